"""Golden fixture pinning the duration -> alignment -> waveform chain of inference.py to the REFERENCE:
runs the reference's own `StyleTTS2.generate` (inference.py:303-319, i.e. text_preprocess, then
`__inference` :224-272 per sentence with prev_d_mean chaining, the [4000:-4000] trim, concat and pad)
in the survey container (never on the GPU box):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_generate.py

inference.py cannot be imported as it is here: it imports librosa, noisereduce, soundfile (via
meldataset), torchaudio, munch (absent) and calls nltk.download at import (a network fetch).  This
script installs import-time stubs for those modules only -- none is called on the generate() path
except nltk's word_tokenize, stubbed as str.split, which is exact for the punctuation-free phoneme
sentences used here -- and builds the StyleTTS2 object without its __init__ (no config file /
checkpoint): get_device buffer, Preprocess, TextCleaner over config_example.yaml's symbols, and the
reference TextEncoder / ProsodyPredictor (models.py) and hifigan Decoder filled with the formula weights
of stts2_mi355x/synth.py.  The RNG draws are made reproducible: the SineGen noise is formula noise
(make_golden.NoisePatch's rule, per sentence), and every dur_stats `normal_(mean, std)` draw is
recorded as z = (draw - mean) / std.  Stored: the sentence token ids, z per sentence, the duration means
returned per sentence and the final waveform, as .npz DATA.
"""
from __future__ import annotations

import importlib.machinery
import os
import sys
import types
import warnings

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from make_golden import HIFI_CFG, REF, fill, import_models, synth  # noqa: E402

warnings.filterwarnings("ignore")
PHONEMES = "hɛloʊ wɝld. ðə sɛkənd wʌn"


def stub(name, **attrs):
    if name in sys.modules:
        return sys.modules[name]
    m = types.ModuleType(name)
    m.__spec__ = importlib.machinery.ModuleSpec(name, None)
    for k, v in attrs.items():
        setattr(m, k, v)
    sys.modules[name] = m
    return m


def import_inference():
    import_models()  # munch / torchaudio stubs, models importable
    stub("librosa")
    stub("noisereduce")
    stub("soundfile")
    ta = sys.modules["torchaudio"]
    ta.transforms.MelSpectrogram = lambda *a, **k: None  # meldataset builds one at import, unused here
    stub("nltk", download=lambda *a, **k: True)
    stub("nltk.tokenize", word_tokenize=lambda s: s.split())
    sys.modules["nltk"].tokenize = sys.modules["nltk.tokenize"]
    import inference  # noqa
    return inference


def main():
    inference = import_inference()
    models = import_models()
    import yaml
    from meldataset import TextCleaner
    from Modules.hifigan import Decoder
    cfg = yaml.safe_load(open(os.path.join(REF, "Configs", "config_example.yaml"), encoding="utf-8"))
    sym = cfg["symbol"]
    symbols = list(sym["pad"]) + list(sym["punctuation"]) + list(sym["letters"]) + list(sym["letters_ipa"]) + \
        list(sym["extend"])
    table = {s: i for i, s in enumerate(symbols)}
    obj = inference.StyleTTS2.__new__(inference.StyleTTS2)
    torch.nn.Module.__init__(obj)
    obj.register_buffer("get_device", torch.empty(0))
    obj.preprocess = inference.Preprocess()
    obj.ref_s = None
    obj.cleaner = TextCleaner(table, debug=False)
    obj.text_encoder = fill(models.TextEncoder(channels=512, kernel_size=5, depth=3, n_symbols=len(table) + 1)).eval()
    obj.predictor = fill(models.ProsodyPredictor(style_dim=128, d_hid=512, nlayers=3, max_dur=50, dropout=0.2)).eval()
    obj.decoder = fill(Decoder(dim_in=512, style_dim=128, dim_out=80, **HIFI_CFG)).eval()
    s = torch.from_numpy(synth.normal("refgen:s", (1, 128)))

    rec = {"tokens": [], "z": [], "means": []}
    state = {"k": 0}
    cleaner_call = obj.cleaner.__call__

    def cleaner(text):
        ids = cleaner_call(text)
        rec["tokens"].append(list(ids))
        return ids
    obj.cleaner = cleaner
    normal_ = torch.Tensor.normal_

    def rec_normal(self, mean=0.0, std=1.0, *a, **k):
        out = normal_(self, mean, std, *a, **k)
        z = (out.double() - float(mean)) / float(std)
        rec["z"].append(z.float().numpy())
        return out

    def randn_like(t, *a, **k):
        if t.dim() == 3 and t.shape[-1] == 9:
            r = torch.from_numpy(synth.source_noise(t.shape[0], t.shape[1], tag=f"refgen{state['k']}"))
            state["k"] += 1
            return r
        return torch.zeros_like(t)
    torch.manual_seed(1234)
    rl, rr = torch.randn_like, torch.rand
    torch.Tensor.normal_, torch.randn_like, torch.rand = rec_normal, randn_like, (lambda *sh, **k: torch.zeros(*sh))
    try:
        wav = obj.generate(PHONEMES, {"style": s, "speed": 1}, stabilize=True, n_merge=1)
    finally:
        torch.Tensor.normal_, torch.randn_like, torch.rand = normal_, rl, rr
    out = {"wav": wav.astype(np.float32), "s": s.numpy(), "n_sentences": np.int64(len(rec["tokens"])),
           "n_symbols": np.int64(len(table) + 1)}
    for i, (t, z) in enumerate(zip(rec["tokens"], rec["z"])):
        out[f"tokens{i}"] = np.array(t, np.int64)
        out[f"z{i}"] = z
    path = os.path.join(HERE, "generate_ref.npz")
    np.savez_compressed(path, **out)
    print(path, os.path.getsize(path), wav.shape, [len(t) for t in rec["tokens"]])


if __name__ == "__main__":
    main()
