"""Generate the golden fixtures in tests/golden/ by running the REFERENCE modules.

Run in the survey container only (needs /root/reference; never on the GPU box):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py

What it does:
  * imports the reference modules read-only (Modules/hifigan.py, Modules/istftnet.py,
    models.py — the latter with import-time stubs for `munch` and `torchaudio`, which are
    absent here and unused by the modules exercised);
  * fills every parameter from the formula in stts2_mi355x/synth.py (by state-dict key);
  * generates inputs from the same formula, and replaces the reference's RNG draws
    (hifigan.py:126 rand, :213 randn_like(sine_waves), :267 randn_like(uv)) by formula
    noise so the GPU box can regenerate the exact noise tensor;
  * records outputs (and a few intermediate taps) as .npz fixtures = DATA only.
"""
from __future__ import annotations

import json
import os
import sys
import types
import warnings

import numpy as np
import torch

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "styletts2-lite_amd"))
sys.path.insert(0, REF)
warnings.filterwarnings("ignore")

from stts2_mi355x import synth  # noqa: E402

HIFI_CFG = dict(resblock_kernel_sizes=[3, 7, 11], upsample_rates=[10, 5, 3, 2], upsample_initial_channel=512,
                resblock_dilation_sizes=[[1, 3, 5], [1, 3, 5], [1, 3, 5]], upsample_kernel_sizes=[20, 10, 6, 4])
ISTFT_CFG = dict(resblock_kernel_sizes=[3, 7, 11], upsample_rates=[10, 6], upsample_initial_channel=512,
                 resblock_dilation_sizes=[[1, 3, 5], [1, 3, 5], [1, 3, 5]], upsample_kernel_sizes=[20, 12],
                 gen_istft_n_fft=20, gen_istft_hop_size=5)


def fill(module, prefix=""):
    sd = module.state_dict()
    new = {}
    for k, v in sd.items():
        if synth.is_fixed_buffer(k):
            new[k] = v
        else:
            new[k] = torch.from_numpy(synth.synth_param(prefix + k, tuple(v.shape)))
    module.load_state_dict(new, strict=True)
    return module


class NoisePatch:
    """Replace torch.rand / torch.randn_like inside the reference's SineGen by formula noise."""

    def __init__(self, noise):
        self.noise = torch.from_numpy(noise)

    def __enter__(self):
        self._rand, self._randn_like = torch.rand, torch.randn_like
        noise = self.noise

        def randn_like(t, *a, **k):
            if t.dim() == 3 and t.shape[-1] == 9:
                assert tuple(t.shape) == tuple(noise.shape), (t.shape, noise.shape)
                return noise.clone()
            return torch.zeros_like(t)  # randn_like(uv): unused by the decoder output

        def rand(*shape, **k):
            return torch.zeros(*shape)  # rand_ini: provably no effect at x300

        torch.randn_like, torch.rand = randn_like, rand
        return self

    def __exit__(self, *a):
        torch.rand, torch.randn_like = self._rand, self._randn_like


def run_decoder(kind, T, B, taps_wanted):
    if kind == "hifigan":
        from Modules.hifigan import Decoder
        dec = Decoder(dim_in=512, style_dim=128, dim_out=80, **HIFI_CFG)
        scale = 300
    else:
        from Modules.istftnet import Decoder
        dec = Decoder(dim_in=512, style_dim=128, dim_out=80, **ISTFT_CFG)
        scale = 300
    dec = fill(dec).eval()
    asr, f0, n, s = synth.decoder_inputs(B, T)
    L = 2 * T * scale
    noise = synth.source_noise(B, L)
    taps = {}
    hooks = []
    if taps_wanted:
        g = dec.generator
        hooks.append(dec.decode[3].register_forward_hook(lambda m, i, o: taps.__setitem__("frontend", o.detach())))
        for i in sorted({0, len(g.ups) - 1}):
            hooks.append(g.noise_res[i].register_forward_hook(
                lambda m, inp, o, i=i: taps.__setitem__(f"noise_res{i}", o.detach())))
            hooks.append(g.ups[i].register_forward_hook(
                lambda m, inp, o, i=i: taps.__setitem__(f"ups{i}", o.detach())))
        hooks.append(g.conv_post.register_forward_hook(lambda m, i, o: taps.__setitem__("post", o.detach())))
        hooks.append(g.m_source.register_forward_hook(lambda m, i, o: taps.__setitem__("har", o[0].detach())))
    with torch.no_grad(), NoisePatch(noise):
        out = dec(torch.from_numpy(asr), torch.from_numpy(f0), torch.from_numpy(n), torch.from_numpy(s))
    for h in hooks:
        h.remove()
    res = {"out": out.numpy().astype(np.float32)}
    for k, v in taps.items():
        res["tap_" + k] = v.numpy().astype(np.float32)
    return res


def import_models():
    """models.py imports munch / torchaudio at module level (models.py:6-11); both are
    absent here and not used by ProsodyPredictor / StyleEncoder: stub them."""
    if "munch" not in sys.modules:
        m = types.ModuleType("munch")

        class Munch(dict):
            __getattr__ = dict.get
        m.Munch = Munch
        sys.modules["munch"] = m
    if "torchaudio" not in sys.modules:
        ta = types.ModuleType("torchaudio")
        ta.transforms = types.SimpleNamespace(MelSpectrogram=None)
        ta.functional = types.SimpleNamespace()
        sys.modules["torchaudio"] = ta
        sys.modules["torchaudio.transforms"] = ta.transforms
        sys.modules["torchaudio.functional"] = ta.functional
    import models  # noqa
    return models


def run_f0n(T, B):
    models = import_models()
    pp = fill(models.ProsodyPredictor(style_dim=128, d_hid=512, nlayers=3, max_dur=50, dropout=0.2)).eval()
    en = np.stack([synth.normal(f"f0n:en:{b}:{T}", (640, T)) for b in range(B)])
    s = np.stack([synth.normal(f"f0n:s:{b}", (128,)) for b in range(B)])
    taps = {}
    h = pp.shared.register_forward_hook(lambda m, i, o: taps.__setitem__("lstm", o[0].detach()))
    with torch.no_grad():
        F0, N = pp.F0Ntrain(torch.from_numpy(en), torch.from_numpy(s))
    h.remove()
    return {"F0": F0.numpy(), "N": N.numpy(), "tap_lstm": taps["lstm"].transpose(-1, -2).contiguous().numpy()}


def run_style(Fr, B):
    models = import_models()
    se = fill(models.StyleEncoder(dim_in=64, style_dim=128, max_conv_dim=512)).eval()
    mel = np.stack([synth.normal(f"style:mel:{b}:{Fr}", (1, 80, Fr)) for b in range(B)])
    with torch.no_grad():
        out = se(torch.from_numpy(mel))
    return {"out": out.numpy()}


def main():
    meta = {"torch": torch.__version__, "numpy": np.__version__,
            "generator": "tests/golden/make_golden.py", "reference": "thewh1teagle/StyleTTS2-lite @ 2025-06-14",
            "cases": {}}
    torch.set_num_threads(8)
    for kind in ("hifigan", "istftnet"):
        for T, B, taps in ((4, 1, True), (4, 2, False), (16, 2, False), (40, 1, False), (400, 1, False)):
            r = run_decoder(kind, T, B, taps)
            name = f"{kind}_T{T}_B{B}"
            np.savez_compressed(os.path.join(HERE, name + ".npz"), **r)
            meta["cases"][name] = {"kind": kind, "T": T, "B": B, "keys": sorted(r.keys()),
                                   "out_absmax": float(np.abs(r["out"]).max()), "out_std": float(r["out"].std())}
            print(name, {k: v.shape for k, v in r.items()}, meta["cases"][name]["out_std"], flush=True)
    for T, B in ((8, 2), (40, 1)):
        r = run_f0n(T, B)
        name = f"f0n_T{T}_B{B}"
        np.savez_compressed(os.path.join(HERE, name + ".npz"), **r)
        meta["cases"][name] = {"kind": "f0n", "T": T, "B": B, "keys": sorted(r.keys())}
        print(name, {k: v.shape for k, v in r.items()}, flush=True)
    for Fr, B in ((80, 2), (241, 1)):
        r = run_style(Fr, B)
        name = f"style_F{Fr}_B{B}"
        np.savez_compressed(os.path.join(HERE, name + ".npz"), **r)
        meta["cases"][name] = {"kind": "style", "F": Fr, "B": B, "keys": sorted(r.keys())}
        print(name, {k: v.shape for k, v in r.items()}, flush=True)
    with open(os.path.join(HERE, "meta.json"), "w") as f:
        json.dump(meta, f, indent=1)


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "probe":
        for kind in ("hifigan", "istftnet"):
            r = run_decoder(kind, 40, 1, True)
            for k, v in r.items():
                print(kind, k, v.shape, "std %.4f absmax %.4f" % (v.std(), np.abs(v).max()))
    else:
        main()
