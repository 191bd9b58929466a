"""Shared test helpers: formula weights for the drop-in modules, golden loading."""
import json
import os

import numpy as np
import torch

from stts2_mi355x import synth

HERE = os.path.dirname(os.path.abspath(__file__))
GOLDEN = os.path.join(HERE, "golden")

HIFI_CFG = dict(resblock_kernel_sizes=[3, 7, 11], upsample_rates=[10, 5, 3, 2], upsample_initial_channel=512,
                resblock_dilation_sizes=[[1, 3, 5], [1, 3, 5], [1, 3, 5]], upsample_kernel_sizes=[20, 10, 6, 4])
ISTFT_CFG = dict(resblock_kernel_sizes=[3, 7, 11], upsample_rates=[10, 6], upsample_initial_channel=512,
                 resblock_dilation_sizes=[[1, 3, 5], [1, 3, 5], [1, 3, 5]], upsample_kernel_sizes=[20, 12],
                 gen_istft_n_fft=20, gen_istft_hop_size=5)


def golden(name):
    return dict(np.load(os.path.join(GOLDEN, name + ".npz")))


def meta():
    with open(os.path.join(GOLDEN, "meta.json")) as f:
        return json.load(f)


def fill_module(module, prefix=""):
    """Load formula weights (stts2_mi355x.synth) into a module by state-dict key."""
    sd = module.state_dict()
    new = {}
    for k, v in sd.items():
        if synth.is_fixed_buffer(k):
            new[k] = v
        else:
            new[k] = torch.from_numpy(synth.synth_param(prefix + k, tuple(v.shape)))
    module.load_state_dict(new, strict=True)
    return module


def make_decoder(kind):
    if kind == "hifigan":
        from stts2_mi355x.hifigan import Decoder
        return fill_module(Decoder(dim_in=512, style_dim=128, dim_out=80, **HIFI_CFG)).eval(), HIFI_CFG
    from stts2_mi355x.istftnet import Decoder
    return fill_module(Decoder(dim_in=512, style_dim=128, dim_out=80, **ISTFT_CFG)).eval(), ISTFT_CFG


def decoder_case(B, T, utt0=0):
    asr, f0, n, s = synth.decoder_inputs(B, T, utt0=utt0)
    noise = synth.source_noise(B, 600 * T, utt0=utt0)
    return [torch.from_numpy(a) for a in (asr, f0, n, s, noise)]


def speech_like(name, L, sr=24000):
    """A reproducible voiced-like clip: a gliding 90-260 Hz fundamental with decaying harmonics,
    a syllabic envelope and formula noise (the mel front-end's test input)."""
    t = np.arange(L, dtype=np.float64) / sr
    f0 = 175 + 85 * np.sin(2 * np.pi * 0.7 * t)
    ph = 2 * np.pi * np.cumsum(f0) / sr
    x = sum(0.3 / h * np.sin(h * ph) for h in range(1, 9))
    env = 0.5 + 0.5 * np.sin(2 * np.pi * 3.1 * t) ** 2
    return (x * env + 0.01 * synth.normal(name, (L,)).astype(np.float64)).astype(np.float32)


DURATION_CASES = ((24, (24, 19, 13)), (60, (60,)))  # (T tokens, lengths per utterance)


def duration_inputs(T, lengths):
    """Duration-path case (tests/golden/make_golden_duration.py): tokens [B,T] int64 (0 past the
    length), lengths [B], style [B,128], alignment [B,T,F] (1-4 frames per token, 0 past the length)."""
    B = len(lengths)
    tok = np.zeros((B, T), np.int64)
    dur = np.zeros((B, T), np.int64)
    for b, n in enumerate(lengths):
        tok[b, :n] = (synth.hash_u01(f"dur:tok:{b}:{T}", n) * 178).astype(np.int64)
        dur[b, :n] = 1 + (synth.hash_u01(f"dur:dur:{b}:{T}", n) * 4).astype(np.int64)
    F = int(dur.sum(1).max())
    aln = np.zeros((B, T, F), np.float32)
    for b in range(B):
        c = 0
        for t in range(T):
            aln[b, t, c:c + dur[b, t]] = 1.0
            c += dur[b, t]
    s = np.stack([synth.normal(f"dur:s:{b}", (128,)) for b in range(B)]).astype(np.float32)
    return tok, np.asarray(lengths, np.int64), s, aln


def make_duration_modules():
    """Drop-in TextEncoder + ProsodyPredictor with the fixtures' formula weights (prefixes te. / pp.)."""
    from stts2_mi355x.models import ProsodyPredictor, TextEncoder
    te = fill_module(TextEncoder(channels=512, kernel_size=5, depth=3, n_symbols=178), "te.").eval()
    pp = fill_module(ProsodyPredictor(style_dim=128, d_hid=512, nlayers=3, max_dur=50, dropout=0.2), "pp.").eval()
    return te, pp
