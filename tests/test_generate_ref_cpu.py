"""CPU: the oracle's restatement of inference.py's duration -> alignment -> waveform chain and generate()
loop (oracle.inference_chain / oracle.generate) against the REFERENCE's own StyleTTS2.generate run on
the same formula weights, inputs, dur_stats draws and SineGen noise (tests/golden/make_golden_generate.py).
This pins the durations / alignment step that was only checked by hand-computed known answers."""
import numpy as np
import torch

from helpers import HIFI_CFG, fill_module, golden
from oracle import stts_oracle as orc
from stts2_mi355x import synth


def modules(n_symbols):
    from stts2_mi355x.hifigan import Decoder
    from stts2_mi355x.models import ProsodyPredictor, TextEncoder
    te = fill_module(TextEncoder(channels=512, kernel_size=5, depth=3, n_symbols=n_symbols)).eval()
    pp = fill_module(ProsodyPredictor(style_dim=128, d_hid=512, nlayers=3, max_dur=50, dropout=0.2)).eval()
    dec = fill_module(Decoder(dim_in=512, style_dim=128, dim_out=80, **HIFI_CFG)).eval()
    return te, pp, dec


def case():
    g = golden("generate_ref")
    n = int(g["n_sentences"])
    sents = [[int(v) for v in g[f"tokens{i}"]] for i in range(n)]
    zs = [torch.from_numpy(g[f"z{i}"]) for i in range(n)]
    nfs = [(lambda F, i=i: torch.from_numpy(synth.source_noise(1, 600 * F, tag=f"refgen{i}"))) for i in range(n)]
    return g, sents, zs, nfs


def test_oracle_generate_matches_reference():
    g, sents, zs, nfs = case()
    te, pp, dec = modules(int(g["n_symbols"]))
    sd = lambda m: {k: v for k, v in m.state_dict().items()}  # noqa: E731
    with torch.no_grad():
        got = orc.generate(sents, torch.from_numpy(g["s"]), sd(te), sd(pp), sd(dec), HIFI_CFG, zs, nfs,
                           stabilize=True)
    assert got.shape == g["wav"].shape
    err = float(np.abs(got - g["wav"]).max())
    print(f"oracle generate vs reference: {got.shape[0]} samples, max-abs {err:.3e}")
    assert err < 1e-4
