"""Pin the CPU oracle (oracle/stts_oracle.py) against the reference's own outputs
(golden fixtures made by importing the reference modules, tests/golden/make_golden.py)."""
import numpy as np
import pytest
import torch

from helpers import decoder_case, golden, make_decoder
from oracle import stts_oracle as orc


def _sd(mod):
    return {k: v.detach() for k, v in mod.state_dict().items()}


@pytest.mark.parametrize("kind", ["hifigan", "istftnet"])
@pytest.mark.parametrize("T,B", [(4, 1), (4, 2), (16, 2), (40, 1)])
def test_decoder_oracle_matches_reference(kind, T, B):
    dec, cfg = make_decoder(kind)
    asr, f0, n, s, noise = decoder_case(B, T)
    g = golden(f"{kind}_T{T}_B{B}")
    taps = {}
    fn = orc.decoder_hifigan if kind == "hifigan" else orc.decoder_istft
    with torch.no_grad():
        out = fn(asr, f0, n, s, _sd(dec), cfg, noise, taps)
    # fp32 reorder floor of the reference itself is <=1.75e-5 at 10 s
    np.testing.assert_allclose(out.numpy(), g["out"], atol=2e-5, rtol=0)
    if "tap_har" in g:  # reference m_source output (sine_merge, [B, L, 1]) and front-end output
        np.testing.assert_allclose(taps["source"].numpy(), g["tap_har"], atol=1e-6, rtol=0)
        np.testing.assert_allclose(taps["frontend"].numpy(), g["tap_frontend"], atol=2e-5, rtol=0)


@pytest.mark.slow
@pytest.mark.parametrize("kind", ["hifigan", "istftnet"])
def test_decoder_oracle_10s(kind):
    dec, cfg = make_decoder(kind)
    asr, f0, n, s, noise = decoder_case(1, 400)
    g = golden(f"{kind}_T400_B1")
    fn = orc.decoder_hifigan if kind == "hifigan" else orc.decoder_istft
    with torch.no_grad():
        out = fn(asr, f0, n, s, _sd(dec), cfg, noise)
    np.testing.assert_allclose(out.numpy(), g["out"], atol=5e-5, rtol=0)


def _predictor():
    from stts2_mi355x.models import ProsodyPredictor
    from helpers import fill_module
    return fill_module(ProsodyPredictor(style_dim=128, d_hid=512, nlayers=3, max_dur=50, dropout=0.2)).eval()


@pytest.mark.parametrize("T,B", [(8, 2), (40, 1)])
def test_f0ntrain_oracle_matches_reference(T, B):
    from stts2_mi355x import synth
    pp = _predictor()
    en = torch.from_numpy(np.stack([synth.normal(f"f0n:en:{b}:{T}", (640, T)) for b in range(B)]))
    s = torch.from_numpy(np.stack([synth.normal(f"f0n:s:{b}", (128,)) for b in range(B)]))
    g = golden(f"f0n_T{T}_B{B}")
    sd = _sd(pp)
    xl = orc.shared_lstm(en, sd)
    np.testing.assert_allclose(xl.numpy(), g["tap_lstm"], atol=1e-5)
    F0, N = orc.f0n_convstacks(torch.from_numpy(g["tap_lstm"]), s, sd)
    np.testing.assert_allclose(F0.numpy(), g["F0"], atol=1e-4, rtol=0)
    np.testing.assert_allclose(N.numpy(), g["N"], atol=1e-4, rtol=0)


@pytest.mark.parametrize("Fr,B", [(80, 2), (241, 1)])
def test_style_encoder_oracle_matches_reference(Fr, B):
    from stts2_mi355x import synth
    from stts2_mi355x.models import StyleEncoder
    from helpers import fill_module
    se = fill_module(StyleEncoder(dim_in=64, style_dim=128, max_conv_dim=512)).eval()
    mel = torch.from_numpy(np.stack([synth.normal(f"style:mel:{b}:{Fr}", (1, 80, Fr)) for b in range(B)]))
    g = golden(f"style_F{Fr}_B{B}")
    out = orc.style_encoder(mel, _sd(se))
    np.testing.assert_allclose(out.numpy(), g["out"], atol=1e-5, rtol=0)
