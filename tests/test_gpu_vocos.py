"""Vocos decoder on the MI355X (STTS_KIND_VOCOS through the C-ABI) against the reference's golden
outputs (tests/golden/make_golden_vocos.py) and the oracle.  North-star bar: fp32 waveform within
1e-3 max-abs of the reference's CPU output."""
import numpy as np
import pytest
import torch

from helpers import golden
from oracle import stts_oracle as orc
from stts2_mi355x import synth
from test_vocos_cpu import make_vocos

pytestmark = pytest.mark.gpu


def _inputs(B, T):
    return [torch.from_numpy(a).cuda() for a in synth.decoder_inputs(B, T, tag="vocos")]


@pytest.mark.parametrize("n_fft,hop,T,B", [(1200, 300, 4, 2), (1024, 256, 16, 1), (1200, 300, 40, 1),
                                           (1200, 300, 400, 1)])
def test_vocos_fp32_matches_reference(n_fft, hop, T, B):
    g = golden(f"vocos_n{n_fft}_T{T}_B{B}")
    dec = make_vocos(n_fft, hop).cuda()
    with torch.no_grad():
        out = dec(*_inputs(B, T), dtype="fp32")
    torch.cuda.synchronize()
    err = np.abs(out.cpu().numpy() - g["out"]).max()
    print(f"vocos n_fft {n_fft} T {T} B {B} fp32 max-abs vs reference {err:.3e}")
    assert out.shape == (B, 1, 2 * T * hop)
    assert err < 1e-3  # north star; measured ~1e-6


def test_vocos_bf16_close_to_fp32():
    dec = make_vocos().cuda()
    x = _inputs(2, 400)
    with torch.no_grad():
        ref = dec(*x, dtype="fp32").cpu().numpy()
        out = dec(*x, dtype="bf16").cpu().numpy()
    err = np.abs(out - ref).max()
    corr = min(np.corrcoef(out[b, 0], ref[b, 0])[0, 1] for b in range(2))
    print(f"vocos bf16 vs fp32 10 s: max-abs {err:.3e} corr {corr:.6f}")
    assert corr > 0.99 and err < 0.1


def test_vocos_batch_rows_independent():
    """B = 3 equals three B = 1 calls (InstanceNorm / LayerNorm / ISTFT are per utterance)."""
    dec = make_vocos().cuda()
    x = _inputs(3, 40)
    with torch.no_grad():
        full = dec(*x, dtype="fp32")
        for b in range(3):
            one = dec(*[t[b:b + 1] for t in x], dtype="fp32")
            assert torch.allclose(one, full[b:b + 1], atol=1e-6, rtol=0)


def test_vocos_vs_oracle_odd_length():
    """T = 7 (14 frames): odd frame counts through the overlap-add edges, against the oracle."""
    dec = make_vocos(1024, 256)
    x = [torch.from_numpy(a) for a in synth.decoder_inputs(1, 7, tag="vocos-odd")]
    with torch.no_grad():
        ref = orc.decoder_vocos(*x, dec.state_dict(), dict(num_layers=8, n_fft=1024, hop=256))
        out = dec.cuda()(*[t.cuda() for t in x], dtype="fp32").cpu()
    assert (out - ref).abs().max().item() < 1e-4


def test_vocos_rejects_noise():
    dec = make_vocos().cuda()
    x = _inputs(1, 4)
    with pytest.raises(ValueError):
        dec.engine("fp32").forward(*x, noise=torch.zeros(1, 2400, 9))
