"""GPU parity: ProsodyPredictor.F0Ntrain conv stacks (HIP) vs the reference golden outputs."""
import numpy as np
import pytest
import torch

from helpers import fill_module, golden
from stts2_mi355x import synth

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _inference():
    """These modules' HIP paths are forward-only (engine.forward_only): run as inference.py does."""
    with torch.no_grad():
        yield


def predictor():
    from stts2_mi355x.models import ProsodyPredictor
    return fill_module(ProsodyPredictor(style_dim=128, d_hid=512, nlayers=3, max_dur=50, dropout=0.2)).eval().cuda()


@pytest.mark.parametrize("T,B", [(8, 2), (40, 1)])
@pytest.mark.parametrize("dtype", ["fp32", "bf16", "bf16x3"])
def test_f0n_convstacks(T, B, dtype):
    pp = predictor()
    g = golden(f"f0n_T{T}_B{B}")
    s = torch.from_numpy(np.stack([synth.normal(f"f0n:s:{b}", (128,)) for b in range(B)])).cuda()
    xl = torch.from_numpy(g["tap_lstm"]).transpose(1, 2).contiguous().cuda()  # [B, T, 512]
    F0, N = pp.f0n_engine(dtype).forward_nlc(xl, s)
    tol = {"fp32": 2e-4, "bf16x3": 5e-4}.get(dtype, 0.1)  # bf16x3: the split accuracy mode
    print(f"f0n T={T} {dtype}: F0 {np.abs(F0.cpu().numpy() - g['F0']).max():.3e} N {np.abs(N.cpu().numpy() - g['N']).max():.3e}")
    assert np.abs(F0.cpu().numpy() - g["F0"]).max() < tol
    assert np.abs(N.cpu().numpy() - g["N"]).max() < tol


def test_f0ntrain_end_to_end():
    pp = predictor()
    T, B = 40, 1
    g = golden(f"f0n_T{T}_B{B}")
    en = torch.from_numpy(np.stack([synth.normal(f"f0n:en:{b}:{T}", (640, T)) for b in range(B)])).cuda()
    s = torch.from_numpy(np.stack([synth.normal(f"f0n:s:{b}", (128,)) for b in range(B)])).cuda()
    F0, N = pp.F0Ntrain(en, s)
    assert np.abs(F0.cpu().numpy() - g["F0"]).max() < 1e-3
    assert np.abs(N.cpu().numpy() - g["N"]).max() < 1e-3
