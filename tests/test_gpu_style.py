"""GPU parity: StyleEncoder (HIP 2-D ResNet) vs the reference golden outputs."""
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


@pytest.mark.parametrize("Fr,B", [(80, 2), (241, 1)])
@pytest.mark.parametrize("dtype", ["fp32", "bf16", "bf16x3"])
def test_style_encoder(Fr, B, dtype):
    from stts2_mi355x.models import StyleEncoder
    se = fill_module(StyleEncoder(dim_in=64, style_dim=128, max_conv_dim=512)).eval().cuda()
    mel = torch.from_numpy(np.stack([synth.normal(f"style:mel:{b}:{Fr}", (1, 80, Fr)) for b in range(B)])).cuda()
    out = se(mel, dtype=dtype).cpu().numpy()
    ref = golden(f"style_F{Fr}_B{B}")["out"]
    err = np.abs(out - ref).max()
    scale = np.abs(ref).max()
    print(f"style F={Fr} {dtype}: max-abs {err:.3e} (ref absmax {scale:.3f})")
    assert err < {"fp32": 1e-4, "bf16x3": 2e-4}.get(dtype, 0.05 * scale)  # bf16x3: the split accuracy mode
