"""GPU: the MultiPeriodDiscriminator forward on the HIP engine (stts_mpd_fwd, through the drop-in
stts2_mi355x.discriminators module) against the fixtures of the REFERENCE module
(tests/golden/mpd_*.npz) and against the oracle at a larger size.

Tolerances: fp32 (exact fp32 MFMA chain, different summation order): 1e-4 relative to each map's
range.  bf16 (bf16 operands and stored maps, 6 layers deep): 3 % of range, correlation >= 0.999."""
import numpy as np
import pytest
import torch

from helpers import golden
from oracle import stts_oracle as orc
from stts2_mi355x import synth

pytestmark = pytest.mark.gpu

_M = {}


def module():
    if "m" not in _M:
        from stts2_mi355x.discriminators import MultiPeriodDiscriminator
        m = MultiPeriodDiscriminator()
        sd = {k: torch.from_numpy(synth.synth_param("mpd." + k, tuple(v.shape))) for k, v in m.state_dict().items()}
        m.load_state_dict(sd)
        _M["m"], _M["sd"] = m.cuda(), sd
    return _M["m"], _M["sd"]


def close(a, b, rel):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    scale = max(1e-3, np.abs(b).max())
    return np.abs(a - b).max() / scale <= rel


@pytest.mark.parametrize("name,maps", [("mpd_B1_T1200", (0, 3, 5)), ("mpd_B2_T1001", ())])
def test_mpd_fp32_matches_reference_fixtures(name, maps):
    m, _ = module()
    g = golden(name)
    with torch.no_grad():
        y_d_rs, y_d_gs, fmap_rs, fmap_gs = m(torch.from_numpy(g["y"]).cuda(), torch.from_numpy(g["y_hat"]).cuda())
    for i in range(5):
        assert tuple(y_d_rs[i].shape) == g[f"score_r{i}"].shape
        assert close(y_d_rs[i].cpu(), g[f"score_r{i}"], 1e-4), (name, i)
        assert close(y_d_gs[i].cpu(), g[f"score_g{i}"], 1e-4), (name, i)
        for j in maps:
            assert tuple(fmap_rs[i][j].shape) == g[f"fmap_r{i}_{j}"].shape
            assert close(fmap_rs[i][j].cpu(), g[f"fmap_r{i}_{j}"], 1e-4), (name, i, j)
            assert close(fmap_gs[i][j].cpu(), g[f"fmap_g{i}_{j}"], 1e-4), (name, i, j)


@pytest.mark.parametrize("dtype,rel", [("fp32", 1e-4), ("bf16", 3e-2)])
def test_mpd_vs_oracle_larger(dtype, rel):
    m, sd = module()
    gen = torch.Generator().manual_seed(3)
    y = torch.randn(2, 1, 9007, generator=gen) * 0.3
    yh = torch.randn(2, 1, 9007, generator=gen) * 0.3
    with torch.no_grad():
        ref = orc.mpd(y, yh, sd)
        out = m(y.cuda(), yh.cuda(), dtype=dtype)
    for k in range(2):  # scores (real, generated)
        for i in range(5):
            assert close(out[k][i].cpu(), ref[k][i], rel), (dtype, k, i)
    for k in (2, 3):  # feature maps
        for i in range(5):
            for j in range(6):
                a, b = out[k][i][j].cpu(), ref[k][i][j]
                assert a.shape == b.shape
                assert close(a, b, rel), (dtype, k, i, j)
                if dtype == "bf16" and b.numel() > 16:
                    assert np.corrcoef(a.flatten(), b.flatten())[0, 1] >= 0.999


@pytest.mark.parametrize("name", ["mpd_B1_T1200", "mpd_B2_T1001"])
def test_mpd_gan_losses_match_reference(name):
    """feature / generator / discriminator losses on the device vs the reference's losses.py values
    stored in the fixture (relative 1e-5)."""
    from stts2_mi355x.discriminators import mpd_gan_losses
    m, _ = module()
    g = golden(name)
    with torch.no_grad():
        fm, gen, disc = mpd_gan_losses(m, torch.from_numpy(g["y"]).cuda(), torch.from_numpy(g["y_hat"]).cuda())
    for got, key in ((fm, "loss_fm"), (gen, "loss_gen"), (disc, "loss_disc")):
        ref = float(g[key])
        assert abs(got.item() - ref) <= 1e-5 * max(1.0, abs(ref)), (key, got.item(), ref)
