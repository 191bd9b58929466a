"""GPU: the MultiResSpecDiscriminator forward (stts_msd_fwd through the drop-in module) against the
REFERENCE module's fixtures (tests/golden/msd_*.npz) and the oracle, its GAN losses against the
reference's values, and the multi-resolution mel loss (stts_mrstft_loss) against the oracle.

Tolerances: fp32 1e-4 of each map's range (exact fp32 MFMA chain, different summation order; the |STFT|
is an fp32 radix-2 FFT like torch.stft's); bf16 3 % of range and correlation >= 0.999; losses 1e-4
relative (fp32), the mel loss 1e-4 relative (parity unpinned upstream: torchaudio is absent, the
oracle restates it)."""
import numpy as np
import pytest
import torch

from helpers import golden
from oracle import stts_oracle as orc
from test_msd_oracle import msd_module

pytestmark = pytest.mark.gpu

_M = {}


def module():
    if "m" not in _M:
        m, sd = msd_module()
        _M["m"], _M["sd"] = m.cuda(), sd
    return _M["m"], _M["sd"]


def close(a, b, rel):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    scale = max(1e-3, np.abs(b).max())
    return np.abs(a - b).max() / scale <= rel


@pytest.mark.parametrize("name", ["msd_B1_T2400", "msd_B2_T1801"])
def test_msd_fp32_matches_reference_fixtures(name):
    m, _ = module()
    g = golden(name)
    with torch.no_grad():
        y_d_rs, y_d_gs, fmap_rs, fmap_gs = m(torch.from_numpy(g["y"]).cuda(), torch.from_numpy(g["y_hat"]).cuda())
    for i in range(3):
        assert tuple(y_d_rs[i].shape) == g[f"score_r{i}"].shape
        assert close(y_d_rs[i].cpu(), g[f"score_r{i}"], 1e-4), (name, i)
        assert close(y_d_gs[i].cpu(), g[f"score_g{i}"], 1e-4), (name, i)
        assert tuple(fmap_rs[i][0].shape) == tuple(g[f"shape_fmap0_{i}"])
        for j in (4, 5):
            assert close(fmap_rs[i][j].cpu(), g[f"fmap_r{i}_{j}"], 1e-4), (name, i, j)
            assert close(fmap_gs[i][j].cpu(), g[f"fmap_g{i}_{j}"], 1e-4), (name, i, j)


@pytest.mark.parametrize("dtype,rel", [("fp32", 1e-4), ("bf16", 3e-2)])
def test_msd_vs_oracle_all_maps(dtype, rel):
    m, sd = module()
    gen = torch.Generator().manual_seed(5)
    y = torch.randn(2, 1, 6007, generator=gen) * 0.3
    yh = torch.randn(2, 1, 6007, generator=gen) * 0.3
    with torch.no_grad():
        ref = orc.msd(y, yh, sd)
        out = m(y.cuda(), yh.cuda(), dtype=dtype)
    for k in range(2):
        for i in range(3):
            assert close(out[k][i].cpu(), ref[k][i], rel), (dtype, k, i)
    for k in (2, 3):
        for i in range(3):
            for j in range(6):
                a, b = out[k][i][j].cpu(), ref[k][i][j]
                assert a.shape == b.shape
                assert close(a, b, rel), (dtype, k, i, j)
                if dtype == "bf16":
                    assert np.corrcoef(a.flatten(), b.flatten())[0, 1] >= 0.999


@pytest.mark.parametrize("name", ["msd_B1_T2400", "msd_B2_T1801"])
def test_msd_gan_losses_match_reference(name):
    from stts2_mi355x.discriminators import msd_gan_losses
    m, _ = module()
    g = golden(name)
    fm, gl, dl = msd_gan_losses(m, torch.from_numpy(g["y"]).cuda(), torch.from_numpy(g["y_hat"]).cuda())
    for got, want in ((fm, g["loss_fm"]), (gl, g["loss_gen"]), (dl, g["loss_disc"])):
        assert abs(got.item() - float(want)) <= 1e-4 * max(1.0, abs(float(want))), (got.item(), want)


@pytest.mark.parametrize("B,T", [(2, 93000), (1, 4801)])
def test_mrstft_loss_vs_oracle(B, T):
    from stts2_mi355x.losses import MultiResolutionSTFTLoss
    gen = torch.Generator().manual_seed(B * 7 + T)
    t = torch.arange(T) / 24000.0
    y = (0.4 * torch.sin(2 * torch.pi * 180 * t) + 0.05 * torch.randn(B, T, generator=gen)).float()
    x = (y + 0.03 * torch.randn(B, T, generator=gen)).float()
    want = orc.mrstft_loss(x.unsqueeze(1), y.unsqueeze(1)).item()
    got = MultiResolutionSTFTLoss()(x.cuda().unsqueeze(1), y.cuda().unsqueeze(1)).item()
    print(f"mrstft B={B} T={T}: hip {got:.8f} oracle {want:.8f}")
    assert abs(got - want) <= 1e-4 * abs(want)
    assert MultiResolutionSTFTLoss()(y.cuda(), y.cuda()).item() == 0.0
