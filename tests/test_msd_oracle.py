"""CPU: the MultiResSpecDiscriminator and multi-resolution mel-loss restatements (oracle) against the
reference's fixtures (tests/golden/make_golden_msd.py), the drop-in's state-dict keys and the native
plan's parameter names."""
import ctypes

import numpy as np
import pytest
import torch

from helpers import golden
from oracle import stts_oracle as orc
from stts2_mi355x import engine as E
from stts2_mi355x import synth


def msd_module():
    from stts2_mi355x.discriminators import MultiResSpecDiscriminator
    m = MultiResSpecDiscriminator()
    sd = {k: torch.from_numpy(synth.synth_param("msd." + k, tuple(v.shape))) for k, v in m.state_dict().items()}
    m.load_state_dict(sd)
    return m, sd


@pytest.mark.parametrize("name", ["msd_B1_T2400", "msd_B2_T1801"])
def test_msd_oracle_matches_reference(name):
    g = golden(name)
    _, sd = msd_module()
    with torch.no_grad():
        y_d_rs, y_d_gs, fmap_rs, fmap_gs = orc.msd(torch.from_numpy(g["y"]), torch.from_numpy(g["y_hat"]), sd)
        fm, gen, disc = orc.gan_losses(y_d_rs, y_d_gs, fmap_rs, fmap_gs)
    for i in range(3):
        assert np.abs(y_d_rs[i].numpy() - g[f"score_r{i}"]).max() < 1e-5
        assert np.abs(y_d_gs[i].numpy() - g[f"score_g{i}"]).max() < 1e-5
        assert tuple(fmap_rs[i][0].shape) == tuple(g[f"shape_fmap0_{i}"])
        for j in (4, 5):
            assert np.abs(fmap_rs[i][j].numpy() - g[f"fmap_r{i}_{j}"]).max() < 1e-5
    assert abs(fm.item() - g["loss_fm"]) < 1e-6 * max(1, abs(g["loss_fm"]))
    assert abs(gen.item() - g["loss_gen"]) < 1e-6 * max(1, abs(g["loss_gen"]))
    assert abs(disc.item() - g["loss_disc"]) < 1e-6 * max(1, abs(g["loss_disc"]))


def test_msd_plan_names_match_state_dict():
    m, _ = msd_module()
    L = E.lib()
    cfg = [3, 1024, 120, 600, 2048, 240, 1200, 512, 50, 240]
    arr = (ctypes.c_int * len(cfg))(*cfg)
    h = ctypes.c_void_p()
    assert L.stts_model_create(E.KIND_MSD, arr, len(cfg), ctypes.byref(h)) == 0
    sd = m.state_dict()
    names = [L.stts_param_name(h, i).decode() for i in range(L.stts_param_count(h))]
    assert sorted(names) == sorted(sd)
    for i, n in enumerate(names):
        assert L.stts_param_numel(h, i) == sd[n].numel(), n
    assert L.stts_workspace_bytes(h, 1, 4, 93000) > 0
    # out elems: per resolution 5 maps x 32 channels + the score map, as the reference's shapes
    T, B = 2400, 2
    want = 0
    for f, hop, _ in orc.MSD_RES:
        H, W = E.msd_geometry(T, f, hop)
        want += sum(B * H * W[j + 1] * 32 for j in range(5)) + B * H * W[5]
    assert L.stts_msd_out_elems(h, B, T) == want
    L.stts_model_destroy(h)


def test_mrstft_oracle_properties():
    """losses.py:24-94 restated (torchaudio is absent here: parity unpinned upstream; the mel filterbank
    restatement is pinned by tests/test_mel_oracle.py's known answers): identical signals give 0, the
    loss is scale-aware and finite, and the three resolutions' frame counts are 1 + T // hop."""
    g = torch.Generator().manual_seed(0)
    y = torch.randn(2, 9000, generator=g) * 0.2
    x = y + torch.randn(2, 9000, generator=g) * 0.02
    assert orc.mrstft_loss(y, y).item() == 0.0
    l1 = orc.mrstft_loss(x, y).item()
    l2 = orc.mrstft_loss(y + (x - y) * 3, y).item()
    assert 0 < l1 < l2 < 1
    for f, hop, w in zip(*orc.MRSTFT.values()):
        assert orc.mel_spectrogram_sr(y, 24000, f, w, hop).shape == (2, 128, 1 + 9000 // hop)
