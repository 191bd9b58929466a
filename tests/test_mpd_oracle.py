"""CPU: the MultiPeriodDiscriminator oracle (oracle/stts_oracle.py: mpd) against the fixtures the
REFERENCE module produced (tests/golden/make_golden_mpd.py), and the drop-in module's state-dict
contract (same keys / shapes as Modules/discriminators.py)."""
import numpy as np
import torch

from helpers import golden
from oracle import stts_oracle as orc
from stts2_mi355x import synth


def mpd_state_dict():
    from stts2_mi355x.discriminators import MultiPeriodDiscriminator
    m = MultiPeriodDiscriminator()
    return {k: torch.from_numpy(synth.synth_param("mpd." + k, tuple(v.shape))) for k, v in m.state_dict().items()}, m


def test_dropin_keys_match_reference_layout():
    sd, m = mpd_state_dict()
    assert len(sd) == 5 * 6 * 3  # 5 periods x (5 convs + conv_post) x (weight_g, weight_v, bias)
    assert tuple(sd["discriminators.0.convs.0.weight_v"].shape) == (32, 1, 5, 1)
    assert tuple(sd["discriminators.4.conv_post.weight_g"].shape) == (1, 1, 1, 1)
    assert [d.period for d in m.discriminators] == [2, 3, 5, 7, 11]


def test_mpd_oracle_matches_reference_fixtures():
    sd, _ = mpd_state_dict()
    for name, maps in (("mpd_B1_T1200", (0, 3, 5)), ("mpd_B2_T1001", ())):
        g = golden(name)
        y, yh = torch.from_numpy(g["y"]), torch.from_numpy(g["y_hat"])
        with torch.no_grad():
            y_d_rs, y_d_gs, fmap_rs, fmap_gs = orc.mpd(y, yh, sd)
        for i in range(5):
            np.testing.assert_allclose(y_d_rs[i].numpy(), g[f"score_r{i}"], rtol=1e-5, atol=1e-5)
            np.testing.assert_allclose(y_d_gs[i].numpy(), g[f"score_g{i}"], rtol=1e-5, atol=1e-5)
            for j in maps:
                np.testing.assert_allclose(fmap_rs[i][j].numpy(), g[f"fmap_r{i}_{j}"], rtol=1e-5, atol=1e-5)
                np.testing.assert_allclose(fmap_gs[i][j].numpy(), g[f"fmap_g{i}_{j}"], rtol=1e-5, atol=1e-5)


def test_mpd_native_layout_sizes():
    """The C-ABI sizes the MPD workspace and output (a forward without statistics must still size
    its buffers: this once returned 0 bytes)."""
    import ctypes
    from stts2_mi355x import engine as E
    L = E.lib()
    h = ctypes.c_void_p()
    arr = (ctypes.c_int * 6)(5, 2, 3, 5, 7, 11)
    assert L.stts_model_create(E.KIND_MPD, arr, 6, ctypes.byref(h)) == 0
    try:
        assert L.stts_param_count(h) == 90
        T, B = 1200, 2
        n = 0
        for p in (2, 3, 5, 7, 11):
            Ls = E.mpd_lengths(T, p)
            n += sum(B * p * Ls[j + 1] * E.MPD_CH[j + 1] for j in range(5)) + B * p * Ls[5]  # + conv_post
        assert L.stts_mpd_out_elems(h, B, T) == n
        for dt in (0, 1):
            assert L.stts_workspace_bytes(h, dt, B, T) >= B * 2 * 600 * 8 * (4 if dt == 0 else 2)
    finally:
        L.stts_model_destroy(h)
