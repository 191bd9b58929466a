"""GPU: the conv1d_igemm engine (one launch through the stts_test_conv1d hook) against
torch.nn.functional fp32 on the CPU: dilation, stride, polyphase ConvTranspose1d,
AdaIN/Snake/LReLU prologues, residual + scale epilogue and the InstanceNorm statistics."""
import ctypes

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from stts2_mi355x import engine as E

pytestmark = pytest.mark.gpu

CASES = [
    # name, Cin, Cout, K, transposed, stride(u), dil, pad, out_pad, L, pro
    ("rb32_k11_d5", 32, 32, 11, 0, 1, 5, 25, 0, 700, 3),
    ("rb64_k7_d3", 64, 64, 7, 0, 1, 3, 9, 0, 333, 3),
    ("rb128_k3_d1", 128, 128, 3, 0, 1, 1, 1, 0, 257, 3),
    ("rb256_k11_d1", 256, 256, 11, 0, 1, 1, 5, 0, 130, 3),
    ("rb32_k3_d1", 32, 32, 3, 0, 1, 1, 1, 0, 1300, 3),
    ("rb32_k7_d3", 32, 32, 7, 0, 1, 3, 9, 0, 517, 3),
    ("rb64_k11_d5", 64, 64, 11, 0, 1, 5, 25, 0, 600, 3),
    ("rb64_k3_d1", 64, 64, 3, 0, 1, 1, 1, 0, 2049, 3),
    ("rb128_k7_d3", 128, 128, 7, 0, 1, 3, 9, 0, 1000, 3),
    ("rb128_k11_d5", 128, 128, 11, 0, 1, 5, 25, 0, 777, 3),
    ("rb256_k3_d5", 256, 256, 3, 0, 1, 5, 5, 0, 600, 3),
    ("rb256_k7_d1", 256, 256, 7, 0, 1, 1, 3, 0, 513, 3),
    # conv1 of a resblock iteration: no residual (bigconv2 RES = false), dilated
    ("rb256_k3_d3_nores", 256, 256, 3, 0, 1, 3, 3, 0, 700, 3),
    ("rb256_k11_d5_nores", 256, 256, 11, 0, 1, 5, 25, 0, 300, 3),
    ("rb128_k11_d5_nores", 128, 128, 11, 0, 1, 5, 25, 0, 1500, 3),
    ("rb128_k7_d1_nores", 128, 128, 7, 0, 1, 1, 3, 0, 511, 3),
    ("front_1090_1024", 1090, 1024, 3, 0, 1, 1, 1, 0, 40, 5),
    # decoder front-end AdainResBlk1d convs on the bigconv2 engine (STTS_OPT_FRONT, bf16)
    ("front_514_1024_nores", 514, 1024, 3, 0, 1, 1, 1, 0, 300, 5),
    ("front_1024_1024", 1024, 1024, 3, 0, 1, 1, 1, 0, 400, 5),
    ("front_1090_512", 1090, 512, 3, 0, 1, 1, 1, 0, 800, 5),
    ("front_1090_512_nopro_nores", 1090, 512, 3, 0, 1, 1, 1, 0, 517, 0),
    ("sc_1x1", 514, 1024, 1, 0, 1, 1, 0, 0, 37, 0),
    ("istft_noise_s6", 22, 256, 12, 0, 6, 1, 3, 0, 481, 0),
    ("post_32_1", 32, 1, 7, 0, 1, 1, 3, 0, 999, 2),
    ("ups0_u10", 512, 256, 20, 1, 10, 1, 5, 0, 23, 2),
    ("ups1_u5", 256, 128, 10, 1, 5, 1, 3, 1, 31, 2),
    ("ups2_u3", 128, 64, 6, 1, 3, 1, 2, 1, 40, 4),
    ("ups3_u2", 64, 32, 4, 1, 2, 1, 1, 0, 77, 2),
    ("istft_ups1_u6", 256, 128, 12, 1, 6, 1, 3, 0, 50, 4),
]


def reference(x, w, b, gb, alpha, slope, res, scale, c):
    name, Cin, Cout, K, tr, st, dil, pad, op, L, pro = c
    v = x.transpose(1, 2)  # [B, Cin, L]
    if pro & 1:
        n = F.instance_norm(v, eps=1e-5)
        g, be = gb[:, :Cin, None], gb[:, Cin:, None]
        v = (1 + g) * n + be
    if pro & 2:
        a = alpha[None, :, None]
        v = v + (1 / a) * torch.sin(a * v) ** 2
    if pro & 4:
        v = F.leaky_relu(v, slope)
    if tr:
        y = F.conv_transpose1d(v, w, b, st, pad, op)
    else:
        y = F.conv1d(v, w, b, st, pad, dil)
    y = y.transpose(1, 2)
    if res is not None:
        y = y + res
    return y * scale


def run_case(case, dtype, stats=True, res_tr=False):
    """res_tr: a residual (scale 1) also for the transposed cases, as the HiFi-GAN upsamplers add the noise
    branch (hifigan.py:335)."""
    name, Cin, Cout, K, tr, st, dil, pad, op, L, pro = case
    g = torch.Generator().manual_seed(hash(name) % 1000)
    B = 2
    x = torch.randn(B, L, Cin, generator=g) * 1.5 + 0.3
    w = torch.randn(*((Cin, Cout, K) if tr else (Cout, Cin, K)), generator=g) / np.sqrt(Cin * K / (st if tr else 1))
    b = torch.randn(Cout, generator=g) * 0.1
    gb = torch.randn(B, 2 * Cin, generator=g) * 0.3
    alpha = torch.rand(Cin, generator=g) + 0.5
    slope = 0.2
    Lout = (L - 1) * st - 2 * pad + K + op if tr else (L + 2 * pad - dil * (K - 1) - 1) // st + 1
    res = torch.randn(B, Lout, Cout, generator=g) if (res_tr or not tr) and not name.endswith("_nores") else None
    scale = 0.70710677 if res is not None and not tr else 1.0
    ref = reference(x, w, b, gb, alpha, slope, res, scale, case)
    dev = "cuda"
    xd, wd, bd, gbd, ad = (t.to(dev).contiguous() for t in (x, w, b, gb, alpha))
    rd = res.to(dev).contiguous() if res is not None else None
    y = torch.empty(B, Lout, Cout, device=dev)
    st_out = torch.zeros(B, Cout, 2, dtype=torch.float64, device=dev)
    P = lambda t: ctypes.c_void_p(t.data_ptr()) if t is not None else ctypes.c_void_p(0)  # noqa: E731
    rc = E.lib().stts_test_conv1d(E.DTYPES[dtype], P(xd), B, L, Cin, P(wd), P(bd), Cout, K, tr, st, dil, pad, op,
                                  pro, P(gbd), P(ad), ctypes.c_float(slope), P(rd), ctypes.c_float(scale), P(y), Lout,
                                  P(st_out if stats else None))
    E.check(rc)
    return ref, y.cpu(), st_out.cpu()


@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
@pytest.mark.parametrize("case", CASES, ids=[c[0] for c in CASES])
def test_conv_engine(case, dtype):
    name = case[0]
    ref, y, s = run_case(case, dtype)
    err = (y - ref).abs().max().item()
    tol = 2e-4 if dtype == "fp32" else 0.03 * max(1.0, ref.abs().max().item() / 4)
    assert err < tol, f"{name} {dtype}: max err {err}"
    yd = y.double()
    if dtype == "fp32":
        np.testing.assert_allclose(s[..., 0].numpy(), yd.sum(1).numpy(), rtol=1e-5, atol=1e-3)
        np.testing.assert_allclose(s[..., 1].numpy(), (yd ** 2).sum(1).numpy(), rtol=1e-5, atol=1e-3)
    else:
        # bf16 mode: the statistics are taken from the fp32 epilogue values, before the bf16
        # store rounds them (relative rounding <= 2^-8 per summand)
        bound_s = yd.abs().sum(1) * 2.0 ** -8 + 1e-3
        bound_q = (yd ** 2).sum(1) * 2.0 ** -7 + 1e-3
        assert ((s[..., 0] - yd.sum(1)).abs() <= bound_s).all(), f"{name}: sum statistics"
        assert ((s[..., 1] - (yd ** 2).sum(1)).abs() <= bound_q).all(), f"{name}: square statistics"


RB_CASES = [c for c in CASES if c[0].startswith("rb")]


@pytest.mark.parametrize("case", RB_CASES, ids=[c[0] for c in RB_CASES])
def test_resconv_engine_matches_general_engine(case):
    """bf16: the specialised resblock engine (resconv.hip) against the general implicit-GEMM
    engine on the same launch: same bf16 operands, fp32 accumulation in a different order."""
    try:
        E.set_option(E.OPT_RESCONV, 1)
        _, y1, s1 = run_case(case, "bf16")
        E.set_option(E.OPT_RESCONV, 0)
        _, y0, s0 = run_case(case, "bf16")
    finally:
        E.set_option(E.OPT_RESCONV, 1)
    scale = max(1.0, y0.abs().max().item())
    err = (y1 - y0).abs().max().item()
    assert err <= 2 ** -7 * scale, f"{case[0]}: engines differ by {err}"
    np.testing.assert_allclose(s1.numpy(), s0.numpy(), rtol=1e-4, atol=1e-2)


WIDE_CASES = [c for c in RB_CASES if c[1] in (128, 256)]


@pytest.mark.parametrize("mode", [2, 3, 4, 5])
@pytest.mark.parametrize("case", WIDE_CASES, ids=[c[0] for c in WIDE_CASES])
def test_bigconv_v2_matches_v1(case, mode):
    """bf16: the C = 128 / 256 resblock engine v2 (bigconv2.hip; mode 2 = automatic, mode 3 =
    4-wave blocks two per CU, mode 4 = 8-wave blocks, mode 5 = C = 256 on 8-wave blocks whose second half
    runs one group behind) against v1 (bigconv.hip) on the same launch:
    same bf16 operands and transform, fp32 accumulation in a different order, statistics from the
    fp32 epilogue values."""
    try:
        E.set_option(E.OPT_BIGCONV, 1)
        _, y1, s1 = run_case(case, "bf16")
        E.set_option(E.OPT_BIGCONV, mode)
        _, y2, s2 = run_case(case, "bf16")
    finally:
        E.reset_options()
    scale = max(1.0, y1.abs().max().item())
    err = (y2 - y1).abs().max().item()
    assert err <= 2 ** -7 * scale, f"{case[0]}: bigconv v2 vs v1 differ by {err}"
    np.testing.assert_allclose(s2.numpy(), s1.numpy(), rtol=1e-4, atol=1e-2)


@pytest.mark.parametrize("case", RB_CASES, ids=[c[0] for c in RB_CASES])
def test_resblock_engines_many_tiles_per_workgroup(case):
    """Persistent grids capped at 3 workgroups: every workgroup walks many tiles and crosses
    utterance boundaries (coefficient switch, statistics flush, cross-tile prefetch)."""
    ref, _, _ = run_case(case, "bf16")
    try:
        E.set_option(E.OPT_GRID_CAP, 3)
        _, y, s = run_case(case, "bf16")
    finally:
        E.set_option(E.OPT_GRID_CAP, 0)
    _, y0, s0 = run_case(case, "bf16")
    scale = max(1.0, y0.abs().max().item())
    assert (y - y0).abs().max().item() <= 2 ** -7 * scale, case[0]
    np.testing.assert_allclose(s.numpy(), s0.numpy(), rtol=1e-4, atol=1e-2)


PP_CASES = [c for c in RB_CASES if c[1] == 64] + [
    ("rb64_k11_d1_long", 64, 64, 11, 0, 1, 1, 5, 0, 9000, 3),
    ("rb64_k7_d5_long_nores", 64, 64, 7, 0, 1, 5, 15, 0, 5000, 3),
    ("rb64_k3_d3_nores", 64, 64, 3, 0, 1, 3, 3, 0, 1111, 3),
]


@pytest.mark.parametrize("cap", [0, 3])
@pytest.mark.parametrize("case", PP_CASES, ids=[c[0] for c in PP_CASES])
def test_resconv_pingpong_matches_lockstep(case, cap):
    """bf16, C = 64: the two-group ping-pong resconv kernel (STTS_OPT_RCPP = 2) against the lock-step
    kernel on the same launch (same MFMA order per tile, so equal outputs; statistics summed in another
    order); cap = 3 makes each group walk many tiles across the two utterances."""
    try:
        E.set_option(E.OPT_GRID_CAP, cap)
        E.set_option(E.OPT_RCPP, 0)
        _, y0, s0 = run_case(case, "bf16")
        E.set_option(E.OPT_RCPP, 2)
        _, y1, s1 = run_case(case, "bf16")
    finally:
        E.reset_options()
    scale = max(1.0, y0.abs().max().item())
    err = (y1 - y0).abs().max().item()
    assert err <= 2 ** -7 * scale, f"{case[0]}: ping-pong vs lock-step differ by {err}"
    np.testing.assert_allclose(s1.numpy(), s0.numpy(), rtol=1e-4, atol=1e-2)


IL_CASES = PP_CASES + [c for c in RB_CASES if c[1] == 32]


@pytest.mark.parametrize("cap", [0, 3])
@pytest.mark.parametrize("case", IL_CASES, ids=[c[0] for c in IL_CASES])
def test_resconv_interleaved_epilogue_bitwise(case, cap):
    """bf16, C = 32 / 64: the lock-step resconv kernel with tile t - 1's epilogue interleaved into tile t's MFMA loop
    (STTS_OPT_EXP bit 32768; the default for the C = 64 residual / running-sum launches, STTS_OPT_RCPP 3) against the
    same kernel without it: same tiles, same MFMA chain and per-lane statistics order, so outputs AND statistics are
    bitwise equal.  cap = 3: ranges across utterances (coefficient switch and flush one step after the tile)."""
    try:
        E.set_option(E.OPT_GRID_CAP, cap)
        E.set_option(E.OPT_RCPP, 0)
        _, y0, s0 = run_case(case, "bf16")
        E.set_option(E.OPT_EXP, 32768)
        _, y1, s1 = run_case(case, "bf16")
    finally:
        E.reset_options()
    assert torch.equal(y1, y0), (case[0], (y1 - y0).abs().max().item())
    assert torch.equal(s1, s0), case[0]


FRONT_CASES = [c for c in CASES if c[0].startswith("front")]


@pytest.mark.parametrize("cap", [0, 3])
@pytest.mark.parametrize("case", FRONT_CASES, ids=[c[0] for c in FRONT_CASES])
def test_front_engine_matches_igemm(case, cap):
    """bf16: the front-end convs on the bigconv2 engine (C_in up to 1120, 256-channel output
    parts, [AdaIN ->] LReLU prologue) against the igemm engine on the same launch; cap = 3 makes
    every workgroup walk many tiles across output parts and utterances."""
    try:
        E.set_option(E.OPT_FRONT, 0)
        _, y0, s0 = run_case(case, "bf16")
        E.set_option(E.OPT_FRONT, 2)  # the engine at any size (default 1 keeps small launches on igemm)
        E.set_option(E.OPT_GRID_CAP, cap)
        _, y1, s1 = run_case(case, "bf16")
    finally:
        E.reset_options()
    scale = max(1.0, y0.abs().max().item())
    err = (y1 - y0).abs().max().item()
    assert err <= 2 ** -7 * scale, f"{case[0]}: front engine vs igemm differ by {err}"
    np.testing.assert_allclose(s1.numpy(), s0.numpy(), rtol=1e-4, atol=1e-2)


@pytest.mark.parametrize("mode", [4, 5])
@pytest.mark.parametrize("case", WIDE_CASES, ids=[c[0] for c in WIDE_CASES])
def test_bigconv_8wave_many_tiles_per_workgroup(case, mode):
    """The 8-wave bigconv2 blocks (STTS_OPT_BIGCONV = 4; at these small sizes the automatic mode
    picks 4-wave blocks; 5: the one-group offset halves at C = 256) with the grid capped at 3 workgroups:
    long tile walks across utterances (coefficient switches, statistics flushes one slot late)."""
    try:
        E.set_option(E.OPT_BIGCONV, mode)
        _, y0, s0 = run_case(case, "bf16")
        E.set_option(E.OPT_GRID_CAP, 3)
        _, y, s = run_case(case, "bf16")
    finally:
        E.reset_options()
    scale = max(1.0, y0.abs().max().item())
    assert (y - y0).abs().max().item() <= 2 ** -7 * scale, case[0]
    np.testing.assert_allclose(s.numpy(), s0.numpy(), rtol=1e-4, atol=1e-2)


PW_CASES = [
    # 1x1 convs without statistics: the pointwise GEMM engine (pwgemm.hip, bf16)
    ("pw_sc_514_1024_nores", 514, 1024, 1, 0, 1, 1, 0, 0, 400, 0),
    ("pw_sc_1090_512_nores", 1090, 512, 1, 0, 1, 1, 0, 0, 333, 0),
    ("pw_vocos1_512_1536_nores", 512, 1536, 1, 0, 1, 1, 0, 0, 800, 1),
    ("pw_vocos2_1536_512", 1536, 512, 1, 0, 1, 1, 0, 0, 257, 0),
    ("pw_head_512_1216_nores", 512, 1216, 1, 0, 1, 1, 0, 0, 130, 0),
    ("pw_64_affine", 96, 64, 1, 0, 1, 1, 0, 0, 77, 1),
    # polyphase ConvTranspose1d upsamplers (2 taps, N = u * Cout): Snake / LReLU prologues
    ("pw_ups1_u5", 256, 128, 10, 1, 5, 1, 3, 1, 31, 2),
    ("pw_ups2_u3", 128, 64, 6, 1, 3, 1, 2, 1, 300, 2),
    ("pw_ups3_u2", 64, 32, 4, 1, 2, 1, 1, 0, 517, 2),
    ("pw_istft_ups0_lrelu", 512, 256, 20, 1, 10, 1, 5, 0, 40, 4),
]


@pytest.mark.parametrize("case", PW_CASES, ids=[c[0] for c in PW_CASES])
def test_pw_engine(case):
    """bf16 1- / 2-tap convs on the short-conv GEMM engine against torch fp32 (3 % of range, as the other
    bf16 engine cases) and against the igemm engine on the same launch (2^-7 of range), outputs and
    InstanceNorm statistics."""
    try:
        E.set_option(E.OPT_PW, 0)
        _, y0, s0 = run_case(case, "bf16")
        E.set_option(E.OPT_PW, 2)  # 2-tap launches too
        ref, y1, s1 = run_case(case, "bf16")
        _, y2, _ = run_case(case, "bf16", stats=False)
    finally:
        E.reset_options()
    scale = max(1.0, ref.abs().max().item())
    assert (y1 - ref).abs().max().item() <= 3e-2 * scale, case[0]
    assert (y1 - y0).abs().max().item() <= 2 ** -7 * scale, case[0]
    assert torch.equal(y1, y2), case[0]
    np.testing.assert_allclose(s1.numpy(), s0.numpy(), rtol=1e-3, atol=1e-1)


UPS_CASES = [c for c in CASES if c[0] in ("ups0_u10", "ups1_u5", "ups2_u3", "ups3_u2")] + [
    ("ups0_u10_long", 512, 256, 20, 1, 10, 1, 5, 0, 700, 2),
    ("ups1_u5_long", 256, 128, 10, 1, 5, 1, 3, 1, 2500, 2),
    ("ups2_u3_long", 128, 64, 6, 1, 3, 1, 2, 1, 3000, 2),
    ("ups3_u2_long", 64, 32, 4, 1, 2, 1, 1, 0, 9000, 2),
]


@pytest.mark.parametrize("cap", [0, 3])
@pytest.mark.parametrize("case", UPS_CASES, ids=[c[0] for c in UPS_CASES])
def test_ups_engine(case, cap):
    """bf16: the HiFi-GAN ups[0] / ups[1] / ups[2] polyphase upsamplers (Snake prologue, noise-branch residual) on the
    bigconv2 engine (ups[2]: 4-wave blocks of 2 output blocks x 2 frame slices of 128 frames) and ups[3] on the resconv
    engine (STTS_OPT_UPS) against torch fp32 and against the igemm engine on the same launch (same
    bf16 operands); cap = 3 makes every workgroup walk many tiles across output parts and utterances."""
    try:
        E.set_option(E.OPT_UPS, 0)
        ref, y0, s0 = run_case(case, "bf16", res_tr=True)
        E.set_option(E.OPT_UPS, 1)
        E.set_option(E.OPT_GRID_CAP, cap)
        _, y1, s1 = run_case(case, "bf16", res_tr=True)
    finally:
        E.reset_options()
    tol = 0.03 * max(1.0, ref.abs().max().item() / 4)
    assert (y1 - ref).abs().max().item() < tol, f"{case[0]}: vs torch fp32"
    scale = max(1.0, y0.abs().max().item())
    err = (y1 - y0).abs().max().item()
    assert err <= 2 ** -7 * scale, f"{case[0]}: ups engine vs igemm differ by {err}"
    # (per-channel fp32 sums over up to 1.4 M outputs, accumulated in a different order by the two engines)
    np.testing.assert_allclose(s1.numpy(), s0.numpy(), rtol=1e-3, atol=1e-1)


@pytest.mark.parametrize("cap", [0, 5])
@pytest.mark.parametrize("case", [c for c in UPS_CASES if c[0].startswith("ups2")], ids=lambda c: c[0])
def test_ups2_wave_layouts(case, cap):
    """bf16 ups[2] (N = 192 = 3 phases x 64) on bigconv2's 12-wave blocks (all three phases in one tile: each window
    DMA'd and transformed once, one statistics copy per phase and frame slice) against the 4-wave blocks of one phase
    per tile part (STTS_OPT_EXP bit 32): every output is the same MFMA chain, so the outputs are bitwise equal; the
    per-channel statistics are the same sums in another fp32 order.  cap = 5 makes workgroups walk many tiles across
    utterances."""
    try:
        E.set_option(E.OPT_GRID_CAP, cap)
        E.set_option(E.OPT_EXP, 32)
        _, y0, s0 = run_case(case, "bf16", res_tr=True)
        E.set_option(E.OPT_EXP, 0)
        _, y1, s1 = run_case(case, "bf16", res_tr=True)
    finally:
        E.reset_options()
    assert torch.equal(y1, y0), f"{case[0]}: 12-wave vs 4-wave outputs differ by {(y1 - y0).abs().max().item()}"
    np.testing.assert_allclose(s1.numpy(), s0.numpy(), rtol=1e-5, atol=1e-2)
