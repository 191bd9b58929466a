"""Conv1d forward / backward of the training step (config 5) on the HIP path vs torch autograd.

train.py:272-327 gets its conv gradients from torch autograd, so autograd (fp64 on the CPU) is the
reference algorithm here; tolerances are relative to the gradient's max magnitude: fp32 1e-4,
bf16 operands (forward, dx and dw: bf16 MFMA operands with fp32 accumulation; db stays an fp64-summed
fp32 reduction in both modes) 2e-2.  The cases are the
conv shapes of the decoder (Modules/hifigan.py) and the discriminators (discriminators.py)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

# (B, Cin, Cout, K, stride, dil, pad, Lin)
CASES = [
    (2, 64, 64, 7, 1, 3, 9, 300),        # resblock conv, dilation 3
    (1, 32, 32, 11, 1, 5, 25, 1000),     # last-stage resblock, dilation 5
    (2, 1090, 1024, 3, 1, 1, 1, 40),     # decoder front-end AdainResBlk1d conv1
    (3, 32, 1, 7, 1, 1, 3, 257),         # conv_post
    (2, 1, 1, 3, 2, 1, 1, 80),           # F0_conv / N_conv (stride 2, one channel)
    (2, 32, 128, 5, 3, 1, 2, 301),       # MPD (5, 1) conv, stride 3 along time
    (1, 512, 256, 1, 1, 1, 0, 37),       # 1x1 shortcut
    (2, 16, 48, 4, 2, 1, 1, 99),         # even kernel, stride 2, ragged length
    (1, 64, 64, 7, 1, 5, 15, 48000),     # long rows: many wgrad slices
    (20, 512, 1024, 5, 3, 1, 2, 36),     # MPD period 5 conv3 at T = 4800 (dx: output padding 2)
    (20, 128, 512, 5, 3, 1, 2, 107),     # MPD period 5 conv2
    (20, 1024, 1024, 5, 1, 1, 2, 12),    # MPD period 5 conv4 (12 rows per column)
    (6, 96, 32, 9, 2, 1, 4, 513),        # MSD (3, 9) stride-2 layer on the time-expanded image (BM 128 x BN 32)
    (5, 96, 32, 9, 2, 1, 4, 65),         # the same, short ragged rows
    (300, 3, 32, 9, 1, 1, 4, 257),       # MSD first (3, 9) layer: Cin = 3 over many rows (many wgrad slices)
]


def _ref(x, w, b, stride, pad, dil, gy):
    xd, wd, bd = (t.double().requires_grad_(True) for t in (x, w, b))
    y = torch.nn.functional.conv1d(xd, wd, bd, stride=stride, padding=pad, dilation=dil)
    y.backward(gy.double())
    return y.detach(), xd.grad, wd.grad, bd.grad


def _rel(a, ref):
    a, ref = a.detach().double().cpu(), ref.detach().double().cpu()
    return float((a - ref).abs().max() / max(ref.abs().max().item(), 1e-30))


@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
@pytest.mark.parametrize("case", CASES, ids=lambda c: "B{}_Ci{}_Co{}_K{}_s{}_d{}_p{}_L{}".format(*c))
def test_conv1d_fwd_bwd(case, dtype):
    from stts2_mi355x.training import conv1d, out_length
    B, Cin, Cout, K, stride, dil, pad, Lin = case
    g = torch.Generator().manual_seed(hash(case) % 2**31)
    x = torch.randn(B, Cin, Lin, generator=g)
    w = torch.randn(Cout, Cin, K, generator=g) / np.sqrt(Cin * K)
    b = torch.randn(Cout, generator=g)
    Lq = out_length(Lin, K, stride, pad, dil)
    gy = torch.randn(B, Cout, Lq, generator=g)
    y_ref, dx_ref, dw_ref, db_ref = _ref(x, w, b, stride, pad, dil, gy)
    xc, wc, bc = (t.cuda().requires_grad_(True) for t in (x, w, b))
    y = conv1d(xc, wc, bc, stride, pad, dil, dtype=dtype)
    assert y.shape == (B, Cout, Lq)
    y.backward(gy.cuda())
    tol = 1e-4 if dtype == "fp32" else 2e-2
    errs = {"y": _rel(y, y_ref), "dx": _rel(xc.grad, dx_ref), "dw": _rel(wc.grad, dw_ref), "db": _rel(bc.grad, db_ref)}
    print(case, dtype, {k: f"{v:.2e}" for k, v in errs.items()})
    assert errs["y"] < tol and errs["dx"] < tol
    assert errs["dw"] < (1e-4 if dtype == "fp32" else 2e-2) and errs["db"] < 1e-5  # db: fp32 in both modes


ACT_CASES = [c for c in CASES if c[2] >= 16] + [(4, 96, 32, 9, 2, 1, 4, 257)]  # + an MSD (3, 9) layer


@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
@pytest.mark.parametrize("case", ACT_CASES, ids=lambda c: "B{}_Ci{}_Co{}_K{}_s{}_d{}_p{}_L{}".format(*c))
def test_conv1d_fused_leaky_relu(case, dtype):
    """conv1d_frames(..., act_slope=0.1) (stts_conv1d_fwd_act, the activation in the conv epilogue).  fp32:
    against torch autograd (fp64) of leaky_relu(conv1d(x), 0.1).  bf16: against the unfused path on the
    same engine (conv1d_frames, then leaky_relu): the gradient mask comes from the output's sign, which the
    bf16 rounding keeps, so the gradients agree to fp32 rounding and the outputs to one bf16 rounding
    (a comparison with fp64 would flip the mask wherever the bf16 conv lands on the other side of 0)."""
    from stts2_mi355x.training import conv1d_frames, leaky_relu, out_length
    B, Cin, Cout, K, stride, dil, pad, Lin = case
    g = torch.Generator().manual_seed(hash(case) % 2**31 + 7)
    x = torch.randn(B, Lin, Cin, generator=g)
    w = torch.randn(Cout, Cin, K, generator=g) / np.sqrt(Cin * K)
    b = torch.randn(Cout, generator=g) * 0.3
    Lq = out_length(Lin, K, stride, pad, dil)
    gy = torch.randn(B, Lq, Cout, generator=g)
    if dtype == "fp32":
        xd, wd, bd = (t.double().requires_grad_(True) for t in (x, w, b))
        yr = torch.nn.functional.leaky_relu(
            torch.nn.functional.conv1d(xd.transpose(1, 2), wd, bd, stride=stride, padding=pad, dilation=dil), 0.1)
        yr = yr.transpose(1, 2)
        yr.backward(gy.double())
        ref = (yr, xd.grad, wd.grad, bd.grad)
        tol = {"y": 1e-4, "dx": 1e-4, "dw": 1e-4, "db": 1e-4}
    else:
        xr, wr, br = (t.cuda().requires_grad_(True) for t in (x, w, b))
        yr = leaky_relu(conv1d_frames(xr, wr, br, stride, pad, dil, dtype=dtype), 0.1)
        yr.backward(gy.cuda())
        ref = (yr, xr.grad, wr.grad, br.grad)
        tol = {"y": 2 ** -7, "dx": 1e-5, "dw": 1e-5, "db": 1e-5}
    xc, wc, bc = (t.cuda().requires_grad_(True) for t in (x, w, b))
    y = conv1d_frames(xc, wc, bc, stride, pad, dil, dtype=dtype, act_slope=0.1)
    y.backward(gy.cuda())
    errs = {"y": _rel(y, ref[0]), "dx": _rel(xc.grad, ref[1]), "dw": _rel(wc.grad, ref[2]), "db": _rel(bc.grad, ref[3])}
    print(case, dtype, {k: f"{v:.2e}" for k, v in errs.items()})
    for k, v in errs.items():
        assert v < tol[k], f"{k}: {v:.2e}"


def test_conv1d_bwd_deterministic_and_partial_outputs():
    """Fixed slice order: two backward passes agree bitwise; dw-only / dx-only calls give the same
    values as the full call."""
    from stts2_mi355x.training import conv1d
    g = torch.Generator().manual_seed(5)
    x = torch.randn(2, 64, 3000, generator=g).cuda()
    w = (torch.randn(64, 64, 3, generator=g) * 0.1).cuda()
    gy = torch.randn(2, 64, 3000, generator=g).cuda()
    outs = []
    for _ in range(2):
        xc, wc = x.clone().requires_grad_(True), w.clone().requires_grad_(True)
        conv1d(xc, wc, None, 1, 1, 1).backward(gy)
        outs.append((xc.grad.clone(), wc.grad.clone()))
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])
    wc = w.clone().requires_grad_(True)
    conv1d(x, wc, None, 1, 1, 1).backward(gy)  # x needs no grad: dx is not computed
    assert torch.equal(wc.grad, outs[0][1])
    xc = x.clone().requires_grad_(True)
    conv1d(xc, w, None, 1, 1, 1).backward(gy)
    assert torch.equal(xc.grad, outs[0][0])


def test_conv1d_module_dropin():
    """training.Conv1d loads an nn.Conv1d state dict and matches its forward and parameter grads."""
    from stts2_mi355x.training import Conv1d
    torch.manual_seed(3)
    ref = torch.nn.Conv1d(48, 80, 5, stride=1, padding=4, dilation=2)
    mod = Conv1d(48, 80, 5, stride=1, padding=4, dilation=2)
    mod.load_state_dict(ref.state_dict())
    x = torch.randn(2, 48, 200)
    ref(x).square().mean().backward()
    mod.cuda()
    mod(x.cuda()).square().mean().backward()
    assert _rel(mod.weight.grad, ref.weight.grad) < 1e-4
    assert _rel(mod.bias.grad, ref.bias.grad) < 1e-4


# (B, Cin, Cout, K, stride, pad, out_pad, Lin): the HiFi-GAN upsamplers (hifigan.py:292-294, u = 10, 5, 3,
# 2 over k = 20, 10, 6, 4), a ragged output_padding case and a stride-1 case
T_CASES = [
    (2, 512, 256, 20, 10, 5, 0, 40),
    (1, 256, 128, 10, 5, 3, 1, 97),
    (2, 128, 64, 6, 3, 2, 1, 300),
    (3, 64, 32, 4, 2, 1, 0, 501),
    (1, 48, 40, 5, 1, 2, 0, 77),
]


@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
@pytest.mark.parametrize("case", T_CASES, ids=lambda c: "B{}_Ci{}_Co{}_K{}_s{}_p{}_op{}_L{}".format(*c))
def test_conv_transpose1d_fwd_bwd(case, dtype):
    from stts2_mi355x.training import conv_transpose1d
    B, Cin, Cout, K, stride, pad, op, Lin = case
    g = torch.Generator().manual_seed(hash(case) % 2**31)
    x = torch.randn(B, Cin, Lin, generator=g)
    w = torch.randn(Cin, Cout, K, generator=g) / np.sqrt(Cin * K / stride)
    b = torch.randn(Cout, generator=g)
    xd_, wd_, bd_ = (t.double().requires_grad_(True) for t in (x, w, b))
    y_ref = torch.nn.functional.conv_transpose1d(xd_, wd_, bd_, stride=stride, padding=pad, output_padding=op)
    gy = torch.randn(y_ref.shape, generator=g)
    y_ref.backward(gy.double())
    xc, wc, bc = (t.cuda().requires_grad_(True) for t in (x, w, b))
    y = conv_transpose1d(xc, wc, bc, stride, pad, op, dtype=dtype)
    assert y.shape == y_ref.shape
    y.backward(gy.cuda())
    tol = 1e-4 if dtype == "fp32" else 2e-2
    errs = {"y": _rel(y, y_ref), "dx": _rel(xc.grad, xd_.grad), "dw": _rel(wc.grad, wd_.grad),
            "db": _rel(bc.grad, bd_.grad)}
    print(case, dtype, {k: f"{v:.2e}" for k, v in errs.items()})
    assert errs["y"] < tol and errs["dx"] < tol
    assert errs["dw"] < tol and errs["db"] < 1e-5


WGW_CASES = CASES  # stride 1, and the strided (2 / 3) discriminator / F0 convs on the phase-split window


@pytest.mark.parametrize("case", WGW_CASES, ids=lambda c: "B{}_Ci{}_Co{}_K{}_s{}_d{}_p{}_L{}".format(*c))
def test_wgrad_window_kernel_matches_per_tap(case):
    """bf16 dw: the all-taps window kernel (k_wgrad_bf16w, STTS_OPT_WGRAD = 1; strides 2 / 3 on a phase-split
    window) against the per-tap kernel (0) on the same inputs: the same bf16 operands, fp32 accumulation in a
    different order."""
    from stts2_mi355x import engine as E
    from stts2_mi355x.training import conv1d, out_length
    B, Cin, Cout, K, stride, dil, pad, Lin = case
    g = torch.Generator().manual_seed(7 + hash(case) % 1000)
    x = torch.randn(B, Cin, Lin, generator=g).cuda()
    w = (torch.randn(Cout, Cin, K, generator=g) / np.sqrt(Cin * K)).cuda()
    gy = torch.randn(B, Cout, out_length(Lin, K, stride, pad, dil), generator=g).cuda()
    dws = []
    try:
        for opt in (1, 0):
            E.set_option(E.OPT_WGRAD, opt)
            wc = w.clone().requires_grad_(True)
            conv1d(x, wc, None, stride, pad, dil, dtype="bf16").backward(gy)
            dws.append(wc.grad.detach().cpu().double())
    finally:
        E.reset_options()
    err = float((dws[0] - dws[1]).abs().max() / dws[1].abs().max())
    assert err < 2e-5, f"window vs per-tap dw differ by {err:.2e} of max"


PLAIN_CASES = [c for c in CASES if c[4] == 1 and c[1] == c[2] and c[1] in (32, 64)]


@pytest.mark.parametrize("case", PLAIN_CASES, ids=lambda c: "B{}_Ci{}_Co{}_K{}_s{}_d{}_p{}_L{}".format(*c))
def test_plain_resconv_matches_igemm(case):
    """bf16 forward and dx of the training step's C = 32 / 64 'same' convs: on the resconv engine with its
    transform set to the identity (STTS_OPT_PLAINRC = 1) against conv1d_igemm (0), same bf16 operands."""
    from stts2_mi355x import engine as E
    from stts2_mi355x.training import conv1d, out_length
    B, Cin, Cout, K, stride, dil, pad, Lin = case
    g = torch.Generator().manual_seed(11 + hash(case) % 1000)
    x = torch.randn(B, Cin, Lin, generator=g).cuda()
    w = (torch.randn(Cout, Cin, K, generator=g) / np.sqrt(Cin * K)).cuda()
    b = torch.randn(Cout, generator=g).cuda()
    gy = torch.randn(B, Cout, out_length(Lin, K, stride, pad, dil), generator=g).cuda()
    outs = []
    try:
        for opt in (1, 0):
            E.set_option(E.OPT_PLAINRC, opt)
            xc = x.clone().requires_grad_(True)
            y = conv1d(xc, w, b, stride, pad, dil, dtype="bf16")
            y.backward(gy)
            outs.append((y.detach().cpu().double(), xc.grad.detach().cpu().double()))
    finally:
        E.reset_options()
    for k, name in enumerate(("y", "dx")):
        a, r = outs[0][k], outs[1][k]
        err = float((a - r).abs().max() / r.abs().max())
        assert err < 2 ** -7, f"{name}: resconv vs igemm differ by {err:.2e} of max"


STRIDED_CASES = [c for c in CASES if c[4] > 1]


@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
@pytest.mark.parametrize("case", STRIDED_CASES, ids=lambda c: "B{}_Ci{}_Co{}_K{}_s{}_d{}_p{}_L{}".format(*c))
def test_folded_strided_conv_matches_engine_stride(case, dtype):
    """Strided convs as stride-1 convs over phase-folded frames (training.FOLD_STRIDED) against
    the engines' own strided path, forward and every gradient (fp32: the same sums in another order)."""
    from stts2_mi355x import training as T
    B, Cin, Cout, K, stride, dil, pad, Lin = case
    g = torch.Generator().manual_seed(3 + hash(case) % 1000)
    x = torch.randn(B, Cin, Lin, generator=g).cuda()
    w = (torch.randn(Cout, Cin, K, generator=g) / np.sqrt(Cin * K)).cuda()
    b = torch.randn(Cout, generator=g).cuda()
    gy = torch.randn(B, Cout, T.out_length(Lin, K, stride, pad, dil), generator=g).cuda()
    res = []
    try:
        for fold in (True, False):
            T.FOLD_STRIDED = fold
            xc, wc, bc = (t.clone().requires_grad_(True) for t in (x, w, b))
            y = T.conv1d(xc, wc, bc, stride, pad, dil, dtype=dtype)
            y.backward(gy)
            res.append([t.detach().double().cpu() for t in (y, xc.grad, wc.grad, bc.grad)])
    finally:
        T.FOLD_STRIDED = False
    tol = 1e-5 if dtype == "fp32" else 2e-2
    for name, a, r in zip(("y", "dx", "dw", "db"), res[0], res[1]):
        err = float((a - r).abs().max() / max(r.abs().max().item(), 1e-30))
        assert err < tol, f"{name}: folded vs strided differ by {err:.2e} of max"


@pytest.mark.parametrize("case", [c for c in CASES if c[2] % 16 == 0],
                         ids=lambda c: "B{}_Ci{}_Co{}_K{}_s{}_d{}_p{}_L{}".format(*c))
def test_bf16_fp32_output_frames(case):
    """STTS_OPT_YF32 (default on): bf16 convs on the general engine store fp32 output frames straight from the
    accumulators.  Against the bf16-output path (option off, + the conversion pass) on the same inputs: y and dx
    differ by at most the one bf16 rounding the option removes (2^-8 of the max), dw / db not at all (fp32
    weight gradients from the same x and dy); and the option's y is at least as close to fp64 as the rounded one."""
    from stts2_mi355x import engine as E
    from stts2_mi355x.training import conv1d_frames, out_length
    B, Cin, Cout, K, stride, dil, pad, Lin = case
    g = torch.Generator().manual_seed(hash(case) % 2**31 + 11)
    x = torch.randn(B, Lin, Cin, generator=g)
    w = torch.randn(Cout, Cin, K, generator=g) / np.sqrt(Cin * K)
    b = torch.randn(Cout, generator=g)
    gy = torch.randn(B, out_length(Lin, K, stride, pad, dil), Cout, generator=g)
    out = {}
    try:
        for yf in (0, 1):
            E.set_option(E.OPT_YF32, yf)
            xc, wc, bc = (t.cuda().requires_grad_(True) for t in (x, w, b))
            y = conv1d_frames(xc, wc, bc, stride, pad, dil, dtype="bf16")
            y.backward(gy.cuda())
            out[yf] = (y.detach(), xc.grad, wc.grad, bc.grad)
    finally:
        E.reset_options()
    yr = torch.nn.functional.conv1d(x.double().transpose(1, 2), w.double(), b.double(), stride=stride, padding=pad,
                                    dilation=dil).transpose(1, 2)
    errs = {k: _rel(a, r) for k, a, r in zip(("y", "dx", "dw", "db"), out[1], out[0])}
    print(case, {k: f"{v:.2e}" for k, v in errs.items()}, f"vs fp64 on {_rel(out[1][0], yr):.2e} off {_rel(out[0][0], yr):.2e}")
    assert errs["y"] <= 2 ** -8 and errs["dx"] <= 2 ** -8 and errs["dw"] == 0 and errs["db"] == 0
    assert _rel(out[1][0], yr) <= _rel(out[0][0], yr) * 1.01


@pytest.mark.parametrize("dtype", ["fp32", "bf16", "bf16x3"])
@pytest.mark.parametrize("case", [c for c in CASES if c[2] == 1] + [(8, 1024, 1, 3, 1, 1, 1, 575)],
                         ids=lambda c: "B{}_Ci{}_Co{}_K{}_s{}_d{}_p{}_L{}".format(*c))
def test_cout1_gemv_forward(case, dtype):
    """STTS_OPT_COUT1 (default on): one-output-channel forwards (conv_post, MPD conv_post 1024 -> 1, the F0 / N
    stride-2 convs) as a GEMV, against torch fp64 (fp32 / bf16x3: 1e-5 of the max; bf16: its rounded operands,
    2e-2) and against the MFMA engine (option off) in the same dtype (1e-5; bf16: one bf16 output rounding)."""
    from stts2_mi355x import engine as E
    from stts2_mi355x.training import conv1d_frames
    B, Cin, Cout, K, stride, dil, pad, Lin = case
    g = torch.Generator().manual_seed(hash(case) % 2**31 + 13)
    x = torch.randn(B, Lin, Cin, generator=g)
    w = torch.randn(Cout, Cin, K, generator=g) / np.sqrt(Cin * K)
    b = torch.randn(Cout, generator=g)
    yr = torch.nn.functional.conv1d(x.double().transpose(1, 2), w.double(), b.double(), stride=stride, padding=pad,
                                    dilation=dil).transpose(1, 2)
    ys = {}
    try:
        for on in (0, 1):
            E.set_option(E.OPT_COUT1, on)
            with torch.no_grad():
                ys[on] = conv1d_frames(x.cuda(), w.cuda(), b.cuda(), stride, pad, dil, dtype=dtype).cpu()
    finally:
        E.reset_options()
    e_ref, e_ab = _rel(ys[1], yr), _rel(ys[1], ys[0])
    print(case, dtype, f"vs fp64 {e_ref:.2e}, vs engine {e_ab:.2e}")
    assert e_ref < (2e-2 if dtype == "bf16" else 1e-5)
    assert e_ab < (2 ** -7 if dtype == "bf16" else 1e-5)
