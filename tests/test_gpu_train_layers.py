"""AdaIN1d + activation, the style Linear, weight norm and a whole AdaINResBlock1 — forward and
backward on the HIP path — against autograd through the oracle's restatement of the reference
(oracle/stts_oracle.py adain1d / snake / adain_resblock1, fp64 on the CPU).  train.py gets these
gradients from torch autograd, so autograd over the reference algorithm is the reference here.
Tolerance: max |error| <= 1e-4 (layers) / 2e-4 (the six-layer resblock) of the max |reference|."""
import os
import re
import sys

import pytest
import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))
import stts_oracle as O  # noqa: E402

pytestmark = pytest.mark.gpu


def _rel(a, ref):
    a, ref = a.detach().double().cpu(), ref.detach().double().cpu()
    return float((a - ref).abs().max() / max(ref.abs().max().item(), 1e-30))


@pytest.mark.parametrize("act", [0, 1, 2], ids=["none", "snake", "lrelu"])
@pytest.mark.parametrize("B,C,L", [(2, 64, 300), (3, 100, 77), (1, 512, 4000)])
def test_adain_act(B, C, L, act):
    from stts2_mi355x.training import adain_act
    g = torch.Generator().manual_seed(B * 1000 + C + act)
    S = 128
    x = torch.randn(B, C, L, generator=g) * 2 + 0.5
    s = torch.randn(B, S, generator=g)
    W = torch.randn(2 * C, S, generator=g) * 0.05
    bfc = torch.randn(2 * C, generator=g) * 0.1
    alpha = 0.5 + torch.rand(1, C, 1, generator=g)
    R = torch.randn(B, C, L, generator=g)
    # reference (fp64): AdaIN1d then the activation
    ref = [t.double().requires_grad_(True) for t in (x, s, W, bfc, alpha)]
    xr, sr, Wr, br, ar = ref
    z = O.adain1d(xr, sr, {"n.fc.weight": Wr, "n.fc.bias": br}, "n")
    y_ref = O.snake(z, ar) if act == 1 else (F.leaky_relu(z, 0.2) if act == 2 else z)
    (y_ref * R.double()).sum().backward()
    dev = [t.cuda().requires_grad_(True) for t in (x, s, W, bfc, alpha)]
    xd, sd, Wd, bd, ad = dev
    y = adain_act(xd.transpose(1, 2), sd, Wd, bd, ad if act == 1 else None, act).transpose(1, 2)
    (y * R.cuda()).sum().backward()
    errs = {"y": _rel(y, y_ref), "dx": _rel(xd.grad, xr.grad), "ds": _rel(sd.grad, sr.grad),
            "dW": _rel(Wd.grad, Wr.grad), "db": _rel(bd.grad, br.grad)}
    if act == 1:
        errs["dalpha"] = _rel(ad.grad, ar.grad)
    print((B, C, L, act), {k: f"{v:.1e}" for k, v in errs.items()})
    for k, v in errs.items():
        assert v < 1e-4, (k, v)


def test_weight_norm_grad():
    from stts2_mi355x.training import weight_norm
    g0 = torch.Generator().manual_seed(1)
    gg = torch.rand(96, 1, 1, generator=g0) + 0.5
    v = torch.randn(96, 64, 7, generator=g0)
    R = torch.randn(96, 64, 7, generator=g0)
    gr, vr = gg.double().requires_grad_(True), v.double().requires_grad_(True)
    (torch._weight_norm(vr, gr, 0) * R.double()).sum().backward()
    gd, vd = gg.cuda().requires_grad_(True), v.cuda().requires_grad_(True)
    w = weight_norm(gd, vd)
    (w * R.cuda()).sum().backward()
    assert _rel(w, torch._weight_norm(v.double(), gg.double(), 0)) < 1e-5
    assert _rel(gd.grad, gr.grad) < 1e-5 and _rel(vd.grad, vr.grad) < 1e-5


@pytest.mark.parametrize("C,K,L", [(64, 7, 500), (32, 11, 1200), (128, 3, 300)])
def test_adain_resblock1_fwd_bwd(C, K, L):
    """One AdaINResBlock1 (dilations 1, 3, 5) end to end: output and every gradient (x, s and all 24
    parameters) against autograd through oracle.adain_resblock1 in fp64."""
    from stts2_mi355x.training import AdaINResBlock1
    torch.manual_seed(C + K)
    B, S = 2, 128
    mod = AdaINResBlock1(C, K, (1, 3, 5), S)
    with torch.no_grad():
        for n, p in mod.named_parameters():
            if "alpha" in n:
                p.uniform_(0.6, 1.4)
            elif "weight_g" in n:
                p.uniform_(0.5, 1.5)
            elif n.endswith("bias"):
                p.normal_(0, 0.1)
            else:
                p.normal_(0, 0.05)
    x = torch.randn(B, C, L)
    s = torch.randn(B, S)
    R = torch.randn(B, C, L)
    sd = {"rb." + k: v.detach().double().requires_grad_(True) for k, v in mod.state_dict().items()}
    xr, sr = x.double().requires_grad_(True), s.double().requires_grad_(True)
    y_ref = O.adain_resblock1(xr, sr, sd, "rb", K, (1, 3, 5))
    (y_ref * R.double()).sum().backward()
    mod.cuda()
    xd, sdv = x.cuda().requires_grad_(True), s.cuda().requires_grad_(True)
    y = mod(xd, sdv)
    (y * R.cuda()).sum().backward()
    errs = {"y": _rel(y, y_ref), "dx": _rel(xd.grad, xr.grad), "ds": _rel(sdv.grad, sr.grad)}
    # convs1's output feeds adain2's InstanceNorm, which cancels a per-channel shift exactly and a
    # per-channel scale up to eps: the true gradient of convs1's bias is 0 and that of weight_g
    # nearly so, a difference of nearly equal dot products.  They are checked against their natural
    # scale instead of their own size: the bias against the largest gradient, weight_g (= <dw, v/|v|>)
    # against max |dw| = max |dv| |v| / g over the rows.
    scale = max(sd["rb." + n].grad.abs().max().item() for n, _ in mod.named_parameters())
    for n, p in mod.named_parameters():
        ref = sd["rb." + n].grad
        if re.match(r"convs1\.\d+\.bias$", n):
            assert p.grad.abs().max().item() < 1e-5 * scale, n
            continue
        if re.match(r"convs1\.\d+\.weight_g$", n):
            pre = n[: -len("weight_g")]
            v, g, dv = sd["rb." + pre + "weight_v"], sd["rb." + n], sd["rb." + pre + "weight_v"].grad
            dw_scale = (dv.flatten(1).norm(dim=1) * v.detach().flatten(1).norm(dim=1) / g.detach().flatten()).max()
            errs[n] = float((p.grad.detach().double().cpu() - ref).abs().max() / dw_scale)
            continue
        errs[n] = _rel(p.grad, ref)
    worst = max(errs, key=errs.get)
    print((C, K, L), "worst", worst, f"{errs[worst]:.2e}", "y", f"{errs['y']:.1e}", "dx", f"{errs['dx']:.1e}")
    for k, v in errs.items():
        assert v < 2e-4, (k, v)


@pytest.mark.parametrize("cin,cout,up,L", [(64, 64, False, 300), (96, 64, False, 155), (64, 32, True, 155),
                                           (1090, 512, True, 40)])
def test_adain_resblk1d_fwd_bwd(cin, cout, up, L):
    """One AdainResBlk1d (the decoder's encode / decode blocks, hifigan.py:359-403), output and every
    gradient against autograd through oracle.adain_resblk1d in fp64."""
    from stts2_mi355x.training import AdainResBlk1d
    torch.manual_seed(cin + cout + up)
    B, S = 2, 128
    mod = AdainResBlk1d(cin, cout, S, upsample=up)
    with torch.no_grad():
        for n, p in mod.named_parameters():
            if "weight_g" in n:
                p.uniform_(0.5, 1.5)
            elif n.endswith("bias"):
                p.normal_(0, 0.1)
            else:
                p.normal_(0, 0.05)
    x = torch.randn(B, cin, L)
    s = torch.randn(B, S)
    Lo = 2 * L if up else L
    R = torch.randn(B, cout, Lo)
    sd = {"blk." + k: v.detach().double().requires_grad_(True) for k, v in mod.state_dict().items()}
    xr, sr = x.double().requires_grad_(True), s.double().requires_grad_(True)
    y_ref = O.adain_resblk1d(xr, sr, sd, "blk", up, cin != cout)
    (y_ref * R.double()).sum().backward()
    mod.cuda()
    xd, sdv = x.cuda().requires_grad_(True), s.cuda().requires_grad_(True)
    y = mod(xd, sdv)
    assert y.shape == y_ref.shape
    (y * R.cuda()).sum().backward()
    errs = {"y": _rel(y, y_ref), "dx": _rel(xd.grad, xr.grad), "ds": _rel(sdv.grad, sr.grad)}
    scale = max(sd["blk." + n].grad.abs().max().item() for n, _ in mod.named_parameters())
    for n, p in mod.named_parameters():
        ref = sd["blk." + n].grad
        if n == "conv1.bias":  # feeds norm2's InstanceNorm: true gradient 0 (see the resblock test)
            assert p.grad.abs().max().item() < 1e-5 * scale, n
            continue
        if n == "conv1.weight_g":
            v, g, dv = sd["blk.conv1.weight_v"], sd["blk." + n], sd["blk.conv1.weight_v"].grad
            dw_scale = (dv.flatten(1).norm(dim=1) * v.detach().flatten(1).norm(dim=1) / g.detach().flatten()).max()
            errs[n] = float((p.grad.detach().double().cpu() - ref).abs().max() / dw_scale)
            continue
        errs[n] = _rel(p.grad, ref)
    worst = max(errs, key=errs.get)
    print((cin, cout, up, L), "worst", worst, f"{errs[worst]:.2e}", "y", f"{errs['y']:.1e}")
    for k, v in errs.items():
        assert v < 2e-4, (k, v)


@pytest.mark.parametrize("period,T", [(2, 6000), (3, 4001), (11, 3000)])
def test_discriminator_p_fwd_bwd(period, T):
    """One MPD DiscriminatorP (discriminators.py:96-129): score, the six feature maps, and the gradients
    of a loss over all of them w.r.t. the input and every parameter, against autograd through
    oracle.discriminator_p in fp64."""
    from stts2_mi355x.training import DiscriminatorP
    torch.manual_seed(period)
    mod = DiscriminatorP(period)
    with torch.no_grad():
        for n, p in mod.named_parameters():
            if "weight_g" in n:
                p.uniform_(0.5, 1.5)
            elif n.endswith("bias"):
                p.normal_(0, 0.05)
    B = 2
    x = torch.randn(B, 1, T) * 0.3
    sd = {"d." + k: v.detach().double().requires_grad_(True) for k, v in mod.state_dict().items()}
    xr = x.double().requires_grad_(True)
    score_r, fmap_r = O.discriminator_p(xr, sd, "d", period)
    Rs = [torch.randn(f.shape) for f in fmap_r]
    loss_r = sum((f * r.double()).sum() for f, r in zip(fmap_r, Rs)) + score_r.square().sum()
    loss_r.backward()
    mod.cuda()
    xd = x.cuda().requires_grad_(True)
    score, fmap = mod(xd)
    assert score.shape == score_r.shape and [f.shape for f in fmap] == [f.shape for f in fmap_r]
    loss = sum((f * r.cuda()).sum() for f, r in zip(fmap, Rs)) + score.square().sum()
    loss.backward()
    errs = {"score": _rel(score, score_r), "dx": _rel(xd.grad, xr.grad)}
    for j, (f, fr) in enumerate(zip(fmap, fmap_r)):
        errs[f"fmap{j}"] = _rel(f, fr)
    for n, p in mod.named_parameters():
        errs[n] = _rel(p.grad, sd["d." + n].grad)
    worst = max(errs, key=errs.get)
    print((period, T), "worst", worst, f"{errs[worst]:.2e}", "dx", f"{errs['dx']:.1e}")
    for k, v in errs.items():
        assert v < 2e-4, (k, v)


def test_discriminator_p_bf16_close():
    """dtype_compute='bf16' (bf16 MFMA operands in the conv forwards, dx and dw; fp32 accumulation) against
    the fp32 run: score within 3 % of its range (measured 0.8 %), input gradient within 10 % (measured
    6.1 %: bf16 rounding compounds through the six dx layers), every parameter gradient (weight_g, weight_v,
    bias of the six convs) within 10 % of its own max."""
    from stts2_mi355x.training import DiscriminatorP
    torch.manual_seed(7)
    m32 = DiscriminatorP(5).cuda()
    m16 = DiscriminatorP(5, dtype_compute="bf16").cuda()
    m16.load_state_dict(m32.state_dict())
    x = torch.randn(2, 1, 5000, device="cuda") * 0.3
    outs = []
    for m in (m32, m16):
        xd = x.clone().requires_grad_(True)
        score, fmap = m(xd)
        (score.square().sum() + sum(f.sum() for f in fmap)).backward()
        outs.append((score.detach(), xd.grad.detach(), {n: p.grad.detach() for n, p in m.named_parameters()}))
    assert _rel(outs[1][0], outs[0][0]) < 3e-2 and _rel(outs[1][1], outs[0][1]) < 1e-1
    perr = {n: _rel(outs[1][2][n], g) for n, g in outs[0][2].items()}
    worst = max(perr, key=perr.get)
    print("bf16 DiscriminatorP parameter gradients: worst", worst, f"{perr[worst]:.2e}")
    assert perr[worst] < 1e-1, (worst, perr[worst])


@pytest.mark.parametrize("dtype", ["fp32", "bf16", "bf16x3"])
@pytest.mark.parametrize("co,kw,stride,pad,act", [(32, 9, 2, 4, 0.1), (32, 3, 1, 1, 0.1), (1, 3, 1, 1, None)])
def test_msd_time_expanded_conv(dtype, co, kw, stride, pad, act):
    """SpecDiscriminator's (3, kw) Conv2d over C = 32 channels with the time expansion inside the conv's window
    loads (stts_conv1d_fwd_tx, training.FUSE_TX) against the materialised x3 + conv1d path in the same dtype
    (same products, another K order: 1e-5 of the max; bf16 1e-4, its output one bf16 ulp) and, in fp32, against
    torch's fp64 Conv2d (1e-5), output and the gradients of image (Cout = 32: stts_conv1d_bwd_tx, no x3), weight
    and bias; with frozen weights the image gradient alone, bit-identical."""
    from stts2_mi355x import training as T
    g = torch.Generator().manual_seed(co * 100 + kw + stride)
    S, H, W, C = 2, 37, 257, 32
    h = torch.randn(S, H, W, C, generator=g)
    w = torch.randn(co, C, 3, kw, generator=g) / (3 * C * kw) ** 0.5
    b = torch.randn(co, generator=g) * 0.1
    gy = torch.randn(S * H, (W + 2 * pad - kw) // stride + 1, co, generator=g)
    res = []
    for fused in (True, False):
        hd, wd, bd = (t.cuda().requires_grad_(True) for t in (h, w, b))
        if fused:
            y = T._ConvTxFn.apply(hd, wd, bd, stride, pad, dtype, act)
        else:
            x3 = T._TimeExpandFn.apply(hd)
            y = T.conv1d_frames(x3.reshape(S * H, W, 3 * C), wd.reshape(co, 3 * C, kw), bd, stride, pad, dtype=dtype,
                                act_slope=act)
        (y * gy.cuda()).sum().backward()
        res.append([t.detach().cpu() for t in (y, hd.grad, wd.grad, bd.grad)])
    # frozen weights (the G step's discriminators): d h alone
    hd = h.cuda().requires_grad_(True)
    (T._ConvTxFn.apply(hd, w.cuda(), b.cuda(), stride, pad, dtype, act) * gy.cuda()).sum().backward()
    assert torch.equal(hd.grad.cpu(), res[0][1])
    for name, a, r in zip(("y", "dh", "dw", "db"), res[0], res[1]):
        assert a.shape == r.shape, name
        # bf16 convs may store bf16 outputs (STTS_OPT_YF32 off, or an engine without fp32 output): the other K
        # order can round y or d h one bf16 ulp apart (2^-8 relative near the max, measured 3.4e-3)
        tol = 1e-2 if (dtype == "bf16" and name in ("y", "dh")) else (1e-4 if dtype == "bf16" else 1e-5)
        assert _rel(a, r) < tol, (name, _rel(a, r))
    if dtype == "fp32":
        hr, wr, br = (t.double().requires_grad_(True) for t in (h, w, b))
        yr = F.conv2d(hr.permute(0, 3, 1, 2), wr, br, stride=(1, stride), padding=(1, pad))
        if act is not None:
            yr = F.leaky_relu(yr, act)
        yr = yr.permute(0, 2, 3, 1).reshape(S * H, -1, co)
        (yr * gy.double()).sum().backward()
        for name, a, r in zip(("y", "dh", "dw", "db"), res[0], (yr, hr.grad, wr.grad, br.grad)):
            assert _rel(a, r) < 1e-5, (name, _rel(a, r))
