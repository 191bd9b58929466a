"""Training-step layers on the HIP path: conv1d, AdaIN1d + Snake /
LeakyReLU, the style Linear, weight norm, and the AdaINResBlock1 built from them, each a
`torch.autograd.Function` whose forward and backward both run as HIP kernels behind the C-ABI.

train.py:272-327 backpropagates the discriminator and generator losses through every nn.Conv1d of
the decoder (Modules/hifigan.py) and the discriminators (Modules/discriminators.py).  `conv1d` is
that layer as a `torch.autograd.Function` over the C-ABI: forward = `stts_conv1d_fwd` (the conv
engine), backward = `stts_conv1d_bwd` (dx on the conv engine as the transposed conv of dy; dw and
db as fp32 MFMA row-slice sums reduced in fixed order).  `Conv1d` is the drop-in nn.Conv1d
(groups = 1, padding_mode 'zeros') whose forward and backward both run there.

Torch tensors are [B, C, L]; the kernels take frames [B][L][C], so the wrapper transposes at the
boundary (plumbing, not compute).
"""
from __future__ import annotations

import ctypes
import math

import torch
from torch import nn

from .engine import _ptr, _require_device, _stream, check, lib

# bf16x3: the split-operand mode (fp32 frames, forward / dx operands as bf16 hi + lo, three MFMAs; dw in fp32)
_DT = {"fp32": 0, "bf16": 1, "bf16x3": 2}
_TRAIN_READY = False
# algorithmic conv work of the autograd path (measurement: tools/bench_train_step.py): 2 B Lq Cout Cin K flops per
# conv forward, the same again per dx and per dw (the transposed conv: 2 B Lin Cin Cout K)
CONV_FLOPS = {"on": False, "fwd": 0.0, "bwd": 0.0}


def _count(kind, flops):
    if CONV_FLOPS["on"]:
        CONV_FLOPS[kind] += flops


def _tl():
    """lib() with the argument types of the training-step entry points (include/stts2_train.h)."""
    global _TRAIN_READY
    L = lib()
    if _TRAIN_READY:
        return L
    vp, i, ll, f, d, ull = (ctypes.c_void_p, ctypes.c_int, ctypes.c_longlong, ctypes.c_float, ctypes.c_double,
                           ctypes.c_ulonglong)
    sig = {
        "stts_snake_workspace_bytes": ([i, i, i], ll),
        "stts_snake_fwd": ([vp, vp, i, i, i, vp, vp], i),
        "stts_snake_bwd": ([vp, vp, vp, i, i, i, vp, vp, vp, ll, vp], i),
        "stts_tanh_fwd": ([vp, ll, vp, vp], i),
        "stts_tanh_bwd": ([vp, vp, ll, vp, vp], i),
        "stts_sum_div": ([vp, i, ll, f, vp, vp], i),
        "stts_div": ([vp, ll, f, vp, vp], i),
        "stts_source_workspace_bytes": ([i, i], ll),
        "stts_source_fwd": ([vp, vp, vp, vp, ull, ll, i, i, i, vp, vp, vp, ll, vp], i),
        "stts_source_bwd": ([vp, vp, vp, i, ll, vp, vp, vp, ll, vp], i),
        "stts_box_smooth_fwd": ([vp, i, i, i, vp, vp], i),
        "stts_box_smooth_bwd": ([vp, i, i, i, vp, vp], i),
        "stts_time_expand3": ([vp, i, i, i, i, vp, vp], i),
        "stts_time_expand3_bwd": ([vp, i, i, i, i, vp, vp], i),
        "stts_stft_mag_workspace_bytes": ([i, ll, i, i, i], ll),
        "stts_stft_mag_fwd": ([vp, i, ll, ll, i, i, i, vp, vp, vp], i),
        "stts_stft_mag_bwd": ([vp, vp, i, ll, i, i, i, vp, vp, ll, vp], i),
        "stts_mrstft_bwd_workspace_bytes": ([i, ll, vp, vp, vp, i, i], ll),
        "stts_mrstft_loss_bwd": ([vp, vp, i, ll, ll, vp, vp, vp, i, i, i, vp, vp, vp, ll, vp], i),
        "stts_gan_workspace_bytes": ([i], ll),
        "stts_gan_loss": ([vp, i, vp, vp, ll, vp], i),
        "stts_gan_loss_bwd": ([vp, vp, vp, i, vp, vp, ll, vp], i),
        "stts_adamw_step": ([vp, i, d, d, d, d, d, ll, vp], i),
        "stts_adamw_step_dev": ([vp, i, d, d, d, d, d, vp, vp], i),
        "stts_source_fwd_seed_dev": ([vp, vp, vp, vp, vp, ll, i, i, i, vp, vp, vp, ll, vp], i),
        "stts_bilstm_workspace_bytes": ([i, i, i], ll),
        "stts_bilstm_fwd_train": ([vp, ll, ll, ll, i, i, i, vp, vp, i, vp, vp, vp, ll, vp], i),
        "stts_bilstm_bwd_workspace_bytes": ([i, i, i, i], ll),
        "stts_bilstm_bwd": ([vp, i, i, i, vp, vp, i, vp, vp, vp, vp, vp, vp, ll, vp], i),
        "stts_dropout": ([vp, ll, f, ull, vp, vp], i),
        "stts_dropout_mask": ([vp, vp, ll, f, vp, vp], i),
        "stts_rowexp_fwd": ([vp, i, i, i, i, i, i, vp, vp], i),
        "stts_rowexp_bwd": ([vp, i, i, i, i, i, i, vp, vp], i),
        "stts_dwconv2d_s2_fwd": ([vp, vp, vp, i, i, i, i, vp, vp], i),
        "stts_dwconv2d_s2_workspace_bytes": ([i], ll),
        "stts_dwconv2d_s2_bwd": ([vp, vp, vp, i, i, i, i, vp, vp, vp, vp, ll, vp], i),
        "stts_avgpool2_fwd": ([vp, i, i, i, i, vp, vp], i),
        "stts_avgpool2_bwd": ([vp, i, i, i, i, vp, vp], i),
        "stts_spatial_mean_fwd": ([vp, i, i, i, vp, vp], i),
        "stts_spatial_mean_bwd": ([vp, i, i, i, vp, vp], i),
        "stts_smooth_l1_loss": ([vp, vp, ll, vp, vp], i),
        "stts_smooth_l1_loss_bwd": ([vp, vp, ll, vp, vp, vp, vp], i),
    }
    for name, (args, res) in sig.items():
        fn = getattr(L, name)
        fn.argtypes, fn.restype = args, res
    _TRAIN_READY = True
    return L


def _ws(nbytes: int, device) -> torch.Tensor:
    return torch.empty(max(int(nbytes), 1), dtype=torch.uint8, device=device)


def out_length(Lin: int, K: int, stride: int, pad: int, dil: int) -> int:
    return (Lin + 2 * pad - dil * (K - 1) - 1) // stride + 1


class _Conv1dFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, bias, stride, pad, dil, dtype, res=None, scale=1.0, act=None):
        """x: frames [B, Lin, Cin] -> y frames [B, Lq, Cout] (+ res, fp32 frames [B, Lq, Cout]);
        act = a leaky-ReLU slope applied in the conv epilogue (stts_conv1d_fwd_act), or None"""
        _require_device()
        B, Lin, Cin = x.shape
        Cout, Cin_w, K = w.shape
        if Cin_w != Cin:
            raise ValueError(f"weight {tuple(w.shape)} does not take {Cin} input channels")
        Lq = out_length(Lin, K, stride, pad, dil)
        dt = _DT[dtype]
        xf = x.detach().to(torch.float32).contiguous()
        wc = w.detach().to(torch.float32).contiguous()
        bc = bias.detach().to(torch.float32).contiguous() if bias is not None else None
        nb = lib().stts_conv1d_fwd_workspace_bytes(dt, B, Lin, Cin, Cout, K, stride, dil, pad, Lq)
        check(int(nb) if nb < 0 else 0, "stts_conv1d_fwd_workspace_bytes")
        ws = _ws(nb, x.device)
        y = torch.empty(B, Lq, Cout, dtype=torch.float32, device=x.device)
        ctx.scale = float(scale)
        ctx.act = act
        if act is not None:
            if res is not None or scale != 1.0:
                raise ValueError("conv1d_frames: the fused leaky ReLU takes no residual / scale")
            check(lib().stts_conv1d_fwd_act(dt, _ptr(xf), _ptr(wc), _ptr(bc), B, Lin, Cin, Cout, K, stride, dil, pad,
                                            Lq, ctypes.c_float(act), _ptr(y), _ptr(ws), int(nb), _stream()),
                  "stts_conv1d_fwd_act")
        elif res is not None and dt != 0:
            # the residual epilogue of stts_conv1d_fwd_res is fp32-only: bf16 runs add it in a second pass
            check(lib().stts_conv1d_fwd(dt, _ptr(xf), _ptr(wc), _ptr(bc), B, Lin, Cin, Cout, K, stride, dil, pad, Lq,
                                        _ptr(y), _ptr(ws), int(nb), _stream()), "stts_conv1d_fwd")
            rc = res.detach().to(torch.float32).contiguous()
            xs = (ctypes.c_void_p * 2)(y.data_ptr(), rc.data_ptr())
            check(_tl().stts_sum_div(xs, 2, y.numel(), ctypes.c_float(1.0 / scale), _ptr(y), _stream()),
                  "stts_sum_div")
        elif res is not None or scale != 1.0:
            rc = res.detach().to(torch.float32).contiguous() if res is not None else None
            check(lib().stts_conv1d_fwd_res(dt, _ptr(xf), _ptr(wc), _ptr(bc), _ptr(rc), ctypes.c_float(scale), B, Lin,
                                            Cin, Cout, K, stride,
                                            dil, pad, Lq, _ptr(y), _ptr(ws), int(nb), _stream()),
                  "stts_conv1d_fwd_res")
        else:
            check(lib().stts_conv1d_fwd(dt, _ptr(xf), _ptr(wc), _ptr(bc), B, Lin, Cin, Cout, K, stride, dil, pad, Lq,
                                        _ptr(y), _ptr(ws), int(nb), _stream()), "stts_conv1d_fwd")
        ctx.save_for_backward(xf, wc, y if act is not None else None)
        ctx.geo = (B, Lin, Cin, Cout, K, stride, dil, pad, Lq, dt, bias is not None)
        _count("fwd", 2.0 * B * Lq * Cout * Cin * K)
        return y

    @staticmethod
    def backward(ctx, gy):
        xf, wc, ya = ctx.saved_tensors
        B, Lin, Cin, Cout, K, stride, dil, pad, Lq, dt, has_bias = ctx.geo
        need_x, need_w, need_b = ctx.needs_input_grad[:3]
        if ctx.scale != 1.0:
            gy = gy * ctx.scale
        dyf = gy.detach().to(torch.float32).contiguous()
        if ctx.act is not None:  # through the fused leaky ReLU, on its output (the slope keeps the sign)
            dpre = torch.empty_like(dyf)
            check(lib().stts_leaky_relu_bwd(_ptr(ya), _ptr(dyf), ya.numel(), ctypes.c_float(ctx.act), _ptr(dpre),
                                            _stream()), "stts_leaky_relu_bwd")
            dyf = dpre
        dev = dyf.device
        nb = lib().stts_conv1d_bwd_workspace_bytes(dt, B, Lin, Cin, Cout, K, stride, dil, pad, Lq)
        check(int(nb) if nb < 0 else 0, "stts_conv1d_bwd_workspace_bytes")
        ws = _ws(nb, dev)
        dx = torch.empty(B, Lin, Cin, dtype=torch.float32, device=dev) if need_x else None
        dw = torch.empty(Cout, Cin, K, dtype=torch.float32, device=dev) if need_w else None
        db = torch.empty(Cout, dtype=torch.float32, device=dev) if (need_b and has_bias) else None
        check(lib().stts_conv1d_bwd(dt, _ptr(xf), _ptr(wc), _ptr(dyf), B, Lin, Cin, Cout, K, stride, dil, pad, Lq,
                                    _ptr(dx), _ptr(dw), _ptr(db), _ptr(ws), int(nb), _stream()), "stts_conv1d_bwd")
        _count("bwd", 2.0 * B * Lq * Cout * Cin * K * ((dx is not None) + (dw is not None)))
        return dx, dw, db, None, None, None, None, (gy if ctx.needs_input_grad[7] else None), None, None


def conv1d(x, weight, bias=None, stride=1, padding=0, dilation=1, dtype="fp32"):
    """torch.nn.functional.conv1d (groups 1, zero padding) with forward and backward on the HIP
    conv engines.  dtype 'bf16' runs the forward and dx with bf16 operands (fp32 accumulation);
    dw / db are always fp32."""
    if dtype not in _DT:
        raise ValueError(f"dtype {dtype!r}: expected one of {list(_DT)}")
    return conv1d_frames(x.transpose(1, 2), weight, bias, stride, padding, dilation, dtype).transpose(1, 2)


# True: stride-2 convs run as stride-1 convs over phase-folded frames (see _fold_strided).  Off by default:
# on the config-5 step it measured slower (103.9 vs 99.3 ms, profiles/r03_bench_train_fold_ab.txt): the
# folded dx has 192 output channels and the per-call weight gather adds launches.  Tests compare both paths.
FOLD_STRIDED = False
# the discriminators' conv -> leaky_relu(0.1) pairs as one launch (stts_conv1d_fwd_act); False = separate passes
FUSE_LRELU = True
_FOLD_MAPS = {}


def _fold_map(K, stride, pad):
    """(K', pad', [(phase, k', t)]) of the stride-1 conv equivalent to a stride-`stride` one: input row
    stride q + t - pad = stride (q + s') + ph, k' = s' - s'_min."""
    key = (K, stride, pad)
    if key not in _FOLD_MAPS:
        js = [t - pad for t in range(K)]
        smin, smax = min(j // stride for j in js), max(j // stride for j in js)
        _FOLD_MAPS[key] = (smax - smin + 1, -smin, [(j % stride, j // stride - smin, t) for t, j in enumerate(js)])
    return _FOLD_MAPS[key]


def _fold_strided(x, weight, stride, padding):
    """A Conv1d(stride s, dilation 1) y[q] = sum_t w[t] x[s q + t - pad] is the stride-1 conv
    y[q] = sum_k' w'[k'] x'[q + k' - pad'] over the frames x'[m] = (x[s m], x[s m + 1], ..., x[s m + s - 1])
    (a free view of the contiguous frames [B, L, C] as [B, L / s, s C], rows padded to a multiple of s),
    with w'[k'][(ph, ci)] = w[t] where s (k' - pad') + ph = t - pad (zero elsewhere).  So the MSD / MPD
    strided convs run on the stride-1 engines (full MFMA columns at N = 32, stride-1 dx and dw) instead of the
    strided igemm tile (64 rows x 128 columns).  Autograd goes through the view and the weight gather."""
    B, Lin, Cin = x.shape
    Cout, _, K = weight.shape
    K2, pad2, taps = _fold_map(K, stride, padding)
    L2 = -(-Lin // stride)
    if L2 * stride != Lin:
        x = torch.nn.functional.pad(x, (0, 0, 0, L2 * stride - Lin))
    x2 = x.reshape(B, L2, stride * Cin)
    w2 = weight.new_zeros(Cout, stride, Cin, K2)
    for ph, k2, t in taps:
        w2[:, ph, :, k2] = weight[:, :, t]
    return x2, w2.reshape(Cout, stride * Cin, K2), pad2


def conv1d_frames(x, weight, bias=None, stride=1, padding=0, dilation=1, dtype="fp32", residual=None, scale=1.0,
                  act_slope=None):
    """conv1d on frames tensors: x [B, Lin, Cin] -> [B, Lq, Cout] (the kernels' native layout);
    `residual` (frames [B, Lq, Cout], fp32 runs) is added and the sum multiplied by `scale` in the
    conv epilogue; `act_slope`: leaky_relu(., act_slope) applied in the epilogue instead (FUSE_LRELU)."""
    if dtype not in _DT:
        raise ValueError(f"dtype {dtype!r}: expected one of {list(_DT)}")
    if residual is None and scale != 1.0:
        raise ValueError("conv1d_frames: `scale` applies to the residual sum; pass a residual or scale 1")
    stride, padding, dilation = int(stride), int(padding), int(dilation)
    if FOLD_STRIDED and stride == 2 and dilation == 1 and residual is None:
        Lq = out_length(x.shape[1], weight.shape[-1], stride, padding, 1)
        x2, w2, pad2 = _fold_strided(x, weight, stride, padding)
        y = _Conv1dFn.apply(x2, w2, bias, 1, pad2, 1, dtype, None, 1.0, act_slope)
        return y[:, :Lq] if y.shape[1] != Lq else y
    return _Conv1dFn.apply(x, weight, bias, stride, padding, dilation, dtype, residual, float(scale), act_slope)


class Conv1d(nn.Conv1d):
    """nn.Conv1d drop-in (same parameters and state dict) computing on the HIP path."""

    def __init__(self, *args, dtype_compute: str = "fp32", **kw):
        super().__init__(*args, **kw)
        if self.groups != 1 or self.padding_mode != "zeros" or isinstance(self.padding, str):
            raise NotImplementedError("HIP Conv1d: groups 1, integer zero padding")
        self.dtype_compute = dtype_compute

    def forward(self, x):
        return conv1d(x, self.weight, self.bias, self.stride[0], self.padding[0], self.dilation[0],
                      self.dtype_compute)


class _ConvT1dFn(torch.autograd.Function):
    """ConvTranspose1d on frames: x [B, Lin, Cin] -> [B, Lout, Cout], w [Cin, Cout, K]."""

    @staticmethod
    def forward(ctx, x, w, bias, stride, pad, out_pad, dtype):
        _require_device()
        B, Lin, Cin = x.shape
        Cin_w, Cout, K = w.shape
        if Cin_w != Cin:
            raise ValueError(f"weight {tuple(w.shape)} does not take {Cin} input channels")
        Lout = (Lin - 1) * stride - 2 * pad + K + out_pad
        dt = _DT[dtype]
        xf, wc, bc = _c(x), _c(w), _c(bias)
        nb = lib().stts_conv_transpose1d_workspace_bytes(dt, B, Lin, Cin, Cout, K, stride, pad, Lout)
        check(int(nb) if nb < 0 else 0, "stts_conv_transpose1d_workspace_bytes")
        ws = _ws(nb, x.device)
        y = torch.empty(B, Lout, Cout, dtype=torch.float32, device=x.device)
        check(lib().stts_conv_transpose1d_fwd(dt, _ptr(xf), _ptr(wc), _ptr(bc), B, Lin, Cin, Cout, K, stride, pad,
                                              Lout, _ptr(y), _ptr(ws), int(nb), _stream()),
              "stts_conv_transpose1d_fwd")
        ctx.save_for_backward(xf, wc)
        ctx.geo = (B, Lin, Cin, Cout, K, stride, pad, Lout, dt, bias is not None)
        _count("fwd", 2.0 * B * Lin * Cin * Cout * K)
        return y

    @staticmethod
    def backward(ctx, gy):
        xf, wc = ctx.saved_tensors
        B, Lin, Cin, Cout, K, stride, pad, Lout, dt, has_bias = ctx.geo
        nx, nw, nbias = ctx.needs_input_grad[:3]
        dy = _c(gy)
        nb = lib().stts_conv_transpose1d_workspace_bytes(dt, B, Lin, Cin, Cout, K, stride, pad, Lout)
        ws = _ws(nb, dy.device)
        dx = torch.empty_like(xf) if nx else None
        dw = torch.empty_like(wc) if nw else None
        db = torch.empty(Cout, dtype=torch.float32, device=dy.device) if (nbias and has_bias) else None
        check(lib().stts_conv_transpose1d_bwd(dt, _ptr(xf), _ptr(wc), _ptr(dy), B, Lin, Cin, Cout, K, stride, pad,
                                              Lout, _ptr(dx), _ptr(dw), _ptr(db), _ptr(ws), int(nb), _stream()),
              "stts_conv_transpose1d_bwd")
        _count("bwd", 2.0 * B * Lin * Cin * Cout * K * ((dx is not None) + (dw is not None)))
        return dx, dw, db, None, None, None, None


def conv_transpose1d_frames(x, weight, bias=None, stride=1, padding=0, output_padding=0, dtype="fp32"):
    """F.conv_transpose1d (groups 1, dilation 1) on frames [B, Lin, Cin] -> [B, Lout, Cout]."""
    if dtype not in _DT:
        raise ValueError(f"dtype {dtype!r}: expected one of {list(_DT)}")
    return _ConvT1dFn.apply(x, weight, bias, int(stride), int(padding), int(output_padding), dtype)


def conv_transpose1d(x, weight, bias=None, stride=1, padding=0, output_padding=0, dtype="fp32"):
    """F.conv_transpose1d on [B, C, L] tensors with forward and backward on the HIP path."""
    return conv_transpose1d_frames(x.transpose(1, 2), weight, bias, stride, padding, output_padding,
                                   dtype).transpose(1, 2)


ACT_NONE, ACT_SNAKE, ACT_LRELU = 0, 1, 2


def _c(t):
    return t.detach().to(torch.float32).contiguous() if t is not None else None


class _LinearFn(torch.autograd.Function):
    """nn.Linear on the device (stts_linear_fwd / stts_linear_bwd): s [B, K], W [N, K] -> [B, N]."""

    @staticmethod
    def forward(ctx, s, W, b):
        _require_device()
        B, K = s.shape
        N = W.shape[0]
        sc, Wc, bc = _c(s), _c(W), _c(b)
        h = torch.empty(B, N, dtype=torch.float32, device=s.device)
        check(lib().stts_linear_fwd(_ptr(sc), _ptr(Wc), _ptr(bc), B, K, N, _ptr(h), _stream()), "stts_linear_fwd")
        ctx.save_for_backward(sc, Wc)
        ctx.has_b = b is not None
        return h

    @staticmethod
    def backward(ctx, dh):
        sc, Wc = ctx.saved_tensors
        B, K = sc.shape
        N = Wc.shape[0]
        dh = _c(dh)
        ns, nw, nb = ctx.needs_input_grad
        ds = torch.empty_like(sc) if ns else None
        dW = torch.empty_like(Wc) if nw else None
        db = torch.empty(N, dtype=torch.float32, device=dh.device) if (nb and ctx.has_b) else None
        check(lib().stts_linear_bwd(_ptr(sc), _ptr(Wc), _ptr(dh), B, K, N, _ptr(ds), _ptr(dW), _ptr(db), _stream()),
              "stts_linear_bwd")
        return ds, dW, db


class _AdaINActFn(torch.autograd.Function):
    """AdaIN1d (InstanceNorm + (1 + gamma), beta) + activation on frames [B, L, C]; gb [B, 2C]."""

    @staticmethod
    def forward(ctx, x, gb, alpha, act):
        _require_device()
        B, L, C = x.shape
        xc, gbc, ac = _c(x), _c(gb), _c(alpha.reshape(-1)) if alpha is not None else None
        nb = lib().stts_adain_act_workspace_bytes(B, L, C)
        check(int(nb) if nb < 0 else 0, "stts_adain_act_workspace_bytes")
        ws = _ws(nb, x.device)
        y = torch.empty_like(xc)
        mr = torch.empty(B, C, 2, dtype=torch.float32, device=x.device)
        check(lib().stts_adain_act_fwd(_ptr(xc), _ptr(gbc), _ptr(ac), act, B, L, C, _ptr(y), _ptr(mr), _ptr(ws),
                                       int(nb), _stream()), "stts_adain_act_fwd")
        ctx.save_for_backward(xc, gbc, ac if ac is not None else xc.new_empty(0), mr)
        ctx.act, ctx.alpha_shape = act, (alpha.shape if alpha is not None else None)
        return y

    @staticmethod
    def backward(ctx, dy):
        xc, gbc, ac, mr = ctx.saved_tensors
        act = ctx.act
        B, L, C = xc.shape
        dy = _c(dy)
        nx, ngb, na = ctx.needs_input_grad[:3]
        nb = lib().stts_adain_act_workspace_bytes(B, L, C)
        ws = _ws(nb, dy.device)
        dx = torch.empty_like(xc) if nx else None
        dgb = torch.empty_like(gbc) if ngb else None
        da = torch.empty(C, dtype=torch.float32, device=dy.device) if (na and act == ACT_SNAKE) else None
        check(lib().stts_adain_act_bwd(_ptr(xc), _ptr(gbc), _ptr(ac if act == ACT_SNAKE else None), act, _ptr(mr),
                                       _ptr(dy), B, L, C, _ptr(dx), _ptr(dgb), _ptr(da), _ptr(ws), int(nb),
                                       _stream()), "stts_adain_act_bwd")
        return dx, dgb, (da.reshape(ctx.alpha_shape) if da is not None else None), None


class _WeightNormFn(torch.autograd.Function):
    """w = g v / ||v|| (norm over all dims but 0): stts_weight_norm / stts_weight_norm_bwd."""

    @staticmethod
    def forward(ctx, g, v):
        _require_device()
        gc, vc = _c(g), _c(v)
        d0 = vc.shape[0]
        w = torch.empty_like(vc)
        check(lib().stts_weight_norm(_ptr(gc), _ptr(vc), d0, vc.numel() // d0, _ptr(w), _stream()),
              "stts_weight_norm")
        ctx.save_for_backward(gc, vc)
        ctx.g_shape = g.shape
        return w

    @staticmethod
    def backward(ctx, dw):
        gc, vc = ctx.saved_tensors
        d0 = vc.shape[0]
        dw = _c(dw)
        dg = torch.empty(d0, dtype=torch.float32, device=dw.device)
        dv = torch.empty_like(vc)
        check(lib().stts_weight_norm_bwd(_ptr(gc), _ptr(vc), _ptr(dw), d0, vc.numel() // d0, _ptr(dg), _ptr(dv),
                                         _stream()), "stts_weight_norm_bwd")
        return dg.reshape(ctx.g_shape), dv


def linear(s, W, b=None):
    return _LinearFn.apply(s, W, b)


def adain_act(x, s, fc_weight, fc_bias, alpha=None, act=ACT_NONE):
    """AdaIN1d(style) on frames x [B, L, C] followed by `act` (Snake needs alpha [C] or [1, C, 1])."""
    return _AdaINActFn.apply(x, linear(s, fc_weight, fc_bias), alpha, int(act))


def weight_norm(g, v):
    return _WeightNormFn.apply(g, v)


class _WNConv(nn.Module):
    """weight_norm(nn.Conv1d) parameter layout (weight_g [Cout, 1, 1], weight_v, bias)."""

    def __init__(self, cin, cout, k, dilation=1, padding=0):
        super().__init__()
        self.weight_g = nn.Parameter(torch.ones(cout, 1, 1))
        self.weight_v = nn.Parameter(torch.randn(cout, cin, k) * 0.02)
        self.bias = nn.Parameter(torch.zeros(cout))
        self.dilation, self.padding = dilation, padding


class _AdaIN(nn.Module):
    def __init__(self, style_dim, C):
        super().__init__()
        self.fc = nn.Linear(style_dim, 2 * C)


class AdaINResBlock1(nn.Module):
    """Trainable Modules/hifigan.py:26-80 AdaINResBlock1 (same parameter names: convs1/convs2 weight-normed,
    adain1/adain2 .fc, alpha1/alpha2), forward and backward on the HIP kernels:
    for each dilation d: xt = Snake(AdaIN1(x)); xt = convs1(xt); xt = Snake(AdaIN2(xt)); xt = convs2(xt);
    x = xt + x.  `forward(x, s)` takes x [B, C, L]; `forward_frames(x, s)` frames [B, L, C]."""

    def __init__(self, channels, kernel_size=3, dilation=(1, 3, 5), style_dim=64):
        super().__init__()
        self.kernel_size, self.dilation = kernel_size, tuple(dilation)
        self.convs1 = nn.ModuleList([_WNConv(channels, channels, kernel_size, d, (kernel_size * d - d) // 2)
                                     for d in dilation])
        self.convs2 = nn.ModuleList([_WNConv(channels, channels, kernel_size, 1, (kernel_size - 1) // 2)
                                     for _ in dilation])
        self.adain1 = nn.ModuleList([_AdaIN(style_dim, channels) for _ in dilation])
        self.adain2 = nn.ModuleList([_AdaIN(style_dim, channels) for _ in dilation])
        self.alpha1 = nn.ParameterList([nn.Parameter(torch.ones(1, channels, 1)) for _ in dilation])
        self.alpha2 = nn.ParameterList([nn.Parameter(torch.ones(1, channels, 1)) for _ in dilation])

    def forward_frames(self, x, s):
        return resblock1_frames(self, x, s)

    def forward(self, x, s):
        return self.forward_frames(x.transpose(1, 2), s).transpose(1, 2)


def resblock1_frames(m, x, s, dtype="fp32"):
    """AdaINResBlock1.forward (hifigan.py:65-74) on frames x [B, L, C] for any module with the reference's
    parameter layout (training.AdaINResBlock1 or the decoder's params.AdaINResBlock1):
    for each dilation: xt = Snake(AdaIN1(x)); xt = convs1(xt); xt = Snake(AdaIN2(xt)); x = convs2(xt) + x."""
    for c1, c2, n1, n2, a1, a2 in zip(m.convs1, m.convs2, m.adain1, m.adain2, m.alpha1, m.alpha2):
        xt = adain_act(x, s, n1.fc.weight, n1.fc.bias, a1, ACT_SNAKE)
        xt = conv1d_frames(xt, weight_norm(c1.weight_g, c1.weight_v), c1.bias, 1, c1.padding, c1.dilation, dtype)
        xt = adain_act(xt, s, n2.fc.weight, n2.fc.bias, a2, ACT_SNAKE)
        x = conv1d_frames(xt, weight_norm(c2.weight_g, c2.weight_v), c2.bias, 1, c2.padding, c2.dilation, dtype,
                          residual=x)  # x = xt + x in convs2's epilogue
    return x


class _PoolFn(torch.autograd.Function):
    """AdainResBlk1d.pool: depthwise ConvTranspose1d(C, C, 3, 2, 1, output_padding 1) on frames."""

    @staticmethod
    def forward(ctx, x, w, bias):
        _require_device()
        B, Lin, C = x.shape
        xc, wc, bc = _c(x), _c(w).reshape(C, 3), _c(bias)
        y = torch.empty(B, 2 * Lin, C, dtype=torch.float32, device=x.device)
        check(lib().stts_pool_fwd(_ptr(xc), _ptr(wc), _ptr(bc), B, Lin, C, _ptr(y), _stream()), "stts_pool_fwd")
        ctx.save_for_backward(xc, wc)
        ctx.w_shape, ctx.has_b = w.shape, bias is not None
        return y

    @staticmethod
    def backward(ctx, gy):
        xc, wc = ctx.saved_tensors
        B, Lin, C = xc.shape
        dy = _c(gy)
        nx, nw, nb_ = ctx.needs_input_grad
        dx = torch.empty_like(xc) if nx else None
        dw = torch.empty(C, 3, dtype=torch.float32, device=dy.device) if nw else None
        db = torch.empty(C, dtype=torch.float32, device=dy.device) if (nb_ and ctx.has_b) else None
        nb = lib().stts_pool_workspace_bytes(B, Lin, C)
        ws = _ws(nb, dy.device)
        check(lib().stts_pool_bwd(_ptr(xc), _ptr(wc), _ptr(dy), B, Lin, C, _ptr(dx), _ptr(dw), _ptr(db), _ptr(ws),
                                  int(nb), _stream()), "stts_pool_bwd")
        return dx, (dw.reshape(ctx.w_shape) if dw is not None else None), db


class _Up2Fn(torch.autograd.Function):
    """nearest x2 upsample of frames (UpSample1d 'half')."""

    @staticmethod
    def forward(ctx, x):
        _require_device()
        B, Lin, C = x.shape
        xc = _c(x)
        y = torch.empty(B, 2 * Lin, C, dtype=torch.float32, device=x.device)
        check(lib().stts_upsample2(_ptr(xc), B, Lin, C, _ptr(y), _stream()), "stts_upsample2")
        ctx.shape = (B, Lin, C)
        return y

    @staticmethod
    def backward(ctx, gy):
        B, Lin, C = ctx.shape
        dy = _c(gy)
        dx = torch.empty(B, Lin, C, dtype=torch.float32, device=dy.device)
        check(lib().stts_upsample2_bwd(_ptr(dy), B, Lin, C, _ptr(dx), _stream()), "stts_upsample2_bwd")
        return dx


class _WNConvT(nn.Module):
    """weight_norm(nn.ConvTranspose1d(C, C, 3, groups=C)) parameter layout (AdainResBlk1d.pool)."""

    def __init__(self, C):
        super().__init__()
        self.weight_g = nn.Parameter(torch.ones(C, 1, 1))
        self.weight_v = nn.Parameter(torch.randn(C, 1, 3) * 0.3)
        self.bias = nn.Parameter(torch.zeros(C))


class AdainResBlk1d(nn.Module):
    """Trainable Modules/hifigan.py:359-403 AdainResBlk1d (the decoder's encode / decode blocks; same
    parameter names), forward and backward on the HIP kernels:
    r = conv2(LReLU(AdaIN2(conv1(pool(LReLU(AdaIN1(x)))))), sc = conv1x1(up2(x)),
    out = (r + sc) / sqrt(2) (the sum and the scale ride in conv2's epilogue).  Dropout p = 0 (the
    decoder's setting)."""

    def __init__(self, dim_in, dim_out, style_dim=64, upsample="none"):
        super().__init__()
        self.upsample = upsample not in ("none", False, None)
        self.learned_sc = dim_in != dim_out
        self.conv1 = _WNConv(dim_in, dim_out, 3, 1, 1)
        self.conv2 = _WNConv(dim_out, dim_out, 3, 1, 1)
        self.norm1 = _AdaIN(style_dim, dim_in)
        self.norm2 = _AdaIN(style_dim, dim_out)
        if self.learned_sc:
            self.conv1x1 = _WNConv(dim_in, dim_out, 1, 1, 0)
            self.conv1x1.bias = None
        if self.upsample:
            self.pool = _WNConvT(dim_in)

    def forward_frames(self, x, s):
        return adain_resblk1d_frames(self, x, s)

    def forward(self, x, s):
        return self.forward_frames(x.transpose(1, 2), s).transpose(1, 2)


def adain_resblk1d_frames(m, x, s, dtype="fp32"):
    """AdainResBlk1d.forward (hifigan.py:384-403, dropout p = 0) on frames x [B, L, C_in] for any module with
    the reference's parameter layout (training.AdainResBlk1d or params.AdainResBlk1d):
    out = (conv2(LReLU(AdaIN2(conv1(pool(LReLU(AdaIN1(x))))))) + conv1x1(up2(x))) / sqrt(2), the sum and the
    scale in conv2's epilogue."""
    up = m.upsample if isinstance(getattr(m, "upsample", None), bool) else m.upsample_type != "none"
    # nn.Dropout(dropout_p) before each conv in train mode (models.py:335, 358-367; the predictor's blocks)
    # (the reference's AdainResBlk1d keeps only self.dropout = nn.Dropout(p), models.py:335: read its p then)
    p_drop = getattr(m, "dropout_p", None)
    if p_drop is None:
        p_drop = getattr(getattr(m, "dropout", None), "p", 0.0)
    p_drop = float(p_drop or 0.0) if m.training else 0.0
    r = adain_act(x, s, m.norm1.fc.weight, m.norm1.fc.bias, None, ACT_LRELU)
    if up:
        r = _PoolFn.apply(r, weight_norm(m.pool.weight_g, m.pool.weight_v), m.pool.bias)
    c1, c2 = m.conv1, m.conv2
    r = conv1d_frames(dropout(r, p_drop), weight_norm(c1.weight_g, c1.weight_v), c1.bias, 1, 1, dtype=dtype)
    r = dropout(adain_act(r, s, m.norm2.fc.weight, m.norm2.fc.bias, None, ACT_LRELU), p_drop)
    sc = _Up2Fn.apply(x) if up else x
    if m.learned_sc:
        sc = conv1d_frames(sc, weight_norm(m.conv1x1.weight_g, m.conv1x1.weight_v), None, 1, 0, dtype=dtype)
    return conv1d_frames(r, weight_norm(c2.weight_g, c2.weight_v), c2.bias, 1, 1, dtype=dtype, residual=sc,
                         scale=1 / math.sqrt(2))


class _LReLUFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, slope):
        _require_device()
        xc = _c(x)
        y = torch.empty_like(xc)
        check(lib().stts_leaky_relu(_ptr(xc), xc.numel(), ctypes.c_float(slope), _ptr(y), _stream()),
              "stts_leaky_relu")
        ctx.save_for_backward(y)
        ctx.slope = slope
        return y

    @staticmethod
    def backward(ctx, gy):
        (y,) = ctx.saved_tensors
        dy = _c(gy)
        dx = torch.empty_like(y)
        check(lib().stts_leaky_relu_bwd(_ptr(y), _ptr(dy), y.numel(), ctypes.c_float(ctx.slope), _ptr(dx),
                                        _stream()), "stts_leaky_relu_bwd")
        return dx, None


def leaky_relu(x, slope):
    return _LReLUFn.apply(x, float(slope))


class _WNConv2dK1(nn.Module):
    """weight_norm(nn.Conv2d(cin, cout, (k, 1), (stride, 1), padding=(pad, 0))) parameter layout."""

    def __init__(self, cin, cout, k, stride, pad):
        super().__init__()
        self.weight_g = nn.Parameter(torch.ones(cout, 1, 1, 1))
        self.weight_v = nn.Parameter(torch.randn(cout, cin, k, 1) * 0.05)
        self.bias = nn.Parameter(torch.zeros(cout))
        self.k, self.stride, self.pad = k, stride, pad


class DiscriminatorP(nn.Module):
    """Trainable Modules/discriminators.py:96-129 DiscriminatorP (weight-norm, k 5, stride 3; same
    parameter names), forward and backward on the HIP kernels.  Each (k, 1) Conv2d is a conv1d along
    the H axis of every one of the `period` columns: the [B, C, H, p] map is kept as frames
    [B * p, H, C] between layers.  forward(x [B, 1, T]) -> (score [B, H * p], fmap [B, C, H, p] x 6)
    as the reference."""

    def __init__(self, period, kernel_size=5, stride=3, dtype_compute="fp32"):
        super().__init__()
        self.period = period
        self.dtype_compute = dtype_compute  # 'bf16': bf16 operands for the conv forwards and dx
        ch = [1, 32, 128, 512, 1024, 1024]
        self.convs = nn.ModuleList([_WNConv2dK1(ch[j], ch[j + 1], kernel_size, stride if j < 4 else 1, 2)
                                    for j in range(5)])
        self.conv_post = _WNConv2dK1(1024, 1, 3, 1, 1)

    def forward(self, x):
        b, c, t = x.shape
        p = self.period
        if t % p != 0:
            x = torch.nn.functional.pad(x, (0, p - t % p), "reflect")  # discriminators.py:112-115
            t = x.shape[-1]
        h = x.reshape(b, c, t // p, p).permute(0, 3, 2, 1).reshape(b * p, t // p, c)  # frames [B p, H, C]
        fmap = []

        def nchw(f):
            return f.reshape(b, p, f.shape[1], f.shape[2]).permute(0, 3, 2, 1)

        for layer in self.convs:
            w = weight_norm(layer.weight_g, layer.weight_v)
            h = conv1d_frames(h, w.reshape(w.shape[0], w.shape[1], layer.k), layer.bias, layer.stride, layer.pad,
                              dtype=self.dtype_compute)
            h = leaky_relu(h, 0.1)
            fmap.append(nchw(h))
        cp = self.conv_post
        w = weight_norm(cp.weight_g, cp.weight_v)
        h = conv1d_frames(h, w.reshape(1, w.shape[1], cp.k), cp.bias, 1, cp.pad, dtype=self.dtype_compute)
        out = nchw(h)
        fmap.append(out)
        return torch.flatten(out, 1, -1), fmap


# ====================================================================== the assembled training step (config 5)
# train.py:267-327: the decoder forward (Modules/hifigan.py:446-475) with its parameters' gradients, the
# discriminators (Modules/discriminators.py) with theirs, the losses (losses.py) and AdamW (optimizers.py).
# Every Function below runs its forward and backward as HIP kernels (include/stts2_train.h).

def _f32(t):
    return t.detach().to(torch.float32).contiguous()


class _SnakeFn(torch.autograd.Function):
    """Snake with a learned alpha (the Generator's stage activations, hifigan.py:329, :343) on frames."""

    @staticmethod
    def forward(ctx, x, alpha):
        _require_device()
        B, L, C = x.shape
        xc, ac = _f32(x), _f32(alpha.reshape(-1))
        y = torch.empty_like(xc)
        check(_tl().stts_snake_fwd(_ptr(xc), _ptr(ac), B, L, C, _ptr(y), _stream()), "stts_snake_fwd")
        ctx.save_for_backward(xc, ac)
        ctx.a_shape = alpha.shape
        return y

    @staticmethod
    def backward(ctx, dy):
        xc, ac = ctx.saved_tensors
        B, L, C = xc.shape
        nx, na = ctx.needs_input_grad
        dyc = _f32(dy)
        dx = torch.empty_like(xc) if nx else None
        da = torch.empty(C, dtype=torch.float32, device=dyc.device) if na else None
        nb = _tl().stts_snake_workspace_bytes(B, L, C)
        ws = _ws(nb, dyc.device)
        check(_tl().stts_snake_bwd(_ptr(xc), _ptr(ac), _ptr(dyc), B, L, C, _ptr(dx), _ptr(da), _ptr(ws), int(nb),
                                   _stream()), "stts_snake_bwd")
        return dx, (da.reshape(ctx.a_shape) if da is not None else None)


def snake(x, alpha):
    return _SnakeFn.apply(x, alpha)


class _TanhFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        _require_device()
        xc = _f32(x)
        y = torch.empty_like(xc)
        check(_tl().stts_tanh_fwd(_ptr(xc), xc.numel(), _ptr(y), _stream()), "stts_tanh_fwd")
        ctx.save_for_backward(y)
        return y

    @staticmethod
    def backward(ctx, dy):
        (y,) = ctx.saved_tensors
        dyc = _f32(dy)
        dx = torch.empty_like(y)
        check(_tl().stts_tanh_bwd(_ptr(y), _ptr(dyc), y.numel(), _ptr(dx), _stream()), "stts_tanh_bwd")
        return dx


def tanh(x):
    return _TanhFn.apply(x)


class _SumDivFn(torch.autograd.Function):
    """(x0 + x1 + ...) / div, added left to right (x + x_source, hifigan.py:334; xs / num_kernels, :342)."""

    @staticmethod
    def forward(ctx, div, *xs):
        _require_device()
        xc = [_f32(x) for x in xs]
        for x in xc[1:]:
            if x.shape != xc[0].shape:
                raise ValueError(f"sum of tensors of shapes {[tuple(t.shape) for t in xc]}")
        y = torch.empty_like(xc[0])
        arr = (ctypes.c_void_p * len(xc))(*[x.data_ptr() for x in xc])
        check(_tl().stts_sum_div(arr, len(xc), y.numel(), ctypes.c_float(div), _ptr(y), _stream()), "stts_sum_div")
        ctx.div, ctx.n = float(div), len(xc)
        return y

    @staticmethod
    def backward(ctx, dy):
        if ctx.div == 1.0:
            g = dy
        else:
            dyc = _f32(dy)
            g = torch.empty_like(dyc)
            check(_tl().stts_div(_ptr(dyc), dyc.numel(), ctypes.c_float(ctx.div), _ptr(g), _stream()), "stts_div")
        # every input gets its own tensor: the inputs may come from concurrent branches (CONCURRENT_BRANCHES), and
        # autograd may accumulate a gradient in place on one stream while another branch's stream still reads a
        # shared one
        out, first = [], True
        for need in ctx.needs_input_grad[1:]:
            out.append((g if first else g.clone()) if need else None)
            first = first and not need
        return (None,) + tuple(out)


def sum_div(xs, div=1.0):
    return _SumDivFn.apply(float(div), *xs)


class _SourceFn(torch.autograd.Function):
    """SourceModuleHnNSF (hifigan.py:221-268): f0_curve [B, n] -> har [B, n*scale]; gradients for l_linear."""

    @staticmethod
    def forward(ctx, f0_curve, lw, lb, noise, seed, utt_offset, scale):
        _require_device()
        B, n = f0_curve.shape
        L = n * scale
        fc, wc, bc = _f32(f0_curve), _f32(lw.reshape(-1)), _f32(lb.reshape(-1))
        nz = _f32(noise) if noise is not None else None
        if nz is not None and tuple(nz.shape) != (B, L, 9):
            raise ValueError(f"noise {tuple(nz.shape)}: expected {(B, L, 9)}")
        sw = torch.empty(B, L, 9, dtype=torch.float32, device=fc.device)
        har = torch.empty(B, L, dtype=torch.float32, device=fc.device)
        nb = _tl().stts_source_workspace_bytes(B, n)
        ws = _ws(nb, fc.device)
        if isinstance(seed, torch.Tensor):  # a device int64 [1] (the capturable step): the kernel reads it
            if not seed.is_cuda or seed.dtype != torch.int64:
                raise TypeError("seed tensor: int64 on the device")
            check(_tl().stts_source_fwd_seed_dev(_ptr(fc), _ptr(wc), _ptr(bc), _ptr(nz), _ptr(seed), int(utt_offset), B,
                                                 n, int(scale), _ptr(sw), _ptr(har), _ptr(ws), int(nb), _stream()),
                  "stts_source_fwd_seed_dev")
        else:
            check(_tl().stts_source_fwd(_ptr(fc), _ptr(wc), _ptr(bc), _ptr(nz),
                                        ctypes.c_ulonglong(int(seed) & (2**64 - 1)), int(utt_offset), B, n, int(scale),
                                        _ptr(sw), _ptr(har), _ptr(ws), int(nb), _stream()), "stts_source_fwd")
        ctx.save_for_backward(sw, har)
        ctx.shapes = (lw.shape, lb.shape, n)
        return har

    @staticmethod
    def backward(ctx, dhar):
        sw, har = ctx.saved_tensors
        lw_shape, lb_shape, n = ctx.shapes
        B, L = har.shape
        nw, nbias = ctx.needs_input_grad[1:3]
        if not (nw or nbias):
            return (None,) * 7
        d = _f32(dhar)
        dW = torch.empty(9, dtype=torch.float32, device=d.device)
        db = torch.empty(1, dtype=torch.float32, device=d.device)
        nbytes = _tl().stts_source_workspace_bytes(B, n)
        ws = _ws(nbytes, d.device)
        check(_tl().stts_source_bwd(_ptr(sw), _ptr(har), _ptr(d), B, L, _ptr(dW), _ptr(db), _ptr(ws), int(nbytes),
                                    _stream()), "stts_source_bwd")
        return None, (dW.reshape(lw_shape) if nw else None), (db.reshape(lb_shape) if nbias else None), None, None, \
            None, None


class _BoxFn(torch.autograd.Function):
    """conv1d(x, ones(1, 1, k), padding k // 2) / k per row (the train-mode smoothing, hifigan.py:453-455)."""

    @staticmethod
    def forward(ctx, x, k):
        _require_device()
        xc = _f32(x)
        B, n = xc.shape
        y = torch.empty_like(xc)
        check(_tl().stts_box_smooth_fwd(_ptr(xc), B, n, int(k), _ptr(y), _stream()), "stts_box_smooth_fwd")
        ctx.k = int(k)
        return y

    @staticmethod
    def backward(ctx, dy):
        d = _f32(dy)
        B, n = d.shape
        dx = torch.empty_like(d)
        check(_tl().stts_box_smooth_bwd(_ptr(d), B, n, ctx.k, _ptr(dx), _stream()), "stts_box_smooth_bwd")
        return dx, None


def box_smooth(x, k):
    return _BoxFn.apply(x, int(k))


def train_smooth(F0_curve, N, rng=None):
    """Decoder.forward's train-mode branch (hifigan.py:447-455): F0_down from [0, 3, 7] and N_down from
    [0, 3, 7, 15], drawn with Python's `random.randint` in the reference's order (so random.seed governs
    them), then the box smoothing on the device."""
    import random as _random
    r = rng or _random
    F0_down = [0, 3, 7][r.randint(0, 2)]
    N_down = [0, 3, 7, 15][r.randint(0, 3)]
    if F0_down:
        F0_curve = box_smooth(F0_curve, F0_down)
    if N_down:
        N = box_smooth(N, N_down)
    return F0_curve, N


class _TimeExpandFn(torch.autograd.Function):
    """x3[s][h][w][c*3 + dh] = y[s][h + dh - 1][w][c]: a (3, kw) Conv2d as a 1-D conv over 3C channels."""

    @staticmethod
    def forward(ctx, y):
        _require_device()
        yc = _f32(y)
        S, H, W, C = yc.shape
        x3 = torch.empty(S, H, W, 3 * C, dtype=torch.float32, device=yc.device)
        check(_tl().stts_time_expand3(_ptr(yc), S, H, W, C, _ptr(x3), _stream()), "stts_time_expand3")
        ctx.shape = (S, H, W, C)
        return x3

    @staticmethod
    def backward(ctx, dx3):
        S, H, W, C = ctx.shape
        d = _f32(dx3)
        dy = torch.empty(S, H, W, C, dtype=torch.float32, device=d.device)
        check(_tl().stts_time_expand3_bwd(_ptr(d), S, H, W, C, _ptr(dy), _stream()), "stts_time_expand3_bwd")
        return dy


# the MSD's (3, kw) Conv2d over C = 32 channels as one launch that time-expands in its window loads
# (stts_conv1d_fwd_tx); False = the materialised x3 + conv1d_frames (tests compare both)
FUSE_TX = True
# (K, stride) of the MSD layers whose bf16 weight gradient reads the image directly (stts_conv1d_wgrad_tx)
_WGRAD_TX = {(3, 1), (9, 2)}


class _ConvTxFn(torch.autograd.Function):
    """SpecDiscriminator's Conv2d(C, Cout, (3, kw), stride (1, s), padding (1, pad)) + optional leaky ReLU on the
    image h [S, H, W, C] -> frames [S H, Lq, Cout], with the time expansion inside the conv (stts_conv1d_fwd_tx,
    weight permuted to dh-major).  Backward: d h by stts_conv1d_bwd_tx (Cout = 32: dy expanded by the engine's
    loads, weight rows reversed) or, for the Cout = 1 out layer, stts_conv1d_bwd on x3 + stts_time_expand3_bwd;
    d w / d b by stts_conv1d_bwd over the materialised x3 (c-major, the weight as it lies)."""

    @staticmethod
    def forward(ctx, h, w, bias, stride, pad, dtype, act):
        _require_device()
        hf = _f32(h)
        S, H, W, C = hf.shape
        co, ci, kh, kw = w.shape
        if ci != C or kh != 3:
            raise ValueError(f"weight {tuple(w.shape)} does not take the [S, H, W, {C}] image")
        Lq = out_length(W, kw, stride, pad, 1)
        dt = _DT[dtype]
        wc = _f32(w)
        wtx = wc.permute(0, 2, 1, 3).contiguous()  # [Cout][3][C][kw]: K index dh C + c
        bc = _f32(bias) if bias is not None else None
        nb = lib().stts_conv1d_fwd_tx_workspace_bytes(dt, S, H, W, C, co, kw, stride, pad, Lq)
        check(int(nb) if nb < 0 else 0, "stts_conv1d_fwd_tx_workspace_bytes")
        ws = _ws(nb, hf.device)
        y = torch.empty(S * H, Lq, co, dtype=torch.float32, device=hf.device)
        check(lib().stts_conv1d_fwd_tx(dt, _ptr(hf), _ptr(wtx), _ptr(bc), S, H, W, C, co, kw, stride, pad, Lq,
                                       int(act is not None), ctypes.c_float(act if act is not None else 0.0), _ptr(y),
                                       _ptr(ws), int(nb), _stream()), "stts_conv1d_fwd_tx")
        ctx.save_for_backward(hf, wc, y if act is not None else None)
        ctx.geo = (S, H, W, C, co, kw, stride, pad, Lq, dt, bias is not None)
        ctx.act = act
        _count("fwd", 2.0 * S * H * Lq * co * 3 * C * kw)
        return y

    @staticmethod
    def backward(ctx, gy):
        hf, wc, ya = ctx.saved_tensors
        S, H, W, C, co, kw, stride, pad, Lq, dt, has_bias = ctx.geo
        need_x, need_w, need_b = ctx.needs_input_grad[:3]
        dyf = _f32(gy)
        if ctx.act is not None:
            dpre = torch.empty_like(dyf)
            check(lib().stts_leaky_relu_bwd(_ptr(ya), _ptr(dyf), ya.numel(), ctypes.c_float(ctx.act), _ptr(dpre),
                                            _stream()), "stts_leaky_relu_bwd")
            dyf = dpre
        dev = dyf.device
        B, Cin = S * H, 3 * C
        dh = None
        if need_x and co == 32:  # d h straight from dy (no dx3 image, no fold)
            wd = wc.flip(2).permute(2, 0, 1, 3).contiguous()  # [3][Cout][C][kw]: chunk j = row dh = 2 - j
            nb = lib().stts_conv1d_bwd_tx_workspace_bytes(dt, S, H, W, C, co, kw, stride, pad, Lq)
            check(int(nb) if nb < 0 else 0, "stts_conv1d_bwd_tx_workspace_bytes")
            ws = _ws(nb, dev)
            dh = torch.empty(S, H, W, C, dtype=torch.float32, device=dev)
            check(lib().stts_conv1d_bwd_tx(dt, _ptr(dyf), _ptr(wd), S, H, W, C, co, kw, stride, pad, Lq, _ptr(dh),
                                           _ptr(ws), int(nb), _stream()), "stts_conv1d_bwd_tx")
            _count("bwd", 2.0 * B * Lq * co * Cin * kw)
            need_x = False
        need_b = need_b and has_bias
        dx3 = dw = db = None
        if not need_x and (need_w or need_b) and dt == 1 and (kw, stride) in _WGRAD_TX:  # bf16: no x3 either
            nb = lib().stts_conv1d_bwd_workspace_bytes(dt, B, W, Cin, co, kw, stride, 1, pad, Lq)
            check(int(nb) if nb < 0 else 0, "stts_conv1d_bwd_workspace_bytes")
            ws = _ws(nb, dev)
            dwt = torch.empty(co, 3, C, kw, dtype=torch.float32, device=dev)
            db = torch.empty(co, dtype=torch.float32, device=dev) if need_b else None
            check(lib().stts_conv1d_wgrad_tx(dt, _ptr(hf), _ptr(dyf), S, H, W, C, co, kw, stride, pad, Lq, _ptr(dwt),
                                             _ptr(db), _ptr(ws), int(nb), _stream()), "stts_conv1d_wgrad_tx")
            _count("bwd", 2.0 * B * Lq * co * Cin * kw)
            dw = dwt.permute(0, 2, 1, 3) if need_w else None  # -> [Cout][C][3][kw]
            need_w = need_b = False
        if need_x or need_w or need_b:  # (the G step's frozen discriminators skip this: d h only)
            x3 = torch.empty(S, H, W, Cin, dtype=torch.float32, device=dev)
            check(_tl().stts_time_expand3(_ptr(hf), S, H, W, C, _ptr(x3), _stream()), "stts_time_expand3")
            nb = lib().stts_conv1d_bwd_workspace_bytes(dt, B, W, Cin, co, kw, stride, 1, pad, Lq)
            check(int(nb) if nb < 0 else 0, "stts_conv1d_bwd_workspace_bytes")
            ws = _ws(nb, dev)
            dx3 = torch.empty(B, W, Cin, dtype=torch.float32, device=dev) if need_x else None
            dw = torch.empty(co, Cin, kw, dtype=torch.float32, device=dev) if need_w else None
            db = torch.empty(co, dtype=torch.float32, device=dev) if need_b else None
            check(lib().stts_conv1d_bwd(dt, _ptr(x3), _ptr(wc), _ptr(dyf), B, W, Cin, co, kw, stride, 1, pad, Lq,
                                        _ptr(dx3), _ptr(dw), _ptr(db), _ptr(ws), int(nb), _stream()),
                  "stts_conv1d_bwd")
            _count("bwd", 2.0 * B * Lq * co * Cin * kw * ((dx3 is not None) + (dw is not None)))
        if dx3 is not None:
            dh = torch.empty(S, H, W, C, dtype=torch.float32, device=dev)
            check(_tl().stts_time_expand3_bwd(_ptr(dx3), S, H, W, C, _ptr(dh), _stream()), "stts_time_expand3_bwd")
        if dw is not None and dw.dim() == 3:
            dw = dw.reshape(co, C, 3, kw)
        return dh, dw, db, None, None, None, None


class _StftMagFn(torch.autograd.Function):
    """|torch.stft(x, n_fft, hop, win, hann(win))| (discriminators.py:11-27) as the [S, F, nb] image."""

    @staticmethod
    def forward(ctx, wave, n_fft, hop, win):
        _require_device()
        w = _f32(wave)
        S, L = w.shape
        F_ = 1 + L // hop
        nb = n_fft // 2 + 1
        mag = torch.empty(S, F_, nb, dtype=torch.float32, device=w.device)
        spec = torch.empty(S, F_, nb, 2, dtype=torch.float32, device=w.device)
        check(_tl().stts_stft_mag_fwd(_ptr(w), S, L, L, n_fft, win, hop, _ptr(mag), _ptr(spec), _stream()),
              "stts_stft_mag_fwd")
        ctx.save_for_backward(spec)
        ctx.geo = (S, L, n_fft, win, hop)
        return mag

    @staticmethod
    def backward(ctx, dmag):
        (spec,) = ctx.saved_tensors
        S, L, n_fft, win, hop = ctx.geo
        d = _f32(dmag)
        dw = torch.empty(S, L, dtype=torch.float32, device=d.device)
        nb = _tl().stts_stft_mag_workspace_bytes(S, L, n_fft, win, hop)
        check(int(nb) if nb < 0 else 0, "stts_stft_mag_workspace_bytes")
        ws = _ws(nb, d.device)
        check(_tl().stts_stft_mag_bwd(_ptr(spec), _ptr(d), S, L, n_fft, win, hop, _ptr(dw), _ptr(ws), int(nb),
                                      _stream()), "stts_stft_mag_bwd")
        return dw, None, None, None


def stft_mag(wave, n_fft, hop, win):
    return _StftMagFn.apply(wave, int(n_fft), int(hop), int(win))


# ---------------------------------------------------------------------- decoder (Modules/hifigan.py)
def _wn_w(layer):
    return weight_norm(layer.weight_g, layer.weight_v)


# independent branches of the generator (the noise branch beside snake -> ups, the num_kernels resblocks of a
# stage) run on their own HIP streams, as discriminators.CONCURRENT does for the sub-discriminators; autograd runs
# each backward op on its forward's stream.  False = one stream (A/B, tests)
CONCURRENT_BRANCHES = True
_BRANCH_STREAMS = {}


def _branches(fns, inputs=()):
    """[f() for f in fns], f i on side stream i, ordered after the caller's stream, which waits for all of them;
    `inputs` (tensors of the caller's stream the branches read or save for backward) are recorded on each side
    stream so the allocator does not hand their memory out before those reads finish."""
    if not CONCURRENT_BRANCHES or len(fns) < 2:
        return [f() for f in fns]
    dev = torch.device("cuda", torch.cuda.current_device())
    key = (dev.index, len(fns))
    if key not in _BRANCH_STREAMS:
        _BRANCH_STREAMS[key] = [torch.cuda.Stream(device=dev) for _ in fns]
    main = torch.cuda.current_stream(dev)
    outs = []
    for f, st in zip(fns, _BRANCH_STREAMS[key]):
        st.wait_stream(main)
        for t in inputs:
            t.record_stream(st)
        with torch.cuda.stream(st):
            outs.append(f())
    for st in _BRANCH_STREAMS[key]:
        main.wait_stream(st)
    for o in outs:
        o.record_stream(main)
    return outs


def generator_forward(g, x, s, f0_curve, noise=None, seed=0, utt_offset=0, dtype="fp32"):
    """Generator.forward (hifigan.py:321-347) on frames x [B, 2T, 512] for a module with the reference's
    parameter layout (stts2_mi355x.hifigan.Generator) -> waveform frames [B, L, 1]."""
    rates, kernels = g.upsample_rates, g.upsample_kernel_sizes
    nk = g.num_kernels
    scale = int(g.upsample_scale)
    har = _SourceFn.apply(f0_curve, g.m_source.l_linear.weight, g.m_source.l_linear.bias, noise, seed, utt_offset,
                          scale).unsqueeze(-1)  # frames [B, L, 1]
    B = har.shape[0]
    for i, (u, k) in enumerate(zip(rates, kernels)):
        nc = g.noise_convs[i]

        def noise_branch(i=i, nc=nc):
            S, P = int(nc.stride), int(nc.padding)
            if S > 1 and nc.weight.shape[-1] == 2 * S and 2 * P == S:
                # Conv1d(1, C, 2S, stride S, padding S/2) (hifigan.py:296-299) as a 2-tap stride-1 conv over
                # S-sample frames: frame r = samples [r S - P, r S - P + S), w'[c][j][t] = w[c][0][t S + j]
                fr = torch.nn.functional.pad(har[..., 0], (P, S - P)).reshape(B, -1, S)
                w2 = nc.weight.reshape(nc.weight.shape[0], 2, S).transpose(1, 2)
                x_src = conv1d_frames(fr, w2, nc.bias, 1, 0, 1, dtype)
            else:
                x_src = conv1d_frames(har, nc.weight, nc.bias, nc.stride, nc.padding, 1, dtype)
            return resblock1_frames(g.noise_res[i], x_src, s, dtype)

        def up_branch(i=i, x=x):
            x = snake(x, g.alphas[i])
            up = g.ups[i]
            return conv_transpose1d_frames(x, _wn_w(up), up.bias, up.stride, up.padding, up.output_padding, dtype)

        x, x_src = _branches([up_branch, noise_branch], (x, har, s))
        x = sum_div([x, x_src])
        rs = _branches([lambda j=j, x=x: resblock1_frames(g.resblocks[i * nk + j], x, s, dtype) for j in range(nk)],
                       (x, s))
        x = sum_div(rs, nk)
    x = snake(x, g.alphas[len(rates)])
    cp = g.conv_post
    x = conv1d_frames(x, _wn_w(cp), cp.bias, 1, cp.padding, 1, dtype)
    return tanh(x)


def decoder_forward(dec, asr, F0_curve, N, s, noise=None, seed=None, utt_offset=0, dtype="fp32"):
    """Decoder.forward (hifigan.py:446-475) with autograd through HIP kernels: asr [B, 512, T], F0_curve and
    N [B, 2T], s [B, style_dim] -> [B, 1, 600 T].  `dec` is stts2_mi355x.hifigan.Decoder (reference
    parameter names); in .train() mode the F0 / N smoothing of :447-455 is applied first (Python's random,
    as the reference).  Activations stay in frames [B, L, C] end to end."""
    _require_device()
    if dtype not in _DT:
        raise ValueError(f"dtype {dtype!r}: expected one of {list(_DT)}")
    if seed is None:
        seed = int(torch.randint(0, 2 ** 62, (1,)).item()) if noise is None else 0
    if dec.training:
        F0_curve, N = train_smooth(F0_curve, N)
    B, _, T = asr.shape
    if F0_curve.shape[-1] != 2 * T or N.shape[-1] != 2 * T:
        raise ValueError(f"F0_curve / N {tuple(F0_curve.shape)} / {tuple(N.shape)}: expected [B, {2 * T}]")
    F0 = conv1d_frames(F0_curve.unsqueeze(-1), _wn_w(dec.F0_conv), dec.F0_conv.bias, 2, 1, 1, dtype)  # [B, T, 1]
    Nc = conv1d_frames(N.unsqueeze(-1), _wn_w(dec.N_conv), dec.N_conv.bias, 2, 1, 1, dtype)
    asr_f = asr.transpose(1, 2)  # frames [B, T, 512]
    x = torch.cat([asr_f, F0, Nc], dim=2)
    x = adain_resblk1d_frames(dec.encode, x, s, dtype)
    ar = dec.asr_res[0]
    asr_res = conv1d_frames(asr_f, _wn_w(ar), ar.bias, 1, 0, 1, dtype)
    res = True
    for block in dec.decode:
        if res:
            x = torch.cat([x, asr_res, F0, Nc], dim=2)
        x = adain_resblk1d_frames(block, x, s, dtype)
        if block.upsample_type != "none":
            res = False
    y = generator_forward(dec.generator, x, s, F0_curve, noise, seed, utt_offset, dtype)  # [B, L, 1]
    return y.reshape(B, 1, -1)


# ---------------------------------------------------------------------- discriminators
def _k1_geom(layer):
    """(k, stride, pad) of a (k, 1) Conv2d: the reference's nn.Conv2d or training._WNConv2dK1."""
    if hasattr(layer, "kernel_size"):
        return layer.kernel_size[0], layer.stride[0], layer.padding[0]
    return layer.k, layer.stride, layer.pad


def discriminator_p_forward(m, x, period, dtype="fp32"):
    """DiscriminatorP.forward (discriminators.py:110-129) for a module with the reference's parameter layout:
    x [B, 1, T] -> (score [B, H*p], fmap: 6 maps [B, C, H, p], permuted views of frames [B*p, H, C])."""
    b, c, t = x.shape
    p = period
    if t % p != 0:
        x = torch.nn.functional.pad(x, (0, p - t % p), "reflect")  # discriminators.py:112-115
        t = x.shape[-1]
    h = x.reshape(b, c, t // p, p).permute(0, 3, 2, 1).reshape(b * p, t // p, c)
    fmap = []

    def nchw(f):
        return f.reshape(b, p, f.shape[1], f.shape[2]).permute(0, 3, 2, 1)

    for layer in m.convs:
        k, st, pad = _k1_geom(layer)
        w = _wn_w(layer)
        wk = w.reshape(w.shape[0], w.shape[1], k)
        if FUSE_LRELU:
            h = conv1d_frames(h, wk, layer.bias, st, pad, dtype=dtype, act_slope=0.1)
        else:
            h = leaky_relu(conv1d_frames(h, wk, layer.bias, st, pad, dtype=dtype), 0.1)
        fmap.append(nchw(h))
    cp = m.conv_post
    k, st, pad = _k1_geom(cp)
    w = _wn_w(cp)
    h = conv1d_frames(h, w.reshape(1, w.shape[1], k), cp.bias, st, pad, dtype=dtype)
    out = nchw(h)
    fmap.append(out)
    return torch.flatten(out, 1, -1), fmap


def spec_discriminator_forward(m, y, dtype="fp32"):
    """SpecDiscriminator.forward (discriminators.py:49-63) for the reference's parameter layout: y [B, 1, T]
    -> (score [B, F*W5], fmap: 6 maps [B, C, F, W], permuted views of frames [B, F, W, C]).  The |STFT|
    image is [B, F frames, nb bins]; each (3, kw) Conv2d is a 1-D conv along the bins over the 3 C
    time-expanded channels (x3[..., c*3 + dh] = row h + dh - 1), so the weight [Cout, C, 3, kw] is the
    [Cout, 3C, kw] conv1d weight as it lies in memory."""
    y = y.reshape(y.shape[0], -1)
    S = y.shape[0]
    h = stft_mag(y, m.fft_size, m.shift_size, m.win_length).unsqueeze(-1)  # [S, F, nb, 1]
    Fr = h.shape[1]
    fmap = []
    layers = list(m.discriminators) + [m.out]
    for j, layer in enumerate(layers):
        w = _wn_w(layer)
        co, ci, kh, kw = w.shape
        act = j < len(layers) - 1
        if (FUSE_TX and (FUSE_LRELU or not act) and ci == 32 and kh == 3 and layer.padding[0] == 1
                and layer.stride[0] == 1):
            out = _ConvTxFn.apply(h, w, layer.bias, layer.stride[1], layer.padding[1], dtype, 0.1 if act else None)
            h = out.reshape(S, Fr, out.shape[1], co)
            fmap.append(h.permute(0, 3, 1, 2))
            continue
        x3 = _TimeExpandFn.apply(h)  # [S, F, W, 3C]
        W3 = x3.shape[2]
        out = conv1d_frames(x3.reshape(S * Fr, W3, 3 * ci), w.reshape(co, ci * kh, kw), layer.bias,
                            layer.stride[1], layer.padding[1], dtype=dtype,
                            act_slope=0.1 if (act and FUSE_LRELU) else None)
        if act and not FUSE_LRELU:
            out = leaky_relu(out, 0.1)
        h = out.reshape(S, Fr, out.shape[1], co)
        fmap.append(h.permute(0, 3, 1, 2))
    return h.reshape(S, -1), fmap


# ------------------------------------------------------------------ dropout (train mode)
class _DropoutFn(torch.autograd.Function):
    """nn.Dropout(p) in train mode on the device (stts_dropout): the mask is a counter draw keyed by a seed from
    torch's default generator, redrawn (not stored) by the backward."""

    @staticmethod
    def forward(ctx, x, p):
        _require_device()
        xc = _c(x)
        seed = int(torch.randint(0, 2 ** 62, (1,)).item())
        y = torch.empty_like(xc)
        check(_tl().stts_dropout(_ptr(xc), xc.numel(), ctypes.c_float(p), ctypes.c_ulonglong(seed), _ptr(y),
                                 _stream()), "stts_dropout")
        ctx.p, ctx.seed = p, seed
        return y

    @staticmethod
    def backward(ctx, dy):
        dyc = _c(dy)
        dx = torch.empty_like(dyc)
        check(_tl().stts_dropout(_ptr(dyc), dyc.numel(), ctypes.c_float(ctx.p), ctypes.c_ulonglong(ctx.seed),
                                 _ptr(dx), _stream()), "stts_dropout")
        return dx, None


class _DropoutMaskFn(torch.autograd.Function):
    """Train-mode dropout with an injected keep mask (stts_dropout_mask), forward and backward."""

    @staticmethod
    def forward(ctx, x, mask, p):
        _require_device()
        xc, mc = _c(x), _c(mask.to(x.device, torch.float32))
        if mc.shape != xc.shape:
            raise ValueError(f"dropout mask {tuple(mc.shape)} for a tensor {tuple(xc.shape)}")
        y = torch.empty_like(xc)
        check(_tl().stts_dropout_mask(_ptr(xc), _ptr(mc), xc.numel(), ctypes.c_float(p), _ptr(y), _stream()),
              "stts_dropout_mask")
        ctx.save_for_backward(mc)
        ctx.p = p
        return y

    @staticmethod
    def backward(ctx, dy):
        (mc,) = ctx.saved_tensors
        dyc = _c(dy)
        dx = torch.empty_like(dyc)
        check(_tl().stts_dropout_mask(_ptr(dyc), _ptr(mc), dyc.numel(), ctypes.c_float(ctx.p), _ptr(dx), _stream()),
              "stts_dropout_mask")
        return dx, None, None


_MASKS = {"fn": None, "k": 0}


def set_dropout_masks(fn):
    """Test hook: fn(k, shape, p) -> the keep mask (0 / 1, any device) of the k-th train-mode dropout call from now on,
    in the REFERENCE module's layout of that tensor (a call site whose layout differs passes ref_transpose); None
    goes back to the device counter draws.  The train-mode fixtures (tests/golden/make_golden_train_text.py) inject
    the same masks into the reference's F.dropout, so both sides drop the same elements."""
    _MASKS["fn"], _MASKS["k"] = fn, 0


def dropout(x, p, ref_transpose=False):
    """nn.Dropout(p) / F.dropout in train mode.  ref_transpose: the reference holds this tensor as x.transpose(1, 2)
    (the TextEncoder's CNN, channels-first there), which is where an injected mask is laid out."""
    if p <= 0:
        return x
    fn = _MASKS["fn"]
    if fn is None:
        return _DropoutFn.apply(x, float(p))
    shape = tuple(x.transpose(1, 2).shape) if ref_transpose else tuple(x.shape)
    m = torch.as_tensor(fn(_MASKS["k"], shape, float(p)), dtype=torch.float32, device=x.device)
    _MASKS["k"] += 1
    if ref_transpose:
        m = m.transpose(1, 2)
    return _DropoutMaskFn.apply(x, m.contiguous(), float(p))


# ------------------------------------------------------------------ ProsodyPredictor.F0Ntrain (models.py:448-461)
class _BiLSTMFn(torch.autograd.Function):
    """Bidirectional nn.LSTM (batch_first) with its backward: stts_bilstm_fwd_train / stts_bilstm_bwd.  x frames
    [B, T, Cin]; ln: None (ProsodyPredictor.shared, full-length rows) or the device int32 text lengths (the packed
    sequences of the text / duration path, texttrain.py); params in torch's order."""

    @staticmethod
    def forward(ctx, x, ln, *params):
        _require_device()
        xc = _c(x)
        B, T, Cin = xc.shape
        ps = [_c(p) for p in params]
        H = ps[1].shape[1]
        arr = (ctypes.c_void_p * 8)(*[p.data_ptr() for p in ps])
        L = _tl()
        nb = int(L.stts_bilstm_workspace_bytes(B, T, H))
        ws = _ws(nb, x.device)
        y = torch.empty(B, T, 2 * H, dtype=torch.float32, device=x.device)
        cs = torch.empty(2, B, T, H, dtype=torch.float32, device=x.device)
        check(L.stts_bilstm_fwd_train(_ptr(xc), T * Cin, Cin, 1, B, T, Cin, _ptr(ln), arr, H, _ptr(y), _ptr(cs),
                                      _ptr(ws), nb, _stream()), "stts_bilstm_fwd_train")
        ctx.save_for_backward(xc, y, cs, ln if ln is not None else torch.empty(0), *ps)
        ctx.has_ln = ln is not None
        return y

    @staticmethod
    def backward(ctx, dy):
        xc, y, cs, ln, *ps = ctx.saved_tensors
        ln = ln if ctx.has_ln else None
        B, T, Cin = xc.shape
        H = ps[1].shape[1]
        dyc = _c(dy)
        need = ctx.needs_input_grad
        dx = torch.empty_like(xc) if need[0] else None
        grads = [torch.empty_like(p) if need[i + 2] else None for i, p in enumerate(ps)]
        arr = (ctypes.c_void_p * 8)(*[p.data_ptr() for p in ps])
        garr = (ctypes.c_void_p * 8)(*[g.data_ptr() if g is not None else None for g in grads])
        L = _tl()
        nb = int(L.stts_bilstm_bwd_workspace_bytes(B, T, Cin, H))
        check(nb if nb < 0 else 0, "stts_bilstm_bwd_workspace_bytes")
        ws = _ws(nb, dy.device)
        check(L.stts_bilstm_bwd(_ptr(xc), B, T, Cin, _ptr(ln), arr, H, _ptr(y), _ptr(cs), _ptr(dyc), _ptr(dx), garr,
                                _ptr(ws), nb, _stream()), "stts_bilstm_bwd")
        return (dx, None, *grads)


def bilstm_frames(lstm, x):
    """lstm = the reference's nn.LSTM(.., bidirectional, batch_first) layout; x frames [B, T, Cin] -> [B, T, 2H]."""
    ps = [lstm.weight_ih_l0, lstm.weight_hh_l0, lstm.bias_ih_l0, lstm.bias_hh_l0, lstm.weight_ih_l0_reverse,
          lstm.weight_hh_l0_reverse, lstm.bias_ih_l0_reverse, lstm.bias_hh_l0_reverse]
    return _BiLSTMFn.apply(x, None, *ps)


def f0ntrain(pp, x, s, dtype="fp32"):
    """ProsodyPredictor.F0Ntrain (models.py:448-461) with autograd: x [B, d_hid + style_dim, T], s [B, style_dim]
    -> (F0 [B, 2T], N [B, 2T]).  The shared BiLSTM, the F0 / N AdainResBlk1d stacks (their dropout in train mode)
    and the 1x1 projections, on frames [B, T, C] throughout."""
    h = bilstm_frames(pp.shared, x.transpose(1, 2).contiguous())
    outs = []
    for blocks, proj in ((pp.F0, pp.F0_proj), (pp.N, pp.N_proj)):
        y = h
        for blk in blocks:
            y = adain_resblk1d_frames(blk, y, s, dtype)
        y = conv1d_frames(y, proj.weight, proj.bias, 1, 0, dtype=dtype)  # [B, 2T, 1]
        outs.append(y[..., 0])
    return outs[0], outs[1]


# ------------------------------------------------------------------ StyleEncoder (models.py:125-150)
class _RowExpFn(torch.autograd.Function):
    """Row expansion of a frames image [B, H, W, C] for a k x k Conv2d with H padding `pad`: [B, Ho, W, C k]."""

    @staticmethod
    def forward(ctx, x, k, pad):
        _require_device()
        xc = _c(x)
        B, H, W, C = xc.shape
        Ho = H + 2 * pad - k + 1
        xe = torch.empty(B, Ho, W, C * k, dtype=torch.float32, device=x.device)
        check(_tl().stts_rowexp_fwd(_ptr(xc), B, H, W, C, k, pad, _ptr(xe), _stream()), "stts_rowexp_fwd")
        ctx.geom = (B, H, W, C, k, pad)
        return xe

    @staticmethod
    def backward(ctx, dxe):
        B, H, W, C, k, pad = ctx.geom
        d = _c(dxe)
        dx = torch.empty(B, H, W, C, dtype=torch.float32, device=d.device)
        check(_tl().stts_rowexp_bwd(_ptr(d), B, H, W, C, k, pad, _ptr(dx), _stream()), "stts_rowexp_bwd")
        return dx, None, None


class _DWConvS2Fn(torch.autograd.Function):
    """LearnedDownSample('half'): depthwise Conv2d(C, C, 3, stride 2, pad 1) on frames images."""

    @staticmethod
    def forward(ctx, x, w, b):
        _require_device()
        xc, wc, bc = _c(x), _c(w), _c(b)
        B, H, W, C = xc.shape
        y = torch.empty(B, (H - 1) // 2 + 1, (W - 1) // 2 + 1, C, dtype=torch.float32, device=x.device)
        check(_tl().stts_dwconv2d_s2_fwd(_ptr(xc), _ptr(wc), _ptr(bc), B, H, W, C, _ptr(y), _stream()),
              "stts_dwconv2d_s2_fwd")
        ctx.save_for_backward(xc, wc)
        ctx.has_b = b is not None
        return y

    @staticmethod
    def backward(ctx, dy):
        xc, wc = ctx.saved_tensors
        B, H, W, C = xc.shape
        d = _c(dy)
        nx, nw, nb_ = ctx.needs_input_grad
        dx = torch.empty_like(xc) if nx else None
        dw = torch.empty_like(wc) if nw else None
        db = torch.empty(C, dtype=torch.float32, device=d.device) if (nb_ and ctx.has_b) else None
        L = _tl()
        nb = int(L.stts_dwconv2d_s2_workspace_bytes(C))
        ws = _ws(nb, d.device)
        check(L.stts_dwconv2d_s2_bwd(_ptr(xc), _ptr(wc), _ptr(d), B, H, W, C, _ptr(dx), _ptr(dw), _ptr(db), _ptr(ws), nb,
                                     _stream()), "stts_dwconv2d_s2_bwd")
        return dx, dw, db


class _AvgPool2Fn(torch.autograd.Function):
    """DownSample('half') on frames images (the last column repeated when W is odd, then 2 x 2 averages)."""

    @staticmethod
    def forward(ctx, x):
        _require_device()
        xc = _c(x)
        B, H, W, C = xc.shape
        y = torch.empty(B, H // 2, (W + 1) // 2, C, dtype=torch.float32, device=x.device)
        check(_tl().stts_avgpool2_fwd(_ptr(xc), B, H, W, C, _ptr(y), _stream()), "stts_avgpool2_fwd")
        ctx.geom = (B, H, W, C)
        return y

    @staticmethod
    def backward(ctx, dy):
        B, H, W, C = ctx.geom
        d = _c(dy)
        dx = torch.empty(B, H, W, C, dtype=torch.float32, device=d.device)
        check(_tl().stts_avgpool2_bwd(_ptr(d), B, H, W, C, _ptr(dx), _stream()), "stts_avgpool2_bwd")
        return dx


class _SpatialMeanFn(torch.autograd.Function):
    """AdaptiveAvgPool2d(1) of a frames image [B, H, W, C] -> [B, C]."""

    @staticmethod
    def forward(ctx, x):
        _require_device()
        xc = _c(x)
        B, H, W, C = xc.shape
        y = torch.empty(B, C, dtype=torch.float32, device=x.device)
        check(_tl().stts_spatial_mean_fwd(_ptr(xc), B, H * W, C, _ptr(y), _stream()), "stts_spatial_mean_fwd")
        ctx.geom = (B, H, W, C)
        return y

    @staticmethod
    def backward(ctx, dy):
        B, H, W, C = ctx.geom
        d = _c(dy)
        dx = torch.empty(B, H, W, C, dtype=torch.float32, device=d.device)
        check(_tl().stts_spatial_mean_bwd(_ptr(d), B, H * W, C, _ptr(dx), _stream()), "stts_spatial_mean_bwd")
        return dx


def conv2d_frames(x, weight, bias, pad, dtype="fp32", residual=None, scale=1.0):
    """Conv2d(k x k, stride 1, padding pad) of a frames image x [B, H, W, Cin] with the reference weight
    [Cout, Cin, k, k]: the row expansion, then the conv1d engine over W (weight read as [Cout, Cin k, k]).
    residual (frames image of the output's shape) and scale ride in the conv's epilogue: (y + residual) * scale."""
    B, H, W, C = x.shape
    co, ci, k, kw = weight.shape
    if ci != C or kw != k:
        raise ValueError(f"conv2d_frames: weight {tuple(weight.shape)} for {C} input channels")
    xe = _RowExpFn.apply(x, k, pad) if k > 1 else x
    Ho = xe.shape[1]
    res = residual.reshape(B * Ho, residual.shape[2], co) if residual is not None else None
    y = conv1d_frames(xe.reshape(B * Ho, W, C * k), weight.reshape(co, C * k, k), bias, 1, pad, 1, dtype,
                      residual=res, scale=scale)
    return y.reshape(B, Ho, y.shape[1], co)


def style_encoder(se, mel, dtype="fp32"):
    """StyleEncoder.forward (models.py:145-150) with autograd: mel [B, 1, n_mels, F] -> [B, style_dim].
    shared = conv3x3 -> 4 x ResBlk('half': (DownSample(conv1x1(x)) + conv2(LReLU(LearnedDownSample(conv1(LReLU(x))))))
    / sqrt(2), models.py:82-123) -> LReLU -> conv5x5 (valid) -> AdaptiveAvgPool2d(1) -> LReLU; unshared = Linear.
    Frames images [B, n_mels, F, C] throughout."""
    blocks = list(se.shared)
    x = mel.permute(0, 2, 3, 1).contiguous()
    c0 = blocks[0]
    x = conv2d_frames(x, c0.weight, c0.bias, 1, dtype)
    for blk in blocks[1:5]:
        sc = x
        if blk.learned_sc:
            sc = conv2d_frames(sc, blk.conv1x1.weight, None, 0, dtype)
        sc = _AvgPool2Fn.apply(sc)
        r = conv2d_frames(leaky_relu(x, 0.2), blk.conv1.weight, blk.conv1.bias, 1, dtype)
        ds = blk.downsample_res.conv
        r = leaky_relu(_DWConvS2Fn.apply(r, ds.weight, ds.bias), 0.2)
        x = conv2d_frames(r, blk.conv2.weight, blk.conv2.bias, 1, dtype, residual=sc, scale=1 / math.sqrt(2))
    c5 = blocks[6]
    x = conv2d_frames(leaky_relu(x, 0.2), c5.weight, c5.bias, 0, dtype)
    h = leaky_relu(_SpatialMeanFn.apply(x), 0.2)
    return linear(h, se.unshared.weight, se.unshared.bias)
