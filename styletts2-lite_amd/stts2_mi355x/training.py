"""Training-step conv layers on the HIP path.

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

import torch
from torch import nn

from .engine import _ptr, _require_device, _stream, check, lib

_DT = {"fp32": 0, "bf16": 1}


def _ws(nbytes: int, device) -> torch.Tensor:
    return torch.empty(max(int(nbytes), 1), dtype=torch.uint8, device=device)


def _frames(t: torch.Tensor) -> torch.Tensor:
    return t.detach().to(torch.float32).transpose(1, 2).contiguous()


def out_length(Lin: int, K: int, stride: int, pad: int, dil: int) -> int:
    return (Lin + 2 * pad - dil * (K - 1) - 1) // stride + 1


class _Conv1dFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, bias, stride, pad, dil, dtype):
        _require_device()
        B, Cin, Lin = x.shape
        Cout, Cin_w, K = w.shape
        if Cin_w != Cin:
            raise ValueError(f"weight {tuple(w.shape)} does not take {Cin} input channels")
        Lq = out_length(Lin, K, stride, pad, dil)
        dt = _DT[dtype]
        xf = _frames(x)
        wc = w.detach().to(torch.float32).contiguous()
        bc = bias.detach().to(torch.float32).contiguous() if bias is not None else None
        nb = lib().stts_conv1d_fwd_workspace_bytes(dt, B, Lin, Cin, Cout, K, stride, dil, pad, Lq)
        check(int(nb) if nb < 0 else 0, "stts_conv1d_fwd_workspace_bytes")
        ws = _ws(nb, x.device)
        y = torch.empty(B, Lq, Cout, dtype=torch.float32, device=x.device)
        check(lib().stts_conv1d_fwd(dt, _ptr(xf), _ptr(wc), _ptr(bc), B, Lin, Cin, Cout, K, stride, dil, pad, Lq,
                                    _ptr(y), _ptr(ws), int(nb), _stream()), "stts_conv1d_fwd")
        ctx.save_for_backward(xf, wc)
        ctx.geo = (B, Lin, Cin, Cout, K, stride, dil, pad, Lq, dt, bias is not None)
        return y.transpose(1, 2)

    @staticmethod
    def backward(ctx, gy):
        xf, wc = ctx.saved_tensors
        B, Lin, Cin, Cout, K, stride, dil, pad, Lq, dt, has_bias = ctx.geo
        need_x, need_w, need_b = ctx.needs_input_grad[:3]
        dyf = _frames(gy)
        dev = dyf.device
        nb = lib().stts_conv1d_bwd_workspace_bytes(dt, B, Lin, Cin, Cout, K, stride, dil, pad, Lq)
        check(int(nb) if nb < 0 else 0, "stts_conv1d_bwd_workspace_bytes")
        ws = _ws(nb, dev)
        dx = torch.empty(B, Lin, Cin, dtype=torch.float32, device=dev) if need_x else None
        dw = torch.empty(Cout, Cin, K, dtype=torch.float32, device=dev) if need_w else None
        db = torch.empty(Cout, dtype=torch.float32, device=dev) if (need_b and has_bias) else None
        check(lib().stts_conv1d_bwd(dt, _ptr(xf), _ptr(wc), _ptr(dyf), B, Lin, Cin, Cout, K, stride, dil, pad, Lq,
                                    _ptr(dx), _ptr(dw), _ptr(db), _ptr(ws), int(nb), _stream()), "stts_conv1d_bwd")
        return (dx.transpose(1, 2) if dx is not None else None), dw, db, None, None, None, None


def conv1d(x, weight, bias=None, stride=1, padding=0, dilation=1, dtype="fp32"):
    """torch.nn.functional.conv1d (groups 1, zero padding) with forward and backward on the HIP
    conv engines.  dtype 'bf16' runs the forward and dx with bf16 operands (fp32 accumulation);
    dw / db are always fp32."""
    if dtype not in _DT:
        raise ValueError(f"dtype {dtype!r}: expected 'fp32' or 'bf16'")
    return _Conv1dFn.apply(x, weight, bias, int(stride), int(padding), int(dilation), dtype)


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
