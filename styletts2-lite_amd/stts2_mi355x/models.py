"""Drop-in `models.ProsodyPredictor` and `models.StyleEncoder` (reference models.py).

Same constructor signatures and state-dict keys as the reference
(ProsodyPredictor models.py:394-466, StyleEncoder models.py:125-150), so checkpoints
load unchanged (reference inference.py:120-122, 158-168).

* `ProsodyPredictor.F0Ntrain(en, s)` (models.py:448-461): the shared BiLSTM stays on
  PyTorch/MIOpen, the F0 / N AdainResBlk1d conv stacks and the
  1x1 projections run as HIP kernels through the C-ABI.
* `StyleEncoder.forward(mel)` (models.py:145-150): the whole 2-D ResNet runs as HIP kernels.
"""
from __future__ import annotations

import torch
import torch.nn as nn

from .params import AdainResBlk1d, Conv1d, Conv2d, Linear


class LinearNorm(nn.Module):
    """reference models.py:152-162 parameter layout (linear_layer)."""

    def __init__(self, in_dim, out_dim, bias=True):
        super().__init__()
        self.linear_layer = nn.Linear(in_dim, out_dim, bias=bias)

    def forward(self, x):
        return self.linear_layer(x)


class AdaLayerNorm(nn.Module):
    """reference models.py:372-392 parameter layout (fc)."""

    def __init__(self, style_dim, channels, eps=1e-5):
        super().__init__()
        self.channels, self.eps = channels, eps
        self.fc = nn.Linear(style_dim, channels * 2)


class DurationEncoder(nn.Module):
    """reference models.py:468-533 parameter layout (lstms = [LSTM, AdaLayerNorm] x nlayers).
    Out of the hot-path scope; parameters only."""

    def __init__(self, sty_dim, d_model, nlayers, dropout=0.1):
        super().__init__()
        self.lstms = nn.ModuleList()
        for _ in range(nlayers):
            self.lstms.append(nn.LSTM(d_model + sty_dim, d_model // 2, num_layers=1, batch_first=True,
                                      bidirectional=True))
            self.lstms.append(AdaLayerNorm(sty_dim, d_model))
        self.dropout, self.d_model, self.sty_dim = dropout, d_model, sty_dim


class ProsodyPredictor(nn.Module):
    """reference models.py:394-466."""

    def __init__(self, style_dim, d_hid, nlayers, max_dur=50, dropout=0.1):
        super().__init__()
        self.style_dim, self.d_hid = int(style_dim), int(d_hid)
        self.text_encoder = DurationEncoder(sty_dim=style_dim, d_model=d_hid, nlayers=nlayers, dropout=dropout)
        self.lstm = nn.LSTM(d_hid + style_dim, d_hid // 2, 1, batch_first=True, bidirectional=True)
        self.duration_proj = LinearNorm(d_hid, max_dur)
        self.shared = nn.LSTM(d_hid + style_dim, d_hid // 2, 1, batch_first=True, bidirectional=True)
        self.F0 = nn.ModuleList([
            AdainResBlk1d(d_hid, d_hid, style_dim, dropout_p=dropout),
            AdainResBlk1d(d_hid, d_hid // 2, style_dim, upsample=True, dropout_p=dropout),
            AdainResBlk1d(d_hid // 2, d_hid // 2, style_dim, dropout_p=dropout)])
        self.N = nn.ModuleList([
            AdainResBlk1d(d_hid, d_hid, style_dim, dropout_p=dropout),
            AdainResBlk1d(d_hid, d_hid // 2, style_dim, upsample=True, dropout_p=dropout),
            AdainResBlk1d(d_hid // 2, d_hid // 2, style_dim, dropout_p=dropout)])
        self.F0_proj = Conv1d(d_hid // 2, 1, 1)
        self.N_proj = Conv1d(d_hid // 2, 1, 1)
        self._engine = None

    def f0n_engine(self, dtype="fp32"):
        from .engine import F0NEngine
        if self._engine is None or self._engine.dtype != dtype or self._engine.stale(self):
            self._engine = F0NEngine(self, dtype=dtype)
        return self._engine

    def F0Ntrain(self, x, s, dtype="fp32"):
        """x = en [B, d_hid+style_dim, T], s [B, style_dim] -> (F0 [B,2T], N [B,2T])."""
        with torch.no_grad():
            self.shared.flatten_parameters() if x.is_cuda else None
            h, _ = self.shared(x.transpose(-1, -2))  # [B, T, d_hid] == NLC, consumed as-is
        return self.f0n_engine(dtype).forward_nlc(h.contiguous(), s)


class LearnedDownSample(nn.Module):
    """reference models.py:13-28 ('half': depthwise Conv2d k3 s2 p1)."""

    def __init__(self, layer_type, dim_in):
        super().__init__()
        self.layer_type = layer_type
        self.conv = Conv2d(dim_in, dim_in, 3, stride=2, padding=1, groups=dim_in)


class ResBlk(nn.Module):
    """reference models.py:82-123 (normalize=False, downsample='half')."""

    def __init__(self, dim_in, dim_out, downsample="half"):
        super().__init__()
        self.dim_in, self.dim_out = dim_in, dim_out
        self.learned_sc = dim_in != dim_out
        self.downsample_res = LearnedDownSample(downsample, dim_in)
        self.conv1 = Conv2d(dim_in, dim_in, 3, 1, 1)
        self.conv2 = Conv2d(dim_in, dim_out, 3, 1, 1)
        if self.learned_sc:
            self.conv1x1 = Conv2d(dim_in, dim_out, 1, 1, 0, bias=False)


class StyleEncoder(nn.Module):
    """reference models.py:125-150."""

    def __init__(self, dim_in=48, style_dim=48, max_conv_dim=384):
        super().__init__()
        blocks = [Conv2d(1, dim_in, 3, 1, 1)]
        dims = []
        for _ in range(4):
            dim_out = min(dim_in * 2, max_conv_dim)
            blocks.append(ResBlk(dim_in, dim_out, downsample="half"))
            dims.append((dim_in, dim_out))
            dim_in = dim_out
        blocks += [nn.LeakyReLU(0.2), Conv2d(dim_out, dim_out, 5, 1, 0), nn.AdaptiveAvgPool2d(1), nn.LeakyReLU(0.2)]
        self.shared = nn.Sequential(*blocks)
        self.unshared = Linear(dim_out, style_dim)
        self.style_dim, self.dims = style_dim, dims
        self._engine = None

    def engine(self, dtype="fp32"):
        from .engine import StyleEngine
        if self._engine is None or self._engine.dtype != dtype or self._engine.stale(self):
            self._engine = StyleEngine(self, dtype=dtype)
        return self._engine

    def forward(self, x, dtype="fp32"):
        """mel [B,1,80,F] -> style [B, style_dim]."""
        return self.engine(dtype).forward(x)
