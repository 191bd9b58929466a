"""Drop-in `models.ProsodyPredictor` and `models.StyleEncoder` (reference models.py).

Same constructor signatures and state-dict keys as the reference
(ProsodyPredictor models.py:394-466, StyleEncoder models.py:125-150), so checkpoints
load unchanged (reference inference.py:120-122, 158-168).

* `ProsodyPredictor.F0Ntrain(en, s)` (models.py:448-461): the shared BiLSTM (HIP recurrence,
  prosody.py), the F0 / N AdainResBlk1d conv stacks and the 1x1 projections run as HIP kernels
  through the C-ABI.
* `ProsodyPredictor.forward(texts, style, text_lengths, alignment, m)` (models.py:417-446) and
  `TextEncoder` (models.py:241-295): the duration path, prosody.py.
* `StyleEncoder.forward(mel)` (models.py:145-150): the whole 2-D ResNet runs as HIP kernels.
* Under autograd (train.py's G step differentiates both, train.py:258, 265, 318, 323-324) F0Ntrain and the
  StyleEncoder take the trainable HIP paths of training.py (f0ntrain, style_encoder) with their backward.
"""
from __future__ import annotations

import torch
import torch.nn as nn

from .params import AdainResBlk1d, Conv1d, Conv2d, Linear
from .prosody import LSTM, AdaLayerNorm, DurationEncoder, TextEncoder, linear_frames, matmul  # noqa: F401


class LinearNorm(nn.Module):
    """reference models.py:152-162 parameter layout (linear_layer)."""

    def __init__(self, in_dim, out_dim, bias=True):
        super().__init__()
        self.linear_layer = nn.Linear(in_dim, out_dim, bias=bias)

    def forward(self, x):
        return self.linear_layer(x)


class ProsodyPredictor(nn.Module):
    """reference models.py:394-466."""

    def __init__(self, style_dim, d_hid, nlayers, max_dur=50, dropout=0.1):
        super().__init__()
        self.style_dim, self.d_hid = int(style_dim), int(d_hid)
        self.text_encoder = DurationEncoder(sty_dim=style_dim, d_model=d_hid, nlayers=nlayers, dropout=dropout)
        self.lstm = LSTM(d_hid + style_dim, d_hid // 2, 1, batch_first=True, bidirectional=True)
        self.duration_proj = LinearNorm(d_hid, max_dur)
        self.shared = LSTM(d_hid + style_dim, d_hid // 2, 1, batch_first=True, bidirectional=True)
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

    def invalidate(self):
        """Drop the packed weights (after writes through `param.data`, which stale() cannot see)."""
        self._engine = None

    def f0n_engine(self, dtype="fp32"):
        from .engine import F0NEngine
        if self._engine is None or self._engine.dtype != dtype or self._engine.stale(self):
            self._engine = F0NEngine(self, dtype=dtype)
        return self._engine

    def forward(self, texts, style, text_lengths, alignment, m=None):
        """reference models.py:417-446: texts = TextEncoder output [B, d_hid, T], style [B, style_dim],
        alignment [B, T, F] -> (duration logits [B, T, max_dur], en [B, d_hid + style_dim, F]).

        Under autograd (train.py:230-233 differentiates it through loss_dur / loss_ce and en) the trainable path runs:
        texttrain.predictor_forward (packed BiLSTMs, AdaLayerNorms, the style concats, duration_proj and en = d^T aln,
        each with its HIP backward; dropout in train mode)."""
        from .texttrain import needs_grad
        if needs_grad(self, texts, style, alignment):
            from .texttrain import predictor_forward
            return predictor_forward(self, texts, style, text_lengths, alignment)
        from .engine import forward_only
        forward_only(self, "ProsodyPredictor")
        dev = self.F0_proj.weight.device
        texts, style, alignment = (t.to(dev, torch.float32) for t in (texts, style, alignment))
        with torch.no_grad():
            d = self.text_encoder(texts, style, text_lengths, m)  # [B, T, d_hid + style_dim]
            x, _ = self.lstm(d, lengths=text_lengths)  # pack -> LSTM -> pad (models.py:421-430)
            lin = self.duration_proj.linear_layer
            duration = linear_frames(x, lin.weight.detach(), lin.bias.detach())  # dropout: eval identity
            en = matmul(d.transpose(-1, -2), alignment)
        return duration.squeeze(-1), en

    def F0Ntrain(self, x, s, dtype="fp32"):
        """x = en [B, d_hid+style_dim, T], s [B, style_dim] -> (F0 [B,2T], N [B,2T]).

        Under autograd (grad mode on and a parameter or an input requiring grad, as train.py:265 calls it) the
        trainable path runs: training.f0ntrain (HIP BiLSTM forward / backward, the AdainResBlk1d stacks with their
        train-mode dropout, the projections); otherwise the fused inference engine."""
        dev = self.F0_proj.weight.device
        if torch.is_grad_enabled() and (any(p.requires_grad for p in self.parameters())
                                        or (isinstance(x, torch.Tensor) and x.requires_grad)
                                        or (isinstance(s, torch.Tensor) and s.requires_grad)):
            from .training import f0ntrain
            return f0ntrain(self, x.to(dev, torch.float32), s.to(dev, torch.float32), dtype)
        in_dev = x.device
        with torch.no_grad():
            h, _ = self.shared(x.to(dev, torch.float32).transpose(-1, -2))  # [B, T, d_hid] frames, HIP BiLSTM
        F0, N = self.f0n_engine(dtype).forward_nlc(h, s)
        return (F0, N) if in_dev.type == "cuda" else (F0.to(in_dev), N.to(in_dev))


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

    def invalidate(self):
        """Drop the packed weights (after writes through `param.data`, which stale() cannot see)."""
        self._engine = None

    def engine(self, dtype="fp32"):
        from .engine import StyleEngine
        if self._engine is None or self._engine.dtype != dtype or self._engine.stale(self):
            self._engine = StyleEngine(self, dtype=dtype)
        return self._engine

    def forward(self, x, dtype="fp32"):
        """mel [B,1,80,F] -> style [B, style_dim].  Under autograd (train.py:258, 324) the trainable path
        (training.style_encoder: the 2-D convs as row expansions + the conv1d engine, with backward); otherwise the
        fused inference engine."""
        if torch.is_grad_enabled() and (any(p.requires_grad for p in self.parameters())
                                        or (isinstance(x, torch.Tensor) and x.requires_grad)):
            from .training import style_encoder
            dev = self.unshared.weight.device
            return style_encoder(self, x.to(dev, torch.float32), dtype)
        return self.engine(dtype).forward(x)
