"""Drop-in `Modules.hifigan.Decoder` (reference Modules/hifigan.py:416-475).

Same constructor signature, same sub-module names and state-dict keys (678 keys,
54,289,492 parameters at style_dim=128), so
`Decoder(...).load_state_dict(ckpt['net']['decoder'])` works unchanged
(reference inference.py:104-111, 158-168).  `forward(asr, F0_curve, N, s)` runs the
whole decoder as HIP kernels for gfx950 through the C-ABI library
(`include/stts2.h`, `stts_decoder_fwd`); there is no PyTorch compute fallback.

When the caller will differentiate the output (grad enabled and a parameter or an input requires grad:
train.py:267 under the G step's backward, :318), the forward instead runs the layer-by-layer HIP
forward / backward of training.decoder_forward, which returns a graph: every parameter, asr, F0_curve,
N and s get their gradients.  In .train() mode the F0 / N smoothing of hifigan.py:447-455 is applied on
both paths (Python's random, as the reference).
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn as nn

from .params import (AdaINResBlock1, AdainResBlk1d, Conv1d, SourceModuleHnNSF, WNConv1d,
                     WNConvT1d)


class Generator(nn.Module):
    """parameter layout of reference hifigan.py:272-319."""

    def __init__(self, style_dim, resblock_kernel_sizes, upsample_rates, upsample_initial_channel,
                 resblock_dilation_sizes, upsample_kernel_sizes):
        super().__init__()
        self.num_kernels = len(resblock_kernel_sizes)
        self.num_upsamples = len(upsample_rates)
        self.upsample_rates = [int(u) for u in upsample_rates]
        self.upsample_kernel_sizes = [int(k) for k in upsample_kernel_sizes]
        self.resblock_kernel_sizes = [int(k) for k in resblock_kernel_sizes]
        self.resblock_dilation_sizes = [list(map(int, d)) for d in resblock_dilation_sizes]
        self.upsample_initial_channel = int(upsample_initial_channel)
        self.upsample_scale = int(np.prod(upsample_rates))
        self.m_source = SourceModuleHnNSF(harmonic_num=8)
        self.noise_convs = nn.ModuleList()
        self.ups = nn.ModuleList()
        self.noise_res = nn.ModuleList()
        for i, (u, k) in enumerate(zip(upsample_rates, upsample_kernel_sizes)):
            c_cur = upsample_initial_channel // (2 ** (i + 1))
            self.ups.append(WNConvT1d(upsample_initial_channel // (2 ** i), c_cur, k, u,
                                      padding=(u // 2 + u % 2), output_padding=u % 2))
            if i + 1 < len(upsample_rates):
                sf = int(np.prod(upsample_rates[i + 1:]))
                self.noise_convs.append(Conv1d(1, c_cur, sf * 2, stride=sf, padding=(sf + 1) // 2))
                self.noise_res.append(AdaINResBlock1(c_cur, 7, [1, 3, 5], style_dim))
            else:
                self.noise_convs.append(Conv1d(1, c_cur, 1))
                self.noise_res.append(AdaINResBlock1(c_cur, 11, [1, 3, 5], style_dim))
        self.resblocks = nn.ModuleList()
        self.alphas = nn.ParameterList()
        self.alphas.append(nn.Parameter(torch.ones(1, upsample_initial_channel, 1)))
        ch = upsample_initial_channel
        for i in range(len(self.ups)):
            ch = upsample_initial_channel // (2 ** (i + 1))
            self.alphas.append(nn.Parameter(torch.ones(1, ch, 1)))
            for k, d in zip(resblock_kernel_sizes, resblock_dilation_sizes):
                self.resblocks.append(AdaINResBlock1(ch, k, d, style_dim))
        self.conv_post = WNConv1d(ch, 1, 7, 1, padding=3)


class Decoder(nn.Module):
    """reference hifigan.py:416-475; forward = the fused HIP decoder, or the autograd path (module docstring)."""

    decoder_type = "hifigan"

    def __init__(self, dim_in=512, F0_channel=512, style_dim=64, dim_out=80,
                 resblock_kernel_sizes=[3, 7, 11], upsample_rates=[10, 5, 3, 2],
                 upsample_initial_channel=512, resblock_dilation_sizes=[[1, 3, 5], [1, 3, 5], [1, 3, 5]],
                 upsample_kernel_sizes=[20, 10, 6, 4]):
        super().__init__()
        self.dim_in, self.style_dim = int(dim_in), int(style_dim)
        self.decode = nn.ModuleList()
        self.encode = AdainResBlk1d(dim_in + 2, 1024, style_dim)
        self.decode.append(AdainResBlk1d(1024 + 2 + 64, 1024, style_dim))
        self.decode.append(AdainResBlk1d(1024 + 2 + 64, 1024, style_dim))
        self.decode.append(AdainResBlk1d(1024 + 2 + 64, 1024, style_dim))
        self.decode.append(AdainResBlk1d(1024 + 2 + 64, 512, style_dim, upsample=True))
        self.F0_conv = WNConv1d(1, 1, 3, stride=2, padding=1)
        self.N_conv = WNConv1d(1, 1, 3, stride=2, padding=1)
        self.asr_res = nn.Sequential(WNConv1d(512, 64, 1))
        self.generator = Generator(style_dim, resblock_kernel_sizes, upsample_rates, upsample_initial_channel,
                                   resblock_dilation_sizes, upsample_kernel_sizes)
        self._engine = None

    # -- HIP path ------------------------------------------------------------------
    def invalidate(self):
        """Drop the packed weights (after writes through `param.data`, which stale() cannot see)."""
        self._engine = None

    def engine(self, dtype: str = "fp32"):
        from .engine import DecoderEngine
        if self._engine is None or self._engine.dtype != dtype or self._engine.stale(self):
            self._engine = DecoderEngine(self, dtype=dtype)
        return self._engine

    def forward(self, asr, F0_curve, N, s, noise=None, seed=None, utt_offset: int = 0, dtype: str = "fp32"):
        """asr [B,512,T], F0_curve [B,2T], N [B,2T], s [B,style_dim] -> [B,1,600T] (float32).

        `noise` [B,600T,9] is the reference's randn_like(sine_waves) draw (hifigan.py:213);
        None draws it on the device from a counter RNG keyed by (seed, utt_offset + b, sample,
        harmonic); seed None takes one draw from torch's default generator (torch.manual_seed
        governs it and successive calls differ, as the reference's draws do)."""
        from . import training
        if torch.is_grad_enabled() and (any(p.requires_grad for p in self.parameters()) or any(
                isinstance(t, torch.Tensor) and t.requires_grad for t in (asr, F0_curve, N, s))):
            return training.decoder_forward(self, asr, F0_curve, N, s, noise=noise, seed=seed, utt_offset=utt_offset,
                                            dtype=dtype)
        if self.training:
            dev = torch.device("cuda", torch.cuda.current_device())
            F0_curve, N = training.train_smooth(torch.as_tensor(F0_curve).to(dev, torch.float32),
                                                torch.as_tensor(N).to(dev, torch.float32))
        return self.engine(dtype).forward(asr, F0_curve, N, s, noise=noise, seed=seed, utt_offset=utt_offset)
