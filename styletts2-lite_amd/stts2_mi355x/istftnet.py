"""Drop-in `Modules.istftnet.Decoder` (reference Modules/istftnet.py:660-721).

Same constructor signature and state-dict keys (including the CustomSTFT buffers
`generator.stft.*`, reference istftnet.py:111-203), forward = HIP decoder.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn as nn

from .params import AdaINResBlock1, AdainResBlk1d, Conv1d, SourceModuleHnNSF, WNConv1d, WNConvT1d


class CustomSTFT(nn.Module):
    """Buffers of reference istftnet.py:111-203 (conv-based STFT/iSTFT bases).

    window = periodic Hann(win_length); forward bases = cos / -sin(2*pi*k*n/N) * window;
    inverse bases = cos / sin(2*pi*n*k/N) * window / N.  Recomputed here from the
    published formula; a loaded checkpoint overwrites them anyway."""

    def __init__(self, filter_length=800, hop_length=200, win_length=800):
        super().__init__()
        self.filter_length = self.n_fft = int(filter_length)
        self.hop_length = int(hop_length)
        self.win_length = int(win_length)
        self.freq_bins = self.n_fft // 2 + 1
        window = torch.hann_window(win_length, periodic=True, dtype=torch.float32)
        if win_length < self.n_fft:
            window = torch.nn.functional.pad(window, (0, self.n_fft - win_length))
        elif win_length > self.n_fft:
            window = window[: self.n_fft]
        self.register_buffer("window", window)
        n = np.arange(self.n_fft)
        k = np.arange(self.freq_bins)
        ang = 2 * np.pi * np.outer(k, n) / self.n_fft
        w = window.numpy()
        self.register_buffer("weight_forward_real", torch.from_numpy(np.cos(ang) * w).float().unsqueeze(1))
        self.register_buffer("weight_forward_imag", torch.from_numpy(-np.sin(ang) * w).float().unsqueeze(1))
        ang_t = 2 * np.pi * np.outer(n, k) / self.n_fft
        iw = w * (1.0 / self.n_fft)
        self.register_buffer("weight_backward_real", torch.from_numpy(np.cos(ang_t).T * iw).float().unsqueeze(1))
        self.register_buffer("weight_backward_imag", torch.from_numpy(np.sin(ang_t).T * iw).float().unsqueeze(1))


class Generator(nn.Module):
    """parameter layout of reference istftnet.py:494-540."""

    def __init__(self, style_dim, resblock_kernel_sizes, upsample_rates, upsample_initial_channel,
                 resblock_dilation_sizes, upsample_kernel_sizes, gen_istft_n_fft, gen_istft_hop_size):
        super().__init__()
        self.num_kernels = len(resblock_kernel_sizes)
        self.num_upsamples = len(upsample_rates)
        self.upsample_rates = [int(u) for u in upsample_rates]
        self.upsample_kernel_sizes = [int(k) for k in upsample_kernel_sizes]
        self.resblock_kernel_sizes = [int(k) for k in resblock_kernel_sizes]
        self.resblock_dilation_sizes = [list(map(int, d)) for d in resblock_dilation_sizes]
        self.upsample_initial_channel = int(upsample_initial_channel)
        self.gen_istft_n_fft = int(gen_istft_n_fft)
        self.gen_istft_hop_size = int(gen_istft_hop_size)
        self.upsample_scale = int(np.prod(upsample_rates)) * int(gen_istft_hop_size)
        self.m_source = SourceModuleHnNSF(harmonic_num=8)
        self.noise_convs = nn.ModuleList()
        self.noise_res = nn.ModuleList()
        self.ups = nn.ModuleList()
        for i, (u, k) in enumerate(zip(upsample_rates, upsample_kernel_sizes)):
            self.ups.append(WNConvT1d(upsample_initial_channel // (2 ** i), upsample_initial_channel // (2 ** (i + 1)),
                                      k, u, padding=(k - u) // 2))
        self.resblocks = nn.ModuleList()
        ch = upsample_initial_channel
        for i in range(len(self.ups)):
            ch = upsample_initial_channel // (2 ** (i + 1))
            for k, d in zip(resblock_kernel_sizes, resblock_dilation_sizes):
                self.resblocks.append(AdaINResBlock1(ch, k, d, style_dim))
            c_cur = ch
            if i + 1 < len(upsample_rates):
                sf = int(np.prod(upsample_rates[i + 1:]))
                self.noise_convs.append(Conv1d(gen_istft_n_fft + 2, c_cur, sf * 2, stride=sf, padding=(sf + 1) // 2))
                self.noise_res.append(AdaINResBlock1(c_cur, 7, [1, 3, 5], style_dim))
            else:
                self.noise_convs.append(Conv1d(gen_istft_n_fft + 2, c_cur, 1))
                self.noise_res.append(AdaINResBlock1(c_cur, 11, [1, 3, 5], style_dim))
        self.post_n_fft = gen_istft_n_fft
        self.conv_post = WNConv1d(ch, self.post_n_fft + 2, 7, 1, padding=3)
        self.stft = CustomSTFT(filter_length=gen_istft_n_fft, hop_length=gen_istft_hop_size,
                               win_length=gen_istft_n_fft)


class Decoder(nn.Module):
    """reference istftnet.py:660-721; forward = HIP decoder (eval semantics)."""

    decoder_type = "istftnet"

    def __init__(self, dim_in=512, F0_channel=512, style_dim=64, dim_out=80,
                 resblock_kernel_sizes=[3, 7, 11], upsample_rates=[10, 6], upsample_initial_channel=512,
                 resblock_dilation_sizes=[[1, 3, 5], [1, 3, 5], [1, 3, 5]], upsample_kernel_sizes=[20, 12],
                 gen_istft_n_fft=20, gen_istft_hop_size=5):
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
                                   resblock_dilation_sizes, upsample_kernel_sizes, gen_istft_n_fft,
                                   gen_istft_hop_size)
        self._engine = None

    def invalidate(self):
        """Drop the packed weights (after writes through `param.data`, which stale() cannot see)."""
        self._engine = None

    def engine(self, dtype: str = "fp32"):
        from .engine import DecoderEngine
        if self._engine is None or self._engine.dtype != dtype or self._engine.stale(self):
            self._engine = DecoderEngine(self, dtype=dtype)
        return self._engine

    def forward(self, asr, F0_curve, N, s, noise=None, seed=None, utt_offset: int = 0, dtype: str = "fp32"):
        from .engine import forward_only
        forward_only(self, "istftnet.Decoder")
        return self.engine(dtype).forward(asr, F0_curve, N, s, noise=noise, seed=seed, utt_offset=utt_offset)
