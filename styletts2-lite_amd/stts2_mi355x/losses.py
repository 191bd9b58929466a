"""Training-step losses on the HIP path, drop-ins for losses.py:

* `MultiResolutionSTFTLoss(fft_sizes, hop_sizes, win_lengths, window=torch.hann_window)`
  (losses.py:66-94): forward(x, y) -> the mean over resolutions of ||y_mag - x_mag||_1 / ||y_mag||_1
  with x_mag = (log(1e-5 + MelSpectrogram(x)) + 4) / 4 (STFTLoss, :35-63), computed by
  `stts_mrstft_loss` (log-mel FFT kernel + fixed-order reductions).  train.py:282 calls it as
  `stft_loss(y_rec, wav)`.

Forward values only: the reference backpropagates through these with autograd; the HIP path has no
backward kernels yet.
"""
from __future__ import annotations

import ctypes

import torch
from torch import nn

from .engine import _dev_f32, _ptr, _require_device, _stream, check, lib


class MultiResolutionSTFTLoss(nn.Module):
    def __init__(self, fft_sizes=(1024, 2048, 512), hop_sizes=(120, 240, 50), win_lengths=(600, 1200, 240),
                 window=torch.hann_window, sample_rate=24000, n_mels=128):
        super().__init__()
        assert len(fft_sizes) == len(hop_sizes) == len(win_lengths)
        if window is not torch.hann_window:
            raise NotImplementedError("the HIP log-mel uses the reference's hann window")
        self.fft_sizes, self.hop_sizes, self.win_lengths = list(fft_sizes), list(hop_sizes), list(win_lengths)
        self.sample_rate, self.n_mels = int(sample_rate), int(n_mels)
        self._ws = None

    def forward(self, x, y):
        """x (predicted), y (ground truth): [B, T] or [B, 1, T] -> 0-dim float32 tensor on the device."""
        _require_device()
        dev = torch.device("cuda", torch.cuda.current_device())
        x, y = _dev_f32(x, dev), _dev_f32(y, dev)
        if x.shape != y.shape:
            raise ValueError(f"x {tuple(x.shape)} and y {tuple(y.shape)} differ")
        L = x.shape[-1]
        x2, y2 = x.reshape(-1, L), y.reshape(-1, L)
        B = x2.shape[0]
        n = len(self.fft_sizes)
        arr = lambda v: (ctypes.c_int * n)(*[int(t) for t in v])  # noqa: E731
        ffts, hops, wins = arr(self.fft_sizes), arr(self.hop_sizes), arr(self.win_lengths)
        nb = lib().stts_mrstft_workspace_bytes(B, L, hops, n, self.n_mels)
        check(int(nb) if nb < 0 else 0, "stts_mrstft_workspace_bytes")
        if self._ws is None or self._ws.numel() < nb or self._ws.device != dev:
            self._ws = torch.empty(int(nb), dtype=torch.uint8, device=dev)
        loss = torch.empty(1, dtype=torch.float64, device=dev)
        check(lib().stts_mrstft_loss(_ptr(x2), _ptr(y2), B, L, L, ffts, hops, wins, n, self.sample_rate, self.n_mels,
                                     _ptr(loss), _ptr(self._ws), int(nb), _stream()), "stts_mrstft_loss")
        return loss[0].float()
