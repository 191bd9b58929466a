"""Training-step losses on the HIP path, drop-ins for losses.py, with autograd:

* `MultiResolutionSTFTLoss(fft_sizes, hop_sizes, win_lengths, window=torch.hann_window)`
  (losses.py:58-94): forward(x, y) = the mean over resolutions of ||y_mag - x_mag||_1 / ||y_mag||_1 with
  x_mag = (log(1e-5 + MelSpectrogram(x)) + 4) / 4 (STFTLoss, :35-55), computed by `stts_mrstft_loss`;
  backward w.r.t. x (train.py:281 `stft_loss(y_rec, wav)`: x = y_rec) by `stts_mrstft_loss_bwd`.
* `feature_loss`, `generator_loss`, `discriminator_loss`, `discriminator_TPRLS_loss`,
  `generator_TPRLS_loss` (:97-147) and the `GeneratorLoss` / `DiscriminatorLoss` modules (:149-190):
  one `stts_gan_loss` launch sequence over all the terms of a call (fixed-order fp64 sums), gradients
  by `stts_gan_loss_bwd`.  They take the reference's lists of tensors (scores [B, n], feature maps of any
  layout as long as the real and generated maps of one layer share it).
"""
from __future__ import annotations

import ctypes

import torch
from torch import nn

from .engine import _ptr, _require_device, _stream, check
from .training import _f32, _tl, _ws

GAN_FEATURE, GAN_GEN, GAN_DISC, GAN_TPRLS = 0, 1, 2, 3


class _GanTerm(ctypes.Structure):
    _fields_ = [("a", ctypes.c_void_p), ("b", ctypes.c_void_p), ("n", ctypes.c_longlong), ("kind", ctypes.c_int)]


def _pair(r, g):
    """(r, g) as contiguous tensors with the same element order (a shared permutation of a permuted view,
    else copies): the terms are order-invariant reductions over aligned elements."""
    if r.shape != g.shape:
        raise ValueError(f"loss operands {tuple(r.shape)} and {tuple(g.shape)} differ")
    order = sorted(range(r.dim()), key=lambda d: (-r.stride(d), d))
    rp, gp = r.permute(order), g.permute(order)
    if rp.is_contiguous() and gp.is_contiguous() and rp.dtype == torch.float32 and gp.dtype == torch.float32:
        return rp, gp
    return r.float().contiguous(), g.float().contiguous()


class _GanFn(torch.autograd.Function):
    """Sum of GAN loss terms (kinds[i] over (ts[2i], ts[2i+1])) -> fp32 scalar; HIP forward and backward."""

    @staticmethod
    def forward(ctx, kinds, *ts):
        _require_device()
        n = len(kinds)
        terms = (_GanTerm * n)()
        for i, k in enumerate(kinds):
            a, b = ts[2 * i], ts[2 * i + 1]
            terms[i] = _GanTerm(a.data_ptr(), b.data_ptr(), a.numel(), int(k))
        nb = _tl().stts_gan_workspace_bytes(n)
        check(int(nb) if nb < 0 else 0, "stts_gan_workspace_bytes")
        ws = _ws(nb, ts[0].device)
        loss = torch.empty(1, dtype=torch.float64, device=ts[0].device)
        check(_tl().stts_gan_loss(terms, n, _ptr(loss), _ptr(ws), int(nb), _stream()), "stts_gan_loss")
        ctx.save_for_backward(*ts)
        ctx.kinds, ctx.ws, ctx.nb = kinds, ws, int(nb)
        return loss[0].to(torch.float32)

    @staticmethod
    def backward(ctx, go):
        ts = ctx.saved_tensors
        kinds = ctx.kinds
        n = len(kinds)
        need = ctx.needs_input_grad[1:]
        terms = (_GanTerm * n)()
        da = (ctypes.c_void_p * n)()
        db = (ctypes.c_void_p * n)()
        grads = []
        for i, k in enumerate(kinds):
            a, b = ts[2 * i], ts[2 * i + 1]
            terms[i] = _GanTerm(a.data_ptr(), b.data_ptr(), a.numel(), int(k))
            ga = torch.empty_like(a) if need[2 * i] else None
            gb = torch.empty_like(b) if need[2 * i + 1] else None
            da[i] = ga.data_ptr() if ga is not None else None
            db[i] = gb.data_ptr() if gb is not None else None
            grads += [ga, gb]
        g = _f32(go.reshape(1))
        check(_tl().stts_gan_loss_bwd(terms, da, db, n, _ptr(g), _ptr(ctx.ws), ctx.nb, _stream()),
              "stts_gan_loss_bwd")
        return (None, *grads)


def gan_terms(terms):
    """terms: list of (kind, a, b) -> the fp32 scalar sum, differentiable w.r.t. every a / b."""
    kinds, ts = [], []
    for kind, a, b in terms:
        a2, b2 = _pair(a, b)
        kinds.append(int(kind))
        ts += [a2, b2]
    return _GanFn.apply(tuple(kinds), *ts)


def feature_loss(fmap_r, fmap_g):
    """losses.py:97-103: 2 * sum over discriminators and layers of mean|rl - gl|."""
    return gan_terms([(GAN_FEATURE, rl, gl) for dr, dg in zip(fmap_r, fmap_g) for rl, gl in zip(dr, dg)])


def generator_loss(disc_outputs):
    """losses.py:120-128 -> (loss, [per-output losses])."""
    per = [gan_terms([(GAN_GEN, dg, dg)]) for dg in disc_outputs]
    return gan_terms([(GAN_GEN, dg, dg) for dg in disc_outputs]), per


def discriminator_loss(disc_real_outputs, disc_generated_outputs):
    """losses.py:106-117 -> (loss, r_losses, g_losses) (the per-output values as Python floats)."""
    loss = gan_terms([(GAN_DISC, dr, dg) for dr, dg in zip(disc_real_outputs, disc_generated_outputs)])
    with torch.no_grad():
        r = [float(gan_terms([(GAN_GEN, dr, dr)])) for dr in disc_real_outputs]  # mean((1 - dr)^2)
        g = [float(gan_terms([(GAN_DISC, torch.ones_like(dg), dg)])) for dg in disc_generated_outputs]
    return loss, r, g


def discriminator_TPRLS_loss(disc_real_outputs, disc_generated_outputs):
    """losses.py:131-138."""
    return gan_terms([(GAN_TPRLS, dr, dg) for dr, dg in zip(disc_real_outputs, disc_generated_outputs)])


def generator_TPRLS_loss(disc_real_outputs, disc_generated_outputs):
    """losses.py:140-147 (its loop binds the real outputs to `dg`: m = median(generated - real))."""
    return gan_terms([(GAN_TPRLS, g, r) for r, g in zip(disc_real_outputs, disc_generated_outputs)])


class GeneratorLoss(nn.Module):
    """losses.py:149-168: feature + generator + TPRLS losses over the MPD and MSD outputs, as one term list."""

    def __init__(self, mpd, msd):
        super().__init__()
        self.mpd = mpd
        self.msd = msd

    def forward(self, y, y_hat):
        y_df_hat_r, y_df_hat_g, fmap_f_r, fmap_f_g = self.mpd(y, y_hat)
        y_ds_hat_r, y_ds_hat_g, fmap_s_r, fmap_s_g = self.msd(y, y_hat)
        terms = []
        # loss_gen_s + loss_gen_f + loss_fm_s + loss_fm_f + loss_rel (the reference's sum; the sum order of
        # the fp64 term values differs from its fp32 additions only in rounding)
        terms += [(GAN_GEN, g, g) for g in y_ds_hat_g]
        terms += [(GAN_GEN, g, g) for g in y_df_hat_g]
        terms += [(GAN_FEATURE, rl, gl) for dr, dg in zip(fmap_s_r, fmap_s_g) for rl, gl in zip(dr, dg)]
        terms += [(GAN_FEATURE, rl, gl) for dr, dg in zip(fmap_f_r, fmap_f_g) for rl, gl in zip(dr, dg)]
        terms += [(GAN_TPRLS, g, r) for r, g in zip(y_df_hat_r, y_df_hat_g)]
        terms += [(GAN_TPRLS, g, r) for r, g in zip(y_ds_hat_r, y_ds_hat_g)]
        return gan_terms(terms)


class DiscriminatorLoss(nn.Module):
    """losses.py:170-190: discriminator + TPRLS losses over the MPD and MSD outputs."""

    def __init__(self, mpd, msd):
        super().__init__()
        self.mpd = mpd
        self.msd = msd

    def forward(self, y, y_hat):
        y_df_hat_r, y_df_hat_g, _, _ = self.mpd(y, y_hat)
        y_ds_hat_r, y_ds_hat_g, _, _ = self.msd(y, y_hat)
        terms = [(GAN_DISC, r, g) for r, g in zip(y_ds_hat_r, y_ds_hat_g)]
        terms += [(GAN_DISC, r, g) for r, g in zip(y_df_hat_r, y_df_hat_g)]
        terms += [(GAN_TPRLS, r, g) for r, g in zip(y_df_hat_r, y_df_hat_g)]
        terms += [(GAN_TPRLS, r, g) for r, g in zip(y_ds_hat_r, y_ds_hat_g)]
        return gan_terms(terms)


# ---------------------------------------------------------------------- multi-resolution mel loss
class _MrstftFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x2, y2, mod):
        B, L = x2.shape
        n = len(mod.fft_sizes)
        arr = lambda v: (ctypes.c_int * n)(*[int(t) for t in v])  # noqa: E731
        ffts, hops, wins = arr(mod.fft_sizes), arr(mod.hop_sizes), arr(mod.win_lengths)
        xc, yc = _f32(x2), _f32(y2)
        dev = xc.device
        nb = _tl().stts_mrstft_workspace_bytes(B, L, hops, n, mod.n_mels)
        check(int(nb) if nb < 0 else 0, "stts_mrstft_workspace_bytes")
        ws = _ws(nb, dev)
        loss = torch.empty(1, dtype=torch.float64, device=dev)
        check(_tl().stts_mrstft_loss(_ptr(xc), _ptr(yc), B, L, L, ffts, hops, wins, n, mod.sample_rate, mod.n_mels,
                                     _ptr(loss), _ptr(ws), int(nb), _stream()), "stts_mrstft_loss")
        ctx.save_for_backward(xc, yc)
        ctx.mod = mod
        return loss[0].to(torch.float32)

    @staticmethod
    def backward(ctx, go):
        xc, yc = ctx.saved_tensors
        mod = ctx.mod
        if ctx.needs_input_grad[1]:
            raise NotImplementedError("MultiResolutionSTFTLoss backward w.r.t. the target y (train.py:281 "
                                      "differentiates the prediction x only)")
        if not ctx.needs_input_grad[0]:
            return None, None, None
        B, L = xc.shape
        n = len(mod.fft_sizes)
        arr = lambda v: (ctypes.c_int * n)(*[int(t) for t in v])  # noqa: E731
        ffts, hops, wins = arr(mod.fft_sizes), arr(mod.hop_sizes), arr(mod.win_lengths)
        nb = _tl().stts_mrstft_bwd_workspace_bytes(B, L, ffts, hops, wins, n, mod.n_mels)
        check(int(nb) if nb < 0 else 0, "stts_mrstft_bwd_workspace_bytes")
        ws = _ws(nb, xc.device)
        dx = torch.empty_like(xc)
        g = _f32(go.reshape(1))
        check(_tl().stts_mrstft_loss_bwd(_ptr(xc), _ptr(yc), B, L, L, ffts, hops, wins, n, mod.sample_rate,
                                         mod.n_mels, _ptr(g), _ptr(dx), _ptr(ws), int(nb), _stream()),
              "stts_mrstft_loss_bwd")
        return dx, None, None


class MultiResolutionSTFTLoss(nn.Module):
    def __init__(self, fft_sizes=(1024, 2048, 512), hop_sizes=(120, 240, 50), win_lengths=(600, 1200, 240),
                 window=torch.hann_window, sample_rate=24000, n_mels=128):
        super().__init__()
        assert len(fft_sizes) == len(hop_sizes) == len(win_lengths)
        if window is not torch.hann_window:
            raise NotImplementedError("the HIP log-mel uses the reference's hann window")
        self.fft_sizes, self.hop_sizes, self.win_lengths = list(fft_sizes), list(hop_sizes), list(win_lengths)
        self.sample_rate, self.n_mels = int(sample_rate), int(n_mels)

    def forward(self, x, y):
        """x (predicted), y (ground truth): [B, T] or [B, 1, T] device tensors -> 0-dim float32 tensor,
        differentiable w.r.t. x."""
        _require_device()
        if x.shape != y.shape:
            raise ValueError(f"x {tuple(x.shape)} and y {tuple(y.shape)} differ")
        L = x.shape[-1]
        dev = torch.device("cuda", torch.cuda.current_device())
        x2 = x.reshape(-1, L).to(dev)
        y2 = y.reshape(-1, L).to(dev)
        return _MrstftFn.apply(x2, y2, self)


class _SmoothL1Fn(torch.autograd.Function):
    """F.smooth_l1_loss(x, y) (beta 1, mean): stts_smooth_l1_loss / _bwd."""

    @staticmethod
    def forward(ctx, x, y):
        _require_device()
        xc, yc = _f32(x), _f32(y)
        if xc.shape != yc.shape:
            raise ValueError(f"smooth_l1_loss: {tuple(xc.shape)} vs {tuple(yc.shape)}")
        loss = torch.empty(1, dtype=torch.float64, device=xc.device)
        check(_tl().stts_smooth_l1_loss(_ptr(xc), _ptr(yc), xc.numel(), _ptr(loss), _stream()), "stts_smooth_l1_loss")
        ctx.save_for_backward(xc, yc)
        return loss[0].to(torch.float32)

    @staticmethod
    def backward(ctx, g):
        xc, yc = ctx.saved_tensors
        nx, ny = ctx.needs_input_grad
        gd = _f32(g.reshape(1))
        dx = torch.empty_like(xc) if nx else None
        dy = torch.empty_like(yc) if ny else None
        check(_tl().stts_smooth_l1_loss_bwd(_ptr(xc), _ptr(yc), xc.numel(), _ptr(gd), _ptr(dx), _ptr(dy), _stream()),
              "stts_smooth_l1_loss_bwd")
        return dx, dy


def smooth_l1_loss(x, y):
    """F.smooth_l1_loss(x, y) as train.py:269-270 calls it (loss_F0_rec = smooth_l1(F0_real, F0_fake) / 10,
    loss_norm_rec = smooth_l1(N_real, N_fake))."""
    return _SmoothL1Fn.apply(x, y)
