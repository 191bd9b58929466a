"""Drop-in MultiPeriodDiscriminator (Modules/discriminators.py:96-156) and MultiResSpecDiscriminator
(:29-94) for the training step: same constructors, sub-module names and
state-dict keys (`discriminators.{i}.convs.{j}.weight_g / weight_v / bias`, `discriminators.{i}.conv_post.*`;
`discriminators.{i}.discriminators.{j}.*`, `discriminators.{i}.out.*`).

Two paths behind one forward(y, y_hat):
  * autograd needed (grad enabled and a parameter or an input requires grad, as in train.py's D and G
    steps): the layer-by-layer HIP forward / backward of training.py (discriminator_p_forward,
    spec_discriminator_forward), gradients for the parameters and the inputs;
  * otherwise the fused forward engines (stts_mpd_fwd, stts_msd_fwd), packed weights, fp32 or bf16.
"""
from __future__ import annotations

import contextlib

import torch
from torch import nn
from torch.nn import Conv2d, Conv2d as _C2
from torch.nn.utils import weight_norm

LRELU_SLOPE = 0.1


def get_padding(kernel_size, dilation=1):
    return int((kernel_size * dilation - dilation) / 2)


class DiscriminatorP(nn.Module):
    """Parameter holder with the reference's layout (discriminators.py:96-106)."""

    def __init__(self, period, kernel_size=5, stride=3, use_spectral_norm=False):
        super().__init__()
        if use_spectral_norm or kernel_size != 5 or stride != 3:
            raise NotImplementedError("the HIP engine implements the reference's weight-norm k5 / s3 configuration")
        self.period = period
        self.convs = nn.ModuleList([
            weight_norm(Conv2d(1, 32, (kernel_size, 1), (stride, 1), padding=(get_padding(5, 1), 0))),
            weight_norm(Conv2d(32, 128, (kernel_size, 1), (stride, 1), padding=(get_padding(5, 1), 0))),
            weight_norm(Conv2d(128, 512, (kernel_size, 1), (stride, 1), padding=(get_padding(5, 1), 0))),
            weight_norm(Conv2d(512, 1024, (kernel_size, 1), (stride, 1), padding=(get_padding(5, 1), 0))),
            weight_norm(Conv2d(1024, 1024, (kernel_size, 1), 1, padding=(2, 0))),
        ])
        self.conv_post = weight_norm(Conv2d(1024, 1, (3, 1), 1, padding=(1, 0)))


class MultiPeriodDiscriminator(nn.Module):
    """MultiPeriodDiscriminator (discriminators.py:132-156) on the HIP engine.

    forward(y, y_hat) -> (y_d_rs, y_d_gs, fmap_rs, fmap_gs) as the reference: one score
    [B, L*p] and six feature maps [B, C, L, p] per period (the maps are permuted views of the
    engine's frames layout).  y and y_hat go through the engine as one batch."""

    def __init__(self, periods=(2, 3, 5, 7, 11)):
        super().__init__()
        self.discriminators = nn.ModuleList([DiscriminatorP(p) for p in periods])
        self._engine = None
        self.dtype_compute = "fp32"  # default dtype of forward() ('bf16': bf16 conv operands, fp32 accumulation)

    def engine(self, dtype="fp32"):
        from .engine import MPDEngine
        if self._engine is None or self._engine.dtype != dtype or self._engine.stale(self):
            self._engine = MPDEngine(self, dtype=dtype)
        return self._engine

    def invalidate(self):
        self._engine = None

    def forward(self, y, y_hat, dtype=None):
        dtype = dtype or self.dtype_compute
        if _needs_graph(self, y, y_hat):
            from .training import discriminator_p_forward
            return _train_forward(lambda d, x: discriminator_p_forward(d, x, d.period, dtype), self.discriminators,
                                  y, y_hat)
        B = y.shape[0]
        res = self.engine(dtype).forward(torch.cat([y, y_hat], 0))
        y_d_rs, y_d_gs, fmap_rs, fmap_gs = [], [], [], []
        for score, fmaps in res:
            y_d_rs.append(score[:B])
            y_d_gs.append(score[B:])
            fmap_rs.append([f[:B] for f in fmaps])
            fmap_gs.append([f[B:] for f in fmaps])
        return y_d_rs, y_d_gs, fmap_rs, fmap_gs


def _needs_graph(module, y, y_hat):
    """True when the caller will differentiate the outputs (train.py's D and G steps)."""
    if not torch.is_grad_enabled():
        return False
    return any(t.requires_grad for t in (y, y_hat) if isinstance(t, torch.Tensor)) or \
        any(p.requires_grad for p in module.parameters())


# the sub-discriminators (periods / resolutions) of one training forward run on their own HIP streams: their
# launches at config-5 sizes fill a fraction of the 256 CUs each (e.g. 192 tiles for an MPD 1024-channel conv), so
# they overlap; autograd runs each backward op on its forward's stream.  False = one stream (A/B, tests)
CONCURRENT = True
_STREAMS = {}


def _side_streams(n, dev):
    key = (dev.index, n)
    if key not in _STREAMS:
        _STREAMS[key] = [torch.cuda.Stream(device=dev) for _ in range(n)]
    return _STREAMS[key]


def _train_forward(run, discs, y, y_hat):
    """The reference's per-discriminator loop (discriminators.py:143-156 / :80-94) on the autograd path.  y and
    y_hat go through one batched call when they need the same graph (the D step: neither requires grad);
    otherwise separately, the side without a gradient under no_grad when no parameter needs one.  With
    CONCURRENT, sub-discriminator i runs on side stream i (ordered after the caller's stream, which waits for
    all of them before it uses the outputs)."""
    dev = torch.device("cuda", torch.cuda.current_device())
    y, y_hat = y.to(device=dev, dtype=torch.float32), y_hat.to(device=dev, dtype=torch.float32)
    B = y.shape[0]
    params_grad = any(p.requires_grad for d in discs for p in d.parameters())
    y_d_rs, y_d_gs, fmap_rs, fmap_gs = [], [], [], []
    main = torch.cuda.current_stream(dev)
    streams = _side_streams(len(discs), dev) if CONCURRENT and len(discs) > 1 else None
    for i, d in enumerate(discs):
        if streams is not None:
            st = streams[i]
            st.wait_stream(main)
            y.record_stream(st)
            y_hat.record_stream(st)
        with torch.cuda.stream(streams[i]) if streams is not None else contextlib.nullcontext():
            if y.requires_grad == y_hat.requires_grad:
                score, fmaps = run(d, torch.cat([y, y_hat], 0))
                r, fr = score[:B], [f[:B] for f in fmaps]
                g, fg = score[B:], [f[B:] for f in fmaps]
            else:
                with torch.set_grad_enabled(params_grad or y.requires_grad):
                    r, fr = run(d, y)
                g, fg = run(d, y_hat)
        y_d_rs.append(r)
        y_d_gs.append(g)
        fmap_rs.append(fr)
        fmap_gs.append(fg)
    if streams is not None:
        for st in streams:
            main.wait_stream(st)
        for t in [*y_d_rs, *y_d_gs, *(f for fs in fmap_rs + fmap_gs for f in fs)]:
            t.record_stream(main)  # made on a side stream, read on the caller's
    return y_d_rs, y_d_gs, fmap_rs, fmap_gs


def mpd_gan_losses(mpd: MultiPeriodDiscriminator, y, y_hat, dtype="fp32"):
    """One MPD forward of (y, y_hat) and, on the device, the reference's
    feature_loss(fmap_rs, fmap_gs), generator_loss(y_d_gs)[0] and discriminator_loss(y_d_rs, y_d_gs)[0]
    (losses.py:97-128) over its outputs -> (feature, generator, discriminator) float64 scalars."""
    with torch.no_grad():  # the fused forward engine (its outputs feed the device loss sums)
        mpd(y, y_hat, dtype=dtype)
    loss = mpd.engine(dtype).gan_losses()
    return loss[0], loss[1], loss[2]


class SpecDiscriminator(nn.Module):
    """Parameter holder with the reference's layout (discriminators.py:29-45)."""

    def __init__(self, fft_size=1024, shift_size=120, win_length=600, window="hann_window", use_spectral_norm=False):
        super().__init__()
        if use_spectral_norm or window != "hann_window":
            raise NotImplementedError("the HIP engine implements the reference's weight-norm / hann configuration")
        self.fft_size, self.shift_size, self.win_length = int(fft_size), int(shift_size), int(win_length)
        self.discriminators = nn.ModuleList([
            weight_norm(_C2(1, 32, kernel_size=(3, 9), padding=(1, 4))),
            weight_norm(_C2(32, 32, kernel_size=(3, 9), stride=(1, 2), padding=(1, 4))),
            weight_norm(_C2(32, 32, kernel_size=(3, 9), stride=(1, 2), padding=(1, 4))),
            weight_norm(_C2(32, 32, kernel_size=(3, 9), stride=(1, 2), padding=(1, 4))),
            weight_norm(_C2(32, 32, kernel_size=(3, 3), stride=(1, 1), padding=(1, 1))),
        ])
        self.out = weight_norm(_C2(32, 1, 3, 1, 1))


class MultiResSpecDiscriminator(nn.Module):
    """MultiResSpecDiscriminator (discriminators.py:65-94) on the HIP engine.

    forward(y, y_hat) -> (y_d_rs, y_d_gs, fmap_rs, fmap_gs) as the reference: per resolution a score
    [B, H*W] and six feature maps [B, C, H, W] (permuted views of the engine's [B][H][W][C] output).
    y and y_hat go through the engine as one batch.  (The reference's forward only runs on CUDA
    tensors: `self.window.to(y.get_device())`, :55; this one takes any device.)"""

    def __init__(self, fft_sizes=(1024, 2048, 512), hop_sizes=(120, 240, 50), win_lengths=(600, 1200, 240),
                 window="hann_window"):
        super().__init__()
        self.discriminators = nn.ModuleList([SpecDiscriminator(f, h, w, window)
                                             for f, h, w in zip(fft_sizes, hop_sizes, win_lengths)])
        self._engine = None
        self.dtype_compute = "fp32"  # default dtype of forward() ('bf16': bf16 conv operands, fp32 accumulation)

    def engine(self, dtype="fp32"):
        from .engine import MSDEngine
        if self._engine is None or self._engine.dtype != dtype or self._engine.stale(self):
            self._engine = MSDEngine(self, dtype=dtype)
        return self._engine

    def invalidate(self):
        self._engine = None

    def forward(self, y, y_hat, dtype=None):
        dtype = dtype or self.dtype_compute
        if _needs_graph(self, y, y_hat):
            from .training import spec_discriminator_forward
            return _train_forward(lambda d, x: spec_discriminator_forward(d, x, dtype), self.discriminators, y,
                                  y_hat)
        B = y.shape[0]
        res = self.engine(dtype).forward(torch.cat([y, y_hat], 0))
        y_d_rs, y_d_gs, fmap_rs, fmap_gs = [], [], [], []
        for score, fmaps in res:
            y_d_rs.append(score[:B])
            y_d_gs.append(score[B:])
            fmap_rs.append([f[:B] for f in fmaps])
            fmap_gs.append([f[B:] for f in fmaps])
        return y_d_rs, y_d_gs, fmap_rs, fmap_gs


def msd_gan_losses(msd: MultiResSpecDiscriminator, y, y_hat, dtype="fp32"):
    """As mpd_gan_losses, over the MultiResSpecDiscriminator outputs."""
    with torch.no_grad():  # the fused forward engine (its outputs feed the device loss sums)
        msd(y, y_hat, dtype=dtype)
    loss = msd.engine(dtype).gan_losses()
    return loss[0], loss[1], loss[2]
