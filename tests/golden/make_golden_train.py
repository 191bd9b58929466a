"""Golden fixtures for the assembled training step (BASELINE config 5), made by
running the REFERENCE modules and their own autograd in the survey container (never on the GPU box):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_train.py

What runs (train.py:267-327 restricted to the decoder and the discriminators):
  * Modules/hifigan.py Decoder (HIFI_CFG, style_dim 128, formula weights, eval as train.py:190 leaves it),
    Modules/discriminators.py MultiPeriodDiscriminator / MultiResSpecDiscriminator (formula weights
    "mpd." / "msd."), losses.py DiscriminatorLoss / GeneratorLoss / MultiResolutionSTFTLoss, and
    torch.optim.AdamW with optimizers.py:65-73's betas (0.0, 0.99), eps 1e-9, weight decay 1e-4;
  * y_rec = decoder(asr, F0, N, s); d_loss = dl(wav, y_rec.detach()); backward; AdamW on msd / mpd;
    g_loss = 5 stft_loss(y_rec, wav) + 1 gl(wav, y_rec); backward; AdamW on the decoder.
Stubs (import-time only, as the other fixture scripts): torchaudio (absent) — its MelSpectrogram,
needed by STFTLoss, is the oracle's restatement (oracle.mel_spectrogram_sr), so the mel loss part is
parity-unpinned upstream; SineGen's noise draws come from the formula (make_golden.NoisePatch);
SpecDiscriminator's CUDA-only `get_device` (make_golden_msd.py).
Stored as .npz DATA: the inputs' gradients in full, y_rec, the losses, and per parameter tensor of each
module a gradient summary (L2 norm, max |g|, the dot product with a formula probe vector, the values at
24 formula indices) and the AdamW update at those indices (tests/golden/train_step_B2_T8.npz).
It also runs the oracle's train_step on the same inputs and prints its deviation from the reference.
"""
from __future__ import annotations

import os
import random
import sys
import warnings

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, HERE)
sys.path.insert(0, ROOT)
from make_golden import HIFI_CFG, NoisePatch, fill  # noqa: E402
from make_golden_mpd import REF, import_losses, synth, waves  # noqa: E402

sys.path.insert(0, REF)
warnings.filterwarnings("ignore")

from oracle import stts_oracle as orc  # noqa: E402

NPROBE = 24
LR_DEC, LR_DISC = 1e-5, 1e-4  # Configs/config_example.yaml:94-95 (ft_lr for the decoder, lr for mpd / msd)


class OracleMel(torch.nn.Module):
    """torchaudio.transforms.MelSpectrogram stand-in (torchaudio is absent): the oracle's restatement."""

    def __init__(self, sample_rate=16000, n_fft=400, win_length=None, hop_length=None, window_fn=None, **kw):
        super().__init__()
        self.sr, self.n_fft, self.win, self.hop = sample_rate, n_fft, win_length or n_fft, hop_length
        assert not kw and window_fn is torch.hann_window

    def forward(self, x):
        return orc.mel_spectrogram_sr(x, self.sr, self.n_fft, self.win, self.hop)


def probe_idx(name, n):
    return np.minimum((synth.hash_u01("probe_idx." + name, NPROBE) * n).astype(np.int64), n - 1)


def summarize(tag, named, rec, deltas=None):
    names = sorted(named)
    l2, mx, dot, idx, val, dval = [], [], [], [], [], []
    for k in names:
        g = named[k].detach().reshape(-1).double().numpy()
        r = synth.normal("probe." + k, (g.size,)).astype(np.float64)
        ix = probe_idx(k, g.size)
        l2.append(np.sqrt((g * g).sum()))
        mx.append(np.abs(g).max())
        dot.append((g * r).sum())
        idx.append(ix)
        val.append(g[ix])
        if deltas is not None:
            dval.append(deltas[k].reshape(-1).double().numpy()[ix])
    rec[f"{tag}.names"] = np.array(names)
    rec[f"{tag}.l2"] = np.array(l2)
    rec[f"{tag}.maxabs"] = np.array(mx)
    rec[f"{tag}.dot"] = np.array(dot)
    rec[f"{tag}.idx"] = np.stack(idx)
    rec[f"{tag}.val"] = np.stack(val)
    if deltas is not None:
        rec[f"{tag}.delta"] = np.stack(dval)


def inputs(B, T):
    asr, f0, n, s = synth.decoder_inputs(B, T, tag="train")
    L = 600 * T
    wav = waves(B, L, 7)
    noise = synth.source_noise(B, L, tag="train_noise")
    return asr, f0, n, s, wav, noise


def main(B=2, T=8):
    torch.manual_seed(0)
    random.seed(0)
    from Modules.discriminators import MultiPeriodDiscriminator, MultiResSpecDiscriminator
    from Modules.hifigan import Decoder
    losses = import_losses()
    sys.modules["torchaudio"].transforms.MelSpectrogram = OracleMel
    dec = fill(Decoder(dim_in=512, style_dim=128, dim_out=80, **HIFI_CFG)).eval()
    mpd = fill(MultiPeriodDiscriminator(), "mpd.").train()
    msd = fill(MultiResSpecDiscriminator(), "msd.").train()
    p0 = {"dec": {k: v.detach().clone() for k, v in dec.state_dict().items()},
          "mpd": {k: v.detach().clone() for k, v in mpd.state_dict().items()},
          "msd": {k: v.detach().clone() for k, v in msd.state_dict().items()}}
    gl, dl = losses.GeneratorLoss(mpd, msd), losses.DiscriminatorLoss(mpd, msd)
    stft_loss = losses.MultiResolutionSTFTLoss()
    mk = lambda m, lr: torch.optim.AdamW(m.parameters(), lr=lr, weight_decay=1e-4, betas=(0.0, 0.99), eps=1e-9)  # noqa
    opt = {"dec": mk(dec, LR_DEC), "mpd": mk(mpd, LR_DISC), "msd": mk(msd, LR_DISC)}

    asr, f0, n, s, wav, noise = inputs(B, T)
    ins = {k: torch.from_numpy(v).requires_grad_(True) for k, v in (("asr", asr), ("F0_curve", f0), ("N", n), ("s", s))}
    wav_t = torch.from_numpy(wav)
    get_device = torch.Tensor.get_device
    torch.Tensor.get_device = lambda self: "cpu"
    rec = {}
    try:
        with NoisePatch(noise):
            y_rec = dec(ins["asr"], ins["F0_curve"], ins["N"], ins["s"])
        for o in opt.values():
            o.zero_grad()
        d_loss = dl(wav_t.detach(), y_rec.detach()).mean()
        d_loss.backward()
        summarize("grad.mpd", {k: p.grad for k, p in mpd.named_parameters()}, rec)
        summarize("grad.msd", {k: p.grad for k, p in msd.named_parameters()}, rec)
        opt["msd"].step()
        opt["mpd"].step()
        for o in opt.values():
            o.zero_grad()
        loss_mel = stft_loss(y_rec, wav_t)
        loss_gen_all = gl(wav_t, y_rec).mean()
        g_loss = 5.0 * loss_mel + 1.0 * loss_gen_all
        g_loss.backward()
        gdec = {k: p.grad for k, p in dec.named_parameters()}
        opt["dec"].step()
    finally:
        torch.Tensor.get_device = get_device
    deltas = {k: p.detach() - p0["dec"][k] for k, p in dec.named_parameters()}
    summarize("grad.dec", gdec, rec, deltas)
    dmpd = {k: p.detach() - p0["mpd"][k] for k, p in mpd.named_parameters()}
    rec["mpd.delta"] = np.stack([dmpd[k].reshape(-1).double().numpy()[probe_idx(k, dmpd[k].numel())]
                                 for k in sorted(dmpd)])
    for k, v in ins.items():
        rec["grad_in." + k] = v.grad.numpy()
    rec["y_rec"] = y_rec.detach().numpy()
    rec["d_loss"] = np.float64(d_loss.item())
    rec["loss_mel"] = np.float64(loss_mel.item())
    rec["loss_gen_all"] = np.float64(loss_gen_all.item())
    rec["g_loss"] = np.float64(g_loss.item())
    rec["B"], rec["T"] = np.int64(B), np.int64(T)
    rec["torch_version"] = np.array(torch.__version__)
    path = os.path.join(HERE, f"train_step_B{B}_T{T}.npz")
    np.savez_compressed(path, **rec)
    print(path, os.path.getsize(path), {k: float(rec[k]) for k in ("d_loss", "loss_mel", "loss_gen_all")})

    # the oracle on the same inputs
    ysd = lambda m: {k: v.detach().clone() for k, v in m.items()}  # noqa: E731
    y_o, l_o, g_o, _ = orc.train_step(ysd(p0["dec"]), ysd(p0["mpd"]), ysd(p0["msd"]), HIFI_CFG,
                                      *[torch.from_numpy(a) for a in (asr, f0, n, s)], wav_t, torch.from_numpy(noise),
                                      lr_dec=LR_DEC, lr_disc=LR_DISC)
    print("oracle y_rec max-abs", (y_o - y_rec.detach()).abs().max().item())
    print("oracle losses", l_o)
    worst = {}
    for tag, gref in (("dec", gdec), ("inputs", {k: v.grad for k, v in ins.items()})):
        for k, g in gref.items():
            go = g_o[tag][k]
            e = (go - g).abs().max().item() / max(g.abs().max().item(), 1e-30)
            worst[(tag, k)] = e
    top = sorted(worst.items(), key=lambda kv: -kv[1])[:8]
    print("oracle worst relative gradient errors:", top)


if __name__ == "__main__":
    main()
