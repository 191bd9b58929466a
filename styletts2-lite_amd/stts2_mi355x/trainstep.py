"""One fine-tune step of the decoder against the discriminators, as train.py:267-327 runs it (BASELINE
config 5), over the drop-in modules: the HIP decoder (hifigan.Decoder, autograd path), the MPD / MSD
(discriminators.py), the losses (losses.py) and AdamW (optim.py).

    step = TrainStep(decoder, mpd, msd)
    losses = step(en, F0_fake, N_fake, s, wav)   # en [B, 512, T], F0 / N [B, 2T], s [B, style_dim], wav [B, 1, 600 T]

does, in the reference's order:
    y_rec = decoder(en, F0_fake, N_fake, s)                                     (train.py:267)
    zero_grad; d_loss = dl(wav.detach(), y_rec.detach()).mean(); backward;
    AdamW step on msd, mpd                                                       (:272-276)
    zero_grad; loss_mel = stft_loss(y_rec, wav); loss_gen_all = gl(wav, y_rec).mean();
    g_loss = lambda_mel loss_mel + lambda_gen loss_gen_all; backward; AdamW on the decoder   (:278-325)
By default the other modules of train.py (text aligner, predictor, style encoder) are outside the step: their
outputs come in as tensors, and their gradients (en.grad, F0.grad, N.grad, s.grad) are left on the inputs when those
require grad.  With `predictor=` and `style_encoder=` the G step also runs them as train.py:258-270 does:

    losses = step(en, None, None, None, wav, p_en=p_en, gt=gt_mel, F0_real=F0_real, N_real=N_real)

computes s = style_encoder(gt.unsqueeze(1)), (F0_fake, N_fake) = predictor.F0Ntrain(p_en, s) (the predictor in
train mode: its dropout), y_rec = decoder(en, F0_fake, N_fake, s), adds lambda_F0 smooth_l1(F0_real, F0_fake) / 10
and lambda_norm smooth_l1(N_real, N_fake) to g_loss (:269-270, 300-307; F0_real comes from the pitch extractor and
N_real = log_norm(gt), both outside this path) and steps AdamW on the predictor and the style encoder after the
decoder's backward (:323-324).  With `text_encoder=` (and the predictor) the step starts where train.py's G step starts
(train.py:217-262), from the tokens:

    losses = step(None, None, None, None, wav, gt=None, F0_real=F0_real, N_real=N_real,
                  text=dict(texts=, input_lengths=, attn=, attn_mono=, mels=, starts=, mel_len=))

t_en = text_encoder(texts, input_lengths) (:217), asr = t_en @ attn (:220-223; attn = s2s_attn or its monotonic
version, the caller's coin), d_gt = attn_mono.sum(-1) (:225), s = style_encoder(mels) (:228), (d, p) =
predictor(t_en, s, input_lengths, attn_mono) (:230-233), the per-utterance crops en / p_en / gt of mel_len frames at
`starts` (:235-251; the caller draws them, as train.py's np.random.randint), then the step above with en, p_en, gt,
plus lambda_dur loss_dur + lambda_ce loss_ce (:286-299, texttrain.duration_losses) in g_loss and AdamW on the text
encoder after the backward (:327).  The aligner's own losses (loss_s2s, loss_mono) and its optimizer step belong to
the text aligner, outside this path; the gradient of asr with respect to attn is left on attn when it requires grad.
`graph=True` (the config-5 step: decoder + discriminators): the step is recorded once in a hipGraph and replayed;
the host then issues one graph launch per step instead of ~5,000 kernel launches through Python autograd.  Every
per-step host scalar lives on the device: the AdamW step counts (optim.AdamW(capturable=True), stts_adamw_step_dev)
and the noise seed (stts_source_fwd_seed_dev, written before each replay).  Call 1 runs eagerly (it also warms the
kernels' one-time setup), call 2 records the graph and replays it, later calls copy their inputs into the graph's
static buffers and replay.  The returned losses are the graph's static outputs (overwritten by the next replay) and
the input gradients land on `static_inputs`; optimizer state["step"] follows after AdamW.sync_steps().
`freeze_d_in_g` (default) turns off requires_grad of the discriminator parameters
during the G step: the reference computes those gradients and discards them (its next iteration starts
with zero_grad before they are used), so skipping them changes no update.
"""
from __future__ import annotations

import torch

from .losses import DiscriminatorLoss, GeneratorLoss, MultiResolutionSTFTLoss, smooth_l1_loss
from .optim import AdamW


def seed_i64(seed):
    """The 64 seed bits the eager path passes as an unsigned long long (training._SourceFn), as the int64 the
    recorded graph's kernel reads (same bits: no seed maps to another stream on one path only)."""
    v = int(seed) & (2 ** 64 - 1)
    return v - 2 ** 64 if v >= 2 ** 63 else v


class TrainStep:
    def __init__(self, decoder, mpd, msd, lr_dec=1e-5, lr_disc=1e-4, lambda_mel=5.0, lambda_gen=1.0, dtype="fp32",
                 freeze_d_in_g=True, capture=False, predictor=None, style_encoder=None, lr_pred=1e-4, lr_style=1e-5,
                 lambda_F0=1.0, lambda_norm=1.0, text_encoder=None, lr_text=1e-4, lambda_dur=1.0, lambda_ce=1.0,
                 graph=False):
        self.decoder, self.mpd, self.msd = decoder, mpd, msd
        self.predictor, self.style_encoder, self.text_encoder = predictor, style_encoder, text_encoder
        self.lambda_dur, self.lambda_ce = float(lambda_dur), float(lambda_ce)
        self.lambda_F0, self.lambda_norm = float(lambda_F0), float(lambda_norm)
        self.capture = capture  # keep copies of the gradients each optimizer step consumed (tests)
        self.captured = {}
        self.dtype = dtype  # the discriminators take it for the duration of each step only (__call__)
        self.gl, self.dl = GeneratorLoss(mpd, msd), DiscriminatorLoss(mpd, msd)
        self.stft_loss = MultiResolutionSTFTLoss()
        self.graph = bool(graph)
        self._graph, self._calls, self.static_inputs, self._static_out = None, 0, None, None
        mk = lambda m, lr: AdamW(m.parameters(), lr=lr, weight_decay=1e-4, betas=(0.0, 0.99), eps=1e-9,  # noqa: E731
                                 capturable=self.graph)
        self.opt = {"decoder": mk(decoder, lr_dec), "mpd": mk(mpd, lr_disc), "msd": mk(msd, lr_disc)}
        # train.py:137-157: the predictor at the general lr, the style encoder at the acoustic ft_lr
        if predictor is not None:
            self.opt["predictor"] = mk(predictor, lr_pred)
        if style_encoder is not None:
            self.opt["style_encoder"] = mk(style_encoder, lr_style)
        if text_encoder is not None:  # train.py:137-157: the text encoder at the general lr
            self.opt["text_encoder"] = mk(text_encoder, lr_text)
        self.lambda_mel, self.lambda_gen = float(lambda_mel), float(lambda_gen)
        self.freeze_d_in_g = freeze_d_in_g

    def zero_grad(self):
        for o in self.opt.values():
            o.zero_grad()

    def __call__(self, en, F0, N, s, wav, noise=None, seed=None, p_en=None, gt=None, F0_real=None, N_real=None,
                 text=None):
        saved = (self.mpd.dtype_compute, self.msd.dtype_compute)
        self.mpd.dtype_compute = self.msd.dtype_compute = self.dtype
        try:
            if self.graph:
                if any(v is not None for v in (p_en, gt, F0_real, N_real, text)):
                    raise NotImplementedError("TrainStep(graph=True) records the config-5 step (decoder + "
                                              "discriminators); the predictor / style / text options run eagerly")
                return self._graphed(en, F0, N, s, wav, noise, seed)
            return self._step(en, F0, N, s, wav, noise, seed, p_en, gt, F0_real, N_real, text)
        finally:  # other users of the same discriminators keep their own compute dtype
            self.mpd.dtype_compute, self.msd.dtype_compute = saved

    def _graphed(self, en, F0, N, s, wav, noise, seed):
        """The recorded step (graph=True): see the module docstring."""
        if seed is None and noise is None:
            seed = int(torch.randint(0, 2 ** 62, (1,)).item())  # (a CPU draw: no device sync)
        if self.decoder.training:
            # train mode draws the F0 / N smoothing with Python's random on the host (hifigan.py:447-455): a recorded
            # graph would replay the first draw forever
            raise ValueError("TrainStep(graph=True) needs the decoder in eval mode (its train-mode smoothing is a "
                             "host-side random draw per step)")
        self._calls += 1
        if self._calls == 1:  # eager: the kernels' one-time setup, the optimizers' device state
            return self._step(en, F0, N, s, wav, noise, seed, None, None, None, None)
        if self._graph is None:
            dev = wav.device
            st = {k: t.detach().clone().requires_grad_(t.requires_grad) for k, t in
                  (("en", en), ("F0", F0), ("N", N), ("s", s))}
            st["wav"] = wav.detach().clone()
            st["noise"] = noise.detach().clone() if noise is not None else None
            st["seed"] = torch.zeros(1, dtype=torch.int64, device=dev)
            self.static_inputs = st
            self._fill(en, F0, N, s, wav, noise, seed)
            g = torch.cuda.CUDAGraph()
            # (the eager call already ran every kernel once on this stream: no side-stream warm-up needed)
            with torch.cuda.graph(g):
                self._static_out = self._step(st["en"], st["F0"], st["N"], st["s"], st["wav"], st["noise"],
                                              None if st["noise"] is not None else st["seed"], None, None, None, None)
            self._graph = g
            # the learning rates are host scalars baked into the recorded AdamW launches
            self._lrs = self._lr_snapshot()
        else:
            if self._lr_snapshot() != self._lrs:
                raise ValueError("TrainStep(graph=True): a learning rate changed after the step was recorded (the "
                                 "replayed AdamW launches carry the recorded values); build a new TrainStep")
            self._fill(en, F0, N, s, wav, noise, seed)
        self._graph.replay()
        return self._static_out

    def _lr_snapshot(self):
        return [g["lr"] for o in self.opt.values() for g in o.param_groups]

    def _fill(self, en, F0, N, s, wav, noise, seed):
        st = self.static_inputs
        with torch.no_grad():
            for k, t in (("en", en), ("F0", F0), ("N", N), ("s", s), ("wav", wav), ("noise", noise)):
                if t is None:
                    continue
                if st[k] is None:
                    raise ValueError("TrainStep(graph=True): the graph was recorded with the device RNG (noise=None)")
                if tuple(t.shape) != tuple(st[k].shape) or t.dtype != st[k].dtype:
                    # (copy_ would broadcast a size-1 dimension silently): a batch of another crop length needs
                    # its own recording
                    raise ValueError(f"TrainStep(graph=True): input {k} is {tuple(t.shape)} {t.dtype}, the graph "
                                     f"was recorded for {tuple(st[k].shape)} {st[k].dtype}")
                if t.data_ptr() != st[k].data_ptr():
                    st[k].copy_(t)
            if noise is None:
                if st["noise"] is not None:
                    raise ValueError("TrainStep(graph=True): the graph was recorded with explicit noise, pass noise=")
                st["seed"].fill_(seed_i64(seed))

    def _text_front(self, text):
        """train.py:217-251: the text encoder, asr, the predictor's forward and the crops."""
        from .prosody import matmul
        from .texttrain import duration_losses
        if self.text_encoder is None or self.predictor is None:
            raise ValueError("TrainStep(text=...) needs text_encoder= and predictor=")
        texts, lens = text["texts"], text["input_lengths"]
        attn, mono = text["attn"], text["attn_mono"]
        t_en = self.text_encoder(texts, lens)  # train.py:217
        asr = matmul(t_en, attn)  # :220-223
        d_gt = mono.sum(axis=-1).detach()  # :225
        mels = text["mels"]
        s_full = self.style_encoder(mels.unsqueeze(1)) if self.style_encoder is not None else text["s"]  # :228
        d, p = self.predictor(t_en, s_full, lens, mono)  # :230-233
        ml, starts = int(text["mel_len"]), [int(v) for v in text["starts"]]
        en = torch.stack([asr[b, :, st:st + ml] for b, st in enumerate(starts)])  # :235-251
        p_en = torch.stack([p[b, :, st:st + ml] for b, st in enumerate(starts)])
        gt = torch.stack([mels[b, :, 2 * st:2 * (st + ml)] for b, st in enumerate(starts)]).detach()
        loss_dur, loss_ce = duration_losses(d, d_gt, lens)  # :286-299
        return en, p_en, gt, loss_dur, loss_ce

    def _step(self, en, F0, N, s, wav, noise, seed, p_en, gt, F0_real, N_real, text=None):
        text_losses = None
        if text is not None:
            en, p_en, gt, loss_dur, loss_ce = self._text_front(text)
            text_losses = (loss_dur, loss_ce)
        if self.style_encoder is not None and gt is not None:
            s = self.style_encoder(gt.unsqueeze(1))  # train.py:258
        if self.predictor is not None and p_en is not None:
            F0, N = self.predictor.F0Ntrain(p_en, s)  # train.py:265
        y_rec = self.decoder(en, F0, N, s, noise=noise, seed=seed, dtype=self.dtype)
        self.zero_grad()
        d_loss = self.dl(wav.detach(), y_rec.detach()).mean()
        d_loss.backward()
        if self.capture:
            for tag, m in (("mpd", self.mpd), ("msd", self.msd)):
                self.captured[tag] = {k: p.grad.detach().clone() for k, p in m.named_parameters() if p.grad is not None}
        self.opt["msd"].step()
        self.opt["mpd"].step()
        self.zero_grad()
        frozen = []
        if self.freeze_d_in_g:
            for m in (self.mpd, self.msd):
                for p in m.parameters():
                    if p.requires_grad:
                        p.requires_grad_(False)
                        frozen.append(p)
        try:
            loss_mel = self.stft_loss(y_rec, wav)
            loss_gen_all = self.gl(wav, y_rec).mean()
            g_loss = self.lambda_mel * loss_mel + self.lambda_gen * loss_gen_all
            extra = {}
            if F0_real is not None:
                extra["loss_F0_rec"] = smooth_l1_loss(F0_real, F0) / 10  # train.py:269
                g_loss = g_loss + self.lambda_F0 * extra["loss_F0_rec"]
            if N_real is not None:
                extra["loss_norm_rec"] = smooth_l1_loss(N_real, N)  # train.py:270
                g_loss = g_loss + self.lambda_norm * extra["loss_norm_rec"]
            if text_losses is not None:  # train.py:300-307: lambda_ce loss_ce + lambda_dur loss_dur
                extra["loss_dur"], extra["loss_ce"] = text_losses
                g_loss = g_loss + self.lambda_ce * text_losses[1] + self.lambda_dur * text_losses[0]
            g_loss.backward()
        finally:
            for p in frozen:
                p.requires_grad_(True)
        if self.capture:
            self.captured["dec"] = {k: p.grad.detach().clone() for k, p in self.decoder.named_parameters()
                                    if p.grad is not None}
            for tag, m in (("predictor", self.predictor), ("style_encoder", self.style_encoder),
                           ("text_encoder", self.text_encoder)):
                if m is not None:
                    self.captured[tag] = {k: p.grad.detach().clone() for k, p in m.named_parameters()
                                          if p.grad is not None}
        for key in ("predictor", "style_encoder", "decoder", "text_encoder"):  # train.py:323-327
            if key in self.opt:
                self.opt[key].step()
        out = {"y_rec": y_rec.detach(), "d_loss": d_loss.detach(), "loss_mel": loss_mel.detach(),
               "loss_gen_all": loss_gen_all.detach(), "g_loss": g_loss.detach()}
        out.update({k: v.detach() for k, v in extra.items()})
        return out
