"""Gradient fixtures of the text / duration path as train.py's G step differentiates it (train.py:217, 220-223,
230-233, 286-299, 318, 323, 327): the REFERENCE TextEncoder (models.py:238-299) and ProsodyPredictor.forward
(:422-446, with the DurationEncoder :468-533), run through their own autograd.

Run in the survey container only (needs /root/reference; never on the GPU box):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_train_text.py

One ragged batch (helpers.DURATION_CASES[0]: T = 24 tokens, lengths 24 / 19 / 13) with formula weights, tokens,
styles and alignments (stts2_mi355x/synth.py, tests/helpers.duration_inputs), twice:
  * train_text_T24_B3.npz: the modules in eval mode (dropout off);
  * train_text_drop_T24_B3.npz: in TRAIN mode, as train.py runs them, with torch.nn.functional.dropout replaced for
    the run by the injected masks synth.dropout_mask(k, shape, p) of the k-th call (y = x mask / (1 - p), torch's
    scaling): the three nn.Dropout(0.2) of the TextEncoder's CNN blocks (models.py:250), the DurationEncoder's
    F.dropout after each LSTM (:512) and the predictor's F.dropout(x, 0.5) before duration_proj (:442), in call
    order.  The HIP path takes the same masks through training.set_dropout_masks (tests/test_gpu_train_text.py).
The chain is train.py's:
    t_en = text_encoder(texts, input_lengths, text_mask)                       (train.py:217)
    asr = t_en @ attn                                                          (:220-223)
    d, p = predictor(t_en, s, input_lengths, attn, text_mask)                  (:230-233)
    loss = sum(asr r_asr) + sum(d r_d) + sum(p r_p) + lambda_dur loss_dur + lambda_ce loss_ce
with loss_dur / loss_ce restated below from train.py:286-299 (d_gt = attn.sum(-1), :225), differentiated in fp64
(the truth) and in fp32 (the reference as it runs).  Stored per parameter tensor: L2 norm, max |g| and the values at
24 formula indices for both dtypes; the input gradient of the style vector, the losses and the outputs in full.
Data only.
"""
from __future__ import annotations

import os
import sys

import numpy as np
import torch
import torch.nn.functional as F

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from make_golden import fill, import_models  # noqa: E402
from make_golden_train_pred import summarize  # noqa: E402
from stts2_mi355x import synth  # noqa: E402

sys.path.insert(0, os.path.dirname(HERE))
from helpers import DURATION_CASES, duration_inputs  # noqa: E402

LAMBDA_DUR, LAMBDA_CE = 1.0, 1.0


def dur_losses(d, d_gt, input_lengths):
    """train.py:286-299, as written there (loss_dur, loss_ce)."""
    loss_ce = 0
    loss_dur = 0
    for _s2s_pred, _text_input, _text_length in zip(d, (d_gt), input_lengths):
        _s2s_pred = _s2s_pred[:_text_length, :]
        _text_input = _text_input[:_text_length].long()
        _s2s_trg = torch.zeros_like(_s2s_pred)
        for p in range(_s2s_trg.shape[0]):
            _s2s_trg[p, :_text_input[p]] = 1
        _dur_pred = torch.sigmoid(_s2s_pred).sum(axis=1)
        loss_dur += F.l1_loss(_dur_pred[1:_text_length - 1], _text_input[1:_text_length - 1])
        loss_ce += F.binary_cross_entropy_with_logits(_s2s_pred.flatten(), _s2s_trg.flatten())
    loss_ce /= d.size(0)
    loss_dur /= d.size(0)
    return loss_dur, loss_ce


class _InjectedDropout:
    """torch.nn.functional.dropout replaced by synth.dropout_mask of the k-th call (train mode only)."""

    def __init__(self):
        self.k = 0

    def __call__(self, x, p=0.5, training=True, inplace=False):
        if not training or p == 0:
            return x
        m = torch.from_numpy(synth.dropout_mask(self.k, tuple(x.shape), p)).to(x.dtype)
        self.k += 1
        return x * m / (1 - p)


def text_case(T, lengths, train=False):
    models = import_models()
    tok, ln, s, aln = duration_inputs(T, lengths)
    B, F_ = len(lengths), aln.shape[2]
    tok_t, ln_t = torch.from_numpy(tok), torch.from_numpy(ln)
    probes = {k: torch.from_numpy(synth.normal(f"tt:probe:{k}:{T}", shp)) for k, shp in
              (("asr", (B, 512, F_)), ("d", (B, T, 50)), ("p", (B, 640, F_)))}
    rec = {"T": np.int64(T), "lengths": ln, "lambda_dur": np.float64(LAMBDA_DUR), "lambda_ce": np.float64(LAMBDA_CE)}
    for tag, dt in (("f64", torch.float64), ("f32", torch.float32)):
        torch.manual_seed(0)
        torch.set_default_dtype(dt)  # (the reference's x_pad buffers are torch.zeros of the default dtype)
        te = fill(models.TextEncoder(channels=512, kernel_size=5, depth=3, n_symbols=178), "te.").train(train).to(dt)
        pp = fill(models.ProsodyPredictor(style_dim=128, d_hid=512, nlayers=3, max_dur=50, dropout=0.2),
                  "pp.").train(train).to(dt)
        saved = F.dropout
        F.dropout = _InjectedDropout()  # (eval mode: never called with training=True)
        m = pp.length_to_mask(ln_t)
        sd = torch.from_numpy(s).to(dt).clone().requires_grad_(True)
        attn = torch.from_numpy(aln).to(dt)
        t_en = te(tok_t, ln_t, m)
        asr = t_en @ attn
        d, p = pp(t_en, sd, ln_t, attn, m)
        ncalls = F.dropout.k
        F.dropout = saved
        if train:
            assert ncalls == 7, ncalls  # 3 CNN blocks + 3 DurationEncoder LSTMs + the duration projection
        d_gt = attn.sum(axis=-1).detach()
        loss_dur, loss_ce = dur_losses(d, d_gt, ln_t)
        loss = ((asr * probes["asr"].to(dt)).sum() + (d * probes["d"].to(dt)).sum() + (p * probes["p"].to(dt)).sum()
                + LAMBDA_DUR * loss_dur + LAMBDA_CE * loss_ce)
        loss.backward()
        params = {**{"te." + k: v for k, v in te.named_parameters()},
                  **{"pp." + k: v for k, v in pp.named_parameters() if v.grad is not None}}
        names = sorted(params)
        rec["names"] = np.array(names)
        summarize(rec, tag, params, names)
        rec[f"{tag}.t_en"], rec[f"{tag}.d"], rec[f"{tag}.p"] = (x.detach().numpy() for x in (t_en, d, p))
        rec[f"{tag}.loss_dur"], rec[f"{tag}.loss_ce"] = float(loss_dur), float(loss_ce)
        rec[f"{tag}.grad_s"] = sd.grad.numpy()
    torch.set_default_dtype(torch.float32)
    return rec


def main():
    torch.set_num_threads(8)
    T, lengths = DURATION_CASES[0]
    for train, tag in ((False, "train_text"), (True, "train_text_drop")):
        rec = text_case(T, lengths, train)
        name = f"{tag}_T{T}_B{len(lengths)}.npz"
        np.savez_compressed(os.path.join(HERE, name), **rec)
        print(name, len(rec["names"]), "parameter tensors;", "loss_dur", rec["f64.loss_dur"], "loss_ce",
              rec["f64.loss_ce"])


if __name__ == "__main__":
    main()
