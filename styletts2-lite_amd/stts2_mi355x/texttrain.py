"""The text / duration path with autograd, as train.py's G step differentiates it (train.py:217, 230-233, 286-299,
318, 323, 327): TextEncoder (models.py:238-299), DurationEncoder (:468-533), ProsodyPredictor.forward (:422-446) and
the duration losses loss_dur / loss_ce (train.py:286-299).  Every op is a `torch.autograd.Function` whose forward and
backward run as HIP kernels behind the C-ABI (include/stts2.h, stts2_train.h):

  * nn.Embedding + masked_fill_          stts_embedding / stts_embedding_bwd
  * weight-norm Conv1d k5                 training.weight_norm + training.conv1d_frames (the conv engine)
  * LayerNorm + LeakyReLU + mask,         stts_row_norm / stts_row_norm_bwd (modes 0 / 1 / 2)
    AdaLayerNorm + style concat + mask,
    the input concat
  * packed-sequence BiLSTM                stts_bilstm_fwd_train / stts_bilstm_bwd with the text lengths
  * dropout (train mode)                  training.dropout (stts_dropout)
  * duration_proj (LinearNorm)            training.linear (stts_linear_fwd / _bwd) over the B T rows
  * en = d^T @ alignment, t_en @ attn     stts_frames_gemm (matmul and both operand gradients)
  * loss_dur + loss_ce                    stts_dur_losses (forward and gradient in one launch)

The drop-in modules (prosody.TextEncoder / DurationEncoder / AdaLayerNorm / LSTM, models.ProsodyPredictor) take these
paths when grad mode is on and a parameter or an input requires grad; under torch.no_grad() (inference.py) they keep
the fused inference kernels.  Tensors live on the HIP device; there is no CPU fallback.
"""
from __future__ import annotations

import ctypes

import torch

from .engine import _ptr, _require_device, _stream, check
from .prosody import _L as _pl, _lengths, frames_gemm
from .training import _c, _tl, _ws, conv1d_frames, dropout, linear, weight_norm

_BOUND = False


def _lib():
    global _BOUND
    L = _tl()
    _pl()
    if not _BOUND:
        vp, i, ll, f = ctypes.c_void_p, ctypes.c_int, ctypes.c_longlong, ctypes.c_float
        sig = {
            "stts_row_norm_bwd_workspace_bytes": ([i, i, i], ll),
            "stts_row_norm_bwd": ([vp, ll, ll, ll, i, i, i, i, vp, vp, ll, f, i, f, vp, vp, ll, ll, i, vp, vp, vp, vp, vp,
                                   vp, ll, vp], i),
            "stts_embedding_bwd": ([vp, i, i, vp, vp, ll, ll, i, i, vp, vp], i),
            "stts_dur_losses_workspace_bytes": ([i], ll),
            "stts_dur_losses": ([vp, ll, ll, i, i, i, vp, vp, ll, vp, vp, vp, vp, vp, ll, vp], i),
        }
        for name, (args, res) in sig.items():
            fn = getattr(L, name)
            fn.argtypes, fn.restype = args, res
        _BOUND = True
    return L


def needs_grad(module, *inputs) -> bool:
    """The autograd path is taken when grad mode is on and a parameter or a tensor input requires grad."""
    if not torch.is_grad_enabled():
        return False
    return any(p.requires_grad for p in module.parameters()) or any(
        isinstance(t, torch.Tensor) and t.requires_grad for t in inputs)


# ------------------------------------------------------------------ nn.Embedding + masked_fill_ (models.py:257-260)
class _EmbeddingFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, weight, tok, ln):
        _require_device()
        B, T = tok.shape
        n_sym, C = weight.shape
        wc = _c(weight)
        h = torch.empty(B, T, C, dtype=torch.float32, device=weight.device)
        err = torch.zeros(1, dtype=torch.int32, device=weight.device)
        check(_pl().stts_embedding(_ptr(tok), B, T, _ptr(wc), n_sym, C, _ptr(ln), _ptr(h), _ptr(err), _stream()),
              "stts_embedding")
        ctx.save_for_backward(tok, ln if ln is not None else torch.empty(0))
        ctx.has_ln, ctx.shape = ln is not None, (n_sym, C)
        ctx.err = err
        return h

    @staticmethod
    def backward(ctx, dh):
        tok, ln = ctx.saved_tensors
        ln = ln if ctx.has_ln else None
        n_sym, C = ctx.shape
        B, T = tok.shape
        dhc = _c(dh)
        dW = torch.empty(n_sym, C, dtype=torch.float32, device=dh.device)
        check(_lib().stts_embedding_bwd(_ptr(tok), B, T, _ptr(ln), _ptr(dhc), dhc.stride(0), dhc.stride(1), n_sym, C,
                                        _ptr(dW), _stream()), "stts_embedding_bwd")
        return dW, None, None


# ------------------------------------------------------------------ row norms (stts_row_norm modes 0 / 1 / 2)
class _RowNormFn(torch.autograd.Function):
    """y [B, T, C + E] = norm(x [B, T, C]) (+ LeakyReLU) | extra [B, E], rows t >= len zero.
    mode 0: LayerNorm(gamma, beta); mode 1: AdaLayerNorm with gb [B, 2C]; mode 2: copy (the input concat)."""

    @staticmethod
    def forward(ctx, x, gamma, beta, gb, extra, mode, eps, slope, ln):
        _require_device()
        B, T, C = x.shape
        E = 0 if extra is None else extra.shape[1]
        xc = _c(x)
        g = _c(gamma if mode == 0 else gb) if mode != 2 else None
        bt = _c(beta) if mode == 0 else None
        ex = _c(extra) if extra is not None else None
        y = torch.empty(B, T, C + E, dtype=torch.float32, device=x.device)
        gb_sb = g.stride(0) if mode == 1 else 0
        check(_pl().stts_row_norm(_ptr(xc), xc.stride(0), xc.stride(1), xc.stride(2), B, T, C, mode, _ptr(g), _ptr(bt),
                                  gb_sb, eps, 0 if slope is None else 1, 0.0 if slope is None else slope, _ptr(ln),
                                  _ptr(ex), E, _ptr(y), y.stride(0), y.stride(1), _stream()), "stts_row_norm")
        ctx.save_for_backward(xc, *(t if t is not None else torch.empty(0) for t in (g, bt, ln)))
        ctx.cfg = (mode, eps, slope, E, ln is not None, gb_sb)
        return y

    @staticmethod
    def backward(ctx, dy):
        xc, g, bt, ln = ctx.saved_tensors
        mode, eps, slope, E, has_ln, gb_sb = ctx.cfg
        ln = ln if has_ln else None
        B, T, C = xc.shape
        dyc = _c(dy)
        need = ctx.needs_input_grad  # x, gamma, beta, gb, extra
        dx = torch.empty(B, T, C, dtype=torch.float32, device=dy.device) if need[0] else None
        dgamma = torch.empty(C, dtype=torch.float32, device=dy.device) if (mode == 0 and need[1]) else None
        dbeta = torch.empty(C, dtype=torch.float32, device=dy.device) if (mode == 0 and need[2]) else None
        dgb = torch.empty(B, 2 * C, dtype=torch.float32, device=dy.device) if (mode == 1 and need[3]) else None
        dex = torch.empty(B, E, dtype=torch.float32, device=dy.device) if (E and need[4]) else None
        L = _lib()
        nb = int(L.stts_row_norm_bwd_workspace_bytes(B, T, C))
        ws = _ws(nb, dy.device)
        check(L.stts_row_norm_bwd(_ptr(xc), xc.stride(0), xc.stride(1), xc.stride(2), B, T, C, mode,
                                  _ptr(g if mode != 2 else None), _ptr(bt if mode == 0 else None), gb_sb, eps,
                                  0 if slope is None else 1, 0.0 if slope is None else slope, _ptr(ln), _ptr(dyc),
                                  dyc.stride(0), dyc.stride(1), E, _ptr(dx), _ptr(dgamma), _ptr(dbeta), _ptr(dgb),
                                  _ptr(dex), _ptr(ws), nb, _stream()), "stts_row_norm_bwd")
        return dx, dgamma, dbeta, dgb, dex, None, None, None, None


def layer_norm_act(x, gamma, beta, eps, slope, ln):
    return _RowNormFn.apply(x, gamma, beta, None, None, 0, float(eps), slope, ln)


def ada_layer_norm(x, gb, eps, ln, extra=None):
    return _RowNormFn.apply(x, None, None, gb, extra, 1, float(eps), None, ln)


def concat_mask(x, extra, ln):
    return _RowNormFn.apply(x, None, None, None, extra, 2, 1e-5, None, ln)


# ------------------------------------------------------------------ packed-sequence BiLSTM
def bilstm(lstm, x, ln):
    """lstm: the reference's nn.LSTM(bidirectional, batch_first) layout; x frames [B, T, Cin]; ln device int32 [B]
    or None -> y [B, T, 2H] (pack -> LSTM -> pad_packed -> zero pad, models.py:267-285)."""
    from .training import _BiLSTMFn
    ps = [lstm.weight_ih_l0, lstm.weight_hh_l0, lstm.bias_ih_l0, lstm.bias_hh_l0, lstm.weight_ih_l0_reverse,
          lstm.weight_hh_l0_reverse, lstm.bias_ih_l0_reverse, lstm.bias_hh_l0_reverse]
    return _BiLSTMFn.apply(x, ln, *ps)


# ------------------------------------------------------------------ batched matmul with both operand gradients
def _mm(a, b):
    from .prosody import matmul
    with torch.no_grad():
        return matmul(a, b)


class _MatmulFn(torch.autograd.Function):
    """a [B, M, K] @ b [B, K, N] (any strides) on stts_frames_gemm; da = dy b^T, db = a^T dy."""

    @staticmethod
    def forward(ctx, a, b):
        ctx.save_for_backward(a, b)
        return _mm(a, b)

    @staticmethod
    def backward(ctx, dy):
        a, b = ctx.saved_tensors
        da = _mm(dy, b.transpose(1, 2)) if ctx.needs_input_grad[0] else None
        db = _mm(a.transpose(1, 2), dy) if ctx.needs_input_grad[1] else None
        return da, db


def matmul(a, b):
    return _MatmulFn.apply(a, b)


# ------------------------------------------------------------------ loss_dur / loss_ce (train.py:286-299)
class _DurLossFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, d, d_gt, ln):
        _require_device()
        B, T, K = d.shape
        dc = _c(d)
        gt = _c(d_gt.to(torch.float32))
        loss = torch.empty(2, dtype=torch.float64, device=d.device)
        L = _lib()
        nb = int(L.stts_dur_losses_workspace_bytes(B))
        ws = _ws(nb, d.device)
        check(L.stts_dur_losses(_ptr(dc), dc.stride(0), dc.stride(1), B, T, K, _ptr(ln), _ptr(gt), gt.stride(0),
                                _ptr(loss), None, None, None, _ptr(ws), nb, _stream()), "stts_dur_losses")
        ctx.save_for_backward(dc, gt, ln if ln is not None else torch.empty(0))
        ctx.has_ln = ln is not None
        out = loss.float()
        return out[0], out[1]

    @staticmethod
    def backward(ctx, g_dur, g_ce):
        dc, gt, ln = ctx.saved_tensors
        ln = ln if ctx.has_ln else None
        B, T, K = dc.shape
        # the upstream scalars stay on the device (the kernel reads them): no host sync
        gd = _c(g_dur.reshape(1)) if g_dur is not None else None
        gc = _c(g_ce.reshape(1)) if g_ce is not None else None
        dz = torch.empty(B, T, K, dtype=torch.float32, device=dc.device)
        loss = torch.empty(2, dtype=torch.float64, device=dc.device)
        L = _lib()
        nb = int(L.stts_dur_losses_workspace_bytes(B))
        ws = _ws(nb, dc.device)
        check(L.stts_dur_losses(_ptr(dc), dc.stride(0), dc.stride(1), B, T, K, _ptr(ln), _ptr(gt), gt.stride(0),
                                _ptr(loss), _ptr(dz), _ptr(gd), _ptr(gc), _ptr(ws), nb, _stream()), "stts_dur_losses")
        return dz, None, None


def duration_losses(d, d_gt, input_lengths):
    """train.py:286-299: (loss_dur, loss_ce) of the predictor's logits d [B, T, max_dur] against d_gt [B, T]
    (= s2s_attn_mono.sum(-1)), over the first input_lengths[b] tokens of each utterance."""
    ln = _lengths(input_lengths, d.shape[0], d.shape[1], d.device)
    return _DurLossFn.apply(d, d_gt.to(d.device), ln)


# ------------------------------------------------------------------ the modules
def text_encoder(te, tokens, input_lengths):
    """TextEncoder.forward (models.py:256-285) with autograd -> [B, channels, T]."""
    dev = te.embedding.weight.device
    if not tokens.is_cuda and tokens.numel() and (int(tokens.min()) < 0 or int(tokens.max()) >= te.n_symbols):
        raise IndexError("TextEncoder: token id outside [0, n_symbols)")  # as nn.Embedding
    tok = tokens.to(device=dev, dtype=torch.int64).contiguous()
    B, T = tok.shape
    ln = _lengths(input_lengths, B, T, dev)
    h = _EmbeddingFn.apply(te.embedding.weight, tok, ln)
    for blk in te.cnn:
        conv, lnm, drop = blk[0], blk[1], blk[3]
        w = weight_norm(conv.weight_g, conv.weight_v)
        y = conv1d_frames(h, w, conv.bias, 1, conv.padding)
        h = layer_norm_act(y, lnm.gamma, lnm.beta, lnm.eps, te.slope, ln)  # LayerNorm -> LeakyReLU -> mask
        if te.training:
            h = dropout(h, float(drop.p), ref_transpose=True)  # (the reference's [B, C, T] layout)
    out = bilstm(te.lstm, h, ln)
    return out.transpose(1, 2)


def duration_encoder(de, x, style, ln):
    """DurationEncoder.forward (models.py:497-523) with autograd: x [B, d_model, T] -> [B, T, d_model + sty_dim]."""
    from .prosody import AdaLayerNorm
    style = style.contiguous() if style.is_contiguous() else style.contiguous()
    h = concat_mask(x.transpose(1, 2), style, ln)  # cat([x, s]) + mask (models.py:499-501)
    for block in de.lstms:
        if isinstance(block, AdaLayerNorm):
            gb = linear(style, block.fc.weight, block.fc.bias)
            h = ada_layer_norm(h, gb, block.eps, ln, extra=style)  # AdaLayerNorm, cat s, mask (:503-507)
        else:
            h = bilstm(block, h, ln)  # pack -> LSTM -> pad (:509-518)
            if de.training and de.dropout > 0:
                h = dropout(h, float(de.dropout))
    return h


def predictor_forward(pp, texts, style, text_lengths, alignment):
    """ProsodyPredictor.forward (models.py:417-446) with autograd: -> (duration logits [B, T, max_dur],
    en [B, d_hid + style_dim, F])."""
    dev = pp.F0_proj.weight.device
    texts, style, alignment = (t.to(dev, torch.float32) for t in (texts, style, alignment))
    B, _, T = texts.shape
    ln = _lengths(text_lengths, B, T, dev)
    d = duration_encoder(pp.text_encoder, texts, style, ln)
    x = bilstm(pp.lstm, d, ln)
    if pp.training:
        x = dropout(x, 0.5)  # nn.functional.dropout(x, 0.5, training=self.training) (models.py:442)
    lin = pp.duration_proj.linear_layer
    duration = linear(x.reshape(B * T, x.shape[-1]), lin.weight, lin.bias).reshape(B, T, -1)
    en = matmul(d.transpose(-1, -2), alignment)
    return duration.squeeze(-1), en
