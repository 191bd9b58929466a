"""Duration / text path on the HIP device, fp32.

Drop-ins for the reference modules in front of the decoder (thewh1teagle/StyleTTS2-lite @ 2025-06-14):

* `LSTM`            nn.LSTM(bidirectional, batch_first, 1 layer) with pack_padded_sequence semantics
                    (models.py:267-279, 420-430, 449, 510-518) -> stts_bilstm_fwd
* `TextEncoder`     models.py:229-295 (embedding, 3 x [wn-Conv1d k5, LayerNorm, LeakyReLU 0.2], BiLSTM)
* `DurationEncoder` models.py:468-533 (nlayers x [BiLSTM, AdaLayerNorm], style concat, masking)
* `matmul`          the alignment products en = d^T @ aln (models.py:432, inference.py:266) and
                    asr = t_en @ aln (inference.py:268)

Every op is a launch in libstts2.so (csrc/prosody.hip) on the current torch stream; parameters are
the modules' own state-dict tensors (same names and shapes as the reference).  There is no CPU or
PyTorch compute fallback: tensors must live on the HIP device.
"""
from __future__ import annotations

import ctypes

import torch
import torch.nn as nn
from torch.nn.utils.rnn import PackedSequence, pack_padded_sequence, pad_packed_sequence

from .engine import _ptr, _stream, check, lib

c_int, c_ll, c_vp, c_float = ctypes.c_int, ctypes.c_longlong, ctypes.c_void_p, ctypes.c_float
_BOUND = False


def _L():
    global _BOUND
    L = lib()
    if not _BOUND:
        L.stts_frames_gemm.argtypes = [c_vp, c_ll, c_ll, c_ll, c_int, c_int, c_int, c_vp, c_ll, c_ll, c_ll, c_ll,
                                       c_int, c_int, c_int, c_vp, c_vp, c_vp, c_ll, c_ll, c_ll, c_int, c_vp]
        L.stts_frames_gemm.restype = c_int
        L.stts_frames_gemm_ws.argtypes = [c_vp, c_ll, c_ll, c_ll, c_int, c_int, c_int, c_vp, c_ll, c_ll, c_ll, c_ll,
                                          c_int, c_int, c_int, c_vp, c_vp, c_vp, c_ll, c_ll, c_ll, c_int, c_vp, c_ll,
                                          c_vp]
        L.stts_frames_gemm_ws.restype = c_int
        L.stts_bilstm_workspace_bytes.argtypes = [c_int, c_int, c_int]
        L.stts_bilstm_workspace_bytes.restype = c_ll
        L.stts_bilstm_fwd.argtypes = [c_vp, c_ll, c_ll, c_ll, c_int, c_int, c_int, c_vp, ctypes.POINTER(c_vp), c_int,
                                      c_vp, c_vp, c_vp, c_vp, c_ll, c_vp]
        L.stts_bilstm_fwd.restype = c_int
        L.stts_set_lstm_group.argtypes = [c_int]
        L.stts_set_lstm_group.restype = c_int
        L.stts_bilstm_error_offset.argtypes = [c_int, c_int, c_int]
        L.stts_bilstm_error_offset.restype = c_ll
        L.stts_set_bilstm_debug.argtypes = [c_int, c_int]
        L.stts_set_bilstm_debug.restype = c_int
        L.stts_row_norm.argtypes = [c_vp, c_ll, c_ll, c_ll, c_int, c_int, c_int, c_int, c_vp, c_vp, c_ll, c_float,
                                    c_int, c_float, c_vp, c_vp, c_int, c_vp, c_ll, c_ll, c_vp]
        L.stts_row_norm.restype = c_int
        L.stts_embedding.argtypes = [c_vp, c_int, c_int, c_vp, c_int, c_int, c_vp, c_vp, c_vp, c_vp]
        L.stts_embedding.restype = c_int
        L.stts_weight_norm.argtypes = [c_vp, c_vp, c_int, c_int, c_vp, c_vp]
        L.stts_weight_norm.restype = c_int
        L.stts_durations.argtypes = [c_vp, c_ll, c_ll, c_int, c_int, c_int, c_vp, c_vp, c_float, c_float, c_float,
                                     c_vp, c_vp, c_vp, c_vp, c_vp]
        L.stts_durations.restype = c_int
        L.stts_expand_frames.argtypes = [c_vp, c_ll, c_ll, c_ll, c_int, c_int, c_int, c_vp, c_int, c_vp, c_vp, c_vp]
        L.stts_expand_frames.restype = c_int
        _BOUND = True
    return L


def set_lstm_group(bg: int) -> None:
    """BiLSTM recurrence kernel: 0 = automatic, -1 = cooperative (H = 256), 1 / 2 / 4 = utterances per
    workgroup of the per-workgroup kernel (A/B testing)."""
    check(_L().stts_set_lstm_group(int(bg)), "stts_set_lstm_group")


def set_bilstm_debug(spin_limit: int = 0, drop: bool = False) -> None:
    """Testing hook of the cooperative recurrence (stts_set_bilstm_debug): waits give up after
    `spin_limit` polls (0 = the default bound) and, with `drop`, one workgroup never publishes."""
    check(_L().stts_set_bilstm_debug(int(spin_limit), 1 if drop else 0), "stts_set_bilstm_debug")


# device error words of BiLSTM launches not yet read by the host (stts_bilstm_error_offset)
_PENDING: list = []


def check_pending() -> None:
    """Read the error words of every BiLSTM launch since the last check (one host sync) and raise
    if a cooperative recurrence timed out (its outputs are then NaN).  Synthesizer calls this at the
    host syncs the reference path already makes (the alignment width, the returned audio)."""
    global _PENDING
    if not _PENDING:
        return
    pend, _PENDING = _PENDING, []
    flags = torch.cat([f for _, f in pend]).cpu()
    bad = [name for (name, _), v in zip(pend, flags.tolist()) if v != 0]
    if bad:
        raise RuntimeError(f"stts_bilstm_fwd: the cooperative recurrence timed out waiting for a peer workgroup "
                           f"({', '.join(bad)}); its outputs are NaN")


def _on_device(t: torch.Tensor, what: str) -> torch.Tensor:
    if not t.is_cuda:
        raise RuntimeError(f"{what}: the HIP path needs device tensors (got {t.device}); no CPU fallback exists")
    if t.dtype != torch.float32:
        raise TypeError(f"{what}: float32 expected, got {t.dtype}")
    return t


def _lengths(lengths, B: int, T: int, device) -> torch.Tensor | None:
    if lengths is None:
        return None
    ln = torch.as_tensor(lengths).to(device=device, dtype=torch.int32).reshape(-1).contiguous()
    if ln.numel() != B:
        raise ValueError(f"lengths has {ln.numel()} entries for a batch of {B}")
    return ln


def frames_gemm(x, xs, B, Tin, Cin, w, wst, N, K, pad, bias, bias2, y, ys, Tout):
    """Raw stts_frames_gemm_ws (include/stts2.h): xs = (b, t, c) strides, wst = (b, n, c, k), ys = (b, t, n).
    Outputs with few 64 x 64 tiles (text-length rows) get a split-K scratch buffer."""
    tiles = ((Tout + 63) // 64) * ((N + 63) // 64) * B
    elems = 16 * B * Tout * N if tiles < 128 and Cin * K >= 256 else 0
    ws = torch.empty(elems, dtype=torch.float32, device=y.device) if elems else None
    check(_L().stts_frames_gemm_ws(_ptr(x), *xs, B, Tin, Cin, _ptr(w), *wst, N, K, pad, _ptr(bias), _ptr(bias2),
                                   _ptr(y), *ys, Tout, _ptr(ws), elems * 4, _stream()), "stts_frames_gemm_ws")


def matmul(a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    """Batched a @ b for 3-D float32 device tensors of any strides ([B,M,K] @ [B,K,N] -> [B,M,N]); under autograd
    (an operand requires grad) with both operand gradients (texttrain.matmul)."""
    if torch.is_grad_enabled() and (a.requires_grad or b.requires_grad):
        from . import texttrain
        return texttrain.matmul(a, b)
    _on_device(a, "matmul"), _on_device(b, "matmul")
    if a.dim() != 3 or b.dim() != 3 or a.shape[0] != b.shape[0] or a.shape[2] != b.shape[1]:
        raise ValueError(f"matmul shapes {tuple(a.shape)} @ {tuple(b.shape)}")
    B, M, K = a.shape
    N = b.shape[2]
    y = torch.empty(B, M, N, dtype=torch.float32, device=a.device)
    if K == 0:
        return y.zero_()
    frames_gemm(a, a.stride(), B, M, K, b, (b.stride(0), b.stride(2), b.stride(1), 0), N, 1, 0, None, None,
                y, y.stride(), M)
    return y


def linear_frames(x: torch.Tensor, weight: torch.Tensor, bias: torch.Tensor | None) -> torch.Tensor:
    """nn.Linear over the last axis of a 3-D [B,T,Cin] tensor (any strides) -> contiguous [B,T,N]."""
    B, T, Cin = x.shape
    N = weight.shape[0]
    y = torch.empty(B, T, N, dtype=torch.float32, device=x.device)
    frames_gemm(x, x.stride(), B, T, Cin, weight, (0, weight.stride(0), weight.stride(1), 0), N, 1, 0, bias, None,
                y, y.stride(), T)
    return y


def row_norm(x, C, mode, gamma=None, beta=None, gb_sb=0, eps=1e-5, slope=None, lengths=None, extra=None):
    """stts_row_norm over a [B,T,C]-indexed view x (any strides) -> contiguous [B,T,C+E]."""
    B, T = x.shape[0], x.shape[1]
    E = 0 if extra is None else extra.shape[1]
    y = torch.empty(B, T, C + E, dtype=torch.float32, device=x.device)
    check(_L().stts_row_norm(_ptr(x), x.stride(0), x.stride(1), x.stride(2), B, T, C, mode, _ptr(gamma), _ptr(beta),
                             gb_sb, eps, 0 if slope is None else 1, 0.0 if slope is None else slope, _ptr(lengths),
                             _ptr(extra), E, _ptr(y), y.stride(0), y.stride(1), _stream()), "stts_row_norm")
    return y


def weight_norm_fold(g: torch.Tensor, v: torch.Tensor) -> torch.Tensor:
    w = torch.empty_like(v)
    d0 = v.shape[0]
    check(_L().stts_weight_norm(_ptr(g), _ptr(v), d0, v.numel() // d0, _ptr(w), _stream()), "stts_weight_norm")
    return w


def durations(logits, lengths=None, z=None, mix=0.0, prev_mean=0.0, speed=1.0):
    """stts_durations (inference.py:247-258): logits [B, T, K] (last axis contiguous) ->
    (dur [B,T] float32, pred [B,T] int32, total [B] int32, dur_mean [B] float32)."""
    _on_device(logits, "durations")
    B, T, K = logits.shape
    if logits.stride(2) != 1:
        logits = logits.contiguous()
    dev = logits.device
    ln = _lengths(lengths, B, T, dev)
    if z is not None:
        z = _on_device(z.reshape(B, T).contiguous(), "durations z")
    dur = torch.empty(B, T, dtype=torch.float32, device=dev)
    pred = torch.empty(B, T, dtype=torch.int32, device=dev)
    total = torch.empty(B, dtype=torch.int32, device=dev)
    dmean = torch.empty(B, dtype=torch.float32, device=dev)
    check(_L().stts_durations(_ptr(logits), logits.stride(0), logits.stride(1), B, T, K, _ptr(ln), _ptr(z),
                              float(mix), float(prev_mean), float(speed), _ptr(dur), _ptr(pred), _ptr(total),
                              _ptr(dmean), _stream()), "stts_durations")
    return dur, pred, total, dmean


def expand_frames(src_btc: torch.Tensor, pred: torch.Tensor, Fmax: int) -> torch.Tensor:
    """stts_expand_frames: src viewed as (b, t, c) (any strides) -> [B, C, Fmax] = src^T @ aln, the
    one-hot alignment of `pred` frames per token (inference.py:259-268) applied as an exact gather."""
    _on_device(src_btc, "expand_frames")
    B, T, C = src_btc.shape
    pred = pred.to(torch.int32).contiguous()
    y = torch.empty(B, C, Fmax, dtype=torch.float32, device=src_btc.device)
    ftok = torch.empty(B, max(Fmax, 1), dtype=torch.int32, device=src_btc.device)
    check(_L().stts_expand_frames(_ptr(src_btc), *src_btc.stride(), B, T, C, _ptr(pred), Fmax, _ptr(ftok), _ptr(y),
                                  _stream()), "stts_expand_frames")
    return y


class LSTM(nn.LSTM):
    """nn.LSTM(input_size, hidden_size, 1, batch_first=True, bidirectional=True) with the HIP forward.

    Same constructor and state-dict keys as torch's (weight_ih_l0, ..., bias_hh_l0_reverse), so the
    reference's checkpoints load unchanged.  `forward(x, hx=None, lengths=None)`:
      * x [B, T, input_size] (any strides), optionally `lengths` [B]: pack_padded_sequence semantics
        (each direction runs over the first lengths[b] steps; later rows are zero), as the reference's
        pack -> LSTM -> pad_packed sequence (models.py:267-279) computes;
      * or x = a PackedSequence, as the reference passes one: the result is packed back the same way.
    Returns (output [B, T, 2H], (h_n [2, B, H], c_n [2, B, H])).
    """

    def forward(self, x, hx=None, lengths=None):
        from .texttrain import needs_grad
        if needs_grad(self, x.data if isinstance(x, PackedSequence) else x):
            # train.py's G step: the packed-sequence BiLSTM with its backward (texttrain.bilstm); (h_n, c_n) are not
            # formed on this path (every reference caller discards them: x, _ = lstm(x))
            from . import texttrain
            if hx is not None:
                raise NotImplementedError("HIP LSTM: only the zero initial state the reference uses (hx=None)")
            if isinstance(x, PackedSequence):
                padded, lens = pad_packed_sequence(x, batch_first=True)
                out, _ = self.forward(padded, lengths=lens)
                return pack_padded_sequence(out, lens, batch_first=True, enforce_sorted=False), None
            _on_device(x, "LSTM")
            return texttrain.bilstm(self, x, _lengths(lengths, x.shape[0], x.shape[1], x.device)), None
        from .engine import forward_only
        forward_only(self, "LSTM")
        if hx is not None:
            raise NotImplementedError("HIP LSTM: only the zero initial state the reference uses (hx=None)")
        if not (self.bidirectional and self.batch_first and self.num_layers == 1 and self.bias
                and self.proj_size == 0):
            raise NotImplementedError("HIP LSTM: bidirectional, batch_first, 1 layer, with bias (as the reference)")
        if isinstance(x, PackedSequence):
            padded, lens = pad_packed_sequence(x, batch_first=True)
            out, hc = self.forward(padded, lengths=lens)
            return pack_padded_sequence(out, lens, batch_first=True, enforce_sorted=False), hc
        _on_device(x, "LSTM")
        B, T, Cin = x.shape
        if Cin != self.input_size:
            raise ValueError(f"LSTM: input size {Cin}, expected {self.input_size}")
        H = self.hidden_size
        ln = _lengths(lengths, B, T, x.device)
        params = [self.weight_ih_l0, self.weight_hh_l0, self.bias_ih_l0, self.bias_hh_l0, self.weight_ih_l0_reverse,
                  self.weight_hh_l0_reverse, self.bias_ih_l0_reverse, self.bias_hh_l0_reverse]
        params = [_on_device(p.detach(), "LSTM parameter").contiguous() for p in params]
        arr = (c_vp * 8)(*[p.data_ptr() for p in params])
        L = _L()
        nb = int(L.stts_bilstm_workspace_bytes(B, T, H))
        ws = torch.empty(max(nb, 1), dtype=torch.uint8, device=x.device)
        y = torch.empty(B, T, 2 * H, dtype=torch.float32, device=x.device)
        hn = torch.empty(2, B, H, dtype=torch.float32, device=x.device)
        cn = torch.empty(2, B, H, dtype=torch.float32, device=x.device)
        check(L.stts_bilstm_fwd(_ptr(x), x.stride(0), x.stride(1), x.stride(2), B, T, Cin, _ptr(ln), arr, H, _ptr(y),
                                _ptr(hn), _ptr(cn), _ptr(ws), nb, _stream()), "stts_bilstm_fwd")
        off = int(L.stts_bilstm_error_offset(B, T, H))
        if B > 0 and off >= 0:
            if len(_PENDING) >= 64:  # bound the list for callers that never sync through check_pending
                check_pending()
            # a 4-byte device copy (async), so the workspace is not kept alive until the check
            _PENDING.append((f"LSTM({self.input_size}, {H}) B={B} T={T}", ws[off:off + 4].view(torch.int32).clone()))
        return y, (hn, cn)


class _LayerNorm(nn.Module):
    """reference models.py:229-240 parameter layout (gamma, beta)."""

    def __init__(self, channels, eps=1e-5):
        super().__init__()
        self.channels, self.eps = channels, eps
        self.gamma = nn.Parameter(torch.ones(channels))
        self.beta = nn.Parameter(torch.zeros(channels))


class _WNConv1d(nn.Module):
    """weight_norm(nn.Conv1d(c, c, k, padding=(k-1)//2)) parameter layout (models.py:245)."""

    def __init__(self, cin, cout, k, padding):
        super().__init__()
        self.cin, self.cout, self.k, self.padding = cin, cout, k, padding
        self.bias = nn.Parameter(torch.zeros(cout))
        self.weight_g = nn.Parameter(torch.ones(cout, 1, 1))
        self.weight_v = nn.Parameter(torch.zeros(cout, cin, k))


class TextEncoder(nn.Module):
    """reference models.py:241-295: same constructor and state-dict keys (embedding.weight,
    cnn.{i}.0.weight_g/_v/bias, cnn.{i}.1.gamma/beta, lstm.*).

    forward(x tokens [B,T] int64, input_lengths [B], m mask [B,T]) -> [B, channels, T] (a view of the
    time-major buffer the kernels produce; rows t >= input_lengths[b] are zero, as the reference's)."""

    def __init__(self, channels, kernel_size, depth, n_symbols, actv=nn.LeakyReLU(0.2)):
        super().__init__()
        self.channels, self.kernel_size, self.n_symbols = channels, kernel_size, n_symbols
        self.slope = float(getattr(actv, "negative_slope", 0.2))
        self.embedding = nn.Embedding(n_symbols, channels)
        pad = (kernel_size - 1) // 2
        self.cnn = nn.ModuleList()
        for _ in range(depth):
            self.cnn.append(nn.Sequential(_WNConv1d(channels, channels, kernel_size, pad), _LayerNorm(channels),
                                          nn.LeakyReLU(self.slope), nn.Dropout(0.2)))
        self.lstm = LSTM(channels, channels // 2, 1, batch_first=True, bidirectional=True)

    def _folded(self, conv):
        """weight_norm fold (stts_weight_norm), cached until the parameters change (load_state_dict,
        optimizer steps bump their versions)."""
        key = (conv.weight_g._version, conv.weight_v._version, conv.weight_g.data_ptr(), conv.weight_v.data_ptr())
        cache = getattr(conv, "_stts_folded", None)
        if cache is None or cache[0] != key:
            cache = (key, weight_norm_fold(conv.weight_g.detach(), conv.weight_v.detach().contiguous()))
            conv._stts_folded = cache
        return cache[1]

    def forward(self, x, input_lengths, m=None):
        from .texttrain import needs_grad
        if needs_grad(self):  # train.py:217 (the text encoder in train mode, optimizer.step('text_encoder'))
            from . import texttrain
            if m is not None and m.shape[-1] != x.shape[-1]:
                raise ValueError(f"mask length {m.shape[-1]} != token length {x.shape[-1]}")
            return texttrain.text_encoder(self, x, input_lengths)
        from .engine import forward_only
        forward_only(self, "TextEncoder")
        if x.dim() != 2:
            raise ValueError(f"tokens must be [B, T], got {tuple(x.shape)}")
        dev = self.embedding.weight.device
        if dev.type != "cuda":
            raise RuntimeError("TextEncoder: the HIP path needs the module on the HIP device; no CPU fallback")
        host_checked = not x.is_cuda
        if host_checked and x.numel() and (int(x.min()) < 0 or int(x.max()) >= self.n_symbols):
            raise IndexError("TextEncoder: token id outside [0, n_symbols)")  # as nn.Embedding
        tok = x.to(device=dev, dtype=torch.int64).contiguous()
        B, T = tok.shape
        if m is not None and m.shape[-1] != T:
            raise ValueError(f"mask length {m.shape[-1]} != token length {T}")
        C = self.channels
        ln = _lengths(input_lengths, B, T, dev)
        h = torch.empty(B, T, C, dtype=torch.float32, device=dev)
        err = None if host_checked else torch.zeros(1, dtype=torch.int32, device=dev)
        emb = _on_device(self.embedding.weight.detach(), "embedding").contiguous()
        check(_L().stts_embedding(_ptr(tok), B, T, _ptr(emb), self.n_symbols, C, _ptr(ln), _ptr(h), _ptr(err),
                                  _stream()), "stts_embedding")
        for blk in self.cnn:
            conv, ln_mod = blk[0], blk[1]
            w = self._folded(conv)
            y = torch.empty(B, T, C, dtype=torch.float32, device=dev)
            frames_gemm(h, h.stride(), B, T, C, w, (0, w.stride(0), w.stride(1), w.stride(2)), C, conv.k,
                        conv.padding, conv.bias.detach(), None, y, y.stride(), T)
            h = row_norm(y, C, 0, gamma=ln_mod.gamma.detach(), beta=ln_mod.beta.detach(), eps=ln_mod.eps,
                         slope=self.slope, lengths=ln)
        out, _ = self.lstm(h, lengths=ln)
        if err is not None and int(err.item()) != 0:  # device tokens: the kernel's flag (one sync)
            raise IndexError("TextEncoder: token id outside [0, n_symbols)")
        return out.transpose(1, 2)


class AdaLayerNorm(nn.Module):
    """reference models.py:372-392 parameter layout (fc)."""

    def __init__(self, style_dim, channels, eps=1e-5):
        super().__init__()
        self.channels, self.eps = channels, eps
        self.fc = nn.Linear(style_dim, channels * 2)

    def forward(self, x, s, lengths=None, extra=None):
        """x [B,T,C] (any strides), s [B,style_dim] -> [B,T,C(+E)]; rows t >= lengths are zero."""
        from .texttrain import needs_grad
        if needs_grad(self, x, s, extra):
            from . import texttrain
            from .training import linear
            gb = linear(s, self.fc.weight, self.fc.bias)
            ln = _lengths(lengths, x.shape[0], x.shape[1], x.device)
            return texttrain.ada_layer_norm(x, gb, self.eps, ln, extra=extra)
        from .engine import forward_only
        forward_only(self, "AdaLayerNorm")
        gb = linear_frames(s.unsqueeze(0), self.fc.weight.detach(), self.fc.bias.detach())[0]
        return row_norm(x, self.channels, 1, gamma=gb, gb_sb=gb.stride(0), eps=self.eps, lengths=lengths,
                        extra=extra)


class DurationEncoder(nn.Module):
    """reference models.py:468-533 (lstms = [LSTM, AdaLayerNorm] x nlayers).

    forward(x [B, d_model, T] (the TextEncoder output), style [B, sty_dim], text_lengths [B], m)
    -> [B, T, d_model + sty_dim], as the reference returns it."""

    def __init__(self, sty_dim, d_model, nlayers, dropout=0.1):
        super().__init__()
        self.lstms = nn.ModuleList()
        for _ in range(nlayers):
            self.lstms.append(LSTM(d_model + sty_dim, d_model // 2, num_layers=1, batch_first=True,
                                   bidirectional=True))
            self.lstms.append(AdaLayerNorm(sty_dim, d_model))
        self.dropout, self.d_model, self.sty_dim = dropout, d_model, sty_dim

    def forward(self, x, style, text_lengths, m=None):
        from .texttrain import needs_grad
        if needs_grad(self, x, style):
            from . import texttrain
            _on_device(x, "DurationEncoder"), _on_device(style, "DurationEncoder style")
            return texttrain.duration_encoder(self, x, style, _lengths(text_lengths, x.shape[0], x.shape[2], x.device))
        from .engine import forward_only
        forward_only(self, "DurationEncoder")
        _on_device(x, "DurationEncoder"), _on_device(style, "DurationEncoder style")
        B, C, T = x.shape
        if C != self.d_model or tuple(style.shape) != (B, self.sty_dim):
            raise ValueError(f"DurationEncoder inputs: x {tuple(x.shape)}, style {tuple(style.shape)}")
        ln = _lengths(text_lengths, B, T, x.device)
        style = style.contiguous()
        h = row_norm(x.transpose(1, 2), C, 2, lengths=ln, extra=style)  # cat([x, s]) + mask (models.py:499-501)
        for block in self.lstms:
            if isinstance(block, AdaLayerNorm):
                h = block(h, style, lengths=ln, extra=style)  # AdaLayerNorm, cat s, mask (models.py:503-507)
            else:
                h, _ = block(h, lengths=ln)  # pack -> LSTM -> pad (models.py:509-518); dropout: eval identity
        return h
