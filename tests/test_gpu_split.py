"""GPU parity of the split-operand accuracy mode (dtype 'bf16x3' = STTS_SPLIT): fp32 activations, every conv's
operands split into bf16 hi + lo parts (hi = bf16(v), lo = bf16(v - hi)) and multiplied as hi*hi + hi*lo + lo*hi
on the bf16 MFMA with fp32 accumulation (conv1d.hip; the lo*lo term, ~2^-18 of a product, is dropped).

Bars: per conv, max |y - y_fp64| / max |y_fp64| <= 2e-5 (the operands carry ~16 significant bits: ~2^-17
relative each; the bf16 throughput mode sits at ~4e-3); the decoders against the REFERENCE golden waveforms
(tests/golden, made from the reference modules) at the north star's 1e-3 max-abs, at 10 s and at config 3's
B = 32 x 10 s against the fp32 path."""
import numpy as np
import pytest
import torch

from helpers import decoder_case, golden, make_decoder

pytestmark = pytest.mark.gpu

SPLIT = 2  # STTS_SPLIT


def _conv_split(x, w, b, stride, pad, dil, dtype=SPLIT):
    """stts_conv1d_fwd on frames x [B, Lin, Cin] -> [B, Lq, Cout] (fp32 tensors on the device)."""
    from stts2_mi355x.engine import _ptr, _stream, check, lib
    B, Lin, Cin = x.shape
    Cout, _, K = w.shape
    Lq = (Lin + 2 * pad - dil * (K - 1) - 1) // stride + 1
    nb = lib().stts_conv1d_fwd_workspace_bytes(dtype, B, Lin, Cin, Cout, K, stride, dil, pad, Lq)
    check(int(nb) if nb < 0 else 0, "stts_conv1d_fwd_workspace_bytes")
    ws = torch.empty(max(int(nb), 1), dtype=torch.uint8, device="cuda")
    y = torch.empty(B, Lq, Cout, device="cuda")
    check(lib().stts_conv1d_fwd(dtype, _ptr(x), _ptr(w), _ptr(b), B, Lin, Cin, Cout, K, stride, dil, pad, Lq, _ptr(y),
                                _ptr(ws), int(nb), _stream()), "stts_conv1d_fwd")
    torch.cuda.synchronize()
    return y


@pytest.mark.parametrize("B,Lin,Cin,Cout,K,stride,dil", [
    (2, 300, 512, 512, 3, 1, 1),      # front-end / C = 512 resblock
    (2, 257, 1090, 1024, 3, 1, 1),    # the 1,090-channel concat (Cin not a multiple of 32)
    (1, 1000, 256, 256, 11, 1, 5),    # C = 256 k11 dilation 5
    (2, 3000, 64, 64, 11, 1, 3),      # C = 64 k11 dilation 3
    (1, 4097, 32, 32, 7, 1, 1),       # C = 32 (ragged length)
    (2, 513, 96, 32, 9, 2, 1),        # stride 2, N = 32 (the MSD layers)
])
def test_split_conv_vs_fp64(B, Lin, Cin, Cout, K, stride, dil):
    torch.manual_seed(1)
    x = torch.randn(B, Lin, Cin, dtype=torch.float64)
    w = torch.randn(Cout, Cin, K, dtype=torch.float64) / (Cin * K) ** 0.5
    b = torch.randn(Cout, dtype=torch.float64)
    pad = dil * (K - 1) // 2
    ref = torch.nn.functional.conv1d(x.transpose(1, 2), w, b, stride=stride, padding=pad, dilation=dil).transpose(1, 2)
    xs, ws_, bs = (t.float().cuda().contiguous() for t in (x, w, b))
    scale = float(ref.abs().max())
    errs = {}
    for name, dt in (("bf16x3", SPLIT), ("fp32", 0), ("bf16", 1)):
        y = _conv_split(xs, ws_, bs, stride, pad, dil, dt).double().cpu()
        assert y.shape == ref.shape
        errs[name] = float((y - ref).abs().max()) / scale
    print(f"conv B{B} L{Lin} {Cin}->{Cout} k{K} s{stride} d{dil}: rel max-abs bf16x3 {errs['bf16x3']:.2e}, "
          f"fp32 {errs['fp32']:.2e}, bf16 {errs['bf16']:.2e}")
    assert errs["bf16x3"] <= 2e-5
    assert errs["bf16x3"] < errs["bf16"] / 20


_DEC = {}


def _dec(kind):
    if kind not in _DEC:
        d, _ = make_decoder(kind)
        _DEC[kind] = d.cuda()
    return _DEC[kind]


def _run(kind, B, T, dtype, sl=slice(None)):
    asr, f0, n, s, nz = (t[sl] for t in decoder_case(B, T))
    with torch.no_grad():
        out = _dec(kind)(asr.cuda(), f0.cuda(), n.cuda(), s.cuda(), noise=nz.cuda(), dtype=dtype)
    torch.cuda.synchronize()
    return out.cpu().numpy()


@pytest.mark.parametrize("kind", ["hifigan", "istftnet"])
@pytest.mark.parametrize("T,B", [(16, 2), (400, 1)])
def test_decoder_split_matches_reference(kind, T, B):
    """The accuracy mode against the reference golden (config 2 = iSTFTNet B 1 x 10 s): north-star 1e-3."""
    out = _run(kind, B, T, "bf16x3")
    ref = golden(f"{kind}_T{T}_B{B}")["out"]
    err = np.abs(out - ref).max()
    print(f"{kind} T={T} B={B} bf16x3 vs reference golden: max-abs {err:.3e}")
    assert err < 1e-3


def test_config3_split_batch32():
    """Config 3's batch (B = 32 x 10 s) in the accuracy mode: utterance 0 vs the reference golden, every
    utterance vs the fp32 path's decode of the same batch, both within the north star's 1e-3."""
    out = _run("hifigan", 32, 400, "bf16x3")
    g = golden("hifigan_T400_B1")["out"][0]
    e0 = float(np.abs(out[0] - g).max())
    ref = _run("hifigan", 32, 400, "fp32")
    err = np.abs(out - ref).reshape(32, -1).max(1)
    print(f"config 3 bf16x3: utterance 0 vs reference golden {e0:.3e}; vs fp32 max over utterances "
          f"{err.max():.3e} (median {np.median(err):.3e})")
    assert e0 < 1e-3 and err.max() < 1e-3



@pytest.mark.parametrize("B,T", [(2, 40), (1, 400)])
def test_ressplit_engine_ab(B, T):
    """The split resblock engine (ressplit.hip: C = 32 in one pass, C = 64 in two input-channel passes through
    an fp32 partial buffer) against the split igemm engine on the same decode (STTS_OPT_RESSPLIT 0 / 1): the
    same split arithmetic in a different summation order."""
    from stts2_mi355x import engine as E
    try:
        E.set_option(E.OPT_BIG64, 0)  # (C = 64 on the split resblock engine, not the bigconv2 engine)
        E.set_option(E.OPT_RESSPLIT, 0)
        ref = _run("hifigan", B, T, "bf16x3")
        E.set_option(E.OPT_RESSPLIT, 1)
        out = _run("hifigan", B, T, "bf16x3")
    finally:
        E.reset_options()
    err = np.abs(out - ref).max()
    print(f"ressplit A/B B={B} T={T}: max-abs {err:.3e}")
    assert err < 2e-5


@pytest.mark.parametrize("B,T,mode", [(2, 40, 5), (1, 400, 5), (3, 64, 5), (2, 40, 1), (3, 64, 1)])
def test_big64_split_engine_ab(B, T, mode):
    """The accuracy mode's C = 64 resblock convs on the bigconv2 engine with 128-frame wave slices
    (STTS_OPT_BIG64 bit 1, bigconv2.hip NF = 4) against the two-pass split resblock engine (STTS_OPT_BIG64 0): the
    same split arithmetic in a different summation order; B = 1 at 10 s also against the reference golden."""
    from stts2_mi355x import engine as E
    try:
        E.set_option(E.OPT_BIG64, 0)
        ref = _run("hifigan", B, T, "bf16x3")
        E.set_option(E.OPT_BIG64, mode)  # (5: 4-wave blocks, the default; 1: 8-wave blocks)
        out = _run("hifigan", B, T, "bf16x3")
    finally:
        E.reset_options()
    err = np.abs(out - ref).max()
    g = golden(f"hifigan_T{T}_B1")["out"][0] if T in (16, 40, 400) and B == 1 else None
    print(f"big64 split A/B B={B} T={T} mode {mode}: max-abs {err:.3e}"
          + (f", vs reference golden {np.abs(out[0] - g).max():.3e}" if g is not None else ""))
    assert np.isfinite(out).all() and err < 2e-5
    if g is not None:
        assert np.abs(out[0] - g).max() < 1e-3


@pytest.mark.parametrize("B,T,mode,front", [(2, 40, 1, 2), (1, 400, 1, 1), (3, 64, 4, 2), (2, 48, 3, 2)])
def test_bigsplit_engine_ab(B, T, mode, front):
    """The split variant of the bigconv2 engine (bigconv2.hip SP: 16-channel groups of bf16 hi + lo windows and
    weights, 3 MFMAs a product; the C = 128 / 256 resblock convs, the front-end k3 convs, ups[0] / ups[1]) against
    the split igemm engine on the same decode (STTS_OPT_BIGSPLIT 0): the same split arithmetic in a different
    summation order.  Modes: production routing, 8-wave blocks everywhere (4), 4-wave blocks everywhere (3);
    STTS_OPT_FRONT 2 forces the front-end engine at these small sizes."""
    from stts2_mi355x import engine as E
    try:
        E.set_option(E.OPT_FRONT, front)
        E.set_option(E.OPT_BIGSPLIT, 0)
        ref = _run("hifigan", B, T, "bf16x3")
        E.set_option(E.OPT_BIGSPLIT, mode)
        out = _run("hifigan", B, T, "bf16x3")
    finally:
        E.reset_options()
    err = np.abs(out - ref).max()
    g = golden(f"hifigan_T{T}_B1")["out"][0] if T in (16, 40, 400) and B == 1 else None
    print(f"bigsplit A/B B={B} T={T} mode {mode}: max-abs {err:.3e}"
          + (f", vs reference golden {np.abs(out[0] - g).max():.3e}" if g is not None else ""))
    assert np.isfinite(out).all() and err < 2e-5
    if g is not None:
        assert np.abs(out[0] - g).max() < 1e-3


@pytest.mark.parametrize("B,T,exp", [(2, 40, 32), (1, 400, 32), (3, 64, 64), (1, 400, 64)])
def test_split_ups_wave_layouts(B, T, exp):
    """The accuracy mode's ups[2] / ups[3] tiles that hold every output phase (the defaults: ups[2] on 12-wave blocks,
    ups[3] with 2 output blocks x 2 frame slices) against one phase per tile part (STTS_OPT_EXP bit 32: ups[2]; bit 64:
    ups[3]): outputs are the same MFMA chains, only the InstanceNorm statistics' fp32 order differs."""
    from stts2_mi355x import engine as E
    try:
        E.set_option(E.OPT_EXP, exp)
        ref = _run("hifigan", B, T, "bf16x3")
        E.set_option(E.OPT_EXP, 0)
        out = _run("hifigan", B, T, "bf16x3")
    finally:
        E.reset_options()
    err = np.abs(out - ref).max()
    g = golden(f"hifigan_T{T}_B1")["out"][0] if T in (16, 40, 400) and B == 1 else None
    print(f"split ups layouts B={B} T={T} exp {exp}: max-abs {err:.3e}"
          + (f", vs reference golden {np.abs(out[0] - g).max():.3e}" if g is not None else ""))
    assert np.isfinite(out).all() and err < 2e-5
    if g is not None:
        assert np.abs(out[0] - g).max() < 1e-3
