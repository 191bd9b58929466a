"""Concurrent resblock branches of the decoder plan (STTS_OPT_BRANCHES, default: batches of at most 4): a generator
stage's resblocks 1 .. n-1 run beside resblock 0 on side HIP streams with their own temporaries and are averaged
after (st_branch_avg), instead of through the running-sum epilogue.  fp32: bit-identical to the running sum (the
same additions in the same order); bf16: the branch outputs are stored (rounded) before the average, so within
bf16 rounding of the running sum; both against the reference golden at B = 1; and inside a captured hipGraph."""
import numpy as np
import pytest
import torch

from helpers import decoder_case, golden, make_decoder

pytestmark = pytest.mark.gpu

_DEC = {}


def _dec(kind):
    if kind not in _DEC:
        d, _ = make_decoder(kind)
        _DEC[kind] = d.cuda()
    return _DEC[kind]


def _run(kind, B, T, dtype, branches, nbranch=None):
    from stts2_mi355x import engine as E
    asr, f0, n, s, nz = decoder_case(B, T)
    try:
        E.set_option(E.OPT_BRANCHES, branches)
        if nbranch is not None:
            E.set_option(E.OPT_NBRANCH, nbranch)
        with torch.no_grad():
            out = _dec(kind)(asr.cuda(), f0.cuda(), n.cuda(), s.cuda(), noise=nz.cuda(), dtype=dtype)
        torch.cuda.synchronize()
    finally:
        E.reset_options()
    return out.cpu().numpy()


@pytest.mark.parametrize("kind", ["hifigan", "istftnet"])
@pytest.mark.parametrize("B,T", [(1, 400), (2, 40), (4, 16)])
def test_branches_fp32_bit_identical(kind, B, T):
    a = _run(kind, B, T, "fp32", 0)
    b = _run(kind, B, T, "fp32", 4)
    print(f"{kind} B={B} T={T} fp32 branches vs running sum: max-abs {np.abs(a - b).max():.3e}")
    assert np.array_equal(a, b)


@pytest.mark.parametrize("B,T", [(1, 400), (4, 40)])
def test_branches_bf16_close(B, T):
    a = _run("hifigan", B, T, "bf16", 0)
    b = _run("hifigan", B, T, "bf16", 4)
    err = float(np.abs(a - b).max())
    print(f"hifigan B={B} T={T} bf16 branches vs running sum: max-abs {err:.3e}")
    assert err < 5e-2  # (bf16 vs fp32 is 1.9e-2 at 10 s; a wrong average would be O(0.1))


def test_branches_golden_b1():
    out = _run("hifigan", 1, 400, "fp32", 4)
    ref = golden("hifigan_T400_B1")["out"]
    err = float(np.abs(out - ref).max())
    print(f"hifigan B=1 T=400 fp32 with branches vs reference golden: {err:.3e}")
    assert err < 1e-3


def test_branches_in_captured_graph():
    from stts2_mi355x.graph import CapturedDecoder
    dec = _dec("hifigan")
    asr, f0, n, s, nz = decoder_case(1, 40)
    run = CapturedDecoder(dec, B=1, T=40, dtype="fp32")
    out = run(asr.cuda(), f0.cuda(), n.cuda(), s.cuda(), noise=nz.cuda()).cpu().numpy()
    ref = _run("hifigan", 1, 40, "fp32", 0)
    assert np.array_equal(out, ref)


@pytest.mark.parametrize("B,T", [(12, 40), (32, 16)])
def test_noise_branches_alone_fp32_bit_identical(B, T):
    """Above the resblock-branch threshold only the noise branches run on a side stream (STTS_OPT_NBRANCH)."""
    a = _run("hifigan", B, T, "fp32", 0, 0)
    b = _run("hifigan", B, T, "fp32", 0, 64)
    assert np.array_equal(a, b)


@pytest.mark.parametrize("B,T", [(1, 16), (2, 24)])
def test_branches_bf16_general_engines_own_splitk(B, T):
    """With the resblock engines off (STTS_OPT_RESCONV 0) the small-batch resblock convs take the general engines,
    incl. the split-K short-conv path (st_pw_split) whose fp32 partials live in per-stream scratch: each side-stream
    resblock has its own, so the concurrent branches equal the one-stream run within bf16 rounding of the average."""
    from stts2_mi355x import engine as E

    def run(branches):
        asr, f0, n, s, nz = decoder_case(B, T)
        try:
            E.set_option(E.OPT_RESCONV, 0)
            E.set_option(E.OPT_BRANCHES, branches)
            E.set_option(E.OPT_NBRANCH, branches)
            with torch.no_grad():
                out = _dec("hifigan")(asr.cuda(), f0.cuda(), n.cuda(), s.cuda(), noise=nz.cuda(), dtype="bf16")
            torch.cuda.synchronize()
        finally:
            E.reset_options()
        return out.cpu().numpy()

    a, b = run(0), run(8)
    err = float(np.abs(a - b).max())
    print(f"hifigan B={B} T={T} bf16 RESCONV=0 branches vs one stream: max-abs {err:.3e}")
    assert np.isfinite(b).all() and err < 2e-2
