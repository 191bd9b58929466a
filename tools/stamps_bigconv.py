"""Phase attribution of the bigconv2 engine by in-kernel s_memtime stamps (STTS_OPT_DEBUG bit 64 +
stts_set_debug_buffer): one launch per shape through the stts_test_conv1d hook at the stage-0 / 1
sizes, per-wave cycle shares of weight waits, window wait, barrier, transform, epilogue, the rest
(MFMA taps + DMA issue).  Diagnostics only.

    python tools/stamps_bigconv.py [--batch 16]
"""
import argparse
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "styletts2-lite_amd")]
import torch  # noqa: E402

from stts2_mi355x import engine as E  # noqa: E402

NAMES = ["w_wait", "x_wait", "barrier", "transform", "epilogue", "total", "rest", "ep_vmwait", "ep_finish", "ep_stats"]


def run(C, K, dil, res, B, L, stamps, skip=0):
    g = torch.Generator().manual_seed(1)
    x = (torch.randn(B, L, C, generator=g) * 1.5).cuda()
    w = (torch.randn(C, C, K, generator=g) / (C * K) ** 0.5).cuda()
    b = (torch.randn(C, generator=g) * 0.1).cuda()
    gb = (torch.randn(B, 2 * C, generator=g) * 0.3).cuda()
    al = (torch.rand(C, generator=g) + 0.5).cuda()
    r = torch.randn(B, L, C, generator=g).cuda() if res else None
    y = torch.empty(B, L, C, device="cuda")
    st = torch.zeros(B, C, 2, dtype=torch.float64, device="cuda")
    P = lambda t: ctypes.c_void_p(t.data_ptr()) if t is not None else ctypes.c_void_p(0)  # noqa: E731
    pad = dil * (K - 1) // 2
    for dbg in (0, 64 | skip):
        E.set_option(E.OPT_DEBUG, dbg)
        stamps.zero_()
        E.check(E.lib().stts_test_conv1d(1, P(x), B, L, C, P(w), P(b), C, K, 0, 1, dil, pad, 0, 3, P(gb), P(al),
                                         ctypes.c_float(0.2), P(r), ctypes.c_float(1.0), P(y), L, P(st)))
        torch.cuda.synchronize()
    E.set_option(E.OPT_DEBUG, 0)
    v = stamps.cpu().tolist()
    tot = v[5] or 1
    waves = max(v[15], 1) * 8
    tag = f" skip={skip:2d}" if skip else ""
    print(f"C={C} K={K:2d} d={dil} res={int(res)}{tag}: cycles/wave {v[5] / waves:9.0f}  " +
          "  ".join(f"{n} {100 * v[i] / tot:4.1f}%" for i, n in enumerate(NAMES) if i != 5), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--skips", default="0", help="comma list of STTS_OPT_DEBUG phase-skip masks (1 transform, "
                    "2 MFMA, 4 epilogue, 8 weight DMA, 16 window DMA, 32 barrier)")
    ap.add_argument("--shapes", default="all", help="'all' or 'short' (one no-res + one res shape per C)")
    a = ap.parse_args()
    torch.cuda.set_device(0)
    stamps = torch.zeros(16, dtype=torch.int64, device="cuda")
    E.check(E.lib().stts_set_debug_buffer(ctypes.c_void_p(stamps.data_ptr())))
    shapes = ((3, 1, False), (3, 1, True), (7, 3, False), (7, 1, True), (11, 5, False), (11, 1, True))
    if a.shapes == "short":
        shapes = ((7, 3, False), (7, 1, True))
    for C, L in ((256, 8000), (128, 40000)):
        for K, dil, res in shapes:
            for skip in (int(x) for x in a.skips.split(",")):
                run(C, K, dil, res, a.batch, L, stamps, skip)
    E.check(E.lib().stts_set_debug_buffer(ctypes.c_void_p(0)))


if __name__ == "__main__":
    main()
