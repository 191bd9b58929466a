"""Phase attribution of the resconv engine (C = 32 / 64 resblock convs) by in-kernel s_memtime stamps
(STTS_OPT_DEBUG bit 64 + stts_set_debug_buffer): one launch per shape through the stts_test_conv1d hook at
the stage-2 / stage-3 frame counts, per-wave shares of the step's phases.  Diagnostics only.

    python tools/stamps_resconv.py [--batch 8] [--skips 0,2]
"""
import argparse
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "styletts2-lite_amd")]
import torch  # noqa: E402

from stts2_mi355x import engine as E  # noqa: E402

NAMES = ["coef+res_issue", "barrier_A", "transform", "win_issue", "barrier_B", "mfma", "epilogue"]


def run(C, K, dil, res, B, L, stamps, skip):
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
    ms = {}
    for dbg in (skip, 64 | skip):
        E.set_option(E.OPT_DEBUG, dbg)
        stamps.zero_()
        a, z = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        E.check(E.lib().stts_test_conv1d(1, P(x), B, L, C, P(w), P(b), C, K, 0, 1, dil, pad, 0, 3, P(gb), P(al),
                                         ctypes.c_float(0.2), P(r), ctypes.c_float(1.0), P(y), L, P(st)))
        z.record()
        torch.cuda.synchronize()
        ms[dbg] = a.elapsed_time(z)
    E.set_option(E.OPT_DEBUG, 0)
    v = stamps.cpu().tolist()
    tot = v[7] or 1
    waves = max(v[15], 1) * (8 if C == 64 else 4)
    tiles = B * ((L + 255) // 256)
    print(f"C={C} K={K:2d} d={dil} res={int(res)} skip={skip}: {ms[skip] * 1e3:6.1f} us (stamped {ms[64 | skip] * 1e3:6.1f}); "
          f"cycles/wave/tile {v[7] / waves / (tiles / max(v[15], 1)):7.0f}  " +
          "  ".join(f"{n} {100 * v[i] / tot:4.1f}%" for i, n in enumerate(NAMES)), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--skips", default="0,2")
    ap.add_argument("--exp", type=int, default=0, help="STTS_OPT_EXP held during the run (8: 3-deep prefetch at C=64)")
    a = ap.parse_args()
    torch.cuda.set_device(0)
    E.set_option(E.OPT_EXP, a.exp)
    stamps = torch.zeros(16, dtype=torch.int64, device="cuda")
    E.check(E.lib().stts_set_debug_buffer(ctypes.c_void_p(stamps.data_ptr())))
    for C, L in ((64, 120000), (32, 240000)):
        for K, dil, res in ((3, 3, False), (3, 1, True), (7, 3, False), (11, 3, False), (11, 1, True)):
            for skip in (int(s) for s in a.skips.split(",")):
                run(C, K, dil, res, a.batch, L, stamps, skip)
    E.check(E.lib().stts_set_debug_buffer(ctypes.c_void_p(0)))


if __name__ == "__main__":
    main()
