"""Phase table of the Vocos pointwise GEMM launches on conv1d_igemm (STTS_OPT_DEBUG bits: 1 window
staging math, 2 MFMAs, 4 epilogue, 8 window loads; results are wrong while set), B x 10 s bf16.

    python tools/vocos_phases.py [--batch 32]
"""
import argparse
import collections
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "styletts2-lite_amd"), os.path.join(ROOT, "tests")]
import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--dtype", default="bf16")
    a = ap.parse_args()
    from stts2_mi355x import engine as E
    from stts2_mi355x import synth
    from test_vocos_cpu import make_vocos
    torch.cuda.set_device(0)
    dec = make_vocos().cuda()
    x = [torch.from_numpy(v).cuda() for v in synth.decoder_inputs(a.batch, 400, tag="bench-vocos")]
    rows = collections.defaultdict(dict)
    with torch.no_grad():
        for dbg in (0, 1, 2, 4, 8, 15):
            E.set_option(E.OPT_DEBUG, dbg)
            for _ in range(2):
                dec(*x, dtype=a.dtype)
            torch.cuda.synchronize()
            E.profile_enable(True)
            dec(*x, dtype=a.dtype)
            torch.cuda.synchronize()
            acc = collections.defaultdict(list)
            for r in E.profile_launches():
                acc[(r["kernel"], r["N"], r["Cin"], r["taps"], r["rows"])].append(r["ms"] * 1e3)
            E.profile_enable(False)
            for k, v in acc.items():
                rows[k][dbg] = (float(np.median(v)), len(v))
    E.reset_options()
    print("kernel, N, Cin, taps, rows: median us per launch (launches) by debug bits 0 / 1 / 2 / 4 / 8 / 15")
    for k in sorted(rows):
        print(k, " | ".join(f"{d}: {rows[k][d][0]:7.1f}" for d in sorted(rows[k])), f"(x{rows[k][0][1]})")


if __name__ == "__main__":
    main()
