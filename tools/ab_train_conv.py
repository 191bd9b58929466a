"""A/B of the training step's bf16 conv engines at config 5 shapes (B = 2 x 93,000 samples): the conv forward,
dx and dw of stts_conv1d_fwd / stts_conv1d_bwd, hipEvent-timed, with an engine option off and on in one
process (STTS_OPT_WGRAD: the all-taps window weight-gradient kernel; STTS_OPT_PLAINRC: the C = 32 / 64 convs
on resconv).  Prints one JSON line per (shape, option value).

    python tools/ab_train_conv.py [--opt 15] [--values 0 1]
"""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "styletts2-lite_amd")]
from stts2_mi355x import engine as E  # noqa: E402
from stts2_mi355x.training import out_length  # noqa: E402

# config 5: B = 2, stage lengths 155 x 2 x (10, 50, 150, 300) frames
SHAPES = [  # (name, B, Cin, Cout, K, stride, dil, pad, Lin)
    ("front_1090_1024_k3", 2, 1090, 1024, 3, 1, 1, 1, 155),
    ("s0_256_k3_d1", 2, 256, 256, 3, 1, 1, 1, 3100),
    ("s0_256_k11_d5", 2, 256, 256, 11, 1, 5, 25, 3100),
    ("s1_128_k7_d3", 2, 128, 128, 7, 1, 3, 9, 15500),
    ("s2_64_k11_d5", 2, 64, 64, 11, 1, 5, 25, 46500),
    ("s3_32_k3_d1", 2, 32, 32, 3, 1, 1, 1, 93000),
    ("s3_32_k11_d5", 2, 32, 32, 11, 1, 5, 25, 93000),
    ("mpd_32_128_k5_s3", 10, 32, 128, 5, 3, 1, 2, 9300),
    ("msd1_3_32_k9", 7444, 3, 32, 9, 1, 1, 4, 257),
    ("msd2_96_32_k9_s2", 7444, 96, 32, 9, 2, 1, 4, 257),
]


def timed(fn, n=10):
    for _ in range(3):
        fn()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(n):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / n


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--opt", type=int, default=E.OPT_WGRAD)
    ap.add_argument("--values", type=int, nargs="+", default=[0, 1])
    a = ap.parse_args()
    L = E.lib()
    dt = 1
    for name, B, Cin, Cout, K, s, d, p, Lin in SHAPES:
        Lq = out_length(Lin, K, s, p, d)
        x = torch.randn(B, Lin, Cin, device="cuda")
        w = torch.randn(Cout, Cin, K, device="cuda") * 0.05
        bias = torch.randn(Cout, device="cuda")
        dy = torch.randn(B, Lq, Cout, device="cuda")
        y = torch.empty(B, Lq, Cout, device="cuda")
        dx = torch.empty_like(x)
        dw = torch.empty_like(w)
        nb = max(L.stts_conv1d_bwd_workspace_bytes(dt, B, Lin, Cin, Cout, K, s, d, p, Lq),
                 L.stts_conv1d_fwd_workspace_bytes(dt, B, Lin, Cin, Cout, K, s, d, p, Lq))
        ws = torch.empty(nb, dtype=torch.uint8, device="cuda")
        flops = 2.0 * B * Lq * Cout * Cin * K
        for v in a.values:
            E.set_option(a.opt, v)
            res = {"shape": name, "opt": a.opt, "value": v}
            calls = {
                "fwd": lambda: E.check(L.stts_conv1d_fwd(dt, E._ptr(x), E._ptr(w), E._ptr(bias), B, Lin, Cin, Cout, K,
                                                         s, d, p, Lq, E._ptr(y), E._ptr(ws), nb, E._stream()), "fwd"),
                "dx": lambda: E.check(L.stts_conv1d_bwd(dt, E._ptr(x), E._ptr(w), E._ptr(dy), B, Lin, Cin, Cout, K, s,
                                                        d, p, Lq, E._ptr(dx), None, None, E._ptr(ws), nb,
                                                        E._stream()), "dx"),
                "dw": lambda: E.check(L.stts_conv1d_bwd(dt, E._ptr(x), E._ptr(w), E._ptr(dy), B, Lin, Cin, Cout, K, s,
                                                        d, p, Lq, None, E._ptr(dw), None, E._ptr(ws), nb,
                                                        E._stream()), "dw"),
            }
            for tag, fn in calls.items():
                ms = timed(fn)
                res[tag + "_ms"] = round(ms, 4)
                res[tag + "_tflops"] = round(flops / ms / 1e9, 1)
            print(json.dumps(res), flush=True)
        E.reset_options()


if __name__ == "__main__":
    main()
