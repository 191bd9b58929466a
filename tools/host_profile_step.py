"""Host-side cost of the config-5 training step: cProfile over the timed steps only (after warmup), to tell
Python / C-ABI issue time from time the host spends blocked on the device.  Prints the top functions by own
time and by cumulative time.  Run on a GPU box: python tools/host_profile_step.py [--dtype bf16] [--steps 3]"""
import argparse
import cProfile
import io
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "styletts2-lite_amd"))

import torch  # noqa: E402

from bench_train_step import build  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dtype", default="bf16")
    ap.add_argument("--steps", type=int, default=3)
    a = ap.parse_args()
    from stts2_mi355x.trainstep import TrainStep
    dec, mpd, msd, (asr, f0, n, s, wav) = build(2, 155)
    dec, mpd, msd = dec.cuda().eval(), mpd.cuda().train(), msd.cuda().train()
    ins = [t.cuda().requires_grad_(True) for t in (asr, f0, n, s)]
    wav = wav.cuda()
    step = TrainStep(dec, mpd, msd, dtype=a.dtype)
    for i in range(2):
        step(*ins, wav, seed=100 + i)
    torch.cuda.synchronize()
    pr = cProfile.Profile()
    t0 = time.perf_counter()
    pr.enable()
    for i in range(a.steps):
        step(*ins, wav, seed=1000 + i)
    pr.disable()
    host = (time.perf_counter() - t0) / a.steps * 1e3
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / a.steps * 1e3
    print(f"host issue {host:.1f} ms / step (under cProfile), wall {wall:.1f} ms / step")
    for key in ("tottime", "cumtime"):
        buf = io.StringIO()
        pstats.Stats(pr, stream=buf).sort_stats(key).print_stats(40)
        print(buf.getvalue())


if __name__ == "__main__":
    main()
