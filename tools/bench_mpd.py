"""MultiPeriodDiscriminator forward on the HIP engine at the training step's shape (BASELINE
configs[4] / SURVEY §8(d) config 5: B = 2 segments of 93,000 samples, real + generated = one batch
of 4).  Median of hipEvent times, algorithmic FLOPs from the conv shapes (SURVEY: MPD forward real +
fake 416.3 GFLOP), the fraction of the dtype's MFMA peak, and the oracle on the host for scale.

    python tools/bench_mpd.py [--segments 2] [--samples 93000] [--iters 10]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "styletts2-lite_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

PEAK = {"bf16": 2.5e15, "fp32": 157.3e12}


def flops(B, T, periods=(2, 3, 5, 7, 11)):
    from stts2_mi355x.engine import MPD_CH, mpd_lengths
    f = 0.0
    for p in periods:
        L = mpd_lengths(T, p)
        for j in range(5):
            f += 2.0 * B * p * L[j + 1] * MPD_CH[j + 1] * MPD_CH[j] * 5
        f += 2.0 * B * p * L[5] * 1024 * 3
    return f


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--segments", type=int, default=2)
    ap.add_argument("--samples", type=int, default=93000)
    ap.add_argument("--iters", type=int, default=10)
    a = ap.parse_args()
    from stts2_mi355x import synth
    from stts2_mi355x.discriminators import MultiPeriodDiscriminator
    torch.cuda.set_device(0)
    m = MultiPeriodDiscriminator()
    sd = {k: torch.from_numpy(synth.synth_param("mpd." + k, tuple(v.shape))) for k, v in m.state_dict().items()}
    m.load_state_dict(sd)
    m = m.cuda()
    gen = torch.Generator().manual_seed(0)
    y = (torch.randn(a.segments, 1, a.samples, generator=gen) * 0.3).cuda()
    yh = (torch.randn(a.segments, 1, a.samples, generator=gen) * 0.3).cuda()
    fl = flops(2 * a.segments, a.samples)
    line = {"workload": f"MultiPeriodDiscriminator forward, {a.segments} segments x {a.samples} samples, real + generated",
            "alg_gflop": fl / 1e9}
    with torch.no_grad():
        for dtype in ("fp32", "bf16"):
            for _ in range(2):
                m(y, yh, dtype=dtype)
            torch.cuda.synchronize()
            ts = []
            for _ in range(a.iters):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                m(y, yh, dtype=dtype)
                e1.record()
                torch.cuda.synchronize()
                ts.append(e0.elapsed_time(e1))
            ms = float(np.median(ts))
            line[dtype] = {"ms": ms, "tflops": fl / ms / 1e9, "mfma_fraction": fl / (ms / 1e3) / PEAK[dtype]}
    # the oracle on the host, one period-set on one real+generated pair (bounded sample)
    from oracle import stts_oracle as orc
    torch.set_num_threads(int(os.environ.get("OMP_NUM_THREADS", "0")) or os.cpu_count() or 1)
    t0 = time.perf_counter()
    with torch.no_grad():
        orc.mpd(y[:1].cpu(), yh[:1].cpu(), sd)
    el = time.perf_counter() - t0
    line["cpu_baseline"] = {"ms_per_segment_pair": el * 1e3, "cores": torch.get_num_threads(), "kind": "port",
                            "sample": "oracle/stts_oracle.py mpd on 1 real + 1 generated segment, fp32 torch-CPU"}
    print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
