"""B = 1 decoder latency: eager forward (~120 launches from Python through the C-ABI) vs the
hipGraph replay of the same forward (stts2_mi355x.graph.CapturedDecoder).  Median of hipEvent
times over --iters calls after warm-up.  One JSON line.

    python tools/bench_graph.py [--batch 1] [--frames 400] [--dtype bf16] [--decoder hifigan]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "styletts2-lite_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402


def timed(fn, iters):
    ts = []
    for _ in range(iters):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    return float(np.median(ts))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1)
    ap.add_argument("--frames", type=int, default=400)
    ap.add_argument("--dtype", default="bf16")
    ap.add_argument("--decoder", default="hifigan")
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    from stts2_mi355x import synth
    from stts2_mi355x.graph import CapturedDecoder
    torch.cuda.set_device(0)
    dec, _ = bench.build_decoder(a.decoder)
    dec = dec.cuda()
    eng = dec.engine(a.dtype)
    asr, f0, n, s = (torch.from_numpy(x).cuda() for x in synth.decoder_inputs(a.batch, a.frames))
    noise = torch.randn(a.batch, 600 * a.frames, 9, device="cuda")
    with torch.no_grad():
        for _ in range(3):
            eng.forward(asr, f0, n, s, noise=noise)
        torch.cuda.synchronize()
        eager = timed(lambda: eng.forward(asr, f0, n, s, noise=noise), a.iters)
        run = CapturedDecoder(dec, a.batch, a.frames, dtype=a.dtype)
        for _ in range(3):
            run(asr, f0, n, s)
        torch.cuda.synchronize()
        graph = timed(lambda: run(asr, f0, n, s), a.iters)
        err = (run(asr, f0, n, s, noise=noise) - eng.forward(asr, f0, n, s, noise=noise)).abs().max().item()
    samples = a.batch * 600 * a.frames
    print(json.dumps({"workload": f"{a.decoder} {a.dtype} decoder, B={a.batch} x {a.frames * 600 // 24000}-s",
                      "eager_ms": eager, "graph_ms": graph, "graph_speedup": eager / graph,
                      "graph_samples_per_s": samples / graph * 1e3, "x_realtime_graph": samples / 24000 / graph * 1e3,
                      "graph_vs_eager_max_abs": err,
                      "note": "graph call = input copies + noise normal_() + replay; eager = noise given"}), flush=True)


if __name__ == "__main__":
    main()
