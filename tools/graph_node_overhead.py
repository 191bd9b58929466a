"""Per-node cost of a hipGraph replay against the same kernels launched on a stream (round 6).

    python tools/graph_node_overhead.py [--kernels 4000] [--numel 4096,1048576,16777216]

Launches N dependent elementwise kernels (torch add_ on one buffer, so each waits for the previous) eagerly and as one
captured torch.cuda.CUDAGraph, and prints the GPU time per kernel of each (hipEvents around the whole sequence, median
of 5) for a few buffer sizes: the difference is the graph's per-node overhead on this runtime.  --fork: every kernel
pair forks onto a side stream and joins back (event record / wait), the pattern of the training step's concurrent
branches, so the graph carries a cross-stream edge pair per two kernels.
"""
import argparse
import json
import statistics

import torch


def timed(fn, reps=5):
    out = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        torch.cuda.synchronize()
        out.append(a.elapsed_time(b))
    return statistics.median(out)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--kernels", type=int, default=4000)
    ap.add_argument("--numel", default="4096,1048576,16777216")
    ap.add_argument("--fork", action="store_true")
    a = ap.parse_args()
    side = torch.cuda.Stream(device=0)
    torch.cuda.set_device(0)
    for numel in (int(x) for x in a.numel.split(",")):
        x = torch.zeros(numel, device="cuda")
        y = torch.zeros(numel, device="cuda")

        def seq():
            if not a.fork:
                for _ in range(a.kernels):
                    x.add_(1.0)
                return
            cur = torch.cuda.current_stream()
            for _ in range(a.kernels // 2):
                side.wait_stream(cur)
                with torch.cuda.stream(side):
                    y.add_(1.0)
                x.add_(1.0)
                cur.wait_stream(side)

        seq()
        torch.cuda.synchronize()
        eager = timed(seq)
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        g = torch.cuda.CUDAGraph()
        with torch.cuda.stream(s):
            seq()  # warm on the capture stream
            torch.cuda.synchronize()
            with torch.cuda.graph(g, stream=s):
                seq()
        torch.cuda.synchronize()
        graph = timed(g.replay)
        print(json.dumps({"fork": a.fork, "numel": numel, "kernels": a.kernels, "eager_us_per_kernel": 1e3 * eager / a.kernels,
                          "graph_us_per_kernel": 1e3 * graph / a.kernels,
                          "graph_minus_eager_us": 1e3 * (graph - eager) / a.kernels}))


if __name__ == "__main__":
    main()
