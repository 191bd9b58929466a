"""Vocos decoder (Modules/vocos.py) on the HIP path at the headline workload's
shape: B = 32 utterances of 10 s (400 asr frames -> 800 STFT frames x hop 300 = 240,000 samples),
the config_example.yaml vocos block (intermediate 1536, 8 ConvNeXt layers, n_fft 1200, hop 300).
Median of hipEvent times per dtype, samples/s, x real time, algorithmic GFLOP (front-end + ConvNeXt
+ head GEMMs), and the oracle on the host for one utterance (bounded CPU sample).

    python tools/bench_vocos.py [--batch 32] [--frames 400] [--iters 10]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "styletts2-lite_amd"), os.path.join(ROOT, "tests")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

PEAK = {"bf16": 2.5e15, "fp32": 157.3e12}


def gflop(T, inter=1536, layers=8, n_fft=1200, d=512):
    """Front-end (encode 4.20 + 3 x 6.09 + decode.3 4.83 GFLOP at T = 400, linear in T)
    + per ConvNeXt layer dwconv 2*7*d + pwconv1/2 2*2*d*inter per frame + head 2*d*(n_fft+2)."""
    front = (4.20 + 3 * 6.09 + 4.83) * T / 400
    F = 2 * T
    return front + F * (layers * (2 * 7 * d + 4 * d * inter) + 2 * d * (n_fft + 2)) / 1e9


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--frames", type=int, default=400)
    ap.add_argument("--iters", type=int, default=10)
    a = ap.parse_args()
    from stts2_mi355x import synth
    from test_vocos_cpu import make_vocos
    torch.cuda.set_device(0)
    dec = make_vocos()
    sd = {k: v.clone() for k, v in dec.state_dict().items()}
    dec = dec.cuda()
    B, T = a.batch, a.frames
    x = [torch.from_numpy(v).cuda() for v in synth.decoder_inputs(B, T, tag="bench-vocos")]
    samples = B * 2 * T * 300
    fl = gflop(T) * B
    line = {"workload": f"vocos decoder, batch {B} x {T} asr frames ({2 * T * 300} samples each), n_fft 1200 hop 300",
            "alg_gflop": fl}
    with torch.no_grad():
        for dtype in ("fp32", "bf16"):
            for _ in range(3):
                dec(*x, dtype=dtype)
            torch.cuda.synchronize()
            ts = []
            for _ in range(a.iters):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                dec(*x, dtype=dtype)
                e1.record()
                torch.cuda.synchronize()
                ts.append(e0.elapsed_time(e1))
            ms = float(np.median(ts))
            line[dtype] = {"ms": ms, "samples_per_s": samples / ms * 1e3, "x_realtime": samples / 24000 / ms * 1e3,
                           "tflops": fl / ms, "mfma_fraction": fl * 1e9 / (ms / 1e3) / PEAK[dtype]}
    from oracle import stts_oracle as orc
    torch.set_num_threads(int(os.environ.get("OMP_NUM_THREADS", "0")) or os.cpu_count() or 1)
    xc = [v[:1].cpu() for v in x]
    t0 = time.perf_counter()
    with torch.no_grad():
        orc.decoder_vocos(*xc, sd, dict(num_layers=8, n_fft=1200, hop=300))
    el = time.perf_counter() - t0
    line["cpu_baseline"] = {"samples_per_s": 2 * T * 300 / el, "cores": torch.get_num_threads(), "kind": "port",
                            "sample": "oracle/stts_oracle.py decoder_vocos on 1 utterance, fp32 torch-CPU"}
    print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
