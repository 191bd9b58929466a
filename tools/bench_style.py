#!/usr/bin/env python3
"""Measurement of the style front-end row: Preprocess.wave_preprocess
(HIP log-mel, mel.hip k_logmel) + StyleEncoder on a batch of 3-s reference chunks, the unit
StyleTTS2.get_styles feeds the encoder (inference.py:195-217).  Prints ONE JSON line.

    python tools/bench_style.py [--batch 32] [--seconds 3] [--steps 20] [--warmup 3]
                                [--dtype fp32|bf16] [--no-cpu-baseline]

Timing: torch.cuda.Event pairs on the current stream (the library launches on it), inputs resident
in HBM.  `mel_roofline` describes k_logmel with its algorithmic work per frame: a 2048-point
radix-2 FFT (11 x 1024 butterflies x 10 flop = 112,640 flop) + 1025 powers (3 flop) + the
80 filters' nonzero taps (2 flop each), and 4 B per input sample read + 320 B per frame written.
The CPU baseline is the oracle (torch.stft + matmul + the StyleEncoder restatement) on the
host's threads over the same chunks.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "styletts2-lite_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

PEAK_FP32 = 157.3e12  # vector fp32 FLOP/s, MI355X
PEAK_HBM = 8.0e12


def timed(fn, steps, warmup):
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0.record()
    for _ in range(steps):
        fn()
    t1.record()
    torch.cuda.synchronize()
    return t0.elapsed_time(t1) / steps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--seconds", type=float, default=3.0)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--dtype", default="fp32", choices=["fp32", "bf16"])
    ap.add_argument("--no-cpu-baseline", action="store_true")
    args = ap.parse_args()

    from helpers import fill_module, speech_like
    from stts2_mi355x.engine import wave_preprocess_batch
    from stts2_mi355x.models import StyleEncoder

    B, L = args.batch, int(24000 * args.seconds)
    F = 1 + L // 300
    dev = torch.device("cuda", 0)
    se_cpu = fill_module(StyleEncoder(dim_in=64, style_dim=128, max_conv_dim=512)).eval()
    sd = {k: v.detach().clone() for k, v in se_cpu.state_dict().items()}
    se = se_cpu.to(dev)
    waves = np.stack([speech_like(f"bench:style:{b}", L) for b in range(B)])
    w = torch.from_numpy(waves).to(dev)

    with torch.no_grad():
        mel_ms = timed(lambda: wave_preprocess_batch(w), args.steps, args.warmup)
        mel = wave_preprocess_batch(w)
        enc_ms = timed(lambda: se(mel.unsqueeze(1), dtype=args.dtype), args.steps, args.warmup)
        both_ms = timed(lambda: se(wave_preprocess_batch(w).unsqueeze(1), dtype=args.dtype), args.steps,
                        args.warmup)

    from oracle import stts_oracle as orc
    fb = orc.melscale_fbanks().numpy()
    taps = int((fb > 0).sum())
    flops_frame = 11 * 1024 * 10 + 3 * 1025 + 2 * taps
    bytes_launch = B * L * 4 + B * F * 80 * 4
    flops_launch = B * F * flops_frame
    line = {
        "metric": "style front-end: 3-s reference chunks/s (log-mel + StyleEncoder)",
        "value": B / (both_ms / 1e3), "unit": "chunks/s", "n_gpus": 1, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": both_ms, "higher_is_better": True, "dtype": args.dtype,
        "data": "synthetic speech-like clips (tests/helpers.speech_like), formula StyleEncoder weights",
        "config": {"workload": f"{B} x {args.seconds:g}-s chunks at 24 kHz ({L} samples, {F} mel frames)",
                   "batch": B},
        "mel_ms": mel_ms, "style_encoder_ms": enc_ms,
        "mel_roofline": {"bound": "latency (LDS / barriers)", "flops_per_frame": flops_frame,
                         "achieved_tflops": flops_launch / (mel_ms / 1e3) / 1e12,
                         "frac_fp32_peak": flops_launch / (mel_ms / 1e3) / PEAK_FP32,
                         "achieved_GBps": bytes_launch / (mel_ms / 1e3) / 1e9,
                         "frac_hbm": bytes_launch / (mel_ms / 1e3) / PEAK_HBM},
    }
    if not args.no_cpu_baseline:
        threads = min(16, os.cpu_count() or 1)
        torch.set_num_threads(threads)
        n = min(B, 8)
        t0 = time.perf_counter()
        with torch.no_grad():
            for b in range(n):
                orc.style_encoder(orc.wave_preprocess(waves[b]).unsqueeze(1), sd)
        dt = time.perf_counter() - t0
        line["cpu_baseline"] = {"value": n / dt, "unit": "chunks/s", "cores": threads, "kind": "port",
                                "sample": f"{n} chunks, oracle wave_preprocess + style_encoder fp32 on torch-CPU"}
    print(json.dumps(line))


if __name__ == "__main__":
    main()
