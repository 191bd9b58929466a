#!/usr/bin/env python3
"""Measurement of the duration / text row.  Prints ONE JSON line.

    python tools/bench_duration.py [--batch 32] [--tokens 130] [--frames 400] [--steps 10] [--warmup 2]
                                   [--no-cpu-baseline]

Workloads (synthetic formula weights, inputs resident in HBM, fp32):
  * duration path: TextEncoder -> DurationEncoder -> predictor.lstm -> duration_proj -> stts_durations
    for B utterances of `tokens` tokens (130 tokens ~ a 10-s utterance at ~3 frames a token);
  * the F0Ntrain shared BiLSTM at B x `frames` (400 frames = 10 s), the largest recurrence of the path;
  * one utterance end to end (Synthesizer.inference: tokens -> waveform, HiFi-GAN decoder fp32 and
    bf16), the reference's own inference.py unit (B = 1: the cooperative BiLSTM recurrence runs).
Timing: torch.cuda.Event pairs on the current stream (the library launches on it).

The BiLSTM recurrence is a chain of `len` dependent steps: its bound is per-step latency, not HBM or
FLOP/s.  `lstm_roofline` still reports its algorithmic work -- per step and direction 4H x H FMAs
(2 flop) over the recurrent weights (4H x H x 4 B, read from L2, not HBM, after the first step) --
against the fp32 vector peak, and the measured time per step.
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

PEAK_FP32 = 157.3e12


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
    ap.add_argument("--tokens", type=int, default=130)
    ap.add_argument("--frames", type=int, default=400)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-e2e", action="store_true", help="skip the one-utterance end-to-end leg")
    ap.add_argument("--e2e-tokens", type=int, default=14,
                    help="tokens of the end-to-end utterance (formula weights give ~25 frames a token: "
                         "14 (+2 pads) ~ 400 frames = 10 s)")
    args = ap.parse_args()

    from helpers import make_decoder, make_duration_modules
    from stts2_mi355x import synth
    from stts2_mi355x.inference import Synthesizer
    from stts2_mi355x.prosody import durations, linear_frames

    B, T, Fr = args.batch, args.tokens, args.frames
    dev = torch.device("cuda", 0)
    te_c, pp_c = make_duration_modules()
    te_sd = {k: v.clone() for k, v in te_c.state_dict().items()}
    pp_sd = {k: v.clone() for k, v in pp_c.state_dict().items()}
    te, pp = te_c.to(dev), pp_c.to(dev)
    tok = torch.from_numpy((synth.hash_u01("bench:dur:tok", B * T) * 177 + 1).astype(np.int64).reshape(B, T)).to(dev)
    ln = torch.full((B,), T, dtype=torch.int32, device=dev)
    s = torch.from_numpy(synth.normal("bench:dur:s", (B, 128))).to(dev)
    z = torch.from_numpy(synth.normal("bench:dur:z", (B, T))).to(dev)

    def duration_path():
        t_en = te(tok, ln)
        d = pp.text_encoder(t_en, s, ln)
        x, _ = pp.lstm(d, lengths=ln)
        lin = pp.duration_proj.linear_layer
        return durations(linear_frames(x, lin.weight, lin.bias), ln, z, mix=0.1)

    en = torch.from_numpy(synth.normal("bench:dur:en", (B, 640, Fr))).to(dev)
    with torch.no_grad():
        dur_ms = timed(duration_path, args.steps, args.warmup)
        lstm_ms = timed(lambda: pp.shared(en.transpose(-1, -2)), args.steps, args.warmup)
        f0n_ms = timed(lambda: pp.F0Ntrain(en, s), args.steps, args.warmup)

    # one utterance end to end (inference.py unit), fp32 and bf16 decoders
    dec, _ = make_decoder("hifigan")
    dec = dec.to(dev)
    tokens1 = [int(v) for v in (synth.hash_u01("bench:e2e:tok", args.e2e_tokens) * 177 + 1)]
    s1 = s[:1]
    e2e = {}
    for dt in (() if args.no_e2e else ("fp32", "bf16")):
        syn = Synthesizer(te, pp, dec, decoder_dtype=dt)
        z1 = torch.zeros(1, args.e2e_tokens + 2, device=dev)
        frames = syn.alignment(tokens1, s1, t=0.1, z=z1)["frames"]
        ms = timed(lambda: syn.inference(tokens1, s1, t=0.1, z=z1), max(2, args.steps // 2), 1)
        e2e[dt] = {"ms": ms, "tokens": args.e2e_tokens + 2, "frames": frames, "samples": 600 * frames,
                   "x_realtime": (600 * frames / 24000) / (ms / 1e3)}

    H = 256
    lstm_flops = 2 * B * Fr * 2 * (4 * H * H + 4 * H * 640)  # recurrence + input projection
    line = {
        "metric": "duration path: utterances/s (TextEncoder + DurationEncoder + duration LSTM + durations)",
        "value": B / (dur_ms / 1e3), "unit": "utterances/s", "n_gpus": 1, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": dur_ms, "higher_is_better": True, "dtype": "fp32",
        "data": "synthetic (formula weights and token ids, synth.py)",
        "config": {"workload": f"{B} utterances x {T} tokens (duration path); shared BiLSTM {B} x {Fr} frames",
                   "batch": B, "tokens": T, "frames": Fr},
        "shared_lstm": {"ms": lstm_ms, "us_per_step": lstm_ms * 1e3 / Fr, "tflops": lstm_flops / (lstm_ms / 1e3) / 1e12},
        "f0ntrain_ms": f0n_ms,
        "end_to_end_one_utterance": e2e,
        "lstm_roofline": {"bound": "latency (dependent steps)", "achieved": lstm_flops / (lstm_ms / 1e3) / 1e12,
                          "peak": PEAK_FP32 / 1e12, "unit": "TFLOP/s",
                          "frac": lstm_flops / (lstm_ms / 1e3) / PEAK_FP32},
    }

    if not args.no_cpu_baseline:
        from oracle import stts_oracle as orc
        nb = min(B, 4)
        torch.set_num_threads(int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1)))
        tok_c, s_c = tok[:nb].cpu(), s[:nb].cpu()
        ln_c = torch.full((nb,), T, dtype=torch.int64)
        t0 = time.perf_counter()
        t_en = orc.text_encoder(tok_c, ln_c, te_sd)
        d = orc.duration_encoder(t_en, s_c, ln_c, pp_sd, "text_encoder.")
        x = orc.bilstm(d, pp_sd, "lstm.", ln_c)
        torch.nn.functional.linear(x, pp_sd["duration_proj.linear_layer.weight"],
                                   pp_sd["duration_proj.linear_layer.bias"])
        dt = time.perf_counter() - t0
        line["cpu_baseline"] = {"value": nb / dt, "unit": "utterances/s", "cores": torch.get_num_threads(),
                                "kind": "port", "sample": f"{nb} utterances x {T} tokens, oracle on torch-CPU"}
    print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
