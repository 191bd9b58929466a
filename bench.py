#!/usr/bin/env python3
"""Throughput benchmark of the MI355X-native StyleTTS2-lite synthesis path.

Headline (BASELINE.json `metric`, `configs[2]`): 24 kHz samples/s and real-time factor of
the HiFi-GAN decoder, bf16, on a batch of 32 ten-second utterances (T = 400 asr frames =
800 F0 frames = 240,000 samples each) per GPU.  One "step" = one decoder forward over the
batch (front-end, harmonic source, 4 upsampling stages, conv_post + tanh), inputs already
resident in HBM.  Weights are the formula weights of stts2_mi355x.synth (the LibriTTS
checkpoint is download-only); inputs are synthetic with the SURVEY.md §8(d) distributions.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--batch 32] [--frames 400]
                    [--decoder hifigan|istftnet] [--dtype bf16|fp32] [--no-cpu-baseline]

N > 1 is launched by torch.distributed.run (one process per GPU, RCCL): utterances are
sharded by rank (weak scaling, no data-path collective); timing is bracketed by a barrier
and device syncs and the max over ranks is reported by rank 0 as ONE JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "styletts2-lite_amd"))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

HIFI_CFG = dict(resblock_kernel_sizes=[3, 7, 11], upsample_rates=[10, 5, 3, 2], upsample_initial_channel=512,
                resblock_dilation_sizes=[[1, 3, 5], [1, 3, 5], [1, 3, 5]], upsample_kernel_sizes=[20, 10, 6, 4])
ISTFT_CFG = dict(resblock_kernel_sizes=[3, 7, 11], upsample_rates=[10, 6], upsample_initial_channel=512,
                 resblock_dilation_sizes=[[1, 3, 5], [1, 3, 5], [1, 3, 5]], upsample_kernel_sizes=[20, 12],
                 gen_istft_n_fft=20, gen_istft_hop_size=5)
PEAK_HBM = 8.0e12        # B/s, MI355X HBM3E (MI355X_MICROARCH.md chip table)
PEAK_MFMA = {"bf16": 2.5e15, "fp32": 157.3e12}  # dense FLOP/s


def build_decoder(kind):
    from stts2_mi355x import synth
    if kind == "hifigan":
        from stts2_mi355x.hifigan import Decoder
        d = Decoder(dim_in=512, style_dim=128, dim_out=80, **HIFI_CFG)
    else:
        from stts2_mi355x.istftnet import Decoder
        d = Decoder(dim_in=512, style_dim=128, dim_out=80, **ISTFT_CFG)
    sd = d.state_dict()
    new = {k: (v if synth.is_fixed_buffer(k) else torch.from_numpy(synth.synth_param(k, tuple(v.shape))))
           for k, v in sd.items()}
    d.load_state_dict(new)
    return d.eval(), (HIFI_CFG if kind == "hifigan" else ISTFT_CFG)


def cpu_baseline(kind, dec, cfg, T, budget_s=12.0):
    """The oracle (CPU restatement of the reference, oracle/stts_oracle.py) on this host's cores,
    one utterance at a time until `budget_s` of CPU work: samples/s."""
    from oracle import stts_oracle as orc
    from stts2_mi355x import synth
    # the GPU box exports OMP_NUM_THREADS = this job's CPU share (nproc reports the whole host)
    torch.set_num_threads(int(os.environ.get("OMP_NUM_THREADS", "0")) or os.cpu_count() or 1)
    sd = {k: v.detach().cpu() for k, v in dec.state_dict().items()}
    fn = orc.decoder_hifigan if kind == "hifigan" else orc.decoder_istft
    done, t0 = 0, time.perf_counter()
    while True:
        asr, f0, n, s = synth.decoder_inputs(1, T, utt0=done)
        noise = synth.source_noise(1, 600 * T, utt0=done)
        with torch.no_grad():
            fn(*(torch.from_numpy(a) for a in (asr, f0, n, s)), sd, cfg, torch.from_numpy(noise))
        done += 1
        el = time.perf_counter() - t0
        if el >= budget_s or done >= 8:
            break
    return {"value": done * 600 * T / el, "unit": "samples/s", "cores": torch.get_num_threads(), "kind": "port",
            "sample": f"{done} x {T * 600 // 24000}-s utterance(s), B=1, oracle/stts_oracle.py "
                      f"{'decoder_hifigan' if kind == 'hifigan' else 'decoder_istft'} fp32 on torch-CPU"}


def roofline(recs, args, el, B, T):
    """Roofline of the dominant kernel (the conv engine with the most hipEvent-timed time in the
    timed region).  achieved = its algorithmic work (SURVEY.md §8(d) byte / flop model, summed over
    its launches) / its measured time; bound = whichever of MFMA / HBM floors is larger for that
    work.  traffic = HBM bytes per launch from the committed rocprofv3 FETCH_SIZE / WRITE_SIZE
    passes (tools/pmc_traffic.py -> profiles/*_traffic.json) when they were taken on this exact
    workload and kernel, else null."""
    fam = {}
    for r in recs:
        f = fam.setdefault(r["kernel"], {"ms": 0.0, "flops": 0.0, "bytes": 0.0, "launches": 0})
        f["ms"] += r["ms"]
        f["flops"] += r["flops"]
        f["bytes"] += r["bytes"]
        f["launches"] += 1
    name, f = max(fam.items(), key=lambda kv: kv[1]["ms"])
    t_k = f["ms"] / 1e3
    t_mfma, t_hbm = f["flops"] / PEAK_MFMA[args.dtype], f["bytes"] / PEAK_HBM
    if t_mfma >= t_hbm:
        roof = {"bound": "mfma", "achieved": f["flops"] / t_k / 1e12, "peak": PEAK_MFMA[args.dtype] / 1e12,
                "unit": "TFLOP/s"}
    else:
        roof = {"bound": "hbm", "achieved": f["bytes"] / t_k / 1e9, "peak": PEAK_HBM / 1e9, "unit": "GB/s"}
    roof["frac"] = roof["achieved"] / roof["peak"]
    roof["traffic"] = None
    roof["kernel"] = name
    roof["launches"] = f["launches"]
    roof["avg_launch_us"] = f["ms"] * 1e3 / f["launches"]
    roof["alg_flops_per_launch"] = f["flops"] / f["launches"]
    roof["alg_bytes_per_launch"] = f["bytes"] / f["launches"]
    roof["kernel_share_of_step"] = f["ms"] / (el * 1e3)
    roof["conv_engines"] = {k: {"ms_per_step": v["ms"] / args.steps, "launches_per_step": v["launches"] // args.steps,
                                "tflops": v["flops"] / (v["ms"] / 1e3) / 1e12,
                                "alg_GBps": v["bytes"] / (v["ms"] / 1e3) / 1e9} for k, v in sorted(fam.items())}
    tr = _pmc_traffic(name, args, B, T)
    if tr is not None:
        roof["traffic"] = tr["hbm_bytes_per_launch"]
        roof["traffic_source"] = tr["source"]
    return roof


def _pmc_traffic(kernel, args, B, T):
    import glob
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "*_traffic.json")), reverse=True):
        try:
            with open(path) as fh:
                d = json.load(fh)
        except (OSError, ValueError):
            continue
        if (d.get("kernel") == kernel and d.get("decoder") == args.decoder and d.get("dtype") == args.dtype
                and d.get("batch") == B and d.get("frames") == T):
            return {"hbm_bytes_per_launch": d["hbm_bytes_per_launch"], "source": os.path.relpath(path, ROOT)}
    return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--batch", type=int, default=32, help="utterances per GPU")
    ap.add_argument("--frames", type=int, default=400, help="asr frames per utterance (400 = 10 s)")
    ap.add_argument("--decoder", default="hifigan", choices=["hifigan", "istftnet"])
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp32"])
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-profile", action="store_true")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        dist = None
        torch.cuda.set_device(0)
    dev = torch.device("cuda", torch.cuda.current_device())

    from stts2_mi355x import engine as E
    from stts2_mi355x import synth

    B, T = args.batch, args.frames
    dec, cfg = build_decoder(args.decoder)
    dec = dec.to(dev)
    utt0 = rank * B  # global utterance ids of this shard
    asr, f0, n, s = (torch.from_numpy(a).to(dev) for a in synth.decoder_inputs(B, T, utt0=utt0))
    eng = dec.engine(args.dtype)
    out = torch.empty(B, 1, 600 * T, device=dev)

    def step(i):
        eng.forward(asr, f0, n, s, noise=None, seed=1234 + i, utt_offset=utt0, out=out)

    for i in range(args.warmup):
        step(i)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    if not args.no_profile:
        E.profile_enable(True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(args.warmup + i)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    prof_recs = E.profile_launches() if not args.no_profile else None
    E.profile_enable(False)
    if dist:
        t = torch.tensor([el], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = t.item()
        dist.barrier()
    if rank != 0:
        if dist:
            dist.destroy_process_group()
        return
    samples = world * B * 600 * T * args.steps
    value = samples / el
    ms = el / args.steps * 1e3
    roof = roofline(prof_recs, args, el, B, T) if prof_recs else None
    line = {
        "metric": "24 kHz audio samples/sec/GPU + real-time factor, 10-s utterance batch",
        "value": value,
        "unit": "samples/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": args.dtype,
        "data": "synthetic (formula weights + SURVEY §8(d) input distributions; device counter-RNG noise)",
        "config": {"workload": f"{args.decoder} decoder, batch {B}/GPU x {T * 600 // 24000}-s utterances "
                               f"({T} asr frames, {600 * T} samples each)",
                   "global_batch": world * B, "frames": T, "decoder": args.decoder,
                   "parallelism": f"dp{world} (utterance shards, no collective on the audio path)"},
        "x_realtime_per_gpu": value / world / 24000.0,
        "roofline": roof,
    }
    if not args.no_cpu_baseline and world == 1:
        line["cpu_baseline"] = cpu_baseline(args.decoder, dec.cpu(), cfg, T)
    print(json.dumps(line), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
