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
                    [--no-profile] [--no-parity-mode] [--no-e2e]

N GPUs = N processes, one per GPU (config 4, BASELINE configs[3]): when WORLD_SIZE is not set
and N > 1, this process spawns `torch.distributed.run --nproc-per-node N` as a child (it never
touches the GPU itself) and exits with the child's status; under torch.distributed.run every rank
reads RANK / LOCAL_RANK / WORLD_SIZE and refuses to run if WORLD_SIZE != --gpus.  Rank r decodes
its contiguous shard of the N x B global utterances (stts2_mi355x.shard.shard_range) with the
device noise keyed by GLOBAL utterance id, so the audio does not depend on N.  There is no
collective on the audio path (weak scaling); the timed region is bracketed by a barrier and
device syncs, and rank 0 prints ONE JSON line with the max over ranks.  A second timed figure
adds the RCCL gather of every rank's audio to rank 0 (`with_gather`).

--selftest-cpu (tests only): gloo on the CPU, the decoder replaced by a deterministic stand-in
of the same output shape, so the spawn / shard / barrier / max / gather plumbing runs without a
GPU (tests/test_bench_launcher.py).
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
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
PEAK_MFMA = {"bf16": 2.5e15, "fp32": 157.3e12, "bf16x3": 2.5e15 / 3}  # dense FLOP/s (bf16x3: 3 bf16 MFMAs a product)
# algorithmic work per output sample (activation bytes: each conv reads its input
# once and writes its output once, everything else fused)
ALG = {"hifigan": {"flops": 2.913e6, "bytes": {"bf16": 9709.0, "fp32": 19417.0, "bf16x3": 19417.0}},
       "istftnet": {"flops": 2.163e6, "bytes": {"bf16": 3632.0, "fp32": 7265.0, "bf16x3": 7265.0}}}
METRIC = "24 kHz audio samples/sec/GPU + real-time factor, 10-s utterance batch"


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


def cpu_baseline(kind, dec, cfg, T, reps=3):
    """The oracle (CPU restatement of the reference, oracle/stts_oracle.py) on this host's cores, timed as
    BASELINE.md plans it: per batch size (B = 1, then B = 4), one untimed warm-up call, then the median of
    `reps` timed calls; samples/s, x real time and ms per batch."""
    from oracle import stts_oracle as orc
    from stts2_mi355x import synth
    # the GPU box exports OMP_NUM_THREADS = this job's CPU share (nproc reports the whole host)
    torch.set_num_threads(int(os.environ.get("OMP_NUM_THREADS", "0")) or os.cpu_count() or 1)
    sd = {k: v.detach().cpu() for k, v in dec.state_dict().items()}
    fn = orc.decoder_hifigan if kind == "hifigan" else orc.decoder_istft

    def leg(Bc):
        asr, f0, n, s = synth.decoder_inputs(Bc, T, utt0=0)
        noise = synth.source_noise(Bc, 600 * T, utt0=0)
        args = [torch.from_numpy(a) for a in (asr, f0, n, s)]
        nz = torch.from_numpy(noise)
        times = []
        for i in range(1 + reps):
            t0 = time.perf_counter()
            with torch.no_grad():
                fn(*args, sd, cfg, nz)
            if i:  # call 0 is the warm-up
                times.append(time.perf_counter() - t0)
        med = float(np.median(times))
        return {"value": Bc * 600 * T / med, "unit": "samples/s", "x_realtime": Bc * 600 * T / med / 24000.0,
                "ms_per_batch": med * 1e3, "ms_per_batch_all": [t * 1e3 for t in times]}

    b1 = leg(1)
    res = dict(b1, cores=torch.get_num_threads(), kind="port",
               sample=f"B=1 x {T * 600 // 24000}-s utterance, 1 warm-up + median of {reps} calls, oracle/stts_oracle.py "
                      f"{'decoder_hifigan' if kind == 'hifigan' else 'decoder_istft'} fp32 on torch-CPU")
    # BASELINE.md plans the CPU figure at B = 1 and B = 4 (the reference's CPU path is slower per sample batched)
    res["b4"] = dict(leg(4), sample=f"B=4 x {T * 600 // 24000}-s utterances, 1 warm-up + median of {reps} calls, "
                                    "same function")
    return res


def roofline(recs, dtype, steps, step_ms, B, T, decoder):
    """Roofline of the dominant kernel (the conv engine with the most hipEvent-timed time in the
    profiled steps).  achieved = its algorithmic work (SURVEY.md §8(d) byte / flop model, summed over
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
    t_mfma, t_hbm = f["flops"] / PEAK_MFMA[dtype], f["bytes"] / PEAK_HBM
    if t_mfma >= t_hbm:
        roof = {"bound": "mfma", "achieved": f["flops"] / t_k / 1e12, "peak": PEAK_MFMA[dtype] / 1e12,
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
    roof["kernel_share_of_step"] = f["ms"] / steps / step_ms
    roof["conv_engines"] = {k: {"ms_per_step": v["ms"] / steps, "launches_per_step": v["launches"] // steps,
                                "tflops": v["flops"] / (v["ms"] / 1e3) / 1e12,
                                "alg_GBps": v["bytes"] / (v["ms"] / 1e3) / 1e9} for k, v in sorted(fam.items())}
    tr = _pmc_traffic(name, dtype, B, T, decoder, f["launches"] // steps)
    if tr is not None:
        roof["traffic"] = tr["hbm_bytes_per_launch"]
        roof["traffic_source"] = tr["source"]
    return roof


def _pmc_traffic(kernel, dtype, B, T, decoder, launches_per_step=None):
    # (a file whose passes counted another number of launches of the family per step was taken on another routing:
    # skipped, so the traffic figure never describes a different set of launches than `achieved`)
    import glob
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "*_traffic.json")), reverse=True):
        try:
            with open(path) as fh:
                d = json.load(fh)
        except (OSError, ValueError):
            continue
        if (d.get("kernel") == kernel and d.get("decoder") == decoder and d.get("dtype") == dtype
                and d.get("batch") == B and d.get("frames") == T
                and (launches_per_step is None or d.get("dispatches", 0) == 2 * launches_per_step)):
            return {"hbm_bytes_per_launch": d["hbm_bytes_per_launch"], "source": os.path.relpath(path, ROOT)}
    return None


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn(args_list, n):
    """N ranks as children of this (GPU-untouched) process: torch.distributed.run, one per GPU."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.abspath(__file__), *args_list]
    return subprocess.call(cmd)


class Stand_in:
    """--selftest-cpu: the decoder's output contract ([B,1,600T] float32, a pure function of the
    GLOBAL utterance ids and the step seed) without a GPU."""

    def forward(self, asr, f0, n, s, noise=None, seed=0, utt_offset=0, out=None):
        B, T = asr.shape[0], asr.shape[2]
        ids = torch.arange(utt_offset, utt_offset + B, dtype=torch.float64).reshape(B, 1, 1)
        t = torch.arange(600 * T, dtype=torch.float64).reshape(1, 1, -1)
        out.copy_(torch.sin(0.001 * t * (ids + 1) + float(seed % 1000)).float())
        return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10, help="timed steps (SURVEY §8(d): median of >= 10)")
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=32, help="utterances per GPU")
    ap.add_argument("--frames", type=int, default=400, help="asr frames per utterance (400 = 10 s)")
    ap.add_argument("--decoder", default="hifigan", choices=["hifigan", "istftnet"])
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp32", "bf16x3"])
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-profile", action="store_true")
    ap.add_argument("--no-parity-mode", action="store_true", help="skip the fp32 figure of the same workload")
    ap.add_argument("--no-accuracy-mode", action="store_true", help="skip the bf16x3 figure of the same workload")
    ap.add_argument("--no-e2e", action="store_true", help="skip the host-to-host (PCIe-inclusive) figure")
    ap.add_argument("--selftest-cpu", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--dump-checksum", default=None, help=argparse.SUPPRESS)
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(spawn(sys.argv[1:], args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: launched with WORLD_SIZE={world} but --gpus {args.gpus}")
    cpu = args.selftest_cpu
    # STTS_BENCH_SHARE_GPU=1 (hardware rehearsal of the N-rank path on a one-GPU box; never a scaling figure): every
    # rank decodes on cuda:0 and the collectives run on gloo, staged through host memory (shard.py)
    share = world > 1 and not cpu and os.environ.get("STTS_BENCH_SHARE_GPU") == "1"
    dist = None
    if world > 1:
        import torch.distributed as dist
        if cpu:
            dist.init_process_group("gloo")
        elif share:
            torch.cuda.set_device(0)
            dist.init_process_group("gloo")
        else:
            torch.cuda.set_device(local)
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))  # RCCL
    elif not cpu:
        torch.cuda.set_device(0)
    dev = torch.device("cpu") if cpu else torch.device("cuda", torch.cuda.current_device())
    cdev = torch.device("cpu") if (cpu or share) else dev  # where the bench's own small collective tensors live

    def sync():
        if not cpu:
            torch.cuda.synchronize()

    from stts2_mi355x import shard, synth
    B_local, T = args.batch, args.frames
    global_batch = world * B_local
    utt0, B = shard.shard_range(global_batch, world, rank)
    if cpu:
        eng, dec, cfg = Stand_in(), None, None
    else:
        from stts2_mi355x import engine as E
        dec, cfg = build_decoder(args.decoder)
        dec = dec.to(dev)
        eng = dec.engine(args.dtype)
    host_in = synth.decoder_inputs(B, T, utt0=utt0)
    asr, f0, n, s = (torch.from_numpy(a).to(dev) for a in host_in)
    out = torch.empty(B, 1, 600 * T, device=dev)

    def step(i, e=eng, o=out):
        e.forward(asr, f0, n, s, noise=None, seed=1234 + i, utt_offset=utt0, out=o)

    def timed(fn, k, w, gather=False):
        """w untimed + k timed calls of fn(i) between barrier + device syncs: max over ranks of the
        wall time, and the per-step device times (events) for the median."""
        for i in range(w):
            fn(i)
        sync()
        if dist:
            dist.barrier()
        sync()
        evs = [] if cpu else [torch.cuda.Event(enable_timing=True) for _ in range(k + 1)]
        t0 = time.perf_counter()
        if evs:
            evs[0].record()
        for i in range(k):
            fn(w + i)
            if gather:
                shard.gather_to_rank0(out, world, rank)
            if evs:
                evs[i + 1].record()
        sync()
        el = time.perf_counter() - t0
        per = [evs[i].elapsed_time(evs[i + 1]) for i in range(k)] if evs else [el * 1e3 / k] * k
        if dist:
            t = torch.tensor([el], dtype=torch.float64, device=cdev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            el = t.item()
            dist.barrier()
        return el, per

    el, per = timed(step, args.steps, args.warmup)
    samples = global_batch * 600 * T * args.steps
    value = samples / el
    ms = el / args.steps * 1e3

    # second figure: the same steps with every rank's audio gathered to rank 0 over RCCL
    with_gather = None
    with_scatter_gather = None
    if dist:
        elg, _ = timed(step, args.steps, 1, gather=True)
        with_gather = {"value": samples / elg, "ms_per_step": elg / args.steps * 1e3,
                       "gathered_bytes_per_step": global_batch * 600 * T * 4}
        # third figure: rank 0 holds the whole global batch's inputs on its device; each step scatters every
        # rank's utterance shard over RCCL (shard.scatter_from_rank0), decodes, and gathers the audio back
        g_in = ([torch.from_numpy(a).to(dev) for a in synth.decoder_inputs(global_batch, T, utt0=0)]
                if rank == 0 else [None] * 4)
        parts = [shard.scatter_from_rank0(g, world, rank, device=dev) for g in g_in]
        # the scattered shard must be this rank's own inputs; the verdict is agreed over all ranks (a collective), so
        # that a mismatch skips this leg everywhere instead of leaving the other ranks waiting in its collectives
        bad = torch.tensor([0 if all(torch.equal(a_, b_) for a_, b_ in zip(parts, (asr, f0, n, s))) else 1],
                           dtype=torch.int32, device=cdev)
        dist.all_reduce(bad, op=dist.ReduceOp.MAX)
        if bad.item():
            with_scatter_gather = {"error": "scattered inputs differ from the shards' own inputs"}
        else:
            def step_sg(i):
                a_, f_, n_, s_ = (shard.scatter_from_rank0(g, world, rank, device=dev) for g in g_in)
                eng.forward(a_, f_, n_, s_, noise=None, seed=1234 + i, utt_offset=utt0, out=out)
                shard.gather_to_rank0(out, world, rank)
            els, _ = timed(step_sg, args.steps, 1)
            with_scatter_gather = {"value": samples / els, "ms_per_step": els / args.steps * 1e3,
                                   "scattered_bytes_per_step": sum(g.numel() * 4 for g in g_in) if rank == 0 else None,
                                   "gathered_bytes_per_step": global_batch * 600 * T * 4}
    if args.dump_checksum is not None:  # tests: the audio of every utterance, gathered to rank 0
        step(0)
        full = shard.gather_to_rank0(out, world, rank) if dist else out
        if rank == 0:
            np.save(args.dump_checksum, full.cpu().numpy())

    prof_recs = None
    if not cpu and not args.no_profile:  # per-launch hipEvents: a separate pass, not the timed one
        # the timed pass runs the production options (the noise branches on a side stream beside the front-end and
        # the stages, STTS_OPT_NBRANCH); this pass runs every conv launch alone, so that its hipEvent duration
        # prices the kernel rather than the overlap
        nb0 = E.get_option(E.OPT_NBRANCH)
        E.set_option(E.OPT_NBRANCH, 0)
        E.profile_enable(True)
        for i in range(2):
            step(100 + i)
        sync()
        prof_recs = E.profile_launches()
        E.profile_enable(False)
        E.set_option(E.OPT_NBRANCH, nb0)
    parity = None
    if not cpu and not args.no_parity_mode and args.dtype != "fp32":
        # the north-star accuracy mode (fp32 storage + exact-fp32 MFMA, 10-s max-abs 2.7e-6 vs the
        # reference) on the same workload
        peng = dec.engine("fp32")
        elp, perp = timed(lambda i: step(i, e=peng), 3, 1)
        parity = {"dtype": "fp32", "steps": 3, "ms_per_step": elp / 3 * 1e3,
                  "value": global_batch * 600 * T * 3 / elp,
                  "hbm_fraction": ALG[args.decoder]["bytes"]["fp32"] * global_batch * 600 * T * 3 / elp / PEAK_HBM,
                  "mfma_fraction": ALG[args.decoder]["flops"] * global_batch * 600 * T * 3 / elp / PEAK_MFMA["fp32"]}
        dec.engine(args.dtype)
    accuracy = None
    if not cpu and not args.no_accuracy_mode and args.dtype == "bf16":
        # the split-operand accuracy mode (fp32 storage, conv operands as bf16 hi + lo on the bf16 MFMA:
        # 10-s max-abs 2.5e-5 vs the reference, tests/test_gpu_split.py) on the same workload
        aeng = dec.engine("bf16x3")
        ela, _ = timed(lambda i: step(i, e=aeng), 3, 1)
        nsm = global_batch * 600 * T * 3
        accuracy = {"dtype": "bf16x3", "steps": 3, "ms_per_step": ela / 3 * 1e3, "value": nsm / ela,
                    "hbm_fraction": ALG[args.decoder]["bytes"]["bf16x3"] * nsm / ela / PEAK_HBM,
                    "mfma_fraction": ALG[args.decoder]["flops"] * nsm / ela / PEAK_MFMA["bf16x3"],
                    "vs_parity_mode": (nsm / ela) / parity["value"] if parity else None}
        if not args.no_profile:  # its own dominant kernel against the bf16x3 peak (2.5 PF / 3), per-launch hipEvents
            nb0 = E.get_option(E.OPT_NBRANCH)
            E.set_option(E.OPT_NBRANCH, 0)
            E.profile_enable(True)
            for i in range(2):
                step(200 + i, e=aeng)
            sync()
            arecs = E.profile_launches()
            E.profile_enable(False)
            E.set_option(E.OPT_NBRANCH, nb0)
            accuracy["roofline"] = roofline(arecs, "bf16x3", 2, accuracy["ms_per_step"], B, T, args.decoder)
        dec.engine(args.dtype)
    e2e = None
    if not cpu and not args.no_e2e:
        # host -> host: pinned host inputs copied in, decoded, audio copied back (PCIe included)
        pins = [torch.from_numpy(a).pin_memory() for a in host_in]
        hout = torch.empty(B, 1, 600 * T).pin_memory()

        def h2h(i):
            a, f, nn_, st = (p.to(dev, non_blocking=True) for p in pins)
            eng.forward(a, f, nn_, st, noise=None, seed=1234 + i, utt_offset=utt0, out=out)
            hout.copy_(out, non_blocking=True)
        ele, _ = timed(h2h, 3, 1)
        e2e = {"value": global_batch * 600 * T * 3 / ele, "ms_per_step": ele / 3 * 1e3,
               "note": "inputs H2D from pinned host memory + decode + audio D2H, per step"}
    if rank != 0:
        if dist:
            dist.destroy_process_group()
        return
    a = ALG[args.decoder]
    line = {
        "metric": METRIC,
        "value": value,
        "unit": "samples/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms,
        "ms_per_step_median": float(np.median(per)),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": args.dtype,
        "data": "synthetic (formula weights + SURVEY §8(d) input distributions; device counter-RNG noise)"
                + (" [SELFTEST: CPU stand-in decoder, not a measurement]" if cpu else ""),
        "config": {"workload": f"{args.decoder} decoder, batch {B_local}/GPU x {T * 600 // 24000}-s utterances "
                               f"({T} asr frames, {600 * T} samples each)",
                   "global_batch": global_batch, "frames": T, "decoder": args.decoder,
                   "parallelism": (f"dp{world} rehearsal: {world} ranks sharing cuda:0 over gloo (STTS_BENCH_SHARE_GPU)" if share
                                   else f"dp{world} (utterance shards, no collective on the audio path)")},
        "x_realtime_per_gpu": value / world / 24000.0,
        "hbm_fraction": a["bytes"][args.dtype] * value / world / PEAK_HBM,
        "mfma_fraction": a["flops"] * value / world / PEAK_MFMA[args.dtype],
        # SURVEY §8(d)'s names: the same two whole-step fractions
        "mfma_or_valu_fraction": a["flops"] * value / world / PEAK_MFMA[args.dtype],
        "roofline": roofline(prof_recs, args.dtype, 2, ms, B, T, args.decoder) if prof_recs else None,
    }
    if with_gather:
        line["with_gather"] = with_gather
    if with_scatter_gather:
        line["with_scatter_gather"] = with_scatter_gather
    if parity:
        line["parity_mode"] = parity
    if accuracy:
        line["accuracy_mode"] = accuracy
    if e2e:
        line["e2e_pcie"] = e2e
    if not cpu and not args.no_cpu_baseline and world == 1:
        line["cpu_baseline"] = cpu_baseline(args.decoder, dec.cpu(), cfg, T)
    print(json.dumps(line), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
