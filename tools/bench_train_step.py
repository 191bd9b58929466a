"""Config-5 training step (BASELINE configs[4]: train.py fine-tune step, decoder + MPD/MSD fwd/bwd,
batch_size 2, max_len 310 -> B = 2 segments of 155 asr frames = 93,000 samples) on one MI355X.

One step = TrainStep (stts2_mi355x/trainstep.py): decoder forward, DiscriminatorLoss fwd/bwd + AdamW on MSD
and MPD, MultiResolutionSTFTLoss + GeneratorLoss fwd/bwd + AdamW on the decoder, all HIP kernels.  Inputs
(en, F0, N, s, wav) synthetic and resident in HBM, formula weights.  Prints one JSON line per dtype:
ms per step (median of hipEvent-timed steps and wall), conv work per step (algorithmic flops of every conv
forward, dx and dw the step launches) and its rate against the dense MFMA peak of the dtype; with
--cpu-baseline also the oracle's step (oracle.train_step, torch CPU autograd) on the host cores.

    python tools/bench_train_step.py [--steps 10] [--warmup 3] [--dtypes fp32,bf16] [--cpu-baseline]
                                     [--opt KEY=VALUE ...] [--no-grad-check]

Each dtype line also carries `grad_vs_fp32`: one captured step of fresh modules (same formula weights, inputs and
noise) in that dtype against the same step in fp32, per module (decoder, MPD, MSD): the normwise gradient error
max |g - g_fp32| / max |g_fp32|, the cosine of the whole gradient vector, and the first-step AdamW update-sign
agreement with fp32 (the bounds the tests hold: tests/test_gpu_train_step.py BF16_STEP_BOUNDS).
"""
import argparse
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "styletts2-lite_amd"), os.path.join(ROOT, "tests")]
import torch  # noqa: E402

PEAK = {"fp32": 157.3e12, "bf16": 2.5e15, "bf16x3": 2.5e15 / 3}  # MI355X dense MFMA (MI355X_MICROARCH.md); bf16x3: 3 MFMAs a product


def build(B, T):
    from helpers import fill_module, make_decoder
    from stts2_mi355x.synth import waves
    from stts2_mi355x import synth
    from stts2_mi355x.discriminators import MultiPeriodDiscriminator, MultiResSpecDiscriminator
    dec, _ = make_decoder("hifigan")
    mpd = fill_module(MultiPeriodDiscriminator(), "mpd.")
    msd = fill_module(MultiResSpecDiscriminator(), "msd.")
    asr, f0, n, s = (torch.from_numpy(a) for a in synth.decoder_inputs(B, T, tag="train"))
    wav = torch.from_numpy(waves(B, 600 * T, 7))
    return dec, mpd, msd, (asr, f0, n, s, wav)


def run_gpu(dtype, B, T, steps, warmup, graph=False):
    from stts2_mi355x import training
    from stts2_mi355x.trainstep import TrainStep
    dec, mpd, msd, (asr, f0, n, s, wav) = build(B, T)
    dec, mpd, msd = dec.cuda().eval(), mpd.cuda().train(), msd.cuda().train()
    ins = [t.cuda().requires_grad_(True) for t in (asr, f0, n, s)]
    wav = wav.cuda()
    # (the conv work of one step, counted on the host while an eager step issues its launches)
    training.CONV_FLOPS.update(on=True, fwd=0.0, bwd=0.0)
    TrainStep(dec, mpd, msd, dtype=dtype)(*ins, wav, seed=99)
    training.CONV_FLOPS["on"] = False
    step = TrainStep(dec, mpd, msd, dtype=dtype, graph=graph)
    for i in range(max(warmup, 3 if graph else 1)):  # graph: call 1 eager, call 2 records + replays
        step(*ins, wav, seed=100 + i)
    torch.cuda.synchronize()
    flops = training.CONV_FLOPS["fwd"] + training.CONV_FLOPS["bwd"]
    ev = []
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    host = []
    for i in range(steps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        h0 = time.perf_counter()
        out = step(*ins, wav, seed=1000 + i)
        host.append((time.perf_counter() - h0) * 1e3)
        b.record()
        ev.append((a, b))
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / steps * 1e3
    ms = statistics.median(x.elapsed_time(y) for x, y in ev)
    return {"metric": "config5 train step", "dtype": dtype, "graph": graph, "B": B, "T_frames": T,
            "samples_per_utt": 600 * T,
            "ms_per_step_median": round(ms, 2), "ms_per_step_wall": round(wall, 2), "steps": steps,
            # the host's time to issue one step (Python autograd + C-ABI calls, no sync): ~ms_per_step = host-bound
            "host_ms_per_step": round(statistics.median(host), 2),
            "conv_gflop_per_step": round(flops / 1e9, 1), "conv_tflops": round(flops / ms / 1e9, 2),
            "frac_of_dense_mfma_peak": round(flops / (ms * 1e-3) / PEAK[dtype], 4),
            "losses": {k: float(out[k]) for k in ("d_loss", "loss_mel", "loss_gen_all")},
            "max_mem_gb": round(torch.cuda.max_memory_allocated() / 2 ** 30, 2)}


def captured_step(dtype, B, T):
    from stts2_mi355x.synth import source_noise
    from stts2_mi355x.trainstep import TrainStep
    dec, mpd, msd, (asr, f0, n, s, wav) = build(B, T)
    dec, mpd, msd = dec.cuda().eval(), mpd.cuda().train(), msd.cuda().train()
    p0 = {tag: {k: v.detach().clone() for k, v in m.named_parameters()} for tag, m in
          (("dec", dec), ("mpd", mpd), ("msd", msd))}
    ins = [t.cuda().requires_grad_(True) for t in (asr, f0, n, s)]
    noise = torch.from_numpy(source_noise(B, 600 * T, tag="train_noise")).cuda()
    step = TrainStep(dec, mpd, msd, dtype=dtype, capture=True)
    step(*ins, wav.cuda(), noise=noise)
    torch.cuda.synchronize()
    upd = {tag: {k: (p.detach() - p0[tag][k]) for k, p in m.named_parameters()} for tag, m in
           (("dec", dec), ("mpd", mpd), ("msd", msd))}
    return step.captured, upd


def grad_check(dtype, B, T, ref):
    got, upd = captured_step(dtype, B, T)
    gref, uref = ref
    out = {}
    for tag in ("dec", "mpd", "msd"):
        a = torch.cat([got[tag][k].reshape(-1).double() for k in sorted(gref[tag])])
        b = torch.cat([gref[tag][k].reshape(-1).double() for k in sorted(gref[tag])])
        ua = torch.cat([upd[tag][k].reshape(-1) for k in sorted(uref[tag])])
        ub = torch.cat([uref[tag][k].reshape(-1) for k in sorted(uref[tag])])
        sig = ub.abs() > 0
        out[tag] = {"normwise": float((a - b).abs().max() / b.abs().max()),
                    "cos": float((a @ b) / (a.norm() * b.norm())),
                    "update_sign_agreement": float((torch.sign(ua[sig]) == torch.sign(ub[sig])).float().mean())}
    return out


def run_cpu(B, T):
    from helpers import HIFI_CFG
    from oracle import stts_oracle as orc
    from stts2_mi355x import synth
    dec, mpd, msd, (asr, f0, n, s, wav) = build(B, T)
    sd = lambda m: {k: v.detach().clone() for k, v in m.state_dict().items()}  # noqa: E731
    noise = torch.from_numpy(synth.source_noise(B, 600 * T, tag="train_noise"))
    t0 = time.perf_counter()
    orc.train_step(sd(dec), sd(mpd), sd(msd), HIFI_CFG, asr, f0, n, s, wav, noise)
    sec = time.perf_counter() - t0
    return {"metric": "config5 train step", "kind": "port", "device": "cpu", "cores": torch.get_num_threads(),
            "ms_per_step": round(sec * 1e3, 1), "sample": "one full config-5 step (B=2 x 93,000 samples)"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--dtypes", default="fp32,bf16")
    ap.add_argument("--B", type=int, default=2)
    ap.add_argument("--T", type=int, default=155)
    ap.add_argument("--cpu-baseline", action="store_true")
    ap.add_argument("--no-fold", action="store_true", help="strided convs on the engines' strided path")
    ap.add_argument("--no-fuse-tx", action="store_true", help="MSD convs on the materialised time expansion (A/B)")
    ap.add_argument("--serial-discs", action="store_true", help="sub-discriminators and generator branches on one stream (A/B)")
    ap.add_argument("--opt", action="append", default=[], help="STTS_OPT_* KEY=VALUE held for the run (A/B)")
    ap.add_argument("--no-grad-check", action="store_true")
    ap.add_argument("--graph", action="store_true", help="TrainStep(graph=True): the step recorded once and replayed")
    a = ap.parse_args()
    if a.no_fold:
        from stts2_mi355x import training
        training.FOLD_STRIDED = False
    if a.serial_discs:
        from stts2_mi355x import discriminators, training
        discriminators.CONCURRENT = False
        training.CONCURRENT_BRANCHES = False
    if a.no_fuse_tx:
        from stts2_mi355x import training
        training.FUSE_TX = False
    from stts2_mi355x import engine as E
    for kv in a.opt:
        k, v = (int(x) for x in kv.split("="))
        E.set_option(k, v)
    ref = None if a.no_grad_check else captured_step("fp32", a.B, a.T)
    for dt in a.dtypes.split(","):
        line = run_gpu(dt, a.B, a.T, a.steps, a.warmup, a.graph)
        if a.opt:
            line["options"] = a.opt
        if ref is not None and dt != "fp32":
            line["grad_vs_fp32"] = grad_check(dt, a.B, a.T, ref)
        print(json.dumps(line), flush=True)
    if a.cpu_baseline:
        torch.set_num_threads(int(os.environ.get("OMP_NUM_THREADS", os.cpu_count())))
        print(json.dumps(run_cpu(a.B, a.T)), flush=True)


if __name__ == "__main__":
    main()
