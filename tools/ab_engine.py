"""A/B of an engine option on the headline workload (HiFi-GAN bf16, B x 10 s): per option value,
interleaved rounds in ONE process (cdna_hip_programming.md §5.4 rule 24), the conv engines'
hipEvent time per step and the per-launch-shape times of the dominant engine.

    python tools/ab_engine.py OPT v1 v2 ... [--batch 32] [--rounds 3]
    OPT: an STTS_OPT_* number (include/stts2.h), e.g. 7 (BIGCONV) 1 2 3
"""
import argparse
import collections
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "styletts2-lite_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("opt", type=int)
    ap.add_argument("values", type=int, nargs="+")
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--frames", type=int, default=400)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--dtype", default="bf16")
    ap.add_argument("--set", action="append", default=[], help="KEY=VALUE options held for every variant")
    a = ap.parse_args()
    fixed = [tuple(int(x) for x in kv.split("=")) for kv in a.set]
    from stts2_mi355x import engine as E
    from stts2_mi355x import synth
    torch.cuda.set_device(0)
    dec, _ = bench.build_decoder("hifigan")
    dec = dec.cuda()
    eng = dec.engine(a.dtype)
    asr, f0, n, s = (torch.from_numpy(x).cuda() for x in synth.decoder_inputs(a.batch, a.frames))
    out = torch.empty(a.batch, 1, 600 * a.frames, device="cuda")
    res = {v: collections.defaultdict(list) for v in a.values}
    step_ms = {v: [] for v in a.values}
    outs = {}
    for r in range(a.rounds):
        for v in a.values:
            for k, fv in fixed:
                E.set_option(k, fv)
            E.set_option(a.opt, v)
            eng.forward(asr, f0, n, s, seed=5, out=out)  # warm
            torch.cuda.synchronize()
            ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            ev0.record()
            eng.forward(asr, f0, n, s, seed=5, out=out)
            ev1.record()
            torch.cuda.synchronize()
            step_ms[v].append(ev0.elapsed_time(ev1))
            if r == 0:
                outs[v] = out.cpu().clone()
            # per-launch events price each kernel alone: the noise branches stay on the caller's stream in this pass
            # (unless the option under test is STTS_OPT_NBRANCH itself)
            if a.opt != E.OPT_NBRANCH:
                E.set_option(E.OPT_NBRANCH, 0)
            E.profile_enable(True)
            eng.forward(asr, f0, n, s, seed=5, out=out)
            torch.cuda.synchronize()
            for rec in E.profile_launches():
                key = (rec["kernel"], rec["N"], rec["taps"], rec["dil"], rec["res_acc"])
                res[v][key].append((rec["ms"], rec["flops"]))
            E.profile_enable(False)
    E.reset_options()
    base = a.values[0]
    summary = {}
    for v in a.values:
        fam = collections.defaultdict(float)
        for key, lst in res[v].items():
            fam[key[0]] += np.median([m for m, _ in lst]) * (len(lst) / a.rounds)
        d = float((outs[v] - outs[base]).abs().max())
        summary[v] = {"step_ms_median": float(np.median(step_ms[v])), "engines_ms": dict(fam),
                      "max_abs_vs_first": d}
        print(f"opt {a.opt}={v}: step {np.median(step_ms[v]):.2f} ms (min {min(step_ms[v]):.2f}); "
              + ", ".join(f"{k} {t:.2f} ms" for k, t in sorted(fam.items())) + f"; max-abs vs {base}: {d:.2e}",
              flush=True)
    keys = sorted({k for v in a.values for k in res[v]}, key=lambda k: (k[0], k[1], k[2], k[3], k[4]))
    print("shape (kernel, N, taps, dil, res|acc<<1): median ms per launch, TF/s")
    for k in keys:
        row = []
        for v in a.values:
            lst = res[v].get(k)
            if lst:
                ms = np.median([m for m, _ in lst])
                row.append(f"{v}: {ms * 1e3:7.1f} us {lst[0][1] / ms / 1e9:6.0f} TF")
        print(f"  {k}: " + " | ".join(row))
    print(json.dumps({"opt": a.opt, "summary": summary}))


if __name__ == "__main__":
    main()
