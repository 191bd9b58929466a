"""A/B of the MultiResSpecDiscriminator engine forward with its stride-2 layers folded (STTS_OPT_MSDFOLD = 1:
stride-1 convs over phase-folded frames, weights folded at pack time) and unfolded (0), at config 5's shape
(real + generated audio, B = 2 x 93,000 samples each): forward + GAN losses time and the largest difference
of the feature maps / scores between the two.  One process, interleaved rounds.

    python tools/ab_msd_fold.py [--iters 10] [--rounds 3]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "styletts2-lite_amd"), os.path.join(ROOT, "tests")]
import torch  # noqa: E402


def timed(fn, iters):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=3)
    a = ap.parse_args()
    from stts2_mi355x import engine as E
    from stts2_mi355x.discriminators import msd_gan_losses
    from test_msd_oracle import msd_module
    torch.cuda.set_device(0)
    gen = torch.Generator().manual_seed(0)
    wav = (torch.randn(2, 1, 93000, generator=gen) * 0.2).cuda()
    yh = (torch.randn(2, 1, 93000, generator=gen) * 0.2).cuda()
    # one module per (fold, dtype): the engine model is created (and the option read) at its first forward
    mods, outs = {}, {}
    with torch.no_grad():
        for v in (0, 1):
            E.set_option(E.OPT_MSDFOLD, v)
            for dt in ("bf16", "fp32"):
                mods[(v, dt)] = msd_module()[0].cuda()
                outs[(v, dt)] = mods[(v, dt)](wav, yh, dtype=dt)
        E.reset_options()
        torch.cuda.synchronize()
        diff = {}
        for dt in ("bf16", "fp32"):
            d = 0.0
            for x0, x1 in zip(torch.utils._pytree.tree_leaves(outs[(0, dt)]), torch.utils._pytree.tree_leaves(outs[(1, dt)])):
                scale = max(1.0, float(x0.abs().max()))
                d = max(d, float((x0 - x1).abs().max()) / scale)
            diff[dt] = d
        res = {}
        for _ in range(a.rounds):
            for v in (0, 1):
                for dt in ("bf16", "fp32"):
                    ms = timed(lambda: msd_gan_losses(mods[(v, dt)], wav, yh, dtype=dt), a.iters)
                    res.setdefault((v, dt), []).append(ms)
    line = {"workload": "MSD forward + GAN losses, real + generated, B = 2 x 93,000 samples",
            "max_rel_diff_fold_vs_strided": diff}
    for (v, dt), lst in sorted(res.items()):
        line[f"fold{v}_{dt}_ms"] = round(min(lst), 3)
    print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
