"""Per-shape attribution of the config-5 training step's conv C-ABI calls (diagnostics): every
stts_conv1d_fwd / _fwd_res / _fwd_act / _bwd and stts_conv_transpose1d_fwd / _bwd call of one bf16 step is
bracketed by hipEvents (the call includes its frame conversions and weight pack), then summed by
(call, dx/dw, B, Lin, Cin, Cout, K, stride, dil).

    python tools/train_conv_shapes.py [--dtype bf16] [--top 30]
"""
import argparse
import collections
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "styletts2-lite_amd"), os.path.join(ROOT, "tests"), os.path.join(ROOT, "tools")]
import torch  # noqa: E402

NAMES = ["stts_conv1d_fwd", "stts_conv1d_fwd_res", "stts_conv1d_fwd_act", "stts_conv1d_bwd",
         "stts_conv_transpose1d_fwd", "stts_conv_transpose1d_bwd",
         # the MSD's time-expanded convs: (S, H, W, C, Cout, K, stride, pad, Lq)
         "stts_conv1d_fwd_tx", "stts_conv1d_bwd_tx", "stts_conv1d_wgrad_tx"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dtype", default="bf16")
    ap.add_argument("--top", type=int, default=30)
    a = ap.parse_args()
    from bench_train_step import build
    from stts2_mi355x import discriminators, training
    from stts2_mi355x import engine as E
    from stts2_mi355x.trainstep import TrainStep
    # one stream, so that each call's events bracket its own work only
    discriminators.CONCURRENT = False
    training.CONCURRENT_BRANCHES = False
    torch.cuda.set_device(0)
    dec, mpd, msd, (asr, f0, n, s, wav) = build(2, 155)
    dec, mpd, msd = dec.cuda().eval(), mpd.cuda().train(), msd.cuda().train()
    ins = [t.cuda().requires_grad_(True) for t in (asr, f0, n, s)]
    wav = wav.cuda()
    step = TrainStep(dec, mpd, msd, dtype=a.dtype)
    step(*ins, wav, seed=1)
    torch.cuda.synchronize()
    L = E.lib()
    recs = []
    orig = {nm: getattr(L, nm) for nm in NAMES}

    def wrap(nm, fn):
        def call(*args):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            rc = fn(*args)
            e1.record()
            ints = [x for x in args[1:] if isinstance(x, int)]
            part = ""
            if nm.endswith("_bwd"):
                ptrs = [x for x in args if not isinstance(x, (int, float))]
                part = "dx" if getattr(ptrs[-5], "value", ptrs[-5]) else ""
                part += "+dw" if getattr(ptrs[-4], "value", ptrs[-4]) else ""
            recs.append((nm, part, tuple(ints[:9]), e0, e1))
            return rc
        return call

    for nm in NAMES:
        setattr(L, nm, wrap(nm, orig[nm]))
    step(*ins, wav, seed=2)
    torch.cuda.synchronize()
    for nm in NAMES:
        setattr(L, nm, orig[nm])
    agg = collections.defaultdict(lambda: [0, 0.0])
    for nm, part, shp, e0, e1 in recs:
        k = (nm.replace("stts_", ""), part, shp)
        agg[k][0] += 1
        agg[k][1] += e0.elapsed_time(e1)
    tot = sum(v[1] for v in agg.values())
    print(f"{len(recs)} conv calls, {tot:.2f} ms inside them (one {a.dtype} step)")
    for k, (c, ms) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:a.top]:
        print(f"{ms:7.2f} ms {c:4d} x  {k[0]:24s} {k[1]:6s} (B, Lin, Cin, Cout, K, stride, dil, pad, Lq) = {k[2]}")


if __name__ == "__main__":
    main()
