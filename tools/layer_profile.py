"""Per-launch roofline table of one decoder forward (conv1d_igemm launches, hipEvent-timed).

    python tools/layer_profile.py [--decoder hifigan] [--dtype bf16] [--batch 32] [--frames 400]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "styletts2-lite_amd"))

import torch  # noqa: E402

import bench  # noqa: E402
from stts2_mi355x import engine as E  # noqa: E402
from stts2_mi355x import synth  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--decoder", default="hifigan")
    ap.add_argument("--dtype", default="bf16")
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--frames", type=int, default=400)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    dec, _ = bench.build_decoder(a.decoder)
    dec = dec.to(dev)
    asr, f0, n, s = (torch.from_numpy(x).to(dev) for x in synth.decoder_inputs(a.batch, a.frames))
    eng = dec.engine(a.dtype)
    out = torch.empty(a.batch, 1, 600 * a.frames, device=dev)
    for i in range(2):
        eng.forward(asr, f0, n, s, seed=i, out=out)
    torch.cuda.synchronize()
    E.profile_enable(True)
    eng.forward(asr, f0, n, s, seed=7, out=out)
    torch.cuda.synchronize()
    recs = E.profile_launches()
    E.profile_enable(False)
    pf, pb = bench.PEAK_MFMA[a.dtype], bench.PEAK_HBM
    print(f"{'i':>3} {'rows':>8} {'N':>5} {'Cin':>5} {'k':>3} {'d':>2} {'ra':>2} {'us':>8} {'TF/s':>7} {'GB/s':>7} "
          f"{'bound':>5} {'frac':>5} {'floor_us':>8} kernel")
    tot, tot_floor = 0.0, 0.0
    for i, r in enumerate(recs):
        t = r["ms"] / 1e3
        tf, gb = r["flops"] / t / 1e12, r["bytes"] / t / 1e9
        t_m, t_h = r["flops"] / pf, r["bytes"] / pb
        bound = "mfma" if t_m >= t_h else "hbm"
        floor = max(t_m, t_h)
        tot += t
        tot_floor += floor
        print(f"{i:3d} {r['B'] * r['rows']:8d} {r['N']:5d} {r['Cin']:5d} {r['taps']:3d} {r['dil']:2d} {r['res_acc']:2d} "
              f"{t * 1e6:8.1f} {tf:7.1f} {gb:7.0f} {bound:>5} {floor / t:5.2f} {floor * 1e6:8.1f} {r['kernel']}")
    print(f"total {tot * 1e3:.3f} ms over {len(recs)} launches; roofline floor {tot_floor * 1e3:.3f} ms "
          f"({tot_floor / tot:.3f})")


if __name__ == "__main__":
    main()
