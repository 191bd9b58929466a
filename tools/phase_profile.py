"""Phase cost of the resblock engines (resconv.hip, bigconv.hip): per-launch times of one decoder forward with
phases skipped through STTS_OPT_DEBUG (1 prologue math, 2 MFMAs, 4 epilogue; bigconv also
8 weight-slice staging, 16 window staging).  Outputs are wrong while a bit is set; only the
timings mean anything.

    python tools/phase_profile.py [modes, e.g. 0,2,8] [bigconv | igemm]

conv1d_igemm (conv1d.hip) bits: 1 window staging, 2 MFMAs, 4 epilogue, 8 window loads.
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "styletts2-lite_amd"))

import torch  # noqa: E402

import bench  # noqa: E402
from stts2_mi355x import engine as E  # noqa: E402
from stts2_mi355x import synth  # noqa: E402


def run(eng, args, dbg):
    E.set_option(E.OPT_DEBUG, dbg)
    for i in range(2):
        eng.forward(*args, seed=i)
    torch.cuda.synchronize()
    E.profile_enable(True)
    eng.forward(*args, seed=7)
    torch.cuda.synchronize()
    recs = E.profile_launches()
    E.profile_enable(False)
    E.set_option(E.OPT_DEBUG, 0)
    return recs


def main():
    dev = torch.device("cuda", 0)
    dec, _ = bench.build_decoder("hifigan")
    dec = dec.to(dev)
    B = int(os.environ.get("PHASE_B", "32"))
    args = tuple(torch.from_numpy(x).to(dev) for x in synth.decoder_inputs(B, 400))
    eng = dec.engine(os.environ.get("PHASE_DT", "bf16"))
    modes = [int(m) for m in sys.argv[1].split(",")] if len(sys.argv) > 1 else [0, 1, 2, 4, 3, 6, 7]
    kernels = ("k_bigconv",) if "bigconv" in sys.argv else ("conv1d_igemm_kernel",) if "igemm" in sys.argv \
        else ("k_resconv", "k_bigconv")
    res = {m: run(eng, args, m) for m in modes}
    print(f"{'i':>3} {'C':>3} {'k':>2} {'d':>1} {'ra':>2} " + " ".join(f"{'dbg' + str(m):>7}" for m in modes))
    tot = {m: 0.0 for m in modes}
    for i, r in enumerate(res[0]):
        if r["kernel"] not in kernels:
            continue
        row = [res[m][i]["ms"] * 1e3 for m in modes]
        for m, v in zip(modes, row):
            tot[m] += v
        print(f"{i:3d} {r['N']:3d} {r['taps']:2d} {r['dil']:1d} {r['res_acc']:2d} " + " ".join(f"{v:7.1f}" for v in row))
    print("total   " + " ".join(f"{tot[m]:7.0f}" for m in modes))


if __name__ == "__main__":
    main()
