"""Phase attribution of the bigconv2 engine on the headline workload (HiFi-GAN bf16, B x 10 s):
one decoder forward with STTS_OPT_DEBUG bit 64 and a debug buffer; the per-wave s_memtime phase
sums are aggregated over every bigconv2 launch of that forward.  Diagnostics only.

    python tools/stamps_decoder.py [--batch 32] [--frames 400]
"""
import argparse
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "styletts2-lite_amd")]
import torch  # noqa: E402

import bench  # noqa: E402

NAMES = ["w_wait", "x_wait", "barrier", "transform", "ep_tail", "total", "rest", "ep_vmwait", "ep_finish", "ep_stats"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--frames", type=int, default=400)
    ap.add_argument("--skips", default="0", help="comma list of extra STTS_OPT_DEBUG phase-skip masks")
    ap.add_argument("--set", action="append", default=[], help="KEY=VALUE options held for the run, e.g. 7=1 "
                    "(resblocks on bigconv v1: the stamps then come from the front-end launches only)")
    a = ap.parse_args()
    ref = None
    for skip in (int(x) for x in a.skips.split(",")):
        out = run(a, skip)
        if ref is None:
            ref = out
        else:  # bits 512 / 1024 change the store path only: the audio must not change
            print(f"  max-abs vs first: {(out - ref).abs().max().item():.3e}")


def run(a, skip):
    from stts2_mi355x import engine as E
    from stts2_mi355x import synth
    torch.cuda.set_device(0)
    for kv in a.set:
        k, v = (int(x) for x in kv.split("="))
        E.set_option(k, v)
    dec, _ = bench.build_decoder("hifigan")
    eng = dec.cuda().engine("bf16")
    asr, f0, n, s = (torch.from_numpy(x).cuda() for x in synth.decoder_inputs(a.batch, a.frames))
    out = torch.empty(a.batch, 1, 600 * a.frames, device="cuda")
    eng.forward(asr, f0, n, s, seed=5, out=out)
    torch.cuda.synchronize()
    stamps = torch.zeros(16, dtype=torch.int64, device="cuda")
    E.check(E.lib().stts_set_debug_buffer(ctypes.c_void_p(stamps.data_ptr())))
    try:
        E.set_option(E.OPT_DEBUG, 64 | skip)
        eng.forward(asr, f0, n, s, seed=5, out=out)
        torch.cuda.synchronize()
    finally:
        E.set_option(E.OPT_DEBUG, 0)
        E.check(E.lib().stts_set_debug_buffer(ctypes.c_void_p(0)))
    v = stamps.cpu().tolist()
    tot = v[5] or 1
    print(f"[skip {skip}] bigconv2 over one B={a.batch} x {a.frames * 600 // 24000}-s forward: {v[15]} workgroups, "
          f"{v[5] / max(v[15] * 8, 1):.0f} cycles per wave-launch")
    for i, nm in enumerate(NAMES):
        if i != 5:
            print(f"  {nm:10s} {100 * v[i] / tot:5.1f} %")
    return out.cpu()


if __name__ == "__main__":
    main()
