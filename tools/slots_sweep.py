#!/usr/bin/env python3
"""A/B: conv-statistics slot spreading (STTS_OPT_STATS_SLOTS) vs batch size, HiFi-GAN bf16, 10-s utterances."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "styletts2-lite_amd"))
import torch  # noqa: E402

import bench  # noqa: E402
from stts2_mi355x import engine as E  # noqa: E402
from stts2_mi355x import synth  # noqa: E402

dec, _ = bench.build_decoder("hifigan")
dec = dec.cuda()
eng = dec.engine("bf16")
for B in [int(b) for b in (sys.argv[1] if len(sys.argv) > 1 else "1,2,4,8,16,32").split(",")]:
    args = tuple(torch.from_numpy(x).cuda() for x in synth.decoder_inputs(B, 400))
    row = []
    for slots in (1, 4, 16, 64):
        E.set_option(5, slots)
        for i in range(2):
            eng.forward(*args, seed=i)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for i in range(3):
            eng.forward(*args, seed=i)
        e1.record()
        torch.cuda.synchronize()
        row.append(e0.elapsed_time(e1) / 3)
    E.set_option(5, 0)
    print(f"B={B:3d}: ms per forward  slots1 {row[0]:.2f}  slots4 {row[1]:.2f}  slots16 {row[2]:.2f}  slots64 {row[3]:.2f}",
          flush=True)
