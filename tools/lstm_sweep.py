#!/usr/bin/env python3
"""A/B sweep of the BiLSTM recurrence grouping (stts_set_lstm_group) over batch sizes: us per step."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "styletts2-lite_amd"))
import torch  # noqa: E402

from stts2_mi355x.prosody import LSTM, set_lstm_group  # noqa: E402

torch.manual_seed(0)
lstm = LSTM(640, 256, 1, batch_first=True, bidirectional=True).cuda()
T = 400
for B in (1, 4, 8, 16, 32, 64):
    x = torch.randn(B, T, 640, device="cuda")
    row = []
    for bg in (-1, 1, 2, 4):
        set_lstm_group(bg)
        for _ in range(2):
            lstm(x)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(5):
            lstm(x)
        e1.record()
        torch.cuda.synchronize()
        row.append(e0.elapsed_time(e1) / 5 * 1e3 / T)
    print(f"B={B:3d} T={T}: us/step (incl. input projection) coop {row[0]:.2f}  bg1 {row[1]:.2f}  bg2 {row[2]:.2f}  bg4 {row[3]:.2f}",
          flush=True)
set_lstm_group(0)
