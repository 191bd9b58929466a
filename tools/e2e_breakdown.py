#!/usr/bin/env python3
"""Stage times of one 10-s utterance through Synthesizer (tokens -> waveform), B = 1, cuda events."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "styletts2-lite_amd"), os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)
import torch  # noqa: E402

from helpers import make_decoder, make_duration_modules  # noqa: E402
from stts2_mi355x import synth  # noqa: E402
from stts2_mi355x.prosody import durations, expand_frames, linear_frames  # noqa: E402

te, pp = (m.cuda() for m in make_duration_modules())
dec, _ = make_decoder("hifigan")
dec = dec.cuda()
ids = [0] + [int(v) for v in (synth.hash_u01("bench:e2e:tok", 14) * 177 + 1)] + [0]
tok = torch.tensor(ids, device="cuda").unsqueeze(0)
s = torch.from_numpy(synth.normal("bench:dur:s", (1, 128))).cuda()
z = torch.zeros(1, len(ids), device="cuda")


def run(rec, dt):
    ev = [torch.cuda.Event(enable_timing=True)]
    ev[0].record()

    def mark(name):
        e = torch.cuda.Event(enable_timing=True)
        e.record()
        ev.append(e)
        rec.append(name)
    with torch.no_grad():
        t_en = te(tok, None); mark("text_encoder")
        d = pp.text_encoder(t_en, s, None); mark("duration_encoder")
        x, _ = pp.lstm(d); mark("duration_lstm")
        lin = pp.duration_proj.linear_layer
        _, pred, total, _ = durations(linear_frames(x, lin.weight, lin.bias), None, z, mix=0.1); mark("durations")
        F = int(total[0].item()); mark("host_read")
        en = expand_frames(d, pred, F); asr = expand_frames(t_en.transpose(1, 2), pred, F); mark("expand")
        F0, N = pp.F0Ntrain(en, s); mark("f0ntrain")
        dec(asr, F0, N, s, dtype=dt); mark("decoder_" + dt)
    torch.cuda.synchronize()
    return [ev[i].elapsed_time(ev[i + 1]) for i in range(len(ev) - 1)]


for dt in ("bf16", "fp32"):
    for _ in range(2):
        run([], dt)
    names = []
    ms = run(names, dt)
    print(dt, " ".join(f"{n} {m:.2f}" for n, m in zip(names, ms)), f"total {sum(ms):.2f} ms", flush=True)
