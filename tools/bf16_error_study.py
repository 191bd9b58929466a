"""Where does the bf16 decoder's error come from?  CPU emulation on the oracle (HiFi-GAN, formula
weights): every conv of the selected stages rounds its (post-prologue) input and its weights to
bf16 (the MFMA operands) and its output to bf16 (the stored activation), accumulating in fp32, as
the HIP bf16 path does.  Prints the waveform max-abs / rms error vs the fp32 oracle for each stage
alone and for all stages.  (Test infrastructure only: the oracle is the checker, nothing here ships.)

    python tools/bf16_error_study.py [T] [bf16|fp16] [all]

(`all`: only the whole-decoder case, for long T.)

With fp16 the operands and the stored activations round to IEEE half (10-bit mantissa, 8x finer than
bf16's 7 bits, range +-65504): the candidate accuracy mode of gfx950's f16 MFMA, which runs at the bf16
rate with the same bytes.  The largest |value| rounded is printed (fp16 overflows above 65504).
"""
import os
import sys

import numpy as np
import torch
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "styletts2-lite_amd"), os.path.join(ROOT, "tests")]
from helpers import decoder_case, make_decoder  # noqa: E402
from oracle import stts_oracle as orc  # noqa: E402

_conv1d, _convT = F.conv1d, F.conv_transpose1d
SEL = set()


def stage(cin, cout):
    if cout == 1 and cin == 32:
        return "post"
    if cin == 1:
        return "noise"
    c = min(cin, cout) if cin != 512 or cout != 256 else 256
    return {256: "s0", 128: "s1", 64: "s2", 32: "s3"}.get(c, "front")


MODE = {"dt": torch.bfloat16, "amax": 0.0}


def bf(x):
    MODE["amax"] = max(MODE["amax"], float(x.abs().max()))
    return x.to(MODE["dt"]).to(torch.float32)


def conv1d(x, w, b=None, *a, **k):
    st = stage(x.shape[1], w.shape[0])
    if st in SEL:
        return bf(_conv1d(bf(x), bf(w), b, *a, **k))
    return _conv1d(x, w, b, *a, **k)


def convT(x, w, b=None, *a, **k):
    st = stage(x.shape[1], w.shape[1])
    if st in SEL:
        return bf(_convT(bf(x), bf(w), b, *a, **k))
    return _convT(x, w, b, *a, **k)


def main():
    T = int(sys.argv[1]) if len(sys.argv) > 1 else 40
    name = sys.argv[2] if len(sys.argv) > 2 else "bf16"
    MODE["dt"] = {"bf16": torch.bfloat16, "fp16": torch.float16}[name]
    torch.set_num_threads(os.cpu_count())
    dec, cfg = make_decoder("hifigan")
    sd = {k: v for k, v in dec.state_dict().items()}
    asr, f0, n, s, noise = decoder_case(1, T)
    F.conv1d, F.conv_transpose1d = conv1d, convT
    with torch.no_grad():
        ref = orc.decoder_hifigan(asr, f0, n, s, sd, cfg, noise).numpy()
        cases = (["front"], ["s0"], ["s1"], ["s2"], ["s3"], ["post"], ["s2", "s3", "post"],
                 ["front", "s0", "s1"], ["front", "s0", "s1", "s2", "s3", "post"])
        if len(sys.argv) > 3 and sys.argv[3] == "all":
            cases = cases[-1:]
        for sel in cases:
            SEL.clear()
            SEL.update(sel)
            out = orc.decoder_hifigan(asr, f0, n, s, sd, cfg, noise).numpy()
            d = out - ref
            print(f"T={T} {name} stages {'+'.join(sel):24s} max-abs {np.abs(d).max():.3e}  rms {np.sqrt((d ** 2).mean()):.3e}"
                  f"  (largest rounded |value| {MODE['amax']:.3g})", flush=True)
            MODE["amax"] = 0.0


if __name__ == "__main__":
    main()
