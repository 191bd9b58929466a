"""Golden fixture pinning the T = 2 conditioning argument of tests/test_gpu_edge.py, made by running the
REFERENCE decoders in the survey container (never on the GPU box):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_edge.py

At T = 2 every InstanceNorm averages two frames; near-equal pairs make the forward ill-conditioned. For
both decoders at (B = 3, T = 2, utterances 5..7 of synth.decoder_case) this stores the reference's fp32
output, the spread of the reference's output under a 1e-6 relative weight perturbation, and its
distance to a float64 run of the same module: the scale against which a GPU result at T = 2 is judged.
"""
from __future__ import annotations

import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from make_golden import HIFI_CFG, ISTFT_CFG, NoisePatch, fill, synth  # noqa: E402


def run(kind):
    if kind == "hifigan":
        from Modules.hifigan import Decoder
        dec = Decoder(dim_in=512, style_dim=128, dim_out=80, **HIFI_CFG)
    else:
        from Modules.istftnet import Decoder
        dec = Decoder(dim_in=512, style_dim=128, dim_out=80, **ISTFT_CFG)
    dec = fill(dec).eval()
    B, T, utt0 = 3, 2, 5
    asr, f0, n, s = synth.decoder_inputs(B, T, utt0=utt0)
    noise = synth.source_noise(B, 600 * T, utt0=utt0)
    args = [torch.from_numpy(a) for a in (asr, f0, n, s)]
    with torch.no_grad(), NoisePatch(noise):
        out = dec(*args).numpy()
    sd = {k: v.clone() for k, v in dec.state_dict().items()}
    pert = {k: (v * (1 + 1e-6 * torch.from_numpy(synth.uniform("edge-pert:" + k, tuple(v.shape))))
                if v.is_floating_point() and not synth.is_fixed_buffer(k) else v) for k, v in sd.items()}
    dec.load_state_dict(pert)
    with torch.no_grad(), NoisePatch(noise):
        out_p = dec(*args).numpy()
    dec.load_state_dict(sd)
    dec = dec.double()
    with torch.no_grad(), NoisePatch(noise.astype(np.float64)):
        out_64 = dec(*[a.double() for a in args]).numpy()
    return {"out": out.astype(np.float32), "spread_perturbed": np.float64(np.abs(out_p - out).max()),
            "spread_fp64": np.float64(np.abs(out_64 - out).max())}


def main():
    torch.set_num_threads(8)
    for kind in ("hifigan", "istftnet"):
        r = run(kind)
        np.savez_compressed(os.path.join(HERE, f"{kind}_T2_B3_edge.npz"), **r)
        print(kind, float(r["spread_perturbed"]), float(r["spread_fp64"]), flush=True)


if __name__ == "__main__":
    main()
