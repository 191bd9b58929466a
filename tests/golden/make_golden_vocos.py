"""Golden fixtures for the Vocos decoder, made by running the REFERENCE
module in the survey container (never on the GPU box):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_vocos.py

Imports /root/reference/Modules/vocos.py read-only (torch, numpy and scipy only), builds
`Decoder(dim_in=512, style_dim=128, intermediate_dim=1536, num_layers=8, gen_istft_n_fft,
gen_istft_hop_size)` as inference.py:112-118 does, fills every parameter from the formula in
stts2_mi355x/synth.py by state-dict key (the `parametrizations.weight.original0/1` weight-norm
keys included), runs forward(asr, F0_curve, N, s) in eval mode on formula inputs and stores the
waveform and two taps as .npz DATA (tests/golden/vocos_*.npz).

Cases: the commented config_example.yaml vocos block (n_fft 1200, hop 300: 600 samples per asr
frame, like the other decoders) and the module defaults (n_fft 1024, hop 256).
"""
from __future__ import annotations

import json
import os
import sys
import warnings

import numpy as np
import torch

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "styletts2-lite_amd"))
sys.path.insert(0, REF)
warnings.filterwarnings("ignore")

from stts2_mi355x import synth  # noqa: E402

CASES = (  # (n_fft, hop, T, B)
    (1200, 300, 4, 2),
    (1200, 300, 40, 1),
    (1200, 300, 400, 1),
    (1024, 256, 16, 1),
)


def fill(module):
    sd = module.state_dict()
    new = {}
    for k, v in sd.items():
        new[k] = v if synth.is_fixed_buffer(k) else torch.from_numpy(synth.synth_param(k, tuple(v.shape)))
    module.load_state_dict(new, strict=True)
    return module


def run(n_fft, hop, T, B):
    from Modules.vocos import Decoder
    torch.manual_seed(0)
    dec = Decoder(dim_in=512, style_dim=128, dim_out=80, intermediate_dim=1536, num_layers=8,
                  gen_istft_n_fft=n_fft, gen_istft_hop_size=hop)
    dec = fill(dec).eval()
    asr, f0, n, s = synth.decoder_inputs(B, T, tag="vocos")
    taps = {}
    hooks = [dec.decode[3].register_forward_hook(lambda m, i, o: taps.__setitem__("frontend", o.detach())),
             dec.generator.final_layer_norm.register_forward_hook(lambda m, i, o: taps.__setitem__("ln", o.detach()))]
    with torch.no_grad():
        out = dec(torch.from_numpy(asr), torch.from_numpy(f0), torch.from_numpy(n), torch.from_numpy(s))
    for h in hooks:
        h.remove()
    res = {"out": out.numpy().astype(np.float32)}
    if T <= 40:
        for k, v in taps.items():
            res["tap_" + k] = v.numpy().astype(np.float32)
    return res


def main():
    torch.set_num_threads(8)
    mpath = os.path.join(HERE, "meta.json")
    meta = json.load(open(mpath))
    for n_fft, hop, T, B in CASES:
        r = run(n_fft, hop, T, B)
        name = f"vocos_n{n_fft}_T{T}_B{B}"
        np.savez_compressed(os.path.join(HERE, name + ".npz"), **r)
        meta["cases"][name] = {"kind": "vocos", "n_fft": n_fft, "hop": hop, "T": T, "B": B, "keys": sorted(r.keys()),
                               "generator": "tests/golden/make_golden_vocos.py",
                               "out_absmax": float(np.abs(r["out"]).max()), "out_std": float(r["out"].std())}
        print(name, {k: v.shape for k, v in r.items()}, meta["cases"][name]["out_std"],
              meta["cases"][name]["out_absmax"], flush=True)
    from Modules.vocos import Decoder
    ref = Decoder(dim_in=512, style_dim=128, dim_out=80, intermediate_dim=1536, num_layers=8,
                  gen_istft_n_fft=1200, gen_istft_hop_size=300)
    meta["vocos_state_dict"] = {k: list(v.shape) for k, v in ref.state_dict().items()}  # the drop-in's key contract
    with open(mpath, "w") as f:
        json.dump(meta, f, indent=1)


if __name__ == "__main__":
    main()
