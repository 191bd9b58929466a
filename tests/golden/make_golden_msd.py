"""Golden fixtures for the MultiResSpecDiscriminator forward and its GAN losses (training step, SURVEY
§8(f) rank 3), made by running the REFERENCE module in the survey container (never on the GPU box):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_msd.py

Imports /root/reference/Modules/discriminators.py read-only and fills its parameters from the formula
in stts2_mi355x/synth.py ("msd." + key).  SpecDiscriminator.forward moves its window with
`self.window.to(y.get_device())` (discriminators.py:55), which only works for CUDA tensors (CPU tensors
report device -1: the "MSD crashes on CPU" of SURVEY §8(c)); during the forward this script makes
Tensor.get_device return "cpu", which changes nothing else.  losses.py needs the torchaudio stub of
make_golden_mpd.py.  Stored: inputs, scores of every resolution, the last two feature maps of every
resolution (the first ones are megabytes) and the reference's three GAN losses, as .npz DATA.
"""
from __future__ import annotations

import os
import sys
import warnings

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from make_golden_mpd import REF, import_losses, synth, waves  # noqa: E402

sys.path.insert(0, REF)
warnings.filterwarnings("ignore")


def main():
    from Modules.discriminators import MultiResSpecDiscriminator
    torch.manual_seed(0)
    msd = MultiResSpecDiscriminator().eval()
    sd = {k: torch.from_numpy(synth.synth_param("msd." + k, tuple(v.shape))) for k, v in msd.state_dict().items()}
    msd.load_state_dict(sd, strict=True)
    L = import_losses()
    get_device = torch.Tensor.get_device
    for B, T in ((1, 2400), (2, 1801)):
        y, yh = waves(B, T, 2), waves(B, T, 3)
        torch.Tensor.get_device = lambda self: "cpu"
        try:
            with torch.no_grad():
                y_d_rs, y_d_gs, fmap_rs, fmap_gs = msd(torch.from_numpy(y), torch.from_numpy(yh))
        finally:
            torch.Tensor.get_device = get_device
        rec = {"y": y, "y_hat": yh,
               "loss_fm": np.float64(L.feature_loss(fmap_rs, fmap_gs).item()),
               "loss_gen": np.float64(L.generator_loss(y_d_gs)[0].item()),
               "loss_disc": np.float64(L.discriminator_loss(y_d_rs, y_d_gs)[0].item())}
        for i in range(len(y_d_rs)):
            rec[f"score_r{i}"] = y_d_rs[i].numpy()
            rec[f"score_g{i}"] = y_d_gs[i].numpy()
            for j in (4, 5):
                rec[f"fmap_r{i}_{j}"] = fmap_rs[i][j].numpy()
                rec[f"fmap_g{i}_{j}"] = fmap_gs[i][j].numpy()
            rec[f"shape_fmap0_{i}"] = np.array(fmap_rs[i][0].shape)
        path = os.path.join(HERE, f"msd_B{B}_T{T}.npz")
        np.savez_compressed(path, **rec)
        print(path, os.path.getsize(path), [y_d_rs[i].shape for i in range(3)])


if __name__ == "__main__":
    main()
