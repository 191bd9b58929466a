"""CPU: the oracle's training step (oracle.train_step: decoder forward, DiscriminatorLoss backward + AdamW on
the MPD / MSD, mel + generator loss backward + AdamW on the decoder; train.py:267-327) reproduces the
reference modules' own autograd and torch's AdamW (tests/golden/train_step_B2_T8.npz, made by
tests/golden/make_golden_train.py) - which makes it the checker of the HIP step (test_gpu_train_step.py)."""
import numpy as np
import torch

from helpers import HIFI_CFG, fill_module, golden, make_decoder
from oracle import stts_oracle as orc
from stts2_mi355x import synth


def test_oracle_train_step_matches_reference():
    from stts2_mi355x.synth import waves
    from stts2_mi355x.discriminators import MultiPeriodDiscriminator, MultiResSpecDiscriminator
    fx = golden("train_step_B2_T8")
    B, T = int(fx["B"]), int(fx["T"])
    dec, _ = make_decoder("hifigan")
    mpd = fill_module(MultiPeriodDiscriminator(), "mpd.")
    msd = fill_module(MultiResSpecDiscriminator(), "msd.")
    sd = lambda m: {k: v.detach().clone() for k, v in m.state_dict().items()}  # noqa: E731
    p0 = sd(dec)
    asr, f0, n, s = (torch.from_numpy(a) for a in synth.decoder_inputs(B, T, tag="train"))
    L = 600 * T
    wav = torch.from_numpy(waves(B, L, 7))
    noise = torch.from_numpy(synth.source_noise(B, L, tag="train_noise"))
    y, losses, grads, params = orc.train_step(sd(dec), sd(mpd), sd(msd), HIFI_CFG, asr, f0, n, s, wav, noise)
    assert np.array_equal(y.numpy(), fx["y_rec"])
    for k in ("d_loss", "loss_mel", "loss_gen_all", "g_loss"):
        assert losses[k] == float(fx[k]), k
    for tag, key in (("dec", "grad.dec"), ("mpd", "grad.mpd"), ("msd", "grad.msd")):
        for i, k in enumerate(str(v) for v in fx[key + ".names"]):
            g = grads[tag][k].reshape(-1).double().numpy()
            assert np.array_equal(g[fx[key + ".idx"][i]], fx[key + ".val"][i]), k
            assert abs(np.sqrt((g * g).sum()) - fx[key + ".l2"][i]) <= 1e-12 * fx[key + ".l2"][i], k
    for k in ("asr", "F0_curve", "N", "s"):
        assert np.array_equal(grads["inputs"][k].numpy(), fx["grad_in." + k]), k
    for i, k in enumerate(str(v) for v in fx["grad.dec.names"]):
        d = (params["dec"][k].double() - p0[k].double()).reshape(-1).numpy()[fx["grad.dec.idx"][i]]
        assert np.array_equal(d, fx["grad.dec.delta"][i]), k
