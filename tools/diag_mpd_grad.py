"""Diagnostic: per-layer gradient of the D loss through one MPD period (HIP vs the oracle in fp64 / fp32)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "styletts2-lite_amd"), os.path.join(ROOT, "tests")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from helpers import fill_module, golden  # noqa: E402
from stts2_mi355x.synth import waves  # noqa: E402
from oracle import stts_oracle as orc  # noqa: E402
from stts2_mi355x import training as T  # noqa: E402
from stts2_mi355x.discriminators import MultiPeriodDiscriminator  # noqa: E402

period, idx = int(sys.argv[1]) if len(sys.argv) > 1 else 5, None
mpd = fill_module(MultiPeriodDiscriminator(), "mpd.")
idx = [d.period for d in mpd.discriminators].index(period)
sd = {k: v.detach().clone() for k, v in mpd.state_dict().items()}
fx = golden("train_step_B2_T8")
y = torch.from_numpy(waves(2, 4800, 7))
yh = torch.from_numpy(fx["y_rec"])
x = torch.cat([y, yh], 0)
d = mpd.discriminators[idx].cuda()
outs = {}
# ours
score, fmap = T.discriminator_p_forward(d, x.cuda(), period)
B4 = x.shape[0]
for j, f in enumerate(fmap):  # the maps are views of the frames tensors [B p, H, C] on the autograd path
    f._base.register_hook(lambda g, j=j, f=f: outs.__setitem__(
        ("ours", j), g.detach().reshape(B4, period, f.shape[2], f.shape[1]).permute(0, 3, 2, 1).cpu().double()))
r, g = score[:2], score[2:]
loss = ((1 - r) ** 2).mean() + (g ** 2).mean()
loss.backward()
gp = {n: p.grad.detach().cpu().double() for n, p in d.named_parameters()}
ref = {}
for dt in (torch.float32, torch.float64):
    lp = {k: v.to(dt).clone().requires_grad_(True) for k, v in sd.items()}
    sc, fm = orc.discriminator_p(x.to(dt), lp, f"discriminators.{idx}", period)
    for j, f in enumerate(fm):
        f.register_hook(lambda gg, j=j, dt=dt: outs.__setitem__((str(dt), j), gg.detach().double()))
    l2 = ((1 - sc[:2]) ** 2).mean() + (sc[2:] ** 2).mean()
    l2.backward()
    ref[dt] = {k[len(f"discriminators.{idx}."):]: v.grad.double() for k, v in lp.items() if k.startswith(f"discriminators.{idx}.")}
for j in range(6):
    a, b, c = outs[("ours", j)], outs[(str(torch.float32), j)], outs[(str(torch.float64), j)]
    s = c.abs().max().item()
    print(f"fmap{j} grad: ours {((a - c).abs().max() / s).item():.2e}  fp32 ref {((b - c).abs().max() / s).item():.2e}  shape {tuple(c.shape)}")
for n in gp:
    a, b, c = gp[n], ref[torch.float32][n], ref[torch.float64][n]
    s = c.abs().max().item()
    print(f"{n:24s} ours {((a - c).abs().max() / s).item():.2e}  fp32 ref {((b - c).abs().max() / s).item():.2e}  max|g| {s:.2e}")
# where does the bias gradient differ: per-row contributions of fmap0's gradient
a, c = outs[("ours", 0)], outs[(str(torch.float64), 0)]
diff = (a - c).abs()
print("fmap0 grad diff: max at", np.unravel_index(int(diff.argmax()), tuple(diff.shape)), "value", diff.max().item(),
      "ref", c.reshape(-1)[int(diff.argmax())].item())
# LeakyReLU kinks: conv outputs whose sign differs from the fp64 forward (their gradient factor is 1 vs 0.1)
with torch.no_grad():
    _, fm_o = T.discriminator_p_forward(d, x.cuda(), period)
    _, fm_64 = orc.discriminator_p(x.double(), {k: v.double() for k, v in sd.items()}, f"discriminators.{idx}", period)
    _, fm_32 = orc.discriminator_p(x.float(), {k: v.float() for k, v in sd.items()}, f"discriminators.{idx}", period)
    for j in range(5):
        a, b, c = fm_o[j].cpu().double(), fm_32[j].double(), fm_64[j]
        print(f"fmap{j}: sign flips vs fp64: ours {int(((a > 0) != (c > 0)).sum())}, fp32 ref {int(((b > 0) != (c > 0)).sum())}"
              f"; forward rel err ours {((a - c).abs().max() / c.abs().max()).item():.1e} ref {((b - c).abs().max() / c.abs().max()).item():.1e}")
