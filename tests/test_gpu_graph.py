"""GPU: hipGraph replay of a decoder forward (stts2_mi355x.graph.CapturedDecoder) against the
eager forward through the C-ABI, and its per-call noise semantics."""
import pytest
import torch

from helpers import decoder_case, make_decoder

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
@pytest.mark.parametrize("B,T", [(1, 40), (2, 16)])
def test_graph_replay_matches_eager(dtype, B, T):
    from stts2_mi355x.graph import CapturedDecoder
    d, _ = make_decoder("hifigan")
    d = d.cuda()
    asr, f0, n, s, nz = (t.cuda() for t in decoder_case(B, T))
    with torch.no_grad():
        ref = d.engine(dtype).forward(asr, f0, n, s, noise=nz).clone()
        run = CapturedDecoder(d, B, T, dtype=dtype)
        out = run(asr, f0, n, s, noise=nz).clone()
        out2 = run(asr, f0, n, s, noise=nz).clone()  # a second replay
    torch.cuda.synchronize()
    assert (out - ref).abs().max().item() < 1e-5  # fp64 statistics atomics may reorder
    assert (out2 - ref).abs().max().item() < 1e-5


def test_graph_noise_follows_torch_rng_and_stale_weights_refuse():
    from stts2_mi355x.graph import CapturedDecoder
    d, _ = make_decoder("hifigan")
    d = d.cuda()
    asr, f0, n, s, _ = (t.cuda() for t in decoder_case(1, 16))
    with torch.no_grad():
        run = CapturedDecoder(d, 1, 16, dtype="bf16")
        torch.manual_seed(7)
        a = run(asr, f0, n, s).clone()
        b = run(asr, f0, n, s).clone()
        torch.manual_seed(7)
        c = run(asr, f0, n, s).clone()
        assert (a - b).abs().max().item() > 1e-4  # fresh noise per call
        assert (a - c).abs().max().item() < 1e-5  # manual_seed reproduces
        d.generator.conv_post.bias.add_(0.1)
        with pytest.raises(RuntimeError, match="weights changed"):
            run(asr, f0, n, s)
