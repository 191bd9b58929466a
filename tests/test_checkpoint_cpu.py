"""Checkpoint tooling: Demo/del_training.ipynb and Extend/extend.ipynb restated
on state dicts (stts2_mi355x.checkpoint), checked against the notebooks' documented behaviour."""
import pytest
import torch

from stts2_mi355x import checkpoint as ck


def fake_ckpt(n_token=178, prefix=""):
    g = torch.Generator().manual_seed(0)
    r = lambda *s: torch.randn(*s, generator=g)  # noqa: E731
    net = {
        "decoder": {prefix + "generator.conv_post.bias": r(1)},
        "predictor": {prefix + "F0_proj.weight": r(1, 256, 1)},
        "text_encoder": {prefix + "embedding.weight": r(n_token, 512)},
        "style_encoder": {prefix + "unshared.weight": r(128, 512)},
        "text_aligner": {prefix + "ctc_linear.2.linear_layer.weight": r(n_token, 512),
                         prefix + "ctc_linear.2.linear_layer.bias": r(n_token),
                         prefix + "asr_s2s.embedding.weight": r(n_token, 256),
                         prefix + "asr_s2s.project_to_n_symbols.weight": r(n_token, 128),
                         prefix + "asr_s2s.project_to_n_symbols.bias": r(n_token)},
        "pitch_extractor": {prefix + "x.weight": r(2, 2)},
        "mpd": {prefix + "y.weight": r(2)},
        "msd": {prefix + "z.weight": r(2)},
        "wd": {prefix + "w.weight": r(2)},
    }
    return {"net": net, "optimizer": {"state": 1}, "epoch": 7, "iters": 99}


def test_prune_keeps_inference_modules_only():
    p = ck.prune_for_inference(fake_ckpt())
    assert list(p) == ["net"]
    assert sorted(p["net"]) == sorted(ck.INFERENCE_MODULES)


@pytest.mark.parametrize("prefix", ["", "module."])
def test_extend_token_table(prefix):
    src = fake_ckpt(178, prefix)
    out = ck.extend_token_table(src, 200, generator=torch.Generator().manual_seed(1))
    assert sorted(out) == ["epoch", "iters", "net", "optimizer", "val_loss"]
    assert out["optimizer"] is None and out["iters"] == 0 and out["epoch"] == 0
    assert sorted(out["net"]) == sorted(ck.TRAINING_MODULES)  # 'wd' dropped (keys_to_keep)
    for mod, p, has_bias in ck.TOKEN_TABLES:
        old = src["net"][mod][prefix + p + ".weight"]
        new = out["net"][mod][p + ".weight"]  # saved without the DataParallel prefix
        assert new.shape == (200, old.shape[1])
        assert torch.equal(new[:178], old)
        assert 0.005 < new[178:].std().item() < 0.015  # randn * 0.01
        if has_bias:
            b = out["net"][mod][p + ".bias"]
            assert torch.equal(b[:178], src["net"][mod][prefix + p + ".bias"]) and torch.all(b[178:] == 0)


def test_extend_rejects_shrink():
    with pytest.raises(ValueError):
        ck.extend_token_table(fake_ckpt(178), 178)
    with pytest.raises(ValueError):
        ck.extend_token_table(fake_ckpt(178), 190, n_token=190)


def test_roundtrip_through_weights_only_load(tmp_path):
    out = ck.extend_token_table(fake_ckpt(), 180)
    f = tmp_path / "extended.pth"
    torch.save(out, f)
    back = ck.load(str(f))
    assert back["net"]["text_encoder"]["embedding.weight"].shape == (180, 512)
    # the extended TextEncoder table loads into the drop-in module built for 180 symbols
    from stts2_mi355x.models import TextEncoder
    te = TextEncoder(channels=512, kernel_size=5, depth=3, n_symbols=180)
    sd = te.state_dict()
    sd["embedding.weight"] = back["net"]["text_encoder"]["embedding.weight"]
    te.load_state_dict(sd)


def test_extend_fills_missing_modules_from_fresh():
    """extend.ipynb saves all eight modules built from the config: one the checkpoint lacks is saved
    freshly initialised.  `fresh` supplies it; without `fresh` it is left out."""
    src = fake_ckpt()
    del src["net"]["mpd"], src["net"]["msd"]
    assert "mpd" not in ck.extend_token_table(src, 180)["net"]
    fresh = {"mpd": {"module.y.weight": torch.ones(2)}, "msd": {"z.weight": torch.zeros(2)},
             "decoder": {"generator.conv_post.bias": torch.full((1,), 9.0)}}
    out = ck.extend_token_table(src, 180, fresh=fresh)
    assert sorted(out["net"]) == sorted(ck.TRAINING_MODULES)
    assert torch.equal(out["net"]["mpd"]["y.weight"], torch.ones(2))
    # modules the checkpoint has keep the checkpoint's values
    assert torch.equal(out["net"]["decoder"]["generator.conv_post.bias"],
                       src["net"]["decoder"]["generator.conv_post.bias"])
