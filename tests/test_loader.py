"""CPU: the drop-in model builder and checkpoint loader (inference.py:70-174) on a synthetic
checkpoint in the reference's format ({'net': {key: state_dict}}, 'module.'-prefixed keys)."""
import torch

from stts2_mi355x.inference import build_models, load_models, symbol_table

# the model_params / symbol layout of the reference's Configs/config*.yaml (values restated here;
# the GPU box has no reference tree)
CONFIG = {
    "symbol": {"pad": "$", "punctuation": ";:,.!?", "letters": "abcdefghijklmnopqrstuvwxyz",
               "letters_ipa": "ɑɐɒæβɔɕç", "extend": ""},
    "model_params": {"dim_in": 64, "hidden_dim": 512, "max_conv_dim": 512, "n_layer": 3, "n_mels": 80,
                     "max_dur": 50, "style_dim": 128, "dropout": 0.2,
                     "decoder": {"type": "hifigan", "resblock_kernel_sizes": [3, 7, 11],
                                 "upsample_rates": [10, 5, 3, 2], "upsample_initial_channel": 512,
                                 "resblock_dilation_sizes": [[1, 3, 5], [1, 3, 5], [1, 3, 5]],
                                 "upsample_kernel_sizes": [20, 10, 6, 4]}},
}


def test_symbol_table():
    table, n_token = symbol_table(CONFIG)
    assert table["$"] == 0 and n_token == len(table) + 1


def test_build_and_load(tmp_path):
    model = build_models(CONFIG)
    assert set(model) == {"decoder", "predictor", "text_encoder", "style_encoder"}
    torch.manual_seed(0)
    net = {}
    for k, m in model.items():
        sd = {n: torch.randn_like(v) for n, v in m.state_dict().items()}
        # the reference's DataParallel checkpoints: 'module.'-prefixed keys for two of them
        net[k] = {("module." + n if k in ("decoder", "predictor") else n): v for n, v in sd.items()}
    path = tmp_path / "ckpt.pth"
    torch.save({"net": net, "epoch": 3}, path)
    fresh = build_models(CONFIG)
    counts = load_models(fresh, str(path))
    for k, m in fresh.items():
        for n, v in m.state_dict().items():
            src = net[k].get(n, net[k].get("module." + n))
            assert torch.equal(v, src), (k, n)
        assert counts[k] == sum(p.numel() for p in m.parameters())
