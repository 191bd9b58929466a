"""Host-side checks of the training-step conv ABI (no GPU): workspace queries validate the geometry
(Lq must be the forward's output length; dilated strided convs are refused) and the drop-in module
refuses what the HIP path does not run."""
import pytest
import torch

from stts2_mi355x import engine as E
from stts2_mi355x.training import Conv1d, out_length


def test_workspace_queries_validate_geometry():
    L = E.lib()
    for fn in (L.stts_conv1d_fwd_workspace_bytes, L.stts_conv1d_bwd_workspace_bytes):
        Lq = out_length(300, 7, 1, 9, 3)
        assert fn(0, 2, 300, 64, 64, 7, 1, 3, 9, Lq) > 0
        assert fn(1, 2, 300, 64, 64, 7, 1, 3, 9, Lq) > 0
        assert fn(0, 2, 300, 64, 64, 7, 1, 3, 9, Lq + 1) == -1   # ST_EINVAL
        # STTS_SPLIT (2): fp32 frames, the fp32 workspace
        assert fn(2, 2, 300, 64, 64, 7, 1, 3, 9, Lq) == fn(0, 2, 300, 64, 64, 7, 1, 3, 9, Lq)
        assert fn(3, 2, 300, 64, 64, 7, 1, 3, 9, Lq) == -2       # ST_EDTYPE
    Lq = out_length(100, 3, 2, 2, 2)
    assert L.stts_conv1d_bwd_workspace_bytes(0, 1, 100, 8, 8, 3, 2, 2, 2, Lq) == -1  # stride 2 with dilation 2
    assert L.stts_conv1d_fwd_workspace_bytes(0, 1, 100, 8, 8, 3, 2, 2, 2, Lq) > 0
    # the MSD's time-expanded conv (stts_conv1d_fwd_tx): the conv1d of S H rows over 3 C = 96 channels; C = 32 only
    Lq = out_length(257, 9, 2, 4, 1)
    tx = L.stts_conv1d_fwd_tx_workspace_bytes
    assert tx(1, 2, 37, 257, 32, 32, 9, 2, 4, Lq) == L.stts_conv1d_fwd_workspace_bytes(1, 74, 257, 96, 32, 9, 2, 1, 4, Lq)
    assert tx(1, 2, 37, 257, 16, 32, 9, 2, 4, Lq) == -1
    assert tx(1, 2, 37, 257, 32, 32, 9, 2, 4, Lq + 1) == -1
    assert tx(3, 2, 37, 257, 32, 32, 9, 2, 4, Lq) == -2
    # its input gradient (stts_conv1d_bwd_tx): the dx of the conv 32 -> 96 over S H rows; Cout = 32 only
    txb = L.stts_conv1d_bwd_tx_workspace_bytes
    assert txb(1, 2, 37, 257, 32, 32, 9, 2, 4, Lq) == L.stts_conv1d_bwd_workspace_bytes(1, 74, 257, 32, 96, 9, 2, 1, 4, Lq)
    assert txb(1, 2, 37, 257, 32, 1, 9, 2, 4, Lq) == -1
    # the weight gradient from the image (stts_conv1d_wgrad_tx): bf16 only, arguments checked before any launch
    wg = L.stts_conv1d_wgrad_tx
    assert wg(0, None, None, 2, 37, 257, 32, 32, 9, 2, 4, Lq, None, None, None, 0, None) == -2
    assert wg(1, None, None, 2, 37, 257, 32, 32, 9, 2, 4, Lq, None, None, None, 0, None) == -1


def test_module_refuses_groups_and_padding_modes():
    with pytest.raises(NotImplementedError):
        Conv1d(8, 8, 3, groups=2)
    with pytest.raises(NotImplementedError):
        Conv1d(8, 8, 3, padding=1, padding_mode="reflect")


def test_forward_without_device_fails_loudly():
    if torch.cuda.is_available():
        pytest.skip("CPU-only check")
    m = Conv1d(4, 4, 3, padding=1)
    with pytest.raises(RuntimeError, match="HIP device"):
        m(torch.randn(1, 4, 10))


def test_training_resblock_matches_reference_layout():
    """training.AdaINResBlock1 has the reference AdaINResBlock1's state-dict keys and shapes (the
    inference-side params.AdaINResBlock1 is pinned to the reference names by test_native_abi)."""
    from stts2_mi355x.params import AdaINResBlock1 as Ref
    from stts2_mi355x.training import AdaINResBlock1
    a = AdaINResBlock1(64, 7, (1, 3, 5), 128).state_dict()
    b = Ref(64, 7, (1, 3, 5), 128).state_dict()
    assert sorted(a) == sorted(b)
    for k in a:
        assert a[k].shape == b[k].shape, k


def test_layer_workspace_queries():
    L = E.lib()
    assert L.stts_adain_act_workspace_bytes(2, 300, 64) > 0
    assert L.stts_adain_act_workspace_bytes(0, 300, 64) == -1


@pytest.mark.parametrize("cin,cout,up", [(1090, 1024, False), (1090, 512, True), (514, 1024, False)])
def test_training_resblk1d_matches_reference_layout(cin, cout, up):
    from stts2_mi355x.params import AdainResBlk1d as Ref
    from stts2_mi355x.training import AdainResBlk1d
    a = AdainResBlk1d(cin, cout, 128, upsample=up).state_dict()
    b = Ref(cin, cout, 128, upsample=up).state_dict()
    assert sorted(a) == sorted(b)
    for k in a:
        assert a[k].shape == b[k].shape, k


def test_training_discriminator_p_matches_reference_layout():
    from stts2_mi355x.discriminators import DiscriminatorP as Ref
    from stts2_mi355x.training import DiscriminatorP
    a = DiscriminatorP(3).state_dict()
    b = Ref(3).state_dict()
    assert sorted(a) == sorted(b)
    for k in a:
        assert a[k].shape == b[k].shape, k
