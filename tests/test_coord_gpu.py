"""The CoordConv U-Net on the MI355X path against the CPU oracle.

The reference is a Keras script that cannot be imported here, so parity is to the oracle's
restatement (oracle.RefCoordConvUNetp / add_coords, whose coordinate channels are pinned to the
closed forms in test_oracle_golden.py) - "parity unpinned" against Keras itself."""
import pytest
import torch

pytestmark = pytest.mark.gpu

from punet import kernels as K  # noqa: E402
from punet import bce_loss  # noqa: E402
from unet import CoordConvUNetp  # noqa: E402
import oracle  # noqa: E402

DEV = torch.device("cuda")


@pytest.mark.parametrize("with_r,c,w", [(False, 3, 17), (True, 3, 17), (True, 1, 19), (False, 1, 19)])
def test_add_coords_kernel(with_r, c, w):
    """c = 1 with r takes the one-float4-per-pixel kernel (the CoordConv U-Net's input)"""
    g = torch.Generator().manual_seed(1)
    x = torch.rand(2, c, 17, w, generator=g)
    got = K.add_coords(x.to(DEV), with_r).cpu()
    ref = oracle.add_coords(x, with_r=with_r).permute(0, 2, 3, 1)
    torch.testing.assert_close(got, ref, rtol=0, atol=2e-7)
    assert torch.equal(got[..., :c + 2], ref[..., :c + 2])


@pytest.mark.parametrize("with_r,depth,base", [(True, 4, 8), (False, 3, 16)])
def test_coordconv_unetp_matches_oracle(with_r, depth, base):
    """fwd (logits through the head), loss and every gradient vs the fp64 oracle, 2 slots, 64x64."""
    torch.manual_seed(21)
    ref = oracle.RefCoordConvUNetp(1, 1, rule="oja", nbf=64, base_ch=base, with_r=with_r, depth=depth)
    torch.manual_seed(21)
    net = CoordConvUNetp(1, 1, DEV, rule="oja", nbf=64, base_ch=base, with_r=with_r, depth=depth)
    for (k, a), (_, b) in zip(net.state_dict().items(), ref.state_dict().items()):
        assert torch.equal(a.cpu(), b), k                     # same seeded init
    g = torch.Generator().manual_seed(4)
    B = 2
    x = torch.rand(B, 1, 64, 64, generator=g)
    t = (torch.rand(B, 64, 64, generator=g) > 0.5).float()
    H = 0.05 * torch.randn(B, 64, 64, generator=g)
    y, hn = net(x.to(DEV), H.to(DEV))
    loss = bce_loss(y, t.to(DEV))
    loss.backward()
    ref = ref.double()
    yr, hr = ref(x.double(), H.double())
    lr_ = oracle.bce_loss(yr, t.double())
    lr_.backward()
    torch.testing.assert_close(y.double().cpu(), yr, rtol=1e-4, atol=1e-6)
    torch.testing.assert_close(hn.double().cpu(), hr, rtol=1e-4, atol=1e-6)
    assert abs(loss.item() - lr_.item()) < 1e-5
    for (k, p), (_, pr) in zip(net.named_parameters(), ref.named_parameters()):
        if k == "eta":
            assert p.grad is None
            continue
        got, want = p.grad.double().cpu(), pr.grad
        rel = ((got - want).norm() / max(want.norm().item(), 1e-30)).item()
        assert rel < 2e-3, (k, rel)
