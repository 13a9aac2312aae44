"""The halo convolution kernel (igemm_halo_x6_kernel: 3x3/s1 layers of width 32/64/128 with the
input halo split once per 16-channel chunk) against the per-tap lean kernel and PyTorch-CPU fp32.

Replaces the same nn.Conv2d(k=3, p=1) + ReLU forward and backward-data of double_conv
(reference src/unet/unet_p.py:184-201) as the per-tap kernel; K order and the MFMA order per
accumulator are the same, so with 16-channel K groups the two kernels are bit-identical, and with
32-channel groups they differ only in the order the two channel halves are summed.
"""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

from punet import kernels as K  # noqa: E402
from punet import trunk as T  # noqa: E402

DEV = "cuda"


def nhwc(t):
    return t.permute(0, 2, 3, 1).contiguous()


def nchw(t):
    return t.permute(0, 3, 1, 2).contiguous()


CASES = [
    # B, H, W, c0, c1, cout, bit-identical to the per-tap kernel.  Bit-identity needs 16-channel K
    # groups and a per-tap launch without split-K (>= 480 tiles): the first two cases
    (8, 128, 128, 48, 0, 64, True),   # fwd on the halo kernel, cgroup 16 (dgrad: N = 48, per-tap)
    (8, 128, 128, 64, 0, 48, True),   # dgrad on the halo kernel, cgroup 16 (fwd: N = 48, per-tap)
    (2, 8, 128, 16, 16, 64, False),   # W 128: 2 row blocks per image, two 16-channel sources
    (1, 16, 64, 48, 0, 128, False),   # W 64: 2 output tiles, 3 chunks
    (2, 32, 32, 64, 64, 128, False),  # W 32: 32-channel K groups (halves summed in another order)
    (1, 4, 128, 32, 96, 64, False),   # unequal concat (the per-tap lean kernel cannot take it)
]


def _run(x0, x1, w, b, dz, split):
    pk = T._Packs()
    y = T.conv3x3(x0, w, b, pk, x1=x1, relu=True)
    d0, d1 = T.conv3x3_dgrad(dz, w, pk, split=split, mask0=x0, mask1=x1)
    return y, d0, d1


@pytest.mark.parametrize("B,H,W,c0,c1,cout,exact", CASES)
def test_halo_conv_fwd_dgrad(B, H, W, c0, c1, cout, exact):
    g = torch.Generator().manual_seed(H * 1000 + W + c0 + 7 * c1 + cout)
    x0 = torch.randn(B, c0, H, W, generator=g)
    x1 = torch.randn(B, c1, H, W, generator=g) if c1 else None
    w = torch.randn(cout, c0 + c1, 3, 3, generator=g) * 0.2
    b = torch.randn(cout, generator=g)
    xcat = torch.cat([x0, x1], 1) if c1 else x0
    xcat.requires_grad_(True)
    wr = w.clone().requires_grad_(True)
    y_ref = torch.relu(F.conv2d(xcat, wr, b, padding=1))
    gy = torch.randn(*y_ref.shape, generator=g)
    y_ref.backward(gy)
    dz = gy * (y_ref > 0).float()
    dx_ref = xcat.grad * (xcat > 0).float()

    dx0 = nhwc(x0).to(DEV)
    dx1 = nhwc(x1).to(DEV) if c1 else None
    dzk = nhwc(dz).to(DEV)
    wd, bd = w.to(DEV), b.to(DEV)
    split = c0 if c1 else None

    assert K.fp32_math() == "split6"
    prev = K.set_conv_halo(True)
    try:
        yh, h0, h1 = _run(dx0, dx1, wd, bd, dzk, split)
        K.set_conv_halo(False)
        yl, l0, l1 = _run(dx0, dx1, wd, bd, dzk, split)
    finally:
        K.set_conv_halo(prev)
    torch.cuda.synchronize()
    dh = torch.cat([h0, h1], 3) if c1 else h0
    dl = torch.cat([l0, l1], 3) if c1 else l0

    # fp32 summation-order tolerance against CPU fp32 (as tests/test_kernels_gpu.py)
    for got, ref in ((nchw(yh), y_ref), (nchw(dh), dx_ref)):
        ref = ref.detach()
        torch.testing.assert_close(got.cpu(), ref, rtol=1e-4, atol=1e-5 * ref.abs().max().item())
    if exact:
        assert torch.equal(yh, yl)
        assert torch.equal(dh, dl)
    else:
        for a, r in ((yh, yl), (dh, dl)):
            torch.testing.assert_close(a, r, rtol=1e-5, atol=1e-6 * r.abs().max().item())
