"""Per-kernel parity of the HIP library against plain PyTorch-CPU fp32 (the oracle's arithmetic).

Every call goes through the C-ABI (punet.kernels -> libplastic_unet.so).  Tolerances are fp32
summation-order tolerances: rtol 1e-4 / atol 1e-5 relative to the output scale.
"""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

from punet import kernels as K  # noqa: E402
from punet import trunk as T  # noqa: E402
from punet.head import PlasticHeadFunction, bce_loss  # noqa: E402
from punet.optim import FusedAdam  # noqa: E402
import oracle  # noqa: E402
from conftest import golden  # noqa: E402

DEV = "cuda"


def rnd(*shape, g, scale=1.0):
    return (torch.randn(*shape, generator=g) * scale).float()


def nhwc(t):
    return t.permute(0, 2, 3, 1).contiguous()


def nchw(t):
    return t.permute(0, 3, 1, 2).contiguous()


def assert_close(got, ref, rtol=1e-4, atol_rel=1e-5):
    got = got.detach().float().cpu()
    ref = ref.detach().float().cpu()
    assert got.shape == ref.shape, (got.shape, ref.shape)
    scale = max(ref.abs().max().item(), 1e-30)
    torch.testing.assert_close(got, ref, rtol=rtol, atol=atol_rel * scale)


CONV_CASES = [
    # B, H, W, c0, c1, cout
    (2, 16, 16, 1, 0, 8),       # single-channel stem kernel (N = 8)
    (2, 37, 70, 1, 0, 16),      # single-channel stem kernel (N = 16): partial 16 x 64 tiles
    (2, 40, 70, 1, 0, 64),      # single-channel stem kernel (N = 64): partial 16 x 64 tiles
    (1, 17, 33, 1, 0, 32),      # single-channel stem kernel (N = 32), odd sizes
    (2, 12, 20, 8, 0, 16),      # vec4 loader, non-square
    (3, 16, 16, 64, 0, 64),     # chunk16 loader, 256x64 tile
    (2, 8, 8, 16, 16, 24),      # two sources (concat), N not a tile multiple
    (1, 8, 8, 8, 8, 8),         # two sources, vec4
    (2, 32, 32, 32, 0, 128),    # 128x128 tile
    (1, 4, 4, 64, 64, 40),      # tiny M, 64x64 tile, split-K (fwd + dgrad with the n0 split)
    (2, 8, 8, 48, 0, 64),       # wgrad 64x128 tile, ragged last k-tile, bias column sums
    (1, 8, 8, 64, 64, 32),      # wgrad 64x128 tile, two sources
    (2, 9, 13, 64, 64, 64),     # wgrad 64x576 6-wave tile (K = 2 x 576), two sources, ragged pixels
    (2, 12, 20, 128, 128, 256), # wgrad split-once planes kernel (128x256): two sources, non-square
    (1, 9, 13, 64, 0, 136),     # planes kernel: N not a tile multiple, ragged pixels, ragged k-tile
    (2, 16, 32, 64, 64, 128),   # halo-reuse wgrad: two sources, 2 x 2 channel tiles, image-row edges
    (1, 32, 16, 192, 0, 64),    # halo-reuse wgrad: 3 input-channel tiles, 16-wide rows (every stage at both edges)
    (8, 64, 64, 64, 0, 64),     # halo2 wgrad (64-channel tile): 8 stages per split, the 3-deep raw ring wraps
    (2, 32, 32, 128, 128, 128), # halo2 wgrad (128-channel tile): two sources, 2 input tiles
    (1, 16, 48, 64, 128, 192),  # halo2 wgrad (64-channel tiles): 3 input x 3 output tiles, 3 stages per row
    (2, 37, 45, 16, 0, 16),     # small-channel direct kernels: several 16x32 tiles, ragged edges
    (1, 19, 70, 4, 4, 4),       # small-channel, two 4-channel sources, N = 4
    (1, 20, 36, 8, 4, 8),       # small-channel wgrad C = 12 (padded item groups), N = 8
    (2, 16, 40, 4, 0, 16),      # small-channel wgrad C = 4, N = 16
    (2, 32, 64, 32, 0, 32),     # 32-channel lean tile (128 x 32): fwd and dgrad, N = 32
    (1, 16, 64, 32, 32, 32),    # 32-channel lean tile, two sources
    (32, 64, 64, 32, 0, 32),    # 256 x 32 lean tile (>= 480 tiles), the C4 64^2 level
]

# 8/16-channel layers on the 16x16x32 MFMA kernel (csrc/smallconv.hip; K.set_smallx6)
SMALL_X6_CASES = [
    (2, 40, 70, 8, 0, 8),       # 8 -> 8: partial 16 x 32 tiles
    (1, 33, 65, 8, 8, 16),      # two 8-channel sources -> 16 (dgrad: 16 -> 8 + 8 with the split)
    (2, 64, 64, 16, 0, 8),      # 16 -> 8 (dgrad 8 -> 16)
    (1, 17, 36, 16, 0, 16),     # 16 -> 16, odd height
    (2, 37, 45, 16, 0, 16),     # ragged edges on both axes
    (1, 17, 36, 8, 0, 8),       # 8 -> 8 row pairs: odd height (the last pair's second row is padding)
    (1, 33, 40, 8, 8, 8),       # 8 + 8 -> 8 row pairs (C = 16: 6 k-steps), odd height
    (2, 3, 20, 16, 0, 8),       # one partial tile, rows past Ho inside the first pair
]


@pytest.mark.parametrize("B,H,W,c0,c1,cout", CONV_CASES)
def test_conv3x3_fwd_dgrad_wgrad(B, H, W, c0, c1, cout):
    g = torch.Generator().manual_seed(B * 1000 + H * 10 + c0 + c1 + cout)
    x0 = rnd(B, c0, H, W, g=g)
    x1 = rnd(B, c1, H, W, g=g) if c1 else None
    w = rnd(cout, c0 + c1, 3, 3, g=g, scale=0.2)
    b = rnd(cout, g=g)
    xcat = torch.cat([x0, x1], 1) if c1 else x0
    xcat.requires_grad_(True)
    wr = w.clone().requires_grad_(True)
    br = b.clone().requires_grad_(True)
    z = F.conv2d(xcat, wr, br, padding=1)
    y = torch.relu(z)
    gy = rnd(*y.shape, g=g)
    y.backward(gy)
    dz = gy * (y > 0).float()

    pk = T._Packs()
    dx0, dx1 = nhwc(x0).to(DEV), (nhwc(x1).to(DEV) if c1 else None)
    yk = T.conv3x3(dx0, w.to(DEV), b.to(DEV), pk, x1=dx1, relu=True)
    assert_close(nchw(yk), y)
    # dgrad (with the split + the relu masks of the sources)
    dzk = nhwc(dz).to(DEV)
    m0 = dx0
    d0, d1 = T.conv3x3_dgrad(dzk, w.to(DEV), pk, split=c0 if c1 else None, mask0=m0,
                             mask1=dx1 if c1 else None)
    ref_dx = xcat.grad * (xcat > 0).float()
    got = torch.cat([d0, d1], 3) if c1 else d0
    assert_close(nchw(got), ref_dx)
    # wgrad + bias grad
    dw, db = T.conv3x3_wgrad(dzk, dx0, dx1)
    assert_close(dw, wr.grad)
    assert_close(db, br.grad)


@pytest.mark.parametrize("C,N", [(4, 4), (8, 8), (12, 8), (16, 16)])
def test_small_channel_wgrad_without_bias(C, N):
    """The small-channel weight gradient with bias_mode 0 (K = 9C is then a multiple of 4, so the
    slab has no bias column): every entry equals the bias_mode 1 run of the same layer - an
    unguarded bias write at column K would land on the next row's tap-0 entry (and one float past
    the slab for the last row of the last block)."""
    g = torch.Generator().manual_seed(C * 10 + N)
    B, H, W = 2, 24, 40
    x = nhwc(rnd(B, C, H, W, g=g)).to(DEV)
    dz = nhwc(rnd(B, N, H, W, g=g)).to(DEV)
    dw0 = torch.full((N, C, 3, 3), float("nan"), device=DEV)
    K.wgrad(batch=B, in_hw=(H, W), out_hw=(H, W), k=3, stride=1, pad=1, rows=dz, n=N, src0=x, c0=C,
            dweight=dw0, bias_mode=0)
    dw1 = torch.empty(N, C, 3, 3, device=DEV)
    db1 = torch.empty(N, device=DEV)
    K.wgrad(batch=B, in_hw=(H, W), out_hw=(H, W), k=3, stride=1, pad=1, rows=dz, n=N, src0=x, c0=C,
            dweight=dw1, bias_mode=1, dbias=db1)
    assert torch.equal(dw0, dw1)
    ref = torch.nn.grad.conv2d_weight(nchw(x).cpu(), (N, C, 3, 3), nchw(dz).cpu(), padding=1)
    assert_close(dw0, ref)


@pytest.mark.gpu
@pytest.mark.parametrize("C,N,bias", [(4, 8, True), (4, 8, False), (3, 8, True), (4, 16, True), (3, 4, False)])
def test_pointwise_wgrad(C, N, bias):
    """The 1x1 small-channel weight gradient (wgrad_pw_kernel, C4's CoordConv conv): against the fp64
    torch gradient, bias_mode 0 equal to bias_mode 1's weights, bitwise run to run."""
    assert K.wgrad_kind(batch=3, hw=(40, 56), n=N, c0=C, k=1) == 6
    g = torch.Generator().manual_seed(C * 100 + N)
    B, H, W = 3, 40, 56
    x = nhwc(rnd(B, C, H, W, g=g)).to(DEV)
    dz = nhwc(rnd(B, N, H, W, g=g)).to(DEV)

    def run():
        dw = torch.full((N, C, 1, 1), float("nan"), device=DEV)
        db = torch.full((N,), float("nan"), device=DEV) if bias else None
        K.wgrad(batch=B, in_hw=(H, W), out_hw=(H, W), k=1, stride=1, pad=0, rows=dz, n=N, src0=x, c0=C,
                dweight=dw, bias_mode=1 if bias else 0, dbias=db)
        return dw, db

    dw, db = run()
    dw2, db2 = run()
    assert torch.equal(dw, dw2) and (not bias or torch.equal(db, db2))
    xr, gr = nchw(x).cpu().double(), nchw(dz).cpu().double()
    ref = torch.einsum("bchw,bnhw->nc", xr, gr).reshape(N, C, 1, 1)
    assert torch.allclose(dw.cpu().double(), ref, rtol=1e-5, atol=1e-4), (dw.cpu().double() - ref).abs().max()
    if bias:
        assert torch.allclose(db.cpu().double(), gr.sum((0, 2, 3)), rtol=1e-5, atol=1e-4)


@pytest.mark.parametrize("B,H,W,c0,c1,cout", SMALL_X6_CASES)
def test_conv3x3_small_channel_x6(B, H, W, c0, c1, cout):
    prev = K.set_smallx6(True)
    try:
        test_conv3x3_fwd_dgrad_wgrad(B, H, W, c0, c1, cout)
    finally:
        K.set_smallx6(prev)


# (1, 4, 512, 64): tiny pixel grid, deep K -> split-K igemm for the shuffled forward and the dgrad
@pytest.mark.parametrize("B,h,cin,cout", [(2, 4, 16, 16), (3, 8, 64, 64), (2, 8, 8, 8), (1, 16, 128, 128),
                                          (1, 4, 512, 64)])
def test_convT2x2(B, h, cin, cout):
    g = torch.Generator().manual_seed(h * 7 + cin)
    x = rnd(B, cin, h, h, g=g).relu().requires_grad_(True)
    w = rnd(cin, cout, 2, 2, g=g, scale=0.3).requires_grad_(True)
    b = rnd(cout, g=g).requires_grad_(True)
    u = F.conv_transpose2d(x, w, b, stride=2)
    gu = rnd(*u.shape, g=g)
    u.backward(gu)
    pk = T._Packs()
    xk = nhwc(x.detach()).to(DEV)
    uk = T.convT2x2(xk, w.detach().to(DEV), b.detach().to(DEV), pk)
    assert_close(nchw(uk), u)
    guk = nhwc(gu).to(DEV)
    dxk = T.convT2x2_dgrad(guk, w.detach().to(DEV), pk, mask=xk)
    assert_close(nchw(dxk), x.grad * (x > 0).float())
    dw, db = T.convT2x2_wgrad(xk, guk)
    assert_close(dw, w.grad)
    assert_close(db, b.grad)


@pytest.mark.parametrize("B,h,cin,cout", [(3, 8, 64, 64), (2, 16, 128, 128), (4, 32, 64, 64)])
def test_convT_bias_grad_run_to_run_bitwise(B, h, cin, cout):
    """The ConvT bias gradient (wgrad_finish4_kernel bias_mode 2: 4 interleaved fp64 chains over the
    flattened (tap, split) sequence) is deterministic: two runs agree bit for bit, weights included,
    and both match the torch gradient."""
    g = torch.Generator().manual_seed(h * 11 + cin)
    x = rnd(B, cin, h, h, g=g).relu()
    gu = rnd(B, cout, 2 * h, 2 * h, g=g)
    xk, guk = nhwc(x).to(DEV), nhwc(gu).to(DEV)
    dw, db = T.convT2x2_wgrad(xk, guk)
    dw2, db2 = T.convT2x2_wgrad(xk, guk)
    assert torch.equal(dw, dw2) and torch.equal(db, db2)
    assert_close(db, gu.sum((0, 2, 3)))
    wr = torch.zeros(cin, cout, 2, 2, requires_grad=True)
    F.conv_transpose2d(x, wr, stride=2).backward(gu)
    assert_close(dw, wr.grad)


@pytest.mark.parametrize("B,H,W,C", [(2, 8, 8, 16), (1, 7, 9, 3), (2, 16, 16, 64)])
def test_maxpool(B, H, W, C):
    g = torch.Generator().manual_seed(H * W + C)
    x = rnd(B, C, H, W, g=g).relu()
    x[:, :, 0:2, 0:2] = 0.5            # ties inside one window: first max wins
    xr = x.clone().requires_grad_(True)
    y = F.max_pool2d(xr, 2)
    gy = rnd(*y.shape, g=g)
    y.backward(gy)
    xk = nhwc(x).to(DEV)
    yk = K.maxpool2_fwd(xk)
    assert torch.equal(nchw(yk).cpu(), y.detach())
    prev = rnd(B, C, H, W, g=g)
    dxk = nhwc(prev).to(DEV)
    K.maxpool2_bwd(xk, nhwc(gy).to(DEV), dxk, relu_mask=True, accumulate=True)
    ref = prev + xr.grad * (x > 0).float()
    assert_close(nchw(dxk), ref, rtol=1e-6, atol_rel=1e-7)
    dxk2 = torch.empty_like(xk)
    K.maxpool2_bwd(xk, nhwc(gy).to(DEV), dxk2, relu_mask=False, accumulate=False)
    assert torch.equal(nchw(dxk2).cpu(), xr.grad)


@pytest.mark.parametrize("rows_hw,C", [((2, 16, 16), 64), ((1, 8, 8), 8), ((3, 5, 7), 128), ((2, 9, 13), 16),
                                         ((2, 17, 11), 32), ((4, 96, 96), 8), ((2, 64, 64), 32)])
def test_outconv(rows_hw, C):
    B, H, W = rows_hw
    g = torch.Generator().manual_seed(C + H)
    x = rnd(B, C, H, W, g=g).relu().requires_grad_(True)
    w = rnd(1, C, 1, 1, g=g).requires_grad_(True)
    b = rnd(1, g=g).requires_grad_(True)
    y = F.conv2d(x, w, b)
    gy = rnd(*y.shape, g=g)
    y.backward(gy)
    xk = nhwc(x.detach()).to(DEV)
    yk = K.outconv_fwd(xk, w.detach().reshape(-1).to(DEV), b.detach().to(DEV))
    assert_close(yk, y[:, 0])
    dxk, dwk, dbk = K.outconv_bwd(xk, w.detach().reshape(-1).to(DEV), gy[:, 0].contiguous().to(DEV), relu_mask=True)
    assert_close(nchw(dxk), x.grad * (x > 0).float())
    assert_close(dwk, w.grad.reshape(-1))
    assert_close(dbk, b.grad)


@pytest.mark.parametrize("rule", ["hebb", "oja"])
@pytest.mark.parametrize("N", [32, 128])
def test_plastic_head_golden(rule, N):
    g = golden("head_%s_N%d.npz" % (rule, N))
    t = {k: torch.from_numpy(v) for k, v in g.items()}
    X = t["X"][None].to(DEV).requires_grad_(True)
    w = t["w"].to(DEV).requires_grad_(True)
    al = t["alpha"].to(DEV).requires_grad_(True)
    eta = t["eta"].to(DEV).requires_grad_(True)
    Y, Hn = PlasticHeadFunction.apply(X, t["H"][None].to(DEV), w, al, eta, 0 if rule == "hebb" else 1, True)
    loss = bce_loss(Y, t["t"].to(DEV))
    loss.backward()
    assert_close(Y[0], t["Y"])
    assert_close(Hn[0], t["Hn"])
    assert abs(loss.item() - float(g["loss"])) <= 1e-6 * abs(float(g["loss"]))
    assert_close(X.grad[0], t["dX"])
    assert_close(w.grad, t["dw"])
    assert_close(al.grad, t["dalpha"])
    assert eta.grad is None          # S3


@pytest.mark.parametrize("rule", ["hebb", "oja"])
def test_trace_update_bit_exact(rule):
    """Elementwise update: same op order as ATen, FP contraction off -> bit-identical to the oracle."""
    g = torch.Generator().manual_seed(3)
    B, N = 32, 128
    H = rnd(B, N, N, g=g, scale=0.3)
    X = rnd(B, N, N, g=g, scale=2.0)
    Y = torch.rand(B, N, N, generator=g)
    eta = torch.tensor([0.0137])
    ref = oracle.trace_update(H, X[:, 0, :], Y[:, 0, :], eta, rule)
    got = K.trace_update(H.to(DEV), X.to(DEV), Y.to(DEV), eta.to(DEV), 0 if rule == "hebb" else 1)
    assert torch.equal(got.cpu(), ref)


@pytest.mark.parametrize("rule", ["hebb", "oja"])
def test_trace_sequence_golden(rule):
    g = golden("trace_seq_%s.npz" % rule)
    w, al, eta = (torch.from_numpy(g[k]).to(DEV) for k in ("w", "alpha", "eta"))
    H = torch.zeros(1, 32, 32, device=DEV)
    for k in range(16):
        Y, H = K.plastic_fwd(torch.from_numpy(g["X"][k])[None].to(DEV), H, w, al, eta, 0 if rule == "hebb" else 1)
        assert_close(Y[0], torch.from_numpy(g["Y"][k]))
        assert_close(H[0], torch.from_numpy(g["H"][k]))


@pytest.mark.parametrize("B,N", [(8, 512), (32, 256), (2, 128)])
def test_plastic_bwd_against_fp64(B, N):
    """pu_plastic_bwd on both tile sizes (64-tiles when the grid has >= 512 blocks: 8 x 512^2,
    32 x 256^2; 32-tiles otherwise) against the fp64 gradients dX = G Weff^T,
    dw = sum_b X_b^T G_b, dalpha = sum_b (X_b^T G_b) . H_b with G = dY (1 - Y) Y."""
    g = torch.Generator().manual_seed(B + N)
    X = rnd(B, N, N, g=g, scale=2.0)
    H = rnd(B, N, N, g=g, scale=0.2)
    w = rnd(N, N, g=g, scale=0.05)
    al = torch.rand(N, N, generator=g) * 0.05
    Y = torch.rand(B, N, N, generator=g)
    dY = rnd(B, N, N, g=g)
    dx, dw, da = K.plastic_bwd(X.to(DEV), H.to(DEV), w.to(DEV), al.to(DEV), Y.to(DEV), dY.to(DEV))
    Gd = dY.double() * (1 - Y.double()) * Y.double()
    weff = w.double()[None] + al.double()[None] * H.double()
    T = torch.einsum("bik,bij->bkj", X.double(), Gd)
    ref_dx = torch.einsum("bij,bkj->bik", Gd, weff)
    for got, ref in ((dx, ref_dx), (dw, T.sum(0)), (da, (T * H.double()).sum(0))):
        got = got.cpu().double()
        assert (got - ref).abs().max().item() <= 1e-5 * ref.abs().max().item() + 1e-6, (got - ref).abs().max()


def test_plastic_head_batched_slots_match_oracle():
    g = torch.Generator().manual_seed(9)
    B, N = 32, 128
    X = rnd(B, N, N, g=g, scale=2.0).requires_grad_(True)
    H = rnd(B, N, N, g=g, scale=0.2)
    w = rnd(N, N, g=g, scale=0.05).requires_grad_(True)
    al = (torch.rand(N, N, generator=g) * 0.05).requires_grad_(True)
    eta = torch.tensor([0.02])
    tg = (torch.rand(B, N, N, generator=g) > 0.5).float()
    Y, Hn = oracle.plastic_head(X, H, w, al, eta, "oja")
    oracle.bce_loss(Y, tg).backward()
    Xd = X.detach().to(DEV).requires_grad_(True)
    wd = w.detach().to(DEV).requires_grad_(True)
    ad = al.detach().to(DEV).requires_grad_(True)
    Yk, Hk = PlasticHeadFunction.apply(Xd, H.to(DEV), wd, ad, eta.to(DEV), 1, True)
    bce_loss(Yk, tg.to(DEV)).backward()
    assert_close(Yk, Y)
    assert_close(Hk, Hn)
    assert_close(Xd.grad, X.grad)
    assert_close(wd.grad, w.grad)
    assert_close(ad.grad, al.grad)


def test_bce_edges_golden():
    g = golden("bce_edge.npz")
    y = torch.from_numpy(g["y"]).to(DEV).requires_grad_(True)
    loss = bce_loss(y, torch.from_numpy(g["t"]).to(DEV))
    loss.backward()
    assert abs(loss.item() - float(g["loss"])) <= 1e-6 * abs(float(g["loss"]))
    assert_close(y.grad, torch.from_numpy(g["dy"]))
    z = torch.from_numpy(g["z"]).to(DEV).requires_grad_(True)
    lz = bce_loss(torch.sigmoid(z), torch.from_numpy(g["tz"]).to(DEV))
    lz.backward()
    assert abs(lz.item() - float(g["lz"])) <= 1e-6 * abs(float(g["lz"]))
    assert_close(z.grad, torch.from_numpy(g["dz"]))


def test_fused_adam_matches_torch_adam():
    g = torch.Generator().manual_seed(1)
    shapes = [(64, 3, 3, 3), (64,), (7,), (1000, 33), (5, 5)]
    ref = [torch.nn.Parameter(rnd(*s, g=g)) for s in shapes]
    dev = [torch.nn.Parameter(p.detach().clone().to(DEV)) for p in ref]
    o1 = torch.optim.Adam(ref, lr=3e-3)
    o2 = FusedAdam(dev, lr=3e-3)
    s1 = torch.optim.lr_scheduler.StepLR(o1, step_size=2, gamma=0.666)
    s2 = torch.optim.lr_scheduler.StepLR(o2, step_size=2, gamma=0.666)
    for step in range(5):
        for a, b in zip(ref, dev):
            gr = rnd(*a.shape, g=g)
            a.grad = gr.clone()
            b.grad = gr.to(DEV)
        dev[2].grad = None      # a parameter without gradient is skipped (eta, S3)
        ref[2].grad = None
        b_ref = [a.detach().clone() for a in ref]
        b_dev = [b.detach().cpu() for b in dev]
        o1.step(); o2.step(); s1.step(); s2.step()
        # each step's update to 1e-6 of its own size (+1 ulp of the parameter): 1-beta2 formed from an
        # fp32-rounded beta2 (1.3e-5 off) fails this
        for a, b, a0, b0 in zip(ref, dev, b_ref, b_dev):
            assert torch.equal(a0, b0)
            du_ref = (a.detach() - a0).double()
            du_dev = (b.detach().cpu() - a0).double()
            bound = 1e-6 * du_ref.abs().max().item() + 1.2e-7 * a0.abs().max().item()
            assert (du_dev - du_ref).abs().max().item() <= bound, (step, a.shape)
            b.data.copy_(a.detach())     # judge every step from the same parameters
    for a, b in zip(ref, dev):
        assert_close(b, a, rtol=1e-6, atol_rel=1e-6)


@pytest.mark.parametrize("B,N", [(32, 128), (128, 128), (3, 50), (2, 200), (1, 512)])
@pytest.mark.parametrize("rule", [0, 1])
def test_fused_head_trace_equals_two_launch_path(B, N, rule):
    """pu_plastic_fwd fuses the trace update into the GEMM (every block recomputes row 0 of its
    column tile).  It must equal, bit for bit, the GEMM followed by the stand-alone update on its
    own Y (the in-place call takes that path), for both tile sizes (32: small grids, 64) and
    ragged N."""
    g = torch.Generator().manual_seed(B * 1000 + N)
    X = rnd(B, N, N, g=g, scale=2.0).to(DEV)
    H = rnd(B, N, N, g=g, scale=0.2).to(DEV)
    w = rnd(N, N, g=g, scale=0.05).to(DEV)
    al = (torch.rand(N, N, generator=g) * 0.05).to(DEV)
    eta = torch.tensor([0.0173], device=DEV)
    Y, Hn = K.plastic_fwd(X, H, w, al, eta, rule, True)
    Y2, none = K.plastic_fwd(X, H, w, al, eta, rule, False)
    assert none is None
    assert torch.equal(Y, Y2)
    Hn2 = K.trace_update(H, X, Y2, eta, rule)
    assert torch.equal(Hn, Hn2)
    Yr, Hr = oracle.plastic_head(X.cpu(), H.cpu(), w.cpu(), al.cpu(), eta.cpu(), "hebb" if rule == 0 else "oja")
    assert_close(Y, Yr)
    assert_close(Hn, Hr)


@pytest.mark.parametrize("rule", [0, 1])
@pytest.mark.parametrize("B,N,C,dt", [(3, 128, 64, torch.float32), (2, 32, 8, torch.float32),
                                      (2, 64, 12, torch.float32), (1, 512, 8, torch.float32),
                                      (2, 48, 128, torch.float32), (3, 128, 64, torch.bfloat16),
                                      # N > 128 whose Weff does not fit one LDS chunk and is not a
                                      # power of two (chunk 72 / 64 / 40 / 32 rows)
                                      (2, 144, 64, torch.float32), (1, 192, 16, torch.float32),
                                      (1, 320, 8, torch.float32), (1, 384, 64, torch.float32),
                                      # 32-row blocks (N >= 256, N % 32 == 0) and the 16-row
                                      # fallback at N = 272
                                      (2, 256, 16, torch.bfloat16), (1, 272, 8, torch.float32),
                                      # the pipelined single-chunk path (C == 4 L) at every L
                                      (4, 64, 4, torch.float32), (2, 112, 32, torch.bfloat16),
                                      # N = 128 with C = 48: L = 16 lanes but C < 64 - the serial
                                      # kernel (the pipelined one would read the next pixel)
                                      (2, 128, 48, torch.float32), (2, 128, 48, torch.bfloat16),
                                      # the pipelined kernel's XCD block order: B % 8 == 0 (each
                                      # slot on one XCD) and B = 9 (one slot straddles two)
                                      (32, 128, 64, torch.float32), (9, 128, 96, torch.bfloat16)])
def test_fused_head_equals_outconv_then_head(rule, B, N, C, dt):
    """pu_plastic_head_fwd (outconv + Weff GEMM on v_mfma_f32_16x16x4_f32 + sigmoid + trace update,
    one launch) is bit-identical to the two-kernel path outconv_fwd -> plastic_fwd: the outconv sum
    uses the same lane tree, and the f32 MFMA is a k-ordered fma chain like the VALU head."""
    g = torch.Generator().manual_seed(N + C)
    feat = torch.randn(B, N, N, C, generator=g).relu_().to(dt).to(DEV)
    wo = (torch.randn(C, generator=g) * 0.2).to(DEV)
    bo = torch.randn(1, generator=g).to(DEV)
    H = (0.2 * torch.randn(B, N, N, generator=g)).to(DEV)
    w = (0.05 * torch.randn(N, N, generator=g)).to(DEV)
    al = (0.05 * torch.rand(N, N, generator=g)).to(DEV)
    eta = torch.tensor([0.0137], device=DEV)
    X, Y, Hn = K.plastic_head_fwd(feat, wo, bo, H, w, al, eta, rule, True)
    X2 = K.outconv_fwd(feat, wo, bo)
    Y2, Hn2 = K.plastic_fwd(X2, H, w, al, eta, rule, True)
    assert torch.equal(X, X2)
    assert torch.equal(Y, Y2)
    assert torch.equal(Hn, Hn2)
    X3, Y3, Hn3 = K.plastic_head_fwd(feat, wo, bo, H, w, al, eta, rule, False)      # eval: no trace
    assert Hn3 is None and torch.equal(Y3, Y) and torch.equal(X3, X)


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_pack_weights_multi_equals_single_packs(dt):
    """pu_pack_weights (every operand of a model, pack + exact bf16 split fused, one launch) is
    bit-identical to pu_pack_weight (+ pu_split_weight6) per operand, for all five layouts, ragged
    K padding and channel-group-major K."""
    from punet._lib import PU_PACK_CONV_FWD, PU_PACK_CONV_DGRAD, PU_PACK_CONVT_FWD, PU_PACK_CONVT_DGRAD
    g = torch.Generator().manual_seed(5)
    specs = [((64, 32, 3, 3), PU_PACK_CONV_FWD, 32), ((64, 32, 3, 3), PU_PACK_CONV_DGRAD, 32),
             ((24, 8, 3, 3), PU_PACK_CONV_FWD, 0), ((8, 1, 3, 3), PU_PACK_CONV_FWD, 0),
             ((48, 64, 2, 2), PU_PACK_CONVT_FWD, 0), ((48, 64, 2, 2), PU_PACK_CONVT_DGRAD, 16),
             ((40, 40, 3, 3), 4, 0), ((128, 96, 3, 3), PU_PACK_CONV_DGRAD, 32)] * 5   # > 32 jobs: 2 batches
    jobs, refs = [], []
    for shape, mode, cg in specs:
        if dt == torch.bfloat16 and cg == 16:
            cg = 32 if shape[1] % 32 == 0 else 0
        w = (torch.randn(*shape, generator=g) * 3).to(DEV)
        d0, d1, kh, kw = shape
        kmin = {0: kh * kw * d1, 1: kh * kw * d0, 2: d0, 3: kh * kw * d1, 4: 4 * d0}[mode]
        k_pad = (kmin + 31) // 32 * 32 if dt == torch.bfloat16 else K.round16(kmin)
        ref = K.pack_weight(w, mode, k_pad, cgroup=cg, dtype=dt)
        out = K.pack_weight(torch.zeros_like(w), mode, k_pad, cgroup=cg, dtype=dt)   # same buffers, zero content
        jobs.append((w, out, getattr(out, "_split6", None)))
        refs.append(ref)
    K.pack_weights(jobs)
    for (w, out, planes), ref in zip(jobs, refs):
        assert torch.equal(out, ref)
        if planes is not None:
            assert torch.equal(planes, ref._split6)


def test_pack_refresh_after_optimizer_is_one_launch():
    """The trunk re-packs every moved parameter at the next forward in one pu_pack_weights call."""
    from unet import UNetp
    torch.manual_seed(0)
    net = UNetp(1, 1, DEV, rule="oja", nbf=64)
    x = torch.rand(1, 1, 64, 64, device=DEV)
    h = net.initialZeroHebb()
    y, _ = net(x, h)
    y.sum().backward()
    opt = FusedAdam(net.parameters(), lr=1e-3)
    opt.step()
    with K.KernelProfiler() as prof:
        net(x, h)
    s = prof.summary()
    assert s["pack_weight"]["launches"] == 1, s.get("pack_weight")


@pytest.mark.parametrize("C,N,relu", [(4, 8, True), (4, 16, False), (8, 8, True), (8, 16, True)])
def test_conv1x1_small_channel(C, N, relu):
    """the direct 1x1 kernel (CoordConv stem, coord_conv_script.py:61-85) vs CPU fp32"""
    from punet._lib import PU_PACK_CONV_FWD
    g = torch.Generator().manual_seed(C * 10 + N)
    B, H, W = 2, 33, 40
    x = rnd(B, C, H, W, g=g)
    w = rnd(N, C, 1, 1, g=g, scale=0.5)
    b = rnd(N, g=g)
    ref = F.conv2d(x, w, b)
    if relu:
        ref = torch.relu(ref)
    pk = T._Packs()
    xd = nhwc(x).to(DEV)
    y = torch.empty(B, H, W, N, device=DEV)
    wd = w.to(DEV)
    K.igemm(batch=B, in_hw=(H, W), out_hw=(H, W), k=1, stride=1, pad=0, src0=xd, c0=C,
            weight=pk.get(wd, PU_PACK_CONV_FWD, K.round16(C)), k_pad=K.round16(C), n=N, bias=b.to(DEV),
            dst0=y, relu=relu)
    assert_close(nchw(y), ref)
