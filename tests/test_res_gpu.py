"""UNetpRes on the MI355X path: the new kernels against torch fp32 on the
CPU, the model against the reference's golden vectors (101x101, odd sizes, both ConvT crops) and
a training-mode step with Dropout2d against the fp64 oracle with the same channel masks."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

from punet import kernels as K  # noqa: E402
from punet import res_trunk as R  # noqa: E402
from punet import bce_loss  # noqa: E402
from unet import UNetpRes  # noqa: E402
import oracle  # noqa: E402
from conftest import golden  # noqa: E402

DEV = torch.device("cuda")


def rnd(*shape, g, scale=1.0):
    return (torch.randn(*shape, generator=g) * scale).float()


def nhwc(t):
    return t.permute(0, 2, 3, 1).contiguous()


def nchw(t):
    return t.permute(0, 3, 1, 2).contiguous()


def assert_close(got, ref, rtol=1e-4, atol_rel=1e-5):
    got = got.detach().float().cpu()
    ref = torch.as_tensor(ref).detach().float().cpu()
    scale = max(ref.abs().max().item(), 1e-30)
    torch.testing.assert_close(got, ref.reshape(got.shape), rtol=rtol, atol=atol_rel * scale)


@pytest.mark.parametrize("B,h,cin,cout,crop", [(2, 6, 16, 8, 1), (1, 12, 32, 16, 0), (2, 5, 64, 32, 1),
                                               (1, 3, 8, 4, 0),
                                               # 8-channel dU: the stride-2 small-channel MFMA dgrad
                                               (2, 16, 8, 8, 1), (1, 20, 16, 8, 0), (2, 37, 16, 8, 1),
                                               (1, 5, 8, 8, 0),
                                               # 16 -> 8 channels: the ConvT forward on the
                                               # small-channel MFMA kernel (2 x 2 sub-pixel conv)
                                               (2, 19, 16, 8, 1), (1, 40, 16, 8, 0)])
def test_convT3x3_s2_crop(B, h, cin, cout, crop):
    """ConvTranspose2d(3, s=2, p=0) + the F.pad crop of unet_p_res.py:214-217: fwd, dgrad, wgrad, bias."""
    g = torch.Generator().manual_seed(h * 100 + cin + crop)
    x = rnd(B, cin, h, h, g=g).relu().requires_grad_(True)
    w = rnd(cin, cout, 3, 3, g=g, scale=0.2).requires_grad_(True)
    b = rnd(cout, g=g).requires_grad_(True)
    full = F.conv_transpose2d(x, w, b, stride=2)            # 2h+1
    u = full[:, :, crop:, crop:]
    gu = rnd(*u.shape, g=g)
    u.backward(gu)
    pk = R._Packs()
    xk = nhwc(x.detach()).to(DEV)
    H2 = 2 * h + 1 - crop
    uk = R.convT3x3(xk, w.detach().to(DEV), b.detach().to(DEV), pk, (H2, H2))
    assert_close(nchw(uk), u)
    guk = nhwc(gu).to(DEV)
    dx = R.convT3x3_dgrad(guk, w.detach().to(DEV), pk, (h, h), mask=xk)
    assert_close(nchw(dx), x.grad * (x > 0).float())
    dw, db = R.convT3x3_wgrad(xk, guk)
    assert_close(dw, w.grad)
    assert_close(db, b.grad)


@pytest.mark.parametrize("B,H,c,split", [(2, 9, 16, None), (1, 16, 32, 16), (2, 7, 8, None)])
def test_residual_conv_epilogues(B, H, c, split):
    """relu(conv(a) + b + r) forward and (conv^T(g) + g_skip) . mask backward (the RESID flag)."""
    g = torch.Generator().manual_seed(B * 7 + H + c)
    a = rnd(B, c, H, H, g=g).relu()
    r = rnd(B, c, H, H, g=g).relu()
    w = rnd(c, c, 3, 3, g=g, scale=0.2)
    bias = rnd(c, g=g)
    y = torch.relu(F.conv2d(a, w, bias, padding=1) + r)
    pk = R._Packs()
    yk = R.conv3x3(nhwc(a).to(DEV), w.to(DEV), bias.to(DEV), pk, resid=nhwc(r).to(DEV))
    assert_close(nchw(yk), y)
    gz = rnd(B, c, H, H, g=g)
    gskip = rnd(B, c, H, H, g=g)
    mask = rnd(B, c, H, H, g=g).relu()
    ref = (F.conv_transpose2d(gz, w, padding=1) + gskip) * (mask > 0).float()
    dk, _ = R.conv3x3_dgrad(nhwc(gz).to(DEV), w.to(DEV), pk, mask0=nhwc(mask).to(DEV), resid=nhwc(gskip).to(DEV))
    assert_close(nchw(dk), ref)


def test_channel_scale_and_column_sum():
    g = torch.Generator().manual_seed(3)
    x = rnd(3, 5, 7, 12, g=g)
    m = (torch.rand(3, 12, generator=g) > 0.5).float() * 2.0
    y = K.channel_scale(x.to(DEV), m.to(DEV))
    assert torch.equal(y.cpu(), x * m[:, None, None, :])
    xb = rnd(5, 64, 48, 8, g=g).to(DEV)            # in place, several grid rows per image
    mb = torch.rand(5, 8, generator=g)
    ref = xb.cpu() * mb[:, None, None, :]
    K.channel_scale(xb, mb.to(DEV), out=xb)
    assert torch.equal(xb.cpu(), ref)
    xs = rnd(3, 5, 7, 6, g=g)                       # odd channel count: scalar path
    ms = torch.rand(3, 6, generator=g)
    assert torch.equal(K.channel_scale(xs.to(DEV), ms.to(DEV)).cpu(), xs * ms[:, None, None, :])
    for rows, cols in ((1000, 8), (70001, 3), (513, 300)):
        a = rnd(rows, cols, g=g)
        s = K.column_sum(a.to(DEV)).cpu()
        torch.testing.assert_close(s, a.double().sum(0).float(), rtol=1e-6, atol=1e-6)
        again = K.column_sum(a.to(DEV)).cpu()
        assert torch.equal(s, again)                # fixed order: bitwise reproducible


@pytest.mark.parametrize("B,H,cout,cin,split", [
    (2, 20, 8, 16, 8),       # 8 -> 8 + 8: small-channel MFMA kernel
    (2, 18, 32, 32, 16),     # 32 -> 16 + 16: lean x6 tile
    (2, 16, 64, 128, 64),    # 64 -> 64 + 64: Winograd
    (1, 8, 64, 128, 64),     # 8x8 grid: Winograd with split-K (the split epilogue kernel)
    (2, 9, 16, 6, 3),        # 3 + 3 channels: the per-element epilogue
])
def test_fused_dropout_scale_in_conv_epilogue(B, H, cout, cin, split):
    """chan_scale (the Dropout2d factors of cat(u, skip), row stride >= the output channels) in the
    split data gradient's epilogue and in the ConvT forward's shuffled epilogue: bitwise equal to
    the separate pu_channel_scale pass over the unscaled outputs."""
    g = torch.Generator().manual_seed(B * 100 + H + cin)
    pk = R._Packs()
    dz = nhwc(rnd(B, cout, H, H, g=g)).to(DEV)
    w = rnd(cout, cin, 3, 3, g=g, scale=0.2).to(DEV)
    skip = nhwc(rnd(B, cin - split, H, H, g=g).relu()).to(DEV)
    ld = (cin + 3) // 4 * 4
    m = ((torch.rand(B, ld, generator=g) >= 0.5).float() * 2.0).to(DEV)
    d0, d1 = R.conv3x3_dgrad(dz, w, pk, split=split, mask1=skip)
    f0, f1 = R.conv3x3_dgrad(dz, w, pk, split=split, mask1=skip, chan_scale=m)
    assert torch.equal(f0, K.channel_scale(d0, m[:, :split].contiguous()))
    assert torch.equal(f1, K.channel_scale(d1, m[:, split:cin].contiguous()))
    # ConvT 3x3 s2 forward (SHUFFLE2): factors per output channel, row stride of the concat mask
    h = H // 2
    x = nhwc(rnd(B, cin, h, h, g=g)).to(DEV)
    wt = rnd(cin, cout, 3, 3, g=g, scale=0.2).to(DEV)
    b = rnd(cout, g=g).to(DEV)
    mt = ((torch.rand(B, cout + 8, generator=g) >= 0.5).float() * 2.0).to(DEV)
    u = R.convT3x3(x, wt, b, pk, (2 * h, 2 * h))
    uf = R.convT3x3(x, wt, b, pk, (2 * h, 2 * h), chan_scale=mt)
    assert torch.equal(uf, K.channel_scale(u, mt[:, :cout].contiguous()))


@pytest.mark.parametrize("B,H,W,C", [(2, 16, 24, 8), (3, 9, 13, 16), (2, 8, 8, 6)])
def test_maxpool_with_fused_dropout_scale(B, H, W, C):
    """pool_drop (unet_p_res.py:62) with the Dropout2d in the pool kernels: forward = maxpool then
    the per-(image, channel) factor, backward = the factor on dy routed to the argmax - bitwise the
    separate pu_channel_scale pass (even / odd sizes, vector and per-element paths)."""
    g = torch.Generator().manual_seed(B * 31 + H + C)
    x = nhwc(rnd(B, C, H, W, g=g)).to(DEV)
    m = ((torch.rand(B, C, generator=g) >= 0.5).float() * 2.0).to(DEV)
    y = K.maxpool2_fwd(x, scale=m)
    assert torch.equal(y, K.channel_scale(K.maxpool2_fwd(x), m))
    dy = rnd(*y.shape, g=g).to(DEV)
    base = rnd(*x.shape, g=g).to(DEV)
    d1 = K.maxpool2_bwd(x, dy, base.clone(), relu_mask=True, accumulate=True, scale=m)
    d2 = K.maxpool2_bwd(x, K.channel_scale(dy, m), base.clone(), relu_mask=True, accumulate=True)
    assert torch.equal(d1, d2)


def _load(net, g, prefix):
    net.load_state_dict({k[len(prefix):]: torch.from_numpy(np.asarray(v)) for k, v in g.items()
                         if k.startswith(prefix)})


def test_unetpres_golden_eval_fwd_bwd():
    """neurons=4 at 101x101 (pool floors 101->50->25->12->6; ConvT crops 13->12 and 51->50, keeps
    25 and 101) against the reference's own outputs and gradients (eval mode, oja)."""
    gi, gg = golden("unetpres_n4.npz"), golden("unetpres_n4_grad.npz")
    net = UNetpRes(1, 1, DEV, neurons=4, rule="oja", nbf=101)
    _load(net, gi, "p.")
    net.eval()
    x = torch.from_numpy(gi["x"]).to(DEV)
    y, hn = net(x, torch.from_numpy(gi["H"]).to(DEV))
    loss = bce_loss(y, torch.from_numpy(gi["t"]).to(DEV))
    loss.backward()
    assert_close(y, gi["Y"])
    assert_close(hn, gi["Hn"])
    assert abs(loss.item() - float(gi["loss"])) < 1e-5
    for k, p in net.named_parameters():
        if k == "eta":
            assert p.grad is None
            continue
        assert_close(p.grad, gg["g." + k], rtol=5e-4, atol_rel=5e-5)


class _MaskDrop(torch.nn.Module):
    def __init__(self, m):
        super().__init__()
        self.m = m

    def forward(self, x):
        return x * self.m[:, :, None, None].to(x.dtype)


def test_unetpres_training_dropout_matches_oracle():
    """Training mode, dropout 0.5 with injected per-sample channel masks, 2 slots at 64x64:
    logits, loss and every gradient against the fp64 oracle with the same masks."""
    torch.manual_seed(11)
    ref = oracle.RefUNetpRes(1, 1, neurons=8, rule="oja", nbf=64, dropout_ratio=0.5)
    net = UNetpRes(1, 1, DEV, neurons=8, rule="oja", nbf=64, dropout_ratio=0.5)
    net.load_state_dict(ref.state_dict())
    g = torch.Generator().manual_seed(5)
    B = 2
    x = torch.rand(B, 1, 64, 64, generator=g)
    t = (torch.rand(B, 64, 64, generator=g) > 0.5).float()
    H = 0.05 * torch.randn(B, 64, 64, generator=g)
    masks = {}

    def mask_fn(name, b, c, p):
        m = (torch.rand(b, c, generator=g) >= p).float() / (1.0 - p)
        masks[name] = m
        return m.to(DEV)

    trunk = net._trunk_plan()
    trunk.mask_fn = mask_fn
    net.train()
    y, hn = net(x.to(DEV), H.to(DEV))
    loss = bce_loss(y, t.to(DEV))
    loss.backward()
    # the oracle in fp64 with the same masks
    ref = ref.double()
    for k in range(1, 5):
        getattr(ref, "pool%d" % k).dpool[1] = _MaskDrop(masks["pool%d" % k])
    for name in ("uconv4", "uconv3", "uconv2", "uconv1"):
        getattr(ref, name).uconv[0] = _MaskDrop(masks[name])
    yr, hr = ref(x.double(), H.double())
    lr_ = oracle.bce_loss(yr, t.double())
    lr_.backward()
    assert_close(y, yr, rtol=1e-4, atol_rel=1e-5)
    assert_close(hn, hr, rtol=1e-4, atol_rel=1e-5)
    assert abs(loss.item() - lr_.item()) < 1e-5
    for (k, p), (_, pr) in zip(net.named_parameters(), ref.named_parameters()):
        if k == "eta":
            continue
        got, want = p.grad.double().cpu(), pr.grad
        rel = ((got - want).norm() / max(want.norm().item(), 1e-30)).item()
        assert rel < 2e-3, (k, rel)


def test_unetpres_batchnorm_golden():
    """UNetpRes(batch_norm=True) on the HIP path vs the reference's golden vectors: train-mode
    fwd/bwd, running statistics after two forwards, eval-mode forward."""
    g = golden("unetpres_bn.npz")
    torch.manual_seed(6)
    ref = oracle.RefUNetpRes(1, 1, neurons=4, dropout_ratio=0.0, rule="oja", nbf=64, batch_norm=True)
    net = UNetpRes(1, 1, DEV, neurons=4, dropout_ratio=0.0, rule="oja", nbf=64, batch_norm=True)
    net.load_state_dict(ref.state_dict())
    net.train()
    xs = torch.from_numpy(g["xs"]).to(DEV)
    hebb = torch.from_numpy(g["hebb"]).to(DEV)
    y, hn = net(xs[0], hebb)
    loss = bce_loss(y, torch.from_numpy(g["t"]).to(DEV))
    loss.backward()
    assert_close(y, g["Y"])
    assert_close(hn, g["Hn"])
    assert abs(loss.item() - float(g["loss"])) < 1e-5
    for k, p in net.named_parameters():
        if k == "eta":
            assert p.grad is None
            continue
        assert_close(p.grad, torch.from_numpy(g["g." + k]), rtol=1e-3, atol_rel=1e-4)
    for k, v in net.state_dict().items():
        if "s1." + k in g:
            assert_close(v, g["s1." + k])
    with torch.no_grad():
        y2, _ = net(xs[1], hebb)
    assert_close(y2, g["Y2"])
    for k, v in net.state_dict().items():
        if "s2." + k in g:
            assert_close(v, g["s2." + k])
    net.eval()
    with torch.no_grad():
        ye, he = net(xs[2], torch.zeros(64, 64, device=DEV))
    assert_close(ye, g["Ye"])
    assert_close(he, g["He"])


def test_unetpres_batchnorm_slots_match_oracle():
    """Three slots in one training step == the oracle's per-slot BatchNorm."""
    torch.manual_seed(3)
    ref = oracle.RefUNetpRes(1, 1, neurons=4, dropout_ratio=0.0, rule="hebb", nbf=32, batch_norm=True)
    net = UNetpRes(1, 1, DEV, neurons=4, dropout_ratio=0.0, rule="hebb", nbf=32, batch_norm=True)
    net.load_state_dict(ref.state_dict())
    gen = torch.Generator().manual_seed(5)
    x = torch.rand(3, 1, 32, 32, generator=gen)
    t = (torch.rand(3, 32, 32, generator=gen) > 0.5).float()
    H = 0.1 * torch.randn(3, 32, 32, generator=gen)
    yr, hr = ref(x, H)
    oracle.bce_loss(yr, t).backward()
    y, h = net(x.to(DEV), H.to(DEV))
    bce_loss(y, t.to(DEV)).backward()
    assert_close(y, yr)
    assert_close(h, hr)
    rsd = ref.state_dict()
    for k, v in net.state_dict().items():
        assert_close(v, rsd[k])
