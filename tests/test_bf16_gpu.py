"""bf16 mixed precision (config C3) on the MI355X path.

Kernel references are torch fp32 on the bf16-ROUNDED operands, so the only differences are the
single bf16 rounding of each kernel output (relative 2^-8 = 3.9e-3) and the fp32 accumulation
order: activations within rtol 8e-3, weight/bias gradients (fp32 outputs of an fp32-accumulated
sum of exact bf16 products) within 2e-4.  The model check is against the fp64 oracle with bars
for a bf16 trunk (logits/Y/loss and gradient relative L2), measured values documented in
DESIGN.md; the 1e-4 parity bar of the north star is the fp32 path's (test_model_gpu.py)."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

from punet import kernels as K  # noqa: E402
from punet import trunk as T  # noqa: E402
from punet import bce_loss  # noqa: E402
from unet import UNetp  # noqa: E402
import oracle  # noqa: E402

DEV = torch.device("cuda")
BF = torch.bfloat16


def rb(t):
    """round to bf16 and back (the operands the kernels actually see)"""
    return t.to(BF).float()


def rnd(*shape, g, scale=1.0):
    return rb(torch.randn(*shape, generator=g) * scale)


def nhwc(t):
    return t.permute(0, 2, 3, 1).contiguous()


def nchw(t):
    return t.permute(0, 3, 1, 2).contiguous()


def close_bf16(got, ref, rtol=8e-3, atol_rel=2e-3):
    got = got.detach().float().cpu()
    ref = ref.detach().float().cpu()
    scale = max(ref.abs().max().item(), 1e-30)
    torch.testing.assert_close(got, ref.reshape(got.shape), rtol=rtol, atol=atol_rel * scale)


def close_f32(got, ref, rtol=2e-4, atol_rel=2e-5):
    got = got.detach().float().cpu()
    ref = ref.detach().float().cpu()
    scale = max(ref.abs().max().item(), 1e-30)
    torch.testing.assert_close(got, ref.reshape(got.shape), rtol=rtol, atol=atol_rel * scale)


CASES = [
    # B, H, W, c0, c1, cout
    (2, 16, 16, 64, 0, 64),       # 256x64 / 128x64 tiles
    (2, 16, 16, 64, 64, 128),     # concat of two sources, 128x128 tile
    (3, 12, 20, 32, 32, 32),      # non-square, N = 32
    (1, 4, 4, 128, 64, 64),       # tiny pixel grid: split-K + bf16 reduce epilogue
    (2, 33, 17, 96, 0, 96),       # ragged tiles, 96 channels
    # halo-reuse wgrad (64-channel multiples, width % 16 == 0): edges, concat, odd stage counts
    (3, 7, 32, 64, 64, 64),       # 7 rows: every stage touches the top or bottom edge
    (1, 5, 48, 128, 0, 192),      # 15 stages, 2 x 3 channel tiles
    (2, 64, 64, 64, 0, 64),       # 512 stages over 512 splits; halo conv (W 64, 4 row blocks)
    # halo conv kernel (width 32/64/128, N % 64 == 0): row blocks, concat, output tiles
    (2, 8, 128, 32, 32, 64),      # W 128: 4 row blocks per image, two sources, split dgrad output
    (1, 16, 32, 64, 0, 128),      # W 32: 2 row blocks, 2 output-channel tiles
    (1, 4, 128, 32, 96, 64),      # unequal concat (the per-tap lean kernel cannot take it)
]


@pytest.mark.parametrize("B,H,W,c0,c1,cout", CASES)
def test_conv3x3_bf16_fwd_dgrad_wgrad(B, H, W, c0, c1, cout):
    g = torch.Generator().manual_seed(B * 100 + H + c0 + c1 + cout)
    x0 = rnd(B, c0, H, W, g=g).relu()
    x1 = rnd(B, c1, H, W, g=g).relu() if c1 else None
    w = rnd(cout, c0 + c1, 3, 3, g=g, scale=0.05)
    b = torch.randn(cout, generator=g)
    xcat = torch.cat([x0, x1], 1) if c1 else x0
    xcat.requires_grad_(True)
    wr = w.clone().requires_grad_(True)
    br = b.clone().requires_grad_(True)
    y = torch.relu(F.conv2d(xcat, wr, br, padding=1))
    gy = rnd(*y.shape, g=g)
    y.backward(gy)
    pk = T._Packs()
    dx0 = nhwc(x0).to(DEV).to(BF)
    dx1 = nhwc(x1).to(DEV).to(BF) if c1 else None
    yk = T.conv3x3(dx0, w.to(DEV), b.to(DEV), pk, x1=dx1)
    assert yk.dtype == BF
    close_bf16(nchw(yk), y)
    dz = (gy * (y > 0).float())
    dzk = nhwc(dz).to(DEV).to(BF)            # dz is bf16-exact (gy rounded, mask 0/1)
    d0, d1 = T.conv3x3_dgrad(dzk, w.to(DEV), pk, split=c0 if c1 else None, mask0=dx0, mask1=dx1)
    got = torch.cat([d0, d1], 3) if c1 else d0
    close_bf16(nchw(got), xcat.grad * (xcat > 0).float())
    dw, db = T.conv3x3_wgrad(dzk, dx0, dx1)
    assert dw.dtype == torch.float32
    close_f32(dw, wr.grad)
    close_f32(db, br.grad)


@pytest.mark.parametrize("B,h,cin,cout", [(2, 8, 64, 64), (1, 4, 512, 512), (2, 16, 128, 64)])
def test_convT2x2_bf16(B, h, cin, cout):
    g = torch.Generator().manual_seed(h * 7 + cin + cout)
    x = rnd(B, cin, h, h, g=g).relu().requires_grad_(True)
    w = rnd(cin, cout, 2, 2, g=g, scale=0.05).requires_grad_(True)
    b = torch.randn(cout, generator=g).requires_grad_(True)
    u = F.conv_transpose2d(x, w, b, stride=2)
    gu = rnd(*u.shape, g=g)
    u.backward(gu)
    pk = T._Packs()
    xk = nhwc(x.detach()).to(DEV).to(BF)
    uk = T.convT2x2(xk, w.detach().to(DEV), b.detach().to(DEV), pk)
    close_bf16(nchw(uk), u)
    guk = nhwc(gu).to(DEV).to(BF)
    dxk = T.convT2x2_dgrad(guk, w.detach().to(DEV), pk, mask=xk)
    close_bf16(nchw(dxk), x.grad * (x > 0).float())
    dw, db = T.convT2x2_wgrad(xk, guk)
    close_f32(dw, w.grad)
    close_f32(db, b.grad)


def test_bf16_maxpool_outconv_convert():
    g = torch.Generator().manual_seed(9)
    x = rnd(2, 8, 8, 64, g=g).relu()
    x[:, 0:2, 0:2, :] = 0.5                      # ties: first max wins, as in fp32
    xb = x.to(DEV).to(BF)
    assert torch.equal(K.maxpool2_fwd(xb).float(), K.maxpool2_fwd(x.to(DEV)))
    dy = rnd(2, 4, 4, 64, g=g)
    dxb = torch.zeros_like(xb)
    K.maxpool2_bwd(xb, dy.to(DEV).to(BF), dxb, relu_mask=True, accumulate=True)
    dxf = torch.zeros(x.shape, device=DEV)
    K.maxpool2_bwd(x.to(DEV), dy.to(DEV), dxf, relu_mask=True, accumulate=True)
    assert torch.equal(dxb.float(), dxf)
    w = torch.randn(64, generator=g)
    bb = torch.randn(1, generator=g)
    close_f32(K.outconv_fwd(xb, w.to(DEV), bb.to(DEV)), K.outconv_fwd(x.to(DEV), w.to(DEV), bb.to(DEV)), rtol=1e-5)
    dl = torch.randn(2, 8, 8, generator=g)
    dxo, dwo, dbo = K.outconv_bwd(xb, w.to(DEV), dl.to(DEV))
    rx, rw, rbb = K.outconv_bwd(x.to(DEV), w.to(DEV), dl.to(DEV))
    close_bf16(dxo, rx)
    close_f32(dwo, rw, rtol=1e-5)
    close_f32(dbo, rbb, rtol=1e-5)
    y = torch.randn(1000, generator=g).to(DEV)
    assert torch.equal(K.to_f32(K.to_bf16(y)), y.to(BF).float())


def test_unetp_bf16_vs_fp64_oracle():
    """depth 4 / base 32 bf16 trunk, 2 slots at 64x64, oja: against the fp64 oracle."""
    torch.manual_seed(3)
    ref = oracle.RefUNetp(1, 1, rule="oja", nbf=64, depth=4, base_ch=32)
    net = UNetp(1, 1, DEV, rule="oja", nbf=64, depth=4, base_ch=32, precision="bf16")
    net.load_state_dict(ref.state_dict())
    g = torch.Generator().manual_seed(8)
    x = torch.rand(2, 1, 64, 64, generator=g)
    t = (torch.rand(2, 64, 64, generator=g) > 0.5).float()
    H = 0.05 * torch.randn(2, 64, 64, generator=g)
    y, hn = net(x.to(DEV), H.to(DEV))
    loss = bce_loss(y, t.to(DEV))
    loss.backward()
    ref = ref.double()
    yr, hr = ref(x.double(), H.double())
    lr_ = oracle.bce_loss(yr, t.double())
    lr_.backward()
    # measured: Y within 5e-6, loss within 1e-8 (the head and loss are fp32; the trunk's bf16
    # rounding reaches Y only through the small w + alpha*H product)
    assert (y.double().cpu() - yr).abs().max().item() < 5e-4
    assert (hn.double().cpu() - hr).abs().max().item() < 5e-4
    assert abs(loss.item() - lr_.item()) < 2e-4
    # trunk gradients: bf16 activations / activation gradients (2^-9 relative rounding per layer)
    # compound through the layers and flip near-zero ReLU masks - measured 0.02-0.16 relative L2
    # per tensor against fp64 (fp32 path: <1e-6); every kernel alone is at its rounding bound
    # (the kernel tests above)
    num = den = 0.0
    for (k, p), (_, pr) in zip(net.named_parameters(), ref.named_parameters()):
        if k == "eta":
            continue
        d = (p.grad.double().cpu() - pr.grad).norm().item()
        rel = d / max(pr.grad.norm().item(), 1e-30)
        assert rel < 0.25, (k, rel)
        num += d * d
        den += pr.grad.norm().item() ** 2
    assert (num / den) ** 0.5 < 0.15


@pytest.mark.parametrize("c0,cout", [(32, 64), (64, 64)])
def test_bf16_halo_conv_bit_identical_to_lean(c0, cout):
    """the register-staged halo kernel sums the same bf16 products in the same order as the per-tap lean kernel
    (unsplit at 8 x 128 x 128: 512 tiles), so forward and dgrad outputs are bit-identical"""
    B, H = 8, 128
    g = torch.Generator(device=DEV).manual_seed(c0 + cout)
    x = torch.randn(B, H, H, c0, device=DEV, generator=g).relu().to(BF)
    w = torch.randn(cout, c0, 3, 3, device=DEV, generator=g) * 0.05
    b = torch.randn(cout, device=DEV, generator=g)
    dz = torch.randn(B, H, H, cout, device=DEV, generator=g).to(BF)
    outs = []
    prev = K.set_conv_halo(1)
    try:
        for halo in (1, 0):               # register-staged halo kernel vs per-tap
            K.set_conv_halo(halo)
            pk = T._Packs()
            y = T.conv3x3(x, w, b, pk)
            d0, _ = T.conv3x3_dgrad(dz, w, pk, mask0=x)
            outs.append((y, d0))
    finally:
        K.set_conv_halo(prev)
    torch.cuda.synchronize()
    assert torch.equal(outs[0][0], outs[1][0])
    assert torch.equal(outs[0][1], outs[1][1])


@pytest.mark.parametrize("B,H,epi", [(8, 128, "relu"), (8, 128, "mask"), (8, 128, "resid"), (9, 128, "accum"),
                                     (8, 128, "plain"), (2, 128, "relu"), (2, 128, "mask")])
def test_bf16_rows_conv_bit_identical_to_lean(B, H, epi):
    """the row-stream kernel (128-wide 64 -> 64 3x3: weights resident in LDS, 16-row strips) sums
    the same bf16 products in the same order as the per-tap lean kernel: bit-identical outputs with
    every epilogue option (bias + ReLU, mask, residual, accumulate).  B >= 8 keeps the lean kernel
    unsplit (>= 512 tiles).  At B = 2 the lean plan splits K and adds its fp32 partial sums in
    another order, so the two bf16 outputs agree to within one bf16 rounding (2 ulp bound)."""
    from punet._lib import PU_PACK_CONV_FWD
    g = torch.Generator(device=DEV).manual_seed(H + B + len(epi))
    x = torch.randn(B, H, 128, 64, device=DEV, generator=g).to(BF)
    w = torch.randn(64, 64, 3, 3, device=DEV, generator=g) * 0.05
    b = torch.randn(64, device=DEV, generator=g)
    aux = torch.randn(B, H, 128, 64, device=DEV, generator=g).to(BF)
    outs = []
    prev = K.set_conv_halo(1)
    try:
        for halo in (1, 0):               # row-stream (the default route for this shape) vs per-tap
            K.set_conv_halo(halo)
            pk = T._Packs()
            wt = pk.get(w, PU_PACK_CONV_FWD, 576, 32, BF)
            out = aux.clone() if epi == "accum" else torch.empty_like(x)
            K.igemm(batch=B, in_hw=(H, 128), out_hw=(H, 128), k=3, stride=1, pad=1, src0=x, c0=64, weight=wt,
                    k_pad=576, n=64, dst0=out, bias=None if epi == "plain" else b, relu=epi == "relu",
                    mask0=aux if epi == "mask" else None, resid=aux if epi == "resid" else None,
                    accum=epi == "accum", cgroup=32)
            outs.append(out)
    finally:
        K.set_conv_halo(prev)
    torch.cuda.synchronize()
    if B >= 8:
        assert torch.equal(outs[0], outs[1])
    else:
        assert torch.allclose(outs[0].float(), outs[1].float(), rtol=2 ** -7, atol=2 ** -12)
        assert (outs[0] != outs[1]).float().mean().item() < 0.05
    ref = torch.nn.functional.conv2d(x.float().permute(0, 3, 1, 2), w.to(BF).float(), None if epi == "plain" else b,
                                     padding=1).permute(0, 2, 3, 1)
    if epi == "relu":
        ref = ref.relu()
    elif epi == "mask":
        ref = torch.where(aux.float() > 0, ref, torch.zeros_like(ref))
    elif epi in ("resid", "accum"):
        ref = ref + aux.float()
    assert torch.allclose(outs[0].float(), ref, rtol=2e-2, atol=2e-2)


@pytest.mark.parametrize("B,H", [(3, 16), (1, 48), (2, 112)])
def test_bf16_rows_conv_strip_edges(B, H):
    """the row-stream kernel on grids of 1, 3 and 7 16-row strips (first / last strip padding rows,
    a strip that is both): fwd (bias + ReLU) and dgrad (mask) within the bf16 bound of torch fp32 on
    the bf16-rounded operands"""
    g = torch.Generator(device=DEV).manual_seed(B * 1000 + H)
    x = torch.randn(B, H, 128, 64, device=DEV, generator=g).relu().to(BF)
    w = torch.randn(64, 64, 3, 3, device=DEV, generator=g) * 0.05
    b = torch.randn(64, device=DEV, generator=g)
    dz = torch.randn(B, H, 128, 64, device=DEV, generator=g).to(BF)
    pk = T._Packs()
    y = T.conv3x3(x, w, b, pk)
    d0, _ = T.conv3x3_dgrad(dz, w, pk, mask0=x)
    torch.cuda.synchronize()
    wb = w.to(BF).float()
    ref = F.conv2d(x.float().permute(0, 3, 1, 2), wb, b, padding=1).relu().permute(0, 2, 3, 1)
    refd = F.conv_transpose2d(dz.float().permute(0, 3, 1, 2), wb, padding=1).permute(0, 2, 3, 1)
    refd = torch.where(x.float() > 0, refd, torch.zeros_like(refd))
    for out, r in ((y, ref), (d0, refd)):
        err = (out.float() - r).abs().max().item()
        assert err <= 2e-2 * r.abs().max().item() + 1e-3, err


@pytest.mark.parametrize("B,H,c0,c1,cout", [(8, 128, 64, 0, 64), (4, 128, 32, 32, 128), (8, 64, 128, 0, 64),
                                            (16, 32, 64, 64, 192), (3, 32, 96, 0, 64)])
def test_bf16_halo2_conv_matches_fp32_and_halo1(B, H, c0, c1, cout):
    """the DMA-ring halo kernel (512-pixel row blocks, 16-channel stages, K order group/half/tap)
    sums the same exact bf16 products as the register-staged kernel in another order: fwd and
    dgrad outputs within 1 bf16 ulp of it, and within the bf16 tolerance of torch fp32 on the
    bf16-rounded operands"""
    g = torch.Generator(device=DEV).manual_seed(H + c0 + c1 + cout)
    x0 = torch.randn(B, H, H, c0, device=DEV, generator=g).relu().to(BF)
    x1 = torch.randn(B, H, H, c1, device=DEV, generator=g).relu().to(BF) if c1 else None
    w = torch.randn(cout, c0 + c1, 3, 3, device=DEV, generator=g) * 0.05
    b = torch.randn(cout, device=DEV, generator=g)
    dz = torch.randn(B, H, H, cout, device=DEV, generator=g).to(BF)
    outs = []
    prev = K.set_conv_halo(2)
    try:
        for halo in (2, 1):
            K.set_conv_halo(halo)
            pk = T._Packs()
            y = T.conv3x3(x0, w, b, pk, x1=x1)
            d0, d1 = T.conv3x3_dgrad(dz, w, pk, split=c0 if c1 else None, mask0=x0, mask1=x1)
            outs.append((y, d0, d1))
    finally:
        K.set_conv_halo(prev)
    torch.cuda.synchronize()
    for a, r in zip(outs[0], outs[1]):
        if a is None:
            continue
        diff = (a.float() - r.float()).abs()
        # one bf16 ulp (8-bit significand) of the larger of the two - a sum within fp32 noise of a
        # rounding midpoint rounds up in one order and down in the other - plus the fp32
        # accumulation noise of a cancelling sum (results near 1e-6 from terms near 0.05)
        ulp = torch.maximum(a.float().abs(), r.float().abs()) * 2.0 ** -7
        assert bool((diff <= ulp + 1e-4).all()), diff.max().item()
    xc = torch.cat([x0, x1], 3) if c1 else x0
    ref = torch.relu(F.conv2d(nchw(xc.float()), rb(w), b, padding=1))
    close_bf16(nchw(outs[0][0]), ref)


def test_bf16_stem_direct_output_and_bf16_rows_wgrad_bitwise():
    """The bf16 trunk's single-channel stem writes its bf16 output directly (PU_EPI_OUT_BF16) and
    its weight gradient reads the bf16 dZ (pu_wgrad math 2): bit for bit what the fp32 output +
    conversion pass and the converted fp32 dZ gave (round-to-nearest-even once; bf16 -> fp32 is
    exact).  Full model forward + backward both ways, then the flag's misuse fails loudly."""
    res = []
    for fused in (True, False):
        orig = T.UNetpTrunk._stem_bf16
        if not fused:
            T.UNetpTrunk._stem_bf16 = lambda self, x: False
        try:
            torch.manual_seed(3)
            net = UNetp(1, 1, DEV, rule="oja", nbf=64, depth=4, base_ch=32, precision="bf16")
            g = torch.Generator().manual_seed(8)
            x = torch.rand(4, 1, 64, 64, generator=g).to(DEV)
            t = (torch.rand(4, 64, 64, generator=g) > 0.5).float().to(DEV)
            H = (0.05 * torch.randn(4, 64, 64, generator=g)).to(DEV)
            y, hn = net(x, H)
            bce_loss(y, t).backward()
            res.append((y.detach(), hn.detach(), {k: p.grad.detach().clone() for k, p in net.named_parameters()
                                                  if p.grad is not None}))
        finally:
            T.UNetpTrunk._stem_bf16 = orig
    assert torch.equal(res[0][0], res[1][0]) and torch.equal(res[0][1], res[1][1])
    for k in res[0][2]:
        assert torch.equal(res[0][2][k], res[1][2][k]), k
    # PU_EPI_OUT_BF16 on anything but the single-channel stem is an argument error
    x = torch.rand(1, 8, 8, 16, device=DEV)
    w = torch.randn(16, 16, 3, 3, device=DEV)
    pk = K.pack_weight(w, 0, 16 * 9)
    with pytest.raises(RuntimeError, match="PU_EPI_OUT_BF16"):
        K.igemm(batch=1, in_hw=(8, 8), out_hw=(8, 8), k=3, stride=1, pad=1, src0=x, c0=16, weight=pk, k_pad=16 * 9,
                n=16, dst0=torch.empty(1, 8, 8, 16, dtype=torch.bfloat16, device=DEV), relu=True)
