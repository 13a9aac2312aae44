"""Winograd F(2x2,3x3) path of the fp32 3x3 convolutions (csrc/winograd.hip) against fp64.

The Winograd kernel does not reproduce the direct kernel's summation order, so it is judged the
way tests/test_precision_gpu.py judges every conv kernel: its max error relative to max|ref|
against the fp64 result, next to ATen's CPU fp32 error on the same op (bound: max(16 x CPU, 4e-6)),
plus rtol 1e-4 parity with CPU fp32 and bitwise run-to-run determinism.  Cases cover the epilogue
variants the U-Net uses (bias + ReLU, residual, ReLU masks, the concat split of the data
gradient, accumulate), the skip concat as two sources, partial tile blocks, non-square and
many-image grids, and the split-K plan of the 8x8 / 16x16 levels."""
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


def rel_err(got, ref):
    got = got.detach().double().cpu()
    return (got - ref).abs().max().item() / ref.abs().max().item()


def check(name, got, cpu32, ref64):
    eg, ec = rel_err(got, ref64), rel_err(cpu32, ref64)
    print("%-34s wino %.2e  cpu32 %.2e" % (name, eg, ec))
    assert eg <= max(16 * ec, 4e-6), (name, eg, ec)
    torch.testing.assert_close(got.detach().float().cpu(), cpu32.float(), rtol=1e-4,
                               atol=1e-5 * cpu32.abs().max().item())


CASES = [
    # B, H, W, c0, c1, cout
    (2, 16, 16, 64, 0, 64),       # one block of 64 tiles x 2 images
    (3, 10, 14, 128, 0, 128),     # 105 tiles: a partial second tile block, 2 channel blocks, non-square
    (2, 8, 8, 64, 64, 64),        # concat (two sources), every tile on an image edge
    (1, 32, 16, 128, 0, 192),     # 3 channel blocks, 8 chunks
    (4, 8, 8, 512, 0, 512),       # split-K (bottom level shape): 64 tiles, 8 channel blocks
    (2, 16, 16, 256, 256, 256),   # split-K with two sources (the 16x16 up level)
    (1, 2, 2, 32, 0, 64),         # a single 2x2 tile
    # > 256 items: the persistent kernel (items streamed per block, next-item prefetch during the
    # epilogue, per-XCD item ranges)
    (5, 128, 128, 64, 0, 64),     # 320 items, 40 per XCD
    (3, 96, 80, 128, 0, 192),     # 270 items: ragged per-XCD ranges (270 % 8 = 6), 3 channel blocks
    # n % 128 == 0 shapes (the 128-channel items under PU_WINO128=1 - test_wino128_bit_identical_..)
    (2, 16, 16, 128, 0, 256),     # 2 channel blocks of 128
    (5, 128, 128, 64, 0, 128),    # 64 -> 128 (direct before 128-channel items), 640 items, persistent
    (7, 96, 80, 128, 0, 128),     # 420 items: ragged per-XCD ranges (420 % 8 = 4)
    (2, 24, 24, 64, 64, 64),      # its data gradient: 64 -> 128 split at 64 (the top concat layer)
]


@pytest.mark.parametrize("B,H,W,c0,c1,cout", CASES)
def test_wino_fwd_dgrad_vs_fp64(B, H, W, c0, c1, cout):
    g = torch.Generator().manual_seed(B * 131 + H * 7 + W + c0 + 3 * c1 + cout)
    C = c0 + c1
    x = torch.randn(B, C, H, W, generator=g).relu()
    w = torch.randn(cout, C, 3, 3, generator=g) * (2.0 / (9 * C)) ** 0.5
    b = torch.randn(cout, generator=g) * 0.1
    dz = torch.randn(B, cout, H, W, generator=g) * (torch.rand(B, cout, H, W, generator=g) > 0.5).float()
    ref = {}
    for dt in (torch.float32, torch.float64):
        xr = x.detach().to(dt).clone().requires_grad_(True)
        z = F.conv2d(xr, w.to(dt), b.to(dt), padding=1)
        z.backward(dz.to(dt))
        ref[dt] = (torch.relu(z).detach(), (xr.grad * (x > 0).to(dt)).detach())
    prev = K.set_wino(True)
    try:
        pk = T._Packs()
        xk = nhwc(x).to(DEV)
        x0, x1 = (xk[..., :c0].contiguous(), xk[..., c0:].contiguous()) if c1 else (xk, None)
        wk = w.to(DEV)
        assert (getattr(pk.get(wk, 0, K.round16(9 * C), K.cgroup_for(c0, c1)), "_wino", None) is not None) \
            == K.wino_wanted(wk, 0)
        y = T.conv3x3(x0, wk, b.to(DEV), pk, x1=x1, relu=True)
        check("wino fwd %dx%dx%d %d+%d->%d" % (B, H, W, c0, c1, cout), nchw(y), ref[torch.float32][0],
              ref[torch.float64][0])
        y2 = T.conv3x3(x0, wk, b.to(DEV), pk, x1=x1, relu=True)
        assert torch.equal(y, y2), "Winograd forward is not deterministic"
        dzk = nhwc(dz).to(DEV)
        d0, d1 = T.conv3x3_dgrad(dzk, wk, pk, split=c0 if c1 else None, mask0=x0, mask1=x1)
        dx = torch.cat([d0, d1], 3) if c1 else d0
        assert (getattr(pk.get(wk, 1, K.round16(9 * cout), K.cgroup_for(cout)), "_wino", None) is not None) \
            == K.wino_wanted(wk, 1)
        check("wino dgrad", nchw(dx), ref[torch.float32][1], ref[torch.float64][1])
    finally:
        K.set_wino(prev)


def test_wino_resid_and_accumulate_epilogues():
    """RESID (the residual add before the ReLU) and ACCUM through the Winograd epilogue, against
    the direct kernel on the same layer (both within fp32 rounding of each other)."""
    g = torch.Generator().manual_seed(11)
    B, H, W, C, N = 2, 12, 8, 64, 64
    x = torch.randn(B, H, W, C, generator=g).to(DEV)
    w = (torch.randn(N, C, 3, 3, generator=g) * 0.05).to(DEV)
    b = torch.randn(N, generator=g).to(DEV)
    r = torch.randn(B, H, W, N, generator=g).to(DEV)
    acc0 = torch.randn(B, H, W, N, generator=g).to(DEV)
    outs = {}
    for on in (True, False):
        prev = K.set_wino(on)
        try:
            pk = T._Packs()
            k_pad = K.round16(9 * C)
            packed = pk.get(w, 0, k_pad, K.cgroup_for(C))
            assert (getattr(packed, "_wino", None) is not None) == on or not on
            o1 = torch.empty(B, H, W, N, device=DEV)
            K.igemm(batch=B, in_hw=(H, W), out_hw=(H, W), k=3, stride=1, pad=1, src0=x, c0=C, weight=packed,
                    k_pad=k_pad, n=N, bias=b, dst0=o1, relu=True, resid=r, cgroup=K.cgroup_for(C))
            o2 = acc0.clone()
            K.igemm(batch=B, in_hw=(H, W), out_hw=(H, W), k=3, stride=1, pad=1, src0=x, c0=C, weight=packed,
                    k_pad=k_pad, n=N, dst0=o2, accum=True, cgroup=K.cgroup_for(C))
            outs[on] = (o1.cpu(), o2.cpu())
        finally:
            K.set_wino(prev)
    for a, bb in zip(outs[True], outs[False]):
        torch.testing.assert_close(a, bb, rtol=1e-5, atol=2e-5 * bb.abs().max().item())


def test_pack_wino_is_G_g_Gt_split_exactly():
    """pu_pack_wino: each (position, n, c) is G g G^T formed in fp64, rounded to fp32, split into
    hi/mid/lo bf16 that sum back to it exactly; forward and the flipped/transposed dgrad kernel."""
    g = torch.Generator().manual_seed(3)
    cout, cin = 64, 32
    w = torch.randn(cout, cin, 3, 3, generator=g, dtype=torch.float64).float()
    G = torch.tensor([[1, 0, 0], [.5, .5, .5], [.5, -.5, .5], [0, 0, 1]], dtype=torch.float64)
    for dgrad in (0, 1):
        n, c = (cout, cin) if not dgrad else (cin, cout)
        gk = w.double() if not dgrad else w.double().transpose(0, 1).flip(2, 3)   # [n][c][3][3]
        U = torch.einsum("ar,ncrs,bs->abnc", G, gk, G).reshape(16, n, c).float()
        out = torch.empty(K.lib().pu_wino_bytes(n, c) // 2, dtype=torch.bfloat16, device=DEV)
        K.pack_wino([(w.to(DEV), out, dgrad)])
        planes = out.cpu().float().reshape(c // 16, 16, 3, n, 16)       # [chunk][xi][plane][n][c16]
        got = planes.permute(1, 2, 3, 0, 4).reshape(16, 3, n, c)
        assert torch.equal(got[:, 0] + got[:, 1] + got[:, 2], U), dgrad
        assert torch.equal(got[:, 0], U.bfloat16().float())


_PERSIST_SCRIPT = r"""
import sys, torch
sys.path.insert(0, sys.argv[2])
from punet import kernels as K, trunk as T
B, H, W, C, N = 5, 128, 128, 64, 64
g = torch.Generator().manual_seed(77)
x = torch.randn(B, H, W, C, generator=g).relu().cuda()
w = (torch.randn(N, C, 3, 3, generator=g) * 0.06).cuda()
b = torch.randn(N, generator=g).cuda()
dz = torch.randn(B, H, W, N, generator=g).cuda()
pk = T._Packs()
y = T.conv3x3(x, w, b, pk, relu=True)
d0, _ = T.conv3x3_dgrad(dz, w, pk, mask0=x)
torch.save({"y": y.cpu(), "d": d0.cpu()}, sys.argv[1])
"""


def test_wino_persistent_equals_one_item_per_block(tmp_path):
    """The persistent kernel (320 items on 256 blocks) and the one-item-per-block launch
    (PU_WINO_PERSIST=0, read once per process - hence two child processes) form the same per-item
    sums in the same order: forward and data gradient bit-identical."""
    import os
    import subprocess
    import sys
    root = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "plastic-unet_amd")
    out = {}
    for persist in ("1", "0"):
        f = str(tmp_path / ("p%s.pt" % persist))
        env = dict(os.environ, PU_WINO_PERSIST=persist, PU_WINO="1", PU_WINO4="0")   # the 8-wave kernel's modes
        r = subprocess.run([sys.executable, "-c", _PERSIST_SCRIPT, f, root], env=env, capture_output=True,
                           text=True, timeout=300)
        assert r.returncode == 0, r.stderr[-2000:]
        out[persist] = torch.load(f, weights_only=True)
    assert torch.equal(out["1"]["y"], out["0"]["y"])
    assert torch.equal(out["1"]["d"], out["0"]["d"])


WGRAD_CASES = [
    # B, H, W, c0, c1, cout
    (2, 16, 16, 64, 0, 64),       # one channel block; 8x8 tile grid (a 16-tile stage spans 2 tile rows)
    (3, 10, 14, 128, 0, 128),     # 105 tiles: a ragged last stage, 2 x 2 channel blocks, non-square
    (2, 8, 8, 64, 64, 64),        # concat (two sources), every tile on an image edge
    (1, 32, 16, 128, 0, 192),     # 3 output blocks
    (4, 8, 8, 512, 0, 512),       # 64 channel blocks x 4 splits (the bottom level)
    (2, 16, 16, 256, 256, 256),   # two 256-channel sources, 8 x 4 blocks
    (8, 64, 64, 64, 0, 64),       # 256 splits of 32 tiles (the top level's shape at bs 8)
    (1, 2, 2, 64, 0, 64),         # a single tile
]


@pytest.mark.parametrize("B,H,W,c0,c1,cout", WGRAD_CASES)
def test_wino_wgrad_vs_fp64(B, H, W, c0, c1, cout):
    """wgrad_wino_x6_kernel (dW = G^T [sum_tiles (A e A^T)(.)(B^T d B)] G, bias as dZ column sums)
    against fp64, next to ATen's CPU fp32 error; bitwise run-to-run determinism; and the kernel
    really is the one dispatched (pu_wgrad_tile kind 5)."""
    g = torch.Generator().manual_seed(B * 17 + H * 5 + W + c0 + 7 * c1 + cout)
    C = c0 + c1
    x = torch.randn(B, C, H, W, generator=g).relu()
    dz = torch.randn(B, cout, H, W, generator=g) * (torch.rand(B, cout, H, W, generator=g) > 0.3).float()
    ref = {}
    for dt in (torch.float32, torch.float64):
        ref[dt] = (torch.nn.grad.conv2d_weight(x.to(dt), (cout, C, 3, 3), dz.to(dt), padding=1),
                   dz.to(dt).sum((0, 2, 3)))
    xk = nhwc(x).to(DEV)
    x0, x1 = (xk[..., :c0].contiguous(), xk[..., c0:].contiguous()) if c1 else (xk, None)
    dzk = nhwc(dz).to(DEV)
    assert K.wgrad_kind(batch=B, hw=(H, W), n=cout, c0=c0, c1=c1) == 5
    dw, db = T.conv3x3_wgrad(dzk, x0, x1)
    check("wino wgrad %dx%dx%d %d+%d->%d" % (B, H, W, c0, c1, cout), dw, ref[torch.float32][0], ref[torch.float64][0])
    check("wino bias grad", db, ref[torch.float32][1], ref[torch.float64][1])
    dw2, db2 = T.conv3x3_wgrad(dzk, x0, x1)
    assert torch.equal(dw, dw2) and torch.equal(db, db2), "Winograd weight gradient is not deterministic"


_W128_SCRIPT = r"""
import sys, torch
sys.path.insert(0, sys.argv[2])
from punet import kernels as K, trunk as T
out = {}
for (B, H, W, c0, c1, N) in [(3, 32, 24, 128, 0, 128), (2, 16, 16, 256, 0, 256), (2, 32, 32, 128, 128, 128),
                             (4, 8, 8, 512, 0, 512), (9, 64, 64, 128, 0, 128)]:
    g = torch.Generator().manual_seed(B + H + c0 + c1 + N)
    C = c0 + c1
    x = torch.randn(B, H, W, C, generator=g).relu().cuda()
    w = (torch.randn(N, C, 3, 3, generator=g) * 0.05).cuda()
    b = torch.randn(N, generator=g).cuda()
    dz = torch.randn(B, H, W, N, generator=g).cuda()
    pk = T._Packs()
    x0, x1 = (x[..., :c0].contiguous(), x[..., c0:].contiguous()) if c1 else (x, None)
    y = T.conv3x3(x0, w, b, pk, x1=x1, relu=True)
    d0, d1 = T.conv3x3_dgrad(dz, w, pk, split=c0 if c1 else None, mask0=x0, mask1=x1)
    out[(B, H, W, c0, c1, N)] = (y.cpu(), d0.cpu(), None if d1 is None else d1.cpu())
torch.save(out, sys.argv[1])
"""


def test_wino128_bit_identical_to_64_channel_items(tmp_path):
    """32-tile x 128-channel Winograd items (wino128_x6_kernel) and 64 x 64 items (PU_WINO128=0,
    read once per process - two child processes) feed every accumulator the same U / V fragments
    in the same MFMA order, then the same output transform: forward and data gradient bitwise equal
    on the layers both take (n % 128 == 0, C >= 128; split-K, concat sources, split outputs,
    persistent item streams)."""
    import os
    import subprocess
    import sys
    root = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "plastic-unet_amd")
    res = {}
    for on in ("1", "0"):
        f = str(tmp_path / ("w%s.pt" % on))
        env = dict(os.environ, PU_WINO4="0", PU_WINO128=on, PU_WINO="1")
        r = subprocess.run([sys.executable, "-c", _W128_SCRIPT, f, root], env=env, capture_output=True, text=True,
                           timeout=300)
        assert r.returncode == 0, r.stderr[-2000:]
        res[on] = torch.load(f, weights_only=True)
    for k in res["1"]:
        for a, b in zip(res["1"][k], res["0"][k]):
            assert (a is None) == (b is None), k
            if a is not None:
                assert torch.equal(a, b), k


_W4_SCRIPT = r"""
import sys, torch
sys.path.insert(0, sys.argv[2])
from punet import kernels as K, trunk as T
out = {}
for (B, H, W, c0, c1, N) in [(2, 16, 16, 64, 0, 64), (3, 10, 14, 128, 0, 128), (2, 8, 8, 64, 64, 64),
                             (1, 32, 16, 128, 0, 192), (4, 8, 8, 512, 0, 512), (2, 16, 16, 256, 256, 256),
                             (1, 2, 2, 32, 0, 64), (5, 128, 128, 64, 0, 64), (3, 96, 80, 128, 0, 192),
                             (2, 24, 24, 128, 128, 128), (2, 24, 24, 64, 64, 64), (3, 16, 16, 64, 0, 128)]:
    g = torch.Generator().manual_seed(B + H + W + c0 + c1 + N)
    C = c0 + c1
    x = torch.randn(B, H, W, C, generator=g).relu().cuda()
    w = (torch.randn(N, C, 3, 3, generator=g) * 0.05).cuda()
    b = torch.randn(N, generator=g).cuda()
    dz = torch.randn(B, H, W, N, generator=g).cuda()
    r = torch.randn(B, H, W, N, generator=g).cuda()
    a0 = torch.randn(B, H, W, N, generator=g).cuda()
    pk = T._Packs()
    x0, x1 = (x[..., :c0].contiguous(), x[..., c0:].contiguous()) if c1 else (x, None)
    y = T.conv3x3(x0, w, b, pk, x1=x1, relu=True)
    d0, d1 = T.conv3x3_dgrad(dz, w, pk, split=c0 if c1 else None, mask0=x0, mask1=x1)
    res = [y.cpu(), d0.cpu(), None if d1 is None else d1.cpu()]
    if not c1:     # the general epilogue: residual + ReLU, accumulate
        k_pad = K.round16(9 * C)
        packed = pk.get(w, 0, k_pad, K.cgroup_for(C))
        o1 = torch.empty(B, H, W, N, device="cuda")
        K.igemm(batch=B, in_hw=(H, W), out_hw=(H, W), k=3, stride=1, pad=1, src0=x, c0=C, weight=packed,
                k_pad=k_pad, n=N, bias=b, dst0=o1, relu=True, resid=r, cgroup=K.cgroup_for(C))
        o2 = a0.clone()
        K.igemm(batch=B, in_hw=(H, W), out_hw=(H, W), k=3, stride=1, pad=1, src0=x, c0=C, weight=packed,
                k_pad=k_pad, n=N, dst0=o2, accum=True, cgroup=K.cgroup_for(C))
        res += [o1.cpu(), o2.cpu()]
    out[(B, H, W, c0, c1, N)] = res
torch.save(out, sys.argv[1])
"""


def test_wino4_bit_identical_to_8_wave_kernel(tmp_path):
    """wino4_x6_kernel (one wave per SIMD, 2 x 2 or 4 x 1 MFMA blocks per position - 64 x 64 or, for
    n % 128 == 0, 32-tile x 128-channel items -, U from L2 into registers) and wino_x6_kernel
    (PU_WINO4=0; read once per process - two child processes) form
    every accumulator from the same U / V planes in the same product order and run the same
    output-transform expression tree: forward, data gradient (masks, concat split), residual and
    accumulate epilogues bitwise equal - one and many items per block, split-K, concat sources,
    ragged tile blocks."""
    import os
    import subprocess
    import sys
    root = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "plastic-unet_amd")
    res = {}
    # (PU_WINO4, PU_WINO4_WIDE, PU_WINO128): the short-reduction concat data gradients take the
    # direct kernel in "100" / "000" and 128-channel Winograd items in the others
    for on in ("100", "000", "110", "120", "001"):
        f = str(tmp_path / ("w%s.pt" % on))
        env = dict(os.environ, PU_WINO4=on[0], PU_WINO4_WIDE=on[1], PU_WINO128=on[2], PU_WINO="1")
        r = subprocess.run([sys.executable, "-c", _W4_SCRIPT, f, root], env=env, capture_output=True, text=True,
                           timeout=300)
        assert r.returncode == 0, r.stderr[-2000:]
        res[on] = torch.load(f, weights_only=True)
    for v, ref in (("100", "000"), ("110", "001"), ("120", "001")):
        for k in res[v]:
            for i, (a, b) in enumerate(zip(res[v][k], res[ref][k])):
                assert (a is None) == (b is None), k
                if a is not None:
                    assert torch.equal(a, b), (v, k, i, (a - b).abs().max().item())


_WW4_SCRIPT = r"""
import sys, torch
sys.path.insert(0, sys.argv[2])
from punet import kernels as K, trunk as T
out = {}
for (B, H, W, c0, c1, N) in [(2, 16, 16, 64, 0, 64), (3, 10, 14, 128, 0, 128), (2, 8, 8, 64, 64, 64),
                             (1, 32, 16, 128, 0, 192), (4, 8, 8, 512, 0, 512), (2, 16, 16, 256, 256, 256),
                             (8, 64, 64, 64, 0, 64), (1, 2, 2, 64, 0, 64)]:
    g = torch.Generator().manual_seed(B + H + W + c0 + c1 + N)
    C = c0 + c1
    x = torch.randn(B, H, W, C, generator=g).relu().cuda()
    dz = (torch.randn(B, H, W, N, generator=g) * (torch.rand(B, H, W, N, generator=g) > 0.3).float()).cuda()
    x0, x1 = (x[..., :c0].contiguous(), x[..., c0:].contiguous()) if c1 else (x, None)
    dw, db = T.conv3x3_wgrad(dz, x0, x1)
    out[(B, H, W, c0, c1, N)] = (dw.cpu(), db.cpu())
torch.save(out, sys.argv[1])
"""


def test_wgrad_wino4_bit_identical_to_8_wave_kernel(tmp_path):
    """wgrad_wino4_x6_kernel (one wave per SIMD, 2 x 2 channel blocks per position, 4-channel
    producer threads, a 4-wave R exchange in the output transform; PU_WW4=1) and
    wgrad_wino_x6_kernel form the same planes, run the same 6 products per accumulator in the same
    order and the same G^T M G expression tree: weight and bias gradients bitwise equal - ragged
    stages, concat sources, several channel blocks, split slabs, a single tile."""
    import os
    import subprocess
    import sys
    root = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "plastic-unet_amd")
    res = {}
    for on in ("1", "0"):
        f = str(tmp_path / ("ww%s.pt" % on))
        env = dict(os.environ, PU_WW4=on)
        r = subprocess.run([sys.executable, "-c", _WW4_SCRIPT, f, root], env=env, capture_output=True, text=True,
                           timeout=300)
        assert r.returncode == 0, r.stderr[-2000:]
        res[on] = torch.load(f, weights_only=True)
    for k in res["1"]:
        for i, (a, b) in enumerate(zip(res["1"][k], res["0"][k])):
            assert torch.equal(a, b), (k, i, (a - b).abs().max().item())
