"""Diagnose the bf16 DMA-ring halo conv (fwd + dgrad) against the register-staged one and torch fp32."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "plastic-unet_amd"))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402
from punet import kernels as K  # noqa: E402
from punet import trunk as T  # noqa: E402

DEV = torch.device("cuda")
BF = torch.bfloat16
for (B, H, c0, c1, cout) in [(8, 128, 64, 0, 64), (2, 32, 64, 0, 64)]:
    g = torch.Generator(device=DEV).manual_seed(H + c0 + c1 + cout)
    x0 = torch.randn(B, H, H, c0, device=DEV, generator=g).relu().to(BF)
    w = torch.randn(cout, c0 + c1, 3, 3, device=DEV, generator=g) * 0.05
    b = torch.randn(cout, device=DEV, generator=g)
    dz = torch.randn(B, H, H, cout, device=DEV, generator=g).to(BF)
    wb = w.to(BF).float()
    yref = F.conv2d(x0.float().permute(0, 3, 1, 2), wb, b, padding=1).relu().permute(0, 2, 3, 1)
    dref = F.conv_transpose2d(dz.float().permute(0, 3, 1, 2), wb, padding=1).permute(0, 2, 3, 1) * (x0.float() > 0)
    res = {}
    for halo in (2, 1, 0):
        K.set_conv_halo(halo)
        pk = T._Packs()
        y = T.conv3x3(x0, w, b, pk).float()
        d0, _ = T.conv3x3_dgrad(dz, w, pk, mask0=x0)
        res[halo] = (y, d0.float())
    torch.cuda.synchronize()
    for k, (name, ref) in enumerate((("fwd", yref), ("dgrad", dref))):
        for halo in (2, 1, 0):
            d = (res[halo][k] - ref).abs()
            print("B%d H%d %s halo%d: max|d - fp32| %.4g at %s (ref %.6g got %.6g)" % (
                B, H, name, halo, d.max().item(), list(torch.unravel_index(d.argmax(), d.shape)),
                ref.flatten()[d.argmax()].item(), res[halo][k].flatten()[d.argmax()].item()))
        a, r = res[2][k], res[1][k]
        dd = (a - r).abs()
        i = dd.argmax()
        print("   halo2 vs halo1 max %.4g at %s: halo2 %.6g halo1 %.6g fp32 %.6g; #diff %d" % (
            dd.max().item(), [int(v) for v in torch.unravel_index(i, dd.shape)], a.flatten()[i].item(),
            r.flatten()[i].item(), ref.flatten()[i].item(), (dd > 0).sum().item()))
        ulp = torch.maximum(a.abs(), r.abs()) * 2.0 ** -7
        bad = (dd > ulp).nonzero()
        for q in bad[:6].tolist():
            print("      >1ulp at", q, "halo2 %.8g halo1 %.8g fp32 %.8g" % (a[tuple(q)].item(), r[tuple(q)].item(),
                                                                         ref[tuple(q)].item()))
K.set_conv_halo(2)
