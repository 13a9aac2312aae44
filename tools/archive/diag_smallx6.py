"""smallconv_x6 vs the VALU direct kernel on the UNetp(bilinear) up4 shapes: outputs and
whether any input / guard memory changed."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "plastic-unet_amd"))
import torch
from punet import kernels as K
from punet import trunk as T
dev = "cuda"
torch.manual_seed(0)
for (B, H, W, c0, c1, n) in [(1, 64, 64, 8, 8, 8), (1, 64, 64, 8, 0, 8), (1, 32, 32, 16, 16, 16), (1, 32, 32, 8, 8, 16)]:
    big = torch.randn(B * H * W * (c0 + c1 + n) * 4 + 4096, device=dev)
    x0 = big[:B * H * W * c0].view(B, H, W, c0).relu()
    x1 = big[B * H * W * c0: B * H * W * (c0 + c1)].view(B, H, W, c1).relu() if c1 else None
    guard = big.clone()
    w = torch.randn(n, c0 + c1, 3, 3, device=dev) * 0.2
    b = torch.randn(n, device=dev)
    dz = torch.randn(B, H, W, n, device=dev)
    res = {}
    for on in (False, True):
        K.set_smallx6(on)
        pk = T._Packs()
        y = T.conv3x3(x0, w, b, pk, x1=x1, relu=True)
        d0, d1 = T.conv3x3_dgrad(dz, w, pk, split=c0 if c1 else None, mask0=x0, mask1=x1)
        torch.cuda.synchronize()
        res[on] = (y.clone(), d0.clone(), None if d1 is None else d1.clone())
        assert torch.equal(big, guard), "inputs modified (smallx6=%s)" % on
    for a, bb, nm in zip(res[False], res[True], ("fwd", "dgrad0", "dgrad1")):
        if a is None:
            continue
        err = (a - bb).abs().max().item() / max(a.abs().max().item(), 1e-30)
        print((B, H, W, c0, c1, n), nm, "rel err %.2e" % err)
