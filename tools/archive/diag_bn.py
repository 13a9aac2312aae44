"""bn_bwd of up4.c0 in UNetp(bn, bilinear) with the small-channel MFMA kernel off / on: the GPU
result vs an fp64 CPU BatchNorm backward of the same inputs, and the input differences."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "plastic-unet_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np
import torch
from unet import UNetp
from punet import bce_loss
from punet import kernels as K
from conftest import golden
DEV = torch.device("cuda")
g = golden("unetp_bn_bilinear.npz")
sd = {k[2:]: torch.from_numpy(np.asarray(v)) for k, v in g.items() if k.startswith("p.")}
xs = torch.from_numpy(np.asarray(g["xs"])); H0 = torch.from_numpy(np.asarray(g["hebb"])); tt = torch.from_numpy(np.asarray(g["t"]))
orig = K.bn_bwd
res = {}
for on in (False, True):
    K.set_smallx6(on)
    calls = []
    def rec(z, gg, mean, rstd, gamma, dgam, dbet, **kw):
        out = orig(z, gg, mean, rstd, gamma, dgam, dbet, **kw)
        torch.cuda.synchronize()
        calls.append([t.detach().double().cpu() for t in (z, gg, mean, rstd, gamma, out, dgam, dbet)])
        return out
    K.bn_bwd = rec
    import punet.trunk as T
    T.K.bn_bwd = rec
    net = UNetp(1, 1, DEV, rule="oja", nbf=64, batch_norm=True, bilinear_upsample=True)
    net.load_state_dict(sd); net.train()
    y, _ = net(xs[0].to(DEV), H0.to(DEV))
    bce_loss(y, tt.to(DEV)).backward()
    torch.cuda.synchronize()
    res[on] = calls
    K.bn_bwd = orig
    T.K.bn_bwd = orig
for i in range(min(4, len(res[False]))):
    a, b = res[False][i], res[True][i]
    names = ("z", "g", "mean", "rstd", "gamma", "dz", "dgam", "dbet")
    diffs = ["%s %.1e" % (n, (x - y).abs().max().item() / max(x.abs().max().item(), 1e-30)) for n, x, y in zip(names, a, b)]
    # fp64 reference BN backward per slot on each run's own inputs
    for tag, c in (("off", a), ("on", b)):
        z, gg, mean, rstd, gamma, dz = c[:6]
        B, H, W, C = z.shape
        zz = z.reshape(B, H * W, C)
        m = zz.mean(1, keepdim=True); v = ((zz - m) ** 2).mean(1, keepdim=True)
        rs = 1.0 / torch.sqrt(v + 1e-5)
        xh = (zz - m) * rs
        gg2 = gg.reshape(B, H * W, C)
        dref = rs * gamma * (gg2 - gg2.mean(1, keepdim=True) - xh * (gg2 * xh).mean(1, keepdim=True))
        e = (dz.reshape(B, H * W, C) - dref).abs().max().item() / dref.abs().max().item()
        diffs.append("%s-vs-fp64 %.1e (|dz| %.1e, |g| %.1e, rstd max %.1e)" % (tag, e, dref.abs().max().item(), gg.abs().max().item(), rs.max().item()))
    print(i, "  ".join(diffs))
