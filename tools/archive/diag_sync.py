"""UNetp(bn, bilinear) up4.conv.conv.0 weight-gradient error vs the golden, small-channel MFMA on,
with and without a device synchronisation after every library call (race test)."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "plastic-unet_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np
import torch
from unet import UNetp
from punet import bce_loss
from punet import kernels as K
from punet import _lib
from conftest import golden
DEV = torch.device("cuda")
g = golden("unetp_bn_bilinear.npz")
sd = {k[2:]: torch.from_numpy(np.asarray(v)) for k, v in g.items() if k.startswith("p.")}
xs = torch.from_numpy(np.asarray(g["xs"])); H0 = torch.from_numpy(np.asarray(g["hebb"])); tt = torch.from_numpy(np.asarray(g["t"]))
L = _lib.load()
def run(tag):
    net = UNetp(1, 1, DEV, rule="oja", nbf=64, batch_norm=True, bilinear_upsample=True)
    net.load_state_dict(sd); net.train()
    y, _ = net(xs[0].to(DEV), H0.to(DEV))
    bce_loss(y, tt.to(DEV)).backward()
    torch.cuda.synchronize()
    for k in ("up4.conv.conv.0.weight", "inc.conv.conv.0.weight"):
        p = dict(net.named_parameters())[k]
        ref = torch.from_numpy(np.asarray(g["g." + k])).reshape(p.shape)
        print("%-8s %-26s rel err %.2e" % (tag, k, (p.grad.cpu() - ref).abs().max().item() / ref.abs().max().item()))
K.set_smallx6(True)
run("async")
names = [n for n, _, _ in _lib.SIGNATURES if n not in ("pu_last_error", "pu_abi_version", "pu_build_id")]
for n in names:
    f = getattr(L, n)
    def wrap(*a, f=f):
        r = f(*a)
        torch.cuda.synchronize()
        return r
    setattr(L, n, wrap)
run("synced")
K.set_smallx6(False)
run("direct")
