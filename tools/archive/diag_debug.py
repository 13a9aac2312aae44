"""Per-layer backward tensors (trunk.debug) of UNetp(bn, bilinear) with the small-channel MFMA
kernel off / on: where do they part?"""
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
xs = torch.from_numpy(np.asarray(g["xs"])); H0 = torch.from_numpy(np.asarray(g["hebb"])); t = torch.from_numpy(np.asarray(g["t"]))
dbg = {}
for on in (False, True):
    K.set_smallx6(on)
    net = UNetp(1, 1, DEV, rule="oja", nbf=64, batch_norm=True, bilinear_upsample=True)
    net.load_state_dict(sd); net.train()
    tr = net._trunk_plan()
    tr.debug = {}
    y, _ = net(xs[0].to(DEV), H0.to(DEV))
    bce_loss(y, t.to(DEV)).backward()
    dbg[on] = {k: v.detach().double().cpu() for k, v in tr.debug.items() if v is not None}
for k in dbg[False]:
    a, b = dbg[False][k], dbg[True][k]
    print("%-12s %-22s rel diff %.2e" % (k, tuple(a.shape), (a - b).abs().max().item() / max(a.abs().max().item(), 1e-30)))
