"""UNetp(batch_norm, bilinear) golden: per-parameter gradient error vs an fp64 oracle run, for
the reference's own fp32 outputs (golden) and the GPU path under both small-channel kernels."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "plastic-unet_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, ROOT)
import numpy as np
import torch
import oracle
from unet import UNetp
from punet import bce_loss
from punet import kernels as K
from conftest import golden

DEV = torch.device("cuda")
g = golden("unetp_bn_bilinear.npz")
sd = {k[2:]: torch.from_numpy(np.asarray(v)) for k, v in g.items() if k.startswith("p.")}
xs = torch.from_numpy(np.asarray(g["xs"]))
H0 = torch.from_numpy(np.asarray(g["hebb"]))
t = torch.from_numpy(np.asarray(g["t"]))
ref = oracle.RefUNetp(1, 1, rule="oja", nbf=64, batch_norm=True, bilinear_upsample=True).double()
ref.load_state_dict({k: v.double() for k, v in sd.items()})
ref.train()
y64, _ = ref(xs[0].double(), H0.double())
oracle.bce_loss(y64, t.double()).backward()
g64 = {k: p.grad for k, p in ref.named_parameters() if p.grad is not None}
outs = {}
for on in (False, True):
    K.set_smallx6(on)
    net = UNetp(1, 1, DEV, rule="oja", nbf=64, batch_norm=True, bilinear_upsample=True)
    net.load_state_dict(sd)
    net.train()
    y, _ = net(xs[0].to(DEV), H0.to(DEV))
    bce_loss(y, t.to(DEV)).backward()
    outs[on] = {k: p.grad.double().cpu() for k, p in net.named_parameters() if p.grad is not None}
print("%-30s %10s %10s %10s" % ("param (err / max|g64|)", "ref fp32", "direct", "x6s"))
for k in g64:
    if k.endswith(".bias") and ".conv." in k:
        continue
    m = g64[k].abs().max().item()
    e_ref = (torch.from_numpy(np.asarray(g["g." + k])).double().reshape(g64[k].shape) - g64[k]).abs().max().item() / m
    e0 = (outs[False][k] - g64[k]).abs().max().item() / m
    e1 = (outs[True][k] - g64[k]).abs().max().item() / m
    print("%-30s %10.2e %10.2e %10.2e" % (k, e_ref, e0, e1))
