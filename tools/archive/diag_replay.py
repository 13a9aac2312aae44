"""Record every conv3x3_dgrad / conv3x3 call of a UNetp(bn, bilinear) training step, replay each
with the small-channel MFMA kernel off and on, and report the calls whose outputs differ."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "plastic-unet_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np
import torch
from unet import UNetp
from punet import bce_loss
from punet import kernels as K
from punet import trunk as T
from conftest import golden
DEV = torch.device("cuda")
g = golden("unetp_bn_bilinear.npz")
sd = {k[2:]: torch.from_numpy(np.asarray(v)) for k, v in g.items() if k.startswith("p.")}
xs = torch.from_numpy(np.asarray(g["xs"])); H0 = torch.from_numpy(np.asarray(g["hebb"])); tt = torch.from_numpy(np.asarray(g["t"]))
calls = []
orig_d, orig_f = T.conv3x3_dgrad, T.conv3x3
MODE = os.environ.get("REPLAY_MODE", "0") == "1"
def rec_d(dz, w, packs, split=None, mask0=None, mask1=None):
    cl = lambda t: None if t is None else t.detach().clone()
    c = ["dgrad", cl(dz), cl(w), split, cl(mask0), cl(mask1)]
    o = orig_d(dz, w, packs, split=split, mask0=mask0, mask1=mask1)
    torch.cuda.synchronize()
    c.append((torch.cat([o[0], o[1]], 3) if o[1] is not None else o[0]).detach().double().cpu())
    calls.append(c)
    return o
def rec_f(x0, w, b, packs, x1=None, relu=True):
    cl = lambda t: None if t is None else t.detach().clone()
    c = ["fwd", cl(x0), cl(w), cl(b), cl(x1), relu]
    o = orig_f(x0, w, b, packs, x1=x1, relu=relu)
    torch.cuda.synchronize()
    c.append(o.detach().double().cpu())
    calls.append(c)
    return o
T.conv3x3_dgrad, T.conv3x3 = rec_d, rec_f
K.set_smallx6(MODE)
net = UNetp(1, 1, DEV, rule="oja", nbf=64, batch_norm=True, bilinear_upsample=True)
net.load_state_dict(sd); net.train()
y, _ = net(xs[0].to(DEV), H0.to(DEV))
bce_loss(y, tt.to(DEV)).backward()
torch.cuda.synchronize()
T.conv3x3_dgrad, T.conv3x3 = orig_d, orig_f
for i, c in enumerate(calls):
    outs = [c[-1]]
    for on in (MODE,):
        K.set_smallx6(on)
        pk = T._Packs()
        if c[0] == "dgrad":
            _, dz, w, split, m0, m1, _ = c
            o = orig_d(dz, w, pk, split=split, mask0=m0, mask1=m1)
            o = torch.cat([o[0], o[1]], 3) if o[1] is not None else o[0]
        else:
            _, x0, w, b, x1, relu, _ = c
            o = orig_f(x0, w, b, pk, x1=x1, relu=relu)
        torch.cuda.synchronize()
        outs.append(o.double().cpu())
    err = (outs[0] - outs[1]).abs().max().item() / max(outs[0].abs().max().item(), 1e-30)
    desc = tuple(c[1].shape) + (tuple(c[2].shape),)
    print("%3d %-5s %-40s rel diff %.2e%s" % (i, c[0], desc, err, "   <---" if err > 1e-5 else ""))
