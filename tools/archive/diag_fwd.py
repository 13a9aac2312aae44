"""Forward intermediates of UNetp(bn, bilinear) with the small-channel MFMA kernel off / on."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "plastic-unet_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np
import torch
from unet import UNetp
from punet import kernels as K
from conftest import golden
DEV = torch.device("cuda")
g = golden("unetp_bn_bilinear.npz")
sd = {k[2:]: torch.from_numpy(np.asarray(v)) for k, v in g.items() if k.startswith("p.")}
xs = torch.from_numpy(np.asarray(g["xs"])); H0 = torch.from_numpy(np.asarray(g["hebb"]))
acts = {}
for on in (False, True):
    K.set_smallx6(on)
    net = UNetp(1, 1, DEV, rule="oja", nbf=64, batch_norm=True, bilinear_upsample=True)
    net.load_state_dict(sd); net.train()
    tr = net._trunk_plan()
    orig = tr.forward
    box = {}
    def fwd(x, params, save, orig=orig, box=box):
        out = orig(x, params, save)
        box["s"] = out[1]
        return out
    tr.forward = fwd
    y, _ = net(xs[0].to(DEV), H0.to(DEV))
    torch.cuda.synchronize()
    flat = {}
    for k, v in box["s"].items():
        if isinstance(v, torch.Tensor):
            flat[k] = v.detach().double().cpu()
        elif isinstance(v, (list, tuple)):
            for i, e in enumerate(v):
                if isinstance(e, torch.Tensor):
                    flat["%s[%d]" % (k, i)] = e.detach().double().cpu()
    acts[on] = flat
for k in acts[False]:
    a, b = acts[False][k], acts[True].get(k)
    if b is None or a.shape != b.shape:
        print(k, "missing/shape"); continue
    flips = int(((a > 0) != (b > 0)).sum().item())
    print("%-16s %-22s rel diff %.2e  relu-mask flips %d%s" % (k, tuple(a.shape), (a - b).abs().max().item() / max(a.abs().max().item(), 1e-30),
                                                         flips, "   (values %s / %s)" % (a[(a > 0) != (b > 0)][:3].tolist(), b[(a > 0) != (b > 0)][:3].tolist()) if flips else ""))
