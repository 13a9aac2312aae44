"""Diagnostic: first-step gradients of the product vs the oracle on the train-capture fixture."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "plastic-unet_amd"), os.path.join(ROOT, "tests")]
import numpy as np, torch
import oracle
from unet import UNetp
from punet import bce_loss
g = np.load(os.path.join(ROOT, "tests/golden/train_capture.npz"))
sd = {k[5:]: torch.from_numpy(g[k]) for k in g.files if k.startswith("init.")}
ref = oracle.RefUNetp(1, 1, rule="oja", nbf=32); ref.load_state_dict(sd)
net = UNetp(1, 1, torch.device("cuda"), rule="oja", nbf=32); net.load_state_dict(sd)
x = torch.from_numpy(g["X_train"][0:1].astype(np.float32)); t = torch.from_numpy(g["y_train"][0].astype(np.float32))
H = torch.zeros(32, 32)
y, _ = ref(x, H); oracle.bce_loss(y, t).backward()
yg, _ = net(x.cuda(), H.cuda()); bce_loss(yg, t.cuda()).backward()
rp = dict(ref.named_parameters())
for k, p in net.named_parameters():
    if p.grad is None: continue
    a, b = p.grad.cpu(), rp[k].grad
    sc = b.abs().max().item()
    rel = ((a - b).abs().max().item()) / max(sc, 1e-30)
    flips = ((a * b) < 0).sum().item()
    tiny = (b.abs() < 1e-6 * sc).sum().item()
    z_ref = (b == 0); z_bad = (z_ref & (a != 0)).sum().item()
    mx = a[z_ref].abs().max().item() if z_ref.any() else 0.0
    print("%-34s max|g| %.3e  relerr %.2e  flips %d/%d  tiny %d  ref==0 %d ours!=0 %d (max %.1e)"
          % (k, sc, rel, flips, b.numel(), tiny, z_ref.sum().item(), z_bad, mx))
