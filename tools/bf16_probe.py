"""bf16 (C3) vs fp32 trunk gradients against the fp64 oracle, per parameter (diagnostic)."""
import sys, torch
sys.path.insert(0, "plastic-unet_amd"); sys.path.insert(0, ".")
from unet import UNetp
from punet import bce_loss
import oracle
DEV = torch.device("cuda")
torch.manual_seed(3)
ref = oracle.RefUNetp(1, 1, rule="oja", nbf=64, depth=4, base_ch=32)
net = UNetp(1, 1, DEV, rule="oja", nbf=64, depth=4, base_ch=32, precision="bf16")
net32 = UNetp(1, 1, DEV, rule="oja", nbf=64, depth=4, base_ch=32)
net.load_state_dict(ref.state_dict()); net32.load_state_dict(ref.state_dict())
g = torch.Generator().manual_seed(8)
x = torch.rand(2, 1, 64, 64, generator=g)
t = (torch.rand(2, 64, 64, generator=g) > 0.5).float()
H = 0.05 * torch.randn(2, 64, 64, generator=g)
outs = []
for n in (net, net32):
    y, hn = n(x.to(DEV), H.to(DEV)); l = bce_loss(y, t.to(DEV)); l.backward(); outs.append((y, hn, l))
ref = ref.double()
yr, hr = ref(x.double(), H.double()); lr_ = oracle.bce_loss(yr, t.double()); lr_.backward()
for name, (y, hn, l) in zip(("bf16", "fp32"), outs):
    print(name, "Ymax", (y.double().cpu() - yr).abs().max().item(), "loss", abs(l.item() - lr_.item()))
for (k, p), (_, p32), (_, pr) in zip(net.named_parameters(), net32.named_parameters(), ref.named_parameters()):
    if k == "eta": continue
    r = lambda a: ((a.double().cpu() - pr.grad).norm() / pr.grad.norm()).item()
    print("%-32s bf16 %.4f  fp32 %.2e" % (k, r(p.grad), r(p32.grad)))
