"""List every pu_conv_igemm call of one C2 training step with the kernel the library picks for it
(pu_conv_igemm_tile), to attribute rocprof lines to layers.   python tools/list_convs.py [--config c3]"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "plastic-unet_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
from punet import kernels as K  # noqa: E402
from punet.engine import Trainer  # noqa: E402
from unet import UNetp  # noqa: E402

bf16 = "--config" in sys.argv and sys.argv[sys.argv.index("--config") + 1] == "c3"
orig = K.igemm
seen = []


PROF = None


def traced(**kw):
    if PROF is None:
        return orig(**kw)
    n0 = len(PROF.records)
    r = orig(**kw)
    seen.append(({k: v for k, v in kw.items() if k in ("batch", "in_hw", "k", "stride", "c0", "c1", "n", "n0")},
                 PROF.records[n0:]))
    return r


K.igemm = traced
dev = torch.device("cuda")
torch.manual_seed(0)
net = UNetp(1, 1, dev, rule="oja", nbf=128, depth=5, base_ch=64, **({"precision": "bf16"} if bf16 else {}))
tr = Trainer(net, lr=1e-4)
x = torch.rand(32, 1, 128, 128, device=dev)
t = (torch.rand(32, 128, 128, device=dev) > 0.5).float()
h = torch.zeros(32, 128, 128, device=dev)
tr.step(x, t, h)                      # packs, caches
with K.KernelProfiler() as prof:
    PROF = prof  # noqa: F811
    tr.step(x, t, h)
torch.cuda.synchronize()
for i, (args, recs) in enumerate(seen):
    print("%2d %-70s %s" % (i, args, ["%s %.1f us" % (r[0], 1e3 * r[3].elapsed_time(r[4])) for r in recs]))
