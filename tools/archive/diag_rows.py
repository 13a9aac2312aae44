"""Where the bf16 row-stream kernel differs from the per-tap lean kernel (diagnostic, GPU)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "plastic-unet_amd"))
import torch  # noqa: E402
from punet import kernels as K  # noqa: E402
from punet import trunk as T  # noqa: E402
from punet._lib import PU_PACK_CONV_FWD  # noqa: E402

DEV, BF = torch.device("cuda"), torch.bfloat16
for B, mode in ((1, "ones"), (1, "randn")):
    g = torch.Generator(device=DEV).manual_seed(7)
    if mode == "ones":
        x = torch.ones(B, 128, 128, 64, device=DEV).to(BF)
        w = torch.zeros(64, 64, 3, 3, device=DEV)
        w[:, :, 1, 1] = 1.0                                   # centre tap only: y[n] = sum_c x[c]
    else:
        x = torch.randn(B, 128, 128, 64, device=DEV, generator=g).to(BF)
        w = torch.randn(64, 64, 3, 3, device=DEV, generator=g) * 0.05
    outs = []
    for halo in (1, 0):
        K.set_conv_halo(halo)
        pk = T._Packs()
        wt = pk.get(w, PU_PACK_CONV_FWD, 576, 32, BF)
        out = torch.empty(B, 128, 128, 64, device=DEV, dtype=BF)
        K.igemm(batch=B, in_hw=(128, 128), out_hw=(128, 128), k=3, stride=1, pad=1, src0=x, c0=64, weight=wt,
                k_pad=576, n=64, dst0=out, cgroup=32)
        outs.append(out.float())
    torch.cuda.synchronize()
    d = (outs[0] - outs[1]).abs()
    print(mode, "max diff", d.max().item(), "frac differing", (d > 0).float().mean().item())
    bad = (d > 0).nonzero()
    if len(bad):
        rows = torch.unique(bad[:, 1]).tolist()
        cols = torch.unique(bad[:, 2]).tolist()
        chans = torch.unique(bad[:, 3]).tolist()
        print(" rows", rows[:40], len(rows))
        print(" cols", cols[:40], len(cols))
        print(" chans", chans[:70], len(chans))
        b0 = bad[0].tolist()
        print(" first", b0, "rows-kernel", outs[0][tuple(b0)].item(), "lean", outs[1][tuple(b0)].item())
    if mode == "ones":
        print(" rows-kernel centre value", outs[0][0, 5, 5, :4].tolist(), "lean", outs[1][0, 5, 5, :4].tolist())
