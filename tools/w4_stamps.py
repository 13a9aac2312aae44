"""Sub-stage timeline of wino4_x6_kernel (diagnostic build -DPU_WPP_STAMP=1, one item per block:
PU_WINO4=1 PU_WINO_PERSIST=0).  Block 0's waves stamp s_memtime at each sub-stage's barrier
arrival, release, and after its MFMAs were issued.  Timing-only tool.

    PU_WINO4=1 PU_WINO_PERSIST=0 PLASTIC_UNET_LIB=plastic-unet_amd/lib/libplastic_unet_w4stamp.so \\
        python tools/w4_stamps.py [layer]"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "plastic-unet_amd"))
import torch  # noqa: E402
from punet import kernels as K, trunk as T  # noqa: E402

LAYERS = {"top": (128, 64, 64), "l2": (64, 128, 128), "l3": (32, 256, 256), "l4": (16, 512, 512)}
name = sys.argv[1] if len(sys.argv) > 1 else "l4"
H, C, N = LAYERS[name]
B = 32
g = torch.Generator().manual_seed(1)
x = torch.randn(B, H, H, C, generator=g).relu().cuda()
w = (torch.randn(N, C, 3, 3, generator=g) * 0.05).cuda()
b = torch.randn(N, generator=g).cuda()
pk = T._Packs()
for _ in range(3):
    T.conv3x3(x, w, b, pk, relu=True)
torch.cuda.synchronize()
NS = 512
buf = (ctypes.c_ulonglong * (8 * NS))()
n = K.lib().pu_wpp_stamps(buf, 8 * NS)
st = [[buf[wv * NS + k] for k in range(NS)] for wv in range(4)]
t0 = min(s[0] for s in st)
for wv in range(4):
    s = st[wv]
    m = next((k for k in range(NS) if s[k] == 0 or s[k] < t0), NS)
    m -= m % 4
    # issued-all, arrival (after lgkmcnt(0)), release, MFMAs issued
    tr = [tuple(s[k + q] - t0 for q in range(4)) for k in range(0, m, 4)]
    lg = [a - i for i, a, _, _ in tr]
    wait = [r - a for _, a, r, _ in tr]
    head = [f - r for _, _, r, f in tr]
    tail = [tr[k + 1][0] - tr[k][3] for k in range(len(tr) - 1)]
    per = [tr[k + 1][2] - tr[k][2] for k in range(len(tr) - 1)]
    f = lambda v: sum(v[2:]) / max(1, len(v) - 2)
    print("wave %d: %3d sub-stages | release->MFMAs issued %5.0f | ->rest issued %5.0f | lgkm wait %5.0f | barrier "
          "wait %5.0f | release->release %5.0f" % (wv, len(tr), f(head), f(tail), f(lg), f(wait), f(per)))
