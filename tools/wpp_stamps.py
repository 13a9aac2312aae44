"""Barrier timeline of the Winograd kernel (diagnostic build, -DPU_WPP_STAMP=1: block 0's per-wave
s_memtime before and after every barrier; the stamp stores shift the kernel's counted vmcnt
waits, so absolute times read high).  Timing-only tool.

    PLASTIC_UNET_LIB=plastic-unet_amd/lib/libplastic_unet_wppstamp.so python tools/wpp_stamps.py [layer]

Prints, per wave, the mean work span (previous release -> this barrier's arrival) and barrier wait
(arrival -> release) of even and odd barrier intervals, in shader cycles."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "plastic-unet_amd"))
import torch  # noqa: E402
from punet import kernels as K, trunk as T  # noqa: E402

LAYERS = {"top": (128, 64, 64), "l2": (64, 128, 128), "l3": (32, 256, 256), "l4": (16, 512, 512)}
name = sys.argv[1] if len(sys.argv) > 1 else "top"
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
assert n == 8 * NS, n
st = [[buf[wv * NS + k] for k in range(NS)] for wv in range(8)]

t0 = min(s[0] for s in st)
for wv in range(8):
    s = st[wv]
    m = next((k for k in range(NS) if s[k] == 0 or s[k] < t0), NS)
    m -= m % 2
    pairs = [(s[k] - t0, s[k + 1] - t0) for k in range(0, m, 2)]   # (ready, released)
    work = {0: [], 1: []}
    wait = {0: [], 1: []}
    for k in range(1, len(pairs)):
        work[k % 2].append(pairs[k][0] - pairs[k - 1][1])
        wait[k % 2].append(pairs[k][1] - pairs[k][0])
    f = lambda v: sum(v) / max(1, len(v))
    print("wave %d: %3d barriers, first release %6d, last %8d | even: work %6.0f wait %6.0f | odd: work %6.0f wait %6.0f"
          % (wv, len(pairs), pairs[0][1], pairs[-1][1], f(work[0]), f(wait[0]), f(work[1]), f(wait[1])))
# per-interval detail of waves 0 and 4 over the first 40 barriers
for wv in (0, 4):
    s = st[wv]
    print("wave %d intervals (work/wait):" % wv,
          " ".join("%d/%d" % (s[k] - s[k - 1], s[k + 1] - s[k]) for k in range(2, min(NS - 1, 82), 2)))

