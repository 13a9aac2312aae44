"""Item timeline of wino4_x6_kernel (diagnostic build -DPU_W4_ITEM_STAMP=1): per block s_memtime at
entry, prologue done, loop done, output-exchange done, stores issued, stores drained, plus HW_ID /
XCC_ID, for the last forward launch of one layer.  Reports phase medians (shader cycles) and, per
CU, the gap between a block's end and the next block's entry.  Timing-only tool.

    PLASTIC_UNET_LIB=plastic-unet_amd/lib/libplastic_unet_w4st.so python tools/w4_items.py [layer]"""
import ctypes
import os
import statistics as st
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "plastic-unet_amd"))
import torch  # noqa: E402
from punet import kernels as K, trunk as T  # noqa: E402

LAYERS = {"top": (128, 64, 64), "l2": (64, 128, 128), "l3": (32, 256, 256), "l4": (16, 512, 512)}
for name in (sys.argv[1:] or ["top", "l4"]):
    H, C, N = LAYERS[name]
    B = 32
    g = torch.Generator().manual_seed(1)
    x = torch.randn(B, H, H, C, generator=g).relu().cuda()
    w = (torch.randn(N, C, 3, 3, generator=g) * 0.05).cuda()
    b = torch.randn(N, generator=g).cuda()
    pk = T._Packs()
    for _ in range(4):
        T.conv3x3(x, w, b, pk, relu=True)
    torch.cuda.synchronize()
    items = B * (H // 2) * (H // 2) // 64 * (N // 64)
    nb = min(items, 4096)
    buf = (ctypes.c_ulonglong * (8 * nb))()
    K.lib().pu_w4_item_stamps(buf, 8 * nb)
    rows = [[buf[i * 8 + k] for k in range(8)] for i in range(nb)]
    ph = {k: [] for k in ("prologue", "loop", "exchange", "epilogue", "drain", "total")}
    for r in rows:
        ph["prologue"].append(r[1] - r[0])
        ph["loop"].append(r[2] - r[1])
        ph["exchange"].append(r[3] - r[2])
        ph["epilogue"].append(r[4] - r[3])
        ph["drain"].append(r[5] - r[4])
        ph["total"].append(r[5] - r[0])
    print("== %s: %d items, C %d -> N %d (%d sub-stages per item)" % (name, items, C, N, 4 * C // 16))
    for k, v in ph.items():
        v = sorted(v)
        print("  %-9s median %7d  p10 %7d  p90 %7d" % (k, st.median(v), v[len(v) // 10], v[9 * len(v) // 10]))
    # per CU (XCC, SE, SH, CU from HW_ID bits 8..15): gap from a block's drained end to the next entry
    cu = {}
    for r in rows:
        cu.setdefault((r[7] & 0xf, (r[6] >> 8) & 0xff), []).append(r)
    gaps, per_cu = [], []
    for key, rs in cu.items():
        rs.sort(key=lambda r: r[0])
        per_cu.append(len(rs))
        for a, c in zip(rs, rs[1:]):
            gaps.append(c[0] - a[5])
    if gaps:
        gaps.sort()
        print("  CUs %d, blocks per CU %s..%s; end -> next entry gap median %d p10 %d p90 %d" % (
            len(cu), min(per_cu), max(per_cu), st.median(gaps), gaps[len(gaps) // 10], gaps[9 * len(gaps) // 10]))
    # span per XCC
    xs = {}
    for r in rows:
        xs.setdefault(r[7] & 0xf, []).append(r)
    for xcc, rs in sorted(xs.items()):
        t0 = min(r[0] for r in rs)
        t1 = max(r[5] for r in rs)
        print("  xcc %d: %d blocks, span %d cycles" % (xcc, len(rs), t1 - t0))
