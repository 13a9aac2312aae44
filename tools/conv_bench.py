"""Per-layer timing of the conv kernels at config-C2 shapes (B=32): fwd, dgrad, wgrad.

    python tools/conv_bench.py [--reps 20] [--layers top,mid,...] [--json out.json]

Prints achieved TFLOP/s per launch (algorithmic FLOPs = 2*M*N*K, K = taps*Cin) against the fp32
MFMA peak.  Used to iterate on igemm/wgrad; bench.py is the end-to-end number.
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "plastic-unet_amd"))

import torch  # noqa: E402

from punet import trunk as T  # noqa: E402
from punet import kernels as K  # noqa: E402

# name: (H, c0, c1, cout)   (B = 32, 3x3 pad 1)
LAYERS = {
    "top": (128, 64, 0, 64),
    "top_cat": (128, 64, 64, 64),
    "l2": (64, 128, 0, 128),
    "l2_cat": (64, 128, 128, 64),
    "l3": (32, 256, 0, 256),
    "l4": (16, 512, 0, 512),
    "l4_cat": (16, 512, 512, 256),
    "bottom": (8, 512, 0, 512),
    "stem": (128, 1, 0, 64),
    # 32-channel levels of C4 (CoordConv base 8 at 64^2) / C5 (UNetpRes n8 at 128^2)
    "c32": (64, 32, 0, 32),
    "c32_cat": (64, 32, 32, 32),
    # small-channel direct-kernel levels of C4/C5 (UNetpRes neurons 8 at 512^2, CoordConv base 8)
    "s8": (512, 8, 0, 8),
    "s8_cat": (512, 8, 8, 8),
    "s16": (256, 16, 0, 16),
    "s16_cat": (256, 16, 16, 16),
}


def timeit(fn, reps):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--layers", default=",".join(LAYERS))
    ap.add_argument("--json", default=None)
    ap.add_argument("--ops", default="fwd,dgrad,wgrad", help="subset of fwd,dgrad,wgrad to time")
    ap.add_argument("--bf16", action="store_true", help="bf16 activations (config C3 kernels)")
    ap.add_argument("--data", default="randn", choices=["randn", "bf16", "zeros"],
                    help="operand values (power/clock probe): bf16 = values exact in bf16 (zero mid/lo planes)")
    a = ap.parse_args()
    dev = torch.device("cuda")
    cu, clk, _ = K.device_info(0)
    peak = 256.0 * cu * (clk / 1e6 if clk else 2.4) / 1e3
    res = {}
    B = a.batch
    for name in a.layers.split(","):
        H, c0, c1, cout = LAYERS[name]
        g = torch.Generator(device=dev).manual_seed(0)
        x0 = torch.randn(B, H, H, c0, device=dev, generator=g).relu_()
        x1 = torch.randn(B, H, H, c1, device=dev, generator=g).relu_() if c1 else None
        w = torch.randn(cout, c0 + c1, 3, 3, device=dev, generator=g) * 0.05
        b = torch.randn(cout, device=dev, generator=g)
        dz = torch.randn(B, H, H, cout, device=dev, generator=g)
        if a.data != "randn":
            for t in (x0, x1, w, dz):
                if t is not None:
                    t.copy_(t.bfloat16().float() if a.data == "bf16" else torch.zeros_like(t))
        if a.bf16:
            x0, dz = x0.bfloat16(), dz.bfloat16()
            x1 = x1.bfloat16() if x1 is not None else None
        pk = T._Packs()
        flops = 2.0 * B * H * H * cout * 9 * (c0 + c1)
        r = {}
        ops = a.ops.split(",")
        if "fwd" in ops:
            r["fwd_ms"] = timeit(lambda: T.conv3x3(x0, w, b, pk, x1=x1), a.reps)
        if c0 > 1 and "dgrad" in ops:
            r["dgrad_ms"] = timeit(lambda: T.conv3x3_dgrad(dz, w, pk, split=c0 if c1 else None, mask0=x0,
                                                           mask1=x1), a.reps)
        if "wgrad" in ops:
            r["wgrad_ms"] = timeit(lambda: T.conv3x3_wgrad(dz, x0, x1), a.reps)
        for k in ("fwd", "dgrad", "wgrad"):
            if k + "_ms" in r:
                r[k + "_TF"] = round(flops / (r[k + "_ms"] * 1e-3) / 1e12, 2)
                r[k + "_frac"] = round(r[k + "_TF"] / peak, 3)
        r["gflop"] = flops / 1e9
        px = B * H * H
        r["fwd_GBs"] = round(4.0 * px * (c0 + c1 + cout) / (r.get("fwd_ms", 1e30) * 1e-3) / 1e9, 1)
        r["dgrad_GBs"] = round(4.0 * px * (cout + 2 * (c0 + c1)) / (r.get("dgrad_ms", 1e30) * 1e-3) / 1e9, 1)
        res[name] = r
        print("%-8s H=%-3d %4d+%-4d->%-4d  fwd %7.3f ms %6.1f TF | dgrad %7.3f ms %6.1f TF | wgrad %7.3f ms %6.1f TF"
              % (name, H, c0, c1, cout, r.get("fwd_ms", 0), r.get("fwd_TF", 0), r.get("dgrad_ms", 0),
                 r.get("dgrad_TF", 0), r.get("wgrad_ms", 0), r.get("wgrad_TF", 0)) +
              ("   [fwd %.0f GB/s, dgrad %.0f GB/s]" % (r["fwd_GBs"], r["dgrad_GBs"]) if c0 + c1 <= 16 else ""), flush=True)
    print("peak fp32 MFMA %.1f TF/s" % peak)
    if a.json:
        json.dump({"peak_TF": peak, "layers": res}, open(a.json, "w"), indent=1)


if __name__ == "__main__":
    main()
