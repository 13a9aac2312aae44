"""Vendor-library context for the conv roofline: MIOpen (torch F.conv2d) fp32 conv3x3 fwd / dgrad /
wgrad at the config-C2 layer shapes, and hipBLASLt (torch.matmul) GEMM rates in fp32 / bf16.

    python tools/vendor_probe.py [--json out.json]

Not part of the product path: it times torch's own kernels on the same device so the achieved
TFLOP/s of the HIP kernels (tools/conv_bench.py) can be read against what the libraries reach.
"""
import argparse
import json

import torch
import torch.nn.functional as F

LAYERS = {  # name: (H, cin, cout), B = 32, 3x3 pad 1
    "top": (128, 64, 64), "top_cat": (128, 128, 64), "l2": (64, 128, 128), "l3": (32, 256, 256),
    "l4": (16, 512, 512), "bottom": (8, 512, 512),
}


def timeit(fn, reps=10):
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
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    dev = torch.device("cuda")
    torch.backends.cudnn.benchmark = True
    res = {"conv_fp32": {}, "gemm": {}}
    for name, (H, cin, cout) in LAYERS.items():
        B = 32
        flops = 2.0 * B * H * H * cout * 9 * cin
        r = {}
        for fmt in ("nchw", "nhwc"):
            mf = torch.channels_last if fmt == "nhwc" else torch.contiguous_format
            x = torch.randn(B, cin, H, H, device=dev).contiguous(memory_format=mf).requires_grad_(True)
            w = (0.05 * torch.randn(cout, cin, 3, 3, device=dev)).contiguous(memory_format=mf).requires_grad_(True)
            y = F.conv2d(x, w, padding=1)
            gy = torch.randn_like(y)
            fwd = timeit(lambda: F.conv2d(x, w, padding=1))
            dg = timeit(lambda: torch.ops.aten.convolution_backward(gy, x, w, None, [1, 1], [1, 1], [1, 1], False,
                                                                    [0, 0], 1, [True, False, False]))
            wg = timeit(lambda: torch.ops.aten.convolution_backward(gy, x, w, None, [1, 1], [1, 1], [1, 1], False,
                                                                    [0, 0], 1, [False, True, False]))
            r[fmt] = {k: round(flops / (ms * 1e-3) / 1e12, 1) for k, ms in (("fwd_TF", fwd), ("dgrad_TF", dg),
                                                                          ("wgrad_TF", wg))}
        res["conv_fp32"][name] = r
        print(name, r, flush=True)
    for dt in (torch.float32, torch.bfloat16):
        for (m, n, k) in ((8192, 8192, 8192), (524288, 64, 576), (131072, 128, 1152), (32768, 256, 2304)):
            A = torch.randn(m, k, device=dev, dtype=dt)
            Bm = torch.randn(k, n, device=dev, dtype=dt)
            ms = timeit(lambda: A @ Bm)
            tf = round(2.0 * m * n * k / (ms * 1e-3) / 1e12, 1)
            res["gemm"]["%s_%dx%dx%d" % (str(dt).split(".")[-1], m, n, k)] = tf
            print("gemm", dt, m, n, k, tf, "TF/s", flush=True)
    if a.json:
        json.dump(res, open(a.json, "w"), indent=1)


if __name__ == "__main__":
    main()
