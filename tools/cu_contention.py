"""CU contention probe (timing only): how long a one-block-per-CU kernel takes when a few CUs are
held by another stream's kernel - the situation of an RCCL all-reduce (its channels are blocks
that stay resident for the collective) overlapping the backward on a multi-GPU node.  A stand-in
for the collective: torch.cuda._sleep (one block spinning for a given number of cycles) on up to
3 side streams.

    python tools/cu_contention.py [--hogs 1] [--us 100]

Prints, per layer and op, the launch's time alone, beside the hog kernels, and the hogs' own time."""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "plastic-unet_amd"))
import torch  # noqa: E402
from punet import trunk as T  # noqa: E402

LAYERS = {"top": (128, 64, 64), "l2": (64, 128, 128), "l3": (32, 256, 256), "l4": (16, 512, 512)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--hogs", type=int, default=1, help="side streams, one 1-block sleep kernel each (<= 3)")
    ap.add_argument("--us", type=float, default=100.0, help="sleep per hog kernel, microseconds")
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--layers", default="top,l3")
    args = ap.parse_args()
    B = 32
    dev = torch.device("cuda")
    sides = [torch.cuda.Stream() for _ in range(max(1, min(3, args.hogs)))]
    g = torch.Generator().manual_seed(1)

    # calibrate _sleep: cycles per microsecond on this clock
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda._sleep(1000)
    torch.cuda.synchronize()
    e0.record()
    torch.cuda._sleep(1_000_000)
    e1.record()
    torch.cuda.synchronize()
    cyc_per_us = 1_000_000 / (e0.elapsed_time(e1) * 1000.0)
    cycles = int(args.us * cyc_per_us)
    print("sleep calibration: %.0f cycles/us -> %d cycles for %.0f us" % (cyc_per_us, cycles, args.us))

    def timed(fn, hog):
        ts = []
        for _ in range(args.reps):
            torch.cuda.synchronize()
            if hog:
                for s in sides[:args.hogs]:
                    with torch.cuda.stream(s):
                        torch.cuda._sleep(cycles)
            # the main stream idles 20 us first, so the hogs are resident when the launch arrives
            torch.cuda._sleep(int(20 * cyc_per_us))
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            fn()
            b.record()
            torch.cuda.synchronize()
            ts.append(a.elapsed_time(b) * 1000.0)
        ts.sort()
        return ts[len(ts) // 2]

    for name in args.layers.split(","):
        H, C, N = LAYERS[name]
        x = torch.randn(B, H, H, C, generator=g).relu().to(dev)
        w = (torch.randn(N, C, 3, 3, generator=g) * 0.05).to(dev)
        bias = torch.randn(N, generator=g).to(dev)
        dz = torch.randn(B, H, H, N, generator=g).to(dev)
        pk = T._Packs()
        ops = {
            "fwd": lambda: T.conv3x3(x, w, bias, pk, relu=True),
            "wgrad": lambda: T.conv3x3_wgrad(dz, x),
        }
        for op, fn in ops.items():
            for _ in range(3):
                fn()
            alone = timed(fn, False)
            beside = timed(fn, True)
            print("%-4s %-5s alone %7.1f us | beside %d hog(s) of %.0f us: %7.1f us (+%.1f)"
                  % (name, op, alone, args.hogs, args.us, beside, beside - alone))


if __name__ == "__main__":
    main()
