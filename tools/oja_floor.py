"""Kernel-duration view of the stand-alone Oja update at the bench batch (bs 32 x 128^2, 4.23 MB)
next to the launch floor, for rocprofv3 --kernel-trace --stats:

    rocprofv3 --kernel-trace --stats -d gpurun_out/oja -o run -- python tools/oja_floor.py

Kernels (distinct names in the trace):
  trace_kernel_v4   Oja update, B=32, N=128: 8*B*N^2 + 8*B*N = 4.23 MB per launch
  trace_kernel      the same update on B=1, N=3 (9 elements): an empty-work launch = the floor of
                    one dependent kernel on this stream (ramp + drain, no bytes)
  trace_kernel_v4   (tagged by size in the log) B=16384: 2.2 GB per launch, the HBM-sized sweep
The bench's HIP-graph figure (oja_update.bs32) includes the ~1-1.5 us kernel boundary; the
kernel-trace duration here is the kernel alone.
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "plastic-unet_amd"))

import torch  # noqa: E402

from punet import kernels as K  # noqa: E402


def main():
    dev = torch.device("cuda")
    eta = torch.full((1,), 0.01, device=dev)
    for B, N, reps in ((1, 3, 200), (32, 128, 200), (16384, 128, 5)):
        H = torch.randn(B, N, N, device=dev)
        X = torch.randn(B, N, N, device=dev)
        Y = torch.rand(B, N, N, device=dev)
        out = torch.empty_like(H)
        for _ in range(reps):
            K.trace_update(H, X, Y, eta, 1, out=out)
        torch.cuda.synchronize()
        print("B=%d N=%d: %d launches, %.3f MB each" % (B, N, reps, (8.0 * B * N * N + 8.0 * B * N) / 1e6), flush=True)
        del H, X, Y, out


if __name__ == "__main__":
    main()
