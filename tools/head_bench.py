"""Fused plastic head forward (pu_plastic_head_fwd) at bs 32 x 128^2, C = 64: us per launch and
algorithmic GB/s (the bench line's oja_update.fused_head_bs32), for the library PLASTIC_UNET_LIB
points at (ablation variants).   python tools/head_bench.py [label] [B N C]  (default 32 128 64 = C2;
32 256 8 = C4)"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "plastic-unet_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
from punet import kernels as K  # noqa: E402
import bench  # noqa: E402

dev = torch.device("cuda", 0)
B, N, C = (int(v) for v in sys.argv[2:5]) if len(sys.argv) >= 5 else (32, 128, 64)
torch.manual_seed(0)
H = 0.1 * torch.randn(B, N, N, device=dev)
w = 0.01 * torch.randn(N, N, device=dev)
a = 0.01 * torch.rand(N, N, device=dev)
eta = torch.full((1,), 0.01, device=dev)
feat = torch.rand(B, N, N, C, device=dev)
wo = 0.1 * torch.randn(C, device=dev)
bo = torch.zeros(1, device=dev)
us, how = bench._launch_time_us(lambda: K.plastic_head_fwd(feat, wo, bo, H, w, a, eta, 1, True), 50)
nbytes = 4.0 * B * N * N * C + 16.0 * B * N * N + 8.0 * N * N
print("%-24s %8.2f us  %7.1f GB/s  %.3f of 8 TB/s  (%s)" % (sys.argv[1] if len(sys.argv) > 1 else
      os.path.basename(os.environ.get("PLASTIC_UNET_LIB", "default")), us, nbytes / us / 1e3, nbytes / us / 8e6, how))
