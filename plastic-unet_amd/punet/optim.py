"""FusedAdam: torch.optim.Adam semantics, one multi-tensor HIP launch per step.

Reference: yaricom/Plastic-UNet src/train.py:66 (``torch.optim.Adam(net.parameters(), lr)``) and
:111 (``optimizer.step()``).  Parameters without a gradient (``eta``, S3) are skipped exactly like
torch's Adam skips them.  The state layout (``step``, ``exp_avg``, ``exp_avg_sq``) is torch's, so
optimizer state_dicts move between the two.  StepLR (train.py:67) works unchanged on top.
"""
import math

import torch
from torch.autograd.graph import increment_version

from . import kernels as K


class FusedAdam(torch.optim.Optimizer):
    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0):
        if lr < 0.0:
            raise ValueError("Invalid learning rate: {}".format(lr))
        if not 0.0 <= eps:
            raise ValueError("Invalid epsilon value: {}".format(eps))
        if not 0.0 <= betas[0] < 1.0 or not 0.0 <= betas[1] < 1.0:
            raise ValueError("Invalid beta parameters: {}".format(betas))
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay))

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        for group in self.param_groups:
            beta1, beta2 = group["betas"]
            by_step = {}
            for p in group["params"]:
                if p.grad is None:
                    continue
                if p.grad.is_sparse:
                    raise RuntimeError("FusedAdam does not support sparse gradients")
                st = self.state[p]
                if len(st) == 0:
                    st["step"] = torch.tensor(0.0)
                    st["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                    st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                st["step"] += 1
                t = int(st["step"].item())
                g = p.grad if p.grad.is_contiguous() else p.grad.contiguous()
                by_step.setdefault(t, []).append((p, g, st["exp_avg"], st["exp_avg_sq"]))
            for t, items in by_step.items():
                bc1 = 1 - beta1 ** t
                bc2 = 1 - beta2 ** t
                step_size = group["lr"] / bc1
                K.adam_multi([i[0] for i in items], [i[1] for i in items], [i[2] for i in items],
                             [i[3] for i in items], beta1, beta2, group["eps"], group["weight_decay"],
                             step_size, math.sqrt(bc2))
                # the kernel writes through raw pointers: bump the version counters so every cache
                # keyed on them (the trunk's packed / split GEMM operands) sees the new values
                increment_version([i[0] for i in items])
        return loss
