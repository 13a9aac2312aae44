"""Data parallelism: one process per GPU, gradients averaged with one RCCL all-reduce per step.

The reference has no parallelism; this is the north_star's DP: the
minibatch is sharded across ranks, parameters start identical (rank-0 broadcast), gradients are
averaged over xGMI by RCCL (torch.distributed backend "nccl" is RCCL on ROCm), and each rank's
plastic traces stay local to its slots (never synchronised).  ``eta`` has no gradient (S3) and is
not communicated.

Gradients land in ONE flat fp32 buffer: the trunk/head backward kernels write straight into views
of it (autograd adopts those views as ``param.grad``), so the all-reduce needs no pack/unpack
copies.  The all-reduce is split into a few large buckets issued in reverse layer order.
"""
import os

import torch
import torch.distributed as dist


def env_world():
    return int(os.environ.get("WORLD_SIZE", "1")), int(os.environ.get("RANK", "0")), \
        int(os.environ.get("LOCAL_RANK", "0"))


def init_from_env(backend=None, timeout_s=600):
    """Initialise the default process group from torchrun's env (MASTER_ADDR=127.0.0.1)."""
    world, rank, local = env_world()
    if world > 1 and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if backend is None:
            backend = "nccl" if torch.cuda.is_available() else "gloo"
        if backend == "nccl":
            torch.cuda.set_device(local)
        import datetime
        dist.init_process_group(backend, timeout=datetime.timedelta(seconds=timeout_s))
    return world, rank, local


@torch.no_grad()
def broadcast_params(module, src=0):
    if dist.is_initialized() and dist.get_world_size() > 1:
        for t in list(module.parameters()) + list(module.buffers()):
            dist.broadcast(t.data, src)


class GradBuffer:
    """Flat gradient storage for ``params`` (in order); ``views[i]`` has ``params[i]``'s shape."""

    def __init__(self, params, device):
        self.params = list(params)
        self.numel = sum(p.numel() for p in self.params)
        self.flat = torch.zeros(self.numel, dtype=torch.float32, device=device)
        self.views = []
        self.offsets = {}
        off = 0
        for p in self.params:
            self.views.append(self.flat[off:off + p.numel()].view_as(p))
            self.offsets[id(p)] = (off, p.numel())
            off += p.numel()

    def view_for(self, p):
        o = self.offsets.get(id(p))
        if o is None:
            return None
        return self.flat[o[0]:o[0] + o[1]].view_as(p)

    def owns_grads(self):
        base = self.flat.data_ptr()
        for p in self.params:
            if p.grad is None or p.grad.data_ptr() != base + 4 * self.offsets[id(p)][0]:
                return False
        return True


def allreduce_mean_(tensors, group=None):
    """Average a list of flat tensors across ranks (RCCL AVG on GPU, SUM/world on gloo)."""
    if not dist.is_initialized():
        return
    world = dist.get_world_size(group)
    if world == 1:
        return
    gloo = dist.get_backend(group) == "gloo"
    for t in tensors:
        if gloo:
            dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
            t.div_(world)
        else:
            dist.all_reduce(t, op=dist.ReduceOp.AVG, group=group)


def allreduce_grads(params, gradbuf=None, group=None, bucket_mb=32):
    """Average the gradients of ``params``.  With a GradBuffer that owns every grad, reduce it in
    buckets of ~bucket_mb (reverse order: decoder/head first); otherwise coalesce, reduce, scatter."""
    if not dist.is_initialized() or dist.get_world_size(group) == 1:
        return
    if gradbuf is not None and gradbuf.owns_grads():
        n = gradbuf.numel
        step = max(1, bucket_mb * (1 << 20) // 4)
        chunks = [gradbuf.flat[s:min(n, s + step)] for s in range(0, n, step)]
        allreduce_mean_(list(reversed(chunks)), group)
        return
    grads = [p.grad for p in params if p.grad is not None]
    if not grads:
        return
    flat = torch.cat([g.reshape(-1) for g in grads])
    allreduce_mean_([flat], group)
    off = 0
    for g in grads:
        g.copy_(flat[off:off + g.numel()].view_as(g))
        off += g.numel()
