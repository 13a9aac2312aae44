"""Data parallelism: one process per GPU, gradients averaged with one RCCL all-reduce per step.

The reference has no parallelism; this is the north_star's DP: the
minibatch is sharded across ranks, parameters start identical (rank-0 broadcast), gradients are
averaged over xGMI by RCCL (torch.distributed backend "nccl" is RCCL on ROCm), and each rank's
plastic traces stay local to its slots (never synchronised).  ``eta`` has no gradient (S3) and is
not communicated.

Gradients land in ONE flat fp32 buffer: the trunk/head backward kernels write straight into views
of it (autograd adopts those views as ``param.grad``), so the all-reduce needs no pack/unpack
copies.  The buffer is laid out in the order the backward produces gradients (head first, then
the trunk from its output layer down to the stem), and ``BucketReducer`` issues an asynchronous
all-reduce for each contiguous bucket the moment its last gradient kernel has been enqueued, so
RCCL runs on its own stream under the remaining backward kernels (overlap); ``finish`` makes the
compute stream wait for the last bucket before Adam.
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
        ts = list(module.parameters()) + list(module.buffers())
        for t in ts:
            dist.broadcast(t.data, src)
        # collectives write in place without bumping version counters; packed-operand caches key on them
        torch.autograd.graph.increment_version(ts)


def rank_generator(device, seed=None, rank=None):
    """A per-rank random generator on ``device`` for the trunk's Dropout2d masks
    (unet_p_res.py:62,69).  Parameters start identical on every rank (broadcast_params), but the
    masks must not: with one shared seed every rank would draw the same channel mask for its slot
    b, so a world of R ranks x B slots would see only B distinct mask sets instead of R x B (the
    single-process global batch).  seed defaults to torch.initial_seed() (what torch.manual_seed
    set), so runs stay reproducible; the rank offset is an odd 64-bit multiplier (distinct
    streams for every rank)."""
    if rank is None:
        rank = dist.get_rank() if dist.is_initialized() else 0
    if seed is None:
        seed = torch.initial_seed()
    g = torch.Generator(device=device)
    g.manual_seed((int(seed) + 0x9E3779B97F4A7C15 * (int(rank) + 1)) % (1 << 63))
    return g


class GradBuffer:
    """Flat gradient storage for ``params`` (in order); ``views[i]`` has ``params[i]``'s shape.
    Every view starts on a 256-byte boundary (``ALIGN`` floats), so the vectorised kernels that
    write and read gradients (wgrad epilogues, Adam) keep their 16-byte accesses whatever the
    parameter sizes are (the outconv bias has 1 element); the padding is zero and never read."""

    ALIGN = 64

    def __init__(self, params, device):
        self.params = list(params)
        self.reducer = None      # BucketReducer: notified by the backward as gradients complete
        self.offsets = {}
        off = 0
        for p in self.params:
            self.offsets[id(p)] = (off, p.numel())
            off += (p.numel() + self.ALIGN - 1) // self.ALIGN * self.ALIGN
        self.numel = off
        self.flat = torch.zeros(self.numel, dtype=torch.float32, device=device)
        self.views = [self.flat[o:o + n].view_as(p) for p, (o, n) in
                      ((p, self.offsets[id(p)]) for p in self.params)]

    def view_for(self, p):
        o = self.offsets.get(id(p))
        if o is None:
            return None
        return self.flat[o[0]:o[0] + o[1]].view_as(p)

    def ready(self, *params):
        """Called by the backward right after enqueuing the kernels that write ``params``' grads."""
        if self.reducer is not None:
            self.reducer.ready(params)

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
    if not dist.is_initialized():
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


class BucketReducer:
    """Overlapped gradient averaging over a GradBuffer.

    The flat buffer is cut into contiguous buckets of about ``bucket_mb`` (never splitting a
    parameter).  ``begin()`` arms it before backward; every ``ready(params)`` call counts those
    parameters off their bucket, and a bucket whose last parameter arrives is all-reduced at once
    with ``async_op=True`` (RCCL runs on its own stream, ordered after the kernels already enqueued
    on the compute stream).  Every rank runs the same backward, so buckets are issued in the same
    order on all ranks.  ``finish()`` issues whatever is left (parameters that never reported, in
    buffer order), then waits: on RCCL ``wait`` only orders the current stream after the
    collective, so the host does not block."""

    def __init__(self, gradbuf, bucket_mb=16, group=None, force=False):
        self.gb = gradbuf
        self.group = group
        self.force = force       # active in a world of one too (exercises the async path)
        cap = max(1, int(bucket_mb * (1 << 20)) // 4)
        self.buckets = []        # [start, end, {param ids}]
        self.bucket_of = {}
        start, ids = 0, set()
        off = 0
        for p in gradbuf.params:
            off = gradbuf.offsets[id(p)][0]
            n = gradbuf.offsets[id(p)][1]
            if ids and off + n - start > cap:
                self.buckets.append((start, off, ids))
                start, ids = off, set()
            ids.add(id(p))
            self.bucket_of[id(p)] = len(self.buckets)
            off += n
        if ids:
            self.buckets.append((start, off, ids))
        self.works = []
        self.pending = None
        self.issued = None
        self.active = False

    def begin(self):
        self.pending = [set(b[2]) for b in self.buckets]
        self.issued = [False] * len(self.buckets)
        self.works = []
        self.active = dist.is_initialized() and (dist.get_world_size(self.group) > 1 or self.force)
        self.gb.reducer = self if self.active else None

    def _issue(self, k):
        s, e, _ = self.buckets[k]
        t = self.gb.flat[s:e]
        gloo = dist.get_backend(self.group) == "gloo"
        op = dist.ReduceOp.SUM if gloo else dist.ReduceOp.AVG
        self.works.append((dist.all_reduce(t, op=op, group=self.group, async_op=True), t, gloo))
        self.issued[k] = True

    def ready(self, params):
        if not self.active:
            return
        for p in params:
            k = self.bucket_of.get(id(p))
            if k is None or self.issued[k]:
                continue
            self.pending[k].discard(id(p))
            if not self.pending[k]:
                self._issue(k)

    def finish(self):
        """Issue the remaining buckets, then order the current stream after every all-reduce.
        Returns the number of buckets that were issued during backward (overlapped)."""
        if not self.active:
            return 0
        early = sum(self.issued)
        for k in range(len(self.buckets)):
            if not self.issued[k]:
                self._issue(k)
        world = dist.get_world_size(self.group)
        for w, t, gloo in self.works:
            w.wait()
            if gloo:
                t.div_(world)
        self.works = []
        self.active = False
        self.gb.reducer = None
        return early
