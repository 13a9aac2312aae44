"""Batched training step of the plastic U-Net (the hot loop of src/train.py:91-112, batched).

    trainer = Trainer(net, lr=3e-4, steplr=1e5)     # FusedAdam + StepLR(gamma .666), per step
    loss, hebb = trainer.step(x, t, hebb)           # fwd -> BCE -> bwd (+ overlapped RCCL all-reduce) -> Adam

Batched semantics: slot b of step s carries its trace to slot b of step
s+1; loss = mean BCE over all slots' pixels (so each slot contributes the reference's per-sample
gradient / B).  Under data parallelism each rank runs its own slots (the global batch is sharded
contiguously by rank) and gradients are averaged across ranks; traces stay per rank.
"""
import torch
import torch.distributed as dist

from . import dp
from .head import bce_loss
from .optim import FusedAdam


class Trainer:
    def __init__(self, net, lr=3e-4, steplr=1e5, gamma=0.666, betas=(0.9, 0.999), eps=1e-8,
                 flat_grads=True, bucket_mb=16, overlap=True, force_reduce=False):
        """force_reduce: run the overlapped all-reduce path even in a world of one rank (tests the
        RCCL async path on a one-GPU box; an AVG over one rank is the identity)"""
        self.net = net
        self.params = list(net.parameters())
        self.opt = FusedAdam(net.parameters(), lr=lr, betas=betas, eps=eps)
        self.sched = torch.optim.lr_scheduler.StepLR(self.opt, gamma=gamma, step_size=int(steplr))
        self.bucket_mb = bucket_mb
        self.gradbuf = None
        self.reducer = None
        self.distributed = dist.is_initialized() and (dist.get_world_size() > 1 or force_reduce)
        if flat_grads and hasattr(net, "_trunk_plan"):
            # flat buffer in gradient-completion order: head (w, alpha), then the trunk's backward order
            trunk = net._trunk_plan()
            order = [net.w, net.alpha] + trunk.backward_order()
            seen = set(id(p) for p in order)
            order += [p for p in self.params if id(p) not in seen]
            trainable = [p for p in order if p is not net.eta]
            self.gradbuf = dp.GradBuffer(trainable, next(net.parameters()).device)
            trunk.gradbuf = self.gradbuf
            if self.distributed and overlap:
                self.reducer = dp.BucketReducer(self.gradbuf, bucket_mb=bucket_mb, force=force_reduce)
        self.overlapped_buckets = 0
        # all-reduce accounting (bench.py's `allreduce` block): set measure_allreduce = True and
        # every step appends (buckets issued, issued during backward, exposed ms) to allreduce_log.
        # Exposed time = the compute stream's wait for the collectives: a HIP event after the last
        # backward kernel is enqueued and one after finish() has ordered the stream behind every
        # bucket (on a CPU / gloo group: the host wall time of finish()).
        self.measure_allreduce = False
        self.allreduce_log = []

    def allreduce_info(self):
        """Static bucket layout of the overlapped reducer (None when it is not active)."""
        if self.reducer is None:
            return None
        return {"buckets": len(self.reducer.buckets),
                "bucket_mb": [round((e - s) * 4 / 1e6, 3) for s, e, _ in self.reducer.buckets],
                "grad_mb": round(self.gradbuf.flat.numel() * 4 / 1e6, 3),
                "nominal_bucket_mb": self.bucket_mb}

    def allreduce_stats(self):
        """Per-step averages over allreduce_log (call after the steps have been synchronised)."""
        if not self.allreduce_log:
            return None
        n = len(self.allreduce_log)
        exposed = []
        for issued, early, ev in self.allreduce_log:
            exposed.append(ev[0].elapsed_time(ev[1]) if isinstance(ev, tuple) else ev)
        return {"steps": n, "buckets_issued": sum(r[0] for r in self.allreduce_log) / n,
                "buckets_overlapped": sum(r[1] for r in self.allreduce_log) / n,
                "exposed_ms_per_step": round(sum(exposed) / n, 4)}

    def _finish_reduce(self):
        if not self.measure_allreduce:
            return self.reducer.finish()
        import time
        issued = len(self.reducer.buckets)
        if self.gradbuf.flat.is_cuda:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            early = self.reducer.finish()
            e1.record()
            self.allreduce_log.append((issued, early, (e0, e1)))
        else:
            t0 = time.perf_counter()
            early = self.reducer.finish()
            self.allreduce_log.append((issued, early, (time.perf_counter() - t0) * 1e3))
        return early

    def step(self, x, t, hebb):
        """One optimisation step on the local batch.  Returns (loss tensor, new hebb), both
        detached and still on the device (no host synchronisation)."""
        for p in self.params:
            p.grad = None
        y, hn = self.net(x, hebb.detach())
        loss = bce_loss(y, t)
        if self.reducer is not None:
            self.reducer.begin()          # buckets all-reduce (async) as the backward completes them
        loss.backward()
        if self.reducer is not None:
            self.overlapped_buckets = self._finish_reduce()
            if not self.gradbuf.owns_grads():       # grads did not land in the buffer: reduce them
                dp.allreduce_grads(self.params, None)
        elif self.distributed:
            dp.allreduce_grads(self.params, self.gradbuf, bucket_mb=self.bucket_mb)
        self.opt.step()
        self.sched.step()
        return loss.detach(), hn.detach()
