"""Batched training step of the plastic U-Net (the hot loop of src/train.py:91-112, batched).

    trainer = Trainer(net, lr=3e-4, steplr=1e5)     # FusedAdam + StepLR(gamma .666), per step
    loss, hebb = trainer.step(x, t, hebb)           # fwd -> BCE -> bwd (+ overlapped RCCL all-reduce) -> Adam

Trainer(..., graph=True) (one rank): after two eager steps the forward + BCE + backward of a step is
captured once into a HIP graph and replayed; the inputs are copied into the graph's static tensors
and the optimizer step runs eagerly after each replay.  The graph holds every kernel launch of the
step - the trunk's operand packing included (captured right after an optimizer step, when every
packed operand is stale) - so the host issues one graph launch instead of several hundred kernel
launches; the kernels and their order are the eager step's (bit-identical results).

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
                 flat_grads=True, bucket_mb=16, overlap=True, force_reduce=False, graph=False):
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
            if self.distributed and dist.get_world_size() > 1 and hasattr(trunk, "mask_gen") \
                    and trunk.mask_gen is None:
                # Dropout2d masks: independent per rank (the parameters are the broadcast ones)
                trunk.mask_gen = dp.rank_generator(next(net.parameters()).device)
        self.overlapped_buckets = 0
        # HIP-graph step (one rank only: the overlapped all-reduce issues collectives from the host
        # during backward); eager warm-up steps first, then capture
        self.graph = bool(graph) and not self.distributed
        self._graph = None
        self._graph_warm = 0
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
        detached and still on the device (no host synchronisation).  With graph=True the returned
        hebb is the graph's output tensor: the next step overwrites it (pass it back in as usual)."""
        if self.graph and x.is_cuda:
            if self._graph is not None or self._graph_warm >= 2:
                return self._graph_step(x, t, hebb)
            self._graph_warm += 1
        return self._eager_step(x, t, hebb)

    @staticmethod
    def _sig(net, *ts):
        return (net.training,) + tuple((tuple(a.shape), a.dtype, a.device) for a in ts)

    def _graph_step(self, x, t, hebb):
        if self._graph is not None and self._sig(self.net, x, t, hebb) != self._gsig:
            # copy_() would broadcast a different batch into the captured one, and an eval-mode
            # call would replay the training graph: anything but the captured step runs eagerly
            return self._eager_step(x, t, hebb)
        if self._graph is None:
            self._gsig = self._sig(self.net, x, t, hebb)
            # capture right after an (eager) optimizer step: every packed operand is stale, so the
            # trunk's refresh launches are part of the graph and run on every replay
            self._sx = x.detach().clone()
            self._st = t.detach().clone()
            self._sh = hebb.detach().clone()
            for p in self.params:
                p.grad = None
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                y, hn = self.net(self._sx, self._sh)
                loss = bce_loss(y, self._st)
                loss.backward()
            self._graph = g
            self._gloss, self._ghn = loss.detach(), hn.detach()
            self._ggrads = [p.grad for p in self.params]
        else:
            self._sx.copy_(x)
            self._st.copy_(t)
            if hebb is not self._sh:
                self._sh.copy_(hebb)
        self._graph.replay()
        # the gradients the graph writes (an eager step in between may have rebound .grad)
        for p, gr in zip(self.params, self._ggrads):
            p.grad = gr
        self.opt.step()
        self.sched.step()
        return self._gloss.clone(), self._ghn

    def _eager_step(self, x, t, hebb):
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
