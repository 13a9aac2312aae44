"""Host -> HBM input pipeline of the training loop: double-buffered, pinned-memory, asynchronous.

The reference copies every sample to the device inside the hot loop (src/train.py:94-95,
``torch.from_numpy(...).to(device)`` per sample, synchronous).  Keeping the whole training set in
HBM instead does not scale past device memory, so batches stream:

  host numpy (any dtype, may be a memmap)  --np.copyto-->  pinned staging slot k
  pinned slot k  --async H2D on a copy stream-->  device slot k   (overlaps the previous step)
  compute stream waits on slot k's copy event, trains on it, then marks slot k consumed

``depth`` slots rotate (2 = double buffering).  A device slot is overwritten only after the
compute stream has recorded that it finished the step reading it; a pinned slot is refilled only
after the copy that read it has completed (host waits on that event).  On a CPU device the same
iterator degenerates to plain copies (test harness for the ordering logic; the product trains on
the GPU).
"""
import numpy as np
import torch


class BatchPrefetcher:
    """Iterate device batches ``(x, y)`` for the index ranges ``ranges`` of host arrays X, Y.

    X: [N, ...] inputs, Y: [N, ...] targets (numpy or torch CPU).  Yielded tensors are float32
    views of the device slot; they stay valid until the iterator advances ``depth - 1`` more
    times (the trainer consumes them within its step)."""

    def __init__(self, X, Y, ranges, device, depth=2):
        self.X, self.Y = X, Y
        self.ranges = list(ranges)
        self.device = torch.device(device)
        self.depth = max(2, int(depth))
        self.gpu = self.device.type == "cuda"
        bmax = max((hi - lo for lo, hi in self.ranges), default=0)
        xs, ys = tuple(np.shape(X)[1:]), tuple(np.shape(Y)[1:])
        self.host, self.dev = [], []
        for _ in range(self.depth if bmax else 0):
            hx = torch.empty((bmax,) + xs, dtype=torch.float32, pin_memory=self.gpu)
            hy = torch.empty((bmax,) + ys, dtype=torch.float32, pin_memory=self.gpu)
            self.host.append((hx, hy))
            self.dev.append((torch.empty((bmax,) + xs, dtype=torch.float32, device=self.device),
                             torch.empty((bmax,) + ys, dtype=torch.float32, device=self.device)))
        if self.gpu:
            self.stream = torch.cuda.Stream(self.device)
            self.copied = [torch.cuda.Event() for _ in range(self.depth)]
            self.consumed = [None] * self.depth
            self.pinned_busy = [None] * self.depth

    def __len__(self):
        return len(self.ranges)

    def _fill(self, i):
        """stage batch i into its pinned slot and issue its H2D copy"""
        k = i % self.depth
        lo, hi = self.ranges[i]
        n = hi - lo
        hx, hy = self.host[k]
        dx, dy = self.dev[k]
        if self.gpu and self.pinned_busy[k] is not None:
            self.pinned_busy[k].synchronize()      # the copy that last read this pinned slot is done
        np.copyto(hx[:n].numpy(), np.asarray(self.X[lo:hi]), casting="same_kind")
        np.copyto(hy[:n].numpy(), np.asarray(self.Y[lo:hi]), casting="same_kind")
        if not self.gpu:
            dx[:n].copy_(hx[:n])
            dy[:n].copy_(hy[:n])
            return
        with torch.cuda.stream(self.stream):
            if self.consumed[k] is not None:
                self.stream.wait_event(self.consumed[k])   # compute finished the step that read slot k
            dx[:n].copy_(hx[:n], non_blocking=True)
            dy[:n].copy_(hy[:n], non_blocking=True)
            self.copied[k].record(self.stream)
        self.pinned_busy[k] = self.copied[k]

    def __iter__(self):
        if not self.ranges:
            return
        if self.gpu:
            # a caller that stops iterating early (zip over the ranges ends before the generator
            # resumes past its last yield) never recorded the last slot's consumed event: order
            # every slot's next copy after all the compute work enqueued so far
            ev = torch.cuda.Event()
            ev.record(torch.cuda.current_stream(self.device))
            self.consumed = [ev] * self.depth
        for j in range(min(self.depth - 1, len(self.ranges))):
            self._fill(j)
        for i, (lo, hi) in enumerate(self.ranges):
            nxt = i + self.depth - 1
            if nxt < len(self.ranges):
                self._fill(nxt)
            k = i % self.depth
            n = hi - lo
            if self.gpu:
                torch.cuda.current_stream(self.device).wait_event(self.copied[k])
            dx, dy = self.dev[k]
            yield dx[:n], dy[:n]
            if self.gpu:
                ev = torch.cuda.Event()
                ev.record(torch.cuda.current_stream(self.device))
                self.consumed[k] = ev
