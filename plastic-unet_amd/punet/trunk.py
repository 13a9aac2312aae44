"""The U-Net trunk of UNetp as one autograd node whose forward and backward are sequences of
HIP kernel launches (no ATen compute ops).

Reference: yaricom/Plastic-UNet src/unet/unet_p.py:54-67 (forward) and the blocks at :179-260;
the backward is what ``loss.backward()`` (src/train.py:110) runs through ATen on the CPU.

Forward (NHWC, fp32), per stage:
  inc     : conv3x3+ReLU, conv3x3+ReLU
  down_i  : MaxPool2d(2) -> conv3x3+ReLU -> conv3x3+ReLU
  up_j    : ConvT2x2s2 (GEMM + pixel-shuffle epilogue) -> conv3x3+ReLU over [skip | upsampled]
            read from two buffers (no concat copy) -> conv3x3+ReLU
  outc    : 1x1 conv C -> 1 (logits)
The CoordConv U-Net of src/coord_conv_script.py:146-200 (config C4) is the same schedule with a
stem - AddCoords fused into the input transpose (pu_add_coords) + 1x1 conv + ReLU - and Keras-style
up stages: ConvT2x2s2 halving the channels and the concat [upsampled | skip] (upsampled FIRST).
Backward fuses every ReLU mask into the producing kernel's epilogue (dgrad / maxpool-bwd /
outconv-bwd multiply by (activation > 0)), writes skip gradients once and lets the max-pool
backward accumulate into them, and gets bias gradients from the weight-gradient GEMM (a ones
column / ones row), so no separate elementwise or reduction passes run.
"""
import os

import torch

from . import kernels as K
from ._lib import PU_PACK_CONV_FWD, PU_PACK_CONV_DGRAD, PU_PACK_CONVT_FWD, PU_PACK_CONVT_DGRAD


# Weight-gradient side stream: the backward enqueues every weight gradient (and its split
# reduction) on a second stream, ordered after the kernel that produced its dZ, so they overlap the
# data-gradient chain.  PU_WSTREAM=1 always, 0 never, unset: bf16 trunks only - measured
# (profiles/r05_experiments/side_stream_ab.txt): C3 (bf16) 8822 -> 8952 img/s, C2 (fp32) 4370 ->
# 4317: the fp32 Winograd kernels hold a whole CU per block (LDS + 2 x 256 VGPRs per SIMD), so
# concurrent launches only queue behind each other and slow both.
_SIDE = {"1": True, "0": False}.get(os.environ.get("PU_WSTREAM", ""), "bf16")


# PU_STEM_BF16=0: the bf16 trunk's stem writes fp32 and converts (A/B runs)
_STEM_BF16 = os.environ.get("PU_STEM_BF16", "1") != "0"
# PU_LAZY_DIRECT=0: refresh every packed direct operand after each optimizer step (A/B runs)
_LAZY = os.environ.get("PU_LAZY_DIRECT", "1") != "0"


class _OnStream:
    """torch.cuda.stream(s) without its per-call device resolution (host time on the backward's
    issue path): make s current, restore the previous stream of s's device on exit."""
    __slots__ = ("s", "prev")

    def __init__(self, s):
        self.s = s

    def __enter__(self):
        self.prev = torch.cuda.current_stream(self.s.device_index)
        torch.cuda.set_stream(self.s)

    def __exit__(self, *exc):
        torch.cuda.set_stream(self.prev)
        return False


def set_side_stream(on):
    """Switch the weight-gradient side stream for backward passes started after this call:
    True / False, or "bf16" (the default: bf16 trunks only)."""
    global _SIDE
    _SIDE = on if on == "bf16" else bool(on)


class _Packs:
    """Packed GEMM operands of the OIHW parameters, rebuilt only when a parameter changes.

    The cache keys on the parameter's storage and checks its version counter (the optimizer and
    the DP broadcast bump it).  ``refresh()`` - called once at the start of every trunk forward -
    re-packs every stale entry in place with ONE multi-tensor launch (pu_pack_weights: pack + exact
    bf16 split fused) instead of two launches per operand at first use."""

    def __init__(self):
        self.cache = {}

    def get(self, w, mode, k_pad, cgroup=0, dtype=torch.float32):
        # keyed by storage (detached views share the parameter's version counter)
        key = (w.data_ptr(), tuple(w.shape), mode, cgroup, dtype)
        ver = w._version
        hit = self.cache.get(key)
        if hit is not None and hit[0] == ver and hit[1]._pack_spec[1] == k_pad:
            return hit[1]
        packed = K.pack_weight(w.detach(), mode, k_pad, cgroup=cgroup, dtype=dtype)
        self.cache[key] = (ver, packed, w)
        return packed

    def refresh(self):
        stale = [(key, w, packed) for key, (ver, packed, w) in self.cache.items()
                 if w._version != ver and w.data_ptr() == key[0]]
        if stale:
            # operands only ever used by the Winograd kernel get their U refreshed, not the
            # direct operand (K._ensure_direct repacks it if a call ever needs it)
            direct = [(w.detach(), packed, getattr(packed, "_split6", None)) for _, w, packed in stale
                      if not (_LAZY and getattr(packed, "_wino_only", False))]
            K.pack_weights(direct, wino=False)
            K.pack_wino([(w.detach(), packed._wino, packed._pack_spec[0] == 1) for _, w, packed in stale
                         if getattr(packed, "_wino", None) is not None])
            for key, w, packed in stale:
                if _LAZY and getattr(packed, "_wino_only", False):
                    packed._direct_ok = False
                self.cache[key] = (w._version, packed, w)


def _grad_sinks(trunk, outc):
    """Views of trunk.gradbuf for trunk.params, or None when a parameter already holds a .grad
    (the backward would then accumulate into an aliased buffer).  With trunk.fused_head the
    outconv weight/bias (params[outc], params[outc+1]) belong to the head: its backward runs first
    and autograd has already adopted their views, so they are not checked."""
    gb = trunk.gradbuf
    if gb is None:
        return None
    skip = (outc, outc + 1) if trunk.fused_head else ()
    if any(p.grad is not None for i, p in enumerate(trunk.params) if i not in skip):
        return None
    return [gb.view_for(p) for p in trunk.params]


def _kp(k, dt):
    """K padded to the kernel's stage: 16 fp32 or 32 bf16 values."""
    return K.round16(k) if dt == torch.float32 else (k + 31) // 32 * 32


def _cg(dt, c0, c1=0):
    """K order of a packed operand: the fp32 kernels' 16/32-channel groups, or 32 for bf16."""
    if dt == torch.float32:
        return K.cgroup_for(c0, c1)
    if c0 % 32 or c1 % 32:
        raise RuntimeError("bf16 convolutions need channel counts that are multiples of 32 (got %d, %d)" % (c0, c1))
    return 32


def conv3x3(x0, w, b, packs, x1=None, relu=True, out_dtype=None):
    """3x3/p1 conv (+bias, ReLU) over the channel concat [x0 | x1] (NHWC).  out_dtype bf16 with an
    fp32 single-channel x0: the stem writes the bf16 trunk's first activation directly."""
    B, H, W, c0 = x0.shape
    c1 = 0 if x1 is None else x1.shape[3]
    cout = w.shape[0]
    dt = x0.dtype
    k_pad = _kp(9 * (c0 + c1), dt)
    g = _cg(dt, c0, c1)
    out = torch.empty(B, H, W, cout, dtype=out_dtype or dt, device=x0.device)
    K.igemm(batch=B, in_hw=(H, W), out_hw=(H, W), k=3, stride=1, pad=1, src0=x0, c0=c0, src1=x1, c1=c1,
            weight=packs.get(w, PU_PACK_CONV_FWD, k_pad, g, dt), k_pad=k_pad, n=cout, bias=b, dst0=out, relu=relu,
            cgroup=g)
    return out


def conv3x3_dgrad(dz, w, packs, split=None, mask0=None, mask1=None):
    """dX = conv(dZ, flipped W^T); optional channel split [0,split) -> d0, rest -> d1 and masks."""
    B, H, W, cout = dz.shape
    cin = w.shape[1]
    dt = dz.dtype
    k_pad = _kp(9 * cout, dt)
    g = _cg(dt, cout)
    n0 = cin if split is None else split
    d0 = torch.empty(B, H, W, n0, dtype=dt, device=dz.device)
    d1 = None if split is None else torch.empty(B, H, W, cin - n0, dtype=dt, device=dz.device)
    K.igemm(batch=B, in_hw=(H, W), out_hw=(H, W), k=3, stride=1, pad=1, src0=dz, c0=cout,
            weight=packs.get(w, PU_PACK_CONV_DGRAD, k_pad, g, dt), k_pad=k_pad, n=cin, dst0=d0, n0=n0, dst1=d1,
            mask0=mask0, mask1=mask1, cgroup=g)
    return d0, d1


def conv3x3_wgrad(dz, x0, x1=None, out=None):
    B, H, W, cout = dz.shape
    c0 = x0.shape[3]
    c1 = 0 if x1 is None else x1.shape[3]
    if out is None:
        dw = torch.empty(cout, c0 + c1, 3, 3, dtype=torch.float32, device=dz.device)
        db = torch.empty(cout, dtype=torch.float32, device=dz.device)
    else:
        dw, db = out
    K.wgrad(batch=B, in_hw=(H, W), out_hw=(H, W), k=3, stride=1, pad=1, rows=dz, n=cout, src0=x0, c0=c0,
            src1=x1, c1=c1, bias_mode=1, dweight=dw, dbias=db)
    return dw, db


def convT2x2(x, w, b, packs):
    """ConvTranspose2d(cin, cout, 2, stride=2): GEMM [B*h*w, cin] x [cin, 4*cout] + pixel shuffle."""
    B, h, wd, cin = x.shape
    cout = w.shape[1]
    dt = x.dtype
    k_pad = _kp(cin, dt)
    out = torch.empty(B, 2 * h, 2 * wd, cout, dtype=dt, device=x.device)
    K.igemm(batch=B, in_hw=(h, wd), out_hw=(h, wd), k=1, stride=1, pad=0, src0=x, c0=cin,
            weight=packs.get(w, PU_PACK_CONVT_FWD, k_pad, 0, dt), k_pad=k_pad, n=4 * cout, bias=b, dst0=out,
            shuffle=True)
    return out


def convT2x2_dgrad(du, w, packs, mask):
    """dX[b,h,w,:] = sum_(i,j) dU[b,2h+i,2w+j,:] W[:, :, i, j]^T, times (mask > 0)."""
    B, H2, W2, cout = du.shape
    cin = w.shape[0]
    dt = du.dtype
    k_pad = _kp(4 * cout, dt)
    g = _cg(dt, cout)
    dx = torch.empty(B, H2 // 2, W2 // 2, cin, dtype=dt, device=du.device)
    K.igemm(batch=B, in_hw=(H2, W2), out_hw=(H2 // 2, W2 // 2), k=2, stride=2, pad=0, src0=du, c0=cout,
            weight=packs.get(w, PU_PACK_CONVT_DGRAD, k_pad, g, dt), k_pad=k_pad, n=cin, dst0=dx, mask0=mask,
            cgroup=g)
    return dx


def convT2x2_wgrad(x, du, out=None):
    B, h, wd, cin = x.shape
    cout = du.shape[3]
    if out is None:
        dw = torch.empty(cin, cout, 2, 2, dtype=torch.float32, device=x.device)
        db = torch.empty(cout, dtype=torch.float32, device=x.device)
    else:
        dw, db = out
    K.wgrad(batch=B, in_hw=(2 * h, 2 * wd), out_hw=(h, wd), k=2, stride=2, pad=0, rows=x, n=cin, src0=du,
            c0=cout, bias_mode=2, dweight=dw, dbias=db)
    return dw, db


def as_nhwc_input(x):
    """Model input [B,C,H,W] -> NHWC.  C == 1 is already NHWC in memory."""
    x = x.contiguous()
    if x.shape[1] == 1:
        B, _, H, W = x.shape
        return x.view(B, H, W, 1)
    return K.nchw_to_nhwc(x)


class UNetpTrunk:
    """Parameter order and kernel schedule of the generalised UNetp trunk (depth D).  Models with a
    ``coord`` stem (CoordConvUNetp) get its w,b appended after outc and ``up_first`` concats.

    Variants of the reference's constructor flags (unet_p.py:9-52):
      batch_norm=True         (:186-193) each conv is Conv -> BatchNorm2d -> ReLU: the conv epilogue
                              keeps bias only, punet.kernels.bn_fwd normalises slot by slot (the
                              reference's batch size 1) and applies the ReLU; backward runs bn_bwd
                              on the masked gradient before the conv's wgrad / dgrad
      bilinear_upsample=True  (:235-236) nn.Upsample(2, bilinear, align_corners=True) in place of
                              the ConvTranspose2d: no parameters, gather-form backward
    """

    def __init__(self, model):
        self.depth = model.depth
        self.coord = getattr(model, "coord", None)
        self.with_r = bool(getattr(model, "with_r", False))
        self.up_first = bool(getattr(model, "up_first", False))
        # activations dtype: float32, or bfloat16 (config C3; fp32 accumulation, fp32 parameters
        # and gradients; the 1-channel stem conv runs in fp32 and its output is rounded once)
        self.dtype = getattr(model, "compute_dtype", torch.float32)
        self.bilinear = bool(getattr(model, "bilinear_upsample", False))
        self.training = True
        self.names = []
        self.packs = _Packs()
        seqs = {"inc": model.inc.conv.conv}
        for i in range(1, self.depth):
            seqs["down%d" % i] = getattr(model, "down%d" % i).mpconv[1].conv
        for j in range(1, self.depth):
            seqs["up%d" % j] = getattr(model, "up%d" % j).conv.conv
        self.params = []
        self.slot = {}           # conv key ("inc.c0", "up2.up", "outc", ...) -> index of its weight
        self.bn = {}             # conv key -> its BatchNorm2d module
        bn_mods = []

        def add(key, w, b):
            self.slot[key] = len(self.params)
            self.params += [w, b]

        # order: inc c0 w,b, c1 w,b ; down_i ... ; up_j: [up w,b], c0 w,b, c1 w,b ; outc w,b ;
        # [coord w,b] ; then the BatchNorm affine parameters (w,b) in conv order
        def add_double(name):
            convs = [m for m in seqs[name] if isinstance(m, torch.nn.Conv2d)]
            norms = [m for m in seqs[name] if isinstance(m, torch.nn.BatchNorm2d)]
            for idx, cm in enumerate(convs):
                add("%s.c%d" % (name, idx), cm.weight, cm.bias)
                if norms:
                    bn_mods.append(("%s.c%d" % (name, idx), norms[idx]))

        add_double("inc")
        for i in range(1, self.depth):
            add_double("down%d" % i)
        for j in range(1, self.depth):
            upm = getattr(model, "up%d" % j).up
            if isinstance(upm, torch.nn.ConvTranspose2d):
                add("up%d.up" % j, upm.weight, upm.bias)
            elif not self.bilinear:
                raise RuntimeError("up%d.up is neither ConvTranspose2d nor bilinear" % j)
            add_double("up%d" % j)
        add("outc", model.outc.conv.weight, model.outc.conv.bias)
        if self.coord is not None:
            add("coord", self.coord.conv.weight, self.coord.conv.bias)
        self.n_core = len(self.params)
        for key, m in bn_mods:
            if m.momentum is None:
                raise NotImplementedError("BatchNorm2d(momentum=None) (cumulative averaging) is not built")
            self.bn[key] = m
            self.slot[key + ".bn"] = len(self.params)
            self.params += [m.weight, m.bias]
        if (self.bn or self.bilinear) and self.dtype != torch.float32:
            raise NotImplementedError("batch_norm / bilinear_upsample run in fp32 (precision='fp32')")
        self.gradbuf = None      # punet.dp.GradBuffer: backward writes grads into its views
        self.debug = None        # dict: when set, backward stores each layer's dZ (tests/diagnostics)
        # True: forward returns the last activation (the outconv runs inside the fused head,
        # punet.head.FusedHeadFunction) and backward receives dL/d(its pre-ReLU) from the head
        self.fused_head = False
        self._ws = None          # weight-gradient side stream (PU_WSTREAM), created on first use
        self._side = None        # the side stream while a backward runs with it, else None

    def _stem_bf16(self, x):
        """bf16 trunk whose first conv is the single-channel stem (no BatchNorm): it writes its bf16
        output directly (PU_EPI_OUT_BF16) and its weight gradient reads the bf16 dZ (pu_wgrad math
        2) - no fp32 copies and conversion passes."""
        return (_STEM_BF16 and self.dtype == torch.bfloat16 and x.dim() == 4 and x.shape[3] == 1 and "inc.c0" not in self.bn
                and self.params[self.slot["inc.c0"]].shape[0] in (8, 16, 32, 64))

    def backward_order(self):
        """Parameters in the order backward() completes their gradients (outc first, stem last;
        each BatchNorm pair completes just before its conv)."""
        order = []
        core = self.params[:self.n_core]
        if self.coord is not None:
            core = core[:-2]
        bn_of = {self.slot[k]: self.slot[k + ".bn"] for k in self.bn}
        for idx in range(len(core) - 2, -2, -2):
            if idx in bn_of:
                j = bn_of[idx]
                order += [self.params[j + 1], self.params[j]]
            order += [core[idx + 1], core[idx]]
        if self.coord is not None:
            order += self.params[self.n_core - 2:self.n_core]
        return order

    def _ready(self, i, n=2):
        """params[i:i+n]'s gradient kernels are enqueued: let an armed BucketReducer know.  With
        the side stream the bucket is issued from it (RCCL then orders after the stream's weight
        gradients), after the stream has caught up with the compute stream (BatchNorm grads)."""
        gb = self.gradbuf
        if gb is None or gb.reducer is None:
            return
        ws = self._side
        if ws is None:
            gb.ready(*self.params[i:i + n])
            return
        ws.wait_stream(torch.cuda.current_stream(ws.device_index))
        with _OnStream(ws):
            gb.ready(*self.params[i:i + n])

    def _wgrad(self, fn, i, out, *reads):
        """Run weight-gradient launcher fn(out) for params[i:i+2] - on the side stream when one is
        active: the stream waits for the compute stream (dZ is its last kernel), the outputs are
        allocated on the compute stream (autograd and the optimizer use them there) and every
        tensor the side stream reads is recorded against it, so the caching allocator does not
        hand its memory out again before the side stream is done with it."""
        ws = self._side
        if ws is None:
            r = fn(out)
        else:
            if out is None:
                out = (torch.empty_like(self.params[i], memory_format=torch.contiguous_format),
                       torch.empty_like(self.params[i + 1]))
            ws.wait_stream(torch.cuda.current_stream(ws.device_index))
            with _OnStream(ws):
                r = fn(out)
            for t in reads:
                if t is not None:
                    t.record_stream(ws)
        self._ready(i)
        return r

    def grad_sinks(self):
        """Views of the flat gradient buffer to write into, or None.  Only used when every
        parameter's .grad is None (autograd then adopts the views; if a .grad already existed it
        would accumulate into an aliased buffer).  With the fused head the outconv parameters
        are the head's (its backward runs first and writes their views), so they do not count."""
        return _grad_sinks(self, self.slot["outc"])

    # -------------------------------------------------------------------------------- forward
    def _conv(self, key, P, s, x0, x1=None, out_dtype=None):
        """conv3x3 (+ BatchNorm) + ReLU of conv `key` over [x0 | x1]."""
        i = self.slot[key]
        bnm = self.bn.get(key)
        if bnm is None:
            return conv3x3(x0, P[i], P[i + 1], self.packs, x1=x1, out_dtype=out_dtype)
        z = conv3x3(x0, P[i], P[i + 1], self.packs, x1=x1, relu=False)
        j = self.slot[key + ".bn"]
        training = self.training or not bnm.track_running_stats
        update = self.training and bnm.track_running_stats
        y, mean, rstd = K.bn_fwd(z, P[j], P[j + 1], bnm.running_mean if (update or not training) else None,
                                 bnm.running_var if (update or not training) else None, bnm.eps, bnm.momentum,
                                 training)
        if update:
            bnm.num_batches_tracked.add_(z.shape[0])     # one reference forward per slot
        if s is not None:
            s[key + ".z"] = z
            s[key + ".stat"] = (mean, rstd)
        return y

    def forward(self, x, params, save):
        P = params
        D = self.depth
        pk = self.packs
        pk.refresh()                   # operands of parameters the optimizer moved: one launch
        s = {"x": x}
        if self.coord is not None:     # stem: 1x1 conv + ReLU over the AddCoords input
            ci = self.slot["coord"]
            cw, cb = P[ci], P[ci + 1]
            B, H, W, ca = x.shape
            x = torch.empty(B, H, W, cw.shape[0], dtype=torch.float32, device=cw.device)
            K.igemm(batch=B, in_hw=(H, W), out_hw=(H, W), k=1, stride=1, pad=0, src0=s["x"], c0=ca,
                    weight=pk.get(cw, PU_PACK_CONV_FWD, K.round16(ca)), k_pad=K.round16(ca), n=cw.shape[0],
                    bias=cb, dst0=x, relu=True)
            s["stem"] = x
        t = self._conv("inc.c0", P, s, x, out_dtype=torch.bfloat16 if self._stem_bf16(x) else None)
        if self.dtype != t.dtype:
            t = K.to_bf16(t)
        s["inc.t"] = t
        y = self._conv("inc.c1", P, s, t)
        skips = [y]
        for i in range(1, D):
            p = K.maxpool2_fwd(skips[-1]); s["down%d.p" % i] = p
            t = self._conv("down%d.c0" % i, P, s, p); s["down%d.t" % i] = t
            y = self._conv("down%d.c1" % i, P, s, t)
            skips.append(y)
        s["skips"] = skips
        y = skips[-1]
        for j in range(1, D):
            skip = skips[D - 1 - j]
            if self.bilinear:
                u = K.upsample_bilinear2x(y)
            else:
                ui = self.slot["up%d.up" % j]
                u = convT2x2(y, P[ui], P[ui + 1], pk)
            s["up%d.u" % j] = u
            if self.up_first:
                t = self._conv("up%d.c0" % j, P, s, u, skip)
            else:
                t = self._conv("up%d.c0" % j, P, s, skip, u)
            s["up%d.t" % j] = t
            y = self._conv("up%d.c1" % j, P, s, t)
            s["up%d.y" % j] = y
        if self.fused_head:
            return y, (s if save else None)
        o = self.slot["outc"]
        logits = K.outconv_fwd(y, P[o].reshape(-1), P[o + 1])
        return logits, (s if save else None)

    # ------------------------------------------------------------------------------- backward
    def _bn_back(self, key, g, s, P, grads, out):
        """g = dL/d(BN output) (ReLU mask applied) -> dL/dz of conv `key`; BatchNorm grads."""
        if key not in self.bn:
            return g
        j = self.slot[key + ".bn"]
        o = out(j)
        mean, rstd = s[key + ".stat"]
        dgam = torch.empty_like(P[j]) if o is None else o[0]
        dbet = torch.empty_like(P[j + 1]) if o is None else o[1]
        dz = K.bn_bwd(s[key + ".z"], g, mean, rstd, P[j], dgam, dbet)
        grads[j], grads[j + 1] = dgam, dbet
        self._ready(j)
        return dz

    def backward(self, s, dlogits, params):
        if dlogits.is_cuda and (_SIDE is True or (_SIDE == "bf16" and self.dtype == torch.bfloat16)):
            if self._ws is None or self._ws.device != dlogits.device:
                self._ws = torch.cuda.Stream(device=dlogits.device)
            self._side = self._ws
        try:
            return self._backward(s, dlogits, params)
        finally:
            if self._side is not None:
                torch.cuda.current_stream(self._side.device_index).wait_stream(self._side)   # grads complete before use
                self._side = None

    def _backward(self, s, dlogits, params):
        D = self.depth
        pk = self.packs
        P = list(params)
        grads = [None] * len(P)
        sink = self.grad_sinks()
        out = (lambda i: None) if sink is None else (lambda i: (sink[i], sink[i + 1]))  # noqa: E731
        sl = self.slot
        skips = s["skips"]

        y_last = s["up%d.y" % (D - 1)]
        outc = sl["outc"]
        if self.fused_head:
            g = dlogits                  # the fused head's outconv backward already applied the mask
        else:
            o = out(outc)
            g, dwo, dbo = K.outconv_bwd(y_last, P[outc].reshape(-1), dlogits, relu_mask=True,
                                        out=None if o is None else (o[0].view(-1), o[1]))
            grads[outc] = dwo.view_as(P[outc])
            grads[outc + 1] = dbo
            self._ready(outc)

        gskip = [None] * (D - 1)
        for j in range(D - 1, 0, -1):
            c0, c1 = sl["up%d.c0" % j], sl["up%d.c1" % j]
            t = s["up%d.t" % j]
            u = s["up%d.u" % j]
            skip = skips[D - 1 - j]
            y_prev = skips[D - 1] if j == 1 else s["up%d.y" % (j - 1)]
            if self.debug is not None:
                self.debug["up%d.c1" % j] = g
            # conv1 of up_j: y_j = relu([bn](conv(t)));  g = dL/d(pre-ReLU)
            g = self._bn_back("up%d.c1" % j, g, s, P, grads, out)
            grads[c1], grads[c1 + 1] = self._wgrad(lambda o: conv3x3_wgrad(g, t, out=o), c1, out(c1), g, t)
            dt, _ = conv3x3_dgrad(g, P[c1], pk, mask0=t)
            dt = self._bn_back("up%d.c0" % j, dt, s, P, grads, out)
            # conv0 over [skip | u]  (up_first: [u | skip])
            if self.up_first:
                grads[c0], grads[c0 + 1] = self._wgrad(lambda o: conv3x3_wgrad(dt, u, skip, out=o), c0, out(c0),
                                                       dt, u, skip)
                du, dskip = conv3x3_dgrad(dt, P[c0], pk, split=u.shape[3], mask1=skip)
            else:
                grads[c0], grads[c0 + 1] = self._wgrad(lambda o: conv3x3_wgrad(dt, skip, u, out=o), c0, out(c0),
                                                       dt, skip, u)
                dskip, du = conv3x3_dgrad(dt, P[c0], pk, split=skip.shape[3], mask0=skip)
            if self.debug is not None:
                self.debug["up%d.c0" % j] = dt
                self.debug["up%d.up" % j] = du
            gskip[D - 1 - j] = dskip
            if self.bilinear:
                g = K.upsample_bilinear2x_bwd(du, mask=y_prev)
            else:
                ui = sl["up%d.up" % j]
                grads[ui], grads[ui + 1] = self._wgrad(lambda o: convT2x2_wgrad(y_prev, du, out=o), ui, out(ui),
                                                       y_prev, du)
                g = convT2x2_dgrad(du, P[ui], pk, mask=y_prev)

        for i in range(D - 1, 0, -1):
            c0, c1 = sl["down%d.c0" % i], sl["down%d.c1" % i]
            t = s["down%d.t" % i]
            p = s["down%d.p" % i]
            if self.debug is not None:
                self.debug["down%d.c1" % i] = g
            g = self._bn_back("down%d.c1" % i, g, s, P, grads, out)
            grads[c1], grads[c1 + 1] = self._wgrad(lambda o: conv3x3_wgrad(g, t, out=o), c1, out(c1), g, t)
            dt, _ = conv3x3_dgrad(g, P[c1], pk, mask0=t)
            dt = self._bn_back("down%d.c0" % i, dt, s, P, grads, out)
            grads[c0], grads[c0 + 1] = self._wgrad(lambda o: conv3x3_wgrad(dt, p, out=o), c0, out(c0), dt, p)
            if self.debug is not None:
                self.debug["down%d.c0" % i] = dt
            dp, _ = conv3x3_dgrad(dt, P[c0], pk)
            g = K.maxpool2_bwd(skips[i - 1], dp, gskip[i - 1], relu_mask=True, accumulate=True)

        t = s["inc.t"]
        c0, c1 = sl["inc.c0"], sl["inc.c1"]
        if self.debug is not None:
            self.debug["inc.c1"] = g
        g = self._bn_back("inc.c1", g, s, P, grads, out)
        grads[c1], grads[c1 + 1] = self._wgrad(lambda o: conv3x3_wgrad(g, t, out=o), c1, out(c1), g, t)
        dt, _ = conv3x3_dgrad(g, P[c1], pk, mask0=t)
        x0 = s["stem"] if self.coord is not None else s["x"]
        if dt.dtype != x0.dtype and not self._stem_bf16(x0):   # bf16 trunk: the fp32 stem's weight gradient
            dt = K.to_f32(dt)
        dt = self._bn_back("inc.c0", dt, s, P, grads, out)
        grads[c0], grads[c0 + 1] = self._wgrad(lambda o: conv3x3_wgrad(dt, x0, out=o), c0, out(c0), dt, x0)
        if self.debug is not None:
            self.debug["inc.c0"] = dt
        if self.coord is not None:     # stem 1x1 conv: dgrad of inc.c0 (masked by the stem ReLU) + wgrad
            dstem, _ = conv3x3_dgrad(dt, P[c0], pk, mask0=x0)
            B, H, W, ca = s["x"].shape
            cs = sl["coord"]
            o = out(cs)
            dw = torch.empty(P[cs].shape, dtype=torch.float32, device=dt.device) if o is None else o[0]
            db = torch.empty(P[cs + 1].shape, dtype=torch.float32, device=dt.device) if o is None else o[1]

            def stem_wgrad(o):
                K.wgrad(batch=B, in_hw=(H, W), out_hw=(H, W), k=1, stride=1, pad=0, rows=dstem,
                        n=P[cs].shape[0], src0=s["x"], c0=ca, bias_mode=1, dweight=o[0], dbias=o[1])
                return o
            grads[cs], grads[cs + 1] = self._wgrad(stem_wgrad, cs, (dw, db), dstem, s["x"])
        return grads


class TrunkFunction(torch.autograd.Function):
    """autograd node: (trunk, save, x NCHW, *trunk params) -> logits [B,H,W] (or, with
    trunk.fused_head, the last activation [B,H,W,C] for the fused head)."""

    @staticmethod
    def forward(ctx, trunk, save, x, *params):
        # ``save`` is decided by the caller: grad mode is always off inside Function.forward
        if trunk.coord is not None:
            xin = K.add_coords(x.detach().contiguous(), trunk.with_r)
        else:
            xin = as_nhwc_input(x.detach())
        detached = [p.detach() for p in params]
        logits, saved = trunk.forward(xin, detached, save)
        ctx.trunk = trunk
        ctx.saved_acts = saved
        ctx.params = detached
        return logits

    @staticmethod
    def backward(ctx, dlogits):
        if ctx.saved_acts is None:
            raise RuntimeError("trunk activations were not saved (forward ran without grad)")
        grads = ctx.trunk.backward(ctx.saved_acts, dlogits.contiguous(), ctx.params)
        ctx.saved_acts = None
        return (None, None, None) + tuple(grads)
