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
import torch

from . import kernels as K
from ._lib import PU_PACK_CONV_FWD, PU_PACK_CONV_DGRAD, PU_PACK_CONVT_FWD, PU_PACK_CONVT_DGRAD


class _Packs:
    """Packed GEMM operands of the OIHW parameters, rebuilt only when a parameter changes."""

    def __init__(self):
        self.cache = {}

    def get(self, w, mode, k_pad, cgroup=0, dtype=torch.float32):
        # keyed by storage (detached views share the parameter's version counter)
        key = (w.data_ptr(), tuple(w.shape), mode, cgroup, dtype)
        ver = w._version
        hit = self.cache.get(key)
        if hit is not None and hit[0] == ver:
            return hit[1]
        packed = K.pack_weight(w.detach(), mode, k_pad, cgroup=cgroup, dtype=dtype)
        self.cache[key] = (ver, packed)
        return packed


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


def conv3x3(x0, w, b, packs, x1=None, relu=True):
    """3x3/p1 conv (+bias, ReLU) over the channel concat [x0 | x1] (NHWC)."""
    B, H, W, c0 = x0.shape
    c1 = 0 if x1 is None else x1.shape[3]
    cout = w.shape[0]
    dt = x0.dtype
    k_pad = _kp(9 * (c0 + c1), dt)
    g = _cg(dt, c0, c1)
    out = torch.empty(B, H, W, cout, dtype=dt, device=x0.device)
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
    ``coord`` stem (CoordConvUNetp) get its w,b appended after outc and ``up_first`` concats."""

    def __init__(self, model):
        self.depth = model.depth
        self.coord = getattr(model, "coord", None)
        self.with_r = bool(getattr(model, "with_r", False))
        self.up_first = bool(getattr(model, "up_first", False))
        # activations dtype: float32, or bfloat16 (config C3; fp32 accumulation, fp32 parameters
        # and gradients; the 1-channel stem conv runs in fp32 and its output is rounded once)
        self.dtype = getattr(model, "compute_dtype", torch.float32)
        self.names = []
        self.packs = _Packs()
        mods = {"inc": model.inc.conv.conv}
        for i in range(1, self.depth):
            mods["down%d" % i] = getattr(model, "down%d" % i).mpconv[1].conv
        for j in range(1, self.depth):
            up = getattr(model, "up%d" % j)
            mods["up%d.up" % j] = up.up
            mods["up%d" % j] = up.conv.conv
        self.params = []
        # order: inc c0 w,b, c1 w,b ; down_i ... ; up_j: up w,b, c0 w,b, c1 w,b ; outc w,b
        for key in ["inc"] + ["down%d" % i for i in range(1, self.depth)]:
            seq = mods[key]
            for idx in (0, 2):
                self.params += [seq[idx].weight, seq[idx].bias]
        for j in range(1, self.depth):
            upm = mods["up%d.up" % j]
            self.params += [upm.weight, upm.bias]
            seq = mods["up%d" % j]
            for idx in (0, 2):
                self.params += [seq[idx].weight, seq[idx].bias]
        self.params += [model.outc.conv.weight, model.outc.conv.bias]
        if self.coord is not None:
            self.params += [self.coord.conv.weight, self.coord.conv.bias]
        self.gradbuf = None      # punet.dp.GradBuffer: backward writes grads into its views
        self.debug = None        # dict: when set, backward stores each layer's dZ (tests/diagnostics)

    def backward_order(self):
        """Parameters in the order backward() completes their gradients (outc first, stem last)."""
        core = self.params[:-2] if self.coord is not None else self.params
        return list(reversed(core)) + (self.params[-2:] if self.coord is not None else [])

    def _ready(self, i, n=2):
        """params[i:i+n]'s gradient kernels are enqueued: let an armed BucketReducer know."""
        gb = self.gradbuf
        if gb is not None and gb.reducer is not None:
            gb.ready(*self.params[i:i + n])

    def grad_sinks(self):
        """Views of the flat gradient buffer to write into, or None.  Only used when every
        parameter's .grad is None (autograd then adopts the views; if a .grad already existed it
        would accumulate into an aliased buffer)."""
        gb = self.gradbuf
        if gb is None or any(p.grad is not None for p in self.params):
            return None
        return [gb.view_for(p) for p in self.params]

    # -------------------------------------------------------------------------------- forward
    def forward(self, x, params, save):
        it = iter(params)
        nxt = lambda: (next(it), next(it))  # noqa: E731
        D = self.depth
        pk = self.packs
        s = {"x": x}
        if self.coord is not None:     # stem: 1x1 conv + ReLU over the AddCoords input
            cw, cb = params[-2], params[-1]
            B, H, W, ca = x.shape
            x = torch.empty(B, H, W, cw.shape[0], dtype=torch.float32, device=cw.device)
            K.igemm(batch=B, in_hw=(H, W), out_hw=(H, W), k=1, stride=1, pad=0, src0=s["x"], c0=ca,
                    weight=pk.get(cw, PU_PACK_CONV_FWD, K.round16(ca)), k_pad=K.round16(ca), n=cw.shape[0],
                    bias=cb, dst0=x, relu=True)
            s["stem"] = x
        w, b = nxt(); t = conv3x3(x, w, b, pk)
        if self.dtype != t.dtype:
            t = K.to_bf16(t)
        s["inc.t"] = t
        w, b = nxt(); y = conv3x3(t, w, b, pk)
        skips = [y]
        for i in range(1, D):
            p = K.maxpool2_fwd(skips[-1]); s["down%d.p" % i] = p
            w, b = nxt(); t = conv3x3(p, w, b, pk); s["down%d.t" % i] = t
            w, b = nxt(); y = conv3x3(t, w, b, pk)
            skips.append(y)
        s["skips"] = skips
        y = skips[-1]
        for j in range(1, D):
            skip = skips[D - 1 - j]
            w, b = nxt(); u = convT2x2(y, w, b, pk); s["up%d.u" % j] = u
            if self.up_first:
                w, b = nxt(); t = conv3x3(u, w, b, pk, x1=skip)
            else:
                w, b = nxt(); t = conv3x3(skip, w, b, pk, x1=u)
            s["up%d.t" % j] = t
            w, b = nxt(); y = conv3x3(t, w, b, pk)
            s["up%d.y" % j] = y
        w, b = nxt()
        logits = K.outconv_fwd(y, w.reshape(-1), b)
        return logits, (s if save else None)

    # ------------------------------------------------------------------------------- backward
    def backward(self, s, dlogits, params):
        D = self.depth
        pk = self.packs
        P = list(params)
        grads = [None] * len(P)
        sink = self.grad_sinks()
        out = (lambda i: None) if sink is None else (lambda i: (sink[i], sink[i + 1]))  # noqa: E731
        # parameter slots (see __init__ order)
        n_enc = 4 * D
        up_base = lambda j: n_enc + 6 * (j - 1)  # noqa: E731
        outc = n_enc + 6 * (D - 1)
        skips = s["skips"]

        y_last = s["up%d.y" % (D - 1)]
        o = out(outc)
        g, dwo, dbo = K.outconv_bwd(y_last, P[outc].reshape(-1), dlogits, relu_mask=True,
                                    out=None if o is None else (o[0].view(-1), o[1]))
        grads[outc] = dwo.view_as(P[outc])
        grads[outc + 1] = dbo
        self._ready(outc)

        gskip = [None] * (D - 1)
        for j in range(D - 1, 0, -1):
            base = up_base(j)
            t = s["up%d.t" % j]
            u = s["up%d.u" % j]
            skip = skips[D - 1 - j]
            y_prev = skips[D - 1] if j == 1 else s["up%d.y" % (j - 1)]
            if self.debug is not None:
                self.debug["up%d.c1" % j] = g
            # conv1 of up_j: y_j = relu(conv(t));  g = dZ
            grads[base + 4], grads[base + 5] = conv3x3_wgrad(g, t, out=out(base + 4))
            self._ready(base + 4)
            dt, _ = conv3x3_dgrad(g, P[base + 4], pk, mask0=t)
            # conv0 over [skip | u]  (up_first: [u | skip])
            if self.up_first:
                grads[base + 2], grads[base + 3] = conv3x3_wgrad(dt, u, skip, out=out(base + 2))
                self._ready(base + 2)
                du, dskip = conv3x3_dgrad(dt, P[base + 2], pk, split=u.shape[3], mask1=skip)
            else:
                grads[base + 2], grads[base + 3] = conv3x3_wgrad(dt, skip, u, out=out(base + 2))
                self._ready(base + 2)
                dskip, du = conv3x3_dgrad(dt, P[base + 2], pk, split=skip.shape[3], mask0=skip)
            if self.debug is not None:
                self.debug["up%d.c0" % j] = dt
                self.debug["up%d.up" % j] = du
            gskip[D - 1 - j] = dskip
            # ConvT
            grads[base], grads[base + 1] = convT2x2_wgrad(y_prev, du, out=out(base))
            self._ready(base)
            g = convT2x2_dgrad(du, P[base], pk, mask=y_prev)

        for i in range(D - 1, 0, -1):
            base = 4 * i
            t = s["down%d.t" % i]
            p = s["down%d.p" % i]
            if self.debug is not None:
                self.debug["down%d.c1" % i] = g
            grads[base + 2], grads[base + 3] = conv3x3_wgrad(g, t, out=out(base + 2))
            self._ready(base + 2)
            dt, _ = conv3x3_dgrad(g, P[base + 2], pk, mask0=t)
            grads[base], grads[base + 1] = conv3x3_wgrad(dt, p, out=out(base))
            self._ready(base)
            if self.debug is not None:
                self.debug["down%d.c0" % i] = dt
            dp, _ = conv3x3_dgrad(dt, P[base], pk)
            g = K.maxpool2_bwd(skips[i - 1], dp, gskip[i - 1], relu_mask=True, accumulate=True)

        t = s["inc.t"]
        if self.debug is not None:
            self.debug["inc.c1"] = g
        grads[2], grads[3] = conv3x3_wgrad(g, t, out=out(2))
        self._ready(2)
        dt, _ = conv3x3_dgrad(g, P[2], pk, mask0=t)
        x0 = s["stem"] if self.coord is not None else s["x"]
        if dt.dtype != x0.dtype:       # bf16 trunk: the fp32 stem's weight gradient
            dt = K.to_f32(dt)
        grads[0], grads[1] = conv3x3_wgrad(dt, x0, out=out(0))
        self._ready(0)
        if self.debug is not None:
            self.debug["inc.c0"] = dt
        if self.coord is not None:     # stem 1x1 conv: dgrad of inc.c0 (masked by the stem ReLU) + wgrad
            dstem, _ = conv3x3_dgrad(dt, P[0], pk, mask0=x0)
            B, H, W, ca = s["x"].shape
            cs = len(P) - 2
            o = out(cs)
            dw = torch.empty(P[cs].shape, dtype=torch.float32, device=dt.device) if o is None else o[0]
            db = torch.empty(P[cs + 1].shape, dtype=torch.float32, device=dt.device) if o is None else o[1]
            K.wgrad(batch=B, in_hw=(H, W), out_hw=(H, W), k=1, stride=1, pad=0, rows=dstem, n=P[cs].shape[0],
                    src0=s["x"], c0=ca, bias_mode=1, dweight=dw, dbias=db)
            grads[cs], grads[cs + 1] = dw, db
            self._ready(cs)
        return grads


class TrunkFunction(torch.autograd.Function):
    """autograd node: (trunk, save, x NCHW, *trunk params) -> logits [B,H,W]."""

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
