"""The UNetpRes trunk (yaricom/Plastic-UNet src/unet/unet_p_res.py:71-113) as HIP kernel sequences.

Each ``down`` / ``middle`` stack (:223-238, :256-272) is Conv3x3 -> residual_block x2 -> ReLU where a
residual_block (:166-189) is  out = conv_B(relu(conv_A(relu(in)))) + relu(in)  - its leading
in-place ReLU rewrites ``in`` before the add (S11).  With r1 = relu(conv0(x)) the stack is

    a1 = relu(A1(r1))          r2 = relu(B1(a1) + r1)          a2 = relu(A2(r2))
    y  = relu(B2(a2) + r2)

five implicit-GEMM convolutions whose epilogues carry bias, the residual add (before the ReLU) and
the ReLU; nothing else is materialised.  Backward, given g = dL/dy * (y > 0):

    g_a2 = B2^T g . (a2>0)     g_o1 = (A2^T g_a2 + g) . (r2>0)     g_a1 = B1^T g_o1 . (a1>0)
    g_z0 = (A1^T g_a1 + g_o1) . (r1>0)      dX = conv0^T g_z0   (split over the two sources)

i.e. the same dgrad kernel with the residual gradient added in its epilogue before the mask.

``up`` (:200-220): ConvTranspose2d(3, s=2, p=0) takes h -> 2h+1 and the negative F.pad crops row and
column 0 when the skip is 2h wide (S13); it runs as one GEMM over the (h+1)^2 grid of 2x2 output
blocks (PU_PACK_CONVT3_FWD) whose shuffle epilogue drops the cropped pixels.  Its dgrad is a
stride-2 3x3 conv (pad = crop) and its wgrad a stride-2 weight-gradient GEMM; the bias gradient
is a column sum.  The concat is [upsampled | skip] (upsampled FIRST, :218) and is read from the
two buffers directly.  Dropout2d (:209, :248) multiplies channels by a per-sample mask
(punet.kernels.channel_scale); masks come from torch's generator (``mask_fn`` may inject them).
"""
import torch

from . import kernels as K
from ._lib import PU_PACK_CONV_FWD, PU_PACK_CONV_DGRAD, PU_PACK_CONVT_DGRAD, PU_PACK_CONVT3_FWD
from .trunk import _Packs, _grad_sinks


# ------------------------------------------------------------------------------ layer helpers
def conv3x3(x0, w, b, packs, x1=None, relu=True, resid=None):
    """3x3/p1 conv over [x0 | x1] (NHWC) + bias (+ resid) (then ReLU)."""
    B, H, W, c0 = x0.shape
    c1 = 0 if x1 is None else x1.shape[3]
    cout = w.shape[0]
    k_pad = K.round16(9 * (c0 + c1))
    g = K.cgroup_for(c0, c1)
    out = torch.empty(B, H, W, cout, dtype=torch.float32, device=x0.device)
    K.igemm(batch=B, in_hw=(H, W), out_hw=(H, W), k=3, stride=1, pad=1, src0=x0, c0=c0, src1=x1, c1=c1,
            weight=packs.get(w, PU_PACK_CONV_FWD, k_pad, g), k_pad=k_pad, n=cout, bias=b, dst0=out, relu=relu,
            cgroup=g, resid=resid)
    return out


def conv3x3_dgrad(dz, w, packs, split=None, mask0=None, mask1=None, resid=None, chan_scale=None):
    """dX = conv(dZ, flipped W^T) (+ resid) (. mask) (* chan_scale[b, c]: the Dropout2d backward);
    optional channel split -> (d0, d1)."""
    B, H, W, cout = dz.shape
    cin = w.shape[1]
    k_pad = K.round16(9 * cout)
    g = K.cgroup_for(cout)
    n0 = cin if split is None else split
    d0 = torch.empty(B, H, W, n0, dtype=torch.float32, device=dz.device)
    d1 = None if split is None else torch.empty(B, H, W, cin - n0, dtype=torch.float32, device=dz.device)
    K.igemm(batch=B, in_hw=(H, W), out_hw=(H, W), k=3, stride=1, pad=1, src0=dz, c0=cout,
            weight=packs.get(w, PU_PACK_CONV_DGRAD, k_pad, g), k_pad=k_pad, n=cin, dst0=d0, n0=n0, dst1=d1,
            mask0=mask0, mask1=mask1, cgroup=g, resid=resid, chan_scale=chan_scale)
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


def _crop(h, out_h):
    crop = 2 * h + 1 - out_h
    if crop not in (0, 1):
        raise RuntimeError("ConvTranspose2d(3, s=2) output %d cannot be padded to the skip size %d "
                           "(unet_p_res.py:215-217 only ever crops one row)" % (2 * h + 1, out_h))
    return crop


def _fusable(m):
    """A Dropout2d mask the conv epilogue can apply (float4 rows: width % 4 == 0, 16-byte aligned
    contiguous rows), else None (a separate pu_channel_scale pass)."""
    if m is None or m.shape[1] % 4 or not m.is_contiguous() or m.data_ptr() % 16:
        return None
    return m


def convT3x3(x, w, b, packs, out_hw, chan_scale=None):
    """ConvTranspose2d(cin, cout, 3, stride=2, padding=0) + crop to out_hw (NHWC); chan_scale
    [B, >= cout] (row stride = its width): per-(image, channel) factors (the Dropout2d of up())."""
    B, h, wd, cin = x.shape
    cout = w.shape[1]
    H2, W2 = out_hw
    crop = _crop(h, H2)
    if _crop(wd, W2) != crop:
        raise RuntimeError("non-square crop")
    k_pad = K.round16(4 * cin)
    out = torch.empty(B, H2, W2, cout, dtype=torch.float32, device=x.device)
    K.igemm(batch=B, in_hw=(h, wd), out_hw=(h + 1, wd + 1), k=2, stride=1, pad=1, src0=x, c0=cin,
            weight=packs.get(w, PU_PACK_CONVT3_FWD, k_pad), k_pad=k_pad, n=4 * cout, bias=b, dst0=out,
            shuffle=True, shuf=(H2, W2, crop), chan_scale=chan_scale)
    return out


def convT3x3_dgrad(du, w, packs, in_hw, mask):
    """dX[i] = sum_r W[:, :, r] dU_full[2i + r] (dU_full[o] = du[o - crop]), times (mask > 0)."""
    B, H2, W2, cout = du.shape
    cin = w.shape[0]
    h, wd = in_hw
    crop = _crop(h, H2)
    k_pad = K.round16(9 * cout)
    g = K.cgroup_for(cout)
    dx = torch.empty(B, h, wd, cin, dtype=torch.float32, device=du.device)
    K.igemm(batch=B, in_hw=(H2, W2), out_hw=(h, wd), k=3, stride=2, pad=crop, src0=du, c0=cout,
            weight=packs.get(w, PU_PACK_CONVT_DGRAD, k_pad, g), k_pad=k_pad, n=cin, dst0=dx, mask0=mask, cgroup=g)
    return dx


def convT3x3_wgrad(x, du, out=None):
    """dW[i][o][r][s] = sum_p x[p][i] dU_full[2p + (r, s)][o] ; db[o] = sum over du pixels."""
    B, h, wd, cin = x.shape
    _, H2, W2, cout = du.shape
    crop = _crop(h, H2)
    if out is None:
        dw = torch.empty(cin, cout, 3, 3, dtype=torch.float32, device=x.device)
        db = torch.empty(cout, dtype=torch.float32, device=x.device)
    else:
        dw, db = out
    K.wgrad(batch=B, in_hw=(H2, W2), out_hw=(h, wd), k=3, stride=2, pad=crop, rows=x, n=cin, src0=du, c0=cout,
            bias_mode=0, dweight=dw)
    K.column_sum(du.view(-1, cout), out=db)
    return dw, db


# --------------------------------------------------------------------------------- the trunk
class ResTrunk:
    """Parameter order and kernel schedule of UNetpRes.  Per stack (conv1..conv4, mid, and the
    middle of uconv4..uconv1): conv0 w,b, block1 A w,b, block1 B w,b, block2 A w,b, block2 B w,b;
    each up stage puts its ConvTranspose2d w,b before its stack; outc w,b last."""

    DOWN = ("conv1", "conv2", "conv3", "conv4")
    UP = ("uconv4", "uconv3", "uconv2", "uconv1")

    def __init__(self, model):
        self.packs = _Packs()
        self.model = model
        self.params = []
        self.slots = {}
        for name in self.DOWN + ("mid",):
            mod = getattr(model, name)
            seq = mod.dconv if name != "mid" else mod.mconv
            self.slots[name] = len(self.params)
            self.params += self._stack_params(seq)
        for name in self.UP:
            mod = getattr(model, name)
            self.slots[name + ".up"] = len(self.params)
            self.params += [mod.dconv.weight, mod.dconv.bias]
            self.slots[name] = len(self.params)
            self.params += self._stack_params(mod.uconv[1].mconv)
        self.slots["outc"] = len(self.params)
        self.params += [model.outc.conv.weight, model.outc.conv.bias]
        # batch_norm=True (unet_p_res.py:171-176): each residual block of the DOWN stacks and mid
        # carries one BatchNorm2d on its ReLU'd input, before conv A (its conv_modules are built
        # without batch_norm, :174-175); the up stages' middle has none (:211).  Affine params
        # appended after outc.
        self.bn = {}             # (stack, block) -> (param index, module)
        for name in self.DOWN + ("mid",):
            mod = getattr(model, name)
            seq = mod.dconv if name != "mid" else mod.mconv
            for blk in (1, 2):
                layers = list(seq[blk].conv)
                if len(layers) == 3:
                    continue
                m = layers[1]
                if not isinstance(m, torch.nn.BatchNorm2d) or m.momentum is None:
                    raise NotImplementedError("UNetpRes BatchNorm layout not recognised")
                self.bn[(name, blk)] = (len(self.params), m)
                self.params += [m.weight, m.bias]
        self.training = True
        self.gradbuf = None
        self.mask_fn = None      # (name, batch, channels, p) -> [B, C] scale; default: bernoulli
        self.mask_gen = None     # torch.Generator for the bernoulli masks (None: torch's default);
                                 # data-parallel Trainers set a per-rank one (punet.dp.rank_generator)
        self.fused_head = False  # as UNetpTrunk.fused_head
        self.debug = None

    @staticmethod
    def _stack_params(seq):
        out = [seq[0].weight, seq[0].bias]
        for blk in (seq[1], seq[2]):
            layers = list(blk.conv)
            convs = layers[1:] if len(layers) == 3 else layers[2:]      # [ReLU, (BN,) A, B]
            for cm in convs:
                conv = cm.conv if isinstance(cm.conv, torch.nn.Conv2d) else cm.conv[0]
                out += [conv.weight, conv.bias]
        return out

    def backward_order(self):
        """Parameters in the order backward() completes their gradients (outc first, conv1 last;
        the BatchNorm affine parameters last - they are small)."""
        n_core = self.slots["outc"] + 2
        return list(reversed(self.params[:n_core])) + list(reversed(self.params[n_core:]))

    def _ready(self, i, n=2):
        """params[i:i+n]'s gradient kernels are enqueued: let an armed BucketReducer know."""
        gb = self.gradbuf
        if gb is not None and gb.reducer is not None:
            gb.ready(*self.params[i:i + n])

    def grad_sinks(self):
        return _grad_sinks(self, self.slots["outc"])

    def _mask(self, name, B, C, p, device):
        if self.mask_fn is not None:
            return self.mask_fn(name, B, C, p)
        return torch.empty(B, C, dtype=torch.float32, device=device).bernoulli_(
            1.0 - p, generator=self.mask_gen).div_(1.0 - p)

    # ---------------------------------------------------------------------------- forward
    def _bn(self, P, key, z, relu, resid=None, save=None):
        j, m = self.bn[key]
        training = self.training or not m.track_running_stats
        update = self.training and m.track_running_stats
        y, mean, rstd = K.bn_fwd(z, P[j], P[j + 1], m.running_mean if (update or not training) else None,
                                 m.running_var if (update or not training) else None, m.eps, m.momentum, training,
                                 relu=relu, resid=resid)
        if update:
            m.num_batches_tracked.add_(z.shape[0])     # one reference forward per slot
        return y, (mean, rstd)

    def _stack_fwd_bn(self, P, i, name, x0, x1=None):
        """conv0 + ReLU, then per residual block: n = BN(r); a = relu(A(n)); r' = relu(B(a) + r)
        (unet_p_res.py:166-189 with batch_norm=True; the add and ReLU fused in B's epilogue)."""
        pk = self.packs
        r = conv3x3(x0, P[i], P[i + 1], pk, x1=x1)
        st = {"x0": x0, "x1": x1}
        for blk in (1, 2):
            ia = i + 2 + 4 * (blk - 1)
            n, sa = self._bn(P, (name, blk), r, relu=False)
            a = conv3x3(n, P[ia], P[ia + 1], pk)
            r_next = conv3x3(a, P[ia + 2], P[ia + 3], pk, resid=r)
            st[blk] = (r, n, a, sa)
            r = r_next
        st["y"] = r
        return r, st

    def _stack_fwd(self, P, i, x0, x1=None):
        pk = self.packs
        r1 = conv3x3(x0, P[i], P[i + 1], pk, x1=x1)
        a1 = conv3x3(r1, P[i + 2], P[i + 3], pk)
        r2 = conv3x3(a1, P[i + 4], P[i + 5], pk, resid=r1)
        a2 = conv3x3(r2, P[i + 6], P[i + 7], pk)
        y = conv3x3(a2, P[i + 8], P[i + 9], pk, resid=r2)
        return y, (x0, x1, r1, a1, r2, a2, y)

    def forward(self, x, params, save, training):
        self.training = training       # BatchNorm: per-slot batch statistics vs running statistics
        self.packs.refresh()           # operands of parameters the optimizer moved: one launch
        P = list(params)
        p_drop = self.model.dropout_ratio
        drop = training and p_drop > 0
        s = {}
        h = x
        skips = []
        for k, name in enumerate(self.DOWN):
            if (name, 1) in self.bn:
                y, st = self._stack_fwd_bn(P, self.slots[name], name, h)
            else:
                y, st = self._stack_fwd(P, self.slots[name], h)
            s[name] = st
            skips.append(y)
            p = p_drop / 2 if k == 0 else p_drop          # pool1 uses dropout_ratio/2 (:39)
            m = self._mask("pool%d" % (k + 1), y.shape[0], y.shape[3], p, y.device) if drop else None
            h = K.maxpool2_fwd(y, scale=m)                # pool_drop (:62): the Dropout2d fused
            if drop:
                s["pool%d.mask" % (k + 1)] = m
        if ("mid", 1) in self.bn:
            y, st = self._stack_fwd_bn(P, self.slots["mid"], "mid", h)
        else:
            y, st = self._stack_fwd(P, self.slots["mid"], h)
        s["mid"] = st
        for j, name in enumerate(self.UP):
            skip = skips[3 - j]
            i = self.slots[name + ".up"]
            # Dropout2d over cat(u, skip) (unet_p_res.py:69): u's channels scaled by the ConvT
            # epilogue (the mask's row stride spans both parts), the skip's by a scaled copy (the
            # unscaled skip stays for MaxPool2d's backward)
            m = self._mask(name, y.shape[0], P[i].shape[1] + skip.shape[3], p_drop, y.device) if drop else None
            u = convT3x3(y, P[i], P[i + 1], self.packs, skip.shape[1:3], chan_scale=_fusable(m))
            s[name + ".in"] = y
            src1 = skip
            if drop:
                cu = u.shape[3]
                if _fusable(m) is None:
                    K.channel_scale(u, m[:, :cu].contiguous(), out=u)
                src1 = K.channel_scale(skip, m[:, cu:].contiguous())
                s[name + ".mask"] = m
            y, st = self._stack_fwd(P, self.slots[name], u, src1)
            s[name] = st
        s["skips"] = skips
        if self.fused_head:
            return y, (s if save else None)
        o = self.slots["outc"]
        logits = K.outconv_fwd(y, P[o].reshape(-1), P[o + 1])
        return logits, (s if save else None)

    # --------------------------------------------------------------------------- backward
    def _stack_bwd(self, P, i, st, g, grads, out, need_dx=True, split=None, mask1=None, chan_scale=None):
        pk = self.packs
        x0, x1, r1, a1, r2, a2, y = st
        dbg = self.debug
        grads[i + 8], grads[i + 9] = conv3x3_wgrad(g, a2, out=out(i + 8))
        self._ready(i + 8)
        g_a2, _ = conv3x3_dgrad(g, P[i + 8], pk, mask0=a2)
        grads[i + 6], grads[i + 7] = conv3x3_wgrad(g_a2, r2, out=out(i + 6))
        self._ready(i + 6)
        g_o1, _ = conv3x3_dgrad(g_a2, P[i + 6], pk, mask0=r2, resid=g)
        grads[i + 4], grads[i + 5] = conv3x3_wgrad(g_o1, a1, out=out(i + 4))
        self._ready(i + 4)
        g_a1, _ = conv3x3_dgrad(g_o1, P[i + 4], pk, mask0=a1)
        grads[i + 2], grads[i + 3] = conv3x3_wgrad(g_a1, r1, out=out(i + 2))
        self._ready(i + 2)
        g_z0, _ = conv3x3_dgrad(g_a1, P[i + 2], pk, mask0=r1, resid=g_o1)
        grads[i], grads[i + 1] = conv3x3_wgrad(g_z0, x0, x1, out=out(i))
        self._ready(i)
        if dbg is not None:
            dbg[i] = (g, g_a2, g_o1, g_a1, g_z0)
        if not need_dx:
            return None, None
        return conv3x3_dgrad(g_z0, P[i], pk, split=split, mask1=mask1, chan_scale=chan_scale)

    def _bn_bwd(self, P, key, z, g, stat, out, grads, add=None, mask=None):
        j, _ = self.bn[key]
        o = out(j)
        dgam = torch.empty_like(P[j]) if o is None else o[0]
        dbet = torch.empty_like(P[j + 1]) if o is None else o[1]
        dz = K.bn_bwd(z, g, stat[0], stat[1], P[j], dgam, dbet, add=add, mask=mask)
        grads[j], grads[j + 1] = dgam, dbet
        self._ready(j)
        return dz

    def _stack_bwd_bn(self, P, i, name, st, g, grads, out, need_dx=True, split=None, mask1=None):
        """g = dL/d(stack output) * (y > 0)."""
        pk = self.packs
        for blk in (2, 1):
            r, n, a, sa = st[blk]
            ia = i + 2 + 4 * (blk - 1)
            grads[ia + 2], grads[ia + 3] = conv3x3_wgrad(g, a, out=out(ia + 2))
            self._ready(ia + 2)
            ga, _ = conv3x3_dgrad(g, P[ia + 2], pk, mask0=a)
            grads[ia], grads[ia + 1] = conv3x3_wgrad(ga, n, out=out(ia))
            self._ready(ia)
            dn, _ = conv3x3_dgrad(ga, P[ia], pk)
            # r feeds the BatchNorm and the residual add: dL/dr = BN^T dn + g, times relu's mask
            g = self._bn_bwd(P, (name, blk), r, dn, sa, out, grads, add=g, mask=r)
        grads[i], grads[i + 1] = conv3x3_wgrad(g, st["x0"], st["x1"], out=out(i))
        self._ready(i)
        if not need_dx:
            return None, None
        return conv3x3_dgrad(g, P[i], pk, split=split, mask1=mask1)

    def backward(self, s, dlogits, params):
        P = list(params)
        grads = [None] * len(P)
        sink = self.grad_sinks()
        out = (lambda i: None) if sink is None else (lambda i: (sink[i], sink[i + 1]))  # noqa: E731
        skips = s["skips"]
        o = self.slots["outc"]
        y_last = s["uconv1"][6]
        if self.fused_head:
            g = dlogits                  # the fused head's outconv backward already applied the mask
        else:
            oo = out(o)
            g, dwo, dbo = K.outconv_bwd(y_last, P[o].reshape(-1), dlogits, relu_mask=True,
                                        out=None if oo is None else (oo[0].view(-1), oo[1]))
            grads[o] = dwo.view_as(P[o])
            grads[o + 1] = dbo
            self._ready(o)
        gskip = [None] * 4
        for j in range(3, -1, -1):                       # uconv1 .. uconv4
            name = self.UP[j]
            st = s[name]
            cu = st[0].shape[3]
            skip = skips[3 - j]
            # the Dropout2d backward of cat(u, skip) in the split data gradient's epilogue
            m = s.get(name + ".mask")
            g_u, g_sk = self._stack_bwd(P, self.slots[name], st, g, grads, out, split=cu, mask1=skip,
                                        chan_scale=_fusable(m))
            if m is not None and _fusable(m) is None:
                K.channel_scale(g_u, m[:, :cu].contiguous(), out=g_u)
                K.channel_scale(g_sk, m[:, cu:].contiguous(), out=g_sk)
            gskip[3 - j] = g_sk
            i = self.slots[name + ".up"]
            x_in = s[name + ".in"]
            grads[i], grads[i + 1] = convT3x3_wgrad(x_in, g_u, out=out(i))
            self._ready(i)
            g = convT3x3_dgrad(g_u, P[i], self.packs, x_in.shape[1:3], mask=x_in)
        if ("mid", 1) in self.bn:
            g_p, _ = self._stack_bwd_bn(P, self.slots["mid"], "mid", s["mid"], g, grads, out)
        else:
            g_p, _ = self._stack_bwd(P, self.slots["mid"], s["mid"], g, grads, out)
        for k in range(3, -1, -1):                       # conv4 .. conv1
            g = K.maxpool2_bwd(skips[k], g_p, gskip[k], relu_mask=True, accumulate=True,
                               scale=s.get("pool%d.mask" % (k + 1)))
            name = self.DOWN[k]
            if (name, 1) in self.bn:
                g_p, _ = self._stack_bwd_bn(P, self.slots[name], name, s[name], g, grads, out, need_dx=k > 0)
            else:
                g_p, _ = self._stack_bwd(P, self.slots[name], s[name], g, grads, out, need_dx=k > 0)
        return grads


class ResTrunkFunction(torch.autograd.Function):
    """autograd node: (trunk, save, training, x NCHW, *params) -> logits [B,H,W]."""

    @staticmethod
    def forward(ctx, trunk, save, training, x, *params):
        from .trunk import as_nhwc_input
        xin = as_nhwc_input(x.detach())
        detached = [p.detach() for p in params]
        logits, saved = trunk.forward(xin, detached, save, training)
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
        return (None, None, None, None) + tuple(grads)
