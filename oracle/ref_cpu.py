"""TEST INFRASTRUCTURE ONLY - plain PyTorch-CPU fp32 restatement of the reference's training path.

Never imported by the product (``plastic-unet_amd/``).  Used by ``tests/`` as the parity checker,
by ``__graft_entry__.smoke()`` as the checker and by ``bench.py`` as the timed ``cpu_baseline``.
Pinned against golden vectors produced by the reference itself (``tests/golden/gen_golden.py``).

Every function cites the reference lines it restates (paths relative to yaricom/Plastic-UNet):

* ``RefUNetp``      - ``src/unet/unet_p.py:9-94`` (model), ``:179-260`` (blocks; the effective
                      re-definitions that shadow ``:96-177``).  Generalised to ``depth``/``base_ch``;
                      ``depth=5, base_ch=8`` is the reference topology, key-for-key.
* ``RefUNetpRes``   - ``src/unet/unet_p_res.py:9-272``.
* ``plastic_head``  - ``src/unet/unet_p.py:69-88`` (== ``unet_p_res.py:115-134``), batched over
                      per-slot traces (SURVEY.md section 8a "Batched semantics").
* ``bce_loss``      - ``src/train.py:70,101-105`` (``nn.BCELoss`` mean, log clamped at -100).
* ``add_coords``    - ``src/coord_conv_script.py:69-96``.
* ``RefCoordConvUNetp`` - ``src/coord_conv_script.py:146-200`` topology with the plastic head of
                      ``unet_p.py:69-88`` in place of the sigmoid output (config C4).
"""
from __future__ import annotations

import math
from collections import OrderedDict

import torch
import torch.nn as nn
import torch.nn.functional as F

__all__ = [
    "unetp_channels", "RefUNetp", "RefUNetpRes", "RefCoordConvUNetp", "plastic_head",
    "trace_update", "plastic_head_sequential", "bce_loss", "add_coords", "ref_train_step", "ref_adam", "ref_steplr",
    "fast_iou_metric", "rle_encode_mask", "det_init_", "ref_eval_net", "ref_train_loop",
]


# ----------------------------------------------------------------------------------------------
# plastic head  (unet_p.py:69-88)
# ----------------------------------------------------------------------------------------------
def trace_update(H, x0, y0, eta, rule):
    """Trace update from ROW 0 of the head input/output (unet_p.py:81-86).

    H: [B,N,N]; x0, y0: [B,N].  Hebb (``:82``): ``(1-eta)*H + eta*outer(x0, y0)``.
    Oja (``:84``): ``H + eta*((x0[:,None] - H*y0[None,:]) * y0[None,:])``; Oja does not decay H.
    """
    if rule == "hebb":
        return (1 - eta) * H + eta * (x0.unsqueeze(2) * y0.unsqueeze(1))
    if rule == "oja":
        y = y0.unsqueeze(1)
        return H + eta * torch.mul(x0.unsqueeze(2) - torch.mul(H, y), y)
    raise ValueError("Must select one learning rule ('hebb' or 'oja')")


def plastic_head(X, H, w, alpha, eta, rule="hebb", alfa_type="free"):
    """``Y_b = sigmoid(X_b (w + alpha*H_b))`` and the trace update, per slot b.

    X, H: [B,N,N] (B=1 is the reference exactly).  'free' and 'yoked' are numerically identical
    in the reference (both elementwise ``alpha*hebb``, unet_p.py:73 vs :75).
    """
    if alfa_type not in ("free", "yoked"):
        raise ValueError("Must select one plasticity coefficient type ('free' or 'yoked')")
    weff = w + torch.mul(alpha, H)
    Y = torch.sigmoid(torch.matmul(X, weff))
    Hn = trace_update(H, X[:, 0, :], Y[:, 0, :], eta, rule)
    return Y, Hn


def plastic_head_sequential(X, H, w, alpha, eta, rule="hebb", alfa_type="free"):
    """``--hebb-mode sequential``: ONE trace threaded through the B samples in order, each sample
    seeing the trace its predecessor left, as B successive reference calls (train.py:91-99) with
    the same parameters.  X [B,N,N], H [N,N] -> Y [B,N,N], H' [N,N].  The trace stays detached
    between samples (train.py:99), so sample b's head sees H_b as a constant."""
    Ys = []
    h = H
    for b in range(X.shape[0]):
        y, hn = plastic_head(X[b:b + 1], h.detach().unsqueeze(0), w, alpha, eta, rule, alfa_type)
        Ys.append(y)
        h = hn[0]
    return torch.cat(Ys), h


def bce_loss(y, t):
    """``nn.BCELoss()`` mean over every element (train.py:70,101-105)."""
    return F.binary_cross_entropy(y.reshape(-1), t.reshape(-1))


# ----------------------------------------------------------------------------------------------
# module trees with the reference's parameter names (state_dict key compatible)
# ----------------------------------------------------------------------------------------------
class _Seq(nn.Module):
    """Holder with a ``conv`` Sequential child (matches ``double_conv.conv`` / ``outconv.conv``)."""


def _double_conv(cin, cout, batch_norm):
    # unet_p.py:184-201 (effective definition) - Conv3x3 [BN] ReLU Conv3x3 [BN] ReLU
    layers = [nn.Conv2d(cin, cout, 3, padding=1)]
    if batch_norm:
        layers.append(nn.BatchNorm2d(cout))
    layers.append(nn.ReLU(inplace=True))
    layers.append(nn.Conv2d(cout, cout, 3, padding=1))
    if batch_norm:
        layers.append(nn.BatchNorm2d(cout))
    layers.append(nn.ReLU(inplace=True))
    m = _Seq()
    m.conv = nn.Sequential(*layers)
    return m


class _Inconv(nn.Module):  # unet_p.py:208-215
    def __init__(self, cin, cout, bn):
        super().__init__()
        self.conv = _double_conv(cin, cout, bn)

    def forward(self, x):
        return self.conv.conv(x)


class _Down(nn.Module):  # unet_p.py:218-228
    def __init__(self, cin, cout, bn):
        super().__init__()
        self.mpconv = nn.Sequential(nn.MaxPool2d(2), _double_conv(cin, cout, bn))

    def forward(self, x):
        return self.mpconv[1].conv(self.mpconv[0](x))


class _Up(nn.Module):  # unet_p.py:231-250
    def __init__(self, cin, cout, bn, bilinear):
        super().__init__()
        self.bilinear = bilinear
        if bilinear:
            self.up = nn.Upsample(scale_factor=2, mode="bilinear", align_corners=True)
        else:
            self.up = nn.ConvTranspose2d(cin // 2, cin // 2, 2, stride=2)
        self.conv = _double_conv(cin, cout, bn)

    def forward(self, x1, x2):
        x1 = self.up(x1)
        # the reference pads the SKIP by the size difference (unet_p.py:242-247); note it takes
        # the W-padding from the H difference and vice versa - zero at the square 2^k sizes.
        dh = x1.size(2) - x2.size(2)
        dw = x1.size(3) - x2.size(3)
        if dh or dw:
            x2 = F.pad(x2, (dh // 2, int(dh / 2), dw // 2, int(dw / 2)))
        return self.conv.conv(torch.cat([x2, x1], dim=1))  # skip FIRST (unet_p.py:248)


class _Outconv(nn.Module):  # unet_p.py:253-260 / unet_p_res.py:191-198
    def __init__(self, cin, cout):
        super().__init__()
        self.conv = nn.Conv2d(cin, cout, 1)

    def forward(self, x):
        return self.conv(x)


def unetp_channels(depth=5, base_ch=8):
    """Encoder widths and (in, out) of each ``up`` for the generalised UNetp trunk.

    ``depth=5, base_ch=8`` reproduces unet_p.py:36-46: enc 8,16,32,64,64 and
    up1(128,32) up2(64,16) up3(32,8) up4(16,8).
    """
    if depth < 2:
        raise ValueError("depth must be >= 2")
    enc = [base_ch * (2 ** i) for i in range(depth - 1)]
    enc.append(enc[-1])
    ups = []
    for j in range(1, depth):
        skip = enc[depth - 1 - j]
        out = enc[depth - 2 - j] if j < depth - 1 else base_ch
        ups.append((2 * skip, out))
    return enc, ups


def _head_params(module, nbf, device=None):
    # unet_p.py:30-32 - RNG order: randn (w), rand (alpha); eta is constant
    module.w = nn.Parameter(.01 * torch.randn(nbf, nbf, device=device), requires_grad=True)
    module.alpha = nn.Parameter(.01 * torch.rand(nbf, nbf, device=device), requires_grad=True)
    module.eta = nn.Parameter(.01 * torch.ones(1, device=device), requires_grad=True)


class _PlasticBase(nn.Module):
    hebb_mode = "slots"

    def _head(self, logits, hebb):
        nbf = self.nbf
        B = logits.shape[0]
        X = logits.reshape(B, nbf, nbf)  # view(nbf, nbf): S7 - N must equal H and W, n_classes 1
        if self.hebb_mode == "sequential":
            if hebb.dim() != 2:
                raise ValueError("hebb_mode='sequential' threads one [nbf,nbf] trace through the batch")
            return plastic_head_sequential(X, hebb, self.w, self.alpha, self.eta, self.rule, self.alfa_type)
        single = hebb.dim() == 2
        H = hebb.unsqueeze(0) if single else hebb
        if H.shape[0] != B:
            raise ValueError("hebb has %d slots but the batch has %d samples" % (H.shape[0], B))
        Y, Hn = plastic_head(X, H, self.w, self.alpha, self.eta, self.rule, self.alfa_type)
        if single:
            return Y[0], Hn[0]
        return Y, Hn

    def initialZeroHebb(self, batch=None):
        shape = (self.nbf, self.nbf) if batch is None else (batch, self.nbf, self.nbf)
        return torch.zeros(*shape, dtype=torch.float)


class RefUNetp(_PlasticBase):
    """UNetp (unet_p.py:8-94), generalised: ``depth``/``base_ch``; optional CoordConv stem."""

    def __init__(self, n_channels, n_classes, device=None, alfa_type="free", rule="hebb", nbf=128,
                 batch_norm=False, bilinear_upsample=False, depth=5, base_ch=8):
        super().__init__()
        self.n_classes, self.n_channels, self.nbf = n_classes, n_channels, nbf
        self.alfa_type, self.rule, self.depth = alfa_type, rule, depth
        _head_params(self, nbf)
        enc, ups = unetp_channels(depth, base_ch)
        self.inc = _Inconv(n_channels, enc[0], batch_norm)
        for i in range(1, depth):
            setattr(self, "down%d" % i, _Down(enc[i - 1], enc[i], batch_norm))
        for j, (cin, cout) in enumerate(ups, 1):
            setattr(self, "up%d" % j, _Up(cin, cout, batch_norm, bilinear_upsample))
        self.outc = _Outconv(base_ch, n_classes)

    def trunk(self, x):
        # Batched semantics with batch_norm=True: the reference trains at batch
        # size 1, so in training mode each slot runs on its own (its own BatchNorm statistics,
        # running statistics updated slot by slot in order).
        if self.training and x.shape[0] > 1 and any(isinstance(m, nn.BatchNorm2d) for m in self.modules()):
            return torch.cat([self._trunk(x[b:b + 1]) for b in range(x.shape[0])])
        return self._trunk(x)

    def _trunk(self, x):
        xs = [self.inc(x)]
        for i in range(1, self.depth):
            xs.append(getattr(self, "down%d" % i)(xs[-1]))
        y = xs[-1]
        for j in range(1, self.depth):
            y = getattr(self, "up%d" % j)(y, xs[self.depth - 1 - j])
        return self.outc(y)

    def forward(self, x, hebb):
        if hebb.dim() == 2 and x.shape[0] != 1 and self.hebb_mode != "sequential":
            raise ValueError("Only batch size: 1 is supported, but was: %d" % x.shape[0])
        return self._head(self.trunk(x), hebb)


# ---------------------------------- UNetpRes (unet_p_res.py) ----------------------------------
class _ConvModule(nn.Module):  # unet_p_res.py:142-164
    def __init__(self, ch, activation=True, batch_norm=False):
        super().__init__()
        conv = nn.Conv2d(ch, ch, kernel_size=3, stride=1, padding=1)
        self.conv = nn.Sequential(conv, nn.BatchNorm2d(ch)) if batch_norm else conv
        self.activation = activation
        if activation:
            self.activ = nn.ReLU(inplace=True)

    def forward(self, x):
        x = self.conv(x)
        return F.relu(x) if self.activation else x


class _ResidualBlock(nn.Module):  # unet_p_res.py:166-189
    def __init__(self, ch, batch_norm=False):
        super().__init__()
        layers = [nn.ReLU(inplace=True)]
        if batch_norm:
            layers.append(nn.BatchNorm2d(ch))
        layers += [_ConvModule(ch), _ConvModule(ch, activation=False)]
        self.conv = nn.Sequential(*layers)

    def forward(self, inp):
        # S11: the leading in-place ReLU rewrites ``inp`` before ``x.add(input)`` (:188), so the
        # skip adds relu(inp), not inp.
        r = F.relu(inp)
        x = r
        for m in list(self.conv)[1:]:
            x = m(x)
        return x + r


def _res_stack(cin, cout, bn):
    # ``down.dconv`` (:262-268) / ``middle.mconv`` (:229-234): Conv3x3, 2 residual blocks, ReLU
    return nn.Sequential(nn.Conv2d(cin, cout, kernel_size=3, padding=1),
                         _ResidualBlock(cout, bn), _ResidualBlock(cout, bn), nn.ReLU(inplace=True))


def _run_stack(seq, x):
    x = seq[0](x)
    x = seq[1](x)
    x = seq[2](x)
    return F.relu(x)


class _ResDown(nn.Module):
    def __init__(self, cin, cout, bn):
        super().__init__()
        self.dconv = _res_stack(cin, cout, bn)

    def forward(self, x):
        return _run_stack(self.dconv, x)


class _Middle(nn.Module):
    def __init__(self, cin, cout, bn):
        super().__init__()
        self.mconv = _res_stack(cin, cout, bn)

    def forward(self, x):
        return _run_stack(self.mconv, x)


class _PoolDrop(nn.Module):  # unet_p_res.py:240-253
    def __init__(self, p):
        super().__init__()
        self.dpool = nn.Sequential(nn.MaxPool2d(2), nn.Dropout2d(p=p, inplace=True))

    def forward(self, x):
        return self.dpool[1](self.dpool[0](x))


class _ResUp(nn.Module):  # unet_p_res.py:200-220
    def __init__(self, cin, cout, p):
        super().__init__()
        self.dconv = nn.ConvTranspose2d(cin, cout, kernel_size=3, stride=2, padding=0)
        # middle(..., batch_norm=False) regardless of the model flag (:211)
        self.uconv = nn.Sequential(nn.Dropout2d(p=p, inplace=True), _Middle(cin, cout, False))

    def forward(self, x1, x2):
        x = self.dconv(x1)                      # n -> 2n+1
        dh = x2.size(2) - x.size(2)
        dw = x2.size(3) - x.size(3)
        if dh or dw:                            # S13: diff -1 crops row/col 0
            x = F.pad(x, (dh // 2, int(dh / 2), dw // 2, int(dw / 2)))
        x = torch.cat([x, x2], dim=1)           # upsampled FIRST (:218)
        return self.uconv[1](self.uconv[0](x))


class RefUNetpRes(_PlasticBase):
    """UNetpRes (unet_p_res.py:9-140)."""

    def __init__(self, n_channels, n_classes, device=None, neurons=16, dropout_ratio=0.5,
                 alfa_type="free", rule="hebb", nbf=128, batch_norm=False, bilinear_upsample=False):
        super().__init__()
        self.n_classes, self.n_channels, self.nbf = n_classes, n_channels, nbf
        self.alfa_type, self.rule = alfa_type, rule
        _head_params(self, nbf)
        n = neurons
        self.conv1 = _ResDown(n_channels, n, batch_norm)
        self.pool1 = _PoolDrop(dropout_ratio / 2)
        self.conv2 = _ResDown(n, n * 2, batch_norm)
        self.pool2 = _PoolDrop(dropout_ratio)
        self.conv3 = _ResDown(n * 2, n * 4, batch_norm)
        self.pool3 = _PoolDrop(dropout_ratio)
        self.conv4 = _ResDown(n * 4, n * 8, batch_norm)
        self.pool4 = _PoolDrop(dropout_ratio)
        self.mid = _Middle(n * 8, n * 16, batch_norm)
        self.uconv4 = _ResUp(n * 16, n * 8, dropout_ratio)
        self.uconv3 = _ResUp(n * 8, n * 4, dropout_ratio)
        self.uconv2 = _ResUp(n * 4, n * 2, dropout_ratio)
        self.uconv1 = _ResUp(n * 2, n, dropout_ratio)
        self.outc = _Outconv(n, n_classes)

    def trunk(self, x):
        # batch_norm=True: per-slot BatchNorm statistics in training mode (see RefUNetp.trunk)
        if self.training and x.shape[0] > 1 and any(isinstance(m, nn.BatchNorm2d) for m in self.modules()):
            return torch.cat([self._trunk(x[b:b + 1]) for b in range(x.shape[0])])
        return self._trunk(x)

    def _trunk(self, x):
        xc1 = self.conv1(x)
        xc2 = self.conv2(self.pool1(xc1))
        xc3 = self.conv3(self.pool2(xc2))
        xc4 = self.conv4(self.pool3(xc3))
        x5 = self.mid(self.pool4(xc4))
        y = self.uconv4(x5, xc4)
        y = self.uconv3(y, xc3)
        y = self.uconv2(y, xc2)
        y = self.uconv1(y, xc1)
        return self.outc(y)

    def forward(self, x, hebb):
        return self._head(self.trunk(x), hebb)


# ------------------------------- CoordConv (coord_conv_script.py) ------------------------------
def add_coords(x, with_r=False):
    """AddCoords (coord_conv_script.py:69-96) on an NCHW tensor.

    Appends ``xx[i,j] = 2*j/(x_dim-1) - 1`` and ``yy[i,j] = 2*i/(y_dim-1) - 1`` (the script builds
    them from ``tf.range`` with x_dim = image height, y_dim = image width: square images only),
    plus ``rr = sqrt((xx-.5)^2 + (yy-.5)^2)`` when ``with_r``.
    """
    B, _, Hh, Ww = x.shape
    j = torch.arange(Ww, dtype=torch.float32)
    i = torch.arange(Hh, dtype=torch.float32)
    xx = (j / (Hh - 1)) * 2 - 1
    yy = (i / (Ww - 1)) * 2 - 1
    xx = xx.view(1, 1, 1, Ww).expand(B, 1, Hh, Ww)
    yy = yy.view(1, 1, Hh, 1).expand(B, 1, Hh, Ww)
    chans = [x, xx, yy]
    if with_r:
        chans.append(torch.sqrt(torch.square(xx - 0.5) + torch.square(yy - 0.5)))
    return torch.cat(chans, dim=1)


class _CoordConv(nn.Module):  # coord_conv_script.py:104-126 (+ the 1x1, 8-filter, ReLU at :153)
    def __init__(self, cin, cout, with_r):
        super().__init__()
        self.with_r = with_r
        self.conv = nn.Conv2d(cin + (3 if with_r else 2), cout, 1)

    def forward(self, x):
        return F.relu(self.conv(add_coords(x, self.with_r)))


class _KUp(nn.Module):
    """Keras up stage (coord_conv_script.py:171-192): ConvT 2x2 s2 halving channels, cat, 2 convs."""

    def __init__(self, cin, cout):
        super().__init__()
        self.up = nn.ConvTranspose2d(cin, cout, 2, stride=2)
        self.conv = _double_conv(2 * cout, cout, False)

    def forward(self, x, skip):
        return self.conv.conv(torch.cat([self.up(x), skip], dim=1))  # upsampled FIRST (:172)


class RefCoordConvUNetp(_PlasticBase):
    """Config C4: the CoordConv U-Net topology (coord_conv_script.py:146-200) with the plastic head
    of unet_p.py:69-88 on its 1-channel logits.  Widths base*[1,2,4,8,16] (the script: 8..128)."""

    def __init__(self, n_channels, n_classes, device=None, alfa_type="free", rule="hebb",
                 nbf=256, base_ch=8, with_r=True, depth=5):
        super().__init__()
        self.n_classes, self.n_channels, self.nbf = n_classes, n_channels, nbf
        self.alfa_type, self.rule, self.depth = alfa_type, rule, depth
        _head_params(self, nbf)
        self.coord = _CoordConv(n_channels, base_ch, with_r)
        enc = [base_ch * 2 ** i for i in range(depth)]
        self.inc = _Inconv(base_ch, enc[0], False)
        for i in range(1, depth):
            setattr(self, "down%d" % i, _Down(enc[i - 1], enc[i], False))
        for j in range(1, depth):
            setattr(self, "up%d" % j, _KUp(enc[depth - j], enc[depth - 1 - j]))
        self.outc = _Outconv(base_ch, n_classes)

    def trunk(self, x):
        xs = [self.inc(self.coord(x))]
        for i in range(1, self.depth):
            xs.append(getattr(self, "down%d" % i)(xs[-1]))
        y = xs[-1]
        for j in range(1, self.depth):
            y = getattr(self, "up%d" % j)(y, xs[self.depth - 1 - j])
        return self.outc(y)

    def forward(self, x, hebb):
        return self._head(self.trunk(x), hebb)


# ----------------------------------------------------------------------------------------------
# training step, optimizer, schedule (train.py:66-112)
# ----------------------------------------------------------------------------------------------
def ref_adam(params, lr):
    return torch.optim.Adam(params, lr=1.0 * lr)          # train.py:66


def ref_steplr(opt, step_size, gamma=0.666):
    return torch.optim.lr_scheduler.StepLR(opt, gamma=gamma, step_size=step_size)  # train.py:67


def ref_train_step(net, opt, sched, x, t, hebb):
    """One step of the reference's hot loop (train.py:91-112), batched over slots.

    Returns (loss, activout, new_hebb).  ``hebb`` is detached like ``Variable(hebb)`` (:99).
    """
    opt.zero_grad()
    y, hn = net(x, hebb.detach())
    loss = bce_loss(y, t)
    loss.backward()
    opt.step()
    if sched is not None:
        sched.step()
    return loss.detach(), y.detach(), hn.detach()


# ----------------------------------------------------------------------------------------------
# host-side metric / RLE used by eval and infer (utils/iou_metric.py:6-24, utils/rle_encode.py:6-17)
# ----------------------------------------------------------------------------------------------
def fast_iou_metric(y_true_in, y_pred_in):
    """utils/iou_metric.py:6-24; with flattened vectors (eval.py:100) each element is a 'batch'."""
    import numpy as np
    A = y_true_in
    B = y_pred_in > 0.5
    metric = []
    thresholds = np.arange(0.5, 1, 0.05)
    for b in range(A.shape[0]):
        t, p = A[b] > 0, B[b] > 0
        inter = np.logical_and(t, p)
        union = np.logical_or(t, p)
        iou = (np.sum(inter > 0) + 1e-10) / (np.sum(union > 0) + 1e-10)
        metric.append(np.mean([iou > th for th in thresholds]))
    return np.mean(metric)


def rle_encode_mask(im):
    """utils/rle_encode.py:6-17 - column-major run-length encoding."""
    import numpy as np
    pixels = np.concatenate([[0], im.flatten(order="F"), [0]])
    runs = np.where(pixels[1:] != pixels[:-1])[0] + 1
    runs[1::2] -= runs[::2]
    return " ".join(str(x) for x in runs)


# ----------------------------------------------------------------------------------------------
# deterministic init used by the golden fixtures for the wide trunks (tests/golden/gen_golden.py)
# ----------------------------------------------------------------------------------------------
def det_init_(net, seed):
    """w ~ .05*N(0,1) (seed+1), alpha ~ .05*U[0,1) (seed+2), eta = .02; every other parameter i
    (state_dict order) ~ U(-b, b), b = 1/sqrt(fan_in), generator seed 1000+i."""
    import numpy as np
    nbf = net.w.shape[0]
    with torch.no_grad():
        net.w.copy_(0.05 * torch.randn(nbf, nbf, generator=torch.Generator().manual_seed(seed + 1)))
        net.alpha.copy_(0.05 * torch.rand(nbf, nbf, generator=torch.Generator().manual_seed(seed + 2)))
        net.eta.fill_(0.02)
        idx = 0
        for k, p in net.state_dict(keep_vars=True).items():
            if k in ("w", "alpha", "eta"):
                continue
            fan = p.shape[1] * (p[0, 0].numel()) if p.dim() > 1 else p.shape[0]
            b = 1.0 / np.sqrt(max(fan, 1))
            p.copy_((torch.rand(p.shape, generator=torch.Generator().manual_seed(1000 + idx)) * 2 - 1) * b)
            idx += 1
    return net


# ----------------------------------------------------------------------------------------------
# the reference's epoch loop and validation (train.py:29-147, eval.py:66-103), bs=1 per step
# ----------------------------------------------------------------------------------------------
def ref_eval_net(net, X_val, y_val):
    """eval.py:66-103: zero trace (S5), trace output discarded, BCE + fast_iou_metric per sample."""
    net.eval()
    val_loss, total_acc = 0.0, 0.0
    with torch.no_grad():
        hebb = net.initialZeroHebb()
        for i, (x, t) in enumerate(zip(X_val, y_val)):
            y, _ = net(torch.from_numpy(x[None].astype("float32")), hebb)
            yf = y.reshape(-1)
            tf = torch.from_numpy(t.astype("float32")).reshape(-1)
            val_loss += bce_loss(yf, tf).item()
            total_acc += fast_iou_metric(y_true_in=tf.numpy(), y_pred_in=yf.numpy())
    return total_acc / (i + 1), val_loss / (i + 1)


def ref_train_loop(net, X_train, y_train, X_val, y_val, epochs, lr, steplr, gamma=0.666,
                   val_every=1):
    """train.py:29-147 without checkpoint I/O.  Returns the lists train() writes to HDF5."""
    import numpy as np
    all_losses, v_train, v_test, v_acc = [], [], [], []
    n = len(X_train)
    opt = ref_adam(net.parameters(), lr)
    sch = ref_steplr(opt, steplr, gamma)
    for epoch in range(epochs):
        net.train()
        hebb = net.initialZeroHebb()                                   # :88 - reset per epoch
        for img, mask in zip(X_train, y_train):
            x = torch.from_numpy(np.array([img.astype(np.float32)]))
            t = torch.from_numpy(mask.astype(np.float32))
            loss, _, hebb = ref_train_step(net, opt, sch, x, t, hebb)
            all_losses.append(loss.item())
        epoch_loss = np.mean(all_losses[-n])                           # S16: indexes ONE element
        if (epoch + 1) % val_every == 0 or epoch + 1 == epochs:
            acc, vloss = ref_eval_net(net, X_val, y_val)
            v_train.append(epoch_loss); v_test.append(vloss); v_acc.append(acc)
    return all_losses, v_train, v_test, v_acc
