"""autograd nodes for the plastic head and BCELoss, each a pair of HIP kernel launches.

Reference: yaricom/Plastic-UNet src/unet/unet_p.py:69-88 (head) and src/train.py:70,101-105
(nn.BCELoss); backward = what loss.backward() (train.py:110) computes for them.
"""
import torch
import torch.nn as nn

from . import kernels as K
from ._lib import PU_RULE_HEBB, PU_RULE_OJA

RULES = {"hebb": PU_RULE_HEBB, "oja": PU_RULE_OJA}

# the 1x1 outconv runs inside the head kernel (pu_plastic_head_fwd) whenever the shapes allow;
# False restores the two-launch path (outconv in the trunk, then pu_plastic_fwd) - tests compare both
FUSE_OUTCONV = True


def fused_head_ok(feat_channels, nbf, seq=False):
    return FUSE_OUTCONV and not seq and feat_channels % 4 == 0 and nbf % 16 == 0 and 16 <= nbf <= 512


class FusedHeadFunction(torch.autograd.Function):
    """(feat [B,N,N,C], outc weight [1,C,1,1], outc bias [1], H [B,N,N], w, alpha, eta) -> (Y, H').

    The reference's outconv (unet_p.py:67, 253-260) and plastic head (:69-88) in one launch; X
    (the logits) is produced inside and kept for the backward, which runs the head backward and
    then the outconv backward (ReLU mask of feat fused), handing the trunk dL/d(pre-ReLU)."""

    @staticmethod
    def forward(ctx, feat, wo, bo, H, w, alpha, eta, rule, update_trace, sink=None):
        # sink: optional (GradBuffer, w, alpha, outc weight, outc bias) - grads into its views
        ctx.sink = sink
        feat = feat.contiguous()
        H = H.detach().contiguous()
        wod = wo.detach().reshape(-1)
        X, y, hn = K.plastic_head_fwd(feat, wod, bo.detach(), H, w.detach(), alpha.detach(), eta.detach(), rule,
                                      update_trace)
        ctx.save_for_backward(feat, wod, X, H, w.detach(), alpha.detach(), y)
        ctx.wo_shape = wo.shape
        ctx.set_materialize_grads(False)
        if hn is not None:
            ctx.mark_non_differentiable(hn)
        return y, hn

    @staticmethod
    def backward(ctx, dy, dhn):
        if dhn is not None:
            raise RuntimeError("backpropagation through the updated plastic trace is not supported: the "
                               "reference detaches it before reuse (src/train.py:99)")
        if dy is None:
            return (None,) * 10
        feat, wod, X, H, w, alpha, y = ctx.saved_tensors
        need_dw = ctx.needs_input_grad[4] or ctx.needs_input_grad[5]
        out_h = out_o = None
        if ctx.sink is not None:
            gb, wp, ap, wop, bop = ctx.sink
            if wp.grad is None and ap.grad is None:
                out_h = (gb.view_for(wp), gb.view_for(ap))
            if wop.grad is None and bop.grad is None:
                out_o = (gb.view_for(wop).view(-1), gb.view_for(bop))
        dx, dw, da = K.plastic_bwd(X, H, w, alpha, y, dy.contiguous(), need_dx=True, need_dw=need_dw, out=out_h)
        if out_h is not None:
            ctx.sink[0].ready(ctx.sink[1], ctx.sink[2])
        dfeat, dwo, dbo = K.outconv_bwd(feat, wod, dx, relu_mask=True, out=out_o)
        if out_o is not None:
            ctx.sink[0].ready(ctx.sink[3], ctx.sink[4])
        return (dfeat, dwo.view(ctx.wo_shape), dbo, None, dw if ctx.needs_input_grad[4] else None,
                da if ctx.needs_input_grad[5] else None, None, None, None, None)


class PlasticHeadFunction(torch.autograd.Function):
    """(X [B,N,N], H [B,N,N], w, alpha, eta) -> (Y, H').

    H' is returned without a gradient path (the reference's callers always detach it before the
    next sample, train.py:99, and no loss depends on it), so eta receives no gradient (S3).
    """

    @staticmethod
    def forward(ctx, X, H, w, alpha, eta, rule, update_trace, sink=None):
        # sink: optional (GradBuffer, w_param, alpha_param) - write dw/dalpha into its views
        ctx.sink = sink
        X = X.contiguous()
        H = H.detach().contiguous()
        y, hn = K.plastic_fwd(X, H, w.detach(), alpha.detach(), eta.detach(), rule, update_trace)
        ctx.save_for_backward(X, H, w.detach(), alpha.detach(), y)
        ctx.set_materialize_grads(False)
        if hn is not None:
            ctx.mark_non_differentiable(hn)
        return y, hn

    @staticmethod
    def backward(ctx, dy, dhn):
        if dhn is not None:
            raise RuntimeError("backpropagation through the updated plastic trace is not supported: the "
                               "reference detaches it before reuse (src/train.py:99)")
        if dy is None:
            return (None,) * 8
        X, H, w, alpha, y = ctx.saved_tensors
        need_dx = ctx.needs_input_grad[0]
        need_dw = ctx.needs_input_grad[2] or ctx.needs_input_grad[3]
        out = None
        if ctx.sink is not None:
            gb, wp, ap = ctx.sink
            if wp.grad is None and ap.grad is None:
                out = (gb.view_for(wp), gb.view_for(ap))
        dx, dw, da = K.plastic_bwd(X, H, w, alpha, y, dy.contiguous(), need_dx=need_dx, need_dw=need_dw, out=out)
        if out is not None:
            ctx.sink[0].ready(ctx.sink[1], ctx.sink[2])
        return (dx, None, dw if ctx.needs_input_grad[2] else None, da if ctx.needs_input_grad[3] else None,
                None, None, None, None)


class SequentialHeadFunction(torch.autograd.Function):
    """hebb_mode='sequential': (X [B,N,N], H [N,N], w, alpha, eta) -> (Y [B,N,N], H' [N,N]).

    One trace threaded through the samples in order - B successive reference calls
    (src/train.py:91-99) sharing the parameters: sample b runs the fused head kernel on the trace
    sample b-1 left.  The traces are detached between samples (train.py:99), so the backward is
    the batched head backward with the per-sample traces H_b as constants (one launch)."""

    @staticmethod
    def forward(ctx, X, H, w, alpha, eta, rule, sink=None):
        ctx.sink = sink
        X = X.contiguous()
        B, N, _ = X.shape
        Hs = torch.empty(B, N, N, dtype=torch.float32, device=X.device)
        Y = torch.empty_like(X)
        h = H.detach().reshape(1, N, N).contiguous()
        wd, ad, ed = w.detach(), alpha.detach(), eta.detach()
        for b in range(B):
            Hs[b].copy_(h[0])
            y, h = K.plastic_fwd(X[b:b + 1], h, wd, ad, ed, rule, True)
            Y[b].copy_(y[0])
        ctx.save_for_backward(X, Hs, wd, ad, Y)
        ctx.set_materialize_grads(False)
        hn = h.reshape(N, N)
        ctx.mark_non_differentiable(hn)
        return Y, hn

    @staticmethod
    def backward(ctx, dy, dhn):
        if dhn is not None:
            raise RuntimeError("backpropagation through the updated plastic trace is not supported: the "
                               "reference detaches it before reuse (src/train.py:99)")
        if dy is None:
            return (None,) * 7
        X, Hs, w, alpha, y = ctx.saved_tensors
        out = None
        if ctx.sink is not None:
            gb, wp, ap = ctx.sink
            if wp.grad is None and ap.grad is None:
                out = (gb.view_for(wp), gb.view_for(ap))
        need_dw = ctx.needs_input_grad[2] or ctx.needs_input_grad[3]
        dx, dw, da = K.plastic_bwd(X, Hs, w, alpha, y, dy.contiguous(), need_dx=ctx.needs_input_grad[0],
                                   need_dw=need_dw, out=out)
        if out is not None:
            ctx.sink[0].ready(ctx.sink[1], ctx.sink[2])
        return (dx, None, dw if ctx.needs_input_grad[2] else None, da if ctx.needs_input_grad[3] else None,
                None, None, None)


class BCELossFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, y, t):
        y = y.contiguous()
        t = t.detach().contiguous()
        ctx.save_for_backward(y, t)
        return K.bce_fwd(y, t)

    @staticmethod
    def backward(ctx, g):
        y, t = ctx.saved_tensors
        return K.bce_bwd(y, t, g), None


def bce_loss(y, t):
    """nn.BCELoss()(y.view(-1), t.view(-1)) on the HIP path (mean, log clamped at -100)."""
    return BCELossFunction.apply(y.reshape(-1), t.reshape(-1))


class BCELoss(nn.Module):
    """Drop-in for ``nn.BCELoss()`` (reduction='mean') on ROCm tensors."""

    def forward(self, input, target):
        return bce_loss(input, target)
