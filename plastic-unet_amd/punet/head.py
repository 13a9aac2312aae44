"""autograd nodes for the plastic head and BCELoss, each a pair of HIP kernel launches.

Reference: yaricom/Plastic-UNet src/unet/unet_p.py:69-88 (head) and src/train.py:70,101-105
(nn.BCELoss); backward = what loss.backward() (train.py:110) computes for them.
"""
import torch
import torch.nn as nn

from . import kernels as K
from ._lib import PU_RULE_HEBB, PU_RULE_OJA

RULES = {"hebb": PU_RULE_HEBB, "oja": PU_RULE_OJA}


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
