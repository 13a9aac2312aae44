"""CoordConvUNetp - the CoordConv U-Net of yaricom/Plastic-UNet src/coord_conv_script.py:146-200
(config C4) with the plastic head of src/unet/unet_p.py:69-88, on the MI355X path.

The reference script is Keras (not importable here); its topology is restated as:
  coord : AddCoords (:69-96; xx, yy and, with_r, rr channels) -> Conv 1x1 -> base_ch, ReLU (:153)
  inc   : 2 x (Conv3x3 + ReLU)                        widths base_ch * 2^i, i < depth (8..128)
  down_i: MaxPool2d(2) -> 2 x (Conv3x3 + ReLU)
  up_j  : ConvTranspose2d(2, s=2) halving the channels -> concat [upsampled | skip] (:171-172,
          upsampled FIRST) -> 2 x (Conv3x3 + ReLU)
  outc  : Conv 1x1 -> n_classes, then the plastic head (sigmoid inside the head).
The module tree / state_dict keys and the construction (RNG) order are those of the oracle's
RefCoordConvUNetp, so seeded inits are identical.  Inputs are floats in [0, 1] (the script's x/255
Lambda, :149, is the caller's image scaling).  forward() runs punet.trunk's kernels; no CPU path.
"""
import torch
import torch.nn as nn

from .unet_p import double_conv, inconv, down, outconv, _check_gpu_tensor

__all__ = ["CoordConvUNetp"]


class coord_conv(nn.Module):  # coord_conv_script.py:104-126 + the 1x1 / 8-filter / ReLU of :153
    def __init__(self, in_ch, out_ch, with_r):
        super().__init__()
        self.with_r = with_r
        self.conv = nn.Conv2d(in_ch + (3 if with_r else 2), out_ch, 1)


class kup(nn.Module):  # coord_conv_script.py:171-192
    def __init__(self, in_ch, out_ch):
        super().__init__()
        self.up = nn.ConvTranspose2d(in_ch, out_ch, 2, stride=2)
        self.conv = double_conv(2 * out_ch, out_ch, False)


class CoordConvUNetp(nn.Module):
    up_first = True      # concat order of the up stages: [upsampled | skip]

    def __init__(self, n_channels, n_classes, device, alfa_type='free', rule='hebb', nbf=256, base_ch=8,
                 with_r=True, depth=5):
        super().__init__()
        self.n_classes = n_classes
        self.n_channels = n_channels
        self.nbf = nbf
        self.torch_dev = device
        self.alfa_type = alfa_type
        self.rule = rule
        self.depth = depth
        self.base_ch = base_ch
        self.with_r = with_r
        self.w = nn.Parameter(.01 * torch.randn(nbf, nbf), requires_grad=True)
        self.alpha = nn.Parameter(.01 * torch.rand(nbf, nbf), requires_grad=True)
        self.eta = nn.Parameter(.01 * torch.ones(1), requires_grad=True)
        self.coord = coord_conv(n_channels, base_ch, with_r)
        enc = [base_ch * 2 ** i for i in range(depth)]
        self.inc = inconv(base_ch, enc[0], batch_norm=False)
        for i in range(1, depth):
            setattr(self, "down%d" % i, down(enc[i - 1], enc[i], batch_norm=False))
        for j in range(1, depth):
            setattr(self, "up%d" % j, kup(enc[depth - j], enc[depth - 1 - j]))
        self.outc = outconv(base_ch, n_classes)
        self.to(device)
        self._trunk = None
        print("CoordConv UNet plastic model with plastic rule [%s] initialized" % self.rule)

    def _trunk_plan(self):
        if self._trunk is None:
            from punet.trunk import UNetpTrunk
            self._trunk = UNetpTrunk(self)
        return self._trunk

    def forward(self, x, hebb):
        single = hebb.dim() == 2
        if single and x.shape[0] != 1:
            raise ValueError("Only batch size: 1 is supported, but was: %d" % x.shape[0])
        if self.alfa_type not in ("free", "yoked"):
            raise ValueError("Must select one plasticity coefficient type ('free' or 'yoked')")
        if self.rule not in ("hebb", "oja"):
            raise ValueError("Must select one learning rule ('hebb' or 'oja')")
        _check_gpu_tensor(x, "x")
        _check_gpu_tensor(hebb, "hebb")
        if self.n_classes != 1:
            raise RuntimeError("the plastic head needs n_classes == 1 (activin = x.view(nbf, nbf))")
        B, C, Hh, Ww = x.shape
        if C != self.n_channels:
            raise RuntimeError("expected input with %d channels, got %d" % (self.n_channels, C))
        if Hh * Ww != self.nbf * self.nbf or Hh != Ww:
            raise RuntimeError("shape '[%d, %d]' is invalid for input of size %d" % (self.nbf, self.nbf, Hh * Ww))
        if Hh % (1 << (self.depth - 1)):
            raise NotImplementedError("image side %d must be divisible by 2^(depth-1)=%d" % (Hh, 1 << (self.depth - 1)))
        H = hebb.unsqueeze(0) if single else hebb
        if H.shape != (B, self.nbf, self.nbf):
            raise ValueError("hebb must be [nbf,nbf] or [B,nbf,nbf]; got %s for batch %d" % (tuple(hebb.shape), B))
        if x.dtype != torch.float32:
            x = x.float()
        from punet.trunk import TrunkFunction
        from punet.head import PlasticHeadFunction, RULES
        trunk = self._trunk_plan()
        trunk.training = self.training
        params = trunk.params
        save = torch.is_grad_enabled() and any(p.requires_grad for p in params)
        from punet.head import fused_head_ok, FusedHeadFunction
        wo, bo = self.outc.conv.weight, self.outc.conv.bias
        trunk.fused_head = fused_head_ok(wo.shape[1], self.nbf, False)
        logits = TrunkFunction.apply(trunk, save, x, *params)
        if trunk.fused_head:
            sink = None if trunk.gradbuf is None else (trunk.gradbuf, self.w, self.alpha, wo, bo)
            Y, Hn = FusedHeadFunction.apply(logits, wo, bo, H, self.w, self.alpha, self.eta, RULES[self.rule], True,
                                            sink)
            return (Y[0], Hn[0]) if single else (Y, Hn)
        sink = None if trunk.gradbuf is None else (trunk.gradbuf, self.w, self.alpha)
        Y, Hn = PlasticHeadFunction.apply(logits, H, self.w, self.alpha, self.eta, RULES[self.rule], True, sink)
        if single:
            return Y[0], Hn[0]
        return Y, Hn

    def initialZeroHebb(self, batch=None):
        shape = (self.nbf, self.nbf) if batch is None else (batch, self.nbf, self.nbf)
        return torch.zeros(*shape, dtype=torch.float, device=self.torch_dev)
