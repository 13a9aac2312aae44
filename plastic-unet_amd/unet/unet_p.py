"""UNetp - drop-in for yaricom/Plastic-UNet ``src/unet/unet_p.py`` on MI355X.

Same class name, constructor signature, defaults, attributes (w, alpha, eta, nbf, rule, alfa_type,
torch_dev, n_channels, n_classes), module tree and state_dict keys as the reference (unet_p.py:9-94,
blocks :179-260), so reference checkpoints load unchanged and seeded initialisation is
bit-identical.  The nn.Conv2d / nn.ConvTranspose2d modules are parameter holders only: forward()
runs the trunk and the plastic head as HIP kernels (punet.trunk / punet.head).  There is no CPU
path - a CPU device raises.

Extensions (keyword-only in spirit, defaults reproduce the reference):
  depth=5, base_ch=8      generalised trunk width/depth (config C2 = depth 5, base 64)
  forward(x [B,C,N,N], hebb [B,N,N]) batches B independent per-slot traces; with hebb [N,N] the
  reference rule "batch size must be 1" applies unchanged.
  hebb_mode='sequential'  one [nbf,nbf] trace threaded through the B samples of a batch in order
                          (forward(x [B,...], hebb [nbf,nbf]) -> (Y [B,nbf,nbf], hebb')), instead of
                          B independent per-slot traces ('slots', the default)
  batch_norm=True         BatchNorm2d per slot (the reference's batch size 1), running statistics
                          updated slot by slot; bilinear_upsample=True: align_corners bilinear 2x
  precision='bf16'        config C3: bf16 activations / packed weights on bf16 MFMA with fp32
                          accumulation; parameters, gradients, Adam, logits and the plastic head
                          stay fp32 (base_ch must be a multiple of 32).
"""
import torch
import torch.nn as nn

__all__ = ["UNetp", "double_conv", "inconv", "down", "up", "outconv", "unetp_channels"]


def unetp_channels(depth=5, base_ch=8):
    """Encoder widths and (in, out) of each up stage; (5, 8) is unet_p.py:36-46 exactly."""
    if depth < 2:
        raise ValueError("depth must be >= 2")
    enc = [base_ch << i for i in range(depth - 1)]
    enc.append(enc[-1])
    ups = []
    for j in range(1, depth):
        skip = enc[depth - 1 - j]
        ups.append((2 * skip, enc[depth - 2 - j] if j < depth - 1 else base_ch))
    return enc, ups


class double_conv(nn.Module):
    """Conv3x3 [BN] ReLU Conv3x3 [BN] ReLU (unet_p.py:179-205) - parameter holder."""

    def __init__(self, in_ch, out_ch, batch_norm):
        super().__init__()
        layers = [nn.Conv2d(in_ch, out_ch, 3, padding=1)]
        if batch_norm:
            layers.append(nn.BatchNorm2d(out_ch))
        layers += [nn.ReLU(inplace=True), nn.Conv2d(out_ch, out_ch, 3, padding=1)]
        if batch_norm:
            layers.append(nn.BatchNorm2d(out_ch))
        layers.append(nn.ReLU(inplace=True))
        self.conv = nn.Sequential(*layers)

    def forward(self, x):
        raise RuntimeError("UNetp blocks are parameter holders; call the UNetp model")


class inconv(nn.Module):  # unet_p.py:208-215
    def __init__(self, in_ch, out_ch, batch_norm=True):
        super().__init__()
        self.conv = double_conv(in_ch, out_ch, batch_norm)


class down(nn.Module):  # unet_p.py:218-228
    def __init__(self, in_ch, out_ch, batch_norm=True):
        super().__init__()
        self.mpconv = nn.Sequential(nn.MaxPool2d(2), double_conv(in_ch, out_ch, batch_norm))


class up(nn.Module):  # unet_p.py:231-250
    def __init__(self, in_ch, out_ch, bilinear=True, batch_norm=True):
        super().__init__()
        if bilinear:
            self.up = nn.Upsample(scale_factor=2, mode="bilinear", align_corners=True)
        else:
            self.up = nn.ConvTranspose2d(in_ch // 2, in_ch // 2, 2, stride=2)
        self.conv = double_conv(in_ch, out_ch, batch_norm)


class outconv(nn.Module):  # unet_p.py:253-260
    def __init__(self, in_ch, out_ch):
        super().__init__()
        self.conv = nn.Conv2d(in_ch, out_ch, 1)


def _check_gpu_tensor(t, what):
    if not (torch.is_tensor(t) and t.is_cuda):
        raise RuntimeError(
            "%s must be a tensor on the ROCm device: this UNetp runs only as HIP kernels on MI355X "
            "(no CPU fallback); got %s" % (what, getattr(t, "device", type(t))))


class UNetp(nn.Module):
    def __init__(self, n_channels, n_classes, device, alfa_type='free', rule='hebb', nbf=128, batch_norm=False,
                 bilinear_upsample=False, depth=5, base_ch=8, precision='fp32', hebb_mode='slots'):
        super().__init__()
        if hebb_mode not in ("slots", "sequential"):
            raise ValueError("hebb_mode must be 'slots' or 'sequential'")
        self.hebb_mode = hebb_mode
        if precision not in ("fp32", "bf16"):
            raise ValueError("precision must be 'fp32' or 'bf16'")
        if precision == "bf16" and base_ch % 32:
            raise ValueError("precision='bf16' needs base_ch to be a multiple of 32 (got %d)" % base_ch)
        self.precision = precision
        self.compute_dtype = torch.bfloat16 if precision == "bf16" else torch.float32
        self.n_classes = n_classes
        self.n_channels = n_channels
        self.nbf = nbf
        self.torch_dev = device
        self.alfa_type = alfa_type
        self.rule = rule
        self.depth = depth
        self.base_ch = base_ch
        self.batch_norm = batch_norm
        self.bilinear_upsample = bilinear_upsample
        # unet_p.py:30-32; created on the CPU generator so seeded init matches the CPU reference
        self.w = nn.Parameter(.01 * torch.randn(nbf, nbf), requires_grad=True)
        self.alpha = nn.Parameter(.01 * torch.rand(nbf, nbf), requires_grad=True)
        self.eta = nn.Parameter(.01 * torch.ones(1), requires_grad=True)
        enc, ups = unetp_channels(depth, base_ch)
        self.inc = inconv(n_channels, enc[0], batch_norm=batch_norm)
        for i in range(1, depth):
            setattr(self, "down%d" % i, down(enc[i - 1], enc[i], batch_norm=batch_norm))
        for j, (cin, cout) in enumerate(ups, 1):
            setattr(self, "up%d" % j, up(cin, cout, batch_norm=batch_norm, bilinear=bilinear_upsample))
        self.outc = outconv(base_ch, n_classes)
        self.to(device)
        self._trunk = None
        print("UNet plastic model with plastic rule [%s] initialized" % self.rule)

    def _trunk_plan(self):
        if self._trunk is None:
            from punet.trunk import UNetpTrunk
            self._trunk = UNetpTrunk(self)
        return self._trunk

    def forward(self, x, hebb):
        single = hebb.dim() == 2
        seq = self.hebb_mode == "sequential"
        if single and x.shape[0] != 1 and not seq:
            raise ValueError("Only batch size: 1 is supported, but was: %d" % x.shape[0])
        if seq and not single:
            raise ValueError("hebb_mode='sequential' threads one [nbf,nbf] trace through the batch")
        if self.alfa_type not in ("free", "yoked"):
            raise ValueError("Must select one plasticity coefficient type ('free' or 'yoked')")
        if self.rule not in ("hebb", "oja"):
            raise ValueError("Must select one learning rule ('hebb' or 'oja')")
        _check_gpu_tensor(x, "x")
        _check_gpu_tensor(hebb, "hebb")
        if (self.batch_norm or self.bilinear_upsample) and self.precision != "fp32":
            raise NotImplementedError("UNetp(batch_norm=True / bilinear_upsample=True) runs with precision='fp32'")
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
        if H.shape != (B if not seq else 1, self.nbf, self.nbf):
            raise ValueError("hebb must be [nbf,nbf] or [B,nbf,nbf]; got %s for batch %d" % (tuple(hebb.shape), B))
        if x.dtype != torch.float32:
            x = x.float()

        from punet.trunk import TrunkFunction
        from punet.head import PlasticHeadFunction, RULES
        trunk = self._trunk_plan()
        trunk.training = self.training      # BatchNorm: per-slot batch statistics vs running statistics
        params = trunk.params
        save = torch.is_grad_enabled() and any(p.requires_grad for p in params)
        from punet.head import fused_head_ok, FusedHeadFunction
        wo, bo = self.outc.conv.weight, self.outc.conv.bias
        trunk.fused_head = fused_head_ok(wo.shape[1], self.nbf, seq)
        logits = TrunkFunction.apply(trunk, save, x, *params)
        if trunk.fused_head:
            sink = None if trunk.gradbuf is None else (trunk.gradbuf, self.w, self.alpha, wo, bo)
            Y, Hn = FusedHeadFunction.apply(logits, wo, bo, H, self.w, self.alpha, self.eta, RULES[self.rule], True,
                                            sink)
            return (Y[0], Hn[0]) if single else (Y, Hn)
        sink = None if trunk.gradbuf is None else (trunk.gradbuf, self.w, self.alpha)
        if seq:
            from punet.head import SequentialHeadFunction
            Y, Hn = SequentialHeadFunction.apply(logits, hebb, self.w, self.alpha, self.eta, RULES[self.rule], sink)
            return (Y[0], Hn) if B == 1 else (Y, Hn)
        Y, Hn = PlasticHeadFunction.apply(logits, H, self.w, self.alpha, self.eta, RULES[self.rule], True, sink)
        if single:
            return Y[0], Hn[0]
        return Y, Hn

    def initialZeroHebb(self, batch=None):
        """Zero trace [nbf,nbf] (unet_p.py:90-94), or [batch,nbf,nbf] per-slot traces."""
        shape = (self.nbf, self.nbf) if batch is None else (batch, self.nbf, self.nbf)
        return torch.zeros(*shape, dtype=torch.float, device=self.torch_dev)
