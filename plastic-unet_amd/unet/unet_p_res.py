"""UNetpRes - drop-in for yaricom/Plastic-UNet ``src/unet/unet_p_res.py`` (module tree / state_dict
compatible; constructor signature and defaults unchanged).

forward() runs the residual trunk as HIP kernels (punet.res_trunk: residual-add conv epilogues,
ConvTranspose2d 3x3 s2 with the row/col-0 crop, Dropout2d channel masks in training mode) and the
plastic head of unet_p_res.py:115-134 (punet.head).  Like UNetp it batches B per-slot traces when
hebb is [B,nbf,nbf]; there is no CPU path.
"""
import torch
import torch.nn as nn

__all__ = ["UNetpRes"]


class conv_module(nn.Module):  # unet_p_res.py:142-164
    def __init__(self, out_ch, kernel_size, stride=1, padding=1, activation=True, batch_norm=False):
        super().__init__()
        conv = nn.Conv2d(out_ch, out_ch, kernel_size=kernel_size, stride=stride, padding=padding)
        self.conv = nn.Sequential(conv, nn.BatchNorm2d(out_ch)) if batch_norm else conv
        self.activation = activation
        if activation:
            self.activ = nn.ReLU(inplace=True)


class residual_block(nn.Module):  # unet_p_res.py:166-189
    def __init__(self, out_ch, batch_norm=False):
        super().__init__()
        layers = [nn.ReLU(inplace=True)]
        if batch_norm:
            layers.append(nn.BatchNorm2d(out_ch))
        layers += [conv_module(out_ch, kernel_size=3), conv_module(out_ch, kernel_size=3, activation=False)]
        self.conv = nn.Sequential(*layers)


class outconv(nn.Module):  # unet_p_res.py:191-198
    def __init__(self, in_ch, out_ch):
        super().__init__()
        self.conv = nn.Conv2d(in_ch, out_ch, kernel_size=1)


def _stack(in_ch, out_ch, batch_norm):
    return nn.Sequential(nn.Conv2d(in_ch, out_ch, kernel_size=3, padding=1),
                         residual_block(out_ch=out_ch, batch_norm=batch_norm),
                         residual_block(out_ch=out_ch, batch_norm=batch_norm), nn.ReLU(inplace=True))


class middle(nn.Module):  # unet_p_res.py:223-238
    def __init__(self, in_ch, out_ch, batch_norm=False):
        super().__init__()
        self.mconv = _stack(in_ch, out_ch, batch_norm)


class down(nn.Module):  # unet_p_res.py:256-272
    def __init__(self, in_ch, out_ch, batch_norm=False):
        super().__init__()
        self.dconv = _stack(in_ch, out_ch, batch_norm)


class pool_drop(nn.Module):  # unet_p_res.py:240-253
    def __init__(self, dropout_ratio):
        super().__init__()
        self.dpool = nn.Sequential(nn.MaxPool2d(2), nn.Dropout2d(p=dropout_ratio, inplace=True))


class up(nn.Module):  # unet_p_res.py:200-220
    def __init__(self, in_ch, out_ch, dropout_ratio, batch_norm=False):
        super().__init__()
        self.dconv = nn.ConvTranspose2d(in_ch, out_ch, kernel_size=3, stride=2, padding=0)
        self.uconv = nn.Sequential(nn.Dropout2d(p=dropout_ratio, inplace=True), middle(in_ch, out_ch, batch_norm=False))


class UNetpRes(nn.Module):
    def __init__(self, n_channels, n_classes, device, neurons=16, dropout_ratio=0.5, alfa_type='free', rule='hebb',
                 nbf=128, batch_norm=False, bilinear_upsample=False, hebb_mode='slots'):
        super().__init__()
        if hebb_mode not in ("slots", "sequential"):
            raise ValueError("hebb_mode must be 'slots' or 'sequential'")
        self.hebb_mode = hebb_mode
        self.n_classes = n_classes
        self.n_channels = n_channels
        self.nbf = nbf
        self.torch_dev = device
        self.alfa_type = alfa_type
        self.rule = rule
        self.neurons = neurons
        self.dropout_ratio = dropout_ratio
        self.w = nn.Parameter(.01 * torch.randn(nbf, nbf), requires_grad=True)
        self.alpha = nn.Parameter(.01 * torch.rand(nbf, nbf), requires_grad=True)
        self.eta = nn.Parameter(.01 * torch.ones(1), requires_grad=True)
        n = neurons
        self.conv1 = down(n_channels, n, batch_norm=batch_norm)
        self.pool1 = pool_drop(dropout_ratio=dropout_ratio / 2)
        self.conv2 = down(n, n * 2, batch_norm=batch_norm)
        self.pool2 = pool_drop(dropout_ratio=dropout_ratio)
        self.conv3 = down(n * 2, n * 4, batch_norm=batch_norm)
        self.pool3 = pool_drop(dropout_ratio=dropout_ratio)
        self.conv4 = down(n * 4, n * 8, batch_norm=batch_norm)
        self.pool4 = pool_drop(dropout_ratio=dropout_ratio)
        self.mid = middle(n * 8, n * 16, batch_norm=batch_norm)
        self.uconv4 = up(n * 16, n * 8, dropout_ratio=dropout_ratio, batch_norm=batch_norm)
        self.uconv3 = up(n * 8, n * 4, dropout_ratio=dropout_ratio, batch_norm=batch_norm)
        self.uconv2 = up(n * 4, n * 2, dropout_ratio=dropout_ratio, batch_norm=batch_norm)
        self.uconv1 = up(n * 2, n * 1, dropout_ratio=dropout_ratio, batch_norm=batch_norm)
        self.outc = outconv(neurons, n_classes)
        self.to(device)
        print("UNet plastic model with plastic rule [%s] initialized" % self.rule)

    def _trunk_plan(self):
        if getattr(self, "_trunk", None) is None:
            from punet.res_trunk import ResTrunk
            self._trunk = ResTrunk(self)
        return self._trunk

    def forward(self, x, hebb):
        from .unet_p import _check_gpu_tensor
        single = hebb.dim() == 2
        B, C, Hh, Ww = x.shape
        seq = self.hebb_mode == "sequential"
        if seq and not single:
            raise ValueError("hebb_mode='sequential' threads one [nbf,nbf] trace through the batch")
        if single and B != 1 and not seq:
            # the reference has no explicit check: activin = x.view(nbf, nbf) fails (S8)
            raise RuntimeError("shape '[%d, %d]' is invalid for input of size %d"
                               % (self.nbf, self.nbf, B * Hh * Ww * self.n_classes))
        if self.alfa_type not in ("free", "yoked"):
            raise ValueError("Must select one plasticity coefficient type ('free' or 'yoked')")
        if self.rule not in ("hebb", "oja"):
            raise ValueError("Must select one learning rule ('hebb' or 'oja')")
        _check_gpu_tensor(x, "x")
        _check_gpu_tensor(hebb, "hebb")
        if self.n_classes != 1:
            raise RuntimeError("the plastic head needs n_classes == 1 (activin = x.view(nbf, nbf))")
        if C != self.n_channels:
            raise RuntimeError("expected input with %d channels, got %d" % (self.n_channels, C))
        if Hh * Ww != self.nbf * self.nbf or Hh != Ww:
            raise RuntimeError("shape '[%d, %d]' is invalid for input of size %d" % (self.nbf, self.nbf, Hh * Ww))
        if Hh < 16:
            raise RuntimeError("UNetpRes needs images of at least 16x16 (four 2x2 poolings)")
        H = hebb.unsqueeze(0) if single else hebb
        if H.shape != (B if not seq else 1, self.nbf, self.nbf):
            raise ValueError("hebb must be [nbf,nbf] or [B,nbf,nbf]; got %s for batch %d" % (tuple(hebb.shape), B))
        if x.dtype != torch.float32:
            x = x.float()
        from punet.res_trunk import ResTrunkFunction
        from punet.head import PlasticHeadFunction, RULES
        trunk = self._trunk_plan()
        params = trunk.params
        save = torch.is_grad_enabled() and any(p.requires_grad for p in params)
        from punet.head import fused_head_ok, FusedHeadFunction
        wo, bo = self.outc.conv.weight, self.outc.conv.bias
        trunk.fused_head = fused_head_ok(wo.shape[1], self.nbf, seq)
        logits = ResTrunkFunction.apply(trunk, save, self.training, x, *params)
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
        shape = (self.nbf, self.nbf) if batch is None else (batch, self.nbf, self.nbf)
        return torch.zeros(*shape, dtype=torch.float, device=self.torch_dev)
