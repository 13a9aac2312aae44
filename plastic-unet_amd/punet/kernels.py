"""torch-tensor wrappers over the C-ABI kernels (one wrapper per entry point of plastic_unet.h).

Every wrapper enqueues on torch's *current* HIP stream and never synchronises.  Tensors must be
fp32, contiguous and resident on the ROCm device; activations are NHWC.
"""
import ctypes
import os

import torch

from . import _lib
from ._lib import (ConvArgs, WgradArgs, PlasticArgs, PlasticHeadArgs, PlasticBwdArgs, AdamTensor, PackJob, WinoJob, check,
                   PU_EPI_RELU, PU_EPI_ACCUM, PU_EPI_SHUFFLE2, PU_EPI_RESID, PU_CONV_NO_HALO, PU_CONV_HALO_V1, PU_CONV_HALO_DMA,
                   PU_CONV_NO_SMALLX6, PU_EPI_OUT_BF16)

__all__ = ["KernelProfiler", "igemm", "wgrad", "pack_weight", "nchw_to_nhwc", "maxpool2_fwd", "maxpool2_bwd",
           "outconv_fwd", "outconv_bwd", "plastic_fwd", "trace_update", "plastic_bwd", "bce_fwd",
           "bce_bwd", "adam_multi", "pack_weights", "round16", "cgroup_for", "device_info", "lib"]


def lib():
    return _lib.load()


# ------------------------------------------------------------------------------ launch profiler
_PROF = None
_MODES = {0: "chunk16", 1: "vec4", 2: "scalar", 3: "direct", 4: "x6", 5: "stem", 6: "wino", 7: "x6s"}

# fp32 GEMM arithmetic of the MFMA convolutions: "split6" (default) = each fp32 product as 6 exact
# bf16 products on the bf16 MFMA pipe (pu_split_weight6 / pu_conv_args.weight6, fp32-accurate);
# "native" = v_mfma_f32_32x32x2_f32.  Read when a weight is packed and when a conv launches.
_FP32_MATH = os.environ.get("PU_FP32_MATH", "split6")


# bf16 3x3/s1 convolutions of width 32/64/128: 2 = the DMA-ring halo kernel (512-pixel
# row blocks, PU_CONV_HALO_DMA), 1 = the register-staged halo kernel (default, as at the C-ABI),
# 0 = the per-tap lean kernel (PU_CONV_HALO:
# A/B runs; tests flip it with set_conv_halo)
_CONV_HALO = int(os.environ.get("PU_CONV_HALO", "1"))


def set_conv_halo(mode):
    """Route eligible bf16 convolutions: 2 DMA-ring halo kernel, 1 (or True) register-staged halo
    kernel - the default, as at the C-ABI -, 0 (or False) per-tap kernel.  Returns the previous
    setting."""
    global _CONV_HALO
    prev, _CONV_HALO = _CONV_HALO, (1 if mode is True else 0 if mode is False else int(mode))
    return prev


def _halo_flags():
    # the C-ABI default (no flag) is the register-staged kernel; 2 opts in to the DMA ring
    return {2: PU_CONV_HALO_DMA, 1: 0}.get(_CONV_HALO, PU_CONV_NO_HALO)


def fp32_math():
    return _FP32_MATH


# fp32 3x3/s1/p1 convolutions (forward and data gradient) on the Winograd F(2x2,3x3) kernel where
# the layer qualifies (PU_WINO=0: the direct 6-product kernels everywhere; A/B runs, tests flip it
# with set_wino)
_WINO = os.environ.get("PU_WINO", "1") != "0"


# fp32 8/16-channel 3x3 convolutions on the 16x16x32 MFMA kernel (csrc/smallconv.hip) or the VALU
# direct kernel (PU_SMALLX6=0; tests flip it with set_smallx6)
_SMALLX6 = os.environ.get("PU_SMALLX6", "1") != "0"


def set_smallx6(on):
    """Route 8/16-channel fp32 3x3 convolutions to the MFMA kernel (True) or the VALU direct one."""
    global _SMALLX6
    prev, _SMALLX6 = _SMALLX6, bool(on)
    return prev


def set_wino(on):
    """Route eligible fp32 3x3 convolutions to the Winograd kernel (True) or the direct kernels.
    Returns the previous setting."""
    global _WINO
    prev, _WINO = _WINO, bool(on)
    return prev


# 32-tile x 128-channel Winograd items (csrc/winograd.hip wino128_use reads the same variables once
# per process): the one-wave-per-SIMD kernel's wide items (PU_WINO4_WIDE=1 everywhere, =2 - the
# default - for the short reductions only, =0 none), or with PU_WINO4=0 the 8-wave PU_WINO128=1 kernel
_WINO4 = os.environ.get("PU_WINO4", "1") != "0"
_WINO128 = os.environ.get("PU_WINO4_WIDE", "2") in ("1", "2") if _WINO4 else \
    os.environ.get("PU_WINO128", "0") == "1"


def wino_wanted(w, mode):
    """Whether a packed conv operand of parameter w (OIHW 3x3) should carry a Winograd operand:
    the reduced channel count a multiple of 32 and the produced one of 64 (the kernel's chunks
    and output blocks)."""
    if mode not in (0, 1) or w.dim() != 4 or w.shape[2:] != (3, 3) or _FP32_MATH != "split6":
        return False
    n, c = (w.shape[0], w.shape[1]) if mode == 0 else (w.shape[1], w.shape[0])
    # csrc wino_ok: a 64-channel reduction into more than 64 outputs only on 128-channel items
    return c % 32 == 0 and n % 64 == 0 and (c >= 128 or n <= 64 or (_WINO128 and n % 128 == 0))


def pack_wino(jobs):
    """pu_pack_wino: jobs = [(w, out, dgrad)] - U = G g G^T of each OIHW weight, exact bf16 planes."""
    if not jobs:
        return
    arr = (WinoJob * len(jobs))()
    nbytes = 0.0
    for i, (w, out, dgrad) in enumerate(jobs):
        _req(w, "w")
        arr[i] = WinoJob(w.data_ptr(), out.data_ptr(), w.shape[0], w.shape[1], int(dgrad))
        nbytes += 4.0 * w.numel() + 2.0 * out.numel()
    with _Rec("pack_wino", nbytes=nbytes):
        check(lib().pu_pack_wino(arr, len(jobs), _stream()), "pu_pack_wino")


def set_fp32_math(mode):
    """'split6' or 'native' (tests / ablations).  Returns the previous mode."""
    global _FP32_MATH
    if mode not in ("split6", "native"):
        raise ValueError("fp32 math must be 'split6' or 'native', got %r" % (mode,))
    prev, _FP32_MATH = _FP32_MATH, mode
    return prev


class KernelProfiler:
    """Brackets every wrapped launch with HIP events on the stream it is launched on, tagged with
    the kernel instantiation and its algorithmic FLOPs / bytes.  Use as a context manager."""

    def __init__(self):
        self.records = []

    def __enter__(self):
        global _PROF
        self._prev, _PROF = _PROF, self
        return self

    def __exit__(self, *exc):
        global _PROF
        _PROF = self._prev
        return False

    def summary(self):
        torch.cuda.synchronize()
        out = {}
        for tag, flops, nbytes, e0, e1 in self.records:
            d = out.setdefault(tag, {"launches": 0, "ms": 0.0, "flops": 0.0, "bytes": 0.0})
            d["launches"] += 1
            d["ms"] += e0.elapsed_time(e1)
            d["flops"] += flops
            d["bytes"] += nbytes
        return out


class _Rec:
    __slots__ = ("tag", "flops", "nbytes", "e0")

    def __init__(self, tag, flops=0.0, nbytes=0.0):
        self.tag, self.flops, self.nbytes = tag, flops, nbytes
        self.e0 = None

    def __enter__(self):
        if _PROF is not None:
            self.e0 = torch.cuda.Event(enable_timing=True)
            self.e0.record()
        return self

    def __exit__(self, *exc):
        if _PROF is not None and self.e0 is not None:
            e1 = torch.cuda.Event(enable_timing=True)
            e1.record()
            _PROF.records.append((self.tag, self.flops, self.nbytes, self.e0, e1))
        return False


def _p(t):
    return None if t is None else t.data_ptr()


_RAW_STREAM = getattr(torch._C, "_cuda_getCurrentRawStream", None)


def _stream():
    """The current stream's raw handle.  torch.cuda.current_stream() resolves the device through
    torch.cuda.is_available() and an environment lookup on every call (~2 us of host time, several
    hundred calls per training step); the raw accessor takes the device index directly."""
    if _RAW_STREAM is not None:
        return _RAW_STREAM(torch._C._cuda_getDevice())
    return torch.cuda.current_stream().cuda_stream


def round16(k):
    return (k + 15) // 16 * 16


def _req(t, name, dtype=torch.float32):
    if t is None:
        return
    if not t.is_cuda:
        raise RuntimeError("%s must be on the ROCm device (got %s); the plastic U-Net path has no CPU "
                           "fallback" % (name, t.device))
    if t.dtype != dtype:
        raise RuntimeError("%s must be %s (got %s)" % (name, dtype, t.dtype))
    if not t.is_contiguous():
        raise RuntimeError("%s must be contiguous" % name)


BF16 = torch.bfloat16


def _act_dtype(t):
    """Activation dtype of a call: float32, or bfloat16 for the bf16 (C3) entry points."""
    return BF16 if t.dtype == BF16 else torch.float32


def device_info(device=0):
    L = lib()
    cu, clk, mem = ctypes.c_int(), ctypes.c_int(), ctypes.c_longlong()
    check(L.pu_device_info(device, ctypes.byref(cu), ctypes.byref(clk), ctypes.byref(mem)), "pu_device_info")
    return cu.value, clk.value, mem.value


def cgroup_for(c0, c1=0):
    """K order for a packed conv operand: 32-channel groups when both sources allow it."""
    if c0 % 32 == 0 and c1 % 32 == 0:
        return 32
    if c0 % 16 == 0 and c1 % 16 == 0:
        return 16
    return 0


def igemm(*, batch, in_hw, out_hw, k, stride, pad, src0, c0, weight, k_pad, n, dst0, n0=None,
          src1=None, c1=0, bias=None, dst1=None, mask0=None, mask1=None, relu=False, accum=False,
          shuffle=False, cgroup=0, resid=None, shuf=(0, 0, 0), chan_scale=None):
    """pu_conv_igemm: implicit-GEMM conv (3x3 fwd/dgrad, ConvT fwd with shuffle, ConvT dgrad).
    resid: residual tensor added before ReLU/mask; shuf = (out_h, out_w, crop) of a SHUFFLE2 grid;
    chan_scale: [batch, ld] per-(image, column) factors applied after the mask (the Dropout2d scale
    of the tensor being produced; SHUFFLE2: per output channel).  A bf16 dst0 with fp32 operands
    is the single-channel stem writing the bf16 trunk's first activation (PU_EPI_OUT_BF16)."""
    dt = _act_dtype(src0)
    out_bf16 = dt == torch.float32 and dst0 is not None and dst0.dtype == BF16
    for t, nm in ((src0, "src0"), (src1, "src1"), (weight, "weight"), (dst0, "dst0"),
                  (dst1, "dst1"), (mask0, "mask0"), (mask1, "mask1"), (resid, "resid")):
        _req(t, nm, BF16 if (out_bf16 and nm == "dst0") else dt)
    _req(bias, "bias")
    _req(chan_scale, "chan_scale")
    flags = (PU_EPI_RELU if relu else 0) | (PU_EPI_ACCUM if accum else 0) | (PU_EPI_SHUFFLE2 if shuffle else 0) \
        | (PU_EPI_RESID if resid is not None else 0) | _halo_flags() | (0 if _SMALLX6 else PU_CONV_NO_SMALLX6) \
        | (PU_EPI_OUT_BF16 if out_bf16 else 0)
    a = ConvArgs(batch, in_hw[0], in_hw[1], out_hw[0], out_hw[1], k, k, stride, pad,
                 _p(src0), c0, _p(src1), c1, _p(weight), k_pad, cgroup, n, _p(bias),
                 _p(dst0), n if n0 is None else n0, _p(dst1), _p(mask0), _p(mask1), flags, None, 0,
                 _p(resid), shuf[0], shuf[1], shuf[2])
    if chan_scale is not None:
        if chan_scale.dim() != 2 or chan_scale.shape[0] != batch:
            raise RuntimeError("chan_scale must be [batch, channels]")
        a.chan_scale, a.chan_scale_ld = chan_scale.data_ptr(), chan_scale.shape[1]
    w6 = getattr(weight, "_split6", None) if (dt != BF16 and _FP32_MATH == "split6") else None
    wn = getattr(weight, "_wino", None) if (w6 is not None and _WINO) else None
    if w6 is not None:
        a.weight6 = w6.data_ptr()
    if wn is not None:
        a.wino = wn.data_ptr()
        # the signature wino_ok reads: shapes, flags, which operands exist, their alignment
        key = (batch, tuple(in_hw), tuple(out_hw), k, stride, pad, c0, c1, n, a.n0, k_pad, cgroup, flags,
               tuple(None if t is None else t.data_ptr() % 16
                     for t in (src0, src1, bias, dst0, dst1, mask0, mask1, resid, chan_scale, weight, w6, wn)))
        _ensure_direct(a, weight, key)
    elif getattr(weight, "_direct_ok", True) is False:     # a direct call (e.g. Winograd switched off)
        _refresh_direct(weight)
    L = lib()
    if dt == BF16:
        _igemm_bf16(L, a, batch, out_hw, k, c0, c1, n, dst0)
        return
    nbytes = L.pu_conv_igemm_workspace_bytes(ctypes.byref(a))
    if nbytes:     # split-K scratch from the caching allocator (stream-ordered reuse)
        ws = torch.empty(nbytes // 4 + 1, dtype=torch.float32, device=dst0.device)
        a.workspace, a.ws_bytes = ws.data_ptr(), nbytes
    if _PROF is None:
        check(L.pu_conv_igemm(ctypes.byref(a), _stream()), "pu_conv_igemm")
        return
    bm, bn, mode, ks = ctypes.c_int(), ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
    L.pu_conv_igemm_tile(ctypes.byref(a), ctypes.byref(bm), ctypes.byref(bn), ctypes.byref(mode), ctypes.byref(ks))
    M = batch * out_hw[0] * out_hw[1]
    tag = "igemm<%dx%d,%s%s>" % (bm.value, bn.value, _MODES[mode.value], ",k%d" % ks.value if ks.value > 1 else "")
    nb = 0.0
    if mode.value in (3, 5, 7):    # small-channel / stem kernels: HBM-bound, report algorithmic bytes
        per = (c0 + c1) + n * (1 + int(accum) + int(resid is not None)) + n0_mask(n, n0, mask0, mask1)
        nb = 4.0 * M * per
    with _Rec(tag, flops=2.0 * M * n * k * k * (c0 + c1), nbytes=nb):
        check(L.pu_conv_igemm(ctypes.byref(a), _stream()), "pu_conv_igemm")


def n0_mask(n, n0, mask0, mask1):
    """channels of the ReLU masks an igemm epilogue reads"""
    n0 = n if n0 is None else n0
    return (n0 if mask0 is not None else 0) + (n - n0 if mask1 is not None else 0)


def _igemm_bf16(L, a, batch, out_hw, k, c0, c1, n, dst0):
    nbytes = L.pu_conv_igemm_bf16_workspace_bytes(ctypes.byref(a))
    if nbytes:
        ws = torch.empty(nbytes // 4 + 1, dtype=torch.float32, device=dst0.device)
        a.workspace, a.ws_bytes = ws.data_ptr(), nbytes
    if _PROF is None:
        check(L.pu_conv_igemm_bf16(ctypes.byref(a), _stream()), "pu_conv_igemm_bf16")
        return
    bm, bn, ks, kind = ctypes.c_int(), ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
    L.pu_conv_igemm_bf16_tile(ctypes.byref(a), ctypes.byref(bm), ctypes.byref(bn), ctypes.byref(ks), ctypes.byref(kind))
    M = batch * out_hw[0] * out_hw[1]
    tag = "igemm_bf16<%dx%d%s%s>" % (bm.value, bn.value, ("", ",lean", ",halo", ",rows")[kind.value],
                                     ",k%d" % ks.value if ks.value > 1 else "")
    with _Rec(tag, flops=2.0 * M * n * k * k * (c0 + c1)):
        check(L.pu_conv_igemm_bf16(ctypes.byref(a), _stream()), "pu_conv_igemm_bf16")


def wgrad(*, batch, in_hw, out_hw, k, stride, pad, rows, n, src0, c0, dweight, src1=None, c1=0,
          bias_mode=0, dbias=None, accumulate=False):
    """pu_wgrad: split-K weight (+bias) gradient into PyTorch's [n][c][k][k] layout (fp32, or
    bf16 rows/sources with fp32 gradients)."""
    # bf16 dZ with an fp32 single-channel source: the bf16 trunk's stem (pu_wgrad math 2)
    stem_bf16 = rows.dtype == BF16 and src0.dtype == torch.float32 and c0 == 1 and src1 is None
    dt = torch.float32 if stem_bf16 else _act_dtype(rows)
    for t, nm in ((rows, "rows"), (src0, "src0"), (src1, "src1")):
        _req(t, nm, BF16 if (stem_bf16 and nm == "rows") else dt)
    _req(dweight, "dweight"); _req(dbias, "dbias")
    a = WgradArgs(batch, in_hw[0], in_hw[1], out_hw[0], out_hw[1], k, k, stride, pad,
                  _p(rows), n, _p(src0), c0, _p(src1), c1, bias_mode, _p(dweight), _p(dbias),
                  1 if accumulate else 0, 2 if stem_bf16 else (1 if (dt != BF16 and _FP32_MATH == "split6") else 0))
    L = lib()
    if dt == BF16:
        nbytes = L.pu_wgrad_bf16_workspace_bytes(ctypes.byref(a))
        ws = torch.empty(max(nbytes // 4, 1), dtype=torch.float32, device=rows.device)
        if nbytes == 0 or _PROF is None:
            check(L.pu_wgrad_bf16(ctypes.byref(a), ws.data_ptr(), nbytes, _stream()), "pu_wgrad_bf16")
            return
        M = batch * out_hw[0] * out_hw[1]
        bn, bk, hl = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        check(L.pu_wgrad_bf16_tile(ctypes.byref(a), ctypes.byref(bn), ctypes.byref(bk), ctypes.byref(hl), None),
              "pu_wgrad_bf16_tile")
        tag = "wgrad_bf16<%dx%d%s>" % (bn.value, bk.value, ",halo" if hl.value else "")
        with _Rec(tag, flops=2.0 * M * n * k * k * (c0 + c1)):
            check(L.pu_wgrad_bf16_phase(ctypes.byref(a), ws.data_ptr(), nbytes, 1, _stream()), "pu_wgrad_bf16")
        with _Rec("wgrad_reduce", nbytes=float(nbytes)):
            check(L.pu_wgrad_bf16_phase(ctypes.byref(a), ws.data_ptr(), nbytes, 2, _stream()), "pu_wgrad_bf16")
        return
    nbytes = L.pu_wgrad_workspace_bytes(ctypes.byref(a))
    if nbytes == 0:
        check(L.pu_wgrad(ctypes.byref(a), None, 0, _stream()), "pu_wgrad")
        return
    ws = torch.empty(max(nbytes // 4, 1), dtype=torch.float32, device=rows.device)
    if _PROF is None:
        check(L.pu_wgrad(ctypes.byref(a), ws.data_ptr(), nbytes, _stream()), "pu_wgrad")
        return
    bn, bk, qv, sp = ctypes.c_int(), ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
    L.pu_wgrad_tile(ctypes.byref(a), ctypes.byref(bn), ctypes.byref(bk), ctypes.byref(qv), ctypes.byref(sp))
    M = batch * out_hw[0] * out_hw[1]
    tag = "wgrad<%dx%d,%s>" % (bn.value, bk.value, ("scalar", "vec4", "direct", "halo", "stem", "wino", "pointwise")[qv.value])
    if a.math == 1 and qv.value in (1, 3, 5):
        tag = tag[:-1] + ",x6>"
    # the GEMM and the split reduction timed apart (they are separate kernels in rocprof too)
    with _Rec(tag, flops=2.0 * M * n * k * k * (c0 + c1)):
        check(L.pu_wgrad_phase(ctypes.byref(a), ws.data_ptr(), nbytes, 1, _stream()), "pu_wgrad_phase")
    with _Rec("wgrad_reduce", nbytes=float(nbytes)):
        check(L.pu_wgrad_phase(ctypes.byref(a), ws.data_ptr(), nbytes, 2, _stream()), "pu_wgrad_phase")


def wgrad_kind(*, batch, hw, n, c0, c1=0, k=3):
    """Which kernel pu_wgrad takes for an fp32 kxk/s1 same-size ('same' padding) weight gradient
    (pu_wgrad_tile's loader kind: 1 float4 GEMM, 2 small-channel direct, 3 halo, 4 stem,
    5 Winograd-domain, 6 pointwise)."""
    a = WgradArgs(batch, hw[0], hw[1], hw[0], hw[1], k, k, 1, (k - 1) // 2, 16, n, 16, c0, 16 if c1 else None, c1, 1,
                  16, 16,
                  0, 1 if _FP32_MATH == "split6" else 0)
    bn, bk, qv, sp = ctypes.c_int(), ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
    check(lib().pu_wgrad_tile(ctypes.byref(a), ctypes.byref(bn), ctypes.byref(bk), ctypes.byref(qv), ctypes.byref(sp)),
          "pu_wgrad_tile")
    return qv.value


def pack_weight(w, mode, k_pad, out=None, cgroup=0, dtype=torch.float32):
    """Pack an fp32 parameter into a GEMM operand (fp32, or bf16 for the C3 kernels)."""
    _req(w, "w")
    d0, d1, kh, kw = w.shape
    taps = kh * kw
    rows = {0: d0, 1: d1, 2: taps * d1, 3: d0, 4: 4 * d1}[mode]
    if out is None:
        out = torch.empty(rows, k_pad, dtype=dtype, device=w.device)
    fn = lib().pu_pack_weight_bf16 if out.dtype == BF16 else lib().pu_pack_weight
    with _Rec("pack_weight", nbytes=4.0 * w.numel() + out.element_size() * out.numel()):
        check(fn(w.data_ptr(), out.data_ptr(), mode, d0, d1, kh, kw, k_pad, cgroup, _stream()), "pu_pack_weight")
    if out.dtype == torch.float32 and _FP32_MATH == "split6" and k_pad % 16 == 0:
        out._split6 = split_weight6(out)      # travels with the packed operand (igemm picks it up)
        # so does the Winograd operand of a 3x3 conv - only while Winograd dispatch is on, so a
        # PU_WINO=0 run neither holds nor refreshes U (set_wino before packing to switch)
        if _WINO and wino_wanted(w, mode):
            n, c = (d0, d1) if mode == 0 else (d1, d0)
            out._wino = torch.empty(lib().pu_wino_bytes(n, c) // 2, dtype=BF16, device=w.device)
            pack_wino([(w, out._wino, mode == 1)])
            # the direct operand of a layer that only ever runs on Winograd is not refreshed after
            # the optimizer step (trunk._Packs.refresh); igemm repacks it on the first call that
            # takes the direct kernel (_ensure_direct)
            out._src, out._direct_ok, out._wino_only = w, True, True
        elif hasattr(out, "_wino"):
            # a U packed from the old weights must not outlive them: repacked in place with
            # Winograd off, then Winograd back on, igemm would otherwise run on the stale U
            del out._wino
            # no Winograd path any more: the direct operand is the one igemm uses, refreshed
            # every step like any other (trunk._Packs.refresh)
            out._wino_only, out._direct_ok = False, True
    out._pack_spec = (mode, k_pad, cgroup)    # pack_weights() refreshes it in place
    return out


def pack_weights(jobs, wino=True):
    """Refresh many packed operands in one launch (pu_pack_weights).  jobs: (w, packed, planes) with
    ``packed`` an output of pack_weight (fp32 or bf16; its mode / k_pad / cgroup are read from the
    attributes pack_weight stored on it) and ``planes`` its split6 planes or None.  wino: also
    refresh the Winograd operands the packed operands carry (one more launch)."""
    if not jobs:
        return
    arr = (PackJob * len(jobs))()
    nbytes = 0.0
    for i, (w, packed, planes) in enumerate(jobs):
        _req(w, "w")
        mode, k_pad, cg = packed._pack_spec
        d0, d1, kh, kw = w.shape
        bf = packed.dtype == BF16
        arr[i] = PackJob(w.data_ptr(), None if bf else packed.data_ptr(), packed.data_ptr() if bf else None,
                         None if planes is None else planes.data_ptr(), mode, d0, d1, kh, kw, k_pad, cg)
        nbytes += 4.0 * w.numel() + packed.element_size() * packed.numel() + (0 if planes is None else 2.0 * planes.numel())
    with _Rec("pack_weight", nbytes=nbytes):
        check(lib().pu_pack_weights(arr, len(jobs), _stream()), "pu_pack_weights")
    for _, packed, _ in jobs:
        if hasattr(packed, "_direct_ok"):
            packed._direct_ok = True
    if wino:
        pack_wino([(w, packed._wino, packed._pack_spec[0] == 1) for w, packed, _ in jobs
                   if getattr(packed, "_wino", None) is not None])


_WINO_TAKES = {}    # call signature -> does pu_conv_igemm take the Winograd kernel for it


def _ensure_direct(a, weight, key):
    """A Winograd-carrying operand on a call: if the library takes the direct kernel for this call
    (pu_conv_igemm_tile's answer, cached per signature), refresh the direct operand if the last
    repack skipped it, and keep refreshing it from now on."""
    takes = _WINO_TAKES.get(key)
    if takes is None:
        bm, bn, mode, ks = ctypes.c_int(), ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        check(lib().pu_conv_igemm_tile(ctypes.byref(a), ctypes.byref(bm), ctypes.byref(bn), ctypes.byref(mode),
                                       ctypes.byref(ks)), "pu_conv_igemm_tile")
        takes = _WINO_TAKES[key] = mode.value == 6
    if not takes:
        weight._wino_only = False
        if not weight._direct_ok:
            _refresh_direct(weight)


def _refresh_direct(weight):
    weight._wino_only = False
    pack_weights([(weight._src, weight, getattr(weight, "_split6", None))], wino=False)


def split_weight6(packed):
    """packed fp32 [n][k_pad] -> bf16 planes [k_pad/16][6][n][8] (hi/mid/lo, exact split)."""
    _req(packed, "packed")
    n, k_pad = packed.shape
    out = torch.empty(k_pad // 16, 6, n, 8, dtype=BF16, device=packed.device)
    with _Rec("pack_weight", nbytes=4.0 * packed.numel() + 6.0 * packed.numel()):
        check(lib().pu_split_weight6(packed.data_ptr(), out.data_ptr(), n, k_pad, _stream()), "pu_split_weight6")
    return out


def to_bf16(x):
    _req(x, "x")
    y = torch.empty(x.shape, dtype=BF16, device=x.device)
    with _Rec("convert", nbytes=6.0 * x.numel()):
        check(lib().pu_convert_f32_bf16(x.data_ptr(), y.data_ptr(), x.numel(), _stream()), "pu_convert_f32_bf16")
    return y


def to_f32(x):
    _req(x, "x", BF16)
    y = torch.empty(x.shape, dtype=torch.float32, device=x.device)
    with _Rec("convert", nbytes=6.0 * x.numel()):
        check(lib().pu_convert_bf16_f32(x.data_ptr(), y.data_ptr(), x.numel(), _stream()), "pu_convert_bf16_f32")
    return y


def nchw_to_nhwc(x):
    _req(x, "x")
    B, C, H, W = x.shape
    out = torch.empty(B, H, W, C, dtype=torch.float32, device=x.device)
    check(lib().pu_nchw_to_nhwc(x.data_ptr(), out.data_ptr(), B, C, H, W, _stream()), "pu_nchw_to_nhwc")
    return out


def channel_scale(x, scale, out=None):
    """Dropout2d on NHWC x [B,H,W,C] with per-(sample, channel) scale [B,C]; out may be x."""
    _req(x, "x"); _req(scale, "scale")
    B, H, W, C = x.shape
    y = torch.empty_like(x) if out is None else out
    with _Rec("channel_scale", nbytes=8.0 * x.numel()):
        check(lib().pu_channel_scale(x.data_ptr(), scale.data_ptr(), y.data_ptr(), B, H * W, C, _stream()),
              "pu_channel_scale")
    return y


def add_coords(x, with_r):
    """NCHW input [B,C,H,W] -> NHWC [B,H,W,C+2(+1)] with the AddCoords channels appended."""
    _req(x, "x")
    B, C, H, W = x.shape
    out = torch.empty(B, H, W, C + 2 + int(with_r), dtype=torch.float32, device=x.device)
    with _Rec("add_coords", nbytes=4.0 * (x.numel() + out.numel())):
        check(lib().pu_add_coords(x.data_ptr(), out.data_ptr(), B, C, H, W, int(with_r), _stream()), "pu_add_coords")
    return out


def column_sum(x2d, out=None, accumulate=False):
    """Deterministic fp64 column sums of a row-major [rows, cols] tensor."""
    _req(x2d, "x")
    rows, cols = x2d.shape
    if out is None:
        out = torch.empty(cols, dtype=torch.float32, device=x2d.device)
    L = lib()
    nbytes = L.pu_column_sum_workspace_bytes(rows, cols)
    ws = torch.empty(nbytes // 4 + 1, dtype=torch.float32, device=x2d.device)
    with _Rec("column_sum", nbytes=4.0 * x2d.numel()):
        check(L.pu_column_sum(x2d.data_ptr(), rows, cols, out.data_ptr(), int(accumulate), ws.data_ptr(), nbytes,
                              _stream()), "pu_column_sum")
    return out


def maxpool2_fwd(x, scale=None):
    """MaxPool2d(2); scale [B, C] (fp32 only): the Dropout2d that follows the pool, fused."""
    dt = _act_dtype(x)
    _req(x, "x", dt)
    B, H, W, C = x.shape
    y = torch.empty(B, H // 2, W // 2, C, dtype=dt, device=x.device)
    with _Rec("maxpool_fwd", nbytes=x.element_size() * (x.numel() + y.numel())):
        if scale is not None:
            _req(x, "x"); _req(scale, "scale")       # fp32 entry point
            check(lib().pu_maxpool2_fwd_scaled(x.data_ptr(), scale.data_ptr(), y.data_ptr(), B, H, W, C, _stream()),
                  "pu_maxpool2_fwd_scaled")
        else:
            fn = lib().pu_maxpool2_fwd_bf16 if dt == BF16 else lib().pu_maxpool2_fwd
            check(fn(x.data_ptr(), y.data_ptr(), B, H, W, C, _stream()), "pu_maxpool2_fwd")
    return y


def maxpool2_bwd(x, dy, dx, relu_mask=True, accumulate=True, scale=None):
    """MaxPool2d(2) backward; scale [B, C] (fp32 only): dy * scale routed (the Dropout2d backward)."""
    dt = _act_dtype(x)
    _req(x, "x", dt); _req(dy, "dy", dt); _req(dx, "dx", dt)
    B, H, W, C = x.shape
    with _Rec("maxpool_bwd", nbytes=x.element_size() * (x.numel() * (3 if accumulate else 2) + dy.numel())):
        if scale is not None:
            _req(x, "x"); _req(scale, "scale")       # fp32 entry point
            check(lib().pu_maxpool2_bwd_scaled(x.data_ptr(), dy.data_ptr(), scale.data_ptr(), dx.data_ptr(), B, H, W,
                                               C, int(relu_mask), int(accumulate), _stream()), "pu_maxpool2_bwd_scaled")
        else:
            fn = lib().pu_maxpool2_bwd_bf16 if dt == BF16 else lib().pu_maxpool2_bwd
            check(fn(x.data_ptr(), dy.data_ptr(), dx.data_ptr(), B, H, W, C, int(relu_mask), int(accumulate),
                     _stream()), "pu_maxpool2_bwd")
    return dx


def outconv_fwd(x, w, b):
    """x [B,H,W,C] NHWC, w [C] (flattened [1,C,1,1]), b [1] -> logits [B,H,W]."""
    dt = _act_dtype(x)
    _req(x, "x", dt); _req(w, "w"); _req(b, "b")
    B, H, W, C = x.shape
    y = torch.empty(B, H, W, dtype=torch.float32, device=x.device)
    fn = lib().pu_outconv_fwd_bf16 if dt == BF16 else lib().pu_outconv_fwd
    with _Rec("outconv_fwd", nbytes=x.element_size() * x.numel() + 4.0 * y.numel()):
        check(fn(x.data_ptr(), w.data_ptr(), _p(b), y.data_ptr(), B * H * W, C, _stream()), "pu_outconv_fwd")
    return y


def outconv_bwd(x, w, dy, relu_mask=True, out=None):
    dt = _act_dtype(x)
    _req(x, "x", dt); _req(w, "w"); _req(dy, "dy")
    B, H, W, C = x.shape
    rows = B * H * W
    dx = torch.empty_like(x)
    if out is None:
        dw = torch.empty(C, dtype=torch.float32, device=x.device)
        db = torch.empty(1, dtype=torch.float32, device=x.device)
    else:
        dw, db = out
    L = lib()
    nbytes = L.pu_outconv_workspace_bytes(rows, C)
    ws = torch.empty(nbytes // 4 + 1, dtype=torch.float32, device=x.device)
    fn = L.pu_outconv_bwd_bf16 if dt == BF16 else L.pu_outconv_bwd
    with _Rec("outconv_bwd", nbytes=x.element_size() * 2.0 * x.numel() + 4.0 * rows):
        check(fn(x.data_ptr(), w.data_ptr(), dy.data_ptr(), dx.data_ptr(), dw.data_ptr(), db.data_ptr(),
                 rows, C, int(relu_mask), ws.data_ptr(), nbytes, _stream()), "pu_outconv_bwd")
    return dx, dw, db


def plastic_fwd(x, hebb, w, alpha, eta, rule, update_trace=True):
    """x, hebb [B,N,N] -> (y [B,N,N], hebb' [B,N,N] or None)."""
    for t, nm in ((x, "x"), (hebb, "hebb"), (w, "w"), (alpha, "alpha"), (eta, "eta")):
        _req(t, nm)
    B, N, _ = x.shape
    y = torch.empty_like(x)
    hn = torch.empty_like(hebb) if update_trace else None
    a = PlasticArgs(B, N, x.data_ptr(), hebb.data_ptr(), w.data_ptr(), alpha.data_ptr(), eta.data_ptr(),
                    y.data_ptr(), _p(hn), rule)
    with _Rec("plastic_fwd", flops=2.0 * B * N ** 3, nbytes=4.0 * (4 * B * N * N + 2 * N * N)):
        check(lib().pu_plastic_fwd(ctypes.byref(a), _stream()), "pu_plastic_fwd")
    return y, hn


def plastic_head_fwd(feat, wo, bo, hebb, w, alpha, eta, rule, update_trace=True):
    """The fused head (pu_plastic_head_fwd): feat [B,N,N,C] NHWC (fp32 / bf16), wo [C], bo [1] ->
    (X [B,N,N] logits, Y [B,N,N], hebb' [B,N,N] or None)."""
    dt = _act_dtype(feat)
    _req(feat, "feat", dt)
    for t, nm in ((wo, "wo"), (bo, "bo"), (hebb, "hebb"), (w, "w"), (alpha, "alpha"), (eta, "eta")):
        _req(t, nm)
    B, N, _, C = feat.shape
    X = torch.empty(B, N, N, dtype=torch.float32, device=feat.device)
    y = torch.empty_like(X)
    hn = torch.empty_like(hebb) if update_trace else None
    a = PlasticHeadArgs(B, N, C, feat.data_ptr(), int(dt == BF16), wo.data_ptr(), bo.data_ptr(), hebb.data_ptr(),
                        w.data_ptr(), alpha.data_ptr(), eta.data_ptr(), X.data_ptr(), y.data_ptr(), _p(hn), rule)
    nbytes = feat.element_size() * feat.numel() + 4.0 * (4 * B * N * N + 2 * N * N)
    with _Rec("plastic_head_fwd", flops=2.0 * B * N ** 3 + 2.0 * B * N * N * C, nbytes=nbytes):
        check(lib().pu_plastic_head_fwd(ctypes.byref(a), _stream()), "pu_plastic_head_fwd")
    return X, y, hn


def trace_update(hebb, x, y, eta, rule, out=None):
    for t, nm in ((hebb, "hebb"), (x, "x"), (y, "y"), (eta, "eta")):
        _req(t, nm)
    B, N, _ = hebb.shape
    out = torch.empty_like(hebb) if out is None else out
    with _Rec("trace_update", nbytes=8.0 * B * N * N + 8.0 * B * N):
        _trace(hebb, x, y, eta, out, B, N, rule)
    return out


def _trace(hebb, x, y, eta, out, B, N, rule):
    check(lib().pu_trace_update(hebb.data_ptr(), x.data_ptr(), y.data_ptr(), eta.data_ptr(), out.data_ptr(), B, N,
                                rule, _stream()), "pu_trace_update")


def plastic_bwd(x, hebb, w, alpha, y, dy, need_dx=True, need_dw=True, out=None):
    for t, nm in ((x, "x"), (hebb, "hebb"), (w, "w"), (alpha, "alpha"), (y, "y"), (dy, "dy")):
        _req(t, nm)
    B, N, _ = x.shape
    dx = torch.empty_like(x) if need_dx else None
    if out is not None and need_dw:
        dw, da = out
    else:
        dw = torch.empty_like(w) if need_dw else None
        da = torch.empty_like(alpha) if need_dw else None
    L = lib()
    nbytes = L.pu_plastic_bwd_workspace_bytes(B, N)
    ws = torch.empty(nbytes // 4 + 1, dtype=torch.float32, device=x.device) if need_dw else None
    a = PlasticBwdArgs(B, N, x.data_ptr(), hebb.data_ptr(), w.data_ptr(), alpha.data_ptr(), y.data_ptr(),
                       dy.data_ptr(), _p(dx), _p(dw), _p(da))
    with _Rec("plastic_bwd", flops=4.0 * B * N ** 3):
        check(L.pu_plastic_bwd(ctypes.byref(a), _p(ws), nbytes if need_dw else 0, _stream()), "pu_plastic_bwd")
    return dx, dw, da


def bce_fwd(y, t):
    _req(y, "y"); _req(t, "t")
    n = y.numel()
    if t.numel() != n:
        raise ValueError("Target size (%s) must be the same as input size (%s)" % (tuple(t.shape), tuple(y.shape)))
    L = lib()
    nbytes = L.pu_bce_workspace_bytes(n)
    ws = torch.empty(nbytes // 4 + 1, dtype=torch.float32, device=y.device)
    loss = torch.empty((), dtype=torch.float32, device=y.device)
    check(L.pu_bce_fwd(y.data_ptr(), t.data_ptr(), n, loss.data_ptr(), ws.data_ptr(), nbytes, _stream()), "pu_bce_fwd")
    return loss


def bce_bwd(y, t, grad_loss):
    _req(y, "y"); _req(t, "t")
    dy = torch.empty_like(y)
    g = grad_loss.contiguous() if grad_loss is not None else None
    check(lib().pu_bce_bwd(y.data_ptr(), t.data_ptr(), y.numel(), _p(g), dy.data_ptr(), _stream()), "pu_bce_bwd")
    return dy


def adam_multi(params, grads, exp_avgs, exp_avg_sqs, beta1, beta2, eps, weight_decay, step_size, bc2_sqrt):
    n = len(params)
    arr = (AdamTensor * max(n, 1))()
    for i, (p, g, m, v) in enumerate(zip(params, grads, exp_avgs, exp_avg_sqs)):
        arr[i] = AdamTensor(p.data_ptr(), g.data_ptr(), m.data_ptr(), v.data_ptr(), p.numel())
    with _Rec("adam", nbytes=28.0 * sum(p.numel() for p in params)):
        check(lib().pu_adam_multi(arr, n, beta1, beta2, eps, weight_decay, step_size, bc2_sqrt, _stream()),
              "pu_adam_multi")


# --------------------------------------------------------------------- BatchNorm2d / bilinear 2x
def bn_fwd(z, gamma, beta, running_mean, running_var, eps, momentum, training, relu=True, resid=None):
    """BatchNorm2d (+ReLU) over NHWC z [B,H,W,C].  training: per-slot statistics over H x W (the
    reference's bs=1 BatchNorm, slot by slot) and B in-order running-statistic updates; else the
    running statistics; resid is added before the ReLU.  Returns (y, save_mean [B,C] or [C], save_rstd)."""
    _req(z, "z"); _req(resid, "resid")
    B, H, W, C = z.shape
    y = torch.empty_like(z)
    shape = (B, C) if training else (C,)
    mean = torch.empty(shape, dtype=torch.float32, device=z.device)
    rstd = torch.empty(shape, dtype=torch.float32, device=z.device)
    L = lib()
    nbytes = L.pu_bn_workspace_bytes(B, H * W, C)
    ws = torch.empty(max(nbytes // 4, 1), dtype=torch.float32, device=z.device)
    with _Rec("batchnorm_fwd", nbytes=4.0 * (3 if training else 2) * z.numel()):
        check(L.pu_bn_fwd(z.data_ptr(), _p(gamma), _p(beta), _p(running_mean), _p(running_var), y.data_ptr(),
                          mean.data_ptr(), rstd.data_ptr(), B, H * W, C, float(eps), float(momentum),
                          1 if training else 0, 1 if relu else 0, _p(resid), ws.data_ptr(), nbytes, _stream()),
              "pu_bn_fwd")
    return y, mean, rstd


def bn_bwd(z, g, mean, rstd, gamma, dgamma=None, dbeta=None, add=None, mask=None):
    """Backward of the training-mode BatchNorm2d given g = dL/d(BN output) (ReLU mask already
    applied): returns dz (+ add, times (mask > 0) when given); writes dgamma / dbeta [C]."""
    _req(z, "z"); _req(g, "g"); _req(add, "add"); _req(mask, "mask")
    B, H, W, C = z.shape
    dz = torch.empty_like(z)
    L = lib()
    nbytes = L.pu_bn_workspace_bytes(B, H * W, C)
    ws = torch.empty(max(nbytes // 4, 1), dtype=torch.float32, device=z.device)
    with _Rec("batchnorm_bwd", nbytes=4.0 * 5 * z.numel()):
        check(L.pu_bn_bwd(z.data_ptr(), g.data_ptr(), mean.data_ptr(), rstd.data_ptr(), _p(gamma), dz.data_ptr(),
                          _p(dgamma), _p(dbeta), B, H * W, C, _p(add), _p(mask), ws.data_ptr(), nbytes, _stream()),
              "pu_bn_bwd")
    return dz


def upsample_bilinear2x(x):
    """nn.Upsample(scale_factor=2, mode='bilinear', align_corners=True) on NHWC x."""
    _req(x, "x")
    B, h, w, C = x.shape
    y = torch.empty(B, 2 * h, 2 * w, C, dtype=torch.float32, device=x.device)
    with _Rec("upsample_fwd", nbytes=4.0 * (x.numel() + y.numel())):
        check(lib().pu_upsample_bilinear2x_fwd(x.data_ptr(), y.data_ptr(), B, h, w, C, _stream()),
              "pu_upsample_bilinear2x_fwd")
    return y


def upsample_bilinear2x_bwd(dy, mask=None):
    """Gradient of upsample_bilinear2x w.r.t. its input, times (mask > 0) when given."""
    _req(dy, "dy"); _req(mask, "mask")
    B, H2, W2, C = dy.shape
    dx = torch.empty(B, H2 // 2, W2 // 2, C, dtype=torch.float32, device=dy.device)
    with _Rec("upsample_bwd", nbytes=4.0 * (dy.numel() + 2 * dx.numel())):
        check(lib().pu_upsample_bilinear2x_bwd(dy.data_ptr(), _p(mask), dx.data_ptr(), B, H2 // 2, W2 // 2, C,
                                               _stream()), "pu_upsample_bilinear2x_bwd")
    return dx
