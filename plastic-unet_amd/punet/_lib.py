"""ctypes binding of libplastic_unet.so (include/plastic_unet.h).

The library is the product's only compute path: importing a kernel wrapper without it raises
immediately - there is no CPU or eager-PyTorch fallback.  load() imports torch first so the HIP
runtime torch ships (libamdhip64.so.7) is the one the library binds to; our kernels then run on
torch's streams and device memory (PU_NO_TORCH=1 skips that: the host-ASan test loads the library
into a torch-free interpreter).
"""
import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("PLASTIC_UNET_LIB",
                          os.path.join(os.path.dirname(HERE), "lib", "libplastic_unet.so"))

c_int, c_ll, c_size, c_float, c_void_p = ctypes.c_int, ctypes.c_longlong, ctypes.c_size_t, ctypes.c_float, ctypes.c_void_p
c_double = ctypes.c_double
P = ctypes.c_void_p

(PU_EPI_RELU, PU_EPI_ACCUM, PU_EPI_SHUFFLE2, PU_EPI_RESID, PU_CONV_NO_HALO, PU_CONV_HALO_V1, PU_CONV_NO_SMALLX6,
 PU_CONV_HALO_DMA, PU_EPI_OUT_BF16) = 1, 2, 4, 8, 16, 32, 64, 128, 256
PU_PACK_CONV_FWD, PU_PACK_CONV_DGRAD, PU_PACK_CONVT_FWD, PU_PACK_CONVT_DGRAD, PU_PACK_CONVT3_FWD = 0, 1, 2, 3, 4
PU_RULE_HEBB, PU_RULE_OJA = 0, 1


ABI_VERSION = 3    # include/plastic_unet.h PU_ABI_VERSION


class ConvArgs(ctypes.Structure):
    _fields_ = [("batch", c_int), ("in_h", c_int), ("in_w", c_int), ("out_h", c_int), ("out_w", c_int),
                ("kh", c_int), ("kw", c_int), ("stride", c_int), ("pad", c_int),
                ("src0", P), ("c0", c_int), ("src1", P), ("c1", c_int),
                ("weight", P), ("k_pad", c_int), ("cgroup", c_int), ("n", c_int), ("bias", P),
                ("dst0", P), ("n0", c_int), ("dst1", P), ("mask0", P), ("mask1", P), ("flags", c_int),
                ("workspace", P), ("ws_bytes", c_size),
                ("resid", P), ("shuf_h", c_int), ("shuf_w", c_int), ("shuf_off", c_int),
                ("weight6", P), ("wino", P), ("chan_scale", P), ("chan_scale_ld", c_int)]


class WgradArgs(ctypes.Structure):
    _fields_ = [("batch", c_int), ("in_h", c_int), ("in_w", c_int), ("out_h", c_int), ("out_w", c_int),
                ("kh", c_int), ("kw", c_int), ("stride", c_int), ("pad", c_int),
                ("rows", P), ("n", c_int), ("src0", P), ("c0", c_int), ("src1", P), ("c1", c_int),
                ("bias_mode", c_int), ("dweight", P), ("dbias", P), ("accumulate", c_int),
                ("math", c_int)]


class PlasticArgs(ctypes.Structure):
    _fields_ = [("batch", c_int), ("nbf", c_int), ("x", P), ("hebb", P), ("w", P), ("alpha", P), ("eta", P),
                ("y", P), ("hebb_out", P), ("rule", c_int)]


class PlasticHeadArgs(ctypes.Structure):
    _fields_ = [("batch", c_int), ("nbf", c_int), ("channels", c_int), ("feat", P), ("feat_bf16", c_int),
                ("out_w", P), ("out_b", P), ("hebb", P), ("w", P), ("alpha", P), ("eta", P), ("x", P), ("y", P),
                ("hebb_out", P), ("rule", c_int)]


class PlasticBwdArgs(ctypes.Structure):
    _fields_ = [("batch", c_int), ("nbf", c_int), ("x", P), ("hebb", P), ("w", P), ("alpha", P), ("y", P),
                ("dy", P), ("dx", P), ("dw", P), ("dalpha", P)]


class AdamTensor(ctypes.Structure):
    _fields_ = [("param", P), ("grad", P), ("exp_avg", P), ("exp_avg_sq", P), ("numel", c_ll)]


class WinoJob(ctypes.Structure):
    _fields_ = [("w", P), ("out", P), ("cout", c_int), ("cin", c_int), ("dgrad", c_int)]


class PackJob(ctypes.Structure):
    _fields_ = [("w", P), ("packed", P), ("packed_bf16", P), ("planes", P), ("mode", c_int), ("d0", c_int),
                ("d1", c_int), ("kh", c_int), ("kw", c_int), ("k_pad", c_int), ("cgroup", c_int)]


# every symbol declared in include/plastic_unet.h: (name, restype, argtypes)
SIGNATURES = [
    ("pu_abi_version", c_int, []),
    ("pu_last_error", ctypes.c_char_p, []),
    ("pu_build_id", ctypes.c_char_p, []),
    ("pu_device_info", c_int, [c_int, ctypes.POINTER(c_int), ctypes.POINTER(c_int), ctypes.POINTER(c_ll)]),
    ("pu_conv_igemm", c_int, [ctypes.POINTER(ConvArgs), P]),
    ("pu_conv_igemm_workspace_bytes", c_size, [ctypes.POINTER(ConvArgs)]),
    ("pu_conv_igemm_tile", c_int, [ctypes.POINTER(ConvArgs), ctypes.POINTER(c_int), ctypes.POINTER(c_int),
                                   ctypes.POINTER(c_int), ctypes.POINTER(c_int)]),
    ("pu_wgrad_workspace_bytes", c_size, [ctypes.POINTER(WgradArgs)]),
    ("pu_wgrad", c_int, [ctypes.POINTER(WgradArgs), P, c_size, P]),
    ("pu_wgrad_phase", c_int, [ctypes.POINTER(WgradArgs), P, c_size, c_int, P]),
    ("pu_wgrad_tile", c_int, [ctypes.POINTER(WgradArgs), ctypes.POINTER(c_int), ctypes.POINTER(c_int),
                              ctypes.POINTER(c_int), ctypes.POINTER(c_int)]),
    ("pu_pack_weight", c_int, [P, P, c_int, c_int, c_int, c_int, c_int, c_int, c_int, P]),
    ("pu_split_weight6", c_int, [P, P, c_int, c_int, P]),
    ("pu_wino_bytes", c_size, [c_int, c_int]),
    ("pu_pack_wino", c_int, [ctypes.POINTER(WinoJob), c_int, P]),
    ("pu_nchw_to_nhwc", c_int, [P, P, c_int, c_int, c_int, c_int, P]),
    ("pu_channel_scale", c_int, [P, P, P, c_int, c_ll, c_int, P]),
    ("pu_conv_igemm_bf16", c_int, [ctypes.POINTER(ConvArgs), P]),
    ("pu_conv_igemm_bf16_workspace_bytes", c_size, [ctypes.POINTER(ConvArgs)]),
    ("pu_conv_igemm_bf16_tile", c_int, [ctypes.POINTER(ConvArgs), ctypes.POINTER(c_int), ctypes.POINTER(c_int),
                                        ctypes.POINTER(c_int), ctypes.POINTER(c_int)]),
    ("pu_wgrad_bf16_workspace_bytes", c_size, [ctypes.POINTER(WgradArgs)]),
    ("pu_wgrad_bf16", c_int, [ctypes.POINTER(WgradArgs), P, c_size, P]),
    ("pu_wgrad_bf16_phase", c_int, [ctypes.POINTER(WgradArgs), P, c_size, c_int, P]),
    ("pu_wgrad_bf16_tile", c_int, [ctypes.POINTER(WgradArgs), ctypes.POINTER(c_int), ctypes.POINTER(c_int),
                                   ctypes.POINTER(c_int), ctypes.POINTER(c_int)]),
    ("pu_pack_weight_bf16", c_int, [P, P, c_int, c_int, c_int, c_int, c_int, c_int, c_int, P]),
    ("pu_convert_f32_bf16", c_int, [P, P, c_ll, P]),
    ("pu_convert_bf16_f32", c_int, [P, P, c_ll, P]),
    ("pu_maxpool2_fwd_bf16", c_int, [P, P, c_int, c_int, c_int, c_int, P]),
    ("pu_maxpool2_bwd_bf16", c_int, [P, P, P, c_int, c_int, c_int, c_int, c_int, c_int, P]),
    ("pu_outconv_fwd_bf16", c_int, [P, P, P, P, c_ll, c_int, P]),
    ("pu_outconv_bwd_bf16", c_int, [P, P, P, P, P, P, c_ll, c_int, c_int, P, c_size, P]),
    ("pu_add_coords", c_int, [P, P, c_int, c_int, c_int, c_int, c_int, P]),
    ("pu_column_sum_workspace_bytes", c_size, [c_ll, c_int]),
    ("pu_column_sum", c_int, [P, c_ll, c_int, P, c_int, P, c_size, P]),
    ("pu_maxpool2_fwd", c_int, [P, P, c_int, c_int, c_int, c_int, P]),
    ("pu_maxpool2_bwd", c_int, [P, P, P, c_int, c_int, c_int, c_int, c_int, c_int, P]),
    ("pu_maxpool2_fwd_scaled", c_int, [P, P, P, c_int, c_int, c_int, c_int, P]),
    ("pu_maxpool2_bwd_scaled", c_int, [P, P, P, P, c_int, c_int, c_int, c_int, c_int, c_int, P]),
    ("pu_outconv_fwd", c_int, [P, P, P, P, c_ll, c_int, P]),
    ("pu_outconv_workspace_bytes", c_size, [c_ll, c_int]),
    ("pu_outconv_bwd", c_int, [P, P, P, P, P, P, c_ll, c_int, c_int, P, c_size, P]),
    ("pu_plastic_fwd", c_int, [ctypes.POINTER(PlasticArgs), P]),
    ("pu_plastic_head_fwd", c_int, [ctypes.POINTER(PlasticHeadArgs), P]),
    ("pu_trace_update", c_int, [P, P, P, P, P, c_int, c_int, c_int, P]),
    ("pu_plastic_bwd_workspace_bytes", c_size, [c_int, c_int]),
    ("pu_plastic_bwd", c_int, [ctypes.POINTER(PlasticBwdArgs), P, c_size, P]),
    ("pu_bce_workspace_bytes", c_size, [c_ll]),
    ("pu_bce_fwd", c_int, [P, P, c_ll, P, P, c_size, P]),
    ("pu_bce_bwd", c_int, [P, P, c_ll, P, P, P]),
    ("pu_bn_workspace_bytes", c_size, [c_int, c_ll, c_int]),
    ("pu_bn_fwd", c_int, [P, P, P, P, P, P, P, P, c_int, c_ll, c_int, c_float, c_float, c_int, c_int, P, P, c_size, P]),
    ("pu_bn_bwd", c_int, [P, P, P, P, P, P, P, P, c_int, c_ll, c_int, P, P, P, c_size, P]),
    ("pu_upsample_bilinear2x_fwd", c_int, [P, P, c_int, c_int, c_int, c_int, P]),
    ("pu_upsample_bilinear2x_bwd", c_int, [P, P, P, c_int, c_int, c_int, c_int, P]),
    ("pu_pack_weights", c_int, [ctypes.POINTER(PackJob), c_int, P]),
    ("pu_adam_multi", c_int, [ctypes.POINTER(AdamTensor), c_int, c_double, c_double, c_double, c_double, c_double,
                              c_double, P]),
]

_lib = None


class LibraryMissing(RuntimeError):
    pass


def load():
    """Load (once) and type the library; raise LibraryMissing if it is not built."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise LibraryMissing(
            "libplastic_unet.so not found at %s - build it with `python plastic-unet_amd/build_native.py` "
            "(the plastic U-Net path has no CPU fallback)" % LIB_PATH)
    if not os.environ.get("PU_NO_TORCH"):
        import torch  # noqa: F401  (loads the HIP runtime the library binds to, before the library)
    lib = ctypes.CDLL(LIB_PATH)
    for name, res, args in SIGNATURES:
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if lib.pu_abi_version() != ABI_VERSION:
        raise LibraryMissing("libplastic_unet.so ABI %d != %d" % (lib.pu_abi_version(), ABI_VERSION))
    _lib = lib
    return lib


def build_id():
    """Source hash the loaded library was built from (see build_native.source_hash)."""
    return load().pu_build_id().decode()


def check(rc, what=""):
    if rc != 0:
        msg = _lib.pu_last_error().decode(errors="replace") if _lib is not None else ""
        raise RuntimeError("%s failed (%d): %s" % (what or "plastic_unet call", rc, msg))
