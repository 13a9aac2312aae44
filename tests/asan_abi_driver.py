"""Run by tests/test_sanitizers.py in a torch-free interpreter with the clang ASan runtime
preloaded and PLASTIC_UNET_LIB = lib/libplastic_unet_asan_host.so (host code only, no device code):
exercises every host path of the C-ABI that needs no GPU - argument validation of every entry
point, the planning / workspace queries over the BASELINE configurations' layer shapes - so
AddressSanitizer sees the boundary's host code.  Exit 0 = no ASan report."""
import ctypes
import importlib.util
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
spec = importlib.util.spec_from_file_location("pu_lib", os.path.join(os.path.dirname(HERE), "plastic-unet_amd",
                                                                      "punet", "_lib.py"))
L = importlib.util.module_from_spec(spec)
spec.loader.exec_module(L)
lib = L.load()
assert lib.pu_abi_version() == L.ABI_VERSION
assert len(lib.pu_build_id()) == 16

A = 0x10000  # 16-byte aligned stand-in device pointers: nothing here dereferences them
calls = 0


def expect_fail(rc):
    global calls
    calls += 1
    assert rc < 0, rc
    assert len(lib.pu_last_error()) > 0


# every structured entry point with empty / inconsistent arguments
expect_fail(lib.pu_conv_igemm(ctypes.byref(L.ConvArgs()), None))
expect_fail(lib.pu_conv_igemm_bf16(ctypes.byref(L.ConvArgs()), None))
expect_fail(lib.pu_wgrad(ctypes.byref(L.WgradArgs()), None, 0, None))
expect_fail(lib.pu_wgrad_bf16(ctypes.byref(L.WgradArgs()), None, 0, None))
expect_fail(lib.pu_plastic_fwd(ctypes.byref(L.PlasticArgs()), None))
expect_fail(lib.pu_plastic_head_fwd(ctypes.byref(L.PlasticHeadArgs()), None))
expect_fail(lib.pu_plastic_bwd(ctypes.byref(L.PlasticBwdArgs()), None, 0, None))
expect_fail(lib.pu_trace_update(None, None, None, None, None, 1, 4, 7, None))
expect_fail(lib.pu_bce_fwd(None, None, 0, None, None, 0, None))
expect_fail(lib.pu_adam_multi(None, 1, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0, None))
bad = (L.AdamTensor * 3)(L.AdamTensor(A, A, A, A, 10), L.AdamTensor(A, None, A, A, 10), L.AdamTensor())
expect_fail(lib.pu_adam_multi(bad, 3, 1e-3, 0.9, 0.999, 1e-8, 0.0, 1.0, None))
expect_fail(lib.pu_pack_weights(None, 1, None))
jobs = (L.PackJob * 3)(L.PackJob(A, A, None, A, 0, 64, 64, 3, 3, 576, 32),    # valid
                       L.PackJob(A, A, None, None, 7, 64, 64, 3, 3, 576, 0),    # bad mode
                       L.PackJob(A, None, None, None, 0, 64, 64, 3, 3, 576, 0)) # no output
expect_fail(lib.pu_pack_weights(jobs, 3, None))
jobs = (L.PackJob * 1)(L.PackJob(A, A + 4, None, None, 0, 64, 64, 3, 3, 576, 0))   # misaligned output
expect_fail(lib.pu_pack_weights(jobs, 1, None))
jobs = (L.PackJob * 1)(L.PackJob(A, A, None, A, 0, 64, 64, 3, 3, 568, 0))       # k_pad < 9 * 64
expect_fail(lib.pu_pack_weights(jobs, 1, None))
h = L.PlasticHeadArgs(2, 100, 64, A, 0, A, A, A, A, A, A, A, A, A, 1)          # nbf not a multiple of 16
expect_fail(lib.pu_plastic_head_fwd(ctypes.byref(h), None))
h = L.PlasticHeadArgs(2, 128, 64, A, 0, A, A, A, A, A, A, A, A, A, 1)          # hebb_out aliasing hebb
expect_fail(lib.pu_plastic_head_fwd(ctypes.byref(h), None))

# planning queries over the trunks' layer shapes (C2/C3 base 64, C4 base 8 at 256, C5 n8 at 512)
shapes = []
for S, chans in ((128, [64, 128, 256, 512, 512]), (256, [8, 16, 32, 64, 128]), (512, [8, 16, 32, 64, 128])):
    for lvl, c in enumerate(chans):
        h = S >> lvl
        for B in (1, 2, 16, 32):
            shapes += [(B, h, c, 0, c), (B, h, c, c, c), (B, h, c, 0, 2 * c), (B, h, 2 * c, 0, c)]
for B, H, c0, c1, n in shapes:
    kp = (9 * (c0 + c1) + 15) // 16 * 16
    for cg in (0, 16, 32):
        if cg and (c0 % cg or c1 % cg):
            continue
        a = L.ConvArgs(B, H, H, H, H, 3, 3, 1, 1, A, c0, A if c1 else None, c1, A, kp, cg, n, A, A, n, None, None,
                       None, 1, None, 0, None, 0, 0, 0, A)
        ws = lib.pu_conv_igemm_workspace_bytes(ctypes.byref(a))
        bm, bn, mode, ks = (ctypes.c_int() for _ in range(4))
        assert lib.pu_conv_igemm_tile(ctypes.byref(a), *(ctypes.byref(v) for v in (bm, bn, mode, ks))) == 0
        assert bm.value > 0 and bn.value > 0 and ws >= 0
        calls += 2
    w = L.WgradArgs(B, H, H, H, H, 3, 3, 1, 1, A, n, A, c0, A if c1 else None, c1, 1, A, A, 0, 1)
    ws = lib.pu_wgrad_workspace_bytes(ctypes.byref(w))
    bn, bk, qv, sp = (ctypes.c_int() for _ in range(4))
    assert lib.pu_wgrad_tile(ctypes.byref(w), *(ctypes.byref(v) for v in (bn, bk, qv, sp))) == 0
    assert ws > 0 and sp.value >= 1
    calls += 2
assert lib.pu_plastic_bwd_workspace_bytes(32, 128) == 32 * 2 * 128 * 128 * 4
print("asan host ABI driver: %d calls, %d shapes, no sanitizer report" % (calls, len(shapes)))
