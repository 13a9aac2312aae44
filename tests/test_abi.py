"""CPU checks of the drop-in boundary: the C-ABI library loads and exports every symbol that
include/plastic_unet.h declares, argument validation fails loudly without touching the GPU, and
the product refuses CPU tensors (no fallback)."""
import ctypes
import os
import re

import pytest
import torch

from conftest import ROOT

HEADER = os.path.join(ROOT, "include", "plastic_unet.h")


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(pu_[a-z0-9_]+)\s*\(", src)))


def test_library_exports_every_header_symbol():
    from punet import _lib
    lib = _lib.load()
    names = declared_functions()
    assert len(names) >= 20
    bound = {n for n, _, _ in _lib.SIGNATURES}
    assert set(names) == bound, set(names) ^ bound
    for n in names:
        assert getattr(lib, n) is not None
    assert lib.pu_abi_version() == _lib.ABI_VERSION == 3


def test_invalid_arguments_return_errors_without_gpu():
    from punet import _lib
    lib = _lib.load()
    a = _lib.ConvArgs()
    rc = lib.pu_conv_igemm(ctypes.byref(a), None)
    assert rc == -1
    assert b"bad grid" in lib.pu_last_error()
    w = _lib.WgradArgs()
    assert lib.pu_wgrad_workspace_bytes(ctypes.byref(w)) == 0
    assert lib.pu_trace_update(None, None, None, None, None, 1, 4, 7, None) == -1
    with pytest.raises(RuntimeError, match="pu_plastic_fwd failed"):
        _lib.check(lib.pu_plastic_fwd(ctypes.byref(_lib.PlasticArgs()), None), "pu_plastic_fwd")


def _conv(lib_mod, B, H, c, n, ws=None, ws_bytes=0):
    A = 0x10000          # 16-byte aligned stand-in pointers: planning never dereferences them
    return lib_mod.ConvArgs(B, H, H, H, H, 3, 3, 1, 1, A, c, None, 0, A, (9 * c + 15) // 16 * 16, 0, n, A,
                            A, n, None, None, None, 1, ws, ws_bytes)


def test_igemm_split_k_plan():
    """Small pixel grids split K (fills the chip), large ones do not; without scratch no split."""
    from punet import _lib
    lib = _lib.load()
    bm, bn, mode, ks = (ctypes.c_int() for _ in range(4))
    bottom = _conv(_lib, 32, 8, 512, 512)                    # C2 8x8 level: 256 tiles of 64x64
    nbytes = lib.pu_conv_igemm_workspace_bytes(ctypes.byref(bottom))
    assert nbytes > 0 and nbytes % (32 * 8 * 8 * 512 * 4) == 0
    lib.pu_conv_igemm_tile(ctypes.byref(bottom), *(ctypes.byref(v) for v in (bm, bn, mode, ks)))
    assert ks.value == 1                                     # no workspace passed -> unsplit
    with_ws = _conv(_lib, 32, 8, 512, 512, 0x20000, nbytes)
    lib.pu_conv_igemm_tile(ctypes.byref(with_ws), *(ctypes.byref(v) for v in (bm, bn, mode, ks)))
    assert ks.value == nbytes // (32 * 8 * 8 * 512 * 4) >= 2
    top = _conv(_lib, 32, 128, 64, 64)                       # 2048 tiles: no split
    assert lib.pu_conv_igemm_workspace_bytes(ctypes.byref(top)) == 0


def test_header_structs_match_ctypes_layout():
    """Field order/size of the ctypes mirrors (a mismatch would corrupt every launch)."""
    from punet import _lib
    src = open(HEADER).read()
    for cname, py in [("pu_conv_args", _lib.ConvArgs), ("pu_wgrad_args", _lib.WgradArgs),
                      ("pu_plastic_args", _lib.PlasticArgs), ("pu_plastic_bwd_args", _lib.PlasticBwdArgs),
                      ("pu_plastic_head_args", _lib.PlasticHeadArgs),
                      ("pu_adam_tensor", _lib.AdamTensor), ("pu_pack_job", _lib.PackJob),
                      ("pu_wino_job", _lib.WinoJob)]:
        body = dict((n, b) for b, n in re.findall(r"typedef struct \{([^}]*)\}\s*(\w+);", src))[cname]
        body = re.sub(r"/\*.*?\*/", "", body, flags=re.S)
        fields = []
        for decl in body.split(";"):
            decl = decl.strip()
            if not decl:
                continue
            decl = re.sub(r"\bconst\b", "", decl)
            for part in decl.split(","):
                fields.append(re.sub(r"[\*\s]", " ", part).split()[-1])
        assert fields == [f for f, _ in py._fields_], (cname, fields)


def test_product_refuses_cpu_tensors():
    from unet import UNetp
    net = UNetp(1, 1, torch.device("cpu"), nbf=32)
    with pytest.raises(RuntimeError, match="ROCm device"):
        net(torch.zeros(1, 1, 32, 32), torch.zeros(32, 32))


def test_reference_batch_rule_kept():
    from unet import UNetp
    net = UNetp(1, 1, torch.device("cpu"), nbf=32)
    with pytest.raises(ValueError, match="Only batch size: 1 is supported, but was: 2"):
        net(torch.zeros(2, 1, 32, 32), torch.zeros(32, 32))


def test_state_dict_and_init_match_reference_keys():
    import oracle
    from unet import UNetp, UNetpRes
    torch.manual_seed(0)
    a = UNetp(1, 1, torch.device("cpu"), rule="oja", nbf=64)
    torch.manual_seed(0)
    b = oracle.RefUNetp(1, 1, rule="oja", nbf=64)
    sa, sb = a.state_dict(), b.state_dict()
    assert list(sa) == list(sb)
    assert all(torch.equal(sa[k], sb[k]) for k in sa)
    torch.manual_seed(5)
    a = UNetpRes(1, 1, torch.device("cpu"), neurons=4, nbf=101)
    torch.manual_seed(5)
    b = oracle.RefUNetpRes(1, 1, neurons=4, nbf=101)
    assert list(a.state_dict()) == list(b.state_dict())
    assert all(torch.equal(a.state_dict()[k], b.state_dict()[k]) for k in a.state_dict())


def test_trunk_parameter_order_covers_every_trunk_parameter():
    from unet import UNetp
    from punet.trunk import UNetpTrunk
    for depth, base in [(5, 8), (4, 16), (5, 64)]:
        m = UNetp(1, 1, torch.device("cpu"), depth=depth, base_ch=base, nbf=64)
        t = UNetpTrunk(m)
        trunk = {id(p) for p in t.params}
        head = {id(m.w), id(m.alpha), id(m.eta)}
        assert trunk | head == {id(p) for p in m.parameters()}
        assert len(t.params) == 4 * depth + 6 * (depth - 1) + 2


def test_wino_plan_reported_and_split_k():
    """pu_conv_igemm_tile reports mode 6 for a Winograd layer, and the 8x8 level splits K."""
    from punet import _lib
    L = _lib.load()
    A = 0x10000

    def args(B, H, c, n, wino, ws=None, ws_bytes=0):
        a = _lib.ConvArgs(B, H, H, H, H, 3, 3, 1, 1, A, c, None, 0, A, 9 * c, 32, n, A, A, n, None, None, None, 1,
                          ws, ws_bytes)
        a.weight6 = A
        a.wino = A if wino else None
        return a
    bm, bn, mode, ks = (ctypes.c_int() for _ in range(4))
    top = args(32, 128, 64, 64, True)
    L.pu_conv_igemm_tile(ctypes.byref(top), *(ctypes.byref(v) for v in (bm, bn, mode, ks)))
    assert (mode.value, ks.value) == (6, 1)
    assert L.pu_conv_igemm_workspace_bytes(ctypes.byref(top)) == 0
    bottom = args(32, 8, 1024, 1024, True)
    nbytes = L.pu_conv_igemm_workspace_bytes(ctypes.byref(bottom))
    assert nbytes > 0
    bottom = args(32, 8, 1024, 1024, True, 0x20000, nbytes)
    L.pu_conv_igemm_tile(ctypes.byref(bottom), *(ctypes.byref(v) for v in (bm, bn, mode, ks)))
    assert mode.value == 6 and ks.value >= 2
    direct = args(32, 128, 64, 64, False)
    L.pu_conv_igemm_tile(ctypes.byref(direct), *(ctypes.byref(v) for v in (bm, bn, mode, ks)))
    assert mode.value == 4


def test_wgrad_dispatch_plan_takes_winograd_on_c2_layers():
    """Planning only (no GPU): the C2 3x3 weight gradients (64-channel blocks, even grids) take the
    Winograd-domain kernel (kind 5), the 8/16-channel and odd-grid ones do not; the workspace is
    the slab of one 512-thread block per CU."""
    from punet import kernels as K
    for (B, H, c0, c1, n) in [(32, 128, 64, 0, 64), (32, 128, 64, 64, 64), (32, 64, 128, 0, 128),
                              (32, 32, 256, 256, 128), (32, 16, 512, 0, 512), (32, 8, 512, 0, 512)]:
        assert K.wgrad_kind(batch=B, hw=(H, H), n=n, c0=c0, c1=c1) == 5, (H, c0, c1, n)
    assert K.wgrad_kind(batch=4, hw=(101, 101), n=64, c0=64) != 5       # odd grid
    assert K.wgrad_kind(batch=4, hw=(64, 64), n=32, c0=32) != 5         # 32-channel layer
    assert K.wgrad_kind(batch=4, hw=(64, 64), n=8, c0=8) == 2            # small-channel direct
    for n in (8, 16, 32, 64):                                            # single-channel stem
        assert K.wgrad_kind(batch=4, hw=(64, 64), n=n, c0=1) == 4, n
    # C4's CoordConv 1x1 (4 -> 8 channels at 256^2) takes the pointwise kernel; a 64-channel 1x1 not
    assert K.wgrad_kind(batch=32, hw=(256, 256), n=8, c0=4, k=1) == 6
    assert K.wgrad_kind(batch=2, hw=(24, 40), n=16, c0=3, k=1) == 6
    assert K.wgrad_kind(batch=2, hw=(24, 40), n=64, c0=64, k=1) != 6
