"""CPU gate on the compiled kernels (no GPU): every kernel of libplastic_unet.so must be free of
scratch memory and VGPR spills.

build_native.py compiles each csrc/*.hip with -Rpass-analysis=kernel-resource-usage and writes the
per-kernel report to build/resource_usage.json.  A spill turns a register-resident accumulator
tile into scratch traffic: round 1's halo weight gradient went from 110 VGPR + 144 AGPR to 256 VGPR
with 125 spilled and ran 3.6x slower while still passing parity - this test is what catches that."""
import json
import os
import sys

from conftest import ROOT

sys.path.insert(0, os.path.join(ROOT, "plastic-unet_amd"))


def _usage():
    import build_native
    build_native.build(verbose=False)       # no-op when the objects are current
    d = json.load(open(build_native.RESOURCES))
    assert d["build_id"] == build_native.source_hash()
    return d["kernels"]


def test_no_kernel_uses_scratch_or_spills_vgprs():
    k = _usage()
    assert len(k) >= 50, "resource report incomplete: %d kernels" % len(k)
    bad = {n: v for n, v in k.items() if v.get("scratch", 0) or v.get("vgpr_spill", 0)}
    assert not bad, "kernels with scratch / VGPR spills:\n" + "\n".join("%s %s" % kv for kv in bad.items())


def test_hot_kernels_keep_their_register_budget():
    """The dominant fp32 kernels keep accumulators in AGPRs and stay at 2 waves per SIMD."""
    k = _usage()
    halo = [v for n, v in k.items() if "wgrad_halo_x6_kernel" in n]
    assert halo, "wgrad_halo_x6_kernel missing"
    for v in halo:
        assert v["occupancy"] >= 2 and v["vgpr"] + v["agpr"] <= 256, v
    lean = [v for n, v in k.items() if "igemm_x6_lean_kernel" in n]
    assert lean and all(v["occupancy"] >= 2 for v in lean), lean


def test_library_reports_its_build_id():
    import build_native
    from punet import _lib
    assert _lib.build_id() == build_native.source_hash()
