"""SURVEY 5 sanitizer / debug builds.

* host AddressSanitizer (CPU, no GPU): build_native's asan_host variant - the host half of every
  source compiled with -fsanitize=address (-Xarch_host) - loaded into a torch-free
  interpreter with the clang ASan runtime preloaded; tests/asan_abi_driver.py drives every entry
  point's validation and the planning / workspace queries over the configurations' layer shapes.
* PU_DEBUG (GPU): the debug variant synchronises after every launch; a short training step of the
  C2 topology at small size runs through it and must match the release library bit for bit."""
import os
import subprocess
import sys

import pytest

from conftest import ROOT, PKG

sys.path.insert(0, PKG)


def test_host_abi_under_address_sanitizer():
    import build_native
    if not build_native.ASAN_RT:
        pytest.skip("clang ASan runtime not found under /opt/rocm/lib/llvm")
    lib = build_native.build_variant("asan_host", verbose=False)
    env = dict(os.environ, PLASTIC_UNET_LIB=lib, PU_NO_TORCH="1", LD_PRELOAD=build_native.ASAN_RT[-1],
               ASAN_OPTIONS="detect_leaks=0:abort_on_error=0:halt_on_error=1")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tests", "asan_abi_driver.py")], env=env,
                       capture_output=True, text=True, timeout=300)
    assert "AddressSanitizer" not in r.stderr, r.stderr[-4000:]
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-4000:])
    assert "no sanitizer report" in r.stdout


_STEP = r"""
import os, sys, json
sys.path.insert(0, %r)
import torch
from unet import UNetp
from punet import bce_loss, _lib
dev = torch.device("cuda")
torch.manual_seed(0)
net = UNetp(1, 1, dev, rule="oja", nbf=64, depth=4, base_ch=32)
g = torch.Generator().manual_seed(1)
x = torch.rand(3, 1, 64, 64, generator=g).to(dev)
t = (torch.rand(3, 64, 64, generator=g) > 0.5).float().to(dev)
H = (0.05 * torch.randn(3, 64, 64, generator=g)).to(dev)
y, hn = net(x, H)
bce_loss(y, t).backward()
torch.cuda.synchronize()
out = {"lib": os.path.basename(_lib.LIB_PATH), "bid": _lib.build_id(), "y": y.double().sum().item(),
       "h": hn.double().sum().item()}
out.update({k: p.grad.double().abs().sum().item() for k, p in net.named_parameters() if p.grad is not None})
print("RESULT " + json.dumps(out))
"""


def _run_step(lib):
    env = dict(os.environ, PLASTIC_UNET_LIB=lib)
    r = subprocess.run([sys.executable, "-c", _STEP % PKG], env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    import json
    return json.loads([l for l in r.stdout.splitlines() if l.startswith("RESULT ")][-1][7:])


@pytest.mark.gpu
def test_pu_debug_library_matches_release():
    """A fwd + bwd of UNetp (depth 4, base 32) through lib/libplastic_unet_debug.so (PU_DEBUG:
    synchronous fault reporting after every launch) gives the release library's results bit for
    bit (the same kernels, only the host-side checks differ)."""
    dbg = os.path.join(PKG, "lib", "libplastic_unet_debug.so")
    rel = os.path.join(PKG, "lib", "libplastic_unet.so")
    if not os.path.exists(dbg):
        pytest.fail("debug library missing: build it with build_native.py --variant debug (build() does)")
    import build_native
    a, b = _run_step(rel), _run_step(dbg)
    assert a["lib"] == "libplastic_unet.so" and b["lib"] == "libplastic_unet_debug.so"
    # both libraries must be builds of THIS tree's sources: a stale variant (built before the last
    # source change) would compare different kernels and fail for the wrong reason (round 4 r04b)
    want_rel, want_dbg = build_native.source_hash(), build_native.source_hash(("PU_DEBUG=1",))
    assert a["bid"] == want_rel, "release library is stale (build id %s, sources %s): rebuild" % (a["bid"], want_rel)
    assert b["bid"] == want_dbg, ("debug library is stale (build id %s, sources %s): "
                                  "build_native.py --variant debug" % (b["bid"], want_dbg))
    for r in (a, b):
        r.pop("lib"), r.pop("bid")
    assert a == b
