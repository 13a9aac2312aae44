"""Build libplastic_unet.so (gfx950) in-tree with hipcc.

    python plastic-unet_amd/build_native.py [--force] [--jobs N] [--variant debug|asan_host]

Objects go to plastic-unet_amd/build/, the library to plastic-unet_amd/lib/libplastic_unet.so
(both git-ignored; the .so travels to the GPU box with the repo snapshot).

Variants (sanitizers / debug):
  debug      lib/libplastic_unet_debug.so: -DPU_DEBUG (every entry point synchronises after its
             launches and reports asynchronous faults as its own error), -O2 -g
  asan_host  lib/libplastic_unet_asan_host.so: the HOST half of every source (argument checks,
             planning, workspace sizing, the C-ABI) with AddressSanitizer (-Xarch_host only: GPU
             ASan is not available on this pool), device code at -O1 - for CPU tests of the
             boundary under LD_PRELOAD of the clang ASan runtime
"""
import argparse
import concurrent.futures as cf
import glob
import hashlib
import json
import os
import re
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
BUILD = os.path.join(HERE, "build")
LIBDIR = os.path.join(HERE, "lib")
LIB = os.path.join(LIBDIR, "libplastic_unet.so")
RESOURCES = os.path.join(BUILD, "resource_usage.json")
INCLUDE = os.path.join(ROOT, "include")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = "gfx950"

CFLAGS = ["-O3", "-std=c++17", "-fPIC", "--offload-arch=" + ARCH, "-I" + INCLUDE, "-I" + CSRC,
          "-Wall", "-Wno-unused-function", "-Wno-unused-variable", "-Wno-unused-but-set-variable",
          "-Wno-unused-result"]
# per-kernel register / scratch report of every compile (kept next to the object, parsed into
# build/resource_usage.json; tests/test_resources.py fails on any scratch use or spill)
RPASS = "-Rpass-analysis=kernel-resource-usage"


def _newer(src_list, target):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(s) > t for s in src_list)


def _compile(src, force, defines=(), tag=""):
    obj = os.path.join(BUILD, os.path.basename(src) + tag + ".o")
    deps = [src] + glob.glob(os.path.join(CSRC, "*.h")) + [os.path.join(INCLUDE, "plastic_unet.h")]
    if not force and not _newer(deps, obj) and os.path.exists(obj + ".resources.txt"):
        return obj, None
    # an entry starting with '-' is passed as a raw compiler flag (ablation variants)
    cmd = [HIPCC] + CFLAGS + [RPASS] + [d if d.startswith("-") else "-D" + d for d in defines] + ["-c", src, "-o", obj]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        return obj, "%s\n%s\n%s" % (" ".join(cmd), r.stdout, r.stderr)
    with open(obj + ".resources.txt", "w") as f:
        f.write(r.stderr)
    return obj, None


_FIELDS = {"VGPRs": "vgpr", "AGPRs": "agpr", "TotalSGPRs": "sgpr", "ScratchSize [bytes/lane]": "scratch",
           "Occupancy [waves/SIMD]": "occupancy", "SGPRs Spill": "sgpr_spill", "VGPRs Spill": "vgpr_spill",
           "LDS Size [bytes/block]": "lds"}


def parse_resources(text):
    """{mangled kernel name: {vgpr, agpr, sgpr, scratch, occupancy, sgpr_spill, vgpr_spill, lds}}
    from hipcc's -Rpass-analysis=kernel-resource-usage remarks."""
    out, cur = {}, None
    for line in text.splitlines():
        m = re.search(r"remark:\s+Function Name: (\S+)", line)
        if m:
            cur = out.setdefault(m.group(1), {})
            continue
        m = re.search(r"remark:\s+([^:]+): (\S+) \[-Rpass-analysis", line)
        if m and cur is not None and m.group(1).strip() in _FIELDS:
            v = m.group(2)
            cur[_FIELDS[m.group(1).strip()]] = int(v) if v.lstrip("-").isdigit() else v
    return out


def source_hash(defines=()):
    """Build id: sha256 over every library source, the public header and the compile flags."""
    h = hashlib.sha256()
    files = sorted(glob.glob(os.path.join(CSRC, "*.hip")) + glob.glob(os.path.join(CSRC, "*.h")))
    for f in files + [os.path.join(INCLUDE, "plastic_unet.h")]:
        h.update(os.path.basename(f).encode())
        with open(f, "rb") as fh:
            h.update(fh.read())
    # flags with this checkout's absolute paths made relative: the id depends on content only
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    h.update(" ".join(CFLAGS + list(defines)).replace(root, "<root>").encode())
    return h.hexdigest()[:16]


def _build_id_object(bid, tag):
    """build/build_id<tag>.o exporting pu_build_id() -> the source hash (rewritten when it changes)."""
    src = os.path.join(BUILD, "build_id%s.cpp" % tag)
    obj = src[:-4] + ".o"
    text = 'extern "C" const char* pu_build_id(void) { return "%s"; }\n' % bid
    if not (os.path.exists(src) and open(src).read() == text and os.path.exists(obj)):
        with open(src, "w") as f:
            f.write(text)
        r = subprocess.run(["g++", "-O2", "-fPIC", "-c", src, "-o", obj], capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError("build id: %s" % r.stderr)
    return obj


def build(force=False, jobs=None, verbose=True, defines=(), lib=None):
    """defines/lib: build an experimental variant (e.g. ablations) into another .so"""
    os.makedirs(BUILD, exist_ok=True)
    os.makedirs(LIBDIR, exist_ok=True)
    srcs = sorted(glob.glob(os.path.join(CSRC, "*.hip")))
    jobs = jobs or min(8, len(srcs))
    tag = ("." + "_".join(d.replace("=", "") for d in defines)) if defines else ""
    target = lib or LIB
    objs, errors = [], []
    with cf.ThreadPoolExecutor(jobs) as ex:
        for obj, err in ex.map(lambda s: _compile(s, force, defines, tag), srcs):
            objs.append(obj)
            if err:
                errors.append(err)
    if errors:
        raise RuntimeError("hipcc failed:\n" + "\n".join(errors))
    bid = source_hash(defines)
    objs.append(_build_id_object(bid, tag))
    if not defines:
        usage = {}
        for o in objs[:-1]:
            rep = o + ".resources.txt"
            if os.path.exists(rep):
                for k, v in parse_resources(open(rep).read()).items():
                    v["source"] = os.path.basename(o).split(".hip")[0] + ".hip"
                    usage[k] = v
        with open(RESOURCES, "w") as f:
            json.dump({"build_id": bid, "kernels": usage}, f, indent=1, sort_keys=True)
    if force or _newer(objs, target):
        cmd = [HIPCC, "-shared", "-fPIC", "--offload-arch=" + ARCH, "-o", target] + objs
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError("link failed:\n%s\n%s" % (r.stdout, r.stderr))
    if verbose:
        print("built", target, "build id", bid)
    return target


ASAN_RT = sorted(glob.glob("/opt/rocm/lib/llvm/lib/clang/*/lib/linux/libclang_rt.asan-x86_64.so"))


def build_variant(kind, verbose=True):
    """Build a sanitizer / debug variant library (see the module docstring); returns its path."""
    os.makedirs(BUILD, exist_ok=True)
    os.makedirs(LIBDIR, exist_ok=True)
    srcs = sorted(glob.glob(os.path.join(CSRC, "*.hip")))
    if kind == "debug":
        return build(defines=("PU_DEBUG=1",), lib=os.path.join(LIBDIR, "libplastic_unet_debug.so"), verbose=verbose)
    if kind != "asan_host":
        raise ValueError("variant must be 'debug' or 'asan_host'")
    target = os.path.join(LIBDIR, "libplastic_unet_asan_host.so")
    flags = ["-O1", "-std=c++17", "-fPIC", "--offload-arch=" + ARCH, "-I" + INCLUDE,
             "-I" + CSRC, "-Xarch_host", "-fsanitize=address", "-Xarch_host", "-fno-omit-frame-pointer"]

    def one(src):
        obj = os.path.join(BUILD, os.path.basename(src) + ".asan_host.o")
        deps = [src] + glob.glob(os.path.join(CSRC, "*.h")) + [os.path.join(INCLUDE, "plastic_unet.h")]
        if _newer(deps, obj):
            r = subprocess.run([HIPCC] + flags + ["-c", src, "-o", obj], capture_output=True, text=True)
            if r.returncode != 0:
                raise RuntimeError("asan_host compile failed: %s\n%s" % (src, r.stderr))
        return obj
    with cf.ThreadPoolExecutor(min(8, len(srcs))) as ex:
        objs = list(ex.map(one, srcs))
    objs.append(_build_id_object(source_hash(("asan_host",)), ".asan_host"))
    if _newer(objs, target):
        r = subprocess.run([HIPCC, "-shared", "-fPIC", "--offload-arch=" + ARCH, "-fsanitize=address", "-o", target] + objs,
                           capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError("asan_host link failed:\n%s" % r.stderr)
    if verbose:
        print("built", target)
    return target


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--jobs", type=int, default=None)
    ap.add_argument("-D", dest="defines", action="append", default=[])
    ap.add_argument("--lib", default=None)
    ap.add_argument("--variant", default=None, choices=["debug", "asan_host"])
    a = ap.parse_args()
    try:
        if a.variant:
            build_variant(a.variant)
        else:
            build(a.force, a.jobs, defines=a.defines, lib=a.lib)
    except RuntimeError as e:
        print(e, file=sys.stderr)
        sys.exit(1)
