"""Build libplastic_unet.so (gfx950) in-tree with hipcc.

    python plastic-unet_amd/build_native.py [--force] [--jobs N]

Objects go to plastic-unet_amd/build/, the library to plastic-unet_amd/lib/libplastic_unet.so
(both git-ignored; the .so travels to the GPU box with the repo snapshot).
"""
import argparse
import concurrent.futures as cf
import glob
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
BUILD = os.path.join(HERE, "build")
LIBDIR = os.path.join(HERE, "lib")
LIB = os.path.join(LIBDIR, "libplastic_unet.so")
INCLUDE = os.path.join(ROOT, "include")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = "gfx950"

CFLAGS = ["-O3", "-std=c++17", "-fPIC", "--offload-arch=" + ARCH, "-I" + INCLUDE, "-I" + CSRC,
          "-Wall", "-Wno-unused-function", "-Wno-unused-variable", "-Wno-unused-but-set-variable",
          "-Wno-unused-result"]


def _newer(src_list, target):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(s) > t for s in src_list)


def _compile(src, force, defines=(), tag=""):
    obj = os.path.join(BUILD, os.path.basename(src) + tag + ".o")
    deps = [src] + glob.glob(os.path.join(CSRC, "*.h")) + [os.path.join(INCLUDE, "plastic_unet.h")]
    if not force and not _newer(deps, obj):
        return obj, None
    cmd = [HIPCC] + CFLAGS + ["-D" + d for d in defines] + ["-c", src, "-o", obj]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        return obj, "%s\n%s\n%s" % (" ".join(cmd), r.stdout, r.stderr)
    return obj, None


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
    if force or _newer(objs, target):
        cmd = [HIPCC, "-shared", "-fPIC", "--offload-arch=" + ARCH, "-o", target] + objs
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError("link failed:\n%s\n%s" % (r.stdout, r.stderr))
    if verbose:
        print("built", target)
    return target


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--jobs", type=int, default=None)
    ap.add_argument("-D", dest="defines", action="append", default=[])
    ap.add_argument("--lib", default=None)
    a = ap.parse_args()
    try:
        build(a.force, a.jobs, defines=a.defines, lib=a.lib)
    except RuntimeError as e:
        print(e, file=sys.stderr)
        sys.exit(1)
