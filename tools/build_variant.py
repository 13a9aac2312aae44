"""Build a timing-only variant library in seconds: ONE source recompiled with extra defines, linked
with the release objects of the others (build_native.build() recompiles every source per variant).

    python tools/build_variant.py <tag> <source.hip> DEF=1 [DEF2=0 ...]
    -> plastic-unet_amd/lib/libplastic_unet_<tag>.so (load with PLASTIC_UNET_LIB=...)
"""
import glob
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "plastic-unet_amd"))
import build_native as bn  # noqa: E402


def main():
    tag, src = sys.argv[1], sys.argv[2]
    defines = tuple(sys.argv[3:])
    bn.build(verbose=False)                      # release objects up to date
    srcp = os.path.join(bn.CSRC, src)
    obj, err = bn._compile(srcp, True, defines, "." + tag)
    if err:
        sys.exit(err)
    objs = [o for o in sorted(glob.glob(os.path.join(bn.BUILD, "*.hip.o"))) if os.path.basename(o) != src + ".o"]
    bid = bn.source_hash(defines)
    objs += [obj, bn._build_id_object(bid, "." + tag)]
    out = os.path.join(bn.LIBDIR, "libplastic_unet_%s.so" % tag)
    r = subprocess.run([bn.HIPCC, "-shared", "-fPIC", "--offload-arch=" + bn.ARCH, "-o", out] + objs,
                       capture_output=True, text=True)
    if r.returncode:
        sys.exit(r.stderr)
    print("built", out, defines)


if __name__ == "__main__":
    main()
