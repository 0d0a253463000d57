"""Experiment helper: link libhlgs.so variants.

    python tools/build_variant.py NAME path/to/variant_of_raster_bwd.hip [csrc file it replaces]
    python tools/build_variant.py NAME --defs "-DHLGS_BWD_WAVES=6 -DHLGS_BWD_CHUNK=64"   (every source rebuilt)
-> hierarchical-lod-gaussians_amd/lib/variants/NAME.so (load it with HLGS_LIBRARY=...)."""
import concurrent.futures as cf
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "hierarchical-lod-gaussians_amd")
sys.path.insert(0, os.path.join(PKG, "hlgs_core"))
import build as B  # noqa: E402


def _link(name, objs):
    out = os.path.join(PKG, "lib", "variants", name + ".so")
    os.makedirs(os.path.dirname(out), exist_ok=True)
    subprocess.run([B.HIPCC, "-shared", f"--offload-arch={B.ARCH}", "-o", out] + objs, check=True)
    print(out)


def with_defs(name, defs):
    csrc = os.path.join(PKG, "csrc")
    odir = os.path.join(PKG, "build", "var", name)
    os.makedirs(odir, exist_ok=True)

    def one(src):
        obj = os.path.join(odir, os.path.splitext(src)[0] + ".o")
        subprocess.run([B.HIPCC] + B.FLAGS + B.PER_FILE.get(src, []) + defs + ["-c", os.path.join(csrc, src), "-o", obj],
                       check=True)
        return obj
    with cf.ThreadPoolExecutor(max_workers=8) as ex:
        objs = list(ex.map(one, B.SOURCES))
    _link(name, objs)


def main(name, variant, replaces="raster_bwd.hip"):
    B.build()
    csrc = os.path.join(PKG, "csrc")
    tmp = os.path.join(csrc, f"_variant_{name}.hip")
    shutil.copy(variant, tmp)
    try:
        obj = os.path.join(PKG, "build", "var", name + ".o")
        os.makedirs(os.path.dirname(obj), exist_ok=True)
        subprocess.run([B.HIPCC] + B.FLAGS + B.PER_FILE.get(replaces, []) + ["-c", tmp, "-o", obj], check=True)
    finally:
        os.remove(tmp)
    objs = [os.path.join(B.OBJDIR, os.path.splitext(s)[0] + ".o") for s in B.SOURCES if s != replaces] + [obj]
    _link(name, objs)


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[2] == "--defs":
        with_defs(sys.argv[1], sys.argv[3].split())
    else:
        main(*sys.argv[1:])
