"""Experiment helper: link libhlgs.so variants that differ in one source file.

    python tools/build_variant.py NAME path/to/variant_of_raster_bwd.hip [csrc file it replaces]
-> hierarchical-lod-gaussians_amd/lib/variants/NAME.so (load it with HLGS_LIBRARY=...)."""
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "hierarchical-lod-gaussians_amd")
sys.path.insert(0, os.path.join(PKG, "hlgs_core"))
import build as B  # noqa: E402


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
    out = os.path.join(PKG, "lib", "variants", name + ".so")
    os.makedirs(os.path.dirname(out), exist_ok=True)
    subprocess.run([B.HIPCC, "-shared", f"--offload-arch={B.ARCH}", "-o", out] + objs, check=True)
    print(out)


if __name__ == "__main__":
    main(*sys.argv[1:])
