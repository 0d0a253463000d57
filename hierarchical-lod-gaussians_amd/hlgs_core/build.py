"""Build libhlgs.so (gfx950) in-tree with hipcc.  No torch headers, no JIT cache: the .so lands in
hierarchical-lod-gaussians_amd/lib/ and travels with the repository snapshot to the GPU box."""
import concurrent.futures as cf
import os
import subprocess
import sys

PKG = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(PKG, "csrc")
LIBDIR = os.path.join(PKG, "lib")
OBJDIR = os.path.join(PKG, "build", "obj")
LIB = os.path.join(LIBDIR, "libhlgs.so")
SOURCES = ["scan.hip", "preprocess.hip", "raster_fwd.hip", "raster_bwd.hip", "gauss_bwd.hip", "lod.hip", "optim.hip", "act.hip", "loss.hip", "stream.hip", "capi.hip", "hier_io.cpp", "spt_build.cpp"]
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("HLGS_ARCH", "gfx950")
FLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-munsafe-fp-atomics", "-fno-slp-vectorize", "-Wall",
         "-Wno-unused-function", "-Wno-unused-variable", "-Wno-unused-but-set-variable"]


def _deps_mtime():
    files = [os.path.join(CSRC, f) for f in os.listdir(CSRC)] + [os.path.join(PKG, "..", "include", "hlgs.h"),
                                                                os.path.abspath(__file__)]  # flags live here
    return max(os.path.getmtime(f) for f in files if os.path.exists(f))


# preprocess.hip, raster_fwd.hip: no a*b+c contraction, so the preprocess (and the key scatter's quadrant masks) round every product and sum as the oracle
# does (-ffp-contract=off there) and its per-Gaussian outputs are bit-identical; the blend's hot
# arithmetic is written with explicit fmaf and is unaffected.
# lod.hip: the same for the LOD sizes (distance, max scale / distance) and interpolation weights, which the
# oracle computes uncontracted: cut decisions and weights are then bit-identical, not only within rounding.
# gauss_bwd.hip: the per-Gaussian backward, likewise (its conic -> cov3D chain is ill-conditioned for wide splats).
PER_FILE = {"preprocess.hip": ["-ffp-contract=off"], "raster_fwd.hip": ["-ffp-contract=off"], "lod.hip": ["-ffp-contract=off"],
            "gauss_bwd.hip": ["-ffp-contract=off"]}


def _compile(src, extra):
    obj = os.path.join(OBJDIR, os.path.splitext(src)[0] + ".o")
    cmd = [HIPCC] + FLAGS + PER_FILE.get(src, []) + extra + ["-c", os.path.join(CSRC, src), "-o", obj]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for {src}:\n{' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    return obj


def variant_switches():
    """Compile-time switches in the product sources (`#if[n]def HLGS_...` / `#if HLGS_...`): there are none.  Measured
    variants live outside the product source (patches under tools/variants/ or git history, built by tools/build_variant.py), so libhlgs.so is
    exactly the tested configuration and no diagnostic or parity-breaking path can be compiled into it."""
    import re
    pat = re.compile(r"^\s*#\s*(ifdef|ifndef|if|elif)\b.*\bHLGS_", re.M)
    hits = []
    for f in sorted(os.listdir(CSRC)):
        for m in pat.finditer(open(os.path.join(CSRC, f)).read()):
            hits.append(f"{f}: {m.group(0).strip()}")
    return hits


def build(force=False, extra=None, verbose=False):
    extra = list(extra or [])
    if any(f.startswith("-D") for f in extra):
        raise ValueError("libhlgs.so is built without defines; experiment variants: tools/build_variant.py")
    sw = variant_switches()
    if sw:
        raise RuntimeError("compile-time variant switches in the product sources:\n" + "\n".join(sw))
    os.makedirs(OBJDIR, exist_ok=True)
    os.makedirs(LIBDIR, exist_ok=True)
    if not force and os.path.exists(LIB) and os.path.getmtime(LIB) >= _deps_mtime():
        if not os.path.exists(os.path.join(LIBDIR, "build_info.json")):
            write_build_info()
        return LIB
    with cf.ThreadPoolExecutor(max_workers=min(len(SOURCES), 8)) as ex:
        objs = list(ex.map(lambda s: _compile(s, extra), SOURCES))
    cmd = [HIPCC, "-shared", f"--offload-arch={ARCH}", "-o", LIB] + objs
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"link failed:\n{' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    write_build_info()
    if verbose:
        print("built", LIB)
    return LIB


def lib_sha16(path=LIB):
    """First 16 hex digits of the library's SHA-256: the build identity profiles are matched against."""
    import hashlib
    with open(path, "rb") as f:
        return hashlib.sha256(f.read()).hexdigest()[:16]


def write_build_info():
    """lib/build_info.json: the library's hash and the git HEAD it was built from (the GPU box gets the tree without
    .git, so the commit is recorded here, at build time)."""
    import json
    head, dirty = None, None
    try:
        root = os.path.dirname(PKG)
        head = subprocess.run(["git", "-C", root, "rev-parse", "HEAD"], capture_output=True, text=True,
                              check=True).stdout.strip()
        dirty = bool(subprocess.run(["git", "-C", root, "status", "--porcelain", "--untracked-files=no", "--",
                                     "hierarchical-lod-gaussians_amd/csrc", "include"], capture_output=True,
                                    text=True).stdout.strip())
    except (OSError, subprocess.CalledProcessError):
        pass
    json.dump(dict(lib_sha16=lib_sha16(), head=head, sources_dirty=dirty),
              open(os.path.join(LIBDIR, "build_info.json"), "w"))


if __name__ == "__main__":
    build(force="--force" in sys.argv, verbose=True)
