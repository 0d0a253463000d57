"""Experiment helper: link libhlgs.so variants for A/B runs.  Variants are never full-file copies in the tree: a variant
is a patch against the product sources, or a file taken from git history.

    python tools/build_variant.py NAME --patch tools/variants/X.patch
        apply a `git diff` of the product sources (paths from the repo root) to a scratch copy of csrc/ and include/,
        rebuild the files it touches, link them with the current objects of every other source
    python tools/build_variant.py NAME --rev COMMIT:PATH PRODUCT_FILE
        PRODUCT_FILE (e.g. raster_bwd.hip) replaced by the text of PATH at COMMIT (`git show`; tools/variants/INDEX.md
        lists the measured rounds-3-5 variants this way)
    python tools/build_variant.py NAME --defs "-DNAME=VALUE ..."   (every source rebuilt with the flags)
-> hierarchical-lod-gaussians_amd/lib/variants/NAME.so (load it with HLGS_LIBRARY=...).  A variant that no longer applies
or compiles fails loudly (tests/test_abi_cpu.py checks the patches under tools/variants/ still apply)."""
import concurrent.futures as cf
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "hierarchical-lod-gaussians_amd")
sys.path.insert(0, os.path.join(PKG, "hlgs_core"))
import build as B  # noqa: E402

CSRC_REL = os.path.join("hierarchical-lod-gaussians_amd", "csrc")


def _link(name, objs):
    out = os.path.join(PKG, "lib", "variants", name + ".so")
    os.makedirs(os.path.dirname(out), exist_ok=True)
    subprocess.run([B.HIPCC, "-shared", f"--offload-arch={B.ARCH}", "-o", out] + objs, check=True)
    print(out)
    return out


def _compile(src_path, product_name, obj):
    os.makedirs(os.path.dirname(obj), exist_ok=True)
    cmd = [B.HIPCC] + B.FLAGS + B.PER_FILE.get(product_name, []) + ["-c", src_path, "-o", obj]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"variant source {src_path} does not compile:\n{r.stderr[-4000:]}")
    return obj


def _scratch_tree(name):
    """A copy of the product sources (csrc/ and include/) laid out as in the repo, so relative includes resolve."""
    tree = os.path.join(PKG, "build", "var", name, "tree")
    shutil.rmtree(tree, ignore_errors=True)
    shutil.copytree(os.path.join(PKG, "csrc"), os.path.join(tree, CSRC_REL))
    shutil.copytree(os.path.join(ROOT, "include"), os.path.join(tree, "include"))
    return tree


def touched_files(patch):
    """Product files a patch changes (the csrc/ names)."""
    out = []
    for line in open(patch):
        if line.startswith("+++ b/"):
            p = line[6:].strip()
            if p.startswith(CSRC_REL + "/"):
                out.append(os.path.basename(p))
            elif not p.startswith("include/"):
                raise ValueError(f"{patch}: touches {p}, outside the product sources")
    return out


def apply_patch(patch, tree, check_only=False):
    cmd = ["patch", "-p1", "--forward", "--batch", "-d", tree, "-i", os.path.abspath(patch)]
    if check_only:
        cmd.insert(1, "--dry-run")
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"{patch} does not apply to the current sources:\n{r.stdout}{r.stderr}")


def with_patch(name, patch):
    B.build()
    tree = _scratch_tree(name)
    apply_patch(patch, tree)
    files = touched_files(patch)
    header_changed = any(line.startswith("+++ b/include/") or line.startswith(f"+++ b/{CSRC_REL}/hlgs_internal.h")
                         or line.startswith(f"+++ b/{CSRC_REL}/hlgs_math.h") for line in open(patch))
    rebuild = list(B.SOURCES) if header_changed else [f for f in files if f in B.SOURCES]
    odir = os.path.join(PKG, "build", "var", name, "obj")
    with cf.ThreadPoolExecutor(max_workers=8) as ex:
        new = dict(zip(rebuild, ex.map(lambda f: _compile(os.path.join(tree, CSRC_REL, f), f,
                                                          os.path.join(odir, os.path.splitext(f)[0] + ".o")), rebuild)))
    objs = [new.get(s, os.path.join(B.OBJDIR, os.path.splitext(s)[0] + ".o")) for s in B.SOURCES]
    return _link(name, objs)


def with_file(name, src_text, replaces):
    B.build()
    tree = _scratch_tree(name)
    path = os.path.join(tree, CSRC_REL, replaces)
    open(path, "w").write(src_text)
    obj = _compile(path, replaces, os.path.join(PKG, "build", "var", name, "obj", os.path.splitext(replaces)[0] + ".o"))
    objs = [obj if s == replaces else os.path.join(B.OBJDIR, os.path.splitext(s)[0] + ".o") for s in B.SOURCES]
    return _link(name, objs)


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
    return _link(name, objs)


def main(argv):
    name, mode = argv[0], argv[1]
    if mode == "--patch":
        with_patch(name, argv[2])
    elif mode == "--rev":
        text = subprocess.check_output(["git", "-C", ROOT, "show", argv[2]]).decode()
        with_file(name, text, argv[3])
    elif mode == "--defs":
        with_defs(name, argv[2].split())
    else:
        raise SystemExit(__doc__)


if __name__ == "__main__":
    main(sys.argv[1:])
