"""Test infrastructure: AddressSanitizer + UndefinedBehaviorSanitizer builds (gcc, CPU only) of
  - the host C++ of libhlgs.so that parses files and builds SPTs (hierarchical-lod-gaussians_amd/csrc/hier_io.cpp,
    spt_build.cpp; they mirror gaussianhierarchy/hierarchy_loader.cpp:26-189 and scene/gaussian_model.py:184-352)
    -> tests/sanitize/build/libhlgs_host_asan.so, loaded through HLGS_LIBRARY (hlgs_core._lib binds what it exports);
  - the C oracle (oracle/hlgs_oracle.c) -> tests/sanitize/build/libhlgs_oracle_asan.so, loaded through HLGS_ORACLE_LIB.
GPU sanitizers are not available on the pool; the kernels are covered by the -m gpu parity tests instead.
tests/test_sanitizers.py runs the CPU suites that exercise these libraries under both sanitizers (LD_PRELOAD of gcc's
libasan, since the Python interpreter is not instrumented)."""
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
CSRC = os.path.join(ROOT, "hierarchical-lod-gaussians_amd", "csrc")
OUT = os.path.join(HERE, "build")
HOST_LIB = os.path.join(OUT, "libhlgs_host_asan.so")
ORACLE_LIB = os.path.join(OUT, "libhlgs_oracle_asan.so")
SAN = ["-fsanitize=address,undefined", "-fno-sanitize-recover=undefined", "-fno-omit-frame-pointer", "-g", "-O1",
       "-fPIC", "-shared"]


def _stale(out, srcs):
    return not os.path.exists(out) or os.path.getmtime(out) < max(os.path.getmtime(s) for s in srcs)


def build():
    os.makedirs(OUT, exist_ok=True)
    host = [os.path.join(CSRC, "hier_io.cpp"), os.path.join(CSRC, "spt_build.cpp"), os.path.join(HERE, "host_shim.cpp")]
    if _stale(HOST_LIB, host + [os.path.join(ROOT, "include", "hlgs.h")]):
        subprocess.check_call(["g++", "-std=c++17"] + SAN + ["-o", HOST_LIB] + host)
    src = os.path.join(ROOT, "oracle", "hlgs_oracle.c")
    if _stale(ORACLE_LIB, [src]):
        subprocess.check_call(["gcc", "-std=c11", "-fno-fast-math", "-ffp-contract=off"] + SAN +
                              ["-o", ORACLE_LIB, src, "-lm"])
    return HOST_LIB, ORACLE_LIB


def libasan():
    return subprocess.run(["gcc", "-print-file-name=libasan.so"], capture_output=True, text=True, check=True).stdout.strip()


if __name__ == "__main__":
    print(build())
