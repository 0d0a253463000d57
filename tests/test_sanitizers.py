"""The host C++ that parses untrusted files and builds SPTs (csrc/hier_io.cpp, csrc/spt_build.cpp) and the C oracle
run clean under AddressSanitizer + UndefinedBehaviorSanitizer (gcc builds, tests/sanitize/build.py).

The CPU suites that drive them -- file round trips, malformed files, SPT construction against its restatement, the
oracle against its float64 restatement and the LOD functions -- run in a child process with gcc's libasan preloaded
(the interpreter is not instrumented), with HLGS_LIBRARY pointing at the sanitized host library and HLGS_ORACLE_LIB at
the sanitized oracle.  Any ASan report or UBSan runtime error aborts the child (-fno-sanitize-recover)."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests", "sanitize"))
import build as SB  # noqa: E402

SUITES = ["tests/test_hier_io.py", "tests/test_hier_malformed.py", "tests/test_spt_build.py", "tests/test_spt_golden.py",
          "tests/test_oracle.py", "tests/test_oracle_lod.py"]


def test_host_code_and_oracle_under_asan_ubsan():
    host, orc = SB.build()
    env = dict(os.environ)
    env.update(LD_PRELOAD=SB.libasan(), ASAN_OPTIONS="detect_leaks=0:abort_on_error=1:allocator_may_return_null=1",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1", HLGS_LIBRARY=host, HLGS_ORACLE_LIB=orc,
               PYTHONPATH=os.pathsep.join([ROOT, os.path.join(ROOT, "hierarchical-lod-gaussians_amd")]))
    r = subprocess.run([sys.executable, "-m", "pytest", "-q", "-x", "-m", "not gpu", "-p", "no:cacheprovider"] + SUITES,
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=900)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-6000:]
    assert "AddressSanitizer" not in out and "runtime error:" not in out, out[-6000:]
    assert " passed" in out
