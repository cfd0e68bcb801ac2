"""CPU: AddressSanitizer + UndefinedBehaviorSanitizer builds (SURVEY.md §5 race/sanitizer plan): the CPU oracle over
the reference KATs (tests/san/oracle_driver.c) and the host side of libdrandhip through its C ABI with no GPU present
(tests/san/host_driver.c; the kernels are untouched — GPU sanitizers are not available on this pool). Each driver
exits non-zero on a failed check and the sanitizers abort on any report. The recipes are tests/san/Makefile, which
(with this file) is listed in .gpurunignore: no GPU run builds or loads a sanitizer build."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SAN = os.path.join(ROOT, "tests", "san")
ENV = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:abort_on_error=1", UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")


def _run(cmd, cwd):
    r = subprocess.run(cmd, cwd=cwd, env=ENV, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-4000:])
    return r.stdout


@pytest.mark.skipif(shutil.which("gcc") is None, reason="gcc missing")
def test_oracle_asan_ubsan():
    _run(["make", "-s", "_build/oracle_san"], SAN)
    out = _run(["./_build/oracle_san"], SAN)
    assert "all checks passed" in out


@pytest.mark.skipif(not os.path.exists(os.path.join(ROOT, "drand_amd", "csrc", "k_prep.o")),
                    reason="kernel objects not built (make -C drand_amd)")
def test_library_host_asan_ubsan():
    _run(["make", "-s", "_build/host_driver"], SAN)
    out = _run(["./_build/host_driver"], SAN)
    assert "all checks passed" in out
