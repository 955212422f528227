"""Host-side AddressSanitizer + UndefinedBehaviorSanitizer run of the C ABI (`make sanitize`,
tests/host_sanitize/abi_driver.cpp).  On the CPU container this exercises every host-only path:
argument validation and error messages, shape arithmetic, tuning hooks and the timing records;
on a GPU box the same driver also allocates, launches, captures and replays a graph of the whole
Generator forward (profiles/r02_host_sanitizer_gpu.txt).  Only leaks inside the ROCm runtime are
suppressed (tests/host_sanitize/lsan.supp)."""
import os
import shutil
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("hipcc") is None and not os.path.exists("/opt/rocm/bin/hipcc"),
                    reason="hipcc not available")
def test_abi_host_paths_under_asan_ubsan():
    jobs = str(min(8, os.cpu_count() or 4))
    subprocess.run(["make", "-j", jobs, "tests/host_sanitize/abi_driver"], cwd=REPO, check=True,
                   stdout=subprocess.DEVNULL, timeout=900)
    env = dict(os.environ, ASAN_OPTIONS="protect_shadow_gap=0:detect_leaks=1:abort_on_error=1",
               LSAN_OPTIONS="suppressions=tests/host_sanitize/lsan.supp", UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run(["./tests/host_sanitize/abi_driver"], cwd=REPO, env=env, capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "ERROR: AddressSanitizer" not in r.stderr and "runtime error" not in r.stderr
