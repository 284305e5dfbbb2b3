"""libcgx's host-only code under AddressSanitizer + UndefinedBehaviorSanitizer
(sanitizers on the host side; GPU sanitizers are not available).
tests/sanitize/Makefile builds the loader (cgx_mm.cpp), the SELL / SELL-P /
row-block planners and the halo planners instrumented; host_check.cpp
drives them on the golden files and synthetic matrices. Any report aborts."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_host_code_is_sanitizer_clean(tmp_path):
    b = subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "tests", "sanitize")],
                       capture_output=True, text=True, timeout=900)
    assert b.returncode == 0, b.stderr[-3000:]
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    r = subprocess.run([os.path.join(ROOT, "build", "sanitize", "host_check"),
                        os.path.join(ROOT, "tests", "golden"), str(tmp_path)],
                       capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0 and "host_check ok" in r.stdout, (r.stdout[-2000:], r.stderr[-4000:])
