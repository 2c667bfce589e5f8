"""CPU: the oracle under host sanitizers.

oracle/selftest.c drives the oracle's entries over seeded random data and
runs the threaded cpu_baseline pipelines against their single-thread results;
it is built with AddressSanitizer + UndefinedBehaviorSanitizer (leaks on)
and with ThreadSanitizer, and both builds must run clean."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("kind,env", [
    ("asan", {"ASAN_OPTIONS": "detect_leaks=1:abort_on_error=0",
              "UBSAN_OPTIONS": "halt_on_error=1:print_stacktrace=1"}),
    ("tsan", {"TSAN_OPTIONS": "halt_on_error=1"}),
])
def test_oracle_selftest_under_sanitizer(tmp_path, kind, env):
    if shutil.which("gcc") is None or shutil.which("make") is None:
        pytest.skip("no gcc / make")
    out = str(tmp_path)
    b = subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "OUT=" + out,
                        "selftest-" + kind], capture_output=True, text=True, timeout=300)
    assert b.returncode == 0, b.stdout + b.stderr
    e = dict(os.environ)
    e.update(env)
    r = subprocess.run([os.path.join(out, "selftest_" + kind)], capture_output=True, text=True,
                       timeout=300, env=e)
    assert r.returncode == 0 and "oracle selftest ok" in r.stdout, r.stdout[-2000:] + r.stderr[-4000:]
