"""Host-side sanitizers for the native runtime: the pure C++ core
(`csrc/runtime/runtime_core.h`) is compiled into `csrc/selftest/runtime_selftest.cpp` with
AddressSanitizer + UndefinedBehaviorSanitizer and with ThreadSanitizer (loader thread pool,
watchdog monitor thread) and run here on the CPU. GPU-side sanitizers are not available on the
MI355X pool; device code is covered by the bitwise-determinism and oracle tests instead."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "csrc", "selftest", "runtime_selftest.cpp")

CONFIGS = {
    "plain": ["-O2"],
    "asan_ubsan": ["-O1", "-g", "-fsanitize=address,undefined", "-fno-omit-frame-pointer",
                   "-fno-sanitize-recover=all"],
    "tsan": ["-O1", "-g", "-fsanitize=thread"],
}


@pytest.mark.skipif(shutil.which("g++") is None, reason="no host compiler")
@pytest.mark.parametrize("cfg", sorted(CONFIGS))
def test_runtime_selftest(tmp_path, cfg):
    exe = tmp_path / f"selftest_{cfg}"
    subprocess.run(["g++", "-std=c++17", *CONFIGS[cfg], "-pthread", SRC, "-o", str(exe)],
                   check=True, capture_output=True, timeout=240)
    env = dict(os.environ, TMPDIR=str(tmp_path),
               ASAN_OPTIONS="verify_asan_link_order=0:detect_leaks=1:abort_on_error=0",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1",
               TSAN_OPTIONS="halt_on_error=1:second_deadlock_stack=1")
    r = subprocess.run([str(exe)], env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0 and "selftest ok" in r.stdout, r.stderr[-4000:]
    assert "WARNING: ThreadSanitizer" not in r.stderr and "ERROR: AddressSanitizer" not in r.stderr
