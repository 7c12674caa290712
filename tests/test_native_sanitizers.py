"""Native runtime under sanitizers (SURVEY §5 "Race detection / sanitizers"):
the shared-memory step ring (1 writer + N reader threads on one mapping) and the
KV block pool (randomised alloc / free / prefix-cache sequences against a
refcount model), built as host-only binaries with ThreadSanitizer and with
AddressSanitizer + UBSan. Any report makes the binary exit non-zero."""
import os
import subprocess

import pytest

from hipserve._build import build_sanitizer_test


@pytest.mark.parametrize("kind", ["thread", "address"])
def test_runtime_under_sanitizer(kind):
    try:
        exe = build_sanitizer_test(kind)
    except RuntimeError as e:
        if "cannot find" in str(e) or "unrecognized" in str(e):
            pytest.skip(f"{kind} sanitizer runtime not available: {e}")
        raise
    # verify_asan_link_order=0: the environment may preload an unrelated library
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1 second_deadlock_stack=1",
               ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:verify_asan_link_order=0",
               UBSAN_OPTIONS="halt_on_error=1")
    msgs = "5000" if kind == "thread" else "20000"
    r = subprocess.run([exe, msgs], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr[-4000:]
    assert "runtime_stress ok" in r.stdout
    assert "WARNING: ThreadSanitizer" not in r.stderr and "ERROR: AddressSanitizer" not in r.stderr
