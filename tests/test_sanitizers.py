"""ASan/UBSan run of the native host runtime (sanitizer build for C++ host code).

The batcher and the libhdf5 shard reader/prefetcher are rebuilt with
``-fsanitize=address,undefined`` (``build.build_sanitized``) and driven by
``tools/asan_native.py`` in a subprocess with the clang ASan runtime preloaded.
A canary program with a deliberate heap overflow proves the sanitizer is live.
Host code only: GPU sanitizers are not used on this platform.
"""
import os
import subprocess
import sys

import pytest

from hetseq_amd.csrc import build

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

pytestmark = pytest.mark.skipif(build.asan_runtime() is None or not os.path.exists(build.SAN_CXX),
                                reason="clang ASan runtime not available")


def _env():
    env = dict(os.environ)
    env["LD_PRELOAD"] = build.asan_runtime()
    env["ASAN_OPTIONS"] = "detect_leaks=0:abort_on_error=0"
    env["UBSAN_OPTIONS"] = "print_stacktrace=1:halt_on_error=1"
    return env


def test_sanitizer_is_live(tmp_path):
    src = tmp_path / "canary.cpp"
    src.write_text("#include <cstdlib>\nint main(int c, char**) { int* a = new int[4]; int r = a[c + 3]; "
                   "delete[] a; return r; }\n")
    exe = tmp_path / "canary"
    subprocess.run([build.SAN_CXX] + build.SAN_FLAGS + [str(src), "-o", str(exe)], check=True)
    r = subprocess.run([str(exe)], env=_env(), capture_output=True, text=True, timeout=60)
    assert r.returncode != 0 and "heap-buffer-overflow" in r.stderr


def test_native_runtime_under_asan_ubsan():
    outs = build.build_sanitized()
    r = subprocess.run([sys.executable, "-u", os.path.join(ROOT, "tools", "asan_native.py"), os.path.dirname(outs[0])],
                       env=_env(), capture_output=True, text=True, timeout=600)
    assert r.returncode == 0 and "SANITIZERS CLEAN" in r.stdout, r.stdout[-2000:] + r.stderr[-4000:]
    assert "runtime error" not in r.stderr, r.stderr[-4000:]  # UBSan findings
