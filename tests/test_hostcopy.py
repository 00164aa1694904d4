"""The host copy pool (infinicache_amd/csrc/hostcopy.cpp) under
ThreadSanitizer and under ASan/UBSan, on the CPU.

The pool spreads the pageable staging copies of a per-object call
(rsgpu.cpp run_host; the Go Split array an EcSet passes,
client/ecRedis.go:384) over a few threads; concurrent callers share it with
try_lock.  tests/hostcopy_check.cpp drives it from several caller threads at
once with batches on both sides of its 12 MiB threshold, ragged and empty
rows, and checks every byte plus guard bytes around each row.  Host code only:
device code is never instrumented."""
import os
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(ROOT, "infinicache_amd", "csrc")
CLANGXX = "/opt/rocm/lib/llvm/bin/clang++"
OUT = os.path.join(ROOT, "tools", "san")


def _build(name, flags):
    if not os.path.exists(CLANGXX):
        pytest.skip("no clang++ in this image")
    os.makedirs(OUT, exist_ok=True)
    exe = os.path.join(OUT, name)
    subprocess.check_call([
        CLANGXX, "-O1", "-g", "-std=c++17", "-fno-omit-frame-pointer", *flags,
        "-D__HIP_PLATFORM_AMD__", "-I/opt/rocm/include", "-I", CSRC,
        os.path.join(HERE, "hostcopy_check.cpp"), os.path.join(CSRC, "hostcopy.cpp"),
        "-o", exe, "-lpthread"])
    return exe


def _run(exe, threads, callers, batches, seed, extra_env):
    env = dict(os.environ, RSGPU_COPY_THREADS=str(threads), **extra_env)
    r = subprocess.run([exe, str(callers), str(batches), str(seed)], env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "WARNING: ThreadSanitizer" not in r.stderr, r.stderr
    assert "ok" in r.stdout


@pytest.mark.parametrize("threads,callers", [(4, 1), (4, 4), (1, 3), (0, 2)])
def test_copy_pool_tsan(threads, callers):
    exe = _build("hostcopy_check_tsan", ["-fsanitize=thread"])
    _run(exe, threads, callers, 8, 11 + threads + callers, {"TSAN_OPTIONS": "halt_on_error=1 exitcode=66"})


def test_copy_pool_asan_ubsan():
    exe = _build("hostcopy_check_asan", ["-fsanitize=address,undefined", "-fno-sanitize-recover=all"])
    _run(exe, 4, 4, 8, 7, {"ASAN_OPTIONS": "halt_on_error=1:detect_leaks=0"})
