"""Host-side AddressSanitizer + UndefinedBehaviorSanitizer over the C ABI
(no sanitizers in the reference; the build runs its host code
under ASan/UBSan).  `make -C infinicache_amd/csrc sanitize` instruments the
host compile of rsgpu.cpp / pipeline.cpp (argument checks, plan and inverse
caches, staging slots, pipelines); device code is never instrumented (the
-fsanitize flags go to -Xarch_host only).  tests/c_abi_client.c and the CPU
oracle (its checker) are built with the same clang and the same runtimes.
Any ASan/UBSan report aborts the client (halt_on_error)."""
import os
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
SAN = os.path.join(ROOT, "tools", "san")
CLANG = "/opt/rocm/lib/llvm/bin/clang"


def _runtime_dir():
    r = subprocess.run([CLANG, "-print-resource-dir"], capture_output=True, text=True, check=True)
    return os.path.join(r.stdout.strip(), "lib", "linux")


@pytest.fixture(scope="module")
def san_client():
    if not os.path.exists(CLANG):
        pytest.skip("no clang in this image")
    subprocess.check_call(["make", "-s", "-j8", "-C", os.path.join(ROOT, "infinicache_amd", "csrc"), "sanitize"])
    out = os.path.join(SAN, "c_abi_client_san")
    rt = _runtime_dir()
    subprocess.check_call([
        CLANG, "-O1", "-g", "-std=c11", "-D_GNU_SOURCE", "-fsanitize=address,undefined",
        "-shared-libasan", "-fno-omit-frame-pointer", "-I", os.path.join(ROOT, "include"),
        "-I", os.path.join(ROOT, "oracle"), os.path.join(HERE, "c_abi_client.c"),
        os.path.join(ROOT, "oracle", "rs_oracle.c"), "-o", out, "-L", SAN, "-l:librsgpu_san.so",
        "-Wl,-rpath," + SAN, "-Wl,-rpath," + rt, "-lpthread"])
    return out


def _run(binary, *args, timeout=300):
    env = dict(os.environ)
    # the HIP runtime keeps process-lifetime allocations: leak checking off
    env["ASAN_OPTIONS"] = "detect_leaks=0:abort_on_error=1"
    env["UBSAN_OPTIONS"] = "print_stacktrace=1:halt_on_error=1"
    return subprocess.run([binary, *args], capture_output=True, text=True, timeout=timeout, env=env)


def test_c_abi_host_paths_under_asan_ubsan(san_client):
    r = _run(san_client)
    assert r.returncode == 0, r.stderr[-4000:] + r.stdout
    assert "host checks ok" in r.stdout
    assert "ERROR: AddressSanitizer" not in r.stderr and "runtime error" not in r.stderr


@pytest.mark.gpu
def test_c_abi_gpu_paths_under_asan_ubsan(gpu, san_client):
    """The host side of every GPU path (staging, pinned DMA, pipelines,
    mixed-pattern images) under ASan/UBSan, with the kernels running."""
    r = _run(san_client, "gpu")
    assert r.returncode == 0, r.stderr[-4000:] + r.stdout
    assert "gpu checks ok" in r.stdout
    assert "ERROR: AddressSanitizer" not in r.stderr and "runtime error" not in r.stderr


def _stress_client(kind):
    """tests/c_abi_stress.c built against librsgpu_san.so (kind "asan": ASan +
    UBSan) or librsgpu_tsan.so ("tsan"), or against the product library
    (kind "plain")."""
    if not os.path.exists(CLANG):
        pytest.skip("no clang in this image")
    src = [os.path.join(HERE, "c_abi_stress.c"), os.path.join(ROOT, "oracle", "rs_oracle.c")]
    inc = ["-I", os.path.join(ROOT, "include"), "-I", os.path.join(ROOT, "oracle")]
    os.makedirs(SAN, exist_ok=True)
    out = os.path.join(SAN, "c_abi_stress_" + kind)
    if kind == "plain":
        lib = os.path.join(ROOT, "infinicache_amd")
        subprocess.check_call([CLANG, "-O2", "-std=c11", "-D_GNU_SOURCE", *inc, *src, "-o", out, "-L", lib,
                               "-l:librsgpu.so", "-Wl,-rpath," + lib, "-lpthread"])
        return out
    subprocess.check_call(["make", "-s", "-j8", "-C", os.path.join(ROOT, "infinicache_amd", "csrc"),
                           "sanitize" if kind == "asan" else "tsan"])
    flags = ["-fsanitize=address,undefined", "-shared-libasan"] if kind == "asan" else ["-fsanitize=thread"]
    lib = "-l:librsgpu_san.so" if kind == "asan" else "-l:librsgpu_tsan.so"
    objs = []
    for f in src:
        o = os.path.join(SAN, kind + "_" + os.path.basename(f) + ".o")
        subprocess.check_call([CLANG, "-O1", "-g", "-std=c11", "-D_GNU_SOURCE", "-fno-omit-frame-pointer", *flags,
                               *inc, "-c", f, "-o", o])
        objs.append(o)
    # linked by the C++ driver: it exports the runtime's C++ interceptors
    # (operator new/delete, the __cxa_guard_* of the library's function-local
    # statics) from the executable, which a C link leaves out
    subprocess.check_call([CLANG + "++", *flags, *objs, "-o", out, "-L", SAN, lib, "-Wl,-rpath," + SAN,
                           "-Wl,-rpath," + _runtime_dir(), "-lpthread"])
    return out


def test_stress_clients_build():
    """The stress client links against all three libraries (the runs need a GPU)."""
    for kind in ("plain", "asan", "tsan"):
        assert os.path.exists(_stress_client(kind))


def _stress(kind, threads, seconds, seed, code=()):
    exe = _stress_client(kind)
    env = dict(os.environ)
    env["ASAN_OPTIONS"] = "detect_leaks=0:abort_on_error=1"
    env["UBSAN_OPTIONS"] = "print_stacktrace=1:halt_on_error=1"
    env["TSAN_OPTIONS"] = ("halt_on_error=1:exitcode=66:second_deadlock_stack=1:suppressions="
                           + os.path.join(HERE, "tsan.supp"))
    r = subprocess.run([exe, str(threads), str(seconds), str(seed), *map(str, code)], capture_output=True, text=True,
                       timeout=seconds + 60, env=env)
    print(r.stdout)
    assert r.returncode == 0, r.stderr[-6000:] + r.stdout
    assert "all bit-exact" in r.stdout
    for bad in ("ERROR: AddressSanitizer", "runtime error", "WARNING: ThreadSanitizer"):
        assert bad not in r.stderr, r.stderr[-6000:]
    return r.stdout


@pytest.mark.gpu
def test_stress_every_route_concurrently(gpu):
    """16 threads on one context, the product library: worker (mailbox image,
    in place, column slices in place and staged), stream path with slot
    growth, copy pool, pinned images freed per call, all at once."""
    _stress("plain", 16, 10, 1)


@pytest.mark.gpu
@pytest.mark.parametrize("code", [(4, 2, 0), (12, 4, 0), (1, 1, 0), (10, 4, 1)])
def test_stress_other_codes(gpu, code):
    """The same routes on other codes: RS(12+4) (four rows per worker pass),
    RS(4+2), RS(1+1), and RS(10+4) on upstream's Cauchy matrix."""
    _stress("plain", 8, 5, 40 + code[0], code)


@pytest.mark.gpu
def test_stress_under_asan_ubsan(gpu):
    _stress("asan", 8, 10, 2)


@pytest.mark.gpu
def test_stress_under_tsan(gpu):
    """Data races in the host side (slots, worker mailboxes and reader epochs,
    deferred frees, copy pool) under ThreadSanitizer with the kernels running."""
    _stress("tsan", 8, 12, 3)
