"""Builds tests/c_abi_client.c with gcc against librsgpu.so (+ the oracle as
the checker) and runs it: the C ABI consumed from plain C, as the cgo shim in
INTEGRATION.md would (no Python, no torch in the process)."""
import os
import subprocess

import pytest

from infinicache_amd import _lib
import oracle

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


@pytest.fixture(scope="module")
def client_bin(tmp_path_factory):
    oracle.build()
    out = str(tmp_path_factory.mktemp("cabi") / "c_abi_client")
    libdir = os.path.dirname(_lib.LIB_PATH)
    odir = os.path.join(ROOT, "oracle")
    subprocess.check_call([
        "gcc", "-O2", "-std=c11", "-Wall", "-Werror", "-I", os.path.join(ROOT, "include"),
        os.path.join(HERE, "c_abi_client.c"), "-o", out,
        "-L", libdir, "-lrsgpu", "-Wl,-rpath," + libdir,
        "-L", odir, "-l:liboracle.so", "-Wl,-rpath," + odir, "-lpthread"])
    return out


def test_c_abi_host_paths(client_bin):
    r = subprocess.run([client_bin], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr + r.stdout
    assert "host checks ok" in r.stdout


@pytest.mark.gpu
def test_c_abi_gpu_paths(gpu, client_bin):
    r = subprocess.run([client_bin, "gpu"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr + r.stdout
    assert "gpu checks ok" in r.stdout
    assert "ecredis replay ok" in r.stdout
    # BASELINE config 3's Get (RS(10+4), 4 MiB: 12 and 13 of 14 shards present)
    assert "ecredis replay ok (RS(10+4), 4194304-B object" in r.stdout


@pytest.mark.gpu
def test_c_abi_exit_with_worker_running(gpu, client_bin):
    """A process that ends with the resident kernel still polling and no
    rsgpu_destroy (a Go client just exits): the library's atexit guard stops
    the worker before the runtime frees its mailboxes."""
    env = dict(os.environ, RSGPU_WORKER_TRACE="1")
    r = subprocess.run([client_bin, "exit_with_worker"], capture_output=True, text=True, timeout=60, env=env)
    assert r.returncode == 0, r.stderr + r.stdout
    assert "exit with the worker running" in r.stdout
    assert "rsgpu worker trace encode+verify" in r.stderr, r.stderr
