"""Property-based checks (hypothesis) of the host layer and the CPU oracle, no
GPU: the size-independent properties the reference's path promises, drawn
over random codes, object sizes and erasure patterns.

  * Split -> encode -> erase up to p shards -> reconstruct -> Join returns the
    object (client/ecRedis.go:382-432 end to end, upstream Split/Join
    semantics of infinicache_amd/ec.py, arithmetic by the numpy oracle);
  * the coding matrix is systematic and MDS: its top k rows are the
    identity and every k-row subset of the (k+p) x k matrix inverts
    (upstream buildMatrix), for both matrix kinds;
  * the C oracle and the numpy oracle agree on random codes and data
    (oracle/rs_oracle.c vs oracle/rs_numpy.py);
  * the RESP codec (infinicache_amd/resp.py, the wire format of
    client/ecRedis.go:233-245,275-277) round-trips arbitrary commands and
    bulk strings, including empty and binary ones, split at any point."""
import io
import itertools
import socket
import threading
import time

import numpy as np
import pytest
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

import infinicache_amd as ia
import oracle
from infinicache_amd import resp
from oracle import rs_numpy as rn

SETTINGS = settings(max_examples=60, deadline=None, suppress_health_check=[HealthCheck.too_slow])


@SETTINGS
@given(k=st.integers(1, 16), p=st.integers(1, 6), data=st.binary(min_size=1, max_size=3000), seed=st.integers(0, 2**32 - 1))
def test_split_encode_erase_reconstruct_join(k, p, data, seed):
    enc = ia.New(k, p)
    sh = enc.Split(data)
    S = len(sh[0])
    assert len(sh) == k + p and all(len(s) == S for s in sh)
    par = rn.encode([sh[i] for i in range(k)], p)  # the p parity rows
    full = [np.asarray(sh[i]).copy() for i in range(k)] + [par[r] for r in range(p)]
    rng = np.random.default_rng(seed)
    lost = set(rng.choice(k + p, int(rng.integers(0, p + 1)), replace=False).tolist())
    got = [None if i in lost else full[i].copy() for i in range(k + p)]
    out = rn.reconstruct(got, k, p)
    for i in range(k + p):
        assert np.array_equal(out[i], full[i]), (k, p, sorted(lost), i)
    buf = io.BytesIO()
    enc.Join(buf, [np.asarray(s) for s in out], len(data))
    assert buf.getvalue() == data


@settings(max_examples=25, deadline=None)
@given(k=st.integers(1, 12), p=st.integers(1, 4), kind=st.sampled_from(["vandermonde", "cauchy"]))
def test_matrix_systematic_and_mds(k, p, kind):
    m = rn.build_matrix(k, p, kind)
    assert m.shape == (k + p, k)
    assert np.array_equal(m[:k], np.eye(k, dtype=np.uint8))
    rows = list(itertools.combinations(range(k + p), k))
    rng = np.random.default_rng(k * 31 + p)
    for r in (rows if len(rows) <= 40 else [rows[i] for i in rng.choice(len(rows), 40, replace=False)]):
        sub = m[list(r)]
        inv = rn.invert(sub)
        assert np.array_equal(rn.matmul(inv, sub), np.eye(k, dtype=np.uint8)), r


@SETTINGS
@given(k=st.integers(1, 20), p=st.integers(1, 8), size=st.integers(1, 700), seed=st.integers(0, 2**32 - 1),
       kind=st.sampled_from(["vandermonde", "cauchy"]))
def test_c_oracle_matches_numpy_oracle(k, p, size, seed, kind):
    rng = np.random.default_rng(seed)
    data = [rng.integers(0, 256, size, dtype=np.uint8) for _ in range(k)]
    e, full = oracle.encode(k, p, data + [bytes(size)] * p, kind)
    assert e == 0
    want = [np.asarray(d) for d in data] + list(rn.encode(data, p, kind))
    for i in range(k + p):
        assert np.array_equal(np.frombuffer(bytes(full[i]), np.uint8), want[i]), i


def _pair():
    a, b = socket.socketpair()
    a.settimeout(5)
    b.settimeout(5)
    return a, b


@SETTINGS
@given(args=st.lists(st.binary(max_size=200), min_size=1, max_size=8))
def test_resp_command_roundtrip(args):
    a, b = _pair()
    try:
        w = resp.Writer(a)
        w.write_multi_bulk_size(len(args))
        for x in args:
            w.write_bulk(x)
        w.flush()
        r = resp.Reader(b)
        assert r.read_command() == args
    finally:
        a.close()
        b.close()


@SETTINGS
@given(payload=st.binary(max_size=5000), chunk=st.integers(1, 64))
def test_resp_bulk_roundtrip_any_split(payload, chunk):
    """A bulk string whose bytes arrive in arbitrary pieces (the socket reader
    fills its buffer as data comes in)."""
    a, b = _pair()
    c, d = _pair()
    try:
        w = resp.Writer(a)
        w.write_bulk(payload)
        w.flush()
        a.shutdown(socket.SHUT_WR)
        wire = b""
        while True:
            x = b.recv(65536)
            if not x:
                break
            wire += x
        assert wire == b"$%d\r\n" % len(payload) + payload + b"\r\n"

        def feed():  # the same bytes in `chunk`-byte pieces, yielding between them
            for i in range(0, len(wire), chunk):
                c.sendall(wire[i:i + chunk])
                time.sleep(0)
        t = threading.Thread(target=feed)
        t.start()
        assert resp.Reader(d).read_bulk() == payload
        t.join(5)
    finally:
        for s_ in (a, b, c, d):
            s_.close()


if __name__ == "__main__":
    pytest.main([__file__, "-q"])
