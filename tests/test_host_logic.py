"""Host-side mirror semantics that run without a GPU: Split / Join (upstream
Join = /root/reference/client/ec.go:83-121), DummyEncoder
(/root/reference/client/ec.go:26-121) and NewEncoder (ec.go:14-24)."""
import io
import os
import sys

import numpy as np
import pytest

import infinicache_amd as ia
from oracle import rs_numpy as rn


def test_split_pads_to_k_plus_p_one_backing_array():
    enc = ia.New(10, 2)
    data = bytes(range(256)) * 4 + b"xyz"  # 1027 bytes
    sh = enc.Split(data)
    assert len(sh) == 12 and all(len(s) == 103 for s in sh)
    assert sh[0].base is sh[11].base  # one backing array, as upstream
    assert np.concatenate(sh).tobytes()[:1027] == data
    assert not np.concatenate(sh)[1027:].any()
    for a, b in zip(sh, rn.split(data, 10, 2)):
        assert np.array_equal(a, b)


def test_split_short_data():
    with pytest.raises(ia.ErrShortData):
        ia.New(10, 2).Split(b"")


def test_split_one_byte():
    sh = ia.New(10, 2).Split(b"\x07")
    assert [len(s) for s in sh] == [1] * 12 and sh[0][0] == 7


def test_join_roundtrip_and_errors():
    enc = ia.New(4, 2)
    data = b"0123456789abcdefXYZ"
    sh = enc.Split(data)
    out = io.BytesIO()
    enc.Join(out, sh, len(data))
    assert out.getvalue() == data
    out = io.BytesIO()
    enc.Join(out, sh, 5)
    assert out.getvalue() == data[:5]
    with pytest.raises(ia.ErrTooFewShards):
        enc.Join(io.BytesIO(), sh[:3], len(data))
    bad = list(sh)
    bad[1] = None
    with pytest.raises(ia.ErrReconstructRequired):
        enc.Join(io.BytesIO(), bad, len(data))
    with pytest.raises(ia.ErrShortData):
        enc.Join(io.BytesIO(), sh, 4 * len(sh[0]) + 1)
    # parity shards missing is fine: Join reads data shards only
    nopar = list(sh[:4]) + [None, None]
    out = io.BytesIO()
    enc.Join(out, nopar, len(data))
    assert out.getvalue() == data


def test_dummy_encoder_semantics():
    d = ia.DummyEncoder(4)
    sh = d.Split(b"0123456789")  # perShard 3: 3,3,3,1 — no padding
    assert [bytes(s) for s in sh] == [b"012", b"345", b"678", b"9"]
    assert d.Verify(sh)
    with pytest.raises(ia.ErrTooFewShards):
        d.Verify(sh[:3])
    with pytest.raises(ia.ErrTooFewShards):
        d.Verify(sh[:3] + [b""])
    with pytest.raises(ia.ErrNotImplemented):
        d.Update(sh, sh)
    assert d.Encode(sh) is None
    out = io.BytesIO()
    d.Join(out, sh, 10)
    assert out.getvalue() == b"0123456789"
    with pytest.raises(ia.ErrShortData):
        d.Split(b"")
    # fewer bytes than shards: ec.go:77-79 stores the empty remainder in the
    # next shard (a non-nil empty slice); later shards stay nil
    sh = d.Split(b"ab")
    assert [None if s is None else bytes(s) for s in sh] == [b"a", b"b", b"", None]


def test_new_encoder_factory(capsys):
    assert isinstance(ia.NewEncoder(10, 0, 32), ia.DummyEncoder)
    assert isinstance(ia.NewEncoder(10, 2, 32), ia.RSEncoder)
    assert ia.NewEncoder(0, 2, 32) is None  # error printed and swallowed
    assert "newEncoder err" in capsys.readouterr().out


def _outcome(fn):
    try:
        return ("ok", fn())
    except Exception as e:  # noqa: BLE001 - the class is the result
        return ("raise", type(e).__name__)


def _need_pyshards(ec):
    """The C marshalling module must be built wherever it can be: skip only
    when this interpreter has no Python.h (the Makefile then builds the
    ctypes path alone), fail when it could have been built but was not."""
    if ec._pyshards is not None:
        return
    import sysconfig
    if not os.path.exists(os.path.join(sysconfig.get_paths()["include"], "Python.h")):
        pytest.skip("no Python.h for this interpreter: csrc/pyshards.c not built, ctypes marshalling only")
    pytest.fail(f"csrc/pyshards.c not built for {sys.executable} "
                f"(make -C infinicache_amd/csrc PY={sys.executable})")


def test_c_marshalling_matches_ctypes_path(monkeypatch):
    """The per-object calls marshal their shard table in C
    (csrc/pyshards.c) when the extension is built; every argument case ends
    exactly as through the ctypes table (the same upstream error, the same
    NoDevice on a GPU-less host, the same refusal of read-only or
    non-contiguous outputs, the same copy of a non-contiguous input)."""
    from infinicache_amd import ec
    _need_pyshards(ec)
    k, p, S = 10, 2, 103
    n = k + p

    def split():
        b = np.zeros(n * S, np.uint8)
        b[:k * S] = np.arange(k * S) % 251
        return [b[i * S:(i + 1) * S] for i in range(n)]

    strided = np.zeros(2 * S, np.uint8)[::2]
    cases = {
        "encode ok": lambda e: e.Encode(split()),
        "encode 11 shards": lambda e: e.Encode(split()[:11]),
        "encode size mismatch": lambda e: e.Encode(split()[:-1] + [np.zeros(S + 1, np.uint8)]),
        "encode all empty": lambda e: e.Encode([np.zeros(0, np.uint8)] * n),
        "encode read-only parity": lambda e: e.Encode(split()[:k] + [bytes(S)] * p),
        "encode strided parity": lambda e: e.Encode(split()[:k] + [strided, np.zeros(S, np.uint8)]),
        "encode strided input": lambda e: e.Encode([strided] + split()[1:]),
        "encode bytes inputs": lambda e: e.Encode([bytes(x) for x in split()[:k]] + [bytearray(S)] * p),
        "verify ok": lambda e: e.Verify(split()),
        "verify nil shard": lambda e: e.Verify([None] + split()[1:]),
        "encode+verify ok": lambda e: e.EncodeVerify(split()),
        "decode ok": lambda e: e.DecodeVerify([None if i in (0, 5) else s for i, s in enumerate(split())]),
        "decode too few": lambda e: e.DecodeVerify([None if i < 3 else s for i, s in enumerate(split())]),
        "reconstruct ok": lambda e: e.Reconstruct([None if i in (1, 11) else s for i, s in enumerate(split())]),
        "reconstruct data": lambda e: e.ReconstructData([None if i in (1, 11) else s for i, s in enumerate(split())]),
        "reconstruct size mismatch": lambda e: e.Reconstruct([None] + split()[1:-1] + [np.zeros(S + 2, np.uint8)]),
    }
    enc = ia.New(k, p)
    fast = {name: _outcome(lambda: f(enc)) for name, f in cases.items()}
    monkeypatch.setattr(ec, "_pyshards", None)
    slow = {name: _outcome(lambda: f(enc)) for name, f in cases.items()}
    assert fast == slow
    if not ia.device_ok(0):
        assert fast["encode ok"] == ("raise", "NoDevice")
        assert fast["encode 11 shards"] == ("raise", "ErrTooFewShards")
        assert fast["encode read-only parity"] == ("raise", "InvalidArgument")


def test_c_batch_marshalling_matches_ctypes_path(monkeypatch):
    """encode_batch / decode_batch(present=...) marshal in C as well; every
    argument case ends exactly as through the ctypes tables."""
    from infinicache_amd import ec
    _need_pyshards(ec)
    k, p = 10, 2
    n = k + p

    def arena(sizes):
        Ss = [(nb + k - 1) // k for nb in sizes]
        buf = np.zeros(sum(n * S for S in Ss), np.uint8)
        out, off = [], 0
        for S in Ss:
            out.append([buf[off + i * S:off + (i + 1) * S] for i in range(n)])
            off += n * S
        return out

    def swapped():
        objs = arena([1000, 2000])
        objs[1][3], objs[1][4] = objs[1][4], objs[1][3]  # not one Split array
        return objs

    def readonly():
        objs = arena([1000])
        objs[0][11] = np.frombuffer(bytes(len(objs[0][11])), np.uint8)
        return objs

    pres = lambda nobj, lost=(0, 5): [[i not in lost for i in range(n)]] * nobj  # noqa: E731
    cases = {
        "enc lists": lambda e: e.encode_batch(arena([1000, 4096, 7])),
        "enc arrays": lambda e: e.encode_batch([np.zeros(n * 100, np.uint8), np.zeros(n * 3, np.uint8)]),
        "enc array not multiple": lambda e: e.encode_batch([np.zeros(n * 100 + 1, np.uint8)]),
        "enc 11 rows": lambda e: e.encode_batch([arena([1000])[0][:11]]),
        "enc rows swapped": lambda e: e.encode_batch(swapped()),
        "enc read-only row": lambda e: e.encode_batch(readonly()),
        "enc empty": lambda e: e.encode_batch([]),
        "enc zero-length": lambda e: e.encode_batch([np.zeros(0, np.uint8)]),
        "dec ok": lambda e: e.decode_batch(arena([1000, 4096]), present=pres(2)),
        "dec size mismatch": lambda e: e.decode_batch([arena([1000])[0][:11] + [np.zeros(7, np.uint8)]],
                                                      present=pres(1)),
        "dec None entry": lambda e: e.decode_batch([[None] + arena([1000])[0][1:]], present=pres(1)),
        "dec 11 shards": lambda e: e.decode_batch([arena([1000])[0][:11]], present=pres(1)),
        "dec read-only output": lambda e: e.decode_batch(readonly(), present=pres(1, lost=(11,))),
        "dec too few present": lambda e: e.decode_batch(arena([1000]), present=pres(1, lost=(0, 1, 2))),
        "dec empty": lambda e: e.decode_batch([], present=[]),
    }
    enc = ia.New(k, p)
    fast = {name: _outcome(lambda: f(enc)) for name, f in cases.items()}
    monkeypatch.setattr(ec, "_pyshards", None)
    slow = {name: _outcome(lambda: f(enc)) for name, f in cases.items()}
    assert fast == slow
    if not ia.device_ok(0):
        assert fast["enc lists"] == ("raise", "NoDevice")
        assert fast["enc rows swapped"] == ("raise", "InvalidArgument")
        assert fast["dec size mismatch"] == ("raise", "ErrShardSize")
