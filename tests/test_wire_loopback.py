"""EcSet/EcGet through the RESP wire format against a loopback proxy
(BASELINE config 1 plumbing).  CPU tests use the
reference's own p == 0 DummyEncoder path (no GF math, no GPU); the gpu tests
run RS(10+2) on the MI355X codec underneath an unchanged object API."""
import socket
import threading

import numpy as np
import pytest

import infinicache_amd as ia
from infinicache_amd import resp
from infinicache_amd.client import MaxLambdaStores, NewClient
from oracle import rs_numpy as rn
from tests.fake_proxy import FakeProxy


@pytest.fixture
def proxy():
    p = FakeProxy()
    yield p
    p.close()


def test_set_command_bytes_match_ecredis_format():
    """The exact bytes of one shard SET (ecRedis.go:233-245) and GET (:275-277)."""
    srv = socket.socket()
    srv.bind(("127.0.0.1", 0))
    srv.listen(16)
    got = []

    def serve():
        conns = [srv.accept()[0] for _ in range(4)]
        for c in conns:
            r, w = resp.Reader(c), resp.Writer(c)
            cmd = r.read_command()
            got.append(cmd)
            w.write_bulk_string(cmd[5 if cmd[0] == b"set" else 3].decode())
            w.write_bulk_string(cmd[2].decode())
            w.write_bulk_string("7")
            w.flush()

    t = threading.Thread(target=serve, daemon=True)
    t.start()
    cli = NewClient(4, 0, 32)  # DummyEncoder: 4 shards, no parity
    assert cli.Dial(["127.0.0.1:%d" % srv.getsockname()[1]])
    placements = [0] * 4
    reqid, ok = cli.EcSet("foo", b"abcdefghijkl", 0, placements)
    t.join(5)
    assert ok and placements == [7, 7, 7, 7]
    cmds = sorted(got, key=lambda c: int(c[2]))
    for i, c in enumerate(cmds):
        assert c[0] == b"set" and c[1] == b"foo" and c[2] == str(i).encode()
        assert 0 <= int(c[3]) < MaxLambdaStores and c[4] == b"400"
        assert c[5] == reqid.encode() and c[6] == b"4" and c[7] == b"0"
        assert c[8] == b"abcdefghijkl"[3 * i:3 * i + 3]
    cli.Close()
    srv.close()


def test_resp_encoding_bytes():
    class Sink:
        def __init__(self):
            self.data = b""

        def sendall(self, b):
            self.data += b

    s = Sink()
    w = resp.Writer(s)
    w.write_cmd_string("get", "foo", "3", "rid", "10", "2")
    w.flush()
    assert s.data == (b"*6\r\n$3\r\nget\r\n$3\r\nfoo\r\n$1\r\n3\r\n$3\r\nrid\r\n"
                      b"$2\r\n10\r\n$1\r\n2\r\n")


def test_dummy_encoder_set_get_roundtrip(proxy):
    cli = NewClient(10, 0, 32)
    assert cli.Dial([proxy.addr])
    data = rn.splitmix64_bytes(0x1F1C, 1, 1 << 20).tobytes()
    _, ok = cli.EcSet("obj", data)
    assert ok and proxy.sets == 10
    _, reader, ok = cli.EcGet("obj", len(data))
    assert ok and reader.read() == data
    assert cli.Data.AllGood
    cli.Close()


def test_get_missing_key_fails(proxy):
    cli = NewClient(4, 0, 32)
    assert cli.Dial([proxy.addr])
    _, reader, ok = cli.EcGet("nope", 10)
    assert not ok and reader is None
    cli.Close()


@pytest.mark.gpu
def test_rs10_2_set_get_1mib(gpu, proxy):
    """BASELINE config 1: client/example Set+Get of one 1 MiB object, RS(10+2)
    (client/example/main.go:12-38 at 1 MiB), codec on the MI355X."""
    cli = NewClient(10, 2, 32)
    assert cli.Dial([proxy.addr])
    data = rn.splitmix64_bytes(0x1F1C, 2, 1 << 20).tobytes()
    placements = [0] * 12
    _, ok = cli.EcSet("foo", data, 0, placements)
    assert ok and proxy.sets == 12
    assert all(0 <= x < MaxLambdaStores for x in placements) and len(set(placements)) == 12
    for _ in range(5):  # random first-d subsets: 2 nil shards each time
        _, reader, ok = cli.EcGet("foo", len(data))
        assert ok and reader.read() == data
        assert not cli.Data.AllGood and cli.Data.Corrupted  # reference's inverted flag
    cli.Close()


@pytest.mark.gpu
def test_rs10_2_every_late_pair(gpu, proxy):
    cli = NewClient(10, 2, 32)
    assert cli.Dial([proxy.addr])
    data = rn.splitmix64_bytes(0x1F1C, 3, 100_003).tobytes()
    assert cli.EcSet("k", data)[1]
    import itertools
    for late in itertools.combinations(range(12), 2):
        proxy.force_late = late
        _, reader, ok = cli.EcGet("k", len(data))
        assert ok and reader.read() == data, late
    cli.Close()


@pytest.mark.gpu
def test_rs10_2_failed_chunk_is_recovered(gpu, proxy):
    """A GET error on one chunk: decode still succeeds (2 late + 1 failed
    would be too many, so force 1 late) and recover() re-SETs the chunk."""
    cli = NewClient(10, 2, 32)
    assert cli.Dial([proxy.addr])
    data = rn.splitmix64_bytes(0x1F1C, 4, 54321).tobytes()
    assert cli.EcSet("r", data)[1]
    original = proxy.store[("r", "3")]
    proxy.store[("r", "3")] = b"junk"
    proxy.fail_chunks = {3}
    proxy.force_late = (7,)
    sets_before = proxy.sets
    _, reader, ok = cli.EcGet("r", len(data))
    assert ok and reader.read() == data
    assert proxy.sets == sets_before + 1
    assert proxy.store[("r", "3")] == original  # re-set with reconstructed bytes
    cli.Close()


@pytest.mark.gpu
def test_rs10_2_corruption_detected_with_extra_shard(gpu, proxy):
    """With 11 bodies (1 late), the extra parity shard is really verified."""
    cli = NewClient(10, 2, 32)
    assert cli.Dial([proxy.addr])
    data = rn.splitmix64_bytes(0x1F1C, 5, 4096).tobytes()
    assert cli.EcSet("c", data)[1]
    proxy.corrupt("c", 11, pos=17)
    proxy.force_late = (2,)
    _, reader, ok = cli.EcGet("c", len(data))
    assert not ok  # Verification failed after reconstruction
    cli.Close()
