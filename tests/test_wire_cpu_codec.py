"""BASELINE config 1 exactly as stated: client/example's Set+Get of one 1 MiB
object, RS(10+2), CPU encode/decode, against a loopback proxy, no GPU.

The client, its Split/Join and the RESP wire format are the product
(infinicache_amd.client / .ec / .resp).  Only the GF arithmetic underneath is
swapped for a test double that calls the CPU oracle (oracle/rs_oracle.c, the
restatement of klauspost/reedsolomon v1.9.3): this tests the plumbing
(client/example/main.go:12-38, ecRedis.go:58-191, the proxy's first-d rule
proxy/lambdastore/connection.go:274-306), not the codec.  The codec itself is
tested bit-exact against the same oracle on the GPU (test_gpu_parity.py)."""
import itertools

import numpy as np
import pytest

import infinicache_amd as ia
import oracle
from infinicache_amd.client import NewClient
from infinicache_amd.ec import RSEncoder, _check
from oracle import rs_numpy as rn
from tests.fake_proxy import FakeProxy


class OracleCodec(RSEncoder):
    """reedsolomon.Encoder whose Encode/Verify/Reconstruct run on the CPU
    oracle (test double); Split/Join/argument handling are the product's."""

    def _store(self, shards, out, idx):
        for i in idx:
            if shards[i] is None or len(shards[i]) == 0:
                shards[i] = out[i].copy()
            else:
                shards[i][:] = out[i]

    def Encode(self, shards):
        e, out = oracle.encode(self.DataShards, self.ParityShards, list(shards))
        _check(e)
        self._store(shards, out, range(self.DataShards, self.Shards))

    def Verify(self, shards):
        e, ok = oracle.verify(self.DataShards, self.ParityShards, list(shards))
        _check(e)
        return ok

    def Reconstruct(self, shards):
        missing = [i for i, s in enumerate(shards) if s is None or len(s) == 0]
        e, out = oracle.reconstruct(self.DataShards, self.ParityShards, list(shards))
        _check(e)
        self._store(shards, out, missing)


@pytest.fixture
def proxy():
    p = FakeProxy()
    yield p
    p.close()


def _cpu_client(k=10, p=2):
    cli = NewClient(k, p, 32, fused_decode=False)  # Encode->Verify, Verify->Reconstruct->Verify
    cli.EC = OracleCodec(k, p)
    return cli


def test_config1_set_get_1mib_cpu_codec(proxy):
    cli = _cpu_client()
    assert cli.Dial([proxy.addr])
    data = rn.splitmix64_bytes(0x1F1C, 0, 1 << 20).tobytes()
    _, ok = cli.EcSet("foo", data)
    assert ok and proxy.sets == 12
    # the stored parity is the oracle's RS(10+2) parity of Split(data)
    sh = rn.split(data, 10, 2)
    par = rn.encode(sh[:10], 2)
    assert proxy.store[("foo", "10")] == par[0].tobytes()
    assert proxy.store[("foo", "11")] == par[1].tobytes()
    for _ in range(3):  # random first-d subsets: 2 nil shards each time
        _, reader, ok = cli.EcGet("foo", len(data))
        assert ok and reader.read() == data
        assert not cli.Data.AllGood and cli.Data.Corrupted  # reference's inverted flag
    cli.Close()


def test_config1_every_late_pair_cpu_codec(proxy):
    cli = _cpu_client()
    assert cli.Dial([proxy.addr])
    data = rn.splitmix64_bytes(0x1F1C, 9, 1024).tobytes()  # the example's 1 KiB object
    assert cli.EcSet("k", data)[1]
    for late in itertools.combinations(range(12), 2):
        proxy.force_late = late
        _, reader, ok = cli.EcGet("k", len(data))
        assert ok and reader.read() == data, late
    cli.Close()


def test_config1_corruption_detected_cpu_codec(proxy):
    cli = _cpu_client()
    assert cli.Dial([proxy.addr])
    data = rn.splitmix64_bytes(0x1F1C, 5, 4096).tobytes()
    assert cli.EcSet("c", data)[1]
    proxy.corrupt("c", 11, pos=17)
    proxy.force_late = (2,)
    _, reader, ok = cli.EcGet("c", len(data))
    assert not ok  # Verification failed after reconstruction
    cli.Close()
