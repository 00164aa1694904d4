"""Mirror of /root/reference/client/example/main.go (BASELINE config 1):
NewClient(10, 2, 32), Dial("127.0.0.1:6378"), EcSet("foo", val), EcGet("foo").

    python examples/client_example.py [--size 1048576] [--addr 127.0.0.1:6378] [--loopback]

--loopback starts the in-process fake proxy (tests/fake_proxy.py) on the given
address instead of expecting a real InfiniCache proxy.  The RS(10+2) codec
underneath runs on the MI355X (infinicache_amd); the object API and the RESP
wire format are the reference's.
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from infinicache_amd.client import NewClient  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=int, default=1 << 20)
    ap.add_argument("--addr", default="127.0.0.1:6378")
    ap.add_argument("--loopback", action="store_true")
    a = ap.parse_args()
    proxy = None
    if a.loopback:
        from tests.fake_proxy import FakeProxy
        host, port = a.addr.rsplit(":", 1)
        proxy = FakeProxy(host, int(port))
    val = os.urandom(a.size)
    cli = NewClient(10, 2, 32)
    if not cli.Dial(a.addr.split(",")):
        sys.exit("Failed to dial")
    t0 = time.time()
    _, ok = cli.EcSet("foo", val)
    if not ok:
        sys.exit("Failed to set")
    print("Set foo %d ns" % int(cli.Data.Duration * 1e9))
    # the first call also initialises the device (HIP context, code object):
    # a second Set shows the steady-state latency
    _, ok = cli.EcSet("foo", val)
    if not ok:
        sys.exit("Failed to set")
    print("Set foo %d ns (second call)" % int(cli.Data.Duration * 1e9))
    _, reader, ok = cli.EcGet("foo", a.size)
    if not ok:
        sys.exit("Failed to get")
    got = reader.read()
    print("Got foo %d ( %d %d ) match=%s" % (int(cli.Data.Duration * 1e9), int(cli.Data.RecLatency * 1e9),
                                            int((cli.Data.Duration - cli.Data.RecLatency) * 1e9),
                                            got == val))
    cli.Close()
    if proxy:
        proxy.close()
    print("total %.3f s" % (time.time() - t0))


if __name__ == "__main__":
    main()
