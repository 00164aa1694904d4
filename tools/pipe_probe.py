"""Config-5 trace through the host pipeline (rsgpu_encode_batch /
rsgpu_decode_batch), each op timed on its own: object GiB/s and the PCIe
bytes it moves (encode: 10 S in, 2 S out; decode: 10 S in, 2 S out).
Measurement only (not a test).

    python tools/pipe_probe.py [reps]
"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import infinicache_amd as ia  # noqa: E402

GiB = float(1 << 30)


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    k, p, nobj = 10, 2, 512
    n = k + p
    rng = np.random.Generator(np.random.PCG64(20200225))
    sizes = np.exp(rng.uniform(np.log(4096), np.log(100 << 20), nobj)).astype(np.int64)
    S = (sizes + k - 1) // k
    offs = np.concatenate([[0], np.cumsum(n * S)])
    enc = ia.New(k, p)
    host = ia.host_alloc(int(offs[-1]))
    host[:] = np.frombuffer(np.random.default_rng(1).bytes(int(offs[-1])), dtype=np.uint8)
    objs = [[host[offs[o] + i * S[o]:offs[o] + (i + 1) * S[o]] for i in range(n)] for o in range(nobj)]
    present = [[i not in (0, 5) for i in range(n)]] * nobj
    tot = int(sizes.sum())
    pcie = int((n * S).sum())  # 10 S in + 2 S out per op
    enc.encode_batch(objs)
    enc.decode_batch(objs, present=present)
    for name, fn in (("encode_batch", lambda: enc.encode_batch(objs)),
                     ("decode_batch", lambda: enc.decode_batch(objs, present=present))):
        ts = []
        for _ in range(reps):
            t0 = time.perf_counter()
            fn()
            ts.append(time.perf_counter() - t0)
        t = sorted(ts)[len(ts) // 2]
        print(f"{name}: {t * 1e3:7.1f} ms  objects {tot / t / GiB:6.2f} GiB/s  PCIe {pcie / t / 1e9:6.2f} GB/s "
              f"(in {10 * int(S.sum()) / t / 1e9:6.2f}, out {2 * int(S.sum()) / t / 1e9:5.2f})", flush=True)


if __name__ == "__main__":
    main()
