"""Variable-size object tables (rsgpu_*_dev_objs, gf_apply_var) against the
fixed-layout launch on the SAME objects: 1024 x 1 MiB RS(10+2), three batch
copies in rotation (cold, as bench.py), HIP events around 20 launches per op,
interleaved rounds.  Prints us per launch and % of 8 TB/s on the algorithmic
bytes.  Measurement only (not a test).

    python tools/var_probe.py [rounds]
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import infinicache_amd as ia  # noqa: E402


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    k, p, nobj, copies = 10, 2, 1024, 3
    n = k + p
    S = (1 << 20) // k + 1
    pitch = (S + 255) // 256 * 256
    stride = n * pitch
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(7)
    allbuf = torch.randint(0, 256, (copies, nobj, n, pitch), dtype=torch.uint8, device=dev, generator=g)
    allbuf[..., S:] = 0
    enc = ia.New(k, p)
    st = torch.cuda.current_stream(dev)
    enc.encode_dev(allbuf, S, pitch, stride, nobj * copies, st)
    bad = torch.zeros(nobj, dtype=torch.int32, device=dev)
    present = [i not in (0, 5) for i in range(n)]
    tabs = [[(allbuf[c].data_ptr() + o * stride, S, pitch) for o in range(nobj)] for c in range(copies)]
    alg = nobj * n * S

    ops = {
        "encode fixed": lambda c: enc.encode_dev(allbuf[c], S, pitch, stride, nobj, st),
        "encode objs": lambda c: enc.encode_dev_objs(tabs[c], st),
        "decode fixed": lambda c: enc.decode_dev(allbuf[c], present, S, pitch, stride, nobj, bad, st),
        "decode objs": lambda c: enc.decode_dev_objs(tabs[c], present, bad, st),
    }
    for _ in range(50):  # clock ramp
        for f in ops.values():
            f(0)
    res = {name: [] for name in ops}
    for _ in range(rounds):
        for name, f in ops.items():
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            f(1)
            e0.record(st)
            for i in range(20):
                f(i % copies)
            e1.record(st)
            e1.synchronize()
            res[name].append(e0.elapsed_time(e1) / 20 * 1e3)
    torch.cuda.synchronize()
    assert int(bad.sum()) == 0
    for name, us in res.items():
        us.sort()
        med = us[len(us) // 2]
        print(f"{name:14s} med {med:7.1f} us  min {us[0]:7.1f}  {alg / (med * 1e-6) / 8e12 * 100:5.1f} % of 8 TB/s",
              flush=True)


if __name__ == "__main__":
    main()
