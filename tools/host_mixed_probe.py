"""Host-side timing of the mixed-pattern decode path (which host call the GPU
waits for): per-call wall time of encode_dev and decode_dev_multi in the
bench's step loop, 1024 x 1 MiB RS(10+2), 3 rotating batch copies."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import infinicache_amd as ia  # noqa: E402

k, p, nobj, copies = 10, 2, 1024, 3
n = k + p
S = ((1 << 20) + k - 1) // k
pitch = (S + 255) // 256 * 256
stride = n * pitch
enc = ia.New(k, p)
buf = torch.randint(0, 256, (copies, nobj, n, pitch), dtype=torch.uint8, device="cuda")
bad = torch.zeros(nobj, dtype=torch.int32, device="cuda")
rng = np.random.default_rng(1)
pres = np.ones((nobj, n), dtype=np.uint8)
for o in range(nobj):
    pres[o, rng.choice(n, p, replace=False)] = 0
st = torch.cuda.current_stream()
te, td = [], []
for it in range(40):
    b = buf[it % copies]
    t0 = time.perf_counter()
    enc.encode_dev(b, S, pitch, stride, nobj, st)
    t1 = time.perf_counter()
    enc.decode_dev_multi(b, pres, S, pitch, stride, nobj, bad, st)
    t2 = time.perf_counter()
    if it >= 5:
        te.append(t1 - t0)
        td.append(t2 - t1)
torch.cuda.synchronize()
print(f"encode_dev host call: p50 {np.median(te)*1e6:.1f} us  max {np.max(te)*1e6:.1f} us")
print(f"decode_dev_multi host call: p50 {np.median(td)*1e6:.1f} us  max {np.max(td)*1e6:.1f} us")
