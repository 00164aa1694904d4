"""Does overlapping the encode of batch i+1 with the decode of batch i (two
HIP streams, event dependencies per batch copy) beat the one-stream
sequence?  Measurement only: the headline's step runs encode
then decode of one batch on one stream, so each kernel's tail (the last
workgroups of a launch running on a part-idle chip) is paid twice a step.

    python tools/overlap_probe.py [steps]
"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

import infinicache_amd as ia  # noqa: E402


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 200
    k, p, nobj, copies = 10, 2, 1024, 3
    n = k + p
    S = (1 << 20) // k + 1
    pitch = (S + 255) // 256 * 256
    stride = n * pitch
    dev = torch.device("cuda", 0)
    enc = ia.New(k, p, device=0)
    g = torch.Generator(device=dev).manual_seed(0x1F1C)
    allbuf = torch.randint(0, 256, (copies, nobj, n, pitch), dtype=torch.uint8, device=dev, generator=g)
    allbuf[..., S:] = 0
    bufs = [allbuf[j] for j in range(copies)]
    present = [i not in (0, 5) for i in range(n)]
    bad = [torch.zeros(nobj, dtype=torch.int32, device=dev) for _ in range(copies)]
    sA = torch.cuda.Stream(dev)
    sB = torch.cuda.Stream(dev)
    for b in bufs:
        enc.encode_dev(b, S, pitch, stride, nobj, sA)
    torch.cuda.synchronize(dev)

    def seq(K):
        for i in range(K):
            b = bufs[i % copies]
            enc.encode_dev(b, S, pitch, stride, nobj, sA)
            enc.decode_dev(b, present, S, pitch, stride, nobj, bad[i % copies], sA)

    ev_enc = [torch.cuda.Event() for _ in range(copies)]
    ev_dec = [torch.cuda.Event() for _ in range(copies)]
    for e in ev_dec:
        e.record(sB)

    def ovl(K):
        for i in range(K):
            j = i % copies
            b = bufs[j]
            sA.wait_event(ev_dec[j])  # the last decode of this copy (it writes rows the encode reads)
            enc.encode_dev(b, S, pitch, stride, nobj, sA)
            ev_enc[j].record(sA)
            sB.wait_event(ev_enc[j])
            enc.decode_dev(b, present, S, pitch, stride, nobj, bad[j], sB)
            ev_dec[j].record(sB)

    bytes_step = 2 * nobj * (1 << 20)
    for name, fn in (("one stream", seq), ("two streams", ovl), ("one stream", seq), ("two streams", ovl)):
        fn(300)
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        fn(steps)
        torch.cuda.synchronize(dev)
        dt = time.perf_counter() - t0
        print(f"{name:12s} {steps} steps: {dt / steps * 1e3:.4f} ms/step, {bytes_step * steps / dt / 2**30:,.1f} GiB/s",
              flush=True)
    # correctness: rows {0, 5} rebuilt from garbage, decode flags clear
    ref = bufs[0].clone()
    torch.cuda.synchronize(dev)
    bufs[0][:, [0, 5], :S] = 7
    torch.cuda.synchronize(dev)  # the fill ran on torch's stream, the decode goes on sA
    enc.decode_dev(bufs[0], present, S, pitch, stride, nobj, bad[0], sA)
    torch.cuda.synchronize(dev)
    print("check:", "bit-exact" if torch.equal(bufs[0][..., :S], ref[..., :S]) and int(bad[0].sum()) == 0 else "FAILED")


if __name__ == "__main__":
    main()
