import time, numpy as np, torch, sys
sys.path.insert(0, '.')
import infinicache_amd as ia
enc = ia.New(10, 2)
k,p,S,nobj=10,2,104858,1024; n=12; pitch=104960
buf = torch.zeros((nobj, n, pitch), dtype=torch.uint8, device='cuda')
bad = torch.zeros(nobj, dtype=torch.int32, device='cuda')
rng = np.random.default_rng(1)
pres = np.ones((nobj, n), dtype=np.uint8)
for o in range(nobj): pres[o, rng.choice(n, 2, replace=False)] = 0
s = torch.cuda.current_stream()
for _ in range(3): enc.decode_dev_multi(buf, pres, S, pitch, n*pitch, nobj, bad, s)
torch.cuda.synchronize()
t = []; t2 = []
for _ in range(20):
    a = time.perf_counter(); enc.decode_dev_multi(buf, pres, S, pitch, n*pitch, nobj, bad, s); t.append(time.perf_counter() - a)
    a = time.perf_counter(); enc.encode_dev(buf, S, pitch, n*pitch, nobj, s); t2.append(time.perf_counter() - a)
    torch.cuda.synchronize()
print("decode_dev_multi host us: median %.1f" % (np.median(t)*1e6), " encode_dev host us: median %.1f" % (np.median(t2)*1e6))
