import os, sys, torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from realtime_stereo_matcher_amd import functional as F
torch.manual_seed(0)
for dt in (torch.float16,):
    n, c, h, w, D = 1, 16, 1, 128, 32
    L = torch.randint(-3, 4, (n, c, h, w), device="cuda").to(dt)
    R = torch.randint(-3, 4, (n, c, h, w), device="cuda").to(dt)
    ref = F.inner_product_volume(L.float(), R.float(), D, algo="valu")
    for algo in ("h2", "ws"):
        got = F.inner_product_volume(L, R, D, algo=algo).float()
        bad = (got - ref).abs() > 1e-3
        print(algo, dt, "bad cells", int(bad.sum()), "of", bad.numel())
        if bad.any():
            idx = bad.nonzero()[:12].tolist()
            for i in idx:
                print("  n,d,y,x", i, "got", got[tuple(i)].item(), "ref", ref[tuple(i)].item())
            # which d rows / x cols are bad
            print("  bad d:", sorted(set(bad.nonzero()[:, 1].tolist()))[:40])
            print("  bad x:", sorted(set(bad.nonzero()[:, 3].tolist()))[:64])
    # single channel test: L = delta at one channel/pixel, R = ones -> out[d, x] = L[x]
    L = torch.zeros(n, c, h, w, device="cuda", dtype=dt); R = torch.zeros_like(L)
    L[0, 0, 0, :] = torch.arange(w, device="cuda").to(dt) / 4
    R[0, 0, 0, :] = 1
    got = F.inner_product_volume(L, R, D, algo="ws").float()
    print("delta test d=0 row:", got[0, 0, 0, :20].tolist())
    print("delta test d=5 row:", got[0, 5, 0, :20].tolist())
