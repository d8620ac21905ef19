import sys, os
sys.path.insert(0, os.getcwd())
import numpy as np, torch
from realtime_stereo_matcher_amd import functional as F
for dt in (torch.float16, torch.bfloat16, torch.float32):
    for (n, c, h, w, D) in [(1, 8, 4, 20, 7), (1, 16, 2, 128, 24), (1, 8, 2, 256, 64), (1, 64, 2, 960, 192)]:
        g = torch.Generator(device="cuda").manual_seed(0)
        L = torch.randn(n, c, h, w, device="cuda", generator=g).to(dt)
        R = torch.randn(n, c, h, w, device="cuda", generator=g).to(dt)
        a = F.inner_product_volume(L, R, D, algo="h2").float()
        b = F.inner_product_volume(L, R, D, algo="valu").float()
        err = (a - b).abs()
        bad = (err > 0.05).nonzero()
        print(dt, (n, c, h, w, D), "maxerr", float(err.max()), "nbad", bad.shape[0], bad[:5].tolist())
