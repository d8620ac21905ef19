"""Debug: fused soft-argmin NaNs with cells near FLT_MAX (C = 16, R = L = +-a)."""
import sys, os
import numpy as np
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from realtime_stereo_matcher_amd import functional as F
from oracle import stereo_oracle as O

rng = np.random.default_rng(7)
sgn = np.where(rng.uniform(size=(1, 16, 2, 128)) < 0.5, -1.0, 1.0)
for top in (1e30, 1e37, 1.5e38, 1.9e38, 2.1e38, 2.5e38, 3.2e38):
    a = np.float32(np.sqrt(top / 16))
    l = (sgn * a).astype(np.float32)
    L = torch.from_numpy(l).cuda()
    for D, keep in ((96, True), (96, False), (256, False)):
        vol, disp = F.inner_product_soft_argmin(L, L, D, keep_volume=keep)
        d = disp.cpu().numpy()
        want = O.softargmin(O.inner_product(l, l, D))
        vnan = int(np.isnan(vol.cpu().numpy()).sum()) if keep else -1
        print(f"top {top:.2e} D {D} keep {keep}: disp nan {int(np.isnan(d).sum())} inf {int(np.isinf(d).sum())} "
              f"max err {float(np.nanmax(np.abs(d - want))):.3e} vol nan {vnan}", flush=True)
