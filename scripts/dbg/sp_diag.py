"""Where does algo "sp" differ from the oracle?  python scripts/dbg/sp_diag.py N C H W D"""
import sys, os
import numpy as np
import torch
sys.path.insert(0, os.getcwd())
from realtime_stereo_matcher_amd import functional as F
from oracle import stereo_oracle as O

n, c, h, w, D = map(int, sys.argv[1:6])
rng = np.random.default_rng(1)
l = rng.standard_normal((n, c, h, w), dtype=np.float32)
r = rng.standard_normal((n, c, h, w), dtype=np.float32)
for algo in ("h2db", "sp"):
    got = F.inner_product_volume(torch.from_numpy(l).cuda(), torch.from_numpy(r).cuda(), D, algo=algo).cpu().numpy()
    want = O.inner_product(l, r, D)
    bad = ~(np.abs(got - want) <= 1e-4)
    print(algo, "bad cells", int(bad.sum()), "of", bad.size, "nan", int(np.isnan(got).sum()))
    if bad.any():
        idx = np.argwhere(bad)
        for ax, name in enumerate("ndyx"):
            v = idx[:, ax]
            u, cnt = np.unique(v, return_counts=True)
            print(f"  {name}: {len(u)} values, range {v.min()}..{v.max()}, top {list(zip(u[np.argsort(-cnt)][:8], np.sort(-cnt)[:8] * -1))}")
        # per (y, x0 tile, d chunk)
        tiles = {}
        for (nn, d, y, x) in idx[:20000]:
            k = (int(nn), int(y), int(x // 128), int(d // 32))
            tiles[k] = tiles.get(k, 0) + 1
        print("  (n, y, tile, dchunk) -> count:", sorted(tiles.items())[:40])
        print("  sample:", [(tuple(i), float(got[tuple(i)]), float(want[tuple(i)])) for i in idx[:6]])
