#!/usr/bin/env python3
"""Host-side replay of the fp16 two-plane band kernel's indexing (csrc/ip_h2.hip), run before any
GPU launch of a changed indexing scheme:   python scripts/check_h2_bounds.py

1. every stage lane's feature loads for every pipeline step of every workgroup stay inside the
   feature tensor (the grid is 2 workgroups per CU);
2. the epilogue's ring writes and reads stay inside the ring, and after block a the ring chunk
   a holds, at (row, column), exactly the accumulator element of band cell (dl = 32a + row, x):
   R row j = x - d (the shear permutation), for every wave and lane;
3. every stored output offset lies inside the (N, D, H, W) volume and every (d, x) cell with
   d < D, x < W of every segment is stored exactly once over the whole grid."""
import sys

import numpy as np

KXT, KSLOT = 128, 32 * 512


def geo(D):
    npass = -(-D // 192)
    pw = (-(-D // npass) + 3) // 4 * 4
    T = 2 if pw <= 32 else 3 if pw <= 64 else 5 if pw <= 128 else 7
    DMAX = 32 * (T - 1)
    RW = KXT + DMAX
    ROWS = RW + KXT
    return T, DMAX, RW, ROWS // 4, npass, pw


def work_lists(N, H, W, D, ncu):
    T, DMAX, RW, GROUPS, npass, pw = geo(D)
    tiles = -(-W // KXT)
    nwork = tiles * H * N * npass
    nwg = max(8, (min(nwork, 2 * ncu) + 7) // 8 * 8)
    q, rr = nwork >> 3, nwork & 7
    for blk in range(nwg):
        grp, gi, gsz = blk & 7, blk >> 3, nwg >> 3
        wbeg = grp * (q + 1) if grp < rr else rr * (q + 1) + (grp - rr) * q
        wend = wbeg + q + (1 if grp < rr else 0)
        if wbeg + gi >= wend:
            continue
        nitems = (wend - (wbeg + gi) + gsz - 1) // gsz
        yield blk, [wbeg + gi + it * gsz for it in range(nitems)]


def decode(w, tiles, npass, H, D, pw, DMAX):
    pas, rest = w % npass, w // npass
    tile, row = rest % tiles, rest // tiles
    y, n = row % H, row // H
    x0, dp = tile * KXT, pas * pw
    return n, y, x0, dp, min(pw, D - dp), x0 - dp - DMAX


def check_loads(N, C, H, W, D, ncu=256):
    T, DMAX, RW, GROUPS, npass, pw = geo(D)
    tiles = -(-W // KXT)
    ITEMS = 2 * GROUPS
    cs, hs, ns = H * W, W, C * H * W
    numel = N * ns
    nks = -(-C // 16)
    bad = 0
    for blk, items in work_lists(N, H, W, D, ncu):
        S = len(items) * nks
        for s in range(S + 2):
            ss = min(s, S - 1)
            it, ks = divmod(ss, nks)
            n, y, x0, dp, Dp, js = decode(items[it], tiles, npass, H, D, pw, DMAX)
            for sq in range(256):
                h = min(sq // GROUPS, 1)
                g = min(sq - h * GROUPS, GROUPS - 1)
                active = sq < ITEMS
                isR = 4 * g < RW
                c0 = ks * 16 + 8 * h
                px = js + 4 * g if isR else x0 + 4 * g - RW
                okp = active and 0 <= px < W
                if okp and px % 4:
                    bad += 1  # 16-B groups must be aligned
                base = n * ns + y * hs + (px if okp else 0) + min(c0, C - 1) * cs
                for kk in range(8):
                    off = kk if C % 16 == 0 else min(kk, max(C - 1 - c0, 0))
                    e = base + off * cs
                    if e < 0 or e + 4 > numel:
                        bad += 1
    return bad


def check_shear(T):
    """Simulate the ring of one full segment; returns the number of mismatches."""
    DMAX = 32 * (T - 1)
    ring = {}  # byte offset within the ring -> (wave, t, i, lane)
    bad = 0
    for a in range(-1, T - 1):
        t = T - 2 - a
        sa, sb = (a + 3) % 3, (a + 4) % 3
        for wave in range(4):
            for lane in range(64):
                lr, hh = lane & 31, lane >> 5
                u = lr - 4 * hh
                wbase = 4 * (32 * wave + lr) + u * 512
                for i in range(16):
                    ci = (i & 3) + 8 * (i >> 2)
                    if sa != 2:
                        addr = wbase + sb * KSLOT - ci * 512
                    else:
                        addr = wbase + 3 * KSLOT - ci * 512 - (3 * KSLOT if u >= ci else 0)
                    if not 0 <= addr < 3 * KSLOT:
                        bad += 1
                        continue
                    ring[addr] = (wave, t, ci + 4 * hh, lr)
        if a < 0:
            continue
        # chunk a is read: rows 8w + hh + 2qq, column 4 lr .. 4 lr + 3
        for wave in range(4):
            for lane in range(64):
                lr, hh = lane & 31, lane >> 5
                srow = 8 * wave + hh
                for qq in range(4):
                    row = srow + 2 * qq
                    dl = 32 * a + row
                    for e in range(4):
                        addr = sa * KSLOT + row * 512 + 16 * lr + 4 * e
                        xcol = 4 * lr + e  # column within the segment
                        src = ring.get(addr)
                        if src is None:
                            bad += 1
                            continue
                        w2, t2, jj, x2 = src
                        # the element holds R row 32(w2+t2)+jj (relative to js) and L column
                        # 32 w2 + x2; its disparity relative to dp is x - j + DMAX - ... :
                        # d_l = (32 w2 + x2) - (32 (w2 + t2) + jj) + DMAX
                        d_l = (32 * w2 + x2) - (32 * (w2 + t2) + jj) + DMAX
                        if 32 * w2 + x2 != xcol or d_l != dl:
                            bad += 1
    return bad


def check_stores(N, H, W, D, ncu=256):
    T, DMAX, RW, GROUPS, npass, pw = geo(D)
    tiles = -(-W // KXT)
    hits = np.zeros(N * D * H * W, np.int32)
    bad = 0
    for blk, items in work_lists(N, H, W, D, ncu):
        for w in items:
            n, y, x0, dp, Dp, js = decode(w, tiles, npass, H, D, pw, DMAX)
            fullx = x0 + KXT <= W
            for a in range(T - 1):
                for wave in range(4):
                    for lane in range(64):
                        lr, hh = lane & 31, lane >> 5
                        srow = 8 * wave + hh
                        okx = x0 + 4 * lr < W
                        for qq in range(4):
                            dl = 32 * a + 2 * qq + srow
                            if dl < Dp and (fullx or okx):
                                base = ((n * D + dp + dl) * H + y) * W + x0 + 4 * lr
                                if base < 0 or base + 4 > hits.size:
                                    bad += 1
                                    continue
                                hits[base:base + 4] += 1
    bad += int((hits != 1).sum())
    return bad


if __name__ == "__main__":
    fails = 0
    for T in (2, 3, 5, 7):
        b = check_shear(T)
        print(f"shear T={T}: mismatches {b}")
        fails += b
    shapes = [(1, 32, 64, 128, 24), (1, 64, 2, 200, 192), (1, 32, 2, 100, 300), (1, 8, 2, 64, 64),
              (2, 20, 3, 260, 100), (1, 48, 2, 132, 33), (1, 16, 1, 1000, 256), (1, 7, 2, 36, 40),
              (1, 64, 2, 960, 192), (1, 33, 2, 512, 31), (1, 64, 3, 960, 192), (2, 17, 3, 64, 24),
              (1, 16, 2, 1920, 256), (1, 8, 2, 64, 201), (1, 4, 3, 20, 7)]
    for sh in shapes:
        b = check_loads(*sh)
        st = check_stores(sh[0], sh[2], sh[3], sh[4])
        print(sh, "out-of-bounds loads:", b, " store coverage errors:", st)
        fails += b + st
    sys.exit(1 if fails else 0)
