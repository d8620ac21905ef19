#!/usr/bin/env python3
"""Host-side bounds check of the warp-specialised band kernel's stage-wave loads
(csrc/ip_ws.hip, load()): replays every lane's addresses for every pipeline step of every
workgroup and asserts they stay inside the feature tensor.  Run before any GPU launch of a
changed indexing scheme:  python scripts/check_ws_bounds.py"""
import sys


def geo(D):
    npass = -(-D // 192)
    pw = -(-D // npass)
    T = 2 if pw <= 32 else 3 if pw <= 64 else 5 if pw <= 128 else 7
    DMAX = 32 * (T - 1)
    RW = 128 + DMAX
    ROWS = RW + 128
    return T, DMAX, RW, ROWS // 4, npass, pw


def check(N, C, H, W, D, ncu=256):
    T, DMAX, RW, GROUPS, npass, pw = geo(D)
    ITEMS = 2 * GROUPS
    tiles = -(-W // 128)
    nwork = tiles * H * N * npass
    nwg = max(8, (min(nwork, ncu) + 7) // 8 * 8)
    q, rr = nwork >> 3, nwork & 7
    cs, hs, ns = H * W, W, C * H * W   # contiguous strides
    numel = N * ns
    nks = -(-C // 16)
    bad = 0
    for blk in range(nwg):
        grp, gi, gsz = blk & 7, blk >> 3, nwg >> 3
        wbeg = grp * (q + 1) if grp < rr else rr * (q + 1) + (grp - rr) * q
        wend = wbeg + q + (1 if grp < rr else 0)
        if wbeg + gi >= wend:
            continue
        nitems = (wend - (wbeg + gi) + gsz - 1) // gsz
        S = nitems * nks
        for s in range(S + 4):
            ss = min(s, S - 1)
            it, ks = divmod(ss, nks)
            w = wbeg + gi + it * gsz
            pas, rest = w % npass, w // npass
            tile, row = rest % tiles, rest // tiles
            y, n = row % H, row // H
            x0, dp = tile * 128, pas * pw
            Dp = min(pw, D - dp)
            Tn = 1 + (Dp - 1 + 31) // 32
            js = x0 - dp - 32 * (Tn - 1)
            for sq in range(256):
                h = min(sq // GROUPS, 1)
                g = min(sq - h * GROUPS, GROUPS - 1)
                active = sq < ITEMS
                isR = 4 * g < RW
                c0 = ks * 16 + 8 * h
                px = js + 4 * g if isR else x0 + 4 * g - RW
                okp = active and 0 <= px < W
                base = n * ns + y * hs + (px if okp else 0) + min(c0, C - 1) * cs
                for kk in range(8):
                    off = kk if C % 16 == 0 else min(kk, max(C - 1 - c0, 0))
                    e = base + off * cs
                    if e < 0 or e + 4 > numel:
                        bad += 1
    return bad


if __name__ == "__main__":
    shapes = [(1, 32, 64, 128, 24), (1, 64, 2, 200, 192), (1, 32, 2, 100, 300), (1, 8, 2, 64, 64),
              (2, 20, 3, 260, 100), (1, 48, 2, 132, 33), (1, 16, 1, 1000, 256), (1, 7, 2, 36, 40),
              (1, 64, 2, 960, 192), (1, 33, 2, 512, 31), (1, 64, 6, 960, 192), (2, 17, 3, 64, 24)]
    fails = 0
    for sh in shapes:
        b = check(*sh)
        print(sh, "out-of-bounds loads:", b)
        fails += b
    sys.exit(1 if fails else 0)
