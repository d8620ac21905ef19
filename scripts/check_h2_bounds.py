#!/usr/bin/env python3
"""Host-side replay of the band kernels' indexing (csrc/ip_h2.hip; the rings of csrc/ip_h2db.hip
and csrc/ip_rs.hip), run before any GPU launch of a changed indexing scheme:
    python scripts/check_h2_bounds.py

1. every stage lane's feature loads and L2 touches, for every step of every workgroup, stay
   inside the feature tensor and inside the lane's channel group -- for the (N, D, H, W) kernels
   (G = 1) and the groupwise kernel (G groups of C/G channels); the grid is 2 workgroups per CU;
2. each wave's epilogue ring: every write and read stays inside the wave's ring, and after
   block a the ring holds chunk a exactly -- the accumulator element of band cell
   (dl = 32 a + row, x) -- in both layouts (NDHW [slot][d][x], NGHWD [x][d circular]); the ring
   writes are bank-conflict free per 32-lane half (ds_write_b32) and the readouts per
   ds_read_b128 lane group (MI355X_MICROARCH.md, LDS table);
3. every stored volume offset lies inside the volume and every cell (d < D, x < W) of every
   (n, g, y) row is stored exactly once over the whole grid, in both layouts, and the fused
   kernel stores every disparity exactly once."""
import sys

import numpy as np

KXT, KSLOT = 128, 4096
_G1 = list(range(0, 4)) + list(range(12, 16)) + list(range(20, 28))
_G2 = list(range(4, 12)) + list(range(16, 20)) + list(range(28, 32))
B128_GROUPS = [_G1, _G2, [l + 32 for l in _G1], [l + 32 for l in _G2]]


def geo(D):
    npass = -(-max(D, 1) // 192)
    pw = (-(-max(D, 1) // npass) + 3) // 4 * 4
    T = 2 if pw <= 32 else 3 if pw <= 64 else 5 if pw <= 128 else 7
    DMAX = 32 * (T - 1)
    RW = KXT + DMAX
    ROWS = RW + KXT
    return T, DMAX, RW, ROWS // 4, npass, pw


def work_lists(N, G, H, W, D, ncu):
    """Mirror of the kernels' Sched (band_common.h): XCD-grouped segment ranges, the D passes of
    a segment consecutive items of one workgroup."""
    T, DMAX, RW, GROUPS, npass, pw = geo(D)
    tiles = -(-W // KXT)
    nwork = tiles * H * N * G * npass
    nwg = max(8, (min(nwork, 2 * ncu) + 7) // 8 * 8)
    nseg = nwork // npass
    q, rr = nseg >> 3, nseg & 7
    for blk in range(nwg):
        grp, gi, gsz = blk & 7, blk >> 3, nwg >> 3
        sbeg = grp * (q + 1) if grp < rr else rr * (q + 1) + (grp - rr) * q
        scnt = q + (1 if grp < rr else 0)
        if gi >= scnt:
            continue
        nitems = ((scnt - gi + gsz - 1) // gsz) * npass
        yield blk, [witem(sbeg, scnt, gi, gsz, npass, it) for it in range(nitems)]


def witem(sbeg, scnt, gi, gsz, npass, i):
    """Mirror of Sched::item(): complete aligned 8-segment blocks rotated by the round."""
    si, p = divmod(i, npass)
    j = gi + si * gsz
    b = j & ~7
    rot = gsz % 8 == 0
    return (sbeg + ((b | ((j + si) & 7)) if rot and b + 8 <= scnt else j)) * npass + p


def decode(w, tiles, npass, G, H, D, pw, DMAX):
    pas, r1 = w % npass, w // npass
    tile, r2 = r1 % tiles, r1 // tiles
    g, row = r2 % G, r2 // G
    y, n = row % H, row // H
    x0, dp = tile * KXT, pas * pw
    return n, y, g, x0, dp, min(pw, D - dp), x0 - dp - DMAX


def check_loads(N, C, H, W, D, G=1, ncu=256):
    T, DMAX, RW, GROUPS, npass, pw = geo(D)
    tiles = -(-W // KXT)
    ITEMS = 2 * GROUPS
    cpg = C // G
    cs, hs, ns = H * W, W, C * H * W
    numel = N * ns
    nks = -(-cpg // 16)
    bad = 0
    for blk, items in work_lists(N, G, H, W, D, ncu):
        for w in items:
            n, y, g, x0, dp, Dp, js = decode(w, tiles, npass, G, H, D, pw, DMAX)
            for ks in range(nks):
                for sq in range(256):
                    h = min(sq // GROUPS, 1)
                    gr = min(sq - h * GROUPS, GROUPS - 1)
                    active = sq < ITEMS
                    isR = 4 * gr < RW
                    cl = ks * 16 + 8 * h
                    px = js + 4 * gr if isR else x0 + 4 * gr - RW
                    okp = active and 0 <= px < W
                    if okp and px % 4:
                        bad += 1  # 4-pixel groups must be aligned
                    rowb = n * ns + y * hs
                    base = rowb + (px if okp else 0) + (g * cpg + min(cl, cpg - 1)) * cs
                    lim = 7 if cpg % 16 == 0 else min(max(cpg - 1 - cl, 0), 7)
                    for kk in range(8):
                        chn = g * cpg + min(cl, cpg - 1) + min(kk, lim)
                        e = base + min(kk, lim) * cs
                        if e < 0 or e + 4 > numel or not g * cpg <= chn < (g + 1) * cpg:
                            bad += 1
                    # the L2 touch of this step: channel cl + (gr & 7) of the same pixel group
                    ct = cl + (gr & 7)
                    if active and 0 <= px < W and ct < cpg:
                        e = rowb + px + (g * cpg + ct) * cs
                        if e < 0 or e + 1 > numel:
                            bad += 1
    return bad


def ring_addr(layout, a, lr, hh, ci):
    u = lr - 4 * hh
    if layout == 0:
        wbase = 4 * lr + 128 * u
        sa, sb = (a + 3) % 3, (a + 4) % 3
        if sa != 2:
            return wbase + sb * KSLOT - ci * 128
        return wbase + 3 * KSLOT - ci * 128 - (3 * KSLOT if u >= ci else 0)
    wbase = 384 * lr + 4 * u
    bp = 32 * ((a + 4) % 3)
    if bp:
        return wbase + 4 * (bp - ci)
    return wbase + 4 * (96 - ci) - (384 if u >= ci else 0)


def read_addr(layout, a, lane, qq):
    """(byte address of the 16-B read, pixel of element 0, local disparity of element 0,
    pixel step, disparity step) of lane's read qq of chunk a"""
    rl, cl = lane >> 3, lane & 7
    if layout == 0:
        return (a % 3) * KSLOT + (8 * qq + rl) * 128 + 16 * cl, 4 * cl, 32 * a + 8 * qq + rl, 1, 0
    return (8 * qq + rl) * 384 + (a % 3) * 128 + 16 * cl, 8 * qq + rl, 32 * a + 4 * cl, 0, 1


def check_shear(T, layout):
    """One wave's ring over a whole segment; returns (mismatches, conflicted lane groups)."""
    DMAX = 32 * (T - 1)
    ring = {}
    bad = conflicts = 0
    for a in range(-1, T - 1):
        t = T - 2 - a
        for i in range(16):
            ci = (i & 3) + 8 * (i >> 2)
            for hh in range(2):
                banks = set()
                for lr in range(32):
                    addr = ring_addr(layout, a, lr, hh, ci)
                    if not 0 <= addr < 3 * KSLOT or addr % 4:
                        bad += 1
                        continue
                    banks.add((addr // 4) % 32)
                    ring[addr] = (t, ci + 4 * hh, lr)  # block, R row in the block, L column
                conflicts += len(banks) != 32
        if a < 0:
            continue
        for qq in range(4):
            for grp in B128_GROUPS:
                banks = set()
                for lane in grp:
                    addr0 = read_addr(layout, a, lane, qq)[0]
                    banks |= {(addr0 // 4 + e) % 64 for e in range(4)}
                conflicts += len(banks) != 64
            for lane in range(64):
                addr0, x, dl, dx, dd = read_addr(layout, a, lane, qq)
                if addr0 % 16 or not 0 <= addr0 < 3 * KSLOT:
                    bad += 1
                    continue
                for e in range(4):
                    src = ring.get(addr0 + 4 * e)
                    if src is None:
                        bad += 1
                        continue
                    t2, jj, x2 = src
                    # wave-relative: L column x2, R row 32 t2 + jj, the window starting DMAX
                    # before the wave's first pixel: d_l = x2 - (32 t2 + jj) + DMAX
                    if x2 != x + e * dx or x2 - 32 * t2 - jj + DMAX != dl + e * dd:
                        bad += 1
    return bad, conflicts


def check_stores(N, H, W, D, G=1, layout=0, ncu=256):
    T, DMAX, RW, GROUPS, npass, pw = geo(D)
    tiles = -(-W // KXT)
    size = N * G * H * W * D
    hits = np.zeros(size, np.int32)
    disp = np.zeros(N * H * W, np.int32)
    dq = layout == 0 or D % 4 == 0
    bad = 0

    def hit(o, cnt):
        nonlocal bad
        if o < 0 or o + cnt > size:
            bad += 1
            return
        hits[o:o + cnt] += 1

    for blk, items in work_lists(N, G, H, W, D, ncu):
        for w in items:
            n, y, g, x0, dp, Dp, js = decode(w, tiles, npass, G, H, D, pw, DMAX)
            fast = dq and x0 + KXT <= W and Dp == DMAX
            for wave in range(4):
                x0w = x0 + 32 * wave
                for a in range(T - 1):
                    for lane in range(64):
                        rl, cl = lane >> 3, lane & 7
                        for qq in range(4):
                            if layout == 0:
                                dl = 32 * a + 8 * qq + rl
                                if fast or (dl < Dp and x0w + 4 * cl < W):
                                    hit(((n * D + dp + dl) * H + y) * W + x0w + 4 * cl, 4)
                            else:
                                pix = x0w + 8 * qq + rl
                                d0 = 32 * a + 4 * cl
                                o = (((n * G + g) * H + y) * W + pix) * D + dp + d0
                                if fast or (pix < W and d0 + 4 <= Dp and dq):
                                    hit(o, 4)
                                elif pix < W:
                                    for e in range(4):
                                        if d0 + e < Dp:
                                            hit(o + e, 1)
                if layout == 0 and npass == 1:  # the fused kernel's disparities: lanes rl == 0
                    for cl in range(8):
                        x = x0w + 4 * cl
                        for e in range(4):
                            if x + e < W:
                                disp[(n * H + y) * W + x + e] += 1
    bad += int((hits != 1).sum())
    if layout == 0 and npass == 1:
        bad += int((disp != 1).sum())
    return bad


def check_rs_ring(T):
    """band_rs's ring (csrc/ip_rs.hip): T-1 chunks of 4 KB per compute wave, chunk m at m*4096;
    block t (a = T-2-t) writes element i of lane (lr, hh) -- local disparity 32 (a+1) + u - c_i,
    u = lr - 4 hh -- at wb + (a+1) 4096 - 128 c_i - 512 (wb = 512 + 128 u + 4 lr), except the
    folded blocks T-1 (a = -1, into chunk 0) and 0 (a = T-2, into chunk T-2):
    ((32768 + 128 u + 4 lr - 128 c_i) & 4095) + (0 | (T-2) 4096).  Written in the order T-1, 0,
    1, ..., T-2, every cell (chunk m, row r, pixel lr) must end up holding local disparity
    32 m + r; every address stays in [0, (T-1) 4096); ds_write_b32 lane groups (0-31, 32-63) are
    conflict free; the readouts (rows 8 qq + rl, 16 B at 16 cl) stay inside their chunk.
    Returns (wrong cells, out-of-range accesses, conflicted lane groups)."""
    size = (T - 1) * KSLOT
    ring = {}
    oob = conf = 0
    for t in [T - 1] + list(range(T - 1)):
        a = T - 2 - t
        for i in range(16):
            ci = (i & 3) + 8 * (i >> 2)
            addrs = []
            for lane in range(64):
                lr, hh = lane & 31, lane >> 5
                u = lr - 4 * hh
                if a in (-1, T - 2):
                    ad = ((32768 + 128 * u + 4 * lr - 128 * ci) & 4095) + (0 if a == -1 else (T - 2) * KSLOT)
                else:
                    ad = (512 + 128 * u + 4 * lr) + (a + 1) * KSLOT - 128 * ci - 512
                if not 0 <= ad < size:
                    oob += 1
                    continue
                ring[ad] = 32 * (a + 1) + u - ci  # the element's local disparity
                addrs.append((lane, ad))
            for half in (0, 1):
                banks = [(ad // 4) % 32 for ln, ad in addrs if ln >> 5 == half]
                if len(set(banks)) != len(banks):
                    conf += 1
    wrong = 0
    for m in range(T - 1):
        for r in range(32):
            for lr in range(32):
                if ring.get(m * KSLOT + r * 128 + 4 * lr) != 32 * m + r:
                    wrong += 1
    for m in range(T - 1):
        for lane in range(64):
            rl, cl = lane >> 3, lane & 7
            for qq in range(4):
                ad = m * KSLOT + qq * 1024 + rl * 128 + 16 * cl
                if not (m * KSLOT <= ad and ad + 16 <= (m + 1) * KSLOT):
                    oob += 1
    return wrong, oob, conf


def check_h2db_ring(T):
    """band_h2db's epilogue ring (csrc/ip_h2db.hip): 2 slots x 4 KB per wave, chunk m in slot m & 1;
    element i of lane (lr, hh) in block t (a = T-2-t) at yi = 4096 + 128 (u - c_i) + 4 lr, XOR
    4096 when a is odd.  Replays the epilogue's order -- for t = T-1 .. 0: write block t, (store
    chunk a-1 from registers), read chunk a -- and checks every read cell of chunk a holds local
    disparity 32 a + row, every access stays in [0, 8192), the writes are conflict free per
    32-lane half.  Returns (wrong cells, out-of-range accesses, conflicted lane groups)."""
    ring = {}
    wrong = oob = conf = 0
    for t in range(T - 1, -1, -1):
        a = T - 2 - t
        for i in range(16):
            ci = (i & 3) + 8 * (i >> 2)
            banks = {0: [], 1: []}
            for lane in range(64):
                lr, hh = lane & 31, lane >> 5
                u = lr - 4 * hh
                yi = 4096 + 128 * (u - ci) + 4 * lr
                ad = (yi ^ 4096) if (a & 1) else yi
                if not 0 <= ad < 2 * KSLOT:
                    oob += 1
                    continue
                ring[ad] = 32 * (a + 1) + u - ci
                banks[hh].append((ad // 4) % 32)
            conf += sum(len(set(b)) != len(b) for b in banks.values())
        if a >= 0:
            for r in range(32):
                for x in range(32):
                    if ring.get((a & 1) * KSLOT + r * 128 + 4 * x) != 32 * a + r:
                        wrong += 1
    return wrong, oob, conf


def check_rs_gw_ring(T):
    """band_rs's groupwise ring (GW): [32 px][DMAX d] fp32 per compute wave (RS = 4 DMAX bytes
    per pixel); element i of lane (lr, hh), block t (a = T-2-t) at wbg + 128 (a+1) - 4 c_i - 16
    with wbg = 16 + lr (RS + 4) - 16 hh, the straddling blocks at lr RS + 4 ((u - c_i) mod 32)
    (+ 128 (T-2) for block 0).  Written T-1, 0, ..., T-2: every cell (px, d) must hold local
    disparity d; accesses stay in [0, 32 RS); ds_write_b32 32-lane groups conflict free."""
    DMAX = 32 * (T - 1)
    RS = 4 * DMAX
    ring = {}
    oob = conf = 0
    for t in [T - 1] + list(range(T - 1)):
        a = T - 2 - t
        for i in range(16):
            ci = (i & 3) + 8 * (i >> 2)
            banks = {0: [], 1: []}
            for lane in range(64):
                lr, hh = lane & 31, lane >> 5
                u = lr - 4 * hh
                if a in (-1, T - 2):
                    ad = lr * RS + 4 * ((u - ci) & 31) + (0 if a == -1 else 128 * (T - 2))
                else:
                    ad = 16 + lr * (RS + 4) - 16 * hh + 128 * (a + 1) - 4 * ci - 16
                if not 0 <= ad < 32 * RS:
                    oob += 1
                    continue
                ring[ad] = (lr, 32 * (a + 1) + u - ci)
                banks[hh].append((ad // 4) % 32)
            conf += sum(len(set(b)) != len(b) for b in banks.values())
    wrong = sum(ring.get(px * RS + 4 * d) != (px, d) for px in range(32) for d in range(DMAX))
    return wrong, oob, conf


if __name__ == "__main__":
    fails = 0
    for T in (3, 5, 7):
        w, o, c = check_rs_gw_ring(T)
        print(f"band_rs groupwise ring T={T}: wrong cells {w}, out-of-range {o}, conflicted lane groups {c}")
        fails += w + o + c
    for T in (3, 5, 7):
        w, o, c = check_h2db_ring(T)
        print(f"band_h2db ring T={T}: wrong cells {w}, out-of-range {o}, conflicted lane groups {c}")
        fails += w + o + c
    for T in (3, 5, 7):
        w, o, c = check_rs_ring(T)
        print(f"band_rs ring T={T}: wrong cells {w}, out-of-range {o}, conflicted lane groups {c}")
        fails += w + o + c
    for layout in (0, 1):
        for T in (2, 3, 5, 7):
            b, c = check_shear(T, layout)
            print(f"shear {'NDHW ' if layout == 0 else 'NGHWD'} T={T}: mismatches {b}, "
                  f"conflicted lane groups {c}")
            fails += b + c
    shapes = [(1, 32, 64, 128, 24), (1, 64, 2, 200, 192), (1, 32, 2, 100, 300), (1, 8, 2, 64, 64),
              (2, 20, 3, 260, 100), (1, 48, 2, 132, 33), (1, 16, 1, 1000, 256), (1, 7, 2, 36, 40),
              (1, 64, 2, 960, 192), (1, 33, 2, 512, 31), (1, 64, 3, 960, 192), (2, 17, 3, 64, 24),
              (1, 16, 2, 1920, 256), (1, 8, 2, 64, 201), (1, 4, 3, 20, 7)]
    for sh in shapes:
        b = check_loads(*sh)
        st = check_stores(sh[0], sh[2], sh[3], sh[4])
        print(sh, "out-of-bounds loads:", b, " store coverage errors:", st)
        fails += b + st
    gshapes = [(1, 32, 3, 260, 100, 4), (2, 48, 2, 132, 33, 3), (1, 256, 2, 960, 192, 8),
               (1, 16, 2, 64, 256, 2), (1, 24, 2, 200, 40, 8), (1, 40, 2, 128, 7, 5)]
    for N, C, H, W, D, G in gshapes:
        b = check_loads(N, C, H, W, D, G)
        st = check_stores(N, H, W, D, G, layout=1)
        print((N, C, H, W, D, G), "groupwise out-of-bounds loads:", b, " store coverage errors:", st)
        fails += b + st
    sys.exit(1 if fails else 0)
