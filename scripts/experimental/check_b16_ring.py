#!/usr/bin/env python3
"""Host replay of band_b16's epilogue shear (csrc/ip_b16.hip) for every block count TB it is built
for: each lane's 4 accumulator elements of block t go to the 2-slot ring of 16 d x 16 x chunks,
each chunk is read back (lane l: row l >> 2, pixels 4 (l & 3) ..) right after the block that
completes it.  Checks, in the wave's LDS program order, that every readout sees exactly the
cell (d, x) it stores and that no write lands on a cell of a chunk still to be read; reports
the bank-conflict degree of the ring writes (ds_write_b32: 32-bank halves) and readouts
(ds_read_b128 lane groups) and of the 16x16x32 fragment reads on band_h2's plane swizzle."""
import sys

SLOT = 1024


def swz(r, h):
    return ((r ^ ((r >> 2) & 3)) << 5) + ((h ^ ((r >> 4) & 1)) << 4)


READ128_GROUPS = [[0, 1, 2, 3, 12, 13, 14, 15] + list(range(20, 28)),
                  list(range(4, 12)) + [16, 17, 18, 19, 28, 29, 30, 31]]
READ128_GROUPS += [[l + 32 for l in g] for g in READ128_GROUPS]


def conflicts_read128(addrs):
    worst = 1
    for g in READ128_GROUPS:
        banks = {}
        for l in g:
            for b in range(4):
                k = (addrs[l] // 4 + b) % 64
                banks[k] = banks.get(k, 0) + 1
        worst = max(worst, max(banks.values()))
    return worst


def conflicts_write32(addrs):
    worst = 1
    for half in (range(0, 32), range(32, 64)):
        banks = {}
        for l in half:
            k = (addrs[l] // 4) % 32
            banks[k] = banks.get(k, 0) + 1
        worst = max(worst, max(banks.values()))
    return worst


def replay(TB):
    ring = {}  # byte address -> (d_local, x_local)
    wmax = rmax = 1
    for t in range(TB - 1, -1, -1):
        a = TB - 2 - t
        for i in range(4):
            addrs = []
            for l in range(64):
                xl, lg = l & 15, l >> 4
                u = xl - 4 * lg - i
                w = 64 * (u & 15) + 4 * xl + (SLOT if u >= 0 else 0)
                if a & 1:
                    w ^= SLOT
                d = 16 * (a + 1) + u  # local disparity of (R row 4 lg + i, pixel xl) in block t
                ring[w] = (d, xl)
                addrs.append(w)
            wmax = max(wmax, conflicts_write32(addrs))
        if a >= 0:
            addrs = []
            for l in range(64):
                r = (a & 1) * SLOT + 16 * l
                addrs.append(r)
                for e in range(4):
                    want = (16 * a + (l >> 2), 4 * (l & 3) + e)
                    got = ring.get(r + 4 * e)
                    if got != want:
                        return f"TB={TB} block {t} lane {l}: readout {got} != {want}"
            rmax = max(rmax, conflicts_read128(addrs))
    # fragment reads of 16x16x32 on the plane swizzle, for every block base (multiples of 16)
    fmax = 1
    for base in range(0, 512, 16):
        addrs = [swz(base + (l & 15), (l >> 4) & 1) + ((l >> 5) * 1 << 20) for l in range(64)]
        fmax = max(fmax, conflicts_read128(addrs))
    return f"TB={TB}: shear ok; ring writes {wmax}-way, readouts {rmax}-way, fragment reads {fmax}-way"


def main():
    bad = False
    for TB in (3, 5, 9, 13):
        msg = replay(TB)
        print(msg)
        bad |= "!=" in msg
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
