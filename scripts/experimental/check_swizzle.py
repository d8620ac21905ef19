#!/usr/bin/env python3
"""Check the LDS chunk swizzle of csrc/ip_mfma.hip against gfx950 bank rules
(MI355X_MICROARCH.md §LDS): fragment reads (ds_read_b128, four 16-lane groups, 64 banks)
must be conflict-free; staging writes (ds_write_b128, 8 contiguous lanes, 32 banks) <= 2-way."""
F = [0, 2, 3, 1]


def addr(r, ch):
    return r * 64 + 16 * (ch ^ F[(r >> 2) & 3])


GROUPS = [list(range(0, 4)) + list(range(12, 16)) + list(range(20, 28)),
          list(range(4, 12)) + list(range(16, 20)) + list(range(28, 32))]
GROUPS += [[g + 32 for g in grp] for grp in GROUPS]


def main():
    worst_r = 1
    for base in range(0, 64, 16):
        for grp in GROUPS:
            slots = [(addr(base + (l & 15), l >> 4) // 16) % 16 for l in grp]
            worst_r = max(worst_r, max(slots.count(s) for s in slots))
    worst_w = 1
    for p in range(4):  # item i -> (chunk i & 3, pixel rows 4*(i >> 2) + p)
        for start in range(0, 512, 8):
            sl = [(addr(4 * (i >> 2) + p, i & 3) // 16) % 8 for i in range(start, start + 8)]
            worst_w = max(worst_w, max(sl.count(s) for s in sl))
    print(f"fragment reads: {worst_r}-way, staging writes: {worst_w}-way")
    assert worst_r == 1 and worst_w <= 2


if __name__ == "__main__":
    main()
