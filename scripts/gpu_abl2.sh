#!/bin/bash
# band_h2 ablation timings at 8 cfg2 pairs per launch: 0 full, 49 memory only (no MFMA, no
# staging writes, no shear), 51 = 49 + loads from one line, 6 = no HBM loads and no stores.
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${1:-abl2}; mkdir -p "$OUT"
for r in 1 2 3; do for ab in 0 49 51 6; do
  echo -n "ablate=$ab: "; timeout -k 10 60 bin/stamps/ip_ab$ab 192 h2 8 > "$OUT/ab.tmp" 2>&1 || { cat "$OUT/ab.tmp"; exit 5; }
  head -1 "$OUT/ab.tmp"
done; done
