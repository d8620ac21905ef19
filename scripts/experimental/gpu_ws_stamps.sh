#!/bin/bash
# Per-role phase stamps of band_h2ws (bin/stamps/ws_stamps*, built by the hipcc lines in
# scripts/ws_stamps.hip).   bash scripts/gpu_ws_stamps.sh TAG bin1 bin2 ...
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/$1; shift; mkdir -p "$OUT"
for b in "$@"; do
  echo "== $b"
  timeout -k 10 60 "$b" > "$OUT/$(basename "$b").log" 2>&1 || { cat "$OUT/$(basename "$b").log"; exit 3; }
  cat "$OUT/$(basename "$b").log"
done
