#!/bin/bash
# Full -m gpu suite, then same-box A/B of the fused passes: the library (role-split FUSE 1 / 2)
# against var_so/nors.so (-DSMCV_NO_RS_FUSE: band_h2db FUSE 1 / band_h2 FUSE 2).
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${1:-fuse}; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1 || { tail -30 "$OUT/gpu_tests.log"; exit 3; }
tail -2 "$OUT/gpu_tests.log"
bash scripts/gpu_ab_var.sh ${1:-fuse} "cfg2_fused,cfg2_fused_nv,cfg4_fused_nv" "default nors"
