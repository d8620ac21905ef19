#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${1:-warp}; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_library_ops.py -m gpu -k "warp or jit or export" -x -q --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; tail -3 "$OUT/pytest.log"; [ $rc -eq 0 ] || { grep -E "Error|assert" "$OUT/pytest.log" | head -20; exit $rc; }
bash scripts/gpu_ab_ops.sh "$1" warp2,warp1 bin/ab/lib_warp8.so bin/ab/lib_wtile.so
