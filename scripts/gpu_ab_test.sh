#!/bin/bash
# Filtered GPU parity tests on the in-tree library, then a same-box A/B of library builds:
#   bash scripts/gpu_ab_test.sh TAG "pytest -k expr" OPS lib1.so lib2.so ...
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=$1; K=$2; OPS=$3; shift 3
OUT=gpurun_out/$TAG; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -k "$K" -x -q --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; tail -3 "$OUT/pytest.log"; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_ab_ops.sh "$TAG" "$OPS" "$@"
