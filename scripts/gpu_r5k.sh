#!/bin/bash
# Round 5: the whole GPU suite on the band_sl build (AUTO volume = band_rs, fused = band_sl) + smoke
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r5k; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests > "$OUT/gpu_tests.log" 2>&1
rc=$?; echo "gpu tests rc=$rc"; grep -E "passed|failed" "$OUT/gpu_tests.log" | tail -2; grep -E "^FAILED" "$OUT/gpu_tests.log" | head -30
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1; echo "smoke rc=$?"; tail -2 "$OUT/smoke.log"
