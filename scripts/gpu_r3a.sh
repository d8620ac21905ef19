#!/bin/bash
# Round 3, first GPU call: the new / changed GPU tests, then the store-pattern micro-benchmark.
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r3a; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_autocast.py tests/test_model_isolation.py tests/test_gpu_v4.py \
  tests/test_model_demo.py "tests/test_gpu_parity.py::test_fused_volume_free_multipass_exact_segments" \
  "tests/test_gpu_parity.py::test_warp_strided_and_errors" "tests/test_gpu_parity.py::test_cfg2_inner_product_full_size" \
  -m gpu -v -s --timeout 300 --timeout-method thread -p no:cacheprovider > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -40 "$OUT/pytest.log" | grep -E "passed|failed|Error|max \||engine" 
hipcc -O3 --offload-arch=gfx950 scripts/micro/store_patterns.hip -o /tmp/store_patterns > "$OUT/build.log" 2>&1 || exit 2
timeout -k 10 120 /tmp/store_patterns > "$OUT/store_patterns.log" 2>&1 || exit 3
cat "$OUT/store_patterns.log"
exit $rc
