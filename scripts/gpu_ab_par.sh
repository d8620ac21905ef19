#!/bin/bash
# A/B timing of library builds plus a parity check of the newest one:
#   bash scripts/gpu_ab_par.sh TAG OPS "pytest -k expr" lib1.so lib2.so ...
# The LAST lib is copied in as realtime_stereo_matcher_amd/libstereocv.so for the tests.
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=$1; OPS=$2; K=$3; shift 3
OUT=gpurun_out/$TAG; mkdir -p "$OUT"; export TMPDIR=/tmp
for lib in "$@"; do last=$lib; done
cp "$last" realtime_stereo_matcher_amd/libstereocv.so
if [ -n "$K" ]; then
  timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
    -p no:cacheprovider -k "$K" > "$OUT/pytest.log" 2>&1
  rc=$?; tail -3 "$OUT/pytest.log"
  if [ $rc -ne 0 ]; then grep -E "FAILED|Error|assert" "$OUT/pytest.log" | head -20; exit $rc; fi
fi
for r in 1 2; do
  for lib in "$@"; do
    STEREOCV_LIB=$lib timeout -k 10 240 python -u scripts/ab_time.py --ops "$OPS" >> "$OUT/ab.jsonl" 2>> "$OUT/ab.err" || { echo "failed on $lib"; tail -5 "$OUT/ab.err"; exit 2; }
  done
done
python3 - "$OUT/ab.jsonl" <<'PY'
import json, sys, collections
rows = [json.loads(l) for l in open(sys.argv[1])]
d = collections.defaultdict(list)
for r in rows: d[(r["op"], r["tag"])].append(r["median_us"])
for (op, tag), v in sorted(d.items()): print(f"{op:16s} {tag:12s} " + " ".join(f"{x:9.1f}" for x in v))
PY
