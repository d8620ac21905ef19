"""CPU checks of bench.py's record plumbing: the committed PMC traffic it quotes belongs to the
same workload (config, pipeline, N=1, default pairs per launch), and the evidence files it
points to carry the gfx950-corrected byte counts."""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def _args(config, pipeline="separate", **kw):
    d = dict(config=config, pipeline=pipeline, algo="auto", batch=None, chunk=None)
    d.update(kw)
    return argparse.Namespace(**d)


def test_committed_traffic_matches_workload():
    for config, pipeline in (("cfg2", "separate"), ("cfg2", "fused-novolume"), ("cfg3", "separate"),
                             ("cfg4", "separate"), ("cfg5", "separate"), ("cfg5", "interweave")):
        a = _args(config, pipeline)
        rel = os.path.join(ROOT, "profiles", bench.EVIDENCE_ROUND, bench.evidence_name(a), "pmc.json")
        if not os.path.exists(rel):
            continue
        kname = bench.kernel_name(bench.CONFIGS[config], pipeline, "auto")
        t = bench.committed_traffic(a, kname)
        if t["traffic"] is None:
            # the committed counter run measured another kernel (the default changed since):
            # the bench quotes nothing rather than another kernel's bytes
            with open(rel) as f:
                ks = json.load(f)["kernels"]
            assert not any(k.startswith(kname.split(" ")[0]) for k in ks), (config, pipeline)
            continue
        assert bench.evidence_name(a) in t["traffic_source"]
        alg = bench.pair_bytes(bench.CONFIGS[config], pipeline) * bench.CONFIGS[config]["chunk"]
        # counted HBM bytes within a few percent of the algorithmic bytes of one launch (cfg4's
        # D = 256 runs in two passes of 128 that each read the features: up to +11 %)
        assert 0.95 * alg <= t["traffic"] <= 1.15 * alg, (config, pipeline, t["traffic"], alg)


def test_committed_traffic_not_quoted_for_other_workloads():
    k = bench.kernel_name(bench.CONFIGS["cfg2"], "separate", "auto")
    assert bench.committed_traffic(_args("cfg2"), k, world=8)["traffic"] is None
    assert bench.committed_traffic(_args("cfg2", chunk=4), k)["traffic"] is None
    assert bench.committed_traffic(_args("cfg2", algo="valu"), k)["traffic"] is None


def test_evidence_summary_consistent():
    path = os.path.join(ROOT, "profiles", bench.EVIDENCE_ROUND, "summary.json")
    if not os.path.exists(path):
        return
    with open(path) as f:
        summary = json.load(f)
    for name, row in summary.items():
        # the rocprofv3 average of the dominant kernel agrees with the HIP events of the same
        # profiled process (round 6 records it; earlier rounds compared with the separate bench
        # process, whose volume buffers may be mapped at another speed, profiles/r05/placement/)
        bench_us = row.get("profiled_bench_avg_kernel_us", row["bench_avg_kernel_us"])
        assert abs(row["rocprof_avg_us"] / bench_us - 1) < 0.1, name
        if "mfma_busy_frac" in row:
            assert 0.0 < row["mfma_busy_frac"] < 1.0
