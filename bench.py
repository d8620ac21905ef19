#!/usr/bin/env python3
"""Headline benchmark: stereo pairs/s of the cost-volume + disparity-regression hot path.

Workloads (--config, BASELINE.json configs[1..4]; inputs synthetic and already resident in HBM):
  cfg2 (default)  1x64x540x960 fp32 features (1/4-res KITTI), inner-product volume D=192
                  (TorchInnerProductCost, cost_volume/inner_product.py:11-42) + soft-argmin
                  (model/mobile_disp_net_c.py:208-220).  Global batch 32, split 32/k over k GPUs
                  (strong scaling).
  cfg3            1x256x540x960 bf16, groupwise volume G=8 D=192, fp32 (N,G,H,W,D) out
                  (TorchGroupwiseCost, cost_volume/groupwise.py:24-56).  4 pairs per GPU, one launch.
  cfg4            16x1080x1920 fp32 per pair, correlation volume D=256 (mean over C,
                  model/mobile_disp_net_c.py:188-205) + soft-argmin; global batch 32 split 32/k
                  (strong scaling, configs[3] / mobile_disp_net_c.py:365-367).
  cfg5            1x128x540x960 fp16, concatenate volume D=64 (cost_volume/concatenate.py:11-41);
                  --pipeline interweave: the v4 shifted interweave volume (mobile_stereo_net_v4.py:
                  443-461) instead.  One pair per GPU.

A STEP is one pass of the hot path over the rank's pairs, launched in chunks of --chunk pairs,
plus -- for N>1 on the regression configs -- the RCCL gather of the per-pair disparities to rank 0
(the only collective).  Pipelines for cfg2: ``separate`` (volume kernel, then the regression
kernel), ``fused`` (one band-kernel pass writes the volume and its soft-argmin), ``fused-novolume``
(the same pass without writing the volume).

    python bench.py [--config cfgN] [--gpus N] [--steps K] [--warmup W] [--pipeline P] ...
    torchrun --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N ...

Rank 0 prints ONE JSON line: ``value`` = pairs processed by all ranks / max-over-ranks wall time of
the K timed steps.  ``roofline`` is the dominant kernel (the volume build, or the fused pass) timed
with HIP events on its launch stream inside the timed region: algorithmic bytes of all its timed
launches / their summed duration.  ``numerics`` compares sampled output rows with the fp64 oracle
after the timed region (checker only).  ``cpu_baseline`` times the eager CPU port of the
reference's op sequence (oracle/torch_port.py, validated against the reference itself by
tests/golden/time_ref_vs_port.py) on the host cores, on a bounded sample (rank 0, N=1 only).
"""
import argparse
import json
import math
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from realtime_stereo_matcher_amd import functional as F  # noqa: E402
from realtime_stereo_matcher_amd.distributed import env_rank, gather_disparities, shard_range  # noqa: E402

METRIC = "stereo pairs/sec + ms/pair, KITTI-res D=192 cost-volume+regression, 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0     # MI355X HBM3E (MI355X_MICROARCH.md, chip-level parameters)
MFMA_BF16_PEAK_TF = 2500.0  # dense bf16/fp16 MFMA (no sparsity)
ARITH_SPLIT = ("fp32 features as a per-item power-of-two scaled, round-to-nearest two-plane fp16 "
               "split; 3 products (hh+hm+mh) per term on v_mfma_f32_32x32x16_f16, fp32 accumulate")

CONFIGS = {
    "cfg2": dict(C=64, H=540, W=960, D=192, dtype=torch.float32, op="inner_product", regress=True,
                 global_batch=32, chunk=32, dname="f32",
                 workload="BASELINE configs[1]: mobile_stereo_net inner_product CV, 1/4-res KITTI "
                          "540x960, C=64, D=192, fp32 + soft-argmin regression"),
    # cfg3: 4 pairs per GPU in one launch (round 6; one pair per launch leaves the persistent grid's
    # ramp and tail in every 0.73 ms launch: 0.62-0.64 against 0.71 at 4 pairs, profiles/r06/ab/r6v_*)
    "cfg3": dict(C=256, H=540, W=960, D=192, G=8, dtype=torch.bfloat16, op="groupwise",
                 regress=False, global_batch=None, per_gpu=4, chunk=4, dname="bf16",
                 workload="BASELINE configs[2]: groupwise cost volume, G=8 C=256 D=192 at 540x960, "
                          "bf16 in, fp32 (N,G,H,W,D) out, MFMA path"),
    "cfg4": dict(C=16, H=1080, W=1920, D=256, dtype=torch.float32, op="correlation", regress=True,
                 global_batch=32, chunk=32, dname="f32",
                 workload="BASELINE configs[3]: mobile_disp_net_c correlation CV, full-res 1080x1920, "
                          "C=16, D=256, fp32 + soft-argmin, global batch 32 sharded over the GPUs"),
    "cfg5": dict(C=128, H=540, W=960, D=64, dtype=torch.float16, op="concat", regress=False,
                 global_batch=None, chunk=1, dname="f16",
                 workload="BASELINE configs[4]: concatenate 4D cost volume, C=128 D=64 at 540x960, "
                          "fp16 (pure write)"),
}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="cfg2", choices=sorted(CONFIGS))
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--global-batch", type=int, default=None,
                    help="pairs per step over all ranks (strong scaling; cfg2/cfg4 default 32)")
    ap.add_argument("--batch", type=int, default=None,
                    help="pairs per GPU per step (weak scaling; overrides --global-batch)")
    ap.add_argument("--chunk", type=int, default=None, help="pairs per kernel launch")
    ap.add_argument("--algo", default="auto", choices=["auto", "sl", "rs", "h2", "h2db", "f32", "mfma", "valu"],
                    help="cfg2 volume kernel of --pipeline separate")
    ap.add_argument("--pipeline", default="separate",
                    choices=["separate", "fused", "fused-novolume", "interweave"])
    ap.add_argument("--features", default=None, choices=["f32", "f16", "bf16"],
                    help="cfg2 / cfg4 feature dtype; f16 / bf16 run under torch.autocast as the "
                         "reference's fp16 mode does (fp32 disparities)")
    ap.add_argument("--cpu-baseline-seconds", type=float, default=12.0,
                    help="bounded CPU-baseline sample length (0 disables)")
    ap.add_argument("--no-check", action="store_true", help="skip the numerics check")
    return ap.parse_args()


# ----------------------------------------------------------------------------- algorithmic bytes
def pair_bytes(cfg, pipeline):
    """Algorithmic bytes per pair of the dominant kernel: read L + R once, write the
    output once (the fused pass: + the disparities; without the volume: only those)."""
    C, H, W, D, es = cfg["C"], cfg["H"], cfg["W"], cfg["D"], cfg["dtype"].itemsize
    feats = 2 * C * H * W * es
    if cfg["op"] == "groupwise":
        return feats + cfg["G"] * H * W * D * 4
    if cfg["op"] == "concat":
        return feats + 2 * C * H * W * D * es
    # disparities: fp32 under autocast (half features), else the feature dtype
    vol, disp = D * H * W * es, H * W * max(es, 4 if cfg.get("autocast") else es)
    if pipeline == "fused":
        return feats + vol + disp
    if pipeline == "fused-novolume":
        return feats + disp
    return feats + vol


def pair_mfma_flops(cfg):
    """Useful flops per pair (2 C per valid output cell)."""
    valid = cfg["H"] * sum(max(0, cfg["W"] - d) for d in range(cfg["D"]))
    return 2 * cfg["C"] * valid


def kernel_name(cfg, pipeline, algo):
    if cfg["op"] == "concat":
        return "shifted_rows_kernel" if pipeline == "interweave" else "concat_kernel"
    if cfg["op"] == "groupwise":  # 16-bit features, 16-channel group steps, one D pass: band_rs
        return "band_rs (NGHWD, bf16)"
    f32 = cfg["dtype"] == torch.float32 and not cfg.get("autocast")
    # fp32 aligned rows with C = 16 or 64: the role-split band kernel for the volume (AUTO, rs);
    # the fused passes on the sliding-window one (one D pass of 65..192 disparities, or C = 16
    # with two passes of <= 128, D <= 256)
    sl_shape = f32 and cfg["C"] in (16, 64) and (64 < cfg["D"] <= 192 or (cfg["C"] == 16 and 192 < cfg["D"] <= 256))
    rs_shape = f32 and cfg["C"] in (16, 64) and cfg["D"] > 64
    if cfg["op"] in ("inner_product", "correlation") and pipeline == "separate":
        # AUTO: the sliding-window kernel (round 6), except the correlation mean at C = 16 with
        # one pass of more than 128 disparities (band_h2db)
        mean16 = cfg["op"] == "correlation" and cfg["C"] == 16 and 128 < cfg["D"] <= 192
        return {"valu": "dot_volume_valu", "f32": "ip_band_f32", "mfma": "ip_band_f32",
                "h2": "band_h2", "h2db": "band_h2db", "rs": "band_rs" if rs_shape else "band_h2db",
                }.get(algo, "band_sl" if sl_shape and not mean16 else "band_h2db")
    if pipeline == "fused":  # volume kept: FUSE 1 (one D pass); D > 192: the two kernels
        if not f32:
            return "band_h2 (fused soft-argmin, volume kept)"
        if cfg["D"] > 192:  # the volume kernel (AUTO), then the regression
            return "band_rs" if rs_shape else "band_h2db"
        return ("band_sl" if sl_shape else "band_h2db") + " (fused soft-argmin, volume kept)"
    if pipeline == "fused-novolume":  # fp32: band_sl FUSE 2; 16-bit features: band_h2 FUSE 2
        return ("band_sl" if sl_shape else "band_h2") + " (fused soft-argmin, volume-free)"
    return "band_h2"


def arithmetic(cfg, pipeline, algo):
    if cfg["op"] == "concat":
        return "copy (bit-exact)"
    if cfg["op"] == "groupwise":
        return "exact bf16 products on v_mfma_f32_32x32x16_bf16, fp32 accumulate, x 1/(C/G)"
    if cfg["op"] == "inner_product" and pipeline == "separate" and algo in ("f32", "mfma"):
        return "exact fp32 products on v_mfma_f32_16x16x4_f32"
    if cfg["op"] == "inner_product" and pipeline == "separate" and algo == "valu":
        return "fp32 FMA (VALU)"
    if cfg.get("autocast"):
        return (f"exact {cfg['dname']} products on v_mfma_f32_32x32x16_{cfg['dname']}, fp32 accumulate"
                + ("; soft-argmin online in fp32/fp64 on the fp32 accumulators, fp32 disparities"
                   if pipeline.startswith("fused") else "; volume rounded to the feature dtype"))
    return ARITH_SPLIT + ("; soft-argmin online in fp32/fp64" if pipeline.startswith("fused") else
                          "; soft-argmin kernel fp64 accumulation")


# ----------------------------------------------------------------------------- the step
def make_step(cfg, a, L, R, ev):
    """Returns step(timed) -> disparities (or None); appends (start, end) HIP events around
    each launch of the dominant kernel when timed."""
    D = cfg["D"]
    chunk = max(1, a.chunk or cfg["chunk"])
    nb = L.shape[0]

    def dominant(l, r):
        if cfg.get("autocast"):  # the reference's fp16 mode: the half features under autocast
            with torch.autocast("cuda", dtype=cfg["dtype"]):
                return dominant_(l, r)
        return dominant_(l, r)

    def dominant_(l, r):
        if cfg["op"] == "inner_product":
            if a.pipeline == "separate":
                return F.inner_product_volume(l, r, D, algo=a.algo), None
            vol, disp = F.inner_product_soft_argmin(l, r, D, keep_volume=a.pipeline == "fused")
            return vol, disp
        if cfg["op"] == "correlation":
            if a.pipeline.startswith("fused"):  # D = 256 volume-free: 2 passes + merge
                return F.inner_product_soft_argmin(l, r, D, mean=True, keep_volume=a.pipeline == "fused")
            return F.correlation_volume(l, r, D), None
        if cfg["op"] == "groupwise":
            return F.groupwise_volume(l, r, cfg["G"], D), None
        if a.pipeline == "interweave":
            return F.interweave_volume(l, r, D), None
        return F.concat_volume(l, r, D), None

    last = {}

    def step(timed):
        disps = []
        for s0 in range(0, nb, chunk):
            l, r = L[s0:s0 + chunk], R[s0:s0 + chunk]
            if timed:
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
            vol, disp = dominant(l, r)
            if timed:
                e.record()
                ev.append((s, e, l.shape[0]))
            if cfg["regress"] and disp is None:
                disp = F.soft_argmin(vol)
            if disp is not None:
                disps.append(disp)
            last["vol"], last["disp"], last["s0"] = vol, disp, s0
        if not disps:
            return None
        return torch.cat(disps, 0) if len(disps) > 1 else disps[0]

    return step, last


# ----------------------------------------------------------------------------- numerics (checker)
def check_numerics(cfg, a, L, R, last):
    """max |got - fp64 oracle| on sampled rows of the LAST chunk's outputs (rows depend only on the
    same rows of L and R).  Test infrastructure only: runs after the timed region."""
    from oracle import stereo_oracle as O
    from oracle.torch_port import soft_argmin_eager, sweep_dot_volume

    H, D = cfg["H"], cfg["D"]
    s0 = last["s0"]
    rows = sorted({0, H // 2, H - 1})
    vol, disp = last["vol"], last["disp"]
    out = {"rows": rows, "pair": s0}

    def host(t):
        t = t.detach()
        if t.dtype == torch.bfloat16:
            t = t.float()
        return t.cpu().numpy()

    lf = host(L[s0:s0 + 1].float())
    rf = host(R[s0:s0 + 1].float())
    errs_v, errs_d, dev32, mean_d, mean32, vdev32 = [], [], [], [], [], []
    for y in rows:
        ly, ry = lf[:, :, y:y + 1], rf[:, :, y:y + 1]
        if cfg["op"] in ("inner_product", "correlation"):
            ref = (O.inner_product(ly, ry, D) if cfg["op"] == "inner_product"
                   else O.correlation_mean(ly, ry, D)).astype(np.float64)
            # the fp64 pipeline (exact volume, fp64 soft-argmin) and torch's fp32 pipeline on the
            # same rows: the fair bar for the end-to-end disparity
            exact = O.softargmin(ref).astype(np.float64)
            v32 = sweep_dot_volume(torch.from_numpy(ly), torch.from_numpy(ry), D,
                                   mean=cfg["op"] == "correlation")
            # torch's own fp32 volume (the reference's op sequence) against the same fp64 rows:
            # the fp32-rounding yardstick for max_abs_err_volume
            vdev32.append(float(np.abs(v32.numpy().astype(np.float64) - ref).max()))
            t32 = soft_argmin_eager(v32)
            d32 = np.abs(t32.numpy().astype(np.float64) - exact)
            dev32.append(float(d32.max()))
            mean32.append(float(d32.mean()))
            if vol is not None:
                errs_v.append(float(np.abs(host(vol[:1, :, y:y + 1]).astype(np.float64) - ref).max()))
            if disp is not None:
                dd = np.abs(host(disp[:1, :, y:y + 1]).astype(np.float64) - exact)
                errs_d.append(float(dd.max()))
                mean_d.append(float(dd.mean()))
        elif cfg["op"] == "groupwise":
            ref = O.groupwise(ly, ry, cfg["G"], D).astype(np.float64)
            errs_v.append(float(np.abs(host(vol[:1, :, y:y + 1]).astype(np.float64) - ref).max()))
        else:
            lh, rh = host(L[s0:s0 + 1, :, y:y + 1]), host(R[s0:s0 + 1, :, y:y + 1])
            if a.pipeline == "interweave":
                ref, got = O.interweave_shifted(lh, rh, D), host(vol[:1, :, :, y:y + 1])
            else:
                ref, got = O.concatenate(lh, rh, D), host(vol[:1, :, y:y + 1])
            errs_v.append(0.0 if np.array_equal(got, ref) else float("inf"))
    if errs_v:
        out["max_abs_err_volume"] = max(errs_v)
    if vdev32:
        out["torch_fp32_volume_dev"] = max(vdev32)
    if errs_d:
        out["max_abs_err_disparity"] = max(errs_d)
    if dev32:
        out["torch_fp32_disparity_dev"] = max(dev32)
        out["torch_fp32_mean_disparity_dev"] = sum(mean32) / len(mean32)
    if mean_d:
        # EPE difference against the exact pipeline (north star: within 1e-4); the per-pixel
        # maximum is bounded by torch fp32's own per-pixel deviation from the same fp64 pipeline
        out["mean_abs_err_disparity"] = sum(mean_d) / len(mean_d)
        out["disparity_ok"] = bool(out["mean_abs_err_disparity"] <= 1e-4 and
                                   out["max_abs_err_disparity"] <= max(out["torch_fp32_disparity_dev"], 1e-4))
    # one row of EVERY pair of the last launch (a different row per pair) against the fp64
    # oracle: the whole persistent-grid launch, not only its first pair
    if cfg["op"] in ("inner_product", "correlation", "groupwise") and vol is not None:
        pairs, worst_v, worst_d = [], 0.0, 0.0
        for j in range(vol.shape[0]):
            y = (37 * j + 11) % H
            ly = host(L[s0 + j:s0 + j + 1, :, y:y + 1].float())
            ry = host(R[s0 + j:s0 + j + 1, :, y:y + 1].float())
            if cfg["op"] == "groupwise":
                ref = O.groupwise(ly, ry, cfg["G"], D).astype(np.float64)
            else:
                ref = (O.inner_product(ly, ry, D) if cfg["op"] == "inner_product"
                       else O.correlation_mean(ly, ry, D)).astype(np.float64)
            worst_v = max(worst_v, float(np.abs(host(vol[j:j + 1, :, y:y + 1]).astype(np.float64) - ref).max()))
            if disp is not None:
                got_v = host(vol[j:j + 1, :, y:y + 1])
                worst_d = max(worst_d, float(np.abs(host(disp[j:j + 1, :, y:y + 1]).astype(np.float64)
                                                    - O.softargmin(got_v)).max()))
            pairs.append([s0 + j, y])
        out["all_pairs_checked"] = pairs
        out["all_pairs_max_abs_err_volume"] = worst_v
        if disp is not None:
            # the regression of each sampled volume row against its fp64 soft-argmin
            out["all_pairs_max_abs_err_regression"] = worst_d
    elif cfg["op"] in ("inner_product", "correlation") and disp is not None:
        # volume-free fused launch: one row of every pair's disparity against the exact fp64
        # pipeline (oracle volume, fp64 soft-argmin); per-pixel bar as above (torch fp32's own
        # deviation on the first pair's rows, at least 1e-4), mean (EPE difference) within 1e-4
        pairs, worst_d, means = [], 0.0, []
        for j in range(disp.shape[0]):
            y = (37 * j + 11) % H
            ly = host(L[s0 + j:s0 + j + 1, :, y:y + 1].float())
            ry = host(R[s0 + j:s0 + j + 1, :, y:y + 1].float())
            ref = (O.inner_product(ly, ry, D) if cfg["op"] == "inner_product"
                   else O.correlation_mean(ly, ry, D)).astype(np.float64)
            dd = np.abs(host(disp[j:j + 1, :, y:y + 1]).astype(np.float64) - O.softargmin(ref))
            worst_d = max(worst_d, float(dd.max()))
            means.append(float(dd.mean()))
            pairs.append([s0 + j, y])
        out["all_pairs_checked"] = pairs
        out["all_pairs_max_abs_err_disparity"] = worst_d
        out["all_pairs_mean_abs_err_disparity"] = sum(means) / len(means)
    out["tolerance"] = 0.0 if cfg["op"] == "concat" else 1e-4
    return out


# ----------------------------------------------------------------------------- CPU baseline
def usable_cores():
    """Cores this process may run on: the affinity mask, capped by a cgroup CPU quota (on the
    GPU box os.cpu_count() reports the whole host, far more than this job's share)."""
    try:
        n = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        n = os.cpu_count() or 1
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, p = f.read().split()[:2]
        if q != "max":
            n = min(n, max(1, math.ceil(int(q) / int(p))))
    except (OSError, ValueError):
        pass
    return max(1, n)


def host_cpu():
    model, phys = "unknown", set()
    try:
        with open("/proc/cpuinfo") as f:
            pid = cid = None
            for line in f:
                k, _, v = line.partition(":")
                k, v = k.strip(), v.strip()
                if k == "model name" and model == "unknown":
                    model = v
                elif k == "physical id":
                    pid = v
                elif k == "core id":
                    cid = v
                elif not k and pid is not None:
                    phys.add((pid, cid))
                    pid = cid = None
    except OSError:
        pass
    return model, len(phys) or None


def cpu_baseline(cfg, a, seconds):
    """The eager CPU port of the reference op sequence (oracle/torch_port.py) on the host cores.
    Rows are independent, so a bounded sample times a band of rows (or whole pairs when one fits
    the budget) and scales to pairs/s; the sample is stated."""
    from oracle import torch_port as P

    threads = usable_cores()
    torch.set_num_threads(threads)
    C, H, W, D = cfg["C"], cfg["H"], cfg["W"], cfg["D"]
    g = torch.Generator().manual_seed(0)

    # the reference's CPU path computes in fp32 (autocast is a GPU mode)
    dt = torch.float32 if cfg.get("autocast") else cfg["dtype"]

    def run(rows):
        l = torch.randn(1, C, rows, W, generator=g).to(dt)
        r = torch.randn(1, C, rows, W, generator=g).to(dt)
        t0 = time.perf_counter()
        if cfg["op"] == "inner_product":
            P.cv_plus_regression(l, r, D)
        elif cfg["op"] == "correlation":
            P.correlation_plus_regression(l, r, D)
        elif cfg["op"] == "groupwise":
            P.sweep_groupwise(l, r, cfg["G"], D)
        elif a.pipeline == "interweave":
            P.sweep_interweave_shifted(l, r, D)
        else:
            P.sweep_concat(l, r, D)
        return time.perf_counter() - t0

    probe_rows = max(1, H // 64)
    run(probe_rows)  # warm-up (thread pool, allocator)
    t_probe = run(probe_rows)
    rows = H if t_probe * H / probe_rows <= seconds / 2 else \
        int(min(H, max(probe_rows, probe_rows * (seconds / 3) / max(t_probe, 1e-9))))
    done_rows, elapsed = 0, 0.0
    while elapsed < seconds or done_rows == 0:
        elapsed += run(rows)
        done_rows += rows
    pairs = done_rows / H
    model, phys = host_cpu()
    what = {"inner_product": "inner-product CV + soft-argmin", "correlation": "correlation CV + soft-argmin",
            "groupwise": "groupwise CV", "concat": "concatenate CV"}[cfg["op"]]
    if cfg["op"] == "concat" and a.pipeline == "interweave":
        what = "shifted interweave volume"
    return {"value": pairs / elapsed, "unit": "pairs/s", "cores": threads, "kind": "port",
            "sample": f"{done_rows} rows of {H} ({pairs:.3f} pairs) of 1x{C}x{H}x{W} "
                      f"{'f32' if cfg.get('autocast') else cfg['dname']}, "
                      f"D={D}, {what}; eager torch CPU port of the reference op sequence, {threads} "
                      f"threads; host: {model}, {os.cpu_count()} logical CPUs, "
                      f"{phys or 'unknown'} physical cores",
            "ms_per_pair": 1e3 * elapsed / pairs}


# ----------------------------------------------------------------------------- PMC traffic
EVIDENCE_ROUND = "r06"


def evidence_name(a):
    suffix = {"separate": "", "fused": "_fused", "fused-novolume": "_fused_novolume",
              "interweave": "_interweave"}[a.pipeline]
    return a.config + suffix + ("" if getattr(a, "features", None) in (None, "f32") else "_" + a.features)


def committed_traffic(a, kernel, world=1):
    """HBM bytes per launch of the dominant kernel from the rocprofv3 --pmc FETCH_SIZE /
    WRITE_SIZE passes of this same command (scripts/gpu_evidence.sh; PMC counters cannot be read
    in the timed run itself), or None when this workload has no committed counter run."""
    rel = os.path.join("profiles", EVIDENCE_ROUND, evidence_name(a), "pmc.json")
    out = {"traffic": None, "traffic_source": None}
    # the committed passes ran this workload at N=1 with the default pairs per launch
    if a.algo != "auto" or a.batch is not None or a.chunk is not None or world != 1:
        return out
    try:
        with open(os.path.join(ROOT, rel)) as f:
            ks = json.load(f)["kernels"]
    except (OSError, ValueError, KeyError):
        return out
    base = kernel.split(" ")[0]
    cands = [v for k, v in ks.items() if k.startswith(base) and "hbm_bytes_per_launch" in v]
    if cands:
        out["traffic"] = round(max(c["hbm_bytes_per_launch"] for c in cands))
        out["traffic_unit"] = "bytes per launch"
        out["traffic_source"] = (rel + ": rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE, separate runs "
                                 "of this command, 2*FETCH_SIZE+WRITE_SIZE (gfx950 correction)")
    return out


# ----------------------------------------------------------------------------- main
def main():
    a = parse()
    cfg = CONFIGS[a.config]
    if a.features not in (None, "f32"):
        if cfg["op"] not in ("inner_product", "correlation") or not a.pipeline.startswith("fused"):
            raise SystemExit("--features f16 / bf16 applies to cfg2 / cfg4 with --pipeline fused*")
        half = {"f16": torch.float16, "bf16": torch.bfloat16}[a.features]
        cfg = dict(cfg, dtype=half, dname=a.features, autocast=True,
                   workload=cfg["workload"] + f"; {a.features} features under torch.autocast")
    if a.pipeline in ("fused", "fused-novolume") and cfg["op"] not in ("inner_product", "correlation"):
        raise SystemExit("--pipeline fused* applies to cfg2 / cfg4 (fused volume + soft-argmin)")
    if a.pipeline == "interweave" and cfg["op"] != "concat":
        raise SystemExit("--pipeline interweave applies to cfg5")
    if a.pipeline != "separate" and a.algo not in ("auto", "h2"):
        raise SystemExit("--algo selects the volume kernel of --pipeline separate")
    rank, world, local = env_rank()
    if world == 1 and a.gpus > 1:
        raise SystemExit("--gpus N>1 must be launched with torchrun --nproc-per-node N")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)

    if a.batch is not None:
        scaling, global_batch = "weak", a.batch * world
        nb = a.batch
    else:
        gb = a.global_batch or cfg["global_batch"]
        if gb is None:  # one-GPU configs: a fixed number of pairs per GPU (replicas)
            nb = cfg.get("per_gpu", 1)
            scaling, global_batch = "weak", world * nb
        else:
            scaling, global_batch = "strong", gb
            s, e = shard_range(gb, rank, world)
            nb = e - s
    C, H, W = cfg["C"], cfg["H"], cfg["W"]
    g = torch.Generator(device=dev).manual_seed(1234 + rank)
    L = torch.randn(nb, C, H, W, device=dev, generator=g).to(cfg["dtype"])
    R = torch.randn(nb, C, H, W, device=dev, generator=g).to(cfg["dtype"])

    ev = []
    step, last = make_step(cfg, a, L, R, ev)

    def run(timed):
        disp = step(timed)
        if cfg["regress"]:
            gather_disparities(disp, global_batch)

    for _ in range(a.warmup):
        run(False)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        run(True)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    kern_ms = sum(s.elapsed_time(e) for s, e, _ in ev)
    launches = max(1, len(ev))
    timed_pairs = sum(n for _, _, n in ev)
    nbytes = pair_bytes(cfg, a.pipeline) * timed_pairs
    achieved = nbytes / (kern_ms * 1e-3) / 1e9 if kern_ms > 0 else 0.0
    pairs = global_batch * a.steps
    rec = {
        "metric": METRIC,
        "value": pairs / elapsed,
        "unit": "pairs/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": 1e3 * elapsed / a.steps,
        "ms_per_pair": 1e3 * elapsed / pairs,
        "higher_is_better": True,
        "scaling": scaling,
        "vs_baseline": None,
        "dtype": cfg["dname"],
        "data": "synthetic (standard-normal features, seeded per rank)",
        "config": {"workload": cfg["workload"], "config": a.config, "C": C, "H": H, "W": W,
                   "D": cfg["D"], **({"G": cfg["G"]} if "G" in cfg else {}),
                   "global_batch": global_batch, "pairs_per_gpu": nb,
                   "pairs_per_launch": min(nb, max(1, a.chunk or cfg["chunk"])),
                   "parallelism": f"dp{world}", "algo": a.algo, "pipeline": a.pipeline,
                   "arithmetic": arithmetic(cfg, a.pipeline, a.algo)},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS,
                     **committed_traffic(a, kernel_name(cfg, a.pipeline, a.algo), world),
                     "kernel": kernel_name(cfg, a.pipeline, a.algo),
                     "avg_kernel_us": 1e3 * kern_ms / launches,
                     "us_per_pair": 1e3 * kern_ms / max(1, timed_pairs),
                     "algorithmic_bytes_per_launch": nbytes / launches,
                     "algorithmic_bytes_per_pair": pair_bytes(cfg, a.pipeline)},
    }
    if cfg["op"] == "groupwise" and kern_ms > 0:
        tf = pair_mfma_flops(cfg) * timed_pairs / (kern_ms * 1e-3) / 1e12
        rec["mfma"] = {"achieved": tf, "peak": MFMA_BF16_PEAK_TF, "unit": "TFLOP/s",
                       "frac": tf / MFMA_BF16_PEAK_TF,
                       "note": "useful flops (2 C per valid cell) / kernel time; the HBM roofline bounds it"}
    if rank == 0 and not a.no_check:
        rec["numerics"] = check_numerics(cfg, a, L, R, last)
    if rank == 0 and world == 1 and a.cpu_baseline_seconds > 0:
        rec["cpu_baseline"] = cpu_baseline(cfg, a, a.cpu_baseline_seconds)
    if rank == 0:
        print(json.dumps(rec), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
