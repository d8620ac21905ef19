#!/usr/bin/env python3
"""Headline benchmark: stereo pairs/s for KITTI-res D=192 cost volume + regression.

Workload (BASELINE.json configs[1], the config the metric is quoted on): per stereo pair,
1x64x540x960 fp32 left/right feature maps (1/4-res KITTI), inner-product cost volume with
D=192 (TorchInnerProductCost, cost_volume/inner_product.py:11-42) followed by the soft-argmin
disparity regression (model/mobile_disp_net_c.py:208-220).  A STEP is one pass of that hot
path over the rank's batch of pairs (inputs already resident in HBM), plus -- for N>1 -- the
RCCL gather of the per-pair disparities to rank 0 (the only collective).

Pipelines (--pipeline):
  separate        (default) the volume kernel (--algo), then the regression kernel reading the
                  (N,D,H,W) volume back -- the reference's two calls;
  fused           one band-kernel launch writes the volume AND its soft-argmin
                  (functional.inner_product_soft_argmin);
  fused-novolume  SURVEY §8f-1: the same kernel without writing the volume.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B] [--pipeline P] [--algo A]
    torchrun --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N ...

Rank 0 prints ONE JSON line.  ``value`` = pairs processed by all ranks / max-over-ranks wall
time of the K timed steps (weak scaling: B pairs per GPU per step).  ``roofline`` is the
dominant kernel (the cost-volume build) timed with HIP events on the launch stream inside
the timed region; ``cpu_baseline`` times the eager CPU port of the reference algorithm
(oracle/torch_port.py) on the host cores on a bounded sample (rank 0, N=1 only).
"""
import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from realtime_stereo_matcher_amd import functional as F  # noqa: E402
from realtime_stereo_matcher_amd.distributed import env_rank, gather_disparities  # noqa: E402

C, H, W, D = 64, 540, 960, 192
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)


def kernel_algorithmic_bytes(batch, pipeline):
    """Algorithmic bytes of the timed (dominant) kernel per launch: read L + R,
    write the (N, D, H, W) fp32 volume once; the fused kernel also writes the disparities."""
    feats, vol, disp = 2 * C * H * W * 4, D * H * W * 4, H * W * 4
    if pipeline == "separate":
        return batch * (feats + vol)
    if pipeline == "fused":
        return batch * (feats + vol + disp)
    return batch * (feats + disp)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--batch", type=int, default=1, help="stereo pairs per GPU per step")
    ap.add_argument("--algo", default="auto", choices=["auto", "h2", "bf16x3", "f32", "mfma", "valu"],
                    help="volume kernel of --pipeline separate")
    ap.add_argument("--pipeline", default="separate", choices=["separate", "fused", "fused-novolume"])
    ap.add_argument("--cpu-baseline-seconds", type=float, default=12.0,
                    help="bounded CPU-baseline sample length (0 disables)")
    return ap.parse_args()


def traffic_from_profiles(kernel_prefix):
    """HBM bytes per launch of the dominant kernel from the committed PMC summary, if any."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(path) as f:
            rec = json.load(f)
        k = rec["kernels"].get(kernel_prefix)
        return None if k is None else k["hbm_bytes_per_launch"]
    except (OSError, KeyError, ValueError):
        return None


def cpu_baseline(seconds):
    """Eager CPU port of the reference algorithm on the host cores, bounded sample."""
    from oracle.torch_port import cv_plus_regression

    threads = torch.get_num_threads()
    g = torch.Generator().manual_seed(0)
    L = torch.randn(1, C, H, W, generator=g)
    R = torch.randn(1, C, H, W, generator=g)
    pairs = 0
    t0 = time.perf_counter()
    while True:
        cv_plus_regression(L, R, D)
        pairs += 1
        if time.perf_counter() - t0 >= seconds:
            break
    dt = time.perf_counter() - t0
    cpu = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    cpu = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return {"value": pairs / dt, "unit": "pairs/s", "cores": threads, "kind": "port",
            "sample": f"{pairs} full cfg2 pair(s) (1x64x540x960 fp32, D=192, CV + soft-argmin), "
                      f"eager torch CPU, {threads} threads, {cpu}",
            "ms_per_pair": 1e3 * dt / pairs}


def main():
    a = parse()
    rank, world, local = env_rank()
    if world != a.gpus:
        if world == 1 and a.gpus > 1:
            raise SystemExit("--gpus N>1 must be launched with torchrun --nproc-per-node N")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)
    B = a.batch
    g = torch.Generator(device=dev).manual_seed(1234 + rank)
    L = torch.randn(B, C, H, W, device=dev, generator=g)
    R = torch.randn(B, C, H, W, device=dev, generator=g)
    global_batch = B * world

    ev = []  # (start, end) around the CV kernel, timed steps only

    if a.pipeline != "separate" and a.algo not in ("auto", "h2"):
        raise SystemExit("--algo selects the volume kernel of --pipeline separate")

    def step(timed):
        if timed:
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
        if a.pipeline == "separate":
            vol = F.inner_product_volume(L, R, D, algo=a.algo)
            if timed:
                e.record()
            disp = F.soft_argmin(vol)  # (B, 1, H, W)
        else:
            _, disp = F.inner_product_soft_argmin(L, R, D, keep_volume=a.pipeline == "fused")
            if timed:
                e.record()
        if timed:
            ev.append((s, e))
        return gather_disparities(disp, global_batch)

    for _ in range(a.warmup):
        step(False)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step(True)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    cv_ms = sum(s.elapsed_time(e) for s, e in ev) / max(1, len(ev))
    nbytes = kernel_algorithmic_bytes(B, a.pipeline)
    achieved = nbytes / (cv_ms * 1e-3) / 1e9
    kname = "band_h2"
    if a.pipeline == "separate":
        kname = {"valu": "dot_volume_valu", "f32": "ip_band_f32", "mfma": "ip_band_f32",
                 "bf16x3": "ip_band_mfma"}.get(a.algo, "band_h2")
    traffic = traffic_from_profiles(kname)
    pairs = global_batch * a.steps
    rec = {
        "metric": "stereo pairs/sec (KITTI-res 540x960x64 inner-product cost volume D=192 + soft-argmin)",
        "value": pairs / elapsed,
        "unit": "pairs/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": 1e3 * elapsed / a.steps,
        "ms_per_pair": 1e3 * elapsed / pairs * world,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic (standard-normal features, seeded per rank)",
        "config": {"workload": "BASELINE configs[1]: mobile_stereo_net inner_product CV, 1/4-res KITTI "
                               "540x960, C=64, D=192, fp32 + soft-argmin regression",
                   "C": C, "H": H, "W": W, "D": D, "batch_per_gpu": B, "global_batch": global_batch,
                   "parallelism": f"dp{world}", "algo": a.algo, "pipeline": a.pipeline},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                     "kernel": kname, "avg_kernel_us": cv_ms * 1e3,
                     "algorithmic_bytes_per_launch": nbytes},
    }
    if rank == 0 and world == 1 and a.cpu_baseline_seconds > 0:
        rec["cpu_baseline"] = cpu_baseline(a.cpu_baseline_seconds)
    if rank == 0:
        print(json.dumps(rec), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
