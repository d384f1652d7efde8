#!/usr/bin/env python3
"""Benchmark: solved trajectories/sec for the 50-knot unicycle + learned-SDF workload (BASELINE.json).

One step = one batched solve (nlot_solve_batch) of B synthetic start/goal instances per GPU of the
metric NLP: benchmark_3's body/bounds/slack penalty, N = 50 knots, learned SDF = the reference
artefact FourierMLP (2-128-128-1, scale 10), linear initial guess.  Instances are independent, so each
rank solves its own seeded batch (weak scaling) and the solved trajectories are gathered to rank 0
over RCCL at the end of every step (the only collective).

value = solved instances of all ranks in the timed steps / max-over-ranks wall time of those steps.

    python bench.py [--gpus N --steps K --warmup W --batch B]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from nlotrajectories_amd import _abi  # noqa: E402
from nlotrajectories_amd.dist import gather_solutions, max_over_ranks, rank_world, sum_over_ranks  # noqa: E402
from nlotrajectories_amd.nn import MlpWeights  # noqa: E402
from nlotrajectories_amd.ops import DeviceMlp, sdf_mlp_eval  # noqa: E402
from nlotrajectories_amd.problem import METRIC_PROBLEM  # noqa: E402
from nlotrajectories_amd.sampling import sample_start_goal  # noqa: E402
from nlotrajectories_amd.solver import last_stats, set_timing, solve_batch  # noqa: E402

PEAK_F32_MFMA_TFLOPS = 157.3  # MI355X_MICROARCH.md: f32-input MFMA = f32 vector peak (dense)
PEAK_BF16_MFMA_TFLOPS = 2500.0  # MI355X_MICROARCH.md: bf16 MFMA, dense
SPLIT_PRODUCTS = 6  # fp32-equivalent product = 6 bf16 MFMA products (nlot_mlp.hip, split-bf16 kernels)
# the MLP kernels emulate fp32 products with 6 bf16 MFMAs: their MFMA roofline for the algorithmic
# (fp32) FLOPs is the dense bf16 peak / 6
PEAK_SPLIT_TFLOPS = PEAK_BF16_MFMA_TFLOPS / SPLIT_PRODUCTS
PEAK_HBM_GBS = 8000.0


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--batch", type=int, default=65536, help="instances per GPU per step (SURVEY.md §8d config 3: 1024 / 16384 / 65536)")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--cpu-sample", type=int, default=48, help="instances for the CPU baseline (0 = skip)")
    ap.add_argument("--cpu-threads", type=int, default=16)
    ap.add_argument("--mu-strategy", choices=["adaptive", "monotone"], default="adaptive",
                    help="adaptive = the reference's IPOPT setting (runner.py:118-120)")
    return ap.parse_args()


def main():
    a = parse()
    rank, local, world = rank_world()
    torch.cuda.set_device(local)
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)
    prob = METRIC_PROBLEM
    w = MlpWeights.artefact()
    mlp = DeviceMlp(w)

    def sdf_gpu(pts):
        v, _, _ = sdf_mlp_eval(mlp, torch.as_tensor(pts, dtype=torch.float32, device=dev), derivatives=False)
        return v.cpu().numpy()

    # start/goal uniform in [-0.3, 1.3]^2, all corners sdf >= 0.02
    x0, xg = sample_start_goal(prob, a.batch, seed=a.seed, sdf=sdf_gpu, rank=rank)
    x0 = torch.tensor(x0, dtype=torch.float64, device=dev)
    xg = torch.tensor(xg, dtype=torch.float64, device=dev)
    opt = _abi.default_options() if a.mu_strategy == "adaptive" else \
        _abi.default_options(mu_strategy=0, barrier_tol_factor=10.0)
    ws = None

    def step():
        r = solve_batch(prob, x0, xg, mlp=mlp, options=opt, workspace=ws)
        solved = (r["status"] == 0)
        if world > 1:  # gather the solutions to every rank (RCCL over xGMI): the only collective
            gather_solutions(r, keys=("X", "U", "cost", "status"))
        return r, int(solved.sum().item())

    from nlotrajectories_amd.solver import workspace_bytes

    ws = torch.empty(workspace_bytes(prob, a.batch), dtype=torch.uint8, device=dev)
    for _ in range(a.warmup):
        step()
    set_timing(True)
    agg = dict(mlp_full_ms=0.0, mlp_full_launches=0, mlp_points_full=0, mlp_value_ms=0.0,
               mlp_value_launches=0, mlp_points_value=0, iterations=0, iterate_ms=0.0,
               mlp_points_full_reused=0)
    slots_in_lds = None
    iters_all, solved_total = [], 0
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        r, ns = step()
        solved_total += ns
        st = last_stats()
        for k in agg:
            agg[k] += st[k]
        slots_in_lds = bool(st["slots_in_lds"])
        iters_all.append(r["iters"][r["status"] == 0].float().mean().item() if ns else 0.0)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    set_timing(False)
    status_counts = torch.bincount(r["status"].long(), minlength=4).cpu().numpy().tolist()
    elapsed = max_over_ranks(elapsed, dev)
    solved_total = sum_over_ranks(solved_total, dev)

    # roofline of the dominant MFMA kernel: the full (value + gradient + Hessian) SDF-MLP launch.  FLOP are
    # counted as executed: the reverse sweep at every point, the forward only where the launch did not take
    # it from the accepted trial point's value launch (forward reuse)
    flop_pt = w.flops_per_point_fwd_grad  # 67,072 for 2-128-128-1
    flop_fwd = w.flops_per_point_fwd      # 33,536
    n_l = max(agg["mlp_full_launches"], 1)
    avg_ms = agg["mlp_full_ms"] / n_l
    reused = agg["mlp_points_full_reused"]
    flop_launch = (agg["mlp_points_full"] * flop_pt - reused * flop_fwd) / n_l
    achieved = flop_launch / (avg_ms * 1e-3) / 1e12 if avg_ms > 0 else 0.0
    traffic = None
    tf = os.path.join(ROOT, "profiles", "mlp_full_traffic.json")
    if os.path.exists(tf):
        with open(tf) as f:
            traffic = json.load(f).get("hbm_bytes_per_launch_per_point")
            if traffic is not None:
                traffic = traffic * agg["mlp_points_full"] / n_l

    cpu = None
    if rank == 0 and world == 1 and a.cpu_sample > 0:
        cpu = cpu_baseline(prob, w, x0.cpu().numpy()[: a.cpu_sample], xg.cpu().numpy()[: a.cpu_sample],
                           a.cpu_threads, opt)

    if rank == 0:
        line = {
            "metric": "solved trajectories/sec (50-knot unicycle+learned-SDF)",
            "value": solved_total / elapsed,
            "unit": "trajectories/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": elapsed / a.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64 (interior-point solver) + f32 (SDF-MLP: fp32-equivalent split-bf16 MFMA products, as "
                     "the reference's fp32 libtorch graph)",
            "data": "synthetic start/goal (seeded, SURVEY.md §8d); learned SDF = reference artefact weights",
            "config": {
                "workload": "metric NLP: unicycle_2nd, rect 0.2x0.08, N=50, rho=10, bounds +-1, "
                            "learned SDF FourierMLP 2-128-128-1 (artefact), linear init, IPOPT tol 1e-4",
                "mu_strategy": a.mu_strategy,
                "instances_per_gpu": a.batch,
                "global_batch": a.batch * world,
                "knots": prob.N + 1,
                "parallelism": f"instances sharded over {world} GPU(s); RCCL all_gather of solutions",
                "solved_per_step_rank0": int((r["status"] == 0).sum().item()),
                "status_counts_rank0": status_counts,
                "mean_iters_solved": float(np.mean(iters_all)),
                "lockstep_global_steps": agg["iterations"] // max(a.steps, 1),
                "solver_step_kernel_ms_per_step": agg["iterate_ms"] / max(a.steps, 1),
                "mlp_ms_per_step": (agg["mlp_full_ms"] + agg["mlp_value_ms"]) / max(a.steps, 1),
                "riccati_slots": "lds" if slots_in_lds else "hbm",
            },
            "roofline": {
                "kernel": "mlp_bf16<128,full> (SDF-MLP value+grad+Hessian; fp32-equivalent products as 6 split "
                          "v_mfma_f32_32x32x16_bf16)",
                "bound": "mfma",
                "achieved": achieved,
                "peak": PEAK_SPLIT_TFLOPS,
                "unit": "TFLOP/s",
                "frac": achieved / PEAK_SPLIT_TFLOPS,
                "peak_note": "dense bf16 MFMA peak 2500 TFLOP/s / 6 split products per fp32-equivalent product; "
                             "the f32-input MFMA peak would be 157.3",
                "traffic": traffic,
                "flop_per_point": flop_pt,
                "forward_reused_frac": reused / max(agg["mlp_points_full"], 1),
                "flop_counting": "executed: 67,072 per point, less the 33,536 forward where it was reused",
                "points_per_launch": agg["mlp_points_full"] / n_l,
                "avg_launch_ms": avg_ms,
                "launches": agg["mlp_full_launches"],
            },
            "cpu_baseline": cpu,
        }
        print(json.dumps(line))
    if world > 1:
        dist.destroy_process_group()


def cpu_baseline(prob, w, x0, xg, threads, opt):
    """The oracle (C restatement, OpenMP over instances) on a bounded sample of the same workload."""
    try:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle as O
    except Exception as e:  # pragma: no cover
        return {"error": str(e)}
    threads = max(1, min(threads, os.cpu_count() or 1))
    hm = O.HostMlp(w)
    t = time.perf_counter()
    r = O.solve_batch(prob, x0, xg, hm, opt=opt, threads=threads)
    dt = time.perf_counter() - t
    ns = int((r["status"] == 0).sum())
    return {"value": ns / dt, "unit": "trajectories/s", "cores": threads, "kind": "port",
            "sample": f"{len(x0)} instances of the same seeded workload (first of rank 0's batch), "
                      f"{ns} solved in {dt:.1f} s on {threads} OpenMP threads"}


if __name__ == "__main__":
    main()
