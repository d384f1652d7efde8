#!/usr/bin/env python3
"""Benchmark: solved trajectories/sec for the 50-knot unicycle + learned-SDF workload (BASELINE.json).

One step = one batch of B synthetic start/goal instances per GPU of the metric NLP solved to completion:
benchmark_3's body/bounds/slack penalty, N = 50 knots, learned SDF = the reference artefact FourierMLP
(2-128-128-1, scale 10), linear initial guess; B = 32,768 by default (so that `--steps 20 --warmup 5` fits
600 s; `--batch 65536` measures ~7 % more).  By default (--continuous on) the K timed batches stream through the
solver in one nlot_solve_batch call with 65,536 instances in flight (continuous batching, NlotSolverOptions.max_active;
slot-indexed state: 22.6 GB of workspace whatever the number of batches), so the latency-bound tail is paid once; every
instance's result is the same as in a call of its own.  Instances are independent, so each rank solves its
own seeded batches (weak scaling) and the solved trajectories are gathered to rank 0 over RCCL after every
solve call (the only collective).

value = solved instances of all ranks in the timed steps / max-over-ranks wall time of those steps.

With --workload stress: BASELINE.json configs[4], the same NLP at N = 256 knots with the 2-256x4-1 ReLU SDF
MLP (seeded, MlpWeights.stress_sdf_mlp), 8192 instances per GPU; the roofline is then the MLP's (f32 MFMA).

    python bench.py [--gpus N --steps K --warmup W --batch B --workload metric|stress]
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
# a progress line on stderr every 30 s from inside the long continuous-batching solve calls
os.environ.setdefault("NLOT_PROGRESS", "30")
sys.path.insert(0, ROOT)

from nlotrajectories_amd import _abi  # noqa: E402
from nlotrajectories_amd.dist import (gather_rank_rows, gather_solutions, max_over_ranks, rank_world,  # noqa: E402
                                      sum_over_ranks)
from nlotrajectories_amd.nn import MlpWeights  # noqa: E402
from nlotrajectories_amd.ops import DeviceMlp, sdf_mlp_eval  # noqa: E402
from nlotrajectories_amd.rrt import rrt_initial_guess  # noqa: E402
from nlotrajectories_amd.problem import B6_PROBLEM, BENCHMARKS, METRIC_PROBLEM, STRESS_PROBLEM  # noqa: E402
from nlotrajectories_amd.sampling import sample_start_goal  # noqa: E402
from nlotrajectories_amd.solver import last_stats, set_timing, solve_batch  # noqa: E402

PEAK_F32_MFMA_TFLOPS = 157.3  # MI355X_MICROARCH.md: f32-input MFMA = f32 vector peak (dense)
PEAK_BF16_MFMA_TFLOPS = 2500.0  # MI355X_MICROARCH.md: bf16 MFMA, dense
SPLIT_PRODUCTS = 6  # fp32-equivalent product = 6 bf16 MFMA products (nlot_mlp.hip, split-bf16 kernels)
# the MLP kernels emulate fp32 products with 6 bf16 MFMAs: their MFMA roofline for the algorithmic
# (fp32) FLOPs is the dense bf16 peak / 6
PEAK_SPLIT_TFLOPS = PEAK_BF16_MFMA_TFLOPS / SPLIT_PRODUCTS
PEAK_HBM_GBS = 8000.0
TIMING_EVERY = int(os.environ.get("NLOT_BENCH_TIMING_EVERY", "8"))  # hipEvents on one global step in 8 (nlot_set_timing)
PEAK_F32_MFMA_NOTE = "dense f32-input MFMA peak (v_mfma_f32_16x16x4_f32; exact fp32 products)"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=4)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--workload", choices=["metric", "stress", "b6"], default="metric",
                    help="metric = BASELINE.json's headline config; stress = configs[4] (2-256x4-1 SDF MLP, N = 256); "
                         "b6 = configs[3] (benchmark 6 Ackermann + ring corridor, N = 100, trained SDF)")
    ap.add_argument("--batch", type=int, default=None,
                    help="instances per GPU per step (metric default 32768, within SURVEY.md §8d config 3's range: the "
                         "driver's --steps 20 --warmup 5 run fits its 600 s budget; 65536 measures ~7 %% more; stress default "
                         "8192 = 65536 over 8 GPUs)")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--cpu-sample", type=int, default=None,
                    help="instances for the CPU baseline on all threads (0 = skip; default 32; 16 stress)")
    ap.add_argument("--cpu-sample-1core", type=int, default=None,
                    help="at least this many instances for the single-core CPU baseline, one at a time until ~8 s (default 2; 1 stress)")
    ap.add_argument("--cpu-threads", type=int, default=None,
                    help="CPU-baseline threads (default: the host's CPU share: min(affinity, cgroup cpu.max quota))")
    ap.add_argument("--cpu-overlap", choices=["on", "off"], default="off",
                    help="off (default since round 5): the CPU baseline runs after the timed region on the host's whole "
                         "CPU share.  on (metric / b6, one rank): during the untimed warm-up on one thread fewer (the "
                         "solver's launch thread keeps one), joined before the timed region; it competes with the "
                         "solver's host thread and measured 7 % lower (0.485 vs 0.522 traj/s, profiles/r05/"
                         "bench_r05ab_*.json), so it is no longer the default")
    ap.add_argument("--continuous", choices=["on", "off"], default="on",
                    help="on (metric / stress): the timed steps' batches flow through the solver with --batch slots "
                         "(continuous batching, NlotSolverOptions.max_active; all of them in one solve call), so one "
                         "batch's latency-bound tail overlaps the next batch's bulk; off: one solve call per batch")
    ap.add_argument("--slots", type=int, default=None,
                    help="continuous batching: instances in flight (default 65536 metric, --batch otherwise; the "
                         "workspace holds the slots' state only, ABI v10)")
    ap.add_argument("--mu-strategy", choices=["adaptive", "monotone"], default="adaptive",
                    help="adaptive = the reference's IPOPT setting (runner.py:118-120)")
    ap.add_argument("--launch-check", action="store_true",
                    help="the multi-rank plumbing alone (self-launch, rank / world, process group, the rank-seeded shards "
                         "gathered to rank 0 in rank order), no solve: tests/test_bench_launch.py runs it on the CPU "
                         "under NLOT_DIST_BACKEND=gloo")
    ap.add_argument("--bounds", choices=["rows", "variable"], default="rows",
                    help="rows = the reference's NLP: the control bounds and slack >= 0 as constraint rows, the form "
                         "CasADi's Opti hands IPOPT (runner.py:67-69,101-103; NlotSolverOptions.general_bounds = 1); "
                         "variable = the same bounds as variable bounds (the GPU's form before round 5)")
    return ap.parse_args()


def batch_calls(steps, continuous, per_call=4):
    """(G, calls): the timed batches per solve call.  Continuous batching streams up to `per_call` batches
    through one call (the workspace grows with them: 19 GiB per 65,536 metric instances); otherwise one call
    per batch.  sum(calls) == steps."""
    if not continuous:
        return 1, [1] * steps
    G = max(1, min(steps, per_call))
    return G, [min(G, steps - i) for i in range(0, steps, G)]


def timed_loop(step, steps, warmup, world, sync, device, after_warmup=None):
    """W untimed warm-up steps, then EXACTLY `steps` timed steps bracketed by a barrier + device sync on
    both sides; returns (per-step results, max-over-ranks elapsed seconds).  after_warmup: called between the two
    (joins host work that overlapped the warm-up)."""
    for _ in range(warmup):
        step()
    if after_warmup is not None:
        after_warmup()
    if world > 1:
        dist.barrier()
    sync()
    t0 = time.perf_counter()
    out = [step() for _ in range(steps)]
    sync()
    if world > 1:
        dist.barrier()
    return out, max_over_ranks(time.perf_counter() - t0, device)


def ric_bytes_per_solve(prob, nr=2):
    """Algorithmic HBM bytes of one instance's Newton solve in k_ric, from the stage layouts
    of nlot_solver.hip: per knot it reads hg = [H | g0 g1] and [A B 0 | c] | M once, writes the gains
    [K | k0 k1 | Kn] and the value function [P | p0 p1 | Gamma] and reads them back in the forward sweep,
    and writes the step (dx, du, ds, y) of each of the nr right-hand sides."""
    nx, nu = prob.nx, prob.nu
    nz, nv, nc = nx + nu + 1, nu + 1, nx
    nab = (nx + nu + 3) & ~1
    ncol = nx + 2 + nc
    hg, abm, gains, vf = nz * (nz + 2), nx * nab + 4, ncol * nv, nx * ncol
    per_knot = hg + abm + 2 * (gains + vf) + nr * (nx + nu + 1 + nx)
    return 8 * (prob.N + 1) * per_knot


def self_launch(n, argv):
    """`--gpus N` (N > 1) with no launcher around this process (WORLD_SIZE unset): start N ranks on this node, one
    process per GPU, with torch.distributed.run (the driver's own form of the command, rendezvous on 127.0.0.1) as a
    child process, and return its exit code.  Called before anything in this process touches the GPU: the ranks are
    children, never an exec of this process."""
    import socket
    import subprocess

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + list(argv)
    print(f"[bench] --gpus {n}: launching {n} ranks: {' '.join(cmd)}", file=sys.stderr, flush=True)
    return subprocess.call(cmd, env=dict(os.environ, NLOT_BENCH_SELF_LAUNCHED="1"))


def draw_b6(batch, seed, rank):
    """benchmark 6's start / goal, xy + U[-0.05, 0.05]^2, seeded per batch and rank."""
    rng = np.random.default_rng(seed + 1000003 * rank)
    x0 = np.repeat(np.array([BENCHMARKS["b6"]["start"]], float), batch, 0)
    xg = np.repeat(np.array([BENCHMARKS["b6"]["goal"]], float), batch, 0)
    x0[:, :2] += rng.uniform(-0.05, 0.05, (batch, 2))
    xg[:, :2] += rng.uniform(-0.05, 0.05, (batch, 2))
    return x0, xg


def launch_check(a, rank, local, world, backend):
    """--launch-check: what a multi-rank bench run does besides solving.  Each rank draws its own seeded shard (the b6
    rule: no SDF needed), the shards are gathered to rank 0 with the bench's collective (gather_solutions), and rank 0
    prints one JSON line: the ranks the process group initialised, the backend, and the gathered shards."""
    t_dev = "cpu"
    if world > 1 and backend == "nccl":  # RCCL gathers device tensors: one GPU per rank
        torch.cuda.set_device(local)
        t_dev = torch.device("cuda", local)
        dist.init_process_group("nccl", device_id=t_dev)
    elif world > 1:
        dist.init_process_group(backend)
    x0, _ = draw_b6(a.batch or 2, a.seed, rank)
    g = gather_solutions({"x0": torch.as_tensor(x0, device=t_dev)}, keys=("x0",))
    pg_world = dist.get_world_size() if dist.is_initialized() else 1
    if rank == 0:
        print(json.dumps({"n_gpus": world, "process_group_world_size": pg_world, "backend": backend if world > 1 else None,
                          "self_launched": os.environ.get("NLOT_BENCH_SELF_LAUNCHED") == "1",
                          "x0": g["x0"].cpu().tolist()}), flush=True)
    if world > 1:
        dist.destroy_process_group()


def main():
    a = parse()
    if "WORLD_SIZE" not in os.environ and a.gpus > 1:
        sys.exit(self_launch(a.gpus, sys.argv[1:]))
    rank, local, world = rank_world()
    if world != a.gpus:  # the line's n_gpus is the ranks that ran: a mismatch is an error, not a relabelling
        print(f"[bench] --gpus {a.gpus} but the launcher started {world} rank(s) (WORLD_SIZE)", file=sys.stderr, flush=True)
        sys.exit(2)
    # NLOT_DIST_BACKEND=gloo: a rehearsal of the multi-rank path with several ranks sharing the visible GPUs
    # (local rank modulo the device count; CPU collectives); the driver's multi-GPU runs use RCCL ("nccl")
    backend = os.environ.get("NLOT_DIST_BACKEND", "nccl")
    if a.launch_check:
        return launch_check(a, rank, local, world, backend)
    ndev = torch.cuda.device_count()  # does not initialise the GPU on this image
    if backend != "nccl":
        local = local % max(ndev, 1)
    elif world > 1 and world > ndev:
        print(f"[bench] {world} ranks over RCCL need {world} GPUs; {ndev} visible", file=sys.stderr, flush=True)
        sys.exit(2)
    torch.cuda.set_device(local)
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    pg = {"world_size": dist.get_world_size() if dist.is_initialized() else 1,
          "backend": dist.get_backend() if dist.is_initialized() else None,
          "launcher": "bench.py --gpus (torch.distributed.run child)" if os.environ.get("NLOT_BENCH_SELF_LAUNCHED") == "1"
          else "torch.distributed.run" if world > 1 else "single process"}
    assert pg["world_size"] == world == a.gpus, pg
    dev = torch.device("cuda", local)
    stress, b6 = a.workload == "stress", a.workload == "b6"
    if a.batch is None:
        a.batch = 8192 if stress else 16384 if b6 else 32768
    if a.cpu_sample is None:  # about 10-30 s of oracle work on the box's 16 threads (metric: inside the warm-up)
        a.cpu_sample = 16 if stress else 32
    if a.cpu_sample_1core is None:
        a.cpu_sample_1core = 1 if stress else 2
    prob = STRESS_PROBLEM if stress else B6_PROBLEM if b6 else METRIC_PROBLEM
    if b6:
        wpath = os.path.join(ROOT, "nlotrajectories_amd", "data", "b6_mlp128_seed0.npz")
        w = MlpWeights.load(wpath)  # trained by scripts/train_sdf.py (NNObstacleTrainer restatement, seed 0)
    else:
        w = MlpWeights.stress_sdf_mlp(seed=0) if stress else MlpWeights.artefact()
    mlp = DeviceMlp(w)
    streaming = w.hidden == 256 or w.n_hidden > 2  # nlot_mlp.hip launch_mlp_strided dispatch

    def sdf_gpu(pts):
        v, _, _ = sdf_mlp_eval(mlp, torch.as_tensor(pts, dtype=torch.float32, device=dev), derivatives=False)
        return v.cpu().numpy()

    def draw(k):  # batch k (warm-up batches first, then the timed ones): a distinct seeded draw per batch and rank
        if b6:  # benchmark 6's start / goal, xy +- U[-0.05, 0.05]^2
            x0, xg = draw_b6(a.batch, a.seed + k, rank)
        else:  # start/goal uniform in [-0.3, 1.3]^2, all corners sdf >= 0.02
            x0, xg = sample_start_goal(prob, a.batch, seed=a.seed + k, sdf=sdf_gpu, rank=rank)
        return (torch.tensor(x0, dtype=torch.float64, device=dev), torch.tensor(xg, dtype=torch.float64, device=dev))

    batches = [draw(k) for k in range(a.warmup + a.steps)]  # resident in HBM before the timed region
    x0, xg = batches[a.warmup]  # the first timed batch (CPU baseline sample)
    opt = _abi.gpu_options() if a.mu_strategy == "adaptive" else \
        _abi.gpu_options(mu_strategy=0, barrier_tol_factor=10.0)
    opt.general_bounds = 1 if a.bounds == "rows" else 0

    from nlotrajectories_amd.solver import workspace_bytes

    # continuous batching: the K timed batches stream through ONE solve call with `slots` concurrent slots (the
    # workspace holds the slots' state, not the instances': ABI v10), so the latency-bound tail is paid once; the
    # per-instance iterations are the same as in one call per batch
    cont = a.continuous == "on" and not b6 and a.steps > 1
    slots = a.slots or (65536 if not (stress or b6) else a.batch)
    G, calls = batch_calls(a.steps, cont, a.steps)
    ws = torch.empty(max(workspace_bytes(prob, a.batch * G, slots if cont else 0),
                         workspace_bytes(prob, a.batch * max(a.warmup, 1), slots)), dtype=torch.uint8, device=dev)
    opt_cont = _abi.gpu_options(**{f: getattr(opt, f) for f, _ in opt._fields_})
    opt_cont.max_active = slots
    agg_keys = ("mlp_full_ms", "mlp_full_launches", "mlp_points_full", "mlp_value_ms", "mlp_value_launches",
                "mlp_points_value", "iterations", "iterate_ms", "mlp_points_full_reused", "ric_ms", "ric_launches",
                "ric_solves", "ric_soc_solves", "ric_resto_solves", "filter_forgotten", "timed_steps",
                "timed_points_full", "timed_points_full_reused", "timed_points_value", "timed_ric_solves")
    agg = {k: 0 for k in agg_keys}
    agg["filter_peak"] = 0  # max over the timed calls
    timing = {"on": False}

    nstep = {"n": 0}

    call_iter = {"i": 0}
    t_solve = {"s": 0.0}  # this rank's own solve-call time inside the timed region (straggler balance)

    def step(first, g=1):
        X_init = None
        bx0 = torch.cat([batches[first + i][0] for i in range(g)])
        bxg = torch.cat([batches[first + i][1] for i in range(g)])
        if b6:  # benchmark 6's own initializer: RRT against the exact ring scene (YAML rrt settings), timed
            X_init, _ = rrt_initial_guess(prob, bx0, bxg, bounds=[[0.0, 0.0], [1.3, 1.3]], step_size=0.02,
                                          max_iter=5000, margin=0.01, seed=a.seed + first + 7919 * rank)
        t0 = time.perf_counter()
        if g > 1:  # g batches through a.batch slots
            r = solve_batch(prob, bx0, bxg, mlp=mlp, options=opt_cont, workspace=ws)
        else:
            r = solve_batch(prob, bx0, bxg, mlp=mlp, options=opt, workspace=ws, X_init=X_init)
        if timing["on"]:
            torch.cuda.synchronize()
            t_solve["s"] += time.perf_counter() - t0
        nstep["n"] += 1
        print(f"[bench] rank {rank} solve {nstep['n']} done", file=sys.stderr, flush=True)
        if timing["on"]:
            st = last_stats()
            for k in agg_keys:
                agg[k] += st[k]
            agg["filter_peak"] = max(agg["filter_peak"], st["filter_peak"])
            agg["filter_capacity"] = st["filter_capacity"]
        if world > 1:  # gather the solutions to rank 0 (RCCL over xGMI): the only collective
            gather_solutions(r, keys=("X", "U", "cost", "status"))
        return r

    def sync():
        torch.cuda.synchronize()
        timing["on"] = not timing["on"]  # hipEvent timing inside the timed steps only
        set_timing(TIMING_EVERY if timing["on"] else 0)

    warm_i = {"i": 0}

    def timed_call():  # the timed region's i-th solve call (the warm-up: its W batches in one call, untimed)
        if not timing["on"]:
            if warm_i["i"] == 0 and cont and a.warmup > 1:
                warm_i["i"] = a.warmup
                return step(0, a.warmup)
            warm_i["i"] += 1
            return step(warm_i["i"] - 1, 1)
        i = call_iter["i"]
        g = calls[i]
        call_iter["i"] += 1
        return step(a.warmup + sum(calls[:i]), g)

    warm_calls = 1 if (cont and a.warmup > 1) else a.warmup  # the W warm-up batches: one continuous call
    # the CPU baseline (rank 0 of a one-rank run, not the stress estimate, which needs the GPU run's iteration counts)
    # overlaps the warm-up: a host thread runs the oracle (ctypes releases the GIL) while the GPU warms up
    cpu_box, cpu_thread = {}, None
    cpu_here = rank == 0 and world == 1 and a.cpu_sample > 0
    if cpu_here and not stress and a.cpu_overlap == "on" and warm_calls > 0:
        import threading

        share, _ = host_cpu_share()
        th = a.cpu_threads or max(1, share - 1)
        x0n, xgn = x0.cpu().numpy(), xg.cpu().numpy()

        def _cpu():
            print("[bench] CPU baseline (oracle), overlapping the warm-up ...", file=sys.stderr, flush=True)
            try:
                cpu_box["r"] = cpu_baseline(prob, w, x0n, xgn, a.cpu_sample, a.cpu_sample_1core, th, opt)
                cpu_box["r"]["overlap"] = ("measured during the untimed GPU warm-up, on one thread fewer than the "
                                           "host share (the solver's launch thread keeps one)")
            except Exception as e:  # pragma: no cover
                cpu_box["r"] = {"error": str(e)}

        cpu_thread = threading.Thread(target=_cpu, daemon=True)
        cpu_thread.start()

    def join_cpu():
        if cpu_thread is not None:
            t = time.perf_counter()
            cpu_thread.join()
            print(f"[bench] CPU baseline joined ({time.perf_counter() - t:.1f} s after the warm-up)", file=sys.stderr,
                  flush=True)

    results, elapsed = timed_loop(timed_call, len(calls), warm_calls, world, sync, dev, after_warmup=join_cpu)
    set_timing(False)
    st_all = torch.cat([x["status"] for x in results]).long()
    it_all = torch.cat([x["iters"] for x in results]).double()
    solved_total = sum_over_ranks(int((st_all == 0).sum().item()), dev)
    iters_solved = [x["iters"][x["status"] == 0].float().mean().item() for x in results if (x["status"] == 0).any()]
    # pooled over the K distinct timed batches of rank 0
    status_counts = torch.bincount(st_all, minlength=len(_abi.STATUS_NAMES)).cpu().numpy().tolist()
    inst_iters = float(it_all.sum().item())  # rank 0's instance-iterations in the timed region
    q = torch.quantile(it_all, torch.tensor([0.5, 0.99], dtype=torch.float64, device=it_all.device)).cpu().tolist()
    rank_rows = gather_rank_rows([rank, t_solve["s"], q[0], q[1], float(it_all.max().item())] + status_counts, dev)

    # rooflines.  Dominant kernel by device time: k_ric (the Newton solve, latency/occupancy-bound fp64 with
    # ~2.8 KB of stage data per knot): HBM roofline on its algorithmic bytes.  The two SDF-MLP launches:
    # split-bf16 MFMA roofline on executed FLOP.
    # the *_ms sums cover the event-timed global steps (one in TIMING_EVERY; each timed step queues ~10 event packets:
    # timing every step cost 1.8 % traj/s, profiles/r05/ab_step_kernel_timing.log): per-launch averages over those
    # steps' launches and the work they did (NlotSolveStats.timed_*, ABI v14); per-step totals scale by all / timed
    n_t = max(agg["timed_steps"], 1)
    t_scale = agg["iterations"] / n_t
    n_r = n_t
    ric_avg_ms = agg["ric_ms"] / n_r
    ric_solves_per_launch = agg["timed_ric_solves"] / n_r
    ric_bytes = ric_bytes_per_solve(prob)
    ric_achieved = ric_solves_per_launch * ric_bytes / (ric_avg_ms * 1e-3) / 1e9 if ric_avg_ms > 0 else 0.0
    # SURVEY.md §8d's algorithmic figure per problem-iteration: 2 * 4 * (nvar + ncon) bytes (read + write the
    # primal-dual iterate; ~7 KB at N = 50)
    nvar = (prob.N + 1) * prob.nx + prob.N * prob.nu + (prob.N + 1)
    ncon = prob.nx + prob.N * prob.nx + prob.nx + (prob.N + 1) * (1 if prob.use_slack else len(prob.body))
    alg_bytes = 2 * 4 * (nvar + ncon)
    ric_alg = ric_solves_per_launch * alg_bytes / (ric_avg_ms * 1e-3) / 1e9 if ric_avg_ms > 0 else 0.0
    ric_traffic = None
    # PMC at bench size (B = 65536): scripts/pmc_traffic.sh + scripts/pmc_traffic.py -> profiles/r05/ (the newest
    # round's file that exists)
    tf = next((t for t in (os.path.join(ROOT, "profiles", r, f) for r, f in
                           (("r06", "pmc_traffic_r06_B65536.json"), ("r05", "pmc_traffic_r05u_B65536.json"))
                           ) if os.path.exists(t)), "")
    pmc = None
    if os.path.exists(tf):
        with open(tf) as f:
            pmc = json.load(f)
        ric_traffic = pmc["k_ric"]["hbm_bytes_per_solve"] * ric_solves_per_launch

    flop_pt = w.flops_per_point_fwd_grad  # 67,072 for 2-128-128-1, 789,504 for 2-256x4-1
    flop_fwd = w.flops_per_point_fwd      # 33,536 / 394,752
    mlp_peak = PEAK_F32_MFMA_TFLOPS if streaming else PEAK_SPLIT_TFLOPS
    n_l = n_t
    avg_ms = agg["mlp_full_ms"] / n_l
    reused = agg["timed_points_full_reused"]
    flop_launch = (agg["timed_points_full"] * flop_pt - reused * flop_fwd) / n_l
    achieved = flop_launch / (avg_ms * 1e-3) / 1e12 if avg_ms > 0 else 0.0
    traffic = None
    if pmc is not None:  # HBM bytes per point of the full launch inside the solve at bench size
        traffic = pmc["mlp_full"]["hbm_bytes_per_point"] * agg["timed_points_full"] / n_l
    n_v = n_t
    v_avg_ms = agg["mlp_value_ms"] / n_v
    v_achieved = agg["timed_points_value"] / n_v * flop_fwd / (v_avg_ms * 1e-3) / 1e12 if v_avg_ms > 0 else 0.0

    def committed(path, **fields):
        """A figure read from a committed profile (not measured by this run): tagged with its file."""
        return dict(fields, source=os.path.relpath(path, ROOT), measured_in_this_run=False)

    def rocprof_avg(name):
        """The kernel's average dispatch duration in the committed rocprofv3 --kernel-trace --stats run of the driver's
        command (the event brackets of this run start at the previous launch's end, so they also hold the queue's packet
        processing and the wait for CUs the side streams hold).  Committed, not this run's."""
        import csv

        path = next((p for p in (os.path.join(ROOT, "profiles", r, f"kernel_stats_{t}_K20_W5.csv")
                                 for r, t in (("r06", "r06s"), ("r06", "r06"), ("r05", "r05ao"))) if os.path.exists(p)),
                    None)
        if path is None:
            return None
        with open(path) as fh:
            for row in csv.DictReader(fh):
                if name in row["Name"]:
                    return committed(path, avg_launch_ms=float(row["AverageNs"]) / 1e6, calls=int(row["Calls"]))
        return None

    cpu = cpu_box.get("r")
    if cpu_here and cpu is None:
        print("[bench] CPU baseline (oracle) ...", file=sys.stderr, flush=True)
        if stress:  # per-iteration estimate (cpu_baseline docstring); iterations of ALL instances per solved one
            tot_it = sum(int(x["iters"].sum().item()) for x in results)
            n_solved = max(sum(int((x["status"] == 0).sum().item()) for x in results), 1)
            cpu = cpu_baseline(prob, w, x0.cpu().numpy(), xg.cpu().numpy(), a.cpu_sample, a.cpu_sample_1core,
                               a.cpu_threads, opt, iter_cap=10, gpu_iters_per_solved=tot_it / n_solved)
        else:
            cpu = cpu_baseline(prob, w, x0.cpu().numpy(), xg.cpu().numpy(), a.cpu_sample, a.cpu_sample_1core,
                               a.cpu_threads, opt)
    if cpu and "ips" in cpu and not cpu.get("estimate"):
        # the sample's traj/s depends on which statuses its few instances draw (a 32-instance sample holds 10-20
        # solved ones): also the measured instance-iteration rate over the GPU run's instance-iterations per solved
        # instance, i.e. the CPU time of this run's whole status mix (an estimate, reported beside the value)
        tot_it = sum(int(x["iters"].sum().item()) for x in results)
        n_solved = max(sum(int((x["status"] == 0).sum().item()) for x in results), 1)
        cpu["full_mix_estimate"] = {
            "value": cpu["ips"] / (tot_it / n_solved), "unit": "trajectories/s", "cores": cpu["cores"],
            "note": f"{cpu['ips']:.1f} instance-iterations/s (the sample) / {tot_it / n_solved:.0f} instance-iterations "
                    f"per solved instance over rank 0's {len(results)} timed call(s)"}

    if rank == 0:
        B_all = a.batch * world
        H, L = w.hidden, w.n_hidden
        kname = (f"mlp_stream<{H},%s> (f32 MFMA 16x16x4, weights streamed through LDS half a layer at a time)"
                 if streaming else f"mlp_bf16<{H},%s> (fp32-equivalent products as 6 split v_mfma_f32_32x32x16_bf16)")
        ric = {
            "kernel": "k_ric (lane-group Riccati Newton solve, fp64)",
            "bound": "hbm",
            # SURVEY.md §8d's algorithmic bytes per problem-iteration (2 * 4 * (nvar + ncon): read + write the
            # primal-dual iterate) x the solves of one launch / this run's event-timed launch average
            "achieved": ric_alg,
            "peak": PEAK_HBM_GBS,
            "unit": "GB/s",
            "frac": ric_alg / PEAK_HBM_GBS,
            "traffic": ric_traffic if not stress else None,
            "algorithmic_bytes_per_solve": alg_bytes,
            "basis": "SURVEY.md §8d algorithmic bytes (2 * 4 * (nvar + ncon) per problem-iteration) per launch / the "
                     "event-timed average launch (hipEvents on the solver's stream, this run)",
            "design_bytes": {"bytes_per_solve": ric_bytes, "achieved": ric_achieved, "frac": ric_achieved / PEAK_HBM_GBS,
                             "note": "the stage layouts k_ric reads and writes (bench.ric_bytes_per_solve, DESIGN.md §7: "
                                     "H, g, A, B, c, M in; gains and value function out and back; 2 right-hand sides)"},
            "solves_per_launch": ric_solves_per_launch,
            "avg_launch_ms": ric_avg_ms,
            "rocprof": rocprof_avg("k_ric<3, false, false>") if not (stress or b6) else None,
            "launches": agg["ric_launches"],
            "timed_launches": agg["timed_steps"],
            "side_stream_solves": {"second_order_corrections": agg["ric_soc_solves"],
                                   "restoration": agg["ric_resto_solves"],
                                   "factorisations_main": agg["ric_solves"]},
            "note": "the kernel is fp64-latency/occupancy-bound; HBM is its roofline.  The second-order corrections "
                    "(substitution with the stored factors, k_ric<DYN, false, true>) and the restoration solves run on "
                    "side streams and are not counted in this launch's solves",
            "traffic_source": (committed(tf, hbm_bytes_per_solve=pmc["k_ric"]["hbm_bytes_per_solve"],
                                         ratio_to_design_bytes=pmc["k_ric"]["ratio_to_algorithmic"],
                                         note="PMC FETCH_SIZE x2 + WRITE_SIZE at B = 65536 (scripts/pmc_traffic.sh); "
                                              "traffic = that x this run's solves per launch")
                               if pmc else "no PMC traffic file"),
        }
        mlp_full = {
            "kernel": kname % "full" + ": SDF-MLP value + gradient + Hessian",
            "bound": "mfma",
            "achieved": achieved,
            "peak": mlp_peak,
            "unit": "TFLOP/s",
            "frac": achieved / mlp_peak,
            "peak_note": PEAK_F32_MFMA_NOTE if streaming else
                         "dense bf16 MFMA peak 2500 TFLOP/s / 6 split products per fp32-equivalent product; "
                         "the f32-input MFMA peak would be 157.3",
            "traffic": traffic if not stress else None,
            "flop_per_point": flop_pt,
            "forward_reused_frac": agg["mlp_points_full_reused"] / max(agg["mlp_points_full"], 1),
            "flop_counting": f"executed: {flop_pt:,} per point (2-{H}x{L + 1}-1 forward + reverse sweep), less the "
                             f"{flop_fwd:,} forward where it was reused",
            "points_per_launch": agg["timed_points_full"] / n_l,
            "avg_launch_ms": avg_ms,
            "launches": agg["mlp_full_launches"],
            "timed_launches": agg["timed_steps"],
            "traffic_source": (committed(tf, hbm_bytes_per_point=pmc["mlp_full"]["hbm_bytes_per_point"],
                                         ratio_to_algorithmic_with_reuse=pmc["mlp_full"]["ratio_to_algorithmic_with_reuse"],
                                         note="PMC in the solve at B = 65536; traffic = that x this run's points per "
                                              "launch (coordinates, the trial's coordinates, value and ReLU pattern in; "
                                              "value + gradient + Hessian out)") if pmc else "no PMC traffic file"),
        }
        mlp_value = {
            "kernel": kname % "value" + ": line-search trial points, value only",
            "bound": "mfma",
            "achieved": v_achieved,
            "peak": mlp_peak,
            "unit": "TFLOP/s",
            "frac": v_achieved / mlp_peak,
            "flop_per_point": flop_fwd,
            "points_per_launch": agg["timed_points_value"] / n_v,
            "avg_launch_ms": v_avg_ms,
            "launches": agg["mlp_value_launches"],
            "timed_launches": agg["timed_steps"],
        }
        if os.environ.get("NLOT_EARLY_VALUE", "1") != "0" and not streaming:
            note = ("per step, the value launch runs in two parts, the first on a fourth stream concurrently with the "
                    "step's evaluations and Newton solves (NLOT_EARLY_VALUE, default since round 4: +1.3 %% traj/s); "
                    "avg_launch_ms sums both parts' event-timed durations, which include that overlap, so frac is a "
                    "lower bound on the kernel's own (0.479 on standalone 3.3 M-point launches, scripts/mlp_bench.py)")
            mlp_value["overlap_note"] = note.replace("%%", "%")
            mlp_full["overlap_note"] = ("the full launch shares the CUs with the early value launch of the previous "
                                        "step's candidates (fourth stream); its event-timed duration includes that")
        # per-dispatch fractions from the profiler (the event brackets above include the streams' overlap): committed
        # from a rocprofv3 --kernel-trace --stats run of this command (scripts/rocprof_fracs.py)
        df = next((d for d in (os.path.join(ROOT, "profiles", r, f"mlp_dispatch_fracs_{t}.json")
                               for r, t in (("r06", "r06s"), ("r06", "r06"), ("r05", "r05ao"))) if os.path.exists(d)), "")
        if os.path.exists(df) and not (stress or b6):
            with open(df) as fh:
                dd = json.load(fh)
            src = os.path.relpath(df, ROOT)
            mlp_full["rocprof_dispatch_frac"] = committed(df, frac=dd["full"]["frac"],
                                                          avg_dispatch_ms=dd["full"]["avg_dispatch_ms"])
            mlp_value["rocprof_dispatch_frac"] = committed(df, frac=dd["value"]["frac"],
                                                           avg_step_ms=dd["value"]["avg_step_ms"])
        # the dominant kernel by device time: k_ric on the metric workload, the SDF-MLP on the stress workload
        if stress:
            rooflines = {"roofline": mlp_full, "roofline_mlp_value": mlp_value, "roofline_ric": ric}
        else:
            rooflines = {"roofline": ric, "roofline_mlp_full": mlp_full, "roofline_mlp_value": mlp_value}
        line = {
            "metric": "solved trajectories/sec (stress: 256-knot unicycle + 2-256x4-1 SDF MLP)" if stress else
                      "solved trajectories/sec (b6: 101-knot Ackermann 2nd-order + ring-corridor learned SDF)" if b6
                      else "solved trajectories/sec (50-knot unicycle+learned-SDF)",
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
            "data": "synthetic start/goal (seeded, SURVEY.md §8d); learned SDF = " +
                    ("seeded kaiming-uniform 2-256x4-1 ReLU net, output bias centred (MlpWeights.stress_sdf_mlp)"
                     if stress else "2-128-128-1 ReLU net trained on benchmark 6's rings by the NNObstacleTrainer "
                     "restatement (seed 0, nlotrajectories_amd/data/b6_mlp128_seed0.npz)" if b6
                     else "reference artefact weights"),
            "config": {
                "workload": ("stress (BASELINE.json configs[4]): unicycle_2nd, rect 0.2x0.08, N=256, dt 0.1, rho=10, "
                             "bounds +-1, SDF MLP 2-256x4-1 ReLU (3 HxH layers), linear init, IPOPT tol 1e-4")
                            if stress else
                            ("b6 (BASELINE.json configs[3]): ackermann_2nd L=0.05, rect 0.08x0.05, N=100, dt 0.05, no "
                             "slack (per-corner sdf >= 0), smooth w=0.5, bounds [+-1, +-2], learned SDF of 4 "
                             "elliptical half rings, RRT init (the YAML's: bounds [0, 1.3]^2, step 0.02, max_iter 5000, "
                             "margin 0.01; inside the timed step), IPOPT tol 1e-4") if b6 else
                            "metric NLP: unicycle_2nd, rect 0.2x0.08, N=50, rho=10, bounds +-1, "
                            "learned SDF FourierMLP 2-128-128-1 (artefact), linear init, IPOPT tol 1e-4",
                "mu_strategy": a.mu_strategy,
                "bounds": ("constraint rows (general_bounds = 1): opti.bounded(umin, U, umax) and slack >= 0 as IPOPT "
                           "sees them from CasADi's Opti (runner.py:67-69,101-103), U and S free"
                           if opt.general_bounds else "variable bounds on U and S (general_bounds = 0)"),
                "instances_per_gpu": a.batch,
                "global_batch": B_all,
                "knots": prob.N + 1,
                "parallelism": f"instances sharded over {world} GPU(s); RCCL gather of solutions to rank 0",
                "process_group": pg,
                "scheduling": (f"continuous batching: the {a.steps} timed batches of {a.batch} instances in "
                               f"{len(calls)} solve call(s) through {slots} concurrent slots (NlotSolverOptions.max_active; "
                               "slot-indexed state, a finished instance's slot goes to the next one); each instance runs "
                               "the same iterations as alone"
                               if cont else "one solve call per batch"),
                "batches": f"{a.steps} distinct seeded draws per rank (seed + k, rank offset), resident in HBM "
                           "before the timed region",
                "solved_per_step_rank0": (int((st_all == 0).sum().item())) / max(a.steps, 1),
                "status_counts_rank0": status_counts,
                "status_counts_note": "summed over rank 0's timed batches",
                "status_rates_rank0": {_abi.STATUS_NAMES[i]: c / max(len(st_all), 1) for i, c in
                                       enumerate(status_counts) if i in _abi.STATUS_NAMES},
                "ipopt_safeguards": ("second-order correction (max_soc 4), watchdog, tiny step, filter reset, soft "
                                     "restoration and the feasibility restoration phase (MinC_1Nrm) all on: IPOPT's "
                                     "defaults (runner.py:113-125)" if opt.resto else
                                     "restoration phase OFF: line-search failures end as line_search_failed"),
                "per_rank": [{"rank": int(rw[0]), "solve_s": rw[1], "iters_p50": rw[2], "iters_p99": rw[3],
                              "iters_max": int(rw[4]), "status_counts": [int(c) for c in rw[5:]]} for rw in rank_rows],
                "mean_iters_solved": float(np.mean(iters_solved)) if iters_solved else 0.0,
                "filters": {"capacity": agg.get("filter_capacity"), "peak_size": agg["filter_peak"],
                            "entries_forgotten": agg["filter_forgotten"],
                            "note": "IPOPT's filters are unbounded lists; 0 forgotten = the GPU's filters behaved as "
                                    "unbounded on every timed instance"},
                "lockstep_global_steps": agg["iterations"] // max(a.steps, 1),
                "solver_step_kernel_ms_per_step": agg["iterate_ms"] * t_scale / max(a.steps, 1),
                "ric_ms_per_step": agg["ric_ms"] * t_scale / max(a.steps, 1),
                "mlp_ms_per_step": (agg["mlp_full_ms"] + agg["mlp_value_ms"]) * t_scale / max(a.steps, 1),
                "event_timing": f"hipEvents on one global step in {TIMING_EVERY} ({agg['timed_steps']} of "
                                f"{agg['iterations']} steps); the *_ms_per_step figures scale their sums by all / timed",
                "instance_iterations_rank0": inst_iters,
                # SDF-MLP work per instance-iteration (DESIGN.md §8f cost model): points the value launches (line-search
                # candidates, speculative ones included) and the full launches evaluate per accepted iteration
                "value_mlp_points_per_instance_iteration": agg["mlp_points_value"] / max(inst_iters, 1.0),
                "full_mlp_points_per_instance_iteration": agg["mlp_points_full"] / max(inst_iters, 1.0),
            },
            **rooflines,
            "cpu_baseline": cpu,
        }
        print(json.dumps(line))
    if world > 1:
        dist.destroy_process_group()


def host_cpu_share():
    """(cores, note): the CPUs this process may use: min(scheduler affinity, cgroup v2 cpu.max quota, rounded down),
    read at run time (the GPU box's affinity lists the whole machine while its cgroup grants a share)."""
    try:
        avail = len(os.sched_getaffinity(0))
    except AttributeError:  # pragma: no cover
        avail = os.cpu_count() or 1
    quota, note = None, f"os.cpu_count() = {os.cpu_count()}, affinity = {avail}"
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
        if q != "max":
            quota = max(1, int(float(q) / float(per)))
            note += f", cgroup cpu.max = {q} / {per} = {float(q) / float(per):.1f} CPUs"
        else:
            note += ", cgroup cpu.max = max"
    except (OSError, ValueError):
        note += ", no cgroup v2 cpu.max"
    cores = min(avail, quota) if quota else avail
    return cores, note


def cpu_baseline(prob, w, x0, xg, n_all, n_one, threads, opt, iter_cap=None, gpu_iters_per_solved=None):
    """The oracle (C restatement) on bounded samples of the same workload: the first n_all instances of rank 0's
    first timed batch in ONE OpenMP call (dynamic schedule, one instance per thread at a time, so a long-running
    instance holds one thread, not a chunk), on the host's CPU share (host_cpu_share) or `threads`; and the first
    n_one of them on one thread.  Parallel efficiency is compared on instance-iterations per second (the two samples
    differ in status mix).

    iter_cap (the stress workload, where one oracle iteration costs ~1 s of fp32 MLP work on a core): the
    sample runs at most iter_cap iterations per instance, and the value is an ESTIMATE = 1 / (measured
    seconds per instance-iteration x the GPU run's iterations per solved instance), stated in `sample`."""
    try:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle as O
    except Exception as e:  # pragma: no cover
        return {"error": str(e)}
    share, host = host_cpu_share()
    threads = max(1, min(threads, share)) if threads else share
    hm = O.HostMlp(w)
    run_opt = type(opt).from_buffer_copy(opt)
    if iter_cap is not None:
        run_opt.max_iter = iter_cap

    def run(n, th):
        t = time.perf_counter()
        r = O.solve_batch(prob, x0[:n], xg[:n], hm, opt=run_opt, threads=th)
        dt = time.perf_counter() - t
        st, its = r["status"], r["iters"]
        print(f"[bench] cpu baseline: {n} instances on {th} thread(s), {dt:.1f} s", file=sys.stderr, flush=True)
        return int((st == 0).sum()), dt, np.bincount(st, minlength=7).tolist(), int(its.sum())

    ns, dt, sc, it = run(n_all, threads)
    ips = it / dt  # instance-iterations per second
    if iter_cap is None:
        out = {"value": ns / dt, "unit": "trajectories/s", "cores": threads, "kind": "port", "ips": ips,
               "sample": f"first {n_all} instances of rank 0's first timed batch: {ns} solved (status counts {sc}), "
                         f"{it} instance-iterations in {dt:.1f} s on {threads} OpenMP threads (host: {host})"}
    else:
        per_it = dt / max(it, 1)
        out = {"value": 1.0 / (per_it * gpu_iters_per_solved), "unit": "trajectories/s", "cores": threads,
               "kind": "port", "estimate": True,
               "sample": f"first {n_all} instances of rank 0's first timed batch, at most {iter_cap} iterations each: "
                         f"{it} instance-iterations in {dt:.1f} s on {threads} OpenMP threads (host: {host}) = "
                         f"{per_it * 1e3:.1f} ms per instance-iteration; value = 1 / (that x the GPU run's "
                         f"{gpu_iters_per_solved:.1f} iterations per solved instance)"}
    if n_one > 0:
        # single core: instances one at a time on one thread until about 8 s of work (a fixed count of 2-3 instances
        # drew anything from 17 to 2,000 instance-iterations), at least n_one of them
        ns1 = dt1 = it1 = 0
        sc1 = [0] * 7
        n1 = 0
        while n1 < len(x0) and (n1 < n_one or dt1 < 8.0):
            t = time.perf_counter()
            r1 = O.solve_batch(prob, x0[n1:n1 + 1], xg[n1:n1 + 1], hm, opt=run_opt, threads=1)
            dt1 += time.perf_counter() - t
            ns1 += int(r1["status"][0] == 0)
            sc1[int(r1["status"][0])] += 1
            it1 += int(r1["iters"][0])
            n1 += 1
        n_one = n1
        print(f"[bench] cpu baseline: {n1} instances on 1 thread, {dt1:.1f} s", file=sys.stderr, flush=True)
        ips1 = it1 / dt1
        out["parallel_efficiency"] = ips / (threads * ips1)
        out["efficiency_note"] = (f"instance-iterations/s: {ips:.1f} on {threads} threads vs {ips1:.2f} on 1 thread")
        if iter_cap is None:
            # a 3-instance sample's traj/s depends on which statuses it draws (half the instances run 1000
            # iterations): the single-core value is the measured instance-iteration rate x the multi-thread sample's
            # instance-iterations per solved instance; the direct figure is kept as indicative
            it_per_solved = it / max(ns, 1)
            out["single_core"] = {"value": ips1 / it_per_solved, "cores": 1,
                                  "sample": f"{ips1:.2f} instance-iterations/s on 1 thread (first {n_one} instances, "
                                            f"{it1} instance-iterations in {dt1:.1f} s) / {it_per_solved:.0f} "
                                            f"instance-iterations per solved instance (the {n_all}-instance sample)",
                                  "direct_indicative": {"value": ns1 / dt1, "solved": ns1, "status_counts": sc1}}
        else:
            out["single_core"] = {"value": 1.0 / (dt1 / max(it1, 1) * gpu_iters_per_solved), "cores": 1,
                                  "estimate": True,
                                  "sample": f"first {n_one} instances, at most {iter_cap} iterations: {it1} "
                                            f"instance-iterations in {dt1:.1f} s on 1 thread"}
    return out


if __name__ == "__main__":
    main()
