"""A/B check of two in-tree builds of libnlot.so on the same seeded metric batch.

    NLOT_LIB=libnlot_v10.so python scripts/ab_solve.py run out_a.npz [B]
    python scripts/ab_solve.py run out_b.npz [B]
    python scripts/ab_solve.py cmp out_a.npz out_b.npz

`run` solves B instances of the metric workload (bench.py's sampler, seed 0) and stores statuses,
iterations, costs and trajectories; `cmp` reports how far two runs differ.
"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def run(out, B):
    import torch

    from nlotrajectories_amd import _abi
    from nlotrajectories_amd.nn import MlpWeights
    from nlotrajectories_amd.ops import DeviceMlp, sdf_mlp_eval
    from nlotrajectories_amd.problem import METRIC_PROBLEM
    from nlotrajectories_amd.sampling import sample_start_goal
    from nlotrajectories_amd.solver import solve_batch

    mlp = DeviceMlp(MlpWeights.artefact())

    def sdf(pts):
        return sdf_mlp_eval(mlp, torch.as_tensor(pts, dtype=torch.float32, device="cuda"), derivatives=False)[0].cpu().numpy()

    x0, xg = sample_start_goal(METRIC_PROBLEM, B, seed=0, sdf=sdf)
    res = {}
    for name, opt in (("adaptive", _abi.gpu_options()),
                      ("monotone", _abi.gpu_options(mu_strategy=0, barrier_tol_factor=10.0))):
        torch.cuda.synchronize()
        t = time.perf_counter()
        r = solve_batch(METRIC_PROBLEM, x0, xg, mlp=mlp, options=opt)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t
        for k in ("X", "U", "cost", "status", "iters"):
            res[f"{name}_{k}"] = r[k].cpu().numpy()
        print(f"{name}: B={B} {dt:.2f} s solved {(res[name + '_status'] == 0).sum()} "
              f"status {np.bincount(res[name + '_status'], minlength=4).tolist()}", flush=True)
    np.savez(out, **res)


def cmp(a, b):
    A, Bz = np.load(a), np.load(b)
    for name in ("adaptive", "monotone"):
        sa, sb = A[f"{name}_status"], Bz[f"{name}_status"]
        ia, ib = A[f"{name}_iters"], Bz[f"{name}_iters"]
        same = (sa == sb) & (ia == ib)
        dX = np.abs(A[f"{name}_X"] - Bz[f"{name}_X"]).reshape(len(sa), -1).max(1)
        dc = np.abs(A[f"{name}_cost"] - Bz[f"{name}_cost"])
        print(f"{name}: status+iters equal {same.mean():.4f}; max|dX| (equal ones) "
              f"median {np.median(dX[same]):.2e} max {dX[same].max():.2e}; max|dcost| {dc[same].max():.2e}; "
              f"solved {(sa == 0).sum()} vs {(sb == 0).sum()}")


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run(sys.argv[2], int(sys.argv[3]) if len(sys.argv) > 3 else 4096)
    else:
        cmp(sys.argv[2], sys.argv[3])
