#!/usr/bin/env python3
"""Oracle outcome fixtures for the solve-level GPU parity tests whose oracle runs are too long for a GPU test.

    python tests/golden/make_oracle_outcomes.py [--threads 8]   ->  tests/golden/oracle_outcomes.npz

For each case it stores the instances (x0, xg, and the initial guesses where the case has its own) and the CPU
oracle's status / final cost / iterations under tests/outcomes.PERTURBATIONS (x0, x0 +- 1e-13 e_x, x0 +- 1e-13 e_y, and
the net summed in reverse order), with IPOPT's settings
(default_options: max_iter 1000, tol 1e-4, adaptive mu, restoration on):

  metric: 128 seeded instances of the headline workload (unicycle_2nd, b3 body, N = 50, artefact FourierMLP; the
          first 128 start/goal pairs of sample_start_goal(seed 0));
  b6:     24 benchmark-6 instances (BASELINE configs[3]: N = 100, the trained ring SDF) from the YAML's RRT initial
          guess, computed by the oracle's RRT restatement (oracle/rrt_oracle.py) and stored, so that the GPU test
          starts both solvers from the identical guess.

The oracle is deterministic (one instance per thread, no reductions across threads), so the GPU box's oracle
build reproduces these numbers bitwise; tests/test_oracle_outcomes_fixture.py re-runs a few instances on the CPU
to catch a fixture that no longer matches the oracle.  Test infrastructure: it imports the oracle only."""
import argparse
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tests"))


def metric_instances(n=128):
    import oracle as O
    from nlotrajectories_amd.nn import MlpWeights
    from nlotrajectories_amd.problem import METRIC_PROBLEM
    from nlotrajectories_amd.sampling import sample_start_goal

    hm = O.HostMlp(MlpWeights.artefact())
    x0, xg = sample_start_goal(METRIC_PROBLEM, n, seed=0, sdf=lambda P: O.mlp_eval(hm, P, want=False)[0])
    return x0, xg


def b6_instances(n=24):
    import rrt_oracle as R
    from nlotrajectories_amd.problem import B6_PROBLEM, BENCHMARKS

    b = BENCHMARKS["b6"]
    rng = np.random.default_rng(4)
    X0 = np.repeat(np.array([b["start"]], float), n, 0)
    XG = np.repeat(np.array([b["goal"]], float), n, 0)
    X0[:, :2] += rng.uniform(-0.05, 0.05, (n, 2))
    XG[:, :2] += rng.uniform(-0.05, 0.05, (n, 2))
    Xi = np.stack([R.rrt_one(B6_PROBLEM, X0[i], XG[i], [[0.0, 0.0], [1.3, 1.3]], step_size=0.02, max_iter=5000,
                             margin=0.01, seed=3, instance=i)[0] for i in range(n)])
    return X0, XG, Xi


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--threads", type=int, default=8)
    ap.add_argument("--out", default=os.path.join(HERE, "oracle_outcomes.npz"))
    ap.add_argument("--only", default=None, help="metric | b6 (keeps the other case from an existing file)")
    a = ap.parse_args()
    import oracle as O
    from outcomes import oracle_outcomes
    from nlotrajectories_amd import _abi
    from nlotrajectories_amd.nn import MlpWeights
    from nlotrajectories_amd.problem import B6_PROBLEM, METRIC_PROBLEM

    opt = _abi.default_options()
    data = dict(np.load(a.out)) if (a.only and os.path.exists(a.out)) else {}
    if a.only in (None, "metric"):
        t = time.time()
        x0, xg = metric_instances()
        out = oracle_outcomes(O, METRIC_PROBLEM, x0, xg, O.HostMlp(MlpWeights.artefact()), opt, threads=a.threads)
        data.update({"metric_x0": x0, "metric_xg": xg, **{f"metric_{k}": v for k, v in out.items()}})
        print(f"metric: {time.time() - t:.0f} s, statuses {np.bincount(out['status'][0], minlength=7).tolist()}",
              flush=True)
    if a.only in (None, "b6"):
        t = time.time()
        X0, XG, Xi = b6_instances()
        hm6 = O.HostMlp(MlpWeights.load(os.path.join(ROOT, "nlotrajectories_amd", "data", "b6_mlp128_seed0.npz")))
        from concurrent.futures import ThreadPoolExecutor

        from outcomes import PERTURBATIONS, mlp_order

        def one(args):  # one perturbation of one instance (ctypes releases the GIL)
            i, (c, d, _) = args
            x = X0[i].copy()
            x[c] += d
            r = O.solve_one(B6_PROBLEM, x, XG[i], hm6, opt=opt, X_init=Xi[i])
            return r["status"], r["cost"], r["iters"], np.concatenate([np.ravel(r["X"]), np.ravel(r["U"])])

        res = []
        with ThreadPoolExecutor(a.threads) as ex:
            for pd in PERTURBATIONS:  # one batch per perturbation: the net's summation order is process-wide
                with mlp_order(pd[2]):
                    res += list(ex.map(one, [(i, pd) for i in range(len(X0))]))
        n, m = len(X0), len(PERTURBATIONS)
        XU = np.stack([r[3] for r in res]).reshape(m, n, -1)
        out = {"status": np.array([r[0] for r in res], np.int32).reshape(m, n),
               "cost": np.array([r[1] for r in res], float).reshape(m, n),
               "iters": np.array([r[2] for r in res], np.int32).reshape(m, n),
               "xdev": np.abs(XU - XU[0]).max(2)}
        data.update({"b6_x0": X0, "b6_xg": XG, "b6_xinit": Xi, **{f"b6_{k}": v for k, v in out.items()}})
        print(f"b6: {time.time() - t:.0f} s, statuses {np.bincount(out['status'][0], minlength=7).tolist()}",
              flush=True)
    np.savez_compressed(a.out, **data)


if __name__ == "__main__":
    main()
