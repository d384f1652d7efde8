#!/usr/bin/env python3
"""Oracle outcome fixtures for the solve-level GPU parity tests whose oracle runs are too long for a GPU test.

    python tests/golden/make_oracle_outcomes.py [--threads 8] [--form rows|varbounds] [--only metric|b6]
    python tests/golden/make_oracle_outcomes.py --form rows|varbounds --add-stpin   (adds {case}_stpin to a file)
    python tests/golden/make_oracle_outcomes.py --form rows|varbounds --add-wide    (adds b6_wide_* to a file)
        rows (default):  tests/golden/oracle_outcomes.npz            (the reference's constraint-row bounds)
        varbounds:       tests/golden/oracle_outcomes_varbounds.npz  (the same bounds as variable bounds)

For each case it stores the instances (x0, xg, and the initial guesses where the case has its own) and the CPU
oracle's status / final cost / iterations / final-iterate deviation under tests/outcomes.PERTURBATIONS (x0,
x0 +- 1e-13 e_x, x0 +- 1e-13 e_y, and the net summed in reverse order), with IPOPT's settings (default_options:
max_iter 1000, tol 1e-4, adaptive mu, restoration on; general_bounds by --form):

  metric: 128 seeded instances of the headline workload (unicycle_2nd, b3 body, N = 50, artefact FourierMLP; the
          first 128 start/goal pairs of sample_start_goal(seed 0));
  b6:     24 benchmark-6 instances (BASELINE configs[3]: N = 100, the trained ring SDF) from the YAML's RRT initial
          guess, computed by the oracle's RRT restatement (oracle/rrt_oracle.py) and stored, so that the GPU test
          starts both solvers from the identical guess.

Per-instance pinned iterates: every run records its iterate at the top of each iteration
(oracle_solve_trace).  For instance i, k_i is the last iteration (at most PIN_CAP = 200, at most the shortest of its
six runs) up to which all five perturbed runs stay within PIN_TOL (max |dX|, |dU|) of the unperturbed run: 1e-5 on
these learned-SDF cases (the reverse-order run changes the fp32 net's outputs at the rounding level, which the
iterates feel at ~1e-7..1e-6 from the first iterations; 1e-5 keeps a 10x margin under the GPU test's 1e-4, the
fp32-MLP iterate tolerance of DESIGN.md §5);
{case}_kpin[i] = k_i, {case}_Xpin / _Upin = the unperturbed iterate at k_i (what max_iter = k_i returns),
{case}_pin_spread = the perturbed runs' largest deviation up to k_i, {case}_stpin = the unperturbed run's status at
max_iter = k_i (max_iter, or the final status where the run ends at the top of iteration k_i: converged, or a
restoration phase that converged to a point the filter rejects; a restoration line-search failure at k_i = iters
happens inside iteration k_i and so returns max_iter).  A GPU test runs every instance to k_i — failed and chaotic
instances included — and compares the iterate and the status.  {case}_trials: the run's trial-point evaluations (IPOPT's
sequential backtracking: one SDF value evaluation of the trial's corners each; DESIGN.md §8f cost model).

b6_wide_status / b6_wide_cost / b6_wide_iters [12, 24]: the b6 instances under tests/outcomes.WIDE (x0 +- 1e-11,
1e-9, 1e-7 e_x, e_y): the oracle's own outcome spread at the size of the GPU's rounding differences (its fp32 net
sums in other orders, its fp64 reductions and Riccati sweeps in other orders in every iteration), against which the
GPU's chaotic b6 outcomes are measured (tests/outcomes.py).

The oracle is deterministic (one instance per thread, no reductions across threads), so the GPU box's oracle
build reproduces these numbers bitwise; tests/test_oracle_outcomes_fixture.py re-runs a few instances on the CPU
to catch a fixture that no longer matches the oracle.  Test infrastructure: it imports the oracle only."""
import argparse
import os
import sys
import time
from concurrent.futures import ThreadPoolExecutor

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

PIN_CAP = 200
PIN_TOL = 1e-5
OUT = {"rows": os.path.join(HERE, "oracle_outcomes.npz"),
       "varbounds": os.path.join(HERE, "oracle_outcomes_varbounds.npz")}


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


def pin(trace0, dev, iters):
    """k_i, and the perturbed runs' largest deviation up to it: dev [m, n, cap] per-iteration deviations of the
    perturbed runs (row 0 unused), iters [m, n] final iterations."""
    m, n, cap = dev.shape
    kpin = np.zeros(n, np.int32)
    spread = np.zeros(n)
    for i in range(n):
        kmax = min(PIN_CAP, cap - 1, int(iters[:, i].min()))
        d = np.nanmax(dev[1:, i, :kmax + 1], axis=0)
        bad = np.nonzero(~(d <= PIN_TOL))[0]
        k = kmax if len(bad) == 0 else int(bad[0]) - 1
        kpin[i] = max(k, 0)
        spread[i] = float(np.nanmax(d[:kpin[i] + 1]))
    return kpin, spread


def pin_status(O, prob, X0, XG, hm, opt, Xi, kpin, threads):
    """The unperturbed run's status at max_iter = k_i, per instance."""
    def one(i):
        o = type(opt).from_buffer_copy(opt)
        o.max_iter = int(kpin[i])
        return O.solve_one(prob, X0[i], XG[i], hm, opt=o, X_init=None if Xi is None else Xi[i])["status"]

    with ThreadPoolExecutor(threads) as ex:
        return np.array(list(ex.map(one, range(len(X0)))), np.int32)


def run_case(O, prob, X0, XG, hm, opt, Xi, threads):
    """Outcomes under every perturbation, with the per-instance pinned iterates."""
    from outcomes import PERTURBATIONS, mlp_order

    n, m = len(X0), len(PERTURBATIONS)

    def one(args):  # one perturbation of one instance (ctypes releases the GIL)
        i, (c, d, _) = args
        x = X0[i].copy()
        x[c] += d
        return O.solve_trace(prob, x, XG[i], hm, opt=opt, X_init=None if Xi is None else Xi[i], cap=PIN_CAP + 1)

    st = np.zeros((m, n), np.int32)
    trials = np.zeros((m, n), np.int32)
    cost = np.zeros((m, n))
    its = np.zeros((m, n), np.int32)
    xdev = np.zeros((m, n))
    dev = np.full((m, n, PIN_CAP + 1), np.nan)
    XU0, T0 = None, None
    with ThreadPoolExecutor(threads) as ex:
        for p, pd in enumerate(PERTURBATIONS):  # one batch per perturbation: the net's summation order is process-wide
            if pd[2] and hm is None:  # no net: the reverse-order run is the unperturbed run
                st[p], cost[p], its[p], xdev[p], dev[p], trials[p] = st[0], cost[0], its[0], xdev[0], 0.0, trials[0]
                continue
            with mlp_order(pd[2]):
                rs = list(ex.map(one, [(i, pd) for i in range(n)]))
            XU = np.stack([np.concatenate([np.ravel(r["X"]), np.ravel(r["U"])]) for r in rs])
            T = np.stack([r["trace"] for r in rs])
            if XU0 is None:
                XU0, T0 = XU, T
            st[p] = [r["status"] for r in rs]
            cost[p] = [r["cost"] for r in rs]
            its[p] = [r["iters"] for r in rs]
            trials[p] = [r["trials"] for r in rs]
            xdev[p] = np.abs(XU - XU0).max(1)
            dev[p] = np.abs(T - T0).max(2)
    kpin, spread = pin(T0, dev, its)
    N, nx, nu = prob.N, prob.nx, prob.nu
    XUp = T0[np.arange(n), kpin]
    stpin = pin_status(O, prob, X0, XG, hm, opt, Xi, kpin, threads)
    return {"status": st, "cost": cost, "iters": its, "xdev": xdev, "trials": trials, "kpin": kpin, "pin_spread": spread,
            "stpin": stpin,
            "Xpin": XUp[:, :(N + 1) * nx].reshape(n, N + 1, nx), "Upin": XUp[:, (N + 1) * nx:].reshape(n, N, nu)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--threads", type=int, default=8)
    ap.add_argument("--form", default="rows", choices=list(OUT))
    ap.add_argument("--out", default=None)
    ap.add_argument("--only", default=None, help="metric | b6 (keeps the other case from an existing file)")
    ap.add_argument("--add-stpin", action="store_true", help="add {case}_stpin to an existing file")
    ap.add_argument("--add-wide", action="store_true", help="add b6_wide_* (outcomes under WIDE) to an existing file")
    a = ap.parse_args()
    out_path = a.out or OUT[a.form]
    import oracle as O
    from nlotrajectories_amd import _abi
    from nlotrajectories_amd.nn import MlpWeights
    from nlotrajectories_amd.problem import B6_PROBLEM, METRIC_PROBLEM

    opt = _abi.default_options(general_bounds=1 if a.form == "rows" else 0)
    data = dict(np.load(out_path)) if (a.only and os.path.exists(out_path)) else {}
    data["general_bounds"] = np.array(opt.general_bounds)

    if a.add_wide:
        from outcomes import WIDE

        data = dict(np.load(out_path))
        opt = _abi.default_options(general_bounds=int(data["general_bounds"]))
        hm6 = O.HostMlp(MlpWeights.load(os.path.join(ROOT, "nlotrajectories_amd", "data", "b6_mlp128_seed0.npz")))
        X0, XG, Xi = data["b6_x0"], data["b6_xg"], data["b6_xinit"]
        n, m = len(X0), len(WIDE)
        t = time.time()

        def one(args):
            i, (c, d, _) = args
            x = X0[i].copy()
            x[c] += d
            r = O.solve_one(B6_PROBLEM, x, XG[i], hm6, opt=opt, X_init=Xi[i])
            return r["status"], r["cost"], r["iters"]

        with ThreadPoolExecutor(a.threads) as ex:
            rs = list(ex.map(one, [(i, pd) for pd in WIDE for i in range(n)]))
        data["b6_wide_status"] = np.array([r[0] for r in rs], np.int32).reshape(m, n)
        data["b6_wide_cost"] = np.array([r[1] for r in rs]).reshape(m, n)
        data["b6_wide_iters"] = np.array([r[2] for r in rs], np.int32).reshape(m, n)
        print(f"b6 wide: {time.time() - t:.0f} s, statuses "
              f"{np.bincount(data['b6_wide_status'].ravel(), minlength=7).tolist()}", flush=True)
        np.savez_compressed(out_path, **data)
        return
    if a.add_stpin:
        data = dict(np.load(out_path))
        opt = _abi.default_options(general_bounds=int(data["general_bounds"]))
        hm6 = O.HostMlp(MlpWeights.load(os.path.join(ROOT, "nlotrajectories_amd", "data", "b6_mlp128_seed0.npz")))
        for case, prob, hm, xi in (("metric", METRIC_PROBLEM, O.HostMlp(MlpWeights.artefact()), None),
                                   ("b6", B6_PROBLEM, hm6, data["b6_xinit"])):
            data[f"{case}_stpin"] = pin_status(O, prob, data[f"{case}_x0"], data[f"{case}_xg"], hm, opt, xi,
                                               data[f"{case}_kpin"], a.threads)
            print(case, "stpin", np.bincount(data[f"{case}_stpin"], minlength=7).tolist(), flush=True)
        np.savez_compressed(out_path, **data)
        return

    def report(case, out, t):
        kp = out["kpin"]
        print(f"{case}: {time.time() - t:.0f} s, statuses {np.bincount(out['status'][0], minlength=7).tolist()}, "
              f"k_pin min / median / max {kp.min()} / {int(np.median(kp))} / {kp.max()}", flush=True)

    if a.only in (None, "metric"):
        t = time.time()
        x0, xg = metric_instances()
        out = run_case(O, METRIC_PROBLEM, x0, xg, O.HostMlp(MlpWeights.artefact()), opt, None, a.threads)
        data.update({"metric_x0": x0, "metric_xg": xg, **{f"metric_{k}": v for k, v in out.items()}})
        report("metric", out, t)
    if a.only in (None, "b6"):
        t = time.time()
        X0, XG, Xi = b6_instances()
        hm6 = O.HostMlp(MlpWeights.load(os.path.join(ROOT, "nlotrajectories_amd", "data", "b6_mlp128_seed0.npz")))
        out = run_case(O, B6_PROBLEM, X0, XG, hm6, opt, Xi, a.threads)
        data.update({"b6_x0": X0, "b6_xg": XG, "b6_xinit": Xi, **{f"b6_{k}": v for k, v in out.items()}})
        report("b6", out, t)
    np.savez_compressed(out_path, **data)


if __name__ == "__main__":
    main()
