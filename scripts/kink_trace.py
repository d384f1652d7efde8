#!/usr/bin/env python3
"""Why the restated IPOPT runs metric instances to max_iter: a per-instance trace.

For each metric instance the restatement fails, the oracle (default options, unbounded filters) is run with its
iterate dump (NLOT_ORACLE_DUMP: per iteration mu, f, E0, dual infeasibility, primal infeasibility, free / fixed mu
mode, X and the knot multipliers), and the last `--tail` iterations are reduced to:

  * fixed_mode_frac: fraction of iterations in the adaptive strategy's fixed mu mode;
  * mu_median, dual_median: the barrier parameter and the dual infeasibility (the error that never falls below tol);
  * relu_flip_frac: fraction of consecutive iterates between which the hidden-layer ReLU pattern (128 units of the
    artefact FourierMLP) changes at one or more of the 204 footprint corners, and the mean number of flipped units;
  * cycle_ratio: min over lags 2..8 of mean ||X_k - X_{k-lag}|| / mean ||X_k - X_{k-1}|| over the last 50 iterations
    (informational: near 1 means the iterates wander rather than repeat; the mode switches break exact cycles);
  * the same instance solved by the same restatement with the ReLUs replaced by softplus(beta = 1000) (an
    oracle-only diagnostic that smooths each kink over |z| < 1e-3 and changes nothing else): the status it reaches.

The point: with the exact Hessian of a ReLU net (zero second derivative of every ReLU, as libtorch / l4casadi give
it), the Newton model does not see the gradient jumps across kinks; where the optimum (or the barrier problem's
solution) sits on a kink, the full Newton steps the filter accepts oscillate across it and the dual infeasibility
stays at the size of the jump.  IPOPT's published algorithm computes the same Newton steps.

    python scripts/kink_trace.py [--cases crosscheck|N] [--tail 200] [--out profiles/r04/kink_trace.json]

CPU only; test infrastructure (uses oracle/)."""
import argparse
import json
import os
import sys
import tempfile
from concurrent.futures import ProcessPoolExecutor

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))


def _solve(args):
    case, x0, xg, dump, softplus = args
    if dump:
        os.environ["NLOT_ORACLE_DUMP"] = dump
    else:
        os.environ.pop("NLOT_ORACLE_DUMP", None)
    if softplus:
        os.environ["NLOT_ORACLE_SOFTPLUS_BETA"] = "1000"
    import oracle as O
    from nlotrajectories_amd import _abi
    from nlotrajectories_amd.nn import MlpWeights
    from nlotrajectories_amd.problem import METRIC_PROBLEM

    hm = O.HostMlp(MlpWeights.artefact())
    if softplus:
        hm.desc.act = 90  # ORACLE_ACT_SOFTPLUS, oracle-only diagnostic
    r = O.solve_one(METRIC_PROBLEM, np.asarray(x0, float), np.asarray(xg, float), hm, opt=_abi.default_options())
    return case, {"status": _abi.STATUS_NAMES[r["status"]], "iters": r["iters"], "cost": r["cost"],
                  "resto_phases": r["resto_phases"], "watchdogs": r["watchdogs"]}


def reduce(dump, tail):
    from nlotrajectories_amd.nn import MlpWeights
    from nlotrajectories_amd.problem import METRIC_PROBLEM as P

    w = MlpWeights.artefact().arrays
    A, b0, W, b1 = w["A"], w["b0"], w["W"].reshape(128, 128), w["b"].reshape(-1)
    fs = MlpWeights.artefact().fourier_scale
    N, nx = P.N, P.nx
    rec = 8 + (N + 1) * nx + (N + 1)
    d = np.fromfile(dump).reshape(-1, rec)[-tail:]
    hd, X = d[:, :8], d[:, 8:8 + (N + 1) * nx].reshape(-1, N + 1, nx)
    body = np.array(P.body)

    def pattern(Xk):
        c, s = np.cos(Xk[:, 2]), np.sin(Xk[:, 2])
        px = Xk[:, None, 0] + c[:, None] * body[None, :, 0] - s[:, None] * body[None, :, 1]
        py = Xk[:, None, 1] + s[:, None] * body[None, :, 0] + c[:, None] * body[None, :, 1]
        p = np.stack([px, py], -1).reshape(-1, 2)
        h0 = np.cos(p @ A.reshape(2, -1) + b0) * fs
        return (h0 @ W.T + b1) > 0

    pats = [pattern(x) for x in X]
    flips = [int((pats[i] != pats[i - 1]).sum()) for i in range(1, len(pats))]
    step = np.array([np.linalg.norm(X[i] - X[i - 1]) for i in range(1, len(X))])
    last = X[-50:]
    s1 = np.mean([np.linalg.norm(last[i] - last[i - 1]) for i in range(1, len(last))])
    ratios = {lag: float(np.mean([np.linalg.norm(last[i] - last[i - lag]) for i in range(lag, len(last))]) / max(s1, 1e-300))
              for lag in range(2, 9)}
    lag = min(ratios, key=ratios.get)
    return {"tail": len(d), "fixed_mode_frac": float((hd[:, 6] == 0).mean()), "mu_median": float(np.median(hd[:, 1])),
            "dual_median": float(np.median(hd[:, 4])), "primal_median": float(np.median(hd[:, 5])),
            "relu_flip_frac": float(np.mean(np.array(flips) > 0)), "relu_units_flipped_mean": float(np.mean(flips)),
            "step_norm_median": float(np.median(step)), "cycle_lag": lag, "cycle_ratio": ratios[lag]}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cases", default="crosscheck")
    ap.add_argument("--tail", type=int, default=200)
    ap.add_argument("--workers", type=int, default=8)
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "r04", "kink_trace.json"))
    a = ap.parse_args()
    doc = json.load(open(os.path.join(ROOT, "tests", "golden", "crosscheck_scipy.json")))
    cases = [(r["case"], r["x0"], r["xg"], r["trust_constr"]["cost"]) for r in doc["instances"]
             if r["case"].startswith("metric")]
    tmp = tempfile.mkdtemp()
    jobs = [(c, x0, xg, os.path.join(tmp, f"{i}.bin"), False) for i, (c, x0, xg, _) in enumerate(cases)]
    jobs += [(c, x0, xg, None, True) for c, x0, xg, _ in cases]
    with ProcessPoolExecutor(a.workers) as ex:
        res = list(ex.map(_solve, jobs))
    n = len(cases)
    rows = []
    for i, (c, x0, xg, tc_cost) in enumerate(cases):
        base, smooth = res[i][1], res[n + i][1]
        row = {"case": c, "restatement": base, "softplus_1000": smooth, "trust_constr_cost": tc_cost}
        if base["status"] != "solved":
            row["trace"] = reduce(jobs[i][3], a.tail)
        rows.append(row)
        print(json.dumps(row), flush=True)
    failed = [r for r in rows if r["restatement"]["status"] != "solved"]
    summary = {
        "cases": n, "restatement_failed": len(failed),
        "failed_with_relu_flips_in_tail": sum(r["trace"]["relu_flip_frac"] > 0.5 for r in failed),
        "failed_dual_inf_median_above_tol": sum(r["trace"]["dual_median"] > 1e-4 for r in failed),
        "failed_but_softplus_solved": sum(r["softplus_1000"]["status"] == "solved" for r in failed),
        "softplus_solved": sum(r["softplus_1000"]["status"] == "solved" for r in rows),
    }
    out = {"generator": "scripts/kink_trace.py", "tail": a.tail, "summary": summary, "instances": rows}
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(summary, indent=1))


if __name__ == "__main__":
    main()
