#!/usr/bin/env python3
"""Do benchmark-6 instances have a feasible point at all?  

The b6 bench line (BASELINE configs[3]: Ackermann 2nd order, N = 100, no slack so every footprint corner must keep
the learned ring SDF >= 0, the YAML's RRT initial guess) solves 7 % of its instances and ends 63 % in a failed
restoration.  This script asks the question the solver status cannot answer: a phase-1 problem that only minimises
the constraint violation of the same NLP,

    min_z 1/2 ||c_eq(z)||^2 + 1/2 ||min(0, c_in(z))||^2   s.t. the control bounds,

solved with scipy's bounded trust-region least squares (least_squares, method 'trf', exact sparse Jacobians from the
oracle's derivatives via scripts/crosscheck_scipy.Nlp) from the RRT initial guess (U = 0).  An instance is reported
feasible when the maximum violation max(|c_eq|, max(0, -c_in)) it reaches is <= 1e-6 (IPOPT's constr_viol_tol is
1e-4).  Also reported: the violation at the RRT guess, and the oracle's (IPOPT restatement's) status on the same
instance.  The instances are tests/golden/oracle_outcomes.npz's b6 set when present (their RRT guesses are stored
there), else 12 seeded ones built here.

    [B6_SOFTPLUS=1] python scripts/b6_feasibility.py [--n 12] [--out profiles/r04/b6_feasibility.json]

B6_SOFTPLUS=1 also runs the oracle's IPOPT restatement with the net's ReLUs replaced by softplus(beta = 1000) (the
kink diagnostic of DESIGN.md §4b) from the same RRT guess and reports its status.

CPU only; test infrastructure (uses the oracle)."""
import argparse
import json
import os
import sys
import time
from concurrent.futures import ProcessPoolExecutor

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "scripts"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
W6 = os.path.join(ROOT, "nlotrajectories_amd", "data", "b6_mlp128_seed0.npz")


def phase1(args):
    i, x0, xg, Xi, oracle_status = args
    import oracle as O
    from scipy.optimize import least_squares
    from scipy import sparse
    from crosscheck_scipy import Nlp
    from nlotrajectories_amd.nn import MlpWeights
    from nlotrajectories_amd.problem import B6_PROBLEM

    hm = O.HostMlp(MlpWeights.load(W6))
    nlp = Nlp(B6_PROBLEM, x0, xg, hm)
    z0 = nlp.z0(Xi)
    bnd = nlp.bounds()
    lo, hi = bnd.lb.copy(), bnd.ub.copy()
    z0 = np.clip(z0, lo + 1e-12 * (np.isfinite(lo)), hi - 1e-12 * (np.isfinite(hi)))
    ne = len(nlp.ceq(z0))

    def res(z):
        return np.concatenate([nlp.ceq(z), np.minimum(0.0, nlp.cin(z))])

    def jac(z):
        ci = nlp.cin(z)
        Ji = nlp.cin_jac(z).tocsr()
        act = sparse.diags((ci < 0).astype(float))
        return sparse.vstack([nlp.ceq_jac(z), act @ Ji]).tocsr()

    def viol(z):
        return max(float(np.abs(nlp.ceq(z)).max()), float(max(0.0, -nlp.cin(z).min())))

    t = time.time()
    r = least_squares(res, z0, jac=jac, bounds=(lo, hi), method="trf", xtol=1e-15, ftol=1e-15, gtol=1e-15,
                      max_nfev=3000)
    smooth = None
    if os.environ.get("B6_SOFTPLUS"):  # the same restatement with the net's ReLUs smoothed (oracle-only diagnostic)
        from nlotrajectories_amd import _abi

        os.environ["NLOT_ORACLE_SOFTPLUS_BETA"] = "1000"
        hs = O.HostMlp(MlpWeights.load(W6))
        hs.desc.act = 90  # ORACLE_ACT_SOFTPLUS
        rs = O.solve_one(B6_PROBLEM, np.asarray(x0, float), np.asarray(xg, float), hs, opt=_abi.default_options(),
                         X_init=Xi)
        smooth = {"status": _abi.STATUS_NAMES[rs["status"]], "iters": rs["iters"], "cost": rs["cost"]}
    out = {"instance": i, "softplus_1000_restatement": smooth, "violation_at_rrt_guess": viol(z0), "min_violation_reached": viol(r.x),
           "equality_violation": float(np.abs(r.fun[:ne]).max()), "corner_sdf_violation": float(np.abs(r.fun[ne:]).max()),
           "feasible_1e-6": bool(viol(r.x) <= 1e-6), "nfev": int(r.nfev), "status": int(r.status),
           "message": r.message, "seconds": time.time() - t, "oracle_status": oracle_status}
    print(json.dumps(out), flush=True)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=12)
    ap.add_argument("--workers", type=int, default=8)
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "r04", "b6_feasibility.json"))
    a = ap.parse_args()
    from nlotrajectories_amd import _abi

    fx = os.path.join(ROOT, "tests", "golden", "oracle_outcomes.npz")
    if os.path.exists(fx) and "b6_x0" in np.load(fx):
        f = np.load(fx)
        X0, XG, Xi, st = f["b6_x0"], f["b6_xg"], f["b6_xinit"], f["b6_status"][0]
        src = "tests/golden/oracle_outcomes.npz (b6 set: RRT guesses of oracle/rrt_oracle.py, seed 3)"
    else:
        sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
        from make_oracle_outcomes import b6_instances

        X0, XG, Xi = b6_instances(a.n)
        st = np.full(len(X0), -1)
        src = "tests/golden/make_oracle_outcomes.b6_instances"
    n = min(a.n, len(X0))
    jobs = [(i, X0[i], XG[i], Xi[i], _abi.STATUS_NAMES.get(int(st[i]), "not run")) for i in range(n)]
    with ProcessPoolExecutor(a.workers) as ex:
        rows = list(ex.map(phase1, jobs))
    feas = [r for r in rows if r["feasible_1e-6"]]
    doc = {"generator": "scripts/b6_feasibility.py", "instances_from": src, "n": n,
           "method": "scipy least_squares trf on [c_eq; min(0, c_in)] with the control bounds, from the RRT guess",
           "feasible (violation <= 1e-6)": len(feas),
           "softplus_1000_solved": sum(1 for r in rows if (r["softplus_1000_restatement"] or {}).get("status") == "solved"),
           "max violation reached (median)": float(np.median([r["min_violation_reached"] for r in rows])),
           "instances": rows}
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    with open(a.out, "w") as fh:
        json.dump(doc, fh, indent=1)
    print(json.dumps({k: v for k, v in doc.items() if k != "instances"}, indent=1))


if __name__ == "__main__":
    main()
