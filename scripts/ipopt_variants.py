#!/usr/bin/env python3
"""Status mix of the oracle's IPOPT restatement under one algorithm variant.

Runs the first B seeded metric instances (bench.py's seed-0 start/goal pairs: unicycle_2nd, b3 body, N = 50,
artefact FourierMLP) through the CPU oracle, one instance per thread, and prints one JSON line with the status
counts, iteration statistics and the filter diagnostics (peak sizes, forgotten entries).  Variants are selected
by the oracle's NLOT_ORACLE_* environment knobs, set by the caller:

    NLOT_ORACLE_FILT_CAP=64 python scripts/ipopt_variants.py --label cap64 --n 256
    python scripts/ipopt_variants.py --label unbounded --n 256 --crosscheck

--crosscheck also runs the 16 metric instances of tests/golden/crosscheck_scipy.json that the round-3
restatement failed (trust-constr reaches a KKT point on all of them) and reports their statuses and costs next
to trust-constr's.  CPU only; test infrastructure (uses oracle/).
"""
import argparse
import json
import os
import sys
import time
from concurrent.futures import ThreadPoolExecutor

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--label", default="default")
    ap.add_argument("--n", type=int, default=256)
    ap.add_argument("--threads", type=int, default=8)
    ap.add_argument("--crosscheck", action="store_true")
    ap.add_argument("--general-bounds", action="store_true")
    ap.add_argument("--mu-strategy", default="adaptive")
    ap.add_argument("--softplus", action="store_true",
                    help="diagnostic: the artefact net with its ReLUs replaced by softplus (beta from "
                         "NLOT_ORACLE_SOFTPLUS_BETA, default 100): is the ReLU nonsmoothness what fails the solves")
    ap.add_argument("--out", default=None, help="append the JSON line to this file")
    ap.add_argument("--per-instance", default=None, help="write per-instance results (npz) here")
    a = ap.parse_args()

    import oracle as O
    from nlotrajectories_amd import _abi
    from nlotrajectories_amd.nn import MlpWeights
    from nlotrajectories_amd.problem import METRIC_PROBLEM
    from nlotrajectories_amd.sampling import sample_start_goal

    hm = O.HostMlp(MlpWeights.artefact())
    sdf_hm = O.HostMlp(MlpWeights.artefact())  # start/goal sampling always uses the ReLU net (same instances)
    if a.softplus:
        hm.desc.act = 90  # ORACLE_ACT_SOFTPLUS (oracle-only diagnostic)
    opt = _abi.default_options()
    opt.general_bounds = int(a.general_bounds)
    opt.mu_strategy = 1 if a.mu_strategy == "adaptive" else 0
    sdf = lambda P: O.mlp_eval(sdf_hm, P, want=False)[0]
    x0, xg = sample_start_goal(METRIC_PROBLEM, a.n, seed=0, sdf=sdf)
    cases = [(f"metric[{i}]", x0[i], xg[i]) for i in range(a.n)]
    cc = {}
    if a.crosscheck:
        doc = json.load(open(os.path.join(ROOT, "tests", "golden", "crosscheck_scipy.json")))
        for r in doc["instances"]:
            if r["case"].startswith("metric") and r["ipopt_restatement"]["status"] != "solved":
                cc[r["case"]] = r
                if int(r["case"][7:-1]) >= a.n:
                    cases.append((r["case"], np.array(r["x0"]), np.array(r["xg"])))

    def run(c):
        t = time.time()
        r = O.solve_one(METRIC_PROBLEM, c[1], c[2], hm, opt=opt)
        r["seconds"] = time.time() - t
        return c[0], r

    t0 = time.time()
    with ThreadPoolExecutor(a.threads) as ex:
        res = dict(ex.map(run, cases))
    wall = time.time() - t0
    names = _abi.STATUS_NAMES
    batch = [res[f"metric[{i}]"] for i in range(a.n)]
    st = np.array([r["status"] for r in batch])
    it = np.array([r["iters"] for r in batch])
    line = {
        "label": a.label, "softplus": a.softplus, "env": {k: v for k, v in os.environ.items() if k.startswith("NLOT_ORACLE")},
        "general_bounds": a.general_bounds, "mu_strategy": a.mu_strategy, "n": a.n,
        "status": {names[k]: int((st == k).sum()) for k in sorted(set(st.tolist()))},
        "iters_mean": float(it.mean()), "iters_p50": float(np.median(it)),
        "solved_iters_mean": float(it[st == 0].mean()) if (st == 0).any() else None,
        "peak_filter": int(max(r["max_filter"] for r in batch)),
        "peak_mu_filter": int(max(r["max_mu_filter"] for r in batch)),
        "instances_forgetting": int(sum((r["filter_forgotten"] + r["mu_filter_forgotten"]) > 0 for r in batch)),
        "cpu_seconds": float(sum(r["seconds"] for r in batch)), "wall_seconds": wall,
    }
    if cc:
        rows = []
        for name, ref in cc.items():
            r = res[name]
            rows.append({"case": name, "status": names[r["status"]], "iters": r["iters"], "cost": r["cost"],
                         "trust_constr_cost": ref["trust_constr"]["cost"],
                         "r03_status": ref["ipopt_restatement"]["status"]})
        line["crosscheck"] = {"n": len(rows), "solved": sum(r["status"] == "solved" for r in rows),
                              "instances": rows}
    if a.per_instance:
        np.savez(a.per_instance, status=st, iters=it, cost=np.array([r["cost"] for r in batch]))
    s = json.dumps(line)
    print(s, flush=True)
    if a.out:
        with open(a.out, "a") as f:
            f.write(s + "\n")


if __name__ == "__main__":
    main()
