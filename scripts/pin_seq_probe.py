#!/usr/bin/env python3
"""How far do the GPU's iterates follow the oracle's, per MLP arithmetic?  (GPU box; diagnostics for DESIGN.md §5.)

For the fixture's instances of a case (tests/golden/oracle_outcomes.npz: b6 = benchmark 6 from the stored RRT guesses,
metric = the headline workload), the oracle's unperturbed run is traced (iterate at the top of every iteration < 201)
and the GPU runs with max_iter = k for k in a ladder, once per net arithmetic: seq (the oracle's own summation order,
NLOT_MLP_ARITH_SEQ), f32 and split_bf16 (the MFMA nets).  Prints, per instance and net, the largest k of the ladder up
to which the GPU iterate stays within 1e-4 / 1e-8 of the oracle's, and a JSON summary line.

    python scripts/pin_seq_probe.py [--case b6|metric] [--n 24] [--threads 16]
"""
import argparse
import json
import os
import sys
from concurrent.futures import ThreadPoolExecutor

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
LADDER = (1, 2, 3, 5, 8, 12, 20, 30, 45, 60, 80, 100, 130, 160)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--case", default="b6", choices=["b6", "metric"])
    ap.add_argument("--n", type=int, default=24)
    ap.add_argument("--threads", type=int, default=16)
    ap.add_argument("--nets", default="seq,f32,split_bf16")
    a = ap.parse_args()
    import oracle as O
    from nlotrajectories_amd import _abi
    from nlotrajectories_amd.nn import MlpWeights
    from nlotrajectories_amd.ops import DeviceMlp
    from nlotrajectories_amd.problem import B6_PROBLEM, METRIC_PROBLEM
    from nlotrajectories_amd.solver import solve_batch

    f = dict(np.load(os.path.join(ROOT, "tests", "golden", "oracle_outcomes.npz")))
    if a.case == "b6":
        prob = B6_PROBLEM
        w = MlpWeights.load(os.path.join(ROOT, "nlotrajectories_amd", "data", "b6_mlp128_seed0.npz"))
    else:
        prob, w = METRIC_PROBLEM, MlpWeights.artefact()
    n = min(a.n, len(f[f"{a.case}_x0"]))
    x0, xg = f[f"{a.case}_x0"][:n], f[f"{a.case}_xg"][:n]
    xi = f[f"{a.case}_xinit"][:n] if f"{a.case}_xinit" in f else None
    opt = _abi.default_options(general_bounds=int(f["general_bounds"]))
    hm = O.HostMlp(w)
    otr = _abi.default_options(general_bounds=int(f["general_bounds"]), max_iter=LADDER[-1] + 1)  # traces to the ladder's end
    with ThreadPoolExecutor(a.threads) as ex:
        rs = list(ex.map(lambda i: O.solve_trace(prob, x0[i], xg[i], hm, opt=otr, X_init=None if xi is None else xi[i]),
                         range(n)))
    T = np.stack([r["trace"] for r in rs])  # [n, 201, nXU]
    its = np.array([r["iters"] for r in rs])
    N, nx = prob.N, prob.nx
    summary = {}
    for net in a.nets.split(","):
        mlp = DeviceMlp(w, net)
        dev = np.full((n, len(LADDER)), np.nan)
        for j, k in enumerate(LADDER):
            o = _abi.default_options(general_bounds=int(f["general_bounds"]), max_iter=k)
            r = solve_batch(prob, x0, xg, mlp=mlp, X_init=xi, options=o)
            XU = np.concatenate([r["X"].cpu().numpy().reshape(n, -1), r["U"].cpu().numpy().reshape(n, -1)], 1)
            ok = its >= k
            dev[ok, j] = np.abs(XU[ok] - T[ok, k]).max(1)
        reach = {}
        for tol in (1e-4, 1e-8):
            kk = []
            for i in range(n):
                good = [LADDER[j] for j in range(len(LADDER)) if not np.isnan(dev[i, j])]
                bad = [LADDER[j] for j in range(len(LADDER)) if not (dev[i, j] <= tol) and not np.isnan(dev[i, j])]
                kk.append(min(bad) if bad else (max(good) if good else 0))
            reach[str(tol)] = kk
        summary[net] = reach
        print(f"[probe] {a.case} {net}: first ladder k outside 1e-4 per instance (or the last k traced): "
              f"{reach['0.0001']}", flush=True)
        print(f"[probe] {a.case} {net}: ... outside 1e-8: {reach['1e-08']}", flush=True)
    print(json.dumps({"case": a.case, "n": n, "oracle_iters": its.tolist(), "ladder": LADDER, "first_outside": summary}))


if __name__ == "__main__":
    main()
