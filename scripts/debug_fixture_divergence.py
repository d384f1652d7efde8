#!/usr/bin/env python3
"""Where do the GPU and the oracle part on a fixture instance (tests/golden/oracle_outcomes.npz: metric or b6 with its
stored RRT guess)?  For growing max_iter = k: status / iterations of both, the GPU-vs-oracle iterate difference, and
the oracle's own response to its reverse-order net sums (NLOT_ORACLE_MLP_REV, tests/outcomes.py) and to a 1e-13 start
change.  GPU debugging aid (run through gpurun); the oracle is the checker.

    python scripts/debug_fixture_divergence.py b6 5 [--ks 5,10,20,...]"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("case", choices=["metric", "b6"])
    ap.add_argument("instance", type=int)
    ap.add_argument("--ks", default="5,10,20,30,40,60,80,100,150,200,300,500,1000")
    a = ap.parse_args()
    import oracle as O
    import torch
    from outcomes import mlp_order

    from nlotrajectories_amd import _abi
    from nlotrajectories_amd.nn import MlpWeights
    from nlotrajectories_amd.ops import DeviceMlp
    from nlotrajectories_amd.problem import B6_PROBLEM, METRIC_PROBLEM
    from nlotrajectories_amd.solver import solve_batch

    f = np.load(os.path.join(ROOT, "tests", "golden", "oracle_outcomes.npz"))
    i = a.instance
    x0, xg = f[f"{a.case}_x0"][i], f[f"{a.case}_xg"][i]
    if a.case == "b6":
        prob = B6_PROBLEM
        w = MlpWeights.load(os.path.join(ROOT, "nlotrajectories_amd", "data", "b6_mlp128_seed0.npz"))
        Xi = f["b6_xinit"][i]
    else:
        prob, w, Xi = METRIC_PROBLEM, MlpWeights.artefact(), None
    hm, mlp = O.HostMlp(w), DeviceMlp(w)
    print(f"{a.case} instance {i}: fixture oracle statuses {f[a.case + '_status'][:, i].tolist()}", flush=True)
    for k in map(int, a.ks.split(",")):
        opt = _abi.default_options(max_iter=k)
        kw = {} if Xi is None else {"X_init": torch.tensor(Xi[None], dtype=torch.float64, device="cuda")}
        rg = solve_batch(prob, x0[None], xg[None], mlp=mlp, options=opt, **kw)
        rc = O.solve_one(prob, x0, xg, hm, opt=opt, X_init=Xi)
        with mlp_order(True):
            rr = O.solve_one(prob, x0, xg, hm, opt=opt, X_init=Xi)
        xp = x0.copy()
        xp[0] += 1e-13
        rp = O.solve_one(prob, xp, xg, hm, opt=opt, X_init=Xi)
        d = max(float(np.abs(rg[n][0].cpu().numpy() - rc[n]).max()) for n in ("X", "U"))
        dr = max(float(np.abs(rr[n] - rc[n]).max()) for n in ("X", "U"))
        dp = max(float(np.abs(rp[n] - rc[n]).max()) for n in ("X", "U"))
        print(f"k {k:5d} gpu {rg['status'][0].item()} {rg['iters'][0].item():5d} oracle {rc['status']} {rc['iters']:5d} "
              f"resto {rc['resto_phases']:3d} soft {rc['soft_resto_steps']:3d} | gpu-oracle {d:.2e} "
              f"oracle-rev {dr:.2e} ({rr['status']} {rr['iters']}) oracle-x+1e-13 {dp:.2e} ({rp['status']})", flush=True)


if __name__ == "__main__":
    main()
