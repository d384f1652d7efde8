#!/usr/bin/env python3
"""Where do a GPU solve and the oracle part?  For one instance of a test case (tests/test_branches_gpu.py cases,
optionally perturbed like the full-solve tests), run both with max_iter = k for growing k and print status,
iterations and the iterate difference next to the oracle's own response to a 1e-13 change of the start.
GPU debugging aid (run through gpurun); uses the oracle as the checker."""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("case")
    ap.add_argument("--instance", type=int, default=-1, help="index of the rng(11) perturbed batch (-1: nominal)")
    ap.add_argument("--ks", default="10,20,40,80,120,160,200,300,400,600,800,1000")
    a = ap.parse_args()
    import oracle as O
    from test_branches_gpu import _cases

    from nlotrajectories_amd import _abi
    from nlotrajectories_amd.solver import solve_batch

    prob, x0, xg = _cases()[a.case]
    x0, xg = np.array(x0, float), np.array(xg, float)
    if a.instance >= 0:
        rng = np.random.default_rng(11)
        B = 12
        X0 = np.repeat(x0[None], B, 0)
        XG = np.repeat(xg[None], B, 0)
        X0[:, :2] += rng.uniform(-0.05, 0.05, (B, 2))
        XG[:, :2] += rng.uniform(-0.05, 0.05, (B, 2))
        x0, xg = X0[a.instance], XG[a.instance]
    for k in map(int, a.ks.split(",")):
        opt = _abi.default_options(max_iter=k)
        rg = solve_batch(prob, x0[None], xg[None], options=opt)
        rc = O.solve_one(prob, x0, xg, opt=opt)
        xp = x0.copy()
        xp[0] += 1e-13
        rp = O.solve_one(prob, xp, xg, opt=opt)
        d = max(float(np.abs(rg[n][0].cpu().numpy() - rc[n]).max()) for n in ("X", "U", "S"))
        sens = max(float(np.abs(rp[n] - rc[n]).max()) for n in ("X", "U", "S"))
        print(f"k {k:5d} gpu {rg['status'][0].item()} {rg['iters'][0].item():5d} oracle {rc['status']} {rc['iters']:5d} "
              f"resto {rc['resto_phases']:3d} soft {rc['soft_resto_steps']:3d} wd {rc['watchdogs']} | gpu-oracle {d:.2e} "
              f"oracle-perturbed {sens:.2e} ({rp['status']} {rp['iters']})", flush=True)


if __name__ == "__main__":
    main()
