#!/usr/bin/env python3
"""Do the restoration solves under the attempt cap give bitwise the same results?  Benchmark 6's fixture instances
(tests/golden/oracle_outcomes.npz: x0, xg, RRT X_init), the cap forced at any batch size (NLOT_RIC_TRIES_MIN=0):
NLOT_RESTO_TRIES=0 twice and =1 once, statuses / iterations / costs / trajectories compared.  GPU box."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    from nlotrajectories_amd import _abi
    from nlotrajectories_amd.nn import MlpWeights
    from nlotrajectories_amd.ops import DeviceMlp
    from nlotrajectories_amd.problem import B6_PROBLEM
    from nlotrajectories_amd.solver import solve_batch

    f = dict(np.load(os.path.join(ROOT, "tests", "golden", "oracle_outcomes.npz")))
    mlp = DeviceMlp(MlpWeights.load(os.path.join(ROOT, "nlotrajectories_amd", "data", "b6_mlp128_seed0.npz")))
    opt = _abi.default_options(general_bounds=int(f["general_bounds"]))
    os.environ["NLOT_RIC_TRIES_MIN"] = "0"
    runs = {}
    for tag, t in (("t0a", "0"), ("t1", "1"), ("t0b", "0")):
        os.environ["NLOT_RESTO_TRIES"] = t
        r = solve_batch(B6_PROBLEM, f["b6_x0"], f["b6_xg"], mlp=mlp, X_init=f["b6_xinit"], options=opt)
        runs[tag] = {k: r[k].cpu().numpy() for k in ("status", "iters", "cost", "X")}
        print(tag, "status", runs[tag]["status"].tolist(), "iters", runs[tag]["iters"].tolist(), flush=True)
    for tag in ("t1", "t0b"):
        eq = [bool(np.array_equal(runs["t0a"][k], runs[tag][k])) for k in ("status", "iters", "cost", "X")]
        diff = np.nonzero(runs["t0a"]["iters"] != runs[tag]["iters"])[0].tolist()
        print(tag, "vs t0a equal (status, iters, cost, X):", eq, "instances with other iteration counts:", diff)


if __name__ == "__main__":
    main()
