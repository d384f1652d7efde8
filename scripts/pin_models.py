#!/usr/bin/env python3
"""Which perturbations move the oracle off its pinned iterates on the instances the GPU misses
(tests/test_pinned_iterates_gpu.py): for each (form, case, instance), the oracle's iterate at max_iter = k_i under
  * the merit function's fp64 sums reversed (NLOT_ORACLE_SUM_REV=1; with the net reversed too),
  * 1 +- eps on every Newton step's primal components (NLOT_ORACLE_STEP_JITTER = 1e-15, 1e-13, 1e-11),
  * six more orders of the net's fp32 sums (NLOT_ORACLE_MLP_REV = 2..7),
against the fixture's pinned iterate (max |dX|, |dU|).  CPU, test infrastructure.

    python scripts/pin_models.py > profiles/r05/pin_models.log"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]

import oracle as O  # noqa: E402
from nlotrajectories_amd import _abi  # noqa: E402
from nlotrajectories_amd.nn import MlpWeights  # noqa: E402
from nlotrajectories_amd.problem import B6_PROBLEM, METRIC_PROBLEM  # noqa: E402

CASES = [("varbounds", "b6", 3), ("varbounds", "b6", 19), ("varbounds", "b6", 21), ("rows", "b6", 19),
         ("rows", "b6", 3), ("rows", "metric", 63), ("rows", "b6", 0)]
MODELS = ([("SUM_REV", {"NLOT_ORACLE_SUM_REV": "1"}), ("SUM_REV+MLP_REV", {"NLOT_ORACLE_SUM_REV": "1",
                                                                          "NLOT_ORACLE_MLP_REV": "1"})] +
          [(f"STEP_JITTER {e}", {"NLOT_ORACLE_STEP_JITTER": e}) for e in ("1e-15", "1e-13", "1e-11")] +
          [(f"MLP order {v}", {"NLOT_ORACLE_MLP_REV": str(v)}) for v in range(2, 8)])


def main():
    hm6 = O.HostMlp(MlpWeights.load(os.path.join(ROOT, "nlotrajectories_amd", "data", "b6_mlp128_seed0.npz")))
    hmm = O.HostMlp(MlpWeights.artefact())
    for form, case, i in CASES:
        f = np.load(os.path.join(ROOT, "tests", "golden",
                                 "oracle_outcomes.npz" if form == "rows" else "oracle_outcomes_varbounds.npz"))
        prob, hm = (B6_PROBLEM, hm6) if case == "b6" else (METRIC_PROBLEM, hmm)
        k = int(f[case + "_kpin"][i])
        o = _abi.default_options(general_bounds=int(f["general_bounds"]), max_iter=k)
        xi = f[case + "_xinit"][i] if case + "_xinit" in f else None
        out = []
        for name, env in MODELS:
            os.environ.update(env)
            r = O.solve_one(prob, f[case + "_x0"][i], f[case + "_xg"][i], hm, opt=o, X_init=xi)
            for v in env:
                os.environ.pop(v)
            d = max(np.abs(r["X"] - f[case + "_Xpin"][i]).max(), np.abs(r["U"] - f[case + "_Upin"][i]).max())
            out.append(f"{name}: {d:.1e}")
        print(f"{form} {case} {i} (k_i {k}): " + "; ".join(out), flush=True)


if __name__ == "__main__":
    main()
