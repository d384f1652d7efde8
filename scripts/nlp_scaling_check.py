#!/usr/bin/env python3
"""Is IPOPT's default NLP scaling a no-op on the metric workload?  

IPOPT scales by default with nlp_scaling_method = gradient-based, nlp_scaling_max_gradient = 100: at the starting
point, the objective gets the factor min(1, 100 / ||grad f||_inf) and every constraint row i the factor
min(1, 100 / ||grad c_i||_inf) (IPOPT's GradientScaling; nlp_scaling_min_value 1e-8).  The restatement applies no
scaling.  This script evaluates those gradients at the reference's starting point (linear X, U = 0, S = 0, and the
same point with S pushed to IPOPT's 0.01) for the first B seeded metric instances and reports the largest row
gradient: below 100 every factor is 1 and the scaling changes nothing.

    python scripts/nlp_scaling_check.py [--n 256] [--out profiles/r04/nlp_scaling_check.json]

CPU only; test infrastructure (the oracle's derivatives, through scripts/crosscheck_scipy.Nlp)."""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "scripts"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=256)
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "r04", "nlp_scaling_check.json"))
    a = ap.parse_args()
    import oracle as O
    from crosscheck_scipy import Nlp
    from nlotrajectories_amd.nn import MlpWeights
    from nlotrajectories_amd.problem import METRIC_PROBLEM
    from nlotrajectories_amd.sampling import sample_start_goal

    hm = O.HostMlp(MlpWeights.artefact())
    x0, xg = sample_start_goal(METRIC_PROBLEM, a.n, seed=0, sdf=lambda P: O.mlp_eval(hm, P, want=False)[0])
    worst = {"objective": 0.0, "equality_rows": 0.0, "inequality_rows": 0.0}
    per = []
    for push in (0.0, 0.01):
        w = {"objective": 0.0, "equality_rows": 0.0, "inequality_rows": 0.0}
        for i in range(a.n):
            nlp = Nlp(METRIC_PROBLEM, x0[i], xg[i], hm)
            z = nlp.z0()
            if nlp.ns:
                z[nlp.iS:] = push
            _, g = nlp.f(z)
            w["objective"] = max(w["objective"], float(np.abs(g).max()))
            Je = nlp.ceq_jac(z)
            w["equality_rows"] = max(w["equality_rows"], float(abs(Je).max()))
            Ji = nlp.cin_jac(z)
            w["inequality_rows"] = max(w["inequality_rows"], float(abs(Ji).max()))
        per.append({"slack_at_start": push, **w})
        for k in worst:
            worst[k] = max(worst[k], w[k])
    doc = {
        "generator": "scripts/nlp_scaling_check.py", "instances": a.n,
        "ipopt_defaults": "nlp_scaling_method gradient-based, nlp_scaling_max_gradient 100",
        "max_abs_gradient_entry": worst, "by_start": per,
        "scaling_is_noop": bool(max(worst.values()) <= 100.0),
        "note": "a row (or the objective) is scaled only if its largest gradient entry exceeds 100; the largest entry "
                "of any row's gradient over all instances is reported",
    }
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(doc, f, indent=1)
    print(json.dumps(doc, indent=1))


if __name__ == "__main__":
    main()
