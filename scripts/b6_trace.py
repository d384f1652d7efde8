#!/usr/bin/env python3
"""Why benchmark-6 instances with a feasible point still fail: a per-iteration trace.

For each of the first --n b6 instances of tests/golden/oracle_outcomes.npz (BASELINE configs[3]: Ackermann 2nd order,
N = 100, no slack, the trained ring SDF, the stored RRT guesses) the oracle runs with IPOPT's settings (default
options: the reference's constraint-row bounds) and NLOT_VERBOSE=1, which prints one line per iteration (mu, f, theta,
E0, dual infeasibility, delta_w, alpha_max, alpha, alpha_z, filter size, watchdog / soft-restoration / tiny-step
flags) and one per restoration iteration.  Each run is reduced to:

  * status, how it ended (oracle info[14]: restoration line search failed, restoration converged to a feasible point
    the original filter rejects, converged infeasible, almost feasible at the restoration's entry, max_iter in or out
    of a restoration phase), iterations, restoration phases, soft-restoration steps, watchdogs, corrections;
  * the main iterations: the share with a shortened step (alpha < alpha_max), with an inertia correction (delta_w >
    0), the largest delta_w, and medians of mu, theta, the dual infeasibility over the last 100;
  * every restoration phase: its iterations, its final theta_R and E0, and how it ended;
  * the phase-1 result of scripts/b6_feasibility.py for the instance (profiles/r04/b6_feasibility.json), when present.

    python scripts/b6_trace.py [--n 12] [--procs 8] [--out profiles/r05/b6_trace.json]

CPU only; test infrastructure (runs the oracle)."""
import argparse
import json
import os
import re
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import sys, json, numpy as np
sys.path.insert(0, {root!r}); sys.path.insert(0, {root!r} + "/oracle")
import oracle as O
from nlotrajectories_amd import _abi
from nlotrajectories_amd.nn import MlpWeights
from nlotrajectories_amd.problem import B6_PROBLEM
f = np.load({root!r} + "/tests/golden/oracle_outcomes.npz")
i = {i}
hm = O.HostMlp(MlpWeights.load({root!r} + "/nlotrajectories_amd/data/b6_mlp128_seed0.npz"))
opt = _abi.default_options(general_bounds={gb})
r = O.solve_one(B6_PROBLEM, f["b6_x0"][i], f["b6_xg"][i], hm, opt=opt, X_init=f["b6_xinit"][i])
print(json.dumps({{k: r[k] for k in ("status", "iters", "cost", "resto_phases", "soft_resto_steps", "watchdogs",
                                    "soc_tried", "term", "constr_viol", "dual_inf", "mu", "trials")}}))
"""

MAIN = re.compile(r"^it\s+(\d+) mu (\S+) f (\S+) th (\S+) E0 (\S+) dual (\S+) dw (\S+) amax (\S+) a (\S+) az (\S+) "
                  r"nf (\d+)(.*)$")
RESTO = re.compile(r"^\s+resto it\s+(\d+) mu (\S+) fR (\S+) thR (\S+) E0 (\S+) a (\S+)$")


def run(i, gb):
    env = dict(os.environ, NLOT_VERBOSE="1", OMP_NUM_THREADS="1")
    p = subprocess.run([sys.executable, "-c", CHILD.format(root=ROOT, i=i, gb=gb)], capture_output=True, text=True,
                       env=env)
    res = json.loads(p.stdout.strip().splitlines()[-1])
    main, phases, cur = [], [], None
    for line in p.stderr.splitlines():
        m = MAIN.match(line)
        if m:
            if cur is not None:
                phases.append(cur)
                cur = None
            it, mu, f, th, E0, dual, dw, amax, a, az, nf = (float(x) for x in m.groups()[:11])
            main.append(dict(it=int(it), mu=mu, f=f, th=th, E0=E0, dual=dual, dw=dw, amax=amax, a=a, az=az,
                             nf=int(nf), flags=m.group(12).strip()))
            continue
        m = RESTO.match(line)
        if m:
            it, mu, fR, thR, E0, a = (float(x) for x in m.groups())
            if cur is None:
                cur = []
            cur.append(dict(it=int(it), mu=mu, fR=fR, thR=thR, E0=E0, a=a))
    if cur is not None:
        phases.append(cur)
    tail = main[-100:]
    med = lambda k: float(np.median([r[k] for r in tail])) if tail else None  # noqa: E731
    res["main_iterations"] = len(main)
    res["main_shortened_frac"] = float(np.mean([r["a"] < r["amax"] for r in main])) if main else None
    res["main_dw_frac"] = float(np.mean([r["dw"] > 0 for r in main])) if main else None
    res["main_dw_max"] = max([r["dw"] for r in main], default=None)
    res["main_last100_median"] = {k: med(k) for k in ("mu", "th", "dual", "E0", "f")}
    res["main_last"] = main[-1] if main else None
    res["restoration_phases"] = [{"iterations": len(ph), "start_iter": ph[0]["it"], "final_thR": ph[-1]["thR"],
                                  "final_E0": ph[-1]["E0"], "final_mu": ph[-1]["mu"], "final_alpha": ph[-1]["a"]}
                                 for ph in phases]
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=12)
    ap.add_argument("--procs", type=int, default=8)
    ap.add_argument("--general-bounds", type=int, default=1)
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "r05", "b6_trace.json"))
    a = ap.parse_args()
    feas = {}
    fp = os.path.join(ROOT, "profiles", "r04", "b6_feasibility.json")
    if os.path.exists(fp):
        for r in json.load(open(fp))["instances"]:
            feas[r["instance"]] = {"feasible_1e-6": r["feasible_1e-6"], "min_violation": r["min_violation_reached"],
                                   "violation_at_rrt_guess": r["violation_at_rrt_guess"]}
    with ThreadPoolExecutor(a.procs) as ex:
        out = list(ex.map(lambda i: run(i, a.general_bounds), range(a.n)))
    for i, r in enumerate(out):
        r["instance"] = i
        r["phase1"] = feas.get(i)
        print(i, r["status"], r["term"], r["iters"], "resto", r["resto_phases"], "feasible",
              (feas.get(i) or {}).get("feasible_1e-6"), flush=True)
    summary = {}
    for r in out:
        key = f"{'feasible' if (r['phase1'] or {}).get('feasible_1e-6') else 'infeasible_or_unknown'}:{r['term']}"
        summary[key] = summary.get(key, 0) + 1
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    json.dump({"generator": "scripts/b6_trace.py", "general_bounds": a.general_bounds, "summary": summary,
               "instances": out}, open(a.out, "w"), indent=1)
    print(json.dumps(summary, indent=1))


if __name__ == "__main__":
    main()
