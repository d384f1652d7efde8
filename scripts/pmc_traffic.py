#!/usr/bin/env python3
"""HBM bytes per unit from the FETCH_SIZE / WRITE_SIZE passes of scripts/pmc_traffic.sh, in the schema bench.py reads
(roofline.traffic): k_ric bytes per factorising Newton solve, full-MLP bytes per point, value-MLP bytes per point.
gfx950 corrections (MI355X_MICROARCH.md, HBM/rocprofv3): FETCH_SIZE counts half the bytes of wide coalesced reads
(x2), both counters in KB = 1024 B.  Per unit = the counter summed over the in-solve dispatches / the solver's own
counts (NlotSolveStats printed by scripts/pmc_solve.py).

    python scripts/pmc_traffic.py gpurun_out/r04pmc profiles/r04/pmc_traffic_r04_B65536.json"""
import collections
import csv
import glob
import json
import os
import re
import sys


def family(name):
    if re.search(r"k_ric<\d+, false, false>", name):
        return "k_ric"
    if re.search(r"k_ric<\d+, false, true>", name):
        return "k_ric_soc"
    if re.search(r"k_ric<\d+, true, false>", name):
        return "k_ric_resto"
    if "mlp_bf16<128, true" in name:
        return "mlp_full"
    if "mlp_bf16<128, false" in name:
        return "mlp_value"
    for k in ("k_iter_a", "k_iter_b", "k_accept", "k_resto_a", "k_resto_b", "k_resto_ls"):
        if k + "<" in name:
            return k
    return None


def main():
    d, out = sys.argv[1], sys.argv[2]
    tot = collections.defaultdict(float)
    for c in ("FETCH_SIZE", "WRITE_SIZE"):
        rows = []
        for path in glob.glob(os.path.join(d, f"pmc_{c}", "**", "*counter_collection.csv"), recursive=True):
            rows += [r for r in csv.DictReader(open(path)) if r["Counter_Name"] == c and family(r["Kernel_Name"])]
        # the first factorising k_ric dispatch is the INIT step's least-squares multiplier solve (every instance, not in
        # NlotSolveStats.ric_solves): excluded, so that bytes per solve are the Newton solves' own (round 5; round 4's
        # file included it: 65,536 LSQ solves over 626,165 counted ones)
        ric = [int(r["Dispatch_Id"]) for r in rows if family(r["Kernel_Name"]) == "k_ric"]
        lsq = min(ric) if ric else None
        for r in rows:
            f = family(r["Kernel_Name"])
            if f == "k_ric" and int(r["Dispatch_Id"]) == lsq:
                f = "k_ric_lsq"
            tot[(f, c)] += float(r["Counter_Value"]) * 1024.0 * (2.0 if c == "FETCH_SIZE" else 1.0)
    st = json.loads(open(os.path.join(d, "pmc_FETCH_SIZE_stats.json")).read().strip().splitlines()[-1])
    pf, pv, reused = st["mlp_points_full"], st["mlp_points_value"], st["mlp_points_full_reused"]
    rf = reused / max(pf, 1)
    # a point whose forward comes from the accepted trial reads its coordinates (8 B), the trial's coordinates for the
    # match (8 B), value (4 B) and ReLU pattern (16 B); the others read their coordinates; all write value, gradient
    # and Hessian (6 floats)
    full_alg = rf * (8 + 8 + 4 + 16 + 24) + (1 - rf) * (8 + 24)
    res = {
        "run": "scripts/pmc_traffic.sh: scripts/pmc_solve.py 65536 8, rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE in separate "
               "passes, --kernel-include-regex k_ric|mlp_bf16; FETCH_SIZE x2 (gfx950), KB = 1024 B; summarised by "
               "scripts/pmc_traffic.py",
        "solver_stats": {k: st[k] for k in ("mlp_points_full", "mlp_points_value", "mlp_points_full_reused",
                                            "mlp_full_launches", "mlp_value_launches", "ric_solves", "ric_launches",
                                            "iterations")},
        "mlp_full": {"fetch_bytes_per_point": tot[("mlp_full", "FETCH_SIZE")] / pf,
                     "write_bytes_per_point": tot[("mlp_full", "WRITE_SIZE")] / pf,
                     "forward_reused_frac": rf, "algorithmic_bytes_per_point_with_reuse": full_alg,
                     "algorithmic_bytes_per_point_plain": 32.0},
        "mlp_value": {"fetch_bytes_per_point": tot[("mlp_value", "FETCH_SIZE")] / pv,
                      "write_bytes_per_point": tot[("mlp_value", "WRITE_SIZE")] / pv,
                      "algorithmic_bytes_per_point": 28.0},
        "k_ric": {"fetch_bytes_per_solve": tot[("k_ric", "FETCH_SIZE")] / st["ric_solves"],
                  "write_bytes_per_solve": tot[("k_ric", "WRITE_SIZE")] / st["ric_solves"],
                  "algorithmic_bytes_per_solve": 143616.0},
    }
    # the phase kernels and the side-stream Newton solves per instance-iteration, next to SURVEY.md
    # §8d's algorithmic 2 * 4 * (nvar + ncon) bytes per problem-iteration
    ii = st.get("instance_iterations")
    if ii:
        res["per_instance_iteration"] = {
            k: {"fetch_bytes": tot[(k, "FETCH_SIZE")] / ii, "write_bytes": tot[(k, "WRITE_SIZE")] / ii,
                "hbm_bytes": (tot[(k, "FETCH_SIZE")] + tot[(k, "WRITE_SIZE")]) / ii}
            for k in ("k_iter_a", "k_iter_b", "k_accept", "k_ric", "k_ric_soc", "k_ric_resto", "k_resto_a", "k_resto_b",
                      "k_resto_ls", "mlp_full", "mlp_value")}
        res["per_instance_iteration"]["instance_iterations"] = ii
        res["per_instance_iteration"]["algorithmic_bytes_survey_8d"] = 5736.0
    for k, u in (("mlp_full", "point"), ("mlp_value", "point"), ("k_ric", "solve")):
        e = res[k]
        e[f"hbm_bytes_per_{u}"] = e[f"fetch_bytes_per_{u}"] + e[f"write_bytes_per_{u}"]
    res["mlp_full"]["ratio_to_algorithmic_with_reuse"] = res["mlp_full"]["hbm_bytes_per_point"] / full_alg
    res["k_ric"]["ratio_to_algorithmic"] = res["k_ric"]["hbm_bytes_per_solve"] / 143616.0
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
