#!/usr/bin/env python3
"""Per-kernel summary of SQ PMC passes (scripts/pmc_solver_sq.sh, scripts/pmc_mlp_sq.sh): counters summed over the
dispatches of each kernel family, then the wave-cycle split (WAIT_ANY = parked on s_waitcnt / barriers, WAIT_INST_ANY
= issue-stalled, ACTIVE_INST_ANY = issuing; they add up to WAVE_CYCLES), instructions per wave and the share of issue
cycles by type.  Usage: python scripts/pmc_sq_summary.py DIR [DIR ...] > summary.json"""
import collections
import csv
import glob
import json
import os
import re
import sys

FAMILIES = [("k_ric<soc>", r"k_ric<\d+, false, true>"), ("k_ric<resto>", r"k_ric<\d+, true"),
            ("k_ric", r"k_ric<\d+, false, false>"), ("k_iter_a", r"k_iter_a<"), ("k_iter_b", r"k_iter_b<"),
            ("k_accept", r"k_accept<"), ("mlp_full", r"mlp_bf16<128, true"), ("mlp_value", r"mlp_bf16<128, false")]


def family(name):
    for f, rx in FAMILIES:
        if re.search(rx, name):
            return f
    return None


def main():
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for d in sys.argv[1:]:
        for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(path)):
                f = family(r["Kernel_Name"])
                if f is None:
                    continue
                agg[f][r["Counter_Name"]] += float(r["Counter_Value"])
                disp[f].add((path, r["Dispatch_Id"]))
    out = {}
    for f, c in agg.items():
        w = c.get("SQ_WAVE_CYCLES", 0.0)
        e = {"dispatches_in_passes": len(disp[f]), "raw": dict(c)}
        if w:
            e["wave_cycle_split"] = {k: c.get(k, 0.0) / w for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY")}
            e["active_split"] = {k: c.get(k, 0.0) / max(c.get("SQ_ACTIVE_INST_ANY", 1.0), 1.0)
                                 for k in ("SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_VMEM", "SQ_ACTIVE_INST_LDS",
                                           "SQ_ACTIVE_INST_SCA") if k in c}
        if c.get("SQ_WAVES"):
            n = c["SQ_WAVES"]
            e["per_wave"] = {k: c[k] / n for k in ("SQ_INSTS", "SQ_INSTS_VALU", "SQ_INSTS_VMEM", "SQ_INSTS_SALU",
                                                   "SQ_INSTS_SMEM", "SQ_INSTS_LDS", "SQ_INSTS_VALU_FMA_F64") if k in c}
        out[f] = e
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
