"""Summarise scripts/pmc_kric_sq.sh: SQ counters of k_ric summed over its launches -> profiles/r02/kric_sq.json.
SQ_WAVE_CYCLES / SQ_WAIT_* / SQ_ACTIVE_INST_* count quad-cycles (MI355X_MICROARCH.md, PMC units); the fractions
below are ratios of those, so the unit cancels."""
import collections
import csv
import json
import sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/r02q/pmc_sq"
import glob

f = glob.glob(f"{root}/**/*counter_collection.csv", recursive=True)[0]
tot = collections.defaultdict(float)
launches = set()
for r in csv.DictReader(open(f)):
    if "k_ric" in r["Kernel_Name"]:
        tot[r["Counter_Name"]] += float(r["Counter_Value"])
        launches.add(r.get("Dispatch_Id", r.get("Correlation_Id")))
w = tot["SQ_WAVE_CYCLES"]
out = {
    "kernel": "k_ric<3> (metric config, B = 16384, one solve)",
    "launches": len(launches),
    "totals": dict(tot),
    "frac_active_inst_any": tot["SQ_ACTIVE_INST_ANY"] / w,
    "frac_active_inst_valu": tot["SQ_ACTIVE_INST_VALU"] / w,
    "frac_wait_any": tot["SQ_WAIT_ANY"] / w,
    "frac_wait_inst_any": tot["SQ_WAIT_INST_ANY"] / w,
    "valu_per_lds_inst": tot["SQ_INSTS_VALU"] / max(1.0, tot["SQ_INSTS_LDS"]),
    "method": "rocprofv3 --pmc (7 SQ counters, one pass, --kernel-include-regex k_ric), scripts/pmc_kric_sq.sh",
}
json.dump(out, open("profiles/r02/kric_sq.json", "w"), indent=1)
print(json.dumps(out, indent=1))
