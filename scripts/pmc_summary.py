"""Summarise the FETCH_SIZE / WRITE_SIZE passes of scripts/gpu_pmc.sh (mlp_bench.py, P points per launch)
into profiles/mlp_full_traffic.json, which bench.py uses for roofline.traffic.

gfx950: FETCH_SIZE counts half the bytes of wide coalesced reads -> doubled (MI355X_MICROARCH.md, HBM);
KB = 1024 B.  The microbenchmark writes 7 floats per point (value, grad 2, Hessian 4); the solver's
launches write 6 (the Hessian's symmetric off-diagonal once), so the per-point figure used by the bench
is fetch + 6 x 4 B."""
import collections
import csv
import json
import os
import sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
P = int(sys.argv[2]) if len(sys.argv) > 2 else 16384 * 204
res = {}
for kind, ctr in (("fetch", "FETCH_SIZE"), ("write", "WRITE_SIZE")):
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(os.path.join(root, kind, "run_counter_collection.csv"))):
        if "mlp_kernel" in r["Kernel_Name"] and r["Counter_Name"] == ctr:
            agg["full" if "true>" in r["Kernel_Name"] else "value"].append(float(r["Counter_Value"]))
    for k, v in agg.items():
        res[f"{k}_{ctr}_KB_mean"] = sum(v) / len(v)
        res[f"{k}_{ctr}_launches"] = len(v)
fetch_pp = res["full_FETCH_SIZE_KB_mean"] * 1024 * 2 / P
write_pp = res["full_WRITE_SIZE_KB_mean"] * 1024 / P
out = {
    "kernel": "mlp_kernel<128,1,full>",
    "points_per_launch": P,
    "fetch_bytes_per_point_corrected": fetch_pp,
    "write_bytes_per_point_microbench": write_pp,
    "hbm_bytes_per_launch_per_point": fetch_pp + 24.0,
    "algorithmic_bytes_per_point": 8 + 24,
    "raw": res,
    "method": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE, separate passes, --kernel-trace only "
              "(scripts/gpu_pmc.sh); FETCH_SIZE x2 (gfx950), KB = 1024 B",
}
json.dump(out, open("profiles/mlp_full_traffic.json", "w"), indent=1)
print(json.dumps(out, indent=1))
