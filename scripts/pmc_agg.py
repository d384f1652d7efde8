"""Aggregate a rocprofv3 counter_collection.csv per kernel (sums over dispatches) -> small JSON."""
import collections
import csv
import json
import sys

agg = collections.defaultdict(collections.Counter)
for r in csv.DictReader(open(sys.argv[1])):
    name = r["Kernel_Name"].split("(")[0].replace("void ", "")
    agg[name][r["Counter_Name"]] += float(r["Counter_Value"])
json.dump({k: dict(v) for k, v in agg.items()}, open(sys.argv[2], "w"), indent=1)
