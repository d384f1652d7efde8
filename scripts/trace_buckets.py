"""Per-active-count buckets of kernel time from a rocprofv3 kernel trace (scripts/gpu_prof*.sh)."""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
names = {"k_iter_a": "ita", "k_ric": "ric", "k_iter_b": "itb", "k_iterate": "iter", "mlp_kernel<128, 1, true>": "full", "mlp_bf16<128, true>": "full", "mlp_bf16<128, false>": "val",
         "mlp_kernel<128, 1, false>": "val", "k_accept": "acc", "k_points": "pts"}
per = collections.defaultdict(list)
for r in rows:
    for k, v in names.items():
        if k in r["Kernel_Name"]:
            per[v].append(r)
acc = per["acc"]
n = len(acc)
# step i: the i-th k_accept launch; its active count = grid / 64
def bucket(a):
    for k in (256, 2048, 8192, 16384, 32768, 65536, 1 << 30):
        if a <= k:
            return k
B = collections.defaultdict(collections.Counter)
# assign every launch to the step whose k_accept ends after it
ends = [int(r["End_Timestamp"]) for r in acc]
import bisect
for v, lst in per.items():
    for r in lst:
        i = bisect.bisect_left(ends, int(r["End_Timestamp"]))
        if i >= n:
            continue
        a = int(acc[i]["Grid_Size_X"]) // 64
        B[bucket(a)][v] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
steps = collections.Counter(bucket(int(r["Grid_Size_X"]) // 64) for r in acc)
wall = collections.Counter()
for i in range(1, n):
    wall[bucket(int(acc[i]["Grid_Size_X"]) // 64)] += ends[i] - ends[i - 1]
for k in sorted(B):
    c = B[k]
    print(f"active<={k:8d} steps {steps[k]:5d} wall {wall[k]/1e6:8.1f} ms  " +
          " ".join(f"{v} {c[v]/1e6:7.1f}" for v in sorted(c)))
print("total wall ms", (ends[-1] - int(per["pts"][0]["Start_Timestamp"])) / 1e6)
