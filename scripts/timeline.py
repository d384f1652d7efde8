#!/usr/bin/env python3
"""Critical path of the solver's global step from a rocprofv3 --kernel-trace CSV (one row per dispatch).

    python scripts/timeline.py RUN_kernel_trace.csv [--min-active 16384]

A global step is the interval between two consecutive k_accept ends.  For the steps whose active count (k_accept's
grid / 64) is at least --min-active (the bulk), per kernel class the mean duration, and the waits that decide the
step's length: k_iter_b starts after both the main Newton solve (k_ric) and the corrections (k_ric<SOC> on the side
stream) end, the second value launch after k_iter_b and the early value launch (fourth stream) and the restoration
chain (third stream).  Reports where the main stream sat idle waiting for a side stream."""
import argparse
import bisect
import collections
import csv
import json

CLASSES = (  # (class, substrings of the kernel name: all must occur); first match wins
    ("ric_soc", "k_ric<", ", false, true>"), ("ric_resto", "k_ric<", ", true, false>"), ("ric", "k_ric<"),
    ("iter_a", "k_iter_a"), ("iter_b", "k_iter_b"), ("accept", "k_accept"), ("resto_a", "k_resto_a"),
    ("resto_b", "k_resto_b"), ("resto_ls", "k_resto_ls"), ("points", "k_points"),
    ("mlp_full", "mlp_bf16<128, true"), ("mlp_value", "mlp_bf16<128, false"), ("mlp_full", "mlp_kernel<128, 1, true>"),
    ("mlp_value", "mlp_kernel<128, 1, false>"), ("admit", "k_admit"), ("init", "k_init_state"),
    ("step_end", "k_step_end"), ("copy", "copyBuffer"), ("fill", "fillBuffer"))


def cls(name):
    for c, *subs in CLASSES:
        if all(s in name for s in subs):
            return c
    return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--min-active", type=int, default=16384)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    rows = []
    for r in csv.DictReader(open(a.trace)):
        c = cls(r["Kernel_Name"])
        if c:
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), c, int(r["Grid_Size_X"]) // 64,
                         r.get("Queue_Id", r.get("Stream_Id", ""))))
    rows.sort()
    acc = [r for r in rows if r[2] == "accept"]
    ends = [r[1] for r in acc]
    steps = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in rows:
        i = bisect.bisect_left(ends, r[1])
        if i < len(acc):
            steps[i][r[2]].append(r)
    bulk = [i for i in range(1, len(acc)) if acc[i][3] >= a.min_active]
    dur = collections.defaultdict(list)
    offs = collections.defaultdict(list)  # (start, end) of each launch relative to the step's start
    waits = collections.defaultdict(list)
    walls = []
    for i in bulk:
        s = steps[i]
        walls.append(ends[i] - ends[i - 1])
        for c, lst in s.items():
            dur[c].append(sum(e - b for b, e, *_ in lst))
            for j, (b, e, *_) in enumerate(sorted(lst)):
                offs[f"{c}#{j}"].append((b - ends[i - 1], e - ends[i - 1]))
        if s.get("iter_b") and s.get("ric"):
            ib = s["iter_b"][0][0]
            ric_end = max(e for b, e, *_ in s["ric"])
            soc_end = max((e for b, e, *_ in s.get("ric_soc", [])), default=0)
            waits["iter_b_after_ric"].append(ib - ric_end)
            waits["soc_end_minus_ric_end"].append(soc_end - ric_end if soc_end else 0)
        if s.get("mlp_value") and s.get("iter_b"):
            ibe = s["iter_b"][0][1]
            v2 = max(s["mlp_value"], key=lambda r: r[0])  # the second (main-stream) part starts last
            waits["value2_start_after_iter_b"].append(v2[0] - ibe)
        if s.get("iter_a") and s.get("mlp_full"):
            waits["iter_a_start_after_full"].append(min(b for b, *_ in s["iter_a"]) - max(e for b, e, *_ in s["mlp_full"]))
        if s.get("accept"):
            acb = s["accept"][0][0]
            prev = max((e for c in ("mlp_value", "resto_ls") for b, e, *_ in s.get(c, []) if e <= acb), default=acb)
            waits["accept_start_after_prev"].append(acb - prev)
    mean = lambda v: sum(v) / len(v) / 1e3 if v else 0.0  # noqa: E731  (us)
    res = {"trace": a.trace, "bulk_steps": len(bulk), "min_active": a.min_active,
           "wall_us_per_step": mean(walls),
           "kernel_us_per_step": {c: mean(v) for c, v in sorted(dur.items())},
           "launch_start_end_us_from_step_start": {
               c: [mean([a for a, _ in v]), mean([b for _, b in v]), len(v)]
               for c, v in sorted(offs.items(), key=lambda kv: sum(a for a, _ in kv[1]) / len(kv[1]))},
           "waits_us": {k: mean(v) for k, v in waits.items()}}
    print(json.dumps(res, indent=1))
    if a.out:
        json.dump(res, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
