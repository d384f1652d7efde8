#!/usr/bin/env python3
"""Per-dispatch roofline fractions of the SDF-MLP launches from a rocprofv3 --kernel-trace --stats run of the bench
(the bench line's event brackets include the early value launch's overlap with the main stream;
the profiler's dispatch durations do not).

    python scripts/rocprof_fracs.py RUN_kernel_stats.csv bench_rocprof.json OUT.json

FLOP per dispatch comes from the same run's bench line (its timed region: points per launch, forward-reuse fraction;
the full launch counts 67,072 FLOP per point less 33,536 per reused forward, the value launch 33,536 per point,
DESIGN.md §7); the duration is the profiler's average over the run's dispatches of that kernel (the value kernel runs
twice per global step, its two parts summed).  Peak: the split-bf16 MFMA roofline, 2.5 PFLOP/s dense / 6 = 416.7
TFLOP/s."""
import csv
import json
import sys

PEAK = 2500.0 / 6.0


def main():
    stats, bench, out = sys.argv[1], sys.argv[2], sys.argv[3]
    rows = {r["Name"]: r for r in csv.DictReader(open(stats))}
    b = json.loads(open(bench).read().strip().splitlines()[-1])
    full = next(r for n, r in rows.items() if "mlp_bf16<128, true" in n)
    val = next(r for n, r in rows.items() if "mlp_bf16<128, false" in n)
    f, v = b["roofline_mlp_full"], b["roofline_mlp_value"]
    steps = f["launches"]  # timed global steps (one full launch each)
    flop_full = f["points_per_launch"] * (67072 - f["forward_reused_frac"] * 33536)
    flop_val = v["points_per_launch"] * 33536  # per global step (both parts)
    per_step_val_calls = int(val["Calls"]) / int(full["Calls"])
    t_full = float(full["AverageNs"]) * 1e-9
    t_val = float(val["AverageNs"]) * 1e-9 * per_step_val_calls
    res = {
        "generator": "scripts/rocprof_fracs.py",
        "stats": stats, "bench": bench, "timed_steps": steps,
        "peak_tflops": PEAK,
        "full": {"flop_per_dispatch": flop_full, "avg_dispatch_ms": t_full * 1e3,
                 "achieved_tflops": flop_full / t_full / 1e12, "frac": flop_full / t_full / 1e12 / PEAK},
        "value": {"flop_per_step": flop_val, "dispatches_per_step": per_step_val_calls,
                  "avg_step_ms": t_val * 1e3, "achieved_tflops": flop_val / t_val / 1e12,
                  "frac": flop_val / t_val / 1e12 / PEAK},
        "event_timed_frac": {"full": f["frac"], "value": v["frac"]},
    }
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
