"""Per-step anatomy of a continuous-batching metric solve (diagnostics, not the product).

    python scripts/step_trace.py run B G SLOTS OUTDIR        # G seeded batches of B through SLOTS slots;
                                                          # writes OUTDIR/steps.txt (NLOT_STEP_LOG) + res.npz
    rocprofv3 --kernel-trace --output-format csv -d D -o trace -- python scripts/step_trace.py run ...
    python scripts/step_trace.py reduce TRACE.csv OUTDIR     # per-step kernel durations -> OUTDIR/kern.npz
    python scripts/step_trace.py report OUTDIR               # tables by active-count bucket

Step s is the s-th k_accept launch; a launch belongs to the first step whose k_accept ends after it starts.
"""
import bisect
import csv
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

STEP_COLS = ["step", "active", "evals", "trials", "unused", "reused", "solves", "resto", "soc", "resto_solves",
             "next_active", "att_sum", "att_max", "att_multi", "resto_att_max"]
KERNELS = [("mlp_full", "mlp_bf16<128, true>"), ("mlp_value", "mlp_bf16<128, false>"),
           ("iter_a", "k_iter_a<"), ("ric", "k_ric<3, false, false>"), ("ric_soc", "k_ric<3, false, true>"),
           ("ric_resto", "k_ric<3, true"), ("iter_b", "k_iter_b<"), ("accept", "k_accept<"),
           ("resto_a", "k_resto_a<"), ("resto_b", "k_resto_b<"), ("resto_ls", "k_resto_ls<"),
           ("points", "k_points"), ("admit", "k_admit"), ("copy", "copyBuffer"), ("fill", "fillBuffer"),
           ("ric_tpi", "k_ric_tpi<"), ("ric_tpi_fwd", "k_ric_tpi_fwd<"), ("soc_tpi", "k_soc_tpi<")]


def run(B, G, slots, outdir):
    os.makedirs(outdir, exist_ok=True)
    log = os.path.join(outdir, "steps.txt")
    if os.path.exists(log):
        os.remove(log)
    import torch

    from nlotrajectories_amd import _abi
    from nlotrajectories_amd.nn import MlpWeights
    from nlotrajectories_amd.ops import DeviceMlp, sdf_mlp_eval
    from nlotrajectories_amd.problem import METRIC_PROBLEM
    from nlotrajectories_amd.sampling import sample_start_goal
    from nlotrajectories_amd.solver import solve_batch

    mlp = DeviceMlp(MlpWeights.artefact())

    def sdf(pts):
        return sdf_mlp_eval(mlp, torch.as_tensor(pts, dtype=torch.float32, device="cuda"), derivatives=False)[0].cpu().numpy()

    xs = [sample_start_goal(METRIC_PROBLEM, B, seed=k, sdf=sdf) for k in range(G)]
    x0 = torch.tensor(np.concatenate([a for a, _ in xs]), dtype=torch.float64, device="cuda")
    xg = torch.tensor(np.concatenate([b for _, b in xs]), dtype=torch.float64, device="cuda")
    opt = _abi.gpu_options()
    opt.max_active = slots
    # warm-up call (kernels loaded), not logged
    solve_batch(METRIC_PROBLEM, x0[:256], xg[:256], mlp=mlp, options=_abi.gpu_options())
    torch.cuda.synchronize()
    os.environ["NLOT_STEP_LOG"] = log  # read once, at the first logged solve
    if os.environ.get("STEP_TIMING") == "1":  # hipEvent timing of the MLP / iterate / k_ric launches, as bench.py's timed steps
        from nlotrajectories_amd.solver import set_timing

        set_timing(True)
    import time
    t = time.perf_counter()
    r = solve_batch(METRIC_PROBLEM, x0, xg, mlp=mlp, options=opt)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t
    st = r["status"].cpu().numpy()
    print(f"B={B} G={G} slots={slots}: {dt:.2f} s, solved {(st == 0).sum()} -> {(st == 0).sum() / dt:.1f} traj/s, "
          f"status {np.bincount(st, minlength=7).tolist()}", flush=True)
    np.savez(os.path.join(outdir, "res.npz"), status=st, iters=r["iters"].cpu().numpy(), cost=r["cost"].cpu().numpy(),
             wall=dt)


def reduce(trace, outdir):
    rows = []
    with open(trace) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    acc = [r for r in rows if "k_accept<" in r[2]]
    # the logged solve is the last one: its steps are the last len(steps) k_accept launches
    steps = np.loadtxt(os.path.join(outdir, "steps.txt"), dtype=np.int64, ndmin=2)
    n = len(steps)
    acc = acc[-n:]
    ends = [a[1] for a in acc]
    t0 = acc[0][0]
    K = np.zeros((n, len(KERNELS)), np.int64)
    for s, e, name in rows:
        if e < t0 - 10_000_000:
            continue
        i = bisect.bisect_left(ends, s)
        if i >= n:
            continue
        for c, (_, pat) in enumerate(KERNELS):
            if pat in name:
                K[i, c] += e - s
                break
    wall = np.diff(np.array([acc[0][0]] + ends, dtype=np.int64))
    np.savez(os.path.join(outdir, "kern.npz"), K=K, wall=wall, names=np.array([k for k, _ in KERNELS]))
    print(f"reduced {len(rows)} launches into {n} steps; wall {wall.sum() / 1e9:.2f} s")


def report(outdir):
    S = np.loadtxt(os.path.join(outdir, "steps.txt"), dtype=np.int64, ndmin=2)
    cols = {c: S[:, i] for i, c in enumerate(STEP_COLS)}
    kp = os.path.join(outdir, "kern.npz")
    Kz = np.load(kp) if os.path.exists(kp) else None
    act = cols["active"]
    edges = [0, 256, 1024, 4096, 8192, 16384, 24576, 32768, 65536, 1 << 30]
    print(f"{len(act)} steps; Newton solves {cols['solves'].sum()}, corrections {cols['soc'].sum()}, "
          f"trial slots {cols['trials'].sum()}, restoration solves {cols['resto_solves'].sum()}")
    hdr = "active<=  steps  mean_act  solves/step  soc/step  trials/step  steps/iter  att/solve  att_max  multi/step"
    if Kz is not None:
        names = list(Kz["names"])
        hdr += "  wall_ms/step " + " ".join(f"{n[:9]:>9}" for n in names if n not in ("copy", "fill", "admit", "points"))
    print(hdr)
    for lo, hi in zip(edges[:-1], edges[1:]):
        m = (act > lo) & (act <= hi)
        if not m.any():
            continue
        line = (f"{hi:8d} {m.sum():6d} {act[m].mean():9.0f} {cols['solves'][m].mean():12.0f} {cols['soc'][m].mean():9.0f}"
                f" {cols['trials'][m].mean():12.0f} {act[m].sum() / max(cols['solves'][m].sum(), 1):10.2f}"
                f" {cols['att_sum'][m].sum() / max(cols['solves'][m].sum(), 1):10.3f} {cols['att_max'][m].mean():8.2f}"
                f" {cols['att_multi'][m].mean():10.0f}")
        if Kz is not None:
            K, wall = Kz["K"], Kz["wall"]
            line += f"  {wall[m].mean() / 1e6:12.3f} " + " ".join(
                f"{K[m, c].mean() / 1e6:9.3f}" for c, n in enumerate(names) if n not in ("copy", "fill", "admit", "points"))
            line += f"   total {wall[m].sum() / 1e9:7.2f} s"
        print(line)
    if Kz is not None:
        print(f"wall total {Kz['wall'].sum() / 1e9:.2f} s")


if __name__ == "__main__":
    cmd = sys.argv[1]
    if cmd == "run":
        run(int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4]), sys.argv[5])
    elif cmd == "reduce":
        reduce(sys.argv[2], sys.argv[3])
    else:
        report(sys.argv[2])
