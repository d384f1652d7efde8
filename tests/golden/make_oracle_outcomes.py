#!/usr/bin/env python3
"""Oracle outcome fixtures for the solve-level GPU parity tests whose oracle runs are too long for a GPU test.

    python tests/golden/make_oracle_outcomes.py [--threads 8] [--only metric|b6]
        -> tests/golden/oracle_outcomes.npz (the reference's NLP form: constraint-row bounds, runner.py:67-69,101-103)

For each case it stores the instances (x0, xg, and the initial guesses where the case has its own) and the CPU
oracle's status / final cost / iterations / final-iterate deviation under tests/outcomes.FIXTURE_PERTURBATIONS, with
IPOPT's settings (default_options: max_iter 1000, tol 1e-4, adaptive mu, restoration on):

  row 0       the unperturbed run;
  rows 1-4    x0 +- 1e-13 e_x, x0 +- 1e-13 e_y (fp64-sized changes: the GPU rounds its fp64 sums, Riccati sweeps and
              libm calls differently in every iteration);
  rows 5-19   the net's fp32 sums in 15 other orders (NLOT_ORACLE_MLP_REV = 1 reversed, 2..7 strided, 8..15 seeded
              random permutations, oracle/nlot_oracle.c): rounding-level changes of the net's outputs, the kind the
              GPU's MFMA nets make (round 6: the round-5 fixture had only the reversed order, so its k_i was optimistic
              for the GPU nets and three after-the-fact excusals covered the difference).

  metric: 128 seeded instances of the headline workload (unicycle_2nd, b3 body, N = 50, artefact FourierMLP; the
          first 128 start/goal pairs of sample_start_goal(seed 0));
  b6:     24 benchmark-6 instances (BASELINE configs[3]: N = 100, the trained ring SDF) from the YAML's RRT initial
          guess, computed by the oracle's RRT restatement (oracle/rrt_oracle.py) and stored, so that the GPU test
          starts both solvers from the identical guess.

Per-instance pinned iterates: every run records its iterate at the top of each iteration (oracle_solve_trace).
  {case}_kpin[i] = k_i, the last iteration (at most PIN_CAP = 200, at most the shortest run) up to which all 19
      perturbed runs stay within PIN_TOL = 1e-5 (max |dX|, |dU|) of the unperturbed run, and at most k_seq below:
      where the GPU's MFMA nets (split-bf16, f32) must still be on the oracle's path;
  {case}_kseq[i], the same over fp64-sized perturbations only (rows 1-4, the merit function's sums reversed,
      +-1e-13 relative noise on every Newton step, and the oracle compiled with FMA contraction: SEQ_EXTRA / FMA_LIB,
      runs capped at 201 iterations, and SEQ_COMBINED: FMA contraction with the other fp64 perturbations at once):
      where the GPU with the oracle's own net arithmetic (NLOT_MLP_ARITH_SEQ: the net bitwise the oracle's) must
      still be on it; k_i is lowered further by NET_COMBINED (FMA contraction, another net order and step noise at
      once, as the GPU's MFMA-net run differs in all three);
  {case}_Xpin / _Upin / _Xseq / _Useq: the unperturbed iterate there (what max_iter = k returns);
  {case}_stpin / _stseq: the unperturbed run's status at max_iter = k (max_iter, or the final status where the run
      ends at the top of iteration k; a restoration line-search failure at k = iters happens inside iteration k and
      so returns max_iter);  {case}_pin_spread: the perturbed runs' largest deviation up to k_i;
  {case}_trials: the run's trial-point evaluations (one SDF value evaluation of the trial's corners each; DESIGN.md
      §8f cost model).

The oracle is deterministic (one instance per thread, no reductions across threads), so the GPU box's oracle
build reproduces these numbers bitwise; tests/test_oracle_outcomes_fixture.py re-runs a few instances on the CPU
to catch a fixture that no longer matches the oracle.  Test infrastructure: it imports the oracle only."""
import argparse
import os
import sys
import time
from concurrent.futures import ThreadPoolExecutor

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

PIN_CAP = 200
PIN_TOL = 1e-5
OUT = os.path.join(HERE, "oracle_outcomes.npz")
N_START = 5  # rows 0-4: the unperturbed run and the four start perturbations


def metric_instances(n=128):
    import oracle as O
    from nlotrajectories_amd.nn import MlpWeights
    from nlotrajectories_amd.problem import METRIC_PROBLEM
    from nlotrajectories_amd.sampling import sample_start_goal

    hm = O.HostMlp(MlpWeights.artefact())
    x0, xg = sample_start_goal(METRIC_PROBLEM, n, seed=0, sdf=lambda P: O.mlp_eval(hm, P, want=False)[0])
    return x0, xg


def b6_instances(n=24):
    import rrt_oracle as R
    from nlotrajectories_amd.problem import B6_PROBLEM, BENCHMARKS

    b = BENCHMARKS["b6"]
    rng = np.random.default_rng(4)
    X0 = np.repeat(np.array([b["start"]], float), n, 0)
    XG = np.repeat(np.array([b["goal"]], float), n, 0)
    X0[:, :2] += rng.uniform(-0.05, 0.05, (n, 2))
    XG[:, :2] += rng.uniform(-0.05, 0.05, (n, 2))
    Xi = np.stack([R.rrt_one(B6_PROBLEM, X0[i], XG[i], [[0.0, 0.0], [1.3, 1.3]], step_size=0.02, max_iter=5000,
                             margin=0.01, seed=3, instance=i)[0] for i in range(n)])
    return X0, XG, Xi


def pin(dev, iters, rows):
    """k, and the perturbed runs' largest deviation up to it, over the perturbed runs `rows`: dev [m, n, cap]
    per-iteration deviations of every run from run 0, iters [m, n] final iterations."""
    m, n, cap = dev.shape
    kpin = np.zeros(n, np.int32)
    spread = np.zeros(n)
    for i in range(n):
        kmax = min(PIN_CAP, cap - 1, int(iters[[0] + list(rows), i].min()))
        d = np.nanmax(dev[list(rows), i, :kmax + 1], axis=0)
        bad = np.nonzero(~(d <= PIN_TOL))[0]
        k = kmax if len(bad) == 0 else int(bad[0]) - 1
        kpin[i] = max(k, 0)
        spread[i] = float(np.nanmax(d[:kpin[i] + 1]))
    return kpin, spread


def pin_status(O, prob, X0, XG, hm, opt, Xi, kpin, threads):
    """The unperturbed run's status at max_iter = k_i, per instance."""
    def one(i):
        o = type(opt).from_buffer_copy(opt)
        o.max_iter = int(kpin[i])
        return O.solve_one(prob, X0[i], XG[i], hm, opt=o, X_init=None if Xi is None else Xi[i])["status"]

    with ThreadPoolExecutor(threads) as ex:
        return np.array(list(ex.map(one, range(len(X0)))), np.int32)


# k_seq's fp64-sized perturbations besides the four start ones: the merit sums reversed, and +-1e-13 relative noise
# on every Newton step (oracle/nlot_oracle.c NLOT_ORACLE_SUM_REV, NLOT_ORACLE_STEP_JITTER): the GPU rounds its fp64
# reductions and Riccati sweeps differently in every iteration, which a start perturbation models only at the start
SEQ_EXTRA = ({"NLOT_ORACLE_SUM_REV": "1"}, {"NLOT_ORACLE_STEP_JITTER": "1e-13"}, {"NLOT_ORACLE_STEP_JITTER": "-1e-13"})
# and the oracle compiled with FMA contraction (oracle/Makefile liboracle_nlot_fma.so): every fp64 operation rounded
# otherwise, as the GPU's code is compiled.  The restoration phase's entry amplifies that to 1e-10 .. 1e-8 within two
# iterations on benchmark 6 (instances 3, 7: 3.5e-10 / 2.0e-11 at iteration 7 where the other perturbations give
# 1e-12), which the start and step perturbations above do not reproduce.  Run in a child process (one library per
# process).
FMA_LIB = "liboracle_nlot_fma.so"


# Combined perturbations (round 6): the GPU's run differs from the oracle's in every respect at once (FMA
# contraction, other fp64 summation orders in its reductions and sweeps, and for the MFMA nets the net's fp32 order)
# where each row above varies one.  Run with the FMA-contracted build (child process): for k_seq, the merit sums
# reversed and step noise, or a start perturbation, on top of FMA contraction; for k_i, each of the net's 15 other
# orders on top of FMA contraction and step noise.
SEQ_COMBINED = ({"env": {"NLOT_ORACLE_SUM_REV": "1", "NLOT_ORACLE_STEP_JITTER": "1e-13"}},
                {"env": {"NLOT_ORACLE_STEP_JITTER": "-1e-13"}, "coord": 0, "d": 1e-13},
                {"env": {"NLOT_ORACLE_SUM_REV": "1"}, "coord": 1, "d": -1e-13})
NET_COMBINED = tuple({"env": {"NLOT_ORACLE_MLP_REV": str(v), "NLOT_ORACLE_STEP_JITTER": "1e-13" if v % 2 else "-1e-13"}}
                     for v in range(1, 16))


def fma_traces(case, data_path, threads, out_path):
    """Child-process side of the FMA rows: for each run of the input's `spec` (JSON list of {env, coord, d}), the
    traces (capped at PIN_CAP + 1 iterations) with the FMA-contracted oracle, as deviations from the input's T0."""
    import json

    import oracle as O
    from nlotrajectories_amd import _abi
    from nlotrajectories_amd.nn import MlpWeights
    from nlotrajectories_amd.problem import B6_PROBLEM, METRIC_PROBLEM

    assert os.path.basename(O.LIB_PATH) == FMA_LIB, O.LIB_PATH
    d = dict(np.load(data_path))
    prob = B6_PROBLEM if case == "b6" else METRIC_PROBLEM
    hm = O.HostMlp(MlpWeights.load(os.path.join(ROOT, "nlotrajectories_amd", "data", "b6_mlp128_seed0.npz"))
                   if case == "b6" else MlpWeights.artefact())
    X0, XG, Xi, T0 = d["x0"], d["xg"], d.get("xinit"), d["T0"]
    o = _abi.default_options(general_bounds=int(d["general_bounds"]), max_iter=PIN_CAP + 1)
    devs, its = [], []
    with ThreadPoolExecutor(threads) as ex:
        for run in json.loads(str(d["spec"])):
            x = X0.copy()
            x[:, run.get("coord", 0)] += run.get("d", 0.0)
            old = {k: os.environ.get(k) for k in run.get("env", {})}
            os.environ.update(run.get("env", {}))
            try:
                rs = list(ex.map(lambda i: O.solve_trace(prob, x[i], XG[i], hm, opt=o,
                                                         X_init=None if Xi is None else Xi[i], cap=PIN_CAP + 1),
                                 range(len(X0))))
            finally:
                for k, v in old.items():
                    if v is None:
                        os.environ.pop(k, None)
                    else:
                        os.environ[k] = v
            devs.append(np.abs(np.stack([r["trace"] for r in rs]) - T0).max(2))
            its.append([r["iters"] for r in rs])
    np.savez(out_path, dev=np.stack(devs), iters=np.array(its, np.int32))


def fma_rows(prob, X0, XG, opt, Xi, T0, spec, threads):
    """Deviation traces [len(spec), n, PIN_CAP + 1] and final iterations of the FMA-contracted oracle's runs `spec`
    from the plain oracle's unperturbed traces T0 (a child process: one oracle library per process)."""
    import json
    import subprocess
    import tempfile

    case = "b6" if prob.N == 100 else "metric"
    with tempfile.TemporaryDirectory() as td:
        src, dst = os.path.join(td, "in.npz"), os.path.join(td, "out.npz")
        np.savez(src, x0=X0, xg=XG, general_bounds=np.array(opt.general_bounds), T0=T0, spec=np.array(json.dumps(spec)),
                 **({"xinit": Xi} if Xi is not None else {}))
        subprocess.run([sys.executable, os.path.abspath(__file__), "--fma-traces", case, src, dst,
                        "--threads", str(threads)], check=True, env=dict(os.environ, NLOT_ORACLE_LIB=FMA_LIB))
        r = np.load(dst)
        return r["dev"], r["iters"]


def seq_pin(O, prob, X0, XG, hm, opt, Xi, threads):
    """k_seq over the four start perturbations and SEQ_EXTRA, from runs capped at PIN_CAP + 1 iterations (traces
    only: a capped run's trace equals the full run's up to the cap)."""
    from outcomes import PERTURBATIONS

    n = len(X0)
    o = type(opt).from_buffer_copy(opt)
    o.max_iter = PIN_CAP + 1
    runs = [(pd, {}) for pd in PERTURBATIONS[:N_START]] + [((0, 0.0, False), e) for e in SEQ_EXTRA]

    def one(args):
        i, (c, d, _) = args
        x = X0[i].copy()
        x[c] += d
        return O.solve_trace(prob, x, XG[i], hm, opt=o, X_init=None if Xi is None else Xi[i], cap=PIN_CAP + 1)

    m = len(runs)
    its = np.zeros((m, n), np.int32)
    dev = np.full((m, n, PIN_CAP + 1), np.nan)
    T0 = None
    with ThreadPoolExecutor(threads) as ex:
        for p, (pd, env) in enumerate(runs):
            old = {k: os.environ.get(k) for k in env}
            os.environ.update(env)
            try:
                rs = list(ex.map(one, [(i, pd) for i in range(n)]))
            finally:
                for k, v in old.items():
                    if v is None:
                        os.environ.pop(k, None)
                    else:
                        os.environ[k] = v
            T = np.stack([r["trace"] for r in rs])
            if T0 is None:
                T0 = T
            its[p] = [r["iters"] for r in rs]
            dev[p] = np.abs(T - T0).max(2)
    # the FMA-contracted build's unperturbed run and SEQ_COMBINED (child process)
    fdev, fits = fma_rows(prob, X0, XG, opt, Xi, T0, [{}] + list(SEQ_COMBINED), threads)
    its = np.concatenate([its, fits])
    dev = np.concatenate([dev, fdev])
    kseq, _ = pin(dev, its, range(1, len(dev)))
    N, nx, nu = prob.N, prob.nx, prob.nu
    XUp = T0[np.arange(n), kseq]
    return {"kseq": kseq, "Xseq": XUp[:, :(N + 1) * nx].reshape(n, N + 1, nx),
            "Useq": XUp[:, (N + 1) * nx:].reshape(n, N, nu), "stseq": pin_status(O, prob, X0, XG, hm, opt, Xi, kseq, threads),
            "T0": T0, "its0": its[0]}


def net_combined_pin(O, prob, X0, XG, hm, opt, Xi, threads, kpin, T0, its0):
    """k_i lowered to where a NET_COMBINED run (FMA build, another net order, step noise) leaves the unperturbed
    run, with the iterate and status there."""
    n = len(X0)
    fdev, fits = fma_rows(prob, X0, XG, opt, Xi, T0, list(NET_COMBINED), threads)
    kc, _ = pin(np.concatenate([np.zeros((1,) + fdev.shape[1:]), fdev]), np.concatenate([its0[None], fits]),
                range(1, len(fdev) + 1))
    k = np.minimum(kpin, kc).astype(np.int32)
    N, nx, nu = prob.N, prob.nx, prob.nu
    XUp = T0[np.arange(n), k]
    return {"kpin": k, "Xpin": XUp[:, :(N + 1) * nx].reshape(n, N + 1, nx),
            "Upin": XUp[:, (N + 1) * nx:].reshape(n, N, nu), "stpin": pin_status(O, prob, X0, XG, hm, opt, Xi, k, threads)}


def clamp_kpin(data, case):
    """k_i covers every perturbation, the fp64-sized ones of k_seq included (the MFMA nets' GPU runs differ from the
    oracle in the fp64 arithmetic too): where k_seq < k_i, k_i = k_seq with k_seq's iterate and status."""
    lo = data[f"{case}_kseq"] < data[f"{case}_kpin"]
    for a, b in (("kpin", "kseq"), ("Xpin", "Xseq"), ("Upin", "Useq"), ("stpin", "stseq")):
        data[f"{case}_{a}"] = np.where(lo.reshape((-1,) + (1,) * (data[f"{case}_{a}"].ndim - 1)),
                                       data[f"{case}_{b}"], data[f"{case}_{a}"])


def run_case(O, prob, X0, XG, hm, opt, Xi, threads):
    """Outcomes under every perturbation, with the per-instance pinned iterates."""
    from outcomes import FIXTURE_PERTURBATIONS, mlp_order

    n, m = len(X0), len(FIXTURE_PERTURBATIONS)

    def one(args):  # one perturbation of one instance (ctypes releases the GIL)
        i, (c, d, _) = args
        x = X0[i].copy()
        x[c] += d
        return O.solve_trace(prob, x, XG[i], hm, opt=opt, X_init=None if Xi is None else Xi[i], cap=PIN_CAP + 1)

    st = np.zeros((m, n), np.int32)
    trials = np.zeros((m, n), np.int32)
    cost = np.zeros((m, n))
    its = np.zeros((m, n), np.int32)
    xdev = np.zeros((m, n))
    dev = np.full((m, n, PIN_CAP + 1), np.nan)
    XU0, T0 = None, None
    t = time.time()
    with ThreadPoolExecutor(threads) as ex:
        for p, pd in enumerate(FIXTURE_PERTURBATIONS):  # one batch per perturbation: the net's order is process-wide
            with mlp_order(pd[2]):
                rs = list(ex.map(one, [(i, pd) for i in range(n)]))
            XU = np.stack([np.concatenate([np.ravel(r["X"]), np.ravel(r["U"])]) for r in rs])
            T = np.stack([r["trace"] for r in rs])
            if XU0 is None:
                XU0, T0 = XU, T
            st[p] = [r["status"] for r in rs]
            cost[p] = [r["cost"] for r in rs]
            its[p] = [r["iters"] for r in rs]
            trials[p] = [r["trials"] for r in rs]
            xdev[p] = np.abs(XU - XU0).max(1)
            dev[p] = np.abs(T - T0).max(2)
            print(f"  perturbation {p} {pd}: {time.time() - t:.0f} s, statuses {np.bincount(st[p], minlength=7).tolist()}",
                  flush=True)
    kpin, spread = pin(dev, its, range(1, m))
    N, nx, nu = prob.N, prob.nx, prob.nu
    XUp = T0[np.arange(n), kpin]
    out = {"status": st, "cost": cost, "iters": its, "xdev": xdev, "trials": trials, "kpin": kpin, "pin_spread": spread,
           "Xpin": XUp[:, :(N + 1) * nx].reshape(n, N + 1, nx), "Upin": XUp[:, (N + 1) * nx:].reshape(n, N, nu),
           "stpin": pin_status(O, prob, X0, XG, hm, opt, Xi, kpin, threads)}
    sq = seq_pin(O, prob, X0, XG, hm, opt, Xi, threads)
    T0s, its0 = sq.pop("T0"), sq.pop("its0")
    out.update(sq)
    out.update(net_combined_pin(O, prob, X0, XG, hm, opt, Xi, threads, kpin, T0s, its0))
    d = {f"c_{k}": v for k, v in out.items()}
    clamp_kpin(d, "c")
    return {k[2:]: v for k, v in d.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--threads", type=int, default=8)
    ap.add_argument("--out", default=OUT)
    ap.add_argument("--only", default=None, help="metric | b6 (keeps the other case from an existing file)")
    ap.add_argument("--seq-pin", action="store_true",
                    help="recompute only the pinned iterations (k_seq, and k_i lowered by NET_COMBINED) in --out")
    ap.add_argument("--fma-traces", nargs=3, default=None, help=argparse.SUPPRESS)  # CASE IN.npz OUT.npz (seq_pin)
    a = ap.parse_args()
    if a.fma_traces:
        return fma_traces(a.fma_traces[0], a.fma_traces[1], a.threads, a.fma_traces[2])
    import oracle as O
    from nlotrajectories_amd import _abi
    from nlotrajectories_amd.nn import MlpWeights
    from nlotrajectories_amd.problem import B6_PROBLEM, METRIC_PROBLEM

    opt = _abi.default_options(general_bounds=1)
    data = dict(np.load(a.out)) if (a.only and os.path.exists(a.out)) else {}
    data["general_bounds"] = np.array(opt.general_bounds)

    if a.seq_pin:
        data = dict(np.load(a.out))
        hm6 = O.HostMlp(MlpWeights.load(os.path.join(ROOT, "nlotrajectories_amd", "data", "b6_mlp128_seed0.npz")))
        for case, prob, hm, xi in (("b6", B6_PROBLEM, hm6, "b6_xinit"), ("metric", METRIC_PROBLEM,
                                                                         O.HostMlp(MlpWeights.artefact()), None)):
            if f"{case}_x0" not in data or a.only not in (None, case):
                continue
            t = time.time()
            X0, XG, Xi = data[f"{case}_x0"], data[f"{case}_xg"], data.get(xi) if xi else None
            out = seq_pin(O, prob, X0, XG, hm, opt, Xi, a.threads)
            T0, its0 = out.pop("T0"), out.pop("its0")
            out.update(net_combined_pin(O, prob, X0, XG, hm, opt, Xi, a.threads, data[f"{case}_kpin"], T0, its0))
            data.update({f"{case}_{k}": v for k, v in out.items()})
            clamp_kpin(data, case)
            for k in ("kseq", "kpin"):
                kp = data[f"{case}_{k}"]
                print(f"{case} {k}: min / median / max {kp.min()} / {int(np.median(kp))} / {kp.max()} "
                      f"({time.time() - t:.0f} s)", flush=True)
        np.savez_compressed(a.out, **data)
        return

    def report(case, out, t):
        for k in ("kpin", "kseq"):
            kp = out[k]
            print(f"{case} {k}: min / median / max {kp.min()} / {int(np.median(kp))} / {kp.max()}", flush=True)
        print(f"{case}: {time.time() - t:.0f} s, statuses {np.bincount(out['status'][0], minlength=7).tolist()}",
              flush=True)

    if a.only in (None, "b6"):
        t = time.time()
        X0, XG, Xi = b6_instances()
        hm6 = O.HostMlp(MlpWeights.load(os.path.join(ROOT, "nlotrajectories_amd", "data", "b6_mlp128_seed0.npz")))
        out = run_case(O, B6_PROBLEM, X0, XG, hm6, opt, Xi, a.threads)
        data = {k: v for k, v in data.items() if not k.startswith("b6_")}
        data.update({"b6_x0": X0, "b6_xg": XG, "b6_xinit": Xi, **{f"b6_{k}": v for k, v in out.items()}})
        report("b6", out, t)
        np.savez_compressed(a.out, **data)
    if a.only in (None, "metric"):
        t = time.time()
        x0, xg = metric_instances()
        out = run_case(O, METRIC_PROBLEM, x0, xg, O.HostMlp(MlpWeights.artefact()), opt, None, a.threads)
        data = {k: v for k, v in data.items() if not k.startswith("metric_")}
        data.update({"metric_x0": x0, "metric_xg": xg, **{f"metric_{k}": v for k, v in out.items()}})
        report("metric", out, t)
        np.savez_compressed(a.out, **data)


if __name__ == "__main__":
    main()
