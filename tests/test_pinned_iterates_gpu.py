"""Per-instance pinning of the headline and benchmark-6 outcomes, failed and chaotic instances
included.

The split-parity tests (tests/outcomes.py) hold the GPU to the oracle's final outcome only where the oracle reproduces
itself, and to the oracle's own spread elsewhere.  Here every instance of tests/golden/oracle_outcomes.npz (and of
oracle_outcomes_varbounds.npz, the variable-bound form) is pinned along its path: k_i is the last iteration (<= 200)
up to which the oracle's five perturbed runs (x0 +- 1e-13 e_x, +- 1e-13 e_y, the net summed in reverse order) stay
within 1e-5 of the unperturbed run (tests/golden/make_oracle_outcomes.py), and the GPU run with max_iter = k_i must
return the oracle's iterate there: X and U within 1e-4 (the fp32-MLP iterate tolerance) and the
oracle's status at max_iter = k_i, solved, max_iter and restoration-failed instances alike.  The reference's
settings (runner.py:110-125) with its constraint-row bounds (runner.py:67-69,101-103).

Two runs per case, one per MLP arithmetic (include/nlot.h NLOT_MLP_ARITH_*: split-bf16, the product default, and
f32 MFMA).  Both are fp32 arithmetic whose MFMA sums round in other orders than the oracle's fp32 net, a perturbation
of the reverse-order net's size that the fixture's five runs sample only five times; k_i is the last iteration they
agree, often one iteration before a decision (filter, mu, restoration entry) flips, so a sixth perturbation can flip
it at k_i already (scripts/pin_probe.py: b6 instance 3 at iteration 6 under the split-bf16 net, 6.7e-6 against the
oracle's 3.5e-6 spread and 7e-2 one iteration later, while the f32 net tracks the oracle to 1.6e-6 through k_i = 20;
metric instance 63 the other way round).  The GPU also rounds its fp64 sums (Riccati sweeps, reductions) in other
orders in every iteration, where the fixture's runs differ only at the start.  So an instance outside 1e-4 is run on
the oracle up to k_i from the twelve WIDE starts (x0 +- 1e-11 .. 1e-7, tests/outcomes.py) and with six more orders of
the net's fp32 sums (NLOT_ORACLE_MLP_REV = 2..7: i -> i m mod H; the fixture's k_i rests on one such sample, the
reversed order): if one of them leaves the pinned iterate by more than 1e-4 there too, k_i was optimistic for the
GPU's perturbation size and the instance is excused (b6 variable-bound instance 3: four of the six orders end 5.0
away at k_i = 87, as both GPU nets do; the oracle is insensitive there to 1e-11 relative noise on every Newton
step).  Per net every remaining instance but 5 % (at least one), and none may miss under both nets: a miss one net
does not share is that net's rounding, not the solver."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
TOL = 1e-4
FILES = {"rows": "oracle_outcomes.npz", "varbounds": "oracle_outcomes_varbounds.npz"}


def _setup(case, artefact, arith):
    from nlotrajectories_amd.nn import MlpWeights
    from nlotrajectories_amd.ops import DeviceMlp
    from nlotrajectories_amd.problem import B6_PROBLEM, METRIC_PROBLEM

    if case == "metric":
        return METRIC_PROBLEM, DeviceMlp(artefact, arith)
    w = MlpWeights.load(os.path.join(os.path.dirname(HERE), "nlotrajectories_amd", "data", "b6_mlp128_seed0.npz"))
    return B6_PROBLEM, DeviceMlp(w, arith)


def _pinned_run(f, case, artefact, arith):
    """GPU iterate deviation from the pinned oracle iterate, and the GPU status, per instance."""
    from nlotrajectories_amd import _abi
    from nlotrajectories_amd.solver import solve_batch

    prob, mlp = _setup(case, artefact, arith)
    x0, xg, kp = f[f"{case}_x0"], f[f"{case}_xg"], f[f"{case}_kpin"]
    xinit = f.get(f"{case}_xinit")
    n = len(x0)
    dev = np.zeros(n)
    sg = np.zeros(n, np.int32)
    for k in np.unique(kp):  # one call per pinned iteration count
        idx = np.nonzero(kp == k)[0]
        opt = _abi.default_options(max_iter=int(k), general_bounds=int(f["general_bounds"]))
        r = solve_batch(prob, x0[idx], xg[idx], mlp=mlp, X_init=None if xinit is None else xinit[idx], options=opt)
        X, U = r["X"].cpu().numpy(), r["U"].cpu().numpy()
        dev[idx] = np.maximum(np.abs(X - f[f"{case}_Xpin"][idx]).reshape(len(idx), -1).max(1),
                              np.abs(U - f[f"{case}_Upin"][idx]).reshape(len(idx), -1).max(1))
        sg[idx] = r["status"].cpu().numpy()
    return dev, sg


def _wide_excused(f, case, form, idx, artefact):
    """Instances among idx whose oracle run from one of the WIDE starts is more than TOL from the pinned iterate at
    k_i (the oracle itself is not pinned there at the GPU's perturbation size)."""
    from concurrent.futures import ThreadPoolExecutor

    import oracle as O
    from outcomes import WIDE, mlp_order
    from nlotrajectories_amd import _abi
    from nlotrajectories_amd.nn import MlpWeights
    from nlotrajectories_amd.problem import B6_PROBLEM, METRIC_PROBLEM

    if case == "metric":
        prob, hm = METRIC_PROBLEM, O.HostMlp(artefact)
    else:
        prob = B6_PROBLEM
        hm = O.HostMlp(MlpWeights.load(os.path.join(os.path.dirname(HERE), "nlotrajectories_amd", "data",
                                                    "b6_mlp128_seed0.npz")))
    N, nx = prob.N, prob.nx
    xi = f.get(f"{case}_xinit")

    def one(args):
        i, (c, d, _) = args
        x = f[f"{case}_x0"][i].copy()
        x[c] += d
        k = int(f[f"{case}_kpin"][i])
        o = _abi.default_options(general_bounds=int(f["general_bounds"]), max_iter=k)
        r = O.solve_one(prob, x, f[f"{case}_xg"][i], hm, opt=o, X_init=None if xi is None else xi[i])
        return max(float(np.abs(r["X"] - f[f"{case}_Xpin"][i]).max()),
                   float(np.abs(r["U"] - f[f"{case}_Upin"][i]).max()))

    orders = (0, 2, 3, 4, 5, 6, 7)  # the net's summation order (one batch per order: the setting is process-wide)
    devs = np.zeros((len(idx), 0))
    with ThreadPoolExecutor(16) as ex:
        for v in orders:
            starts = WIDE if v == 0 else ((0, 0.0, False),)
            with mlp_order(v):
                d = np.array(list(ex.map(one, [(int(i), pd) for i in idx for pd in starts]))).reshape(len(idx), -1)
            devs = np.concatenate([devs, d], 1)
    for i, d in zip(idx, devs):
        print(f"[pinned] {case} {form} instance {int(i)} (k_i {int(f[f'{case}_kpin'][i])}): oracle from the WIDE starts "
              f"max |dev| {d[:len(WIDE)].max():.2e}, with other net orders {np.array2string(d[len(WIDE):], precision=1)}",
              flush=True)
    return {int(i) for i, d in zip(idx, devs) if d.max() > TOL}


@pytest.mark.parametrize("form", list(FILES))
@pytest.mark.parametrize("case", ["metric", "b6"])
def test_pinned_iterates_match_oracle(case, form, artefact):
    from outcomes import reproducible
    from nlotrajectories_amd import _abi

    path = os.path.join(HERE, "golden", FILES[form])
    if not os.path.exists(path):
        pytest.skip(f"{FILES[form]} not generated")
    f = dict(np.load(path))
    kp, st0 = f[f"{case}_kpin"], f[f"{case}_status"][0]
    # the oracle's status at max_iter = k_i (the fixture's {case}_stpin: max_iter, or the final status where the run
    # ends at the top of iteration k_i; a restoration line-search failure at k_i = iters happens inside the iteration)
    want = f[f"{case}_stpin"]
    R = reproducible({k: f[f"{case}_{k}"] for k in ("status", "cost", "xdev")})
    bad = {}
    for arith in ("f32", "split_bf16"):
        dev, sg = _pinned_run(f, case, artefact, arith)
        for name, g in (("solved", st0 == 0), ("max_iter", st0 == _abi.NLOT_MAXITER),
                        ("restoration failed", st0 == 4), ("other", ~np.isin(st0, (0, 1, 4))),
                        ("reproducible", R), ("chaotic", ~R)):
            if g.any():
                print(f"[pinned] {case} {form} {arith} {name}: {int(g.sum())} instances, k_i min / median / max "
                      f"{kp[g].min()} / {int(np.median(kp[g]))} / {kp[g].max()}, max |gpu - oracle| "
                      f"{dev[g].max():.2e}", flush=True)
        b = np.nonzero((dev > TOL) | (sg != want))[0]
        bad[arith] = b
        print(f"[pinned] {case} {form} {arith}: {len(b)} of {len(kp)} outside",
              [(int(i), int(kp[i]), float(dev[i]), int(sg[i]), int(want[i])) for i in b], flush=True)
    union = np.union1d(bad["f32"], bad["split_bf16"])
    exc = _wide_excused(f, case, form, union, artefact) if len(union) else set()
    left = {a: np.array([i for i in bad[a] if int(i) not in exc], int) for a in bad}
    print(f"[pinned] {case} {form}: excused (the oracle leaves the path too) {sorted(exc)}; left {left}", flush=True)
    cap = max(1, int(0.05 * len(kp)))
    assert len(left["f32"]) <= cap and len(left["split_bf16"]) <= cap, left
    assert len(np.intersect1d(left["f32"], left["split_bf16"])) == 0, left
