"""Per-instance pinning of the headline and benchmark-6 outcomes, failed and chaotic
instances included, with no excusals.

The split-parity tests (tests/outcomes.py) hold the GPU to the oracle's final outcome only where the oracle reproduces
itself, and to the oracle's own spread elsewhere.  Here every instance of tests/golden/oracle_outcomes.npz is pinned
along its path (the reference's settings, runner.py:110-125, with its constraint-row bounds, runner.py:67-69,101-103):
the GPU run with max_iter = k must return the oracle's iterate there, X and U within 1e-4 (the fp32-MLP iterate
tolerance), and the oracle's status at max_iter = k, for every instance, solved, max_iter and
restoration-failed alike.  k per net arithmetic (include/nlot.h NLOT_MLP_ARITH_*):

  * seq (the net in the oracle's own summation order: bitwise the oracle's net for benchmark 6's ReLU-input net,
    within the libm's ulp for the artefact's Fourier layer): k_seq, the last iteration (<= 200) up to which the
    oracle's runs from x0 +- 1e-13 e_x, e_y stay within 1e-5 of the unperturbed run.  What is left between GPU and
    oracle is the solver's fp64 (other summation orders, FMA contraction, libm), so this pins the solver itself;
  * split_bf16 (the product default) and f32 (the MFMA nets): k_i, the same over all 19 perturbed runs of the fixture,
    the four starts and 15 other orders of the net's fp32 sums (tests/golden/make_oracle_outcomes.py).  The MFMA nets
    round their sums in other orders than the oracle's net, a perturbation those orders sample.

Round 5 pinned the MFMA nets at a k_i measured with one other net order, so k_i was optimistic for them, and an
excusal (the oracle leaving the path too under other orders or wider starts, checked after the fact) with a 5 %-per-net
cap covered the difference.  Both are gone: the perturbation set that defines k_i is now the one that excused, plus
(round 6) combined perturbations, the FMA-contracted oracle with another net order and step noise at once, as the
GPU's run differs in all of them together.

The bar: the product net (split_bf16) leaves the pinned path on no instance.  The selectable alternatives (f32, seq)
are held to the sampling bound of the definition itself: k is the minimum over K perturbed runs, so a run
exchangeable with them leaves before all of them with probability 1 / (K + 1) per instance, and a strict zero would
fail a correct net on most 24-instance batches; the count may not exceed the binomial 99.9 % quantile (miss_bound).
Every miss is printed with its k, deviation and statuses (DESIGN.md §5 lists them)."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
TOL = 1e-4
PRODUCT_NET = "split_bf16"
# perturbed runs that define k (tests/golden/make_oracle_outcomes.py): k_seq over the four starts, SEQ_EXTRA's 3,
# the FMA build and SEQ_COMBINED's 3; k_i over the fixture's 19, k_seq's 7 others and NET_COMBINED's 15
K_RUNS = {"pin": 19 + 7 + 15, "seq": 4 + 3 + 1 + 3}


def miss_bound(n, k_runs, alpha=1e-3):
    """Largest count of instances on which a run exchangeable with the k_runs perturbed ones leaves the path before
    all of them (probability 1 / (k_runs + 1) each, independent instances), at false-failure rate alpha."""
    from scipy.stats import binom

    return int(binom.isf(alpha, n, 1.0 / (k_runs + 1)))


def _setup(case, artefact, arith):
    from nlotrajectories_amd.nn import MlpWeights
    from nlotrajectories_amd.ops import DeviceMlp
    from nlotrajectories_amd.problem import B6_PROBLEM, METRIC_PROBLEM

    if case == "metric":
        return METRIC_PROBLEM, DeviceMlp(artefact, arith)
    w = MlpWeights.load(os.path.join(os.path.dirname(HERE), "nlotrajectories_amd", "data", "b6_mlp128_seed0.npz"))
    return B6_PROBLEM, DeviceMlp(w, arith)


def _pinned_run(f, case, artefact, arith, tag):
    """GPU iterate deviation from the pinned oracle iterate, and the GPU status, per instance."""
    from nlotrajectories_amd import _abi
    from nlotrajectories_amd.solver import solve_batch

    prob, mlp = _setup(case, artefact, arith)
    x0, xg, kp = f[f"{case}_x0"], f[f"{case}_xg"], f[f"{case}_k{tag}"]
    xinit = f.get(f"{case}_xinit")
    n = len(x0)
    dev = np.zeros(n)
    sg = np.zeros(n, np.int32)
    for k in np.unique(kp):  # one call per pinned iteration count
        idx = np.nonzero(kp == k)[0]
        opt = _abi.default_options(max_iter=int(k), general_bounds=int(f["general_bounds"]))
        r = solve_batch(prob, x0[idx], xg[idx], mlp=mlp, X_init=None if xinit is None else xinit[idx], options=opt)
        X, U = r["X"].cpu().numpy(), r["U"].cpu().numpy()
        dev[idx] = np.maximum(np.abs(X - f[f"{case}_X{tag}"][idx]).reshape(len(idx), -1).max(1),
                              np.abs(U - f[f"{case}_U{tag}"][idx]).reshape(len(idx), -1).max(1))
        sg[idx] = r["status"].cpu().numpy()
    return dev, sg


@pytest.mark.parametrize("arith", ["seq", "split_bf16", "f32"])
@pytest.mark.parametrize("case", ["metric", "b6"])
def test_pinned_iterates_match_oracle(case, arith, artefact):
    from outcomes import reproducible
    from nlotrajectories_amd import _abi

    f = dict(np.load(os.path.join(HERE, "golden", "oracle_outcomes.npz")))
    tag = "seq" if arith == "seq" else "pin"
    kp, st0 = f[f"{case}_k{tag}"], f[f"{case}_status"][0]
    # the oracle's status at max_iter = k (max_iter, or the final status where the run ends at the top of iteration
    # k; a restoration line-search failure at k = iters happens inside the iteration)
    want = f[f"{case}_st{tag}"]
    R = reproducible({k: f[f"{case}_{k}"] for k in ("status", "cost", "xdev")})
    dev, sg = _pinned_run(f, case, artefact, arith, tag)
    for name, g in (("solved", st0 == 0), ("max_iter", st0 == _abi.NLOT_MAXITER), ("restoration failed", st0 == 4),
                    ("other", ~np.isin(st0, (0, 1, 4))), ("reproducible", R), ("chaotic", ~R)):
        if g.any():
            print(f"[pinned] {case} {arith} {name}: {int(g.sum())} instances, k_{tag} min / median / max "
                  f"{kp[g].min()} / {int(np.median(kp[g]))} / {kp[g].max()}, max |gpu - oracle| {dev[g].max():.2e}",
                  flush=True)
    bad = np.nonzero((dev > TOL) | (sg != want))[0]
    allowed = 0 if arith == PRODUCT_NET else miss_bound(len(kp), K_RUNS[tag])
    print(f"[pinned] {case} {arith}: {len(bad)} of {len(kp)} outside (allowed {allowed})",
          [(int(i), int(kp[i]), float(dev[i]), int(sg[i]), int(want[i])) for i in bad], flush=True)
    assert len(bad) <= allowed, [(int(i), int(kp[i]), float(dev[i]), int(sg[i]), int(want[i])) for i in bad]
