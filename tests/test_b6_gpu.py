"""BASELINE.json configs[3] on the GPU: benchmark 6 (ackermann_2nd, no slack = per-corner constraints, smooth
w = 0.5) at N = 100 with the learned SDF trained on its ring corridor (data/b6_mlp128_seed0.npz).  Iterates vs
the oracle (fp32 MLP on both sides: 1e-4, or 20x the oracle's own response to a 1e-13 start perturbation), and
a seeded batch with the YAML's RRT initial guess against the oracle's outcomes (tests/outcomes.py split parity)."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
DATA = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "nlotrajectories_amd", "data")


def _setup():
    import oracle as O
    from nlotrajectories_amd.nn import MlpWeights
    from nlotrajectories_amd.ops import DeviceMlp
    from nlotrajectories_amd.problem import B6_PROBLEM, BENCHMARKS

    w = MlpWeights.load(os.path.join(DATA, "b6_mlp128_seed0.npz"))
    return O, B6_PROBLEM, BENCHMARKS["b6"], DeviceMlp(w), O.HostMlp(w)


def test_b6_iterates_match_oracle():
    O, prob, b, mlp, hm = _setup()
    from nlotrajectories_amd import _abi
    from nlotrajectories_amd.solver import solve_batch

    x0, xg = np.array(b["start"], float), np.array(b["goal"], float)
    x0[1] += 0.02  # off the corridor's centre line by a little
    for k in (1, 3, 8):
        opt = _abi.gpu_options(max_iter=k)
        rg = solve_batch(prob, x0[None], xg[None], mlp=mlp, options=opt)
        rc = O.solve_one(prob, x0, xg, hm, opt=opt)
        xp = x0.copy()
        xp[0] += 1e-13
        rp = O.solve_one(prob, xp, xg, hm, opt=opt)
        sens = max(float(np.abs(rp[n] - rc[n]).max()) for n in ("X", "U"))
        d = {n: float(np.abs(rg[n][0].cpu().numpy() - rc[n]).max()) for n in ("X", "U")}
        print("b6 k", k, "status", rc["status"], rg["status"][0].item(), d, "oracle sensitivity", sens, flush=True)
        assert rg["status"][0].item() == rc["status"]
        for n, v in d.items():
            assert v <= max(1e-4, 20 * sens), (k, n, v)


def test_b6_batch_matches_oracle():
    """24 seeded benchmark-6 instances (BASELINE configs[3]: N = 100, trained ring SDF) from the YAML's RRT initial
    guess: the instances, the guesses (the oracle's RRT restatement, oracle/rrt_oracle.py; the batched GPU RRT
    reproduces it, tests/test_rrt.py) and the oracle's outcomes under the fixture's 20 runs (x0, x0 +- 1e-13 e_x, e_y,
    the net's fp32 sums in 15 other orders) are the fixture tests/golden/oracle_outcomes.npz (its 1000-iteration
    N = 100 solves take an hour of CPU).  Split parity (tests/outcomes.py), per net on its own: identical status and
    final cost within 1e-4 on every instance the oracle reproduces under all 20 runs; on the chaotic ones a status
    agreement at least the lowest of the 19 perturbed runs' (no slack).  Three nets (include/nlot.h
    NLOT_MLP_ARITH_*): seq (the oracle's own summation order, bitwise its net here), f32 and the product's split-bf16.
    A solve floor (the GPU solves at least as many instances as the perturbed oracle run that solves fewest, less one,
    and at least one; jointly solved instances end within 10 % of the oracle's cost — the chaotic group's status
    agreement alone would pass a GPU that solves nothing here, where the oracle's statuses are mostly failures); and
    every instance the GPU reports solved satisfies its constraints (dynamics, start / terminal states, per-corner
    learned SDF >= 0 without slack)."""
    import os

    O, prob, b, _, hm = _setup()
    from outcomes import WIDE, net_parity, oracle_outcomes
    from nlotrajectories_amd import _abi
    from nlotrajectories_amd.nn import MlpWeights
    from nlotrajectories_amd.ops import DeviceMlp
    from nlotrajectories_amd.solver import solve_batch

    f = dict(np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "oracle_outcomes.npz")))
    X0, XG, Xi = f["b6_x0"], f["b6_xg"], f["b6_xinit"]
    out = {k: f[f"b6_{k}"] for k in ("status", "cost", "iters", "xdev")}
    opt = _abi.default_options()
    widen = lambda i: oracle_outcomes(O, prob, X0[i], XG[i], hm, opt=opt, X_init=Xi[i], perturbations=WIDE)
    w = MlpWeights.load(os.path.join(DATA, "b6_mlp128_seed0.npz"))
    res = {}
    for arith in ("seq", "f32", "split_bf16"):
        r = solve_batch(prob, X0, XG, mlp=DeviceMlp(w, arith), X_init=Xi, options=opt)
        res[arith] = (r["status"].cpu().numpy(), r["cost"].cpu().numpy())
        print("b6 batch statuses", arith, "gpu", res[arith][0].tolist(), flush=True)
    print("b6 batch statuses oracle", out["status"][0].tolist(), flush=True)
    net_parity("b6 (24, RRT init)", out, res, widen=widen)
    st, cost = res["split_bf16"]
    floor = max(1, int(min((out["status"][k] == 0).sum() for k in range(out["status"].shape[0]))) - 1)
    both = (st == 0) & (out["status"][0] == 0)
    rel = np.abs(cost - out["cost"][0]) / np.abs(out["cost"][0])
    print(f"b6 solved: gpu {int((st == 0).sum())}, floor {floor}, jointly {int(both.sum())}, "
          f"max relative cost difference {rel[both].max() if both.any() else 0.0:.3g}", flush=True)
    assert (st == 0).sum() >= floor
    assert (rel[both] <= 0.1).all(), rel[both]
    X, U = r["X"].cpu().numpy(), r["U"].cpu().numpy()
    for i in np.where(st == 0)[0]:
        assert np.abs(X[i, 0] - X0[i]).max() < 1e-4
        assert np.abs(X[i, -1, [0, 1, 3, 4, 5, 6]] - XG[i, [0, 1, 3, 4, 5, 6]]).max() < 1e-4
        F = X[i, :-1] + prob.dt * np.stack([O.dynamics(prob, X[i, k], U[i, k]) for k in range(prob.N)])
        assert np.abs(X[i, 1:] - F).max() < 1e-4
        # per-corner learned SDF >= 0 (no slack), to the constraint tolerance
        c = np.concatenate([O.corners(prob, X[i, k]) for k in range(prob.N + 1)])
        v, _, _ = O.mlp_eval(hm, c, want=False)
        assert v.min() > -1e-4
