"""tests/golden/oracle_outcomes.npz (the reference's constraint-row bounds) still describes this oracle (CPU): the GPU
parity tests compare against its stored oracle outcomes (tests/outcomes.py) and pinned iterates
(tests/test_pinned_iterates_gpu.py), so a change of the oracle's arithmetic must regenerate it
(tests/golden/make_oracle_outcomes.py).  Re-runs the fixture's quickest instances (fewest iterations) at x0, two
perturbed starts and two other net orders (reversed, a seeded random permutation) and asks for bitwise the same
status, iterations and final cost, and a few pinned iterates (max_iter = k_i, k_seq) bitwise."""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)


def _fixture():
    return dict(np.load(os.path.join(HERE, "golden", "oracle_outcomes.npz")))


def test_fixture_layout():
    from outcomes import FIXTURE_PERTURBATIONS, reproducible

    f = _fixture()
    m = len(FIXTURE_PERTURBATIONS)
    assert int(f["general_bounds"]) == 1
    for case, n, N, nx in (("metric", 128, 50, 5), ("b6", 24, 100, 7)):
        assert f[f"{case}_x0"].shape[0] == n and f[f"{case}_status"].shape == (m, n)
        assert f[f"{case}_cost"].shape == (m, n) and f[f"{case}_iters"].shape == (m, n)
        assert f[f"{case}_xdev"].shape == (m, n) and (f[f"{case}_xdev"][0] == 0).all()
        assert f[f"{case}_trials"].shape == (m, n) and (f[f"{case}_trials"] >= 0).all()
        st, it = f[f"{case}_status"][0], f[f"{case}_iters"][0]
        for tag in ("pin", "seq"):
            kp = f[f"{case}_k{tag}"]
            assert kp.shape == (n,) and (kp >= 0).all() and (kp <= 200).all() and (kp <= it).all()
            assert f[f"{case}_X{tag}"].shape == (n, N + 1, nx) and f[f"{case}_U{tag}"].shape == (n, N, 2)
            sp = f[f"{case}_st{tag}"]
            assert sp.shape == (n,) and ((sp == 1) | ((kp == it) & (sp == st))).all()
        # k_seq (start perturbations only) is never shorter than k_i (every perturbation)
        assert (f[f"{case}_kseq"] >= f[f"{case}_kpin"]).all()
        assert (f[f"{case}_pin_spread"] <= 1e-5).all()
    assert f["b6_xinit"].shape == (24, 101, 7)
    # the split has both groups on the headline workload (tests/outcomes.py)
    R = reproducible({k: f[f"metric_{k}"] for k in ("status", "cost", "xdev")})
    print("metric fixture: reproducible", int(R.sum()), "of", len(R))
    assert 0 < R.sum() < len(R)


def test_fixture_matches_oracle():
    import oracle as O
    from outcomes import FIXTURE_PERTURBATIONS, mlp_order
    from nlotrajectories_amd import _abi
    from nlotrajectories_amd.nn import MlpWeights
    from nlotrajectories_amd.problem import B6_PROBLEM, METRIC_PROBLEM

    f = _fixture()
    opt = _abi.default_options(general_bounds=int(f["general_bounds"]))
    hm = O.HostMlp(MlpWeights.artefact())
    its = f["metric_iters"][0]
    for i in np.argsort(its, kind="stable")[:4]:
        for r in (0, 1, 3, 5, len(FIXTURE_PERTURBATIONS) - 1):
            coord, d, rev = FIXTURE_PERTURBATIONS[r]
            x0 = f["metric_x0"][i].copy()
            x0[coord] += d
            with mlp_order(rev):
                res = O.solve_one(METRIC_PROBLEM, x0, f["metric_xg"][i], hm, opt=opt)
            assert res["status"] == f["metric_status"][r, i] and res["iters"] == f["metric_iters"][r, i], (i, r)
            assert res["cost"] == f["metric_cost"][r, i], (i, r, res["cost"], f["metric_cost"][r, i])
    hm6 = O.HostMlp(MlpWeights.load(os.path.join(os.path.dirname(HERE), "nlotrajectories_amd", "data",
                                                 "b6_mlp128_seed0.npz")))
    i = int(np.argmin(f["b6_iters"][0]))
    res = O.solve_one(B6_PROBLEM, f["b6_x0"][i], f["b6_xg"][i], hm6, opt=opt, X_init=f["b6_xinit"][i])
    assert res["status"] == f["b6_status"][0, i] and res["iters"] == f["b6_iters"][0, i]
    assert res["cost"] == f["b6_cost"][0, i]
    # pinned iterates: the unperturbed run stopped at max_iter = k returns the stored iterate bitwise
    for tag in ("pin", "seq"):
        kp = f[f"metric_k{tag}"]
        for i in list(np.argsort(kp, kind="stable")[:2]) + [int(np.argmax(kp))]:
            o = _abi.default_options(general_bounds=int(f["general_bounds"]), max_iter=int(kp[i]))
            res = O.solve_one(METRIC_PROBLEM, f["metric_x0"][i], f["metric_xg"][i], hm, opt=o)
            assert (res["X"] == f[f"metric_X{tag}"][i]).all() and (res["U"] == f[f"metric_U{tag}"][i]).all(), (i, kp[i])
            assert res["status"] == f[f"metric_st{tag}"][i], (i, kp[i])
