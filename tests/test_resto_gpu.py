"""IPOPT's feasibility restoration phase (MinC_1NrmRestorationPhase) and soft restoration on the GPU vs the oracle
(runner.py:113-125 runs IPOPT with its defaults, which restore whenever the filter line search fails).

Iterates: after k iterations (restoration iterations count, as in IPOPT; an instance stopped inside a restoration
phase reports the restoration iterate on both sides) GPU X / U / S equal the oracle's within 1e-7 (1e-6 beyond 10
iterations) or 20x the oracle's own response to a 1e-13 change of the start, on cases whose restoration phases the
oracle reports (b2 without slack; benchmark 6's solver settings at N = 100: restoration from iteration 3, solved
at 32; benchmark 6's ring scene: 20 restoration phases).  Status and iteration count are compared where the
oracle reproduces its own under that change of the start.  Full solves: the restoration statuses appear on the
GPU, and outcomes agree with the oracle per instance as well as the oracle agrees with itself."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ITERS = {
    # b2 without slack from the YAML's start is chaotic from iteration 5 on (the oracle's own response to a 1e-13
    # change of the start reaches 5e-3): a perturbed pair that stays reproducible through its restoration phase
    "b2_no_slack_p5": (5, 10, 15, 20, 30),
    "b6_settings_N100": (2, 3, 4, 6, 10, 20, 40),
    "b6_elliptical_rings": (3, 4, 8, 15, 30),
}


def _case(name):
    from test_branches_gpu import _cases

    if name == "b2_no_slack_p5":  # the 6th draw of rng(5) around the YAML's start / goal
        prob, x0, xg = _cases()["b2_no_slack"]
        rng = np.random.default_rng(5)
        for _ in range(6):
            a, g = np.array(x0, float), np.array(xg, float)
            a[:2] += rng.uniform(-0.05, 0.05, 2)
            g[:2] += rng.uniform(-0.05, 0.05, 2)
        return prob, a.tolist(), g.tolist()
    return _cases()[name]


@pytest.mark.parametrize("name", list(ITERS))
def test_restoration_iterates_match_oracle(name):
    import oracle as O
    from nlotrajectories_amd import _abi
    from nlotrajectories_amd.solver import solve_batch

    prob, x0, xg = _case(name)
    resto_seen = 0
    for k in ITERS[name]:
        opt = _abi.default_options(max_iter=k)
        rg = solve_batch(prob, np.array([x0], float), np.array([xg], float), options=opt)
        rc = O.solve_one(prob, np.array(x0, float), np.array(xg, float), opt=opt)
        xp = np.array(x0, float)
        xp[0] += 1e-13
        rp = O.solve_one(prob, xp, np.array(xg, float), opt=opt)
        sens = max(float(np.abs(rp[n] - rc[n]).max()) for n in ("X", "U", "S"))
        dx = {n: float(np.abs(rg[n][0].cpu().numpy() - rc[n]).max()) for n in ("X", "U", "S")}
        print(name, "k", k, "status", rc["status"], "iters", rc["iters"], "resto phases", rc["resto_phases"],
              "soft", rc["soft_resto_steps"], dx, "oracle sensitivity", sens, flush=True)
        resto_seen = max(resto_seen, rc["resto_phases"])
        if rp["status"] == rc["status"] and rp["iters"] == rc["iters"]:  # outcome reproducible by the oracle itself
            assert rg["status"][0].item() == rc["status"], (name, k)
            assert rg["iters"][0].item() == rc["iters"], (name, k)
        tol = max(1e-7 if k <= 10 else 1e-6, 20 * sens)
        for n, v in dx.items():
            assert v <= tol, (name, k, n, v)
    assert resto_seen >= 1, name


@pytest.mark.parametrize("name", ["b2_no_slack", "b6_settings_N100", "b5_ackermann2nd_squares", "b6_elliptical_rings"])
def test_restoration_full_solves_match_oracle(name):
    """12 perturbed start/goal pairs: per-instance status equality with the oracle (both with restoration) on
    >= 75 %, final cost within 1e-4 relative on jointly solved instances (>= 80 % of them), and without slack
    (every corner constraint hard: the starts are infeasible for the linear initial guess) at least half solve
    where the round-2 GPU path solved none."""
    import oracle as O
    from nlotrajectories_amd import _abi
    from nlotrajectories_amd.solver import solve_batch

    prob, x0, xg = _case(name)
    rng = np.random.default_rng(11)
    B = 12
    X0 = np.repeat(np.array([x0], float), B, 0)
    XG = np.repeat(np.array([xg], float), B, 0)
    X0[:, :2] += rng.uniform(-0.05, 0.05, (B, 2))
    XG[:, :2] += rng.uniform(-0.05, 0.05, (B, 2))
    opt = _abi.default_options()
    rg = solve_batch(prob, X0, XG, options=opt)
    rc = O.solve_batch(prob, X0, XG, opt=opt, threads=8)
    xp = X0.copy()
    xp[:, 0] += 1e-13
    rp = O.solve_batch(prob, xp, XG, opt=opt, threads=8)
    sg = rg["status"].cpu().numpy()
    both = (sg == 0) & (rc["status"] == 0)
    rel = np.abs(rg["cost"].cpu().numpy() - rc["cost"]) / np.abs(rc["cost"])
    self_agree = (rp["status"] == rc["status"]).mean()
    print(name, "gpu", sg.tolist(), "oracle", rc["status"].tolist(), "perturbed oracle", rp["status"].tolist(),
          "iters gpu", rg["iters"].cpu().numpy().tolist(), "oracle", rc["iters"].tolist(), "rel cost",
          np.round(rel[both], 8).tolist(), flush=True)
    if name == "b6_elliptical_rings":
        # the analytic ring scene in casadi mode signs its distance by a quadrant test: the corridor
        # reads negative everywhere, the NLP is infeasible, and which failure (restoration failed / max_iter) ends
        # a run is decided by chaotic restoration phases with mu ~ 1e2 on both sides: compare solved / unsolved
        assert ((sg == 0) == (rc["status"] == 0)).mean() >= min(0.75, ((rp["status"] == 0) == (rc["status"] == 0)).mean() - 2 / B)
    else:
        assert (sg == rc["status"]).mean() >= min(0.75, self_agree - 2 / B)
    if both.any():
        # final costs at tol 1e-4 are loose where the NLP is flat (b2 without slack: the oracle restarted at its own
        # solution moves the cost by up to 1.5e-3): 1e-4 on 80 % of the jointly solved instances, or the GPU's
        # differences within 3x the oracle's own run-to-run envelope (1e-13 start perturbation), quartile and max
        selfb = both & (rp["status"] == 0)
        rel_self = np.abs(rp["cost"] - rc["cost"])[selfb] / np.abs(rc["cost"][selfb])
        q_self = np.quantile(rel_self, 0.75) if len(rel_self) else 0.0
        m_self = rel_self.max() if len(rel_self) else 0.0
        print(name, "cost envelope: gpu q75 / max", np.quantile(rel[both], 0.75), rel[both].max(), "oracle self",
              q_self, m_self, flush=True)
        assert (rel[both] <= 1e-4).mean() >= 0.8 or (
            np.quantile(rel[both], 0.75) <= 3 * max(1e-4, q_self) and rel[both].max() <= 3 * max(1e-4, m_self))
    if name in ("b2_no_slack", "b6_settings_N100"):
        assert (sg == 0).sum() >= B // 2


def test_restoration_statuses_on_metric(artefact):
    """64 seeded metric instances: the instances whose line search fails now go through the soft restoration and
    the restoration phase (or stop at an almost feasible point, theta <= 1e-2 tol, as IPOPT does): restoration
    statuses appear, no line-search-failed status (2) remains, and the GPU solves the instances the oracle does."""
    import torch

    import oracle as O
    from nlotrajectories_amd import _abi
    from nlotrajectories_amd.ops import DeviceMlp
    from nlotrajectories_amd.problem import METRIC_PROBLEM
    from nlotrajectories_amd.sampling import sample_start_goal
    from nlotrajectories_amd.solver import solve_batch

    tm = artefact.torch_module()
    sdf = lambda P: tm(torch.tensor(np.asarray(P), dtype=torch.float32)).detach().numpy()[:, 0]
    x0, xg = sample_start_goal(METRIC_PROBLEM, 64, seed=0, sdf=sdf)
    opt = _abi.default_options()
    rg = solve_batch(METRIC_PROBLEM, x0, xg, mlp=DeviceMlp(artefact), options=opt)
    rc = O.solve_batch(METRIC_PROBLEM, x0, xg, O.HostMlp(artefact), opt=opt, threads=16)  # the box's CPU share
    sg = rg["status"].cpu().numpy()
    print("metric gpu", np.bincount(sg, minlength=7).tolist(), "oracle", np.bincount(rc["status"], minlength=7).tolist(),
          "agree", (sg == rc["status"]).mean(), flush=True)
    assert (sg == _abi.NLOT_LS_FAILED).sum() == 0 and ((sg == 4) | (sg == 5)).sum() > 0
    # max_iter vs restoration_failed is decided late along chaotic paths: the solved / unsolved outcome is compared
    assert ((sg == 0) == (rc["status"] == 0)).mean() >= 0.85
