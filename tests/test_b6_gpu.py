"""BASELINE.json configs[3] on the GPU: benchmark 6 (ackermann_2nd, no slack = per-corner constraints, smooth
w = 0.5) at N = 100 with the learned SDF trained on its ring corridor (data/b6_mlp128_seed0.npz).  Iterates vs
the oracle (fp32 MLP on both sides: 1e-4, or 20x the oracle's own response to a 1e-13 start perturbation), and
a seeded batch with the YAML's RRT initial guess that solves where the oracle solves."""
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


def test_b6_batch_solves_where_the_oracle_solves():
    """24 seeded benchmark-6 instances with the YAML's RRT initial guess (the batched GPU RRT reproduces the
    oracle's RRT restatement; tests/test_rrt.py): instances 2 and 4 are solved by the oracle (77 and 412
    iterations, restoration on).  Both are chaotic in the oracle itself (measured on the CPU: instance 2 under
    +-1e-13 start perturbations ends at costs 7.36, 7.13, 7.16 or restoration-failed; instance 4 under 1e-12
    noise on the initial guess ends restoration-failed or at max_iter), so a per-instance 1e-4 cost match cannot
    be asked of any other floating-point order.  Asserted: the GPU solves at least one of them, within 10 % of
    the oracle's cost (the spread of the oracle's own solved outcomes), and every instance the GPU reports solved
    satisfies its constraints (dynamics, start / terminal states, per-corner learned SDF >= 0 without slack)."""
    O, prob, b, mlp, hm = _setup()
    import rrt_oracle as R
    from nlotrajectories_amd import _abi
    from nlotrajectories_amd.rrt import rrt_initial_guess
    from nlotrajectories_amd.solver import solve_batch

    rng = np.random.default_rng(4)
    B = 24
    X0 = np.repeat(np.array([b["start"]], float), B, 0)
    XG = np.repeat(np.array([b["goal"]], float), B, 0)
    X0[:, :2] += rng.uniform(-0.05, 0.05, (B, 2))
    XG[:, :2] += rng.uniform(-0.05, 0.05, (B, 2))
    rrt = dict(step_size=0.02, max_iter=5000, margin=0.01, seed=3)
    Xi, ok = rrt_initial_guess(prob, X0, XG, [[0.0, 0.0], [1.3, 1.3]], **rrt)
    r = solve_batch(prob, X0, XG, mlp=mlp, X_init=Xi)
    st, cost = r["status"].cpu().numpy(), r["cost"].cpu().numpy()
    print("b6 batch statuses", st.tolist(), flush=True)
    joint = []
    for i in (2, 4):
        Xr, _ = R.rrt_one(prob, X0[i], XG[i], [[0.0, 0.0], [1.3, 1.3]], instance=i, **rrt)
        rc = O.solve_one(prob, X0[i], XG[i], hm, opt=_abi.default_options(), X_init=Xr)
        print("instance", i, "oracle", rc["status"], rc["iters"], rc["cost"], "gpu", st[i], r["iters"][i].item(), cost[i],
              flush=True)
        assert rc["status"] == 0
        if st[i] == 0:
            joint.append(abs(cost[i] - rc["cost"]) / abs(rc["cost"]))
    assert joint and max(joint) <= 0.1, joint
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
