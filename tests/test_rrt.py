"""RRT initializer (core/trajectory_initialization.py:58-239): the oracle restatement on the CPU, and the GPU's
batched nlot_rrt_init against it (`-m gpu`).  The benchmark YAMLs' own RRT settings (rrt_bounds, step_size
0.02, max_iter 5000, margin) come from the reference's Config dumps in tests/golden/nlp_golden.json."""
import json
import os

import numpy as np
import torch
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = json.load(open(os.path.join(HERE, "golden", "nlp_golden.json")))
CASES = ["benchmark_1_dot_circle.yaml", "benchmark_2_unicycle_circle.yaml", "benchmark_3_unicycle_convex.yaml",
         "benchmark_4_dot_nonconvex.yaml", "benchmark_5_ackermann_circle.yaml", "benchmark_6_ackermann_wave.yaml"]


def _case(fn):
    from nlotrajectories_amd.config import Config

    cfg = Config.model_validate(GOLD["configs"][fn])
    ini = GOLD["configs"][fn]["solver"]["initializer"][0]
    kw = dict(bounds=ini["rrt_bounds"], step_size=ini["step_size"], max_iter=ini["max_iter"], margin=ini["margin"])
    return cfg.to_problem().with_(sdf="analytic"), np.array(cfg.body.start_state), np.array(cfg.body.goal_state), kw


def test_oracle_rrt_paths_join_start_and_goal():
    import rrt_oracle as R

    for fn in CASES[:2] + CASES[3:4]:
        prob, x0, xg, kw = _case(fn)
        X, ok = R.rrt_one(prob, x0, xg, seed=0, **kw)
        assert ok, fn
        assert X.shape == (prob.N + 1, prob.nx)
        np.testing.assert_allclose(X[0, :2], x0[:2], atol=1e-12)
        np.testing.assert_allclose(X[-1, :2], xg[:2], atol=1e-12)
        assert np.all(X[:, 2:] == 0.0)  # lifted with zeros (:233-235)


def test_oracle_rrt_failure_is_reported():
    import rrt_oracle as R

    prob, x0, xg, kw = _case(CASES[1])
    kw["max_iter"] = 3
    X, ok = R.rrt_one(prob, x0, xg, seed=0, **kw)
    assert not ok  # the reference raises RuntimeError("RRT failed to find a path within max_iter.")
    np.testing.assert_allclose(X, np.linspace(x0, xg, prob.N + 1), atol=1e-15)


def test_oracle_inflation_as_written():
    """RectangleGeometry: max |np.min(body point)| + margin (not the corner norm, :108-111); others 0."""
    import rrt_oracle as R
    from nlotrajectories_amd.problem import Problem

    p = Problem(shape="rectangle", length=0.2, width=0.1, obstacles=[{"type": "circle", "center": (0, 0), "radius": 1}])
    assert abs(R.inflation(p, 0.01) - 0.11) < 1e-15
    assert R.inflation(p.with_(shape="triangle"), 0.01) == 0.0


@pytest.mark.gpu
@pytest.mark.parametrize("fn", CASES)
def test_gpu_rrt_matches_oracle(fn):
    """Same draws, same tree, same shortcuts: X_init within 1e-9 of the oracle (scipy's LAPACK spline solve
    vs the kernel's Thomas algorithm differ by rounding) for 6 perturbed starts per benchmark scene."""
    import rrt_oracle as R
    from nlotrajectories_amd.rrt import rrt_initial_guess

    prob, x0, xg, kw = _case(fn)
    rng = np.random.default_rng(7)
    B = 6
    X0 = np.repeat(x0[None], B, 0)
    X0[1:, :2] += rng.uniform(-0.02, 0.02, (B - 1, 2))
    XG = np.repeat(xg[None], B, 0)
    Xg, okg = rrt_initial_guess(prob, X0, XG, seed=3, **kw)
    Xg, okg = Xg.cpu().numpy(), okg.cpu().numpy()
    for b in range(B):
        Xc, okc = R.rrt_one(prob, X0[b], XG[b], seed=3, instance=b, **kw)
        err = float(np.abs(Xg[b] - Xc).max())
        print(fn, b, "ok", okc, bool(okg[b]), "max |dX|", err, flush=True)
        assert bool(okg[b]) == okc
        assert err < 1e-9, (fn, b, err)


@pytest.mark.gpu
def test_gpu_rrt_chunked_equals_one_call(monkeypatch):
    """rrt_initial_guess splits a batch into nlot_rrt_init calls of CHUNK instances (bounded workspace); the draws
    are keyed by the global instance index (NlotRrtOptions.first_instance), so the result equals one call's."""
    import nlotrajectories_amd.rrt as rrt

    prob, x0, xg, kw = _case(CASES[0])
    rng = np.random.default_rng(11)
    B = 13
    X0 = np.repeat(x0[None], B, 0)
    X0[:, :2] += rng.uniform(-0.02, 0.02, (B, 2))
    XG = np.repeat(xg[None], B, 0)
    Xa, oka = rrt.rrt_initial_guess(prob, X0, XG, seed=5, **kw)
    monkeypatch.setattr(rrt, "CHUNK", 4)
    Xb, okb = rrt.rrt_initial_guess(prob, X0, XG, seed=5, **kw)
    assert torch.equal(Xa, Xb) and torch.equal(oka, okb)


@pytest.mark.gpu
def test_gpu_rrt_concurrent_streams():
    """Two rrt_initial_guess calls in flight on two streams (each call allocates its own workspace on its stream):
    both results equal the sequential ones (a shared cached workspace let such calls corrupt each
    other's trees)."""
    import nlotrajectories_amd.rrt as rrt

    prob, x0, xg, kw = _case(CASES[0])
    rng = np.random.default_rng(12)
    B = 64
    X0 = np.repeat(x0[None], B, 0)
    X0[:, :2] += rng.uniform(-0.02, 0.02, (B, 2))
    XG = np.repeat(xg[None], B, 0)
    Xa, oka = rrt.rrt_initial_guess(prob, X0, XG, seed=5, **kw)
    Xb, okb = rrt.rrt_initial_guess(prob, X0, XG, seed=6, **kw)
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    with torch.cuda.stream(s1):
        Xc, okc = rrt.rrt_initial_guess(prob, X0, XG, seed=5, **kw)
    with torch.cuda.stream(s2):
        Xd, okd = rrt.rrt_initial_guess(prob, X0, XG, seed=6, **kw)
    torch.cuda.synchronize()
    assert torch.equal(Xa, Xc) and torch.equal(oka, okc)
    assert torch.equal(Xb, Xd) and torch.equal(okb, okd)


# ---- reference-pinned fixtures (tests/golden/make_rrt_golden.py: the REFERENCE's RRTInitializer driven like
# run_benchmark.py:116-127, its `random` replaced by the counter-based stream; circle / square scenes) ----
RRT_GOLD = json.load(open(os.path.join(HERE, "golden", "rrt_golden.json")))["cases"]


def _gold_problem(c):
    from nlotrajectories_amd.config import Config

    return Config.model_validate(GOLD["configs"][c["yaml"]]).to_problem().with_(sdf="analytic")


@pytest.mark.parametrize("i", range(len(RRT_GOLD)))
def test_oracle_rrt_matches_reference_rrt(i):
    """The restatement reproduces the reference's X_init (tree, intermediate points, shortcuts, CubicSpline)."""
    import rrt_oracle as R

    c = RRT_GOLD[i]
    X, ok = R.rrt_one(_gold_problem(c), np.array(c["x0"]), np.array(c["xg"]), c["bounds"], step_size=c["step_size"],
                      max_iter=c["max_iter"], margin=c["margin"], seed=c["seed"], instance=c["instance"])
    assert ok == c["ok"]
    np.testing.assert_allclose(X, np.array(c["X_init"]), atol=1e-12, rtol=0)


@pytest.mark.gpu
@pytest.mark.parametrize("yaml", sorted({c["yaml"] for c in RRT_GOLD}))
def test_gpu_rrt_matches_reference_rrt(yaml):
    """nlot_rrt_init on the scene's 4 instances (batch index = the fixture's instance) against the reference's X_init:
    1e-9 (the kernel's Thomas spline solve vs scipy's LAPACK)."""
    from nlotrajectories_amd.rrt import rrt_initial_guess

    cs = sorted([c for c in RRT_GOLD if c["yaml"] == yaml], key=lambda c: c["instance"])
    c0 = cs[0]
    Xg, okg = rrt_initial_guess(_gold_problem(c0), np.array([c["x0"] for c in cs]), np.array([c["xg"] for c in cs]),
                                c0["bounds"], step_size=c0["step_size"], max_iter=c0["max_iter"], margin=c0["margin"],
                                seed=c0["seed"])
    Xg, okg = Xg.cpu().numpy(), okg.cpu().numpy()
    for b, c in enumerate(cs):
        err = float(np.abs(Xg[b] - np.array(c["X_init"])).max())
        print(yaml, b, "max |dX| vs reference", err, flush=True)
        assert bool(okg[b]) == c["ok"] and err < 1e-9
