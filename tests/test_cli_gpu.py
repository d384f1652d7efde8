"""run-benchmark end to end on the GPU: restated b2 (analytic SDF) and b3 (learned SDF, artefact weights),
linear initializer; the result CSV carries the reference header with all 20 columns."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
CFG = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "configs")


def _b2_easy(tmp_path):
    """benchmark_2's YAML with a start/goal pair well clear of the obstacle (converges in ~16 iterations on
    both sides; the YAML's own diagonal start/goal takes ~300 path-sensitive iterations under IPOPT's
    settings, where GPU and oracle may end in different outcomes)."""
    import yaml

    cfg = yaml.safe_load(open(os.path.join(CFG, "benchmark_2_unicycle_circle.yaml")))
    cfg["body"]["start_state"] = [0.0, 0.95, 0.0, 0.0, 0.0]
    cfg["body"]["goal_state"] = [1.0, 0.95, 0.0, 0.0, 0.0]
    f = tmp_path / "benchmark_2_unicycle_circle.yaml"
    f.write_text(yaml.safe_dump(cfg))
    return str(f)


def test_run_benchmark_cli(tmp_path):
    from nlotrajectories_amd.cli import CSV_HEADER, main

    name = "benchmark_2_unicycle_circle"
    main(["--config", _b2_easy(tmp_path), "--initializer", "linear", "--results", str(tmp_path)])
    rows = open(tmp_path / f"{name}_results.csv").read().strip().split("\n")
    assert rows[0] == CSV_HEADER
    vals = rows[1].split(",")
    assert len(vals) == 20
    assert float(vals[10]) >= 1.0 - 1e-6  # objective: at least the straight-line length to the goal


def test_run_benchmark_returns_trajectory(tmp_path):
    from nlotrajectories_amd.cli import run_benchmark

    X, U, status = run_benchmark(_b2_easy(tmp_path), initializer="linear", verbose=False)
    assert status == "success" and X.shape == (5, 51) and U.shape == (2, 50)
    assert np.abs(X[:, 0] - [0, 0.95, 0, 0, 0]).max() < 1e-4


def test_learned_config_matches_oracle():
    """benchmark_3 with the learned SDF (artefact weights): the CLI's outcome equals the oracle's on the
    same NLP (both end in a line-search failure from the linear guess under the adaptive setting)."""
    import oracle as O
    from nlotrajectories_amd.cli import run_benchmark
    from nlotrajectories_amd.config import Config
    from nlotrajectories_amd.nn import MlpWeights

    f = os.path.join(CFG, "benchmark_3_unicycle_convex.yaml")
    X, U, status = run_benchmark(f, initializer="linear", weights="artefact", verbose=False)
    cfg = Config.load(f)
    from nlotrajectories_amd import _abi

    rc = O.solve_one(cfg.to_problem(), cfg.body.start_state, cfg.body.goal_state, O.HostMlp(MlpWeights.artefact()),
                     opt=_abi.gpu_options())
    assert status == ("success" if rc["status"] == 0 else "failed")
    assert X.shape == (5, 41) and U.shape == (2, 40)


def test_run_benchmark_with_the_yaml_rrt_initializer(tmp_path):
    """The shipped YAML's own initializer (rrt, the default of every benchmark) now runs: the GPU RRT's path
    (seeded) starts the solve, and the run returns a trajectory from the start state."""
    from nlotrajectories_amd.cli import run_benchmark

    X, U, status = run_benchmark(_b2_easy(tmp_path), verbose=False)
    print("rrt-initialised b2:", status, flush=True)
    assert status in ("success", "failed") and X.shape == (5, 51) and U.shape == (2, 50)
    assert np.abs(X[:2, 0] - [0.0, 0.95]).max() < 1e-4
