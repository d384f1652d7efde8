"""`run-benchmark --config X.yaml` on the GPU solver: the reference's scripts/run_benchmark.py:49-226 flow
(load + validate the YAML, build the NLP, solve, report objective / solver time / final state, SDF-quality
metrics, append the results CSV) with nlot_solve_batch in place of CasADi/IPOPT.

    python -m nlotrajectories_amd.cli --config benchmark_2_unicycle_circle.yaml --initializer linear

Differences from the reference, all loud:
  * initializer `rrt` (every shipped YAML) runs the batched GPU RRT (rrt.py) with a seeded counter-based
    random stream (the reference draws from Python's unseeded `random`); --initializer linear|default override
    it (default = CasADi's zero initial guess, run_benchmark.py:113-114 / DefualtInitializer);
  * solver.mode l4casadi trains a network in the reference (NNObstacleTrainer); here `--weights train` does the
    same (the seeded restatement in trainer.py, on the GPU), or the weights come from --weights (an .npz written
    by MlpWeights.save, e.g. data/b6_mlp128_seed0.npz, or the shipped artefact with --weights artefact);
  * solver.type sqpmethod is not provided (the reference's default benchmarks all use ipopt);
  * plots are not produced; the CSV row always carries all 20 header columns (the reference writes 17
    values under a 20-column header).
"""
from __future__ import annotations

import argparse
import sys
import time
from pathlib import Path

import numpy as np
import torch

from . import _abi, scene
from .config import Config
from .nn import MlpWeights
from .ops import DeviceMlp, sdf_mlp_eval
from .solver import solve_batch

CSV_HEADER = ("solver_mode,model_type,num_hidden_layers,hidden_dim,activation_function,omega_0,"
              "surface_loss_weight,eikonal_weight,num_steps,init_mode,objective_value,solver_time,mse,iou,"
              "hausdorff,chamfer,surface_loss,enforce_heading,use_smooth,smooth_weight")


def _metrics(cfg: Config, mlp, n=1000, lo=-1.0, hi=2.0):
    """run_benchmark.py:35-46 compute_metrics: approximated vs exact SDF on an n x n grid of [-1, 2]^2."""
    obs = cfg.obstacle_dicts()
    x = np.linspace(lo, hi, n)
    X, Y = np.meshgrid(x, x)
    try:
        exact = scene.exact_sdf(obs, X, Y)
    except NotImplementedError:
        return (None,) * 5
    if mlp is not None:
        pts = torch.tensor(np.stack([X.ravel(), Y.ravel()], 1), dtype=torch.float32, device="cuda")
        approx = sdf_mlp_eval(mlp, pts, derivatives=False)[0].cpu().numpy().astype(np.float64).reshape(X.shape)
    else:
        approx = scene.approximated_sdf(obs, X, Y)
    return (scene.mse(exact, approx), scene.iou(exact, approx), scene.hausdorff(exact, approx, X, Y),
            scene.chamfer(exact, approx, X, Y), scene.surface_loss(exact, approx))


def _fmt(v, spec):
    return "None" if v is None else format(v, spec)


def run_benchmark(config_path, initializer="yaml", weights=None, results_dir="results", verbose=True,
                  options=None, metrics=True):
    """Returns (X_opt [nx, N+1], U_opt [nu, N], status str) like RunBenchmark.run (runner.py:148-153)."""
    config_path = Path(config_path)
    cfg = Config.load(config_path)
    if cfg.solver.type != "ipopt":
        raise NotImplementedError("solver.type sqpmethod is not provided (only the IPOPT restatement)")
    init = cfg.solver.initializer.choice.mode if initializer == "yaml" else initializer
    prob = cfg.to_problem()
    mlp = None
    if prob.sdf == "mlp":
        if weights is None:
            raise ValueError("solver.mode l4casadi: pass --weights train (train the config's network, as the "
                             "reference does), --weights <file.npz> or --weights artefact")
        if weights == "train":  # run_benchmark.py:84-95
            from .trainer import train_for_config

            model, _ = train_for_config(cfg, verbose=verbose)
            w = MlpWeights.from_module(model)
        else:
            w = MlpWeights.artefact() if weights == "artefact" else MlpWeights.load(weights)
        mlp = DeviceMlp(w)
    x0 = np.asarray(cfg.body.start_state, float)[None]
    xg = np.asarray(cfg.body.goal_state, float)[None]
    if x0.shape[1] != prob.nx or xg.shape[1] != prob.nx:
        raise ValueError(f"start/goal states must have {prob.nx} entries for {prob.dynamics}")
    X_init = np.zeros((1, prob.N + 1, prob.nx)) if init == "default" else None  # CasADi default guess
    if init == "rrt":  # RRTInitializer (run_benchmark.py:118-131) on the GPU, against the exact scene
        from .rrt import rrt_initial_guess

        ic = cfg.solver.initializer.choice
        X_init, ok = rrt_initial_guess(prob, x0, xg, bounds=ic.rrt_bounds, step_size=ic.step_size,
                                       max_iter=ic.max_iter, margin=ic.margin)
        if not bool(ok[0]):
            raise RuntimeError("RRT failed to find a path within max_iter.")
    opt = options or _abi.gpu_options()
    torch.cuda.synchronize()
    t0 = time.time()
    r = solve_batch(prob, x0, xg, mlp=mlp, options=opt, X_init=X_init)
    torch.cuda.synchronize()
    solver_time = time.time() - t0
    X = r["X"][0].cpu().numpy().T
    U = r["U"][0].cpu().numpy().T
    st = int(r["status"][0])
    status = "success" if st == 0 else "failed"
    if status == "failed":
        if verbose:
            names = {1: "maximum iterations", 2: "line search failure", 3: "numerical failure"}
            print(f"[IPOPT Error] {names.get(st, st)} after {int(r['iters'][0])} iterations")
            print("Dynamics violation:", np.linalg.norm(X[:, 1:] - X[:, :-1] - prob.dt * _f(prob, X[:, :-1], U)))
        return X, U, status
    obj = float(r["cost"][0])
    if not verbose:
        return X, U, status
    print("Objective value:", obj)
    print("Computation time for the solver:", solver_time)
    m = _metrics(cfg, mlp) if metrics else (None,) * 5
    for name, v in zip(("MSE", "IoU", "Hausdorff", "Chamfer", "Surface loss"), m):
        print(f"{name}:", v)
    print("Optimization complete.")
    print("Final state:", X[:, -1])
    out = Path(results_dir)
    out.mkdir(parents=True, exist_ok=True)
    f = out / f"{config_path.stem}_results.csv"
    new = not f.exists()
    mc = cfg.model
    with open(f, "a") as fh:
        if new:
            fh.write(CSV_HEADER + "\n")
        if cfg.solver.mode == "l4casadi":
            head = (f"{cfg.solver.mode},{mc.type},{mc.num_hidden_layers},{mc.hidden_dim},{mc.activation_function},"
                    f"{mc.omega_0},{mc.surface_loss_weight},{mc.eikonal_loss_weight}")
        else:
            head = f"{cfg.solver.mode},None,None,None,None,None,None,None"
        fh.write(f"{head},{cfg.solver.N},{init},{obj:3f},{solver_time:2f},{_fmt(m[0], '6f')},{_fmt(m[1], '6f')},"
                 f"{_fmt(m[2], '6f')},{_fmt(m[3], '6f')},{_fmt(m[4], '6f')},{cfg.solver.enforce_heading},"
                 f"{cfg.solver.use_smooth},{cfg.solver.smooth_weight}\n")
    return X, U, status


def _f(prob, X, U):
    """Continuous dynamics f(x, u) column-wise for the failure diagnostic (core/dynamics.py)."""
    x, u = X, U
    d = prob.dynamics
    if d == "point_1st":
        return np.stack([u[0], u[1], 0 * u[0], 0 * u[0]])
    if d == "point_2nd":
        return np.stack([x[2], x[3], u[0], u[1]])
    if d == "unicycle":
        return np.stack([u[0] * np.cos(x[2]), u[0] * np.sin(x[2]), u[1]])
    if d == "unicycle_2nd":
        return np.stack([x[3] * np.cos(x[2]), x[3] * np.sin(x[2]), x[4], u[0], u[1]])
    L = prob.wheelbase
    if d == "ackermann":
        return np.stack([u[0] * np.cos(x[2]), u[0] * np.sin(x[2]), u[0] * np.tan(x[3]) / L, u[1]])
    return np.stack([x[4] * np.cos(x[2]), x[4] * np.sin(x[2]), x[4] * np.tan(x[3]) / L, x[6],
                     (x[6] / (1 + x[3] ** 2) * x[4] + np.tan(x[3]) * u[0]) / L, u[0], u[1]])


def main(argv=None):
    ap = argparse.ArgumentParser(prog="run-benchmark")
    ap.add_argument("--config", type=str, required=True, help="Path to benchmark YAML config")
    ap.add_argument("--initializer", choices=["yaml", "linear", "default", "rrt"], default="yaml",
                    help="override the YAML initializer (yaml = the config's own, rrt for every shipped one)")
    ap.add_argument("--weights", type=str, default=None, help="learned-SDF weights: 'train' (NNObstacleTrainer), an .npz, or 'artefact'")
    ap.add_argument("--results", type=str, default="results")
    a = ap.parse_args(argv)
    run_benchmark(Path(a.config), initializer=a.initializer, weights=a.weights, results_dir=a.results)


if __name__ == "__main__":
    sys.exit(main())
