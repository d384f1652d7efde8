"""Dump GPU iterates after k accepted steps (max_iter = k) for a benchmark_2 instance, for comparison with
the oracle on the CPU.  python scripts/debug_iterates.py [tag] [opts as key=value ...]  (tag "tiny": the
tiny-step parity case of tests/test_solver_gpu.py)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from nlotrajectories_amd import _abi  # noqa: E402
from nlotrajectories_amd.problem import BENCHMARKS  # noqa: E402
from nlotrajectories_amd.solver import solve_batch  # noqa: E402

tag = sys.argv[1] if len(sys.argv) > 1 else "b2"
b = BENCHMARKS["b2"]
x0, xg, kw = b["start"], b["goal"], {}
if tag == "tiny":
    x0, xg, kw = [0.0, 0.05, 0.0, 0.0, 0.0], [1.0, 0.1, 0.0, 0.0, 0.0], dict(tiny_step_tol=0.1, tiny_step_y_tol=1e3)
elif tag == "tiny2":
    x0, xg, kw = [0.0, 0.8, 0.0, 0.0, 0.0], [1.0, 0.9, 0.0, 0.0, 0.0], dict(tiny_step_tol=0.05, tiny_step_y_tol=1e3)
out = {}
for k in range(0, 14):
    r = solve_batch(b["problem"], np.array([x0]), np.array([xg]), options=_abi.gpu_options(max_iter=k, **kw))
    out[f"X{k}"] = r["X"][0].cpu().numpy(); out[f"U{k}"] = r["U"][0].cpu().numpy(); out[f"S{k}"] = r["S"][0].cpu().numpy()
    out[f"st{k}"] = r["status"][0].item(); out[f"it{k}"] = r["iters"][0].item()
os.makedirs("gpurun_out", exist_ok=True)
np.savez(f"gpurun_out/iterates_{tag}.npz", **out)
print("ok")
