"""Dump GPU iterates after k accepted steps (max_iter = k) for the benchmark_2 instance."""
import sys, os
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from nlotrajectories_amd import _abi
from nlotrajectories_amd.problem import BENCHMARKS
from nlotrajectories_amd.solver import solve_batch
b = BENCHMARKS["b2"]
out = {}
for k in [0, 1, 2, 3, 4, 6, 8, 12, 20]:
    r = solve_batch(b["problem"], np.array([b["start"]]), np.array([b["goal"]]), options=_abi.gpu_options(max_iter=k))
    out[f"X{k}"] = r["X"][0].cpu().numpy(); out[f"U{k}"] = r["U"][0].cpu().numpy(); out[f"S{k}"] = r["S"][0].cpu().numpy()
    out[f"st{k}"] = r["status"][0].item(); out[f"it{k}"] = r["iters"][0].item()
os.makedirs("gpurun_out", exist_ok=True)
np.savez("gpurun_out/iterates_b2.npz", **out)
print("ok")
