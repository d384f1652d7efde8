"""Single-instance iteration latency of the product build: B=1 (and B=64) solves capped at max_iter, wall
time per lock-step step, with set_timing for the k_iterate share."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from nlotrajectories_amd import _abi  # noqa: E402
from nlotrajectories_amd.nn import MlpWeights  # noqa: E402
from nlotrajectories_amd.ops import DeviceMlp, sdf_mlp_eval  # noqa: E402
from nlotrajectories_amd.problem import METRIC_PROBLEM  # noqa: E402
from nlotrajectories_amd.sampling import sample_start_goal  # noqa: E402
from nlotrajectories_amd.solver import last_stats, set_timing, solve_batch  # noqa: E402

mlp = DeviceMlp(MlpWeights.artefact())


def sdf(pts):
    return sdf_mlp_eval(mlp, torch.as_tensor(pts, dtype=torch.float32, device="cuda"), derivatives=False)[0].cpu().numpy()


for B in (1, 64):
    x0, xg = sample_start_goal(METRIC_PROBLEM, B, seed=3, sdf=sdf)
    opt = _abi.gpu_options(max_iter=40)
    solve_batch(METRIC_PROBLEM, x0, xg, mlp=mlp, options=opt)
    set_timing(True)
    torch.cuda.synchronize()
    t = time.perf_counter()
    r = solve_batch(METRIC_PROBLEM, x0, xg, mlp=mlp, options=opt)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t
    st = last_stats()
    set_timing(False)
    steps = st["iterations"]
    print(f"B={B}: {steps} steps, {dt / steps * 1e6:.0f} us/step wall, k_iterate {st['iterate_ms'] / steps * 1e3:.0f} "
          f"us/step, mlp {(st['mlp_full_ms'] + st['mlp_value_ms']) / steps * 1e3:.0f} us/step", flush=True)
