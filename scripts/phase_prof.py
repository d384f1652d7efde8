"""Phase timer run (needs libnlot_prof.so, NLOT_LIB=libnlot_prof.so): per-iteration phase times of
instance 0 at batch sizes 1 and B, printed by the device."""
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
from nlotrajectories_amd.solver import solve_batch  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 1
iters = int(sys.argv[2]) if len(sys.argv) > 2 else 12
mlp = DeviceMlp(MlpWeights.artefact())


def sdf(pts):
    return sdf_mlp_eval(mlp, torch.as_tensor(pts, dtype=torch.float32, device="cuda"), derivatives=False)[0].cpu().numpy()


x0, xg = sample_start_goal(METRIC_PROBLEM, max(B, 1), seed=0, sdf=sdf)
torch.cuda.synchronize()
t = time.perf_counter()
r = solve_batch(METRIC_PROBLEM, x0, xg, mlp=mlp, options=_abi.gpu_options(max_iter=iters))
torch.cuda.synchronize()
print(f"B={B} max_iter={iters} wall {time.perf_counter() - t:.3f} s", flush=True)
