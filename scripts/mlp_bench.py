"""MLP kernel microbenchmark: full (value + grad + Hessian) and value-only launches on the metric-size
point set (16384 instances x 204 corners), hipEvent-timed, with achieved TFLOP/s (fp32-equivalent flops) and the
fraction of the split-bf16 peak (2.5 PF/s dense bf16 / 6 products = 416.7 TF/s).  NLOT_LIB selects the build."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from nlotrajectories_amd.nn import MlpWeights  # noqa: E402
from nlotrajectories_amd.ops import DeviceMlp, sdf_mlp_eval  # noqa: E402

stress = len(sys.argv) > 2 and sys.argv[2] == "stress"  # python scripts/mlp_bench.py P [stress]
P = int(sys.argv[1]) if len(sys.argv) > 1 else 16384 * 204
w = MlpWeights.stress_sdf_mlp(0) if stress else MlpWeights.artefact()
mlp = DeviceMlp(w)
pts = (torch.rand(P, 2, device="cuda") * 1.6 - 0.3).contiguous()
for full in (True, False):
    for _ in range(2):
        sdf_mlp_eval(mlp, pts, derivatives=full)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    n = 10
    e0.record()
    for _ in range(n):
        sdf_mlp_eval(mlp, pts, derivatives=full)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / n
    flop = P * (w.flops_per_point_fwd_grad if full else w.flops_per_point_fwd)
    print(f"{'full ' if full else 'value'} P={P} {ms:.3f} ms  {flop / ms / 1e9:.1f} TFLOP/s  "
          f"(frac {flop / ms / 1e9 / 416.7:.3f} of the split-bf16 peak)", flush=True)
