#!/usr/bin/env python3
"""Short metric solve at bench size for PMC passes (scripts/pmc_r03.sh): B instances of bench.py's workload
(sampler seed 0), max_iter iterations, IPOPT defaults; prints the solver's launch statistics as one JSON line
(points per MLP launch, Newton solves per k_ric launch) so per-dispatch counters can be turned into bytes/unit.

    python scripts/pmc_solve.py [B] [max_iter]
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch

    from nlotrajectories_amd import _abi
    from nlotrajectories_amd.nn import MlpWeights
    from nlotrajectories_amd.ops import DeviceMlp, sdf_mlp_eval
    from nlotrajectories_amd.problem import METRIC_PROBLEM
    from nlotrajectories_amd.sampling import sample_start_goal
    from nlotrajectories_amd.solver import last_stats, solve_batch

    B = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
    it = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    mlp = DeviceMlp(MlpWeights.artefact())

    def sdf(pts):
        return sdf_mlp_eval(mlp, torch.as_tensor(pts, dtype=torch.float32, device="cuda"), derivatives=False)[0].cpu().numpy()

    x0, xg = sample_start_goal(METRIC_PROBLEM, B, seed=0, sdf=sdf)
    x0 = torch.tensor(x0, device="cuda")
    xg = torch.tensor(xg, device="cuda")
    r = solve_batch(METRIC_PROBLEM, x0, xg, mlp=mlp, options=_abi.gpu_options(max_iter=it))
    torch.cuda.synchronize()
    st = last_stats()
    st["B"], st["max_iter"] = B, it
    st["status_counts"] = torch.bincount(r["status"].long(), minlength=7).tolist()
    st["instance_iterations"] = int(r["iters"].long().sum().item())
    print(json.dumps(st), flush=True)


if __name__ == "__main__":
    main()
