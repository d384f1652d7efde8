#!/usr/bin/env python3
"""Does running the instance set as K concurrent solver calls (one host thread, one stream and one workspace each)
beat one call?  The K call chains interleave on the GPU: one chain's MFMA-bound MLP launches overlap another's
latency-bound Newton solves and the tails of each other's kernels.  Every instance runs the same iterations either way
(slot-independent arithmetic), so the results are compared bitwise.

    python scripts/concurrent_solve.py B G SLOTS K     (B x G seeded metric instances, as scripts/step_trace.py)

K Python threads, each calling solve_batch on its own torch stream.  Measured slower: 1299 traj/s for
one call against 1054 (K = 2) and 984 (K = 4); an in-library variant (one host thread and stream per group) 1122 and 856."""
import os
import sys
import threading
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    B, G, slots, K = (int(v) for v in sys.argv[1:5])
    mode = "py"
    import torch

    from nlotrajectories_amd import _abi
    from nlotrajectories_amd.nn import MlpWeights
    from nlotrajectories_amd.ops import DeviceMlp, sdf_mlp_eval
    from nlotrajectories_amd.problem import METRIC_PROBLEM
    from nlotrajectories_amd.sampling import sample_start_goal
    from nlotrajectories_amd.solver import solve_batch, workspace_bytes

    mlp = DeviceMlp(MlpWeights.artefact())

    def sdf(pts):
        return sdf_mlp_eval(mlp, torch.as_tensor(pts, dtype=torch.float32, device="cuda"), derivatives=False)[0].cpu().numpy()

    xs = [sample_start_goal(METRIC_PROBLEM, B, seed=k, sdf=sdf) for k in range(G)]
    x0 = torch.tensor(np.concatenate([a for a, _ in xs]), dtype=torch.float64, device="cuda")
    xg = torch.tensor(np.concatenate([b for _, b in xs]), dtype=torch.float64, device="cuda")
    n = len(x0)
    solve_batch(METRIC_PROBLEM, x0[:256], xg[:256], mlp=mlp, options=_abi.gpu_options())
    torch.cuda.synchronize()

    def opt_for(s):
        o = _abi.gpu_options()
        o.max_active = s
        return o

    # one call through `slots` slots
    ws1 = torch.empty(workspace_bytes(METRIC_PROBLEM, n, slots), dtype=torch.uint8, device="cuda")
    t = time.perf_counter()
    r1 = solve_batch(METRIC_PROBLEM, x0, xg, mlp=mlp, options=opt_for(slots), workspace=ws1)
    torch.cuda.synchronize()
    t1 = time.perf_counter() - t
    st1 = r1["status"].cpu().numpy()
    del ws1
    # K concurrent calls over contiguous parts, slots / K each
    parts = np.array_split(np.arange(n), K)
    streams = [torch.cuda.Stream() for _ in range(K)]
    wss = [torch.empty(workspace_bytes(METRIC_PROBLEM, len(p), slots // K), dtype=torch.uint8, device="cuda")
           for p in parts]
    out = [None] * K
    torch.cuda.synchronize()

    def work(i):
        with torch.cuda.stream(streams[i]):
            p = parts[i]
            out[i] = solve_batch(METRIC_PROBLEM, x0[p[0]:p[-1] + 1], xg[p[0]:p[-1] + 1], mlp=mlp,
                                 options=opt_for(slots // K), workspace=wss[i])
        streams[i].synchronize()

    t = time.perf_counter()
    th = [threading.Thread(target=work, args=(i,)) for i in range(K)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    torch.cuda.synchronize()
    tk = time.perf_counter() - t
    stk = torch.cat([o["status"] for o in out]).cpu().numpy()
    same = {k: bool((torch.cat([o[k] for o in out]) == r1[k]).all().item()) for k in ("status", "iters", "cost")}
    print(f"[{mode}] n={n} slots={slots}: one call {t1:.2f} s ({(st1 == 0).sum() / t1:.1f} traj/s); {K} concurrent calls "
          f"{tk:.2f} s ({(stk == 0).sum() / tk:.1f} traj/s); bitwise same {same}", flush=True)


if __name__ == "__main__":
    main()
