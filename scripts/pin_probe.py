#!/usr/bin/env python3
"""Where a pinned-iterate mismatch starts (tests/test_pinned_iterates_gpu.py): for the given fixture instances, the GPU
iterate at max_iter = k for k = 1..K against the unperturbed oracle trace (oracle_solve_trace) and the oracle's own
perturbed runs (the +-1e-13 starts and the reverse-order net), one line per k.

    python scripts/pin_probe.py --case b6 --inst 3 --kmax 24 [--arith split_bf16|f32|seq]

GPU box; test infrastructure (runs the oracle as the checker).  NLOT_MLP=f32 in the environment switches the GPU's
SDF net to its fp32 path for an A/B against the split-bf16 default."""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--case", default="b6")
    ap.add_argument("--inst", type=int, nargs="+", default=[3])
    ap.add_argument("--kmax", type=int, default=24)
    ap.add_argument("--kmin", type=int, default=1)
    ap.add_argument("--kstep", type=int, default=1)
    ap.add_argument("--arith", default="split_bf16", choices=["split_bf16", "f32", "seq"])
    a = ap.parse_args()
    import oracle as O
    from outcomes import PERTURBATIONS, mlp_order

    sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
    from make_oracle_outcomes import SEQ_EXTRA
    from nlotrajectories_amd import _abi
    from nlotrajectories_amd.nn import MlpWeights
    from nlotrajectories_amd.ops import DeviceMlp
    from nlotrajectories_amd.problem import B6_PROBLEM, METRIC_PROBLEM
    from nlotrajectories_amd.solver import solve_batch

    f = dict(np.load(os.path.join(ROOT, "tests", "golden", "oracle_outcomes.npz")))
    if a.case == "b6":
        prob = B6_PROBLEM
        w = MlpWeights.load(os.path.join(ROOT, "nlotrajectories_amd", "data", "b6_mlp128_seed0.npz"))
    else:
        prob, w = METRIC_PROBLEM, MlpWeights.artefact()
    hm, mlp = O.HostMlp(w), DeviceMlp(w, a.arith)
    gb = int(f["general_bounds"])
    N, nx, nu = prob.N, prob.nx, prob.nu
    for i in a.inst:
        x0, xg = f[f"{a.case}_x0"][i], f[f"{a.case}_xg"][i]
        xi = f[f"{a.case}_xinit"][i] if f"{a.case}_xinit" in f else None
        opt = _abi.default_options(general_bounds=gb)
        traces = []
        o_tr = _abi.default_options(general_bounds=gb, max_iter=a.kmax + 1)
        if a.arith == "seq":  # the fp64-sized perturbations of k_seq (make_oracle_outcomes.SEQ_EXTRA)
            runs = [(pd, {}) for pd in PERTURBATIONS[:5]] + [((0, 0.0, False), e) for e in SEQ_EXTRA]
        else:
            runs = [(pd, {}) for pd in PERTURBATIONS]
        for (c, d, rev), env in runs:
            x = x0.copy()
            x[c] += d
            os.environ.update(env)
            with mlp_order(rev):
                traces.append(O.solve_trace(prob, x, xg, hm, opt=o_tr, X_init=xi, cap=a.kmax + 1)["trace"])
            for k_ in env:
                os.environ.pop(k_, None)
        T0 = traces[0]
        print(f"instance {i}: kpin {int(f[f'{a.case}_kpin'][i])}, kseq {int(f[f'{a.case}_kseq'][i])}, "
              f"oracle status {int(f[f'{a.case}_status'][0, i])} "
              f"iters {int(f[f'{a.case}_iters'][0, i])}, net {a.arith}", flush=True)
        for k in range(a.kmin, a.kmax + 1, a.kstep):
            o = _abi.default_options(general_bounds=gb, max_iter=k)
            r = solve_batch(prob, x0[None], xg[None], mlp=mlp, X_init=None if xi is None else xi[None], options=o)
            g = np.concatenate([r["X"][0].cpu().numpy().ravel(), r["U"][0].cpu().numpy().ravel()])
            dg = float(np.nanmax(np.abs(g - T0[k])))
            dall = [float(np.nanmax(np.abs(t[k] - T0[k]))) for t in traces[1:]]
            dself = max(dall)
            dX = np.abs(g[:(N + 1) * nx] - T0[k][:(N + 1) * nx]).reshape(N + 1, nx)
            kk, jj = np.unravel_index(int(np.nanargmax(dX)), dX.shape)
            print(f"  k {k:3d} status {int(r['status'][0])} |gpu - oracle| {dg:.3e}  oracle self {dself:.3e} "
                  f"({' '.join(f'{v:.1e}' for v in dall)})  argmax X[{kk},{jj}]", flush=True)


if __name__ == "__main__":
    main()
