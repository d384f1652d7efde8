#!/usr/bin/env python3
"""Is a GPU net arithmetic's error against the fp64 truth a rounding-like spread, or does it carry a bias?  (GPU box;
diagnostics for DESIGN.md §5.)

For the artefact FourierMLP and benchmark 6's trained ReLU net, at 200,000 seeded points: value and gradient from
each GPU arithmetic (split_bf16, f32, seq) and from the oracle in several fp32 summation orders, minus torch fp64.
Prints per arithmetic the mean, the standard deviation and the mean / (std / sqrt(n)) of the value error, and the
same for the gradient components, as one JSON line.  A rounding-like arithmetic has a mean within a few standard
errors of 0 and a spread like the oracle orders'.

    python scripts/net_bias_probe.py [--n 200000]
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tests"))


def stats(e):
    e = np.asarray(e, np.float64)
    m, s = float(e.mean()), float(e.std())
    return {"mean": m, "std": s, "z": m / (s / np.sqrt(len(e))) if s > 0 else 0.0, "max_abs": float(np.abs(e).max())}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=200000)
    a = ap.parse_args()
    import torch

    import oracle as O
    from outcomes import mlp_order
    from nlotrajectories_amd.nn import MlpWeights
    from nlotrajectories_amd.ops import DeviceMlp, sdf_mlp_eval

    nets = {"artefact": MlpWeights.artefact(),
            "b6": MlpWeights.load(os.path.join(ROOT, "nlotrajectories_amd", "data", "b6_mlp128_seed0.npz"))}
    rng = np.random.default_rng(11)
    pts = rng.uniform(-0.3, 1.3, size=(a.n, 2)).astype(np.float32)
    out = {}
    for name, w in nets.items():
        m = w.torch_module().double()
        p64 = torch.tensor(pts, dtype=torch.float64, requires_grad=True)
        f = m(p64)[:, 0]
        (g,) = torch.autograd.grad(f.sum(), p64)
        f64, g64 = f.detach().numpy(), g.numpy()
        res = {}
        for arith in ("split_bf16", "f32", "seq"):
            v, gg, _ = (x.cpu().numpy() for x in sdf_mlp_eval(DeviceMlp(w, arith), torch.tensor(pts, device="cuda")))
            res[f"gpu_{arith}"] = {"f": stats(v - f64), "gx": stats(gg[:, 0] - g64[:, 0]), "gy": stats(gg[:, 1] - g64[:, 1])}
        hm = O.HostMlp(w)
        for v_ in (0, 1, 2, 8, 9):
            with mlp_order(v_):
                v, gg, _ = O.mlp_eval(hm, pts)
            res[f"oracle_order_{v_}"] = {"f": stats(v - f64), "gx": stats(gg[:, 0] - g64[:, 0]),
                                         "gy": stats(gg[:, 1] - g64[:, 1])}
        out[name] = res
        for k, r in res.items():
            print(f"[bias] {name} {k}: f mean {r['f']['mean']:+.3e} std {r['f']['std']:.3e} z {r['f']['z']:+.1f} | "
                  f"gx z {r['gx']['z']:+.1f} gy z {r['gy']['z']:+.1f}", flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
