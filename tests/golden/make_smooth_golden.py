"""Golden vectors of the smooth-activation SDF networks, computed by the REFERENCE's own modules (runs only where
/root/reference exists; the output tests/golden/smooth_golden.npz is what travels).

The reference's core/nn_architectures.py (FourierMLP with activation_function tanh / sigmoid / leaky_relu,
:42-72; SIREN with SineLayer, :8-26,75-100) is imported from the reference tree (torch only), built under
torch.manual_seed(seed) with the reference's own initialisers, and evaluated in fp64 with torch autograd: value,
gradient and Hessian at seeded points (the quantities jac_ / jac_adj1_nn_sdf trace, gen/nn_sdf.cpp:57-104).  The
weights are stored flattened in this package's kernel layout (nlotrajectories_amd.nn.MlpWeights: A (in, out), b0,
W (out, in) per hidden layer, b, w_out, b_out, scale / omega_0, act), read from the reference module's parameters.

    python tests/golden/make_smooth_golden.py [--reference /root/reference]
"""
import argparse
import importlib.util
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ACT = {"ReLU": 0, "tanh": 1, "sigmoid": 2, "leaky_relu": 3, "sine": 4}  # include/nlot.h NLOT_ACT_*
# (name, architecture, hidden, num_layers, scale or omega_0, activation, seed)
CASES = [
    ("fourier_tanh", "fourier", 64, 3, 1.0, "tanh", 1),
    ("fourier_sigmoid_2x", "fourier", 128, 4, 2.0, "sigmoid", 2),
    ("fourier_leaky", "fourier", 64, 3, 1.0, "leaky_relu", 3),
    ("siren", "siren", 64, 3, 30.0, "sine", 4),
    ("siren_w5_3x", "siren", 128, 5, 5.0, "sine", 5),
]


def load_reference(ref):
    path = os.path.join(ref, "src", "nlotrajectories", "core", "nn_architectures.py")
    spec = importlib.util.spec_from_file_location("ref_nn_architectures", path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def flatten(model, arch, scale, act):
    g = lambda t: t.detach().double().numpy().astype(np.float32)
    if arch == "fourier":
        A, b0 = g(model.fourier.weights), g(model.fourier.bias)
        hidden = list(model.layers)
        W = [g(l.weight) for l in hidden]
        b = [g(l.bias) for l in hidden]
        in_kind = 1
    else:
        first, hidden = model.layers[0], list(model.layers[1:])
        A, b0 = g(first.linear.weight).T.copy(), g(first.linear.bias)
        W = [g(l.linear.weight) for l in hidden]
        b = [g(l.linear.bias) for l in hidden]
        in_kind = 0
    H = A.shape[1]
    return dict(in_kind=np.int32(in_kind), hidden=np.int32(H), n_hidden=np.int32(len(W)), fourier_scale=np.float32(scale),
                b_out=np.float32(g(model.output_layer.bias)[0]), act=np.int32(ACT[act]), A=A, b0=b0,
                W=np.stack(W) if W else np.zeros((0, H, H), np.float32),
                b=np.stack(b) if b else np.zeros((0, H), np.float32), w_out=g(model.output_layer.weight)[0])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reference", default="/root/reference")
    a = ap.parse_args()
    if not os.path.isdir(a.reference):
        print("reference tree absent; nothing to do")
        return 0
    ref = load_reference(a.reference)
    rng = np.random.default_rng(7)
    pts = rng.uniform(-0.5, 1.5, size=(256, 2)).astype(np.float32)  # the training box of run_benchmark.py:96
    out = {"p": pts}
    for name, arch, H, L, sc, act, seed in CASES:
        torch.manual_seed(seed)
        if arch == "fourier":
            m = ref.FourierMLP(2, H, 1, num_layers=L, scale=sc, activation_function=act)
        else:
            m = ref.SIREN(2, H, 1, num_layers=L, omega_0=sc)
        m.eval()
        w = flatten(m, arch, sc, act)
        # the fp32 weights as the kernels hold them, evaluated by the reference module in fp64
        md = m.double()
        with torch.no_grad():
            for prm, (k, v) in zip(md.parameters(), dict(md.named_parameters()).items()):
                prm.copy_(prm.float().double())
        P = torch.tensor(pts, dtype=torch.float64)
        f = lambda p: md(p[None])[0, 0]
        out[f"{name}/f"] = torch.func.vmap(f)(P).detach().numpy()
        out[f"{name}/grad"] = torch.func.vmap(torch.func.grad(f))(P).detach().numpy()
        out[f"{name}/hess"] = torch.func.vmap(torch.func.hessian(f))(P).detach().numpy()
        for k, v in w.items():
            out[f"{name}/{k}"] = v
        print(name, "f range", float(out[f"{name}/f"].min()), float(out[f"{name}/f"].max()))
    np.savez_compressed(os.path.join(HERE, "smooth_golden.npz"), **out)
    return 0


if __name__ == "__main__":
    sys.exit(main())
