"""Golden-vector generator (test infrastructure; runs only where /root/reference exists).

What it produces (all committed, small):
  nlotrajectories_amd/data/nn_sdf_artefact.npz
      The learned-SDF weights of the reference artefact `_l4c_generated/nn_sdf.pt`, extracted as
      RAW DATA: the zip members `nn_sdf/constants/{0..5}` are little-endian fp32 arrays.  Nothing in
      the archive is unpickled or executed (no torch.jit.load, no pickle).  Shapes follow the
      TorchScript graph text `nn_sdf/code/__torch__/torch/fx/graph_module/___torch_mangle_0.py`:
          mm(x, c0) + c1 -> cos -> *10 -> addmm(c2, ., c3) -> relu -> addmm(c4, ., c5)
      c0 = A (2,128), c1 = b0 (128), c2 = b1 (128), c3 = W1 stored (out,in) [nn.Linear.weight],
      c4 = b2 (1), c5 = w2 (128).  The (out,in) orientation of c3 is pinned by the known answers
      captured from the reference artefact in SURVEY.md §8c (f(0,0) = 0.2995333, ...), which this
      script re-checks before writing anything.
  tests/golden/mlp_artefact_golden.npz
      Seeded points p (fp32) with f, grad f, lam*grad f (adj1) and lam*hess f (jac_adj1) computed by
      the REFERENCE's own module `src/nlotrajectories/core/nn_architectures.py:42-72` (FourierMLP,
      imported from the reference tree; torch only) loaded with the artefact weights, derivatives by
      torch autograd — the same quantities l4casadi traces into jac_/adj1_/jac_adj1_nn_sdf.pt
      (gen/nn_sdf.cpp:57-104).  Both fp32 (as libtorch evaluates the artefact, gen/nn_sdf.cpp casts
      double->float) and fp64 columns are stored.
  tests/golden/kat_survey.json
      Known answers captured from the reference in SURVEY.md §8c (artefact MLP values at 5 points,
      Unicycle2ndOrder.dynamics, rectangle corners, approximated SDF at the corners, soft_min).

Run:  python tests/golden/make_golden.py
"""
import importlib.util
import json
import os
import sys
import zipfile

import numpy as np
import torch

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))

KNOWN = {  # SURVEY.md §8c "Known answers (captured this session)", artefact, lambda = 1
    "points": [[0, 0], [0.5, 0.5], [1, 1], [0.25, 0.75], [1.2, 0.37]],
    "f": [0.2995333, -0.1712036, 0.1847260, 0.0516005, -0.0386944],
    "grad": [[-0.969588, -0.183145], [-0.281356, -0.689222], [-0.342374, 0.844196],
             [-0.115402, -0.784186], [0.146473, 0.137436]],
    "hess": {"0": [[-6.6451, -0.6239], [-0.6239, -1.6373]],
             "1": [[4.7842, 0.2450], [0.2450, -11.2047]]},
}

KAT_NLP = {  # SURVEY.md §8c, reference code evaluated numerically, b2 config
    "unicycle_2nd_dynamics": {"x": [0.3, 0.2, 0.7, 0.5, -0.1], "u": [0.4, -0.3],
                              "f": [0.38242109, 0.32210884, -0.1, 0.4, -0.3]},
    "rect_corners": {"pose": [0.3, 0.2, 0.7], "length": 0.2, "width": 0.1,
                     "corners": [[0.25573, 0.09734], [0.19130, 0.17382],
                                 [0.34427, 0.30266], [0.40870, 0.22618]]},
    "circle_b2_approx_sdf_at_corners": {"center": [0.5, 0.5], "radius": 0.2, "margin": 0.05,
                                        "values": [0.2209646, 0.1990945, 0.0013809, 0.0386419]},
    "soft_min": {"args": [0.1, 0.3], "alpha": 10.0, "value": 0.0873072},
}


def extract_weights():
    z = zipfile.ZipFile(os.path.join(REF, "_l4c_generated", "nn_sdf.pt"))
    c = [np.frombuffer(z.read(f"nn_sdf/constants/{i}"), dtype="<f4").copy() for i in range(6)]
    w = {
        "A": c[0].reshape(2, 128),      # fourier.weights (in, out)
        "b0": c[1],                     # fourier.bias
        "W1": c[3].reshape(128, 128),   # layers[0].weight (out, in)
        "b1": c[2],                     # layers[0].bias
        "w2": c[5].reshape(1, 128),     # output_layer.weight (out=1, in)
        "b2": c[4].reshape(1),          # output_layer.bias
    }
    return w


def load_reference_fourier_mlp(w):
    path = os.path.join(REF, "src", "nlotrajectories", "core", "nn_architectures.py")
    spec = importlib.util.spec_from_file_location("ref_nn_architectures", path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    # artefact: FourierMLP(2, 128, 1, num_layers=3, scale=10) -> one hidden Linear(128,128)+ReLU
    model = mod.FourierMLP(input_dim=2, hidden_dim=128, output_dim=1, num_layers=3, scale=10.0)
    sd = {
        "fourier.weights": torch.from_numpy(w["A"]),
        "fourier.bias": torch.from_numpy(w["b0"]),
        "layers.0.weight": torch.from_numpy(w["W1"]),
        "layers.0.bias": torch.from_numpy(w["b1"]),
        "output_layer.weight": torch.from_numpy(w["w2"]),
        "output_layer.bias": torch.from_numpy(w["b2"]),
    }
    model.load_state_dict(sd)
    model.eval()
    return model


def derivs(model, pts, lam, dtype):
    m = model.to(dtype)
    p = torch.tensor(pts, dtype=dtype, requires_grad=True)
    f = m(p)[:, 0]
    (g,) = torch.autograd.grad(f.sum(), p, create_graph=True)
    H = torch.zeros(len(pts), 2, 2, dtype=dtype)
    for j in range(2):
        (hj,) = torch.autograd.grad(g[:, j].sum(), p, retain_graph=True)
        H[:, j, :] = hj
    lam_t = torch.tensor(lam, dtype=dtype)
    return (f.detach().numpy(), g.detach().numpy(), (lam_t[:, None] * g).detach().numpy(),
            (lam_t[:, None, None] * H).detach().numpy())


def main():
    if not os.path.isdir(REF):
        print("reference tree absent; nothing to do")
        return 0
    w = extract_weights()
    model = load_reference_fourier_mlp(w)
    # pin the weight layout against the survey's known answers before writing anything
    f_k, g_k, _, h_k = derivs(model, KNOWN["points"], [1.0] * 5, torch.float64)
    assert np.allclose(f_k, KNOWN["f"], atol=2e-6), f_k
    assert np.allclose(g_k, KNOWN["grad"], atol=2e-5), g_k
    assert np.allclose(h_k[0], KNOWN["hess"]["0"], atol=2e-3), h_k[0]
    assert np.allclose(h_k[1], KNOWN["hess"]["1"], atol=2e-3), h_k[1]

    data_dir = os.path.join(REPO, "nlotrajectories_amd", "data")
    os.makedirs(data_dir, exist_ok=True)
    np.savez(os.path.join(data_dir, "nn_sdf_artefact.npz"), arch=np.array("fourier"),
             scale=np.float32(10.0), **w)

    rng = np.random.default_rng(0)
    pts = np.concatenate([
        np.array(KNOWN["points"], dtype=np.float64),
        rng.uniform(-0.5, 1.5, size=(2043, 2)),      # the training box of run_benchmark.py:96
        rng.uniform(-3.0, 4.0, size=(200, 2)),       # far field
    ]).astype(np.float32)
    lam = rng.uniform(-2.0, 2.0, size=len(pts)).astype(np.float32)
    out = {"p": pts, "lam": lam}
    for name, dt in (("f32", torch.float32), ("f64", torch.float64)):
        f, g, adj, hes = derivs(model, pts.astype(np.float64 if dt == torch.float64 else np.float32),
                                lam.astype(np.float64 if dt == torch.float64 else np.float32), dt)
        out[f"f_{name}"], out[f"grad_{name}"] = f, g
        out[f"adj1_{name}"], out[f"jac_adj1_{name}"] = adj, hes
    np.savez_compressed(os.path.join(HERE, "mlp_artefact_golden.npz"), **out)
    with open(os.path.join(HERE, "kat_survey.json"), "w") as fh:
        json.dump({"mlp_artefact": KNOWN, "nlp": KAT_NLP}, fh, indent=1)
    print("wrote", len(pts), "golden MLP points")
    return 0


if __name__ == "__main__":
    sys.exit(main())
