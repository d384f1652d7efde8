"""Smooth-activation SDF networks (tanh / sigmoid / leaky ReLU hidden layers, SIREN's sine; the reference's
core/nn_architectures.py:8-100 and l4casadi's naive MLP, `model.activation_function` / `model.type: siren` of
run_benchmark.py:55-83).  Their Hessian has a term from every layer, so the kernel (mlp_smooth) and the oracle
carry value, gradient and Hessian forward; both are checked against torch fp64 autograd of the same module.

Tolerances (fp32 evaluation, as the reference's libtorch graph): value 2e-5 absolute (|f| <~ 2), gradient and
Hessian 2e-5 of their largest entry (5e-5 for SIREN's omega_0 = 30 scaling)."""
import numpy as np
import pytest
import torch


def _nets():
    from nlotrajectories_amd.nn import SIREN, FourierMLP, MultiLayerPerceptron

    torch.manual_seed(0)
    return {
        "fourier_tanh_2x": FourierMLP(2, 64, 1, num_layers=4, scale=2.0, activation_function="tanh"),
        "fourier_sigmoid": FourierMLP(2, 128, 1, num_layers=3, scale=3.0, activation_function="sigmoid"),
        "mlp_tanh_256x3": MultiLayerPerceptron(2, 256, 1, 3, "Tanh"),
        "mlp_sigmoid": MultiLayerPerceptron(2, 128, 1, 2, "Sigmoid"),
        "mlp_leaky": MultiLayerPerceptron(2, 64, 1, 3, "LeakyReLU"),
        "mlp_tanh_0hidden": MultiLayerPerceptron(2, 64, 1, 1, "Tanh"),
        "siren": SIREN(2, 128, 1, num_layers=3, omega_0=30),
        "siren_4": SIREN(2, 64, 1, num_layers=5, omega_0=30),
    }


def _torch_f64(w, pts):
    """value, gradient, Hessian of the restated module in fp64 (torch.func)."""
    md = w.torch_module().double().requires_grad_(False)
    P = torch.tensor(pts, dtype=torch.float64)
    f = lambda p: md(p[None])[0, 0]
    v = torch.func.vmap(f)(P).numpy()
    g = torch.func.vmap(torch.func.grad(f))(P).numpy()
    h = torch.func.vmap(torch.func.hessian(f))(P).numpy()
    return v, g, h


def _check(v, g, h, ref, tol):
    rv, rg, rh = ref
    np.testing.assert_allclose(v, rv, atol=2e-5, rtol=0)
    np.testing.assert_allclose(g, rg, atol=tol * max(np.abs(rg).max(), 1e-3), rtol=0)
    np.testing.assert_allclose(h, rh, atol=tol * max(np.abs(rh).max(), 1e-3), rtol=0)


@pytest.mark.parametrize("name", list(_nets()))
def test_weights_roundtrip(name):
    """from_module -> torch_module reproduces the module (names, activation, omega_0, layer count)."""
    from nlotrajectories_amd.nn import MlpWeights

    m = _nets()[name]
    w = MlpWeights.from_module(m)
    x = torch.rand(64, 2) * 2 - 0.5
    with torch.no_grad():
        np.testing.assert_allclose(w.torch_module()(x).numpy(), m(x).numpy(), atol=1e-6, rtol=0)


@pytest.mark.parametrize("name", list(_nets()))
def test_oracle_smooth_matches_torch_f64(name):
    import oracle as O
    from nlotrajectories_amd.nn import MlpWeights

    w = MlpWeights.from_module(_nets()[name])
    pts = np.random.default_rng(1).uniform(-0.5, 1.5, (64, 2)).astype(np.float32)
    v, g, h = O.mlp_eval(O.HostMlp(w), pts)
    _check(v, g, h.reshape(-1, 2, 2), _torch_f64(w, pts), 5e-5 if "siren" in name else 2e-5)


@pytest.mark.gpu
@pytest.mark.parametrize("name", list(_nets()))
def test_kernel_smooth_matches_oracle_and_torch(name):
    import oracle as O
    from nlotrajectories_amd.nn import MlpWeights
    from nlotrajectories_amd.ops import DeviceMlp, sdf_mlp_eval

    w = MlpWeights.from_module(_nets()[name])
    dm = DeviceMlp(w)
    rng = np.random.default_rng(2)
    for P in (1, 7, 8, 9, 1000):  # ragged tiles of 8 points
        pts = rng.uniform(-0.5, 1.5, (P, 2)).astype(np.float32)
        lam = rng.uniform(-2, 2, P).astype(np.float32)
        pt = torch.tensor(pts, device="cuda")
        v, g, h = (t.cpu().numpy() for t in sdf_mlp_eval(dm, pt))
        _, ga, ha = (t.cpu().numpy() for t in sdf_mlp_eval(dm, pt, lam=torch.tensor(lam, device="cuda")))
        vv = sdf_mlp_eval(dm, pt, derivatives=False)[0].cpu().numpy()
        np.testing.assert_array_equal(vv, v)  # the value-only launch computes the same value
        ref = _torch_f64(w, pts)
        tol = 5e-5 if "siren" in name else 2e-5
        _check(v, g, h, ref, tol)
        _check(v, ga, ha, (ref[0], lam[:, None] * ref[1], lam[:, None, None] * ref[2]), tol)
        ov, og, oh = O.mlp_eval(O.HostMlp(w), pts)
        np.testing.assert_allclose(v, ov, atol=2e-6 * max(1, np.abs(ov).max()), rtol=0)
        np.testing.assert_allclose(h[:, 0, 1], h[:, 1, 0])


@pytest.mark.gpu
@pytest.mark.parametrize("act", ["tanh", "sigmoid"])
def test_solver_iterates_smooth_sdf(artefact, act):
    """Learned-SDF solve with a smooth net (the artefact's weights under tanh / sigmoid hidden layers): the
    Newton iterates after k = 1, 3 equal the oracle's to 1e-4 (fp32 MLP on both sides)."""
    import dataclasses

    import oracle as O
    from nlotrajectories_amd import _abi
    from nlotrajectories_amd.ops import DeviceMlp
    from nlotrajectories_amd.problem import METRIC_PROBLEM
    from nlotrajectories_amd.solver import solve_batch

    w = dataclasses.replace(artefact, act={"tanh": _abi.ACT_TANH, "sigmoid": _abi.ACT_SIGMOID}[act])
    mlp, hm = DeviceMlp(w), O.HostMlp(w)
    x0, xg = [0, 0, 0.785, 0, 0], [1, 1, 0.785, 0, 0]
    for k in (1, 3):
        opt = _abi.gpu_options(max_iter=k)
        rg = solve_batch(METRIC_PROBLEM, np.array([x0]), np.array([xg]), mlp=mlp, options=opt)
        rc = O.solve_one(METRIC_PROBLEM, x0, xg, hm, opt=opt)
        assert rg["iters"][0].item() == rc["iters"]
        np.testing.assert_allclose(rg["X"][0].cpu().numpy(), rc["X"], atol=1e-4)
        np.testing.assert_allclose(rg["U"][0].cpu().numpy(), rc["U"], atol=1e-4)


# ---- reference-pinned fixtures (tests/golden/make_smooth_golden.py: the REFERENCE's FourierMLP(tanh | sigmoid |
# leaky_relu) and SIREN modules, core/nn_architectures.py:8-100, seeded, fp64 autograd) ----
REF_CASES = ["fourier_tanh", "fourier_sigmoid_2x", "fourier_leaky", "siren", "siren_w5_3x"]


def _golden_net(name):
    import os

    from nlotrajectories_amd.nn import MlpWeights

    z = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "smooth_golden.npz"))
    g = lambda k: z[f"{name}/{k}"]
    w = MlpWeights(int(g("in_kind")), int(g("hidden")), int(g("n_hidden")), float(g("fourier_scale")),
                   float(g("b_out")), {k: g(k).astype(np.float32) for k in ("A", "b0", "W", "b", "w_out")}, int(g("act")))
    return w, z["p"], (g("f"), g("grad"), g("hess"))


@pytest.mark.parametrize("name", REF_CASES)
def test_oracle_smooth_matches_reference_golden(name):
    import oracle as O

    w, pts, ref = _golden_net(name)
    v, g, h = O.mlp_eval(O.HostMlp(w), pts)
    _check(v, g, h.reshape(-1, 2, 2), ref, 5e-5 if "siren" in name else 2e-5)


@pytest.mark.gpu
@pytest.mark.parametrize("name", REF_CASES)
def test_kernel_smooth_matches_reference_golden(name):
    from nlotrajectories_amd.ops import DeviceMlp, sdf_mlp_eval

    w, pts, ref = _golden_net(name)
    v, g, h = (t.cpu().numpy() for t in sdf_mlp_eval(DeviceMlp(w), torch.tensor(pts, device="cuda:0")))
    _check(v, g, h.reshape(-1, 2, 2), ref, 5e-5 if "siren" in name else 2e-5)
