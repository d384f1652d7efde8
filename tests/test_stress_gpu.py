"""The stress configuration on the GPU (BASELINE.json configs[4]): the 2-256x4-1 ReLU SDF MLP (three 256x256
HxH layers, seeded kaiming-uniform as core/sdf/l4casadi.py:69-74) through the layer-streaming MFMA kernel,
against torch fp64; a deeper Fourier net on the same kernel; and the solver at N = 256 knots with that MLP
as the learned SDF, against the oracle."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _torch64(w):
    m = w.torch_module().double()
    return m


def _check_vs_torch(w, P=3000, seed=0):
    from nlotrajectories_amd.ops import DeviceMlp, sdf_mlp_eval

    rng = np.random.default_rng(seed)
    pts = rng.uniform(-0.5, 1.5, size=(P, 2)).astype(np.float32)
    lam = rng.uniform(-1, 1, size=P).astype(np.float32)
    d = DeviceMlp(w)
    t = torch.tensor(pts, device="cuda")
    v, g, h = (x.cpu().numpy() for x in sdf_mlp_eval(d, t, lam=torch.tensor(lam, device="cuda")))
    vv, _, _ = sdf_mlp_eval(d, t, derivatives=False)
    m = _torch64(w)
    x = torch.tensor(pts, dtype=torch.float64, requires_grad=True)
    f = m(x)[:, 0]
    (gr,) = torch.autograd.grad(f, x, grad_outputs=torch.tensor(lam, dtype=torch.float64), create_graph=True)
    hs = [torch.autograd.grad(gr[:, a].sum(), x, retain_graph=True)[0] for a in range(2)]
    H = torch.stack(hs, 1).detach().numpy()
    f64, g64 = f.detach().numpy(), gr.detach().numpy()
    fs, gs = max(1.0, np.abs(f64).max()), max(1.0, np.abs(g64).max())
    print(w.hidden, w.n_hidden, "max |f| err", np.abs(v - f64).max(), "max |grad| err", np.abs(g - g64).max(),
          "max |H| err", np.abs(h - H).max())
    # fp32 chain through 4 layers of width 256: absolute error relative to max |f| / |grad|
    assert np.abs(v - f64).max() <= 2e-5 * fs
    assert np.abs(g - g64).max() <= 1e-4 * gs
    assert np.abs(h - H).max() <= 1e-4 * max(1.0, np.abs(H).max())
    np.testing.assert_array_equal(vv.cpu().numpy(), v)  # value-only launch == full launch's value


def test_stress_mlp_256x4_vs_torch():
    from nlotrajectories_amd.nn import MlpWeights

    _check_vs_torch(MlpWeights.stress_sdf_mlp(seed=0))


def test_stream_kernel_fourier_three_layers_vs_torch():
    from nlotrajectories_amd import _abi
    from nlotrajectories_amd.nn import FourierMLP, MlpWeights

    torch.manual_seed(3)
    m = FourierMLP(2, 128, 1, num_layers=5, scale=2.0)  # 3 HxH layers: beyond the LDS-resident kernels
    w = MlpWeights.from_module(m)
    assert w.in_kind == _abi.MLP_IN_FOURIER and w.n_hidden == 3
    _check_vs_torch(w, seed=1)


def test_stress_solver_N256_iterates_match_oracle():
    """N = 256 knots (5 passes of a wavefront over the knots) with the stress MLP as the learned SDF:
    GPU iterates equal the oracle's after 1 and 3 iterations (fp32 MLP on both sides: 1e-4)."""
    import oracle as O
    from nlotrajectories_amd import _abi
    from nlotrajectories_amd.nn import MlpWeights
    from nlotrajectories_amd.ops import DeviceMlp
    from nlotrajectories_amd.problem import STRESS_PROBLEM
    from nlotrajectories_amd.solver import solve_batch

    w = MlpWeights.stress_sdf_mlp(seed=0)
    mlp, hm = DeviceMlp(w), O.HostMlp(w)
    from nlotrajectories_amd.sampling import sample_start_goal

    sdf = lambda P: O.mlp_eval(hm, P, want=False)[0]
    x0, xg = sample_start_goal(STRESS_PROBLEM, 2, seed=0, sdf=sdf)
    for k in (1, 3):
        opt = _abi.gpu_options(max_iter=k)
        rg = solve_batch(STRESS_PROBLEM, x0, xg, mlp=mlp, options=opt)
        for b in range(2):
            rc = O.solve_one(STRESS_PROBLEM, x0[b], xg[b], hm, opt=opt)
            assert rg["status"][b].item() == rc["status"]
            np.testing.assert_allclose(rg["X"][b].cpu().numpy(), rc["X"], atol=1e-4)
            np.testing.assert_allclose(rg["U"][b].cpu().numpy(), rc["U"], atol=1e-4)
