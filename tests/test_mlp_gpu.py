"""GPU parity of the batched SDF-MLP kernel (nn_sdf / jac_nn_sdf / adj1_nn_sdf / jac_adj1_nn_sdf)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", params=["split_bf16", "f32"])
def dmlp(artefact, request):
    """The artefact net with each MFMA arithmetic (include/nlot.h NLOT_MLP_ARITH_*; the parity tests run both)."""
    from nlotrajectories_amd.ops import DeviceMlp

    return DeviceMlp(artefact, request.param)


def test_mlp_matches_reference_golden(dmlp, golden):
    """Against the reference module's fp32 autograd values (tests/golden/make_golden.py)."""
    from nlotrajectories_amd.ops import sdf_mlp_eval

    p = torch.tensor(golden["p"], device="cuda")
    lam = torch.tensor(golden["lam"], device="cuda")
    v, g, h = sdf_mlp_eval(dmlp, p)
    _, ga, ha = sdf_mlp_eval(dmlp, p, lam=lam)
    v, g, h, ga, ha = (t.cpu().numpy() for t in (v, g, h, ga, ha))
    f64 = golden["f_f64"]
    # fp32 forward of a 2-128-128-1 net with |W| sums ~ 1e2: absolute tolerance 2e-5 on f (|f| <~ 2)
    np.testing.assert_allclose(v, f64, atol=2e-5, rtol=0)
    gs = np.abs(golden["grad_f64"]).max()
    np.testing.assert_allclose(g, golden["grad_f64"], atol=2e-5 * max(gs, 1), rtol=0)
    np.testing.assert_allclose(ga, golden["adj1_f64"], atol=5e-5 * max(gs, 1), rtol=0)
    hs = np.abs(golden["jac_adj1_f64"]).max()
    np.testing.assert_allclose(ha, golden["jac_adj1_f64"], atol=2e-5 * hs, rtol=0)
    np.testing.assert_allclose(h[:, 0, 1], h[:, 1, 0])


def test_mlp_matches_oracle_and_value_path(dmlp, artefact):
    import oracle as O
    from nlotrajectories_amd.ops import sdf_mlp_eval

    rng = np.random.default_rng(3)
    for P in (1, 31, 32, 33, 127, 128, 129, 4097):
        pts = rng.uniform(-0.6, 1.6, size=(P, 2)).astype(np.float32)
        lam = rng.uniform(-1, 1, size=P).astype(np.float32)
        hm = O.HostMlp(artefact)
        ov, og, oh = O.mlp_eval(hm, pts, lam)
        t = torch.tensor(pts, device="cuda")
        v, g, h = (x.cpu().numpy() for x in sdf_mlp_eval(dmlp, t, lam=torch.tensor(lam, device="cuda")))
        vv, _, _ = sdf_mlp_eval(dmlp, t, derivatives=False)
        np.testing.assert_allclose(v, ov, atol=1e-5)
        np.testing.assert_array_equal(vv.cpu().numpy(), v)  # value-only kernel == full kernel's value
        np.testing.assert_allclose(g, og, atol=5e-5 * max(1, np.abs(og).max()))
        np.testing.assert_allclose(h, oh, atol=5e-5 * max(1, np.abs(oh).max()))


def test_split_bf16_is_fp32_equivalent(dmlp, golden, artefact):
    """The 2-128-128-1 kernels run the hidden GEMM as six split-bf16 MFMA products, or as f32 MFMA
    products (NLOT_MLP_ARITH_F32).  Their error against the fp64 truth must be no larger than an fp32 evaluation's: at
    most twice the oracle's (plain fp32 FMA chain) error plus one fp32 ulp of max|f|, for f and for grad f."""
    import oracle as O
    from nlotrajectories_amd.ops import sdf_mlp_eval

    pts = np.asarray(golden["p"], dtype=np.float32)
    v, g, _ = (x.cpu().numpy().astype(np.float64) for x in sdf_mlp_eval(dmlp, torch.tensor(pts, device="cuda")))
    ov, og, _ = O.mlp_eval(O.HostMlp(artefact), pts, np.ones(len(pts), np.float32))
    f64, g64 = golden["f_f64"], golden["grad_f64"]
    fs, gs = np.abs(f64).max(), np.abs(g64).max()
    assert np.abs(v - f64).max() <= 2 * np.abs(ov - f64).max() + 1.2e-7 * fs
    assert np.abs(g - g64).max() <= 2 * np.abs(og - g64).max() + 1.2e-7 * gs


def test_relu_mlp_128_split_bf16_vs_torch():
    """ReLU input layer, H = 128, one hidden layer: the split-bf16 kernels' other input-layer branch.
    A plain bf16 GEMM would miss the value tolerance by ~100x."""
    from nlotrajectories_amd.nn import MlpWeights
    from nlotrajectories_amd.ops import DeviceMlp, sdf_mlp_eval

    w = MlpWeights.random_relu_mlp(hidden=128, n_hidden=1, seed=4)
    m = w.torch_module().double()
    pts = torch.rand(3000, 2, dtype=torch.float64) * 2 - 0.5
    pts.requires_grad_(True)
    f = m(pts)[:, 0]
    (g,) = torch.autograd.grad(f.sum(), pts)
    dm = DeviceMlp(w)
    v, gg, hh = sdf_mlp_eval(dm, pts.detach().float().cuda())
    vv, _, _ = sdf_mlp_eval(dm, pts.detach().float().cuda(), derivatives=False)
    np.testing.assert_array_equal(vv.cpu().numpy(), v.cpu().numpy())
    np.testing.assert_allclose(v.cpu().numpy(), f.detach().numpy(), atol=1e-5 * max(1, f.abs().max().item()))
    np.testing.assert_allclose(gg.cpu().numpy(), g.numpy(), atol=1e-4 * max(1, g.abs().max().item()))
    assert float(hh.abs().max()) == 0.0


def test_mlp_relu_two_layer_vs_torch():
    """l4casadi naive MLP (ReLU input layer, 2 hidden layers): value & grad vs torch fp64; hess = 0."""
    from nlotrajectories_amd.nn import MlpWeights
    from nlotrajectories_amd.ops import DeviceMlp, sdf_mlp_eval

    w = MlpWeights.random_relu_mlp(hidden=64, n_hidden=2, seed=1)
    m = w.torch_module().double()
    pts = torch.rand(1000, 2, dtype=torch.float64) * 2 - 0.5
    pts.requires_grad_(True)
    f = m(pts)[:, 0]
    (g,) = torch.autograd.grad(f.sum(), pts)
    v, gg, hh = sdf_mlp_eval(DeviceMlp(w), pts.detach().float().cuda())
    np.testing.assert_allclose(v.cpu().numpy(), f.detach().numpy(), atol=1e-4 * max(1, f.abs().max().item()))
    np.testing.assert_allclose(gg.cpu().numpy(), g.numpy(), atol=1e-4 * max(1, g.abs().max().item()))
    assert float(hh.abs().max()) == 0.0


@pytest.mark.parametrize("net", ["b6_trained", "relu_64x2", "relu_256x3"])
def test_seq_arith_bitwise_oracle(net):
    """NLOT_MLP_ARITH_SEQ (include/nlot.h, ABI v15): every sum a sequential fp32 FMA chain in index order, the oracle's
    default order (oracle/nlot_oracle.c oracle_mlp_point).  For ReLU-input nets (benchmark 6's trained 2-128-128-1 net,
    l4casadi's naive MLPs) value, lam*gradient and the value-only launch are bitwise the oracle's."""
    import os

    import oracle as O
    from nlotrajectories_amd.nn import MlpWeights
    from nlotrajectories_amd.ops import DeviceMlp, sdf_mlp_eval

    if net == "b6_trained":
        w = MlpWeights.load(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                         "nlotrajectories_amd", "data", "b6_mlp128_seed0.npz"))
    elif net == "relu_64x2":
        w = MlpWeights.random_relu_mlp(hidden=64, n_hidden=2, seed=1)
    else:
        w = MlpWeights.random_relu_mlp(hidden=256, n_hidden=3, seed=2)
    rng = np.random.default_rng(7)
    pts = rng.uniform(-0.2, 1.4, size=(5000, 2)).astype(np.float32)
    lam = rng.uniform(-2, 2, size=5000).astype(np.float32)
    dm = DeviceMlp(w, "seq")
    t = torch.tensor(pts, device="cuda")
    v, g, h = (x.cpu().numpy() for x in sdf_mlp_eval(dm, t, lam=torch.tensor(lam, device="cuda")))
    vv, _, _ = sdf_mlp_eval(dm, t, derivatives=False)
    ov, og, oh = O.mlp_eval(O.HostMlp(w), pts, lam)
    np.testing.assert_array_equal(v, ov)
    np.testing.assert_array_equal(vv.cpu().numpy(), ov)
    np.testing.assert_array_equal(g, og)
    np.testing.assert_array_equal(h, oh)


def test_seq_arith_fourier_nearly_bitwise(artefact):
    """The artefact FourierMLP through NLOT_MLP_ARITH_SEQ: the same sums as the oracle's; the input layer's cos / sin
    are the fp64 functions rounded to fp32 on both sides (device ocml vs host libm), which differ only where the two
    fp64 results straddle an fp32 rounding boundary (~2^-28 of the arguments): all but a few of 4000 points x 128 units
    bitwise, and the outputs bitwise on at least 99.9 % of the points."""
    import oracle as O
    from nlotrajectories_amd.ops import DeviceMlp, sdf_mlp_eval

    rng = np.random.default_rng(8)
    pts = rng.uniform(-0.3, 1.3, size=(4000, 2)).astype(np.float32)
    lam = rng.uniform(-2, 2, size=4000).astype(np.float32)
    v, g, h = (x.cpu().numpy() for x in sdf_mlp_eval(DeviceMlp(artefact, "seq"), torch.tensor(pts, device="cuda"),
                                                    lam=torch.tensor(lam, device="cuda")))
    ov, og, oh = O.mlp_eval(O.HostMlp(artefact), pts, lam)
    same = float(((v == ov) & (g == og).all(1) & (h == oh).all((1, 2))).mean())
    print(f"[seq] Fourier net: {same:.4f} of the points bitwise equal (value, gradient, Hessian), max |dv| "
          f"{np.abs(v - ov).max():.2e}", flush=True)
    assert same >= 0.999
    np.testing.assert_allclose(v, ov, atol=2e-6)
    np.testing.assert_allclose(g, og, atol=2e-5 * max(1, np.abs(og).max()))
