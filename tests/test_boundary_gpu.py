"""The drop-in boundary on the GPU: the CasADi-external entry points of libnlot.so called exactly as CasADi
calls gen/nn_sdf.cpp's (arg/res/iw/w/mem, one 1x2 point per call, host doubles), and the L4CasADi /
NNObstacle wrappers with the reference's signatures, against the reference-generated golden vectors."""
import ctypes as C

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

DP = C.POINTER(C.c_double)


def _call(L, fn, args, n_out):
    """fn(arg, res, iw, w, mem) with CasADi's calling convention; returns the res buffers."""
    arrs = [np.ascontiguousarray(a, np.float64) for a in args]
    argv = (DP * len(arrs))(*[a.ctypes.data_as(DP) for a in arrs])
    outs = [np.zeros(n) for n in n_out]
    resv = (DP * len(outs))(*[o.ctypes.data_as(DP) if len(o) else None for o in outs])
    f = getattr(L, fn)
    f.restype = C.c_int
    f.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int]
    rc = f(argv, resv, None, None, 0)
    return rc, outs


def test_casadi_external_entry_points(artefact, golden):
    from nlotrajectories_amd import _lib
    from nlotrajectories_amd.ops import DeviceMlp

    L = _lib.lib()
    m = DeviceMlp(artefact)
    assert L.nlot_casadi_bind(m.handle) == 0
    for fn, n_in, n_out in (("nn_sdf", 1, 1), ("jac_nn_sdf", 2, 1), ("adj1_nn_sdf", 3, 1), ("jac_adj1_nn_sdf", 4, 3)):
        getattr(L, fn + "_n_in").restype = C.c_longlong
        getattr(L, fn + "_n_out").restype = C.c_longlong
        assert getattr(L, fn + "_n_in")() == n_in and getattr(L, fn + "_n_out")() == n_out, fn
    L.nn_sdf_sparsity_in.restype = C.POINTER(C.c_longlong)
    L.nn_sdf_sparsity_in.argtypes = [C.c_longlong]
    sp = L.nn_sdf_sparsity_in(0)
    assert (sp[0], sp[1], sp[2]) == (1, 2, 1)  # gen/nn_sdf.cpp:36 — 1 x 2 dense
    idx = np.random.default_rng(5).choice(len(golden["p"]), 48, replace=False)
    gs = max(1.0, np.abs(golden["grad_f64"]).max())
    hs = np.abs(golden["jac_adj1_f64"]).max()
    for i in idx:
        p, lam = golden["p"][i].astype(np.float64), float(golden["lam"][i])
        rc, (v,) = _call(L, "nn_sdf", [p], [1])
        assert rc == 0 and abs(v[0] - golden["f_f64"][i]) < 2e-5
        rc, (g,) = _call(L, "jac_nn_sdf", [p, v], [2])
        assert rc == 0 and np.abs(g - golden["grad_f64"][i]).max() < 5e-5 * gs
        rc, (ga,) = _call(L, "adj1_nn_sdf", [p, v, [lam]], [2])
        assert rc == 0 and np.abs(ga - golden["adj1_f64"][i]).max() < 5e-5 * gs
        rc, (h, r1, r2) = _call(L, "jac_adj1_nn_sdf", [p, v, [lam], ga], [4, 0, 0])
        assert rc == 0 and np.abs(h.reshape(2, 2) - golden["jac_adj1_f64"][i]).max() < 5e-5 * hs
    # only res[0] of jac_adj1 exists (gen/nn_sdf.cpp:93-101 throws invalid_argument; here: return 1)
    rc, _ = _call(L, "jac_adj1_nn_sdf", [golden["p"][0], [0.0], [1.0], [0.0, 0.0]], [4, 1, 0])
    assert rc == 1
    # destroying the bound model unbinds it (no use-after-free): the next call fails cleanly
    del m
    import gc

    gc.collect()
    rc, _ = _call(L, "nn_sdf", [golden["p"][0]], [1])
    assert rc == 1 and b"no model bound" in L.nlot_last_error()


def test_l4casadi_wrapper_signature(artefact, golden):
    """L4CasADi(model, device=..., name=...) on the reference FourierMLP module; NNObstacle.approximated_sdf."""
    from nlotrajectories_amd.l4casadi import L4CasADi, NNObstacle

    model = artefact.torch_module()
    l4c = L4CasADi(model, device="cpu", name="nn_sdf")
    p = torch.tensor(golden["p"][:300])
    lam = torch.tensor(golden["lam"][:300])
    f = l4c(p)
    assert f.shape == (300, 1) and f.device.type == "cpu"
    np.testing.assert_allclose(f[:, 0].numpy(), golden["f_f64"][:300], atol=2e-5)
    gs = max(1.0, np.abs(golden["grad_f64"]).max())
    np.testing.assert_allclose(l4c.jac(p).numpy(), golden["grad_f64"][:300], atol=5e-5 * gs)
    hs = np.abs(golden["jac_adj1_f64"]).max()
    for i in range(0, 300, 37):  # per-point adjoint seeds as CasADi passes them
        np.testing.assert_allclose(l4c.adj1(p[i:i + 1], lam[i]).numpy()[0], golden["adj1_f64"][i], atol=5e-5 * gs)
        np.testing.assert_allclose(l4c.jac_adj1(p[i:i + 1], lam[i]).numpy()[0], golden["jac_adj1_f64"][i],
                                   atol=5e-5 * hs)
    obs = NNObstacle(None, l4c)
    xs, ys = golden["p"][:300, 0].reshape(20, 15), golden["p"][:300, 1].reshape(20, 15)
    v = obs.approximated_sdf(xs, ys)
    assert v.shape == (20, 15)
    np.testing.assert_allclose(v.ravel(), golden["f_f64"][:300], atol=2e-5)
    # the wrapper plugs into the batched solver as the learned SDF
    from nlotrajectories_amd.problem import METRIC_PROBLEM
    from nlotrajectories_amd.solver import solve_batch

    r = solve_batch(METRIC_PROBLEM, np.array([[0, 0, 0.785, 0, 0.0]]), np.array([[1, 1, 0.785, 0, 0.0]]), mlp=obs,
                    options=__import__("nlotrajectories_amd._abi", fromlist=["x"]).gpu_options(max_iter=2))
    assert r["iters"][0].item() == 2
    with pytest.raises(ValueError):
        L4CasADi(model, generate_jac_jac=True)


def test_hess_without_grad(artefact):
    """nlot_sdf_mlp_eval with grad = NULL and hess != NULL (jac_adj1 alone) equals the full call's Hessian."""
    import ctypes as C

    from nlotrajectories_amd._lib import lib, stream_ptr
    from nlotrajectories_amd.ops import DeviceMlp, sdf_mlp_eval

    dm = DeviceMlp(artefact)
    pts = torch.tensor(np.random.default_rng(5).uniform(-0.5, 1.5, (333, 2)), dtype=torch.float32, device="cuda")
    lam = torch.linspace(-2, 2, 333, device="cuda")
    v, _, h = sdf_mlp_eval(dm, pts, lam=lam)
    val = torch.empty(333, device="cuda")
    hess = torch.full((333, 2, 2), float("nan"), device="cuda")
    p = lambda t: C.c_void_p(t.data_ptr())
    assert lib().nlot_sdf_mlp_eval(dm.handle, p(pts), 333, p(val), None, p(lam), p(hess), stream_ptr()) == 0
    torch.cuda.synchronize()
    assert torch.equal(val, v) and torch.equal(hess, h)
