"""Device-side entry points on torch tensors (thin wrappers over the C ABI, no CPU fallback)."""
from __future__ import annotations

import ctypes as C

import numpy as np
import torch

from . import _abi
from ._lib import check, lib, require_gpu, stream_ptr
from .nn import MlpWeights


class DeviceMlp:
    """Device-resident learned-SDF weights (NlotMlp handle).  arith: "split_bf16" (the default: three-way bf16 operand
    split, six MFMA products per fp32 product) or "f32" (v_mfma_f32 products, the reference's fp32 net); both fp32
    arithmetic, differing at the rounding level (include/nlot.h, NLOT_MLP_ARITH_*).  "seq" (ReLU nets; tests): every
    sum a sequential fp32 FMA chain in index order, the oracle's default order, one thread per point."""

    ARITH = {"split_bf16": 0, "f32": 1, "seq": 2}

    def __init__(self, weights: MlpWeights, arith: str = "split_bf16"):
        require_gpu()
        self.weights = weights
        self.arith = arith
        self._arrs = {k: np.ascontiguousarray(v, np.float32) for k, v in weights.arrays.items()}
        fp = lambda a: a.ctypes.data_as(C.POINTER(C.c_float))
        d = _abi.NlotMlpDesc(in_kind=weights.in_kind, hidden=weights.hidden, n_hidden=weights.n_hidden, act=weights.act,
                             fourier_scale=weights.fourier_scale, b_out=weights.b_out)
        d.A, d.b0, d.W, d.b, d.w_out = (fp(self._arrs[k]) for k in ("A", "b0", "W", "b", "w_out"))
        h = lib().nlot_mlp_create_ex(C.byref(d), self.ARITH[arith])
        if not h:
            raise RuntimeError("nlot_mlp_create_ex: " + lib().nlot_last_error().decode())
        self.handle = C.c_void_p(h)

    def __del__(self):
        h = getattr(self, "handle", None)
        if h:
            try:
                lib().nlot_mlp_destroy(h)
            except Exception:
                pass
            self.handle = None


def _ptr(t):
    return C.c_void_p(t.data_ptr()) if t is not None else None


def sdf_mlp_eval(mlp: DeviceMlp, pts: torch.Tensor, lam: torch.Tensor = None, derivatives: bool = True):
    """nn_sdf family on the GPU: pts [P,2] fp32 cuda -> (val [P], lam*grad [P,2], lam*hess [P,2,2]).

    With derivatives=False only the value is computed (nn_sdf); lam=None means lam = 1 (jac_nn_sdf).
    """
    assert pts.is_cuda and pts.dtype == torch.float32 and pts.dim() == 2 and pts.shape[1] == 2
    pts = pts.contiguous()
    P = pts.shape[0]
    val = torch.empty(P, device=pts.device, dtype=torch.float32)
    grad = hess = None
    if derivatives:
        grad = torch.empty(P, 2, device=pts.device, dtype=torch.float32)
        hess = torch.empty(P, 2, 2, device=pts.device, dtype=torch.float32)
    if lam is not None:
        lam = lam.to(device=pts.device, dtype=torch.float32).contiguous()
    check(lib().nlot_sdf_mlp_eval(mlp.handle, _ptr(pts), P, _ptr(val), _ptr(grad), _ptr(lam), _ptr(hess),
                                  stream_ptr()), "nlot_sdf_mlp_eval")
    return val, grad, hess
