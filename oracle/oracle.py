"""ctypes front-end of the CPU oracle (liboracle_nlot.so).  TEST INFRASTRUCTURE ONLY.

Imported only by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg.  The product
package never imports this module.  See nlot_oracle.c for what is restated from where.
"""
import ctypes as C
import os
import subprocess

import numpy as np

from nlotrajectories_amd import _abi

HERE = os.path.dirname(os.path.abspath(__file__))
# NLOT_ORACLE_LIB=liboracle_nlot_fma.so: the FMA-contracted build (oracle/Makefile; fixture generation only)
LIB_PATH = os.path.join(HERE, os.environ.get("NLOT_ORACLE_LIB", "liboracle_nlot.so"))


def build(force: bool = False) -> str:
    srcs = [os.path.join(HERE, "nlot_oracle.c"), os.path.join(HERE, "..", "include", "nlot.h")]
    if force or not os.path.exists(LIB_PATH) or any(os.path.getmtime(LIB_PATH) < os.path.getmtime(s) for s in srcs) \
            or not os.path.exists(os.path.join(HERE, "liboracle_nlot_fma.so")):
        subprocess.run(["make", "-C", HERE, "-s"], check=True)
    return LIB_PATH


_lib = None


def lib():
    global _lib
    if _lib is None:
        build()
        L = C.CDLL(LIB_PATH)
        dp, fp, ip = C.POINTER(C.c_double), C.POINTER(C.c_float), C.POINTER(C.c_int)
        L.oracle_mlp_eval.argtypes = [C.POINTER(_abi.NlotMlpDesc), fp, C.c_long, fp, fp, fp, fp]
        L.oracle_sdf_eval.argtypes = [C.POINTER(_abi.NlotProblem), C.POINTER(_abi.NlotMlpDesc), dp, C.c_long, dp]
        L.oracle_soft_min.argtypes = [dp, C.c_int, C.c_double]
        L.oracle_soft_min.restype = C.c_double
        L.oracle_dynamics.argtypes = [C.POINTER(_abi.NlotProblem), dp, dp, dp]
        L.oracle_corners.argtypes = [C.POINTER(_abi.NlotProblem), dp, dp]
        L.oracle_knot_constraints.argtypes = [C.POINTER(_abi.NlotProblem), C.POINTER(_abi.NlotMlpDesc), dp,
                                              C.c_double, dp, dp]
        L.oracle_solve_one.argtypes = [C.POINTER(_abi.NlotProblem), C.POINTER(_abi.NlotSolverOptions),
                                       C.POINTER(_abi.NlotMlpDesc), dp, dp, dp, dp, dp, dp, dp, ip, dp]
        L.oracle_solve_warm.argtypes = [C.POINTER(_abi.NlotProblem), C.POINTER(_abi.NlotSolverOptions),
                                         C.POINTER(_abi.NlotMlpDesc), dp, dp, dp, dp, dp, dp, dp, dp, dp, ip, dp]
        L.oracle_solve_trace.argtypes = [C.POINTER(_abi.NlotProblem), C.POINTER(_abi.NlotSolverOptions),
                                         C.POINTER(_abi.NlotMlpDesc), dp, dp, dp, dp, dp, dp, dp, ip, dp, dp, C.c_int]
        L.oracle_solve_batch.argtypes = [C.POINTER(_abi.NlotProblem), C.POINTER(_abi.NlotSolverOptions),
                                         C.POINTER(_abi.NlotMlpDesc), dp, dp, dp, dp, dp, dp, dp, ip, ip,
                                         C.c_long, C.c_int]
        for n in ("oracle_sizeof_problem", "oracle_sizeof_options", "oracle_sizeof_mlpdesc", "oracle_sizeof_stats"):
            getattr(L, n).restype = C.c_int
        assert L.oracle_sizeof_problem() == C.sizeof(_abi.NlotProblem)
        assert L.oracle_sizeof_options() == C.sizeof(_abi.NlotSolverOptions)
        assert L.oracle_sizeof_mlpdesc() == C.sizeof(_abi.NlotMlpDesc)
        _lib = L
    return _lib


def _dp(a):
    return a.ctypes.data_as(C.POINTER(C.c_double)) if a is not None else None


def _fp(a):
    return a.ctypes.data_as(C.POINTER(C.c_float)) if a is not None else None


class HostMlp:
    """Host copy of the MLP weights in NlotMlpDesc form (arrays kept alive)."""

    def __init__(self, w):
        self.w = {k: np.ascontiguousarray(v, dtype=np.float32) for k, v in w.arrays.items()}
        d = _abi.NlotMlpDesc()
        d.in_kind, d.hidden, d.n_hidden, d.act = w.in_kind, w.hidden, w.n_hidden, getattr(w, "act", 0)
        d.fourier_scale, d.b_out = w.fourier_scale, w.b_out
        d.A, d.b0 = _fp(self.w["A"]), _fp(self.w["b0"])
        d.W, d.b = _fp(self.w["W"]), _fp(self.w["b"])
        d.w_out = _fp(self.w["w_out"])
        self.desc = d


def mlp_eval(hm: HostMlp, pts, lam=None, want=True):
    pts = np.ascontiguousarray(pts, dtype=np.float32)
    P = len(pts)
    val = np.zeros(P, np.float32)
    grad = np.zeros((P, 2), np.float32) if want else None
    hess = np.zeros((P, 2, 2), np.float32) if want else None
    lam_a = None if lam is None else np.ascontiguousarray(lam, dtype=np.float32)
    lib().oracle_mlp_eval(C.byref(hm.desc), _fp(pts), P, _fp(val), _fp(grad), _fp(lam_a), _fp(hess))
    return val, grad, hess


def sdf_eval(problem, pts, hm: HostMlp = None):
    pc = problem.to_c()
    pts = np.ascontiguousarray(pts, dtype=np.float64)
    out = np.zeros((len(pts), 6))
    lib().oracle_sdf_eval(C.byref(pc), C.byref(hm.desc) if hm else None, _dp(pts), len(pts), _dp(out))
    return out


def soft_min(vals, alpha=10.0):
    v = np.ascontiguousarray(vals, dtype=np.float64)
    return lib().oracle_soft_min(_dp(v), len(v), alpha)


def dyn_map(problem, x, u):
    """(F, A, B) of the defect map x_{k+1} = F(x_k, u_k): Euler or, with problem.integrator 'rk4', RK4."""
    pc = problem.to_c()
    nx, nu = problem.nx, problem.nu
    F, A, B = np.zeros(nx), np.zeros((nx, nx)), np.zeros((nx, nu))
    lib().oracle_dyn_map(C.byref(pc), _dp(np.ascontiguousarray(x, np.float64)), _dp(np.ascontiguousarray(u, np.float64)),
                         _dp(F), _dp(A), _dp(B))
    return F, A, B


def dynamics(problem, x, u):
    pc = problem.to_c()
    x = np.ascontiguousarray(x, np.float64)
    u = np.ascontiguousarray(u, np.float64)
    f = np.zeros(problem.nx)
    lib().oracle_dynamics(C.byref(pc), _dp(x), _dp(u), _dp(f))
    return f


def corners(problem, pose):
    pc = problem.to_c()
    pose = np.ascontiguousarray(pose, np.float64)
    out = np.zeros((len(problem.body), 2))
    lib().oracle_corners(C.byref(pc), _dp(pose), _dp(out))
    return out


def knot_constraints(problem, xk, sk=0.0, hm: HostMlp = None):
    pc = problem.to_c()
    xk = np.ascontiguousarray(xk, np.float64)
    d = np.zeros(8)
    g = np.zeros((8, 3))
    m = lib().oracle_knot_constraints(C.byref(pc), C.byref(hm.desc) if hm else None, _dp(xk), sk, _dp(d), _dp(g))
    return d[:m], g[:m]


# oracle/nlot_oracle.c TERM_*: how a run ended (info[14])
TERM_NAMES = ("solved", "max_iter", "max_iter_in_restoration", "restoration_line_search_failed",
              "restoration_converged_feasible_rejected_by_filter", "restoration_converged_infeasible",
              "almost_feasible_at_restoration_entry", "numeric", "tiny_step", "line_search_failed")


def solve_one(problem, x0, xg, hm: HostMlp = None, opt=None, X_init=None, U_init=None, S_init=None):
    pc = problem.to_c()
    opt = opt or _abi.default_options()
    N, nx, nu = problem.N, problem.nx, problem.nu
    X = np.zeros((N + 1, nx))
    U = np.zeros((N, nu))
    S = np.zeros(N + 1)
    cost = np.zeros(1)
    it = (C.c_int * 1)()
    info = np.zeros(16)
    x0 = np.ascontiguousarray(x0, np.float64)
    xg = np.ascontiguousarray(xg, np.float64)
    Xi = None if X_init is None else np.ascontiguousarray(X_init, np.float64)
    Ui = None if U_init is None else np.ascontiguousarray(U_init, np.float64)
    Si = None if S_init is None else np.ascontiguousarray(S_init, np.float64)
    st = lib().oracle_solve_warm(C.byref(pc), C.byref(opt), C.byref(hm.desc) if hm else None, _dp(x0), _dp(xg),
                                 _dp(Xi), _dp(Ui), _dp(Si), _dp(X), _dp(U), _dp(S), _dp(cost), it, _dp(info))
    ev = int(info[7])
    return dict(status=st, X=X, U=U, S=S, cost=float(cost[0]), iters=int(it[0]), dual_inf=info[1],
                constr_viol=info[2], lin_resid=info[3], mu=info[4], E0=info[5], resto_phases=int(info[6]),
                watchdogs=ev // 1000000, soft_resto_steps=(ev // 10000) % 100, soc_tried=(ev // 100) % 100,
                tiny_steps=ev % 100, theta_fail=float(info[8]), max_filter=int(info[9]),
                max_mu_filter=int(info[10]), filter_forgotten=int(info[11]), mu_filter_forgotten=int(info[12]),
                trials=int(info[13]), term=TERM_NAMES[int(info[14])])


def solve_trace(problem, x0, xg, hm: HostMlp = None, opt=None, X_init=None, cap=201):
    """solve_one plus the iterate (X, U) at the top of every iteration it < cap: trace[it] = the point a run with
    max_iter = it returns; rows past the final iteration stay NaN."""
    pc = problem.to_c()
    opt = opt or _abi.default_options()
    N, nx, nu = problem.N, problem.nx, problem.nu
    X, U, S = np.zeros((N + 1, nx)), np.zeros((N, nu)), np.zeros(N + 1)
    cost, info = np.zeros(1), np.zeros(16)
    it = (C.c_int * 1)()
    tr = np.full((cap, (N + 1) * nx + N * nu), np.nan)
    x0 = np.ascontiguousarray(x0, np.float64)
    xg = np.ascontiguousarray(xg, np.float64)
    Xi = None if X_init is None else np.ascontiguousarray(X_init, np.float64)
    st = lib().oracle_solve_trace(C.byref(pc), C.byref(opt), C.byref(hm.desc) if hm else None, _dp(x0), _dp(xg),
                                  _dp(Xi), _dp(X), _dp(U), _dp(S), _dp(cost), it, _dp(info), _dp(tr), cap)
    return dict(status=st, X=X, U=U, S=S, cost=float(cost[0]), iters=int(it[0]), trace=tr, trials=int(info[13]),
                resto_phases=int(info[6]))


def solve_batch(problem, x0, xg, hm: HostMlp = None, opt=None, threads=0):
    pc = problem.to_c()
    opt = opt or _abi.default_options()
    B = len(x0)
    N, nx, nu = problem.N, problem.nx, problem.nu
    X = np.zeros((B, N + 1, nx))
    U = np.zeros((B, N, nu))
    S = np.zeros((B, N + 1))
    cost = np.zeros(B)
    status = np.zeros(B, np.int32)
    iters = np.zeros(B, np.int32)
    x0 = np.ascontiguousarray(x0, np.float64)
    xg = np.ascontiguousarray(xg, np.float64)
    ip = C.POINTER(C.c_int)
    lib().oracle_solve_batch(C.byref(pc), C.byref(opt), C.byref(hm.desc) if hm else None, _dp(x0), _dp(xg), None,
                             _dp(X), _dp(U), _dp(S), _dp(cost), status.ctypes.data_as(ip),
                             iters.ctypes.data_as(ip), B, threads)
    return dict(status=status, X=X, U=U, S=S, cost=cost, iters=iters)
