// Batched trajectory optimisation on the GPU: B independent instances of the NLP of
// RunBenchmark.run (/root/reference/src/nlotrajectories/core/runner.py:44-108), solved with a
// restatement of IPOPT's primal-dual filter line-search algorithm (runner.py:113-133)
// whose Newton systems are solved by a stage-wise Riccati recursion.
//
// Layout: every per-instance array is structure-of-arrays with the instance index fastest
// (element i of instance b at [i * cap + b]), so the one-thread-per-instance kernels below read and
// write whole 256/512-byte lines per wave.  The learned-SDF points of all active instances are
// compacted into one list per global step and evaluated by the MFMA kernel (nlot_mlp.hip).
//
// Per-instance phase machine (one global step = one launch of each kernel):
//   INIT -> [corners, MLP full, k_iterate: slack push, least-squares multipliers, then EVAL work]
//   EVAL -> [corners, MLP full, k_iterate: evaluate, converge?, mu update, inertia-corrected
//            Newton step, step bounds]                                              -> LS
//   LS   -> [trial corners, MLP value, k_accept: filter test at alpha; accept -> EVAL,
//            reject -> alpha/2 (next step), alpha < alpha_min -> DONE(LS_FAILED)]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <vector>

#include "nlot_device.h"
#include "nlot_internal.h"

namespace nlot {

enum Phase { PH_INIT = 0, PH_EVAL = 1, PH_LS = 2, PH_DONE = 3 };
enum Scal {
    SC_MU, SC_TAU, SC_DWLAST, SC_THMAX, SC_THMIN, SC_ALPHA, SC_AMAX, SC_AMIN, SC_AZ, SC_THETA, SC_PHI, SC_GD,
    SC_DW, SC_DC, SC_STATUS, SC_ITERS, SC_PHASE, SC_TRIALS, SC_NFILT, SC_RANK, SC_E0, SC_COUNT
};
constexpr int FILT_MAX = 64;
constexpr int MMAX = 4;  // inequalities per knot (rectangle without slack)

struct Ws {
    double *X, *U, *S, *T, *yi, *yk, *yt, *yd, *zl, *zu, *zs, *vt;
    double *dv, *Jd, *Hd, *rci, *rcd, *rct, *rcq;
    double *Kf, *kf, *Kn, *Pm, *pv, *Gm;
    double *dX, *dU, *dS, *dT, *yi_n, *yk_n, *yt_n, *yd_n, *dzl, *dzu, *dzs, *dvt;
    double *sc, *filt;
    float* pts;  // [P_per][cap][2]
    float* mo;   // [6][P_per][cap]
    int* cnt;    // [0] eval points count, [1] trial count, [2] not-done count
    int64_t cap;
};

struct Dims {
    int N, nx, nu, ns, M, nc, nb, nv, sd;  // nv = nu + ns (stage k < N)
    int tidx[8];
    int ppk;  // SDF points per knot (corners, or 1 for a dot)
};

static Dims make_dims(const NlotProblem& p) {
    Dims d{};
    d.N = p.N;
    d.nx = p.nx;
    d.nu = p.nu;
    d.ns = p.use_slack ? 1 : 0;
    d.nb = p.shape == NLOT_SHAPE_DOT ? 1 : p.n_body;
    d.M = p.shape == NLOT_SHAPE_DOT ? 1 : (p.use_slack ? 1 : p.n_body);
    d.sd = (p.shape == NLOT_SHAPE_POLYGON && p.use_slack) ? 1 : 0;
    d.nv = p.nu + d.ns;
    d.nc = 0;
    for (int i = 0; i < p.nx; ++i)
        if (p.enforce_heading || i != 2) d.tidx[d.nc++] = i;
    d.ppk = d.nb;
    return d;
}

// workspace carving (host and device agree on the order)
#define NLOT_WS_ARRAYS(X_)                                                                             \
    X_(X, (N + 1) * nx) X_(U, N * nu) X_(S, N + 1) X_(T, (N + 1) * M) X_(yi, nx) X_(yk, N * nx) X_(yt, nc) \
    X_(yd, (N + 1) * M) X_(zl, N * nu) X_(zu, N * nu) X_(zs, N + 1) X_(vt, (N + 1) * M)                \
    X_(dv, (N + 1) * M) X_(Jd, (N + 1) * M * 3) X_(Hd, (N + 1) * 6) X_(rci, nx) X_(rcd, N * nx)         \
    X_(rct, nc) X_(rcq, (N + 1) * M) X_(Kf, (N + 1) * nv * nx) X_(kf, (N + 1) * nv)                     \
    X_(Kn, (N + 1) * nv * nc) X_(Pm, (N + 1) * nx * nx) X_(pv, (N + 1) * nx) X_(Gm, (N + 1) * nx * nc) \
    X_(dX, (N + 1) * nx) X_(dU, N * nu) X_(dS, N + 1) X_(dT, (N + 1) * M) X_(yi_n, nx) X_(yk_n, N * nx) \
    X_(yt_n, nc) X_(yd_n, (N + 1) * M) X_(dzl, N * nu) X_(dzu, N * nu) X_(dzs, N + 1)                  \
    X_(dvt, (N + 1) * M) X_(sc, SC_COUNT) X_(filt, 2 * FILT_MAX)

static size_t ws_doubles_per_instance(const Dims& d) {
    const int N = d.N, nx = d.nx, nu = d.nu, M = d.M, nc = d.nc, nv = d.nv;
    size_t n = 0;
#define NLOT_CNT(name, cnt) n += (size_t)(cnt);
    NLOT_WS_ARRAYS(NLOT_CNT)
#undef NLOT_CNT
    return n;
}

static size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

static size_t ws_bytes(const Dims& d, int64_t B, bool mlp) {
    size_t b = align256(ws_doubles_per_instance(d) * (size_t)B * sizeof(double));
    if (mlp) {
        const size_t P = (size_t)d.ppk * (d.N + 1);
        b += align256(P * (size_t)B * 2 * sizeof(float));
        b += align256(6 * P * (size_t)B * sizeof(float));
    }
    b += 256;  // counters
    return b;
}

static Ws carve(const Dims& d, int64_t B, bool mlp, void* base) {
    Ws w{};
    w.cap = B;
    const int N = d.N, nx = d.nx, nu = d.nu, M = d.M, nc = d.nc, nv = d.nv;
    double* q = (double*)base;
#define NLOT_TAKE(name, cnt)   \
    w.name = q;                \
    q += (size_t)(cnt) * (size_t)B;
    NLOT_WS_ARRAYS(NLOT_TAKE)
#undef NLOT_TAKE
    char* c = (char*)base + align256(ws_doubles_per_instance(d) * (size_t)B * sizeof(double));
    if (mlp) {
        const size_t P = (size_t)d.ppk * (N + 1);
        w.pts = (float*)c;
        c += align256(P * (size_t)B * 2 * sizeof(float));
        w.mo = (float*)c;
        c += align256(6 * P * (size_t)B * sizeof(float));
    }
    w.cnt = (int*)c;
    return w;
}

#define AT(arr, i) (ws.arr[(size_t)(i) * ws.cap + b])
#define SC(i) (ws.sc[(size_t)(i) * ws.cap + b])

// ---------------------------------------------------------------------------------------------
// per-corner SDF: learned (MLP output of this step's compacted list) or analytic
// ---------------------------------------------------------------------------------------------
__device__ inline HD corner_sdf(const NlotProblem& p, const Ws& ws, int rank, int cntv, int pidx, double cx,
                                double cy) {
    if (p.sdf_kind == NLOT_SDF_ANALYTIC) return sdf_scene(p, cx, cy, true);
    const size_t P = 0;  // unused
    (void)P;
    // MLP outputs: [q][pidx * cap + rank]
    const int64_t stride = (int64_t)ws.cap;
    const int64_t plane = (int64_t)((p.shape == NLOT_SHAPE_DOT ? 1 : p.n_body) * (p.N + 1)) * stride;
    const int64_t o = (int64_t)pidx * stride + rank;
    (void)cntv;
    HD h;
    h.v = ws.mo[o];
    h.gx = ws.mo[plane + o];
    h.gy = ws.mo[2 * plane + o];
    h.hxx = ws.mo[3 * plane + o];
    h.hxy = ws.mo[4 * plane + o];
    h.hyy = ws.mo[5 * plane + o];
    return h;
}

// Inequality functions at a knot (geometry.py:63-67, 107-117; utils.py:18-33): values d[j]
// (slack excluded), pose gradients g[j][3], and Hw = sum_j w[j] d2 d_j / dpose2 (if w != null).
__device__ inline void knot_eval(const NlotProblem& p, const Dims& dm, const Ws& ws, int rank, int k,
                                 const double* xk, double* d, double (*g)[3], const double* w, double* Hw) {
    const double x = xk[0], y = xk[1];
    if (p.shape == NLOT_SHAPE_DOT) {
        HD f = corner_sdf(p, ws, rank, 0, k, x, y);
        d[0] = f.v;
        if (g) { g[0][0] = f.gx; g[0][1] = f.gy; g[0][2] = 0; }
        if (Hw) {
            Hw[0] = w[0] * f.hxx; Hw[1] = w[0] * f.hxy; Hw[2] = 0;
            Hw[3] = w[0] * f.hyy; Hw[4] = 0; Hw[5] = 0;
        }
        return;
    }
    double sn, cs;
    sincos(xk[2], &sn, &cs);
    double phi[MMAX], gp[MMAX][3], Hp[MMAX][6];  // Hp: xx xy xt yy yt tt
    for (int i = 0; i < dm.nb; ++i) {
        const double bx = p.body[i][0], by = p.body[i][1];
        const double cx = x + cs * bx - sn * by, cy = y + sn * bx + cs * by;  // geometry.py:78-83
        const double ex = -(cy - y), ey = cx - x;                            // d c / d theta
        HD f = corner_sdf(p, ws, rank, 0, k * dm.nb + i, cx, cy);
        phi[i] = f.v;
        gp[i][0] = f.gx;
        gp[i][1] = f.gy;
        gp[i][2] = f.gx * ex + f.gy * ey;
        Hp[i][0] = f.hxx;
        Hp[i][1] = f.hxy;
        Hp[i][2] = f.hxx * ex + f.hxy * ey;
        Hp[i][3] = f.hyy;
        Hp[i][4] = f.hxy * ex + f.hyy * ey;
        Hp[i][5] = ex * (f.hxx * ex + f.hxy * ey) + ey * (f.hxy * ex + f.hyy * ey) - f.gx * (cx - x) - f.gy * (cy - y);
    }
    if (p.use_slack) {  // soft_min over corners (not max-shifted, as utils.py:30-31)
        const double al = p.softmin_alpha;
        double e[MMAX], sum = 0;
        for (int i = 0; i < dm.nb; ++i) {
            e[i] = exp(-al * phi[i]);
            sum += e[i];
        }
        d[0] = -log(sum) / al;
        double gd[3] = {0, 0, 0};
        for (int i = 0; i < dm.nb; ++i)
            for (int a = 0; a < 3; ++a) gd[a] += (e[i] / sum) * gp[i][a];
        if (g)
            for (int a = 0; a < 3; ++a) g[0][a] = gd[a];
        if (Hw) {
            double H[6] = {0, 0, 0, 0, 0, 0};
            const int ia[6] = {0, 0, 0, 1, 1, 2}, ib[6] = {0, 1, 2, 1, 2, 2};
            for (int i = 0; i < dm.nb; ++i) {
                const double wi = e[i] / sum;
                for (int q = 0; q < 6; ++q) H[q] += wi * (Hp[i][q] - al * gp[i][ia[q]] * gp[i][ib[q]]);
            }
            for (int q = 0; q < 6; ++q) Hw[q] = w[0] * (H[q] + al * gd[ia[q]] * gd[ib[q]]);
        }
    } else {
        for (int i = 0; i < dm.nb; ++i) {
            d[i] = phi[i];
            if (g)
                for (int a = 0; a < 3; ++a) g[i][a] = gp[i][a];
        }
        if (Hw) {
            for (int q = 0; q < 6; ++q) Hw[q] = 0;
            for (int i = 0; i < dm.nb; ++i)
                for (int q = 0; q < 6; ++q) Hw[q] += w[i] * Hp[i][q];
        }
    }
}

// objective value (runner.py:80-96)
__device__ inline double objective(const NlotProblem& p, const Dims& dm, const Ws& ws, int b, const double* dXs,
                                   const double* dUs, const double* dSs, double al) {
    (void)dXs; (void)dUs; (void)dSs;
    const int nx = dm.nx, nu = dm.nu, N = dm.N;
    double f = 0;
    for (int k = 0; k < N; ++k) {
        const double dx = (AT(X, (k + 1) * nx) + al * AT(dX, (k + 1) * nx)) - (AT(X, k * nx) + al * AT(dX, k * nx));
        const double dy = (AT(X, (k + 1) * nx + 1) + al * AT(dX, (k + 1) * nx + 1)) -
                          (AT(X, k * nx + 1) + al * AT(dX, k * nx + 1));
        f += sqrt(dx * dx + dy * dy + p.path_eps);
    }
    if (p.use_slack) {
        double q = 0;
        for (int k = 0; k <= N; ++k) {
            const double s = AT(S, k) + al * AT(dS, k);
            q += s * s;
        }
        f += p.slack_penalty * q;
    }
    if (p.use_smooth) {
        double q = 0;
        for (int k = 0; k < N - 1; ++k)
            for (int i = 0; i < nu; ++i) {
                const double u = AT(U, k * nu + i) + al * AT(dU, k * nu + i);
                q += u * u;
            }
        f += p.smooth_weight * q;
    }
    return f;
}

// ---------------------------------------------------------------------------------------------
// Stage-wise Newton system and its Riccati solve
// ---------------------------------------------------------------------------------------------
enum { MODE_NEWTON = 0, MODE_LSQ = 1 };

template <int DYN>
struct Solver {
    using D = Dyn<DYN>;
    static constexpr int NX = D::NX, NU = D::NU, NV = NU + 1, NZ = NX + NV, NC = NX;

    // Condensed stage matrix H (nz x nz) and gradient g (nz) of stage k.
    __device__ static void stage(const NlotProblem& p, const Dims& dm, const Ws& ws, int b, int k, int mode,
                                 double dw, double (*H)[NZ], double* g) {
        const int N = dm.N, nu = NU, M = dm.M;
        const int nvk = (k < N ? nu : 0) + dm.ns, nz = NX + nvk, iu = NX, is = NX + (k < N ? nu : 0);
        const double mu = SC(SC_MU), kappa_d = 1e-5;
#pragma unroll
        for (int i = 0; i < NZ; ++i) {
            g[i] = 0;
#pragma unroll
            for (int j = 0; j < NZ; ++j) H[i][j] = 0;
        }
        double x[NX];
#pragma unroll
        for (int i = 0; i < NX; ++i) x[i] = AT(X, k * NX + i);
        // objective gradient and (Newton) Hessian of the path-length terms
        for (int seg = k - 1; seg <= k; ++seg) {
            if (seg < 0 || seg >= N) continue;
            const double dx = AT(X, (seg + 1) * NX) - AT(X, seg * NX);
            const double dy = AT(X, (seg + 1) * NX + 1) - AT(X, seg * NX + 1);
            const double r2 = dx * dx + dy * dy + p.path_eps, r = sqrt(r2), r3 = r2 * r;
            const double sgn = seg == k ? -1.0 : 1.0;
            g[0] += sgn * dx / r;
            g[1] += sgn * dy / r;
            if (mode == MODE_NEWTON) {
                H[0][0] += (r2 - dx * dx) / r3;
                H[0][1] += -dx * dy / r3;
                H[1][0] += -dx * dy / r3;
                H[1][1] += (r2 - dy * dy) / r3;
            }
        }
        if (p.use_slack) g[is] += 2.0 * p.slack_penalty * AT(S, k);
        if (p.use_smooth && k < N - 1)
#pragma unroll
            for (int i = 0; i < NU; ++i) g[iu + i] += 2.0 * p.smooth_weight * AT(U, k * NU + i);
        if (mode == MODE_NEWTON) {
            if (p.use_slack) H[is][is] += 2.0 * p.slack_penalty;
            if (p.use_smooth && k < N - 1)
#pragma unroll
                for (int i = 0; i < NU; ++i) H[iu + i][iu + i] += 2.0 * p.smooth_weight;
            if (k < N) {  // dynamics c_k = x_{k+1} - F_k  =>  W -= sum_i y_i d2F_i
                double u[NU], l[NX], Hz[NX + NU][NX + NU];
#pragma unroll
                for (int i = 0; i < NU; ++i) u[i] = AT(U, k * NU + i);
#pragma unroll
                for (int i = 0; i < NX; ++i) l[i] = AT(yk, k * NX + i);
#pragma unroll
                for (int i = 0; i < NX + NU; ++i)
#pragma unroll
                    for (int j = 0; j < NX + NU; ++j) Hz[i][j] = 0;
                D::hess(x, u, l, p.dt, p.wheelbase, Hz);
#pragma unroll
                for (int i = 0; i < NX + NU; ++i)
#pragma unroll
                    for (int j = 0; j < NX + NU; ++j) H[i][j] -= Hz[i][j];
            }
            // knot inequality curvature sum_j yd_j d2 d_j (pose block x, y, theta)
            {
                const int ia[6] = {0, 0, 0, 1, 1, 2}, ib[6] = {0, 1, 2, 1, 2, 2};
#pragma unroll
                for (int q = 0; q < 6; ++q) {
                    if (ia[q] >= NX || ib[q] >= NX) continue;
                    const double v = AT(Hd, k * 6 + q);
                    H[ia[q]][ib[q]] += v;
                    if (ia[q] != ib[q]) H[ib[q]][ia[q]] += v;
                }
            }
            if (k < N)
#pragma unroll
                for (int i = 0; i < NU; ++i) {
                    const double uu = AT(U, k * NU + i), sl = uu - p.umin[i], su = p.umax[i] - uu;
                    H[iu + i][iu + i] += AT(zl, k * NU + i) / sl + AT(zu, k * NU + i) / su;
                    g[iu + i] += -mu / sl + mu / su;
                }
            if (dm.ns) {
                const double s = AT(S, k);
                H[is][is] += AT(zs, k) / s;
                g[is] += -mu / s + kappa_d * mu;
            }
            for (int i = 0; i < nz; ++i) H[i][i] += dw;
        } else {
            for (int i = 0; i < nz; ++i) H[i][i] = 1.0;
            if (k < N)
#pragma unroll
                for (int i = 0; i < NU; ++i) g[iu + i] += -AT(zl, k * NU + i) + AT(zu, k * NU + i);
            if (dm.ns) g[is] += -AT(zs, k);
        }
        // eliminated inequality slacks t
        for (int j = 0; j < M; ++j) {
            double J[NZ];
#pragma unroll
            for (int a = 0; a < NZ; ++a) J[a] = 0;
#pragma unroll
            for (int a = 0; a < 3; ++a)
                if (a < NX) J[a] = AT(Jd, (k * M + j) * 3 + a);
            if (dm.sd) J[is] = 1.0;
            const double t = AT(T, k * M + j), v = AT(vt, k * M + j);
            double Dj, rhs;
            if (mode == MODE_NEWTON) {
                Dj = v / t + dw;
                rhs = Dj * AT(rcq, k * M + j) + (-mu / t + kappa_d * mu);
            } else {
                Dj = 1.0;
                rhs = -v;
            }
#pragma unroll
            for (int a = 0; a < NZ; ++a) {
                g[a] += J[a] * rhs;
#pragma unroll
                for (int c = 0; c < NZ; ++c) H[a][c] += Dj * J[a] * J[c];
            }
        }
    }

    // path-length cross block M_k (positions of x_k vs x_{k+1}) = -G_k
    __device__ static void cross(const NlotProblem& p, const Ws& ws, int b, int k, int mode, double (*Mk)[2]) {
        Mk[0][0] = Mk[0][1] = Mk[1][0] = Mk[1][1] = 0;
        if (mode != MODE_NEWTON) return;
        const double dx = AT(X, (k + 1) * NX) - AT(X, k * NX), dy = AT(X, (k + 1) * NX + 1) - AT(X, k * NX + 1);
        const double r2 = dx * dx + dy * dy + p.path_eps, r = sqrt(r2), r3 = r2 * r;
        Mk[0][0] = -(r2 - dx * dx) / r3;
        Mk[0][1] = Mk[1][0] = dx * dy / r3;
        Mk[1][1] = -(r2 - dy * dy) / r3;
    }

    // Backward Riccati with the terminal multiplier carried along, then the forward sweep.
    // Residuals of the right-hand side come from rci/rcd/rct/rcq (zero in LSQ mode).
    // Returns 0, or 1 when the inertia test fails.
    __device__ static int riccati(const NlotProblem& p, const Dims& dm, const Ws& ws, int b, int mode, double dw) {
        const int N = dm.N, nc = dm.nc, ns = dm.ns;
        double P[NX][NX], pp[NX], G[NX][NC], Psi[NC][NC], psi[NC];
#pragma unroll
        for (int i = 0; i < NX; ++i) {
            pp[i] = 0;
#pragma unroll
            for (int j = 0; j < NX; ++j) P[i][j] = 0;
#pragma unroll
            for (int c = 0; c < NC; ++c) G[i][c] = 0;
        }
#pragma unroll
        for (int a = 0; a < NC; ++a) {
            psi[a] = 0;
#pragma unroll
            for (int c = 0; c < NC; ++c) Psi[a][c] = 0;
        }
        int negsum = 0;
        SC(SC_DC) = 0.0;
        for (int k = N; k >= 0; --k) {
            const int nv = (k < N ? NU : 0) + ns, nz = NX + nv;
            double H[NZ][NZ], g[NZ];
            stage(p, dm, ws, b, k, mode, dw, H, g);
            double A[NX][NX], Bu[NX][NU], c[NX];
            // [A B] with the slack column zero;  c = F_k - x_{k+1} = -rcd_k
#pragma unroll
            for (int i = 0; i < NX; ++i) {
                c[i] = 0;
#pragma unroll
                for (int j = 0; j < NX; ++j) A[i][j] = 0;
#pragma unroll
                for (int j = 0; j < NU; ++j) Bu[i][j] = 0;
            }
            if (k < N) {
                double x[NX], u[NU];
#pragma unroll
                for (int i = 0; i < NX; ++i) x[i] = AT(X, k * NX + i);
#pragma unroll
                for (int i = 0; i < NU; ++i) u[i] = AT(U, k * NU + i);
                D::jac(x, u, p.dt, p.wheelbase, A, Bu);
#pragma unroll
                for (int i = 0; i < NX; ++i) c[i] = mode == MODE_NEWTON ? -AT(rcd, k * NX + i) : 0.0;
                double Mk[2][2];
                cross(p, ws, b, k, mode, Mk);
                // substitute dx_{k+1} = A dx + B dv + c into dx_k' M dx_{k+1}
#pragma unroll
                for (int i = 0; i < 2; ++i) {
#pragma unroll
                    for (int j = 0; j < NX; ++j) {
                        const double ma = Mk[i][0] * A[0][j] + Mk[i][1] * A[1][j];
                        H[i][j] += ma;
                        H[j][i] += ma;
                    }
#pragma unroll
                    for (int j = 0; j < NU; ++j) {
                        const double mb = Mk[i][0] * Bu[0][j] + Mk[i][1] * Bu[1][j];
                        H[i][NX + j] += mb;
                        H[NX + j][i] += mb;
                    }
                    g[i] += Mk[i][0] * c[0] + Mk[i][1] * c[1];
                }
            }
            // AB = [A | B | 0]  (NX x NZ)
            double AB[NX][NZ];
#pragma unroll
            for (int i = 0; i < NX; ++i) {
#pragma unroll
                for (int j = 0; j < NX; ++j) AB[i][j] = A[i][j];
#pragma unroll
                for (int j = 0; j < NV; ++j) AB[i][NX + j] = j < NU ? Bu[i][j] : 0.0;
            }
            double PAB[NX][NZ], Pcp[NX];
#pragma unroll
            for (int i = 0; i < NX; ++i) {
#pragma unroll
                for (int j = 0; j < NZ; ++j) {
                    double t = 0;
#pragma unroll
                    for (int q = 0; q < NX; ++q) t += P[i][q] * AB[q][j];
                    PAB[i][j] = t;
                }
                double t = pp[i];
#pragma unroll
                for (int q = 0; q < NX; ++q) t += P[i][q] * c[q];
                Pcp[i] = t;
            }
            // Q = H' + AB' P AB, q = g' + AB'(P c + p), QN = AB' G
            double Q[NZ][NZ], q[NZ], QN[NZ][NC];
#pragma unroll
            for (int i = 0; i < NZ; ++i) {
#pragma unroll
                for (int j = 0; j < NZ; ++j) {
                    double t = H[i][j];
#pragma unroll
                    for (int r = 0; r < NX; ++r) t += AB[r][i] * PAB[r][j];
                    Q[i][j] = t;
                }
                double t = g[i];
#pragma unroll
                for (int r = 0; r < NX; ++r) t += AB[r][i] * Pcp[r];
                q[i] = t;
#pragma unroll
                for (int cc = 0; cc < NC; ++cc) {
                    double u = 0;
#pragma unroll
                    for (int r = 0; r < NX; ++r) u += AB[r][i] * G[r][cc];
                    QN[i][cc] = u;
                }
            }
            // stage control block: slack at position NX + nv - 1 when k == N (no u at the last knot)
            int vidx[NV];
#pragma unroll
            for (int v = 0; v < NV; ++v) vidx[v] = NX + v;
            // stage() places the slack at NX + (k < N ? NU : 0): at the last knot it is column NX
            if (k == N) vidx[0] = NX;
            double Kk[NV][NX], kk[NV], Kn[NV][NC];
#pragma unroll
            for (int v = 0; v < NV; ++v) {
                kk[v] = 0;
#pragma unroll
                for (int j = 0; j < NX; ++j) Kk[v][j] = 0;
#pragma unroll
                for (int cc = 0; cc < NC; ++cc) Kn[v][cc] = 0;
            }
            if (nv > 0) {
                double L[NV][NV];
                int perm[NV], nneg;
#pragma unroll
                for (int i = 0; i < NV; ++i)
#pragma unroll
                    for (int j = 0; j < NV; ++j) L[i][j] = (i < nv && j < nv) ? Q[vidx[i]][vidx[j]] : 0.0;
                if (ldl_factor<NV>(L, nv, perm, &nneg)) return 1;
                negsum += nneg;
                if (negsum > nc) return 1;
                double col[NV];
#pragma unroll
                for (int j = 0; j < NX; ++j) {
#pragma unroll
                    for (int v = 0; v < NV; ++v) col[v] = v < nv ? -Q[vidx[v]][j] : 0.0;
                    ldl_solve1<NV>(L, nv, perm, col);
#pragma unroll
                    for (int v = 0; v < NV; ++v) Kk[v][j] = col[v];
                }
#pragma unroll
                for (int v = 0; v < NV; ++v) col[v] = v < nv ? -q[vidx[v]] : 0.0;
                ldl_solve1<NV>(L, nv, perm, col);
#pragma unroll
                for (int v = 0; v < NV; ++v) kk[v] = col[v];
#pragma unroll
                for (int cc = 0; cc < NC; ++cc) {
                    if (cc >= nc) break;
#pragma unroll
                    for (int v = 0; v < NV; ++v) col[v] = v < nv ? -QN[vidx[v]][cc] : 0.0;
                    ldl_solve1<NV>(L, nv, perm, col);
#pragma unroll
                    for (int v = 0; v < NV; ++v) Kn[v][cc] = col[v];
                }
            }
            // store gains
#pragma unroll
            for (int v = 0; v < NV; ++v) {
                if (v >= dm.nv) continue;
                AT(kf, k * dm.nv + v) = kk[v];
#pragma unroll
                for (int j = 0; j < NX; ++j) AT(Kf, (k * dm.nv + v) * NX + j) = Kk[v][j];
#pragma unroll
                for (int cc = 0; cc < NC; ++cc)
                    if (cc < nc) AT(Kn, (k * dm.nv + v) * nc + cc) = Kn[v][cc];
            }
            // value function of stage k
            double Pn[NX][NX], pn[NX], Gn[NX][NC];
#pragma unroll
            for (int i = 0; i < NX; ++i) {
#pragma unroll
                for (int j = 0; j < NX; ++j) {
                    double t = Q[i][j];
#pragma unroll
                    for (int v = 0; v < NV; ++v)
                        if (v < nv) t += Q[i][vidx[v]] * Kk[v][j];
                    Pn[i][j] = t;
                }
                double t = q[i];
#pragma unroll
                for (int v = 0; v < NV; ++v)
                    if (v < nv) t += Q[i][vidx[v]] * kk[v];
                pn[i] = t;
#pragma unroll
                for (int cc = 0; cc < NC; ++cc) {
                    double u = QN[i][cc];
#pragma unroll
                    for (int v = 0; v < NV; ++v)
                        if (v < nv) u += Q[i][vidx[v]] * Kn[v][cc];
                    Gn[i][cc] = u;
                }
            }
#pragma unroll
            for (int i = 0; i < NX; ++i)
#pragma unroll
                for (int j = 0; j < i; ++j) {
                    const double a = 0.5 * (Pn[i][j] + Pn[j][i]);
                    Pn[i][j] = Pn[j][i] = a;
                }
#pragma unroll
            for (int a = 0; a < NC; ++a) {
                if (a >= nc) continue;
#pragma unroll
                for (int cc = 0; cc < NC; ++cc) {
                    if (cc >= nc) continue;
                    double t = 0;
#pragma unroll
                    for (int v = 0; v < NV; ++v)
                        if (v < nv) t += QN[vidx[v]][a] * Kn[v][cc];
                    Psi[a][cc] += t;
                }
                double t = 0;
#pragma unroll
                for (int r = 0; r < NX; ++r) t += G[r][a] * c[r];
#pragma unroll
                for (int v = 0; v < NV; ++v)
                    if (v < nv) t += QN[vidx[v]][a] * kk[v];
                psi[a] += t;
            }
            if (k == N) {  // terminal equality C x_N = xg_sel
#pragma unroll
                for (int i = 0; i < NX; ++i)
#pragma unroll
                    for (int cc = 0; cc < NC; ++cc) Gn[i][cc] = 0;
                for (int cc = 0; cc < nc; ++cc) {
                    Gn[dm.tidx[cc]][cc] = 1.0;
                    psi[cc] = mode == MODE_NEWTON ? AT(rct, cc) : 0.0;
                }
            }
#pragma unroll
            for (int i = 0; i < NX; ++i) {
                AT(pv, k * NX + i) = pn[i];
#pragma unroll
                for (int j = 0; j < NX; ++j) AT(Pm, (k * NX + i) * NX + j) = Pn[i][j];
#pragma unroll
                for (int cc = 0; cc < NC; ++cc)
                    if (cc < nc) AT(Gm, (k * NX + i) * nc + cc) = Gn[i][cc];
            }
#pragma unroll
            for (int i = 0; i < NX; ++i) {
                pp[i] = pn[i];
#pragma unroll
                for (int j = 0; j < NX; ++j) P[i][j] = Pn[i][j];
#pragma unroll
                for (int cc = 0; cc < NC; ++cc) G[i][cc] = Gn[i][cc];
            }
        }
        // terminal multiplier (Sylvester inertia check, delta_c on the terminal block if needed)
        double dx0[NX], nu_[NC];
#pragma unroll
        for (int i = 0; i < NX; ++i) dx0[i] = mode == MODE_NEWTON ? -AT(rci, i) : 0.0;
#pragma unroll
        for (int cc = 0; cc < NC; ++cc) nu_[cc] = 0;
        if (nc) {
            double L[NC][NC];
            int perm[NC], nneg;
#pragma unroll
            for (int i = 0; i < NC; ++i)
#pragma unroll
                for (int j = 0; j < NC; ++j) L[i][j] = (i < nc && j < nc) ? -Psi[i][j] : 0.0;
            int st = ldl_factor<NC>(L, nc, perm, &nneg);
            if (st == 2 || nneg != negsum) {
                const double dc = 1e-8 * pow(SC(SC_MU), 0.25);
#pragma unroll
                for (int i = 0; i < NC; ++i)
#pragma unroll
                    for (int j = 0; j < NC; ++j) L[i][j] = (i < nc && j < nc) ? -Psi[i][j] + (i == j ? dc : 0.0) : 0.0;
                if (ldl_factor<NC>(L, nc, perm, &nneg)) return 1;
                if (nneg != negsum) return 1;
                SC(SC_DC) = dc;
            }
#pragma unroll
            for (int cc = 0; cc < NC; ++cc) {
                if (cc >= nc) continue;
                double t = psi[cc];
#pragma unroll
                for (int r = 0; r < NX; ++r) t += G[r][cc] * dx0[r];
                nu_[cc] = t;
            }
            ldl_solve1<NC>(L, nc, perm, nu_);
        } else if (negsum) {
            return 1;
        }
        // forward sweep
        double dx[NX];
#pragma unroll
        for (int i = 0; i < NX; ++i) dx[i] = dx0[i];
        for (int k = 0; k <= N; ++k) {
            const int nv = (k < N ? NU : 0) + ns;
            double dvv[NV];
#pragma unroll
            for (int v = 0; v < NV; ++v) {
                dvv[v] = 0;
                if (v >= nv) continue;
                double t = AT(kf, k * dm.nv + v);
#pragma unroll
                for (int j = 0; j < NX; ++j) t += AT(Kf, (k * dm.nv + v) * NX + j) * dx[j];
#pragma unroll
                for (int cc = 0; cc < NC; ++cc)
                    if (cc < nc) t += AT(Kn, (k * dm.nv + v) * nc + cc) * nu_[cc];
                dvv[v] = t;
            }
#pragma unroll
            for (int i = 0; i < NX; ++i) AT(dX, k * NX + i) = dx[i];
            if (k < N)
#pragma unroll
                for (int i = 0; i < NU; ++i) AT(dU, k * NU + i) = dvv[i];
            if (ns) AT(dS, k) = dvv[nv - 1];
            if (k == 0) {
#pragma unroll
                for (int i = 0; i < NX; ++i) {
                    double t = AT(pv, i);
#pragma unroll
                    for (int j = 0; j < NX; ++j) t += AT(Pm, i * NX + j) * dx[j];
#pragma unroll
                    for (int cc = 0; cc < NC; ++cc)
                        if (cc < nc) t += AT(Gm, i * nc + cc) * nu_[cc];
                    AT(yi_n, i) = -t;
                }
            }
            if (k < N) {
                double x[NX], u[NU], A[NX][NX], Bu[NX][NU], dn[NX];
#pragma unroll
                for (int i = 0; i < NX; ++i) x[i] = AT(X, k * NX + i);
#pragma unroll
                for (int i = 0; i < NU; ++i) u[i] = AT(U, k * NU + i);
                D::jac(x, u, p.dt, p.wheelbase, A, Bu);
#pragma unroll
                for (int i = 0; i < NX; ++i) {
                    double t = mode == MODE_NEWTON ? -AT(rcd, k * NX + i) : 0.0;
#pragma unroll
                    for (int j = 0; j < NX; ++j) t += A[i][j] * dx[j];
#pragma unroll
                    for (int j = 0; j < NU; ++j) t += Bu[i][j] * dvv[j];
                    dn[i] = t;
                }
                double Mk[2][2];
                cross(p, ws, b, k, mode, Mk);
#pragma unroll
                for (int i = 0; i < NX; ++i) {
                    double t = AT(pv, (k + 1) * NX + i);
#pragma unroll
                    for (int j = 0; j < NX; ++j) t += AT(Pm, ((k + 1) * NX + i) * NX + j) * dn[j];
#pragma unroll
                    for (int cc = 0; cc < NC; ++cc)
                        if (cc < nc) t += AT(Gm, ((k + 1) * NX + i) * nc + cc) * nu_[cc];
                    double mt = i < 2 ? Mk[0][i] * dx[0] + Mk[1][i] * dx[1] : 0.0;
                    AT(yk_n, k * NX + i) = -t - mt;
                }
#pragma unroll
                for (int i = 0; i < NX; ++i) dx[i] = dn[i];
            }
        }
#pragma unroll
        for (int cc = 0; cc < NC; ++cc)
            if (cc < nc) AT(yt_n, cc) = nu_[cc];
        return 0;
    }
};

// ---------------------------------------------------------------------------------------------
// kernels
// ---------------------------------------------------------------------------------------------
__global__ void k_init_state(NlotProblem p, Dims dm, NlotSolverOptions o, Ws ws, const double* __restrict__ x0,
                             const double* __restrict__ xg, const double* __restrict__ Xinit, int B) {
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= B) return;
    const int N = dm.N, nx = dm.nx, nu = dm.nu, M = dm.M;
    const double k1 = o.bound_push, k2 = o.bound_frac;
    for (int k = 0; k <= N; ++k)
        for (int i = 0; i < nx; ++i) {
            double v;
            if (Xinit) v = Xinit[((size_t)b * (N + 1) + k) * nx + i];
            else v = x0[(size_t)b * nx + i] + (xg[(size_t)b * nx + i] - x0[(size_t)b * nx + i]) * ((double)k / (double)N);
            AT(X, k * nx + i) = v;  // LinearInitializer (trajectory_initialization.py:54-55)
        }
    for (int k = 0; k < N; ++k)
        for (int i = 0; i < nu; ++i) {
            const double lo = p.umin[i], hi = p.umax[i];
            const double pl = fmin(k1 * fmax(1.0, fabs(lo)), k2 * (hi - lo));
            const double pu = fmin(k1 * fmax(1.0, fabs(hi)), k2 * (hi - lo));
            AT(U, k * nu + i) = fmin(fmax(0.0, lo + pl), hi - pu);
            AT(zl, k * nu + i) = 1.0;
            AT(zu, k * nu + i) = 1.0;
        }
    for (int k = 0; k <= N; ++k) {
        AT(S, k) = dm.ns ? fmax(0.0, k1) : 0.0;
        AT(zs, k) = 1.0;
        AT(dS, k) = 0.0;
    }
    for (int i = 0; i < (N + 1) * nx; ++i) AT(dX, i) = 0.0;  // step arrays start defined (0 * garbage = NaN)
    for (int i = 0; i < N * nu; ++i) AT(dU, i) = 0.0;
    for (int q = 0; q < (N + 1) * M; ++q) AT(dT, q) = 0.0;
    for (int q = 0; q < (N + 1) * M; ++q) AT(vt, q) = 1.0;
    SC(SC_MU) = o.mu_init;
    SC(SC_TAU) = fmax(0.99, 1.0 - o.mu_init);
    SC(SC_DWLAST) = 0;
    SC(SC_STATUS) = -1;
    SC(SC_ITERS) = 0;
    SC(SC_PHASE) = PH_INIT;
    SC(SC_NFILT) = 0;
    SC(SC_E0) = 0;
}

// corners of X (+ alpha dX) for instances in the given phases, compacted into the MLP point list
__global__ void k_points(NlotProblem p, Dims dm, Ws ws, int B, int trial) {
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= B) return;
    const int ph = (int)SC(SC_PHASE);
    const bool want = trial ? ph == PH_LS : (ph == PH_INIT || ph == PH_EVAL);
    if (!want) return;
    const int rank = atomicAdd(&ws.cnt[trial ? 1 : 0], 1);
    SC(SC_RANK) = rank;
    const double al = trial ? SC(SC_ALPHA) : 0.0;
    const int nx = dm.nx;
    for (int k = 0; k <= dm.N; ++k) {
        const double x = AT(X, k * nx) + al * AT(dX, k * nx);
        const double y = AT(X, k * nx + 1) + al * AT(dX, k * nx + 1);
        if (p.shape == NLOT_SHAPE_DOT) {
            const size_t o = ((size_t)k * ws.cap + rank) * 2;
            ws.pts[o] = (float)x;  // CasADi double -> fp32 (gen/nn_sdf.cpp)
            ws.pts[o + 1] = (float)y;
            continue;
        }
        const double th = AT(X, k * nx + 2) + al * AT(dX, k * nx + 2);
        double sn, cs;
        sincos(th, &sn, &cs);
        for (int i = 0; i < dm.nb; ++i) {
            const double bx = p.body[i][0], by = p.body[i][1];
            const size_t o = ((size_t)(k * dm.nb + i) * ws.cap + rank) * 2;
            ws.pts[o] = (float)(x + cs * bx - sn * by);
            ws.pts[o + 1] = (float)(y + sn * bx + cs * by);
        }
    }
}

__device__ inline double frac_to_bound(double sl, double dsl, double tau, double amax) {
    if (dsl < 0) {
        const double a = -tau * sl / dsl;
        if (a < amax) return a;
    }
    return amax;
}

template <int DYN>
__global__ void __launch_bounds__(64) k_iterate(NlotProblem p, Dims dm, NlotSolverOptions o, Ws ws, int B,
                                                const double* __restrict__ x0, const double* __restrict__ xg) {
    using SV = Solver<DYN>;
    constexpr int NX = SV::NX, NU = SV::NU;
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= B) return;
    const int ph = (int)SC(SC_PHASE);
    if (ph != PH_INIT && ph != PH_EVAL) return;
    const int N = dm.N, M = dm.M, nc = dm.nc;
    const int rank = (int)SC(SC_RANK);
    const double k1 = o.bound_push;
    const double* x0b = x0 + (size_t)b * NX;
    const double* xgb = xg + (size_t)b * NX;

    // ---- knot data: d, J_d (y_d-weighted Hessian later) ----
    auto eval_knots = [&](bool with_hess) {
        for (int k = 0; k <= N; ++k) {
            double xk[NX], d[MMAX], gk[MMAX][3], w[MMAX], Hw[6];
#pragma unroll
            for (int i = 0; i < NX; ++i) xk[i] = AT(X, k * NX + i);
            for (int j = 0; j < M; ++j) w[j] = AT(yd, k * M + j);
            knot_eval(p, dm, ws, rank, k, xk, d, gk, w, with_hess ? Hw : nullptr);
            for (int j = 0; j < M; ++j) {
                const double dj = d[j] + (dm.sd ? AT(S, k) : 0.0);
                AT(dv, k * M + j) = dj;
                for (int a = 0; a < 3; ++a) AT(Jd, (k * M + j) * 3 + a) = gk[j][a];
            }
            if (with_hess)
                for (int q = 0; q < 6; ++q) AT(Hd, k * 6 + q) = Hw[q];
        }
    };
    auto residuals = [&]() {  // c(x) at the current point (IPOPT sign)
#pragma unroll
        for (int i = 0; i < NX; ++i) AT(rci, i) = AT(X, i) - x0b[i];
        for (int cc = 0; cc < nc; ++cc) AT(rct, cc) = AT(X, N * NX + dm.tidx[cc]) - xgb[dm.tidx[cc]];
        for (int k = 0; k < N; ++k) {
            double x[NX], u[NU], f[NX];
#pragma unroll
            for (int i = 0; i < NX; ++i) x[i] = AT(X, k * NX + i);
#pragma unroll
            for (int i = 0; i < NU; ++i) u[i] = AT(U, k * NU + i);
            Dyn<DYN>::f(x, u, p.wheelbase, f);
#pragma unroll
            for (int i = 0; i < NX; ++i) AT(rcd, k * NX + i) = AT(X, (k + 1) * NX + i) - (x[i] + p.dt * f[i]);
        }
        for (int q = 0; q < (N + 1) * M; ++q) AT(rcq, q) = AT(dv, q) - AT(T, q);
    };

    if (ph == PH_INIT) {
        eval_knots(false);
        for (int q = 0; q < (N + 1) * M; ++q) AT(T, q) = fmax(AT(dv, q), k1);  // slack push
        for (int q = 0; q < (N + 1) * M; ++q) AT(yd, q) = 0.0;
        // least-squares equality multipliers (IPOPT LeastSquareMultipliers)
        if (SV::riccati(p, dm, ws, b, MODE_LSQ, 0.0) == 0) {
            double ymax = 0;
            for (int k = 0; k <= N; ++k)
                for (int j = 0; j < M; ++j) {
                    double w = 0;
                    for (int a = 0; a < 3 && a < NX; ++a) w += AT(Jd, (k * M + j) * 3 + a) * AT(dX, k * NX + a);
                    if (dm.sd) w += AT(dS, k);
                    const double v = w - AT(vt, k * M + j);
                    AT(yd, k * M + j) = v;
                    ymax = fmax(ymax, fabs(v));
                }
            for (int i = 0; i < NX; ++i) ymax = fmax(ymax, fabs(AT(yi, i) = AT(yi_n, i)));
            for (int i = 0; i < N * NX; ++i) ymax = fmax(ymax, fabs(AT(yk, i) = AT(yk_n, i)));
            for (int cc = 0; cc < nc; ++cc) ymax = fmax(ymax, fabs(AT(yt, cc) = AT(yt_n, cc)));
            if (ymax > o.constr_mult_init_max) {
                for (int i = 0; i < NX; ++i) AT(yi, i) = 0;
                for (int i = 0; i < N * NX; ++i) AT(yk, i) = 0;
                for (int cc = 0; cc < nc; ++cc) AT(yt, cc) = 0;
                for (int q = 0; q < (N + 1) * M; ++q) AT(yd, q) = 0;
            }
        } else {
            for (int i = 0; i < NX; ++i) AT(yi, i) = 0;
            for (int i = 0; i < N * NX; ++i) AT(yk, i) = 0;
            for (int cc = 0; cc < nc; ++cc) AT(yt, cc) = 0;
            for (int q = 0; q < (N + 1) * M; ++q) AT(yd, q) = 0;
        }
    }
    eval_knots(true);
    residuals();

    // ---- theta / phi at the current point ----
    const double mu0 = SC(SC_MU);
    auto theta_phi = [&](double mu, double* th, double* ph_) {
        double t = 0, bar = 0, lin = 0;
        for (int i = 0; i < NX; ++i) t += fabs(AT(rci, i));
        for (int cc = 0; cc < nc; ++cc) t += fabs(AT(rct, cc));
        for (int i = 0; i < N * NX; ++i) t += fabs(AT(rcd, i));
        for (int q = 0; q < (N + 1) * M; ++q) {
            t += fabs(AT(rcq, q));
            bar += log(AT(T, q));
            lin += AT(T, q);
        }
        for (int k = 0; k < N; ++k)
            for (int i = 0; i < NU; ++i) {
                const double u = AT(U, k * NU + i);
                bar += log(u - p.umin[i]) + log(p.umax[i] - u);
            }
        if (dm.ns)
            for (int k = 0; k <= N; ++k) {
                bar += log(AT(S, k));
                lin += AT(S, k);
            }
        *th = t;
        *ph_ = objective(p, dm, ws, b, nullptr, nullptr, nullptr, 0.0) - mu * bar + 1e-5 * mu * lin;
    };
    if (ph == PH_INIT) {
        double th0, p0;
        theta_phi(mu0, &th0, &p0);
        SC(SC_THMAX) = 1e4 * fmax(1.0, th0);
        SC(SC_THMIN) = 1e-4 * fmax(1.0, th0);
        SC(SC_NFILT) = 0;
    }

    // ---- optimality measures (IPOPT scaled E_0 / E_mu) ----
    double dual = 0, primal = 0, c0 = 0, cmu = 0, cviol = 0, ysum = 0, zsum = 0;
    int nzc = 0;
    {
        for (int k = 0; k <= N; ++k) {
            double r[NX];
            // objective gradient w.r.t. x_k (path length)
#pragma unroll
            for (int i = 0; i < NX; ++i) r[i] = 0;
            for (int seg = k - 1; seg <= k; ++seg) {
                if (seg < 0 || seg >= N) continue;
                const double dx = AT(X, (seg + 1) * NX) - AT(X, seg * NX);
                const double dy = AT(X, (seg + 1) * NX + 1) - AT(X, seg * NX + 1);
                const double rr = sqrt(dx * dx + dy * dy + p.path_eps);
                const double sgn = seg == k ? -1.0 : 1.0;
                r[0] += sgn * dx / rr;
                r[1] += sgn * dy / rr;
            }
            if (k > 0)
#pragma unroll
                for (int i = 0; i < NX; ++i) r[i] += AT(yk, (k - 1) * NX + i);
            double A[NX][NX], Bu[NX][NU];
            if (k < N) {
                double x[NX], u[NU];
#pragma unroll
                for (int i = 0; i < NX; ++i) x[i] = AT(X, k * NX + i);
#pragma unroll
                for (int i = 0; i < NU; ++i) u[i] = AT(U, k * NU + i);
                Dyn<DYN>::jac(x, u, p.dt, p.wheelbase, A, Bu);
#pragma unroll
                for (int j = 0; j < NX; ++j) {
                    double t = 0;
#pragma unroll
                    for (int i = 0; i < NX; ++i) t += A[i][j] * AT(yk, k * NX + i);
                    r[j] -= t;
                }
            }
            if (k == 0)
#pragma unroll
                for (int i = 0; i < NX; ++i) r[i] += AT(yi, i);
            if (k == N)
                for (int cc = 0; cc < nc; ++cc) r[dm.tidx[cc]] += AT(yt, cc);
            for (int j = 0; j < M; ++j)
                for (int a = 0; a < 3 && a < NX; ++a) r[a] += AT(Jd, (k * M + j) * 3 + a) * AT(yd, k * M + j);
#pragma unroll
            for (int i = 0; i < NX; ++i) dual = fmax(dual, fabs(r[i]));
            if (k < N)
#pragma unroll
                for (int i = 0; i < NU; ++i) {
                    double t = -AT(zl, k * NU + i) + AT(zu, k * NU + i);
                    if (p.use_smooth && k < N - 1) t += 2.0 * p.smooth_weight * AT(U, k * NU + i);
#pragma unroll
                    for (int a = 0; a < NX; ++a) t -= Bu[a][i] * AT(yk, k * NX + a);
                    dual = fmax(dual, fabs(t));
                }
            if (dm.ns) {
                double t = 2.0 * p.slack_penalty * AT(S, k) - AT(zs, k);
                if (dm.sd)
                    for (int j = 0; j < M; ++j) t += AT(yd, k * M + j);
                dual = fmax(dual, fabs(t));
            }
            for (int j = 0; j < M; ++j) dual = fmax(dual, fabs(-AT(yd, k * M + j) - AT(vt, k * M + j)));
        }
        for (int i = 0; i < NX; ++i) primal = fmax(primal, fabs(AT(rci, i)));
        for (int cc = 0; cc < nc; ++cc) primal = fmax(primal, fabs(AT(rct, cc)));
        for (int i = 0; i < N * NX; ++i) primal = fmax(primal, fabs(AT(rcd, i)));
        cviol = primal;
        for (int q = 0; q < (N + 1) * M; ++q) {
            primal = fmax(primal, fabs(AT(rcq, q)));
            cviol = fmax(cviol, fmax(0.0, -AT(dv, q)));
        }
        auto compl_ = [&](double z, double s) {
            c0 = fmax(c0, fabs(z * s));
            cmu = fmax(cmu, fabs(z * s - mu0));
            zsum += fabs(z);
            nzc++;
        };
        for (int k = 0; k < N; ++k)
            for (int i = 0; i < NU; ++i) {
                const double u = AT(U, k * NU + i);
                compl_(AT(zl, k * NU + i), u - p.umin[i]);
                compl_(AT(zu, k * NU + i), p.umax[i] - u);
            }
        if (dm.ns)
            for (int k = 0; k <= N; ++k) compl_(AT(zs, k), AT(S, k));
        for (int q = 0; q < (N + 1) * M; ++q) compl_(AT(vt, q), AT(T, q));
        for (int i = 0; i < NX; ++i) ysum += fabs(AT(yi, i));
        for (int i = 0; i < N * NX; ++i) ysum += fabs(AT(yk, i));
        for (int cc = 0; cc < nc; ++cc) ysum += fabs(AT(yt, cc));
        for (int q = 0; q < (N + 1) * M; ++q) ysum += fabs(AT(yd, q));
    }
    const int ny = NX + N * NX + nc + (N + 1) * M;
    const double sd = fmax(100.0, (ysum + zsum) / (double)(ny + nzc)) / 100.0;
    const double scc = fmax(100.0, zsum / (double)nzc) / 100.0;
    const double E0 = fmax(fmax(dual / sd, primal), c0 / scc);
    SC(SC_E0) = E0;
    const int iters = (int)SC(SC_ITERS);
    if (!isfinite(E0)) {
        SC(SC_STATUS) = NLOT_NUMERIC;
        SC(SC_PHASE) = PH_DONE;
        return;
    }
    if (E0 <= o.tol && dual <= o.dual_inf_tol && cviol <= o.constr_viol_tol && c0 <= o.compl_inf_tol) {
        SC(SC_STATUS) = NLOT_SOLVED;
        SC(SC_PHASE) = PH_DONE;
        return;
    }
    if (iters >= o.max_iter) {
        SC(SC_STATUS) = NLOT_MAXITER;
        SC(SC_PHASE) = PH_DONE;
        return;
    }
    // ---- monotone barrier update ----
    double mu = mu0;
    if (iters > 0) {
        const double kap = o.barrier_tol_factor;
        double cm = cmu;
        for (;;) {
            const double Emu = fmax(fmax(dual / sd, primal), cm / scc);
            if (Emu > kap * mu) break;
            double nm = fmin(0.2 * mu, pow(mu, 1.5));
            nm = fmax(nm, fmin(o.tol, o.compl_inf_tol) / (kap + 1.0));
            if (nm >= mu) break;
            mu = nm;
            SC(SC_MU) = mu;
            SC(SC_TAU) = fmax(0.99, 1.0 - mu);
            SC(SC_NFILT) = 0;
            cm = 0;  // recompute the complementarity error for the new mu
            for (int k = 0; k < N; ++k)
                for (int i = 0; i < NU; ++i) {
                    const double u = AT(U, k * NU + i);
                    cm = fmax(cm, fabs(AT(zl, k * NU + i) * (u - p.umin[i]) - mu));
                    cm = fmax(cm, fabs(AT(zu, k * NU + i) * (p.umax[i] - u) - mu));
                }
            if (dm.ns)
                for (int k = 0; k <= N; ++k) cm = fmax(cm, fabs(AT(zs, k) * AT(S, k) - mu));
            for (int q = 0; q < (N + 1) * M; ++q) cm = fmax(cm, fabs(AT(vt, q) * AT(T, q) - mu));
        }
    }
    // ---- search direction with inertia correction ----
    double dw = 0.0;
    if (SV::riccati(p, dm, ws, b, MODE_NEWTON, 0.0)) {
        const double last = SC(SC_DWLAST);
        dw = last == 0.0 ? 1e-4 : fmax(1e-20, last / 3.0);
        for (;;) {
            if (!SV::riccati(p, dm, ws, b, MODE_NEWTON, dw)) break;
            dw *= (last == 0.0) ? 100.0 : 8.0;
            if (dw > 1e40) break;
        }
        if (dw > 1e40) {
            SC(SC_STATUS) = NLOT_NUMERIC;
            SC(SC_PHASE) = PH_DONE;
            return;
        }
        SC(SC_DWLAST) = dw;
    }
    SC(SC_DW) = dw;
    // ---- recover dt, yd+, dz ----
    const double kappa_d = 1e-5, tau = SC(SC_TAU);
    for (int k = 0; k <= N; ++k)
        for (int j = 0; j < M; ++j) {
            const int q = k * M + j;
            double Jdz = 0;
            for (int a = 0; a < 3 && a < NX; ++a) Jdz += AT(Jd, q * 3 + a) * AT(dX, k * NX + a);
            if (dm.sd) Jdz += AT(dS, k);
            const double t = AT(T, q), v = AT(vt, q);
            const double dt_ = Jdz + AT(rcq, q);
            AT(dT, q) = dt_;
            AT(yd_n, q) = (v / t + dw) * dt_ + (-mu / t + kappa_d * mu);
            AT(dvt, q) = mu / t - v - (v / t) * dt_;
        }
    for (int k = 0; k < N; ++k)
        for (int i = 0; i < NU; ++i) {
            const int q = k * NU + i;
            const double u = AT(U, q), sl = u - p.umin[i], su = p.umax[i] - u, du = AT(dU, q);
            AT(dzl, q) = mu / sl - AT(zl, q) - (AT(zl, q) / sl) * du;
            AT(dzu, q) = mu / su - AT(zu, q) + (AT(zu, q) / su) * du;
        }
    if (dm.ns)
        for (int k = 0; k <= N; ++k) {
            const double s = AT(S, k);
            AT(dzs, k) = mu / s - AT(zs, k) - (AT(zs, k) / s) * AT(dS, k);
        }
    // ---- fraction to the boundary ----
    double amax = 1.0, az = 1.0;
    for (int k = 0; k < N; ++k)
        for (int i = 0; i < NU; ++i) {
            const int q = k * NU + i;
            const double u = AT(U, q);
            amax = frac_to_bound(u - p.umin[i], AT(dU, q), tau, amax);
            amax = frac_to_bound(p.umax[i] - u, -AT(dU, q), tau, amax);
            az = frac_to_bound(AT(zl, q), AT(dzl, q), tau, az);
            az = frac_to_bound(AT(zu, q), AT(dzu, q), tau, az);
        }
    if (dm.ns)
        for (int k = 0; k <= N; ++k) {
            amax = frac_to_bound(AT(S, k), AT(dS, k), tau, amax);
            az = frac_to_bound(AT(zs, k), AT(dzs, k), tau, az);
        }
    for (int q = 0; q < (N + 1) * M; ++q) {
        amax = frac_to_bound(AT(T, q), AT(dT, q), tau, amax);
        az = frac_to_bound(AT(vt, q), AT(dvt, q), tau, az);
    }
    // ---- line-search reference values ----
    double theta, phi;
    theta_phi(mu, &theta, &phi);
    double gd = 0;
    for (int k = 0; k <= N; ++k) {  // objective gradient . d
        for (int seg = k - 1; seg <= k; ++seg) {
            if (seg < 0 || seg >= N) continue;
            const double dx = AT(X, (seg + 1) * NX) - AT(X, seg * NX);
            const double dy = AT(X, (seg + 1) * NX + 1) - AT(X, seg * NX + 1);
            const double rr = sqrt(dx * dx + dy * dy + p.path_eps);
            const double sgn = seg == k ? -1.0 : 1.0;
            gd += sgn * (dx / rr) * AT(dX, k * NX) + sgn * (dy / rr) * AT(dX, k * NX + 1);
        }
    }
    for (int k = 0; k < N; ++k)
        for (int i = 0; i < NU; ++i) {
            const int q = k * NU + i;
            const double u = AT(U, q);
            double gu = -mu / (u - p.umin[i]) + mu / (p.umax[i] - u);
            if (p.use_smooth && k < N - 1) gu += 2.0 * p.smooth_weight * u;
            gd += gu * AT(dU, q);
        }
    if (dm.ns)
        for (int k = 0; k <= N; ++k) {
            const double s = AT(S, k);
            gd += (2.0 * p.slack_penalty * s - mu / s + kappa_d * mu) * AT(dS, k);
        }
    for (int q = 0; q < (N + 1) * M; ++q) gd += (-mu / AT(T, q) + kappa_d * mu) * AT(dT, q);
    const double gt = 1e-5, gp = 1e-8, delta = 1.0, sth = 1.1, sph = 2.3;
    double amin = gt;
    if (gd < 0) {
        amin = fmin(gt, gp * theta / (-gd));
        if (theta <= SC(SC_THMIN)) amin = fmin(amin, delta * pow(theta, sth) / pow(-gd, sph));
    }
    amin *= 0.05;
    SC(SC_THETA) = theta;
    SC(SC_PHI) = phi;
    SC(SC_GD) = gd;
    SC(SC_AMAX) = amax;
    SC(SC_AMIN) = amin;
    SC(SC_AZ) = az;
    SC(SC_ALPHA) = amax;
    SC(SC_TRIALS) = 0;
    SC(SC_PHASE) = PH_LS;
}

__device__ inline int cmp_le(double lhs, double rhs, double bas) { return lhs - rhs <= 10.0 * 2.220446049250313e-16 * fabs(bas); }

template <int DYN>
__global__ void __launch_bounds__(64) k_accept(NlotProblem p, Dims dm, NlotSolverOptions o, Ws ws, int B,
                                               const double* __restrict__ x0, const double* __restrict__ xg) {
    constexpr int NX = Dyn<DYN>::NX, NU = Dyn<DYN>::NU;
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= B) return;
    int ph = (int)SC(SC_PHASE);
    if (ph == PH_LS) {
        const int N = dm.N, M = dm.M, nc = dm.nc;
        const double al = SC(SC_ALPHA), mu = SC(SC_MU);
        const int rank = (int)SC(SC_RANK);
        const double* x0b = x0 + (size_t)b * NX;
        const double* xgb = xg + (size_t)b * NX;
        // theta and phi at the trial point x + al d
        double th = 0, bar = 0, lin = 0;
        for (int i = 0; i < NX; ++i) th += fabs(AT(X, i) + al * AT(dX, i) - x0b[i]);
        for (int cc = 0; cc < nc; ++cc) {
            const int ix = N * NX + dm.tidx[cc];
            th += fabs(AT(X, ix) + al * AT(dX, ix) - xgb[dm.tidx[cc]]);
        }
        for (int k = 0; k < N; ++k) {
            double x[NX], u[NU], f[NX];
#pragma unroll
            for (int i = 0; i < NX; ++i) x[i] = AT(X, k * NX + i) + al * AT(dX, k * NX + i);
#pragma unroll
            for (int i = 0; i < NU; ++i) u[i] = AT(U, k * NU + i) + al * AT(dU, k * NU + i);
            Dyn<DYN>::f(x, u, p.wheelbase, f);
#pragma unroll
            for (int i = 0; i < NX; ++i)
                th += fabs(AT(X, (k + 1) * NX + i) + al * AT(dX, (k + 1) * NX + i) - (x[i] + p.dt * f[i]));
        }
        for (int k = 0; k <= N; ++k) {
            double xk[NX], d[MMAX];
#pragma unroll
            for (int i = 0; i < NX; ++i) xk[i] = AT(X, k * NX + i) + al * AT(dX, k * NX + i);
            knot_eval(p, dm, ws, rank, k, xk, d, nullptr, nullptr, nullptr);
            const double sk = AT(S, k) + al * AT(dS, k);
            for (int j = 0; j < M; ++j) {
                const double t = AT(T, k * M + j) + al * AT(dT, k * M + j);
                th += fabs(d[j] + (dm.sd ? sk : 0.0) - t);
                bar += log(t);
                lin += t;
            }
        }
        for (int k = 0; k < N; ++k)
            for (int i = 0; i < NU; ++i) {
                const double u = AT(U, k * NU + i) + al * AT(dU, k * NU + i);
                bar += log(u - p.umin[i]) + log(p.umax[i] - u);
            }
        if (dm.ns)
            for (int k = 0; k <= N; ++k) {
                const double s = AT(S, k) + al * AT(dS, k);
                bar += log(s);
                lin += s;
            }
        const double pht = objective(p, dm, ws, b, nullptr, nullptr, nullptr, al) - mu * bar + 1e-5 * mu * lin;
        const double theta = SC(SC_THETA), phi = SC(SC_PHI), gd = SC(SC_GD);
        const double gt = 1e-5, gp = 1e-8, delta = 1.0, sth = 1.1, sph = 2.3, eta = 1e-8;
        // IPOPT FilterLSAcceptor::CheckAcceptabilityOfTrialPoint
        int ok = isfinite(th) && isfinite(pht) && th <= SC(SC_THMAX);
        const int ftype = gd < 0 && al * pow(-gd, sph) > delta * pow(theta, sth);
        const int armijo = cmp_le(pht - phi, eta * al * gd, phi);
        if (ok) {
            if (ftype && theta <= SC(SC_THMIN)) {
                ok = armijo;
            } else {
                ok = cmp_le(th, (1.0 - gt) * theta, theta) || cmp_le(pht - phi, -gp * theta, phi);
                if (ok && pht > phi) {
                    const double bas = fabs(phi) > 10.0 ? log10(fabs(phi)) : 1.0;
                    if (log10(pht - phi) > 5.0 + bas) ok = 0;
                }
            }
        }
        int nf = (int)SC(SC_NFILT);
        if (ok)
            for (int i = 0; i < nf; ++i) {
                const double ft = AT(filt, 2 * i), fp = AT(filt, 2 * i + 1);
                if (!(th <= ft || pht <= fp)) {
                    ok = 0;
                    break;
                }
            }
        if (ok) {
            if (!(ftype && armijo)) {  // augment the filter with (1-gt) theta, phi - gp theta
                const double ntv = (1.0 - gt) * theta, npv = phi - gp * theta;
                int w = 0;
                for (int i = 0; i < nf; ++i) {
                    const double ft = AT(filt, 2 * i), fp = AT(filt, 2 * i + 1);
                    if (!(ft >= ntv && fp >= npv)) {
                        AT(filt, 2 * w) = ft;
                        AT(filt, 2 * w + 1) = fp;
                        ++w;
                    }
                }
                nf = w;
                if (nf == FILT_MAX) {
                    for (int i = 0; i + 1 < FILT_MAX; ++i) {
                        AT(filt, 2 * i) = AT(filt, 2 * (i + 1));
                        AT(filt, 2 * i + 1) = AT(filt, 2 * (i + 1) + 1);
                    }
                    nf--;
                }
                AT(filt, 2 * nf) = ntv;
                AT(filt, 2 * nf + 1) = npv;
                SC(SC_NFILT) = nf + 1;
            }
            // accept: primal and multipliers with alpha, bound multipliers with alpha_z + safeguard
            for (int i = 0; i < (N + 1) * NX; ++i) AT(X, i) += al * AT(dX, i);
            for (int i = 0; i < N * NU; ++i) AT(U, i) += al * AT(dU, i);
            if (dm.ns)
                for (int k = 0; k <= N; ++k) AT(S, k) += al * AT(dS, k);
            for (int q = 0; q < (N + 1) * M; ++q) AT(T, q) += al * AT(dT, q);
            for (int i = 0; i < NX; ++i) AT(yi, i) += al * (AT(yi_n, i) - AT(yi, i));
            for (int i = 0; i < N * NX; ++i) AT(yk, i) += al * (AT(yk_n, i) - AT(yk, i));
            for (int cc = 0; cc < nc; ++cc) AT(yt, cc) += al * (AT(yt_n, cc) - AT(yt, cc));
            for (int q = 0; q < (N + 1) * M; ++q) AT(yd, q) += al * (AT(yd_n, q) - AT(yd, q));
            const double az = SC(SC_AZ), ks = 1e10;
            auto zupd = [&](double z, double dz, double sl) {
                double zn = z + az * dz;
                return fmax(fmin(zn, ks * mu / sl), mu / (ks * sl));
            };
            for (int k = 0; k < N; ++k)
                for (int i = 0; i < NU; ++i) {
                    const int q = k * NU + i;
                    const double u = AT(U, q);
                    AT(zl, q) = zupd(AT(zl, q), AT(dzl, q), u - p.umin[i]);
                    AT(zu, q) = zupd(AT(zu, q), AT(dzu, q), p.umax[i] - u);
                }
            if (dm.ns)
                for (int k = 0; k <= N; ++k) AT(zs, k) = zupd(AT(zs, k), AT(dzs, k), AT(S, k));
            for (int q = 0; q < (N + 1) * M; ++q) AT(vt, q) = zupd(AT(vt, q), AT(dvt, q), AT(T, q));
            SC(SC_ITERS) = SC(SC_ITERS) + 1;
            SC(SC_PHASE) = PH_EVAL;
            ph = PH_EVAL;
        } else {
            const double na = 0.5 * al;
            SC(SC_TRIALS) = SC(SC_TRIALS) + 1;
            if (na < SC(SC_AMIN)) {
                SC(SC_STATUS) = NLOT_LS_FAILED;
                SC(SC_PHASE) = PH_DONE;
                ph = PH_DONE;
            } else {
                SC(SC_ALPHA) = na;
            }
        }
    }
    if (ph != PH_DONE) atomicAdd(&ws.cnt[2], 1);
}

__global__ void k_finalize(NlotProblem p, Dims dm, Ws ws, int B, double* Xo, double* Uo, double* So, double* cost,
                           int32_t* status, int32_t* iters) {
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= B) return;
    const int N = dm.N, nx = dm.nx, nu = dm.nu;
    for (int i = 0; i < (N + 1) * nx; ++i) Xo[(size_t)b * (N + 1) * nx + i] = AT(X, i);
    for (int i = 0; i < N * nu; ++i) Uo[(size_t)b * N * nu + i] = AT(U, i);
    if (So)
        for (int k = 0; k <= N; ++k) So[(size_t)b * (N + 1) + k] = dm.ns ? AT(S, k) : 0.0;
    for (int i = 0; i < (N + 1) * nx; ++i) AT(dX, i) = 0;
    for (int i = 0; i < N * nu; ++i) AT(dU, i) = 0;
    for (int k = 0; k <= N; ++k) AT(dS, k) = 0;
    cost[b] = objective(p, dm, ws, b, nullptr, nullptr, nullptr, 0.0);
    int st = (int)SC(SC_STATUS);
    status[b] = st < 0 ? NLOT_MAXITER : st;
    iters[b] = (int)SC(SC_ITERS);
}

// ---------------------------------------------------------------------------------------------
// host driver
// ---------------------------------------------------------------------------------------------
static thread_local NlotSolveStats g_stats;
static bool g_timing = false;

static int validate(const NlotProblem* p, const NlotSolverOptions* o, const NlotMlp* mlp, int64_t B) {
    if (!p || !o) { set_error("null problem/options"); return NLOT_ERR_INVALID; }
    static const int NXS[6] = {4, 4, 3, 5, 4, 7};
    if (p->dynamics < 0 || p->dynamics > 5 || p->nx != NXS[p->dynamics] || p->nu != 2) {
        set_error("dynamics / nx / nu mismatch");
        return NLOT_ERR_INVALID;
    }
    if (p->N < 2 || p->N > 4096 || p->dt <= 0) { set_error("N must be in [2, 4096], dt > 0"); return NLOT_ERR_INVALID; }
    if (p->shape == NLOT_SHAPE_POLYGON && (p->n_body < 1 || p->n_body > MMAX)) {
        set_error("polygon footprint: 1..4 corners"); return NLOT_ERR_INVALID;
    }
    if (p->shape == NLOT_SHAPE_POLYGON && p->nx < 3) { set_error("polygon footprint needs a heading state"); return NLOT_ERR_INVALID; }
    if (p->sdf_kind == NLOT_SDF_MLP && !mlp) { set_error("learned SDF requires an NlotMlp"); return NLOT_ERR_INVALID; }
    if (p->sdf_kind == NLOT_SDF_ANALYTIC && (p->n_obs < 1 || p->n_obs > NLOT_MAX_OBS)) {
        set_error("analytic SDF needs 1..16 obstacles"); return NLOT_ERR_INVALID;
    }
    for (int i = 0; i < p->nu; ++i)
        if (!(p->umin[i] < p->umax[i])) { set_error("control bounds must satisfy min < max"); return NLOT_ERR_INVALID; }
    if (o->max_soc != 0) { set_error("max_soc > 0 is not implemented on the GPU path (DESIGN.md §4)"); return NLOT_ERR_INVALID; }
    if (o->mu_strategy != 0) { set_error("only the monotone mu strategy is implemented"); return NLOT_ERR_INVALID; }
    if (B <= 0 || B > (int64_t)1 << 26) { set_error("B out of range"); return NLOT_ERR_INVALID; }
    return NLOT_OK;
}

template <int DYN>
static int run(const NlotProblem& p, const NlotSolverOptions& o, const NlotMlp* mlp, const double* x0, const double* xg,
               const double* Xinit, double* X, double* U, double* S, double* cost, int32_t* status, int32_t* iters,
               int64_t B, void* workspace, hipStream_t st) {
    const Dims dm = make_dims(p);
    const bool use_mlp = p.sdf_kind == NLOT_SDF_MLP;
    Ws ws = carve(dm, B, use_mlp, workspace);
    const int Bi = (int)B;
    const int tpb = 64, grid = (Bi + tpb - 1) / tpb;
    const int64_t P = (int64_t)dm.ppk * (dm.N + 1);
    g_stats = NlotSolveStats{};
    hipLaunchKernelGGL(k_init_state, dim3(grid), dim3(tpb), 0, st, p, dm, o, ws, x0, xg, Xinit, Bi);
    NLOT_HIP_CHECK(hipGetLastError());
    int* hcnt = nullptr;
    NLOT_HIP_CHECK(hipHostMalloc((void**)&hcnt, 4 * sizeof(int), hipHostMallocDefault));
    hipEvent_t ev[4] = {nullptr, nullptr, nullptr, nullptr};
    if (g_timing && use_mlp)
        for (auto& e : ev) hipEventCreate(&e);
    // upper bound on global steps: every accepted iteration takes at most (1 + backtracks) steps
    const int max_steps = (o.max_iter + 2) * 64;
    int rc = NLOT_OK;
    for (int step = 0; step < max_steps; ++step) {
        NLOT_HIP_CHECK(hipMemsetAsync(ws.cnt, 0, 4 * sizeof(int), st));
        if (use_mlp) {
            hipLaunchKernelGGL(k_points, dim3(grid), dim3(tpb), 0, st, p, dm, ws, Bi, 0);
            MlpOut mo{};
            const int64_t plane = P * B;
            mo.val = ws.mo; mo.gx = ws.mo + plane; mo.gy = ws.mo + 2 * plane; mo.hxx = ws.mo + 3 * plane;
            mo.hxy = ws.mo + 4 * plane; mo.hyx = mo.hxy; mo.hyy = ws.mo + 5 * plane;
            mo.sv = mo.sg = mo.sh = 1;
            if (ev[0]) hipEventRecord(ev[0], st);
            rc = launch_mlp_strided(mlp->dev, ws.pts, B, ws.cnt + 0, (int)P, B, nullptr, mo, true, st);
            if (rc) break;
            if (ev[0]) hipEventRecord(ev[1], st);
            hipLaunchKernelGGL(k_iterate<DYN>, dim3(grid), dim3(tpb), 0, st, p, dm, o, ws, Bi, x0, xg);
            hipLaunchKernelGGL(k_points, dim3(grid), dim3(tpb), 0, st, p, dm, ws, Bi, 1);
            if (ev[0]) hipEventRecord(ev[2], st);
            rc = launch_mlp_strided(mlp->dev, ws.pts, B, ws.cnt + 1, (int)P, B, nullptr, mo, false, st);
            if (rc) break;
            if (ev[0]) hipEventRecord(ev[3], st);
            g_stats.mlp_full_launches++;
            g_stats.mlp_value_launches++;
        } else {
            hipLaunchKernelGGL(k_iterate<DYN>, dim3(grid), dim3(tpb), 0, st, p, dm, o, ws, Bi, x0, xg);
        }
        hipLaunchKernelGGL(k_accept<DYN>, dim3(grid), dim3(tpb), 0, st, p, dm, o, ws, Bi, x0, xg);
        NLOT_HIP_CHECK(hipGetLastError());
        NLOT_HIP_CHECK(hipMemcpyAsync(hcnt, ws.cnt, 4 * sizeof(int), hipMemcpyDeviceToHost, st));
        NLOT_HIP_CHECK(hipStreamSynchronize(st));
        g_stats.iterations = step + 1;
        g_stats.mlp_points_full += (int64_t)hcnt[0] * P;
        g_stats.mlp_points_value += (int64_t)hcnt[1] * P;
        if (ev[0]) {
            float a = 0, c = 0;
            hipEventElapsedTime(&a, ev[0], ev[1]);
            hipEventElapsedTime(&c, ev[2], ev[3]);
            g_stats.mlp_full_ms += a;
            g_stats.mlp_value_ms += c;
        }
        if (hcnt[2] == 0) break;
    }
    for (auto& e : ev)
        if (e) hipEventDestroy(e);
    hipHostFree(hcnt);
    if (rc) return rc;
    hipLaunchKernelGGL(k_finalize, dim3(grid), dim3(tpb), 0, st, p, dm, ws, Bi, X, U, S, cost, status, iters);
    NLOT_HIP_CHECK(hipGetLastError());
    NLOT_HIP_CHECK(hipStreamSynchronize(st));
    return NLOT_OK;
}

}  // namespace nlot

extern "C" size_t nlot_solve_workspace_size(const NlotProblem* p, int64_t B) {
    if (!p) return 0;
    nlot::Dims d = nlot::make_dims(*p);
    return nlot::ws_bytes(d, B, p->sdf_kind == NLOT_SDF_MLP);
}

extern "C" int32_t nlot_solve_batch(const NlotProblem* p, const NlotSolverOptions* o, const NlotMlp* mlp,
                                    const double* x0, const double* xg, const double* Xinit, double* X, double* U,
                                    double* S, double* cost, int32_t* status, int32_t* iters, int64_t B,
                                    void* workspace, size_t wbytes, void* stream) {
    using namespace nlot;
    int rc = validate(p, o, mlp, B);
    if (rc) return rc;
    if (!x0 || !xg || !X || !U || !cost || !status || !iters || !workspace) {
        set_error("nlot_solve_batch: null pointer");
        return NLOT_ERR_INVALID;
    }
    if (wbytes < nlot_solve_workspace_size(p, B)) {
        set_error("nlot_solve_batch: workspace too small");
        return NLOT_ERR_WORKSPACE;
    }
    hipStream_t st = (hipStream_t)stream;
    switch (p->dynamics) {
    case NLOT_POINT_1ST: return run<NLOT_POINT_1ST>(*p, *o, mlp, x0, xg, Xinit, X, U, S, cost, status, iters, B, workspace, st);
    case NLOT_POINT_2ND: return run<NLOT_POINT_2ND>(*p, *o, mlp, x0, xg, Xinit, X, U, S, cost, status, iters, B, workspace, st);
    case NLOT_UNICYCLE: return run<NLOT_UNICYCLE>(*p, *o, mlp, x0, xg, Xinit, X, U, S, cost, status, iters, B, workspace, st);
    case NLOT_UNICYCLE_2ND: return run<NLOT_UNICYCLE_2ND>(*p, *o, mlp, x0, xg, Xinit, X, U, S, cost, status, iters, B, workspace, st);
    case NLOT_ACKERMANN: return run<NLOT_ACKERMANN>(*p, *o, mlp, x0, xg, Xinit, X, U, S, cost, status, iters, B, workspace, st);
    case NLOT_ACKERMANN_2ND: return run<NLOT_ACKERMANN_2ND>(*p, *o, mlp, x0, xg, Xinit, X, U, S, cost, status, iters, B, workspace, st);
    }
    set_error("unknown dynamics");
    return NLOT_ERR_INVALID;
}

extern "C" void nlot_set_timing(int32_t en) { nlot::g_timing = en != 0; }
extern "C" void nlot_last_stats(NlotSolveStats* out) {
    if (out) *out = nlot::g_stats;
}
