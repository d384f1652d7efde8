/*
 * nlot_oracle.c — CPU restatement of the reference's NLP hot path.  TEST INFRASTRUCTURE ONLY.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg load this library (as the
 * checker / the timed CPU baseline).  The product (libnlot.so, nlotrajectories_amd/) never links
 * or calls it.
 *
 * What is restated (file:line under /root/reference):
 *   - NLP definition of RunBenchmark.run                      src/nlotrajectories/core/runner.py:44-108
 *       decision variables X, U, slack                         runner.py:46-47, 66-69
 *       start / terminal equalities (enforce_heading)          runner.py:50-56
 *       explicit-Euler dynamics defects                        runner.py:59-64
 *       per-knot SDF constraints                               runner.py:73-77 -> geometry.py:63-67,107-117
 *       cost: path length + slack + smooth penalties           runner.py:80-98
 *       control bounds                                          runner.py:101-103
 *   - dynamics f(x,u), 6 models                                core/dynamics.py:33-148
 *   - footprint corners + soft-min                              core/geometry.py:78-83,125-144; core/utils.py:18-33
 *   - analytic SDFs (circle, smooth square, union)              core/sdf/casadi.py:33-41,69-118,385-386
 *   - learned SDF (FourierMLP / naive MLP, fp32 like libtorch)  core/nn_architectures.py:30-72; gen/nn_sdf.cpp:57-104
 *   - IPOPT (external dependency, CasADi 3.7.0's bundled IPOPT, poetry.lock:90-91) is restated from its
 *     published algorithm (Waechter & Biegler 2006): primal-dual barrier method, monotone and adaptive
 *     (quality-function oracle) mu updates, fraction-to-boundary rule, inertia-corrected Newton step, filter
 *     line search with second-order corrections, watchdog, tiny-step rule, filter reset, soft restoration and
 *     the feasibility restoration phase (MinC_1Nrm); the bounds as Opti's constraint rows (general_bounds,
 *     runner.py:67-69,101-103) or as variable bounds.  Deviations are listed in DESIGN.md §4.
 *
 * Derivatives use a small second-order forward-mode "jet" (value, gradient, Hessian), so this file is
 * an independent derivation from the hand-written derivatives of the HIP kernels.
 */
#include <float.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../include/nlot.h"

#ifdef _OPENMP
#include <omp.h>
#endif

/* ============================================================================================ */
/* Second-order jets                                                                           */
/* ============================================================================================ */
#define JD 10
#define JH (JD * (JD + 1) / 2)
typedef struct {
    int n;
    double v;
    double g[JD];
    double h[JH]; /* lower triangle, row i col j<=i at i*(i+1)/2+j */
} jet;

static inline int hix(int i, int j) { return i >= j ? i * (i + 1) / 2 + j : j * (j + 1) / 2 + i; }

static jet jconst(int n, double c) {
    jet r;
    memset(&r, 0, sizeof r);
    r.n = n;
    r.v = c;
    return r;
}
static jet jvar(int n, double v, int i) {
    jet r = jconst(n, v);
    r.g[i] = 1.0;
    return r;
}
static jet jadd(jet a, jet b) {
    jet r = a;
    r.v += b.v;
    for (int i = 0; i < a.n; ++i) r.g[i] += b.g[i];
    for (int i = 0; i < a.n * (a.n + 1) / 2; ++i) r.h[i] += b.h[i];
    return r;
}
static jet jscale(jet a, double c) {
    jet r = a;
    r.v *= c;
    for (int i = 0; i < a.n; ++i) r.g[i] *= c;
    for (int i = 0; i < a.n * (a.n + 1) / 2; ++i) r.h[i] *= c;
    return r;
}
static jet jsub(jet a, jet b) { return jadd(a, jscale(b, -1.0)); }
static jet jaddc(jet a, double c) {
    a.v += c;
    return a;
}
static jet jmul(jet a, jet b) {
    jet r = jconst(a.n, a.v * b.v);
    for (int i = 0; i < a.n; ++i) r.g[i] = a.g[i] * b.v + a.v * b.g[i];
    for (int i = 0; i < a.n; ++i)
        for (int j = 0; j <= i; ++j) {
            int q = hix(i, j);
            r.h[q] = a.h[q] * b.v + a.v * b.h[q] + a.g[i] * b.g[j] + a.g[j] * b.g[i];
        }
    return r;
}
/* r = f(a) with f(a.v)=f0, f'=f1, f''=f2 */
static jet junary(jet a, double f0, double f1, double f2) {
    jet r = jconst(a.n, f0);
    for (int i = 0; i < a.n; ++i) r.g[i] = f1 * a.g[i];
    for (int i = 0; i < a.n; ++i)
        for (int j = 0; j <= i; ++j) {
            int q = hix(i, j);
            r.h[q] = f1 * a.h[q] + f2 * a.g[i] * a.g[j];
        }
    return r;
}
static jet jsin(jet a) { return junary(a, sin(a.v), cos(a.v), -sin(a.v)); }
static jet jcos(jet a) { return junary(a, cos(a.v), -sin(a.v), -cos(a.v)); }
static jet jtan(jet a) {
    double t = tan(a.v), s2 = 1.0 + t * t;
    return junary(a, t, s2, 2.0 * t * s2);
}
static jet jexp(jet a) {
    double e = exp(a.v);
    return junary(a, e, e, e);
}
static jet jlog(jet a) { return junary(a, log(a.v), 1.0 / a.v, -1.0 / (a.v * a.v)); }
static jet jsqrt(jet a) {
    double s = sqrt(a.v);
    return junary(a, s, 0.5 / s, -0.25 / (s * a.v));
}
static jet jrecip(jet a) { return junary(a, 1.0 / a.v, -1.0 / (a.v * a.v), 2.0 / (a.v * a.v * a.v)); }
static jet jdiv(jet a, jet b) { return jmul(a, jrecip(b)); }
static jet jsq(jet a) { return jmul(a, a); }

/* phi(cx(z), cy(z)) given phi's value / gradient / Hessian in (cx, cy) */
static jet jcompose2(double f, const double g[2], const double H[3] /*xx,xy,yy*/, jet cx, jet cy) {
    jet r = jconst(cx.n, f);
    for (int i = 0; i < cx.n; ++i) r.g[i] = g[0] * cx.g[i] + g[1] * cy.g[i];
    for (int i = 0; i < cx.n; ++i)
        for (int j = 0; j <= i; ++j) {
            int q = hix(i, j);
            r.h[q] = g[0] * cx.h[q] + g[1] * cy.h[q] + H[0] * cx.g[i] * cx.g[j] +
                     H[1] * (cx.g[i] * cy.g[j] + cy.g[i] * cx.g[j]) + H[2] * cy.g[i] * cy.g[j];
        }
    return r;
}

/* ============================================================================================ */
/* Learned SDF — fp32 like the reference's libtorch evaluation (gen/nn_sdf.cpp:57-104)           */
/* ============================================================================================ */
/* out: [0]=f [1..2]=lam*grad [3..5]=lam*hess (xx,xy,yy).  lam scales the adjoint seed
 * (adj1 / jac_adj1, gen/nn_sdf.cpp:79-104); lam = 1 gives jac_nn_sdf.  want = 0: value only. */
#define ORACLE_ACT_SOFTPLUS 90 /* not in the ABI: a diagnostic of the oracle (ReLU-kink experiment) */
/* s, s', s'' of a smooth hidden activation (core/nn_architectures.py:47-52; SineLayer :8-26 with omega_0) */
static void oracle_act3(int act, float omega, float z, float* s, float* d1, float* d2) {
    switch (act) {
        case NLOT_ACT_TANH: *s = tanhf(z); *d1 = 1.f - *s * *s; *d2 = -2.f * *s * *d1; break;
        case NLOT_ACT_SIGMOID: *s = 1.f / (1.f + expf(-z)); *d1 = *s * (1.f - *s); *d2 = *d1 * (1.f - 2.f * *s); break;
        case NLOT_ACT_LEAKY_RELU: *s = z > 0.f ? z : 0.01f * z; *d1 = z > 0.f ? 1.f : 0.01f; *d2 = 0.f; break;
        case NLOT_ACT_SINE: {
            const float u = omega * z;
            *s = sinf(u); *d1 = omega * cosf(u); *d2 = -omega * omega * *s;
            break;
        }
        case ORACLE_ACT_SOFTPLUS: { /* diagnostic only (scripts/ipopt_variants.py): ReLU smoothed, beta from env */
            static float beta = 0.f;
            if (beta == 0.f) beta = getenv("NLOT_ORACLE_SOFTPLUS_BETA") ? (float)atof(getenv("NLOT_ORACLE_SOFTPLUS_BETA")) : 100.f;
            const float t = beta * z, e = expf(-fabsf(t)), sg = t >= 0.f ? 1.f / (1.f + e) : e / (1.f + e);
            *s = fmaxf(z, 0.f) + log1pf(e) / beta;
            *d1 = sg;
            *d2 = beta * sg * (1.f - sg);
            break;
        }
        default: *s = z > 0.f ? z : 0.f; *d1 = z > 0.f ? 1.f : 0.f; *d2 = 0.f;
    }
}

/* Smooth nets: value, gradient and Hessian carried forward through every layer (the Hessian has a term
 * from each activation), 6 components per hidden unit: a, a_x, a_y, a_xx, a_xy, a_yy. */
static void oracle_mlp_point_smooth(const NlotMlpDesc* m, float px, float py, float lam, int want, float out[6]) {
    enum { HM = 256 };
    const int H = m->hidden;
    float a[6][HM], z[6][HM];
    for (int k = 0; k < H; ++k) {
        const float ax = m->A[k], ay = m->A[H + k];
        const float zz = fmaf(py, ay, px * ax) + m->b0[k];
        float s, d1, d2;
        if (m->in_kind == NLOT_MLP_IN_FOURIER) {
            s = cosf(zz) * m->fourier_scale;
            d1 = -m->fourier_scale * sinf(zz);
            d2 = -m->fourier_scale * cosf(zz);
        } else {
            oracle_act3(m->act, m->fourier_scale, zz, &s, &d1, &d2);
        }
        a[0][k] = s;
        a[1][k] = d1 * ax;
        a[2][k] = d1 * ay;
        a[3][k] = d2 * ax * ax;
        a[4][k] = d2 * ax * ay;
        a[5][k] = d2 * ay * ay;
    }
    for (int l = 0; l < m->n_hidden; ++l) {
        const float* W = m->W + (size_t)l * H * H;
        const float* b = m->b + (size_t)l * H;
        for (int j = 0; j < H; ++j)
            for (int c = 0; c < 6; ++c) {
                float t = 0.f;
                for (int k = 0; k < H; ++k) t = fmaf(W[(size_t)j * H + k], a[c][k], t);
                z[c][j] = t;
            }
        for (int j = 0; j < H; ++j) {
            float s, d1, d2;
            oracle_act3(m->act, m->fourier_scale, z[0][j] + b[j], &s, &d1, &d2);
            a[0][j] = s;
            a[1][j] = d1 * z[1][j];
            a[2][j] = d1 * z[2][j];
            a[3][j] = d2 * z[1][j] * z[1][j] + d1 * z[3][j];
            a[4][j] = d2 * z[1][j] * z[2][j] + d1 * z[4][j];
            a[5][j] = d2 * z[2][j] * z[2][j] + d1 * z[5][j];
        }
    }
    float o[6] = {0, 0, 0, 0, 0, 0};
    for (int c = 0; c < 6; ++c)
        for (int j = 0; j < H; ++j) o[c] = fmaf(m->w_out[j], a[c][j], o[c]);
    out[0] = o[0] + m->b_out;
    for (int c = 1; c < 6; ++c) out[c] = want ? lam * o[c] : 0.f;
}

/* NLOT_ORACLE_MLP_REV=1 (test infrastructure, tests/outcomes.py): every fp32 dot product of the ReLU net (hidden
 * layers, output layer, reverse sweep, input-layer contraction) accumulates in the reverse index order.  The result
 * differs from the default only by fp32 rounding: the same kind of difference the GPU's split-bf16 MFMA sums make, so
 * a solve whose outcome changes under it is not reproducible at the GPU's arithmetic.  Read per call (toggled
 * between whole batches by the Python side).  NLOT_ORACLE_MLP_REV=v >= 2: the index order i -> (i * m_v) mod H with
 * an odd multiplier m_v (a permutation for H a power of two): more samples of the same kind of difference
 * (tests/test_pinned_iterates_gpu.py).  v >= 8 (round 6): a pseudo-random permutation of the index seeded by v
 * (Fisher-Yates over a splitmix64 stream), the same one for every sum of the call. */
static int mlp_rev(void) {
    const char* e = getenv("NLOT_ORACLE_MLP_REV");
    return e ? atoi(e) : 0;
}
static int mlp_perm_mult(int v) {
    static const int m[8] = {1, 1, 3, 5, 7, 11, 13, 17};
    return m[v & 7];
}
/* NLOT_ORACLE_MLP_BIAS=b (test infrastructure, round 6): b added to the net's fp32 value: a model of the split-bf16
 * GPU net's measured offset against every fp32 summation order (-5e-9 / -4e-9 on the artefact / benchmark-6 nets,
 * scripts/net_bias_probe.py), for the fixture's pinned iterations */
static float mlp_bias(void) {
    const char* e = getenv("NLOT_ORACLE_MLP_BIAS");
    return e ? (float)atof(e) : 0.f;
}
static void mlp_perm_random(int v, int H, int* perm) {
    uint64_t x = 0x9E3779B97F4A7C15ull * (uint64_t)(v + 1);
    for (int i = 0; i < H; ++i) perm[i] = i;
    for (int i = H - 1; i > 0; --i) {
        x += 0x9E3779B97F4A7C15ull;
        uint64_t z = x;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        z ^= z >> 31;
        const int j = (int)(z % (uint64_t)(i + 1));
        const int t = perm[i];
        perm[i] = perm[j];
        perm[j] = t;
    }
}

void oracle_mlp_point(const NlotMlpDesc* m, float px, float py, float lam, int want, float out[6]) {
    enum { HM = 256, LM = 8 };
    const int H = m->hidden;
    const int rv = mlp_rev();
    const int rvm = mlp_perm_mult(rv);
    int perm[HM];
    if (rv >= 8) mlp_perm_random(rv, H, perm);
#define RIX(i) (rv == 0 ? (i) : rv == 1 ? H - 1 - (i) : rv >= 8 ? perm[i] : ((i) * rvm) % H)
    if (m->act != NLOT_ACT_RELU) {
        oracle_mlp_point_smooth(m, px, py, lam, want, out);
        return;
    }
    float z0[HM], h[HM], hn[HM];
    unsigned char mask[LM + 1][HM];
    for (int k = 0; k < H; ++k) {
        /* p @ A + b0  (torch.mm then add, graph ___torch_mangle_0.py) */
        float z = fmaf(py, m->A[H + k], px * m->A[k]) + m->b0[k];
        z0[k] = z;
        if (m->in_kind == NLOT_MLP_IN_FOURIER) {
            /* nn_architectures.py:38.  The fp32 cos as the fp64 cos rounded to fp32: correctly rounded in all but
             * ~2^-28 of the arguments, so any fp32 libm (libtorch's included) is within an ulp of it, and the GPU's
             * NLOT_MLP_ARITH_SEQ net forms the same value (round 6; cosf of glibc and of the device differ in the last
             * bit on ~60 % of the artefact's arguments) */
            h[k] = (float)cos((double)z) * m->fourier_scale;
            mask[0][k] = 1;
        } else {
            mask[0][k] = z > 0.f;
            h[k] = z > 0.f ? z : 0.f;
        }
    }
    for (int l = 0; l < m->n_hidden; ++l) {
        const float* W = m->W + (size_t)l * H * H;
        const float* b = m->b + (size_t)l * H;
        for (int j = 0; j < H; ++j) {
            float a = 0.f;
            for (int kq = 0; kq < H; ++kq) {
                const int k = RIX(kq);
                a = fmaf(W[(size_t)j * H + k], h[k], a);
            }
            a += b[j];
            mask[l + 1][j] = a > 0.f;
            hn[j] = a > 0.f ? a : 0.f;
        }
        memcpy(h, hn, sizeof(float) * H);
    }
    float f = 0.f;
    for (int jq = 0; jq < H; ++jq) f = fmaf(m->w_out[RIX(jq)], h[RIX(jq)], f);
    out[0] = f + m->b_out;
    if (mlp_bias() != 0.f) out[0] += mlp_bias();
    out[1] = out[2] = out[3] = out[4] = out[5] = 0.f;
    if (!want) return;
    /* reverse sweep: delta = d f / d h_l */
    float d[HM], dn[HM];
    for (int j = 0; j < H; ++j) d[j] = lam * m->w_out[j];
    for (int l = m->n_hidden - 1; l >= 0; --l) {
        const float* W = m->W + (size_t)l * H * H;
        for (int j = 0; j < H; ++j) d[j] = mask[l + 1][j] ? d[j] : 0.f;
        for (int k = 0; k < H; ++k) dn[k] = 0.f;
        for (int jq = 0; jq < H; ++jq) {
            const int j = RIX(jq);
            for (int k = 0; k < H; ++k) dn[k] = fmaf(W[(size_t)j * H + k], d[j], dn[k]);
        }
        memcpy(d, dn, sizeof(float) * H);
    }
    float gx = 0.f, gy = 0.f, hxx = 0.f, hxy = 0.f, hyy = 0.f;
    for (int kq = 0; kq < H; ++kq) {
        const int k = RIX(kq);
        float ax = m->A[k], ay = m->A[H + k], dz, c2;
        if (m->in_kind == NLOT_MLP_IN_FOURIER) {
            dz = d[k] * (-m->fourier_scale * (float)sin((double)z0[k]));
            c2 = d[k] * (-m->fourier_scale * (float)cos((double)z0[k]));
        } else {
            dz = mask[0][k] ? d[k] : 0.f;
            c2 = 0.f; /* ReLU input layer: piecewise linear, Hessian 0 a.e. */
        }
        gx = fmaf(ax, dz, gx);
        gy = fmaf(ay, dz, gy);
        hxx = fmaf(ax * ax, c2, hxx);
        hxy = fmaf(ax * ay, c2, hxy);
        hyy = fmaf(ay * ay, c2, hyy);
    }
    out[1] = gx;
    out[2] = gy;
    out[3] = hxx;
    out[4] = hxy;
    out[5] = hyy;
#undef RIX
}

/* Batched form of the nn_sdf family (same argument meaning as nlot_sdf_mlp_eval, host buffers). */
void oracle_mlp_eval(const NlotMlpDesc* m, const float* pts, long P, float* val, float* grad,
                     const float* lam, float* hess) {
    int want = (grad != NULL) || (hess != NULL);
#pragma omp parallel for schedule(static)
    for (long i = 0; i < P; ++i) {
        float o[6];
        oracle_mlp_point(m, pts[2 * i], pts[2 * i + 1], lam ? lam[i] : 1.f, want, o);
        val[i] = o[0];
        if (grad) {
            grad[2 * i] = o[1];
            grad[2 * i + 1] = o[2];
        }
        if (hess) {
            hess[4 * i + 0] = o[3];
            hess[4 * i + 1] = o[4];
            hess[4 * i + 2] = o[4];
            hess[4 * i + 3] = o[5];
        }
    }
}

/* ============================================================================================ */
/* Analytic SDFs (core/sdf/casadi.py), in 2-D jets over the point (x, y): value, gradient, Hessian       */
/* ============================================================================================ */
typedef struct {
    double v, gx, gy, hxx, hxy, hyy;
} j2;
static j2 k2(double c) { j2 r = {c, 0, 0, 0, 0, 0}; return r; }
static j2 add2(j2 a, j2 b) { j2 r = {a.v + b.v, a.gx + b.gx, a.gy + b.gy, a.hxx + b.hxx, a.hxy + b.hxy, a.hyy + b.hyy}; return r; }
static j2 sub2(j2 a, j2 b) { j2 r = {a.v - b.v, a.gx - b.gx, a.gy - b.gy, a.hxx - b.hxx, a.hxy - b.hxy, a.hyy - b.hyy}; return r; }
static j2 addc2(j2 a, double c) { a.v += c; return a; }
static j2 sc2(double c, j2 a) { j2 r = {c * a.v, c * a.gx, c * a.gy, c * a.hxx, c * a.hxy, c * a.hyy}; return r; }
static j2 divc2(j2 a, double c) { j2 r = {a.v / c, a.gx / c, a.gy / c, a.hxx / c, a.hxy / c, a.hyy / c}; return r; }
static j2 mul2(j2 a, j2 b) {
    j2 r = {a.v * b.v, a.gx * b.v + a.v * b.gx, a.gy * b.v + a.v * b.gy, a.hxx * b.v + a.v * b.hxx + 2 * a.gx * b.gx,
            a.hxy * b.v + a.v * b.hxy + a.gx * b.gy + a.gy * b.gx, a.hyy * b.v + a.v * b.hyy + 2 * a.gy * b.gy};
    return r;
}
static j2 chain2(j2 a, double f0, double f1, double f2) {
    j2 r = {f0, f1 * a.gx, f1 * a.gy, f1 * a.hxx + f2 * a.gx * a.gx, f1 * a.hxy + f2 * a.gx * a.gy,
            f1 * a.hyy + f2 * a.gy * a.gy};
    return r;
}
static j2 sqrt2(j2 a) { double q = sqrt(a.v); return chain2(a, q, 0.5 / q, -0.25 / (q * a.v)); }
static j2 exp2_(j2 a) { double e = exp(a.v); return chain2(a, e, e, e); }
static j2 log2_(j2 a) { return chain2(a, log(a.v), 1.0 / a.v, -1.0 / (a.v * a.v)); }
static j2 tanh2(j2 a) { double t = tanh(a.v), d = 1 - t * t; return chain2(a, t, d, -2 * t * d); }

static j2 sdf_circle(const NlotObstacle* o, j2 x, j2 y) { /* casadi.py:33-41 */
    j2 dx = addc2(x, -o->cx), dy = addc2(y, -o->cy);
    return addc2(sqrt2(add2(mul2(dx, dx), mul2(dy, dy))), -(o->size + o->margin));
}
/* SquareObstacle soft helpers casadi.py:81-105 (soft_abs eps 1e-6); TrapezoidObstacle's casadi.py:288-312 (1e-8) */
static j2 sabs2(j2 v, double eps) { return sqrt2(addc2(mul2(v, v), eps)); }
static j2 smax2(j2 a, j2 b, double eps) { return sc2(0.5, add2(add2(a, b), sabs2(sub2(a, b), eps))); }
static j2 smin2(j2 a, j2 b, double eps) { return sc2(0.5, sub2(add2(a, b), sabs2(sub2(a, b), eps))); }
static j2 sdf_square(const NlotObstacle* o, j2 x, j2 y) { /* casadi.py:69-118 */
    double half = o->size / 2 + o->margin;
    j2 dx = sabs2(addc2(x, -o->cx), 1e-6), dy = sabs2(addc2(y, -o->cy), 1e-6);
    j2 d_x = addc2(dx, -half), d_y = addc2(dy, -half), zero = k2(0.0);
    j2 dxo = smax2(d_x, zero, 1e-6), dyo = smax2(d_y, zero, 1e-6);
    j2 outside = sqrt2(add2(mul2(dxo, dxo), mul2(dyo, dyo)));
    j2 inside = smin2(smax2(d_x, d_y, 1e-6), zero, 1e-6);
    return add2(outside, inside);
}
/* soft_min, core/utils.py:18-33 (no max-shift, exactly as written): sum of exp(-alpha v_i) in order, then
   -1/alpha log */
static j2 soft_min_fin(j2 sum, double alpha) { return sc2(-1.0 / alpha, log2_(sum)); }
/* PolygonObstacle.approximated_sdf casadi.py:150-186: soft_min of the distances to the edge segments (hard
   clamp of the projection parameter), signed by tanh(100 (x - cx)(y - cy)) about the centroid */
static j2 sdf_polygon(const NlotProblem* p, const NlotObstacle* o, j2 x, j2 y) {
    const double(*V)[2] = p->verts + o->v0;
    const double a = p->softmin_alpha;
    j2 sum = k2(0.0);
    for (int e = 0; e < o->nv; ++e) {
        const int e1 = e + 1 < o->nv ? e + 1 : 0;
        const double x0 = V[e][0], y0 = V[e][1], dx = V[e1][0] - x0, dy = V[e1][1] - y0;
        const double seg = dx * dx + dy * dy + 1e-6;
        j2 traw = divc2(add2(sc2(dx, addc2(x, -x0)), sc2(dy, addc2(y, -y0))), seg);
        j2 t = traw.v < 0.0 ? k2(0.0) : traw.v > 1.0 ? k2(1.0) : traw;
        j2 qx = sub2(x, addc2(sc2(dx, t), x0)), qy = sub2(y, addc2(sc2(dy, t), y0));
        sum = add2(sum, exp2_(sc2(-a, sqrt2(add2(mul2(qx, qx), mul2(qy, qy))))));
    }
    j2 md = soft_min_fin(sum, a);
    j2 sign = tanh2(sc2(100.0, mul2(addc2(x, -o->cx), addc2(y, -o->cy))));
    return addc2(mul2(sign, md), -o->margin);
}
/* TrapezoidObstacle.approximated_sdf casadi.py:317-374 */
static j2 sdf_trapezoid(const NlotProblem* p, const NlotObstacle* o, j2 x, j2 y) {
    const double(*V)[2] = p->verts + o->v0;
    const int nv = o->nv;
    j2 zero = k2(0.0), one = k2(1.0), inner_max = zero, outside = zero;
    for (int e = 0; e < nv; ++e) { /* half-plane distances, soft max folded left to right */
        const int e1 = e + 1 < nv ? e + 1 : 0;
        const double x0 = V[e][0], y0 = V[e][1], ex = V[e1][0] - x0, ey = V[e1][1] - y0;
        const double nl = sqrt(ey * ey + ex * ex + 1e-6), nx = ey / nl, ny = -ex / nl;
        j2 d = addc2(add2(sc2(nx, addc2(x, -x0)), sc2(ny, addc2(y, -y0))), -o->margin);
        inner_max = e == 0 ? d : smax2(inner_max, d, 1e-8);
    }
    j2 inside = smin2(inner_max, zero, 1e-8);
    for (int e = 0; e < nv; ++e) { /* distances to the segments, smooth clamp, soft min folded */
        const int e1 = e + 1 < nv ? e + 1 : 0;
        const double x0 = V[e][0], y0 = V[e][1], ex = V[e1][0] - x0, ey = V[e1][1] - y0;
        const double seg = ex * ex + ey * ey + 1e-6;
        j2 t = smin2(one, smax2(zero, divc2(add2(sc2(ex, addc2(x, -x0)), sc2(ey, addc2(y, -y0))), seg), 1e-8), 1e-8);
        j2 qx = sub2(x, addc2(sc2(ex, t), x0)), qy = sub2(y, addc2(sc2(ey, t), y0));
        j2 dist = sqrt2(addc2(add2(mul2(qx, qx), mul2(qy, qy)), 1e-6));
        outside = e == 0 ? dist : smin2(outside, dist, 1e-8);
    }
    return addc2(add2(outside, inside), -o->margin);
}
static j2 sdf_prim(const NlotProblem* p, const NlotObstacle* o, j2 x, j2 y) {
    switch (o->type) {
    case NLOT_OBS_CIRCLE: return sdf_circle(o, x, y);
    case NLOT_OBS_SQUARE: return sdf_square(o, x, y);
    case NLOT_OBS_POLYGON: return sdf_polygon(p, o, x, y);
    default: return sdf_trapezoid(p, o, x, y);
    }
}
/* MultiObstacle.approximated_sdf casadi.py:385-386 — soft_min even for one obstacle; a group (a MultiObstacle
   in the scene: ConvexEllipticRing / ConvexSObstacle) is soft_min'ed first and enters as one term.  Evaluated
   in (x, y) and composed with the corner's jet (as the GPU's 2-D hyper-duals). */
static jet sdf_analytic(const NlotProblem* p, jet cx, jet cy) {
    const double a = p->softmin_alpha;
    j2 x = {cx.v, 1, 0, 0, 0, 0}, y = {cy.v, 0, 1, 0, 0, 0}, sum = k2(0.0);
    for (int i = 0; i < p->n_obs;) {
        j2 v;
        if (p->obs[i].group < 0) {
            v = sdf_prim(p, &p->obs[i], x, y);
            ++i;
        } else {
            const int g = p->obs[i].group;
            j2 in = k2(0.0);
            for (; i < p->n_obs && p->obs[i].group == g; ++i) in = add2(in, exp2_(sc2(-a, sdf_prim(p, &p->obs[i], x, y))));
            v = soft_min_fin(in, a);
        }
        sum = add2(sum, exp2_(sc2(-a, v)));
    }
    j2 s = soft_min_fin(sum, a);
    double g[2] = {s.gx, s.gy}, H[3] = {s.hxx, s.hxy, s.hyy};
    return jcompose2(s.v, g, H, cx, cy);
}

/* soft_min, core/utils.py:18-33, over jets of any dimension (the footprint's corner soft_min) */
static jet soft_min_j(const jet* a, int n, double alpha) {
    jet s = jconst(a[0].n, 0.0);
    for (int i = 0; i < n; ++i) s = jadd(s, jexp(jscale(a[i], -alpha)));
    return jscale(jlog(s), -1.0 / alpha);
}

/* SDF of the scene at world point (cx, cy) given as jets (any dimension). */
static jet sdf_point(const NlotProblem* p, const NlotMlpDesc* m, jet cx, jet cy, int want) {
    if (p->sdf_kind == NLOT_SDF_ANALYTIC) return sdf_analytic(p, cx, cy);
    float o[6];
    /* NNObstacle.approximated_sdf -> l4casadi forward: CasADi double cast to float (gen/nn_sdf.cpp) */
    oracle_mlp_point(m, (float)cx.v, (float)cy.v, 1.f, want, o);
    double g[2] = {o[1], o[2]}, H[3] = {o[3], o[4], o[5]};
    if (!want) return jconst(cx.n, (double)o[0]);
    return jcompose2((double)o[0], g, H, cx, cy);
}

/* Batched scene SDF at points (value, gradient, Hessian); out [P][6]. */
void oracle_sdf_eval(const NlotProblem* p, const NlotMlpDesc* m, const double* pts, long P, double* out) {
    for (long i = 0; i < P; ++i) {
        jet x = jvar(2, pts[2 * i], 0), y = jvar(2, pts[2 * i + 1], 1);
        jet s = sdf_point(p, m, x, y, 1);
        out[6 * i + 0] = s.v;
        out[6 * i + 1] = s.g[0];
        out[6 * i + 2] = s.g[1];
        out[6 * i + 3] = s.h[hix(0, 0)];
        out[6 * i + 4] = s.h[hix(1, 0)];
        out[6 * i + 5] = s.h[hix(1, 1)];
    }
}

double oracle_soft_min(const double* v, int n, double alpha) {
    jet a[64];
    for (int i = 0; i < n; ++i) a[i] = jconst(1, v[i]);
    return soft_min_j(a, n, alpha).v;
}

/* ============================================================================================ */
/* Dynamics (core/dynamics.py)                                                                  */
/* ============================================================================================ */
/* f(x, u) as jets over z = (x, u); n = nx + nu */
static void dyn_f(const NlotProblem* p, const jet* x, const jet* u, jet* f) {
    int n = x[0].n;
    switch (p->dynamics) {
    case NLOT_POINT_1ST: /* dynamics.py:40-41 */
        f[0] = u[0];
        f[1] = u[1];
        f[2] = jconst(n, 0.0);
        f[3] = jconst(n, 0.0);
        break;
    case NLOT_POINT_2ND: /* dynamics.py:51-56 */
        f[0] = x[2];
        f[1] = x[3];
        f[2] = u[0];
        f[3] = u[1];
        break;
    case NLOT_UNICYCLE: /* dynamics.py:66-73 */
        f[0] = jmul(u[0], jcos(x[2]));
        f[1] = jmul(u[0], jsin(x[2]));
        f[2] = u[1];
        break;
    case NLOT_UNICYCLE_2ND: /* dynamics.py:83-96 */
        f[0] = jmul(x[3], jcos(x[2]));
        f[1] = jmul(x[3], jsin(x[2]));
        f[2] = x[4];
        f[3] = u[0];
        f[4] = u[1];
        break;
    case NLOT_ACKERMANN: /* dynamics.py:109-118 */
        f[0] = jmul(u[0], jcos(x[2]));
        f[1] = jmul(u[0], jsin(x[2]));
        f[2] = jscale(jmul(u[0], jtan(x[3])), 1.0 / p->wheelbase);
        f[3] = u[1];
        break;
    case NLOT_ACKERMANN_2ND: { /* dynamics.py:131-148, vector order reproduced as written */
        jet th = x[2], psi = x[3], v = x[4], psid = x[6], a = u[0], al = u[1];
        f[0] = jmul(v, jcos(th));
        f[1] = jmul(v, jsin(th));
        f[2] = jscale(jmul(v, jtan(psi)), 1.0 / p->wheelbase);
        f[3] = psid;
        /* domega = 1/L * (dpsi / (1 + psi^2) * v + tan(psi) * a) */
        f[4] = jscale(jadd(jmul(jdiv(psid, jaddc(jsq(psi), 1.0)), v), jmul(jtan(psi), a)), 1.0 / p->wheelbase);
        f[5] = a;
        f[6] = al;
        break;
    }
    default:
        for (int i = 0; i < p->nx; ++i) f[i] = jconst(n, NAN);
    }
}

/* The defect map F(x, u) = x + dt f (Euler) or the RK4 step, with A = dF/dx [nx][nx], B = dF/du [nx][nu] */
static void dyn_eval(const NlotProblem* p, const double* x, const double* u, const double* lam, double* F,
                     double* A, double* B, double* Hl);
void oracle_dyn_map(const NlotProblem* p, const double* x, const double* u, double* F, double* A, double* B) {
    dyn_eval(p, x, u, NULL, F, A, B, NULL);
}

void oracle_dynamics(const NlotProblem* p, const double* x, const double* u, double* f) {
    int n = p->nx + p->nu;
    jet xj[8], uj[4], fj[8];
    for (int i = 0; i < p->nx; ++i) xj[i] = jconst(n, x[i]);
    for (int i = 0; i < p->nu; ++i) uj[i] = jconst(n, u[i]);
    dyn_f(p, xj, uj, fj);
    for (int i = 0; i < p->nx; ++i) f[i] = fj[i].v;
}

/* The opt-in RK4 defect map (NLOT_INTEG_RK4, not the reference's NLP): the effective rate
   f_eff = (k1 + 2 k2 + 2 k3 + k4) / 6 with stage points x + k dt/2, x + k dt/2, x + k dt, so that
   F = x + dt f_eff; the GPU's DynRk4 (nlot_device.h) uses the same operation order. */
static void dyn_feff(const NlotProblem* p, const jet* x, const jet* u, jet* fe) {
    if (p->integrator != NLOT_INTEG_RK4) {
        dyn_f(p, x, u, fe);
        return;
    }
    const int nx = p->nx;
    const double dt = p->dt;
    jet k[8], xs[8];
    dyn_f(p, x, u, k);
    for (int i = 0; i < nx; ++i) { fe[i] = k[i]; xs[i] = jadd(x[i], jscale(k[i], 0.5 * dt)); }
    dyn_f(p, xs, u, k);
    for (int i = 0; i < nx; ++i) { fe[i] = jadd(fe[i], jscale(k[i], 2.0)); xs[i] = jadd(x[i], jscale(k[i], 0.5 * dt)); }
    dyn_f(p, xs, u, k);
    for (int i = 0; i < nx; ++i) { fe[i] = jadd(fe[i], jscale(k[i], 2.0)); xs[i] = jadd(x[i], jscale(k[i], dt)); }
    dyn_f(p, xs, u, k);
    for (int i = 0; i < nx; ++i) fe[i] = jscale(jadd(fe[i], k[i]), 1.0 / 6.0);
}

/* F = x + dt f(x,u) (runner.py:62-63; f_eff under RK4): value, A = dF/dx, B = dF/du, Hl = sum_i lam_i d2F_i/dz2 */
static void dyn_eval(const NlotProblem* p, const double* x, const double* u, const double* lam, double* F,
                     double* A, double* B, double* Hl) {
    int nx = p->nx, nu = p->nu, n = nx + nu;
    jet xj[8], uj[4], fj[8];
    for (int i = 0; i < nx; ++i) xj[i] = jvar(n, x[i], i);
    for (int i = 0; i < nu; ++i) uj[i] = jvar(n, u[i], nx + i);
    dyn_feff(p, xj, uj, fj);
    for (int i = 0; i < nx; ++i) {
        F[i] = x[i] + p->dt * fj[i].v;
        if (A)
            for (int j = 0; j < nx; ++j) A[i * nx + j] = (i == j ? 1.0 : 0.0) + p->dt * fj[i].g[j];
        if (B)
            for (int j = 0; j < nu; ++j) B[i * nu + j] = p->dt * fj[i].g[nx + j];
    }
    if (Hl) {
        for (int a = 0; a < n; ++a)
            for (int b = 0; b < n; ++b) {
                double s = 0;
                for (int i = 0; i < nx; ++i) s += lam[i] * fj[i].h[hix(a, b)];
                Hl[a * n + b] = p->dt * s;
            }
    }
}

/* ============================================================================================ */
/* Geometry: corners and per-knot SDF constraints (core/geometry.py)                            */
/* ============================================================================================ */
void oracle_corners(const NlotProblem* p, const double* pose, double* out) { /* geometry.py:78-83 */
    double c = cos(pose[2]), s = sin(pose[2]);
    for (int i = 0; i < p->n_body; ++i) {
        out[2 * i] = pose[0] + c * p->body[i][0] - s * p->body[i][1];
        out[2 * i + 1] = pose[1] + s * p->body[i][0] + c * p->body[i][1];
    }
}

/* number of inequality constraints per knot */
static int knot_m(const NlotProblem* p) {
    if (p->shape == NLOT_SHAPE_DOT) return 1;
    return p->use_slack ? 1 : p->n_body;
}

/* Inequality functions at knot k w.r.t. pose (x, y, theta) = state[0..2] (jets, n = 3).
 * The slack s_k enters linearly with coefficient 1 (geometry.py:116-117) and is added by callers.
 * dot:      d = sdf(x, y)                                    geometry.py:63-67 (slack ignored, bug F7b)
 * slack:    d = soft_min_i sdf(c_i) (+ s_k)                  geometry.py:115-117, margin 0 (runner.py:76)
 * no slack: d_i = sdf(c_i), one per corner                   geometry.py:112-114
 * (densify_polygon with num_points=0 returns the corners, geometry.py:85-105) */
static int knot_ineq(const NlotProblem* p, const NlotMlpDesc* m, const double* xk, int want, jet* d) {
    jet X = jvar(3, xk[0], 0), Y = jvar(3, xk[1], 1);
    if (p->shape == NLOT_SHAPE_DOT) {
        d[0] = sdf_point(p, m, X, Y, want);
        return 1;
    }
    jet T = jvar(3, xk[2], 2);
    jet c = jcos(T), s = jsin(T);
    jet phi[NLOT_MAX_BODY];
    for (int i = 0; i < p->n_body; ++i) {
        double bx = p->body[i][0], by = p->body[i][1];
        jet cx = jadd(X, jsub(jscale(c, bx), jscale(s, by)));
        jet cy = jadd(Y, jadd(jscale(s, bx), jscale(c, by)));
        phi[i] = sdf_point(p, m, cx, cy, want);
    }
    if (p->use_slack) {
        d[0] = soft_min_j(phi, p->n_body, p->softmin_alpha);
        return 1;
    }
    for (int i = 0; i < p->n_body; ++i) d[i] = phi[i];
    return p->n_body;
}

/* value of the per-knot inequality functions (including slack) — exported for tests */
int oracle_knot_constraints(const NlotProblem* p, const NlotMlpDesc* m, const double* xk, double sk, double* d,
                            double* grad3) {
    jet dj[NLOT_MAX_BODY];
    int mm = knot_ineq(p, m, xk, 1, dj);
    for (int j = 0; j < mm; ++j) {
        d[j] = dj[j].v + ((p->use_slack && p->shape != NLOT_SHAPE_DOT) ? sk : 0.0);
        if (grad3)
            for (int i = 0; i < 3; ++i) grad3[3 * j + i] = dj[j].g[i];
    }
    return mm;
}

/* ============================================================================================ */
/* Small dense linear algebra                                                                   */
/* ============================================================================================ */
/* In-place Cholesky of the n x n row-major SPD matrix a (lower factor).  Returns 0 on success,
 * 1 when a pivot is not safely positive (the inertia test of the Newton system). */
static int ldl(double* a, int n, int* perm, int* nneg) {
    double scale = 1e-300;
    for (int i = 0; i < n; ++i)
        for (int j = 0; j < n; ++j) scale = fmax(scale, fabs(a[i * n + j]));
    for (int i = 0; i < n; ++i) perm[i] = i;
    *nneg = 0;
    for (int j = 0; j < n; ++j) {
        int pv = j;
        for (int i = j + 1; i < n; ++i)
            if (fabs(a[i * n + i]) > fabs(a[pv * n + pv])) pv = i;
        if (pv != j) { /* symmetric swap of rows/cols j and pv */
            for (int c = 0; c < n; ++c) {
                double t = a[j * n + c];
                a[j * n + c] = a[pv * n + c];
                a[pv * n + c] = t;
            }
            for (int r = 0; r < n; ++r) {
                double t = a[r * n + j];
                a[r * n + j] = a[r * n + pv];
                a[r * n + pv] = t;
            }
            int t = perm[j];
            perm[j] = perm[pv];
            perm[pv] = t;
        }
        double d = a[j * n + j];
        if (!(fabs(d) > 1e-13 * scale) || !isfinite(d)) return 2;
        if (d < 0) (*nneg)++;
        double col[16];
        for (int i = j + 1; i < n; ++i) col[i] = a[i * n + j];
        for (int i = j + 1; i < n; ++i) {
            for (int k = j + 1; k <= i; ++k) a[i * n + k] -= col[i] * col[k] / d;
            a[i * n + j] = col[i] / d;
        }
        for (int i = j + 1; i < n; ++i) /* keep the trailing block symmetric (upper mirrors lower) */
            for (int k = i + 1; k < n; ++k) a[i * n + k] = a[k * n + i];
    }
    return 0;
}
/* Solve (P' L D L' P) X = Bm in place, X n x m */
static void ldl_solve(const double* a, int n, const int* perm, double* Bm, int m);
int oracle_ldl_test(double* a, int n, double* b, int* nneg) {
    int perm[16];
    int st = ldl(a, n, perm, nneg);
    if (!st) ldl_solve(a, n, perm, b, 1);
    return st;
}
static void ldl_solve(const double* a, int n, const int* perm, double* Bm, int m) {
    double t[16];
    for (int c = 0; c < m; ++c) {
        for (int i = 0; i < n; ++i) t[i] = Bm[perm[i] * m + c];
        for (int i = 0; i < n; ++i)
            for (int k = 0; k < i; ++k) t[i] -= a[i * n + k] * t[k];
        for (int i = 0; i < n; ++i) t[i] /= a[i * n + i];
        for (int i = n - 1; i >= 0; --i)
            for (int k = i + 1; k < n; ++k) t[i] -= a[k * n + i] * t[k];
        for (int i = 0; i < n; ++i) Bm[perm[i] * m + c] = t[i];
    }
}

/* ============================================================================================ */
/* Solver state                                                                                 */
/* ============================================================================================ */
/* Filters (line search, adaptive-mu progress, restoration): IPOPT's Filter is an unbounded list from which
 * dominated entries are removed (Filter::AddEntry).  At most one entry enters per iteration (plus one per
 * restoration entry), so a capacity of 2 max_iter + 64 never overflows: the list is unbounded in effect.
 * NLOT_ORACLE_FILT_CAP forces a smaller capacity that forgets the oldest entry (round-3 behaviour, kept only
 * to measure that variant). */
#define FILT_MIN 64
#define XMAX 8
#define VMAX 5
#define ZMAX (XMAX + VMAX)
#define CMAX 8

typedef struct {
    const NlotProblem* p;
    const NlotMlpDesc* m;
    const NlotSolverOptions* o;
    int nx, nu, ns, N, M, nc, sd; /* sd: slack enters d (polygon + slack) */
    int tidx[CMAX];
    double x0[XMAX], xg[XMAX];
    /* iterate */
    double *X, *U, *S, *T;
    double *yi, *yk, *yt, *yd;
    double *zl, *zu, *zs, *vt;
    /* evaluation at current iterate */
    double f;
    double *gX, *gU, *gS;
    double *F, *A, *B, *Hdyn;
    double *dv, *Jd, *Hd;
    double *Gs; /* path-length Hessian per segment, 2x2 */
    /* Newton system (stage-wise) */
    double *H, *g; /* (N+1) * ZMAX*ZMAX, (N+1) * ZMAX — condensed, unsubstituted */
    double *Kf, *kf, *Kn; /* (N+1) * VMAX*XMAX, VMAX, VMAX*CMAX */
    double *Pm, *pv, *Gm; /* (N+1) * XMAX*XMAX, XMAX, XMAX*CMAX */
    double dx0[XMAX], rN[CMAX];
    double *cdef; /* N * nx dynamics offsets */
    /* equality residuals c(x) in IPOPT sign: x0-x0bar | x_{k+1}-F_k | C x_N - xg | d - t (the RHS) */
    double *rci, *rcd, *rct, *rcq;
    /* step */
    double *dX, *dU, *dS, *dT;
    double *yi_n, *yk_n, *yt_n, *yd_n;
    double *dzl, *dzu, *dzs, *dvt;
    /* scalars */
    double mu, tau, dw_last, theta_max, theta_min;
    int nfilt, fcap;
    int filt_ovf, afilt_ovf, max_nfilt, max_nafilt; /* overflows (forgotten entries) and peak sizes: diagnostics */
    double *filt_theta, *filt_phi;
    /* adaptive mu (IpAdaptiveMuUpdate): free/fixed mode, mu_max and the obj-constr progress filter */
    int free_mode, nafilt;
    double mu_dc; /* mu for delta_c (the iterate's mu; the affine solve uses mu = 0 in the RHS) */
    double mu_max, *af_f, *af_th;
    double lin_resid; /* debug: max residual of the linear KKT system */
    double dc_used;   /* delta_c applied to the terminal block in the last solve */
    /* ---- feasibility restoration problem (IPOPT MinC_1NrmRestorationPhase), active when resto = 1:
     *   min rho sum(p + n) + zeta/2 ||D_R (x - x_R)||^2  s.t.  c(x) - p + n = 0,  p, n >= 0
     * over every equality row (initial state, dynamics, terminal state, d(x) - t).  Row layout:
     * [init nx][dynamics N*nx][terminal nc][inequality (N+1)*M]. */
    int resto, ne;
    int rej_filter, last_rej_filter, n_filt_rej, n_filt_resets; /* IPOPT filter reset heuristic (trigger 5, max 5) */
    int n_soc_tried, n_soc_acc;                                  /* second-order corrections started / accepted */
    long n_trials; /* trial-point merit evaluations (one SDF value evaluation of the trial's corners each) */
    int term; /* diagnostics: how the run ended (TERM_*) */
    double rho, zeta;
    double *XR, *UR, *SR, *DRX, *DRU, *DRS; /* reference point and its proximity scaling */
    double *rp, *rn, *rzp, *rzn;            /* p, n and their bound multipliers */
    double *rdp, *rdn, *rdzp, *rdzn;        /* their steps */
    double *Dsoft, *esoft;                  /* per row: compliance and offset of the soft equality */
    /* ---- general-constraint bounds (o->general_bounds = 1): CasADi Opti hands the reference's control bounds
     * (opti.bounded(umin, U, umax), runner.py:100-104) and slack >= 0 (runner.py:67-69) to IPOPT as constraint
     * rows g(x) = U_ki, g(x) = S_k, so IPOPT sees d(x) - sigma = 0 with the bounds on its slack sigma, and U, S
     * free.  Bound row b: control b = k nu + i (umin_i <= sigma <= umax_i), then slack rows N nu + k (sigma >= 0);
     * zbl / zbu are sigma's bound multipliers, yb the row multiplier, rcb = U - sigma (or S - sigma). */
    int gcb, nb;
    /* IPOPT bound_relax_factor (variant, NLOT_ORACLE_BOUND_RELAX = r): every bound relaxed by r max(1, |bound|)
     * (TNLPAdapter); prel is the problem with the relaxed control bounds, brel the relaxation of the zero bounds
     * of S and of the inequality slacks (the bound distances are S + brel and T = d(x) + brel). */
    double brel;
    NlotProblem prel;
    double *sb, *yb, *zbl, *zbu, *rcb, *dsb, *yb_n, *dzbl, *dzbu;
    double *arena;
    unsigned long long jit_ctr; /* NLOT_ORACLE_STEP_JITTER's stream position (per solve: deterministic) */
} Sol;
static int row_d(const Sol* s, int k, int i) { return s->nx + k * s->nx + i; }
static int row_t(const Sol* s, int j) { return s->nx + s->N * s->nx + j; }
static int row_q(const Sol* s, int q) { return s->nx + s->N * s->nx + s->nc + q; }
static int row_b(const Sol* s, int b) { return row_q(s, (s->N + 1) * s->M) + b; } /* restoration row of bound row b */
/* bound row b: its variable, bounds (one-sided rows have no upper bound) */
static double bvar(const Sol* s, const double* U, const double* S, int b) {
    return b < s->N * s->nu ? U[b] : S[b - s->N * s->nu];
}
static double blo(const Sol* s, int b) { return b < s->N * s->nu ? s->p->umin[b % s->nu] : -s->brel; }
static int bhi_on(const Sol* s, int b) { return b < s->N * s->nu; }
static double bhi(const Sol* s, int b) { return b < s->N * s->nu ? s->p->umax[b % s->nu] : 0.0; }

static int nv_of(const Sol* s, int k) { return (k < s->N ? s->nu : 0) + s->ns; }

static int sol_alloc(Sol* s) {
    int N = s->N, nx = s->nx, nu = s->nu, M = s->M;
    size_t n = 0;
#define TAKE(ptr, cnt) n += (size_t)(cnt);
#define ALLOCS                                                                                   \
    TAKE(X, (N + 1) * nx) TAKE(U, N * nu) TAKE(S, (N + 1)) TAKE(T, (N + 1) * M) TAKE(yi, nx)     \
    TAKE(yk, N * nx) TAKE(yt, CMAX) TAKE(yd, (N + 1) * M) TAKE(zl, N * nu) TAKE(zu, N * nu)       \
    TAKE(zs, (N + 1)) TAKE(vt, (N + 1) * M) TAKE(gX, (N + 1) * nx) TAKE(gU, N * nu)               \
    TAKE(gS, (N + 1)) TAKE(F, N * nx) TAKE(A, N * nx * nx) TAKE(B, N * nx * nu)                   \
    TAKE(Hdyn, N * (nx + nu) * (nx + nu)) TAKE(dv, (N + 1) * M) TAKE(Jd, (N + 1) * M * 3)         \
    TAKE(Hd, (N + 1) * 9) TAKE(Gs, N * 4) TAKE(H, (N + 1) * ZMAX * ZMAX) TAKE(g, (N + 1) * ZMAX)  \
    TAKE(Kf, (N + 1) * VMAX * XMAX) TAKE(kf, (N + 1) * VMAX) TAKE(Kn, (N + 1) * VMAX * CMAX)      \
    TAKE(Pm, (N + 1) * XMAX * XMAX) TAKE(pv, (N + 1) * XMAX) TAKE(Gm, (N + 1) * XMAX * CMAX)      \
    TAKE(cdef, N * nx) TAKE(dX, (N + 1) * nx) TAKE(dU, N * nu) TAKE(dS, (N + 1))                 \
    TAKE(dT, (N + 1) * M) TAKE(yi_n, nx) TAKE(yk_n, N * nx) TAKE(yt_n, CMAX)                     \
    TAKE(yd_n, (N + 1) * M) TAKE(dzl, N * nu) TAKE(dzu, N * nu) TAKE(dzs, (N + 1))               \
    TAKE(dvt, (N + 1) * M) TAKE(rci, XMAX) TAKE(rcd, N * nx) TAKE(rct, CMAX) TAKE(rcq, (N + 1) * M)         \
    TAKE(XR, (N + 1) * nx) TAKE(UR, N * nu) TAKE(SR, N + 1) TAKE(DRX, (N + 1) * nx) TAKE(DRU, N * nu)           \
    TAKE(DRS, N + 1) TAKE(rp, NE) TAKE(rn, NE) TAKE(rzp, NE) TAKE(rzn, NE) TAKE(rdp, NE) TAKE(rdn, NE)          \
    TAKE(rdzp, NE) TAKE(rdzn, NE) TAKE(Dsoft, NE) TAKE(esoft, NE) TAKE(sb, NB) TAKE(yb, NB) TAKE(zbl, NB)           \
    TAKE(zbu, NB) TAKE(rcb, NB) TAKE(dsb, NB) TAKE(yb_n, NB) TAKE(dzbl, NB) TAKE(dzbu, NB)                  \
    TAKE(filt_theta, FC) TAKE(filt_phi, FC) TAKE(af_f, FC) TAKE(af_th, FC)
    const int FC = s->fcap;
    const int NB = N * nu + N + 1;
    const int NE = nx + N * nx + CMAX + (N + 1) * M + NB;
    ALLOCS
#undef TAKE
    s->arena = (double*)calloc(n, sizeof(double));
    if (!s->arena) return 1;
    double* q = s->arena;
#define TAKE(ptr, cnt) s->ptr = q; q += (size_t)(cnt);
    ALLOCS
#undef TAKE
    return 0;
}

/* ============================================================================================ */
/* NLP evaluation (runner.py:44-108)                                                            */
/* ============================================================================================ */
/* NLOT_ORACLE_SUM_REV=1 (test infrastructure, tests/test_pinned_iterates_gpu.py): the merit function's fp64 sums
 * (theta, the barrier terms, the objective and the restoration objective: the values the filter and Armijo tests
 * compare) accumulate in the reverse index order.  The result differs from the default only by fp64 rounding: the
 * kind of difference the GPU's wave reductions make in every iteration (another summation order), where the
 * fixture's perturbed runs differ only at the start.  Read per call (toggled between whole batches). */
static int sum_rev(void) {
    const char* e = getenv("NLOT_ORACLE_SUM_REV");
    return e && e[0] == '1';
}
#define SRV(i, n) (srv ? (n) - 1 - (i) : (i))

/* objective value at (X, U, S)  — runner.py:80-96 */
static double objective(const Sol* s, const double* X, const double* U, const double* S) {
    const NlotProblem* p = s->p;
    int nx = s->nx, nu = s->nu, N = s->N;
    const int srv = sum_rev();
    double f = 0;
    for (int k_ = 0; k_ < N; ++k_) {
        const int k = SRV(k_, N);
        double dx = X[(k + 1) * nx] - X[k * nx], dy = X[(k + 1) * nx + 1] - X[k * nx + 1];
        f += sqrt(dx * dx + dy * dy + p->path_eps);
    }
    if (p->use_slack) {
        double q = 0;
        for (int k = 0; k <= N; ++k) q += S[SRV(k, N + 1)] * S[SRV(k, N + 1)];
        f += p->slack_penalty * q;
    }
    if (p->use_smooth) {
        double q = 0;
        for (int k = 0; k < N - 1; ++k) /* sum_{k < N-1} ||u_k||^2, runner.py:92-95 (bug F7c kept) */
            for (int i = 0; i < nu; ++i) q += U[SRV(k, N - 1) * nu + i] * U[SRV(k, N - 1) * nu + i];
        f += p->smooth_weight * q;
    }
    return f;
}

/* Restoration objective rho sum(p + n) + zeta/2 ||D_R (x - x_R)||^2 over x = (X, U, S). */
static double objective_resto(const Sol* s, const double* X, const double* U, const double* S, const double* p,
                              const double* n) {
    int nx = s->nx, nu = s->nu, N = s->N;
    const int srv = sum_rev();
    double a = 0, q = 0;
    for (int i_ = 0; i_ < s->ne; ++i_) {
        const int i = SRV(i_, s->ne);
        a += p[i] + n[i];
    }
    for (int i_ = 0; i_ < (N + 1) * nx; ++i_) {
        const int i = SRV(i_, (N + 1) * nx);
        q += pow(s->DRX[i] * (X[i] - s->XR[i]), 2);
    }
    for (int i_ = 0; i_ < N * nu; ++i_) {
        const int i = SRV(i_, N * nu);
        q += pow(s->DRU[i] * (U[i] - s->UR[i]), 2);
    }
    if (s->ns)
        for (int k_ = 0; k_ <= N; ++k_) {
            const int k = SRV(k_, N + 1);
            q += pow(s->DRS[k] * (S[k] - s->SR[k]), 2);
        }
    return s->rho * a + 0.5 * s->zeta * q;
}

/* Equality residuals c(x) (IPOPT sign) at a point; any output may be NULL.  rcb (bound rows, general_bounds)
 * = U - sigma / S - sigma at the slacks SB. */
static void residuals(const Sol* s, const double* X, const double* U, const double* S, const double* T,
                      const double* SB, double* rci, double* rcd, double* rct, double* rcq, double* rcb) {
    const NlotProblem* p = s->p;
    int nx = s->nx, nu = s->nu, N = s->N, M = s->M;
    for (int i = 0; i < nx; ++i) rci[i] = X[i] - s->x0[i];
    for (int j = 0; j < s->nc; ++j) rct[j] = X[N * nx + s->tidx[j]] - s->xg[s->tidx[j]];
    for (int k = 0; k < N; ++k) {
        double Fk[XMAX];
        dyn_eval(p, X + k * nx, U + k * nu, NULL, Fk, NULL, NULL, NULL);
        for (int i = 0; i < nx; ++i) rcd[k * nx + i] = X[(k + 1) * nx + i] - Fk[i];
    }
    for (int k = 0; k <= N; ++k) {
        jet d[NLOT_MAX_BODY];
        knot_ineq(p, s->m, X + k * nx, 0, d);
        for (int j = 0; j < M; ++j) rcq[k * M + j] = d[j].v + (s->sd ? S[k] : 0.0) + s->brel - T[k * M + j];
    }
    if (rcb)
        for (int q = 0; q < s->nb; ++q) rcb[q] = bvar(s, U, S, q) - SB[q];
}

/* barrier terms of the bounded quantities: variable bounds of U, S, or (general_bounds) the bound rows' slacks;
 * the inequality slacks T.  bar = sum of logs, lin = sum of the one-sided slacks (kappa_d damping) */
static void barrier_terms(const Sol* s, const double* U, const double* S, const double* T, const double* SB,
                          double* bar_out, double* lin_out) {
    const NlotProblem* p = s->p;
    int nu = s->nu, N = s->N, M = s->M;
    const int srv = sum_rev();
    double bar = 0, lin = 0;
    for (int q_ = 0; q_ < (N + 1) * M; ++q_) {
        const int q = SRV(q_, (N + 1) * M);
        bar += log(T[q]);
        lin += T[q];
    }
    if (s->gcb) {
        for (int q_ = 0; q_ < s->nb; ++q_) {
            const int q = SRV(q_, s->nb);
            bar += log(SB[q] - blo(s, q));
            if (bhi_on(s, q)) bar += log(bhi(s, q) - SB[q]);
            else lin += SB[q];
        }
    } else {
        for (int k_ = 0; k_ < N; ++k_) {
            const int k = SRV(k_, N);
            for (int i = 0; i < nu; ++i) bar += log(U[k * nu + i] - p->umin[i]) + log(p->umax[i] - U[k * nu + i]);
        }
        if (s->ns)
            for (int k_ = 0; k_ <= N; ++k_) {
                const int k = SRV(k_, N + 1);
                bar += log(S[k] + s->brel);
                lin += S[k] + s->brel;
            }
    }
    *bar_out = bar;
    *lin_out = lin;
}

/* Constraint violation theta = ||c||_1 (incl. d - t and the bound rows) and barrier value phi_mu at a point;
 * the residual arrays (may be NULL) receive c(x). */
static void merit_r(const Sol* s, const double* X, const double* U, const double* S, const double* T, const double* SB,
                    double mu, double* theta, double* phi, double* rci, double* rcd, double* rct, double* rcq,
                    double* rcb) {
    int nx = s->nx, N = s->N, M = s->M;
    double bi[XMAX], bt[CMAX];
    double* bd = (double*)malloc(sizeof(double) * (N * nx + (N + 1) * M + s->nb + 1));
    double* bq = bd + N * nx;
    double* bb = bq + (N + 1) * M;
    if (!rci) rci = bi;
    if (!rct) rct = bt;
    if (!rcd) rcd = bd;
    if (!rcq) rcq = bq;
    if (!rcb) rcb = bb;
    residuals(s, X, U, S, T, SB, rci, rcd, rct, rcq, rcb);
    double th = 0, bar, lin;
    const int srv = sum_rev();
    for (int i = 0; i < nx; ++i) th += fabs(rci[SRV(i, nx)]);
    for (int j = 0; j < s->nc; ++j) th += fabs(rct[SRV(j, s->nc)]);
    for (int i = 0; i < N * nx; ++i) th += fabs(rcd[SRV(i, N * nx)]);
    for (int q = 0; q < (N + 1) * M; ++q) th += fabs(rcq[SRV(q, (N + 1) * M)]);
    for (int q = 0; q < s->nb; ++q) th += fabs(rcb[SRV(q, s->nb)]);
    free(bd);
    barrier_terms(s, U, S, T, SB, &bar, &lin);
    const double kappa_d = 1e-5;
    *theta = th;
    *phi = objective(s, X, U, S) - mu * bar + kappa_d * mu * lin;
}
/* Restoration merit at (x, t, p, n): theta_R = ||c(x) - p + n||_1 over every row (d - t and bound rows included),
 * phi_R = restoration objective - mu sum ln(bound slacks incl. p, n) + kappa_d mu sum(one-sided slacks). */
static void merit_resto(const Sol* s, const double* X, const double* U, const double* S, const double* T,
                        const double* SB, const double* pp, const double* nn, double mu, double* theta, double* phi,
                        double* rci, double* rcd, double* rct, double* rcq, double* rcb) {
    int nx = s->nx, N = s->N, M = s->M;
    double bi[XMAX], bt[CMAX];
    double* bd = (double*)malloc(sizeof(double) * (N * nx + (N + 1) * M + s->nb + 1));
    double* bq = bd + N * nx;
    double* bb = bq + (N + 1) * M;
    if (!rci) rci = bi;
    if (!rct) rct = bt;
    if (!rcd) rcd = bd;
    if (!rcq) rcq = bq;
    if (!rcb) rcb = bb;
    residuals(s, X, U, S, T, SB, rci, rcd, rct, rcq, rcb);
    for (int i = 0; i < nx; ++i) rci[i] += -pp[i] + nn[i];
    for (int k = 0; k < N; ++k)
        for (int i = 0; i < nx; ++i) rcd[k * nx + i] += -pp[row_d(s, k, i)] + nn[row_d(s, k, i)];
    for (int j = 0; j < s->nc; ++j) rct[j] += -pp[row_t(s, j)] + nn[row_t(s, j)];
    for (int q = 0; q < (N + 1) * M; ++q) rcq[q] += -pp[row_q(s, q)] + nn[row_q(s, q)];
    for (int q = 0; q < s->nb; ++q) rcb[q] += -pp[row_b(s, q)] + nn[row_b(s, q)];
    double th = 0, bar, lin;
    const int srv = sum_rev();
    for (int i = 0; i < nx; ++i) th += fabs(rci[SRV(i, nx)]);
    for (int j = 0; j < s->nc; ++j) th += fabs(rct[SRV(j, s->nc)]);
    for (int i = 0; i < N * nx; ++i) th += fabs(rcd[SRV(i, N * nx)]);
    for (int q = 0; q < (N + 1) * M; ++q) th += fabs(rcq[SRV(q, (N + 1) * M)]);
    for (int q = 0; q < s->nb; ++q) th += fabs(rcb[SRV(q, s->nb)]);
    free(bd);
    barrier_terms(s, U, S, T, SB, &bar, &lin);
    for (int i_ = 0; i_ < s->ne; ++i_) {
        const int i = SRV(i_, s->ne);
        bar += log(pp[i]) + log(nn[i]);
        lin += pp[i] + nn[i];
    }
    *theta = th;
    *phi = objective_resto(s, X, U, S, pp, nn) - mu * bar + 1e-5 * mu * lin;
}

static void merit(const Sol* s, const double* X, const double* U, const double* S, const double* T, const double* SB,
                  double mu, double* theta, double* phi, double* fout) {
    merit_r(s, X, U, S, T, SB, mu, theta, phi, NULL, NULL, NULL, NULL, NULL);
    if (fout) *fout = objective(s, X, U, S);
}

/* Full evaluation at the current iterate: gradients, Jacobians, Lagrangian-Hessian pieces. */
static void eval_full(Sol* s) {
    const NlotProblem* p = s->p;
    int nx = s->nx, nu = s->nu, N = s->N, M = s->M, nz = nx + nu;
    s->f = objective(s, s->X, s->U, s->S);
    memset(s->gX, 0, sizeof(double) * (N + 1) * nx);
    memset(s->gU, 0, sizeof(double) * N * nu);
    memset(s->gS, 0, sizeof(double) * (N + 1));
    for (int k = 0; k < N; ++k) { /* path length, runner.py:82-86 */
        double dx = s->X[(k + 1) * nx] - s->X[k * nx], dy = s->X[(k + 1) * nx + 1] - s->X[k * nx + 1];
        double r2 = dx * dx + dy * dy + p->path_eps, r = sqrt(r2), r3 = r2 * r;
        s->gX[(k + 1) * nx] += dx / r;
        s->gX[(k + 1) * nx + 1] += dy / r;
        s->gX[k * nx] -= dx / r;
        s->gX[k * nx + 1] -= dy / r;
        s->Gs[4 * k + 0] = (r2 - dx * dx) / r3;
        s->Gs[4 * k + 1] = -dx * dy / r3;
        s->Gs[4 * k + 2] = -dx * dy / r3;
        s->Gs[4 * k + 3] = (r2 - dy * dy) / r3;
    }
    if (p->use_slack)
        for (int k = 0; k <= N; ++k) s->gS[k] = 2.0 * p->slack_penalty * s->S[k];
    if (p->use_smooth)
        for (int k = 0; k < N - 1; ++k)
            for (int i = 0; i < nu; ++i) s->gU[k * nu + i] = 2.0 * p->smooth_weight * s->U[k * nu + i];
    for (int k = 0; k < N; ++k) {
        double Fk[XMAX];
        dyn_eval(p, s->X + k * nx, s->U + k * nu, s->yk + k * nx, Fk, s->A + k * nx * nx, s->B + k * nx * nu,
                 s->Hdyn + k * nz * nz);
        for (int i = 0; i < nx; ++i) {
            s->F[k * nx + i] = Fk[i];
            s->rcd[k * nx + i] = s->X[(k + 1) * nx + i] - Fk[i];
        }
    }
    for (int i = 0; i < nx; ++i) s->rci[i] = s->X[i] - s->x0[i];
    for (int j = 0; j < s->nc; ++j) s->rct[j] = s->X[N * nx + s->tidx[j]] - s->xg[s->tidx[j]];
    for (int q = 0; q < s->nb; ++q) s->rcb[q] = bvar(s, s->U, s->S, q) - s->sb[q];
    if (s->resto) { /* c(x) - p + n, and the restoration objective's gradient (no path-length terms) */
        for (int i = 0; i < nx; ++i) s->rci[i] += -s->rp[i] + s->rn[i];
        for (int q = 0; q < s->nb; ++q) s->rcb[q] += -s->rp[row_b(s, q)] + s->rn[row_b(s, q)];
        for (int k = 0; k < N; ++k)
            for (int i = 0; i < nx; ++i) s->rcd[k * nx + i] += -s->rp[row_d(s, k, i)] + s->rn[row_d(s, k, i)];
        for (int j = 0; j < s->nc; ++j) s->rct[j] += -s->rp[row_t(s, j)] + s->rn[row_t(s, j)];
        s->f = objective_resto(s, s->X, s->U, s->S, s->rp, s->rn);
        for (int i = 0; i < (N + 1) * nx; ++i) s->gX[i] = s->zeta * s->DRX[i] * s->DRX[i] * (s->X[i] - s->XR[i]);
        for (int i = 0; i < N * nu; ++i) s->gU[i] = s->zeta * s->DRU[i] * s->DRU[i] * (s->U[i] - s->UR[i]);
        for (int k = 0; k <= N; ++k) s->gS[k] = s->ns ? s->zeta * s->DRS[k] * s->DRS[k] * (s->S[k] - s->SR[k]) : 0.0;
        memset(s->Gs, 0, sizeof(double) * 4 * N);
    }
    for (int k = 0; k <= N; ++k) {
        jet d[NLOT_MAX_BODY];
        knot_ineq(p, s->m, s->X + k * nx, 1, d);
        double* Hd = s->Hd + 9 * k;
        memset(Hd, 0, sizeof(double) * 9);
        for (int j = 0; j < M; ++j) {
            s->dv[k * M + j] = d[j].v + (s->sd ? s->S[k] : 0.0);
            s->rcq[k * M + j] = s->dv[k * M + j] + s->brel - s->T[k * M + j];
            if (s->resto) s->rcq[k * M + j] += -s->rp[row_q(s, k * M + j)] + s->rn[row_q(s, k * M + j)];
            for (int a = 0; a < 3; ++a) s->Jd[(k * M + j) * 3 + a] = d[j].g[a];
            double w = s->yd[k * M + j];
            for (int a = 0; a < 3; ++a)
                for (int b = 0; b < 3; ++b) Hd[a * 3 + b] += w * d[j].h[hix(a, b)];
        }
    }
}

/* Optimality measures (IPOPT's OptimalityErrorConvergenceCheck / curr_barrier_error). */
typedef struct {
    double dual, primal, compl0, complmu, sd, sc, cviol;
    /* for the quality-function mu oracle (IpQualityFunctionMuOracle, 2-norm-squared) */
    double dual_sq, primal_sq, avg_compl;
    int n_dual, n_pri, n_comp;
    /* 1-norms for the primal-dual system error of the soft restoration phase */
    double dual_1, primal_1, complmu_1;
} Errs;

/* The residual arrays rci/rcd/rct/rcq must hold c(x) (minus p plus n in the restoration problem), as
 * eval_full leaves them. */
static void errors(const Sol* s, Errs* e) {
    const NlotProblem* p = s->p;
    int nx = s->nx, nu = s->nu, N = s->N, M = s->M;
    double dual = 0, primal = 0, c0 = 0, cmu = 0, cviol = 0, ysum = 0, zsum = 0;
    double dsq = 0, psq = 0, csum = 0, d1 = 0, p1 = 0, c1 = 0;
    int ny = 0, nzc = 0, ndual = 0, npri = 0;
#define DUAL(v)                                                                                  \
    do {                                                                                         \
        double vv = (v);                                                                         \
        dual = fmax(dual, fabs(vv));                                                             \
        dsq += vv * vv;                                                                          \
        d1 += fabs(vv);                                                                          \
        ndual++;                                                                                 \
    } while (0)
    /* dual infeasibility: grad L over x, u, s, t */
    for (int k = 0; k <= N; ++k) {
        double r[XMAX];
        for (int i = 0; i < nx; ++i) r[i] = s->gX[k * nx + i];
        if (k > 0)
            for (int i = 0; i < nx; ++i) r[i] += s->yk[(k - 1) * nx + i];
        if (k < N)
            for (int j = 0; j < nx; ++j) {
                double t = 0;
                for (int i = 0; i < nx; ++i) t += s->A[k * nx * nx + i * nx + j] * s->yk[k * nx + i];
                r[j] -= t;
            }
        if (k == 0)
            for (int i = 0; i < nx; ++i) r[i] += s->yi[i];
        if (k == N)
            for (int j = 0; j < s->nc; ++j) r[s->tidx[j]] += s->yt[j];
        for (int j = 0; j < M; ++j)
            for (int a = 0; a < 3; ++a) r[a] += s->Jd[(k * M + j) * 3 + a] * s->yd[k * M + j];
        for (int i = 0; i < nx; ++i) DUAL(r[i]);
        if (k < N)
            for (int i = 0; i < nu; ++i) {
                double t = s->gcb ? s->gU[k * nu + i] + s->yb[k * nu + i]
                                  : s->gU[k * nu + i] - s->zl[k * nu + i] + s->zu[k * nu + i];
                for (int a = 0; a < nx; ++a) t -= s->B[k * nx * nu + a * nu + i] * s->yk[k * nx + a];
                DUAL(t);
            }
        if (s->ns) {
            double t = s->gcb ? s->gS[k] + s->yb[N * nu + k] : s->gS[k] - s->zs[k];
            if (s->sd)
                for (int j = 0; j < M; ++j) t += s->yd[k * M + j];
            DUAL(t);
        }
        for (int j = 0; j < M; ++j) DUAL(-s->yd[k * M + j] - s->vt[k * M + j]);
    }
    for (int q = 0; q < s->nb; ++q) /* bound-row slacks: -y - z_L + z_U */
        DUAL(-s->yb[q] - s->zbl[q] + (bhi_on(s, q) ? s->zbu[q] : 0.0));
    /* primal infeasibility (c, d - t) and unscaled constraint violation */
#define PRI(v)                                                                                   \
    do {                                                                                         \
        double vv = (v);                                                                         \
        primal = fmax(primal, fabs(vv));                                                         \
        psq += vv * vv;                                                                          \
        p1 += fabs(vv);                                                                          \
        npri++;                                                                                  \
    } while (0)
    for (int i = 0; i < nx; ++i) PRI(s->rci[i]);
    for (int j = 0; j < s->nc; ++j) PRI(s->rct[j]);
    for (int i = 0; i < N * nx; ++i) PRI(s->rcd[i]);
    cviol = primal;
    for (int q = 0; q < (N + 1) * M; ++q) {
        PRI(s->rcq[q]);
        cviol = fmax(cviol, fmax(0.0, -s->dv[q]));
    }
    for (int q = 0; q < s->nb; ++q) { /* bound rows: d(x) = U or S against [d_L, d_U] */
        PRI(s->rcb[q]);
        const double v = bvar(s, s->U, s->S, q);
        cviol = fmax(cviol, fmax(0.0, blo(s, q) - v));
        if (bhi_on(s, q)) cviol = fmax(cviol, fmax(0.0, v - bhi(s, q)));
    }
#undef PRI
    /* complementarity */
#define COMPL(z, sl)                                                                             \
    do {                                                                                         \
        double zz = (z), ss = (sl);                                                              \
        c0 = fmax(c0, fabs(zz * ss));                                                            \
        cmu = fmax(cmu, fabs(zz * ss - s->mu));                                                  \
        c1 += fabs(zz * ss - s->mu);                                                             \
        csum += zz * ss;                                                                         \
        zsum += fabs(zz);                                                                        \
        nzc++;                                                                                   \
    } while (0)
    if (s->gcb) {
        for (int q = 0; q < s->nb; ++q) {
            COMPL(s->zbl[q], s->sb[q] - blo(s, q));
            if (bhi_on(s, q)) COMPL(s->zbu[q], bhi(s, q) - s->sb[q]);
        }
    } else {
        for (int k = 0; k < N; ++k)
            for (int i = 0; i < nu; ++i) {
                COMPL(s->zl[k * nu + i], s->U[k * nu + i] - p->umin[i]);
                COMPL(s->zu[k * nu + i], p->umax[i] - s->U[k * nu + i]);
            }
        if (s->ns)
            for (int k = 0; k <= N; ++k) COMPL(s->zs[k], s->S[k] + s->brel);
    }
    for (int k = 0; k <= N; ++k)
        for (int j = 0; j < M; ++j) COMPL(s->vt[k * M + j], s->T[k * M + j]);
    if (s->resto) /* p and n rows: rho -+ y - z = 0, z p = mu, z n = mu */
        for (int i = 0; i < s->ne; ++i) {
            double y = i < nx ? s->yi[i]
                       : i < row_t(s, 0) ? s->yk[i - nx]
                       : i < row_q(s, 0) ? s->yt[i - row_t(s, 0)]
                       : i < row_b(s, 0) ? s->yd[i - row_q(s, 0)]
                                         : s->yb[i - row_b(s, 0)];
            DUAL(s->rho - y - s->rzp[i]);
            DUAL(s->rho + y - s->rzn[i]);
            COMPL(s->rzp[i], s->rp[i]);
            COMPL(s->rzn[i], s->rn[i]);
        }
#undef COMPL
#undef DUAL
    for (int i = 0; i < nx; ++i) ysum += fabs(s->yi[i]);
    for (int i = 0; i < N * nx; ++i) ysum += fabs(s->yk[i]);
    for (int j = 0; j < s->nc; ++j) ysum += fabs(s->yt[j]);
    for (int i = 0; i < (N + 1) * M; ++i) ysum += fabs(s->yd[i]);
    for (int i = 0; i < s->nb; ++i) ysum += fabs(s->yb[i]);
    ny = nx + N * nx + s->nc + (N + 1) * M + s->nb;
    const double smax = 100.0;
    e->sd = fmax(smax, (ysum + zsum) / (double)(ny + nzc)) / smax;
    e->sc = fmax(smax, zsum / (double)nzc) / smax;
    e->dual = dual;
    e->primal = primal;
    e->compl0 = c0;
    e->complmu = cmu;
    e->cviol = cviol;
    e->dual_sq = dsq;
    e->primal_sq = psq;
    e->n_dual = ndual;
    e->n_pri = npri;
    e->n_comp = nzc;
    e->avg_compl = nzc ? csum / nzc : 0.0;
    e->dual_1 = d1;
    e->primal_1 = p1;
    e->complmu_1 = c1;
}

/* IPOPT's primal-dual system error (soft restoration phase): mean absolute residual of the primal-dual
 * system at barrier parameter mu, sum of 1-norms / element count.  errors() must have run with s->mu =
 * the mu wanted. */
static double pd_error(const Errs* e) {
    return (e->dual_1 + e->primal_1 + e->complmu_1) / (double)(e->n_dual + e->n_pri + e->n_comp);
}

/* ============================================================================================ */
/* Newton system: stage matrices + Riccati recursion                                            */
/* ============================================================================================ */
enum { MODE_NEWTON = 0, MODE_LSQ = 1 };

/* Build the condensed stage-wise system:
 *   min sum_k 1/2 z_k' H_k z_k + g_k' z_k + sum_k dx_k' M_k dx_{k+1}
 *   s.t. dx_0 = dx0, dx_{k+1} = A_k dx_k + B_k dv_k + c_k, C dx_N = rN
 * H_k includes W_kk + Sigma + dw I + J_d' D J_d (IPOPT slacks t and their duals eliminated). */
/* bound row q (general_bounds) in the condensed stage system: sigma (and in the restoration problem p, n) eliminated.
 * bg = sigma's barrier gradient, Sig = its barrier Hessian; Newton: D = Sig + dw, rhs = D r + bg (r = U - sigma);
 * restoration: D = 1 / C, rhs = (r - E) / C as for the inequality rows; least squares: D = 1, rhs = -(z_L - z_U). */
static void bound_sig(const Sol* s, int q, double* Sig, double* bg) {
    const double mu = s->mu, kappa_d = 1e-5, sl = s->sb[q] - blo(s, q);
    *Sig = s->zbl[q] / sl;
    *bg = -mu / sl;
    if (bhi_on(s, q)) {
        const double su = bhi(s, q) - s->sb[q];
        *Sig += s->zbu[q] / su;
        *bg += mu / su;
    } else {
        *bg += kappa_d * mu;
    }
}
static void bound_row(const Sol* s, int q, int mode, double dw, double* D, double* rhs) {
    const double kappa_d = 1e-5, mu = s->mu;
    if (mode != MODE_NEWTON) {
        *D = 1.0;
        *rhs = -(s->zbl[q] - (bhi_on(s, q) ? s->zbu[q] : 0.0));
        return;
    }
    double Sig, bg;
    bound_sig(s, q, &Sig, &bg);
    const double st = Sig + dw;
    if (s->resto) {
        const int r = row_b(s, q);
        const double pp = s->rp[r], nn = s->rn[r];
        const double sp = s->rzp[r] / pp + dw, sn = s->rzn[r] / nn + dw;
        const double C = 1.0 / st + 1.0 / sp + 1.0 / sn;
        const double E = -bg / st + (mu / pp - s->rho - kappa_d * mu) / sp - (mu / nn - s->rho - kappa_d * mu) / sn;
        *D = 1.0 / C;
        *rhs = (s->rcb[q] - E) / C;
    } else {
        *D = st;
        *rhs = st * s->rcb[q] + bg;
    }
}

static void build(Sol* s, int mode, double dw) {
    const NlotProblem* p = s->p;
    int nx = s->nx, nu = s->nu, N = s->N, M = s->M, nzd = nx + nu;
    const double kappa_d = 1e-5;
    double mu = s->mu;
    for (int k = 0; k <= N; ++k) {
        int nvk = nv_of(s, k), nzk = nx + nvk, iu = nx, is = nx + (k < N ? nu : 0);
        double* H = s->H + (size_t)k * ZMAX * ZMAX;
        double* g = s->g + (size_t)k * ZMAX;
        memset(H, 0, sizeof(double) * ZMAX * ZMAX);
        memset(g, 0, sizeof(double) * ZMAX);
#define HH(i, j) H[(i)*nzk + (j)]
        for (int i = 0; i < nx; ++i) g[i] = s->gX[k * nx + i];
        if (k < N)
            for (int i = 0; i < nu; ++i) g[iu + i] = s->gU[k * nu + i];
        if (s->ns) g[is] = s->gS[k];
        if (mode == MODE_NEWTON) {
            /* objective Hessian */
            for (int a = 0; a < 2; ++a)
                for (int b = 0; b < 2; ++b) {
                    if (k < N) HH(a, b) += s->Gs[4 * k + 2 * a + b];
                    if (k > 0) HH(a, b) += s->Gs[4 * (k - 1) + 2 * a + b];
                }
            if (s->resto) { /* restoration objective: zeta D_R^2 (its only curvature besides the constraints) */
                for (int i = 0; i < nx; ++i) HH(i, i) += s->zeta * s->DRX[k * nx + i] * s->DRX[k * nx + i];
                if (k < N)
                    for (int i = 0; i < nu; ++i) HH(iu + i, iu + i) += s->zeta * s->DRU[k * nu + i] * s->DRU[k * nu + i];
                if (s->ns) HH(is, is) += s->zeta * s->DRS[k] * s->DRS[k];
            } else {
                if (p->use_slack) HH(is, is) += 2.0 * p->slack_penalty;
                if (p->use_smooth && k < N - 1)
                    for (int i = 0; i < nu; ++i) HH(iu + i, iu + i) += 2.0 * p->smooth_weight;
            }
            /* dynamics constraint c_k = x_{k+1} - F_k: W += -sum_i y_i d2F_i */
            if (k < N)
                for (int a = 0; a < nzd; ++a)
                    for (int b = 0; b < nzd; ++b) HH(a, b) -= s->Hdyn[(size_t)k * nzd * nzd + a * nzd + b];
            /* knot inequality curvature  sum_j yd_j d2 d_j (pose block) */
            for (int a = 0; a < 3; ++a)
                for (int b = 0; b < 3; ++b)
                    if (a < nx && b < nx) HH(a, b) += s->Hd[9 * k + a * 3 + b];
            /* bound barriers Sigma and barrier gradient (variable bounds; general_bounds: the bound rows below) */
            if (k < N && !s->gcb)
                for (int i = 0; i < nu; ++i) {
                    double sl = s->U[k * nu + i] - p->umin[i], su = p->umax[i] - s->U[k * nu + i];
                    HH(iu + i, iu + i) += s->zl[k * nu + i] / sl + s->zu[k * nu + i] / su;
                    g[iu + i] += -mu / sl + mu / su;
                }
            if (s->ns && !s->gcb) {
                HH(is, is) += s->zs[k] / (s->S[k] + s->brel);
                g[is] += -mu / (s->S[k] + s->brel) + kappa_d * mu;
            }
            for (int i = 0; i < nzk; ++i) HH(i, i) += dw;
        } else {
            for (int i = 0; i < nzk; ++i) HH(i, i) = 1.0;
            if (k < N && !s->gcb)
                for (int i = 0; i < nu; ++i) g[iu + i] += -s->zl[k * nu + i] + s->zu[k * nu + i];
            if (s->ns && !s->gcb) g[is] += -s->zs[k];
        }
        /* general_bounds: bound rows U_ki - sigma = 0 / S_k - sigma = 0 with sigma's barrier eliminated like t below
         * (J = the unit vector of the variable) */
        for (int c = 0; c < (s->gcb ? nvk : 0); ++c) {
            const int q = c < nvk - s->ns ? k * nu + c : N * nu + k; /* stage column iu + c: controls, then slack */
            double D, rhs;
            bound_row(s, q, mode, dw, &D, &rhs);
            HH(iu + c, iu + c) += D;
            g[iu + c] += rhs;
        }
        /* eliminated inequality slacks t (IPOPT d(x) - t = 0, t >= 0) */
        for (int j = 0; j < M; ++j) {
            double J[ZMAX];
            memset(J, 0, sizeof J);
            for (int a = 0; a < 3 && a < nx; ++a) J[a] = s->Jd[(k * M + j) * 3 + a];
            if (s->sd) J[is] = 1.0;
            double D, rhs;
            double t = s->T[k * M + j], v = s->vt[k * M + j];
            if (mode == MODE_NEWTON && s->resto) {
                /* t, p and n of the row eliminated: y~ = (J dz + r - E) / C (restoration) */
                const int r = row_q(s, k * M + j);
                const double pp = s->rp[r], nn = s->rn[r], st = v / t + dw;
                const double sp = s->rzp[r] / pp + dw, sn = s->rzn[r] / nn + dw;
                const double C = 1.0 / st + 1.0 / sp + 1.0 / sn;
                const double E = (mu / t - kappa_d * mu) / st + (mu / pp - s->rho - kappa_d * mu) / sp -
                                 (mu / nn - s->rho - kappa_d * mu) / sn;
                D = 1.0 / C;
                rhs = (s->rcq[k * M + j] - E) / C;
            } else if (mode == MODE_NEWTON) {
                D = v / t + dw;
                rhs = D * s->rcq[k * M + j] + (-mu / t + kappa_d * mu);
            } else {
                D = 1.0;
                rhs = -v;
            }
            for (int a = 0; a < nzk; ++a) {
                g[a] += J[a] * rhs;
                for (int b = 0; b < nzk; ++b) HH(a, b) += D * J[a] * J[b];
            }
        }
#undef HH
    }
    if (mode == MODE_NEWTON) {
        if (s->resto) /* soft equality rows: J dz - D y~ = -r + e (p, n eliminated) */
            for (int i = 0; i < row_q(s, 0); ++i) {
                const double pp = s->rp[i], nn = s->rn[i];
                const double sp = s->rzp[i] / pp + dw, sn = s->rzn[i] / nn + dw;
                s->Dsoft[i] = 1.0 / sp + 1.0 / sn;
                s->esoft[i] = (mu / pp - s->rho - kappa_d * mu) / sp - (mu / nn - s->rho - kappa_d * mu) / sn;
            }
        for (int i = 0; i < nx; ++i) s->dx0[i] = -s->rci[i] + (s->resto ? s->esoft[i] : 0.0);
        for (int j = 0; j < s->nc; ++j) s->rN[j] = -s->rct[j] + (s->resto ? s->esoft[row_t(s, j)] : 0.0);
        for (int k = 0; k < N; ++k)
            for (int i = 0; i < nx; ++i)
                s->cdef[k * nx + i] = -s->rcd[k * nx + i] + (s->resto ? s->esoft[row_d(s, k, i)] : 0.0);
    } else {
        memset(s->dx0, 0, sizeof s->dx0);
        memset(s->rN, 0, sizeof s->rN);
        memset(s->cdef, 0, sizeof(double) * N * nx);
    }
}

/* Cross block M_k between positions of x_k and x_{k+1} (path length), Newton mode only. */
static void cross(const Sol* s, int mode, int k, double* Mk) {
    int nx = s->nx;
    memset(Mk, 0, sizeof(double) * XMAX * XMAX);
    if (mode != MODE_NEWTON || s->resto) return; /* the restoration objective has no path-length term */
    for (int a = 0; a < 2; ++a)
        for (int b = 0; b < 2; ++b) Mk[a * nx + b] = -s->Gs[4 * k + 2 * a + b];
}

/* Restoration rows (p, n eliminated) make the dynamics / initial-state equalities soft: x' = y + w with
 * cost 1/2 w' D^{-1} w.  Minimising the value function (P, p + G nu, Psi, psi) of x' over w gives the
 * value function of y:  P <- (I + P D)^{-1} P,  [p | G] <- (I + P D)^{-1} [p | G],
 * Psi -= G' D (I + P D)^{-1} G,  psi -= G' D (I + P D)^{-1} p,  computed through the symmetric
 * K = I + S P S (S = D^{1/2}): (I + P D)^{-1} X = S^{-1} K^{-1} S X,  D (I + P D)^{-1} = S K^{-1} S.
 * Returns 1 if K is not positive definite (D^{-1} + P indefinite: wrong inertia). */
static int soft_transform(int nx, int nc, const double* D, double* P, double* pv, double* G, double* Psi,
                          double* psi) {
    double S[XMAX], K[XMAX * XMAX], Z[XMAX * (XMAX + 1 + CMAX)];
    int perm[XMAX], nneg, m = nx + 1 + nc;
    for (int i = 0; i < nx; ++i) S[i] = sqrt(D[i]);
    for (int i = 0; i < nx; ++i)
        for (int j = 0; j < nx; ++j) K[i * nx + j] = (i == j ? 1.0 : 0.0) + S[i] * P[i * nx + j] * S[j];
    if (ldl(K, nx, perm, &nneg) || nneg) return 1;
    for (int i = 0; i < nx; ++i) {
        for (int j = 0; j < nx; ++j) Z[i * m + j] = S[i] * P[i * nx + j];
        Z[i * m + nx] = S[i] * pv[i];
        for (int c = 0; c < nc; ++c) Z[i * m + nx + 1 + c] = S[i] * G[i * nc + c];
    }
    ldl_solve(K, nx, perm, Z, m); /* Z = K^{-1} S [P | p | G] */
    for (int a = 0; a < nc; ++a) {
        double t = 0;
        for (int r = 0; r < nx; ++r) t += S[r] * G[r * nc + a] * Z[r * m + nx];
        psi[a] -= t;
        for (int b = 0; b < nc; ++b) {
            double u = 0;
            for (int r = 0; r < nx; ++r) u += S[r] * G[r * nc + a] * Z[r * m + nx + 1 + b];
            Psi[a * nc + b] -= u;
        }
    }
    for (int i = 0; i < nx; ++i) {
        for (int j = 0; j < nx; ++j) P[i * nx + j] = Z[i * m + j] / S[i];
        pv[i] = Z[i * m + nx] / S[i];
        for (int c = 0; c < nc; ++c) G[i * nc + c] = Z[i * m + nx + 1 + c] / S[i];
    }
    for (int i = 0; i < nx; ++i)
        for (int j = 0; j < i; ++j) P[i * nx + j] = P[j * nx + i] = 0.5 * (P[i * nx + j] + P[j * nx + i]);
    return 0;
}
/* x' = y + w* = S K^{-1} (S^{-1} y - S (p + G nu)) for the value function (P, p, G) of x' (untransformed). */
static void soft_forward(int nx, int nc, const double* D, const double* P, const double* pv, const double* G,
                         const double* nu, const double* y, double* xo) {
    double S[XMAX], K[XMAX * XMAX], r[XMAX];
    int perm[XMAX], nneg;
    for (int i = 0; i < nx; ++i) S[i] = sqrt(D[i]);
    for (int i = 0; i < nx; ++i)
        for (int j = 0; j < nx; ++j) K[i * nx + j] = (i == j ? 1.0 : 0.0) + S[i] * P[i * nx + j] * S[j];
    ldl(K, nx, perm, &nneg);
    for (int i = 0; i < nx; ++i) {
        double q = pv[i];
        for (int c = 0; c < nc; ++c) q += G[i * nc + c] * nu[c];
        r[i] = y[i] / S[i] - S[i] * q;
    }
    ldl_solve(K, nx, perm, r, 1);
    for (int i = 0; i < nx; ++i) xo[i] = S[i] * r[i];
}

/* Backward Riccati + terminal multiplier + forward sweep.  Returns 0, or 1 for wrong inertia. */
static int riccati(Sol* s, int mode) {
    int nx = s->nx, nu = s->nu, N = s->N, nc = s->nc, negsum = 0;
    double Pn[XMAX * XMAX], pn[XMAX], Gn[XMAX * CMAX], Psi[CMAX * CMAX], psi[CMAX];
    memset(Pn, 0, sizeof Pn);
    memset(pn, 0, sizeof pn);
    memset(Gn, 0, sizeof Gn);
    memset(Psi, 0, sizeof Psi);
    memset(psi, 0, sizeof psi);
    for (int k = N; k >= 0; --k) {
        int nv = nv_of(s, k), nz = nx + nv;
        double Hp[ZMAX * ZMAX], gp[ZMAX], Ak[XMAX * XMAX], Bk[XMAX * VMAX], ck[XMAX];
        memcpy(Hp, s->H + (size_t)k * ZMAX * ZMAX, sizeof(double) * nz * nz);
        memcpy(gp, s->g + (size_t)k * ZMAX, sizeof(double) * nz);
        memset(Ak, 0, sizeof Ak);
        memset(Bk, 0, sizeof Bk);
        memset(ck, 0, sizeof ck);
        if (k < N) {
            memcpy(Ak, s->A + (size_t)k * nx * nx, sizeof(double) * nx * nx);
            for (int i = 0; i < nx; ++i)
                for (int j = 0; j < nu; ++j) Bk[i * nv + j] = s->B[(size_t)k * nx * nu + i * nu + j];
            memcpy(ck, s->cdef + (size_t)k * nx, sizeof(double) * nx);
            /* substitute dx_{k+1} = A dx + B dv + c into the cross term dx_k' M_k dx_{k+1} */
            double Mk[XMAX * XMAX];
            cross(s, mode, k, Mk);
            double MA[XMAX * XMAX], MB[XMAX * VMAX], Mc[XMAX];
            for (int i = 0; i < nx; ++i) {
                for (int j = 0; j < nx; ++j) {
                    double t = 0;
                    for (int q = 0; q < nx; ++q) t += Mk[i * nx + q] * Ak[q * nx + j];
                    MA[i * nx + j] = t;
                }
                for (int j = 0; j < nv; ++j) {
                    double t = 0;
                    for (int q = 0; q < nx; ++q) t += Mk[i * nx + q] * Bk[q * nv + j];
                    MB[i * nv + j] = t;
                }
                double t = 0;
                for (int q = 0; q < nx; ++q) t += Mk[i * nx + q] * ck[q];
                Mc[i] = t;
            }
            for (int i = 0; i < nx; ++i) {
                for (int j = 0; j < nx; ++j) Hp[i * nz + j] += MA[i * nx + j] + MA[j * nx + i];
                for (int j = 0; j < nv; ++j) {
                    Hp[i * nz + nx + j] += MB[i * nv + j];
                    Hp[(nx + j) * nz + i] += MB[i * nv + j];
                }
                gp[i] += Mc[i];
            }
        }
        if (s->resto && k < N && soft_transform(nx, nc, s->Dsoft + row_d(s, k, 0), Pn, pn, Gn, Psi, psi)) return 1;
        /* Q = H' + [A B]' P [A B] ; q = g' + [A B]'(P c + p) */
        double AB[XMAX * ZMAX], PAB[XMAX * ZMAX], Pcp[XMAX];
        for (int i = 0; i < nx; ++i) {
            for (int j = 0; j < nx; ++j) AB[i * nz + j] = Ak[i * nx + j];
            for (int j = 0; j < nv; ++j) AB[i * nz + nx + j] = Bk[i * nv + j];
        }
        for (int i = 0; i < nx; ++i) {
            for (int j = 0; j < nz; ++j) {
                double t = 0;
                for (int q = 0; q < nx; ++q) t += Pn[i * nx + q] * AB[q * nz + j];
                PAB[i * nz + j] = t;
            }
            double t = pn[i];
            for (int q = 0; q < nx; ++q) t += Pn[i * nx + q] * ck[q];
            Pcp[i] = t;
        }
        double Q[ZMAX * ZMAX], q[ZMAX], QN[ZMAX * CMAX];
        for (int i = 0; i < nz; ++i) {
            for (int j = 0; j < nz; ++j) {
                double t = Hp[i * nz + j];
                for (int r = 0; r < nx; ++r) t += AB[r * nz + i] * PAB[r * nz + j];
                Q[i * nz + j] = t;
            }
            double t = gp[i];
            for (int r = 0; r < nx; ++r) t += AB[r * nz + i] * Pcp[r];
            q[i] = t;
            for (int c = 0; c < nc; ++c) {
                double u = 0;
                for (int r = 0; r < nx; ++r) u += AB[r * nz + i] * Gn[r * nc + c];
                QN[i * nc + c] = u;
            }
        }
        /* factor Q_vv, feedback gains */
        double L[VMAX * VMAX], Kk[VMAX * XMAX], kk[VMAX], Knk[VMAX * CMAX];
        if (nv > 0) {
            for (int i = 0; i < nv; ++i)
                for (int j = 0; j < nv; ++j) L[i * nv + j] = Q[(nx + i) * nz + nx + j];
            /* inertia: pivoted LDL^T counts the negative eigenvalues of each
             * stage block; with Psi_0 below this gives the exact inertia of the Newton matrix. */
            int perm[VMAX], nneg;
            if (ldl(L, nv, perm, &nneg)) return 1; /* singular stage block */
            if (s->resto && nneg) return 1;        /* every constraint is soft: the Hessian must be PD */
            negsum += nneg;
            if (negsum > nc) return 1; /* more negatives than the terminal block can absorb */
            for (int i = 0; i < nv; ++i) {
                for (int j = 0; j < nx; ++j) Kk[i * nx + j] = -Q[(nx + i) * nz + j];
                kk[i] = -q[nx + i];
                for (int c = 0; c < nc; ++c) Knk[i * nc + c] = -QN[(nx + i) * nc + c];
            }
            ldl_solve(L, nv, perm, Kk, nx);
            ldl_solve(L, nv, perm, kk, 1);
            if (nc) ldl_solve(L, nv, perm, Knk, nc);
        }
        memcpy(s->Kf + (size_t)k * VMAX * XMAX, Kk, sizeof(double) * VMAX * XMAX);
        memcpy(s->kf + (size_t)k * VMAX, kk, sizeof(double) * VMAX);
        memcpy(s->Kn + (size_t)k * VMAX * CMAX, Knk, sizeof(double) * VMAX * CMAX);
        /* value function of stage k */
        double P[XMAX * XMAX], pp[XMAX], G[XMAX * CMAX];
        for (int i = 0; i < nx; ++i) {
            for (int j = 0; j < nx; ++j) {
                double t = Q[i * nz + j];
                for (int v = 0; v < nv; ++v) t += Q[i * nz + nx + v] * Kk[v * nx + j];
                P[i * nx + j] = t;
            }
            double t = q[i];
            for (int v = 0; v < nv; ++v) t += Q[i * nz + nx + v] * kk[v];
            pp[i] = t;
            for (int c = 0; c < nc; ++c) {
                double u = QN[i * nc + c];
                for (int v = 0; v < nv; ++v) u += Q[i * nz + nx + v] * Knk[v * nc + c];
                G[i * nc + c] = u;
            }
        }
        for (int i = 0; i < nx; ++i)
            for (int j = 0; j < i; ++j) {
                double a = 0.5 * (P[i * nx + j] + P[j * nx + i]);
                P[i * nx + j] = P[j * nx + i] = a;
            }
        for (int a = 0; a < nc; ++a) {
            for (int b = 0; b < nc; ++b) {
                double t = 0;
                for (int v = 0; v < nv; ++v) t += QN[(nx + v) * nc + a] * Knk[v * nc + b];
                Psi[a * nc + b] += t;
            }
            double t = 0;
            for (int r = 0; r < nx; ++r) t += Gn[r * nc + a] * ck[r];
            for (int v = 0; v < nv; ++v) t += QN[(nx + v) * nc + a] * kk[v];
            psi[a] += t;
        }
        if (k == N) { /* terminal equality C x_N = xg_sel enters here */
            memset(G, 0, sizeof G);
            for (int c = 0; c < nc; ++c) {
                G[s->tidx[c] * nc + c] = 1.0;
                psi[c] = -s->rN[c];
            }
        }
        memcpy(s->Pm + (size_t)k * XMAX * XMAX, P, sizeof P);
        memcpy(s->pv + (size_t)k * XMAX, pp, sizeof pp);
        memcpy(s->Gm + (size_t)k * XMAX * CMAX, G, sizeof G);
        memcpy(Pn, P, sizeof P);
        memcpy(pn, pp, sizeof pp);
        memcpy(Gn, G, sizeof G);
    }
    /* terminal multiplier: -Psi_0 nu = Gamma_0' dx0 + psi_0 (IPOPT delta_c if singular) */
    double nu_[CMAX];
    s->dc_used = 0.0;
    if (s->resto && soft_transform(nx, nc, s->Dsoft, Pn, pn, Gn, Psi, psi)) return 1; /* soft initial state */
    if (s->resto) { /* soft terminal rows: (-Psi + D_t) nu = Gamma' dx0 + psi, positive definite */
        double L[CMAX * CMAX];
        int perm[CMAX], nneg;
        for (int i = 0; i < nc * nc; ++i) L[i] = -Psi[i];
        for (int i = 0; i < nc; ++i) L[i * nc + i] += s->Dsoft[row_t(s, i)];
        if (ldl(L, nc, perm, &nneg) || nneg) return 1;
        for (int c = 0; c < nc; ++c) {
            double t = psi[c];
            for (int r = 0; r < nx; ++r) t += Gn[r * nc + c] * s->dx0[r];
            nu_[c] = t;
        }
        ldl_solve(L, nc, perm, nu_, 1);
    } else if (nc) {
        /* inertia (Sylvester over the Riccati eliminations): the Newton matrix has the wanted
         * inertia iff #neg(Psi_0) = nc - sum_k #neg(Q_vv,k) and Psi_0 is nonsingular. */
        double L[CMAX * CMAX];
        int perm[CMAX], nneg;
        for (int i = 0; i < nc * nc; ++i) L[i] = -Psi[i];
        int st = ldl(L, nc, perm, &nneg); /* nneg counts negatives of -Psi = positives of Psi */
        if (st == 2 || nneg != negsum) {
            /* (near-)rank-deficient terminal block (e.g. no lateral motion of a unicycle at v = 0):
             * IPOPT's delta_c on those rows; a genuine inertia defect survives it. */
            double dc = 1e-8 * pow(s->mu_dc, 0.25); /* delta_c from the iterate's mu */
            for (int i = 0; i < nc * nc; ++i) L[i] = -Psi[i];
            for (int i = 0; i < nc; ++i) L[i * nc + i] += dc;
            if (ldl(L, nc, perm, &nneg)) return 1;
            if (nneg != negsum) return 1; /* wrong inertia */
            s->dc_used = dc;
        }
        for (int c = 0; c < nc; ++c) {
            double t = psi[c];
            for (int r = 0; r < nx; ++r) t += Gn[r * nc + c] * s->dx0[r];
            nu_[c] = t;
        }
        ldl_solve(L, nc, perm, nu_, 1);
    } else if (negsum) {
        return 1;
    }
    /* forward sweep */
    double dx[XMAX];
    memcpy(dx, s->dx0, sizeof(double) * nx);
    if (s->resto) soft_forward(nx, nc, s->Dsoft, s->Pm, s->pv, s->Gm, nu_, s->dx0, dx);
    for (int k = 0; k <= N; ++k) {
        int nv = nv_of(s, k);
        const double *Kk = s->Kf + (size_t)k * VMAX * XMAX, *kk = s->kf + (size_t)k * VMAX,
                     *Knk = s->Kn + (size_t)k * VMAX * CMAX;
        double dvv[VMAX];
        for (int v = 0; v < nv; ++v) {
            double t = kk[v];
            for (int j = 0; j < nx; ++j) t += Kk[v * nx + j] * dx[j];
            for (int c = 0; c < nc; ++c) t += Knk[v * nc + c] * nu_[c];
            dvv[v] = t;
        }
        memcpy(s->dX + k * nx, dx, sizeof(double) * nx);
        if (k < N)
            for (int i = 0; i < nu; ++i) s->dU[k * nu + i] = dvv[i];
        if (s->ns) s->dS[k] = dvv[nv - 1];
        if (k == 0) { /* initial-state multiplier */
            const double *P = s->Pm, *pp = s->pv, *G = s->Gm;
            for (int i = 0; i < nx; ++i) {
                double t = pp[i];
                for (int j = 0; j < nx; ++j) t += P[i * nx + j] * dx[j];
                for (int c = 0; c < nc; ++c) t += G[i * nc + c] * nu_[c];
                s->yi_n[i] = -t;
            }
        }
        if (k < N) {
            double dn[XMAX];
            const double* Ak = s->A + (size_t)k * nx * nx;
            for (int i = 0; i < nx; ++i) {
                double t = s->cdef[k * nx + i];
                for (int j = 0; j < nx; ++j) t += Ak[i * nx + j] * dx[j];
                for (int j = 0; j < nu; ++j) t += s->B[(size_t)k * nx * nu + i * nu + j] * dvv[j];
                dn[i] = t;
            }
            if (s->resto) { /* soft dynamics: dx_{k+1} = y + w* */
                double y_[XMAX];
                memcpy(y_, dn, sizeof(double) * nx);
                soft_forward(nx, nc, s->Dsoft + row_d(s, k, 0), s->Pm + (size_t)(k + 1) * XMAX * XMAX,
                             s->pv + (size_t)(k + 1) * XMAX, s->Gm + (size_t)(k + 1) * XMAX * CMAX, nu_, y_, dn);
            }
            /* dynamics multiplier y_k = -grad V_{k+1}(dx_{k+1}) - M_k' dx_k */
            const double *P = s->Pm + (size_t)(k + 1) * XMAX * XMAX, *pp = s->pv + (size_t)(k + 1) * XMAX,
                         *G = s->Gm + (size_t)(k + 1) * XMAX * CMAX;
            double Mk[XMAX * XMAX];
            cross(s, mode, k, Mk);
            for (int i = 0; i < nx; ++i) {
                double t = pp[i];
                for (int j = 0; j < nx; ++j) t += P[i * nx + j] * dn[j];
                for (int c = 0; c < nc; ++c) t += G[i * nc + c] * nu_[c];
                double mt = 0;
                for (int j = 0; j < nx; ++j) mt += Mk[j * nx + i] * dx[j];
                s->yk_n[k * nx + i] = -t - mt;
            }
            memcpy(dx, dn, sizeof(double) * nx);
        }
    }
    for (int c = 0; c < nc; ++c) s->yt_n[c] = nu_[c];
    return 0;
}

/* Max residual of the full (unsubstituted) linear KKT system for the computed step (debug). */
static double linear_residual(Sol* s, int mode) {
    int nx = s->nx, nu = s->nu, N = s->N, nc = s->nc;
    double res = 0;
    for (int k = 0; k <= N; ++k) {
        int nv = nv_of(s, k), nz = nx + nv;
        double z[ZMAX], r[ZMAX];
        for (int i = 0; i < nx; ++i) z[i] = s->dX[k * nx + i];
        if (k < N)
            for (int i = 0; i < nu; ++i) z[nx + i] = s->dU[k * nu + i];
        if (s->ns) z[nz - 1] = s->dS[k];
        const double* H = s->H + (size_t)k * ZMAX * ZMAX;
        for (int i = 0; i < nz; ++i) {
            double t = s->g[(size_t)k * ZMAX + i];
            for (int j = 0; j < nz; ++j) t += H[i * nz + j] * z[j];
            r[i] = t;
        }
        double Mk[XMAX * XMAX];
        if (k < N) {
            cross(s, mode, k, Mk);
            for (int i = 0; i < nx; ++i)
                for (int j = 0; j < nx; ++j) r[i] += Mk[i * nx + j] * s->dX[(k + 1) * nx + j];
        }
        if (k > 0) {
            cross(s, mode, k - 1, Mk);
            for (int i = 0; i < nx; ++i)
                for (int j = 0; j < nx; ++j) r[i] += Mk[j * nx + i] * s->dX[(k - 1) * nx + j];
            for (int i = 0; i < nx; ++i) r[i] += s->yk_n[(k - 1) * nx + i];
        }
        if (k < N) {
            for (int j = 0; j < nx; ++j)
                for (int i = 0; i < nx; ++i) r[j] -= s->A[(size_t)k * nx * nx + i * nx + j] * s->yk_n[k * nx + i];
            for (int j = 0; j < nu; ++j)
                for (int i = 0; i < nx; ++i) r[nx + j] -= s->B[(size_t)k * nx * nu + i * nu + j] * s->yk_n[k * nx + i];
        }
        if (k == 0)
            for (int i = 0; i < nx; ++i) r[i] += s->yi_n[i];
        if (k == N)
            for (int c = 0; c < nc; ++c) r[s->tidx[c]] += s->yt_n[c];
        for (int i = 0; i < nz; ++i) res = fmax(res, fabs(r[i]));
    }
    for (int i = 0; i < nx; ++i) res = fmax(res, fabs(s->dX[i] - s->dx0[i]));
    for (int k = 0; k < N; ++k)
        for (int i = 0; i < nx; ++i) {
            double t = s->dX[(k + 1) * nx + i] - s->cdef[k * nx + i];
            for (int j = 0; j < nx; ++j) t -= s->A[(size_t)k * nx * nx + i * nx + j] * s->dX[k * nx + j];
            for (int j = 0; j < nu; ++j) t -= s->B[(size_t)k * nx * nu + i * nu + j] * s->dU[k * nu + j];
            res = fmax(res, fabs(t));
        }
    for (int c = 0; c < nc; ++c) /* regularised row: C dx - dc nu = rN */
        res = fmax(res, fabs(s->dX[N * nx + s->tidx[c]] - s->dc_used * s->yt_n[c] - s->rN[c]));
    return res;
}

/* Recover dt, yd+, dz from the primal step (Newton mode); in the restoration problem also dp, dn, dzp, dzn. */
static void recover(Sol* s, double dw) {
    const NlotProblem* p = s->p;
    int nx = s->nx, nu = s->nu, N = s->N, M = s->M;
    const double kappa_d = 1e-5;
    double mu = s->mu;
    /* p, n of one restoration row given its new multiplier y~ */
    #define PN_STEP(r, yn)                                                                                 \
    do {                                                                                                   \
        const double pp_ = s->rp[r], nn_ = s->rn[r];                                                       \
        const double sp_ = s->rzp[r] / pp_ + dw, sn_ = s->rzn[r] / nn_ + dw;                               \
        s->rdp[r] = ((yn) - s->rho - kappa_d * mu + mu / pp_) / sp_;                                       \
        s->rdn[r] = (-(yn) - s->rho - kappa_d * mu + mu / nn_) / sn_;                                      \
        s->rdzp[r] = mu / pp_ - s->rzp[r] - (s->rzp[r] / pp_) * s->rdp[r];                                 \
        s->rdzn[r] = mu / nn_ - s->rzn[r] - (s->rzn[r] / nn_) * s->rdn[r];                                 \
    } while (0)
    for (int k = 0; k <= N; ++k)
        for (int j = 0; j < M; ++j) {
            int q = k * M + j;
            double Jdz = 0;
            for (int a = 0; a < 3 && a < nx; ++a) Jdz += s->Jd[q * 3 + a] * s->dX[k * nx + a];
            if (s->sd) Jdz += s->dS[k];
            double t = s->T[q], v = s->vt[q];
            if (s->resto) {
                const int r = row_q(s, q);
                const double pp = s->rp[r], nn = s->rn[r], st = v / t + dw;
                const double sp = s->rzp[r] / pp + dw, sn = s->rzn[r] / nn + dw;
                const double C = 1.0 / st + 1.0 / sp + 1.0 / sn;
                const double E = (mu / t - kappa_d * mu) / st + (mu / pp - s->rho - kappa_d * mu) / sp -
                                 (mu / nn - s->rho - kappa_d * mu) / sn;
                const double yn = (Jdz + s->rcq[q] - E) / C;
                s->yd_n[q] = yn;
                s->dT[q] = (yn + mu / t - kappa_d * mu) / st;
                PN_STEP(r, yn);
            } else {
                double dt = Jdz + s->rcq[q];
                s->dT[q] = dt;
                s->yd_n[q] = (v / t + dw) * dt + (-mu / t + kappa_d * mu);
            }
            s->dvt[q] = mu / t - v - (v / t) * s->dT[q];
        }
    if (s->resto) {
        for (int i = 0; i < nx; ++i) PN_STEP(i, s->yi_n[i]);
        for (int k = 0; k < N; ++k)
            for (int i = 0; i < nx; ++i) PN_STEP(row_d(s, k, i), s->yk_n[k * nx + i]);
        for (int j = 0; j < s->nc; ++j) PN_STEP(row_t(s, j), s->yt_n[j]);
    }
    /* general_bounds: the bound rows' slack step, row multiplier and slack bound multipliers */
    for (int q = 0; q < s->nb; ++q) {
        const double dvar = bvar(s, s->dU, s->dS, q);
        double Sig, bg;
        bound_sig(s, q, &Sig, &bg);
        const double st = Sig + dw;
        if (s->resto) {
            double D, rhs;
            bound_row(s, q, MODE_NEWTON, dw, &D, &rhs);
            const double yn = D * dvar + rhs; /* (J dz + r - E) / C */
            s->yb_n[q] = yn;
            s->dsb[q] = (yn - bg) / st;
            PN_STEP(row_b(s, q), yn);
        } else {
            s->dsb[q] = dvar + s->rcb[q];
            s->yb_n[q] = st * s->dsb[q] + bg;
        }
        const double sl = s->sb[q] - blo(s, q);
        s->dzbl[q] = mu / sl - s->zbl[q] - (s->zbl[q] / sl) * s->dsb[q];
        if (bhi_on(s, q)) {
            const double su = bhi(s, q) - s->sb[q];
            s->dzbu[q] = mu / su - s->zbu[q] + (s->zbu[q] / su) * s->dsb[q];
        } else {
            s->dzbu[q] = 0.0;
        }
    }
    #undef PN_STEP
    if (s->gcb) return;
    for (int k = 0; k < N; ++k)
        for (int i = 0; i < nu; ++i) {
            int q = k * nu + i;
            double sl = s->U[q] - p->umin[i], su = p->umax[i] - s->U[q], du = s->dU[q];
            s->dzl[q] = mu / sl - s->zl[q] - (s->zl[q] / sl) * du;
            s->dzu[q] = mu / su - s->zu[q] + (s->zu[q] / su) * du;
        }
    if (s->ns)
        for (int k = 0; k <= N; ++k) s->dzs[k] = mu / (s->S[k] + s->brel) - s->zs[k] - (s->zs[k] / (s->S[k] + s->brel)) * s->dS[k];
}

/* ============================================================================================ */
/* IPOPT main loop (restated)                                                                   */
/* ============================================================================================ */
static double frac_to_bound(double sl, double dsl, double tau, double amax) {
    if (dsl < 0) {
        double a = -tau * sl / dsl;
        if (a < amax) return a;
    }
    return amax;
}

static int cmp_le(double lhs, double rhs, double bas) { /* IPOPT Compare_le */
    return lhs - rhs <= 10.0 * DBL_EPSILON * fabs(bas);
}

static void filter_add(Sol* s, double theta, double phi) {
    const double gt = 1e-5, gp = 1e-8;
    double nt = (1.0 - gt) * theta, np = phi - gp * theta;
    int w = 0;
    for (int i = 0; i < s->nfilt; ++i) /* drop entries dominated by the new one */
        if (!(s->filt_theta[i] >= nt && s->filt_phi[i] >= np)) {
            s->filt_theta[w] = s->filt_theta[i];
            s->filt_phi[w] = s->filt_phi[i];
            ++w;
        }
    s->nfilt = w;
    if (s->nfilt == s->fcap) { /* only under NLOT_ORACLE_FILT_CAP: forget the oldest entry */
        memmove(s->filt_theta, s->filt_theta + 1, sizeof(double) * (s->fcap - 1));
        memmove(s->filt_phi, s->filt_phi + 1, sizeof(double) * (s->fcap - 1));
        s->nfilt--;
        s->filt_ovf++;
    }
    s->filt_theta[s->nfilt] = nt;
    s->filt_phi[s->nfilt] = np;
    s->nfilt++;
    if (s->nfilt > s->max_nfilt) s->max_nfilt = s->nfilt;
}
static int filter_ok(const Sol* s, double theta, double phi) {
    for (int i = 0; i < s->nfilt; ++i)
        if (!(theta <= s->filt_theta[i] || phi <= s->filt_phi[i])) return 0;
    return 1;
}

/* IPOPT filter acceptance of a trial point (FilterLSAcceptor::CheckAcceptabilityOfTrialPoint). */
static int ls_accept(const Sol* s, double theta, double phi, double gd, double alpha, double tht, double pht,
                     int* armijo_ftype) {
    const double gt = 1e-5, gp = 1e-8, delta = 1.0, sth = 1.1, sph = 2.3, eta = 1e-8;
    if (!(isfinite(tht) && isfinite(pht)) || tht > s->theta_max) return 0;
    int ftype = gd < 0 && alpha * pow(-gd, sph) > delta * pow(theta, sth);
    int armijo = cmp_le(pht - phi, eta * alpha * gd, phi);
    int ok;
    if (ftype && theta <= s->theta_min) {
        ok = armijo;
    } else {
        ok = cmp_le(tht, (1.0 - gt) * theta, theta) || cmp_le(pht - phi, -gp * theta, phi);
        if (ok && pht > phi) { /* obj_max_inc = 5 */
            double bas = fabs(phi) > 10.0 ? log10(fabs(phi)) : 1.0;
            if (log10(pht - phi) > 5.0 + bas) ok = 0;
        }
    }
    if (ok) {
        ok = filter_ok(s, tht, pht);
        ((Sol*)s)->rej_filter = !ok; /* rejected by the filter after the sufficient-decrease test passed */
    } else {
        ((Sol*)s)->rej_filter = 0;
    }
    if (ok) *armijo_ftype = ftype && armijo;
    return ok;
}

static double primal_frac(const Sol* s, double tau) {
    const NlotProblem* p = s->p;
    int nu = s->nu, N = s->N, M = s->M;
    double a = 1.0;
    for (int k = 0; k < (s->gcb ? 0 : N); ++k)
        for (int i = 0; i < nu; ++i) {
            int q = k * nu + i;
            a = frac_to_bound(s->U[q] - p->umin[i], s->dU[q], tau, a);
            a = frac_to_bound(p->umax[i] - s->U[q], -s->dU[q], tau, a);
        }
    if (s->ns && !s->gcb)
        for (int k = 0; k <= N; ++k) a = frac_to_bound(s->S[k] + s->brel, s->dS[k], tau, a);
    for (int q = 0; q < s->nb; ++q) {
        a = frac_to_bound(s->sb[q] - blo(s, q), s->dsb[q], tau, a);
        if (bhi_on(s, q)) a = frac_to_bound(bhi(s, q) - s->sb[q], -s->dsb[q], tau, a);
    }
    for (int q = 0; q < (N + 1) * M; ++q) a = frac_to_bound(s->T[q], s->dT[q], tau, a);
    if (s->resto)
        for (int i = 0; i < s->ne; ++i) {
            a = frac_to_bound(s->rp[i], s->rdp[i], tau, a);
            a = frac_to_bound(s->rn[i], s->rdn[i], tau, a);
        }
    return a;
}
static double dual_frac(const Sol* s, double tau) {
    int nu = s->nu, N = s->N, M = s->M;
    double a = 1.0;
    for (int q = 0; q < (s->gcb ? 0 : N * nu); ++q) {
        a = frac_to_bound(s->zl[q], s->dzl[q], tau, a);
        a = frac_to_bound(s->zu[q], s->dzu[q], tau, a);
    }
    if (s->ns && !s->gcb)
        for (int k = 0; k <= N; ++k) a = frac_to_bound(s->zs[k], s->dzs[k], tau, a);
    for (int q = 0; q < s->nb; ++q) {
        a = frac_to_bound(s->zbl[q], s->dzbl[q], tau, a);
        if (bhi_on(s, q)) a = frac_to_bound(s->zbu[q], s->dzbu[q], tau, a);
    }
    for (int q = 0; q < (N + 1) * M; ++q) a = frac_to_bound(s->vt[q], s->dvt[q], tau, a);
    if (s->resto)
        for (int i = 0; i < s->ne; ++i) {
            a = frac_to_bound(s->rzp[i], s->rdzp[i], tau, a);
            a = frac_to_bound(s->rzn[i], s->rdzn[i], tau, a);
        }
    return a;
}
/* the full step: its arrays and their lengths (step_len doubles in all) */
#define STEP_ARRAYS(s_)                                                                                            \
    double* arrs[] = {s_->dX,  s_->dU,  s_->dS,  s_->dT,  s_->yi_n, s_->yk_n, s_->yt_n, s_->yd_n,                  \
                      s_->dzl, s_->dzu, s_->dzs, s_->dvt, s_->dsb,  s_->yb_n, s_->dzbl, s_->dzbu};                 \
    int lens[] = {(N + 1) * nx, N * nu, N + 1, (N + 1) * M, nx, N * nx, CMAX, (N + 1) * M, N * nu, N * nu, N + 1,   \
                  (N + 1) * M, s_->nb, s_->nb, s_->nb, s_->nb};
static int step_len(const Sol* s) {
    int nx = s->nx, nu = s->nu, N = s->N, M = s->M;
    return (N + 1) * nx + 3 * N * nu + 2 * (N + 1) + 3 * (N + 1) * M + nx + N * nx + CMAX + 4 * s->nb;
}
/* save (dir=0) / restore (dir=1) the full step */
static void step_save(Sol* s, double* buf, int dir) {
    int nx = s->nx, nu = s->nu, N = s->N, M = s->M;
    STEP_ARRAYS(s)
    for (int i = 0; i < 16; ++i) {
        if (dir == 0) memcpy(buf, arrs[i], sizeof(double) * lens[i]);
        else memcpy(arrs[i], buf, sizeof(double) * lens[i]);
        buf += lens[i];
    }
}
static void res_save(Sol* s, double* buf, int dir) {
    int nx = s->nx, N = s->N, M = s->M;
    double* arrs[] = {s->rci, s->rcd, s->rct, s->rcq, s->rcb};
    int lens[] = {XMAX, N * nx, CMAX, (N + 1) * M, s->nb};
    for (int i = 0; i < 5; ++i) {
        if (dir == 0) memcpy(buf, arrs[i], sizeof(double) * lens[i]);
        else memcpy(arrs[i], buf, sizeof(double) * lens[i]);
        buf += lens[i];
    }
}


/* ============================================================================================ */
/* Adaptive barrier update (runner.py:118-121: mu_strategy "adaptive", mu_oracle                */
/* "quality-function", barrier_tol_factor 0.05) — restated from IPOPT 3.14's AdaptiveMuUpdate   */
/* and QualityFunctionMuOracle (Nocedal, Waechter, Waltz, SIAM J. Optim. 19(4), 2009) with      */
/* IPOPT's defaults: adaptive_mu_globalization obj-constr-filter (filter_margin_fact 1e-5,      */
/* filter_max_margin 1), adaptive_mu_monotone_init_factor 0.8, mu_max_fact 1e3, mu_min 1e-11,   */
/* sigma in [1e-6, 1e2], quality_function_norm_type 2-norm-squared, no centrality/balancing    */
/* term, quality_function_max_section_steps 8, quality_function_section_sigma_tol 1e-2.         */
/* ============================================================================================ */
#define AMU_MU_MIN 1e-11
static double afilt_margin(double th) { return 1e-5 * fmin(1.0, th); }
static int afilt_acceptable(const Sol* s, double f, double th) {
    const double m = afilt_margin(th);
    for (int i = 0; i < s->nafilt; ++i)
        if (f + m >= s->af_f[i] && th + m >= s->af_th[i]) return 0;
    return 1;
}
static void afilt_add(Sol* s, double f, double th) {
    const double m = afilt_margin(th), nf = f - m, nt = th - m;
    int w = 0;
    for (int i = 0; i < s->nafilt; ++i)
        if (!(s->af_f[i] >= nf && s->af_th[i] >= nt)) {
            s->af_f[w] = s->af_f[i];
            s->af_th[w] = s->af_th[i];
            ++w;
        }
    s->nafilt = w;
    if (s->nafilt == s->fcap) { /* only under NLOT_ORACLE_FILT_CAP: forget the oldest entry */
        memmove(s->af_f, s->af_f + 1, sizeof(double) * (s->fcap - 1));
        memmove(s->af_th, s->af_th + 1, sizeof(double) * (s->fcap - 1));
        s->nafilt--;
        s->afilt_ovf++;
    }
    s->af_f[s->nafilt] = nf;
    s->af_th[s->nafilt] = nt;
    s->nafilt++;
    if (s->nafilt > s->max_nafilt) s->max_nafilt = s->nafilt;
}

/* step = aff + sigma * cen over every step array (layout of step_save) */
static void step_combine(Sol* s, const double* aff, const double* cen, double sigma) {
    int nx = s->nx, nu = s->nu, N = s->N, M = s->M;
    STEP_ARRAYS(s)
    for (int a = 0; a < 16; ++a) {
        for (int i = 0; i < lens[a]; ++i) arrs[a][i] = aff[i] + sigma * cen[i];
        aff += lens[a];
        cen += lens[a];
    }
}

typedef struct {
    const double *aff, *cen;
    double avg;
    const Errs* e;
} QfCtx;

/* quality function q(sigma) of the linearised KKT error after the fraction-to-boundary step */
static double qf_eval(Sol* s, const QfCtx* q, double sigma) {
    const NlotProblem* p = s->p;
    int nu = s->nu, N = s->N, M = s->M;
    step_combine(s, q->aff, q->cen, sigma);
    /* tau inside q(sigma) is a reconstruction; NLOT_ORACLE_QF_TAU=curr uses the current iteration's
     * tau instead (variant) */
    static int tau_curr = -1;
    if (tau_curr < 0) tau_curr = getenv("NLOT_ORACLE_QF_TAU") && !strcmp(getenv("NLOT_ORACLE_QF_TAU"), "curr");
    const double tau = tau_curr ? s->tau : fmax(0.99, 1.0 - sigma * q->avg);
    const double ap = primal_frac(s, tau), ad = dual_frac(s, tau);
    double csq = 0;
#define CQ(sl, dsl, z, dz)                                                                       \
    do {                                                                                         \
        double c_ = ((sl) + ap * (dsl)) * ((z) + ad * (dz));                                     \
        csq += c_ * c_;                                                                          \
    } while (0)
    for (int k = 0; k < (s->gcb ? 0 : N); ++k)
        for (int i = 0; i < nu; ++i) {
            int j = k * nu + i;
            CQ(s->U[j] - p->umin[i], s->dU[j], s->zl[j], s->dzl[j]);
            CQ(p->umax[i] - s->U[j], -s->dU[j], s->zu[j], s->dzu[j]);
        }
    if (s->ns && !s->gcb)
        for (int k = 0; k <= N; ++k) CQ(s->S[k] + s->brel, s->dS[k], s->zs[k], s->dzs[k]);
    for (int q = 0; q < s->nb; ++q) {
        CQ(s->sb[q] - blo(s, q), s->dsb[q], s->zbl[q], s->dzbl[q]);
        if (bhi_on(s, q)) CQ(bhi(s, q) - s->sb[q], -s->dsb[q], s->zbu[q], s->dzbu[q]);
    }
    for (int j = 0; j < (N + 1) * M; ++j) CQ(s->T[j], s->dT[j], s->vt[j], s->dvt[j]);
#undef CQ
    const Errs* e = q->e;
    return (1.0 - ad) * (1.0 - ad) * e->dual_sq / e->n_dual + (1.0 - ap) * (1.0 - ap) * e->primal_sq / e->n_pri +
           csq / e->n_comp;
}

/* golden-section search for the minimiser of q over [lo, up] (sigma space, or log10 sigma);
 * q_lo / q_up < 0 mean "not evaluated yet" (QualityFunctionMuOracle::PerformGoldenSection[Log]) */
static double qf_golden(Sol* s, const QfCtx* q, double sig_up, double q_up, double sig_lo, double q_lo, int lg) {
    const double gfac = (3.0 - sqrt(5.0)) / 2.0;
#define TO_T(x) (lg ? log10(x) : (x))
#define TO_S(t) (lg ? pow(10.0, (t)) : (t))
    const double t_up0 = TO_T(sig_up), t_lo0 = TO_T(sig_lo);
    double up = t_up0, lo = t_lo0;
    double m1 = lo + gfac * (up - lo), m2 = lo + (1.0 - gfac) * (up - lo);
    double q1 = qf_eval(s, q, TO_S(m1)), q2 = qf_eval(s, q, TO_S(m2));
    int n = 0;
    while (n < 8 && (TO_S(up) - TO_S(lo)) >= 1e-2 * TO_S(up)) {
        ++n;
        if (q1 > q2) {
            lo = m1;
            q_lo = q1;
            m1 = m2;
            q1 = q2;
            m2 = lo + (1.0 - gfac) * (up - lo);
            q2 = qf_eval(s, q, TO_S(m2));
        } else {
            up = m2;
            q_up = q2;
            m2 = m1;
            q2 = q1;
            m1 = lo + gfac * (up - lo);
            q1 = qf_eval(s, q, TO_S(m1));
        }
    }
    double sig, qq;
    if (q1 < q2) {
        sig = TO_S(m1);
        qq = q1;
    } else {
        sig = TO_S(m2);
        qq = q2;
    }
    if (up == t_up0) {
        if (q_up < 0) q_up = qf_eval(s, q, TO_S(up));
        if (q_up < qq) sig = TO_S(up);
    } else if (lo == t_lo0) {
        if (q_lo < 0) q_lo = qf_eval(s, q, TO_S(lo));
        if (q_lo < qq) sig = TO_S(lo);
    }
#undef TO_T
#undef TO_S
    return sig;
}

/* QualityFunctionMuOracle::CalculateMu: sigma minimising q, mu = sigma * avg_compl */
static double qf_sigma(Sol* s, const QfCtx* q, double mu_min, double mu_max) {
    const double avg = q->avg;
    const double sig_up = fmin(100.0, mu_max / avg), sig_lo = fmax(1e-6, mu_min / avg);
    if (sig_lo >= sig_up) return sig_up;
    if (sig_up <= 1.0) return qf_golden(s, q, sig_up, -1.0, sig_lo, -1.0, 1);
    if (sig_lo >= 1.0) return qf_golden(s, q, sig_up, -1.0, sig_lo, -1.0, 0);
    const double sig_1m = 1.0 - fmax(1e-4, 1e-2);
    const double q_1m = qf_eval(s, q, sig_1m), q_1 = qf_eval(s, q, 1.0);
    if (q_1m > q_1) return qf_golden(s, q, sig_up, -1.0, 1.0, q_1, 0);
    return qf_golden(s, q, sig_1m, q_1m, fmax(sig_lo, 1e-300), -1.0, 1);
}

/* ============================================================================================ */
/* Globalisation safeguards of IPOPT's BacktrackingLineSearch (restated):           */
/* second-order correction, watchdog, soft restoration, tiny-step test, and the feasibility       */
/* restoration phase (MinC_1NrmRestorationPhase).                                                 */
/* ============================================================================================ */
/* iterate (primal + equality/bound multipliers; restoration p, n, zp, zn) save (dir 0) / load (dir 1) */
static int iter_len(const Sol* s) {
    int nx = s->nx, nu = s->nu, N = s->N, M = s->M;
    return (N + 1) * nx + 3 * N * nu + 2 * (N + 1) + 3 * (N + 1) * M + nx + N * nx + CMAX + 4 * s->ne + 4 * s->nb;
}
static void iter_io(Sol* s, double* buf, int dir) {
    int nx = s->nx, nu = s->nu, N = s->N, M = s->M;
    double* arrs[] = {s->X, s->U, s->S, s->T, s->yi, s->yk, s->yt, s->yd, s->zl, s->zu, s->zs, s->vt,
                      s->rp, s->rn, s->rzp, s->rzn, s->sb, s->yb, s->zbl, s->zbu};
    int lens[] = {(N + 1) * nx, N * nu, N + 1, (N + 1) * M, nx, N * nx, CMAX, (N + 1) * M, N * nu, N * nu, N + 1,
                  (N + 1) * M, s->ne, s->ne, s->ne, s->ne, s->nb, s->nb, s->nb, s->nb};
    for (int i = 0; i < 20; ++i) {
        if (dir == 0) memcpy(buf, arrs[i], sizeof(double) * lens[i]);
        else memcpy(arrs[i], buf, sizeof(double) * lens[i]);
        buf += lens[i];
    }
}

typedef struct { /* trial point buffers */
    double *X, *U, *S, *T, *P, *N, *SB;
} Trial;

static void trial_primal(const Sol* s, double a, Trial* t) {
    int nx = s->nx, nu = s->nu, N = s->N, M = s->M;
    for (int i = 0; i < (N + 1) * nx; ++i) t->X[i] = s->X[i] + a * s->dX[i];
    for (int i = 0; i < N * nu; ++i) t->U[i] = s->U[i] + a * s->dU[i];
    for (int k = 0; k <= N; ++k) t->S[k] = s->S[k] + a * s->dS[k];
    for (int q = 0; q < (N + 1) * M; ++q) t->T[q] = s->T[q] + a * s->dT[q];
    for (int q = 0; q < s->nb; ++q) t->SB[q] = s->sb[q] + a * s->dsb[q];
    if (s->resto)
        for (int i = 0; i < s->ne; ++i) {
            t->P[i] = s->rp[i] + a * s->rdp[i];
            t->N[i] = s->rn[i] + a * s->rdn[i];
        }
}
static void trial_merit(const Sol* s, const Trial* t, double mu, double* th, double* ph, double* rci, double* rcd,
                        double* rct, double* rcq, double* rcb) {
    ((Sol*)s)->n_trials++;
    if (s->resto) merit_resto(s, t->X, t->U, t->S, t->T, t->SB, t->P, t->N, mu, th, ph, rci, rcd, rct, rcq, rcb);
    else merit_r(s, t->X, t->U, t->S, t->T, t->SB, mu, th, ph, rci, rcd, rct, rcq, rcb);
}

/* accept the trial point: primal (and equality multipliers, IPOPT alpha_for_y = primal) with alpha, bound
 * multipliers with alpha_z and the kappa_Sigma safeguard */
static void accept_step(Sol* s, double al, double az, const Trial* t) {
    const NlotProblem* p = s->p;
    int nx = s->nx, nu = s->nu, N = s->N, M = s->M;
    const double mu = s->mu, ks = 1e10;
    memcpy(s->X, t->X, sizeof(double) * (N + 1) * nx);
    memcpy(s->U, t->U, sizeof(double) * N * nu);
    memcpy(s->S, t->S, sizeof(double) * (N + 1));
    memcpy(s->T, t->T, sizeof(double) * (N + 1) * M);
    for (int i = 0; i < nx; ++i) s->yi[i] += al * (s->yi_n[i] - s->yi[i]);
    for (int i = 0; i < N * nx; ++i) s->yk[i] += al * (s->yk_n[i] - s->yk[i]);
    for (int i = 0; i < s->nc; ++i) s->yt[i] += al * (s->yt_n[i] - s->yt[i]);
    for (int i = 0; i < (N + 1) * M; ++i) s->yd[i] += al * (s->yd_n[i] - s->yd[i]);
    memcpy(s->sb, t->SB, sizeof(double) * s->nb);
    for (int i = 0; i < s->nb; ++i) s->yb[i] += al * (s->yb_n[i] - s->yb[i]);
#define ZUPD(z, dz, sl)                                                                          \
    do {                                                                                         \
        double zn = (z) + az * (dz), sv = (sl);                                                  \
        zn = fmax(fmin(zn, ks * mu / sv), mu / (ks * sv));                                       \
        (z) = zn;                                                                                \
    } while (0)
    for (int k = 0; k < (s->gcb ? 0 : N); ++k)
        for (int i = 0; i < nu; ++i) {
            int q = k * nu + i;
            ZUPD(s->zl[q], s->dzl[q], s->U[q] - p->umin[i]);
            ZUPD(s->zu[q], s->dzu[q], p->umax[i] - s->U[q]);
        }
    if (s->ns && !s->gcb)
        for (int k = 0; k <= N; ++k) ZUPD(s->zs[k], s->dzs[k], s->S[k] + s->brel);
    for (int q = 0; q < s->nb; ++q) {
        ZUPD(s->zbl[q], s->dzbl[q], s->sb[q] - blo(s, q));
        if (bhi_on(s, q)) ZUPD(s->zbu[q], s->dzbu[q], bhi(s, q) - s->sb[q]);
    }
    for (int q = 0; q < (N + 1) * M; ++q) ZUPD(s->vt[q], s->dvt[q], s->T[q]);
    if (s->resto) {
        memcpy(s->rp, t->P, sizeof(double) * s->ne);
        memcpy(s->rn, t->N, sizeof(double) * s->ne);
        for (int i = 0; i < s->ne; ++i) {
            ZUPD(s->rzp[i], s->rdzp[i], s->rp[i]);
            ZUPD(s->rzn[i], s->rdzn[i], s->rn[i]);
        }
    }
#undef ZUPD
}

/* directional derivative of the barrier merit along the step (IPOPT gradBarrTDelta) */
static double barrier_gd(const Sol* s) {
    const NlotProblem* p = s->p;
    int nx = s->nx, nu = s->nu, N = s->N, M = s->M;
    const double kappa_d = 1e-5, mu = s->mu;
    double gd = 0;
    for (int i = 0; i < (N + 1) * nx; ++i) gd += s->gX[i] * s->dX[i];
    for (int k = 0; k < N; ++k)
        for (int i = 0; i < nu; ++i) {
            int q = k * nu + i;
            gd += (s->gcb ? s->gU[q] : s->gU[q] - mu / (s->U[q] - p->umin[i]) + mu / (p->umax[i] - s->U[q])) * s->dU[q];
        }
    if (s->ns)
        for (int k = 0; k <= N; ++k) gd += (s->gcb ? s->gS[k] : s->gS[k] - mu / (s->S[k] + s->brel) + kappa_d * mu) * s->dS[k];
    for (int q = 0; q < s->nb; ++q) {
        double Sig, bg;
        bound_sig(s, q, &Sig, &bg);
        gd += bg * s->dsb[q];
    }
    for (int q = 0; q < (N + 1) * M; ++q) gd += (-mu / s->T[q] + kappa_d * mu) * s->dT[q];
    if (s->resto)
        for (int i = 0; i < s->ne; ++i)
            gd += (s->rho + kappa_d * mu - mu / s->rp[i]) * s->rdp[i] + (s->rho + kappa_d * mu - mu / s->rn[i]) * s->rdn[i];
    return gd;
}

/* Newton step with IPOPT's inertia correction (delta_w); 0 ok, 1 failed */
/* NLOT_ORACLE_STEP_JITTER=eps (test infrastructure, tests/test_pinned_iterates_gpu.py): every Newton step's primal
 * components are scaled by 1 +- eps (a fixed pseudo-random sign per component and step): a model of the rounding
 * differences of another fp64 summation order in the KKT solve (the GPU's lane-group Riccati sweeps), injected in
 * every iteration where the fixture's perturbed runs differ only at the start.  0 or unset: off (the default).  The
 * sign stream restarts with every solve (round 6: it was per thread, so a run depended on the runs its thread did
 * before). */
static void step_jitter(Sol* s) {
    const char* e = getenv("NLOT_ORACLE_STEP_JITTER");
    const double eps = e ? atof(e) : 0.0;
    if (eps == 0.0) return;
    const int nX = (s->N + 1) * s->nx, nU = s->N * s->nu;
    for (int i = 0; i < nX + nU + s->N + 1; ++i) {
        unsigned long long h = (++s->jit_ctr) * 0x9E3779B97F4A7C15ull;
        h ^= h >> 31;
        const double f = 1.0 + ((h >> 7) & 1 ? eps : -eps);
        if (i < nX) s->dX[i] *= f;
        else if (i < nX + nU) s->dU[i - nX] *= f;
        else s->dS[i - nX - nU] *= f;
    }
}

static int newton_step(Sol* s, double* dw_out) {
    double dw = 0.0;
    build(s, MODE_NEWTON, dw);
    if (riccati(s, MODE_NEWTON)) {
        dw = s->dw_last == 0.0 ? 1e-4 : fmax(1e-20, s->dw_last / 3.0);
        for (;;) {
            build(s, MODE_NEWTON, dw);
            if (!riccati(s, MODE_NEWTON)) break;
            dw *= (s->dw_last == 0.0) ? 100.0 : 8.0;
            if (dw > 1e40) return 1;
        }
        s->dw_last = dw;
    }
    *dw_out = dw;
    step_jitter(s);
    return 0;
}

typedef struct { /* line-search reference values (the current point, or the watchdog's) */
    double theta, phi, gd, alpha_test;
    int fixed_test; /* 1: acceptance uses alpha_test instead of the trial's alpha (watchdog) */
} LsRef;

/* IPOPT DoBacktrackingLineSearch: alpha = amax, amax/2, ... down to amin; on the first trial, if theta did
 * not decrease, up to max_soc second-order corrections (not in the restoration problem).  Returns 1 when a
 * point was accepted (alpha, az, the f-type/Armijo flag out; the step arrays hold the accepted step). */
static int backtrack(Sol* s, const LsRef* ref, double amax, double az0, double amin, double tau, int skip_first,
                     int only_full, double dw, Trial* t, double* alpha_out, double* az_out, int* ftype_armijo) {
    const NlotSolverOptions* o = s->o;
    int nx = s->nx, N = s->N, M = s->M;
    const int nsave = step_len(s);
    const int nres = XMAX + N * nx + CMAX + (N + 1) * M + s->nb;
    double tri[XMAX], trt[CMAX];
    double* trd = (double*)malloc(sizeof(double) * (N * nx + (N + 1) * M + s->nb + 1));
    double* trq = trd + N * nx;
    double* trb = trq + (N + 1) * M;
    double alpha = skip_first ? 0.5 * amax : amax, az = az0;
    int accepted = 0, ntr = skip_first ? 1 : 0;
    s->last_rej_filter = 0;
    for (;;) {
        ++ntr;
        trial_primal(s, alpha, t);
        double tht, pht;
        trial_merit(s, t, s->mu, &tht, &pht, tri, trd, trt, trq, trb);
        const double at = ref->fixed_test ? ref->alpha_test : alpha;
        if (ls_accept(s, ref->theta, ref->phi, ref->gd, at, tht, pht, ftype_armijo)) {
            accepted = 1;
            break;
        }
        s->last_rej_filter = s->rej_filter;
        if (only_full) break;
        /* second-order correction (IPOPT max_soc, kappa_soc): c_soc = alpha c(x) + c(x + alpha d) */
        if (ntr == 1 && !s->resto && o->max_soc > 0 && tht >= ref->theta) {
            int soc_ok = 0;
            s->n_soc_tried++;
            double* save = (double*)malloc(sizeof(double) * (nsave + nres));
            double* c0 = save + nsave;
            step_save(s, save, 0);
            res_save(s, c0, 0);
            double *ci = s->rci, *cd = s->rcd, *ct = s->rct, *cq = s->rcq, *cb = s->rcb;
            for (int i = 0; i < nx; ++i) ci[i] = alpha * ci[i] + tri[i];
            for (int i = 0; i < N * nx; ++i) cd[i] = alpha * cd[i] + trd[i];
            for (int i = 0; i < s->nc; ++i) ct[i] = alpha * ct[i] + trt[i];
            for (int i = 0; i < (N + 1) * M; ++i) cq[i] = alpha * cq[i] + trq[i];
            for (int i = 0; i < s->nb; ++i) cb[i] = alpha * cb[i] + trb[i];
            double th_old = tht;
            for (int pc = 0; pc < o->max_soc; ++pc) {
                build(s, MODE_NEWTON, dw);
                if (riccati(s, MODE_NEWTON)) break; /* same matrix: cannot fail, but be safe */
                recover(s, dw);
                const double asoc = primal_frac(s, tau);
                trial_primal(s, asoc, t);
                double ths, phs;
                trial_merit(s, t, s->mu, &ths, &phs, tri, trd, trt, trq, trb);
                if (ls_accept(s, ref->theta, ref->phi, ref->gd, alpha, ths, phs, ftype_armijo)) {
                    soc_ok = 1;
                    alpha = asoc;
                    az = dual_frac(s, tau);
                    break;
                }
                if (ths > o->kappa_soc * th_old) break;
                th_old = ths;
                for (int i = 0; i < nx; ++i) ci[i] = asoc * ci[i] + tri[i];
                for (int i = 0; i < N * nx; ++i) cd[i] = asoc * cd[i] + trd[i];
                for (int i = 0; i < s->nc; ++i) ct[i] = asoc * ct[i] + trt[i];
                for (int i = 0; i < (N + 1) * M; ++i) cq[i] = asoc * cq[i] + trq[i];
                for (int i = 0; i < s->nb; ++i) cb[i] = asoc * cb[i] + trb[i];
            }
            res_save(s, c0, 1);
            if (!soc_ok) step_save(s, save, 1);
            free(save);
            if (soc_ok) {
                s->n_soc_acc++;
                accepted = 1;
                break;
            }
        }
        alpha *= 0.5;
        if (alpha < amin) break;
    }
    free(trd);
    *alpha_out = alpha;
    *az_out = az;
    return accepted;
}

/* IPOPT DetectTinyStep: primal step tiny relative to the iterate, multiplier step small, nearly feasible */
static int tiny_step(const Sol* s, const Errs* e) {
    const NlotSolverOptions* o = s->o;
    if (!(o->tiny_step_tol > 0)) return 0;
    int nx = s->nx, nu = s->nu, N = s->N, M = s->M;
    double mx = 0, my = 0, ya = 0;
    for (int i = 0; i < (N + 1) * nx; ++i) mx = fmax(mx, fabs(s->dX[i]) / (1.0 + fabs(s->X[i])));
    for (int i = 0; i < N * nu; ++i) mx = fmax(mx, fabs(s->dU[i]) / (1.0 + fabs(s->U[i])));
    if (s->ns)
        for (int k = 0; k <= N; ++k) mx = fmax(mx, fabs(s->dS[k]) / (1.0 + fabs(s->S[k])));
    for (int q = 0; q < (N + 1) * M; ++q) mx = fmax(mx, fabs(s->dT[q]) / (1.0 + fabs(s->T[q])));
    for (int q = 0; q < s->nb; ++q) mx = fmax(mx, fabs(s->dsb[q]) / (1.0 + fabs(s->sb[q])));
    if (mx > o->tiny_step_tol) return 0;
    for (int i = 0; i < nx; ++i) {
        my = fmax(my, fabs(s->yi_n[i] - s->yi[i]));
        ya = fmax(ya, fabs(s->yi[i]));
    }
    for (int i = 0; i < N * nx; ++i) {
        my = fmax(my, fabs(s->yk_n[i] - s->yk[i]));
        ya = fmax(ya, fabs(s->yk[i]));
    }
    for (int i = 0; i < s->nc; ++i) {
        my = fmax(my, fabs(s->yt_n[i] - s->yt[i]));
        ya = fmax(ya, fabs(s->yt[i]));
    }
    for (int q = 0; q < (N + 1) * M; ++q) {
        my = fmax(my, fabs(s->yd_n[q] - s->yd[q]));
        ya = fmax(ya, fabs(s->yd[q]));
    }
    for (int q = 0; q < s->nb; ++q) {
        my = fmax(my, fabs(s->yb_n[q] - s->yb[q]));
        ya = fmax(ya, fabs(s->yb[q]));
    }
    if (my / (1.0 + ya) > o->tiny_step_y_tol) return 0;
    return e->primal < 1e-4;
}

static void sol_setup(Sol* s, const NlotProblem* p, const NlotSolverOptions* o, const NlotMlpDesc* m,
                      const double* x0, const double* xg) {
    memset(s, 0, sizeof *s);
    s->p = p;
    s->m = m;
    s->o = o;
    s->nx = p->nx;
    s->nu = p->nu;
    s->ns = p->use_slack ? 1 : 0;
    s->N = p->N;
    s->M = knot_m(p);
    s->sd = (p->shape == NLOT_SHAPE_POLYGON && p->use_slack) ? 1 : 0;
    s->nc = 0;
    for (int i = 0; i < p->nx; ++i) /* runner.py:51-56 */
        if (p->enforce_heading || i != 2) s->tidx[s->nc++] = i;
    memcpy(s->x0, x0, sizeof(double) * p->nx);
    memcpy(s->xg, xg, sizeof(double) * p->nx);
    s->gcb = o->general_bounds ? 1 : 0;
    s->nb = s->gcb ? s->N * s->nu + s->ns * (s->N + 1) : 0;
    s->ne = s->nx + s->N * s->nx + s->nc + (s->N + 1) * s->M + s->nb;
    s->fcap = 2 * (o->max_iter > 0 ? o->max_iter : 0) + FILT_MIN;
    const char* br = getenv("NLOT_ORACLE_BOUND_RELAX");
    if (br && atof(br) > 0.0) {
        const double r = atof(br);
        s->prel = *p;
        for (int i = 0; i < p->nu; ++i) {
            s->prel.umin[i] -= r * fmax(1.0, fabs(p->umin[i]));
            s->prel.umax[i] += r * fmax(1.0, fabs(p->umax[i]));
        }
        s->p = &s->prel;
        s->brel = r;
    }
    const char* fc = getenv("NLOT_ORACLE_FILT_CAP");
    if (fc && atoi(fc) > 0 && atoi(fc) < s->fcap) s->fcap = atoi(fc);
}

/* how a run ended (diagnostic, info[14]) */
enum { TERM_SOLVED = 0, TERM_MAXITER = 1, TERM_MAXITER_RESTO = 2, TERM_RESTO_LS = 3, TERM_RESTO_FEAS_REJECTED = 4,
       TERM_RESTO_INFEASIBLE = 5, TERM_ALMOST_FEASIBLE = 6, TERM_NUMERIC = 7, TERM_TINY = 8, TERM_LS = 9 };

/* Per-iteration trace (test infrastructure: oracle_solve_trace): the iterate (X, U) at the top of iteration it, i.e.
 * the point a run with max_iter = it returns (inside a restoration phase: the restoration iterate, as the GPU solver
 * reports it).  Thread-local, so parallel runs trace independently. */
static __thread double* g_trace;
static __thread int g_trace_cap;
static void trace_rec(const Sol* s, int it, const double* X, const double* U) {
    if (!g_trace || it < 0 || it >= g_trace_cap) return;
    const size_t nX = (size_t)(s->N + 1) * s->nx, nU = (size_t)s->N * s->nu;
    memcpy(g_trace + (size_t)it * (nX + nU), X, sizeof(double) * nX);
    memcpy(g_trace + (size_t)it * (nX + nU) + nX, U, sizeof(double) * nU);
}

/* IPOPT MinC_1NrmRestorationPhase (Waechter & Biegler 2006 §3.3, IPOPT's documented defaults), run on the
 * restoration workspace r for the current point of s.  Returns 0 when it found a point acceptable to the
 * original filter (s then holds it: equality multipliers 0 as constr_mult_reset_threshold = 0, bound
 * multipliers by one complementarity Newton step over the whole restoration, reset to 1 above
 * bound_mult_reset_threshold), else a status.  *iter counts restoration iterations (max_iter covers both). */
static int restoration(Sol* s, Sol* r, int* iter, double* lin_resid) {
    const NlotProblem* p = s->p;
    const NlotSolverOptions* o = s->o;
    int nx = s->nx, nu = s->nu, N = s->N, M = s->M;
    const double kappa_d = 1e-5, gt = 1e-5, gp = 1e-8;
    /* reference point x_R and the original merit there */
    double th_R, ph_R;
    merit(s, s->X, s->U, s->S, s->T, s->sb, s->mu, &th_R, &ph_R, NULL);
    residuals(s, s->X, s->U, s->S, s->T, s->sb, s->rci, s->rcd, s->rct, s->rcq, s->rcb);
    double cmax = 0;
    for (int i = 0; i < nx; ++i) cmax = fmax(cmax, fabs(s->rci[i]));
    for (int i = 0; i < N * nx; ++i) cmax = fmax(cmax, fabs(s->rcd[i]));
    for (int j = 0; j < s->nc; ++j) cmax = fmax(cmax, fabs(s->rct[j]));
    for (int q = 0; q < (N + 1) * M; ++q) cmax = fmax(cmax, fabs(s->rcq[q]));
    for (int q = 0; q < s->nb; ++q) cmax = fmax(cmax, fabs(s->rcb[q]));
    memcpy(r->X, s->X, sizeof(double) * (N + 1) * nx);
    memcpy(r->U, s->U, sizeof(double) * N * nu);
    memcpy(r->S, s->S, sizeof(double) * (N + 1));
    memcpy(r->T, s->T, sizeof(double) * (N + 1) * M);
    memcpy(r->sb, s->sb, sizeof(double) * s->nb);
    memcpy(r->XR, s->X, sizeof(double) * (N + 1) * nx);
    memcpy(r->UR, s->U, sizeof(double) * N * nu);
    memcpy(r->SR, s->S, sizeof(double) * (N + 1));
    for (int i = 0; i < (N + 1) * nx; ++i) r->DRX[i] = fmin(1.0, 1.0 / fabs(r->XR[i]));
    for (int i = 0; i < N * nu; ++i) r->DRU[i] = fmin(1.0, 1.0 / fabs(r->UR[i]));
    for (int k = 0; k <= N; ++k) r->DRS[k] = fmin(1.0, 1.0 / fabs(r->SR[k]));
    const double mu = fmax(s->mu, cmax);
    r->mu = mu;
    r->mu_dc = mu;
    r->tau = fmax(0.99, 1.0 - mu);
    r->rho = o->resto_penalty_parameter;
    r->zeta = o->resto_proximity_weight * sqrt(mu);
    /* p, n minimising the restoration barrier problem for fixed x (IPOPT eq. (33)) */
    for (int i = 0; i < r->ne; ++i) {
        const double c = i < nx ? s->rci[i]
                         : i < row_t(s, 0) ? s->rcd[i - nx]
                         : i < row_q(s, 0) ? s->rct[i - row_t(s, 0)]
                         : i < row_b(s, 0) ? s->rcq[i - row_q(s, 0)]
                                           : s->rcb[i - row_b(s, 0)];
        const double a = (mu - r->rho * c) / (2.0 * r->rho);
        const double n = a + sqrt(a * a + mu * c / (2.0 * r->rho));
        r->rn[i] = n;
        r->rp[i] = c + n;
        r->rzp[i] = mu / r->rp[i];
        r->rzn[i] = mu / r->rn[i];
    }
    for (int i = 0; i < N * nu; ++i) {
        r->zl[i] = fmin(r->rho, s->zl[i]);
        r->zu[i] = fmin(r->rho, s->zu[i]);
    }
    for (int k = 0; k <= N; ++k) r->zs[k] = fmin(r->rho, s->zs[k]);
    for (int q = 0; q < (N + 1) * M; ++q) r->vt[q] = fmin(r->rho, s->vt[q]);
    for (int q = 0; q < s->nb; ++q) {
        r->zbl[q] = fmin(r->rho, s->zbl[q]);
        r->zbu[q] = fmin(r->rho, s->zbu[q]);
    }
    memset(r->yb, 0, sizeof(double) * s->nb);
    memset(r->yi, 0, sizeof(double) * nx);
    memset(r->yk, 0, sizeof(double) * N * nx);
    memset(r->yt, 0, sizeof(double) * CMAX);
    memset(r->yd, 0, sizeof(double) * (N + 1) * M);
    r->nfilt = 0;
    r->dw_last = 0;
    {
        double th0, ph0;
        merit_resto(r, r->X, r->U, r->S, r->T, r->sb, r->rp, r->rn, r->mu, &th0, &ph0, NULL, NULL, NULL, NULL, NULL);
        r->theta_max = 1e4 * fmax(1.0, th0);
        r->theta_min = 1e-4 * fmax(1.0, th0);
    }
    const int ntr = (N + 1) * nx + N * nu + (N + 1) + (N + 1) * M + 2 * r->ne + r->nb;
    double* tb = (double*)malloc(sizeof(double) * ntr);
    Trial t = {tb, tb + (N + 1) * nx, tb + (N + 1) * nx + N * nu, tb + (N + 1) * nx + N * nu + N + 1,
               tb + (N + 1) * nx + N * nu + N + 1 + (N + 1) * M, tb + (N + 1) * nx + N * nu + N + 1 + (N + 1) * M + r->ne,
               tb + (N + 1) * nx + N * nu + N + 1 + (N + 1) * M + 2 * r->ne};
    const double kap = o->barrier_tol_factor;
    const double mu_floor = fmin(o->tol, o->compl_inf_tol) / (kap + 1.0);
    int status = NLOT_RESTO_FAILED, first = 1;
    Errs e;
    for (;;) {
        eval_full(r);
        errors(r, &e);
        trace_rec(s, *iter, r->X, r->U);
        double E0 = fmax(fmax(e.dual / e.sd, e.primal), e.compl0 / e.sc);
        if (!isfinite(E0)) {
            status = NLOT_NUMERIC;
            break;
        }
        if (!first) { /* RestoConvergenceCheck: back to the regular iteration? */
            double th_o, ph_o;
            merit(s, r->X, r->U, r->S, r->T, r->sb, s->mu, &th_o, &ph_o, NULL);
            if (th_o <= o->required_infeasibility_reduction * th_R && filter_ok(s, th_o, ph_o) &&
                (cmp_le(th_o, (1.0 - gt) * th_R, th_R) || cmp_le(ph_o - ph_R, -gp * th_R, ph_R))) {
                status = 0;
                break;
            }
            if (E0 <= o->tol) { /* the restoration problem converged to an unacceptable point */
                const double thr = o->resto_failure_feasibility_threshold > 0 ? o->resto_failure_feasibility_threshold
                                                                              : 1e2 * o->tol;
                double pinf = 0;
                residuals(s, r->X, r->U, r->S, r->T, r->sb, s->rci, s->rcd, s->rct, s->rcq, s->rcb);
                for (int i = 0; i < nx; ++i) pinf = fmax(pinf, fabs(s->rci[i]));
                for (int i = 0; i < N * nx; ++i) pinf = fmax(pinf, fabs(s->rcd[i]));
                for (int j = 0; j < s->nc; ++j) pinf = fmax(pinf, fabs(s->rct[j]));
                for (int q = 0; q < (N + 1) * M; ++q) pinf = fmax(pinf, fabs(s->rcq[q]));
                for (int q = 0; q < s->nb; ++q) pinf = fmax(pinf, fabs(s->rcb[q]));
                status = pinf <= thr ? NLOT_RESTO_FAILED : NLOT_INFEASIBLE;
                s->term = pinf <= thr ? TERM_RESTO_FEAS_REJECTED : TERM_RESTO_INFEASIBLE;
                break;
            }
        }
        first = 0;
        if (*iter >= o->max_iter) {
            status = NLOT_MAXITER;
            s->term = TERM_MAXITER_RESTO;
            break;
        }
        /* monotone barrier update inside the restoration phase */
        for (;;) {
            double Emu = fmax(fmax(e.dual / e.sd, e.primal), e.complmu / e.sc);
            if (Emu > kap * r->mu) break;
            double nm = fmax(fmin(0.2 * r->mu, pow(r->mu, 1.5)), mu_floor);
            if (nm >= r->mu) break;
            r->mu = nm;
            r->tau = fmax(0.99, 1.0 - nm);
            r->nfilt = 0;
            errors(r, &e);
        }
        r->mu_dc = r->mu;
        double dw;
        if (newton_step(r, &dw)) {
            status = NLOT_NUMERIC;
            break;
        }
        recover(r, dw);
        const double tau = r->tau, amax = primal_frac(r, tau), az = dual_frac(r, tau);
        double theta, phi;
        merit_resto(r, r->X, r->U, r->S, r->T, r->sb, r->rp, r->rn, r->mu, &theta, &phi, NULL, NULL, NULL, NULL, NULL);
        const double gd = barrier_gd(r);
        double amin = 1e-5;
        if (gd < 0) {
            amin = fmin(1e-5, 1e-8 * theta / (-gd));
            if (theta <= r->theta_min) amin = fmin(amin, pow(theta, 1.1) / pow(-gd, 2.3));
        }
        amin *= 0.05;
        LsRef ref = {theta, phi, gd, 0.0, 0};
        double alpha, azz;
        int fa = 0;
        int ok = backtrack(r, &ref, amax, az, amin, tau, 0, 0, dw, &t, &alpha, &azz, &fa);
        if (getenv("NLOT_VERBOSE"))
            fprintf(stderr, "  resto it %3d mu %.2e fR %.6f thR %.2e E0 %.2e a %.2e\n", *iter, r->mu, r->f, theta, E0, alpha);
        if (!ok) {
            status = NLOT_RESTO_FAILED;
            s->term = TERM_RESTO_LS;
            break;
        }
        if (!fa) filter_add(r, theta, phi);
        accept_step(r, alpha, azz, &t);
        ++*iter;
    }
    free(tb);
    (void)lin_resid;
    if (status) {
        /* the instance ends inside the restoration phase: its output is the restoration iterate (the GPU solver's
         * arrays hold it); IPOPT would report the original problem's last iterate */
        memcpy(s->X, r->X, sizeof(double) * (N + 1) * nx);
        memcpy(s->U, r->U, sizeof(double) * N * nu);
        memcpy(s->S, r->S, sizeof(double) * (N + 1));
        return status;
    }
    /* back to the regular problem */
    double* zold = (double*)malloc(sizeof(double) * 4 * (2 * N * nu + (N + 1) + (N + 1) * M));
    const double mu0 = s->mu;
    double az = 1.0;
#define DZ(z, so, sn) ((mu0 - (z) * (sn)) / (so))
    for (int q = 0; q < s->nb; ++q) {
        s->dzbl[q] = DZ(s->zbl[q], s->sb[q] - blo(s, q), r->sb[q] - blo(s, q));
        s->dzbu[q] = bhi_on(s, q) ? DZ(s->zbu[q], bhi(s, q) - s->sb[q], bhi(s, q) - r->sb[q]) : 0.0;
    }
    for (int k = 0; k < (s->gcb ? 0 : N); ++k)
        for (int i = 0; i < nu; ++i) {
            int q = k * nu + i;
            s->dzl[q] = DZ(s->zl[q], s->U[q] - p->umin[i], r->U[q] - p->umin[i]);
            s->dzu[q] = DZ(s->zu[q], p->umax[i] - s->U[q], p->umax[i] - r->U[q]);
        }
    if (s->ns && !s->gcb)
        for (int k = 0; k <= N; ++k) s->dzs[k] = DZ(s->zs[k], s->S[k] + s->brel, r->S[k] + s->brel);
    for (int q = 0; q < (N + 1) * M; ++q) s->dvt[q] = DZ(s->vt[q], s->T[q], r->T[q]);
#undef DZ
    az = dual_frac(s, s->tau);
    double zmax = 0;
    for (int q = 0; q < s->nb; ++q) {
        s->zbl[q] += az * s->dzbl[q];
        zmax = fmax(zmax, s->zbl[q]);
        if (bhi_on(s, q)) {
            s->zbu[q] += az * s->dzbu[q];
            zmax = fmax(zmax, s->zbu[q]);
        }
    }
    for (int i = 0; i < (s->gcb ? 0 : N * nu); ++i) {
        s->zl[i] += az * s->dzl[i];
        s->zu[i] += az * s->dzu[i];
        zmax = fmax(zmax, fmax(s->zl[i], s->zu[i]));
    }
    if (s->ns && !s->gcb)
        for (int k = 0; k <= N; ++k) {
            s->zs[k] += az * s->dzs[k];
            zmax = fmax(zmax, s->zs[k]);
        }
    for (int q = 0; q < (N + 1) * M; ++q) {
        s->vt[q] += az * s->dvt[q];
        zmax = fmax(zmax, s->vt[q]);
    }
    if (zmax > o->bound_mult_reset_threshold) {
        for (int i = 0; i < N * nu; ++i) s->zl[i] = s->zu[i] = 1.0;
        for (int k = 0; k <= N; ++k) s->zs[k] = 1.0;
        for (int q = 0; q < (N + 1) * M; ++q) s->vt[q] = 1.0;
        for (int q = 0; q < s->nb; ++q) s->zbl[q] = s->zbu[q] = 1.0;
    }
    free(zold);
    memcpy(s->X, r->X, sizeof(double) * (N + 1) * nx);
    memcpy(s->U, r->U, sizeof(double) * N * nu);
    memcpy(s->S, r->S, sizeof(double) * (N + 1));
    memcpy(s->T, r->T, sizeof(double) * (N + 1) * M);
    memcpy(s->sb, r->sb, sizeof(double) * s->nb);
    memset(s->yi, 0, sizeof(double) * nx);
    memset(s->yk, 0, sizeof(double) * N * nx);
    memset(s->yt, 0, sizeof(double) * CMAX);
    memset(s->yd, 0, sizeof(double) * (N + 1) * M);
    memset(s->yb, 0, sizeof(double) * s->nb);
    (void)kappa_d;
    return 0;
}

/* info[0] = final objective, [1] = max dual inf, [2] = constr viol, [3] = max linear-KKT residual
 * seen, [4] = final mu, [5] = E_0 (scaled overall error), [6] = restoration phases, [7] = watchdog /
 * soft-restoration / SOC / tiny-step events (packed: 1e6 * watchdog + 1e4 * soft + 1e2 * soc tried + tiny),
 * [8] = theta (1-norm) at the last line-search failure, -1 if none, [9] / [10] = peak size of the line-search
 * (incl. restoration) / adaptive-mu filter, [11] / [12] = their forgotten entries (NLOT_ORACLE_FILT_CAP only),
 * [13] = trial-point merit evaluations (sequential line-search trials incl. corrections, soft and restoration steps),
 * [14] = how the run ended (TERM_*: restoration line search failed / converged to a feasible point the original filter
 * rejects / converged infeasible, almost feasible at the restoration's entry, max_iter inside restoration, ...).
 * info holds >= 16 doubles. */
/* oracle_solve_one with an initial guess for the controls and slacks too (Uinit / Sinit, NULL = the reference's
 * U = S = 0), pushed into their bounds as IPOPT pushes a starting point; test infrastructure (warm starts from a
 * returned solution: is it a local optimum of the same NLP). */
int oracle_solve_warm(const NlotProblem* p, const NlotSolverOptions* o, const NlotMlpDesc* m, const double* x0,
                      const double* xg, const double* Xinit, const double* Uinit, const double* Sinit, double* Xout,
                      double* Uout, double* Sout, double* cost, int* iters_out, double* info);
int oracle_solve_one(const NlotProblem* p, const NlotSolverOptions* o, const NlotMlpDesc* m, const double* x0,
                     const double* xg, const double* Xinit, double* Xout, double* Uout, double* Sout, double* cost,
                     int* iters_out, double* info) {
    return oracle_solve_warm(p, o, m, x0, xg, Xinit, NULL, NULL, Xout, Uout, Sout, cost, iters_out, info);
}
/* oracle_solve_one that also records the iterate (X, U) at the top of every iteration it < trace_cap into
 * trace[it * ((N+1) nx + N nu)] (test infrastructure: per-instance iterate fixtures) */
int oracle_solve_trace(const NlotProblem* p, const NlotSolverOptions* o, const NlotMlpDesc* m, const double* x0,
                       const double* xg, const double* Xinit, double* Xout, double* Uout, double* Sout, double* cost,
                       int* iters_out, double* info, double* trace, int trace_cap) {
    g_trace = trace;
    g_trace_cap = trace_cap;
    const int st = oracle_solve_warm(p, o, m, x0, xg, Xinit, NULL, NULL, Xout, Uout, Sout, cost, iters_out, info);
    g_trace = NULL;
    g_trace_cap = 0;
    return st;
}
int oracle_solve_warm(const NlotProblem* p, const NlotSolverOptions* o, const NlotMlpDesc* m, const double* x0,
                      const double* xg, const double* Xinit, const double* Uinit, const double* Sinit, double* Xout,
                      double* Uout, double* Sout, double* cost, int* iters_out, double* info) {
    Sol sol, *s = &sol, rsol, *r = &rsol;
    sol_setup(s, p, o, m, x0, xg);
    if (sol_alloc(s)) return NLOT_NUMERIC;
    int r_alloc = 0;
    int nx = s->nx, nu = s->nu, N = s->N, M = s->M;
    const double k1 = o->bound_push, k2 = o->bound_frac;
    const int nsave = step_len(s);
    double lin_resid = 0;
    double* qf_aff = (double*)malloc(sizeof(double) * 2 * nsave);
    double* qf_cen = qf_aff + nsave;
    /* ---- initial point: LinearInitializer (trajectory_initialization.py:54-55), U = S = 0 ---- */
    for (int k = 0; k <= N; ++k)
        for (int i = 0; i < nx; ++i)
            s->X[k * nx + i] = Xinit ? Xinit[k * nx + i] : x0[i] + (xg[i] - x0[i]) * ((double)k / (double)N);
    for (int k = 0; k < N; ++k)
        for (int i = 0; i < nu; ++i) {
            double lo = p->umin[i], hi = p->umax[i];
            double pl = fmin(k1 * fmax(1.0, fabs(lo)), k2 * (hi - lo));
            double pu = fmin(k1 * fmax(1.0, fabs(hi)), k2 * (hi - lo));
            const double pushed = fmin(fmax(Uinit ? Uinit[k * nu + i] : 0.0, lo + pl), hi - pu);
            /* general_bounds: U is free (Opti's initial value 0) and its row slack starts pushed into the bounds */
            s->U[k * nu + i] = s->gcb ? (Uinit ? Uinit[k * nu + i] : 0.0) : pushed;
            if (s->gcb) s->sb[k * nu + i] = pushed;
        }
    for (int k = 0; k <= N; ++k) {
        const double s0 = Sinit ? Sinit[k] : 0.0;
        s->S[k] = (s->ns && !s->gcb) ? fmax(s0, k1 - s->brel) : (s->ns ? s0 : 0.0);
        if (s->gcb && s->ns) s->sb[N * nu + k] = fmax(s0, k1); /* slack_bound_push of d(x0) = S_k */
    }
    for (int q = 0; q < s->nb; ++q) s->zbl[q] = s->zbu[q] = 1.0;
    for (int k = 0; k <= N; ++k) {
        jet d[NLOT_MAX_BODY];
        knot_ineq(p, m, s->X + k * nx, 0, d);
        for (int j = 0; j < M; ++j) s->T[k * M + j] = fmax(d[j].v + (s->sd ? s->S[k] : 0.0) + s->brel, k1);
    }
    for (int i = 0; i < N * nu; ++i) s->zl[i] = s->zu[i] = 1.0;
    for (int k = 0; k <= N; ++k) s->zs[k] = 1.0;
    for (int i = 0; i < (N + 1) * M; ++i) s->vt[i] = 1.0;
    s->mu = o->mu_init;
    s->mu_dc = s->mu;
    s->tau = fmax(0.99, 1.0 - s->mu);
    /* ---- least-squares equality multipliers (IPOPT LeastSquareMultipliers) ---- */
    eval_full(s);
    build(s, MODE_LSQ, 0.0);
    if (riccati(s, MODE_LSQ) == 0) {
        double ymax = 0;
        for (int k = 0; k <= N; ++k)
            for (int j = 0; j < M; ++j) {
                int q = k * M + j;
                double w = 0;
                for (int a = 0; a < 3 && a < nx; ++a) w += s->Jd[q * 3 + a] * s->dX[k * nx + a];
                if (s->sd) w += s->dS[k];
                s->yd[q] = w - s->vt[q];
                ymax = fmax(ymax, fabs(s->yd[q]));
            }
        for (int q = 0; q < s->nb; ++q) { /* bound rows: y = J dz - (z_L - z_U), J the unit vector */
            s->yb[q] = bvar(s, s->dU, s->dS, q) - (s->zbl[q] - (bhi_on(s, q) ? s->zbu[q] : 0.0));
            ymax = fmax(ymax, fabs(s->yb[q]));
        }
        memcpy(s->yi, s->yi_n, sizeof(double) * nx);
        memcpy(s->yk, s->yk_n, sizeof(double) * N * nx);
        memcpy(s->yt, s->yt_n, sizeof(double) * s->nc);
        for (int i = 0; i < nx; ++i) ymax = fmax(ymax, fabs(s->yi[i]));
        for (int i = 0; i < N * nx; ++i) ymax = fmax(ymax, fabs(s->yk[i]));
        for (int i = 0; i < s->nc; ++i) ymax = fmax(ymax, fabs(s->yt[i]));
        if (ymax > o->constr_mult_init_max) {
            memset(s->yi, 0, sizeof(double) * nx);
            memset(s->yk, 0, sizeof(double) * N * nx);
            memset(s->yt, 0, sizeof(double) * CMAX);
            memset(s->yd, 0, sizeof(double) * (N + 1) * M);
            memset(s->yb, 0, sizeof(double) * s->nb);
        }
    }
    {
        double th0, ph0;
        merit(s, s->X, s->U, s->S, s->T, s->sb, s->mu, &th0, &ph0, NULL);
        s->theta_max = 1e4 * fmax(1.0, th0);
        s->theta_min = 1e-4 * fmax(1.0, th0);
    }
    s->nfilt = 0;
    s->dw_last = 0;
    int status = NLOT_MAXITER, iter = 0;
    Errs e;
    const int ntr = (N + 1) * nx + N * nu + (N + 1) + (N + 1) * M + s->nb;
    double* tb = (double*)malloc(sizeof(double) * ntr);
    Trial t = {tb, tb + (N + 1) * nx, tb + (N + 1) * nx + N * nu, tb + (N + 1) * nx + N * nu + N + 1, NULL, NULL,
               tb + (N + 1) * nx + N * nu + N + 1 + (N + 1) * M};
    /* watchdog (IPOPT StartWatchDog / StopWatchDog): saved iterate, direction and reference values */
    const int nit = iter_len(s);
    double* wd_it = (double*)malloc(sizeof(double) * (nit + nsave));
    double* wd_dir = wd_it + nit;
    int in_wd = 0, wd_short = 0, wd_trial = 0, in_soft = 0, soft_cnt = 0, tiny_last = 0;
    int n_resto = 0, n_wd = 0, n_soft = 0, n_tiny = 0;
    double theta_fail = -1.0; /* theta of the last iterate whose line search failed (diagnostic) */
    LsRef wd_ref = {0, 0, 0, 0, 1};
    double wd_amax = 1, wd_az = 1, wd_amin = 0, wd_mu = 0, wd_tau = 0;
    FILE* dump = getenv("NLOT_ORACLE_DUMP") ? fopen(getenv("NLOT_ORACLE_DUMP"), "wb") : NULL; /* diagnostics */
    for (;;) {
        eval_full(s);
        errors(s, &e);
        trace_rec(s, iter, s->X, s->U);
        double E0 = fmax(fmax(e.dual / e.sd, e.primal), e.compl0 / e.sc);
        if (dump) { /* [iter, mu, f, E0, dual, primal, free mode, resto phases], X and yd, one record per iteration */
            const double hd[8] = {(double)iter, s->mu, s->f, E0, e.dual, e.primal, (double)s->free_mode,
                                  (double)n_resto};
            fwrite(hd, sizeof(double), 8, dump);
            fwrite(s->X, sizeof(double), (size_t)(N + 1) * nx, dump);
            fwrite(s->yd, sizeof(double), (size_t)(N + 1) * M, dump);
        }
        if (info) info[5] = E0;
        if (!isfinite(E0)) {
            status = NLOT_NUMERIC;
            break;
        }
        if (E0 <= o->tol && e.dual <= o->dual_inf_tol && e.cviol <= o->constr_viol_tol &&
            e.compl0 <= o->compl_inf_tol) {
            status = NLOT_SOLVED;
            break;
        }
        if (iter >= o->max_iter) {
            status = NLOT_MAXITER;
            break;
        }
        /* ---- barrier parameter ---- */
        const double kap = o->barrier_tol_factor;
        const double mu_floor = fmin(o->tol, o->compl_inf_tol) / (kap + 1.0);
        int use_qf = 0, ls_reset = 0;
        if (o->mu_strategy == 0) { /* IPOPT MonotoneMuUpdate, fast decrease allowed */
            if (iter > 0) {
                for (;;) {
                    double Emu = fmax(fmax(e.dual / e.sd, e.primal), e.complmu / e.sc);
                    if (Emu > kap * s->mu && !tiny_last) break;
                    double nm = fmin(0.2 * s->mu, pow(s->mu, 1.5));
                    nm = fmax(nm, mu_floor);
                    if (nm >= s->mu) break;
                    s->mu = nm;
                    s->tau = fmax(0.99, 1.0 - s->mu);
                    s->nfilt = 0;
                    ls_reset = 1;
                    errors(s, &e); /* complmu depends on mu */
                    tiny_last = 0;
                }
            }
        } else { /* IPOPT AdaptiveMuUpdate::UpdateBarrierParameter */
            if (iter == 0) {
                s->mu_max = 1e3 * e.avg_compl; /* mu_max_fact * initial average complementarity */
                s->free_mode = 1;
                s->nafilt = 0;
            }
            double th_c, ph_c;
            merit(s, s->X, s->U, s->S, s->T, s->sb, s->mu, &th_c, &ph_c, NULL);
            const double f_c = s->f;
            /* fixed mode: back to free mode as soon as the point makes sufficient progress w.r.t. the progress
             * filter ("Switching back to free mu mode", checked every iteration); otherwise one Fiacco-McCormick
             * decrease once the barrier problem is solved ("Reducing mu ... in fixed mu mode") */
            if (!s->free_mode) {
                if (afilt_acceptable(s, f_c, th_c)) {
                    s->free_mode = 1; /* RememberCurrentPointAsAccepted below */
                } else {
                    double Emu = fmax(fmax(e.dual / e.sd, e.primal), e.complmu / e.sc);
                    if (Emu <= kap * s->mu) {
                        double nm = fmax(fmin(0.2 * s->mu, pow(s->mu, 1.5)), mu_floor);
                        if (nm < s->mu) {
                            s->mu = nm;
                            s->tau = fmax(0.99, 1.0 - s->mu);
                            s->nfilt = 0;
                            ls_reset = 1;
                            errors(s, &e);
                        }
                    }
                }
            }
            if (s->free_mode) {
                if (afilt_acceptable(s, f_c, th_c)) {
                    afilt_add(s, f_c, th_c); /* RememberCurrentPointAsAccepted */
                } else { /* insufficient progress: fixed mode at 0.8 * average complementarity */
                    s->free_mode = 0;
                    s->mu = fmin(fmax(0.8 * e.avg_compl, AMU_MU_MIN), s->mu_max);
                    s->tau = fmax(0.99, 1.0 - s->mu);
                    s->nfilt = 0;
                    ls_reset = 1;
                    errors(s, &e);
                }
            }
            use_qf = s->free_mode;
        }
        /* ---- search direction with inertia correction ---- */
        const double mu_it = s->mu;
        s->mu_dc = mu_it;
        if (use_qf) s->mu = 0.0; /* free mode: affine-scaling step first */
        double dw;
        if (newton_step(s, &dw)) {
            status = NLOT_NUMERIC;
            break;
        }
        lin_resid = fmax(lin_resid, linear_residual(s, MODE_NEWTON));
        recover(s, dw);
        if (use_qf) { /* QualityFunctionMuOracle: centering step, sigma search, mu = sigma avg */
            step_save(s, qf_aff, 0);
            s->mu = e.avg_compl;
            build(s, MODE_NEWTON, dw);
            if (riccati(s, MODE_NEWTON)) { /* same matrix as the affine solve: cannot fail */
                status = NLOT_NUMERIC;
                break;
            }
            recover(s, dw);
            step_save(s, qf_cen, 0);
            for (int i = 0; i < nsave; ++i) qf_cen[i] -= qf_aff[i];
            QfCtx qc = {qf_aff, qf_cen, e.avg_compl, &e};
            double sigma = qf_sigma(s, &qc, AMU_MU_MIN, s->mu_max);
            double mu = fmin(fmax(sigma * e.avg_compl, AMU_MU_MIN), s->mu_max);
            step_combine(s, qf_aff, qf_cen, mu / e.avg_compl);
            s->mu = mu;
            s->tau = fmax(0.99, 1.0 - mu);
            s->nfilt = 0; /* the line-search filter belongs to one barrier problem */
            ls_reset = 1;
        } else {
            s->mu = mu_it;
        }
        if (ls_reset) { /* a new barrier problem: BacktrackingLineSearch::Reset ends the soft restoration and the
                         * watchdog (and clears the filter, above) */
            in_soft = soft_cnt = 0;
            in_wd = wd_short = 0;
        }
        /* ---- step sizes: fraction to the boundary; line-search reference values ---- */
        const double tau = s->tau;
        double amax = primal_frac(s, tau), az = dual_frac(s, tau);
        double theta, phi;
        merit(s, s->X, s->U, s->S, s->T, s->sb, s->mu, &theta, &phi, NULL);
        const double gd = barrier_gd(s);
        double amin = 1e-5;
        if (gd < 0) {
            amin = fmin(1e-5, 1e-8 * theta / (-gd));
            if (theta <= s->theta_min) amin = fmin(amin, pow(theta, 1.1) / pow(-gd, 2.3));
        }
        amin *= 0.05;
        /* ---- line search (IPOPT BacktrackingLineSearch::FindAcceptableTrialPoint) ---- */
        LsRef ref = {theta, phi, gd, 0.0, 0};
        double alpha = amax, azz = az;
        int accepted = 0, fa = 0, is_tiny = 0, augment = 1;
        if (!in_soft && !in_wd && tiny_step(s, &e)) { /* tiny step: take the full step, no filter */
            is_tiny = 1;
            ++n_tiny;
            trial_primal(s, amax, &t);
            accepted = 1;
            augment = 0;
            if (tiny_last) { /* twice in a row: IPOPT STOP_AT_TINY_STEP */
                accept_step(s, amax, az, &t);
                ++iter;
                status = NLOT_TINY_STEP;
                break;
            }
        } else if (in_soft) {
            accepted = 0; /* soft restoration continues below */
        } else {
            if (!in_wd && o->watchdog_shortened_iter_trigger > 0 && wd_short >= o->watchdog_shortened_iter_trigger) {
                /* StartWatchDog: remember the point, its direction and reference values */
                in_wd = 1;
                wd_trial = 0;
                ++n_wd;
                iter_io(s, wd_it, 0);
                step_save(s, wd_dir, 0);
                wd_ref = (LsRef){theta, phi, gd, amax, 1};
                wd_amax = amax;
                wd_az = az;
                wd_amin = amin;
                wd_mu = s->mu;
                wd_tau = tau;
            }
            int skip_first = 0;
            for (;;) {
                const LsRef* rf = in_wd ? &wd_ref : &ref;
                accepted = backtrack(s, rf, amax, az, amin, tau, skip_first, in_wd, dw, &t, &alpha, &azz, &fa);
                if (in_wd) {
                    if (accepted) {
                        in_wd = 0;
                    } else if (++wd_trial > o->watchdog_trial_iter_max) {
                        /* StopWatchDog: back to the watchdog point and direction, backtrack from alpha_max/2 */
                        in_wd = 0;
                        wd_short = 0;
                        iter_io(s, wd_it, 1);
                        step_save(s, wd_dir, 1);
                        s->mu = wd_mu;
                        s->tau = wd_tau;
                        amax = wd_amax;
                        az = wd_az;
                        amin = wd_amin;
                        ref = (LsRef){wd_ref.theta, wd_ref.phi, wd_ref.gd, 0.0, 0};
                        eval_full(s); /* residuals of the watchdog point (second-order corrections) */
                        skip_first = 1;
                        continue;
                    } else { /* tentative step: accepted without the acceptance test */
                        accepted = 1;
                        alpha = amax;
                        azz = az;
                        trial_primal(s, amax, &t);
                        fa = 0;
                    }
                }
                break;
            }
            if (accepted) wd_short = (alpha < amax) ? wd_short + 1 : 0;
            /* IPOPT filter reset heuristic: the filter is cleared when in filter_reset_trigger (5) successive
             * iterations the last rejected trial was rejected by the filter (at most max_filter_resets = 5) */
            if (accepted && s->n_filt_resets < 5) {
                s->n_filt_rej = s->last_rej_filter ? s->n_filt_rej + 1 : 0;
                if (s->n_filt_rej >= 5) {
                    s->nfilt = 0;
                    s->n_filt_resets++;
                    s->n_filt_rej = 0;
                }
            }
        }
        if (!accepted && o->soft_resto_pderror_reduction_factor > 0 && o->resto) {
            /* soft restoration phase (IPOPT TrySoftRestoStep): the damped full step if it is acceptable to
             * the filter, or if it reduces the primal-dual error by the factor */
            if (in_soft && ++soft_cnt > o->max_soft_resto_iters) {
                accepted = 0;
            } else {
                const double a = fmin(amax, az);
                trial_primal(s, a, &t);
                double tht, pht;
                trial_merit(s, &t, s->mu, &tht, &pht, NULL, NULL, NULL, NULL, NULL);
                int ft = 0, sat = ls_accept(s, ref.theta, ref.phi, ref.gd, 0.0, tht, pht, &ft);
                int ok = sat;
                if (!ok) {
                    const double mu_pd = (o->mu_strategy == 1 && s->free_mode) ? 0.0 : s->mu;
                    const double mu_keep = s->mu;
                    s->mu = mu_pd;
                    Errs ec;
                    errors(s, &ec);
                    const double pd_c = pd_error(&ec);
                    s->mu = mu_keep;
                    double* snap = (double*)malloc(sizeof(double) * (nit + nsave));
                    iter_io(s, snap, 0);
                    step_save(s, snap + nit, 0);
                    accept_step(s, a, a, &t);
                    eval_full(s);
                    s->mu = mu_pd;
                    errors(s, &ec);
                    s->mu = mu_keep;
                    const double pd_t = pd_error(&ec);
                    ok = isfinite(pd_t) && pd_t <= o->soft_resto_pderror_reduction_factor * pd_c;
                    iter_io(s, snap, 1); /* the caller accepts the trial point itself */
                    step_save(s, snap + nit, 1);
                    eval_full(s);
                    free(snap);
                }
                if (ok) {
                    accepted = 1;
                    alpha = azz = a;
                    augment = 0;
                    ++n_soft;
                    if (sat) {
                        in_soft = 0;
                        soft_cnt = 0;
                    } else {
                        in_soft = 1;
                    }
                } else {
                    accepted = 0;
                }
            }
        }
        if (getenv("NLOT_VERBOSE"))
            fprintf(stderr, "it %3d mu %.2e f %.6f th %.2e E0 %.2e dual %.2e dw %.1e amax %.2e a %.2e az %.2e nf %d%s%s%s\n",
                    iter, s->mu, s->f, theta, E0, e.dual, dw, amax, alpha, azz, s->nfilt, in_wd ? " W" : "",
                    in_soft ? " s" : "", is_tiny ? " T" : "");
        if (!accepted) {
            theta_fail = ref.theta;
            if (!o->resto) {
                status = NLOT_LS_FAILED;
                break;
            }
            /* IPOPT BacktrackingLineSearch::FindAcceptableTrialPoint: the restoration phase is not entered at
             * an almost feasible point (theta <= 1e-2 tol); without an acceptable iterate to fall back to
             * (acceptable_tol 1e-6 < tol here, so none) IPOPT stops with Restoration_Failed. */
            if (ref.theta <= 1e-2 * o->tol) {
                status = NLOT_RESTO_FAILED;
                s->term = TERM_ALMOST_FEASIBLE;
                break;
            }
            /* ---- feasibility restoration phase ---- */
            /* the current point enters the filter first: FilterLSAcceptor::PrepareRestoPhaseStart augments it with
             * the line search's reference values (the watchdog point's after StopWatchDog, where s is back at
             * that point) */
            filter_add(s, ref.theta, ref.phi);
            if (!r_alloc) {
                sol_setup(r, p, o, m, x0, xg);
                r->resto = 1;
                if (sol_alloc(r)) {
                    status = NLOT_NUMERIC;
                    break;
                }
                r_alloc = 1;
            }
            ++n_resto;
            int st = restoration(s, r, &iter, &lin_resid);
            if (st) {
                status = st;
                break;
            }
            in_soft = soft_cnt = 0;
            in_wd = wd_short = 0;
            tiny_last = 0;
            continue;
        }
        if (augment && !fa) filter_add(s, ref.theta, ref.phi);
        accept_step(s, alpha, azz, &t);
        tiny_last = is_tiny;
        ++iter;
    }
    if (dump) fclose(dump);
    free(tb);
    free(wd_it);
    free(qf_aff);
    memcpy(Xout, s->X, sizeof(double) * (N + 1) * nx);
    memcpy(Uout, s->U, sizeof(double) * N * nu);
    if (Sout) memcpy(Sout, s->S, sizeof(double) * (N + 1));
    *cost = objective(s, s->X, s->U, s->S);
    *iters_out = iter;
    if (info) {
        info[0] = *cost;
        info[1] = e.dual;
        info[2] = e.cviol;
        info[3] = lin_resid;
        info[4] = s->mu;
        info[6] = n_resto;
        info[7] = 1e6 * n_wd + 1e4 * n_soft + 1e2 * (s->n_soc_tried > 99 ? 99 : s->n_soc_tried) + n_tiny;
        info[8] = theta_fail;
        const int mr = r_alloc ? r->max_nfilt : 0;
        info[9] = s->max_nfilt > mr ? s->max_nfilt : mr;
        info[10] = s->max_nafilt;
        info[11] = s->filt_ovf + (r_alloc ? r->filt_ovf : 0);
        info[12] = s->afilt_ovf;
        info[13] = (double)(s->n_trials + (r_alloc ? r->n_trials : 0));
        /* [14] how the run ended (TERM_*): the status, told apart by where it came from */
        info[14] = status == NLOT_SOLVED ? TERM_SOLVED : status == NLOT_NUMERIC ? TERM_NUMERIC
                   : status == NLOT_TINY_STEP ? TERM_TINY : status == NLOT_LS_FAILED ? TERM_LS
                   : status == NLOT_MAXITER && s->term != TERM_MAXITER_RESTO ? TERM_MAXITER : s->term;
    }
    if (r_alloc) free(r->arena);
    free(s->arena);
    return status;
}

/* Batch of B independent instances, OpenMP over instances (the CPU baseline). */
int oracle_solve_batch(const NlotProblem* p, const NlotSolverOptions* o, const NlotMlpDesc* m, const double* x0,
                       const double* xg, const double* Xinit, double* X, double* U, double* S, double* cost,
                       int* status, int* iters, long B, int nthreads) {
    int nx = p->nx, nu = p->nu, N = p->N;
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel for schedule(dynamic, 1)
#endif
    for (long b = 0; b < B; ++b) {
        status[b] = oracle_solve_one(p, o, m, x0 + b * nx, xg + b * nx, Xinit ? Xinit + b * (N + 1) * nx : NULL,
                                     X + b * (N + 1) * nx, U + b * N * nu, S ? S + b * (N + 1) : NULL, cost + b,
                                     iters + b, NULL);
    }
    (void)nthreads;
    return 0;
}

void oracle_default_options(NlotSolverOptions* o) {
    memset(o, 0, sizeof *o);
    o->tol = 1e-4;
    o->max_iter = 1000;
    o->mu_strategy = 1;          /* adaptive + quality-function oracle (runner.py:118-119) */
    o->mu_init = 0.1;
    o->barrier_tol_factor = 0.05; /* runner.py:120 */
    o->dual_inf_tol = 1.0;
    o->constr_viol_tol = 1e-4;
    o->compl_inf_tol = 1e-4;
    o->constr_mult_init_max = 1e3;
    o->bound_push = 1e-2;
    o->bound_frac = 1e-2;
    o->max_soc = 4; /* IPOPT defaults from here on */
    o->resto = 1;
    o->watchdog_shortened_iter_trigger = 10;
    o->watchdog_trial_iter_max = 3;
    o->max_soft_resto_iters = 10;
    o->kappa_soc = 0.99;
    o->tiny_step_tol = 10 * DBL_EPSILON;
    o->tiny_step_y_tol = 1e-2;
    o->soft_resto_pderror_reduction_factor = 0.9999;
    o->required_infeasibility_reduction = 0.9;
    o->resto_penalty_parameter = 1000.0;
    o->resto_proximity_weight = 1.0;
    o->bound_mult_reset_threshold = 1000.0;
    o->resto_failure_feasibility_threshold = 0.0;
    o->general_bounds = 1; /* the bounds as constraint rows, CasADi Opti's form (runner.py:67-69,101-103) */
}

int oracle_sizeof_problem(void) { return (int)sizeof(NlotProblem); }
int oracle_sizeof_options(void) { return (int)sizeof(NlotSolverOptions); }
int oracle_sizeof_mlpdesc(void) { return (int)sizeof(NlotMlpDesc); }
int oracle_sizeof_stats(void) { return (int)sizeof(NlotSolveStats); }

/* NLP pieces for an independent solver (scripts/crosscheck_scipy.py): the knot inequalities with their pose
 * gradients and the w-weighted pose Hessian sum_j w_j d2 d_j / dpose2 (3x3 row-major) ... */
int oracle_knot_constraints_h(const NlotProblem* p, const NlotMlpDesc* m, const double* xk, double sk, const double* w,
                              double* d, double* grad3, double* hess9) {
    jet dj[NLOT_MAX_BODY];
    int mm = knot_ineq(p, m, xk, 1, dj);
    for (int a = 0; a < 9; ++a) hess9[a] = 0.0;
    for (int j = 0; j < mm; ++j) {
        d[j] = dj[j].v + ((p->use_slack && p->shape != NLOT_SHAPE_DOT) ? sk : 0.0);
        for (int i = 0; i < 3; ++i) grad3[3 * j + i] = dj[j].g[i];
        for (int a = 0; a < 3; ++a)
            for (int b = 0; b < 3; ++b) hess9[a * 3 + b] += w[j] * dj[j].h[hix(a, b)];
    }
    return mm;
}
/* ... and the defect map F(x, u) (Euler or RK4) with its Jacobians and the lambda-weighted Hessian
 * sum_i lambda_i d2 F_i / d(x, u)2 ((nx + nu)^2 row-major). */
void oracle_dyn_hess(const NlotProblem* p, const double* x, const double* u, const double* lam, double* F, double* A,
                     double* B, double* H) {
    dyn_eval(p, x, u, lam, F, A, B, H);
}
