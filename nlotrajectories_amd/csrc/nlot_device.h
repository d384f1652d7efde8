// Device-side model library of the batched solver: dynamics with hand-derived first and second
// derivatives, analytic SDFs, footprint corners + soft-min chain rule, small dense LDL^T.
// (Independent of the oracle, which derives the same quantities with forward-mode jets.)
#pragma once
#include <hip/hip_runtime.h>

#include "../../include/nlot.h"

namespace nlot {

// ---------------------------------------------------------------------------------------------
// Dynamics F(x,u) = x + dt f(x,u)  (runner.py:62-63).  For each model:
//   eval: F, A = dF/dx (NX x NX), B = dF/du (NX x NU)
//   hess: Hz += sum_i lam_i d2F_i/dz2 over z = (x, u)   ((NX+NU)^2, symmetric)
// ---------------------------------------------------------------------------------------------
template <int DYN> struct Dyn;

template <> struct Dyn<NLOT_POINT_1ST> {  // dynamics.py:33-41  f = (u0, u1, 0, 0)
    static constexpr int NX = 4, NU = 2;
    __device__ __forceinline__ static void f(const double* x, const double* u, double, double* o, double = 0) {
        o[0] = u[0]; o[1] = u[1]; o[2] = 0; o[3] = 0; (void)x;
    }
    __device__ __forceinline__ static void jac(const double* x, const double* u, double dt, double, double (*A)[NX], double (*B)[NU]) {
        for (int i = 0; i < NX; ++i) { for (int j = 0; j < NX; ++j) A[i][j] = i == j; B[i][0] = B[i][1] = 0; }
        B[0][0] = dt; B[1][1] = dt; (void)x; (void)u;
    }
    __device__ __forceinline__ static void hess(const double*, const double*, const double*, double, double, double (*)[NX + NU]) {}
};

template <> struct Dyn<NLOT_POINT_2ND> {  // dynamics.py:44-56  f = (vx, vy, ax, ay)
    static constexpr int NX = 4, NU = 2;
    __device__ __forceinline__ static void f(const double* x, const double* u, double, double* o, double = 0) {
        o[0] = x[2]; o[1] = x[3]; o[2] = u[0]; o[3] = u[1];
    }
    __device__ __forceinline__ static void jac(const double*, const double*, double dt, double, double (*A)[NX], double (*B)[NU]) {
        for (int i = 0; i < NX; ++i) { for (int j = 0; j < NX; ++j) A[i][j] = i == j; B[i][0] = B[i][1] = 0; }
        A[0][2] = dt; A[1][3] = dt; B[2][0] = dt; B[3][1] = dt;
    }
    __device__ __forceinline__ static void hess(const double*, const double*, const double*, double, double, double (*)[NX + NU]) {}
};

template <> struct Dyn<NLOT_UNICYCLE> {  // dynamics.py:59-73  f = (v c, v s, w), u = (v, w)
    static constexpr int NX = 3, NU = 2;
    __device__ __forceinline__ static void f(const double* x, const double* u, double, double* o, double = 0) {
        double s, c; sincos(x[2], &s, &c);
        o[0] = u[0] * c; o[1] = u[0] * s; o[2] = u[1];
    }
    __device__ __forceinline__ static void jac(const double* x, const double* u, double dt, double, double (*A)[NX], double (*B)[NU]) {
        double s, c; sincos(x[2], &s, &c);
        for (int i = 0; i < NX; ++i) { for (int j = 0; j < NX; ++j) A[i][j] = i == j; B[i][0] = B[i][1] = 0; }
        A[0][2] = -dt * u[0] * s; A[1][2] = dt * u[0] * c;
        B[0][0] = dt * c; B[1][0] = dt * s; B[2][1] = dt;
    }
    __device__ __forceinline__ static void hess(const double* x, const double* u, const double* l, double dt, double, double (*H)[NX + NU]) {
        double s, c; sincos(x[2], &s, &c);
        H[2][2] += dt * (-l[0] * u[0] * c - l[1] * u[0] * s);
        double t = dt * (-l[0] * s + l[1] * c);
        H[2][3] += t; H[3][2] += t;
    }
};

template <> struct Dyn<NLOT_UNICYCLE_2ND> {  // dynamics.py:76-96  f = (v c, v s, w, a, alpha)
    static constexpr int NX = 5, NU = 2;
    __device__ __forceinline__ static void f(const double* x, const double* u, double, double* o, double = 0) {
        double s, c; sincos(x[2], &s, &c);
        o[0] = x[3] * c; o[1] = x[3] * s; o[2] = x[4]; o[3] = u[0]; o[4] = u[1];
    }
    __device__ __forceinline__ static void jac(const double* x, const double*, double dt, double, double (*A)[NX], double (*B)[NU]) {
        double s, c; sincos(x[2], &s, &c);
        for (int i = 0; i < NX; ++i) { for (int j = 0; j < NX; ++j) A[i][j] = i == j; B[i][0] = B[i][1] = 0; }
        A[0][2] = -dt * x[3] * s; A[0][3] = dt * c;
        A[1][2] = dt * x[3] * c;  A[1][3] = dt * s;
        A[2][4] = dt;
        B[3][0] = dt; B[4][1] = dt;
    }
    __device__ __forceinline__ static void hess(const double* x, const double*, const double* l, double dt, double, double (*H)[NX + NU]) {
        double s, c; sincos(x[2], &s, &c);
        H[2][2] += dt * (-l[0] * x[3] * c - l[1] * x[3] * s);
        double t = dt * (-l[0] * s + l[1] * c);
        H[2][3] += t; H[3][2] += t;
    }
};

template <> struct Dyn<NLOT_ACKERMANN> {  // dynamics.py:99-118  f = (v c, v s, v tan(psi)/L, psidot)
    static constexpr int NX = 4, NU = 2;
    __device__ __forceinline__ static void f(const double* x, const double* u, double L, double* o, double = 0) {
        double s, c; sincos(x[2], &s, &c);
        o[0] = u[0] * c; o[1] = u[0] * s; o[2] = u[0] * tan(x[3]) / L; o[3] = u[1];
    }
    __device__ __forceinline__ static void jac(const double* x, const double* u, double dt, double L, double (*A)[NX], double (*B)[NU]) {
        double s, c; sincos(x[2], &s, &c);
        double tp = tan(x[3]), sec2 = 1 + tp * tp;
        for (int i = 0; i < NX; ++i) { for (int j = 0; j < NX; ++j) A[i][j] = i == j; B[i][0] = B[i][1] = 0; }
        A[0][2] = -dt * u[0] * s; A[1][2] = dt * u[0] * c; A[2][3] = dt * u[0] * sec2 / L;
        B[0][0] = dt * c; B[1][0] = dt * s; B[2][0] = dt * tp / L; B[3][1] = dt;
    }
    __device__ __forceinline__ static void hess(const double* x, const double* u, const double* l, double dt, double L, double (*H)[NX + NU]) {
        double s, c; sincos(x[2], &s, &c);
        double tp = tan(x[3]), sec2 = 1 + tp * tp;
        H[2][2] += dt * (-l[0] * u[0] * c - l[1] * u[0] * s);
        double t = dt * (-l[0] * s + l[1] * c);          // d2/dtheta dv
        H[2][4] += t; H[4][2] += t;
        H[3][3] += dt * l[2] * u[0] * 2.0 * sec2 * tp / L;  // d2/dpsi2
        double q = dt * l[2] * sec2 / L;                  // d2/dpsi dv
        H[3][4] += q; H[4][3] += q;
    }
};

template <> struct Dyn<NLOT_ACKERMANN_2ND> {  // dynamics.py:121-148, output order reproduced as written
    static constexpr int NX = 7, NU = 2;
    __device__ __forceinline__ static void f(const double* x, const double* u, double L, double* o, double = 0) {
        double s, c; sincos(x[2], &s, &c);
        double tp = tan(x[3]), q = 1 + x[3] * x[3];
        o[0] = x[4] * c; o[1] = x[4] * s; o[2] = x[4] * tp / L; o[3] = x[6];
        o[4] = (x[6] / q * x[4] + tp * u[0]) / L;  // "domega" lands in the v slot (bug F7a kept)
        o[5] = u[0]; o[6] = u[1];
    }
    __device__ __forceinline__ static void jac(const double* x, const double* u, double dt, double L, double (*A)[NX], double (*B)[NU]) {
        double s, c; sincos(x[2], &s, &c);
        double tp = tan(x[3]), sec2 = 1 + tp * tp, q = 1 + x[3] * x[3], dq = -2 * x[3] / (q * q);
        for (int i = 0; i < NX; ++i) { for (int j = 0; j < NX; ++j) A[i][j] = i == j; B[i][0] = B[i][1] = 0; }
        A[0][2] = -dt * x[4] * s; A[0][4] = dt * c;
        A[1][2] = dt * x[4] * c;  A[1][4] = dt * s;
        A[2][3] = dt * x[4] * sec2 / L; A[2][4] = dt * tp / L;
        A[3][6] = dt;
        A[4][3] = dt * (x[6] * x[4] * dq + sec2 * u[0]) / L;
        A[4][4] += dt * x[6] / q / L;
        A[4][6] = dt * x[4] / q / L;
        B[4][0] = dt * tp / L; B[5][0] = dt; B[6][1] = dt;
    }
    __device__ __forceinline__ static void hess(const double* x, const double* u, const double* l, double dt, double L, double (*H)[NX + NU]) {
        double s, c; sincos(x[2], &s, &c);
        double tp = tan(x[3]), sec2 = 1 + tp * tp, q = 1 + x[3] * x[3];
        double dq = -2 * x[3] / (q * q), d2q = (6 * x[3] * x[3] - 2) / (q * q * q);  // d(1/q), d2(1/q)
        H[2][2] += dt * (-l[0] * x[4] * c - l[1] * x[4] * s);
        double t = dt * (-l[0] * s + l[1] * c);  // theta-v
        H[2][4] += t; H[4][2] += t;
        double g33 = l[2] * x[4] * 2 * sec2 * tp / L + l[4] * (x[6] * x[4] * d2q + u[0] * 2 * sec2 * tp) / L;
        H[3][3] += dt * g33;
        double g34 = l[2] * sec2 / L + l[4] * x[6] * dq / L;  // psi-v
        H[3][4] += dt * g34; H[4][3] += dt * g34;
        double g36 = l[4] * x[4] * dq / L;                    // psi-psidot
        H[3][6] += dt * g36; H[6][3] += dt * g36;
        double g37 = l[4] * sec2 / L;                         // psi-a
        H[3][7] += dt * g37; H[7][3] += dt * g37;
        double g46 = l[4] / q / L;                            // v-psidot
        H[4][6] += dt * g46; H[6][4] += dt * g46;
    }
};

// ---------------------------------------------------------------------------------------------
// RK4 defects (opt-in, NlotProblem.integrator = NLOT_INTEG_RK4; not the reference's discretisation, which is
// Euler, runner.py:62-63).  Dyn<D + NLOT_RK4_BIAS> keeps the Euler-shaped interface of Dyn<D>: its f is the
// effective rate f_eff = (k1 + 2 k2 + 2 k3 + k4) / 6, so F = x + dt f_eff is the classical RK4 step, and its
// jac / hess differentiate f_eff exactly with second-order forward jets over z = (x, u) (the oracle does the
// same with its jets, in the same operation order).
// ---------------------------------------------------------------------------------------------
constexpr int NLOT_RK4_BIAS = 8;

template <int N>
struct Jt {  // value, gradient, lower-triangular Hessian over N variables
    double v, g[N], h[N * (N + 1) / 2];
};
template <int N> __device__ inline Jt<N> jt_const(double c) {
    Jt<N> r;
    r.v = c;
    for (int i = 0; i < N; ++i) r.g[i] = 0;
    for (int i = 0; i < N * (N + 1) / 2; ++i) r.h[i] = 0;
    return r;
}
template <int N> __device__ inline Jt<N> jt_var(double c, int i) { Jt<N> r = jt_const<N>(c); r.g[i] = 1; return r; }
template <int N> __device__ inline Jt<N> operator+(const Jt<N>& a, const Jt<N>& b) {
    Jt<N> r;
    r.v = a.v + b.v;
    for (int i = 0; i < N; ++i) r.g[i] = a.g[i] + b.g[i];
    for (int i = 0; i < N * (N + 1) / 2; ++i) r.h[i] = a.h[i] + b.h[i];
    return r;
}
template <int N> __device__ inline Jt<N> operator*(const Jt<N>& a, double c) {
    Jt<N> r;
    r.v = a.v * c;
    for (int i = 0; i < N; ++i) r.g[i] = a.g[i] * c;
    for (int i = 0; i < N * (N + 1) / 2; ++i) r.h[i] = a.h[i] * c;
    return r;
}
template <int N> __device__ inline Jt<N> jt_addc(Jt<N> a, double c) { a.v += c; return a; }
template <int N> __device__ inline Jt<N> operator*(const Jt<N>& a, const Jt<N>& b) {
    Jt<N> r;
    r.v = a.v * b.v;
    for (int i = 0; i < N; ++i) r.g[i] = a.g[i] * b.v + a.v * b.g[i];
    for (int i = 0, q = 0; i < N; ++i)
        for (int j = 0; j <= i; ++j, ++q) r.h[q] = a.h[q] * b.v + a.v * b.h[q] + a.g[i] * b.g[j] + a.g[j] * b.g[i];
    return r;
}
template <int N> __device__ inline Jt<N> jt_unary(const Jt<N>& a, double f0, double f1, double f2) {
    Jt<N> r;
    r.v = f0;
    for (int i = 0; i < N; ++i) r.g[i] = f1 * a.g[i];
    for (int i = 0, q = 0; i < N; ++i)
        for (int j = 0; j <= i; ++j, ++q) r.h[q] = f1 * a.h[q] + f2 * a.g[i] * a.g[j];
    return r;
}
// scalar helpers with one spelling for double and jets (the oracle's jet operations, nlot_oracle.c)
__device__ inline double tsin(double a) { return sin(a); }
__device__ inline double tcos(double a) { return cos(a); }
__device__ inline double ttan(double a) { return tan(a); }
__device__ inline double trecip(double a) { return 1.0 / a; }
__device__ inline double taddc(double a, double c) { return a + c; }
__device__ inline double tconst(double c, double) { return c; }
template <int N> __device__ inline Jt<N> tsin(const Jt<N>& a) { return jt_unary(a, sin(a.v), cos(a.v), -sin(a.v)); }
template <int N> __device__ inline Jt<N> tcos(const Jt<N>& a) { return jt_unary(a, cos(a.v), -sin(a.v), -cos(a.v)); }
template <int N> __device__ inline Jt<N> ttan(const Jt<N>& a) {
    const double t = tan(a.v), s2 = 1.0 + t * t;
    return jt_unary(a, t, s2, 2.0 * t * s2);
}
template <int N> __device__ inline Jt<N> trecip(const Jt<N>& a) {
    return jt_unary(a, 1.0 / a.v, -1.0 / (a.v * a.v), 2.0 / (a.v * a.v * a.v));
}
template <int N> __device__ inline Jt<N> taddc(const Jt<N>& a, double c) { return jt_addc(a, c); }
template <int N> __device__ inline Jt<N> tconst(double c, const Jt<N>&) { return jt_const<N>(c); }

// f(x, u) of model D for a double or jet scalar, in the oracle's operation order (dyn_f, nlot_oracle.c)
template <int D, class T>
__device__ inline void fgen(const T* x, const T* u, double L, T* f) {
    if constexpr (D == NLOT_POINT_1ST) {
        f[0] = u[0]; f[1] = u[1]; f[2] = tconst(0.0, x[0]); f[3] = tconst(0.0, x[0]);
    } else if constexpr (D == NLOT_POINT_2ND) {
        f[0] = x[2]; f[1] = x[3]; f[2] = u[0]; f[3] = u[1];
    } else if constexpr (D == NLOT_UNICYCLE) {
        f[0] = u[0] * tcos(x[2]); f[1] = u[0] * tsin(x[2]); f[2] = u[1];
    } else if constexpr (D == NLOT_UNICYCLE_2ND) {
        f[0] = x[3] * tcos(x[2]); f[1] = x[3] * tsin(x[2]); f[2] = x[4]; f[3] = u[0]; f[4] = u[1];
    } else if constexpr (D == NLOT_ACKERMANN) {
        f[0] = u[0] * tcos(x[2]); f[1] = u[0] * tsin(x[2]); f[2] = (u[0] * ttan(x[3])) * (1.0 / L); f[3] = u[1];
    } else {  // ackermann_2nd, vector order as written (domega in the v slot)
        f[0] = x[4] * tcos(x[2]); f[1] = x[4] * tsin(x[2]); f[2] = (x[4] * ttan(x[3])) * (1.0 / L); f[3] = x[6];
        f[4] = ((x[6] * trecip(taddc(x[3] * x[3], 1.0))) * x[4] + ttan(x[3]) * u[0]) * (1.0 / L);
        f[5] = u[0]; f[6] = u[1];
    }
}
// f_eff = (k1 + 2 k2 + 2 k3 + k4) / 6 with stage points x + k (dt / 2), x + k (dt / 2), x + k dt
template <int D, int NX, class T>
__device__ inline void rk4_feff(const T* x, const T* u, double dt, double L, T* fe) {
    T k[NX], xs[NX];
    fgen<D>(x, u, L, k);
#pragma unroll
    for (int i = 0; i < NX; ++i) { fe[i] = k[i]; xs[i] = x[i] + k[i] * (0.5 * dt); }
    fgen<D>(xs, u, L, k);
#pragma unroll
    for (int i = 0; i < NX; ++i) { fe[i] = fe[i] + k[i] * 2.0; xs[i] = x[i] + k[i] * (0.5 * dt); }
    fgen<D>(xs, u, L, k);
#pragma unroll
    for (int i = 0; i < NX; ++i) { fe[i] = fe[i] + k[i] * 2.0; xs[i] = x[i] + k[i] * dt; }
    fgen<D>(xs, u, L, k);
#pragma unroll
    for (int i = 0; i < NX; ++i) fe[i] = (fe[i] + k[i]) * (1.0 / 6.0);
}
template <int D, int NX, int NU>
__device__ __noinline__ void rk4_jets(const double* x, const double* u, double dt, double L, Jt<NX + NU>* fe) {
    constexpr int N = NX + NU;
    Jt<N> xj[NX], uj[NU];
    for (int i = 0; i < NX; ++i) xj[i] = jt_var<N>(x[i], i);
    for (int i = 0; i < NU; ++i) uj[i] = jt_var<N>(u[i], NX + i);
    rk4_feff<D, NX>(xj, uj, dt, L, fe);
}

template <int D>
struct DynRk4 {
    static constexpr int NX = Dyn<D>::NX, NU = Dyn<D>::NU, N = NX + NU;
    __device__ static void f(const double* x, const double* u, double L, double* o, double dt) {
        rk4_feff<D, NX>(x, u, dt, L, o);
    }
    __device__ static void jac(const double* x, const double* u, double dt, double L, double (*A)[NX], double (*B)[NU]) {
        Jt<N> fe[NX];
        rk4_jets<D, NX, NU>(x, u, dt, L, fe);
        for (int i = 0; i < NX; ++i) {
            for (int j = 0; j < NX; ++j) A[i][j] = (i == j ? 1.0 : 0.0) + dt * fe[i].g[j];
            for (int j = 0; j < NU; ++j) B[i][j] = dt * fe[i].g[NX + j];
        }
    }
    __device__ static void hess(const double* x, const double* u, const double* l, double dt, double L, double (*H)[N]) {
        Jt<N> fe[NX];
        rk4_jets<D, NX, NU>(x, u, dt, L, fe);
        for (int a = 0; a < N; ++a)
            for (int b = 0; b < N; ++b) {
                const int q = a >= b ? a * (a + 1) / 2 + b : b * (b + 1) / 2 + a;
                double s = 0;
                for (int i = 0; i < NX; ++i) s += l[i] * fe[i].h[q];
                H[a][b] += dt * s;
            }
    }
};
template <> struct Dyn<NLOT_POINT_1ST + NLOT_RK4_BIAS> : DynRk4<NLOT_POINT_1ST> {};
template <> struct Dyn<NLOT_POINT_2ND + NLOT_RK4_BIAS> : DynRk4<NLOT_POINT_2ND> {};
template <> struct Dyn<NLOT_UNICYCLE + NLOT_RK4_BIAS> : DynRk4<NLOT_UNICYCLE> {};
template <> struct Dyn<NLOT_UNICYCLE_2ND + NLOT_RK4_BIAS> : DynRk4<NLOT_UNICYCLE_2ND> {};
template <> struct Dyn<NLOT_ACKERMANN + NLOT_RK4_BIAS> : DynRk4<NLOT_ACKERMANN> {};
template <> struct Dyn<NLOT_ACKERMANN_2ND + NLOT_RK4_BIAS> : DynRk4<NLOT_ACKERMANN_2ND> {};

// ---------------------------------------------------------------------------------------------
// 2-D hyper-dual number (value, gradient, Hessian in (x, y)) for the analytic SDFs
// ---------------------------------------------------------------------------------------------
struct HD {
    double v, gx, gy, hxx, hxy, hyy;
};
__device__ __forceinline__ HD hd_var_x(double x) { return {x, 1, 0, 0, 0, 0}; }
__device__ __forceinline__ HD hd_var_y(double y) { return {y, 0, 1, 0, 0, 0}; }
__device__ __forceinline__ HD hd_const(double c) { return {c, 0, 0, 0, 0, 0}; }
__device__ __forceinline__ HD operator+(HD a, HD b) { return {a.v + b.v, a.gx + b.gx, a.gy + b.gy, a.hxx + b.hxx, a.hxy + b.hxy, a.hyy + b.hyy}; }
__device__ __forceinline__ HD operator-(HD a, HD b) { return {a.v - b.v, a.gx - b.gx, a.gy - b.gy, a.hxx - b.hxx, a.hxy - b.hxy, a.hyy - b.hyy}; }
__device__ __forceinline__ HD operator+(HD a, double c) { a.v += c; return a; }
__device__ __forceinline__ HD operator*(double c, HD a) { return {c * a.v, c * a.gx, c * a.gy, c * a.hxx, c * a.hxy, c * a.hyy}; }
__device__ __forceinline__ HD operator*(HD a, HD b) {
    return {a.v * b.v, a.gx * b.v + a.v * b.gx, a.gy * b.v + a.v * b.gy,
            a.hxx * b.v + a.v * b.hxx + 2 * a.gx * b.gx,
            a.hxy * b.v + a.v * b.hxy + a.gx * b.gy + a.gy * b.gx,
            a.hyy * b.v + a.v * b.hyy + 2 * a.gy * b.gy};
}
__device__ __forceinline__ HD hd_chain(HD a, double f0, double f1, double f2) {
    return {f0, f1 * a.gx, f1 * a.gy, f1 * a.hxx + f2 * a.gx * a.gx, f1 * a.hxy + f2 * a.gx * a.gy,
            f1 * a.hyy + f2 * a.gy * a.gy};
}
__device__ __forceinline__ HD hd_sqrt(HD a) { double s = sqrt(a.v); return hd_chain(a, s, 0.5 / s, -0.25 / (s * a.v)); }
__device__ __forceinline__ HD hd_exp(HD a) { double e = exp(a.v); return hd_chain(a, e, e, e); }
__device__ __forceinline__ HD hd_log(HD a) { return hd_chain(a, log(a.v), 1.0 / a.v, -1.0 / (a.v * a.v)); }

// CircleObstacle.approximated_sdf (core/sdf/casadi.py:33-41): |p - c| - (r + m)
__device__ __forceinline__ HD sdf_circle(double cx, double cy, double r, double m, double x, double y) {
    double dx = x - cx, dy = y - cy, rr = sqrt(dx * dx + dy * dy);
    double nx = dx / rr, ny = dy / rr;
    return {rr - (r + m), nx, ny, (1 - nx * nx) / rr, -nx * ny / rr, (1 - ny * ny) / rr};
}
// SquareObstacle.approximated_sdf (core/sdf/casadi.py:69-118)
__device__ __forceinline__ HD sdf_square(double cx, double cy, double size, double m, double x, double y) {
    const double half = size / 2 + m;
    HD X = hd_var_x(x) + (-cx), Y = hd_var_y(y) + (-cy);
    HD dx = hd_sqrt(X * X + 1e-6), dy = hd_sqrt(Y * Y + 1e-6);
    HD d_x = dx + (-half), d_y = dy + (-half);
    auto smax = [](HD a, HD b) { HD d = a - b; return 0.5 * (a + b + hd_sqrt(d * d + 1e-6)); };
    auto smin = [](HD a, HD b) { HD d = a - b; return 0.5 * (a + b - hd_sqrt(d * d + 1e-6)); };
    HD z = hd_const(0.0);
    HD xo = smax(d_x, z), yo = smax(d_y, z);
    HD outside = hd_sqrt(xo * xo + yo * yo);
    HD inside = smin(smax(d_x, d_y), z);
    return outside + inside;
}
__device__ __forceinline__ HD hd_tanh(HD a) { double t = tanh(a.v), d = 1 - t * t; return hd_chain(a, t, d, -2 * t * d); }
__device__ __forceinline__ HD hd_divc(HD a, double c) { return {a.v / c, a.gx / c, a.gy / c, a.hxx / c, a.hxy / c, a.hyy / c}; }
// PolygonObstacle.approximated_sdf (casadi.py:150-186; EllipticRingObstacle is a polygon of its arc points):
// soft_min of the edge-segment distances (hard clamp of the projection), signed by tanh(100 (x - cx)(y - cy))
__device__ __forceinline__ HD sdf_polygon(const NlotProblem& p, const NlotObstacle& o, double x, double y) {
    const double(*V)[2] = p.verts + o.v0;
    const double a = p.softmin_alpha;
    HD X = hd_var_x(x), Y = hd_var_y(y), sum = hd_const(0.0);
    for (int e = 0; e < o.nv; ++e) {
        const int e1 = e + 1 < o.nv ? e + 1 : 0;
        const double x0 = V[e][0], y0 = V[e][1], dx = V[e1][0] - x0, dy = V[e1][1] - y0;
        const double seg = dx * dx + dy * dy + 1e-6;
        HD traw = hd_divc(dx * (X + (-x0)) + dy * (Y + (-y0)), seg);
        HD t = traw.v < 0.0 ? hd_const(0.0) : traw.v > 1.0 ? hd_const(1.0) : traw;
        HD qx = X - (dx * t + x0), qy = Y - (dy * t + y0);
        sum = sum + hd_exp((-a) * hd_sqrt(qx * qx + qy * qy));
    }
    HD md = (-1.0 / a) * hd_log(sum);
    HD sign = hd_tanh(100.0 * ((X + (-o.cx)) * (Y + (-o.cy))));
    return sign * md + (-o.margin);
}
// TrapezoidObstacle.approximated_sdf (casadi.py:317-374), soft helpers with soft_abs eps 1e-8 (casadi.py:288-312)
__device__ __forceinline__ HD sdf_trapezoid(const NlotProblem& p, const NlotObstacle& o, double x, double y) {
    const double(*V)[2] = p.verts + o.v0;
    auto smax = [](HD a, HD b) { HD d = a - b; return 0.5 * (a + b + hd_sqrt(d * d + 1e-8)); };
    auto smin = [](HD a, HD b) { HD d = a - b; return 0.5 * (a + b - hd_sqrt(d * d + 1e-8)); };
    HD X = hd_var_x(x), Y = hd_var_y(y), zero = hd_const(0.0), one = hd_const(1.0), inner_max = zero, outside = zero;
    for (int e = 0; e < o.nv; ++e) {
        const int e1 = e + 1 < o.nv ? e + 1 : 0;
        const double x0 = V[e][0], y0 = V[e][1], ex = V[e1][0] - x0, ey = V[e1][1] - y0;
        const double nl = sqrt(ey * ey + ex * ex + 1e-6), nx = ey / nl, ny = -ex / nl;
        HD d = nx * (X + (-x0)) + ny * (Y + (-y0)) + (-o.margin);
        inner_max = e == 0 ? d : smax(inner_max, d);
    }
    HD inside = smin(inner_max, zero);
    for (int e = 0; e < o.nv; ++e) {
        const int e1 = e + 1 < o.nv ? e + 1 : 0;
        const double x0 = V[e][0], y0 = V[e][1], ex = V[e1][0] - x0, ey = V[e1][1] - y0;
        const double seg = ex * ex + ey * ey + 1e-6;
        HD t = smin(one, smax(zero, hd_divc(ex * (X + (-x0)) + ey * (Y + (-y0)), seg)));
        HD qx = X - (ex * t + x0), qy = Y - (ey * t + y0);
        HD dist = hd_sqrt(qx * qx + qy * qy + 1e-6);
        outside = e == 0 ? dist : smin(outside, dist);
    }
    return outside + inside + (-o.margin);
}
__device__ __forceinline__ HD sdf_prim(const NlotProblem& p, const NlotObstacle& o, double x, double y) {
    switch (o.type) {
        case NLOT_OBS_CIRCLE: return sdf_circle(o.cx, o.cy, o.size, o.margin, x, y);
        case NLOT_OBS_SQUARE: return sdf_square(o.cx, o.cy, o.size, o.margin, x, y);
        case NLOT_OBS_POLYGON: return sdf_polygon(p, o, x, y);
        default: return sdf_trapezoid(p, o, x, y);
    }
}
// MultiObstacle.approximated_sdf (casadi.py:385-386): soft_min over obstacles, utils.py:18-33; a group (a
// MultiObstacle inside the scene: ConvexEllipticRing, ConvexSObstacle) is soft_min'ed first, one term
__device__ __forceinline__ HD sdf_scene(const NlotProblem& p, double x, double y, bool derivs) {
    const double a = p.softmin_alpha;
    HD sum = hd_const(0.0);
    for (int i = 0; i < p.n_obs;) {
        HD v;
        const int g = p.obs[i].group;
        if (g < 0) {
            v = sdf_prim(p, p.obs[i], x, y);
            ++i;
        } else {
            HD in = hd_const(0.0);
            for (; i < p.n_obs && p.obs[i].group == g; ++i) in = in + hd_exp((-a) * sdf_prim(p, p.obs[i], x, y));
            v = (-1.0 / a) * hd_log(in);
        }
        sum = sum + hd_exp((-a) * v);
    }
    (void)derivs;
    return (-1.0 / a) * hd_log(sum);
}

// ---------------------------------------------------------------------------------------------
// Small dense symmetric indefinite LDL^T (1x1 diagonal pivoting on the largest |a_ii|).
// Returns 0 (nneg = negative pivots) or 2 if numerically singular.  n <= NMAX compile-time.
// ---------------------------------------------------------------------------------------------
template <int NMAX>
__device__ __forceinline__ int ldl_factor(double (*a)[NMAX], int n, int* perm, int* nneg) {
    double scale = 1e-300;
#pragma unroll
    for (int i = 0; i < NMAX; ++i)
#pragma unroll
        for (int j = 0; j < NMAX; ++j)
            if (i < n && j < n) scale = fmax(scale, fabs(a[i][j]));
#pragma unroll
    for (int i = 0; i < NMAX; ++i) perm[i] = i;
    *nneg = 0;
#pragma unroll
    for (int j = 0; j < NMAX; ++j) {
        if (j >= n) break;
        int pv = j;
        double best = fabs(a[j][j]);
#pragma unroll
        for (int i = j + 1; i < NMAX; ++i)
            if (i < n && fabs(a[i][i]) > best) {
                best = fabs(a[i][i]);
                pv = i;
            }
        if (pv != j) {  // symmetric swap j <-> pv with compile-time register indices only
#pragma unroll
            for (int c = 0; c < NMAX; ++c) {
                double rowp = 0;
#pragma unroll
                for (int r = 0; r < NMAX; ++r)
                    if (r == pv) rowp = a[r][c];
#pragma unroll
                for (int r = 0; r < NMAX; ++r)
                    if (r == pv) a[r][c] = a[j][c];
                a[j][c] = rowp;
            }
#pragma unroll
            for (int r = 0; r < NMAX; ++r) {
                double colp = 0;
#pragma unroll
                for (int c = 0; c < NMAX; ++c)
                    if (c == pv) colp = a[r][c];
#pragma unroll
                for (int c = 0; c < NMAX; ++c)
                    if (c == pv) a[r][c] = a[r][j];
                a[r][j] = colp;
            }
            int pp = 0;
#pragma unroll
            for (int r = 0; r < NMAX; ++r)
                if (r == pv) pp = perm[r];
#pragma unroll
            for (int r = 0; r < NMAX; ++r)
                if (r == pv) perm[r] = perm[j];
            perm[j] = pp;
        }
        double d = a[j][j];
        if (!(fabs(d) > 1e-13 * scale) || !isfinite(d)) return 2;
        if (d < 0) (*nneg)++;
        double col[NMAX];
#pragma unroll
        for (int i = 0; i < NMAX; ++i) col[i] = (i > j && i < n) ? a[i][j] : 0.0;
#pragma unroll
        for (int i = 0; i < NMAX; ++i) {
            if (i <= j || i >= n) continue;
#pragma unroll
            for (int k = 0; k < NMAX; ++k)
                if (k > j && k <= i) a[i][k] -= col[i] * col[k] / d;
            a[i][j] = col[i] / d;
        }
#pragma unroll
        for (int i = 0; i < NMAX; ++i)
#pragma unroll
            for (int k = 0; k < NMAX; ++k)
                if (i > j && k > i && k < n && i < n) a[i][k] = a[k][i];
    }
    return 0;
}
// Solve with the factor for one right-hand side (in place).
template <int NMAX>
__device__ __forceinline__ void ldl_solve1(const double (*a)[NMAX], int n, const int* perm, double* x) {
    double t[NMAX];
#pragma unroll
    for (int i = 0; i < NMAX; ++i) t[i] = 0;
    // t = P x  (perm[i] = original index at position i)
#pragma unroll
    for (int i = 0; i < NMAX; ++i)
#pragma unroll
        for (int q = 0; q < NMAX; ++q)
            if (i < n && perm[i] == q) t[i] = x[q];
#pragma unroll
    for (int i = 0; i < NMAX; ++i)
#pragma unroll
        for (int k = 0; k < NMAX; ++k)
            if (i < n && k < i) t[i] -= a[i][k] * t[k];
#pragma unroll
    for (int i = 0; i < NMAX; ++i)
        if (i < n) t[i] /= a[i][i];
#pragma unroll
    for (int i = NMAX - 1; i >= 0; --i)
#pragma unroll
        for (int k = 0; k < NMAX; ++k)
            if (i < n && k > i && k < n) t[i] -= a[k][i] * t[k];
#pragma unroll
    for (int i = 0; i < NMAX; ++i)
#pragma unroll
        for (int q = 0; q < NMAX; ++q)
            if (i < n && perm[i] == q) x[q] = t[i];
}

}  // namespace nlot
