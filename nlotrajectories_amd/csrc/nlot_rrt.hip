// Batched RRT initializer (core/trajectory_initialization.py:58-239, RRTInitializer) for gfx950.
//
// One wavefront per instance.  The scalar control flow of the reference's loop runs redundantly on all 64 lanes
// (every lane holds the same values); the two data-parallel parts spread over the lanes:
//   * nearest node: the lanes scan the tree with a stride of 64 and reduce (distance, index) — the first index
//     on ties, as np.argmin;
//   * collision checks: the sample points of a segment (i / n along it, n = ceil(|p2 - p1| / step)) are spread
//     over the lanes and OR-reduced.
// The tree and the path buffers live in the caller's workspace (instance-major); lane 0 writes them and a
// workgroup fence publishes each write to the other lanes.  The path post-processing (intermediate points at
// turns > 60 degrees, greedy shortcuts, not-a-knot cubic spline as scipy's CubicSpline builds it) is serial on
// every lane except the shortcut's collision checks.
//
// Randomness: the reference draws from Python's global `random` (unseeded); here a counter-based splitmix64 of
// (seed, instance, iteration, draw) — the same stream oracle/rrt_oracle.py draws, so the trees are comparable.
#include <cmath>

#include "nlot_internal.h"

namespace nlot {
namespace {

__host__ __device__ inline uint64_t mix64(uint64_t z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
// uniform double in [0, 1): draw k (0: goal test, 1: x, 2: y) of iteration it of instance b
__device__ inline double u01(uint64_t key, int it, int k) {
    return (double)(mix64(key ^ (uint64_t)(4 * (int64_t)it + k)) >> 11) * 0x1.0p-53;
}

// MultiObstacle.sdf (casadi.py:381-383): the minimum of the obstacles' exact SDFs (a group's too)
//   circle  casadi.py:33-38      square  casadi.py:54-67
//   polygon / trapezoid  PolygonObstacle.sdf casadi.py:135-148: distance to the boundary, negative inside
__device__ double exact_sdf(const NlotProblem& p, double x, double y) {
    double best = INFINITY;
    for (int i = 0; i < p.n_obs; ++i) {
        const NlotObstacle& o = p.obs[i];
        double v;
        if (o.type == NLOT_OBS_CIRCLE) {
            const double dx = x - o.cx, dy = y - o.cy;
            v = sqrt(dx * dx + dy * dy) - (o.size + o.margin);
        } else if (o.type == NLOT_OBS_SQUARE) {
            const double half = o.size / 2 + o.margin;
            const double dx = fabs(x - o.cx) - half, dy = fabs(y - o.cy) - half;
            const double ox = fmax(dx, 0.0), oy = fmax(dy, 0.0);
            v = sqrt(ox * ox + oy * oy) + fmin(fmax(dx, dy), 0.0);
        } else {
            const double(*V)[2] = p.verts + o.v0;
            double d = INFINITY;
            bool inside = false;
            for (int e = 0; e < o.nv; ++e) {
                const int e1 = e + 1 < o.nv ? e + 1 : 0;
                const double x0 = V[e][0], y0 = V[e][1], x1 = V[e1][0], y1 = V[e1][1];
                const double ex = x1 - x0, ey = y1 - y0;
                double t = ((x - x0) * ex + (y - y0) * ey) / (ex * ex + ey * ey);
                t = fmin(fmax(t, 0.0), 1.0);
                const double qx = x - (x0 + t * ex), qy = y - (y0 + t * ey);
                d = fmin(d, sqrt(qx * qx + qy * qy));
                if ((y0 > y) != (y1 > y) && x < x0 + (y - y0) * ex / (y1 - y0)) inside = !inside;
            }
            v = (inside ? -d : d) - o.margin;
        }
        best = fmin(best, v);
    }
    return best;
}

__device__ inline int wave_any(int v) {
    for (int o = 32; o > 0; o >>= 1) v |= __shfl_xor(v, o);
    return v;
}

// trajectory_initialization.py:115-128 / 131-138: every sample point p1 + (p2 - p1) (i / n), i = 0..n, has
// sdf >= inflation (all lanes return the same answer)
__device__ bool collision_free(const NlotProblem& p, double x1, double y1, double x2, double y2, double step,
                               double infl, int lane) {
    const double dx = x2 - x1, dy = y2 - y1;
    const double dist = sqrt(dx * dx + dy * dy);
    const int n = max(1, (int)ceil(dist / step));
    int hit = 0;
    for (int i = lane; i <= n; i += 64) {
        const double f = (double)i / (double)n;
        if (exact_sdf(p, x1 + dx * f, y1 + dy * f) < infl) hit = 1;
    }
    return !wave_any(hit);
}

// np.linspace(a, b, num)[i]: i * ((b - a) / (num - 1)) + a, the last one exactly b
__device__ inline double linspace_at(double a, double b, int num, int i) {
    if (num == 1) return a;
    if (i == num - 1) return b;
    return (double)i * ((b - a) / (double)(num - 1)) + a;
}

struct InstWs {
    double *nx, *ny, *px, *py, *qx, *qy, *s, *lo, *di, *up, *rb, *slope, *d1;
    int* par;
};
__device__ inline InstWs inst_ws(double* base, int cap) {
    InstWs w;
    w.nx = base;
    w.ny = w.nx + cap;
    w.par = (int*)(w.ny + cap);
    w.px = w.ny + 2 * cap;  // path buffers hold up to 2 cap points (intermediate points at most double it)
    w.py = w.px + 2 * cap;
    w.qx = w.py + 2 * cap;
    w.qy = w.qx + 2 * cap;
    w.s = w.qy + 2 * cap;  // spline: parameter, tridiagonal system, slopes, derivatives (one coordinate at a time)
    w.lo = w.s + 2 * cap;
    w.di = w.lo + 2 * cap;
    w.up = w.di + 2 * cap;
    w.rb = w.up + 2 * cap;
    w.slope = w.rb + 2 * cap;
    w.d1 = w.slope + 2 * cap;
    return w;
}
__host__ __device__ constexpr size_t inst_ws_doubles(int cap) { return (size_t)cap * 3 + (size_t)22 * cap; }

// scipy CubicSpline(s, y, bc_type='not-a-knot') first derivatives d1[0..m) (scipy/interpolate/_cubic.py): the
// n = 2 line, the n = 3 parabola, or the banded system with the not-a-knot end rows; solved here by the Thomas
// algorithm (scipy: LAPACK gbsv with partial pivoting; the two agree to rounding)
__device__ void spline_slopes(const InstWs& w, const double* y, int m) {
    double *s = w.s, *sl = w.slope, *d = w.d1;
    for (int i = 0; i + 1 < m; ++i) sl[i] = (y[i + 1] - y[i]) / (s[i + 1] - s[i]);
    if (m == 2) {
        d[0] = d[1] = sl[0];
        return;
    }
    if (m == 3) {  // A = [[1, 1, 0], [dx1, 2 (dx0 + dx1), dx0], [0, 1, 1]], b = [2 sl0, 3 (dx0 sl1 + dx1 sl0), 2 sl1]
        const double dx0 = s[1] - s[0], dx1 = s[2] - s[1];
        const double b0 = 2 * sl[0], b1 = 3 * (dx0 * sl[1] + dx1 * sl[0]), b2 = 2 * sl[1];
        // d0 = b0 - d1, d2 = b2 - d1: dx1 (b0 - d1) + 2 (dx0 + dx1) d1 + dx0 (b2 - d1) = b1
        const double dm = (b1 - dx1 * b0 - dx0 * b2) / (2 * (dx0 + dx1) - dx1 - dx0);
        d[0] = b0 - dm;
        d[1] = dm;
        d[2] = b2 - dm;
        return;
    }
    double *lo = w.lo, *di = w.di, *up = w.up, *rb = w.rb;  // row i: lo[i] d[i-1] + di[i] d[i] + up[i] d[i+1]
    for (int i = 1; i + 1 < m; ++i) {
        const double dxm = s[i] - s[i - 1], dxp = s[i + 1] - s[i];
        lo[i] = dxp;
        di[i] = 2 * (dxm + dxp);
        up[i] = dxm;
        rb[i] = 3 * (dxp * sl[i - 1] + dxm * sl[i]);
    }
    {  // not-a-knot start: dx1 d0 + (s2 - s0) d1 = ((dx0 + 2 dd) dx1 sl0 + dx0^2 sl1) / dd
        const double dx0 = s[1] - s[0], dx1 = s[2] - s[1], dd = s[2] - s[0];
        di[0] = dx1;
        up[0] = dd;
        rb[0] = ((dx0 + 2 * dd) * dx1 * sl[0] + dx0 * dx0 * sl[1]) / dd;
    }
    {  // not-a-knot end: (s[-1] - s[-3]) d[-2] + dx[-2] d[-1] = (dx[-1]^2 sl[-2] + (2 dd + dx[-1]) dx[-2] sl[-1]) / dd
        const double dxl = s[m - 1] - s[m - 2], dxp = s[m - 2] - s[m - 3], dd = s[m - 1] - s[m - 3];
        lo[m - 1] = dd;
        di[m - 1] = dxp;
        rb[m - 1] = (dxl * dxl * sl[m - 3] + (2 * dd + dxl) * dxp * sl[m - 2]) / dd;
    }
    // Thomas: the first row has two unknowns (d0, d1) and the second three; eliminate forward
    for (int i = 1; i < m; ++i) {
        const double f = lo[i] / di[i - 1];
        di[i] -= f * up[i - 1];
        rb[i] -= f * rb[i - 1];
    }
    d[m - 1] = rb[m - 1] / di[m - 1];
    for (int i = m - 2; i >= 0; --i) d[i] = (rb[i] - up[i] * d[i + 1]) / di[i];
}

// CubicHermiteSpline coefficients and PPoly evaluation (Horner, interval by searchsorted side='right')
__device__ double spline_eval(const InstWs& w, const double* y, int m, double v) {
    const double* s = w.s;
    int i = 0;
    while (i + 1 < m - 1 && s[i + 1] <= v) ++i;
    const double dx = s[i + 1] - s[i], sl = w.slope[i], d0 = w.d1[i], d1 = w.d1[i + 1];
    const double t = (d0 + d1 - 2 * sl) / dx;
    const double c0 = t / dx, c1 = (sl - d0) / dx - t, c2 = d0, c3 = y[i];
    const double q = v - s[i];
    return ((c0 * q + c1) * q + c2) * q + c3;
}

__global__ __launch_bounds__(64) void k_rrt(const NlotProblem* __restrict__ pp, NlotRrtOptions o,
                                            const double* __restrict__ x0, const double* __restrict__ xg,
                                            double* __restrict__ Xinit, int32_t* __restrict__ ok, double* ws, int64_t B,
                                            double infl) {
    const int64_t b = blockIdx.x;
    if (b >= B) return;
    const int lane = threadIdx.x;
    const NlotProblem& p = *pp;
    const int nx = p.nx, npts = p.N + 1, cap = o.max_iter + 2;
    const InstWs w = inst_ws(ws + (size_t)b * inst_ws_doubles(cap), cap);
    const double sx = x0[b * nx], sy = x0[b * nx + 1], gx = xg[b * nx], gy = xg[b * nx + 1];
    const double step = o.step_size;
    const uint64_t key = mix64(o.seed ^ mix64((uint64_t)(b + o.first_instance)));
    if (lane == 0) {
        w.nx[0] = sx;
        w.ny[0] = sy;
        w.par[0] = -1;
    }
    __threadfence_block();
    int n = 1, final_parent = -1;
    for (int it = 0; it < o.max_iter; ++it) {
        double rx, ry;
        if (u01(key, it, 0) < o.goal_sample_rate) {
            rx = gx;
            ry = gy;
        } else {
            rx = o.bounds[0][0] + (o.bounds[1][0] - o.bounds[0][0]) * u01(key, it, 1);
            ry = o.bounds[0][1] + (o.bounds[1][1] - o.bounds[0][1]) * u01(key, it, 2);
        }
        // nearest (first index on ties)
        double bd = INFINITY;
        int bi = 0x7fffffff;
        for (int j = lane; j < n; j += 64) {
            const double dx = rx - w.nx[j], dy = ry - w.ny[j];
            const double dd = sqrt(dx * dx + dy * dy);
            if (dd < bd) {
                bd = dd;
                bi = j;
            }
        }
        for (int off = 32; off > 0; off >>= 1) {
            const double od = __shfl_xor(bd, off);
            const int oi = __shfl_xor(bi, off);
            if (od < bd || (od == bd && oi < bi)) {
                bd = od;
                bi = oi;
            }
        }
        const double ax = w.nx[bi], ay = w.ny[bi];
        const double dx = rx - ax, dy = ry - ay;
        const double nrm = sqrt(dx * dx + dy * dy);
        if (nrm == 0.0) continue;
        const double qx = ax + (dx / nrm) * step, qy = ay + (dy / nrm) * step;
        if (!collision_free(p, ax, ay, qx, qy, step, infl, lane)) continue;
        if (lane == 0) {
            w.nx[n] = qx;
            w.ny[n] = qy;
            w.par[n] = bi;
        }
        __threadfence_block();
        ++n;
        const double ex = qx - gx, ey = qy - gy;
        if (sqrt(ex * ex + ey * ey) < step) {  // the goal joins the tree (no collision check, as the reference)
            final_parent = n - 1;
            break;
        }
    }
    double* X = Xinit + (size_t)b * npts * nx;
    if (final_parent < 0) {  // the reference raises RuntimeError("RRT failed to find a path within max_iter.")
        for (int i = lane; i < npts * nx; i += 64) {
            const int k = i / nx, c = i % nx;
            X[i] = linspace_at(x0[b * nx + c], xg[b * nx + c], npts, k);
        }
        if (lane == 0) ok[b] = 0;
        return;
    }
    // raw path start -> goal
    int m = 1;
    for (int j = final_parent; j >= 0; j = w.par[j]) ++m;
    if (lane == 0) {
        w.px[m - 1] = gx;
        w.py[m - 1] = gy;
        int k = m - 2;
        for (int j = final_parent; j >= 0; j = w.par[j], --k) {
            w.px[k] = w.nx[j];
            w.py[k] = w.ny[j];
        }
        // insert_intermediate_points (:161-173): a midpoint before every point whose turn exceeds 60 degrees
        int q = 0;
        w.qx[q] = w.px[0];
        w.qy[q++] = w.py[0];
        for (int i = 1; i + 1 < m; ++i) {
            const double v1x = w.px[i] - w.px[i - 1], v1y = w.py[i] - w.py[i - 1];
            const double v2x = w.px[i + 1] - w.px[i], v2y = w.py[i + 1] - w.py[i];
            const double c = (v1x * v2x + v1y * v2y) / (sqrt(v1x * v1x + v1y * v1y) * sqrt(v2x * v2x + v2y * v2y));
            const double deg = acos(fmin(fmax(c, -1.0), 1.0)) * 57.29577951308232;
            if (deg > 60.0) {
                w.qx[q] = (w.px[i] + w.px[i - 1]) / 2;
                w.qy[q++] = (w.py[i] + w.py[i - 1]) / 2;
            }
            w.qx[q] = w.px[i];
            w.qy[q++] = w.py[i];
        }
        w.qx[q] = w.px[m - 1];
        w.qy[q++] = w.py[m - 1];
        w.par[0] = q;  // hand the count to the other lanes (the tree is no longer needed)
    }
    __threadfence_block();
    const int mq = w.par[0];
    // _shortcut_path (:130-150): from each kept point, the farthest later point reachable collision-free
    int mp = 1, i = 0;
    if (lane == 0) {
        w.px[0] = w.qx[0];
        w.py[0] = w.qy[0];
    }
    while (i < mq - 1) {
        int j = mq - 1;
        while (j > i + 1) {
            if (collision_free(p, w.qx[i], w.qy[i], w.qx[j], w.qy[j], step, infl, lane)) break;
            --j;
        }
        if (lane == 0) {
            w.px[mp] = w.qx[j];
            w.py[mp] = w.qy[j];
        }
        ++mp;
        i = j;
    }
    __threadfence_block();
    // _bspline_curve (:152-159): the straight line for <= 2 points, else a not-a-knot cubic spline per coordinate
    // over s = linspace(0, 1, mp), at linspace(0, 1, npts)
    if (mp <= 2) {
        for (int k = lane; k < npts; k += 64) {
            X[k * nx + 0] = linspace_at(w.px[0], w.px[mp - 1], npts, k);
            X[k * nx + 1] = linspace_at(w.py[0], w.py[mp - 1], npts, k);
        }
    } else {
        for (int c = 0; c < 2; ++c) {
            const double* y = c == 0 ? w.px : w.py;
            if (lane == 0) {
                for (int k = 0; k < mp; ++k) w.s[k] = linspace_at(0.0, 1.0, mp, k);
                spline_slopes(w, y, mp);
            }
            __threadfence_block();
            for (int k = lane; k < npts; k += 64) X[k * nx + c] = spline_eval(w, y, mp, linspace_at(0.0, 1.0, npts, k));
            __threadfence_block();
        }
    }
    for (int k = lane; k < npts; k += 64)
        for (int c = 2; c < nx; ++c) X[k * nx + c] = 0.0;  // lifted with zeros (:233-235)
    if (lane == 0) ok[b] = 1;
}

}  // namespace
}  // namespace nlot

// workspace: the device copy of NlotProblem (kernels read it through a pointer), then the instance buffers
static constexpr size_t kRrtHdr = 16384;
static_assert(sizeof(NlotProblem) <= kRrtHdr, "RRT workspace header");

extern "C" size_t nlot_rrt_workspace_size(const NlotRrtOptions* opt, int64_t B) {
    if (!opt || opt->max_iter < 1 || B < 0) return 0;
    return kRrtHdr + nlot::inst_ws_doubles(opt->max_iter + 2) * sizeof(double) * (size_t)B;
}

extern "C" int32_t nlot_rrt_init(const NlotProblem* prob, const NlotRrtOptions* opt, const double* x0,
                                 const double* xg, double* X_init, int32_t* ok, int64_t B, void* workspace,
                                 size_t workspace_bytes, void* stream) {
    using namespace nlot;
    if (!prob || !opt || !x0 || !xg || !X_init || !ok || B < 0) {
        set_error("nlot_rrt_init: null argument");
        return NLOT_ERR_INVALID;
    }
    if (B == 0) return NLOT_OK;
    if (opt->max_iter < 1 || !(opt->step_size > 0) || prob->nx < 2 || prob->N < 1 || prob->n_obs < 0 ||
        prob->n_obs > NLOT_MAX_OBS || prob->n_verts < 0 || prob->n_verts > NLOT_MAX_VERTS ||
        !(opt->bounds[1][0] >= opt->bounds[0][0]) || !(opt->bounds[1][1] >= opt->bounds[0][1])) {
        set_error("nlot_rrt_init: invalid problem or options (max_iter >= 1, step_size > 0, bounds min <= max)");
        return NLOT_ERR_INVALID;
    }
    for (int i = 0; i < prob->n_obs; ++i) {
        const NlotObstacle& q = prob->obs[i];
        if ((q.type == NLOT_OBS_POLYGON || q.type == NLOT_OBS_TRAPEZOID) && (q.v0 < 0 || q.nv < 2 || q.v0 + q.nv > prob->n_verts)) {
            set_error("nlot_rrt_init: polygon vertex range outside verts[0, n_verts)");
            return NLOT_ERR_INVALID;
        }
    }
    if (!workspace || workspace_bytes < nlot_rrt_workspace_size(opt, B)) {
        set_error("nlot_rrt_init: workspace smaller than nlot_rrt_workspace_size");
        return NLOT_ERR_WORKSPACE;
    }
    // footprint inflation (trajectory_initialization.py:108-113): for a RectangleGeometry the largest |min
    // coordinate| over the body points (as written: np.min of each point, not its norm) + margin; else 0
    double infl = 0.0;
    if (prob->shape == NLOT_SHAPE_POLYGON && prob->n_body == 4) {
        for (int i = 0; i < prob->n_body; ++i) infl = fmax(infl, fabs(fmin(prob->body[i][0], prob->body[i][1])));
        infl += opt->margin;
    }
    hipStream_t st = (hipStream_t)stream;
    NlotProblem* dP = (NlotProblem*)workspace;
    NLOT_HIP_CHECK(hipMemcpyAsync(dP, prob, sizeof(NlotProblem), hipMemcpyHostToDevice, st));
    hipLaunchKernelGGL(k_rrt, dim3((unsigned)B), dim3(64), 0, st, dP, *opt, x0, xg, X_init, ok,
                       (double*)((char*)workspace + kRrtHdr), B, infl);
    NLOT_HIP_CHECK(hipGetLastError());
    return NLOT_OK;
}
