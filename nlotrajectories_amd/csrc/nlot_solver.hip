// Batched trajectory optimisation on the GPU: B independent instances of the NLP of
// RunBenchmark.run (/root/reference/src/nlotrajectories/core/runner.py:44-108), solved with a
// restatement of IPOPT's primal-dual filter line-search algorithm (runner.py:113-133)
// whose Newton systems are solved by a stage-wise Riccati recursion.
//
// MI355X mapping: ONE WAVEFRONT PER INSTANCE, except the Riccati solve.
//   * k_iter_a / k_iter_b / k_accept: lanes over knots for everything that is per knot (SDF chain rule +
//     soft-min, dynamics and their derivatives, condensed stage matrices, residuals, optimality
//     measures); scalars of the algorithm come from wave reductions (shuffles), broadcast from lane 0 so
//     every lane takes the same branch;
//   * k_ric: 16 lanes per instance (one per column of the extended stage matrix), 4 instances per
//     wavefront; the recursion is sequential in the knot index, stage inputs arrive by global->LDS DMA;
//   * per-instance arrays are instance-major (a wave touches one contiguous block);
//   * the learned-SDF corner points of all instances that need them in a step are compacted
//     (rank-major) into one list and evaluated by the MFMA kernel (nlot_mlp.hip) in a single launch;
//     the kernel that moves an instance into a phase appends the points that phase needs;
//   * the host launches only the still-active instances (active list rebuilt every step).
//
// Per-instance phase machine (one global step = one launch of each kernel):
//   INIT -> [corners (k_points), MLP full, k_iter_a: slack push, least-squares multipliers (k_ric), then
//            the EVAL work]
//   EVAL -> [MLP full, k_iter_a: evaluate, converge?, mu update, stage matrices; k_ric: inertia-corrected
//            Newton step; k_iter_b: sigma choice, step bounds, first trial corners]          -> LS
//   LS   -> [MLP value, k_accept: filter test at the candidates; accept -> EVAL (new corners),
//            reject -> next halvings (next step), alpha < alpha_min -> DONE(LS_FAILED)]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <type_traits>
#include <cmath>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <vector>

#include "nlot_device.h"
#include "nlot_internal.h"

namespace nlot {

// PH_SOFT1 / PH_SOFT2: IPOPT's soft restoration step (BacktrackingLineSearch::TrySoftRestoStep) — the damped
// step's filter test on a value launch, then (not filter-acceptable) the primal-dual error at the tentatively
// accepted point on a full launch.  PH_RINIT: first step of a feasibility restoration phase (its point's full
// evaluation, then MinC_1NrmRestorationPhase's initialisation); while SC_RESTO = 1 the EVAL / LS phases belong to
// the restoration problem (k_resto_a / k_ric<DYN, true> / k_resto_b / k_resto_ls).
enum Phase { PH_INIT = 0, PH_EVAL = 1, PH_LS = 2, PH_DONE = 3, PH_SOC = 4, PH_SOFT1 = 5, PH_SOFT2 = 6, PH_RINIT = 7 };
// k_iter_a's passes (run() launches SOC on the side stream at the start of a step and EVAL after the full MLP launch)
enum IterPass { PASS_ALL = 0, PASS_INIT = 1, PASS_SOC = 2, PASS_EVAL = 3 };

// Minimum waves per SIMD the per-instance kernels are compiled for (register budget 512 / w per lane),
// and the depth of k_ric's stage ring (its LDS per wavefront sets k_ric's occupancy).  These kernels wait
// on memory most of their cycles (SQ_WAIT_ANY 56-73 %), so residency is speed.
// Defaults: the best of each knob measured alone at B = 65536 (profiles/r01/variants_v14.log).
#ifndef NLOT_WPE_A
#define NLOT_WPE_A 2
#endif
#ifndef NLOT_WPE_B
#define NLOT_WPE_B 2
#endif
#ifndef NLOT_WPE_ACC
#define NLOT_WPE_ACC 3
#endif
#ifndef NLOT_WPE_RIC
#define NLOT_WPE_RIC 2  // k_ric at 2 waves/SIMD: 12 % less k_ric time at the metric config than 1 (r02i A/B)
#endif
#ifndef NLOT_WPE_SOC
#define NLOT_WPE_SOC 2  // the correction (substitution) instantiation of k_ric
#endif
#ifndef NLOT_RIC_RING
#define NLOT_RIC_RING 2
#endif
// the restoration phases run few wavefronts (the instances in restoration), so their latency, not residency, counts
#ifndef NLOT_WPE_RA
#define NLOT_WPE_RA NLOT_WPE_A  // k_resto_a
#endif
#ifndef NLOT_WPE_RLS
#define NLOT_WPE_RLS NLOT_WPE_ACC  // k_resto_ls
#endif
#ifndef NLOT_WPE_RRIC
#define NLOT_WPE_RRIC NLOT_WPE_RIC  // k_ric<DYN, true>
#endif
#if !defined(NLOT_RIC_FENCED) && !defined(NLOT_RIC_INORDER)
#define NLOT_RIC_INORDER
#endif
enum Scal {
    SC_MU, SC_TAU, SC_DWLAST, SC_THMAX, SC_THMIN, SC_ALPHA, SC_AMAX, SC_AMIN, SC_AZ, SC_THETA, SC_PHI, SC_GD,
    SC_DW, SC_DC, SC_STATUS, SC_ITERS, SC_PHASE, SC_TRIALS, SC_NFILT, SC_RANK, SC_E0, SC_NCAND,
    SC_FREE, SC_MUMAX, SC_NAF,  // adaptive mu: free-mode flag, mu_max, progress-filter entries
    // hand-off k_iter_a -> k_ric -> k_iter_b: Newton-solve state (0 idle, 1 pending, 2 solved, 3 LSQ
    // failed), its barrier parameters and right-hand-side count, and the optimality scalars the
    // quality-function oracle needs
    SC_RIC, SC_RMU0, SC_RMU1, SC_RNR, SC_USEQF, SC_AVG, SC_DSQ, SC_PSQ, SC_NZC,
    SC_ACCSLOT,  // trial-list slot of the accepted line-search candidate (forward reuse), -1 if none
    // IPOPT's globalisation safeguards: second-order correction (count in progress, the
    // original trial's alpha and alpha_z, theta of the last corrected trial), k_ric's fixed delta_w (-1: the
    // inertia-correction loop), watchdog (active, shortened-step counter, trials, reference values and the
    // saved line-search scalars), tiny step (this iteration, the previous one), max primal infeasibility
    SC_SOCK, SC_SOCA, SC_SOCAZ, SC_SOCTH, SC_RICFIX,
    SC_WD, SC_WDSHORT, SC_WDTRIAL, SC_WDTH, SC_WDPH, SC_WDGD, SC_WDAT, SC_WDAZ, SC_WDAMIN, SC_WDMU, SC_WDTAU,
    SC_TINY, SC_TINYLAST, SC_PRIMAL,
    // IPOPT's filter reset heuristic: last rejection of this line search was by the filter, successive such
    // iterations, resets done
    SC_LASTREJF, SC_NFREJ, SC_NFRES,
    // soft restoration: active, iterations, primal-dual error at the current point and the mu it was taken at
    SC_INSOFT, SC_SOFTCNT, SC_PDC, SC_MUPD,
    // feasibility restoration (MinC_1Nrm): active, first iteration, the original problem's mu / tau / last
    // delta_w, theta_R and phi_R at the restoration's start, rho, zeta, the restoration's theta_max / theta_min
    // and filter entries, restoration phases started (statistics)
    SC_RESTO, SC_RFIRST, SC_RMUO, SC_RTAUO, SC_RDWO, SC_THR, SC_PHR, SC_RHO, SC_ZETA, SC_RTHMAX, SC_RTHMIN,
    SC_RNFILT, SC_NRESTO,
    // inertia correction carried over to the next global step (k_ric's attempt cap): the next delta_w to try (-1:
    // none pending) and the delta_w already added into hg
    SC_RETRY, SC_DWHG,
    SC_COUNT
};
// Filters (line search, adaptive-mu progress, restoration): IPOPT's Filter is an unbounded list from which
// dominated entries are removed.  At most one entry enters per iteration (the line-search filter can grow to
// 2 max_iter + O(1) in principle); the largest size measured over the round-4 metric bench was 613 (bench.py
// config.filters), so 1024 entries per filter are unbounded in effect there.  An overflow forgets the oldest entry;
// it is counted (NlotSolveStats.filter_forgotten, the restoration filter included) and reported by bench.py.
constexpr int FILT_MAX = 1024;
// ints per step-parity counter set (workspace counters: 2 sets): [0..8) the phase machine's counts (Ws::cnt), [8..11)
// diagnostics of the factorising Newton solves (attempts summed, their maximum, solves needing more than one), [11]
// the largest filter size reached and [12] filter entries forgotten at capacity (diagnostics), [15] the most
// factorisations one restoration Newton solve took (diagnostics), [13]
// where k_admit's slots start in the active list.  After the two sets: the free-slot count and k_admit's error flag.
constexpr int CSET = 16;
constexpr int NSPEC = 8;  // step lengths evaluated per line-search round after a first rejection
constexpr int MMAX = 4;  // inequalities per knot (rectangle without slack)

struct Dims {
    int N, nx, nu, ns, M, nc, nb, nv, sd;  // nv = nu + ns (stage k < N)
    int tidx[8];
    int ppk;  // SDF points per knot (corners, or 1 for a dot)
    // general bounds (NlotSolverOptions.general_bounds): the control bounds and slack >= 0 as constraint rows, the way
    // CasADi's Opti hands them to IPOPT (runner.py:67-69,101-103).  ngb = bound rows N nu + ns (N + 1) (the workspace
    // always holds their arrays: the workspace size does not depend on the options); gcb = 1 selects the form
    int ngb, gcb;
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
    d.ngb = p.N * p.nu + d.ns * (p.N + 1);
    d.gcb = 0;  // run() sets it from the options
    return d;
}

// Riccati storage per knot (one Newton solve with up to two right-hand sides):
//   slot (LDS when it fits, else HBM): [A B 0] (nx x nz) | c | M (2x2) | K (nv x nx) | k (2 x nv) | Kn (nv x nc)
//     — everything the sequential forward sweep reads;
//   hg (HBM): H (nz x nz) | g (2 x nz) — built in parallel over knots, read once by the backward sweep
//     (prefetched one stage ahead);
//   vf (HBM): P (nx x nx) | p (2 x nx) | Gamma (nx x nc) — written by the backward sweep, read by the
//     parallel multiplier pass.  (nz = nx + nu + 1, nv = nu + 1, nc = nx.)
//   Layouts (row-major, ncol = nx + 2 + nc gain columns K | k_0 | k_1 | Kn):
//     slot = [A B 0 | c | pad] (nx x ab_row) | M | GN (ncol x nv);  hg = [H | g_0 g_1] (nz x (nz+2)) (the
//     Riccati lane of column j reads row j, H being symmetric, or a g column top to bottom);
//     vf = [P | p_0 p_1 | Gamma] (nx x ncol).
__host__ __device__ constexpr int ab_row(int nx, int nu) { return (nx + nu + 2 + 1) & ~1; }  // [A B 0 | c], even
__host__ __device__ constexpr int slot_len(int nx, int nu) {
    return nx * ab_row(nx, nu) + 4 + (nx + 2 + nx) * (nu + 1);
}
__host__ __device__ constexpr int hg_len(int nx, int nu) { return (nx + nu + 1) * (nx + nu + 3); }
__host__ __device__ constexpr int vf_len(int nx, int nu) { return nx * (nx + 2 + nx); }
// quality-function oracle step buffers (affine / centering): dX dU dS yi yk yt | dT dzl dzu dzs dvt | dsb (the
// bound rows' slack step, general bounds)
__host__ __device__ constexpr int qf_len(int N, int nx, int nu, int M, int ngb) {
    return (N + 1) * nx + N * nu + (N + 1) + nx + N * nx + 8 + (N + 1) * M + 2 * N * nu + (N + 1) + (N + 1) * M + ngb;
}

// an iterate (X U S T yi yk yt yd zl zu zs vt sb yb) or a step (dX dU dS dT yi_n yk_n yt_n yd_n dzl dzu dzs dvt dsb
// yb_n): the save areas of the second-order correction and the watchdog
__host__ __device__ constexpr int it_len(int N, int nx, int nu, int M, int ngb) {
    return (N + 1) * nx + 3 * N * nu + 2 * (N + 1) + 3 * (N + 1) * M + nx + N * nx + 8 + 2 * ngb;
}

// restoration rows (oracle Sol::rp ...): [initial state nx][dynamics N nx][terminal nc][inequalities (N+1) M]
// [bound rows ngb (general bounds)], allocated with the terminal block padded to 8
__host__ __device__ constexpr int ne_len(int N, int nx, int M, int ngb) { return nx + N * nx + 8 + (N + 1) * M + ngb; }

// a stored pivoted LDL^T factor of an n x n block (ldl_factor's in-place form, then the permutation): the Q_vv
// factor of every stage and the terminal block's, kept by each Newton solve for the second-order corrections
__host__ __device__ constexpr int ldl_len(int n) { return n * n + n; }

// instance-major arrays: (name, per-instance length)
#define NLOT_WS_ARRAYS(X_)                                                                             \
    X_(X, (N + 1) * nx) X_(U, N * nu) X_(S, N + 1) X_(T, (N + 1) * M) X_(yi, nx) X_(yk, N * nx) X_(yt, 8) \
    X_(yd, (N + 1) * M) X_(zl, N * nu) X_(zu, N * nu) X_(zs, N + 1) X_(vt, (N + 1) * M)                \
    X_(dv, (N + 1) * M) X_(Jd, (N + 1) * M * 3) X_(Hd, (N + 1) * 6) X_(rci, nx) X_(rcd, N * nx)         \
    X_(rct, 8) X_(rcq, (N + 1) * M) X_(dX, (N + 1) * nx) X_(dU, N * nu) X_(dS, N + 1)                  \
    X_(dT, (N + 1) * M) X_(yi_n, nx) X_(yk_n, N * nx) X_(yt_n, 8) X_(yd_n, (N + 1) * M)                \
    X_(dzl, N * nu) X_(dzu, N * nu) X_(dzs, N + 1) X_(dvt, (N + 1) * M) X_(sc, SC_COUNT)               \
    X_(filt, 2 * FILT_MAX) X_(afilt, 2 * FILT_MAX) X_(qa, qf_len(N, nx, nu, M, ngb)) X_(qc, qf_len(N, nx, nu, M, ngb)) \
    X_(stg, (N + 1) * slot_len(nx, nu)) X_(hg, (N + 1) * hg_len(nx, nu)) X_(vf, (N + 1) * vf_len(nx, nu))   \
    X_(dX2, (N + 1) * nx) X_(dU2, N * nu) X_(dS2, N + 1) X_(yi2, nx) X_(yk2, N * nx) X_(yt2, 8)         \
    X_(sts, it_len(N, nx, nu, M, ngb)) X_(rcs, nx + N * nx + 8 + (N + 1) * M + ngb)                     \
    X_(wdi, it_len(N, nx, nu, M, ngb)) X_(wdd, it_len(N, nx, nu, M, ngb))                               \
    X_(rp, ne_len(N, nx, M, ngb)) X_(rn, ne_len(N, nx, M, ngb)) X_(rzp, ne_len(N, nx, M, ngb))           \
    X_(rzn, ne_len(N, nx, M, ngb)) X_(rdp, ne_len(N, nx, M, ngb)) X_(rdn, ne_len(N, nx, M, ngb))         \
    X_(rdzp, ne_len(N, nx, M, ngb)) X_(rdzn, ne_len(N, nx, M, ngb)) X_(dsoft, ne_len(N, nx, M, ngb))     \
    X_(esoft, ne_len(N, nx, M, ngb)) X_(rfilt, 2 * FILT_MAX)                                            \
    X_(qfac, (N + 1) * ldl_len(nu + 1)) X_(tfac, ldl_len(nx)) X_(x0s, nx) X_(xgs, nx) X_(phi, N * nx * (nx + 2)) \
    X_(sb, ngb) X_(yb, ngb) X_(rcb, ngb) X_(dsb, ngb) X_(yb_n, ngb)

struct Ws {
#define NLOT_DECL(name, cnt) \
    double* name;            \
    int L_##name;
    NLOT_WS_ARRAYS(NLOT_DECL)
#undef NLOT_DECL
    float* pts;  // compacted corner list, rank-major [rank][P][2]
    float* mo;   // MLP outputs [6][cap * P] (rank-major within a plane)
    // trial lists by global-step parity q: the full launch of step s + 1 reuses step s's accepted
    // candidate while k_accept of step s already emits the candidates of step s + 1
    float* tpts[2];      // trial corner list [slot][P][2] (slot = rank + candidate), cap * NSPEC slots
    float* tval[2];      // its values [slot][P]
    uint32_t* tmask[2];  // its hidden-layer ReLU patterns [4][slot][P]
    int* tsrc;           // per evaluation rank: trial slot whose forward the full launch may reuse, or -1
    int* cnt;  // counters of step parity q at cnt + CSET q: [0] evaluation ranks, [1] trial slots, [2] next active
               // count, [3] full-launch points whose forward was reused, [4] Newton solves, [5] restoration list count,
               // [6] second-order corrections, [7] restoration Newton solves
    int* act[2]; // active instance lists (ping-pong)
    int* actr[2]; // the instances of act in a restoration phase (count: counter [5] of the step's set)
    int* ricl;    // this step's factorising Newton solves (count: counter [4]), compacted by k_iter_a for k_ric
    int* socl;    // this step's second-order corrections (count: counter [6])
    // Slots: every array above is indexed by slot (cap slots); sinst[slot] is the instance a slot holds.  An instance
    // leaving the active list (k_accept) writes its outputs (o*, instance-indexed, caller-owned) and frees its slot
    // (freel, count at cnt[2 CSET]); k_admit gives free slots to the next instances, k_init_state starts them.
    int* sinst;
    int* freel;
    double *oX, *oU, *oS, *ocost;
    int32_t *ostat, *oiters;
    int64_t cap;
    int ppk;
    int prio;  // NLOT_SETPRIO: the side-stream chains (restoration solves, corrections) raise their waves' issue priority
};

static size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

// doubles of all instance-major arrays for B instances, each array rounded up to 256 bytes
static size_t ws_doubles(const Dims& d, int64_t B) {
    const int N = d.N, nx = d.nx, nu = d.nu, M = d.M, ngb = d.ngb;
    size_t n = 0;
#define NLOT_CNT(name, cnt) n += ((size_t)(cnt) * (size_t)B + 31) & ~(size_t)31;
    NLOT_WS_ARRAYS(NLOT_CNT)
#undef NLOT_CNT
    return n;
}

constexpr size_t kHdr = 32768;  // device copies of NlotProblem, Dims, Ws (kernels read them through pointers:
                                // a by-value struct argument indexed at run time is copied to scratch)
constexpr size_t kHdrProblem = 0, kHdrDims = 24576, kHdrWs = 28672;  // NlotProblem ~14.5 KB (vertex pool)

static size_t ws_bytes(const Dims& d, int64_t B, bool mlp) {
    size_t b = kHdr + align256(ws_doubles(d, B) * sizeof(double));
    if (mlp) {  // corner list and outputs sized for NSPEC line-search candidates per instance
        const size_t P = (size_t)d.ppk * (d.N + 1);
        b += align256(P * (size_t)B * NSPEC * 2 * sizeof(float));
        b += align256(6 * P * (size_t)B * NSPEC * sizeof(float));
        b += 2 * align256(P * (size_t)B * NSPEC * 2 * sizeof(float));     // tpts, per step parity
        b += 2 * align256(P * (size_t)B * NSPEC * sizeof(float));         // tval
        b += 2 * align256(4 * P * (size_t)B * NSPEC * sizeof(uint32_t));  // tmask
        b += align256((size_t)B * sizeof(int));                    // tsrc
    }
    b += align256(2 * (size_t)B * sizeof(int));
    b += align256(2 * (size_t)B * sizeof(int));  // restoration lists
    b += 2 * align256((size_t)B * sizeof(int));  // Newton-solve and correction lists
    b += 2 * align256((size_t)B * sizeof(int));  // slot -> instance, free slots
    b += 256;  // counters (2 sets of CSET ints)
    return b;
}

static Ws carve(const Dims& d, int64_t B, bool mlp, void* base) {
    Ws w{};
    w.cap = B;
    w.ppk = d.ppk;
    const int N = d.N, nx = d.nx, nu = d.nu, M = d.M, ngb = d.ngb;
    base = (char*)base + kHdr;
    double* q = (double*)base;
#define NLOT_TAKE(name, cnt)          \
    w.name = q;                       \
    w.L_##name = (int)(cnt);          \
    q += ((size_t)(cnt) * (size_t)B + 31) & ~(size_t)31;
    NLOT_WS_ARRAYS(NLOT_TAKE)
#undef NLOT_TAKE
    char* c = (char*)base + align256(ws_doubles(d, B) * sizeof(double));
    if (mlp) {
        const size_t P = (size_t)d.ppk * (N + 1);
        w.pts = (float*)c;
        c += align256(P * (size_t)B * NSPEC * 2 * sizeof(float));
        w.mo = (float*)c;
        c += align256(6 * P * (size_t)B * NSPEC * sizeof(float));
        for (int q = 0; q < 2; ++q) {
            w.tpts[q] = (float*)c;
            c += align256(P * (size_t)B * NSPEC * 2 * sizeof(float));
            w.tval[q] = (float*)c;
            c += align256(P * (size_t)B * NSPEC * sizeof(float));
            w.tmask[q] = (uint32_t*)c;
            c += align256(4 * P * (size_t)B * NSPEC * sizeof(uint32_t));
        }
        w.tsrc = (int*)c;
        c += align256((size_t)B * sizeof(int));
    }
    w.act[0] = (int*)c;
    w.act[1] = (int*)c + B;
    c += align256(2 * (size_t)B * sizeof(int));
    w.actr[0] = (int*)c;
    w.actr[1] = (int*)c + B;
    c += align256(2 * (size_t)B * sizeof(int));
    w.ricl = (int*)c;
    c += align256((size_t)B * sizeof(int));
    w.socl = (int*)c;
    c += align256((size_t)B * sizeof(int));
    w.sinst = (int*)c;
    c += align256((size_t)B * sizeof(int));
    w.freel = (int*)c;
    c += align256((size_t)B * sizeof(int));
    w.cnt = (int*)c;
    return w;
}

// element i of instance b's array (instance-major)
#define AT(arr, i) (ws.arr[(size_t)b * ws.L_##arr + (i)])
#define SC(i) AT(sc, i)
// General bounds (Dims::gcb; oracle Sol::gcb): CasADi's Opti passes opti.bounded(umin, U, umax) and slack >= 0
// (runner.py:67-69,101-103) to IPOPT as constraint rows d(x) = U_ki, d(x) = S_k, i.e. rows d(x) - sb = 0 whose slack
// sb carries the bounds, with U and S free.  Bound row q: control q = k nu + i, then slack rows N nu + k.  The bounded
// quantity of a row is sb (general bounds) or the variable itself (variable bounds); its bound multipliers live in
// zl / zu (controls) and zs (slacks) in both forms.  BVU / BVS: the bounded value, BDU / BDS: its step.
#define BVU(e) (dm.gcb ? AT(sb, (e)) : AT(U, (e)))
#define BVS(k) (dm.gcb ? AT(sb, dm.N * dm.nu + (k)) : AT(S, (k)))
#define BDU(e) (dm.gcb ? AT(dsb, (e)) : AT(dU, (e)))
#define BDS(k) (dm.gcb ? AT(dsb, dm.N * dm.nu + (k)) : AT(dS, (k)))

// save (to buf) or load (from buf) an iterate, a step, or the residual rows, lane-strided
#define NLOT_ITER_ARRAYS(F_) F_(X) F_(U) F_(S) F_(T) F_(yi) F_(yk) F_(yt) F_(yd) F_(zl) F_(zu) F_(zs) F_(vt) F_(sb) F_(yb)
#define NLOT_STEP_ARRAYS(F_) \
    F_(dX) F_(dU) F_(dS) F_(dT) F_(yi_n) F_(yk_n) F_(yt_n) F_(yd_n) F_(dzl) F_(dzu) F_(dzs) F_(dvt) F_(dsb) F_(yb_n)
#define NLOT_RES_ARRAYS(F_) F_(rci) F_(rcd) F_(rct) F_(rcq) F_(rcb)
#define NLOT_IO(name)                                                              \
    {                                                                              \
        double* a_ = &AT(name, 0);                                                 \
        const int n_ = ws.L_##name;                                                \
        for (int i_ = lane; i_ < n_; i_ += 64) {                                   \
            if (save) buf[off + i_] = a_[i_];                                      \
            else a_[i_] = buf[off + i_];                                           \
        }                                                                          \
        off += n_;                                                                 \
    }
// Host grid bounds ("lists and their grid bounds").  The phase kernels' grids are the host's last known
// active count and the Newton / correction solves' grids that count over the group size: upper bounds of the device's
// counts (the active set only shrinks between admissions, and a solve list is a subset of it).  Should a device count
// ever exceed its grid, the instances past it would skip their step silently; block 0 checks, sets the error flag
// cnt[2 CSET + 1] to `code` (GRID_*), and the host fails the call at its next synchronisation.  The restoration kernels
// do not need it: they stride over their exact list count (the host's bound for them is a heuristic).
enum { GRID_ADMIT = 1, GRID_ACTIVE = 2, GRID_SOLVE = 3 };
__device__ __forceinline__ void grid_guard(const Ws& ws, int count, int per_block, int code) {
    if (blockIdx.x == 0 && threadIdx.x == 0 && count > (int)gridDim.x * per_block) ws.cnt[2 * CSET + 1] = code;
}

// the host's message for the error flag cnt[2 CSET + 1] (grid_guard codes)
static const char* grid_error(int code) {
    switch (code) {
    case GRID_ADMIT: return "nlot_solve_batch: slot bookkeeping mismatch (admission found fewer free slots than expected)";
    case GRID_ACTIVE: return "nlot_solve_batch: an active list outgrew its launch grid (host bound below the device count)";
    case GRID_SOLVE: return "nlot_solve_batch: a solve list outgrew its launch grid (host bound below the device count)";
    default: return "nlot_solve_batch: unknown device error flag";
    }
}

__device__ inline void iter_io(const Ws& ws, int64_t b, int lane, double* buf, bool save) {
    int off = 0;
    NLOT_ITER_ARRAYS(NLOT_IO)
}
__device__ inline void step_io(const Ws& ws, int64_t b, int lane, double* buf, bool save) {
    int off = 0;
    NLOT_STEP_ARRAYS(NLOT_IO)
}
__device__ inline void res_io(const Ws& ws, int64_t b, int lane, double* buf, bool save) {
    int off = 0;
    NLOT_RES_ARRAYS(NLOT_IO)
}
#undef NLOT_IO

// lane-strided update of n workspace elements in chunks of CH elements per lane: a chunk's NV loads per element are
// all issued before its stores (the compiler may not move a load above a store into the same workspace), so an array
// costs one memory round trip per chunk instead of one per 64 elements; ld(i, v) loads, st(i, v) computes and stores
template <int CH, int NV, class Ld, class St>
__device__ __forceinline__ void chunked_update(int n, int lane, Ld&& ld, St&& st) {
    for (int i0 = lane; i0 < n; i0 += 64 * CH) {
        double v[CH][NV];
#pragma unroll
        for (int r = 0; r < CH; ++r)
            if (i0 + 64 * r < n) ld(i0 + 64 * r, v[r]);
#pragma unroll
        for (int r = 0; r < CH; ++r)
            if (i0 + 64 * r < n) st(i0 + 64 * r, v[r]);
    }
}

// A lane-strided pass whose first chunk is loaded ahead (load), then consumed exactly as chunked_update would
// (run: the same elements in the same order, later chunks loaded as they come): several reductions' loads issued
// together cost one memory round trip instead of one each, with the arithmetic unchanged
template <int CH, int NV>
struct Pre {
    double v[CH][NV];
    template <class Ld>
    __device__ __forceinline__ void load(int n, int lane, Ld&& ld) {
#pragma unroll
        for (int r = 0; r < CH; ++r)
            if (lane + 64 * r < n) ld(lane + 64 * r, v[r]);
    }
    template <class Ld, class St>
    __device__ __forceinline__ void run(int n, int lane, Ld&& ld, St&& st) {
#pragma unroll
        for (int r = 0; r < CH; ++r)
            if (lane + 64 * r < n) st(lane + 64 * r, v[r]);
        if (n > 64 * CH) chunked_update<4, NV>(n, lane + 64 * CH, ld, st);
    }
};

// ---- wave-level helpers (64 lanes; results broadcast from lane 0 so every lane branches alike) ----
__device__ inline double wsum(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    return __shfl(v, 0);
}
__device__ inline double wmax(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmax(v, __shfl_xor(v, o));
    return __shfl(v, 0);
}
__device__ inline double wmin(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmin(v, __shfl_xor(v, o));
    return __shfl(v, 0);
}
__device__ inline void wsync() { __syncthreads(); }  // one-wave workgroups: barrier + LDS/global fence
// value of v in lane l (compile-time-uniform l) broadcast to the wave through two v_readlane_b32
__device__ __forceinline__ double bcast_lane(double v, int l) {
    const long long bits = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_readlane((int)bits, l);
    const int hi = __builtin_amdgcn_readlane((int)(bits >> 32), l);
    return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}
// LDS-only workgroup sync (s_waitcnt lgkmcnt(0) + s_barrier): outstanding global stores are not waited
// for.  Used inside the Riccati recursion when its slots live in LDS; the global fallback needs wsync.
template <bool LDS>
__device__ __forceinline__ void xsync() {
    if constexpr (LDS) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
    } else {
        __syncthreads();
    }
}

// ---------------------------------------------------------------------------------------------
// per-corner SDF: learned (MLP output of this step's compacted list) or analytic
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ HD corner_sdf(const NlotProblem& p, const Ws& ws, int rank, int pidx, double cx, double cy,
                                         const float* tval = nullptr) {
    if (p.sdf_kind == NLOT_SDF_ANALYTIC) return sdf_scene(p, cx, cy, true);
    if (tval) {  // value launch of this step's trial list (slot = rank)
        HD h{};
        h.v = tval[(int64_t)rank * ws.ppk * (p.N + 1) + pidx];
        return h;
    }
    // MLP outputs of this step's compacted list, rank-major: quantity q of point pidx of the
    // instance with compaction rank r at mo[q * plane + r * P + pidx]
    const int64_t P = (int64_t)ws.ppk * (p.N + 1);
    const int64_t plane = P * ws.cap * NSPEC;
    const int64_t o = (int64_t)rank * P + pidx;
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
__device__ __forceinline__ void knot_eval(const NlotProblem& p, const Dims& dm, const Ws& ws, int rank, int k,
                                 const double* xk, double* d, double (*g)[3], const double* w, double* Hw,
                                 const float* tval = nullptr) {
    const double x = xk[0], y = xk[1];
    if (p.shape == NLOT_SHAPE_DOT) {
        HD f = corner_sdf(p, ws, rank, k, x, y, tval);
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
#pragma unroll
    for (int i = 0; i < MMAX; ++i) {
        if (i >= dm.nb) break;
        const double bx = p.body[i][0], by = p.body[i][1];
        const double cx = x + cs * bx - sn * by, cy = y + sn * bx + cs * by;  // geometry.py:78-83
        const double ex = -(cy - y), ey = cx - x;                            // d c / d theta
        HD f = corner_sdf(p, ws, rank, k * dm.nb + i, cx, cy, tval);
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
#pragma unroll
        for (int i = 0; i < MMAX; ++i) {
            if (i >= dm.nb) break;
            e[i] = exp(-al * phi[i]);
            sum += e[i];
        }
        d[0] = -log(sum) / al;
        double gd[3] = {0, 0, 0};
#pragma unroll
        for (int i = 0; i < MMAX; ++i)
            if (i < dm.nb)
#pragma unroll
                for (int a = 0; a < 3; ++a) gd[a] += (e[i] / sum) * gp[i][a];
        if (g)
            for (int a = 0; a < 3; ++a) g[0][a] = gd[a];
        if (Hw) {
            double H[6] = {0, 0, 0, 0, 0, 0};
            const int ia[6] = {0, 0, 0, 1, 1, 2}, ib[6] = {0, 1, 2, 1, 2, 2};
#pragma unroll
            for (int i = 0; i < MMAX; ++i) {
                if (i >= dm.nb) break;
                const double wi = e[i] / sum;
#pragma unroll
                for (int q = 0; q < 6; ++q) H[q] += wi * (Hp[i][q] - al * gp[i][ia[q]] * gp[i][ib[q]]);
            }
            for (int q = 0; q < 6; ++q) Hw[q] = w[0] * (H[q] + al * gd[ia[q]] * gd[ib[q]]);
        }
    } else {
#pragma unroll
        for (int i = 0; i < MMAX; ++i) {
            if (i >= dm.nb) break;
            d[i] = phi[i];
            if (g)
#pragma unroll
                for (int a = 0; a < 3; ++a) g[i][a] = gp[i][a];
        }
        if (Hw) {
#pragma unroll
            for (int q = 0; q < 6; ++q) Hw[q] = 0;
#pragma unroll
            for (int i = 0; i < MMAX; ++i)
                if (i < dm.nb)
#pragma unroll
                    for (int q = 0; q < 6; ++q) Hw[q] += w[i] * Hp[i][q];
        }
    }
}

// ---------------------------------------------------------------------------------------------
// Stage-wise Newton system and its Riccati solve
// ---------------------------------------------------------------------------------------------
enum { MODE_NEWTON = 0, MODE_LSQ = 1 };

#ifdef NLOT_PHASE_PROF
#define PROF_T(v) const long long v = wall_clock64()
#define PROF_ACC(acc, v0) acc += wall_clock64() - v0
#else
#define PROF_T(v)
#define PROF_ACC(acc, v0)
#endif

template <int DYN>
struct Solver {
    using D = Dyn<DYN>;
    static constexpr int NX = D::NX, NU = D::NU, NV = NU + 1, NZ = NX + NV, NC = NX;

    // Condensed stage matrix H (nz x nz) and gradient g (nz) of stage k, written to o[0, NZ*NZ) and
    // o[NZ*NZ, NZ*NZ+NZ).  H is accumulated in its structured blocks (pose 3x3, pose-slack, slack,
    // control diagonal, dynamics curvature) and emitted dense once, so it never occupies 64 doubles
    // of registers.
    // Two right-hand sides: g_r = g(mu_r) for r < nr, written as o = [H | g_0 g_1] (NZ x (NZ+2)); g is
    // affine in mu, accumulated as base + mu * coefficient.
    // GONLY: only the g columns are written (a second-order correction: H is the iteration's, already factorised)
    template <bool GONLY = false>
    __device__ __forceinline__ static void stage(const NlotProblem& p, const Dims& dm, const Ws& ws, int b, int k, int mode,
                                                 double dw, double mu0, double mu1, int nr, double* o) {
        const int N = dm.N, M = dm.M;
        const double kappa_d = 1e-5;
        const bool newton = mode == MODE_NEWTON;
        double Pp[3][3], ps[3], gp[NX], gu[NU], uu[NU], ss = 0, gs = 0;
        double gpm[3] = {0, 0, 0}, gum[NU], gsm = 0;  // d g / d mu
#pragma unroll
        for (int i = 0; i < 3; ++i) {
            ps[i] = 0;
#pragma unroll
            for (int j = 0; j < 3; ++j) Pp[i][j] = 0;
        }
#pragma unroll
        for (int i = 0; i < NX; ++i) gp[i] = 0;
#pragma unroll
        for (int i = 0; i < NU; ++i) gu[i] = uu[i] = gum[i] = 0;
        // objective gradient and (Newton) Hessian of the path-length terms
        for (int seg = k - 1; seg <= k; ++seg) {
            if (seg < 0 || seg >= N) continue;
            const double dx = AT(X, (seg + 1) * NX) - AT(X, seg * NX);
            const double dy = AT(X, (seg + 1) * NX + 1) - AT(X, seg * NX + 1);
            const double r2 = dx * dx + dy * dy + p.path_eps, r = sqrt(r2), r3 = r2 * r;
            const double sgn = seg == k ? -1.0 : 1.0;
            gp[0] += sgn * dx / r;
            gp[1] += sgn * dy / r;
            if (newton) {
                Pp[0][0] += (r2 - dx * dx) / r3;
                Pp[0][1] += -dx * dy / r3;
                Pp[1][0] += -dx * dy / r3;
                Pp[1][1] += (r2 - dy * dy) / r3;
            }
        }
        const double Sk = AT(S, k);
        if (p.use_slack) gs += 2.0 * p.slack_penalty * Sk;
        if (p.use_smooth && k < N - 1)
#pragma unroll
            for (int i = 0; i < NU; ++i) gu[i] += 2.0 * p.smooth_weight * AT(U, k * NU + i);
        double Hz[NX + NU][NX + NU];  // dynamics curvature: constant sparsity, folds to a few registers
#pragma unroll
        for (int i = 0; i < NX + NU; ++i)
#pragma unroll
            for (int j = 0; j < NX + NU; ++j) Hz[i][j] = 0;
        if (newton) {
            if (p.use_slack) ss += 2.0 * p.slack_penalty;
            if (p.use_smooth && k < N - 1)
#pragma unroll
                for (int i = 0; i < NU; ++i) uu[i] += 2.0 * p.smooth_weight;
            if (k < N) {  // dynamics c_k = x_{k+1} - F_k  =>  W -= sum_i y_i d2F_i
                double x[NX], u[NU], l[NX];
#pragma unroll
                for (int i = 0; i < NX; ++i) x[i] = AT(X, k * NX + i);
#pragma unroll
                for (int i = 0; i < NU; ++i) u[i] = AT(U, k * NU + i);
#pragma unroll
                for (int i = 0; i < NX; ++i) l[i] = AT(yk, k * NX + i);
                D::hess(x, u, l, p.dt, p.wheelbase, Hz);
            }
            // knot inequality curvature sum_j yd_j d2 d_j (pose block x, y, theta)
            {
                const int ia[6] = {0, 0, 0, 1, 1, 2}, ib[6] = {0, 1, 2, 1, 2, 2};
#pragma unroll
                for (int q = 0; q < 6; ++q) {
                    const double v = AT(Hd, k * 6 + q);
                    Pp[ia[q]][ib[q]] += v;
                    if (ia[q] != ib[q]) Pp[ib[q]][ia[q]] += v;
                }
            }
            // bound barriers: Sigma on the diagonal, the barrier gradient (affine in mu).  General bounds: the row
            // d(x) - sb = 0 with sb's barrier eliminated (oracle bound_row): D = Sigma + dw, rhs = D rcb + grad barrier
            if (k < N)
#pragma unroll
                for (int i = 0; i < NU; ++i) {
                    const double uv = BVU(k * NU + i), sl = uv - p.umin[i], su = p.umax[i] - uv;
                    const double sig = AT(zl, k * NU + i) / sl + AT(zu, k * NU + i) / su;
                    if (dm.gcb) {
                        uu[i] += sig + dw;
                        gu[i] += (sig + dw) * AT(rcb, k * NU + i);
                    } else {
                        uu[i] += sig;
                    }
                    gum[i] += -1.0 / sl + 1.0 / su;
                }
            if (dm.ns) {
                const double sv = BVS(k), sig = AT(zs, k) / sv;
                if (dm.gcb) {
                    ss += sig + dw;
                    gs += (sig + dw) * AT(rcb, N * NU + k);
                } else {
                    ss += sig;
                }
                gsm += -1.0 / sv + kappa_d;
            }
        } else {  // least squares: D = 1 on a bound row (general bounds), rhs -(z_L - z_U) either way
            if (k < N)
#pragma unroll
                for (int i = 0; i < NU; ++i) {
                    gu[i] += -AT(zl, k * NU + i) + AT(zu, k * NU + i);
                    if (dm.gcb) uu[i] += 1.0;
                }
            if (dm.ns) {
                gs += -AT(zs, k);
                if (dm.gcb) ss += 1.0;
            }
        }
        // eliminated inequality slacks t:  H += J' D J, g += J' rhs, J = (d d_j/d pose, 1 on the slack)
        for (int j = 0; j < M; ++j) {
            double J[3];
#pragma unroll
            for (int a = 0; a < 3; ++a) J[a] = AT(Jd, (k * M + j) * 3 + a);
            const double t = AT(T, k * M + j), v = AT(vt, k * M + j);
            double Dj, rhs, rhm = 0;
            if (newton) {
                Dj = v / t + dw;
                rhs = Dj * AT(rcq, k * M + j);
                rhm = -1.0 / t + kappa_d;
            } else {
                Dj = 1.0;
                rhs = -v;
            }
#pragma unroll
            for (int a = 0; a < 3; ++a) {
                gp[a] += J[a] * rhs;
                gpm[a] += J[a] * rhm;
#pragma unroll
                for (int c = 0; c < 3; ++c) Pp[a][c] += Dj * J[a] * J[c];
                if (dm.sd) ps[a] += Dj * J[a];
            }
            if (dm.sd) {
                ss += Dj;
                gs += rhs;
                gsm += rhm;
            }
        }
        // emit dense H, g; the slack column is NX + NU (k < N) or NX (k == N): compile-time per branch
        const double dg = newton ? dw : 1.0;
        auto emit = [&](auto has_u) {
            constexpr bool HU = decltype(has_u)::value;
            constexpr int is = HU ? NX + NU : NX;
            const bool hs = dm.ns != 0;
            const int nz = is + (hs ? 1 : 0);
#pragma unroll
            for (int i = 0; i < NZ; ++i) {
#pragma unroll
                for (int j = 0; j < NZ; ++j) {
                    double h = 0;
                    if (i < 3 && j < 3) h += Pp[i][j];
                    if (HU && i == j && i >= NX && i < NX + NU) h += uu[i - NX];
                    if (HU && i < NX + NU && j < NX + NU) h -= Hz[i][j];
                    if (hs) {
                        if (i == is && j == is) h += ss;
                        if (i == is && j < 3) h += ps[j];
                        if (j == is && i < 3) h += ps[i];
                    }
                    if (i == j && i < nz) h += dg;
                    if constexpr (!GONLY) o[i * (NZ + 2) + j] = h;
                }
                double gi = 0, gm = 0;
                if (i < NX) {
                    gi = gp[i];
                    if (i < 3) gm = gpm[i];
                } else if (HU && i < NX + NU) {
                    gi = gu[i - NX];
                    gm = gum[i - NX];
                }
                if (hs && i == is) {
                    gi = gs;
                    gm = gsm;
                }
                o[i * (NZ + 2) + NZ] = gi + mu0 * gm;
                o[i * (NZ + 2) + NZ + 1] = nr > 1 ? gi + mu1 * gm : 0.0;
            }
        };
        if (k < N) emit(std::true_type{});
        else emit(std::false_type{});
    }

    // path-length cross block M_k (positions of x_k vs x_{k+1}) = -G_k
    __device__ __forceinline__ static void cross(const NlotProblem& p, const Ws& ws, int b, int k, int mode, double (*Mk)[2]) {
        Mk[0][0] = Mk[0][1] = Mk[1][0] = Mk[1][1] = 0;
        if (mode != MODE_NEWTON) return;
        const double dx = AT(X, (k + 1) * NX) - AT(X, k * NX), dy = AT(X, (k + 1) * NX + 1) - AT(X, k * NX + 1);
        const double r2 = dx * dx + dy * dy + p.path_eps, r = sqrt(r2), r3 = r2 * r;
        Mk[0][0] = -(r2 - dx * dx) / r3;
        Mk[0][1] = Mk[1][0] = dx * dy / r3;
        Mk[1][1] = -(r2 - dy * dy) / r3;
    }

    // ---------------- stage layouts of the Riccati recursion (k_ric) ----------------
    //   slot: ABc = [A B 0 | c | pad] (NX x NAB) | M (2x2) | GN[c][v] (NCOL x NV: K^T | k_0 | k_1 | Kn^T)
    //   hg:   [H | g_0 g_1] (NZ x (NZ+2));  vf / VE: [P | p_0 p_1 | G] (NX x NCOL)
    //   QE:   [Q | q_0 q_1 | QN] (NZ x NQE);  W: [P AB | P c + p_0 | P c + p_1 | G] (NX x NQE)
    //   PE:   [Psi | psi_0 psi_1] (NC x (NC+2))
    static constexpr int NCOL = NX + 2 + NC, NQE = NZ + 2 + NC, NAB = ab_row(NX, NU);
    static constexpr int SLOT = slot_len(NX, NU), HG = hg_len(NX, NU), VF = vf_len(NX, NU);
    static constexpr int sAB = 0, sM = NX * NAB, sGN = sM + 4;
    static_assert(sGN + NCOL * NV == SLOT, "slot layout");
    static_assert(NZ * (NZ + 2) == HG && NX * NCOL == VF, "hg / vf layout");

    // gain column c <-> QE column
    __host__ __device__ static constexpr int qe_col(int c) { return c < NX ? c : NZ + (c - NX); }

    // Build every stage's matrices in parallel (lane = knot): [H | g] -> hg (HBM); [A B 0 | c], M -> slot.
    // GONLY: hg's g columns and the slot's c column only (second-order correction: A, B and M are the iteration's,
    // which the forward sweep leaves in place)
    template <bool LDS, bool GONLY = false>
    __device__ static void build_stages(const NlotProblem& p, const Dims& dm, const Ws& ws, int b, int lane, int mode,
                                        double dw, double mu0, double mu1, int nr, double* SL, int stride = 64) {
        const int N = dm.N;
        for (int k = lane; k <= N; k += stride) {
            double* o = SL + (size_t)k * SLOT;
            stage<GONLY>(p, dm, ws, b, k, mode, dw, mu0, mu1, nr, &AT(hg, k * HG));
            if constexpr (GONLY) {
#pragma unroll
                for (int i = 0; i < NX; ++i)
                    o[sAB + i * NAB + NZ] = (k < N && mode == MODE_NEWTON) ? -AT(rcd, k * NX + i) : 0.0;
                continue;
            }
            double A[NX][NX], Bu[NX][NU];
#pragma unroll
            for (int i = 0; i < NX; ++i) {
#pragma unroll
                for (int j = 0; j < NX; ++j) A[i][j] = 0;
#pragma unroll
                for (int j = 0; j < NU; ++j) Bu[i][j] = 0;
            }
            double Mk[2][2] = {{0, 0}, {0, 0}};
            if (k < N) {
                double x[NX], u[NU];
#pragma unroll
                for (int i = 0; i < NX; ++i) x[i] = AT(X, k * NX + i);
#pragma unroll
                for (int i = 0; i < NU; ++i) u[i] = AT(U, k * NU + i);
                D::jac(x, u, p.dt, p.wheelbase, A, Bu);
                cross(p, ws, b, k, mode, Mk);
            }
#pragma unroll
            for (int i = 0; i < NX; ++i) {
#pragma unroll
                for (int j = 0; j < NZ; ++j) o[sAB + i * NAB + j] = j < NX ? A[i][j] : (j < NX + NU ? Bu[i][j - NX] : 0.0);
                o[sAB + i * NAB + NZ] = (k < N && mode == MODE_NEWTON) ? -AT(rcd, k * NX + i) : 0.0;
#pragma unroll
                for (int j = NZ + 1; j < NAB; ++j) o[sAB + i * NAB + j] = 0.0;
            }
            o[sM + 0] = Mk[0][0];
            o[sM + 1] = Mk[0][1];
            o[sM + 2] = Mk[1][0];
            o[sM + 3] = Mk[1][1];
        }
        __syncthreads();  // hg is in HBM: full fence
    }

    // ---------------- the feasibility restoration problem (IPOPT MinC_1NrmRestorationPhase) ----------------
    //   min rho sum(p + n) + zeta/2 ||D_R (x - x_R)||^2  s.t.  c(x) - p + n = 0, p, n >= 0  (every equality row,
    //   d(x) - t included).  Newton system (oracle build(), resto branch): the objective's curvature is zeta D_R^2;
    //   on an inequality row t, p and n are eliminated (D = 1 / C, rhs = (r - E) / C); on an equality row p and n
    //   are eliminated into a soft equality J dz - D y = -r + e (dsoft, esoft), folded into the Riccati recursion
    //   by k_ric<DYN, true>.  x_R and the original bound multipliers are the iterate saved in wdi at the start.
    __device__ __forceinline__ static void stage_resto(const NlotProblem& p, const Dims& dm, const Ws& ws, int b, int k,
                                                       double dw, double mu, double* o) {
        const int N = dm.N, M = dm.M, nc = dm.nc;
        const double kappa_d = 1e-5, rho = SC(SC_RHO), zeta = SC(SC_ZETA);
        const double* ori = &AT(wdi, 0);
        const int oU = ws.L_X, oS = oU + ws.L_U;
        double Pp[3][3], ps[3], hx[NX], gp[NX], gu[NU], uu[NU], ss = 0, gs = 0;
#pragma unroll
        for (int i = 0; i < 3; ++i) {
            ps[i] = 0;
#pragma unroll
            for (int j = 0; j < 3; ++j) Pp[i][j] = 0;
        }
#pragma unroll
        for (int i = 0; i < NX; ++i) {  // proximity term: gradient zeta D_R^2 (x - x_R), curvature zeta D_R^2
            const double xr = ori[k * NX + i], dr = fmin(1.0, 1.0 / fabs(xr));
            hx[i] = zeta * dr * dr;
            gp[i] = hx[i] * (AT(X, k * NX + i) - xr);
        }
#pragma unroll
        for (int i = 0; i < NU; ++i) {
            uu[i] = gu[i] = 0;
            if (k < N) {
                const double ur = ori[oU + k * NU + i], dr = fmin(1.0, 1.0 / fabs(ur));
                uu[i] = zeta * dr * dr;
                gu[i] = uu[i] * (AT(U, k * NU + i) - ur);
            }
        }
        const double Sk = AT(S, k);
        if (dm.ns) {
            const double sr = ori[oS + k], dr = fmin(1.0, 1.0 / fabs(sr));
            ss = zeta * dr * dr;
            gs = ss * (Sk - sr);
        }
        double Hz[NX + NU][NX + NU];
#pragma unroll
        for (int i = 0; i < NX + NU; ++i)
#pragma unroll
            for (int j = 0; j < NX + NU; ++j) Hz[i][j] = 0;
        if (k < N) {  // dynamics c_k = x_{k+1} - F_k  =>  W -= sum_i y_i d2F_i
            double x[NX], u[NU], l[NX];
#pragma unroll
            for (int i = 0; i < NX; ++i) x[i] = AT(X, k * NX + i);
#pragma unroll
            for (int i = 0; i < NU; ++i) u[i] = AT(U, k * NU + i);
#pragma unroll
            for (int i = 0; i < NX; ++i) l[i] = AT(yk, k * NX + i);
            D::hess(x, u, l, p.dt, p.wheelbase, Hz);
        }
        {
            const int ia[6] = {0, 0, 0, 1, 1, 2}, ib[6] = {0, 1, 2, 1, 2, 2};
#pragma unroll
            for (int q = 0; q < 6; ++q) {
                const double v = AT(Hd, k * 6 + q);
                Pp[ia[q]][ib[q]] += v;
                if (ia[q] != ib[q]) Pp[ib[q]][ia[q]] += v;
            }
        }
        // bound barriers; general bounds: the bound row with sb, p and n eliminated (bound_row_resto)
        if (k < N)
#pragma unroll
            for (int i = 0; i < NU; ++i) {
                const double uv = BVU(k * NU + i), sl = uv - p.umin[i], su = p.umax[i] - uv;
                const double sig = AT(zl, k * NU + i) / sl + AT(zu, k * NU + i) / su, bg = -mu / sl + mu / su;
                if (dm.gcb) {
                    double Db;
                    gu[i] += bound_row_resto(dm, ws, b, k * NU + i, sig, bg, dw, mu, &Db);
                    uu[i] += Db;
                } else {
                    uu[i] += sig;
                    gu[i] += bg;
                }
            }
        if (dm.ns) {
            const double sv = BVS(k), sig = AT(zs, k) / sv, bg = -mu / sv + kappa_d * mu;
            if (dm.gcb) {
                double Db;
                gs += bound_row_resto(dm, ws, b, N * NU + k, sig, bg, dw, mu, &Db);
                ss += Db;
            } else {
                ss += sig;
                gs += bg;
            }
        }
        const int q0 = NX + N * NX + nc;  // first inequality row
        for (int j = 0; j < M; ++j) {
            double J[3];
#pragma unroll
            for (int a = 0; a < 3; ++a) J[a] = AT(Jd, (k * M + j) * 3 + a);
            const int r = q0 + k * M + j;
            const double t = AT(T, k * M + j), v = AT(vt, k * M + j), pp = AT(rp, r), nn = AT(rn, r);
            const double st = v / t + dw, sp = AT(rzp, r) / pp + dw, sn = AT(rzn, r) / nn + dw;
            const double C = 1.0 / st + 1.0 / sp + 1.0 / sn;
            const double E = (mu / t - kappa_d * mu) / st + (mu / pp - rho - kappa_d * mu) / sp -
                             (mu / nn - rho - kappa_d * mu) / sn;
            const double Dj = 1.0 / C, rhs = (AT(rcq, k * M + j) - E) / C;
#pragma unroll
            for (int a = 0; a < 3; ++a) {
                gp[a] += J[a] * rhs;
#pragma unroll
                for (int c = 0; c < 3; ++c) Pp[a][c] += Dj * J[a] * J[c];
                if (dm.sd) ps[a] += Dj * J[a];
            }
            if (dm.sd) {
                ss += Dj;
                gs += rhs;
            }
        }
        auto emit = [&](auto has_u) {
            constexpr bool HU = decltype(has_u)::value;
            constexpr int is = HU ? NX + NU : NX;
            const bool hs = dm.ns != 0;
            const int nz = is + (hs ? 1 : 0);
#pragma unroll
            for (int i = 0; i < NZ; ++i) {
#pragma unroll
                for (int j = 0; j < NZ; ++j) {
                    double h = 0;
                    if (i < 3 && j < 3) h += Pp[i][j];
                    if (i == j && i < NX) h += hx[i];
                    if (HU && i == j && i >= NX && i < NX + NU) h += uu[i - NX];
                    if (HU && i < NX + NU && j < NX + NU) h -= Hz[i][j];
                    if (hs) {
                        if (i == is && j == is) h += ss;
                        if (i == is && j < 3) h += ps[j];
                        if (j == is && i < 3) h += ps[i];
                    }
                    if (i == j && i < nz) h += dw;
                    o[i * (NZ + 2) + j] = h;
                }
                double gi = 0;
                if (i < NX) gi = gp[i];
                else if (HU && i < NX + NU) gi = gu[i - NX];
                if (hs && i == is) gi = gs;
                o[i * (NZ + 2) + NZ] = gi;
                o[i * (NZ + 2) + NZ + 1] = 0.0;
            }
        };
        if (k < N) emit(std::true_type{});
        else emit(std::false_type{});
    }

    // general bounds in the restoration problem (oracle bound_row, resto branch): bound row q with its slack sb (barrier
    // Hessian sig, gradient bg) and its p, n eliminated like an inequality row's t, p, n: D = 1 / C, rhs = (r - E) / C,
    // C = 1/(sig + dw) + 1/(zp/p + dw) + 1/(zn/n + dw), r = rcb (c - p + n); returns rhs, D in *Dq
    __device__ __forceinline__ static double bound_row_resto(const Dims& dm, const Ws& ws, int b, int q, double sig,
                                                             double bg, double dw, double mu, double* Dq) {
        const double kappa_d = 1e-5, rho = SC(SC_RHO);
        const int r = NX + dm.N * NX + dm.nc + (dm.N + 1) * dm.M + q;
        const double pp = AT(rp, r), nn = AT(rn, r);
        const double st = sig + dw, sp = AT(rzp, r) / pp + dw, sn = AT(rzn, r) / nn + dw;
        const double C = 1.0 / st + 1.0 / sp + 1.0 / sn;
        const double E = -bg / st + (mu / pp - rho - kappa_d * mu) / sp - (mu / nn - rho - kappa_d * mu) / sn;
        *Dq = 1.0 / C;
        return (AT(rcb, q) - E) / C;
    }

    // the soft equality rows' compliance and offset (oracle build(), resto branch) for delta_w dw, rows lane.. by
    // stride: D = 1/sp + 1/sn, e = (mu/p - rho - kd mu)/sp - (mu/n - rho - kd mu)/sn, sp = zp/p + dw, sn = zn/n + dw
    __device__ static void soft_rows(const Dims& dm, const Ws& ws, int b, int lane, int stride, double dw, double mu) {
        const double kappa_d = 1e-5, rho = SC(SC_RHO);
        const int nrow = NX + dm.N * NX + dm.nc;
        for (int i = lane; i < nrow; i += stride) {
            const double pp = AT(rp, i), nn = AT(rn, i);
            const double sp = AT(rzp, i) / pp + dw, sn = AT(rzn, i) / nn + dw;
            AT(dsoft, i) = 1.0 / sp + 1.0 / sn;
            AT(esoft, i) = (mu / pp - rho - kappa_d * mu) / sp - (mu / nn - rho - kappa_d * mu) / sn;
        }
    }

    // every stage of the restoration Newton system (lane = knot): hg, and the slot [A B 0 | c + e] with M = 0
    __device__ static void build_stages_resto(const NlotProblem& p, const Dims& dm, const Ws& ws, int b, int lane,
                                              double dw, double mu, double* SL) {
        const int N = dm.N;
        soft_rows(dm, ws, b, lane, 64, dw, mu);
        __syncthreads();
        for (int k = lane; k <= N; k += 64) {
            double* o = SL + (size_t)k * SLOT;
            stage_resto(p, dm, ws, b, k, dw, mu, &AT(hg, k * HG));
            double A[NX][NX], Bu[NX][NU];
#pragma unroll
            for (int i = 0; i < NX; ++i) {
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
            }
#pragma unroll
            for (int i = 0; i < NX; ++i) {
#pragma unroll
                for (int j = 0; j < NZ; ++j) o[sAB + i * NAB + j] = j < NX ? A[i][j] : (j < NX + NU ? Bu[i][j - NX] : 0.0);
                o[sAB + i * NAB + NZ] = k < N ? -AT(rcd, k * NX + i) + AT(esoft, NX + k * NX + i) : 0.0;
#pragma unroll
                for (int j = NZ + 1; j < NAB; ++j) o[sAB + i * NAB + j] = 0.0;
            }
            o[sM + 0] = o[sM + 1] = o[sM + 2] = o[sM + 3] = 0.0;  // the restoration objective has no path length
        }
        __syncthreads();
    }
};

// ---------------------------------------------------------------------------------------------
// Lane-group Riccati (kernel k_ric): G lanes per instance, 64 / G instances per wavefront.
// Lane j of a group owns column j of the stage's extended matrices.  It keeps W[:, j] and QE[:, j]
// in registers, plus its gain column and (terminal columns) its row of [Psi | psi].  LDS holds only
// what other lanes read: the staged [A B 0 | c] | M of the stage (double-buffered; HBM loads run a
// few stages ahead in registers), the value function, the three control columns of QE (Q_vv, Q_xv)
// and the gains.  Per stage: 3 wave-local LDS syncs, each followed by one batch of 16-byte reads;
// the 3x3 pivots are inverted once (reciprocals).
// ---------------------------------------------------------------------------------------------
template <int DYN>
struct RicG {
    using SV = Solver<DYN>;
    static constexpr int NX = SV::NX, NU = SV::NU, NV = SV::NV, NZ = SV::NZ, NC = SV::NC;
    static constexpr int NCOL = SV::NCOL, NQE = SV::NQE, NAB = SV::NAB;
    static constexpr int G = NQE <= 16 ? 16 : 32;  // lanes per instance (>= one per QE column)
    static constexpr int IPW = 64 / G;             // instances per wavefront
    static constexpr int NABM = NX * NAB + 4;      // [A B 0 | c | pad] | M, contiguous at the start of a slot
    static constexpr int ev(int n) { return n + (n & 1); }  // rows padded to 16 bytes
    static constexpr int NXP = ev(NX), NZP = ev(NZ), NCOLP = ev(NCOL);
    // Stage inputs arrive by global -> LDS DMA (global_load_lds_dwordx4: lane l of the wave lands 16 bytes
    // at base + 16 l, i.e. G * 16 bytes per group per instruction), RING stages ahead; no VGPRs held.
    static constexpr int DW = 2 * G;                       // doubles per group per DMA instruction
    static constexpr int NDH = (SV::HG + DW - 1) / DW;     // DMA instructions for hg
    static constexpr int NDA = (NABM + DW - 1) / DW;       // ... for [A B 0 | c] | M
    static constexpr int NDMA = NDH + NDA, RING = NLOT_RIC_RING;
    static_assert(SV::sAB == 0 && SV::sM == NX * NAB && NCOL <= NQE && NQE <= G && NV <= 4 && NAB % 2 == 0,
                  "RicG layout");
    struct alignas(16) Sh {  // per instance; every row starts on a 16-byte boundary
        double VE[NX][NCOLP];         // value function [P | p_0 p_1 | Gamma] of the stage after
        double QT[NV][NZP];           // columns NX .. NX+NV-1 of QE, transposed
        double VU[NCOL][NXP];         // value update before symmetrisation, column-major
        double cols[NCOL][4];         // gains
        double PE[NC][NC + 2];
    };
};
typedef double d2v __attribute__((ext_vector_type(2)));

// k_ric's LDS hand-offs between the lanes of its single wavefront.  NLOT_RIC_INORDER (the default) relies
// on the LDS unit executing one wavefront's DS instructions in issue order (a ds_read issued after a
// ds_write sees it), so only the compiler's order is pinned; NLOT_RIC_FENCED waits for the LDS queue and
// barriers instead (same results, measured slower).
__device__ __forceinline__ void ric_sync() {
#ifdef NLOT_RIC_INORDER
    asm volatile("" ::: "memory");
#else
    xsync<true>();
#endif
}
// before a DMA refills a ring slot: the slot's reads have returned
__device__ __forceinline__ void ric_sync_reads() {
#ifdef NLOT_RIC_INORDER
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0); vmcnt and expcnt not waited
    asm volatile("" ::: "memory");
#else
    xsync<true>();
#endif
}

// Newton (or least-squares) solve of the instances whose stage matrices k_iter_a built (SC_RIC = 1),
// with IPOPT's inertia correction: on a wrong inertia the group rebuilds its stages with the next
// delta_w and factorises again.  Outputs: dX dU dS yi_n yk_n yt_n (and the second right-hand side).
// waves per SIMD of k_ric: NLOT_WPE_RIC (restoration: NLOT_WPE_RRIC; corrections: NLOT_WPE_SOC), except
// ackermann_2nd (nx = 7), whose larger stage spills 384 B/lane at 2
template <int DYN, bool RESTO, bool SOC>
struct RicWpe {
    static constexpr int value = SOC ? NLOT_WPE_SOC : DYN % NLOT_RK4_BIAS == NLOT_ACKERMANN_2ND ? 1
                                                  : RESTO ? NLOT_WPE_RRIC : NLOT_WPE_RIC;
};
// RESTO = true: the restoration problem's Newton solve (instances with SC_RESTO = 1, list ws.actr): every
// equality row is soft (p, n eliminated, oracle soft_transform): before stage k uses the value function of
// x_{k+1} it becomes that of y = x_{k+1} - w (P <- (I + P D)^-1 P, [p | G] likewise, Psi / psi corrected), the
// initial state likewise after the sweep, the terminal rows get (-Psi + D_t) nu = ..., and the forward sweep
// maps x_{k+1} = (I + D P)^-1 (y - D (p + G nu)); every stage block must be positive definite.
// SOC = true: the second-order corrections (SC_RICFIX >= 0) by substitution with the stored factors; the SOC = false
// launch skips them (separate instantiations: the substitution's registers stay out of the factorising sweep's).
#ifdef NLOT_RIC_PROF
// tuning builds only: k_ric's phase times summed over its groups (wall clock, 10 ns), per instantiation kind
// (0 Newton, 1 correction, 2 restoration) x [backward, F1, F2, F3 + multipliers, solves]; printed by run()
__device__ unsigned long long g_ric_prof[3][5];
#endif
template <int DYN, bool RESTO, bool SOC = false>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(RicWpe<DYN, RESTO, SOC>::value))) void k_ric(const NlotProblem* __restrict__ pp_, const Dims* __restrict__ dd_,
                                            const Ws* __restrict__ ws_, const int* __restrict__ active, int n_active,
                                            const int* __restrict__ nact, int mode, int* __restrict__ diag,
                                            int max_tries) {
    using R = RicG<DYN>;
    using SV = Solver<DYN>;
    constexpr int NX = R::NX, NU = R::NU, NV = R::NV, NZ = R::NZ, NC = R::NC, NCOL = R::NCOL, NQE = R::NQE;
    constexpr int NAB = R::NAB, G = R::G, NABM = R::NABM, NCOLP = R::NCOLP, DW = R::DW, NDH = R::NDH, NDA = R::NDA;
    constexpr int NDMA = R::NDMA, RING = R::RING;
    constexpr int SLOT = SV::SLOT, HG = SV::HG, VF = SV::VF, sAB = SV::sAB, sM = SV::sM, sGN = SV::sGN;
    const NlotProblem& p = *pp_;
    const Dims& dm = *dd_;
    const Ws& ws = *ws_;
    // the side-stream chains share CUs with the main Newton solve and gate the step's later kernels: with
    // NLOT_SETPRIO their waves win the SIMD's issue arbitration (s_setprio; arithmetic unchanged)
    if ((RESTO || SOC) && ws.prio) __builtin_amdgcn_s_setprio(2);
    __shared__ typename R::Sh shg[R::IPW];
    __shared__ __attribute__((aligned(16))) double ring[RING][NDMA][R::IPW][DW];  // DMA'd stage inputs
    const int grp = threadIdx.x / G, l = threadIdx.x % G, gb = grp * G;
    // RESTO: grid-stride over the whole restoration list (the host sizes the grid by a stale bound, which the list can
    // outgrow within a synchronisation window; an instance left out would repeat k_resto_a's evaluation, whose
    // barrier update is not idempotent); else one instance per group, at most the grid's
    const int nlist = RESTO ? *nact : std::min(n_active, *nact);
    if constexpr (!RESTO) grid_guard(ws, *nact, R::IPW, GRID_SOLVE);
    auto body = [&](const int si) {
    const int b = active[si];
    if ((int)SC(SC_RIC) != 1) return;
    if ((SC(SC_RESTO) != 0.0) != RESTO) return;
    if (!RESTO && (SC(SC_RICFIX) >= 0.0) != SOC) return;
    // least squares: the INIT instances only (phase read, not SC_RIC: the side stream's corrections set theirs concurrently)
    if (mode == MODE_LSQ && (int)SC(SC_PHASE) != PH_INIT) return;
    typename R::Sh& sh = shg[grp];
    const int N = dm.N, nc = dm.nc, ns = dm.ns;
    const double mu0 = SC(SC_RMU0), last_dw = SC(SC_DWLAST);
    const int nr = (int)SC(SC_RNR);
    double* SL = &AT(stg, 0);
    const int j = l;  // QE column of this lane
    const int gc = j < NX ? j : ((j >= NZ && j < NQE) ? NX + (j - NZ) : -1);  // gain column (qe_col^-1)
    const int a_pe = j - (NZ + 2);                                              // [Psi | psi] row
    const bool own_pe = a_pe >= 0 && a_pe < NC;
    double nu_[2][NC], dx0[NX];
    const int neg_lim = RESTO ? 0 : nc;  // negative stage pivots the terminal block can absorb (none: all rows soft)
    // a Newton solve keeps its factors (Q_vv per stage, the terminal block) for the second-order corrections
    constexpr int QFL = ldl_len(NV);
    const bool keep_fac = !RESTO && mode == MODE_NEWTON;
    const int q0r = NX + N * NX + nc;   // restoration rows: first inequality row (terminal rows at q0r - nc)

    // backward sweep + terminal multipliers; 0, or 1 on a wrong inertia (uniform within the group)
    auto backward = [&]() -> int {
        for (int e = l; e < NX * NCOLP; e += G) (&sh.VE[0][0])[e] = 0.0;
        double pe[NC + 2];
#pragma unroll
        for (int c = 0; c < NC + 2; ++c) pe[c] = 0.0;
        if (mode == MODE_NEWTON && l == 0) SC(SC_DC) = 0.0;
        // Stage inputs from HBM (written by k_iter_a, read once) stream into the LDS ring by DMA, RING
        // stages ahead.  Group grp's double e of a stage's hg lands at ring[slot][e / DW][grp][e % DW], the
        // [A B 0 | c] | M block at ring[slot][NDH + e / DW][grp][e % DW].
        double w[NX], q[NZ], gcol[NV], vr[NX];
        auto issue = [&](int k) {  // DMA of stage k (every lane of the group; one 16-byte piece each)
            if (k < 0) return;
            const int slot = k % RING;
            const double* hgk = &AT(hg, k * HG);
            const double* abk = SL + (size_t)k * SLOT;
#pragma unroll
            for (int t = 0; t < NDH; ++t) {
                const int e = t * DW + 2 * l;
                __builtin_amdgcn_global_load_lds((const void*)(hgk + (e < HG ? e : 0)),
                                                 (__attribute__((address_space(3))) void*)&ring[slot][t][0][0], 16, 0, 0);
            }
#pragma unroll
            for (int t = 0; t < NDA; ++t) {
                const int e = t * DW + 2 * l;
                __builtin_amdgcn_global_load_lds((const void*)(abk + (e < NABM ? e : 0)),
                                                 (__attribute__((address_space(3))) void*)&ring[slot][NDH + t][0][0], 16, 0,
                                                 0);
            }
        };
        // wait until at most `n` DMA instructions (plus whatever vector-memory stores came after them) are
        // outstanding: vmcnt counts stores too, so this is conservative (the ring stays ~2 stages ahead)
        auto wait_dma = [&](int n) {
            // s_waitcnt encoding (gfx9): vmcnt[3:0] | expcnt[6:4] = 7 | lgkmcnt[11:8] = 15 | vmcnt[5:4] << 14
            constexpr int base = (7 << 4) | (15 << 8);
            switch (n) {
                case 0: __builtin_amdgcn_s_waitcnt(base | 0); break;
                default: __builtin_amdgcn_s_waitcnt(base | (((RING - 1) * NDMA) & 15) | ((((RING - 1) * NDMA) >> 4) << 14)); break;
            }
            asm volatile("" ::: "memory");
        };
#pragma unroll
        for (int r = 0; r < RING; ++r) issue(N - r);
        int negsum = 0;
        // RESTO: the value function in sh.VE becomes that of y = x - w for the soft rows with compliance Dp[0..NX):
        // columns [P | p | G] <- S^-1 K^-1 S [P | p | G] (K = I + S P S, S = D^1/2, redundantly factorised by every
        // lane), Psi -= G' D G~, psi -= G' D p~ (the terminal lanes' registers).  1 if K is not positive definite.
        auto soft_step = [&](const double* Dp) -> int {
            double Dd[NX], Sd[NX], K[NX][NX], v[NX], ga[NX];
#pragma unroll
            for (int i = 0; i < NX; ++i) {
                Dd[i] = Dp[i];
                Sd[i] = sqrt(Dd[i]);
            }
#pragma unroll
            for (int i = 0; i < NX; ++i)
#pragma unroll
                for (int c = 0; c < NX; ++c) K[i][c] = (i == c ? 1.0 : 0.0) + Sd[i] * sh.VE[i][c] * Sd[c];
            int perm[NX], nneg;
            if (ldl_factor<NX>(K, NX, perm, &nneg) || nneg) return 1;
#pragma unroll
            for (int i = 0; i < NX; ++i) {
                v[i] = gc >= 0 ? Sd[i] * sh.VE[i][gc] : 0.0;
                ga[i] = own_pe ? sh.VE[i][NX + 2 + a_pe] : 0.0;
            }
            ric_sync();
            if (gc >= 0) {
                ldl_solve1<NX>(K, NX, perm, v);
#pragma unroll
                for (int i = 0; i < NX; ++i) sh.VE[i][gc] = v[i] / Sd[i];
            }
            ric_sync();
            if (own_pe) {
#pragma unroll
                for (int c = 0; c < NC + 2; ++c) {
                    const int vc_ = c < NC ? NX + 2 + c : NX + (c - NC);
                    double t = 0;
#pragma unroll
                    for (int i = 0; i < NX; ++i) t += Dd[i] * ga[i] * sh.VE[i][vc_];
                    pe[c] -= t;
                }
            }
            return 0;
        };
        const bool wcol = j < NZ + 2;              // W column j is P AB (+ p_r), not a Gamma pass-through
        const int cc = j < NZ ? j : NZ;            // AB column (the c column for the p_r columns)
        const int jc = j >= NZ && j < NQE ? NX + j - NZ : 0;  // VE column carried into W
        const bool vlane = j >= NX && j < NX + NV;  // control columns: Q_vv, Q_xv
        ric_sync();
#ifdef NLOT_PHASE_PROF
        long long ph[5] = {0, 0, 0, 0, 0};
#endif
        for (int k = N; k >= 0; --k) {
#ifdef NLOT_PHASE_PROF
            long long tq = wall_clock64();
#endif
            const int nv = (k < N ? NU : 0) + ns;
            if constexpr (RESTO)
                if (k < N && soft_step(&AT(dsoft, NX + k * NX))) return 1;  // soft dynamics rows of stage k
            wait_dma(k >= RING - 1 ? 1 : 0);  // stage k's DMA landed (the later RING-1 stages may be in flight)
            const double* hrow = &ring[k % RING][0][grp][0];  // hg of stage k, element e at (e / DW) * IPW * DW + e % DW
            auto HGe = [&](int e) { return hrow[(e / DW) * (R::IPW * DW) + e % DW]; };
            const double* abase = &ring[k % RING][NDH][grp][0];
            auto ABe = [&](int e) { return abase[(e / DW) * (R::IPW * DW) + e % DW]; };
            double hcur[NZ];  // column j of [H | g_0 g_1]: row j of the symmetric H, or a g column read down; zero
                              // beyond nr
            {
                const int jg = j < NZ + 2 ? j : NZ;
#pragma unroll
                for (int i = 0; i < NZ; ++i) {
                    const double v = HGe(j < NZ ? j * (NZ + 2) + i : i * (NZ + 2) + jg);
                    hcur[i] = j < NZ + nr ? v : 0.0;
                }
            }
            // ---- batch 1: P (rows of VE), this lane's VE column and AB column, M ----
            double P[NX][NX], vc[NX], abc[NX];
#pragma unroll
            for (int r = 0; r < NX; ++r) {
                const d2v* row = reinterpret_cast<const d2v*>(&sh.VE[r][0]);
#pragma unroll
                for (int c2 = 0; c2 < NX / 2; ++c2) {
                    const d2v v = row[c2];
                    P[r][2 * c2] = v.x;
                    P[r][2 * c2 + 1] = v.y;
                }
                if (NX & 1) P[r][NX - 1] = sh.VE[r][NX - 1];
                vc[r] = sh.VE[r][jc];
                abc[r] = ABe(r * NAB + cc);
            }
            const d2v m01 = d2v{ABe(NX * NAB), ABe(NX * NAB + 1)}, m23 = d2v{ABe(NX * NAB + 2), ABe(NX * NAB + 3)};
            // (1) W[:, j] = [P AB | P c + p_0 | P c + p_1 | G][:, j]
#pragma unroll
            for (int r = 0; r < NX; ++r) {
                double t = j < NZ ? 0.0 : vc[r];
#pragma unroll
                for (int qq = 0; qq < NX; ++qq) t += P[r][qq] * abc[qq];
                w[r] = wcol ? t : vc[r];
            }
            // (2) QE[:, j] = [H | g] + cross + AB' W  (cross: path-length coupling through the dynamics)
            const double mj0 = j == 0 ? m01.x : m23.x, mj1 = j == 0 ? m01.y : m23.y;
#pragma unroll
            for (int i = 0; i < NZ; ++i) {
                double ab_i[NX];
#pragma unroll
                for (int r = 0; r < NX; ++r) ab_i[r] = ABe(r * NAB + i);
                double t = hcur[i];
                if (i < 2) {
                    const double x = (i == 0 ? m01.x : m23.x) * abc[0] + (i == 0 ? m01.y : m23.y) * abc[1];
                    t = wcol ? t + x : t;
                }
                {
                    const double x = mj0 * ab_i[0] + mj1 * ab_i[1];
                    t = (wcol && j < 2) ? t + x : t;
                }
#pragma unroll
                for (int r = 0; r < NX; ++r) t += ab_i[r] * w[r];
                q[i] = t;
            }
            if (vlane) {
                d2v* dst = reinterpret_cast<d2v*>(&sh.QT[j - NX][0]);
#pragma unroll
                for (int i2 = 0; i2 < NZ / 2; ++i2) dst[i2] = d2v{q[2 * i2], q[2 * i2 + 1]};
                if (NZ & 1) sh.QT[j - NX][NZ - 1] = q[NZ - 1];
            }
#ifdef NLOT_PHASE_PROF
            { const long long t = wall_clock64(); ph[0] += t - tq; tq = t; }
#endif
            ric_sync();
            // ---- batch 2: the control columns of QE (Q_vv, Q_xv), read from LDS where they are used (holding all
            //      NV x NZ of them in registers across the factorisation spilled the factorising sweep) ----
            auto Qv = [&](int v, int i) { return sh.QT[v][i]; };
#ifdef NLOT_PHASE_PROF
            { const long long t = wall_clock64(); ph[1] += t - tq; tq = t; }
#endif
            // (3) Q_vv factorised by every lane (identical, uniform inertia decision); lane j solves its
            //     gain column in registers
#pragma unroll
            for (int v = 0; v < NV; ++v) gcol[v] = 0.0;
            if (nv == 3 && NV == 3) {
                // pivoted LDL^T of the symmetric 3x3 (pivot order of ldl_factor: largest diagonal first,
                // then the larger remaining diagonal), reciprocal pivots
                auto qv = [&](int a, int c) {  // Q_vv[a][c] = QE[NX + a][NX + c] = Qv(c, NX + a) (static a, c)
                    return Qv(c, NX + a);
                };
                double scale = 1e-300;
#pragma unroll
                for (int a = 0; a < 3; ++a)
#pragma unroll
                    for (int c = 0; c < 3; ++c) scale = fmax(scale, fabs(qv(a, c)));
                const double a00 = qv(0, 0), a11 = qv(1, 1), a22 = qv(2, 2);
                int pv = 0;
                if (fabs(a11) > fabs(a00)) pv = 1;
                if (fabs(a22) > fabs(pv == 1 ? a11 : a00)) pv = 2;
                int o0 = pv, o1 = pv == 1 ? 0 : 1, o2 = pv == 2 ? 0 : 2;
                // pivoted entries by LDS address (a register array indexed at run time would go to scratch)
                const double d0 = sh.QT[o0][NX + o0], c1 = sh.QT[o0][NX + o1], c2 = sh.QT[o0][NX + o2];
                const double e11 = sh.QT[o1][NX + o1], e21 = sh.QT[o1][NX + o2], e22 = sh.QT[o2][NX + o2];
                if (!(fabs(d0) > 1e-13 * scale) || !isfinite(d0)) return 1;
                const double i0 = 1.0 / d0;
                double l10 = c1 * i0, l20 = c2 * i0;
                double b11 = e11 - c1 * l10;
                const double b21 = e21 - c2 * l10;
                double b22 = e22 - c2 * l20;
                if (fabs(b22) > fabs(b11)) {  // swap positions 1 and 2 (rows of L included)
                    const int t = o1;
                    o1 = o2;
                    o2 = t;
                    const double tb = b11;
                    b11 = b22;
                    b22 = tb;
                    const double tl = l10;
                    l10 = l20;
                    l20 = tl;
                }
                const double d1 = b11;
                if (!(fabs(d1) > 1e-13 * scale) || !isfinite(d1)) return 1;
                const double i1 = 1.0 / d1, l21 = b21 * i1, d2 = b22 - b21 * l21;
                if (!(fabs(d2) > 1e-13 * scale) || !isfinite(d2)) return 1;
                const double i2 = 1.0 / d2;
                negsum += (d0 < 0) + (d1 < 0) + (d2 < 0);
                if (negsum > neg_lim) return 1;
                if (keep_fac && l == 0) {  // ldl_factor's form: L below the diagonal, D on it, then the permutation
                    const double f[QFL] = {d0, 0.0, 0.0, l10, d1, 0.0, l20, l21, d2, (double)o0, (double)o1, (double)o2};
                    double* qf = &AT(qfac, k * QFL);
#pragma unroll
                    for (int e = 0; e < QFL; ++e) qf[e] = f[e];
                }
                if (gc >= 0) {
                    const double x0 = q[NX], x1 = q[NX + 1], x2 = q[NX + 2];
                    // permutations as exact 0/1 blends (selects by a run-time index become scratch arrays)
                    auto pick = [&](int o) { return (o == 0 ? 1.0 : 0.0) * x0 + (o == 1 ? 1.0 : 0.0) * x1 + (o == 2 ? 1.0 : 0.0) * x2; };
                    double t0 = pick(o0), t1 = pick(o1), t2 = pick(o2);
                    t1 -= l10 * t0;
                    t2 -= l20 * t0;
                    t2 -= l21 * t1;
                    t0 *= i0;
                    t1 *= i1;
                    t2 *= i2;
                    t1 -= l21 * t2;
                    t0 -= l10 * t1;
                    t0 -= l20 * t2;
#pragma unroll
                    for (int v = 0; v < 3; ++v)
                        gcol[v] = -((o0 == v ? 1.0 : 0.0) * t0 + (o1 == v ? 1.0 : 0.0) * t1 + (o2 == v ? 1.0 : 0.0) * t2);
                }
            } else if (nv > 0) {
                double L[NV][NV];
                int perm[NV], nneg;
#pragma unroll
                for (int a = 0; a < NV; ++a)
#pragma unroll
                    for (int c = 0; c < NV; ++c) L[a][c] = (a < nv && c < nv) ? Qv(c, NX + a) : 0.0;
                if (ldl_factor<NV>(L, nv, perm, &nneg)) return 1;
                negsum += nneg;
                if (negsum > neg_lim) return 1;
                if (keep_fac && l == 0) {
                    double* qf = &AT(qfac, k * QFL);
#pragma unroll
                    for (int a = 0; a < NV; ++a) {
#pragma unroll
                        for (int c = 0; c < NV; ++c) qf[a * NV + c] = L[a][c];
                        qf[NV * NV + a] = (double)perm[a];
                    }
                }
                if (gc >= 0) {
                    double col[NV];
#pragma unroll
                    for (int v = 0; v < NV; ++v) col[v] = v < nv ? -q[NX + v] : 0.0;
                    ldl_solve1<NV>(L, nv, perm, col);
#pragma unroll
                    for (int v = 0; v < NV; ++v) gcol[v] = v < nv ? col[v] : 0.0;
                }
            }
            // (4a) gains to LDS and to the slot (forward sweep); raw value update of column gc
            if (gc >= 0) {
                double* GN = SL + (size_t)k * SLOT + sGN;
                d2v* cd = reinterpret_cast<d2v*>(&sh.cols[gc][0]);
                cd[0] = d2v{gcol[0], NV > 1 ? gcol[NV > 1 ? 1 : 0] : 0.0};
                if (NV > 2) cd[1] = d2v{gcol[NV > 2 ? 2 : 0], 0.0};
#pragma unroll
                for (int v = 0; v < NV; ++v) GN[gc * NV + v] = gcol[v];
#pragma unroll
                for (int i = 0; i < NX; ++i) {
                    double t = q[i];
#pragma unroll
                    for (int v = 0; v < NV; ++v) t += Qv(v, i) * gcol[v];
                    vr[i] = t;
                }
                d2v* vd = reinterpret_cast<d2v*>(&sh.VU[gc][0]);
#pragma unroll
                for (int i2 = 0; i2 < NX / 2; ++i2) vd[i2] = d2v{vr[2 * i2], vr[2 * i2 + 1]};
                if (NX & 1) sh.VU[gc][NX - 1] = vr[NX - 1];
            }
#ifdef NLOT_PHASE_PROF
            { const long long t = wall_clock64(); ph[2] += t - tq; tq = t; }
#endif
            ric_sync();
            // ---- batch 3: transposed raw values (symmetrisation), gains of the terminal columns ----
            if (gc >= 0) {
                double tr[NX];
#pragma unroll
                for (int i = 0; i < NX; ++i) tr[i] = sh.VU[i][gc < NX ? gc : 0];
                double* vfk = &AT(vf, k * VF);
#pragma unroll
                for (int i = 0; i < NX; ++i) {
                    double t = vr[i];
                    if (gc < NX && gc != i) t = 0.5 * (t + tr[i]);
                    if (k == N && gc >= NX + 2) {
                        const int c3 = gc - NX - 2;
                        t = (c3 < nc && dm.tidx[c3] == i) ? 1.0 : 0.0;
                    }
                    sh.VE[i][gc] = t;
                    vfk[i * NCOL + gc] = t;
                }
            }
            // (4c) terminal system rows [Psi | psi_0 psi_1] (lanes of the terminal columns, registers)
            if (own_pe) {
#pragma unroll
                for (int c = 0; c < NC; ++c) {
                    const d2v* cs = reinterpret_cast<const d2v*>(&sh.cols[NX + 2 + c][0]);
                    const d2v g01 = cs[0], g23 = cs[1];
                    const double gv[4] = {g01.x, g01.y, g23.x, g23.y};
                    double t = 0;
#pragma unroll
                    for (int v = 0; v < NV; ++v) t += q[NX + v] * gv[v];
                    pe[c] += t;
                }
#pragma unroll
                for (int rr = 0; rr < 2; ++rr) {
                    if (k == N) {
                        pe[NC + rr] = (a_pe < nc && mode == MODE_NEWTON)
                                          ? AT(rct, a_pe) - (RESTO ? AT(esoft, q0r - nc + a_pe) : 0.0)
                                          : 0.0;
                    } else {
                        const d2v* cs = reinterpret_cast<const d2v*>(&sh.cols[NX + rr][0]);
                        const d2v g01 = cs[0], g23 = cs[1];
                        const double gv[4] = {g01.x, g01.y, g23.x, g23.y};
                        double t = 0;
#pragma unroll
                        for (int qq = 0; qq < NX; ++qq) t += w[qq] * ABe(qq * NAB + NZ);
#pragma unroll
                        for (int v = 0; v < NV; ++v) t += q[NX + v] * gv[v];
                        pe[NC + rr] += t;
                    }
                }
            }
            ric_sync_reads();  // every read of slot k % RING is complete before the DMA refills it
            issue(k - RING);
#ifdef NLOT_PHASE_PROF
            { const long long t = wall_clock64(); ph[3] += t - tq; tq = t; }
#endif
            ric_sync();
#ifdef NLOT_PHASE_PROF
            ph[4] += wall_clock64() - tq;
#endif
        }
#ifdef NLOT_PHASE_PROF
        if (b == 0 && l == 0 && SC(SC_ITERS) < 3)
            printf("RICG stage phases: WQ %lld syncA+Qv %lld ldl+gains+VU %lld sym+PE+stage %lld syncC %lld (x10ns, sum over stages)\n",
                   ph[0], ph[1], ph[2], ph[3], ph[4]);
#endif
        if constexpr (RESTO)
            if (soft_step(&AT(dsoft, 0))) return 1;  // soft initial-state rows
        if (own_pe)
#pragma unroll
            for (int c = 0; c < NC + 2; ++c) sh.PE[a_pe][c] = pe[c];
        __syncthreads();  // gains (slot) and vf in HBM are read across lanes by the forward sweep
        // terminal multipliers (every lane, identical): -Psi nu_r = G0' dx0 + psi_r, delta_c on the terminal block
#pragma unroll
        for (int i = 0; i < NX; ++i) dx0[i] = mode == MODE_NEWTON ? -AT(rci, i) + (RESTO ? AT(esoft, i) : 0.0) : 0.0;
#pragma unroll
        for (int rr = 0; rr < 2; ++rr)
#pragma unroll
            for (int cc = 0; cc < NC; ++cc) nu_[rr][cc] = 0.0;
        if (RESTO && nc) {  // soft terminal rows: (-Psi + D_t) nu = G0' dx0 + psi, positive definite
            double L[NC][NC];
            int perm[NC], nneg;
#pragma unroll
            for (int i = 0; i < NC; ++i)
#pragma unroll
                for (int c = 0; c < NC; ++c)
                    L[i][c] = (i < nc && c < nc) ? -sh.PE[i][c] + (i == c ? AT(dsoft, q0r - nc + i) : 0.0)
                                                 : 0.0;
            if (ldl_factor<NC>(L, nc, perm, &nneg) || nneg) return 1;
#pragma unroll
            for (int cc = 0; cc < NC; ++cc) {
                double t = 0;
                if (cc < nc) {
                    t = sh.PE[cc][NC];
#pragma unroll
                    for (int r = 0; r < NX; ++r) t += sh.VE[r][NX + 2 + cc] * dx0[r];
                }
                nu_[0][cc] = t;
            }
            ldl_solve1<NC>(L, nc, perm, nu_[0]);
        } else if (nc) {
            double L[NC][NC];
            int perm[NC], nneg;
#pragma unroll
            for (int i = 0; i < NC; ++i)
#pragma unroll
                for (int c = 0; c < NC; ++c) L[i][c] = (i < nc && c < nc) ? -sh.PE[i][c] : 0.0;
            int f = ldl_factor<NC>(L, nc, perm, &nneg);
            if (f == 2 || nneg != negsum) {
                const double dc = 1e-8 * pow(SC(SC_MU), 0.25);
#pragma unroll
                for (int i = 0; i < NC; ++i)
#pragma unroll
                    for (int c = 0; c < NC; ++c) L[i][c] = (i < nc && c < nc) ? -sh.PE[i][c] + (i == c ? dc : 0.0) : 0.0;
                if (ldl_factor<NC>(L, nc, perm, &nneg)) return 1;
                if (nneg != negsum) return 1;
                if (l == 0) SC(SC_DC) = dc;
            }
            if (keep_fac && l == 0) {
                double* tf = &AT(tfac, 0);
#pragma unroll
                for (int a = 0; a < NC; ++a) {
#pragma unroll
                    for (int c = 0; c < NC; ++c) tf[a * NC + c] = L[a][c];
                    tf[NC * NC + a] = (double)perm[a];
                }
            }
#pragma unroll
            for (int rr = 0; rr < 2; ++rr) {
                if (rr >= nr) break;
#pragma unroll
                for (int cc = 0; cc < NC; ++cc) {
                    double t = 0;
                    if (cc < nc) {
                        t = sh.PE[cc][NC + rr];
#pragma unroll
                        for (int r = 0; r < NX; ++r) t += sh.VE[r][NX + 2 + cc] * dx0[r];
                    }
                    nu_[rr][cc] = t;
                }
                ldl_solve1<NC>(L, nc, perm, nu_[rr]);
            }
        } else if (negsum) {
            return 1;
        }
        return 0;
    };

    // Second-order correction (SC_RICFIX >= 0): the matrix is the iteration's (same iterate, multipliers and
    // delta_w), only the right-hand side changed (g and c from the corrected residuals, k_iter_a).  So no
    // factorisation: a backward substitution with the stored Q_vv factors and gains, the value function's P and
    // Gamma kept from the iteration's sweep, and the recursion of the right-hand-side terms alone:
    //   w = P' c + p',  q = g + M c + AB' w,  k = -Q_vv^-1 q_v,  p = q_x + K' q_v,  psi += Gamma'(c + B k)
    // (p = q_x + Q_xv k = q_x + K' q_v since K = -Q_vv^-1 Q_vx).  Lanes i < NX carry w, p and the open-loop
    // offset e = c + B k; lanes i < NZ carry q; every lane solves the NV x NV system; lanes a < NC carry psi.
    // Writes k_0 into the gains and p_0 into vf (the forward sweep's inputs), nu_[0] and dx0.
    auto backward_rhs = [&]() {
        const int li = l < NZ ? l : 0, lx = l < NX ? l : 0, lm = l < 2 ? l : 0, la = l < NC ? l : 0;
        // one stage's inputs of this lane (row lx / column li / terminal column la; the stored Q_vv factor one element
        // per lane, shuffled where the solve needs it), SD - 1 stages ahead: a stage is a few shuffles and ~40 fused
        // multiply-adds, an HBM round trip several microseconds under the bulk's load
        constexpr int SD = 3;
        static_assert(QFL <= G, "one factor element per lane");
        struct In {
            double cl, g, m0, m1, P[NX], ab[NX], gam[NX], qfl, kt[NV], bu[NU];
        };
        auto load = [&](int k, In& d) {
            const double* slot = SL + (size_t)k * SLOT;
            const double* vn = &AT(vf, (k < N ? k + 1 : N) * VF);  // the stage after (k < N; clamped, unused at N)
            d.cl = slot[sAB + lx * NAB + NZ];
            d.g = AT(hg, k * HG + li * (NZ + 2) + NZ);
            d.m0 = slot[sM + 2 * lm];
            d.m1 = slot[sM + 2 * lm + 1];
#pragma unroll
            for (int r = 0; r < NX; ++r) {
                d.P[r] = vn[lx * NCOL + r];
                d.ab[r] = slot[sAB + r * NAB + li];
                d.gam[r] = vn[r * NCOL + NX + 2 + la];
            }
            d.qfl = AT(qfac, k * QFL + (l < QFL ? l : 0));
#pragma unroll
            for (int v = 0; v < NV; ++v) d.kt[v] = slot[sGN + lx * NV + v];
#pragma unroll
            for (int v = 0; v < NU; ++v) d.bu[v] = slot[sAB + lx * NAB + NX + v];
        };
        double pn = 0.0, psi = 0.0;
        // three buffers with static names (a rotated array of structs costs register copies), each refilled with the
        // stage SD below the one it held as soon as that stage is done
        In b0, b1, b2;
        static_assert(SD == 3, "three stage buffers");
        load(N, b0);
        if (N >= 1) load(N - 1, b1);
        if (N >= 2) load(N - 2, b2);
        auto stage_k = [&](const int k, const In& cur) {
            const int nv = (k < N ? NU : 0) + ns;
            const bool kn = k < N;
            const double cl = kn && l < NX ? cur.cl : 0.0;
            double c[NX];
#pragma unroll
            for (int r = 0; r < NX; ++r) c[r] = __shfl(cl, gb + r);
            double wl = pn;
#pragma unroll
            for (int qq = 0; qq < NX; ++qq) wl += cur.P[qq] * c[qq];
            double w[NX];
#pragma unroll
            for (int r = 0; r < NX; ++r) w[r] = __shfl(kn ? wl : 0.0, gb + r);
            double ql = cur.g;
            if (kn) {
                if (l < 2) ql += cur.m0 * c[0] + cur.m1 * c[1];
#pragma unroll
                for (int r = 0; r < NX; ++r) ql += cur.ab[r] * w[r];
            }
            double qvv[NV], kv[NV];  // q_v, then k = -Q_vv^-1 q_v
#pragma unroll
            for (int v = 0; v < NV; ++v) {
                qvv[v] = __shfl(ql, gb + NX + v);
                kv[v] = v < nv ? -qvv[v] : 0.0;
            }
            if (nv > 0) {
                double L[NV][NV];
                int perm[NV];
#pragma unroll
                for (int a = 0; a < NV; ++a) {
#pragma unroll
                    for (int cc = 0; cc < NV; ++cc) L[a][cc] = __shfl(cur.qfl, gb + a * NV + cc);
                    perm[a] = (int)__shfl(cur.qfl, gb + NV * NV + a);
                }
                ldl_solve1<NV>(L, nv, perm, kv);
            }
            double* GN = SL + (size_t)k * SLOT + sGN;
            if (l < NV) {
                double v = 0;
#pragma unroll
                for (int vv = 0; vv < NV; ++vv) v = vv == l ? kv[vv] : v;
                GN[NX * NV + l] = v;  // k_0
            }
            double pl = ql, el = cl;
#pragma unroll
            for (int v = 0; v < NV; ++v) pl += cur.kt[v] * qvv[v];
#pragma unroll
            for (int v = 0; v < NU; ++v) el += cur.bu[v] * kv[v];
            if (l < NX) AT(vf, k * VF + lx * NCOL + NX) = pl;  // p_0
            if (!kn) {
                psi = l < nc ? AT(rct, la) : 0.0;
            } else {
                double e[NX];
#pragma unroll
                for (int r = 0; r < NX; ++r) e[r] = __shfl(el, gb + r);
#pragma unroll
                for (int r = 0; r < NX; ++r) psi += cur.gam[r] * e[r];
            }
            pn = pl;
        };
        for (int k = N; k >= 0;) {
            stage_k(k, b0);
            if (k - SD >= 0) load(k - SD, b0);
            if (--k < 0) break;
            stage_k(k, b1);
            if (k - SD >= 0) load(k - SD, b1);
            if (--k < 0) break;
            stage_k(k, b2);
            if (k - SD >= 0) load(k - SD, b2);
            --k;
        }
#pragma unroll
        for (int i = 0; i < NX; ++i) dx0[i] = -AT(rci, i);
#pragma unroll
        for (int rr = 0; rr < 2; ++rr)
#pragma unroll
            for (int cc = 0; cc < NC; ++cc) nu_[rr][cc] = 0.0;
        if (nc) {  // (-Psi + delta_c) nu = psi + Gamma_0' dx0 with the stored factor
            double t = psi;
            if (l < nc)
#pragma unroll
                for (int r = 0; r < NX; ++r) t += AT(vf, r * NCOL + NX + 2 + li) * dx0[r];
#pragma unroll
            for (int cc = 0; cc < NC; ++cc) {
                const double v = __shfl(t, gb + cc);
                nu_[0][cc] = cc < nc ? v : 0.0;
            }
            double L[NC][NC];
            int perm[NC];
            const double* f = &AT(tfac, 0);
#pragma unroll
            for (int a = 0; a < NC; ++a) {
#pragma unroll
                for (int cc = 0; cc < NC; ++cc) L[a][cc] = f[a * NC + cc];
                perm[a] = (int)f[NC * NC + a];
            }
            ldl_solve1<NC>(L, nc, perm, nu_[0]);
        }
        __syncthreads();  // k_0 and p_0 in HBM are read across lanes by the forward sweep
    };

    // delta_w enters the stage matrices linearly: H(dw) = H(0) + dw (I_nz + sum_q Jx_q Jx_q'),
    // g(dw) = g(0) + dw sum_q Jx_q c_q, with Jx_q = (d d_q/d pose, 1 on the slack when it enters d_q) and
    // c_q = rcq (stage(): D_q = v/t + dw); general bounds add dw e_b e_b' and dw e_b rcb_b per bound row b (D_b = Sigma_b
    // + dw on the control / slack column).  A retry adds (dw_new - dw_old) times that to hg in place.
    auto add_dw = [&](double ddw) {
        const int M = dm.M, sd = dm.sd;
        const bool hs = ns != 0;
        for (int k = l; k <= N; k += G) {
            double* o = &AT(hg, k * HG);
            const int is = k < N ? NX + NU : NX, nz = is + (hs ? 1 : 0);
            for (int i = 0; i < nz; ++i) o[i * (NZ + 2) + i] += ddw;
            if (dm.gcb) {  // bound rows: the control columns (k < N) and the slack column
                for (int i = NX; i < nz; ++i) {
                    const int qb = i < is ? k * NU + (i - NX) : N * NU + k;
                    const double r = ddw * AT(rcb, qb);
                    o[i * (NZ + 2) + i] += ddw;
                    o[i * (NZ + 2) + NZ] += r;
                    if (nr > 1) o[i * (NZ + 2) + NZ + 1] += r;
                }
            }
            for (int qq = 0; qq < M; ++qq) {
                double J[3];
#pragma unroll
                for (int a = 0; a < 3; ++a) J[a] = AT(Jd, (k * M + qq) * 3 + a);
                const double r = ddw * AT(rcq, k * M + qq);
#pragma unroll
                for (int a = 0; a < 3; ++a) {
#pragma unroll
                    for (int c = 0; c < 3; ++c) o[a * (NZ + 2) + c] += ddw * J[a] * J[c];
                    o[a * (NZ + 2) + NZ] += J[a] * r;
                    if (nr > 1) o[a * (NZ + 2) + NZ + 1] += J[a] * r;
                    if (sd) {
                        o[is * (NZ + 2) + a] += ddw * J[a];
                        o[a * (NZ + 2) + is] += ddw * J[a];
                    }
                }
                if (sd) {
                    o[is * (NZ + 2) + is] += ddw;
                    o[is * (NZ + 2) + NZ] += r;
                    if (nr > 1) o[is * (NZ + 2) + NZ + 1] += r;
                }
            }
        }
        __syncthreads();
    };

    // RESTO: the restoration system is not affine in delta_w (an inequality row's D = 1 / C, C = 1/(v/t + dw) +
    // 1/(zp/p + dw) + 1/(zn/n + dw)): the retry adds the differences of D J J' and J rhs per row, the diagonal
    // step, and recomputes the soft equality rows (dsoft / esoft, the slots' c columns)
    auto add_dw_resto = [&](double dw_old, double dw_new) {
        const int M = dm.M, sd = dm.sd;
        const bool hs = ns != 0;
        const double kappa_d = 1e-5, rho = SC(SC_RHO);
        SV::soft_rows(dm, ws, b, l, G, dw_new, mu0);
        __syncthreads();
        auto dr = [&](int r, int q, double dw_, double* Dq) {  // D and rhs of inequality row q (restoration row r)
            const double t = AT(T, q), v = AT(vt, q), pp = AT(rp, r), nn = AT(rn, r);
            const double st = v / t + dw_, sp = AT(rzp, r) / pp + dw_, sn = AT(rzn, r) / nn + dw_;
            const double C = 1.0 / st + 1.0 / sp + 1.0 / sn;
            const double E = (mu0 / t - kappa_d * mu0) / st + (mu0 / pp - rho - kappa_d * mu0) / sp -
                             (mu0 / nn - rho - kappa_d * mu0) / sn;
            *Dq = 1.0 / C;
            return (AT(rcq, q) - E) / C;
        };
        for (int k = l; k <= N; k += G) {
            double* o = &AT(hg, k * HG);
            const int is = k < N ? NX + NU : NX, nz = is + (hs ? 1 : 0);
            for (int i = 0; i < nz; ++i) o[i * (NZ + 2) + i] += dw_new - dw_old;
            for (int qq = 0; qq < M; ++qq) {
                double J[3], D0, D1;
#pragma unroll
                for (int a = 0; a < 3; ++a) J[a] = AT(Jd, (k * M + qq) * 3 + a);
                const int q = k * M + qq;
                const double r0 = dr(q0r + q, q, dw_old, &D0), r1 = dr(q0r + q, q, dw_new, &D1);
                const double dD = D1 - D0, dg = r1 - r0;
#pragma unroll
                for (int a = 0; a < 3; ++a) {
#pragma unroll
                    for (int c = 0; c < 3; ++c) o[a * (NZ + 2) + c] += dD * J[a] * J[c];
                    o[a * (NZ + 2) + NZ] += J[a] * dg;
                    if (sd) {
                        o[is * (NZ + 2) + a] += dD * J[a];
                        o[a * (NZ + 2) + is] += dD * J[a];
                    }
                }
                if (sd) {
                    o[is * (NZ + 2) + is] += dD;
                    o[is * (NZ + 2) + NZ] += dg;
                }
            }
            if (dm.gcb) {  // bound rows (sb, p, n eliminated): the differences of D and rhs on their columns
                for (int i = NX; i < nz; ++i) {
                    const int qb = i < is ? k * NU + (i - NX) : N * NU + k;
                    double sig, bg, D0, D1;
                    if (i < is) {
                        const double lo = p.umin[i - NX], hi = p.umax[i - NX], uv = BVU(qb);
                        sig = AT(zl, qb) / (uv - lo) + AT(zu, qb) / (hi - uv);
                        bg = -mu0 / (uv - lo) + mu0 / (hi - uv);
                    } else {
                        const double sv = BVS(k);
                        sig = AT(zs, k) / sv;
                        bg = -mu0 / sv + kappa_d * mu0;
                    }
                    const double r0 = SV::bound_row_resto(dm, ws, b, qb, sig, bg, dw_old, mu0, &D0);
                    const double r1 = SV::bound_row_resto(dm, ws, b, qb, sig, bg, dw_new, mu0, &D1);
                    o[i * (NZ + 2) + i] += D1 - D0;
                    o[i * (NZ + 2) + NZ] += r1 - r0;
                }
            }
            if (k < N)
                for (int i = 0; i < NX; ++i)
                    SL[(size_t)k * SLOT + sAB + i * NAB + NZ] = -AT(rcd, k * NX + i) + AT(esoft, NX + k * NX + i);
        }
        __syncthreads();
    };

    // inertia correction (IPOPT): delta_w = 0, then 1e-4 (or last / 3), x100 (x8 once one was used)
    const double fixdw = SC(SC_RICFIX);  // >= 0: second-order correction, stages built with this delta_w
    const bool fixed = fixdw >= 0.0;
    double dw = fixed ? fixdw : 0.0, dw_in_hg = dw;
    // an inertia correction this instance started in an earlier launch (the attempt cap deferred it): hg holds
    // dw_in_hg, the next delta_w of IPOPT's sequence is dw (the same sequence as in one launch)
    const bool resume = !SOC && mode == MODE_NEWTON && !fixed && SC(SC_RETRY) >= 0.0;
    if (resume) {
        dw = SC(SC_RETRY);
        dw_in_hg = SC(SC_DWHG);
    }
    int fail = 0;
#ifdef NLOT_PHASE_PROF
    long long t_build = 0, t_back = 0;
    int n_att = 0;
    PROF_T(tr0);
#endif
#ifdef NLOT_RIC_PROF
    const long long rp0 = wall_clock64();
#endif
    if constexpr (SOC) backward_rhs();
    int n_tries = 0;
    bool deferred = false;
    for (int attempt = resume ? 1 : 0; !SOC; ++attempt) {
        ++n_tries;
#ifdef NLOT_PHASE_PROF
        PROF_T(ta);
        ++n_att;
#endif
        if (attempt > 0) {
            if constexpr (RESTO) add_dw_resto(dw_in_hg, dw);
            else add_dw(dw - dw_in_hg);
            dw_in_hg = dw;
        }
#ifdef NLOT_PHASE_PROF
        PROF_T(tb);
        t_build += tb - ta;
#endif
        fail = backward();
#ifdef NLOT_PHASE_PROF
        t_back += wall_clock64() - tb;
#endif
        if (!fail || mode != MODE_NEWTON || fixed) break;
        dw = dw == 0.0 ? (last_dw == 0.0 ? 1e-4 : fmax(1e-20, last_dw / 3.0)) : dw * (last_dw == 0.0 ? 100.0 : 8.0);
        if (dw > 1e40) break;
        // attempt cap: a wrong inertia after max_tries factorisations in this launch continues in the next global
        // step's launch, so one instance's long delta_w sequence does not hold the whole launch (restoration solves
        // too: their chain joins the main stream before the second value launch)
        if (n_tries >= max_tries && (int)SC(SC_PHASE) == PH_EVAL) {
            deferred = true;
            break;
        }
    }
#ifdef NLOT_PHASE_PROF
    PROF_T(tr1);
#endif
    if (diag && l == 0 && !SOC && !RESTO && mode == MODE_NEWTON) {  // diagnostics (CSET [8..11))
        atomicAdd(diag, n_tries);
        atomicMax(diag + 1, n_tries);
        if (n_tries > 1) atomicAdd(diag + 2, 1);
    }
    if (diag && l == 0 && RESTO) atomicMax(diag, n_tries);  // restoration solves: most factorisations (CSET [15])
    if (deferred) {  // SC_RIC stays 1: k_iter_b (k_resto_b) and k_accept pass the instance by, k_iter_a lists it
                     // again (k_resto_a keeps its stages)
        if (l == 0) {
            SC(SC_RETRY) = dw;
            SC(SC_DWHG) = dw_in_hg;
        }
        return;
    }
    if (fail) {
        __syncthreads();
        if (l == 0) {
            if (fixed) {
                SC(SC_RIC) = 4;  // the correction's solve failed: k_iter_b resumes the backtracking
            } else if (mode == MODE_NEWTON) {
                SC(SC_STATUS) = NLOT_NUMERIC;
                SC(SC_PHASE) = PH_DONE;
                SC(SC_RIC) = 0;
            } else {
                SC(SC_RIC) = 3;
            }
        }
        return;
    }

#ifdef NLOT_RIC_PROF
    constexpr int rpk = SOC ? 1 : RESTO ? 2 : 0;
    long long rpt = wall_clock64();
    if (l == 0 && mode == MODE_NEWTON) {
        atomicAdd(&g_ric_prof[rpk][0], (unsigned long long)(rpt - rp0));
        atomicAdd(&g_ric_prof[rpk][4], 1ull);
    }
    auto rp_mark = [&](int i) {
        const long long t = wall_clock64();
        if (l == 0 && mode == MODE_NEWTON) atomicAdd(&g_ric_prof[rpk][i], (unsigned long long)(t - rpt));
        rpt = t;
    };
#else
    auto rp_mark = [](int) {};
#endif
    // forward sweep.  (F1) closed-loop maps per knot, in parallel over knots: row i of stage k's phi block is
    // [Phi_i | off_0,i off_1,i] with Phi = A + B K, off_r = c + B (k_r + Kn nu_r); the slot's [A B 0 | c] stays, so a
    // second-order correction (same A, B, K: the same Phi) recomputes the offsets only, and k_iter_a rebuilds only c
    static_assert(NU + 1 == NV, "slack is the last control column");
    constexpr int PR = NX + 2;  // phi row: Phi_i | off_0,i | off_1,i
    for (int k = l; k < N; k += G) {
        double* slot = SL + (size_t)k * SLOT;
        double* ph = &AT(phi, (size_t)k * NX * PR);
        const double* GN = slot + sGN;
        double dv[2][NU], Kt[NU][NX];
#pragma unroll
        for (int rr = 0; rr < 2; ++rr)
#pragma unroll
            for (int v = 0; v < NU; ++v) {
                double t = GN[(NX + rr) * NV + v];
#pragma unroll
                for (int cc = 0; cc < NC; ++cc) t += GN[(NX + 2 + cc) * NV + v] * nu_[rr][cc];
                dv[rr][v] = t;
            }
#pragma unroll
        for (int v = 0; v < NU; ++v)
#pragma unroll
            for (int c = 0; c < NX; ++c) Kt[v][c] = GN[c * NV + v];
        // every row of [A B | c] in registers before the first store (the stores into phi might alias the slot for
        // the compiler: row by row, each row was a dependent HBM round trip; ~4-10 us each under the bulk's load)
        double ab[NX][NX + NU + 1];
#pragma unroll
        for (int i = 0; i < NX; ++i) {
            const double* r_ = slot + sAB + i * NAB;
#pragma unroll
            for (int c = 0; c < NX + NU; ++c) ab[i][c] = (SOC && c < NX) ? 0.0 : r_[c];
            ab[i][NX + NU] = r_[NZ];
        }
#pragma unroll
        for (int i = 0; i < NX; ++i) {
            double* pr = ph + i * PR;
            const double* Bi = &ab[i][NX];
            double o0 = ab[i][NX + NU], o1 = ab[i][NX + NU];
#pragma unroll
            for (int v = 0; v < NU; ++v) {
                o0 += Bi[v] * dv[0][v];
                o1 += Bi[v] * dv[1][v];
            }
            if constexpr (!SOC) {
#pragma unroll
                for (int c = 0; c < NX; ++c) {
                    double t = ab[i][c];
#pragma unroll
                    for (int v = 0; v < NU; ++v) t += Bi[v] * Kt[v][c];
                    pr[c] = t;
                }
            }
            pr[NX] = o0;
            pr[NX + 1] = o1;
        }
        if constexpr (RESTO) {  // soft dynamics rows: x_{k+1} = S K^-1 S^-1 (Phi x_k + off - D (p + G nu))
            const double* v1 = &AT(vf, (k + 1) * VF);
            double Dd[NX], Sd[NX], K[NX][NX], w[NX], col[NX];
#pragma unroll
            for (int i = 0; i < NX; ++i) {
                Dd[i] = AT(dsoft, NX + k * NX + i);
                Sd[i] = sqrt(Dd[i]);
                double t = v1[i * NCOL + NX];
#pragma unroll
                for (int cc = 0; cc < NC; ++cc) t += v1[i * NCOL + NX + 2 + cc] * nu_[0][cc];
                w[i] = t;
            }
#pragma unroll
            for (int i = 0; i < NX; ++i)
#pragma unroll
                for (int c = 0; c < NX; ++c) K[i][c] = (i == c ? 1.0 : 0.0) + Sd[i] * v1[i * NCOL + c] * Sd[c];
            int perm[NX], nneg;
            ldl_factor<NX>(K, NX, perm, &nneg);  // positive definite: the backward sweep factorised it
#pragma unroll 1
            for (int c = 0; c <= NX; ++c) {  // the NX columns of Phi, then the offset
#pragma unroll
                for (int i = 0; i < NX; ++i) {
                    const double y = ph[i * PR + c];
                    col[i] = (c < NX ? y : y - Dd[i] * w[i]) / Sd[i];
                }
                ldl_solve1<NX>(K, NX, perm, col);
#pragma unroll
                for (int i = 0; i < NX; ++i) ph[i * PR + c] = Sd[i] * col[i];
            }
        }
    }
    __syncthreads();
    rp_mark(1);
    // (F2) the chain dx_{k+1} = Phi_k dx_k + off_k: lane i < NX of the group carries dx[i] of both
    //      right-hand sides; the other components arrive by group shuffles; rows prefetched a stage ahead
    double* dXo[2] = {&AT(dX, 0), &AT(dX2, 0)};
    double* dUo[2] = {&AT(dU, 0), &AT(dU2, 0)};
    double* dSo[2] = {&AT(dS, 0), &AT(dS2, 0)};
    {
        const int li = l < NX ? l : 0;
        double xv = 0;
        if constexpr (RESTO) {  // soft initial-state rows: x_0 = S K^-1 S^-1 (dx0 - D (p_0 + G_0 nu))
            const double* v0 = &AT(vf, 0);
            double Dd[NX], Sd[NX], K[NX][NX], col[NX];
#pragma unroll
            for (int i = 0; i < NX; ++i) {
                Dd[i] = AT(dsoft, i);
                Sd[i] = sqrt(Dd[i]);
                double t = v0[i * NCOL + NX];
#pragma unroll
                for (int cc = 0; cc < NC; ++cc) t += v0[i * NCOL + NX + 2 + cc] * nu_[0][cc];
                col[i] = (dx0[i] - Dd[i] * t) / Sd[i];
            }
#pragma unroll
            for (int i = 0; i < NX; ++i)
#pragma unroll
                for (int c = 0; c < NX; ++c) K[i][c] = (i == c ? 1.0 : 0.0) + Sd[i] * v0[i * NCOL + c] * Sd[c];
            int perm[NX], nneg;
            ldl_factor<NX>(K, NX, perm, &nneg);
            ldl_solve1<NX>(K, NX, perm, col);
#pragma unroll
            for (int i = 0; i < NX; ++i) dx0[i] = Sd[i] * col[i];
        }
#pragma unroll
        for (int i = 0; i < NX; ++i)
            if (i == l) xv = dx0[i];
        double x[2] = {xv, xv};
        constexpr int FRING = 4;  // rows of the next FRING knots in flight (HBM latency)
        double row[NX + 2], rr_[FRING][NX + 2];
        auto load_row = [&](int k, double* rw) {
            if (k >= N) return;
            const double* sl = &AT(phi, ((size_t)k * NX + li) * PR);
#pragma unroll
            for (int c = 0; c < NX + 2; ++c) rw[c] = sl[c];
        };
#pragma unroll
        for (int r = 0; r < FRING; ++r) load_row(r, rr_[r]);
        for (int k = 0; k < N; ++k) {
#pragma unroll
            for (int c = 0; c < NX + 2; ++c) row[c] = rr_[0][c];
#pragma unroll
            for (int r = 0; r + 1 < FRING; ++r)
#pragma unroll
                for (int c = 0; c < NX + 2; ++c) rr_[r][c] = rr_[r + 1][c];
            load_row(k + FRING, rr_[FRING - 1]);
            if (l < NX) {
                dXo[0][k * NX + l] = x[0];
                if (nr > 1) dXo[1][k * NX + l] = x[1];
            }
#pragma unroll
            for (int rr = 0; rr < 2; ++rr) {
                double t = row[NX + rr];
#pragma unroll
                for (int c = 0; c < NX; ++c) t += row[c] * __shfl(x[rr], gb + c);
                x[rr] = t;
            }
        }
        if (l < NX) {
            dXo[0][N * NX + l] = x[0];
            if (nr > 1) dXo[1][N * NX + l] = x[1];
        }
    }
    __syncthreads();  // dX visible to every lane
    rp_mark(2);
    // (F3) controls and slacks in parallel over knots: dv_k = k_r + K dx_k + Kn nu_r
    // (both right-hand sides per knot: the gains and both dx_k loaded once, before the first store)
    for (int k = l; k <= N; k += G) {
        const double* GN = SL + (size_t)k * SLOT + sGN;
        double gn[NCOL * NV], dxk[2][NX];
#pragma unroll
        for (int e = 0; e < NCOL * NV; ++e) gn[e] = GN[e];
#pragma unroll
        for (int rr = 0; rr < 2; ++rr)
#pragma unroll
            for (int c = 0; c < NX; ++c) dxk[rr][c] = rr < nr ? dXo[rr][k * NX + c] : 0.0;
#pragma unroll
        for (int rr = 0; rr < 2; ++rr) {
            if (rr >= nr) break;
            double dv[NV];
#pragma unroll
            for (int v = 0; v < NV; ++v) {
                double t = gn[(NX + rr) * NV + v];
#pragma unroll
                for (int c = 0; c < NX; ++c) t += gn[c * NV + v] * dxk[rr][c];
#pragma unroll
                for (int cc = 0; cc < NC; ++cc) t += gn[(NX + 2 + cc) * NV + v] * nu_[rr][cc];
                dv[v] = t;
            }
            if (k < N)
#pragma unroll
                for (int v = 0; v < NU; ++v) dUo[rr][k * NU + v] = dv[v];
            if (ns) dSo[rr][k] = k < N ? dv[NU] : dv[0];
        }
    }
    // equality multipliers in parallel over knots: y_k = -grad V_{k+1}(dx_{k+1}) - M_k' dx_k,
    // y_init = -grad V_0(dx_0)
    double* yio[2] = {&AT(yi_n, 0), &AT(yi2, 0)};
    double* yko[2] = {&AT(yk_n, 0), &AT(yk2, 0)};
    double* yto[2] = {&AT(yt_n, 0), &AT(yt2, 0)};
    // (both right-hand sides per knot: the value function block, M and both dx loaded once, before the first store)
    for (int k = l - 1; k < N; k += G) {
        const double* v1 = &AT(vf, (k + 1) * VF);
        double vb[NX * NCOL], xn[2][NX], d01[2][2], s0[4];
#pragma unroll
        for (int e = 0; e < NX * NCOL; ++e) vb[e] = v1[e];
#pragma unroll
        for (int rr = 0; rr < 2; ++rr) {
#pragma unroll
            for (int c = 0; c < NX; ++c) xn[rr][c] = rr < nr ? dXo[rr][(k + 1) * NX + c] : 0.0;
            d01[rr][0] = (rr < nr && k >= 0) ? dXo[rr][k * NX] : 0.0;
            d01[rr][1] = (rr < nr && k >= 0) ? dXo[rr][k * NX + 1] : 0.0;
        }
#pragma unroll
        for (int e = 0; e < 4; ++e) s0[e] = k >= 0 ? SL[(size_t)k * SLOT + sM + e] : 0.0;
#pragma unroll
        for (int rr = 0; rr < 2; ++rr) {
            if (rr >= nr) break;
            double mx0 = 0, mx1 = 0;
            if (k >= 0) {
                const double d0 = d01[rr][0], d1 = d01[rr][1];
                mx0 = s0[0] * d0 + s0[2] * d1;
                mx1 = s0[1] * d0 + s0[3] * d1;
            }
#pragma unroll
            for (int i = 0; i < NX; ++i) {
                double t = vb[i * NCOL + NX + rr];
#pragma unroll
                for (int c = 0; c < NX; ++c) t += vb[i * NCOL + c] * xn[rr][c];
#pragma unroll
                for (int cc = 0; cc < NC; ++cc) t += vb[i * NCOL + NX + 2 + cc] * nu_[rr][cc];
                if (k < 0) {
                    yio[rr][i] = -t;
                } else {
                    const double mt = i == 0 ? mx0 : (i == 1 ? mx1 : 0.0);
                    yko[rr][k * NX + i] = -t - mt;
                }
            }
        }
    }
#pragma unroll
    for (int rr = 0; rr < 2; ++rr) {
        if (rr >= nr) break;
        if (l < nc) {
            double v = 0;
#pragma unroll
            for (int cc = 0; cc < NC; ++cc)
                if (cc == l) v = nu_[rr][cc];
            yto[rr][l] = v;
        }
    }
    __syncthreads();
    rp_mark(3);
#ifdef NLOT_PHASE_PROF
    if (b == 0 && l == 0 && SC(SC_ITERS) < 8)
        printf("RICG it %d attempts %d build %lld backward %lld forward %lld total %lld (x10ns)\n", (int)SC(SC_ITERS),
               n_att, t_build, t_back, wall_clock64() - tr1, wall_clock64() - tr0);
#endif
    if (l == 0) {
        if (dw > 0.0 && mode == MODE_NEWTON && !fixed) SC(SC_DWLAST) = dw;
        SC(SC_RETRY) = -1.0;
        SC(SC_DW) = dw;
        SC(SC_RIC) = 2;
    }
    };
    if constexpr (RESTO) {
        for (int si = blockIdx.x * R::IPW + grp; si < nlist; si += gridDim.x * R::IPW) {
            body(si);
            __syncthreads();
        }
    } else {
        const int si = blockIdx.x * R::IPW + grp;
        if (si < nlist) body(si);
    }
}

// ---------------------------------------------------------------------------------------------
// kernels (one 64-lane workgroup = one instance; grid = active instances)
// ---------------------------------------------------------------------------------------------
static __global__ __launch_bounds__(64) void k_init_state(const NlotProblem* __restrict__ pp_, const Dims* __restrict__ dd_, NlotSolverOptions o, Ws ws,
                                                   const double* __restrict__ x0, const double* __restrict__ xg,
                                                   const double* __restrict__ Xinit, const int* __restrict__ adm,
                                                   const int* __restrict__ cadm) {
    const NlotProblem& p = *pp_;
    const Dims& dm = *dd_;
    const int lane = threadIdx.x;
    // the first fill (adm = NULL): slot i holds instance i; an admission: the slots k_admit appended to the next
    // active list at adm[cadm[13] ..], holding the instances k_admit assigned (ws.sinst).  k_admit admitted
    // cadm[2] - cadm[13] of them (fewer than the host's grid on a shortfall, which it flags): blocks past that exit
    if (adm && (int)blockIdx.x >= cadm[2] - cadm[13]) return;
    const int b = adm ? adm[cadm[13] + (int)blockIdx.x] : (int)blockIdx.x;
    const int64_t inst = adm ? ws.sinst[b] : b;
    const int N = dm.N, nx = dm.nx, nu = dm.nu, M = dm.M;
    const double k1 = o.bound_push, k2 = o.bound_frac;
    for (int i = lane; i < nx; i += 64) {
        AT(x0s, i) = x0[inst * nx + i];
        AT(xgs, i) = xg[inst * nx + i];
    }
    for (int e = lane; e < (N + 1) * nx; e += 64) {
        const int k = e / nx, i = e % nx;
        const double v = Xinit ? Xinit[((size_t)inst * (N + 1) + k) * nx + i]
                               : x0[inst * nx + i] + (xg[inst * nx + i] - x0[inst * nx + i]) * ((double)k / (double)N);
        AT(X, e) = v;  // LinearInitializer (trajectory_initialization.py:54-55)
        AT(dX, e) = 0.0;
    }
    for (int e = lane; e < N * nu; e += 64) {
        const int i = e % nu;
        const double lo = p.umin[i], hi = p.umax[i];
        const double pl = fmin(k1 * fmax(1.0, fabs(lo)), k2 * (hi - lo));
        const double pu = fmin(k1 * fmax(1.0, fabs(hi)), k2 * (hi - lo));
        const double pushed = fmin(fmax(0.0, lo + pl), hi - pu);
        // general bounds: U is free (Opti's initial value 0) and its row slack starts pushed into the bounds
        AT(U, e) = dm.gcb ? 0.0 : pushed;
        AT(zl, e) = 1.0;
        AT(zu, e) = 1.0;
        AT(dU, e) = 0.0;
        if (dm.gcb) {
            AT(sb, e) = pushed;
            AT(yb, e) = 0.0;
            AT(dsb, e) = 0.0;
        }
    }
    for (int k = lane; k <= N; k += 64) {
        AT(S, k) = (dm.ns && !dm.gcb) ? fmax(0.0, k1) : 0.0;
        AT(zs, k) = 1.0;
        AT(dS, k) = 0.0;
        if (dm.gcb && dm.ns) {  // slack_bound_push of the row d(x0) = S_k = 0
            AT(sb, N * nu + k) = fmax(0.0, k1);
            AT(yb, N * nu + k) = 0.0;
            AT(dsb, N * nu + k) = 0.0;
        }
    }
    for (int q = lane; q < (N + 1) * M; q += 64) {
        AT(vt, q) = 1.0;
        AT(dT, q) = 0.0;
    }
    if (lane == 0) {
        SC(SC_MU) = o.mu_init;
        SC(SC_TAU) = fmax(0.99, 1.0 - o.mu_init);
        SC(SC_DWLAST) = 0;
        SC(SC_STATUS) = -1;
        SC(SC_ITERS) = 0;
        SC(SC_PHASE) = PH_INIT;
        SC(SC_ACCSLOT) = -1;
        SC(SC_NFILT) = 0;
        SC(SC_E0) = 0;
        SC(SC_SOCK) = 0;
        SC(SC_RICFIX) = -1;
        SC(SC_WD) = 0;
        SC(SC_WDSHORT) = 0;
        SC(SC_WDTRIAL) = 0;
        SC(SC_TINY) = 0;
        SC(SC_TINYLAST) = 0;
        SC(SC_LASTREJF) = 0;
        SC(SC_NFREJ) = 0;
        SC(SC_NFRES) = 0;
        SC(SC_INSOFT) = 0;
        SC(SC_SOFTCNT) = 0;
        SC(SC_RESTO) = 0;
        SC(SC_RNFILT) = 0;
        SC(SC_NRESTO) = 0;
        SC(SC_RETRY) = -1.0;
        if (!adm) {
            ws.act[0][b] = b;
            ws.sinst[b] = b;
        }
    }
}

// End of global step s (one wave, after k_accept): the step's counter sets go to the host's pinned ring slot and the
// free-slot count / admission flag to its flag pair (plain vector stores into mapped host memory, visible once the
// stream's synchronisation sees the kernel complete); then the finished set C = cnt + CSET q is cleared for step s + 1
// (its Cn) and the next step's set takes its early value launch's base, Cn[14] = Cn[1] (the candidates listed up to
// now).  One launch in place of a D2H copy, a fill and a D2D copy per step (each a queue packet of its own).
static __global__ __launch_bounds__(64) void k_step_end(int* __restrict__ cnt, int q, int* __restrict__ ring,
                                                        int* __restrict__ hflag) {
    const int l = threadIdx.x;
    const int v = l < 2 * CSET + 2 ? cnt[l] : 0;
    const int base = __shfl(v, CSET * (q ^ 1) + 1);
    if (l < 2 * CSET) ring[l] = v;
    else if (l < 2 * CSET + 2) hflag[l - 2 * CSET] = v;
    if (l >= CSET * q && l < CSET * q + CSET) cnt[l] = 0;
    else if (l == CSET * (q ^ 1) + 14) cnt[l] = base;
}

// continuous batching: instances first .. first + n - 1 take the n most recently freed slots, which join the active
// list of the next step (its count cnt[2]; the position they start at goes to cnt[13] for k_init_state).  The host
// asks for n <= the free slots (capacity - next active count); a shortfall sets the error flag cnt[2 CSET + 1].
static __global__ __launch_bounds__(1024) void k_admit(int* __restrict__ act, int* __restrict__ cnt, int* __restrict__ sinst,
                                                        const int* __restrict__ freel, int* __restrict__ gcnt, int first,
                                                        int n) {
    const int base = cnt[2], nf = gcnt[0];
    if (nf < n) {
        if (threadIdx.x == 0) gcnt[1] = GRID_ADMIT;
        n = nf;
    }
    for (int t = threadIdx.x; t < n; t += blockDim.x) {
        const int slot = freel[nf - n + t];
        act[base + t] = slot;
        sinst[slot] = first + t;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        cnt[2] = base + n;
        cnt[13] = base;
        gcnt[0] = nf - n;
    }
}

// number of step lengths of a later line-search round starting at alpha a: a, a/2, ... while >= alpha_min,
// at most nspec (speculative backtracking: the same accepted alpha as sequential halving, because the
// acceptance test of one candidate does not depend on the others; the first round tries alpha_max alone)
__device__ __forceinline__ int n_later(double a, double amin, int nspec) {
    int n = 1;
    for (int j = 1; j < nspec; ++j) {
        a *= 0.5;
        if (a < amin) break;
        ++n;
    }
    return n;
}

// Corners of X + a_c dX (a_c = a0 2^-c, c < ncand) of instance b, appended to a compacted point list:
// the evaluation list pts (!trial; a0 = 0, ncand = 1) or the trial list tp.  Without a learned SDF there
// are no lists: only the candidate count is recorded.  cnt: the counters of
// the global step that evaluates them.  Called with uniform arguments by the kernel that moves the
// instance into the phase needing them: k_iter_b (first line-search round), k_accept (accepted: the new
// iterate; rejected: the next round), k_points (first step).  Lane = knot: one sincos per knot.
__device__ void emit_points(const NlotProblem& p, const Dims& dm, const Ws& ws, int b, int lane, int* cnt,
                            bool trial, float* tp, int ncand, double a0) {
    if (!ws.pts) {
        if (lane == 0) SC(SC_NCAND) = ncand;
        return;
    }
    int rank = 0;
    if (lane == 0) {
        rank = atomicAdd(&cnt[trial ? 1 : 0], ncand);
        SC(SC_RANK) = rank;
        SC(SC_NCAND) = ncand;
        if (!trial && ws.tsrc) ws.tsrc[rank] = (int)SC(SC_ACCSLOT);
    }
    rank = __shfl(rank, 0);
    const int nx = dm.nx, nb = dm.nb;
    float* dst = trial ? tp : ws.pts;
    for (int cnd = 0; cnd < ncand; ++cnd) {
        const double al = trial ? ldexp(a0, -cnd) : 0.0;
        float* o0 = dst + (size_t)(rank + cnd) * dm.ppk * (dm.N + 1) * 2;
        for (int k = lane; k <= dm.N; k += 64) {
            const double x = AT(X, k * nx) + al * AT(dX, k * nx);
            const double y = AT(X, k * nx + 1) + al * AT(dX, k * nx + 1);
            float* o = o0 + (size_t)k * nb * 2;
            if (p.shape == NLOT_SHAPE_DOT) {
                o[0] = (float)x;  // CasADi double -> fp32 (gen/nn_sdf.cpp)
                o[1] = (float)y;
            } else {
                const double th = AT(X, k * nx + 2) + al * AT(dX, k * nx + 2);
                double sn, cs;
                sincos(th, &sn, &cs);
                for (int i = 0; i < nb; ++i) {
                    const double bx = p.body[i][0], by = p.body[i][1];
                    o[2 * i] = (float)(x + cs * bx - sn * by);
                    o[2 * i + 1] = (float)(y + sn * bx + cs * by);
                }
            }
        }
    }
}

// first global step: the corners of every instance (phase INIT)
static __global__ __launch_bounds__(64) void k_points(const NlotProblem* __restrict__ pp_, const Dims* __restrict__ dd_,
                                               const Ws* __restrict__ ws_, const int* __restrict__ active, int* cnt) {
    const Ws& ws = *ws_;
    grid_guard(ws, cnt[2], 1, GRID_ACTIVE);
    if ((int)blockIdx.x >= cnt[2]) return;  // the host's count may exceed the device's (k_admit shortfall)
    const int b = active[blockIdx.x];
    if ((int)SC(SC_PHASE) != PH_INIT) return;
    emit_points(*pp_, *dd_, ws, b, threadIdx.x, cnt, false, nullptr, 1, 0.0);
}

__device__ inline double frac_to_bound(double sl, double dsl, double tau, double amax) {
    if (dsl < 0) {
        const double a = -tau * sl / dsl;
        if (a < amax) return a;
    }
    return amax;
}
__device__ inline int cmp_le(double lhs, double rhs, double bas) {
    return lhs - rhs <= 10.0 * 2.220446049250313e-16 * fabs(bas);
}

// objective at X + al dX (runner.py:80-96), wave-parallel
__device__ inline double objective_w(const NlotProblem& p, const Dims& dm, const Ws& ws, int b, int lane, double al) {
    const int nx = dm.nx, nu = dm.nu, N = dm.N;
    double f = 0;
    for (int k = lane; k < N; k += 64) {
        const double dx = (AT(X, (k + 1) * nx) + al * AT(dX, (k + 1) * nx)) - (AT(X, k * nx) + al * AT(dX, k * nx));
        const double dy = (AT(X, (k + 1) * nx + 1) + al * AT(dX, (k + 1) * nx + 1)) -
                          (AT(X, k * nx + 1) + al * AT(dX, k * nx + 1));
        f += sqrt(dx * dx + dy * dy + p.path_eps);
    }
    double sq = 0, uq = 0;
    if (p.use_slack)
        for (int k = lane; k <= N; k += 64) {
            const double s = AT(S, k) + al * AT(dS, k);
            sq += s * s;
        }
    if (p.use_smooth)
        for (int e = lane; e < (N - 1) * nu; e += 64) {
            const double u = AT(U, e) + al * AT(dU, e);
            uq += u * u;
        }
    return wsum(f) + p.slack_penalty * wsum(sq) + p.smooth_weight * wsum(uq);
}

// A filter update by the whole wave (uniform control flow, every lane calls): drop the entries (ft, fp) with
// ft >= a && fp >= c (the new entry dominates them), keep the rest in order, append (a, c), forgetting the oldest entry
// at capacity; the filter's count lives in SC(sc_n).  The kept entries of each 64-entry chunk move down in one
// ballot-compacted store (destinations never pass the chunk's own entries, so a chunk's loads complete before any store
// reaches them; later chunks are not touched), instead of lane 0's serial load -> store chain (one memory round trip
// per entry).  cs (may be null): the step's counter set — [11] peak size, [12] entries forgotten.  Returns the new count.
__device__ inline int filter_update(const Ws& ws, int b, double* filt, int sc_n, double a, double c, int* cs, int lane) {
    const int nfc = (int)SC(sc_n);
    int w = 0;
    for (int base = 0; base < nfc; base += 64) {
        const int i = base + lane;
        double ft = 0.0, fp = 0.0;
        bool keep = false;
        if (i < nfc) {
            ft = filt[2 * i];
            fp = filt[2 * i + 1];
            keep = !(ft >= a && fp >= c);
        }
        const uint64_t m = __ballot(keep);
        if (keep) {
            const int d = w + __popcll(m & ((1ull << lane) - 1ull));
            filt[2 * d] = ft;
            filt[2 * d + 1] = fp;
        }
        w += __popcll(m);
    }
    wsync();
    if (lane == 0) {
        if (w == FILT_MAX) {  // never reached on the bench workloads (NlotSolveStats.filter_forgotten)
            for (int i = 0; i + 1 < FILT_MAX; ++i) {
                filt[2 * i] = filt[2 * (i + 1)];
                filt[2 * i + 1] = filt[2 * (i + 1) + 1];
            }
            w--;
            if (cs) atomicAdd(cs + 12, 1);
        }
        filt[2 * w] = a;
        filt[2 * w + 1] = c;
        SC(sc_n) = w + 1;
        if (cs) atomicMax(cs + 11, w + 1);
    }
    if (w == FILT_MAX) w--;
    wsync();
    return w + 1;
}

// IPOPT filter augmentation with the iterate's (theta, phi): margins gamma_theta = 1e-5, gamma_phi = 1e-8.  filt: the
// original problem's filter (count SC_NFILT) or the restoration's (SC_RNFILT).  Whole wave.
__device__ inline void filter_add(const Ws& ws, int b, double* filt, int sc_n, double theta, double phi, int* cs,
                                  int lane) {
    const double gt = 1e-5, gp = 1e-8, ntv = (1.0 - gt) * theta, npv = phi - gp * theta;
    filter_update(ws, b, filt, sc_n, ntv, npv, cs, lane);
}

// The line search of the original problem failed and the soft restoration did not help: IPOPT's feasibility
// restoration phase (BacktrackingLineSearch::FindAcceptableTrialPoint).  At an almost feasible point (theta <=
// 1e-2 tol) IPOPT does not restore: without an acceptable iterate to fall back to it stops with Restoration_Failed.
// Otherwise the current point enters the filter with the line search's reference values and the instance moves to
// PH_RINIT: the next step's full launch evaluates its corners (emitted here into that step's list, counters
// cnt_next), and k_resto_a initialises the restoration problem there.  Returns the new phase (uniform).
__device__ int resto_enter(const NlotSolverOptions& o, const NlotProblem& p, const Dims& dm, const Ws& ws, int b,
                           int lane, int* cnt_next) {
    const double th = SC(SC_THETA);
    wsync();
    if (th <= 1e-2 * o.tol) {
        if (lane == 0) {
            SC(SC_STATUS) = NLOT_RESTO_FAILED;
            SC(SC_PHASE) = PH_DONE;
        }
        wsync();
        return PH_DONE;
    }
    filter_add(ws, b, &AT(filt, 0), SC_NFILT, th, SC(SC_PHI), cnt_next, lane);
    if (lane == 0) {
        SC(SC_RESTO) = 1;
        SC(SC_PHASE) = PH_RINIT;
        SC(SC_ACCSLOT) = -1;
    }
    wsync();
    emit_points(p, dm, ws, b, lane, cnt_next, false, nullptr, 1, 0.0);
    return PH_RINIT;
}

// The backtracking line search of the original problem ended (alpha < alpha_min): IPOPT TrySoftRestoStep first
// (phase PH_SOFT1: the step min(alpha_max, alpha_z) for both primal and dual variables, one trial point emitted
// into (tp, cnt)), else the restoration phase, else (resto = 0) NLOT_LS_FAILED.  Returns the new phase.
__device__ int ls_failed(const NlotSolverOptions& o, const NlotProblem& p, const Dims& dm, const Ws& ws, int b, int lane,
                         float* tp, int* cnt, int* cnt_next) {
    if (!o.resto) {
        wsync();
        if (lane == 0) {
            SC(SC_STATUS) = NLOT_LS_FAILED;
            SC(SC_PHASE) = PH_DONE;
        }
        wsync();
        return PH_DONE;
    }
    if (o.soft_resto_pderror_reduction_factor > 0) {
        const double a = fmin(SC(SC_AMAX), SC(SC_AZ));
        wsync();
        if (lane == 0) {
            SC(SC_ALPHA) = a;
            SC(SC_PHASE) = PH_SOFT1;
        }
        wsync();
        emit_points(p, dm, ws, b, lane, cnt, true, tp, 1, a);
        return PH_SOFT1;
    }
    return resto_enter(o, p, dm, ws, b, lane, cnt_next);
}

// k_iter_a: evaluation, optimality test, barrier update, then the stage matrices of the Newton system
// (k_ric solves it).  pass (IterPass): INIT = slack push and the least-squares multiplier system of the instances in
// INIT (their first step); SOC = the second-order corrections' stages only (side stream, at the start of the step: they
// need no MLP evaluation); EVAL = everything but the corrections; ALL = both.  (INIT instances first take their
// least-squares multipliers from k_ric's solve).
#ifdef NLOT_KPROF
// tuning builds only: phase times of the per-instance kernels summed over their waves (wall clock, 10 ns), [kernel]
// [phase]; slot 15 counts the waves that reached the last mark; printed by run()
__device__ unsigned long long g_kprof[4][16];
#define KPROF_INIT long long kp_t = wall_clock64()
#define KPROF(kid, ph)                                                                              \
    do {                                                                                             \
        const long long kp_n = wall_clock64();                                                       \
        if (threadIdx.x == 0) atomicAdd(&g_kprof[kid][ph], (unsigned long long)(kp_n - kp_t));     \
        kp_t = kp_n;                                                                                 \
    } while (0)
#define KPROF_COUNT(kid) \
    if (threadIdx.x == 0) atomicAdd(&g_kprof[kid][15], 1ull)
#else
#define KPROF_INIT
#define KPROF(kid, ph)
#define KPROF_COUNT(kid)
#endif
template <int DYN>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(NLOT_WPE_A))) void k_iter_a(const NlotProblem* __restrict__ pp_, const Dims* __restrict__ dd_, NlotSolverOptions o, const Ws* __restrict__ ws_,
                                               const int* __restrict__ active, const double* __restrict__ x0,
                                               const double* __restrict__ xg, int pass, int* cnt, int* cnt_next) {
    const bool init_pass = pass == PASS_INIT;
    grid_guard(*ws_, cnt[2], 1, GRID_ACTIVE);
    if ((int)blockIdx.x >= cnt[2]) return;  // grid sized by a stale (larger) host count: steps run ahead of the host
    const NlotProblem& p = *pp_;
    const Dims& dm = *dd_;
    const Ws& ws = *ws_;
    using SV = Solver<DYN>;
    constexpr int NX = SV::NX, NU = SV::NU;
    const int b = active[blockIdx.x], lane = threadIdx.x;
    if (SC(SC_RESTO) != 0.0) return;  // k_resto_a
    const int ph = (int)SC(SC_PHASE);
    if (ph != PH_INIT && ph != PH_EVAL && ph != PH_SOC && ph != PH_SOFT2) return;
    if (ph == PH_EVAL && SC(SC_RETRY) >= 0.0) {  // k_ric's inertia correction continues (attempt cap): stages kept
        if (lane == 0 && (pass == PASS_ALL || pass == PASS_EVAL)) ws.ricl[atomicAdd(&cnt[4], 1)] = b;
        return;
    }
    if (init_pass && ph != PH_INIT) return;
    if ((pass == PASS_SOC) != (ph == PH_SOC) && pass != PASS_ALL && !init_pass) return;
    double* SL = &AT(stg, 0);
    if (ph == PH_SOC) {
        // second-order correction: the same Newton matrix (the iteration's delta_w, no inertia loop) with the
        // corrected constraint residuals c_soc in rci/rcd/rct/rcq (written by k_accept)
        const double dw = SC(SC_DW), mu = SC(SC_MU);
        SV::template build_stages<false, true>(p, dm, ws, b, lane, MODE_NEWTON, dw, mu, 0.0, 1, SL);
        if (lane == 0) {
            SC(SC_RMU0) = mu;
            SC(SC_RMU1) = 0.0;
            SC(SC_RNR) = 1;
            SC(SC_USEQF) = 0.0;
            SC(SC_RICFIX) = dw;
            SC(SC_RIC) = 1;
            ws.socl[atomicAdd(&cnt[6], 1)] = b;  // k_ric<DYN, false, true>'s list (and the statistics)
        }
        return;
    }
    KPROF_INIT;
    const int N = dm.N, M = dm.M, nc = dm.nc;
    const int rank = (int)SC(SC_RANK);
    const double k1 = o.bound_push;
    const double* x0b = x0 + (size_t)b * NX;
    const double* xgb = xg + (size_t)b * NX;

    auto eval_knots = [&](bool with_hess) {
        for (int k = lane; k <= N; k += 64) {
            double xk[NX], d[MMAX], gk[MMAX][3], w[MMAX], Hw[6];
#pragma unroll
            for (int i = 0; i < NX; ++i) xk[i] = AT(X, k * NX + i);
#pragma unroll
            for (int j = 0; j < MMAX; ++j) w[j] = (with_hess && j < M) ? AT(yd, k * M + j) : 0.0;
            knot_eval(p, dm, ws, rank, k, xk, d, gk, w, with_hess ? Hw : nullptr);
#pragma unroll
            for (int j = 0; j < MMAX; ++j) {
                if (j >= M) break;
                AT(dv, k * M + j) = d[j] + (dm.sd ? AT(S, k) : 0.0);
#pragma unroll
                for (int a = 0; a < 3; ++a) AT(Jd, (k * M + j) * 3 + a) = gk[j][a];
            }
            if (with_hess)
                for (int q = 0; q < 6; ++q) AT(Hd, k * 6 + q) = Hw[q];
        }
        wsync();
    };
    const int ngb = dm.gcb ? dm.ngb : 0;  // bound rows (general bounds)
    auto zero_mults = [&]() {
        for (int i = lane; i < NX; i += 64) AT(yi, i) = 0;
        for (int i = lane; i < N * NX; i += 64) AT(yk, i) = 0;
        for (int i = lane; i < nc; i += 64) AT(yt, i) = 0;
        for (int q = lane; q < (N + 1) * M; q += 64) AT(yd, q) = 0;
        for (int q = lane; q < ngb; q += 64) AT(yb, q) = 0;
    };

    const double mu0 = SC(SC_MU);
    if (ph == PH_INIT && init_pass) {
        eval_knots(false);
        for (int q = lane; q < (N + 1) * M; q += 64) {
            AT(T, q) = fmax(AT(dv, q), k1);  // slack push
            AT(yd, q) = 0.0;
        }
        wsync();
        // least-squares equality multipliers (IPOPT LeastSquareMultipliers): the system, solved by k_ric
        SV::template build_stages<false>(p, dm, ws, b, lane, MODE_LSQ, 0.0, mu0, 0.0, 1, SL);
        if (lane == 0) {
            SC(SC_RMU0) = mu0;
            SC(SC_RMU1) = 0.0;
            SC(SC_RNR) = 1;
            SC(SC_RIC) = 1;
        }
        return;
    }
    if (ph == PH_INIT) {
        if ((int)SC(SC_RIC) == 2) {
            double ymax = 0;
            for (int k = lane; k <= N; k += 64)
                for (int j = 0; j < M; ++j) {
                    double w = 0;
                    for (int a = 0; a < 3 && a < NX; ++a) w += AT(Jd, (k * M + j) * 3 + a) * AT(dX, k * NX + a);
                    if (dm.sd) w += AT(dS, k);
                    const double v = w - AT(vt, k * M + j);
                    AT(yd, k * M + j) = v;
                    ymax = fmax(ymax, fabs(v));
                }
            for (int i = lane; i < NX; i += 64) ymax = fmax(ymax, fabs(AT(yi, i) = AT(yi_n, i)));
            for (int i = lane; i < N * NX; i += 64) ymax = fmax(ymax, fabs(AT(yk, i) = AT(yk_n, i)));
            for (int i = lane; i < nc; i += 64) ymax = fmax(ymax, fabs(AT(yt, i) = AT(yt_n, i)));
            // bound rows: y = J dz - (z_L - z_U), J the unit vector of the control / slack
            for (int q = lane; q < ngb; q += 64) {
                const double v = q < N * NU ? AT(dU, q) - (AT(zl, q) - AT(zu, q)) : AT(dS, q - N * NU) - AT(zs, q - N * NU);
                AT(yb, q) = v;
                ymax = fmax(ymax, fabs(v));
            }
            ymax = wmax(ymax);
            wsync();
            if (ymax > o.constr_mult_init_max) zero_mults();
        } else {
            zero_mults();
        }
        wsync();
        if (lane == 0) SC(SC_RIC) = 0;
    }
    KPROF(0, 0);  // entry, INIT work
    eval_knots(true);
    KPROF(0, 1);  // SDF chain rule at the corners
    // residuals c(x) (IPOPT sign)
    for (int i = lane; i < NX; i += 64) AT(rci, i) = AT(X, i) - x0b[i];
    for (int i = lane; i < nc; i += 64) AT(rct, i) = AT(X, N * NX + dm.tidx[i]) - xgb[dm.tidx[i]];
    for (int k = lane; k < N; k += 64) {
        double x[NX], u[NU], f[NX];
#pragma unroll
        for (int i = 0; i < NX; ++i) x[i] = AT(X, k * NX + i);
#pragma unroll
        for (int i = 0; i < NU; ++i) u[i] = AT(U, k * NU + i);
        Dyn<DYN>::f(x, u, p.wheelbase, f, p.dt);
#pragma unroll
        for (int i = 0; i < NX; ++i) AT(rcd, k * NX + i) = AT(X, (k + 1) * NX + i) - (x[i] + p.dt * f[i]);
    }
    chunked_update<4, 2>((N + 1) * M, lane, [&](int q, double* v) { v[0] = AT(dv, q); v[1] = AT(T, q); },
                         [&](int q, const double* v) { AT(rcq, q) = v[0] - v[1]; });
    for (int q = lane; q < ngb; q += 64)  // bound rows U - sb, S - sb
        AT(rcb, q) = (q < N * NU ? AT(U, q) : AT(S, q - N * NU)) - AT(sb, q);
    wsync();

    // the lane-strided sums below: every pass's first chunk loaded ahead (Pre), consumed in the same per-lane order
    auto theta_phi = [&](double mu, double* th, double* phv, double* fout = nullptr) {
        double t = 0, bar = 0, lin = 0;
        auto tsum = [&](int, const double* v) { t += fabs(v[0]); };
        chunked_update<4, 1>(NX, lane, [&](int i, double* v) { v[0] = AT(rci, i); }, tsum);
        chunked_update<4, 1>(nc, lane, [&](int i, double* v) { v[0] = AT(rct, i); }, tsum);
        chunked_update<4, 1>(N * NX, lane, [&](int i, double* v) { v[0] = AT(rcd, i); }, tsum);
        chunked_update<4, 2>((N + 1) * M, lane, [&](int q, double* v) { v[0] = AT(rcq, q); v[1] = AT(T, q); },
                             [&](int, const double* v) {
                                 t += fabs(v[0]);
                                 bar += log(v[1]);
                                 lin += v[1];
                             });
        chunked_update<4, 1>(N * NU, lane, [&](int e, double* v) { v[0] = BVU(e); },
                             [&](int e, const double* v) {
                                 const double u = v[0];
                                 bar += log(u - p.umin[e % NU]) + log(p.umax[e % NU] - u);
                             });
        if (dm.ns)
            chunked_update<4, 1>(N + 1, lane, [&](int k, double* v) { v[0] = BVS(k); },
                                 [&](int, const double* v) {
                                     bar += log(v[0]);
                                     lin += v[0];
                                 });
        chunked_update<4, 1>(ngb, lane, [&](int q, double* v) { v[0] = AT(rcb, q); }, tsum);
        *th = wsum(t);
        const double fo = objective_w(p, dm, ws, b, lane, 0.0);
        *phv = fo - mu * wsum(bar) + 1e-5 * mu * wsum(lin);
        if (fout) *fout = fo;
    };
    if (ph == PH_INIT) {
        double th0, p0;
        theta_phi(mu0, &th0, &p0);
        if (lane == 0) {
            SC(SC_THMAX) = 1e4 * fmax(1.0, th0);
            SC(SC_THMIN) = 1e-4 * fmax(1.0, th0);
            SC(SC_NFILT) = 0;
        }
    }

    KPROF(0, 2);  // residuals (and theta / phi at INIT)
    // ---- optimality measures (IPOPT scaled E_0 / E_mu) ----
    double dual = 0, primal = 0, c0 = 0, cmu = 0, cviol = 0, ysum = 0, zsum = 0, nzc = 0;
    double dsq = 0, psq = 0, csum = 0;  // quality-function oracle: ||grad L||^2, ||c, d - t||^2, sum z s
    double d1 = 0, p1 = 0;              // soft restoration: 1-norms of the dual and primal residuals
    // The passes below only read: their first chunks are all loaded here, ahead of the dual residuals' knot loop, and
    // consumed in the original order (Pre) — one memory round trip instead of one per pass (13 passes)
    const int nnu = N * NU;
    auto ld_bs = [&](int q, double* v) {  // bound-row slacks: y, z_L (z_S), z_U
        v[0] = AT(yb, q);
        v[1] = q < nnu ? AT(zl, q) : AT(zs, q - nnu);
        v[2] = q < nnu ? AT(zu, q) : 0.0;
    };
    auto ld_rci = [&](int i, double* v) { v[0] = AT(rci, i); };
    auto ld_rct = [&](int i, double* v) { v[0] = AT(rct, i); };
    auto ld_rcd = [&](int i, double* v) { v[0] = AT(rcd, i); };
    auto ld_rcq = [&](int q, double* v) { v[0] = AT(rcq, q); v[1] = AT(dv, q); };
    auto ld_rcb = [&](int q, double* v) { v[0] = AT(rcb, q); v[1] = q < nnu ? AT(U, q) : AT(S, q - nnu); };
    auto ld_cu = [&](int e, double* v) { v[0] = BVU(e); v[1] = AT(zl, e); v[2] = AT(zu, e); };
    auto ld_zs = [&](int k, double* v) { v[0] = AT(zs, k); v[1] = BVS(k); };
    auto ld_vt = [&](int q, double* v) { v[0] = AT(vt, q); v[1] = AT(T, q); };
    auto ld_yi = [&](int i, double* v) { v[0] = AT(yi, i); };
    auto ld_yk = [&](int i, double* v) { v[0] = AT(yk, i); };
    auto ld_yt = [&](int i, double* v) { v[0] = AT(yt, i); };
    auto ld_yd = [&](int q, double* v) { v[0] = AT(yd, q); };
    auto ld_yb = [&](int q, double* v) { v[0] = AT(yb, q); };
    Pre<3, 3> p_bs;
    Pre<1, 1> p_rci, p_rct, p_yi, p_yt, p_yd;
    Pre<4, 1> p_rcd, p_yk;
    Pre<1, 2> p_rcq, p_zs, p_vt;
    Pre<3, 2> p_rcb;
    Pre<2, 3> p_cu;
    Pre<3, 1> p_yb;
    p_bs.load(ngb, lane, ld_bs);
    p_rci.load(NX, lane, ld_rci);
    p_rct.load(nc, lane, ld_rct);
    p_rcd.load(N * NX, lane, ld_rcd);
    p_rcq.load((N + 1) * M, lane, ld_rcq);
    p_rcb.load(ngb, lane, ld_rcb);
    p_cu.load(N * NU, lane, ld_cu);
    if (dm.ns) p_zs.load(N + 1, lane, ld_zs);
    p_vt.load((N + 1) * M, lane, ld_vt);
    p_yi.load(NX, lane, ld_yi);
    p_yk.load(N * NX, lane, ld_yk);
    p_yt.load(nc, lane, ld_yt);
    p_yd.load((N + 1) * M, lane, ld_yd);
    p_yb.load(ngb, lane, ld_yb);
    for (int k = lane; k <= N; k += 64) {
        double r[NX];
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
#pragma unroll
            for (int i = 0; i < NX; ++i)
                for (int cc = 0; cc < nc; ++cc)
                    if (dm.tidx[cc] == i) r[i] += AT(yt, cc);
        for (int j = 0; j < M; ++j)
            for (int a = 0; a < 3 && a < NX; ++a) r[a] += AT(Jd, (k * M + j) * 3 + a) * AT(yd, k * M + j);
#pragma unroll
        for (int i = 0; i < NX; ++i) {
            dual = fmax(dual, fabs(r[i]));
            dsq += r[i] * r[i];
            d1 += fabs(r[i]);
        }
        if (k < N)
#pragma unroll
            for (int i = 0; i < NU; ++i) {  // general bounds: the bound row's multiplier instead of z_L, z_U
                double t = dm.gcb ? AT(yb, k * NU + i) : -AT(zl, k * NU + i) + AT(zu, k * NU + i);
                if (p.use_smooth && k < N - 1) t += 2.0 * p.smooth_weight * AT(U, k * NU + i);
#pragma unroll
                for (int a = 0; a < NX; ++a) t -= Bu[a][i] * AT(yk, k * NX + a);
                dual = fmax(dual, fabs(t));
                dsq += t * t;
                d1 += fabs(t);
            }
        if (dm.ns) {
            double t = 2.0 * p.slack_penalty * AT(S, k) + (dm.gcb ? AT(yb, N * NU + k) : -AT(zs, k));
            if (dm.sd)
                for (int j = 0; j < M; ++j) t += AT(yd, k * M + j);
            dual = fmax(dual, fabs(t));
            dsq += t * t;
            d1 += fabs(t);
        }
        for (int j = 0; j < M; ++j) {
            const double t = -AT(yd, k * M + j) - AT(vt, k * M + j);
            dual = fmax(dual, fabs(t));
            dsq += t * t;
            d1 += fabs(t);
        }
    }
    p_bs.run(ngb, lane, ld_bs, [&](int q, const double* v) {  // bound-row slacks: -y - z_L + z_U
        const double t = q < nnu ? -v[0] - v[1] + v[2] : -v[0] - v[1];
        dual = fmax(dual, fabs(t));
        dsq += t * t;
        d1 += fabs(t);
    });
    auto pri_ = [&](double v) {
        primal = fmax(primal, fabs(v));
        psq += v * v;
        p1 += fabs(v);
    };
    auto pri1 = [&](int, const double* v) { pri_(v[0]); };
    p_rci.run(NX, lane, ld_rci, pri1);
    p_rct.run(nc, lane, ld_rct, pri1);
    p_rcd.run(N * NX, lane, ld_rcd, pri1);
    cviol = wmax(primal);
    p_rcq.run((N + 1) * M, lane, ld_rcq, [&](int, const double* v) {
        pri_(v[0]);
        cviol = fmax(cviol, fmax(0.0, -v[1]));
    });
    p_rcb.run(ngb, lane, ld_rcb, [&](int q, const double* v) {  // bound rows: d(x) = U or S against its bounds
        pri_(v[0]);
        if (q < nnu) {
            const double u = v[1];
            cviol = fmax(cviol, fmax(0.0, fmax(p.umin[q % NU] - u, u - p.umax[q % NU])));
        } else {
            cviol = fmax(cviol, fmax(0.0, -v[1]));
        }
    });
    auto compl_ = [&](double z, double s) {
        c0 = fmax(c0, fabs(z * s));
        cmu = fmax(cmu, fabs(z * s - mu0));
        csum += z * s;
        zsum += fabs(z);
        nzc += 1;
    };
    p_cu.run(N * NU, lane, ld_cu, [&](int e, const double* v) {
        compl_(v[1], v[0] - p.umin[e % NU]);
        compl_(v[2], p.umax[e % NU] - v[0]);
    });
    auto compl2 = [&](int, const double* v) { compl_(v[0], v[1]); };
    if (dm.ns) p_zs.run(N + 1, lane, ld_zs, compl2);
    p_vt.run((N + 1) * M, lane, ld_vt, compl2);
    auto ysum1 = [&](int, const double* v) { ysum += fabs(v[0]); };
    p_yi.run(NX, lane, ld_yi, ysum1);
    p_yk.run(N * NX, lane, ld_yk, ysum1);
    p_yt.run(nc, lane, ld_yt, ysum1);
    p_yd.run((N + 1) * M, lane, ld_yd, ysum1);
    p_yb.run(ngb, lane, ld_yb, ysum1);
    dual = wmax(dual);
    primal = wmax(primal);
    cviol = wmax(cviol);
    c0 = wmax(c0);
    cmu = wmax(cmu);
    zsum = wsum(zsum);
    ysum = wsum(ysum);
    nzc = wsum(nzc);
    const double csum_w = wsum(csum), dsq_w = wsum(dsq), psq_w = wsum(psq);
    const double d1_w = wsum(d1), p1_w = wsum(p1);
    const double ny = NX + N * NX + nc + (N + 1) * M + ngb;
    const double sd = fmax(100.0, (ysum + zsum) / (ny + nzc)) / 100.0;
    const double scc = fmax(100.0, zsum / nzc) / 100.0;
    const double E0 = fmax(fmax(dual / sd, primal), c0 / scc);
    // IPOPT's primal-dual system error at barrier parameter m (soft restoration): sum of the 1-norms of the dual,
    // primal and complementarity residuals over the element count
    KPROF(0, 3);  // optimality measures
    const double n_pd = (double)((N + 1) * NX + N * NU + dm.ns * (N + 1) + (N + 1) * M + ngb) +
                        (double)(NX + nc + N * NX + (N + 1) * M + ngb) + nzc;
    auto pd_error = [&](double m) {
        double c1 = 0;
        for (int e = lane; e < N * NU; e += 64) {
            const double u = BVU(e);
            c1 += fabs(AT(zl, e) * (u - p.umin[e % NU]) - m) + fabs(AT(zu, e) * (p.umax[e % NU] - u) - m);
        }
        if (dm.ns)
            for (int k = lane; k <= N; k += 64) c1 += fabs(AT(zs, k) * BVS(k) - m);
        for (int q = lane; q < (N + 1) * M; q += 64) c1 += fabs(AT(vt, q) * AT(T, q) - m);
        return (d1_w + p1_w + wsum(c1)) / n_pd;
    };
    if (ph == PH_SOFT2) {
        // the soft restoration's tentatively accepted point (k_accept): accepted if its primal-dual error fell by
        // the factor, then this is the next iteration's evaluation; else back to the saved point and restoration
        const double pd_t = pd_error(SC(SC_MUPD));
        const bool ok = isfinite(pd_t) && pd_t <= o.soft_resto_pderror_reduction_factor * SC(SC_PDC);
        wsync();
        if (!ok) {
            double* buf = &AT(sts, 0);
            iter_io(ws, b, lane, buf, false);
            wsync();
            resto_enter(o, p, dm, ws, b, lane, cnt_next);
            return;
        }
        if (lane == 0) {
            SC(SC_ITERS) = SC(SC_ITERS) + 1;
            SC(SC_INSOFT) = 1;
            SC(SC_TINYLAST) = 0;
            SC(SC_PHASE) = PH_EVAL;
        }
        wsync();
    }
    const int iters = (int)SC(SC_ITERS);
    wsync();
    auto finish = [&](int status) {
        if (lane == 0) {
            SC(SC_E0) = E0;
            SC(SC_STATUS) = status;
            SC(SC_PHASE) = PH_DONE;
        }
    };
    if (!isfinite(E0)) return finish(NLOT_NUMERIC);
    if (E0 <= o.tol && dual <= o.dual_inf_tol && cviol <= o.constr_viol_tol && c0 <= o.compl_inf_tol)
        return finish(NLOT_SOLVED);
    if (iters >= o.max_iter) return finish(NLOT_MAXITER);
    // ---- barrier parameter: monotone (IPOPT MonotoneMuUpdate) or adaptive (AdaptiveMuUpdate with the
    //      quality-function oracle, runner.py:118-120; restated in oracle/nlot_oracle.c) ----
    const double kap = o.barrier_tol_factor;
    const double mu_floor = fmin(o.tol, o.compl_inf_tol) / (kap + 1.0);
    constexpr double kMuMin = 1e-11;
    double mu = mu0, tau = SC(SC_TAU);
    bool reset_filter = false;
    auto compl_mu = [&](double m) {
        double cm = 0;
        chunked_update<4, 3>(N * NU, lane, [&](int e, double* v) { v[0] = BVU(e); v[1] = AT(zl, e); v[2] = AT(zu, e); },
                             [&](int e, const double* v) {
                                 cm = fmax(cm, fabs(v[1] * (v[0] - p.umin[e % NU]) - m));
                                 cm = fmax(cm, fabs(v[2] * (p.umax[e % NU] - v[0]) - m));
                             });
        auto cm2 = [&](int, const double* v) { cm = fmax(cm, fabs(v[0] * v[1] - m)); };
        if (dm.ns) chunked_update<4, 2>(N + 1, lane, [&](int k, double* v) { v[0] = AT(zs, k); v[1] = BVS(k); }, cm2);
        chunked_update<4, 2>((N + 1) * M, lane, [&](int q, double* v) { v[0] = AT(vt, q); v[1] = AT(T, q); }, cm2);
        return wmax(cm);
    };
    bool tiny_last = o.mu_strategy == 0 && SC(SC_TINYLAST) != 0.0;  // a tiny step forces a decrease
    auto barrier_decrease = [&](double cm) {  // Fiacco-McCormick: decrease while the barrier problem is solved
        for (;;) {
            const double Emu = fmax(fmax(dual / sd, primal), cm / scc);
            if (Emu > kap * mu && !tiny_last) break;
            tiny_last = false;
            const double nm = fmax(fmin(0.2 * mu, pow(mu, 1.5)), mu_floor);
            if (nm >= mu) break;
            mu = nm;
            tau = fmax(0.99, 1.0 - mu);
            reset_filter = true;
            cm = compl_mu(mu);
        }
    };
    bool use_qf = false;
    const double avg = csum_w / nzc;
    if (o.mu_strategy == 0) {
        if (iters > 0) barrier_decrease(cmu);
    } else {
        double mu_max = SC(SC_MUMAX);
        bool free_ = SC(SC_FREE) != 0.0;
        int naf = (int)SC(SC_NAF);
        if (iters == 0) {
            mu_max = 1e3 * avg;
            free_ = true;
            naf = 0;
        }
        double th_c, ph_c, f_c;
        theta_phi(mu0, &th_c, &ph_c, &f_c);
        auto af_ok = [&]() {  // obj-constr progress filter (margin 1e-5 min(1, theta)); entries lane-parallel
            const double m = 1e-5 * fmin(1.0, th_c);
            bool bad = false;
            for (int i = lane; i < naf; i += 64)
                if (f_c + m >= AT(afilt, 2 * i) && th_c + m >= AT(afilt, 2 * i + 1)) bad = true;
            return __ballot(bad) == 0ull;
        };
        // fixed mode (IPOPT AdaptiveMuUpdate): back to free mode as soon as the point makes sufficient progress
        // w.r.t. the progress filter (checked every iteration; remembered below), else one Fiacco-McCormick
        // decrease once the barrier problem is solved
        if (!free_) {
            if (af_ok()) {
                free_ = true;
            } else if (fmax(fmax(dual / sd, primal), cmu / scc) <= kap * mu) {
                const double nm = fmax(fmin(0.2 * mu, pow(mu, 1.5)), mu_floor);
                if (nm < mu) {
                    mu = nm;
                    tau = fmax(0.99, 1.0 - mu);
                    reset_filter = true;
                }
            }
        }
        int naf_new = naf;
        if (free_) {
            if (af_ok()) {  // remember the point: drop dominated entries, append (oldest forgotten at capacity)
                const double m = 1e-5 * fmin(1.0, th_c), nf = f_c - m, nt = th_c - m;
                wsync();
                if (lane == 0) SC(SC_NAF) = naf;  // the count filter_update reads (the iteration-0 reset included)
                wsync();
                naf_new = filter_update(ws, b, &AT(afilt, 0), SC_NAF, nf, nt, cnt, lane);
            } else {  // insufficient progress: fixed mode at 0.8 x average complementarity
                free_ = false;
                mu = fmin(fmax(0.8 * avg, kMuMin), mu_max);
                tau = fmax(0.99, 1.0 - mu);
                reset_filter = true;
            }
        }
        if (lane == 0) {
            SC(SC_NAF) = naf_new;
            SC(SC_FREE) = free_ ? 1.0 : 0.0;
            SC(SC_MUMAX) = mu_max;
        }
        use_qf = free_;
    }
    const double mu_pd = (o.mu_strategy == 1 && use_qf) ? 0.0 : mu;  // soft restoration's mu (free mode: 0)
    const double pd_c = pd_error(mu_pd);
    wsync();
    if (lane == 0) {
        SC(SC_MU) = mu;
        SC(SC_TAU) = tau;
        if (reset_filter) {  // a new barrier problem: BacktrackingLineSearch::Reset (filter, soft restoration, watchdog)
            SC(SC_NFILT) = 0;
            SC(SC_INSOFT) = 0;
            SC(SC_SOFTCNT) = 0;
            SC(SC_WD) = 0;
            SC(SC_WDSHORT) = 0;
        }
        SC(SC_PDC) = pd_c;
        SC(SC_MUPD) = mu_pd;
    }
    wsync();
    KPROF(0, 4);  // convergence test, mu update (theta / phi, progress filter), primal-dual error
    // ---- Newton system (free mode: affine mu = 0 and centering mu = avg right-hand sides): stage
    //      matrices here, factorisation + inertia correction in k_ric, the rest in k_iter_b ----
    SV::template build_stages<false>(p, dm, ws, b, lane, MODE_NEWTON, 0.0, use_qf ? 0.0 : mu, avg, use_qf ? 2 : 1, SL);
    KPROF(0, 5);  // stage matrices
    KPROF_COUNT(0);
    if (lane == 0) {
        SC(SC_E0) = E0;
        SC(SC_RMU0) = use_qf ? 0.0 : mu;
        SC(SC_RMU1) = avg;
        SC(SC_RNR) = use_qf ? 2 : 1;
        SC(SC_USEQF) = use_qf ? 1.0 : 0.0;
        SC(SC_AVG) = avg;
        SC(SC_DSQ) = dsq_w;
        SC(SC_PSQ) = psq_w;
        SC(SC_NZC) = nzc;
        SC(SC_PRIMAL) = primal;
        SC(SC_RICFIX) = -1.0;
        SC(SC_RIC) = 1;
        ws.ricl[atomicAdd(&cnt[4], 1)] = b;  // k_ric's list of Newton solves (and the statistics)
    }
}

// k_iter_b: after k_ric's solve — the quality-function mu oracle (free mode: sigma search over the
// affine and centering steps), recovery of the slack/bound-multiplier steps, fraction to the boundary
// and the line-search reference values.
template <int DYN>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(NLOT_WPE_B))) void k_iter_b(const NlotProblem* __restrict__ pp_, const Dims* __restrict__ dd_, NlotSolverOptions o, const Ws* __restrict__ ws_,
                                               const int* __restrict__ active, int* cnt, float* tp, int* cnt_next) {
    grid_guard(*ws_, cnt[2], 1, GRID_ACTIVE);
    if ((int)blockIdx.x >= cnt[2]) return;
    const NlotProblem& p = *pp_;
    const Dims& dm = *dd_;
    const Ws& ws = *ws_;
    using SV = Solver<DYN>;
    constexpr int NX = SV::NX, NU = SV::NU;
    const int b = active[blockIdx.x], lane = threadIdx.x;
    if (SC(SC_RESTO) != 0.0) return;  // k_resto_b
    const int ric = (int)SC(SC_RIC);
    if (ric == 4) {  // a second-order correction's solve failed: restore the step, halve the original alpha
        double* rb = &AT(rcs, 0);
        double* sb = &AT(sts, 0);
        {
            double* buf = rb;
            const bool save = false;
            res_io(ws, b, lane, buf, save);
            buf = sb;
            step_io(ws, b, lane, buf, save);
        }
        const double na = 0.5 * SC(SC_SOCA);
        const bool failed = na < SC(SC_AMIN);
        wsync();
        if (lane == 0) {
            SC(SC_RIC) = 0;
            SC(SC_SOCK) = 0;
            SC(SC_AZ) = SC(SC_SOCAZ);
            SC(SC_TRIALS) = 1;
            SC(SC_ALPHA) = na;
            if (!failed) SC(SC_PHASE) = PH_LS;
        }
        wsync();
        if (failed) ls_failed(o, *pp_, *dd_, ws, b, lane, tp, cnt, cnt_next);
        else emit_points(*pp_, *dd_, ws, b, lane, cnt, true, tp, 1, na);
        return;
    }
    if (ric != 2) return;
    KPROF_INIT;
    const bool soc = (int)SC(SC_PHASE) == PH_SOC;
    const int N = dm.N, M = dm.M;
    const double dw = SC(SC_DW), avg = SC(SC_AVG), dsq_w = SC(SC_DSQ), psq_w = SC(SC_PSQ), nzc = SC(SC_NZC);
    const bool use_qf = SC(SC_USEQF) != 0.0;
    double mu = SC(SC_MU), tau = SC(SC_TAU);
    const int ngb = dm.gcb ? dm.ngb : 0;  // bound rows (general bounds)
    const int n_dual_ = (N + 1) * NX + N * NU + dm.ns * (N + 1) + (N + 1) * M + ngb;
    const int n_pri_ = NX + dm.nc + N * NX + (N + 1) * M + ngb;
    const int nc = dm.nc;
    constexpr double kMuMin = 1e-11;
    (void)o;
    // the lane-strided sums: every pass's first chunk loaded ahead (Pre), consumed in the same per-lane order as the
    // plain loops they replace (one memory round trip instead of one per pass and per 64 elements)
    auto theta_phi = [&](double mu, double* th, double* phv, double* fout = nullptr) {
        double t = 0, bar = 0, lin = 0;
        auto tsum = [&](int, const double* v) { t += fabs(v[0]); };
        auto l_rci = [&](int i, double* v) { v[0] = AT(rci, i); };
        auto l_rct = [&](int i, double* v) { v[0] = AT(rct, i); };
        auto l_rcd = [&](int i, double* v) { v[0] = AT(rcd, i); };
        auto l_rcq = [&](int q, double* v) { v[0] = AT(rcq, q); v[1] = AT(T, q); };
        auto l_bu = [&](int e, double* v) { v[0] = BVU(e); };
        auto l_bs = [&](int k, double* v) { v[0] = BVS(k); };
        auto l_rcb = [&](int q, double* v) { v[0] = AT(rcb, q); };
        Pre<1, 1> q_rci, q_rct, q_bs;
        Pre<4, 1> q_rcd;
        Pre<1, 2> q_rcq;
        Pre<2, 1> q_bu;
        Pre<3, 1> q_rcb;
        q_rci.load(NX, lane, l_rci);
        q_rct.load(nc, lane, l_rct);
        q_rcd.load(N * NX, lane, l_rcd);
        q_rcq.load((N + 1) * M, lane, l_rcq);
        q_bu.load(N * NU, lane, l_bu);
        if (dm.ns) q_bs.load(N + 1, lane, l_bs);
        q_rcb.load(ngb, lane, l_rcb);
        q_rci.run(NX, lane, l_rci, tsum);
        q_rct.run(nc, lane, l_rct, tsum);
        q_rcd.run(N * NX, lane, l_rcd, tsum);
        q_rcq.run((N + 1) * M, lane, l_rcq, [&](int, const double* v) {
            t += fabs(v[0]);
            bar += log(v[1]);
            lin += v[1];
        });
        q_bu.run(N * NU, lane, l_bu, [&](int e, const double* v) {
            const double u = v[0];
            bar += log(u - p.umin[e % NU]) + log(p.umax[e % NU] - u);
        });
        if (dm.ns)
            q_bs.run(N + 1, lane, l_bs, [&](int, const double* v) {
                bar += log(v[0]);
                lin += v[0];
            });
        q_rcb.run(ngb, lane, l_rcb, tsum);
        *th = wsum(t);
        const double fo = objective_w(p, dm, ws, b, lane, 0.0);
        *phv = fo - mu * wsum(bar) + 1e-5 * mu * wsum(lin);
        if (fout) *fout = fo;
    };
    // QualityFunctionMuOracle buffers: Riccati outputs + recovered slack/dual steps, affine (qa) and
    // centering minus affine (qc)
    {
        const int oU = (N + 1) * NX, oS = oU + N * NU, oyi = oS + N + 1, oyk = oyi + NX, oyt = oyk + N * NX,
                  oT = oyt + 8, ozl = oT + (N + 1) * M, ozu = ozl + N * NU, ozs = ozu + N * NU, ovt = ozs + N + 1,
                  odb = ovt + (N + 1) * M;
        // the steps of the bounded quantities: the bound rows' slacks (general bounds) or U and S
        const int oBU = dm.gcb ? odb : oU, oBS = dm.gcb ? odb + N * NU : oS;
        // store the Riccati outputs and the recovered slack/dual steps at barrier parameter m (cen: minus aff)
        // (cen: the second right-hand side's arrays dX2 ...)
        auto qf_store = [&](double m, bool cen) {
            double* dst = cen ? &AT(qc, 0) : &AT(qa, 0);
            const double* aff = &AT(qa, 0);
            const double* sX = cen ? &AT(dX2, 0) : &AT(dX, 0);
            const double* sU = cen ? &AT(dU2, 0) : &AT(dU, 0);
            const double* sS = cen ? &AT(dS2, 0) : &AT(dS, 0);
            const double* syi = cen ? &AT(yi2, 0) : &AT(yi_n, 0);
            const double* syk = cen ? &AT(yk2, 0) : &AT(yk_n, 0);
            const double* syt = cen ? &AT(yt2, 0) : &AT(yt_n, 0);
            auto put = [&](int i, double v) { dst[i] = cen ? v - aff[i] : v; };
            for (int i = lane; i < (N + 1) * NX; i += 64) put(i, sX[i]);
            for (int i = lane; i < N * NU; i += 64) put(oU + i, sU[i]);
            for (int i = lane; i <= N; i += 64) put(oS + i, sS[i]);
            for (int i = lane; i < NX; i += 64) put(oyi + i, syi[i]);
            for (int i = lane; i < N * NX; i += 64) put(oyk + i, syk[i]);
            for (int i = lane; i < 8; i += 64) put(oyt + i, syt[i]);
            for (int k = lane; k <= N; k += 64) {
                for (int j = 0; j < M; ++j) {
                    const int q = k * M + j;
                    double Jdz = 0;
                    for (int a = 0; a < 3 && a < NX; ++a) Jdz += AT(Jd, q * 3 + a) * sX[k * NX + a];
                    if (dm.sd) Jdz += sS[k];
                    const double t = AT(T, q), v = AT(vt, q), dt_ = Jdz + AT(rcq, q);
                    put(oT + q, dt_);
                    put(ovt + q, m / t - v - (v / t) * dt_);
                }
                if (dm.ns) {  // general bounds: the row slack's step d_sb = dS + rcb
                    const double sk = BVS(k), ds = dm.gcb ? sS[k] + AT(rcb, N * NU + k) : sS[k];
                    put(ozs + k, m / sk - AT(zs, k) - (AT(zs, k) / sk) * ds);
                    if (dm.gcb) put(odb + N * NU + k, ds);
                }
            }
            for (int e = lane; e < N * NU; e += 64) {
                const double u = BVU(e), sl = u - p.umin[e % NU], su = p.umax[e % NU] - u;
                const double du = dm.gcb ? sU[e] + AT(rcb, e) : sU[e];
                put(ozl + e, m / sl - AT(zl, e) - (AT(zl, e) / sl) * du);
                put(ozu + e, m / su - AT(zu, e) + (AT(zu, e) / su) * du);
                if (dm.gcb) put(odb + e, du);
            }
            wsync();
        };
        if (use_qf) {
        qf_store(0.0, false);
        qf_store(avg, true);
        const double* qa_ = &AT(qa, 0);
        const double* qc_ = &AT(qc, 0);
        const double dual_t = dsq_w / (double)n_dual_, pri_t = psq_w / (double)n_pri_;
        // Fast path (N + 1 <= 64 knots, N NU <= 128): every complementarity pair a lane owns (<= 6) is
        // cached in registers once; q(sigma) is then FMA work plus three wave reductions, and the
        // fraction to the boundary is tau / max(-dslack / slack) (reciprocals precomputed, no division
        // per pair).  Other sizes take the generic loop below.
        const bool qf_fast = N * NU <= 128 && N + 1 <= 64 && (N + 1) * M <= 64;
        constexpr int QP = 6;
        double c_sl[QP], c_isl[QP], c_da[QP], c_dc[QP], c_z[QP], c_iz[QP], c_za[QP], c_zc[QP];
        if (qf_fast) {
            auto put = [&](int j, double sl, double da, double dc, double z, double za, double zc) {
                c_sl[j] = sl;
                c_isl[j] = 1.0 / sl;
                c_da[j] = da;
                c_dc[j] = dc;
                c_z[j] = z;
                c_iz[j] = 1.0 / z;
                c_za[j] = za;
                c_zc[j] = zc;
            };
            auto none = [&](int j) {
                c_sl[j] = 1.0; c_isl[j] = 0.0; c_da[j] = c_dc[j] = 0.0;
                c_z[j] = 0.0; c_iz[j] = 0.0; c_za[j] = c_zc[j] = 0.0;
            };
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const int e = lane + 64 * h;
                if (e < N * NU) {
                    const double u = BVU(e), da = qa_[oBU + e], dc = qc_[oBU + e];
                    put(2 * h, u - p.umin[e % NU], da, dc, AT(zl, e), qa_[ozl + e], qc_[ozl + e]);
                    put(2 * h + 1, p.umax[e % NU] - u, -da, -dc, AT(zu, e), qa_[ozu + e], qc_[ozu + e]);
                } else {
                    none(2 * h);
                    none(2 * h + 1);
                }
            }
            if (dm.ns && lane <= N) put(4, BVS(lane), qa_[oBS + lane], qc_[oBS + lane], AT(zs, lane), qa_[ozs + lane],
                                        qc_[ozs + lane]);
            else none(4);
            if (lane < (N + 1) * M) put(5, AT(T, lane), qa_[oT + lane], qc_[oT + lane], AT(vt, lane), qa_[ovt + lane],
                                        qc_[ovt + lane]);
            else none(5);
        }
        auto qf = [&](double sig) {  // q(sigma): 2-norm-squared, per-element averaged (oracle qf_eval)
            const double tq = fmax(0.99, 1.0 - sig * avg);
            if (qf_fast) {
                double rp = 0.0, rd = 0.0;
#pragma unroll
                for (int j = 0; j < QP; ++j) {
                    rp = fmax(rp, -(c_da[j] + sig * c_dc[j]) * c_isl[j]);
                    rd = fmax(rd, -(c_za[j] + sig * c_zc[j]) * c_iz[j]);
                }
                rp = wmax(rp);
                rd = wmax(rd);
                const double ap = rp > 0.0 ? fmin(1.0, tq / rp) : 1.0, ad = rd > 0.0 ? fmin(1.0, tq / rd) : 1.0;
                double csq = 0.0;
#pragma unroll
                for (int j = 0; j < QP; ++j) {
                    const double c = (c_sl[j] + ap * (c_da[j] + sig * c_dc[j])) * (c_z[j] + ad * (c_za[j] + sig * c_zc[j]));
                    csq += c * c;
                }
                csq = wsum(csq);
                return (1.0 - ad) * (1.0 - ad) * dual_t + (1.0 - ap) * (1.0 - ap) * pri_t + csq / nzc;
            }
            double ap = 1.0, ad = 1.0;
            for (int e = lane; e < N * NU; e += 64) {
                const double u = BVU(e), du = qa_[oBU + e] + sig * qc_[oBU + e];
                ap = frac_to_bound(u - p.umin[e % NU], du, tq, ap);
                ap = frac_to_bound(p.umax[e % NU] - u, -du, tq, ap);
                ad = frac_to_bound(AT(zl, e), qa_[ozl + e] + sig * qc_[ozl + e], tq, ad);
                ad = frac_to_bound(AT(zu, e), qa_[ozu + e] + sig * qc_[ozu + e], tq, ad);
            }
            if (dm.ns)
                for (int k = lane; k <= N; k += 64) {
                    ap = frac_to_bound(BVS(k), qa_[oBS + k] + sig * qc_[oBS + k], tq, ap);
                    ad = frac_to_bound(AT(zs, k), qa_[ozs + k] + sig * qc_[ozs + k], tq, ad);
                }
            for (int q = lane; q < (N + 1) * M; q += 64) {
                ap = frac_to_bound(AT(T, q), qa_[oT + q] + sig * qc_[oT + q], tq, ap);
                ad = frac_to_bound(AT(vt, q), qa_[ovt + q] + sig * qc_[ovt + q], tq, ad);
            }
            ap = wmin(ap);
            ad = wmin(ad);
            double csq = 0;
            auto cq = [&](double sl, double dsl, double z, double dz) {
                const double c = (sl + ap * dsl) * (z + ad * dz);
                csq += c * c;
            };
            for (int e = lane; e < N * NU; e += 64) {
                const double u = BVU(e), du = qa_[oBU + e] + sig * qc_[oBU + e];
                cq(u - p.umin[e % NU], du, AT(zl, e), qa_[ozl + e] + sig * qc_[ozl + e]);
                cq(p.umax[e % NU] - u, -du, AT(zu, e), qa_[ozu + e] + sig * qc_[ozu + e]);
            }
            if (dm.ns)
                for (int k = lane; k <= N; k += 64)
                    cq(BVS(k), qa_[oBS + k] + sig * qc_[oBS + k], AT(zs, k), qa_[ozs + k] + sig * qc_[ozs + k]);
            for (int q = lane; q < (N + 1) * M; q += 64)
                cq(AT(T, q), qa_[oT + q] + sig * qc_[oT + q], AT(vt, q), qa_[ovt + q] + sig * qc_[ovt + q]);
            csq = wsum(csq);
            return (1.0 - ad) * (1.0 - ad) * dual_t + (1.0 - ap) * (1.0 - ap) * pri_t + csq / nzc;
        };
        // sigma search (oracle qf_sigma / qf_golden) as a state machine with one q() call site
        const double mu_max = SC(SC_MUMAX);
        const double sig_up = fmin(100.0, mu_max / avg), sig_lo = fmax(1e-6, kMuMin / avg);
        const double gfac = (3.0 - sqrt(5.0)) / 2.0;
        enum { EV_1M, EV_1, EV_M1, EV_M2, EV_N1, EV_N2, EV_UP, EV_LO, LOOP, FINAL, DONE };
        bool lg = false;
        double tu0 = 0, tl0 = 0, up = 0, lo = 0, m1 = 0, m2 = 0, q1 = 0, q2 = 0, q_up = -1, q_lo = -1, q1m = 0,
               qq = 0, sig = sig_up;
        int nsec = 0, st;
        auto toS = [&](double t_) { return lg ? pow(10.0, t_) : t_; };
        auto start = [&](double su, double qu, double sl, double ql, bool l) {
            lg = l;
            tu0 = up = lg ? log10(su) : su;
            tl0 = lo = lg ? log10(sl) : sl;
            q_up = qu;
            q_lo = ql;
            m1 = lo + gfac * (up - lo);
            m2 = lo + (1.0 - gfac) * (up - lo);
            nsec = 0;
        };
        if (sig_lo >= sig_up) {
            st = DONE;
        } else if (sig_up <= 1.0) {
            start(sig_up, -1.0, sig_lo, -1.0, true);
            st = EV_M1;
        } else if (sig_lo >= 1.0) {
            start(sig_up, -1.0, sig_lo, -1.0, false);
            st = EV_M1;
        } else {
            st = EV_1M;
        }
        while (st != DONE) {
            const double x = st == EV_1M ? 0.99
                           : st == EV_1  ? 1.0
                           : (st == EV_M1 || st == EV_N1) ? toS(m1)
                           : (st == EV_M2 || st == EV_N2) ? toS(m2)
                           : st == EV_UP ? toS(up)
                                         : toS(lo);
            const double qv = qf(x);
            switch (st) {
                case EV_1M: q1m = qv; st = EV_1; break;
                case EV_1:
                    if (q1m > qv) start(sig_up, -1.0, 1.0, qv, false);
                    else start(0.99, q1m, sig_lo, -1.0, true);
                    st = EV_M1;
                    break;
                case EV_M1: q1 = qv; st = EV_M2; break;
                case EV_M2: q2 = qv; st = LOOP; break;
                case EV_N1: q1 = qv; st = LOOP; break;
                case EV_N2: q2 = qv; st = LOOP; break;
                case EV_UP: q_up = qv; st = FINAL; break;
                default: q_lo = qv; st = FINAL; break;
            }
            while (st == LOOP || st == FINAL) {
                if (st == LOOP) {
                    if (nsec < 8 && (toS(up) - toS(lo)) >= 1e-2 * toS(up)) {
                        ++nsec;
                        if (q1 > q2) {
                            lo = m1; q_lo = q1; m1 = m2; q1 = q2;
                            m2 = lo + (1.0 - gfac) * (up - lo);
                            st = EV_N2;
                        } else {
                            up = m2; q_up = q2; m2 = m1; q2 = q1;
                            m1 = lo + gfac * (up - lo);
                            st = EV_N1;
                        }
                    } else {
                        sig = q1 < q2 ? toS(m1) : toS(m2);
                        qq = q1 < q2 ? q1 : q2;
                        if (up == tu0) st = q_up < 0 ? EV_UP : FINAL;
                        else if (lo == tl0) st = q_lo < 0 ? EV_LO : FINAL;
                        else st = DONE;
                    }
                } else {
                    if (up == tu0) {
                        if (q_up < qq) sig = toS(up);
                    } else if (lo == tl0) {
                        if (q_lo < qq) sig = toS(lo);
                    }
                    st = DONE;
                }
            }
        }
        mu = fmin(fmax(sig * avg, kMuMin), mu_max);
        sig = mu / avg;
        tau = fmax(0.99, 1.0 - mu);
        // the step for the chosen sigma: affine + sigma centering (chunked: loads before stores)
        auto comb = [&](int n, int oa, double* dst) {
            chunked_update<4, 2>(n, lane, [&](int i, double* v) { v[0] = qa_[oa + i]; v[1] = qc_[oa + i]; },
                                 [&](int i, const double* v) { dst[i] = v[0] + sig * v[1]; });
        };
        comb((N + 1) * NX, 0, &AT(dX, 0));
        comb(N * NU, oU, &AT(dU, 0));
        comb(N + 1, oS, &AT(dS, 0));
        comb(NX, oyi, &AT(yi_n, 0));
        comb(N * NX, oyk, &AT(yk_n, 0));
        comb(8, oyt, &AT(yt_n, 0));
        wsync();
        if (lane == 0) {  // a new barrier problem: BacktrackingLineSearch::Reset (filter, soft restoration, watchdog)
            SC(SC_MU) = mu;
            SC(SC_TAU) = tau;
            SC(SC_NFILT) = 0;
            SC(SC_INSOFT) = 0;
            SC(SC_SOFTCNT) = 0;
            SC(SC_WD) = 0;
            SC(SC_WDSHORT) = 0;
        }
        wsync();
        }
    }
    KPROF(1, 0);  // quality-function mu oracle (free mode) / sigma choice
    // ---- recover dt, yd+, dz; fraction to the boundary; line-search reference values ----
    const double kappa_d = 1e-5;
    double amax = 1.0, az = 1.0, gd = 0;
    for (int k = lane; k <= N; k += 64) {
        // every input of the knot loaded before its first store (the stores might alias them for the compiler: each
        // group of loads after a store was another dependent round trip); the arithmetic below is unchanged
        double jd[MMAX][3], tq[MMAX], vq[MMAX], rq[MMAX], dxk[3], xs[3][2];
#pragma unroll
        for (int j = 0; j < MMAX; ++j) {
            if (j >= M) break;
            const int q = k * M + j;
#pragma unroll
            for (int a = 0; a < 3; ++a) jd[j][a] = a < NX ? AT(Jd, q * 3 + a) : 0.0;
            tq[j] = AT(T, q);
            vq[j] = AT(vt, q);
            rq[j] = AT(rcq, q);
        }
#pragma unroll
        for (int a = 0; a < 3; ++a) dxk[a] = a < NX ? AT(dX, k * NX + a) : 0.0;
        const double dSk = (dm.sd || dm.ns) ? AT(dS, k) : 0.0;
        const int qb = N * NU + k;
        const double Sk = dm.ns ? AT(S, k) : 0.0, zsk = dm.ns ? AT(zs, k) : 0.0;
        const double sbk = (dm.ns && dm.gcb) ? AT(sb, qb) : 0.0, rcbk = (dm.ns && dm.gcb) ? AT(rcb, qb) : 0.0;
#pragma unroll
        for (int r = 0; r < 3; ++r) {  // knots k - 1, k, k + 1 (x, y) of the path-length term
            const int kk = k - 1 + r;
            xs[r][0] = (kk >= 0 && kk <= N) ? AT(X, kk * NX) : 0.0;
            xs[r][1] = (kk >= 0 && kk <= N) ? AT(X, kk * NX + 1) : 0.0;
        }
#pragma unroll
        for (int j = 0; j < MMAX; ++j) {
            if (j >= M) break;
            const int q = k * M + j;
            double Jdz = 0;
            for (int a = 0; a < 3 && a < NX; ++a) Jdz += jd[j][a] * dxk[a];
            if (dm.sd) Jdz += dSk;
            const double t = tq[j], v = vq[j];
            const double dt_ = Jdz + rq[j];
            const double dvt_ = mu / t - v - (v / t) * dt_;
            AT(dT, q) = dt_;
            AT(yd_n, q) = (v / t + dw) * dt_ + (-mu / t + kappa_d * mu);
            AT(dvt, q) = dvt_;
            amax = frac_to_bound(t, dt_, tau, amax);
            az = frac_to_bound(v, dvt_, tau, az);
            gd += (-mu / t + kappa_d * mu) * dt_;
        }
        if (dm.ns) {
            if (dm.gcb) {  // the bound row S - sb: sb's step, the row multiplier (oracle recover)
                const double s = Sk, ds = dSk, sv = sbk, db = ds + rcbk;
                const double sig = zsk / sv, bg = -mu / sv + kappa_d * mu;
                const double dzs_ = mu / sv - zsk - sig * db;
                AT(dsb, qb) = db;
                AT(yb_n, qb) = (sig + dw) * db + bg;
                AT(dzs, k) = dzs_;
                amax = frac_to_bound(sv, db, tau, amax);
                az = frac_to_bound(zsk, dzs_, tau, az);
                gd += 2.0 * p.slack_penalty * s * ds + bg * db;
            } else {
                const double s = Sk, ds = dSk;
                const double dzs_ = mu / s - zsk - (zsk / s) * ds;
                AT(dzs, k) = dzs_;
                amax = frac_to_bound(s, ds, tau, amax);
                az = frac_to_bound(zsk, dzs_, tau, az);
                gd += (2.0 * p.slack_penalty * s - mu / s + kappa_d * mu) * ds;
            }
        }
#pragma unroll
        for (int r = 0; r < 2; ++r) {  // path-length gradient . dx_k: segments k - 1 and k
            const int seg = k - 1 + r;
            if (seg < 0 || seg >= N) continue;
            const double dx = xs[r + 1][0] - xs[r][0];
            const double dy = xs[r + 1][1] - xs[r][1];
            const double rr = sqrt(dx * dx + dy * dy + p.path_eps);
            const double sgn = seg == k ? -1.0 : 1.0;
            gd += sgn * (dx / rr) * dxk[0] + sgn * (dy / rr) * dxk[1];
        }
    }
    // the controls' bound rows in chunks of 2 x 64 (loads before stores; same element order as the plain loop)
    chunked_update<2, 6>(N * NU, lane,
                         [&](int e, double* v) {
                             v[0] = AT(U, e);
                             v[1] = AT(dU, e);
                             v[2] = dm.gcb ? AT(sb, e) : 0.0;
                             v[3] = dm.gcb ? AT(rcb, e) : 0.0;
                             v[4] = AT(zl, e);
                             v[5] = AT(zu, e);
                         },
                         [&](int e, const double* v) {
        const int i = e % NU, k = e / NU;
        const double zle = v[4], zue = v[5];
        if (dm.gcb) {  // the bound row U - sb: sb's step d_sb = dU + rcb, the row multiplier (oracle recover)
            const double u = v[0], du = v[1], bv = v[2], sl = bv - p.umin[i], su = p.umax[i] - bv;
            const double db = du + v[3];
            const double dzl_ = mu / sl - zle - (zle / sl) * db;
            const double dzu_ = mu / su - zue + (zue / su) * db;
            const double sig = zle / sl + zue / su, bg = -mu / sl + mu / su;
            AT(dsb, e) = db;
            AT(yb_n, e) = (sig + dw) * db + bg;
            AT(dzl, e) = dzl_;
            AT(dzu, e) = dzu_;
            amax = frac_to_bound(sl, db, tau, amax);
            amax = frac_to_bound(su, -db, tau, amax);
            az = frac_to_bound(zle, dzl_, tau, az);
            az = frac_to_bound(zue, dzu_, tau, az);
            if (p.use_smooth && k < N - 1) gd += 2.0 * p.smooth_weight * u * du;
            gd += bg * db;
            return;
        }
        const double u = v[0], sl = u - p.umin[i], su = p.umax[i] - u, du = v[1];
        const double dzl_ = mu / sl - zle - (zle / sl) * du;
        const double dzu_ = mu / su - zue + (zue / su) * du;
        AT(dzl, e) = dzl_;
        AT(dzu, e) = dzu_;
        amax = frac_to_bound(sl, du, tau, amax);
        amax = frac_to_bound(su, -du, tau, amax);
        az = frac_to_bound(zle, dzl_, tau, az);
        az = frac_to_bound(zue, dzu_, tau, az);
        double gu = -mu / sl + mu / su;
        if (p.use_smooth && k < N - 1) gu += 2.0 * p.smooth_weight * u;
        gd += gu * du;
                         });
    amax = wmin(amax);
    az = wmin(az);
    gd = wsum(gd);
    wsync();
    KPROF(1, 1);  // step recovery, fraction to the boundary, gradient term
    if (soc) {  // second-order corrected direction: its fraction-to-boundary step is the one trial point
        if (lane == 0) {
            SC(SC_RIC) = 0;
            SC(SC_ALPHA) = amax;
            SC(SC_AZ) = az;
            SC(SC_PHASE) = PH_LS;
        }
        wsync();
        emit_points(p, dm, ws, b, lane, cnt, true, tp, 1, amax);
        return;
    }
    double theta, phi;
    theta_phi(mu, &theta, &phi);
    const double gt = 1e-5, gp = 1e-8, delta = 1.0, sth = 1.1, sph = 2.3;
    double amin = gt;
    if (gd < 0) {
        amin = fmin(gt, gp * theta / (-gd));
        if (theta <= SC(SC_THMIN)) amin = fmin(amin, delta * pow(theta, sth) / pow(-gd, sph));
    }
    amin *= 0.05;
    // IPOPT DetectTinyStep (not while the watchdog runs): primal step tiny relative to the iterate, multiplier
    // step small, nearly feasible -> the full step is taken without a line search
    const bool in_wd = SC(SC_WD) != 0.0, in_soft = SC(SC_INSOFT) != 0.0;
    bool tiny = false;
    if (o.tiny_step_tol > 0 && !in_wd && !in_soft) {
        double mx = 0, my = 0, ya = 0;
        for (int i = lane; i < (N + 1) * NX; i += 64) mx = fmax(mx, fabs(AT(dX, i)) / (1.0 + fabs(AT(X, i))));
        for (int i = lane; i < N * NU; i += 64) mx = fmax(mx, fabs(AT(dU, i)) / (1.0 + fabs(AT(U, i))));
        if (dm.ns)
            for (int k = lane; k <= N; k += 64) mx = fmax(mx, fabs(AT(dS, k)) / (1.0 + fabs(AT(S, k))));
        for (int q = lane; q < (N + 1) * M; q += 64) mx = fmax(mx, fabs(AT(dT, q)) / (1.0 + fabs(AT(T, q))));
        for (int q = lane; q < ngb; q += 64) mx = fmax(mx, fabs(AT(dsb, q)) / (1.0 + fabs(AT(sb, q))));
        auto ystep = [&](double yn, double y) {
            my = fmax(my, fabs(yn - y));
            ya = fmax(ya, fabs(y));
        };
        for (int i = lane; i < NX; i += 64) ystep(AT(yi_n, i), AT(yi, i));
        for (int i = lane; i < N * NX; i += 64) ystep(AT(yk_n, i), AT(yk, i));
        for (int i = lane; i < nc; i += 64) ystep(AT(yt_n, i), AT(yt, i));
        for (int q = lane; q < (N + 1) * M; q += 64) ystep(AT(yd_n, q), AT(yd, q));
        for (int q = lane; q < ngb; q += 64) ystep(AT(yb_n, q), AT(yb, q));
        mx = wmax(mx);
        my = wmax(my);
        ya = wmax(ya);
        tiny = mx <= o.tiny_step_tol && my / (1.0 + ya) <= o.tiny_step_y_tol && SC(SC_PRIMAL) < 1e-4;
    }
    // IPOPT StartWatchDog: after watchdog_shortened_iter_trigger shortened steps in a row, remember the point,
    // its direction and reference values; the next watchdog_trial_iter_max iterations try full steps only
    const bool start_wd = !tiny && !in_wd && !in_soft && o.watchdog_shortened_iter_trigger > 0 &&
                          SC(SC_WDSHORT) >= o.watchdog_shortened_iter_trigger;
    if (start_wd) {
        double* buf = &AT(wdi, 0);
        iter_io(ws, b, lane, buf, true);
        buf = &AT(wdd, 0);
        step_io(ws, b, lane, buf, true);
    }
    wsync();
    if (lane == 0) {
        SC(SC_RIC) = 0;
        SC(SC_THETA) = theta;
        SC(SC_PHI) = phi;
        SC(SC_GD) = gd;
        SC(SC_AMAX) = amax;
        SC(SC_AMIN) = amin;
        SC(SC_AZ) = az;
        SC(SC_ALPHA) = amax;
        SC(SC_TRIALS) = 0;
        SC(SC_SOCK) = 0;
        SC(SC_LASTREJF) = 0;
        SC(SC_TINY) = tiny ? 1.0 : 0.0;
        SC(SC_PHASE) = PH_LS;
        if (start_wd) {
            SC(SC_WD) = 1;
            SC(SC_WDTRIAL) = 0;
            SC(SC_WDTH) = theta;
            SC(SC_WDPH) = phi;
            SC(SC_WDGD) = gd;
            SC(SC_WDAT) = amax;
            SC(SC_WDAZ) = az;
            SC(SC_WDAMIN) = amin;
            SC(SC_WDMU) = mu;
            SC(SC_WDTAU) = tau;
        }
    }
    wsync();  // dX complete
    if (in_soft) {
        // soft restoration phase (IPOPT): no line search; after max_soft_resto_iters soft steps the restoration
        // phase, else the next soft step (PH_SOFT1, min(alpha_max, alpha_z), this step's trial list)
        const int sc = (int)SC(SC_SOFTCNT) + 1;
        wsync();
        if (lane == 0) SC(SC_SOFTCNT) = sc;
        if (sc > o.max_soft_resto_iters) {
            resto_enter(o, p, dm, ws, b, lane, cnt_next);
        } else {
            if (lane == 0) {
                SC(SC_ALPHA) = fmin(amax, az);
                SC(SC_PHASE) = PH_SOFT1;
            }
            wsync();
            emit_points(p, dm, ws, b, lane, cnt, true, tp, 1, fmin(amax, az));
        }
        return;
    }
    KPROF(1, 2);  // theta / phi, tiny step, watchdog, soft restoration
    // the first line-search round: alpha_max alone (none for a tiny step)
    emit_points(p, dm, ws, b, lane, cnt, true, tp, tiny ? 0 : 1, amax);
    KPROF(1, 3);  // trial corners
    KPROF_COUNT(1);
}

// An instance leaves the active list (k_accept): its outputs (X, U, S, cost = the objective at X, status, iterations;
// run_benchmark.py:146-167) go to the caller's arrays at its instance index, and its slot joins the free list.
__device__ void retire(const NlotProblem& p, const Dims& dm, const Ws& ws, int b, int lane) {
    const int N = dm.N, nx = dm.nx, nu = dm.nu;
    const size_t inst = (size_t)ws.sinst[b];
    for (int i = lane; i < (N + 1) * nx; i += 64) ws.oX[inst * (N + 1) * nx + i] = AT(X, i);
    for (int i = lane; i < N * nu; i += 64) ws.oU[inst * N * nu + i] = AT(U, i);
    if (ws.oS)
        for (int k = lane; k <= N; k += 64) ws.oS[inst * (N + 1) + k] = dm.ns ? AT(S, k) : 0.0;
    const double c = objective_w(p, dm, ws, b, lane, 0.0);
    if (lane == 0) {
        ws.ocost[inst] = c;
        const int st = (int)SC(SC_STATUS);
        ws.ostat[inst] = st < 0 ? NLOT_MAXITER : st;
        ws.oiters[inst] = (int)SC(SC_ITERS);
        ws.freel[atomicAdd(&ws.cnt[2 * CSET], 1)] = b;
    }
}

template <int DYN>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(NLOT_WPE_ACC))) void k_accept(const NlotProblem* __restrict__ pp_, const Dims* __restrict__ dd_, NlotSolverOptions o, const Ws* __restrict__ ws_,
                                               const int* __restrict__ active, int* __restrict__ next,
                                               int* __restrict__ nextr, const double* __restrict__ x0,
                                               const double* __restrict__ xg, int* cnt, int* cnt_next, float* tp_next,
                                               const float* tval, int nspec_next) {
    grid_guard(*ws_, cnt[2], 1, GRID_ACTIVE);
    if ((int)blockIdx.x >= cnt[2]) return;
    const NlotProblem& p = *pp_;
    const Dims& dm = *dd_;
    const Ws& ws = *ws_;
    constexpr int NX = Dyn<DYN>::NX, NU = Dyn<DYN>::NU;
    const int b = active[blockIdx.x], lane = threadIdx.x;
    int ph = (int)SC(SC_PHASE);
    // instances in a restoration phase: k_resto_ls ran their line search; here they only join the next lists
    if (SC(SC_RESTO) == 0.0 && (ph == PH_LS || ph == PH_SOFT1)) {
        const int N = dm.N, M = dm.M, nc = dm.nc;
        const double a0 = SC(SC_ALPHA), mu = SC(SC_MU);
        const int rank0 = (int)SC(SC_RANK), ncand = (int)SC(SC_NCAND);  // as emitted
        const double* x0b = x0 + (size_t)b * NX;
        const double* xgb = xg + (size_t)b * NX;
        const double gt = 1e-5, gp = 1e-8, delta = 1.0, sth = 1.1, sph = 2.3, eta = 1e-8;
        const int nf = (int)SC(SC_NFILT);
        const bool in_wd = SC(SC_WD) != 0.0, tiny = SC(SC_TINY) != 0.0;
        const int sock = (int)SC(SC_SOCK);
        // theta and phi at the trial point x + al d (candidate trial-list slot `rank`); with `store`, the
        // residual rows become keep * rc + c(x + al d) (the second-order correction's right-hand side)
        auto trial = [&](double al, int rank, bool store, double keep, double* th_o, double* ph_o) {
            double th = 0, bar = 0, lin = 0;
            for (int i = lane; i < NX; i += 64) {
                const double c = AT(X, i) + al * AT(dX, i) - x0b[i];
                th += fabs(c);
                if (store) AT(rci, i) = keep * AT(rci, i) + c;
            }
            for (int cc = lane; cc < nc; cc += 64) {
                const int ix = N * NX + dm.tidx[cc];
                const double c = AT(X, ix) + al * AT(dX, ix) - xgb[dm.tidx[cc]];
                th += fabs(c);
                if (store) AT(rct, cc) = keep * AT(rct, cc) + c;
            }
            for (int k = lane; k <= N; k += 64) {
                double xk[NX];
#pragma unroll
                for (int i = 0; i < NX; ++i) xk[i] = AT(X, k * NX + i) + al * AT(dX, k * NX + i);
                if (k < N) {
                    double u[NU], f[NX];
#pragma unroll
                    for (int i = 0; i < NU; ++i) u[i] = AT(U, k * NU + i) + al * AT(dU, k * NU + i);
                    Dyn<DYN>::f(xk, u, p.wheelbase, f, p.dt);
#pragma unroll
                    for (int i = 0; i < NX; ++i) {
                        const double c = AT(X, (k + 1) * NX + i) + al * AT(dX, (k + 1) * NX + i) - (xk[i] + p.dt * f[i]);
                        th += fabs(c);
                        if (store) AT(rcd, k * NX + i) = keep * AT(rcd, k * NX + i) + c;
                    }
                    if (dm.gcb) {  // bound rows U - sb, the barrier of sb
#pragma unroll
                        for (int i = 0; i < NU; ++i) {
                            const int qb = k * NU + i;
                            const double sv = AT(sb, qb) + al * AT(dsb, qb), c = u[i] - sv;
                            th += fabs(c);
                            if (store) AT(rcb, qb) = keep * AT(rcb, qb) + c;
                            bar += log(sv - p.umin[i]) + log(p.umax[i] - sv);
                        }
                    } else {
#pragma unroll
                        for (int i = 0; i < NU; ++i) bar += log(u[i] - p.umin[i]) + log(p.umax[i] - u[i]);
                    }
                }
                double d[MMAX];
                knot_eval(p, dm, ws, rank, k, xk, d, nullptr, nullptr, nullptr, tval);
                const double sk = AT(S, k) + al * AT(dS, k);
                for (int j = 0; j < M; ++j) {
                    const double t = AT(T, k * M + j) + al * AT(dT, k * M + j);
                    const double c = d[j] + (dm.sd ? sk : 0.0) - t;
                    th += fabs(c);
                    if (store) AT(rcq, k * M + j) = keep * AT(rcq, k * M + j) + c;
                    bar += log(t);
                    lin += t;
                }
                if (dm.ns) {
                    if (dm.gcb) {  // bound row S - sb
                        const int qb = N * NU + k;
                        const double sv = AT(sb, qb) + al * AT(dsb, qb), c = sk - sv;
                        th += fabs(c);
                        if (store) AT(rcb, qb) = keep * AT(rcb, qb) + c;
                        bar += log(sv);
                        lin += sv;
                    } else {
                        bar += log(sk);
                        lin += sk;
                    }
                }
            }
            *th_o = wsum(th);
            const double fo = objective_w(p, dm, ws, b, lane, al);
            *ph_o = fo - mu * wsum(bar) + 1e-5 * mu * wsum(lin);
        };
        // IPOPT FilterLSAcceptor::CheckAcceptabilityOfTrialPoint against reference values (rth, rph, rgd) with
        // step size `at` for the switching condition / Armijo test
        int rejf = 0;  // the last acceptance test failed on the filter after the sufficient-decrease test passed
        auto acceptable = [&](double rth, double rph, double rgd, double at, double th, double pht, int* fa) {
            int ok = isfinite(th) && isfinite(pht) && th <= SC(SC_THMAX);
            const int ftype = rgd < 0 && at * pow(-rgd, sph) > delta * pow(rth, sth);
            const int armijo = cmp_le(pht - rph, eta * at * rgd, rph);
            if (ok) {
                if (ftype && rth <= SC(SC_THMIN)) {
                    ok = armijo;
                } else {
                    ok = cmp_le(th, (1.0 - gt) * rth, rth) || cmp_le(pht - rph, -gp * rth, rph);
                    if (ok && pht > rph) {
                        const double bas = fabs(rph) > 10.0 ? log10(fabs(rph)) : 1.0;
                        if (log10(pht - rph) > 5.0 + bas) ok = 0;
                    }
                }
            }
            if (ok) {
                int bad = 0;
                for (int i = lane; i < nf; i += 64) {
                    const double ft = AT(filt, 2 * i), fp = AT(filt, 2 * i + 1);
                    if (!(th <= ft || pht <= fp)) bad = 1;
                }
                ok = wmax((double)bad) == 0.0;
                rejf = !ok;
            } else {
                rejf = 0;
            }
            *fa = ok && ftype && armijo;
            return ok;
        };
        // accept the trial point x + al d: primal and equality multipliers with al, bound multipliers with az and
        // IPOPT's kappa_Sigma safeguard
        auto accept_point = [&](double al, double az) {
            const double ks = 1e10;
            auto zupd = [&](double z, double dz, double sl) {
                const double zn = z + az * dz;
                return fmax(fmin(zn, ks * mu / sl), mu / (ks * sl));
            };
            chunked_update<4, 2>((N + 1) * NX, lane, [&](int i, double* v) { v[0] = AT(X, i); v[1] = AT(dX, i); },
                   [&](int i, const double* v) { AT(X, i) = v[0] + al * v[1]; });
            if (dm.gcb) {  // general bounds: U and S free; the bound rows' slacks carry the bound multipliers
                chunked_update<4, 2>(N * NU, lane, [&](int e, double* v) { v[0] = AT(U, e); v[1] = AT(dU, e); },
                       [&](int e, const double* v) { AT(U, e) = v[0] + al * v[1]; });
                if (dm.ns)
                    chunked_update<4, 2>(N + 1, lane, [&](int k, double* v) { v[0] = AT(S, k); v[1] = AT(dS, k); },
                           [&](int k, const double* v) { AT(S, k) = v[0] + al * v[1]; });
                chunked_update<4, 4>(dm.ngb, lane,
                       [&](int q, double* v) { v[0] = AT(sb, q); v[1] = AT(dsb, q); v[2] = AT(yb, q); v[3] = AT(yb_n, q); },
                       [&](int q, const double* v) {
                           const double sv = v[0] + al * v[1];
                           AT(sb, q) = sv;
                           AT(yb, q) = v[2] + al * (v[3] - v[2]);
                           if (q < N * NU) {
                               AT(zl, q) = zupd(AT(zl, q), AT(dzl, q), sv - p.umin[q % NU]);
                               AT(zu, q) = zupd(AT(zu, q), AT(dzu, q), p.umax[q % NU] - sv);
                           } else {
                               AT(zs, q - N * NU) = zupd(AT(zs, q - N * NU), AT(dzs, q - N * NU), sv);
                           }
                       });
            } else {
            chunked_update<4, 6>(N * NU, lane,
                   [&](int e, double* v) {
                       v[0] = AT(U, e); v[1] = AT(dU, e); v[2] = AT(zl, e); v[3] = AT(dzl, e); v[4] = AT(zu, e);
                       v[5] = AT(dzu, e);
                   },
                   [&](int e, const double* v) {
                       const double u = v[0] + al * v[1];
                       AT(U, e) = u;
                       AT(zl, e) = zupd(v[2], v[3], u - p.umin[e % NU]);
                       AT(zu, e) = zupd(v[4], v[5], p.umax[e % NU] - u);
                   });
            if (dm.ns)
                chunked_update<4, 4>(N + 1, lane, [&](int k, double* v) { v[0] = AT(S, k); v[1] = AT(dS, k); v[2] = AT(zs, k); v[3] = AT(dzs, k); },
                       [&](int k, const double* v) {
                           const double s_ = v[0] + al * v[1];
                           AT(S, k) = s_;
                           AT(zs, k) = zupd(v[2], v[3], s_);
                       });
            }
            chunked_update<4, 6>((N + 1) * M, lane,
                   [&](int q, double* v) {
                       v[0] = AT(T, q); v[1] = AT(dT, q); v[2] = AT(vt, q); v[3] = AT(dvt, q); v[4] = AT(yd, q);
                       v[5] = AT(yd_n, q);
                   },
                   [&](int q, const double* v) {
                       const double t = v[0] + al * v[1];
                       AT(T, q) = t;
                       AT(vt, q) = zupd(v[2], v[3], t);
                       AT(yd, q) = v[4] + al * (v[5] - v[4]);
                   });
            chunked_update<4, 2>(NX, lane, [&](int i, double* v) { v[0] = AT(yi, i); v[1] = AT(yi_n, i); },
                   [&](int i, const double* v) { AT(yi, i) = v[0] + al * (v[1] - v[0]); });
            chunked_update<4, 2>(N * NX, lane, [&](int i, double* v) { v[0] = AT(yk, i); v[1] = AT(yk_n, i); },
                   [&](int i, const double* v) { AT(yk, i) = v[0] + al * (v[1] - v[0]); });
            chunked_update<4, 2>(nc, lane, [&](int i, double* v) { v[0] = AT(yt, i); v[1] = AT(yt_n, i); },
                   [&](int i, const double* v) { AT(yt, i) = v[0] + al * (v[1] - v[0]); });
        };
        if (ph == PH_SOFT1) {
            // IPOPT TrySoftRestoStep: the step a = min(alpha_max, alpha_z) for primal and dual variables is taken if
            // the filter accepts it (the switching condition at alpha 0), or if it reduces the primal-dual error by
            // soft_resto_pderror_reduction_factor (PH_SOFT2: tentatively accepted, evaluated by the next step)
            double th, pht;
            int fa = 0;
            trial(a0, rank0, false, 0.0, &th, &pht);
            const int sat = acceptable(SC(SC_THETA), SC(SC_PHI), SC(SC_GD), 0.0, th, pht, &fa);
            wsync();
            if (!sat) {
                double* buf = &AT(sts, 0);
                iter_io(ws, b, lane, buf, true);
                wsync();
            }
            accept_point(a0, a0);
            wsync();
            if (lane == 0) {
                SC(SC_AZ) = a0;
                SC(SC_ACCSLOT) = (double)rank0;
                SC(SC_SOCK) = 0;
                if (sat) {
                    SC(SC_ITERS) = SC(SC_ITERS) + 1;
                    SC(SC_INSOFT) = 0;
                    SC(SC_SOFTCNT) = 0;
                    SC(SC_TINYLAST) = 0;
                    SC(SC_PHASE) = PH_EVAL;
                } else {
                    SC(SC_PHASE) = PH_SOFT2;
                }
            }
            ph = sat ? PH_EVAL : PH_SOFT2;
            wsync();
            emit_points(p, dm, ws, b, lane, cnt_next, false, nullptr, 1, 0.0);
        } else {
        KPROF_INIT;
        const double theta = SC(SC_THETA), phi = SC(SC_PHI), gd = SC(SC_GD);
        double rth = theta, rph = phi, rgd = gd, at_fix = -1.0;
        if (in_wd) {  // watchdog: the watchdog point's reference values and its alpha_max as the test step
            rth = SC(SC_WDTH);
            rph = SC(SC_WDPH);
            rgd = SC(SC_WDGD);
            at_fix = SC(SC_WDAT);
        }
        if (sock > 0) at_fix = SC(SC_SOCA);  // a corrected trial is tested with the original alpha
        int ok = 0, fa = 0, cnd = 0;
        double al = a0, th = 0, pht = 0;
        int lastrej = (int)SC(SC_LASTREJF);
        if (tiny) {
            ok = 1;
            al = SC(SC_AMAX);
        } else {
            for (cnd = 0; cnd < ncand && !ok; ++cnd) {
                al = ldexp(a0, -cnd);
                trial(al, rank0 + cnd, false, 0.0, &th, &pht);
                ok = acceptable(rth, rph, rgd, at_fix >= 0 ? at_fix : al, th, pht, &fa);
                if (!ok && sock == 0) lastrej = rejf;  // corrected trials do not count (as the oracle)
            }
        }
        if (lane == 0) SC(SC_LASTREJF) = lastrej;
        KPROF(2, 0);  // trial points: theta / phi, acceptance tests
        int next_round = 0;  // 1: emit the next backtracking round from SC_ALPHA; 2: PH_SOC
        bool tentative = false;
        wsync();
        if (!ok) {
            if (sock > 0) {  // a corrected trial was rejected
                if (th > o.kappa_soc * SC(SC_SOCTH) || sock >= o.max_soc) {  // give up: the original step, halved
                    double* buf = &AT(rcs, 0);
                    res_io(ws, b, lane, buf, false);
                    buf = &AT(sts, 0);
                    step_io(ws, b, lane, buf, false);
                    wsync();
                    if (lane == 0) {
                        SC(SC_SOCK) = 0;
                        SC(SC_AZ) = SC(SC_SOCAZ);
                        SC(SC_ALPHA) = 0.5 * SC(SC_SOCA);
                        SC(SC_TRIALS) = 1;
                    }
                    next_round = 1;
                } else {  // c_soc = alpha_soc c_soc + c(x + alpha_soc d_soc), solve again
                    trial(a0, rank0, true, a0, &th, &pht);
                    if (lane == 0) {
                        SC(SC_SOCTH) = th;
                        SC(SC_SOCK) = sock + 1;
                    }
                    next_round = 2;
                }
            } else if (in_wd) {
                const int wt = (int)SC(SC_WDTRIAL) + 1;
                if (wt > o.watchdog_trial_iter_max) {  // StopWatchDog: back to the watchdog point and direction
                    double* buf = &AT(wdi, 0);
                    iter_io(ws, b, lane, buf, false);
                    buf = &AT(wdd, 0);
                    step_io(ws, b, lane, buf, false);
                    wsync();
                    if (lane == 0) {
                        SC(SC_WD) = 0;
                        SC(SC_WDSHORT) = 0;
                        SC(SC_LASTREJF) = 0;
                        SC(SC_MU) = SC(SC_WDMU);
                        SC(SC_TAU) = SC(SC_WDTAU);
                        SC(SC_AMAX) = SC(SC_WDAT);
                        SC(SC_AZ) = SC(SC_WDAZ);
                        SC(SC_AMIN) = SC(SC_WDAMIN);
                        SC(SC_THETA) = SC(SC_WDTH);
                        SC(SC_PHI) = SC(SC_WDPH);
                        SC(SC_GD) = SC(SC_WDGD);
                        SC(SC_ALPHA) = 0.5 * SC(SC_WDAT);
                        SC(SC_TRIALS) = 1;
                    }
                    next_round = 1;
                } else {  // a tentative full step, accepted without the test
                    if (lane == 0) SC(SC_WDTRIAL) = wt;
                    ok = 1;
                    tentative = true;
                    al = SC(SC_AMAX);
                    cnd = 1;
                    fa = 0;
                }
            } else if ((int)SC(SC_TRIALS) == 0 && o.max_soc > 0 && th >= theta) {
                // second-order correction of the rejected full step: save the step and the residuals, then
                // c_soc = alpha c(x) + c(x + alpha d)
                double* buf = &AT(sts, 0);
                step_io(ws, b, lane, buf, true);
                buf = &AT(rcs, 0);
                res_io(ws, b, lane, buf, true);
                wsync();
                trial(a0, rank0, true, a0, &th, &pht);
                if (lane == 0) {
                    SC(SC_SOCAZ) = SC(SC_AZ);
                    SC(SC_SOCA) = a0;
                    SC(SC_SOCTH) = th;
                    SC(SC_SOCK) = 1;
                }
                next_round = 2;
            } else {
                if (lane == 0) {
                    SC(SC_ALPHA) = ldexp(a0, -ncand);
                    SC(SC_TRIALS) = SC(SC_TRIALS) + ncand;
                }
                next_round = 1;
            }
        }
        wsync();
        KPROF(2, 1);  // rejection: second-order correction's residuals, watchdog, next round
        if (ok) {
            // filter augmentation with the current point's values unless an f-type step met Armijo (or the
            // step is tiny: IPOPT takes it without the filter)
            // IPOPT filter reset heuristic (filter_reset_trigger 5, max_filter_resets 5): the filter is cleared
            // when the last rejected trial of 5 successive line searches was rejected by the filter
            if (!tiny && lane == 0 && SC(SC_NFRES) < 5) {
                SC(SC_NFREJ) = lastrej ? SC(SC_NFREJ) + 1 : 0;
                if (SC(SC_NFREJ) >= 5) {
                    SC(SC_NFILT) = 0;
                    SC(SC_NFRES) = SC(SC_NFRES) + 1;
                    SC(SC_NFREJ) = 0;
                }
            }
            wsync();  // lane 0's filter reset above
            if (!tiny && !fa) filter_add(ws, b, &AT(filt, 0), SC_NFILT, theta, phi, cnt, lane);
            // accept: primal and multipliers with alpha, bound multipliers with alpha_z + safeguard
            accept_point(al, SC(SC_AZ));
            const bool stop_tiny = tiny && SC(SC_TINYLAST) != 0.0;  // IPOPT STOP_AT_TINY_STEP
            ph = stop_tiny ? PH_DONE : PH_EVAL;
            if (lane == 0) {
                SC(SC_ITERS) = SC(SC_ITERS) + 1;
                SC(SC_PHASE) = ph;
                if (stop_tiny) SC(SC_STATUS) = NLOT_TINY_STEP;
                // the candidate the loop stepped past is the accepted one (no slot for a tiny step)
                SC(SC_ACCSLOT) = tiny ? -1.0 : (double)(rank0 + cnd - 1);
                if (in_wd && !tentative) SC(SC_WD) = 0;
                if (!tiny) SC(SC_WDSHORT) = al < SC(SC_AMAX) ? SC(SC_WDSHORT) + 1 : 0;
                SC(SC_SOCK) = 0;
                SC(SC_TINYLAST) = tiny ? 1.0 : 0.0;
            }
            // corners of the new iterate, for the next step's full launch
            wsync();  // X complete
            KPROF(2, 2);  // accepted: filter, the new iterate
            if (!stop_tiny) emit_points(p, dm, ws, b, lane, cnt_next, false, nullptr, 1, 0.0);
            KPROF(2, 3);  // corners of the new iterate
        } else if (next_round == 2) {
            ph = PH_SOC;
            if (lane == 0) SC(SC_PHASE) = PH_SOC;
        } else {
            const double na = SC(SC_ALPHA);
            if (na < SC(SC_AMIN)) {
                ph = ls_failed(o, p, dm, ws, b, lane, tp_next, cnt_next, cnt_next);
            } else {
                emit_points(p, dm, ws, b, lane, cnt_next, true, tp_next, n_later(na, SC(SC_AMIN), nspec_next), na);
            }
            KPROF(2, 4);  // rejected: next round's corners
        }
        KPROF_COUNT(2);
        }  // PH_LS
    }
    wsync();
    if (SC(SC_RESTO) == 2.0) {  // back from a restoration phase in this step's k_resto_a (k_resto_a, "returning")
        wsync();
        if (lane == 0) {
            SC(SC_RESTO) = 0;
            SC(SC_ACCSLOT) = -1;
        }
        wsync();
        emit_points(p, dm, ws, b, lane, cnt_next, false, nullptr, 1, 0.0);
    }
    wsync();
    ph = (int)SC(SC_PHASE);
    if (ph == PH_DONE) {
        retire(p, dm, ws, b, lane);
    } else if (lane == 0) {  // the next step's active list (and restoration list) and counts
        next[atomicAdd(&cnt_next[2], 1)] = b;
        if (SC(SC_RESTO) != 0.0) nextr[atomicAdd(&cnt_next[5], 1)] = b;
    }
}

// ---------------------------------------------------------------------------------------------
// Feasibility restoration phase (IPOPT MinC_1NrmRestorationPhase; oracle restoration()): instances with
// SC_RESTO = 1, list ws.actr.  The restoration problem's iterate lives in the ordinary arrays (X U S T, y, z) plus
// p, n, z_p, z_n per equality row; the original iterate (x_R and its bound multipliers) is saved in wdi.
//   k_resto_a  (PH_RINIT: initialisation, then) evaluation, back-to-the-original-problem test, convergence,
//              monotone mu, restoration stage matrices (k_ric<DYN, true> solves them)
//   k_resto_b  p, n, t and bound-multiplier steps, fraction to the boundary, line-search reference values
//   k_resto_ls filter line search of the restoration problem (no second-order correction, watchdog or soft step)
// ---------------------------------------------------------------------------------------------
template <int DYN>
struct Resto {
    static constexpr int NX = Dyn<DYN>::NX, NU = Dyn<DYN>::NU;
    // restoration rows: every equality row, the bound rows last (general bounds)
    __device__ static int n_rows(const Dims& dm) {
        return NX + dm.N * NX + dm.nc + (dm.N + 1) * dm.M + (dm.gcb ? dm.ngb : 0);
    }
    // multiplier of restoration row i (the row's equality multiplier)
    __device__ static double yrow(const Dims& dm, const Ws& ws, int b, int i) {
        const int rt = NX + dm.N * NX, rq = rt + dm.nc, rb = rq + (dm.N + 1) * dm.M;
        return i < NX ? AT(yi, i) : i < rt ? AT(yk, i - NX) : i < rq ? AT(yt, i - rt) : i < rb ? AT(yd, i - rq)
                                                                                               : AT(yb, i - rb);
    }
    // sum over the rows of p + n, and of log p + log n (wave-reduced)
    __device__ static void pn_sums(const Dims& dm, const Ws& ws, int b, int lane, double al, double* lin, double* bar) {
        const int ne = n_rows(dm);
        double l = 0, g = 0;
        for (int i = lane; i < ne; i += 64) {
            const double pp = AT(rp, i) + al * AT(rdp, i), nn = AT(rn, i) + al * AT(rdn, i);
            l += pp + nn;
            g += log(pp) + log(nn);
        }
        *lin = wsum(l);
        *bar = wsum(g);
    }
    // zeta / 2 ||D_R (x + al dx - x_R)||^2 over x = (X, U, S)
    __device__ static double proximity(const Dims& dm, const Ws& ws, int b, int lane, double al) {
        const double* ori = &AT(wdi, 0);
        const int N = dm.N, oU = ws.L_X, oS = oU + ws.L_U;
        double q = 0;
        auto add = [&](double x, double xr) {
            const double dr = fmin(1.0, 1.0 / fabs(xr)), v = dr * (x - xr);
            q += v * v;
        };
        for (int i = lane; i < (N + 1) * NX; i += 64) add(AT(X, i) + al * AT(dX, i), ori[i]);
        for (int i = lane; i < N * NU; i += 64) add(AT(U, i) + al * AT(dU, i), ori[oU + i]);
        if (dm.ns)
            for (int k = lane; k <= N; k += 64) add(AT(S, k) + al * AT(dS, k), ori[oS + k]);
        return 0.5 * SC(SC_ZETA) * wsum(q);
    }
};

template <int DYN>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(NLOT_WPE_RA))) void k_resto_a(
    const NlotProblem* __restrict__ pp_, const Dims* __restrict__ dd_, NlotSolverOptions o, const Ws* __restrict__ ws_,
    const int* __restrict__ actr, const double* __restrict__ x0, const double* __restrict__ xg, int* cnt) {
    const NlotProblem& p = *pp_;
    const Dims& dm = *dd_;
    const Ws& ws = *ws_;
    using SV = Solver<DYN>;
    using RS = Resto<DYN>;
    constexpr int NX = SV::NX, NU = SV::NU;
    const int lane = threadIdx.x, nlist = cnt[5];
    // grid-stride over the restoration list (the host sizes the grid by a stale bound)
    auto body = [&](const int b) {
    if (SC(SC_RESTO) == 0.0) return;
    const int ph = (int)SC(SC_PHASE);
    if (ph != PH_RINIT && ph != PH_EVAL) return;
    // k_ric<DYN, true>'s inertia correction continues (attempt cap): the stages and the delta_w state are kept
    if (ph == PH_EVAL && SC(SC_RETRY) >= 0.0) return;
    const bool init = ph == PH_RINIT;
    const int N = dm.N, M = dm.M, nc = dm.nc, rank = (int)SC(SC_RANK);
    const int rt = NX + N * NX, rq = rt + nc, rb = rq + (N + 1) * M, ne = RS::n_rows(dm), ngb = ne - rb;
    const double kappa_d = 1e-5;
    const double* x0b = x0 + (size_t)b * NX;
    const double* xgb = xg + (size_t)b * NX;
    double* ori = &AT(wdi, 0);
    const int oU = ws.L_X, oS = oU + ws.L_U, oT = oS + ws.L_S, oyi = oT + ws.L_T, oyk = oyi + ws.L_yi,
              oyt = oyk + ws.L_yk, oyd = oyt + ws.L_yt, ozl = oyd + ws.L_yd, ozu = ozl + ws.L_zl, ozs = ozu + ws.L_zu,
              ovt = ozs + ws.L_zs, osb = ovt + ws.L_vt;
    (void)oyi; (void)oyk; (void)oyt; (void)oyd;
    // ---- evaluation at X: constraint values and Jacobians; the restoration multipliers weight Hd (0 at PH_RINIT)
    for (int k = lane; k <= N; k += 64) {
        double xk[NX], d[MMAX], gk[MMAX][3], w[MMAX], Hw[6];
#pragma unroll
        for (int i = 0; i < NX; ++i) xk[i] = AT(X, k * NX + i);
#pragma unroll
        for (int j = 0; j < MMAX; ++j) w[j] = (!init && j < M) ? AT(yd, k * M + j) : 0.0;
        knot_eval(p, dm, ws, rank, k, xk, d, gk, w, Hw);
#pragma unroll
        for (int j = 0; j < MMAX; ++j) {
            if (j >= M) break;
            AT(dv, k * M + j) = d[j] + (dm.sd ? AT(S, k) : 0.0);
#pragma unroll
            for (int a = 0; a < 3; ++a) AT(Jd, (k * M + j) * 3 + a) = gk[j][a];
        }
        for (int q = 0; q < 6; ++q) AT(Hd, k * 6 + q) = init ? 0.0 : Hw[q];
    }
    wsync();
    // ---- the original constraints c(x) (IPOPT sign): theta_o = ||c||_1, pinf = ||c||_inf
    for (int i = lane; i < NX; i += 64) AT(rci, i) = AT(X, i) - x0b[i];
    for (int i = lane; i < nc; i += 64) AT(rct, i) = AT(X, N * NX + dm.tidx[i]) - xgb[dm.tidx[i]];
    for (int k = lane; k < N; k += 64) {
        double x[NX], u[NU], f[NX];
#pragma unroll
        for (int i = 0; i < NX; ++i) x[i] = AT(X, k * NX + i);
#pragma unroll
        for (int i = 0; i < NU; ++i) u[i] = AT(U, k * NU + i);
        Dyn<DYN>::f(x, u, p.wheelbase, f, p.dt);
#pragma unroll
        for (int i = 0; i < NX; ++i) AT(rcd, k * NX + i) = AT(X, (k + 1) * NX + i) - (x[i] + p.dt * f[i]);
    }
    for (int q = lane; q < (N + 1) * M; q += 64) AT(rcq, q) = AT(dv, q) - AT(T, q);
    for (int q = lane; q < ngb; q += 64) AT(rcb, q) = (q < N * NU ? AT(U, q) : AT(S, q - N * NU)) - AT(sb, q);
    wsync();
    auto crow = [&](int i) {  // c of restoration row i
        return i < NX ? AT(rci, i) : i < rt ? AT(rcd, i - NX) : i < rq ? AT(rct, i - rt) : i < rb ? AT(rcq, i - rq)
                                                                                                 : AT(rcb, i - rb);
    };
    double th_o = 0, pinf = 0;
    for (int i = lane; i < ne; i += 64) {
        const double c = fabs(crow(i));
        th_o += c;
        pinf = fmax(pinf, c);
    }
    th_o = wsum(th_o);
    pinf = wmax(pinf);
    // the original barrier merit at this point with the original problem's mu: ln of every bound slack, the linear
    // damping on one-sided ones
    auto phi_orig = [&](double mu_o) {
        double bar = 0, lin = 0;
        for (int q = lane; q < (N + 1) * M; q += 64) {
            bar += log(AT(T, q));
            lin += AT(T, q);
        }
        for (int e = lane; e < N * NU; e += 64) {
            const double u = BVU(e);
            bar += log(u - p.umin[e % NU]) + log(p.umax[e % NU] - u);
        }
        if (dm.ns)
            for (int k = lane; k <= N; k += 64) {
                bar += log(BVS(k));
                lin += BVS(k);
            }
        return objective_w(p, dm, ws, b, lane, 0.0) - mu_o * wsum(bar) + kappa_d * mu_o * wsum(lin);
    };
    if (init) {
        // MinC_1Nrm initialisation: x_R = x, mu = max(mu, ||c||_inf), p / n minimising the barrier problem for fixed
        // x (IPOPT eq. (33)), bound multipliers capped at rho, equality multipliers 0
        const double mu_o = SC(SC_MU), ph_R = phi_orig(mu_o);
        iter_io(ws, b, lane, ori, true);
        const double mu = fmax(mu_o, pinf), rho = o.resto_penalty_parameter;
        wsync();
        for (int i = lane; i < ne; i += 64) {
            const double c = crow(i);
            const double a = (mu - rho * c) / (2.0 * rho);
            const double n = a + sqrt(a * a + mu * c / (2.0 * rho));
            AT(rn, i) = n;
            AT(rp, i) = c + n;
            AT(rzp, i) = mu / (c + n);
            AT(rzn, i) = mu / n;
        }
        for (int e = lane; e < N * NU; e += 64) {
            AT(zl, e) = fmin(rho, AT(zl, e));
            AT(zu, e) = fmin(rho, AT(zu, e));
        }
        for (int k = lane; k <= N; k += 64) AT(zs, k) = fmin(rho, AT(zs, k));
        for (int q = lane; q < (N + 1) * M; q += 64) {
            AT(vt, q) = fmin(rho, AT(vt, q));
            AT(yd, q) = 0.0;
        }
        for (int i = lane; i < NX; i += 64) AT(yi, i) = 0.0;
        for (int i = lane; i < N * NX; i += 64) AT(yk, i) = 0.0;
        for (int i = lane; i < 8; i += 64) AT(yt, i) = 0.0;
        for (int q = lane; q < ngb; q += 64) AT(yb, q) = 0.0;
        wsync();
        // the restoration's theta_max / theta_min from its merit at the start (proximity term 0 at x_R)
        double th0 = 0;
        for (int i = lane; i < ne; i += 64) th0 += fabs(crow(i) - AT(rp, i) + AT(rn, i));
        th0 = wsum(th0);
        if (lane == 0) {
            SC(SC_RMUO) = mu_o;
            SC(SC_RTAUO) = SC(SC_TAU);
            SC(SC_RDWO) = SC(SC_DWLAST);
            SC(SC_DWLAST) = 0.0;
            SC(SC_THR) = th_o;
            SC(SC_PHR) = ph_R;
            SC(SC_RHO) = rho;
            SC(SC_ZETA) = o.resto_proximity_weight * sqrt(mu);
            SC(SC_RTHMAX) = 1e4 * fmax(1.0, th0);
            SC(SC_RTHMIN) = 1e-4 * fmax(1.0, th0);
            SC(SC_RNFILT) = 0;
            SC(SC_MU) = mu;
            SC(SC_TAU) = fmax(0.99, 1.0 - mu);
            SC(SC_RFIRST) = 1;
            SC(SC_PHASE) = PH_EVAL;
            SC(SC_NRESTO) = SC(SC_NRESTO) + 1;
        }
        wsync();
    }
    const bool first = SC(SC_RFIRST) != 0.0;
    const double rho = SC(SC_RHO), zeta = SC(SC_ZETA), mu0 = SC(SC_MU);
    // ---- the restoration problem's residuals c(x) - p + n
    for (int i = lane; i < NX; i += 64) AT(rci, i) += -AT(rp, i) + AT(rn, i);
    for (int i = lane; i < N * NX; i += 64) AT(rcd, i) += -AT(rp, NX + i) + AT(rn, NX + i);
    for (int j = lane; j < nc; j += 64) AT(rct, j) += -AT(rp, rt + j) + AT(rn, rt + j);
    for (int q = lane; q < (N + 1) * M; q += 64) AT(rcq, q) += -AT(rp, rq + q) + AT(rn, rq + q);
    for (int q = lane; q < ngb; q += 64) AT(rcb, q) += -AT(rp, rb + q) + AT(rn, rb + q);
    wsync();
    // ---- optimality measures of the restoration problem (oracle errors(), resto branch)
    double dual = 0, primal = 0, c0 = 0, cmu = 0, ysum = 0, zsum = 0, nzc = 0;
    auto dual_ = [&](double v) { dual = fmax(dual, fabs(v)); };
    for (int k = lane; k <= N; k += 64) {
        double r[NX];
#pragma unroll
        for (int i = 0; i < NX; ++i) {
            const double xr = ori[k * NX + i], dr = fmin(1.0, 1.0 / fabs(xr));
            r[i] = zeta * dr * dr * (AT(X, k * NX + i) - xr);
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
#pragma unroll
            for (int i = 0; i < NX; ++i)
                for (int cc = 0; cc < nc; ++cc)
                    if (dm.tidx[cc] == i) r[i] += AT(yt, cc);
        for (int j = 0; j < M; ++j)
            for (int a = 0; a < 3 && a < NX; ++a) r[a] += AT(Jd, (k * M + j) * 3 + a) * AT(yd, k * M + j);
#pragma unroll
        for (int i = 0; i < NX; ++i) dual_(r[i]);
        if (k < N)
#pragma unroll
            for (int i = 0; i < NU; ++i) {
                const double ur = ori[oU + k * NU + i], dr = fmin(1.0, 1.0 / fabs(ur));
                double t = zeta * dr * dr * (AT(U, k * NU + i) - ur) +
                           (dm.gcb ? AT(yb, k * NU + i) : -AT(zl, k * NU + i) + AT(zu, k * NU + i));
#pragma unroll
                for (int a = 0; a < NX; ++a) t -= Bu[a][i] * AT(yk, k * NX + a);
                dual_(t);
            }
        if (dm.ns) {
            const double sr = ori[oS + k], dr = fmin(1.0, 1.0 / fabs(sr));
            double t = zeta * dr * dr * (AT(S, k) - sr) + (dm.gcb ? AT(yb, N * NU + k) : -AT(zs, k));
            if (dm.sd)
                for (int j = 0; j < M; ++j) t += AT(yd, k * M + j);
            dual_(t);
        }
        for (int j = 0; j < M; ++j) dual_(-AT(yd, k * M + j) - AT(vt, k * M + j));
    }
    auto compl_ = [&](double z, double sl) {
        c0 = fmax(c0, fabs(z * sl));
        cmu = fmax(cmu, fabs(z * sl - mu0));
        zsum += fabs(z);
        nzc += 1;
    };
    for (int i = lane; i < ne; i += 64) {  // p and n rows: rho -+ y - z = 0, z p = mu, z n = mu
        const double y = RS::yrow(dm, ws, b, i);
        dual_(rho - y - AT(rzp, i));
        dual_(rho + y - AT(rzn, i));
        compl_(AT(rzp, i), AT(rp, i));
        compl_(AT(rzn, i), AT(rn, i));
        primal = fmax(primal, fabs(crow(i)));
        ysum += fabs(y);
    }
    for (int e = lane; e < N * NU; e += 64) {
        const double u = BVU(e);
        compl_(AT(zl, e), u - p.umin[e % NU]);
        compl_(AT(zu, e), p.umax[e % NU] - u);
    }
    if (dm.ns)
        for (int k = lane; k <= N; k += 64) compl_(AT(zs, k), BVS(k));
    for (int q = lane; q < (N + 1) * M; q += 64) compl_(AT(vt, q), AT(T, q));
    for (int q = lane; q < ngb; q += 64)  // bound-row slacks: -y - z_L + z_U
        dual_(q < N * NU ? -AT(yb, q) - AT(zl, q) + AT(zu, q) : -AT(yb, q) - AT(zs, q - N * NU));
    dual = wmax(dual);
    primal = wmax(primal);
    c0 = wmax(c0);
    cmu = wmax(cmu);
    zsum = wsum(zsum);
    ysum = wsum(ysum);
    nzc = wsum(nzc);
    const double sd = fmax(100.0, (ysum + zsum) / ((double)ne + nzc)) / 100.0;
    const double scc = fmax(100.0, zsum / nzc) / 100.0;
    const double E0 = fmax(fmax(dual / sd, primal), c0 / scc);
    const int iters = (int)SC(SC_ITERS);
    wsync();
    auto finish = [&](int status) {
        if (lane == 0) {
            SC(SC_E0) = E0;
            SC(SC_STATUS) = status;
            SC(SC_PHASE) = PH_DONE;
        }
    };
    if (!isfinite(E0)) return finish(NLOT_NUMERIC);
    if (!first) {
        // RestoConvergenceCheck: back to the original problem once theta_o <= kappa_resto theta_R and the point is
        // acceptable to the original filter (sufficient decrease against (theta_R, phi_R))
        const double mu_o = SC(SC_RMUO), th_R = SC(SC_THR), ph_R = SC(SC_PHR);
        const double ph_o = phi_orig(mu_o);
        const double gt = 1e-5, gp = 1e-8;
        int bad = 0;
        const int nf = (int)SC(SC_NFILT);
        for (int i = lane; i < nf; i += 64)
            if (!(th_o <= AT(filt, 2 * i) || ph_o <= AT(filt, 2 * i + 1))) bad = 1;
        const bool back = th_o <= o.required_infeasibility_reduction * th_R && wmax((double)bad) == 0.0 &&
                          (cmp_le(th_o, (1.0 - gt) * th_R, th_R) || cmp_le(ph_o - ph_R, -gp * th_R, ph_R));
        if (back) {
            // leave the restoration phase: the bound multipliers of the original problem take one complementarity
            // Newton step from their saved values over the whole phase (fraction to the boundary with the original
            // tau), reset to 1 above bound_mult_reset_threshold; the equality multipliers restart at 0
            const double tau_o = SC(SC_RTAUO);
            double az = 1.0, zmax = 0;
            auto dz = [&](double z, double so, double sn) { return (mu_o - z * sn) / so; };
            // the bounded quantities at x_R and now: U / S, or the bound rows' slacks (general bounds)
            const int oBU = dm.gcb ? osb : oU, oBS = dm.gcb ? osb + N * NU : oS;
            for (int e = lane; e < N * NU; e += 64) {
                const double lo = p.umin[e % NU], hi = p.umax[e % NU], uo = ori[oBU + e], un = BVU(e);
                AT(dzl, e) = dz(ori[ozl + e], uo - lo, un - lo);
                AT(dzu, e) = dz(ori[ozu + e], hi - uo, hi - un);
                az = frac_to_bound(ori[ozl + e], AT(dzl, e), tau_o, az);
                az = frac_to_bound(ori[ozu + e], AT(dzu, e), tau_o, az);
            }
            if (dm.ns)
                for (int k = lane; k <= N; k += 64) {
                    AT(dzs, k) = dz(ori[ozs + k], ori[oBS + k], BVS(k));
                    az = frac_to_bound(ori[ozs + k], AT(dzs, k), tau_o, az);
                }
            for (int q = lane; q < (N + 1) * M; q += 64) {
                AT(dvt, q) = dz(ori[ovt + q], ori[oT + q], AT(T, q));
                az = frac_to_bound(ori[ovt + q], AT(dvt, q), tau_o, az);
            }
            az = wmin(az);
            for (int e = lane; e < N * NU; e += 64) {
                AT(zl, e) = ori[ozl + e] + az * AT(dzl, e);
                AT(zu, e) = ori[ozu + e] + az * AT(dzu, e);
                zmax = fmax(zmax, fmax(AT(zl, e), AT(zu, e)));
            }
            if (dm.ns)
                for (int k = lane; k <= N; k += 64) {
                    AT(zs, k) = ori[ozs + k] + az * AT(dzs, k);
                    zmax = fmax(zmax, AT(zs, k));
                }
            for (int q = lane; q < (N + 1) * M; q += 64) {
                AT(vt, q) = ori[ovt + q] + az * AT(dvt, q);
                zmax = fmax(zmax, AT(vt, q));
                AT(yd, q) = 0.0;
            }
            zmax = wmax(zmax);
            if (zmax > o.bound_mult_reset_threshold) {
                for (int e = lane; e < N * NU; e += 64) AT(zl, e) = AT(zu, e) = 1.0;
                for (int k = lane; k <= N; k += 64) AT(zs, k) = 1.0;
                for (int q = lane; q < (N + 1) * M; q += 64) AT(vt, q) = 1.0;
            }
            for (int i = lane; i < NX; i += 64) AT(yi, i) = 0.0;
            for (int i = lane; i < N * NX; i += 64) AT(yk, i) = 0.0;
            for (int i = lane; i < 8; i += 64) AT(yt, i) = 0.0;
            for (int q = lane; q < ngb; q += 64) AT(yb, q) = 0.0;
            wsync();
            // SC_RESTO = 2, "returning": k_resto_a runs on the restoration stream concurrently with this step's
            // k_iter_a, which passes the instance by; k_accept (after the join) ends the phase and lists the point's
            // corners for the next step's full launch, whose k_iter_a takes the iteration from there (the same
            // evaluation one global step later: the instance's arithmetic is unchanged)
            if (lane == 0) {
                SC(SC_MU) = mu_o;
                SC(SC_TAU) = tau_o;
                SC(SC_DWLAST) = SC(SC_RDWO);
                SC(SC_RESTO) = 2;
                SC(SC_INSOFT) = 0;
                SC(SC_SOFTCNT) = 0;
                SC(SC_WD) = 0;
                SC(SC_WDSHORT) = 0;
                SC(SC_TINYLAST) = 0;
            }
            return;
        }
        if (E0 <= o.tol) {  // the restoration problem converged at a point the original problem does not accept
            const double thr = o.resto_failure_feasibility_threshold > 0 ? o.resto_failure_feasibility_threshold
                                                                          : 1e2 * o.tol;
            return finish(pinf <= thr ? NLOT_RESTO_FAILED : NLOT_INFEASIBLE);
        }
    }
    if (lane == 0) SC(SC_RFIRST) = 0;
    if (iters >= o.max_iter) return finish(NLOT_MAXITER);
    // ---- monotone barrier update inside the restoration phase
    const double kap = o.barrier_tol_factor, mu_floor = fmin(o.tol, o.compl_inf_tol) / (kap + 1.0);
    double mu = mu0, tau = SC(SC_TAU);
    bool reset_filter = false;
    for (;;) {
        const double Emu = fmax(fmax(dual / sd, primal), cmu / scc);
        if (Emu > kap * mu) break;
        const double nm = fmax(fmin(0.2 * mu, pow(mu, 1.5)), mu_floor);
        if (nm >= mu) break;
        mu = nm;
        tau = fmax(0.99, 1.0 - mu);
        reset_filter = true;
        double cm = 0;
        auto cmx = [&](double z, double sl) { cm = fmax(cm, fabs(z * sl - mu)); };
        for (int i = lane; i < ne; i += 64) {
            cmx(AT(rzp, i), AT(rp, i));
            cmx(AT(rzn, i), AT(rn, i));
        }
        for (int e = lane; e < N * NU; e += 64) {
            const double u = BVU(e);
            cmx(AT(zl, e), u - p.umin[e % NU]);
            cmx(AT(zu, e), p.umax[e % NU] - u);
        }
        if (dm.ns)
            for (int k = lane; k <= N; k += 64) cmx(AT(zs, k), BVS(k));
        for (int q = lane; q < (N + 1) * M; q += 64) cmx(AT(vt, q), AT(T, q));
        cmu = wmax(cm);
    }
    wsync();
    if (lane == 0) {
        SC(SC_MU) = mu;
        SC(SC_TAU) = tau;
        if (reset_filter) SC(SC_RNFILT) = 0;
    }
    wsync();
    SV::build_stages_resto(p, dm, ws, b, lane, 0.0, mu, &AT(stg, 0));
    if (lane == 0) {
        SC(SC_E0) = E0;
        SC(SC_RMU0) = mu;
        SC(SC_RMU1) = 0.0;
        SC(SC_RNR) = 1;
        SC(SC_USEQF) = 0.0;
        SC(SC_RICFIX) = -1.0;
        SC(SC_RIC) = 1;
        atomicAdd(&cnt[7], 1);  // statistics: restoration Newton solves (k_ric<DYN, true>)
    }
    };
    for (int idx = blockIdx.x; idx < nlist; idx += gridDim.x) {
        body(actr[idx]);
        wsync();
    }
}

template <int DYN>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(NLOT_WPE_B))) void k_resto_b(
    const NlotProblem* __restrict__ pp_, const Dims* __restrict__ dd_, NlotSolverOptions o, const Ws* __restrict__ ws_,
    const int* __restrict__ actr, int* cnt, float* tp) {
    const NlotProblem& p = *pp_;
    const Dims& dm = *dd_;
    const Ws& ws = *ws_;
    if (ws.prio) __builtin_amdgcn_s_setprio(2);  // NLOT_SETPRIO (see k_ric)
    using SV = Solver<DYN>;
    using RS = Resto<DYN>;
    constexpr int NX = Dyn<DYN>::NX, NU = Dyn<DYN>::NU;
    const int lane = threadIdx.x, nlist = cnt[5];
    auto body = [&](const int b) {
    if (SC(SC_RESTO) == 0.0 || (int)SC(SC_RIC) != 2) return;
    (void)o;
    const int N = dm.N, M = dm.M, nc = dm.nc;
    const int rt = NX + N * NX, rq = rt + nc, rb = rq + (N + 1) * M, ne = RS::n_rows(dm);
    const double kappa_d = 1e-5, dw = SC(SC_DW), mu = SC(SC_MU), tau = SC(SC_TAU), rho = SC(SC_RHO),
                 zeta = SC(SC_ZETA);
    const double* ori = &AT(wdi, 0);
    const int oU = ws.L_X, oS = oU + ws.L_U;
    double amax = 1.0, az = 1.0, gd = 0;
    // p, n and their multipliers' steps of row r given its new multiplier yn (oracle PN_STEP)
    auto pn_step = [&](int r, double yn) {
        const double pp = AT(rp, r), nn = AT(rn, r);
        const double sp = AT(rzp, r) / pp + dw, sn = AT(rzn, r) / nn + dw;
        const double dp = (yn - rho - kappa_d * mu + mu / pp) / sp, dn = (-yn - rho - kappa_d * mu + mu / nn) / sn;
        const double dzp = mu / pp - AT(rzp, r) - (AT(rzp, r) / pp) * dp, dzn = mu / nn - AT(rzn, r) - (AT(rzn, r) / nn) * dn;
        AT(rdp, r) = dp;
        AT(rdn, r) = dn;
        AT(rdzp, r) = dzp;
        AT(rdzn, r) = dzn;
        amax = frac_to_bound(pp, dp, tau, amax);
        amax = frac_to_bound(nn, dn, tau, amax);
        az = frac_to_bound(AT(rzp, r), dzp, tau, az);
        az = frac_to_bound(AT(rzn, r), dzn, tau, az);
        gd += (rho + kappa_d * mu - mu / pp) * dp + (rho + kappa_d * mu - mu / nn) * dn;
    };
    for (int k = lane; k <= N; k += 64) {
        for (int j = 0; j < M; ++j) {  // t, p and n of the inequality row from its new multiplier y~
            const int q = k * M + j, r = rq + q;
            double Jdz = 0;
            for (int a = 0; a < 3 && a < NX; ++a) Jdz += AT(Jd, q * 3 + a) * AT(dX, k * NX + a);
            if (dm.sd) Jdz += AT(dS, k);
            const double t = AT(T, q), v = AT(vt, q), pp = AT(rp, r), nn = AT(rn, r);
            const double st = v / t + dw, sp = AT(rzp, r) / pp + dw, sn = AT(rzn, r) / nn + dw;
            const double C = 1.0 / st + 1.0 / sp + 1.0 / sn;
            const double E = (mu / t - kappa_d * mu) / st + (mu / pp - rho - kappa_d * mu) / sp -
                             (mu / nn - rho - kappa_d * mu) / sn;
            const double yn = (Jdz + AT(rcq, q) - E) / C;
            const double dt_ = (yn + mu / t - kappa_d * mu) / st;
            const double dvt_ = mu / t - v - (v / t) * dt_;
            AT(yd_n, q) = yn;
            AT(dT, q) = dt_;
            AT(dvt, q) = dvt_;
            pn_step(r, yn);
            amax = frac_to_bound(t, dt_, tau, amax);
            az = frac_to_bound(v, dvt_, tau, az);
            gd += (-mu / t + kappa_d * mu) * dt_;
        }
        if (dm.ns) {
            const double s_ = AT(S, k), ds = AT(dS, k), sr = ori[oS + k], dr = fmin(1.0, 1.0 / fabs(sr));
            if (dm.gcb) {  // bound row S - sb with sb, p and n eliminated (oracle recover, resto branch)
                const int qb = N * NU + k;
                const double sv = AT(sb, qb), sig = AT(zs, k) / sv, bg = -mu / sv + kappa_d * mu;
                double Db;
                const double rhs = SV::bound_row_resto(dm, ws, b, qb, sig, bg, dw, mu, &Db);
                const double yn = Db * ds + rhs, db = (yn - bg) / (sig + dw);
                const double dzs_ = mu / sv - AT(zs, k) - sig * db;
                AT(yb_n, qb) = yn;
                AT(dsb, qb) = db;
                AT(dzs, k) = dzs_;
                pn_step(rb + qb, yn);
                amax = frac_to_bound(sv, db, tau, amax);
                az = frac_to_bound(AT(zs, k), dzs_, tau, az);
                gd += zeta * dr * dr * (s_ - sr) * ds + bg * db;
            } else {
                const double dzs_ = mu / s_ - AT(zs, k) - (AT(zs, k) / s_) * ds;
                AT(dzs, k) = dzs_;
                amax = frac_to_bound(s_, ds, tau, amax);
                az = frac_to_bound(AT(zs, k), dzs_, tau, az);
                gd += (zeta * dr * dr * (s_ - sr) - mu / s_ + kappa_d * mu) * ds;
            }
        }
#pragma unroll
        for (int i = 0; i < NX; ++i) {
            const double xr = ori[k * NX + i], dr = fmin(1.0, 1.0 / fabs(xr));
            gd += zeta * dr * dr * (AT(X, k * NX + i) - xr) * AT(dX, k * NX + i);
        }
    }
    for (int i = lane; i < NX; i += 64) pn_step(i, AT(yi_n, i));
    for (int i = lane; i < N * NX; i += 64) pn_step(NX + i, AT(yk_n, i));
    for (int j = lane; j < nc; j += 64) pn_step(rt + j, AT(yt_n, j));
    for (int e = lane; e < N * NU; e += 64) {
        if (dm.gcb) {  // bound row U - sb with sb, p and n eliminated (oracle recover, resto branch)
            const double u = AT(U, e), du = AT(dU, e), ur = ori[oU + e], dr = fmin(1.0, 1.0 / fabs(ur));
            const double sv = AT(sb, e), sl = sv - p.umin[e % NU], su = p.umax[e % NU] - sv;
            const double sig = AT(zl, e) / sl + AT(zu, e) / su, bg = -mu / sl + mu / su;
            double Db;
            const double rhs = SV::bound_row_resto(dm, ws, b, e, sig, bg, dw, mu, &Db);
            const double yn = Db * du + rhs, db = (yn - bg) / (sig + dw);
            const double dzl_ = mu / sl - AT(zl, e) - (AT(zl, e) / sl) * db;
            const double dzu_ = mu / su - AT(zu, e) + (AT(zu, e) / su) * db;
            AT(yb_n, e) = yn;
            AT(dsb, e) = db;
            AT(dzl, e) = dzl_;
            AT(dzu, e) = dzu_;
            pn_step(rb + e, yn);
            amax = frac_to_bound(sl, db, tau, amax);
            amax = frac_to_bound(su, -db, tau, amax);
            az = frac_to_bound(AT(zl, e), dzl_, tau, az);
            az = frac_to_bound(AT(zu, e), dzu_, tau, az);
            gd += zeta * dr * dr * (u - ur) * du + bg * db;
            continue;
        }
        const double u = AT(U, e), sl = u - p.umin[e % NU], su = p.umax[e % NU] - u, du = AT(dU, e);
        const double ur = ori[oU + e], dr = fmin(1.0, 1.0 / fabs(ur));
        const double dzl_ = mu / sl - AT(zl, e) - (AT(zl, e) / sl) * du;
        const double dzu_ = mu / su - AT(zu, e) + (AT(zu, e) / su) * du;
        AT(dzl, e) = dzl_;
        AT(dzu, e) = dzu_;
        amax = frac_to_bound(sl, du, tau, amax);
        amax = frac_to_bound(su, -du, tau, amax);
        az = frac_to_bound(AT(zl, e), dzl_, tau, az);
        az = frac_to_bound(AT(zu, e), dzu_, tau, az);
        gd += (zeta * dr * dr * (u - ur) - mu / sl + mu / su) * du;
    }
    amax = wmin(amax);
    az = wmin(az);
    gd = wsum(gd);
    // the restoration merit at the current point: theta = ||c - p + n||_1, phi = its objective - mu sum ln(bound
    // slacks incl. p, n) + kappa_d mu sum(one-sided slacks)
    double th = 0, bar = 0, lin = 0;
    for (int i = lane; i < NX; i += 64) th += fabs(AT(rci, i));
    for (int i = lane; i < nc; i += 64) th += fabs(AT(rct, i));
    for (int i = lane; i < N * NX; i += 64) th += fabs(AT(rcd, i));
    for (int q = lane; q < (N + 1) * M; q += 64) {
        th += fabs(AT(rcq, q));
        bar += log(AT(T, q));
        lin += AT(T, q);
    }
    for (int e = lane; e < N * NU; e += 64) {
        const double u = BVU(e);
        bar += log(u - p.umin[e % NU]) + log(p.umax[e % NU] - u);
    }
    if (dm.ns)
        for (int k = lane; k <= N; k += 64) {
            bar += log(BVS(k));
            lin += BVS(k);
        }
    for (int q = lane; q < ne - rb; q += 64) th += fabs(AT(rcb, q));  // bound rows (c - p + n)
    double pn_lin, pn_bar;
    RS::pn_sums(dm, ws, b, lane, 0.0, &pn_lin, &pn_bar);
    const double theta = wsum(th);
    const double phi = rho * pn_lin + RS::proximity(dm, ws, b, lane, 0.0) - mu * (wsum(bar) + pn_bar) +
                       kappa_d * mu * (wsum(lin) + pn_lin);
    const double gt = 1e-5, gp = 1e-8;
    double amin = gt;
    if (gd < 0) {
        amin = fmin(gt, gp * theta / (-gd));
        if (theta <= SC(SC_RTHMIN)) amin = fmin(amin, pow(theta, 1.1) / pow(-gd, 2.3));
    }
    amin *= 0.05;
    (void)ne;
    wsync();
    if (lane == 0) {
        SC(SC_RIC) = 0;
        SC(SC_THETA) = theta;
        SC(SC_PHI) = phi;
        SC(SC_GD) = gd;
        SC(SC_AMAX) = amax;
        SC(SC_AMIN) = amin;
        SC(SC_AZ) = az;
        SC(SC_ALPHA) = amax;
        SC(SC_TRIALS) = 0;
        SC(SC_TINY) = 0;
        SC(SC_PHASE) = PH_LS;
    }
    wsync();
    emit_points(p, dm, ws, b, lane, cnt, true, tp, 1, amax);
    };
    for (int idx = blockIdx.x; idx < nlist; idx += gridDim.x) {
        body(actr[idx]);
        wsync();
    }
}

template <int DYN>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(NLOT_WPE_RLS))) void k_resto_ls(
    const NlotProblem* __restrict__ pp_, const Dims* __restrict__ dd_, NlotSolverOptions o, const Ws* __restrict__ ws_,
    const int* __restrict__ actr, const double* __restrict__ x0, const double* __restrict__ xg, int* cnt,
    int* cnt_next, float* tp_next, const float* tval, int nspec_next) {
    const NlotProblem& p = *pp_;
    const Dims& dm = *dd_;
    const Ws& ws = *ws_;
    using RS = Resto<DYN>;
    constexpr int NX = Dyn<DYN>::NX, NU = Dyn<DYN>::NU;
    const int lane = threadIdx.x, nlist = cnt[5];
    auto body = [&](const int b) {
    if (SC(SC_RESTO) == 0.0 || (int)SC(SC_PHASE) != PH_LS) return;
    (void)o;
    const int N = dm.N, M = dm.M, nc = dm.nc;
    const int rt = NX + N * NX, rq = rt + nc, rb = rq + (N + 1) * M, ne = RS::n_rows(dm);
    const double a0 = SC(SC_ALPHA), mu = SC(SC_MU), rho = SC(SC_RHO), kappa_d = 1e-5;
    const int rank0 = (int)SC(SC_RANK), ncand = (int)SC(SC_NCAND);
    const double* x0b = x0 + (size_t)b * NX;
    const double* xgb = xg + (size_t)b * NX;
    const double gt = 1e-5, gp = 1e-8, delta = 1.0, sth = 1.1, sph = 2.3, eta = 1e-8;
    // the restoration merit at x + al d, p + al dp, n + al dn (trial-list slot `rank`)
    auto trial = [&](double al, int rank, double* th_o, double* ph_o) {
        double th = 0, bar = 0, lin = 0;
        auto pr = [&](int r) { return (AT(rp, r) + al * AT(rdp, r)) - (AT(rn, r) + al * AT(rdn, r)); };
        for (int i = lane; i < NX; i += 64) th += fabs(AT(X, i) + al * AT(dX, i) - x0b[i] - pr(i));
        for (int cc = lane; cc < nc; cc += 64) {
            const int ix = N * NX + dm.tidx[cc];
            th += fabs(AT(X, ix) + al * AT(dX, ix) - xgb[dm.tidx[cc]] - pr(rt + cc));
        }
        for (int k = lane; k <= N; k += 64) {
            double xk[NX];
#pragma unroll
            for (int i = 0; i < NX; ++i) xk[i] = AT(X, k * NX + i) + al * AT(dX, k * NX + i);
            if (k < N) {
                double u[NU], f[NX];
#pragma unroll
                for (int i = 0; i < NU; ++i) u[i] = AT(U, k * NU + i) + al * AT(dU, k * NU + i);
                Dyn<DYN>::f(xk, u, p.wheelbase, f, p.dt);
#pragma unroll
                for (int i = 0; i < NX; ++i)
                    th += fabs(AT(X, (k + 1) * NX + i) + al * AT(dX, (k + 1) * NX + i) - (xk[i] + p.dt * f[i]) -
                               pr(NX + k * NX + i));
                if (dm.gcb) {  // bound rows U - sb - p + n, the barrier of sb
#pragma unroll
                    for (int i = 0; i < NU; ++i) {
                        const int qb = k * NU + i;
                        const double sv = AT(sb, qb) + al * AT(dsb, qb);
                        th += fabs(u[i] - sv - pr(rb + qb));
                        bar += log(sv - p.umin[i]) + log(p.umax[i] - sv);
                    }
                } else {
#pragma unroll
                    for (int i = 0; i < NU; ++i) bar += log(u[i] - p.umin[i]) + log(p.umax[i] - u[i]);
                }
            }
            double d[MMAX];
            knot_eval(p, dm, ws, rank, k, xk, d, nullptr, nullptr, nullptr, tval);
            const double sk = AT(S, k) + al * AT(dS, k);
            for (int j = 0; j < M; ++j) {
                const double t = AT(T, k * M + j) + al * AT(dT, k * M + j);
                th += fabs(d[j] + (dm.sd ? sk : 0.0) - t - pr(rq + k * M + j));
                bar += log(t);
                lin += t;
            }
            if (dm.ns) {
                if (dm.gcb) {  // bound row S - sb - p + n
                    const int qb = N * NU + k;
                    const double sv = AT(sb, qb) + al * AT(dsb, qb);
                    th += fabs(sk - sv - pr(rb + qb));
                    bar += log(sv);
                    lin += sv;
                } else {
                    bar += log(sk);
                    lin += sk;
                }
            }
        }
        double pn_lin, pn_bar;
        RS::pn_sums(dm, ws, b, lane, al, &pn_lin, &pn_bar);
        *th_o = wsum(th);
        *ph_o = rho * pn_lin + RS::proximity(dm, ws, b, lane, al) - mu * (wsum(bar) + pn_bar) +
                kappa_d * mu * (wsum(lin) + pn_lin);
    };
    const double rth = SC(SC_THETA), rph = SC(SC_PHI), rgd = SC(SC_GD);
    const int nf = (int)SC(SC_RNFILT);
    auto acceptable = [&](double at, double th, double pht, int* fa) {  // against the restoration's filter
        int ok = isfinite(th) && isfinite(pht) && th <= SC(SC_RTHMAX);
        const int ftype = rgd < 0 && at * pow(-rgd, sph) > delta * pow(rth, sth);
        const int armijo = cmp_le(pht - rph, eta * at * rgd, rph);
        if (ok) {
            if (ftype && rth <= SC(SC_RTHMIN)) {
                ok = armijo;
            } else {
                ok = cmp_le(th, (1.0 - gt) * rth, rth) || cmp_le(pht - rph, -gp * rth, rph);
                if (ok && pht > rph) {
                    const double bas = fabs(rph) > 10.0 ? log10(fabs(rph)) : 1.0;
                    if (log10(pht - rph) > 5.0 + bas) ok = 0;
                }
            }
        }
        if (ok) {
            int bad = 0;
            for (int i = lane; i < nf; i += 64)
                if (!(th <= AT(rfilt, 2 * i) || pht <= AT(rfilt, 2 * i + 1))) bad = 1;
            ok = wmax((double)bad) == 0.0;
        }
        *fa = ok && ftype && armijo;
        return ok;
    };
    int ok = 0, fa = 0, cnd = 0;
    double al = a0;
    for (cnd = 0; cnd < ncand && !ok; ++cnd) {
        al = ldexp(a0, -cnd);
        double th, pht;
        trial(al, rank0 + cnd, &th, &pht);
        ok = acceptable(al, th, pht, &fa);
    }
    wsync();
    if (!ok) {
        const double na = ldexp(a0, -ncand);
        if (lane == 0) {
            SC(SC_ALPHA) = na;
            SC(SC_TRIALS) = SC(SC_TRIALS) + ncand;
            if (na < SC(SC_AMIN)) {  // the restoration phase's line search failed: IPOPT Restoration_Failed
                SC(SC_STATUS) = NLOT_RESTO_FAILED;
                SC(SC_PHASE) = PH_DONE;
            }
        }
        wsync();
        if (!(na < SC(SC_AMIN))) emit_points(p, dm, ws, b, lane, cnt_next, true, tp_next, n_later(na, SC(SC_AMIN), nspec_next), na);
        return;
    }
    if (!fa) filter_add(ws, b, &AT(rfilt, 0), SC_RNFILT, rth, rph, cnt, lane);  // peak / forgotten statistics too
    // accept: primal, p, n and equality multipliers with alpha; bound multipliers (z_p, z_n included) with alpha_z
    const double az = SC(SC_AZ), ks = 1e10;
    auto zupd = [&](double z, double dz, double sl) {
        const double zn = z + az * dz;
        return fmax(fmin(zn, ks * mu / sl), mu / (ks * sl));
    };
    for (int i = lane; i < (N + 1) * NX; i += 64) AT(X, i) += al * AT(dX, i);
    if (dm.gcb) {  // U, S free; the bound rows' slacks and multipliers
        for (int e = lane; e < N * NU; e += 64) AT(U, e) += al * AT(dU, e);
        if (dm.ns)
            for (int k = lane; k <= N; k += 64) AT(S, k) += al * AT(dS, k);
        for (int q = lane; q < dm.ngb; q += 64) {
            const double sv = AT(sb, q) + al * AT(dsb, q);
            AT(sb, q) = sv;
            AT(yb, q) += al * (AT(yb_n, q) - AT(yb, q));
            if (q < N * NU) {
                AT(zl, q) = zupd(AT(zl, q), AT(dzl, q), sv - p.umin[q % NU]);
                AT(zu, q) = zupd(AT(zu, q), AT(dzu, q), p.umax[q % NU] - sv);
            } else {
                AT(zs, q - N * NU) = zupd(AT(zs, q - N * NU), AT(dzs, q - N * NU), sv);
            }
        }
    } else {
    for (int e = lane; e < N * NU; e += 64) {
        const double u = AT(U, e) + al * AT(dU, e);
        AT(U, e) = u;
        AT(zl, e) = zupd(AT(zl, e), AT(dzl, e), u - p.umin[e % NU]);
        AT(zu, e) = zupd(AT(zu, e), AT(dzu, e), p.umax[e % NU] - u);
    }
    if (dm.ns)
        for (int k = lane; k <= N; k += 64) {
            const double s_ = AT(S, k) + al * AT(dS, k);
            AT(S, k) = s_;
            AT(zs, k) = zupd(AT(zs, k), AT(dzs, k), s_);
        }
    }
    for (int q = lane; q < (N + 1) * M; q += 64) {
        const double t = AT(T, q) + al * AT(dT, q);
        AT(T, q) = t;
        AT(vt, q) = zupd(AT(vt, q), AT(dvt, q), t);
        AT(yd, q) += al * (AT(yd_n, q) - AT(yd, q));
    }
    for (int i = lane; i < NX; i += 64) AT(yi, i) += al * (AT(yi_n, i) - AT(yi, i));
    for (int i = lane; i < N * NX; i += 64) AT(yk, i) += al * (AT(yk_n, i) - AT(yk, i));
    for (int i = lane; i < nc; i += 64) AT(yt, i) += al * (AT(yt_n, i) - AT(yt, i));
    for (int i = lane; i < ne; i += 64) {
        const double pp = AT(rp, i) + al * AT(rdp, i), nn = AT(rn, i) + al * AT(rdn, i);
        AT(rp, i) = pp;
        AT(rn, i) = nn;
        AT(rzp, i) = zupd(AT(rzp, i), AT(rdzp, i), pp);
        AT(rzn, i) = zupd(AT(rzn, i), AT(rdzn, i), nn);
    }
    wsync();
    if (lane == 0) {
        SC(SC_ITERS) = SC(SC_ITERS) + 1;
        SC(SC_PHASE) = PH_EVAL;
        SC(SC_ACCSLOT) = (double)(rank0 + cnd - 1);
    }
    wsync();
    emit_points(p, dm, ws, b, lane, cnt_next, false, nullptr, 1, 0.0);
    };
    for (int idx = blockIdx.x; idx < nlist; idx += gridDim.x) {
        body(actr[idx]);
        wsync();
    }
}

// ---------------------------------------------------------------------------------------------
// host driver
// ---------------------------------------------------------------------------------------------
// Per-dynamics compile units (Makefile): NLOT_UNIT = D >= 0 instantiates run<D> and run<D + NLOT_RK4_BIAS> only;
// NLOT_UNIT = -1 holds the C ABI, the statistics and the dispatch; without NLOT_UNIT (tuning builds) one unit does all.
#ifndef NLOT_UNIT
static thread_local NlotSolveStats g_stats;
static int g_timing = 0;  // nlot_set_timing: 0 off; k: one step in each group of k, at position (step / k) % k (rotating)
#else
extern thread_local NlotSolveStats g_stats;
extern int g_timing;
#if NLOT_UNIT < 0
thread_local NlotSolveStats g_stats;
int g_timing = 0;
#endif
#endif

static int validate(const NlotProblem* p, const NlotSolverOptions* o, const NlotMlp* mlp, int64_t B) {
    if (!p || !o) { set_error("null problem/options"); return NLOT_ERR_INVALID; }
    static const int NXS[6] = {4, 4, 3, 5, 4, 7};
    if (p->dynamics < 0 || p->dynamics > 5 || p->nx != NXS[p->dynamics] || p->nu != 2) {
        set_error("dynamics / nx / nu mismatch");
        return NLOT_ERR_INVALID;
    }
    if (p->N < 2 || p->N > 4096 || p->dt <= 0) { set_error("N must be in [2, 4096], dt > 0"); return NLOT_ERR_INVALID; }
    if (o->general_bounds != 0 && o->general_bounds != 1) {
        set_error("general_bounds: 0 variable bounds, 1 constraint rows (CasADi Opti's form)");
        return NLOT_ERR_INVALID;
    }
    if (p->integrator != NLOT_INTEG_EULER && p->integrator != NLOT_INTEG_RK4) {
        set_error("integrator must be NLOT_INTEG_EULER or NLOT_INTEG_RK4"); return NLOT_ERR_INVALID;
    }
    if (p->shape == NLOT_SHAPE_POLYGON && (p->n_body < 1 || p->n_body > MMAX)) {
        set_error("polygon footprint: 1..4 corners"); return NLOT_ERR_INVALID;
    }
    if (p->shape == NLOT_SHAPE_POLYGON && p->nx < 3) { set_error("polygon footprint needs a heading state"); return NLOT_ERR_INVALID; }
    if (p->sdf_kind == NLOT_SDF_MLP && !mlp) { set_error("learned SDF requires an NlotMlp"); return NLOT_ERR_INVALID; }
    if (p->sdf_kind == NLOT_SDF_ANALYTIC && (p->n_obs < 1 || p->n_obs > NLOT_MAX_OBS)) {
        set_error("analytic SDF needs 1..NLOT_MAX_OBS (128) obstacles"); return NLOT_ERR_INVALID;
    }
    if (p->sdf_kind == NLOT_SDF_ANALYTIC) {
        if (p->n_verts < 0 || p->n_verts > NLOT_MAX_VERTS) { set_error("n_verts out of range"); return NLOT_ERR_INVALID; }
        for (int i = 0; i < p->n_obs; ++i) {
            const NlotObstacle& q = p->obs[i];
            if (q.type < NLOT_OBS_CIRCLE || q.type > NLOT_OBS_TRAPEZOID) { set_error("unknown obstacle type"); return NLOT_ERR_INVALID; }
            const bool poly = q.type == NLOT_OBS_POLYGON || q.type == NLOT_OBS_TRAPEZOID;
            if (poly && (q.nv < (q.type == NLOT_OBS_TRAPEZOID ? 4 : 2) || (q.type == NLOT_OBS_TRAPEZOID && q.nv != 4) ||
                         q.v0 < 0 || q.v0 + q.nv > p->n_verts)) {
                set_error("polygon / trapezoid obstacle: vertex range outside verts[0, n_verts) (a trapezoid has 4)");
                return NLOT_ERR_INVALID;
            }
        }
    }
    for (int i = 0; i < p->nu; ++i)
        if (!(p->umin[i] < p->umax[i])) { set_error("control bounds must satisfy min < max"); return NLOT_ERR_INVALID; }
    if (o->max_iter < 0 || o->max_iter > 10000000) { set_error("max_iter must be in [0, 1e7]"); return NLOT_ERR_INVALID; }
    if (o->resto && (o->resto_penalty_parameter <= 0 || o->required_infeasibility_reduction <= 0 ||
                     o->required_infeasibility_reduction >= 1 || o->resto_proximity_weight < 0)) {
        set_error("restoration options: rho > 0, 0 < kappa_resto < 1, proximity weight >= 0");
        return NLOT_ERR_INVALID;
    }
    if (o->max_soc < 0 || o->watchdog_shortened_iter_trigger < 0 || o->watchdog_trial_iter_max < 0) {
        set_error("max_soc / watchdog options must be >= 0");
        return NLOT_ERR_INVALID;
    }
    if (o->mu_strategy != 0 && o->mu_strategy != 1) { set_error("mu_strategy: 0 monotone, 1 adaptive"); return NLOT_ERR_INVALID; }
    if (B <= 0 || B > (int64_t)1 << 26) { set_error("B out of range"); return NLOT_ERR_INVALID; }
    return NLOT_OK;
}

template <int DYN>
int run(const NlotProblem& p, const NlotSolverOptions& o, const NlotMlp* mlp, const double* x0, const double* xg,
               const double* Xinit, double* X, double* U, double* S, double* cost, int32_t* status, int32_t* iters,
               int64_t B, void* workspace, hipStream_t st) {
    Dims dm = make_dims(p);
    dm.gcb = o.general_bounds ? 1 : 0;
    const bool use_mlp = p.sdf_kind == NLOT_SDF_MLP;
    // slots: min(B, max_active) (continuous batching) or B; the workspace holds the slots' state only
    const int cap_slots = (int)(o.max_active > 0 && o.max_active < B ? o.max_active : B);
    Ws ws = carve(dm, cap_slots, use_mlp, workspace);
    ws.oX = X;
    ws.oU = U;
    ws.oS = S;
    ws.ocost = cost;
    ws.ostat = status;
    ws.oiters = iters;
    ws.prio = getenv("NLOT_SETPRIO") ? atoi(getenv("NLOT_SETPRIO")) : 0;
    NlotProblem* dP = (NlotProblem*)((char*)workspace + kHdrProblem);
    Dims* dD = (Dims*)((char*)workspace + kHdrDims);
    Ws* dW = (Ws*)((char*)workspace + kHdrWs);
    static_assert(sizeof(NlotProblem) <= kHdrDims - kHdrProblem && sizeof(Dims) <= kHdrWs - kHdrDims &&
                  sizeof(Ws) <= kHdr - kHdrWs, "workspace header");
    NLOT_HIP_CHECK(hipMemcpyAsync(dP, &p, sizeof(NlotProblem), hipMemcpyHostToDevice, st));
    NLOT_HIP_CHECK(hipMemcpyAsync(dD, &dm, sizeof(Dims), hipMemcpyHostToDevice, st));
    NLOT_HIP_CHECK(hipMemcpyAsync(dW, &ws, sizeof(Ws), hipMemcpyHostToDevice, st));
    const int Bi = (int)B;
    const int64_t P = (int64_t)dm.ppk * (dm.N + 1);
    g_stats = NlotSolveStats{};
    g_stats.filter_capacity = FILT_MAX;
    hipLaunchKernelGGL(k_init_state, dim3(cap_slots), dim3(64), 0, st, dP, dD, o, ws, x0, xg, Xinit, nullptr, nullptr);
    NLOT_HIP_CHECK(hipGetLastError());
    // Steps run ahead of the host: every kernel reads its step's active count on the device (cnt[2] of the
    // step's counter set, written by the previous step's k_accept), and grids are sized by the host's last
    // known count, an upper bound (the active set only shrinks).  The host waits once per KPIPE steps: it
    // then learns the counts (the D2H copies of each step's counters land in a pinned ring) and whether any
    // instance is still active; the at most KPIPE - 1 steps launched past the end exit at once.
    constexpr int KPIPE = 8;
    // host-side resources released on every return path (NLOT_HIP_CHECK returns early)
    struct Res {
        int* hcnt = nullptr;
        hipEvent_t ev[KPIPE][10] = {};  // [8], [9]: the early value launch (NLOT_EARLY_VALUE) on its stream
        hipEvent_t noev[10] = {};       // the untimed steps' (no events)
        bool timed[KPIPE] = {};         // the ring slot's step was timed
        hipStream_t s2 = nullptr, s3 = nullptr, s4 = nullptr;       // side streams: SOC / restoration / early values
        hipEvent_t e_a = nullptr, e_soc = nullptr, e_r = nullptr, e_s = nullptr, e_v0 = nullptr, e_v1 = nullptr;
        ~Res() {
            for (auto& r : ev)
                for (auto& e : r)
                    if (e) (void)hipEventDestroy(e);
            for (hipEvent_t e : {e_a, e_soc, e_r, e_s, e_v0, e_v1})
                if (e) (void)hipEventDestroy(e);
            if (s2) (void)hipStreamDestroy(s2);
            if (s3) (void)hipStreamDestroy(s3);
            if (s4) (void)hipStreamDestroy(s4);
            if (hcnt) (void)hipHostFree(hcnt);
        }
    } res;
    // + 2: the free-slot count and k_admit's error flag, read at every synchronisation
    NLOT_HIP_CHECK(hipHostMalloc((void**)&res.hcnt, (KPIPE * 2 * CSET + 2) * sizeof(int),
                                 hipHostMallocMapped | hipHostMallocCoherent));
    // The second-order corrections (substitution, short) and the restoration instances' Newton solves (a longer
    // sequential sweep, few instances) touch disjoint instances from the main Newton solve: they run on a side
    // stream, forked after k_iter_a, so their latency hides under k_ric's; k_iter_b joins the corrections, the
    // value-MLP launch joins the restoration chain (k_resto_b appends to the same trial list).
    // NLOT_STREAM_PRIO (A/B knob, measured neutral in round 4): 1 = the restoration stream at the highest priority,
    // 2 = the correction stream too; unset: default-priority streams
    int stream_prio = 0;
    if (const char* e = getenv("NLOT_STREAM_PRIO")) stream_prio = atoi(e);
    if (stream_prio > 0) {
        int prio_least = 0, prio_greatest = 0;
        NLOT_HIP_CHECK(hipDeviceGetStreamPriorityRange(&prio_least, &prio_greatest));
        if (stream_prio >= 2) NLOT_HIP_CHECK(hipStreamCreateWithPriority(&res.s2, hipStreamNonBlocking, prio_greatest));
        else NLOT_HIP_CHECK(hipStreamCreateWithFlags(&res.s2, hipStreamNonBlocking));
        NLOT_HIP_CHECK(hipStreamCreateWithPriority(&res.s3, hipStreamNonBlocking, prio_greatest));
    } else {
        NLOT_HIP_CHECK(hipStreamCreateWithFlags(&res.s2, hipStreamNonBlocking));
        NLOT_HIP_CHECK(hipStreamCreateWithFlags(&res.s3, hipStreamNonBlocking));
    }
    NLOT_HIP_CHECK(hipEventCreateWithFlags(&res.e_a, hipEventDisableTiming));
    NLOT_HIP_CHECK(hipEventCreateWithFlags(&res.e_soc, hipEventDisableTiming));
    NLOT_HIP_CHECK(hipEventCreateWithFlags(&res.e_r, hipEventDisableTiming));
    NLOT_HIP_CHECK(hipEventCreateWithFlags(&res.e_s, hipEventDisableTiming));
    NLOT_HIP_CHECK(hipEventCreateWithFlags(&res.e_v0, hipEventDisableTiming));
    NLOT_HIP_CHECK(hipEventCreateWithFlags(&res.e_v1, hipEventDisableTiming));
    NLOT_HIP_CHECK(hipStreamCreateWithFlags(&res.s4, hipStreamNonBlocking));
    hipStream_t s2 = res.s2, s3 = res.s3, s4 = res.s4;
    // stream layout of the step (A/B knobs NLOT_SOC_FORK, NLOT_EARLY_VALUE).  The early value launch (the previous
    // step's line-search candidates evaluated on a fourth stream while this step's evaluations and Newton solves run)
    // is on by default since round 4: +1.3 % at the bench's scheduling with the round-4 MLP kernels (bitwise-equal
    // results, scripts/gpu_r04q.sh; neutral in round 3 when the full MLP launch held one 512-VGPR wave per SIMD)
    int soc_fork = 0, early_value = 1;
    if (const char* e = getenv("NLOT_SOC_FORK")) soc_fork = std::max(0, std::min(2, atoi(e)));
    if (const char* e = getenv("NLOT_EARLY_VALUE")) early_value = atoi(e) != 0;
    const int t_every = g_timing;
    g_stats.timing_every = t_every;
    if (t_every)
        for (int k = 0; k < KPIPE; ++k)
            for (int i = 0; i < 10; ++i) NLOT_HIP_CHECK(hipEventCreate(&res.ev[k][i]));
    MlpOut mo{}, mo_t[2] = {};
    MlpReuse reuse[2] = {};
    if (use_mlp) {
        const int64_t plane = P * (int64_t)cap_slots * NSPEC;  // the MLP output planes hold the slots' points
        mo.val = ws.mo; mo.gx = ws.mo + plane; mo.gy = ws.mo + 2 * plane; mo.hxx = ws.mo + 3 * plane;
        mo.hxy = ws.mo + 4 * plane; mo.hyx = mo.hxy; mo.hyy = ws.mo + 5 * plane;
        mo.sv = mo.sg = mo.sh = 1;
        // trial lists (by step parity): values + ReLU patterns, reused by the next full launch at the
        // accepted point
        static const bool no_reuse = getenv("NLOT_MLP_REUSE") && strcmp(getenv("NLOT_MLP_REUSE"), "0") == 0;
        for (int q = 0; q < 2; ++q) {
            mo_t[q].val = ws.tval[q];
            mo_t[q].sv = 1;
            mo_t[q].mask = ws.tmask[q];
            mo_t[q].mask_plane = plane;
            reuse[q] = MlpReuse{no_reuse ? nullptr : ws.tsrc, ws.tpts[q], ws.tval[q], ws.tmask[q], plane, nullptr};
        }
    }
    g_stats.slots_in_lds = 0;  // stage slots live in the HBM workspace; k_ric stages them through LDS
    const int ric_blocks_per = RicG<DYN>::IPW;
    // speculation while one value launch stays below ~56 GFLOP of forward work: 8192 instances of the metric
    // (P = 204 corners x 33,536 FLOP; measured best of {512, 2048, 8192} x {1, 2} at B = 65536), 138 of the
    // stress config (P = 1028 x 394,752 FLOP)
    int spec_threshold = 8192, spec_bulk = 2;  // 2 step lengths per later round in the bulk: -1.5 % (r03 ab8)
    if (use_mlp) {
        const double H = mlp->dev.H, fwd = 2.0 * (2.0 * H + mlp->dev.n_hidden * H * H + H);
        spec_threshold = (int)std::max(1.0, std::min(1e9, 5.6e10 / (fwd * (double)P)));
    }
    if (const char* e = getenv("NLOT_SPEC_THRESHOLD")) spec_threshold = atoi(e);
    if (const char* e = getenv("NLOT_SPEC_BULK")) spec_bulk = std::max(1, std::min(NSPEC, atoi(e)));
    // k_ric's inertia-correction attempts per launch while more than ric_tries_min instances are active (the rest of
    // an instance's delta_w sequence continues in the next step's launch)
    // (round 5, after the restoration solves joined the cap: at every batch size, +0.8 % metric, +4.9 % benchmark 6,
    // profiles/r05/ab_tries_min_r05az.log; the results do not depend on it)
    int ric_tries = 1, ric_tries_min = 0;
    if (const char* e = getenv("NLOT_RIC_TRIES")) ric_tries = std::max(1, atoi(e));
    if (const char* e = getenv("NLOT_RIC_TRIES_MIN")) ric_tries_min = atoi(e);
    // the same cap for the restoration solves (side stream; NLOT_RESTO_TRIES=0: every attempt in one launch)
    bool resto_tries = true;
    if (const char* e = getenv("NLOT_RESTO_TRIES")) resto_tries = atoi(e) != 0;
    double progress_s = 0, t_prog = 0;
    if (const char* e = getenv("NLOT_PROGRESS")) progress_s = atof(e);
    t_prog = progress_s;
    const auto t_prog0 = std::chrono::steady_clock::now();
    int kpipe = KPIPE;
    if (const char* e = getenv("NLOT_PIPE")) kpipe = std::max(1, std::min(KPIPE, atoi(e)));
    // a safety net against a phase-machine bug, not an iteration limit (max_iter bounds every instance): at most
    // 64 global steps per iteration per admission wave
    const int64_t waves = (B + std::max(1, o.max_active > 0 && o.max_active < Bi ? o.max_active : Bi) - 1) /
                          std::max(1, o.max_active > 0 && o.max_active < Bi ? o.max_active : Bi);
    const int64_t max_steps = ((int64_t)o.max_iter + 2) * 64 * (waves + 1);
    // Continuous batching (o.max_active = capacity < B): the first `capacity` instances start; whenever a host
    // synchronisation finds at least capacity / 32 slots free, the next instances (index order) join the active
    // list and run their INIT step (corners, slack push, least-squares multipliers) in the next step.  Every
    // instance runs the same iteration sequence whenever it starts, so the results do not depend on capacity;
    // what changes is that the latency-bound tail of one group overlaps the bulk of the next.
    const int capacity = cap_slots;
    const int min_admit = std::max(1, capacity / 32);
    int next_admit = capacity;
    bool init_step = true;  // this step runs the INIT pass (step 0, and the step after an admission)
    // grid bound of the restoration kernels (they read the exact list count on the device): every active instance
    // until a synchronisation shows how many are restoring (an instance enters at most one step before)
    // NLOT_RESTO_BOUND=n (test knob, tests/test_resto_gpu.py::test_resto_grid_bound_same_results): the bound forced to
    // at most n, so that the restoration lists outgrow their grids and the kernels' stride over the exact count runs on
    // every restoring step (the results must not change)
    int resto_force = 0;
    if (const char* e = getenv("NLOT_RESTO_BOUND")) resto_force = std::max(1, atoi(e));
    int resto_bound = o.resto ? (resto_force ? std::min(Bi, resto_force) : Bi) : 0;
    int rc = NLOT_OK, n_active = capacity, cur = 0, synced = 0;
    int64_t step = 0;
    NLOT_HIP_CHECK(hipMemsetAsync(ws.cnt, 0, 64 * sizeof(int), st));  // both sets, the free-slot count, error flag
    res.hcnt[0] = capacity;  // step 0's active count (cnt[2] of counter set 0)
    NLOT_HIP_CHECK(hipMemcpyAsync(ws.cnt + 2, res.hcnt, sizeof(int), hipMemcpyHostToDevice, st));
    NLOT_HIP_CHECK(hipStreamSynchronize(st));  // the pinned source is reused below
    // the step's counter bookkeeping as one kernel (k_step_end) writing the pinned ring, or (NLOT_STEP_KERNEL=0) as
    // the D2H / fill / D2D copies it replaces
    bool step_kernel = true;
    if (const char* e = getenv("NLOT_STEP_KERNEL")) step_kernel = atoi(e) != 0;
    int* dcnt = nullptr;
    NLOT_HIP_CHECK(hipHostGetDevicePointer((void**)&dcnt, res.hcnt, 0));
    // fold the counters of steps synced .. last into g_stats (after a synchronisation); updates n_active
    // NLOT_STEP_LOG=path (diagnostics, scripts/step_trace.py): one line per global step appended to path —
    // step, active, full-eval instances, trial slots, reused points, Newton solves, restoration count, corrections,
    // restoration solves, next active
    const char* step_log = getenv("NLOT_STEP_LOG");
    std::vector<int> slog;
    auto fold = [&](int64_t last) {
        for (int64_t sj = synced; sj <= last; ++sj) {
            const int j = (int)(sj % kpipe), qj = (int)(sj & 1);
            const int* hc = res.hcnt + 2 * CSET * j + CSET * qj;
            const int next_active = res.hcnt[2 * CSET * j + CSET * (qj ^ 1) + 2];
            if (step_log) {
                slog.push_back((int)sj);
                slog.push_back(n_active);
                for (int c = 0; c < 8; ++c) slog.push_back(c == 2 ? 0 : hc[c]);
                slog.push_back(next_active);
                for (int c = 8; c < 11; ++c) slog.push_back(hc[c]);
            slog.push_back(hc[15]);
            }
            g_stats.iterations = (int)(sj + 1);
            if (use_mlp) {
                g_stats.mlp_points_full += (int64_t)hc[0] * P;
                g_stats.mlp_points_value += (int64_t)hc[1] * P;
                g_stats.mlp_points_full_reused += (int64_t)hc[3];
                g_stats.mlp_full_launches++;
                g_stats.mlp_value_launches++;
            }
            g_stats.ric_launches++;
            g_stats.ric_solves += hc[4];
            g_stats.ric_soc_solves += hc[6];
            g_stats.ric_resto_solves += hc[7];
            g_stats.filter_peak = std::max(g_stats.filter_peak, hc[11]);
            g_stats.filter_forgotten += hc[12];
            hipEvent_t* e = res.ev[j];
            if (res.timed[j]) {
                g_stats.timed_steps++;
                g_stats.timed_ric_solves += hc[4];
                if (use_mlp) {
                    g_stats.timed_points_full += (int64_t)hc[0] * P;
                    g_stats.timed_points_value += (int64_t)hc[1] * P;
                    g_stats.timed_points_full_reused += (int64_t)hc[3];
                }
            }
            if (res.timed[j] && use_mlp) {
                float a = 0, c = 0;
                (void)hipEventElapsedTime(&a, e[0], e[1]);
                (void)hipEventElapsedTime(&c, e[2], e[3]);
                g_stats.mlp_full_ms += a;
                g_stats.mlp_value_ms += c;
                if (early_value) {
                    float v0 = 0;
                    (void)hipEventElapsedTime(&v0, e[8], e[9]);
                    g_stats.mlp_value_ms += v0;
                }
            }
            if (res.timed[j]) {
                float a = 0, r = 0;
                (void)hipEventElapsedTime(&a, e[4], e[5]);
                (void)hipEventElapsedTime(&r, e[6], e[7]);
                g_stats.iterate_ms += a;
                g_stats.ric_ms += r;
            }
            n_active = next_active;
            if (n_active == 0) break;  // the later steps of this window found nothing to do
        }
        synced = last + 1;
    };
    // the factorising Newton solves (main stream): the lane-group k_ric
    auto launch_ric = [&](const int* list, const int* count, int mode, int* diag, int tries) {
        hipLaunchKernelGGL((k_ric<DYN, false>), dim3((n_active + ric_blocks_per - 1) / ric_blocks_per), dim3(64), 0,
                           st, dP, dD, dW, list, n_active, count, mode, diag, tries);
    };
    for (step = 0; step < max_steps && n_active > 0; ++step) {
        const int* act = ws.act[cur];
        int* nxt = ws.act[cur ^ 1];
        const int* actr = ws.actr[cur];
        int* nxtr = ws.actr[cur ^ 1];
        const int kq = step % kpipe;
        // one step in t_every, at a position in its group of t_every steps that rotates from group to group: the
        // host's synchronisations (and so admissions, INIT steps) fall at a fixed position of the KPIPE window, so a
        // fixed sampling phase would time one kind of step only
        res.timed[kq] = t_every > 0 && step % t_every == (step / t_every) % t_every;
        hipEvent_t* ev = res.timed[kq] ? res.ev[kq] : res.noev;
        // Point lists are appended to by the kernel that moves an instance into the phase needing them
        // (k_iter_b: first line-search round; k_accept: the new iterate, or the next round), so the lists
        // and counters of step s + 1 fill while step s runs: both alternate by step parity q.
        const int q = step & 1;
        int* C = ws.cnt + CSET * q;
        int* Cn = ws.cnt + CSET * (q ^ 1);
        if (!step_kernel) NLOT_HIP_CHECK(hipMemsetAsync(Cn, 0, CSET * sizeof(int), st));
        // the second-order corrections' chain (k_iter_a's SOC pass: their stages; k_ric<DYN, false, true>: the
        // substitutions) needs no MLP evaluation: it forks to the side stream at the start of the step (soc_fork 1),
        // after the full MLP launch (2), or after the one k_iter_a launch that also does the evaluations (0)
        auto soc_chain = [&](bool with_pass) {
            NLOT_HIP_CHECK(hipEventRecord(res.e_s, st));
            NLOT_HIP_CHECK(hipStreamWaitEvent(s2, res.e_s, 0));
            if (with_pass)
                hipLaunchKernelGGL(k_iter_a<DYN>, dim3(n_active), dim3(64), 0, s2, dP, dD, o, dW, act, ws.x0s, ws.xgs,
                                   (int)PASS_SOC, C, Cn);
            hipLaunchKernelGGL((k_ric<DYN, false, true>), dim3((n_active + ric_blocks_per - 1) / ric_blocks_per),
                               dim3(64), 0, s2, dP, dD, dW, ws.socl, n_active, C + 6, (int)MODE_NEWTON, nullptr, 1 << 30);
            NLOT_HIP_CHECK(hipEventRecord(res.e_soc, s2));
            return NLOT_OK;
        };
        if (soc_fork == 1) NLOT_HIP_CHECK((hipError_t)(soc_chain(true) == NLOT_OK ? hipSuccess : hipErrorUnknown));
        // the value launch's first part: the candidates the previous step's k_accept / k_resto_ls listed (ranks
        // [0, C[14]), C[14] = C[1] now) evaluate on a side stream while this step's evaluations and Newton solves run;
        // the second part (after k_iter_b) covers the candidates added since (ranks [C[14], C[1]))
        if (use_mlp && early_value) {
            if (!step_kernel) NLOT_HIP_CHECK(hipMemcpyAsync(C + 14, C + 1, sizeof(int), hipMemcpyDeviceToDevice, st));
            NLOT_HIP_CHECK(hipEventRecord(res.e_v0, st));
            NLOT_HIP_CHECK(hipStreamWaitEvent(s4, res.e_v0, 0));
            if (ev[0]) (void)hipEventRecord(ev[8], s4);
            rc = launch_mlp_strided(mlp->dev, ws.tpts[q], (int64_t)n_active * NSPEC, C + 14, (int)P, 0, nullptr,
                                    mo_t[q], false, s4);
            if (ev[0]) (void)hipEventRecord(ev[9], s4);
            if (rc) break;
            NLOT_HIP_CHECK(hipEventRecord(res.e_v1, s4));
        }
        // speculative backtracking only while the GPU is latency-bound (few active instances); in the
        // throughput-bound bulk it would multiply the value-MLP work for the same accepted steps
        const int nspec = n_active > spec_threshold ? spec_bulk : NSPEC;
        if (use_mlp) {
            if (init_step) hipLaunchKernelGGL(k_points, dim3(n_active), dim3(64), 0, st, dP, dD, dW, act, C);
            if (ev[0]) (void)hipEventRecord(ev[0], st);
            // contiguous rank-major list: P_per = 1, count = (#instances) * P read on the device
            MlpReuse ru = reuse[q ^ 1];  // the previous step's trial list
            ru.nreused = C + 3;          // statistics: points whose forward was reused
            rc = launch_mlp_strided(mlp->dev, ws.pts, n_active, C + 0, (int)P, 0, nullptr, mo, true, st, &ru);
            if (rc) break;
            if (ev[0]) (void)hipEventRecord(ev[1], st);
        }
        if (soc_fork == 2) NLOT_HIP_CHECK((hipError_t)(soc_chain(true) == NLOT_OK ? hipSuccess : hipErrorUnknown));
        if (ev[4]) (void)hipEventRecord(ev[4], st);
        // restoration phases (list actr, count C[5]) on a stream of their own, forked once the step's evaluations are
        // in (they need nothing else of the step; disjoint instances): k_resto_a, their Newton solves, k_resto_b.  An
        // instance k_resto_a returns to the original problem is passed by this step's k_iter_a and continues next
        // step (k_accept); round 5: k_resto_a (one long wavefront per restoring instance, ~0.5 ms) left the main
        // stream's critical path
        const int n_resto = std::min(n_active, resto_bound);
        if (n_resto > 0) {
            NLOT_HIP_CHECK(hipEventRecord(res.e_a, st));
            NLOT_HIP_CHECK(hipStreamWaitEvent(s3, res.e_a, 0));
            hipLaunchKernelGGL(k_resto_a<DYN>, dim3(n_resto), dim3(64), 0, s3, dP, dD, o, dW, actr, ws.x0s, ws.xgs, C);
            hipLaunchKernelGGL((k_ric<DYN, true>), dim3((n_resto + ric_blocks_per - 1) / ric_blocks_per), dim3(64), 0, s3,
                               dP, dD, dW, actr, n_resto, C + 5, (int)MODE_NEWTON, C + 15,
                               resto_tries && n_active > ric_tries_min ? ric_tries : 1 << 30);
            hipLaunchKernelGGL(k_resto_b<DYN>, dim3(n_resto), dim3(64), 0, s3, dP, dD, o, dW, actr, C,
                               use_mlp ? ws.tpts[q] : nullptr);
            NLOT_HIP_CHECK(hipEventRecord(res.e_r, s3));
        }
        if (init_step) {  // INIT: slack push + least-squares multipliers (one Riccati solve)
            hipLaunchKernelGGL(k_iter_a<DYN>, dim3(n_active), dim3(64), 0, st, dP, dD, o, dW, act, ws.x0s, ws.xgs,
                               (int)PASS_INIT, C, Cn);
            launch_ric(act, C + 2, (int)MODE_LSQ, nullptr, 1 << 30);
        }
        hipLaunchKernelGGL(k_iter_a<DYN>, dim3(n_active), dim3(64), 0, st, dP, dD, o, dW, act, ws.x0s, ws.xgs,
                           (int)(soc_fork == 0 ? PASS_ALL : PASS_EVAL), C, Cn);
        if (soc_fork == 0) NLOT_HIP_CHECK((hipError_t)(soc_chain(false) == NLOT_OK ? hipSuccess : hipErrorUnknown));
        // the Newton solves and the corrections run over the compacted lists k_iter_a wrote (ws.ricl / ws.socl,
        // counts C[4] / C[6]; the grids are host bounds, blocks past the count exit): one group per instance that
        // has work, so a launch holds as many wavefronts as it has solves / 4
        if (ev[6]) (void)hipEventRecord(ev[6], st);
        launch_ric(ws.ricl, C + 4, (int)MODE_NEWTON, C + 8, n_active > ric_tries_min ? ric_tries : 1 << 30);
        if (ev[6]) (void)hipEventRecord(ev[7], st);
        NLOT_HIP_CHECK(hipStreamWaitEvent(st, res.e_soc, 0));
        hipLaunchKernelGGL(k_iter_b<DYN>, dim3(n_active), dim3(64), 0, st, dP, dD, o, dW, act, C,
                           use_mlp ? ws.tpts[q] : nullptr, Cn);
        if (n_resto > 0) NLOT_HIP_CHECK(hipStreamWaitEvent(st, res.e_r, 0));
        if (ev[4]) (void)hipEventRecord(ev[5], st);
        if (use_mlp) {
            // the wait for the early part comes before the timing event: ev[2]..ev[3] is the second part's own time
            if (early_value) NLOT_HIP_CHECK(hipStreamWaitEvent(st, res.e_v1, 0));
            if (ev[0]) (void)hipEventRecord(ev[2], st);
            MlpReuse vb{};
            vb.base = C + 14;
            rc = launch_mlp_strided(mlp->dev, ws.tpts[q], (int64_t)n_active * NSPEC, C + 1, (int)P, 0, nullptr,
                                    mo_t[q], false, st, early_value ? &vb : nullptr);
            if (rc) break;
            if (ev[0]) (void)hipEventRecord(ev[3], st);
        }
        // the next round's candidate count uses this step's nspec (n_active only shrinks: speculation
        // starts at most KPIPE steps late; the accepted alpha is the same either way)
        if (n_resto > 0)
            hipLaunchKernelGGL(k_resto_ls<DYN>, dim3(n_resto), dim3(64), 0, st, dP, dD, o, dW, actr, ws.x0s, ws.xgs, C, Cn,
                               use_mlp ? ws.tpts[q ^ 1] : nullptr, use_mlp ? ws.tval[q] : nullptr, nspec);
        hipLaunchKernelGGL(k_accept<DYN>, dim3(n_active), dim3(64), 0, st, dP, dD, o, dW, act, nxt, nxtr, ws.x0s, ws.xgs, C, Cn,
                           use_mlp ? ws.tpts[q ^ 1] : nullptr, use_mlp ? ws.tval[q] : nullptr, nspec);
        NLOT_HIP_CHECK(hipGetLastError());
        // this step's counters (C) and the next step's active count (Cn[2]), before step + 1 clears C
        int* hflag = res.hcnt + KPIPE * 2 * CSET;
        if (step_kernel) {
            hipLaunchKernelGGL(k_step_end, dim3(1), dim3(64), 0, st, ws.cnt, q, dcnt + 2 * CSET * kq,
                               dcnt + KPIPE * 2 * CSET);
        } else {
            NLOT_HIP_CHECK(hipMemcpyAsync(res.hcnt + 2 * CSET * kq, ws.cnt, 2 * CSET * sizeof(int),
                                          hipMemcpyDeviceToHost, st));
        }
        cur ^= 1;
        init_step = false;
        if (kq != kpipe - 1) continue;
        if (!step_kernel)
            NLOT_HIP_CHECK(hipMemcpyAsync(hflag, ws.cnt + 2 * CSET, 2 * sizeof(int), hipMemcpyDeviceToHost, st));
        NLOT_HIP_CHECK(hipStreamSynchronize(st));
        if (hflag[1] != 0) {  // k_admit's shortfall or a list that outgrew its grid (grid_guard): fail now, not at the end
            set_error(grid_error(hflag[1]));
            return NLOT_ERR_INVALID;
        }
        // restoration lists of the window: the next launches' grid bound (their kernels read the exact count)
        int rmax = 0;
        for (int j = 0; j <= kq; ++j) rmax = std::max(rmax, res.hcnt[2 * CSET * j + CSET * (((step - kq + j) & 1) ^ 1) + 5]);
        resto_bound = std::min(Bi, 2 * rmax + 256);
        if (resto_force) resto_bound = std::min(resto_bound, resto_force);
        fold(step);
        if (progress_s > 0) {  // NLOT_PROGRESS=seconds: a line on stderr now and then (long continuous calls)
            const double t = std::chrono::duration<double>(std::chrono::steady_clock::now() - t_prog0).count();
            if (t >= t_prog) {
                fprintf(stderr, "[nlot] %.0f s: step %lld, %d active, %d of %d instances admitted\n", t, (long long)step,
                        n_active, next_admit, Bi);
                fflush(stderr);
                t_prog = t + progress_s;
            }
        }
        if (next_admit < Bi && (capacity - n_active >= min_admit || n_active == 0)) {
            // instances next_admit .. next_admit + n_new - 1 take free slots (the free-slot count is capacity - the
            // next active count: every instance that left the list freed its slot), join the next step's active
            // list, and start (k_init_state on those slots)
            const int n_new = std::min(capacity - n_active, Bi - next_admit);
            int* Cadm = ws.cnt + CSET * ((step + 1) & 1);
            hipLaunchKernelGGL(k_admit, dim3(1), dim3(1024), 0, st, ws.act[cur], Cadm, ws.sinst, ws.freel,
                               ws.cnt + 2 * CSET, next_admit, n_new);
            hipLaunchKernelGGL(k_init_state, dim3(n_new), dim3(64), 0, st, dP, dD, o, ws, x0, xg, Xinit, ws.act[cur],
                               Cadm);
            NLOT_HIP_CHECK(hipGetLastError());
            next_admit += n_new;
            n_active += n_new;
            init_step = true;
        }
    }
    if (rc) return rc;
    if (synced < step) {  // a window the loop left before its synchronisation point
        NLOT_HIP_CHECK(hipStreamSynchronize(st));
        fold(step - 1);
    }
#ifdef NLOT_KPROF
    {
        unsigned long long kp[4][16];
        NLOT_HIP_CHECK(hipStreamSynchronize(st));
        NLOT_HIP_CHECK(hipMemcpyFromSymbol(kp, HIP_SYMBOL(g_kprof), sizeof(kp)));
        const char* kn[4] = {"k_iter_a", "k_iter_b", "k_accept", "k_resto"};
        for (int k = 0; k < 4; ++k)
            if (kp[k][15]) {
                fprintf(stderr, "[kprof] %s waves %llu: us per wave", kn[k], kp[k][15]);
                for (int i = 0; i < 15; ++i)
                    if (kp[k][i]) fprintf(stderr, " [%d] %.2f", i, kp[k][i] * 1e-2 / kp[k][15]);
                fprintf(stderr, "\n");
            }
        const unsigned long long z[4][16] = {};
        NLOT_HIP_CHECK(hipMemcpyToSymbol(HIP_SYMBOL(g_kprof), z, sizeof(z)));
    }
#endif
#ifdef NLOT_RIC_PROF
    {
        unsigned long long hp[3][5];
        NLOT_HIP_CHECK(hipStreamSynchronize(st));
        NLOT_HIP_CHECK(hipMemcpyFromSymbol(hp, HIP_SYMBOL(g_ric_prof), sizeof(hp)));
        const char* kinds[3] = {"newton", "correction", "restoration"};
        for (int k = 0; k < 3; ++k)
            if (hp[k][4])
                fprintf(stderr, "[ric_prof] %s solves %llu: us per solve backward %.2f F1 %.2f F2 %.2f F3+mult %.2f\n",
                        kinds[k], hp[k][4], hp[k][0] * 1e-2 / hp[k][4], hp[k][1] * 1e-2 / hp[k][4],
                        hp[k][2] * 1e-2 / hp[k][4], hp[k][3] * 1e-2 / hp[k][4]);
        const unsigned long long z[3][5] = {};
        NLOT_HIP_CHECK(hipMemcpyToSymbol(HIP_SYMBOL(g_ric_prof), z, sizeof(z)));
    }
#endif
    if (n_active > 0 || next_admit < Bi) {
        set_error("nlot_solve_batch: the global step cap was reached with instances unfinished (phase-machine bug)");
        return NLOT_ERR_INVALID;
    }
    if (step_log && !slog.empty()) {
        if (FILE* f = fopen(step_log, "a")) {
            for (size_t i = 0; i < slog.size(); i += 15) {
                for (int c = 0; c < 15; ++c) fprintf(f, c ? " %d" : "%d", slog[i + c]);
                fputc('\n', f);
            }
            fclose(f);
        }
    }
    // every instance wrote its outputs when it left the active list (k_accept -> retire)
    NLOT_HIP_CHECK(hipMemcpyAsync(res.hcnt, ws.cnt + 2 * CSET, 2 * sizeof(int), hipMemcpyDeviceToHost, st));
    NLOT_HIP_CHECK(hipStreamSynchronize(st));
    if (res.hcnt[1] != 0 || res.hcnt[0] != capacity) {
        set_error(res.hcnt[1] != 0 ? grid_error(res.hcnt[1])
                                   : "nlot_solve_batch: slot bookkeeping mismatch (free slots at the end != capacity)");
        return NLOT_ERR_INVALID;
    }
    return NLOT_OK;
}

#define NLOT_RUN_SIG(D)                                                                                            \
    int run<D>(const NlotProblem&, const NlotSolverOptions&, const NlotMlp*, const double*, const double*,          \
               const double*, double*, double*, double*, double*, int32_t*, int32_t*, int64_t, void*, hipStream_t)
#if defined(NLOT_UNIT) && NLOT_UNIT >= 0
template NLOT_RUN_SIG(NLOT_UNIT);
template NLOT_RUN_SIG(NLOT_UNIT + NLOT_RK4_BIAS);
#elif defined(NLOT_UNIT)
#define NLOT_EXTERN_RUN(D) extern template NLOT_RUN_SIG(D); extern template NLOT_RUN_SIG(D + NLOT_RK4_BIAS);
NLOT_EXTERN_RUN(0) NLOT_EXTERN_RUN(1) NLOT_EXTERN_RUN(2) NLOT_EXTERN_RUN(3) NLOT_EXTERN_RUN(4) NLOT_EXTERN_RUN(5)
#undef NLOT_EXTERN_RUN
#endif
#undef NLOT_RUN_SIG

}  // namespace nlot

#if !defined(NLOT_UNIT) || NLOT_UNIT < 0
extern "C" size_t nlot_solve_workspace_size(const NlotProblem* p, int64_t B) {
    if (!p) return 0;
    nlot::Dims d = nlot::make_dims(*p);
    return nlot::ws_bytes(d, B, p->sdf_kind == NLOT_SDF_MLP);
}
extern "C" size_t nlot_solve_workspace_size_slots(const NlotProblem* p, int64_t B, int32_t max_active) {
    return nlot_solve_workspace_size(p, max_active > 0 && max_active < B ? (int64_t)max_active : B);
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
    if (wbytes < nlot_solve_workspace_size_slots(p, B, o->max_active)) {
        set_error("nlot_solve_batch: workspace too small");
        return NLOT_ERR_WORKSPACE;
    }
    hipStream_t st = (hipStream_t)stream;
    // the dynamics model and the integrator select the instantiation (Euler: DYN; RK4: DYN + NLOT_RK4_BIAS)
#ifdef NLOT_ONLY_DYN  // kernel-tuning builds (make tune): the one instantiation
    if (p->dynamics + (p->integrator == NLOT_INTEG_RK4 ? NLOT_RK4_BIAS : 0) == NLOT_ONLY_DYN)
        return run<NLOT_ONLY_DYN>(*p, *o, mlp, x0, xg, Xinit, X, U, S, cost, status, iters, B, workspace, st);
    set_error("tuning build (NLOT_ONLY_DYN): this dynamics model is not compiled in");
    return NLOT_ERR_INVALID;
#endif
#define NLOT_RUN(D) return run<D>(*p, *o, mlp, x0, xg, Xinit, X, U, S, cost, status, iters, B, workspace, st)
#ifndef NLOT_ONLY_DYN
    switch (p->dynamics + (p->integrator == NLOT_INTEG_RK4 ? NLOT_RK4_BIAS : 0)) {
    case NLOT_POINT_1ST: NLOT_RUN(NLOT_POINT_1ST);
    case NLOT_POINT_2ND: NLOT_RUN(NLOT_POINT_2ND);
    case NLOT_UNICYCLE: NLOT_RUN(NLOT_UNICYCLE);
    case NLOT_UNICYCLE_2ND: NLOT_RUN(NLOT_UNICYCLE_2ND);
    case NLOT_ACKERMANN: NLOT_RUN(NLOT_ACKERMANN);
    case NLOT_ACKERMANN_2ND: NLOT_RUN(NLOT_ACKERMANN_2ND);
    case NLOT_POINT_1ST + NLOT_RK4_BIAS: NLOT_RUN(NLOT_POINT_1ST + NLOT_RK4_BIAS);
    case NLOT_POINT_2ND + NLOT_RK4_BIAS: NLOT_RUN(NLOT_POINT_2ND + NLOT_RK4_BIAS);
    case NLOT_UNICYCLE + NLOT_RK4_BIAS: NLOT_RUN(NLOT_UNICYCLE + NLOT_RK4_BIAS);
    case NLOT_UNICYCLE_2ND + NLOT_RK4_BIAS: NLOT_RUN(NLOT_UNICYCLE_2ND + NLOT_RK4_BIAS);
    case NLOT_ACKERMANN + NLOT_RK4_BIAS: NLOT_RUN(NLOT_ACKERMANN + NLOT_RK4_BIAS);
    case NLOT_ACKERMANN_2ND + NLOT_RK4_BIAS: NLOT_RUN(NLOT_ACKERMANN_2ND + NLOT_RK4_BIAS);
    }
#endif
#undef NLOT_RUN
    set_error("unknown dynamics");
    return NLOT_ERR_INVALID;
}

extern "C" void nlot_set_timing(int32_t every) { nlot::g_timing = every > 0 ? every : 0; }
extern "C" void nlot_last_stats(NlotSolveStats* out) {
    if (out) *out = nlot::g_stats;
}
#endif  // C ABI unit
