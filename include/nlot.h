/*
 * nlot.h — C ABI of the MI355X-native batched trajectory optimiser (libnlot.so).
 *
 * This is the drop-in boundary for the reference's NLP constraint-evaluation hot path
 * (SURVEY.md §8b).  Everything is plain C: POD structs, caller-owned pointers, int return codes,
 * an explicit hipStream_t passed as void*, no exceptions and no global mutable state on the
 * compute entry points (each call uses only its arguments and the caller's workspace).
 *
 * Replaced reference interfaces (file:line under /root/reference):
 *   nlot_sdf_mlp_eval        <- gen/nn_sdf.cpp:57-60  nn_sdf        (value)
 *                               gen/nn_sdf.cpp:67-70  jac_nn_sdf    (gradient)
 *                               gen/nn_sdf.cpp:79-83  adj1_nn_sdf   (lambda * gradient)
 *                               gen/nn_sdf.cpp:91-104 jac_adj1_nn_sdf (lambda * Hessian)
 *                           batched over P points on the device instead of one 1x2 point per call.
 *   nlot_solve_batch         <- src/nlotrajectories/core/runner.py:44-153 RunBenchmark.run
 *                               (NLP of runner.py:46-108 solved by CasADi Opti + IPOPT,
 *                               runner.py:113-133) for B independent start/goal instances.
 *   nn_sdf / jac_nn_sdf / adj1_nn_sdf / jac_adj1_nn_sdf and their _n_in/_n_out/_sparsity_*
 *                            <- gen/nn_sdf.cpp:36-104, same CasADi external signatures, served by
 *                               the model bound with nlot_casadi_bind (host buffers, like CasADi).
 */
#ifndef NLOT_H
#define NLOT_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define NLOT_ABI_VERSION 15

/* ---- error codes ------------------------------------------------------------------------- */
#define NLOT_OK 0
#define NLOT_ERR_INVALID -1    /* bad argument / unsupported configuration */
#define NLOT_ERR_HIP -2        /* HIP runtime error */
#define NLOT_ERR_WORKSPACE -3  /* workspace too small */

/* ---- per-problem solve status (output array `status`) ----------------------------------- */
#define NLOT_SOLVED 0             /* IPOPT "Solve_Succeeded" analogue: E_0 <= tol + abs. tols */
#define NLOT_MAXITER 1            /* max_iter reached (IPOPT Maximum_Iterations_Exceeded)     */
#define NLOT_LS_FAILED 2          /* alpha < alpha_min with restoration switched off (opt.resto = 0) */
#define NLOT_NUMERIC 3            /* non-finite values / inertia correction failed            */
#define NLOT_RESTO_FAILED 4       /* IPOPT Restoration_Failed: restoration line search failed, or it
                                     converged to a feasible point the filter does not accept  */
#define NLOT_INFEASIBLE 5         /* IPOPT Infeasible_Problem_Detected (restoration converged to a
                                     point of local infeasibility)                              */
#define NLOT_TINY_STEP 6          /* IPOPT Search_Direction_Becomes_Too_Small                  */

/* ---- dynamics (core/dynamics.py:7-13, DYNAMICS_CLASS_MAP 151-158) ------------------------ */
enum NlotDynamics {
    NLOT_POINT_1ST = 0,   /* PointMass1stOrder  dynamics.py:33-41  nx=4 nu=2 */
    NLOT_POINT_2ND = 1,   /* PointMass2ndOrder  dynamics.py:44-56  nx=4 nu=2 */
    NLOT_UNICYCLE = 2,    /* Unicycle           dynamics.py:59-73  nx=3 nu=2 */
    NLOT_UNICYCLE_2ND = 3,/* Unicycle2ndOrder   dynamics.py:76-96  nx=5 nu=2 */
    NLOT_ACKERMANN = 4,   /* Ackermann          dynamics.py:99-118 nx=4 nu=2 */
    NLOT_ACKERMANN_2ND = 5/* Ackermann2ndOrder  dynamics.py:121-148 nx=7 nu=2 (vector order as-is) */
};

/* ---- robot geometry (core/geometry.py) --------------------------------------------------- */
enum NlotShape {
    NLOT_SHAPE_DOT = 0,     /* DotGeometry geometry.py:59-70: sdf(x,y) >= 0, slack ignored      */
    NLOT_SHAPE_POLYGON = 1  /* PolygonGeometry geometry.py:73-117 (rectangle 125-135, triangle
                               138-144): soft-min over corners + slack, or per-corner >= 0       */
};

/* ---- analytic obstacles (core/sdf/casadi.py) ---------------------------------------------- */
enum NlotObstacleType {
    NLOT_OBS_CIRCLE = 0,    /* CircleObstacle.approximated_sdf casadi.py:33-41 */
    NLOT_OBS_SQUARE = 1,    /* SquareObstacle.approximated_sdf casadi.py:69-118 */
    NLOT_OBS_POLYGON = 2,   /* PolygonObstacle.approximated_sdf casadi.py:150-186 (EllipticRingObstacle
                               casadi.py:193-248 is a polygon of its arc points); (cx, cy) = centroid */
    NLOT_OBS_TRAPEZOID = 3  /* TrapezoidObstacle.approximated_sdf casadi.py:317-374 (4 vertices) */
};

enum NlotIntegrator {
    NLOT_INTEG_EULER = 0, /* x_{k+1} = x_k + dt f(x_k, u_k), runner.py:62-63 */
    NLOT_INTEG_RK4 = 1    /* x_{k+1} = x_k + dt (k1 + 2 k2 + 2 k3 + k4) / 6 (opt-in, non-parity) */
};

enum NlotSdfKind {
    NLOT_SDF_ANALYTIC = 0, /* MultiObstacle.approximated_sdf casadi.py:385-386 (soft_min union) */
    NLOT_SDF_MLP = 1       /* NNObstacle.approximated_sdf l4casadi.py:241-257 (learned)         */
};

#define NLOT_MAX_OBS 128   /* primitive obstacles (a discr_s of 30 arc points is 58 trapezoids) */
#define NLOT_MAX_VERTS 512 /* polygon / trapezoid vertices of all obstacles */
#define NLOT_MAX_BODY 8
#define NLOT_MAX_NU 4

typedef struct NlotObstacle {
    int32_t type;      /* NlotObstacleType */
    int32_t group;     /* -1: a term of the scene's soft_min; g >= 0: consecutive obstacles of group g are first
                          soft_min'ed together (a MultiObstacle inside the scene: ConvexEllipticRing casadi.py:393-445,
                          ConvexSObstacle casadi.py:448-525), and that value is the scene's term */
    int32_t v0, nv;    /* polygon / trapezoid: vertices verts[v0 .. v0 + nv) in the reference's point order */
    double cx, cy;     /* circle / square: center; polygon: centroid (mean of the points, casadi.py:133) */
    double size;       /* circle: radius; square: side length */
    double margin;
} NlotObstacle;

/* One NLP of runner.py:44-108 (all B instances share it; start/goal differ per instance). */
typedef struct NlotProblem {
    int32_t dynamics;        /* NlotDynamics */
    int32_t shape;           /* NlotShape */
    int32_t nx, nu;          /* must match the dynamics */
    int32_t n_body;          /* polygon corner count (rectangle 4, triangle 3) */
    int32_t N;               /* knots - 1 (solver.N) */
    double body[NLOT_MAX_BODY][2]; /* corners in body frame, geometry.py:125-144 order */
    double wheelbase;        /* Ackermann L */
    double dt;
    int32_t use_slack;       /* runner.py:66-69 */
    int32_t use_smooth;      /* runner.py:91-96 */
    double slack_penalty;    /* rho */
    double smooth_weight;    /* w */
    int32_t enforce_heading; /* runner.py:51-56 */
    int32_t sdf_kind;        /* NlotSdfKind */
    double umin[NLOT_MAX_NU], umax[NLOT_MAX_NU]; /* runner.py:101-103 */
    double softmin_alpha;    /* utils.py:18 alpha = 10 */
    double path_eps;         /* runner.py:81 epsilon = 1e-8 */
    int32_t n_obs;
    int32_t n_verts;
    NlotObstacle obs[NLOT_MAX_OBS];
    double verts[NLOT_MAX_VERTS][2];
    int32_t integrator;      /* NLOT_INTEG_EULER (the reference's defects, runner.py:62-63; default) or NLOT_INTEG_RK4
                                (opt-in classical RK4 step as the defect map; not the reference's NLP) */
    int32_t pad2_;
} NlotProblem;

/* IPOPT options (runner.py:113-125 + IPOPT defaults).  See DESIGN.md §4 for the restatement. */
typedef struct NlotSolverOptions {
    double tol;                  /* 1e-4 (runner.py:118) */
    int32_t max_iter;            /* 1000 (runner.py:117) */
    int32_t mu_strategy;         /* 0 = monotone (Fiacco-McCormick), 1 = adaptive with the quality-function
                                    oracle (the reference's setting, runner.py:118-119; default) */
    double mu_init;              /* 0.1 */
    double barrier_tol_factor;   /* kappa_eps (IPOPT default 10; the reference sets 0.05, runner.py:120) */
    double dual_inf_tol;         /* 1 */
    double constr_viol_tol;      /* 1e-4 */
    double compl_inf_tol;        /* 1e-4 */
    double constr_mult_init_max; /* 1e3 */
    double bound_push;           /* 1e-2 */
    double bound_frac;           /* 1e-2 */
    int32_t max_soc;             /* second-order corrections per iteration (IPOPT default 4) */
    int32_t resto;               /* 1: feasibility restoration phase on line-search failure (IPOPT) */
    int32_t watchdog_shortened_iter_trigger; /* 10 (IPOPT default; 0 switches the watchdog off) */
    int32_t watchdog_trial_iter_max;         /* 3 */
    int32_t max_soft_resto_iters;            /* 10 */
    int32_t max_active;          /* solver scheduling, not an IPOPT option: 0 = all B instances from the start;
                                    n > 0 = continuous batching, at most n instances in flight and the next ones
                                    admitted (in index order) as others finish — per-instance results are the same */
    double kappa_soc;                        /* 0.99 */
    double tiny_step_tol;                    /* 10 eps = 2.22e-15 */
    double tiny_step_y_tol;                  /* 1e-2 */
    double soft_resto_pderror_reduction_factor; /* 0.9999 (0 switches the soft restoration off) */
    double required_infeasibility_reduction; /* kappa_resto = 0.9 */
    double resto_penalty_parameter;          /* rho = 1000 */
    double resto_proximity_weight;           /* zeta = weight * sqrt(mu), weight 1 */
    double bound_mult_reset_threshold;       /* 1000 */
    double resto_failure_feasibility_threshold; /* 0 means 1e2 * tol (IPOPT default) */
    int32_t general_bounds;      /* 1 (default since ABI v12): the control bounds and slack >= 0 as constraint rows
                                    g(x) = U, g(x) = S with bounded IPOPT slacks, U and S free — the NLP CasADi Opti
                                    hands IPOPT (runner.py:67-69,101-103); 0: the same bounds as variable bounds */
    int32_t pad_gb_;
} NlotSolverOptions;

/* Learned SDF: an l4casadi-wrappable torch model, flattened.
 *   FourierMLP (core/nn_architectures.py:30-72):  h0 = scale * cos(p @ A + b0)         (in_kind 1)
 *   l4c.naive.MultiLayerPerceptron:              h0 = act(p @ A + b0)                  (in_kind 0)
 *   SIREN (core/nn_architectures.py:8-26,75-100): in_kind 0 with act = NLOT_ACT_SINE, fourier_scale = omega_0
 *   then n_hidden x  h_{l+1} = act(W_l h_l + b_l);   f = w_out . h + b_out.
 * ReLU nets run on the MFMA kernels (n_hidden 1-4); the smooth activations on the hyper-dual kernel
 * (value, gradient and Hessian propagated forward through every layer; n_hidden 0-4), DESIGN.md §7.
 * All weights fp32 (the reference's l4casadi path evaluates the TorchScript graph in fp32,
 * gen/nn_sdf.cpp casts the CasADi doubles to float).  Host OR device pointers depending on the
 * consumer (nlot_mlp_create copies host arrays to the device). */
#define NLOT_MLP_IN_LINEAR_RELU 0
#define NLOT_MLP_IN_FOURIER 1
/* activations (core/nn_architectures.py:47-52 names; l4casadi naive: ReLU/Tanh/Sigmoid/LeakyReLU) */
#define NLOT_ACT_RELU 0
#define NLOT_ACT_TANH 1
#define NLOT_ACT_SIGMOID 2
#define NLOT_ACT_LEAKY_RELU 3 /* negative slope 0.01 (F.leaky_relu / nn.LeakyReLU default) */
#define NLOT_ACT_SINE 4       /* sin(omega_0 z), SineLayer nn_architectures.py:8-26; omega_0 in fourier_scale */

typedef struct NlotMlpDesc {
    int32_t in_kind;       /* NLOT_MLP_IN_* */
    int32_t hidden;        /* H (multiple of 32, <= 256) */
    int32_t n_hidden;      /* hidden HxH layers (>= 0) */
    int32_t act;           /* NLOT_ACT_* of the hidden layers (and of the input layer when in_kind 0) */
    float fourier_scale;   /* FourierFeatureLayer.scale (in_kind 1); omega_0 when act = NLOT_ACT_SINE */
    float b_out;
    const float* A;        /* [2][H]  (in, out) */
    const float* b0;       /* [H] */
    const float* W;        /* [n_hidden][H][H]  (out, in) = nn.Linear.weight */
    const float* b;        /* [n_hidden][H] */
    const float* w_out;    /* [H] */
} NlotMlpDesc;

typedef struct NlotMlp NlotMlp; /* opaque device-resident weights */

/* ---- version / errors --------------------------------------------------------------------- */
int32_t nlot_abi_version(void);
/* Last error message of the calling thread (thread-local; never NULL). */
const char* nlot_last_error(void);
/* Fill `opt` with the defaults documented above. */
void nlot_default_options(NlotSolverOptions* opt);

/* ---- learned-SDF weights ------------------------------------------------------------------- */
/* Copies the host arrays of `desc` to device memory; returns NULL on error (see nlot_last_error). */
NlotMlp* nlot_mlp_create(const NlotMlpDesc* desc);
/* The net's MFMA arithmetic (ABI v13).  Both are fp32 arithmetic (products exact in the fp32 accumulator); they
 * differ in the MFMA sums' order and so at the rounding level:
 *   NLOT_MLP_ARITH_SPLIT_BF16  operands split into three bf16 parts, six bf16 MFMA products per fp32 product (the
 *                              default of nlot_mlp_create: 2.65x the f32-MFMA peak)
 *   NLOT_MLP_ARITH_F32         v_mfma_f32 products (the reference's fp32 net, gen/nn_sdf.cpp, at the f32 peak)
 *   NLOT_MLP_ARITH_SEQ         (ABI v15; ReLU nets) every sum a sequential fp32 FMA chain in index order, one thread per
 *                              point: a fixed, documented summation order (the test oracle's), for bitwise-reproducible
 *                              comparisons; not a throughput path */
#define NLOT_MLP_ARITH_SPLIT_BF16 0
#define NLOT_MLP_ARITH_F32 1
#define NLOT_MLP_ARITH_SEQ 2
NlotMlp* nlot_mlp_create_ex(const NlotMlpDesc* desc, int32_t arith);
void nlot_mlp_destroy(NlotMlp* mlp);

/* Batched SDF-MLP evaluation on the device (the nn_sdf family, gen/nn_sdf.cpp:57-104).
 *   pts  [P][2] fp32 device, row-major.   val [P] (required).
 *   grad [P][2] or NULL: df/dp.             lam [P] or NULL (NULL = 1): adjoint seed.
 *   hess [P][2][2] or NULL: lam * d2f/dp2 (jac_adj1).  When lam != NULL, grad is lam * df/dp (adj1).
 * `stream` is a hipStream_t (NULL = default stream). Asynchronous. */
int32_t nlot_sdf_mlp_eval(const NlotMlp* mlp, const float* pts, int64_t P, float* val, float* grad,
                          const float* lam, float* hess, void* stream);

/* ---- batched trajectory optimisation ------------------------------------------------------ */
/* Bytes of device workspace nlot_solve_batch needs for B instances. */
size_t nlot_solve_workspace_size(const NlotProblem* prob, int64_t B);
/* Bytes for B instances streamed through max_active slots (continuous batching, ABI v10): the workspace holds the
 * slots' state only, so it depends on min(B, max_active), not on B (max_active <= 0: all B at once). */
size_t nlot_solve_workspace_size_slots(const NlotProblem* prob, int64_t B, int32_t max_active);

/* Solve B independent instances of `prob` (start x0[b], goal xg[b]) on the device.
 *   x0, xg    [B][nx] fp64 device
 *   X_init    [B][N+1][nx] fp64 device, or NULL = LinearInitializer (trajectory_initialization.py:54-55)
 *   X         [B][N+1][nx] fp64 device (out)   U [B][N][nu] fp64 (out)   S [B][N+1] fp64 or NULL
 *   cost      [B] fp64 (out: objective value, runner.py:80-98 / run_benchmark.py:166)
 *   status    [B] int32 (out: NLOT_SOLVED ...)   iters [B] int32 (out)
 *   mlp       required iff prob->sdf_kind == NLOT_SDF_MLP
 *   workspace >= nlot_solve_workspace_size_slots(prob, B, opt->max_active) bytes of device memory (per-slot state;
 *             an instance writes its outputs when it finishes, and its slot goes to the next instance).
 * Returns when all instances finished (the host drives the iteration loop on `stream`). */
int32_t nlot_solve_batch(const NlotProblem* prob, const NlotSolverOptions* opt, const NlotMlp* mlp,
                         const double* x0, const double* xg, const double* X_init, double* X,
                         double* U, double* S, double* cost, int32_t* status, int32_t* iters,
                         int64_t B, void* workspace, size_t workspace_bytes, void* stream);

/* Per-solve counters of the last nlot_solve_batch on this thread (host side, for benchmarking). */
typedef struct NlotSolveStats {
    int32_t iterations;        /* lock-step iterations run */
    int32_t ls_rounds;         /* line-search rounds launched */
    int64_t mlp_points_full;   /* points evaluated with value+grad+hess */
    int64_t mlp_points_value;  /* points evaluated value-only (trial points) */
    double mlp_full_ms;        /* summed device time of the full MLP launches (hipEvents) */
    double mlp_value_ms;       /* summed device time of the value-only MLP launches */
    int32_t mlp_full_launches;
    int32_t mlp_value_launches;
    double iterate_ms;         /* summed device time of the solver-step (k_iterate) launches */
    int32_t slots_in_lds;      /* 1: Riccati stage slots held in LDS, 0: in the HBM workspace */
    int32_t pad_;
    int64_t mlp_points_full_reused; /* full-launch points whose forward came from the accepted trial point */
    double ric_ms;             /* summed device time of the Newton-solve (k_ric) launches (hipEvents) */
    int32_t ric_launches;
    int32_t pad2_;
    int64_t ric_solves;        /* instance Newton solves (factorisations) those launches performed */
    int64_t ric_soc_solves;    /* second-order corrections: substitutions with the stored factors (side stream) */
    int64_t ric_resto_solves;  /* restoration-phase Newton solves (side stream) */
    int32_t filter_capacity;   /* entries per filter (line search, adaptive-mu progress, restoration); ABI v11 */
    int32_t filter_peak;       /* the largest size any filter reached */
    int64_t filter_forgotten;  /* entries forgotten at capacity (IPOPT's filter is unbounded: 0 = faithful) */
    /* ABI v14: the *_ms sums above cover the timed global steps only (nlot_set_timing); these count them and the
     * work their launches did (one full MLP, one value MLP in up to two parts, one k_ric launch per step) */
    int32_t timed_steps;
    int32_t timing_every;
    int64_t timed_points_full;
    int64_t timed_points_full_reused;
    int64_t timed_points_value;
    int64_t timed_ric_solves;
} NlotSolveStats;
/* hipEvent timing of the MLP, solver-step and k_ric launches inside nlot_solve_batch: 0 off, 1 every global step,
 * k > 1 one step in each group of k consecutive steps, at the position (group index mod k) (a sample over every
 * position: each timed step adds ~10 event packets to the queue, ~2 % of the step time when every step is timed). */
void nlot_set_timing(int32_t every);
void nlot_last_stats(NlotSolveStats* out);

/* ---- CasADi external compatibility shim (gen/nn_sdf.cpp:36-104) ----------------------------
 * A CasADi user can `casadi.external("nn_sdf", "libnlot.so")` after binding a model.  These are
 * host functions on double buffers owned by CasADi, one 1x2 point per call, exactly like the
 * generated file; they run the MLP on the GPU synchronously.  Bind with nlot_casadi_bind (the
 * reference's static global L4CasADi object, gen/nn_sdf.cpp:3). */
typedef double casadi_real_t;
typedef long long int casadi_int_t;
int32_t nlot_casadi_bind(const NlotMlp* mlp);

/* ---- RRT initializer (core/trajectory_initialization.py:58-239, RRTInitializer) ----------------- */
typedef struct NlotRrtOptions {
    double bounds[2][2];       /* [[xmin, ymin], [xmax, ymax]] sampling box (YAML rrt_bounds) */
    double step_size;          /* extension step (0.05) */
    double margin;             /* safety distance added to the footprint inflation (0.01) */
    double goal_sample_rate;   /* probability of sampling the goal (0.05) */
    uint64_t seed;             /* counter-based RNG seed (the reference draws from Python's global `random`) */
    int32_t max_iter;          /* tree extensions tried (1000) */
    int32_t first_instance;    /* index of instance 0 of this call in the caller's batch (the random stream is keyed by
                                  it: a batch split into calls draws as one call; 0 otherwise) */
} NlotRrtOptions;

/* Bytes of device workspace nlot_rrt_init needs for B instances (tree, path and spline buffers). */
size_t nlot_rrt_workspace_size(const NlotRrtOptions* opt, int64_t B);

/* Batched RRTInitializer.get_initial_guess: per instance, an RRT in the xy plane from x0[b][0:2] to xg[b][0:2]
 * against the scene's EXACT SDF (MultiObstacle.sdf, casadi.py:381-383; the footprint by point inflation,
 * trajectory_initialization.py:108-113), the path with intermediate points at turns > 60 degrees, greedy
 * shortcuts and a not-a-knot cubic spline resampled to N + 1 points; other states 0 (:233-236).
 *   x0, xg   [B][nx] fp64 device      X_init [B][N+1][nx] fp64 device (out)
 *   ok       [B] int32 device (out): 1, or 0 where the reference raises "RRT failed to find a path within max_iter"
 *            (X_init of that instance is then the straight line)
 * Requires prob->sdf_kind-independent obstacles: the analytic scene in prob->obs (the training target in l4casadi
 * mode). Asynchronous on `stream`. */
int32_t nlot_rrt_init(const NlotProblem* prob, const NlotRrtOptions* opt, const double* x0, const double* xg,
                      double* X_init, int32_t* ok, int64_t B, void* workspace, size_t workspace_bytes, void* stream);
casadi_int_t nn_sdf_n_in(void);
casadi_int_t nn_sdf_n_out(void);
const casadi_int_t* nn_sdf_sparsity_in(casadi_int_t i);
const casadi_int_t* nn_sdf_sparsity_out(casadi_int_t i);
int nn_sdf(const casadi_real_t** arg, casadi_real_t** res, casadi_int_t* iw, casadi_real_t* w, int mem);
casadi_int_t jac_nn_sdf_n_in(void);
casadi_int_t jac_nn_sdf_n_out(void);
int jac_nn_sdf(const casadi_real_t** arg, casadi_real_t** res, casadi_int_t* iw, casadi_real_t* w, int mem);
casadi_int_t adj1_nn_sdf_n_in(void);
casadi_int_t adj1_nn_sdf_n_out(void);
int adj1_nn_sdf(const casadi_real_t** arg, casadi_real_t** res, casadi_int_t* iw, casadi_real_t* w, int mem);
casadi_int_t jac_adj1_nn_sdf_n_in(void);
casadi_int_t jac_adj1_nn_sdf_n_out(void);
int jac_adj1_nn_sdf(const casadi_real_t** arg, casadi_real_t** res, casadi_int_t* iw, casadi_real_t* w, int mem);

#ifdef __cplusplus
}
#endif
#endif /* NLOT_H */
