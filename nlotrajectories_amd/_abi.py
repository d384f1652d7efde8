"""ctypes mirrors of the plain-C structs in include/nlot.h (layout must match the header)."""
import ctypes as C

NLOT_OK = 0
NLOT_SOLVED, NLOT_MAXITER, NLOT_LS_FAILED, NLOT_NUMERIC = 0, 1, 2, 3
NLOT_RESTO_FAILED, NLOT_INFEASIBLE, NLOT_TINY_STEP = 4, 5, 6
STATUS_NAMES = {0: "solved", 1: "max_iter", 2: "line_search_failed", 3: "numeric", 4: "restoration_failed",
                5: "infeasible", 6: "tiny_step"}

# NlotDynamics (core/dynamics.py:7-13)
DYNAMICS = {"point_1st": 0, "point_2nd": 1, "unicycle": 2, "unicycle_2nd": 3, "ackermann": 4,
            "ackermann_2nd": 5}
STATE_DIM = {"point_1st": 4, "point_2nd": 4, "unicycle": 3, "unicycle_2nd": 5, "ackermann": 4,
             "ackermann_2nd": 7}
CONTROL_DIM = {k: 2 for k in DYNAMICS}
SHAPE_DOT, SHAPE_POLYGON = 0, 1
OBS_CIRCLE, OBS_SQUARE, OBS_POLYGON, OBS_TRAPEZOID = 0, 1, 2, 3
INTEG_EULER, INTEG_RK4 = 0, 1
SDF_ANALYTIC, SDF_MLP = 0, 1
MLP_IN_LINEAR_RELU, MLP_IN_FOURIER = 0, 1
# hidden activations (include/nlot.h NLOT_ACT_*)
ACT_RELU, ACT_TANH, ACT_SIGMOID, ACT_LEAKY_RELU, ACT_SINE = 0, 1, 2, 3, 4
MAX_OBS, MAX_VERTS, MAX_BODY, MAX_NU = 128, 512, 8, 4


class NlotObstacle(C.Structure):
    _fields_ = [("type", C.c_int32), ("group", C.c_int32), ("v0", C.c_int32), ("nv", C.c_int32),
                ("cx", C.c_double), ("cy", C.c_double), ("size", C.c_double), ("margin", C.c_double)]


class NlotProblem(C.Structure):
    _fields_ = [
        ("dynamics", C.c_int32), ("shape", C.c_int32), ("nx", C.c_int32), ("nu", C.c_int32),
        ("n_body", C.c_int32), ("N", C.c_int32), ("body", (C.c_double * 2) * MAX_BODY),
        ("wheelbase", C.c_double), ("dt", C.c_double), ("use_slack", C.c_int32),
        ("use_smooth", C.c_int32), ("slack_penalty", C.c_double), ("smooth_weight", C.c_double),
        ("enforce_heading", C.c_int32), ("sdf_kind", C.c_int32), ("umin", C.c_double * MAX_NU),
        ("umax", C.c_double * MAX_NU), ("softmin_alpha", C.c_double), ("path_eps", C.c_double),
        ("n_obs", C.c_int32), ("n_verts", C.c_int32), ("obs", NlotObstacle * MAX_OBS),
        ("verts", (C.c_double * 2) * MAX_VERTS), ("integrator", C.c_int32), ("pad2_", C.c_int32),
    ]


class NlotSolverOptions(C.Structure):
    _fields_ = [
        ("tol", C.c_double), ("max_iter", C.c_int32), ("mu_strategy", C.c_int32),
        ("mu_init", C.c_double), ("barrier_tol_factor", C.c_double), ("dual_inf_tol", C.c_double),
        ("constr_viol_tol", C.c_double), ("compl_inf_tol", C.c_double),
        ("constr_mult_init_max", C.c_double), ("bound_push", C.c_double), ("bound_frac", C.c_double),
        ("max_soc", C.c_int32), ("resto", C.c_int32), ("watchdog_shortened_iter_trigger", C.c_int32),
        ("watchdog_trial_iter_max", C.c_int32), ("max_soft_resto_iters", C.c_int32), ("max_active", C.c_int32),
        ("kappa_soc", C.c_double), ("tiny_step_tol", C.c_double), ("tiny_step_y_tol", C.c_double),
        ("soft_resto_pderror_reduction_factor", C.c_double), ("required_infeasibility_reduction", C.c_double),
        ("resto_penalty_parameter", C.c_double), ("resto_proximity_weight", C.c_double),
        ("bound_mult_reset_threshold", C.c_double), ("resto_failure_feasibility_threshold", C.c_double),
        ("general_bounds", C.c_int32), ("pad_gb_", C.c_int32),
    ]


class NlotMlpDesc(C.Structure):
    _fields_ = [
        ("in_kind", C.c_int32), ("hidden", C.c_int32), ("n_hidden", C.c_int32), ("act", C.c_int32),
        ("fourier_scale", C.c_float), ("b_out", C.c_float), ("A", C.POINTER(C.c_float)),
        ("b0", C.POINTER(C.c_float)), ("W", C.POINTER(C.c_float)), ("b", C.POINTER(C.c_float)),
        ("w_out", C.POINTER(C.c_float)),
    ]


class NlotSolveStats(C.Structure):
    _fields_ = [
        ("iterations", C.c_int32), ("ls_rounds", C.c_int32), ("mlp_points_full", C.c_int64),
        ("mlp_points_value", C.c_int64), ("mlp_full_ms", C.c_double), ("mlp_value_ms", C.c_double),
        ("mlp_full_launches", C.c_int32), ("mlp_value_launches", C.c_int32),
        ("iterate_ms", C.c_double), ("slots_in_lds", C.c_int32), ("pad_", C.c_int32),
        ("mlp_points_full_reused", C.c_int64), ("ric_ms", C.c_double), ("ric_launches", C.c_int32),
        ("pad2_", C.c_int32), ("ric_solves", C.c_int64), ("ric_soc_solves", C.c_int64),
        ("ric_resto_solves", C.c_int64), ("filter_capacity", C.c_int32), ("filter_peak", C.c_int32),
        ("filter_forgotten", C.c_int64), ("timed_steps", C.c_int32), ("timing_every", C.c_int32),
        ("timed_points_full", C.c_int64), ("timed_points_full_reused", C.c_int64), ("timed_points_value", C.c_int64),
        ("timed_ric_solves", C.c_int64),
    ]


# IPOPT's globalisation safeguards switched off: the round-1 algorithm (plain filter line search)
SAFEGUARDS_OFF = dict(max_soc=0, resto=0, watchdog_shortened_iter_trigger=0, soft_resto_pderror_reduction_factor=0.0,
                      tiny_step_tol=0.0)


def default_options(**kw) -> NlotSolverOptions:
    """IPOPT settings of runner.py:113-125 plus IPOPT defaults."""
    o = NlotSolverOptions(tol=1e-4, max_iter=1000, mu_strategy=1, mu_init=0.1,
                          barrier_tol_factor=0.05, dual_inf_tol=1.0, constr_viol_tol=1e-4,
                          compl_inf_tol=1e-4, constr_mult_init_max=1e3, bound_push=1e-2,
                          bound_frac=1e-2, max_soc=4, resto=1, watchdog_shortened_iter_trigger=10,
                          watchdog_trial_iter_max=3, max_soft_resto_iters=10, kappa_soc=0.99,
                          tiny_step_tol=10 * 2.220446049250313e-16, tiny_step_y_tol=1e-2,
                          soft_resto_pderror_reduction_factor=0.9999, required_infeasibility_reduction=0.9,
                          resto_penalty_parameter=1000.0, resto_proximity_weight=1.0,
                          bound_mult_reset_threshold=1000.0, resto_failure_feasibility_threshold=0.0,
                          general_bounds=1)
    for k, v in kw.items():
        setattr(o, k, v)
    return o


def gpu_options(**kw) -> NlotSolverOptions:
    """The IPOPT settings the GPU path runs: since round 3 exactly default_options() (second-order corrections,
    watchdog, tiny-step test, soft restoration and the feasibility restoration phase).  Kept as a
    name for callers; NO_RESTO gives the round-2 behaviour (line-search failure ends an instance)."""
    return default_options(**kw)


# restoration switched off: an instance whose line search fails ends with NLOT_LS_FAILED (round-2 GPU behaviour)
NO_RESTO = dict(resto=0, soft_resto_pderror_reduction_factor=0.0)


class NlotRrtOptions(C.Structure):
    """include/nlot.h NlotRrtOptions (RRTInitializer arguments, trajectory_initialization.py:68-81)."""
    _fields_ = [("bounds", (C.c_double * 2) * 2), ("step_size", C.c_double), ("margin", C.c_double),
                ("goal_sample_rate", C.c_double), ("seed", C.c_uint64), ("max_iter", C.c_int32), ("first_instance", C.c_int32)]
