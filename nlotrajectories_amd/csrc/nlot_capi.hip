// C-ABI plumbing of libnlot.so: version, thread-local errors, defaults, and the CasADi external
// compatibility shim (gen/nn_sdf.cpp:36-104 signatures).
#include <hip/hip_runtime.h>

#include <cstring>
#include <mutex>
#include <string>

#include "nlot_internal.h"

namespace nlot {
static thread_local std::string g_err;
void set_error(const std::string& msg) { g_err = msg; }
}  // namespace nlot

extern "C" int32_t nlot_abi_version(void) { return NLOT_ABI_VERSION; }
extern "C" const char* nlot_last_error(void) { return nlot::g_err.c_str(); }

extern "C" void nlot_default_options(NlotSolverOptions* o) {
    if (!o) return;
    std::memset(o, 0, sizeof(*o));
    o->tol = 1e-4;               // runner.py:118
    o->max_iter = 1000;          // runner.py:117
    o->mu_strategy = 1;          // adaptive + quality-function oracle (runner.py:118-119)
    o->mu_init = 0.1;
    o->barrier_tol_factor = 0.05;  // runner.py:120
    o->dual_inf_tol = 1.0;
    o->constr_viol_tol = 1e-4;
    o->compl_inf_tol = 1e-4;
    o->constr_mult_init_max = 1e3;
    o->bound_push = 1e-2;
    o->bound_frac = 1e-2;
    o->max_soc = 4;                          // IPOPT defaults from here on
    o->resto = 1;
    o->watchdog_shortened_iter_trigger = 10;
    o->watchdog_trial_iter_max = 3;
    o->max_soft_resto_iters = 10;
    o->kappa_soc = 0.99;
    o->tiny_step_tol = 10 * 2.220446049250313e-16;
    o->tiny_step_y_tol = 1e-2;
    o->soft_resto_pderror_reduction_factor = 0.9999;
    o->required_infeasibility_reduction = 0.9;
    o->resto_penalty_parameter = 1000.0;
    o->resto_proximity_weight = 1.0;
    o->bound_mult_reset_threshold = 1000.0;
    o->resto_failure_feasibility_threshold = 0.0;
    o->general_bounds = 1;  // opti.bounded / subject_to(slack >= 0) as constraint rows (runner.py:67-69,101-103)
}

// ------------------------------------------------------------------------------------------------
// CasADi external shim.  gen/nn_sdf.cpp:3 constructs ONE static global L4CasADi model at dlopen; the
// equivalent here is the model bound by nlot_casadi_bind.  Each call evaluates one 1x2 point (the
// sparsity of gen/nn_sdf.cpp:36-37) on the GPU synchronously; CasADi owns arg/res (host doubles).
// ------------------------------------------------------------------------------------------------
namespace {
const NlotMlp* g_bound = nullptr;  // cleared by nlot_mlp_destroy (casadi_unbind)
int g_bound_dev = 0;               // device the bound model lives on
std::mutex g_mu;
float* g_dev[64] = {};  // per device: [0..1] point, [2] lam, [3] val, [4..5] grad, [6..9] hess
const casadi_int_t s_in0[3] = {1, 2, 1};
const casadi_int_t s_out0[3] = {1, 1, 1};

int shim_eval(const double* x, const double* adj, double* val, double* grad, double* hess) {
    std::lock_guard<std::mutex> lk(g_mu);
    if (!g_bound) {
        nlot::set_error("nn_sdf: no model bound (nlot_casadi_bind)");
        return 1;
    }
    int prev = 0;
    if (hipGetDevice(&prev) != hipSuccess || hipSetDevice(g_bound_dev) != hipSuccess) return 1;
    struct Restore {
        int d;
        ~Restore() { (void)hipSetDevice(d); }
    } restore{prev};
    float*& scratch = g_dev[g_bound_dev & 63];
    if (!scratch && hipMalloc(&scratch, 16 * sizeof(float)) != hipSuccess) return 1;
    float* g_dev = scratch;
    float h[16] = {0};
    h[0] = (float)x[0];  // CasADi double -> fp32, as the TorchScript graph requires
    h[1] = (float)x[1];
    h[2] = adj ? (float)adj[0] : 1.f;
    if (hipMemcpy(g_dev, h, 3 * sizeof(float), hipMemcpyHostToDevice) != hipSuccess) return 1;
    bool full = grad || hess;
    if (nlot_sdf_mlp_eval(g_bound, g_dev, 1, g_dev + 3, full ? g_dev + 4 : nullptr, full ? g_dev + 2 : nullptr,
                          hess ? g_dev + 6 : nullptr, nullptr) != NLOT_OK)
        return 1;
    if (hipMemcpy(h + 3, g_dev + 3, 7 * sizeof(float), hipMemcpyDeviceToHost) != hipSuccess) return 1;
    if (val) val[0] = h[3];
    if (grad) {
        grad[0] = h[4];
        grad[1] = h[5];
    }
    if (hess) /* column-major 2x2 (symmetric) */
        for (int i = 0; i < 4; ++i) hess[i] = h[6 + i];
    return 0;
}
}  // namespace

extern "C" int32_t nlot_casadi_bind(const NlotMlp* mlp) {
    std::lock_guard<std::mutex> lk(g_mu);
    g_bound = mlp;
    g_bound_dev = mlp ? mlp->device : 0;
    return NLOT_OK;
}

void nlot::casadi_unbind(const NlotMlp* m) {
    std::lock_guard<std::mutex> lk(g_mu);
    if (g_bound == m) g_bound = nullptr;
}

extern "C" casadi_int_t nn_sdf_n_in(void) { return 1; }
extern "C" casadi_int_t nn_sdf_n_out(void) { return 1; }
extern "C" const casadi_int_t* nn_sdf_sparsity_in(casadi_int_t i) { return i == 0 ? s_in0 : nullptr; }
extern "C" const casadi_int_t* nn_sdf_sparsity_out(casadi_int_t i) { return i == 0 ? s_out0 : nullptr; }
extern "C" int nn_sdf(const casadi_real_t** arg, casadi_real_t** res, casadi_int_t*, casadi_real_t*, int) {
    return shim_eval(arg[0], nullptr, res[0], nullptr, nullptr);
}
// jac [i0, out_o0] -> [jac_o0_i0]  (gen/nn_sdf.cpp:64-70)
extern "C" casadi_int_t jac_nn_sdf_n_in(void) { return 2; }
extern "C" casadi_int_t jac_nn_sdf_n_out(void) { return 1; }
extern "C" int jac_nn_sdf(const casadi_real_t** arg, casadi_real_t** res, casadi_int_t*, casadi_real_t*, int) {
    double v;
    return shim_eval(arg[0], nullptr, &v, res[0], nullptr);
}
// adj1 [i0, out_o0, adj_o0] -> [out_adj_i0]  (gen/nn_sdf.cpp:76-83)
extern "C" casadi_int_t adj1_nn_sdf_n_in(void) { return 3; }
extern "C" casadi_int_t adj1_nn_sdf_n_out(void) { return 1; }
extern "C" int adj1_nn_sdf(const casadi_real_t** arg, casadi_real_t** res, casadi_int_t*, casadi_real_t*, int) {
    double v;
    return shim_eval(arg[0], arg[2], &v, res[0], nullptr);
}
// jac_adj1 [i0, out_o0, adj_o0, out_adj_i0] -> [jac_adj_i0_i0, -, -]  (gen/nn_sdf.cpp:88-104):
// only res[0] is provided, exactly like the generated file (which throws; this returns 1).
extern "C" casadi_int_t jac_adj1_nn_sdf_n_in(void) { return 4; }
extern "C" casadi_int_t jac_adj1_nn_sdf_n_out(void) { return 3; }
extern "C" int jac_adj1_nn_sdf(const casadi_real_t** arg, casadi_real_t** res, casadi_int_t*, casadi_real_t*, int) {
    if (res[1] != nullptr || res[2] != nullptr || res[0] == nullptr) {
        nlot::set_error("jac_adj1_nn_sdf: only jac_adj_i0_i0 is provided (as in L4CasADi)");
        return 1;
    }
    double v, g[2];
    return shim_eval(arg[0], arg[2], &v, g, res[0]);
}
