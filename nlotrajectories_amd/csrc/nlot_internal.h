// Internal declarations shared by the HIP translation units of libnlot.so (not part of the ABI).
#pragma once
#include <hip/hip_runtime.h>

#include <atomic>
#include <cstdint>
#include <cstdio>
#include <string>

#include "../../include/nlot.h"

namespace nlot {

// thread-local last error (nlot_last_error)
void set_error(const std::string& msg);

#define NLOT_HIP_CHECK(expr)                                                                        \
    do {                                                                                           \
        hipError_t e_ = (expr);                                                                    \
        if (e_ != hipSuccess) {                                                                    \
            ::nlot::set_error(std::string(#expr) + ": " + hipGetErrorString(e_));                  \
            return NLOT_ERR_HIP;                                                                   \
        }                                                                                          \
    } while (0)

// One-time per-device kernel attribute (the dynamic-LDS limit): `done` is a bit mask over device ids
// kept per kernel instantiation, so a process driving several GPUs sets it on each of them, and
// concurrent callers at worst set it twice (idempotent).
inline hipError_t set_lds_attr_once(std::atomic<uint64_t>& done, const void* fn, int bytes) {
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    const uint64_t bit = 1ull << (dev & 63);
    if (done.load(std::memory_order_acquire) & bit) return hipSuccess;
    e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
    if (e == hipSuccess) done.fetch_or(bit, std::memory_order_acq_rel);
    return e;
}
// Compute units of the current device (cached per device id).
int device_cus();
// The CasADi shim drops its binding when the bound model is destroyed (nlot_capi.hip).
void casadi_unbind(const NlotMlp* m);

// Device-resident learned-SDF weights (opaque NlotMlp of the ABI).
struct MlpDev {
    int arith;       // NLOT_MLP_ARITH_* (nlot_mlp_create_ex)
    int in_kind;     // NLOT_MLP_IN_*
    int H;           // hidden width
    int n_hidden;    // HxH layers
    int act;         // NLOT_ACT_* (ReLU: the MFMA kernels; smooth activations: mlp_smooth)
    float scale;     // fourier scale; omega_0 for NLOT_ACT_SINE
    float b_out;
    const float* A;     // [2][H]
    const float* b0;    // [H]
    const float* W;     // [n_hidden][H][H] (out, in)
    const float* b;     // [n_hidden][H]
    const float* w_out; // [H]
    const void* Wp;     // [3][H][H] bf16 planes (hi, mid, lo) of layer 0, for the split-bf16 value kernel
    const float* Wt;    // [n_hidden][H][H] (in, out): transposed HxH layers for mlp_smooth (smooth nets only)
};

// Output addressing of the MLP kernel: element q of point i goes to ptr_q[i * stride_q].
struct MlpOut {
    float* val;
    float* gx;
    float* gy;
    float* hxx;
    float* hxy;
    float* hyx;  // may alias hxy (SoA) or be the [1][0] slot of an AoS 2x2
    float* hyy;
    int sv, sg, sh;
    uint32_t* mask;      // value launches: the hidden layer's ReLU pattern, 4 words per point (or null)
    int64_t mask_plane;  // word w of point i at mask[w * mask_plane + i]
};

// Forward reuse for full launches: the instance with compaction rank r has, when src[r] >= 0, been
// evaluated by a value launch at trial slot src[r] (tpts, tval, tmask: points, values, ReLU patterns of
// that launch, point i of slot s at s * P_per + i).  Where the trial point equals the point, the full
// kernel takes f and the pattern from there and skips the forward GEMM (same arithmetic: same result).
struct MlpReuse {
    const int* src;
    const float* tpts;
    const float* tval;
    const uint32_t* tmask;
    int64_t plane;
    int* nreused;  // if set: += the number of points whose forward was reused (statistics)
    // if set (ld == 0, mlp_bf16 only): the launch covers ranks [*base, cnt) instead of [0, cnt) (the solver splits a
    // step's value launch in two: the candidates known at the start of the step, then those k_iter_b adds)
    const int* base;
};

// Launch the MFMA SDF-MLP kernel on cnt * P_per points, cnt = *n_dev if n_dev else n (n = upper bound
// that sizes the persistent grid).  Point g lives at g (ld == 0) or (g % cnt) + (g / cnt) * ld.
// full = value + lam*grad + lam*hess; else value only.
int launch_mlp_strided(const MlpDev& w, const float* pts, int64_t n, const int* n_dev, int P_per, int64_t ld,
                       const float* lam, const MlpOut& out, bool full, hipStream_t stream,
                       const MlpReuse* reuse = nullptr);

}  // namespace nlot

struct NlotMlp {
    nlot::MlpDev dev;
    void* block;  // single device allocation holding all arrays
    int device;   // HIP device the arrays live on
};
