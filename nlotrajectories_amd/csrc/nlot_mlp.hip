// Batched learned-SDF MLP: value, lambda*gradient and lambda*Hessian at P points (gfx950).
//
// Replaces the per-point CasADi externals nn_sdf / jac_nn_sdf / adj1_nn_sdf / jac_adj1_nn_sdf
// (/root/reference/_l4c_generated/nn_sdf.cpp:57-104), whose TorchScript graphs evaluate
//   f(p) = w_out . relu(W_l ... relu(W_0 h0 + b_0) ...) + b_out,   h0 = scale*cos(p A + b0)  (FourierMLP,
//   core/nn_architectures.py:30-72)  or  h0 = relu(p A + b0)  (l4casadi naive MLP)
// in fp32, one 1x2 point per call.  Here one launch evaluates every corner of every knot of every
// active problem.
//
// Mapping (MI355X, wave64, f32-input MFMA v_mfma_f32_32x32x2_f32 = exact k-ordered fp32 FMA chain):
//   * a wave owns 32 points; a 256-thread block owns 128 points per tile and loops over tiles
//     (persistent grid: the weights are staged into LDS once per block);
//   * forward GEMM:  Z^T[hidden j][point i] = W[j][:] . h[:][i]  — A operand = W from LDS
//     (row stride H+1 floats: the 32 rows a ds_read_b32 touches land in 32 distinct banks),
//     B operand = the hidden activations of the point held by the lane;  the input layer h0 is
//     computed on the fly per k-step (1 cos per lane per MFMA k-step, hidden under the MFMA);
//   * the accumulator layout (hidden unit in registers, point in lanes) is exactly the B-operand
//     layout of the next product, so every further hidden layer and the whole reverse sweep
//     (G^T = W^T (lam*w_out .* mask)) chain register-to-register with no LDS transpose;
//   * the gradient / Hessian w.r.t. the 2-D input are contractions over the hidden units of the
//     input layer: per-lane partial sums + one cross-half shuffle.  For a Fourier input layer
//     lam*d2f/dp2 = A diag(g .* (-scale cos z)) A^T (g = df/dh0), for a ReLU input layer it is 0.
#include <hip/hip_runtime.h>

#include <atomic>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "nlot_internal.h"

namespace nlot {

typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int kMaxResidentLayers = 2;

// sin and cos of a Fourier-layer argument (|x| up to ~1e3 here: weights ~N(0, 9.4^2), inputs in the
// workspace box): 3-part Cody-Waite reduction by pi/2 with FMA, Cephes sinf/cosf minimax polynomials on
// [-pi/4, pi/4] (~1 ulp), quadrant by select.  No slow path: ~20 instructions for both.
__device__ __forceinline__ void sincos_fourier(float x, float* sn, float* cs) {
    const float j = rintf(x * 0.636619772367581343f);
    float r = fmaf(j, -1.57079637050628662109375f, x);
    r = fmaf(j, 4.37113900018624283e-8f, r);
    r = fmaf(j, 1.71512451e-15f, r);
    const float r2 = r * r;
    const float ps = fmaf(fmaf(fmaf(-1.9515295891e-4f, r2, 8.3321608736e-3f), r2, -1.6666654611e-1f), r2 * r, r);
    const float pc = fmaf(fmaf(fmaf(fmaf(2.443315711809948e-5f, r2, -1.388731625493765e-3f), r2,
                                    4.166664568298827e-2f), r2, -0.5f), r2, 1.0f);
    const int q = (int)j & 3;
    const float s0 = (q & 1) ? pc : ps, c0 = (q & 1) ? ps : pc;
    *sn = (q & 2) ? -s0 : s0;
    *cs = ((q + 1) & 2) ? -c0 : c0;
}

// Fourier-layer argument in turns for the transcendental unit (v_sin_f32 / v_cos_f32 give sin and cos of
// 2 pi t): r = x - 2 pi j in [-pi, pi] by a two-part Cody-Waite reduction with FMA (the first product is
// exact; the dropped third part, |j| * 3.4e-15, stays below 1e-12 for |x| <= 1e3), then r / (2 pi).  The
// split-bf16 kernels use it: 4 instructions and one 8-cycle transcendental per sin or cos, against ~14 for
// the polynomials and quadrant selects of sincos_fourier.
__device__ __forceinline__ float turns_fourier(float x) {
    const float j = rintf(x * 0.159154943091895336f);
    float r = fmaf(j, -6.28318548202514648f, x);
    r = fmaf(j, 1.74845560e-7f, r);
    return r * 0.159154943091895336f;
}

// row index (hidden unit) held by register r of a 32x32 accumulator on lane-half hl
__device__ __forceinline__ int acc_row(int r, int hl) { return (r & 3) + 8 * (r >> 2) + 4 * hl; }

// FULL kernels with one hidden layer run 512-thread blocks (8 waves = 2 per SIMD) sharing one LDS copy of
// the weights, with a per-wave [64][33] staging tile for the reverse sweep (two k-halves at a time).
__host__ __device__ constexpr size_t mlp_lds_floats(int H, int L, bool staged) {
    return (size_t)L * H * (H + 1) + 4 * H + (size_t)L * H + (staged ? (size_t)8 * 64 * 33 : 0);
}
__host__ __device__ constexpr bool mlp_staged(int H, int L) {
    return L == 1 && H % 64 == 0 && mlp_lds_floats(H, L, true) * 4 <= 160 * 1024;
}
__host__ __device__ constexpr int mlp_threads(int H, int L, bool full) { return full && mlp_staged(H, L) ? 512 : 256; }

template <int H, int L, bool FULL>
// Point g of the launch (g < cnt * P_per, cnt = *cnt_dev when given: the solver's compacted instances)
// lives at address g (ld == 0, contiguous rank-major list) or (g % cnt) + (g / cnt) * ld of pts/lam/out.
__global__ __launch_bounds__(mlp_threads(H, L, FULL), (FULL || L > 1) ? 1 : 2) void mlp_kernel(MlpDev w, const float* __restrict__ pts, int64_t cnt_host,
                                                      const int* __restrict__ cnt_dev, int P_per, int64_t ld,
                                                      const float* __restrict__ lam, MlpOut out) {
    constexpr int HP = H + 1;   // padded LDS row
    constexpr int NT = H / 32;  // 32x32 tiles along the hidden dimension
    extern __shared__ __attribute__((aligned(16))) float smem[];
    float* sW = smem;                                   // [L][H][HP]
    float* sA0 = sW + (size_t)L * H * HP;               // [H]
    float* sA1 = sA0 + H;                               // [H]
    float* sb0 = sA1 + H;                               // [H]
    float* sb = sb0 + H;                                // [L][H]
    float* sw = sb + L * H;                             // [H]
    // FULL kernels whose LDS budget allows: a per-wave [H][33] staging tile for the reverse sweep's
    // operand and for df/dh0 (runtime k-loops instead of fully unrolled register chains: no spills)
    constexpr bool STAGED = FULL && mlp_staged(H, L);
    float* sStage = sw + H;                             // [8 waves][64][33] when STAGED
    constexpr int TP = mlp_threads(H, L, FULL) / 2;     // points per block tile (32 per wave)

    for (int idx = threadIdx.x; idx < L * H * H; idx += blockDim.x) {
        int l = idx / (H * H), rem = idx - l * H * H, j = rem / H, k = rem - j * H;
        sW[(size_t)l * H * HP + j * HP + k] = w.W[idx];
    }
    for (int idx = threadIdx.x; idx < H; idx += blockDim.x) {
        sA0[idx] = w.A[idx];
        sA1[idx] = w.A[H + idx];
        sb0[idx] = w.b0[idx];
        sw[idx] = w.w_out[idx];
    }
    for (int idx = threadIdx.x; idx < L * H; idx += blockDim.x) sb[idx] = w.b[idx];
    __syncthreads();

    const int64_t cnt = cnt_dev ? (int64_t)(*cnt_dev) : cnt_host;
    const int64_t npts = cnt * P_per;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int il = lane & 31, hl = lane >> 5;
    const bool fourier = w.in_kind == NLOT_MLP_IN_FOURIER;
    const float scale = w.scale;

    for (int64_t tile = blockIdx.x; tile * TP < npts; tile += gridDim.x) {
        const int64_t gi = tile * TP + wave * 32 + il;
        const bool valid = gi < npts;
        const int64_t pi = valid ? (ld == 0 ? gi : (gi % cnt) + (gi / cnt) * ld) : 0;
        float px = 0.f, py = 0.f;
        if (valid) {
            px = pts[2 * pi];
            py = pts[2 * pi + 1];
        }
        // ---------------- input layer + first hidden GEMM ----------------
        f32x16 acc[NT];
#pragma unroll
        for (int t = 0; t < NT; ++t) acc[t] = f32x16{};
#pragma unroll 4
        for (int s = 0; s < H / 2; ++s) {
            const int k = 2 * s + hl;
            const float z = fmaf(py, sA1[k], px * sA0[k]) + sb0[k];
            float h0;
            if (fourier) {
                float sn, cs;
                sincos_fourier(z, &sn, &cs);
                h0 = cs * scale;
            } else {
                h0 = z > 0.f ? z : 0.f;
            }
#pragma unroll
            for (int t = 0; t < NT; ++t) {
                const float a = sW[(t * 32 + il) * HP + k];
                acc[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, h0, acc[t], 0, 0, 0);
            }
        }
        uint64_t mask[L];
        // bias + ReLU of layer 0
        {
            uint64_t m = 0;
#pragma unroll
            for (int t = 0; t < NT; ++t)
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const float v = acc[t][r] + sb[t * 32 + acc_row(r, hl)];
                    const bool on = v > 0.f;
                    acc[t][r] = on ? v : 0.f;
                    m |= (uint64_t)on << (t * 16 + r);
                }
            mask[0] = m;
        }
        // ---------------- further hidden layers (register-chained) ----------------
#pragma unroll
        for (int l = 1; l < L; ++l) {
            const float* Wl = sW + (size_t)l * H * HP;
            f32x16 nacc[NT];
#pragma unroll
            for (int t = 0; t < NT; ++t) nacc[t] = f32x16{};
#pragma unroll
            for (int ti = 0; ti < NT; ++ti)
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int kk = ti * 32 + acc_row(r, hl);
                    const float bv = acc[ti][r];
#pragma unroll
                    for (int t = 0; t < NT; ++t) {
                        const float a = Wl[(t * 32 + il) * HP + kk];
                        nacc[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, bv, nacc[t], 0, 0, 0);
                    }
                }
            uint64_t m = 0;
#pragma unroll
            for (int t = 0; t < NT; ++t)
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const float v = nacc[t][r] + sb[l * H + t * 32 + acc_row(r, hl)];
                    const bool on = v > 0.f;
                    acc[t][r] = on ? v : 0.f;
                    m |= (uint64_t)on << (t * 16 + r);
                }
            mask[l] = m;
        }
        // ---------------- output layer ----------------
        float fpart = 0.f;
#pragma unroll
        for (int t = 0; t < NT; ++t)
#pragma unroll
            for (int r = 0; r < 16; ++r) fpart = fmaf(sw[t * 32 + acc_row(r, hl)], acc[t][r], fpart);
        const float f = fpart + __shfl_xor(fpart, 32) + w.b_out;

        if constexpr (!FULL) {
            if (valid && hl == 0) out.val[pi * out.sv] = f;
            continue;
        } else {
            // ---------------- reverse sweep ----------------
            const float lm = lam ? (valid ? lam[pi] : 0.f) : 1.f;
            float gx = 0.f, gy = 0.f, hxx = 0.f, hxy = 0.f, hyy = 0.f;
            if constexpr (STAGED) {
                float* sE = sStage + wave * (64 * 33);  // [k within the half][point], padded
                const uint64_t m = mask[0];
                f32x16 g[NT];
#pragma unroll
                for (int t = 0; t < NT; ++t) g[t] = f32x16{};
                // g = W^T e with e = lam * w_out .* mask, staged 64 rows of k at a time
#pragma unroll
                for (int hh = 0; hh < H / 64; ++hh) {
                    __syncthreads();
#pragma unroll
                    for (int tt = 0; tt < 2; ++tt)
#pragma unroll
                        for (int r = 0; r < 16; ++r) {
                            const int t = 2 * hh + tt, kl = tt * 32 + acc_row(r, hl);
                            sE[kl * 33 + il] = ((m >> (t * 16 + r)) & 1) ? lm * sw[t * 32 + acc_row(r, hl)] : 0.f;
                        }
                    __syncthreads();
#pragma unroll 4
                    for (int s = 0; s < 32; ++s) {
                        const int kl = 2 * s + hl, k = hh * 64 + kl;
                        const float bv = sE[kl * 33 + il];
#pragma unroll
                        for (int t = 0; t < NT; ++t) {
                            const float a = sW[k * HP + t * 32 + il];
                            g[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, bv, g[t], 0, 0, 0);
                        }
                    }
                }
                // g = df/dh0 (x lam): contract with the input layer's derivatives, lane = (k, point)
#pragma unroll
                for (int hh = 0; hh < H / 64; ++hh) {
                    __syncthreads();
#pragma unroll
                    for (int tt = 0; tt < 2; ++tt)
#pragma unroll
                        for (int r = 0; r < 16; ++r) sE[(tt * 32 + acc_row(r, hl)) * 33 + il] = g[2 * hh + tt][r];
                    __syncthreads();
#pragma unroll 2
                    for (int s = 0; s < 32; ++s) {
                        const int kl = 2 * s + hl, k = hh * 64 + kl;
                        const float ax = sA0[k], ay = sA1[k];
                        const float z = fmaf(py, ay, px * ax) + sb0[k];
                        const float d = sE[kl * 33 + il];
                        float dz, c2;
                        if (fourier) {
                            float sn, cs;
                            sincos_fourier(z, &sn, &cs);
                            dz = d * (-scale * sn);
                            c2 = d * (-scale * cs);
                        } else {
                            dz = z > 0.f ? d : 0.f;
                            c2 = 0.f;
                        }
                        gx = fmaf(ax, dz, gx);
                        gy = fmaf(ay, dz, gy);
                        hxx = fmaf(ax * ax, c2, hxx);
                        hxy = fmaf(ax * ay, c2, hxy);
                        hyy = fmaf(ay * ay, c2, hyy);
                    }
                }
            } else {
            // e = lam * w_out .* mask_top  (in place, accumulator layout)
            {
                const uint64_t m = mask[L - 1];
#pragma unroll
                for (int t = 0; t < NT; ++t)
#pragma unroll
                    for (int r = 0; r < 16; ++r)
                        acc[t][r] = ((m >> (t * 16 + r)) & 1) ? lm * sw[t * 32 + acc_row(r, hl)] : 0.f;
            }
#pragma unroll
            for (int l = L - 1; l >= 0; --l) {
                const float* Wl = sW + (size_t)l * H * HP;
                f32x16 g[NT];
#pragma unroll
                for (int t = 0; t < NT; ++t) g[t] = f32x16{};
#pragma unroll
                for (int tj = 0; tj < NT; ++tj)
#pragma unroll
                    for (int r = 0; r < 16; ++r) {
                        const int jj = tj * 32 + acc_row(r, hl);
                        const float bv = acc[tj][r];
#pragma unroll
                        for (int t = 0; t < NT; ++t) {
                            const float a = Wl[jj * HP + t * 32 + il];
                            g[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, bv, g[t], 0, 0, 0);
                        }
                    }
                if (l > 0) {
                    const uint64_t m = mask[l - 1];
#pragma unroll
                    for (int t = 0; t < NT; ++t)
#pragma unroll
                        for (int r = 0; r < 16; ++r) acc[t][r] = ((m >> (t * 16 + r)) & 1) ? g[t][r] : 0.f;
                } else {
#pragma unroll
                    for (int t = 0; t < NT; ++t) acc[t] = g[t];
                }
            }
            // acc = df/dh0 (x lam); contract with the input layer's derivatives
#pragma unroll
            for (int t = 0; t < NT; ++t)
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int k = t * 32 + acc_row(r, hl);
                    const float ax = sA0[k], ay = sA1[k];
                    const float z = fmaf(py, ay, px * ax) + sb0[k];
                    const float d = acc[t][r];
                    float dz, c2;
                    if (fourier) {
                        float sn, cs;
                        sincos_fourier(z, &sn, &cs);
                        dz = d * (-scale * sn);
                        c2 = d * (-scale * cs);
                    } else {
                        dz = z > 0.f ? d : 0.f;
                        c2 = 0.f;
                    }
                    gx = fmaf(ax, dz, gx);
                    gy = fmaf(ay, dz, gy);
                    hxx = fmaf(ax * ax, c2, hxx);
                    hxy = fmaf(ax * ay, c2, hxy);
                    hyy = fmaf(ay * ay, c2, hyy);
                }
            }
            gx += __shfl_xor(gx, 32);
            gy += __shfl_xor(gy, 32);
            hxx += __shfl_xor(hxx, 32);
            hxy += __shfl_xor(hxy, 32);
            hyy += __shfl_xor(hyy, 32);
            if (valid && hl == 0) {
                out.val[pi * out.sv] = f;
                if (out.gx) {
                    out.gx[pi * out.sg] = gx;
                    out.gy[pi * out.sg] = gy;
                }
                if (out.hxx) {
                    out.hxx[pi * out.sh] = hxx;
                    out.hxy[pi * out.sh] = hxy;
                    if (out.hyx != out.hxy) out.hyx[pi * out.sh] = hxy;
                    out.hyy[pi * out.sh] = hyy;
                }
            }
        }
    }
}

// ---------------------------------------------------------------------------------------------
// Split-bf16 MFMA kernels with fp32-equivalent products (Fourier / ReLU input layer, one HxH layer).
// Both operands are split into three bf16 parts, x = x_hi + x_mid + x_lo (8 + 8 + 8 significant bits,
// exact up to 2^-24 relative), and each 32x32x16 block takes the six products down to 2^-24:
// hi.hi, hi.mid, mid.hi, hi.lo, lo.hi, mid.mid — every product exact in the fp32 accumulator, the dropped
// ones below fp32 rounding.  6 v_mfma_f32_32x32x16_bf16 (6 x 32 cycles) replace 8 v_mfma_f32_32x32x2_f32
// (8 x 64 cycles) per 16 k.  The weight planes are split once at nlot_mlp_create (MlpDev::Wp) and staged
// once per block as one row-major image; the forward GEMM reads it by rows (ds_read_b128), the reverse
// sweep G = W^T (lam w_out .* mask) by transposed reads (ds_read_b64_tr_b16) — one image for both.  The
// input-layer activations are split as they are computed, directly in the B-operand layout (lane l:
// point l & 31, k = 16 s + 8 (l >> 5) + j); the reverse sweep's B operand is the forward accumulator
// (mask and w_out) split in place (accumulator-as-operand k order).
// ---------------------------------------------------------------------------------------------
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void split3(float x, __bf16& h, __bf16& m, __bf16& l) {
#pragma clang fp contract(off)  // x is the rounded fp32 input: never fuse its producer into the subtractions
    h = (__bf16)x;
    const float r = x - (float)h;  // exact
    m = (__bf16)r;
    l = (__bf16)(r - (float)m);    // exact difference
}

// The five smaller split products of one k block from a zero accumulator, then the hi x hi products into the running
// sum, then the two added by a VALU add (round to nearest).  One v_mfma_f32_32x32x16_bf16 aligns its addends (the
// accumulator and its 16 products) to the largest of them and keeps about two bits below that one's fp32 ulp
// (scripts/mfma_round_probe.hip), so small products added straight to a large running sum lose their low bits.
__device__ __forceinline__ f32x16 mfma6s(const bf16x8& ah, const bf16x8& am, const bf16x8& al, const bf16x8& bh,
                                         const bf16x8& bm, const bf16x8& bl, f32x16 acc) {
    f32x16 acs = __builtin_amdgcn_mfma_f32_32x32x16_bf16(am, bm, f32x16{}, 0, 0, 0);
    acs = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al, bh, acs, 0, 0, 0);
    acs = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bl, acs, 0, 0, 0);
    acs = __builtin_amdgcn_mfma_f32_32x32x16_bf16(am, bh, acs, 0, 0, 0);
    acs = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bm, acs, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bh, acc, 0, 0, 0);
    return acc + acs;
}
// The five smaller products into a running accumulator of their own (NLOT_MLP_TWOACC_REV=2: one VALU add per output
// tile instead of one per k block; the small-product sum stays ~2^-8 of the main one, so it keeps its low bits too)
__device__ __forceinline__ f32x16 mfma5s(const bf16x8& ah, const bf16x8& am, const bf16x8& al, const bf16x8& bh,
                                         const bf16x8& bm, const bf16x8& bl, f32x16 acs) {
    acs = __builtin_amdgcn_mfma_f32_32x32x16_bf16(am, bm, acs, 0, 0, 0);
    acs = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al, bh, acs, 0, 0, 0);
    acs = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bl, acs, 0, 0, 0);
    acs = __builtin_amdgcn_mfma_f32_32x32x16_bf16(am, bh, acs, 0, 0, 0);
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bm, acs, 0, 0, 0);
}
// Where it is used (round 6, profiles/r06/ab_split_two_acc/): in the reverse sweep (G = W^T e, the
// gradient and Hessian) by default, as mfma5s's running small-product accumulator (NLOT_MLP_TWOACC_REV=2; mfma6s per
// k block is 1, the direct accumulation 0): with the direct accumulation the product net left benchmark 6's pinned
// path on instances where no fp32 summation order of the oracle's net does; the running form costs 3.6 % less than
// mfma6s on the full launch (1.513 / 1.569 ms, profiles/r06/ab_rev_acc/).  In the forward GEMMs only with
// NLOT_MLP_TWOACC_FWD=1 (it halves the value's -5e-9 offset but the value kernel spills at 3 waves per SIMD: -20 %
// there, -5 % traj/s)
#ifndef NLOT_MLP_TWOACC_FWD
#define NLOT_MLP_TWOACC_FWD 0
#endif
#ifndef NLOT_MLP_TWOACC_REV
#define NLOT_MLP_TWOACC_REV 2
#endif

// six split-bf16 products, smallest terms first
__device__ __forceinline__ f32x16 mfma6(const bf16x8& ah, const bf16x8& am, const bf16x8& al, const bf16x8& bh,
                                        const bf16x8& bm, const bf16x8& bl, f32x16 acc) {
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(am, bm, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al, bh, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bl, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(am, bh, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bm, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bh, acc, 0, 0, 0);
    return acc;
}

// A fragment (32x32x16) of W^T from the row-major plane image by two transposed reads: lane group
// g = lane / 16 covers columns c0 = col0 + 16 (g & 1) .. +15 of W; lane 4q + p of the group supplies row
// r0 + q, columns c0 + 4p .. +3, and receives its own column's 4 rows.  Rows follow the
// accumulator-as-operand k order: element jj of lane half h is row jbase + 8 (jj >> 2) + 4 h + (jj & 3).
template <int RS>
__device__ __forceinline__ bf16x8 wt_frag(const __bf16* plane, int jbase, int col0, int lane) {
    const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3, h = g >> 1;
    const int c0 = col0 + 16 * (g & 1);
    const __bf16* a0 = plane + (size_t)(jbase + 4 * h + q) * RS + c0 + 4 * p;
    const __bf16* a1 = a0 + (size_t)8 * RS;
    const bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((__attribute__((address_space(3))) bf16x4*)(a0));
    const bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((__attribute__((address_space(3))) bf16x4*)(a1));
    return bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
}

// one weight image per CU, shared by NLOT_MLP_*_THREADS / 256 waves per SIMD: value-only launches 3; FULL (value +
// reverse sweep) NLOT_MLP_FULL_THREADS / 256.  Round 4: the input layer is a template parameter (no per-element
// branch on the kind), its weights are read as float4 runs (a lane's 8 consecutive k of a 16-wide k block), and the
// reverse sweep's contraction re-reads its LDS operands every tile (an opaque zero offset keeps the compiler from
// hoisting 192 loop-invariant floats into registers across the tile loop, which had pinned FULL at one wave per
// SIMD: 256 VGPRs + 184 AGPRs, or 504 B/lane of scratch at two).
#ifndef NLOT_MLP_VALUE_THREADS
#define NLOT_MLP_VALUE_THREADS 768
#endif
#ifndef NLOT_MLP_FULL_THREADS
#define NLOT_MLP_FULL_THREADS 512
#endif
__host__ __device__ constexpr int bf16_threads(bool full) { return full ? NLOT_MLP_FULL_THREADS : NLOT_MLP_VALUE_THREADS; }

template <int H>
__host__ __device__ constexpr size_t mlp_bf16_lds_bytes() {
    return (size_t)3 * H * (H + 8) * 2 + (size_t)8 * H * 4;
}

// a zero the compiler cannot see through (a VGPR written by an opaque move): added to an LDS offset inside a loop,
// it keeps loop-invariant LDS reads in the loop
__device__ __forceinline__ int opaque_zero() {
    int z;
    asm volatile("v_mov_b32 %0, 0" : "=v"(z));
    return z;
}

__device__ __forceinline__ void lds8(const float* p, float (&o)[8]) {
    const float4 a = *reinterpret_cast<const float4*>(p), b = *reinterpret_cast<const float4*>(p + 4);
    o[0] = a.x, o[1] = a.y, o[2] = a.z, o[3] = a.w, o[4] = b.x, o[5] = b.y, o[6] = b.z, o[7] = b.w;
}

// input-layer activation of z = p @ A + b0 (nn_architectures.py:38 for the Fourier layer)
template <bool FOUR>
__device__ __forceinline__ float in_act(float z, float scale) {
    if constexpr (FOUR) {
        // rounded product (no contraction into split3's subtraction): h0 is the fp32 value the oracle forms
#pragma clang fp contract(off)
        return __builtin_amdgcn_cosf(turns_fourier(z)) * scale;
    } else {
        return z > 0.f ? z : 0.f;
    }
}

template <int H, bool FULL, bool FOUR>
__global__ __launch_bounds__(bf16_threads(FULL), 1) void mlp_bf16(MlpDev w, const float* __restrict__ pts, int64_t cnt_host,
                                                            const int* __restrict__ cnt_dev, int P_per, int64_t ld,
                                                            const float* __restrict__ lam, MlpOut out, MlpReuse ru) {
    constexpr int RS = H + 8;    // padded plane row (bf16): 16-byte rows offset by 4 banks
    constexpr int NT = H / 32;   // 32-row tiles
    constexpr int NKB = H / 16;  // 16-wide k blocks
    extern __shared__ __attribute__((aligned(16))) float smem[];
    __bf16* sWp = reinterpret_cast<__bf16*>(smem);                  // [3][H][RS]
    float* sA0 = reinterpret_cast<float*>(sWp + (size_t)3 * H * RS);  // [H]
    float* sA1 = sA0 + H;
    float* sb0 = sA1 + H;
    float* sb = sb0 + H;
    float* sw = sb + H;
    float* sq = sw + H;  // [3][H]: A0^2, A0 A1, A1^2 (the Fourier Hessian's per-k factors, as the oracle rounds them)
    __shared__ int s_reused;
    for (int idx = threadIdx.x; idx < 3 * H * H / 8; idx += blockDim.x) {  // 16-byte chunks of the planes
        const int pr = idx / (H / 8), c8 = idx % (H / 8);                   // pr = plane * H + row
        *reinterpret_cast<uint4*>(sWp + (size_t)pr * RS + c8 * 8) = reinterpret_cast<const uint4*>(w.Wp)[idx];
    }
    for (int idx = threadIdx.x; idx < H; idx += blockDim.x) {
        const float a0 = w.A[idx], a1 = w.A[H + idx];
        sA0[idx] = a0;
        sA1[idx] = a1;
        sb0[idx] = w.b0[idx];
        sb[idx] = w.b[idx];
        sw[idx] = w.w_out[idx];
        sq[idx] = a0 * a0;
        sq[H + idx] = a0 * a1;
        sq[2 * H + idx] = a1 * a1;
    }
    if (threadIdx.x == 0) s_reused = 0;
    __syncthreads();

    const int64_t cnt = cnt_dev ? (int64_t)(*cnt_dev) : cnt_host;
    const int64_t npts = cnt * P_per;
    const int64_t g0 = (ru.base && ld == 0) ? (int64_t)(*ru.base) * P_per : 0;  // first point of the launch
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int il = lane & 31, hl = lane >> 5;
    const float scale = w.scale;
    constexpr int TP = bf16_threads(FULL) / 2;  // points per block tile (32 per wave)
    if constexpr (!FULL) {
        // Value-only launches, software-pipelined inside the wave: the B fragment (input-layer activations, split)
        // of k block s + 1 — or, in the last block, block 0 of the wave's NEXT tile — is computed between the MFMAs
        // of block s (2 elements per 32x32 output tile), so a wave's VALU work issues into its own MFMA gaps
        // instead of alternating with them.  Same arithmetic per point as the FULL forward below.
        static_assert(8 % NT == 0, "two input-layer elements per output tile and k block");
        constexpr int EPT = 8 / NT;
        const int64_t G = gridDim.x;
        auto point = [&](int64_t tile, float& x, float& y) {
            const int64_t gi = g0 + tile * TP + wave * 32 + il;
            x = y = 0.f;
            if (gi < npts) {
                const int64_t pi = ld == 0 ? gi : (gi % cnt) + (gi / cnt) * ld;
                x = pts[2 * pi];
                y = pts[2 * pi + 1];
            }
        };
        float cx, cy, nx, ny;
        point(blockIdx.x, cx, cy);
        point(blockIdx.x + G, nx, ny);
        bf16x8 bh, bm, bl;
        {
            float a0[8], a1[8], c0[8];
            lds8(sA0 + 8 * hl, a0);
            lds8(sA1 + 8 * hl, a1);
            lds8(sb0 + 8 * hl, c0);
#pragma unroll
            for (int jj = 0; jj < 8; ++jj) {
                __bf16 a, b, c;
                split3(in_act<FOUR>(fmaf(cy, a1[jj], cx * a0[jj]) + c0[jj], scale), a, b, c);
                bh[jj] = a;
                bm[jj] = b;
                bl[jj] = c;
            }
        }
        for (int64_t tile = blockIdx.x; g0 + tile * TP < npts; tile += G) {
            float fx, fy;
            point(tile + 2 * G, fx, fy);
            f32x16 acc[NT];
#pragma unroll
            for (int t = 0; t < NT; ++t) acc[t] = f32x16{};
#pragma unroll 1
            for (int s = 0; s < NKB; ++s) {
                const bool last = s == NKB - 1;
                const int sn = last ? 0 : s + 1;
                const float qx = last ? nx : cx, qy = last ? ny : cy;
                float a0[8], a1[8], c0[8];
                const int kn = 16 * sn + 8 * hl;
                lds8(sA0 + kn, a0);
                lds8(sA1 + kn, a1);
                lds8(sb0 + kn, c0);
                bf16x8 nh, nm, nl;
#pragma unroll
                for (int t = 0; t < NT; ++t) {
                    const __bf16* rowp = sWp + (size_t)(t * 32 + il) * RS + 16 * s + 8 * hl;
                    const bf16x8 ah = *reinterpret_cast<const bf16x8*>(rowp);
                    const bf16x8 am = *reinterpret_cast<const bf16x8*>(rowp + (size_t)H * RS);
                    const bf16x8 al = *reinterpret_cast<const bf16x8*>(rowp + (size_t)2 * H * RS);
                    acc[t] = NLOT_MLP_TWOACC_FWD ? mfma6s(ah, am, al, bh, bm, bl, acc[t]) : mfma6(ah, am, al, bh, bm, bl, acc[t]);
#pragma unroll
                    for (int u = 0; u < EPT; ++u) {
                        const int jj = t * EPT + u;
                        __bf16 a, b, c;
                        split3(in_act<FOUR>(fmaf(qy, a1[jj], qx * a0[jj]) + c0[jj], scale), a, b, c);
                        nh[jj] = a;
                        nm[jj] = b;
                        nl[jj] = c;
                    }
                }
                bh = nh;
                bm = nm;
                bl = nl;
            }
            float fpart = 0.f;
            uint64_t mk = 0;
#pragma unroll
            for (int t = 0; t < NT; ++t)
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int j = t * 32 + acc_row(r, hl);
                    const float v = acc[t][r] + sb[j];
                    const int on = min(max(__float_as_int(v), 0), 1);
                    fpart = fmaf(sw[j], fmaxf(v, 0.f), fpart);
                    mk |= (uint64_t)on << (t * 16 + r);
                }
            const float fw = fpart + __shfl_xor(fpart, 32) + w.b_out;
            const int64_t gi = g0 + tile * TP + wave * 32 + il;
            if (gi < npts) {
                const int64_t pi = ld == 0 ? gi : (gi % cnt) + (gi / cnt) * ld;
                if (hl == 0) out.val[pi * out.sv] = fw;
                if (out.mask) {
                    out.mask[(2 * hl) * out.mask_plane + pi] = (uint32_t)mk;
                    out.mask[(2 * hl + 1) * out.mask_plane + pi] = (uint32_t)(mk >> 32);
                }
            }
            cx = nx;
            cy = ny;
            nx = fx;
            ny = fy;
        }
        return;
    }

    // A block's tiles are tile0, tile0 + G, ...: each tile's inputs (point, the reuse source and, one tile later,
    // the source's trial point / value / ReLU pattern) are loaded ahead, so the dependent global round trips of a
    // tile overlap the previous tile's MFMA work
    struct TileIn {
        float px, py;
        int src;
    };
    struct ReuseIn {
        float tx, ty, tv;
        uint32_t m0, m1;
    };
    const bool reuse_on = FULL && ru.src && ld == 0;
    auto load_in = [&](int64_t tile, TileIn& a) {
        const int64_t gi = g0 + tile * TP + wave * 32 + il;
        a.px = a.py = 0.f;
        a.src = -1;
        if (gi < npts) {
            const int64_t pi = ld == 0 ? gi : (gi % cnt) + (gi / cnt) * ld;
            a.px = pts[2 * pi];
            a.py = pts[2 * pi + 1];
            if (reuse_on) a.src = ru.src[gi / P_per];
        }
    };
    auto load_reuse = [&](int64_t tile, const TileIn& a, ReuseIn& r) {
        r.tx = r.ty = r.tv = 0.f;
        r.m0 = r.m1 = 0u;
        if (reuse_on && a.src >= 0) {
            const int64_t gi = g0 + tile * TP + wave * 32 + il;
            const int64_t q = (int64_t)a.src * P_per + (gi - (gi / P_per) * P_per);
            r.tx = ru.tpts[2 * q];
            r.ty = ru.tpts[2 * q + 1];
            r.tv = ru.tval[q];
            r.m0 = ru.tmask[(2 * hl) * ru.plane + q];
            r.m1 = ru.tmask[(2 * hl + 1) * ru.plane + q];
        }
    };
    const int64_t G = gridDim.x;
    TileIn in0, in1;
    ReuseIn re0;
    load_in(blockIdx.x, in0);
    load_reuse(blockIdx.x, in0, re0);
    load_in(blockIdx.x + G, in1);
    for (int64_t tile = blockIdx.x; g0 + tile * TP < npts; tile += G) {
        TileIn in2;
        ReuseIn re1;
        load_in(tile + 2 * G, in2);
        load_reuse(tile + G, in1, re1);
        const int64_t gi = g0 + tile * TP + wave * 32 + il;
        const bool valid = gi < npts;
        const int64_t pi = valid ? (ld == 0 ? gi : (gi % cnt) + (gi / cnt) * ld) : 0;
        const float px = in0.px, py = in0.py;
        // ---------------- forward reuse (full launches after an accepted trial point) ----------------
        float f = 0.f;
        uint64_t mask = 0;
        bool have = false;
        if (reuse_on && valid && in0.src >= 0 && re0.tx == px && re0.ty == py) {
            f = re0.tv;
            mask = (uint64_t)re0.m0 | ((uint64_t)re0.m1 << 32);
            have = true;
        }
        const bool skip = __all(have || !valid);  // wave-uniform
        if (FULL && skip && ru.nreused) {
            const uint64_t vb = __ballot(valid && hl == 0);
            if (lane == 0) atomicAdd(&s_reused, (int)__popcll(vb));
        }
        if (!skip) {  // the forward for all 32 points of the wave
        // ---------------- input layer + hidden GEMM ----------------
        f32x16 acc[NT];
#pragma unroll
        for (int t = 0; t < NT; ++t) acc[t] = f32x16{};
#pragma unroll 1
        for (int s = 0; s < NKB; ++s) {
            // the lane's 8 consecutive k of this block: k = 16 s + 8 hl + jj
            float a0[8], a1[8], c0[8];
            const int k0 = 16 * s + 8 * hl;
            lds8(sA0 + k0, a0);
            lds8(sA1 + k0, a1);
            lds8(sb0 + k0, c0);
            bf16x8 bh, bm, bl;
#pragma unroll
            for (int jj = 0; jj < 8; ++jj) {
                const float z = fmaf(py, a1[jj], px * a0[jj]) + c0[jj];
                __bf16 a, b, c;
                split3(in_act<FOUR>(z, scale), a, b, c);
                bh[jj] = a;
                bm[jj] = b;
                bl[jj] = c;
            }
#pragma unroll
            for (int t = 0; t < NT; ++t) {
                const __bf16* rowp = sWp + (size_t)(t * 32 + il) * RS + 16 * s + 8 * hl;
                const bf16x8 ah = *reinterpret_cast<const bf16x8*>(rowp);
                const bf16x8 am = *reinterpret_cast<const bf16x8*>(rowp + (size_t)H * RS);
                const bf16x8 al = *reinterpret_cast<const bf16x8*>(rowp + (size_t)2 * H * RS);
                acc[t] = NLOT_MLP_TWOACC_FWD ? mfma6s(ah, am, al, bh, bm, bl, acc[t]) : mfma6(ah, am, al, bh, bm, bl, acc[t]);
            }
        }
        // ---------------- bias + ReLU + output layer (accumulator layout of the f32 MFMA: acc_row) ----------------
        float fpart = 0.f;
        uint64_t mk = 0;
#pragma unroll
        for (int t = 0; t < NT; ++t)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int j = t * 32 + acc_row(r, hl);
                const float v = acc[t][r] + sb[j];
                // on = v > 0 without a compare: the int image of a float is > 0 exactly for v > 0 (-0 and the
                // negatives have the sign bit); clamp(., 0, 1) is one v_med3_i32, max(v, 0) one v_max_f32
                const int on = min(max(__float_as_int(v), 0), 1);
                fpart = fmaf(sw[j], fmaxf(v, 0.f), fpart);
                mk |= (uint64_t)on << (t * 16 + r);
            }
        const float fw = fpart + __shfl_xor(fpart, 32) + w.b_out;
        if (!have) {
            f = fw;
            mask = mk;
        }
        }  // forward
        if constexpr (!FULL) {
            if (valid) {
                if (hl == 0) out.val[pi * out.sv] = f;
                if (out.mask) {
                    out.mask[(2 * hl) * out.mask_plane + pi] = (uint32_t)mask;
                    out.mask[(2 * hl + 1) * out.mask_plane + pi] = (uint32_t)(mask >> 32);
                }
            }
        } else {
            // ---------------- reverse sweep: G = W^T e, e = lam * w_out .* mask ----------------
            // e is split once into the B fragments of all 2 NT k-steps (blk = 2 tj + sl: accumulator registers
            // 8 sl .. 8 sl + 7 of output tile tj, permuted k order; 3 NT x 2 x 4 VGPRs); then output tile tk of
            // G = W^T e accumulates over the k-steps while the contraction of tile tk - 1 (whose accumulator is
            // complete) runs between its MFMAs: 2 of its 16 rows per k-step
            const float lm = lam ? (valid ? lam[pi] : 0.f) : 1.f;
            constexpr int NB = 2 * NT;
            bf16x8 Bh[NB], Bm[NB], Bl[NB];
#pragma unroll
            for (int blk = 0; blk < NB; ++blk) {
                const int tj = blk >> 1, sl = blk & 1;
#pragma unroll
                for (int jj = 0; jj < 8; ++jj) {
                    const int r = 8 * sl + jj;
                    const float e = ((mask >> (tj * 16 + r)) & 1) ? lm * sw[tj * 32 + acc_row(r, hl)] : 0.f;
                    __bf16 a, b, c;
                    split3(e, a, b, c);
                    Bh[blk][jj] = a;
                    Bm[blk][jj] = b;
                    Bl[blk][jj] = c;
                }
            }
            // g = df/dh0 (x lam): contract with the input layer's derivatives (lane: k rows, point); the four rows
            // of a register quad are consecutive k: one 16-byte read per input-layer vector
            float gx = 0.f, gy = 0.f, hxx = 0.f, hxy = 0.f, hyy = 0.f;
            const int zo = opaque_zero();
            auto contract2 = [&](const f32x16& gp, int tp, int r0) {  // rows r0, r0 + 1 of output tile tp
                const int r4 = r0 >> 2, rr0 = r0 & 3;
                const int k0 = tp * 32 + 8 * r4 + 4 * hl + zo;
                const float4 A0 = *reinterpret_cast<const float4*>(sA0 + k0);
                const float4 A1 = *reinterpret_cast<const float4*>(sA1 + k0);
                const float4 B0 = *reinterpret_cast<const float4*>(sb0 + k0);
                float4 Q0, Q1, Q2;  // A0^2, A0 A1, A1^2 (staged once per block)
                if constexpr (FOUR) {
                    Q0 = *reinterpret_cast<const float4*>(sq + k0);
                    Q1 = *reinterpret_cast<const float4*>(sq + H + k0);
                    Q2 = *reinterpret_cast<const float4*>(sq + 2 * H + k0);
                }
#pragma unroll
                for (int u = 0; u < 2; ++u) {
                    const int rr = rr0 + u;
                    const float ax = rr == 0 ? A0.x : rr == 1 ? A0.y : rr == 2 ? A0.z : A0.w;
                    const float ay = rr == 0 ? A1.x : rr == 1 ? A1.y : rr == 2 ? A1.z : A1.w;
                    const float bz = rr == 0 ? B0.x : rr == 1 ? B0.y : rr == 2 ? B0.z : B0.w;
                    const float z = fmaf(py, ay, px * ax) + bz;
                    const float d = gp[r0 + u];
                    if constexpr (FOUR) {  // the factor -scale is applied to the sums
                        const float qxx = rr == 0 ? Q0.x : rr == 1 ? Q0.y : rr == 2 ? Q0.z : Q0.w;
                        const float qxy = rr == 0 ? Q1.x : rr == 1 ? Q1.y : rr == 2 ? Q1.z : Q1.w;
                        const float qyy = rr == 0 ? Q2.x : rr == 1 ? Q2.y : rr == 2 ? Q2.z : Q2.w;
                        const float tz = turns_fourier(z);
                        const float dz = d * __builtin_amdgcn_sinf(tz);
                        const float c2 = d * __builtin_amdgcn_cosf(tz);
                        gx = fmaf(ax, dz, gx);
                        gy = fmaf(ay, dz, gy);
                        hxx = fmaf(qxx, c2, hxx);
                        hxy = fmaf(qxy, c2, hxy);
                        hyy = fmaf(qyy, c2, hyy);
                    } else {  // ReLU input layer: piecewise linear, Hessian 0 a.e.
                        const float dz = z > 0.f ? d : 0.f;
                        gx = fmaf(ax, dz, gx);
                        gy = fmaf(ay, dz, gy);
                    }
                }
            };
            static_assert(NB == 8, "2 contraction rows per k-step cover a 16-row output tile");
            f32x16 gprev = f32x16{};
#pragma unroll
            for (int tk = 0; tk < NT; ++tk) {
                f32x16 g = f32x16{}, gs = f32x16{};
#pragma unroll
                for (int blk = 0; blk < NB; ++blk) {
                    const int jbase = 16 * blk;  // 32 tj + 16 sl
                    const bf16x8 ah = wt_frag<RS>(sWp, jbase, 32 * tk, lane);
                    const bf16x8 am = wt_frag<RS>(sWp + (size_t)H * RS, jbase, 32 * tk, lane);
                    const bf16x8 al = wt_frag<RS>(sWp + (size_t)2 * H * RS, jbase, 32 * tk, lane);
                    if constexpr (NLOT_MLP_TWOACC_REV == 2) {
                        gs = mfma5s(ah, am, al, Bh[blk], Bm[blk], Bl[blk], gs);
                        g = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, Bh[blk], g, 0, 0, 0);
                    } else {
                        g = NLOT_MLP_TWOACC_REV ? mfma6s(ah, am, al, Bh[blk], Bm[blk], Bl[blk], g)
                                                : mfma6(ah, am, al, Bh[blk], Bm[blk], Bl[blk], g);
                    }
                    if (tk > 0) contract2(gprev, tk - 1, 2 * blk);
                }
                if constexpr (NLOT_MLP_TWOACC_REV == 2) g += gs;
                gprev = g;
            }
#pragma unroll
            for (int r0 = 0; r0 < 16; r0 += 2) contract2(gprev, NT - 1, r0);
            const float sg = FOUR ? -scale : 1.f;
            gx = sg * (gx + __shfl_xor(gx, 32));
            gy = sg * (gy + __shfl_xor(gy, 32));
            hxx = sg * (hxx + __shfl_xor(hxx, 32));
            hxy = sg * (hxy + __shfl_xor(hxy, 32));
            hyy = sg * (hyy + __shfl_xor(hyy, 32));
            if (valid && hl == 0) {
                out.val[pi * out.sv] = f;
                if (out.gx) {
                    out.gx[pi * out.sg] = gx;
                    out.gy[pi * out.sg] = gy;
                }
                if (out.hxx) {
                    out.hxx[pi * out.sh] = hxx;
                    out.hxy[pi * out.sh] = hxy;
                    if (out.hyx != out.hxy) out.hyx[pi * out.sh] = hxy;
                    out.hyy[pi * out.sh] = hyy;
                }
            }
        }
        in0 = in1;  // the next tile's inputs (loaded during this tile)
        in1 = in2;
        re0 = re1;
    }
    if (FULL && ru.nreused) {  // statistics: full-launch points whose forward was reused
        __syncthreads();
        if (threadIdx.x == 0 && s_reused) atomicAdd(ru.nreused, s_reused);
    }
}

int device_cus() {
    static std::atomic<int> cus[64];
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return 256;
    std::atomic<int>& c = cus[dev & 63];
    int v = c.load(std::memory_order_relaxed);
    if (v == 0) {
        hipDeviceProp_t prop;
        v = (hipGetDeviceProperties(&prop, dev) == hipSuccess && prop.multiProcessorCount > 0) ? prop.multiProcessorCount
                                                                                               : 256;
        c.store(v, std::memory_order_relaxed);
    }
    return v;
}
static int num_cus() { return device_cus(); }

template <int H, int L, bool FULL>
static int launch_t(const MlpDev& w, const float* pts, int64_t n, const int* n_dev, int P_per, int64_t ld,
                    const float* lam, const MlpOut& out, hipStream_t stream, const MlpReuse* reuse) {
    const size_t lds = sizeof(float) * mlp_lds_floats(H, L, FULL && mlp_staged(H, L));
    static std::atomic<uint64_t> attr_set{0};
    NLOT_HIP_CHECK(set_lds_attr_once(attr_set, (const void*)mlp_kernel<H, L, FULL>, 160 * 1024));
    if constexpr (L == 1 && H == 128) {
        // split-bf16 MFMA kernels (fp32-equivalent products); a net created with NLOT_MLP_ARITH_F32 (no planes) or
        // NLOT_MLP=f32 in the environment takes the f32-MFMA kernels
        static const bool use_bf16 = !(getenv("NLOT_MLP") && strcmp(getenv("NLOT_MLP"), "f32") == 0);
        if (use_bf16 && w.Wp) {
            constexpr size_t lv = mlp_bf16_lds_bytes<H>();
            static std::atomic<uint64_t> attr_v{0}, attr_f{0};
            NLOT_HIP_CHECK(set_lds_attr_once(attr_v, (const void*)mlp_bf16<H, FULL, false>, (int)lv));
            NLOT_HIP_CHECK(set_lds_attr_once(attr_f, (const void*)mlp_bf16<H, FULL, true>, (int)lv));
            constexpr int NTB = bf16_threads(FULL);
            const int64_t tiles = (n * P_per + NTB / 2 - 1) / (NTB / 2);
            const int64_t cap = num_cus();
            const int grid = (int)(tiles < cap ? (tiles > 0 ? tiles : 1) : cap);
            const MlpReuse ru = reuse ? *reuse : MlpReuse{};
            if (w.in_kind == NLOT_MLP_IN_FOURIER)
                hipLaunchKernelGGL((mlp_bf16<H, FULL, true>), dim3(grid), dim3(NTB), lv, stream, w, pts, n, n_dev,
                                   P_per, ld, lam, out, ru);
            else
                hipLaunchKernelGGL((mlp_bf16<H, FULL, false>), dim3(grid), dim3(NTB), lv, stream, w, pts, n, n_dev,
                                   P_per, ld, lam, out, ru);
            NLOT_HIP_CHECK(hipGetLastError());
            return NLOT_OK;
        }
    }
    constexpr int NTH = mlp_threads(H, L, FULL);
    int64_t tiles = (n * P_per + NTH / 2 - 1) / (NTH / 2);
    // resident blocks per CU: VGPR-limited (FULL: 1 wave/SIMD) and LDS-limited
    int64_t cap = (int64_t)num_cus() * ((!FULL && L == 1 && lds <= 80 * 1024) ? 2 : 1);
    int grid = (int)(tiles < cap ? (tiles > 0 ? tiles : 1) : cap);
    hipLaunchKernelGGL((mlp_kernel<H, L, FULL>), dim3(grid), dim3(NTH), lds, stream, w, pts, n, n_dev, P_per, ld, lam, out);
    NLOT_HIP_CHECK(hipGetLastError());
    return NLOT_OK;
}

// ---------------------------------------------------------------------------------------------
// Layer-streaming kernel for nets whose weights do not fit in LDS (the stress config 2-256x4-1: three
// 256x256 HxH layers = 768 KB of fp32; any H in {64, 128, 256} with up to kMaxStreamLayers HxH layers).
// f32-input MFMA v_mfma_f32_16x16x4_f32 (exact fp32 products): a wave owns 16 points (column = point),
// 16-unit tiles in 4 registers per lane (row 4 (lane >> 4) + i), and that accumulator is the B operand of
// the next layer's product with k = 16 T + 4 (lane >> 4) + i (k order permuted consistently on A).
// Weights pass through LDS a quarter layer (a "unit") at a time, software-pipelined: the global loads of
// unit u + 1 are issued into registers before the MFMAs of unit u, so their L2 latency hides under the
// 8192 MFMA cycles per wave of a quarter (H = 256).  A unit is stored with a row stride of H/4 + 4 floats,
// so every ds_read_b32 of an A operand (16 consecutive outputs x 4 k of the lane groups) hits 64 banks:
//   forward  y = W h:     rows j0 .. j0 + H/4 of W, k-major: sW[k][j - j0]
//   reverse  g = W^T e:   columns i0 .. i0 + H/4, as sW[j][i - i0]
// 4 waves (one per SIMD with the whole 512-register file; 64 points per block tile) share each unit: the
// weights cross L2 -> LDS 4 L x 4 B H^2 per 64 points for value + reverse sweep (3 MB at H = 256, L = 3).
// ---------------------------------------------------------------------------------------------
constexpr int kMaxStreamLayers = 4;
__host__ __device__ constexpr int stream_stride(int H) { return H / 4 + 4; }
__host__ __device__ constexpr size_t stream_lds_floats(int H) {
    return (size_t)H * stream_stride(H) + (size_t)4 * H + (size_t)kMaxStreamLayers * H;
}
typedef float f32x4 __attribute__((ext_vector_type(4)));

template <int H, bool FULL>
__global__ __launch_bounds__(256, 1) void mlp_stream(MlpDev w, const float* __restrict__ pts, int64_t cnt_host,
                                                     const int* __restrict__ cnt_dev, int P_per, int64_t ld,
                                                     const float* __restrict__ lam, MlpOut out) {
    constexpr int Q = H / 4, NQ = Q / 16, NT = H / 16, RS = stream_stride(H);
    constexpr int PF = H * H / 4096;  // float4 of a unit per thread (Q x H floats over 256 threads)
    static_assert(PF >= 1 && NQ >= 1, "H >= 64");
    extern __shared__ __attribute__((aligned(16))) float smem[];
    float* sW = smem;                  // the staged unit [H][RS]
    float* sA0 = sW + (size_t)H * RS;  // [H]
    float* sA1 = sA0 + H;              // [H]
    float* sb0 = sA1 + H;              // [H]
    float* sw = sb0 + H;               // [H]
    float* sbl = sw + H;               // [kMaxStreamLayers][H]: HxH layer biases
    const int L = w.n_hidden;
    for (int idx = threadIdx.x; idx < H; idx += 256) {
        sA0[idx] = w.A[idx];
        sA1[idx] = w.A[H + idx];
        sb0[idx] = w.b0[idx];
        sw[idx] = w.w_out[idx];
    }
    for (int idx = threadIdx.x; idx < L * H; idx += 256) sbl[idx] = w.b[idx];
    __syncthreads();  // the input layer is read by every wave before the first staging barrier
    const int64_t cnt = cnt_dev ? (int64_t)(*cnt_dev) : cnt_host;
    const int64_t npts = cnt * P_per;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int pn = lane & 15, lg = lane >> 4;  // point of the lane, lane group (k / row offset 4 lg)
    const bool fourier = w.in_kind == NLOT_MLP_IN_FOURIER;
    const float scale = w.scale;
    // units of one block tile: forward (layer l, quarter q) = 4 l + q; FULL adds the reverse sweep,
    // 4 L + 4 (L - 1 - l) + q
    const int U = FULL ? 8 * L : 4 * L;
    float4 pf[PF];
    // Forward units: a wave covers 16 rows x 16 k per float4 pass (lane = jj + 16 kk: row 16 jb + jj, k = 16 kq +
    // 4 kk .. + 3), so each transposed ds_write_b32 hits bank 16 kk + jj + const: 64 distinct banks.
    // Reverse units: 16-byte row pieces, stored as they are.
    // Per-thread parts of the unit addresses; the rest are compile-time offsets per r (a runtime-indexed
    // address set would be hoisted out of the tile loop into registers)
    constexpr int KQ = H / 16, QC = Q / 4;
    const int jj = threadIdx.x & 15, kk = (threadIdx.x >> 4) & 3, w4 = threadIdx.x >> 6;
    const int fwd_g = jj * H + 16 * w4 + 4 * kk, fwd_s = (16 * w4 + 4 * kk) * RS + jj;
    const int rev_g = (threadIdx.x / QC) * H + 4 * (threadIdx.x % QC), rev_s = (threadIdx.x / QC) * RS + 4 * (threadIdx.x % QC);
    auto fetch = [&](int u) {
        const bool fwd = u < 4 * L;
        const int l = fwd ? (u >> 2) : L - 1 - ((u - 4 * L) >> 2), q = u & 3;
        const float* src = w.W + (size_t)l * H * H + (fwd ? q * Q * H + fwd_g : q * Q + rev_g);
        if (fwd) {
#pragma unroll
            for (int r = 0; r < PF; ++r)
                pf[r] = *reinterpret_cast<const float4*>(src + 16 * ((4 * r) / KQ) * H + 16 * ((4 * r) % KQ));
        } else {
#pragma unroll
            for (int r = 0; r < PF; ++r) pf[r] = *reinterpret_cast<const float4*>(src + (256 * r / QC) * H);
        }
    };
    auto commit = [&](int u) {
        if (u < 4 * L) {
#pragma unroll
            for (int r = 0; r < PF; ++r) {
                float* d = sW + fwd_s + 16 * ((4 * r) % KQ) * RS + 16 * ((4 * r) / KQ);
                d[0] = pf[r].x;
                d[RS] = pf[r].y;
                d[2 * RS] = pf[r].z;
                d[3 * RS] = pf[r].w;
            }
        } else {
#pragma unroll
            for (int r = 0; r < PF; ++r) *reinterpret_cast<float4*>(sW + rev_s + (256 * r / QC) * RS) = pf[r];
        }
    };
    // acc_q[t] += W_unit(16 t + pn, k) B(k), k over all H (both sweeps read the unit as sW[k][16 t + pn]); the A
    // operands of group (T, i) are loaded one group ahead of its MFMAs (one wave per SIMD: nothing else hides the
    // LDS latency)
    auto unit_mfma = [&](f32x4* accq, const f32x4* bsrc) {
        float a_cur[NQ];
#pragma unroll
        for (int t = 0; t < NQ; ++t) a_cur[t] = sW[(4 * lg) * RS + 16 * t + pn];
#pragma unroll
        for (int T = 0; T < NT; ++T)
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                float a_nxt[NQ];
                if (4 * T + i + 1 < 4 * NT) {
                    const int kn = 16 * ((4 * T + i + 1) >> 2) + 4 * lg + ((i + 1) & 3);
#pragma unroll
                    for (int t = 0; t < NQ; ++t) a_nxt[t] = sW[kn * RS + 16 * t + pn];
                }
                const float bv = bsrc[T][i];
#pragma unroll
                for (int t = 0; t < NQ; ++t) accq[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a_cur[t], bv, accq[t], 0, 0, 0);
#pragma unroll
                for (int t = 0; t < NQ; ++t) a_cur[t] = a_nxt[t];
                asm volatile("" ::: "memory");  // bound the LDS loads the scheduler hoists (register file)
            }
    };
    fetch(0);
    constexpr int TP = 64;  // points per block tile (4 waves x 16, one per SIMD with the whole register file)
    for (int64_t tile = blockIdx.x; tile * TP < npts; tile += gridDim.x) {
        const int64_t gi = tile * TP + wave * 16 + pn;
        const bool valid = gi < npts;
        const int64_t pi = valid ? (ld == 0 ? gi : (gi % cnt) + (gi / cnt) * ld) : 0;
        float px = 0.f, py = 0.f;
        if (valid) {
            px = pts[2 * pi];
            py = pts[2 * pi + 1];
        }
        f32x4 acc[NT];
        uint32_t mask[kMaxStreamLayers][NT / 8 > 0 ? NT / 8 : 1];  // ReLU bit 4 (t & 7) + i of word t >> 3
        // input layer h0 (unit k = 16 T + 4 lg + i of the lane's point), computed once into the B registers
#pragma unroll
        for (int T = 0; T < NT; ++T)
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int k = 16 * T + 4 * lg + i;
                const float z = fmaf(py, sA1[k], px * sA0[k]) + sb0[k];
                if (fourier) {
                    float sn, cs;
                    sincos_fourier(z, &sn, &cs);
                    acc[T][i] = cs * scale;
                } else {
                    acc[T][i] = z > 0.f ? z : 0.f;
                }
            }
        // ---------------- forward through the HxH layers ----------------
#pragma unroll 1
        for (int l = 0; l < L; ++l) {
            f32x4 nacc[NT];
#pragma unroll
            for (int t = 0; t < NT; ++t) nacc[t] = f32x4{};
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int u = 4 * l + q;
                __syncthreads();
                commit(u);
                __syncthreads();
                fetch(u + 1 < U ? u + 1 : 0);
                unit_mfma(nacc + q * NQ, acc);
            }
            const float* bl = sbl + l * H;
#pragma unroll
            for (int t = 0; t < NT; ++t) {
                uint32_t m = 0;
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const float v = nacc[t][i] + bl[16 * t + 4 * lg + i];
                    const bool on = v > 0.f;
                    acc[t][i] = on ? v : 0.f;
                    m |= (uint32_t)on << (4 * (t & 7) + i);
                }
                if constexpr (FULL) {  // layer index is runtime: predicated writes keep the masks in registers
#pragma unroll
                    for (int ll = 0; ll < kMaxStreamLayers; ++ll)
                        if (ll == l) mask[ll][t >> 3] = (t & 7) == 0 ? m : (mask[ll][t >> 3] | m);
                }
            }
        }
        auto lsum = [](float v) {  // sum over the 4 lane groups (the 4 k / row offsets of a point)
            v += __shfl_xor(v, 16);
            return v + __shfl_xor(v, 32);
        };
        float fpart = 0.f;
#pragma unroll
        for (int t = 0; t < NT; ++t)
#pragma unroll
            for (int i = 0; i < 4; ++i) fpart = fmaf(sw[16 * t + 4 * lg + i], acc[t][i], fpart);
        const float f = lsum(fpart) + w.b_out;
        if constexpr (!FULL) {
            if (valid && lg == 0) out.val[pi * out.sv] = f;
            continue;
        } else {
            // ---------------- reverse sweep: e = lam w_out .* mask_top; g = W_l^T e; e = g .* mask_{l-1} ----
            const float lm = lam ? (valid ? lam[pi] : 0.f) : 1.f;
            auto mask_of = [&](int l, int word) {  // mask[l][word] for a runtime l, by selects
                uint32_t m = mask[0][word];
#pragma unroll
                for (int ll = 1; ll < kMaxStreamLayers; ++ll) m = ll == l ? mask[ll][word] : m;
                return m;
            };
#pragma unroll
            for (int t = 0; t < NT; ++t)
#pragma unroll
                for (int i = 0; i < 4; ++i)
                    acc[t][i] = ((mask_of(L - 1, t >> 3) >> (4 * (t & 7) + i)) & 1) ? lm * sw[16 * t + 4 * lg + i] : 0.f;
#pragma unroll 1
            for (int l = L - 1; l >= 0; --l) {
                f32x4 g[NT];
#pragma unroll
                for (int t = 0; t < NT; ++t) g[t] = f32x4{};
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const int u = 4 * L + 4 * (L - 1 - l) + q;
                    __syncthreads();
                    commit(u);
                    __syncthreads();
                    fetch(u + 1 < U ? u + 1 : 0);
                    unit_mfma(g + q * NQ, acc);
                }
                if (l > 0) {
#pragma unroll
                    for (int t = 0; t < NT; ++t)
#pragma unroll
                        for (int i = 0; i < 4; ++i) acc[t][i] = ((mask_of(l - 1, t >> 3) >> (4 * (t & 7) + i)) & 1) ? g[t][i] : 0.f;
                } else {
#pragma unroll
                    for (int t = 0; t < NT; ++t) acc[t] = g[t];
                }
            }
            // acc = lam df/dh0: contract with the input layer's derivatives (lane = (k, point))
            float gx = 0.f, gy = 0.f, hxx = 0.f, hxy = 0.f, hyy = 0.f;
#pragma unroll
            for (int t = 0; t < NT; ++t)
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const int k = 16 * t + 4 * lg + i;
                    const float ax = sA0[k], ay = sA1[k];
                    const float z = fmaf(py, ay, px * ax) + sb0[k];
                    const float d = acc[t][i];
                    float dz, c2;
                    if (fourier) {
                        float sn, cs;
                        sincos_fourier(z, &sn, &cs);
                        dz = d * (-scale * sn);
                        c2 = d * (-scale * cs);
                    } else {
                        dz = z > 0.f ? d : 0.f;
                        c2 = 0.f;
                    }
                    gx = fmaf(ax, dz, gx);
                    gy = fmaf(ay, dz, gy);
                    hxx = fmaf(ax * ax, c2, hxx);
                    hxy = fmaf(ax * ay, c2, hxy);
                    hyy = fmaf(ay * ay, c2, hyy);
                }
            gx = lsum(gx);
            gy = lsum(gy);
            hxx = lsum(hxx);
            hxy = lsum(hxy);
            hyy = lsum(hyy);
            if (valid && lg == 0) {
                out.val[pi * out.sv] = f;
                if (out.gx) {
                    out.gx[pi * out.sg] = gx;
                    out.gy[pi * out.sg] = gy;
                }
                if (out.hxx) {
                    out.hxx[pi * out.sh] = hxx;
                    out.hxy[pi * out.sh] = hxy;
                    if (out.hyx != out.hxy) out.hyx[pi * out.sh] = hxy;
                    out.hyy[pi * out.sh] = hyy;
                }
            }
        }
    }
}

template <int H, bool FULL>
static int launch_stream(const MlpDev& w, const float* pts, int64_t n, const int* n_dev, int P_per, int64_t ld,
                         const float* lam, const MlpOut& out, hipStream_t stream) {
    const size_t lds = sizeof(float) * stream_lds_floats(H);
    static std::atomic<uint64_t> attr{0};
    NLOT_HIP_CHECK(set_lds_attr_once(attr, (const void*)mlp_stream<H, FULL>, (int)lds));
    const int64_t tiles = (n * P_per + 63) / 64;
    const int64_t cap = device_cus();
    const int grid = (int)(tiles < cap ? (tiles > 0 ? tiles : 1) : cap);
    hipLaunchKernelGGL((mlp_stream<H, FULL>), dim3(grid), dim3(256), lds, stream, w, pts, n, n_dev, P_per, ld, lam, out);
    NLOT_HIP_CHECK(hipGetLastError());
    return NLOT_OK;
}

// ---------------------------------------------------------------------------------------------
// Smooth activations (tanh, sigmoid, leaky ReLU, SIREN's sine; core/nn_architectures.py:8-100 and
// l4casadi's naive MLP): the Hessian has a term from every layer, so value, gradient and Hessian are
// carried FORWARD through the net as hyper-duals in fp32 — per hidden unit the 6 components
// (a, a_x, a_y, a_xx, a_xy, a_yy) of a point, with z = W a + b linear in all of them and, per unit,
//   a = s(z), a_x = s'(z) z_x, a_xx = s''(z) z_x^2 + s'(z) z_xx, a_xy = s''(z) z_x z_y + s'(z) z_xy, ...
// A block of 256 threads owns a tile of kSmoothPB points: thread t computes hidden unit t % H for the
// points of group t / H; the layer's activations of the tile sit in LDS as [k][point][component] (one
// broadcast float4 stream per k), the weights come transposed ([in][out]: a coalesced row per k) from L2.
// These nets are not on the metric path (the reference's YAMLs use ReLU); the bound is the fp32 VALU at
// 6 H^2 FMA per point and layer.
// ---------------------------------------------------------------------------------------------
constexpr int kSmoothPB = 8;

// s(z), s'(z), s''(z) of the activation
__device__ __forceinline__ void act3(int act, float omega, float z, float& s, float& d1, float& d2) {
    if (act == NLOT_ACT_TANH) {
        s = tanhf(z);
        d1 = 1.f - s * s;
        d2 = -2.f * s * d1;
    } else if (act == NLOT_ACT_SIGMOID) {
        s = 1.f / (1.f + expf(-z));
        d1 = s * (1.f - s);
        d2 = d1 * (1.f - 2.f * s);
    } else if (act == NLOT_ACT_LEAKY_RELU) {
        s = z > 0.f ? z : 0.01f * z;
        d1 = z > 0.f ? 1.f : 0.01f;
        d2 = 0.f;
    } else if (act == NLOT_ACT_SINE) {
        const float u = omega * z;  // torch: sin(omega_0 * linear(x)), the product rounded first
        s = sinf(u);
        const float c = cosf(u);
        d1 = omega * c;
        d2 = -omega * omega * s;
    } else {  // ReLU
        s = z > 0.f ? z : 0.f;
        d1 = z > 0.f ? 1.f : 0.f;
        d2 = 0.f;
    }
}

template <int H, bool FULL>
__global__ __launch_bounds__(256) void mlp_smooth(MlpDev w, const float* __restrict__ pts, int64_t cnt_host,
                                                  const int* __restrict__ cnt_dev, int P_per, int64_t ld,
                                                  const float* __restrict__ lam, MlpOut out) {
    constexpr int NC = FULL ? 6 : 1;            // hyper-dual components carried
    constexpr int NG = 256 / H;                 // point groups of a block
    constexpr int PPT = kSmoothPB / NG;         // points per thread
    constexpr int ROW = kSmoothPB * NC;         // floats per k in LDS
    static_assert(NG >= 1 && PPT >= 1 && (PPT * NC) % 2 == 0, "mlp_smooth shape");
    __shared__ __attribute__((aligned(16))) float act_s[H * ROW];
    __shared__ float pxy[kSmoothPB][2];
    __shared__ float lam_s[kSmoothPB];
    __shared__ int64_t pidx[kSmoothPB];
    const int64_t cnt = cnt_dev ? (int64_t)(*cnt_dev) : cnt_host;
    const int64_t npts = cnt * P_per;
    const int t = threadIdx.x, i = t % H, grp = t / H, p0 = grp * PPT;
    const int act = w.act, L = w.n_hidden;
    const float omega = w.scale;
    const bool fourier = w.in_kind == NLOT_MLP_IN_FOURIER;
    for (int64_t tile = blockIdx.x; tile * kSmoothPB < npts; tile += gridDim.x) {
        if (t < kSmoothPB) {
            const int64_t gi = tile * kSmoothPB + t;
            const bool valid = gi < npts;
            const int64_t pi = valid ? (ld == 0 ? gi : (gi % cnt) + (gi / cnt) * ld) : -1;
            pidx[t] = pi;
            pxy[t][0] = valid ? pts[2 * pi] : 0.f;
            pxy[t][1] = valid ? pts[2 * pi + 1] : 0.f;
            lam_s[t] = (valid && lam) ? lam[pi] : 1.f;
        }
        __syncthreads();
        // input layer: z = p A + b0 (as torch: p @ A then + b0), dz/dp = (A0, A1), d2z = 0
        const float a0 = w.A[i], a1 = w.A[H + i], bb = w.b0[i];
#pragma unroll
        for (int q = 0; q < PPT; ++q) {
            const int p = p0 + q;
            const float z = fmaf(pxy[p][1], a1, pxy[p][0] * a0) + bb;
            float s, d1, d2;
            if (fourier) {  // scale * cos(z) (nn_architectures.py:38)
                const float sn = sinf(z), cs = cosf(z);
                s = cs * w.scale;
                d1 = -w.scale * sn;
                d2 = -w.scale * cs;
            } else {
                act3(act, omega, z, s, d1, d2);
            }
            float* dst = act_s + i * ROW + p * NC;
            dst[0] = s;
            if constexpr (FULL) {
                dst[1] = d1 * a0;
                dst[2] = d1 * a1;
                dst[3] = d2 * a0 * a0;
                dst[4] = d2 * a0 * a1;
                dst[5] = d2 * a1 * a1;
            }
        }
        __syncthreads();
        // hidden layers
#pragma unroll 1
        for (int l = 0; l < L; ++l) {
            const float* Wt = w.Wt + (size_t)l * H * H + i;
            float acc[PPT * NC];
#pragma unroll
            for (int e = 0; e < PPT * NC; ++e) acc[e] = 0.f;
            const float* src = act_s + p0 * NC;
#pragma unroll 4
            for (int k = 0; k < H; ++k) {
                const float wk = Wt[(size_t)k * H];
                const float2* ak = reinterpret_cast<const float2*>(src + k * ROW);
#pragma unroll
                for (int e2 = 0; e2 < PPT * NC / 2; ++e2) {
                    const float2 v = ak[e2];
                    acc[2 * e2] = fmaf(wk, v.x, acc[2 * e2]);
                    acc[2 * e2 + 1] = fmaf(wk, v.y, acc[2 * e2 + 1]);
                }
            }
            const float bl = w.b[(size_t)l * H + i];
            __syncthreads();  // every thread has read the layer's input
#pragma unroll
            for (int q = 0; q < PPT; ++q) {
                const float* z = acc + q * NC;
                float s, d1, d2;
                act3(act, omega, z[0] + bl, s, d1, d2);
                float* dst = act_s + i * ROW + (p0 + q) * NC;
                dst[0] = s;
                if constexpr (FULL) {
                    dst[1] = d1 * z[1];
                    dst[2] = d1 * z[2];
                    dst[3] = fmaf(d2 * z[1], z[1], d1 * z[3]);
                    dst[4] = fmaf(d2 * z[1], z[2], d1 * z[4]);
                    dst[5] = fmaf(d2 * z[2], z[2], d1 * z[5]);
                }
            }
            __syncthreads();
        }
        // output layer: thread (point, component) contracts w_out over the hidden units
        if (t < ROW) {
            const int p = t / NC, c = t % NC;
            float s = 0.f;
            for (int k = 0; k < H; ++k) s = fmaf(w.w_out[k], act_s[k * ROW + t], s);
            const int64_t pi = pidx[p];
            if (pi >= 0) {
                const float lm = lam_s[p];
                if (c == 0) out.val[pi * out.sv] = s + w.b_out;
                if constexpr (FULL) {
                    if (c == 1 && out.gx) out.gx[pi * out.sg] = lm * s;
                    if (c == 2 && out.gy) out.gy[pi * out.sg] = lm * s;
                    if (out.hxx) {
                        if (c == 3) out.hxx[pi * out.sh] = lm * s;
                        if (c == 4) {
                            out.hxy[pi * out.sh] = lm * s;
                            if (out.hyx != out.hxy) out.hyx[pi * out.sh] = lm * s;
                        }
                        if (c == 5) out.hyy[pi * out.sh] = lm * s;
                    }
                }
            }
        }
        __syncthreads();  // the tile's LDS is reused by the next one
    }
}

template <int H, bool FULL>
static int launch_smooth(const MlpDev& w, const float* pts, int64_t n, const int* n_dev, int P_per, int64_t ld,
                         const float* lam, const MlpOut& out, hipStream_t stream) {
    const int64_t tiles = (n * P_per + kSmoothPB - 1) / kSmoothPB;
    const int64_t cap = (int64_t)device_cus() * 8;
    const int grid = (int)(tiles < cap ? (tiles > 0 ? tiles : 1) : cap);
    hipLaunchKernelGGL((mlp_smooth<H, FULL>), dim3(grid), dim3(256), 0, stream, w, pts, n, n_dev, P_per, ld, lam, out);
    NLOT_HIP_CHECK(hipGetLastError());
    return NLOT_OK;
}

// ---------------------------------------------------------------------------------------------
// NLOT_MLP_ARITH_SEQ (ABI v15): the ReLU net in the reference order of every sum.  One thread per point; each dot
// product is a sequential fmaf chain over its index in increasing order with the bias added after it, FMA
// contraction off: the expression sequence of the oracle's default order (oracle/nlot_oracle.c oracle_mlp_point,
// NLOT_ORACLE_MLP_REV unset).  For a Linear + ReLU input layer (benchmark 6's trained net, l4casadi's naive MLP) the
// outputs are bitwise the oracle's; a Fourier input layer's cos / sin are the fp64 functions rounded to fp32 on both
// sides (the correctly rounded fp32 values except where the two libms' fp64 results straddle an fp32 rounding
// boundary, about once in 2^28 evaluations).  Test arithmetic: it takes the net's rounding out of a GPU-vs-oracle comparison, so that what is left
// is the solver's fp64 (tests/test_pinned_iterates_gpu.py).  Not a throughput path: VALU chains, per-thread arrays
// in scratch.  The value launches write no ReLU patterns and the full launches reuse no forward (both optional).
// ---------------------------------------------------------------------------------------------
template <int H, bool FULL>
__global__ __launch_bounds__(64) void mlp_seq(MlpDev w, const float* __restrict__ pts, int64_t cnt_host,
                                              const int* __restrict__ cnt_dev, int P_per, int64_t ld,
                                              const float* __restrict__ lam, MlpOut out) {
#pragma clang fp contract(off)
    constexpr int MW = H / 32;
    const int64_t cnt = cnt_dev ? (int64_t)(*cnt_dev) : cnt_host;
    const int64_t npts = cnt * P_per;
    const int L = w.n_hidden;
    const bool fourier = w.in_kind == NLOT_MLP_IN_FOURIER;
    for (int64_t gi = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; gi < npts; gi += (int64_t)gridDim.x * blockDim.x) {
        const int64_t pi = ld == 0 ? gi : (gi % cnt) + (gi / cnt) * ld;
        const float px = pts[2 * pi], py = pts[2 * pi + 1];
        float z0[H], h[H], hn[H];
        uint32_t mask[kMaxStreamLayers + 1][MW];
        for (int k = 0; k < H; ++k) {  // p @ A + b0 (graph ___torch_mangle_0.py)
            const float z = fmaf(py, w.A[H + k], px * w.A[k]) + w.b0[k];
            z0[k] = z;
            h[k] = fourier ? (float)cos((double)z) * w.scale : (z > 0.f ? z : 0.f);
        }
        for (int q = 0; q < MW; ++q) {
            uint32_t m = 0;
            for (int t = 0; t < 32; ++t) m |= (fourier || z0[32 * q + t] > 0.f) ? (1u << t) : 0u;
            mask[0][q] = m;
        }
        for (int l = 0; l < L; ++l) {
            const float* W = w.W + (size_t)l * H * H;
            for (int j = 0; j < H; ++j) {
                float a = 0.f;
                for (int k = 0; k < H; ++k) a = fmaf(W[(size_t)j * H + k], h[k], a);
                a += w.b[(size_t)l * H + j];
                hn[j] = a > 0.f ? a : 0.f;
            }
            for (int q = 0; q < MW; ++q) {
                uint32_t m = 0;
                for (int t = 0; t < 32; ++t) m |= hn[32 * q + t] > 0.f ? (1u << t) : 0u;
                mask[l + 1][q] = m;
            }
            for (int j = 0; j < H; ++j) h[j] = hn[j];
        }
        float f = 0.f;
        for (int j = 0; j < H; ++j) f = fmaf(w.w_out[j], h[j], f);
        out.val[pi * out.sv] = f + w.b_out;
        if constexpr (FULL) {
            // reverse sweep: d = df/dh_l, each column sum dn[k] = sum_j W[j][k] d[j] over j in increasing order
            const float lm = lam ? lam[pi] : 1.f;
            float* d = h;
            float* dn = hn;
            for (int j = 0; j < H; ++j) d[j] = lm * w.w_out[j];
            for (int l = L - 1; l >= 0; --l) {
                const float* W = w.W + (size_t)l * H * H;
                for (int j = 0; j < H; ++j) d[j] = (mask[l + 1][j >> 5] >> (j & 31)) & 1u ? d[j] : 0.f;
                for (int k = 0; k < H; ++k) {
                    float t = 0.f;
                    for (int j = 0; j < H; ++j) t = fmaf(W[(size_t)j * H + k], d[j], t);
                    dn[k] = t;
                }
                float* s = d;
                d = dn;
                dn = s;
            }
            float gx = 0.f, gy = 0.f, hxx = 0.f, hxy = 0.f, hyy = 0.f;
            for (int k = 0; k < H; ++k) {
                const float ax = w.A[k], ay = w.A[H + k];
                float dz, c2;
                if (fourier) {
                    dz = d[k] * (-w.scale * (float)sin((double)z0[k]));
                    c2 = d[k] * (-w.scale * (float)cos((double)z0[k]));
                } else {
                    dz = (mask[0][k >> 5] >> (k & 31)) & 1u ? d[k] : 0.f;
                    c2 = 0.f;  // ReLU input layer: piecewise linear, Hessian 0 a.e.
                }
                gx = fmaf(ax, dz, gx);
                gy = fmaf(ay, dz, gy);
                hxx = fmaf(ax * ax, c2, hxx);
                hxy = fmaf(ax * ay, c2, hxy);
                hyy = fmaf(ay * ay, c2, hyy);
            }
            if (out.gx) {
                out.gx[pi * out.sg] = gx;
                out.gy[pi * out.sg] = gy;
            }
            if (out.hxx) {
                out.hxx[pi * out.sh] = hxx;
                out.hxy[pi * out.sh] = hxy;
                if (out.hyx != out.hxy) out.hyx[pi * out.sh] = hxy;
                out.hyy[pi * out.sh] = hyy;
            }
        }
    }
}

template <int H, bool FULL>
static int launch_seq(const MlpDev& w, const float* pts, int64_t n, const int* n_dev, int P_per, int64_t ld,
                      const float* lam, const MlpOut& out, hipStream_t stream) {
    const int64_t blocks = (n * P_per + 63) / 64;
    const int64_t cap = (int64_t)device_cus() * 16;
    const int grid = (int)(blocks < cap ? (blocks > 0 ? blocks : 1) : cap);
    hipLaunchKernelGGL((mlp_seq<H, FULL>), dim3(grid), dim3(64), 0, stream, w, pts, n, n_dev, P_per, ld, lam, out);
    NLOT_HIP_CHECK(hipGetLastError());
    return NLOT_OK;
}

int launch_mlp_strided(const MlpDev& w, const float* pts, int64_t n, const int* n_dev, int P_per, int64_t ld,
                       const float* lam, const MlpOut& out, bool full, hipStream_t stream, const MlpReuse* reuse) {
    if (n <= 0) return NLOT_OK;
    if (w.arith == NLOT_MLP_ARITH_SEQ) {  // ReLU nets only (nlot_mlp_create_ex checks)
#define NLOT_SEQ_CASE(HH)                                                                      \
    if (w.H == HH) return full ? launch_seq<HH, true>(w, pts, n, n_dev, P_per, ld, lam, out, stream) \
                               : launch_seq<HH, false>(w, pts, n, n_dev, P_per, ld, lam, out, stream);
        NLOT_SEQ_CASE(64)
        NLOT_SEQ_CASE(128)
        NLOT_SEQ_CASE(256)
#undef NLOT_SEQ_CASE
        set_error("MLP kernel: hidden width must be 64, 128 or 256 (DESIGN.md §7)");
        return NLOT_ERR_INVALID;
    }
    if (w.act != NLOT_ACT_RELU) {  // smooth activations: forward hyper-duals (the ReLU masks / reuse do not apply)
        if (w.n_hidden < 0 || w.n_hidden > kMaxStreamLayers) {
            set_error("MLP kernel: 0 to 4 hidden HxH layers are supported for smooth activations");
            return NLOT_ERR_INVALID;
        }
#define NLOT_SMOOTH_CASE(HH)                                                                     \
    if (w.H == HH) return full ? launch_smooth<HH, true>(w, pts, n, n_dev, P_per, ld, lam, out, stream) \
                               : launch_smooth<HH, false>(w, pts, n, n_dev, P_per, ld, lam, out, stream);
        NLOT_SMOOTH_CASE(64)
        NLOT_SMOOTH_CASE(128)
        NLOT_SMOOTH_CASE(256)
#undef NLOT_SMOOTH_CASE
        set_error("MLP kernel: hidden width must be 64, 128 or 256 (DESIGN.md §7)");
        return NLOT_ERR_INVALID;
    }
    if (w.n_hidden < 1 || w.n_hidden > kMaxStreamLayers) {
        set_error("MLP kernel: 1 to 4 hidden HxH layers are supported (DESIGN.md §7)");
        return NLOT_ERR_INVALID;
    }
    // weights beyond LDS (H = 256, or more than 2 HxH layers): the layer-streaming kernel
    if (w.H == 256 || w.n_hidden > kMaxResidentLayers) {
        if (w.H == 256) return full ? launch_stream<256, true>(w, pts, n, n_dev, P_per, ld, lam, out, stream)
                                    : launch_stream<256, false>(w, pts, n, n_dev, P_per, ld, lam, out, stream);
        if (w.H == 128) return full ? launch_stream<128, true>(w, pts, n, n_dev, P_per, ld, lam, out, stream)
                                    : launch_stream<128, false>(w, pts, n, n_dev, P_per, ld, lam, out, stream);
        if (w.H == 64) return full ? launch_stream<64, true>(w, pts, n, n_dev, P_per, ld, lam, out, stream)
                                   : launch_stream<64, false>(w, pts, n, n_dev, P_per, ld, lam, out, stream);
    }
#define NLOT_MLP_CASE(HH, LL)                                                                      \
    if (w.H == HH && w.n_hidden == LL)                                                             \
        return full ? launch_t<HH, LL, true>(w, pts, n, n_dev, P_per, ld, lam, out, stream, reuse) \
                    : launch_t<HH, LL, false>(w, pts, n, n_dev, P_per, ld, lam, out, stream, reuse);
    NLOT_MLP_CASE(64, 1)
    NLOT_MLP_CASE(64, 2)
    NLOT_MLP_CASE(128, 1)
    NLOT_MLP_CASE(128, 2)
#undef NLOT_MLP_CASE
    {
        set_error("MLP kernel: hidden width must be 64, 128 or 256 (DESIGN.md §7)");
        return NLOT_ERR_INVALID;
    }
}

}  // namespace nlot

// ------------------------------------------------------------------------------------------------
// C ABI
// ------------------------------------------------------------------------------------------------
extern "C" NlotMlp* nlot_mlp_create(const NlotMlpDesc* d) { return nlot_mlp_create_ex(d, NLOT_MLP_ARITH_SPLIT_BF16); }

extern "C" NlotMlp* nlot_mlp_create_ex(const NlotMlpDesc* d, int32_t arith) {
    using namespace nlot;
    if (arith != NLOT_MLP_ARITH_SPLIT_BF16 && arith != NLOT_MLP_ARITH_F32 && arith != NLOT_MLP_ARITH_SEQ) {
        set_error("nlot_mlp_create_ex: arith must be NLOT_MLP_ARITH_SPLIT_BF16, NLOT_MLP_ARITH_F32 or NLOT_MLP_ARITH_SEQ");
        return nullptr;
    }
    if (arith == NLOT_MLP_ARITH_SEQ && d && d->act != NLOT_ACT_RELU) {
        set_error("nlot_mlp_create_ex: NLOT_MLP_ARITH_SEQ is defined for ReLU nets only");
        return nullptr;
    }
    if (!d || !d->A || !d->b0 || !d->w_out || (d->n_hidden > 0 && (!d->W || !d->b))) {
        set_error("nlot_mlp_create: null descriptor or weight pointer");
        return nullptr;
    }
    if (d->act < NLOT_ACT_RELU || d->act > NLOT_ACT_SINE ||
        (d->in_kind != NLOT_MLP_IN_FOURIER && d->in_kind != NLOT_MLP_IN_LINEAR_RELU)) {
        set_error("nlot_mlp_create: activation must be NLOT_ACT_* and the input layer Fourier or Linear+act");
        return nullptr;
    }
    const bool smooth = d->act != NLOT_ACT_RELU;
    if ((d->hidden != 64 && d->hidden != 128 && d->hidden != 256) || d->n_hidden < (smooth ? 0 : 1) ||
        d->n_hidden > kMaxStreamLayers) {
        set_error("nlot_mlp_create: hidden width 64/128/256 with 1-4 hidden HxH layers supported (0-4 for smooth "
                  "activations; DESIGN.md §7)");
        return nullptr;
    }
    const int H = d->hidden, L = d->n_hidden;
    const size_t nA = 2 * H, nb0 = H, nW = (size_t)L * H * H, nb = (size_t)L * H, nw = H;
    const bool split = arith == NLOT_MLP_ARITH_SPLIT_BF16;
    const size_t nWp = split ? (size_t)3 * H * H / 2 : 0;  // bf16 planes of layer 0, in float units
    const size_t nWt = smooth ? nW : 0;        // transposed HxH layers (mlp_smooth)
    const size_t total = nA + nb0 + nW + nb + nw + nWp + nWt + 4;
    float* blk = nullptr;
    if (hipMalloc(&blk, total * sizeof(float)) != hipSuccess) {
        set_error("nlot_mlp_create: hipMalloc failed");
        return nullptr;
    }
    float* p = blk;
    auto put = [&](const float* src, size_t cnt) -> float* {
        float* dst = p;
        if (cnt) hipMemcpy(dst, src, cnt * sizeof(float), hipMemcpyHostToDevice);
        p += cnt;
        return dst;
    };
    NlotMlp* m = new NlotMlp;
    m->block = blk;
    m->device = 0;
    (void)hipGetDevice(&m->device);
    m->dev.arith = arith;
    m->dev.in_kind = d->in_kind;
    m->dev.H = H;
    m->dev.n_hidden = L;
    m->dev.act = d->act;
    m->dev.scale = d->fourier_scale;
    m->dev.b_out = d->b_out;
    m->dev.A = put(d->A, nA);
    m->dev.b0 = put(d->b0, nb0);
    m->dev.W = put(d->W, nW);
    m->dev.b = put(d->b, nb);
    m->dev.w_out = put(d->w_out, nw);
    m->dev.Wp = nullptr;
    if (L > 0 && split) {  // layer-0 weights split into three bf16 planes, round-to-nearest-even at each step (host, exact)
        std::vector<uint16_t> planes((size_t)3 * H * H);
        auto bf16_rne = [](float x) -> uint16_t {
            uint32_t u;
            memcpy(&u, &x, 4);
            return (uint16_t)((u + 0x7FFFu + ((u >> 16) & 1u)) >> 16);
        };
        auto bf16_f = [](uint16_t h) -> float {
            const uint32_t u = (uint32_t)h << 16;
            float f;
            memcpy(&f, &u, 4);
            return f;
        };
        for (size_t i = 0; i < (size_t)H * H; ++i) {
            const float x = d->W[i];
            const uint16_t hi = bf16_rne(x);
            const float r = x - bf16_f(hi);
            const uint16_t mid = bf16_rne(r);
            const uint16_t lo = bf16_rne(r - bf16_f(mid));
            planes[i] = hi;
            planes[(size_t)H * H + i] = mid;
            planes[(size_t)2 * H * H + i] = lo;
        }
        m->dev.Wp = put(reinterpret_cast<const float*>(planes.data()), nWp);
    }
    m->dev.Wt = nullptr;
    if (smooth && L > 0) {  // [l][in][out] for mlp_smooth's coalesced rows
        std::vector<float> wt(nW);
        for (int l = 0; l < L; ++l)
            for (int o = 0; o < H; ++o)
                for (int k = 0; k < H; ++k) wt[(size_t)l * H * H + (size_t)k * H + o] = d->W[(size_t)l * H * H + (size_t)o * H + k];
        m->dev.Wt = put(wt.data(), nWt);
    }
    if (hipDeviceSynchronize() != hipSuccess) {
        set_error("nlot_mlp_create: copy failed");
        hipFree(blk);
        delete m;
        return nullptr;
    }
    return m;
}

extern "C" void nlot_mlp_destroy(NlotMlp* m) {
    if (!m) return;
    nlot::casadi_unbind(m);
    hipFree(m->block);
    delete m;
}

extern "C" int32_t nlot_sdf_mlp_eval(const NlotMlp* mlp, const float* pts, int64_t P, float* val, float* grad,
                                     const float* lam, float* hess, void* stream) {
    using namespace nlot;
    if (!mlp || !pts || !val || P < 0) {
        set_error("nlot_sdf_mlp_eval: null argument");
        return NLOT_ERR_INVALID;
    }
    MlpOut o{};
    o.val = val;
    o.sv = 1;
    if (grad) {
        o.gx = grad;
        o.gy = grad + 1;
        o.sg = 2;
    }
    if (hess) {
        o.hxx = hess;
        o.hxy = hess + 1;
        o.hyx = hess + 2;
        o.hyy = hess + 3;
        o.sh = 4;
    }
    const bool full = grad || hess;  // every kernel skips a null grad or hess plane (jac_adj1 alone is allowed)
    return launch_mlp_strided(mlp->dev, pts, P, nullptr, 1, 0, lam, o, full, (hipStream_t)stream);
}
