// How does v_mfma_f32_32x32x16_bf16 round its fp32 accumulation?  (Diagnostics for DESIGN.md §5, GPU box.)
//
// A = all-ones (bf16 1.0), so C[m][n] = acc[m][n] + sum_k B[k][n]: each column n is one test of how 16 exact bf16
// products are added to an fp32 accumulator.  Printed per column: the expected value under (a) exact sum then one
// round-to-nearest-even, (b) round toward zero, and the hardware's result (hex).
//     hipcc --offload-arch=gfx950 -O2 -o /tmp/mfma_round_probe scripts/mfma_round_probe.hip && /tmp/mfma_round_probe
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

__global__ void probe(const float* bcols, const float* acc_in, float* out) {
    const int lane = threadIdx.x, col = lane & 31, hl = lane >> 5;
    bf16x8 a, b;
    for (int j = 0; j < 8; ++j) {
        a[j] = (__bf16)1.0f;
        b[j] = (__bf16)bcols[col * 16 + 8 * hl + j];  // exactly representable values only
    }
    f32x16 acc;
    for (int r = 0; r < 16; ++r) acc[r] = acc_in[col];
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc, 0, 0, 0);
    if (hl == 0) out[col] = acc[0];  // row 0
}

static uint32_t bits(float f) {
    uint32_t u;
    memcpy(&u, &f, 4);
    return u;
}

int main() {
    float B[32 * 16] = {}, acc[32] = {}, out[32] = {};
    const char* what[32] = {};
    int n = 0;
    auto col = [&](const char* w, float a) {
        what[n] = w;
        acc[n] = a;
        return n++;
    };
    const float u23 = ldexpf(1.f, -23), u24 = ldexpf(1.f, -24);
    int c;
    c = col("1 + 0.75 ulp (one product)", 1.f);
    B[c * 16] = 1.5f * u24;
    c = col("1 + 16 x 0.047 ulp (= 0.75 ulp)", 1.f);
    for (int k = 0; k < 16; ++k) B[c * 16 + k] = 1.5f * ldexpf(1.f, -28);
    c = col("1 - 0.25 ulp(below 1)", 1.f);
    B[c * 16] = -0.25f * u24;
    c = col("-1 - 0.75 ulp", -1.f);
    B[c * 16] = -1.5f * u24;
    c = col("1 + 0.5 ulp (tie, even = 1)", 1.f);
    B[c * 16] = 0.5f * u23;
    c = col("(1 + ulp) + 0.5 ulp (tie, even = 1 + 2 ulp)", 1.f + u23);
    B[c * 16] = 0.5f * u23;
    c = col("1 + 0.4 ulp", 1.f);
    B[c * 16] = ldexpf(1.625f, -25);  // 0.406 ulp
    c = col("1 + 0.6 ulp", 1.f);
    B[c * 16] = ldexpf(1.1875f, -24);  // 0.594 ulp
    c = col("0 + (1 + 2^-8) - 1 (cancellation)", 0.f);
    B[c * 16] = 1.f + ldexpf(1.f, -7);
    B[c * 16 + 1] = -1.f;
    c = col("1e-3 + 16 products of mixed sign", 1e-3f);
    for (int k = 0; k < 16; ++k) B[c * 16 + k] = (k & 1 ? -1.f : 1.f) * ldexpf(1.f + (k & 7) / 8.f, -20 - k);
    // the accumulation window: 16 equal small addends of either sign against a unit accumulator (or a unit product)
    for (int sgn = 1; sgn >= -1; sgn -= 2)
        for (int k = 24; k <= 30; k += 2) {
            static char lbl[64][64];
            snprintf(lbl[n], 64, "acc 1 + 16 x (%+d.5 * 2^-%d)", sgn, k);
            c = col(lbl[n], 1.f);
            for (int q = 0; q < 16; ++q) B[c * 16 + q] = sgn * 1.5f * ldexpf(1.f, -k);
        }
    for (int sgn = 1; sgn >= -1; sgn -= 2)
        for (int k = 26; k <= 30; k += 4) {
            static char lbl2[64][64];
            snprintf(lbl2[n], 64, "acc 0, product 1 + 15 x (%+d.5 * 2^-%d)", sgn, k);
            c = col(lbl2[n], 0.f);
            B[c * 16] = 1.f;
            for (int q = 1; q < 16; ++q) B[c * 16 + q] = sgn * 1.5f * ldexpf(1.f, -k);
        }
    float *dB, *dA, *dO;
    hipMalloc(&dB, sizeof B);
    hipMalloc(&dA, sizeof acc);
    hipMalloc(&dO, sizeof out);
    hipMemcpy(dB, B, sizeof B, hipMemcpyHostToDevice);
    hipMemcpy(dA, acc, sizeof acc, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, dB, dA, dO);
    hipMemcpy(out, dO, sizeof out, hipMemcpyDeviceToHost);
    for (int i = 0; i < n; ++i) {
        double exact = acc[i];
        for (int k = 0; k < 16; ++k) exact += (double)(float)(__bf16)B[i * 16 + k];
        const float rne = (float)exact;
        float rz = rne;
        if ((double)rne != exact && fabs((double)rne) > fabs(exact)) rz = nextafterf(rne, 0.f);
        printf("%-46s exact %.12e  RNE %08x  RZ %08x  MFMA %08x  %-5s  (MFMA - exact) / 2^-30 = %+.3f\n", what[i], exact,
               bits(rne), bits(rz), bits(out[i]), bits(out[i]) == bits(rne) ? "=RNE" : bits(out[i]) == bits(rz) ? "=RZ" : "other",
               ((double)out[i] - exact) * 1073741824.0);
    }
    return 0;
}
