// Probe: does v_mfma_f32_32x32x16_f16 honour fp16 subnormal inputs, and does the f32 accumulator
// keep small products (as the bf16 form does, mfma_bf16_precision.hip)?
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstring>
#include <cmath>
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

__global__ void mm(const _Float16* A, const _Float16* B, const float* C, float* D) {
    int l = threadIdx.x;
    f16x8 a, b;
    for (int j = 0; j < 8; ++j) {
        a[j] = A[(l & 31) * 16 + 8 * (l >> 5) + j];
        b[j] = B[(8 * (l >> 5) + j) * 32 + (l & 31)];
    }
    f32x16 c;
    for (int r = 0; r < 16; ++r) c[r] = C[((r & 3) + 8 * (r >> 2) + 4 * (l >> 5)) * 32 + (l & 31)];
    c = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
    for (int r = 0; r < 16; ++r) D[((r & 3) + 8 * (r >> 2) + 4 * (l >> 5)) * 32 + (l & 31)] = c[r];
}

static float run(float c00, float a0, float b0) {
    static _Float16 hA[32 * 16], hB[16 * 32];
    static float hC[32 * 32], hD[32 * 32];
    memset(hA, 0, sizeof hA); memset(hB, 0, sizeof hB); memset(hC, 0, sizeof hC);
    hA[0] = (_Float16)a0; hB[0] = (_Float16)b0; hC[0] = c00;
    _Float16 *dA, *dB; float *dC, *dD;
    (void)hipMalloc(&dA, sizeof hA); (void)hipMalloc(&dB, sizeof hB); (void)hipMalloc(&dC, sizeof hC); (void)hipMalloc(&dD, sizeof hD);
    (void)hipMemcpy(dA, hA, sizeof hA, hipMemcpyHostToDevice); (void)hipMemcpy(dB, hB, sizeof hB, hipMemcpyHostToDevice);
    (void)hipMemcpy(dC, hC, sizeof hC, hipMemcpyHostToDevice);
    mm<<<1, 64>>>(dA, dB, dC, dD);
    (void)hipMemcpy(hD, dD, sizeof hD, hipMemcpyDeviceToHost);
    (void)hipFree(dA); (void)hipFree(dB); (void)hipFree(dC); (void)hipFree(dD);
    return hD[0];
}

int main() {
    printf("# subnormal fp16 inputs (min normal 2^-14): D = a*b with b = 1\n");
    for (int k = 13; k <= 24; ++k) {
        float a = ldexpf(1.0f, -k);
        float d = run(0.f, a, 1.0f);
        printf("a=2^-%d  D=%.6g  %s\n", k, d, d == a ? "exact" : (d == 0.f ? "FLUSHED" : "inexact"));
    }
    printf("# subnormal*normal product 2^-20 * 2^10\n");
    float d = run(0.f, ldexpf(1.0f, -20), 1024.f);
    printf("D=%.6g expect %.6g\n", d, ldexpf(1.0f, -10));
    printf("# C=1 plus product 2^-k (f32 accumulate)\n");
    for (int k = 16; k <= 26; k += 2) {
        float dd = run(1.0f, ldexpf(1.0f, -k / 2), ldexpf(1.0f, -(k - k / 2)));
        printf("k=%d D-1=%.6g expect %.6g\n", k, dd - 1.0f, ldexpf(1.0f, -k));
    }
    return 0;
}
