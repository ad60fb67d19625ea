// Probe: how v_mfma_f32_32x32x16_bf16 adds small products to a large accumulator, and whether the
// in-kernel 3-piece split is exact.  Prints one line per experiment.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstring>
#include <cmath>
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef unsigned short u16x8 __attribute__((ext_vector_type(8)));

// D = A(32x16) B(16x32) + C, lane l supplies A[l&31][8*(l>>5)+j], B[8*(l>>5)+j][l&31].
__global__ void mm(const unsigned short* A, const unsigned short* B, const float* C, float* D) {
    int l = threadIdx.x;
    u16x8 a, b;
    for (int j = 0; j < 8; ++j) {
        a[j] = A[(l & 31) * 16 + 8 * (l >> 5) + j];
        b[j] = B[(8 * (l >> 5) + j) * 32 + (l & 31)];
    }
    f32x16 c;
    for (int r = 0; r < 16; ++r) c[r] = C[((r & 3) + 8 * (r >> 2) + 4 * (l >> 5)) * 32 + (l & 31)];
    c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), c, 0, 0, 0);
    for (int r = 0; r < 16; ++r) D[((r & 3) + 8 * (r >> 2) + 4 * (l >> 5)) * 32 + (l & 31)] = c[r];
}

static unsigned short bf(float x) { unsigned u; memcpy(&u, &x, 4); return (unsigned short)(u >> 16); }

static float run(float c00, const float* prods, int np) {
    // A[0][k] = prods[k], B[k][0] = 1 -> D[0][0] = c00 + sum prods
    static unsigned short hA[32 * 16], hB[16 * 32];
    static float hC[32 * 32], hD[32 * 32];
    memset(hA, 0, sizeof hA); memset(hB, 0, sizeof hB); memset(hC, 0, sizeof hC);
    for (int k = 0; k < np; ++k) { hA[k] = bf(prods[k]); hB[k * 32] = bf(1.0f); }
    hC[0] = c00;
    unsigned short *dA, *dB; float *dC, *dD;
    hipMalloc(&dA, sizeof hA); hipMalloc(&dB, sizeof hB); hipMalloc(&dC, sizeof hC); hipMalloc(&dD, sizeof hD);
    hipMemcpy(dA, hA, sizeof hA, hipMemcpyHostToDevice); hipMemcpy(dB, hB, sizeof hB, hipMemcpyHostToDevice);
    hipMemcpy(dC, hC, sizeof hC, hipMemcpyHostToDevice);
    mm<<<1, 64>>>(dA, dB, dC, dD);
    hipMemcpy(hD, dD, sizeof hD, hipMemcpyDeviceToHost);
    hipFree(dA); hipFree(dB); hipFree(dC); hipFree(dD);
    return hD[0];
}

int main() {
    printf("# exp1: C=1, one product 2^-k\n");
    for (int k = 6; k <= 26; k += 2) {
        float p = ldexpf(1.0f, -k);
        float d = run(1.0f, &p, 1);
        printf("k=%2d  D-1=%.9g  expect=%.9g  %s\n", k, d - 1.0f, p, (d - 1.0f) == p ? "exact" : "LOST/ROUNDED");
    }
    printf("# exp2: C=0, products {1, 2^-k}\n");
    for (int k = 6; k <= 26; k += 2) {
        float p[2] = {1.0f, ldexpf(1.0f, -k)};
        float d = run(0.0f, p, 2);
        printf("k=%2d  D-1=%.9g  expect=%.9g  %s\n", k, d - 1.0f, p[1], (d - 1.0f) == p[1] ? "exact" : "LOST/ROUNDED");
    }
    printf("# exp3: C=1, 16 products of 2^-k each\n");
    for (int k = 10; k <= 30; k += 2) {
        float p[16]; for (int i = 0; i < 16; ++i) p[i] = ldexpf(1.0f, -k);
        float d = run(1.0f, p, 16);
        float e = 16 * ldexpf(1.0f, -k);
        printf("k=%2d  D-1=%.9g  expect=%.9g  %s\n", k, d - 1.0f, e, (d - 1.0f) == e ? "exact" : "LOST/ROUNDED");
    }
    printf("# exp4: C=1, product 1.5*2^-k (2 significant bits)\n");
    for (int k = 10; k <= 24; k += 2) {
        float p = 1.5f * ldexpf(1.0f, -k);
        float d = run(1.0f, &p, 1);
        printf("k=%2d  D-1=%.9g  expect=%.9g\n", k, d - 1.0f, p);
    }
    return 0;
}
