// Probe 2: accuracy model of v_mfma_f32_32x32x16_bf16 on random data.  For each of 32x32 outputs,
// compare D = C + sum_k A[i][k] B[k][j] against the exact value (double) rounded to fp32, in units
// of ulp(|exact|) and of ulp(max(|C|, max|product|)).  Scales: C ~ N(0,1), products ~ 2^-s.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstring>
#include <cmath>
#include <cstdlib>
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef unsigned short u16x8 __attribute__((ext_vector_type(8)));

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
static float fb(unsigned short h) { unsigned u = (unsigned)h << 16; float f; memcpy(&f, &u, 4); return f; }
static double gauss() {
    double u1 = (rand() + 1.0) / (RAND_MAX + 2.0), u2 = (rand() + 1.0) / (RAND_MAX + 2.0);
    return sqrt(-2 * log(u1)) * cos(6.283185307179586 * u2);
}
static double ulp(double x) { int e; frexp(x == 0 ? 1e-30 : x, &e); return ldexp(1.0, e - 24); }

int main() {
    static unsigned short hA[32 * 16], hB[16 * 32];
    static float hC[32 * 32], hD[32 * 32];
    unsigned short *dA, *dB; float *dC, *dD;
    (void)hipMalloc(&dA, sizeof hA); (void)hipMalloc(&dB, sizeof hB);
    (void)hipMalloc(&dC, sizeof hC); (void)hipMalloc(&dD, sizeof hD);
    for (int s : {0, 4, 8, 12, 16, 20}) {
        for (int cz = 0; cz < 2; ++cz) {
            double max_ulp_exact = 0, max_ulp_big = 0, sum_err = 0, sum_abs = 0;
            int n_exact = 0, n = 0;
            for (int rep = 0; rep < 20; ++rep) {
                for (int i = 0; i < 32 * 16; ++i) hA[i] = bf((float)(gauss() * ldexp(1.0, -s / 2)));
                for (int i = 0; i < 16 * 32; ++i) hB[i] = bf((float)(gauss() * ldexp(1.0, -(s - s / 2))));
                for (int i = 0; i < 32 * 32; ++i) hC[i] = cz ? 0.f : (float)gauss();
                (void)hipMemcpy(dA, hA, sizeof hA, hipMemcpyHostToDevice);
                (void)hipMemcpy(dB, hB, sizeof hB, hipMemcpyHostToDevice);
                (void)hipMemcpy(dC, hC, sizeof hC, hipMemcpyHostToDevice);
                mm<<<1, 64>>>(dA, dB, dC, dD);
                (void)hipMemcpy(hD, dD, sizeof hD, hipMemcpyDeviceToHost);
                for (int i = 0; i < 32; ++i)
                    for (int j = 0; j < 32; ++j) {
                        double ex = hC[i * 32 + j], big = fabs(hC[i * 32 + j]);
                        for (int k = 0; k < 16; ++k) {
                            double p = (double)fb(hA[i * 16 + k]) * fb(hB[k * 32 + j]);
                            ex += p;
                            big = fmax(big, fabs(p));
                        }
                        double d = hD[i * 32 + j];
                        double e = d - ex;
                        max_ulp_exact = fmax(max_ulp_exact, fabs(e) / ulp(ex));
                        max_ulp_big = fmax(max_ulp_big, fabs(e) / ulp(big));
                        n_exact += (d == (double)(float)ex);
                        sum_err += e;
                        sum_abs += fabs(e) / ulp(big);
                        ++n;
                    }
            }
            printf("products~2^-%2d C=%s: max err %.2f ulp(exact) %.3f ulp(max term); mean |err| %.3f ulp(max term); "
                   "bias %+.3e; %d/%d equal RNE(exact)\n", s, cz ? "0   " : "N(0,1)", max_ulp_exact, max_ulp_big,
                   sum_abs / n, sum_err / n, n_exact, n);
        }
    }
    return 0;
}
