// Weight re-packing for the split-precision kernels, on the device in one launch per weight: the
// layouts of kernels.pack_x6 / kernels.pack_f16x3 (the torch-op definitions, kept as the reference
// and compared bit for bit in tests/test_gpu_train.py).  The training step re-packs every weight
// after each optimizer step (train_ddpm.py:110-111); ~20 torch ops per weight made that a
// host-launch-bound few thousand small kernels per iteration.
//
// Input w: [N][ldw] fp32, columns K = ntaps * C0 (segment 0, column tap * C0 + c) + C1 (the 1x1
// residual segment).  Output per N tile t (BN rows) a row of int16 bit patterns:
//   segment 0, S0 = ntaps * C0 / 16 steps: [step][piece P0][k-half 2][BN][8]
//   segment 1, S1 = C1 / 16 steps:          [step][piece P1][k-half 2][BN][8]
// step order 'halo' (order == 0): s = (c / 16) * ntaps + tap; 'natural' (order == 1): s = k / 16.
// mode 0 (bf16x6): P0 = P1 = 3 exact truncated bf16 pieces, no scale.
// mode 1 (f16x3): per row n a power-of-two scale 2^sW[n], sW = clamp(14 - ceil(log2 max|w[n, k]|),
//   -60, 60) over segment 0 (and segment 1 when res_f16), 0 for an all-zero row; segment 0 as two
//   round-to-nearest fp16 pieces (h, fp16(v - h)); segment 1 as two fp16 pieces (res_f16) or three
//   bf16 pieces, same scale; wsinv[n] = 2^-sW[n].  Rows n >= N (tile padding) are zero, wsinv 1.
#include <hip/hip_fp16.h>

#include "wc_x6.hpp"

namespace {

constexpr int PK_THREADS = 256;

__device__ __forceinline__ unsigned short bf16_hi(float v) { return (unsigned short)(__float_as_uint(v) >> 16); }
__device__ __forceinline__ float bf16_val(unsigned short p) { return __uint_as_float((unsigned)p << 16); }

__global__ __launch_bounds__(PK_THREADS) void pack_split_kernel(const float* __restrict__ w, int ldw, int N, int C0,
                                                                int ntaps, int C1, int order, int mode, int res_f16,
                                                                int BN, short* __restrict__ out,
                                                                float* __restrict__ wsinv) {
    const int n = blockIdx.x;
    const int t = n / BN, nn = n - t * BN;
    const int K0 = ntaps * C0, K = K0 + C1;
    const bool live = n < N;
    const float* row = w + (long)(live ? n : 0) * ldw;
    // per-row power-of-two scale (f16x3)
    int sw = 0;
    if (mode == 1) {
        __shared__ float red[PK_THREADS / 64];
        const int Ks = res_f16 ? K : K0;
        float m = 0.f;
        if (live)
            for (int k = threadIdx.x; k < Ks; k += PK_THREADS) m = fmaxf(m, fabsf(row[k]));
        m = wave_max(m);
        if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
        __syncthreads();
        m = red[0];
        for (int i = 1; i < PK_THREADS / 64; ++i) m = fmaxf(m, red[i]);
        if (m > 0.f) {
            int e;
            const float fr = frexpf(m, &e);             // m = fr * 2^e, fr in [0.5, 1)
            const int cl = (fr == 0.5f) ? e - 1 : e;    // ceil(log2 m)
            sw = min(60, max(-60, 14 - cl));
        }
        if (threadIdx.x == 0) wsinv[n] = ldexpf(1.f, -sw);
    }
    const float sc = ldexpf(1.f, sw);
    const int P0 = mode == 1 ? 2 : 3;
    const int P1 = (mode == 1 && res_f16) ? 2 : 3;
    const long S0 = K0 / 16, S1 = C1 / 16;
    const long trow = (S0 * P0 + S1 * P1) * 2 * BN * 8;
    short* dst = out + t * trow;
    for (int k = threadIdx.x; k < K; k += PK_THREADS) {
        const float v = live ? row[k] * sc : 0.f;  // exact: power-of-two scale
        long s;
        int kk, P;
        long base;
        bool f16;
        if (k < K0) {
            if (order == 0) {
                const int tap = k / C0, c = k - tap * C0;
                s = (long)(c >> 4) * ntaps + tap;
                kk = c & 15;
            } else {
                s = k >> 4;
                kk = k & 15;
            }
            P = P0;
            base = 0;
            f16 = mode == 1;
        } else {
            const int k1 = k - K0;
            s = k1 >> 4;
            kk = k1 & 15;
            P = P1;
            base = S0 * P0 * 2 * BN * 8;
            f16 = mode == 1 && res_f16;
        }
        const long idx0 = base + (s * P * 2 + (kk >> 3)) * BN * 8 + nn * 8 + (kk & 7);
        const long pstride = 2L * BN * 8;
        if (f16) {  // (the bf16 single-piece build: the bf16 piece, wcx6::split2_one)
            unsigned short h, l;
            wcx6::split2_one(v, h, l);
            dst[idx0] = (short)h;
            dst[idx0 + pstride] = (short)l;
        } else {
            const unsigned short p0 = bf16_hi(v);
            const float r1 = v - bf16_val(p0);
            const unsigned short p1 = bf16_hi(r1);
            const float r2 = r1 - bf16_val(p1);
            dst[idx0] = (short)p0;
            dst[idx0 + pstride] = (short)p1;
            dst[idx0 + 2 * pstride] = (short)bf16_hi(r2);
        }
    }
}

}  // namespace

extern "C" int wc_pack_split(const float* w, int ldw, int N, int C0, int ntaps, int C1, int order, int mode,
                             int res_f16, int BN, void* out, int64_t out_bytes, float* wsinv, void* stream) {
    if (!w || !out || (mode == 1 && !wsinv)) return WC_E_ARG;
    if (N <= 0 || C0 <= 0 || C0 % 16 || C1 < 0 || C1 % 16 || ntaps < 1 || ldw < ntaps * C0 + C1) return WC_E_SHAPE;
    if ((order != 0 && order != 1) || (mode != 0 && mode != 1) || (BN != 64 && BN != 128)) return WC_E_ARG;
    if (order == 0 && ntaps != 9 && ntaps != 4) return WC_E_ARG;
    const long Np = (long)(N + BN - 1) / BN * BN;
    const long S0 = (long)ntaps * C0 / 16, S1 = C1 / 16;
    const int P0 = mode == 1 ? 2 : 3, P1 = (mode == 1 && res_f16) ? 2 : 3;
    const long bytes = (Np / BN) * (S0 * P0 + S1 * P1) * 2 * BN * 8 * 2;
    if (out_bytes != bytes) return WC_E_SHAPE;
    wc_last_kernel = "pack_split_kernel";
    hipLaunchKernelGGL(pack_split_kernel, dim3((unsigned)Np), dim3(PK_THREADS), 0, reinterpret_cast<hipStream_t>(stream),
                       w, ldw, N, C0, ntaps, C1, order, mode, res_f16, BN, reinterpret_cast<short*>(out), wsinv);
    WC_CHECK_LAUNCH();
    return WC_OK;
}
