// Kernels for the older 128-px UNet (reference diffusion_model/models/old_modules.py:126-360):
// 2x2 average pooling, x2 bilinear upsampling (align_corners=False), channel LayerNorm, and the
// noise-level sinusoid broadcast into its concat channels.  All NHWC fp32 views; HBM-bound.
#include "wc_common.hpp"

namespace {

int grid_for(long n, int threads) {
    long g = (n + threads - 1) / threads;
    if (g > 16384) g = 16384;
    return (int)(g < 1 ? 1 : g);
}

// nn.AvgPool2d(2) (old_modules.py:185): ((v00 + v01) + v10) + v11, then / 4, as ATen's loop.
__global__ __launch_bounds__(256) void avgpool2_kernel(const float* __restrict__ in, int ldi,
                                                       float* __restrict__ out, int ldo, int B, int Ho,
                                                       int Wo, int C) {
    const int q = C / 4;
    const long total = (long)B * Ho * Wo * q;
    for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
         i += (long)gridDim.x * blockDim.x) {
        const int c4 = (int)(i % q);
        const long pix = i / q;
        const int x = (int)(pix % Wo);
        const int y = (int)((pix / Wo) % Ho);
        const int b = (int)(pix / ((long)Wo * Ho));
        const long r0 = ((long)(b * 2 * Ho + 2 * y) * (2 * Wo) + 2 * x) * ldi + c4 * 4;
        const long r1 = r0 + (long)(2 * Wo) * ldi;
        const f32x4 a = *reinterpret_cast<const f32x4*>(in + r0);
        const f32x4 bq = *reinterpret_cast<const f32x4*>(in + r0 + ldi);
        const f32x4 c = *reinterpret_cast<const f32x4*>(in + r1);
        const f32x4 d = *reinterpret_cast<const f32x4*>(in + r1 + ldi);
        *reinterpret_cast<f32x4*>(out + pix * ldo + c4 * 4) = (((a + bq) + c) + d) / 4.0f;
    }
}

// nn.Upsample(scale_factor=2, mode='bilinear', align_corners=False) (old_modules.py:219):
// src = 0.5*(dst + 0.5) - 0.5 clamped at 0, i0 = floor, i1 = min(i0 + 1, in - 1).
__global__ __launch_bounds__(256) void upsample2_kernel(const float* __restrict__ in, int ldi,
                                                        float* __restrict__ out, int ldo, int B, int Hi,
                                                        int Wi, int C) {
    const int q = C / 4;
    const int Ho = 2 * Hi, Wo = 2 * Wi;
    const long total = (long)B * Ho * Wo * q;
    for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
         i += (long)gridDim.x * blockDim.x) {
        const int c4 = (int)(i % q);
        const long pix = i / q;
        const int x = (int)(pix % Wo);
        const int y = (int)((pix / Wo) % Ho);
        const int b = (int)(pix / ((long)Wo * Ho));
        float sy = fmaxf(0.5f * ((float)y + 0.5f) - 0.5f, 0.f);
        float sx = fmaxf(0.5f * ((float)x + 0.5f) - 0.5f, 0.f);
        const int y0 = (int)sy, x0 = (int)sx;
        const int y1 = y0 + (y0 < Hi - 1 ? 1 : 0), x1 = x0 + (x0 < Wi - 1 ? 1 : 0);
        const float ly1 = sy - (float)y0, lx1 = sx - (float)x0;
        const float ly0 = 1.f - ly1, lx0 = 1.f - lx1;
        const float* base = in + (long)b * Hi * Wi * ldi + c4 * 4;
        const f32x4 v00 = *reinterpret_cast<const f32x4*>(base + ((long)y0 * Wi + x0) * ldi);
        const f32x4 v01 = *reinterpret_cast<const f32x4*>(base + ((long)y0 * Wi + x1) * ldi);
        const f32x4 v10 = *reinterpret_cast<const f32x4*>(base + ((long)y1 * Wi + x0) * ldi);
        const f32x4 v11 = *reinterpret_cast<const f32x4*>(base + ((long)y1 * Wi + x1) * ldi);
        *reinterpret_cast<f32x4*>(out + pix * ldo + c4 * 4) =
            ly0 * (lx0 * v00 + lx1 * v01) + ly1 * (lx0 * v10 + lx1 * v11);
    }
}

// LayerNorm over the channels of every pixel (nn.LayerNorm([C]) on (B, N, C) tokens,
// old_modules.py:80-85).  One wave per pixel; two-pass mean / biased variance.
__global__ __launch_bounds__(256) void layernorm_kernel(const float* __restrict__ in, int ldi,
                                                        const float* __restrict__ g,
                                                        const float* __restrict__ bta, float eps,
                                                        float* __restrict__ out, int ldo, long P,
                                                        int C) {
    const int lane = threadIdx.x & 63;
    const long wave = ((long)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const long nw = ((long)gridDim.x * blockDim.x) >> 6;
    for (long p = wave; p < P; p += nw) {
        const float* row = in + p * ldi;
        float s = 0.f;
        for (int c = lane; c < C; c += 64) s += row[c];
        const float mean = wave_sum(s) / (float)C;
        float v = 0.f;
        for (int c = lane; c < C; c += 64) {
            const float d = row[c] - mean;
            v = fmaf(d, d, v);
        }
        const float rstd = 1.0f / sqrtf(wave_sum(v) / (float)C + eps);
        float* o = out + p * ldo;
        for (int c = lane; c < C; c += 64) o[c] = (row[c] - mean) * rstd * g[c] + bta[c];
    }
}

// UNet.sinusoidal_embedding + nearest upsample (old_modules.py:283-317): channel k of pixel
// (b, y, x) = sin(ang_k * noise_b) for k < K, cos(ang_{k-K} * noise_b) otherwise.
__global__ __launch_bounds__(256) void noise_embed_kernel(const float* __restrict__ noise,
                                                          const float* __restrict__ ang, int K,
                                                          float* __restrict__ out, int ldo, int B,
                                                          int HW) {
    const long total = (long)B * HW * 2 * K;
    for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
         i += (long)gridDim.x * blockDim.x) {
        const int k = (int)(i % (2 * K));
        const long pix = i / (2 * K);
        const int b = (int)(pix / HW);
        const float a = ang[k % K] * noise[b];
        out[pix * ldo + k] = k < K ? sinf(a) : cosf(a);
    }
}

}  // namespace

extern "C" int wc_avgpool2x2(const float* in, int ldi, float* out, int ldo, int B, int H, int W,
                             int C, void* stream) {
    if (!in || !out) return WC_E_ARG;
    if (C % 4 || ldi % 4 || ldo % 4 || H % 2 || W % 2) return WC_E_SHAPE;
    long total = (long)B * (H / 2) * (W / 2) * (C / 4);
    hipLaunchKernelGGL(avgpool2_kernel, dim3(grid_for(total, 256)), dim3(256), 0,
                       reinterpret_cast<hipStream_t>(stream), in, ldi, out, ldo, B, H / 2, W / 2, C);
    WC_CHECK_LAUNCH();
    return WC_OK;
}

extern "C" int wc_upsample2x_bilinear(const float* in, int ldi, float* out, int ldo, int B, int H,
                                      int W, int C, void* stream) {
    if (!in || !out) return WC_E_ARG;
    if (C % 4 || ldi % 4 || ldo % 4) return WC_E_SHAPE;
    long total = (long)B * 4 * H * W * (C / 4);
    hipLaunchKernelGGL(upsample2_kernel, dim3(grid_for(total, 256)), dim3(256), 0,
                       reinterpret_cast<hipStream_t>(stream), in, ldi, out, ldo, B, H, W, C);
    WC_CHECK_LAUNCH();
    return WC_OK;
}

extern "C" int wc_layernorm_channels(const float* in, int ldi, const float* gamma, const float* beta,
                                     float eps, float* out, int ldo, int64_t P, int C, void* stream) {
    if (!in || !out || !gamma || !beta) return WC_E_ARG;
    if (C <= 0 || P <= 0) return WC_E_SHAPE;
    hipLaunchKernelGGL(layernorm_kernel, dim3(grid_for(P * 64, 256)), dim3(256), 0,
                       reinterpret_cast<hipStream_t>(stream), in, ldi, gamma, beta, eps, out, ldo,
                       (long)P, C);
    WC_CHECK_LAUNCH();
    return WC_OK;
}

extern "C" int wc_noise_embed(const float* noise, const float* ang, int K, float* out, int ldo,
                              int B, int HW, void* stream) {
    if (!noise || !ang || !out) return WC_E_ARG;
    if (K <= 0 || B <= 0 || HW <= 0) return WC_E_SHAPE;
    long total = (long)B * HW * 2 * K;
    hipLaunchKernelGGL(noise_embed_kernel, dim3(grid_for(total, 256)), dim3(256), 0,
                       reinterpret_cast<hipStream_t>(stream), noise, ang, K, out, ldo, B, HW);
    WC_CHECK_LAUNCH();
    return WC_OK;
}
