// Swift-SRGAN x4 generator (reference srgan_model/models.py:65-92), the depthwise half of every
// SeperableConv2d (:6-21): nn.Conv2d(C, C, K, padding=K//2, groups=C) on an NHWC fp32 view.  The
// pointwise half, BatchNorm (folded), PReLU, PixelShuffle (as four output maps), the residual adds
// and the (tanh + 1)/2 head run in wc_conv_igemm's epilogue.
//
// Tile: 32 x 8 output pixels x NQ channel quads per workgroup.  The (8+K-1) x (32+K-1) halo of
// those channels is staged in LDS once (zero padding written explicitly); each thread owns one
// column and NQ rows of one quad and slides down the K taps of a column so that every halo row it
// reads feeds all of its rows (K+NQ-1 LDS reads per tap column instead of K*NQ).  fp32 FMAs in the
// torch tap order (ky-major, kx-minor) starting from the bias.
// Memory-bound: one read of the input (+ halo re-reads from LDS), one write of the output.
#include "wc_common.hpp"

namespace {

constexpr int DW_TW = 32;
constexpr int DW_TH = 8;
constexpr int DW_NT = 256;

template <int K, int NQ>
__global__ __launch_bounds__(DW_NT) void dwconv_kernel(const float* __restrict__ x, int ldx, float* __restrict__ out,
                                                      int ldo, const float* __restrict__ w,
                                                      const float* __restrict__ bias, int H, int W, int C,
                                                      int tiles_x, int tiles_y) {
    constexpr int HW_ = DW_TW + K - 1;
    constexpr int HH = DW_TH + K - 1;
    constexpr int R = DW_TH * NQ * DW_TW / DW_NT;  // rows per thread (NQ = 4 -> 4, NQ = 1 -> 1)
    static_assert(R * DW_NT == DW_TH * NQ * DW_TW, "tile / thread mapping");
    __shared__ f32x4 halo[HH * HW_ * NQ];
    __shared__ f32x4 wsm[K * K * NQ];

    const int tile = blockIdx.x;
    const int tx = tile % tiles_x;
    const int ty = (tile / tiles_x) % tiles_y;
    const int b = tile / (tiles_x * tiles_y);
    const int c0 = blockIdx.y * NQ * 4;
    const int x0 = tx * DW_TW, y0 = ty * DW_TH;
    const int nq = min(NQ, (C - c0) / 4);  // quads present in this channel group

    for (int i = threadIdx.x; i < HH * HW_ * NQ; i += DW_NT) {
        const int q = i % NQ;
        const int hp = i / NQ;
        const int hx = hp % HW_, hy = hp / HW_;
        const int gy = y0 + hy - K / 2, gx = x0 + hx - K / 2;
        f32x4 v = {0.f, 0.f, 0.f, 0.f};
        if (q < nq && gy >= 0 && gy < H && gx >= 0 && gx < W)
            v = *reinterpret_cast<const f32x4*>(x + ((long)(b * H + gy) * W + gx) * ldx + c0 + 4 * q);
        halo[i] = v;
    }
    for (int i = threadIdx.x; i < K * K * NQ; i += DW_NT) {
        const int q = i % NQ, tap = i / NQ;
        f32x4 v = {0.f, 0.f, 0.f, 0.f};
        if (q < nq) {
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] = w[(long)(c0 + 4 * q + e) * K * K + tap];
        }
        wsm[i] = v;
    }
    __syncthreads();

    const int q = threadIdx.x % NQ;
    const int col = (threadIdx.x / NQ) % DW_TW;
    const int r0 = (threadIdx.x / (NQ * DW_TW)) * R;
    if (q >= nq) return;
    f32x4 bv = {0.f, 0.f, 0.f, 0.f};
    if (bias) bv = *reinterpret_cast<const f32x4*>(bias + c0 + 4 * q);
    f32x4 acc[R];
#pragma unroll
    for (int r = 0; r < R; ++r) acc[r] = bv;
    // torch order: for each output, taps ky-major, kx-minor.  Iterating ky outermost keeps that order
    // per output while each halo row is read once per (ky, kx) for all R rows.  K = 9 keeps the ky loop
    // rolled: fully unrolled, the 9 x 9 x R halo reads were hoisted into 512 registers and spilled (346
    // VGPR spills, 4.96 ms for the 1024^2 64-channel head of the SRGAN)
    constexpr int KY_UNROLL = K <= 3 ? K : 1;
#pragma unroll KY_UNROLL
    for (int ky = 0; ky < K; ++ky) {
#pragma unroll
        for (int kx = 0; kx < K; ++kx) {
            const f32x4 wv = wsm[(ky * K + kx) * NQ + q];
#pragma unroll
            for (int r = 0; r < R; ++r) {
                const f32x4 hv = halo[((r0 + r + ky) * HW_ + col + kx) * NQ + q];
#pragma unroll
                for (int e = 0; e < 4; ++e) acc[r][e] = fmaf(hv[e], wv[e], acc[r][e]);
            }
        }
    }
    const int gx = x0 + col;
    if (gx >= W) return;
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int gy = y0 + r0 + r;
        if (gy < H) *reinterpret_cast<f32x4*>(out + ((long)(b * H + gy) * W + gx) * ldo + c0 + 4 * q) = acc[r];
    }
}

template <int K>
int launch_dw(const float* x, int ldx, float* out, int ldo, const float* w, const float* bias, int B, int H, int W,
              int C, hipStream_t s) {
    const int tiles_x = (W + DW_TW - 1) / DW_TW, tiles_y = (H + DW_TH - 1) / DW_TH;
    const long ntiles = (long)B * tiles_x * tiles_y;
    if (ntiles >= (1L << 31)) return WC_E_SHAPE;
    if (C >= 16) {
        wc_last_kernel = K == 3 ? "dwconv_kernel<3, 4>" : "dwconv_kernel<9, 4>";
        hipLaunchKernelGGL((dwconv_kernel<K, 4>), dim3((unsigned)ntiles, (C + 15) / 16), dim3(DW_NT), 0, s, x, ldx,
                           out, ldo, w, bias, H, W, C, tiles_x, tiles_y);
    } else {
        wc_last_kernel = K == 3 ? "dwconv_kernel<3, 1>" : "dwconv_kernel<9, 1>";
        hipLaunchKernelGGL((dwconv_kernel<K, 1>), dim3((unsigned)ntiles, C / 4), dim3(DW_NT), 0, s, x, ldx, out, ldo,
                           w, bias, H, W, C, tiles_x, tiles_y);
    }
    WC_CHECK_LAUNCH();
    return WC_OK;
}

}  // namespace

extern "C" int wc_dwconv(const float* x, int ldx, float* out, int ldo, const float* w, const float* bias, int B,
                         int H, int W, int C, int K, void* stream) {
    if (!x || !out || !w) return WC_E_ARG;
    if (B < 1 || H < 1 || W < 1 || C < 4 || C % 4 || ldx % 4 || ldo % 4 || ldx < C || ldo < C) return WC_E_SHAPE;
    if (((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(out)) & 15) != 0) return WC_E_SHAPE;
    if (bias && (reinterpret_cast<uintptr_t>(bias) & 15) != 0) return WC_E_SHAPE;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    switch (K) {
        case 3: return launch_dw<3>(x, ldx, out, ldo, w, bias, B, H, W, C, s);
        case 9: return launch_dw<9>(x, ldx, out, ldo, w, bias, B, H, W, C, s);
        default: return WC_E_SHAPE;
    }
}
