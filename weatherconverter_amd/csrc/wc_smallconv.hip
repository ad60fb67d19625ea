// Training kernels of the UNet's two 3-channel convs (reference unet_base.py:400 conv_in, 3 -> 64;
// :448-449,483-485 norm_out -> SiLU -> conv_out, 64 -> 3), the pieces of train_ddpm.py:94-114's
// loss.backward() that a split-precision MFMA tile handles badly: with 3 channels on one side of the
// GEMM an MFMA tile pads that side 20x (the generic kernels took 2.3 / 0.57 / 0.51 ms per B=32
// iteration, profiles/r05_train_bf16_launch_shapes.txt).  These are fp32 VALU kernels bound by the
// 64-channel tensor's HBM traffic:
//   head_dgrad_kernel   dz[b][y][x][c] = sum_{n, ky, kx} g[b][n][y + 1 - ky][x + 1 - kx] w[n][c][ky][kx]
//                       (the transposed conv of the NCHW loss gradient; one read of g, one write of dz)
//   head_wgrad_kernel   dW[n][c][ky][kx] = sum_{b, y, x} g[b][n][y][x] act[b][y + ky - 1][x + kx - 1][c],
//                       act = SiLU(x sc + sh) (the forward's prologue, silu_fast), zero outside the image
//   stem_wgrad_kernel   dW[n][c][ky][kx] = sum_{b, y, x} g[b][y][x][n] x[b][c][y + ky - 1][x + kx - 1]
// The weight gradients write one partial per workgroup (a 64 x 16-pixel band of one image) and
// small_reduce_kernel adds the partials in a fixed two-level order: deterministic run to run.
// Every product is an fp32 FMA (at least the reference's precision).
#include "wc_common.hpp"

namespace {

constexpr int ST = 16;          // pixel tile edge
constexpr int HT = ST + 2;      // halo edge
constexpr int BAND = 4;         // 16-row tiles per weight-gradient workgroup (a 64 x 16 band)
constexpr int RED_CHUNK = 64;   // partials per first-level reduce group

typedef float f32x2v __attribute__((ext_vector_type(2)));

WC_DEVICE float silu_head(float y) { return y * __builtin_amdgcn_rcpf(1.0f + __expf(-y)); }

// ---- head data gradient: thread = (channel quad cq, tile row pr), sweeping the tile row's 16 pixels;
// the g halo of the 16 x 16 tile in LDS (read as broadcasts), the thread's weights [n][tap] x 4 channels
// in registers (wp is [NO][9][C]); the 16 quads of one pixel store 256 contiguous bytes
template <int NO>
__global__ __launch_bounds__(256) void head_dgrad_kernel(const float* __restrict__ g, const float* __restrict__ wp, int C,
                                                         int H, int W, float* __restrict__ dz, int ldz, int tiles_x,
                                                         int tiles_y) {
    __shared__ float gs[NO][HT][HT];
    const int tile = blockIdx.x;
    const int tx = tile % tiles_x, ty = (tile / tiles_x) % tiles_y, b = tile / (tiles_x * tiles_y);
    const int x0 = tx * ST, y0 = ty * ST;
    for (int i = threadIdx.x; i < NO * HT * HT; i += 256) {
        const int n = i / (HT * HT), r = (i / HT) % HT, col = i % HT;
        const int gy = y0 - 1 + r, gx = x0 - 1 + col;
        gs[n][r][col] = ((unsigned)gy < (unsigned)H && (unsigned)gx < (unsigned)W)
                            ? g[(((long)b * NO + n) * H + gy) * W + gx] : 0.f;
    }
    const int cq = threadIdx.x & 15, pr = threadIdx.x >> 4;
    const int c = blockIdx.y * 64 + 4 * cq;
    const bool cok = c < C;
    f32x4 wv[NO][9];
#pragma unroll
    for (int n = 0; n < NO; ++n)
#pragma unroll
        for (int t = 0; t < 9; ++t)
            wv[n][t] = cok ? *reinterpret_cast<const f32x4*>(wp + ((long)n * 9 + t) * C + c) : f32x4{0.f, 0.f, 0.f, 0.f};
    __syncthreads();
    const int y = y0 + pr;
    if (!cok || y >= H) return;
    float* orow = dz + ((long)b * H + y) * W * ldz + c;
    for (int x = 0; x < ST; ++x) {
        f32x2v a01 = {0.f, 0.f}, a23 = {0.f, 0.f};
#pragma unroll
        for (int n = 0; n < NO; ++n)
#pragma unroll
            for (int ky = 0; ky < 3; ++ky)
#pragma unroll
                for (int kx = 0; kx < 3; ++kx) {
                    const float v = gs[n][pr + 2 - ky][x + 2 - kx];
                    const f32x4 w4 = wv[n][ky * 3 + kx];
                    a01 = __builtin_elementwise_fma(f32x2v{v, v}, f32x2v{w4.x, w4.y}, a01);
                    a23 = __builtin_elementwise_fma(f32x2v{v, v}, f32x2v{w4.z, w4.w}, a23);
                }
        if (x0 + x < W) *reinterpret_cast<f32x4*>(orow + (long)(x0 + x) * ldz) = f32x4{a01.x, a01.y, a23.x, a23.y};
    }
}

// ---- head weight gradient: workgroup = a band of BAND 16 x 16 tiles (one image, 16 columns), thread =
// (channel cl of a 16-channel chunk, tile row r); per tile the g tile (NO x 16 x 16) and, per chunk, the
// act halo [18 rows][18 px][16 ch] (row stride 304 floats: the 4 tile rows of a wave land in 4 disjoint
// 16-bank groups) in LDS; acc[chunk][n][tap] in registers for the whole band, then per chunk a fixed-order
// sum over the 16 rows through LDS into the workgroup's partial [NO][C][9]
constexpr int AROW = HT * 16 + 16;

template <int NO, int NCH>
__global__ __launch_bounds__(256) void head_wgrad_kernel(const float* __restrict__ x, int ldx,
                                                         const float* __restrict__ scale,
                                                         const float* __restrict__ shift, const float* __restrict__ g,
                                                         int H, int W, float* __restrict__ part, int tiles_x,
                                                         int bands_y) {
    constexpr int C = 16 * NCH;
    constexpr int L = NO * C * 9;
    __shared__ float gs[NO][ST][ST];
    __shared__ __attribute__((aligned(16))) float buf[ST * 16 * 27 > HT * AROW ? ST * 16 * 27 : HT * AROW];
    const int wg = blockIdx.x;
    const int tx = wg % tiles_x, by = (wg / tiles_x) % bands_y, b = wg / (tiles_x * bands_y);
    const int x0 = tx * ST;
    const int cl = threadIdx.x & 15, r = threadIdx.x >> 4;
    float acc[NCH][NO][9];
#pragma unroll
    for (int ch = 0; ch < NCH; ++ch)
#pragma unroll
        for (int n = 0; n < NO; ++n)
#pragma unroll
            for (int t = 0; t < 9; ++t) acc[ch][n][t] = 0.f;
    for (int tb = 0; tb < BAND; ++tb) {
        const int y0 = (by * BAND + tb) * ST;
        if (y0 >= H) break;
        __syncthreads();  // the previous tile's reads of gs / buf are done
        for (int i = threadIdx.x; i < NO * ST * ST; i += 256) {
            const int n = i / (ST * ST), yy = (i / ST) % ST, xx = i % ST;
            const int gy = y0 + yy, gx = x0 + xx;
            gs[n][yy][xx] = (gy < H && gx < W) ? g[(((long)b * NO + n) * H + gy) * W + gx] : 0.f;
        }
#pragma unroll
        for (int ch = 0; ch < NCH; ++ch) {
            if (ch) __syncthreads();  // the previous chunk's reads of buf are done
            // halo item i = (pixel i / 4, channel quad i % 4): GN affine + SiLU, zero outside the image
            for (int i = threadIdx.x; i < HT * HT * 4; i += 256) {
                const int q = i & 3, hp = i >> 2, hx = hp % HT, hy = hp / HT;
                const int gy = y0 - 1 + hy, gx = x0 - 1 + hx;
                f32x4 v = {0.f, 0.f, 0.f, 0.f};
                if ((unsigned)gy < (unsigned)H && (unsigned)gx < (unsigned)W) {
                    const int c = ch * 16 + 4 * q;
                    const f32x4 a = *reinterpret_cast<const f32x4*>(x + (((long)b * H + gy) * W + gx) * ldx + c);
                    const f32x4 sc = *reinterpret_cast<const f32x4*>(scale + (long)b * C + c);
                    const f32x4 sh = *reinterpret_cast<const f32x4*>(shift + (long)b * C + c);
#pragma unroll
                    for (int e = 0; e < 4; ++e) v[e] = silu_head(fmaf(a[e], sc[e], sh[e]));
                }
                *reinterpret_cast<f32x4*>(buf + hy * AROW + hx * 16 + 4 * q) = v;
            }
            __syncthreads();
            if (y0 + r < H) {
                for (int xx = 0; xx < ST; ++xx) {
                    float gv[NO];
#pragma unroll
                    for (int n = 0; n < NO; ++n) gv[n] = gs[n][r][xx];
#pragma unroll
                    for (int ky = 0; ky < 3; ++ky)
#pragma unroll
                        for (int kx = 0; kx < 3; ++kx) {
                            const float a = buf[(r + ky) * AROW + (xx + kx) * 16 + cl];
#pragma unroll
                            for (int n = 0; n < NO; ++n) acc[ch][n][ky * 3 + kx] = fmaf(gv[n], a, acc[ch][n][ky * 3 + kx]);
                        }
                }
            }
        }
    }
    // per chunk: the 16 rows' sums of each (channel, n, tap), rows added in order 0..15
    float* dst = part + (long)wg * L;
#pragma unroll
    for (int ch = 0; ch < NCH; ++ch) {
        __syncthreads();
#pragma unroll
        for (int n = 0; n < NO; ++n)
#pragma unroll
            for (int t = 0; t < 9; ++t) buf[(r * 16 + cl) * 27 + n * 9 + t] = acc[ch][n][t];
        __syncthreads();
        for (int o = threadIdx.x; o < 16 * NO * 9; o += 256) {
            const int c = o / (NO * 9), nt = o % (NO * 9), n = nt / 9, t = nt % 9;
            float s = 0.f;
            for (int rr = 0; rr < ST; ++rr) s += buf[(rr * 16 + c) * 27 + nt];
            dst[((long)n * C + ch * 16 + c) * 9 + t] = s;
        }
    }
}

// ---- stem weight gradient: the same band / thread layout with the roles swapped: thread = (output
// channel nl of a 16-channel chunk, tile row r); the NCHW input halo (CI x 18 x 18, all channels) in LDS
// once per tile, the g tile [16 rows][16 px][16 ch] (row stride 272 floats) per chunk
constexpr int GROW = ST * 16 + 16;

template <int CI, int NCH>
__global__ __launch_bounds__(256) void stem_wgrad_kernel(const float* __restrict__ xin, const float* __restrict__ g,
                                                         int ldg, int H, int W, float* __restrict__ part, int tiles_x,
                                                         int bands_y) {
    constexpr int N = 16 * NCH;
    constexpr int L = N * CI * 9;
    __shared__ float xs[CI][HT][HT];
    __shared__ __attribute__((aligned(16))) float buf[ST * 16 * CI * 9 > ST * GROW ? ST * 16 * CI * 9 : ST * GROW];
    const int wg = blockIdx.x;
    const int tx = wg % tiles_x, by = (wg / tiles_x) % bands_y, b = wg / (tiles_x * bands_y);
    const int x0 = tx * ST;
    const int nl = threadIdx.x & 15, r = threadIdx.x >> 4;
    float acc[NCH][CI][9];
#pragma unroll
    for (int ch = 0; ch < NCH; ++ch)
#pragma unroll
        for (int c = 0; c < CI; ++c)
#pragma unroll
            for (int t = 0; t < 9; ++t) acc[ch][c][t] = 0.f;
    for (int tb = 0; tb < BAND; ++tb) {
        const int y0 = (by * BAND + tb) * ST;
        if (y0 >= H) break;
        __syncthreads();
        for (int i = threadIdx.x; i < CI * HT * HT; i += 256) {
            const int c = i / (HT * HT), hy = (i / HT) % HT, hx = i % HT;
            const int gy = y0 - 1 + hy, gx = x0 - 1 + hx;
            xs[c][hy][hx] = ((unsigned)gy < (unsigned)H && (unsigned)gx < (unsigned)W)
                                ? xin[(((long)b * CI + c) * H + gy) * W + gx] : 0.f;
        }
#pragma unroll
        for (int ch = 0; ch < NCH; ++ch) {
            if (ch) __syncthreads();
            for (int i = threadIdx.x; i < ST * ST * 4; i += 256) {  // (pixel i / 4, quad i % 4)
                const int q = i & 3, p = i >> 2, xx = p % ST, yy = p / ST;
                const int gy = y0 + yy, gx = x0 + xx;
                f32x4 v = {0.f, 0.f, 0.f, 0.f};
                if (gy < H && gx < W)
                    v = *reinterpret_cast<const f32x4*>(g + (((long)b * H + gy) * W + gx) * ldg + ch * 16 + 4 * q);
                *reinterpret_cast<f32x4*>(buf + yy * GROW + xx * 16 + 4 * q) = v;
            }
            __syncthreads();
            if (y0 + r < H) {
                for (int xx = 0; xx < ST; ++xx) {
                    const float gv = buf[r * GROW + xx * 16 + nl];
#pragma unroll
                    for (int c = 0; c < CI; ++c)
#pragma unroll
                        for (int ky = 0; ky < 3; ++ky)
#pragma unroll
                            for (int kx = 0; kx < 3; ++kx)
                                acc[ch][c][ky * 3 + kx] = fmaf(gv, xs[c][r + ky][xx + kx], acc[ch][c][ky * 3 + kx]);
                }
            }
        }
    }
    float* dst = part + (long)wg * L;
#pragma unroll
    for (int ch = 0; ch < NCH; ++ch) {
        __syncthreads();
#pragma unroll
        for (int c = 0; c < CI; ++c)
#pragma unroll
            for (int t = 0; t < 9; ++t) buf[(r * 16 + nl) * (CI * 9) + c * 9 + t] = acc[ch][c][t];
        __syncthreads();
        for (int o = threadIdx.x; o < 16 * CI * 9; o += 256) {
            const int n = o / (CI * 9), ct = o % (CI * 9);
            float s = 0.f;
            for (int rr = 0; rr < ST; ++rr) s += buf[(rr * 16 + n) * (CI * 9) + ct];
            dst[(long)(ch * 16 + n) * (CI * 9) + ct] = s;
        }
    }
}

// ---- fixed-order reduction of the partials: level 1 sums RED_CHUNK consecutive partials per group
// (ascending), level 2 the groups (ascending) into out (written, or added with accumulate)
__global__ __launch_bounds__(256) void small_reduce1_kernel(const float* __restrict__ part, int nparts, int L,
                                                            float* __restrict__ part2) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= L) return;
    const int s0 = blockIdx.y * RED_CHUNK, s1 = min(nparts, s0 + RED_CHUNK);
    float s = 0.f;
    for (int sp = s0; sp < s1; ++sp) s += part[(long)sp * L + i];
    part2[(long)blockIdx.y * L + i] = s;
}

__global__ __launch_bounds__(256) void small_reduce2_kernel(const float* __restrict__ part2, int ngroups, int L,
                                                            float* __restrict__ out, int accumulate) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= L) return;
    float s = 0.f;
    for (int gi = 0; gi < ngroups; ++gi) s += part2[(long)gi * L + i];
    out[i] = accumulate ? out[i] + s : s;
}

int small_reduce(const float* part, int nparts, int L, float* part2, float* out, int accumulate, hipStream_t s) {
    const int ng = (nparts + RED_CHUNK - 1) / RED_CHUNK;
    hipLaunchKernelGGL(small_reduce1_kernel, dim3((L + 255) / 256, ng), dim3(256), 0, s, part, nparts, L, part2);
    WC_CHECK_LAUNCH();
    hipLaunchKernelGGL(small_reduce2_kernel, dim3((L + 255) / 256), dim3(256), 0, s, part2, ng, L, out, accumulate);
    WC_CHECK_LAUNCH();
    return WC_OK;
}

long band_workgroups(int B, int H, int W) { return (long)B * ((H + ST * BAND - 1) / (ST * BAND)) * ((W + ST - 1) / ST); }

}  // namespace

extern "C" int64_t wc_small_wgrad_workspace(int B, int H, int W, int L) {
    if (B <= 0 || H <= 0 || W <= 0 || L <= 0) return -1;
    const long nw = band_workgroups(B, H, W);
    return (int64_t)(nw + (nw + RED_CHUNK - 1) / RED_CHUNK) * L;
}

extern "C" int wc_head_dgrad(const float* g, int B, int NO, int H, int W, const float* w_p, int C, float* dz, int ldz,
                             void* stream) {
    if (!g || !w_p || !dz) return WC_E_ARG;
    if (B <= 0 || H <= 0 || W <= 0 || NO < 1 || NO > 4 || C <= 0 || C % 4 || ldz < C || ldz % 4) return WC_E_SHAPE;
    if (((reinterpret_cast<uintptr_t>(w_p) | reinterpret_cast<uintptr_t>(dz)) & 15) != 0) return WC_E_SHAPE;
    const int tiles_x = (W + ST - 1) / ST, tiles_y = (H + ST - 1) / ST;
    const long n = (long)B * tiles_x * tiles_y;
    if (n >= (1L << 31)) return WC_E_SHAPE;
    const dim3 grid((unsigned)n, (unsigned)((C + 63) / 64));
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    switch (NO) {
        case 1: wc_last_kernel = "head_dgrad_kernel<1>";
            hipLaunchKernelGGL(head_dgrad_kernel<1>, grid, dim3(256), 0, s, g, w_p, C, H, W, dz, ldz, tiles_x, tiles_y); break;
        case 2: wc_last_kernel = "head_dgrad_kernel<2>";
            hipLaunchKernelGGL(head_dgrad_kernel<2>, grid, dim3(256), 0, s, g, w_p, C, H, W, dz, ldz, tiles_x, tiles_y); break;
        case 3: wc_last_kernel = "head_dgrad_kernel<3>";
            hipLaunchKernelGGL(head_dgrad_kernel<3>, grid, dim3(256), 0, s, g, w_p, C, H, W, dz, ldz, tiles_x, tiles_y); break;
        default: wc_last_kernel = "head_dgrad_kernel<4>";
            hipLaunchKernelGGL(head_dgrad_kernel<4>, grid, dim3(256), 0, s, g, w_p, C, H, W, dz, ldz, tiles_x, tiles_y); break;
    }
    WC_CHECK_LAUNCH();
    return WC_OK;
}

extern "C" int wc_head_wgrad(const float* x, int ldx, const float* scale, const float* shift, const float* g, int B,
                             int NO, int H, int W, int C, float* work, int64_t work_floats, float* dw, int accumulate,
                             void* stream) {
    if (!x || !scale || !shift || !g || !work || !dw) return WC_E_ARG;
    if (B <= 0 || H <= 0 || W <= 0 || NO != 3 || (C != 32 && C != 64) || ldx < C || ldx % 4) return WC_E_SHAPE;
    if (((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(scale) | reinterpret_cast<uintptr_t>(shift)) &
         15) != 0)
        return WC_E_SHAPE;
    const int L = NO * C * 9;
    if (work_floats != wc_small_wgrad_workspace(B, H, W, L)) return WC_E_SHAPE;
    const long nw = band_workgroups(B, H, W);
    if (nw >= (1L << 31) || nw * L >= (1L << 40)) return WC_E_SHAPE;
    const int tiles_x = (W + ST - 1) / ST, bands_y = (H + ST * BAND - 1) / (ST * BAND);
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    if (C == 64) {
        hipLaunchKernelGGL((head_wgrad_kernel<3, 4>), dim3((unsigned)nw), dim3(256), 0, s, x, ldx, scale, shift, g, H, W,
                           work, tiles_x, bands_y);
    } else {
        hipLaunchKernelGGL((head_wgrad_kernel<3, 2>), dim3((unsigned)nw), dim3(256), 0, s, x, ldx, scale, shift, g, H, W,
                           work, tiles_x, bands_y);
    }
    WC_CHECK_LAUNCH();
    wc_last_kernel = C == 64 ? "head_wgrad_kernel<3, 4>" : "head_wgrad_kernel<3, 2>";
    return small_reduce(work, (int)nw, L, work + nw * L, dw, accumulate, s);
}

extern "C" int wc_stem_wgrad(const float* x_nchw, int CI, const float* g, int ldg, int B, int H, int W, int N,
                             float* work, int64_t work_floats, float* dw, int accumulate, void* stream) {
    if (!x_nchw || !g || !work || !dw) return WC_E_ARG;
    if (B <= 0 || H <= 0 || W <= 0 || CI != 3 || (N != 32 && N != 64) || ldg < N || ldg % 4) return WC_E_SHAPE;
    if ((reinterpret_cast<uintptr_t>(g) & 15) != 0) return WC_E_SHAPE;
    const int L = N * CI * 9;
    if (work_floats != wc_small_wgrad_workspace(B, H, W, L)) return WC_E_SHAPE;
    const long nw = band_workgroups(B, H, W);
    if (nw >= (1L << 31) || nw * L >= (1L << 40)) return WC_E_SHAPE;
    const int tiles_x = (W + ST - 1) / ST, bands_y = (H + ST * BAND - 1) / (ST * BAND);
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    if (N == 64) {
        hipLaunchKernelGGL((stem_wgrad_kernel<3, 4>), dim3((unsigned)nw), dim3(256), 0, s, x_nchw, g, ldg, H, W, work,
                           tiles_x, bands_y);
    } else {
        hipLaunchKernelGGL((stem_wgrad_kernel<3, 2>), dim3((unsigned)nw), dim3(256), 0, s, x_nchw, g, ldg, H, W, work,
                           tiles_x, bands_y);
    }
    WC_CHECK_LAUNCH();
    wc_last_kernel = N == 64 ? "stem_wgrad_kernel<3, 4>" : "stem_wgrad_kernel<3, 2>";
    return small_reduce(work, (int)nw, L, work + nw * L, dw, accumulate, s);
}
