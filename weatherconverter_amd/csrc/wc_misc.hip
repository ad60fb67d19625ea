// Small kernels of the DDPM hot path: time embedding, stem conv, scheduler step, forward
// noising, counter-based Gaussian noise and the semantic-gradient-guidance update.
#include "wc_common.hpp"

#include <math.h>
#include <stdio.h>

namespace {

// --------------------------------------------------------------------------------------------
// Time embedding (reference get_time_embedding unet_base.py:7-30; t_proj :395-397;
// t_emb_layers :98-100 = SiLU -> Linear).  One launch computes, per timestep row,
//   e = [sin(t/f_k), cos(t/f_k)],  f_k = 10000^(k/(D/2))   (fp32 pow/sin/cos as torch)
//   h = W2 SiLU(W1 e + b1) + b2                              (t_proj)
//   out[p] = proj_w[p] . SiLU(h) + proj_b[p]                 (all ResBlock projections)
// Every workgroup recomputes the 2x D^2 MLP (cheap) and owns 256 projection rows.
// --------------------------------------------------------------------------------------------
constexpr int TE_THREADS = 256;

__global__ __launch_bounds__(TE_THREADS) void temb_kernel(const int64_t* __restrict__ t, int D,
                                                          const float* __restrict__ w1,
                                                          const float* __restrict__ b1,
                                                          const float* __restrict__ w2,
                                                          const float* __restrict__ b2,
                                                          const float* __restrict__ pw,
                                                          const float* __restrict__ pb, int P,
                                                          float* __restrict__ out) {
    __shared__ float e[256], h[256];
    const int row = blockIdx.y;
    const int half = D / 2;
    const float tv = (float)t[row];
    for (int k = threadIdx.x; k < half; k += TE_THREADS) {
        float f = powf(10000.0f, (float)k / (float)half);
        float a = tv / f;
        e[k] = sinf(a);
        e[k + half] = cosf(a);
    }
    __syncthreads();
    for (int j = threadIdx.x; j < D; j += TE_THREADS) {
        float acc = 0.f;
        const float* wr = w1 + (long)j * D;
        for (int k = 0; k < D; ++k) acc = fmaf(wr[k], e[k], acc);
        h[j] = wc_silu(acc + b1[j]);
    }
    __syncthreads();
    for (int j = threadIdx.x; j < D; j += TE_THREADS) {
        float acc = 0.f;
        const float* wr = w2 + (long)j * D;
        for (int k = 0; k < D; ++k) acc = fmaf(wr[k], h[k], acc);
        e[j] = wc_silu(acc + b2[j]);  // SiLU of t_proj output = input of every t_emb_layer
    }
    __syncthreads();
    const int p = blockIdx.x * TE_THREADS + threadIdx.x;
    if (p < P) {
        const float* wr = pw + (long)p * D;
        float acc = 0.f;
        for (int k = 0; k < D; k += 4) {
            f32x4 w = *reinterpret_cast<const f32x4*>(wr + k);
            acc = fmaf(w.x, e[k], acc);
            acc = fmaf(w.y, e[k + 1], acc);
            acc = fmaf(w.z, e[k + 2], acc);
            acc = fmaf(w.w, e[k + 3], acc);
        }
        out[(long)row * P + p] = acc + pb[p];
    }
}

// --------------------------------------------------------------------------------------------
// conv_in: 3x3 pad-1 conv from the NCHW image to an NHWC view (unet_base.py:400,456).  The
// NCHW->NHWC transpose is fused here.
// conv_in_px_kernel<COUT, CIN, GN>: thread = pixel, all COUT outputs in registers; the Cin*9 inputs
// are loaded once per pixel (coalesced across the wave), weights are LDS broadcasts.  The outputs
// leave through a per-wave LDS tile, 32 channels at a time: each store instruction then writes eight
// pixels' 128 contiguous bytes (whole lines; thread-per-pixel 16-byte stores at the skip buffer's
// 512-byte pixel pitch touched a line per lane).  GN: the wave's 64 pixels are one GroupNorm
// 64-pixel block, and its (mean, M2) tile partials are computed from the same LDS tile with
// gn_partials_kernel's lane map and summation order (wc_gn.hip): bit-identical partials without the
// separate pass over the output.
// conv_in_kernel (any Cout % 4): thread = (pixel, 4 output channels).
// Both accumulate bias, then (ci, ky, kx) in order, one fma each (out-of-image taps add 0 * w).
// --------------------------------------------------------------------------------------------
constexpr int CI_TS = 36;  // LDS tile row pitch (floats): 32 channels + 4, conflict-free b128 access
constexpr size_t CI_TILE_BYTES = 4 * 64 * CI_TS * sizeof(float);

template <int COUT, int CIN, bool GN>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(3))) void conv_in_px_kernel(const float* __restrict__ x, int B, int Cin, int H, int W,
                                                         const float* __restrict__ w, const float* __restrict__ bias,
                                                         float* __restrict__ out, int ldo, float* __restrict__ part,
                                                         int ncb, int sw, int cb_off) {
    static_assert(COUT % 32 == 0, "conv_in_px: 32-channel store rounds");
    // GN (wc_conv_in_gn): w is already [Cin*9][COUT]; every weight is wave-uniform, so the taps read them
    // as scalar loads (s_load_dwordx16) straight into SGPR operands of the FMAs: no LDS staging, no LDS
    // broadcast reads.  Else w is the PyTorch [COUT][Cin*9] and is staged transposed into LDS.
    extern __shared__ float ws[];  // (not GN) [Cin*9][COUT]; then 4 wave tiles [64 px][CI_TS]
    const int K = Cin * 9;
    const float* wk = w;
    float* tiles = ws;
    if constexpr (!GN) {
        for (int i = threadIdx.x; i < K * COUT; i += blockDim.x) {
            const int co = i % COUT, k = i / COUT;
            ws[i] = w[(long)co * K + k];
        }
        __syncthreads();
        wk = ws;
        tiles = ws + CIN * 9 * COUT;
    }
    const int lane = threadIdx.x & 63;
    float* tile = tiles + (threadIdx.x >> 6) * 64 * CI_TS;
    const long npix = (long)B * H * W;
    const long pix0 = (long)blockIdx.x * blockDim.x + (threadIdx.x & ~63);  // the wave's first pixel
    // lanes past the end compute a copy of the last pixel (no branch around the loads), never stored
    const long pix = min(pix0 + lane, npix - 1);
    const int xw = (int)(pix % W);
    const int yh = (int)((pix / W) % H);
    const int b = (int)(pix / ((long)W * H));
    float acc[COUT];
#pragma unroll
    for (int c = 0; c < COUT; ++c) acc[c] = bias[c];
    // the pixel's CIN * 9 inputs first, all loads in flight together, then the taps in order
    float xin[CIN * 9];
#pragma unroll
    for (int k = 0; k < CIN * 9; ++k) {
        const int ci = k / 9, t = k % 9;
        const int iy = yh + t / 3 - 1, ix = xw + t % 3 - 1;
        xin[k] = ((unsigned)iy < (unsigned)H && (unsigned)ix < (unsigned)W) ? x[(((long)b * CIN + ci) * H + iy) * W + ix]
                                                                            : 0.f;
    }
#pragma unroll
    for (int k = 0; k < CIN * 9; ++k) {
        const float v = xin[k];
        const f32x4* wr = reinterpret_cast<const f32x4*>(wk + k * COUT);
#pragma unroll
        for (int q = 0; q < COUT / 4; ++q) {
            const f32x4 wv = wr[q];
            acc[4 * q + 0] = fmaf(v, wv.x, acc[4 * q + 0]);
            acc[4 * q + 1] = fmaf(v, wv.y, acc[4 * q + 1]);
            acc[4 * q + 2] = fmaf(v, wv.z, acc[4 * q + 2]);
            acc[4 * q + 3] = fmaf(v, wv.w, acc[4 * q + 3]);
        }
    }
    const int q = lane & 7, row = lane >> 3;  // (channel quad, pixel row) of the store / GN lane map
    // the GN partials [npix / 64][ncb][32 / sw][2] as a range-checked buffer (GN only)
    const __amdgpu_buffer_rsrc_t srd_part = __builtin_amdgcn_make_buffer_rsrc(
        part, (short)0, GN ? (int)((npix / 64) * ncb * (32 / sw) * 8) : 0, 0x00020000);
    // branch-free stores (a divergent branch around them made the compiler spill the accumulators):
    // a row past the end holds the clamped last pixel's values (lanes past the end computed it), so it
    // is stored to that pixel again, the same bytes
    float* orow[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) orow[i] = out + min(pix0 + row + 8 * i, npix - 1) * ldo + 4 * q;
#pragma unroll
    for (int cb = 0; cb < COUT / 32; ++cb) {
        // the tile is this wave's own: a wave's LDS operations complete in order, so only the compiler
        // has to be kept from moving them across (no workgroup barrier)
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int j = 0; j < 8; ++j)
            *reinterpret_cast<f32x4*>(tile + lane * CI_TS + 4 * j) =
                f32x4{acc[32 * cb + 4 * j], acc[32 * cb + 4 * j + 1], acc[32 * cb + 4 * j + 2], acc[32 * cb + 4 * j + 3]};
        __builtin_amdgcn_wave_barrier();
        f32x4 v[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) v[i] = *reinterpret_cast<const f32x4*>(tile + (row + 8 * i) * CI_TS + 4 * q);
#pragma unroll
        for (int i = 0; i < 8; ++i)
            *reinterpret_cast<f32x4*>(orow[i] + 32 * cb) = v[i];
        if constexpr (GN) {
            // gn_partials_kernel (wc_gn.hip) on this 64-pixel block x 32 channels, same lanes, same order
            const int qw = sw / 4;
            float sum = 0.f;
#pragma unroll
            for (int i = 0; i < 8; ++i) sum += (v[i].x + v[i].y) + (v[i].z + v[i].w);
#pragma unroll
            for (int o = 1; o < 8; o <<= 1) {
                const float t = __shfl_xor(sum, o, 64);
                sum = o < qw ? sum + t : sum;
            }
            sum += __shfl_xor(sum, 8, 64);
            sum += __shfl_xor(sum, 16, 64);
            sum += __shfl_xor(sum, 32, 64);
            const float mean = sum / (64.0f * (float)sw);
            float m2 = 0.f;
#pragma unroll
            for (int i = 0; i < 8; ++i)
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const float d = v[i][e] - mean;
                    m2 = fmaf(d, d, m2);
                }
#pragma unroll
            for (int o = 1; o < 8; o <<= 1) {
                const float t = __shfl_xor(m2, o, 64);
                m2 = o < qw ? m2 + t : m2;
            }
            m2 += __shfl_xor(m2, 8, 64);
            m2 += __shfl_xor(m2, 16, 64);
            m2 += __shfl_xor(m2, 32, 64);
            // after the butterflies every lane of a sub-slot holds its (mean, M2): all of them store it
            // (the same bytes to one address).  A wave that starts past the last pixel (the grid is
            // rounded up to 4 waves) has no partial slot: the stores go through a buffer resource
            // sized to the partials, whose range check drops them (a branch around them, even a
            // wave-uniform one, made the compiler spill: 75 -> 150 us per launch)
            const long bp = pix0 / 64;  // b * np64 + p (HW % 64 == 0)
            const unsigned o = (unsigned)(((bp * ncb + cb_off + cb) * (32 / sw) + q / qw) * 2 * 4);
            __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, mean), srd_part, o, 0, 0);
            __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, m2), srd_part, o + 4u, 0, 0);
        }
    }
}

__global__ __launch_bounds__(256) void conv_in_kernel(const float* __restrict__ x, int B, int Cin,
                                                      int H, int W, const float* __restrict__ w,
                                                      const float* __restrict__ bias, int Cout,
                                                      float* __restrict__ out, int ldo) {
    extern __shared__ float ws[];  // [Cin*9][Cout]
    const int K = Cin * 9;
    for (int i = threadIdx.x; i < K * Cout; i += blockDim.x) {
        int co = i % Cout, k = i / Cout;
        ws[i] = w[(long)co * K + k];
    }
    __syncthreads();
    const int qpp = Cout / 4;
    const long total = (long)B * H * W * qpp;
    for (long idx = (long)blockIdx.x * blockDim.x + threadIdx.x; idx < total;
         idx += (long)gridDim.x * blockDim.x) {
        const int q = (int)(idx % qpp);
        const long pix = idx / qpp;
        const int xw = (int)(pix % W);
        const int yh = (int)((pix / W) % H);
        const int b = (int)(pix / ((long)W * H));
        f32x4 acc = *reinterpret_cast<const f32x4*>(bias + q * 4);
        for (int ci = 0; ci < Cin; ++ci) {
            const float* plane = x + ((long)b * Cin + ci) * H * W;
#pragma unroll
            for (int ky = 0; ky < 3; ++ky) {
                const int iy = yh + ky - 1;
#pragma unroll
                for (int kx = 0; kx < 3; ++kx) {
                    const int ix = xw + kx - 1;
                    const float v = ((unsigned)iy < (unsigned)H && (unsigned)ix < (unsigned)W) ? plane[(long)iy * W + ix] : 0.f;
                    const f32x4 wv = *reinterpret_cast<const f32x4*>(ws + ((ci * 3 + ky) * 3 + kx) * Cout + q * 4);
                    acc.x = fmaf(v, wv.x, acc.x);
                    acc.y = fmaf(v, wv.y, acc.y);
                    acc.z = fmaf(v, wv.z, acc.z);
                    acc.w = fmaf(v, wv.w, acc.w);
                }
            }
        }
        *reinterpret_cast<f32x4*>(out + pix * ldo + q * 4) = acc;
    }
}

// --------------------------------------------------------------------------------------------
// Head: norm_out -> SiLU -> conv_out (unet_base.py:448-449,483-485), 3x3 pad-1 conv from an NHWC
// view with the GroupNorm affine + SiLU applied on load, to NO <= 4 output channels stored NCHW.
// With 3 outputs an MFMA tile wastes 20x its work; this kernel is HBM-bound instead: one 16x16
// pixel tile per workgroup (thread = pixel), 16-channel chunks whose 18x18 halo is transformed
// once into LDS, weights read as wave-uniform scalars.  fp32 FMAs (the reference's precision).
// w layout: [C/16][9 taps][16 ch][4] (outputs padded to 4).
// --------------------------------------------------------------------------------------------
constexpr int HD_T = 16;

// The next chunk's halo (raw values and their GN affine) is loaded into registers while the
// current chunk computes, so the loads' latency is hidden; NOC = 3 skips the padded 4th output.
constexpr int HD_ITEMS = (HD_T + 2) * (HD_T + 2) * 4;
constexpr int HD_PER_T = (HD_ITEMS + 255) / 256;

template <int NOC>
__global__ __launch_bounds__(256) void head_conv_kernel(const float* __restrict__ x, int ldx,
                                                        const float* __restrict__ scale,
                                                        const float* __restrict__ shift, int B, int H, int W,
                                                        int C, const float* __restrict__ w,
                                                        const float* __restrict__ bias, int NO,
                                                        float* __restrict__ out, int tiles_x, int tiles_y) {
    // halo image [channel quad][pixel]: with the lane -> pixel map below every ds_read_b128 lane group
    // ({0-3,12-15,20-27}, {4-11,16-19,28-31}, +32) reads 16 consecutive pixels of one halo row, so all
    // 9 tap offsets are bank-conflict-free (the [pixel][quad] image with thread = row-major pixel was
    // 4-way conflicted: 2.8e7 conflict cycles per step, profiles/r03j_pmc_step.txt)
    __shared__ f32x4 halo[HD_ITEMS];
    constexpr int HPIX = (HD_T + 2) * (HD_T + 2);
    const int tile = blockIdx.x;
    const int tx = tile % tiles_x, ty = (tile / tiles_x) % tiles_y, b = tile / (tiles_x * tiles_y);
    const int x0 = tx * HD_T, y0 = ty * HD_T;
    const int lane = threadIdx.x & 63, l32 = lane & 31;
    const int grp = ((l32 >= 4 && l32 < 12) || (l32 >= 16 && l32 < 20) || l32 >= 28) ? 1 : 0;
    const int px = l32 < 4 ? l32 : l32 < 12 ? l32 - 4 : l32 < 20 ? l32 - 8 : l32 < 28 ? l32 - 12 : l32 - 16;
    const int py = (threadIdx.x >> 6) * 4 + (lane >> 5) * 2 + grp;
    typedef float f32x2v __attribute__((ext_vector_type(2)));
    f32x2v acc01 = {bias[0], NO > 1 ? bias[1] : 0.f};
    float acc2 = NO > 2 ? bias[2] : 0.f, acc3 = (NOC > 3 && NO > 3) ? bias[3] : 0.f;
    // halo item i = threadIdx.x + 256 k: pixel i >> 2, channels 4 (i & 3) ..
    long goff[HD_PER_T];
    unsigned inb = 0, val = 0;
#pragma unroll
    for (int k = 0; k < HD_PER_T; ++k) {
        const int i = threadIdx.x + 256 * k;
        const int hp = i >> 2;
        const int hx = hp % (HD_T + 2), hy = hp / (HD_T + 2);
        const int gy = y0 + hy - 1, gx = x0 + hx - 1;
        const bool ok = i < HD_ITEMS && gy >= 0 && gy < H && gx >= 0 && gx < W;
        val |= (i < HD_ITEMS ? 1u : 0u) << k;
        inb |= (ok ? 1u : 0u) << k;
        goff[k] = ok ? ((long)(b * H + gy) * W + gx) * ldx + 4 * (i & 3) : 0;
    }
    // every item of a thread has the same channel quad (256 items apart): one scale / shift each
    f32x4 ra[HD_PER_T], rs, rh;
    auto load = [&](int c0) {
        const int c = c0 + 4 * (threadIdx.x & 3);
        rs = *reinterpret_cast<const f32x4*>(scale + (long)b * C + c);
        rh = *reinterpret_cast<const f32x4*>(shift + (long)b * C + c);
#pragma unroll
        for (int k = 0; k < HD_PER_T; ++k)
            if ((inb >> k) & 1u) ra[k] = *reinterpret_cast<const f32x4*>(x + goff[k] + c0);
    };
    load(0);
    for (int c0 = 0; c0 < C; c0 += 16) {
        __syncthreads();  // previous chunk's reads done
#pragma unroll
        for (int k = 0; k < HD_PER_T; ++k) {
            if (!((val >> k) & 1u)) continue;
            f32x4 v = {0.f, 0.f, 0.f, 0.f};
            if ((inb >> k) & 1u) {
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    // SiLU with v_rcp_f32 (as the conv prologues' silu_fast) instead of an IEEE division:
                    // the division's ten instructions per value were a quarter of this kernel's VALU
                    const float y = fmaf(ra[k][e], rs[e], rh[e]);
                    v[e] = y * __builtin_amdgcn_rcpf(1.0f + __expf(-y));
                }
            }
            const int i = threadIdx.x + 256 * k;
            halo[(i & 3) * HPIX + (i >> 2)] = v;  // zero padding after the prologue, as the reference pads
        }
        __syncthreads();
        if (c0 + 16 < C) load(c0 + 16);
        const float* wc = w + (long)(c0 / 16) * 9 * 16 * 4;
#pragma unroll
        for (int tap = 0; tap < 9; ++tap) {
            const int hy = py + tap / 3, hx = px + tap % 3;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const f32x4 a = halo[q * HPIX + hy * (HD_T + 2) + hx];
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const f32x4 wv = *reinterpret_cast<const f32x4*>(wc + ((tap * 16) + 4 * q + e) * 4);
                    // outputs 0 and 1 as one packed FMA (v_pk_fma_f32, the same fused products)
                    acc01 = __builtin_elementwise_fma(f32x2v{a[e], a[e]}, f32x2v{wv.x, wv.y}, acc01);
                    acc2 = fmaf(a[e], wv.z, acc2);
                    if constexpr (NOC > 3) acc3 = fmaf(a[e], wv.w, acc3);
                }
            }
        }
    }
    const int gx = x0 + px, gy = y0 + py;
    if (gx < W && gy < H) {
        const long o = ((long)b * NO * H + gy) * W + gx;
        const long ps = (long)H * W;
        out[o] = acc01.x;
        if (NO > 1) out[o + ps] = acc01.y;
        if (NO > 2) out[o + 2 * ps] = acc2;
        if (NOC > 3 && NO > 3) out[o + 3 * ps] = acc3;
    }
}

// --------------------------------------------------------------------------------------------
// Philox4x32-10 (Salmon et al. 2011) + Box-Muller.  Counter = (element/4, global sample, step, 0),
// key = seed.  Independent of batch sharding by construction.
// --------------------------------------------------------------------------------------------
WC_DEVICE uint4 philox4x32_10(uint4 ctr, uint2 key) {
    const uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u;
    const uint32_t W0 = 0x9E3779B9u, W1 = 0xBB67AE85u;
#pragma unroll
    for (int i = 0; i < 10; ++i) {
        uint32_t hi0 = __umulhi(M0, ctr.x), lo0 = M0 * ctr.x;
        uint32_t hi1 = __umulhi(M1, ctr.z), lo1 = M1 * ctr.z;
        ctr = make_uint4(hi1 ^ ctr.y ^ key.x, lo1, hi0 ^ ctr.w ^ key.y, lo0);
        key.x += W0;
        key.y += W1;
    }
    return ctr;
}

WC_DEVICE f32x4 normal4(uint64_t seed, uint32_t e4, uint32_t sample, uint32_t step) {
    uint4 r = philox4x32_10(make_uint4(e4, sample, step, 0u),
                            make_uint2((uint32_t)seed, (uint32_t)(seed >> 32)));
    const float inv = 2.3283064365386963e-10f;  // 2^-32
    float u0 = ((float)r.x + 0.5f) * inv, u1 = ((float)r.y + 0.5f) * inv;
    float u2 = ((float)r.z + 0.5f) * inv, u3 = ((float)r.w + 0.5f) * inv;
    float ra = sqrtf(-2.f * logf(u0)), rb = sqrtf(-2.f * logf(u2));
    float sa, ca, sb, cb;
    sincosf(6.283185307179586f * u1, &sa, &ca);
    sincosf(6.283185307179586f * u3, &sb, &cb);
    return f32x4{ra * ca, ra * sa, rb * cb, rb * sb};
}

// Reverse step (linear_noise_scheduler.py:96-116 / :63-77).  Operation order and rounding follow
// the reference's tensor ops exactly (IEEE division, FP contraction pinned off: sigma*z is rounded
// before the add, as the reference's separate tensor ops), so with identical tables and z the
// result is bitwise equal to the PyTorch CPU path.
__global__ __launch_bounds__(256) void ddpm_step_kernel(const float* __restrict__ x,
                                                        const float* __restrict__ eps,
                                                        const float* __restrict__ z,
                                                        float* __restrict__ xo,
                                                        float* __restrict__ szo, int64_t n4,
                                                        int64_t per4, float beta, float s1m,
                                                        float sqa, float sigma, int mode,
                                                        uint64_t seed, int64_t sample0,
                                                        int64_t step) {
#pragma clang fp contract(off)
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4;
         i += (int64_t)gridDim.x * blockDim.x) {
        f32x4 xv = reinterpret_cast<const f32x4*>(x)[i];
        f32x4 ev = reinterpret_cast<const f32x4*>(eps)[i];
        f32x4 zv = f32x4{0.f, 0.f, 0.f, 0.f};
        if (mode == WC_NOISE_TENSOR) {
            zv = reinterpret_cast<const f32x4*>(z)[i];
        } else if (mode == WC_NOISE_PHILOX) {
            int64_t smp = i / per4;
            zv = normal4(seed, (uint32_t)(i - smp * per4), (uint32_t)(sample0 + smp), (uint32_t)step);
        }
        f32x4 r, sq;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            float m = __fsub_rn(xv[k], __fdiv_rn(__fmul_rn(beta, ev[k]), s1m));
            m = __fdiv_rn(m, sqa);
            float sz = __fmul_rn(sigma, zv[k]);
            asm volatile("" : "+v"(sz));  // sigma*z is rounded before the add (no FMA), as the reference
            if (szo) {
                r[k] = m;
                sq[k] = sz;
            } else {
                r[k] = (mode == WC_NOISE_NONE) ? m : __fadd_rn(m, sz);
            }
        }
        reinterpret_cast<f32x4*>(xo)[i] = r;
        if (szo) reinterpret_cast<f32x4*>(szo)[i] = sq;
    }
}

__global__ __launch_bounds__(256) void add_noise_kernel(const float* __restrict__ x0,
                                                        const float* __restrict__ nz,
                                                        const float* __restrict__ ca,
                                                        const float* __restrict__ cb,
                                                        float* __restrict__ out, int64_t n4,
                                                        int64_t per4) {
#pragma clang fp contract(off)
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4;
         i += (int64_t)gridDim.x * blockDim.x) {
        int64_t smp = i / per4;
        const float a = ca[smp], bb = cb[smp];
        f32x4 xv = reinterpret_cast<const f32x4*>(x0)[i];
        f32x4 nv = reinterpret_cast<const f32x4*>(nz)[i];
        f32x4 r;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            float p0 = __fmul_rn(a, xv[k]), p1 = __fmul_rn(bb, nv[k]);
            asm volatile("" : "+v"(p0), "+v"(p1));  // both products rounded before the add
            r[k] = __fadd_rn(p0, p1);
        }
        reinterpret_cast<f32x4*>(out)[i] = r;
    }
}

__global__ __launch_bounds__(256) void philox_kernel(float* __restrict__ out, int64_t n4,
                                                     int64_t per4, uint64_t seed, int64_t sample0,
                                                     int64_t step) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4;
         i += (int64_t)gridDim.x * blockDim.x) {
        int64_t smp = i / per4;
        reinterpret_cast<f32x4*>(out)[i] =
            normal4(seed, (uint32_t)(i - smp * per4), (uint32_t)(sample0 + smp), (uint32_t)step);
    }
}

// --------------------------------------------------------------------------------------------
// SGG update (sgg/sgg.py:16-22 + seg_model/inference.py:39-43).  One thread per output pixel of
// the S x S latent: 4x4 average pool of the 4S x 4S gradient per channel (fp32, as F.avg_pool2d),
// then the std-weighted L2 magnitude and the mean update in fp64 as the reference's numpy path.
// mode 0: magnitude over channels per sample (reference semantics at batch 1);
// mode 1: reference semantics for batch > 1 (D4): squeeze(0) is a no-op, so the numpy sum runs
//         over the BATCH axis and the magnitude is per channel.
// --------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void sgg_kernel(const float* __restrict__ grad,
                                                  const float* __restrict__ mu,
                                                  const float* __restrict__ sigma,
                                                  float* __restrict__ xt, float* __restrict__ mag,
                                                  int nb, int S, float lam, double s0, double s1,
                                                  double s2, int mode) {
    const int S4 = 4 * S;
    const long total = (long)S * S;
    const double stdv[3] = {s0, s1, s2};
    for (long pix = (long)blockIdx.x * blockDim.x + threadIdx.x; pix < total;
         pix += (long)gridDim.x * blockDim.x) {
        const int y = (int)(pix / S), x = (int)(pix % S);
        if (mode == 0) {
            for (int b = 0; b < nb; ++b) {
                double acc = 0.0;
                for (int c = 0; c < 3; ++c) {
                    const float* g = grad + (((long)b * 3 + c) * S4 + 4 * y) * S4 + 4 * x;
                    float s = 0.f;
                    for (int dy = 0; dy < 4; ++dy)
                        for (int dx = 0; dx < 4; ++dx) s += g[(long)dy * S4 + dx];
                    double v = (double)(s / 16.f) * stdv[c];
                    acc += v * v;
                }
                double m = sqrt(acc);
                if (mag) mag[(long)b * total + pix] = (float)m;
                for (int c = 0; c < 3; ++c) {
                    long o = ((long)b * 3 + c) * total + pix;
                    double sg = (double)__fmul_rn(lam, sigma[o]);
                    xt[o] = (float)(((double)mu[o] + sg * m) + (double)sigma[o]);
                }
            }
        } else {
            for (int c = 0; c < 3; ++c) {
                double acc = 0.0;
                for (int b = 0; b < nb; ++b) {
                    const float* g = grad + (((long)b * 3 + c) * S4 + 4 * y) * S4 + 4 * x;
                    float s = 0.f;
                    for (int dy = 0; dy < 4; ++dy)
                        for (int dx = 0; dx < 4; ++dx) s += g[(long)dy * S4 + dx];
                    double v = (double)(s / 16.f) * stdv[c];
                    acc += v * v;
                }
                double m = sqrt(acc);
                if (mag) mag[(long)c * total + pix] = (float)m;
                for (int b = 0; b < nb; ++b) {
                    long o = ((long)b * 3 + c) * total + pix;
                    double sg = (double)__fmul_rn(lam, sigma[o]);
                    xt[o] = (float)(((double)mu[o] + sg * m) + (double)sigma[o]);
                }
            }
        }
    }
}

int grid_for(int64_t n, int threads) {
    int64_t g = (n + threads - 1) / threads;
    if (g > 8192) g = 8192;
    if (g < 1) g = 1;
    return (int)g;
}

}  // namespace

extern "C" int wc_temb(const int64_t* t, int nt, int D, const float* w1, const float* b1,
                       const float* w2, const float* b2, const float* proj_w,
                       const float* proj_b, int P, float* out, void* stream) {
    if (!t || !w1 || !b1 || !w2 || !b2 || !proj_w || !proj_b || !out) return WC_E_ARG;
    if (D <= 0 || D > 256 || D % 4 != 0 || nt <= 0 || P <= 0) return WC_E_SHAPE;
    dim3 grid((P + TE_THREADS - 1) / TE_THREADS, nt);
    hipLaunchKernelGGL(temb_kernel, grid, dim3(TE_THREADS), 0, reinterpret_cast<hipStream_t>(stream),
                       t, D, w1, b1, w2, b2, proj_w, proj_b, P, out);
    WC_CHECK_LAUNCH();
    return WC_OK;
}

extern "C" int wc_conv_in(const float* x, int B, int Cin, int H, int W, const float* w,
                          const float* b, int Cout, float* out, int ldo, void* stream) {
    if (!x || !w || !b || !out) return WC_E_ARG;
    if (Cin < 1 || Cin > 16 || Cout % 4 != 0 || ldo % 4 != 0) return WC_E_SHAPE;
    size_t lds = (size_t)Cin * 9 * Cout * sizeof(float);
    if (lds > 64 * 1024) return WC_E_SHAPE;
    if (Cout == 64 && Cin == 3 && (reinterpret_cast<uintptr_t>(out) & 15) == 0 &&
        (reinterpret_cast<uintptr_t>(b) & 15) == 0) {
        const long npix = (long)B * H * W;
        wc_last_kernel = "conv_in_px_kernel<64, 3, false>";
        hipLaunchKernelGGL((conv_in_px_kernel<64, 3, false>), dim3((unsigned)((npix + 255) / 256)), dim3(256),
                           lds + CI_TILE_BYTES, reinterpret_cast<hipStream_t>(stream), x, B, Cin, H, W, w, b, out,
                           ldo, nullptr, 0, 0, 0);
        WC_CHECK_LAUNCH();
        return WC_OK;
    }
    long total = (long)B * H * W * (Cout / 4);
    hipLaunchKernelGGL(conv_in_kernel, dim3(grid_for(total, 256)), dim3(256), lds,
                       reinterpret_cast<hipStream_t>(stream), x, B, Cin, H, W, w, b, Cout, out, ldo);
    WC_CHECK_LAUNCH();
    return WC_OK;
}

extern "C" int wc_conv_in_gn(const float* x, int B, int Cin, int H, int W, const float* w, const float* b,
                             int Cout, float* out, int ldo, float* part, int ncb, int sw, int c0, void* stream) {
    if (!x || !w || !b || !out || !part) return WC_E_ARG;
    if (Cin != 3 || Cout != 64 || ldo % 4 != 0 || ldo < Cout || (H * W) % 64 != 0 || c0 % 32 != 0 || c0 < 0 ||
        (reinterpret_cast<uintptr_t>(w) & 15) != 0 ||
        c0 + Cout > ncb * 32 || (sw != 4 && sw != 8 && sw != 16 && sw != 32) ||
        ((reinterpret_cast<uintptr_t>(out) | reinterpret_cast<uintptr_t>(b)) & 15) != 0)
        return WC_E_SHAPE;
    const long npix = (long)B * H * W;
    const size_t lds = CI_TILE_BYTES;
    wc_last_kernel = "conv_in_px_kernel<64, 3, true>";
    hipLaunchKernelGGL((conv_in_px_kernel<64, 3, true>), dim3((unsigned)((npix + 255) / 256)), dim3(256), lds,
                       reinterpret_cast<hipStream_t>(stream), x, B, Cin, H, W, w, b, out, ldo, part, ncb, sw,
                       c0 / 32);
    WC_CHECK_LAUNCH();
    return WC_OK;
}

extern "C" int wc_head_conv(const float* x, int ldx, const float* scale, const float* shift, int B, int H,
                            int W, int C, const float* w, const float* bias, int NO, float* out, void* stream) {
    if (!x || !scale || !shift || !w || !bias || !out) return WC_E_ARG;
    if (NO < 1 || NO > 4 || C < 16 || C % 16 || ldx % 4 || ldx < C) return WC_E_SHAPE;
    if (((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(w) | reinterpret_cast<uintptr_t>(scale) |
          reinterpret_cast<uintptr_t>(shift)) & 15) != 0)
        return WC_E_SHAPE;
    const int tiles_x = (W + HD_T - 1) / HD_T, tiles_y = (H + HD_T - 1) / HD_T;
    const long n = (long)B * tiles_x * tiles_y;
    if (n >= (1L << 31)) return WC_E_SHAPE;
    if (NO == 3) {
        wc_last_kernel = "head_conv_kernel<3>";
        hipLaunchKernelGGL(head_conv_kernel<3>, dim3((unsigned)n), dim3(256), 0, reinterpret_cast<hipStream_t>(stream),
                           x, ldx, scale, shift, B, H, W, C, w, bias, NO, out, tiles_x, tiles_y);
    } else {
        wc_last_kernel = "head_conv_kernel<4>";
        hipLaunchKernelGGL(head_conv_kernel<4>, dim3((unsigned)n), dim3(256), 0, reinterpret_cast<hipStream_t>(stream),
                           x, ldx, scale, shift, B, H, W, C, w, bias, NO, out, tiles_x, tiles_y);
    }
    WC_CHECK_LAUNCH();
    return WC_OK;
}

extern "C" int wc_ddpm_step(const float* x, const float* eps, const float* z, float* x_out,
                            float* sz_out, int64_t B, int64_t per_sample, float beta, float s1m,
                            float sqrt_alpha, float sigma, int noise_mode, uint64_t seed,
                            int64_t sample0, int64_t step, void* stream) {
    if (!x || !eps || !x_out) return WC_E_ARG;
    if (noise_mode < 0 || noise_mode > 2 || (noise_mode == WC_NOISE_TENSOR && !z)) return WC_E_ARG;
    if (per_sample % 4 != 0) return WC_E_SHAPE;
    int64_t n4 = B * per_sample / 4;
    hipLaunchKernelGGL(ddpm_step_kernel, dim3(grid_for(n4, 256)), dim3(256), 0,
                       reinterpret_cast<hipStream_t>(stream), x, eps, z, x_out, sz_out, n4, per_sample / 4,
                       beta, s1m, sqrt_alpha, sigma, noise_mode, seed, sample0, step);
    WC_CHECK_LAUNCH();
    return WC_OK;
}

extern "C" int wc_add_noise(const float* x0, const float* noise, const float* coef_a,
                            const float* coef_b, float* out, int64_t B, int64_t per_sample,
                            void* stream) {
    if (!x0 || !noise || !coef_a || !coef_b || !out) return WC_E_ARG;
    if (per_sample % 4 != 0) return WC_E_SHAPE;
    int64_t n4 = B * per_sample / 4;
    hipLaunchKernelGGL(add_noise_kernel, dim3(grid_for(n4, 256)), dim3(256), 0,
                       reinterpret_cast<hipStream_t>(stream), x0, noise, coef_a, coef_b, out, n4,
                       per_sample / 4);
    WC_CHECK_LAUNCH();
    return WC_OK;
}

extern "C" int wc_philox_normal(float* out, int64_t B, int64_t per_sample, uint64_t seed,
                                int64_t sample0, int64_t step, void* stream) {
    if (!out) return WC_E_ARG;
    if (per_sample % 4 != 0) return WC_E_SHAPE;
    int64_t n4 = B * per_sample / 4;
    hipLaunchKernelGGL(philox_kernel, dim3(grid_for(n4, 256)), dim3(256), 0,
                       reinterpret_cast<hipStream_t>(stream), out, n4, per_sample / 4, seed,
                       sample0, step);
    WC_CHECK_LAUNCH();
    return WC_OK;
}

extern "C" int wc_sgg_update(const float* grad, const float* mu, const float* sigma,
                             float* xt_out, float* mag_out, int nb, int S, float lambda_,
                             double std0, double std1, double std2, int sum_batch, void* stream) {
    if (!grad || !mu || !sigma || !xt_out) return WC_E_ARG;
    if (nb < 1 || S < 1) return WC_E_SHAPE;
    long total = (long)S * S;
    wc_last_kernel = "sgg_kernel";
    hipLaunchKernelGGL(sgg_kernel, dim3(grid_for(total, 256)), dim3(256), 0,
                       reinterpret_cast<hipStream_t>(stream), grad, mu, sigma, xt_out, mag_out, nb,
                       S, lambda_, std0, std1, std2, sum_batch ? 1 : 0);
    WC_CHECK_LAUNCH();
    return WC_OK;
}

// wc_source_hash: defined in the build's generated object (weatherconverter_amd/_build.py source_hash)
extern "C" const char* wc_source_hash(void);
extern "C" const char* wc_version(void) {
    static char v[96] = {0};
    if (!v[0]) snprintf(v, sizeof v, "weatherconverter_amd 0.1 gfx950 src:%s", wc_source_hash());
    return v;
}

// In-graph launch timing: one wave reads the GPU's constant-rate wall clock (wall_clock64, the
// 100 MHz real-time counter) and lane 0 stores it to slots[index] with an ordinary vector store.  Stamp
// launches captured around the named launches of a graph give their durations as the graph runs them.
__global__ __launch_bounds__(64) void stamp_kernel(unsigned long long* __restrict__ slots, int index) {
    const unsigned long long t = wall_clock64();
    if (threadIdx.x == 0) slots[index] = t;
}

extern "C" int wc_stamp(unsigned long long* slots, int index, void* stream) {
    if (!slots || index < 0) return WC_E_ARG;
    hipLaunchKernelGGL(stamp_kernel, dim3(1), dim3(64), 0, reinterpret_cast<hipStream_t>(stream), slots, index);
    WC_CHECK_LAUNCH();
    return WC_OK;
}

extern "C" int wc_wall_clock_khz(int* khz) {
    if (!khz) return WC_E_ARG;
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e == hipSuccess) e = hipDeviceGetAttribute(khz, hipDeviceAttributeWallClockRate, dev);
    return e == hipSuccess ? WC_OK : (int)e;
}

// The instantiation name of the kernel this host thread launched last through a named launcher
// (rocprofv3's demangled form), then cleared: "" when the last entry point did not name its kernel.
extern "C" const char* wc_last_kernel_name(void) {
    const char* n = wc_last_kernel;
    wc_last_kernel = "";
    return n;
}
