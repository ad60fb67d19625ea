// GroupNorm statistics for NHWC fp32 views (reference: nn.GroupNorm(8, C), unet_base.py:90 etc.).
//
// Pass 1 (wc_gn_stats): grid = B * splits workgroups, each streaming whole pixel rows (all C
// channels, float4 loads: full cache lines, ~HBM rate) of one pixel range of one image.  Thread t
// keeps one fixed 4-channel slice (so one group) and accumulates shifted sums around its own first
// element (pivot), which keeps the moments free of E[x^2]-E[x]^2 cancellation; the workgroup then
// merges the (n, mean, M2) of each group's threads with Chan's formula in a fixed order.
// HBM-bound: 4 B/element.  (Channel counts with C/4 > 256 use a per-group fallback kernel.)
// Pass 2 (wc_gn_finalize): one workgroup per batch element merges the split partials (again
// Chan, fixed order => deterministic) and emits the per-(b, c) affine
//   scale = gamma * rstd,   shift = beta - mean * rstd * gamma,
// consumed by the conv prologue (GroupNorm-apply + SiLU fused into the next conv's loads).
#include "wc_common.hpp"

namespace {

constexpr int GN_THREADS = 256;

// Splits per image depend on the image only (not on B), so the partials of one image merge in the
// same order whatever batch it runs in: a batch-sharded run is bit-identical to a single-rank run.
// The counts are what the former "~2048 workgroups" rule gave at the benched B=16.
int splits_for(int /*B*/, int HW, int C) {
    if (C / 4 > GN_THREADS) {  // fallback kernel: B * splits * G workgroups
        const int max_by_hw = HW / 64 < 1 ? 1 : HW / 64;
        return max_by_hw > 16 ? 16 : max_by_hw;
    }
    const int max_by_hw = HW / 16 < 1 ? 1 : HW / 16;  // whole pixel rows per workgroup
    return max_by_hw > 128 ? 128 : max_by_hw;
}

// Whole-row kernel: thread t handles channel quad q = t % Q of pixels p_begin + t / Q + k * R.
__global__ __launch_bounds__(GN_THREADS) void gn_stats_rows_kernel(const float* __restrict__ x, int HW,
                                                                   int C, int ldc, int G, int splits,
                                                                   float* __restrict__ partials) {
    const int split = blockIdx.x % splits;
    const int b = blockIdx.x / splits;
    const int Q = C / 4;
    const int R = GN_THREADS / Q;  // pixel rows per iteration (threads >= R*Q idle)
    const int cpg = C / G;
    const int q = threadIdx.x % Q;
    const int r = threadIdx.x / Q;
    const int pps = (HW + splits - 1) / splits;
    const int p_begin = split * pps;
    const int p_end = min(HW, p_begin + pps);
    float n = 0.f, s = 0.f, ss = 0.f, pivot = 0.f;
    if (r < R) {
        const float* base = x + (long)b * HW * ldc + q * 4;
        bool have = false;
        for (int p = p_begin + r; p < p_end; p += R) {
            const f32x4 v = *reinterpret_cast<const f32x4*>(base + (long)p * ldc);
            if (!have) { pivot = v.x; have = true; }
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const float d = v[i] - pivot;
                s += d;
                ss = fmaf(d, d, ss);
            }
            n += 4.f;
        }
    }
    __shared__ float sn[GN_THREADS], sm[GN_THREADS], sq[GN_THREADS];
    sn[threadIdx.x] = n;
    sm[threadIdx.x] = n > 0.f ? pivot + s / n : 0.f;
    sq[threadIdx.x] = n > 0.f ? fmaxf(ss - s * (s / n), 0.f) : 0.f;
    __syncthreads();
    if (threadIdx.x < G) {  // group g: quads [g*cpg/4, (g+1)*cpg/4) of every row, fixed order
        const int g = threadIdx.x;
        float N0 = 0.f, M0 = 0.f, Q0 = 0.f;
        for (int rr = 0; rr < R; ++rr)
            for (int qq = g * (cpg / 4); qq < (g + 1) * (cpg / 4); ++qq) {
                const int t = rr * Q + qq;
                chan_merge(N0, M0, Q0, sn[t], sm[t], sq[t]);
            }
        float* o = partials + (((long)b * splits + split) * G + g) * 2;
        o[0] = M0;
        o[1] = Q0;
    }
}

__global__ __launch_bounds__(GN_THREADS) void gn_stats_kernel(const float* __restrict__ x, int HW,
                                                              int C, int ldc, int G, int splits,
                                                              float* __restrict__ partials) {
    const int g = blockIdx.x % G;
    const int split = (blockIdx.x / G) % splits;
    const int b = blockIdx.x / (G * splits);
    const int cpg = C / G;
    const int q_per_pix = cpg / 4;  // float4 per pixel within the group
    const int pps = (HW + splits - 1) / splits;
    const int p_begin = split * pps;
    const int p_end = min(HW, p_begin + pps);
    const long total = (long)max(0, p_end - p_begin) * q_per_pix;

    const float* base = x + ((long)b * HW + p_begin) * ldc + g * cpg;
    float n = 0.f, s = 0.f, ss = 0.f, pivot = 0.f;
    bool have = false;
    for (long idx = threadIdx.x; idx < total; idx += GN_THREADS) {
        long pix = idx / q_per_pix;
        int q = (int)(idx - pix * q_per_pix);
        f32x4 v = *reinterpret_cast<const f32x4*>(base + pix * ldc + q * 4);
        if (!have) { pivot = v.x; have = true; }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            float d = v[i] - pivot;
            s += d;
            ss = fmaf(d, d, ss);
        }
        n += 4.f;
    }
    float mean = 0.f, m2 = 0.f;
    if (n > 0.f) {
        mean = pivot + s / n;
        m2 = fmaxf(ss - s * (s / n), 0.f);
    }
    // wave merge
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        float nb = __shfl_xor(n, o, 64), mb = __shfl_xor(mean, o, 64), m2b = __shfl_xor(m2, o, 64);
        chan_merge(n, mean, m2, nb, mb, m2b);
    }
    __shared__ float red[3][GN_THREADS / 64];
    const int wave = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) { red[0][wave] = n; red[1][wave] = mean; red[2][wave] = m2; }
    __syncthreads();
    if (threadIdx.x == 0) {
        float N0 = red[0][0], M0 = red[1][0], Q0 = red[2][0];
        for (int w = 1; w < GN_THREADS / 64; ++w) chan_merge(N0, M0, Q0, red[0][w], red[1][w], red[2][w]);
        float* o = partials + (((long)b * splits + split) * G + g) * 2;
        o[0] = M0;
        o[1] = Q0;
    }
}

__global__ __launch_bounds__(GN_THREADS) void gn_finalize_kernel(
    const float* __restrict__ partials, int HW, int C, int G, int splits,
    const float* __restrict__ gamma, const float* __restrict__ beta, float eps,
    float* __restrict__ scale, float* __restrict__ shift, float* __restrict__ bound) {
    const int b = blockIdx.x;
    const int cpg = C / G;
    const int pps = (HW + splits - 1) / splits;
    __shared__ float s_mean[32], s_rstd[32], s_bound[32];
    // 32 lanes per group: lane j merges splits j, j+32, ... then a 32-lane butterfly.
    const int g = threadIdx.x / 32;
    const int j = threadIdx.x % 32;
    if (g < G) {
        float n = 0.f, mean = 0.f, m2 = 0.f;
        for (int sp = j; sp < splits; sp += 32) {
            int pb = sp * pps;
            int pe = min(HW, pb + pps);
            float cnt = (float)max(0, pe - pb) * (float)cpg;
            const float* pp = partials + (((long)b * splits + sp) * G + g) * 2;
            chan_merge(n, mean, m2, cnt, pp[0], pp[1]);
        }
#pragma unroll
        for (int o = 16; o > 0; o >>= 1) {
            float nb = __shfl_xor(n, o, 32), mb = __shfl_xor(mean, o, 32), m2b = __shfl_xor(m2, o, 32);
            chan_merge(n, mean, m2, nb, mb, m2b);
        }
        if (j == 0) {
            float var = n > 0.f ? m2 / n : 0.f;  // biased, as torch
            s_mean[g] = mean;
            s_rstd[g] = 1.0f / sqrtf(fmaxf(var, 0.f) + eps);
            // Samuelson: every element of the group lies within sqrt(n - 1) population standard
            // deviations of the mean; 1e-3 relative slack covers the fp32 moments' rounding.
            s_bound[g] = (fabsf(mean) + sqrtf(fmaxf(n - 1.f, 0.f)) * sqrtf(fmaxf(var, 0.f))) * 1.001f;
        }
    }
    __syncthreads();
    if (bound && threadIdx.x == 0) {
        float m = 0.f;
        for (int gg = 0; gg < G; ++gg) m = fmaxf(m, s_bound[gg]);
        bound[b] = m;
    }
    for (int c = threadIdx.x; c < C; c += GN_THREADS) {
        int gg = c / cpg;
        float r = s_rstd[gg];
        float ga = gamma ? gamma[c] : 1.f;
        float be = beta ? beta[c] : 0.f;
        float sc = r * ga;
        scale[(long)b * C + c] = sc;
        shift[(long)b * C + c] = be - s_mean[gg] * sc;
    }
}

// ---- tile partials (the format the split-precision conv epilogues emit, wcx6::gn_tile_partials) ----
// part[((b * np64 + p) * ncb + cb) * (32 / sw) + sub] = (mean, M2) over pixel block p (64 pixels) x
// the sw channels of sub-slot sub of 32-channel block cb.  One wave per (b, p, cb): lane = channel
// quad (0..7) + 8 * pixel row (0..7), 8 pixel rows per pass, two passes over the registers.
__global__ __launch_bounds__(256) void gn_partials_kernel(const float* __restrict__ x, int ldx, int HW, int ncbv,
                                                          int np64, float* __restrict__ part, int ncb, int sw,
                                                          int cb_off, long nwaves) {
    const long wv = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (wv >= nwaves) return;
    const int lane = threadIdx.x & 63;
    const int cbl = (int)(wv % ncbv);
    const long bp = wv / ncbv;  // b * np64 + p
    const int p = (int)(bp % np64);
    const long b = bp / np64;
    const int q = lane & 7, row = lane >> 3;
    const float* base = x + (b * HW + (long)p * 64 + row) * ldx + cbl * 32 + 4 * q;
    f32x4 v[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = *reinterpret_cast<const f32x4*>(base + (long)i * 8 * ldx);
    const int qw = sw / 4;  // quads per sub-slot
    float sum = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i) sum += (v[i].x + v[i].y) + (v[i].z + v[i].w);
    for (int o = 1; o < qw; o <<= 1) sum += __shfl_xor(sum, o, 64);
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
    for (int o = 1; o < qw; o <<= 1) m2 += __shfl_xor(m2, o, 64);
    m2 += __shfl_xor(m2, 8, 64);
    m2 += __shfl_xor(m2, 16, 64);
    m2 += __shfl_xor(m2, 32, 64);
    if (row == 0 && (q % qw) == 0) {
        float* o = part + ((bp * ncb + cb_off + cbl) * (32 / sw) + q / qw) * 2;
        o[0] = mean;
        o[1] = m2;
    }
}

// Per (b, group) merge of the tile partials of the view's channels [c0, c0 + C): one wave per group
// (workgroup = image).  Every partial covers the same n0 = 64*sw values, so the merge is the exact
// equal-count identity  mean = avg(m_i),  M2 = sum(M2_i) + n0 * sum((m_i - mean)^2): up to
// 64 * GNF_KC partials per group in one round of loads kept in registers for both passes (the launch is
// latency-bound: 57 per sampling step), larger groups in two streaming passes; lane butterflies in a
// fixed order (deterministic, per image); then the same per-(b, c) affine (and optional bound) as
// gn_finalize.
constexpr int GNF_THREADS = 512;
constexpr int GNF_KC = 32;  // register-cached partials per lane (groups of up to 2048 items)

// KC: rounds of 64 partials per group kept in registers (the power of two >= items / 64, chosen on the
// host), 0 = the streaming form for larger groups
template <int KC>
__global__ __launch_bounds__(GNF_THREADS) void gn_finalize_part_kernel(
    const float* __restrict__ part, int np64, int ncb, int sw, int c0, int C, int G,
    const float* __restrict__ gamma, const float* __restrict__ beta, float eps, float* __restrict__ scale,
    float* __restrict__ shift, float* __restrict__ bound) {
    const int b = blockIdx.x;
    const int cpg = C / G;
    const int spg = cpg / sw;  // sub-slots per group
    const int spb = 32 / sw;   // sub-slots per 32-channel block
    __shared__ float s_mean[8], s_rstd[8], s_bound[8];
    const int g = threadIdx.x >> 6;
    const int j = threadIdx.x & 63;
    const float n0 = 64.0f * (float)sw;
    if (g < G) {
        const int NS = ncb * spb;
        const int items = np64 * spg;
        float mean, q;
        if constexpr (KC > 0) {
            // the group's (slot, pixel block) partials flattened, item i = j + 64 k -> slot i / np64,
            // block i % np64: every load of the lane issued at once (no dependent rounds), and the
            // values kept in registers for the M2 pass
            const float* gbase = part + ((long)b * np64 * NS + (c0 + g * cpg) / sw) * 2;
            float mk[KC > 0 ? KC : 1], qk[KC > 0 ? KC : 1];
            // (slot, block) of item j + 64 k stepped without division: 64 = ds * np64 + dr, dr < np64
            const int ds = 64 / np64, dr = 64 - ds * np64;
            int sl = j / np64, pp = j - sl * np64;
#pragma unroll
            for (int k = 0; k < KC; ++k) {
                // KC = the rounds the group's items need (host); in the last one, lanes past the end
                // load the group's first partial and contribute 0 (no branch)
                const bool ok = j + 64 * k < items;
                const float2 v = *reinterpret_cast<const float2*>(gbase + (ok ? 2 * sl + 2 * NS * pp : 0));
                mk[k] = ok ? v.x : 0.f;
                qk[k] = ok ? v.y : 0.f;
                pp += dr;
                const int wrap = pp >= np64;
                pp -= wrap ? np64 : 0;
                sl += ds + wrap;
            }
            float sm = 0.f;
#pragma unroll
            for (int k = 0; k < KC; ++k) sm += mk[k];
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) sm += __shfl_xor(sm, o, 64);
            mean = sm / (float)items;
            q = 0.f;
#pragma unroll
            for (int k = 0; k < KC; ++k) {
                if (j + 64 * k < items) {
                    const float d = mk[k] - mean;
                    q += fmaf(n0 * d, d, qk[k]);
                }
            }
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) q += __shfl_xor(q, o, 64);
        } else {
            // sub-slot (pixel block pp, global slot gs) sits at ((b * np64 + pp) * NS + gs) * 2, and a
            // group's spg slots are contiguous: stream each slot's np64 partials with a fixed lane
            // stride, four loads in flight per lane, no index division
            const long pstride = 2L * NS * 64;  // one lane step (64 pixel blocks)
            const float* base = part + ((long)b * np64 * NS + (c0 + g * cpg) / sw) * 2 + (long)j * NS * 2;
            float sm = 0.f;
            for (int s = 0; s < spg; ++s) {
                const float* ps = base + 2 * s;
                float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
                int pp = j;
                for (; pp + 192 < np64; pp += 256, ps += 4 * pstride) {
                    a0 += ps[0];
                    a1 += ps[pstride];
                    a2 += ps[2 * pstride];
                    a3 += ps[3 * pstride];
                }
                for (; pp < np64; pp += 64, ps += pstride) a0 += ps[0];
                sm += (a0 + a1) + (a2 + a3);
            }
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) sm += __shfl_xor(sm, o, 64);
            mean = sm / (float)items;
            q = 0.f;
            for (int s = 0; s < spg; ++s) {
                const float* ps = base + 2 * s;
                float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
                int pp = j;
                for (; pp + 192 < np64; pp += 256, ps += 4 * pstride) {
                    float d;
                    d = ps[0] - mean;
                    a0 += fmaf(n0 * d, d, ps[1]);
                    d = ps[pstride] - mean;
                    a1 += fmaf(n0 * d, d, ps[pstride + 1]);
                    d = ps[2 * pstride] - mean;
                    a2 += fmaf(n0 * d, d, ps[2 * pstride + 1]);
                    d = ps[3 * pstride] - mean;
                    a3 += fmaf(n0 * d, d, ps[3 * pstride + 1]);
                }
                for (; pp < np64; pp += 64, ps += pstride) {
                    const float d = ps[0] - mean;
                    a0 += fmaf(n0 * d, d, ps[1]);
                }
                q += (a0 + a1) + (a2 + a3);
            }
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) q += __shfl_xor(q, o, 64);
        }
        if (j == 0) {
            const float n = n0 * (float)items;
            const float var = fmaxf(q / n, 0.f);  // biased, as torch
            s_mean[g] = mean;
            s_rstd[g] = 1.0f / sqrtf(var + eps);
            s_bound[g] = (fabsf(mean) + sqrtf(fmaxf(n - 1.f, 0.f)) * sqrtf(var)) * 1.001f;
        }
    }
    __syncthreads();
    if (bound && threadIdx.x == 0) {
        float m = 0.f;
        for (int gg = 0; gg < G; ++gg) m = fmaxf(m, s_bound[gg]);
        bound[b] = m;
    }
    for (int c = threadIdx.x; c < C; c += GNF_THREADS) {
        const int gg = c / cpg;
        const float r = s_rstd[gg];
        const float ga = gamma ? gamma[c] : 1.f;
        const float be = beta ? beta[c] : 0.f;
        const float sc = r * ga;
        scale[(long)b * C + c] = sc;
        shift[(long)b * C + c] = be - s_mean[gg] * sc;
    }
}

}  // namespace

extern "C" int wc_gn_partials(const float* x, int ldx, int B, int HW, int C, float* part, int ncb, int sw, int c0,
                              void* stream) {
    if (!x || !part) return WC_E_ARG;
    if ((sw != 4 && sw != 8 && sw != 16 && sw != 32) || C % 32 || c0 % 32 || c0 < 0 || c0 + C > ncb * 32 ||
        HW % 64 || ldx % 4 || (reinterpret_cast<uintptr_t>(x) & 15) != 0)
        return WC_E_SHAPE;
    const int np64 = HW / 64;
    const long nwaves = (long)B * np64 * (C / 32);
    hipLaunchKernelGGL(gn_partials_kernel, dim3((unsigned)((nwaves + 3) / 4)), dim3(256), 0,
                       reinterpret_cast<hipStream_t>(stream), x, ldx, HW, C / 32, np64, part, ncb, sw, c0 / 32,
                       nwaves);
    WC_CHECK_LAUNCH();
    return WC_OK;
}

extern "C" int wc_gn_finalize_part(const float* part, int B, int HW, int ncb, int sw, int c0, int C, int groups,
                                   const float* gamma, const float* beta, float eps, float* scale, float* shift,
                                   float* bound, void* stream) {
    if (!part || !scale || !shift) return WC_E_ARG;
    if (groups < 1 || groups > 8 || C % groups || (C / groups) % sw || c0 % sw || HW % 64 || c0 + C > ncb * 32 ||
        (sw != 4 && sw != 8 && sw != 16 && sw != 32))
        return WC_E_SHAPE;
    const int items = (HW / 64) * (C / groups / sw), rounds = (items + 63) / 64;
    const int kc = rounds <= 1 ? 1 : rounds <= 2 ? 2 : rounds <= 4 ? 4 : rounds <= 8 ? 8 : rounds <= 16 ? 16
                 : rounds <= GNF_KC ? GNF_KC : 0;
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    const int np64 = HW / 64;
#define WC_GNF(KC)                                                                                              \
    hipLaunchKernelGGL(gn_finalize_part_kernel<KC>, dim3(B), dim3(GNF_THREADS), 0, st, part, np64, ncb, sw, c0, C, \
                       groups, gamma, beta, eps, scale, shift, bound)
    switch (kc) {
        case 1: WC_GNF(1); break;
        case 2: WC_GNF(2); break;
        case 4: WC_GNF(4); break;
        case 8: WC_GNF(8); break;
        case 16: WC_GNF(16); break;
        case GNF_KC: WC_GNF(GNF_KC); break;
        default: WC_GNF(0); break;
    }
#undef WC_GNF
    WC_CHECK_LAUNCH();
    return WC_OK;
}

extern "C" int wc_gn_num_splits(int B, int HW, int C) { return splits_for(B, HW, C); }

extern "C" int wc_gn_stats(const float* x, int B, int HW, int C, int ldc, int groups,
                           float* partials, void* stream) {
    if (!x || !partials) return WC_E_ARG;
    if (groups < 1 || groups > 8 || C % groups != 0 || (C / groups) % 4 != 0 || ldc % 4 != 0)
        return WC_E_SHAPE;
    if ((reinterpret_cast<uintptr_t>(x) & 15) != 0) return WC_E_SHAPE;
    int splits = splits_for(B, HW, C);
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    if (C / 4 <= GN_THREADS) {
        hipLaunchKernelGGL(gn_stats_rows_kernel, dim3(B * splits), dim3(GN_THREADS), 0, st, x, HW, C, ldc,
                           groups, splits, partials);
    } else {
        hipLaunchKernelGGL(gn_stats_kernel, dim3(B * splits * groups), dim3(GN_THREADS), 0, st, x, HW, C,
                           ldc, groups, splits, partials);
    }
    WC_CHECK_LAUNCH();
    return WC_OK;
}

extern "C" int wc_gn_finalize(const float* partials, int B, int HW, int C, int groups,
                              const float* gamma, const float* beta, float eps, float* scale,
                              float* shift, void* stream) {
    if (!partials || !scale || !shift) return WC_E_ARG;
    if (groups < 1 || groups > 8 || C % groups != 0) return WC_E_SHAPE;
    int splits = splits_for(B, HW, C);
    hipLaunchKernelGGL(gn_finalize_kernel, dim3(B), dim3(GN_THREADS), 0,
                       reinterpret_cast<hipStream_t>(stream), partials, HW, C, groups, splits,
                       gamma, beta, eps, scale, shift, nullptr);
    WC_CHECK_LAUNCH();
    return WC_OK;
}

extern "C" int wc_gn_finalize_bound(const float* partials, int B, int HW, int C, int groups,
                                    const float* gamma, const float* beta, float eps, float* scale,
                                    float* shift, float* bound, void* stream) {
    if (!partials || !scale || !shift || !bound) return WC_E_ARG;
    if (groups < 1 || groups > 8 || C % groups != 0) return WC_E_SHAPE;
    int splits = splits_for(B, HW, C);
    hipLaunchKernelGGL(gn_finalize_kernel, dim3(B), dim3(GN_THREADS), 0,
                       reinterpret_cast<hipStream_t>(stream), partials, HW, C, groups, splits,
                       gamma, beta, eps, scale, shift, bound);
    WC_CHECK_LAUNCH();
    return WC_OK;
}
