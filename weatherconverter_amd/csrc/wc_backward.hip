// Backward-pass kernels of the DDPM UNet training step (reference diffusion_model/train_ddpm.py:106-114:
// loss.backward() through unet_base.Unet, then Adam).  gfx950 / CDNA4, wave64.
//
//  * conv_wgrad_kernel  dW[m][k] = sum over pixels of G[pixel][m] * X_k[pixel], where X_k is the
//    conv's own input as the forward read it: column k = (tap, channel) of segment 0 with the same
//    tap offsets, stride and zero padding, optionally through the forward's GroupNorm(+SiLU)
//    prologue (the activation is recomputed, not stored), then the raw 1x1 residual segment.
//    One GEMM with M = G channels, N = K columns, K = B*Hm*Wm pixels on fp32 MFMA
//    (v_mfma_f32_32x32x2_f32, exact fp32 products): both operands are NHWC pixel rows, which is
//    exactly the [k][m] / [k][n] order the 32x32x2 fragments read (lane = m or n, lane half = k),
//    so the tiles are staged straight from HBM rows into LDS with no transpose.  The pixel
//    reduction is split across workgroups (partials [split][M][K]) and summed in a fixed order
//    by wgrad_reduce_kernel, which also scatters into the parameter's own layout: results are
//    deterministic run to run.
//  * gnb_*  GroupNorm(8)(+SiLU) backward: per-(b, c) sums of dy and dy*xhat over pixel splits,
//    per-image coefficients (dx = a*dy + k0 + k1*xhat), dgamma / dbeta, and the elementwise
//    apply that recomputes xhat and the SiLU derivative from the stored pre-norm input.  The
//    same reduction without a normalised input is the per-(b, c) channel sum (bias / temb grads).
//  * gemm_small / silu / colsum / temb helpers for the time-embedding MLP (B x 128 matrices).
//  * nchw_to_nhwc: the loss gradient (NCHW, the UNet output layout) into a padded NHWC view.
#include <algorithm>

#include "wc_x6.hpp"

namespace {

constexpr unsigned OOB = 0x80000000u;
constexpr int SRD_BYTES = 0x7FFFFFFF;
constexpr int SRD_FLAGS = 0x00020000;

WC_DEVICE __amdgpu_buffer_rsrc_t make_srd(const float* p) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(p), (short)0, SRD_BYTES, SRD_FLAGS);
}
WC_DEVICE f32x4 bload4(__amdgpu_buffer_rsrc_t r, unsigned off) {
    return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0));
}
WC_DEVICE float silu_grad(float y) {  // d/dy [y * sigmoid(y)]
    const float s = 1.0f / (1.0f + __expf(-y));
    return s * (1.0f + y * (1.0f - s));
}

// ============================================================================================
// conv weight gradient
// ============================================================================================
constexpr int WG_THREADS = 256;
constexpr int WG_KP = 32;  // pixels per K-step

struct WgDev {
    const float* g;
    int M, ldg;
    const float* src0;
    int C0, ldc0, H0, W0, sy, sx, ntaps;
    int dy[WC_MAX_TAPS], dx[WC_MAX_TAPS];
    const float* scale;
    const float* shift;
    const float* src1;
    int C1, ldc1, H1, W1;
    int Hm, Wm;
    long P;     // pixels = B*Hm*Wm
    int K0, Kc; // segment-0 columns (ntaps*C0), all columns (+ C1)
    float* part;
    long pps;   // pixels per split (multiple of WG_KP)
    int ntm, ntn;
    // F3: per-image bounds (device [B]) of G, segment 0 and segment 1; xe0 = segment 0's static exponent
    const float* gb;
    const float* xb0;
    const float* xb1;
    int xe0, B;
};

// PRO: 0 raw, 1 GN affine, 2 GN affine + SiLU (segment 0 only, as the forward prologue).
// X6: bf16x6 (both operands split exactly into 3 bf16 pieces; the 6 piece products with i + j <= 2
// on v_mfma_f32_32x32x16_bf16).  The pieces stay in LDS as [pixel][channel] rows — the order they
// arrive in from HBM — and the MFMA fragments, which need 8 consecutive PIXELS per lane, are read
// with ds_read_b64_tr_b16 (gfx950's transposing LDS read: per 16-lane group a 4-row x 16-column
// block delivered column-major).  Row bytes = 2*width + 64 (== 64 mod 256): the four rows of a
// half-wave's read land on disjoint banks.  Else fp32 MFMA 32x32x2 on fp32 rows.
// F3 (with X6): f16x3 instead — G x 2^sg, segment 0 x 2^sx0, segment 1 x 2^sx1 split into two fp16
// pieces (products h*h + h*l + l*h), s = 13 - floor(log2 bound) from the batch max of the per-image
// bounds (segment 0: at most its static exponent xe0); the epilogue removes 2^-(sg + sx) per column.
// Pixels per K-step (per barrier): 16 for the split forms, 32 for fp32 (32 pixels per barrier measured
// slower for the f16x3 tiles, 292 vs 264 us at the 1x1 shapes, and for the single-piece tiles, 392 vs
// 352 us on the GroupNorm-affine 1x1 form: profiles/r06_train_wgrad_ab.txt).
template <bool X6>
constexpr int wg_kp() { return X6 ? 16 : WG_KP; }
// LDS piece planes: the single-piece builds (WC_SINGLE16, one 16-bit piece per operand) stage the high
// piece only (the low piece is zero there and mfma_f16c drops its products)
template <bool X6, bool F3>
constexpr int wg_nps() { return !X6 ? 0 : (F3 && WC_SINGLE16) ? 1 : F3 ? 2 : 3; }

template <int BM, int BN, int PRO, bool X6, bool F3 = false>
__global__ __launch_bounds__(WG_THREADS, 2) void conv_wgrad_kernel(WgDev p) {
    static_assert(!F3 || X6, "F3 runs the X6 structure");
    constexpr int NP = F3 ? 2 : 3;
    constexpr int NPS = wg_nps<X6, F3>();
    constexpr int WAVES_M = BM / 64, WAVES_N = BN / 64;
    static_assert(WAVES_M * WAVES_N == 4, "4 waves of 64x64");
    constexpr int KP = wg_kp<X6>();
    constexpr int AS = BM + 32, BS = BN + 32;  // fp32 LDS row strides: lane halves on disjoint banks
    constexpr int ASB = BM * 2 + 64, BSB = BN * 2 + 64;  // X6 row bytes
    constexpr int APL = KP * ASB, BPL = KP * BSB;        // X6 bytes of one piece plane
    constexpr int A_PER_T = KP * BM / 4 / WG_THREADS;
    constexpr int B_PER_T = KP * BN / 4 / WG_THREADS;
    constexpr int STAGE = X6 ? NPS * (APL + BPL) : KP * (AS + BS) * 4;  // bytes
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;
    const int wm = wave / WAVES_N, wn = wave % WAVES_N;
    const int l32 = lane & 31, half = lane >> 5;

    // XCD-aware bijective order: the ntm x ntn tiles of one pixel split (which all read that split's G
    // and input rows) are consecutive logical blocks and land on one XCD, whose L2 then serves their
    // re-reads (round-robin placement fetched the rows into every XCD's L2, once per tile)
    int t = blockIdx.x;
    {
        const int nblk = gridDim.x, q = nblk / 8, r = nblk % 8, xcd = t % 8;
        t = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + t / 8;
    }
    const int tn = t % p.ntn;
    t /= p.ntn;
    const int tm = t % p.ntm;
    const int sp = t / p.ntm;
    const int m0 = tm * BM, n0 = tn * BN;
    const long pbeg = (long)sp * p.pps;
    long pend = pbeg + p.pps;
    if (pend > p.P) pend = p.P;
    const int nsteps = (int)((pend - pbeg + KP - 1) / KP);
    const int HWm = p.Hm * p.Wm;
    int sg = 0, sx0 = 0, sx1 = 0;
    if constexpr (F3) {
        auto exp_of = [&](const float* bnd, int cap) {
            float m = 0.f;
            for (int b = 0; b < p.B; ++b) m = fmaxf(m, bnd[b]);
            int e = cap;
            if (m > 0.f) e = min(cap, 13 - ((int)((__float_as_uint(m) >> 23) & 0xffu) - 127));
            return max(e, -100);
        };
        sg = exp_of(p.gb, 60);
        sx0 = p.xb0 ? exp_of(p.xb0, p.xe0) : p.xe0;
        sx1 = p.xb1 ? exp_of(p.xb1, 60) : 0;
    }
    const float gsc = ldexpf(1.f, sg), xsc0 = ldexpf(1.f, sx0), xsc1 = ldexpf(1.f, sx1);

    // fixed per-thread column coordinates
    int arow[A_PER_T], acol[A_PER_T];
#pragma unroll
    for (int j = 0; j < A_PER_T; ++j) {
        const int i = tid + WG_THREADS * j;
        arow[j] = i / (BM / 4);
        acol[j] = 4 * (i % (BM / 4));
    }
    int brow[B_PER_T], bcol[B_PER_T], bseg[B_PER_T], bc[B_PER_T], bdy[B_PER_T], bdx[B_PER_T];
#pragma unroll
    for (int j = 0; j < B_PER_T; ++j) {
        const int i = tid + WG_THREADS * j;
        brow[j] = i / (BN / 4);
        bcol[j] = 4 * (i % (BN / 4));
        const int k = n0 + bcol[j];
        if (k < p.K0) {
            const int tp = k / p.C0;
            bseg[j] = 0;
            bc[j] = k - tp * p.C0;
            bdy[j] = p.dy[tp];
            bdx[j] = p.dx[tp];
        } else if (k < p.Kc) {
            bseg[j] = 1;
            bc[j] = k - p.K0;
            bdy[j] = 0;
            bdx[j] = 0;
        } else {
            bseg[j] = 2;  // past the last column
            bc[j] = 0;
            bdy[j] = 0;
            bdx[j] = 0;
        }
    }
    const __amdgpu_buffer_rsrc_t srdg = make_srd(p.g);
    const __amdgpu_buffer_rsrc_t srd0 = make_srd(p.src0);
    const __amdgpu_buffer_rsrc_t srd1 = make_srd(p.src1 ? p.src1 : p.src0);
    const __amdgpu_buffer_rsrc_t srdsc = make_srd(PRO ? p.scale : p.src0);
    const __amdgpu_buffer_rsrc_t srdsh = make_srd(PRO ? p.shift : p.src0);

    f32x4 ra[A_PER_T], rb[B_PER_T];
    // pixel coordinates of each B item, advanced by KP pixels per K-step (no per-step division)
    int bb_[B_PER_T], by_[B_PER_T], bx_[B_PER_T];
#pragma unroll
    for (int j = 0; j < B_PER_T; ++j) {
        const int px = (int)pbeg + brow[j];
        bb_[j] = px / HWm;
        const int r = px - bb_[j] * HWm;
        by_[j] = r / p.Wm;
        bx_[j] = r - by_[j] * p.Wm;
    }
    const int ipend = (int)pend;
    // raw loads of the next K-step are issued before the current step's MFMAs; the GroupNorm(+SiLU)
    // prologue runs after them, in store(), so the loads' latency hides under the MFMAs
    unsigned binb = 0;  // bit j: B item j is a real (in-image) input value
    f32x4 bsc[PRO ? B_PER_T : 1], bsh[PRO ? B_PER_T : 1];
    auto load = [&](int s) {
        const int pb0 = (int)pbeg + s * KP;
#pragma unroll
        for (int j = 0; j < A_PER_T; ++j) {
            const int px = pb0 + arow[j];
            const bool ok = px < ipend && m0 + acol[j] < p.M;
            ra[j] = bload4(srdg, ok ? (unsigned)(px * p.ldg + m0 + acol[j]) * 4u : OOB);
        }
        binb = 0;
#pragma unroll
        for (int j = 0; j < B_PER_T; ++j) {
            const int px = pb0 + brow[j];
            const int b = bb_[j], y = by_[j], x = bx_[j];
            unsigned off = OOB;
            if (px < ipend && bseg[j] < 2) {
                if (bseg[j] == 0) {
                    const int iy = y * p.sy + bdy[j], ix = x * p.sx + bdx[j];
                    if ((unsigned)iy < (unsigned)p.H0 && (unsigned)ix < (unsigned)p.W0) {
                        off = (unsigned)(((b * p.H0 + iy) * p.W0 + ix) * p.ldc0 + bc[j]) * 4u;
                        binb |= 1u << j;
                    }
                } else {
                    off = (unsigned)(((b * p.H1 + y) * p.W1 + x) * p.ldc1 + bc[j]) * 4u;
                }
            }
            // the buffer descriptor must be wave-uniform: one load per segment, the other masked off
            rb[j] = bload4(srd0, bseg[j] == 0 ? off : OOB) + bload4(srd1, bseg[j] == 1 ? off : OOB);
            if constexpr (PRO != 0) {
                const unsigned o = (unsigned)(b * p.C0 + bc[j]) * 4u;
                const bool pro = bseg[j] == 0 && px < ipend;
                bsc[j] = bload4(srdsc, pro ? o : OOB);
                bsh[j] = bload4(srdsh, pro ? o : OOB);
            }
            // advance to the next K-step's pixel
            int nx = x + KP, ny = y, nb = b;
            while (nx >= p.Wm) {
                nx -= p.Wm;
                if (++ny == p.Hm) {
                    ny = 0;
                    ++nb;
                }
            }
            bb_[j] = nb;
            by_[j] = ny;
            bx_[j] = nx;
        }
    };
    auto store = [&](int buf) {
        unsigned char* a = lds + buf * STAGE;
        unsigned char* bb = a + (X6 ? NPS * APL : KP * AS * 4);
#pragma unroll
        for (int j = 0; j < A_PER_T; ++j) {
            if constexpr (F3) {
                wcx6::u32x2 h, l;
                wcx6::split2_f16(ra[j] * gsc, h, l);
                unsigned char* d = a + arow[j] * ASB + acol[j] * 2;
                *reinterpret_cast<wcx6::u32x2*>(d) = h;
                if constexpr (NPS > 1) *reinterpret_cast<wcx6::u32x2*>(d + APL) = l;
            } else if constexpr (X6) {
                wcx6::u32x2 p0, p1, p2;
                wcx6::split3(ra[j], p0, p1, p2);
                unsigned char* d = a + arow[j] * ASB + acol[j] * 2;
                *reinterpret_cast<wcx6::u32x2*>(d) = p0;
                *reinterpret_cast<wcx6::u32x2*>(d + APL) = p1;
                *reinterpret_cast<wcx6::u32x2*>(d + 2 * APL) = p2;
            } else {
                *reinterpret_cast<f32x4*>(a + (arow[j] * AS + acol[j]) * 4) = ra[j];
            }
        }
#pragma unroll
        for (int j = 0; j < B_PER_T; ++j) {
            f32x4 v = rb[j];
            if constexpr (PRO != 0) {
                if (bseg[j] == 0) {
                    v = v * bsc[j] + bsh[j];
                    if constexpr (PRO == 2) {
                        v.x = wc_silu(v.x); v.y = wc_silu(v.y); v.z = wc_silu(v.z); v.w = wc_silu(v.w);
                    }
                    if (!((binb >> j) & 1u)) v = f32x4{0.f, 0.f, 0.f, 0.f};  // padding after the prologue
                }
            }
            if constexpr (F3) {
                wcx6::u32x2 h, l;
                wcx6::split2_f16(v * (bseg[j] == 1 ? xsc1 : xsc0), h, l);
                unsigned char* d = bb + brow[j] * BSB + bcol[j] * 2;
                *reinterpret_cast<wcx6::u32x2*>(d) = h;
                if constexpr (NPS > 1) *reinterpret_cast<wcx6::u32x2*>(d + BPL) = l;
            } else if constexpr (X6) {
                wcx6::u32x2 p0, p1, p2;
                wcx6::split3(v, p0, p1, p2);
                unsigned char* d = bb + brow[j] * BSB + bcol[j] * 2;
                *reinterpret_cast<wcx6::u32x2*>(d) = p0;
                *reinterpret_cast<wcx6::u32x2*>(d + BPL) = p1;
                *reinterpret_cast<wcx6::u32x2*>(d + 2 * BPL) = p2;
            } else {
                *reinterpret_cast<f32x4*>(bb + (brow[j] * BS + bcol[j]) * 4) = v;
            }
        }
    };

    f32x16 acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

    if (nsteps > 0) {
        load(0);
        store(0);
    }
    __syncthreads();
    // X6 fragment addresses: lane = 16 g + 4 q + p supplies row 8 kh + q (kh = g >> 1), columns
    // 16 (g & 1) + 4 p .. + 3 of its 32-column block; it receives column (lane & 31), 4 pixels
    const int tq = (lane & 15) >> 2, tp = lane & 3, tg = lane >> 4;
    const int tr_a = (8 * (tg >> 1) + tq) * ASB + (wm * 64 + 16 * (tg & 1) + 4 * tp) * 2;
    const int tr_b = (8 * (tg >> 1) + tq) * BSB + (wn * 64 + 16 * (tg & 1) + 4 * tp) * 2;
    auto tr_frag = [&](const unsigned char* q0, int rs) {
        typedef short v4s __attribute__((ext_vector_type(4)));
        const v4s lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4s*)(q0));
        const v4s hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4s*)(q0 + 4 * rs));
        const wcx6::u32x2 l2 = __builtin_bit_cast(wcx6::u32x2, lo), h2 = __builtin_bit_cast(wcx6::u32x2, hi);
        return wcx6::u32x4{l2.x, l2.y, h2.x, h2.y};
    };
    for (int s = 0; s < nsteps; ++s) {
        const int buf = s & 1;
        if (s + 1 < nsteps) load(s + 1);
        if constexpr (F3) {
#pragma unroll
            for (int ks = 0; ks < KP / 16; ++ks) {  // 16-pixel MFMA K-steps of the stage
                const unsigned char* a = lds + buf * STAGE + tr_a + ks * 16 * ASB;
                const unsigned char* bb = lds + buf * STAGE + NPS * APL + tr_b + ks * 16 * BSB;
                wcx6::u32x4 fa[2][2], fb[2][2];
#pragma unroll
                for (int pc = 0; pc < 2; ++pc) {
                    if (pc >= NPS) {  // single-piece builds: the low piece is never read (mfma_f16c drops it)
#pragma unroll
                        for (int i = 0; i < 2; ++i) fa[i][pc] = fb[i][pc] = wcx6::u32x4{0u, 0u, 0u, 0u};
                        continue;
                    }
#pragma unroll
                    for (int mb = 0; mb < 2; ++mb) fa[mb][pc] = tr_frag(a + pc * APL + mb * 64, ASB);
#pragma unroll
                    for (int nb = 0; nb < 2; ++nb) fb[nb][pc] = tr_frag(bb + pc * BPL + nb * 64, BSB);
                }
#pragma unroll
                for (int mb = 0; mb < 2; ++mb)
#pragma unroll
                    for (int nb = 0; nb < 2; ++nb) {
                        acc[mb][nb] = wcx6::mfma_f16(fa[mb][0], fb[nb][0], acc[mb][nb]);
                        acc[mb][nb] = wcx6::mfma_f16c(fa[mb][0], fb[nb][1], acc[mb][nb]);
                        acc[mb][nb] = wcx6::mfma_f16c(fa[mb][1], fb[nb][0], acc[mb][nb]);
                    }
            }
        } else if constexpr (X6) {
            const unsigned char* a = lds + buf * STAGE + tr_a;
            const unsigned char* bb = lds + buf * STAGE + 3 * APL + tr_b;
            wcx6::u32x4 fa[2][3], fb[2][3];
#pragma unroll
            for (int pc = 0; pc < 3; ++pc) {
#pragma unroll
                for (int mb = 0; mb < 2; ++mb) fa[mb][pc] = tr_frag(a + pc * APL + mb * 64, ASB);
#pragma unroll
                for (int nb = 0; nb < 2; ++nb) fb[nb][pc] = tr_frag(bb + pc * BPL + nb * 64, BSB);
            }
#pragma unroll
            for (int mb = 0; mb < 2; ++mb)
#pragma unroll
                for (int nb = 0; nb < 2; ++nb) acc[mb][nb] = wcx6::mfma_bf16(fa[mb][0], fb[nb][0], acc[mb][nb]);
#pragma unroll
            for (int mb = 0; mb < 2; ++mb)
#pragma unroll
                for (int nb = 0; nb < 2; ++nb) {
                    acc[mb][nb] = wcx6::mfma_bf16(fa[mb][0], fb[nb][1], acc[mb][nb]);
                    acc[mb][nb] = wcx6::mfma_bf16(fa[mb][1], fb[nb][0], acc[mb][nb]);
                }
#pragma unroll
            for (int mb = 0; mb < 2; ++mb)
#pragma unroll
                for (int nb = 0; nb < 2; ++nb) {
                    acc[mb][nb] = wcx6::mfma_bf16(fa[mb][0], fb[nb][2], acc[mb][nb]);
                    acc[mb][nb] = wcx6::mfma_bf16(fa[mb][1], fb[nb][1], acc[mb][nb]);
                    acc[mb][nb] = wcx6::mfma_bf16(fa[mb][2], fb[nb][0], acc[mb][nb]);
                }
        } else {
            const float* a = reinterpret_cast<const float*>(lds + buf * STAGE) + wm * 64 + l32;
            const float* bb = reinterpret_cast<const float*>(lds + buf * STAGE) + KP * AS + wn * 64 + l32;
#pragma unroll
            for (int kk = 0; kk < KP / 2; ++kk) {
                const int row = 2 * kk + half;
                const float a0 = a[row * AS], a1 = a[row * AS + 32];
                const float b0 = bb[row * BS], b1 = bb[row * BS + 32];
                acc[0][0] = mfma32(a0, b0, acc[0][0]);
                acc[0][1] = mfma32(a0, b1, acc[0][1]);
                acc[1][0] = mfma32(a1, b0, acc[1][0]);
                acc[1][1] = mfma32(a1, b1, acc[1][1]);
            }
        }
        if (s + 1 < nsteps) store(buf ^ 1);
        __syncthreads();
    }

    // partial[sp][m][k]
    float* out = p.part + (long)sp * p.M * p.Kc;
#pragma unroll
    for (int mb = 0; mb < 2; ++mb)
#pragma unroll
        for (int nb = 0; nb < 2; ++nb) {
            const int k = n0 + wn * 64 + nb * 32 + l32;
            const float un = F3 ? ldexpf(1.f, -(sg + (k < p.K0 ? sx0 : sx1))) : 1.f;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int m = m0 + wm * 64 + mb * 32 + (r & 3) + 8 * (r >> 2) + 4 * half;
                if (m < p.M && k < p.Kc) out[(long)m * p.Kc + k] = F3 ? acc[mb][nb][r] * un : acc[mb][nb][r];
            }
        }
}

__global__ __launch_bounds__(256) void wgrad_reduce_kernel(const float* __restrict__ part, int splits, int step,
                                                           int M, int Kc, int K0, int C0, int Cw, float* __restrict__ dw0,
                                                           long sM0, long sC0, long sT0, float* __restrict__ dw1,
                                                           long sM1, int accumulate) {
    const long i = (long)blockIdx.x * 256 + threadIdx.x;
    const long n = (long)M * Kc;
    if (i >= n) return;
    float s = 0.f;
    for (int sp = 0; sp < splits; sp += step) s += part[(long)sp * n + i];
    const int m = (int)(i / Kc);
    const int k = (int)(i - (long)m * Kc);
    float* dst;
    if (k < K0) {
        const int t = k / C0, c = k - t * C0;
        if (c >= Cw) return;
        dst = dw0 + m * sM0 + c * sC0 + t * sT0;
    } else {
        if (!dw1) return;
        dst = dw1 + m * sM1 + (k - K0);
    }
    *dst = accumulate ? *dst + s : s;
}

// First level of the split reduction when there are many splits: workgroup (chunk, grp) sums slabs
// [grp * RG, grp * RG + RG) of 256 consecutive elements (4 waves, wave w takes slabs w, w + 4, ...,
// float4 per lane; the wave sums meet in LDS in wave order) and writes the result over slab grp * RG
// in place.  The second level (wgrad_reduce_kernel, step RG) adds the groups' slabs in order: a fixed
// summation tree, so results stay deterministic, with the partial slabs read by
// (n / 256) x (splits / RG) workgroups instead of one serial loop per element.
constexpr int RG = 32;
__global__ __launch_bounds__(256) void wgrad_reduce_groups_kernel(float* __restrict__ part, int splits, long n4) {
    __shared__ f32x4 red[3][64];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const long e = (long)blockIdx.x * 64 + lane;  // float4 index
    const int g0 = blockIdx.y * RG, g1 = min(splits, g0 + RG);
    f32x4* p4 = reinterpret_cast<f32x4*>(part);
    f32x4 s = {0.f, 0.f, 0.f, 0.f};
    if (e < n4)
#pragma unroll 4
        for (int sp = g0 + w; sp < g1; sp += 4) s += p4[(long)sp * n4 + e];
    if (w) red[w - 1][lane] = s;
    __syncthreads();
    if (w == 0 && e < n4) p4[(long)g0 * n4 + e] = ((s + red[0][lane]) + red[1][lane]) + red[2][lane];
}
template <int BM, int BN, int PRO, bool X6, bool F3 = false>
int wgrad_launch(const WgDev& d, int grid, hipStream_t s) {
    constexpr int KP = wg_kp<X6>();
    constexpr int bytes =
        2 * (X6 ? wg_nps<X6, F3>() * KP * ((BM * 2 + 64) + (BN * 2 + 64)) : KP * ((BM + 32) + (BN + 32)) * 4);
    static bool attr_set = false;
    if (!attr_set && bytes > 64 * 1024) {
        hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&conv_wgrad_kernel<BM, BN, PRO, X6, F3>),
                                           hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
        if (e != hipSuccess) return (int)e;
        attr_set = true;
    }
    WC_SET_NAME("conv_wgrad_kernel", {WC_TI(BM), WC_TI(BN), WC_TI(PRO), WC_TB(X6), WC_TB(F3)});
    hipLaunchKernelGGL((conv_wgrad_kernel<BM, BN, PRO, X6, F3>), dim3(grid), dim3(WG_THREADS), bytes, s, d);
    WC_CHECK_LAUNCH();
    return WC_OK;
}

template <int BM, int BN>
int wgrad_dispatch(const WgDev& d, int pro, int mode, int grid, hipStream_t s) {  // mode 0 fp32, 1 x6, 2 f16x3
    if (mode == 2) {
        switch (pro) {
            case 0: return wgrad_launch<BM, BN, 0, true, true>(d, grid, s);
            case 1: return wgrad_launch<BM, BN, 1, true, true>(d, grid, s);
            default: return wgrad_launch<BM, BN, 2, true, true>(d, grid, s);
        }
    }
    if (mode == 1) {
        switch (pro) {
            case 0: return wgrad_launch<BM, BN, 0, true>(d, grid, s);
            case 1: return wgrad_launch<BM, BN, 1, true>(d, grid, s);
            default: return wgrad_launch<BM, BN, 2, true>(d, grid, s);
        }
    }
    switch (pro) {
        case 0: return wgrad_launch<BM, BN, 0, false>(d, grid, s);
        case 1: return wgrad_launch<BM, BN, 1, false>(d, grid, s);
        default: return wgrad_launch<BM, BN, 2, false>(d, grid, s);
    }
}

// ============================================================================================
// GroupNorm(+SiLU) backward and per-(b, c) channel sums
// ============================================================================================
constexpr int GB_THREADS = 256;

// part[((b*splits + sp)*C + c)*2 + {0, 1}] = (sum dy, sum dy*xhat) over the split's pixels, with
// xhat = x*sc0[b,c] + sh0[b,c] (sc0 = rstd, sh0 = -mean*rstd), y = gamma*xhat + beta and
// dy = dz * SiLU'(y) (or dz).  HAS_X = false: plain sums of dz (second entry 0).
template <bool HAS_X, bool SILU>
__global__ __launch_bounds__(GB_THREADS) void gnb_reduce_kernel(const float* __restrict__ dz, int ldz,
                                                                 const float* __restrict__ x, int ldx,
                                                                 const float* __restrict__ sc0,
                                                                 const float* __restrict__ sh0,
                                                                 const float* __restrict__ gamma,
                                                                 const float* __restrict__ beta, int HW, int C,
                                                                 int splits, int pps, int nq, float* __restrict__ part,
                                                                 float* __restrict__ part3) {
    __shared__ f32x4 red[3][GB_THREADS];
    const int ncb = C / 4 / nq;
    int t = blockIdx.x;
    const int cb = t % ncb;
    t /= ncb;
    const int sp = t % splits;
    const int b = t / splits;
    const int q = threadIdx.x % nq;
    const int r = threadIdx.x / nq;
    const int R = GB_THREADS / nq;
    const int c = (cb * nq + q) * 4;
    const int p0 = sp * pps;
    const int p1 = min(HW, p0 + pps);
    f32x4 s1 = f32x4{0.f, 0.f, 0.f, 0.f}, s2 = s1, s3 = s1;
    f32x4 a = s1, o = s1, g = f32x4{1.f, 1.f, 1.f, 1.f}, be = s1;
    if constexpr (HAS_X) {
        a = *reinterpret_cast<const f32x4*>(sc0 + (long)b * C + c);
        o = *reinterpret_cast<const f32x4*>(sh0 + (long)b * C + c);
        if (gamma) g = *reinterpret_cast<const f32x4*>(gamma + c);
        if (beta) be = *reinterpret_cast<const f32x4*>(beta + c);
    }
    for (int px = p0 + r; px < p1; px += R) {
        const long pix = (long)b * HW + px;
        f32x4 d = *reinterpret_cast<const f32x4*>(dz + pix * ldz + c);
        if constexpr (HAS_X) {
            const f32x4 xh = *reinterpret_cast<const f32x4*>(x + pix * ldx + c) * a + o;
            if constexpr (SILU) {
                const f32x4 y = g * xh + be;
                d.x *= silu_grad(y.x); d.y *= silu_grad(y.y); d.z *= silu_grad(y.z); d.w *= silu_grad(y.w);
            }
            s2 += d * xh;
            s3 += xh;
        }
        s1 += d;
    }
    red[0][threadIdx.x] = s1;
    red[1][threadIdx.x] = s2;
    red[2][threadIdx.x] = s3;
    __syncthreads();
    if (r == 0) {
        for (int k = 1; k < R; ++k) {
            s1 += red[0][k * nq + q];
            s2 += red[1][k * nq + q];
            s3 += red[2][k * nq + q];
        }
        float* dst = part + (((long)b * splits + sp) * C + c) * 2;
        *reinterpret_cast<f32x4*>(dst) = f32x4{s1.x, s2.x, s1.y, s2.y};
        *reinterpret_cast<f32x4*>(dst + 4) = f32x4{s1.z, s2.z, s1.w, s2.w};
        if (HAS_X && part3) *reinterpret_cast<f32x4*>(part3 + ((long)b * splits + sp) * C + c) = s3;
    }
}

// Workgroup (image b, channel block of cw channels): sums[b][c] = (sum dy, sum dy*xhat) over the splits
// in a fixed order (slice k of the 256 / cw slices sums splits k, k + nsl, ...; the slices are added in
// order).  With coef the block is one GroupNorm group (cw = C / G): A = sum_c gamma_c s1_c and
// Bs = sum_c gamma_c s2_c by a fixed butterfly in wave 0, n = cw*HW, and
// coef[b][c] = (rstd*gamma_c, -rstd*A/n, -rstd*Bs/n) so that dx = c0*dy + c1 + c2*xhat.
// (One workgroup per image with a 64-split chain per channel took ~20 us a launch; this grid is
// B x blocks.)
__global__ __launch_bounds__(GB_THREADS) void gnb_finalize_kernel(const float* __restrict__ part, int splits, int C,
                                                                   int cw, int HW, const float* __restrict__ sc0,
                                                                   const float* __restrict__ gamma,
                                                                   float* __restrict__ sums, float* __restrict__ coef,
                                                                   const float* __restrict__ part3,
                                                                   float* __restrict__ dsum) {
    __shared__ float red[3][GB_THREADS];
    __shared__ float gs[2];
    const int b = blockIdx.x;
    const int nsl = GB_THREADS / cw;
    const int ch = threadIdx.x % cw, sl = threadIdx.x / cw;
    const int c = blockIdx.y * cw + ch;
    const bool act = sl < nsl && c < C;
    const bool want3 = part3 && dsum && coef;
    float s1 = 0.f, s2 = 0.f, s3 = 0.f;
    if (act) {
        const wcx6::f32x2* pp = reinterpret_cast<const wcx6::f32x2*>(part + ((long)b * splits * C + c) * 2);
#pragma unroll 4
        for (int sp = sl; sp < splits; sp += nsl) {
            const wcx6::f32x2 v = pp[(long)sp * C];
            s1 += v.x;
            s2 += v.y;
        }
        if (want3) {
            const float* p3 = part3 + (long)b * splits * C + c;
#pragma unroll 4
            for (int sp = sl; sp < splits; sp += nsl) s3 += p3[(long)sp * C];
        }
    }
    red[0][threadIdx.x] = s1;
    red[1][threadIdx.x] = s2;
    red[2][threadIdx.x] = s3;
    __syncthreads();
    const bool lead = sl == 0 && c < C;
    float ga = 1.f;
    if (lead) {
        for (int k = 1; k < nsl; ++k) {
            s1 += red[0][k * cw + ch];
            s2 += red[1][k * cw + ch];
            s3 += red[2][k * cw + ch];
        }
        sums[((long)b * C + c) * 2] = s1;
        sums[((long)b * C + c) * 2 + 1] = s2;
        if (gamma) ga = gamma[c];
    }
    if (!coef) return;
    __syncthreads();
    if (sl == 0) {
        red[0][ch] = lead ? ga * s1 : 0.f;
        red[1][ch] = lead ? ga * s2 : 0.f;
    }
    __syncthreads();
    if (threadIdx.x < 64) {
        float A = 0.f, Bs = 0.f;
        for (int k = threadIdx.x; k < cw; k += 64) {
            A += red[0][k];
            Bs += red[1][k];
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            A += __shfl_xor(A, o, 64);
            Bs += __shfl_xor(Bs, o, 64);
        }
        if (threadIdx.x == 0) {
            gs[0] = A;
            gs[1] = Bs;
        }
    }
    __syncthreads();
    if (lead) {
        const float inv_n = 1.0f / ((float)cw * (float)HW);
        const float rstd = sc0[(long)b * C + c];
        const f32x4 cf = f32x4{rstd * ga, -rstd * gs[0] * inv_n, -rstd * gs[1] * inv_n, 0.f};
        *reinterpret_cast<f32x4*>(coef + ((long)b * C + c) * 4) = cf;
        // sum over the image's pixels of dx = c0 dy + c1 + c2 xhat, in closed form from the same sums
        if (want3) {
            dsum[((long)b * C + c) * 2] = cf.x * s1 + (float)HW * cf.y + cf.z * s3;
            dsum[((long)b * C + c) * 2 + 1] = 0.f;
        }
    }
}

// out[c] (+)= sum_b sums[(b*C + c)*2 + idx]   (fixed order)
__global__ __launch_bounds__(256) void bsum_kernel(const float* __restrict__ sums, int B, int C, int idx,
                                                   float* __restrict__ out, int accumulate) {
    const int c = blockIdx.x * 256 + threadIdx.x;
    if (c >= C) return;
    float s = 0.f;
    for (int b = 0; b < B; ++b) s += sums[((long)b * C + c) * 2 + idx];
    out[c] = accumulate ? out[c] + s : s;
}

// Many bsums in one launch: job y = blockIdx.y does out[c] (+)= sum_b sums[(b*C + c)*2 + idx] (the
// order of bsum_kernel; the caller gives each output at most one job per launch).
__global__ __launch_bounds__(256) void bsum_batch_kernel(const wc_bsum_job* __restrict__ jobs, int B) {
    const wc_bsum_job j = jobs[blockIdx.y];
    for (int c = blockIdx.x * 256 + threadIdx.x; c < j.C; c += gridDim.x * 256) {
        float s = 0.f;
        for (int b = 0; b < B; ++b) s += j.sums[((long)b * j.C + c) * 2 + j.idx];
        j.out[c] = j.accumulate ? j.out[c] + s : s;
    }
}

// dx (+)= coef0*dy + coef1 + coef2*xhat, elementwise over (b, pixel, 4 channels)
template <bool SILU, bool ACC>
WC_DEVICE f32x4 gnb_apply_one(const float* __restrict__ dz, int ldz, const float* __restrict__ x, int ldx,
                              const float* __restrict__ sc0, const float* __restrict__ sh0,
                              const float* __restrict__ gamma, const float* __restrict__ beta,
                              const float* __restrict__ coef, float* __restrict__ dx, int lddx, long i, int HW, int C,
                              int& b) {
    const int C4 = C / 4;
    const long pix = i / C4;
    const int c = (int)(i - pix * C4) * 4;
    b = (int)(pix / HW);
    const long bc = (long)b * C + c;
    f32x4 d = *reinterpret_cast<const f32x4*>(dz + pix * ldz + c);
    const f32x4 xh = *reinterpret_cast<const f32x4*>(x + pix * ldx + c) * *reinterpret_cast<const f32x4*>(sc0 + bc) +
                     *reinterpret_cast<const f32x4*>(sh0 + bc);
    if constexpr (SILU) {
        const f32x4 g = gamma ? *reinterpret_cast<const f32x4*>(gamma + c) : f32x4{1.f, 1.f, 1.f, 1.f};
        const f32x4 be = beta ? *reinterpret_cast<const f32x4*>(beta + c) : f32x4{0.f, 0.f, 0.f, 0.f};
        const f32x4 y = g * xh + be;
        d.x *= silu_grad(y.x); d.y *= silu_grad(y.y); d.z *= silu_grad(y.z); d.w *= silu_grad(y.w);
    }
    f32x4 res;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
        const f32x4 cf = *reinterpret_cast<const f32x4*>(coef + (bc + e) * 4);
        res[e] = cf.x * d[e] + cf.y + cf.z * xh[e];
    }
    f32x4* o = reinterpret_cast<f32x4*>(dx + pix * lddx + c);
    if constexpr (ACC) res += *o;
    *o = res;
    return res;
}

template <bool SILU, bool ACC>
__global__ __launch_bounds__(256) void gnb_apply_kernel(const float* __restrict__ dz, int ldz, const float* __restrict__ x,
                                                        int ldx, const float* __restrict__ sc0,
                                                        const float* __restrict__ sh0, const float* __restrict__ gamma,
                                                        const float* __restrict__ beta, const float* __restrict__ coef,
                                                        float* __restrict__ dx, int lddx, long n4, int HW, int C) {
    const long i = (long)blockIdx.x * 256 + threadIdx.x;
    if (i >= n4) return;
    int b;
    gnb_apply_one<SILU, ACC>(dz, ldz, x, ldx, sc0, sh0, gamma, beta, coef, dx, lddx, i, HW, C, b);
}

// The same, also raising absmax[b] to the max |dx| WRITTEN per image (after the accumulate: the
// final value of every element it writes, so absmax over all writers of a tensor bounds the tensor).
// Workgroup k walks the float4 range [k per, (k + 1) per) (per a multiple of 1024), four elements per
// thread per round with every load of the round issued before its first store (vmcnt counts stores:
// a load after a store would wait for the store); the maxima go out once per workgroup when the range
// lies in one image (the usual case: all B slots share one L2 line, so the atomics are kept few), per
// lane otherwise.
template <bool SILU, bool ACC>
__global__ __launch_bounds__(256) void gnb_apply_absmax_kernel(
    const float* __restrict__ dz, int ldz, const float* __restrict__ x, int ldx, const float* __restrict__ sc0,
    const float* __restrict__ sh0, const float* __restrict__ gamma, const float* __restrict__ beta,
    const float* __restrict__ coef, float* __restrict__ dx, int lddx, long n4, int HW, int C, long per,
    float* __restrict__ absmax) {
    __shared__ float wm[4];
    const long i0 = (long)blockIdx.x * per;
    const long i1 = min(n4, i0 + per);
    const int C4 = C / 4;
    const long per_img = (long)HW * C4;
    const int bfirst = (int)(i0 / per_img), blast = (int)((i1 - 1) / per_img);
    float m = 0.f;
    int bc = bfirst;
    for (long base = i0 + threadIdx.x; base < i1; base += 1024) {
        f32x4 d[4], xv[4], o[4];
        long pofs[4];
        int bb[4], cc[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const long i = min(base + 256 * u, i1 - 1);  // past the range: a repeat of the last element, not stored
            const long pix = i / C4;
            cc[u] = (int)(i - pix * C4) * 4;
            bb[u] = (int)(pix / HW);
            pofs[u] = pix;
            d[u] = *reinterpret_cast<const f32x4*>(dz + pix * ldz + cc[u]);
            xv[u] = *reinterpret_cast<const f32x4*>(x + pix * ldx + cc[u]);
            if constexpr (ACC) o[u] = *reinterpret_cast<const f32x4*>(dx + pix * lddx + cc[u]);
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const long bc4 = (long)bb[u] * C + cc[u];
            const f32x4 xh = xv[u] * *reinterpret_cast<const f32x4*>(sc0 + bc4) + *reinterpret_cast<const f32x4*>(sh0 + bc4);
            f32x4 dd = d[u];
            if constexpr (SILU) {
                const f32x4 g = gamma ? *reinterpret_cast<const f32x4*>(gamma + cc[u]) : f32x4{1.f, 1.f, 1.f, 1.f};
                const f32x4 be = beta ? *reinterpret_cast<const f32x4*>(beta + cc[u]) : f32x4{0.f, 0.f, 0.f, 0.f};
                const f32x4 y = g * xh + be;
                dd.x *= silu_grad(y.x); dd.y *= silu_grad(y.y); dd.z *= silu_grad(y.z); dd.w *= silu_grad(y.w);
            }
            f32x4 r;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const f32x4 cf = *reinterpret_cast<const f32x4*>(coef + (bc4 + e) * 4);
                r[e] = cf.x * dd[e] + cf.y + cf.z * xh[e];
            }
            if constexpr (ACC) r += o[u];
            o[u] = r;
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            if (base + 256 * u >= i1) continue;
            *reinterpret_cast<f32x4*>(dx + pofs[u] * lddx + cc[u]) = o[u];
            const float v = fmaxf(fmaxf(fabsf(o[u].x), fabsf(o[u].y)), fmaxf(fabsf(o[u].z), fabsf(o[u].w)));
            if (bfirst != blast && bb[u] != bc) {  // a range crossing images: flush the lane's maximum
                atomicMax(reinterpret_cast<unsigned*>(absmax) + bc, __float_as_uint(m));
                bc = bb[u];
                m = 0.f;
            }
            m = fmaxf(m, v);
        }
    }
    if (bfirst == blast) {  // one image: one atomic for the workgroup
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
        if ((threadIdx.x & 63) == 0) wm[threadIdx.x >> 6] = m;
        __syncthreads();
        if (threadIdx.x == 0)
            atomicMax(reinterpret_cast<unsigned*>(absmax) + bfirst,
                      __float_as_uint(fmaxf(fmaxf(wm[0], wm[1]), fmaxf(wm[2], wm[3]))));
    } else {
        atomicMax(reinterpret_cast<unsigned*>(absmax) + bc, __float_as_uint(m));
    }
}

// ============================================================================================
// small dense helpers (time-embedding MLP: B x 128 rows)
// ============================================================================================
// C[m][n] = alpha * sum_k A[m*sam + k*sak] * B[k*sbk + n*sbn] + beta*C[m][n]  (beta = 0: no read)
__global__ __launch_bounds__(256) void gemm_small_kernel(int M, int N, int K, const float* __restrict__ A, long sam,
                                                         long sak, const float* __restrict__ Bm, long sbk, long sbn,
                                                         float* __restrict__ Cm, long ldc, float alpha, float beta) {
    const long i = (long)blockIdx.x * 256 + threadIdx.x;
    if (i >= (long)M * N) return;
    const int m = (int)(i / N), n = (int)(i - (long)m * N);
    float s = 0.f;
    for (int k = 0; k < K; ++k) s = fmaf(A[m * sam + k * sak], Bm[k * sbk + n * sbn], s);
    float* c = Cm + m * ldc + n;
    *c = beta != 0.f ? alpha * s + beta * *c : alpha * s;
}

// The same with one wave per output for long K (the time-embedding input gradient: K = all ResBlock
// channels): lanes stride K, then a fixed butterfly (deterministic).
__global__ __launch_bounds__(256) void gemm_small_wave_kernel(int M, int N, int K, const float* __restrict__ A, long sam,
                                                              long sak, const float* __restrict__ Bm, long sbk,
                                                              long sbn, float* __restrict__ Cm, long ldc, float alpha,
                                                              float beta) {
    const long o = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (o >= (long)M * N) return;
    const int m = (int)(o / N), n = (int)(o - (long)m * N);
    float s = 0.f;
    for (int k = lane; k < K; k += 64) s = fmaf(A[m * sam + k * sak], Bm[k * sbk + n * sbn], s);
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off, 64);
    if (lane == 0) {
        float* c = Cm + m * ldc + n;
        *c = beta != 0.f ? alpha * s + beta * *c : alpha * s;
    }
}

// mode 0: out = silu(y); mode 1: out = dz * silu'(y)
__global__ __launch_bounds__(256) void silu_kernel(const float* __restrict__ y, const float* __restrict__ dz,
                                                   float* __restrict__ out, long n, int mode) {
    const long i = (long)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    out[i] = mode == 0 ? wc_silu(y[i]) : dz[i] * silu_grad(y[i]);
}

// out[n] (+)= sum_r X[r*ldx + n]
__global__ __launch_bounds__(256) void colsum_kernel(const float* __restrict__ X, int R, int N, long ldx,
                                                     float* __restrict__ out, int accumulate) {
    const int n = blockIdx.x * 256 + threadIdx.x;
    if (n >= N) return;
    float s = 0.f;
    for (int r = 0; r < R; ++r) s += X[r * ldx + n];
    out[n] = accumulate ? out[n] + s : s;
}

// reference get_time_embedding (unet_base.py:7-30): [sin(t/f_k), cos(t/f_k)], f_k = 10000^(k/half)
__global__ __launch_bounds__(256) void time_embedding_kernel(const int64_t* __restrict__ t, int nt, int D,
                                                             float* __restrict__ out) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    const int half = D / 2;
    if (i >= nt * half) return;
    const int row = i / half, k = i - row * half;
    const float f = powf(10000.0f, (float)k / (float)half);
    const float a = (float)t[row] / f;
    out[(long)row * D + k] = sinf(a);
    out[(long)row * D + k + half] = cosf(a);
}

__global__ __launch_bounds__(256) void nchw_to_nhwc_kernel(const float* __restrict__ src, int C, int HW, long total,
                                                           float* __restrict__ dst, int ldc) {
    const long i = (long)blockIdx.x * 256 + threadIdx.x;
    if (i >= total) return;  // total = B*HW*ldc
    const long pix = i / ldc;
    const int c = (int)(i - pix * ldc);
    const long b = pix / HW;
    const long p = pix - b * HW;
    dst[i] = c < C ? src[(b * C + c) * HW + p] : 0.f;
}

inline unsigned blocks_for(long n, int per) { return (unsigned)((n + per - 1) / per); }

// absmax[b] = max |x| over image b of an NHWC view (C channels at pixel stride ldx); the caller zeroes
// absmax.  Grid (chunks, B): each workgroup reduces a contiguous pixel range of one image, one atomic
// per workgroup (|x| >= 0 orders like its unsigned bits, so the max is exact and order-free).
__global__ __launch_bounds__(256) void absmax_images_kernel(const float* __restrict__ x, int ldx, int HW, int C4,
                                                           int ppb, float* __restrict__ absmax) {
    const int b = blockIdx.y;
    const long p0 = (long)blockIdx.x * ppb;
    const long p1 = min((long)HW, p0 + ppb);
    const float* img = x + (long)b * HW * ldx;
    float m = 0.f;
    auto take = [&](const float* q) {
        const f32x4 v = *reinterpret_cast<const f32x4*>(q);
        m = fmaxf(m, fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w))));
    };
    if (C4 <= 256) {
        // thread = (pixel offset, channel quad), fixed for the whole range: no per-element index division
        // (the 64-bit divide per float4 held this pass to ~1.8 TB/s)
        const int per = 256 / C4;  // pixels per pass
        const int c4 = threadIdx.x % C4, pxo = threadIdx.x / C4;
        if (pxo < per) {
            const float* q = img + (p0 + pxo) * ldx + 4 * c4;
            const long stride = (long)per * ldx;
#pragma unroll 4
            for (long px = p0 + pxo; px < p1; px += per, q += stride) take(q);
        }
    } else {
        for (long px = p0; px < p1; ++px)
            for (int c4 = threadIdx.x; c4 < C4; c4 += 256) take(img + px * ldx + 4 * c4);
    }
    wcx6::block_absmax_atomic(absmax, b, m);
}

}  // namespace

// ---------------------------------------------------------------------------------------------
static int conv_wgrad_any(const wc_wgrad_args* a, float* part, int splits, int mode, const float* gb, int xe0,
                          const float* xb0, const float* xb1, void* stream) {
    if (!a || !a->g || !part || a->nseg < 1 || a->nseg > 2) return WC_E_ARG;
    if (mode == 2 && (!gb || (a->nseg == 2 && !xb1) || xe0 < -100 || xe0 > 60)) return WC_E_ARG;
    const wc_conv_seg& s0 = a->seg[0];
    if (!s0.src) return WC_E_ARG;
    if (a->M <= 0 || a->M % 4 || a->ldg % 4 || s0.C <= 0 || s0.C % 4 || s0.ldc % 4) return WC_E_SHAPE;
    if (s0.ntaps < 1 || s0.ntaps > WC_MAX_TAPS || splits < 1 || s0.sy < 1 || s0.sx < 1) return WC_E_SHAPE;
    if (a->B < 1 || a->Hm < 1 || a->Wm < 1) return WC_E_SHAPE;
    if ((s0.scale == nullptr) != (s0.shift == nullptr)) return WC_E_ARG;
    if (((reinterpret_cast<uintptr_t>(a->g) | reinterpret_cast<uintptr_t>(s0.src)) & 15) != 0) return WC_E_SHAPE;
    const long P = (long)a->B * a->Hm * a->Wm;
    if (P <= 0 || (long)a->B * s0.H * s0.W * s0.ldc * 4 >= (1L << 31) || P * a->ldg * 4 >= (1L << 31))
        return WC_E_SHAPE;
    WgDev d{};
    d.g = a->g; d.M = a->M; d.ldg = a->ldg;
    d.src0 = s0.src; d.C0 = s0.C; d.ldc0 = s0.ldc; d.H0 = s0.H; d.W0 = s0.W; d.sy = s0.sy; d.sx = s0.sx;
    d.ntaps = s0.ntaps;
    for (int t = 0; t < s0.ntaps; ++t) { d.dy[t] = s0.dy[t]; d.dx[t] = s0.dx[t]; }
    d.scale = s0.scale; d.shift = s0.shift;
    d.K0 = s0.ntaps * s0.C;
    d.Kc = d.K0;
    if (a->nseg == 2) {
        const wc_conv_seg& s1 = a->seg[1];
        if (!s1.src || s1.scale) return WC_E_ARG;
        if (s1.C <= 0 || s1.C % 4 || s1.ldc % 4 || (reinterpret_cast<uintptr_t>(s1.src) & 15) != 0) return WC_E_SHAPE;
        if (s1.ntaps != 1 || s1.dy[0] != 0 || s1.dx[0] != 0) return WC_E_SHAPE;
        // the 1x1 residual segment is read at the pixel itself (stride 1, the gradient's grid)
        if (s0.sy != 1 || s0.sx != 1 || s1.sy != 1 || s1.sx != 1 || s1.H != a->Hm || s1.W != a->Wm)
            return WC_E_SHAPE;
        if ((long)a->B * s1.H * s1.W * s1.ldc * 4 >= (1L << 31)) return WC_E_SHAPE;
        d.src1 = s1.src; d.C1 = s1.C; d.ldc1 = s1.ldc; d.H1 = s1.H; d.W1 = s1.W;
        d.Kc += s1.C;
    }
    d.Hm = a->Hm; d.Wm = a->Wm; d.P = P;
    const bool narrow = a->M <= 64;
    const int BM = narrow ? 64 : 128, BN = narrow ? 256 : 128;
    d.ntm = (a->M + BM - 1) / BM;
    d.ntn = (d.Kc + BN - 1) / BN;
    d.pps = ((P + splits - 1) / splits + WG_KP - 1) / WG_KP * WG_KP;
    const long nsp = (P + d.pps - 1) / d.pps;
    if (nsp != splits) return WC_E_SHAPE;  // the caller sizes part by wc_conv_wgrad_splits
    d.part = part;
    d.gb = gb; d.xb0 = xb0; d.xb1 = xb1; d.xe0 = xe0; d.B = a->B;
    const long grid = (long)d.ntm * d.ntn * splits;
    if (grid > (1L << 30)) return WC_E_SHAPE;
    const int pro = s0.scale ? (s0.silu ? 2 : 1) : 0;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    return narrow ? wgrad_dispatch<64, 256>(d, pro, mode, (int)grid, s) : wgrad_dispatch<128, 128>(d, pro, mode, (int)grid, s);
}

extern "C" int wc_conv_wgrad(const wc_wgrad_args* a, float* part, int splits, void* stream) {
    return conv_wgrad_any(a, part, splits, 0, nullptr, 0, nullptr, nullptr, stream);
}

extern "C" int wc_conv_wgrad_x6(const wc_wgrad_args* a, float* part, int splits, void* stream) {
    return conv_wgrad_any(a, part, splits, 1, nullptr, 0, nullptr, nullptr, stream);
}

extern "C" int wc_conv_wgrad_f16x3(const wc_wgrad_args* a, float* part, int splits, const float* gbound, int x_exp0,
                                   const float* xbound0, const float* xbound1, void* stream) {
    return conv_wgrad_any(a, part, splits, 2, gbound, x_exp0, xbound0, xbound1, stream);
}

extern "C" int wc_conv_wgrad_splits(int M, int Kc, int64_t P, int target_blocks) {
    const bool narrow = M <= 64;
    const int BM = narrow ? 64 : 128, BN = narrow ? 256 : 128;
    const long tiles = (long)((M + BM - 1) / BM) * ((Kc + BN - 1) / BN);
    long sp = (target_blocks + tiles - 1) / tiles;
    const long maxsp = (P + 255) / 256;  // at least 8 K-steps per split
    if (sp > maxsp) sp = maxsp;
    if (sp < 1) sp = 1;
    // the kernel's pixels-per-split rounding may need fewer splits to cover P
    const long pps = ((P + sp - 1) / sp + WG_KP - 1) / WG_KP * WG_KP;
    return (int)((P + pps - 1) / pps);
}

extern "C" int wc_wgrad_reduce(float* part, int splits, int M, int Kc, int K0, int C0, int Cw, float* dw0,
                               int64_t sM0, int64_t sC0, int64_t sT0, float* dw1, int64_t sM1, int accumulate,
                               void* stream) {
    if (!part || !dw0 || splits < 1 || M <= 0 || Kc <= 0 || K0 <= 0 || C0 <= 0 || K0 % C0 || K0 > Kc) return WC_E_ARG;
    if (Kc > K0 && !dw1) return WC_E_ARG;
    const long n = (long)M * Kc;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    int step = 1;
    if (splits > RG && n % 4 == 0 && (reinterpret_cast<uintptr_t>(part) & 15) == 0) {
        // part is scratch: the group sums overwrite the first slab of each group
        const long n4 = n / 4;
        const int ng = (splits + RG - 1) / RG;
        hipLaunchKernelGGL(wgrad_reduce_groups_kernel, dim3((unsigned)((n4 + 63) / 64), (unsigned)ng), dim3(256), 0, s,
                           part, splits, n4);
        WC_CHECK_LAUNCH();
        step = RG;
    }
    wc_last_kernel = "wgrad_reduce_kernel";
    hipLaunchKernelGGL(wgrad_reduce_kernel, dim3(blocks_for(n, 256)), dim3(256), 0, s, part, splits, step, M, Kc, K0,
                       C0, Cw, dw0, (long)sM0, (long)sC0, (long)sT0, dw1, (long)sM1, accumulate);
    WC_CHECK_LAUNCH();
    return WC_OK;
}

// channel quads per workgroup: the largest power of two <= 64 dividing C/4 (the threads' rows then
// tile the 256-thread workgroup exactly)
static int gnb_nq(int C) {
    const int q = C / 4;
    if (C % 4 || q < 1) return -1;
    int nq = 64;
    while (q % nq) nq >>= 1;
    return nq;
}

extern "C" int wc_gn_bwd_splits(int B, int HW) {
    int sp = 1024 / (B < 1 ? 1 : B);
    const int maxsp = HW / 16 < 1 ? 1 : HW / 16;
    sp = sp > maxsp ? maxsp : sp;
    sp = sp > 256 ? 256 : sp;
    return sp < 1 ? 1 : sp;
}

extern "C" int wc_gn_bwd_reduce(const float* dz, int ldz, const float* x, int ldx, const float* sc0, const float* sh0,
                                const float* gamma, const float* beta, int silu, int B, int HW, int C, int splits,
                                float* part, float* part3, void* stream) {
    if (!dz || !part || (x && (!sc0 || !sh0)) || (part3 && !x)) return WC_E_ARG;
    const int nq = gnb_nq(C);
    if (nq < 0 || ldz % 4 || (x && ldx % 4) || splits < 1 || B < 1 || HW < 1) return WC_E_SHAPE;
    const int pps = (HW + splits - 1) / splits;
    const long grid = (long)B * splits * (C / 4 / nq);
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    if (!x)
        hipLaunchKernelGGL((gnb_reduce_kernel<false, false>), dim3((unsigned)grid), dim3(GB_THREADS), 0, s, dz, ldz, x,
                           ldx, sc0, sh0, gamma, beta, HW, C, splits, pps, nq, part, part3);
    else if (silu)
        hipLaunchKernelGGL((gnb_reduce_kernel<true, true>), dim3((unsigned)grid), dim3(GB_THREADS), 0, s, dz, ldz, x, ldx,
                           sc0, sh0, gamma, beta, HW, C, splits, pps, nq, part, part3);
    else
        hipLaunchKernelGGL((gnb_reduce_kernel<true, false>), dim3((unsigned)grid), dim3(GB_THREADS), 0, s, dz, ldz, x,
                           ldx, sc0, sh0, gamma, beta, HW, C, splits, pps, nq, part, part3);
    WC_CHECK_LAUNCH();
    return WC_OK;
}

extern "C" int wc_gn_bwd_finalize(const float* part, int B, int splits, int C, int groups, int HW, const float* sc0,
                                  const float* gamma, float* sums, float* coef, const float* part3, float* dsum,
                                  void* stream) {
    if (!part || !sums || (coef && !sc0) || ((part3 != nullptr) != (dsum != nullptr)) || (dsum && !coef))
        return WC_E_ARG;
    if (C < 1 || B < 1 || splits < 1 || (coef && (groups < 1 || C % groups))) return WC_E_SHAPE;
    const int cw = coef ? C / groups : (C < 64 ? C : 64);
    if (cw > GB_THREADS) return WC_E_SHAPE;
    hipLaunchKernelGGL(gnb_finalize_kernel, dim3(B, (C + cw - 1) / cw), dim3(GB_THREADS), 0,
                       reinterpret_cast<hipStream_t>(stream), part, splits, C, cw, HW, sc0, gamma, sums, coef, part3, dsum);
    WC_CHECK_LAUNCH();
    return WC_OK;
}

extern "C" int wc_bsum(const float* sums, int B, int C, int idx, float* out, int accumulate, void* stream) {
    if (!sums || !out || idx < 0 || idx > 1) return WC_E_ARG;
    hipLaunchKernelGGL(bsum_kernel, dim3(blocks_for(C, 256)), dim3(256), 0, reinterpret_cast<hipStream_t>(stream), sums,
                       B, C, idx, out, accumulate);
    WC_CHECK_LAUNCH();
    return WC_OK;
}

extern "C" int wc_bsum_batch(const wc_bsum_job* jobs, int njobs, int B, int max_c, void* stream) {
    if (!jobs || njobs < 0 || B < 1 || max_c < 0) return WC_E_ARG;
    if (njobs == 0 || max_c == 0) return WC_OK;
    if (njobs > 65535) return WC_E_SHAPE;
    hipLaunchKernelGGL(bsum_batch_kernel, dim3(blocks_for(max_c, 256), njobs), dim3(256), 0,
                       reinterpret_cast<hipStream_t>(stream), jobs, B);
    WC_CHECK_LAUNCH();
    return WC_OK;
}

extern "C" int wc_gn_bwd_apply(const float* dz, int ldz, const float* x, int ldx, const float* sc0, const float* sh0,
                               const float* gamma, const float* beta, int silu, const float* coef, int B, int HW, int C,
                               float* dx, int lddx, int accumulate, float* absmax, void* stream) {
    if (!dz || !x || !sc0 || !sh0 || !coef || !dx) return WC_E_ARG;
    if (C % 4 || ldz % 4 || ldx % 4 || lddx % 4) return WC_E_SHAPE;
    if (((reinterpret_cast<uintptr_t>(dz) | reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(dx)) & 15) != 0)
        return WC_E_SHAPE;
    const long n4 = (long)B * HW * (C / 4);
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    if (absmax) {
        const long nb = std::min<long>(blocks_for(n4, 1024), 2048);
        const long per = ((n4 + nb - 1) / nb + 1023) / 1024 * 1024;
        const dim3 g((unsigned)((n4 + per - 1) / per));
#define WC_GNB_APPLY(S, A)                                                                                       \
    hipLaunchKernelGGL((gnb_apply_absmax_kernel<S, A>), g, dim3(256), 0, s, dz, ldz, x, ldx, sc0, sh0, gamma, beta, \
                       coef, dx, lddx, n4, HW, C, per, absmax)
        if (silu) {
            if (accumulate) WC_GNB_APPLY(true, true); else WC_GNB_APPLY(true, false);
        } else {
            if (accumulate) WC_GNB_APPLY(false, true); else WC_GNB_APPLY(false, false);
        }
#undef WC_GNB_APPLY
        WC_CHECK_LAUNCH();
        return WC_OK;
    }
    const dim3 g(blocks_for(n4, 256));
#define WC_GNB_APPLY(S, A) \
    hipLaunchKernelGGL((gnb_apply_kernel<S, A>), g, dim3(256), 0, s, dz, ldz, x, ldx, sc0, sh0, gamma, beta, coef, dx, lddx, n4, HW, C)
    if (silu) {
        if (accumulate) WC_GNB_APPLY(true, true); else WC_GNB_APPLY(true, false);
    } else {
        if (accumulate) WC_GNB_APPLY(false, true); else WC_GNB_APPLY(false, false);
    }
#undef WC_GNB_APPLY
    WC_CHECK_LAUNCH();
    return WC_OK;
}

extern "C" int wc_gemm_small(int M, int N, int K, const float* A, int64_t sam, int64_t sak, const float* Bm, int64_t sbk,
                             int64_t sbn, float* Cm, int64_t ldc, float alpha, float beta, void* stream) {
    if (!A || !Bm || !Cm) return WC_E_ARG;
    if (M <= 0 || N <= 0 || K <= 0) return WC_E_SHAPE;
    if (K >= 256) {
        wc_last_kernel = "gemm_small_wave_kernel";
        hipLaunchKernelGGL(gemm_small_wave_kernel, dim3(blocks_for((long)M * N, 4)), dim3(256), 0,
                           reinterpret_cast<hipStream_t>(stream), M, N, K, A, (long)sam, (long)sak, Bm, (long)sbk,
                           (long)sbn, Cm, (long)ldc, alpha, beta);
        WC_CHECK_LAUNCH();
        return WC_OK;
    }
    hipLaunchKernelGGL(gemm_small_kernel, dim3(blocks_for((long)M * N, 256)), dim3(256), 0,
                       reinterpret_cast<hipStream_t>(stream), M, N, K, A, (long)sam, (long)sak, Bm, (long)sbk,
                       (long)sbn, Cm, (long)ldc, alpha, beta);
    WC_CHECK_LAUNCH();
    return WC_OK;
}

extern "C" int wc_silu(const float* y, const float* dz, float* out, int64_t n, int mode, void* stream) {
    if (!y || !out || (mode == 1 && !dz) || mode < 0 || mode > 1) return WC_E_ARG;
    if (n <= 0) return WC_E_SHAPE;
    hipLaunchKernelGGL(silu_kernel, dim3(blocks_for(n, 256)), dim3(256), 0, reinterpret_cast<hipStream_t>(stream), y, dz,
                       out, (long)n, mode);
    WC_CHECK_LAUNCH();
    return WC_OK;
}

extern "C" int wc_colsum(const float* X, int R, int N, int64_t ldx, float* out, int accumulate, void* stream) {
    if (!X || !out) return WC_E_ARG;
    if (R <= 0 || N <= 0) return WC_E_SHAPE;
    hipLaunchKernelGGL(colsum_kernel, dim3(blocks_for(N, 256)), dim3(256), 0, reinterpret_cast<hipStream_t>(stream), X, R,
                       N, (long)ldx, out, accumulate);
    WC_CHECK_LAUNCH();
    return WC_OK;
}

extern "C" int wc_time_embedding(const int64_t* t, int nt, int D, float* out, void* stream) {
    if (!t || !out) return WC_E_ARG;
    if (nt <= 0 || D <= 0 || D % 2) return WC_E_SHAPE;
    hipLaunchKernelGGL(time_embedding_kernel, dim3(blocks_for((long)nt * (D / 2), 256)), dim3(256), 0,
                       reinterpret_cast<hipStream_t>(stream), t, nt, D, out);
    WC_CHECK_LAUNCH();
    return WC_OK;
}

extern "C" int wc_nchw_to_nhwc(const float* src, int B, int C, int H, int W, float* dst, int ldc, void* stream) {
    if (!src || !dst) return WC_E_ARG;
    if (B <= 0 || C <= 0 || ldc < C || H <= 0 || W <= 0) return WC_E_SHAPE;
    const long total = (long)B * H * W * ldc;
    hipLaunchKernelGGL(nchw_to_nhwc_kernel, dim3(blocks_for(total, 256)), dim3(256), 0,
                       reinterpret_cast<hipStream_t>(stream), src, C, H * W, total, dst, ldc);
    WC_CHECK_LAUNCH();
    return WC_OK;
}

// Per-image max |x| of an NHWC view (the range bound of a gradient operand on f16x3): see
// absmax_images_kernel.  absmax must be zeroed by the caller.
extern "C" int wc_absmax_images(const float* x, int ldx, int B, int HW, int C, float* absmax, void* stream) {
    if (!x || !absmax) return WC_E_ARG;
    if (B <= 0 || HW <= 0 || C <= 0 || C % 4 || ldx % 4 || (reinterpret_cast<uintptr_t>(x) & 15)) return WC_E_SHAPE;
    const int ppb = 512;  // pixels per workgroup
    const dim3 grid((unsigned)((HW + ppb - 1) / ppb), (unsigned)B);
    hipLaunchKernelGGL(absmax_images_kernel, grid, dim3(256), 0, reinterpret_cast<hipStream_t>(stream), x, ldx, HW, C / 4,
                       ppb, absmax);
    WC_CHECK_LAUNCH();
    return WC_OK;
}
