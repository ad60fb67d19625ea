// General implicit-GEMM convolution on bf16x6 split-precision MFMA for gfx950: any tap grid,
// input stride, 1x1 residual segment and output map (NHWC view / parity-strided / NCHW) — the
// same contract as wc_conv_igemm (wc_conv.hip), at the bf16x6 arithmetic of wc_conv6.hip.
//
// Used for the convs the halo-tiled 3x3 kernel does not take: the attention in/out projections
// (1x1, GN-affine prologue / residual epilogue), the 4x4 stride-2 down convs, the four parity
// sub-convs of each ConvTranspose2d, and 3x3 convs whose grid does not tile (head, small levels).
//
// Structure (as wc_conv.hip, with 16-channel K-steps):
//   * GEMM view M = B*Hm*Wm output positions, N = output channels, K-step = 16 channels of one
//     tap (segment 0, tap-major) or of the 1x1 residual segment.  The weight is pre-split by the
//     host into [N tile][K-step][piece 3][k-half 2][BN][8] bf16 (K in natural order).
//   * 4 waves, each a 64x64 sub-tile of 2x2 32x32 accumulators; per K-step 24 MFMAs
//     (piece-order sums 0, 1, 2 of both operands).
//   * The global loads of step k+1 are issued before the MFMAs of step k; after them the A
//     values get the GN(+SiLU) prologue, zero padding, the exact 3-piece split, and are written
//     into the other LDS buffer with the step's weight pieces; one barrier per step.
//   * LDS images are [piece][k-half][row][8 bf16] (16-byte row slots): the ds_read_b128 lane
//     groups {0-3,12-15,20-27} / {4-11,16-19,28-31} read 16 rows distinct mod 16 ->
//     conflict-free with no swizzle.
#include <type_traits>

#include "wc_x6.hpp"

namespace {

using namespace wcx6;

constexpr int NT = 256;
constexpr int BK = 16;  // channels per K-step

struct IgDev {
    const float* src0;
    int C0, ldc0, H0, W0, sy, sx;
    int kh, kw, ty0, tdy, tx0, tdx;  // tap (ky, kx) reads input (y*sy + ty0 + ky*tdy, x*sx + tx0 + kx*tdx)
    const float* scale;
    const float* shift;
    const float* src1;
    int C1, ldc1;
    int B, Hm, Wm, N, M;
    const void* w6;
    const float* bias;
    const float* temb;
    int temb_ld;
    const float* res;
    int ldres;
    float* out;
    int ldo;
    int Ho, Wo, osy, osx, ooy, oox, out_nchw;
    int ident;
    int steps0, steps;
    int cpt;             // 16-channel chunks per tap of segment 0
    int ntiles_n;
    float ascale;        // f16x3: 2^a_exp applied to the A values before splitting (else 1)
    float ainv;          // 2^-a_exp
    const float* wsinv;  // f16x3: 2^-sW[n] (else NULL)
    const float* abound; // f16x3: per-image bound of the segment-0 values (UNIB only), or NULL
    int a_exp;           // f16x3: static exponent (the per-image bound may lower it)
    float* absmax;       // optional per-image max |out| (atomic)
    float* gn_part;      // optional GroupNorm tile partials (UNIB only; wcx6::gn_tile_partials)
    int gn_ncb, gn_sw, gn_c0, gn_p64, gn_np64;
    unsigned short* qkv3;  // optional: attention in-projection written pre-split (wc_conv_igemm_f16x3_qkv)
    const unsigned char* a3;  // PA: segment 0 already scaled and split (wc_split_f16x3_tiled layout)
    int qC, qD;            // C and the head dim of that projection
    float qscale[3];       // 2^exps of q, k, v
};

// F3: segment 0 in f16x3 (2 fp16 pieces), else bf16x6; segment 1 is always bf16x6.  NPL: LDS
// planes per operand stage (piece x k-half): 4 for an f16x3 launch without segment 1, else 6.
template <int BM, int BN, bool F3, int NPL>
struct IgTile {
    static constexpr int WAVES_M = BM / 64;
    static constexpr int WAVES_N = BN / 64;
    static_assert(WAVES_M * WAVES_N == 4, "4 waves of 64x64");
    static_assert(NPL == 6 || (F3 && NPL == 4), "4-plane stages hold f16x3 segment-0 steps only");
    static constexpr int A_PER_T = BM * (BK / 4) / NT;  // float4 per thread per step
    static constexpr int APLANE = BM * 16;              // bytes of one (piece, k-half) plane
    static constexpr int BPLANE = BN * 16;
    static constexpr int ASTAGE = NPL * APLANE;
    static constexpr int BSTAGE = NPL * BPLANE;
    static constexpr int STAGE = ASTAGE + BSTAGE;
    static constexpr int BSTEP0 = (F3 ? 4 : 6) * BPLANE;  // weight bytes of a segment-0 step
    static constexpr int BSTEP1 = 6 * BPLANE;             // ... of a segment-1 step
    static constexpr int B_PER_T = (BSTAGE / 16 + NT - 1) / NT;
    static constexpr int B_FULL = BSTEP0 / 16 / NT;       // items j < B_FULL valid in every step
};

// Output-tile order of the GEMM grids.  XCD-aware bijection first (blocks b and b + 8 share an XCD:
// consecutive logical tiles land on one XCD's L2), then, within the logical order, bands of WC_IG_GM
// M-tiles walked N-tile by N-tile (M fastest inside a band): the ~64 workgroups an XCD runs at once
// then hold about 8 A row-tiles and 8 B column-tiles instead of ~4 A tiles and every B tile -- the
// qkv projections' B (C x 3C, up to 7 MB pre-split) does not fit a 4 MB L2 and was refetched for
// every M-tile.  WC_IG_GM = 1 is the plain N-fastest order.
#ifndef WC_IG_GM
#define WC_IG_GM 8
#endif
WC_DEVICE void ig_tile_order(int ntn, int& tm, int& tn) {
    const int nblk = gridDim.x;
    int bid = blockIdx.x;
    {
        const int q = nblk / 8, r = nblk % 8, xcd = bid % 8;
        bid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + bid / 8;
    }
    const int ntm = nblk / ntn;
    const int band = bid / (WC_IG_GM * ntn), rem = bid - band * (WC_IG_GM * ntn);
    const int gm = min(WC_IG_GM, ntm - band * WC_IG_GM);  // the last band may be narrower
    tn = rem / gm;
    tm = band * WC_IG_GM + rem % gm;
}

// PRO: 0 raw, 1 GN affine, 2 GN affine + SiLU.  UNIB: tiles never straddle images.  ACT: epilogue
// activation (template, see wc_conv.hip).  F3: segment 0 on f16x3 (caller bounds |a| 2^a_exp).
// TR (the pre-split qkv epilogue only): accumulate the transposed block (lanes = pixels, rows =
// channels; the same products, B and A fragments swapped in the MFMA).
// The pre-split qkv form (TR, BN 128) is held to 3 waves per SIMD (174 -> 168 VGPRs, 5 spilled).
// P1 (UNIB, f16x3 segment 0 only): a pointwise 1x1 stride-1 conv whose tiles are whole rows of one
// image (the attention projections): no tap stepping, no bounds or padding logic per element.
// PA (with P1): the A operand arrives pre-scaled and pre-split in the LDS stage order
// (wc_split_f16x3_tiled), so both operands of a K-step are 16 KiB copied HBM/L2 -> LDS by
// LDS-DMA (4 wave-instructions per wave, no registers, no VALU) into a 3-stage ring: the copy of
// step s + 2 is issued while step s computes, one barrier per step.  (Measured and dropped: a 4-stage
// ring walked in pairs of steps, one barrier per pair: 254 vs 274 TF/s at two instead of three
// workgroups per CU -- the projections are not barrier-bound.)
template <int BM, int BN, int PRO, bool UNIB, int ACT, bool F3, int NPL, bool TR = false, bool P1 = false,
          bool PA = false>
__global__ __launch_bounds__(NT, (TR && BN == 128) ? 3 : 2) void conv_igemm_x6_kernel(IgDev p) {
    using T = IgTile<BM, BN, F3, NPL>;
    static_assert(!PA || (P1 && F3 && NPL == 4 && UNIB && PRO == 0), "PA: pre-split pointwise f16x3");
    // PA: the 3 ring stages are distinct LDS objects, so the compiler sees that a step's fragment
    // reads cannot alias the LDS-DMA in flight into another stage (one array would make it wait
    // vmcnt(0) before every read, i.e. for the copy just issued)
    // (PA: 48 KiB of stages, three workgroups per CU)
    __shared__ __attribute__((aligned(16))) unsigned char smem[PA ? T::STAGE : 2 * T::STAGE];
    __shared__ __attribute__((aligned(16))) unsigned char smem_b[PA ? T::STAGE : 16];
    __shared__ __attribute__((aligned(16))) unsigned char smem_c[PA ? T::STAGE : 16];

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;
    const int wm = wave / T::WAVES_N;
    const int wn = wave % T::WAVES_N;

    int tile_m, tile_n;
    ig_tile_order(p.ntiles_n, tile_m, tile_n);
    const int m0 = tile_m * BM;
    const int n0 = tile_n * BN;
    const int HWm = p.Hm * p.Wm;

    // ---- staging coordinates: thread = (row prow + 64 j, channel quad q4) ----
    const int q4 = tid & 3;
    const int prow = tid >> 2;  // 0..63
    int pb[T::A_PER_T], ys[T::A_PER_T], xs[T::A_PER_T], org0[T::A_PER_T], org1[T::A_PER_T];
#pragma unroll
    for (int j = 0; j < T::A_PER_T; ++j) {
        const int m = m0 + prow + 64 * j;
        if (m < p.M) {
            const int b = m / HWm;
            const int r = m - b * HWm;
            const int y = r / p.Wm;
            const int x = r - y * p.Wm;
            pb[j] = b;
            ys[j] = y * p.sy;
            xs[j] = x * p.sx;
            org0[j] = ((b * p.H0 + ys[j]) * p.W0 + xs[j]) * p.ldc0 + q4 * 4;
            org1[j] = ((b * p.H0 + ys[j]) * p.W0 + xs[j]) * p.ldc1 + q4 * 4;
        } else {
            pb[j] = -1; ys[j] = -(1 << 24); xs[j] = 0; org0[j] = 0; org1[j] = 0;
        }
    }
    const int b_tile = m0 / HWm;
    // f16x3 scale: the static exponent, lowered per image by the producer's bound (tile = 1 image)
    float ascale = 1.f, ainv = 1.f;
    if constexpr (F3) {
        int s_exp = p.a_exp;
        if (UNIB && p.abound) {
            const float bnd = p.abound[b_tile];
            const int e = (int)((__float_as_uint(bnd) >> 23) & 0xffu) - 127;
            if (bnd > 0.f) s_exp = min(s_exp, 13 - e);
            s_exp = max(s_exp, -100);
        }
        ascale = ldexpf(1.0f, s_exp);
        ainv = ldexpf(1.0f, -s_exp);
    }
    // LDS byte offset of this thread's 8-byte A write within a piece plane set
    const int a_wr = (q4 >> 1) * T::APLANE + prow * 16 + (q4 & 1) * 8;

    const __amdgpu_buffer_rsrc_t srd0 = make_srd(p.src0);
    const __amdgpu_buffer_rsrc_t srd1 = make_srd(p.src1 ? p.src1 : p.src0);
    const __amdgpu_buffer_rsrc_t srdw = make_srd(p.w6);
    const __amdgpu_buffer_rsrc_t srdsc = make_srd(PRO ? p.scale : p.src0);
    const __amdgpu_buffer_rsrc_t srdsh = make_srd(PRO ? p.shift : p.src0);

    // Two register stages: the loads of K-step s + 2 are issued before the MFMAs of step s and
    // written to LDS after those of step s + 1, so a load has two K-steps (not one) to land.
    constexpr int NSC = UNIB ? 1 : T::A_PER_T;
    f32x4 ra[2][T::A_PER_T];
    u32x4 rb[2][T::B_PER_T];
    f32x4 rsc[2][NSC], rsh[2][NSC];
    unsigned aval0 = 0u, aval1 = 0u;

    const unsigned wtile =
        (unsigned)tile_n * (unsigned)(p.steps0 * T::BSTEP0 + (p.steps - p.steps0) * T::BSTEP1);
    auto load_w = [&](int st, auto RS) {
        constexpr int rs = decltype(RS)::value;
        const bool s1 = st >= p.steps0;
        const unsigned base = wtile + (s1 ? (unsigned)(p.steps0 * T::BSTEP0 + (st - p.steps0) * T::BSTEP1)
                                          : (unsigned)(st * T::BSTEP0));
        const int items = (s1 ? T::BSTEP1 : T::BSTEP0) / 16;
        const bool live = st < p.steps;
#pragma unroll
        for (int j = 0; j < T::B_PER_T; ++j) {
            const int i = tid + NT * j;
            rb[rs][j] = bload_u4(srdw, live && (j < T::B_FULL || i < items) ? base + (unsigned)i * 16u : OOB);
        }
    };
    // K-step st = (tap, 16-channel chunk), tap-major; taps row-major over the kh x kw grid.  load0 is
    // called for st = 0, 1, 2, ... in order, so the (chunk, tap) position advances incrementally: a
    // division by the runtime chunk / tap counts per step cost ~60 scalar instructions, and the CU's
    // one scalar unit serves all of its waves (SQ_INSTS_SALU was 7.4 per MFMA on the projections)
    int nx_c0 = 0, nx_ky = 0, nx_kx = 0;
    auto load0 = [&](int st, auto RS) {
        constexpr int rs = decltype(RS)::value;
        const int c0 = nx_c0, ky = nx_ky, kx = nx_kx;
        nx_c0 += BK;
        if constexpr (P1) {  // every row of the tile is an in-bounds pixel of one image
            const bool live = st < p.steps;
#pragma unroll
            for (int j = 0; j < T::A_PER_T; ++j)
                ra[rs][j] = bload_f4(srd0, live ? (unsigned)(org0[j] + c0) * 4u : OOB);
            if constexpr (PRO != 0) {
                const unsigned o = live ? (unsigned)(b_tile * p.C0 + c0 + q4 * 4) * 4u : OOB;
                rsc[rs][0] = bload_f4(srdsc, o);
                rsh[rs][0] = bload_f4(srdsh, o);
            }
            load_w(st, RS);
            return;
        }
        if (nx_c0 == p.C0) {
            nx_c0 = 0;
            if (++nx_kx == p.kw) {
                nx_kx = 0;
                ++nx_ky;
            }
        }
        const int dy = p.ty0 + ky * p.tdy, dx = p.tx0 + kx * p.tdx;
        const int tap_off = (dy * p.W0 + dx) * p.ldc0 + c0;
        const bool live = st < p.steps;
        unsigned av = 0;
#pragma unroll
        for (int j = 0; j < T::A_PER_T; ++j) {
            const int iy = ys[j] + dy, ix = xs[j] + dx;
            const bool ok = live && (unsigned)iy < (unsigned)p.H0 && (unsigned)ix < (unsigned)p.W0;
            av |= (ok ? 1u : 0u) << j;
            ra[rs][j] = bload_f4(srd0, ok ? (unsigned)(org0[j] + tap_off) * 4u : OOB);
        }
        if constexpr (rs == 0) aval0 = av; else aval1 = av;
        if constexpr (PRO != 0) {
            const int c = c0 + q4 * 4;
            if constexpr (UNIB) {
                const unsigned o = live ? (unsigned)(b_tile * p.C0 + c) * 4u : OOB;
                rsc[rs][0] = bload_f4(srdsc, o);
                rsh[rs][0] = bload_f4(srdsh, o);
            } else {
#pragma unroll
                for (int j = 0; j < T::A_PER_T; ++j) {
                    const unsigned o = live && pb[j] >= 0 ? (unsigned)(pb[j] * p.C0 + c) * 4u : OOB;
                    rsc[rs][j] = bload_f4(srdsc, o);
                    rsh[rs][j] = bload_f4(srdsh, o);
                }
            }
        }
        load_w(st, RS);
    };
    auto load1 = [&](int st, auto RS) {
        constexpr int rs = decltype(RS)::value;
        const int c1 = (st - p.steps0) * BK;
        const bool live = st < p.steps;
        unsigned av = 0;
#pragma unroll
        for (int j = 0; j < T::A_PER_T; ++j) {
            av |= (pb[j] >= 0 ? 1u : 0u) << j;
            ra[rs][j] = bload_f4(srd1, live && pb[j] >= 0 ? (unsigned)(org1[j] + c1) * 4u : OOB);
        }
        if constexpr (rs == 0) aval0 = av; else aval1 = av;
        load_w(st, RS);
    };
    // Every K-loop iteration issues its loads unconditionally (steps past the end load nothing:
    // all offsets out of range), so the compiler's vmcnt waits see one straight-line issue order
    // and count only the younger stage's loads (a conditional issue made it wait for vmcnt(0)).
    auto load_step = [&](int st, auto RS) {
        if (NPL == 4 || st < p.steps0) load0(st, RS);
        else load1(st, RS);
    };

    // register stage rs (holding K-step st) -> LDS stage buf
    auto store = [&](unsigned char* buf, int st, auto RS) {
        constexpr int rs = decltype(RS)::value;
        const bool pro = st < p.steps0;
#pragma unroll
        for (int j = 0; j < T::A_PER_T; ++j) {
            f32x4 v = ra[rs][j];
            if constexpr (PRO != 0) {
                if (pro) {
                    v = v * rsc[rs][UNIB ? 0 : j] + rsh[rs][UNIB ? 0 : j];
                    if constexpr (PRO == 2) {
                        v.x = silu_fast(v.x); v.y = silu_fast(v.y);
                        v.z = silu_fast(v.z); v.w = silu_fast(v.w);
                    }
                }
            }
            if (!P1 && !(((rs == 0 ? aval0 : aval1) >> j) & 1u)) v = f32x4{0.f, 0.f, 0.f, 0.f};  // padding after the prologue
            unsigned char* d = buf + a_wr + j * 64 * 16;
            if constexpr (F3) v = v * ascale;
            if (F3 && pro) {
                u32x2 a0, a1;
                split2_f16(v, a0, a1);
                *reinterpret_cast<u32x2*>(d) = a0;
                *reinterpret_cast<u32x2*>(d + 2 * T::APLANE) = a1;
            } else if constexpr (NPL == 6) {
                u32x2 a0, a1, a2;
                split3(v, a0, a1, a2);
                *reinterpret_cast<u32x2*>(d) = a0;
                *reinterpret_cast<u32x2*>(d + 2 * T::APLANE) = a1;
                *reinterpret_cast<u32x2*>(d + 4 * T::APLANE) = a2;
            }
        }
        unsigned char* bb = buf + T::ASTAGE;
        const int items = (pro ? T::BSTEP0 : T::BSTEP1) / 16;
#pragma unroll
        for (int j = 0; j < T::B_PER_T; ++j) {
            const int i = tid + NT * j;
            if (j < T::B_FULL || i < items) *reinterpret_cast<u32x4*>(bb + i * 16) = rb[rs][j];
        }
    };

    f32x16 acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

    const int l32 = lane & 31;
    const int half = lane >> 5;
    const int a_rd = half * T::APLANE + (wm * 64 + l32) * 16;
    const int b_rd = T::ASTAGE + half * T::BPLANE + (wn * 64 + l32) * 16;

    auto compute6 = [&](const unsigned char* buf) {
        if constexpr (NPL == 6) {
            u32x4 fa[2][3], fb[2][3];
#pragma unroll
            for (int pc = 0; pc < 3; ++pc) {
#pragma unroll
                for (int mb = 0; mb < 2; ++mb)
                    fa[mb][pc] = *reinterpret_cast<const u32x4*>(buf + a_rd + mb * 32 * 16 + pc * 2 * T::APLANE);
#pragma unroll
                for (int nb = 0; nb < 2; ++nb)
                    fb[nb][pc] = *reinterpret_cast<const u32x4*>(buf + b_rd + nb * 32 * 16 + pc * 2 * T::BPLANE);
            }
#pragma unroll
            for (int mb = 0; mb < 2; ++mb)
#pragma unroll
                for (int nb = 0; nb < 2; ++nb) acc[mb][nb] = mfma_bf16(fa[mb][0], fb[nb][0], acc[mb][nb]);
#pragma unroll
            for (int mb = 0; mb < 2; ++mb)
#pragma unroll
                for (int nb = 0; nb < 2; ++nb) {
                    acc[mb][nb] = mfma_bf16(fa[mb][0], fb[nb][1], acc[mb][nb]);
                    acc[mb][nb] = mfma_bf16(fa[mb][1], fb[nb][0], acc[mb][nb]);
                }
#pragma unroll
            for (int mb = 0; mb < 2; ++mb)
#pragma unroll
                for (int nb = 0; nb < 2; ++nb) {
                    acc[mb][nb] = mfma_bf16(fa[mb][0], fb[nb][2], acc[mb][nb]);
                    acc[mb][nb] = mfma_bf16(fa[mb][1], fb[nb][1], acc[mb][nb]);
                    acc[mb][nb] = mfma_bf16(fa[mb][2], fb[nb][0], acc[mb][nb]);
                }
        }
    };
    auto compute3 = [&](const unsigned char* buf) {
        u32x4 fa[2][2], fb[2][2];
#pragma unroll
        for (int pc = 0; pc < 2; ++pc) {
#pragma unroll
            for (int mb = 0; mb < 2; ++mb)
                fa[mb][pc] = *reinterpret_cast<const u32x4*>(buf + a_rd + mb * 32 * 16 + pc * 2 * T::APLANE);
#pragma unroll
            for (int nb = 0; nb < 2; ++nb)
                fb[nb][pc] = *reinterpret_cast<const u32x4*>(buf + b_rd + nb * 32 * 16 + pc * 2 * T::BPLANE);
        }
#pragma unroll
        for (int mb = 0; mb < 2; ++mb)
#pragma unroll
            for (int nb = 0; nb < 2; ++nb)
                acc[mb][nb] = TR ? mfma_f16(fb[nb][0], fa[mb][0], acc[mb][nb]) : mfma_f16(fa[mb][0], fb[nb][0], acc[mb][nb]);
#pragma unroll
        for (int mb = 0; mb < 2; ++mb)
#pragma unroll
            for (int nb = 0; nb < 2; ++nb) {
                acc[mb][nb] = TR ? mfma_f16c(fb[nb][1], fa[mb][0], acc[mb][nb]) : mfma_f16c(fa[mb][0], fb[nb][1], acc[mb][nb]);
                acc[mb][nb] = TR ? mfma_f16c(fb[nb][0], fa[mb][1], acc[mb][nb]) : mfma_f16c(fa[mb][1], fb[nb][0], acc[mb][nb]);
            }
    };
    // the data of K-step `step` is segment 0 iff step < steps0
    auto compute = [&](const unsigned char* buf, bool seg0) {
        if (F3 && seg0) compute3(buf);
        else compute6(buf);
    };

    if constexpr (PA) {
        // ---- K loop on pre-split operands: LDS-DMA ring of 3 stages (step s in stage s % 3) ----
        const unsigned char* asrc = p.a3 + (long)(m0 / BM) * p.steps * 8192 + tid * 16;
        const unsigned char* bsrc = reinterpret_cast<const unsigned char*>(p.w6) +
                                    (long)tile_n * p.steps * T::BSTEP0 + tid * 16;
        static_assert(T::ASTAGE == 8192 && T::BSTEP0 == 8192, "PA: 128 x 16 A and B steps");
        auto stage = [&](auto S) -> unsigned char* {
            constexpr int SV = decltype(S)::value;
            if constexpr (SV == 0) return smem;
            else if constexpr (SV == 1) return smem_b;
            else return smem_c;
        };
        // The copies are issued as inline assembly, outside the compiler's wait tracking (which
        // cannot tell the ring's stages apart and waits for every copy in flight before each
        // step's barrier, shrinking the copy's window from two steps to one); the ring's own
        // s_waitcnt vmcnt below orders them.  M0 (the LDS base of an LDS-DMA) is written only here.
        auto dma = [&](int st, unsigned char* buf) {
            const unsigned dst = __builtin_amdgcn_readfirstlane(
                (unsigned)(uintptr_t)(__attribute__((address_space(3))) unsigned char*)(buf) + wave * 1024);
            const unsigned char* a0 = asrc + (long)st * 8192;
            const unsigned char* b0 = bsrc + (long)st * T::BSTEP0;
            asm volatile(
                "s_mov_b32 m0, %4\n\t"
                "global_load_lds_dwordx4 %0, off\n\t"
                "s_add_u32 m0, %4, 0x1000\n\t"
                "global_load_lds_dwordx4 %1, off\n\t"
                "s_add_u32 m0, %4, 0x2000\n\t"
                "global_load_lds_dwordx4 %2, off\n\t"
                "s_add_u32 m0, %4, 0x3000\n\t"
                "global_load_lds_dwordx4 %3, off"
                :
                : "v"(a0), "v"(a0 + 4096), "v"(b0), "v"(b0 + 4096), "s"(dst)
                : "memory", "m0");
        };
        const std::integral_constant<int, 0> S0;
        const std::integral_constant<int, 1> S1;
        const std::integral_constant<int, 2> S2;
        auto kstep = [&](auto S, int step) {
            constexpr int SV = decltype(S)::value;
            // this wave's copy of step `step` landed (the younger step + 1 may still fly), then
            // everyone's; and every wave is done with step - 1, whose stage step + 2 reuses
            if (step + 1 < p.steps) asm volatile("s_waitcnt vmcnt(4)\n\ts_barrier" ::: "memory");
            else asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
            if (step + 2 < p.steps) dma(step + 2, stage(std::integral_constant<int, (SV + 2) % 3>{}));
            compute3(stage(S));
        };
        dma(0, smem);
        if (p.steps > 1) dma(1, smem_b);
        int step = 0;
        for (; step + 3 <= p.steps; step += 3) {
            kstep(S0, step);
            kstep(S1, step + 1);
            kstep(S2, step + 2);
        }
        if (step < p.steps) kstep(S0, step);
        if (step + 1 < p.steps) kstep(S1, step + 1);
    } else {
    // ---- K loop: one barrier per step, two steps per iteration (register stages 0 / 1) ----
    const std::integral_constant<int, 0> R0;
    const std::integral_constant<int, 1> R1;
    load_step(0, R0);
    load_step(1, R1);
    store(smem, 0, R0);
    __syncthreads();
    for (int step = 0; step < p.steps; step += 2) {
        load_step(step + 2, R0);
        compute(smem, step < p.steps0);
        if (step + 1 >= p.steps) break;
        store(smem + T::STAGE, step + 1, R1);
        __syncthreads();
        load_step(step + 3, R1);
        compute(smem + T::STAGE, step + 1 < p.steps0);
        if (step + 2 >= p.steps) break;
        store(smem, step + 2, R0);
        __syncthreads();
    }
    }

    // ---- epilogue: pre-split attention projection (wc_conv_igemm_f16x3_qkv, TR) ----
    // acc[mb][nb][r] = output (pixel m-block col l32, channel n-block row); a 32-channel block lies
    // in one (part, head) since D % 32 == 0.  q / k: rows 8j + 4 half + 0..3 are 4 consecutive
    // dims of one 8-dim group -> one 8-byte store per piece, 64 lanes = 512 contiguous bytes.
    // v: 2-byte stores at the pixel's key-order position, 64 contiguous bytes per half-wave.
    if constexpr (TR) {
        if (UNIB && p.qkv3) {
            // the tile's bias and 2^-(sA + sW[n]) through LDS: global loads between the stores
            // would wait for the stores' acks (vmcnt counts both), LDS reads do not
            __syncthreads();  // the last K-step's fragment reads are done
            float* sbias = reinterpret_cast<float*>(smem);
            if (tid < BN) {
                const int n = n0 + tid;
                sbias[tid] = (n < p.N && p.bias) ? p.bias[n] : 0.f;
                sbias[BN + tid] = n < p.N ? (F3 ? p.wsinv[n] * ainv : 1.0f) : 0.f;
            }
            __syncthreads();
            const long img = (long)b_tile * 6 * p.qC * HWm;
            const long plane = (long)p.qD * HWm;  // one piece of one head
#pragma unroll
            for (int nb = 0; nb < 2; ++nb) {
                const int nblk = n0 + wn * 64 + nb * 32;
                if (nblk >= p.N) continue;
                const int part = nblk / p.qC;
                const int c0 = nblk - part * p.qC;
                const int head = c0 / p.qD, d0 = c0 - head * p.qD;
                const float sc = p.qscale[part];
#pragma unroll
                for (int mb = 0; mb < 2; ++mb) {
                    const int pix = m0 - b_tile * HWm + wm * 64 + mb * 32 + l32;
                    if (part < 2) {
                        unsigned short* dst = p.qkv3 + img + (long)((part * (p.qC / p.qD) + head) * 2) * plane +
                                              ((long)(d0 >> 3) * HWm + pix) * 8 + 4 * half;
#pragma unroll
                        for (int j = 0; j < 4; ++j) {
                            f32x4 v;
#pragma unroll
                            for (int e = 0; e < 4; ++e) {
                                const int n = nblk + 8 * j + 4 * half + e;
                                v[e] = (acc[mb][nb][4 * j + e] * sbias[BN + n - n0] + sbias[n - n0]) * sc;
                            }
                            u32x2 ph, pl;
                            split2_f16(v, ph, pl);
                            *reinterpret_cast<u32x2*>(dst + (long)j * HWm * 8) = ph;
                            *reinterpret_cast<u32x2*>(dst + plane + (long)j * HWm * 8) = pl;
                        }
                    } else {
                        const long pos = (pix & ~31) + attn_key_pos(pix & 31);
                        unsigned short* dst = p.qkv3 + img + 4L * p.qC * HWm + (long)(head * 2) * plane + pos;
#pragma unroll
                        for (int r = 0; r < 16; ++r) {
                            const int row = (r & 3) + 8 * (r >> 2) + 4 * half;
                            const int n = nblk + row;
                            const float v = (acc[mb][nb][r] * sbias[BN + n - n0] + sbias[n - n0]) * sc;
                            unsigned short h, l;
                            split2_one(v, h, l);
                            dst[(long)(d0 + row) * HWm] = h;
                            dst[plane + (long)(d0 + row) * HWm] = l;
                        }
                    }
                }
            }
            return;
        }
        // ---- transposed NHWC epilogue (the pointwise projections, UNIB, identity map, N % 32 == 0):
        // a lane holds pixel l32 of each 32-row block and channels 8 j + 4 half .. + 3 of each
        // 32-channel block, so residual loads and output stores are 16-byte vectors (16 per lane
        // instead of 64 scalar ones); per-channel bias and scale through LDS
        if constexpr (UNIB) {
            __syncthreads();  // the last K-step's fragment reads are done
            float* sbias = reinterpret_cast<float*>(smem);
            if (tid < BN) {
                const int n = n0 + tid;
                sbias[tid] = (n < p.N && p.bias) ? p.bias[n] : 0.f;
                sbias[BN + tid] = n < p.N ? (F3 ? p.wsinv[n] * ainv : 1.0f) : 0.f;
            }
            __syncthreads();
            const __amdgpu_buffer_rsrc_t srd_out = make_srd(p.out + (long)b_tile * HWm * p.ldo);
            const __amdgpu_buffer_rsrc_t srd_res = make_srd(p.res ? p.res + (long)b_tile * HWm * p.ldres : p.out);
            const int prow = m0 - b_tile * HWm + wm * 64 + l32;  // pixel of this lane in block mb = 0
            const int ncol = wn * 64 + 4 * half;                  // tile channel of j = 0 in block nb = 0
            const bool nok[2] = {n0 + wn * 64 < p.N, n0 + wn * 64 + 32 < p.N};
            f32x4 rv[2][2][4];
            if (p.res) {
#pragma unroll
                for (int mb = 0; mb < 2; ++mb)
#pragma unroll
                    for (int nb = 0; nb < 2; ++nb)
#pragma unroll
                        for (int j = 0; j < 4; ++j)
                            rv[mb][nb][j] = bload_f4(srd_res, nok[nb] ? (unsigned)((prow + 32 * mb) * p.ldres + n0 + ncol +
                                                                                  32 * nb + 8 * j) * 4u : OOB);
            }
            float vmax = 0.f;
#pragma unroll
            for (int nb = 0; nb < 2; ++nb) {
                if (!nok[nb]) continue;
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const int c = ncol + 32 * nb + 8 * j;
                    const f32x4 badd = *reinterpret_cast<const f32x4*>(sbias + c);
                    const f32x4 bmul = *reinterpret_cast<const f32x4*>(sbias + BN + c);
#pragma unroll
                    for (int mb = 0; mb < 2; ++mb) {
                        f32x4 v = f32x4{acc[mb][nb][4 * j], acc[mb][nb][4 * j + 1], acc[mb][nb][4 * j + 2],
                                        acc[mb][nb][4 * j + 3]} * bmul + badd;
                        if (p.res) v += rv[mb][nb][j];
                        bstore_f4(srd_out, (unsigned)((prow + 32 * mb) * p.ldo + n0 + c) * 4u, v);
                        vmax = fmaxf(vmax, fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w))));
#pragma unroll
                        for (int e = 0; e < 4; ++e) acc[mb][nb][4 * j + e] = v[e];
                    }
                }
            }
            if (p.absmax) block_absmax_atomic(p.absmax, b_tile, vmax);
            if (p.gn_part) {
                GnTile g{p.gn_part, p.gn_ncb, p.gn_sw, (long)b_tile * p.gn_np64 + p.gn_p64 + (m0 - b_tile * HWm) / 64 + wm,
                         (p.gn_c0 + n0 + wn * 64) / 32};
                gn_tile_partials_tr(acc, g, nok[1] ? 2 : (nok[0] ? 1 : 0));
            }
        }
        return;
    }

    // ---- epilogue (as wc_conv.hip) ----
    const int HWo = p.Ho * p.Wo;
    float vmax = 0.f;  // absmax: per image; tiles straddling images take the per-value atomic below
    if constexpr (UNIB) {
        // the tile is one image: 32-bit buffer offsets from that image's base, temb hoisted, and the
        // output position of a 32-row block from one division (32 | Wm) instead of one per element
        const __amdgpu_buffer_rsrc_t srd_out =
            make_srd(p.out + (p.out_nchw ? (long)b_tile * p.N * HWo : (long)b_tile * HWo * p.ldo));
        const __amdgpu_buffer_rsrc_t srd_res = make_srd(p.res ? p.res + (long)b_tile * HWo * p.ldres : p.out);
        // identity output map: every residual value of the tile is loaded before the first store
        // (vmcnt counts stores too, so a load issued after a store waits for that store's ack --
        // one residual load per element between the stores serialised the epilogue on them)
        float rv[2][2][16];
        const bool pre = p.res && p.ident;
        float ebn[2], emul[2];  // per-channel terms of both column blocks, also before any store
#pragma unroll
        for (int nb = 0; nb < 2; ++nb) {
            const int n = n0 + wn * 64 + nb * 32 + l32;
            const bool ok = n < p.N;
            ebn[nb] = (ok && p.bias) ? p.bias[n] : 0.f;
            if (ok && p.temb) ebn[nb] += p.temb[b_tile * p.temb_ld + n];
            emul[nb] = (F3 && ok) ? p.wsinv[n] * ainv : 1.0f;
        }
        if (pre) {
#pragma unroll
            for (int mb = 0; mb < 2; ++mb)
#pragma unroll
                for (int nb = 0; nb < 2; ++nb) {
                    const int rr0 = m0 - b_tile * HWm + wm * 64 + mb * 32;
                    const int n = n0 + wn * 64 + nb * 32 + l32;
#pragma unroll
                    for (int r = 0; r < 16; ++r) {
                        const int row = (r & 3) + 8 * (r >> 2) + 4 * half;
                        rv[mb][nb][r] = bload_f1(srd_res, n < p.N ? (unsigned)((rr0 + row) * p.ldres + n) * 4u : OOB);
                    }
                }
        }
#pragma unroll
        for (int mb = 0; mb < 2; ++mb) {
            const int rr0 = m0 - b_tile * HWm + wm * 64 + mb * 32;  // pixel of row 0 in the image
            const bool fast = (p.Wm & 31) == 0;
            const int my0 = rr0 / p.Wm, mx0 = rr0 - my0 * p.Wm;
#pragma unroll
            for (int nb = 0; nb < 2; ++nb) {
                const int n = n0 + wn * 64 + nb * 32 + l32;
                if (n >= p.N) continue;
                const float bn = ebn[nb], mul = emul[nb];
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int row = (r & 3) + 8 * (r >> 2) + 4 * half;
                    float v = (F3 ? acc[mb][nb][r] * mul : acc[mb][nb][r]) + bn;
                    if constexpr (ACT == WC_ACT_GELU) v = 0.5f * v * (1.0f + erff(v * 0.70710678118654752f));
                    else if constexpr (ACT == WC_ACT_SILU) v = v / (1.0f + __expf(-v));
                    int opix;  // output pixel within the image
                    int oy = 0, ox = 0;
                    if (p.ident) {
                        opix = rr0 + row;
                    } else {
                        int my = my0, mx = mx0 + row;
                        if (!fast) {
                            my = (rr0 + row) / p.Wm;
                            mx = rr0 + row - my * p.Wm;
                        }
                        oy = my * p.osy + p.ooy;
                        ox = mx * p.osx + p.oox;
                        opix = oy * p.Wo + ox;
                    }
                    if (pre) v += rv[mb][nb][r];
                    else if (p.res) v += bload_f1(srd_res, (unsigned)(opix * p.ldres + n) * 4u);
                    if (p.out_nchw) bstore_f1(srd_out, (unsigned)(n * HWo + opix) * 4u, v);
                    else bstore_f1(srd_out, (unsigned)(opix * p.ldo + n) * 4u, v);
                    vmax = fmaxf(vmax, fabsf(v));
                    acc[mb][nb][r] = v;
                }
            }
        }
        if (p.absmax) block_absmax_atomic(p.absmax, b_tile, vmax);  // the tile is image b_tile
        if (p.gn_part) {  // this wave's 64 GEMM rows are one pixel block of image b_tile
            GnTile g{p.gn_part, p.gn_ncb, p.gn_sw,
                     (long)b_tile * p.gn_np64 + p.gn_p64 + (m0 - b_tile * HWm) / 64 + wm,
                     (p.gn_c0 + n0 + wn * 64) / 32};
            gn_tile_partials(acc, g, min(2, max(0, (p.N - n0 - wn * 64) / 32)));
        }
        return;
    }
#pragma unroll
    for (int mb = 0; mb < 2; ++mb) {
        const int mbase = m0 + wm * 64 + mb * 32;
        const int b0 = mbase / HWm;
        const int bnd = (b0 + 1) * HWm;
#pragma unroll
        for (int nb = 0; nb < 2; ++nb) {
            const int n = n0 + wn * 64 + nb * 32 + l32;
            if (n >= p.N) continue;
            const float bn = p.bias ? p.bias[n] : 0.f;
            const float mul = F3 ? p.wsinv[n] * ainv : 1.0f;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int row = (r & 3) + 8 * (r >> 2) + 4 * half;
                const int m = mbase + row;
                if (m >= p.M) continue;
                int b = (HWm >= 32) ? b0 + (m >= bnd ? 1 : 0) : m / HWm;
                float v = (F3 ? acc[mb][nb][r] * mul : acc[mb][nb][r]) + bn;
                if (p.temb) v += p.temb[b * p.temb_ld + n];
                if constexpr (ACT == WC_ACT_GELU) v = 0.5f * v * (1.0f + erff(v * 0.70710678118654752f));
                else if constexpr (ACT == WC_ACT_SILU) v = v / (1.0f + __expf(-v));
                if (p.ident) {
                    if (p.res) v += p.res[(long)m * p.ldres + n];
                    p.out[(long)m * p.ldo + n] = v;
                    if (p.absmax) {
                        if constexpr (UNIB) vmax = fmaxf(vmax, fabsf(v));
                        else atomicMax(reinterpret_cast<unsigned*>(p.absmax) + b, __float_as_uint(fabsf(v)));
                    }
                    acc[mb][nb][r] = v;
                } else {
                    const int rr = m - b * HWm;
                    const int my = rr / p.Wm;
                    const int mx = rr - my * p.Wm;
                    const int oy = my * p.osy + p.ooy;
                    const int ox = mx * p.osx + p.oox;
                    const long pix = (long)(b * p.Ho + oy) * p.Wo + ox;
                    if (p.res) v += p.res[pix * p.ldres + n];
                    if (p.out_nchw)
                        p.out[((long)b * p.N + n) * HWo + (long)oy * p.Wo + ox] = v;
                    else
                        p.out[pix * p.ldo + n] = v;
                    if (p.absmax) {
                        if constexpr (UNIB) vmax = fmaxf(vmax, fabsf(v));
                        else atomicMax(reinterpret_cast<unsigned*>(p.absmax) + b, __float_as_uint(fabsf(v)));
                    }
                    acc[mb][nb][r] = v;
                }
            }
        }
    }
}

template <int BM, int BN, int PRO, bool UNIB, int ACT = WC_ACT_NONE, bool F3 = false>
int launch(const IgDev& d, hipStream_t stream) {
    IgDev p = d;
    const int tiles_m = (p.M + BM - 1) / BM;
    p.ntiles_n = (p.N + BN - 1) / BN;
    dim3 grid(tiles_m * p.ntiles_n);
    const bool p1 = p.kh == 1 && p.kw == 1 && p.ty0 == 0 && p.tx0 == 0 && p.sy == 1 && p.sx == 1 &&
                    p.steps == p.steps0 && p.H0 == p.Hm && p.W0 == p.Wm;
    if constexpr (F3 && UNIB && PRO == 0 && ACT == WC_ACT_NONE && BM == 128 && BN == 128) {
        if (p.a3) {  // pre-split A operand: LDS-DMA pipeline, transposed accumulators (both epilogues)
            WC_SET_NAME("conv_igemm_x6_kernel", {WC_TI(BM), WC_TI(BN), WC_TI(0), WC_TB(true), WC_TI(ACT), WC_TB(true),
                                                 WC_TI(4), WC_TB(true), WC_TB(true), WC_TB(true)});
            hipLaunchKernelGGL((conv_igemm_x6_kernel<BM, BN, 0, true, ACT, true, 4, true, true, true>), grid, dim3(NT),
                               0, stream, p);
            WC_CHECK_LAUNCH();
            return WC_OK;
        }
    }
    if (p.a3) return WC_E_ARG;
    if constexpr (F3 && UNIB && PRO == 1 && ACT == WC_ACT_NONE) {
        if (p.qkv3) {  // pre-split attention projection
            if (p1) {
                WC_SET_NAME("conv_igemm_x6_kernel", {WC_TI(BM), WC_TI(BN), WC_TI(PRO), WC_TB(UNIB), WC_TI(ACT), WC_TB(F3), WC_TI(4), WC_TB(true), WC_TB(true), WC_TB(false)});
                hipLaunchKernelGGL((conv_igemm_x6_kernel<BM, BN, PRO, UNIB, ACT, F3, 4, true, true>), grid, dim3(NT), 0, stream, p);
            } else {
                WC_SET_NAME("conv_igemm_x6_kernel", {WC_TI(BM), WC_TI(BN), WC_TI(PRO), WC_TB(UNIB), WC_TI(ACT), WC_TB(F3), WC_TI(4), WC_TB(true), WC_TB(false), WC_TB(false)});
                hipLaunchKernelGGL((conv_igemm_x6_kernel<BM, BN, PRO, UNIB, ACT, F3, 4, true>), grid, dim3(NT), 0, stream, p);
            }
            WC_CHECK_LAUNCH();
            return WC_OK;
        }
    }
    if (p.qkv3) return WC_E_ARG;
    if constexpr (F3 && UNIB && PRO <= 1 && ACT == WC_ACT_NONE && BN == 128) {
        if (p1 && p.ident && p.N % 32 == 0 && p.ldo % 4 == 0 && (reinterpret_cast<uintptr_t>(p.out) & 15) == 0 &&
            (!p.res || (p.ldres % 4 == 0 && (reinterpret_cast<uintptr_t>(p.res) & 15) == 0))) {
            // the projections: transposed accumulators for the vector epilogue
            WC_SET_NAME("conv_igemm_x6_kernel", {WC_TI(BM), WC_TI(BN), WC_TI(PRO), WC_TB(UNIB), WC_TI(ACT), WC_TB(F3), WC_TI(4), WC_TB(true), WC_TB(true), WC_TB(false)});
            hipLaunchKernelGGL((conv_igemm_x6_kernel<BM, BN, PRO, UNIB, ACT, F3, 4, true, true>), grid, dim3(NT), 0, stream, p);
            WC_CHECK_LAUNCH();
            return WC_OK;
        }
    }
    if (F3 && p.steps == p.steps0) {  // f16x3 segment 0 only: 4-plane LDS stages
        WC_SET_NAME("conv_igemm_x6_kernel", {WC_TI(BM), WC_TI(BN), WC_TI(PRO), WC_TB(UNIB), WC_TI(ACT), WC_TB(F3),
                                             WC_TI(F3 ? 4 : 6), WC_TB(false), WC_TB(false), WC_TB(false)});
        hipLaunchKernelGGL((conv_igemm_x6_kernel<BM, BN, PRO, UNIB, ACT, F3, F3 ? 4 : 6>), grid, dim3(NT), 0, stream, p);
    } else {
        WC_SET_NAME("conv_igemm_x6_kernel", {WC_TI(BM), WC_TI(BN), WC_TI(PRO), WC_TB(UNIB), WC_TI(ACT), WC_TB(F3), WC_TI(6),
                                             WC_TB(false), WC_TB(false), WC_TB(false)});
        hipLaunchKernelGGL((conv_igemm_x6_kernel<BM, BN, PRO, UNIB, ACT, F3, 6>), grid, dim3(NT), 0, stream, p);
    }
    WC_CHECK_LAUNCH();
    return WC_OK;
}

template <int BM, int BN>
int dispatch(const IgDev& d, int pro, int act, bool f3, hipStream_t s) {
    const bool unib = (d.Hm * d.Wm) % BM == 0;
    if (d.gn_part && !unib) return WC_E_SHAPE;  // tile partials need tiles inside one image
    if (f3) {  // f16x3: no epilogue activation instantiated
        if (act != WC_ACT_NONE) return WC_E_ARG;
        switch (pro * 2 + (unib ? 1 : 0)) {
            case 0: return launch<BM, BN, 0, false, WC_ACT_NONE, true>(d, s);
            case 1: return launch<BM, BN, 0, true, WC_ACT_NONE, true>(d, s);
            case 2: return launch<BM, BN, 1, false, WC_ACT_NONE, true>(d, s);
            case 3: return launch<BM, BN, 1, true, WC_ACT_NONE, true>(d, s);
            case 4: return launch<BM, BN, 2, false, WC_ACT_NONE, true>(d, s);
            default: return launch<BM, BN, 2, true, WC_ACT_NONE, true>(d, s);
        }
    }
    if (act != WC_ACT_NONE) {  // activations are instantiated for a raw segment 0 only
        if (pro != 0) return WC_E_ARG;
        if (act == WC_ACT_GELU)
            return unib ? launch<BM, BN, 0, true, WC_ACT_GELU>(d, s) : launch<BM, BN, 0, false, WC_ACT_GELU>(d, s);
        return unib ? launch<BM, BN, 0, true, WC_ACT_SILU>(d, s) : launch<BM, BN, 0, false, WC_ACT_SILU>(d, s);
    }
    switch (pro * 2 + (unib ? 1 : 0)) {
        case 0: return launch<BM, BN, 0, false>(d, s);
        case 1: return launch<BM, BN, 0, true>(d, s);
        case 2: return launch<BM, BN, 1, false>(d, s);
        case 3: return launch<BM, BN, 1, true>(d, s);
        case 4: return launch<BM, BN, 2, false>(d, s);
        default: return launch<BM, BN, 2, true>(d, s);
    }
}

}  // namespace

namespace {

// Shared host validation (wc_conv_igemm's contract with C % 16); fills d.
int prepare(const wc_conv_args* a, const void* w6, IgDev& d, long& k) {
    if (!a || !w6 || !a->out) return WC_E_ARG;
    if (a->nseg < 1 || a->nseg > 2) return WC_E_ARG;
    if (a->act < WC_ACT_NONE || a->act > WC_ACT_SILU) return WC_E_ARG;
    const wc_conv_seg& s0 = a->seg[0];
    if (!s0.src) return WC_E_ARG;
    if ((s0.scale == nullptr) != (s0.shift == nullptr)) return WC_E_ARG;
    if (s0.C <= 0 || s0.C % BK || s0.ldc % 4 || (reinterpret_cast<uintptr_t>(s0.src) & 15)) return WC_E_SHAPE;
    if (s0.ntaps < 1 || s0.ntaps > WC_MAX_TAPS || s0.kbase != 0) return WC_E_SHAPE;
    if ((long)a->B * s0.H * s0.W * s0.ldc * 4 >= (1L << 31)) return WC_E_SHAPE;  // 2 GiB SRD range
    int kw = 1;
    while (kw < s0.ntaps && s0.dy[kw] == s0.dy[0]) ++kw;
    if (s0.ntaps % kw != 0) return WC_E_SHAPE;
    const int kh = s0.ntaps / kw;
    const int tdx = kw > 1 ? s0.dx[1] - s0.dx[0] : 0;
    const int tdy = kh > 1 ? s0.dy[kw] - s0.dy[0] : 0;
    for (int t = 0; t < s0.ntaps; ++t)
        if (s0.dy[t] != s0.dy[0] + (t / kw) * tdy || s0.dx[t] != s0.dx[0] + (t % kw) * tdx) return WC_E_SHAPE;
    d = IgDev{};
    d.src0 = s0.src; d.C0 = s0.C; d.ldc0 = s0.ldc; d.H0 = s0.H; d.W0 = s0.W; d.sy = s0.sy; d.sx = s0.sx;
    d.kh = kh; d.kw = kw; d.ty0 = s0.dy[0]; d.tdy = tdy; d.tx0 = s0.dx[0]; d.tdx = tdx;
    d.scale = s0.scale; d.shift = s0.shift;
    k = (long)s0.ntaps * s0.C;
    if (a->nseg == 2) {
        const wc_conv_seg& s1 = a->seg[1];
        if (!s1.src || s1.scale) return WC_E_ARG;
        if (s1.C <= 0 || s1.C % BK || s1.ldc % 4 || (reinterpret_cast<uintptr_t>(s1.src) & 15)) return WC_E_SHAPE;
        if (s1.ntaps != 1 || s1.dy[0] != 0 || s1.dx[0] != 0) return WC_E_SHAPE;
        if (s1.H != s0.H || s1.W != s0.W || s1.sy != s0.sy || s1.sx != s0.sx) return WC_E_SHAPE;
        if (s1.kbase != k) return WC_E_SHAPE;
        if ((long)a->B * s1.H * s1.W * s1.ldc * 4 >= (1L << 31)) return WC_E_SHAPE;
        d.src1 = s1.src; d.C1 = s1.C; d.ldc1 = s1.ldc;
        k += s1.C;
    }
    const long M = (long)a->B * a->Hm * a->Wm;
    if (M <= 0 || M > (1L << 30) || a->N <= 0) return WC_E_SHAPE;
    if (reinterpret_cast<uintptr_t>(w6) & 15) return WC_E_SHAPE;
    d.B = a->B; d.Hm = a->Hm; d.Wm = a->Wm; d.N = a->N; d.M = (int)M;
    d.w6 = w6; d.bias = a->bias; d.temb = a->temb; d.temb_ld = a->temb_ld;
    d.res = a->res; d.ldres = a->ldres; d.out = a->out; d.ldo = a->ldo;
    d.Ho = a->Ho; d.Wo = a->Wo; d.osy = a->osy; d.osx = a->osx; d.ooy = a->ooy; d.oox = a->oox;
    d.out_nchw = a->out_nchw;
    d.ident = !a->out_nchw && a->osy == 1 && a->osx == 1 && a->ooy == 0 && a->oox == 0 &&
              a->Ho == a->Hm && a->Wo == a->Wm;
    // the single-image-tile epilogue addresses one image of the output / residual with 32-bit offsets
    const long hwo = (long)a->Ho * a->Wo;
    if ((a->out_nchw ? hwo * a->N : hwo * a->ldo) * 4 >= (1L << 31) || (a->res && hwo * a->ldres * 4 >= (1L << 31)))
        return WC_E_SHAPE;
    d.steps0 = (int)((long)s0.ntaps * s0.C / BK);
    d.cpt = s0.C / BK;
    d.steps = (int)(k / BK);
    d.wsinv = nullptr; d.abound = nullptr; d.a_exp = 0;
    d.qkv3 = nullptr; d.qC = d.qD = 0;
    d.absmax = a->absmax_out;
    d.gn_part = a->gn_part;
    if (a->gn_part) {  // N whole 32-channel blocks at a 32-aligned offset, NHWC output
        const int sw = a->gn_sw;
        if ((sw != 4 && sw != 8 && sw != 16 && sw != 32) || a->N % 32 || a->gn_c0 % 32 || a->gn_c0 < 0 ||
            a->gn_c0 + a->N > a->gn_ncb * 32 || a->out_nchw || (a->Hm * a->Wm) % 64 || a->gn_p64 < 0 ||
            a->gn_p64 + a->Hm * a->Wm / 64 > a->gn_np64)
            return WC_E_SHAPE;
        d.gn_ncb = a->gn_ncb; d.gn_sw = sw; d.gn_c0 = a->gn_c0; d.gn_p64 = a->gn_p64; d.gn_np64 = a->gn_np64;
    }
    return WC_OK;
}

}  // namespace

extern "C" int wc_conv_igemm_x6(const wc_conv_args* a, const void* w6, int64_t w6_bytes, void* stream) {
    IgDev d;
    long k;
    const int st = prepare(a, w6, d, k);
    if (st != WC_OK) return st;
    const int BN = wc_conv3x3_x6_tile_n(a->N);
    const long ntn = (a->N + BN - 1) / BN;
    if (w6_bytes != ntn * (k / BK) * (long)BN * 96 || w6_bytes >= (1L << 31)) return WC_E_SHAPE;
    const int pro = a->seg[0].scale ? (a->seg[0].silu ? 2 : 1) : 0;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    if (BN == 64) return dispatch<256, 64>(d, pro, a->act, false, s);
    return dispatch<128, 128>(d, pro, a->act, false, s);
}

extern "C" int wc_conv_igemm_f16x3_qkv(const wc_conv_args* a, const void* w3, int64_t w3_bytes, int a_exp,
                                       const float* w_inv_scale, void* qkv3, int C, int heads, const int* exps,
                                       void* stream) {
    if (!a || !qkv3 || !exps || !w_inv_scale) return WC_E_ARG;
    if (C <= 0 || heads <= 0 || C % heads || (C / heads) % 32 || a->N != 3 * C) return WC_E_SHAPE;
    if (a->nseg != 1 || a->res || a->temb || a->absmax_out || a->gn_part || a->out_nchw || a->act) return WC_E_ARG;
    if (a->seg[0].ntaps != 1 || a->seg[0].dy[0] || a->seg[0].dx[0] || a->seg[0].sy != 1 || a->seg[0].sx != 1)
        return WC_E_SHAPE;
    if ((a->Hm * a->Wm) % 128 || (reinterpret_cast<uintptr_t>(qkv3) & 15)) return WC_E_SHAPE;
    if (a_exp < -60 || a_exp > 60) return WC_E_ARG;
    for (int i = 0; i < 3; ++i)
        if (exps[i] < -60 || exps[i] > 60) return WC_E_ARG;
    IgDev d;
    long k;
    wc_conv_args aa = *a;
    aa.out = reinterpret_cast<float*>(qkv3);  // unused by the split epilogue; keeps prepare's checks uniform
    aa.ldo = a->N;
    aa.Ho = a->Hm; aa.Wo = a->Wm; aa.osy = aa.osx = 1; aa.ooy = aa.oox = 0;
    const int st = prepare(&aa, w3, d, k);
    if (st != WC_OK) return st;
    const int BN = wc_conv3x3_x6_tile_n(a->N);
    if (BN != 128) return WC_E_SHAPE;
    const long ntn = (a->N + BN - 1) / BN;
    if (w3_bytes != ntn * (long)d.steps0 * BN * 64 || w3_bytes >= (1L << 31)) return WC_E_SHAPE;
    d.a_exp = a_exp;
    d.wsinv = w_inv_scale;
    d.qkv3 = reinterpret_cast<unsigned short*>(qkv3);
    d.qC = C;
    d.qD = C / heads;
    for (int i = 0; i < 3; ++i) d.qscale[i] = ldexpf(1.0f, exps[i]);
    const int pro = a->seg[0].scale ? (a->seg[0].silu ? 2 : 1) : 0;
    return dispatch<128, 128>(d, pro, WC_ACT_NONE, true, reinterpret_cast<hipStream_t>(stream));
}

extern "C" int wc_conv_igemm_f16x3(const wc_conv_args* a, const void* w3, int64_t w3_bytes, int a_exp,
                                   const float* w_inv_scale, const float* a_bound, void* stream) {
    IgDev d;
    long k;
    const int st = prepare(a, w3, d, k);
    if (st != WC_OK) return st;
    if (!w_inv_scale || a_exp < -60 || a_exp > 60) return WC_E_ARG;
    const int BN = wc_conv3x3_x6_tile_n(a->N);
    const long ntn = (a->N + BN - 1) / BN;
    const long s1 = d.steps - d.steps0;
    if (w3_bytes != ntn * ((long)d.steps0 * BN * 64 + s1 * BN * 96) || w3_bytes >= (1L << 31)) return WC_E_SHAPE;
    d.a_exp = a_exp;
    d.wsinv = w_inv_scale;
    d.abound = a_bound;
    const int BM = BN == 64 ? 256 : 128;
    if (a_bound && (d.Hm * d.Wm) % BM != 0) return WC_E_SHAPE;  // per-image scale needs 1-image tiles
    const int pro = a->seg[0].scale ? (a->seg[0].silu ? 2 : 1) : 0;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    if (BN == 64) return dispatch<256, 64>(d, pro, a->act, true, s);
    return dispatch<128, 128>(d, pro, a->act, true, s);
}

// ---- pointwise projections on a pre-split A operand (PA) ----

namespace {

// a3[mt][ks][piece][k-half][row 128][8 x fp16] from the fp32 rows of an NHWC view: optional GroupNorm
// affine (+ SiLU), x 2^a_exp, two-piece round-to-nearest fp16 split (wcx6::split2_f16).  A wave owns
// 64 rows x 32 channels in 8 rounds of 8 rows: lane = (row 8, channel quad 8), so each load instruction
// reads 8 whole 128-byte row segments (a lane per row read 64 separate lines per instruction: 0.56 of
// HBM); each lane splits its quad and stores the two 8-byte halves of its fragments, so for a fixed
// (16-channel step, k-half, piece) the 8 rows' 16-byte fragments land as one contiguous 128 bytes.
__global__ __launch_bounds__(256) void split_tiled_kernel(const float* __restrict__ src, int ldc, int HW, int K,
                                                          const float* __restrict__ scale,
                                                          const float* __restrict__ shift, int silu, float ascale,
                                                          unsigned char* __restrict__ a3) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int g32 = blockIdx.y * 4 + wave;
    if (g32 * 32 >= K) return;
    const int row0 = blockIdx.x * 64;
    const int b = row0 / HW;  // HW % 128 == 0: the 64 rows are one image's
    const int q = lane & 7, rl = lane >> 3;
    const int c = g32 * 32 + 4 * q;
    f32x4 v[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = *reinterpret_cast<const f32x4*>(src + (long)(row0 + 8 * i + rl) * ldc + c);
    if (scale) {
        const f32x4 sc = *reinterpret_cast<const f32x4*>(scale + (long)b * K + c);
        const f32x4 sh = *reinterpret_cast<const f32x4*>(shift + (long)b * K + c);
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            v[i] = v[i] * sc + sh;
            if (silu) {
                v[i].x = silu_fast(v[i].x); v[i].y = silu_fast(v[i].y);
                v[i].z = silu_fast(v[i].z); v[i].w = silu_fast(v[i].w);
            }
        }
    }
    // quad q: channels 4q .. 4q + 3 of the 32 = step 2 g32 + q / 4, k-half (q / 2) % 2, 8-byte half q % 2
    const int mt = row0 >> 7, KS = K / 16;
    const long step = (long)mt * KS + 2 * g32 + (q >> 2);
    unsigned char* base = a3 + ((step * 2 * 2 + ((q >> 1) & 1)) * 128 + (row0 & 127) + rl) * 16 + (q & 1) * 8;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        u32x2 ph, pl;
        split2_f16(v[i] * ascale, ph, pl);
        *reinterpret_cast<u32x2*>(base + i * 8 * 16) = ph;
        *reinterpret_cast<u32x2*>(base + i * 8 * 16 + 2 * 128 * 16) = pl;
    }
}

// The pre-split projection GEMM, H = 64-row blocks per wave: H = 2 (proj_pa256_kernel) = 256 x 128
// tiles, each wave 128 pixels x 64 channels (4 x 2 transposed 32x32 accumulators, 24 MFMAs per
// K-step), a 3-stage LDS-DMA ring of 24 KiB stages (the A rows of two consecutive 128-row a3 tiles +
// the B step), two workgroups per CU.  WR (H = 1, proj_pa_wr_kernel: 128 x 128 tiles): the B
// fragments go from L2 straight into registers two steps ahead (three register sets, as the halo
// conv's weights) and only A rides the LDS-DMA ring (8 KiB stages): half the LDS traffic per MFMA.
// Same fragments, products and per-accumulator order as conv_igemm_x6_kernel<128, 128, ..., PA>
// (transposed accumulation): the results are bit-identical to it (tests/test_x6.py).  QKV: the
// pre-split attention epilogue.
// DA (with WR): the A fragments also go from the pre-split rows straight into registers two steps
// ahead: no LDS and no barrier in the K loop (each wave streams its own operands; the two waves
// sharing A rows or B columns read them twice, through the CU's L1).
template <bool QKV, int H, bool WR, bool DA = false>
__global__ __launch_bounds__(NT, H == 2 || DA ? 2 : 3) void proj_pa_kernel(IgDev p) {
    static_assert((H == 2 && !WR && !DA) || (H == 1 && WR), "the instantiated forms");
    constexpr int BM = 128 * H, BN = 128;
    constexpr int APLANE = 128 * 16, BPLANE = BN * 16;  // one (piece, k-half) plane of a 128-row half / of B
    constexpr int AHALF = 4 * APLANE;                    // 8 KiB: one a3 step of 128 rows
    constexpr int STAGE = H * AHALF + (WR ? 0 : 4 * BPLANE);
    constexpr int NDMA = 2 * H + (WR ? 0 : 2);           // LDS-DMA wave-instructions per step
    __shared__ __attribute__((aligned(16))) unsigned char st0[STAGE];
    __shared__ __attribute__((aligned(16))) unsigned char st1[STAGE];
    __shared__ __attribute__((aligned(16))) unsigned char st2[STAGE];
    __shared__ __attribute__((aligned(16))) float sbias[2 * BN];

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;
    const int wm = wave >> 1, wn = wave & 1;
    int tile_m, tile_n;
    ig_tile_order(p.ntiles_n, tile_m, tile_n);
    const int m0 = tile_m * BM;
    const int n0 = tile_n * BN;
    const int HWm = p.Hm * p.Wm;
    const int b_tile = m0 / HWm;
    const float ainv = ldexpf(1.0f, -p.a_exp);
    const int steps = p.steps;

    const unsigned char* asrc0 = p.a3 + (long)(H * tile_m) * steps * AHALF + tid * 16;
    const unsigned char* asrc1 = asrc0 + (long)steps * AHALF;
    const unsigned char* bsrc = reinterpret_cast<const unsigned char*>(p.w6) + (long)tile_n * steps * (4 * BPLANE) + tid * 16;
    auto stage = [&](auto S) -> unsigned char* {
        constexpr int SV = decltype(S)::value;
        if constexpr (SV == 0) return st0;
        else if constexpr (SV == 1) return st1;
        else return st2;
    };
    // LDS-DMA wave-instructions (1 KiB each) per wave: the A halves, then (not WR) B; inline
    // assembly outside the compiler's wait tracking, ordered by the ring's own s_waitcnt (as the
    // 128 x 128 form)
    auto dma1 = [&](unsigned dst, const unsigned char* src) {
        asm volatile("s_mov_b32 m0, %1\n\tglobal_load_lds_dwordx4 %0, off" : : "v"(src), "s"(dst) : "memory", "m0");
    };
    auto dma = [&](int st, unsigned char* buf) {
        const unsigned dst = __builtin_amdgcn_readfirstlane(
            (unsigned)(uintptr_t)(__attribute__((address_space(3))) unsigned char*)(buf) + wave * 1024);
        const unsigned char* a0 = asrc0 + (long)st * AHALF;
        dma1(dst, a0);
        dma1(dst + 0x1000, a0 + 4096);
        if constexpr (H == 2) {
            const unsigned char* a1 = asrc1 + (long)st * AHALF;
            dma1(dst + 0x2000, a1);
            dma1(dst + 0x3000, a1 + 4096);
        }
        if constexpr (!WR) {
            const unsigned char* b0 = bsrc + (long)st * (4 * BPLANE);
            dma1(dst + H * 0x2000, b0);
            dma1(dst + H * 0x2000 + 0x1000, b0 + 4096);
        }
    };
    // WR: B fragments of step st into register set `set` (steps past the end re-read the last one:
    // every load issued unconditionally keeps the compiler's vmcnt counts straight)
    u32x4 wreg[WR ? 3 : 1][2][2];
    const __amdgpu_buffer_rsrc_t srdw = make_srd(p.w6);
    const unsigned wlane = (unsigned)((lane >> 5) * BPLANE + (wn * 64 + (lane & 31)) * 16);
    const int wtile = tile_n * steps * (4 * BPLANE);
    u32x4 areg[DA ? 3 : 1][2][2];  // DA: [set][mb][piece]
    const __amdgpu_buffer_rsrc_t srda = make_srd(p.a3 + (long)tile_m * steps * AHALF);
    const unsigned alane = (unsigned)((lane >> 5) * APLANE + (wm * 64 + (lane & 31)) * 16);
    auto load_a = [&](int set, int st) {
        if constexpr (DA) {
            const int off = (st < steps ? st : steps - 1) * AHALF;
#pragma unroll
            for (int mb = 0; mb < 2; ++mb)
#pragma unroll
                for (int pc = 0; pc < 2; ++pc)
                    areg[set][mb][pc] = bload_u4s(srda, alane + (unsigned)(mb * 32 * 16 + pc * 2 * APLANE), off);
        }
    };
    auto load_b = [&](int set, int st) {
        if constexpr (WR) {
            const int off = wtile + (st < steps ? st : steps - 1) * (4 * BPLANE);
#pragma unroll
            for (int nb = 0; nb < 2; ++nb)
#pragma unroll
                for (int pc = 0; pc < 2; ++pc)
                    wreg[set][nb][pc] = bload_u4s(srdw, wlane + (unsigned)(nb * 32 * 16 + pc * 2 * BPLANE), off);
        }
    };

    f32x16 acc[H][2][2];  // [64-row block of the wave][mb in the block][nb]; transposed (lanes = pixels)
#pragma unroll
    for (int h = 0; h < H; ++h)
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j)
#pragma unroll
                for (int r = 0; r < 16; ++r) acc[h][i][j][r] = 0.f;
    const int l32 = lane & 31;
    const int half = lane >> 5;
    // row r0 = wm * 64 H + 32 mb of the tile: A half r0 / 128, row r0 % 128 of it
    const int a_rd = ((wm * 64 * H) >> 7) * AHALF + ((wm * 64 * H) & 127) * 16 + half * APLANE + l32 * 16;
    const int b_rd = H * AHALF + half * BPLANE + (wn * 64 + l32) * 16;
    auto compute = [&](const unsigned char* buf, int set) {
        u32x4 fa[2 * H][2], fb[2][2];
#pragma unroll
        for (int pc = 0; pc < 2; ++pc) {
#pragma unroll
            for (int mb = 0; mb < 2 * H; ++mb) {
                if constexpr (DA) fa[mb][pc] = areg[set][mb & 1][pc];
                else fa[mb][pc] = *reinterpret_cast<const u32x4*>(buf + a_rd + mb * 32 * 16 + pc * 2 * APLANE);
            }
            if constexpr (!WR) {
#pragma unroll
                for (int nb = 0; nb < 2; ++nb)
                    fb[nb][pc] = *reinterpret_cast<const u32x4*>(buf + b_rd + nb * 32 * 16 + pc * 2 * BPLANE);
            } else {
#pragma unroll
                for (int nb = 0; nb < 2; ++nb) fb[nb][pc] = wreg[set][nb][pc];
            }
        }
#pragma unroll
        for (int mb = 0; mb < 2 * H; ++mb)
#pragma unroll
            for (int nb = 0; nb < 2; ++nb)
                acc[mb >> 1][mb & 1][nb] = mfma_f16(fb[nb][0], fa[mb][0], acc[mb >> 1][mb & 1][nb]);
#pragma unroll
        for (int mb = 0; mb < 2 * H; ++mb)
#pragma unroll
            for (int nb = 0; nb < 2; ++nb) {
                f32x16& a = acc[mb >> 1][mb & 1][nb];
                a = mfma_f16c(fb[nb][1], fa[mb][0], a);
                a = mfma_f16c(fb[nb][0], fa[mb][1], a);
            }
    };
    const std::integral_constant<int, 0> S0;
    const std::integral_constant<int, 1> S1;
    const std::integral_constant<int, 2> S2;
    // Step s (stage and B set s % 3): issue B(s + 2) and the copy of s + 2, then wait for this wave's
    // copy of s (younger ops may fly: not WR, the copy of s + 1; WR, B(s + 1) and the copy of s + 1),
    // barrier (everyone's copy landed; everyone is done with s - 1, whose stage s + 2 reuses).  WR:
    // the compiler's own wait for B(s) counts only the B loads after it (8), which leaves the copy
    // of s + 1 in flight (in-order vmcnt: B(s + 1) and older are complete by then).
    auto kstep = [&](auto S, int step) {
        constexpr int SV = decltype(S)::value;
        if constexpr (WR) {
            if (step + 1 < steps) asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" : : "n"(4 + NDMA) : "memory");
            else asm volatile("s_waitcnt vmcnt(4)\n\ts_barrier" ::: "memory");
            load_b((SV + 2) % 3, step + 2);
        } else {
            if (step + 1 < steps) asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" : : "n"(NDMA) : "memory");
            else asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
        }
        if (step + 2 < steps) dma(step + 2, stage(std::integral_constant<int, (SV + 2) % 3>{}));
        compute(stage(S), SV);
    };
    int step = 0;
    if constexpr (DA) {
        auto kstep_d = [&](auto S) {
            constexpr int SV = decltype(S)::value;
            load_a((SV + 2) % 3, step + 2);
            load_b((SV + 2) % 3, step + 2);
            // keep the loads at the head of their step (the scheduler otherwise sinks them behind the
            // MFMAs, leaving one step of cover and a vmcnt(0) per iteration)
            __builtin_amdgcn_sched_barrier(0);
            compute(st0, SV);
            __builtin_amdgcn_sched_barrier(0);
        };
        load_a(0, 0);
        load_b(0, 0);
        load_a(1, 1);
        load_b(1, 1);
        for (; step + 3 <= steps; step += 3) {
            kstep_d(S0);
            ++step;
            kstep_d(S1);
            ++step;
            kstep_d(S2);
            step -= 2;
        }
        if (step < steps) kstep_d(S0);
        ++step;
        if (step < steps) kstep_d(S1);
    } else {
    load_b(0, 0);
    dma(0, st0);
    load_b(1, 1);
    if (steps > 1) dma(1, st1);
    for (; step + 3 <= steps; step += 3) {
        kstep(S0, step);
        kstep(S1, step + 1);
        kstep(S2, step + 2);
    }
    if (step < steps) kstep(S0, step);
    if (step + 1 < steps) kstep(S1, step + 1);
    }

    // per-channel bias and 2^-(sA + sW[n]) of the tile through LDS (global loads between the
    // epilogue's stores would wait for their acks: vmcnt counts both)
    if (tid < BN) {
        const int n = n0 + tid;
        sbias[tid] = p.bias ? p.bias[n] : 0.f;
        sbias[BN + tid] = p.wsinv[n] * ainv;
    }
    __syncthreads();
    const int prow0 = m0 - b_tile * HWm + wm * 64 * H + l32;  // pixel of this lane in block mb = 0
    if constexpr (QKV) {
        // as conv_igemm_x6_kernel's pre-split qkv epilogue, over 4 row blocks
        const long img = (long)b_tile * 6 * p.qC * HWm;
        const long plane = (long)p.qD * HWm;
#pragma unroll
        for (int nb = 0; nb < 2; ++nb) {
            const int nblk = n0 + wn * 64 + nb * 32;
            const int part = nblk / p.qC;
            const int c0 = nblk - part * p.qC;
            const int head = c0 / p.qD, d0 = c0 - head * p.qD;
            const float sc = p.qscale[part];
#pragma unroll
            for (int mb = 0; mb < 2 * H; ++mb) {
                const f32x16& a = acc[mb >> 1][mb & 1][nb];
                const int pix = prow0 + mb * 32;
                if (part < 2) {
                    unsigned short* dst = p.qkv3 + img + (long)((part * (p.qC / p.qD) + head) * 2) * plane +
                                          ((long)(d0 >> 3) * HWm + pix) * 8 + 4 * half;
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        f32x4 v;
#pragma unroll
                        for (int e = 0; e < 4; ++e) {
                            const int n = nblk + 8 * j + 4 * half + e;
                            v[e] = (a[4 * j + e] * sbias[BN + n - n0] + sbias[n - n0]) * sc;
                        }
                        u32x2 ph, pl;
                        split2_f16(v, ph, pl);
                        *reinterpret_cast<u32x2*>(dst + (long)j * HWm * 8) = ph;
                        *reinterpret_cast<u32x2*>(dst + plane + (long)j * HWm * 8) = pl;
                    }
                } else {
                    const long pos = (pix & ~31) + attn_key_pos(pix & 31);
                    unsigned short* dst = p.qkv3 + img + 4L * p.qC * HWm + (long)(head * 2) * plane + pos;
#pragma unroll
                    for (int r = 0; r < 16; ++r) {
                        const int row = (r & 3) + 8 * (r >> 2) + 4 * half;
                        const int n = nblk + row;
                        const float v = (a[r] * sbias[BN + n - n0] + sbias[n - n0]) * sc;
                        unsigned short h, l;
                        split2_one(v, h, l);
                        dst[(long)(d0 + row) * HWm] = h;
                        dst[plane + (long)(d0 + row) * HWm] = l;
                    }
                }
            }
        }
    } else {
        // as conv_igemm_x6_kernel's transposed NHWC epilogue: 16-byte residual loads (all before the
        // first store) and stores, per-image absmax, GroupNorm tile partials per 64-row pair
        const __amdgpu_buffer_rsrc_t srd_out = make_srd(p.out + (long)b_tile * HWm * p.ldo);
        const __amdgpu_buffer_rsrc_t srd_res = make_srd(p.res ? p.res + (long)b_tile * HWm * p.ldres : p.out);
        const int ncol = wn * 64 + 4 * half;
        float vmax = 0.f;
        f32x4 rv[H][2][2][4];
        if (p.res) {
#pragma unroll
            for (int h = 0; h < H; ++h)
#pragma unroll
                for (int i = 0; i < 2; ++i)
#pragma unroll
                    for (int nb = 0; nb < 2; ++nb)
#pragma unroll
                        for (int j = 0; j < 4; ++j)
                            rv[h][i][nb][j] = bload_f4(srd_res, (unsigned)((prow0 + 32 * (2 * h + i)) * p.ldres + n0 + ncol +
                                                                          32 * nb + 8 * j) * 4u);
        }
#pragma unroll
        for (int h = 0; h < H; ++h) {
#pragma unroll
            for (int nb = 0; nb < 2; ++nb) {
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const int c = ncol + 32 * nb + 8 * j;
                    const f32x4 badd = *reinterpret_cast<const f32x4*>(sbias + c);
                    const f32x4 bmul = *reinterpret_cast<const f32x4*>(sbias + BN + c);
#pragma unroll
                    for (int i = 0; i < 2; ++i) {
                        f32x16& a = acc[h][i][nb];
                        f32x4 v = f32x4{a[4 * j], a[4 * j + 1], a[4 * j + 2], a[4 * j + 3]} * bmul + badd;
                        if (p.res) v += rv[h][i][nb][j];
                        bstore_f4(srd_out, (unsigned)((prow0 + 32 * (2 * h + i)) * p.ldo + n0 + c) * 4u, v);
                        vmax = fmaxf(vmax, fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w))));
#pragma unroll
                        for (int e = 0; e < 4; ++e) a[4 * j + e] = v[e];
                    }
                }
            }
        }
        if (p.absmax) block_absmax_atomic(p.absmax, b_tile, vmax);
        if (p.gn_part) {
#pragma unroll
            for (int h = 0; h < H; ++h) {
                GnTile g{p.gn_part, p.gn_ncb, p.gn_sw,
                         (long)b_tile * p.gn_np64 + p.gn_p64 + (m0 - b_tile * HWm) / 64 + H * wm + h,
                         (p.gn_c0 + n0 + wn * 64) / 32};
                gn_tile_partials_tr(acc[h], g, 2);
            }
        }
    }
}

// Form of the two pre-split projection GEMMs.  g_pa256 -- 0: the 128 x 128 LDS-DMA form only;
// 2: the 256 x 128 form wherever the pixels per image are a multiple of 256; 1 (default): the
// 256 x 128 form for the pre-split qkv epilogue at >= 2048 of its tiles, the one place it measured
// faster (64^2, C 512 -> 1536: 341 vs 373 us; the out-projections and the smaller qkv grids ran
// 4-16 % slower at two workgroups per CU, tools/proj_probe.py).  wc_proj_set_tile for tests.
int g_pa256 = 1;

template <bool QKV, int H, bool WR, bool DA = false>
void launch_pa_form(const IgDev& d, hipStream_t stream) {
    IgDev p = d;
    p.ntiles_n = p.N / 128;
    dim3 grid((p.M / (128 * H)) * p.ntiles_n);
    WC_SET_NAME("proj_pa_kernel", {WC_TB(QKV), WC_TI(H), WC_TB(WR), WC_TB(DA)});
    hipLaunchKernelGGL((proj_pa_kernel<QKV, H, WR, DA>), grid, dim3(NT), 0, stream, p);
}

int launch_pa(const IgDev& d, hipStream_t stream) {
    const bool fits = (d.Hm * d.Wm) % 256 == 0 && d.N % 128 == 0 && !d.abound;
    const long tiles256 = (long)(d.M / 256) * (d.N / 128);
    if (fits && (g_pa256 == 2 || (g_pa256 == 1 && d.qkv3 && tiles256 >= 2048))) {
        if (d.qkv3) launch_pa_form<true, 2, false>(d, stream);
        else launch_pa_form<false, 2, false>(d, stream);
        WC_CHECK_LAUNCH();
        return WC_OK;
    }
    return launch<128, 128, 0, true, WC_ACT_NONE, true>(d, stream);
}

// shared checks of the two PA entry points: the A operand's view shape in args->seg[0] (1x1,
// stride 1, no prologue: a3 already carries it), a3 of M x C x 4 bytes
int prepare_pa(const wc_conv_args* a, const void* a3, int64_t a3_bytes, const void* w3, IgDev& d, long& k) {
    if (!a3 || (reinterpret_cast<uintptr_t>(a3) & 15)) return WC_E_ARG;
    if (a->nseg != 1 || a->seg[0].scale || a->act) return WC_E_ARG;
    const wc_conv_seg& s0 = a->seg[0];
    if (s0.ntaps != 1 || s0.dy[0] || s0.dx[0] || s0.sy != 1 || s0.sx != 1 || s0.H != a->Hm || s0.W != a->Wm)
        return WC_E_SHAPE;
    if ((a->Hm * a->Wm) % 128 || s0.C % 32 || a->N % 128) return WC_E_SHAPE;
    const int st = prepare(a, w3, d, k);
    if (st != WC_OK) return st;
    if (a3_bytes != (long)d.M * s0.C * 4) return WC_E_SHAPE;
    d.a3 = reinterpret_cast<const unsigned char*>(a3);
    return WC_OK;
}

}  // namespace

extern "C" int wc_split_f16x3_tiled(const float* src, int ldc, int B, int HW, int C, const float* scale,
                                    const float* shift, int silu, int a_exp, void* a3, int64_t a3_bytes,
                                    void* stream) {
    if (!src || !a3 || (scale == nullptr) != (shift == nullptr)) return WC_E_ARG;
    if (a_exp < -60 || a_exp > 60) return WC_E_ARG;
    if (B <= 0 || HW <= 0 || HW % 128 || C <= 0 || C % 32 || ldc < C || ldc % 4) return WC_E_SHAPE;
    if ((reinterpret_cast<uintptr_t>(src) & 15) || (reinterpret_cast<uintptr_t>(a3) & 15)) return WC_E_SHAPE;
    if (scale && ((reinterpret_cast<uintptr_t>(scale) & 15) || (reinterpret_cast<uintptr_t>(shift) & 15)))
        return WC_E_SHAPE;
    const long M = (long)B * HW;
    if (a3_bytes != M * C * 4 || M > (1L << 30)) return WC_E_SHAPE;
    dim3 grid((unsigned)(M / 64), (unsigned)((C / 32 + 3) / 4));
    wc_last_kernel = "split_tiled_kernel";
    hipLaunchKernelGGL(split_tiled_kernel, grid, dim3(256), 0, reinterpret_cast<hipStream_t>(stream), src, ldc, HW, C,
                       scale, shift, silu, ldexpf(1.0f, a_exp), reinterpret_cast<unsigned char*>(a3));
    WC_CHECK_LAUNCH();
    return WC_OK;
}

extern "C" int wc_proj_f16x3(const wc_conv_args* a, const void* a3, int64_t a3_bytes, const void* w3,
                             int64_t w3_bytes, int a_exp, const float* w_inv_scale, void* stream) {
    if (!a || !w_inv_scale || a_exp < -60 || a_exp > 60) return WC_E_ARG;
    IgDev d;
    long k;
    const int st = prepare_pa(a, a3, a3_bytes, w3, d, k);
    if (st != WC_OK) return st;
    if (!d.ident || d.ldo % 4 || (reinterpret_cast<uintptr_t>(d.out) & 15)) return WC_E_SHAPE;
    if (d.res && (d.ldres % 4 || (reinterpret_cast<uintptr_t>(d.res) & 15))) return WC_E_SHAPE;
    if (a->temb) return WC_E_ARG;
    if (w3_bytes != (long)(a->N / 128) * d.steps0 * 128 * 64 || w3_bytes >= (1L << 31)) return WC_E_SHAPE;
    d.a_exp = a_exp;
    d.wsinv = w_inv_scale;
    return launch_pa(d, reinterpret_cast<hipStream_t>(stream));
}

extern "C" int wc_proj_f16x3_qkv(const wc_conv_args* a, const void* a3, int64_t a3_bytes, const void* w3,
                                 int64_t w3_bytes, int a_exp, const float* w_inv_scale, void* qkv3, int C, int heads,
                                 const int* exps, void* stream) {
    if (!a || !qkv3 || !exps || !w_inv_scale || a_exp < -60 || a_exp > 60) return WC_E_ARG;
    if (C <= 0 || heads <= 0 || C % heads || (C / heads) % 32 || a->N != 3 * C) return WC_E_SHAPE;
    if (a->res || a->temb || a->absmax_out || a->gn_part || a->out_nchw) return WC_E_ARG;
    if (reinterpret_cast<uintptr_t>(qkv3) & 15) return WC_E_SHAPE;
    for (int i = 0; i < 3; ++i)
        if (exps[i] < -60 || exps[i] > 60) return WC_E_ARG;
    wc_conv_args aa = *a;
    aa.out = reinterpret_cast<float*>(qkv3);  // unused by the split epilogue; keeps prepare's checks uniform
    aa.ldo = a->N;
    aa.Ho = a->Hm; aa.Wo = a->Wm; aa.osy = aa.osx = 1; aa.ooy = aa.oox = 0;
    IgDev d;
    long k;
    const int st = prepare_pa(&aa, a3, a3_bytes, w3, d, k);
    if (st != WC_OK) return st;
    if (w3_bytes != (long)(a->N / 128) * d.steps0 * 128 * 64 || w3_bytes >= (1L << 31)) return WC_E_SHAPE;
    d.a_exp = a_exp;
    d.wsinv = w_inv_scale;
    d.qkv3 = reinterpret_cast<unsigned short*>(qkv3);
    d.qC = C;
    d.qD = C / heads;
    for (int i = 0; i < 3; ++i) d.qscale[i] = ldexpf(1.0f, exps[i]);
    return launch_pa(d, reinterpret_cast<hipStream_t>(stream));
}

extern "C" int wc_proj_set_tile(int rows) {
    // 0 the default choice, 128 / 256 the LDS-DMA forms
    if (rows != 0 && rows != 128 && rows != 256) return WC_E_ARG;
    const int prev = g_pa256 == 0 ? 128 : g_pa256 == 2 ? 256 : 0;
    g_pa256 = rows == 128 ? 0 : rows == 256 ? 2 : 1;
    return prev;
}
