// 3x3 stride-1 convolution on split-precision MFMA for gfx950: bf16x6 and f16x3.
//
// bf16x6.  Every fp32 operand v is split EXACTLY into three bf16 pieces by truncation:
// v0 = v with the low 16 bits cleared, v1 = (v - v0) likewise, v2 = v - v0 - v1 (at most 8
// significant bits, so it is exact in bf16).  The product a*w is accumulated as the six terms
// a_i*w_j with i + j <= 2, each an exact bf16 x bf16 product summed in fp32 by
// v_mfma_f32_32x32x16_bf16.  The dropped terms a1w2 + a2w1 + a2w2 are < 3*2^-24 |a w|, the size
// of one fp32 rounding, so the result stays inside the fp32 tolerance of the reference conv.  A
// 32x32x16 block costs 6 bf16 MFMAs (192 cycles) instead of 8 fp32 MFMAs (512 cycles).
//
// f16x3 (only for a GroupNorm-applied segment 0, whose magnitude has a static bound).  a' =
// a * 2^sA and w' = w * 2^sW[n] (exact power-of-two scales) are split into two fp16 pieces by
// round-to-nearest (h = fp16(v), l = fp16(v - h): v = h + l to ~2^-22 relative, l may be
// subnormal — the f16 MFMA honours subnormal inputs, tools/probes/mfma_f16_subnormal.hip), and
// a'w' = h_a h_w + h_a l_w + l_a h_w on v_mfma_f32_32x32x16_f16: 3 MFMAs per block, half the
// bf16x6 work.  No overflow is possible: a GN output z = (x - mean)/sqrt(var + eps) obeys
// |z| <= sqrt(n - 1) (Samuelson), so |gamma z + beta| <= sqrt(n-1) max|gamma| + max|beta| =: bound,
// and the host picks sA with bound * 2^sA <= 2^14 (fp16 max 65504).  The 1x1 residual segment
// (raw input, no static bound) stays bf16x6 with the same scales, so every product carries the
// factor 2^(sA + sW[n]), removed exactly in the epilogue.
//
// Tiling (implicit GEMM, M = output pixels, N = output channels, K = (16-channel chunk, tap)).
// A workgroup owns a TH x 16 pixel tile of one image and BN output channels; each of its 4 waves
// owns 4 image rows x 16 columns (64 pixels) x 64 channels as 2 x 2 32x32 accumulators.
//   * Per 16-channel chunk the (TH+2) x 18 input HALO is loaded once, GroupNorm-applied (+SiLU),
//     zero-padded, split into its pieces and written to LDS.  All 9 taps then read their A
//     fragments from that one halo image at a constant per-tap offset, so the prologue VALU is
//     paid (TH+2)*18/(TH*16) times per input element instead of 9 times.  The halo loads are
//     issued one K-step before the chunk's last and consumed in it (see the K loop for why).
//   * A K-step is one tap of a chunk (bf16x6) or two (f16x3, 24 MFMAs per wave either way): the
//     taps' 16 x BN weight pieces (pre-split and pre-laid-out by the host in the exact LDS order)
//     are staged through registers one step ahead; one barrier per step.  The next chunk's halo
//     is written at the chunk's last K-step, into the other halo buffer.
//   * The fused 1x1 residual_input_conv (raw input, same pixel) runs as extra chunks with one
//     tap (the halo centre).
// LDS images.  Halo: [piece][k-half 2][pixel (TH+2)*18][8 x 16-bit]; weights: [piece][k-half]
// [BN][8 x 16-bit].  The MFMA row -> pixel map is chosen so that each ds_read_b128 lane group
// ({0-3,12-15,20-27}, {4-11,16-19,28-31}, +32) reads 16 consecutive pixels of one image row:
// 16 distinct 16-byte slots, bank-conflict-free for every tap offset.
//
// Fused work (reference unet_base.py ResBlock, :87-109 / :146-150), as in wc_conv.hip:
// prologue SiLU(v*scale[b,c] + shift[b,c]) with zero padding applied after it; epilogue
// + bias[n] + temb[b,n], activation, + residual view, NHWC store.
#include <stdlib.h>

#include "wc_x6.hpp"

namespace {

using namespace wcx6;

constexpr int NT = 256;
constexpr int HWD = 18;  // halo row width: 16 output columns + 2

struct X6Dev {
    const float* src0;
    int C0, ldc0;
    const float* scale;
    const float* shift;
    const float* src1;
    int C1, ldc1;
    int B, H, W, N;
    const void* w6;
    const float* bias;
    const float* temb;
    int temb_ld;
    const float* res;
    int ldres;
    float* out;
    int ldo;
    int act;
    int nck0, nck1;       // 16-channel chunks of segment 0 (3x3) and segment 1 (1x1 residual)
    int a_exp;            // f16x3: static exponent sA of the segment-0 bound (else 0)
    const float* abound;  // f16x3: per-image bound of every A value (segment 1 in fp16), or NULL
    const float* wsinv;   // f16x3: 2^-sW[n] per output channel (else NULL)
    float* absmax;        // optional per-image max |out| (atomic)
    float* gn_part;       // optional GroupNorm tile partials of the output (wcx6::gn_tile_partials)
    int gn_ncb, gn_sw, gn_c0, gn_np64;
    int tiles_x, tiles_y, ntiles_n;
    int s2d_cpp, Hi, Wi;  // S2D: 16-channel chunks per phase (C / 16) and the input's H, W
};

// F3: segment 0 in f16x3 (2 pieces), else bf16x6 (3 pieces).  R16: segment 1 in f16x3 too (needs
// the per-image bound), else bf16x6.
// GL: weights staged by LDS-DMA (global_load_lds_dwordx4 straight into the LDS image the host
// pre-laid out) at three taps (one halo row) per K-step: 36 MFMAs per wave between barriers and
// no weight registers; else register-staged, one tap per K-step.
// MAP: 0 = 3x3 stride 1; 1 = 4x4/s2 down conv over the space-to-depth input (2x2 taps); 2 = the
// 4x4/s2 transposed conv, one output parity per workgroup (2x2 taps of the 3x3 frame).
template <int TH, int BN, bool RES, bool F3, bool R16, bool GL = false, int MAP = 0, int WR = 0>
struct X6Tile {
    static constexpr int BM = TH * 16;
    static constexpr int WAVES_N = BN / 64;
    static constexpr int WAVES_M = 4 / WAVES_N;
    static_assert(WAVES_M * 64 == BM, "each wave owns 4 image rows x 16 columns");
    static constexpr int NP0 = F3 ? 2 : 3;              // pieces of segment 0
    static constexpr int NP1 = R16 ? 2 : 3;             // pieces of segment 1
    static constexpr int NPH = RES && NP1 > NP0 ? NP1 : NP0;  // halo planes per k-half
    static constexpr int HPIX = (TH + 2) * HWD;          // halo pixels
    static constexpr int HPLANE = HPIX * 16;             // bytes of one (piece, k-half) halo plane
    static constexpr int HSTAGE = 2 * NPH * HPLANE;      // one halo buffer
    static constexpr int BPLANE = BN * 16;               // bytes of one (piece, k-half) weight plane
    static constexpr int BSTEP0 = 2 * NP0 * BPLANE;      // one segment-0 weight step
    static constexpr int BSTEP1 = 2 * NP1 * BPLANE;      // one segment-1 weight step
    // taps per K-step (2 for f16x3 measured slower: 302 vs 322 TF/s, larger LDS weight stage)
    static constexpr int TPS = GL ? 3 : 1;
    static constexpr int NTAP = MAP ? 4 : 9;             // taps per chunk (MAP 1, 2: 2x2 taps)
    static constexpr int NMT = (NTAP + TPS - 1) / TPS;    // K-steps per 16-channel chunk
    static constexpr int BSTEPM = TPS * BSTEP0;           // weight bytes of a full segment-0 K-step
    static constexpr int BSTAGE = (RES && BSTEP1 > BSTEPM) ? BSTEP1 : BSTEPM;  // LDS weight buffer
    // WR: weight fragments go from global (L2) straight into registers, no LDS weight stage.
    // WR 3 (nck1 == nck0): residual chunk c rides in 3x3 chunk c as a tenth step; its TH x 16
    // centre goes to two more halo-shaped buffers after the halo's own (same A addressing)
    static constexpr int LDS = 2 * HSTAGE + (WR ? (WR == 3 ? 2 * HSTAGE : 0) : 2 * BSTAGE);
    static constexpr int H_ITEMS = HPIX * 4;             // float4 items of one halo chunk
    static constexpr int H_PER_T = (H_ITEMS + NT - 1) / NT;
    static constexpr int C_PER_T = TH * 16 * 4 / NT;      // float4 items of one residual centre chunk
    static_assert(C_PER_T * NT == TH * 16 * 4, "whole centre items per thread");
    static constexpr int B_PER_T = (BSTAGE / 16 + NT - 1) / NT;
    // weight items j < B_FULL of every thread are valid in every step (both segments; the last
    // K-step of a chunk may carry a single tap)
    static constexpr int B_FULL = (RES ? (BSTEP0 < BSTEP1 ? BSTEP0 : BSTEP1) : BSTEP0) / 16 / NT;
};

// MFMA row r (0..31) -> pixel (dy, dx) of a 2 x 16 strip: the ds_read_b128 lane group
// {0-3, 12-15, 20-27} is row dy = 0, the group {4-11, 16-19, 28-31} row dy = 1.
WC_DEVICE int row_dy(int r) { return ((r >= 4 && r < 12) || (r >= 16 && r < 20) || r >= 28) ? 1 : 0; }
WC_DEVICE int row_dx(int r) {
    return r < 4 ? r : r < 12 ? r - 4 : r < 20 ? r - 8 : r < 28 ? r - 12 : r - 16;
}

// PRO: 0 = raw segment 0, 1 = GN affine, 2 = GN affine + SiLU.  RES: segment 1 present.
// TH = 8 tiles without a residual or with an fp16 one are held to 3 waves per SIMD (<= 168
// VGPRs; the two-deep residual staging would otherwise take the R16 form to 178 and 2 waves, and
// 3 waves cost it one spilled VGPR); the other forms run at 2.
template <int TH, int BN, int PRO, bool RES, bool F3, bool R16, bool GL, int MAP = 0, int WR = 0>
__global__ __launch_bounds__(NT, (TH == 8 && (!RES || (F3 && R16))) ? 3 : 2) void conv3x3_x6_kernel(
    X6Dev p) {
    using T = X6Tile<TH, BN, RES, F3, R16, GL, MAP, WR>;
    static_assert(!WR || (F3 && (!RES || R16) && !GL && (MAP == 0 || TH == 8) && T::TPS == 1),
                  "WR: the f16x3 3x3 forms with 2-piece weights in every step");
    constexpr bool S2D = MAP == 1, CT = MAP == 2;
    static_assert(!MAP || (!RES && !GL && PRO == 0), "MAP 1, 2: raw single-segment register-staged forms");
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;
    const int wm = wave / T::WAVES_N;
    const int wn = wave % T::WAVES_N;

    // XCD-aware bijective tile order (as wc_conv.hip): consecutive logical tiles, which share
    // halo rows and weights, land on one XCD's L2.
    const int nblk = gridDim.x;
    int bid = blockIdx.x;
    {
        int q = nblk / 8, r = nblk % 8, xcd = bid % 8;
        bid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + bid / 8;
    }
    // CT: the four output parities of one tile are consecutive blocks (one halo, one L2)
    const int par = CT ? (bid & 3) : 0;
    if (CT) bid >>= 2;
    const int tile_n = bid % p.ntiles_n;
    int tt = bid / p.ntiles_n;
    const int txi = tt % p.tiles_x;
    tt /= p.tiles_x;
    const int tyi = tt % p.tiles_y;
    const int b = tt / p.tiles_y;
    const int y0 = tyi * TH, x0 = txi * 16, n0 = tile_n * BN;
    // f16x3 scale of this image: the static exponent, lowered so that the per-image bound (which
    // covers segment 1's raw input) also fits: bound * 2^s < 2^14 with s = 13 - floor(log2 bound)
    int s_exp = p.a_exp;
    if (F3 && p.abound) {
        const float bnd = p.abound[b];
        const int e = (int)((__float_as_uint(bnd) >> 23) & 0xffu) - 127;
        if (bnd > 0.f) s_exp = min(s_exp, 13 - e);
        s_exp = max(s_exp, -100);
    }
    const float ascale = ldexpf(1.0f, s_exp), ainv = ldexpf(1.0f, -s_exp);
    const int S0 = T::NMT * p.nck0;  // segment-0 K-steps
    const int S = S0 + (RES ? p.nck1 : 0);
    const unsigned seg0_bytes = (unsigned)(T::NTAP * p.nck0 * T::BSTEP0);
    const unsigned wtile = CT ? (unsigned)(tile_n * 4 + par) * seg0_bytes
                              : (unsigned)tile_n * (seg0_bytes + (unsigned)((RES ? p.nck1 : 0) * T::BSTEP1));

    // ---- halo staging coordinates: item i = tid + NT*j is halo pixel i>>2, channels 4*(i&3).. ----
    const int q = tid & 3;
    // S2D: halo pixel (hy, hx) is the 2x2 input block (BY, BX) = (y0 - 1 + hy, x0 - 1 + hx) of
    // input pixels (2 BY - 1 + py, 2 BX - 1 + px); its in-bounds bits per phase row / column
    int hoff0[T::H_PER_T];
    // item j's halo pixel is (tid >> 2) + 64 j: one LDS base, item j at + 1024 j (immediate offsets)
    const int hlds0 = (q >> 1) * T::HPLANE + (tid >> 2) * 16 + (q & 1) * 8;
    unsigned hin = 0, hval = 0, hr0 = 0, hr1 = 0, hc0 = 0, hc1 = 0;
#pragma unroll
    for (int j = 0; j < T::H_PER_T; ++j) {
        const int i = tid + NT * j;
        const int P = i >> 2;
        const int hy = P / HWD;
        const int hx = P - hy * HWD;
        const int iy = y0 - 1 + hy, ix = x0 - 1 + hx;
        const bool valid = i < T::H_ITEMS;
        hval |= (valid ? 1u : 0u) << j;
        if constexpr (S2D) {
            const int y2 = 2 * iy - 1, x2 = 2 * ix - 1;
            hr0 |= (valid && (unsigned)y2 < (unsigned)p.Hi ? 1u : 0u) << j;
            hr1 |= (valid && (unsigned)(y2 + 1) < (unsigned)p.Hi ? 1u : 0u) << j;
            hc0 |= ((unsigned)x2 < (unsigned)p.Wi ? 1u : 0u) << j;
            hc1 |= ((unsigned)(x2 + 1) < (unsigned)p.Wi ? 1u : 0u) << j;
            hoff0[j] = ((b * p.Hi + y2) * p.Wi + x2) * p.ldc0 + 4 * q;  // used only with a phase in bounds
        } else {
            const bool inb = valid && (unsigned)iy < (unsigned)p.H && (unsigned)ix < (unsigned)p.W;
            hin |= (inb ? 1u : 0u) << j;
            const int pix = (b * p.H + iy) * p.W + ix;
            hoff0[j] = inb ? (pix * p.ldc0 + 4 * q) * 4 : (int)OOB;  // byte offset, chunk 0
        }
    }
    unsigned hinc = hin;  // in-bounds bits of the chunk in the halo registers

    const __amdgpu_buffer_rsrc_t srd0 = make_srd(p.src0);
    const __amdgpu_buffer_rsrc_t srd1 = make_srd(RES ? p.src1 : p.src0);
    const __amdgpu_buffer_rsrc_t srdw = make_srd(p.w6);
    const __amdgpu_buffer_rsrc_t srdsc = make_srd(PRO ? p.scale : p.src0);
    const __amdgpu_buffer_rsrc_t srdsh = make_srd(PRO ? p.shift : p.src0);

    f32x4 rh[T::H_PER_T];
    // residual (segment-1) chunks: only the TH x 16 halo centre is read (1x1 tap), so they are
    // staged as centre items, two register sets deep (chunk c in set c & 1): a chunk's loads have
    // two K-steps to land instead of one
    f32x4 rc[RES ? 2 : 1][RES ? T::C_PER_T : 1];
    const int cq = tid & 3, cpx = (tid >> 2) & 15, cpy = tid >> 6;  // item tid + NT j: row cpy + 4 j
    const unsigned coff0 = (unsigned)(((b * p.H + y0 + cpy) * p.W + x0 + cpx) * p.ldc1 + 4 * cq);
    const unsigned cstep = (unsigned)(4 * p.W * p.ldc1);
    const int clds0 = (cq >> 1) * T::HPLANE + ((cpy + 1) * HWD + cpx + 1) * 16 + (cq & 1) * 8;
    f32x4 rsc = {1.f, 1.f, 1.f, 1.f}, rsh = {0.f, 0.f, 0.f, 0.f};
    u32x4 rb[GL ? 1 : T::B_PER_T];

    auto load_ss = [&](int c) {  // GroupNorm scale / shift of chunk c
        if constexpr (PRO != 0) {
            const unsigned o = (unsigned)(b * p.C0 + c * 16 + 4 * q) * 4u;
            rsc = bload_f4(srdsc, o);
            rsh = bload_f4(srdsh, o);
        }
    };
    auto load_halo0 = [&](int c, bool ss = true) {
        if constexpr (S2D) {  // chunk c = (phase (py, px), 16 channels): phase-major over 4C channels
            const int ph = c / p.s2d_cpp;
            const int py = ph >> 1, px = ph & 1;
            hinc = (py ? hr1 : hr0) & (px ? hc1 : hc0);
            const int d = (py * p.Wi + px) * p.ldc0 + (c - ph * p.s2d_cpp) * 16;
#pragma unroll
            for (int j = 0; j < T::H_PER_T; ++j)
                rh[j] = bload_f4(srd0, ((hinc >> j) & 1u) ? (unsigned)(hoff0[j] + d) * 4u : OOB);
        } else {
#pragma unroll
            for (int j = 0; j < T::H_PER_T; ++j)
                rh[j] = bload_f4s(srd0, (unsigned)hoff0[j], c * 64);
        }
        if (ss) load_ss(c);
    };
    // seg0: prologue + (F3: scale, 2 fp16 pieces | 3 bf16 pieces); seg1: (F3: scale) 3 bf16 pieces
    auto write_halo = [&](int hs, bool seg0) {
        unsigned char* base = smem + hs * T::HSTAGE;
#pragma unroll
        for (int j = 0; j < T::H_PER_T; ++j) {
            if (j >= T::H_ITEMS / NT && !((hval >> j) & 1u)) continue;  // only the last item can be partial
            f32x4 v = rh[j];
            if constexpr (PRO != 0) {
                if (seg0) {
                    v = v * rsc + rsh;
                    if constexpr (PRO == 2) {
                        v.x = silu_fast(v.x); v.y = silu_fast(v.y);
                        v.z = silu_fast(v.z); v.w = silu_fast(v.w);
                    }
                }
            }
            if (!((hinc >> j) & 1u)) v = f32x4{0.f, 0.f, 0.f, 0.f};  // padding after the prologue
            if constexpr (F3) v = v * ascale;
            if ((F3 && seg0) || (R16 && !seg0)) {
                u32x2 a0, a1;
                split2_f16(v, a0, a1);
                *reinterpret_cast<u32x2*>(base + hlds0 + 1024 * j) = a0;
                *reinterpret_cast<u32x2*>(base + 2 * T::HPLANE + hlds0 + 1024 * j) = a1;
            } else {
                u32x2 a0, a1, a2;
                split3(v, a0, a1, a2);
                *reinterpret_cast<u32x2*>(base + hlds0 + 1024 * j) = a0;
                *reinterpret_cast<u32x2*>(base + 2 * T::HPLANE + hlds0 + 1024 * j) = a1;
                *reinterpret_cast<u32x2*>(base + 4 * T::HPLANE + hlds0 + 1024 * j) = a2;
            }
        }
    };
    // live = false: the same loads at an out-of-range offset (zeros, no traffic), so that the
    // number of loads in flight does not depend on a runtime condition (see load_w below)
    auto load_center = [&](auto P, int c, bool live = true) {
        constexpr int PV = decltype(P)::value;
        const unsigned v = live ? coff0 * 4u : OOB;
#pragma unroll
        for (int j = 0; j < T::C_PER_T; ++j)
            rc[PV][j] = bload_f4s(srd1, v, (int)(((unsigned)j * cstep + (unsigned)c * 16u) * 4u));
    };
    // segment-1 centre -> halo buffer hs: raw input (F3: scaled), R16: 2 fp16 pieces, else 3 bf16
    auto write_center = [&](auto P, int hs) {
        constexpr int PV = decltype(P)::value;
        unsigned char* base = smem + hs * T::HSTAGE + clds0;
#pragma unroll
        for (int j = 0; j < T::C_PER_T; ++j) {
            f32x4 v = rc[PV][j];
            if constexpr (F3) v = v * ascale;
            unsigned char* d = base + j * 4 * HWD * 16;
            if constexpr (R16) {
                u32x2 a0, a1;
                split2_f16(v, a0, a1);
                *reinterpret_cast<u32x2*>(d) = a0;
                *reinterpret_cast<u32x2*>(d + 2 * T::HPLANE) = a1;
            } else {
                u32x2 a0, a1, a2;
                split3(v, a0, a1, a2);
                *reinterpret_cast<u32x2*>(d) = a0;
                *reinterpret_cast<u32x2*>(d + 2 * T::HPLANE) = a1;
                *reinterpret_cast<u32x2*>(d + 4 * T::HPLANE) = a2;
            }
        }
    };
    const std::integral_constant<int, 0> I0;
    const std::integral_constant<int, 1> I1;
    // weight step s (segment-0 steps are BSTEP0 bytes, segment-1 steps BSTEP1)
    // K-step s -> (byte offset of its weights, 16-byte items): segment-0 step s is taps
    // TPS*(s % NMT) .. of chunk s / NMT (the host packs taps of a chunk contiguously)
    auto step_w = [&](int s, unsigned& off, int& items) {
        if (RES && s >= S0) {
            off = wtile + seg0_bytes + (unsigned)((s - S0) * T::BSTEP1);
            items = T::BSTEP1 / 16;
        } else {
            const int c = s / T::NMT, t0 = (s - c * T::NMT) * T::TPS;
            const int nt = T::NTAP - t0 < T::TPS ? T::NTAP - t0 : T::TPS;
            off = wtile + (unsigned)((c * T::NTAP + t0) * T::BSTEP0);
            items = nt * T::BSTEP0 / 16;
        }
    };
    // LDS-DMA: each wave-instruction writes 1 KiB lane-linearly at a wave-uniform LDS base; the
    // host's weight image is already in LDS order, so item i goes to byte 16 i of the stage
    auto glds_b = [&](int s) {
        unsigned base;
        int items;
        step_w(s, base, items);
        const unsigned char* src = reinterpret_cast<const unsigned char*>(p.w6) + base + tid * 16;
        unsigned char* dst = smem + 2 * T::HSTAGE + (s & 1) * T::BSTAGE + wave * 1024;
#pragma unroll
        for (int j = 0; j < T::B_PER_T; ++j) {
            if (j < T::B_FULL || tid + NT * j < items)
                __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void*)(src + j * NT * 16),
                                                 (__attribute__((address_space(3))) void*)(dst + j * NT * 16), 16, 0, 0);
        }
    };
    auto load_b = [&](int s) {
        if constexpr (GL) return;
        unsigned base;
        int items;
        step_w(s < S ? s : S - 1, base, items);  // issued unconditionally: see load_w
#pragma unroll
        for (int j = 0; j < T::B_PER_T; ++j) {
            const int i = tid + NT * j;
            const bool ok = j < T::B_FULL || i < items;
            rb[j] = bload_u4s(srdw, ok ? (unsigned)i * 16u : OOB, (int)base);
        }
    };
    auto write_b = [&](int bs, int s) {
        if constexpr (GL) return;
        unsigned char* base = smem + 2 * T::HSTAGE + bs * T::BSTAGE;
        unsigned off_unused;
        int items;
        step_w(s, off_unused, items);
#pragma unroll
        for (int j = 0; j < T::B_PER_T; ++j) {
            const int i = tid + NT * j;
            if (j < T::B_FULL || i < items) *reinterpret_cast<u32x4*>(base + i * 16) = rb[j];
        }
    };

    // ---- fragment addressing ----
    const int l32 = lane & 31;
    const int half = lane >> 5;
    int abase[2];
#pragma unroll
    for (int mb = 0; mb < 2; ++mb)
        abase[mb] = half * T::HPLANE + ((4 * wm + 2 * mb + row_dy(l32)) * HWD + row_dx(l32)) * 16;
    const int bbase = 2 * T::HSTAGE + half * T::BPLANE + (wn * 64 + l32) * 16;

    f32x16 acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

    // bf16x6 step (segment 0 without F3, and segment 1)
    auto compute6 = [&](int hs, int toff, int bs) {
        const unsigned char* ha = smem + hs * T::HSTAGE + toff * 16;
        const unsigned char* hb = smem + bs * T::BSTAGE;
        u32x4 fa[2][3], fb[2][3];
#pragma unroll
        for (int pc = 0; pc < 3; ++pc) {
#pragma unroll
            for (int mb = 0; mb < 2; ++mb)
                fa[mb][pc] = *reinterpret_cast<const u32x4*>(ha + abase[mb] + pc * 2 * T::HPLANE);
#pragma unroll
            for (int nb = 0; nb < 2; ++nb)
                fb[nb][pc] = *reinterpret_cast<const u32x4*>(hb + bbase + nb * 32 * 16 + pc * 2 * T::BPLANE);
        }
        // piece-order sums 0, 1, 2: the first MFMAs need only the piece-0 fragments
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
    };
    // f16x3 step (segment 0 with F3)
    auto compute3 = [&](int hs, int toff, int bs, int tt) {
        const unsigned char* ha = smem + hs * T::HSTAGE + toff * 16;
        const unsigned char* hb = smem + bs * T::BSTAGE + tt * T::BSTEP0;
        u32x4 fa[2][2], fb[2][2];
#pragma unroll
        for (int pc = 0; pc < 2; ++pc) {
#pragma unroll
            for (int mb = 0; mb < 2; ++mb)
                fa[mb][pc] = *reinterpret_cast<const u32x4*>(ha + abase[mb] + pc * 2 * T::HPLANE);
#pragma unroll
            for (int nb = 0; nb < 2; ++nb)
                fb[nb][pc] = *reinterpret_cast<const u32x4*>(hb + bbase + nb * 32 * 16 + pc * 2 * T::BPLANE);
        }
#pragma unroll
        for (int mb = 0; mb < 2; ++mb)
#pragma unroll
            for (int nb = 0; nb < 2; ++nb) acc[mb][nb] = mfma_f16(fa[mb][0], fb[nb][0], acc[mb][nb]);
#pragma unroll
        for (int mb = 0; mb < 2; ++mb)
#pragma unroll
            for (int nb = 0; nb < 2; ++nb) {
                acc[mb][nb] = mfma_f16c(fa[mb][0], fb[nb][1], acc[mb][nb]);
                acc[mb][nb] = mfma_f16c(fa[mb][1], fb[nb][0], acc[mb][nb]);
            }
    };
    auto compute0 = [&](int hs, int toff, int bs, int tt) {
        if constexpr (F3) compute3(hs, toff, bs, tt);
        else compute6(hs, toff, bs);
    };

    if constexpr (WR) {
        // ---- K loop, weights in registers: a K-step (chunk, tap) reads its A fragments from the
        // chunk's halo image in LDS and its B fragments from a register set filled one step ahead
        // straight from L2 (the host's weight image is already in fragment order); the only LDS
        // writes are the next chunk's halo at the chunk's last tap, so there is ONE barrier per
        // chunk (9 taps x 12 MFMAs) instead of one per tap.  Set parity is compile-time: step
        // s = 9c + mt uses set (c + mt) & 1, and chunks run in pairs.
        // two register sets (the next step's fragments land while this one computes), also for the
        // residual forms: the last 3x3 chunk is peeled (compile-time), so the residual centres it
        // stages are not live through the chunk loop
        // WR 2 (9-tap grids): the last tap's weights go out two taps ahead, into a third set, so the
        // next chunk's halo loads can be issued before them (three taps of cover, not one)
        constexpr bool LA2 = WR == 2 && MAP == 0;
        constexpr int NS = LA2 ? 3 : 2;
        u32x4 wreg[NS][2][2];  // [set][nb][piece]
        const unsigned wlane = (unsigned)(half * T::BPLANE + (wn * 64 + l32) * 16);
        // Every weight / centre load is issued unconditionally (a step past the end re-reads the last
        // one, unused): with a load behind a branch the compiler's vmcnt bookkeeping must assume the
        // skipped path at the join and waits for ALL loads in flight, i.e. for the next step's
        // weights in the middle of this step, on every other step.
        auto load_w = [&](int set, int st) {
            unsigned off;
            int items_unused;
            step_w(st < S ? st : S - 1, off, items_unused);  // wave-uniform: the scalar offset
#pragma unroll
            for (int nb = 0; nb < 2; ++nb)
#pragma unroll
                for (int pc = 0; pc < 2; ++pc)
                    wreg[set][nb][pc] = bload_u4s(srdw, wlane + (unsigned)(nb * 32 * 16 + pc * 2 * T::BPLANE), (int)off);
        };
        auto compute_w = [&](int set, int hs, int toff) {
            const unsigned char* ha = smem + hs * T::HSTAGE + toff * 16;
            u32x4 fa[2][2];
#pragma unroll
            for (int pc = 0; pc < 2; ++pc)
#pragma unroll
                for (int mb = 0; mb < 2; ++mb)
                    fa[mb][pc] = *reinterpret_cast<const u32x4*>(ha + abase[mb] + pc * 2 * T::HPLANE);
#pragma unroll
            for (int mb = 0; mb < 2; ++mb)
#pragma unroll
                for (int nb = 0; nb < 2; ++nb) acc[mb][nb] = mfma_f16(fa[mb][0], wreg[set][nb][0], acc[mb][nb]);
#pragma unroll
            for (int mb = 0; mb < 2; ++mb)
#pragma unroll
                for (int nb = 0; nb < 2; ++nb) {
                    acc[mb][nb] = mfma_f16c(fa[mb][0], wreg[set][nb][1], acc[mb][nb]);
                    acc[mb][nb] = mfma_f16c(fa[mb][1], wreg[set][nb][0], acc[mb][nb]);
                }
        };
        // Chunk c uses halo buffer and weight-set parity PV = (nck0 - 1 - c) & 1, counted from the
        // end, so the peeled last 3x3 chunk always has PV = 0 (two compile-time variants of it
        // flowing into one epilogue made the register allocator spill hundreds of VGPRs).
        // weight set of step mt of a chunk of parity PV: (mt + PV) & 1 for 9 taps (odd: the chunk
        // parity carries the alternation across chunks), mt & 1 for the 2x2 tap grids
        constexpr int NTAP = T::NTAP, TODD = NTAP & 1;
        const int pv0 = (p.nck0 - 1) & 1;
        // WR 3: the centre of a chunk (rc set 0) into centre buffer hs (halo-shaped, after the halo's)
        auto write_cf = [&](int hs) { write_center(I0, 2 + hs); };
        load_halo0(0);
        if constexpr (WR == 3 && RES) load_center(I0, 0);
        if (TODD && pv0 && WR != 3) load_w(1, 0);
        else load_w(0, 0);
        write_halo(pv0, true);
        if constexpr (WR == 3 && RES) write_cf(pv0);
        __syncthreads();
        auto chunk = [&](auto P, auto L, int c) {
            constexpr int PV = decltype(P)::value;  // the chunk's halo buffer and set parity
            constexpr bool LAST = decltype(L)::value != 0;  // the last 3x3 chunk (compile-time)
#pragma unroll
            for (int mt = 0; mt < NTAP; ++mt) {
                const int st = NTAP * c + mt;
                constexpr bool EARLY = LA2 && !LAST;
                if (EARLY && mt == NTAP - 3) {
                    load_w((mt + 1 + TODD * PV) & 1, st + 1);
                    load_w(NS - 1, st + 2);
                    load_halo0(c + 1, false);  // scale / shift (L2) in the last tap: 8 registers fewer
                } else if (EARLY && mt == NTAP - 1) {
                    load_w((mt + 1 + TODD * PV) & 1, st + 1);
                    load_ss(c + 1);
                } else if (!(EARLY && mt == NTAP - 2)) {
                    load_w((mt + 1 + TODD * PV) & 1, st + 1);
                    if (mt == NTAP - 2) {
                        if constexpr (!LAST) load_halo0(c + 1);
                        else if constexpr (RES) load_center(I0, 0);
                    }
                }
                // keep the next step's loads at the head of this one (the scheduler otherwise sinks
                // them behind this step's MFMAs, leaving a few hundred cycles for an L2 round trip)
                __builtin_amdgcn_sched_barrier(0);
                if constexpr (RES && LAST) {
                    if (mt == 8) load_center(I1, p.nck1 > 1 ? 1 : 0);
                }
                // tap offset in the halo; CT parity (py, px): tap (i, j) reads input offset (py - i, px - j)
                const int toff = S2D ? ((mt >> 1) + 1) * HWD + (mt & 1) + 1
                               : CT  ? ((par >> 1) - (mt >> 1) + 1) * HWD + (par & 1) - (mt & 1) + 1
                                     : (mt / 3) * HWD + mt % 3;
                compute_w((EARLY && mt == NTAP - 1) ? NS - 1 : (mt + TODD * PV) & 1, PV, toff);
            }
            if constexpr (!LAST) write_halo(PV ^ 1, true);
            else if constexpr (RES) write_center(I0, PV ^ 1);
            __syncthreads();
        };
        // residual chunk cc: centre register set cc & 1, halo buffer and weight set (nck0 + cc) & 1
        auto residual = [&](auto Q0) {
            if constexpr (RES) {
                constexpr int Q = decltype(Q0)::value;
                const int S0w = 9 * p.nck0;
                auto rstep = [&](auto P, auto QQ, int cc) {
                    constexpr int PV = decltype(P)::value, QV = decltype(QQ)::value;
                    const int st = S0w + cc;
                    const bool more = st + 1 < S;
                    load_w(QV ^ 1, st + 1);
                    load_center(P, cc + 2 < p.nck1 ? cc + 2 : p.nck1 - 1);
                    __builtin_amdgcn_sched_barrier(0);
                    compute_w(QV, QV, HWD + 1);  // the halo centre = the output pixel
                    if (more) write_center(std::integral_constant<int, PV ^ 1>{}, QV ^ 1);
                    __syncthreads();
                };
                int cc = 0;
                for (; cc + 1 < p.nck1; cc += 2) {
                    rstep(I0, std::integral_constant<int, Q>{}, cc);
                    rstep(I1, std::integral_constant<int, Q ^ 1>{}, cc + 1);
                }
                if (cc < p.nck1) rstep(I0, std::integral_constant<int, Q>{}, cc);
            }
        };
        const std::integral_constant<int, 0> NL;
        const std::integral_constant<int, 1> LL;
        if constexpr (WR == 3 && RES) {
            // ---- residual interleaved: chunk c = 9 taps of segment 0 + the 1x1 step of segment-1
            // chunk c (nck1 == nck0). Ten steps per chunk, so the weight set of step mt is mt & 1
            // for every chunk; the centre of chunk c + 1 is loaded with its halo and written to the
            // other buffer's centre region at the chunk's end: no separate residual phase, no
            // barrier per 1x1 step.
            // weights of step (c, mt): taps in segment 0, mt == 9 the segment-1 step c; past the
            // end: the last step again (issued unconditionally, unused)
            auto load_wf = [&](int set, int c, int mt) {
                if (c >= p.nck0) { c = p.nck0 - 1; mt = 9; }
                const unsigned off = mt < 9 ? wtile + (unsigned)((9 * c + mt) * T::BSTEP0)
                                            : wtile + seg0_bytes + (unsigned)(c * T::BSTEP1);
#pragma unroll
                for (int nb = 0; nb < 2; ++nb)
#pragma unroll
                    for (int pc = 0; pc < 2; ++pc)
                        wreg[set][nb][pc] = bload_u4s(srdw, wlane + (unsigned)(nb * 32 * 16 + pc * 2 * T::BPLANE), (int)off);
            };
            auto compute_cf = [&](int set, int hs) { compute_w(set, 2 + hs, HWD + 1); };
            auto chunk_f = [&](auto P, auto L, int c) {
                constexpr int PV = decltype(P)::value;
                constexpr bool LAST = decltype(L)::value != 0;
#pragma unroll
                for (int mt = 0; mt < 10; ++mt) {
                    load_wf((mt + 1) & 1, mt < 9 ? c : c + 1, mt < 9 ? mt + 1 : 0);
                    if constexpr (!LAST) {  // GN scale / shift (L2) last: 8 registers fewer through taps 7-8
                        if (mt == 7) load_halo0(c + 1, false);
                        if (mt == 8) load_center(I0, c + 1);
                        if (mt == 9) load_ss(c + 1);
                    }
                    __builtin_amdgcn_sched_barrier(0);
                    if (mt < 9) compute_w(mt & 1, PV, (mt / 3) * HWD + mt % 3);
                    else compute_cf(1, PV);
                }
                if constexpr (!LAST) {
                    write_halo(PV ^ 1, true);
                    write_cf(PV ^ 1);
                    __syncthreads();
                }
            };
            // (the prologue above wrote chunk 0's halo and centre into buffer pv0 and loaded step
            // (0, 0)'s weights into set 0)
            int c = 0;
            if (pv0) chunk_f(I1, NL, c++);
            for (; c + 1 < p.nck0 - 1; c += 2) {
                chunk_f(I0, NL, c);
                chunk_f(I1, NL, c + 1);
            }
            chunk_f(I0, LL, p.nck0 - 1);
        } else {
        int c = 0;
        if (pv0) chunk(I1, NL, c++);  // nck0 even: the leading odd chunk
        for (; c + 1 < p.nck0 - 1; c += 2) {
            chunk(I0, NL, c);
            chunk(I1, NL, c + 1);
        }
        chunk(I0, LL, p.nck0 - 1);
        residual(I1);  // the residual centres follow in halo buffer 1, weight set 1
        }
    } else {
        // ---- K loop: steps = (chunk, tap) of segment 0, then the chunks of segment 1 ----
        load_halo0(0);
        if constexpr (GL) glds_b(0);
        load_b(0);
        write_halo(0, true);
        write_b(0, 0);
        __syncthreads();
        int s = 0;
        for (int c = 0; c < p.nck0; ++c) {
            const int hs = c & 1;
    #pragma unroll
            for (int mt = 0; mt < T::NMT; ++mt) {
                const bool more = s + 1 < S;
                if constexpr (GL) {
                    if (more) glds_b(s + 1);  // buffer (s+1)&1 was last read in step s-1
                }
                load_b(s + 1);
                // The next chunk's halo loads go out one K-step before the last, after that step's
                // weight loads: vmcnt drains in issue order, so a halo load issued earlier would be
                // waited for by every later step's weight-tile wait (an HBM-latency stall per chunk).
                // After the last chunk come residual centres 0 (one step early) and 1 (in the last).
                // Every load is issued in every chunk (the last chunk re-reads its own halo, the
                // centres of the other chunks go to an out-of-range offset): a load behind a runtime
                // branch makes the compiler wait for all loads in flight at the next weight wait.
                if (mt == T::NMT - 2) {
                    load_halo0(c + 1 < p.nck0 ? c + 1 : c);
                    if constexpr (RES) load_center(I0, 0, c + 1 == p.nck0);
                }
                if constexpr (RES) {
                    if (mt == T::NMT - 1) load_center(I1, 1, c + 1 == p.nck0 && p.nck1 > 1);
                }
                __builtin_amdgcn_sched_barrier(0);
    #pragma unroll
                for (int tt = 0; tt < T::TPS; ++tt) {
                    const int tp = mt * T::TPS + tt;
                    if (tp < T::NTAP) {
                        // CT parity (py, px): tap (i, j) reads input offset (py - i, px - j) (engine._CT_TAPS)
                        const int toff = S2D ? ((tp >> 1) + 1) * HWD + (tp & 1) + 1
                                       : CT  ? ((par >> 1) - (tp >> 1) + 1) * HWD + (par & 1) - (tp & 1) + 1
                                             : (tp / 3) * HWD + tp % 3;
                        compute0(hs, toff, s & 1, tt);
                    }
                }
                if (more) write_b((s + 1) & 1, s + 1);
                if (mt == T::NMT - 1) {
                    if (c + 1 < p.nck0) write_halo(hs ^ 1, true);
                    else if constexpr (RES) write_center(I0, hs ^ 1);
                }
                __syncthreads();
                ++s;
            }
        }
        if constexpr (RES) {
            // residual chunk c (centre set c & 1): issue centre c + 2 into this set, compute, write
            // centre c + 1 (loaded a step earlier) into the other halo buffer
            auto rstep = [&](auto P, int c) {
                constexpr int PV = decltype(P)::value;
                const int hs = (p.nck0 + c) & 1;
                const bool more = s + 1 < S;
                if constexpr (GL) {
                    if (more) glds_b(s + 1);
                }
                load_b(s + 1);
                load_center(P, c + 2, c + 2 < p.nck1);
                __builtin_amdgcn_sched_barrier(0);
                if constexpr (R16) compute3(hs, HWD + 1, s & 1, 0);  // the halo centre = the output pixel
                else compute6(hs, HWD + 1, s & 1);
                if (more) {
                    write_b((s + 1) & 1, s + 1);
                    write_center(std::integral_constant<int, PV ^ 1>{}, hs ^ 1);
                }
                __syncthreads();
                ++s;
            };
            int c = 0;
            for (; c + 1 < p.nck1; c += 2) {
                rstep(I0, c);
                rstep(I1, c + 1);
            }
            if (c < p.nck1) rstep(I0, c);
        }

    }

    // ---- epilogue: (F3: x 2^-(sA + sW[n])) + bias + temb, activation, + residual, NHWC store ----
    // 32-bit buffer offsets from the image's base (the tile is one image): one multiply per row,
    // no 64-bit address arithmetic per element
    const long img_px = (long)b * p.H * p.W * (CT ? 4 : 1);
    const __amdgpu_buffer_rsrc_t srd_out = make_srd(p.out + img_px * p.ldo);
    const __amdgpu_buffer_rsrc_t srd_res = make_srd(p.res ? p.res + img_px * p.ldres : p.out);
    float vmax = 0.f;
    // per-channel bias / temb / scale of both column blocks loaded before the first store (a load
    // issued after stores waits for their acks: vmcnt counts both)
    float eadd[2], emul[2];
#pragma unroll
    for (int nb = 0; nb < 2; ++nb) {
        const int n = n0 + wn * 64 + nb * 32 + l32;
        const bool ok = n < p.N;
        eadd[nb] = (ok && p.bias) ? p.bias[n] : 0.f;
        if (ok && p.temb) eadd[nb] += p.temb[b * p.temb_ld + n];
        emul[nb] = (F3 && ok) ? p.wsinv[n] * ainv : 1.0f;
    }
    // Fast path (no activation, the whole column tile inside N: every UNet 3x3 conv): straight-line
    // code, per 32 x 32 block 16 residual loads issued together, then 16 stores; row offsets in the
    // scalar buffer offset.  The general path below branches per element on the activation and per
    // block on n < N, and the compiler then waits for each residual load right after issuing it.
    const bool fast = p.act == WC_ACT_NONE && n0 + BN <= p.N;
    auto epi_fast = [&](auto HR) {
        constexpr bool HASRES = decltype(HR)::value;
#pragma unroll
        for (int mb = 0; mb < 2; ++mb) {
            const int pix0 = CT ? (2 * (y0 + 4 * wm + 2 * mb) + (par >> 1)) * 2 * p.W + 2 * x0 + (par & 1)
                                : (y0 + 4 * wm + 2 * mb) * p.W + x0;
#pragma unroll
            for (int nb = 0; nb < 2; ++nb) {
                const int n = n0 + wn * 64 + nb * 32 + l32;
                const float add = eadd[nb], mul = emul[nb];
                float rv[16];
                if constexpr (HASRES) {
                    const unsigned vres = (unsigned)(pix0 * p.ldres + n) * 4u;
#pragma unroll
                    for (int r = 0; r < 16; ++r) {
                        const int row = (r & 3) + 8 * (r >> 2) + 4 * half;
                        const int dpx = CT ? (row_dy(row) ? 4 * p.W : 0) + 2 * row_dx(row)
                                           : (row_dy(row) ? p.W : 0) + row_dx(row);
                        rv[r] = bload_f1s(srd_res, vres, dpx * p.ldres * 4);
                    }
                }
                const unsigned vout = (unsigned)(pix0 * p.ldo + n) * 4u;
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int row = (r & 3) + 8 * (r >> 2) + 4 * half;
                    const int dpx = CT ? (row_dy(row) ? 4 * p.W : 0) + 2 * row_dx(row)
                                       : (row_dy(row) ? p.W : 0) + row_dx(row);
                    float v = (F3 ? acc[mb][nb][r] * mul : acc[mb][nb][r]) + add;
                    if constexpr (HASRES) v += rv[r];
                    bstore_f1s(srd_out, vout, dpx * p.ldo * 4, v);
                    vmax = fmaxf(vmax, fabsf(v));
                    acc[mb][nb][r] = v;
                }
            }
        }
    };
    if (fast) {
        if (p.res) epi_fast(std::true_type{});
        else epi_fast(std::false_type{});
    } else
#pragma unroll
    for (int mb = 0; mb < 2; ++mb) {
        // pixel (dy 0, dx 0) of this 32-row block; CT: output pixel (2y + py, 2x + px) of 2H x 2W
        const int pix0 = CT ? (2 * (y0 + 4 * wm + 2 * mb) + (par >> 1)) * 2 * p.W + 2 * x0 + (par & 1)
                            : (y0 + 4 * wm + 2 * mb) * p.W + x0;
#pragma unroll
        for (int nb = 0; nb < 2; ++nb) {
            const int n = n0 + wn * 64 + nb * 32 + l32;
            if (n >= p.N) continue;
            const float add = eadd[nb], mul = emul[nb];
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int row = (r & 3) + 8 * (r >> 2) + 4 * half;
                const int pix = CT ? pix0 + (row_dy(row) ? 4 * p.W : 0) + 2 * row_dx(row)
                                   : pix0 + (row_dy(row) ? p.W : 0) + row_dx(row);
                float v = (F3 ? acc[mb][nb][r] * mul : acc[mb][nb][r]) + add;
                if (p.act == WC_ACT_GELU) v = 0.5f * v * (1.0f + erff(v * 0.70710678118654752f));
                else if (p.act == WC_ACT_SILU) v = v / (1.0f + __expf(-v));
                if (p.res) v += bload_f1(srd_res, (unsigned)(pix * p.ldres + n) * 4u);
                bstore_f1(srd_out, (unsigned)(pix * p.ldo + n) * 4u, v);
                vmax = fmaxf(vmax, fabsf(v));
                acc[mb][nb][r] = v;
            }
        }
    }
    if (p.absmax) block_absmax_atomic(p.absmax, b, vmax);  // the whole tile is image b
    if (p.gn_part) {
        // this wave's 64 pixels (4 rows x 16 columns of the tile) are pixel block p64 of image b
        GnTile g{p.gn_part, p.gn_ncb, p.gn_sw,
                 (long)b * p.gn_np64 + par * (p.H * p.W / 64) + (tyi * p.tiles_x + txi) * T::WAVES_M + wm,
                 (p.gn_c0 + n0 + wn * 64) / 32};
        gn_tile_partials(acc, g, min(2, max(0, (p.N - n0 - wn * 64) / 32)));
    }
}

template <int TH, int BN, int PRO, bool RES, bool F3, bool R16 = false, bool GL = false, int MAP = 0, int WR = 0>
int launch6(const X6Dev& d, hipStream_t stream) {
    using T = X6Tile<TH, BN, RES, F3, R16, GL, MAP, WR>;
    static const int lds = T::LDS;
    static bool attr_set = false;  // > 64 KiB of dynamic LDS needs an explicit opt-in
    if (!attr_set) {
        hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&conv3x3_x6_kernel<TH, BN, PRO, RES, F3, R16, GL, MAP, WR>),
                                           hipFuncAttributeMaxDynamicSharedMemorySize, lds);
        if (e != hipSuccess) return (int)e;
        attr_set = true;
    }
    X6Dev p = d;
    p.tiles_x = p.W / 16;
    p.tiles_y = p.H / TH;
    p.ntiles_n = (p.N + BN - 1) / BN;
    dim3 grid(p.B * p.tiles_y * p.tiles_x * p.ntiles_n * (MAP == 2 ? 4 : 1));
    WC_SET_NAME("conv3x3_x6_kernel", {WC_TI(TH), WC_TI(BN), WC_TI(PRO), WC_TB(RES), WC_TB(F3), WC_TB(R16), WC_TB(GL),
                                      WC_TI(MAP), WC_TI(WR)});
    hipLaunchKernelGGL((conv3x3_x6_kernel<TH, BN, PRO, RES, F3, R16, GL, MAP, WR>), grid, dim3(NT), lds, stream, p);
    WC_CHECK_LAUNCH();
    return WC_OK;
}

template <int TH, int BN>
int dispatch6(const X6Dev& d, int pro, bool res, bool f3, hipStream_t s) {
    // f16x3 weight fragments straight from L2 into registers one K-step ahead, one barrier per 16-channel
    // chunk (same-box A/Bs against LDS-staged weights: conv1 338 -> 356 TF/s; 64-channel forms 27.10 ->
    // 27.00 ms/step); the residual 1x1 chunks interleaved with the 3x3 chunks when the two segments have
    // as many chunks (WR 3).  Measured and removed: LDS-DMA weight staging (292 vs 318
    // TF/s), the last tap's weights two taps ahead (the step did not gain), the one-wave-per-SIMD
    // software-pipelined form (no faster: 425 vs 427 TF/s at 64^2, slower at 256^2).
    if constexpr (TH == 16) {
        if (f3 && pro == 2 && (!res || d.abound != nullptr))
            return res ? launch6<TH, BN, 2, true, true, true, false, 0, 1>(d, s)
                       : launch6<TH, BN, 2, false, true, false, false, 0, 1>(d, s);
    }
    if constexpr (TH == 8) {
        if (f3 && !res) {
            return pro == 1 ? launch6<TH, BN, 1, false, true, false, false, 0, true>(d, s)
                            : launch6<TH, BN, 2, false, true, false, false, 0, true>(d, s);
        }
        if (f3 && res && d.abound != nullptr && pro == 2) {
            if (d.nck1 == d.nck0) return launch6<TH, BN, 2, true, true, true, false, 0, 3>(d, s);
            return launch6<TH, BN, 2, true, true, true, false, 0, true>(d, s);
        }
    }
    if (f3) {  // f16x3 needs the GN prologue (the static bound); pro is 1 or 2 here
        const bool r16 = res && d.abound != nullptr;
        switch ((pro - 1) * 3 + (res ? (r16 ? 2 : 1) : 0)) {
            case 0: return launch6<TH, BN, 1, false, true>(d, s);
            case 1: return launch6<TH, BN, 1, true, true>(d, s);
            case 2: return launch6<TH, BN, 1, true, true, true>(d, s);
            case 3: return launch6<TH, BN, 2, false, true>(d, s);
            case 4: return launch6<TH, BN, 2, true, true>(d, s);
            default: return launch6<TH, BN, 2, true, true, true>(d, s);
        }
    }
    switch (pro * 2 + (res ? 1 : 0)) {
        case 0: return launch6<TH, BN, 0, false, false>(d, s);
        case 1: return launch6<TH, BN, 0, true, false>(d, s);
        case 2: return launch6<TH, BN, 1, false, false>(d, s);
        case 3: return launch6<TH, BN, 1, true, false>(d, s);
        case 4: return launch6<TH, BN, 2, false, false>(d, s);
        default: return launch6<TH, BN, 2, true, false>(d, s);
    }
}

bool is_3x3(const wc_conv_seg& s) {
    if (s.ntaps != 9) return false;
    for (int t = 0; t < 9; ++t)
        if (s.dy[t] != t / 3 - 1 || s.dx[t] != t % 3 - 1) return false;
    return true;
}

// Shared host validation; fills d and returns the number of K-steps (or a negative status).
int prepare(const wc_conv_args* a, const void* w, X6Dev& d, int& BN, int& TH) {
    if (!a || !w || !a->out) return WC_E_ARG;
    if (a->nseg < 1 || a->nseg > 2) return WC_E_ARG;
    const wc_conv_seg& s0 = a->seg[0];
    if (!s0.src) return WC_E_ARG;
    if ((s0.scale == nullptr) != (s0.shift == nullptr)) return WC_E_ARG;
    if (a->act < WC_ACT_NONE || a->act > WC_ACT_SILU) return WC_E_ARG;
    BN = wc_conv3x3_x6_tile_n(a->N);
    TH = BN == 64 ? 16 : 8;
    if (!is_3x3(s0) || s0.sy != 1 || s0.sx != 1 || s0.kbase != 0) return WC_E_SHAPE;
    if (s0.C <= 0 || s0.C % 16 || s0.ldc % 4 || (reinterpret_cast<uintptr_t>(s0.src) & 15)) return WC_E_SHAPE;
    if (s0.H != a->Hm || s0.W != a->Wm || a->Hm % TH || a->Wm % 16) return WC_E_SHAPE;
    if (a->B <= 0 || a->N <= 0) return WC_E_SHAPE;
    if ((long)a->B * s0.H * s0.W * s0.ldc * 4 >= (1L << 31)) return WC_E_SHAPE;  // 2 GiB SRD range
    if (reinterpret_cast<uintptr_t>(w) & 15) return WC_E_SHAPE;
    d = X6Dev{};
    d.src0 = s0.src; d.C0 = s0.C; d.ldc0 = s0.ldc; d.scale = s0.scale; d.shift = s0.shift;
    d.nck0 = s0.C / 16;
    if (a->nseg == 2) {
        const wc_conv_seg& s1 = a->seg[1];
        if (!s1.src || s1.scale) return WC_E_ARG;
        if (s1.ntaps != 1 || s1.dy[0] != 0 || s1.dx[0] != 0 || s1.sy != 1 || s1.sx != 1) return WC_E_SHAPE;
        if (s1.H != s0.H || s1.W != s0.W || s1.kbase != 9 * s0.C) return WC_E_SHAPE;
        if (s1.C <= 0 || s1.C % 16 || s1.ldc % 4 || (reinterpret_cast<uintptr_t>(s1.src) & 15)) return WC_E_SHAPE;
        if ((long)a->B * s1.H * s1.W * s1.ldc * 4 >= (1L << 31)) return WC_E_SHAPE;
        d.src1 = s1.src; d.C1 = s1.C; d.ldc1 = s1.ldc; d.nck1 = s1.C / 16;
    }
    if (a->out_nchw || a->Ho != a->Hm || a->Wo != a->Wm || a->osy != 1 || a->osx != 1 || a->ooy || a->oox)
        return WC_E_SHAPE;
    // the epilogue addresses one image of the output / residual with 32-bit buffer offsets
    if ((long)a->Hm * a->Wm * a->ldo * 4 >= (1L << 31) || (a->res && (long)a->Hm * a->Wm * a->ldres * 4 >= (1L << 31)))
        return WC_E_SHAPE;
    d.B = a->B; d.H = a->Hm; d.W = a->Wm; d.N = a->N;
    d.w6 = w; d.bias = a->bias; d.temb = a->temb; d.temb_ld = a->temb_ld;
    d.res = a->res; d.ldres = a->ldres; d.out = a->out; d.ldo = a->ldo; d.act = a->act;
    d.a_exp = 0; d.abound = nullptr; d.wsinv = nullptr;
    d.absmax = a->absmax_out;
    d.gn_part = a->gn_part;
    if (a->gn_part) {  // N whole 32-channel blocks at a 32-aligned offset; 64-pixel blocks per image
        const int sw = a->gn_sw;
        if ((sw != 4 && sw != 8 && sw != 16 && sw != 32) || a->N % 32 || a->gn_c0 % 32 || a->gn_c0 < 0 ||
            a->gn_c0 + a->N > a->gn_ncb * 32 || a->gn_p64 != 0 || a->gn_np64 * 64 != a->Hm * a->Wm)
            return WC_E_SHAPE;
        d.gn_ncb = a->gn_ncb; d.gn_sw = sw; d.gn_c0 = a->gn_c0; d.gn_np64 = a->gn_np64;
    }
    return WC_OK;
}

}  // namespace

extern "C" int wc_conv3x3_x6_tile_n(int N) { return N <= 64 ? 64 : 128; }

extern "C" int wc_conv3x3_x6(const wc_conv_args* a, const void* w6, int64_t w6_bytes, void* stream) {
    X6Dev d;
    int BN, TH;
    const int st = prepare(a, w6, d, BN, TH);
    if (st != WC_OK) return st;
    const long ntn = (a->N + BN - 1) / BN;
    const long steps = 9L * d.nck0 + d.nck1;
    if (w6_bytes != ntn * steps * (long)BN * 96 || w6_bytes >= (1L << 31)) return WC_E_SHAPE;
    const int pro = a->seg[0].scale ? (a->seg[0].silu ? 2 : 1) : 0;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    if (BN == 64) return dispatch6<16, 64>(d, pro, a->nseg == 2, false, s);
    return dispatch6<8, 128>(d, pro, a->nseg == 2, false, s);
}

extern "C" int wc_conv3x3_f16x3(const wc_conv_args* a, const void* w3, int64_t w3_bytes, int a_exp,
                                const float* w_inv_scale, const float* a_bound, void* stream) {
    X6Dev d;
    int BN, TH;
    const int st = prepare(a, w3, d, BN, TH);
    if (st != WC_OK) return st;
    if (!w_inv_scale) return WC_E_ARG;
    // segment 0 needs a range bound: the GN prologue's static one, or (a raw single segment, e.g. a
    // data gradient in the training backward) the per-image bound a_bound
    if (!a->seg[0].scale && (!a_bound || a->nseg != 1)) return WC_E_ARG;
    if (a_exp < -60 || a_exp > 60) return WC_E_ARG;
    const long ntn = (a->N + BN - 1) / BN;
    const long res_step = a_bound ? 64 : 96;  // segment 1 in fp16 (2 pieces) when bounded, else bf16x6
    if (w3_bytes != ntn * (9L * d.nck0 * BN * 64 + (long)d.nck1 * BN * res_step) || w3_bytes >= (1L << 31))
        return WC_E_SHAPE;
    d.a_exp = a_exp;
    d.abound = a_bound;
    d.wsinv = w_inv_scale;
    const int pro = a->seg[0].scale ? (a->seg[0].silu ? 2 : 1) : 0;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    if (pro == 0) {  // raw segment under the per-image bound: the weights-in-registers forms
        if (BN == 64) return launch6<16, 64, 0, false, true, false, false, 0, 1>(d, s);
        return launch6<8, 128, 0, false, true, false, false, 0, 1>(d, s);
    }
    if (BN == 64) return dispatch6<16, 64>(d, pro, a->nseg == 2, true, s);
    return dispatch6<8, 128>(d, pro, a->nseg == 2, true, s);
}

// 4x4 stride-2 pad-1 conv (the UNet down-sampling conv) as a 2x2 stride-1 conv over the
// space-to-depth view of its input: output (oy, ox) = sum over taps (a, b) in {0,1}^2 of block
// (oy + a, ox + b), block (BY, BX) = input pixels (2 BY - 1 + py, 2 BX - 1 + px) as 4C channels
// (phase-major), so the weight tap (ky, kx) = (2a + py, 2b + px).  The halo kernel runs it with a
// 2x2 tap grid and the block -> pixel map in its halo loader: each input value is staged once per
// tile instead of once per tap.  Raw input on f16x3 under the producer's per-image bound.
extern "C" int wc_conv4x4s2_f16x3(const wc_conv_args* a, const void* w3, int64_t w3_bytes, const float* w_inv_scale,
                                  const float* a_bound, void* stream) {
    if (!a || !w3 || !a->out || !w_inv_scale || !a_bound) return WC_E_ARG;
    if (a->nseg != 1 || a->act != WC_ACT_NONE) return WC_E_ARG;
    const wc_conv_seg& s0 = a->seg[0];
    if (!s0.src || s0.scale || s0.shift) return WC_E_ARG;
    if (s0.ntaps != 16 || s0.sy != 2 || s0.sx != 2 || s0.kbase != 0) return WC_E_SHAPE;
    for (int t = 0; t < 16; ++t)
        if (s0.dy[t] != t / 4 - 1 || s0.dx[t] != t % 4 - 1) return WC_E_SHAPE;
    const int BN = wc_conv3x3_x6_tile_n(a->N);
    if (BN != 128) return WC_E_SHAPE;  // the TH = 8 x BN = 128 form only (N > 64)
    if (s0.C <= 0 || s0.C % 16 || s0.ldc % 4 || (reinterpret_cast<uintptr_t>(s0.src) & 15)) return WC_E_SHAPE;
    if (a->B <= 0 || a->Hm % 8 || a->Wm % 16 || s0.H != 2 * a->Hm || s0.W != 2 * a->Wm) return WC_E_SHAPE;
    if ((long)a->B * s0.H * s0.W * s0.ldc * 4 >= (1L << 31)) return WC_E_SHAPE;
    if (reinterpret_cast<uintptr_t>(w3) & 15) return WC_E_SHAPE;
    if (a->out_nchw || a->Ho != a->Hm || a->Wo != a->Wm || a->osy != 1 || a->osx != 1 || a->ooy || a->oox)
        return WC_E_SHAPE;
    if ((long)a->Hm * a->Wm * a->ldo * 4 >= (1L << 31)) return WC_E_SHAPE;  // per image: offsets from its base
    if (a->res && ((long)a->Hm * a->Wm * a->ldres * 4 >= (1L << 31) || a->ldres % 4)) return WC_E_SHAPE;
    X6Dev d{};
    d.res = a->res; d.ldres = a->ldres;  // epilogue: out = conv + res (the training data gradient accumulates)
    d.src0 = s0.src; d.C0 = 4 * s0.C; d.ldc0 = s0.ldc;
    d.nck0 = 4 * s0.C / 16;
    d.s2d_cpp = s0.C / 16; d.Hi = s0.H; d.Wi = s0.W;
    d.B = a->B; d.H = a->Hm; d.W = a->Wm; d.N = a->N;
    d.w6 = w3; d.bias = a->bias; d.temb = a->temb; d.temb_ld = a->temb_ld;
    d.out = a->out; d.ldo = a->ldo; d.act = WC_ACT_NONE;
    d.a_exp = 60; d.abound = a_bound; d.wsinv = w_inv_scale;
    d.absmax = a->absmax_out;
    d.gn_part = a->gn_part;
    if (a->gn_part) {
        const int sw = a->gn_sw;
        if ((sw != 4 && sw != 8 && sw != 16 && sw != 32) || a->N % 32 || a->gn_c0 % 32 || a->gn_c0 < 0 ||
            a->gn_c0 + a->N > a->gn_ncb * 32 || a->gn_p64 != 0 || a->gn_np64 * 64 != a->Hm * a->Wm)
            return WC_E_SHAPE;
        d.gn_ncb = a->gn_ncb; d.gn_sw = sw; d.gn_c0 = a->gn_c0; d.gn_np64 = a->gn_np64;
    }
    const long ntn = (a->N + BN - 1) / BN;
    if (w3_bytes != ntn * 4L * d.nck0 * BN * 64 || w3_bytes >= (1L << 31)) return WC_E_SHAPE;
    return launch6<8, 128, 0, false, true, false, false, 1, true>(d, reinterpret_cast<hipStream_t>(stream));
}

// ConvTranspose2d(C, N, 4, stride 2, padding 1) (the UNet up-sampling conv) in one launch: output
// parity (py, px) is a 2x2 stride-1 conv over the input, tap (i, j) at input offset (py - i, px - j)
// (engine._CT_TAPS), written to pixels (2y + py, 2x + px); the four parities of a tile are four
// consecutive workgroups of the halo kernel reading one halo.
extern "C" int wc_convtr4x4s2_f16x3(const wc_conv_args* a, const void* w3, int64_t w3_bytes, const float* w_inv_scale,
                                   const float* a_bound, void* stream) {
    if (!a || !w3 || !a->out || !w_inv_scale || !a_bound) return WC_E_ARG;
    if (a->nseg != 1 || a->act != WC_ACT_NONE) return WC_E_ARG;
    const wc_conv_seg& s0 = a->seg[0];
    if (!s0.src || s0.scale || s0.shift) return WC_E_ARG;
    if (s0.sy != 1 || s0.sx != 1 || s0.kbase != 0) return WC_E_SHAPE;
    const int BN = wc_conv3x3_x6_tile_n(a->N);
    const int TH = BN == 64 ? 16 : 8;
    if (s0.C <= 0 || s0.C % 16 || s0.ldc % 4 || (reinterpret_cast<uintptr_t>(s0.src) & 15)) return WC_E_SHAPE;
    if (a->B <= 0 || a->N <= 0 || s0.H != a->Hm || s0.W != a->Wm || a->Hm % TH || a->Wm % 16) return WC_E_SHAPE;
    if ((long)a->B * s0.H * s0.W * s0.ldc * 4 >= (1L << 31)) return WC_E_SHAPE;
    if (reinterpret_cast<uintptr_t>(w3) & 15) return WC_E_SHAPE;
    if (a->out_nchw || a->Ho != 2 * a->Hm || a->Wo != 2 * a->Wm || a->osy != 2 || a->osx != 2 || a->ooy || a->oox ||
        a->temb)
        return WC_E_SHAPE;
    if (4L * a->Hm * a->Wm * a->ldo * 4 >= (1L << 31)) return WC_E_SHAPE;  // per image: offsets from its base
    if (a->res && (4L * a->Hm * a->Wm * a->ldres * 4 >= (1L << 31) || a->ldres % 4)) return WC_E_SHAPE;
    X6Dev d{};
    d.res = a->res; d.ldres = a->ldres;  // epilogue: out = conv + res, at the parity's output pixel
    d.src0 = s0.src; d.C0 = s0.C; d.ldc0 = s0.ldc; d.nck0 = s0.C / 16;
    d.B = a->B; d.H = a->Hm; d.W = a->Wm; d.N = a->N;
    d.w6 = w3; d.bias = a->bias;
    d.out = a->out; d.ldo = a->ldo; d.act = WC_ACT_NONE;
    d.a_exp = 60; d.abound = a_bound; d.wsinv = w_inv_scale;
    d.absmax = a->absmax_out;
    d.gn_part = a->gn_part;
    if (a->gn_part) {  // the parities' pixel blocks: parity p owns blocks p*HW/64 .. of the 4HW/64
        const int sw = a->gn_sw;
        if ((sw != 4 && sw != 8 && sw != 16 && sw != 32) || a->N % 32 || a->gn_c0 % 32 || a->gn_c0 < 0 ||
            a->gn_c0 + a->N > a->gn_ncb * 32 || a->gn_p64 != 0 || a->gn_np64 * 64 != 4 * a->Hm * a->Wm)
            return WC_E_SHAPE;
        d.gn_ncb = a->gn_ncb; d.gn_sw = sw; d.gn_c0 = a->gn_c0; d.gn_np64 = a->gn_np64;
    }
    const long ntn = (a->N + BN - 1) / BN;
    if (w3_bytes != ntn * 4L * 4L * d.nck0 * BN * 64 || w3_bytes >= (1L << 31)) return WC_E_SHAPE;
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    if (BN == 64) return launch6<16, 64, 0, false, true, false, false, 2>(d, st);
    return launch6<8, 128, 0, false, true, false, false, 2, true>(d, st);
}
