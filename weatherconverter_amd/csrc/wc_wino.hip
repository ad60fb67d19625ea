// ResBlock 3x3 stride-1 conv on f16x3 MFMA through a Winograd F(2,3) transform along x.
//
// The direct halo kernel (wc_conv6.hip) spends 9 MFMA K-steps per 16-channel chunk per output
// pixel.  Along x a 3-tap filter over two outputs is the minimal filtering algorithm F(2,3): with the
// four input values d0..d3 of an output pair (input columns 2t-1 .. 2t+2) and the three taps g0..g2
// of one kernel row,
//     V0 = d0 - d2,  V1 = d1 + d2,  V2 = d2 - d1,  V3 = d1 - d3            (input transform)
//     U0 = g0,  U1 = (g0 + g1 + g2) / 2,  U2 = (g0 - g1 + g2) / 2,  U3 = g2   (filter transform, host)
//     M_p = sum over (c, kernel row) of V_p U_p                               (4 GEMMs, one per p)
//     y0 = M0 + M1 + M2,  y1 = M1 - M2 - M3                                  (output transform)
// so an output pair costs 3 rows x 4 positions = 12 K-steps instead of 18: 1.5x fewer MFMAs for the
// same algorithmic work.  Along y the conv stays direct (the kernel row is a halo-row offset), which
// keeps the accumulator state at 2x the output tile and the transform VALU light.
//
// Arithmetic (f16x3, as wc_conv6.hip): V is formed in fp32 from the GN+SiLU prologue output scaled
// by 2^s (|V| <= 2 x the Samuelson bound, so the host passes the GN exponent and the kernel uses
// s = a_exp - 1), then split into two round-to-nearest fp16 pieces; U is formed in float64 on the
// host, scaled per output channel by 2^sW[n] (max |U| 2^sW <= 2^14) and split the same way.
// Products h_V h_U + h_V l_U + l_V h_U accumulate in fp32 in the MFMA.  Errors: the fp32 rounding of
// each V (one add) and of the transforms' sums, at fp32-class size (tests/test_wino.py bounds the
// whole conv against a float64 direct conv at <= 4x the direct kernel's own error).
//
// The fused 1x1 residual_input_conv (raw block input X, unet_base.py:146-150) enters the transform
// domain exactly: y0 += r(x_2t) is M0 += x_2t W_r, and y1 += r(x_2t+1) is M3 += (-x_2t+1) W_r, so
// one residual chunk is two position GEMMs sharing one weight fragment (12 MFMAs per wave, the
// direct kernel's count).
//
// Tiling.  A workgroup owns TH image rows x 16 columns (8 output pairs = "tiles" per row) x BN
// channels; each of its 4 waves owns 8 rows x 8 tiles (64 tiles = 128 pixels, two 32-row MFMA
// blocks) x 32 channels x the 4 positions: acc[4][2] = 128 accumulator registers, 2 waves per SIMD.
// Per 16-channel chunk the (TH+2) x 18 input halo is loaded once (items of one halo row x 6 pixels
// x 4 channels: two tiles), GN+SiLU-transformed, Winograd-transformed and split by VALU, and
// written to LDS as [piece][position][k-half][halo row][tile] 16-byte fragments; every K-step
// (kernel row dy, position p) then reads its A fragments at a constant halo-row offset dy.  The
// MFMA row -> (row, tile) map makes each ds_read_b128 lane group read 16 consecutive fragments
// (two image rows x 8 tiles): conflict-free.  Weight fragments go from L2 straight into three
// register sets two K-steps ahead (12 steps per chunk: the set of a step is compile-time); one
// barrier per chunk.  Residual chunks follow the 3x3 chunks (one K-step each, centre values of two
// chunks in flight).
//
// Epilogue as the direct kernel: x 2^-(s + sW[n]), + bias + temb, + residual view, NHWC store,
// GroupNorm tile partials (each wave's two 64-pixel blocks), per-image absmax.
// Reference: unet_base.py:87-109 (ResBlock convs), :146-150 (forward), SURVEY.md §8 row a3.
#include <stdlib.h>

#include "wc_x6.hpp"

// Ablation switches for timing experiments only (wrong results; tools/wino_ab.sh): bit 0 no SiLU, 1 no
// GN/SiLU prologue, 2 no halo transform/split/LDS write in the K loop, 3 no weight loads in the K loop,
// 4 no barrier in the K loop, 5 no halo loads in the K loop, 6 no A-fragment reads in the K loop, 7 no
// output stores.
#ifndef WC_ABL
#define WC_ABL 0
#endif
#ifndef WC_WINO_SCALAR
#define WC_WINO_SCALAR 0
#endif

namespace {

using namespace wcx6;

constexpr int NT = 256;

// 16 bytes per lane from a buffer straight into LDS at the wave-uniform base dst + 16 lane (device-only
// helper: the target builtin must not appear in a kernel body the host pass parses)
WC_DEVICE void wino_lds16(__amdgpu_buffer_rsrc_t srd, void* dst, unsigned voff, int soff) {
    __builtin_amdgcn_raw_ptr_buffer_load_lds(srd, (__attribute__((address_space(3))) void*)dst, 16, voff, soff, 0, 0);
}

struct WDev {
    const float* src0;
    int C0, ldc0;
    const float* scale;
    const float* shift;
    const float* src1;
    int C1, ldc1;
    int B, H, W, N;
    const void* w;
    const float* bias;
    const float* temb;
    int temb_ld;
    const float* res;
    int ldres;
    float* out;
    int ldo;
    int nck0, nck1;
    int a_exp;            // s of the transformed segment 0 (the GN exponent - 1)
    const float* abound;  // per-image bound of segment 1's raw values (or NULL without residual)
    const float* wsinv;   // 2^-sW[n]
    float* absmax;
    float* gn_part;
    int gn_ncb, gn_sw, gn_c0, gn_np64;
    int tiles_x, tiles_y, ntiles_n;
    const unsigned char* vpre;  // PRO 3: segment 0 pre-transformed and split (wino_vsplit_kernel layout)
    long vimg;                  // PRO 3: bytes of one image's V
    // PRO 0 (a training data gradient dz of a GroupNorm(+SiLU) input x): the GroupNorm backward's
    // per-channel sums of the written values (wc_conv3x3_wino_f16x3_gnb), gnb_reduce_kernel's
    // (sum dy, sum dy xhat) [, sum xhat] with xhat = x sc0 + sh0, dy = dz SiLU'(gamma xhat + beta)
    const float* gb_x;
    int gb_ldx, gb_silu;
    const float* gb_sc0;
    const float* gb_sh0;
    const float* gb_gamma;
    const float* gb_beta;
    float* gb_part;   // [B][splits][N][2], split = (tile, wave row)
    float* gb_part3;  // [B][splits][N] or NULL
};

WC_DEVICE float wino_silu_grad(float y) {  // d/dy [y sigmoid(y)], as wc_backward.hip's silu_grad
    const float s = 1.0f / (1.0f + __expf(-y));
    return s * (1.0f + y * (1.0f - s));
}

// MB: 32-tile MFMA row blocks per wave (4 image rows x 8 tiles each): 2 (two waves per SIMD) or 4 (one
// wave per SIMD, 512 registers: each weight fragment feeds twice the MFMAs, halving the vector-memory
// traffic per MFMA that the two-wave form is bound by)
// NW: waves per workgroup, 4 or 8 (one 8-wave workgroup per CU at two waves per SIMD: its halo's GN+SiLU /
// transform / split VALU and loads feed twice the MFMA work -- BN = 256 channels over 8 rows, or BN = 128
// over 16 rows).  The weights stay packed in 128-channel tiles (wc_conv3x3_wino_tile_n): a 256-channel
// workgroup reads two of them.
// Planes of the pre-split layout per 16-channel chunk: (piece 2) x (position 4) x (k-half 2), or in the
// single-piece builds (WC_SINGLE16: the 16-bit training lines, one piece per operand) the high piece's 8
// planes only -- the low piece is zero there, so the pass writes and the conv copies half the bytes.
constexpr int VPL = WC_SINGLE16 ? 8 : 16;

template <int TH, int BN, int MB = 2, int NW = 4, bool VP = false>
struct WTile {
    static constexpr int NT = 64 * NW;
    static constexpr int WAVES_N = BN / 32;
    static constexpr int WAVES_M = NW / WAVES_N;
    static_assert(WAVES_N * WAVES_M == NW && WAVES_M * 4 * MB == TH, "each wave owns 4 MB rows x 8 tiles x 32 channels");
    static constexpr int PBN = BN > 128 ? 128 : BN;  // channels per packed weight tile
    static constexpr int HR = TH + 2;            // halo rows
    // one (piece, position, k-half) plane of [halo row][tile] 16-byte fragments; the 16 extra bytes make
    // the k-half stride 16 mod 128 so the item writes of a 16-lane group hit 16 distinct 8-byte slots
    // (VP, PRO 3: the planes arrive by LDS-DMA in 1-KiB pieces, no item writes: no pad, planes contiguous)
    static constexpr int PSTR = HR * 128 + (VP ? 0 : 16);
    // VP: the chunk's VPL planes of HR rows x 8 tiles arrive as 1-KiB LDS-DMA pieces, piece i of wave w is
    // w + NW i (the last round partial when the count is not a multiple of NW)
    static constexpr int DPIECES = VPL * HR * 8 / 64;
    static_assert(!VP || VPL * HR * 8 == DPIECES * 64, "VP: the halo stage is a whole number of 1-KiB pieces");
    static constexpr int DPW = (DPIECES + NW - 1) / NW;
    static constexpr int HSTAGE = 16 * PSTR;     // planes (piece 2) x (position 4) x (k-half 2)
    static constexpr int CPSTR = TH * 128 + 16;  // residual centre plane ([row][tile])
    static constexpr int CSTAGE = 8 * CPSTR;     // (piece 2) x (position 0 / 3) x (k-half 2)
    static constexpr int ITEMS = HR * 16;        // (halo row, tile pair, channel quad)
    static constexpr int I_PER_T = (ITEMS + NT - 1) / NT;
    static constexpr int C_PER_T = TH * 16 * 4 / NT;  // centre float4 items per thread
    static constexpr int BSTEP = PBN * 64;       // weight bytes of one K-step: [piece 2][k-half 2][PBN][8]
    static constexpr int STEPS = 12;             // (kernel row, position) per chunk
};

// MFMA row r (0..31) -> (row, tile) of a 4-row x 8-tile block: the ds_read_b128 lane group
// {0-3, 12-15, 20-27} reads rows 0-1 x tiles 0-7 (16 consecutive fragments), {4-11, 16-19, 28-31}
// rows 2-3.  (grp, idx) as wc_conv6.hip's row_dy / row_dx.
WC_DEVICE int wg_grp(int r) { return ((r >= 4 && r < 12) || (r >= 16 && r < 20) || r >= 28) ? 1 : 0; }
WC_DEVICE int wg_idx(int r) { return r < 4 ? r : r < 12 ? r - 4 : r < 20 ? r - 8 : r < 28 ? r - 12 : r - 16; }
WC_DEVICE int wg_row(int r) { return 2 * wg_grp(r) + (wg_idx(r) >> 3); }
WC_DEVICE int wg_tile(int r) { return wg_idx(r) & 7; }

// PRO: 2 = GroupNorm affine + SiLU prologue on segment 0 (static Samuelson bound), 0 = raw segment 0
// under the per-image bound abound (the training data gradients), 3 = segment 0 already GN+SiLU'd,
// Winograd-transformed and split by wino_vsplit_kernel (the same arithmetic, once per input instead of
// once per output-channel tile): its halo planes are copied into LDS by LDS-DMA, no item VALU.  RES: the
// fused 1x1 residual segment (raw input, f16x3 under the per-image bound abound).
template <int TH, int BN, int PRO, bool RES, int MB = 2, int NW = 4>
__global__ __launch_bounds__(64 * NW) __attribute__((amdgpu_waves_per_eu(MB == 4 ? 1 : 2, MB == 4 ? 1 : 2)))
void conv3x3_wino_kernel(WDev p) {
    static_assert((PRO == 2 || PRO == 0 || PRO == 3) && !(PRO == 0 && RES),
                  "GN+SiLU (+ residual), pre-split GN+SiLU (+ residual) or one raw segment");
    constexpr bool VP = PRO == 3;
    using T = WTile<TH, BN, MB, NW, VP>;
    constexpr int NT = T::NT;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    unsigned char* const cbase = smem + 2 * T::HSTAGE;  // residual centre buffers

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;
    const int wm = wave / T::WAVES_N;
    const int wn = wave % T::WAVES_N;

    // XCD-aware bijective tile order (wc_conv6.hip): consecutive logical tiles on one XCD's L2
    const int nblk = gridDim.x;
    int bid = blockIdx.x;
    {
        int q = nblk / 8, r = nblk % 8, xcd = bid % 8;
        bid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + bid / 8;
    }
    const int tile_n = bid % p.ntiles_n;
    int tt = bid / p.ntiles_n;
    const int txi = tt % p.tiles_x;
    tt /= p.tiles_x;
    const int tyi = tt % p.tiles_y;
    const int b = tt / p.tiles_y;
    const int y0 = tyi * TH, x0 = txi * 16, n0 = tile_n * BN;

    // s: the transformed segment 0 needs |V| 2^s <= 2^14 (p.a_exp already counts V's doubling); a raw
    // value under the per-image bound needs bound * 2^s < 2^14 (residual: s <= 13 - e; a raw segment 0,
    // doubled by the transform: s <= 12 - e)
    int s_exp = p.a_exp;
    if ((RES || PRO == 0) && p.abound) {
        const float bnd = p.abound[b];
        const int e = (int)((__float_as_uint(bnd) >> 23) & 0xffu) - 127;
        if (bnd > 0.f) s_exp = min(s_exp, (PRO == 0 ? 12 : 13) - e);
        s_exp = max(s_exp, -100);
    }
    const float ascale = ldexpf(1.0f, s_exp), ainv = ldexpf(1.0f, -s_exp);
    const int S0 = T::STEPS * p.nck0;
    const int S = S0 + (RES ? p.nck1 : 0);
    // residual chunk r < nri rides in 3x3 chunk r as a 13th K-step; the rest (nck1 > nck0) follow as a
    // tail phase, one K-step and one barrier each
    // (TH = 16: the centre staging of four items per thread does not fit beside the halo's; all tail)
    constexpr bool RI = RES && (T::C_PER_T <= 2 || MB == 4);
    const int nri = RI ? min(p.nck0, p.nck1) : 0;
    const int ntail = RES ? p.nck1 - nri : 0;
    constexpr int WPT = T::PBN / 32;  // waves per packed weight tile
    const unsigned wtile = (unsigned)(tile_n * (BN / T::PBN) + wn / WPT) * (unsigned)(S * T::BSTEP);

    const __amdgpu_buffer_rsrc_t srd0 = make_srd(p.src0);
    const __amdgpu_buffer_rsrc_t srd1 = make_srd(RES ? p.src1 : p.src0);
    const __amdgpu_buffer_rsrc_t srdw = make_srd(p.w);
    const __amdgpu_buffer_rsrc_t srdsc = make_srd(PRO == 2 ? p.scale : p.src0);
    const __amdgpu_buffer_rsrc_t srdsh = make_srd(PRO == 2 ? p.shift : p.src0);
    // VP: this image's pre-split planes [chunk][plane VPL][row H][tile W/2] x 16 B; per-lane byte offsets
    // of this wave's LDS-DMA pieces (chunk 0; a chunk is a scalar offset), OOB for halo rows outside
    // the image (the load returns zeros: the padding rows' V)
    const __amdgpu_buffer_rsrc_t srdv = make_srd(VP ? (const void*)(p.vpre + (long)b * p.vimg) : (const void*)p.src0);
    unsigned voff[VP ? T::DPW : 1];
    if constexpr (VP) {
#pragma unroll
        for (int i = 0; i < T::DPW; ++i) {
            const int f = (wave + NW * i) * 64 + lane;  // 16-byte fragment of the stage
            const int P = f / (T::HR * 8), r = (f >> 3) % T::HR, tl = f & 7;
            const int y = y0 - 1 + r;
            voff[i] = (unsigned)y < (unsigned)p.H ? (unsigned)(((P * p.H + y) * (p.W / 2) + (x0 >> 1) + tl) * 16) : OOB;
        }
    }
    const int vchunk = VPL * p.H * (p.W / 2) * 16;  // bytes of one 16-channel chunk's planes
    auto dma_halo = [&](int c, int hs) {
        if constexpr (VP) {
            unsigned char* dst = smem + hs * T::HSTAGE + wave * 1024;
#pragma unroll
            for (int i = 0; i < T::DPW; ++i)
                if (T::DPIECES % NW == 0 || wave + NW * i < T::DPIECES)  // wave-uniform: the partial last round
                    wino_lds16(srdv, dst + i * NW * 1024, voff[i], c * vchunk);
        }
    };

    // ---- halo items: item i = tid + NT j = (halo row i >> 4, tile pair (i >> 2) & 3, quad i & 3) ----
    const int q = tid & 3;
    int hbase[T::I_PER_T];  // byte offset of the item's first pixel (chunk 0); OOB pixels re-masked per load
    unsigned hin[T::I_PER_T];
    int hwr[T::I_PER_T];  // LDS byte offset of the item's (piece 0, position 0) fragment slot
    const int hpx = p.ldc0 * 4;  // bytes between horizontally adjacent pixels
#pragma unroll
    for (int j = 0; j < T::I_PER_T; ++j) {
        // item tid + NT j: the items fill waves 0 .. in order (spreading them thinner over all four waves
        // would not shorten any wave's instruction stream, only add wave 3's)
        const int i = tid + NT * j;
        const int hrow = i >> 4, tp = (i >> 2) & 3;
        const bool valid = i < T::ITEMS;
        const int iy = y0 - 1 + hrow;
        hin[j] = 0;
#pragma unroll
        for (int k = 0; k < 6; ++k) {
            const int ix = x0 - 1 + 4 * tp + k;
            const bool inb = valid && (unsigned)iy < (unsigned)p.H && (unsigned)ix < (unsigned)p.W;
            hin[j] |= (inb ? 1u : 0u) << k;
        }
        hbase[j] = (((b * p.H + iy) * p.W + x0 - 1 + 4 * tp) * p.ldc0 + 4 * q) * 4;
        hwr[j] = valid ? (q >> 1) * T::PSTR + (hrow * 8 + 2 * tp) * 16 + (q & 1) * 8 : -1;
    }
    f32x4 rh[T::I_PER_T][6];
    f32x4 rsc, rsh;
    auto load_ss = [&](int c) {
        if constexpr (PRO == 2) {
            const unsigned o = (unsigned)(b * p.C0 + c * 16 + 4 * q) * 4u;
            rsc = bload_f4(srdsc, o);
            rsh = bload_f4(srdsh, o);
        }
    };
    auto load_slot = [&](int j, int c) {  // item slot j of chunk c (every load issued; OOB pixels read 0)
#pragma unroll
        for (int k = 0; k < 6; ++k)
            rh[j][k] = bload_f4s(srd0, ((hin[j] >> k) & 1u) ? (unsigned)(hbase[j] + k * hpx) : OOB, c * 64);
    };
    auto load_halo = [&](int c) {
        if constexpr (VP) return;
#pragma unroll
        for (int j = 0; j < T::I_PER_T; ++j) load_slot(j, c);
        load_ss(c);
    };
    // GN + SiLU prologue of pixels k0 .. k1 - 1 of slot j, in place (zero padding after it), x 2^s
#if WC_WINO_SCALAR
    // Scalar form (no packed-f32 VALU: v_pk_fma / v_pk_mul cost several times a plain VALU op beside
    // MFMAs, MI355X_MICROARCH.md): the chunk's GN scale / shift are pre-multiplied by 2^s once, so
    // a' = x sc' + sh' = (x sc + sh) 2^s exactly, the exp2 argument is a' (-log2 e 2^-s) = a (-log2 e)
    // exactly, and a' / (1 + 2^u) = SiLU(a) 2^s: the same bits as the vector form, one multiply fewer.
    const float cu = -1.4426950408889634f * ainv;
    auto prologue = [&](int j, int k0, int k1) {
        if constexpr (PRO == 2) {
            if (j == 0 && k0 == 0) {
                rsc = rsc * ascale;
                rsh = rsh * ascale;
            }
        }
        auto act = [&](f32x4 a) {
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                float v;
                if constexpr (PRO == 2) {
                    const float ap = __builtin_fmaf(a[e], rsc[e], rsh[e]);
                    const float r = __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(ap * cu));
                    v = ap * r;
                } else {
                    v = a[e] * ascale;
                }
                a[e] = v;
            }
            return a;
        };
#pragma unroll
        for (int k = k0; k < k1; ++k) {
            const f32x4 zero = {0.f, 0.f, 0.f, 0.f};
#if WC_WINO_SCALAR == 2
            // the select over the expression itself: clang branches around each pixel's activation
            rh[j][k] = ((hin[j] >> k) & 1u) ? act(rh[j][k]) : zero;
#else
            const f32x4 a = act(rh[j][k]);
            rh[j][k] = ((hin[j] >> k) & 1u) ? a : zero;
#endif
        }
    };
#else
    auto prologue = [&](int j, int k0, int k1) {
#pragma unroll
        for (int k = k0; k < k1; ++k) {
            f32x4 a = rh[j][k];
            if constexpr (PRO == 2 && !(WC_ABL & 2)) {
                a = a * rsc + rsh;
                if constexpr (!(WC_ABL & 1)) {
                    a.x = silu_fast(a.x); a.y = silu_fast(a.y);
                    a.z = silu_fast(a.z); a.w = silu_fast(a.w);
                }
            }
            rh[j][k] = ((hin[j] >> k) & 1u) ? a * ascale : f32x4{0.f, 0.f, 0.f, 0.f};
        }
    };
#endif
    // Winograd input transform of tile t (0, 1) of slot j, 2-piece fp16 split, 8 fragment writes into
    // halo buffer hs
    auto transform = [&](int j, int t, int hs, int p0 = 0, int p1 = 4) {
        if (hwr[j] < 0) return;  // idle item slot (ITEMS is not a multiple of NT)
        unsigned char* base = smem + hs * T::HSTAGE + hwr[j] + t * 16;
        const f32x4 d0 = rh[j][2 * t], d1 = rh[j][2 * t + 1], d2 = rh[j][2 * t + 2], d3 = rh[j][2 * t + 3];
#if WC_WINO_SCALAR
        f32x4 V[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            V[0][e] = d0[e] - d2[e];
            V[1][e] = d1[e] + d2[e];
            V[2][e] = d2[e] - d1[e];
            V[3][e] = d1[e] - d3[e];
        }
#else
        const f32x4 V[4] = {d0 - d2, d1 + d2, d2 - d1, d1 - d3};
#endif
#pragma unroll
        for (int pos = p0; pos < p1; ++pos) {
            u32x2 a0, a1;
            split2_f16(V[pos], a0, a1);
            unsigned char* d = base + pos * 2 * T::PSTR;
            *reinterpret_cast<u32x2*>(d) = a0;
            *reinterpret_cast<u32x2*>(d + 8 * T::PSTR) = a1;
        }
    };
    auto write_items = [&](int hs) {
        if constexpr (VP) return;
#pragma unroll
        for (int j = 0; j < T::I_PER_T; ++j) {
            prologue(j, 0, 6);
            transform(j, 0, hs);
            transform(j, 1, hs);
        }
    };

    // ---- residual centre items: item i = tid + NT j = (row i >> 6, pixel (i >> 2) & 15, quad i & 3) ----
    f32x4 rc[2][RES ? T::C_PER_T : 1];
    const int cpx = (tid >> 2) & 15, crow0 = tid >> 6;  // item j: row crow0 + NW j
    const unsigned coff0 = (unsigned)(((b * p.H + y0 + crow0) * p.W + x0 + cpx) * p.ldc1 + 4 * q);
    const unsigned cstep = (unsigned)(NW * p.W * p.ldc1);
    // position 0 takes x at even columns, position 3 takes -x at odd columns (plane index 1)
    const int cwr0 = (cpx & 1) * 2 * T::CPSTR + (q >> 1) * T::CPSTR + (crow0 * 8 + (cpx >> 1)) * 16 + (q & 1) * 8;
    // live = false: the same loads at an out-of-range offset (zeros, no traffic): every load is issued
    // unconditionally (a load behind a runtime branch makes the compiler drain vmcnt at the join)
    auto load_centre = [&](auto P, int c, bool live = true) {
        constexpr int PV = decltype(P)::value;
        const unsigned v = live ? coff0 * 4u : OOB;
#pragma unroll
        for (int j = 0; j < T::C_PER_T; ++j)
            rc[PV][j] = bload_f4s(srd1, v, (int)(((unsigned)j * cstep + (unsigned)c * 16u) * 4u));
    };
    auto write_centre = [&](auto P, int cs) {
        constexpr int PV = decltype(P)::value;
        unsigned char* base = cbase + cs * T::CSTAGE + cwr0;
        const float sg = (cpx & 1) ? -ascale : ascale;
#pragma unroll
        for (int j = 0; j < T::C_PER_T; ++j) {
            u32x2 a0, a1;
            split2_f16(rc[PV][j] * sg, a0, a1);
            unsigned char* d = base + j * NW * 8 * 16;  // + NW rows
            *reinterpret_cast<u32x2*>(d) = a0;
            *reinterpret_cast<u32x2*>(d + 4 * T::CPSTR) = a1;
        }
    };

    // ---- fragment addressing ----
    const int l32 = lane & 31;
    const int half = lane >> 5;
    int abase[MB];
#pragma unroll
    for (int mb = 0; mb < MB; ++mb) abase[mb] = ((4 * MB * wm + 4 * mb + wg_row(l32)) * 8 + wg_tile(l32)) * 16;
    const unsigned wlane = (unsigned)(half * T::PBN * 16 + ((wn % WPT) * 32 + l32) * 16);

    u32x4 wreg[3][2];  // [set][piece]
    // weight fragments of K-step st (past the end: the last step again, unused): issued unconditionally
    // weight fragments of 3x3 K-step st (st >= S0: tail residual step st - S0; past the end: the last
    // step again, unused): issued unconditionally
    auto load_w = [&](int set, int st) {
        int s = st < S0 ? st : S0 + nri + (st - S0);
        s = s < S ? s : S - 1;
        const int off = (int)(wtile + (unsigned)s * T::BSTEP);
#pragma unroll
        for (int pc = 0; pc < 2; ++pc) wreg[set][pc] = bload_u4s(srdw, wlane + (unsigned)(pc * 2 * T::PBN * 16), off);
    };
    u32x4 wres[2];  // the interleaved residual step's weights (their own set: the 3-set cycle stays 12-periodic)
    auto load_wres = [&](int r) {
        const int s = S0 + r < S ? S0 + r : S - 1;
        const int off = (int)(wtile + (unsigned)s * T::BSTEP);
#pragma unroll
        for (int pc = 0; pc < 2; ++pc) wres[pc] = bload_u4s(srdw, wlane + (unsigned)(pc * 2 * T::PBN * 16), off);
    };

    f32x16 acc[4][MB];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < MB; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

    // K-step (kernel row dy, position pos) of the chunk in halo buffer hs, weights in set
    // A fragments of a K-step, two register sets: the fragments of step st + 1 are read from LDS while
    // step st's MFMAs run (a step is only 6 MFMAs per wave; reading its own fragments at its head left
    // the LDS latency exposed at every step)
    u32x4 fa[2][MB][2];  // [set][mb][piece]
    auto read_a = [&](int fs, int hs, int dy, int pos) {
        const unsigned char* ha = smem + hs * T::HSTAGE + (pos * 2 + half) * T::PSTR + dy * 128;
#pragma unroll
        for (int mb = 0; mb < MB; ++mb)
#pragma unroll
            for (int pc = 0; pc < 2; ++pc)
                fa[fs][mb][pc] = *reinterpret_cast<const u32x4*>(ha + pc * 8 * T::PSTR + abase[mb]);
    };
    auto mfma_a = [&](int fs, int set, int pos) {
#pragma unroll
        for (int mb = 0; mb < MB; ++mb) acc[pos][mb] = mfma_f16(fa[fs][mb][0], wreg[set][0], acc[pos][mb]);
#pragma unroll
        for (int mb = 0; mb < MB; ++mb) {
            acc[pos][mb] = mfma_f16c(fa[fs][mb][0], wreg[set][1], acc[pos][mb]);
            acc[pos][mb] = mfma_f16c(fa[fs][mb][1], wreg[set][0], acc[pos][mb]);
        }
    };
    // residual K-step: positions 0 and 3 from centre buffer cs, one weight fragment
    auto compute_res = [&](const u32x4 (&w)[2], int cs) {
        const unsigned char* ca = cbase + cs * T::CSTAGE + half * T::CPSTR;
#pragma unroll
        for (int r = 0; r < 2; ++r) {  // position 0 (x_even), position 3 (-x_odd): 16 fragment registers at a time
            u32x4 fr[MB][2];  // [mb][piece]
#pragma unroll
            for (int mb = 0; mb < MB; ++mb)
#pragma unroll
                for (int pc = 0; pc < 2; ++pc)
                    fr[mb][pc] = *reinterpret_cast<const u32x4*>(ca + (pc * 4 + r * 2) * T::CPSTR + abase[mb]);
#pragma unroll
            for (int mb = 0; mb < MB; ++mb) {
                f32x16& a = acc[r ? 3 : 0][mb];
                a = mfma_f16(fr[mb][0], w[0], a);
                a = mfma_f16c(fr[mb][0], w[1], a);
                a = mfma_f16c(fr[mb][1], w[0], a);
            }
        }
    };

    const std::integral_constant<int, 0> I0;
    const std::integral_constant<int, 1> I1;
    // ---- K loop over the 3x3 chunks: chunk c in halo buffer c & 1; step st of a chunk uses weight
    // set st % 3 (12 steps per chunk), the weights of step st + 2 are issued at its head ----
    // Chunk c uses halo buffer (nck0 - 1 - c) & 1, counted from the end, so the peeled last chunk is one
    // compile-time variant flowing into the epilogue (two variants joining there make the register
    // allocator spill, as in wc_conv6.hip)
    const int pv0 = (p.nck0 - 1) & 1;
    load_halo(0);
    dma_halo(0, pv0);
    if constexpr (RI) load_centre(I0, 0, nri > 0);
    load_w(0, 0);
    load_w(1, 1);
    write_items(pv0);
    if constexpr (RI) write_centre(I0, pv0);
    if constexpr (VP) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's LDS-DMA pieces landed
    __syncthreads();
    // The next chunk's halo item slot j goes out at step load_at(j) (after that step's weight loads:
    // vmcnt drains in issue order, so the weight waits of the following steps wait for it only from
    // three steps later); its prologue (step pro_at(j)) and transform (tiles 0 / 1 at the next two
    // steps) run under the MFMAs of those steps, into the other halo buffer, which nobody reads this
    // chunk.  One slot (TH = 8): loads at 6, VALU at 9-11; two (TH = 16): 4 / 6-8 and 7 / 9-11.  The
    // next chunk's residual centre rides with slot 0 and is split into the other centre buffer at step 11;
    // this chunk's residual step (weights from step 7) runs after step 11.
    // One slot (TH = 8): the halo goes out at step 2 and its VALU is spread thin over steps 5-11 (prologue
    // two pixels a step at 5-7, then each tile's positions 0-1 / 2-3 a step at 8-11), so that it fits the
    // vector-issue slots the MFMAs leave.  Two slots (TH = 16, registers for both only briefly): slot 0
    // loads at 3, prologue at 5, tiles at 6 and 7; slot 1 loads at 7, prologue at 9, tiles at 10 and 11.
    constexpr int HALO_AT = T::I_PER_T == 1 ? 2 : 3;
    auto load_at = [](int j) { return T::I_PER_T == 1 ? 2 : (j == 0 ? 3 : 7); };
    auto pro_at = [](int j) { return j == 0 ? 5 : 9; };
    // the slot's VALU at step st (relative step k = st - pro_at(j))
    auto slot_work = [&](int j, int k, int hs) {
        if constexpr (VP) return;
        if constexpr (WC_ABL & 4) {
            if (k >= 0 && k < 3) prologue(j, 2 * k, 2 * k + 2);
            return;
        }
        if constexpr (T::I_PER_T == 1) {
            if (k >= 0 && k < 3) prologue(j, 2 * k, 2 * k + 2);
            if (k >= 3 && k < 7) transform(j, (k - 3) >> 1, hs, ((k - 3) & 1) * 2, ((k - 3) & 1) * 2 + 2);
        } else {
            if (k == 0) prologue(j, 0, 6);
            if (k == 1 || k == 2) transform(j, k - 1, hs);
        }
    };
    auto chunk = [&](auto P, auto L, int c) {
        constexpr int PV = decltype(P)::value;
        constexpr bool LAST = decltype(L)::value != 0;
        read_a(0, PV, 0, 0);  // step 0's fragments (the halo buffer was written before the last barrier)
#pragma unroll
        for (int st = 0; st < T::STEPS; ++st) {
            if (!(WC_ABL & 8) || c == 0) load_w((st + 2) % 3, T::STEPS * c + st + 2);
            if constexpr (!LAST) {
#pragma unroll
                for (int j = 0; j < T::I_PER_T; ++j)
                    if (!(WC_ABL & 32) && st == load_at(j)) load_slot(j, c + 1);
                if (st == HALO_AT) {
                    dma_halo(c + 1, PV ^ 1);
                    load_ss(c + 1);
                    if constexpr (RI) load_centre(I0, c + 1, c + 1 < nri);
                }
            } else if constexpr (RES) {  // the tail's first two centres
                if (st == HALO_AT) load_centre(I0, nri, ntail > 0);
                if (st == HALO_AT + 1) load_centre(I1, nri + 1, ntail > 1);
            }
            if constexpr (RI) {
                if (st == 9) load_wres(c);
            }
            __builtin_amdgcn_sched_barrier(0);
            if (st + 1 < T::STEPS && (!(WC_ABL & 64) || c == 0)) read_a((st + 1) & 1, PV, (st + 1) >> 2, (st + 1) & 3);
            mfma_a(st & 1, st % 3, st & 3);
            if constexpr (!LAST) {
#pragma unroll
                for (int j = 0; j < T::I_PER_T; ++j) slot_work(j, st - pro_at(j), PV ^ 1);
                if constexpr (RI) {
                    if (st == 9) write_centre(I0, PV ^ 1);
                }
            }
        }
        if constexpr (RES) {
            if constexpr (RI) {
                if (c < nri) compute_res(wres, PV);
            }
            if constexpr (LAST) {
                if (ntail > 0) write_centre(I0, 1);  // tail chunk k in centre buffer (k + 1) & 1
            }
        }
        // VP: this wave's LDS-DMA pieces of the next chunk (issued at step HALO_AT, followed by at least
        // 18 weight loads) have landed once at most the last 4 vector-memory ops (the next chunk's first
        // two weight steps) are outstanding: vmcnt counts loads in issue order
        if constexpr (VP && !LAST) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
        if constexpr (!(WC_ABL & 16)) __syncthreads();
    };
    const std::integral_constant<int, 0> NL;
    const std::integral_constant<int, 1> LL;
    {
        int c = 0;
        if (pv0) chunk(I1, NL, c++);
        for (; c + 1 < p.nck0 - 1; c += 2) {
            chunk(I0, NL, c);
            chunk(I1, NL, c + 1);
        }
        chunk(I0, LL, p.nck0 - 1);
    }
    if constexpr (RES) {
        // tail residual chunk nri + k: weights in set k & 1 (the last 3x3 chunk's prefetch put tail steps 0
        // and 1 in sets 0 and 1; from here the load of step k + 2 is issued after step k's MFMAs), centre
        // registers k & 1, centre buffer (k + 1) & 1
        auto tstep = [&](auto P, int k) {
            constexpr int PV = decltype(P)::value;
            compute_res(wreg[PV], PV ^ 1);
            load_w(PV, S0 + k + 2);
            load_centre(P, nri + k + 2, k + 2 < ntail);
            __builtin_amdgcn_sched_barrier(0);
            if (k + 1 < ntail) write_centre(std::integral_constant<int, PV ^ 1>{}, PV);
            __syncthreads();
        };
        int k = 0;
        for (; k + 1 < ntail; k += 2) {
            tstep(I0, k);
            tstep(I1, k + 1);
        }
        if (k < ntail) tstep(I0, k);
    }

    // ---- epilogue: output transform, x 2^-(s + sW[n]), + bias + temb, + residual view, NHWC store ----
    const long img_px = (long)b * p.H * p.W;
    const __amdgpu_buffer_rsrc_t srd_out = make_srd(p.out + img_px * p.ldo);
    const __amdgpu_buffer_rsrc_t srd_res = make_srd(p.res ? p.res + img_px * p.ldres : p.out);
    const int n = n0 + wn * 32 + l32;
    const bool nok = n < p.N;
    float eadd = (nok && p.bias) ? p.bias[n] : 0.f;
    if (nok && p.temb) eadd += p.temb[b * p.temb_ld + n];
    const float emul = nok ? p.wsinv[n] * ainv : 0.f;
    float vmax = 0.f;
    float gs1 = 0.f, gs2 = 0.f, gs3 = 0.f;  // GroupNorm-backward sums of this lane's channel (PRO 0)
    // accumulator register r of block mb is MFMA row (r & 3) + 8 (r >> 2) + 4 half: the four registers of
    // a group j = r >> 2 are four consecutive tiles of one image row.  One per-lane byte offset per
    // (mb, j) and the tile steps (r & 3) x 2 pixels as wave-uniform scalar offsets: no per-store VALU.
    const int so_px = 4 * p.ldo;  // bytes between horizontally adjacent output pixels
    const int so_rs = 4 * p.ldres;
#pragma unroll
    for (int mb = 0; mb < MB; ++mb) {
        unsigned vo[4], vr[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int row = 8 * j + 4 * half;
            const int pix = (y0 + 4 * MB * wm + 4 * mb + wg_row(row)) * p.W + x0 + 2 * wg_tile(row);
            vo[j] = (unsigned)(pix * p.ldo + n) * 4u;
            vr[j] = (unsigned)(pix * p.ldres + (nok ? n : 0)) * 4u;
        }
        float rv[2][16];
        if (p.res) {
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                rv[0][r] = bload_f1s(srd_res, vr[r >> 2], (r & 3) * 2 * so_rs);
                rv[1][r] = bload_f1s(srd_res, vr[r >> 2], ((r & 3) * 2 + 1) * so_rs);
            }
        }
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const float m0 = acc[0][mb][r], m1 = acc[1][mb][r], m2 = acc[2][mb][r], m3 = acc[3][mb][r];
            float ya = ((m0 + m1) + m2) * emul + eadd;
            float yb = ((m1 - m2) - m3) * emul + eadd;
            if (p.res) {
                ya += rv[0][r];
                yb += rv[1][r];
            }
            acc[0][mb][r] = ya;
            acc[1][mb][r] = yb;
            vmax = fmaxf(vmax, fmaxf(fabsf(ya), fabsf(yb)));
        }
        if constexpr (PRO == 0) {
            if (p.gb_part) {  // the same 32 values against x at the same pixels (loads issued first)
                const __amdgpu_buffer_rsrc_t srd_x = make_srd(p.gb_x + img_px * p.gb_ldx);
                const int so_x = 4 * p.gb_ldx;
                float xv[2][16];
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int j = r >> 2;
                    const int row = 8 * j + 4 * half;
                    const int pix = (y0 + 4 * MB * wm + 4 * mb + wg_row(row)) * p.W + x0 + 2 * wg_tile(row);
                    const unsigned vx = nok ? (unsigned)(pix * p.gb_ldx + n) * 4u : OOB;
                    xv[0][r] = bload_f1s(srd_x, vx, (r & 3) * 2 * so_x);
                    xv[1][r] = bload_f1s(srd_x, vx, ((r & 3) * 2 + 1) * so_x);
                }
                const long bn = (long)b * p.N + (nok ? n : 0);
                const float sc0 = p.gb_sc0[bn], sh0 = p.gb_sh0[bn];
                const float ga = p.gb_gamma ? p.gb_gamma[nok ? n : 0] : 1.f;
                const float be = p.gb_beta ? p.gb_beta[nok ? n : 0] : 0.f;
#pragma unroll
                for (int r = 0; r < 16; ++r)
#pragma unroll
                    for (int e = 0; e < 2; ++e) {
                        const float xh = xv[e][r] * sc0 + sh0;
                        float d = acc[e][mb][r];
                        if (p.gb_silu) d *= wino_silu_grad(ga * xh + be);
                        gs1 += d;
                        gs2 += d * xh;
                        gs3 += xh;
                    }
            }
        }
        if (nok) {
            if constexpr (WC_ABL & 128) {  // ablation: no output stores (one store only if a sum hits a magic value)
                float sum = 0.f;
#pragma unroll
                for (int r = 0; r < 16; ++r) sum += acc[0][mb][r] + acc[1][mb][r];
                if (sum == 1234.5678f) bstore_f1s(srd_out, vo[0], 0, sum);
            } else {
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    bstore_f1s(srd_out, vo[r >> 2], (r & 3) * 2 * so_px, acc[0][mb][r]);
                    bstore_f1s(srd_out, vo[r >> 2], ((r & 3) * 2 + 1) * so_px, acc[1][mb][r]);
                }
            }
        }
    }
    if (!nok) vmax = 0.f;
    if (p.absmax) block_absmax_atomic(p.absmax, b, vmax);
    if constexpr (PRO == 0) {
        if (p.gb_part) {  // the two lanes of a channel (rows 0-3 / 4-7 of each block) add, lane half 0 writes
            gs1 += __shfl_xor(gs1, 32, 64);
            gs2 += __shfl_xor(gs2, 32, 64);
            gs3 += __shfl_xor(gs3, 32, 64);
            const int splits = p.tiles_y * p.tiles_x * T::WAVES_M;
            const long sp = (long)b * splits + ((long)tyi * p.tiles_x + txi) * T::WAVES_M + wm;
            if (nok && half == 0) {
                p.gb_part[(sp * p.N + n) * 2] = gs1;
                p.gb_part[(sp * p.N + n) * 2 + 1] = gs2;
                if (p.gb_part3) p.gb_part3[sp * p.N + n] = gs3;
            }
        }
    }
    if (p.gn_part) {
        // this wave's 64-pixel blocks (4 rows x 16 px each), numbered by pixel position alone (image 4-row
        // block r4 -> ((r4 / 2) * tiles_x + tile x) * 2 + r4 % 2), so every tile height / wave form writes the
        // same partial to the same slot and the GroupNorm merge order (and result) does not depend on the form
        const int r4 = tyi * (TH / 4) + MB * wm;
#pragma unroll
        for (int mb = 0; mb < MB; ++mb) {
            const f32x16 blk[2][1] = {{acc[0][mb]}, {acc[1][mb]}};
            GnTile g{p.gn_part, p.gn_ncb, p.gn_sw,
                     (long)b * p.gn_np64 + (long)(((r4 + mb) >> 1) * p.tiles_x + txi) * 2 + ((r4 + mb) & 1),
                     (p.gn_c0 + n0 + wn * 32) / 32};
            gn_tile_partials(blk, g, p.N - n0 - wn * 32 >= 32 ? 1 : 0);
        }
    }
}

template <int TH, int BN, int PRO, bool RES, int MB = 2, int NW = 4>
int launch_wino(const WDev& d, hipStream_t stream) {
    using T = WTile<TH, BN, MB, NW, PRO == 3>;  // the layout the kernel itself uses (PRO 3: unpadded planes)
    constexpr int lds = 2 * T::HSTAGE + (RES ? 2 * T::CSTAGE : 0);
    static bool attr_set = false;  // > 64 KiB of dynamic LDS needs an explicit opt-in
    if (!attr_set) {
        hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&conv3x3_wino_kernel<TH, BN, PRO, RES, MB, NW>),
                                           hipFuncAttributeMaxDynamicSharedMemorySize, lds);
        if (e != hipSuccess) return (int)e;
        attr_set = true;
    }
    WDev p = d;
    p.tiles_x = p.W / 16;
    p.tiles_y = p.H / TH;
    p.ntiles_n = (p.N + BN - 1) / BN;
    dim3 grid(p.B * p.tiles_y * p.tiles_x * p.ntiles_n);
    WC_SET_NAME("conv3x3_wino_kernel", {WC_TI(TH), WC_TI(BN), WC_TI(PRO), WC_TB(RES), WC_TI(MB), WC_TI(NW)});
    hipLaunchKernelGGL((conv3x3_wino_kernel<TH, BN, PRO, RES, MB, NW>), grid, dim3(T::NT), lds, stream, p);
    WC_CHECK_LAUNCH();
    return WC_OK;
}

}  // namespace

extern "C" int wc_conv3x3_wino_tile_n(int N) { return N <= 64 ? 64 : 128; }

namespace {

// Argument checks and the kernel parameters shared by wc_conv3x3_wino_f16x3 and its pre-split form.
int wino_setup(const wc_conv_args* a, const void* w, int64_t w_bytes, int a_exp, const float* w_inv_scale,
               const float* a_bound, WDev& d, int& pro, bool& res, int& BN) {
    if (!a || !w || !a->out || !w_inv_scale) return WC_E_ARG;
    if (a->nseg < 1 || a->nseg > 2) return WC_E_ARG;
    const wc_conv_seg& s0 = a->seg[0];
    if (!s0.src || (s0.scale == nullptr) != (s0.shift == nullptr)) return WC_E_ARG;
    // segment 0: the GN + SiLU prologue (its static bound), or one raw segment under a_bound
    pro = s0.scale ? 2 : 0;
    if (pro == 2 && !s0.silu) return WC_E_ARG;
    if (pro == 0 && (!a_bound || a->nseg != 1)) return WC_E_ARG;
    if (a->act != WC_ACT_NONE) return WC_E_ARG;
    if (a_exp < -60 || a_exp > 60) return WC_E_ARG;
    BN = wc_conv3x3_wino_tile_n(a->N);
    const int TH = BN == 64 ? 16 : 8;
    if (s0.ntaps != 9 || s0.sy != 1 || s0.sx != 1 || s0.kbase != 0) return WC_E_SHAPE;
    for (int t = 0; t < 9; ++t)
        if (s0.dy[t] != t / 3 - 1 || s0.dx[t] != t % 3 - 1) return WC_E_SHAPE;
    if (s0.C <= 0 || s0.C % 16 || s0.ldc % 4 || (reinterpret_cast<uintptr_t>(s0.src) & 15)) return WC_E_SHAPE;
    if (a->B <= 0 || a->N <= 0 || s0.H != a->Hm || s0.W != a->Wm || a->Hm % TH || a->Wm % 16) return WC_E_SHAPE;
    if ((long)a->B * s0.H * s0.W * s0.ldc * 4 >= (1L << 31)) return WC_E_SHAPE;
    if (reinterpret_cast<uintptr_t>(w) & 15) return WC_E_SHAPE;
    d = WDev{};
    d.src0 = s0.src; d.C0 = s0.C; d.ldc0 = s0.ldc; d.scale = s0.scale; d.shift = s0.shift;
    d.nck0 = s0.C / 16;
    res = a->nseg == 2;
    if (res) {
        const wc_conv_seg& s1 = a->seg[1];
        if (!s1.src || s1.scale || !a_bound) return WC_E_ARG;  // the residual runs on f16x3 under a_bound
        if (s1.ntaps != 1 || s1.dy[0] != 0 || s1.dx[0] != 0 || s1.sy != 1 || s1.sx != 1) return WC_E_SHAPE;
        if (s1.H != s0.H || s1.W != s0.W || s1.kbase != 9 * s0.C) return WC_E_SHAPE;
        if (s1.C <= 0 || s1.C % 16 || s1.ldc % 4 || (reinterpret_cast<uintptr_t>(s1.src) & 15)) return WC_E_SHAPE;
        if ((long)a->B * s1.H * s1.W * s1.ldc * 4 >= (1L << 31)) return WC_E_SHAPE;
        d.src1 = s1.src; d.C1 = s1.C; d.ldc1 = s1.ldc; d.nck1 = s1.C / 16;
    }
    if (a->out_nchw || a->Ho != a->Hm || a->Wo != a->Wm || a->osy != 1 || a->osx != 1 || a->ooy || a->oox)
        return WC_E_SHAPE;
    if ((long)a->Hm * a->Wm * a->ldo * 4 >= (1L << 31) || (a->res && (long)a->Hm * a->Wm * a->ldres * 4 >= (1L << 31)))
        return WC_E_SHAPE;
    d.B = a->B; d.H = a->Hm; d.W = a->Wm; d.N = a->N;
    d.w = w; d.bias = a->bias; d.temb = a->temb; d.temb_ld = a->temb_ld;
    d.res = a->res; d.ldres = a->ldres; d.out = a->out; d.ldo = a->ldo;
    d.a_exp = a_exp - 1;  // |V| <= 2 x the GN bound
    d.abound = (res || pro == 0) ? a_bound : nullptr;
    d.wsinv = w_inv_scale;
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
    if (w_bytes != ntn * (12L * d.nck0 + d.nck1) * BN * 64 || w_bytes >= (1L << 31)) return WC_E_SHAPE;
    return WC_OK;
}

// bytes of one image's pre-split planes: [chunk C/16][plane VPL][row H][tile W/2] x 16 B
long wino_vimg(int C, int H, int W) { return (long)(C / 16) * VPL * H * (W / 2) * 16; }

// ---- wino_vsplit_kernel: segment 0 of a GN+SiLU Winograd conv, transformed and split once ----
// Workgroup = R = 256 / W image rows of one image and NCK 16-channel chunks (NCK = 2 where C % 32 == 0:
// a pixel's 32 channels are one whole 128-byte line, read by one workgroup -- with one chunk per
// workgroup the two halves of every line went to workgroups on different XCDs and were fetched twice).
// Stage 1: the rows' pixels -1 .. W (4 NCK lanes per pixel, 16 B each) through GN affine + SiLU + 2^s
// with zero padding, once per element, into LDS as fp32 [chunk][row][pixel][quad].  Stage 2: thread =
// (row, tile t, channel octet h), for each chunk: the tile's four pixels 2t - 1 .. 2t + 2 from LDS, the
// input transform V0..V3 and the two-piece fp16 split, stored as 16-byte fragments at
// [b][chunk][plane = piece 8 + position 2 + h][y][t] -- for fixed (plane, row) consecutive lanes write
// consecutive tiles.  The same operations in the same order as the conv kernel's items (prologue /
// transform, PRO 2): the planes are bit for bit the LDS image those items write.  s per image as the
// conv: a_exp - 1, clamped to 13 - e(res_bound[b]) under a residual.
#ifndef VS_IPT
#define VS_IPT 4
#endif
template <int NCK>
__global__ __launch_bounds__(256) void wino_vsplit_kernel(const float* __restrict__ src, int ldc, int B, int H,
                                                          int W, int C, const float* __restrict__ scale,
                                                          const float* __restrict__ shift, int a_exp1,
                                                          const float* __restrict__ res_bound,
                                                          unsigned char* __restrict__ vout, long vimg) {
    extern __shared__ __attribute__((aligned(16))) f32x4 act[];  // [NCK][R][W + 2][4 quads + 1 pad]
    const int R = 256 / W, ngrp = C / (16 * NCK), nyb = (H + R - 1) / R;
    const int kg = blockIdx.x % ngrp;
    const int yb = (blockIdx.x / ngrp) % nyb;
    const int b = blockIdx.x / (ngrp * nyb);
    const int y0 = yb * R;
    const int tid = threadIdx.x;
    int s_exp = a_exp1;
    if (res_bound) {
        const float bnd = res_bound[b];
        const int e = (int)((__float_as_uint(bnd) >> 23) & 0xffu) - 127;
        if (bnd > 0.f) s_exp = min(s_exp, 13 - e);
        s_exp = max(s_exp, -100);
    }
    const float ascale = ldexpf(1.0f, s_exp);
    // stage 1: item = (row, padded pixel, quad of the NCK x 16 channels); VS_IPT items per thread in
    // flight.  256 % (4 NCK) == 0, so a thread's channel quad -- and its GN scale / shift -- is the same
    // for every item it takes: loaded once
    const int W2 = W + 2, items = R * W2 * 4 * NCK, cstride = R * W2 * 5;
    const int qt = tid % (4 * NCK), ct = kg * 16 * NCK + 4 * qt;
    const f32x4 sct = *reinterpret_cast<const f32x4*>(scale + (long)b * C + ct);
    const f32x4 sht = *reinterpret_cast<const f32x4*>(shift + (long)b * C + ct);
    for (int i0 = tid; i0 < items; i0 += VS_IPT * 256) {
        f32x4 v[VS_IPT];
        bool inb[VS_IPT];
        int slot[VS_IPT];
#pragma unroll
        for (int u = 0; u < VS_IPT; ++u) {
            const int i = min(i0 + u * 256, items - 1);  // past the end: a repeat of the last item, not stored
            const int px = (i / (4 * NCK)) % W2 - 1, r = (i / (4 * NCK)) / W2;
            const int y = y0 + r;
            inb[u] = (unsigned)px < (unsigned)W && y < H;
            v[u] = *reinterpret_cast<const f32x4*>(src + ((long)(b * H + min(y, H - 1)) * W + min(max(px, 0), W - 1)) * ldc + ct);
            // a pixel is 5 slots (4 quads + pad): stage 2's lanes, two pixels apart, then read distinct banks
            slot[u] = (qt >> 2) * cstride + (r * W2 + px + 1) * 5 + (qt & 3);
        }
#pragma unroll
        for (int u = 0; u < VS_IPT; ++u) {
            if (i0 + u * 256 >= items) break;
            f32x4 a = v[u] * sct + sht;
            a.x = silu_fast(a.x); a.y = silu_fast(a.y);
            a.z = silu_fast(a.z); a.w = silu_fast(a.w);
            act[slot[u]] = inb[u] ? a * ascale : f32x4{0.f, 0.f, 0.f, 0.f};
        }
    }
    __syncthreads();
    // stage 2
    const int T2 = W / 2;
    const int t = tid % T2, h = (tid / T2) & 1, r = tid / W;
    const int y = y0 + r;
    // R * W <= 256 threads own a (row, tile, octet): when W does not divide 256 the trailing threads
    // (r == R) would read past stage 1's rows and write the next workgroup's first row
    if (r >= R || y >= H) return;
    const long plane = (long)H * T2 * 16;
    const long frag = ((long)y * T2 + t) * 16;
#pragma unroll
    for (int ck = 0; ck < NCK; ++ck) {
        unsigned char* vb = vout + (long)b * vimg + (long)(kg * NCK + ck) * VPL * H * T2 * 16;
        u32x2 pc[2][4][2];  // [quad of the octet][position][piece]
#pragma unroll
        for (int qq = 0; qq < 2; ++qq) {
            const f32x4* ar = act + ck * cstride + (r * W2 + 2 * t) * 5 + 2 * h + qq;  // pixel 2t - 1 is padded index 2t
            const f32x4 d0 = ar[0], d1 = ar[5], d2 = ar[10], d3 = ar[15];
            const f32x4 V[4] = {d0 - d2, d1 + d2, d2 - d1, d1 - d3};
#pragma unroll
            for (int pos = 0; pos < 4; ++pos) split2_f16(V[pos], pc[qq][pos][0], pc[qq][pos][1]);
        }
#pragma unroll
        for (int pos = 0; pos < 4; ++pos)
#pragma unroll
            for (int piece = 0; piece < VPL / 8; ++piece)  // (single-piece builds: the high piece only)
                *reinterpret_cast<u32x4*>(vb + (piece * 8 + pos * 2 + h) * plane + frag) =
                    u32x4{pc[0][pos][piece].x, pc[0][pos][piece].y, pc[1][pos][piece].x, pc[1][pos][piece].y};
    }
}

}  // namespace

extern "C" int wc_conv3x3_wino_f16x3(const wc_conv_args* a, const void* w, int64_t w_bytes, int a_exp,
                                     const float* w_inv_scale, const float* a_bound, void* stream) {
    WDev d;
    int pro, BN;
    bool res;
    const int st = wino_setup(a, w, w_bytes, a_exp, w_inv_scale, a_bound, d, pro, res, BN);
    if (st != WC_OK) return st;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    if (pro == 0) return BN == 64 ? launch_wino<16, 64, 0, false>(d, s) : launch_wino<8, 128, 0, false>(d, s);
    if (BN == 64) return res ? launch_wino<16, 64, 2, true>(d, s) : launch_wino<16, 64, 2, false>(d, s);
    return res ? launch_wino<8, 128, 2, true>(d, s) : launch_wino<8, 128, 2, false>(d, s);
}

extern "C" int wc_conv3x3_wino_gnb_splits(int N, int H, int W) {
    const int BN = wc_conv3x3_wino_tile_n(N), TH = BN == 64 ? 16 : 8;
    if (N <= 0 || H <= 0 || W <= 0 || H % TH || W % 16) return -1;
    const int waves_m = 4 / (BN / 32);
    return (H / TH) * (W / 16) * waves_m;
}

extern "C" int wc_conv3x3_wino_f16x3_gnb(const wc_conv_args* a, const void* w, int64_t w_bytes, int a_exp,
                                         const float* w_inv_scale, const float* a_bound, const wc_gnb_epi* g,
                                         void* stream) {
    WDev d;
    int pro, BN;
    bool res;
    const int st = wino_setup(a, w, w_bytes, a_exp, w_inv_scale, a_bound, d, pro, res, BN);
    if (st != WC_OK) return st;
    if (pro != 0 || !g || !g->x || !g->sc0 || !g->sh0 || !g->part) return WC_E_ARG;
    if (g->ldx < d.N || g->splits != wc_conv3x3_wino_gnb_splits(d.N, d.H, d.W)) return WC_E_SHAPE;
    if ((long)d.B * d.H * d.W * g->ldx * 4 >= (1L << 31)) return WC_E_SHAPE;
    d.gb_x = g->x; d.gb_ldx = g->ldx; d.gb_silu = g->silu ? 1 : 0;
    d.gb_sc0 = g->sc0; d.gb_sh0 = g->sh0; d.gb_gamma = g->gamma; d.gb_beta = g->beta;
    d.gb_part = g->part; d.gb_part3 = g->part3;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    return BN == 64 ? launch_wino<16, 64, 0, false>(d, s) : launch_wino<8, 128, 0, false>(d, s);
}

extern "C" int wc_wino_vsplit_bytes(int B, int C, int H, int W, int64_t* bytes) {
    if (!bytes || B <= 0 || C <= 0 || C % 16 || H <= 0 || W <= 0 || W % 16) return WC_E_SHAPE;
    *bytes = (int64_t)B * wino_vimg(C, H, W);
    return WC_OK;
}

extern "C" int wc_wino_vsplit_f16x3(const wc_conv_args* a, int a_exp, const float* a_bound, void* vout, int64_t v_bytes,
                                    void* stream) {
    if (!a || !vout || a->nseg < 1 || a->nseg > 2) return WC_E_ARG;
    const wc_conv_seg& s0 = a->seg[0];
    if (!s0.src || !s0.scale || !s0.shift || !s0.silu) return WC_E_ARG;  // the GN + SiLU segment only
    if (a->nseg == 2 && !a_bound) return WC_E_ARG;
    if (a_exp < -60 || a_exp > 60) return WC_E_ARG;
    if (s0.C <= 0 || s0.C % 16 || s0.ldc % 4 || (reinterpret_cast<uintptr_t>(s0.src) & 15) || s0.W % 16)
        return WC_E_SHAPE;
    if ((reinterpret_cast<uintptr_t>(vout) & 15) || v_bytes != (int64_t)a->B * wino_vimg(s0.C, s0.H, s0.W))
        return WC_E_SHAPE;
    if (s0.W > 256) return WC_E_SHAPE;  // R = 256 / W rows per workgroup
    const int R = 256 / s0.W;
    const int nck = s0.C % 32 == 0 ? 2 : 1;
    const long nblk = (long)a->B * ((s0.H + R - 1) / R) * (s0.C / (16 * nck));
    const size_t lds = (size_t)nck * R * (s0.W + 2) * 5 * sizeof(f32x4);
    if (lds > 64 * 1024) return WC_E_SHAPE;
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    const float* rb = a->nseg == 2 ? a_bound : nullptr;
    unsigned char* vo = reinterpret_cast<unsigned char*>(vout);
    const long vimg = wino_vimg(s0.C, s0.H, s0.W);
    if (nck == 2) {
        WC_SET_NAME("wino_vsplit_kernel", {WC_TI(2)});
        hipLaunchKernelGGL(wino_vsplit_kernel<2>, dim3((unsigned)nblk), dim3(256), lds, st, s0.src, s0.ldc, a->B, s0.H,
                           s0.W, s0.C, s0.scale, s0.shift, a_exp - 1, rb, vo, vimg);
    } else {
        WC_SET_NAME("wino_vsplit_kernel", {WC_TI(1)});
        hipLaunchKernelGGL(wino_vsplit_kernel<1>, dim3((unsigned)nblk), dim3(256), lds, st, s0.src, s0.ldc, a->B, s0.H,
                           s0.W, s0.C, s0.scale, s0.shift, a_exp - 1, rb, vo, vimg);
    }
    WC_CHECK_LAUNCH();
    return WC_OK;
}

extern "C" int wc_conv3x3_wino_f16x3_vp(const wc_conv_args* a, const void* w, int64_t w_bytes, int a_exp,
                                        const float* w_inv_scale, const float* a_bound, const void* vpre,
                                        int64_t v_bytes, void* stream) {
    WDev d;
    int pro, BN;
    bool res;
    const int st = wino_setup(a, w, w_bytes, a_exp, w_inv_scale, a_bound, d, pro, res, BN);
    if (st != WC_OK) return st;
    if (pro != 2 || !vpre || (reinterpret_cast<uintptr_t>(vpre) & 15)) return WC_E_ARG;
    d.vimg = wino_vimg(d.C0, d.H, d.W);
    if (v_bytes != (int64_t)d.B * d.vimg || d.vimg >= (1L << 31)) return WC_E_SHAPE;
    d.vpre = reinterpret_cast<const unsigned char*>(vpre);
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    if (BN == 64) return res ? launch_wino<16, 64, 3, true>(d, s) : launch_wino<16, 64, 3, false>(d, s);
    return res ? launch_wino<8, 128, 3, true>(d, s) : launch_wino<8, 128, 3, false>(d, s);
}

// The same with 8-wave workgroups of 256 output channels (N % 256 == 0): each halo plane copy feeds
// twice the MFMAs, one workgroup per CU.  Measured slower alone at every batch (B = 2..16: +3..17 %)
// but faster beside a concurrent launch stream (the two-group sampling graph: 23.36-23.37 vs
// 23.52-23.53 ms/step), so the caller picks it (profiles/r06_wino_vp8_ab.txt).
extern "C" int wc_conv3x3_wino_f16x3_vp8(const wc_conv_args* a, const void* w, int64_t w_bytes, int a_exp,
                                         const float* w_inv_scale, const float* a_bound, const void* vpre,
                                         int64_t v_bytes, void* stream) {
    WDev d;
    int pro, BN;
    bool res;
    const int st = wino_setup(a, w, w_bytes, a_exp, w_inv_scale, a_bound, d, pro, res, BN);
    if (st != WC_OK) return st;
    if (pro != 2 || !vpre || (reinterpret_cast<uintptr_t>(vpre) & 15)) return WC_E_ARG;
    if (BN != 128 || d.N % 256) return WC_E_SHAPE;
    d.vimg = wino_vimg(d.C0, d.H, d.W);
    if (v_bytes != (int64_t)d.B * d.vimg || d.vimg >= (1L << 31)) return WC_E_SHAPE;
    d.vpre = reinterpret_cast<const unsigned char*>(vpre);
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    return res ? launch_wino<8, 256, 3, true, 2, 8>(d, s) : launch_wino<8, 256, 3, false, 2, 8>(d, s);
}

// ---- device re-pack for wc_conv3x3_wino_f16x3 (training: the weights change every step) ----
// One workgroup per output channel n (of the N-tile-padded count): max |U|, |w_res| over the row, the
// power-of-two scale 2^sW with max * 2^sW <= 2^14 (sW from the exponent: exact, no log2), then every
// value of the row: U in float64 (g0, (g0 + g1 + g2) / 2, (g0 - g1 + g2) / 2, g2) x 2^sW, rounded once
// to fp32, split into two round-to-nearest fp16 pieces -- the same IEEE operations in the same order as
// kernels.pack_wino's torch definition, so the two are bit-identical.
namespace {

__device__ double wino_u(const float* row, int C0, int ky, int pos, int c) {
    const double g0 = row[(ky * 3 + 0) * C0 + c], g1 = row[(ky * 3 + 1) * C0 + c], g2 = row[(ky * 3 + 2) * C0 + c];
    switch (pos) {
        case 0: return g0;
        case 1: return ((g0 + g1) + g2) * 0.5;
        case 2: return ((g0 - g1) + g2) * 0.5;
        default: return g2;
    }
}

// The same for channels c .. c + 7 of an LDS row with tap stride ld (16-byte aligned): two 16-byte reads
// per tap instead of eight scalar ones (lanes 8 channels apart hit one bank eight ways).
__device__ void wino_u8(const float* row, int ld, int ky, int pos, int c, double* v) {
    f32x4 g[3][2];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        g[k][0] = *reinterpret_cast<const f32x4*>(row + (ky * 3 + k) * ld + c);
        g[k][1] = *reinterpret_cast<const f32x4*>(row + (ky * 3 + k) * ld + c + 4);
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) {
        const double g0 = g[0][e >> 2][e & 3], g1 = g[1][e >> 2][e & 3], g2 = g[2][e >> 2][e & 3];
        v[e] = pos == 0 ? g0 : pos == 1 ? ((g0 + g1) + g2) * 0.5 : pos == 2 ? ((g0 - g1) + g2) * 0.5 : g2;
    }
}

// The row of output channel n: the 3x3 values at row3[(ky * 3 + kx) * C0 + c], the residual ones (C1)
// at rres[j]; live = n < N (padding rows are zeros).
__device__ void pack_wino_row(const float* row3, int ld, bool vec, const float* rres, bool live, int n, int C0, int C1,
                              int BN, short* __restrict__ out, float* __restrict__ wsinv) {
    // items of 8 consecutive channels (one 16-byte fragment per piece): 12 (ky, pos) x C0 / 8, then C1 / 8
    const int c8 = C0 / 8, n0 = 12 * c8, nall = n0 + C1 / 8;
    auto values = [&](int it, double* v) {
        if (it < n0) {
            const int kp = it / c8, c = (it - kp * c8) * 8;
            if (vec) {
                wino_u8(row3, ld, kp / 4, kp % 4, c, v);
            } else {
#pragma unroll
                for (int e = 0; e < 8; ++e) v[e] = wino_u(row3, ld, kp / 4, kp % 4, c + e);
            }
        } else {
            const int c = (it - n0) * 8;
#pragma unroll
            for (int e = 0; e < 8; ++e) v[e] = rres[c + e];
        }
    };
    double m = 0.0;
    if (live) {
        for (int it = threadIdx.x; it < nall; it += blockDim.x) {
            double v[8];
            values(it, v);
#pragma unroll
            for (int e = 0; e < 8; ++e) m = fmax(m, fabs(v[e]));
        }
    }
    __shared__ double red[256];
    red[threadIdx.x] = m;
    __syncthreads();
    for (int s = 128; s > 0; s >>= 1) {
        if ((int)threadIdx.x < s) red[threadIdx.x] = fmax(red[threadIdx.x], red[threadIdx.x + s]);
        __syncthreads();
    }
    const double amax = red[0];
    int sw = 0;
    if (amax > 0.0) {
        int e;
        const double mant = frexp(amax, &e);  // amax = mant 2^e, mant in [0.5, 1)
        sw = (mant == 0.5 ? 15 : 14) - e;     // floor(log2(2^14 / amax))
        sw = sw < -60 ? -60 : sw > 60 ? 60 : sw;
    }
    const double scale = ldexp(1.0, sw);
    if (threadIdx.x == 0) wsinv[n] = ldexpf(1.0f, -sw);
    const int T = n / BN, nn = n % BN;
    const long rowlen = (long)(12 * (C0 / 16) + C1 / 16) * 2 * 2 * BN * 8;  // int16 per N tile
    short* trow = out + (long)T * rowlen;
    const int plane = 2 * BN * 8;  // distance between the two pieces (int16 units)
    for (int it = threadIdx.x; it < nall; it += blockDim.x) {
        double v[8];
        if (live) values(it, v);
        else
#pragma unroll
            for (int e = 0; e < 8; ++e) v[e] = 0.0;
        long o;
        if (it < n0) {
            const int kp = it / c8, c = (it - kp * c8) * 8, ky = kp / 4, pos = kp % 4;
            const int chunk = c / 16, kh = (c % 16) / 8;
            o = ((((long)(chunk * 3 + ky) * 4 + pos) * 2 * 2 + kh) * BN + nn) * 8;  // piece 0
        } else {
            const int c = (it - n0) * 8;
            const int chunk = c / 16, kh = (c % 16) / 8;
            o = (long)(C0 / 16) * 12 * 2 * 2 * BN * 8 + (((long)chunk * 2 * 2 + kh) * BN + nn) * 8;
        }
        unsigned hp[4], lp[4];
#pragma unroll
        for (int e = 0; e < 8; e += 2) {
            unsigned short h0, l0, h1, l1;
            float a = (float)(v[e] * scale), b = (float)(v[e + 1] * scale);
            // materialize the fp32 values: without this the compiler folds double -> fp32 -> fp16 into one
            // double -> fp16 rounding, which differs on fp16 ties (the definition rounds twice, fp32 first)
            asm volatile("" : "+v"(a), "+v"(b));
            split2_one(a, h0, l0);
            split2_one(b, h1, l1);
            hp[e / 2] = (unsigned)h0 | ((unsigned)h1 << 16);
            lp[e / 2] = (unsigned)l0 | ((unsigned)l1 << 16);
        }
        *reinterpret_cast<u32x4*>(trow + o) = u32x4{hp[0], hp[1], hp[2], hp[3]};
        *reinterpret_cast<u32x4*>(trow + o + plane) = u32x4{lp[0], lp[1], lp[2], lp[3]};
    }
}

__global__ __launch_bounds__(256) void pack_wino_kernel(const float* __restrict__ w, int K, int N, int C0, int C1,
                                                        int BN, short* __restrict__ out, float* __restrict__ wsinv) {
    const int n = blockIdx.x;
    const bool live = n < N;
    const float* row = w + (long)(live ? n : 0) * K;
    pack_wino_row(row, C0, false, row + 9 * C0, live, n, C0, C1, BN, out, wsinv);
}

// The same from the module's own [Co][Ci][3][3] weight (no host re-layout): TRANSPOSED = false, the conv
// itself (N = Co, C0 = Ci; value (n, tap, c) = w[n][c][tap]), the residual row n of wres [N][C1];
// TRANSPOSED = true, its data gradient (N = Ci, C0 = Co; value (n, tap, c) = w[c][n][8 - tap], the
// flipped, transposed filter), no residual.  The row goes through LDS in the packed order first, so the
// values -- and the pieces -- are those of pack_wino_kernel on the host re-layout.
// Stage output channel n's 3x3 values into LDS in the packed order row3[tap * (C0 + 4) + c] (the 4-float
// pad puts the nine taps of one channel, written by neighbouring lanes, in different banks), eight loads
// in flight per thread (a load-then-store loop waited out one memory latency per element).
// TRANSPOSED reads the flipped, transposed filter w[c][n][8 - tap].
__device__ void stage_row3(const float* __restrict__ w, bool transposed, int N, int n, int C0, float* row3) {
    const int lim = 9 * C0, ld = C0 + 4;
    for (int i0 = threadIdx.x; i0 < lim; i0 += 8 * 256) {
        float v[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const int i = i0 + k * 256;
            const int c = i / 9, t = i - 9 * c;
            v[k] = i < lim ? (transposed ? w[((long)c * N + n) * 9 + t] : w[(long)n * lim + i]) : 0.f;
        }
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const int i = i0 + k * 256;
            const int c = i / 9, t = i - 9 * c;
            if (i < lim) row3[(transposed ? 8 - t : t) * ld + c] = v[k];
        }
    }
}

template <bool TRANSPOSED>
__global__ __launch_bounds__(256) void pack_wino_raw_kernel(const float* __restrict__ w, const float* __restrict__ wres,
                                                            int N, int C0, int C1, int BN, short* __restrict__ out,
                                                            float* __restrict__ wsinv) {
    extern __shared__ float row3[];  // [9][C0]
    const int n = blockIdx.x;
    const bool live = n < N;
    if (live) stage_row3(w, TRANSPOSED, N, n, C0, row3);  // i walks the source in memory order
    __syncthreads();
    pack_wino_row(row3, C0 + 4, true, wres + (long)(live ? n : 0) * C1, live, n, C0, C1, BN, out, wsinv);
}

// Many raw packs in one launch (the training step's ~80 per-iteration Winograd packs): workgroup g runs
// output channel g - wg0 of the job with the largest wg0 <= g (binary search over the sorted wg0s).
__global__ __launch_bounds__(256) void pack_wino_batch_kernel(const wc_wino_pack_job* __restrict__ jobs, int njobs) {
    extern __shared__ float row3[];
    __shared__ int s_wg0[256];
    const int g = blockIdx.x;
    // the jobs' first workgroups in LDS in one round of loads, then the search (one dependent global
    // load per search step cost a memory latency each)
    const bool lds = njobs <= 256;
    if (lds && (int)threadIdx.x < njobs) s_wg0[threadIdx.x] = jobs[threadIdx.x].wg0;
    __syncthreads();
    int lo = 0, hi = njobs - 1;
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if ((lds ? s_wg0[mid] : jobs[mid].wg0) <= g) lo = mid;
        else hi = mid - 1;
    }
    const wc_wino_pack_job jb = jobs[lo];
    const int n = g - jb.wg0;
    const bool live = n < jb.N;
    const int C0 = jb.C0, N = jb.N;
    if (live) stage_row3(jb.w, jb.transposed != 0, N, n, C0, row3);
    __syncthreads();
    pack_wino_row(row3, C0 + 4, true, jb.wres + (long)(live ? n : 0) * jb.C1, live, n, C0, jb.C1, jb.BN,
                  reinterpret_cast<short*>(jb.out), jb.wsinv);
}

}  // namespace

extern "C" int wc_pack_wino(const float* w, int N, int C0, int C1, void* out, int64_t out_bytes, float* w_inv_scale,
                            void* stream) {
    if (!w || !out || !w_inv_scale) return WC_E_ARG;
    if (N <= 0 || C0 <= 0 || C0 % 16 || C1 < 0 || C1 % 16) return WC_E_SHAPE;
    const int BN = wc_conv3x3_wino_tile_n(N);
    const long ntn = (N + BN - 1) / BN;
    if (out_bytes != ntn * (12L * (C0 / 16) + C1 / 16) * BN * 64) return WC_E_SHAPE;
    hipLaunchKernelGGL(pack_wino_kernel, dim3((unsigned)(ntn * BN)), dim3(256), 0, reinterpret_cast<hipStream_t>(stream),
                       w, 9 * C0 + C1, N, C0, C1, BN, reinterpret_cast<short*>(out), w_inv_scale);
    wc_last_kernel = "pack_wino_kernel";
    WC_CHECK_LAUNCH();
    return WC_OK;
}

extern "C" int wc_pack_wino_batch(const wc_wino_pack_job* jobs, int njobs, int total_wg, int max_c0, void* stream) {
    if (!jobs || njobs < 0 || total_wg < 0) return WC_E_ARG;
    if (njobs == 0) return WC_OK;
    if (max_c0 <= 0 || 9L * (max_c0 + 4) * 4 > 64 * 1024 || total_wg <= 0) return WC_E_SHAPE;
    hipLaunchKernelGGL(pack_wino_batch_kernel, dim3((unsigned)total_wg), dim3(256), (size_t)9 * (max_c0 + 4) * sizeof(float),
                       reinterpret_cast<hipStream_t>(stream), jobs, njobs);
    wc_last_kernel = "pack_wino_batch_kernel";
    WC_CHECK_LAUNCH();
    return WC_OK;
}

extern "C" int wc_pack_wino_raw(const float* w, const float* wres, int N, int C0, int C1, int transposed, void* out,
                                int64_t out_bytes, float* w_inv_scale, void* stream) {
    if (!w || !out || !w_inv_scale || (C1 && !wres) || (transposed && C1)) return WC_E_ARG;
    if (N <= 0 || C0 <= 0 || C0 % 16 || C1 < 0 || C1 % 16 || 9L * (C0 + 4) * 4 > 64 * 1024) return WC_E_SHAPE;
    const int BN = wc_conv3x3_wino_tile_n(N);
    const long ntn = (N + BN - 1) / BN;
    if (out_bytes != ntn * (12L * (C0 / 16) + C1 / 16) * BN * 64) return WC_E_SHAPE;
    const size_t lds = (size_t)9 * (C0 + 4) * sizeof(float);
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    if (transposed)
        hipLaunchKernelGGL(pack_wino_raw_kernel<true>, dim3((unsigned)(ntn * BN)), dim3(256), lds, s, w, wres, N, C0, C1,
                           BN, reinterpret_cast<short*>(out), w_inv_scale);
    else
        hipLaunchKernelGGL(pack_wino_raw_kernel<false>, dim3((unsigned)(ntn * BN)), dim3(256), lds, s, w, wres, N, C0,
                           C1, BN, reinterpret_cast<short*>(out), w_inv_scale);
    wc_last_kernel = "pack_wino_raw_kernel";
    WC_CHECK_LAUNCH();
    return WC_OK;
}
