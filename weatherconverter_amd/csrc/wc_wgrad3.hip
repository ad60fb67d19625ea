// Weight gradient of a 3x3 stride-1 pad-1 convolution, halo-tiled, on bf16x6 split-precision MFMA
// (gfx950).  Backward of the ResBlock convs (reference unet_base.py:92-94,106 through
// train_ddpm.py:110 loss.backward()):
//
//   dW[m][tap][c] = sum over pixels p of G[p][m] * X~[p + off(tap)][c]
//
// G = the output gradient (NHWC, M channels), X~ = the conv's input as the forward read it: the
// GroupNorm(+SiLU) prologue recomputed from the stored pre-norm tensor, zero padded after it.
//
// The generic wc_conv_wgrad GEMM stages the im2col operand, so every input value is loaded,
// normalised, SiLU'd and split nine times (once per tap column) and each 16-pixel K-step ends in a
// barrier.  Here a workgroup owns BM output channels x 32 input channels x all 9 taps and walks
// TH x 16-pixel blocks: per block the (TH+2) x 18 input halo is loaded, transformed and split ONCE
// into LDS, and each 16-pixel row of the block is one K-step whose nine taps read their B
// fragments from that halo at a constant pixel offset (ds_read_b64_tr_b16 on [pixel][channel]
// rows: the MFMA wants 8 consecutive PIXELS per lane).  The A fragments (G^T, 8 pixels of one
// channel per lane) go straight from L2 into registers one K-step ahead and are reused by all nine
// taps: 54 MFMAs per wave per K-step (9 taps x 6 piece products), one barrier per block.
//
// Arithmetic (F3 = false, bf16x6): both operands split exactly into three bf16 pieces
// (wcx6::split3), the six products with i + j <= 2 accumulated in fp32 (as wc_conv_wgrad_x6).
// F3 = true (f16x3): X~ * 2^x_exp (the forward's static exponent of the GroupNorm(+SiLU) output,
// Samuelson bound) and G * 2^sg split into two round-to-nearest fp16 pieces, products h*h + h*l +
// l*h (27 MFMAs per wave per K-step); sg = 13 - floor(log2 max_b gbound[b]) from the per-image absmax
// of G that the f16x3 data gradient already measured, so |G| * 2^sg < 2^14.  One exponent for the
// whole batch: a pixel split may cross images, and every product carries the same factor, which the
// epilogue removes exactly (power of two).  Results: partial sums per pixel split [split][M][9*C0]
// (column = tap*C0 + c, the layout of wc_conv_wgrad), reduced in a fixed order by wc_wgrad_reduce:
// deterministic run to run.
#include "wc_x6.hpp"

namespace {

using namespace wcx6;

constexpr int W3_NT = 256;
constexpr int W3_HW = 18;  // halo row: 16 + 2 pixels

struct W3Dev {
    const float* g;
    int M, ldg;
    const float* x;
    int C0, ldc0;
    const float* scale;
    const float* shift;
    int B, H, W;
    float* part;
    int Kc;          // partial row length: 9 * C0
    int nblk, bps;   // TH x 16 blocks in the batch; blocks per split
    int nmt, nct;    // m tiles, c tiles
    int x_exp;              // F3: exponent of X~
    const float* gbound;    // F3: per-image max |G| [B]
};

// WM waves along M (32 output channels each), 4 / WM along C (32 input channels each); TH rows per
// block.  PRO: 0 raw input, 1 GN affine, 2 GN affine + SiLU.
template <int WM, int TH, int PRO, bool F3 = false>
struct W3Cfg {
    static constexpr int NPC = F3 ? 2 : 3;                         // operand pieces
    static constexpr int WC = 4 / WM;
    static constexpr int BM = 32 * WM, BC = 32 * WC, CPL = WC;    // c planes of 32 channels
    static constexpr int HP = (TH + 2) * W3_HW;                     // halo pixels
    static constexpr int ROW = 64;                                  // bytes of one pixel row of one plane
    static constexpr int PLANE = HP * ROW;                          // one (piece, c-plane) plane
    static constexpr int BUF = NPC * CPL * PLANE;                   // one halo buffer
    static constexpr int LDS = 2 * BUF;
    static constexpr int ITEMS = HP * CPL * 8;                      // float4 items of one halo
    static constexpr int HJ = (ITEMS + W3_NT - 1) / W3_NT;
    static_assert(W3_NT % (8 * CPL) == 0, "each thread keeps its channel quad and plane");
};

template <int WM, int TH, int PRO, bool F3>
__global__ __launch_bounds__(W3_NT, 2) void conv_wgrad3_kernel(W3Dev p) {
    using Cf = W3Cfg<WM, TH, PRO, F3>;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;
    const int wm = wave / Cf::WC, wc = wave % Cf::WC;
    const int l32 = lane & 31, half = lane >> 5;

    // XCD-aware bijective order (as the forward kernels): the (m, c) tiles of one pixel split, which
    // read the same G rows and input halos, are consecutive logical blocks on one XCD's L2
    const int nblk = gridDim.x;
    int bid = blockIdx.x;
    {
        const int q = nblk / 8, r = nblk % 8, xcd = bid % 8;
        bid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + bid / 8;
    }
    const int mt = bid % p.nmt;
    int t = bid / p.nmt;
    const int ct = t % p.nct;
    const int sp = t / p.nct;
    const int m0 = mt * Cf::BM, c0 = ct * Cf::BC;
    const int k0 = sp * p.bps;
    const int k1 = min(p.nblk, k0 + p.bps);
    const int bx_n = p.W / 16, by_n = p.H / TH;
    // F3 scales: X~ by its static exponent, G by the batch's absmax bound
    float xsc = 1.f, gsc = 1.f, unscale = 1.f;
    if constexpr (F3) {
        float gm = 0.f;
        for (int b = 0; b < p.B; ++b) gm = fmaxf(gm, p.gbound[b]);
        int sg = 60;
        if (gm > 0.f) sg = min(60, 13 - ((int)((__float_as_uint(gm) >> 23) & 0xffu) - 127));
        sg = max(sg, -100);
        xsc = ldexpf(1.f, p.x_exp);
        gsc = ldexpf(1.f, sg);
        unscale = ldexpf(1.f, -(sg + p.x_exp));
    }

    const __amdgpu_buffer_rsrc_t srdg = make_srd(p.g);
    const __amdgpu_buffer_rsrc_t srdx = make_srd(p.x);
    const __amdgpu_buffer_rsrc_t srdsc = make_srd(PRO ? p.scale : p.x);
    const __amdgpu_buffer_rsrc_t srdsh = make_srd(PRO ? p.shift : p.x);

    // ---- halo items: thread keeps channel quad q and plane cp; item j is halo pixel hp0 + j*HPS ----
    const int q = tid & 7;
    const int cp = (tid >> 3) % Cf::CPL;
    const int hp0 = tid / (8 * Cf::CPL);
    constexpr int HPS = W3_NT / (8 * Cf::CPL);  // halo pixels advanced per item
    const int hch = c0 + cp * 32 + 4 * q;       // first channel of the thread's quad
    f32x4 rh[Cf::HJ];
    unsigned hin = 0;  // bit j: item j is an in-image pixel
    int hb_img = 0;    // image of the staged halo
    auto load_halo = [&](int k) {
        const bool live = k < k1;
        const int kk = live ? k : k1 - 1;
        const int b = kk / (bx_n * by_n);
        const int rem = kk - b * (bx_n * by_n);
        const int by = rem / bx_n, bx = rem - by * bx_n;
        const int y0 = by * TH - 1, x0 = bx * 16 - 1;
        hin = 0;
#pragma unroll
        for (int j = 0; j < Cf::HJ; ++j) {
            const int hp = hp0 + j * HPS;
            const int hy = hp / W3_HW, hx = hp - hy * W3_HW;
            const int iy = y0 + hy, ix = x0 + hx;
            const bool in = live && hp < Cf::HP && (unsigned)iy < (unsigned)p.H && (unsigned)ix < (unsigned)p.W;
            hin |= (in ? 1u : 0u) << j;
            rh[j] = bload_f4(srdx, in ? (unsigned)((((b * p.H + iy) * p.W + ix) * p.ldc0 + hch) * 4) : OOB);
        }
        hb_img = b;
    };
    auto write_halo = [&](int buf) {
        unsigned char* base = smem + buf * Cf::BUF + cp * Cf::PLANE + q * 8;
        // GN scale / shift of the image (L2; loaded here, not with the halo: 8 registers fewer
        // through the K-steps)
        f32x4 rsc = {1.f, 1.f, 1.f, 1.f}, rsh = {0.f, 0.f, 0.f, 0.f};
        if constexpr (PRO != 0) {
            const unsigned o = (unsigned)((hb_img * p.C0 + hch) * 4);
            rsc = bload_f4(srdsc, o);
            rsh = bload_f4(srdsh, o);
        }
#pragma unroll
        for (int j = 0; j < Cf::HJ; ++j) {
            const int hp = hp0 + j * HPS;
            if (j >= Cf::HP / HPS && hp >= Cf::HP) continue;  // only the last item can be past the halo
            f32x4 v = rh[j];
            if constexpr (PRO != 0) {
                v = v * rsc + rsh;
                if constexpr (PRO == 2) {
                    if constexpr (F3) {  // v_rcp instead of an IEEE division (~10 VALU ops a value):
                        // ~1 ulp of fp32, far below the two fp16 pieces' 22 bits
                        v.x = silu_fast(v.x); v.y = silu_fast(v.y); v.z = silu_fast(v.z); v.w = silu_fast(v.w);
                    } else {
                        v.x = wc_silu(v.x); v.y = wc_silu(v.y); v.z = wc_silu(v.z); v.w = wc_silu(v.w);
                    }
                }
            }
            if (!((hin >> j) & 1u)) v = f32x4{0.f, 0.f, 0.f, 0.f};  // zero padding after the prologue
            unsigned char* d = base + hp * Cf::ROW;
            if constexpr (F3) {
                u32x2 h, l;
                split2_f16(v * xsc, h, l);
                *reinterpret_cast<u32x2*>(d) = h;
                *reinterpret_cast<u32x2*>(d + Cf::CPL * Cf::PLANE) = l;
            } else {
                u32x2 a0, a1, a2;
                split3(v, a0, a1, a2);
                *reinterpret_cast<u32x2*>(d) = a0;
                *reinterpret_cast<u32x2*>(d + Cf::CPL * Cf::PLANE) = a1;
                *reinterpret_cast<u32x2*>(d + 2 * Cf::CPL * Cf::PLANE) = a2;
            }
        }
    };

    // ---- A operand: G^T, lane (m = l32, k-half) holds 8 consecutive pixels of one channel ----
    const unsigned gl = (unsigned)((8 * half * p.ldg + m0 + wm * 32 + l32) * 4);
    float gr[8];
    auto load_g = [&](int k, int r) {
        const bool live = k < k1;
        const int kk = live ? k : k1 - 1;
        const int b = kk / (bx_n * by_n);
        const int rem = kk - b * (bx_n * by_n);
        const int by = rem / bx_n, bx = rem - by * bx_n;
        const int pix = (b * p.H + by * TH + r) * p.W + bx * 16;  // first pixel of the K-step
        const unsigned v = live ? gl : OOB;
#pragma unroll
        for (int j = 0; j < 8; ++j) gr[j] = bload_f1s(srdg, v, (pix + j) * p.ldg * 4);
    };

    // ---- B operand: X~ pieces, 8 consecutive halo pixels of channel l32 per lane (transposing read) ----
    const int tq = (lane & 15) >> 2, tp = lane & 3, tg = lane >> 4;
    const int tr_off = (8 * (tg >> 1) + tq) * Cf::ROW + (16 * (tg & 1) + 4 * tp) * 2 + wc * Cf::PLANE;
    auto tr_frag = [&](const unsigned char* q0) {
        typedef short v4s __attribute__((ext_vector_type(4)));
        const v4s lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4s*)(q0));
        const v4s hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4s*)(q0 + 4 * Cf::ROW));
        const u32x2 l2 = __builtin_bit_cast(u32x2, lo), h2 = __builtin_bit_cast(u32x2, hi);
        return u32x4{l2.x, l2.y, h2.x, h2.y};
    };

    f32x16 acc[9];
#pragma unroll
    for (int i = 0; i < 9; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[i][r] = 0.f;

    if (k0 < k1) {
        load_halo(k0);
        load_g(k0, 0);
        write_halo(0);
        __syncthreads();
        for (int k = k0; k < k1; ++k) {
            const int buf = (k - k0) & 1;
            const unsigned char* hb = smem + buf * Cf::BUF + tr_off;
#pragma unroll
            for (int r = 0; r < TH; ++r) {
                // this K-step's A pieces (loaded one step ahead), then the next step's loads
                u32x4 af[Cf::NPC];
                if constexpr (F3) {
                    u32x2 a0, a1, b0, b1;
                    split2_f16(f32x4{gr[0], gr[1], gr[2], gr[3]} * gsc, a0, a1);
                    split2_f16(f32x4{gr[4], gr[5], gr[6], gr[7]} * gsc, b0, b1);
                    af[0] = u32x4{a0.x, a0.y, b0.x, b0.y};
                    af[1] = u32x4{a1.x, a1.y, b1.x, b1.y};
                } else {
                    u32x2 a0, a1, a2, b0, b1, b2;
                    split3(f32x4{gr[0], gr[1], gr[2], gr[3]}, a0, a1, a2);
                    split3(f32x4{gr[4], gr[5], gr[6], gr[7]}, b0, b1, b2);
                    af[0] = u32x4{a0.x, a0.y, b0.x, b0.y};
                    af[1] = u32x4{a1.x, a1.y, b1.x, b1.y};
                    af[Cf::NPC - 1] = u32x4{a2.x, a2.y, b2.x, b2.y};
                }
                if (r + 1 < TH) load_g(k, r + 1);
                else load_g(k + 1, 0);
                // the next block's halo goes out in the block's first K-step (after that step's G
                // loads), TH - 1 K-steps before write_halo needs it: its registers are live through
                // the block's last K-step anyway, so the peak register count is unchanged, and the
                // HBM latency of a first-touch halo is covered (with the fast SiLU below: 2.5-4 % on
                // the ResBlock shapes, profiles/r04_wgrad3_ab.txt)
                if (r == 0) load_halo(k + 1);
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int tap = 0; tap < 9; ++tap) {
                    const int dy = tap / 3, dx = tap % 3;  // halo offset of the tap's first pixel
                    const unsigned char* q0 = hb + ((r + dy) * W3_HW + dx) * Cf::ROW;
                    u32x4 bf[Cf::NPC];
#pragma unroll
                    for (int pc = 0; pc < Cf::NPC; ++pc) bf[pc] = tr_frag(q0 + pc * Cf::CPL * Cf::PLANE);
                    if constexpr (F3) {
                        acc[tap] = mfma_f16(af[0], bf[0], acc[tap]);
                        acc[tap] = mfma_f16c(af[0], bf[1], acc[tap]);
                        acc[tap] = mfma_f16c(af[1], bf[0], acc[tap]);
                    } else {
                        acc[tap] = mfma_bf16(af[0], bf[0], acc[tap]);
                        acc[tap] = mfma_bf16(af[0], bf[1], acc[tap]);
                        acc[tap] = mfma_bf16(af[1], bf[0], acc[tap]);
                        acc[tap] = mfma_bf16(af[0], bf[Cf::NPC - 1], acc[tap]);
                        acc[tap] = mfma_bf16(af[1], bf[1], acc[tap]);
                        acc[tap] = mfma_bf16(af[Cf::NPC - 1], bf[0], acc[tap]);
                    }
                }
            }
            write_halo(buf ^ 1);  // (past the last block: an unused write of zeros)
            __syncthreads();
        }
    }

    // ---- partial[sp][m][tap * C0 + c] ----
    float* out = p.part + (long)sp * p.M * p.Kc;
    const int c = c0 + wc * 32 + l32;
#pragma unroll
    for (int tap = 0; tap < 9; ++tap) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int m = m0 + wm * 32 + (r & 3) + 8 * (r >> 2) + 4 * half;
            out[(long)m * p.Kc + tap * p.C0 + c] = F3 ? acc[tap][r] * unscale : acc[tap][r];
        }
    }
}

template <int WM, int TH, int PRO, bool F3>
int launch_w3(const W3Dev& d, int grid, hipStream_t s) {
    using Cf = W3Cfg<WM, TH, PRO, F3>;
    static bool attr_set = false;
    if (!attr_set) {
        hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&conv_wgrad3_kernel<WM, TH, PRO, F3>),
                                           hipFuncAttributeMaxDynamicSharedMemorySize, Cf::LDS);
        if (e != hipSuccess) return (int)e;
        attr_set = true;
    }
    WC_SET_NAME("conv_wgrad3_kernel", {WC_TI(WM), WC_TI(TH), WC_TI(PRO), WC_TB(F3)});
    hipLaunchKernelGGL((conv_wgrad3_kernel<WM, TH, PRO, F3>), dim3(grid), dim3(W3_NT), Cf::LDS, s, d);
    WC_CHECK_LAUNCH();
    return WC_OK;
}

// (WM, TH) per output-channel count: 128-channel M tiles with 8-row blocks, or (M % 128 != 0)
// 64-channel tiles x 64 input channels with 2-row blocks (two workgroups per CU either way)
inline void w3_shape(int M, int& WM, int& TH) {
    if (M % 128 == 0) { WM = 4; TH = 8; }
    else { WM = 2; TH = 2; }
}

}  // namespace

// Number of pixel splits (= partial slabs) wc_conv_wgrad3 uses: about target_blocks workgroups,
// at most one split per 4 pixel blocks.
extern "C" int wc_conv_wgrad3_splits(int M, int C0, int B, int H, int W, int target_blocks) {
    if (M <= 0 || C0 <= 0 || B <= 0 || H <= 0 || W <= 0) return 1;
    int WM, TH;
    w3_shape(M, WM, TH);
    const int BM = 32 * WM, BC = 128 / WM;
    const long tiles = (long)((M + BM - 1) / BM) * ((C0 + BC - 1) / BC);
    const long nblk = (long)B * (H / TH) * (W / 16);
    long sp = (target_blocks + tiles - 1) / tiles;
    if (sp > nblk / 4) sp = nblk / 4;
    if (sp < 1) sp = 1;
    const long bps = (nblk + sp - 1) / sp;
    return (int)((nblk + bps - 1) / bps);
}

// Segment 0 of `a` must be the 3x3 stride-1 tap grid (-1..1, row-major) at the gradient's own grid
// (H, W), optional GN(+SiLU) prologue; M % 64 == 0 (M % 128 == 0 uses the 128-channel tiles), C0 % 32
// == 0 (% 64 for the 64-channel tiles), W % 16 == 0, H % TH == 0.  a->nseg must be 1 (the residual
// 1x1 segment goes through wc_conv_wgrad).  part: [splits][M][9*C0] floats, splits from
// wc_conv_wgrad3_splits; then wc_wgrad_reduce(part, splits, M, 9*C0, 9*C0, C0, ...) as for
// wc_conv_wgrad.
template <bool F3>
int launch_w3_any(int WM, int pro, const W3Dev& d, int grid, hipStream_t s) {
    if (WM == 4) {
        switch (pro) {
            case 0: return launch_w3<4, 8, 0, F3>(d, grid, s);
            case 1: return launch_w3<4, 8, 1, F3>(d, grid, s);
            default: return launch_w3<4, 8, 2, F3>(d, grid, s);
        }
    }
    switch (pro) {
        case 0: return launch_w3<2, 2, 0, F3>(d, grid, s);
        case 1: return launch_w3<2, 2, 1, F3>(d, grid, s);
        default: return launch_w3<2, 2, 2, F3>(d, grid, s);
    }
}

static int conv_wgrad3_any(const wc_wgrad_args* a, float* part, int splits, bool f3, int x_exp, const float* gbound,
                           void* stream) {
    if (!a || !a->g || !part || a->nseg != 1) return WC_E_ARG;
    if (f3 && (!gbound || x_exp < -100 || x_exp > 60)) return WC_E_ARG;
    const wc_conv_seg& s0 = a->seg[0];
    if (!s0.src || (s0.scale == nullptr) != (s0.shift == nullptr)) return WC_E_ARG;
    if (s0.ntaps != 9 || s0.sy != 1 || s0.sx != 1 || s0.kbase != 0) return WC_E_SHAPE;
    for (int t = 0; t < 9; ++t)
        if (s0.dy[t] != t / 3 - 1 || s0.dx[t] != t % 3 - 1) return WC_E_SHAPE;
    int WM, TH;
    w3_shape(a->M, WM, TH);
    const int BC = 128 / WM;
    if (a->M <= 0 || a->M % 64 || s0.C <= 0 || s0.C % BC || s0.ldc % 4 || a->ldg % 4) return WC_E_SHAPE;
    if (a->B < 1 || s0.H != a->Hm || s0.W != a->Wm || a->Wm % 16 || a->Hm % TH) return WC_E_SHAPE;
    if (((reinterpret_cast<uintptr_t>(a->g) | reinterpret_cast<uintptr_t>(s0.src)) & 15) != 0) return WC_E_SHAPE;
    if ((long)a->B * a->Hm * a->Wm * s0.ldc * 4 >= (1L << 31) || (long)a->B * a->Hm * a->Wm * a->ldg * 4 >= (1L << 31))
        return WC_E_SHAPE;
    W3Dev d{};
    d.g = a->g; d.M = a->M; d.ldg = a->ldg;
    d.x = s0.src; d.C0 = s0.C; d.ldc0 = s0.ldc; d.scale = s0.scale; d.shift = s0.shift;
    d.B = a->B; d.H = a->Hm; d.W = a->Wm;
    d.part = part; d.Kc = 9 * s0.C;
    d.nblk = a->B * (a->Hm / TH) * (a->Wm / 16);
    d.nmt = a->M / (32 * WM);
    d.nct = s0.C / BC;
    if (splits < 1 || splits > d.nblk) return WC_E_SHAPE;
    d.bps = (d.nblk + splits - 1) / splits;
    if ((d.nblk + d.bps - 1) / d.bps != splits) return WC_E_SHAPE;  // as wc_conv_wgrad3_splits sizes it
    const long grid = (long)splits * d.nct * d.nmt;
    if (grid > (1L << 30)) return WC_E_SHAPE;
    const int pro = s0.scale ? (s0.silu ? 2 : 1) : 0;
    d.x_exp = x_exp;
    d.gbound = gbound;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    return f3 ? launch_w3_any<true>(WM, pro, d, (int)grid, s) : launch_w3_any<false>(WM, pro, d, (int)grid, s);
}

extern "C" int wc_conv_wgrad3(const wc_wgrad_args* a, float* part, int splits, void* stream) {
    return conv_wgrad3_any(a, part, splits, false, 0, nullptr, stream);
}

// f16x3 form: x_exp = the forward's exponent of segment 0's (GroupNorm-bounded) operand, gbound[B] =
// per-image max |G| (wc_absmax_images); same partial layout and reduce.
extern "C" int wc_conv_wgrad3_f16x3(const wc_wgrad_args* a, float* part, int splits, int x_exp, const float* gbound,
                                    void* stream) {
    return conv_wgrad3_any(a, part, splits, true, x_exp, gbound, stream);
}
