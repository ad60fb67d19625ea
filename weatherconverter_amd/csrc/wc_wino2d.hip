// ResBlock 3x3 conv on f16x3 MFMA through the 2D Winograd transform F(2x2, 3x3), position-major, for
// the wide convs (>= 4 output-channel tiles) whose input is pre-split once per element.
//
// F(2x2, 3x3): a 2x2 output tile needs the 4x4 input patch d (rows 2ty - 1 .. 2ty + 2, columns
// 2tx - 1 .. 2tx + 2); with B^T = [[1, 0, -1, 0], [0, 1, 1, 0], [0, -1, 1, 0], [0, 1, 0, -1]],
// G = [[1, 0, 0], [1/2, 1/2, 1/2], [1/2, -1/2, 1/2], [0, 0, 1]], A^T = [[1, 1, 1, 0], [0, 1, -1, -1]]:
//     V = B^T d B (16 positions P = (p, q)),  U = G g G^T,  M_P = sum_c V_P U_P,  y = A^T M A
// 16 products per 2x2 tile and input channel against the direct conv's 36 and the 1D F(2,3) form's 24
// (wc_wino.hip): 2/3 of the 1D form's MFMA work.  The 1D kernel keeps the accumulators of all four
// of its positions live; with 16 positions that state is 4 accumulators per output (the round-4 2D
// attempt, DESIGN.md §9, ran 2.7x slower from exactly that: one 32-row block per wave, each weight
// fragment feeding 3 MFMAs).  This kernel is POSITION-MAJOR instead: the K loop runs over (P, channel
// chunk) with P outermost, so a wave holds one position's M (2 blocks) plus the four outputs' y;
// when a position's chunks are done its M is folded into y (y_ij += A^T[i][p] A^T[j][q] M, the
// coefficients 0 / +-1: exact adds) and restarted.  A wave owns 64 tiles (256 pixels) x 32 output
// channels: every weight fragment feeds 6 MFMAs (the 1D form's ratio) over 2x the pixels, so the
// weight bytes per output are 2/3 of the 1D form's.
//
// Operands.  wino2d_vsplit_kernel applies GroupNorm + SiLU, x 2^s, the transform and the two-piece
// fp16 split once per 2x2 tile and writes the planes [b][chunk][piece][P][k-half][TY][TX] x 16 B (8
// channels); the fused 1x1 residual (raw input X under its per-image bound, unet_base.py:146-150)
// adds four more "positions", the tile's four pixels, whose planes hold X x 2^s split the same way and
// whose products go straight into y_ij.  The conv copies each K-step's A operand (2 pieces x 2 k-halves
// x 64 tiles, 4 KiB) into LDS by LDS-DMA (one 1-KiB wave-instruction per wave per step) through a
// 3-stage ring of 6-step stages, one barrier per stage; the weights (pre-split on the host, the
// filter transform in float64) go from L2 straight into three register sets two steps ahead.
// Range: |V| <= 4 max|d|, so the GN exponent drops by two (a_exp - 2); with a residual the shared
// exponent is also <= 13 - e(bound of X), as the 1D form.
// Epilogue: x 2^-(s + sW[n]), + bias + temb, + residual view, NHWC store, per-image absmax, GroupNorm
// tile partials in the slots the 1D kernels write (64-pixel blocks numbered by position).
// Reference: unet_base.py:87-109 (ResBlock convs), :146-150 (forward), SURVEY.md §8 row a3.
#include "wc_x6.hpp"

namespace {

using namespace wcx6;

constexpr int W2_NT = 256;
constexpr int W2_G = 6;                  // K-steps per LDS stage (a multiple of the 3 weight sets)
constexpr int W2_NS = 3;                 // ring stages
constexpr int W2_STEP = 4096;            // A bytes of one K-step: [piece 2][k-half 2][64 tiles][16 B]
constexpr int W2_STAGE = W2_G * W2_STEP;
constexpr int W2_LDS = W2_NS * W2_STAGE;
constexpr int W2_BN = 128;
constexpr int W2_BSTEP = W2_BN * 64;     // weight bytes of one K-step: [piece 2][k-half 2][128][8 fp16]

WC_DEVICE void lds16(__amdgpu_buffer_rsrc_t srd, void* dst, unsigned voff, int soff) {
    __builtin_amdgcn_raw_ptr_buffer_load_lds(srd, (__attribute__((address_space(3))) void*)dst, 16, voff, soff, 0, 0);
}

// the per-image exponent shared by the transformed segment and the residual (both kernels)
WC_DEVICE int w2_exp(int a_exp2, const float* abound, int b) {
    int s = a_exp2;
    if (abound) {
        const float bnd = abound[b];
        const int e = (int)((__float_as_uint(bnd) >> 23) & 0xffu) - 127;
        if (bnd > 0.f) s = min(s, 13 - e);
        s = max(s, -100);
    }
    return s;
}

struct W2Dev {
    const unsigned char* v;   // segment-0 planes, image b at v + b * vimg
    long vimg;
    const unsigned char* vr;  // residual planes, image b at vr + b * rimg (RES)
    long rimg;
    int B, H, W, N, TY, TX;
    int nck0, nck1, spad;     // 16-channel chunks of the segments; K-steps padded to a multiple of W2_G
    const void* w;
    const float* bias;
    const float* temb;
    int temb_ld;
    const float* res;
    int ldres;
    float* out;
    int ldo;
    int a_exp2;               // a_exp - 2
    const float* abound;
    const float* wsinv;
    float* absmax;
    float* gn_part;
    int gn_ncb, gn_sw, gn_c0, gn_np64;
    int mtiles_x, mtiles_y, ntiles_n;
};

template <bool RES>
__global__ __launch_bounds__(W2_NT) __attribute__((amdgpu_waves_per_eu(2, 2))) void conv3x3_wino2d_kernel(W2Dev p) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int tid = threadIdx.x, lane = tid & 63;
    // wave-uniform in an SGPR: the LDS-DMA's LDS base (M0) and scalar offset derive from it (as a VGPR
    // value the compiler wraps every DMA in a waterfall loop)
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int l32 = lane & 31, half = lane >> 5;
    // XCD-aware bijective tile order (wc_conv6.hip): consecutive logical tiles -- the N tiles of one
    // pixel block, which share its A planes -- on one XCD's L2
    int bid = blockIdx.x;
    {
        const int nblk = gridDim.x, q = nblk / 8, r = nblk % 8, xcd = bid % 8;
        bid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + bid / 8;
    }
    const int tile_n = bid % p.ntiles_n;
    int tt = bid / p.ntiles_n;
    const int mtx = tt % p.mtiles_x;
    tt /= p.mtiles_x;
    const int mty = tt % p.mtiles_y;
    const int b = tt / p.mtiles_y;
    const int ty0 = mty * 8, tx0 = mtx * 8, n0 = tile_n * W2_BN;
    const int s_exp = w2_exp(p.a_exp2, RES ? p.abound : nullptr, b);
    const float ainv = ldexpf(1.0f, -s_exp);
    const int nck0 = p.nck0, nck1 = RES ? p.nck1 : 0, nck1d = RES ? p.nck1 : 1;  // nck1d: divisor
    const int S0 = 16 * nck0, S = S0 + 4 * nck1, SP = p.spad;

    // LDS-DMA: wave w copies plane (piece w >> 1, k-half w & 1) of each K-step; lane = tile m
    // (8 x 8 tiles, row-major), one 16-byte fragment each
    const long plane = (long)p.TY * p.TX * 16;
    const unsigned vlane = (unsigned)(((ty0 + (lane >> 3)) * p.TX + tx0 + (lane & 7)) * 16);
    const int dpc = wave >> 1, dkh = wave & 1;
    const __amdgpu_buffer_rsrc_t srd0 = make_srd(p.v + (long)b * p.vimg);
    const __amdgpu_buffer_rsrc_t srdr = make_srd(RES ? (const void*)(p.vr + (long)b * p.rimg) : (const void*)p.v);
    // K-step position (segment, group, chunk): segment 0 = (position P, chunk c), 1 = (residual pixel o,
    // chunk c1), 2 = padding; one division per stage, then scalar increments
    struct Pos {
        int seg, g, c;
    };
    auto pos_of = [&](int st) {
        if (st < S0) return Pos{0, st / nck0, st % nck0};
        if (RES && st < S) return Pos{1, (st - S0) / nck1d, (st - S0) % nck1d};
        return Pos{2, 0, 0};
    };
    auto advance = [&](Pos& q) {
        if (q.seg == 2) return;
        if (++q.c == (q.seg == 0 ? nck0 : nck1d)) {
            q.c = 0;
            if (++q.g == (q.seg == 0 ? 16 : 4)) q = Pos{RES && q.seg == 0 ? 1 : 2, 0, 0};
        }
    };
    auto dma_step = [&](const Pos& q, unsigned char* dst) {
        if (q.seg == 0) {
            lds16(srd0, dst, vlane, (int)((((long)(q.c * 2 + dpc) * 16 + q.g) * 2 + dkh) * plane));
        } else if (RES && q.seg == 1) {
            lds16(srdr, dst, vlane, (int)((((long)(q.c * 2 + dpc) * 4 + q.g) * 2 + dkh) * plane));
        } else {
            lds16(srd0, dst, OOB, 0);  // a padding step: zeros, no traffic
        }
    };
    auto stage_buf = [&](int k) { return smem + (k % W2_NS) * W2_STAGE; };
    auto dma_stage = [&](int k) {
        unsigned char* base = stage_buf(k) + wave * 1024;
        Pos q = pos_of(k * W2_G);
#pragma unroll
        for (int s = 0; s < W2_G; ++s) {
            dma_step(q, base + s * W2_STEP);
            advance(q);
        }
    };

    // weights: K-step st of segment 0 is weight step st ((P, c) position-major), residual step
    // (o, c1) is weight step S0 + c1; padding steps re-read the last one (unused)
    const __amdgpu_buffer_rsrc_t srdw = make_srd(p.w);
    const unsigned wlane = (unsigned)(half * W2_BN * 16 + (wave * 32 + l32) * 16);
    const long wtile = (long)tile_n * (S0 + nck1) * W2_BSTEP;
    u32x4 wreg[3][2];
    auto load_w = [&](int set, int st) {
        int ws = st < S0 ? st : (st < S ? S0 + (st - S0) % nck1d : S0 + nck1 - 1);
        const int off = (int)(wtile + (long)ws * W2_BSTEP);
#pragma unroll
        for (int pc = 0; pc < 2; ++pc) wreg[set][pc] = bload_u4s(srdw, wlane + (unsigned)(pc * 2 * W2_BN * 16), off);
    };

    f32x16 M[2], Y[4][2];
#pragma unroll
    for (int mb = 0; mb < 2; ++mb) {
#pragma unroll
        for (int r = 0; r < 16; ++r) M[mb][r] = 0.f;
#pragma unroll
        for (int o = 0; o < 4; ++o)
#pragma unroll
            for (int r = 0; r < 16; ++r) Y[o][mb][r] = 0.f;
    }
    u32x4 fa[2][2][2];  // [set][mb][piece]
    auto read_a = [&](int fs, const unsigned char* sb) {
#pragma unroll
        for (int mb = 0; mb < 2; ++mb)
#pragma unroll
            for (int pc = 0; pc < 2; ++pc)
                fa[fs][mb][pc] = *reinterpret_cast<const u32x4*>(sb + ((pc * 2 + half) * 64 + 32 * mb + l32) * 16);
    };
    // the two blocks' chains interleaved: no MFMA waits on the one issued just before it
    auto mfma_step = [&](int fs, int set) {
#pragma unroll
        for (int mb = 0; mb < 2; ++mb) M[mb] = mfma_f16(fa[fs][mb][0], wreg[set][0], M[mb]);
#pragma unroll
        for (int mb = 0; mb < 2; ++mb) M[mb] = mfma_f16c(fa[fs][mb][0], wreg[set][1], M[mb]);
#pragma unroll
        for (int mb = 0; mb < 2; ++mb) M[mb] = mfma_f16c(fa[fs][mb][1], wreg[set][0], M[mb]);
    };
    // a group (one position's chunks, or one residual pixel's) ends at a step whose chunk is the last:
    // y_o += coef_o M, M = 0 (coef = A^T[i][p] A^T[j][q] in {0, +-1}: exact adds; residual pixel o: 1 at o)
    auto fold = [&](const Pos& q) {
        float cf[4];
        if (q.seg == 0) {
            const int pp = q.g >> 2, qq = q.g & 3;
            const float a0p = pp < 3 ? 1.f : 0.f, a1p = pp == 0 ? 0.f : (pp == 1 ? 1.f : -1.f);
            const float a0q = qq < 3 ? 1.f : 0.f, a1q = qq == 0 ? 0.f : (qq == 1 ? 1.f : -1.f);
            cf[0] = a0p * a0q; cf[1] = a0p * a1q; cf[2] = a1p * a0q; cf[3] = a1p * a1q;
        } else {
#pragma unroll
            for (int j = 0; j < 4; ++j) cf[j] = j == q.g ? 1.f : 0.f;
        }
#pragma unroll
        for (int o = 0; o < 4; ++o)
#pragma unroll
            for (int mb = 0; mb < 2; ++mb)
#pragma unroll
                for (int r = 0; r < 16; ++r) Y[o][mb][r] = __builtin_fmaf(cf[o], M[mb][r], Y[o][mb][r]);
#pragma unroll
        for (int mb = 0; mb < 2; ++mb)
#pragma unroll
            for (int r = 0; r < 16; ++r) M[mb][r] = 0.f;
    };
    auto group_end = [&](const Pos& q) {
        return q.seg != 2 && q.c == (q.seg == 0 ? nck0 : nck1d) - 1;
    };

    // ---- K loop: stage k (W2_G steps) computes from ring buffer k % 3 while stage k + 2 is copied in;
    // per wave and stage W2_G LDS-DMA + 2 W2_G weight loads: at a stage's end the next stage's copies
    // (issued one stage earlier) are complete once at most 3 W2_G + 4 vector-memory ops are outstanding
    const int nstages = SP / W2_G;
    dma_stage(0);
    dma_stage(1);
    load_w(0, 0);
    load_w(1, 1);
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(W2_G + 4) : "memory");
    __syncthreads();
    Pos cq = pos_of(0);  // the computed step's position
    for (int k = 0; k < nstages; ++k) {
        dma_stage(k + 2);
        const unsigned char* sb = stage_buf(k);
        read_a(0, sb);
#pragma unroll
        for (int s = 0; s < W2_G; ++s) {
            const int st = k * W2_G + s;
            load_w((s + 2) % 3, st + 2);
            __builtin_amdgcn_sched_barrier(0);
            if (s + 1 < W2_G) read_a((s + 1) & 1, sb + (s + 1) * W2_STEP);
            mfma_step(s & 1, s % 3);
            if (group_end(cq)) fold(cq);
            advance(cq);
        }
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(3 * W2_G + 4) : "memory");
        __syncthreads();
    }

    // ---- epilogue: x 2^-(s + sW[n]), + bias + temb, + residual view, NHWC store, absmax, GN partials ----
    const long img_px = (long)b * p.H * p.W;
    const __amdgpu_buffer_rsrc_t srd_out = make_srd(p.out + img_px * p.ldo);
    const __amdgpu_buffer_rsrc_t srd_res = make_srd(p.res ? p.res + img_px * p.ldres : p.out);
    const int n = n0 + wave * 32 + l32;
    const bool nok = n < p.N;
    float eadd = (nok && p.bias) ? p.bias[n] : 0.f;
    if (nok && p.temb) eadd += p.temb[b * p.temb_ld + n];
    const float emul = nok ? p.wsinv[n] * ainv : 0.f;
    float vmax = 0.f;
    // accumulator register r of block mb: MFMA row (r & 3) + 8 (r >> 2) + 4 half = tile (tile row 4 mb +
    // (r >> 2), tile column (r & 3) + 4 half); output o = (i, j) is pixel (2 (ty0 + tr) + i, 2 (tx0 + tc) + j)
#pragma unroll
    for (int mb = 0; mb < 2; ++mb)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int tr = 4 * mb + (r >> 2), tc = (r & 3) + 4 * half;
#pragma unroll
            for (int o = 0; o < 4; ++o) {
                const int y = 2 * (ty0 + tr) + (o >> 1), x = 2 * (tx0 + tc) + (o & 1);
                float v = Y[o][mb][r] * emul + eadd;
                if (p.res) v += bload_f1(srd_res, (unsigned)((y * p.W + x) * p.ldres + (nok ? n : 0)) * 4u);
                Y[o][mb][r] = v;
                vmax = fmaxf(vmax, fabsf(v));
                if (nok) bstore_f1(srd_out, (unsigned)((y * p.W + x) * p.ldo + n) * 4u, v);
            }
        }
    if (!nok) vmax = 0.f;
    if (p.absmax) block_absmax_atomic(p.absmax, b, vmax);
    if (p.gn_part && p.N - n0 - wave * 32 >= 32) {
        // 64-pixel blocks (4 pixel rows x 16 columns): block (mb, g) = registers 8 g .. 8 g + 7 of the four
        // outputs, both lane halves; slot numbered by position as the 1D kernels number it
        const int sw = p.gn_sw;
        const float inv_n = 1.0f / (64.0f * (float)sw);
        const int tiles_x16 = p.W / 16;
#pragma unroll
        for (int mb = 0; mb < 2; ++mb)
#pragma unroll
            for (int g = 0; g < 2; ++g) {
                float s = 0.f;
#pragma unroll
                for (int o = 0; o < 4; ++o)
#pragma unroll
                    for (int r = 8 * g; r < 8 * g + 8; ++r) s += Y[o][mb][r];
                const float mean = gn_seg_sum(s, sw) * inv_n;
                float q = 0.f;
#pragma unroll
                for (int o = 0; o < 4; ++o)
#pragma unroll
                    for (int r = 8 * g; r < 8 * g + 8; ++r) {
                        const float d = Y[o][mb][r] - mean;
                        q = fmaf(d, d, q);
                    }
                const float m2 = gn_seg_sum(q, sw);
                const int r4 = ty0 / 2 + 2 * mb + g;
                const long pix64 = (long)b * p.gn_np64 + ((r4 >> 1) * tiles_x16 + mtx) * 2 + (r4 & 1);
                const int c = lane & 31;
                if (lane < 32 && (c & (sw - 1)) == 0) {
                    const long idx = ((pix64 * p.gn_ncb + (p.gn_c0 + n0 + wave * 32) / 32) * (32 / sw) + c / sw) * 2;
                    p.gn_part[idx] = mean;
                    p.gn_part[idx + 1] = m2;
                }
            }
    }
}

// ---- wino2d_vsplit_kernel: the A planes of conv3x3_wino2d_kernel.  Segment-0 workgroups: 32 tiles x 32
// channels (thread = tile, channel quad): the tile's 4x4 patch through GN affine + SiLU + 2^s (zero
// outside the image), V = B^T d B, two fp16 pieces per value, 8-byte halves of the 16-byte fragments
// (8 lanes read one pixel's 128-byte line; for a fixed plane the lanes store 128-byte runs).  Residual
// workgroups (RES): the tile's four pixels of X x 2^s, split the same way, as positions 0..3.
__global__ __launch_bounds__(256) void wino2d_vsplit_kernel(const float* __restrict__ src, int ldc, int C0,
                                                            const float* __restrict__ scale,
                                                            const float* __restrict__ shift,
                                                            const float* __restrict__ src1, int ldc1, int C1, int H,
                                                            int W, int a_exp2, const float* __restrict__ abound,
                                                            unsigned char* __restrict__ v, long vimg,
                                                            unsigned char* __restrict__ vr, long rimg, int nb0) {
    const int TX = W / 2, TY = H / 2, tb_per_img = TY * TX / 32;
    const long plane = (long)TY * TX * 16;
    const int q8 = threadIdx.x & 7, tl = threadIdx.x >> 3;
    int blk = blockIdx.x;
    const bool res = blk >= nb0;
    if (res) blk -= nb0;
    const int ng = (res ? C1 : C0) / 32;
    const int grp = blk % ng, tb = (blk / ng) % tb_per_img, b = blk / (ng * tb_per_img);
    const int t = tb * 32 + tl, ty = t / TX, tx = t % TX;
    const float ascale = ldexpf(1.0f, w2_exp(a_exp2, abound, b));
    const int c = grp * 32 + 4 * q8;
    const int chunk = c / 16, kh = (c % 16) / 8, hf = (c % 8) / 4;
    const long frag = ((long)ty * TX + tx) * 16 + hf * 8;
    if (!res) {
        const f32x4 sc = *reinterpret_cast<const f32x4*>(scale + (long)b * C0 + c);
        const f32x4 sh = *reinterpret_cast<const f32x4*>(shift + (long)b * C0 + c);
        f32x4 d[4][4];
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int y = 2 * ty - 1 + i, x = 2 * tx - 1 + j;
                f32x4 a = {0.f, 0.f, 0.f, 0.f};
                if ((unsigned)y < (unsigned)H && (unsigned)x < (unsigned)W) {
                    const f32x4 r = *reinterpret_cast<const f32x4*>(src + (((long)b * H + y) * W + x) * ldc + c);
#pragma unroll
                    for (int e = 0; e < 4; ++e) a[e] = silu_fast(fmaf(r[e], sc[e], sh[e])) * ascale;
                }
                d[i][j] = a;
            }
        // rows: u[p][j] = (B^T d)[p][j]; columns: V[p][q] = (u B)[p][q]
        f32x4 u[4][4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            u[0][j] = d[0][j] - d[2][j];
            u[1][j] = d[1][j] + d[2][j];
            u[2][j] = d[2][j] - d[1][j];
            u[3][j] = d[1][j] - d[3][j];
        }
        unsigned char* vb = v + (long)b * vimg;
#pragma unroll
        for (int pp = 0; pp < 4; ++pp) {
            const f32x4 V[4] = {u[pp][0] - u[pp][2], u[pp][1] + u[pp][2], u[pp][2] - u[pp][1], u[pp][1] - u[pp][3]};
#pragma unroll
            for (int qq = 0; qq < 4; ++qq) {
                u32x2 h, l;
                split2_f16(V[qq], h, l);
                const int P = pp * 4 + qq;
                *reinterpret_cast<u32x2*>(vb + (((long)(chunk * 2 + 0) * 16 + P) * 2 + kh) * plane + frag) = h;
                *reinterpret_cast<u32x2*>(vb + (((long)(chunk * 2 + 1) * 16 + P) * 2 + kh) * plane + frag) = l;
            }
        }
    } else {
        unsigned char* rb = vr + (long)b * rimg;
#pragma unroll
        for (int o = 0; o < 4; ++o) {
            const int y = 2 * ty + (o >> 1), x = 2 * tx + (o & 1);
            const f32x4 a = *reinterpret_cast<const f32x4*>(src1 + (((long)b * H + y) * W + x) * ldc1 + c) * ascale;
            u32x2 h, l;
            split2_f16(a, h, l);
            *reinterpret_cast<u32x2*>(rb + (((long)(chunk * 2 + 0) * 4 + o) * 2 + kh) * plane + frag) = h;
            *reinterpret_cast<u32x2*>(rb + (((long)(chunk * 2 + 1) * 4 + o) * 2 + kh) * plane + frag) = l;
        }
    }
}

// shared checks; fills d (everything but the plane pointers)
int wino2d_setup(const wc_conv_args* a, int a_exp, const float* a_bound, W2Dev& d) {
    if (!a || !a->out || a->nseg < 1 || a->nseg > 2) return WC_E_ARG;
    const wc_conv_seg& s0 = a->seg[0];
    if (!s0.src || !s0.scale || !s0.shift || !s0.silu) return WC_E_ARG;  // the GN + SiLU segment
    if (a->act != WC_ACT_NONE || a_exp < -60 || a_exp > 60) return WC_E_ARG;
    if (s0.ntaps != 9 || s0.sy != 1 || s0.sx != 1 || s0.kbase != 0) return WC_E_SHAPE;
    for (int t = 0; t < 9; ++t)
        if (s0.dy[t] != t / 3 - 1 || s0.dx[t] != t % 3 - 1) return WC_E_SHAPE;
    if (s0.C <= 0 || s0.C % 32 || s0.ldc % 4 || (reinterpret_cast<uintptr_t>(s0.src) & 15)) return WC_E_SHAPE;
    if (a->B <= 0 || a->N <= 0 || s0.H != a->Hm || s0.W != a->Wm || a->Hm % 16 || a->Wm % 16) return WC_E_SHAPE;
    if ((long)a->B * s0.H * s0.W * s0.ldc * 4 >= (1L << 31)) return WC_E_SHAPE;
    d = W2Dev{};
    d.nck0 = s0.C / 16;
    const bool res = a->nseg == 2;
    if (res) {
        const wc_conv_seg& s1 = a->seg[1];
        if (!s1.src || s1.scale || !a_bound) return WC_E_ARG;
        if (s1.ntaps != 1 || s1.dy[0] != 0 || s1.dx[0] != 0 || s1.sy != 1 || s1.sx != 1) return WC_E_SHAPE;
        if (s1.H != s0.H || s1.W != s0.W || s1.kbase != 9 * s0.C) return WC_E_SHAPE;
        if (s1.C <= 0 || s1.C % 32 || s1.ldc % 4 || (reinterpret_cast<uintptr_t>(s1.src) & 15)) return WC_E_SHAPE;
        if ((long)a->B * s1.H * s1.W * s1.ldc * 4 >= (1L << 31)) return WC_E_SHAPE;
        d.nck1 = s1.C / 16;
    }
    if (a->out_nchw || a->Ho != a->Hm || a->Wo != a->Wm || a->osy != 1 || a->osx != 1 || a->ooy || a->oox)
        return WC_E_SHAPE;
    if ((long)a->Hm * a->Wm * a->ldo * 4 >= (1L << 31) || (a->res && (long)a->Hm * a->Wm * a->ldres * 4 >= (1L << 31)))
        return WC_E_SHAPE;
    d.B = a->B; d.H = a->Hm; d.W = a->Wm; d.N = a->N; d.TY = a->Hm / 2; d.TX = a->Wm / 2;
    const int S = 16 * d.nck0 + 4 * d.nck1;
    d.spad = (S + W2_G - 1) / W2_G * W2_G;
    d.a_exp2 = a_exp - 2;
    d.abound = res ? a_bound : nullptr;
    d.mtiles_x = d.TX / 8; d.mtiles_y = d.TY / 8; d.ntiles_n = (a->N + W2_BN - 1) / W2_BN;
    d.vimg = (long)16 * s0.C * d.H * d.W;
    d.rimg = res ? (long)4 * a->seg[1].C * d.H * d.W : 0;
    if (d.vimg >= (1L << 31) || d.rimg >= (1L << 31)) return WC_E_SHAPE;
    return WC_OK;
}

}  // namespace

extern "C" int wc_wino2d_bytes(int B, int C0, int C1, int H, int W, int64_t* v_bytes, int64_t* r_bytes) {
    if (!v_bytes || !r_bytes || B <= 0 || C0 <= 0 || C0 % 32 || C1 < 0 || C1 % 32 || H % 16 || W % 16 || H <= 0 || W <= 0)
        return WC_E_SHAPE;
    *v_bytes = (int64_t)B * 16 * C0 * H * W;
    *r_bytes = (int64_t)B * 4 * C1 * H * W;
    return WC_OK;
}

extern "C" int wc_wino2d_vsplit_f16x3(const wc_conv_args* a, int a_exp, const float* a_bound, void* v, int64_t v_bytes,
                                      void* vr, int64_t r_bytes, void* stream) {
    W2Dev d;
    const int st = wino2d_setup(a, a_exp, a_bound, d);
    if (st != WC_OK) return st;
    const bool res = a->nseg == 2;
    if (!v || (reinterpret_cast<uintptr_t>(v) & 15) || v_bytes != (int64_t)d.B * d.vimg) return WC_E_SHAPE;
    if (res && (!vr || (reinterpret_cast<uintptr_t>(vr) & 15) || r_bytes != (int64_t)d.B * d.rimg)) return WC_E_SHAPE;
    const wc_conv_seg& s0 = a->seg[0];
    const int tb = d.TY * d.TX / 32;
    const long nb0 = (long)d.B * tb * (s0.C / 32);
    const long nb1 = res ? (long)d.B * tb * (a->seg[1].C / 32) : 0;
    if (nb0 + nb1 >= (1L << 31)) return WC_E_SHAPE;
    wc_last_kernel = "wino2d_vsplit_kernel";
    hipLaunchKernelGGL(wino2d_vsplit_kernel, dim3((unsigned)(nb0 + nb1)), dim3(256), 0,
                       reinterpret_cast<hipStream_t>(stream), s0.src, s0.ldc, s0.C, s0.scale, s0.shift,
                       res ? a->seg[1].src : s0.src, res ? a->seg[1].ldc : s0.ldc, res ? a->seg[1].C : 0, d.H, d.W,
                       d.a_exp2, res ? a_bound : nullptr, reinterpret_cast<unsigned char*>(v), d.vimg,
                       reinterpret_cast<unsigned char*>(res ? vr : v), d.rimg, (int)nb0);
    WC_CHECK_LAUNCH();
    return WC_OK;
}

extern "C" int wc_conv3x3_wino2d_f16x3(const wc_conv_args* a, const void* w, int64_t w_bytes, int a_exp,
                                       const float* w_inv_scale, const float* a_bound, const void* v, int64_t v_bytes,
                                       const void* vr, int64_t r_bytes, void* stream) {
    W2Dev d;
    const int st = wino2d_setup(a, a_exp, a_bound, d);
    if (st != WC_OK) return st;
    const bool res = a->nseg == 2;
    if (!w || !w_inv_scale || (reinterpret_cast<uintptr_t>(w) & 15)) return WC_E_ARG;
    if (!v || (reinterpret_cast<uintptr_t>(v) & 15) || v_bytes != (int64_t)d.B * d.vimg) return WC_E_SHAPE;
    if (res && (!vr || (reinterpret_cast<uintptr_t>(vr) & 15) || r_bytes != (int64_t)d.B * d.rimg)) return WC_E_SHAPE;
    const long wsteps = 16L * d.nck0 + d.nck1;
    if (w_bytes != (long)d.ntiles_n * wsteps * W2_BSTEP || w_bytes >= (1L << 31)) return WC_E_SHAPE;
    d.v = reinterpret_cast<const unsigned char*>(v);
    d.vr = reinterpret_cast<const unsigned char*>(res ? vr : v);
    d.w = w; d.bias = a->bias; d.temb = a->temb; d.temb_ld = a->temb_ld;
    d.res = a->res; d.ldres = a->ldres; d.out = a->out; d.ldo = a->ldo;
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
    const long nblk = (long)d.B * d.mtiles_y * d.mtiles_x * d.ntiles_n;
    if (nblk >= (1L << 31)) return WC_E_SHAPE;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    static bool attr_set[2] = {false, false};
    if (!attr_set[res]) {
        hipError_t e = hipFuncSetAttribute(res ? reinterpret_cast<const void*>(&conv3x3_wino2d_kernel<true>)
                                               : reinterpret_cast<const void*>(&conv3x3_wino2d_kernel<false>),
                                           hipFuncAttributeMaxDynamicSharedMemorySize, W2_LDS);
        if (e != hipSuccess) return (int)e;
        attr_set[res] = true;
    }
    if (res) {
        WC_SET_NAME("conv3x3_wino2d_kernel", {WC_TB(true)});
        hipLaunchKernelGGL(conv3x3_wino2d_kernel<true>, dim3((unsigned)nblk), dim3(W2_NT), W2_LDS, s, d);
    } else {
        WC_SET_NAME("conv3x3_wino2d_kernel", {WC_TB(false)});
        hipLaunchKernelGGL(conv3x3_wino2d_kernel<false>, dim3((unsigned)nblk), dim3(W2_NT), W2_LDS, s, d);
    }
    WC_CHECK_LAUNCH();
    return WC_OK;
}
