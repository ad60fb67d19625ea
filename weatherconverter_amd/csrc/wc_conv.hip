// Implicit-GEMM convolution on fp32 MFMA for gfx950.
//
// GEMM view: M = B*Hm*Wm output positions (NHWC pixels), N = output channels, K = sum over
// segments of ntaps*C (tap-major, channel-minor; the packed weight is [N][K], K contiguous).
// One workgroup = 4 waves computing a BM x BN tile; each wave owns a 64x64 sub-tile made of 2x2
// v_mfma_f32_32x32x2_f32 accumulators (64 accumulator registers per lane).  A K-step stages 32
// input channels of one tap for BM pixels and the matching 32 K-columns of BN weight rows.
//
// Pipeline (one barrier per K-step): the global loads of step k+1 are issued before the 64 MFMAs
// of step k; after the MFMAs the wave applies the GroupNorm+SiLU prologue to them and writes them
// into the OTHER LDS buffer; then one barrier.  Two workgroups per CU let one block's prologue VALU
// run beside the other block's MFMAs on each SIMD.
//
// Loads are raw buffer loads (SRD with a 2 GiB range): a padding tap or an out-of-range row gets
// an out-of-range offset and reads 0 with no branch.  Per-thread pixel offsets are computed once;
// a K-step only adds the uniform tap offset (dy*W + dx)*ldc + c0, advanced by a scalar state
// machine (segment, tap, channel block).
//
// LDS tiles are [rows][32 floats] (128 B rows, no padding) with the 16-byte chunk index XOR-ed by
// ((row >> 1) & 7): the ds_read_b128 fragment reads (16 lanes = 16 distinct rows, same chunk) and
// the ds_write_b128 staging writes (8 lanes = 8 chunks of one row) are both bank-conflict-free.
//
// Fused work (reference unet_base.py ResBlock, :87-109 / :146-150):
//   prologue  (segment 0)    v <- SiLU(v*scale[b,c] + shift[b,c])   [GroupNorm-apply (+ SiLU)]
//                            zero padding is applied AFTER the prologue, as Conv2d pads the
//                            SiLU output
//   segment 1 (optional)     the 1x1 residual_input_conv appended as extra K columns (raw input)
//   epilogue                 + bias[n] + temb[b,n] + residual view, NHWC or NCHW store
#include "wc_common.hpp"

namespace {

constexpr int BK = 32;  // channels per K-step (one LDS row = 128 B)
constexpr int NTHREADS = 256;
constexpr unsigned OOB = 0x80000000u;  // byte offset past the SRD range -> load returns 0
constexpr int SRD_BYTES = 0x7FFFFFFF;
constexpr int SRD_FLAGS = 0x00020000;

struct SegDev {
    const float* src;
    int C, ldc, H, W, sy, sx, ntaps, kbase;
    int dy[WC_MAX_TAPS];
    int dx[WC_MAX_TAPS];
    const float* scale;
    const float* shift;
};

struct ConvDev {
    SegDev seg[2];
    int nseg;
    int B, Hm, Wm, N, M;
    const float* w;
    int ldw;
    const float* bias;
    const float* temb;
    int temb_ld;
    const float* res;
    int ldres;
    float* out;
    int ldo;
    int Ho, Wo, osy, osx, ooy, oox, out_nchw;
    int ident;    // output position == GEMM row (plain NHWC store)
    int steps;    // total K-steps
    int ntiles_n; // N tiles
};

template <int BM, int BN>
struct Tile {
    static constexpr int WAVES_M = BM / 64;
    static constexpr int WAVES_N = BN / 64;
    static_assert(WAVES_M * WAVES_N == 4, "4 waves of 64x64");
    static constexpr int A_PER_T = BM * (BK / 4) / NTHREADS;  // float4 per thread
    static constexpr int B_PER_T = BN * (BK / 4) / NTHREADS;
    static constexpr int STAGE = (BM + BN) * BK;              // floats per LDS buffer
};

WC_DEVICE float silu_fast(float v) {
    // v * sigmoid(v) with v_exp_f32 and v_rcp_f32 (~2 ulp); exp overflow gives rcp(inf) = 0.
    return v * __builtin_amdgcn_rcpf(1.0f + __expf(-v));
}

WC_DEVICE f32x4 bload4(__amdgpu_buffer_rsrc_t r, unsigned off) {
    return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0));
}

WC_DEVICE __amdgpu_buffer_rsrc_t make_srd(const float* p) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(p), (short)0, SRD_BYTES, SRD_FLAGS);
}

// PRO: 0 = raw segment 0, 1 = GN affine, 2 = GN affine + SiLU.
// UNIB: every tile lies inside one image (Hm*Wm % BM == 0) -> one (scale, shift) per step.
template <int BM, int BN, int PRO, bool UNIB>
__global__ __launch_bounds__(NTHREADS, 2) void conv_igemm_kernel(ConvDev p) {
    using T = Tile<BM, BN>;
    __shared__ __attribute__((aligned(16))) float lds[2 * T::STAGE];

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;
    const int wm = wave / T::WAVES_N;
    const int wn = wave % T::WAVES_N;

    // XCD-aware tile order (bijective): consecutive logical tiles, which share A rows, are placed
    // on the same XCD so their im2col re-reads hit one L2.
    const int nblk = gridDim.x;
    int bid = blockIdx.x;
    {
        int q = nblk / 8, r = nblk % 8, xcd = bid % 8;
        bid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + bid / 8;
    }
    const int tile_m = bid / p.ntiles_n;
    const int tile_n = bid % p.ntiles_n;
    const int m0 = tile_m * BM;
    const int n0 = tile_n * BN;
    const int HWm = p.Hm * p.Wm;

    // ---- per-thread staging coordinates ----
    const int q4 = tid & 7;     // 16-byte chunk (4 channels) within the 32-channel step
    const int prow = tid >> 3;  // 0..31
    const int wsw = ((q4 ^ ((prow >> 1) & 7)) << 2);  // swizzled column of this thread's writes
    int pb[T::A_PER_T], py[T::A_PER_T], px[T::A_PER_T];
#pragma unroll
    for (int j = 0; j < T::A_PER_T; ++j) {
        int m = m0 + prow + 32 * j;
        if (m < p.M) {
            int b = m / HWm;
            int r = m - b * HWm;
            pb[j] = b;
            py[j] = r / p.Wm;
            px[j] = r - py[j] * p.Wm;
        } else {
            pb[j] = -1; py[j] = -(1 << 20); px[j] = 0;  // never in range
        }
    }
    const int b_tile = m0 / HWm;  // the image of the whole tile when UNIB

    // ---- scalar K-step state machine for the NEXT load ----
    int ls = 0, ltap = 0, lc0 = 0;   // segment, tap, channel block of the next load
    // per-segment, per-thread pixel origin offsets (floats) and sampling coordinates
    int org[T::A_PER_T], ys[T::A_PER_T], xs[T::A_PER_T];
    __amdgpu_buffer_rsrc_t srd_a = make_srd(p.seg[0].src);
    __amdgpu_buffer_rsrc_t srd_w = make_srd(p.w);
    __amdgpu_buffer_rsrc_t srd_sc = make_srd(PRO ? p.seg[0].scale : p.w);
    __amdgpu_buffer_rsrc_t srd_sh = make_srd(PRO ? p.seg[0].shift : p.w);
    int sH = p.seg[0].H, sW = p.seg[0].W, sldc = p.seg[0].ldc, sC = p.seg[0].C;
    int sntaps = p.seg[0].ntaps, skbase = p.seg[0].kbase;

    auto set_segment = [&](int s) {
        const SegDev& sg = p.seg[s];
        srd_a = make_srd(sg.src);
        sH = sg.H; sW = sg.W; sldc = sg.ldc; sC = sg.C; sntaps = sg.ntaps; skbase = sg.kbase;
#pragma unroll
        for (int j = 0; j < T::A_PER_T; ++j) {
            ys[j] = py[j] * sg.sy;
            xs[j] = px[j] * sg.sx;
            org[j] = pb[j] < 0 ? 0 : ((pb[j] * sg.H + ys[j]) * sg.W + xs[j]) * sg.ldc + q4 * 4;
        }
    };
    set_segment(0);

    f32x4 ra[T::A_PER_T];
    f32x4 rb[T::B_PER_T];
    f32x4 rsc[UNIB ? 1 : T::A_PER_T], rsh[UNIB ? 1 : T::A_PER_T];
    unsigned aval = 0;
    bool stage_pro = PRO != 0;  // whether the staged data (in ra) takes the prologue

    auto load_step = [&]() {
        const int dy = p.seg[ls].dy[ltap], dx = p.seg[ls].dx[ltap];
        const int tap_off = (dy * sW + dx) * sldc + lc0;
        aval = 0;
#pragma unroll
        for (int j = 0; j < T::A_PER_T; ++j) {
            const int iy = ys[j] + dy, ix = xs[j] + dx;
            const bool ok = (unsigned)iy < (unsigned)sH && (unsigned)ix < (unsigned)sW;
            aval |= (ok ? 1u : 0u) << j;
            ra[j] = bload4(srd_a, ok ? (unsigned)(org[j] + tap_off) * 4u : OOB);
        }
        stage_pro = PRO != 0 && ls == 0;
        if constexpr (PRO != 0) {
            if (ls == 0) {
                const int c = lc0 + q4 * 4;
                if constexpr (UNIB) {
                    rsc[0] = bload4(srd_sc, (unsigned)(b_tile * sC + c) * 4u);
                    rsh[0] = bload4(srd_sh, (unsigned)(b_tile * sC + c) * 4u);
                } else {
#pragma unroll
                    for (int j = 0; j < T::A_PER_T; ++j) {
                        const unsigned o = pb[j] >= 0 ? (unsigned)(pb[j] * sC + c) * 4u : OOB;
                        rsc[j] = bload4(srd_sc, o);
                        rsh[j] = bload4(srd_sh, o);
                    }
                }
            }
        }
        const int kcol = skbase + ltap * sC + lc0 + q4 * 4;
#pragma unroll
        for (int j = 0; j < T::B_PER_T; ++j) {
            const int n = n0 + prow + 32 * j;
            rb[j] = bload4(srd_w, n < p.N ? (unsigned)(n * p.ldw + kcol) * 4u : OOB);
        }
        // advance the state machine (uniform scalar branches)
        lc0 += BK;
        if (lc0 == sC) {
            lc0 = 0;
            if (++ltap == sntaps) {
                ltap = 0;
                if (++ls < p.nseg) set_segment(ls);
            }
        }
    };

    auto store_step = [&](float* buf) {
        if constexpr (PRO != 0) {
            if (stage_pro) {
#pragma unroll
                for (int j = 0; j < T::A_PER_T; ++j) {
                    f32x4 v = ra[j] * rsc[UNIB ? 0 : j] + rsh[UNIB ? 0 : j];
                    if constexpr (PRO == 2) {
                        v.x = silu_fast(v.x); v.y = silu_fast(v.y);
                        v.z = silu_fast(v.z); v.w = silu_fast(v.w);
                    }
                    ra[j] = v;
                }
            }
        }
#pragma unroll
        for (int j = 0; j < T::A_PER_T; ++j) {
            f32x4 v = ((aval >> j) & 1u) ? ra[j] : f32x4{0.f, 0.f, 0.f, 0.f};
            *reinterpret_cast<f32x4*>(buf + (prow + 32 * j) * BK + wsw) = v;
        }
        float* bbuf = buf + BM * BK;
#pragma unroll
        for (int j = 0; j < T::B_PER_T; ++j)
            *reinterpret_cast<f32x4*>(bbuf + (prow + 32 * j) * BK + wsw) = rb[j];
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
    const int rsw = (l32 >> 1) & 7;  // row swizzle of this lane's fragment rows
    int koff[4];
#pragma unroll
    for (int kq = 0; kq < 4; ++kq) koff[kq] = ((half * 4 + kq) ^ rsw) << 2;
    const int a_row = (wm * 64 + l32) * BK;
    const int b_row = BM * BK + (wn * 64 + l32) * BK;

    auto compute = [&](const float* buf) {
        f32x4 a0 = *reinterpret_cast<const f32x4*>(buf + a_row + koff[0]);
        f32x4 a1 = *reinterpret_cast<const f32x4*>(buf + a_row + 32 * BK + koff[0]);
        f32x4 b0 = *reinterpret_cast<const f32x4*>(buf + b_row + koff[0]);
        f32x4 b1 = *reinterpret_cast<const f32x4*>(buf + b_row + 32 * BK + koff[0]);
#pragma unroll
        for (int kq = 0; kq < 4; ++kq) {
            f32x4 na0, na1, nb0, nb1;
            if (kq < 3) {  // prefetch the next chunk's fragments under this chunk's MFMAs
                na0 = *reinterpret_cast<const f32x4*>(buf + a_row + koff[kq + 1]);
                na1 = *reinterpret_cast<const f32x4*>(buf + a_row + 32 * BK + koff[kq + 1]);
                nb0 = *reinterpret_cast<const f32x4*>(buf + b_row + koff[kq + 1]);
                nb1 = *reinterpret_cast<const f32x4*>(buf + b_row + 32 * BK + koff[kq + 1]);
            }
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                acc[0][0] = mfma32(a0[j], b0[j], acc[0][0]);
                acc[0][1] = mfma32(a0[j], b1[j], acc[0][1]);
                acc[1][0] = mfma32(a1[j], b0[j], acc[1][0]);
                acc[1][1] = mfma32(a1[j], b1[j], acc[1][1]);
            }
            if (kq < 3) { a0 = na0; a1 = na1; b0 = nb0; b1 = nb1; }
        }
    };

    load_step();
    store_step(lds);
    __syncthreads();

    for (int step = 0; step < p.steps; ++step) {
        float* cur = lds + (step & 1) * T::STAGE;
        float* nxt = lds + ((step & 1) ^ 1) * T::STAGE;
        const bool more = step + 1 < p.steps;
        if (more) load_step();
        compute(cur);
        if (more) store_step(nxt);
        __syncthreads();
    }

    // ---- epilogue ----
    const int HWo = p.Ho * p.Wo;
#pragma unroll
    for (int mb = 0; mb < 2; ++mb) {
        const int mbase = m0 + wm * 64 + mb * 32;
        const int b0 = mbase / HWm;
        const int bnd = (b0 + 1) * HWm;  // first row of the next image
#pragma unroll
        for (int nb = 0; nb < 2; ++nb) {
            const int n = n0 + wn * 64 + nb * 32 + l32;
            if (n >= p.N) continue;
            const float bn = p.bias ? p.bias[n] : 0.f;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int row = (r & 3) + 8 * (r >> 2) + 4 * half;
                const int m = mbase + row;
                if (m >= p.M) continue;
                int b = (HWm >= 32) ? b0 + (m >= bnd ? 1 : 0) : m / HWm;
                float v = acc[mb][nb][r] + bn;
                if (p.temb) v += p.temb[b * p.temb_ld + n];
                if (p.ident) {
                    if (p.res) v += p.res[(long)m * p.ldres + n];
                    p.out[(long)m * p.ldo + n] = v;
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
                }
            }
        }
    }
}

template <int BM, int BN, int PRO, bool UNIB>
int launch(const ConvDev& d, hipStream_t stream) {
    ConvDev p = d;
    int tiles_m = (p.M + BM - 1) / BM;
    p.ntiles_n = (p.N + BN - 1) / BN;
    dim3 grid(tiles_m * p.ntiles_n);
    hipLaunchKernelGGL((conv_igemm_kernel<BM, BN, PRO, UNIB>), grid, dim3(NTHREADS), 0, stream, p);
    WC_CHECK_LAUNCH();
    return WC_OK;
}

template <int BM, int BN>
int dispatch(const ConvDev& d, int pro, hipStream_t s) {
    const bool unib = (d.Hm * d.Wm) % BM == 0;
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

extern "C" int wc_conv_igemm(const wc_conv_args* a, void* stream) {
    if (!a || !a->w || !a->out) return WC_E_ARG;
    if (a->nseg < 1 || a->nseg > 2) return WC_E_ARG;
    ConvDev d{};
    long k = 0;
    for (int s = 0; s < a->nseg; ++s) {
        const wc_conv_seg& sg = a->seg[s];
        if (!sg.src) return WC_E_ARG;
        if (sg.C <= 0 || sg.C % BK != 0 || sg.ldc % 4 != 0) return WC_E_SHAPE;
        if (sg.ntaps < 1 || sg.ntaps > WC_MAX_TAPS) return WC_E_SHAPE;
        if ((reinterpret_cast<uintptr_t>(sg.src) & 15) != 0) return WC_E_SHAPE;
        if ((sg.scale == nullptr) != (sg.shift == nullptr)) return WC_E_ARG;
        if (s == 1 && sg.scale) return WC_E_ARG;  // the residual segment is read raw
        // every byte offset the kernel forms must stay below the 2 GiB buffer range
        if ((long)a->B * sg.H * sg.W * sg.ldc * 4 >= (1L << 31)) return WC_E_SHAPE;
        SegDev& o = d.seg[s];
        o.src = sg.src; o.C = sg.C; o.ldc = sg.ldc; o.H = sg.H; o.W = sg.W;
        o.sy = sg.sy; o.sx = sg.sx; o.ntaps = sg.ntaps; o.kbase = sg.kbase;
        for (int t = 0; t < sg.ntaps; ++t) { o.dy[t] = sg.dy[t]; o.dx[t] = sg.dx[t]; }
        o.scale = sg.scale; o.shift = sg.shift;
        if (sg.kbase + sg.ntaps * sg.C > a->ldw) return WC_E_SHAPE;
        k += (long)sg.ntaps * sg.C;
    }
    if (a->ldw % 4 != 0 || (reinterpret_cast<uintptr_t>(a->w) & 15) != 0) return WC_E_SHAPE;
    if ((long)a->N * a->ldw * 4 >= (1L << 31)) return WC_E_SHAPE;
    d.nseg = a->nseg;
    d.B = a->B; d.Hm = a->Hm; d.Wm = a->Wm; d.N = a->N;
    long M = (long)a->B * a->Hm * a->Wm;
    if (M <= 0 || M > (1L << 30) || a->N <= 0) return WC_E_SHAPE;
    d.M = (int)M;
    d.w = a->w; d.ldw = a->ldw; d.bias = a->bias; d.temb = a->temb; d.temb_ld = a->temb_ld;
    d.res = a->res; d.ldres = a->ldres; d.out = a->out; d.ldo = a->ldo;
    d.Ho = a->Ho; d.Wo = a->Wo; d.osy = a->osy; d.osx = a->osx; d.ooy = a->ooy; d.oox = a->oox;
    d.out_nchw = a->out_nchw;
    d.ident = !a->out_nchw && a->osy == 1 && a->osx == 1 && a->ooy == 0 && a->oox == 0 &&
              a->Ho == a->Hm && a->Wo == a->Wm;
    d.steps = (int)(k / BK);
    const int pro = a->seg[0].scale ? (a->seg[0].silu ? 2 : 1) : 0;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    // 64-column outputs (C_out = 64 stages, the 3-channel head) use a 256x64 tile.
    if (a->N <= 64) return dispatch<256, 64>(d, pro, s);
    return dispatch<128, 128>(d, pro, s);
}
