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

struct ConvDev {
    // segment 0: the conv input, read through a kh x kw tap grid, optional GN prologue
    const float* src0;
    int C0, ldc0, H0, W0, sy, sx;
    int kh, kw, ty0, tdy, tx0, tdx;  // tap (ky, kx) reads input (y*sy + ty0 + ky*tdy, x*sx + tx0 + kx*tdx)
    const float* scale;
    const float* shift;
    // segment 1 (optional): raw 1x1 input at the same pixel (the fused residual_input_conv)
    const float* src1;
    int C1, ldc1, kbase1;
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
    int steps0;   // K-steps of segment 0
    int steps;    // total K-steps
    int ntiles_n; // N tiles
    const float* act_param;  // PReLU slopes [N]
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
// ACT: epilogue activation (WC_ACT_*), a template parameter: a runtime branch to an inlined erff
// makes the 64-element epilogue too large to unroll, which moves the accumulators to scratch and
// slows every instantiation ~1.8x.
template <int BM, int BN, int PRO, bool UNIB, int ACT>
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

    // ---- per-thread staging coordinates (fixed for the whole K loop) ----
    const int q4 = tid & 7;     // 16-byte chunk (4 channels) within the 32-channel step
    const int prow = tid >> 3;  // 0..31
    const int wsw = ((q4 ^ ((prow >> 1) & 7)) << 2);  // swizzled column of this thread's writes
    int pb[T::A_PER_T], ys[T::A_PER_T], xs[T::A_PER_T], org0[T::A_PER_T], org1[T::A_PER_T];
#pragma unroll
    for (int j = 0; j < T::A_PER_T; ++j) {
        const int m = m0 + prow + 32 * j;
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
            pb[j] = -1; ys[j] = -(1 << 24); xs[j] = 0; org0[j] = 0; org1[j] = 0;  // never in range
        }
    }
    const int b_tile = m0 / HWm;  // the image of the whole tile when UNIB

    const __amdgpu_buffer_rsrc_t srd0 = make_srd(p.src0);
    const __amdgpu_buffer_rsrc_t srd1 = make_srd(p.src1 ? p.src1 : p.src0);
    const __amdgpu_buffer_rsrc_t srdw = make_srd(p.w);
    const __amdgpu_buffer_rsrc_t srdsc = make_srd(PRO ? p.scale : p.w);
    const __amdgpu_buffer_rsrc_t srdsh = make_srd(PRO ? p.shift : p.w);

    f32x4 ra[T::A_PER_T];
    f32x4 rb[T::B_PER_T];
    f32x4 rsc[UNIB ? 1 : T::A_PER_T], rsh[UNIB ? 1 : T::A_PER_T];
    unsigned aval = 0;

    // scalar state of the NEXT load in segment 0: tap (ky, kx) and channel block c0
    int ky = 0, kx = 0, c0 = 0;

    auto load_w = [&](int kcol) {
#pragma unroll
        for (int j = 0; j < T::B_PER_T; ++j) {
            const int n = n0 + prow + 32 * j;
            rb[j] = bload4(srdw, n < p.N ? (unsigned)(n * p.ldw + kcol) * 4u : OOB);
        }
    };
    auto load0 = [&]() {
        const int dy = p.ty0 + ky * p.tdy, dx = p.tx0 + kx * p.tdx;
        const int tap_off = (dy * p.W0 + dx) * p.ldc0 + c0;
        aval = 0;
#pragma unroll
        for (int j = 0; j < T::A_PER_T; ++j) {
            const int iy = ys[j] + dy, ix = xs[j] + dx;
            const bool ok = (unsigned)iy < (unsigned)p.H0 && (unsigned)ix < (unsigned)p.W0;
            aval |= (ok ? 1u : 0u) << j;
            ra[j] = bload4(srd0, ok ? (unsigned)(org0[j] + tap_off) * 4u : OOB);
        }
        if constexpr (PRO != 0) {
            const int c = c0 + q4 * 4;
            if constexpr (UNIB) {
                rsc[0] = bload4(srdsc, (unsigned)(b_tile * p.C0 + c) * 4u);
                rsh[0] = bload4(srdsh, (unsigned)(b_tile * p.C0 + c) * 4u);
            } else {
#pragma unroll
                for (int j = 0; j < T::A_PER_T; ++j) {
                    const unsigned o = pb[j] >= 0 ? (unsigned)(pb[j] * p.C0 + c) * 4u : OOB;
                    rsc[j] = bload4(srdsc, o);
                    rsh[j] = bload4(srdsh, o);
                }
            }
        }
        load_w((ky * p.kw + kx) * p.C0 + c0 + q4 * 4);
        // advance (branch-free scalar selects)
        c0 += BK;
        const bool wc = c0 == p.C0;
        c0 = wc ? 0 : c0;
        kx += wc ? 1 : 0;
        const bool wx = kx == p.kw;
        kx = wx ? 0 : kx;
        ky += wx ? 1 : 0;
    };
    int c1 = 0;  // next channel block of segment 1
    auto load1 = [&]() {
        aval = 0;
#pragma unroll
        for (int j = 0; j < T::A_PER_T; ++j) {
            aval |= (pb[j] >= 0 ? 1u : 0u) << j;
            ra[j] = bload4(srd1, pb[j] >= 0 ? (unsigned)(org1[j] + c1) * 4u : OOB);
        }
        load_w(p.kbase1 + c1 + q4 * 4);
        c1 += BK;
    };

    auto store = [&](float* buf, bool pro) {
        if constexpr (PRO != 0) {
            if (pro) {
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

    // MFMAs of k-chunks [KQ0, KQ1) (4 channels each); fragments of chunk kq+1 are read under chunk kq.
    f32x4 fa0, fa1, fb0, fb1;
    auto frag = [&](const float* buf, int kq) {
        fa0 = *reinterpret_cast<const f32x4*>(buf + a_row + koff[kq]);
        fa1 = *reinterpret_cast<const f32x4*>(buf + a_row + 32 * BK + koff[kq]);
        fb0 = *reinterpret_cast<const f32x4*>(buf + b_row + koff[kq]);
        fb1 = *reinterpret_cast<const f32x4*>(buf + b_row + 32 * BK + koff[kq]);
    };
    auto compute = [&](const float* buf, int kq0, int kq1, bool prefetch_next_step_frag) {
#pragma unroll
        for (int kq = kq0; kq < kq1; ++kq) {
            const f32x4 a0 = fa0, a1 = fa1, b0 = fb0, b1 = fb1;
            if (kq < 3) frag(buf, kq + 1);
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                acc[0][0] = mfma32(a0[j], b0[j], acc[0][0]);
                acc[0][1] = mfma32(a0[j], b1[j], acc[0][1]);
                acc[1][0] = mfma32(a1[j], b0[j], acc[1][0]);
                acc[1][1] = mfma32(a1[j], b1[j], acc[1][1]);
            }
        }
        (void)prefetch_next_step_frag;
    };

    // ---- K loop: one barrier per step; phase A loads segment 0, phase B segment 1 ----
    // Per step: [next step's buffer loads] [MFMA chunks 0-1] [MFMA chunks 2-3 interleaved with the
    // prologue VALU and the LDS writes of the next step, 1 MFMA : 5 VALU] [barrier].  The loads have
    // 32 MFMAs (~2k cycles) to land before the interleaved half consumes them.
#define WC_INTERLEAVE()                                                         \
    do {                                                                        \
        _Pragma("unroll") for (int i_ = 0; i_ < 32; ++i_) {                     \
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0); /* MFMA */       \
            __builtin_amdgcn_sched_group_barrier(0x002, 5, 0); /* VALU */       \
            if (i_ % 4 == 3)                                                    \
                __builtin_amdgcn_sched_group_barrier(0x200, 1, 0); /* DS wr */  \
        }                                                                       \
    } while (0)

    if (p.steps0 > 0) { load0(); store(lds, true); } else { load1(); store(lds, false); }
    __syncthreads();
    int step = 0;
    for (; step < p.steps0 - 1; ++step) {
        float* cur = lds + (step & 1) * T::STAGE;
        float* nxt = lds + ((step & 1) ^ 1) * T::STAGE;
        load0();
        __builtin_amdgcn_sched_barrier(0);  // keep the next step's loads ahead of the MFMAs
        frag(cur, 0);
        compute(cur, 0, 2, false);
        __builtin_amdgcn_sched_barrier(0);
        compute(cur, 2, 4, false);
        store(nxt, true);
        WC_INTERLEAVE();
        __builtin_amdgcn_sched_barrier(0);
        __syncthreads();
    }
    for (; step < p.steps - 1; ++step) {
        float* cur = lds + (step & 1) * T::STAGE;
        float* nxt = lds + ((step & 1) ^ 1) * T::STAGE;
        load1();
        __builtin_amdgcn_sched_barrier(0);
        frag(cur, 0);
        compute(cur, 0, 2, false);
        __builtin_amdgcn_sched_barrier(0);
        compute(cur, 2, 4, false);
        store(nxt, false);
        WC_INTERLEAVE();
        __builtin_amdgcn_sched_barrier(0);
        __syncthreads();
    }
    frag(lds + (step & 1) * T::STAGE, 0);
    compute(lds + (step & 1) * T::STAGE, 0, 4, false);
#undef WC_INTERLEAVE

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
                if constexpr (ACT == WC_ACT_GELU) v = 0.5f * v * (1.0f + erff(v * 0.70710678118654752f));
                else if constexpr (ACT == WC_ACT_SILU) v = v / (1.0f + __expf(-v));
                else if constexpr (ACT == WC_ACT_PRELU) v = v >= 0.f ? v : p.act_param[n] * v;
                else if constexpr (ACT == WC_ACT_TANH01) v = (tanhf(v) + 1.0f) * 0.5f;
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

template <int BM, int BN, int PRO, bool UNIB, int ACT = WC_ACT_NONE>
int launch(const ConvDev& d, hipStream_t stream) {
    ConvDev p = d;
    int tiles_m = (p.M + BM - 1) / BM;
    p.ntiles_n = (p.N + BN - 1) / BN;
    dim3 grid(tiles_m * p.ntiles_n);
    hipLaunchKernelGGL((conv_igemm_kernel<BM, BN, PRO, UNIB, ACT>), grid, dim3(NTHREADS), 0, stream, p);
    WC_CHECK_LAUNCH();
    return WC_OK;
}

template <int BM, int BN>
int dispatch(const ConvDev& d, int pro, int act, hipStream_t s) {
    const bool unib = (d.Hm * d.Wm) % BM == 0;
    if (act != WC_ACT_NONE) {  // activations are instantiated for a raw segment 0 only
        if (pro != 0) return WC_E_ARG;
        if (act == WC_ACT_GELU)
            return unib ? launch<BM, BN, 0, true, WC_ACT_GELU>(d, s) : launch<BM, BN, 0, false, WC_ACT_GELU>(d, s);
        if (act == WC_ACT_PRELU)
            return unib ? launch<BM, BN, 0, true, WC_ACT_PRELU>(d, s) : launch<BM, BN, 0, false, WC_ACT_PRELU>(d, s);
        if (act == WC_ACT_TANH01)
            return unib ? launch<BM, BN, 0, true, WC_ACT_TANH01>(d, s) : launch<BM, BN, 0, false, WC_ACT_TANH01>(d, s);
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

extern "C" int wc_conv_igemm(const wc_conv_args* a, void* stream) {
    if (!a || !a->w || !a->out) return WC_E_ARG;
    if (a->nseg < 1 || a->nseg > 2) return WC_E_ARG;
    if (a->absmax_out || a->gn_part) return WC_E_ARG;  // output bounds / GN partials: split-precision kernels
    ConvDev d{};
    const wc_conv_seg& s0 = a->seg[0];
    if (!s0.src) return WC_E_ARG;
    if (s0.C <= 0 || s0.C % BK != 0 || s0.ldc % 4 != 0) return WC_E_SHAPE;
    if (s0.ntaps < 1 || s0.ntaps > WC_MAX_TAPS) return WC_E_SHAPE;
    if ((reinterpret_cast<uintptr_t>(s0.src) & 15) != 0) return WC_E_SHAPE;
    if ((s0.scale == nullptr) != (s0.shift == nullptr)) return WC_E_ARG;
    if (s0.kbase != 0) return WC_E_SHAPE;
    if ((long)a->B * s0.H * s0.W * s0.ldc * 4 >= (1L << 31)) return WC_E_SHAPE;  // 2 GiB SRD range
    // the taps must form a kh x kw grid: tap t = (ty0 + (t / kw) * tdy, tx0 + (t % kw) * tdx)
    int kw = 1;
    while (kw < s0.ntaps && s0.dy[kw] == s0.dy[0]) ++kw;
    if (s0.ntaps % kw != 0) return WC_E_SHAPE;
    const int kh = s0.ntaps / kw;
    const int tdx = kw > 1 ? s0.dx[1] - s0.dx[0] : 0;
    const int tdy = kh > 1 ? s0.dy[kw] - s0.dy[0] : 0;
    for (int t = 0; t < s0.ntaps; ++t)
        if (s0.dy[t] != s0.dy[0] + (t / kw) * tdy || s0.dx[t] != s0.dx[0] + (t % kw) * tdx) return WC_E_SHAPE;
    d.src0 = s0.src; d.C0 = s0.C; d.ldc0 = s0.ldc; d.H0 = s0.H; d.W0 = s0.W; d.sy = s0.sy; d.sx = s0.sx;
    d.kh = kh; d.kw = kw; d.ty0 = s0.dy[0]; d.tdy = tdy; d.tx0 = s0.dx[0]; d.tdx = tdx;
    d.scale = s0.scale; d.shift = s0.shift;
    long k = (long)s0.ntaps * s0.C;
    if (a->nseg == 2) {
        // the fused residual: raw 1x1 read of a view with the same spatial grid as segment 0
        const wc_conv_seg& s1 = a->seg[1];
        if (!s1.src || s1.scale) return WC_E_ARG;
        if (s1.C <= 0 || s1.C % BK != 0 || s1.ldc % 4 != 0) return WC_E_SHAPE;
        if ((reinterpret_cast<uintptr_t>(s1.src) & 15) != 0) return WC_E_SHAPE;
        if (s1.ntaps != 1 || s1.dy[0] != 0 || s1.dx[0] != 0) return WC_E_SHAPE;
        if (s1.H != s0.H || s1.W != s0.W || s1.sy != s0.sy || s1.sx != s0.sx) return WC_E_SHAPE;
        if (s1.kbase != k) return WC_E_SHAPE;
        if ((long)a->B * s1.H * s1.W * s1.ldc * 4 >= (1L << 31)) return WC_E_SHAPE;
        d.src1 = s1.src; d.C1 = s1.C; d.ldc1 = s1.ldc; d.kbase1 = s1.kbase;
        k += s1.C;
    }
    if (k > a->ldw) return WC_E_SHAPE;
    if (a->ldw % 4 != 0 || (reinterpret_cast<uintptr_t>(a->w) & 15) != 0) return WC_E_SHAPE;
    if ((long)a->N * a->ldw * 4 >= (1L << 31)) return WC_E_SHAPE;
    d.B = a->B; d.Hm = a->Hm; d.Wm = a->Wm; d.N = a->N;
    long M = (long)a->B * a->Hm * a->Wm;
    if (M <= 0 || M > (1L << 30) || a->N <= 0) return WC_E_SHAPE;
    d.M = (int)M;
    d.w = a->w; d.ldw = a->ldw; d.bias = a->bias; d.temb = a->temb; d.temb_ld = a->temb_ld;
    d.res = a->res; d.ldres = a->ldres; d.out = a->out; d.ldo = a->ldo;
    d.Ho = a->Ho; d.Wo = a->Wo; d.osy = a->osy; d.osx = a->osx; d.ooy = a->ooy; d.oox = a->oox;
    d.out_nchw = a->out_nchw;
    if (a->act < WC_ACT_NONE || a->act > WC_ACT_TANH01) return WC_E_ARG;
    if (a->act == WC_ACT_PRELU && !a->act_param) return WC_E_ARG;
    d.act_param = a->act_param;
    d.ident = !a->out_nchw && a->osy == 1 && a->osx == 1 && a->ooy == 0 && a->oox == 0 &&
              a->Ho == a->Hm && a->Wo == a->Wm;
    d.steps0 = (int)((long)s0.ntaps * s0.C / BK);
    d.steps = (int)(k / BK);
    const int pro = s0.scale ? (s0.silu ? 2 : 1) : 0;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    // 64-column outputs (C_out = 64 stages, the 3-channel head) use a 256x64 tile.
    if (a->N <= 64) return dispatch<256, 64>(d, pro, a->act, s);
    return dispatch<128, 128>(d, pro, a->act, s);
}
