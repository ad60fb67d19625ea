// Implicit-GEMM convolution on fp32 MFMA for gfx950.
//
// GEMM view: M = B*Hm*Wm output positions (NHWC pixels), N = output channels, K = sum over
// segments of ntaps*C (tap-major, channel-minor; the packed weight is [N][K], K contiguous).
// One workgroup = 4 waves computing a BM x BN tile; each wave owns a 64x64 sub-tile made of 2x2
// v_mfma_f32_32x32x2_f32 accumulators (64 AGPR/VGPR per lane).  A K-step stages 32 input channels
// of one tap for BM pixels and the matching 32 K-rows of BN weights through LDS; the next step's
// global loads are issued before the current step's MFMAs (register staging, written to LDS after
// the barrier), so HBM/L2 latency hides under 64 MFMAs per wave.
//
// Fused work (reference unet_base.py ResBlock, :87-109 / :146-150):
//   prologue  (per segment)  v <- SiLU(v*scale[b,c] + shift[b,c])   [GroupNorm-apply + SiLU]
//                            zero padding is applied AFTER the prologue, as Conv2d pads the
//                            SiLU output
//   segment 2 (optional)     the 1x1 residual_input_conv appended as extra K columns
//   epilogue                 + bias[n] + temb[b,n] + residual view, NHWC or NCHW store
//
// LDS tiles are [rows][36] floats: a 144-byte row stride (9 16-byte slots) makes the
// ds_read_b128 fragment reads (16 lanes = 16 distinct rows, same column) conflict-free.
#include "wc_common.hpp"

namespace {

constexpr int BK = 32;        // channels per K-step
constexpr int LDS_STRIDE = 36;  // floats per LDS row
constexpr int NTHREADS = 256;

struct SegDev {
    const float* src;
    int C, ldc, H, W, sy, sx, ntaps, kbase;
    int dy[WC_MAX_TAPS];
    int dx[WC_MAX_TAPS];
    const float* scale;
    const float* shift;
    int silu;
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
    int steps0;   // K-steps of segment 0 (= ntaps * C / BK)
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
};

// Decode K-step -> (segment, tap, channel offset).
WC_DEVICE void decode_step(const ConvDev& p, int step, int& s, int& tap, int& c0) {
    if (step < p.steps0) {
        s = 0;
        int cpt = p.seg[0].C / BK;
        tap = step / cpt;
        c0 = (step - tap * cpt) * BK;
    } else {
        s = 1;
        int st = step - p.steps0;
        int cpt = p.seg[1].C / BK;
        tap = st / cpt;
        c0 = (st - tap * cpt) * BK;
    }
}

template <int BM, int BN>
__global__ __launch_bounds__(NTHREADS, 2) void conv_igemm_kernel(ConvDev p) {
    using T = Tile<BM, BN>;
    __shared__ __attribute__((aligned(16))) float lds[(BM + BN) * LDS_STRIDE];
    float* As = lds;
    float* Bs = lds + BM * LDS_STRIDE;

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;
    const int wm = wave / T::WAVES_N;
    const int wn = wave % T::WAVES_N;

    // XCD-aware tile order: consecutive logical tiles (which share A rows) on one XCD.
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

    // ---- per-thread staging coordinates ----
    const int q4 = tid & 7;      // float4 column within the 32-channel step
    const int prow = tid >> 3;   // 0..31
    const int HWm = p.Hm * p.Wm;
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
            pb[j] = -1; py[j] = 0; px[j] = 0;
        }
    }

    f32x4 ra[T::A_PER_T];
    f32x4 rb[T::B_PER_T];
    f32x4 rsc[T::A_PER_T], rsh[T::A_PER_T];
    bool aval[T::A_PER_T];

    auto load_step = [&](int step) {
        int s, tap, c0;
        decode_step(p, step, s, tap, c0);
        const SegDev& sg = p.seg[s];
        const int dy = sg.dy[tap], dx = sg.dx[tap];
        const int c = c0 + q4 * 4;
#pragma unroll
        for (int j = 0; j < T::A_PER_T; ++j) {
            int iy = py[j] * sg.sy + dy;
            int ix = px[j] * sg.sx + dx;
            bool ok = pb[j] >= 0 && iy >= 0 && iy < sg.H && ix >= 0 && ix < sg.W;
            aval[j] = ok;
            if (ok) {
                long off = ((long)(pb[j] * sg.H + iy) * sg.W + ix) * sg.ldc + c;
                ra[j] = *reinterpret_cast<const f32x4*>(sg.src + off);
                if (sg.scale) {
                    rsc[j] = *reinterpret_cast<const f32x4*>(sg.scale + pb[j] * sg.C + c);
                    rsh[j] = *reinterpret_cast<const f32x4*>(sg.shift + pb[j] * sg.C + c);
                }
            }
        }
        const int kcol = sg.kbase + tap * sg.C + c0 + q4 * 4;
#pragma unroll
        for (int j = 0; j < T::B_PER_T; ++j) {
            int n = n0 + prow + 32 * j;
            if (n < p.N)
                rb[j] = *reinterpret_cast<const f32x4*>(p.w + (long)n * p.ldw + kcol);
            else
                rb[j] = f32x4{0.f, 0.f, 0.f, 0.f};
        }
        return s;
    };

    auto store_step = [&](int s) {
        const SegDev& sg = p.seg[s];
#pragma unroll
        for (int j = 0; j < T::A_PER_T; ++j) {
            f32x4 v = ra[j];
            if (aval[j]) {
                if (sg.scale) {
                    v = v * rsc[j] + rsh[j];
                    if (sg.silu) {
                        v.x = wc_silu(v.x); v.y = wc_silu(v.y);
                        v.z = wc_silu(v.z); v.w = wc_silu(v.w);
                    }
                }
            } else {
                v = f32x4{0.f, 0.f, 0.f, 0.f};
            }
            *reinterpret_cast<f32x4*>(As + (prow + 32 * j) * LDS_STRIDE + q4 * 4) = v;
        }
#pragma unroll
        for (int j = 0; j < T::B_PER_T; ++j)
            *reinterpret_cast<f32x4*>(Bs + (prow + 32 * j) * LDS_STRIDE + q4 * 4) = rb[j];
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
    const float* a_base = As + (wm * 64 + l32) * LDS_STRIDE + half * 16;
    const float* b_base = Bs + (wn * 64 + l32) * LDS_STRIDE + half * 16;

    int s_cur = load_step(0);
    store_step(s_cur);
    __syncthreads();

    for (int step = 0; step < p.steps; ++step) {
        int s_next = 0;
        if (step + 1 < p.steps) s_next = load_step(step + 1);

#pragma unroll
        for (int kq = 0; kq < 4; ++kq) {
            f32x4 a0 = *reinterpret_cast<const f32x4*>(a_base + kq * 4);
            f32x4 a1 = *reinterpret_cast<const f32x4*>(a_base + 32 * LDS_STRIDE + kq * 4);
            f32x4 b0 = *reinterpret_cast<const f32x4*>(b_base + kq * 4);
            f32x4 b1 = *reinterpret_cast<const f32x4*>(b_base + 32 * LDS_STRIDE + kq * 4);
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                acc[0][0] = mfma32(a0[j], b0[j], acc[0][0]);
                acc[0][1] = mfma32(a0[j], b1[j], acc[0][1]);
                acc[1][0] = mfma32(a1[j], b0[j], acc[1][0]);
                acc[1][1] = mfma32(a1[j], b1[j], acc[1][1]);
            }
        }
        __syncthreads();
        if (step + 1 < p.steps) {
            store_step(s_next);
            __syncthreads();
        }
    }

    // ---- epilogue ----
    const int HWo = p.Ho * p.Wo;
#pragma unroll
    for (int nb = 0; nb < 2; ++nb) {
        const int n = n0 + wn * 64 + nb * 32 + l32;
        if (n >= p.N) continue;
        const float bn = p.bias ? p.bias[n] : 0.f;
#pragma unroll
        for (int mb = 0; mb < 2; ++mb) {
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int row = (r & 3) + 8 * (r >> 2) + 4 * half;
                const int m = m0 + wm * 64 + mb * 32 + row;
                if (m >= p.M) continue;
                const int b = m / HWm;
                const int rr = m - b * HWm;
                const int my = rr / p.Wm;
                const int mx = rr - my * p.Wm;
                const int oy = my * p.osy + p.ooy;
                const int ox = mx * p.osx + p.oox;
                float v = acc[mb][nb][r] + bn;
                if (p.temb) v += p.temb[b * p.temb_ld + n];
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

template <int BM, int BN>
int launch(const ConvDev& d, hipStream_t stream) {
    ConvDev p = d;
    int tiles_m = (p.M + BM - 1) / BM;
    p.ntiles_n = (p.N + BN - 1) / BN;
    dim3 grid(tiles_m * p.ntiles_n);
    hipLaunchKernelGGL((conv_igemm_kernel<BM, BN>), grid, dim3(NTHREADS), 0, stream, p);
    WC_CHECK_LAUNCH();
    return WC_OK;
}

}  // namespace

extern "C" int wc_conv_igemm(const wc_conv_args* a, void* stream) {
    if (!a || !a->w || !a->out) return WC_E_ARG;
    if (a->nseg < 1 || a->nseg > 2) return WC_E_ARG;
    ConvDev d{};
    int k = 0;
    for (int s = 0; s < a->nseg; ++s) {
        const wc_conv_seg& sg = a->seg[s];
        if (!sg.src) return WC_E_ARG;
        if (sg.C <= 0 || sg.C % BK != 0 || sg.ldc % 4 != 0) return WC_E_SHAPE;
        if (sg.ntaps < 1 || sg.ntaps > WC_MAX_TAPS) return WC_E_SHAPE;
        if ((reinterpret_cast<uintptr_t>(sg.src) & 15) != 0) return WC_E_SHAPE;
        if ((sg.scale == nullptr) != (sg.shift == nullptr)) return WC_E_ARG;
        SegDev& o = d.seg[s];
        o.src = sg.src; o.C = sg.C; o.ldc = sg.ldc; o.H = sg.H; o.W = sg.W;
        o.sy = sg.sy; o.sx = sg.sx; o.ntaps = sg.ntaps; o.kbase = sg.kbase;
        for (int t = 0; t < sg.ntaps; ++t) { o.dy[t] = sg.dy[t]; o.dx[t] = sg.dx[t]; }
        o.scale = sg.scale; o.shift = sg.shift; o.silu = sg.silu;
        if (sg.kbase + sg.ntaps * sg.C > a->ldw) return WC_E_SHAPE;
        k += sg.ntaps * sg.C;
    }
    if (a->ldw % 4 != 0 || (reinterpret_cast<uintptr_t>(a->w) & 15) != 0) return WC_E_SHAPE;
    d.nseg = a->nseg;
    d.B = a->B; d.Hm = a->Hm; d.Wm = a->Wm; d.N = a->N;
    long M = (long)a->B * a->Hm * a->Wm;
    if (M <= 0 || M > (1L << 30) || a->N <= 0) return WC_E_SHAPE;
    d.M = (int)M;
    d.w = a->w; d.ldw = a->ldw; d.bias = a->bias; d.temb = a->temb; d.temb_ld = a->temb_ld;
    d.res = a->res; d.ldres = a->ldres; d.out = a->out; d.ldo = a->ldo;
    d.Ho = a->Ho; d.Wo = a->Wo; d.osy = a->osy; d.osx = a->osx; d.ooy = a->ooy; d.oox = a->oox;
    d.out_nchw = a->out_nchw;
    d.steps0 = a->seg[0].ntaps * a->seg[0].C / BK;
    d.steps = k / BK;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    // 64-column outputs (C_out = 64 stages, the 3-channel head) use a 256x64 tile.
    if (a->N <= 64) return launch<256, 64>(d, s);
    return launch<128, 128>(d, s);
}
