// Self-attention backward on fp32 MFMA for gfx950 (the training backward of the softmax(QK^T*s)V
// core of nn.MultiheadAttention, reference unet_base.py:115,159; train_ddpm.py:110 loss.backward()).
//
// Forward contract (wc_attention_fwd_lse): lse[b][h][q] = log2 sum_k exp2(s_qk * scale*log2(e)), so
// P_qk = exp2(s_qk*scale_log2 - lse_q) is recomputed exactly without storing the N x N scores.
// With Dv_q = sum_d dO_qd O_qd (attn_bwd_prep_kernel):
//     dS = P o (dP - Dv),  dP = dO V^T,  dV = P^T dO,  dK = scale dS^T Q,  dQ = scale dS K.
// Two kernels, no atomics (deterministic):
//   attn_bwd_dkdv_kernel  a wave owns 32 keys; loops over 32-query tiles (Q, dO, lse, Dv staged in
//       LDS): S = Q K^T and dP = dO V^T with keys on the lanes (the accumulator register r holds
//       query (r&3)+8(r>>2)+4*half), so P and dS are directly the B operand of
//       dV^T += dO^T P and dK^T += Q^T dS (the forward kernel's register-reuse trick, transposed).
//   attn_bwd_dq_kernel    a wave owns 32 queries; loops over 32-key tiles: S^T = K Q^T and
//       dP^T = V dO^T with queries on the lanes, dS^T feeds dQ^T += K^T dS^T.
// The wave's own rows (K, V for dK/dV; Q, dO for dQ) stay in registers for the whole loop and the
// other side's 32-row tiles go through LDS, shared by the workgroup's 4 waves (one per SIMD); exact
// fp32 products.
#include "wc_common.hpp"

namespace {

template <int D>
struct BwdCfg {
    static constexpr int DH = D / 2;                // d-values per lane half in the QK^T / dO V^T loops
    static constexpr int DP = (D + 31) / 32 * 32;   // padded head dim of the d-row accumulators
    static constexpr int NDB = DP / 32;
    static constexpr int RS = D + 4;                // LDS row stride (floats)
    static constexpr int W = 4;                     // waves per workgroup (one per SIMD)
    static constexpr int SLACK = 32;                // reads of pad columns d >= D stay inside LDS
    static constexpr int LDS_FLOATS = 2 * 32 * RS + SLACK + 64;
};

// A wave owns 32 keys: its K and V rows stay in registers (lane = key, the half's d range), the
// 32-query tiles of Q and dO go through LDS, shared by the workgroup's 4 waves.
template <int D>
__global__ __launch_bounds__(256, 1) void attn_bwd_dkdv_kernel(
    const float* __restrict__ qkv, int ldq, const float* __restrict__ dO, int lddo, const float* __restrict__ lse,
    const float* __restrict__ Dv, float* __restrict__ dqkv, int lddq, int N, int C, float scale_log2, float scale) {
    using Cf = BwdCfg<D>;
    constexpr int RS = Cf::RS, NT = 256;
    extern __shared__ __attribute__((aligned(16))) float smem[];
    float* Qs = smem;                     // [32][RS] query tile
    float* Os = Qs + 32 * RS;             // [32][RS] dO tile
    float* Ls = Os + 32 * RS + Cf::SLACK; // [32] lse, then [32] Dv

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int l32 = lane & 31, half = lane >> 5;
    const int head = blockIdx.y, b = blockIdx.z, H = gridDim.y;
    const float* base = qkv + (long)b * N * ldq;
    const float* dob = dO + (long)b * N * lddo;
    const int qcol = head * D, kcol = C + head * D, vcol = 2 * C + head * D;
    const int key = blockIdx.x * 128 + wave * 32 + l32;

    float kreg[Cf::DH], vreg[Cf::DH];
#pragma unroll
    for (int i = 0; i < Cf::DH; i += 4) {
        f32x4 kv = f32x4{0.f, 0.f, 0.f, 0.f}, vv = kv;
        if (key < N) {
            kv = *reinterpret_cast<const f32x4*>(base + (long)key * ldq + kcol + half * Cf::DH + i);
            vv = *reinterpret_cast<const f32x4*>(base + (long)key * ldq + vcol + half * Cf::DH + i);
        }
        kreg[i] = kv.x; kreg[i + 1] = kv.y; kreg[i + 2] = kv.z; kreg[i + 3] = kv.w;
        vreg[i] = vv.x; vreg[i + 1] = vv.y; vreg[i + 2] = vv.z; vreg[i + 3] = vv.w;
    }

    f32x16 dvT[Cf::NDB], dkT[Cf::NDB];
#pragma unroll
    for (int d = 0; d < Cf::NDB; ++d)
#pragma unroll
        for (int r = 0; r < 16; ++r) { dvT[d][r] = 0.f; dkT[d][r] = 0.f; }

    const int ntiles = (N + 31) / 32;
    for (int t = 0; t < ntiles; ++t) {
        const int q0 = t * 32;
        __syncthreads();  // previous tile consumed
        for (int i = tid; i < 32 * (D / 4); i += NT) {
            const int r = i / (D / 4), c4 = i % (D / 4);
            const int q = q0 + r;
            f32x4 qv = f32x4{0.f, 0.f, 0.f, 0.f}, ov = qv;
            if (q < N) {
                qv = *reinterpret_cast<const f32x4*>(base + (long)q * ldq + qcol + c4 * 4);
                ov = *reinterpret_cast<const f32x4*>(dob + (long)q * lddo + head * D + c4 * 4);
            }
            *reinterpret_cast<f32x4*>(Qs + r * RS + c4 * 4) = qv;
            *reinterpret_cast<f32x4*>(Os + r * RS + c4 * 4) = ov;
        }
        if (tid < 32) {
            const int q = q0 + tid;
            Ls[tid] = q < N ? lse[((long)b * H + head) * N + q] : INFINITY;  // P = 0 for padding queries
            Ls[32 + tid] = q < N ? Dv[((long)b * H + head) * N + q] : 0.f;
        }
        __syncthreads();

        // S = Q K^T, dP = dO V^T: rows = queries, lane = key
        f32x16 s, dp;
#pragma unroll
        for (int r = 0; r < 16; ++r) { s[r] = 0.f; dp[r] = 0.f; }
        const float* qr = Qs + l32 * RS + half * Cf::DH;
        const float* orw = Os + l32 * RS + half * Cf::DH;
#pragma unroll
        for (int i = 0; i < Cf::DH; i += 4) {
            const f32x4 a = *reinterpret_cast<const f32x4*>(qr + i);
            const f32x4 a2 = *reinterpret_cast<const f32x4*>(orw + i);
            s = mfma32(a.x, kreg[i], s); s = mfma32(a.y, kreg[i + 1], s);
            s = mfma32(a.z, kreg[i + 2], s); s = mfma32(a.w, kreg[i + 3], s);
            dp = mfma32(a2.x, vreg[i], dp); dp = mfma32(a2.y, vreg[i + 1], dp);
            dp = mfma32(a2.z, vreg[i + 2], dp); dp = mfma32(a2.w, vreg[i + 3], dp);
        }
        // P and dS in place (register r <-> query row (r&3) + 8(r>>2) + 4 half of the tile)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int qi = (r & 3) + 8 * (r >> 2) + 4 * half;
            const float pr = exp2f(s[r] * scale_log2 - Ls[qi]);
            s[r] = pr;
            dp[r] = pr * (dp[r] - Ls[32 + qi]);
        }
        // dV^T += dO^T P, dK^T += Q^T dS
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int qi = (r & 3) + 8 * (r >> 2) + 4 * half;
            const float* op = Os + qi * RS + l32;
            const float* qp = Qs + qi * RS + l32;
#pragma unroll
            for (int d = 0; d < Cf::NDB; ++d) {
                dvT[d] = mfma32(op[d * 32], s[r], dvT[d]);
                dkT[d] = mfma32(qp[d * 32], dp[r], dkT[d]);
            }
        }
    }

    if (key < N) {
        float* row = dqkv + ((long)b * N + key) * lddq;
#pragma unroll
        for (int d = 0; d < Cf::NDB; ++d) {
#pragma unroll
            for (int r = 0; r < 16; r += 4) {
                const int dv = d * 32 + 8 * (r >> 2) + 4 * half;
                if (dv < D) {
                    *reinterpret_cast<f32x4*>(row + kcol + dv) =
                        f32x4{dkT[d][r], dkT[d][r + 1], dkT[d][r + 2], dkT[d][r + 3]} * scale;
                    *reinterpret_cast<f32x4*>(row + vcol + dv) = f32x4{dvT[d][r], dvT[d][r + 1], dvT[d][r + 2], dvT[d][r + 3]};
                }
            }
        }
    }
}

// A wave owns 32 queries: Q and dO rows in registers, 32-key tiles of K and V through LDS.
template <int D>
__global__ __launch_bounds__(256, 1) void attn_bwd_dq_kernel(
    const float* __restrict__ qkv, int ldq, const float* __restrict__ dO, int lddo, const float* __restrict__ lse,
    const float* __restrict__ Dv, float* __restrict__ dqkv, int lddq, int N, int C, float scale_log2, float scale) {
    using Cf = BwdCfg<D>;
    constexpr int RS = Cf::RS, NT = 256;
    extern __shared__ __attribute__((aligned(16))) float smem[];
    float* Ks = smem;             // [32][RS] key tile
    float* Vs = Ks + 32 * RS;     // [32][RS]

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int l32 = lane & 31, half = lane >> 5;
    const int head = blockIdx.y, b = blockIdx.z, H = gridDim.y;
    const float* base = qkv + (long)b * N * ldq;
    const float* dob = dO + (long)b * N * lddo;
    const int qcol = head * D, kcol = C + head * D, vcol = 2 * C + head * D;
    const int qme = blockIdx.x * 128 + wave * 32 + l32;

    float qreg[Cf::DH], oreg[Cf::DH];
#pragma unroll
    for (int i = 0; i < Cf::DH; i += 4) {
        f32x4 qv = f32x4{0.f, 0.f, 0.f, 0.f}, ov = qv;
        if (qme < N) {
            qv = *reinterpret_cast<const f32x4*>(base + (long)qme * ldq + qcol + half * Cf::DH + i);
            ov = *reinterpret_cast<const f32x4*>(dob + (long)qme * lddo + head * D + half * Cf::DH + i);
        }
        qreg[i] = qv.x; qreg[i + 1] = qv.y; qreg[i + 2] = qv.z; qreg[i + 3] = qv.w;
        oreg[i] = ov.x; oreg[i + 1] = ov.y; oreg[i + 2] = ov.z; oreg[i + 3] = ov.w;
    }
    const float lq = qme < N ? lse[((long)b * H + head) * N + qme] : INFINITY;
    const float dq = qme < N ? Dv[((long)b * H + head) * N + qme] : 0.f;

    f32x16 dqT[Cf::NDB];
#pragma unroll
    for (int d = 0; d < Cf::NDB; ++d)
#pragma unroll
        for (int r = 0; r < 16; ++r) dqT[d][r] = 0.f;

    const int ntiles = (N + 31) / 32;
    for (int t = 0; t < ntiles; ++t) {
        const int k0 = t * 32;
        __syncthreads();
        for (int i = tid; i < 32 * (D / 4); i += NT) {
            const int r = i / (D / 4), c4 = i % (D / 4);
            const int key = k0 + r;
            f32x4 kv = f32x4{0.f, 0.f, 0.f, 0.f}, vv = kv;
            if (key < N) {
                kv = *reinterpret_cast<const f32x4*>(base + (long)key * ldq + kcol + c4 * 4);
                vv = *reinterpret_cast<const f32x4*>(base + (long)key * ldq + vcol + c4 * 4);
            }
            *reinterpret_cast<f32x4*>(Ks + r * RS + c4 * 4) = kv;
            *reinterpret_cast<f32x4*>(Vs + r * RS + c4 * 4) = vv;
        }
        __syncthreads();

        // S^T = K Q^T, dP^T = V dO^T: rows = keys, lane = query
        f32x16 s, dp;
#pragma unroll
        for (int r = 0; r < 16; ++r) { s[r] = 0.f; dp[r] = 0.f; }
        const float* kr = Ks + l32 * RS + half * Cf::DH;
        const float* vr = Vs + l32 * RS + half * Cf::DH;
#pragma unroll
        for (int i = 0; i < Cf::DH; i += 4) {
            const f32x4 a = *reinterpret_cast<const f32x4*>(kr + i);
            const f32x4 a2 = *reinterpret_cast<const f32x4*>(vr + i);
            s = mfma32(a.x, qreg[i], s); s = mfma32(a.y, qreg[i + 1], s);
            s = mfma32(a.z, qreg[i + 2], s); s = mfma32(a.w, qreg[i + 3], s);
            dp = mfma32(a2.x, oreg[i], dp); dp = mfma32(a2.y, oreg[i + 1], dp);
            dp = mfma32(a2.z, oreg[i + 2], dp); dp = mfma32(a2.w, oreg[i + 3], dp);
        }
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int key = k0 + (r & 3) + 8 * (r >> 2) + 4 * half;
            const float pr = key < N ? exp2f(s[r] * scale_log2 - lq) : 0.f;
            dp[r] = pr * (dp[r] - dq);
        }
        // dQ^T += K^T dS^T
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int ki = (r & 3) + 8 * (r >> 2) + 4 * half;
            const float* kp = Ks + ki * RS + l32;
#pragma unroll
            for (int d = 0; d < Cf::NDB; ++d) dqT[d] = mfma32(kp[d * 32], dp[r], dqT[d]);
        }
    }

    if (qme < N) {
        float* row = dqkv + ((long)b * N + qme) * lddq + qcol;
#pragma unroll
        for (int d = 0; d < Cf::NDB; ++d) {
#pragma unroll
            for (int r = 0; r < 16; r += 4) {
                const int dv = d * 32 + 8 * (r >> 2) + 4 * half;
                if (dv < D)
                    *reinterpret_cast<f32x4*>(row + dv) = f32x4{dqT[d][r], dqT[d][r + 1], dqT[d][r + 2], dqT[d][r + 3]} * scale;
            }
        }
    }
}

// Dv[b][h][q] = sum_d dO[b, q, h*D + d] * O[b, q, h*D + d].  16 lanes per (b, q, h) row, rows in
// memory order (b, q, h): a wave reads four heads' rows of one pixel, consecutive 16-byte pieces across
// the lanes (a thread per row striding through its own row touched 64 cache lines per load); each lane
// sums d = 4 l + 64 k in order, then a fixed xor butterfly over the 16 lanes (deterministic).
__global__ __launch_bounds__(256) void attn_bwd_prep_kernel(const float* __restrict__ O, int ldo,
                                                            const float* __restrict__ dO, int lddo, int B, int N,
                                                            int H, int D, float* __restrict__ Dv) {
    const long r = (long)blockIdx.x * 16 + (threadIdx.x >> 4);
    const int l = threadIdx.x & 15;
    const bool live = r < (long)B * N * H;
    const long rr = live ? r : 0;
    const int h = (int)(rr % H);
    const long bq = rr / H;
    const float* o = O + bq * ldo + h * D;
    const float* g = dO + bq * lddo + h * D;
    float s = 0.f;
    if (live)
        for (int d = 4 * l; d < D; d += 64) {
            const f32x4 a = *reinterpret_cast<const f32x4*>(o + d);
            const f32x4 c = *reinterpret_cast<const f32x4*>(g + d);
            s = fmaf(a.x, c.x, s); s = fmaf(a.y, c.y, s); s = fmaf(a.z, c.z, s); s = fmaf(a.w, c.w, s);
        }
#pragma unroll
    for (int m = 8; m > 0; m >>= 1) s += __shfl_xor(s, m, 16);
    if (live && l == 0) {
        const int q = (int)(bq % N);
        const int b = (int)(bq / N);
        Dv[((long)b * H + h) * N + q] = s;
    }
}

template <int D>
int launch_bwd(const float* qkv, int ldq, const float* dO, int lddo, const float* lse, const float* Dv, float* dqkv,
               int lddq, int B, int N, int C, int heads, float scale, hipStream_t s, int parts = 3) {
    using Cf = BwdCfg<D>;
    const size_t lds = (size_t)Cf::LDS_FLOATS * sizeof(float);
    static bool attr_set = false;
    if (!attr_set && lds > 64 * 1024) {
        hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&attn_bwd_dkdv_kernel<D>),
                                           hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (e != hipSuccess) return (int)e;
        e = hipFuncSetAttribute(reinterpret_cast<const void*>(&attn_bwd_dq_kernel<D>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (e != hipSuccess) return (int)e;
        attr_set = true;
    }
    const dim3 grid((N + 127) / 128, heads, B);
    const float scale_log2 = scale * 1.4426950408889634f;
    if (parts & 1) {
        WC_SET_NAME("attn_bwd_dkdv_kernel", {WC_TI(D)});
        hipLaunchKernelGGL(attn_bwd_dkdv_kernel<D>, grid, dim3(256), lds, s, qkv, ldq, dO, lddo, lse, Dv, dqkv, lddq, N,
                           C, scale_log2, scale);
        WC_CHECK_LAUNCH();
    }
    if (parts & 2) {
        WC_SET_NAME("attn_bwd_dq_kernel", {WC_TI(D)});
        hipLaunchKernelGGL(attn_bwd_dq_kernel<D>, grid, dim3(256), lds, s, qkv, ldq, dO, lddo, lse, Dv, dqkv, lddq, N,
                           C, scale_log2, scale);
        WC_CHECK_LAUNCH();
    }
    return WC_OK;
}

}  // namespace

extern "C" int wc_attention_bwd(const float* qkv, int ld_qkv, const float* out, int ld_out, const float* dout,
                                int ld_dout, const float* lse, float* dv_work, float* dqkv, int ld_dqkv, int B, int N,
                                int C, int heads, float scale, void* stream) {
    if (!qkv || !out || !dout || !lse || !dv_work || !dqkv) return WC_E_ARG;
    if (heads <= 0 || C % heads || B <= 0 || N <= 0) return WC_E_SHAPE;
    if (ld_qkv % 4 || ld_out % 4 || ld_dout % 4 || ld_dqkv % 4 || ld_qkv < 3 * C || ld_dqkv < 3 * C || ld_out < C ||
        ld_dout < C)
        return WC_E_SHAPE;
    const int D = C / heads;
    if (D % 4) return WC_E_SHAPE;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    const long n = (long)B * heads * N;
    hipLaunchKernelGGL(attn_bwd_prep_kernel, dim3((unsigned)((n + 15) / 16)), dim3(256), 0, s, out, ld_out, dout,
                       ld_dout, B, N, heads, D, dv_work);
    WC_CHECK_LAUNCH();
    switch (D) {
        case 8: return launch_bwd<8>(qkv, ld_qkv, dout, ld_dout, lse, dv_work, dqkv, ld_dqkv, B, N, C, heads, scale, s);
        case 16: return launch_bwd<16>(qkv, ld_qkv, dout, ld_dout, lse, dv_work, dqkv, ld_dqkv, B, N, C, heads, scale, s);
        case 32: return launch_bwd<32>(qkv, ld_qkv, dout, ld_dout, lse, dv_work, dqkv, ld_dqkv, B, N, C, heads, scale, s);
        case 64: return launch_bwd<64>(qkv, ld_qkv, dout, ld_dout, lse, dv_work, dqkv, ld_dqkv, B, N, C, heads, scale, s);
        case 128:
            return launch_bwd<128>(qkv, ld_qkv, dout, ld_dout, lse, dv_work, dqkv, ld_dqkv, B, N, C, heads, scale, s);
        case 192:
            return launch_bwd<192>(qkv, ld_qkv, dout, ld_dout, lse, dv_work, dqkv, ld_dqkv, B, N, C, heads, scale, s);
        default: return WC_E_SHAPE;
    }
}

// Dv = rowsum(dO o O) per (image, head, query) only (the first step of the backward; used by the
// split-precision backward wc_attention_bwd6).
extern "C" int wc_attention_bwd_prep(const float* out, int ld_out, const float* dout, int ld_dout, int B, int N,
                                     int heads, int D, float* dv_work, void* stream) {
    if (!out || !dout || !dv_work) return WC_E_ARG;
    if (B <= 0 || N <= 0 || heads <= 0 || D <= 0 || D % 4 || ld_out % 4 || ld_dout % 4) return WC_E_SHAPE;
    const long n = (long)B * heads * N;
    hipLaunchKernelGGL(attn_bwd_prep_kernel, dim3((unsigned)((n + 15) / 16)), dim3(256), 0,
                       reinterpret_cast<hipStream_t>(stream), out, ld_out, dout, ld_dout, B, N, heads, D, dv_work);
    WC_CHECK_LAUNCH();
    return WC_OK;
}

// The fp32-MFMA dK / dV kernel alone at head dim 192, after wc_attention_bwd_prep (the f16x3 backward
// runs its dQ kernel beside it: wc_attention_bwd6.hip).
extern "C" int wc_attention_bwd_dkdv192(const float* qkv, int ld_qkv, const float* dout, int ld_dout, const float* lse,
                                        const float* dv_work, float* dqkv, int ld_dqkv, int B, int N, int C,
                                        int heads, float scale, void* stream) {
    if (!qkv || !dout || !lse || !dv_work || !dqkv) return WC_E_ARG;
    if (heads <= 0 || C != 192 * heads || B <= 0 || N <= 0) return WC_E_SHAPE;
    if (ld_qkv % 4 || ld_dout % 4 || ld_dqkv % 4 || ld_qkv < 3 * C || ld_dqkv < 3 * C || ld_dout < C) return WC_E_SHAPE;
    return launch_bwd<192>(qkv, ld_qkv, dout, ld_dout, lse, dv_work, dqkv, ld_dqkv, B, N, C, heads, scale,
                           reinterpret_cast<hipStream_t>(stream), 1);
}
