// Flash-style self-attention on fp32 MFMA for gfx950 (replaces the softmax(QK^T*scale)V core of
// nn.MultiheadAttention(C, 4, batch_first=True), reference unet_base.py:115,159).
//
// Workgroup = 4 waves = 128 query rows of one (batch, head); each wave owns 32 query rows.
// K/V tiles of 32 keys are staged through LDS and shared by the 4 waves.  Per tile and wave:
//   S^T = K Q^T       D/2 x v_mfma_f32_32x32x2_f32 (A = K rows from LDS via ds_read_b128,
//                     B = Q^T from registers/LDS).  The accumulator holds key rows x query columns,
//                     so every lane owns ONE query: the online-softmax row max / row sum are
//                     in-lane over 16 registers plus one lane^32 exchange.
//   O^T += V^T P^T    16 x (Dp/32) MFMAs; the S^T accumulator register r IS the B operand of
//                     k-substep r (key order permuted identically on the V side), so P never
//                     leaves registers, and O^T's column is again the lane's query, so the
//                     softmax rescale is a per-lane multiply.
// The N x N score matrix is never materialised; everything is exact f32 arithmetic with the
// softmax in the exp2 domain.
#include "wc_common.hpp"

namespace {

constexpr int ATT_THREADS = 256;
constexpr int KT = 32;  // keys per tile

template <int D>
struct AttCfg {
    static constexpr int DH = D / 2;                 // d-values per lane half in QK^T
    static constexpr int DP = (D + 31) / 32 * 32;    // padded head dim for PV blocks
    static constexpr int NDB = DP / 32;              // PV 32-wide blocks
    static constexpr int KS = D + 4;                 // K row stride (floats), odd # of 16B slots
    static constexpr bool QREG = D <= 128;           // Q kept in registers
    static constexpr int QS = D + 4;                 // Q row stride in LDS when !QREG
};

template <int D>
__global__ __launch_bounds__(ATT_THREADS, 1) void attention_kernel(const float* __restrict__ qkv,
                                                                   int ldq, float* __restrict__ out,
                                                                   int ldo, int N, int C,
                                                                   float scale_log2, float* __restrict__ lse) {
    using Cf = AttCfg<D>;
    extern __shared__ __attribute__((aligned(16))) float smem[];
    float* Ks = smem;                       // [KT][KS]
    float* Vs = Ks + KT * Cf::KS;           // [KT][DP]
    float* Qs = Vs + KT * Cf::DP;           // [128][QS] (only when !QREG)

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;
    const int l32 = lane & 31;
    const int half = lane >> 5;
    const int head = blockIdx.y;
    const int b = blockIdx.z;
    const int q0 = blockIdx.x * 128 + wave * 32;
    const float* base = qkv + (long)b * N * ldq;
    const int qcol = head * D;
    const int kcol = C + head * D;
    const int vcol = 2 * C + head * D;

    // zero the V pad columns once (D = 16 only)
    if (Cf::DP != D) {
        for (int i = tid; i < KT * Cf::DP; i += ATT_THREADS) {
            int c = i % Cf::DP;
            if (c >= D) Vs[i] = 0.f;
        }
    }

    // ---- Q fragment: lane (q = l32, half) needs Q[q][half*DH + i], i < DH ----
    float qreg[Cf::QREG ? Cf::DH : 1];
    const int qrow = q0 + l32;
    if constexpr (Cf::QREG) {
#pragma unroll
        for (int i = 0; i < Cf::DH; i += 4) {
            f32x4 v = f32x4{0.f, 0.f, 0.f, 0.f};
            if (qrow < N) v = *reinterpret_cast<const f32x4*>(base + (long)qrow * ldq + qcol + half * Cf::DH + i);
            qreg[i] = v.x; qreg[i + 1] = v.y; qreg[i + 2] = v.z; qreg[i + 3] = v.w;
        }
    } else {
        for (int i = tid; i < 128 * (D / 4); i += ATT_THREADS) {
            int r = i / (D / 4), c4 = i % (D / 4);
            int qr = blockIdx.x * 128 + r;
            f32x4 v = f32x4{0.f, 0.f, 0.f, 0.f};
            if (qr < N) v = *reinterpret_cast<const f32x4*>(base + (long)qr * ldq + qcol + c4 * 4);
            *reinterpret_cast<f32x4*>(Qs + r * Cf::QS + c4 * 4) = v;
        }
    }

    f32x16 o[Cf::NDB];
#pragma unroll
    for (int d = 0; d < Cf::NDB; ++d)
#pragma unroll
        for (int r = 0; r < 16; ++r) o[d][r] = 0.f;
    float m_run = -INFINITY, l_run = 0.f;

    const int ntiles = (N + KT - 1) / KT;
    for (int t = 0; t < ntiles; ++t) {
        const int kv0 = t * KT;
        __syncthreads();  // previous tile fully consumed (and Q/V-pad staged on t == 0)
        // stage K and V tile: 32 rows x D floats each
        for (int i = tid; i < KT * (D / 4); i += ATT_THREADS) {
            int r = i / (D / 4), c4 = i % (D / 4);
            int key = kv0 + r;
            f32x4 kv = f32x4{0.f, 0.f, 0.f, 0.f}, vv = kv;
            if (key < N) {
                const float* row = base + (long)key * ldq;
                kv = *reinterpret_cast<const f32x4*>(row + kcol + c4 * 4);
                vv = *reinterpret_cast<const f32x4*>(row + vcol + c4 * 4);
            }
            *reinterpret_cast<f32x4*>(Ks + r * Cf::KS + c4 * 4) = kv;
            *reinterpret_cast<f32x4*>(Vs + r * Cf::DP + c4 * 4) = vv;
        }
        __syncthreads();

        // ---- S^T = K Q^T ----
        f32x16 s;
#pragma unroll
        for (int r = 0; r < 16; ++r) s[r] = 0.f;
        const float* krow = Ks + l32 * Cf::KS + half * Cf::DH;
        const float* qrowp = Qs + (wave * 32 + l32) * Cf::QS + half * Cf::DH;
#pragma unroll
        for (int i = 0; i < Cf::DH; i += 4) {
            f32x4 a = *reinterpret_cast<const f32x4*>(krow + i);
            f32x4 qb;
            if constexpr (Cf::QREG) {
                qb = f32x4{qreg[i], qreg[i + 1], qreg[i + 2], qreg[i + 3]};
            } else {
                qb = *reinterpret_cast<const f32x4*>(qrowp + i);
            }
            s = mfma32(a.x, qb.x, s);
            s = mfma32(a.y, qb.y, s);
            s = mfma32(a.z, qb.z, s);
            s = mfma32(a.w, qb.w, s);
        }

        // ---- online softmax over keys (rows), per query (lane) ----
        float mloc = -INFINITY;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int key = kv0 + (r & 3) + 8 * (r >> 2) + 4 * half;
            float v = (key < N) ? s[r] * scale_log2 : -INFINITY;
            s[r] = v;
            mloc = fmaxf(mloc, v);
        }
        mloc = fmaxf(mloc, __shfl_xor(mloc, 32, 64));
        const float m_new = fmaxf(m_run, mloc);
        const float alpha = exp2f(m_run - m_new);
        float lsum = 0.f;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            float pv = exp2f(s[r] - m_new);
            s[r] = pv;
            lsum += pv;
        }
        lsum += __shfl_xor(lsum, 32, 64);
        l_run = l_run * alpha + lsum;
        m_run = m_new;
#pragma unroll
        for (int d = 0; d < Cf::NDB; ++d)
#pragma unroll
            for (int r = 0; r < 16; ++r) o[d][r] *= alpha;

        // ---- O^T += V^T P^T ----
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int key = (r & 3) + 8 * (r >> 2) + 4 * half;
            const float* vrow = Vs + key * Cf::DP + l32;
#pragma unroll
            for (int d = 0; d < Cf::NDB; ++d) o[d] = mfma32(vrow[d * 32], s[r], o[d]);
        }
    }

    // ---- epilogue: O[q][dv] = O^T[dv][q] / l ----
    if (qrow < N) {
        const float inv = 1.0f / l_run;
        // log2-domain log-sum-exp of the scaled scores (training backward): P = exp2(s*scale_log2 - lse)
        if (lse && half == 0) lse[((long)b * gridDim.y + head) * N + qrow] = m_run + __log2f(l_run);
        float* orow = out + ((long)b * N + qrow) * ldo + head * D;
#pragma unroll
        for (int d = 0; d < Cf::NDB; ++d) {
#pragma unroll
            for (int r = 0; r < 16; r += 4) {
                const int dv = d * 32 + 8 * (r >> 2) + 4 * half;
                if (dv < D) {
                    f32x4 v = f32x4{o[d][r] * inv, o[d][r + 1] * inv, o[d][r + 2] * inv, o[d][r + 3] * inv};
                    *reinterpret_cast<f32x4*>(orow + dv) = v;
                }
            }
        }
    }
}

template <int D>
int launch_att(const float* qkv, int ldq, float* out, int ldo, int B, int N, int C, int heads,
               float scale, hipStream_t stream, float* lse = nullptr) {
    using Cf = AttCfg<D>;
    size_t lds = (size_t)(KT * Cf::KS + KT * Cf::DP) * sizeof(float);
    if (!Cf::QREG) lds += (size_t)128 * Cf::QS * sizeof(float);
    static bool attr_set = false;  // >64 KiB dynamic LDS (D = 192 keeps Q in LDS): opt in once
    if (!attr_set && lds > 64 * 1024) {
        hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&attention_kernel<D>),
                                           hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (e != hipSuccess) return (int)e;
        attr_set = true;
    }
    dim3 grid((N + 127) / 128, heads, B);
    const float scale_log2 = scale * 1.4426950408889634f;
    hipLaunchKernelGGL(attention_kernel<D>, grid, dim3(ATT_THREADS), lds, stream, qkv, ldq, out,
                       ldo, N, C, scale_log2, lse);
    WC_CHECK_LAUNCH();
    return WC_OK;
}

}  // namespace

static int attention_fwd_any(const float* qkv, int ld_qkv, float* out, int ld_out, int B, int N, int C, int heads,
                             float scale, void* stream, float* lse) {
    if (!qkv || !out) return WC_E_ARG;
    if (heads <= 0 || C % heads != 0 || ld_qkv % 4 != 0 || ld_out % 4 != 0) return WC_E_SHAPE;
    if (ld_qkv < 3 * C || ld_out < C) return WC_E_SHAPE;
    const int D = C / heads;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    switch (D) {
        case 8: return launch_att<8>(qkv, ld_qkv, out, ld_out, B, N, C, heads, scale, s, lse);
        case 16: return launch_att<16>(qkv, ld_qkv, out, ld_out, B, N, C, heads, scale, s, lse);
        case 24: return launch_att<24>(qkv, ld_qkv, out, ld_out, B, N, C, heads, scale, s, lse);
        case 48: return launch_att<48>(qkv, ld_qkv, out, ld_out, B, N, C, heads, scale, s, lse);
        case 96: return launch_att<96>(qkv, ld_qkv, out, ld_out, B, N, C, heads, scale, s, lse);
        case 160: return launch_att<160>(qkv, ld_qkv, out, ld_out, B, N, C, heads, scale, s, lse);
        case 32: return launch_att<32>(qkv, ld_qkv, out, ld_out, B, N, C, heads, scale, s, lse);
        case 64: return launch_att<64>(qkv, ld_qkv, out, ld_out, B, N, C, heads, scale, s, lse);
        case 128: return launch_att<128>(qkv, ld_qkv, out, ld_out, B, N, C, heads, scale, s, lse);
        case 192: return launch_att<192>(qkv, ld_qkv, out, ld_out, B, N, C, heads, scale, s, lse);
        default: return WC_E_SHAPE;
    }
}

extern "C" int wc_attention_fwd(const float* qkv, int ld_qkv, float* out, int ld_out, int B,
                                int N, int C, int heads, float scale, void* stream) {
    return attention_fwd_any(qkv, ld_qkv, out, ld_out, B, N, C, heads, scale, stream, nullptr);
}

extern "C" int wc_attention_fwd_lse(const float* qkv, int ld_qkv, float* out, int ld_out, float* lse, int B, int N,
                                    int C, int heads, float scale, void* stream) {
    if (!lse) return WC_E_ARG;
    return attention_fwd_any(qkv, ld_qkv, out, ld_out, B, N, C, heads, scale, stream, lse);
}
