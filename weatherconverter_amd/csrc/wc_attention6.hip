// Flash attention on split-precision MFMA for gfx950 (head dims D % 32 == 0).  Same contract as
// wc_attention_fwd (wc_attention.hip): softmax(Q K^T * scale) V per (batch, head), replacing the
// core of nn.MultiheadAttention(C, 4, batch_first=True) (unet_base.py:115,159).
//
// Arithmetic (fp32-class, fp32 accumulation):
//   bf16x6  every fp32 operand (Q, K, V and the probabilities P) split exactly into three bf16
//           pieces (wc_x6.hpp split3); six products per block on v_mfma_f32_32x32x16_bf16.
//   f16x3   Q, K, V scaled by caller-chosen powers of two 2^eq, 2^ek, 2^ev with |x| 2^e < 2^15
//           (static bounds from the in-projection and its GroupNorm, see kernels.py), P by 2^14,
//           each split into two round-to-nearest fp16 pieces; three products per block on
//           v_mfma_f32_32x32x16_f16.  The scales fold into the softmax multiplier and the final
//           1/l, so no extra arithmetic is spent on them.
//
// Structure:
//   * workgroup = 4 waves x 32 queries of one (batch, head); Q is split once into registers.
//   * K/V tiles of 32 keys, double-buffered in LDS: the next tile's global loads are issued before
//     the MFMAs of the current tile and split into the other buffer after them; one barrier/tile.
//   * S^T = K Q^T per 16 head dims.  The accumulator holds keys x queries, so each lane owns one
//     query and the online softmax is in-lane (+ one lane^32 exchange).
//   * O^T += V^T P^T: the S^T registers of a 16-key chunk ARE the lane's B operand (P^T), split in
//     registers; V is staged transposed ([piece][dim][32 keys]) in the matching key permutation
//     (key_pos below), its 16-byte slots XOR-swizzled by (dim >> 2) & 3 so each ds_read_b128 lane
//     group reads 16 distinct slots.
#include "wc_x6.hpp"

namespace {

using namespace wcx6;

constexpr int NT = 256;
constexpr int KT = 32;  // keys per tile
// 1 (default): the pre-split d = 128 forms read a tile's K fragments all at once and its V fragments
// before the softmax (one LDS latency per phase, the V reads under the softmax VALU; 252 VGPRs, still
// two waves per SIMD): 1549 -> 1514 us on the 64 x 64 attention, same box.  0 for A/B builds.
#ifndef WC_ATT_PREF
#define WC_ATT_PREF 1
#endif

template <int D, bool F3>
struct Ax6 {
    static_assert(D % 32 == 0, "split-precision attention needs D % 32 == 0");
    static constexpr int NP = F3 ? 2 : 3;               // pieces per operand
    static constexpr int NCH = D / 16;                  // QK^T K-steps
    static constexpr int NDB = D / 32;                  // O^T 32-dim blocks
    static constexpr int KPLANE = KT * 16;              // bytes of one (piece, chunk, k-half) K plane
    static constexpr int KBYTES = NP * NCH * 2 * KPLANE; // K pieces of one tile
    static constexpr int VPLANE = D * KT * 2;           // bytes of one V^T piece
    static constexpr int VBYTES = NP * VPLANE;
    static constexpr int STAGE = KBYTES + VBYTES;
    static constexpr int LDS = 2 * STAGE;
    static constexpr int KPT = KT * D / 4 / NT;         // K float4 items per thread
    static constexpr int VITEMS = (KT / 2) * (D / 4);   // V (key pair, dim quad) items
    static constexpr int VPT = (VITEMS + NT - 1) / NT;
};

// 16-byte buffer load per lane straight into LDS at the wave-uniform base dst (device-only helper:
// the target builtins must not appear in the kernel body the host pass parses)
WC_DEVICE void buf_lds16(__amdgpu_buffer_rsrc_t srd, void* dst, unsigned voff, int soff) {
    __builtin_amdgcn_raw_ptr_buffer_load_lds(srd, (__attribute__((address_space(3))) void*)dst, 16, voff, soff, 0, 0);
}
WC_DEVICE int uniform_int(int v) { return __builtin_amdgcn_readfirstlane(v); }

// position of key k (0..31) in the permuted K16 order of the PV MFMA (see header)
WC_DEVICE int key_pos(int k) { return attn_key_pos(k); }

// The three bf16 piece bit patterns (hi16 = the piece) of 4 floats, per element.
WC_DEVICE void split3_elems(f32x4 v, unsigned (&u)[3][4]) {
#pragma unroll
    for (int e = 0; e < 4; ++e) {
        const float x = v[e];
        const unsigned a = __float_as_uint(x);
        const float r1 = x - __uint_as_float(a & 0xffff0000u);
        const unsigned c = __float_as_uint(r1);
        const float r2 = r1 - __uint_as_float(c & 0xffff0000u);
        u[0][e] = a;
        u[1][e] = c;
        u[2][e] = __float_as_uint(r2);
    }
}

// 16-bit pieces of 8 consecutive values as MFMA operands: NP x u32x4
template <bool F3>
WC_DEVICE void pieces8(f32x4 v0, f32x4 v1, u32x4 (&out)[F3 ? 2 : 3]) {
    if constexpr (F3) {
        u32x2 a0, a1, b0, b1;
        split2_f16(v0, a0, a1);
        split2_f16(v1, b0, b1);
        out[0] = u32x4{a0.x, a0.y, b0.x, b0.y};
        out[1] = u32x4{a1.x, a1.y, b1.x, b1.y};
    } else {
        u32x2 a0, a1, a2, b0, b1, b2;
        split3(v0, a0, a1, a2);
        split3(v1, b0, b1, b2);
        out[0] = u32x4{a0.x, a0.y, b0.x, b0.y};
        out[1] = u32x4{a1.x, a1.y, b1.x, b1.y};
        out[2] = u32x4{a2.x, a2.y, b2.x, b2.y};
    }
}

template <bool F3>
WC_DEVICE void mfma_split(f32x16& acc, const u32x4 (&a)[F3 ? 2 : 3], const u32x4 (&b)[F3 ? 2 : 3]) {
    if constexpr (F3) {
        acc = mfma_f16(a[0], b[0], acc);
        acc = mfma_f16c(a[0], b[1], acc);
        acc = mfma_f16c(a[1], b[0], acc);
    } else {
        acc = mfma_bf16(a[0], b[0], acc);
        acc = mfma_bf16(a[0], b[1], acc);
        acc = mfma_bf16(a[1], b[0], acc);
        acc = mfma_bf16(a[0], b[2], acc);
        acc = mfma_bf16(a[1], b[1], acc);
        acc = mfma_bf16(a[2], b[0], acc);
    }
}

// qs, ks, vs: scales applied to Q, K, V before splitting (1 for bf16x6); score_mul multiplies the
// raw S^T accumulator into the exp2 domain; out_mul multiplies O / l at the end.
// f16x3 up to D = 128 fits 256 registers (two waves per SIMD: one wave's softmax / staging VALU
// runs under the other's MFMAs); the larger forms keep Q and O in 512 registers at one wave.
// PRE (f16x3 only): qkv is the pre-split projection of wc_conv_igemm_f16x3_qkv (already scaled by
// 2^exps; qs, ks, vs unused); K and V^T tiles are copied into LDS by LDS-DMA in their final image.
// O3 (PRE only): `out` is the A operand of the out-projection GEMM (wc_proj_f16x3): O x 2^ev split
// into fp16 pieces in the a3 layout of wc_split_f16x3_tiled (C % 32 == 0, N % 128 == 0), bit for bit
// what that split pass makes of the fp32 O.
template <int D, bool F3, bool PRE = false, bool O3 = false>
__global__ __launch_bounds__(NT, F3 && D <= 128 ? 2 : 1) void attention_x6_kernel(const float* __restrict__ qkv, int ldq,
                                                             float* __restrict__ out, int ldo, int N,
                                                             int C, float score_mul, float qs, float ks,
                                                             float vs, float ps, float out_mul,
                                                             float* __restrict__ lse) {
    static_assert(!PRE || F3, "pre-split operands are f16x3");
    using A = Ax6<D, F3>;
    constexpr int NP = A::NP;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;
    const int l32 = lane & 31;
    const int half = lane >> 5;
    // XCD-aware bijective order: the workgroups of one (batch, head) — which all stream the same
    // K/V — are consecutive logical blocks and land on one XCD, so its L2 holds that K/V once
    // (round-robin placement would pull it into all eight L2s).
    const int nqb = (N + 127) / 128;
    const int nblk = gridDim.x;
    int bid = blockIdx.x;
    {
        int q = nblk / 8, r = nblk % 8, xcd = bid % 8;
        bid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + bid / 8;
    }
    const int heads = C / D;
    const int head = (bid / nqb) % heads;
    const int b = bid / (nqb * heads);
    const int q0 = (bid % nqb) * 128 + wave * 32;
    const float* base = qkv + (long)b * N * ldq;
    const int qcol = head * D;
    const int kcol = C + head * D;
    const int vcol = 2 * C + head * D;
    const __amdgpu_buffer_rsrc_t srd = make_srd(base);
    // pre-split layout (wc_kernels.h, wc_conv_igemm_f16x3_qkv), in fp16 elements
    const unsigned short* q3 = reinterpret_cast<const unsigned short*>(qkv) + (long)b * 6 * C * N;
    const long hplane = (long)D * N;  // one piece of one head
    const unsigned short* Qp = q3 + (long)(head * 2) * hplane;
    const unsigned short* Kp = q3 + (long)((C / D + head) * 2) * hplane;
    const unsigned short* Vp = q3 + 4L * C * N + (long)(head * 2) * hplane;

    // ---- Q pieces: lane (query l32, half) holds Q[q][16 ch + 8 half + j] ----
    const int qrow = q0 + l32;
    u32x4 qp[A::NCH][NP];
#pragma unroll
    for (int ch = 0; ch < A::NCH; ++ch) {
        if constexpr (PRE) {
#pragma unroll
            for (int pc = 0; pc < NP; ++pc) {
                const u32x4* src = reinterpret_cast<const u32x4*>(Qp + pc * hplane + ((long)(2 * ch + half) * N + qrow) * 8);
                qp[ch][pc] = qrow < N ? *src : u32x4{0u, 0u, 0u, 0u};
            }
        } else {
            const unsigned o = (unsigned)(qrow * ldq + qcol + 16 * ch + 8 * half) * 4u;
            const f32x4 v0 = bload_f4(srd, qrow < N ? o : OOB) * qs;
            const f32x4 v1 = bload_f4(srd, qrow < N ? o + 16u : OOB) * qs;
            pieces8<F3>(v0, v1, qp[ch]);
        }
    }
    // LDS-DMA of tile t into buf (PRE): D/16 wave-instructions per wave, half K (plane pairs, key
    // slots XOR-swizzled as write_tile does), half V^T (16 dim rows, 16-byte slots swizzled)
    // Buffer loads: per-lane 32-bit byte offsets from the image's pre-split base, fixed for the
    // whole key loop; the tile enters as the scalar offset, the LDS base (M0) is wave-uniform.
    constexpr int G = D / 8;  // K planes per piece = V^T row groups of 16 per piece x 2
    const int wv = uniform_int(wave);
    unsigned kvoff[G / 4], vvoff[G / 4];
    __amdgpu_buffer_rsrc_t srd3 = make_srd(q3);
    if constexpr (PRE) {
#pragma unroll
        for (int j = 0; j < G / 4; ++j) {
            const int i = wave + 4 * j;  // 0 .. G-1: (piece, plane pair)
            const int pc = i / (G / 2), pp = i % (G / 2);
            const int pl = 2 * pp + (lane >> 5), key = (lane & 31) ^ (pl & 15);
            kvoff[j] = (unsigned)((Kp - q3) + pc * hplane + ((long)pl * N + key) * 8) * 2u;
        }
#pragma unroll
        for (int j = 0; j < G / 4; ++j) {
            const int i = wave + 4 * j;  // 0 .. G-1: (piece, 16-row block)
            const int pc = i / (D / 16), r0 = 16 * (i % (D / 16));
            const int row = r0 + (lane >> 2), slot = (lane & 3) ^ ((row >> 2) & 3);
            vvoff[j] = (unsigned)((Vp - q3) + pc * hplane + (long)row * N + slot * 8) * 2u;
        }
    }
    auto dma_tile = [&](int t, unsigned char* buf) {
        const int kv0 = t * KT;
#pragma unroll
        for (int j = 0; j < G / 4; ++j) {
            const int i = wv + 4 * j;
            const int pc = i / (G / 2), pp = i % (G / 2);
            unsigned char* dst = buf + (pc * G + 2 * pp) * A::KPLANE;
            buf_lds16(srd3, dst, kvoff[j], kv0 * 16);
        }
#pragma unroll
        for (int j = 0; j < G / 4; ++j) {
            const int i = wv + 4 * j;
            const int pc = i / (D / 16), r0 = 16 * (i % (D / 16));
            unsigned char* dst = buf + A::KBYTES + pc * A::VPLANE + r0 * (KT * 2);
            buf_lds16(srd3, dst, vvoff[j], kv0 * 2);
        }
    };

    // ---- staging coordinates ----
    // K: item i -> key i / (D/4), dims 4*(i % (D/4)) .. +3 (a wave reads whole key rows).  In LDS
    // plane pl = (16-dim chunk, k-half) the key's 16-byte slot is key ^ (pl & 15): the 16 lanes of a
    // ds_write_b64 group (one key, 8 planes x 2 halves) then hit 16 distinct bank pairs, where the
    // unswizzled image (planes 512 B apart) put them on one bank pair.
    int k_goff[A::KPT], k_key[A::KPT], k_lds[A::KPT];
#pragma unroll
    for (int j = 0; j < A::KPT; ++j) {
        const int i = tid + NT * j;
        const int key = i / (D / 4), d4 = i % (D / 4);
        const int pl = (d4 >> 2) * 2 + ((d4 >> 1) & 1);
        k_key[j] = key;
        k_goff[j] = key * ldq + kcol + 4 * d4;
        k_lds[j] = (pl * KT + (key ^ (pl & 15))) * 16 + (d4 & 1) * 8;
    }
    // V: item i -> keys 2kp, 2kp+1 (kp = i % 16) and dims 4*d4 .. +3 (d4 = i / 16): a 32-lane
    // ds_write_b32 group covers 16 key pairs x 2 dim quads, 2-way on the banks (free), where
    // dim-quad-major items put 32 lanes on 4 banks.
    int v_goff[A::VPT], v_key[A::VPT], v_pos[A::VPT], v_d[A::VPT];
#pragma unroll
    for (int j = 0; j < A::VPT; ++j) {
        const int i = tid + NT * j;
        const int kp = i % (KT / 2), d4 = i / (KT / 2);
        v_key[j] = i < A::VITEMS ? 2 * kp : 1 << 20;  // invalid items never load nor store
        v_goff[j] = 2 * kp * ldq + vcol + 4 * d4;
        v_pos[j] = key_pos(2 * kp);
        v_d[j] = 4 * d4;
    }

    f32x4 rk[A::KPT], rv[A::VPT][2];
    auto load_tile = [&](int t) {
        const int kv0 = t * KT;
#pragma unroll
        for (int j = 0; j < A::KPT; ++j)
            rk[j] = bload_f4(srd, kv0 + k_key[j] < N ? (unsigned)(kv0 * ldq + k_goff[j]) * 4u : OOB);
#pragma unroll
        for (int j = 0; j < A::VPT; ++j) {
            const unsigned o = (unsigned)(kv0 * ldq + v_goff[j]) * 4u;
            rv[j][0] = bload_f4(srd, kv0 + v_key[j] < N ? o : OOB);
            rv[j][1] = bload_f4(srd, kv0 + v_key[j] + 1 < N ? o + (unsigned)ldq * 4u : OOB);
        }
    };
    auto write_tile = [&](unsigned char* buf) {
#pragma unroll
        for (int j = 0; j < A::KPT; ++j) {
            if constexpr (F3) {
                u32x2 p0, p1;
                split2_f16(rk[j] * ks, p0, p1);
                *reinterpret_cast<u32x2*>(buf + k_lds[j]) = p0;
                *reinterpret_cast<u32x2*>(buf + A::NCH * 2 * A::KPLANE + k_lds[j]) = p1;
            } else {
                u32x2 p0, p1, p2;
                split3(rk[j], p0, p1, p2);
                *reinterpret_cast<u32x2*>(buf + k_lds[j]) = p0;
                *reinterpret_cast<u32x2*>(buf + A::NCH * 2 * A::KPLANE + k_lds[j]) = p1;
                *reinterpret_cast<u32x2*>(buf + 2 * A::NCH * 2 * A::KPLANE + k_lds[j]) = p2;
            }
        }
        unsigned char* vb = buf + A::KBYTES;
#pragma unroll
        for (int j = 0; j < A::VPT; ++j) {
            if (v_key[j] >= KT) continue;
            const int pos = v_pos[j];
            if constexpr (F3) {
                const f32x4 va = rv[j][0] * vs, vb4 = rv[j][1] * vs;
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const int d = v_d[j] + e;
                    const int off = d * (KT * 2) + (((pos >> 3) ^ ((d >> 2) & 3)) << 4) + (pos & 7) * 2;
                    unsigned h, l;  // keys 2kp (low half) and 2kp + 1 of dim d, split as one pair
                    split2_pair(f32x2{va[e], vb4[e]}, h, l);
                    *reinterpret_cast<unsigned*>(vb + off) = h;
                    *reinterpret_cast<unsigned*>(vb + A::VPLANE + off) = l;
                }
            } else {
                unsigned ua[3][4], ub[3][4];
                split3_elems(rv[j][0], ua);
                split3_elems(rv[j][1], ub);
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const int d = v_d[j] + e;
                    const int off = d * (KT * 2) + (((pos >> 3) ^ ((d >> 2) & 3)) << 4) + (pos & 7) * 2;
#pragma unroll
                    for (int pc = 0; pc < 3; ++pc)
                        *reinterpret_cast<unsigned*>(vb + pc * A::VPLANE + off) = hi_pair(ub[pc][e], ua[pc][e]);
                }
            }
        }
    };

    f32x16 o[A::NDB];
#pragma unroll
    for (int d = 0; d < A::NDB; ++d)
#pragma unroll
        for (int r = 0; r < 16; ++r) o[d][r] = 0.f;
    float m_run = -INFINITY, l_run = 0.f;

    const int ntiles = (N + KT - 1) / KT;
    if constexpr (PRE) {
        dma_tile(0, smem);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else {
        load_tile(0);
        write_tile(smem);
    }
    __syncthreads();
    for (int t = 0; t < ntiles; ++t) {
        const unsigned char* cur = smem + (t & 1) * A::STAGE;
        const int kv0 = t * KT;
        if constexpr (PRE) {
            if (t + 1 < ntiles) dma_tile(t + 1, smem + ((t + 1) & 1) * A::STAGE);  // buffer last read in tile t - 1
        } else {
            if (t + 1 < ntiles) load_tile(t + 1);
        }

        // ---- S^T = K Q^T ----
        f32x16 s;
#pragma unroll
        for (int r = 0; r < 16; ++r) s[r] = 0.f;
#if WC_ATT_PREF
        if constexpr (PRE && D == 128) {
            // all of the tile's K fragments first (one LDS latency for the whole S, not one per chunk)
            u32x4 kf[A::NCH][NP];
#pragma unroll
            for (int ch = 0; ch < A::NCH; ++ch)
#pragma unroll
                for (int pc = 0; pc < NP; ++pc)
                    kf[ch][pc] = *reinterpret_cast<const u32x4*>(cur + ((pc * A::NCH + ch) * 2 + half) * A::KPLANE +
                                                                  (l32 ^ ((ch * 2 + half) & 15)) * 16);
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int ch = 0; ch < A::NCH; ++ch) mfma_split<F3>(s, kf[ch], qp[ch]);
        } else
#endif
        {
#pragma unroll
        for (int ch = 0; ch < A::NCH; ++ch) {
            u32x4 kf[NP];
#pragma unroll
            for (int pc = 0; pc < NP; ++pc)
                kf[pc] = *reinterpret_cast<const u32x4*>(cur + ((pc * A::NCH + ch) * 2 + half) * A::KPLANE +
                                                          (l32 ^ ((ch * 2 + half) & 15)) * 16);
            mfma_split<F3>(s, kf, qp[ch]);
        }
        }
#if WC_ATT_PREF
        // the tile's V fragments issued before the softmax, whose VALU covers their latency
        u32x4 vpre[(PRE && D == 128) ? 2 : 1][(PRE && D == 128) ? A::NDB : 1][NP];
        if constexpr (PRE && D == 128) {
#pragma unroll
            for (int c = 0; c < 2; ++c)
#pragma unroll
                for (int db = 0; db < A::NDB; ++db) {
                    const int d = db * 32 + l32;
                    const int off = A::KBYTES + d * (KT * 2) + (((2 * c + half) ^ ((d >> 2) & 3)) << 4);
#pragma unroll
                    for (int pc = 0; pc < NP; ++pc)
                        vpre[c][db][pc] = *reinterpret_cast<const u32x4*>(cur + off + pc * A::VPLANE);
                }
        }
#endif

        // ---- online softmax over keys, per query (lane) ----
        // The running max is kept in the exp2 domain: max(s) * score_mul = max(s * score_mul)
        // (score_mul > 0, rounding is monotonic), and each probability is one fma + v_exp_f32:
        // p = 2^(s * score_mul + EP - m) carries the f16x3 prescale 2^EP of P exactly in the
        // exponent (l carries it too, and out_mul omits it)
        float mloc = -INFINITY;
        if (PRE || kv0 + KT <= N) {  // full tile (wave-uniform; PRE needs N % KT == 0): no key mask
#pragma unroll
            for (int r = 0; r < 16; ++r) mloc = fmaxf(mloc, s[r]);
        } else {
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int key = kv0 + (r & 3) + 8 * (r >> 2) + 4 * half;
                if (key >= N) s[r] = -INFINITY;
                mloc = fmaxf(mloc, s[r]);
            }
        }
        mloc = fmaxf(mloc, __shfl_xor(mloc, 32, 64));
        const float m_new = fmaxf(m_run, mloc * score_mul);
        const float alpha = __builtin_amdgcn_exp2f(m_run - m_new);  // v_exp_f32 (results < 2^-126 flush: negligible)
        const float nb = (F3 ? 14.0f : 0.0f) - m_new;
#pragma unroll
        for (int r = 0; r < 16; ++r) s[r] = __builtin_amdgcn_exp2f(fmaf(s[r], score_mul, nb));
        // row sum as a packed-add tree (8 instructions, not 16)
        f32x2 ts[4];
#pragma unroll
        for (int i = 0; i < 4; ++i)
            ts[i] = f32x2{s[4 * i], s[4 * i + 1]} + f32x2{s[4 * i + 2], s[4 * i + 3]};
        const f32x2 u = (ts[0] + ts[1]) + (ts[2] + ts[3]);
        float lsum = u.x + u.y;
        lsum += __shfl_xor(lsum, 32, 64);
        l_run = l_run * alpha + lsum;
        m_run = m_new;
        // alpha == 1 exactly when no lane's running max moved: skipping the multiply is then exact
        if (__builtin_amdgcn_ballot_w64(alpha != 1.0f)) {
#pragma unroll
            for (int d = 0; d < A::NDB; ++d)
#pragma unroll
                for (int r = 0; r < 16; ++r) o[d][r] *= alpha;
        }

        // ---- O^T += V^T P^T: two 16-key chunks ----
#pragma unroll
        for (int c = 0; c < 2; ++c) {
            u32x4 pp[NP];
            pieces8<F3>(f32x4{s[8 * c + 0], s[8 * c + 1], s[8 * c + 2], s[8 * c + 3]},
                        f32x4{s[8 * c + 4], s[8 * c + 5], s[8 * c + 6], s[8 * c + 7]}, pp);
#pragma unroll
            for (int db = 0; db < A::NDB; ++db) {
                const int d = db * 32 + l32;
                const int off = A::KBYTES + d * (KT * 2) + (((2 * c + half) ^ ((d >> 2) & 3)) << 4);
#if WC_ATT_PREF
                if constexpr (PRE && D == 128) {
                    (void)off;
                    mfma_split<F3>(o[db], vpre[c][db], pp);
                    continue;
                }
#endif
                u32x4 vf[NP];
#pragma unroll
                for (int pc = 0; pc < NP; ++pc)
                    vf[pc] = *reinterpret_cast<const u32x4*>(cur + off + pc * A::VPLANE);
                mfma_split<F3>(o[db], vf, pp);
            }
        }

        if constexpr (PRE) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's DMA of tile t + 1 landed
        } else {
            if (t + 1 < ntiles) write_tile(smem + ((t + 1) & 1) * A::STAGE);
        }
        __syncthreads();
    }

    // ---- epilogue: O[q][dv] = O^T[dv][q] / l ----
    if constexpr (O3) {
        if (qrow < N) {
            const float inv = out_mul / l_run;
            const long m = (long)b * N + qrow;  // GEMM row (pixel of the batch)
            const long rowbase = ((m >> 7) * (C / 16)) * 4 * 128 * 16 + (m & 127) * 16 + 8 * half;
            unsigned char* a3 = reinterpret_cast<unsigned char*>(out);
#pragma unroll
            for (int d = 0; d < A::NDB; ++d) {
#pragma unroll
                for (int r = 0; r < 16; r += 4) {
                    const int c = head * D + d * 32 + 8 * (r >> 2) + 4 * half;  // c % 8 == 4 half
                    const f32x4 v = f32x4{o[d][r] * inv, o[d][r + 1] * inv, o[d][r + 2] * inv, o[d][r + 3] * inv} * vs;
                    u32x2 ph, pl;
                    split2_f16(v, ph, pl);
                    unsigned char* dst = a3 + rowbase + ((long)(c >> 4) * 4 + ((c >> 3) & 1)) * 128 * 16;
                    *reinterpret_cast<u32x2*>(dst) = ph;                 // piece 0
                    *reinterpret_cast<u32x2*>(dst + 2 * 128 * 16) = pl;  // piece 1
                }
            }
        }
        return;
    }
    // log-sum-exp of the scaled scores for the backward (wc_attention_bwd's contract):
    // lse = log2 sum_k 2^(s_k * scale * log2 e) = m + log2(l) - EP, EP the f16x3 P prescale
    if (lse != nullptr && half == 0 && qrow < N)
        lse[((long)b * heads + head) * N + qrow] = m_run + log2f(l_run) - (F3 ? 14.0f : 0.0f);
    if (qrow < N) {
        const float inv = out_mul / l_run;
        float* orow = out + ((long)b * N + qrow) * ldo + head * D;
#pragma unroll
        for (int d = 0; d < A::NDB; ++d) {
#pragma unroll
            for (int r = 0; r < 16; r += 4) {
                const int dv = d * 32 + 8 * (r >> 2) + 4 * half;
                *reinterpret_cast<f32x4*>(orow + dv) =
                    f32x4{o[d][r] * inv, o[d][r + 1] * inv, o[d][r + 2] * inv, o[d][r + 3] * inv};
            }
        }
    }
}

template <int D, bool F3, bool PRE = false, bool O3 = false>
int launch_att6(const float* qkv, int ldq, float* out, int ldo, int B, int N, int C, int heads,
                float scale, int eq, int ek, int ev, hipStream_t stream, float* lse = nullptr) {
    using A = Ax6<D, F3>;
    static bool attr_set = false;
    if (!attr_set) {
        hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&attention_x6_kernel<D, F3, PRE, O3>),
                                           hipFuncAttributeMaxDynamicSharedMemorySize, A::LDS);
        if (e != hipSuccess) return (int)e;
        attr_set = true;
    }
    // P carries 2^14 under f16x3 (small probabilities stay in the fp16 normal range); it is added
    // in the exp2 argument inside the kernel and cancels in O / l
    const float score_mul = scale * 1.4426950408889634f * ldexpf(1.f, -(eq + ek));
    dim3 grid(((N + 127) / 128) * heads * B);
    WC_SET_NAME("attention_x6_kernel", {WC_TI(D), WC_TB(F3), WC_TB(PRE), WC_TB(O3)});
    hipLaunchKernelGGL((attention_x6_kernel<D, F3, PRE, O3>), grid, dim3(NT), A::LDS, stream, qkv, ldq, out, ldo, N, C,
                       score_mul, ldexpf(1.f, eq), ldexpf(1.f, ek), ldexpf(1.f, ev), 1.0f, ldexpf(1.f, -ev), lse);
    WC_CHECK_LAUNCH();
    return WC_OK;
}

template <bool F3>
int dispatch_att6(const float* qkv, int ld_qkv, float* out, int ld_out, int B, int N, int C, int heads,
                  float scale, int eq, int ek, int ev, hipStream_t s, float* lse = nullptr) {
    if (!qkv || !out) return WC_E_ARG;
    if (heads <= 0 || C % heads != 0 || ld_qkv % 4 != 0 || ld_out % 4 != 0) return WC_E_SHAPE;
    if (ld_qkv < 3 * C || ld_out < C || N <= 0 || B <= 0) return WC_E_SHAPE;
    if ((reinterpret_cast<uintptr_t>(qkv) & 15) || (reinterpret_cast<uintptr_t>(out) & 15)) return WC_E_SHAPE;
    if ((long)N * ld_qkv * 4 >= (1L << 31)) return WC_E_SHAPE;  // per-image SRD range
    if (eq < -60 || eq > 60 || ek < -60 || ek > 60 || ev < -60 || ev > 60) return WC_E_ARG;
    switch (C / heads) {
        case 32: return launch_att6<32, F3>(qkv, ld_qkv, out, ld_out, B, N, C, heads, scale, eq, ek, ev, s, lse);
        case 64: return launch_att6<64, F3>(qkv, ld_qkv, out, ld_out, B, N, C, heads, scale, eq, ek, ev, s, lse);
        case 96: return launch_att6<96, F3>(qkv, ld_qkv, out, ld_out, B, N, C, heads, scale, eq, ek, ev, s, lse);
        case 128: return launch_att6<128, F3>(qkv, ld_qkv, out, ld_out, B, N, C, heads, scale, eq, ek, ev, s, lse);
        case 160: return launch_att6<160, F3>(qkv, ld_qkv, out, ld_out, B, N, C, heads, scale, eq, ek, ev, s, lse);
        case 192: return launch_att6<192, F3>(qkv, ld_qkv, out, ld_out, B, N, C, heads, scale, eq, ek, ev, s, lse);
        default: return WC_E_SHAPE;
    }
}

int dispatch_att_presplit(const void* qkv3, float* out, int ld_out, int B, int N, int C, int heads, float scale,
                          int eq, int ek, int ev, hipStream_t s) {
    if (!qkv3 || !out) return WC_E_ARG;
    if (heads <= 0 || C % heads != 0 || ld_out % 4 != 0 || ld_out < C || N <= 0 || B <= 0 || N % KT) return WC_E_SHAPE;
    if ((reinterpret_cast<uintptr_t>(qkv3) & 15) || (reinterpret_cast<uintptr_t>(out) & 15)) return WC_E_SHAPE;
    if (eq < -60 || eq > 60 || ek < -60 || ek > 60 || ev < -60 || ev > 60) return WC_E_ARG;
    const float* q = reinterpret_cast<const float*>(qkv3);
    switch (C / heads) {
        case 32: return launch_att6<32, true, true>(q, 0, out, ld_out, B, N, C, heads, scale, eq, ek, ev, s);
        case 64: return launch_att6<64, true, true>(q, 0, out, ld_out, B, N, C, heads, scale, eq, ek, ev, s);
        case 96: return launch_att6<96, true, true>(q, 0, out, ld_out, B, N, C, heads, scale, eq, ek, ev, s);
        case 128: return launch_att6<128, true, true>(q, 0, out, ld_out, B, N, C, heads, scale, eq, ek, ev, s);
        case 160: return launch_att6<160, true, true>(q, 0, out, ld_out, B, N, C, heads, scale, eq, ek, ev, s);
        case 192: return launch_att6<192, true, true>(q, 0, out, ld_out, B, N, C, heads, scale, eq, ek, ev, s);
        default: return WC_E_SHAPE;
    }
}

int dispatch_att_presplit_a3(const void* qkv3, void* a3, int64_t a3_bytes, int B, int N, int C, int heads,
                             float scale, int eq, int ek, int ev, hipStream_t s) {
    if (!qkv3 || !a3) return WC_E_ARG;
    if (heads <= 0 || C % heads != 0 || C % 32 || N <= 0 || B <= 0 || N % 128) return WC_E_SHAPE;
    if ((reinterpret_cast<uintptr_t>(qkv3) & 15) || (reinterpret_cast<uintptr_t>(a3) & 15)) return WC_E_SHAPE;
    if (a3_bytes != (long)B * N * C * 4) return WC_E_SHAPE;
    if (eq < -60 || eq > 60 || ek < -60 || ek > 60 || ev < -60 || ev > 60) return WC_E_ARG;
    const float* q = reinterpret_cast<const float*>(qkv3);
    float* o = reinterpret_cast<float*>(a3);
    switch (C / heads) {
        case 32: return launch_att6<32, true, true, true>(q, 0, o, C, B, N, C, heads, scale, eq, ek, ev, s);
        case 64: return launch_att6<64, true, true, true>(q, 0, o, C, B, N, C, heads, scale, eq, ek, ev, s);
        case 96: return launch_att6<96, true, true, true>(q, 0, o, C, B, N, C, heads, scale, eq, ek, ev, s);
        case 128: return launch_att6<128, true, true, true>(q, 0, o, C, B, N, C, heads, scale, eq, ek, ev, s);
        case 160: return launch_att6<160, true, true, true>(q, 0, o, C, B, N, C, heads, scale, eq, ek, ev, s);
        case 192: return launch_att6<192, true, true, true>(q, 0, o, C, B, N, C, heads, scale, eq, ek, ev, s);
        default: return WC_E_SHAPE;
    }
}

}  // namespace

extern "C" int wc_attention_fwd_f16x3_presplit_a3(const void* qkv3, void* a3, int64_t a3_bytes, int B, int N, int C,
                                                  int heads, float scale, int q_exp, int k_exp, int v_exp,
                                                  void* stream) {
    return dispatch_att_presplit_a3(qkv3, a3, a3_bytes, B, N, C, heads, scale, q_exp, k_exp, v_exp,
                                    reinterpret_cast<hipStream_t>(stream));
}

extern "C" int wc_attention_fwd_f16x3_presplit(const void* qkv3, float* out, int ld_out, int B, int N, int C,
                                               int heads, float scale, int q_exp, int k_exp, int v_exp,
                                               void* stream) {
    return dispatch_att_presplit(qkv3, out, ld_out, B, N, C, heads, scale, q_exp, k_exp, v_exp,
                                 reinterpret_cast<hipStream_t>(stream));
}

extern "C" int wc_attention_fwd_x6(const float* qkv, int ld_qkv, float* out, int ld_out, int B, int N,
                                   int C, int heads, float scale, void* stream) {
    return dispatch_att6<false>(qkv, ld_qkv, out, ld_out, B, N, C, heads, scale, 0, 0, 0,
                                reinterpret_cast<hipStream_t>(stream));
}

extern "C" int wc_attention_fwd_f16x3(const float* qkv, int ld_qkv, float* out, int ld_out, int B, int N,
                                      int C, int heads, float scale, int q_exp, int k_exp, int v_exp,
                                      void* stream) {
    return dispatch_att6<true>(qkv, ld_qkv, out, ld_out, B, N, C, heads, scale, q_exp, k_exp, v_exp,
                               reinterpret_cast<hipStream_t>(stream));
}

// The same split-precision forwards, also writing the softmax log-sum-exp lse[b][head][query]
// (float32 [B][heads][N], the contract of wc_attention_fwd_lse / wc_attention_bwd): the training
// forward's attention on the sampler's arithmetic.
extern "C" int wc_attention_fwd_f16x3_lse(const float* qkv, int ld_qkv, float* out, int ld_out, float* lse, int B,
                                          int N, int C, int heads, float scale, int q_exp, int k_exp, int v_exp,
                                          void* stream) {
    if (!lse) return WC_E_ARG;
    return dispatch_att6<true>(qkv, ld_qkv, out, ld_out, B, N, C, heads, scale, q_exp, k_exp, v_exp,
                               reinterpret_cast<hipStream_t>(stream), lse);
}

extern "C" int wc_attention_fwd_x6_lse(const float* qkv, int ld_qkv, float* out, int ld_out, float* lse, int B, int N,
                                       int C, int heads, float scale, void* stream) {
    if (!lse) return WC_E_ARG;
    return dispatch_att6<false>(qkv, ld_qkv, out, ld_out, B, N, C, heads, scale, 0, 0, 0,
                                reinterpret_cast<hipStream_t>(stream), lse);
}
