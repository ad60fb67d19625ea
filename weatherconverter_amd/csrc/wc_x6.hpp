// Shared helpers of the bf16x6 split-precision kernels (wc_conv6.hip, wc_igemm6.hip).
#pragma once
#include "wc_common.hpp"

namespace wcx6 {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x2 __attribute__((ext_vector_type(2)));

constexpr unsigned OOB = 0x80000000u;  // byte offset past the SRD range -> load returns 0
constexpr int SRD_BYTES = 0x7FFFFFFF;
constexpr int SRD_FLAGS = 0x00020000;

WC_DEVICE __amdgpu_buffer_rsrc_t make_srd(const void* p) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, SRD_BYTES, SRD_FLAGS);
}
WC_DEVICE f32x4 bload_f4(__amdgpu_buffer_rsrc_t r, unsigned off) {
    return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0));
}
WC_DEVICE u32x4 bload_u4(__amdgpu_buffer_rsrc_t r, unsigned off) {
    return __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0));
}

// per-lane offset voff plus a wave-uniform (SGPR) offset soff: loop-invariant lane offsets need no
// per-load VALU (OOB in voff still reads 0: the range check is on voff + the immediate)
WC_DEVICE f32x4 bload_f4s(__amdgpu_buffer_rsrc_t r, unsigned voff, int soff) {
    return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, voff, soff, 0));
}
WC_DEVICE u32x4 bload_u4s(__amdgpu_buffer_rsrc_t r, unsigned voff, int soff) {
    return __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(r, voff, soff, 0));
}

WC_DEVICE float bload_f1(__amdgpu_buffer_rsrc_t r, unsigned off) {
    return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, off, 0, 0));
}
WC_DEVICE void bstore_f1(__amdgpu_buffer_rsrc_t r, unsigned off, float v) {
    __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, v), r, off, 0, 0);
}

WC_DEVICE float bload_f1s(__amdgpu_buffer_rsrc_t r, unsigned voff, int soff) {
    return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, voff, soff, 0));
}
WC_DEVICE void bstore_f1s(__amdgpu_buffer_rsrc_t r, unsigned voff, int soff, float v) {
    __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, v), r, voff, soff, 0);
}

WC_DEVICE void bstore_f4(__amdgpu_buffer_rsrc_t r, unsigned off, f32x4 v) {
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), r, off, 0, 0);
}

WC_DEVICE f32x16 mfma_bf16(u32x4 a, u32x4 b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, a),
                                                   __builtin_bit_cast(bf16x8, b), c, 0, 0, 0);
}

// A correction product of the f16x3 split (h*l or l*h).  The single-piece builds drop them: every
// f16x3 kernel then computes with one 16-bit piece per operand (h*h), fp32 accumulation, the same
// power-of-two range scaling.  -DWC_SINGLE16=1 (libwc_kernels_single16.so, the 16-bit training line):
// the piece is fp16; -DWC_SINGLE16=2 (libwc_kernels_bf16.so, the bf16 training line of BASELINE
// config 3): the piece is bf16 (round to nearest even) on v_mfma_f32_32x32x16_bf16, and every pack /
// pre-split writer emits bf16 bits through the helpers below.
#ifndef WC_SINGLE16
#define WC_SINGLE16 0
#endif
WC_DEVICE f32x16 mfma_f16(u32x4 a, u32x4 b, f32x16 c) {
#if WC_SINGLE16 == 2
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), c,
                                                   0, 0, 0);
#else
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b), c,
                                                  0, 0, 0);
#endif
}
WC_DEVICE f32x16 mfma_f16c(u32x4 a, u32x4 b, f32x16 c) {
#if WC_SINGLE16
    (void)a;
    (void)b;
    return c;
#else
    return mfma_f16(a, b, c);
#endif
}

WC_DEVICE float silu_fast(float v) { return v * __builtin_amdgcn_rcpf(1.0f + __expf(-v)); }

// High halves of two fp32 bit patterns packed into one dword: (hi16(hi) << 16) | hi16(lo).
WC_DEVICE unsigned hi_pair(unsigned hi, unsigned lo) { return __builtin_amdgcn_perm(hi, lo, 0x07060302u); }

// Exact three-piece bf16 split of 4 floats by truncation: v = p0 + p1 + p2 exactly, each piece
// 8 significant bits (wc_conv6.hip header comment).
// NOTE: bit-cast a scalar copy, never the subscript v[e] directly: hipcc (ROCm 7.2 clang) lowers
// __builtin_bit_cast(unsigned, v[e]) of an ext_vector element to element 0 for every e
// (tools/probes/bitcast_vector_element.hip reproduces it).
WC_DEVICE void split3(f32x4 v, u32x2& p0, u32x2& p1, u32x2& p2) {
    unsigned u0[4], u1[4], u2[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
        const float x = v[e];
        const unsigned a = __float_as_uint(x);
        const float r1 = x - __uint_as_float(a & 0xffff0000u);
        const unsigned c = __float_as_uint(r1);
        const float r2 = r1 - __uint_as_float(c & 0xffff0000u);
        u0[e] = a;
        u1[e] = c;
        u2[e] = __float_as_uint(r2);
    }
    p0 = u32x2{hi_pair(u0[1], u0[0]), hi_pair(u0[3], u0[2])};
    p1 = u32x2{hi_pair(u1[1], u1[0]), hi_pair(u1[3], u1[2])};
    p2 = u32x2{hi_pair(u2[1], u2[0]), hi_pair(u2[3], u2[2])};
}

// Two-piece fp16 split by round-to-nearest: h = fp16(v), l = fp16(v - h) (v - h is exact in fp32),
// so v = h + l to 2^-22 |v| (or 2^-25 absolute when l is subnormal).  Callers bound |v| < 2^15.
// Two values at a time: v_cvt_pk_f16_f32 (gfx950, RNE) -> 2 x v_cvt_f32_f16 -> v_pk_add_f32 ->
// v_cvt_pk_f16_f32, 2.5 VALU per value, already packed as the MFMA operand wants.
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef _Float16 f16x2v __attribute__((ext_vector_type(2)));
// l = fp16(v - h) by v_fma_mix (f32 v, f16 h): v - h is exact in fp32 (at most 12 significant bits
// below h), so rounding the exact fma result to fp16 once is bit for bit the convert-back / subtract /
// convert sequence, in 3 instructions per pair instead of 5-6
typedef __bf16 bf16x2v __attribute__((ext_vector_type(2)));
WC_DEVICE void split2_pair(f32x2 v, unsigned& h, unsigned& l) {
#if WC_SINGLE16 == 2
    h = __builtin_bit_cast(unsigned, __builtin_convertvector(v, bf16x2v));  // v_cvt_pk_bf16_f32 (RNE)
    l = 0u;  // the single-piece line has no correction products
#else
    const f16x2v hh = __builtin_convertvector(v, f16x2v);
    h = __builtin_bit_cast(unsigned, hh);
    asm("v_fma_mixlo_f16 %0, %1, 1.0, -%2 op_sel_hi:[0,0,1]\n\t"
        "v_fma_mixhi_f16 %0, %3, 1.0, -%2 op_sel:[0,0,1] op_sel_hi:[0,0,1]"
        : "=&v"(l) : "v"(v.x), "v"(h), "v"(v.y));
#endif
}
// The two 16-bit pieces of one value (h = piece(v), l = piece(v - h); bf16 line: l = 0), as bit patterns.
WC_DEVICE void split2_one(float v, unsigned short& h, unsigned short& l) {
#if WC_SINGLE16 == 2
    h = __builtin_bit_cast(unsigned short, (__bf16)v);
    l = 0;
#else
    const _Float16 hh = (_Float16)v;
    h = __builtin_bit_cast(unsigned short, hh);
    l = __builtin_bit_cast(unsigned short, (_Float16)(v - (float)hh));
#endif
}
WC_DEVICE void split2_f16(f32x4 v, u32x2& ph, u32x2& pl) {
    unsigned h0, l0, h1, l1;
    split2_pair(f32x2{v.x, v.y}, h0, l0);
    split2_pair(f32x2{v.z, v.w}, h1, l1);
    ph = u32x2{h0, h1};
    pl = u32x2{l0, l1};
}

// Position of key k (0..31) of a 32-key tile in the K16 order of the attention P V^T MFMA: inside
// each 16-key half, keys 4-7 and 8-11 swap places (wc_attention6.hip header).
WC_DEVICE int attn_key_pos(int k) {
    const int c = k >> 4, kk = k & 15;
    return 16 * c + 8 * ((kk >> 2) & 1) + (kk & 3) + 4 * (kk >> 3);
}

// Raise absmax[b] to the wave's max of m (|values| >= 0: their float bits order like unsigned ints).
WC_DEVICE void wave_absmax_atomic(float* absmax, int b, float m) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
    if ((threadIdx.x & 63) == 0) atomicMax(reinterpret_cast<unsigned*>(absmax) + b, __float_as_uint(m));
}

// The workgroup's max |value| in one atomic (the wave maxima meet in LDS): many same-address
// device atomics serialise -- one per wave cost the attention out-projection up to 40 % of its
// time (tools/probes/proj_epi_probe.py).  Every thread of the block must call it.
WC_DEVICE void block_absmax_atomic(float* absmax, int b, float m) {
    __shared__ float wmax[16];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
    if ((threadIdx.x & 63) == 0) wmax[threadIdx.x >> 6] = m;
    __syncthreads();
    if (threadIdx.x == 0) {
        float r = wmax[0];
        for (int i = 1; i < (int)(blockDim.x >> 6); ++i) r = fmaxf(r, wmax[i]);
        atomicMax(reinterpret_cast<unsigned*>(absmax) + b, __float_as_uint(r));
    }
}

// GroupNorm tile partials from a wave's 64 x 64 output block (2 x 2 MFMA 32x32 blocks whose
// acc[mb][nb][r] already hold the FINAL stored values).  For each valid 32-channel column block nb
// and each sub-slot of sw channels in it: (mean, M2) over the 64 pixels x sw channels, two passes
// over the registers (no E[x^2] - E[x]^2 cancellation), lane butterflies in a fixed order
// (deterministic).  Written to part[((pix64 * ncb + cb) * (32 / sw) + sub) * 2 + {0, 1}].
struct GnTile {
    float* part;
    int ncb, sw;  // channel blocks of 32 in the tensor, sub-slot width (4, 8, 16 or 32)
    long pix64;   // b * np64 + p64 of this wave's 64 pixels
    int cb0;      // column block of nb = 0
};
WC_DEVICE float gn_seg_sum(float v, int sw) {
    for (int o = 1; o < sw; o <<= 1) v += __shfl_xor(v, o, 64);
    return v + __shfl_xor(v, 32, 64);
}
template <int NB>
WC_DEVICE void gn_tile_partials(const f32x16 (&acc)[2][NB], const GnTile& g, int nvalid) {
    const int lane = threadIdx.x & 63;
    const float inv_n = 1.0f / (64.0f * (float)g.sw);
#pragma unroll
    for (int nb = 0; nb < NB; ++nb) {
        if (nb >= nvalid) break;
        float s = 0.f;
#pragma unroll
        for (int mb = 0; mb < 2; ++mb)
#pragma unroll
            for (int r = 0; r < 16; ++r) s += acc[mb][nb][r];
        const float mean = gn_seg_sum(s, g.sw) * inv_n;
        float q = 0.f;
#pragma unroll
        for (int mb = 0; mb < 2; ++mb)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const float d = acc[mb][nb][r] - mean;
                q = fmaf(d, d, q);
            }
        const float m2 = gn_seg_sum(q, g.sw);
        const int c = lane & 31;
        if (lane < 32 && (c & (g.sw - 1)) == 0) {
            const long idx = ((g.pix64 * g.ncb + g.cb0 + nb) * (32 / g.sw) + c / g.sw) * 2;
            g.part[idx] = mean;
            g.part[idx + 1] = m2;
        }
    }
}

// The same partials from the TRANSPOSED accumulators of conv_igemm_x6_kernel<..., TR> (lanes =
// pixels): acc[mb][nb][4 j + e] is pixel 32 mb + (lane & 31) of the wave's 64, channel
// 8 j + 4 (lane / 32) + e of column block nb.  A sub-slot of sw channels is the lane's quads
// (j, half) with (8 j + 4 half) / sw equal, reduced over the 32 pixels of each half (and over the
// halves for sw >= 8); two passes over the registers, fixed butterfly order.
template <int NB>
WC_DEVICE void gn_tile_partials_tr(const f32x16 (&acc)[2][NB], const GnTile& g, int nvalid) {
    const int lane = threadIdx.x & 63, half = lane >> 5;
    const float inv_n = 1.0f / (64.0f * (float)g.sw);
    const int lsw = __builtin_ctz((unsigned)g.sw);  // sw is a power of two
    auto red = [&](float v) {
        for (int o = 1; o < 32; o <<= 1) v += __shfl_xor(v, o, 64);
        if (g.sw >= 8) v += __shfl_xor(v, 32, 64);
        return v;
    };
#pragma unroll
    for (int nb = 0; nb < NB; ++nb) {
        if (nb >= nvalid) break;
        // quad sums over e and mb; sub-slot of quad (j, half): (8 j + 4 half) / sw
        float qs[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            float t = 0.f;
#pragma unroll
            for (int mb = 0; mb < 2; ++mb)
#pragma unroll
                for (int e = 0; e < 4; ++e) t += acc[mb][nb][4 * j + e];
            qs[j] = t;
        }
        const int nsub = 32 >> lsw;  // sub-slots in the block: 8, 4, 2, 1
        float mean[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            // the lane's part of the sub-slot containing quad j: quads j' with (8 j' + 4 h) / sw equal
            const int s = (8 * j + 4 * half) >> lsw;
            float t = 0.f;
#pragma unroll
            for (int jj = 0; jj < 4; ++jj)
                if (((8 * jj + 4 * half) >> lsw) == s) t += qs[jj];
            mean[j] = red(t) * inv_n;
        }
        float q2[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            float t = 0.f;
#pragma unroll
            for (int mb = 0; mb < 2; ++mb)
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const float d = acc[mb][nb][4 * j + e] - mean[j];
                    t = fmaf(d, d, t);
                }
            q2[j] = t;
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int s = (8 * j + 4 * half) >> lsw;
            float t = 0.f;
#pragma unroll
            for (int jj = 0; jj < 4; ++jj)
                if (((8 * jj + 4 * half) >> lsw) == s) t += q2[jj];
            const float m2 = red(t);
            // one writer per sub-slot: lane 0 of the half owning its first quad, at its first j
            const bool first_j = ((8 * j + 4 * half) & (g.sw - 1)) == 0;
            if ((lane & 31) == 0 && first_j && s < nsub) {
                const long idx = ((g.pix64 * g.ncb + g.cb0 + nb) * nsub + s) * 2;
                g.part[idx] = mean[j];
                g.part[idx + 1] = m2;
            }
        }
    }
}

}  // namespace wcx6
