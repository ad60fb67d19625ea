// Self-attention backward on bf16x6 split-precision MFMA for gfx950 (head dims D % 32 == 0): the same
// contract and algorithm as wc_attention_bwd (wc_attention_bwd.hip) — the training backward of the
// softmax(QK^T*s)V core of nn.MultiheadAttention (reference unet_base.py:115,159 under
// train_ddpm.py:110) — with every product on v_mfma_f32_32x32x16_bf16 instead of fp32 MFMA.
//
// Arithmetic: each fp32 operand (Q, K, V, dO and the recomputed P and dS) is split exactly into three
// bf16 pieces (wcx6::split3, v = v0 + v1 + v2); the six products with i + j <= 2 accumulate in fp32.
// The dropped terms are < 3*2^-24 relative per product: fp32-class, no range bound needed (dO and dS
// have none).  A 32x32x16 block costs 6 x 32 cycles here against 8 x 64 on fp32 MFMA.
//
//   attn_bwd6_dkdv_kernel  a wave owns 32 keys (K, V rows in registers as bf16 pieces; D <= 128 — at
//       D = 192 the two-piece forms keep the V rows in LDS and split the output dims over workgroups,
//       the single-piece builds run the whole width in one); 32-query tiles of Q and dO are staged once
//       per tile as pieces in LDS ([piece][query][dim], shared by the 4 waves).
//         S = Q K^T, dP = dO V^T     rows = queries (A: ds_read_b128 from the tile), cols = keys (B: regs)
//         P, dS in the accumulator registers (lane = key, register r = query (r&3)+8(r>>2)+4 half)
//         dV^T += dO^T P, dK^T += Q^T dS   A: the tile read transposed (ds_read_b64_tr_b16) in the
//             query order the accumulator registers hold (per lane half: queries 4h+0..3, 8+4h+0..3 of
//             each 16-query chunk), B: the P / dS registers split in place.
//   attn_bwd6_dq_kernel    a wave owns 32 queries; 32-key tiles of K and V staged as pieces; S^T,
//       dP^T with lane = query, dQ^T += K^T dS^T.
// No atomics, fixed reduction order: deterministic.
//
// F3 = true (wc_attention_bwd_f16x3): the same kernels on f16x3 — every operand scaled by a power of
// two and split into two round-to-nearest fp16 pieces, products h*h + h*l + l*h on
// v_mfma_f32_32x32x16_f16 (3 MFMAs per block instead of 6).  The exponents come from range bounds:
// Q, K, V from the forward's in-projection bounds (eq, ek, ev: |Q| 2^eq <= 2^14 ...); dO from its
// per-image absmax (dobound[b], |dO| 2^edo < 2^14); P in [0, 1] at 2^14; dS = P (dP - D) with
// |dP_ij| = |dO_i . V_j| <= d max|dO| max|V| and |D_i| = |dO_i . O_i| <= d max|dO| max|V| (O is a
// convex combination of V rows), so |dS| < 2^(e_do + 2 + log2 d + 14 - ev) and
// eds = ev - e_do - 2 - log2 d puts it below 2^14 (e_do = floor(log2 max|dO|)).  Accumulators carry
// the products' power-of-two factors, removed exactly before use / in the epilogue.
#include "wc_x6.hpp"

namespace {

using namespace wcx6;

template <int D, bool F3 = false>
struct B6Cfg {
    static_assert(D % 32 == 0, "split-precision attention backward: D % 32 == 0");
    static constexpr int NP = F3 ? 2 : 3;   // operand pieces
    // pieces kept in LDS: the single-piece builds (WC_SINGLE16) never read the f16x3 low piece, so their
    // tiles hold the high piece only (half the LDS: two workgroups per CU at D = 128)
    static constexpr int NPS = F3 && WC_SINGLE16 ? 1 : NP;
    static constexpr int NCH = D / 16;      // 16-dim K-steps of S / dP
    static constexpr int NDB = D / 32;      // 32-dim output blocks
    static constexpr int RSB = 2 * D + 80;  // tile row bytes (odd multiple of 16: conflict-free b128 reads)
    static constexpr int PLANE = 32 * RSB;  // one piece of one 32-row tile
    static constexpr int TILE = NPS * PLANE; // the pieces
    static constexpr int STAGE = 2 * TILE + 2 * 32 * 4;  // two tiles (Q, dO or K, V) + lse / Dv
    static constexpr int LDS = 2 * STAGE;                // double-buffered: tile t + 1 staged under tile t
    static constexpr int IPT = D / 32;                   // float4 items per thread of one 32 x D tile
    // own rows kept as pieces (else fp32, split per use); the single-piece builds hold one piece, so
    // D = 192 rows fit as pieces there too (half the registers of the fp32 rows)
    static constexpr bool PRESPLIT = D <= 128 || NPS == 1;
    static constexpr int VROWB = NCH * NPS * 64 * 16;  // one wave's own rows as pieces in get() order (VL)
    static constexpr int LDS_VL = STAGE + 4 * VROWB;  // VL: one Q / dO stage + the four waves' V rows
};

// Split-precision pieces of 8 consecutive values as MFMA operands: three exact bf16 pieces, or (F3)
// two fp16 pieces of v * sc.
template <bool F3>
WC_DEVICE void pieces8(const float* v, float sc, u32x4 (&out)[F3 ? 2 : 3]);
template <>
WC_DEVICE void pieces8<true>(const float* v, float sc, u32x4 (&out)[2]) {
    u32x2 a0, a1, b0, b1;
    split2_f16(f32x4{v[0], v[1], v[2], v[3]} * sc, a0, a1);
    split2_f16(f32x4{v[4], v[5], v[6], v[7]} * sc, b0, b1);
    out[0] = u32x4{a0.x, a0.y, b0.x, b0.y};
    out[1] = u32x4{a1.x, a1.y, b1.x, b1.y};
}
template <>
WC_DEVICE void pieces8<false>(const float* v, float, u32x4 (&out)[3]) {
    u32x2 a0, a1, a2, b0, b1, b2;
    split3(f32x4{v[0], v[1], v[2], v[3]}, a0, a1, a2);
    split3(f32x4{v[4], v[5], v[6], v[7]}, b0, b1, b2);
    out[0] = u32x4{a0.x, a0.y, b0.x, b0.y};
    out[1] = u32x4{a1.x, a1.y, b1.x, b1.y};
    out[2] = u32x4{a2.x, a2.y, b2.x, b2.y};
}
template <bool F3>
WC_DEVICE void pieces8(const f32x16& v, int off, float sc, u32x4 (&out)[F3 ? 2 : 3]) {
    float t[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) t[j] = v[off + j];
    pieces8<F3>(t, sc, out);
}
WC_DEVICE void mfmaP(f32x16& acc, const u32x4 (&a)[2], const u32x4 (&b)[2]) {
    acc = mfma_f16(a[0], b[0], acc);
    acc = mfma_f16c(a[0], b[1], acc);
    acc = mfma_f16c(a[1], b[0], acc);
}

WC_DEVICE void mfmaP(f32x16& acc, const u32x4 (&a)[3], const u32x4 (&b)[3]) {
    acc = mfma_bf16(a[0], b[0], acc);
    acc = mfma_bf16(a[0], b[1], acc);
    acc = mfma_bf16(a[1], b[0], acc);
    acc = mfma_bf16(a[0], b[2], acc);
    acc = mfma_bf16(a[1], b[1], acc);
    acc = mfma_bf16(a[2], b[0], acc);
}

// A wave's own 32 rows (lane = row l32) of a [rows][D] fp32 matrix, the dims its lane half feeds:
// for K-step ch the lane holds dims 16 ch + 8 half .. + 7.  Kept either as bf16 pieces (PRESPLIT) or as
// fp32 values split per use.
template <int D, bool F3>
struct OwnRows {
    using Cf = B6Cfg<D, F3>;
    u32x4 pc[Cf::PRESPLIT ? Cf::NCH : 1][Cf::NP];
    float fv[Cf::PRESPLIT ? 1 : Cf::NCH * 8];
    float sc = 1.f;
    WC_DEVICE void load(const float* row, bool ok, int half, float scale) {
        sc = scale;
#pragma unroll
        for (int ch = 0; ch < Cf::NCH; ++ch) {
            float v[8];
            f32x4 a = f32x4{0.f, 0.f, 0.f, 0.f}, b = a;
            if (ok) {
                a = *reinterpret_cast<const f32x4*>(row + 16 * ch + 8 * half);
                b = *reinterpret_cast<const f32x4*>(row + 16 * ch + 8 * half + 4);
            }
            v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
            if constexpr (Cf::PRESPLIT) {
                pieces8<F3>(v, sc, pc[ch]);
            } else {
#pragma unroll
                for (int j = 0; j < 8; ++j) fv[8 * ch + j] = v[j];
            }
        }
    }
    WC_DEVICE void get(int ch, u32x4 (&out)[Cf::NP]) const {
        if constexpr (Cf::PRESPLIT) {
#pragma unroll
            for (int pp = 0; pp < Cf::NP; ++pp) out[pp] = pc[ch][pp];
        } else {
            pieces8<F3>(fv + 8 * ch, sc, out);
        }
    }
};

// A 32-row x D tile (rows r0.., fp32 rows at `base` with pitch ld, columns col..) staged into LDS as
// three bf16 piece planes [piece][row][dim] (row pitch RSB bytes); rows >= N are zero.  Split in two
// halves so the next tile's global loads are in flight while the current tile computes.
template <int D, bool F3>
struct TileStage {
    using Cf = B6Cfg<D, F3>;
    f32x4 v[Cf::IPT];
    WC_DEVICE void load(const float* base, long ld, int col, int r0, int N, int tid) {
#pragma unroll
        for (int j = 0; j < Cf::IPT; ++j) {
            const int i = tid + 256 * j;
            const int r = i / (D / 4), c4 = i % (D / 4);
            const int row = r0 + r;
            v[j] = f32x4{0.f, 0.f, 0.f, 0.f};
            if (row < N) v[j] = *reinterpret_cast<const f32x4*>(base + (long)row * ld + col + 4 * c4);
        }
    }
    WC_DEVICE void store(unsigned char* dst, int tid, float sc) const {
#pragma unroll
        for (int j = 0; j < Cf::IPT; ++j) {
            const int i = tid + 256 * j;
            const int r = i / (D / 4), c4 = i % (D / 4);
            unsigned char* d = dst + r * Cf::RSB + c4 * 8;
            if constexpr (F3) {
                u32x2 h, l;
                split2_f16(v[j] * sc, h, l);
                *reinterpret_cast<u32x2*>(d) = h;
                if constexpr (Cf::NPS > 1) *reinterpret_cast<u32x2*>(d + Cf::PLANE) = l;
            } else {
                u32x2 p0, p1, p2;
                split3(v[j], p0, p1, p2);
                *reinterpret_cast<u32x2*>(d) = p0;
                *reinterpret_cast<u32x2*>(d + Cf::PLANE) = p1;
                *reinterpret_cast<u32x2*>(d + 2 * Cf::PLANE) = p2;
            }
        }
    }
};

// A operand rows = tile rows (lane = row l32), K-step ch: 8 dims per lane half (ds_read_b128).
template <int D, bool F3>
WC_DEVICE void tile_rows(const unsigned char* tile, int l32, int half, int ch, u32x4 (&out)[F3 ? 2 : 3]) {
    using Cf = B6Cfg<D, F3>;
    const unsigned char* p = tile + l32 * Cf::RSB + (16 * ch + 8 * half) * 2;
#pragma unroll
    for (int pc = 0; pc < Cf::NP; ++pc)
        out[pc] = pc < Cf::NPS ? *reinterpret_cast<const u32x4*>(p + pc * Cf::PLANE) : u32x4{0u, 0u, 0u, 0u};
}

// A operand = tile^T (rows = the 32 dims of block db, K = 16 tile rows of chunk c) in the row order
// of the accumulator registers: lane half h gets rows 16c + 4h + 0..3 and 16c + 8 + 4h + 0..3
// (ds_read_b64_tr_b16: lane 16g + 4q + p supplies row base + q, dims 16(g & 1) + 4p .. + 3; the lane
// receives dim l32 of the 4 rows its 16-lane group supplied).
template <int D, bool F3>
WC_DEVICE void tile_cols(const unsigned char* tile, int lane, int db, int c, u32x4 (&out)[F3 ? 2 : 3]) {
    using Cf = B6Cfg<D, F3>;
    const int g = lane >> 4, q = (lane & 15) >> 2, p = lane & 3;
    const int row = 16 * c + 4 * (g >> 1) + q;
    const unsigned char* base = tile + row * Cf::RSB + (32 * db + 16 * (g & 1) + 4 * p) * 2;
    typedef short v4s __attribute__((ext_vector_type(4)));
#pragma unroll
    for (int pc = 0; pc < Cf::NP; ++pc) {
        if (pc >= Cf::NPS) {
            out[pc] = u32x4{0u, 0u, 0u, 0u};
            continue;
        }
        const unsigned char* a = base + pc * Cf::PLANE;
        const v4s lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4s*)(a));
        const v4s hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4s*)(a + 8 * Cf::RSB));
        const u32x2 l2 = __builtin_bit_cast(u32x2, lo), h2 = __builtin_bit_cast(u32x2, hi);
        out[pc] = u32x4{l2.x, l2.y, h2.x, h2.y};
    }
}

// Per-image power-of-two factors of the F3 operands (all 1 for bf16x6).
struct BwdScales {
    float sq = 1.f, sk = 1.f, sv = 1.f, sdo = 1.f, sds = 1.f, sp = 1.f;
    int eq = 0, ek = 0, ev = 0, edo = 0, eds = 0, ep = 0;
};
template <int D, bool F3>
WC_DEVICE BwdScales bwd_scales(int eq, int ek, int ev, const float* dobound, int b) {
    BwdScales r;
    if constexpr (F3) {
        constexpr int LOGD = D == 32 ? 5 : D == 64 ? 6 : D == 128 ? 7 : 8;
        const float m = dobound[b];
        int edo = 60, eds = 60;
        if (m > 0.f) {
            const int e = (int)((__float_as_uint(m) >> 23) & 0xffu) - 127;  // floor(log2 max|dO|)
            edo = min(60, 13 - e);
            eds = min(60, ev - e - 2 - LOGD);
        }
        r.eq = eq; r.ek = ek; r.ev = ev; r.edo = max(edo, -100); r.eds = max(eds, -100); r.ep = 14;
        r.sq = ldexpf(1.f, eq); r.sk = ldexpf(1.f, ek); r.sv = ldexpf(1.f, ev);
        r.sdo = ldexpf(1.f, r.edo); r.sds = ldexpf(1.f, r.eds); r.sp = 16384.f;
    }
    return r;
}

// DS: the output dims split over DS workgroups (each computes S and dP in full, and dK / dV — or dQ —
// for D / DS of the dims): at D = 192 the whole width does not fit one wave's registers.
// VL: the wave's own V rows live in LDS as pieces in the order the MFMAs read them ([K-step][piece]
// [lane] 16-byte fragments, one ds_read_b128 each, conflict-free) instead of registers, and the Q / dO
// tiles are single-staged to make room (the next tile's global loads still fly under the MFMAs): at
// D = 192 the K and V rows together would take 192 registers and the kernel spilled.
template <int D, bool F3, int DS = 1, bool VL = false>
__global__ __launch_bounds__(256, F3 && WC_SINGLE16 && D <= 64 ? 2 : 1) void attn_bwd6_dkdv_kernel(
    const float* __restrict__ qkv, int ldq, const float* __restrict__ dO, int lddo, const float* __restrict__ lse,
    const float* __restrict__ Dv, float* __restrict__ dqkv, int lddq, int N, int C, float scale_log2, float scale,
    int eq, int ek, int ev, const float* __restrict__ dobound, float* __restrict__ amx) {
    using Cf = B6Cfg<D, F3>;
    constexpr int NP = Cf::NP;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];  // 2 stages: Q, dO tiles, lse, Dv

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int l32 = lane & 31, half = lane >> 5;
    const int head = blockIdx.y, b = blockIdx.z, H = gridDim.y;
    const float* base = qkv + (long)b * N * ldq;
    const float* dob = dO + (long)b * N * lddo;
    const int qcol = head * D, kcol = C + head * D, vcol = 2 * C + head * D;
    constexpr int NDBP = Cf::NDB / DS;  // output blocks of this workgroup
    static_assert(Cf::NDB % DS == 0, "DS divides the 32-dim output blocks");
    const int db0 = (int)(blockIdx.x % DS) * NDBP;
    const int key = (int)(blockIdx.x / DS) * 128 + wave * 32 + l32;
    const BwdScales sc = bwd_scales<D, F3>(eq, ek, ev, dobound, b);
    const float s_log2 = scale_log2 * ldexpf(1.f, -(sc.eq + sc.ek));  // S carries 2^(eq + ek)
    const float dp_un = ldexpf(1.f, -(sc.edo + sc.ev));               // dP carries 2^(edo + ev)

    OwnRows<D, F3> kr, vr;
    kr.load(base + (long)key * ldq + kcol, key < N, half, sc.sk);
    constexpr int NSTAGE = VL ? 1 : 2;
    unsigned char* vls = smem + NSTAGE * Cf::STAGE + wave * Cf::VROWB;
    if constexpr (VL) {
        const float* row = base + (long)key * ldq + vcol;
#pragma unroll
        for (int ch = 0; ch < Cf::NCH; ++ch) {
            float v[8];
            f32x4 a = f32x4{0.f, 0.f, 0.f, 0.f}, c = a;
            if (key < N) {
                a = *reinterpret_cast<const f32x4*>(row + 16 * ch + 8 * half);
                c = *reinterpret_cast<const f32x4*>(row + 16 * ch + 8 * half + 4);
            }
            v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = c.x; v[5] = c.y; v[6] = c.z; v[7] = c.w;
            u32x4 pc[NP];
            pieces8<F3>(v, sc.sv, pc);
#pragma unroll
            for (int pp = 0; pp < Cf::NPS; ++pp) *reinterpret_cast<u32x4*>(vls + ((ch * Cf::NPS + pp) * 64 + lane) * 16) = pc[pp];
        }
    } else {
        vr.load(base + (long)key * ldq + vcol, key < N, half, sc.sv);
    }

    f32x16 dvT[NDBP], dkT[NDBP];
#pragma unroll
    for (int d = 0; d < NDBP; ++d)
#pragma unroll
        for (int r = 0; r < 16; ++r) { dvT[d][r] = 0.f; dkT[d][r] = 0.f; }

    const int ntiles = (N + 31) / 32;
    TileStage<D, F3> sq, so;
    float rl = INFINITY, rdv = 0.f;
    auto gload = [&](int t) {
        const int q0 = t * 32;
        sq.load(base, ldq, qcol, q0, N, tid);
        so.load(dob, lddo, head * D, q0, N, tid);
        if (tid < 32) {
            const int q = q0 + tid;
            rl = q < N ? lse[((long)b * H + head) * N + q] : INFINITY;  // P = 0 for padding queries
            rdv = q < N ? Dv[((long)b * H + head) * N + q] : 0.f;
        }
    };
    auto swrite = [&](int buf) {
        unsigned char* st = smem + buf * Cf::STAGE;
        sq.store(st, tid, sc.sq);
        so.store(st + Cf::TILE, tid, sc.sdo);
        if (tid < 32) {
            float* l = reinterpret_cast<float*>(st + 2 * Cf::TILE);
            l[tid] = rl;
            l[32 + tid] = rdv;
        }
    };
    gload(0);
    swrite(0);
    __syncthreads();
    for (int t = 0; t < ntiles; ++t) {
        unsigned char* Qs = smem + (NSTAGE == 2 ? (t & 1) : 0) * Cf::STAGE;
        unsigned char* Os = Qs + Cf::TILE;
        const float* Ls = reinterpret_cast<const float*>(Qs + 2 * Cf::TILE);
        if (t + 1 < ntiles) gload(t + 1);  // in flight under this tile's MFMAs
        // S = Q K^T, dP = dO V^T: rows = queries, lane = key
        f32x16 s, dp;
#pragma unroll
        for (int r = 0; r < 16; ++r) { s[r] = 0.f; dp[r] = 0.f; }
#pragma unroll
        for (int ch = 0; ch < Cf::NCH; ++ch) {
            u32x4 a[NP], bk[NP];
            tile_rows<D, F3>(Qs, l32, half, ch, a);
            kr.get(ch, bk);
            mfmaP(s, a, bk);
            tile_rows<D, F3>(Os, l32, half, ch, a);
            if constexpr (VL) {
#pragma unroll
                for (int pp = 0; pp < NP; ++pp)
                    bk[pp] = pp < Cf::NPS ? *reinterpret_cast<const u32x4*>(vls + ((ch * Cf::NPS + pp) * 64 + lane) * 16)
                                          : u32x4{0u, 0u, 0u, 0u};
            } else {
                vr.get(ch, bk);
            }
            mfmaP(dp, a, bk);
        }
        // P and dS in place (register r <-> query (r&3) + 8(r>>2) + 4 half of the tile)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int qi = (r & 3) + 8 * (r >> 2) + 4 * half;
            // one fma + v_exp_f32 (results below 2^-126 flush to 0: negligible, as the forward)
            const float pr = __builtin_amdgcn_exp2f(fmaf(s[r], s_log2, -Ls[qi]));
            s[r] = pr;
            dp[r] = pr * (F3 ? dp[r] * dp_un - Ls[32 + qi] : dp[r] - Ls[32 + qi]);
        }
        // dV^T += dO^T P, dK^T += Q^T dS over the two 16-query chunks
#pragma unroll
        for (int c = 0; c < 2; ++c) {
            u32x4 pp[NP], ds[NP];
            pieces8<F3>(s, 8 * c, sc.sp, pp);
            pieces8<F3>(dp, 8 * c, sc.sds, ds);
#pragma unroll
            for (int db = 0; db < NDBP; ++db) {
                u32x4 a[NP];
                tile_cols<D, F3>(Os, lane, db0 + db, c, a);
                mfmaP(dvT[db], a, pp);
                tile_cols<D, F3>(Qs, lane, db0 + db, c, a);
                mfmaP(dkT[db], a, ds);
            }
        }
        if constexpr (NSTAGE == 2) {
            if (t + 1 < ntiles) swrite((t + 1) & 1);  // the other stage: last read in tile t - 1
        } else if (t + 1 < ntiles) {
            __syncthreads();  // every wave is done with the single stage
            swrite(0);
        }
        __syncthreads();
    }

    float vmax = 0.f;
    if (key < N) {
        const float kun = scale * ldexpf(1.f, -(sc.eq + sc.eds)), vun = ldexpf(1.f, -(sc.edo + sc.ep));
        float* row = dqkv + ((long)b * N + key) * lddq;
#pragma unroll
        for (int d = 0; d < NDBP; ++d) {
#pragma unroll
            for (int r = 0; r < 16; r += 4) {
                const int dv = (db0 + d) * 32 + 8 * (r >> 2) + 4 * half;
                const f32x4 kk = f32x4{dkT[d][r], dkT[d][r + 1], dkT[d][r + 2], dkT[d][r + 3]} * kun;
                const f32x4 vv0 = f32x4{dvT[d][r], dvT[d][r + 1], dvT[d][r + 2], dvT[d][r + 3]};
                const f32x4 vv = F3 ? vv0 * vun : vv0;
                *reinterpret_cast<f32x4*>(row + kcol + dv) = kk;
                *reinterpret_cast<f32x4*>(row + vcol + dv) = vv;
                vmax = fmaxf(vmax, fmaxf(fmaxf(fmaxf(fabsf(kk.x), fabsf(kk.y)), fmaxf(fabsf(kk.z), fabsf(kk.w))),
                                         fmaxf(fmaxf(fabsf(vv.x), fabsf(vv.y)), fmaxf(fabsf(vv.z), fabsf(vv.w)))));
            }
        }
    }
    if (amx) block_absmax_atomic(amx, b, vmax);  // the workgroup is one image
}

template <int D, bool F3, int DS = 1>
__global__ __launch_bounds__(256, F3 && WC_SINGLE16 && D <= 128 ? 2 : 1) void attn_bwd6_dq_kernel(
    const float* __restrict__ qkv, int ldq, const float* __restrict__ dO, int lddo, const float* __restrict__ lse,
    const float* __restrict__ Dv, float* __restrict__ dqkv, int lddq, int N, int C, float scale_log2, float scale,
    int eq, int ek, int ev, const float* __restrict__ dobound, float* __restrict__ amx) {
    using Cf = B6Cfg<D, F3>;
    constexpr int NP = Cf::NP;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];  // 2 stages: K, V tiles

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int l32 = lane & 31, half = lane >> 5;
    const int head = blockIdx.y, b = blockIdx.z, H = gridDim.y;
    const float* base = qkv + (long)b * N * ldq;
    const float* dob = dO + (long)b * N * lddo;
    const int qcol = head * D, kcol = C + head * D, vcol = 2 * C + head * D;
    constexpr int NDBP = Cf::NDB / DS;
    static_assert(Cf::NDB % DS == 0, "DS divides the 32-dim output blocks");
    const int db0 = (int)(blockIdx.x % DS) * NDBP;
    const int qme = (int)(blockIdx.x / DS) * 128 + wave * 32 + l32;
    const BwdScales sc = bwd_scales<D, F3>(eq, ek, ev, dobound, b);
    const float s_log2 = scale_log2 * ldexpf(1.f, -(sc.eq + sc.ek));
    const float dp_un = ldexpf(1.f, -(sc.edo + sc.ev));

    OwnRows<D, F3> qr, orr;
    qr.load(base + (long)qme * ldq + qcol, qme < N, half, sc.sq);
    orr.load(dob + (long)qme * lddo + head * D, qme < N, half, sc.sdo);
    const float lq = qme < N ? lse[((long)b * H + head) * N + qme] : INFINITY;
    const float dq = qme < N ? Dv[((long)b * H + head) * N + qme] : 0.f;

    f32x16 dqT[NDBP];
#pragma unroll
    for (int d = 0; d < NDBP; ++d)
#pragma unroll
        for (int r = 0; r < 16; ++r) dqT[d][r] = 0.f;

    const int ntiles = (N + 31) / 32;
    TileStage<D, F3> sk, sv;
    auto gload = [&](int t) {
        sk.load(base, ldq, kcol, t * 32, N, tid);
        sv.load(base, ldq, vcol, t * 32, N, tid);
    };
    auto swrite = [&](int buf) {
        unsigned char* st = smem + buf * Cf::STAGE;
        sk.store(st, tid, sc.sk);
        sv.store(st + Cf::TILE, tid, sc.sv);
    };
    gload(0);
    swrite(0);
    __syncthreads();
    for (int t = 0; t < ntiles; ++t) {
        const int k0 = t * 32;
        unsigned char* Ks = smem + (t & 1) * Cf::STAGE;
        unsigned char* Vs = Ks + Cf::TILE;
        if (t + 1 < ntiles) gload(t + 1);  // in flight under this tile's MFMAs
        // S^T = K Q^T, dP^T = V dO^T: rows = keys, lane = query
        f32x16 s, dp;
#pragma unroll
        for (int r = 0; r < 16; ++r) { s[r] = 0.f; dp[r] = 0.f; }
#pragma unroll
        for (int ch = 0; ch < Cf::NCH; ++ch) {
            u32x4 a[NP], bq[NP];
            tile_rows<D, F3>(Ks, l32, half, ch, a);
            qr.get(ch, bq);
            mfmaP(s, a, bq);
            tile_rows<D, F3>(Vs, l32, half, ch, a);
            orr.get(ch, bq);
            mfmaP(dp, a, bq);
        }
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int key = k0 + (r & 3) + 8 * (r >> 2) + 4 * half;
            const float pr = key < N ? __builtin_amdgcn_exp2f(fmaf(s[r], s_log2, -lq)) : 0.f;
            dp[r] = pr * (F3 ? dp[r] * dp_un - dq : dp[r] - dq);
        }
        // dQ^T += K^T dS^T
#pragma unroll
        for (int c = 0; c < 2; ++c) {
            u32x4 ds[NP];
            pieces8<F3>(dp, 8 * c, sc.sds, ds);
#pragma unroll
            for (int db = 0; db < NDBP; ++db) {
                u32x4 a[NP];
                tile_cols<D, F3>(Ks, lane, db0 + db, c, a);
                mfmaP(dqT[db], a, ds);
            }
        }
        if (t + 1 < ntiles) swrite((t + 1) & 1);
        __syncthreads();
    }

    float vmax = 0.f;
    if (qme < N) {
        const float qun = scale * ldexpf(1.f, -(sc.ek + sc.eds));
        float* row = dqkv + ((long)b * N + qme) * lddq + qcol;
#pragma unroll
        for (int d = 0; d < NDBP; ++d) {
#pragma unroll
            for (int r = 0; r < 16; r += 4) {
                const int dv = (db0 + d) * 32 + 8 * (r >> 2) + 4 * half;
                const f32x4 qq = f32x4{dqT[d][r], dqT[d][r + 1], dqT[d][r + 2], dqT[d][r + 3]} * qun;
                *reinterpret_cast<f32x4*>(row + dv) = qq;
                vmax = fmaxf(vmax, fmaxf(fmaxf(fabsf(qq.x), fabsf(qq.y)), fmaxf(fabsf(qq.z), fabsf(qq.w))));
            }
        }
    }
    if (amx) block_absmax_atomic(amx, b, vmax);
}

template <int D, bool F3, int DS = 1>
int launch_bwd6(const float* qkv, int ldq, const float* dO, int lddo, const float* lse, const float* Dv, float* dqkv,
                int lddq, int B, int N, int C, int heads, float scale, int eq, int ek, int ev, const float* dobound,
                float* amx, hipStream_t s) {
    using Cf = B6Cfg<D, F3>;
    static bool attr_set = false;
    if (!attr_set) {
        hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&attn_bwd6_dkdv_kernel<D, F3, DS>),
                                           hipFuncAttributeMaxDynamicSharedMemorySize, Cf::LDS);
        if (e != hipSuccess) return (int)e;
        e = hipFuncSetAttribute(reinterpret_cast<const void*>(&attn_bwd6_dq_kernel<D, F3, DS>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, Cf::LDS);
        if (e != hipSuccess) return (int)e;
        attr_set = true;
    }
    const dim3 grid((N + 127) / 128 * DS, heads, B);
    const float scale_log2 = scale * 1.4426950408889634f;
    WC_SET_NAME("attn_bwd6_dkdv_kernel", {WC_TI(D), WC_TB(F3), WC_TI(DS)});
    hipLaunchKernelGGL((attn_bwd6_dkdv_kernel<D, F3, DS>), grid, dim3(256), Cf::LDS, s, qkv, ldq, dO, lddo, lse, Dv, dqkv,
                       lddq, N, C, scale_log2, scale, eq, ek, ev, dobound, amx);
    WC_CHECK_LAUNCH();
    WC_SET_NAME("attn_bwd6_dq_kernel", {WC_TI(D), WC_TB(F3), WC_TI(DS)});
    hipLaunchKernelGGL((attn_bwd6_dq_kernel<D, F3, DS>), grid, dim3(256), Cf::LDS, s, qkv, ldq, dO, lddo, lse, Dv, dqkv,
                       lddq, N, C, scale_log2, scale, eq, ek, ev, dobound, amx);
    WC_CHECK_LAUNCH();
    return WC_OK;
}

}  // namespace

// Dv[b][h][q] = sum_d dO O over the head (wc_attention_bwd's prep step) must already be in dv_work
// (wc_attention_bwd6 runs it itself through wc_attention_bwd_prep).
extern "C" int wc_attention_bwd_prep(const float* out, int ld_out, const float* dout, int ld_dout, int B, int N,
                                     int heads, int D, float* dv_work, void* stream);
extern "C" int wc_attention_bwd_dkdv192(const float* qkv, int ld_qkv, const float* dout, int ld_dout, const float* lse,
                                        const float* dv_work, float* dqkv, int ld_dqkv, int B, int N, int C,
                                        int heads, float scale, void* stream);

// the D = 192 dK / dV kernel with V rows in LDS, output dims in DS parts (2: no spills, S and dP computed
// twice; 1: computed once, 216 bytes of scratch per lane; WC_DKDV192_DS selects, default 2)
template <int DS>
int launch_dkdv192(const float* qkv, int ld_qkv, const float* dout, int ld_dout, const float* lse, const float* dv_work,
                   float* dqkv, int ld_dqkv, int B, int N, int C, int heads, float scale, int eq, int ek, int ev,
                   const float* dobound, float* amx, hipStream_t s) {
    using Cf = B6Cfg<192, true>;
    static bool attr_set = false;
    if (!attr_set) {
        hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&attn_bwd6_dkdv_kernel<192, true, DS, true>),
                                           hipFuncAttributeMaxDynamicSharedMemorySize, Cf::LDS_VL);
        if (e != hipSuccess) return (int)e;
        attr_set = true;
    }
    WC_SET_NAME("attn_bwd6_dkdv_kernel", {WC_TI(192), WC_TB(true), WC_TI(DS), WC_TB(true)});
    hipLaunchKernelGGL((attn_bwd6_dkdv_kernel<192, true, DS, true>), dim3((N + 127) / 128 * DS, heads, B), dim3(256),
                       Cf::LDS_VL, s, qkv, ld_qkv, dout, ld_dout, lse, dv_work, dqkv, ld_dqkv, N, C,
                       scale * 1.4426950408889634f, scale, eq, ek, ev, dobound, amx);
    WC_CHECK_LAUNCH();
    return WC_OK;
}

static int attention_bwd_split(const float* qkv, int ld_qkv, const float* out, int ld_out, const float* dout,
                               int ld_dout, const float* lse, float* dv_work, float* dqkv, int ld_dqkv, int B, int N,
                               int C, int heads, float scale, bool f3, int eq, int ek, int ev, const float* dobound,
                               float* amx, void* stream) {
    if (!qkv || !out || !dout || !lse || !dv_work || !dqkv || (f3 && !dobound)) return WC_E_ARG;
    if (heads <= 0 || C % heads || B <= 0 || N <= 0) return WC_E_SHAPE;
    if (ld_qkv % 4 || ld_out % 4 || ld_dout % 4 || ld_dqkv % 4 || ld_qkv < 3 * C || ld_dqkv < 3 * C || ld_out < C ||
        ld_dout < C)
        return WC_E_SHAPE;
    if ((reinterpret_cast<uintptr_t>(qkv) | reinterpret_cast<uintptr_t>(dout) | reinterpret_cast<uintptr_t>(dqkv)) & 15)
        return WC_E_SHAPE;
    if (f3 && (eq < -60 || eq > 60 || ek < -60 || ek > 60 || ev < -60 || ev > 60)) return WC_E_ARG;
    const int D = C / heads;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    int st = wc_attention_bwd_prep(out, ld_out, dout, ld_dout, B, N, heads, D, dv_work, stream);
    if (st != WC_OK) return st;
#define WC_BWD6(DD)                                                                                                    \
    (f3 ? launch_bwd6<DD, true>(qkv, ld_qkv, dout, ld_dout, lse, dv_work, dqkv, ld_dqkv, B, N, C, heads, scale, eq, ek, \
                                ev, dobound, amx, s)                                                                   \
        : launch_bwd6<DD, false>(qkv, ld_qkv, dout, ld_dout, lse, dv_work, dqkv, ld_dqkv, B, N, C, heads, scale, 0, 0, \
                                 0, nullptr, amx, s))
    switch (D) {
        case 32: return WC_BWD6(32);
        case 64: return WC_BWD6(64);
        case 128: return WC_BWD6(128);
        case 192: {
            // f16x3 only: dQ with the output dims in three parts (its own Q / dO rows fit at a third of
            // the accumulators); dK / dV with the V rows in LDS (VL, launch_dkdv192), or
            // (no dqkv_absmax: the caller asked for the fp32-MFMA kernel, which raises no bound) on fp32 MFMA
            if (!f3) return WC_E_SHAPE;
            using Cf = B6Cfg<192, true>;
            const bool fp32_dkdv = amx == nullptr;
#if WC_SINGLE16
            // single-piece builds: one piece per row and tile, so the whole width fits one wave (rows as
            // pieces; dK / dV with the V rows in LDS): no output split, S and dP computed once per kernel
            // instead of 2 (dK / dV) and 3 (dQ) times
            if (!fp32_dkdv) {
                st = launch_dkdv192<1>(qkv, ld_qkv, dout, ld_dout, lse, dv_work, dqkv, ld_dqkv, B, N, C, heads, scale, eq,
                                       ek, ev, dobound, amx, s);
                if (st != WC_OK) return st;
                static bool attr1 = false;
                if (!attr1) {
                    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&attn_bwd6_dq_kernel<192, true, 1>),
                                                       hipFuncAttributeMaxDynamicSharedMemorySize, Cf::LDS);
                    if (e != hipSuccess) return (int)e;
                    attr1 = true;
                }
                WC_SET_NAME("attn_bwd6_dq_kernel", {WC_TI(192), WC_TB(true), WC_TI(1)});
                hipLaunchKernelGGL((attn_bwd6_dq_kernel<192, true, 1>), dim3((N + 127) / 128, heads, B), dim3(256), Cf::LDS,
                                   s, qkv, ld_qkv, dout, ld_dout, lse, dv_work, dqkv, ld_dqkv, N, C,
                                   scale * 1.4426950408889634f, scale, eq, ek, ev, dobound, amx);
                WC_CHECK_LAUNCH();
                return WC_OK;
            }
#endif
            if (fp32_dkdv) {
                st = wc_attention_bwd_dkdv192(qkv, ld_qkv, dout, ld_dout, lse, dv_work, dqkv, ld_dqkv, B, N, C, heads,
                                              scale, stream);
                if (st != WC_OK) return st;
            }
            static bool attr_set = false;
            if (!attr_set) {
                hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&attn_bwd6_dq_kernel<192, true, 3>),
                                                   hipFuncAttributeMaxDynamicSharedMemorySize, Cf::LDS);
                if (e != hipSuccess) return (int)e;
                attr_set = true;
            }
            const float scale_log2 = scale * 1.4426950408889634f;
            if (!fp32_dkdv) {
                // output dims in two workgroups (DS = 2: no scratch; one workgroup spilled 216 B/lane and
                // was no faster, removed)
                st = launch_dkdv192<2>(qkv, ld_qkv, dout, ld_dout, lse, dv_work, dqkv, ld_dqkv, B, N, C, heads, scale,
                                       eq, ek, ev, dobound, amx, s);
                if (st != WC_OK) return st;
            }
            WC_SET_NAME("attn_bwd6_dq_kernel", {WC_TI(192), WC_TB(true), WC_TI(3)});
            hipLaunchKernelGGL((attn_bwd6_dq_kernel<192, true, 3>), dim3((N + 127) / 128 * 3, heads, B), dim3(256),
                               Cf::LDS, s, qkv, ld_qkv, dout, ld_dout, lse, dv_work, dqkv, ld_dqkv, N, C, scale_log2,
                               scale, eq, ek, ev, dobound, fp32_dkdv ? nullptr : amx);
            WC_CHECK_LAUNCH();
            return WC_OK;
        }
        default: return WC_E_SHAPE;
    }
#undef WC_BWD6
}

extern "C" int wc_attention_bwd6(const float* qkv, int ld_qkv, const float* out, int ld_out, const float* dout,
                                 int ld_dout, const float* lse, float* dv_work, float* dqkv, int ld_dqkv, int B, int N,
                                 int C, int heads, float scale, void* stream) {
    return attention_bwd_split(qkv, ld_qkv, out, ld_out, dout, ld_dout, lse, dv_work, dqkv, ld_dqkv, B, N, C, heads,
                               scale, false, 0, 0, 0, nullptr, nullptr, stream);
}

// f16x3 form: eq / ek / ev the forward's exponents of Q, K, V (|Q| 2^eq <= 2^14 ...), dobound[B] the
// per-image max |dO| (device memory); dqkv_absmax (optional, [B]) raised to the max |dqkv| written.
extern "C" int wc_attention_bwd_f16x3(const float* qkv, int ld_qkv, const float* out, int ld_out, const float* dout,
                                      int ld_dout, const float* lse, float* dv_work, float* dqkv, int ld_dqkv, int B,
                                      int N, int C, int heads, float scale, int eq, int ek, int ev,
                                      const float* dobound, float* dqkv_absmax, void* stream) {
    return attention_bwd_split(qkv, ld_qkv, out, ld_out, dout, ld_dout, lse, dv_work, dqkv, ld_dqkv, B, N, C, heads,
                               scale, true, eq, ek, ev, dobound, dqkv_absmax, stream);
}
