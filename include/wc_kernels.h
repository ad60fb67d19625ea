/*
 * wc_kernels.h — C ABI of the WeatherConverter MI355X (gfx950) hot-path kernels.
 *
 * The reference (xXCoffeeColaXc/WeatherConverter, 100 % Python) has no FFI of its own: its hot
 * path is PyTorch eager ops called from the Python API listed in SURVEY.md §8(b).  Each entry
 * point below replaces a group of those eager ops; the reference call site it stands in for is
 * cited per function.  The Python drop-in layer (weatherconverter_amd/) binds these through ctypes
 * (see INTEGRATION.md).
 *
 * Conventions
 *  - All tensors are caller-owned device memory (torch storage).  Nothing here allocates or frees.
 *  - Activations are NHWC fp32 "views": (ptr, C, ldc) where ldc >= C is the per-pixel stride in
 *    floats, so channel slices of a wider buffer (the UNet skip concat) are addressed in place.
 *  - Every function is asynchronous on the given hipStream_t (passed as void*) and never syncs.
 *  - Return 0 on success, a positive hipError_t on a launch error, or a negative WC_E_* code when
 *    a shape is outside what the kernel supports (the Python layer raises RuntimeError; there is
 *    no silent fallback).
 */
#ifndef WC_KERNELS_H
#define WC_KERNELS_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define WC_OK 0
#define WC_E_SHAPE (-1)   /* unsupported shape / alignment */
#define WC_E_ARG (-2)     /* null pointer or bad enum */

/* ------------------------------------------------------------------------------------------ */
/* Implicit-GEMM convolution on fp32 MFMA (v_mfma_f32_32x32x2_f32).                            */
/* ------------------------------------------------------------------------------------------ */

#define WC_MAX_TAPS 16

/* One K-segment of the implicit GEMM: a source view read through `ntaps` spatial taps.  The K
 * index of the packed weight is (kbase + tap * C + c). */
typedef struct wc_conv_seg {
    const float* src;   /* NHWC view base (already offset to its first channel) */
    int C;              /* channels read from this view (multiple of 32) */
    int ldc;            /* pixel stride of the view, floats */
    int H, W;           /* spatial extent of the source */
    int sy, sx;         /* stride of the input sampling grid */
    int ntaps;          /* 1..WC_MAX_TAPS */
    int dy[WC_MAX_TAPS];
    int dx[WC_MAX_TAPS];
    /* Optional fused GroupNorm-apply prologue: v = v*scale[b*C+c] + shift[b*C+c]; NULL = none. */
    const float* scale;
    const float* shift;
    int silu;           /* apply SiLU after the affine (only meaningful with scale/shift) */
    int kbase;          /* first K column of this segment in the packed weight */
} wc_conv_seg;

typedef struct wc_conv_args {
    wc_conv_seg seg[2];
    int nseg;
    /* GEMM grid: M = B*Hm*Wm output positions, N output channels. */
    int B, Hm, Wm;
    int N;
    const float* w;     /* packed weight [N][ldw] with K contiguous */
    int ldw;
    const float* bias;  /* [N] or NULL */
    const float* temb;  /* per-(batch, n) add, temb[b*temb_ld + n]; temb_ld = 0 broadcasts */
    int temb_ld;
    const float* res;   /* residual view added in the epilogue (same spatial map as out) or NULL */
    int ldres;
    float* out;         /* output view */
    int ldo;
    int Ho, Wo;         /* output spatial extent */
    int osy, osx, ooy, oox; /* output position = (my*osy + ooy, mx*osx + oox) */
    int out_nchw;       /* 1: write out[(b*N + n)*Ho*Wo + oy*Wo + ox] (ldo ignored) */
    int act;            /* epilogue activation after bias/temb, before the residual add:
                           WC_ACT_NONE / WC_ACT_GELU (exact erf) / WC_ACT_SILU / WC_ACT_PRELU /
                           WC_ACT_TANH01; wc_conv_igemm accepts an activation only with a raw
                           segment 0 (no scale/shift) */
    float* absmax_out;  /* optional, per image [B] (caller-zeroed): atomically raised to max |out| of
                           the image's written values (a bound for a later f16x3 consumer);
                           split-precision kernels only (the fp32 kernel returns WC_E_ARG) */
    const float* act_param; /* WC_ACT_PRELU: per-output-channel slopes [N] (else ignored) */
    /* Optional GroupNorm tile partials of the output (split-precision kernels; see wc_gn_partials):
     * the written channels are [gn_c0, gn_c0 + N) of a tensor with gn_ncb*32 channels; the output
     * rows are pixel blocks gn_p64 .. of the tensor's gn_np64 blocks of 64 per image. */
    float* gn_part;
    int gn_ncb, gn_sw, gn_c0, gn_p64, gn_np64;
} wc_conv_args;

#define WC_ACT_NONE 0
#define WC_ACT_GELU 1
#define WC_ACT_SILU 2
#define WC_ACT_PRELU 3  /* v >= 0 ? v : act_param[n] * v (nn.PReLU(num_parameters=N)); fp32 kernel only */
#define WC_ACT_TANH01 4 /* (tanh(v) + 1) / 2 (Swift-SRGAN output, srgan_model/models.py:92); fp32 only */

/* Replaces: nn.Conv2d 3x3/1x1/4x4-s2 and nn.ConvTranspose2d (per output parity), the GN+SiLU
 * prologue of nn.Sequential(GroupNorm, SiLU, Conv2d), the temb broadcast add, the 1x1
 * residual_input_conv and the residual add — unet_base.py:87-109,123-129,146-150,333-334,348
 * and the attention in/out projections of nn.MultiheadAttention (unet_base.py:115,159). */
int wc_conv_igemm(const wc_conv_args* args, void* stream);

/* ------------------------------------------------------------------------------------------ */
/* 3x3 stride-1 convolution on bf16x6 split-precision MFMA (v_mfma_f32_32x32x16_bf16).         */
/* ------------------------------------------------------------------------------------------ */

/* Every fp32 operand is split exactly into three bf16 pieces by truncation (v = v0 + v1 + v2,
 * 8 significant bits each) and the products v_i*w_j with i + j <= 2 are accumulated in fp32.
 * The dropped terms are < 3*2^-24 relative per product, the order of fp32 rounding.
 *
 * Same arguments as wc_conv_igemm, restricted to: segment 0 = 3x3 taps (-1..1 row-major) at
 * stride 1 on an Hm x Wm grid equal to its source, C % 16 == 0; optional segment 1 = raw 1x1 at
 * the same pixel, C % 16 == 0; plain NHWC output at the same grid; Hm % TH == 0 and
 * Wm % 16 == 0 where TH = 8 (BN = 128) or 16 (BN = 64, used when N <= 64).
 * args->w / ldw are ignored; w6 is the weight re-packed by the caller as
 *   [ceil(N/BN)][steps][piece 3][k-half 2][BN][8] bf16 bit patterns,
 * steps = 9*(C0/16) (channel-chunk major, tap minor) + C1/16, w6_bytes its size in bytes.
 * Replaces the same reference layers as wc_conv_igemm's 3x3 case (unet_base.py:92,106). */
int wc_conv3x3_x6(const wc_conv_args* args, const void* w6, int64_t w6_bytes, void* stream);
/* The same conv with segment 0 on f16x3 (two round-to-nearest fp16 pieces of a*2^s and of
 * w*2^sW[n], three f16 MFMAs per block).  Requires the GN prologue on segment 0: the caller picks
 * a_exp with (sqrt(n_group - 1) * max|gamma| + max|beta|) * 2^a_exp <= 2^14, which bounds every
 * scaled A value below the fp16 range (Samuelson's inequality on the normalized group).
 * a_bound (optional, per image, e.g. wc_gn_finalize_bound of segment 1's input): image b uses
 * s = min(a_exp, 13 - floor(log2 a_bound[b])), which also bounds segment 1's raw values, and
 * segment 1 runs on f16x3 as well; without it s = a_exp and segment 1 stays bf16x6.
 * w3 layout per N tile: [9*C0/16 steps][piece 2][k-half 2][BN][8] fp16 bits (scaled by 2^sW[n]),
 * then [C1/16 steps][piece 2 (fp16, a_bound given) or 3 (bf16)][k-half 2][BN][8] (same scale);
 * w_inv_scale[n] = 2^-sW[n]. */
int wc_conv3x3_f16x3(const wc_conv_args* args, const void* w3, int64_t w3_bytes, int a_exp,
                     const float* w_inv_scale, const float* a_bound, void* stream);
/* (wc_conv3x3_f16x3 also takes a raw segment 0 without the GN prologue when a_bound is given and
 * nseg == 1: s = min(a_exp, 13 - floor(log2 a_bound[b])) per image, e.g. a_exp = 60 and a_bound from
 * wc_absmax_images — the 3x3 data gradients of the training backward, unet_base.py:92,106.) */
/* The output-channel tile (BN) wc_conv3x3_x6 and wc_conv_igemm_x6 use for N output channels. */
int wc_conv3x3_x6_tile_n(int N);
/* The ResBlock 3x3 conv (GN+SiLU prologue on segment 0, optional fused 1x1 residual segment 1; or
 * one raw segment 0 under the per-image bound a_bound, s = min(a_exp - 1, 12 - floor(log2 a_bound[b])))
 * through a Winograd F(2,3) transform along x on f16x3 (csrc/wc_wino.hip): per output pair and
 * kernel row, V = (d0-d2, d1+d2, d2-d1, d1-d3) of the prologue output, U = (g0, (g0+g1+g2)/2,
 * (g0-g1+g2)/2, g2), M_p = sum V_p U_p, y = (M0+M1+M2, M1-M2-M3): 12 MFMA K-steps per chunk instead
 * of 18 per output pair.  Same contract as wc_conv3x3_f16x3 (a_exp is the GroupNorm exponent; the
 * kernel uses a_exp - 1 for the doubled V range) except: segment 0 must carry the GN scale/shift and
 * SiLU, no epilogue activation, and a segment 1 needs a_bound (it runs on f16x3: the residual enters
 * the transform domain as M0 += x_even W_r, M3 += -x_odd W_r).  w layout per N tile (BN =
 * wc_conv3x3_wino_tile_n(N)): [C0/16][kernel row 3][position 4][piece 2][k-half 2][BN][8] fp16 bits of
 * U * 2^sW[n], then [C1/16][piece 2][k-half 2][BN][8] of the residual weight (same scale);
 * w_inv_scale[n] = 2^-sW[n].  H % (BN == 64 ? 16 : 8) == 0, W % 16 == 0.
 * Replaces unet_base.py:92,106 (+ :107-109 residual_input_conv), forward :146-150. */
int wc_conv3x3_wino_f16x3(const wc_conv_args* args, const void* w, int64_t w_bytes, int a_exp,
                          const float* w_inv_scale, const float* a_bound, void* stream);
int wc_conv3x3_wino_tile_n(int N);
/* The GN + SiLU segment 0 of a wc_conv3x3_wino_f16x3 conv, transformed and split ONCE (instead of once
 * per output-channel tile inside the conv): segment 0 of `args` (scale / shift / silu set, W % 16 == 0)
 * GroupNorm-affine'd, SiLU'd, scaled by 2^s (s = a_exp - 1, per image clamped to 13 - e(a_bound[b]) when
 * args has a residual segment -- the conv's own exponent), Winograd input-transformed (V0..V3 of every
 * output pair) and split into two fp16 pieces, stored in the conv's LDS image order:
 * vout[b][C/16][plane 16][H][W/2] x 16 bytes (wc_wino_vsplit_bytes; the single-piece training builds
 * store the high piece's 8 planes only, their low piece being zero).  Bit for bit what the conv's own
 * prologue computes. */
int wc_wino_vsplit_bytes(int B, int C, int H, int W, int64_t* bytes);
int wc_wino_vsplit_f16x3(const wc_conv_args* args, int a_exp, const float* a_bound, void* vout, int64_t v_bytes,
                         void* stream);
/* wc_conv3x3_wino_f16x3 reading segment 0 from wc_wino_vsplit_f16x3's output (same args, a_exp, a_bound):
 * its halo planes go into LDS by LDS-DMA with no per-item VALU; bit-identical results. */
int wc_conv3x3_wino_f16x3_vp(const wc_conv_args* args, const void* w, int64_t w_bytes, int a_exp,
                             const float* w_inv_scale, const float* a_bound, const void* vpre, int64_t v_bytes,
                             void* stream);
/* wc_conv3x3_wino_f16x3_vp with 8-wave workgroups of 256 output channels (N % 256 == 0; same results bit
 * for bit): each halo plane copy feeds twice the MFMAs.  Slower alone, faster beside a concurrent
 * stream of launches (the two-group sampling graph picks it). */
int wc_conv3x3_wino_f16x3_vp8(const wc_conv_args* args, const void* w, int64_t w_bytes, int a_exp,
                              const float* w_inv_scale, const float* a_bound, const void* vpre, int64_t v_bytes,
                              void* stream);
/* wc_conv3x3_wino_f16x3 on one raw segment (a training data gradient dz, under a_bound) whose epilogue
 * also forms the GroupNorm(+SiLU) backward's sums of the values it writes (the pass wc_gn_bwd_reduce
 * makes over dz, without re-reading dz): with xhat = x*sc0 + sh0 at the same pixel and channel and
 * dy = dz * SiLU'(gamma*xhat + beta) (silu) or dz, part[B][splits][N][2] = (sum dy, sum dy*xhat) and
 * part3[B][splits][N] (optional) = sum xhat per (image, 8- or 16-row x 16-column tile, wave row);
 * splits = wc_conv3x3_wino_gnb_splits(N, H, W).  wc_gn_bwd_finalize takes them as the reduce's. */
typedef struct wc_gnb_epi {
    const float* x;
    int ldx, silu;
    const float* sc0;
    const float* sh0;
    const float* gamma;
    const float* beta;
    float* part;
    float* part3;
    int splits, pad;
} wc_gnb_epi;
int wc_conv3x3_wino_gnb_splits(int N, int H, int W);
int wc_conv3x3_wino_f16x3_gnb(const wc_conv_args* args, const void* w, int64_t w_bytes, int a_exp,
                              const float* w_inv_scale, const float* a_bound, const wc_gnb_epi* g, void* stream);
/* Device re-pack of a [N][9*C0 + C1] fp32 ResBlock conv weight (K = (ky*3 + kx, c), then the 1x1
 * residual columns) into wc_conv3x3_wino_f16x3's layout and w_inv_scale[ceil(N/BN)*BN]: the F(2,3)
 * filter transform in float64, the per-channel power-of-two scale, one rounding to fp32, two fp16
 * pieces (bit-identical to kernels.pack_wino's definition).  out_bytes must equal the layout size. */
int wc_pack_wino(const float* w, int N, int C0, int C1, void* out, int64_t out_bytes, float* w_inv_scale,
                 void* stream);
/* wc_pack_wino from the module's own [Co][Ci][3][3] fp32 weight (no host re-layout; bit-identical to
 * wc_pack_wino of engine.pack_conv's layout): transposed = 0, the conv (N = Co, C0 = Ci) with the optional
 * 1x1 residual wres [N][C1]; transposed = 1, its data gradient (N = Ci, C0 = Co: the flipped transposed
 * filter), C1 = 0.  9 * (C0 + 4) * 4 <= 64 KiB (the row staged in LDS, padded). */
int wc_pack_wino_raw(const float* w, const float* wres, int N, int C0, int C1, int transposed, void* out,
                     int64_t out_bytes, float* w_inv_scale, void* stream);
/* Many wc_pack_wino_raw in one launch.  jobs: a DEVICE array of njobs descriptors sorted by wg0, job j
 * covering workgroups [wg0, wg0 + its N-tile-padded N) of the total_wg; out / wsinv sized as
 * wc_pack_wino_raw's; max_c0 >= every job's C0 (9 * (max_c0 + 4) * 4 <= 64 KiB).  The caller validates shapes
 * (kernels.pack_wino_raw_batch does, as wc_pack_wino_raw). */
typedef struct wc_wino_pack_job {
    const float* w;
    const float* wres;
    void* out;
    float* wsinv;
    int N, C0, C1, transposed, BN, wg0, pad0, pad1;
} wc_wino_pack_job;
int wc_pack_wino_batch(const wc_wino_pack_job* jobs, int njobs, int total_wg, int max_c0, void* stream);

/* General implicit-GEMM conv at the same bf16x6 arithmetic: exactly wc_conv_igemm's contract
 * (tap grids, input strides, the 1x1 residual segment, output maps, NCHW store; an activation
 * only with a raw segment 0) with channel counts C % 16 == 0.  args->w / ldw are ignored; w6 is
 * the weight pre-split as [ceil(N/BN)][K/16][piece 3][k-half 2][BN][8] bf16 bit patterns with K
 * in wc_conv_igemm's natural order (tap-major, then the residual columns).
 * Replaces the same reference layers as wc_conv_igemm (unet_base.py:115,129,159,334 and the
 * old UNet's Linear layers, old_modules.py:87-95). */
int wc_conv_igemm_x6(const wc_conv_args* args, const void* w6, int64_t w6_bytes, void* stream);
/* wc_conv_igemm_x6 with segment 0 on f16x3 (as wc_conv3x3_f16x3; no epilogue activation).  The
 * caller guarantees |a| * 2^a_exp <= 2^14 for every segment-0 value after the prologue, or passes
 * a_bound (per image, >= max |a| of the image's segment-0 values after the prologue, e.g. the
 * producer's absmax_out): image b then uses s = min(a_exp, 13 - floor(log2 a_bound[b])), which
 * needs tiles within one image ((Hm*Wm) % BM == 0, BM = 256 for N <= 64 else 128).  w3 layout
 * per N tile: [ntaps*C0/16 steps][piece 2][k-half 2][BN][8] fp16 bits, then
 * [C1/16][piece 3][k-half 2][BN][8] bf16 bits, all scaled by 2^sW[n]; w_inv_scale[n] = 2^-sW[n].
 * Replaces the attention in/out projections (unet_base.py:115,159), the head conv (:483-485), the
 * down-sampling convs (:231) and the up-sampling transposed convs (:300). */
int wc_conv_igemm_f16x3(const wc_conv_args* args, const void* w3, int64_t w3_bytes, int a_exp,
                        const float* w_inv_scale, const float* a_bound, void* stream);
/* The down-sampling Conv2d(C, N, 4, stride 2, padding 1) (unet_base.py:129,163) on f16x3 as a
 * 2x2 stride-1 conv over the space-to-depth view of its raw input: block (BY, BX) = input pixels
 * (2BY-1+py, 2BX-1+px), 4C channels phase-major (py, px, c), run by the halo-tiled kernel of
 * wc_conv3x3_f16x3 with a 2x2 tap grid.  args: one raw segment with the 16 taps (ky-1, kx-1),
 * stride 2, input 2Hm x 2Wm; Hm % 8 == 0, Wm % 16 == 0, N > 64 (else WC_E_SHAPE: use
 * wc_conv_igemm_f16x3); no residual, activation or output map.  a_bound[b] >= max |x| of image b
 * (the producer's absmax_out) sets its scale as in wc_conv_igemm_f16x3.  w3 layout per N tile:
 * [(4C/16) chunks x 4 taps (a, b) steps][piece 2][k-half 2][BN][8] fp16 bits of the weight
 * w[n][c][2a+py][2b+px] at s2d channel (2py+px)C + c, scaled by 2^sW[n]; w_inv_scale[n] = 2^-sW[n]. */
int wc_conv4x4s2_f16x3(const wc_conv_args* args, const void* w3, int64_t w3_bytes, const float* w_inv_scale,
                       const float* a_bound, void* stream);
/* The up-sampling ConvTranspose2d(C, N, 4, stride 2, padding 1) (unet_base.py:333-334,348) on
 * f16x3 in one launch of the halo-tiled kernel: output parity (py, px) is a 2x2 stride-1 conv over
 * the raw input, tap (i, j) at input offset (py - i, px - j) with weight rows ky = 1, 3 (py 0) or
 * 0, 2 (py 1) for i = 0, 1, columns likewise, stored at output pixel
 * (2y + py, 2x + px).  args: one raw segment (taps ignored, stride 1) over the Hm x Wm input grid;
 * output view Ho = 2Hm, Wo = 2Wm with osy = osx = 2, ooy = oox = 0; Hm % TH == 0 (TH = 16 for
 * N <= 64 else 8), Wm % 16 == 0; no residual, temb or activation.  GN partials: gn_np64 = 4HmWm/64,
 * gn_p64 = 0 (parity p writes blocks p*HmWm/64 ..).  a_bound as wc_conv4x4s2_f16x3.  w3 layout
 * per N tile: [parity 4][(C/16) chunks x 4 taps][piece 2][k-half 2][BN][8] fp16 bits, one scale
 * 2^sW[n] for all parities; w_inv_scale[n] = 2^-sW[n]. */
int wc_convtr4x4s2_f16x3(const wc_conv_args* args, const void* w3, int64_t w3_bytes, const float* w_inv_scale,
                        const float* a_bound, void* stream);
/* wc_conv_igemm_f16x3 for the attention in-projection (1x1, N = 3C output channels [q | k | v],
 * unet_base.py:115,159 in_proj_weight/in_proj_bias), whose epilogue writes the projection already
 * in the f16x3 form wc_attention_fwd_f16x3_presplit reads instead of fp32 rows: value v of part
 * p (q, k, v) is scaled by 2^exps[p] and split into two round-to-nearest fp16 pieces (h, l) that
 * are stored per image b (image stride 6*C*HW fp16 elements) as
 *   q, k:  [part 2][head][piece 2][d / 8][pixel HW][d % 8]
 *   v:     at 4*C*HW: [head][piece 2][d][HW] with pixels permuted inside every 32-pixel group into
 *          the key order of the attention kernel's P V^T MFMA (so its V^T tiles are contiguous rows).
 * args->out is ignored (may be NULL); requires args->N == 3*C, C % heads == 0, (C/heads) % 32 == 0,
 * HW % 128 == 0 and no residual / temb / absmax / GN partial outputs. */
int wc_conv_igemm_f16x3_qkv(const wc_conv_args* args, const void* w3, int64_t w3_bytes, int a_exp,
                            const float* w_inv_scale, void* qkv3, int C, int heads, const int* exps,
                            void* stream);
/* wc_attention_fwd_f16x3_presplit whose output is the out-projection's pre-split A operand: O x
 * 2^v_exp in the a3 layout of wc_split_f16x3_tiled (C % 32 == 0, N % 128 == 0, a3_bytes =
 * B*N*C*4), bit for bit that split of the fp32 output, for wc_proj_f16x3 at a_exp = v_exp. */
int wc_attention_fwd_f16x3_presplit_a3(const void* qkv3, void* a3, int64_t a3_bytes, int B, int N, int C, int heads,
                                       float scale, int q_exp, int k_exp, int v_exp, void* stream);
/* The attention projections (unet_base.py:110-116 in_proj / out_proj) on an A operand split
 * beforehand: wc_split_f16x3_tiled writes, from the rows of an NHWC view (B images x HW pixels,
 * C channels; HW % 128 == 0, C % 32 == 0, 16-byte aligned, ldc % 4 == 0) optionally through a
 * GroupNorm affine scale/shift[B][C] (+ SiLU), the values x 2^a_exp as two round-to-nearest fp16
 * pieces in the GEMM's LDS stage order: a3[B*HW/128][C/16][piece 2][k-half 2][128][8] (4 bytes
 * per element; a3_bytes = B*HW*C*4).  The caller guarantees |value| * 2^a_exp <= 2^14. */
int wc_split_f16x3_tiled(const float* src, int ldc, int B, int HW, int C, const float* scale, const float* shift,
                         int silu, int a_exp, void* a3, int64_t a3_bytes, void* stream);
/* wc_conv_igemm_f16x3 (1x1, no prologue) whose A operand is a3 from wc_split_f16x3_tiled at the same
 * a_exp: both operands of every K-step are copied to LDS by LDS-DMA.  args->seg[0] describes the
 * view a3 was made from (1x1 tap, stride 1); N % 128 == 0; identity output map into a 16-byte
 * aligned view (ldo % 4 == 0), optional residual view (same), bias, absmax_out, GN partials. */
int wc_proj_f16x3(const wc_conv_args* args, const void* a3, int64_t a3_bytes, const void* w3, int64_t w3_bytes,
                  int a_exp, const float* w_inv_scale, void* stream);
/* wc_conv_igemm_f16x3_qkv on a pre-split A operand (the GroupNorm affine applied by the split). */
int wc_proj_f16x3_qkv(const wc_conv_args* args, const void* a3, int64_t a3_bytes, const void* w3, int64_t w3_bytes,
                      int a_exp, const float* w_inv_scale, void* qkv3, int C, int heads, const int* exps,
                      void* stream);
/* Form of the two pre-split projection GEMMs above: 0 (default) the measured choice (256 x 128
 * tiles for wc_proj_f16x3_qkv at >= 2048 of them, else 128 x 128), 256 (wherever the pixels per
 * image are a multiple of 256) or 128 (the 128 x 128 LDS-DMA form).  Both forms give bit-identical
 * results.  Returns the previous setting (or WC_E_ARG).  Process-wide, not thread-safe against
 * concurrent launches. */
int wc_proj_set_tile(int rows);

/* ------------------------------------------------------------------------------------------ */
/* GroupNorm statistics (replaces nn.GroupNorm(8, C) reductions, unet_base.py:90,104,110,448)  */
/* ------------------------------------------------------------------------------------------ */

/* Number of per-batch pixel splits used by wc_gn_stats for a given shape (partials sizing). */
int wc_gn_num_splits(int B, int HW, int C);
/* partials: float[B][splits][groups][2] (mean, M2 of the split), count derivable from shape. */
int wc_gn_stats(const float* x, int B, int HW, int C, int ldc, int groups, float* partials,
                void* stream);
/* Combine partials → per-(b, c) affine: scale = rstd*gamma, shift = beta - mean*rstd*gamma. */
int wc_gn_finalize(const float* partials, int B, int HW, int C, int groups, const float* gamma,
                   const float* beta, float eps, float* scale, float* shift, void* stream);
/* The same, plus bound[b] = max over groups of |mean| + sqrt(n - 1) * std (x 1.001): every element
 * of image b of the INPUT x is at most this in magnitude (Samuelson's inequality; n = HW*C/groups). */
int wc_gn_finalize_bound(const float* partials, int B, int HW, int C, int groups, const float* gamma,
                         const float* beta, float eps, float* scale, float* shift, float* bound,
                         void* stream);
/* Tile partials (the format the split-precision conv epilogues emit through wc_conv_args.gn_part):
 * part = float[B][HW/64][ncb][32/sw][2], (mean, M2) over each 64-pixel block x sw-channel sub-slot
 * of a tensor with ncb*32 channels.  wc_gn_partials fills the slots of the view x (channels
 * [c0, c0 + C) of that tensor; C, c0 multiples of 32; HW % 64 == 0) from memory. */
int wc_gn_partials(const float* x, int ldx, int B, int HW, int C, float* part, int ncb, int sw, int c0,
                   void* stream);
/* GroupNorm of the view channels [c0, c0 + C) (groups over that range) from tile partials: the
 * per-(b, c) affine of wc_gn_finalize (and, if bound != NULL, wc_gn_finalize_bound's bound). */
int wc_gn_finalize_part(const float* part, int B, int HW, int ncb, int sw, int c0, int C, int groups,
                        const float* gamma, const float* beta, float eps, float* scale, float* shift,
                        float* bound, void* stream);

/* ------------------------------------------------------------------------------------------ */
/* Flash attention, fp32 MFMA (replaces nn.MultiheadAttention's softmax(QK^T/sqrt(d))V,        */
/* unet_base.py:115,159,214,257,320,365).                                                      */
/* ------------------------------------------------------------------------------------------ */

/* qkv: [B*N][ld_qkv] rows holding q | k | v (C each, head h at columns h*d); out: [B*N][ld_out]. */
int wc_attention_fwd(const float* qkv, int ld_qkv, float* out, int ld_out, int B, int N, int C,
                     int heads, float scale, void* stream);
/* Same contract on bf16x6 split-precision MFMA (exact 3-piece bf16 split of Q, K, V and of the
 * softmax probabilities, six products per block, fp32 accumulation); head dim C/heads % 32 == 0. */
int wc_attention_fwd_x6(const float* qkv, int ld_qkv, float* out, int ld_out, int B, int N, int C,
                        int heads, float scale, void* stream);
/* Same contract on f16x3: Q, K, V are scaled by 2^q_exp, 2^k_exp, 2^v_exp (the caller guarantees
 * |x| * 2^exp <= 2^14, e.g. from the in-projection row norms and the GroupNorm bound) and the
 * probabilities by 2^14, each split into two round-to-nearest fp16 pieces, three f16 MFMAs per block;
 * the scales are removed in the softmax multiplier and the final 1/l. */
int wc_attention_fwd_f16x3(const float* qkv, int ld_qkv, float* out, int ld_out, int B, int N, int C,
                           int heads, float scale, int q_exp, int k_exp, int v_exp, void* stream);
/* wc_attention_fwd_f16x3 / wc_attention_fwd_x6 also writing the softmax log-sum-exp
 * lse[(b*heads + h)*N + q] = log2 sum_k 2^(s_qk * scale * log2 e) (float32 [B][heads][N], the
 * contract of wc_attention_fwd_lse that wc_attention_bwd reads): the training forward
 * (train_ddpm.py:106-108) on the sampler's split-precision attention. */
int wc_attention_fwd_f16x3_lse(const float* qkv, int ld_qkv, float* out, int ld_out, float* lse, int B, int N,
                               int C, int heads, float scale, int q_exp, int k_exp, int v_exp, void* stream);
int wc_attention_fwd_x6_lse(const float* qkv, int ld_qkv, float* out, int ld_out, float* lse, int B, int N, int C,
                            int heads, float scale, void* stream);
/* wc_attention_fwd_f16x3 reading the pre-split projection written by wc_conv_igemm_f16x3_qkv with
 * exponents (q_exp, k_exp, v_exp): the K and V^T tiles are copied into LDS by LDS-DMA (no split
 * or transpose work in the key loop); results are bit-identical to wc_attention_fwd_f16x3 on the
 * fp32 projection.  N % 32 == 0, head dim % 32 == 0. */
int wc_attention_fwd_f16x3_presplit(const void* qkv3, float* out, int ld_out, int B, int N, int C, int heads,
                                    float scale, int q_exp, int k_exp, int v_exp, void* stream);

/* ------------------------------------------------------------------------------------------ */
/* Time embedding: sinusoid + t_proj MLP + every ResBlock's SiLU→Linear projection in one launch */
/* (replaces get_time_embedding unet_base.py:7-30, t_proj :395-397,462, t_emb_layers :98-100). */
/* ------------------------------------------------------------------------------------------ */

/* t: int64[nt]; w1,b1,w2,b2: t_proj Linear weights [D][D]/[D]; proj_w: concatenated rows
 * [P][D], proj_b: [P]; out: [nt][P].  D = temb_dim (even, <= 256). */
int wc_temb(const int64_t* t, int nt, int D, const float* w1, const float* b1, const float* w2,
            const float* b2, const float* proj_w, const float* proj_b, int P, float* out,
            void* stream);

/* ------------------------------------------------------------------------------------------ */
/* Stem / head                                                                                 */
/* ------------------------------------------------------------------------------------------ */

/* conv_in: NCHW input (B, Cin<=4, H, W) → NHWC view, 3x3 pad 1 (unet_base.py:400,456). */
int wc_conv_in(const float* x, int B, int Cin, int H, int W, const float* w, const float* b,
               int Cout, float* out, int ldo, void* stream);
/* conv_in for the 3 -> 64 stem with the output's GroupNorm tile partials (the wc_gn_partials format
 * and arithmetic, bit-identical) from the same launch: part / ncb / sw as wc_gn_partials, c0 = the
 * output view's first channel in the partials tensor (% 32); H*W % 64 == 0.  w is the weight
 * TRANSPOSED, [Cin*9][Cout] (k = ci*9 + ky*3 + kx), 16-byte aligned; results bit-identical to
 * wc_conv_in with the PyTorch layout.  Replaces the stem conv (unet_base.py:456) followed by the first
 * GroupNorm's statistics pass (unet_base.py:97). */
int wc_conv_in_gn(const float* x, int B, int Cin, int H, int W, const float* w, const float* b, int Cout,
                  float* out, int ldo, float* part, int ncb, int sw, int c0, void* stream);
/* Head (unet_base.py:448-449,483-485): out = conv3x3(SiLU(x*scale[b,c] + shift[b,c])) + bias for
 * NO <= 4 output channels, x an NHWC view (C % 16 == 0), out NCHW (B, NO, H, W), pad 1 after the
 * prologue.  w packed as [C/16][9 taps (ky-major)][16 channels][4 outputs, zero-padded]. */
int wc_head_conv(const float* x, int ldx, const float* scale, const float* shift, int B, int H, int W,
                 int C, const float* w, const float* bias, int NO, float* out, void* stream);

/* ------------------------------------------------------------------------------------------ */
/* Scheduler (linear_noise_scheduler.py)                                                       */
/* ------------------------------------------------------------------------------------------ */

/* Noise source for the reverse step. */
#define WC_NOISE_NONE 0     /* t == 0: x' = mean */
#define WC_NOISE_TENSOR 1   /* z given as a device tensor (torch-CPU-compatible mode) */
#define WC_NOISE_PHILOX 2   /* z generated in-kernel: Philox4x32-10(seed, sample, step) */

/* x_out = (x - coef_eps*eps ... ) exactly as sample_prev_timestep (:96-116) /
 * sample_prev_timestep2 (:63-77):  mean = (x - (beta*eps)/s1m) / sqrt_alpha;  x' = mean + sigma*z.
 * sz_out == NULL: x_out = x' (fused sampling step).  sz_out != NULL: x_out = mean and
 * sz_out = sigma*z, the (mean, sigma) pair the reference method returns.
 * The per-step scalars are computed on the host in fp32 exactly as the reference computes them.
 * Elements are NCHW (B, C, H, W) contiguous; Philox noise is keyed by the GLOBAL sample index
 * (sample0 + b) so results do not depend on how samples are sharded over ranks. */
int wc_ddpm_step(const float* x, const float* eps, const float* z, float* x_out, float* sz_out,
                 int64_t B,
                 int64_t per_sample, float beta, float s1m, float sqrt_alpha, float sigma,
                 int noise_mode, uint64_t seed, int64_t sample0, int64_t step, void* stream);

/* add_noise / add_noise2 (:30-61): out = a[t_b]*x0 + b[t_b]*noise with per-sample coefficients
 * (coef_a/coef_b: float[B], already gathered for each sample's t on the device). */
int wc_add_noise(const float* x0, const float* noise, const float* coef_a, const float* coef_b,
                 float* out, int64_t B, int64_t per_sample, void* stream);

/* Standard normal fill, Philox4x32-10 keyed by (seed, sample0 + b, step); out is (B, per_sample). */
int wc_philox_normal(float* out, int64_t B, int64_t per_sample, uint64_t seed, int64_t sample0,
                     int64_t step, void* stream);

/* ------------------------------------------------------------------------------------------ */
/* Semantic-gradient guidance update (sgg/sgg.py:16-22, seg_model/inference.py:39-43)          */
/* ------------------------------------------------------------------------------------------ */

/* grad: (nb, 3, 4S, 4S) input-gradient of the segmenter loss; mu, sigma: (nb, 3, S, S).
 * m[y][x] = sqrt(sum_c (avgpool4(grad)_c * std_c)^2); mu_hat = mu + lambda*sigma*m;
 * xt = mu_hat + sigma.  `sum_batch` = 1 reproduces the reference's batch-1 squeeze semantics
 * for nb > 1 (D4: the magnitude sums over the batch axis too).  mag_out (optional) receives m. */
int wc_sgg_update(const float* grad, const float* mu, const float* sigma, float* xt_out,
                  float* mag_out, int nb, int S, float lambda_, double std0, double std1,
                  double std2, int sum_batch, void* stream);

/* ------------------------------------------------------------------------------------------ */
/* Older 128-px UNet (diffusion_model/models/old_modules.py:126-360)                          */
/* ------------------------------------------------------------------------------------------ */

/* nn.AvgPool2d(2) on an NHWC view (old_modules.py:185,192). */
int wc_avgpool2x2(const float* in, int ldi, float* out, int ldo, int B, int H, int W, int C,
                  void* stream);
/* nn.Upsample(scale_factor=2, mode='bilinear'), align_corners=False (old_modules.py:219,222). */
int wc_upsample2x_bilinear(const float* in, int ldi, float* out, int ldo, int B, int H, int W,
                           int C, void* stream);
/* nn.LayerNorm([C]) over the channels of P pixels (old_modules.py:80-85,90,93). */
int wc_layernorm_channels(const float* in, int ldi, const float* gamma, const float* beta,
                          float eps, float* out, int ldo, int64_t P, int C, void* stream);
/* sinusoidal_embedding + nearest upsample (old_modules.py:283-317): out[pix][k] =
 * sin(ang[k]*noise[b]) for k < K, cos(ang[k-K]*noise[b]) for K <= k < 2K. */
int wc_noise_embed(const float* noise, const float* ang, int K, float* out, int ldo, int B,
                   int HW, void* stream);

/* ------------------------------------------------------------------------------------------ */
/* Training step (diffusion_model/train_ddpm.py:94-114)                                       */
/* ------------------------------------------------------------------------------------------ */

/* Size (in doubles) of the workspace wc_mse_loss needs. */
int wc_mse_workspace_doubles(void);
/* criterion = torch.nn.MSELoss() (train_ddpm.py:177, :107): loss[0] = mean((a - b)^2) over n
 * elements, fp64 accumulation in a fixed order (deterministic).  grad (optional, same shape) =
 * grad_scale * (a - b), i.e. d loss / d a for grad_scale = 2/n.  a, b, grad 16-byte aligned. */
int wc_mse_loss(const float* a, const float* b, int64_t n, float* grad, float grad_scale,
                double* workspace, float* loss, void* stream);

/* ---- UNet backward (loss.backward(), train_ddpm.py:110; the layers of unet_base.py:87-488) ---- */

/* Conv weight gradient: dW[m][k] = sum over the B*Hm*Wm pixel grid of g[pixel][m] * X_k[pixel],
 * where X_k is column k of the conv's own input exactly as the forward read it (wc_conv_args
 * segments: segment 0 through its taps / stride / zero padding, optionally through the forward's
 * GroupNorm(+SiLU) prologue scale/shift/silu, then the raw 1x1 segment 1).  K column order as the
 * forward's packed weight: (tap, channel) of segment 0, then segment 1's channels.  fp32 MFMA.
 * g: NHWC view with M channels (M % 4 == 0) and pixel stride ldg.  The pixel sum is split over
 * `splits` workgroup rows (wc_conv_wgrad_splits); partial sums go to part[splits][M][Kc] and
 * wc_wgrad_reduce adds them in a fixed order (deterministic).
 * Replaces the weight gradients of every nn.Conv2d / ConvTranspose2d / in_proj / out_proj. */
typedef struct wc_wgrad_args {
    const float* g;
    int M, ldg;
    wc_conv_seg seg[2];
    int nseg;
    int B, Hm, Wm;
} wc_wgrad_args;
int wc_conv_wgrad(const wc_wgrad_args* args, float* part, int splits, void* stream);
/* The same weight gradient on bf16x6 split-precision MFMA (both operands split exactly into three
 * bf16 pieces, the 6 piece products with i + j <= 2; fragments read pixel-contiguous from
 * [pixel][channel] LDS rows with gfx950's transposing ds_read_b64_tr_b16).  Same arguments. */
int wc_conv_wgrad_x6(const wc_wgrad_args* args, float* part, int splits, void* stream);
/* The same weight gradient on f16x3 (two fp16 pieces per operand, products h*h + h*l + l*h):
 * gbound[B] = per-image max |g|; segment 0 scaled by 2^min(x_exp0, 13 - floor(log2 max xbound0)) (xbound0
 * may be NULL: the static exponent x_exp0 of a GroupNorm-bounded operand, |x| 2^x_exp0 <= 2^14);
 * segment 1 (if any) by its per-image bound xbound1[B].  Device arrays; same partials and reduce. */
int wc_conv_wgrad_f16x3(const wc_wgrad_args* args, float* part, int splits, const float* gbound, int x_exp0,
                        const float* xbound0, const float* xbound1, void* stream);
/* The split count wc_conv_wgrad accepts for (M, Kc, P = B*Hm*Wm) aiming at ~target_blocks workgroups. */
int wc_conv_wgrad_splits(int M, int Kc, int64_t P, int target_blocks);
/* Halo-tiled weight gradient of a 3x3 stride-1 pad-1 conv on bf16x6 (the ResBlock convs' backward,
 * unet_base.py:92-94,106 under train_ddpm.py:110): a->seg[0] the 3x3 tap grid at the gradient's
 * own grid (optional GN(+SiLU) prologue), a->nseg == 1; M % 64 == 0, C0 % 32 == 0 (% 64 when
 * M % 128 != 0), Wm % 16 == 0, Hm % 8 == 0 (% 2 when M % 128 != 0).  Writes the same partials as
 * wc_conv_wgrad ([splits][M][9*C0], column = tap*C0 + c), reduced by wc_wgrad_reduce; splits from
 * wc_conv_wgrad3_splits. */
int wc_conv_wgrad3(const wc_wgrad_args* args, float* part, int splits, void* stream);
/* The same halo-tiled weight gradient on f16x3: segment 0's operand (a GroupNorm(+SiLU) output) scaled
 * by 2^x_exp, the forward conv's exponent for it (|X~| * 2^x_exp <= 2^14, Samuelson bound), and G by
 * 2^sg with sg = 13 - floor(log2 max_b gbound[b]); gbound[B] = per-image max |G| (wc_absmax_images,
 * device memory).  Two fp16 pieces per operand, products h*h + h*l + l*h, the common power-of-two
 * factor removed in the epilogue.  Same partials and reduce as wc_conv_wgrad3. */
int wc_conv_wgrad3_f16x3(const wc_wgrad_args* args, float* part, int splits, int x_exp, const float* gbound,
                         void* stream);
int wc_conv_wgrad3_splits(int M, int C0, int B, int H, int W, int target_blocks);
/* absmax[b] = max |x| over image b of the NHWC view (x, ldx) with C channels (C % 4 == 0, 16-byte
 * aligned); absmax [B] float32 zeroed by the caller.  The per-image range bound that lets the training
 * backward run its data-gradient convs on f16x3 (train_ddpm.py:110). */
int wc_absmax_images(const float* x, int ldx, int B, int HW, int C, float* absmax, void* stream);

/* Weight re-pack for the split-precision kernels in one launch (the layouts of kernels.pack_x6 /
 * pack_f16x3, see wc_pack.hip): w [N][ldw] fp32 with K = ntaps*C0 + C1 columns; order 0 'halo'
 * (16-channel chunk, tap) steps or 1 'natural' K/16 steps; mode 0 bf16x6 (3 truncated bf16 pieces),
 * mode 1 f16x3 (per-row power-of-two scale, wsinv[n] = 2^-sW[n], segment 0 as 2 fp16 pieces, segment 1
 * as 2 fp16 pieces with res_f16 else 3 bf16); BN the output-channel tile (64 or 128); out_bytes the
 * exact packed size.  Replaces the per-step host-side packing of every weight in the training step
 * (train_ddpm.py:110-111 re-runs the forward on updated weights). */
int wc_pack_split(const float* w, int ldw, int N, int C0, int ntaps, int C1, int order, int mode, int res_f16,
                  int BN, void* out, int64_t out_bytes, float* wsinv, void* stream);
/* dW = sum_split part: column k < K0 is (tap t = k / C0, channel c = k % C0), written (c < Cw only)
 * to dw0[m*sM0 + c*sC0 + t*sT0]; columns k >= K0 to dw1[m*sM1 + k - K0].  accumulate: += .
 * part is scratch: with more than 32 splits the sums of each group of 32 slabs (in a fixed order)
 * overwrite the group's first slab, and the groups are then added in order. */
int wc_wgrad_reduce(float* part, int splits, int M, int Kc, int K0, int C0, int Cw, float* dw0,
                    int64_t sM0, int64_t sC0, int64_t sT0, float* dw1, int64_t sM1, int accumulate,
                    void* stream);

/* GroupNorm(groups)(+SiLU) backward over NHWC views (reference nn.GroupNorm(8, C) -> nn.SiLU()).
 * sc0/sh0 [B][C]: the normalisation without affine (rstd, -mean*rstd: wc_gn_finalize with NULL
 * gamma/beta), so xhat = x*sc0 + sh0; y = gamma*xhat + beta; dy = dz * SiLU'(y) (silu) or dz.
 * reduce: part[B][splits][C][2] = (sum dy, sum dy*xhat) per pixel split (wc_gn_bwd_splits);
 *         x == NULL: plain per-(b, c) sums of dz (bias / time-embedding gradients).
 * finalize: sums[B][C][2] in a fixed order; with coef: coef[B][C][4] = (rstd*gamma, -rstd*A/n,
 *         -rstd*Bs/n, 0), A / Bs the group sums of gamma*sum dy / gamma*sum dy*xhat.
 *         part3 (optional, x != NULL, [B][splits][C]): the splits' sums of xhat; given to the finalize
 *         with dsum [B][C][2] (and coef), dsum[b][c][0] = the image's sum over pixels of the value the
 *         apply writes (accumulate off), c0*sum dy + HW*c1 + c2*sum xhat, second entry 0: the next
 *         layer's bias / time-embedding gradient without a pass over dx.
 * bsum: out[c] (+)= sum_b sums[b][c][idx]  (idx 0: dbeta / bias grad, 1: dgamma).
 * apply: dx (+)= coef0*dy + coef1 + coef2*xhat.  C % 4 == 0, 16-byte aligned views.  absmax (optional,
 *         [B], caller-zeroed or carried over): raised to the max |dx| written per image, so that over
 *         every writer of a gradient tensor it bounds the tensor (the f16x3 backward's range bound). */
int wc_gn_bwd_splits(int B, int HW);
int wc_gn_bwd_reduce(const float* dz, int ldz, const float* x, int ldx, const float* sc0, const float* sh0,
                     const float* gamma, const float* beta, int silu, int B, int HW, int C, int splits,
                     float* part, float* part3, void* stream);
int wc_gn_bwd_finalize(const float* part, int B, int splits, int C, int groups, int HW, const float* sc0,
                       const float* gamma, float* sums, float* coef, const float* part3, float* dsum,
                       void* stream);
int wc_bsum(const float* sums, int B, int C, int idx, float* out, int accumulate, void* stream);
/* Many wc_bsum in one launch (the training backward's deferred dgamma / dbeta / bias sums): jobs is a
 * DEVICE array of njobs descriptors, max_c >= every job's C; no two jobs of one launch share an output. */
typedef struct wc_bsum_job {
    const float* sums;
    float* out;
    int C, idx, accumulate, pad;
} wc_bsum_job;
int wc_bsum_batch(const wc_bsum_job* jobs, int njobs, int B, int max_c, void* stream);
int wc_gn_bwd_apply(const float* dz, int ldz, const float* x, int ldx, const float* sc0, const float* sh0,
                    const float* gamma, const float* beta, int silu, const float* coef, int B, int HW, int C,
                    float* dx, int lddx, int accumulate, float* absmax, void* stream);

/* Attention forward that also writes lse[b][h][q] = log2 sum_k exp2(s_qk * scale * log2 e) (fp32
 * MFMA kernel of wc_attention_fwd), and its backward: dqkv (same [q | k | v] column layout as
 * qkv) from qkv, the forward output `out`, its gradient dout and lse; dv_work: B*heads*N floats.
 * Head dims 8, 16, 32, 64, 128, 192.  Deterministic (no atomics).
 * Replaces the backward of nn.MultiheadAttention's attention core (unet_base.py:115,159). */
int wc_attention_fwd_lse(const float* qkv, int ld_qkv, float* out, int ld_out, float* lse, int B, int N, int C,
                         int heads, float scale, void* stream);
int wc_attention_bwd(const float* qkv, int ld_qkv, const float* out, int ld_out, const float* dout, int ld_dout,
                     const float* lse, float* dv_work, float* dqkv, int ld_dqkv, int B, int N, int C, int heads,
                     float scale, void* stream);
/* The same backward on bf16x6 split-precision MFMA (exact 3-piece bf16 split of Q, K, V, dO and the
 * recomputed P and dS; six products per block, fp32 accumulation); head dim C/heads in {32, 64, 128};
 * qkv, dout, dqkv 16-byte aligned. */
int wc_attention_bwd6(const float* qkv, int ld_qkv, const float* out, int ld_out, const float* dout, int ld_dout,
                      const float* lse, float* dv_work, float* dqkv, int ld_dqkv, int B, int N, int C, int heads,
                      float scale, void* stream);
/* The same backward on f16x3 (two round-to-nearest fp16 pieces per operand, three products per block):
 * Q, K, V scaled by 2^eq, 2^ek, 2^ev — the training forward's exponents from the in-projection bounds
 * (|Q| 2^eq <= 2^14 ...); dO by 2^edo from dobound[b] = per-image max |dO| (device, wc_absmax_images);
 * P by 2^14; dS by 2^eds with the bound |dS| <= 2 d max|dO| max|V|.  Head dim in {32, 64, 128}, or 192
 * (dQ on f16x3; dK / dV on f16x3 with the V rows in LDS when dqkv_absmax is given, on fp32 MFMA, which
 * raises no bound, when it is NULL: the caller's choice is the one argument, no environment switch).
 * dqkv_absmax (optional, [B], caller-zeroed): raised to the max |dqkv| written per image. */
/* The fp32-MFMA dK / dV kernel of wc_attention_bwd alone, head dim 192, after wc_attention_bwd_prep:
 * wc_attention_bwd_f16x3 pairs it with its f16x3 dQ kernel at that width. */
int wc_attention_bwd_dkdv192(const float* qkv, int ld_qkv, const float* dout, int ld_dout, const float* lse,
                             const float* dv_work, float* dqkv, int ld_dqkv, int B, int N, int C, int heads,
                             float scale, void* stream);
int wc_attention_bwd_f16x3(const float* qkv, int ld_qkv, const float* out, int ld_out, const float* dout,
                           int ld_dout, const float* lse, float* dv_work, float* dqkv, int ld_dqkv, int B, int N,
                           int C, int heads, float scale, int eq, int ek, int ev, const float* dobound,
                           float* dqkv_absmax, void* stream);
/* Its first step alone: dv_work[(b*heads + h)*N + q] = sum_d dout[b, q, h*D + d] * out[b, q, h*D + d]. */
int wc_attention_bwd_prep(const float* out, int ld_out, const float* dout, int ld_dout, int B, int N, int heads,
                          int D, float* dv_work, void* stream);

/* Small dense helpers for the time-embedding MLP backward (t_proj, t_emb_layers: B x 128):
 * C[m][n] = alpha*sum_k A[m*sam + k*sak]*B[k*sbk + n*sbn] + beta*C[m][n] (beta 0: C not read);
 * silu: mode 0 out = silu(y), mode 1 out = dz*silu'(y); colsum: out[n] (+)= sum_r X[r*ldx + n];
 * time embedding: get_time_embedding (unet_base.py:7-30) of nt timesteps, D columns. */
int wc_gemm_small(int M, int N, int K, const float* A, int64_t sam, int64_t sak, const float* B, int64_t sbk,
                  int64_t sbn, float* C, int64_t ldc, float alpha, float beta, void* stream);
int wc_silu(const float* y, const float* dz, float* out, int64_t n, int mode, void* stream);
int wc_colsum(const float* X, int R, int N, int64_t ldx, float* out, int accumulate, void* stream);
int wc_time_embedding(const int64_t* t, int nt, int D, float* out, void* stream);
/* NCHW (B, C, H, W) -> NHWC with ldc >= C channels per pixel, channels C..ldc-1 zero. */
int wc_nchw_to_nhwc(const float* src, int B, int C, int H, int W, float* dst, int ldc, void* stream);

/* ------------------------------------------------------------------------------------------ */
/* Swift-SRGAN generator (srgan_model/models.py:6-92)                                         */
/* ------------------------------------------------------------------------------------------ */

/* Depthwise half of SeperableConv2d (:9-17): nn.Conv2d(C, C, K, stride 1, padding K//2, groups=C)
 * on NHWC views (row strides ldx / ldo in floats), w = torch weight (C, 1, K, K), bias [C] or NULL.
 * K in {3, 9}; C % 4 == 0 (pad channels with zero weights).  The pointwise half, folded BatchNorm,
 * PReLU, PixelShuffle and tanh run in wc_conv_igemm (WC_ACT_PRELU / WC_ACT_TANH01, output maps). */
int wc_dwconv(const float* x, int ldx, float* out, int ldo, const float* w, const float* bias, int B,
              int H, int W, int C, int K, void* stream);

/* Training ends (train_ddpm.py:94-114 loss.backward() through unet_base.py:400 conv_in and
 * :448-449,483-485 norm_out -> SiLU -> conv_out): fp32 VALU kernels for the two 3-channel convs, whose
 * MFMA tiles would be 20x padding.
 * wc_head_dgrad: dz (NHWC view, row stride ldz) = the transposed 3x3 conv of g (NCHW (B, NO, H, W), the
 *   loss gradient of conv_out) with w_p = conv_out.weight re-laid [NO][9 taps][C] (C % 4 == 0, NO <= 4).
 * wc_head_wgrad: dw [NO][C][3][3] (=) sum over pixels of g times SiLU(x*scale[b,c] + shift[b,c]) (the
 *   forward's prologue on the NHWC view x, zero padding after it) at each tap; NO = 3, C in {32, 64}.
 * wc_stem_wgrad: dw [N][CI][3][3] (=) sum over pixels of g (NHWC, N in {32, 64} channels, row stride
 *   ldg) times the NCHW input x (CI = 3) at each tap.
 * The weight gradients take a workspace of wc_small_wgrad_workspace(B, H, W, dw elements) floats (per-
 * band partials, summed in a fixed order: deterministic); accumulate = 1 adds into dw. */
int64_t wc_small_wgrad_workspace(int B, int H, int W, int L);
int wc_head_dgrad(const float* g, int B, int NO, int H, int W, const float* w_p, int C, float* dz, int ldz,
                  void* stream);
int wc_head_wgrad(const float* x, int ldx, const float* scale, const float* shift, const float* g, int B,
                  int NO, int H, int W, int C, float* work, int64_t work_floats, float* dw, int accumulate,
                  void* stream);
int wc_stem_wgrad(const float* x_nchw, int CI, const float* g, int ldg, int B, int H, int W, int N,
                  float* work, int64_t work_floats, float* dw, int accumulate, void* stream);

/* Library identification: "weatherconverter_amd 0.1 gfx950 src:<digest>", where the digest (also alone
 * from wc_source_hash) is the one weatherconverter_amd/_build.py source_hash() computed over the kernel
 * sources, this header and the compiler flags the library was built from.  The Python loader refuses a
 * library whose digest differs from the tree's (no reference counterpart: build provenance). */
const char* wc_version(void);
const char* wc_source_hash(void);

/* Instrumentation (no reference counterpart): the exact template instantiation of the kernel the
 * calling host thread launched last through one of the entry points above, in the demangled form
 * rocprofv3 reports (e.g. "conv3x3_x6_kernel<8, 128, 2, false, true, false, false, 0, 1>"), or ""
 * when that entry point does not name its kernel.  Reading it clears it.  bench.py keys its
 * per-launch HIP-event timings by this name so they line up with the rocprofv3 kernel trace. */
const char* wc_last_kernel_name(void);
/* Instrumentation (no reference counterpart): a one-wave kernel that writes the GPU's constant-rate
 * wall clock (wall_clock64) to slots[index].  Captured into a HIP graph around each named launch
 * (kernels.stamp_timing), the stamps time every launch as the replayed graph runs it -- bench.py's
 * roofline duration (torch refuses timed event-record nodes in ROCm graph capture). */
int wc_stamp(unsigned long long* slots, int index, void* stream);
/* The wall clock's rate in kHz (hipDeviceAttributeWallClockRate of the current device). */
int wc_wall_clock_khz(int* khz);

#ifdef __cplusplus
}
#endif
#endif /* WC_KERNELS_H */
