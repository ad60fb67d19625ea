// Host-side AddressSanitizer check of the C ABI (include/wc_kernels.h).
//
// Built by tools/asan/run.sh with `-Xarch_host -fsanitize=address`, so only the host code of every
// entry point is instrumented (GPU ASan is not available on this pool).  It needs no GPU: every call
// below is rejected by the argument / shape validation before any launch, or is a host-only sizing
// helper.  What it proves: the validation code reads nothing outside the caller's structs, and each
// rejection returns the documented WC_E_* code (the Python layer turns these into RuntimeError).
#include <cstdio>
#include <cstring>
#include <vector>

#include "wc_kernels.h"

static int failures = 0;

#define EXPECT(expr, want)                                                                       \
    do {                                                                                         \
        const int got_ = (expr);                                                                 \
        if (got_ != (want)) {                                                                    \
            std::printf("FAIL %s:%d %s -> %d (want %d)\n", __FILE__, __LINE__, #expr, got_, want); \
            ++failures;                                                                          \
        }                                                                                        \
    } while (0)

int main() {
    // Host buffers stand in for device pointers: none of them is dereferenced by the host code.
    std::vector<float> buf(1 << 12, 0.f);
    float* p = buf.data();
    wc_conv_args a;
    std::memset(&a, 0, sizeof(a));

    // Convolution entry points: null struct / weights / output, bad segment count, bad channels.
    EXPECT(wc_conv_igemm(nullptr, nullptr), WC_E_ARG);
    EXPECT(wc_conv_igemm(&a, nullptr), WC_E_ARG);
    a.w = p;
    a.out = p;
    a.nseg = 3;
    EXPECT(wc_conv_igemm(&a, nullptr), WC_E_ARG);
    a.nseg = 1;
    EXPECT(wc_conv_igemm(&a, nullptr), WC_E_ARG);  // seg[0].src == NULL
    a.seg[0].src = p;
    a.seg[0].C = 30;  // not a multiple of the K tile
    a.seg[0].ldc = 32;
    EXPECT(wc_conv_igemm(&a, nullptr), WC_E_SHAPE);
    EXPECT(wc_conv3x3_x6(nullptr, p, 0, nullptr), WC_E_ARG);
    EXPECT(wc_conv3x3_f16x3(nullptr, p, 0, 0, p, nullptr, nullptr), WC_E_ARG);
    a.seg[0].scale = p;  // scale without shift
    EXPECT(wc_conv3x3_f16x3(&a, p, 0, 0, p, nullptr, nullptr), WC_E_ARG);
    a.seg[0].scale = nullptr;
    EXPECT(wc_conv_igemm_x6(nullptr, p, 0, nullptr), WC_E_ARG);
    // Winograd conv: null struct, a raw segment without its per-image bound, a raw segment that is
    // not a 3x3 grid; tile width; the device pack's null / channel / size checks.
    EXPECT(wc_conv3x3_wino_f16x3(nullptr, p, 0, 0, p, p, nullptr), WC_E_ARG);
    EXPECT(wc_conv3x3_wino_f16x3(&a, p, 0, 0, p, nullptr, nullptr), WC_E_ARG);
    EXPECT(wc_conv3x3_wino_f16x3(&a, p, 0, 0, p, p, nullptr), WC_E_SHAPE);  // ntaps 0, C = 30
    EXPECT(wc_conv3x3_wino_tile_n(64), 64);
    EXPECT(wc_conv3x3_wino_tile_n(65), 128);
    EXPECT(wc_pack_wino(nullptr, 128, 32, 0, p, 0, p, nullptr), WC_E_ARG);
    EXPECT(wc_pack_wino(p, 128, 30, 0, p, 0, p, nullptr), WC_E_SHAPE);
    EXPECT(wc_pack_wino(p, 128, 32, 0, p, 12, p, nullptr), WC_E_SHAPE);  // wrong output size

    // Attention: null operands, heads not dividing C, unsupported head width, misaligned strides.
    EXPECT(wc_attention_fwd(nullptr, 96, p, 32, 1, 64, 32, 4, 1.f, nullptr), WC_E_ARG);
    EXPECT(wc_attention_fwd(p, 96, p, 32, 1, 64, 30, 4, 1.f, nullptr), WC_E_SHAPE);
    EXPECT(wc_attention_fwd(p, 96, p, 32, 1, 64, 36, 9, 1.f, nullptr), WC_E_SHAPE);  // D = 4
    EXPECT(wc_attention_fwd(p, 90, p, 32, 1, 64, 32, 4, 1.f, nullptr), WC_E_SHAPE);
    EXPECT(wc_attention_fwd_lse(p, 96, p, 32, nullptr, 1, 64, 32, 4, 1.f, nullptr), WC_E_ARG);
    EXPECT(wc_attention_fwd_f16x3(nullptr, 96, p, 32, 1, 64, 32, 4, 1.f, 0, 0, 0, nullptr), WC_E_ARG);

    // Sampler / training element-wise entry points.
    EXPECT(wc_ddpm_step(nullptr, p, p, p, nullptr, 1, 16, 0.f, 0.f, 1.f, 0.f, 0, 0, 0, 0, nullptr), WC_E_ARG);
    EXPECT(wc_ddpm_step(p, p, p, p, nullptr, 1, 15, 0.f, 0.f, 1.f, 0.f, 0, 0, 0, 0, nullptr), WC_E_SHAPE);
    EXPECT(wc_ddpm_step(p, p, p, p, nullptr, 1, 16, 0.f, 0.f, 1.f, 0.f, 7, 0, 0, 0, nullptr), WC_E_ARG);
    EXPECT(wc_mse_loss(nullptr, p, 16, nullptr, 1.f, nullptr, p, nullptr), WC_E_ARG);
    std::vector<double> ws(wc_mse_workspace_doubles());
    EXPECT(wc_mse_loss(p, p, 0, nullptr, 1.f, ws.data(), p, nullptr), WC_E_SHAPE);
    EXPECT(wc_mse_loss(p + 1, p, 16, nullptr, 1.f, ws.data(), p, nullptr), WC_E_SHAPE);  // misaligned

    // Round-3 training entry points: weight gradients, split-precision attention backward, bounds.
    wc_wgrad_args wg;
    std::memset(&wg, 0, sizeof(wg));
    EXPECT(wc_conv_wgrad3(nullptr, p, 1, nullptr), WC_E_ARG);
    EXPECT(wc_conv_wgrad3_f16x3(&wg, p, 1, 0, p, nullptr), WC_E_ARG);  // g == NULL
    wg.g = p;
    wg.nseg = 1;
    wg.seg[0].src = p;
    EXPECT(wc_conv_wgrad3_f16x3(&wg, p, 1, 0, nullptr, nullptr), WC_E_ARG);  // no gradient bound
    EXPECT(wc_conv_wgrad3_f16x3(&wg, p, 1, 99, p, nullptr), WC_E_ARG);       // exponent out of range
    EXPECT(wc_conv_wgrad3(&wg, p, 1, nullptr), WC_E_SHAPE);                   // not a 3x3 tap grid
    EXPECT(wc_conv_wgrad_f16x3(nullptr, p, 1, p, 0, nullptr, nullptr, nullptr), WC_E_ARG);
    EXPECT(wc_conv_wgrad_f16x3(&wg, p, 1, nullptr, 0, nullptr, nullptr, nullptr), WC_E_ARG);  // no G bound
    wg.nseg = 2;
    wg.seg[1].src = p;
    EXPECT(wc_conv_wgrad_f16x3(&wg, p, 1, p, 0, nullptr, nullptr, nullptr), WC_E_ARG);  // segment 1 unbounded
    EXPECT(wc_wgrad_reduce(nullptr, 1, 4, 4, 4, 4, 4, p, 0, 0, 0, nullptr, 0, 0, nullptr), WC_E_ARG);
    EXPECT(wc_wgrad_reduce(p, 1, 4, 8, 4, 4, 4, p, 0, 0, 0, nullptr, 0, 0, nullptr), WC_E_ARG);  // dw1 missing
    EXPECT(wc_attention_bwd_f16x3(p, 96, p, 32, p, 32, p, p, p, 96, 1, 64, 32, 4, 1.f, 0, 0, 0, nullptr, nullptr,
                                  nullptr), WC_E_ARG);  // no dO bound
    EXPECT(wc_attention_bwd_f16x3(p, 96, p, 32, p, 32, p, p, p, 96, 1, 64, 32, 4, 1.f, 99, 0, 0, p, nullptr, nullptr),
           WC_E_ARG);  // exponent out of range
    EXPECT(wc_attention_bwd_f16x3(p, 96, p, 32, p, 32, p, p, p, 96, 1, 64, 30, 4, 1.f, 0, 0, 0, p, nullptr, nullptr),
           WC_E_SHAPE);  // heads do not divide C
    EXPECT(wc_attention_bwd_dkdv192(p, 96, p, 32, p, p, p, 96, 1, 64, 32, 4, 1.f, nullptr), WC_E_SHAPE);  // D != 192
    EXPECT(wc_attention_bwd6(nullptr, 96, p, 32, p, 32, p, p, p, 96, 1, 64, 32, 4, 1.f, nullptr), WC_E_ARG);
    EXPECT(wc_gn_bwd_apply(nullptr, 4, p, 4, p, p, nullptr, nullptr, 1, p, 1, 16, 4, p, 4, 0, p, nullptr), WC_E_ARG);
    EXPECT(wc_gn_bwd_apply(p, 3, p, 4, p, p, nullptr, nullptr, 1, p, 1, 16, 4, p, 4, 0, p, nullptr), WC_E_SHAPE);
    EXPECT(wc_absmax_images(nullptr, 4, 1, 16, 4, p, nullptr), WC_E_ARG);
    EXPECT(wc_pack_split(p, 144, 4, 16, 9, 0, 0, 0, 0, 100, p, 0, p, nullptr), WC_E_ARG);  // BN not 64 / 128

    // Kernel-form selectors: out-of-range modes rejected, valid ones return the previous setting.
    EXPECT(wc_conv3x3_set_onewave(2), WC_E_ARG);
    EXPECT(wc_proj_set_tile(64), WC_E_ARG);
    if (wc_conv3x3_set_onewave(1) != 0 || wc_conv3x3_set_onewave(0) != 1 || wc_proj_set_tile(256) != 0 ||
        wc_proj_set_tile(-128) != 256 || wc_proj_set_tile(128) != -128 || wc_proj_set_tile(0) != 128) {
        std::printf("FAIL kernel-form selectors\n");
        ++failures;
    }
    // the 256-row projection launcher checks run before any launch (null / misaligned A operand)
    EXPECT(wc_proj_f16x3_qkv(&a, nullptr, 0, p, 0, 0, p, p, 128, 4, nullptr, nullptr), WC_E_ARG);

    // Host-only sizing helpers must be positive and deterministic.
    if (wc_conv3x3_x6_tile_n(64) != 64 || wc_conv3x3_x6_tile_n(320) != 128) {
        std::printf("FAIL wc_conv3x3_x6_tile_n\n");
        ++failures;
    }
    if (wc_gn_num_splits(16, 4096, 320) <= 0 || wc_gn_bwd_splits(16, 4096) <= 0 ||
        wc_conv_wgrad_splits(320, 2880, 65536, 1024) <= 0 || wc_mse_workspace_doubles() <= 0 ||
        wc_conv_wgrad3_splits(128, 128, 32, 256, 256, 512) <= 0 ||
        wc_conv_wgrad3_splits(128, 128, 32, 256, 256, 512) != wc_conv_wgrad3_splits(128, 128, 32, 256, 256, 512)) {
        std::printf("FAIL sizing helpers\n");
        ++failures;
    }

    std::printf("abi_validation: %d failure(s)\n", failures);
    return failures == 0 ? 0 : 1;
}
