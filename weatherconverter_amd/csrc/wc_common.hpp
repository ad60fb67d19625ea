// Shared device helpers for the WeatherConverter MI355X (gfx950 / CDNA4) kernels.
// Every kernel in this library is written for wave64 CDNA4 only: no CUDA shims, no dual paths.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <initializer_list>
#include <string>

#include "../../include/wc_kernels.h"

#define WC_DEVICE __device__ __forceinline__

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

// Status codes (see include/wc_kernels.h).
#define WC_CHECK_LAUNCH()                                                       \
    do {                                                                        \
        hipError_t _e = hipGetLastError();                                      \
        if (_e != hipSuccess) return (int)_e;                                   \
    } while (0)

WC_DEVICE float wc_silu(float v) {
    // v * sigmoid(v); v_exp_f32 based exp and a true division keep this within ~1 ulp of
    // torch.nn.functional.silu's fp32 result.
    return v / (1.0f + __expf(-v));
}

// fp32 MFMA 32x32x2: D[32x32] += A[32x2] * B[2x32].  Lane l supplies A[l&31][l>>5] and
// B[l>>5][l&31]; D element (row, col) for register r is row = (r&3) + 8*(r>>2) + 4*(l>>5),
// col = l&31.  Exact f32 fma chain (MI355X_MICROARCH.md, Matrix cores).
WC_DEVICE f32x16 mfma32(float a, float b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}

WC_DEVICE int wc_lane() { return __lane_id(); }

// Instantiation name of the kernel the calling host thread launched last, in the demangled form
// rocprofv3 prints ("conv3x3_x6_kernel<8, 128, 2, false, true, false, false, 0, 1>"), read once per
// launch through wc_last_kernel_name() so per-launch timings can be keyed exactly as the profiler
// keys them.  Templated launchers build their name once (a function-local static string).
inline thread_local const char* wc_last_kernel = "";
struct WcTArg {
    long v;
    bool is_bool;
};
#define WC_TI(x) WcTArg{(long)(x), false}
#define WC_TB(x) WcTArg{(long)(x), true}
inline std::string wc_tname(const char* base, std::initializer_list<WcTArg> args) {
    std::string s(base);
    s += '<';
    bool first = true;
    for (const WcTArg& a : args) {
        if (!first) s += ", ";
        first = false;
        s += a.is_bool ? (a.v ? "true" : "false") : std::to_string(a.v);
    }
    s += '>';
    return s;
}
#define WC_SET_NAME(...)                                            \
    do {                                                            \
        static const std::string _wc_nm = wc_tname(__VA_ARGS__);    \
        wc_last_kernel = _wc_nm.c_str();                            \
    } while (0)

// Wave-level reductions over 64 lanes.
WC_DEVICE float wave_sum(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}
WC_DEVICE float wave_max(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
    return v;
}

// Chan et al. pairwise merge of (count, mean, M2) partial moments; used by GroupNorm so that
// the variance never goes through E[x^2] - E[x]^2 cancellation.
WC_DEVICE void chan_merge(float& n, float& mean, float& m2, float nb, float meanb, float m2b) {
    float nt = n + nb;
    if (nt <= 0.f) return;
    float delta = meanb - mean;
    float fb = nb / nt;
    mean = mean + delta * fb;
    m2 = m2 + m2b + delta * delta * n * fb;
    n = nt;
}
