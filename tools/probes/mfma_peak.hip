// Attainable dense MFMA rate on this MI355X under load (not the 2.4 GHz data-sheet figure): every
// wave of a full-chip grid (8 waves per SIMD) issues back-to-back v_mfma_f32_32x32x16_f16 (or _bf16, or the fp32
// 32x32x2) on four independent accumulators with random operands, for long enough (~0.1 s per launch, 5 launches) that
// the power manager has settled the clock.  Reported: TFLOP/s of the raw MFMA stream and its fraction
// of the data-sheet peak; the f16x3 conv's MFMA rate divided by this is its fraction of what the chip
// sustains.   hipcc --offload-arch=gfx950 -O3 -o mfma_peak mfma_peak.hip && ./mfma_peak
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4v __attribute__((ext_vector_type(4)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

template <int MODE>  // 0 f16 32x32x16, 1 bf16 32x32x16, 2 fp32 32x32x2, 3 f16 16x16x32
__global__ __launch_bounds__(256) void mfma_stream(const u32x4* __restrict__ ops, float* __restrict__ out, int iters) {
    const int lane = threadIdx.x & 63;
    u32x4 a[4], b[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        a[j] = ops[(j * 2) * 64 + lane];
        b[j] = ops[(j * 2 + 1) * 64 + lane];
    }
    f32x16 acc[4];
    f32x4v acc4[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[j][r] = 0.f;
#pragma unroll
        for (int r = 0; r < 4; ++r) acc4[j][r] = 0.f;
    }
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            if constexpr (MODE == 3)
                acc4[j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, a[j]),
                                                                 __builtin_bit_cast(f16x8, b[j]), acc4[j], 0, 0, 0);
            else if constexpr (MODE == 0)
                acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8, a[j]),
                                                                __builtin_bit_cast(f16x8, b[j]), acc[j], 0, 0, 0);
            else if constexpr (MODE == 1)
                acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, a[j]),
                                                                 __builtin_bit_cast(bf16x8, b[j]), acc[j], 0, 0, 0);
            else
                acc[j] = __builtin_amdgcn_mfma_f32_32x32x2f32(__builtin_bit_cast(float, a[j].x),
                                                              __builtin_bit_cast(float, b[j].x), acc[j], 0, 0, 0);
        }
    }
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
#pragma unroll
        for (int r = 0; r < 16; ++r) s += acc[j][r];
#pragma unroll
        for (int r = 0; r < 4; ++r) s += acc4[j][r];
    }
    out[blockIdx.x * 256 + threadIdx.x] = s;
}

#define CK(x)                                                                        \
    do {                                                                             \
        hipError_t e_ = (x);                                                         \
        if (e_ != hipSuccess) {                                                      \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            return 1;                                                                \
        }                                                                            \
    } while (0)

template <int MODE>
int run(const u32x4* ops, float* out, int grid, int wps, const char* name, double flop_per_mfma, double peak_tf) {
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const int iters = (MODE == 2 ? 20000 : MODE == 3 ? 200000 : 100000) * 8 / wps;  // ~0.1 s per launch
    hipLaunchKernelGGL(mfma_stream<MODE>, dim3(grid), dim3(256), 0, 0, ops, out, iters / 10);  // warm-up
    CK(hipDeviceSynchronize());
    for (int rep = 0; rep < 3; ++rep) {
        CK(hipEventRecord(e0));
        hipLaunchKernelGGL(mfma_stream<MODE>, dim3(grid), dim3(256), 0, 0, ops, out, iters);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms = 0.f;
        CK(hipEventElapsedTime(&ms, e0, e1));
        const double flops = (double)grid * 4 /*waves*/ * iters * 4 /*accs*/ * flop_per_mfma;
        const double tf = flops / (ms * 1e-3) / 1e12;
        printf("{\"mfma\": \"%s\", \"waves_per_simd\": %d, \"rep\": %d, \"ms\": %.3f, \"tflops\": %.1f, "
               "\"datasheet_peak\": %.1f, \"frac\": %.4f}\n",
               name, wps, rep, ms, tf, peak_tf, tf / peak_tf);
    }
    return 0;
}

int main() {
    int ncu = 0;
    CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
    const int grid8 = ncu * 8;  // 8 workgroups = 32 waves per CU (8 per SIMD)
    std::vector<unsigned> h(8 * 64 * 4);
    unsigned x = 12345u;
    for (auto& v : h) {  // random fp16 / bf16 pairs of magnitude ~1 (exponent bits fixed near 0)
        x = x * 1664525u + 1013904223u;
        const unsigned lo = 0x3800u | (x >> 22), hi = 0x3800u | ((x >> 12) & 0x3ffu);
        v = lo | (hi << 16) | ((x & 1u) << 15);
    }
    u32x4* ops;
    float* out;
    CK(hipMalloc(&ops, h.size() * 4));
    CK(hipMalloc(&out, (size_t)grid8 * 256 * 4));
    CK(hipMemcpy(ops, h.data(), h.size() * 4, hipMemcpyHostToDevice));
    const char* only = getenv("MFMA_PEAK_ONLY");  // "f16": the 32x32x16 f16 sweep over waves per SIMD only
    for (int wps : {8, 4, 3, 2, 1}) {  // waves per SIMD (grid = wps 4-wave workgroups per CU)
        const int grid = ncu * wps;
        if (run<0>(ops, out, grid, wps, "f32_32x32x16_f16", 32768.0, 2516.6)) return 1;
        if (only) continue;
        if (run<3>(ops, out, grid, wps, "f32_16x16x32_f16", 16384.0, 2516.6)) return 1;
        if (run<1>(ops, out, grid, wps, "f32_32x32x16_bf16", 32768.0, 2516.6)) return 1;
        if (run<2>(ops, out, grid, wps, "f32_32x32x2_f32", 4096.0, 157.3)) return 1;
    }
    CK(hipFree(ops));
    CK(hipFree(out));
    return 0;
}
