// Training-side kernels (reference diffusion_model/train_ddpm.py:94-114): the MSE loss between the
// UNet's noise prediction and the drawn noise (criterion = torch.nn.MSELoss(), mean reduction),
// fused with the gradient of that loss.
//
// Pass 1: grid-stride float4 sweep, each thread accumulates (a - b)^2 in fp64 (the mean of ~6e6
// squares keeps its fp32 result exact to the last bit this way), optionally writes
// grad = scale * (a - b); the workgroup reduces in a fixed order into partials[block].
// Pass 2: one workgroup sums the partials in a fixed order -> loss = sum / n (deterministic).
// HBM-bound: 8 B/element read (+4 B written with the gradient).
#include "wc_common.hpp"

namespace {

constexpr int MSE_THREADS = 256;
constexpr int MSE_PARTS = 1024;  // == wc_mse_workspace_doubles()

__global__ __launch_bounds__(MSE_THREADS) void mse_partial_kernel(const float* __restrict__ a,
                                                                   const float* __restrict__ b, int64_t n,
                                                                   float* __restrict__ grad, float scale,
                                                                   double* __restrict__ partials) {
    const int64_t n4 = n / 4;
    double s = 0.0;
    for (int64_t i = (int64_t)blockIdx.x * MSE_THREADS + threadIdx.x; i < n4; i += (int64_t)gridDim.x * MSE_THREADS) {
        const f32x4 av = reinterpret_cast<const f32x4*>(a)[i];
        const f32x4 bv = reinterpret_cast<const f32x4*>(b)[i];
        const f32x4 d = av - bv;
#pragma unroll
        for (int k = 0; k < 4; ++k) s = fma((double)d[k], (double)d[k], s);
        if (grad) reinterpret_cast<f32x4*>(grad)[i] = d * scale;
    }
    // scalar tail (n % 4), handled by block 0
    if (blockIdx.x == 0 && threadIdx.x < (int)(n - n4 * 4)) {
        const int64_t i = n4 * 4 + threadIdx.x;
        const float d = a[i] - b[i];
        s = fma((double)d, (double)d, s);
        if (grad) grad[i] = d * scale;
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
    __shared__ double red[MSE_THREADS / 64];
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0) {
        double t = 0.0;
        for (int w = 0; w < MSE_THREADS / 64; ++w) t += red[w];
        partials[blockIdx.x] = t;
    }
}

__global__ __launch_bounds__(MSE_THREADS) void mse_final_kernel(const double* __restrict__ partials, int nparts,
                                                                 int64_t n, float* __restrict__ loss) {
    __shared__ double red[MSE_THREADS];
    double s = 0.0;
    for (int i = threadIdx.x; i < nparts; i += MSE_THREADS) s += partials[i];
    red[threadIdx.x] = s;
    __syncthreads();
    for (int w = MSE_THREADS / 2; w > 0; w >>= 1) {
        if (threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
        __syncthreads();
    }
    if (threadIdx.x == 0) loss[0] = (float)(red[0] / (double)n);
}

}  // namespace

extern "C" int wc_mse_workspace_doubles(void) { return MSE_PARTS; }

extern "C" int wc_mse_loss(const float* a, const float* b, int64_t n, float* grad, float grad_scale,
                           double* workspace, float* loss, void* stream) {
    if (!a || !b || !workspace || !loss) return WC_E_ARG;
    if (n <= 0) return WC_E_SHAPE;
    if (((reinterpret_cast<uintptr_t>(a) | reinterpret_cast<uintptr_t>(b) | reinterpret_cast<uintptr_t>(grad)) & 15) != 0)
        return WC_E_SHAPE;
    const int64_t n4 = n / 4;
    int64_t blocks = (n4 + MSE_THREADS * 8 - 1) / (MSE_THREADS * 8);
    blocks = blocks < 1 ? 1 : blocks > MSE_PARTS ? MSE_PARTS : blocks;
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    hipLaunchKernelGGL(mse_partial_kernel, dim3((unsigned)blocks), dim3(MSE_THREADS), 0, st, a, b, n, grad, grad_scale,
                       workspace);
    WC_CHECK_LAUNCH();
    hipLaunchKernelGGL(mse_final_kernel, dim3(1), dim3(MSE_THREADS), 0, st, workspace, (int)blocks, n, loss);
    WC_CHECK_LAUNCH();
    return WC_OK;
}
