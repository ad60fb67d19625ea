// Reproducer (device-only compile, inspect the ISA): with ROCm 7.2 hipcc,
// __builtin_bit_cast(unsigned, v[e]) on an ext_vector_type element lowers to element 0 for every
// e, so all four v_and_b32 below use the same source register.  Bit-cast a scalar copy instead.
//   hipcc -O3 --offload-arch=gfx950 --cuda-device-only -S bitcast_vector_element.hip -o - | grep v_and_b32
#include <hip/hip_runtime.h>
typedef float f32x4 __attribute__((ext_vector_type(4)));
__global__ void k(const f32x4* in, unsigned* o) {
    f32x4 v = in[threadIdx.x];
#pragma unroll
    for (int e = 0; e < 4; ++e) o[4 * threadIdx.x + e] = __builtin_bit_cast(unsigned, v[e]) & 0xffff0000u;
}
