// Calibration kernel (tools only): back-to-back v_mfma_f32_32x32x16_bf16 on register operands,
// 8 independent accumulators per wave, `waves` waves per workgroup, one workgroup per CU slot.
// Measures the MFMA rate the chip sustains under full load (clock included) - the practical
// ceiling the trunk kernels' roofline fractions are read against.
#include <hip/hip_runtime.h>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float floatx16 __attribute__((ext_vector_type(16)));

__global__ __launch_bounds__(512) void k_mfma_peak(float* out, int iters) {
    floatx16 acc[8];
    for (int i = 0; i < 8; ++i)
        for (int e = 0; e < 16; ++e) acc[i][e] = 0.f;
    bf16x8 a, b;
    for (int e = 0; e < 8; ++e) {
        a[e] = (__bf16)(float)(threadIdx.x & 7);
        b[e] = (__bf16)(float)(e + 1);
    }
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int i = 0; i < 8; ++i) acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc[i], 0, 0, 0);
    }
    float s = 0.f;
    for (int i = 0; i < 8; ++i)
        for (int e = 0; e < 16; ++e) s += acc[i][e];
    if (s == 12345.678f) out[threadIdx.x] = s;  // keep the loop alive
}

extern "C" int mfma_peak_launch(float* out, int blocks, int threads, int iters, void* stream) {
    k_mfma_peak<<<blocks, threads, 0, (hipStream_t)stream>>>(out, iters);
    return (int)hipGetLastError();
}
