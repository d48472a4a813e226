// Test-only kernels (not part of the product library libgreedymml_hip.so): built into
// tests/native/libgm_testkit.so by greedy_multimodal_learning_amd/build.py and loaded by the
// residency tests (tests/testkit.py).
#include <hip/hip_runtime.h>

namespace {

// one workgroup per CU when lds_bytes is the whole LDS: spins on the 100 MHz real-time
// counter, sleeping between polls, until `ticks` have passed - a stand-in for a resident
// collective kernel holding CUs
__global__ void k_hold_cus(unsigned long long ticks) {
    extern __shared__ int lds[];
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(8);
    if (threadIdx.x == 0) lds[0] = 0;
}

}  // namespace

// `blocks` workgroups of `threads` threads, each holding `lds_bytes` of LDS (up to 160 KiB: one
// workgroup per CU), spinning for `usec` microseconds.  0 on success, -1 on bad arguments, else
// the HIP error of the launch.
extern "C" int gmt_hold_cus(int blocks, int threads, int lds_bytes, unsigned usec, void* stream) {
    if (blocks < 1 || blocks > 4096 || threads < 64 || threads > 1024 || lds_bytes < 4 || lds_bytes > 160 * 1024 ||
        usec > 10000000u)
        return -1;
    if (lds_bytes > 64 * 1024)
        hipFuncSetAttribute(reinterpret_cast<const void*>(k_hold_cus), hipFuncAttributeMaxDynamicSharedMemorySize,
                            lds_bytes);
    hipLaunchKernelGGL(k_hold_cus, dim3(blocks), dim3(threads), lds_bytes, static_cast<hipStream_t>(stream),
                       (unsigned long long)usec * 100ull);
    return (int)hipGetLastError();
}
