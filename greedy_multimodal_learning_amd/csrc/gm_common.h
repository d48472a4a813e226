// Internal helpers shared by the HIP translation units of libgreedymml_hip.so.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstdio>
#include <cstdint>

#include "greedymml.h"

namespace gm {

// ---- error reporting (thread-local text, no exceptions across the ABI) ----
void set_error(const char* fmt, ...);
int check_launch(const char* what);

#define GM_REQUIRE(cond, ...)                 \
    do {                                      \
        if (!(cond)) {                        \
            ::gm::set_error(__VA_ARGS__);     \
            return GM_E_ARG;                  \
        }                                     \
    } while (0)

// ---- element access ----
template <typename T> struct Elem;
template <> struct Elem<float> {
    static __device__ __forceinline__ float ld(const float* p) { return *p; }
    static __device__ __forceinline__ void st(float* p, float v) { *p = v; }
};
// bf16 stored as raw uint16 (upper half of an f32)
template <> struct Elem<uint16_t> {
    static __device__ __forceinline__ float ld(const uint16_t* p) {
        return __uint_as_float(((uint32_t)*p) << 16);
    }
    static __device__ __forceinline__ void st(uint16_t* p, float v) { *p = f2bf(v); }
    static __device__ __forceinline__ uint16_t f2bf(float v) {
        __bf16 h = (__bf16)v;  // v_cvt_pk_bf16_f32: RNE, NaN-preserving
        return __builtin_bit_cast(uint16_t, h);
    }
};

// ReLU with PyTorch's NaN semantics (torch.relu = clamp_min propagates NaN; fmaxf(NaN, 0) would
// return 0 and hide a diverged activation from the NaN-loss stop)
__device__ __forceinline__ float relu_nan(float z) { return (z > 0.f || z != z) ? z : 0.f; }

// The gradient join's masked addend (a ReLU output's dz = dy where the forward's mask bit is set;
// batchnorm.hip's 1-bit mask: bit e of byte i is element 8 i + e): the bf16 pair x keeps the
// halves whose bits (b & 1: low, b & 2: high) are set - exactly the dres the BN backward wrote
__device__ __forceinline__ uint32_t mask_bf2(uint32_t x, uint32_t b) {
    return x & ((b & 1u ? 0x0000ffffu : 0u) | (b & 2u ? 0xffff0000u : 0u));
}

__device__ __forceinline__ float bf_lo(uint32_t w) { return __uint_as_float(w << 16); }
__device__ __forceinline__ float bf_hi(uint32_t w) { return __uint_as_float(w & 0xffff0000u); }
__device__ __forceinline__ uint32_t pack_bf2(float lo, float hi) {
    return (uint32_t)Elem<uint16_t>::f2bf(lo) | ((uint32_t)Elem<uint16_t>::f2bf(hi) << 16);
}

// Group i of 8 consecutive channels of an NHWC activation: one 16-byte vector for
// bf16, two for fp32 (the reference-precision trunk).  Values travel as fp32.
template <typename E> struct V8;
template <> struct V8<uint16_t> {
    static __device__ __forceinline__ void ld(const void* base, long long i, float* f) {
        const uint4 u = static_cast<const uint4*>(base)[i];
        f[0] = bf_lo(u.x); f[1] = bf_hi(u.x); f[2] = bf_lo(u.y); f[3] = bf_hi(u.y);
        f[4] = bf_lo(u.z); f[5] = bf_hi(u.z); f[6] = bf_lo(u.w); f[7] = bf_hi(u.w);
    }
    static __device__ __forceinline__ void st(void* base, long long i, const float* f) {
        static_cast<uint4*>(base)[i] =
            make_uint4(pack_bf2(f[0], f[1]), pack_bf2(f[2], f[3]), pack_bf2(f[4], f[5]), pack_bf2(f[6], f[7]));
    }
};
template <> struct V8<float> {
    static __device__ __forceinline__ void ld(const void* base, long long i, float* f) {
        const float4* p = static_cast<const float4*>(base) + 2 * i;
        const float4 a = p[0], b = p[1];
        f[0] = a.x; f[1] = a.y; f[2] = a.z; f[3] = a.w; f[4] = b.x; f[5] = b.y; f[6] = b.z; f[7] = b.w;
    }
    static __device__ __forceinline__ void st(void* base, long long i, const float* f) {
        float4* p = static_cast<float4*>(base) + 2 * i;
        p[0] = make_float4(f[0], f[1], f[2], f[3]);
        p[1] = make_float4(f[4], f[5], f[6], f[7]);
    }
};

// 64-lane wave sum (gfx950 wave64)
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}
__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// unsigned fast division by a runtime constant (host-side precomputed magic)
struct FastDiv {
    uint32_t d, m, s;
    FastDiv() : d(1), m(0), s(0) {}
    explicit FastDiv(uint32_t div) : d(div) {
        s = 0;
        while ((1ull << s) < div) ++s;
        m = (uint32_t)((((1ull << 32) * ((1ull << s) - div)) / div) + 1);
    }
    __device__ __forceinline__ uint32_t div(uint32_t n) const {
        uint32_t t = __umulhi(n, m);
        return (uint32_t)(((uint64_t)t + n) >> s);
    }
};

inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

// ---- in-launch hand-off health (fused BatchNorm, split-K turnstile) ----------------
// A spin that runs out of its poll budget sets a bit in its translation unit's sticky
// device fault word and poisons its result (NaN) instead of applying stale data;
// gm_device_faults() (abi.hip) reports the OR of all fault words.
unsigned spin_limit();                         // host: poll budget passed to the kernels
// the device residency plan (gm_set_residency): who else can hold CU slots while a
// launch whose workgroups wait on each other runs
struct Residency {
    int streams, sharers, reserved_cus;
};
const Residency& residency();
int usable_cus(int cus);                       // cus - reserved (at least cus / 4)
unsigned bn_faults_read(bool clear);           // batchnorm.hip
unsigned conv_faults_read(bool clear);         // conv_igemm.hip

// ---- cross-workgroup hand-off without fences (cdna_hip_programming.md, in-launch
// split-K recipe, sc1 form): the producer writes with sc1 (write-through) stores,
// drains vmcnt, barriers and publishes with a relaxed agent-scope atomic; the
// consumer observes the atomic and reads with sc1 loads (L2-served, never stale) ----
template <typename T>
__device__ __forceinline__ void st_sc1(T* p, T v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// sc1 accesses through a buffer resource: plain (non-atomic) instructions, so many
// stay in flight; cache-policy bit 16 = sc1 on gfx950
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc_of(const void* base) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, 0x7fffffff, 0x00020000);
}
__device__ __forceinline__ float4 ld_sc1_f32x4(__amdgpu_buffer_rsrc_t r, unsigned off_bytes) {
    return __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(r, off_bytes, 0, 16));
}
__device__ __forceinline__ void st_sc1_f32x4(__amdgpu_buffer_rsrc_t r, unsigned off_bytes, float4 v) {
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned, v), r,
                                           off_bytes, 0, 16);
}

}  // namespace gm
