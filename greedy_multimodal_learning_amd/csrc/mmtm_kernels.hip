// MMTM squeeze / excitation-scale kernels for gfx950 (wave64).
//
// Spatial reduction (squeeze and its backward) and channel re-scale of
// MMTM_mitigate (reference src/balanced_mmtm.py:49-154).  HBM-bound: every
// kernel streams its activations exactly once with 16-byte vector loads where
// alignment allows, accumulates in fp32 and reduces with wave shuffles + LDS.
//
//   NCHW: one wave per (b,c) row of HW contiguous elements; the row is read with
//         the widest aligned vector (2..16 B/lane) and reduced by wave shuffles.
//   NHWC: a 256-thread workgroup per (b, HW-split); each thread owns 16 B of
//         channels, walks pixels, then the pixel lanes are reduced through LDS.
//         Splits write fp32 partials which a second pass sums in fixed order
//         (deterministic, no float atomics).
#include <cstring>

#include <cstdlib>

#include "gm_common.h"

namespace gm {

constexpr int kMaxProb = 4;

struct RedProb {
    const void* x;
    const void* dy;
    float* out;
    const float* e;
    int C, HW, ld_out, ld_e;
    float scale;
    int row_start;   // NCHW: first global row (b*C + c) of this problem
    int wg_start;    // NHWC: first workgroup of this problem
    int S;           // NHWC: HW splits
    int hw_per;      // NHWC: pixels per split
    int cw, ncs;     // NHWC: channels per slab (<= 4096 B of them), slabs (C = cw * ncs)
    float* part;     // NHWC partials [B][S][C] (S > 1)
};
struct RedArgs {
    RedProb p[kMaxProb];
    int nprob, B;
    const gm_gate_state* gate;  // gated form: the substituted modality's outputs x 0
    int mod[kMaxProb];          // gated form: modality of each problem (-2: never substituted)
};

// the modality whose scale the on-device gate substitutes, or -1 (reads only the
// curation_mode / caring prefix shared by gm_gate_state and gm_gate_state_n)
__device__ __forceinline__ int gate_sub(const gm_gate_state* g) {
    if (!g) return -1;
    return g->curation_mode ? g->caring : -1;
}

// gm_mmtm_mask_rows2's factor of problem pi under the gate (0 for the substituted one)
__device__ __forceinline__ float gate_factor(const RedArgs& a, int pi) {
    const int sub = gate_sub(a.gate);
    return (sub >= 0 && a.mod[pi] == sub) ? 0.f : 1.f;
}

__device__ __forceinline__ float epilogue(float g, const RedProb& p, int b, int c, float k = 1.f) {
    g *= p.scale;
    if (p.e) {
        float e = p.e[(size_t)b * p.ld_e + c];
        g = g * ((1.0f - e) * e);
    }
    return g * k;  // gm_mmtm_mask_rows2's factor, applied in place of that launch
}

// ---- vector loaders: VB bytes per lane -> N floats ----
template <typename T, int VB> struct VecLd;
template <int VB> struct VecLd<float, VB> {
    static constexpr int N = VB / 4;
    static __device__ __forceinline__ void ld(const float* p, float* v) {
        if constexpr (VB == 16) { float4 t = *(const float4*)p; v[0] = t.x; v[1] = t.y; v[2] = t.z; v[3] = t.w; }
        else if constexpr (VB == 8) { float2 t = *(const float2*)p; v[0] = t.x; v[1] = t.y; }
        else { v[0] = *p; }
    }
};
template <int VB> struct VecLd<uint16_t, VB> {
    static constexpr int N = VB / 2;
    static __device__ __forceinline__ void ld(const uint16_t* p, float* v) {
        if constexpr (VB == 16) {
            uint4 t = *(const uint4*)p;
            v[0] = bf_lo(t.x); v[1] = bf_hi(t.x); v[2] = bf_lo(t.y); v[3] = bf_hi(t.y);
            v[4] = bf_lo(t.z); v[5] = bf_hi(t.z); v[6] = bf_lo(t.w); v[7] = bf_hi(t.w);
        } else if constexpr (VB == 8) {
            uint2 t = *(const uint2*)p;
            v[0] = bf_lo(t.x); v[1] = bf_hi(t.x); v[2] = bf_lo(t.y); v[3] = bf_hi(t.y);
        } else if constexpr (VB == 4) {
            uint32_t t = *(const uint32_t*)p;
            v[0] = bf_lo(t); v[1] = bf_hi(t);
        } else {
            v[0] = __uint_as_float(((uint32_t)*p) << 16);
        }
    }
};

// ---------------- NCHW: one wave per row ----------------
template <typename T, int VB, bool BWD>
__global__ __launch_bounds__(256) void k_rowreduce_nchw(RedArgs a, int total_rows) {
    using L = VecLd<T, VB>;
    constexpr int N = L::N;
    const int lane = threadIdx.x & 63;
    const int wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const int nwaves = (gridDim.x * blockDim.x) >> 6;
    for (int row = wave; row < total_rows; row += nwaves) {
        int pi = 0;
#pragma unroll
        for (int q = 1; q < kMaxProb; ++q)
            if (q < a.nprob && row >= a.p[q].row_start) pi = q;
        const RedProb& p = a.p[pi];
        const int r = row - p.row_start;
        const size_t base = (size_t)r * p.HW;
        const T* x = (const T*)p.x + base;
        const T* dy = BWD ? (const T*)p.dy + base : nullptr;
        const int nvec = p.HW / N;
        float acc = 0.f;
        for (int i = lane; i < nvec; i += 64) {
            float vx[N];
            L::ld(x + (size_t)i * N, vx);
            if constexpr (BWD) {
                float vd[N];
                L::ld(dy + (size_t)i * N, vd);
#pragma unroll
                for (int j = 0; j < N; ++j) acc = fmaf(vx[j], vd[j], acc);
            } else {
#pragma unroll
                for (int j = 0; j < N; ++j) acc += vx[j];
            }
        }
        acc = wave_sum(acc);
        if (lane == 0) {
            const int b = r / p.C, c = r - b * p.C;
            p.out[(size_t)b * p.ld_out + c] = epilogue(acc, p, b, c, gate_factor(a, pi));
        }
    }
}

// ---------------- NHWC: workgroup per (b, split) ----------------
// U: pixels per thread whose 16-B loads are issued together (the loop is HBM-latency-bound:
// bytes in flight per CU, not instructions, set its rate)
// NTH: threads per workgroup (256 or 1024: the waves per CU at B x slabs workgroups)
// NT: nontemporal (streaming) loads - the activations are read once
template <typename T, bool BWD, int U, int NTH, bool NT = false>
__global__ __launch_bounds__(NTH) void k_colreduce_nhwc(RedArgs a) {
    constexpr int N = 16 / (int)sizeof(T);  // channels per thread (16 B)
    __shared__ float red[NTH * N];
    int pi = 0;
#pragma unroll
    for (int q = 1; q < kMaxProb; ++q)
        if (q < a.nprob && (int)blockIdx.x >= a.p[q].wg_start) pi = q;
    const RedProb& p = a.p[pi];
    const int w = blockIdx.x - p.wg_start;
    // workgroup = (b, split s, channel slab cs); a slab is <= 4096 B of one pixel's channels
    const int per_b = p.S * p.ncs;
    const int b = w / per_b, rem = w - b * per_b;
    const int s = rem / p.ncs, cs = rem - s * p.ncs;
    const int CW = p.cw, c0 = cs * CW;
    const int tpp = CW / N;           // threads per pixel
    const int ppi = NTH / tpp;        // pixels per iteration
    const int t = threadIdx.x;
    const int cc = t % tpp, pl = t / tpp;
    const int hw0 = s * p.hw_per, hw1 = min(p.HW, hw0 + p.hw_per);
    float acc[N];
#pragma unroll
    for (int j = 0; j < N; ++j) acc[j] = 0.f;
    if (pl < ppi) {
        const size_t bbase = (size_t)b * p.HW * p.C + c0 + (size_t)cc * N;
        auto one = [&](int hw) {
            const size_t off = bbase + (size_t)hw * p.C;
            float vx[N];
            if constexpr (NT && sizeof(T) == 2) {
                typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
                const u32x4 t4 = __builtin_nontemporal_load((const u32x4*)((const T*)p.x + off));
                vx[0] = bf_lo(t4.x); vx[1] = bf_hi(t4.x); vx[2] = bf_lo(t4.y); vx[3] = bf_hi(t4.y);
                vx[4] = bf_lo(t4.z); vx[5] = bf_hi(t4.z); vx[6] = bf_lo(t4.w); vx[7] = bf_hi(t4.w);
            } else {
                VecLd<T, 16>::ld((const T*)p.x + off, vx);
            }
            if constexpr (BWD) {
                float vd[N];
                VecLd<T, 16>::ld((const T*)p.dy + off, vd);
#pragma unroll
                for (int j = 0; j < N; ++j) acc[j] = fmaf(vx[j], vd[j], acc[j]);
            } else {
#pragma unroll
                for (int j = 0; j < N; ++j) acc[j] += vx[j];
            }
        };
        int hw = hw0 + pl;
        // U pixels per thread per round: their loads are independent, so all U are in
        // flight together (an HBM-latency-bound loop otherwise)
        for (; hw + (U - 1) * ppi < hw1; hw += U * ppi) {
#pragma unroll
            for (int u = 0; u < U; ++u) one(hw + u * ppi);
        }
        if constexpr (U > 4) {
            for (; hw + 3 * ppi < hw1; hw += 4 * ppi) {
#pragma unroll
                for (int u = 0; u < 4; ++u) one(hw + u * ppi);
            }
        }
        for (; hw < hw1; hw += ppi) one(hw);
    }
    // LDS layout [pl][CW]: thread (cc, pl) writes its N channels
    if (pl < ppi) {
#pragma unroll
        for (int j = 0; j < N; ++j) red[pl * CW + cc * N + j] = acc[j];
    }
    __syncthreads();
    // two-level fixed-order sum over the ppi pixel lanes: R = NTH / CW threads per channel
    // each sum a strided share, then one thread per channel sums the R shares
    const int R = CW <= NTH ? NTH / CW : 1;
    __shared__ float red2[NTH];
    if (R > 1) {
        if (t < R * CW) {
            const int c = t % CW, r = t / CW;
            float v = 0.f;
            for (int q = r; q < ppi; q += R) v += red[q * CW + c];
            red2[r * CW + c] = v;
        }
        __syncthreads();
    }
    for (int c = t; c < CW; c += NTH) {
        float v = 0.f;
        if (R > 1) {
            for (int r = 0; r < R; ++r) v += red2[r * CW + c];
        } else {
            for (int q = 0; q < ppi; ++q) v += red[q * CW + c];
        }
        if (p.S == 1) {
            p.out[(size_t)b * p.ld_out + c0 + c] = epilogue(v, p, b, c0 + c, gate_factor(a, pi));
        } else {
            p.part[((size_t)b * p.S + s) * p.C + c0 + c] = v;
        }
    }
}


__global__ __launch_bounds__(256) void k_reduce_partials(RedArgs a) {
    // grid: (ceil(maxC/256), B, nprob)
    const RedProb& p = a.p[blockIdx.z];
    const int b = blockIdx.y;
    const int c = blockIdx.x * 256 + threadIdx.x;
    if (c >= p.C || p.S <= 1) return;
    const float* src = p.part + (size_t)b * p.S * p.C + c;
    float v = 0.f;
    for (int s = 0; s < p.S; ++s) v += src[(size_t)s * p.C];
    p.out[(size_t)b * p.ld_out + c] = epilogue(v, p, b, c, gate_factor(a, (int)blockIdx.z));
}

// ---------------- channel scale (fwd) / apply (bwd) ----------------
struct ScaleProb {
    const void* x;
    void* y;
    const float* s;
    const float* a;
    int C, HW, ld_s, ld_a;
    float alpha;
    FastDiv div_hw;   // NCHW row = flat / HW
    FastDiv div_c;    // NHWC: pixel = flat / C
    FastDiv div_hwc;  // NHWC: b = flat / (HW*C)
    long long vec_start;  // first global vector index of this problem
    long long nvec;
};
struct ScaleArgs {
    ScaleProb p[kMaxProb];
    int nprob;
    long long total_vec;
    const gm_gate_state* gate;  // gated form: the problem whose modality is gate_sub() reads
    const float* alt[kMaxProb];   // its alt row broadcast (ld 0)
    int mod[kMaxProb];            // modality of each problem (-2: never substituted)
};

template <typename T, int N, int LAYOUT, bool ROWCONST>
__global__ __launch_bounds__(256) void k_channel_scale(ScaleArgs a) {
    const long long stride = (long long)gridDim.x * blockDim.x;
    const int sub = gate_sub(a.gate);
    for (long long v = (long long)blockIdx.x * blockDim.x + threadIdx.x; v < a.total_vec; v += stride) {
        int pi = 0;
#pragma unroll
        for (int q = 1; q < kMaxProb; ++q)
            if (q < a.nprob && v >= a.p[q].vec_start) pi = q;
        const ScaleProb& p = a.p[pi];
        const bool subst = sub >= 0 && a.mod[pi] == sub;
        const float* ps = subst ? a.alt[pi] : p.s;  // substituted: the running average row
        const int ld_s = subst ? 0 : p.ld_s;
        const uint32_t i0 = (uint32_t)((v - p.vec_start) * N);
        const T* x = (const T*)p.x + i0;
        T* y = (T*)p.y + i0;
        float vx[N], sc[N], ad[N];
        VecLd<T, N * (int)sizeof(T)>::ld(x, vx);
        if (LAYOUT == GM_NCHW) {
            if (ROWCONST) {
                const uint32_t row = p.div_hw.div(i0);
                const uint32_t b = row / (uint32_t)p.C, c = row - b * (uint32_t)p.C;
                const float s0 = ps[(size_t)b * ld_s + c];
                const float a0 = p.a ? p.a[(size_t)b * p.ld_a + c] * p.alpha : 0.f;
#pragma unroll
                for (int j = 0; j < N; ++j) { sc[j] = s0; ad[j] = a0; }
            } else {
#pragma unroll
                for (int j = 0; j < N; ++j) {
                    const uint32_t row = p.div_hw.div(i0 + j);
                    const uint32_t b = row / (uint32_t)p.C, c = row - b * (uint32_t)p.C;
                    sc[j] = ps[(size_t)b * ld_s + c];
                    ad[j] = p.a ? p.a[(size_t)b * p.ld_a + c] * p.alpha : 0.f;
                }
            }
        } else {
            const uint32_t b = p.div_hwc.div(i0);
            const uint32_t c0 = i0 - p.div_c.div(i0) * (uint32_t)p.C;
            const float* sp = ps + (size_t)b * ld_s + c0;
            if constexpr (N % 4 == 0) {
#pragma unroll
                for (int j = 0; j < N; j += 4) {
                    const float4 t = *(const float4*)(sp + j);
                    sc[j] = t.x; sc[j + 1] = t.y; sc[j + 2] = t.z; sc[j + 3] = t.w;
                }
                if (p.a) {
                    const float* ap = p.a + (size_t)b * p.ld_a + c0;
#pragma unroll
                    for (int j = 0; j < N; j += 4) {
                        const float4 t = *(const float4*)(ap + j);
                        ad[j] = t.x * p.alpha; ad[j + 1] = t.y * p.alpha;
                        ad[j + 2] = t.z * p.alpha; ad[j + 3] = t.w * p.alpha;
                    }
                } else {
#pragma unroll
                    for (int j = 0; j < N; ++j) ad[j] = 0.f;
                }
            } else {
#pragma unroll
                for (int j = 0; j < N; ++j) {
                    sc[j] = sp[j];
                    ad[j] = p.a ? p.a[(size_t)b * p.ld_a + c0 + j] * p.alpha : 0.f;
                }
            }
        }
        float o[N];
#pragma unroll
        for (int j = 0; j < N; ++j) o[j] = p.a ? fmaf(vx[j], sc[j], ad[j]) : vx[j] * sc[j];
        if constexpr (sizeof(T) == 2) {
            if constexpr (N == 8) {
                uint4 w;
                w.x = pack_bf2(o[0], o[1]); w.y = pack_bf2(o[2], o[3]);
                w.z = pack_bf2(o[4], o[5]); w.w = pack_bf2(o[6], o[7]);
                *(uint4*)y = w;
            } else {
#pragma unroll
                for (int j = 0; j < N; ++j) Elem<uint16_t>::st((uint16_t*)y + j, o[j]);
            }
        } else {
            if constexpr (N == 4) {
                *(float4*)y = make_float4(o[0], o[1], o[2], o[3]);
            } else {
#pragma unroll
                for (int j = 0; j < N; ++j) ((float*)y)[j] = o[j];
            }
        }
    }
}

// ---------------- running averages ----------------
// grid: ceil(C/64) blocks of 256 threads; wave w sums rows b = w, w+4, ... of 64
// consecutive channels (coalesced), the 4 partials are added in fixed order.
__global__ __launch_bounds__(256) void k_running_avg(const float* e, int ld, int B, int C,
                                                     const float* rv, const float* rs,
                                                     float* ov, float* os, int step) {
    __shared__ float part[4][64];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int c = blockIdx.x * 64 + lane;
    float m = 0.f;
    if (c < C) {
#pragma unroll 4
        for (int b = w; b < B; b += 4) m += e[(size_t)b * ld + c];
    }
    part[w][lane] = m;
    __syncthreads();
    if (w != 0 || c >= C) return;
    m = ((part[0][lane] + part[1][lane]) + part[2][lane]) + part[3][lane];
    m = m / (float)B;
    const float k = (float)step, k1 = (float)(step + 1);
    ov[c] = (m + rv[c] * k) / k1;
    os[c] = (m + rs[c] * k) / k1;
}

// graph-capturable form: one workgroup, step counter in device memory, averages
// updated in place; the counter is advanced after every thread has read it
__global__ __launch_bounds__(256) void k_running_avg_dev(const float* e, int ld, int B, int C, float* rv, float* rs,
                                                         int* step, int increment) {
    // one thread per channel (all 256 of them busy, no serial 64-channel passes), the
    // batch mean in the same order as before: four partial sums over b = w, w+4, ...
    // combined ((p0 + p1) + p2) + p3
    const int st = *step;
    const float k = (float)st, k1 = (float)(st + 1);
    for (int c = threadIdx.x; c < C; c += 256) {
        float p[4] = {0.f, 0.f, 0.f, 0.f};
        int b = 0;
        for (; b + 16 <= B; b += 16) {
            float v[16];
#pragma unroll
            for (int u = 0; u < 16; ++u) v[u] = e[(size_t)(b + u) * ld + c];
#pragma unroll
            for (int u = 0; u < 16; ++u) p[u & 3] += v[u];
        }
        for (; b < B; ++b) p[b & 3] += e[(size_t)b * ld + c];
        float m = ((p[0] + p[1]) + p[2]) + p[3];
        m = m / (float)B;
        rv[c] = (m + rv[c] * k) / k1;
        if (rs != rv) rs[c] = (m + rs[c] * k) / k1;
    }
    __syncthreads();  // every thread has read *step
    if (threadIdx.x == 0 && increment) *step = st + 1;
}

static bool aligned(const void* p, int bytes) { return ((uintptr_t)p % bytes) == 0; }

}  // namespace gm

using namespace gm;

// ======================= host entry points =======================

// k_colreduce_nhwc form: pixels in flight per thread (4, 8, 16) and threads per workgroup
// (256, 1024); gm_mmtm_set_reduce_form, an A/B knob
static int g_red_unroll = -1, g_red_threads = -1;
static int red_unroll() {
    if (g_red_unroll < 0) {
        g_red_unroll = 4;
    }
    return g_red_unroll;
}
static int red_threads() {
    if (g_red_threads < 0) {
        g_red_threads = 256;
    }
    return g_red_threads;
}
static int g_red_nt = [] {
    return 1;
}();
extern "C" int gm_mmtm_set_reduce_form(int threads, int unroll) {
    g_red_nt = threads < 0;  // negative threads: nontemporal loads (forward, bf16; the default)
    if (threads < 0) threads = -threads;
    GM_REQUIRE(unroll == 4 || unroll == 8 || unroll == 16, "reduce unroll must be 4, 8 or 16 (got %d)", unroll);
    GM_REQUIRE(threads == 256 || threads == 1024, "reduce threads must be 256 or 1024 (got %d)", threads);
    g_red_unroll = unroll;
    g_red_threads = threads;
    return GM_OK;
}

static int red_wgs() {
    static int w = [] {
        // workgroups wanted for the NHWC squeeze:
        // 128: from B = 64 up one workgroup per (sample, view) and no partials pass (measured
        // 25-30 us/step faster at C2 than 512, which split each map 4 ways at B = 64)
        return 128;
    }();
    return w;
}

static int red_setup(const gm_spatial_reduce* in, int nprob, int B, int dtype, int layout,
                     RedArgs& a, size_t& scratch_need, int& nwg, int& vb) {
    GM_REQUIRE(in && nprob >= 1 && nprob <= kMaxProb, "spatial_reduce: nprob must be 1..%d", kMaxProb);
    GM_REQUIRE(B >= 1, "spatial_reduce: B must be >= 1");
    GM_REQUIRE(dtype == GM_F32 || dtype == GM_BF16, "spatial_reduce: bad dtype %d", dtype);
    GM_REQUIRE(layout == GM_NCHW || layout == GM_NHWC, "spatial_reduce: bad layout %d", layout);
    const int es = dtype == GM_F32 ? 4 : 2;
    memset(&a, 0, sizeof(a));
    a.nprob = nprob;
    a.B = B;
    scratch_need = 0;
    const bool bwd = in[0].dy != nullptr;
    int rows = 0, wgs = 0;
    vb = 16;
    for (int i = 0; i < nprob; ++i) {
        const gm_spatial_reduce& s = in[i];
        GM_REQUIRE(s.x && s.out && s.C >= 1 && s.HW >= 1, "spatial_reduce[%d]: null pointer or empty shape", i);
        GM_REQUIRE((s.dy != nullptr) == bwd, "spatial_reduce: all problems must agree on forward/backward");
        GM_REQUIRE(s.ld_out >= s.C, "spatial_reduce[%d]: ld_out < C", i);
        GM_REQUIRE(!s.e || s.ld_e >= 0, "spatial_reduce[%d]: bad ld_e", i);
        RedProb& p = a.p[i];
        p.x = s.x; p.dy = s.dy; p.out = s.out; p.e = s.e;
        p.C = s.C; p.HW = s.HW; p.ld_out = s.ld_out; p.ld_e = s.ld_e; p.scale = s.scale;
        if (layout == GM_NCHW) {
            p.row_start = rows;
            rows += B * s.C;
            while (vb > es && (((size_t)s.HW * es) % vb != 0 || !aligned(s.x, vb) ||
                               (s.dy && !aligned(s.dy, vb))))
                vb >>= 1;
        } else {
            GM_REQUIRE((s.C * es) % 16 == 0 && (s.C * es <= 4096 || (s.C * es) % 4096 == 0),
                       "spatial_reduce[%d]: NHWC needs C*elem %% 16 == 0 and <= 4096 B or a multiple of it (C=%d)",
                       i, s.C);
            p.cw = s.C * es <= 4096 ? s.C : 4096 / es;
            p.ncs = s.C / p.cw;
            GM_REQUIRE(aligned(s.x, 16) && (!s.dy || aligned(s.dy, 16)),
                       "spatial_reduce[%d]: NHWC tensors must be 16-byte aligned", i);
            const int tpp = p.cw * es / 16, ppi = red_threads() / tpp;
            // per-problem split independent of how many problems share the launch, so a
            // modality's reduction order (and bits) never depends on its batch-mates
            const int per = red_wgs() / 2;
            int S = (per + B - 1) / B;
            const int maxS = (s.HW + 2 * ppi - 1) / (2 * ppi);
            S = S < 1 ? 1 : (S > maxS ? maxS : S);
            if (S < 1) S = 1;
            p.hw_per = (s.HW + S - 1) / S;
            S = (s.HW + p.hw_per - 1) / p.hw_per;
            p.S = S;
            p.wg_start = wgs;
            wgs += B * S * p.ncs;
            if (S > 1) scratch_need += (size_t)B * S * s.C * sizeof(float);
        }
    }
    nwg = layout == GM_NCHW ? rows : wgs;
    return GM_OK;
}

extern "C" size_t gm_spatial_reduce_scratch(const gm_spatial_reduce* p, int nprob, int B, int dtype,
                                            int layout) {
    RedArgs a;
    size_t need = 0;
    int nwg = 0, vb = 0;
    if (red_setup(p, nprob, B, dtype, layout, a, need, nwg, vb) != GM_OK) return 0;
    return need;
}

template <typename T>
static void launch_rows(RedArgs& a, int rows, int vb, bool bwd, hipStream_t st) {
    const int waves_per_wg = 4;
    int grid = (rows + waves_per_wg - 1) / waves_per_wg;
    if (grid > 8192) grid = 8192;
#define GM_ROWS(VB)                                                                   \
    if (bwd) k_rowreduce_nchw<T, VB, true><<<grid, 256, 0, st>>>(a, rows);            \
    else k_rowreduce_nchw<T, VB, false><<<grid, 256, 0, st>>>(a, rows);
    if (vb == 16) { GM_ROWS(16) }
    else if (vb == 8) { GM_ROWS(8) }
    else if (vb == 4) { GM_ROWS(4) }
    else if constexpr (sizeof(T) == 2) { GM_ROWS(2) }
#undef GM_ROWS
}

static int spatial_reduce_impl(const gm_spatial_reduce* in, int nprob, int B, int dtype, int layout,
                               const gm_gate_state* gate, const int* mods, void* scratch, size_t scratch_bytes,
                               void* stream) {
    RedArgs a;
    size_t need = 0;
    int nwg = 0, vb = 16;
    int rc = red_setup(in, nprob, B, dtype, layout, a, need, nwg, vb);
    if (rc) return rc;
    a.gate = gate;
    for (int i = 0; i < kMaxProb; ++i) a.mod[i] = (mods && i < nprob) ? mods[i] : -2;
    hipStream_t st = as_stream(stream);
    const bool bwd = in[0].dy != nullptr;
    if (layout == GM_NCHW) {
        if (dtype == GM_F32) launch_rows<float>(a, nwg, vb, bwd, st);
        else launch_rows<uint16_t>(a, nwg, vb, bwd, st);
        return check_launch("k_rowreduce_nchw");
    }
    GM_REQUIRE(scratch_bytes >= need && (need == 0 || scratch), "spatial_reduce: scratch %zu < %zu bytes",
               scratch_bytes, need);
    size_t off = 0;
    int maxC = 0, anyS = 0;
    for (int i = 0; i < nprob; ++i) {
        RedProb& p = a.p[i];
        if (p.S > 1) {
            p.part = (float*)((char*)scratch + off);
            off += (size_t)B * p.S * p.C * sizeof(float);
            anyS = 1;
        }
        if (p.C > maxC) maxC = p.C;
    }
#define GM_COLRED(T, U, NTH)                                                  \
    if (bwd) k_colreduce_nhwc<T, true, U, NTH><<<nwg, NTH, 0, st>>>(a);      \
    else k_colreduce_nhwc<T, false, U, NTH><<<nwg, NTH, 0, st>>>(a);
    const int u = red_unroll(), wide = red_threads() == 1024;
    if (dtype == GM_BF16 && !bwd && g_red_nt) {
        if (wide) k_colreduce_nhwc<uint16_t, false, 4, 1024, true><<<nwg, 1024, 0, st>>>(a);
        else if (u >= 8) k_colreduce_nhwc<uint16_t, false, 8, 256, true><<<nwg, 256, 0, st>>>(a);
        else k_colreduce_nhwc<uint16_t, false, 4, 256, true><<<nwg, 256, 0, st>>>(a);
    } else if (dtype == GM_F32) {
        if (wide) { GM_COLRED(float, 4, 1024) } else if (u >= 8) { GM_COLRED(float, 8, 256) } else { GM_COLRED(float, 4, 256) }
    } else if (wide) {
        if (u >= 8) { GM_COLRED(uint16_t, 8, 1024) } else { GM_COLRED(uint16_t, 4, 1024) }
    } else {
        if (u >= 16) { GM_COLRED(uint16_t, 16, 256) } else if (u >= 8) { GM_COLRED(uint16_t, 8, 256) } else { GM_COLRED(uint16_t, 4, 256) }
    }
#undef GM_COLRED
    rc = check_launch("k_colreduce_nhwc");
    if (rc || !anyS) return rc;
    dim3 g((maxC + 255) / 256, B, nprob);
    k_reduce_partials<<<g, 256, 0, st>>>(a);
    return check_launch("k_reduce_partials");
}

extern "C" int gm_mmtm_spatial_reduce(const gm_spatial_reduce* in, int nprob, int B, int dtype, int layout,
                                      void* scratch, size_t scratch_bytes, void* stream) {
    return spatial_reduce_impl(in, nprob, B, dtype, layout, nullptr, nullptr, scratch, scratch_bytes, stream);
}

extern "C" int gm_mmtm_spatial_reduce_gated(const gm_spatial_reduce* in, int nprob, int B, int dtype, int layout,
                                            const gm_gate_state* gate, void* scratch, size_t scratch_bytes,
                                            void* stream) {
    GM_REQUIRE(gate && nprob >= 2, "spatial_reduce_gated: gate and the two modalities' problems (0, 1) required");
    const int mods[kMaxProb] = {0, 1, -2, -2};
    return spatial_reduce_impl(in, nprob, B, dtype, layout, gate, mods, scratch, scratch_bytes, stream);
}

extern "C" int gm_mmtm_spatial_reduce_gated_n(const gm_spatial_reduce* in, int nprob, int B, int dtype, int layout,
                                              const gm_gate_state* gate, const int* mods, void* scratch,
                                              size_t scratch_bytes, void* stream) {
    GM_REQUIRE(gate && mods && nprob >= 1 && nprob <= kMaxProb,
               "spatial_reduce_gated_n: gate, 1..%d problems and their modality ids required", kMaxProb);
    for (int i = 0; i < nprob; ++i)
        GM_REQUIRE(mods[i] >= -2 && mods[i] < 64, "spatial_reduce_gated_n: bad modality id %d", mods[i]);
    return spatial_reduce_impl(in, nprob, B, dtype, layout, gate, mods, scratch, scratch_bytes, stream);
}

static int channel_scale_impl(const gm_channel_scale* in, int nprob, int B, int dtype, int layout,
                              const gm_gate_state* gate, const int* mods, const float* const* alts, void* stream) {
    GM_REQUIRE(in && nprob >= 1 && nprob <= kMaxProb, "channel_scale: nprob must be 1..%d", kMaxProb);
    GM_REQUIRE(B >= 1, "channel_scale: B must be >= 1");
    GM_REQUIRE(dtype == GM_F32 || dtype == GM_BF16, "channel_scale: bad dtype");
    GM_REQUIRE(layout == GM_NCHW || layout == GM_NHWC, "channel_scale: bad layout");
    const int es = dtype == GM_F32 ? 4 : 2;
    int N = 16 / es;
    bool rowconst = true;
    for (int i = 0; i < nprob; ++i) {
        const gm_channel_scale& s = in[i];
        GM_REQUIRE(s.x && s.y && s.s && s.C >= 1 && s.HW >= 1, "channel_scale[%d]: null pointer or empty", i);
        GM_REQUIRE(s.ld_s >= 0 && (!s.a || s.ld_a >= 0), "channel_scale[%d]: negative ld", i);
        const size_t numel = (size_t)B * s.C * s.HW;
        GM_REQUIRE(numel < (1ull << 32), "channel_scale[%d]: tensor too large for 32-bit indexing", i);
        if (!aligned(s.x, 16) || !aligned(s.y, 16) || numel % N) N = 1;
        if (layout == GM_NHWC && (s.C % N || !aligned(s.s, 16) || s.ld_s % 4 ||
                                  (s.a && (!aligned(s.a, 16) || s.ld_a % 4))))
            N = 1;
        if (layout == GM_NCHW && s.HW % N) rowconst = false;
    }
    ScaleArgs a;
    memset(&a, 0, sizeof(a));
    a.nprob = nprob;
    long long vs = 0;
    for (int i = 0; i < nprob; ++i) {
        const gm_channel_scale& s = in[i];
        ScaleProb& p = a.p[i];
        p.x = s.x; p.y = s.y; p.s = s.s; p.a = s.a;
        p.C = s.C; p.HW = s.HW; p.ld_s = s.ld_s; p.ld_a = s.ld_a; p.alpha = s.alpha;
        p.div_hw = FastDiv((uint32_t)s.HW);
        p.div_c = FastDiv((uint32_t)s.C);
        p.div_hwc = FastDiv((uint32_t)(s.HW * s.C));
        p.vec_start = vs;
        p.nvec = (long long)B * s.C * s.HW / N;
        vs += p.nvec;
    }
    a.total_vec = vs;
    a.gate = gate;
    for (int i = 0; i < kMaxProb; ++i) {
        a.mod[i] = (mods && i < nprob) ? mods[i] : -2;
        a.alt[i] = (alts && i < nprob) ? alts[i] : nullptr;
    }
    hipStream_t st = as_stream(stream);
    long long g = (vs + 255) / 256;
    if (g > 16384) g = 16384;
    const int grid = (int)g;
#define GM_SC(T, NN, LAY, RC) k_channel_scale<T, NN, LAY, RC><<<grid, 256, 0, st>>>(a)
    if (dtype == GM_F32) {
        if (N == 4) {
            if (layout == GM_NHWC) GM_SC(float, 4, GM_NHWC, true);
            else if (rowconst) GM_SC(float, 4, GM_NCHW, true);
            else GM_SC(float, 4, GM_NCHW, false);
        } else {
            if (layout == GM_NHWC) GM_SC(float, 1, GM_NHWC, true);
            else GM_SC(float, 1, GM_NCHW, true);
        }
    } else {
        if (N == 8) {
            if (layout == GM_NHWC) GM_SC(uint16_t, 8, GM_NHWC, true);
            else if (rowconst) GM_SC(uint16_t, 8, GM_NCHW, true);
            else GM_SC(uint16_t, 8, GM_NCHW, false);
        } else {
            if (layout == GM_NHWC) GM_SC(uint16_t, 1, GM_NHWC, true);
            else GM_SC(uint16_t, 1, GM_NCHW, true);
        }
    }
#undef GM_SC
    return check_launch("k_channel_scale");
}

extern "C" int gm_mmtm_channel_scale(const gm_channel_scale* in, int nprob, int B, int dtype, int layout,
                                     void* stream) {
    return channel_scale_impl(in, nprob, B, dtype, layout, nullptr, nullptr, nullptr, stream);
}

extern "C" int gm_mmtm_channel_scale_gated(const gm_channel_scale* in, int nprob, int B, int dtype, int layout,
                                           const gm_gate_state* gate, const float* alt0, const float* alt1,
                                           void* stream) {
    GM_REQUIRE(gate && alt0 && alt1 && nprob >= 2, "channel_scale_gated: gate, two alternative rows and the two "
               "modalities' problems (0, 1) are required");
    GM_REQUIRE(aligned(alt0, 16) && aligned(alt1, 16), "channel_scale_gated: alternative rows must be 16-B aligned");
    const int mods[kMaxProb] = {0, 1, -2, -2};
    const float* alts[kMaxProb] = {alt0, alt1, nullptr, nullptr};
    return channel_scale_impl(in, nprob, B, dtype, layout, gate, mods, alts, stream);
}

extern "C" int gm_mmtm_channel_scale_gated_n(const gm_channel_scale* in, int nprob, int B, int dtype, int layout,
                                             const gm_gate_state* gate, const int* mods, const float* const* alts,
                                             void* stream) {
    GM_REQUIRE(gate && mods && alts && nprob >= 1 && nprob <= kMaxProb,
               "channel_scale_gated_n: gate, 1..%d problems, their modality ids and alternative rows required",
               kMaxProb);
    for (int i = 0; i < nprob; ++i) {
        GM_REQUIRE(mods[i] >= -2 && mods[i] < 64, "channel_scale_gated_n: bad modality id %d", mods[i]);
        GM_REQUIRE(mods[i] < 0 || (alts[i] && aligned(alts[i], 16)),
                   "channel_scale_gated_n: problem %d needs a 16-B aligned alternative row", i);
    }
    return channel_scale_impl(in, nprob, B, dtype, layout, gate, mods, alts, stream);
}

extern "C" int gm_mmtm_running_avg(const float* e_v, int ld_e, int B, int C, const float* ra_v_old,
                                   const float* ra_s_old, float* ra_v_new, float* ra_s_new, int step,
                                   void* stream) {
    GM_REQUIRE(e_v && ra_v_old && ra_s_old && ra_v_new && ra_s_new, "running_avg: null pointer");
    GM_REQUIRE(B >= 1 && C >= 1 && ld_e >= C && step >= 0, "running_avg: bad shape");
    k_running_avg<<<(C + 63) / 64, 256, 0, as_stream(stream)>>>(e_v, ld_e, B, C, ra_v_old, ra_s_old,
                                                                  ra_v_new, ra_s_new, step);
    return check_launch("k_running_avg");
}

extern "C" int gm_mmtm_running_avg_dev(const float* e_v, int ld_e, int B, int C, float* ra_v, float* ra_s,
                                       int* step, int increment, void* stream) {
    GM_REQUIRE(e_v && ra_v && ra_s && step, "running_avg_dev: null pointer");
    GM_REQUIRE(B >= 1 && C >= 1 && ld_e >= C, "running_avg_dev: bad shape");
    k_running_avg_dev<<<1, 256, 0, as_stream(stream)>>>(e_v, ld_e, B, C, ra_v, ra_s, step, increment);
    return check_launch("k_running_avg_dev");
}
