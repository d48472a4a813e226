// Training-mode BatchNorm2d over NHWC bf16 activations, fused with the residual
// add and ReLU that follow it in the torchvision ResNet blocks (the reference's
// trunk, src/model.py:65-106 via torchvision.models.resnet18).
//
// Forward  y = relu?( (x - mean) * invstd * gamma + beta  (+ residual) )
//   1. k_bn_reduce<FWD>: per-block fp32 partial sums of x and x^2 per channel; the
//      last-arriving block (agent-scope release/acquire ticket) combines the
//      partials in fp64 (fixed order: deterministic), writes save_mean/save_invstd,
//      the per-channel affine coefficients and the running-stat update
//      (momentum, unbiased variance - torch.nn.functional.batch_norm semantics).
//   2. k_bn_apply: one pass, 16-byte vectors, coefficients held in registers.
// Backward (dz = dy * (y > 0) when relu):
//   1. k_bn_reduce<BWD>: S1 = sum dz, S2 = sum dz*(x-mean) -> dbeta = S1,
//      dgamma = S2*invstd, dx = a*dz + b*x + c per channel.
//   2. k_bn_apply_bwd: dx (and dres = dz for the residual branch).
// Bytes per element (bf16): fwd 2 (stats) + 4..6 (apply); bwd 4..6 + 6..8.
// The reduce + apply kernels are templated on the element type E: bf16 (the
// performance trunk) or fp32 (the reference-precision trunk, gm_bn_*_f32); the
// single-launch fused kernels are bf16 only.
#include <cstdlib>
#include <initializer_list>
#include <type_traits>

#include "gm_common.h"

namespace gm {
namespace {

constexpr int kT = 256;          // threads per block
constexpr int kMaxC = 2048;      // channels supported (ResNet-50 ends at 2048)
constexpr size_t kHdr = 256;     // scratch header (ticket counters)
constexpr int kMaxRC = 512;      // row chunks per channel slice (partials the last block combines)
constexpr int kRedF = 4096;      // LDS floats of the row-group combine (rpp * 2 * SW == 4096)

// 2-D reduce grid: (row chunk, 64-channel slice), ~512 blocks (2x for large maps).  Every block
// streams a [rows x SW] strip (SW = min(C, 64) channels, 128-B row segments),
// unrolled x8 so ~32 KB per block is in flight, and writes one partial row of
// 2*SW floats; ONE ticketed level per slice: the last-arriving block combines the
// slice's <= kMaxRC partial rows with all 256 threads (16-B sc1 loads, all in
// flight at once, fp64, fixed order) and finalizes.  One dependent memory round
// trip after the ticket instead of two ticket levels: the small maps of layer3/4
// are latency-, not bandwidth-bound.
struct Plan {
    int SW, tpr_log, rpp;  // slice width, log2(threads per row), rows per pass
    int nslice, nrc;       // slices, row chunks per slice
    long long rpb;         // rows per block
    size_t off_coef, off_p1, bytes;
};

inline int ilog2(int v) {
    int l = 0;
    while ((1 << l) < v) ++l;
    return l;
}

inline int bn_blocks() {
    static int b = [] {
        return 512;
    }();
    return b;
}

inline Plan make_plan(long long M, int C) {
    Plan p;
    p.SW = C < 64 ? C : 64;
    p.tpr_log = ilog2(p.SW / 8);
    p.rpp = kT >> p.tpr_log;
    p.nslice = C / p.SW;
    long long want = bn_blocks() / p.nslice;
    if (M * C >= (16ll << 20)) want *= 2;  // large maps: bandwidth-bound, more blocks
    if (want < 1) want = 1;
    if (want > kMaxRC) want = kMaxRC;
    long long rpb = (M + want - 1) / want;
    rpb = (rpb + p.rpp - 1) / p.rpp * p.rpp;
    p.rpb = rpb;
    p.nrc = (int)((M + rpb - 1) / rpb);
    const size_t cnt = (size_t)p.nslice * sizeof(unsigned);
    p.off_coef = (cnt + kHdr - 1) / kHdr * kHdr;
    p.off_p1 = p.off_coef + (size_t)4 * C * sizeof(float);
    p.bytes = p.off_p1 + (size_t)p.nslice * p.nrc * 2 * p.SW * sizeof(double);  // fp64 partials (fp32 path)
    return p;
}

inline size_t scratch_bytes(long long M, int C) { return make_plan(M, C).bytes; }

__device__ __forceinline__ void unpack8(uint4 u, float* f) {
    f[0] = bf_lo(u.x); f[1] = bf_hi(u.x); f[2] = bf_lo(u.y); f[3] = bf_hi(u.y);
    f[4] = bf_lo(u.z); f[5] = bf_hi(u.z); f[6] = bf_lo(u.w); f[7] = bf_hi(u.w);
}
__device__ __forceinline__ uint4 pack8(const float* f) {
    return make_uint4(pack_bf2(f[0], f[1]), pack_bf2(f[2], f[3]), pack_bf2(f[4], f[5]), pack_bf2(f[6], f[7]));
}

// The ReLU mask of 8 stored bf16 values as one byte (bit j: value j > 0 - the bf16 half in
// 0x0001 .. 0x7f80, positive and not NaN: exactly the backward's y > 0 test on the stored y, also
// for the NaN poison a spin timeout writes), and back as 8 bf16 values (1.0 where set) that the
// y-mask code paths test unchanged
__device__ __forceinline__ unsigned mask_byte(uint4 w) {
    const unsigned v[4] = {w.x, w.y, w.z, w.w};
    unsigned b = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        b |= ((v[k] & 0xffffu) - 1u < 0x7f80u ? 1u : 0u) << (2 * k);
        b |= ((v[k] >> 16) - 1u < 0x7f80u ? 1u : 0u) << (2 * k + 1);
    }
    return b;
}
__device__ __forceinline__ uint4 mask_vals(unsigned b) {
    unsigned v[4];
#pragma unroll
    for (int k = 0; k < 4; ++k)
        v[k] = ((b >> (2 * k)) & 1u ? 0x3f80u : 0u) | ((b >> (2 * k + 1)) & 1u ? 0x3f800000u : 0u);
    return make_uint4(v[0], v[1], v[2], v[3]);
}

// Pin loaded values at this point: every load issued before is complete here, and none is sunk
// past it to its first use (the compiler otherwise issues a streaming loop's loads one round
// trip at a time - the ReLU mask bytes after the 16-B vectors had landed)
typedef unsigned pin_u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void pin(uint4& v) {
    pin_u32x4 w = {v.x, v.y, v.z, v.w};
    asm volatile("" : "+v"(w));
    v = make_uint4(w.x, w.y, w.z, w.w);
}
__device__ __forceinline__ void pin(unsigned& v) { asm volatile("" : "+v"(v)); }

// Per-view-group operands: a grouped launch (gm_bn_*_grouped_bf16) normalises G views
// stacked along the batch, each with its own parameters, statistics and scratch, in one
// grid (blockIdx.z = group); every kernel starts from group_args().
constexpr int kMaxBnG = 16;  // view groups per grouped launch (C5: 12 views)
struct BnGroup {
    const void* x;
    const void* dy;
    const void* y;
    const float* gamma;
    const float* beta;
    float* rmean;
    float* rvar;
    float* save_mean;
    float* save_invstd;
    float* dgamma;
    float* dbeta;
    long long* nbt;
    float* coef_out;
    const float* fcoef;
    const uint4* res;
    uint4* yout;
    uint4* dres_out;
    uint8_t* mask_out;      // fwd (relu + residual), optional: the ReLU mask, one byte per 8 channels
    const uint8_t* ymask;   // bwd: that mask in place of y (k_bn_bwd_fused<BWD_RELU, ..., YM>)
};

struct ReduceArgs {
    long long M;
    int C, tpr_log, relu, accumulate;
    int SW, nrc;
    long long rpb;
    const void* x;       // fwd: x; bwd: x   (E elements)
    const void* dy;      // bwd
    const void* y;       // bwd relu mask
    const float* gamma;
    const float* beta;
    float* rmean;
    float* rvar;
    float momentum, eps;
    float* save_mean;    // fwd: out; bwd: in
    float* save_invstd;  // fwd: out; bwd: in
    float* dgamma;
    float* dbeta;
    unsigned* counter;   // [nslice] tickets (zero between calls)
    long long* nbt;      // num_batches_tracked (fwd, may be null)
    float* coef;         // [4][C]
    float* part;         // [nslice][nrc][SW][2] fp32 per-block partials
    float* coef_out;     // fwd, optional: the affine coefficients sc[C], sh[C] for the backward
    const float* fcoef;  // BWD_RELUX: the forward's sc[C], sh[C]
    unsigned* gen;       // fused fwd: [nslice] generation words (coefficients published)
    const uint4* res;    // fused fwd: residual
    uint4* yout;         // fused fwd: output / fused bwd: dx
    uint4* dres_out;     // fused bwd: dres
    uint8_t* mask_out;   // fused fwd, optional: ReLU mask bytes (bit j: channel 8 v + j of vector v > 0)
    const uint8_t* ymask;  // fused bwd: the mask in place of y
    unsigned spin_limit; // fused: poll budget of the coefficient hand-off
    int redundant;       // fused, small maps: every block combines the partial rows itself
    unsigned long long scr_stride;  // bytes between the groups' coefficient + partial areas
    unsigned hdr_words;             // words between the groups' ticket / generation headers
    BnGroup grp[kMaxBnG];           // grp[blockIdx.z] replaces the per-group pointers above
};

// this block's group: its pointers and its slice of the scratch (tickets, coefficients,
// partials, generation words)
__device__ __forceinline__ ReduceArgs group_args(const ReduceArgs& a0) {
    ReduceArgs a = a0;
    const int g = blockIdx.z;
    const BnGroup& q = a0.grp[g];
    a.x = q.x; a.dy = q.dy; a.y = q.y;
    a.gamma = q.gamma; a.beta = q.beta; a.rmean = q.rmean; a.rvar = q.rvar;
    a.save_mean = q.save_mean; a.save_invstd = q.save_invstd;
    a.dgamma = q.dgamma; a.dbeta = q.dbeta; a.nbt = q.nbt;
    a.coef_out = q.coef_out; a.fcoef = q.fcoef;
    a.res = q.res; a.yout = q.yout; a.dres_out = q.dres_out;
    a.mask_out = q.mask_out; a.ymask = q.ymask;
    const unsigned long long off = (unsigned long long)g * a0.scr_stride;
    a.counter = a0.counter + g * a0.hdr_words;
    a.coef = reinterpret_cast<float*>(reinterpret_cast<char*>(a0.coef) + off);
    a.part = reinterpret_cast<float*>(reinterpret_cast<char*>(a0.part) + off);
    if (a0.gen) a.gen = a0.gen + g * a0.hdr_words;
    return a;
}

// sticky fault word of this translation unit (gm_device_faults): a fused launch whose
// coefficient hand-off timed out
__device__ unsigned g_bn_fault = 0;

// Wait (thread 0, bounded) until the slice's generation word moves past g0; on
// timeout raise the fault bit and return false in EVERY thread of the block (the
// caller then applies NaN coefficients instead of stale ones).
__device__ __forceinline__ bool wait_generation(const unsigned* gen, unsigned g0, unsigned limit, float* flag) {
    if (threadIdx.x == 0) {
        unsigned it = 0;
        bool ok = true;
        while (__hip_atomic_load(gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == g0) {
            if (++it >= limit) {
                ok = false;
                break;
            }
            __builtin_amdgcn_s_sleep(2);
        }
        if (!ok) atomicOr(&g_bn_fault, GM_FAULT_BN_SPIN);
        *flag = ok ? 1.f : 0.f;
    }
    __syncthreads();
    return *flag != 0.f;
}

// BWD_RELUX: the relu mask recomputed from x and the forward's affine coefficients
// (z = x*sc + sh > 0, the forward's own fp32 value) instead of read back from y
enum { FWD = 0, BWD = 1, BWD_RELU = 2, BWD_RELUX = 3 };  // relu as a template arg: no per-load branch

template <int MODE, typename E>
__device__ __forceinline__ void accum(const ReduceArgs& a, long long v, const float* mu, float* s1, float* s2,
                                      const float* fsc, const float* fsh) {
    float xf[8];
    V8<E>::ld(a.x, v, xf);
    if (MODE == FWD) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            s1[j] += xf[j];
            s2[j] = fmaf(xf[j], xf[j], s2[j]);
        }
    } else {
        float d[8];
        V8<E>::ld(a.dy, v, d);
        if (MODE == BWD_RELU) {
            float yf[8];
            V8<E>::ld(a.y, v, yf);
#pragma unroll
            for (int j = 0; j < 8; ++j) d[j] = yf[j] > 0.f ? d[j] : 0.f;
        }
        if (MODE == BWD_RELUX) {
#pragma unroll
            for (int j = 0; j < 8; ++j) d[j] = fmaf(xf[j], fsc[j], fsh[j]) > 0.f ? d[j] : 0.f;
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            s1[j] += d[j];
            s2[j] = fmaf(d[j], xf[j] - mu[j], s2[j]);
        }
    }
}

// accum() on already loaded vectors (zero vectors contribute nothing in every mode)
template <int MODE>
__device__ __forceinline__ void accum_vals(uint4 ux, uint4 ud, uint4 uy, const float* mu, float* s1, float* s2,
                                          const float* fsc = nullptr, const float* fsh = nullptr) {
    float xf[8];
    unpack8(ux, xf);
    if (MODE == FWD) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            s1[j] += xf[j];
            s2[j] = fmaf(xf[j], xf[j], s2[j]);
        }
    } else {
        float d[8];
        unpack8(ud, d);
        if (MODE == BWD_RELU) {
            float yf[8];
            unpack8(uy, yf);
#pragma unroll
            for (int j = 0; j < 8; ++j) d[j] = yf[j] > 0.f ? d[j] : 0.f;
        }
        if (MODE == BWD_RELUX) {
#pragma unroll
            for (int j = 0; j < 8; ++j) d[j] = fmaf(xf[j], fsc[j], fsh[j]) > 0.f ? d[j] : 0.f;
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            s1[j] += d[j];
            s2[j] = fmaf(d[j], xf[j] - mu[j], s2[j]);
        }
    }
}

// per-channel operands of finalize(), loaded by every block BEFORE its ticket so the
// last block's dependent chain after the ticket has one memory round trip fewer
struct FinOps {
    float g, b, rm, rv;  // FWD: gamma, beta, running mean/var; BWD: gamma, -, save_mean, save_invstd
};

template <int MODE>
__device__ __forceinline__ FinOps fin_load(const ReduceArgs& a, int c) {
    FinOps f;
    f.g = a.gamma[c];
    if (MODE == FWD) {
        f.b = a.beta[c];
        f.rm = a.rmean ? a.rmean[c] : 0.f;
        f.rv = a.rmean ? a.rvar[c] : 0.f;
    } else {
        f.b = 0.f;
        f.rm = a.save_mean[c];
        f.rv = a.save_invstd[c];
    }
    return f;
}

// SC1: the coefficients are published with write-through stores (read by the other
// blocks of the same launch in the fused forward, k_bn_fwd_fused)
template <int MODE, bool SC1 = false, bool CENTER = false>
__device__ __forceinline__ void finalize(const ReduceArgs& a, int c, double S1, double S2, double invM,
                                         const FinOps& f) {
    const int C = a.C;
    const double g = (double)f.g;
    if (MODE == FWD) {
        const double mean = S1 * invM;
        double var = S2 * invM - mean * mean;
        if (var < 0.0) var = 0.0;
        const double invstd = 1.0 / sqrt(var + (double)a.eps);
        const double sc = g * invstd;
        a.coef[c] = (float)sc;
        a.coef[C + c] = (float)((double)f.b - mean * sc);
        if (SC1) {
            st_sc1(&a.coef[c], a.coef[c]);
            st_sc1(&a.coef[C + c], a.coef[C + c]);
        }
        if (a.coef_out) {
            a.coef_out[c] = a.coef[c];
            a.coef_out[C + c] = a.coef[C + c];
        }
        a.save_mean[c] = (float)mean;
        a.save_invstd[c] = (float)invstd;
        if (a.rmean) {
            const double m = (double)a.momentum;
            const double unb = a.M > 1 ? var * (double)a.M / (double)(a.M - 1) : var;
            a.rmean[c] = (float)((1.0 - m) * (double)f.rm + m * mean);
            a.rvar[c] = (float)((1.0 - m) * (double)f.rv + m * unb);
        }
    } else {
        const double mean = (double)f.rm;
        const double is = (double)f.rv;
        const double ca = g * is;
        const double cb = -g * is * is * is * S2 * invM;
        a.coef[c] = (float)ca;
        a.coef[C + c] = (float)cb;
        if (CENTER) {  // dx = ca*dz + cb*(x - mean) + cc (fp32 path: no cb*x - cb*mean cancellation)
            a.coef[2 * C + c] = (float)(-ca * S1 * invM);
            a.coef[3 * C + c] = (float)mean;
        } else {
            a.coef[2 * C + c] = (float)(-ca * S1 * invM - cb * mean);
        }
        if (SC1) {
            st_sc1(&a.coef[c], a.coef[c]);
            st_sc1(&a.coef[C + c], a.coef[C + c]);
            st_sc1(&a.coef[2 * C + c], a.coef[2 * C + c]);
        }
        const float dg = (float)(S2 * is), db = (float)S1;
        if (a.accumulate) {
            a.dgamma[c] += dg;
            a.dbeta[c] += db;
        } else {
            a.dgamma[c] = dg;
            a.dbeta[c] = db;
        }
    }
}

// Cross-workgroup hand-off without fences (cdna_hip_programming.md, in-launch
// split-K recipe, sc1 form): partials are written with agent-scope atomic stores
// (write-through sc1), every wave drains vmcnt, the block barriers, lane 0 takes a
// relaxed agent-scope ticket; the block that draws the last ticket reads the
// partials back with agent-scope atomic loads (sc1), so no L2 write-back or
// invalidate is needed.  Returns true in that last block.

__device__ __forceinline__ bool ticket(unsigned* ctr, unsigned n, float* flag) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        const unsigned tk = __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const bool last = tk == n - 1;
        if (last) __hip_atomic_store(ctr, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // reset
        *flag = last ? 1.f : 0.f;
    }
    __syncthreads();
    return *flag != 0.f;
}

template <int MODE, bool SC1 = false>
__device__ __forceinline__ void combine_finalize(const ReduceArgs& a, int cs, float* red, const FinOps& fo);

// One launch: partial sums per (row chunk, channel slice) + one ticketed combine
// per slice + per-channel finalize.
template <int MODE, typename E>
__global__ __launch_bounds__(kT) void k_bn_reduce(ReduceArgs a0) {
    const ReduceArgs a = group_args(a0);
    __shared__ float red[kRedF + 4];  // the one LDS object: row-group partials, flag
    const int t = threadIdx.x;
    const int C = a.C, SW = a.SW;
    const int rc = blockIdx.x, cs = blockIdx.y;
    const int tpr = 1 << a.tpr_log;
    const int cg = t & (tpr - 1);
    const int r0 = t >> a.tpr_log;
    const int rpp = kT >> a.tpr_log;
    const long long vpr = C >> 3;                     // 16-B vectors per row
    const int c0 = cs * SW + cg * 8;                  // first channel of this thread

    float fsc[8], fsh[8];
    if (MODE == BWD_RELUX) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            fsc[j] = a.fcoef[c0 + j];
            fsh[j] = a.fcoef[C + c0 + j];
        }
    }
    float mu[8];
    if (MODE != FWD) {
#pragma unroll
        for (int j = 0; j < 8; ++j) mu[j] = a.save_mean[c0 + j];
    }
    float s1[8], s2[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) s1[j] = s2[j] = 0.f;

    const long long rbeg = (long long)rc * a.rpb;
    long long rend = rbeg + a.rpb;
    if (rend > a.M) rend = a.M;
    long long r = rbeg + r0;
    const long long cv = c0 >> 3;
    const long long st = (long long)rpp * vpr;
    for (; r + 7 * rpp < rend; r += 8 * rpp) {
        const long long v = r * vpr + cv;
#pragma unroll
        for (int u = 0; u < 8; ++u) accum<MODE, E>(a, v + u * st, mu, s1, s2, fsc, fsh);
    }
    if (MODE == FWD && std::is_same<E, uint16_t>::value && r < rend) {  // the tail as ONE predicated batch
        const uint4* X = static_cast<const uint4*>(a.x);
        uint4 vx[8];
        const uint4 z = make_uint4(0u, 0u, 0u, 0u);
#pragma unroll
        for (int u = 0; u < 8; ++u) vx[u] = X[(r + u * rpp < rend ? r + u * rpp : r) * vpr + cv];
#pragma unroll
        for (int u = 0; u < 8; ++u) accum_vals<MODE>(r + u * rpp < rend ? vx[u] : z, z, z, mu, s1, s2);
    } else {
        for (; r < rend; r += rpp) accum<MODE, E>(a, r * vpr + cv, mu, s1, s2, fsc, fsh);
    }

    // row-group combine in LDS: red[r0][SW][2]  (rpp * 2SW == 4096 floats)
    const int S2w = 2 * SW;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        red[r0 * S2w + (cg * 8 + j) * 2] = s1[j];
        red[r0 * S2w + (cg * 8 + j) * 2 + 1] = s2[j];
    }
    __syncthreads();
    float* p1 = a.part + ((size_t)cs * a.nrc + rc) * S2w;
    if (t < S2w) {
        float acc = 0.f;
        for (int i = 0; i < rpp; ++i) acc += red[i * S2w + t];
        st_sc1(&p1[t], acc);
    }
    FinOps fo{};
    if (t < SW) fo = fin_load<MODE>(a, cs * SW + t);  // in flight with the partial store
    // the last block of the slice combines its nrc partial rows: lane group of L
    // threads per row (one float4 each), G = 256/L row groups, rows g, g+G, ...
    if (!ticket(a.counter + cs, (unsigned)a.nrc, &red[kRedF])) return;
    combine_finalize<MODE>(a, cs, red, fo);
}

// The last block of a slice: combine the slice's nrc partial rows (lane group of L
// threads per row, one float4 each, G = 256/L row groups, rows g, g+G, ...) in fp64
// and finalize the slice's channels.
template <int MODE, bool SC1>
__device__ __forceinline__ void combine_finalize(const ReduceArgs& a, int cs, float* red, const FinOps& fo) {
    const int t = threadIdx.x;
    const int SW = a.SW, S2w = 2 * SW;
    if (MODE == FWD && a.nbt && cs == 0 && t == 0) *a.nbt += 1;
    const int L = S2w >> 2, G = kT / L;  // L in {4..32}, G in {8..64}
    const int lv = t % L, g = t / L;
    const auto rq = rsrc_of(a.part + (size_t)cs * a.nrc * S2w);
    double d0 = 0.0, d1 = 0.0, d2 = 0.0, d3 = 0.0;
    for (int i0 = g; i0 < a.nrc; i0 += 8 * G) {  // 8 independent 16-B loads in flight
        float4 v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int i = i0 + u * G;
            v[u] = i < a.nrc ? ld_sc1_f32x4(rq, (unsigned)(i * S2w + 4 * lv) * 4u) : make_float4(0.f, 0.f, 0.f, 0.f);
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            d0 += (double)v[u].x; d1 += (double)v[u].y; d2 += (double)v[u].z; d3 += (double)v[u].w;
        }
    }
    __syncthreads();  // red[] is free again
    double* rd = reinterpret_cast<double*>(red);  // [G][S2w] doubles: G * S2w == 2 * kT <= kRedF / 2
    rd[g * S2w + 4 * lv + 0] = d0;
    rd[g * S2w + 4 * lv + 1] = d1;
    rd[g * S2w + 4 * lv + 2] = d2;
    rd[g * S2w + 4 * lv + 3] = d3;
    __syncthreads();
    if (t < SW) {
        double S1 = 0.0, S2 = 0.0;
        for (int i = 0; i < G; ++i) {
            S1 += rd[i * S2w + 2 * t];
            S2 += rd[i * S2w + 2 * t + 1];
        }
        finalize<MODE, SC1>(a, cs * SW + t, S1, S2, 1.0 / (double)a.M, fo);
    }
}

// ---------------------------------------------------------------------------------
// The stem's max-pool backward gathered straight into its BatchNorm + ReLU backward
// (torchvision stem: relu(bn1(x)) -> MaxPool2d(3, 2, 1); reference src/model.py:65-106).
// The pool gradient dz (input resolution, 205 MB at C2) is never written: each thread owns
// a 2 x 2 block of input pixels (rows 2k, 2k+1, columns 2l, 2l+1) x 8 channels and gathers
// their pool gradient from the (at most) 2 x 2 windows (k..k+1, l..l+1) that can select
// them - one window read serves four pixels instead of the per-pixel gather's one (four
// times fewer L2 reads than k_maxpool_bwd) - summed in k_maxpool_bwd's order (window row,
// then column, ascending) and rounded to bf16 as k_maxpool_bwd stores it, then masked by
// the forward's ReLU (x*sc + sh > 0).  Pass 1 (APPLY = false) reduces S1 = sum dz,
// S2 = sum dz*(x - mean) per channel into partial rows + the ticketed fp64 combine and
// finalize of k_bn_reduce; pass 2 applies dx = ca*dz + cb*x + cc.  HBM: pass 1 reads x and
// the pooled gradient + argmax, pass 2 the same and writes dx - against k_maxpool_bwd
// (read pooled, write dz) + the BN backward (read dz and x twice, write dx).
// With xs (the forward's selected raw x per pooled output) pass 1 needs no pixel gather:
// S1 and S2 are linear in the per-pixel gradient, so they sum over the pooled outputs -
// dy_pool * mask(xs) and dy_pool * mask(xs) * (xs - mean) - reading the pooled gradient and
// xs (a quarter of the pixels, 2 x 51 MB at C2) instead of x, the gradient and the argmax.
// (The per-pixel bf16 rounding of the gathered gradient, which pass 2 applies to dx, is not
// applied to these sums: they are the fp32 sums of the same terms.)
struct StemPoolGeo {
    int Ng, H, W, P, Q;      // images per view group, input and pooled sizes
    long long items;         // owner blocks x channel groups per view group
    long long ipb;           // items per block (pass 1; a multiple of kT)
    const uint2* idx;        // [G*Ng][P][Q][C] window-relative argmax bytes
    const uint4* gp;         // [G*Ng][P][Q][C] bf16 pool gradient
    const uint4* xs;         // [G*Ng][P][Q][C] bf16 selected x (optional)
};

typedef unsigned u32x4v_t __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint4 ld_nt16(const uint4* p) {  // streamed once: nontemporal
    const u32x4v_t v = __builtin_nontemporal_load(reinterpret_cast<const u32x4v_t*>(p));
    return make_uint4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ void st_nt16(uint4* p, uint4 v) {
    const u32x4v_t w = {v.x, v.y, v.z, v.w};
    __builtin_nontemporal_store(w, reinterpret_cast<u32x4v_t*>(p));
}

template <bool APPLY>
__global__ __launch_bounds__(kT) void k_stem_pool_bn_bwd(ReduceArgs a0, StemPoolGeo pg) {
    const ReduceArgs a = group_args(a0);
    __shared__ float red[kRedF + 4];
    const int t = threadIdx.x;
    const int C = a.C, C8 = C >> 3;
    const int g = blockIdx.z;
    const long long goff = (long long)g * pg.Ng * pg.P * pg.Q * C8;  // this group's pooled vectors
    const uint2* __restrict__ IDX = pg.idx + goff;
    const uint4* __restrict__ GP = pg.gp + goff;
    const uint4* __restrict__ X = static_cast<const uint4*>(a.x);
    float fsc[8], fsh[8], mu[8], ca[8], cb[8], cc[8];
    const int cg0 = t % C8;  // fixed per thread in pass 1 (kT and the block base are multiples of C8)
    auto ld_coef = [&](const float* p, int cg, float* v) {
        const float4 u0 = *reinterpret_cast<const float4*>(p + cg * 8);
        const float4 u1 = *reinterpret_cast<const float4*>(p + cg * 8 + 4);
        v[0] = u0.x; v[1] = u0.y; v[2] = u0.z; v[3] = u0.w; v[4] = u1.x; v[5] = u1.y; v[6] = u1.z; v[7] = u1.w;
    };
    ld_coef(a.fcoef, cg0, fsc);
    ld_coef(a.fcoef + C, cg0, fsh);
    if (!APPLY) ld_coef(a.save_mean, cg0, mu);
    else {
        ld_coef(a.coef, cg0, ca);
        ld_coef(a.coef + C, cg0, cb);
        ld_coef(a.coef + 2 * C, cg0, cc);
    }
    float s1[8], s2[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) s1[j] = s2[j] = 0.f;
    // one owner block x channel group, in two phases (loads, then arithmetic) so that a
    // thread keeps UI items' loads in flight together
    struct Item {
        uint2 iv[4];
        uint4 gq[4], xv[4];
        int n, k, l, cg;
        unsigned okw;  // bit u: window u exists (a select on the loaded value instead would
                       // make hipcc branch around the load and drain vmcnt per window)
    };
    // 32-bit index math (a group's pooled and input vectors are < 2^31: checked on the host)
    const unsigned QC8 = (unsigned)pg.Q * C8, WC8 = (unsigned)pg.W * C8;
    auto load = [&](long long i64, Item& it) {
        const unsigned i = (unsigned)i64;
        const unsigned ob = i / (unsigned)C8;
        it.cg = (int)(i - ob * (unsigned)C8);
        const unsigned r1 = ob / (unsigned)pg.Q;
        it.l = (int)(ob - r1 * (unsigned)pg.Q);
        const unsigned nn = r1 / (unsigned)pg.P;
        it.k = (int)(r1 - nn * (unsigned)pg.P);
        it.n = (int)nn;
        const int k = it.k, l = it.l;
        // windows (k + wr, l + wc); pixel (dh, dw) of the block is covered by window
        // (k + wr, l + wc) iff wr <= dh and wc <= dw (and the window exists)
        const unsigned o0 = i;  // the block's own window (k, l) = pooled vector i
        it.okw = 0u;
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int wr = u >> 1, wc = u & 1;
            const bool ok = k + wr < pg.P && l + wc < pg.Q;
            const unsigned o = ok ? o0 + (unsigned)wr * QC8 + (unsigned)wc * (unsigned)C8 : o0;
            it.iv[u] = IDX[o];
            it.gq[u] = GP[o];
            it.okw |= ok ? (1u << u) : 0u;
        }
        const unsigned x0 = ((nn * (unsigned)pg.H + 2u * (unsigned)k) * (unsigned)pg.W + 2u * (unsigned)l) * C8 + it.cg;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int dh = q >> 1, dw = q & 1;
            const bool in = 2 * k + dh < pg.H && 2 * l + dw < pg.W;
            it.xv[q] = ld_nt16(&X[in ? x0 + (unsigned)dh * WC8 + (unsigned)dw * (unsigned)C8 : x0]);
        }
    };
    auto compute = [&](const Item& it) {
        const int n = it.n, k = it.k, l = it.l, cg = it.cg;
        float gv[4][8];
#pragma unroll
        for (int u = 0; u < 4; ++u) unpack8(it.gq[u], gv[u]);
        // a missing window's argmax bytes become 0xff (never a position 0..8): one select per
        // window here instead of a mask AND per channel compare below
        uint2 ivm[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) ivm[u] = ((it.okw >> u) & 1u) ? it.iv[u] : make_uint2(~0u, ~0u);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int dh = q >> 1, dw = q & 1;
            const int h = 2 * k + dh, w = 2 * l + dw;
            if (h >= pg.H || w >= pg.W) continue;
            float d[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) d[j] = 0.f;
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int wr = u >> 1, wc = u & 1;
                if (wr > dh || wc > dw) continue;
                // position of pixel (h, w) in window (k + wr, l + wc): rows 2(k+wr)-1 .., cols 2(l+wc)-1 ..
                // (h - 2k = dh, w - 2l = dw: a compile-time constant per (q, u))
                const uint32_t pos = (uint32_t)((dh - 2 * wr + 1) * 3 + (dw - 2 * wc + 1));
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const uint32_t b = ((j < 4 ? ivm[u].x : ivm[u].y) >> (8 * (j & 3))) & 0xffu;
                    if (b == pos) d[j] += gv[u][j];
                }
            }
            float xf[8];
            unpack8(it.xv[q], xf);
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const float dr = __uint_as_float((uint32_t)Elem<uint16_t>::f2bf(d[j]) << 16);  // k_maxpool_bwd's bf16 dz
                d[j] = fmaf(xf[j], fsc[j], fsh[j]) > 0.f ? dr : 0.f;
            }
            if (APPLY) {
                float o[8];
#pragma unroll
                for (int j = 0; j < 8; ++j) o[j] = fmaf(ca[j], d[j], fmaf(cb[j], xf[j], cc[j]));
                st_nt16(&reinterpret_cast<uint4*>(a.yout)[(((long long)n * pg.H + h) * pg.W + w) * C8 + cg], pack8(o));
            } else {
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    s1[j] += d[j];
                    s2[j] = fmaf(d[j], xf[j] - mu[j], s2[j]);
                }
            }
        }
    };
    auto item = [&](long long i) {
        Item it;
        load(i, it);
        compute(it);
    };
    if (APPLY) {
        // (the coefficient registers hold channel group cg0: a grid-stride step is a multiple of C8)
        // two items' loads in flight per thread
        const long long stride = (long long)gridDim.x * kT;
        long long i = (long long)blockIdx.x * kT + t;
        for (; i + stride < pg.items; i += 2 * stride) {
            Item u, v;
            load(i, u);
            load(i + stride, v);
            compute(u);
            compute(v);
        }
        if (i < pg.items) item(i);
        return;
    }
    const int rc = blockIdx.x;
    const long long i0 = (long long)rc * pg.ipb;
    const long long i1 = i0 + pg.ipb < pg.items ? i0 + pg.ipb : pg.items;
    if (pg.xs) {
        // pooled outputs i (an item index is a pooled (n, k, l, cg) vector: the same decode)
        const uint4* __restrict__ XS = pg.xs + goff;
        for (long long i = i0 + t; i < i1; i += 4 * kT) {
            uint4 gq[4], xq[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {  // four vectors' loads in flight
                const long long iu = i + u * kT < i1 ? i + u * kT : i;
                gq[u] = GP[iu];
                xq[u] = XS[iu];
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                if (i + u * kT >= i1) break;
                float gv[8], xf[8];
                unpack8(gq[u], gv);
                unpack8(xq[u], xf);
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const float d = fmaf(xf[j], fsc[j], fsh[j]) > 0.f ? gv[j] : 0.f;
                    s1[j] += d;
                    s2[j] = fmaf(d, xf[j] - mu[j], s2[j]);
                }
            }
        }
    } else {
        for (long long i = i0 + t; i < i1; i += kT) item(i);  // (two items in flight per thread: slower)
    }
    // row-group combine in LDS as k_bn_reduce: red[r0][SW][2], r0 = t / C8 (C8 threads per row)
    const int S2w = 2 * C, r0 = t / C8, rpp = kT / C8;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        red[r0 * S2w + (cg0 * 8 + j) * 2] = s1[j];
        red[r0 * S2w + (cg0 * 8 + j) * 2 + 1] = s2[j];
    }
    __syncthreads();
    float* p1 = a.part + (size_t)rc * S2w;
    if (t < S2w) {
        float acc = 0.f;
        for (int i = 0; i < rpp; ++i) acc += red[i * S2w + t];
        st_sc1(&p1[t], acc);
    }
    FinOps fo{};
    if (t < C) fo = fin_load<BWD_RELUX>(a, t);
    if (!ticket(a.counter, (unsigned)a.nrc, &red[kRedF])) return;
    combine_finalize<BWD_RELUX>(a, 0, red, fo);
}

// Finalize of BatchNorm forward statistics whose per-workgroup partial rows were written by
// the producer (k_conv_stem's epilogue): one block per view group combines the rows in fp64
// (fixed order) and finalizes as k_bn_reduce's last block does.  a0.part / a0.coef: group 0's
// rows and coefficient area, the groups scr_stride bytes apart.
// 1024 threads per (64-channel slice, group): 32 lanes per partial row (one float4 each), 32
// row groups with 8 rows' loads in flight each (the producers' rows are many - a 3x3 layer-2
// convolution writes one per 64-pixel slab - and the combine sits on the forward's critical
// path), fp64, then the row groups combined in a fixed order.
constexpr int kFinT = 1024;
__global__ __launch_bounds__(kFinT) void k_bn_stats_finalize(ReduceArgs a0) {
    const ReduceArgs a = group_args(a0);
    __shared__ double rd[kFinT / 32][128];
    const int t = threadIdx.x, cs = blockIdx.y;  // channel slice cs (64 channels)
    const int lv = t & 31, rg = t >> 5;
    FinOps fo;
    {  // every thread, no branch (a conditional load here cost wave 0 a waited round trip
       // before its row loads); threads t >= 64 load channel t % 64's again, unused
        const int c = cs * 64 + (t & 63);
        const float* rm = a.rmean ? a.rmean : a.gamma;
        const float* rv = a.rmean ? a.rvar : a.gamma;
        fo.g = a.gamma[c];
        fo.b = a.beta[c];
        fo.rm = rm[c];
        fo.rv = rv[c];
    }
    const float4* rows = reinterpret_cast<const float4*>(a.part + (size_t)cs * a.nrc * 128);
    double d0 = 0.0, d1 = 0.0, d2 = 0.0, d3 = 0.0;
    for (int i0 = rg; i0 < a.nrc; i0 += 8 * 32) {
        float4 v[8];  // clamped rows, all eight loads in flight, then the value select (a
#pragma unroll    // conditional load compiled to a branch and a full wait per row)
        for (int u = 0; u < 8; ++u) v[u] = rows[(size_t)min(i0 + u * 32, a.nrc - 1) * 32 + lv];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            if (i0 + u * 32 >= a.nrc) v[u] = make_float4(0.f, 0.f, 0.f, 0.f);
            d0 += (double)v[u].x; d1 += (double)v[u].y; d2 += (double)v[u].z; d3 += (double)v[u].w;
        }
    }
    rd[rg][4 * lv] = d0; rd[rg][4 * lv + 1] = d1; rd[rg][4 * lv + 2] = d2; rd[rg][4 * lv + 3] = d3;
    __syncthreads();
    if (t < 64) {
        double S1 = 0.0, S2 = 0.0;
        for (int i = 0; i < kFinT / 32; ++i) {
            S1 += rd[i][2 * t];
            S2 += rd[i][2 * t + 1];
        }
        finalize<FWD>(a, cs * 64 + t, S1, S2, 1.0 / (double)a.M, fo);  // (rm / rv unused without rmean)
        if (a.nbt && cs == 0 && t == 0) *a.nbt += 1;
    }
}

// The backward's statistics (sum dz, sum dz * (x - mean) per channel) from producer partial
// rows (the input-gradient convolution's epilogue, gm_conv2d_dgrad_grouped_bn_stats_bf16):
// combined like k_bn_stats_finalize, then finalize<BWD> - dgamma / dbeta (accumulate) and the
// apply's coefficients ca, cb, cc at coef0 + g * cstride (the partial rows' group blocks are
// packed: no room for 3 C coefficients at their end).
__global__ __launch_bounds__(kFinT) void k_bn_bwd_stats_finalize(ReduceArgs a0, float* coef0, long long cstride) {
    ReduceArgs a = group_args(a0);
    a.coef = coef0 + blockIdx.z * cstride;
    __shared__ double rd[kFinT / 32][128];
    const int t = threadIdx.x, cs = blockIdx.y;
    const int lv = t & 31, rg = t >> 5;
    const FinOps fo = fin_load<BWD>(a, cs * 64 + (t & 63));  // every thread: no branch, no early wait
    const float4* rows = reinterpret_cast<const float4*>(a.part + (size_t)cs * a.nrc * 128);
    double d0 = 0.0, d1 = 0.0, d2 = 0.0, d3 = 0.0;
    for (int i0 = rg; i0 < a.nrc; i0 += 8 * 32) {
        float4 v[8];  // clamped rows, all eight loads in flight, then the value select (a
#pragma unroll    // conditional load compiled to a branch and a full wait per row)
        for (int u = 0; u < 8; ++u) v[u] = rows[(size_t)min(i0 + u * 32, a.nrc - 1) * 32 + lv];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            if (i0 + u * 32 >= a.nrc) v[u] = make_float4(0.f, 0.f, 0.f, 0.f);
            d0 += (double)v[u].x; d1 += (double)v[u].y; d2 += (double)v[u].z; d3 += (double)v[u].w;
        }
    }
    rd[rg][4 * lv] = d0; rd[rg][4 * lv + 1] = d1; rd[rg][4 * lv + 2] = d2; rd[rg][4 * lv + 3] = d3;
    __syncthreads();
    if (t < 64) {
        double S1 = 0.0, S2 = 0.0;
        for (int i = 0; i < kFinT / 32; ++i) {
            S1 += rd[i][2 * t];
            S2 += rd[i][2 * t + 1];
        }
        finalize<BWD>(a, cs * 64 + t, S1, S2, 1.0 / (double)a.M, fo);
    }
}

// ---------------------------------------------------------------------------------
// Redundant-finalize hand-off of the single-launch kernels for small maps (a.redundant):
// the last-arriving block no longer combines, finalizes, publishes the coefficients and a
// generation word that the other blocks poll and then read the coefficients from - four
// dependent memory round trips after the last partial row lands.  Every block polls the
// slice's ticket counter itself (the partial rows' writers add to it after their sc1
// stores: cdna_hip_programming.md Guideline 16, the sc1 poll row), combines the <= nrc
// partial rows (sc1 loads, fp64, the fixed order of combine_finalize: every block computes
// the same coefficients) and keeps the coefficients in LDS; the block whose ticket came
// last also writes the side outputs (statistics, running averages, counter, coef_out /
// dgamma, dbeta) through finalize().  The counter then counts a second round (each block
// once it has seen nrc arrivals), and the block completing that round re-zeroes it, so
// no poller can miss the value nrc and the ticket words are zero between calls again.
__device__ __forceinline__ bool arrive(unsigned* ctr, unsigned n, float* flag) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        const unsigned tk = __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        *flag = tk == n - 1 ? 1.f : 0.f;
    }
    __syncthreads();
    return *flag != 0.f;
}

__device__ __forceinline__ bool wait_count(unsigned* ctr, unsigned n, unsigned limit, float* flag) {
    if (threadIdx.x == 0) {
        unsigned it = 0;
        bool ok = true;
        while (__hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < n) {
            if (++it >= limit) {
                ok = false;
                break;
            }
            __builtin_amdgcn_s_sleep(1);
        }
        if (!ok) atomicOr(&g_bn_fault, GM_FAULT_BN_SPIN);
        *flag = ok ? 1.f : 0.f;
    }
    __syncthreads();
    return *flag != 0.f;
}

__device__ __forceinline__ void depart(unsigned* ctr, unsigned n) {
    if (threadIdx.x == 0) {
        const unsigned tk = __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (tk == 2 * n - 1) __hip_atomic_store(ctr, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

// the slice's coefficients into cf[3][SW] (LDS): FWD sc, sh; BWD ca, cb, cc (bf16 form)
template <int MODE>
__device__ __forceinline__ void combine_coefs(const ReduceArgs& a, int cs, float* red, const FinOps& fo, bool last,
                                              float* cf) {
    const int t = threadIdx.x;
    const int SW = a.SW, S2w = 2 * SW;
    const int L = S2w >> 2, G = kT / L;
    const int lv = t % L, g = t / L;
    const auto rq = rsrc_of(a.part + (size_t)cs * a.nrc * S2w);
    double d0 = 0.0, d1 = 0.0, d2 = 0.0, d3 = 0.0;
    for (int i0 = g; i0 < a.nrc; i0 += 8 * G) {
        float4 v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int i = i0 + u * G;
            v[u] = i < a.nrc ? ld_sc1_f32x4(rq, (unsigned)(i * S2w + 4 * lv) * 4u) : make_float4(0.f, 0.f, 0.f, 0.f);
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            d0 += (double)v[u].x; d1 += (double)v[u].y; d2 += (double)v[u].z; d3 += (double)v[u].w;
        }
    }
    __syncthreads();
    double* rd = reinterpret_cast<double*>(red);
    rd[g * S2w + 4 * lv + 0] = d0;
    rd[g * S2w + 4 * lv + 1] = d1;
    rd[g * S2w + 4 * lv + 2] = d2;
    rd[g * S2w + 4 * lv + 3] = d3;
    __syncthreads();
    if (t < SW) {
        double S1 = 0.0, S2 = 0.0;
        for (int i = 0; i < G; ++i) {
            S1 += rd[i * S2w + 2 * t];
            S2 += rd[i * S2w + 2 * t + 1];
        }
        const double invM = 1.0 / (double)a.M;
        const int c = cs * SW + t;
        if (last) {
            if (MODE == FWD && a.nbt && cs == 0 && t == 0) *a.nbt += 1;
            finalize<MODE, false>(a, c, S1, S2, invM, fo);
        }
        const double gg = (double)fo.g;
        if (MODE == FWD) {
            const double mean = S1 * invM;
            double var = S2 * invM - mean * mean;
            if (var < 0.0) var = 0.0;
            const double invstd = 1.0 / sqrt(var + (double)a.eps);
            const double sc = gg * invstd;
            cf[t] = (float)sc;
            cf[SW + t] = (float)((double)fo.b - mean * sc);
        } else {
            const double mean = (double)fo.rm, is = (double)fo.rv;
            const double ca = gg * is, cb = -gg * is * is * is * S2 * invM;
            cf[t] = (float)ca;
            cf[SW + t] = (float)cb;
            cf[2 * SW + t] = (float)(-ca * S1 * invM - cb * mean);
        }
    }
    __syncthreads();
}

// The reference-precision (fp32) reduce: the reference's CPU BatchNorm accumulates its
// sums in double (ATen acc_type<float> on the CPU), and long fp32 sums of gradients with
// mixed signs lose the digits the parameter gradients are made of (1e-3 relative at
// 224x224 maps, measured).  So every level accumulates in fp64: per-thread sums, the
// row-group combine, the per-block partials (sc1 stores, 8 B) and the last block's
// combine; the centred backward coefficients (finalize<CENTER>).
template <int MODE>
__global__ __launch_bounds__(kT) void k_bn_reduce_f64(ReduceArgs a0) {
    const ReduceArgs a = group_args(a0);
    __shared__ double red[kRedF];  // rpp * 2 * SW == 4096 doubles
    __shared__ float flag;
    const int t = threadIdx.x;
    const int C = a.C, SW = a.SW;
    const int rc = blockIdx.x, cs = blockIdx.y;
    const int tpr = 1 << a.tpr_log;
    const int cg = t & (tpr - 1);
    const int r0 = t >> a.tpr_log;
    const int rpp = kT >> a.tpr_log;
    const long long vpr = C >> 3;
    const int c0 = cs * SW + cg * 8;
    const float* X = static_cast<const float*>(a.x);
    const float* DY = static_cast<const float*>(a.dy);
    const float* Y = static_cast<const float*>(a.y);
    double fsc[8], fsh[8], mu[8], s1[8], s2[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        fsc[j] = MODE == BWD_RELUX ? (double)a.fcoef[c0 + j] : 0.0;
        fsh[j] = MODE == BWD_RELUX ? (double)a.fcoef[C + c0 + j] : 0.0;
        mu[j] = MODE != FWD ? (double)a.save_mean[c0 + j] : 0.0;
        s1[j] = s2[j] = 0.0;
    }
    const long long rbeg = (long long)rc * a.rpb;
    long long rend = rbeg + a.rpb;
    if (rend > a.M) rend = a.M;
    for (long long r = rbeg + r0; r < rend; r += rpp) {
        const long long e = r * C + c0;
        float xf[8], d[8];
        V8<float>::ld(X + e, 0, xf);
        if (MODE != FWD) V8<float>::ld(DY + e, 0, d);
        if (MODE == BWD_RELU) {
            float yf[8];
            V8<float>::ld(Y + e, 0, yf);
#pragma unroll
            for (int j = 0; j < 8; ++j) d[j] = yf[j] > 0.f ? d[j] : 0.f;
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            if (MODE == BWD_RELUX) d[j] = fmaf(xf[j], (float)fsc[j], (float)fsh[j]) > 0.f ? d[j] : 0.f;
            if (MODE == FWD) {
                s1[j] += (double)xf[j];
                s2[j] = fma((double)xf[j], (double)xf[j], s2[j]);
            } else {
                s1[j] += (double)d[j];
                s2[j] = fma((double)d[j], (double)xf[j] - mu[j], s2[j]);
            }
        }
    }
    const int S2w = 2 * SW;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        red[r0 * S2w + (cg * 8 + j) * 2] = s1[j];
        red[r0 * S2w + (cg * 8 + j) * 2 + 1] = s2[j];
    }
    __syncthreads();
    double* p1 = reinterpret_cast<double*>(a.part) + ((size_t)cs * a.nrc + rc) * S2w;
    if (t < S2w) {
        double acc = 0.0;
        for (int i = 0; i < rpp; ++i) acc += red[i * S2w + t];
        st_sc1(&p1[t], acc);
    }
    FinOps fo{};
    if (t < SW) fo = fin_load<MODE>(a, cs * SW + t);
    if (!ticket(a.counter + cs, (unsigned)a.nrc, &flag)) return;
    if (MODE == FWD && a.nbt && cs == 0 && t == 0) *a.nbt += 1;
    const double* pp = reinterpret_cast<const double*>(a.part) + (size_t)cs * a.nrc * S2w;
    if (t < S2w) {  // fixed order over the row chunks
        double acc = 0.0;
        for (int i = 0; i < a.nrc; ++i)
            acc += __hip_atomic_load(pp + (size_t)i * S2w + t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        red[t] = acc;
    }
    __syncthreads();
    if (t < SW) finalize<MODE, false, true>(a, cs * SW + t, red[2 * t], red[2 * t + 1], 1.0 / (double)a.M, fo);
}

// Fused forward for maps whose grid is co-resident (fused_plan) and whose rows
// fit NR 16-B vectors per thread: the block keeps its x strip in registers, takes
// its ticket, the slice's last block finalizes and publishes the coefficients
// (write-through stores, then a generation word), the other blocks spin on the
// generation word (bounded) and every block applies y = relu?(x*sc + sh (+res)) from
// its registers.  One launch and one read of x instead of two launches and two reads.

template <bool RES, bool RELU, int NR>
__global__ __launch_bounds__(kT, NR == 16 ? 2 : NR == 8 ? 3 : 4) void k_bn_fwd_fused(ReduceArgs a0) {  // NR 0: streaming
    const ReduceArgs a = group_args(a0);
    __shared__ float red[kRedF + 4];
    const int t = threadIdx.x;
    const int C = a.C, SW = a.SW;
    const int rc = blockIdx.x, cs = blockIdx.y;
    const int tpr = 1 << a.tpr_log;
    const int cg = t & (tpr - 1);
    const int r0 = t >> a.tpr_log;
    const int rpp = kT >> a.tpr_log;
    const long long vpr = C >> 3;
    const int c0 = cs * SW + cg * 8;
    const long long cv = c0 >> 3;
    unsigned* gen = a.gen + cs;
    unsigned g0 = 0;
    if (t == 0) g0 = __hip_atomic_load(gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint4* X = static_cast<const uint4*>(a.x);

    const long long rbeg = (long long)rc * a.rpb;
    long long rend = rbeg + a.rpb;
    if (rend > a.M) rend = a.M;
    const uint4 z = make_uint4(0u, 0u, 0u, 0u);
    constexpr int NV = NR > 0 ? NR : 1;
    uint4 v[NV];
    float s1[8], s2[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) s1[j] = s2[j] = 0.f;
    if (NR > 0) {
#pragma unroll
        for (int u = 0; u < NV; ++u) {  // clamped loads (always valid), then a value select
            const long long r = rbeg + r0 + (long long)u * rpp;
            const uint4 w = X[(r < rend ? r : rend - 1) * vpr + cv];
            v[u] = r < rend ? w : z;
        }
#pragma unroll
        for (int u = 0; u < NV; ++u) accum_vals<FWD>(v[u], z, z, nullptr, s1, s2);
    } else {  // streaming: 8 rows in flight per thread, x re-read (L2 / MALL) by the apply
        long long r = rbeg + r0;
        const long long st = (long long)rpp * vpr;
        for (; r + 7 * rpp < rend; r += 8 * rpp) {
            uint4 w[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) w[u] = X[r * vpr + cv + u * st];
#pragma unroll
            for (int u = 0; u < 8; ++u) accum_vals<FWD>(w[u], z, z, nullptr, s1, s2);
        }
        for (; r < rend; r += rpp) accum_vals<FWD>(X[r * vpr + cv], z, z, nullptr, s1, s2);
    }

    const int S2w = 2 * SW;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        red[r0 * S2w + (cg * 8 + j) * 2] = s1[j];
        red[r0 * S2w + (cg * 8 + j) * 2 + 1] = s2[j];
    }
    __syncthreads();
    float* p1 = a.part + ((size_t)cs * a.nrc + rc) * S2w;
    if (t < S2w) {
        float acc = 0.f;
        for (int i = 0; i < rpp; ++i) acc += red[i * S2w + t];
        st_sc1(&p1[t], acc);
    }
    FinOps fo{};
    if (t < SW) fo = fin_load<FWD>(a, cs * SW + t);
    bool fresh = true;
    float sc[8], sh[8];
    if (a.redundant) {
        __shared__ float cf[3 * 64];
        const bool last = arrive(a.counter + cs, (unsigned)a.nrc, &red[kRedF]);
        fresh = wait_count(a.counter + cs, (unsigned)a.nrc, a.spin_limit, &red[kRedF + 1]);
        combine_coefs<FWD>(a, cs, red, fo, last, cf);
        depart(a.counter + cs, (unsigned)a.nrc);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            sc[j] = cf[cg * 8 + j];
            sh[j] = cf[SW + cg * 8 + j];
        }
    } else {
        if (ticket(a.counter + cs, (unsigned)a.nrc, &red[kRedF])) {
            combine_finalize<FWD, true>(a, cs, red, fo);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
            if (t == 0) __hip_atomic_store(gen, g0 + 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        } else {
            fresh = wait_generation(gen, g0, a.spin_limit, &red[kRedF + 1]);
        }
        const auto rq = rsrc_of(a.coef);
        const float4 sa = ld_sc1_f32x4(rq, (unsigned)c0 * 4u), sb = ld_sc1_f32x4(rq, (unsigned)(c0 + 4) * 4u);
        const float4 ha = ld_sc1_f32x4(rq, (unsigned)(C + c0) * 4u), hb = ld_sc1_f32x4(rq, (unsigned)(C + c0 + 4) * 4u);
        sc[0] = sa.x; sc[1] = sa.y; sc[2] = sa.z; sc[3] = sa.w; sc[4] = sb.x; sc[5] = sb.y; sc[6] = sb.z; sc[7] = sb.w;
        sh[0] = ha.x; sh[1] = ha.y; sh[2] = ha.z; sh[3] = ha.w; sh[4] = hb.x; sh[5] = hb.y; sh[6] = hb.z; sh[7] = hb.w;
    }
    if (!fresh) {  // timed out: never apply stale coefficients (the fault word is set)
#pragma unroll
        for (int j = 0; j < 8; ++j) sc[j] = sh[j] = __builtin_nanf("");
    }
    auto apply = [&](uint4 xv, long long i) {
        float f[8], q[8];
        unpack8(xv, f);
        if (RES) unpack8(a.res[i], q);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            float zz = fmaf(f[j], sc[j], sh[j]);
            if (RES) zz += q[j];
            f[j] = RELU ? relu_nan(zz) : zz;
            if (!fresh) f[j] = __builtin_nanf("");  // poisoned (fmaxf would turn NaN into 0)
        }
        const uint4 w = pack8(f);
        a.yout[i] = w;
        if (RES && RELU && a.mask_out) a.mask_out[i] = (uint8_t)mask_byte(w);
    };
    if (NR > 0) {
#pragma unroll
        for (int u = 0; u < NV; ++u) {
            const long long r = rbeg + r0 + (long long)u * rpp;
            if (r < rend) apply(v[u], r * vpr + cv);
        }
    } else {
        long long r = rbeg + r0;
        const long long st = (long long)rpp * vpr;
        for (; r + 3 * rpp < rend; r += 4 * rpp) {
            uint4 w[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) w[u] = X[r * vpr + cv + u * st];
#pragma unroll
            for (int u = 0; u < 4; ++u) apply(w[u], r * vpr + cv + u * st);
        }
        for (; r < rend; r += rpp) apply(X[r * vpr + cv], r * vpr + cv);
    }
}

// Fused backward, same scheme as k_bn_fwd_fused: the block holds its x / dy (/ y)
// strip in registers (NR 4 or 8) or re-reads it (NR 0), the slice's last block
// publishes (a, b, c) and every block writes dx = a*dz + b*x + c (and dres = dz).
template <int MODE, bool DRES, int NR, bool YM = false>
__global__ __launch_bounds__(kT, NR == 8 ? 2 : 3) void k_bn_bwd_fused(ReduceArgs a0) {
    const ReduceArgs a = group_args(a0);
    __shared__ float red[kRedF + 4];
    const int t = threadIdx.x;
    const int C = a.C, SW = a.SW;
    const int rc = blockIdx.x, cs = blockIdx.y;
    const int tpr = 1 << a.tpr_log;
    const int cg = t & (tpr - 1);
    const int r0 = t >> a.tpr_log;
    const int rpp = kT >> a.tpr_log;
    const long long vpr = C >> 3;
    const int c0 = cs * SW + cg * 8;
    const long long cv = c0 >> 3;
    unsigned* gen = a.gen + cs;
    unsigned g0 = 0;
    if (t == 0) g0 = __hip_atomic_load(gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint4* X = static_cast<const uint4*>(a.x);
    const uint4* DY = static_cast<const uint4*>(a.dy);
    const uint4* Y = static_cast<const uint4*>(a.y);
    // y for the ReLU mask, or (YM) the forward's mask byte expanded to 1.0 / 0 bf16 values
    auto ldy = [&](long long i) { return YM ? mask_vals(a.ymask[i]) : Y[i]; };
    float mu[8], fsc[8], fsh[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        mu[j] = a.save_mean[c0 + j];
        if (MODE == BWD_RELUX) {
            fsc[j] = a.fcoef[c0 + j];
            fsh[j] = a.fcoef[C + c0 + j];
        }
    }
    const long long rbeg = (long long)rc * a.rpb;
    long long rend = rbeg + a.rpb;
    if (rend > a.M) rend = a.M;
    const uint4 z = make_uint4(0u, 0u, 0u, 0u);
    constexpr int NV = NR > 0 ? NR : 1;
    constexpr int NY = MODE == BWD_RELU ? NV : 1;
    // streaming rows in flight (register budget: y's vectors; the mask bytes (YM) cost one each)
    constexpr int US = MODE == BWD_RELU && !YM ? 2 : 4;
    uint4 vx[NV], vd[NV], vy[NY];
    float s1[8], s2[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) s1[j] = s2[j] = 0.f;
    if (NR > 0) {
#pragma unroll
        for (int u = 0; u < NV; ++u) {  // clamped loads, then value selects (zero rows add nothing)
            const long long r = rbeg + r0 + (long long)u * rpp;
            const long long i = (r < rend ? r : rend - 1) * vpr + cv;
            const uint4 wx = X[i], wd = DY[i];
            vx[u] = r < rend ? wx : z;
            vd[u] = r < rend ? wd : z;
            if (MODE == BWD_RELU) vy[u] = ldy(i);
        }
#pragma unroll
        for (int u = 0; u < NV; ++u)
            accum_vals<MODE>(vx[u], vd[u], MODE == BWD_RELU ? vy[u < NY ? u : 0] : z, mu, s1, s2, fsc, fsh);
    } else {
        long long r = rbeg + r0;
        const long long st = (long long)rpp * vpr;
        for (; r + (US - 1) * rpp < rend; r += US * rpp) {
            uint4 wx[US], wd[US], wy[US];
            unsigned wm[US];
#pragma unroll
            for (int u = 0; u < US; ++u) {
                const long long i = r * vpr + cv + u * st;
                wx[u] = X[i];
                wd[u] = DY[i];
                if (MODE == BWD_RELU && YM) wm[u] = a.ymask[i];
                else if (MODE == BWD_RELU) wy[u] = Y[i];
            }
#pragma unroll
            for (int u = 0; u < US; ++u) {
                pin(wx[u]);
                pin(wd[u]);
                if (MODE == BWD_RELU && YM) pin(wm[u]);
                else if (MODE == BWD_RELU) pin(wy[u]);
            }
#pragma unroll
            for (int u = 0; u < US; ++u)
                accum_vals<MODE>(wx[u], wd[u], MODE == BWD_RELU ? (YM ? mask_vals(wm[u]) : wy[u]) : z, mu, s1, s2, fsc,
                                 fsh);
        }
        for (; r < rend; r += rpp) {
            const long long i = r * vpr + cv;
            accum_vals<MODE>(X[i], DY[i], MODE == BWD_RELU ? ldy(i) : z, mu, s1, s2, fsc, fsh);
        }
    }

    const int S2w = 2 * SW;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        red[r0 * S2w + (cg * 8 + j) * 2] = s1[j];
        red[r0 * S2w + (cg * 8 + j) * 2 + 1] = s2[j];
    }
    __syncthreads();
    float* p1 = a.part + ((size_t)cs * a.nrc + rc) * S2w;
    if (t < S2w) {
        float acc = 0.f;
        for (int i = 0; i < rpp; ++i) acc += red[i * S2w + t];
        st_sc1(&p1[t], acc);
    }
    FinOps fo{};
    if (t < SW) fo = fin_load<MODE>(a, cs * SW + t);
    bool fresh = true;
    float ca[8], cb[8], cc[8];
    if (a.redundant) {
        __shared__ float cf[3 * 64];
        const bool last = arrive(a.counter + cs, (unsigned)a.nrc, &red[kRedF]);
        fresh = wait_count(a.counter + cs, (unsigned)a.nrc, a.spin_limit, &red[kRedF + 1]);
        combine_coefs<MODE>(a, cs, red, fo, last, cf);
        depart(a.counter + cs, (unsigned)a.nrc);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            ca[j] = cf[cg * 8 + j];
            cb[j] = cf[SW + cg * 8 + j];
            cc[j] = cf[2 * SW + cg * 8 + j];
        }
    } else {
        if (ticket(a.counter + cs, (unsigned)a.nrc, &red[kRedF])) {
            combine_finalize<MODE, true>(a, cs, red, fo);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
            if (t == 0) __hip_atomic_store(gen, g0 + 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        } else {
            fresh = wait_generation(gen, g0, a.spin_limit, &red[kRedF + 1]);
        }
        const auto rq = rsrc_of(a.coef);
        auto ld8 = [&](int off, float* o) {
            const float4 p = ld_sc1_f32x4(rq, (unsigned)(off + c0) * 4u), q = ld_sc1_f32x4(rq, (unsigned)(off + c0 + 4) * 4u);
            o[0] = p.x; o[1] = p.y; o[2] = p.z; o[3] = p.w; o[4] = q.x; o[5] = q.y; o[6] = q.z; o[7] = q.w;
        };
        ld8(0, ca);
        ld8(C, cb);
        ld8(2 * C, cc);
    }
    if (!fresh) {  // timed out: never apply stale coefficients (the fault word is set)
#pragma unroll
        for (int j = 0; j < 8; ++j) ca[j] = cb[j] = cc[j] = __builtin_nanf("");
    }
    auto out = [&](uint4 ux, uint4 ud, uint4 uy, long long i) {
        float d[8], xf[8];
        unpack8(ud, d);
        unpack8(ux, xf);
        if (MODE == BWD_RELU) {
            float yf[8];
            unpack8(uy, yf);
#pragma unroll
            for (int j = 0; j < 8; ++j) d[j] = yf[j] > 0.f ? d[j] : 0.f;
        }
        if (MODE == BWD_RELUX) {
#pragma unroll
            for (int j = 0; j < 8; ++j) d[j] = fmaf(xf[j], fsc[j], fsh[j]) > 0.f ? d[j] : 0.f;
        }
        if (DRES) a.dres_out[i] = pack8(d);
        float o[8];
#pragma unroll
        for (int j = 0; j < 8; ++j)
            o[j] = fmaf(ca[j], d[j], fmaf(cb[j], xf[j], cc[j]));
        a.yout[i] = pack8(o);
    };
    if (NR > 0) {
#pragma unroll
        for (int u = 0; u < NV; ++u) {
            const long long r = rbeg + r0 + (long long)u * rpp;
            if (r < rend) out(vx[u], vd[u], MODE == BWD_RELU ? vy[u < NY ? u : 0] : z, r * vpr + cv);
        }
    } else {
        long long r = rbeg + r0;
        const long long st = (long long)rpp * vpr;
        for (; r + (US - 1) * rpp < rend; r += US * rpp) {
            uint4 wx[US], wd[US], wy[US];
            unsigned wm[US];
#pragma unroll
            for (int u = 0; u < US; ++u) {
                const long long i = r * vpr + cv + u * st;
                wx[u] = X[i];
                wd[u] = DY[i];
                if (MODE == BWD_RELU && YM) wm[u] = a.ymask[i];
                else if (MODE == BWD_RELU) wy[u] = Y[i];
            }
#pragma unroll
            for (int u = 0; u < US; ++u) {
                pin(wx[u]);
                pin(wd[u]);
                if (MODE == BWD_RELU && YM) pin(wm[u]);
                else if (MODE == BWD_RELU) pin(wy[u]);
            }
#pragma unroll
            for (int u = 0; u < US; ++u)
                out(wx[u], wd[u], MODE == BWD_RELU ? (YM ? mask_vals(wm[u]) : wy[u]) : z, r * vpr + cv + u * st);
        }
        for (; r < rend; r += rpp) {
            const long long i = r * vpr + cv;
            out(X[i], DY[i], MODE == BWD_RELU ? ldy(i) : z, i);
        }
    }
}

struct ApplyArgs {
    long long nvec;      // M * C / 8
    int tpr_log;
    int relu;
    const void* x;       // E elements
    const void* res;     // fwd residual / bwd: y (relu mask)
    const void* dy;      // bwd
    void* out;           // fwd y / bwd dx
    void* out2;          // bwd dres
    const float* coef;   // [4][C]
    int C;
    const float* fcoef;  // bwd MASKX: the forward's sc[C], sh[C]
    long long gvec;      // view groups (gridDim.y): group g's x / res / dy / out / out2 gvec
    long long cgs;       // vectors and its coefficients cgs floats after group 0's
    long long fcgs;      // bwd MASKX: group g's fcoef fcgs floats after group 0's
    uint8_t* mask_out;   // fwd (relu + residual), optional: the ReLU mask bytes (as gvec)
};

__device__ __forceinline__ void load_coef(const float* p, int cg, float* c) {
    const float4 a = reinterpret_cast<const float4*>(p)[cg * 2];
    const float4 b = reinterpret_cast<const float4*>(p)[cg * 2 + 1];
    c[0] = a.x; c[1] = a.y; c[2] = a.z; c[3] = a.w; c[4] = b.x; c[5] = b.y; c[6] = b.z; c[7] = b.w;
}

template <bool RES, bool RELU, typename E>
__global__ __launch_bounds__(kT) void k_bn_apply(ApplyArgs a) {
    const long long stride = (long long)gridDim.x * kT;  // multiple of C/8
    long long v = (long long)blockIdx.x * kT + threadIdx.x;
    const int cg = (int)(v & ((1 << a.tpr_log) - 1));
    const long long go = blockIdx.y * a.gvec;  // view group blockIdx.y
    const float* coef = a.coef + blockIdx.y * a.cgs;
    float sc[8], sh[8];
    load_coef(coef, cg, sc);
    load_coef(coef + a.C, cg, sh);
    auto fin = [&](long long i, float* f, const float* r) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            float z = fmaf(f[j], sc[j], sh[j]);
            if (RES) z += r[j];
            f[j] = RELU ? relu_nan(z) : z;
        }
        V8<E>::st(a.out, i, f);
        if (RES && RELU && std::is_same<E, uint16_t>::value && a.mask_out) a.mask_out[i] = (uint8_t)mask_byte(pack8(f));
    };
    auto one = [&](long long i) {
        i += go;
        float f[8];
        V8<E>::ld(a.x, i, f);
        float r[8];
        if (RES) V8<E>::ld(a.res, i, r);
        fin(i, f, r);
    };
    if constexpr (std::is_same<E, uint16_t>::value) {
        // four vectors' 16-B loads issued before the first use (as k_bn_apply_bwd)
        typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
        constexpr int U = 4;
        const u32x4* XX = static_cast<const u32x4*>(a.x) + go;
        const u32x4* RR = static_cast<const u32x4*>(a.res) + go;
        for (; v + (U - 1) * stride < a.nvec; v += U * stride) {
            u32x4 rx[U], rr[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                rx[u] = XX[v + u * stride];
                if (RES) rr[u] = RR[v + u * stride];
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                asm volatile("" : "+v"(rx[u]));
                if (RES) asm volatile("" : "+v"(rr[u]));
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                float f[8], r[8];
                unpack8(make_uint4(rx[u].x, rx[u].y, rx[u].z, rx[u].w), f);
                if (RES) unpack8(make_uint4(rr[u].x, rr[u].y, rr[u].z, rr[u].w), r);
                fin(go + v + u * stride, f, r);
            }
        }
        for (; v < a.nvec; v += stride) one(v);
        return;
    }
    for (; v + stride < a.nvec; v += 2 * stride) {
        one(v);
        one(v + stride);
    }
    if (v < a.nvec) one(v);
}

template <bool RELU, bool DRES, bool MASKX, typename E>
__global__ __launch_bounds__(kT) void k_bn_apply_bwd(ApplyArgs a) {
    constexpr bool CENTER = std::is_same<E, float>::value;  // finalize<CENTER>: slot 3 = mean
    const long long stride = (long long)gridDim.x * kT;
    long long v = (long long)blockIdx.x * kT + threadIdx.x;
    const int cg = (int)(v & ((1 << a.tpr_log) - 1));
    const long long go = blockIdx.y * a.gvec;  // view group blockIdx.y
    const float* coef = a.coef + blockIdx.y * a.cgs;
    float ca[8], cb[8], cc[8], fs[8], fh[8], mu[8];
    load_coef(coef, cg, ca);
    load_coef(coef + a.C, cg, cb);
    load_coef(coef + 2 * a.C, cg, cc);
    if (CENTER) load_coef(coef + 3 * a.C, cg, mu);
    if (MASKX) {
        load_coef(a.fcoef + blockIdx.y * a.fcgs, cg, fs);
        load_coef(a.fcoef + blockIdx.y * a.fcgs + a.C, cg, fh);
    }
    constexpr bool YR = RELU && !MASKX;  // the mask read from y
    auto ld = [&](long long i, float* d, float* xf, float* yf) {
        V8<E>::ld(a.dy, go + i, d);
        V8<E>::ld(a.x, go + i, xf);
        if (YR) V8<E>::ld(a.res, go + i, yf);
    };
    auto out = [&](long long i, float* d, const float* xf, const float* yf) {
        if (RELU && MASKX) {
#pragma unroll
            for (int j = 0; j < 8; ++j) d[j] = fmaf(xf[j], fs[j], fh[j]) > 0.f ? d[j] : 0.f;
        } else if (RELU) {
#pragma unroll
            for (int j = 0; j < 8; ++j) d[j] = yf[j] > 0.f ? d[j] : 0.f;
        }
        if (DRES) V8<E>::st(a.out2, go + i, d);
        float o[8];
#pragma unroll
        for (int j = 0; j < 8; ++j)
            o[j] = CENTER ? fmaf(ca[j], d[j], fmaf(cb[j], xf[j] - mu[j], cc[j])) : fmaf(ca[j], d[j], fmaf(cb[j], xf[j], cc[j]));
        V8<E>::st(a.out, go + i, o);
    };
    // U vectors' loads issued before the first store (the pointers may alias as far as the
    // compiler knows: one vector at a time serialised load -> wait -> store, 32 B in flight)
    constexpr int U = 4;
    if constexpr (std::is_same<E, uint16_t>::value) {  // raw 16-B loads first, unpacked after
        typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
        const u32x4* DY = static_cast<const u32x4*>(a.dy) + go;
        const u32x4* XX = static_cast<const u32x4*>(a.x) + go;
        const u32x4* YY = static_cast<const u32x4*>(a.res) + go;
        auto u4 = [](u32x4 w) { return make_uint4(w.x, w.y, w.z, w.w); };
        for (; v + (U - 1) * stride < a.nvec; v += U * stride) {
            u32x4 rd[U], rx[U], ry[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                rd[u] = DY[v + u * stride];
                rx[u] = XX[v + u * stride];
                if (YR) ry[u] = YY[v + u * stride];
            }
            // every load issued before the first use (the compiler otherwise sinks each load to
            // its use: one vector's 32 B in flight per thread)
#pragma unroll
            for (int u = 0; u < U; ++u) {
                asm volatile("" : "+v"(rd[u]), "+v"(rx[u]));
                if (YR) asm volatile("" : "+v"(ry[u]));
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                float d[8], xf[8], yf[8];
                unpack8(u4(rd[u]), d);
                unpack8(u4(rx[u]), xf);
                if (YR) unpack8(u4(ry[u]), yf);
                out(v + u * stride, d, xf, yf);
            }
        }
    } else {
        for (; v + (U - 1) * stride < a.nvec; v += U * stride) {
            float d[U][8], xf[U][8], yf[U][YR ? 8 : 1];
#pragma unroll
            for (int u = 0; u < U; ++u) ld(v + u * stride, d[u], xf[u], yf[u]);
#pragma unroll
            for (int u = 0; u < U; ++u) out(v + u * stride, d[u], xf[u], yf[u]);
        }
    }
    for (; v < a.nvec; v += stride) {
        float d[8], xf[8], yf[YR ? 8 : 1];
        ld(v, d, xf, yf);
        out(v, d, xf, yf);
    }
}

__global__ void k_bn_infer_coef(int C, const float* gamma, const float* beta, const float* rm, const float* rv,
                                float eps, float* coef) {
    const int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= C) return;
    const double is = 1.0 / sqrt((double)rv[c] + (double)eps);
    const double sc = (double)gamma[c] * is;
    coef[c] = (float)sc;
    coef[C + c] = (float)((double)beta[c] - (double)rm[c] * sc);
}

inline int apply_grid(long long nvec, int C) {
    // ~4 vectors per thread, grid a multiple of nothing in particular: kT is a
    // multiple of C/8 so the channel group of a thread is fixed
    long long g = (nvec + kT * 4 - 1) / (kT * 4);
    if (g > 8192) g = 8192;
    if (g < 1) g = 1;
    (void)C;
    return (int)g;
}

constexpr int kGenOff = 32;  // generation words: header words [32, 32 + nslice) (nslice <= 32)

// Plan of the fused forward: rows per thread NR in {4, 8, 16} (the register-held
// strip) and a grid that stays co-resident even when `concurrency` such launches run
// at once on different streams (the view trunks): grid <= CUs * occupancy / concurrency,
// the occupancy MEASURED for the kernel instantiations that can be launched
// (hipOccupancyMaxActiveBlocksPerMultiprocessor, the minimum over their variants) and
// the concurrency set by the caller (gm_bn_set_concurrency: the number of trunk streams
// that run concurrently plus headroom; default 4).  A grid
// that could exceed the resident capacity would let spinning blocks wait on blocks that
// cannot be scheduled (the spin is bounded and then faults loudly, see wait_generation).
// Returns NR (pl rewritten), -1 for the streaming variant (x re-read by the apply phase;
// gm_bn_set_fused_mode(1) disables it) or 0: use the two-kernel path (gm_bn_set_fused_mode(0)).
int g_concurrency = [] {
    const int v = 4;
    return v >= 1 ? v : 4;  // 0 / garbage: the default (never a division by zero)
}();
int g_fused_env = [] {
    return 2;  // read once; 0 = two-kernel path, 1 = no streaming variant
}();

template <typename K>
int occ_min(std::initializer_list<K> ks) {
    int best = 1 << 30;
    for (K k : ks) {
        int n = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, reinterpret_cast<const void*>(k), kT, 0) != hipSuccess)
            n = 0;
        best = n < best ? n : best;
    }
    return best == (1 << 30) ? 0 : best;
}

struct Occ {
    int fwd[4];  // NR 4, 8, 16, streaming
    int bwd[3];  // NR 4, 8, streaming
};

const Occ& occupancy() {
    static const Occ o = [] {
        Occ r{};
#define GM_F(NR) occ_min({k_bn_fwd_fused<true, true, NR>, k_bn_fwd_fused<true, false, NR>, \
                          k_bn_fwd_fused<false, true, NR>, k_bn_fwd_fused<false, false, NR>})
#define GM_B(NR) occ_min({k_bn_bwd_fused<BWD_RELUX, false, NR>, k_bn_bwd_fused<BWD_RELU, true, NR>, \
                          k_bn_bwd_fused<BWD_RELU, false, NR>, k_bn_bwd_fused<BWD, false, NR>,       \
                          k_bn_bwd_fused<BWD_RELU, true, NR, true>, k_bn_bwd_fused<BWD_RELU, false, NR, true>})
        r.fwd[0] = GM_F(4); r.fwd[1] = GM_F(8); r.fwd[2] = GM_F(16); r.fwd[3] = GM_F(0);
        r.bwd[0] = GM_B(4); r.bwd[1] = GM_B(8); r.bwd[2] = GM_B(0);
#undef GM_F
#undef GM_B
        return r;
    }();
    return o;
}

int device_cus() {
    static const int cus = [] {
        int dev = 0, n = 0;
        if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) !=
                                                     hipSuccess)
            return 0;
        return n;
    }();
    return cus;
}

// the redundant-finalize hand-off (every block combines the partial rows): small maps only,
// where a block's extra partial-row reads are a few KB
static int g_bn_redundant_max = [] {
    return 16;  // measured: 8 / 16 help layer 4 (~1-1.3 us a launch), 32+ slow layer 3
}();
inline int redundant_ok(int nrc) { return nrc <= g_bn_redundant_max ? 1 : 0; }

inline int fused_plan(long long M, int C, Plan& pl, bool bwd = false, int G = 1) {
    if (g_fused_env == 0) return 0;
    // co-residency under the device residency plan (gm_set_residency): CUs held by
    // never-yielding kernels (RCCL) are not counted, and every process sharing the GPU
    // may run its own launches at once
    const Residency& rs = residency();
    const int cus = usable_cus(device_cus());
    // a grouped launch (G views in one grid) holds G plans' worth of workgroups at once
    const int conc = (g_concurrency > rs.streams ? g_concurrency : rs.streams) * rs.sharers * G;
    const Plan base = make_plan(M, C);
    const Occ& oc = occupancy();
    const int nrs[3] = {4, 8, 16};
    const int occ_reg[3] = {bwd ? oc.bwd[0] : oc.fwd[0], bwd ? oc.bwd[1] : oc.fwd[1], bwd ? 0 : oc.fwd[2]};
    for (int i = 0; i < 3; ++i) {
        if (occ_reg[i] <= 0) continue;
        const long long budget = (long long)cus * occ_reg[i] / conc;
        long long want = budget / base.nslice;
        if (want < 1) continue;
        long long rpb = (M + want - 1) / want;
        rpb = (rpb + base.rpp - 1) / base.rpp * base.rpp;
        if (rpb / base.rpp > nrs[i]) continue;
        const long long nrc = (M + rpb - 1) / rpb;
        if (nrc > base.nrc) continue;  // partials area sized by the base plan
        pl = base;
        pl.rpb = rpb;
        pl.nrc = (int)nrc;
        return nrs[i];
    }
    if (g_fused_env >= 2) {  // streaming variant: any map size
        const int occ_s = bwd ? oc.bwd[2] : oc.fwd[3];
        long long want = (long long)cus * occ_s / conc / base.nslice;
        if (want >= 1) {
            long long rpb = (M + want - 1) / want;
            rpb = (rpb + base.rpp - 1) / base.rpp * base.rpp;
            const long long nrc = (M + rpb - 1) / rpb;
            if (nrc <= base.nrc) {
                pl = base;
                pl.rpb = rpb;
                pl.nrc = (int)nrc;
                return -1;
            }
        }
    }
    return 0;
}

int check_common(long long M, int C, const void* scratch, size_t bytes, const char* fn) {
    if (M <= 0 || C < 8 || C > kMaxC || (C & (C - 1)) != 0) {
        set_error("%s: need M > 0 and C a power of two in [8, %d] (M=%lld C=%d)", fn, kMaxC, M, C);
        return GM_E_ARG;
    }
    if (!scratch || bytes < scratch_bytes(M, C)) {
        set_error("%s: scratch %zu bytes < required %zu", fn, bytes, scratch_bytes(M, C));
        return GM_E_SCRATCH;
    }
    return GM_OK;
}

}  // namespace
}  // namespace gm

using namespace gm;

extern "C" size_t gm_bn_scratch(long long M, int C) {
    if (M <= 0 || C < 8 || C > kMaxC) return 0;
    return scratch_bytes(M, C);
}

namespace {

// Grouped scratch layout (the gm_bn_*_grouped_bf16 calls; never mixed with ungrouped calls
// on one buffer): kMaxBnG fixed 256-byte headers (each group's tickets and generation
// words: they stay at the same place whatever the shape, so a ticket word is only ever
// a ticket word and stays zero between calls), then per group its coefficients and
// partials (no zero invariant) at a shape-dependent stride.
constexpr size_t kGrpHdr = kMaxBnG * kHdr;
inline size_t group_stride(long long M, int C) {
    const Plan p = make_plan(M, C);
    return (p.bytes - p.off_coef + 255) / 256 * 256;
}
inline size_t grouped_bytes(long long M, int C, int G) { return kGrpHdr + G * group_stride(M, C); }

// the scratch pointers of a call: ungrouped layout (header, coefficients, partials) or
// the grouped one above
void set_scratch(ReduceArgs& a, const Plan& pl, char* s, bool grouped) {
    a.counter = reinterpret_cast<unsigned*>(s);
    if (grouped) {
        a.coef = reinterpret_cast<float*>(s + kGrpHdr);
        a.part = reinterpret_cast<float*>(s + kGrpHdr + (pl.off_p1 - pl.off_coef));
        a.scr_stride = group_stride(a.M, a.C);
        a.hdr_words = kHdr / sizeof(unsigned);
    } else {
        a.coef = reinterpret_cast<float*>(s + pl.off_coef);
        a.part = reinterpret_cast<float*>(s + pl.off_p1);
        a.scr_stride = 0;
        a.hdr_words = 0;
    }
}

// the G descriptors of a grouped call must agree on everything but their pointers
int check_groups_fwd(const gm_bn_fwd* ps, int G, const char* fn) {
    GM_REQUIRE(ps && G >= 1 && G <= kMaxBnG, "%s: 1..%d groups (got %d)", fn, kMaxBnG, G);
    for (int g = 0; g < G; ++g) {
        const gm_bn_fwd& p = ps[g], &q = ps[0];
        GM_REQUIRE(p.x && p.gamma && p.beta && p.save_mean && p.save_invstd, "%s: null argument (group %d)", fn, g);
        GM_REQUIRE(!p.running_mean == !p.running_var, "%s: running_mean/var both or neither", fn);
        GM_REQUIRE(p.M == q.M && p.C == q.C && p.relu == q.relu && !p.residual == !q.residual &&
                       !p.running_mean == !q.running_mean && !p.num_batches_tracked == !q.num_batches_tracked &&
                       !p.coef_out == !q.coef_out && !p.y == !q.y && p.momentum == q.momentum && p.eps == q.eps,
                   "%s: group %d differs from group 0 in shape or options", fn, g);
    }
    return GM_OK;
}

int check_groups_bwd(const gm_bn_bwd* ps, int G, const char* fn) {
    GM_REQUIRE(ps && G >= 1 && G <= kMaxBnG, "%s: 1..%d groups (got %d)", fn, kMaxBnG, G);
    for (int g = 0; g < G; ++g) {
        const gm_bn_bwd& p = ps[g], &q = ps[0];
        GM_REQUIRE(p.dy && p.x && p.gamma && p.save_mean && p.save_invstd && p.dx && p.dgamma && p.dbeta,
                   "%s: null argument (group %d)", fn, g);
        GM_REQUIRE(!p.relu || p.y || (p.fwd_coef && !p.dres),
                   "%s: relu needs the forward output y (or fwd_coef, without a residual)", fn);
        GM_REQUIRE(p.M == q.M && p.C == q.C && p.relu == q.relu && !p.y == !q.y && !p.dres == !q.dres &&
                       !p.fwd_coef == !q.fwd_coef && p.accumulate == q.accumulate,
                   "%s: group %d differs from group 0 in shape or options", fn, g);
    }
    return GM_OK;
}

int check_scratch(long long M, int C, int G, bool grouped, const void* scratch, size_t bytes, const char* fn) {
    int rc = check_common(M, C, scratch, bytes, fn);
    if (rc) return rc;
    const size_t need = grouped ? grouped_bytes(M, C, G) : scratch_bytes(M, C);
    if (bytes < need) {
        set_error("%s: scratch %zu bytes < required %zu for %d groups", fn, bytes, need, G);
        return GM_E_SCRATCH;
    }
    return GM_OK;
}

// shared fields from group 0, per-group pointers into grp[], scratch split per group
void fill_fwd(ReduceArgs& a, const gm_bn_fwd* ps, int G, bool grouped, const Plan& pl, char* s) {
    const gm_bn_fwd* p = ps;
    a.M = p->M; a.C = p->C; a.tpr_log = pl.tpr_log; a.rpb = pl.rpb;
    a.SW = pl.SW; a.nrc = pl.nrc;
    a.momentum = p->momentum; a.eps = p->eps;
    set_scratch(a, pl, s, grouped);
    for (int g = 0; g < G; ++g) {
        BnGroup& q = a.grp[g];
        q.x = ps[g].x;
        q.gamma = ps[g].gamma; q.beta = ps[g].beta;
        q.rmean = ps[g].running_mean; q.rvar = ps[g].running_var;
        q.save_mean = ps[g].save_mean; q.save_invstd = ps[g].save_invstd;
        q.nbt = ps[g].num_batches_tracked;
        q.coef_out = ps[g].coef_out;
        q.res = static_cast<const uint4*>(ps[g].residual);
        q.yout = static_cast<uint4*>(ps[g].y);
        q.mask_out = static_cast<uint8_t*>(ps[g].relu_mask);
    }
    BnGroup& q = a.grp[0];  // the single-group fields (host bookkeeping only: kernels read grp[])
    a.x = q.x; a.gamma = q.gamma; a.beta = q.beta; a.rmean = q.rmean; a.rvar = q.rvar;
    a.save_mean = q.save_mean; a.save_invstd = q.save_invstd; a.nbt = q.nbt; a.coef_out = q.coef_out;
}

template <typename E>
int bn_fwd_train(const gm_bn_fwd* ps, int G, bool grouped, void* scratch, size_t bytes, void* stream,
                 const char* fn) {
    int rc = check_groups_fwd(ps, G, fn);
    if (rc) return rc;
    const gm_bn_fwd* p = ps;
    GM_REQUIRE(p->y, "%s: null argument (y)", fn);
    if ((rc = check_scratch(p->M, p->C, G, grouped, scratch, bytes, fn))) return rc;
    const Plan pl = make_plan(p->M, p->C);
    char* s = static_cast<char*>(scratch);
    ReduceArgs a{};
    fill_fwd(a, ps, G, grouped, pl, s);
    hipStream_t st = as_stream(stream);
    Plan fp;
    const int nr = std::is_same<E, uint16_t>::value ? fused_plan(p->M, p->C, fp, false, G) : 0;
    if (nr) {
        a.rpb = fp.rpb;
        a.nrc = fp.nrc;
        a.gen = reinterpret_cast<unsigned*>(s) + kGenOff;
        a.spin_limit = spin_limit();
        a.redundant = redundant_ok(a.nrc);
        const dim3 g(fp.nrc, fp.nslice, G);
        const bool res = p->residual != nullptr, relu = p->relu != 0;
#define GM_BN_FUSED_LAUNCH(NR)                                                                        \
    if (res && relu) hipLaunchKernelGGL((k_bn_fwd_fused<true, true, NR>), g, dim3(kT), 0, st, a);     \
    else if (res) hipLaunchKernelGGL((k_bn_fwd_fused<true, false, NR>), g, dim3(kT), 0, st, a);       \
    else if (relu) hipLaunchKernelGGL((k_bn_fwd_fused<false, true, NR>), g, dim3(kT), 0, st, a);      \
    else hipLaunchKernelGGL((k_bn_fwd_fused<false, false, NR>), g, dim3(kT), 0, st, a);
        if (nr < 0) { GM_BN_FUSED_LAUNCH(0) }
        else if (nr == 4) { GM_BN_FUSED_LAUNCH(4) }
        else if (nr == 8) { GM_BN_FUSED_LAUNCH(8) }
        else { GM_BN_FUSED_LAUNCH(16) }
#undef GM_BN_FUSED_LAUNCH
        return check_launch("k_bn_fwd_fused");
    }
    const dim3 rg(pl.nrc, pl.nslice, G);
    if (std::is_same<E, float>::value) hipLaunchKernelGGL((k_bn_reduce_f64<FWD>), rg, dim3(kT), 0, st, a);
    else hipLaunchKernelGGL((k_bn_reduce<FWD, E>), rg, dim3(kT), 0, st, a);
    if ((rc = check_launch("k_bn_reduce<fwd>"))) return rc;
    for (int gi = 0; gi < G; ++gi) {  // the apply: one launch per group
        ApplyArgs b{};
        b.nvec = p->M * (p->C / 8); b.tpr_log = ilog2(p->C / 8); b.C = p->C; b.relu = p->relu;
        b.x = ps[gi].x; b.res = ps[gi].residual; b.out = ps[gi].y;
        b.mask_out = static_cast<uint8_t*>(ps[gi].relu_mask);
        b.coef = reinterpret_cast<float*>(reinterpret_cast<char*>(a.coef) + gi * a.scr_stride);
        const int g = apply_grid(b.nvec, p->C);
        if (p->residual) {
            if (p->relu) hipLaunchKernelGGL((k_bn_apply<true, true, E>), dim3(g), dim3(kT), 0, st, b);
            else hipLaunchKernelGGL((k_bn_apply<true, false, E>), dim3(g), dim3(kT), 0, st, b);
        } else {
            if (p->relu) hipLaunchKernelGGL((k_bn_apply<false, true, E>), dim3(g), dim3(kT), 0, st, b);
            else hipLaunchKernelGGL((k_bn_apply<false, false, E>), dim3(g), dim3(kT), 0, st, b);
        }
        if ((rc = check_launch("k_bn_apply"))) return rc;
    }
    return GM_OK;
}

template <typename E>
int bn_fwd_infer(const gm_bn_fwd* p, void* scratch, size_t bytes, void* stream, const char* fn) {
    GM_REQUIRE(p && p->x && p->y && p->gamma && p->beta && p->running_mean && p->running_var, "%s: null argument",
               fn);
    int rc = check_common(p->M, p->C, scratch, bytes, fn);
    if (rc) return rc;
    char* s = static_cast<char*>(scratch);
    float* coef = reinterpret_cast<float*>(s + make_plan(p->M, p->C).off_coef);
    hipStream_t st = as_stream(stream);
    hipLaunchKernelGGL(k_bn_infer_coef, dim3((p->C + 255) / 256), dim3(256), 0, st, p->C, p->gamma, p->beta,
                       p->running_mean, p->running_var, p->eps, coef);
    if ((rc = check_launch("k_bn_infer_coef"))) return rc;
    ApplyArgs b{};
    b.nvec = p->M * (p->C / 8); b.tpr_log = ilog2(p->C / 8); b.C = p->C; b.relu = p->relu;
    b.x = p->x; b.res = p->residual; b.out = p->y; b.coef = coef;
    const int g = apply_grid(b.nvec, p->C);
    if (p->residual) {
        if (p->relu) hipLaunchKernelGGL((k_bn_apply<true, true, E>), dim3(g), dim3(kT), 0, st, b);
        else hipLaunchKernelGGL((k_bn_apply<true, false, E>), dim3(g), dim3(kT), 0, st, b);
    } else {
        if (p->relu) hipLaunchKernelGGL((k_bn_apply<false, true, E>), dim3(g), dim3(kT), 0, st, b);
        else hipLaunchKernelGGL((k_bn_apply<false, false, E>), dim3(g), dim3(kT), 0, st, b);
    }
    return check_launch("k_bn_apply");
}

template <typename E>
int bn_bwd(const gm_bn_bwd* ps, int G, bool grouped, void* scratch, size_t bytes, void* stream, const char* fn) {
    int rc = check_groups_bwd(ps, G, fn);
    if (rc) return rc;
    const gm_bn_bwd* p = ps;
    const bool maskx = p->relu && !p->y;
    if ((rc = check_scratch(p->M, p->C, G, grouped, scratch, bytes, fn))) return rc;
    const Plan pl = make_plan(p->M, p->C);
    char* s = static_cast<char*>(scratch);
    ReduceArgs a{};
    a.M = p->M; a.C = p->C; a.tpr_log = pl.tpr_log; a.rpb = pl.rpb; a.relu = p->relu;
    a.SW = pl.SW; a.nrc = pl.nrc;
    a.accumulate = p->accumulate;
    set_scratch(a, pl, s, grouped);
    for (int g = 0; g < G; ++g) {
        BnGroup& q = a.grp[g];
        q.x = ps[g].x; q.dy = ps[g].dy; q.y = ps[g].y;
        q.gamma = ps[g].gamma;
        q.save_mean = const_cast<float*>(ps[g].save_mean);
        q.save_invstd = const_cast<float*>(ps[g].save_invstd);
        q.dgamma = ps[g].dgamma; q.dbeta = ps[g].dbeta;
        q.fcoef = ps[g].fwd_coef;
        q.yout = static_cast<uint4*>(ps[g].dx);
        q.dres_out = static_cast<uint4*>(ps[g].dres);
        q.ymask = static_cast<const uint8_t*>(ps[g].relu_mask);
    }
    hipStream_t st = as_stream(stream);
    Plan fp;
    const int nr = (std::is_same<E, uint16_t>::value && (!p->dres || p->relu)) ? fused_plan(p->M, p->C, fp, true, G)
                                                                               : 0;
    if (nr) {
        a.rpb = fp.rpb;
        a.nrc = fp.nrc;
        a.gen = reinterpret_cast<unsigned*>(s) + kGenOff;
        a.spin_limit = spin_limit();
        a.redundant = redundant_ok(a.nrc);
        const dim3 g(fp.nrc, fp.nslice, G);
        const bool ym = p->relu && p->relu_mask && !maskx;  // the forward's mask bytes in place of y
#define GM_BN_BWD_FUSED_LAUNCH(NR)                                                                                  \
    if (maskx) hipLaunchKernelGGL((k_bn_bwd_fused<BWD_RELUX, false, NR>), g, dim3(kT), 0, st, a);                   \
    else if (ym && p->dres) hipLaunchKernelGGL((k_bn_bwd_fused<BWD_RELU, true, NR, true>), g, dim3(kT), 0, st, a);  \
    else if (ym) hipLaunchKernelGGL((k_bn_bwd_fused<BWD_RELU, false, NR, true>), g, dim3(kT), 0, st, a);            \
    else if (p->relu && p->dres) hipLaunchKernelGGL((k_bn_bwd_fused<BWD_RELU, true, NR>), g, dim3(kT), 0, st, a);   \
    else if (p->relu) hipLaunchKernelGGL((k_bn_bwd_fused<BWD_RELU, false, NR>), g, dim3(kT), 0, st, a);             \
    else hipLaunchKernelGGL((k_bn_bwd_fused<BWD, false, NR>), g, dim3(kT), 0, st, a);
        if (nr < 0) { GM_BN_BWD_FUSED_LAUNCH(0) }
        else if (nr == 4) { GM_BN_BWD_FUSED_LAUNCH(4) }
        else { GM_BN_BWD_FUSED_LAUNCH(8) }
#undef GM_BN_BWD_FUSED_LAUNCH
        return check_launch("k_bn_bwd_fused");
    }
    const dim3 rg(pl.nrc, pl.nslice, G);
    if (std::is_same<E, float>::value) {  // reference precision: fp64 accumulation
        if (maskx) hipLaunchKernelGGL((k_bn_reduce_f64<BWD_RELUX>), rg, dim3(kT), 0, st, a);
        else if (p->relu) hipLaunchKernelGGL((k_bn_reduce_f64<BWD_RELU>), rg, dim3(kT), 0, st, a);
        else hipLaunchKernelGGL((k_bn_reduce_f64<BWD>), rg, dim3(kT), 0, st, a);
    } else if (maskx) hipLaunchKernelGGL((k_bn_reduce<BWD_RELUX, E>), rg, dim3(kT), 0, st, a);
    else if (p->relu) hipLaunchKernelGGL((k_bn_reduce<BWD_RELU, E>), rg, dim3(kT), 0, st, a);
    else hipLaunchKernelGGL((k_bn_reduce<BWD, E>), rg, dim3(kT), 0, st, a);
    if ((rc = check_launch("k_bn_reduce<bwd>"))) return rc;
    for (int gi = 0; gi < G; ++gi) {  // the apply: one launch per group
        const gm_bn_bwd* q = ps + gi;
        ApplyArgs b{};
        b.nvec = p->M * (p->C / 8); b.tpr_log = ilog2(p->C / 8); b.C = p->C; b.relu = p->relu;
        b.x = q->x; b.res = q->y; b.dy = q->dy; b.out = q->dx;
        b.out2 = q->dres;
        b.coef = reinterpret_cast<float*>(reinterpret_cast<char*>(a.coef) + gi * a.scr_stride);
        b.fcoef = q->fwd_coef;
        const int g = apply_grid(b.nvec, p->C);
        if (maskx) {
            hipLaunchKernelGGL((k_bn_apply_bwd<true, false, true, E>), dim3(g), dim3(kT), 0, st, b);
        } else if (p->relu) {
            if (p->dres) hipLaunchKernelGGL((k_bn_apply_bwd<true, true, false, E>), dim3(g), dim3(kT), 0, st, b);
            else hipLaunchKernelGGL((k_bn_apply_bwd<true, false, false, E>), dim3(g), dim3(kT), 0, st, b);
        } else {
            if (p->dres) hipLaunchKernelGGL((k_bn_apply_bwd<false, true, false, E>), dim3(g), dim3(kT), 0, st, b);
            else hipLaunchKernelGGL((k_bn_apply_bwd<false, false, false, E>), dim3(g), dim3(kT), 0, st, b);
        }
        if ((rc = check_launch("k_bn_apply_bwd"))) return rc;
    }
    return GM_OK;
}

int bn_fwd_stats(const gm_bn_fwd* ps, int G, bool grouped, void* scratch, size_t bytes, void* stream,
                 const char* fn) {
    int rc = check_groups_fwd(ps, G, fn);
    if (rc) return rc;
    const gm_bn_fwd* p = ps;
    GM_REQUIRE(p->coef_out, "%s: coef_out required", fn);
    if ((rc = check_scratch(p->M, p->C, G, grouped, scratch, bytes, fn))) return rc;
    const Plan pl = make_plan(p->M, p->C);
    ReduceArgs a{};
    fill_fwd(a, ps, G, grouped, pl, static_cast<char*>(scratch));
    hipLaunchKernelGGL((k_bn_reduce<FWD, uint16_t>), dim3(pl.nrc, pl.nslice, G), dim3(kT), 0, as_stream(stream), a);
    return check_launch("k_bn_reduce<fwd>");
}

}  // namespace

namespace gm {
unsigned bn_faults_read(bool clear) {
    unsigned v = 0;
    if (hipMemcpyFromSymbol(&v, HIP_SYMBOL(g_bn_fault), sizeof(v), 0, hipMemcpyDeviceToHost) != hipSuccess) return ~0u;
    if (clear && v) {
        const unsigned z = 0;
        (void)hipMemcpyToSymbol(HIP_SYMBOL(g_bn_fault), &z, sizeof(z), 0, hipMemcpyHostToDevice);
    }
    return v;
}
}  // namespace gm

extern "C" int gm_bn_set_concurrency(int n) {
    GM_REQUIRE(n >= 1 && n <= 1024, "gm_bn_set_concurrency: n must be in [1, 1024] (got %d)", n);
    gm::g_concurrency = n;
    return GM_OK;
}

extern "C" int gm_bn_set_fused_mode(int mode) {
    GM_REQUIRE(mode >= 0 && mode <= 2, "gm_bn_set_fused_mode: mode must be 0, 1 or 2 (got %d)", mode);
    gm::g_fused_env = mode;
    return GM_OK;
}

// Statistics half of the training forward only (one reduce launch): save_mean/invstd,
// running statistics, num_batches_tracked and the affine coefficients in coef_out
// (required); no y.  The apply is fused into the consumer (gm_bn_relu_maxpool2d_fwd_bf16).
extern "C" int gm_bn_fwd_stats_bf16(const gm_bn_fwd* p, void* scratch, size_t bytes, void* stream) {
    return bn_fwd_stats(p, 1, false, scratch, bytes, stream, "gm_bn_fwd_stats_bf16");
}

extern "C" size_t gm_bn_scratch_grouped(long long M, int C, int G) {
    if (M <= 0 || C < 8 || C > kMaxC || G < 1 || G > kMaxBnG) return 0;
    return grouped_bytes(M, C, G);
}

extern "C" int gm_bn_fwd_train_grouped_bf16(const gm_bn_fwd* ps, int G, void* scratch, size_t bytes, void* stream) {
    return bn_fwd_train<uint16_t>(ps, G, true, scratch, bytes, stream, "gm_bn_fwd_train_grouped_bf16");
}
extern "C" int gm_bn_bwd_grouped_bf16(const gm_bn_bwd* ps, int G, void* scratch, size_t bytes, void* stream) {
    return bn_bwd<uint16_t>(ps, G, true, scratch, bytes, stream, "gm_bn_bwd_grouped_bf16");
}
extern "C" int gm_bn_fwd_stats_grouped_bf16(const gm_bn_fwd* ps, int G, void* scratch, size_t bytes, void* stream) {
    return bn_fwd_stats(ps, G, true, scratch, bytes, stream, "gm_bn_fwd_stats_grouped_bf16");
}

extern "C" int gm_bn_fwd_train_bf16(const gm_bn_fwd* p, void* scratch, size_t bytes, void* stream) {
    return bn_fwd_train<uint16_t>(p, 1, false, scratch, bytes, stream, "gm_bn_fwd_train_bf16");
}
extern "C" int gm_bn_fwd_infer_bf16(const gm_bn_fwd* p, void* scratch, size_t bytes, void* stream) {
    return bn_fwd_infer<uint16_t>(p, scratch, bytes, stream, "gm_bn_fwd_infer_bf16");
}
extern "C" int gm_bn_bwd_bf16(const gm_bn_bwd* p, void* scratch, size_t bytes, void* stream) {
    return bn_bwd<uint16_t>(p, 1, false, scratch, bytes, stream, "gm_bn_bwd_bf16");
}
extern "C" int gm_bn_fwd_train_f32(const gm_bn_fwd* p, void* scratch, size_t bytes, void* stream) {
    return bn_fwd_train<float>(p, 1, false, scratch, bytes, stream, "gm_bn_fwd_train_f32");
}
extern "C" int gm_bn_fwd_infer_f32(const gm_bn_fwd* p, void* scratch, size_t bytes, void* stream) {
    return bn_fwd_infer<float>(p, scratch, bytes, stream, "gm_bn_fwd_infer_f32");
}
extern "C" int gm_bn_bwd_f32(const gm_bn_bwd* p, void* scratch, size_t bytes, void* stream) {
    return bn_bwd<float>(p, 1, false, scratch, bytes, stream, "gm_bn_bwd_f32");
}

// The stem's BatchNorm + ReLU + max-pool backward in two launches (k_stem_pool_bn_bwd):
// d describes one view group's pool (N images, k 3, stride 2, pad 1, C 64); ps[g] the BN
// backward of group g with relu, fwd_coef (the mask from x) and no y / dres; ps[g].dy unused.
// apply = false: pass 1 only (statistics, dgamma / dbeta, the coefficients ca, cb, cc); the
// weight gradient of the stem then forms dx itself (gm_conv2d_wgrad_stem_bn_grouped_bf16).
static int stem_pool_bwd(const gm_pool_desc* d, int G, const void* dy_pool, const void* idx, const void* xsel,
                         const gm_bn_bwd* ps, void* scratch, size_t bytes, bool apply, const float** bcoef,
                         long long* bcoef_gs, void* stream, const char* fn) {
    GM_REQUIRE(d && dy_pool && idx && ps && G >= 1 && G <= kMaxBnG, "%s: bad arguments", fn);
    GM_REQUIRE(d->k == 3 && d->stride == 2 && d->pad == 1 && d->C == 64 && d->N >= 1 && d->H >= 2 && d->W >= 2,
               "%s: the stem's pool only (k 3, stride 2, pad 1, C 64)", fn);
    const int P = (d->H + 2 - 3) / 2 + 1, Q = (d->W + 2 - 3) / 2 + 1;
    GM_REQUIRE((d->H + 1) / 2 == P && (d->W + 1) / 2 == Q, "%s: pool geometry", fn);
    for (int g = 0; g < G; ++g) {
        const gm_bn_bwd& p = ps[g];
        GM_REQUIRE(p.M == (long long)d->N * d->H * d->W && p.C == d->C && p.relu && p.fwd_coef && !p.y && !p.dres &&
                       p.x && (p.dx || !apply) && p.gamma && p.save_mean && p.save_invstd && p.dgamma && p.dbeta &&
                       p.accumulate == ps[0].accumulate,
                   "%s: group %d: BN backward must be M = N*H*W, C, relu with fwd_coef, no y / dres", fn, g);
    }
    int rc;
    if ((rc = check_scratch(ps[0].M, ps[0].C, G, true, scratch, bytes, fn))) return rc;
    const Plan pl = make_plan(ps[0].M, ps[0].C);
    ReduceArgs a{};
    a.M = ps[0].M; a.C = ps[0].C; a.relu = 1; a.SW = ps[0].C; a.tpr_log = 3;
    a.accumulate = ps[0].accumulate;
    set_scratch(a, pl, static_cast<char*>(scratch), true);
    for (int g = 0; g < G; ++g) {
        BnGroup& q = a.grp[g];
        q.x = ps[g].x;
        q.gamma = ps[g].gamma;
        q.save_mean = const_cast<float*>(ps[g].save_mean);
        q.save_invstd = const_cast<float*>(ps[g].save_invstd);
        q.dgamma = ps[g].dgamma; q.dbeta = ps[g].dbeta;
        q.fcoef = ps[g].fwd_coef;
        q.yout = static_cast<uint4*>(ps[g].dx);
    }
    StemPoolGeo pg;
    pg.Ng = d->N; pg.H = d->H; pg.W = d->W; pg.P = P; pg.Q = Q;
    pg.items = (long long)d->N * P * Q * (d->C / 8);
    GM_REQUIRE((long long)d->N * d->H * d->W * (d->C / 8) < (1ll << 31), "%s: a group's map exceeds 2^31 vectors", fn);
    // pass-1 partial rows: at most the plan's (the grouped scratch holds pl.nrc rows per group)
    int nrc = pl.nrc < kMaxRC ? pl.nrc : kMaxRC;
    pg.ipb = (pg.items + nrc - 1) / nrc;
    pg.ipb = (pg.ipb + kT - 1) / kT * kT;
    nrc = (int)((pg.items + pg.ipb - 1) / pg.ipb);
    a.nrc = nrc;
    pg.idx = static_cast<const uint2*>(idx);
    pg.gp = static_cast<const uint4*>(dy_pool);
    pg.xs = static_cast<const uint4*>(xsel);
    hipStream_t st = as_stream(stream);
    hipLaunchKernelGGL((k_stem_pool_bn_bwd<false>), dim3(nrc, 1, G), dim3(kT), 0, st, a, pg);
    if ((rc = check_launch("k_stem_pool_bn_bwd<reduce>"))) return rc;
    if (!apply) {  // group g's ca, cb, cc: a.coef + g * scr_stride bytes (group_args)
        *bcoef = a.coef;
        *bcoef_gs = (long long)(a.scr_stride / sizeof(float));
        return GM_OK;
    }
    long long grid = (pg.items + kT - 1) / kT;
    if (grid > 4096) grid = 4096;
    hipLaunchKernelGGL((k_stem_pool_bn_bwd<true>), dim3((unsigned)grid, 1, G), dim3(kT), 0, st, a, pg);
    return check_launch("k_stem_pool_bn_bwd<apply>");
}

extern "C" int gm_bn_relu_maxpool2d_bwd_grouped_bf16(const gm_pool_desc* d, int G, const void* dy_pool,
                                                     const void* idx, const void* xsel, const gm_bn_bwd* ps,
                                                     void* scratch, size_t bytes, void* stream) {
    return stem_pool_bwd(d, G, dy_pool, idx, xsel, ps, scratch, bytes, true, nullptr, nullptr, stream,
                         "gm_bn_relu_maxpool2d_bwd_grouped_bf16");
}

extern "C" int gm_bn_relu_maxpool2d_bwd_stats_grouped_bf16(const gm_pool_desc* d, int G, const void* dy_pool,
                                                           const void* idx, const void* xsel, const gm_bn_bwd* ps,
                                                           void* scratch, size_t bytes, const float** bcoef,
                                                           long long* bcoef_gs, void* stream) {
    const char* fn = "gm_bn_relu_maxpool2d_bwd_stats_grouped_bf16";
    GM_REQUIRE(bcoef && bcoef_gs, "%s: null coefficient outputs", fn);
    return stem_pool_bwd(d, G, dy_pool, idx, xsel, ps, scratch, bytes, false, bcoef, bcoef_gs, stream, fn);
}

// BatchNorm forward statistics from producer partial rows (gm_conv2d_fwd_grouped_bn_stats_bf16,
// the stem's gm_conv2d_fwd_grouped_stats_bf16): stats = [G] x ([C / 64 slices][rows][64 x (sum,
// sum of squares)] then 2C floats of coefficient scratch); ps[g] as for
// gm_bn_fwd_stats_grouped_bf16 (C a multiple of 64).  One block per (slice, group).
extern "C" int gm_bn_fwd_stats_finalize_grouped(const gm_bn_fwd* ps, int G, float* stats, int rows, void* stream) {
    const char* fn = "gm_bn_fwd_stats_finalize_grouped";
    int rc = check_groups_fwd(ps, G, fn);
    if (rc) return rc;
    const int C = ps[0].C;
    GM_REQUIRE(stats && rows >= 1 && C >= 64 && C % 64 == 0 && ps[0].M >= 1, "%s: C a multiple of 64, rows >= 1",
               fn);
    ReduceArgs a{};
    a.M = ps[0].M; a.C = C; a.SW = 64; a.tpr_log = 3; a.nrc = rows;
    a.momentum = ps[0].momentum; a.eps = ps[0].eps;
    a.part = stats;
    a.coef = stats + (size_t)rows * 2 * C;
    a.scr_stride = (unsigned long long)(rows + 1) * 2 * C * sizeof(float);
    a.hdr_words = 0;
    for (int g = 0; g < G; ++g) {
        BnGroup& q = a.grp[g];
        q.x = ps[g].x;
        q.gamma = ps[g].gamma; q.beta = ps[g].beta;
        q.rmean = ps[g].running_mean; q.rvar = ps[g].running_var;
        q.save_mean = ps[g].save_mean; q.save_invstd = ps[g].save_invstd;
        q.nbt = ps[g].num_batches_tracked;
        q.coef_out = ps[g].coef_out;
    }
    hipLaunchKernelGGL(k_bn_stats_finalize, dim3(1, C / 64, G), dim3(kFinT), 0, as_stream(stream), a);
    return check_launch("k_bn_stats_finalize");
}

// The apply after gm_bn_fwd_stats_finalize_grouped: y = relu?(x*sc + sh (+ residual)), the
// coefficients read from the statistics buffer; one launch for the G groups when their
// tensors are evenly strided (the view-batched trunk), else one per group.
extern "C" int gm_bn_fwd_apply_grouped_bf16(const gm_bn_fwd* ps, int G, const float* stats, int rows, void* stream) {
    const char* fn = "gm_bn_fwd_apply_grouped_bf16";
    int rc = check_groups_fwd(ps, G, fn);
    if (rc) return rc;
    const gm_bn_fwd* p = ps;
    const int C = p->C;
    GM_REQUIRE(stats && rows >= 1 && C >= 64 && C % 64 == 0 && p->y, "%s: C a multiple of 64, rows >= 1, y", fn);
    const long long gs = p->M * C;  // elements
    bool strided = true;
    for (int g = 1; g < G; ++g) {
        const uint16_t* x0 = static_cast<const uint16_t*>(p->x);
        strided = strided && ps[g].x == x0 + g * gs &&
                  ps[g].y == static_cast<uint16_t*>(p->y) + g * gs &&
                  (!p->residual || ps[g].residual == static_cast<const uint16_t*>(p->residual) + g * gs) &&
                  (!p->relu_mask || ps[g].relu_mask == static_cast<uint8_t*>(p->relu_mask) + g * gs / 8);
    }
    const long long cgs = (long long)(rows + 1) * 2 * C;
    hipStream_t st = as_stream(stream);
    const int ng = strided ? 1 : G;
    for (int gi = 0; gi < ng; ++gi) {
        ApplyArgs b{};
        b.nvec = p->M * (C / 8); b.tpr_log = ilog2(C / 8); b.C = C; b.relu = p->relu;
        b.x = ps[gi].x; b.res = ps[gi].residual; b.out = ps[gi].y;
        b.mask_out = static_cast<uint8_t*>(ps[gi].relu_mask);
        b.coef = stats + gi * cgs + (size_t)rows * 2 * C;
        b.gvec = strided ? gs / 8 : 0;
        b.cgs = strided ? cgs : 0;
        const dim3 g(apply_grid(b.nvec, C), strided ? G : 1);
        if (p->residual) {
            if (p->relu) hipLaunchKernelGGL((k_bn_apply<true, true, uint16_t>), g, dim3(kT), 0, st, b);
            else hipLaunchKernelGGL((k_bn_apply<true, false, uint16_t>), g, dim3(kT), 0, st, b);
        } else {
            if (p->relu) hipLaunchKernelGGL((k_bn_apply<false, true, uint16_t>), g, dim3(kT), 0, st, b);
            else hipLaunchKernelGGL((k_bn_apply<false, false, uint16_t>), g, dim3(kT), 0, st, b);
        }
        if ((rc = check_launch("k_bn_apply"))) return rc;
    }
    return GM_OK;
}

// The BatchNorm backward from producer statistics (include/greedymml.h): stats as written by
// gm_conv2d_dgrad_grouped_bn_stats_bf16 - [G] x ([C / 64][rows][64 x (sum dz, sum dz (x - mean))]
// + 2C floats), then G x 4C floats of backward coefficients.  ps[g]: the backward descriptor
// (relu with fwd_coef - the mask recomputed from x - or no relu; no dres), C a multiple of 64.
extern "C" size_t gm_bn_bwd_stats_coef_offset(int C, int G, int rows) {
    return (size_t)G * 2 * C * (size_t)(rows + 1);
}

static int check_bwd_from_stats(const gm_bn_bwd* ps, int G, const float* stats, int rows, const char* fn) {
    int rc = check_groups_bwd(ps, G, fn);
    if (rc) return rc;
    const int C = ps[0].C;
    GM_REQUIRE(stats && rows >= 1 && C >= 64 && C % 64 == 0 && ps[0].M >= 1, "%s: C a multiple of 64, rows >= 1",
               fn);
    GM_REQUIRE(!ps[0].dres && (!ps[0].relu || ps[0].fwd_coef),
               "%s: relu needs fwd_coef (mask from x); no residual gradient", fn);
    return GM_OK;
}

extern "C" int gm_bn_bwd_stats_finalize_grouped(const gm_bn_bwd* ps, int G, float* stats, int rows, void* stream) {
    const char* fn = "gm_bn_bwd_stats_finalize_grouped";
    int rc = check_bwd_from_stats(ps, G, stats, rows, fn);
    if (rc) return rc;
    const int C = ps[0].C;
    ReduceArgs a{};
    a.M = ps[0].M; a.C = C; a.SW = 64; a.tpr_log = 3; a.nrc = rows;
    a.accumulate = ps[0].accumulate;
    a.part = stats;
    a.coef = stats;
    a.scr_stride = (unsigned long long)(rows + 1) * 2 * C * sizeof(float);
    a.hdr_words = 0;
    for (int g = 0; g < G; ++g) {
        BnGroup& q = a.grp[g];
        q.x = ps[g].x; q.dy = ps[g].dy;
        q.gamma = ps[g].gamma;
        q.save_mean = const_cast<float*>(ps[g].save_mean);
        q.save_invstd = const_cast<float*>(ps[g].save_invstd);
        q.dgamma = ps[g].dgamma; q.dbeta = ps[g].dbeta;
    }
    float* coef0 = stats + gm_bn_bwd_stats_coef_offset(C, G, rows);
    hipLaunchKernelGGL(k_bn_bwd_stats_finalize, dim3(1, C / 64, G), dim3(kFinT), 0, as_stream(stream), a, coef0,
                       (long long)4 * C);
    return check_launch("k_bn_bwd_stats_finalize");
}

extern "C" int gm_bn_bwd_apply_grouped_bf16(const gm_bn_bwd* ps, int G, const float* stats, int rows, void* stream) {
    const char* fn = "gm_bn_bwd_apply_grouped_bf16";
    int rc = check_bwd_from_stats(ps, G, stats, rows, fn);
    if (rc) return rc;
    const gm_bn_bwd* p = ps;
    const int C = p->C;
    GM_REQUIRE(p->dx && p->dy && p->x, "%s: null argument (dx, dy, x)", fn);
    const long long gs = p->M * C;
    bool strided = true;
    for (int g = 1; g < G; ++g)
        strided = strided && ps[g].x == static_cast<const uint16_t*>(p->x) + g * gs &&
                  ps[g].dy == static_cast<const uint16_t*>(p->dy) + g * gs &&
                  ps[g].dx == static_cast<uint16_t*>(p->dx) + g * gs &&
                  (!p->relu || ps[g].fwd_coef == p->fwd_coef + (size_t)g * 2 * C);
    const float* coef0 = stats + gm_bn_bwd_stats_coef_offset(C, G, rows);
    hipStream_t st = as_stream(stream);
    const int ng = strided ? 1 : G;
    for (int gi = 0; gi < ng; ++gi) {
        ApplyArgs b{};
        b.nvec = p->M * (C / 8); b.tpr_log = ilog2(C / 8); b.C = C; b.relu = p->relu;
        b.x = ps[gi].x; b.dy = ps[gi].dy; b.out = ps[gi].dx;
        b.coef = coef0 + (size_t)gi * 4 * C;
        b.fcoef = ps[gi].fwd_coef;
        b.gvec = strided ? gs / 8 : 0;
        b.cgs = strided ? 4 * C : 0;
        b.fcgs = strided ? 2 * C : 0;
        const dim3 g(apply_grid(b.nvec, C), strided ? G : 1);
        if (p->relu) hipLaunchKernelGGL((k_bn_apply_bwd<true, false, true, uint16_t>), g, dim3(kT), 0, st, b);
        else hipLaunchKernelGGL((k_bn_apply_bwd<false, false, false, uint16_t>), g, dim3(kT), 0, st, b);
        if ((rc = check_launch("k_bn_apply_bwd"))) return rc;
    }
    return GM_OK;
}
