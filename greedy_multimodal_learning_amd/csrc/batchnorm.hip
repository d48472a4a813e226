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
#include "gm_common.h"

namespace gm {
namespace {

constexpr int kT = 256;          // threads per block
constexpr int kMaxC = 2048;      // channels supported (ResNet-50 ends at 2048)
constexpr size_t kHdr = 256;     // scratch header (ticket counter)
constexpr int kFlag = 2 * kMaxC; // LDS slot of the last-arriver flag

struct Plan {
    int nblk;        // reduce blocks
    int tpr_log;     // log2(threads per row) = log2(C/8)
    long long rpb;   // rows per block
};

inline int ilog2(int v) {
    int l = 0;
    while ((1 << l) < v) ++l;
    return l;
}

inline Plan make_plan(long long M, int C) {
    Plan p;
    p.tpr_log = ilog2(C / 8);
    const int rpp = kT / (C / 8);
    // bound the partials the last block combines (nblk * 2C floats <= 128 KB) and
    // give every block >= 64 KB of x
    long long by_bytes = (M * C * 2 + 65535) / 65536;
    long long cap = 16384 / C;
    if (cap < 4) cap = 4;
    long long nb = by_bytes < cap ? by_bytes : cap;
    if (nb < 1) nb = 1;
    long long rpb = (M + nb - 1) / nb;
    rpb = (rpb + rpp - 1) / rpp * rpp;
    p.rpb = rpb;
    p.nblk = (int)((M + rpb - 1) / rpb);
    return p;
}

inline size_t scratch_bytes(long long M, int C) {
    Plan p = make_plan(M, C);
    return kHdr + (size_t)4 * C * sizeof(float) + (size_t)p.nblk * 2 * C * sizeof(float);
}

__device__ __forceinline__ void unpack8(uint4 u, float* f) {
    f[0] = bf_lo(u.x); f[1] = bf_hi(u.x); f[2] = bf_lo(u.y); f[3] = bf_hi(u.y);
    f[4] = bf_lo(u.z); f[5] = bf_hi(u.z); f[6] = bf_lo(u.w); f[7] = bf_hi(u.w);
}
__device__ __forceinline__ uint4 pack8(const float* f) {
    return make_uint4(pack_bf2(f[0], f[1]), pack_bf2(f[2], f[3]), pack_bf2(f[4], f[5]), pack_bf2(f[6], f[7]));
}

struct ReduceArgs {
    long long M;
    int C, tpr_log, relu, accumulate;
    long long rpb;
    const uint4* x;      // fwd: x; bwd: x
    const uint4* dy;     // bwd
    const uint4* y;      // bwd relu mask
    const float* gamma;
    const float* beta;
    float* rmean;
    float* rvar;
    float momentum, eps;
    float* save_mean;    // fwd: out; bwd: in
    float* save_invstd;  // fwd: out; bwd: in
    float* dgamma;
    float* dbeta;
    unsigned* counter;
    long long* nbt;      // num_batches_tracked (fwd, may be null)
    float* coef;         // [4][C]
    float* part;         // [nblk][2C]
};

enum { FWD = 0, BWD = 1, BWD_RELU = 2 };  // relu as a template arg: no per-load branch

template <int MODE>
__device__ __forceinline__ void accum(const ReduceArgs& a, long long v, const float* mu, float* s1, float* s2) {
    float xf[8];
    unpack8(a.x[v], xf);
    if (MODE == FWD) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            s1[j] += xf[j];
            s2[j] = fmaf(xf[j], xf[j], s2[j]);
        }
    } else {
        float d[8];
        unpack8(a.dy[v], d);
        if (MODE == BWD_RELU) {
            float yf[8];
            unpack8(a.y[v], yf);
#pragma unroll
            for (int j = 0; j < 8; ++j) d[j] = yf[j] > 0.f ? d[j] : 0.f;
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            s1[j] += d[j];
            s2[j] = fmaf(d[j], xf[j] - mu[j], s2[j]);
        }
    }
}

template <int MODE>
__device__ __forceinline__ void finalize(const ReduceArgs& a, int c, double S1, double S2, double invM) {
    const int C = a.C;
    const double g = (double)a.gamma[c];
    if (MODE == FWD) {
        const double mean = S1 * invM;
        double var = S2 * invM - mean * mean;
        if (var < 0.0) var = 0.0;
        const double invstd = 1.0 / sqrt(var + (double)a.eps);
        const double sc = g * invstd;
        a.coef[c] = (float)sc;
        a.coef[C + c] = (float)((double)a.beta[c] - mean * sc);
        a.save_mean[c] = (float)mean;
        a.save_invstd[c] = (float)invstd;
        if (a.rmean) {
            const double m = (double)a.momentum;
            const double unb = a.M > 1 ? var * (double)a.M / (double)(a.M - 1) : var;
            a.rmean[c] = (float)((1.0 - m) * (double)a.rmean[c] + m * mean);
            a.rvar[c] = (float)((1.0 - m) * (double)a.rvar[c] + m * unb);
        }
    } else {
        const double mean = (double)a.save_mean[c];
        const double is = (double)a.save_invstd[c];
        const double ca = g * is;
        const double cb = -g * is * is * is * S2 * invM;
        a.coef[c] = (float)ca;
        a.coef[C + c] = (float)cb;
        a.coef[2 * C + c] = (float)(-ca * S1 * invM - cb * mean);
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

// One launch: partial sums + last-arriver finalize.
template <int MODE>
__global__ __launch_bounds__(kT) void k_bn_reduce(ReduceArgs a) {
    __shared__ float red[kFlag + 4];  // the one LDS object: row-group partials, flag, fp64 combine
    const int t = threadIdx.x;
    const int C = a.C;
    const int tpr = 1 << a.tpr_log;
    const int cg = t & (tpr - 1);
    const int r0 = t >> a.tpr_log;
    const int rpp = kT >> a.tpr_log;
    const long long vpr = C >> 3;  // vectors per row

    float mu[8];
    if (MODE != FWD) {
#pragma unroll
        for (int j = 0; j < 8; ++j) mu[j] = a.save_mean[cg * 8 + j];
    }
    float s1[8], s2[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) s1[j] = s2[j] = 0.f;

    const long long rbeg = (long long)blockIdx.x * a.rpb;
    long long rend = rbeg + a.rpb;
    if (rend > a.M) rend = a.M;
    long long r = rbeg + r0;
    for (; r + 3 * rpp < rend; r += 4 * rpp) {
        const long long v = r * vpr + cg;
        const long long st = (long long)rpp * vpr;
        accum<MODE>(a, v, mu, s1, s2);
        accum<MODE>(a, v + st, mu, s1, s2);
        accum<MODE>(a, v + 2 * st, mu, s1, s2);
        accum<MODE>(a, v + 3 * st, mu, s1, s2);
    }
    for (; r < rend; r += rpp) accum<MODE>(a, r * vpr + cg, mu, s1, s2);

    // row-group combine in LDS: red[r0][C][2]  (rpp * 2C == 4096 floats)
    const int C2 = 2 * C;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        red[r0 * C2 + (cg * 8 + j) * 2] = s1[j];
        red[r0 * C2 + (cg * 8 + j) * 2 + 1] = s2[j];
    }
    __syncthreads();
    float* part = a.part + (size_t)blockIdx.x * C2;  // [nblk][C][2]
    for (int col = t; col < C2; col += kT) {
        float acc = 0.f;
        for (int i = 0; i < rpp; ++i) acc += red[i * C2 + col];
        part[col] = acc;
    }
    // hand-off: plain stores -> drain -> barrier -> agent release -> ticket
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (t == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        unsigned tk = __hip_atomic_fetch_add(a.counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        red[kFlag] = (tk == gridDim.x - 1) ? 1.f : 0.f;
    }
    __syncthreads();
    if (red[kFlag] == 0.f) return;
    if (t == 0) {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        *a.counter = 0u;  // leave the ticket at zero for the next call
        if (MODE == FWD && a.nbt) *a.nbt += 1;
    }
    __syncthreads();

    // last block: combine the nblk partial rows in fp64, in passes of <= kT float4
    // columns (= 2*kT channels); thread = (float4 column, row group)
    const int nb = gridDim.x;
    const int ncol4 = C2 >> 2;
    const int w4 = ncol4 < kT ? ncol4 : kT;
    const int groups = kT / w4;
    double* dred = reinterpret_cast<double*>(red);  // [groups][w4*4]
    const float4* p4 = reinterpret_cast<const float4*>(a.part);
    const double invM = 1.0 / (double)a.M;
    for (int base = 0; base < ncol4; base += w4) {
        const int c4 = base + t % w4;
        const int g = t / w4;
        double acc[4] = {0.0, 0.0, 0.0, 0.0};
        int b = g;
        for (; b + 3 * groups < nb; b += 4 * groups) {
            const float4 q0 = p4[(size_t)b * ncol4 + c4];
            const float4 q1 = p4[(size_t)(b + groups) * ncol4 + c4];
            const float4 q2 = p4[(size_t)(b + 2 * groups) * ncol4 + c4];
            const float4 q3 = p4[(size_t)(b + 3 * groups) * ncol4 + c4];
            acc[0] += ((double)q0.x + (double)q1.x) + ((double)q2.x + (double)q3.x);
            acc[1] += ((double)q0.y + (double)q1.y) + ((double)q2.y + (double)q3.y);
            acc[2] += ((double)q0.z + (double)q1.z) + ((double)q2.z + (double)q3.z);
            acc[3] += ((double)q0.w + (double)q1.w) + ((double)q2.w + (double)q3.w);
        }
        for (; b < nb; b += groups) {
            const float4 q = p4[(size_t)b * ncol4 + c4];
            acc[0] += q.x; acc[1] += q.y; acc[2] += q.z; acc[3] += q.w;
        }
        __syncthreads();  // previous pass done with dred
#pragma unroll
        for (int j = 0; j < 4; ++j) dred[g * w4 * 4 + (t % w4) * 4 + j] = acc[j];
        __syncthreads();
        for (int cl = t; cl < w4 * 2; cl += kT) {  // channels of this pass
            double S1 = 0.0, S2 = 0.0;
            for (int i = 0; i < groups; ++i) {
                S1 += dred[i * w4 * 4 + 2 * cl];
                S2 += dred[i * w4 * 4 + 2 * cl + 1];
            }
            finalize<MODE>(a, base * 2 + cl, S1, S2, invM);
        }
    }
}

struct ApplyArgs {
    long long nvec;      // M * C / 8
    int tpr_log;
    int relu;
    const uint4* x;
    const uint4* res;    // fwd residual / bwd: y (relu mask)
    const uint4* dy;     // bwd
    uint4* out;          // fwd y / bwd dx
    uint4* out2;         // bwd dres
    const float* coef;   // [4][C]
    int C;
};

__device__ __forceinline__ void load_coef(const float* p, int cg, float* c) {
    const float4 a = reinterpret_cast<const float4*>(p)[cg * 2];
    const float4 b = reinterpret_cast<const float4*>(p)[cg * 2 + 1];
    c[0] = a.x; c[1] = a.y; c[2] = a.z; c[3] = a.w; c[4] = b.x; c[5] = b.y; c[6] = b.z; c[7] = b.w;
}

template <bool RES, bool RELU>
__global__ __launch_bounds__(kT) void k_bn_apply(ApplyArgs a) {
    const long long stride = (long long)gridDim.x * kT;  // multiple of C/8
    long long v = (long long)blockIdx.x * kT + threadIdx.x;
    const int cg = (int)(v & ((1 << a.tpr_log) - 1));
    float sc[8], sh[8];
    load_coef(a.coef, cg, sc);
    load_coef(a.coef + a.C, cg, sh);
    auto one = [&](long long i) {
        float f[8];
        unpack8(a.x[i], f);
        float r[8];
        if (RES) unpack8(a.res[i], r);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            float z = fmaf(f[j], sc[j], sh[j]);
            if (RES) z += r[j];
            f[j] = RELU ? fmaxf(z, 0.f) : z;
        }
        a.out[i] = pack8(f);
    };
    for (; v + stride < a.nvec; v += 2 * stride) {
        one(v);
        one(v + stride);
    }
    if (v < a.nvec) one(v);
}

template <bool RELU, bool DRES>
__global__ __launch_bounds__(kT) void k_bn_apply_bwd(ApplyArgs a) {
    const long long stride = (long long)gridDim.x * kT;
    long long v = (long long)blockIdx.x * kT + threadIdx.x;
    const int cg = (int)(v & ((1 << a.tpr_log) - 1));
    float ca[8], cb[8], cc[8];
    load_coef(a.coef, cg, ca);
    load_coef(a.coef + a.C, cg, cb);
    load_coef(a.coef + 2 * a.C, cg, cc);
    auto one = [&](long long i) {
        float d[8], xf[8];
        unpack8(a.dy[i], d);
        unpack8(a.x[i], xf);
        if (RELU) {
            float yf[8];
            unpack8(a.res[i], yf);
#pragma unroll
            for (int j = 0; j < 8; ++j) d[j] = yf[j] > 0.f ? d[j] : 0.f;
        }
        if (DRES) a.out2[i] = pack8(d);
        float o[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] = fmaf(ca[j], d[j], fmaf(cb[j], xf[j], cc[j]));
        a.out[i] = pack8(o);
    };
    for (; v + stride < a.nvec; v += 2 * stride) {
        one(v);
        one(v + stride);
    }
    if (v < a.nvec) one(v);
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

extern "C" int gm_bn_fwd_train_bf16(const gm_bn_fwd* p, void* scratch, size_t bytes, void* stream) {
    GM_REQUIRE(p && p->x && p->y && p->gamma && p->beta && p->save_mean && p->save_invstd,
               "gm_bn_fwd_train_bf16: null argument");
    GM_REQUIRE(!p->running_mean == !p->running_var, "gm_bn_fwd_train_bf16: running_mean/var both or neither");
    int rc = check_common(p->M, p->C, scratch, bytes, "gm_bn_fwd_train_bf16");
    if (rc) return rc;
    const Plan pl = make_plan(p->M, p->C);
    char* s = static_cast<char*>(scratch);
    ReduceArgs a{};
    a.M = p->M; a.C = p->C; a.tpr_log = pl.tpr_log; a.rpb = pl.rpb;
    a.x = static_cast<const uint4*>(p->x);
    a.gamma = p->gamma; a.beta = p->beta; a.rmean = p->running_mean; a.rvar = p->running_var;
    a.momentum = p->momentum; a.eps = p->eps;
    a.save_mean = p->save_mean; a.save_invstd = p->save_invstd;
    a.nbt = p->num_batches_tracked;
    a.counter = reinterpret_cast<unsigned*>(s);
    a.coef = reinterpret_cast<float*>(s + kHdr);
    a.part = a.coef + 4 * p->C;
    hipStream_t st = as_stream(stream);
    hipLaunchKernelGGL(k_bn_reduce<FWD>, dim3(pl.nblk), dim3(kT), 0, st, a);
    if ((rc = check_launch("k_bn_reduce<fwd>"))) return rc;
    ApplyArgs b{};
    b.nvec = p->M * (p->C / 8); b.tpr_log = pl.tpr_log; b.C = p->C; b.relu = p->relu;
    b.x = a.x; b.res = static_cast<const uint4*>(p->residual); b.out = static_cast<uint4*>(p->y);
    b.coef = a.coef;
    const int g = apply_grid(b.nvec, p->C);
    if (p->residual) {
        if (p->relu) hipLaunchKernelGGL((k_bn_apply<true, true>), dim3(g), dim3(kT), 0, st, b);
        else hipLaunchKernelGGL((k_bn_apply<true, false>), dim3(g), dim3(kT), 0, st, b);
    } else {
        if (p->relu) hipLaunchKernelGGL((k_bn_apply<false, true>), dim3(g), dim3(kT), 0, st, b);
        else hipLaunchKernelGGL((k_bn_apply<false, false>), dim3(g), dim3(kT), 0, st, b);
    }
    return check_launch("k_bn_apply");
}

extern "C" int gm_bn_fwd_infer_bf16(const gm_bn_fwd* p, void* scratch, size_t bytes, void* stream) {
    GM_REQUIRE(p && p->x && p->y && p->gamma && p->beta && p->running_mean && p->running_var,
               "gm_bn_fwd_infer_bf16: null argument");
    int rc = check_common(p->M, p->C, scratch, bytes, "gm_bn_fwd_infer_bf16");
    if (rc) return rc;
    char* s = static_cast<char*>(scratch);
    float* coef = reinterpret_cast<float*>(s + kHdr);
    hipStream_t st = as_stream(stream);
    hipLaunchKernelGGL(k_bn_infer_coef, dim3((p->C + 255) / 256), dim3(256), 0, st, p->C, p->gamma, p->beta,
                       p->running_mean, p->running_var, p->eps, coef);
    if ((rc = check_launch("k_bn_infer_coef"))) return rc;
    ApplyArgs b{};
    b.nvec = p->M * (p->C / 8); b.tpr_log = ilog2(p->C / 8); b.C = p->C; b.relu = p->relu;
    b.x = static_cast<const uint4*>(p->x); b.res = static_cast<const uint4*>(p->residual);
    b.out = static_cast<uint4*>(p->y); b.coef = coef;
    const int g = apply_grid(b.nvec, p->C);
    if (p->residual) {
        if (p->relu) hipLaunchKernelGGL((k_bn_apply<true, true>), dim3(g), dim3(kT), 0, st, b);
        else hipLaunchKernelGGL((k_bn_apply<true, false>), dim3(g), dim3(kT), 0, st, b);
    } else {
        if (p->relu) hipLaunchKernelGGL((k_bn_apply<false, true>), dim3(g), dim3(kT), 0, st, b);
        else hipLaunchKernelGGL((k_bn_apply<false, false>), dim3(g), dim3(kT), 0, st, b);
    }
    return check_launch("k_bn_apply");
}

extern "C" int gm_bn_bwd_bf16(const gm_bn_bwd* p, void* scratch, size_t bytes, void* stream) {
    GM_REQUIRE(p && p->dy && p->x && p->gamma && p->save_mean && p->save_invstd && p->dx && p->dgamma && p->dbeta,
               "gm_bn_bwd_bf16: null argument");
    GM_REQUIRE(!p->relu || p->y, "gm_bn_bwd_bf16: relu needs the forward output y");
    int rc = check_common(p->M, p->C, scratch, bytes, "gm_bn_bwd_bf16");
    if (rc) return rc;
    const Plan pl = make_plan(p->M, p->C);
    char* s = static_cast<char*>(scratch);
    ReduceArgs a{};
    a.M = p->M; a.C = p->C; a.tpr_log = pl.tpr_log; a.rpb = pl.rpb; a.relu = p->relu;
    a.accumulate = p->accumulate;
    a.x = static_cast<const uint4*>(p->x); a.dy = static_cast<const uint4*>(p->dy);
    a.y = static_cast<const uint4*>(p->y);
    a.gamma = p->gamma;
    a.save_mean = const_cast<float*>(p->save_mean); a.save_invstd = const_cast<float*>(p->save_invstd);
    a.dgamma = p->dgamma; a.dbeta = p->dbeta;
    a.counter = reinterpret_cast<unsigned*>(s);
    a.coef = reinterpret_cast<float*>(s + kHdr);
    a.part = a.coef + 4 * p->C;
    hipStream_t st = as_stream(stream);
    if (p->relu) hipLaunchKernelGGL(k_bn_reduce<BWD_RELU>, dim3(pl.nblk), dim3(kT), 0, st, a);
    else hipLaunchKernelGGL(k_bn_reduce<BWD>, dim3(pl.nblk), dim3(kT), 0, st, a);
    if ((rc = check_launch("k_bn_reduce<bwd>"))) return rc;
    ApplyArgs b{};
    b.nvec = p->M * (p->C / 8); b.tpr_log = pl.tpr_log; b.C = p->C; b.relu = p->relu;
    b.x = a.x; b.res = a.y; b.dy = a.dy; b.out = static_cast<uint4*>(p->dx);
    b.out2 = static_cast<uint4*>(p->dres); b.coef = a.coef;
    const int g = apply_grid(b.nvec, p->C);
    if (p->relu) {
        if (p->dres) hipLaunchKernelGGL((k_bn_apply_bwd<true, true>), dim3(g), dim3(kT), 0, st, b);
        else hipLaunchKernelGGL((k_bn_apply_bwd<true, false>), dim3(g), dim3(kT), 0, st, b);
    } else {
        if (p->dres) hipLaunchKernelGGL((k_bn_apply_bwd<false, true>), dim3(g), dim3(kT), 0, st, b);
        else hipLaunchKernelGGL((k_bn_apply_bwd<false, false>), dim3(g), dim3(kT), 0, st, b);
    }
    return check_launch("k_bn_apply_bwd");
}
