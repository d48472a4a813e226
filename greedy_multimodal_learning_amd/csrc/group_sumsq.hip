// Per-branch weight/gradient norms (+ fused SGD) for the conditional-learning-
// speed gate: one multi-tensor pass over all parameters and gradients.
//
// Reference: Bias_Mitigation_Strong.compute_BDR (src/callbacks.py:199-233) runs
// `(p**2).sum().item()` and `(g**2).sum().item()` for each of the 142 parameter
// tensors (284 host syncs per step) and then torch.optim.SGD updates them
// (train.py:48-51).  Here: ONE streaming pass.  The virtual concatenation of all
// tensors is cut into fixed chunks; each workgroup streams its chunk with 16-byte
// loads, accumulates per-thread fp32 partials per tensor segment, folds them into
// fp64 per-group sums, and writes one fp64 row per workgroup; a second 1-block
// pass adds the rows in fixed order.  HBM bytes/step: 8*N (read p, g) without the
// update, 12*N with it (read p, g; write p).  Deterministic.
#include "gm_common.h"
#include "gate_rule.h"

namespace gm {

constexpr int kChunk = 16384;     // minimum elements per workgroup
constexpr int kMaxRows = 4096;    // larger totals get longer chunks (fewer rows to finalize)
constexpr int kMaxGroups = 32;  // group_mask bits; 8-group instantiation for <= 4 branches

// Elements per workgroup: 16384, or a multiple of 4096 keeping the grid (= the finalize
// rows) at <= kMaxRows.  C2 (23.8 M elements) stays at 16384; C5 (415 M) gets 102400:
// 4055 rows instead of 25 345, which cost the 1-block finalize 0.71 ms.
__host__ __device__ inline long long chunk_elems(long long total) {
    const long long per = (total + kMaxRows - 1) / kMaxRows;
    const long long c = (per + 4095) / 4096 * 4096;
    return c > kChunk ? c : kChunk;
}

__device__ __forceinline__ int find_tensor(const gm_tensor* t, int nt, long long e) {
    int lo = 0, hi = nt - 1;
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (t[mid].offset <= e) lo = mid; else hi = mid - 1;
    }
    return lo;
}

// Streams elements [tb, te) of one tensor: accumulates w^2 and (gscale*g)^2 into sw, sg
// and applies the SGD update in place.
template <bool SGD>
__device__ __forceinline__ void stream_segment(const gm_tensor& T, long long tb, long long te,
                                               float gscale, float lr, float& sw, float& sg) {
    float* __restrict__ p = T.param;
    const float* __restrict__ gr = T.grad;
    // scalar head up to 16-byte alignment of p (and g)
    long long a = tb;
    const bool vec_ok = gr == nullptr || (((uintptr_t)(p + a) ^ (uintptr_t)(gr + a)) & 15) == 0;
    long long head = a;
    if (vec_ok) {
        while (head < te && ((uintptr_t)(p + head) & 15)) ++head;
    } else {
        head = te;
    }
    for (long long i = a + threadIdx.x; i < head; i += 256) {
        const float w = p[i];
        const float g = gr ? gr[i] * gscale : 0.f;
        sw = fmaf(w, w, sw);
        sg = fmaf(g, g, sg);
        if (SGD && gr) p[i] = fmaf(-lr, g, w);
    }
    const long long nv = (te - head) >> 2;
    float4* pv = (float4*)(p + head);
    const float4* gv = (const float4*)(gr ? gr + head : nullptr);
    long long i0 = threadIdx.x;
    if (gr) {
        // 4 independent 16-B loads of each stream in flight per thread
        for (; i0 + 3 * 256 < nv; i0 += 4 * 256) {
            float4 w[4], g[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) { w[u] = pv[i0 + u * 256]; g[u] = gv[i0 + u * 256]; }
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                sw = fmaf(w[u].x, w[u].x, sw); sw = fmaf(w[u].y, w[u].y, sw);
                sw = fmaf(w[u].z, w[u].z, sw); sw = fmaf(w[u].w, w[u].w, sw);
                g[u].x *= gscale; g[u].y *= gscale; g[u].z *= gscale; g[u].w *= gscale;
                sg = fmaf(g[u].x, g[u].x, sg); sg = fmaf(g[u].y, g[u].y, sg);
                sg = fmaf(g[u].z, g[u].z, sg); sg = fmaf(g[u].w, g[u].w, sg);
                if (SGD)
                    pv[i0 + u * 256] = make_float4(fmaf(-lr, g[u].x, w[u].x), fmaf(-lr, g[u].y, w[u].y),
                                                   fmaf(-lr, g[u].z, w[u].z), fmaf(-lr, g[u].w, w[u].w));
            }
        }
    }
    for (long long i = i0; i < nv; i += 256) {
        const float4 w = pv[i];
        sw = fmaf(w.x, w.x, sw); sw = fmaf(w.y, w.y, sw);
        sw = fmaf(w.z, w.z, sw); sw = fmaf(w.w, w.w, sw);
        if (gr) {
            float4 g = gv[i];
            g.x *= gscale; g.y *= gscale; g.z *= gscale; g.w *= gscale;
            sg = fmaf(g.x, g.x, sg); sg = fmaf(g.y, g.y, sg);
            sg = fmaf(g.z, g.z, sg); sg = fmaf(g.w, g.w, sg);
            if (SGD)
                pv[i] = make_float4(fmaf(-lr, g.x, w.x), fmaf(-lr, g.y, w.y),
                                    fmaf(-lr, g.z, w.z), fmaf(-lr, g.w, w.w));
        }
    }
    for (long long i = head + nv * 4 + threadIdx.x; i < te; i += 256) {
        const float w = p[i];
        const float g = gr ? gr[i] * gscale : 0.f;
        sw = fmaf(w, w, sw);
        sg = fmaf(g, g, sg);
        if (SGD && gr) p[i] = fmaf(-lr, g, w);
    }
}

template <bool SGD, int MG>
__global__ __launch_bounds__(256) void k_group_sumsq(const gm_tensor* __restrict__ tab, int nt,
                                                     long long total, int ngroups, float gscale,
                                                     float lr, long long chunk, double* __restrict__ rows) {
    __shared__ double sred[4][2 * MG];
    const long long e0 = (long long)blockIdx.x * chunk;
    const long long e1 = min(total, e0 + chunk);
    double gw[MG], gg[MG];
#pragma unroll
    for (int g = 0; g < MG; ++g) { gw[g] = 0.0; gg[g] = 0.0; }
    int ti = find_tensor(tab, nt, e0);
    long long e = e0;
    while (e < e1) {
        const gm_tensor T = tab[ti];
        const long long tb = e - T.offset;                       // first local element
        const long long te = min(T.n, e1 - T.offset);            // end (exclusive)
        float sw = 0.f, sg = 0.f;
        stream_segment<SGD>(T, tb, te, gscale, lr, sw, sg);
        const unsigned m = T.group_mask;
#pragma unroll
        for (int g = 0; g < MG; ++g)
            if (g < ngroups && ((m >> g) & 1u)) { gw[g] += (double)sw; gg[g] += (double)sg; }
        e = T.offset + te;
        ++ti;
    }
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
    for (int g = 0; g < MG; ++g) {
        if (g >= ngroups) break;
        const double w = wave_sum_d(gw[g]);
        const double s = wave_sum_d(gg[g]);
        if (lane == 0) { sred[wave][2 * g] = w; sred[wave][2 * g + 1] = s; }
    }
    __syncthreads();
    if (threadIdx.x < 2 * ngroups) {
        const int j = threadIdx.x;
        rows[(size_t)blockIdx.x * 2 * ngroups + j] = ((sred[0][j] + sred[1][j]) + sred[2][j]) + sred[3][j];
    }
}

// Many-group form (N-branch gates, up to 32 groups).  The per-thread fp64 arrays of the
// form above cost 128 VGPRs at 32 groups (2.6 TB/s on C5).  Segments are uniform across
// the workgroup, so here each thread keeps ONE fp64 pair for the current run of tensors
// with the same group mask; when the mask changes (a few times per chunk) the workgroup
// reduces the run in fixed order and thread 0 adds it to the LDS per-group sums.
__device__ __forceinline__ void flush_run(double& aw, double& ag, unsigned mask, int ngroups,
                                          double (*sred)[2], double* acc) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const double w = wave_sum_d(aw), g = wave_sum_d(ag);
    if (lane == 0) { sred[wave][0] = w; sred[wave][1] = g; }
    __syncthreads();
    if (threadIdx.x == 0) {
        const double tw = ((sred[0][0] + sred[1][0]) + sred[2][0]) + sred[3][0];
        const double tg = ((sred[0][1] + sred[1][1]) + sred[2][1]) + sred[3][1];
        for (int k = 0; k < ngroups; ++k)
            if ((mask >> k) & 1u) { acc[2 * k] += tw; acc[2 * k + 1] += tg; }
    }
    __syncthreads();
    aw = 0.0;
    ag = 0.0;
}

template <bool SGD>
__global__ __launch_bounds__(256) void k_group_sumsq_runs(const gm_tensor* __restrict__ tab, int nt,
                                                          long long total, int ngroups, float gscale,
                                                          float lr, long long chunk, double* __restrict__ rows) {
    __shared__ double sred[4][2];
    __shared__ double acc[2 * kMaxGroups];
    if (threadIdx.x < 2 * kMaxGroups) acc[threadIdx.x] = 0.0;
    const long long e0 = (long long)blockIdx.x * chunk;
    const long long e1 = min(total, e0 + chunk);
    int ti = find_tensor(tab, nt, e0);
    unsigned cur = tab[ti].group_mask;
    double aw = 0.0, ag = 0.0;
    long long e = e0;
    while (e < e1) {
        const gm_tensor T = tab[ti];
        if (T.group_mask != cur) {
            flush_run(aw, ag, cur, ngroups, sred, acc);
            cur = T.group_mask;
        }
        const long long tb = e - T.offset;
        const long long te = min(T.n, e1 - T.offset);
        float sw = 0.f, sg = 0.f;
        stream_segment<SGD>(T, tb, te, gscale, lr, sw, sg);
        aw += (double)sw;
        ag += (double)sg;
        e = T.offset + te;
        ++ti;
    }
    flush_run(aw, ag, cur, ngroups, sred, acc);
    if (threadIdx.x < 2 * ngroups) rows[(size_t)blockIdx.x * 2 * ngroups + threadIdx.x] = acc[threadIdx.x];
}

// 1024 threads stream the [nrows][w] row block as one flat array with fully coalesced
// 8-byte loads: thread t < S (S = the largest multiple of w <= 1024) owns column t % w and
// reads elements t, t + S, ... (8 in flight).  The former form gave each thread whole
// 128-B rows (every load instruction touched 64 cache lines; 13 us on the serial end of
// the C2 step for 1451 rows).  Then per column 32 fixed partial sums of its slots and
// their fixed-order total => deterministic.  (Threads t >= S hold 0 and take no part.)
constexpr int kFinT = 1024;
// gate (optional): the on-device gate's state - gm_gate_state (gate_n 0) or gm_gate_state_n (1) -
// whose step rule thread 0 applies to the finished sums (gm_group_sumsq_gate: no gate launch)
__global__ __launch_bounds__(kFinT) void k_group_finalize(const double* __restrict__ rows, int nrows,
                                                          int ngroups, double* __restrict__ out,
                                                          void* gate = nullptr, int gate_n = 0) {
    __shared__ double s[kFinT];
    __shared__ double tot_s[2 * kMaxGroups];
    __shared__ double part[32 * 2 * kMaxGroups];
    const int w = 2 * ngroups;
    const int S = (kFinT / w) * w, R = S / w;  // R row slots per column
    const int t = threadIdx.x;
    const long long n = (long long)nrows * w;
    double acc = 0.0;
    if (t < S) {
        long long e = t;
        for (; e + 7ll * S < n; e += 8ll * S) {
            double v[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) v[u] = rows[e + u * (long long)S];
#pragma unroll
            for (int u = 0; u < 8; ++u) acc += v[u];
        }
        for (; e < n; e += S) acc += rows[e];
    }
    s[t] = acc;
    __syncthreads();
    const int P = min(32, R);  // partial sums per column (R = kFinT / w >= 16)
    if (t < P * w) {  // column c = t % w, partial q = t / w over slots q, q + P, ...
        const int c = t % w, q = t / w;
        double p = 0.0;
        for (int j = q; j < R; j += P) p += s[j * w + c];
        part[q * w + c] = p;
    }
    __syncthreads();
    if (t < w) {
        double tot = 0.0;
        for (int q = 0; q < P; ++q) tot += part[q * w + t];
        out[t] = tot;
        tot_s[t] = tot;
    }
    if (gate == nullptr) return;  // (uniform)
    __syncthreads();
    if (t == 0) {
        if (gate_n) gate_strong_rule_n(tot_s, static_cast<gm_gate_state_n*>(gate));
        else gate_strong_rule(tot_s, static_cast<gm_gate_state*>(gate));
    }
}

}  // namespace gm

using namespace gm;

extern "C" size_t gm_group_sumsq_scratch(long long total) {
    if (total <= 0) return 0;
    const long long nb = (total + chunk_elems(total) - 1) / chunk_elems(total);
    return (size_t)nb * 2 * kMaxGroups * sizeof(double);
}

static int group_sumsq(const gm_tensor* table, int nt, long long total, int ngroups, float gscale, float lr,
                       double* out, void* scratch, size_t scratch_bytes, void* gate, int gate_n, void* stream) {
    GM_REQUIRE(table && nt >= 1 && total >= 1, "group_sumsq: empty tensor table");
    GM_REQUIRE(ngroups >= 1 && ngroups <= kMaxGroups, "group_sumsq: ngroups must be 1..%d", kMaxGroups);
    GM_REQUIRE(out, "group_sumsq: null output");
    const long long chunk = chunk_elems(total);
    const long long nb = (total + chunk - 1) / chunk;
    GM_REQUIRE(nb < (1ll << 31), "group_sumsq: too many elements");
    GM_REQUIRE(scratch && scratch_bytes >= gm_group_sumsq_scratch(total),
               "group_sumsq: scratch %zu < %zu bytes", scratch_bytes, gm_group_sumsq_scratch(total));
    hipStream_t st = as_stream(stream);
    double* rows = (double*)scratch;
    if (ngroups <= 8) {
        if (lr != 0.f)
            k_group_sumsq<true, 8><<<(int)nb, 256, 0, st>>>(table, nt, total, ngroups, gscale, lr, chunk, rows);
        else
            k_group_sumsq<false, 8><<<(int)nb, 256, 0, st>>>(table, nt, total, ngroups, gscale, lr, chunk, rows);
    } else {  // N-branch gates (C5: 12 branches -> 24 groups)
        if (lr != 0.f)
            k_group_sumsq_runs<true><<<(int)nb, 256, 0, st>>>(table, nt, total, ngroups, gscale, lr, chunk, rows);
        else
            k_group_sumsq_runs<false><<<(int)nb, 256, 0, st>>>(table, nt, total, ngroups, gscale, lr, chunk, rows);
    }
    int rc = check_launch("k_group_sumsq");
    if (rc) return rc;
    k_group_finalize<<<1, kFinT, 0, st>>>(rows, (int)nb, ngroups, out, gate, gate_n);
    return check_launch("k_group_finalize");
}

extern "C" int gm_group_sumsq(const gm_tensor* table, int nt, long long total, int ngroups, float gscale,
                              float lr, double* out, void* scratch, size_t scratch_bytes, void* stream) {
    return group_sumsq(table, nt, total, ngroups, gscale, lr, out, scratch, scratch_bytes, nullptr, 0, stream);
}

extern "C" int gm_group_sumsq_gate(const gm_tensor* table, int nt, long long total, int ngroups, float gscale,
                                   float lr, double* out, void* scratch, size_t scratch_bytes, void* gate,
                                   int gate_n, void* stream) {
    GM_REQUIRE(gate, "group_sumsq_gate: null gate state");
    // (main, bypass) groups per branch: 4 for the two-branch gate, 2 nb for the N-branch one (nb in
    // the state: the rule reads 4 nb sums)
    GM_REQUIRE(gate_n ? (ngroups >= 4 && ngroups % 2 == 0) : ngroups == 4,
               "group_sumsq_gate: %d groups do not match the %s gate", ngroups, gate_n ? "N-branch" : "two-branch");
    return group_sumsq(table, nt, total, ngroups, gscale, lr, out, scratch, scratch_bytes, gate, gate_n ? 1 : 0,
                       stream);
}
