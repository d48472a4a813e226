// Branch-summed cross-entropy of the training step (reference train.py:22-29 blend_loss:
// loss = sum over branches of F.cross_entropy(logits_branch, y), mean over the batch)
// and its gradient, for all branches in one launch each.  Replaces ~20 small
// PyTorch kernels (log_softmax / nll_loss forward and backward per branch, fills,
// the branch sum) at the end of the step.
//
//   gm_xent_fwd: rows r = br*B + b; lse_r = log sum_n exp(x[r,n]) (max-shifted fp32,
//                as log_softmax), loss = sum_br (1/B) sum_b (lse_r - x[r, y_b]); one
//                workgroup (a wave per row), row losses combined in fp64 in a fixed
//                order: deterministic.
//                A label outside [0, N) makes the loss NaN (PyTorch asserts).
//   gm_xent_bwd: dx[r,n] = g * (exp(x[r,n] - lse_r) - [n == y_b]) / B, g = *gout
//                (the loss's incoming gradient, read on the device).
#include "gm_common.h"

namespace gm {
namespace {

constexpr int kXT = 256;

// Forward: one wave per row (lanes over the classes, wave max / sum by shuffles), four
// rows per wave in flight, 16 waves.  The former thread-per-row form walked a row's N
// logits twice one dependent load at a time (10 us for 128 rows x 40 classes, on the
// serial path between the heads and the backward).  Row losses are summed per wave in
// its fixed row order, then over the waves in fixed order (fp64): deterministic.
constexpr int kXF = 1024, kXW = kXF / 64, kXU = 4;

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
    return v;
}

__global__ __launch_bounds__(kXF) void k_xent_fwd(const float* __restrict__ x, int rows, int B, int N,
                                                  const long long* __restrict__ y, float* __restrict__ lse,
                                                  float* __restrict__ loss) {
    __shared__ double wsum[kXW];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    double acc = 0.0;  // lane 0's running row-loss sum
    for (int rb = wave; rb < rows; rb += kXU * kXW) {
        float m[kXU], sm[kXU];
#pragma unroll
        for (int u = 0; u < kXU; ++u) {
            const int r = rb + u * kXW;
            m[u] = -INFINITY;
            if (r < rows)
                for (int n = lane; n < N; n += 64) m[u] = fmaxf(m[u], x[(size_t)r * N + n]);
        }
#pragma unroll
        for (int u = 0; u < kXU; ++u) m[u] = wave_max(m[u]);
#pragma unroll
        for (int u = 0; u < kXU; ++u) {
            const int r = rb + u * kXW;
            sm[u] = 0.f;
            if (r < rows)
                for (int n = lane; n < N; n += 64) sm[u] += expf(x[(size_t)r * N + n] - m[u]);
        }
#pragma unroll
        for (int u = 0; u < kXU; ++u) sm[u] = wave_sum(sm[u]);
        if (lane == 0) {
#pragma unroll
            for (int u = 0; u < kXU; ++u) {
                const int r = rb + u * kXW;
                if (r >= rows) break;
                const float l = m[u] + logf(sm[u]);
                lse[r] = l;
                const long long lab = y[r % B];
                acc += (double)((lab >= 0 && lab < N) ? l - x[(size_t)r * N + lab] : NAN);
            }
        }
    }
    if (lane == 0) wsum[wave] = acc;
    __syncthreads();
    if (threadIdx.x == 0) {
        double t = 0.0;
        for (int w = 0; w < kXW; ++w) t += wsum[w];
        *loss = (float)(t / (double)B);
    }
}

__global__ __launch_bounds__(kXT) void k_xent_bwd(const float* __restrict__ x, const float* __restrict__ lse,
                                                  int rows, int B, int N, const long long* __restrict__ y,
                                                  const float* __restrict__ gout, float* __restrict__ dx) {
    const long long i = (long long)blockIdx.x * kXT + threadIdx.x;
    if (i >= (long long)rows * N) return;
    const int r = (int)(i / N), n = (int)(i - (long long)r * N);
    const float g = *gout / (float)B;
    const float p = expf(x[i] - lse[r]);
    dx[i] = g * (p - (y[r % B] == n ? 1.f : 0.f));
}

}  // namespace
}  // namespace gm

using namespace gm;

extern "C" int gm_xent_fwd(const float* logits, int nbranch, int B, int N, const long long* labels, float* lse,
                           float* loss, void* stream) {
    GM_REQUIRE(logits && labels && lse && loss, "gm_xent_fwd: null argument");
    GM_REQUIRE(nbranch > 0 && B > 0 && N > 0, "gm_xent_fwd: need nbranch, B, N > 0");
    hipLaunchKernelGGL(k_xent_fwd, dim3(1), dim3(kXF), 0, as_stream(stream), logits, nbranch * B, B, N, labels,
                       lse, loss);
    return check_launch("k_xent_fwd");
}

extern "C" int gm_xent_bwd(const float* logits, const float* lse, int nbranch, int B, int N,
                           const long long* labels, const float* gout, float* dlogits, void* stream) {
    GM_REQUIRE(logits && lse && labels && gout && dlogits, "gm_xent_bwd: null argument");
    GM_REQUIRE(nbranch > 0 && B > 0 && N > 0, "gm_xent_bwd: need nbranch, B, N > 0");
    const long long n = (long long)nbranch * B * N;
    hipLaunchKernelGGL(k_xent_bwd, dim3((unsigned)((n + kXT - 1) / kXT)), dim3(kXT), 0, as_stream(stream), logits,
                       lse, nbranch * B, B, N, labels, gout, dlogits);
    return check_launch("k_xent_bwd");
}
