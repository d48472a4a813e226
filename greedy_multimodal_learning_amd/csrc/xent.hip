// Branch-summed cross-entropy of the training step (reference train.py:22-29 blend_loss:
// loss = sum over branches of F.cross_entropy(logits_branch, y), mean over the batch)
// and its gradient, for all branches in one launch each.  Replaces ~20 small
// PyTorch kernels (log_softmax / nll_loss forward and backward per branch, fills,
// the branch sum) at the end of the step.
//
//   gm_xent_fwd: rows r = br*B + b; lse_r = log sum_n exp(x[r,n]) (max-shifted fp32,
//                as log_softmax), loss = sum_br (1/B) sum_b (lse_r - x[r, y_b]); one
//                workgroup, row losses combined in fp64 in a fixed order: deterministic.
//                A label outside [0, N) makes the loss NaN (PyTorch asserts).
//   gm_xent_bwd: dx[r,n] = g * (exp(x[r,n] - lse_r) - [n == y_b]) / B, g = *gout
//                (the loss's incoming gradient, read on the device).
#include "gm_common.h"

namespace gm {
namespace {

constexpr int kXT = 256;

__device__ __forceinline__ float row_lse(const float* x, int N) {
    float m = -INFINITY;
    for (int n = 0; n < N; ++n) m = fmaxf(m, x[n]);
    float s = 0.f;
    for (int n = 0; n < N; ++n) s += expf(x[n] - m);
    return m + logf(s);
}

__global__ __launch_bounds__(kXT) void k_xent_fwd(const float* __restrict__ x, int rows, int B, int N,
                                                  const long long* __restrict__ y, float* __restrict__ lse,
                                                  float* __restrict__ loss) {
    __shared__ double red[kXT];
    const int t = threadIdx.x;
    double acc = 0.0;
    for (int r = t; r < rows; r += kXT) {
        const float* xr = x + (size_t)r * N;
        const float l = row_lse(xr, N);
        lse[r] = l;
        const long long lab = y[r % B];
        const float v = (lab >= 0 && lab < N) ? l - xr[lab] : NAN;
        acc += (double)v;
    }
    red[t] = acc;
    __syncthreads();
    for (int s = kXT / 2; s > 0; s >>= 1) {
        if (t < s) red[t] += red[t + s];
        __syncthreads();
    }
    if (t == 0) *loss = (float)(red[0] / (double)B);
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
    hipLaunchKernelGGL(k_xent_fwd, dim3(1), dim3(kXT), 0, as_stream(stream), logits, nbranch * B, B, N, labels,
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
