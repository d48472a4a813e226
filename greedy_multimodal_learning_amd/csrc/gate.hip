// On-device conditional-learning-speed gate: the curation decision of
// Bias_Mitigation_Strong.on_backward_end (reference src/callbacks.py:199-267) made by a
// one-thread kernel right after the fused norms+SGD pass, and the MMTM curation
// substitution (src/balanced_mmtm.py:135-152) driven by the resulting device flags, so a
// training step needs no host synchronisation: one hipGraph serves every curation
// setting and steps are enqueued back to back.
//
// State (gm_gate_state, device memory, owned by the caller):
//   curation_mode, caring (-1 = None), curation_step, unlock, window, n_curated (steps
//   that ran curated, a statistic), eps, M = {bypass0, bypass1, main0, main1}, d_bdr.
// Step rule, exactly the reference's (fp64, C log10 = numpy's IEEE behaviour):
//   unlocked & not curating: M += g/w ratios; d = log10(Mb0/Mm0) - log10(Mb1/Mm1);
//                            |d| > eps -> curate, caring = d < 0 ? 1 : 0; else caring 0
//   unlocked & curating:     curation_step += 1; stop at the window
//   locked:                  d as above, no curation, caring 0
#include <cstddef>

#include "gm_common.h"
#include "gate_rule.h"

namespace gm {
namespace {

// the gated MMTM kernels read curation_mode / caring through a gm_gate_state pointer
static_assert(offsetof(gm_gate_state_n, curation_mode) == offsetof(gm_gate_state, curation_mode) &&
                  offsetof(gm_gate_state_n, caring) == offsetof(gm_gate_state, caring) &&
                  offsetof(gm_gate_state_n, unlock) == offsetof(gm_gate_state, unlock),
              "gm_gate_state_n must share gm_gate_state's prefix");

__global__ void k_gate_strong(const double* __restrict__ s, gm_gate_state* st) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    gate_strong_rule(s, st);
}

// N branches (C4 / C5): gate_strong_rule_n (gate_rule.h)
__global__ void k_gate_strong_n(const double* __restrict__ s, gm_gate_state_n* st) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    gate_strong_rule_n(s, st);
}

// effective MMTM scales under the device flags: the cared-for modality's scale is the
// (already updated) running average broadcast over the batch, the other stays live;
// mask[m] = 0 for the substituted modality (its excitation path gets no gradient)
__global__ __launch_bounds__(256) void k_select_scale(const float* __restrict__ e_v, int ld_v,
                                                      const float* __restrict__ e_s, int ld_s,
                                                      const float* __restrict__ ra_v,
                                                      const float* __restrict__ ra_s, int B, int Cv, int Cs,
                                                      const gm_gate_state* __restrict__ st, float* __restrict__ s_v,
                                                      float* __restrict__ s_s, float* __restrict__ mask) {
    const int cur = st->curation_mode, car = st->caring;
    const bool sub_v = cur && car == 0, sub_s = cur && car == 1;
    const long long nv = (long long)B * Cv, ns = (long long)B * Cs;
    for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < nv + ns; i += (long long)gridDim.x * 256) {
        if (i < nv) {
            const int b = (int)(i / Cv), c = (int)(i - (long long)b * Cv);
            s_v[i] = sub_v ? ra_v[c] : e_v[(size_t)b * ld_v + c];
        } else {
            const long long j = i - nv;
            const int b = (int)(j / Cs), c = (int)(j - (long long)b * Cs);
            s_s[j] = sub_s ? ra_s[c] : e_s[(size_t)b * ld_s + c];
        }
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        mask[0] = sub_v ? 0.f : 1.f;
        mask[1] = sub_s ? 0.f : 1.f;
    }
}

__global__ __launch_bounds__(256) void k_mask_rows(float* __restrict__ a, long long n, const float* __restrict__ m) {
    const float k = *m;
    for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long long)gridDim.x * 256) a[i] *= k;
}

// both modalities' rows in one launch: a[i] *= m[0], b[i] *= m[1]
__global__ __launch_bounds__(256) void k_mask_rows2(float* __restrict__ a, long long na, float* __restrict__ b,
                                                    long long nb, const float* __restrict__ m) {
    const float ka = m[0], kb = m[1];
    const long long st = (long long)gridDim.x * 256;
    for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < na + nb; i += st) {
        if (i < na) a[i] *= ka;
        else b[i - na] *= kb;
    }
}

}  // namespace
}  // namespace gm

using namespace gm;

extern "C" int gm_gate_strong_step(const double* sums, gm_gate_state* state, void* stream) {
    GM_REQUIRE(sums && state, "gm_gate_strong_step: null pointer");
    k_gate_strong<<<1, 64, 0, as_stream(stream)>>>(sums, state);
    return check_launch("k_gate_strong");
}

extern "C" int gm_gate_strong_step_n(const double* sums, gm_gate_state_n* state, void* stream) {
    GM_REQUIRE(sums && state, "gm_gate_strong_step_n: null pointer");
    k_gate_strong_n<<<1, 64, 0, as_stream(stream)>>>(sums, state);
    return check_launch("k_gate_strong_n");
}

extern "C" int gm_mmtm_select_scale(const float* e_v, int ld_v, const float* e_s, int ld_s, const float* ra_v,
                                    const float* ra_s, int B, int Cv, int Cs, const gm_gate_state* state,
                                    float* s_v, float* s_s, float* mask, void* stream) {
    GM_REQUIRE(e_v && e_s && ra_v && ra_s && state && s_v && s_s && mask && B > 0 && Cv > 0 && Cs > 0,
               "gm_mmtm_select_scale: bad arguments");
    const long long n = (long long)B * (Cv + Cs);
    int g = (int)((n + 255) / 256);
    g = g > 1024 ? 1024 : g;
    k_select_scale<<<g, 256, 0, as_stream(stream)>>>(e_v, ld_v, e_s, ld_s, ra_v, ra_s, B, Cv, Cs, state, s_v, s_s,
                                                     mask);
    return check_launch("k_select_scale");
}

extern "C" int gm_mmtm_mask_rows(float* a, long long n, const float* mask, void* stream) {
    GM_REQUIRE(a && mask && n > 0, "gm_mmtm_mask_rows: bad arguments");
    int g = (int)((n + 255) / 256);
    g = g > 1024 ? 1024 : g;
    k_mask_rows<<<g, 256, 0, as_stream(stream)>>>(a, n, mask);
    return check_launch("k_mask_rows");
}

extern "C" int gm_mmtm_mask_rows2(float* a, long long na, float* b, long long nb, const float* mask, void* stream) {
    GM_REQUIRE(a && b && mask && na > 0 && nb > 0, "gm_mmtm_mask_rows2: bad arguments");
    long long g = (na + nb + 255) / 256;
    g = g > 1024 ? 1024 : g;
    k_mask_rows2<<<(int)g, 256, 0, as_stream(stream)>>>(a, na, b, nb, mask);
    return check_launch("k_mask_rows2");
}
