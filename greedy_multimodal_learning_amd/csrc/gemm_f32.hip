// Small fp32 GEMMs of the MMTM joint FC on MFMA (gfx950 v_mfma_f32_16x16x4_f32).
//
// The MMTM layers are [B, 2C] x [2C, C'] and [B, C'] x [C', C] with B <= 256 and
// C <= 512 (plus their weight/input gradients): a few MFLOP, L2-resident, so the
// kernel is latency/parallelism-bound, not HBM- or MFMA-bound.  Design:
//   * each wave computes one 16x16 output tile over a K range with the exact-f32
//     MFMA (an fmaf chain: same numerics as the fp32 reference's FMA GEMMs);
//   * a 256-thread workgroup holds TM x TN tiles x KS K-splits (TM*TN*KS = 4);
//     split-K partial tiles are summed through LDS in fixed order (deterministic);
//   * operands are generic strided views (ld0 = 0 broadcasts a row, ptr = NULL
//     means an all-ones operand) so transposes, concatenated inputs and bias
//     gradients need no copies; up to 6 problems run in one launch;
//   * fused epilogue: bias, relu / sigmoid, relu-backward mask, accumulate.
#include <cstring>

#include "gm_common.h"

namespace gm {

constexpr int kMaxGemm = 6;
typedef float floatx4 __attribute__((ext_vector_type(4)));

struct GemmArgs {
    gm_gemm p[kMaxGemm];
    int tile_start[kMaxGemm + 1];
    int tiles_n[kMaxGemm];  // workgroup tiles along N
    int cfg[kMaxGemm];      // TM | TN<<4 | KS<<8
    int nprob;
};

// One K-segment of a wave's 16x16 tile: k in [k0, k1) (segment-local), stepping 4.
// Lane (li, lk) reads A[m0+li][k+lk] and B[k+lk][n0+li]; pointers advance by
// 4*ld1 / 4*ld0 per step.  8 steps (32 k) per iteration with the next
// iteration's 16 loads issued before this iteration's 8 MFMAs (register
// double-buffer), so L2 latency hides behind MFMA issue.
__device__ __forceinline__ void seg_mma(floatx4& acc, const gm_operand& A, const gm_operand& B,
                                        int m, int n, bool mrow, bool ncol, int lk, int k0, int k1) {
    if (k1 <= k0) return;
    const bool aone = A.ptr == nullptr;
    const float* pa = aone ? nullptr : A.ptr + (long)m * A.ld0 + (long)(k0 + lk) * A.ld1;
    const float* pb = B.ptr + (long)(k0 + lk) * B.ld0 + (long)n * B.ld1;
    const long sa = 4l * A.ld1, sb = 4l * B.ld0;
    const bool va = mrow && !aone, vb = ncol;
    const float one = mrow ? 1.0f : 0.0f;
    int k = k0;
    constexpr int U = 8;
    if (k + 4 * U <= k1) {
        float ac[U], bc[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            ac[u] = va ? pa[u * sa] : one;
            bc[u] = vb ? pb[u * sb] : 0.f;
        }
        for (; k + 8 * U <= k1; k += 4 * U) {
            float an[U], bn[U];
            const float* qa = pa + U * sa;
            const float* qb = pb + U * sb;
#pragma unroll
            for (int u = 0; u < U; ++u) {
                an[u] = va ? qa[u * sa] : one;
                bn[u] = vb ? qb[u * sb] : 0.f;
            }
#pragma unroll
            for (int u = 0; u < U; ++u) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(ac[u], bc[u], acc, 0, 0, 0);
#pragma unroll
            for (int u = 0; u < U; ++u) { ac[u] = an[u]; bc[u] = bn[u]; }
            if (!aone) pa = qa;
            pb = qb;
        }
#pragma unroll
        for (int u = 0; u < U; ++u) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(ac[u], bc[u], acc, 0, 0, 0);
        k += 4 * U;
        if (!aone) pa += U * sa;
        pb += U * sb;
    }
    for (; k < k1; k += 4) {
        const bool in = (k + lk) < k1;
        const float av = (in && va) ? *pa : ((in && aone) ? one : 0.f);
        const float bv = (in && vb) ? *pb : 0.f;
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bv, acc, 0, 0, 0);
        if (!aone) pa += sa;
        pb += sb;
    }
}

__global__ __launch_bounds__(256) void k_gemm_f32(GemmArgs a) {
    __shared__ floatx4 red[4][64];
    int pi = 0;
#pragma unroll
    for (int q = 1; q < kMaxGemm; ++q)
        if (q < a.nprob && (int)blockIdx.x >= a.tile_start[q]) pi = q;
    const gm_gemm& p = a.p[pi];
    const int TM = a.cfg[pi] & 15, TN = (a.cfg[pi] >> 4) & 15, KS = (a.cfg[pi] >> 8) & 15;
    const int wg = blockIdx.x - a.tile_start[pi];
    const int wm = wg / a.tiles_n[pi], wn = wg - wm * a.tiles_n[pi];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int tile = wave / KS, ks = wave - tile * KS;
    const int tm = tile / TN, tn = tile - tm * TN;
    const int m0 = (wm * TM + tm) * 16, n0 = (wn * TN + tn) * 16;
    const int li = lane & 15, lk = lane >> 4;
    const int K0 = p.K[0], Ktot = p.K[0] + p.K[1];
    // K range of this split (global k, multiple of 4 per split)
    const int k4 = (Ktot + 3) >> 2;
    const int per = (k4 + KS - 1) / KS;
    const int kb = min(Ktot, ks * per * 4), ke = min(Ktot, (ks + 1) * per * 4);
    const bool mrow = (m0 + li) < p.M, ncol = (n0 + li) < p.N;
    const int mm = mrow ? m0 + li : 0, nn = ncol ? n0 + li : 0;
    floatx4 acc = {0.f, 0.f, 0.f, 0.f};
    seg_mma(acc, p.A[0], p.B[0], mm, nn, mrow, ncol, lk, kb, min(ke, K0));
    if (p.K[1] > 0)
        seg_mma(acc, p.A[1], p.B[1], mm, nn, mrow, ncol, lk, max(kb, K0) - K0, ke - K0);
    if (KS > 1) {
        red[wave][lane] = acc;
        __syncthreads();
        if (ks != 0) return;
        for (int s = 1; s < KS; ++s) {
            const floatx4 o = red[wave + s][lane];
            acc[0] += o[0]; acc[1] += o[1]; acc[2] += o[2]; acc[3] += o[3];
        }
    }
    // C/D map of 16x16x4: col = lane&15, row = (lane>>4)*4 + r
    const int n = n0 + li;
    if (n >= p.N) return;
    const float bias = p.bias ? p.bias[n] : 0.f;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const int m = m0 + lk * 4 + r;
        if (m >= p.M) continue;
        float v = acc[r] + bias;
        if (p.act == 1) v = v > 0.f ? v : 0.f;
        else if (p.act == 2) v = 1.0f / (1.0f + expf(-v));
        if (p.mask) v = p.mask[(size_t)m * p.ld_mask + n] > 0.f ? v : 0.f;
        float* c = p.C + (size_t)m * p.ld_c + n;
        *c = p.accumulate ? *c + v : v;
    }
}

}  // namespace gm

using namespace gm;

extern "C" int gm_gemm_f32(const gm_gemm* in, int nprob, void* stream) {
    GM_REQUIRE(in && nprob >= 1 && nprob <= kMaxGemm, "gemm_f32: nprob must be 1..%d", kMaxGemm);
    GemmArgs a;
    memset(&a, 0, sizeof(a));
    a.nprob = nprob;
    int tiles = 0;
    for (int i = 0; i < nprob; ++i) {
        const gm_gemm& p = in[i];
        GM_REQUIRE(p.M >= 1 && p.N >= 1 && p.K[0] >= 0 && p.K[1] >= 0 && p.K[0] + p.K[1] >= 1,
                   "gemm_f32[%d]: bad shape M=%d N=%d K=%d+%d", i, p.M, p.N, p.K[0], p.K[1]);
        GM_REQUIRE(p.C && p.ld_c >= p.N, "gemm_f32[%d]: bad C / ld_c", i);
        GM_REQUIRE(p.act >= 0 && p.act <= 2, "gemm_f32[%d]: bad act %d", i, p.act);
        GM_REQUIRE(!p.mask || p.ld_mask >= p.N, "gemm_f32[%d]: bad ld_mask", i);
        for (int s = 0; s < 2; ++s)
            if (p.K[s] > 0)
                GM_REQUIRE(p.B[s].ptr, "gemm_f32[%d]: segment %d has no B operand", i, s);
        a.p[i] = p;
        const int Kt = p.K[0] + p.K[1];
        int KS = Kt >= 512 ? 4 : (Kt >= 128 ? 2 : 1);
        int TM, TN;
        const int rest = 4 / KS;
        if (rest == 1) { TM = TN = 1; }
        else if (rest == 2) { if (p.M >= p.N) { TM = 2; TN = 1; } else { TM = 1; TN = 2; } }
        else {
            if (p.M <= 16) { TM = 1; TN = 4; }
            else if (p.N <= 16) { TM = 4; TN = 1; }
            else { TM = 2; TN = 2; }
        }
        const int tm = (p.M + 16 * TM - 1) / (16 * TM), tn = (p.N + 16 * TN - 1) / (16 * TN);
        a.cfg[i] = TM | (TN << 4) | (KS << 8);
        a.tiles_n[i] = tn;
        a.tile_start[i] = tiles;
        tiles += tm * tn;
    }
    a.tile_start[nprob] = tiles;
    k_gemm_f32<<<tiles, 256, 0, as_stream(stream)>>>(a);
    return check_launch("k_gemm_f32");
}
