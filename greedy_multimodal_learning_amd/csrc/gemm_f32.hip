// Small fp32 GEMMs of the MMTM joint FC on MFMA (gfx950 v_mfma_f32_16x16x4_f32).
//
// The MMTM layers are [B, 2C] x [2C, C'] and [B, C'] x [C', C] with B <= 256 and
// C <= 512 (plus their weight/input gradients): a few MFLOP, L2-resident, so the
// kernel is latency/parallelism-bound, not HBM- or MFMA-bound.  Design:
//   * each wave computes one 16x16 output tile over a K range with the exact-f32
//     MFMA (an fmaf chain: same numerics as the fp32 reference's FMA GEMMs);
//   * a 1024-thread workgroup holds TM x TN tiles x KS K-splits (TM*TN*KS = 16 waves),
//     KS up to 16 so a wave's dependent chain is at most ~64 k (two rounds of loads in
//     flight) - the MMTM GEMMs are L2-latency chains, not MFMA work; split-K partial
//     tiles are summed through LDS in fixed order (deterministic);
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
    int cfg[kMaxGemm];      // TM | TN<<5 | KS<<10
    int nprob;
    int vec;  // 1: the float4 K-segment form where the operands allow it (A/B knob)
};

// One K-segment of a wave's 16x16 tile: k in [k0, k1) (segment-local), stepping 4.
// Lane (li, lk) reads A[m0+li][k+lk] and B[k+lk][n0+li]; pointers advance by
// 4*ld1 / 4*ld0 per step.  8 steps (32 k) per iteration with the next
// iteration's 16 loads issued before this iteration's 8 MFMAs (register
// double-buffer), so L2 latency hides behind MFMA issue.  Every load is
// unconditional from a clamped, in-range address and the validity select comes
// after it: a "load or constant" select on a per-lane condition makes hipcc branch
// around each load with a vmcnt(0) inside (cdna_hip_programming.md §5 trap 4c),
// i.e. one dependent L2 round trip per k-step.
template <int U>
__device__ __forceinline__ void seg_mma(floatx4& acc, const gm_operand& A, const gm_operand& B,
                                        int m, int n, bool mrow, bool ncol, int lk, int k0, int k1) {
    if (k1 <= k0) return;
    const bool aone = A.ptr == nullptr;
    // an all-ones A operand loads (and ignores) B's in-range elements
    const float* pa = aone ? B.ptr : A.ptr + (long)m * A.ld0 + (long)(k0 + lk) * A.ld1;
    const float* pb = B.ptr + (long)(k0 + lk) * B.ld0 + (long)n * B.ld1;
    const long sa = aone ? 0 : 4l * A.ld1, sb = 4l * B.ld0;
    const bool va = mrow && !aone, vb = ncol;
    const float one = mrow ? 1.0f : 0.0f;
    int k = k0;
    if (k + 4 * U <= k1) {
        float ac[U], bc[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            ac[u] = pa[u * sa];
            bc[u] = pb[u * sb];
        }
        for (; k + 8 * U <= k1; k += 4 * U) {
            float an[U], bn[U];
            const float* qa = pa + U * sa;
            const float* qb = pb + U * sb;
#pragma unroll
            for (int u = 0; u < U; ++u) {
                an[u] = qa[u * sa];
                bn[u] = qb[u * sb];
            }
#pragma unroll
            for (int u = 0; u < U; ++u)
                acc = __builtin_amdgcn_mfma_f32_16x16x4f32(va ? ac[u] : one, vb ? bc[u] : 0.f, acc, 0, 0, 0);
#pragma unroll
            for (int u = 0; u < U; ++u) { ac[u] = an[u]; bc[u] = bn[u]; }
            pa = qa;
            pb = qb;
        }
#pragma unroll
        for (int u = 0; u < U; ++u)
            acc = __builtin_amdgcn_mfma_f32_16x16x4f32(va ? ac[u] : one, vb ? bc[u] : 0.f, acc, 0, 0, 0);
        k += 4 * U;
        pa += U * sa;
        pb += U * sb;
    }
    // tail (< 4U k): lanes past k1 re-read the segment's last k and contribute zero
    for (; k < k1; k += 4) {
        const bool in = (k + lk) < k1;
        const long back = in ? 0 : (long)(k + lk - (k1 - 1));
        const float al = pa[-back * (aone ? 0 : A.ld1)];
        const float bl = pb[-back * B.ld0];
        const float av = in ? (va ? al : (aone ? one : 0.f)) : 0.f;
        const float bv = (in && vb) ? bl : 0.f;
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bv, acc, 0, 0, 0);
        pa += sa;
        pb += sb;
    }
}

// The same K-segment on 16-k groups with 16-byte loads along k where an operand is
// k-contiguous (A.ld1 == 1 / B.ld0 == 1, 16-B aligned rows): the four MFMAs of a group
// take k = kg + 4*lk + q in MFMA q (any k -> (lane, instruction) assignment is valid
// when A and B agree), so lane lk's float4 at kg + 4*lk feeds all four; a k-strided
// operand loads its four scalars at those same k.  A strided fp32 load touches one
// cache line per lane row for 4 B of it: the float4 form asks the TA for 4x fewer lines.
// UG groups (16*UG k) per load round, the next round in flight under this one's MFMAs.
template <bool VA, bool VB, int UG>
__device__ __forceinline__ void seg_mma_v(floatx4& acc, const gm_operand& A, const gm_operand& B, int m, int n,
                                          bool mrow, bool ncol, int lk, int k0, int k1) {
    const bool aone = A.ptr == nullptr;
    const bool va = mrow && !aone, vb = ncol;
    const float one = mrow ? 1.0f : 0.0f;
    const float* pa = aone ? B.ptr : A.ptr + (long)m * A.ld0;
    const float* pb = B.ptr + (long)n * B.ld1;
    const long sa = aone ? 0 : A.ld1, sb = B.ld0;
    auto load = [&](int kg, float (&a)[4], float (&b)[4]) {
        const int k = kg + 4 * lk;
        if constexpr (VA) {
            const float4 t = *reinterpret_cast<const float4*>(pa + k);
            a[0] = t.x; a[1] = t.y; a[2] = t.z; a[3] = t.w;
        } else {
#pragma unroll
            for (int q = 0; q < 4; ++q) a[q] = pa[(long)(k + q) * sa];
        }
        if constexpr (VB) {
            const float4 t = *reinterpret_cast<const float4*>(pb + k);
            b[0] = t.x; b[1] = t.y; b[2] = t.z; b[3] = t.w;
        } else {
#pragma unroll
            for (int q = 0; q < 4; ++q) b[q] = pb[(long)(k + q) * sb];
        }
    };
    auto mma = [&](const float (&a)[4], const float (&b)[4]) {
#pragma unroll
        for (int q = 0; q < 4; ++q)
            acc = __builtin_amdgcn_mfma_f32_16x16x4f32(va ? a[q] : one, vb ? b[q] : 0.f, acc, 0, 0, 0);
    };
    int kg = k0;
    if (kg + 16 * UG <= k1) {
        float ac[UG][4], bc[UG][4];
#pragma unroll
        for (int g = 0; g < UG; ++g) load(kg + 16 * g, ac[g], bc[g]);
        for (; kg + 32 * UG <= k1; kg += 16 * UG) {
            float an[UG][4], bn[UG][4];
#pragma unroll
            for (int g = 0; g < UG; ++g) load(kg + 16 * (UG + g), an[g], bn[g]);
#pragma unroll
            for (int g = 0; g < UG; ++g) mma(ac[g], bc[g]);
#pragma unroll
            for (int g = 0; g < UG; ++g)
#pragma unroll
                for (int q = 0; q < 4; ++q) { ac[g][q] = an[g][q]; bc[g][q] = bn[g][q]; }
        }
#pragma unroll
        for (int g = 0; g < UG; ++g) mma(ac[g], bc[g]);
        kg += 16 * UG;
    }
    for (; kg + 16 <= k1; kg += 16) {
        float a[4], b[4];
        load(kg, a, b);
        mma(a, b);
    }
    if (kg < k1) seg_mma<4>(acc, A, B, m, n, mrow, ncol, lk, kg, k1);  // < 16 k left
}

// one K-segment: the float4 form where the operands allow it (uniform per problem)
template <int U>
__device__ __forceinline__ void seg_any(int vec, floatx4& acc, const gm_operand& A, const gm_operand& B, int m,
                                        int n, bool mrow, bool ncol, int lk, int k0, int k1) {
    if (k1 <= k0) return;
    const bool va4 = A.ptr != nullptr && A.ld1 == 1 && (A.ld0 & 3) == 0 && ((uintptr_t)A.ptr & 15) == 0;
    const bool vb4 = B.ld0 == 1 && (B.ld1 & 3) == 0 && ((uintptr_t)B.ptr & 15) == 0;
    if (vec == 0 || (!va4 && !vb4)) seg_mma<U>(acc, A, B, m, n, mrow, ncol, lk, k0, k1);
    else if (va4 && vb4) seg_mma_v<true, true, U / 4>(acc, A, B, m, n, mrow, ncol, lk, k0, k1);
    else if (va4) seg_mma_v<true, false, U / 4>(acc, A, B, m, n, mrow, ncol, lk, k0, k1);
    else seg_mma_v<false, true, U / 4>(acc, A, B, m, n, mrow, ncol, lk, k0, k1);
}

// GEMM forms (gm_gemm_set_waves A/B knob): waves per workgroup x k-steps per load round
struct GemmForm { int nw, u; };
// forms 4 / 5: timing diagnostics of form 1 (outputs meaningless): arguments and one
// store only / everything but the operand loads and MFMAs
constexpr GemmForm kForms[] = {{4, 8}, {4, 16}, {8, 16}, {16, 8}};
static int g_gemm_form = 1, g_gemm_vec = 1, g_gemm_outer = 1;

// The MMTM GEMMs are dependent-latency chains (kernel arguments -> operand loads ->
// MFMAs -> epilogue loads -> store), not MFMA work: every round trip costs ~1-2 us.  So
// the problem index is the grid's y (no tile-table lookup before the argument loads),
// the epilogue's operands (bias, relu mask, accumulated C) are loaded together with the
// first operand round, and a wave's K range is at most two load rounds.
template <int NW, int U>
__global__ __launch_bounds__(NW * 64) void k_gemm_f32(GemmArgs a) {
    __shared__ floatx4 red[NW][64];
    const int pi = blockIdx.y;
    const gm_gemm& p = a.p[pi];
    const int cfg = a.cfg[pi];
    const int TM = cfg & 31, TN = (cfg >> 5) & 31, KS = (cfg >> 10) & 31;
    const int wg = blockIdx.x;
    if (wg >= a.tile_start[pi + 1] - a.tile_start[pi]) return;
    const int wm = wg / a.tiles_n[pi], wn = wg - wm * a.tiles_n[pi];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int tile = wave / KS, ks = wave - tile * KS;
    const int tm = tile / TN, tn = tile - tm * TN;
    const int m0 = (wm * TM + tm) * 16, n0 = (wn * TN + tn) * 16;
    const int li = lane & 15, lk = lane >> 4;
    const int K0 = p.K[0], Ktot = p.K[0] + p.K[1];
    // K range of this split (global k, a multiple of 16 per split)
    const int k16 = (Ktot + 15) >> 4;
    const int per = (k16 + KS - 1) / KS;
    const int kb = min(Ktot, ks * per * 16), ke = min(Ktot, (ks + 1) * per * 16);
    const bool mrow = (m0 + li) < p.M, ncol = (n0 + li) < p.N;
    const int mm = mrow ? m0 + li : 0, nn = ncol ? n0 + li : 0;
    // epilogue operands, in flight with the first operand round (clamped addresses)
    float bias = 0.f, mk[4] = {1.f, 1.f, 1.f, 1.f}, co[4] = {0.f, 0.f, 0.f, 0.f};
    if (ks == 0) {
        if (p.bias) bias = p.bias[nn];
        if (p.mask) {
#pragma unroll
            for (int r = 0; r < 4; ++r) mk[r] = p.mask[(size_t)min(m0 + lk * 4 + r, p.M - 1) * p.ld_mask + nn];
        }
        if (p.accumulate) {
#pragma unroll
            for (int r = 0; r < 4; ++r) co[r] = p.C[(size_t)min(m0 + lk * 4 + r, p.M - 1) * p.ld_c + nn];
        }
    }
    floatx4 acc = {0.f, 0.f, 0.f, 0.f};
    seg_any<U>(a.vec, acc, p.A[0], p.B[0], mm, nn, mrow, ncol, lk, kb, min(ke, K0));
    if (p.K[1] > 0)
        seg_any<U>(a.vec, acc, p.A[1], p.B[1], mm, nn, mrow, ncol, lk, max(kb, K0) - K0, ke - K0);
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
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const int m = m0 + lk * 4 + r;
        float v = acc[r] + bias;
        if (p.act == 1) v = relu_nan(v);
        else if (p.act == 2) v = 1.0f / (1.0f + expf(-v));
        v = mk[r] > 0.f ? v : 0.f;
        if (m < p.M) p.C[(size_t)m * p.ld_c + n] = co[r] + v;
    }
}

// ---------------------------------------------------------------------------------
// Outer-product shapes: K <= 128 with a large M x N output - the MMTM weight gradients at C5
// (fc_squeeze: dW[2048][24576] = dz^T[2048][32] . sq[32][24576], 201 MB of fp32 output written,
// and read back when accumulating).  k_gemm_f32 gives each wave one 16 x 16 tile and its
// epilogue stores 64-B row segments: 0.5 TB/s on that shape (407 us).  Here a 256-thread
// workgroup owns a 64 x 256 output tile; every thread keeps 8 rows x 8 columns (two float4
// column chunks 128 floats apart, so a wave's stores are whole 512-B row segments) in registers
// and runs an in-order fmaf chain over k, its operands loaded straight from global memory as
// float4s (A: the 8 rows of the thread's row group - the same address across the 32 lanes of
// the group; B: the thread's 8 columns), 4 k-steps in flight.  No LDS: the kernel runs beside
// the weight-gradient stream's one-workgroup-per-CU 156 KB ring kernels, which an LDS-staged
// form (40 KB per workgroup) kept off the CUs - C5 +0.5 ms/step in an A/B although its own
// launches were faster.  Bound: the output write (+ read when accumulating).
constexpr int kOM = 64, kON = 256, kOU = 4;

struct OuterArgs {
    gm_gemm p[kMaxGemm];
    int tiles_m[kMaxGemm];
    int tile_start[kMaxGemm + 1];
};

__global__ __launch_bounds__(256) void k_gemm_outer(OuterArgs a) {
    const int pi = blockIdx.y;
    const gm_gemm& p = a.p[pi];
    const int wg = blockIdx.x;
    if (wg >= a.tile_start[pi + 1] - a.tile_start[pi]) return;
    const int tm = wg % a.tiles_m[pi], tn = wg / a.tiles_m[pi];  // tm fastest: neighbours share B
    const int t = threadIdx.x, cg = t & 31, rg = t >> 5;
    const int m0 = tm * kOM + 8 * rg, n0 = tn * kON + 4 * cg;
    const int K = p.K[0];
    // A[m][k] = A.ptr[m + k * ld1] (ld0 == 1), B[k][n] = B.ptr[k * ld0 + n] (ld1 == 1); rows / columns
    // past M / N read a clamped in-range float4 and are never stored
    const float* pa = p.A[0].ptr + min(m0, p.M - 8);
    const long sa = p.A[0].ld1;
    const float* pb0 = p.B[0].ptr + min(n0, p.N - 4);
    const float* pb1 = p.B[0].ptr + min(n0 + 128, p.N - 4);
    const long sb = p.B[0].ld0;
    float acc[8][8];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[i][j] = 0.f;
    auto fma8 = [&](const float4& a0, const float4& a1, const float4& b0, const float4& b1) __attribute__((always_inline)) {
        const float av[8] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w};
        const float bv[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
#pragma unroll
        for (int i = 0; i < 8; ++i)
#pragma unroll
            for (int j = 0; j < 8; ++j) acc[i][j] = fmaf(av[i], bv[j], acc[i][j]);
    };
    int k = 0;
    for (; k + kOU <= K; k += kOU) {  // kOU k-steps' loads in flight, then their FMAs in k order
        float4 a0[kOU], a1[kOU], b0[kOU], b1[kOU];
#pragma unroll
        for (int u = 0; u < kOU; ++u) {
            const long ka = (long)(k + u) * sa, kb = (long)(k + u) * sb;
            a0[u] = *reinterpret_cast<const float4*>(pa + ka);
            a1[u] = *reinterpret_cast<const float4*>(pa + ka + 4);
            b0[u] = *reinterpret_cast<const float4*>(pb0 + kb);
            b1[u] = *reinterpret_cast<const float4*>(pb1 + kb);
        }
#pragma unroll
        for (int u = 0; u < kOU; ++u) fma8(a0[u], a1[u], b0[u], b1[u]);
    }
    for (; k < K; ++k) {
        const float4 a0 = *reinterpret_cast<const float4*>(pa + (long)k * sa);
        const float4 a1 = *reinterpret_cast<const float4*>(pa + (long)k * sa + 4);
        const float4 b0 = *reinterpret_cast<const float4*>(pb0 + (long)k * sb);
        const float4 b1 = *reinterpret_cast<const float4*>(pb1 + (long)k * sb);
        fma8(a0, a1, b0, b1);
    }
    // the clamped rows / columns: the thread's registers hold rows min(m0, M - 8) + i and columns
    // min(n0, N - 4) + j; store only the thread's own in-range outputs
    const int mb = min(m0, p.M - 8), nb0 = min(n0, p.N - 4), nb1 = min(n0 + 128, p.N - 4);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const int m = mb + i;
        if (m < m0 || m >= m0 + 8) continue;  // (a clamped row group: rows another group owns)
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int nb = h ? nb1 : nb0, n = n0 + 128 * h;
            if (n >= p.N) continue;
            float* c = p.C + (size_t)m * p.ld_c + nb;
            float4 v = make_float4(acc[i][4 * h], acc[i][4 * h + 1], acc[i][4 * h + 2], acc[i][4 * h + 3]);
            if (nb == n) {  // a whole float4 chunk of this thread
                if (p.accumulate) {
                    const float4 o = *reinterpret_cast<const float4*>(c);
                    v.x += o.x; v.y += o.y; v.z += o.z; v.w += o.w;
                }
                *reinterpret_cast<float4*>(c) = v;
            } else {  // the last, clamped chunk: columns nb + q >= n are this thread's
                const float vv[4] = {v.x, v.y, v.z, v.w};
                for (int q = n - nb; q < 4; ++q) c[q] = (p.accumulate ? c[q] : 0.f) + vv[q];
            }
        }
    }
}

// a problem the outer-product kernel takes: one K segment of at most 128, a large output, no
// bias / activation / mask, row-contiguous operands (A[m][k] = A[m + k ld1], B[k][n] = B[k ld0 + n]),
// M >= 8 and N >= 4, float4-aligned operand rows and C rows
static bool outer_ok(const gm_gemm& p) {
    const gm_operand& A = p.A[0];
    const gm_operand& B = p.B[0];
    return p.K[1] == 0 && p.K[0] >= 1 && p.K[0] <= 128 && (long long)p.M * p.N >= (1ll << 20) && p.M >= 8 &&
           p.N >= 4 && !p.bias && !p.mask && p.act == 0 && A.ptr && A.ld0 == 1 && (A.ld1 & 3) == 0 &&
           ((uintptr_t)A.ptr & 15) == 0 && B.ld1 == 1 && (B.ld0 & 3) == 0 && ((uintptr_t)B.ptr & 15) == 0 &&
           (p.ld_c & 3) == 0 && ((uintptr_t)p.C & 15) == 0;
}

}  // namespace gm

using namespace gm;

static int launch_gemm_f32(const gm_gemm* in, int nprob, hipStream_t st);

extern "C" int gm_gemm_f32(const gm_gemm* in, int nprob, void* stream) {
    GM_REQUIRE(in && nprob >= 1 && nprob <= kMaxGemm, "gemm_f32: nprob must be 1..%d", kMaxGemm);
    hipStream_t st = as_stream(stream);
    // the outer-product problems (k_gemm_outer) and the rest (k_gemm_f32): independent problems,
    // two launches on one stream
    gm_gemm rest[kMaxGemm];
    int nrest = 0;
    OuterArgs o;
    memset(&o, 0, sizeof(o));
    int nout = 0, maxt = 0;
    for (int i = 0; i < nprob; ++i) {
        const gm_gemm& p = in[i];
        if (g_gemm_outer && p.M >= 1 && p.N >= 1 && p.C && p.ld_c >= p.N && p.A[0].ptr && p.B[0].ptr && outer_ok(p)) {
            o.p[nout] = p;
            o.tiles_m[nout] = (p.M + kOM - 1) / kOM;
            const int t = o.tiles_m[nout] * ((p.N + kON - 1) / kON);
            o.tile_start[nout + 1] = o.tile_start[nout] + t;
            maxt = t > maxt ? t : maxt;
            ++nout;
        } else {
            rest[nrest++] = p;
        }
    }
    if (nrest) {
        const int rc = launch_gemm_f32(rest, nrest, st);
        if (rc) return rc;
    }
    if (nout) {
        k_gemm_outer<<<dim3(maxt, nout), 256, 0, st>>>(o);
        return check_launch("k_gemm_outer");
    }
    return GM_OK;
}

static int launch_gemm_f32(const gm_gemm* in, int nprob, hipStream_t st) {
    GemmArgs a;
    memset(&a, 0, sizeof(a));
    a.nprob = nprob;
    int tiles = 0, maxt = 0;
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
        // K splits: about two load rounds (8U k) per wave, at most the workgroup's waves
        const GemmForm f = kForms[g_gemm_form];
        const int NW = f.nw;
        int KS = 1;
        while (KS < NW && KS * 8 * f.u < Kt) KS *= 2;
        const int mt16 = (p.M + 15) / 16, nt16 = (p.N + 15) / 16;
        int TM = 1, TN = 1;
        while (TM * TN * KS < NW) {
            if (TN < nt16 && (TN <= TM || TM >= mt16)) TN *= 2;
            else if (TM < mt16) TM *= 2;
            else TN *= 2;
        }
        const int tm = (p.M + 16 * TM - 1) / (16 * TM), tn = (p.N + 16 * TN - 1) / (16 * TN);
        a.cfg[i] = TM | (TN << 5) | (KS << 10);
        a.tiles_n[i] = tn;
        a.tile_start[i] = tiles;
        tiles += tm * tn;
        if (tm * tn > maxt) maxt = tm * tn;
    }
    a.tile_start[nprob] = tiles;
    a.vec = g_gemm_vec;
    const dim3 grid(maxt, nprob);
    switch (g_gemm_form) {
        case 0: k_gemm_f32<4, 8><<<grid, 256, 0, st>>>(a); break;
        case 1: k_gemm_f32<4, 16><<<grid, 256, 0, st>>>(a); break;
        case 2: k_gemm_f32<8, 16><<<grid, 512, 0, st>>>(a); break;
        default: k_gemm_f32<16, 8><<<grid, 1024, 0, st>>>(a); break;
    }
    return check_launch("k_gemm_f32");
}

extern "C" int gm_gemm_set_form(int form) {
    g_gemm_vec = !(form & 256);    // bit 8: scalar k-steps only
    g_gemm_outer = !(form & 512);  // bit 9: no outer-product kernel (every problem on k_gemm_f32)
    form &= 255;
    GM_REQUIRE(form >= 0 && form < (int)(sizeof(kForms) / sizeof(kForms[0])), "gemm form must be 0..3 (got %d)",
               form);
    g_gemm_form = form;
    return GM_OK;
}
