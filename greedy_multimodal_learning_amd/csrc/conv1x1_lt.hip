// 1x1 / stride-1 / pad-0 convolutions in NHWC are plain GEMMs over the pixels (the ResNet-50
// bottleneck's reduce / expand convolutions: 70 launches of the C5 step, where the generic
// im2col kernel ran at 0.09 of the MFMA peak) - they go to hipBLASLt, the vendor GEMM library,
// instead of a conv kernel (no tap decode, no halo, library tiles for any M x N x K).
// Reference: torchvision Bottleneck conv1 / conv3 (resnet.py, the C5 workload's trunk,
// SURVEY §8 row f4), autocast bf16.
//
// Layouts (row-major, per view group g at the group strides): x [M][C], w [K][C] (KRSC with
// R = S = 1), wt [C][K] (the channel-transposed copy the input gradient takes), y / dy [M][K],
// dw [K][C] fp32.  In hipBLASLt's column-major terms (a row-major [r][c] matrix is a
// column-major c x r one):
//   fwd   Y^T  (K x M) = op_T(w: C x K) . (x: C x M)
//   dgrad dX^T (C x M) = op_T(wt: K x C) . (dy: K x M)       (+ addend as the C matrix)
//   wgrad dW^T (C x K) = (x: C x M) . op_T(dy: K x M)         (fp32 out, beta = accumulate)
// The view groups are the GEMM batch (strided).  Algorithms come from hipBLASLt's heuristic
// with no workspace (nothing allocated), cached per problem; a handle per stream, created on
// first use (eager warm-up steps run before any graph capture).  OFF by default: the C5
// training step faulted with it (an illegal address inside the step, r04) while every
// isolated shape, the C5 ones at 12 view groups included, matches fp32 PyTorch
// (test_conv1x1_gemm_vs_fp32); GM_CONV1X1_LT=1 / gm_conv_set_1x1_gemm(1) turn it on.
#include <hipblaslt/hipblaslt.h>

#include <cstdint>
#include <cstring>
#include <map>
#include <mutex>
#include <tuple>

#include "gm_common.h"

namespace gm {
namespace {

int g_conv_lt = [] {
    const char* e = getenv("GM_CONV1X1_LT");  // 1: the 1x1 shapes take hipBLASLt (default: im2col)
    return e ? atoi(e) : 0;
}();

// one handle per stream: the step runs weight gradients on a side stream beside the main
// chain, and a handle's internal state must not be shared by concurrent GEMMs
std::mutex g_lt_mu;
hipblasLtHandle_t lt_handle(hipStream_t st) {
    static std::map<hipStream_t, hipblasLtHandle_t> hs;
    std::lock_guard<std::mutex> g(g_lt_mu);
    auto it = hs.find(st);
    if (it != hs.end()) return it->second;
    hipblasLtHandle_t x = nullptr;
    if (hipblasLtCreate(&x) != HIPBLAS_STATUS_SUCCESS) x = nullptr;
    hs[st] = x;
    return x;
}

struct LtPlan {
    hipblasLtMatmulDesc_t op = nullptr;
    hipblasLtMatrixLayout_t la = nullptr, lb = nullptr, lc = nullptr, ld = nullptr;
    hipblasLtMatmulAlgo_t algo;
    bool ok = false, bad = false;  // bad: no workspace-free algorithm (the caller falls back)
};

// (transA, transB, m, n, k, lda, ldb, ldc, batch, sa, sb, sc, d_f32, c_is_d)
using LtKey = std::tuple<int, int, long long, long long, long long, long long, long long, long long, int, long long,
                         long long, long long, int>;

std::map<LtKey, LtPlan> g_lt_plans;

hipblasLtMatrixLayout_t layout(hipDataType t, long long rows, long long cols, long long ld, int batch, long long stride) {
    hipblasLtMatrixLayout_t l = nullptr;
    if (hipblasLtMatrixLayoutCreate(&l, t, (uint64_t)rows, (uint64_t)cols, ld) != HIPBLAS_STATUS_SUCCESS) return nullptr;
    if (batch > 1) {
        int32_t b = batch;
        int64_t s = stride;
        hipblasLtMatrixLayoutSetAttribute(l, HIPBLASLT_MATRIX_LAYOUT_BATCH_COUNT, &b, sizeof(b));
        hipblasLtMatrixLayoutSetAttribute(l, HIPBLASLT_MATRIX_LAYOUT_STRIDED_BATCH_OFFSET, &s, sizeof(s));
    }
    return l;
}

// D (m x n, column-major, ld ldc) = alpha op(A) op(B) + beta C, bf16 A / B, C and D bf16 or fp32
int lt_gemm(bool ta, bool tb, long long m, long long n, long long k, const void* A, long long lda, long long sa,
            const void* B, long long ldb, long long sb, const void* C, void* D, long long ldc, long long sc,
            bool d_f32, int batch, float beta, hipStream_t st, const char* fn) {
    hipblasLtHandle_t h = lt_handle(st);
    GM_REQUIRE(h != nullptr, "%s: hipblasLtCreate failed", fn);
    const LtKey key{ta, tb, m, n, k, lda, ldb, ldc, batch, sa, sb, sc, d_f32};
    LtPlan* pl;
    {
        std::lock_guard<std::mutex> g(g_lt_mu);
        pl = &g_lt_plans[key];
        if (pl->bad) return GM_E_UNSUP;
        if (!pl->ok) {
            const hipDataType dt = d_f32 ? HIP_R_32F : HIP_R_16BF;
            GM_REQUIRE(hipblasLtMatmulDescCreate(&pl->op, HIPBLAS_COMPUTE_32F, HIP_R_32F) == HIPBLAS_STATUS_SUCCESS,
                       "%s: hipblasLtMatmulDescCreate", fn);
            const int32_t opa = ta ? HIPBLAS_OP_T : HIPBLAS_OP_N, opb = tb ? HIPBLAS_OP_T : HIPBLAS_OP_N;
            hipblasLtMatmulDescSetAttribute(pl->op, HIPBLASLT_MATMUL_DESC_TRANSA, &opa, sizeof(opa));
            hipblasLtMatmulDescSetAttribute(pl->op, HIPBLASLT_MATMUL_DESC_TRANSB, &opb, sizeof(opb));
            pl->la = layout(HIP_R_16BF, ta ? k : m, ta ? m : k, lda, batch, sa);
            pl->lb = layout(HIP_R_16BF, tb ? n : k, tb ? k : n, ldb, batch, sb);
            pl->lc = layout(dt, m, n, ldc, batch, sc);
            pl->ld = layout(dt, m, n, ldc, batch, sc);
            GM_REQUIRE(pl->la && pl->lb && pl->lc && pl->ld, "%s: hipblasLtMatrixLayoutCreate", fn);
            hipblasLtMatmulPreference_t pref = nullptr;
            hipblasLtMatmulPreferenceCreate(&pref);
            uint64_t ws = 0;  // no workspace: the library allocates nothing
            hipblasLtMatmulPreferenceSetAttribute(pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES, &ws, sizeof(ws));
            // the first candidate that needs no workspace (the preference alone does not
            // guarantee it: a solution with a workspace requirement would write through a
            // null workspace)
            hipblasLtMatmulHeuristicResult_t res[16];
            int found = 0;
            const hipblasStatus_t s =
                hipblasLtMatmulAlgoGetHeuristic(h, pl->op, pl->la, pl->lb, pl->lc, pl->ld, pref, 16, res, &found);
            hipblasLtMatmulPreferenceDestroy(pref);
            int pick = -1;
            for (int i = 0; s == HIPBLAS_STATUS_SUCCESS && i < found && pick < 0; ++i)
                if (res[i].state == HIPBLAS_STATUS_SUCCESS && res[i].workspaceSize == 0) pick = i;
            if (pick < 0) {  // none: this problem takes the im2col kernel
                pl->bad = true;
                return GM_E_UNSUP;
            }
            pl->algo = res[pick].algo;
            pl->ok = true;
        }
    }
    const float alpha = 1.f;
    const hipblasStatus_t s = hipblasLtMatmul(h, pl->op, &alpha, A, pl->la, B, pl->lb, &beta, C ? C : D, pl->lc, D,
                                              pl->ld, &pl->algo, nullptr, 0, st);
    GM_REQUIRE(s == HIPBLAS_STATUS_SUCCESS, "%s: hipblasLtMatmul failed (%d)", fn, (int)s);
    return check_launch(fn);
}

}  // namespace

// 1x1 / stride 1 / pad 0 (both axes), channels the GEMM can take
bool conv1x1_lt_ok(int R, int S, int sh, int sw, int ph, int pw, long long M) {
    return g_conv_lt && R == 1 && S == 1 && sh == 1 && sw == 1 && ph == 0 && pw == 0 && M >= 1;
}

int conv1x1_lt_fwd(long long M, int C, int K, int G, const void* x, long long gs_x, const void* w, long long gs_w,
                   void* y, long long gs_y, hipStream_t st) {
    return lt_gemm(true, false, K, M, C, w, C, gs_w, x, C, gs_x, nullptr, y, K, gs_y, false, G, 0.f, st,
                   "conv1x1 fwd (hipBLASLt)");
}

int conv1x1_lt_dgrad(long long M, int C, int K, int G, const void* dy, long long gs_dy, const void* wt, long long gs_wt,
                     void* dx, long long gs_dx, const void* addend, hipStream_t st) {
    return lt_gemm(true, false, C, M, K, wt, K, gs_wt, dy, K, gs_dy, addend, dx, C, gs_dx, false, G,
                   addend ? 1.f : 0.f, st, "conv1x1 dgrad (hipBLASLt)");
}

int conv1x1_lt_wgrad(long long M, int C, int K, int G, const void* dy, long long gs_dy, const void* x, long long gs_x,
                     float* dw, long long gs_dw, int accumulate, hipStream_t st) {
    return lt_gemm(false, true, C, K, M, x, C, gs_x, dy, K, gs_dy, nullptr, dw, C, gs_dw, true, G,
                   accumulate ? 1.f : 0.f, st, "conv1x1 wgrad (hipBLASLt)");
}

}  // namespace gm

extern "C" int gm_conv_set_1x1_gemm(int on) {
    gm::g_conv_lt = on ? 1 : 0;
    return GM_OK;
}
