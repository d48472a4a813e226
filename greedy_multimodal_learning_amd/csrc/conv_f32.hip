// Reference-precision (fp32) ResNet trunk convolutions on the exact-f32 MFMA
// (gfx950 v_mfma_f32_32x32x2_f32: every product rounded once, fp32 accumulate - the
// numerics of the reference's fp32 Conv2d, src/model.py:65-106 via torchvision).
//
// One implicit-GEMM kernel serves the three passes; NHWC activations, KRSC weights:
//   fwd   : y [pix=(n,p,q)][k]   = sum_{(r,s,c)} x[n, p*st-pad+r, q*st-pad+s, c] * w[k][r][s][c]
//   dgrad : dx[pix=(n,h,w)][c]   = sum_{(r,s,k)} dy[n, (h+pad-r)/st, (w+pad-s)/st, k] * w[k][r][s][c]
//                                  (taps whose offset is not a multiple of the stride add nothing)
//   wgrad : dw[k][(r,s,c)]       = sum_{pix=(n,p,q)} dy[pix][k] * x[n, p*st-pad+r, q*st-pad+s, c]
// GEMM C[M][N] = sum_kk A(m,kk) B(kk,n).  Workgroup tile (64*TM) x (64*TN), BK = 16,
// 4 waves in 2x2, each wave (32*TM) x (32*TN) of 32x32 MFMA tiles.  Operands are
// gathered (im2col on the fly) with 16-byte loads whenever the channel counts are
// multiples of 4 (every ResNet layer but the RGB stem, which takes the element path),
// staged through LDS (double buffer, register prefetch of the next k-tile, rows padded
// to 32 mod 64 dwords so the MFMA fragment reads are conflict-free).  Long reductions
// (wgrad over all pixels, small-M layers) are split over workgroups into fp32 slabs
// summed in a fixed order by a second kernel: deterministic, no float atomics.
#include <cstring>

#include "gm_common.h"

namespace gm {
namespace {

constexpr int kBK = 16;
constexpr int kPad = 32;  // row stride = 64*T + 32 == 32 (mod 64) dwords
typedef float floatx16 __attribute__((ext_vector_type(16)));

enum { FWD = 0, DGRAD = 1, WGRAD = 2 };

struct F32Args {
    int M, N, Kr;                  // GEMM shape (Kr = reduction length)
    int Nb, H, W, C, K, R, S, st, pad, P, Q;
    const float* x;
    const float* w;
    const float* dy;
    float* out;
    const float* addend;           // dgrad: added to the result (gradient join), may be null
    int accumulate;                // out += result
    int ktiles, kt_per_split;      // k-tiles in total / per split (blockIdx.z)
    float* part;                   // splits > 1: [splits][M][N] fp32 slabs
    FastDiv fd_C, fd_S, fd_K, fd_Q, fd_P, fd_W, fd_H, fd_st;
};

// ---- operand element access --------------------------------------------------
// Row decode of an output / input pixel index.
struct Pix {
    int n, a, b;  // (n, p, q) or (n, h, w)
};
__device__ __forceinline__ Pix dec_pix(unsigned m, const FastDiv& fq, const FastDiv& fp, int Q, int P) {
    const unsigned t = fq.div(m);
    const unsigned n = fp.div(t);
    return Pix{(int)n, (int)(t - n * P), (int)(m - t * Q)};
}

// x[n, h, w, c..c+V) with zero outside the image
template <int V>
__device__ __forceinline__ void ld_x(const F32Args& a, int n, int h, int w, int c, float* o) {
    if ((unsigned)h < (unsigned)a.H && (unsigned)w < (unsigned)a.W) {
        const float* p = a.x + (((long long)n * a.H + h) * a.W + w) * a.C + c;
        if (V == 4) {
            const float4 v = *reinterpret_cast<const float4*>(p);
            o[0] = v.x; o[1] = v.y; o[2] = v.z; o[3] = v.w;
        } else {
            o[0] = *p;
        }
    } else {
#pragma unroll
        for (int j = 0; j < V; ++j) o[j] = 0.f;
    }
}

// A(m, kk..kk+V) for FWD (x gather) and DGRAD (dy gather); pixel row pre-decoded.
template <int MODE, int V>
__device__ __forceinline__ void ld_a(const F32Args& a, const Pix& px, bool mok, int kk, float* o) {
    if (!mok || kk >= a.Kr) {
#pragma unroll
        for (int j = 0; j < V; ++j) o[j] = 0.f;
        return;
    }
    if (MODE == FWD) {
        const unsigned rs = a.fd_C.div((unsigned)kk);
        const int c = kk - (int)rs * a.C;
        const unsigned r = a.fd_S.div(rs);
        const int s = (int)(rs - r * a.S);
        ld_x<V>(a, px.n, px.a * a.st - a.pad + (int)r, px.b * a.st - a.pad + s, c, o);
    } else {  // DGRAD: kk = (r, s, k), k fastest
        const unsigned rs = a.fd_K.div((unsigned)kk);
        const int k = kk - (int)rs * a.K;
        const unsigned r = a.fd_S.div(rs);
        const int s = (int)(rs - r * a.S);
        const int hp = px.a + a.pad - (int)r, wp = px.b + a.pad - s;
        const unsigned p = a.fd_st.div((unsigned)(hp < 0 ? 0 : hp)), q = a.fd_st.div((unsigned)(wp < 0 ? 0 : wp));
        const bool ok = hp >= 0 && wp >= 0 && (int)p * a.st == hp && (int)q * a.st == wp && (int)p < a.P &&
                        (int)q < a.Q;
        if (ok) {
            const float* src = a.dy + (((long long)px.n * a.P + p) * a.Q + q) * a.K + k;
            if (V == 4) {
                const float4 v = *reinterpret_cast<const float4*>(src);
                o[0] = v.x; o[1] = v.y; o[2] = v.z; o[3] = v.w;
            } else {
                o[0] = *src;
            }
        } else {
#pragma unroll
            for (int j = 0; j < V; ++j) o[j] = 0.f;
        }
    }
}

// ---- the kernel ------------------------------------------------------------------
// VEC: 16-byte operand loads (C % 4 == 0 and K % 4 == 0), else element loads.
template <int MODE, bool VEC, int TM, int TN>
__global__ __launch_bounds__(256) void k_conv_f32(F32Args a) {
    constexpr int BM = 64 * TM, BN = 64 * TN;
    constexpr int LA = BM + kPad, LB = BN + kPad;
    __shared__ float As[2][kBK][LA];
    __shared__ float Bs[2][kBK][LB];
    const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
    const int wm = wave & 1, wn = wave >> 1;
    const int m0 = blockIdx.x * BM, n0 = blockIdx.y * BN;
    const int kt0 = blockIdx.z * a.kt_per_split;
    int kt1 = kt0 + a.kt_per_split;
    if (kt1 > a.ktiles) kt1 = a.ktiles;

    // A-operand chunks of this thread: FWD/DGRAD rows are pixels, loaded along kk
    // (VEC: chunk c -> row c>>2, 4 kk at 4*(c&3); element: e -> row e>>4, kk e&15);
    // WGRAD rows are output channels, loaded along m (chunk c -> kk c / (BM/4), m 4*(c % (BM/4))).
    constexpr int NA = VEC ? TM : 4 * TM;   // VEC: BM*4/256 chunks; element: BM*16/256 elements
    constexpr int NB = VEC ? TN : 4 * TN;
    Pix apx[(MODE != WGRAD) ? NA : 1];
    bool aok[(MODE != WGRAD) ? NA : 1];
    if (MODE != WGRAD) {
#pragma unroll
        for (int i = 0; i < NA; ++i) {
            const int e = t + i * 256;
            const int mi = VEC ? (e >> 2) : (e >> 4);
            const int m = m0 + mi;
            aok[i] = m < a.M;
            apx[i] = MODE == FWD ? dec_pix(aok[i] ? m : 0, a.fd_Q, a.fd_P, a.Q, a.P)
                                 : dec_pix(aok[i] ? m : 0, a.fd_W, a.fd_H, a.W, a.H);
        }
    }
    // B-operand column decode for WGRAD (cols are (r, s, c)), fixed per thread
    int bh[(MODE == WGRAD) ? NB : 1], bw[(MODE == WGRAD) ? NB : 1], bc[(MODE == WGRAD) ? NB : 1];
    bool bok[(MODE == WGRAD) ? NB : 1];
    if (MODE == WGRAD) {
#pragma unroll
        for (int i = 0; i < NB; ++i) {
            const int e = t + i * 256;
            const int n = n0 + (VEC ? 4 * (e % (BN / 4)) : (e % BN));
            bok[i] = n < a.N;
            const unsigned rs = a.fd_C.div((unsigned)(bok[i] ? n : 0));
            bc[i] = (bok[i] ? n : 0) - (int)rs * a.C;
            const unsigned r = a.fd_S.div(rs);
            bh[i] = (int)r - a.pad;
            bw[i] = (int)(rs - r * a.S) - a.pad;
        }
    }

    float ra[NA][VEC ? 4 : 1], rb[NB][VEC ? 4 : 1];
    auto load = [&](int kt) {
        const int kb = kt * kBK;
#pragma unroll
        for (int i = 0; i < NA; ++i) {
            const int e = t + i * 256;
            if (MODE != WGRAD) {
                const int kk = kb + (VEC ? 4 * (e & 3) : (e & 15));
                ld_a<MODE, VEC ? 4 : 1>(a, apx[i], aok[i], kk, ra[i]);
            } else {  // A(m = k, kk = pix) = dy[pix][k]
                const int kk = kb + (VEC ? e / (BM / 4) : e / BM);
                const int m = m0 + (VEC ? 4 * (e % (BM / 4)) : e % BM);
                const bool ok = kk < a.Kr && m < a.M;
                const float* p = a.dy + (long long)(ok ? kk : 0) * a.K + (ok ? m : 0);
                if (VEC) {
                    const float4 v = ok ? *reinterpret_cast<const float4*>(p) : make_float4(0.f, 0.f, 0.f, 0.f);
                    ra[i][0] = v.x; ra[i][1] = v.y; ra[i][2] = v.z; ra[i][3] = v.w;
                } else {
                    ra[i][0] = ok ? *p : 0.f;
                }
            }
        }
#pragma unroll
        for (int i = 0; i < NB; ++i) {
            const int e = t + i * 256;
            if (MODE == FWD) {  // B(kk, n) = w[n][kk]: along kk
                const int n = n0 + (VEC ? (e >> 2) : (e >> 4));
                const int kk = kb + (VEC ? 4 * (e & 3) : (e & 15));
                const bool ok = n < a.N && kk < a.Kr;
                const float* p = a.w + (long long)(ok ? n : 0) * a.Kr + (ok ? kk : 0);
                if (VEC) {
                    const float4 v = ok ? *reinterpret_cast<const float4*>(p) : make_float4(0.f, 0.f, 0.f, 0.f);
                    rb[i][0] = v.x; rb[i][1] = v.y; rb[i][2] = v.z; rb[i][3] = v.w;
                } else {
                    rb[i][0] = ok ? *p : 0.f;
                }
            } else if (MODE == DGRAD) {  // B(kk = (r,s,k), n = c) = w[k][r][s][c]: along n
                const int kk = kb + (VEC ? e / (BN / 4) : e / BN);
                const int n = n0 + (VEC ? 4 * (e % (BN / 4)) : e % BN);
                const bool ok = n < a.N && kk < a.Kr;
                const unsigned rs = a.fd_K.div((unsigned)(ok ? kk : 0));
                const int k = (ok ? kk : 0) - (int)rs * a.K;
                const float* p = a.w + ((long long)k * a.R * a.S + rs) * a.C + (ok ? n : 0);
                if (VEC) {
                    const float4 v = ok ? *reinterpret_cast<const float4*>(p) : make_float4(0.f, 0.f, 0.f, 0.f);
                    rb[i][0] = v.x; rb[i][1] = v.y; rb[i][2] = v.z; rb[i][3] = v.w;
                } else {
                    rb[i][0] = ok ? *p : 0.f;
                }
            } else {  // WGRAD: B(kk = pix, n = (r,s,c)) = x patch: along n
                const int kk = kb + (VEC ? e / (BN / 4) : e / BN);
                if (kk < a.Kr && bok[i]) {
                    const Pix px = dec_pix((unsigned)kk, a.fd_Q, a.fd_P, a.Q, a.P);
                    ld_x<VEC ? 4 : 1>(a, px.n, px.a * a.st + bh[i], px.b * a.st + bw[i], bc[i], rb[i]);
                } else {
#pragma unroll
                    for (int j = 0; j < (VEC ? 4 : 1); ++j) rb[i][j] = 0.f;
                }
            }
        }
    };
    auto store = [&](int buf) {
#pragma unroll
        for (int i = 0; i < NA; ++i) {
            const int e = t + i * 256;
            if (MODE != WGRAD) {
                if (VEC) {
                    const int mi = e >> 2, kq = 4 * (e & 3);
#pragma unroll
                    for (int j = 0; j < 4; ++j) As[buf][kq + j][mi] = ra[i][j];
                } else {
                    As[buf][e & 15][e >> 4] = ra[i][0];
                }
            } else {
                if (VEC) {
                    const int kk = e / (BM / 4), mi = 4 * (e % (BM / 4));
                    *reinterpret_cast<float4*>(&As[buf][kk][mi]) = make_float4(ra[i][0], ra[i][1], ra[i][2], ra[i][3]);
                } else {
                    As[buf][e / BM][e % BM] = ra[i][0];
                }
            }
        }
#pragma unroll
        for (int i = 0; i < NB; ++i) {
            const int e = t + i * 256;
            if (MODE == FWD) {
                if (VEC) {
                    const int ni = e >> 2, kq = 4 * (e & 3);
#pragma unroll
                    for (int j = 0; j < 4; ++j) Bs[buf][kq + j][ni] = rb[i][j];
                } else {
                    Bs[buf][e & 15][e >> 4] = rb[i][0];
                }
            } else {
                if (VEC) {
                    const int kk = e / (BN / 4), ni = 4 * (e % (BN / 4));
                    *reinterpret_cast<float4*>(&Bs[buf][kk][ni]) = make_float4(rb[i][0], rb[i][1], rb[i][2], rb[i][3]);
                } else {
                    Bs[buf][e / BN][e % BN] = rb[i][0];
                }
            }
        }
    };

    floatx16 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

    const int li = lane & 31, lk = lane >> 5;
    if (kt0 < kt1) {
        load(kt0);
        store(0);
        __syncthreads();
        for (int kt = kt0; kt < kt1; ++kt) {
            const int buf = (kt - kt0) & 1;
            if (kt + 1 < kt1) load(kt + 1);
#pragma unroll
            for (int k2 = 0; k2 < kBK; k2 += 2) {
                float fa[TM], fb[TN];
#pragma unroll
                for (int i = 0; i < TM; ++i) fa[i] = As[buf][k2 + lk][wm * 32 * TM + i * 32 + li];
#pragma unroll
                for (int j = 0; j < TN; ++j) fb[j] = Bs[buf][k2 + lk][wn * 32 * TN + j * 32 + li];
#pragma unroll
                for (int i = 0; i < TM; ++i)
#pragma unroll
                    for (int j = 0; j < TN; ++j)
                        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[i], fb[j], acc[i][j], 0, 0, 0);
            }
            if (kt + 1 < kt1) store(buf ^ 1);
            __syncthreads();
        }
    }

    // C/D map of 32x32: col = lane & 31, row = (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5)
    const bool split = gridDim.z > 1;
    float* dst = split ? a.part + (size_t)blockIdx.z * a.M * a.N : a.out;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) {
            const int n = n0 + wn * 32 * TN + j * 32 + li;
            if (n >= a.N) continue;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int m = m0 + wm * 32 * TM + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * lk;
                if (m >= a.M) continue;
                const size_t o = (size_t)m * a.N + n;
                float v = acc[i][j][r];
                if (!split) {
                    if (a.addend) v += a.addend[o];
                    if (a.accumulate) v += dst[o];
                }
                dst[o] = v;
            }
        }
}

// splits > 1: out[i] = sum_s part[s][i] (+ addend) (+ out), fixed order
__global__ __launch_bounds__(256) void k_conv_f32_splitk_sum(const float* __restrict__ part, int splits, long long n,
                                                            const float* __restrict__ addend, int accumulate,
                                                            float* __restrict__ out) {
    for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long long)gridDim.x * 256) {
        float v = 0.f;
        for (int s = 0; s < splits; ++s) v += part[(size_t)s * n + i];
        if (addend) v += addend[i];
        if (accumulate) v += out[i];
        out[i] = v;
    }
}

struct Plan {
    F32Args a;
    int TM, TN, splits;
    bool vec;
    dim3 grid;
    size_t scratch;
};

int cus() {
    static const int n = [] {
        int dev = 0, c = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
            return 256;
        return c;
    }();
    return n;
}

int make_plan(const gm_conv_f32* p, Plan& pl, const char* fn) {
    if (!p) {
        set_error("%s: null descriptor", fn);
        return GM_E_ARG;
    }
    const gm_conv_desc& d = p->d;
    if (p->mode < 0 || p->mode > 2 || d.N < 1 || d.H < 1 || d.W < 1 || d.C < 1 || d.K < 1 || d.R < 1 || d.S < 1 ||
        d.stride < 1 || d.pad < 0) {
        set_error("%s: bad descriptor (mode=%d N=%d H=%d W=%d C=%d K=%d R=%d S=%d stride=%d pad=%d)", fn, p->mode, d.N,
                  d.H, d.W, d.C, d.K, d.R, d.S, d.stride, d.pad);
        return GM_E_ARG;
    }
    const int P = (d.H + 2 * d.pad - d.R) / d.stride + 1, Q = (d.W + 2 * d.pad - d.S) / d.stride + 1;
    if (P < 1 || Q < 1) {
        set_error("%s: empty output", fn);
        return GM_E_ARG;
    }
    F32Args& a = pl.a;
    memset(&a, 0, sizeof(a));
    a.Nb = d.N; a.H = d.H; a.W = d.W; a.C = d.C; a.K = d.K; a.R = d.R; a.S = d.S;
    a.st = d.stride; a.pad = d.pad; a.P = P; a.Q = Q;
    const long long npix = (long long)d.N * P * Q, nin = (long long)d.N * d.H * d.W;
    const long long rsc = (long long)d.R * d.S * d.C, rsk = (long long)d.R * d.S * d.K;
    long long M, N, Kr;
    if (p->mode == FWD) { M = npix; N = d.K; Kr = rsc; }
    else if (p->mode == DGRAD) { M = nin; N = d.C; Kr = rsk; }
    else { M = d.K; N = rsc; Kr = npix; }
    if (M >= (1ll << 31) || N >= (1ll << 31) || Kr >= (1ll << 31) || M * N >= (1ll << 40) ||
        npix * d.K >= (1ll << 40) || nin * d.C >= (1ll << 40)) {
        set_error("%s: problem too large", fn);
        return GM_E_ARG;
    }
    a.M = (int)M; a.N = (int)N; a.Kr = (int)Kr;
    a.fd_C = FastDiv((uint32_t)d.C); a.fd_S = FastDiv((uint32_t)d.S); a.fd_K = FastDiv((uint32_t)d.K);
    a.fd_Q = FastDiv((uint32_t)Q); a.fd_P = FastDiv((uint32_t)P); a.fd_W = FastDiv((uint32_t)d.W);
    a.fd_H = FastDiv((uint32_t)d.H); a.fd_st = FastDiv((uint32_t)d.stride);
    pl.vec = (d.C % 4 == 0) && (d.K % 4 == 0);
    const long long big = (M + 127) / 128 * ((N + 127) / 128);
    pl.TM = pl.TN = (big >= cus()) ? 2 : 1;
    const int BM = 64 * pl.TM, BN = 64 * pl.TN;
    const long long tiles = (M + BM - 1) / BM * ((N + BN - 1) / BN);
    a.ktiles = (int)((Kr + kBK - 1) / kBK);
    // split the reduction when the tiles alone leave the chip idle; >= 8 k-tiles per split
    int splits = 1;
    const long long target = 2ll * cus();
    if (tiles < target && a.ktiles >= 16) {
        long long s = (target + tiles - 1) / tiles;
        long long maxs = a.ktiles / 8;
        if (s > maxs) s = maxs;
        if (s > 64) s = 64;
        splits = (int)(s < 1 ? 1 : s);
    }
    a.kt_per_split = (a.ktiles + splits - 1) / splits;
    splits = (a.ktiles + a.kt_per_split - 1) / a.kt_per_split;
    pl.splits = splits;
    pl.grid = dim3((unsigned)((M + BM - 1) / BM), (unsigned)((N + BN - 1) / BN), (unsigned)splits);
    pl.scratch = splits > 1 ? (size_t)splits * M * N * sizeof(float) : 0;
    return GM_OK;
}

template <int MODE>
void launch(const Plan& pl, hipStream_t st) {
#define GM_F32_L(V, TM, TN) hipLaunchKernelGGL((k_conv_f32<MODE, V, TM, TN>), pl.grid, dim3(256), 0, st, pl.a)
    if (pl.vec) {
        if (pl.TM == 2) GM_F32_L(true, 2, 2); else GM_F32_L(true, 1, 1);
    } else {
        if (pl.TM == 2) GM_F32_L(false, 2, 2); else GM_F32_L(false, 1, 1);
    }
#undef GM_F32_L
}

}  // namespace
}  // namespace gm

using namespace gm;

extern "C" size_t gm_conv2d_f32_scratch(const gm_conv_f32* p) {
    Plan pl;
    if (make_plan(p, pl, "gm_conv2d_f32_scratch")) return 0;
    return pl.scratch;
}

extern "C" int gm_conv2d_f32(const gm_conv_f32* p, void* scratch, size_t scratch_bytes, void* stream) {
    Plan pl;
    int rc = make_plan(p, pl, "gm_conv2d_f32");
    if (rc) return rc;
    GM_REQUIRE(p->out, "gm_conv2d_f32: null output");
    GM_REQUIRE(p->mode == WGRAD ? (p->x && p->dy) : p->mode == FWD ? (p->x && p->w) : (p->dy && p->w),
               "gm_conv2d_f32: null operand for mode %d", p->mode);
    GM_REQUIRE(!p->addend || p->mode == DGRAD, "gm_conv2d_f32: addend is a dgrad option");
    if (pl.scratch) {
        if (!scratch || scratch_bytes < pl.scratch) {
            set_error("gm_conv2d_f32: scratch %zu bytes < required %zu", scratch_bytes, pl.scratch);
            return GM_E_SCRATCH;
        }
    }
    pl.a.x = p->x; pl.a.w = p->w; pl.a.dy = p->dy; pl.a.out = p->out; pl.a.addend = p->addend;
    pl.a.accumulate = p->accumulate;
    pl.a.part = static_cast<float*>(scratch);
    hipStream_t st = as_stream(stream);
    if (p->mode == FWD) launch<FWD>(pl, st);
    else if (p->mode == DGRAD) launch<DGRAD>(pl, st);
    else launch<WGRAD>(pl, st);
    if ((rc = check_launch("k_conv_f32"))) return rc;
    if (pl.splits > 1) {
        const long long n = (long long)pl.a.M * pl.a.N;
        long long g = (n + 1023) / 1024;
        if (g > 8192) g = 8192;
        hipLaunchKernelGGL(k_conv_f32_splitk_sum, dim3((unsigned)(g < 1 ? 1 : g)), dim3(256), 0, st, pl.a.part,
                           pl.splits, n, p->addend, p->accumulate, p->out);
        return check_launch("k_conv_f32_splitk_sum");
    }
    return GM_OK;
}
