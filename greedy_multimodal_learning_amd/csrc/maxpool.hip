// MaxPool2d of the ResNet stem (torchvision: kernel 3, stride 2, padding 1;
// reference src/model.py:65-106 via torchvision.models.resnet18), NHWC bf16.
//
// Forward writes y and a 1-byte window-relative argmax per output element
// (PyTorch stores an int64 flat index: 8x the bytes).  Tie/NaN rule follows
// PyTorch's max_pool2d kernels: scan the window row-major and take a value when
// `v > max || isnan(v)`, starting from -inf at the first in-bounds position.
// Backward is a gather: each input pixel visits the <= ceil(k/s)^2 windows that
// cover it and sums the dy of those whose argmax is that pixel (fp32, fixed
// order), so no atomics and dx is written exactly once.  Element type E: bf16 (the
// performance trunk) or fp32 (the reference-precision trunk), 8 channels per access.
#include <type_traits>

#include "gm_common.h"

namespace gm {
namespace {

template <typename E>
__device__ __forceinline__ float round_to(float v) {
    if constexpr (std::is_same<E, uint16_t>::value) return __uint_as_float((uint32_t)Elem<uint16_t>::f2bf(v) << 16);
    else return v;
}

struct PoolArgs {
    int N, H, W, C8;  // C8 = C / 8 (16-byte channel groups)
    int P, Q, k, s, pad;
    FastDiv fd_c8, fd_q, fd_p, fd_w, fd_h, fd_s;  // index decode without integer division
    FastDiv fd_ng;  // images per view group (BNRELU: group g = n / Ng reads coef + g*2C)
};

// BNRELU: the pooled values are relu(x*sc + sh) rounded to E, i.e. the stem's BatchNorm +
// ReLU applied on the fly (coef = sc[C], sh[C]): the normalised activation is never
// written, bit-identical to BN-apply (fmaf, fmaxf, RNE store) followed by the plain pool.
// xsel (optional): the raw input value each output selected (its argmax's x), so the BN
// backward's channel sums need only the pooled tensors (k_stem_pool_bn_bwd pass 1)
template <typename E, bool BNRELU = false>
__global__ __launch_bounds__(256) void k_maxpool_fwd(PoolArgs a, const void* __restrict__ x, void* __restrict__ y,
                                                     uint2* __restrict__ idx, const float* __restrict__ coef = nullptr,
                                                     void* __restrict__ xsel = nullptr) {
    const unsigned total = (unsigned)a.N * a.P * a.Q * a.C8;  // < 2^31 (checked on the host)
    for (unsigned i = blockIdx.x * 256 + threadIdx.x; i < total; i += gridDim.x * 256) {
        unsigned t = a.fd_c8.div(i);
        const int cg = (int)(i - t * a.C8);
        unsigned t2 = a.fd_q.div(t);
        const int q = (int)(t - t2 * a.Q);
        const unsigned n_ = a.fd_p.div(t2);
        const int p = (int)(t2 - n_ * a.P);
        const int n = (int)n_;
        const int h0 = p * a.s - a.pad, w0 = q * a.s - a.pad;
        float m[8], xs[8];
        uint32_t ix[8];
        float sc[8], sh[8];
        if (BNRELU) {
            const float* cf = coef + (size_t)a.fd_ng.div((unsigned)n) * (a.C8 * 16);
            const float4* c4 = reinterpret_cast<const float4*>(cf + cg * 8);
            const float4* s4 = reinterpret_cast<const float4*>(cf + a.C8 * 8 + cg * 8);
            const float4 c0 = c4[0], c1 = c4[1], s0 = s4[0], s1 = s4[1];
            sc[0] = c0.x; sc[1] = c0.y; sc[2] = c0.z; sc[3] = c0.w; sc[4] = c1.x; sc[5] = c1.y; sc[6] = c1.z; sc[7] = c1.w;
            sh[0] = s0.x; sh[1] = s0.y; sh[2] = s0.z; sh[3] = s0.w; sh[4] = s1.x; sh[5] = s1.y; sh[6] = s1.z; sh[7] = s1.w;
        }
        const int hs = h0 < 0 ? 0 : h0, ws = w0 < 0 ? 0 : w0;
        const uint32_t first = (uint32_t)((hs - h0) * a.k + (ws - w0));
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            m[j] = -__builtin_huge_valf();
            xs[j] = 0.f;
            ix[j] = first;
        }
        if (a.k == 3) {
            // 3 x 3 windows (the ResNet stem): the nine loads in flight at once, out-of-image
            // positions clamped to (hs, ws) and skipped in the row-major scan below
            // 32-bit vector indices (the map has < 2^31 16-B vectors: checked on the host):
            // the clamped corner (hs, ws) and the window origin, then constant offsets per tap
            float v[9][8];
            const int xc = ((n * a.H + hs) * a.W + ws) * a.C8 + cg;
            const int x00 = xc + ((h0 - hs) * a.W + (w0 - ws)) * a.C8;
            const int WC8 = a.W * a.C8;
#pragma unroll
            for (int u = 0; u < 9; ++u) {
                const int h = h0 + u / 3, w = w0 + u % 3;
                const bool in = h >= 0 && h < a.H && w >= 0 && w < a.W;
                V8<E>::ld(x, in ? x00 + (u / 3) * WC8 + (u % 3) * a.C8 : xc, v[u]);
            }
#pragma unroll
            for (int u = 0; u < 9; ++u) {
                const int h = h0 + u / 3, w = w0 + u % 3;
                if (h < 0 || h >= a.H || w < 0 || w >= a.W) continue;
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const float z = BNRELU ? round_to<E>(relu_nan(fmaf(v[u][j], sc[j], sh[j]))) : v[u][j];
                    if (z > m[j] || __builtin_isnan(z)) {
                        m[j] = z;
                        xs[j] = v[u][j];
                        ix[j] = (uint32_t)u;
                    }
                }
            }
        } else
        for (int r = 0; r < a.k; ++r) {
            const int h = h0 + r;
            if (h < 0 || h >= a.H) continue;
            for (int c = 0; c < a.k; ++c) {
                const int w = w0 + c;
                if (w < 0 || w >= a.W) continue;
                float v[8], raw[8];
                V8<E>::ld(x, (((long long)n * a.H + h) * a.W + w) * a.C8 + cg, v);
#pragma unroll
                for (int j = 0; j < 8; ++j) raw[j] = v[j];
                if (BNRELU) {
#pragma unroll
                    for (int j = 0; j < 8; ++j) v[j] = round_to<E>(relu_nan(fmaf(v[j], sc[j], sh[j])));
                }
                const uint32_t pos = (uint32_t)(r * a.k + c);
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    if (v[j] > m[j] || __builtin_isnan(v[j])) {
                        m[j] = v[j];
                        xs[j] = raw[j];
                        ix[j] = pos;
                    }
                }
            }
        }
        V8<E>::st(y, i, m);  // the max of E values is an E value: the store is exact
        if (xsel) V8<E>::st(xsel, i, xs);  // an E value loaded from x: exact
        idx[i] = make_uint2(ix[0] | ix[1] << 8 | ix[2] << 16 | ix[3] << 24, ix[4] | ix[5] << 8 | ix[6] << 16 | ix[7] << 24);
    }
}

template <typename E>
__global__ __launch_bounds__(256) void k_maxpool_bwd(PoolArgs a, const void* __restrict__ dy,
                                                     const uint2* __restrict__ idx, void* __restrict__ dx) {
    const unsigned total = (unsigned)a.N * a.H * a.W * a.C8;
    for (unsigned i = blockIdx.x * 256 + threadIdx.x; i < total; i += gridDim.x * 256) {
        unsigned t = a.fd_c8.div(i);
        const int cg = (int)(i - t * a.C8);
        unsigned t2 = a.fd_w.div(t);
        const int w = (int)(t - t2 * a.W);
        const unsigned n_ = a.fd_h.div(t2);
        const int h = (int)(t2 - n_ * a.H);
        const int n = (int)n_;
        // windows p with p*s - pad <= h <= p*s - pad + k - 1
        int plo = h + a.pad - a.k + 1;
        plo = plo <= 0 ? 0 : (int)a.fd_s.div((unsigned)(plo + a.s - 1));
        int phi = (int)a.fd_s.div((unsigned)(h + a.pad));
        if (phi > a.P - 1) phi = a.P - 1;
        int qlo = w + a.pad - a.k + 1;
        qlo = qlo <= 0 ? 0 : (int)a.fd_s.div((unsigned)(qlo + a.s - 1));
        int qhi = (int)a.fd_s.div((unsigned)(w + a.pad));
        if (qhi > a.Q - 1) qhi = a.Q - 1;
        float g[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) g[j] = 0.f;
        if (a.k == 3 && a.s == 2) {
            // the ResNet stem's pool: at most 2 x 2 windows; all eight loads in flight at
            // once (addresses clamped to a valid window, contributions predicated), summed
            // in the generic loop's order (p, then q, ascending)
            uint2 iv[4];
            float dv[4][8];
            bool ok[4];
            uint32_t pos[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int p = phi - 1 + (u >> 1), q = qhi - 1 + (u & 1);
                ok[u] = p >= plo && q >= qlo;
                const int pc = ok[u] ? p : phi, qc = ok[u] ? q : qhi;
                const long long o = (((long long)n * a.P + pc) * a.Q + qc) * a.C8 + cg;
                iv[u] = idx[o];
                V8<E>::ld(dy, o, dv[u]);
                pos[u] = (uint32_t)((h - (p * a.s - a.pad)) * a.k + (w - (q * a.s - a.pad)));
            }
#pragma unroll
            for (int u = 0; u < 4; ++u)
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const uint32_t b = ((j < 4 ? iv[u].x : iv[u].y) >> (8 * (j & 3))) & 0xffu;
                    if (ok[u] && b == pos[u]) g[j] += dv[u][j];
                }
            V8<E>::st(dx, i, g);
            continue;
        }
        for (int p = plo; p <= phi; ++p) {
            for (int q = qlo; q <= qhi; ++q) {
                const long long o = (((long long)n * a.P + p) * a.Q + q) * a.C8 + cg;
                const uint2 iv = idx[o];
                const uint32_t pos = (uint32_t)((h - (p * a.s - a.pad)) * a.k + (w - (q * a.s - a.pad)));
                float d[8];
                V8<E>::ld(dy, o, d);
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const uint32_t b = ((j < 4 ? iv.x : iv.y) >> (8 * (j & 3))) & 0xffu;
                    if (b == pos) g[j] += d[j];
                }
            }
        }
        V8<E>::st(dx, i, g);
    }
}

int prep(const gm_pool_desc* d, PoolArgs& a, const char* fn) {
    if (!d) {
        set_error("%s: null descriptor", fn);
        return GM_E_ARG;
    }
    if (d->N <= 0 || d->H <= 0 || d->W <= 0 || d->C <= 0 || d->C % 8 || d->k < 1 || d->k > 15 || d->stride < 1 ||
        d->pad < 0 || 2 * d->pad > d->k) {
        set_error("%s: unsupported N=%d H=%d W=%d C=%d k=%d s=%d pad=%d (C%%8==0, k<=15, pad<=k/2)", fn, d->N, d->H,
                  d->W, d->C, d->k, d->stride, d->pad);
        return GM_E_ARG;
    }
    a.N = d->N; a.H = d->H; a.W = d->W; a.C8 = d->C / 8;
    a.k = d->k; a.s = d->stride; a.pad = d->pad;
    a.P = (d->H + 2 * d->pad - d->k) / d->stride + 1;
    a.Q = (d->W + 2 * d->pad - d->k) / d->stride + 1;
    if (a.P <= 0 || a.Q <= 0) {
        set_error("%s: empty output", fn);
        return GM_E_ARG;
    }
    if ((long long)a.N * a.H * a.W * a.C8 >= (1ll << 31)) {
        set_error("%s: tensor too large (N*H*W*C/8 >= 2^31)", fn);
        return GM_E_ARG;
    }
    a.fd_c8 = FastDiv((uint32_t)a.C8);
    a.fd_q = FastDiv((uint32_t)a.Q);
    a.fd_p = FastDiv((uint32_t)a.P);
    a.fd_w = FastDiv((uint32_t)a.W);
    a.fd_h = FastDiv((uint32_t)a.H);
    a.fd_s = FastDiv((uint32_t)a.s);
    a.fd_ng = FastDiv((uint32_t)a.N);
    return GM_OK;
}

inline int grid_for(long long n) {
    long long g = (n + 255) / 256;
    if (g > 16384) g = 16384;
    return (int)(g < 1 ? 1 : g);
}

}  // namespace
}  // namespace gm

using namespace gm;

template <typename E>
int pool_fwd(const gm_pool_desc* d, const void* x, void* y, void* idx, void* stream, const char* fn) {
    PoolArgs a;
    int rc = prep(d, a, fn);
    if (rc) return rc;
    GM_REQUIRE(x && y && idx, "%s: null pointer", fn);
    const long long n = (long long)a.N * a.P * a.Q * a.C8;
    hipLaunchKernelGGL(k_maxpool_fwd<E>, dim3(grid_for(n)), dim3(256), 0, as_stream(stream), a, x, y,
                       static_cast<uint2*>(idx));
    return check_launch("k_maxpool_fwd");
}

template <typename E>
int pool_bwd(const gm_pool_desc* d, const void* dy, const void* idx, void* dx, void* stream, const char* fn) {
    PoolArgs a;
    int rc = prep(d, a, fn);
    if (rc) return rc;
    GM_REQUIRE(dy && idx && dx, "%s: null pointer", fn);
    const long long n = (long long)a.N * a.H * a.W * a.C8;
    hipLaunchKernelGGL(k_maxpool_bwd<E>, dim3(grid_for(n)), dim3(256), 0, as_stream(stream), a, dy,
                       static_cast<const uint2*>(idx), dx);
    return check_launch("k_maxpool_bwd");
}

extern "C" int gm_maxpool2d_fwd_bf16(const gm_pool_desc* d, const void* x, void* y, void* idx, void* stream) {
    return pool_fwd<uint16_t>(d, x, y, idx, stream, "gm_maxpool2d_fwd_bf16");
}

// G view groups of d->N images each, stacked along the batch; group g applies the
// coefficients coef + g*2C; xsel (optional, y-shaped) receives each output's selected raw x
extern "C" int gm_bn_relu_maxpool2d_fwd_grouped_bf16(const gm_pool_desc* d, int G, const void* x, const float* coef,
                                                     void* y, void* idx, void* xsel, void* stream) {
    const char* fn = "gm_bn_relu_maxpool2d_fwd_grouped_bf16";
    GM_REQUIRE(d && G >= 1 && G <= 64, "%s: 1..64 groups", fn);
    gm_pool_desc dg = *d;
    dg.N = d->N * G;
    PoolArgs a;
    int rc = prep(&dg, a, fn);
    if (rc) return rc;
    a.fd_ng = FastDiv((uint32_t)d->N);
    GM_REQUIRE(x && coef && y && idx, "%s: null pointer", fn);
    const long long n = (long long)a.N * a.P * a.Q * a.C8;
    hipLaunchKernelGGL((k_maxpool_fwd<uint16_t, true>), dim3(grid_for(n)), dim3(256), 0, as_stream(stream), a, x, y,
                       static_cast<uint2*>(idx), coef, xsel);
    return check_launch("k_maxpool_fwd<bnrelu>");
}

extern "C" int gm_bn_relu_maxpool2d_fwd_bf16(const gm_pool_desc* d, const void* x, const float* coef, void* y,
                                             void* idx, void* stream) {
    return gm_bn_relu_maxpool2d_fwd_grouped_bf16(d, 1, x, coef, y, idx, nullptr, stream);
}

extern "C" int gm_maxpool2d_bwd_bf16(const gm_pool_desc* d, const void* dy, const void* idx, void* dx, void* stream) {
    return pool_bwd<uint16_t>(d, dy, idx, dx, stream, "gm_maxpool2d_bwd_bf16");
}

extern "C" int gm_maxpool2d_fwd_f32(const gm_pool_desc* d, const void* x, void* y, void* idx, void* stream) {
    return pool_fwd<float>(d, x, y, idx, stream, "gm_maxpool2d_fwd_f32");
}

extern "C" int gm_maxpool2d_bwd_f32(const gm_pool_desc* d, const void* dy, const void* idx, void* dx, void* stream) {
    return pool_bwd<float>(d, dy, idx, dx, stream, "gm_maxpool2d_bwd_f32");
}
