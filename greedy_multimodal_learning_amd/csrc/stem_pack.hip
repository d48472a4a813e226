// Pixel-pair packing of the RGB stem (conv.py stem path): ONE launch builds both
//   the input view  xp[n][hp][wq][8]  = {x[n, c, hp-pad, 2wq+j-pad] : j in 0..1, c in 0..3}
//                   (zero outside the image and for c >= C0), bf16, from an fp32 or bf16
//                   NCHW-strided x (e.g. x[:, view] of the [B, V, 3, H, W] batch), and
//   the weight view wp[k][r][sq][8]  = {w[k, c, r, 2sq+j] : j in 0..1, c in 0..3}
//                   (zero for s >= S or c >= C0), bf16 from the fp32 [K, C0, R, S] weight at
//                   any strides (the model's channels_last parameter, no contiguous copy).
// Each thread writes one 16-B element (2 pixels x 4 channels); reads are coalesced per
// channel plane.  Replaces the zero-fill + strided cast/copy PyTorch launches of the
// input and of the weight (4 launches per view).
#include "gm_common.h"

namespace gm {
namespace {

constexpr int kPT = 256;

__device__ __forceinline__ unsigned short bf16_of(float f) {
    unsigned u = __float_as_uint(f);
    if ((u & 0x7fffffffu) > 0x7f800000u) return (unsigned short)0x7fc0;  // NaN, as c10::BFloat16
    u += 0x7fffu + ((u >> 16) & 1u);  // round to nearest even
    return (unsigned short)(u >> 16);
}

template <bool BF16>
__device__ __forceinline__ unsigned short load_bf16(const void* p, long long i) {
    if (BF16) return static_cast<const unsigned short*>(p)[i];
    return bf16_of(static_cast<const float*>(p)[i]);
}

template <bool BF16>
__global__ __launch_bounds__(kPT) void k_stem_pack(gm_stem_pack a, long long nx, int nw) {
    const long long i = (long long)blockIdx.x * kPT + threadIdx.x;
    unsigned short v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = 0;
    if (i < nx) {  // input element (n, hp, wq)
        const int Wq = a.Wp >> 1;
        const long long nh = i / Wq;
        const int wq = (int)(i - nh * Wq);
        const int n = (int)(nh / a.Hp), hp = (int)(nh - (long long)n * a.Hp);
        const int h = hp - a.pad;
        if (h >= 0 && h < a.H) {
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                const int w = 2 * wq + j - a.pad;
                if (w >= 0 && w < a.W) {
                    const long long base = (long long)n * a.sn + (long long)h * a.sh + (long long)w * a.sw;
                    for (int c = 0; c < a.C0; ++c) v[4 * j + c] = load_bf16<BF16>(a.x, base + (long long)c * a.sc);
                }
            }
        }
        uint4 o;
        o.x = v[0] | ((unsigned)v[1] << 16); o.y = v[2] | ((unsigned)v[3] << 16);
        o.z = v[4] | ((unsigned)v[5] << 16); o.w = v[6] | ((unsigned)v[7] << 16);
        reinterpret_cast<uint4*>(a.xp)[i] = o;
    } else if (i < nx + nw) {  // weight element (k, r, sq)
        const long long e = i - nx;
        const int Sq = (a.S + 1) >> 1;
        const int k = (int)(e / (a.R * Sq));
        const int rs = (int)(e - (long long)k * a.R * Sq);
        const int r = rs / Sq, sq = rs - r * Sq;
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const int s = 2 * sq + j;
            if (s < a.S)
                for (int c = 0; c < a.C0; ++c)
                    v[4 * j + c] = bf16_of(a.w[(long long)k * a.wk + (long long)c * a.wc + (long long)r * a.wr +
                                               (long long)s * a.ws]);
        }
        uint4 o;
        o.x = v[0] | ((unsigned)v[1] << 16); o.y = v[2] | ((unsigned)v[3] << 16);
        o.z = v[4] | ((unsigned)v[5] << 16); o.w = v[6] | ((unsigned)v[7] << 16);
        reinterpret_cast<uint4*>(a.wp)[e] = o;
    }
}

}  // namespace
}  // namespace gm

using namespace gm;

extern "C" int gm_stem_pack_bf16(const gm_stem_pack* p, void* stream) {
    GM_REQUIRE(p && p->x && p->xp, "gm_stem_pack_bf16: null argument");
    GM_REQUIRE(p->C0 >= 1 && p->C0 <= 4 && p->N > 0 && p->H > 0 && p->W > 0 && p->pad >= 0,
               "gm_stem_pack_bf16: need 1 <= C0 <= 4 and a non-empty image");
    GM_REQUIRE(p->Hp >= p->H + p->pad && p->Wp >= p->W + p->pad && (p->Wp & 1) == 0,
               "gm_stem_pack_bf16: pair view %dx%d too small for %dx%d + pad %d (Wp even)", p->Hp, p->Wp, p->H,
               p->W, p->pad);
    GM_REQUIRE(p->dtype == GM_F32 || p->dtype == GM_BF16, "gm_stem_pack_bf16: x must be fp32 or bf16");
    GM_REQUIRE(!p->w || (p->wp && p->K > 0 && p->R > 0 && p->S > 0), "gm_stem_pack_bf16: bad weight");
    gm_stem_pack q = *p;
    if (q.w && !q.wk && !q.wc && !q.wr && !q.ws) {  // contiguous [K, C0, R, S]
        q.ws = 1;
        q.wr = q.S;
        q.wc = (long long)q.R * q.S;
        q.wk = (long long)q.C0 * q.R * q.S;
    }
    p = &q;
    const long long nx = (long long)p->N * p->Hp * (p->Wp / 2);
    const int nw = p->w ? p->K * p->R * ((p->S + 1) / 2) : 0;
    const long long tot = nx + nw;
    const dim3 g((unsigned)((tot + kPT - 1) / kPT));
    if (p->dtype == GM_BF16)
        hipLaunchKernelGGL(k_stem_pack<true>, g, dim3(kPT), 0, as_stream(stream), *p, nx, nw);
    else
        hipLaunchKernelGGL(k_stem_pack<false>, g, dim3(kPT), 0, as_stream(stream), *p, nx, nw);
    return check_launch("k_stem_pack");
}
