// bf16 implicit-GEMM convolution on MFMA (gfx950), NHWC activations, KRSC weights.
//
// One kernel serves the ResNet trunk's forward convolutions and their input
// gradients (the trunk of reference src/model.py:53-106, torchvision ResNet):
//
//   out[b, p*oS+oH, q*oS+oW, n] = sum_{t < ntap} sum_c in[b, p*sA+dh_t, q*sA+dw_t, c] * wt[n, tap_t, c]
//
//   forward  : one class, taps (r,s) with dh = r - pad, dw = s - pad, sA = stride, oS = 1;
//   dgrad    : input = dY, weights = transpose(W) [Ci][R][S][Co], sA = 1; the output
//              pixels split into stride^2 parity classes (ph, pw), each with only the
//              taps r where (ph + pad - r) % stride == 0 and dh = (ph + pad - r)/stride,
//              so a strided convolution's input gradient wastes no MFMA work.
//
// GEMM view: M = B*P*Q output pixels, N = output channels, K = ntap*C (c fastest).
// Tiles BM x BN x 64; 256 threads = 2x2 waves, each wave (BM/2)x(BN/2) built from
// v_mfma_f32_32x32x16_bf16 tiles; operands staged global -> LDS by LDS-DMA
// (global_load_lds_dwordx4; double-buffered, next tile's DMA under this tile's MFMAs),
// LDS rows of 128 B XOR-swizzled by ((row>>1)&7) (applied on the DMA source address)
// so the ds_read_b128 fragment reads are conflict-free; fp32 accumulation; weights are
// the MFMA A operand so each lane holds 4 consecutive output channels of one pixel and
// the epilogue writes 8-B NHWC chunks directly.  Out-of-range taps read zeros.
#include <algorithm>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <type_traits>

#include "gm_common.h"

namespace gm {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float floatx16 __attribute__((ext_vector_type(16)));

constexpr int kMaxTap = 49;
constexpr int kMaxCls = 4;

struct ConvCls {
    uint16_t* out;
    int P, Q;                 // GEMM output grid of this class
    int oS, oH, oW;           // output pixel = (p*oS + oH, q*oS + oW)
    int ntap;
    int tile_start;           // first workgroup of this class
    int tiles_m;
    short tw[kMaxTap];        // weight tap index (r*S + s)
    signed char dh[kMaxTap], dw[kMaxTap];
    // the same taps as an Rc x Sc grid (tap = i*Sc + j): dh = cdh[i], dw = cdw[j],
    // weight tap = crs[i] + cs[j]; i = (tap * smag) >> 8 (exact for tap < ntap).  The
    // kernel reads them as 4-bit fields: pk_dh/pk_dw hold dh+8 / dw+8, pk_r/pk_s the
    // weight row r_i / column s_j (weight tap = r_i * Sw + s_j).
    int Rc, Sc, smag;
    int dh0, sh, dw0, sw;     // dh_i = dh0 + sh*i, dw_j = dw0 + sw*j (sh, sw = +-1)
    unsigned pk_dh, pk_dw, pk_r, pk_s;
    FastDiv fd_pq, fd_q;      // output pixel -> (b, p, q)
    signed char cdh[8], cdw[8];
    unsigned char crs[8], cs[8];
};

struct ConvArgs {
    const uint16_t* in;       // [N][Hi][Wi][C]
    const uint16_t* wt;       // [Nout][T][C]
    int N, Hi, Wi, C, logC;
    int Nout, T;              // output channels, taps per weight row
    int Sw;                   // weight columns (S)
    int Ho, Wo;               // full output spatial dims
    int sAh, sAw;             // input strides of the GEMM's A rows (H, W)
    int ncls;
    int xcd;                  // remap block ids so consecutive tiles share an XCD (L2)
    // split-K (lean kernel): grid = splits x tiles, split-major; split s of a tile takes
    // k-tiles [s*nk/S, (s+1)*nk/S) and the tile's splits hand their fp32 accumulators
    // on in order 0 -> 1 -> ... -> S-1 through ws (turnstile flags[tile], zero between
    // launches); the last split writes the output.  Deterministic (fixed order).
    const uint16_t* addend;   // dgrad, optional: out = conv + addend (same layout as out)
    // with it, optional: the addend's 1-bit mask (mask_bf2; group g at amask + g * gs_out / 8) -
    // out = conv + (addend where the bit is set), the addend never aliasing out
    const uint8_t* amask;
    int splits, tiles_total;
    float* ws;                // [tiles][MT*NT*16/4][256] float4
    unsigned* flags;          // [tiles]
    unsigned spin_limit;      // poll budget of the turnstile wait
    // view groups in one launch (the view-batched trunk): group g's input, weights and output
    // (and addend) sit gs_in / gs_wt / gs_out elements after group 0's; tiled kernels give
    // group g the tiles [g * tiles_g, (g + 1) * tiles_g), persistent ones gridDim / G workgroups
    int G, tiles_g;
    long long gs_in, gs_wt, gs_out;
    // forward, optional: BatchNorm statistics of the stored (bf16) output from the epilogue -
    // per group [Nout / 64 slices][stats_rows][64 channels][sum, sum of squares] fp32 partial
    // rows (k_conv_rw: one per persistent workgroup; store_tile_lds: one per output tile), then
    // 2 Nout floats of coefficient area: group g at stats + g * 2 Nout (stats_rows + 1)
    // (gm_bn_fwd_stats_finalize_grouped combines them)
    float* stats;
    int stats_rows;
    // input gradient, optional (with stats): the statistics of the BatchNorm backward whose dy
    // this launch writes - the BN's input x (out's layout), its forward coefficients sc, sh
    // ([G][2 Nout]) and save_mean ([G][Nout]): partial rows of (sum dz, sum dz (x - mean)) with
    // dz = dy where x sc + sh > 0 (the forward's ReLU; gm_bn_bwd_stats_finalize_grouped)
    const uint16_t* bnx;
    const float* bncoef;
    const float* bnmean;
    ConvCls cls[kMaxCls];
};

typedef float f32x2 __attribute__((ext_vector_type(2)));  // channel pairs: packed fp32 math

// BatchNorm statistics of one stored 16-B chunk (8 channels) into s1 / s2 (channel pairs):
// forward - sum y, sum y^2 of the stored values v; backward (BnB) - sum dz, sum dz (x - mean)
// of the stored input gradient v with x's chunk xv.  Invalid chunks arrive as zeros (no sum).
struct BnB {
    f32x2 sc[4], sh[4], mu[4];
};
__device__ __forceinline__ void bnb_load(const ConvArgs& a, int grp, int n, BnB& q) {
    const float* cf = a.bncoef + (size_t)grp * 2 * a.Nout + n;
    const float* mu = a.bnmean + (size_t)grp * a.Nout + n;
    const float4 s0 = *reinterpret_cast<const float4*>(cf), s1 = *reinterpret_cast<const float4*>(cf + 4);
    const float4 h0 = *reinterpret_cast<const float4*>(cf + a.Nout), h1 = *reinterpret_cast<const float4*>(cf + a.Nout + 4);
    const float4 m0 = *reinterpret_cast<const float4*>(mu), m1 = *reinterpret_cast<const float4*>(mu + 4);
    q.sc[0] = {s0.x, s0.y}; q.sc[1] = {s0.z, s0.w}; q.sc[2] = {s1.x, s1.y}; q.sc[3] = {s1.z, s1.w};
    q.sh[0] = {h0.x, h0.y}; q.sh[1] = {h0.z, h0.w}; q.sh[2] = {h1.x, h1.y}; q.sh[3] = {h1.z, h1.w};
    q.mu[0] = {m0.x, m0.y}; q.mu[1] = {m0.z, m0.w}; q.mu[2] = {m1.x, m1.y}; q.mu[3] = {m1.z, m1.w};
}
__device__ __forceinline__ void bn_acc_fwd(const unsigned (&v)[4], f32x2 (&s1)[4], f32x2 (&s2)[4]) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const f32x2 f = {bf_lo(v[k]), bf_hi(v[k])};
        s1[k] += f;
        s2[k] = __builtin_elementwise_fma(f, f, s2[k]);
    }
}
__device__ __forceinline__ void bn_acc_bwd(const unsigned (&v)[4], const unsigned (&xv)[4], const BnB& q,
                                           f32x2 (&s1)[4], f32x2 (&s2)[4]) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        f32x2 d = {bf_lo(v[k]), bf_hi(v[k])};
        const f32x2 x = {bf_lo(xv[k]), bf_hi(xv[k])};
        const f32x2 z = __builtin_elementwise_fma(x, q.sc[k], q.sh[k]);  // fmaf(x, sc, sh) > 0: the
        d.x = z.x > 0.f ? d.x : 0.f;                                       // single-launch backward's mask
        d.y = z.y > 0.f ? d.y : 0.f;
        s1[k] += d;
        s2[k] = __builtin_elementwise_fma(d, x - q.mu[k], s2[k]);
    }
}

// sticky fault word of this translation unit (gm_device_faults): a split whose
// turnstile wait timed out
__device__ unsigned g_conv_fault = 0;

__device__ __forceinline__ int swz(int row, int chunk) { return chunk ^ ((row >> 1) & 7); }

// Workgroups are dealt round-robin over the 8 XCDs (b and b+8 share one).  The
// bijective remap gives each XCD a contiguous range of tile ids (tm fastest), so
// the tiles of one output-channel column - one weight slice - stay in one L2.
__device__ __forceinline__ int block_id(int xcd) {
    const int b = blockIdx.x;
    if (!xcd) return b;
    const int n = gridDim.x, q = n >> 3, r = n & 7, x = b & 7;
    return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + (b >> 3);
}

__device__ __attribute__((aligned(16))) const uint4 g_zero16[1] = {{0u, 0u, 0u, 0u}};

// bits i in [0, n) with 0 <= x + d0 + s*i < lim (s = +-1): one contiguous range
__device__ __forceinline__ unsigned span_mask(int x, int d0, int s, int n, int lim) {
    int lo, hi;
    if (s > 0) {
        lo = -(x + d0);
        hi = lim - 1 - (x + d0);
    } else {
        lo = x + d0 - (lim - 1);
        hi = x + d0;
    }
    lo = lo < 0 ? 0 : lo;
    hi = hi > n - 1 ? n - 1 : hi;
    return lo > hi ? 0u : ((2u << hi) - (1u << lo));
}

// ---- shared epilogue: D[n][m] layout: lane -> pixel m (col = lane&31), registers
// 4g..4g+3 -> channels 8g + 4h + 0..3: 8-byte NHWC stores, no LDS.  Through buffer
// resources, the stores and the addend loads (fused gradient join) are issued for the
// whole tile with no per-element branch: out-of-tile positions get an offset past the
// buffer's range, which the hardware drops (stores) or reads as zero (loads), so the
// addend loads are all in flight together instead of one dependent round trip per store.
// MASK: the masked addend (a.amask) is handled here - store_tile_lds's fallback; the kernels that
// store through store_tile directly (k_conv_igemm, k_conv_halo) get their masked addend
// materialised in dx before the launch (demask) and so keep their registers.
template <int MT, int NT, int BM, int BN, bool MASK = false>
__device__ __forceinline__ void store_tile(const ConvArgs& a, const ConvCls& cl, int m0, int n0, int wm, int wn,
                                           int fr, int fh, int M, floatx16 (&acc)[MT][NT], long long goff = 0) {
    const int PQ = cl.P * cl.Q;
    uint16_t* const outp = cl.out + goff;  // this group's output (and addend)
    const uint16_t* const addp = a.addend ? a.addend + goff : nullptr;
    const size_t out_bytes = (size_t)a.N * a.Ho * a.Wo * a.Nout * 2;
    if (out_bytes < 0x7ffff000u) {
        const auto orsrc = __builtin_amdgcn_make_buffer_rsrc(outp, 0, (int)out_bytes, 0x00020000);
        unsigned off[MT];
        bool mok[MT];
#pragma unroll
        for (int i = 0; i < MT; ++i) {
            int m = m0 + wm * (BM / 2) + i * 32 + fr;
            mok[i] = m < M;
            m = mok[i] ? m : m0;
            const int b = (int)cl.fd_pq.div((uint32_t)m), pq = m - b * PQ;
            const int p = (int)cl.fd_q.div((uint32_t)pq), q = pq - p * cl.Q;
            const int ho = p * cl.oS + cl.oH, wo = q * cl.oS + cl.oW;
            off[i] = (unsigned)(((b * a.Ho + ho) * a.Wo + wo) * a.Nout) * 2u;
        }
        auto boff = [&](int i, int j, int gq) {
            const int n = n0 + wn * (BN / 2) + j * 32 + 8 * gq + 4 * fh;
            return (mok[i] && n < a.Nout) ? off[i] + (unsigned)n * 2u : 0xfffffff0u;
        };
        typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
        u32x2 av[MT][NT][4];
        if (a.addend) {
            const auto arsrc = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t*>(addp), 0, (int)out_bytes,
                                                                 0x00020000);
#pragma unroll
            for (int i = 0; i < MT; ++i)
#pragma unroll
                for (int j = 0; j < NT; ++j)
#pragma unroll
                    for (int gq = 0; gq < 4; ++gq)
                        av[i][j][gq] = __builtin_amdgcn_raw_buffer_load_b64(arsrc, boff(i, j, gq), 0, 0);
            if (MASK && a.amask) {  // (Nout % 32 == 0) one mask dword per 32 channels: gq's byte, fh's nibble
                const auto mrsrc = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(a.amask + goff / 8), 0,
                                                                     (int)(out_bytes >> 4), 0x00020000);
#pragma unroll
                for (int i = 0; i < MT; ++i)
#pragma unroll
                    for (int j = 0; j < NT; ++j) {
                        const unsigned w = __builtin_amdgcn_raw_buffer_load_b32(mrsrc, (boff(i, j, 0) - 8u * fh) >> 4,
                                                                                0, 0) >> (4 * fh);
#pragma unroll
                        for (int gq = 0; gq < 4; ++gq) {
                            av[i][j][gq].x = mask_bf2(av[i][j][gq].x, w >> (8 * gq));
                            av[i][j][gq].y = mask_bf2(av[i][j][gq].y, w >> (8 * gq + 2));
                        }
                    }
            }
        }
#pragma unroll
        for (int i = 0; i < MT; ++i)
#pragma unroll
            for (int j = 0; j < NT; ++j)
#pragma unroll
                for (int gq = 0; gq < 4; ++gq) {
                    float o0 = acc[i][j][4 * gq], o1 = acc[i][j][4 * gq + 1];
                    float o2 = acc[i][j][4 * gq + 2], o3 = acc[i][j][4 * gq + 3];
                    if (a.addend) {
                        o0 += bf_lo(av[i][j][gq].x); o1 += bf_hi(av[i][j][gq].x);
                        o2 += bf_lo(av[i][j][gq].y); o3 += bf_hi(av[i][j][gq].y);
                    }
                    const u32x2 v = {pack_bf2(o0, o1), pack_bf2(o2, o3)};
                    __builtin_amdgcn_raw_buffer_store_b64(v, orsrc, boff(i, j, gq), 0, 0);
                }
        return;
    }
#pragma unroll
    for (int i = 0; i < MT; ++i) {  // outputs of 2 GB or more: 64-bit addressing
        const int m = m0 + wm * (BM / 2) + i * 32 + fr;
        if (m >= M) continue;
        const int b = (int)cl.fd_pq.div((uint32_t)m), pq = m - b * PQ;
        const int p = (int)cl.fd_q.div((uint32_t)pq), q = pq - p * cl.Q;
        const int ho = p * cl.oS + cl.oH, wo = q * cl.oS + cl.oW;
        uint16_t* dst = outp + ((size_t)(b * a.Ho + ho) * a.Wo + wo) * a.Nout;
#pragma unroll
        for (int j = 0; j < NT; ++j)
#pragma unroll
            for (int gq = 0; gq < 4; ++gq) {
                const int n = n0 + wn * (BN / 2) + j * 32 + 8 * gq + 4 * fh;
                if (n >= a.Nout) continue;
                float o0 = acc[i][j][4 * gq], o1 = acc[i][j][4 * gq + 1];
                float o2 = acc[i][j][4 * gq + 2], o3 = acc[i][j][4 * gq + 3];
                if (a.addend) {
                    uint2 av = *(const uint2*)(addp + (dst - outp) + n);
                    if (MASK && a.amask) {
                        const size_t e = (size_t)goff + (size_t)(dst - outp) + n;
                        const unsigned b = (unsigned)a.amask[e >> 3] >> (e & 4);
                        av.x = mask_bf2(av.x, b);
                        av.y = mask_bf2(av.y, b >> 2);
                    }
                    o0 += bf_lo(av.x); o1 += bf_hi(av.x); o2 += bf_lo(av.y); o3 += bf_hi(av.y);
                }
                uint2 v;
                v.x = pack_bf2(o0, o1);
                v.y = pack_bf2(o2, o3);
                *(uint2*)(dst + n) = v;
            }
    }
}

// The same epilogue through LDS for the 256-thread tiled kernels (2 x 2 waves of MT x NT
// fragments, the k-loop's LDS idle: every DMA has landed, the caller's barrier-free reads
// end at the __syncthreads below): the tile's BM pixel rows of BN channels are assembled in
// LDS - bf16, or fp32 with the fused gradient-join addend (added before the one rounding) -
// 16-B chunks XOR-swizzled by pixel, and leave as 16-B stores, BN / 8 lanes per contiguous
// pixel row segment.  The direct 8-B stores from the MFMA layout touch 32 pixel rows per
// instruction: 13 % of the layer-3 halo launch (41.4 us with, 36.0 without them).  Falls
// back to store_tile when the LDS is too small or the output needs 64-bit offsets.
template <int MT, int NT, int BM, int BN>
__device__ __forceinline__ void store_tile_lds(const ConvArgs& a, const ConvCls& cl, int m0, int n0, int wm, int wn,
                                               int fr, int fh, int M, floatx16 (&acc)[MT][NT], long long goff,
                                               char* lds, int lds_bytes, int t, int grp) {
    static_assert(BM == 64 * MT && BN == 64 * NT, "store_tile_lds: 2 x 2 waves of MT x NT fragments");
    const size_t out_bytes = (size_t)a.N * a.Ho * a.Wo * a.Nout * 2;
    const bool f32 = a.addend != nullptr;
    if (out_bytes >= 0x7ffff000u || BM * BN * (f32 ? 4 : 2) + 4 * (BN / 8) * 64 > lds_bytes) {
        store_tile<MT, NT, BM, BN, true>(a, cl, m0, n0, wm, wn, fr, fh, M, acc, goff);
        return;
    }
    constexpr int CH = BN / 8, CF = BN / 4;  // bf16 / fp32 16-B chunks per pixel row
    constexpr int NU = BM * CH / 256;          // output chunks per thread
    __syncthreads();  // every wave is done with the k-loop's LDS
    if (f32) {
#pragma unroll
        for (int i = 0; i < MT; ++i)
#pragma unroll
            for (int j = 0; j < NT; ++j)
#pragma unroll
                for (int gq = 0; gq < 4; ++gq) {
                    const int px = wm * (BM / 2) + i * 32 + fr, c = wn * (CF / 2) + 8 * j + 2 * gq + fh;
                    *reinterpret_cast<float4*>(lds + px * (BN * 4) + ((c ^ (px & (CF - 1))) << 4)) =
                        make_float4(acc[i][j][4 * gq], acc[i][j][4 * gq + 1], acc[i][j][4 * gq + 2], acc[i][j][4 * gq + 3]);
                }
    } else {
#pragma unroll
        for (int i = 0; i < MT; ++i)
#pragma unroll
            for (int j = 0; j < NT; ++j)
#pragma unroll
                for (int gq = 0; gq < 4; ++gq) {
                    const int px = wm * (BM / 2) + i * 32 + fr, c = wn * (CH / 2) + 4 * j + gq;
                    *reinterpret_cast<uint2*>(lds + px * (BN * 2) + ((c ^ (px & (CH - 1))) << 4) + 8 * fh) =
                        make_uint2(pack_bf2(acc[i][j][4 * gq], acc[i][j][4 * gq + 1]),
                                   pack_bf2(acc[i][j][4 * gq + 2], acc[i][j][4 * gq + 3]));
                }
    }
    __syncthreads();
    // this thread's chunks: pixel row px = e / CH, chunk c = e % CH of e = t + 256 u
    const int PQ = cl.P * cl.Q;
    // dense classes (forward, stride-1 input gradient): output pixel m is NHWC row m
    const bool dense = cl.oS == 1 && cl.oH == 0 && cl.oW == 0 && cl.P == a.Ho && cl.Q == a.Wo;
    unsigned off[NU];  // (computed branch-free per lane: a per-lane branch in these unrolled loops
                       // serialises them)
    if (dense) {
#pragma unroll
        for (int u = 0; u < NU; ++u) {
            const int e = t + 256 * u, px = e / CH, c = e - px * CH;
            const int m = m0 + px, n = n0 + 8 * c;
            const unsigned o = (unsigned)m * (unsigned)a.Nout * 2u + (unsigned)n * 2u;
            off[u] = (m < M) & (n < a.Nout) ? o : 0xfffffff0u;
        }
    } else {
#pragma unroll
        for (int u = 0; u < NU; ++u) {
            const int e = t + 256 * u, px = e / CH, c = e - px * CH;
            const int n = n0 + 8 * c;
            const int m = min(m0 + px, M - 1);
            const int b = (int)cl.fd_pq.div((uint32_t)m), pq = m - b * PQ;
            const int p = (int)cl.fd_q.div((uint32_t)pq), q = pq - p * cl.Q;
            const unsigned o = (unsigned)((((b * a.Ho + p * cl.oS + cl.oH) * a.Wo + q * cl.oS + cl.oW) * a.Nout + n) * 2);
            off[u] = (m0 + px < M) & (n < a.Nout) ? o : 0xfffffff0u;
        }
    }
    uint16_t* const outp = cl.out + goff;
    const auto orsrc = __builtin_amdgcn_make_buffer_rsrc(outp, 0, (int)out_bytes, 0x00020000);
    typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
    if (f32) {
        const auto arsrc = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t*>(a.addend + goff), 0, (int)out_bytes,
                                                             0x00020000);
        u32x4 av[NU];
#pragma unroll
        for (int u = 0; u < NU; ++u) av[u] = __builtin_amdgcn_raw_buffer_load_b128(arsrc, off[u], 0, 0);
        if (a.amask) {  // one mask byte per 16-B chunk: byte off / 16 (past the range: 0)
            const auto mrsrc = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(a.amask + goff / 8), 0,
                                                                 (int)(out_bytes >> 4), 0x00020000);
            unsigned mb[NU];
#pragma unroll
            for (int u = 0; u < NU; ++u) mb[u] = __builtin_amdgcn_raw_buffer_load_b8(mrsrc, off[u] >> 4, 0, 0);
#pragma unroll
            for (int u = 0; u < NU; ++u) {
                av[u].x = mask_bf2(av[u].x, mb[u]);
                av[u].y = mask_bf2(av[u].y, mb[u] >> 2);
                av[u].z = mask_bf2(av[u].z, mb[u] >> 4);
                av[u].w = mask_bf2(av[u].w, mb[u] >> 6);
            }
        }
#pragma unroll
        for (int u = 0; u < NU; ++u) {
            const int e = t + 256 * u, px = e / CH, c = e - px * CH;
            const float4 f0 = *reinterpret_cast<const float4*>(lds + px * (BN * 4) + (((2 * c) ^ (px & (CF - 1))) << 4));
            const float4 f1 = *reinterpret_cast<const float4*>(lds + px * (BN * 4) + (((2 * c + 1) ^ (px & (CF - 1))) << 4));
            const u32x4 o = {pack_bf2(f0.x + bf_lo(av[u].x), f0.y + bf_hi(av[u].x)),
                             pack_bf2(f0.z + bf_lo(av[u].y), f0.w + bf_hi(av[u].y)),
                             pack_bf2(f1.x + bf_lo(av[u].z), f1.y + bf_hi(av[u].z)),
                             pack_bf2(f1.z + bf_lo(av[u].w), f1.w + bf_hi(av[u].w))};
            __builtin_amdgcn_raw_buffer_store_b128(o, orsrc, off[u], 0, 0);
        }
        return;
    }
    u32x4 v[NU];
#pragma unroll
    for (int u = 0; u < NU; ++u) {
        const int e = t + 256 * u, px = e / CH, c = e - px * CH;
        v[u] = *reinterpret_cast<const u32x4*>(lds + px * (BN * 2) + ((c ^ (px & (CH - 1))) << 4));
    }
#pragma unroll
    for (int u = 0; u < NU; ++u) __builtin_amdgcn_raw_buffer_store_b128(v[u], orsrc, off[u], 0, 0);
    if (a.stats) {
        // BatchNorm statistics of the stored values (forward: y; input gradient: the BN
        // backward's dz against x): this thread's chunk c = t % CH (8 channels) over its NU
        // pixels, then the lanes sharing c (c + CH k: xor 8 / 16 / 32) and the four waves (LDS
        // past the tile) - one partial row per output tile, row m0 / BM
        f32x2 s1[4], s2[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) s1[k] = s2[k] = f32x2{0.f, 0.f};
        if (a.bnx) {
            const auto xrsrc = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t*>(a.bnx + goff), 0,
                                                                 (int)out_bytes, 0x00020000);
            u32x4 xv[NU];
#pragma unroll
            for (int u = 0; u < NU; ++u) xv[u] = __builtin_amdgcn_raw_buffer_load_b128(xrsrc, off[u], 0, 0);
            const int n = n0 + 8 * (t % CH);
            BnB q;
            bnb_load(a, grp, n < a.Nout ? n : 0, q);
#pragma unroll
            for (int u = 0; u < NU; ++u) {
                const bool ok = off[u] != 0xfffffff0u;
                const unsigned w4[4] = {ok ? v[u].x : 0u, ok ? v[u].y : 0u, ok ? v[u].z : 0u, ok ? v[u].w : 0u};
                const unsigned x4[4] = {xv[u].x, xv[u].y, xv[u].z, xv[u].w};
                bn_acc_bwd(w4, x4, q, s1, s2);
            }
        } else {
#pragma unroll
            for (int u = 0; u < NU; ++u) {
                const bool ok = off[u] != 0xfffffff0u;
                const unsigned w4[4] = {ok ? v[u].x : 0u, ok ? v[u].y : 0u, ok ? v[u].z : 0u, ok ? v[u].w : 0u};
                bn_acc_fwd(w4, s1, s2);
            }
        }
        float r[16];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            r[4 * k] = s1[k].x; r[4 * k + 1] = s2[k].x; r[4 * k + 2] = s1[k].y; r[4 * k + 3] = s2[k].y;
        }
        const int lane = t & 63, wave = t >> 6;
#pragma unroll
        for (int q = 0; q < 16; ++q) {
            float x = r[q];
            if (CH == 8) x += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x128, 0xf, 0xf, false));
            x += __int_as_float(__builtin_amdgcn_ds_swizzle(__float_as_int(x), 0x401f));
            x += __shfl_xor(x, 32);
            r[q] = x;
        }
        float* red = reinterpret_cast<float*>(lds + BM * BN * 2);  // [4 waves][CH chunks][16]
        if (lane < CH) {
#pragma unroll
            for (int q = 0; q < 4; ++q)
                *reinterpret_cast<float4*>(red + (wave * CH + lane) * 16 + 4 * q) =
                    make_float4(r[4 * q], r[4 * q + 1], r[4 * q + 2], r[4 * q + 3]);
        }
        __syncthreads();
        if (t < BN) {  // channel n0 + t: chunk t / 8, channel j = t % 8 of it
            const int c = t >> 3, j = t & 7;
            float S1 = 0.f, S2 = 0.f;
#pragma unroll
            for (int w = 0; w < 4; ++w) {
                S1 += red[(w * CH + c) * 16 + 2 * j];
                S2 += red[(w * CH + c) * 16 + 2 * j + 1];
            }
            const int n = n0 + t;
            if (n < a.Nout) {
                float* sp = a.stats + (size_t)grp * 2 * a.Nout * (a.stats_rows + 1);
                *reinterpret_cast<float2*>(sp + ((size_t)(n >> 6) * a.stats_rows + m0 / BM) * 128 + (n & 63) * 2) =
                    make_float2(S1, S2);
            }
        }
    }
}

template <int BM, int BN, bool UT, int ST>
__global__ __launch_bounds__(256) void k_conv_igemm(ConvArgs a) {
    constexpr int BK = 64;
    constexpr int AR = BM / 32;       // A rows per thread
    constexpr int BR = BN / 32;       // B rows per thread
    constexpr int MT = BM / 64, NT = BN / 64;  // 32x32 MFMA tiles per wave
    constexpr int G = AR + BR;        // LDS-DMA instructions per wave per k-tile
    extern __shared__ __attribute__((aligned(16))) uint4 smem[];
    uint4* As = smem;                           // [ST][BM][8] (16-B chunks)
    uint4* Bs = smem + ST * BM * 8;             // [ST][BN][8]

    const int bid = block_id(a.xcd);
    int ci = 0;
#pragma unroll
    for (int q = 1; q < kMaxCls; ++q)
        if (q < a.ncls && bid >= a.cls[q].tile_start) ci = q;
    const ConvCls& cl = a.cls[ci];
    const int wgid = bid - cl.tile_start;
    const int tm = wgid % cl.tiles_m, tn = wgid / cl.tiles_m;
    const int m0 = tm * BM, n0 = tn * BN;
    const int PQ = cl.P * cl.Q;
    const int M = a.N * PQ;
    const int Ktot = cl.ntap * a.C;
    const int nk = (Ktot + BK - 1) / BK;

    const int t = threadIdx.x;
    const int lane = t & 63, wave = t >> 6;
    // tap table -> LDS (static indices only into the kernel-argument struct)
    int* tapt = (int*)(smem + ST * (BM + BN) * 8);
#pragma unroll
    for (int i = 0; i < kMaxTap; ++i)
        if (t == i && i < cl.ntap)
            tapt[i] = (int)cl.tw[i] | ((int)(cl.dh[i] + 128) << 8) | ((int)(cl.dw[i] + 128) << 16);
    __syncthreads();
    const int wm = wave >> 1, wn = wave & 1;
    const int slot = lane & 7;                  // 16-B LDS slot this lane's DMA fills

    // Staging is LDS-DMA (global_load_lds_dwordx4): a wave instruction writes 64 x 16 B
    // = 8 rows x 128 B linearly, so the XOR swizzle moves to the SOURCE: the lane that
    // fills slot s of row r loads global chunk s ^ f(r).  Zero taps (padding) read a
    // 16-B zero block of the code object.
    const uint16_t* a_ptr[AR];
    int a_h[AR], a_w[AR], a_gc[AR];
#pragma unroll
    for (int j = 0; j < AR; ++j) {
        const int row = (wave * AR + j) * 8 + (lane >> 3);
        const int m = m0 + row;
        a_gc[j] = slot ^ ((row >> 1) & 7);
        if (m < M) {
            const int b = m / PQ, pq = m - b * PQ;
            const int p = pq / cl.Q, q = pq - p * cl.Q;
            a_h[j] = p * a.sAh;
            a_w[j] = q * a.sAw;
            a_ptr[j] = a.in + ((size_t)((b * a.Hi + a_h[j]) * a.Wi + a_w[j]) << a.logC);
        } else {
            a_h[j] = -(1 << 28);  // never valid
            a_w[j] = 0;
            a_ptr[j] = a.in;
        }
    }
    const uint16_t* b_ptr[BR];
    bool b_ok[BR];
    int b_gc[BR];
#pragma unroll
    for (int j = 0; j < BR; ++j) {
        const int row = (wave * BR + j) * 8 + (lane >> 3);
        const int n = n0 + row;
        b_gc[j] = slot ^ ((row >> 1) & 7);
        b_ok[j] = n < a.Nout;
        b_ptr[j] = a.wt + (size_t)(b_ok[j] ? n : 0) * a.T * a.C;
    }
    typedef __attribute__((address_space(1))) const void* gptr_t;
    typedef __attribute__((address_space(3))) void* lptr_t;
    auto issue = [&](int kt, int buf) {
        if constexpr (UT) {
            // C >= 64: a 64-wide k-tile lies inside one tap -> ONE table read per tile
            const int k = kt * BK;
            const int te = __builtin_amdgcn_readfirstlane(tapt[k >> a.logC]);
            const int dh = ((te >> 8) & 0xff) - 128, dw = ((te >> 16) & 0xff) - 128;
            const int c0 = k & (a.C - 1);
            const int aoff = ((dh * a.Wi + dw) << a.logC) + c0;
            const int boff = (te & 0xff) * a.C + c0;
#pragma unroll
            for (int j = 0; j < AR; ++j) {
                const bool ok = (unsigned)(a_h[j] + dh) < (unsigned)a.Hi && (unsigned)(a_w[j] + dw) < (unsigned)a.Wi;
                const void* src = ok ? (const void*)(a_ptr[j] + aoff + a_gc[j] * 8) : (const void*)g_zero16;
                __builtin_amdgcn_global_load_lds((gptr_t)src, (lptr_t)(As + (buf * BM + (wave * AR + j) * 8) * 8),
                                                 16, 0, 0);
            }
#pragma unroll
            for (int j = 0; j < BR; ++j) {
                const void* src = b_ok[j] ? (const void*)(b_ptr[j] + boff + b_gc[j] * 8) : (const void*)g_zero16;
                __builtin_amdgcn_global_load_lds((gptr_t)src, (lptr_t)(Bs + (buf * BN + (wave * BR + j) * 8) * 8),
                                                 16, 0, 0);
            }
        } else {
#pragma unroll
            for (int j = 0; j < AR; ++j) {
                const int k = kt * BK + a_gc[j] * 8;
                const bool kin = k < Ktot;
                const int te = tapt[kin ? (k >> a.logC) : 0];
                const int c = k & (a.C - 1);
                const int dh = ((te >> 8) & 0xff) - 128, dw = ((te >> 16) & 0xff) - 128;
                const int hi = a_h[j] + dh, wi = a_w[j] + dw;
                const bool ok = kin && (unsigned)hi < (unsigned)a.Hi && (unsigned)wi < (unsigned)a.Wi;
                const void* src = ok ? (const void*)(a_ptr[j] + (((dh * a.Wi + dw) << a.logC) + c))
                                     : (const void*)g_zero16;
                __builtin_amdgcn_global_load_lds((gptr_t)src, (lptr_t)(As + (buf * BM + (wave * AR + j) * 8) * 8),
                                                 16, 0, 0);
            }
#pragma unroll
            for (int j = 0; j < BR; ++j) {
                const int k = kt * BK + b_gc[j] * 8;
                const bool kin = k < Ktot;
                const int te = tapt[kin ? (k >> a.logC) : 0];
                const int c = k & (a.C - 1);
                const void* src = (kin && b_ok[j]) ? (const void*)(b_ptr[j] + (te & 0xff) * a.C + c)
                                                   : (const void*)g_zero16;
                __builtin_amdgcn_global_load_lds((gptr_t)src, (lptr_t)(Bs + (buf * BN + (wave * BR + j) * 8) * 8),
                                                 16, 0, 0);
            }
        }
    };

    floatx16 acc[MT][NT];
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int j = 0; j < NT; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

    const int fr = lane & 31, fh = lane >> 5;
    auto compute = [&](int buf) {
#pragma unroll
        for (int ks = 0; ks < 4; ++ks) {
            const int chunk = ks * 2 + fh;
            bf16x8 af[MT], bfr[NT];
#pragma unroll
            for (int i = 0; i < MT; ++i) {
                const int row = wm * (BM / 2) + i * 32 + fr;
                af[i] = __builtin_bit_cast(bf16x8, As[(buf * BM + row) * 8 + swz(row, chunk)]);
            }
#pragma unroll
            for (int j = 0; j < NT; ++j) {
                const int row = wn * (BN / 2) + j * 32 + fr;
                bfr[j] = __builtin_bit_cast(bf16x8, Bs[(buf * BN + row) * 8 + swz(row, chunk)]);
            }
#pragma unroll
            for (int i = 0; i < MT; ++i)
#pragma unroll
                for (int j = 0; j < NT; ++j)
                    // weights as the MFMA A operand, pixels as B: D[n][m], so each lane ends
                    // up holding 4 consecutive output channels of ONE pixel per register group
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(bfr[j], af[i], acc[i][j], 0, 0, 0);
        }
    };
    if constexpr (ST == 2) {
        // 2 LDS buffers: the DMA of tile kt+1 runs under the MFMAs of tile kt; the barrier
        // at the end of each step (vmcnt(0) + s_barrier) publishes it.
        if (nk > 0) issue(0, 0);
        __syncthreads();
        for (int kt = 0; kt < nk; ++kt) {
            const int buf = kt & 1;
            if (kt + 1 < nk) issue(kt + 1, buf ^ 1);
            compute(buf);
            __syncthreads();
        }
    } else {
        // 3 LDS buffers, two k-tiles in flight: step kt waits only for ITS tile
        // (counted vmcnt leaves tile kt+1's G DMAs outstanding), one raw barrier per
        // step publishes it and retires the reads of buffer (kt-1)%3, which tile kt+2
        // then refills under this step's MFMAs.
        if (nk > 0) issue(0, 0);
        if (nk > 1) issue(1, 1);
        int buf = 0, nbuf = 2;
        for (int kt = 0; kt < nk; ++kt) {
            if (kt + 1 < nk)
                asm volatile("s_waitcnt vmcnt(%0)" ::"n"(G) : "memory");
            else
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_s_barrier();
            asm volatile("" ::: "memory");
            if (kt + 2 < nk) issue(kt + 2, nbuf);
            compute(buf);
            buf = buf == ST - 1 ? 0 : buf + 1;
            nbuf = nbuf == ST - 1 ? 0 : nbuf + 1;
        }
    }

    store_tile<MT, NT, BM, BN>(a, cl, m0, n0, wm, wn, fr, fh, M, acc);
}

// Lean variant for C >= 64 (a 64-wide k-tile lies inside one tap) and <= 32 taps:
//  * per-row tap validity precomputed as a bitmask (one bit test per DMA, no bounds math),
//  * wave index in an SGPR, so every LDS-DMA destination (M0) is scalar arithmetic,
//  * per-lane LDS fragment offsets precomputed and the k-loop unrolled by the two
//    buffers, so every ds_read_b128 is base VGPR + immediate (no address VALU),
//  * the tap-table entry of the next k-tile is read one step ahead.
// PIPE 0: two LDS stages, issue(k+1) -> compute(k) -> __syncthreads (vmcnt(0) drain).
// PIPE 2 / 3: an LDS ring of PIPE stages with ONE raw barrier per k-tile: wait with a
// counted vmcnt for tile k only (PIPE 3 leaves tile k+1's DMA in flight across the
// barrier), barrier, refill the stage compute(k-1) released, compute(k) with the next
// k-step's fragments read from LDS under the current k-step's MFMAs.
template <int BM, int BN, int PIPE>
__global__ __launch_bounds__(256) void k_conv_igemm_ut(ConvArgs a) {
    constexpr int BK = 64;
    constexpr int AR = BM / 32, BR = BN / 32;
    constexpr int MT = BM / 64, NT = BN / 64;
    constexpr int SA = BM * 128, SB = BN * 128;  // bytes per stage
    constexpr int NST = PIPE == 3 ? 3 : 2;      // LDS stages
    constexpr int G = AR + BR;                   // LDS-DMA instructions per wave per k-tile
    extern __shared__ __attribute__((aligned(16))) uint4 smem[];
    char* lds = reinterpret_cast<char*>(smem);   // [A0..A(NST-1)][B0..B(NST-1)]

    int bid = block_id(a.xcd);
    int split = 0;
    if (a.splits > 1) {
        split = bid / a.tiles_total;
        bid -= split * a.tiles_total;
    }
    const int tid = bid;  // launch-wide tile index: split-K slab and turnstile word
    int g = 0;            // view group
    if (a.G > 1) {
        g = bid / a.tiles_g;
        bid -= g * a.tiles_g;
    }
    const uint16_t* const gin = a.in + g * a.gs_in;
    const uint16_t* const gwt = a.wt + g * a.gs_wt;
    int ci = 0;
#pragma unroll
    for (int q = 1; q < kMaxCls; ++q)
        if (q < a.ncls && bid >= a.cls[q].tile_start) ci = q;
    const ConvCls& cl = a.cls[ci];
    const int wgid = bid - cl.tile_start;
    // tile order: with the XCD remap, tm fastest (an XCD's contiguous tile range shares a
    // weight slice); without it (split-K needs the dispatch order), tn fastest, so that
    // with a power-of-two column count the round-robin XCD dealing (block b on XCD b % 8)
    // keeps each weight slice on the same XCD(s) - L2-resident instead of re-fetched
    const int tiles_n = (a.Nout + BN - 1) / BN;
    const int tm = a.xcd ? wgid % cl.tiles_m : wgid / tiles_n;
    const int tn = a.xcd ? wgid / cl.tiles_m : wgid - tm * tiles_n;
    const int m0 = tm * BM, n0 = tn * BN;
    const int PQ = cl.P * cl.Q;
    const int M = a.N * PQ;
    const int nk_all = (cl.ntap * a.C) / BK;
    const int kt0 = split * nk_all / a.splits;
    const int nk = (split + 1) * nk_all / a.splits - kt0;

    const int t = threadIdx.x;
    const int lane = t & 63;
    const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
    const int wm = wave >> 1, wn = wave & 1;
    const int slot = lane & 7;
    // the class's tap grid, unpacked in SGPRs from 4-bit fields
    const unsigned pk_dh = cl.pk_dh, pk_dw = cl.pk_dw, pk_r = cl.pk_r, pk_s = cl.pk_s;

    // per A row: pixel base pointer and the tap validity as two bitmasks over the
    // grid's rows (bit i: h + cdh[i] in range) and columns (bit j: w + cdw[j] in range)
    const uint16_t* a_ptr[AR];
    unsigned a_vr[AR], a_vs[AR];
#pragma unroll
    for (int j = 0; j < AR; ++j) {
        const int row = (wave * AR + j) * 8 + (lane >> 3);
        const int m = m0 + row;
        const int gc = slot ^ ((row >> 1) & 7);
        const int b = (int)cl.fd_pq.div((uint32_t)m), pq = m - b * PQ;
        const int p = (int)cl.fd_q.div((uint32_t)pq), q = pq - p * cl.Q;
        const int h = p * a.sAh, w = q * a.sAw;
        // dh_i = dh_0 + sh*i with sh = +-1 (fwd: r - pad; dgrad class: (ph+pad-r)/st), so
        // the valid grid rows are one contiguous bit range [lo, hi]; same for columns
        const unsigned vr = span_mask(h, cl.dh0, cl.sh, cl.Rc, a.Hi);
        const unsigned vs = span_mask(w, cl.dw0, cl.sw, cl.Sc, a.Wi);
        const bool in = m < M;
        a_vr[j] = in ? vr : 0u;
        a_vs[j] = vs;
        a_ptr[j] = gin + (in ? ((size_t)((b * a.Hi + h) * a.Wi + w) << a.logC) : 0) + gc * 8;
    }
    const uint16_t* b_ptr[BR];
    bool b_ok[BR];
#pragma unroll
    for (int j = 0; j < BR; ++j) {
        const int row = (wave * BR + j) * 8 + (lane >> 3);
        const int n = n0 + row;
        const int gc = slot ^ ((row >> 1) & 7);
        b_ok[j] = n < a.Nout;
        b_ptr[j] = gwt + (size_t)(b_ok[j] ? n : 0) * a.T * a.C + gc * 8;
    }
    // per-lane fragment byte offsets inside a stage: row*128 + swizzled 16-B chunk
    const int fr = lane & 31, fh = lane >> 5;
    int a_rd[MT][4], b_rd[NT][4];
#pragma unroll
    for (int i = 0; i < MT; ++i) {
        const int row = wm * (BM / 2) + i * 32 + fr;
#pragma unroll
        for (int ks = 0; ks < 4; ++ks) a_rd[i][ks] = row * 128 + (swz(row, ks * 2 + fh) << 4);
    }
#pragma unroll
    for (int j = 0; j < NT; ++j) {
        const int row = wn * (BN / 2) + j * 32 + fr;
#pragma unroll
        for (int ks = 0; ks < 4; ++ks) b_rd[j][ks] = NST * SA + row * 128 + (swz(row, ks * 2 + fh) << 4);
    }

    typedef __attribute__((address_space(1))) const void* gptr_t;
    typedef __attribute__((address_space(3))) void* lptr_t;
    auto issue = [&](int kt, int buf) {
        const int k = (kt0 + kt) * BK;
        const int tap = __builtin_amdgcn_readfirstlane(k >> a.logC);
        const int ti = (tap * cl.smag) >> 8, tj = tap - ti * cl.Sc;
        const int dh = (int)((pk_dh >> (4 * ti)) & 15u) - 8, dw = (int)((pk_dw >> (4 * tj)) & 15u) - 8;
        const int tw = (int)((pk_r >> (4 * ti)) & 15u) * a.Sw + (int)((pk_s >> (4 * tj)) & 15u);
        const int c0 = k & (a.C - 1);
        const long aoff = (long)(((dh * a.Wi + dw) << a.logC) + c0);
        const long boff = (long)(tw * a.C + c0);
#pragma unroll
        for (int j = 0; j < AR; ++j) {
            const bool ok = ((a_vr[j] >> ti) & (a_vs[j] >> tj)) & 1u;
            const void* src = ok ? (const void*)(a_ptr[j] + aoff) : (const void*)g_zero16;
            __builtin_amdgcn_global_load_lds((gptr_t)src, (lptr_t)(lds + buf * SA + (wave * AR + j) * 1024), 16, 0,
                                             0);
        }
#pragma unroll
        for (int j = 0; j < BR; ++j) {
            const void* src = b_ok[j] ? (const void*)(b_ptr[j] + boff) : (const void*)g_zero16;
            __builtin_amdgcn_global_load_lds((gptr_t)src,
                                             (lptr_t)(lds + NST * SA + buf * SB + (wave * BR + j) * 1024), 16, 0, 0);
        }
    };

    floatx16 acc[MT][NT];
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int j = 0; j < NT; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
    auto compute = [&](int buf) {
#pragma unroll
        for (int ks = 0; ks < 4; ++ks) {
            bf16x8 af[MT], bfr[NT];
#pragma unroll
            for (int i = 0; i < MT; ++i)
                af[i] = *reinterpret_cast<const bf16x8*>(lds + buf * SA + a_rd[i][ks]);
#pragma unroll
            for (int j = 0; j < NT; ++j)
                bfr[j] = *reinterpret_cast<const bf16x8*>(lds + buf * SB + b_rd[j][ks]);
#pragma unroll
            for (int i = 0; i < MT; ++i)
#pragma unroll
                for (int j = 0; j < NT; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(bfr[j], af[i], acc[i][j], 0, 0, 0);
        }
    };
    if constexpr (PIPE == 0) {
        issue(0, 0);
        __syncthreads();
        int kt = 0;
        for (; kt + 1 < nk; kt += 2) {  // tiles kt (buffer 0) and kt+1 (buffer 1)
            issue(kt + 1, 1);
            compute(0);
            __syncthreads();
            if (kt + 2 < nk) issue(kt + 2, 0);
            compute(1);
            __syncthreads();
        }
        if (kt < nk) compute(0);  // odd tile count: the last tile sits in buffer 0
    } else {
        // fragments of k-step ks+1 are read while k-step ks's MFMAs run
        auto compute_pf = [&](int buf) {
            bf16x8 af[2][MT], bfr[2][NT];
#pragma unroll
            for (int i = 0; i < MT; ++i) af[0][i] = *reinterpret_cast<const bf16x8*>(lds + buf * SA + a_rd[i][0]);
#pragma unroll
            for (int j = 0; j < NT; ++j) bfr[0][j] = *reinterpret_cast<const bf16x8*>(lds + buf * SB + b_rd[j][0]);
#pragma unroll
            for (int ks = 0; ks < 4; ++ks) {
                const int c = ks & 1;
                if (ks < 3) {
#pragma unroll
                    for (int i = 0; i < MT; ++i)
                        af[c ^ 1][i] = *reinterpret_cast<const bf16x8*>(lds + buf * SA + a_rd[i][ks + 1]);
#pragma unroll
                    for (int j = 0; j < NT; ++j)
                        bfr[c ^ 1][j] = *reinterpret_cast<const bf16x8*>(lds + buf * SB + b_rd[j][ks + 1]);
                }
#pragma unroll
                for (int i = 0; i < MT; ++i)
#pragma unroll
                    for (int j = 0; j < NT; ++j)
                        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(bfr[c][j], af[c][i], acc[i][j], 0, 0, 0);
            }
            // emitted order: k-step ks + 1's reads BEFORE k-step ks's MFMAs, so they stay in
            // flight under the matrix pipe.  (Threading them between the MFMAs, one read per
            // MFMA, issued each k-step's last read after its MFMAs into a register an MFMA had
            // just released, and the lgkmcnt(0) the compiler put before the next MFMAs then
            // exposed that read's whole LDS latency once per k-step.)
            constexpr int NR = MT + NT, NM = MT * NT;
            __builtin_amdgcn_sched_group_barrier(0x100, NR, 0);
#pragma unroll
            for (int ks = 0; ks < 3; ++ks) {
                __builtin_amdgcn_sched_group_barrier(0x100, NR, 0);
                __builtin_amdgcn_sched_group_barrier(0x008, NM, 0);
            }
            __builtin_amdgcn_sched_group_barrier(0x008, NM, 0);
        };
        // s_waitcnt immediates (gfx9 encoding: vmcnt[3:0] + [15:14], expcnt[6:4], lgkmcnt[11:8])
        constexpr int kWaitTile = (G & 15) | (7 << 4) | (15 << 8) | (((G >> 4) & 3) << 14);  // vmcnt(G)
        constexpr int kWaitAll = (7 << 4) | (15 << 8);                                       // vmcnt(0)
        issue(0, 0);
        if (NST == 3 && nk > 1) issue(1, 1);
        int s = 0;  // stage of tile kt
        for (int kt = 0; kt < nk; ++kt) {
            if (NST == 3 && kt + 1 < nk) __builtin_amdgcn_s_waitcnt(kWaitTile);  // tile kt+1 stays in flight
            else __builtin_amdgcn_s_waitcnt(kWaitAll);
            __builtin_amdgcn_s_barrier();
            if (kt + NST - 1 < nk) {
                int sn = s + NST - 1;
                if (sn >= NST) sn -= NST;
                issue(kt + NST - 1, sn);
            }
            compute_pf(s);
            if (++s == NST) s = 0;
        }
    }

    if (a.splits > 1) {
        constexpr int NQ = MT * NT * 4;  // float4 groups of accumulators per lane
        const auto rs = rsrc_of(a.ws + (size_t)tid * NQ * 256 * 4);
        if (split > 0) {  // wait for the previous split's running sum, then add it
            __shared__ int late;
            if (t == 0) {  // bounded: a broken hand-off never hangs, it faults loudly
                unsigned n = 0;
                bool ok = true;
                while (__hip_atomic_load(a.flags + tid, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) !=
                       (unsigned)split) {
                    if (++n >= a.spin_limit) {
                        ok = false;
                        break;
                    }
                    __builtin_amdgcn_s_sleep(2);
                }
                if (!ok) atomicOr(&g_conv_fault, GM_FAULT_SPLITK_SPIN);
                late = ok ? 0 : 1;
            }
            __syncthreads();
            if (late) {  // poison: the running sum was not handed over (the fault word is set)
#pragma unroll
                for (int i = 0; i < MT; ++i)
#pragma unroll
                    for (int j = 0; j < NT; ++j)
#pragma unroll
                        for (int r = 0; r < 16; ++r) acc[i][j][r] = __builtin_nanf("");
            }
#pragma unroll
            for (int i = 0; i < MT; ++i)
#pragma unroll
                for (int j = 0; j < NT; ++j)
#pragma unroll
                    for (int g = 0; g < 4; ++g) {
                        const float4 v = ld_sc1_f32x4(rs, (unsigned)((((i * NT + j) * 4 + g) * 256 + t) * 16));
                        acc[i][j][4 * g] += v.x;
                        acc[i][j][4 * g + 1] += v.y;
                        acc[i][j][4 * g + 2] += v.z;
                        acc[i][j][4 * g + 3] += v.w;
                    }
        }
        if (split < a.splits - 1) {  // publish the running sum to the next split
#pragma unroll
            for (int i = 0; i < MT; ++i)
#pragma unroll
                for (int j = 0; j < NT; ++j)
#pragma unroll
                    for (int g = 0; g < 4; ++g)
                        st_sc1_f32x4(rs, (unsigned)((((i * NT + j) * 4 + g) * 256 + t) * 16),
                                     make_float4(acc[i][j][4 * g], acc[i][j][4 * g + 1], acc[i][j][4 * g + 2],
                                                 acc[i][j][4 * g + 3]));
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
            if (t == 0) __hip_atomic_store(a.flags + tid, (unsigned)(split + 1), __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT);
            return;
        }
        if (t == 0) __hip_atomic_store(a.flags + tid, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }

    store_tile_lds<MT, NT, BM, BN>(a, cl, m0, n0, wm, wn, fr, fh, M, acc, g * a.gs_out, lds, NST * (SA + SB), t, g);
}

// ---------------------------------------------------------------------------------
// 3x3 / stride-1 / pad-1 convolutions (the ResNet trunk's 13 main convolutions per view
// and their stride-1 input gradients) with the A operand staged ONCE per 64-channel
// chunk as a halo instead of once per tap (implicit-GEMM im2col re-stages every input
// pixel 9 times).  The lean kernel above is bound by the per-CU LDS-DMA rate
// (~26 B/clk/CU measured: tools/conv_ab.py diagnostics), so bytes staged per FLOP is
// the lever: per 64-deep k-tile the A stage shrinks from 16 KB to (halo / 9) ~3-6 KB.
//
// Geometry.  An M tile is 128 consecutive output pixels (b, p, q) of the flat
// N*H*W order (it may span rows and images).  Input rows live in a "padded row" space:
// image b's row h is padded row b*(H+1) + 1 + h, and padded rows b*(H+1) are zero rows
// (one between consecutive images, one after the last), columns are padded by one zero
// column each side.  Output (b, p, q) with tap offset (dh, dw) in [-1, 1]^2 reads halo
// pixel ((b*(H+1) + 1 + p + dh) - pr0) * (W+2) + (1 + q + dw), pr0 the tile's first
// padded row - so every tap reads in-range LDS and padding is real zeros (DMA'd from a
// zero vector), with no per-lane predicates.  Halo pixels are 128-B LDS rows (64
// channels) with the 16-B chunk XOR-swizzled by ((pixel >> 1) & 7), applied on the DMA
// source as everywhere in this file.
//
// Schedule: k-tiles run chunk-major, tap-minor (k = chunk * 9 + tap); the halo of a
// chunk is loaded at the chunk's first k-tile (one buffer; the other co-resident
// workgroup of the CU hides that stall), the B operand (weights) through the usual
// 2-stage ring with one barrier per k-tile.  Epilogue and split-K turnstile as in the
// lean kernel.
// s_barrier that is also a compiler memory barrier: without the fences the scheduler may
// move an LDS access of the next tile above the raw barrier (it is not a memory fence)
__device__ __forceinline__ void lds_barrier() {
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}

// LDS fragment read as inline asm (k_conv_rw, k_conv_stem): hipcc does not see these as
// LDS accesses, so it neither drains the LDS-DMA in flight before them nor counts them;
// the kernels wait for them explicitly (lgkmcnt(0) tied to the fragments about to be used)
template <int OFF>
__device__ __forceinline__ bf16x8 lds_rd128(unsigned addr) {
    bf16x8 d;
    asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(d) : "v"(addr), "i"(OFF));
    return d;
}

struct HaloArgs {
    int halo_bytes;           // LDS bytes of the halo region (multiple of 1 KB)
    FastDiv fd_w2, fd_h1;     // W + 2, H + 1
};

// BM = 256 (one workgroup per CU): the weight bytes staged per FLOP - the binding
// LDS-DMA traffic of the BM = 128 form - halve; the halo is double-buffered and the
// next chunk's halo is DMA'd in pieces under the current chunk's first eight k-tiles
// (the BM = 128 form relies on its co-resident second workgroup to hide that load).
template <int BM, int BN, int NB>
__global__ __launch_bounds__(BM == 256 ? 512 : 256) void k_conv_halo(ConvArgs a, HaloArgs h) {
    constexpr int BK = 64;  // NB: stages of the weight (B) ring, 2 or 3
    constexpr bool kHB2 = BM == 256;  // double-buffered halo, prefetched in pieces
    constexpr int NW = BM == 256 ? 8 : 4;  // waves: (NW/2) x 2, each a 64x64 sub-tile
    constexpr int NT_ = NW * 64;           // threads
    constexpr int BR = BN / (8 * NW);      // B-stage DMA instructions per wave
    constexpr int MT = 2, NT = BN / 64;
    constexpr int SB = BN * 128;
    extern __shared__ __attribute__((aligned(16))) uint4 smem[];
    char* lds = reinterpret_cast<char*>(smem);  // [halo (x2 when kHB2)][B0][B1]([B2])
    const int HB = h.halo_bytes;
    const int BOFF = kHB2 ? 2 * HB : HB;  // start of the B ring

    int bid = blockIdx.x;
    int split = 0;
    if (a.splits > 1) {
        split = bid / a.tiles_total;
        bid -= split * a.tiles_total;
    }
    const ConvCls& cl = a.cls[0];
    // tn fastest: blocks are dealt round-robin over the 8 XCDs (b on XCD b % 8), so with a
    // power-of-two column count each XCD's blocks share one weight slice (L2-resident)
    const int tiles_n = (a.Nout + BN - 1) / BN;
    const int tm = bid / tiles_n, tn = bid - tm * tiles_n;
    const int m0 = tm * BM, n0 = tn * BN;
    const int H = a.Hi, W = a.Wi, W2 = W + 2, H1 = H + 1;
    const int PQ = cl.P * cl.Q;  // == H * W (stride 1, same size)
    const int M = a.N * PQ;
    const int nk_all = 9 * (a.C >> 6);
    const int kt0 = split * nk_all / a.splits;
    const int nk = (split + 1) * nk_all / a.splits - kt0;

    const int t = threadIdx.x;
    const int lane = t & 63;
    const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
    const int wm = wave >> 1, wn = wave & 1;
    const int slot = lane & 7;
    const unsigned pk_dh = cl.pk_dh, pk_dw = cl.pk_dw, pk_r = cl.pk_r, pk_s = cl.pk_s;

    // tile's padded row range
    int pr0, npix;
    {
        const int b0 = (int)cl.fd_pq.div((uint32_t)m0), q0 = m0 - b0 * PQ;
        const int p0 = (int)cl.fd_q.div((uint32_t)q0);
        const int m1 = min(m0 + BM, M) - 1;
        const int b1 = (int)cl.fd_pq.div((uint32_t)m1), q1 = m1 - b1 * PQ;
        const int p1 = (int)cl.fd_q.div((uint32_t)q1);
        pr0 = b0 * H1 + p0;
        npix = (b1 * H1 + p1 + 2 - pr0 + 1) * W2;
    }
    pr0 = __builtin_amdgcn_readfirstlane(pr0);
    npix = __builtin_amdgcn_readfirstlane(npix);
    const int nI = (npix + 7) >> 3;  // halo DMA instructions of the workgroup

    // A fragments: per MFMA row block i the lane's output pixel's halo index (tap 0,0)
    const int fr = lane & 31, fh = lane >> 5;
    int hbase[MT];
#pragma unroll
    for (int i = 0; i < MT; ++i) {
        int m = m0 + wm * (MT * 32) + i * 32 + fr;
        m = m < M ? m : m0;  // rows past M read a valid pixel; their outputs are not stored
        const int b = (int)cl.fd_pq.div((uint32_t)m), pq = m - b * PQ;
        const int p = (int)cl.fd_q.div((uint32_t)pq), q = pq - p * cl.Q;
        hbase[i] = (b * H1 + 1 + p - pr0) * W2 + 1 + q;
    }
    // B rows (weights [Nout][9][C])
    const uint16_t* b_ptr[BR];
    bool b_ok[BR];
#pragma unroll
    for (int j = 0; j < BR; ++j) {
        const int row = (wave * BR + j) * 8 + (lane >> 3);
        const int n = n0 + row;
        const int gc = slot ^ ((row >> 1) & 7);
        b_ok[j] = n < a.Nout;
        b_ptr[j] = a.wt + (size_t)(b_ok[j] ? n : 0) * a.T * a.C + gc * 8;
    }
    int b_rd[NT][4];
#pragma unroll
    for (int j = 0; j < NT; ++j) {
        const int row = wn * (BN / 2) + j * 32 + fr;
#pragma unroll
        for (int ks = 0; ks < 4; ++ks) b_rd[j][ks] = BOFF + row * 128 + (swz(row, ks * 2 + fh) << 4);
    }

    typedef __attribute__((address_space(1))) const void* gptr_t;
    typedef __attribute__((address_space(3))) void* lptr_t;
    // the halo of channel chunk cc: instructions I = wave, wave+4, ... of nI, 8 pixels each
    // (instructions [I0, I1) only, into halo buffer hb)
    auto issue_halo_part = [&](int cc, int hb, int I0, int I1) {
        const int cbase = cc << 6;
        char* dst = lds + hb * HB;
        for (int I = I0 + wave; I < I1; I += NW) {
            const int hp = I * 8 + (lane >> 3);
            const void* src = (const void*)g_zero16;
            if (hp < npix) {
                const int r = (int)h.fd_w2.div((uint32_t)hp), c = hp - r * W2;
                const int pr = pr0 + r;
                const int b = (int)h.fd_h1.div((uint32_t)pr), rr = pr - b * H1;
                if (rr != 0 && c != 0 && c != W + 1 && b < a.N) {
                    const int gc = slot ^ ((hp >> 1) & 7);
                    src = (const void*)(a.in + ((size_t)((b * H + rr - 1) * W + c - 1) << a.logC) + cbase + gc * 8);
                }
            }
            __builtin_amdgcn_global_load_lds((gptr_t)src, (lptr_t)(dst + I * 1024), 16, 0, 0);
        }
    };
    auto issue_halo = [&](int cc) { issue_halo_part(cc, kHB2 ? (cc & 1) : 0, 0, nI); };
    // the kHB2 prefetch: piece tp (0..7) of the next chunk's halo, NW instructions a
    // multiple so every wave issues whole rounds
    const int nIp = (nI + 8 * NW - 1) / (8 * NW) * NW;  // instructions per piece
    auto issue_b = [&](int kt, int buf) {
        const int k = kt0 + kt;
        const int cc = k / 9, tp = k - cc * 9;
        const int ti = tp / 3, tj = tp - ti * 3;
        const int tw = (int)((pk_r >> (4 * ti)) & 15u) * a.Sw + (int)((pk_s >> (4 * tj)) & 15u);
        const long boff = (long)(tw * a.C + (cc << 6));
#pragma unroll
        for (int j = 0; j < BR; ++j) {
            const void* src = b_ok[j] ? (const void*)(b_ptr[j] + boff) : (const void*)g_zero16;
            __builtin_amdgcn_global_load_lds((gptr_t)src, (lptr_t)(lds + BOFF + buf * SB + (wave * BR + j) * 1024), 16,
                                             0, 0);
        }
    };

    floatx16 acc[MT][NT];
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int j = 0; j < NT; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

    auto compute = [&](int buf, int toff, int hoff) {
        int abase[MT];
#pragma unroll
        for (int i = 0; i < MT; ++i) {
            const int hp = hbase[i] + toff;
            abase[i] = hoff + ((hp << 7) | ((((hp >> 1) & 7) ^ fh) << 4));  // chunk (2ks+fh)^swz = this ^ (ks<<5)
        }
        bf16x8 af[2][MT], bfr[2][NT];
#pragma unroll
        for (int i = 0; i < MT; ++i) af[0][i] = *reinterpret_cast<const bf16x8*>(lds + abase[i]);
#pragma unroll
        for (int j = 0; j < NT; ++j) bfr[0][j] = *reinterpret_cast<const bf16x8*>(lds + buf * SB + b_rd[j][0]);
#pragma unroll
        for (int ks = 0; ks < 4; ++ks) {
            const int c = ks & 1;
            if (ks < 3) {
#pragma unroll
                for (int i = 0; i < MT; ++i)
                    af[c ^ 1][i] = *reinterpret_cast<const bf16x8*>(lds + (abase[i] ^ ((ks + 1) << 5)));
#pragma unroll
                for (int j = 0; j < NT; ++j)
                    bfr[c ^ 1][j] = *reinterpret_cast<const bf16x8*>(lds + buf * SB + b_rd[j][ks + 1]);
            }
#pragma unroll
            for (int i = 0; i < MT; ++i)
#pragma unroll
                for (int j = 0; j < NT; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(bfr[c][j], af[c][i], acc[i][j], 0, 0, 0);
        }
        constexpr int NR = MT + NT, NM = MT * NT;  // next k-step's reads before these MFMAs
        __builtin_amdgcn_sched_group_barrier(0x100, NR, 0);
#pragma unroll
        for (int ks = 0; ks < 3; ++ks) {
            __builtin_amdgcn_sched_group_barrier(0x100, NR, 0);
            __builtin_amdgcn_sched_group_barrier(0x008, NM, 0);
        }
        __builtin_amdgcn_sched_group_barrier(0x008, NM, 0);
    };

    constexpr int kWaitAll = (7 << 4) | (15 << 8);  // s_waitcnt vmcnt(0)
    issue_halo(kt0 / 9);
    issue_b(0, 0);
    if (NB == 3 && nk > 1) issue_b(1, 1);
    constexpr int kWaitB = (BR & 15) | (7 << 4) | (15 << 8);  // vmcnt(BR): the newest B stage stays in flight
    int sb = 0;  // B stage of k-tile kt
    for (int kt = 0; kt < nk; ++kt) {
        const int k = kt0 + kt;
        const int tp = k % 9;
        if (NB == 3 && kt + 1 < nk) __builtin_amdgcn_s_waitcnt(kWaitB);
        else __builtin_amdgcn_s_waitcnt(kWaitAll);
        __builtin_amdgcn_s_barrier();
        if (!kHB2 && kt > 0 && tp == 0) {  // next channel chunk: every wave is done with the old halo
            issue_halo(k / 9);
            __builtin_amdgcn_s_waitcnt(kWaitAll);
            __builtin_amdgcn_s_barrier();
        }
        // kHB2: the next chunk's halo goes to the other buffer (last read by the previous
        // chunk, whose k-tiles every wave has passed at this barrier), issued before this
        // k-tile's B stage so the counted B waits stay valid, landed by the chunk's first wait
        if (kHB2 && kt - tp + 9 < nk) {
            // pieces [lo, hi): a split that starts mid-chunk issues the pieces it skipped
            const int lo = kt == 0 ? 0 : tp, hi = tp < 8 ? tp + 1 : 8;
            const int cn = k / 9 + 1;
            if (lo < hi) issue_halo_part(cn, cn & 1, lo * nIp, min(hi * nIp, nI));
        }
        if (kt + NB - 1 < nk) {
            int sn = sb + NB - 1;
            if (sn >= NB) sn -= NB;
            issue_b(kt + NB - 1, sn);
        }
        const int ti = tp / 3, tj = tp - ti * 3;
        const int dh = (int)((pk_dh >> (4 * ti)) & 15u) - 8, dw = (int)((pk_dw >> (4 * tj)) & 15u) - 8;
        compute(sb, dh * W2 + dw, kHB2 ? ((k / 9) & 1) * HB : 0);
        if (++sb == NB) sb = 0;
    }

    if (a.splits > 1) {
        constexpr int NQ = MT * NT * 4;  // float4 groups of accumulators per lane
        const auto rs = rsrc_of(a.ws + (size_t)bid * NQ * NT_ * 4);
        if (split > 0) {  // wait for the previous split's running sum, then add it
            __shared__ int late;
            if (t == 0) {  // bounded: a broken hand-off never hangs, it faults loudly
                unsigned n = 0;
                bool ok = true;
                while (__hip_atomic_load(a.flags + bid, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) !=
                       (unsigned)split) {
                    if (++n >= a.spin_limit) {
                        ok = false;
                        break;
                    }
                    __builtin_amdgcn_s_sleep(2);
                }
                if (!ok) atomicOr(&g_conv_fault, GM_FAULT_SPLITK_SPIN);
                late = ok ? 0 : 1;
            }
            __syncthreads();
            if (late) {  // poison: the running sum was not handed over (the fault word is set)
#pragma unroll
                for (int i = 0; i < MT; ++i)
#pragma unroll
                    for (int j = 0; j < NT; ++j)
#pragma unroll
                        for (int r = 0; r < 16; ++r) acc[i][j][r] = __builtin_nanf("");
            }
#pragma unroll
            for (int i = 0; i < MT; ++i)
#pragma unroll
                for (int j = 0; j < NT; ++j)
#pragma unroll
                    for (int g = 0; g < 4; ++g) {
                        const float4 v = ld_sc1_f32x4(rs, (unsigned)((((i * NT + j) * 4 + g) * NT_ + t) * 16));
                        acc[i][j][4 * g] += v.x;
                        acc[i][j][4 * g + 1] += v.y;
                        acc[i][j][4 * g + 2] += v.z;
                        acc[i][j][4 * g + 3] += v.w;
                    }
        }
        if (split < a.splits - 1) {  // publish the running sum to the next split
#pragma unroll
            for (int i = 0; i < MT; ++i)
#pragma unroll
                for (int j = 0; j < NT; ++j)
#pragma unroll
                    for (int g = 0; g < 4; ++g)
                        st_sc1_f32x4(rs, (unsigned)((((i * NT + j) * 4 + g) * NT_ + t) * 16),
                                     make_float4(acc[i][j][4 * g], acc[i][j][4 * g + 1], acc[i][j][4 * g + 2],
                                                 acc[i][j][4 * g + 3]));
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
            if (t == 0) __hip_atomic_store(a.flags + bid, (unsigned)(split + 1), __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT);
            return;
        }
        if (t == 0) __hip_atomic_store(a.flags + bid, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }

    // (BM = 256: two 128-row halves of wave rows 0-1 and 2-3)
    store_tile<MT, NT, 128, BN>(a, cl, m0 + (wm >> 1) * 128, n0, wm & 1, wn, fr, fh, M, acc);
}

// ---------------------------------------------------------------------------------
// k_conv_h9: the halo-staged 3x3 / stride-1 convolution (forward and stride-1 input
// gradient, C a multiple of 64) with its nine taps UNROLLED.  k_conv_halo decodes the
// tap of every k-tile at run time (k / 9, tap / 3, packed-field shifts, the ring stage
// modulo, per-DMA pointer selects): ~45 scalar and ~40 vector instructions per 16 MFMAs
// per wave, which at two waves per SIMD issue-bind the loop (ISA census, round 3).  Here
// the k-loop runs over 64-channel chunks with the nine taps as compile-time steps, so
//   * the weight-ring stage of a tap is tap % 3 (nine is a multiple of the ring depth):
//     the B fragment addresses are precomputed lane offsets + an immediate;
//   * each tap's halo offset and weight tap index are decoded ONCE per workgroup (the A
//     fragment address of tap t / fragment i is a precomputed VGPR);
//   * the halo pixel decode (two fast divides per DMA instruction) is done once per tile,
//     not once per channel chunk; chunks only add their channel base;
//   * weights are DMA'd without per-lane bounds selects (Nout % BN == 0 is required).
// Split-K splits whole channel chunks (splits <= C / 64) and hands the fp32 running sum
// on through the same turnstile as k_conv_halo.  One workgroup = 128 output pixels x BN
// channels, 4 waves of 64x64 (v_mfma_f32_32x32x16_bf16), two workgroups per CU.
constexpr int kH9MaxQ = 12;  // halo DMA instructions per wave (nI <= 48)

// NB: weight-ring stages (NB - 2 stay in flight across a k-tile).  Weights and halo both by
// LDS-DMA.  Measured and dropped (r03-r04): register-staged weights, a register prefetch of
// the next chunk's halo, weight pieces spread between the k-slices' MFMAs (0.05-0.07 ms/step
// slower or neutral).
template <int BN, int NB>
__global__ __launch_bounds__(256, 2) void k_conv_h9(ConvArgs a, HaloArgs h) {
    constexpr int BM = 128, MT = 2, NT = BN / 64, NW = 4;
    static_assert(NB >= 2 && NB <= 8, "ring depth");
    constexpr int BR = BN / (8 * NW);  // weight DMA instructions per wave per k-tile
    constexpr int SB = BN * 128;       // bytes of one ring stage
    extern __shared__ __attribute__((aligned(16))) uint4 smem[];
    char* lds = reinterpret_cast<char*>(smem);  // [halo][B0]..[B(NB-1)]
    const int HB = h.halo_bytes;

    int bid = blockIdx.x;
    int split = 0;
    if (a.splits > 1) {
        split = bid / a.tiles_total;
        bid -= split * a.tiles_total;
    }
    const int tid = bid;  // launch-wide tile index: split-K slab and turnstile word
    int g = 0;            // view group
    if (a.G > 1) {
        g = bid / a.tiles_g;
        bid -= g * a.tiles_g;
    }
    const uint16_t* const gin = a.in + g * a.gs_in;
    const uint16_t* const gwt = a.wt + g * a.gs_wt;
    const ConvCls& cl = a.cls[0];
    const int tiles_n = a.Nout / BN;
    const int tm = bid / tiles_n, tn = bid - tm * tiles_n;
    const int m0 = tm * BM, n0 = tn * BN;
    const int H = a.Hi, W = a.Wi, W2 = W + 2, H1 = H + 1;
    const int PQ = cl.P * cl.Q;
    const int M = a.N * PQ;
    const int nch = a.C >> 6;
    const int c0 = split * nch / a.splits, c1 = (split + 1) * nch / a.splits;

    const int t = threadIdx.x;
    const int lane = t & 63;
    const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
    const int wm = wave >> 1, wn = wave & 1;
    const int slot = lane & 7;
    const int fr = lane & 31, fh = lane >> 5;

    // the tile's padded halo rows
    int pr0, npix;
    {
        const int b0 = (int)cl.fd_pq.div((uint32_t)m0), q0 = m0 - b0 * PQ;
        const int p0 = (int)cl.fd_q.div((uint32_t)q0);
        const int m1 = min(m0 + BM, M) - 1;
        const int b1 = (int)cl.fd_pq.div((uint32_t)m1), q1 = m1 - b1 * PQ;
        const int p1 = (int)cl.fd_q.div((uint32_t)q1);
        pr0 = b0 * H1 + p0;
        npix = (b1 * H1 + p1 + 2 - pr0 + 1) * W2;
    }
    pr0 = __builtin_amdgcn_readfirstlane(pr0);
    npix = __builtin_amdgcn_readfirstlane(npix);
    const int nI = (npix + 7) >> 3;
    const int nq = (nI - wave + NW - 1) / NW;  // this wave's halo instructions

    // per-tap halo offset and weight tap (uniform), decoded once
    int toff[9], twc[9];
#pragma unroll
    for (int tp = 0; tp < 9; ++tp) {
        const int ti = tp / 3, tj = tp % 3;
        const int dh = (int)((cl.pk_dh >> (4 * ti)) & 15u) - 8, dw = (int)((cl.pk_dw >> (4 * tj)) & 15u) - 8;
        toff[tp] = __builtin_amdgcn_readfirstlane(dh * W2 + dw);
        const int tw = (int)((cl.pk_r >> (4 * ti)) & 15u) * a.Sw + (int)((cl.pk_s >> (4 * tj)) & 15u);
        twc[tp] = __builtin_amdgcn_readfirstlane(tw * a.C);
    }
    // A fragment addresses (ks = 0) per tap and row block: chunk (2ks+fh) ^ swz(pixel)
    int aad[9][MT];
#pragma unroll
    for (int i = 0; i < MT; ++i) {
        int m = m0 + wm * (MT * 32) + i * 32 + fr;
        m = m < M ? m : m0;  // rows past M read a valid pixel; their outputs are not stored
        const int b = (int)cl.fd_pq.div((uint32_t)m), pq = m - b * PQ;
        const int p = (int)cl.fd_q.div((uint32_t)pq), q = pq - p * cl.Q;
        const int hb = (b * H1 + 1 + p - pr0) * W2 + 1 + q;
#pragma unroll
        for (int tp = 0; tp < 9; ++tp) {
            const int hp = hb + toff[tp];
            aad[tp][i] = (hp << 7) | ((((hp >> 1) & 7) ^ fh) << 4);
        }
    }
    // B: weight rows of this wave's DMA instructions ([Nout][9][C]), source-swizzled
    const uint16_t* b_src[BR];
#pragma unroll
    for (int j = 0; j < BR; ++j) {
        const int row = (wave * BR + j) * 8 + (lane >> 3);
        b_src[j] = gwt + (size_t)(n0 + row) * a.T * a.C + ((slot ^ ((row >> 1) & 7)) << 3);
    }
    int b_rd[NT][4];
#pragma unroll
    for (int j = 0; j < NT; ++j) {
        const int row = wn * (BN / 2) + j * 32 + fr;
#pragma unroll
        for (int ks = 0; ks < 4; ++ks) b_rd[j][ks] = HB + row * 128 + (swz(row, ks * 2 + fh) << 4);
    }
    // halo sources of this wave's DMA instructions: channel-0 element offset or -1 (zero)
    int hsrc[kH9MaxQ];
#pragma unroll
    for (int q = 0; q < kH9MaxQ; ++q) {
        hsrc[q] = -1;
        const int hp = (wave + NW * q) * 8 + (lane >> 3);
        if (q < nq && hp < npix) {
            const int r = (int)h.fd_w2.div((uint32_t)hp), c = hp - r * W2;
            const int pr = pr0 + r;
            const int b = (int)h.fd_h1.div((uint32_t)pr), rr = pr - b * H1;
            if (rr != 0 && c != 0 && c != W + 1 && b < a.N)
                hsrc[q] = (((b * H + rr - 1) * W + c - 1) << a.logC) + ((slot ^ ((hp >> 1) & 7)) << 3);
        }
    }

    typedef __attribute__((address_space(1))) const void* gptr_t;
    typedef __attribute__((address_space(3))) void* lptr_t;
    auto issue_halo = [&](int cc) {
        const int cbase = cc << 6;
#pragma unroll
        for (int q = 0; q < kH9MaxQ; ++q) {
            if (q < nq) {
                const void* src = hsrc[q] >= 0 ? (const void*)(gin + hsrc[q] + cbase) : (const void*)g_zero16;
                __builtin_amdgcn_global_load_lds((gptr_t)src, (lptr_t)(lds + (wave + NW * q) * 1024), 16, 0, 0);
            }
        }
    };
    // k-tile (chunk cc, tap tp) -> ring stage st
    auto issue_b = [&](int cc, int tp, int st) {
        const int off = twc[tp] + (cc << 6);
#pragma unroll
        for (int j = 0; j < BR; ++j)
            __builtin_amdgcn_global_load_lds((gptr_t)(b_src[j] + off),
                                             (lptr_t)(lds + HB + st * SB + (wave * BR + j) * 1024), 16, 0, 0);
    };

    floatx16 acc[MT][NT];
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int j = 0; j < NT; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

    auto compute = [&](int tp, int st) {
        bf16x8 af[2][MT], bfr[2][NT];
#pragma unroll
        for (int i = 0; i < MT; ++i) af[0][i] = *reinterpret_cast<const bf16x8*>(lds + aad[tp][i]);
#pragma unroll
        for (int j = 0; j < NT; ++j) bfr[0][j] = *reinterpret_cast<const bf16x8*>(lds + st * SB + b_rd[j][0]);
#pragma unroll
        for (int ks = 0; ks < 4; ++ks) {
            const int c = ks & 1;
            if (ks < 3) {
#pragma unroll
                for (int i = 0; i < MT; ++i)
                    af[c ^ 1][i] = *reinterpret_cast<const bf16x8*>(lds + (aad[tp][i] ^ ((ks + 1) << 5)));
#pragma unroll
                for (int j = 0; j < NT; ++j)
                    bfr[c ^ 1][j] = *reinterpret_cast<const bf16x8*>(lds + st * SB + b_rd[j][ks + 1]);
            }
#pragma unroll
            for (int i = 0; i < MT; ++i)
#pragma unroll
                for (int j = 0; j < NT; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(bfr[c][j], af[c][i], acc[i][j], 0, 0, 0);
        }
        constexpr int NR = MT + NT, NM = MT * NT;
        // slice ks + 1's fragment reads are issued BEFORE slice ks's MFMAs (the compiler's
        // counted lgkmcnt then waits for slice ks's reads only, slice ks + 1's stay in
        // flight under the MFMAs).  The read/MFMA interleave this replaces issued each
        // slice's last read after its MFMAs, into a register an MFMA had just released,
        // and waited lgkmcnt(0) on it: one exposed LDS round trip per k-slice.
        __builtin_amdgcn_sched_group_barrier(0x100, NR, 0);
#pragma unroll
        for (int ks = 0; ks < 3; ++ks) {
            __builtin_amdgcn_sched_group_barrier(0x100, NR, 0);
            __builtin_amdgcn_sched_group_barrier(0x008, NM, 0);
        }
        __builtin_amdgcn_sched_group_barrier(0x008, NM, 0);
    };

    // vmcnt(n): all but the wave's n newest vector-memory operations done
    auto wait_vm = [](int n) {
        switch (n) {
        case 0: __builtin_amdgcn_s_waitcnt((7 << 4) | (15 << 8)); break;
        case 1: __builtin_amdgcn_s_waitcnt(1 | (7 << 4) | (15 << 8)); break;
        case 2: __builtin_amdgcn_s_waitcnt(2 | (7 << 4) | (15 << 8)); break;
        case 3: __builtin_amdgcn_s_waitcnt(3 | (7 << 4) | (15 << 8)); break;
        case 4: __builtin_amdgcn_s_waitcnt(4 | (7 << 4) | (15 << 8)); break;
        case 5: __builtin_amdgcn_s_waitcnt(5 | (7 << 4) | (15 << 8)); break;
        case 6: __builtin_amdgcn_s_waitcnt(6 | (7 << 4) | (15 << 8)); break;
        case 7: __builtin_amdgcn_s_waitcnt(7 | (7 << 4) | (15 << 8)); break;
        case 8: __builtin_amdgcn_s_waitcnt(8 | (7 << 4) | (15 << 8)); break;
        case 9: __builtin_amdgcn_s_waitcnt(9 | (7 << 4) | (15 << 8)); break;
        case 10: __builtin_amdgcn_s_waitcnt(10 | (7 << 4) | (15 << 8)); break;
        case 11: __builtin_amdgcn_s_waitcnt(11 | (7 << 4) | (15 << 8)); break;
        default: __builtin_amdgcn_s_waitcnt(12 | (7 << 4) | (15 << 8)); break;
        }
    };
    static_assert((NB - 2) * BR <= 12, "counted wait range");
    const int nkt = (c1 - c0) * 9;
    issue_halo(c0);
#pragma unroll
    for (int k = 0; k < NB - 1; ++k)
        if (k < nkt) issue_b(c0 + k / 9, k % 9, k);
    int sb = 0;  // ring slot of k-tile kt
    int kt = 0;
    for (int cc = c0; cc < c1; ++cc) {
#pragma unroll
        for (int tp = 0; tp < 9; ++tp, ++kt) {
            // stages issued after k-tile kt: min(NB - 2, nkt - 1 - kt), left in flight
            const int ahead = min(NB - 2, nkt - 1 - kt);
            wait_vm(ahead * BR);
            __builtin_amdgcn_s_barrier();
            if (tp == 0 && cc > c0) {  // every wave is done with the previous chunk's halo
                issue_halo(cc);
                wait_vm(0);
                __builtin_amdgcn_s_barrier();
            }
            int sn = sb + NB - 1;
            if (sn >= NB) sn -= NB;
            if (kt + NB - 1 < nkt) {
                if (tp + NB - 1 < 9) issue_b(cc, tp + NB - 1, sn);
                else issue_b(cc + 1, tp + NB - 1 - 9, sn);
            }
            compute(tp, sb);
            if (++sb == NB) sb = 0;
        }
    }

    if (a.splits > 1) {
        constexpr int NQ = MT * NT * 4;  // float4 groups of accumulators per lane
        const auto rs = rsrc_of(a.ws + (size_t)tid * NQ * 256 * 4);
        if (split > 0) {  // wait for the previous split's running sum, then add it
            __shared__ int late;
            if (t == 0) {  // bounded: a broken hand-off never hangs, it faults loudly
                unsigned n = 0;
                bool ok = true;
                while (__hip_atomic_load(a.flags + tid, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) !=
                       (unsigned)split) {
                    if (++n >= a.spin_limit) {
                        ok = false;
                        break;
                    }
                    __builtin_amdgcn_s_sleep(2);
                }
                if (!ok) atomicOr(&g_conv_fault, GM_FAULT_SPLITK_SPIN);
                late = ok ? 0 : 1;
            }
            __syncthreads();
            if (late) {
#pragma unroll
                for (int i = 0; i < MT; ++i)
#pragma unroll
                    for (int j = 0; j < NT; ++j)
#pragma unroll
                        for (int r = 0; r < 16; ++r) acc[i][j][r] = __builtin_nanf("");
            }
#pragma unroll
            for (int i = 0; i < MT; ++i)
#pragma unroll
                for (int j = 0; j < NT; ++j)
#pragma unroll
                    for (int g = 0; g < 4; ++g) {
                        const float4 v = ld_sc1_f32x4(rs, (unsigned)((((i * NT + j) * 4 + g) * 256 + t) * 16));
                        acc[i][j][4 * g] += v.x;
                        acc[i][j][4 * g + 1] += v.y;
                        acc[i][j][4 * g + 2] += v.z;
                        acc[i][j][4 * g + 3] += v.w;
                    }
        }
        if (split < a.splits - 1) {  // publish the running sum to the next split
#pragma unroll
            for (int i = 0; i < MT; ++i)
#pragma unroll
                for (int j = 0; j < NT; ++j)
#pragma unroll
                    for (int g = 0; g < 4; ++g)
                        st_sc1_f32x4(rs, (unsigned)((((i * NT + j) * 4 + g) * 256 + t) * 16),
                                     make_float4(acc[i][j][4 * g], acc[i][j][4 * g + 1], acc[i][j][4 * g + 2],
                                                 acc[i][j][4 * g + 3]));
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
            if (t == 0) __hip_atomic_store(a.flags + tid, (unsigned)(split + 1), __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT);
            return;
        }
        if (t == 0) __hip_atomic_store(a.flags + tid, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    store_tile_lds<MT, NT, 128, BN>(a, cl, m0, n0, wm, wn, fr, fh, M, acc, g * a.gs_out, lds, HB + NB * SB, t, g);
}

// ---------------------------------------------------------------------------------
// 3x3 / stride-1 convolutions with 64 input and 64 output channels (ResNet layer 1:
// forward and input gradient).  The whole weight tensor (9 taps x 64 x 64 bf16 = 72 KB)
// stays resident in LDS for the life of a persistent workgroup, which walks output tiles
// of RT whole image rows (RT*W <= 128 pixels; MFMA rows past RT*W are padding whose
// outputs are not stored).  A tile's input is its (RT+2) x (W+2) zero-bordered halo
// (29 KB at 56x56), DMA'd into the second of two halo buffers while the MFMAs of the
// current tile run, so the only bytes staged per tile are the halo - instead of nine
// 16 KB im2col A tiles plus 72 KB of weights in the im2col kernel - and the k-loop is
// LDS reads + MFMAs only.  Halo pixels are 128-B rows XOR-swizzled as in k_conv_halo;
// weights are [tap][n][128 B] with the same swizzle on n.
struct RwArgs {
    int RT;        // image rows per tile
    int tpi;       // tiles per image (H / RT)
    int tiles;     // N * tpi
    int hbytes;    // one halo buffer (multiple of 1 KB)
    int nI;        // halo DMA instructions per tile
    int npix;      // (RT + 2) * (W + 2)
    FastDiv fd_w2, fd_tpi;
};

constexpr int kRwWeightBytes = 9 * 64 * 128;

template <int Form = 0>  // one form (the template keeps the symbol of earlier profiles)
__global__ __launch_bounds__(256) void k_conv_rw(ConvArgs a, RwArgs r) {
    extern __shared__ __attribute__((aligned(16))) uint4 smem[];
    char* lds = reinterpret_cast<char*>(smem);  // [weights][halo 0][halo 1]
    constexpr int WB = kRwWeightBytes;
    const ConvCls& cl = a.cls[0];
    const int H = a.Hi, W = a.Wi, W2 = W + 2;
    const int t = threadIdx.x, lane = t & 63;
    const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
    const int wm = wave >> 1, wn = wave & 1;
    const int slot = lane & 7, fr = lane & 31, fh = lane >> 5;
    const unsigned pk_dh = cl.pk_dh, pk_dw = cl.pk_dw, pk_r = cl.pk_r, pk_s = cl.pk_s;
    typedef __attribute__((address_space(1))) const void* gptr_t;
    typedef __attribute__((address_space(3))) void* lptr_t;
    // view groups: gridDim / G workgroups per group, each walking that group's tiles
    int g = 0, tl = blockIdx.x, nwg = gridDim.x;
    if (a.G > 1) {
        nwg = gridDim.x / a.G;
        g = tl / nwg;
        tl -= g * nwg;
    }
    if (tl >= r.tiles || g >= a.G) return;
    const uint16_t* const gin = a.in + g * a.gs_in;
    const uint16_t* const gwt = a.wt + g * a.gs_wt;
    const uint16_t* const gadd = a.addend ? a.addend + g * a.gs_out : nullptr;

    // weights, once: instruction I = tap (I >> 3), rows n = 8 (I & 7) .. + 7
    for (int I = wave; I < 72; I += 4) {
        const int tp = I >> 3, n = (I & 7) * 8 + (lane >> 3);
        const int ti = tp / 3, tj = tp - ti * 3;
        const int tw = (int)((pk_r >> (4 * ti)) & 15u) * a.Sw + (int)((pk_s >> (4 * tj)) & 15u);
        const int gc = slot ^ ((n >> 1) & 7);
        __builtin_amdgcn_global_load_lds((gptr_t)(gwt + ((size_t)n * a.T + tw) * 64 + gc * 8),
                                         (lptr_t)(lds + I * 1024), 16, 0, 0);
    }
    // the halo of tile tl (image b, output rows p0 .. p0+RT-1) into buffer bb.  The halo's
    // geometry relative to the tile origin is the same for every tile, so each lane's
    // source offsets (kMaxHI instructions per wave at most) are decoded once: per tile only
    // the origin and the image-border rows (top row valid iff p0 > 0, bottom iff p0+RT < H).
    constexpr int kMaxHI = 12;
    int h_rel[kMaxHI];
    unsigned h_cls = 0;  // 2 bits per instruction: 0 always, 1 top row, 2 bottom row, 3 never
#pragma unroll
    for (int j = 0; j < kMaxHI; ++j) {
        const int I = wave + 4 * j;
        const int hp = I * 8 + (lane >> 3);
        const int rr = (int)r.fd_w2.div((uint32_t)hp), c = hp - rr * W2;
        const int gc = slot ^ ((hp >> 1) & 7);
        h_rel[j] = ((rr - 1) * W + c - 1) * 64 + gc * 8;
        unsigned k = rr == 0 ? 1u : rr == r.RT + 1 ? 2u : 0u;
        if (I >= r.nI || hp >= r.npix || c == 0 || c == W + 1) k = 3u;
        h_cls |= k << (2 * j);
    }
    auto issue_halo = [&](int tile, int bb) {
        const int b = (int)r.fd_tpi.div((uint32_t)tile);
        const int p0 = (tile - b * r.tpi) * r.RT;
        const uint16_t* origin = gin + ((size_t)(b * H + p0) * W << 6);
        const unsigned okmask = 1u | (p0 > 0 ? 2u : 0u) | (p0 + r.RT < H ? 4u : 0u);  // bit k: class k valid
        char* base = lds + WB + bb * r.hbytes;
#pragma unroll
        for (int j = 0; j < kMaxHI; ++j) {
            const int I = wave + 4 * j;
            if (I >= r.nI) break;
            const bool ok = (okmask >> ((h_cls >> (2 * j)) & 3u)) & 1u;
            const void* src = ok ? (const void*)(origin + h_rel[j]) : (const void*)g_zero16;
            __builtin_amdgcn_global_load_lds((gptr_t)src, (lptr_t)(base + I * 1024), 16, 0, 0);
        }
    };
    issue_halo(tl, 0);

    // tile-invariant fragment geometry: MFMA row block i of this wave -> tile pixel
    const int valid = r.RT * W;
    int hbase[2], prow[2], pcol[2];
    bool pok[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        int m = wm * 64 + i * 32 + fr;
        pok[i] = m < valid;
        m = pok[i] ? m : 0;
        prow[i] = m / W;
        pcol[i] = m - prow[i] * W;
        hbase[i] = (prow[i] + 1) * W2 + pcol[i] + 1;
    }
    const int nb = wn * 32 + fr;
    const int b0 = nb * 128 + ((fh ^ ((nb >> 1) & 7)) << 4);  // B fragment, tap 0, k-step 0
    int b_ks[4];  // per k-step (the tap adds an immediate tap * 8192)
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) b_ks[ks] = b0 ^ (ks << 5);

    constexpr int kWaitAll = (7 << 4) | (15 << 8);  // s_waitcnt vmcnt(0)
    constexpr int kStores = 8;                      // epilogue stores per wave per tile (addend path)
    constexpr int kWaitStores = kStores | (7 << 4) | (15 << 8);  // vmcnt(kStores)
    constexpr int kWaitStores4 = 4 | (7 << 4) | (15 << 8);       // LDS-tile path: 4 16-B stores
    __builtin_amdgcn_s_waitcnt(kWaitAll);
    lds_barrier();
    const size_t out_bytes = (size_t)a.N * a.Ho * a.Wo * a.Nout * 2;
    const __amdgpu_buffer_rsrc_t orsrc =
        __builtin_amdgcn_make_buffer_rsrc(cl.out + g * a.gs_out, 0, (int)(out_bytes < 0x7fffffffu ? out_bytes : 0x7fffffffu),
                                          0x00020000);

    // BatchNorm statistics (a.stats; forward: y, input gradient: the BN backward's dz against
    // a.bnx): this thread's channel group t % 8 summed over the pixels it stores, combined over
    // the workgroup after the last tile (partial row wg)
    const int wg = tl;
    f32x2 bs1[4], bs2[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) bs1[k] = bs2[k] = f32x2{0.f, 0.f};
    BnB bq;
    if (a.stats && a.bnx) bnb_load(a, g, 8 * (t & 7), bq);
    const __amdgpu_buffer_rsrc_t xrsrc = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<uint16_t*>(a.bnx ? a.bnx + g * a.gs_out : cl.out), 0,
        (int)(out_bytes < 0x7fffffffu ? out_bytes : 0x7fffffffu), 0x00020000);
    int bb = 0;
    for (; tl < r.tiles; tl += nwg) {
        const int nx = tl + nwg;
        const int b = (int)r.fd_tpi.div((uint32_t)tl);
        const int p0 = (tl - b * r.tpi) * r.RT;
        const unsigned tbase = (unsigned)(((size_t)(b * a.Ho + p0) * a.Wo) * a.Nout * 2);
        // backward statistics: the BN input's chunks of this tile, loaded under the MFMAs
        // (issued before the next halo's DMA so their wait does not include it)
        __attribute__((ext_vector_type(4))) unsigned xv[4];
        if (a.stats && a.bnx && !a.addend) {
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int e = t + 256 * u;
                xv[u] = __builtin_amdgcn_raw_buffer_load_b128(xrsrc, (e >> 3) < valid ? tbase + (unsigned)e * 16u
                                                                                     : 0xfffffff0u, 0, 0);
            }
        }
        if (nx < r.tiles) issue_halo(nx, bb ^ 1);  // buffer bb^1 was released by the last barrier
        const int hoff = WB + bb * r.hbytes;

        floatx16 acc[2];
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int e = 0; e < 16; ++e) acc[i][e] = 0.f;
        bf16x8 af[2][2], bfr[2];
        unsigned abase[2];
        const unsigned lds0 = (unsigned)(uintptr_t)(__attribute__((address_space(3))) char*)lds;
        auto tap_base = [&](int tp) {
            const int ti = tp / 3, tj = tp - ti * 3;
            const int dh = (int)((pk_dh >> (4 * ti)) & 15u) - 8, dw = (int)((pk_dw >> (4 * tj)) & 15u) - 8;
            const int toff = dh * W2 + dw;
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                const int hp = hbase[i] + toff;
                abase[i] = lds0 + ((unsigned)(hoff + (hp << 7)) | (unsigned)((((hp >> 1) & 7) ^ fh) << 4));
            }
        };
        auto load_b = [&](auto tpc, int ks, int c) {
            constexpr int TP = decltype(tpc)::value;  // ds offsets are 16-bit: tap 8 moves the base
            if constexpr (TP < 8) bfr[c] = lds_rd128<TP * 8192>(lds0 + (unsigned)b_ks[ks]);
            else bfr[c] = lds_rd128<0>(lds0 + (unsigned)b_ks[ks] + TP * 8192u);
        };
        auto load = [&](int k, int c) {  // k-step k = 4 * tap + ks
            const int tp = k >> 2, ks = k & 3;
            if (ks == 0) tap_base(tp);
#pragma unroll
            for (int i = 0; i < 2; ++i) af[c][i] = lds_rd128<0>(abase[i] ^ (unsigned)(ks << 5));
            switch (tp) {
                case 0: load_b(std::integral_constant<int, 0>{}, ks, c); break;
                case 1: load_b(std::integral_constant<int, 1>{}, ks, c); break;
                case 2: load_b(std::integral_constant<int, 2>{}, ks, c); break;
                case 3: load_b(std::integral_constant<int, 3>{}, ks, c); break;
                case 4: load_b(std::integral_constant<int, 4>{}, ks, c); break;
                case 5: load_b(std::integral_constant<int, 5>{}, ks, c); break;
                case 6: load_b(std::integral_constant<int, 6>{}, ks, c); break;
                case 7: load_b(std::integral_constant<int, 7>{}, ks, c); break;
                default: load_b(std::integral_constant<int, 8>{}, ks, c); break;
            }
        };
        // one k-step of fragments in flight under the MFMAs: wait for everything, issue the
        // next k-step's reads, then this k-step's MFMAs (counted waits that keep two
        // k-steps in flight are not used: k_conv_stem showed sporadic wrong tiles with them)
        load(0, 0);
#pragma unroll
        for (int k = 0; k < 36; ++k) {
            const int c = k & 1;
            asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(af[c][0]), "+v"(af[c][1]), "+v"(bfr[c]));
            if (k + 1 < 36) load(k + 1, c ^ 1);
            __builtin_amdgcn_sched_barrier(0);  // the next k-step's reads go out before these MFMAs
#pragma unroll
            for (int i = 0; i < 2; ++i)
                acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(bfr[c], af[c][i], acc[i], 0, 0, 0);
            __builtin_amdgcn_sched_barrier(0);
        }

        if (!a.addend) {
            // epilogue through LDS: the tile's RT whole image rows are one contiguous NHWC
            // block, assembled in LDS (16-B chunks XOR-swizzled by pixel) and written with
            // 16-B stores instead of 8 B per lane at a 128-B stride
            char* ot = lds + WB + 2 * r.hbytes;
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                const int m = wm * 64 + i * 32 + fr;
#pragma unroll
                for (int gq = 0; gq < 4; ++gq) {
                    const int chunk = (wn * 4 + gq) ^ (m & 7);
                    *reinterpret_cast<uint2*>(ot + m * 128 + chunk * 16 + 8 * fh) =
                        make_uint2(pack_bf2(acc[i][4 * gq], acc[i][4 * gq + 1]),
                                   pack_bf2(acc[i][4 * gq + 2], acc[i][4 * gq + 3]));
                }
            }
            __syncthreads();
            uint4 vv[4];  // the four reads together, then the stores (then the statistics)
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int e = t + 256 * u;  // 16-B chunk e of the tile: pixel e / 8, chunk e % 8
                const int m = e >> 3, j = e & 7;
                vv[u] = *reinterpret_cast<const uint4*>(ot + (m < valid ? m : 0) * 128 + ((j ^ (m & 7)) << 4));
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int e = t + 256 * u;
                __builtin_amdgcn_raw_buffer_store_b128(
                    __builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned, vv[u]), orsrc,
                    (e >> 3) < valid ? tbase + (unsigned)e * 16u : 0xfffffff0u, 0, 0);
            }
            if (a.stats && a.bnx) {
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const bool ok = ((t + 256 * u) >> 3) < valid;
                    const unsigned w4[4] = {ok ? vv[u].x : 0u, ok ? vv[u].y : 0u, ok ? vv[u].z : 0u,
                                            ok ? vv[u].w : 0u};
                    const unsigned x4[4] = {xv[u].x, xv[u].y, xv[u].z, xv[u].w};
                    bn_acc_bwd(w4, x4, bq, bs1, bs2);
                }
            } else if (a.stats) {
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const bool ok = ((t + 256 * u) >> 3) < valid;
                    const unsigned w4[4] = {ok ? vv[u].x : 0u, ok ? vv[u].y : 0u, ok ? vv[u].z : 0u,
                                            ok ? vv[u].w : 0u};
                    bn_acc_fwd(w4, bs1, bs2);
                }
            }
            // the next tile's halo (issued before these stores) has landed; the stores may
            // still be in flight.  Then every wave is done with buffer bb and the LDS tile.
            __builtin_amdgcn_s_waitcnt(kWaitStores4);
            lds_barrier();
            bb ^= 1;
            continue;
        }
        // epilogue with the fused gradient join: rows p0 + prow, columns pcol; 4 consecutive
        // output channels per store, the addend loaded for the whole tile first (its loads in
        // flight together), added in fp32 before the one rounding to bf16
        size_t off[2];
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const int ho = (p0 + prow[i]) * cl.oS + cl.oH, wo = pcol[i] * cl.oS + cl.oW;
            off[i] = ((size_t)(b * a.Ho + ho) * a.Wo + wo) * a.Nout + wn * 32 + 4 * fh;
        }
        uint2 av[2][4];
        if (a.addend) {
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int gq = 0; gq < 4; ++gq)
                    av[i][gq] = *(const uint2*)(gadd + off[i] + 8 * gq);  // rows past RT*W read row 0
            if (a.amask) {  // element e's bit: byte e / 8, nibble (e / 4) & 1
                const uint8_t* const gm = a.amask + g * a.gs_out / 8;
#pragma unroll
                for (int i = 0; i < 2; ++i)
#pragma unroll
                    for (int gq = 0; gq < 4; ++gq) {
                        const size_t e = off[i] + 8 * gq;
                        const unsigned b = (unsigned)gm[e >> 3] >> (e & 4);
                        av[i][gq].x = mask_bf2(av[i][gq].x, b);
                        av[i][gq].y = mask_bf2(av[i][gq].y, b >> 2);
                    }
            }
        }
#pragma unroll
        for (int i = 0; i < 2; ++i) {
#pragma unroll
            for (int gq = 0; gq < 4; ++gq) {
                float o0 = acc[i][4 * gq], o1 = acc[i][4 * gq + 1];
                float o2 = acc[i][4 * gq + 2], o3 = acc[i][4 * gq + 3];
                if (a.addend) {
                    o0 += bf_lo(av[i][gq].x); o1 += bf_hi(av[i][gq].x);
                    o2 += bf_lo(av[i][gq].y); o3 += bf_hi(av[i][gq].y);
                }
                typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
                const u32x2 v = {pack_bf2(o0, o1), pack_bf2(o2, o3)};
                // every wave issues exactly kStores stores (padding rows get an offset past
                // the buffer's range, which the hardware drops), so the wait below can count them
                __builtin_amdgcn_raw_buffer_store_b64(v, orsrc, pok[i] ? (unsigned)((off[i] + 8 * gq) * 2) : 0xfffffff0u,
                                                      0, 0);
            }
        }
        // the next tile's halo (issued before these stores) has landed; the stores may
        // still be in flight.  Then every wave is done with buffer bb.
        __builtin_amdgcn_s_waitcnt(kWaitStores);
        lds_barrier();
        bb ^= 1;
    }
    if (a.stats) {  // the partial row: [32 thread rows][64 channels][2] combined in the free LDS tile
        float* red = reinterpret_cast<float*>(lds + WB + 2 * r.hbytes);  // 16 KB
        const int r0 = t >> 3, cg = t & 7;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            red[r0 * 128 + (cg * 8 + 2 * k) * 2] = bs1[k].x;
            red[r0 * 128 + (cg * 8 + 2 * k) * 2 + 1] = bs2[k].x;
            red[r0 * 128 + (cg * 8 + 2 * k + 1) * 2] = bs1[k].y;
            red[r0 * 128 + (cg * 8 + 2 * k + 1) * 2 + 1] = bs2[k].y;
        }
        __syncthreads();
        if (t < 128) {
            float s = 0.f;
            for (int i = 0; i < 32; ++i) s += red[i * 128 + t];
            a.stats[((size_t)g * (a.stats_rows + 1) + wg) * 128 + t] = s;
        }
    }
}

// ---------------------------------------------------------------------------------
// The ResNet stem on its pixel-pair view (conv.py: a 7 x 4 filter over 8-channel pairs,
// strides (2, 1), K = 224, 64 output channels, no padding).  A workgroup walks a
// contiguous run of output rows of one image, TWO rows per iteration:
//  * the weights live in VGPRs (each lane its 2 x 14 B fragments, 112 VGPRs), so the
//    LDS feeds only the pixel operand;
//  * input rows stream through an LDS ring of "units" of two input rows (unit u = rows
//    2u, 2u + 1, slot u % 8), fetched once per workgroup by register-staged global loads
//    two iterations ahead (no LDS-DMA: every LDS access is compiler-visible, so its waits
//    are exact);
//  * output rows p, p + 1 share input rows (row p + 1's tap row r is row p's r + 2): one
//    pixel fragment of input row j feeds row p's MFMAs (tap row j) and row p + 1's (tap
//    row j - 2) - 18 fragment reads for 56 MFMAs per wave, where the row-at-a-time form
//    with weights in LDS read 84;
//  * wave w owns output columns 32 w .. 32 w + 31 and all 64 channels; its 8 KB output
//    tile is private (no barrier between the MFMAs and the stores), leaving as whole
//    128-B pixel rows.
// One barrier per iteration (the ring).  The row-at-a-time kernel this replaces spent
// 121 us per step: per-k-step address math and an LDS round trip + barrier per row.
constexpr int kStemRing = 8;
struct StemArgs {
    int N, P;      // images, output rows per image
    int cpi, L;    // chunks (workgroups) per image, output rows per chunk (even)
    int uchunks;   // 16-B chunks per unit (2 * Wi)
    int upitch;    // LDS bytes per ring slot (uchunks * 16)
    int ichunks;   // 16-B chunks per image (Hi * Wi)
    float* stats;  // optional: per-workgroup BatchNorm partial rows of the stored output
                   // ([G][stats_rows][64 x (sum, sum of squares)] + 128 floats per group)
    int stats_rows;  // workgroups per group (N * cpi: the rows of each group's partials)
};

template <int R, int S>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2, 2))) void k_conv_stem(ConvArgs a, StemArgs r) {
    static_assert(S % 2 == 0 && R >= 2, "k_conv_stem: even pair-tap count per row");
    constexpr int KS = R * S / 2;  // k-steps (two taps of 8 channels each)
    constexpr int H2 = S / 2;      // k-steps per tap row
    extern __shared__ __attribute__((aligned(16))) uint4 smem[];
    char* lds = reinterpret_cast<char*>(smem);  // [ring 8 x upitch][4 wave tiles x 8 KB]
    const ConvCls& cl = a.cls[0];
    const int Wi = a.Wi, Q = cl.Q;
    const int t = threadIdx.x, lane = t & 63;
    const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
    const int fr = lane & 31, fh = lane >> 5;
    const int per = r.stats_rows;
    const int g = blockIdx.x / per, wg = blockIdx.x - g * per;
    if (g >= a.G) return;
    const int b = wg / r.cpi, c = wg - b * r.cpi;
    const int p0 = c * r.L, p1 = min(cl.P, p0 + r.L);
    const uint4* const img = reinterpret_cast<const uint4*>(a.in + g * a.gs_in) + (size_t)b * r.ichunks;
    char* const tile = lds + kStemRing * r.upitch + wave * 8192;

    // weights -> VGPRs: fragment (k-step ks, channel block cb) = channel 32 cb + fr, tap 2 ks + fh
    bf16x8 wf[KS][2];
    {
        const uint4* wsrc = reinterpret_cast<const uint4*>(a.wt + g * a.gs_wt);
#pragma unroll
        for (int ks = 0; ks < KS; ++ks)
#pragma unroll
            for (int cb = 0; cb < 2; ++cb)
                wf[ks][cb] = __builtin_bit_cast(bf16x8, wsrc[(cb * 32 + fr) * (2 * KS) + 2 * ks + fh]);
    }
    // two units (u, u + 1: 2 * uchunks 16-B chunks, contiguous in the image) per iteration:
    // thread t holds chunks t and t + 256 (2 * uchunks <= 512); zeros past the image
    auto fetch = [&](int u, uint4 (&v)[2]) __attribute__((always_inline)) {
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int cc = t + 256 * h;
            const int gi = u * r.uchunks + cc;
            v[h] = (cc < 2 * r.uchunks && gi < r.ichunks) ? img[gi] : make_uint4(0, 0, 0, 0);
        }
    };
    auto stash = [&](int u, const uint4 (&v)[2]) __attribute__((always_inline)) {
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int cc = t + 256 * h;
            if (cc < 2 * r.uchunks) {
                const int hi = cc >= r.uchunks;
                const int uu = u + hi;
                *reinterpret_cast<uint4*>(lds + (uu & (kStemRing - 1)) * r.upitch + (cc - hi * r.uchunks) * 16) = v[h];
            }
        }
    };
    // prologue: units p0 .. p0 + 4 into the ring (iteration 0's window), units of
    // iterations 1 and 2 into the register stages
    {
        uint4 v0[2], v1[2], v2[2];
        fetch(p0, v0);
        fetch(p0 + 2, v1);
        fetch(p0 + 4, v2);
        stash(p0, v0);
        stash(p0 + 2, v1);
        stash(p0 + 4, v2);  // (unit p0 + 5 too: part of iteration 1's window, rewritten there)
    }
    uint4 sa[2], sb[2];  // register stages: units for iterations i + 1 (written at i) and i + 2
    fetch(p0 + 5, sa);
    fetch(p0 + 7, sb);

    float bs1[8], bs2[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) bs1[j] = bs2[j] = 0.f;
    const int q = wave * 32 + fr;
    const int qc = q < Q ? q : 0;
    const size_t out_bytes = (size_t)a.N * a.Ho * a.Wo * a.Nout * 2;
    const __amdgpu_buffer_rsrc_t orsrc =
        __builtin_amdgcn_make_buffer_rsrc(cl.out + g * a.gs_out, 0, (int)(out_bytes < 0x7fffffffu ? out_bytes : 0x7fffffffu),
                                          0x00020000);

    auto iteration = [&](int p, uint4 (&cur)[2]) __attribute__((always_inline)) {
        __syncthreads();  // units p .. p + 4 are in the ring; iteration p - 2's reads are done
        stash(p + 5, cur);  // iteration p + 2's new units into the slots of units p - 3, p - 2
        fetch(p + 9, cur);  // ... and the iteration after next's into the registers

        floatx16 acc[2][2];
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int cb = 0; cb < 2; ++cb)
#pragma unroll
                for (int e = 0; e < 16; ++e) acc[i][cb][e] = 0.f;
        unsigned sl[5];  // ring slot bases of units p .. p + 4
#pragma unroll
        for (int d = 0; d < 5; ++d) sl[d] = (unsigned)(((p + d) & (kStemRing - 1)) * r.upitch);
        // pixel fragment (input row j, tap pair h): lane (q, fh) <- pixel pair q + 2 h + fh
#pragma unroll
        for (int j = 0; j < R + 2; ++j) {
#pragma unroll
            for (int h = 0; h < H2; ++h) {
                const bf16x8 af = *reinterpret_cast<const bf16x8*>(lds + sl[j >> 1] +
                                                                   (((j & 1) * Wi + qc + 2 * h + fh) << 4));
                if (j < R) {
#pragma unroll
                    for (int cb = 0; cb < 2; ++cb)
                        acc[0][cb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wf[j * H2 + h][cb], af, acc[0][cb], 0, 0, 0);
                }
                if (j >= 2) {
#pragma unroll
                    for (int cb = 0; cb < 2; ++cb)
                        acc[1][cb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wf[(j - 2) * H2 + h][cb], af, acc[1][cb],
                                                                            0, 0, 0);
                }
            }
        }
        // the wave's tile: [row i][pixel fr][64 channels] bf16, 16-B chunks XOR-swizzled by pixel
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int cb = 0; cb < 2; ++cb)
#pragma unroll
                for (int gq = 0; gq < 4; ++gq) {
                    const int chunk = (cb * 4 + gq) ^ (fr & 7);
                    *reinterpret_cast<uint2*>(tile + (i * 32 + fr) * 128 + chunk * 16 + 8 * fh) =
                        make_uint2(pack_bf2(acc[i][cb][4 * gq], acc[i][cb][4 * gq + 1]),
                                   pack_bf2(acc[i][cb][4 * gq + 2], acc[i][cb][4 * gq + 3]));
                }
        // 8 KB = 64 pixel rows of 128 B: store u covers pixel rows 8 u .. 8 u + 7, lane ->
        // (pixel row 8 u + lane / 8, chunk lane % 8): the channel group is lane % 8
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int pr = 8 * u + (lane >> 3), j = lane & 7;
            const int i = pr >> 5, px = pr & 31;
            const int qq = wave * 32 + px;
            const bool ok = qq < Q && p + i < p1;
            const uint4 v = *reinterpret_cast<const uint4*>(tile + pr * 128 + ((j ^ (px & 7)) << 4));
            const unsigned off = (unsigned)((((size_t)(b * a.Ho + p + i) * a.Wo + qq) * 64 + j * 8) * 2);
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned, v),
                                                   orsrc, ok ? off : 0xfffffff0u, 0, 0);
            if (r.stats) {
                const uint32_t w4[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
                for (int jj = 0; jj < 8; ++jj) {
                    const float f = ok ? __uint_as_float((jj & 1) ? (w4[jj >> 1] & 0xffff0000u) : (w4[jj >> 1] << 16))
                                       : 0.f;
                    bs1[jj] += f;
                    bs2[jj] = fmaf(f, f, bs2[jj]);
                }
            }
        }
    };
    // iterations alternate the two register stages (stage a: units written at even iterations)
    for (int p = p0; p < p1; p += 4) {
        iteration(p, sa);
        if (p + 2 < p1) iteration(p + 2, sb);
    }
    if (r.stats) {  // the workgroup's partial row: [32 thread rows][64 channels][2] combined in LDS
        __syncthreads();
        float* red = reinterpret_cast<float*>(lds);  // the ring (>= 16 KB)
        const int r0 = t >> 3, cg = t & 7;
#pragma unroll
        for (int jj = 0; jj < 8; ++jj) {
            red[r0 * 128 + (cg * 8 + jj) * 2] = bs1[jj];
            red[r0 * 128 + (cg * 8 + jj) * 2 + 1] = bs2[jj];
        }
        __syncthreads();
        if (t < 128) {
            float acc = 0.f;
            for (int i = 0; i < 32; ++i) acc += red[i * 128 + t];
            r.stats[((size_t)g * (r.stats_rows + 1) + wg) * 128 + t] = acc;
        }
    }
}

// zero the output pixels no dgrad class covers (e.g. odd pixels of a 1x1/s2 dgrad), or
// copy the addend there when the dgrad is fused with a gradient join
__global__ void k_zero_bf16(uint16_t* p, size_t n, const uint16_t* src, const uint8_t* msk = nullptr) {
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    for (; i * 8 < n; i += (size_t)gridDim.x * blockDim.x) {
        uint4 v = src ? *(const uint4*)(src + i * 8) : make_uint4(0, 0, 0, 0);
        if (msk) {  // the masked addend: byte i covers these 8 elements
            const unsigned b = msk[i];
            v.x = mask_bf2(v.x, b); v.y = mask_bf2(v.y, b >> 2); v.z = mask_bf2(v.z, b >> 4); v.w = mask_bf2(v.w, b >> 6);
        }
        *(uint4*)(p + i * 8) = v;
    }
}

// W[Co][T][Ci] -> Wt[Ci][T][Co] (bf16), for the input-gradient convolution
__global__ void k_transpose_w(const uint16_t* w, uint16_t* wt, int Co, int T, int Ci) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    const int n = Co * T * Ci;
    if (i >= n) return;
    const int c = i % Ci, tk = (i / Ci) % T, k = i / (Ci * T);
    wt[((size_t)c * T + tk) * Co + k] = w[i];
}

static int ilog2(int v) {
    int l = 0;
    while ((1 << l) < v) ++l;
    return (1 << l) == v ? l : -1;
}

}  // namespace gm

using namespace gm;

static bool lean_path() {
    static bool on = [] {
        return true;
    }();
    return on;
}

static bool grid_ok(const ConvCls& c, int S);
static void pack_grid(ConvCls& c, int S);

// main-loop form of the lean kernel (k_conv_igemm_ut PIPE); gm_conv_set_pipe() at run time (A/B in
// one process).  -1 (default): PIPE 2 - one raw barrier per k-tile with a counted wait - which
// measured 2-6 % faster than PIPE 0 on the strided first convolutions of layers 2-4 as the step
// launches them (r06, profiles/r06_strided_ab.txt); the halo kernels stay eligible
static int g_conv_pipe = -1;
static int conv_pipe() { return g_conv_pipe; }

template <int BM, int BN, int PIPE>
static void launch_ut(const ConvArgs& a, int grid, hipStream_t st) {
    constexpr int NST = PIPE == 3 ? 3 : 2;
    const size_t lds = (size_t)NST * (BM + BN) * 128;
    static bool attr = false;  // idempotent, safe to race
    if (!attr) {
        (void)hipFuncSetAttribute((const void*)k_conv_igemm_ut<BM, BN, PIPE>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)lds);
        attr = true;
    }
    k_conv_igemm_ut<BM, BN, PIPE><<<grid, 256, lds, st>>>(a);
}

// the masked addend materialised over dx (k_zero_bf16's masked copy; every group, contiguous),
// which then is the addend in place - for the kernels whose epilogue reads no mask
static int demask(ConvArgs& a, hipStream_t st) {
    if (!a.amask) return GM_OK;
    const size_t n = (size_t)(a.G > 1 ? a.G : 1) * a.N * a.Ho * a.Wo * a.Nout;
    uint16_t* dx = a.cls[0].out;
    k_zero_bf16<<<(int)((n / 8 + 255) / 256 < 4096 ? (n / 8 + 255) / 256 : 4096), 256, 0, st>>>(dx, n, a.addend,
                                                                                               a.amask);
    a.addend = dx;
    a.amask = nullptr;
    return check_launch("k_zero_bf16");
}

template <int BM, int BN, int ST>
static int launch_igemm(ConvArgs& a, hipStream_t st) {
    if (int rc = demask(a, st)) return rc;
    int tiles = 0;
    for (int i = 0; i < a.ncls; ++i) {
        ConvCls& c = a.cls[i];
        const int M = a.N * c.P * c.Q;
        c.tiles_m = (M + BM - 1) / BM;
        c.tile_start = tiles;
        tiles += c.tiles_m * ((a.Nout + BN - 1) / BN);
    }
    if (tiles == 0) return GM_OK;
    a.tiles_g = tiles;
    tiles *= a.G;  // view groups: G x the tiles of one group
    a.tiles_total = tiles;
    if (a.splits < 1) a.splits = 1;
    const size_t lds = (size_t)ST * (BM + BN) * 128 + kMaxTap * 4 + 12;
    static bool attr_set = false;  // idempotent, safe to race
    if (!attr_set) {
        (void)hipFuncSetAttribute((const void*)k_conv_igemm<BM, BN, true, ST>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)lds);
        (void)hipFuncSetAttribute((const void*)k_conv_igemm<BM, BN, false, ST>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)lds);
        attr_set = true;
    }
    bool grid = true;
    for (int i = 0; i < a.ncls; ++i) grid = grid && grid_ok(a.cls[i], a.Sw);
    if (a.C >= 64 && grid && lean_path()) {
        const int pipe = conv_pipe() < 0 ? 2 : conv_pipe();
        if (pipe == 3) launch_ut<BM, BN, 3>(a, tiles * a.splits, st);
        else if (pipe == 2) launch_ut<BM, BN, 2>(a, tiles * a.splits, st);
        else launch_ut<BM, BN, 0>(a, tiles * a.splits, st);
    } else if (a.splits > 1) {
        set_error("conv: split-K needs the lean kernel");
        return GM_E_ARG;
    } else if (a.G > 1) {
        set_error("conv: view groups need the lean, halo or resident-weight kernels (C >= 64)");
        return GM_E_UNSUP;
    } else if (a.C >= 64) {
        k_conv_igemm<BM, BN, true, ST><<<tiles, 256, lds, st>>>(a);
    } else {
        k_conv_igemm<BM, BN, false, ST><<<tiles, 256, lds, st>>>(a);
    }
    return check_launch("k_conv_igemm");
}

static int stages() {
    static int s = [] {
        return 2;  // (3 stages: one workgroup per CU, slower)
    }();
    return s;
}

// XCD remap of the tile order (ConvArgs::xcd: each XCD a contiguous tile range, tm fastest, so one
// weight slice stays in one L2): measured no gain (r01; r06: a split-aware tn-fastest remap, whose
// XCDs share each pixel range's im2col rows, 3.62 vs 3.59 ms/step) - off
static int xcd_remap() { return 0; }

static int tile_bias() {
    static int b = [] {
        return 1024;
    }();
    return b;
}

static int g_splitk_target = [] {
    return 384;  // workgroups wanted from split-K; 0 disables it
}();
static int splitk_target() { return g_splitk_target; }

static int splitk_mink() {
    static int t = [] {
        return 16;  // minimum k-tiles per split
    }();
    return t;
}

enum { T128x128 = 0, T128x64 = 1, T64x64 = 2 };
struct TilePick {
    int tile, splits, tiles;
};

static bool lean_ok(const ConvArgs& a) {
    bool grid = a.C >= 64 && lean_path();
    for (int i = 0; i < a.ncls; ++i) grid = grid && grid_ok(a.cls[i], a.Sw);
    return grid;
}

static int conv_cus() {
    static int n = [] {
        int dev = 0, c = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || c <= 0)
            c = 256;
        return c;
    }();
    return n;
}

// enough workgroups to fill 256 CUs with the largest tile that does (128x128: 4
// independent accumulators per wave, so one workgroup per CU keeps the MFMA pipe fed);
// when 128x128 tiles alone are too few (layers 3/4: small M, long K), split K over
// 2-4 workgroups per tile (turnstile hand-off, lean kernel only) instead of shrinking
// the tile, which halves the staged bytes per FLOP against 64x64.
static TilePick pick_tile(const ConvArgs& a) {
    long M = 0;
    int t128 = 0, nkmin = 1 << 30;
    for (int i = 0; i < a.ncls; ++i) {
        const long Mi = (long)a.N * a.cls[i].P * a.cls[i].Q;
        M += Mi * a.G;
        t128 += a.G * (int)((Mi + 127) / 128) * ((a.Nout + 127) / 128);
        const int nk = a.cls[i].ntap * a.C / 64;
        nkmin = nk < nkmin ? nk : nkmin;
    }
    const long wgs = tile_bias();  // workgroups wanted before a larger tile is taken
    if (a.Nout >= 128 && M / 128 * (a.Nout / 128) >= wgs / 4) return {T128x128, 1, t128};
    const int want = splitk_target();
    if (want > 0 && a.Nout >= 128 && a.C >= 64 && t128 > 0 && lean_ok(a)) {
        int S = (want + t128 - 1) / t128;
        if (S > 4) S = 4;
        while (S > 1 && nkmin / S < splitk_mink()) --S;  // long enough splits to amortize the hand-off
        // deadlock freedom of the turnstile: a waiting split holds its CU slot while the
        // split it waits on may still be queued behind OTHER launches' waiting splits (the
        // other trunk's stream; another process when ranks share the device) or behind
        // kernels that never yield (RCCL collectives overlapping backward).  Keep the
        // waiting workgroups of one launch (tiles x (S-1)) within two slots per usable CU
        // (CUs minus the reserved ones) divided by the launches that can wait at once -
        // the residency plan's streams x sharers (gm_set_residency; S = 4 at layer 4 timed
        // out with two ranks sharing one GPU before the plan counted them)
        const Residency& rs = residency();
        while (S > 1 && (long)t128 * (S - 1) > (long)usable_cus(conv_cus()) * 2 / (rs.streams * rs.sharers)) --S;
        if (S >= 2) return {T128x128, S, t128};
    }
    if (M / 128 * ((a.Nout + 63) / 64) >= wgs * 3 / 4) return {T128x64, 1, 0};
    return {T64x64, 1, 0};
}

// turnstile words live in a FIXED region at the start of the workspace (never overlapped
// by any call's slabs, whatever its tile count), so they stay zero between calls that
// share the workspace
constexpr int kMaxSplitTiles = 16384;
static size_t splitk_flag_bytes(int /*tiles*/) { return (size_t)kMaxSplitTiles * 4; }

static size_t splitk_bytes(const TilePick& p) {
    if (p.splits <= 1) return 0;
    return splitk_flag_bytes(p.tiles) + (size_t)p.tiles * 16 * 256 * 16;  // 128x128: 16 float4 per lane
}

static int g_conv_halo = [] {
    return 1;
}();

// the halo kernel serves one-class, 3x3 tap grids with offsets in [-1, 1] at stride 1
// and same-size output (forward 3x3/s1/p1 and its input gradient), C a multiple of 64;
// returns the halo LDS bytes (0 = not eligible)
static int halo_bytes(const ConvArgs& a, int BM = 128) {
    // C >= 128 (two or more chunks): with one chunk (ResNet layer 1) the whole halo must
    // land before the first k-tile and the im2col kernel measured faster (tools/conv_ab.py)
    if (!g_conv_halo || a.ncls != 1 || a.C < 128 || (a.C & 63) || a.sAh != 1 || a.sAw != 1) return 0;
    const ConvCls& c = a.cls[0];
    if (c.ntap != 9 || c.Rc != 3 || c.Sc != 3 || c.oS != 1 || c.P != a.Hi || c.Q != a.Wi || a.Ho != a.Hi ||
        a.Wo != a.Wi || !grid_ok(c, a.Sw))
        return 0;
    for (int i = 0; i < 3; ++i)
        if (c.cdh[i] < -1 || c.cdh[i] > 1 || c.cdw[i] < -1 || c.cdw[i] > 1) return 0;
    const int H1 = a.Hi + 1, W2 = a.Wi + 2, PQ = c.P * c.Q, M = a.N * PQ;
    int maxpix = 0;
    for (int m0 = 0; m0 < M; m0 += BM) {
        const int m1 = (m0 + BM < M ? m0 + BM : M) - 1;
        const int b0 = m0 / PQ, p0 = (m0 - b0 * PQ) / c.Q;
        const int b1 = m1 / PQ, p1 = (m1 - b1 * PQ) / c.Q;
        const int npix = (b1 * H1 + p1 + 2 - (b0 * H1 + p0) + 1) * W2;
        maxpix = npix > maxpix ? npix : maxpix;
    }
    return (maxpix + 7) / 8 * 1024;
}

template <int BN, int NB, int BM = 128>
static int launch_halo_v(ConvArgs& a, int hb, hipStream_t st) {
    if (int rc = demask(a, st)) return rc;
    ConvCls& c = a.cls[0];
    const int M = a.N * c.P * c.Q;
    c.tiles_m = (M + BM - 1) / BM;
    c.tile_start = 0;
    a.tiles_total = c.tiles_m * ((a.Nout + BN - 1) / BN);
    if (a.splits < 1) a.splits = 1;
    HaloArgs h;
    h.halo_bytes = hb;
    h.fd_w2 = FastDiv((uint32_t)(a.Wi + 2));
    h.fd_h1 = FastDiv((uint32_t)(a.Hi + 1));
    const size_t lds = (size_t)hb * (BM == 256 ? 2 : 1) + NB * (size_t)BN * 128;
    static size_t attr = 0;  // largest dynamic LDS granted so far (idempotent, safe to race)
    if (lds > attr) {
        const hipError_t e = hipFuncSetAttribute((const void*)k_conv_halo<BM, BN, NB>,
                                                 hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (e != hipSuccess) {
            set_error("k_conv_halo: %zu B of LDS refused (%s)", lds, hipGetErrorString(e));
            return GM_E_UNSUP;
        }
        attr = lds;
    }
    k_conv_halo<BM, BN, NB><<<a.tiles_total * a.splits, BM == 256 ? 512 : 256, lds, st>>>(a, h);
    return check_launch("k_conv_halo");
}

static int g_conv_stem = [] {
    return 1;  // 0: the pixel-pair stem takes the im2col kernel
}();

// k_conv_stem serves the pixel-pair stem: one-class forward convolutions over 8-channel
// elements with 64 output channels, no padding, strides (2, 1), a 7 x 4 filter and output
// columns <= 128; returns its LDS bytes (0 = not eligible)
static size_t stem_plan(const ConvArgs& a, StemArgs& r) {
    if (!g_conv_stem || a.ncls != 1 || a.C != 8 || a.Nout != 64 || a.sAw != 1 || a.sAh != 2) return 0;
    const ConvCls& c = a.cls[0];
    if (c.oS != 1 || c.oH != 0 || c.oW != 0 || c.Q > 128 || c.ntap != a.T || a.Sw != 4 || a.T != 28) return 0;
    for (int tp = 0; tp < c.ntap; ++tp) {  // forward taps without padding: (r, s) = (dh, dw), weight tap tp
        const int rr = tp / a.Sw, ss = tp - rr * a.Sw;
        if (c.tw[tp] != tp || c.dh[tp] != rr || c.dw[tp] != ss) return 0;
    }
    const int R = a.T / a.Sw;
    if ((c.P - 1) * a.sAh + R > a.Hi || c.Q - 1 + a.Sw > a.Wi) return 0;
    if ((size_t)a.N * a.Ho * a.Wo * a.Nout * 2 >= 0x7ffff000u) return 0;
    if ((long long)a.Hi * a.Wi >= (1ll << 27)) return 0;
    r.N = a.N;
    r.P = c.P;
    r.uchunks = 2 * a.Wi;
    if (r.uchunks > 256) return 0;  // two units per iteration over 256 threads x 2 chunks
    r.upitch = r.uchunks * 16;
    r.ichunks = a.Hi * a.Wi;
    // chunks of an even number of rows: about two workgroups per CU over all view groups
    const int target = a.G > 0 ? 512 / a.G : 512;
    const int cpi0 = std::max(1, std::min((c.P + 1) / 2, target / std::max(1, a.N)));
    r.L = (c.P + cpi0 - 1) / cpi0;
    r.L += r.L & 1;
    r.cpi = (c.P + r.L - 1) / r.L;  // no empty chunk
    r.stats_rows = a.N * r.cpi;
    r.stats = nullptr;
    const size_t lds = (size_t)kStemRing * r.upitch + 4 * 8192;
    return lds <= 80 * 1024 ? lds : 0;  // two workgroups per CU
}

static int launch_stem(const ConvArgs& a, const StemArgs& r, size_t lds, hipStream_t st) {
    static size_t granted = 0;
    if (lds > granted) {
        const hipError_t e =
            hipFuncSetAttribute((const void*)k_conv_stem<7, 4>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (e != hipSuccess) {
            set_error("k_conv_stem: %zu B of LDS refused (%s)", lds, hipGetErrorString(e));
            return GM_E_UNSUP;
        }
        granted = lds;
    }
    // N * cpi workgroups per view group (about two per CU in all)
    k_conv_stem<7, 4><<<r.stats_rows * a.G, 256, lds, st>>>(a, r);
    return check_launch("k_conv_stem");
}

static int g_conv_rw = [] {
    return 1;  // 0: layer-1 shapes take the im2col kernel
}();

// the resident-weight kernel serves one-class 3x3 / stride-1 / same-size convolutions with
// C = Nout = 64 and tap offsets in [-1, 1]; returns its LDS bytes (0 = not eligible)
static size_t rw_plan(const ConvArgs& a, RwArgs& r) {
    if (!g_conv_rw || a.ncls != 1 || a.C != 64 || a.Nout != 64 || a.T != 9 || a.sAh != 1 || a.sAw != 1) return 0;
    const ConvCls& c = a.cls[0];
    if (c.ntap != 9 || c.Rc != 3 || c.Sc != 3 || c.oS != 1 || c.P != a.Hi || c.Q != a.Wi || a.Ho != a.Hi ||
        a.Wo != a.Wi || !grid_ok(c, a.Sw) || a.Wi > 128)
        return 0;
    if ((size_t)a.N * a.Ho * a.Wo * a.Nout * 2 >= 0x7ffff000u) return 0;  // 32-bit buffer offsets
    for (int i = 0; i < 3; ++i)
        if (c.cdh[i] < -1 || c.cdh[i] > 1 || c.cdw[i] < -1 || c.cdw[i] > 1) return 0;
    int RT = 128 / a.Wi;
    if (RT > a.Hi) RT = a.Hi;
    while (RT > 1 && a.Hi % RT) --RT;
    r.RT = RT;
    r.tpi = a.Hi / RT;
    r.tiles = a.N * r.tpi;
    r.npix = (RT + 2) * (a.Wi + 2);
    r.nI = (r.npix + 7) / 8;
    if (r.nI > 48) return 0;  // k_conv_rw decodes at most 12 halo instructions per wave
    r.hbytes = r.nI * 1024;
    r.fd_w2 = FastDiv((uint32_t)(a.Wi + 2));
    r.fd_tpi = FastDiv((uint32_t)r.tpi);
    const size_t lds = (size_t)kRwWeightBytes + 2 * (size_t)r.hbytes + 128 * 128;
    return lds <= 160 * 1024 ? lds : 0;
}

// persistent: one workgroup per CU, split evenly over the view groups (workgroups per group)
static int rw_per(const ConvArgs& a, const RwArgs& r) {
    return r.tiles < 256 / a.G ? r.tiles : (256 / a.G > 0 ? 256 / a.G : 1);
}
static int launch_rw(const ConvArgs& a, const RwArgs& r, size_t lds, hipStream_t st) {
    static bool granted = false;  // the whole LDS (idempotent, safe to race)
    if (!granted) {
        const int mx = 160 * 1024;
        const hipError_t e = hipFuncSetAttribute((const void*)k_conv_rw<0>, hipFuncAttributeMaxDynamicSharedMemorySize, mx);
        if (e != hipSuccess) {
            set_error("k_conv_rw: %d B of LDS refused (%s)", mx, hipGetErrorString(e));
            return GM_E_UNSUP;
        }
        granted = true;
    }
    const int grid = rw_per(a, r) * a.G;
    k_conv_rw<0><<<grid, 256, lds, st>>>(a, r);
    return check_launch("k_conv_rw");
}

static int g_conv_h9 = [] {
    return 1;  // 0: the halo shapes take k_conv_halo (A/B)
}();
// k_conv_h9 when eligible: Nout a multiple of BN, at most 48 halo DMA instructions, the
// halo + 3 weight stages within half the CU's LDS (two workgroups per CU), splits over
// whole channel chunks.  Returns 0 when not taken.
template <int BN, int NB>
static int launch_h9(ConvArgs& a, int hb, hipStream_t st) {
    ConvCls& c = a.cls[0];
    const int M = a.N * c.P * c.Q;
    c.tiles_m = (M + 127) / 128;
    c.tile_start = 0;
    a.tiles_g = c.tiles_m * (a.Nout / BN);
    a.tiles_total = a.tiles_g * a.G;
    if (a.splits < 1) a.splits = 1;
    HaloArgs h;
    h.halo_bytes = hb;
    h.fd_w2 = FastDiv((uint32_t)(a.Wi + 2));
    h.fd_h1 = FastDiv((uint32_t)(a.Hi + 1));
    const size_t lds = (size_t)hb + NB * (size_t)BN * 128;
    static size_t attr = 0;
    if (lds > attr) {
        const hipError_t e =
            hipFuncSetAttribute((const void*)k_conv_h9<BN, NB>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (e != hipSuccess) {
            set_error("k_conv_h9: %zu B of LDS refused (%s)", lds, hipGetErrorString(e));
            return GM_E_UNSUP;
        }
        attr = lds;
    }
    k_conv_h9<BN, NB><<<dim3(a.tiles_total * a.splits), 256, lds, st>>>(a, h);
    const int rc = check_launch("k_conv_h9");
    return rc == GM_OK ? 1 : rc;
}

// (BN, NB) of k_conv_h9 for a shape: gm_conv_set_h9(1) = automatic - the deepest weight
// ring (<= 3 stages) of 128-channel tiles that keeps two workgroups per CU; a forced
// form (BN << 8 | NB, A/B runs) when it fits.  0 when not eligible.
static int h9_form(const ConvArgs& a, int hb, int BNmax) {
    if (!g_conv_h9 || hb / 1024 > 4 * kH9MaxQ || a.N * a.cls[0].P * a.cls[0].Q >= (1 << 30) / 8) return 0;
    const int budget = 80 * 1024 - 256;
    auto fits = [&](int bn, int nb) { return bn <= BNmax && a.Nout % bn == 0 && hb + nb * bn * 128 <= budget; };
    if (g_conv_h9 > 1) {
        const int bn = g_conv_h9 >> 8, nb = g_conv_h9 & 255;
        return fits(bn, nb) ? g_conv_h9 : 0;
    }
    for (int nb = 3; nb >= 2; --nb)
        if (fits(128, nb)) return 128 << 8 | nb;
    return fits(64, 4) ? 64 << 8 | 4 : 0;
}

// k_conv_h9 when eligible (Nout a multiple of BN, at most 48 halo DMA instructions, splits
// over whole channel chunks).  Returns 1 when launched, 0 when not taken.
template <int BN>
static int try_h9(ConvArgs& a, int hb, hipStream_t st) {
    if (a.splits > (a.C >> 6)) return 0;
    const int f = h9_form(a, hb, BN);
    if (!f) return 0;
    switch (f) {
    case 128 << 8 | 2: return launch_h9<128, 2>(a, hb, st);
    case 128 << 8 | 3: return launch_h9<128, 3>(a, hb, st);
    case 64 << 8 | 3: return launch_h9<64, 3>(a, hb, st);
    case 64 << 8 | 4: return launch_h9<64, 4>(a, hb, st);
    case 64 << 8 | 5: return launch_h9<64, 5>(a, hb, st);
    default: return 0;
    }
}

template <int BN>
static int launch_halo(ConvArgs& a, int hb, hipStream_t st) {
    const int p = conv_pipe();
    if (p <= 0 || p == 3) {
        const int r = try_h9<BN>(a, hb, st);
        if (r == 1) return GM_OK;
        if (r != 0) return r;
    }
    // a third weight stage when two workgroups per CU still fit (or when asked: pipe 3)
    if (p == 3 || hb + 3 * BN * 128 <= 80 * 1024 - 256) return launch_halo_v<BN, 3>(a, hb, st);
    return launch_halo_v<BN, 2>(a, hb, st);
}

// 256-pixel halo tiles (one workgroup per CU, BN = 128): eligible when the double
// halo plus a 3-stage weight ring fits the CU's LDS.  Tiles too few to fill the chip
// split K (2-4 ways, >= 16 k-tiles each) through the turnstile when the workspace holds
// the 256x128 slabs.  Returns 0 when not taken.
struct Halo256Plan {
    int hb = 0;        // one halo buffer's LDS bytes (0: not taken)
    int tiles = 0, splits = 1;
    size_t ws = 0;     // split-K workspace bytes (turnstile words + 256x128 fp32 slabs)
};

// the 256-pixel form (gm_conv_set_halo(2)): shapes with fewer 256x128 tiles keep the 128-pixel form;
// K is split when the tiles do not fill the chip
static const int g_h256_mintiles = 192;
static const int g_h256_split = 1;

static Halo256Plan halo256_plan(const ConvArgs& a) {
    Halo256Plan p;
    if (g_conv_halo != 2 || a.Nout % 128) return p;
    const int hb = halo_bytes(a, 256);
    if (hb <= 0 || 2 * hb + 3 * 128 * 128 > 160 * 1024) return p;
    const int M = a.N * a.cls[0].P * a.cls[0].Q;
    p.tiles = (M + 255) / 256 * (a.Nout / 128);
    if (p.tiles < g_h256_mintiles) return p;
    p.hb = hb;
    const int nk = 9 * (a.C >> 6);
    int S = (p.tiles >= 192 || !g_h256_split) ? 1 : 256 / p.tiles;
    S = S > 4 ? 4 : S;
    while (S > 1 && nk / S < 16) --S;
    // waiters within the device's slots (one workgroup per CU here) per concurrent launch: see pick_tile
    const Residency& rs = residency();
    while (S > 1 && (long)p.tiles * (S - 1) > (long)usable_cus(conv_cus()) / (rs.streams * rs.sharers)) --S;
    if (p.tiles > kMaxSplitTiles) S = 1;
    p.splits = S;
    if (S > 1) p.ws = splitk_flag_bytes(p.tiles) + (size_t)p.tiles * 32 * 256 * 16;
    return p;
}

static int try_halo256(ConvArgs& a, hipStream_t st, void* ws, size_t ws_bytes) {
    const Halo256Plan pl = halo256_plan(a);
    if (pl.hb <= 0) return 0;
    const int hb = pl.hb, tiles = pl.tiles;
    int S = pl.splits;
    if (S > 1 && (!ws || ws_bytes < pl.ws)) S = 1;
    a.splits = S;
    a.xcd = 0;
    if (S > 1) {
        a.spin_limit = spin_limit();
        a.flags = static_cast<unsigned*>(ws);
        a.ws = reinterpret_cast<float*>(static_cast<char*>(ws) + splitk_flag_bytes(tiles));
    }
    const int rc = launch_halo_v<128, 3, 256>(a, hb, st);
    return rc == GM_OK ? 1 : rc;
}

static int pick_and_launch(ConvArgs& a, hipStream_t st, void* ws, size_t ws_bytes) {
    const bool three = stages() == 3;
    if (a.G < 1) a.G = 1;
    if (a.G == 1) {
        const int r = try_halo256(a, st, ws, ws_bytes);
        if (r == 1) return GM_OK;
        if (r != 0) return r;
    }
    {
        RwArgs r;
        const size_t lds = rw_plan(a, r);
        if (lds > 0) {
            a.stats_rows = rw_per(a, r);  // (a.stats: one partial row per workgroup)
            return launch_rw(a, r, lds, st);
        }
    }
    {
        StemArgs r;
        const size_t lds = stem_plan(a, r);
        if (lds > 0) return launch_stem(a, r, lds, st);  // (no statistics: r.stats null)
    }
    TilePick p = pick_tile(a);
    if (p.splits > 1 && (!ws || ws_bytes < splitk_bytes(p) || p.tiles > kMaxSplitTiles)) {  // the unsplit choice
        long M = 0;
        for (int i = 0; i < a.ncls; ++i) M += (long)a.N * a.cls[i].P * a.cls[i].Q * a.G;
        p = {M / 128 * ((a.Nout + 63) / 64) >= tile_bias() * 3 / 4 ? T128x64 : T64x64, 1, 0};
    }
    a.splits = p.splits;
    a.xcd = p.splits > 1 ? 0 : xcd_remap();  // split-K relies on split-major dispatch order
    if (p.splits > 1) {
        a.spin_limit = spin_limit();
        a.flags = static_cast<unsigned*>(ws);
        a.ws = reinterpret_cast<float*>(static_cast<char*>(ws) + splitk_flag_bytes(p.tiles));
    }
    const int hb = halo_bytes(a);
    const long long Mg = (long long)a.N * a.cls[0].P * a.cls[0].Q;
    a.stats_rows = (int)((Mg + 127) / 128);  // (a.stats: one partial row per 128-pixel tile)
    if (hb > 0 && hb + 2 * 128 * 128 <= 160 * 1024 && a.G > 1) {
        // view groups: k_conv_h9 when it takes the shape, else the lean kernel below
        if (p.tile != T128x128) a.splits = 1;
        const int r = (p.tile == T128x128 || a.Nout >= 128) ? try_h9<128>(a, hb, st) : try_h9<64>(a, hb, st);
        if (r == 1) return GM_OK;
        if (r != 0) return r;
        if (a.splits != p.splits) p.tile = a.Nout >= 128 ? T128x64 : T64x64;
    } else if (hb > 0 && hb + 2 * 128 * 128 <= 160 * 1024) {
        if (p.tile == T128x128) return launch_halo<128>(a, hb, st);
        a.splits = 1;  // (split-K is only chosen with 128x128 tiles)
        if (a.Nout >= 128) return launch_halo<128>(a, hb, st);
        return launch_halo<64>(a, hb, st);
    }
    if (p.tile == T64x64) a.stats_rows = (int)((Mg + 63) / 64);
    switch (p.tile) {
    case T128x128: return three ? launch_igemm<128, 128, 3>(a, st) : launch_igemm<128, 128, 2>(a, st);
    case T128x64: return three ? launch_igemm<128, 64, 3>(a, st) : launch_igemm<128, 64, 2>(a, st);
    default: return three ? launch_igemm<64, 64, 3>(a, st) : launch_igemm<64, 64, 2>(a, st);
    }
}

// the class's taps as a grid: rows r (stride-compatible with the class parity ph) and
// columns s (with pw); fwd is the st = 1 case with every (r, s) - same order as tw/dh/dw
static void set_grid(ConvCls& c, const gm_conv_desc* d, int st, int ph, int pw) {
    c.Rc = c.Sc = 0;
    for (int r = 0; r < d->R && c.Rc < 8; ++r) {
        if (((ph + d->pad - r) % st + st) % st) continue;
        c.cdh[c.Rc] = (signed char)((ph + d->pad - r) / st);
        c.crs[c.Rc++] = (unsigned char)(r * d->S);
    }
    for (int s = 0; s < d->S && c.Sc < 8; ++s) {
        if (((pw + d->pad - s) % st + st) % st) continue;
        c.cdw[c.Sc] = (signed char)((pw + d->pad - s) / st);
        c.cs[c.Sc++] = (unsigned char)s;
    }
    c.smag = c.Sc > 0 ? (256 + c.Sc - 1) / c.Sc : 0;
    c.fd_pq = FastDiv((uint32_t)(c.P * c.Q > 0 ? c.P * c.Q : 1));
    c.fd_q = FastDiv((uint32_t)(c.Q > 0 ? c.Q : 1));
    pack_grid(c, d->S);
}

// forward taps read dh = r - pad, i.e. the dgrad formula with st = 1 and a sign flip
static void set_grid_fwd(ConvCls& c, const gm_conv_desc_hw* d) {
    c.Rc = d->R < 8 ? d->R : 8;
    c.Sc = d->S < 8 ? d->S : 8;
    for (int r = 0; r < c.Rc; ++r) {
        c.cdh[r] = (signed char)(r - d->pad_h);
        c.crs[r] = (unsigned char)(r * d->S);
    }
    for (int s = 0; s < c.Sc; ++s) {
        c.cdw[s] = (signed char)(s - d->pad_w);
        c.cs[s] = (unsigned char)s;
    }
    c.smag = (256 + c.Sc - 1) / c.Sc;
    c.fd_pq = FastDiv((uint32_t)(c.P * c.Q));
    c.fd_q = FastDiv((uint32_t)c.Q);
    pack_grid(c, d->S);
}

static void pack_grid(ConvCls& c, int S) {
    c.dh0 = c.cdh[0];
    c.sh = c.Rc > 1 ? c.cdh[1] - c.cdh[0] : 1;
    c.dw0 = c.cdw[0];
    c.sw = c.Sc > 1 ? c.cdw[1] - c.cdw[0] : 1;
    c.pk_dh = c.pk_dw = c.pk_r = c.pk_s = 0;
    for (int i = 0; i < c.Rc; ++i) {
        c.pk_dh |= (unsigned)((c.cdh[i] + 8) & 15) << (4 * i);
        c.pk_r |= (unsigned)((c.crs[i] / S) & 15) << (4 * i);
    }
    for (int j = 0; j < c.Sc; ++j) {
        c.pk_dw |= (unsigned)((c.cdw[j] + 8) & 15) << (4 * j);
        c.pk_s |= (unsigned)(c.cs[j] & 15) << (4 * j);
    }
}

// the lean kernel's tap grid must reproduce the tap list exactly (order, offsets, weights)
static bool grid_ok(const ConvCls& c, int S) {
    if (c.Rc * c.Sc != c.ntap || c.Rc > 8 || c.Sc > 8) return false;
    if ((c.sh != 1 && c.sh != -1) || (c.sw != 1 && c.sw != -1)) return false;
    for (int i = 0; i < c.Rc; ++i)
        if (c.cdh[i] != c.dh0 + c.sh * i) return false;
    for (int j = 0; j < c.Sc; ++j)
        if (c.cdw[j] != c.dw0 + c.sw * j) return false;
    for (int t = 0; t < c.ntap; ++t) {
        const int i = (t * c.smag) >> 8, j = t - i * c.Sc;
        if (i != t / c.Sc) return false;
        const int dh = (int)((c.pk_dh >> (4 * i)) & 15u) - 8, dw = (int)((c.pk_dw >> (4 * j)) & 15u) - 8;
        const int tw = (int)((c.pk_r >> (4 * i)) & 15u) * S + (int)((c.pk_s >> (4 * j)) & 15u);
        if (dh != c.dh[t] || dw != c.dw[t] || tw != c.tw[t]) return false;
    }
    return true;
}

static int check_desc(const gm_conv_desc* d) {
    GM_REQUIRE(d && d->N > 0 && d->H > 0 && d->W > 0 && d->C > 0 && d->K > 0 && d->R > 0 && d->S > 0,
               "conv: empty shape");
    GM_REQUIRE(d->stride >= 1 && d->pad >= 0, "conv: bad stride/pad");
    GM_REQUIRE(d->R * d->S <= kMaxTap, "conv: at most %d taps", kMaxTap);
    GM_REQUIRE(ilog2(d->C) >= 3, "conv: C must be a power of two >= 8 (got %d)", d->C);
    GM_REQUIRE(d->K % 8 == 0, "conv: K must be a multiple of 8 (got %d)", d->K);
    return GM_OK;
}

static int check_desc_hw(const gm_conv_desc_hw* d) {
    GM_REQUIRE(d && d->N > 0 && d->H > 0 && d->W > 0 && d->C > 0 && d->K > 0 && d->R > 0 && d->S > 0,
               "conv: empty shape");
    GM_REQUIRE(d->stride_h >= 1 && d->stride_w >= 1 && d->pad_h >= 0 && d->pad_w >= 0, "conv: bad stride/pad");
    GM_REQUIRE(d->R * d->S <= kMaxTap, "conv: at most %d taps", kMaxTap);
    GM_REQUIRE(ilog2(d->C) >= 3, "conv: C must be a power of two >= 8 (got %d)", d->C);
    GM_REQUIRE(d->K % 8 == 0, "conv: K must be a multiple of 8 (got %d)", d->K);
    GM_REQUIRE(d->H + 2 * d->pad_h >= d->R && d->W + 2 * d->pad_w >= d->S, "conv: filter larger than input");
    return GM_OK;
}

static void fwd_setup(const gm_conv_desc_hw* d, const void* x, const void* w, void* y, ConvArgs& a) {
    const int P = (d->H + 2 * d->pad_h - d->R) / d->stride_h + 1;
    const int Q = (d->W + 2 * d->pad_w - d->S) / d->stride_w + 1;
    memset(&a, 0, sizeof(a));
    a.in = (const uint16_t*)x;
    a.wt = (const uint16_t*)w;
    a.N = d->N; a.Hi = d->H; a.Wi = d->W; a.C = d->C; a.logC = ilog2(d->C);
    a.Nout = d->K; a.T = d->R * d->S; a.Sw = d->S;
    a.Ho = P; a.Wo = Q; a.sAh = d->stride_h; a.sAw = d->stride_w;
    a.ncls = 1;
    a.G = 1;
    ConvCls& c = a.cls[0];
    c.out = (uint16_t*)y;
    c.P = P; c.Q = Q; c.oS = 1; c.oH = 0; c.oW = 0;
    c.ntap = d->R * d->S;
    for (int r = 0; r < d->R; ++r)
        for (int s = 0; s < d->S; ++s) {
            const int i = r * d->S + s;
            c.tw[i] = (short)i;
            c.dh[i] = (signed char)(r - d->pad_h);
            c.dw[i] = (signed char)(s - d->pad_w);
        }
    set_grid_fwd(c, d);
}

// returns false when some output pixels belong to no parity class (they must be zeroed)
static bool dgrad_setup(const gm_conv_desc* d, const void* dy, const void* wt, void* dx, ConvArgs& a) {
    const int st = d->stride;
    const int P = (d->H + 2 * d->pad - d->R) / st + 1;
    const int Q = (d->W + 2 * d->pad - d->S) / st + 1;
    memset(&a, 0, sizeof(a));
    a.in = (const uint16_t*)dy;
    a.wt = (const uint16_t*)wt;
    a.N = d->N; a.Hi = P; a.Wi = Q; a.C = d->K; a.logC = ilog2(d->K);
    a.Nout = d->C; a.T = d->R * d->S; a.Sw = d->S;
    a.Ho = d->H; a.Wo = d->W; a.sAh = a.sAw = 1;
    a.G = 1;
    bool full = true;
    for (int ph = 0; ph < st; ++ph)
        for (int pw = 0; pw < st; ++pw) {
            ConvCls& c = a.cls[a.ncls];
            c.out = (uint16_t*)dx;
            c.P = (d->H - ph + st - 1) / st;
            c.Q = (d->W - pw + st - 1) / st;
            c.oS = st; c.oH = ph; c.oW = pw;
            int n = 0;
            for (int r = 0; r < d->R; ++r) {
                if (((ph + d->pad - r) % st + st) % st) continue;
                for (int sx = 0; sx < d->S; ++sx) {
                    if (((pw + d->pad - sx) % st + st) % st) continue;
                    c.tw[n] = (short)(r * d->S + sx);
                    c.dh[n] = (signed char)((ph + d->pad - r) / st);
                    c.dw[n] = (signed char)((pw + d->pad - sx) / st);
                    ++n;
                }
            }
            c.ntap = n;
            if (n == 0 || c.P <= 0 || c.Q <= 0) { full = false; continue; }
            set_grid(c, d, st, ph, pw);
            ++a.ncls;
        }
    return full;
}

static int check_dgrad(const gm_conv_desc* d) {
    int rc = check_desc(d);
    if (rc) return rc;
    GM_REQUIRE(ilog2(d->K) >= 3, "conv dgrad: K must be a power of two >= 8 (got %d)", d->K);
    GM_REQUIRE(d->stride * d->stride <= kMaxCls, "conv dgrad: stride %d unsupported", d->stride);
    return GM_OK;
}

static gm_conv_desc_hw to_hw(const gm_conv_desc* d) {
    return gm_conv_desc_hw{d->N, d->H, d->W, d->C, d->K, d->R, d->S, d->stride, d->stride, d->pad, d->pad};
}

namespace gm {
unsigned conv_faults_read(bool clear) {
    unsigned v = 0;
    if (hipMemcpyFromSymbol(&v, HIP_SYMBOL(g_conv_fault), sizeof(v), 0, hipMemcpyDeviceToHost) != hipSuccess)
        return ~0u;
    if (clear && v) {
        const unsigned z = 0;
        (void)hipMemcpyToSymbol(HIP_SYMBOL(g_conv_fault), &z, sizeof(z), 0, hipMemcpyHostToDevice);
    }
    return v;
}
}  // namespace gm

extern "C" int gm_conv_set_splitk(int target) {
    GM_REQUIRE(target >= 0, "gm_conv_set_splitk: target must be >= 0");
    g_splitk_target = target;
    return GM_OK;
}

extern "C" int gm_conv_set_h9(int on) {
    g_conv_h9 = on;
    return GM_OK;
}


extern "C" int gm_conv_set_halo(int on) {
    g_conv_halo = on < 0 ? 0 : on > 2 ? 2 : on;
    return GM_OK;
}

extern "C" int gm_conv_set_stem(int on) {
    g_conv_stem = on ? 1 : 0;
    return GM_OK;
}

extern "C" int gm_conv_set_rw(int on) {
    g_conv_rw = on ? 1 : 0;  // 0: the layer-1 shapes take the im2col kernel
    return GM_OK;
}

extern "C" int gm_conv_set_pipe(int pipe) {
    GM_REQUIRE(pipe == -1 || pipe == 0 || pipe == 2 || pipe == 3, "gm_conv_set_pipe: -1 (default), 0, 2 or 3");
    g_conv_pipe = pipe;
    return GM_OK;
}


// 1x1 / s1 / p0 convolutions as plain GEMMs (conv1x1.hip, k_gemm_ring)
namespace gm {
bool conv1x1_ok(int R, int S, int sh, int sw, int ph, int pw, long long M, int Kr, int N);
bool conv1x1s_ok(int R, int S, int sh, int sw, int ph, int pw, long long M, int Kr, int N);
int conv1x1_gemm(long long M, int Kr, int N, int G, const void* A, long long gsA, const void* B, long long gsB,
                 void* out, long long gsO, const void* addend, hipStream_t st, const char* fn,
                 float* stats = nullptr, const uint16_t* bnx = nullptr, const float* bncoef = nullptr,
                 const float* bnmean = nullptr, const uint8_t* amask = nullptr, const int* sgeo = nullptr);
}  // namespace gm

extern "C" int gm_conv2d_fwd_hw_bf16(const gm_conv_desc_hw* d, const void* x, const void* w, void* y,
                                     void* stream) {
    int rc = check_desc_hw(d);
    if (rc) return rc;
    GM_REQUIRE(x && w && y, "conv fwd: null pointer");
    {
        const long long M = (long long)d->N * d->H * d->W;
        if (gm::conv1x1_ok(d->R, d->S, d->stride_h, d->stride_w, d->pad_h, d->pad_w, M, d->C, d->K))
            return gm::conv1x1_gemm(M, d->C, d->K, 1, x, 0, w, 0, y, 0, nullptr, as_stream(stream), "conv1x1 fwd");
    }
    ConvArgs a;
    fwd_setup(d, x, w, y, a);
    return pick_and_launch(a, as_stream(stream), nullptr, 0);
}

extern "C" int gm_conv2d_fwd_ex_bf16(const gm_conv_desc* d, const void* x, const void* w, void* y, void* ws,
                                     size_t ws_bytes, void* stream) {
    int rc = check_desc(d);
    if (rc) return rc;
    GM_REQUIRE(x && w && y, "conv fwd: null pointer");
    const gm_conv_desc_hw h = to_hw(d);
    {
        const long long M = (long long)d->N * d->H * d->W;
        if (gm::conv1x1_ok(d->R, d->S, d->stride, d->stride, d->pad, d->pad, M, d->C, d->K))
            return gm::conv1x1_gemm(M, d->C, d->K, 1, x, 0, w, 0, y, 0, nullptr, as_stream(stream), "conv1x1 fwd");
    }
    ConvArgs a;
    fwd_setup(&h, x, w, y, a);
    return pick_and_launch(a, as_stream(stream), ws, ws_bytes);
}

extern "C" int gm_conv2d_fwd_bf16(const gm_conv_desc* d, const void* x, const void* w, void* y, void* stream) {
    return gm_conv2d_fwd_ex_bf16(d, x, w, y, nullptr, 0, stream);
}

// G view groups in one launch: group g reads x + g*N*H*W*C with the weight w + g*w_stride
// and writes y + g*N*P*Q*K (the views stacked along the batch, one weight per view)
extern "C" int gm_conv2d_fwd_grouped_bf16(const gm_conv_desc_hw* d, int G, const void* x, const void* w,
                                          long long w_stride, void* y, void* ws, size_t ws_bytes, void* stream) {
    int rc = check_desc_hw(d);
    if (rc) return rc;
    GM_REQUIRE(x && w && y, "conv fwd: null pointer");
    GM_REQUIRE(G >= 1 && G <= 64, "conv fwd: view groups must be 1..64 (got %d)", G);
    GM_REQUIRE(G == 1 || w_stride >= (long long)d->K * d->R * d->S * d->C ||
                   -w_stride >= (long long)d->K * d->R * d->S * d->C,
               "conv fwd: group weight stride %lld shorter than one weight", w_stride);
    {
        const long long M = (long long)d->N * d->H * d->W;
        if (gm::conv1x1_ok(d->R, d->S, d->stride_h, d->stride_w, d->pad_h, d->pad_w, M, d->C, d->K))
            return gm::conv1x1_gemm(M, d->C, d->K, G, x, M * d->C, w, w_stride, y, M * d->K, nullptr,
                                    as_stream(stream), "conv1x1 fwd");
        const int P = (d->H - 1) / 2 + 1, Q = (d->W - 1) / 2 + 1;
        const long long Mo = (long long)d->N * P * Q;
        if (gm::conv1x1s_ok(d->R, d->S, d->stride_h, d->stride_w, d->pad_h, d->pad_w, Mo, d->C, d->K) &&
            M * d->C < (1ll << 30)) {  // the downsample: A rows gathered at stride 2
            const int geo[6] = {2, d->H, d->W, P, Q, 0};
            return gm::conv1x1_gemm(Mo, d->C, d->K, G, x, M * d->C, w, w_stride, y, Mo * d->K, nullptr,
                                    as_stream(stream), "conv1x1/s2 fwd", nullptr, nullptr, nullptr, nullptr, nullptr,
                                    geo);
        }
    }
    ConvArgs a;
    fwd_setup(d, x, w, y, a);
    a.G = G;
    a.gs_in = (long long)d->N * d->H * d->W * d->C;
    a.gs_wt = w_stride;
    a.gs_out = (long long)d->N * a.cls[0].P * a.cls[0].Q * d->K;
    return pick_and_launch(a, as_stream(stream), ws, ws_bytes);
}

// The stem convolution (k_conv_stem's shapes) with the BatchNorm statistics of its output
// accumulated in its epilogue: partial rows per workgroup, finalized by
// gm_bn_fwd_stats_finalize_grouped (no statistics pass over the 205 MB output).
// Forward convolution + the BatchNorm statistics of its stored output from the epilogue
// (include/greedymml.h).  The statistics buffer: an upper bound of the partial rows either
// statistics kernel takes for the shape.
extern "C" size_t gm_conv2d_fwd_bn_stats_floats(const gm_conv_desc_hw* d, int G) {
    if (check_desc_hw(d) || G < 1 || G > 64) return 0;
    ConvArgs a;
    fwd_setup(d, reinterpret_cast<const void*>(16), reinterpret_cast<const void*>(16), reinterpret_cast<void*>(16), a);
    a.G = G;
    const long long M = (long long)d->N * a.cls[0].P * a.cls[0].Q;
    long long rows = (M + 63) / 64;  // k_gemm_ring, 64-pixel tiles: one row per 64 pixels
    if (rows < 256) rows = 256;       // k_conv_rw, k_conv_stem: one per workgroup
    StemArgs r;
    if (stem_plan(a, r) > 0 && r.stats_rows > rows) rows = r.stats_rows;
    return (size_t)G * 2 * d->K * (size_t)(rows + 1);
}

extern "C" int gm_conv2d_fwd_grouped_bn_stats_bf16(const gm_conv_desc_hw* d, int G, const void* x, const void* w,
                                                   long long w_stride, void* y, float* stats, size_t stats_floats,
                                                   int* rows_out, void* ws, size_t ws_bytes, void* stream) {
    int rc = check_desc_hw(d);
    if (rc) return rc;
    GM_REQUIRE(x && w && y && stats && rows_out, "conv fwd bn stats: null pointer");
    GM_REQUIRE(G >= 1 && G <= 64, "conv fwd bn stats: view groups must be 1..64 (got %d)", G);
    GM_REQUIRE(G == 1 || w_stride >= (long long)d->K * d->R * d->S * d->C ||
                   -w_stride >= (long long)d->K * d->R * d->S * d->C,
               "conv fwd bn stats: group weight stride %lld shorter than one weight", w_stride);
    const size_t need = gm_conv2d_fwd_bn_stats_floats(d, G);
    GM_REQUIRE(stats_floats >= need, "conv fwd bn stats: %zu floats < %zu", stats_floats, need);
    ConvArgs a;
    fwd_setup(d, x, w, y, a);
    const long long M = (long long)d->N * a.cls[0].P * a.cls[0].Q;
    if (d->K % 64 != 0 || (size_t)M * d->K * 2 >= 0x7ffff000u) {
        set_error("conv fwd bn stats: K %% 64 != 0 or a group's output past 32-bit offsets");
        return GM_E_UNSUP;
    }
    if (gm::conv1x1_ok(d->R, d->S, d->stride_h, d->stride_w, d->pad_h, d->pad_w, M, d->C, d->K)) {
        *rows_out = (int)((M + 63) / 64);
        return gm::conv1x1_gemm(M, d->C, d->K, G, x, M * d->C, w, w_stride, y, M * d->K, nullptr,
                                as_stream(stream), "conv1x1 fwd", stats);
    }
    {
        const long long Mi = (long long)d->N * d->H * d->W;
        if (gm::conv1x1s_ok(d->R, d->S, d->stride_h, d->stride_w, d->pad_h, d->pad_w, M, d->C, d->K) &&
            Mi * d->C < (1ll << 30)) {  // the downsample: A rows gathered at stride 2 (M = output pixels)
            const int geo[6] = {2, d->H, d->W, a.cls[0].P, a.cls[0].Q, 0};
            *rows_out = (int)((M + 63) / 64);
            return gm::conv1x1_gemm(M, d->C, d->K, G, x, Mi * d->C, w, w_stride, y, M * d->K, nullptr,
                                    as_stream(stream), "conv1x1/s2 fwd", stats, nullptr, nullptr, nullptr, nullptr,
                                    geo);
        }
    }
    a.G = G;
    a.gs_in = (long long)d->N * d->H * d->W * d->C;
    a.gs_wt = w_stride;
    a.gs_out = M * d->K;
    // every view-grouped forward kernel stages its output tile through LDS (k_conv_rw,
    // store_tile_lds of k_conv_h9 / k_conv_igemm_ut; k_gemm_ring above), where the sums are a
    // few VALU per stored 16-B chunk.  (Summed in the MFMA layout instead - a 32-lane reduction
    // per value, one row per 64-pixel slab - they cost more than the statistics read: r05.)
    if (a.G < 2) {
        set_error("conv fwd bn stats: view groups (G >= 2) only");
        return GM_E_UNSUP;
    }
    StemArgs sr;
    if (stem_plan(a, sr) > 0) {  // the stem's statistics come from gm_conv2d_fwd_grouped_stats_bf16
        set_error("conv fwd bn stats: stem shapes take the stem statistics entry point");
        return GM_E_UNSUP;
    }
    a.stats = stats;
    rc = pick_and_launch(a, as_stream(stream), ws, ws_bytes);
    *rows_out = a.stats_rows;
    if (rc == GM_OK && a.stats_rows == 0) {  // a kernel without the staged epilogue ran
        set_error("conv fwd bn stats: the kernel chosen for this shape writes no statistics");
        return GM_E_UNSUP;
    }
    return rc;
}

extern "C" int gm_conv_stem_stats_rows(const gm_conv_desc_hw* d, int G) {
    if (check_desc_hw(d) || G < 1 || G > 64) return 0;
    ConvArgs a;
    fwd_setup(d, reinterpret_cast<const void*>(16), reinterpret_cast<const void*>(16), reinterpret_cast<void*>(16), a);
    a.G = G;
    StemArgs r;
    if (stem_plan(a, r) == 0 || a.Nout != 64) return 0;
    return r.stats_rows;
}

extern "C" int gm_conv2d_fwd_grouped_stats_bf16(const gm_conv_desc_hw* d, int G, const void* x, const void* w,
                                                long long w_stride, void* y, float* stats, int stats_rows,
                                                void* stream) {
    int rc = check_desc_hw(d);
    if (rc) return rc;
    GM_REQUIRE(x && w && y && stats, "conv fwd stats: null pointer");
    GM_REQUIRE(G >= 1 && G <= 64, "conv fwd stats: view groups must be 1..64 (got %d)", G);
    GM_REQUIRE(G == 1 || w_stride >= (long long)d->K * d->R * d->S * d->C ||
                   -w_stride >= (long long)d->K * d->R * d->S * d->C,
               "conv fwd stats: group weight stride %lld shorter than one weight", w_stride);
    ConvArgs a;
    fwd_setup(d, x, w, y, a);
    a.G = G;
    a.gs_in = (long long)d->N * d->H * d->W * d->C;
    a.gs_wt = w_stride;
    a.gs_out = (long long)d->N * a.cls[0].P * a.cls[0].Q * d->K;
    StemArgs r;
    const size_t lds = stem_plan(a, r);
    GM_REQUIRE(lds > 0 && a.Nout == 64, "conv fwd stats: only the stem kernel's shapes (64 output channels)");
    GM_REQUIRE(stats_rows == r.stats_rows, "conv fwd stats: stats_rows %d != gm_conv_stem_stats_rows %d",
               stats_rows, r.stats_rows);
    r.stats = stats;
    return launch_stem(a, r, lds, as_stream(stream));
}

// The input gradient with a masked gradient-join addend: dx = dgrad + (addend where the 1-bit mask
// is set) - the identity branch's dz = dy . [y > 0] of a block-output ReLU read from its dy and the
// BatchNorm forward's mask bits (batchnorm.hip) instead of a materialised dres.  dx != addend.
static int dgrad_grouped(const gm_conv_desc* d, int G, const void* dy, const void* wt, long long wt_stride, void* dx,
                         const void* addend, const uint8_t* amask, void* ws, size_t ws_bytes, void* stream);

extern "C" int gm_conv2d_dgrad_grouped_masked_bf16(const gm_conv_desc* d, int G, const void* dy, const void* wt,
                                                   long long wt_stride, void* dx, const void* addend,
                                                   const void* addend_mask, void* ws, size_t ws_bytes, void* stream) {
    GM_REQUIRE(addend && addend_mask, "conv dgrad masked: null addend or mask");
    GM_REQUIRE(addend != dx, "conv dgrad masked: the addend must not alias dx");
    GM_REQUIRE(d && d->C % 32 == 0, "conv dgrad masked: C must be a multiple of 32 (one mask dword per 32 channels)");
    return dgrad_grouped(d, G, dy, wt, wt_stride, dx, addend, static_cast<const uint8_t*>(addend_mask), ws, ws_bytes,
                         stream);
}

extern "C" int gm_conv2d_dgrad_grouped_bf16(const gm_conv_desc* d, int G, const void* dy, const void* wt,
                                            long long wt_stride, void* dx, const void* addend, void* ws,
                                            size_t ws_bytes, void* stream) {
    return dgrad_grouped(d, G, dy, wt, wt_stride, dx, addend, nullptr, ws, ws_bytes, stream);
}

static int dgrad_grouped(const gm_conv_desc* d, int G, const void* dy, const void* wt, long long wt_stride, void* dx,
                         const void* addend, const uint8_t* amask, void* ws, size_t ws_bytes, void* stream) {
    int rc = check_dgrad(d);
    if (rc) return rc;
    GM_REQUIRE(dy && wt && dx, "conv dgrad: null pointer");
    GM_REQUIRE(G >= 1 && G <= 64, "conv dgrad: view groups must be 1..64 (got %d)", G);
    GM_REQUIRE(G == 1 || wt_stride >= (long long)d->K * d->R * d->S * d->C ||
                   -wt_stride >= (long long)d->K * d->R * d->S * d->C,
               "conv dgrad: group weight stride %lld shorter than one weight", wt_stride);
    const int P = (d->H + 2 * d->pad - d->R) / d->stride + 1;
    const int Q = (d->W + 2 * d->pad - d->S) / d->stride + 1;
    {
        const long long M = (long long)d->N * d->H * d->W;
        if (gm::conv1x1_ok(d->R, d->S, d->stride, d->stride, d->pad, d->pad, M, d->K, d->C))
            return gm::conv1x1_gemm(M, d->K, d->C, G, dy, M * d->K, wt, wt_stride, dx, M * d->C, addend,
                                    as_stream(stream), "conv1x1 dgrad", nullptr, nullptr, nullptr, nullptr, amask);
        const long long Mo = (long long)d->N * P * Q;
        if (d->stride == 2 && gm::conv1x1s_ok(d->R, d->S, 2, 2, d->pad, d->pad, Mo, d->K, d->C) &&
            M * d->C < (1ll << 30)) {
            // the downsample's input gradient: dy rows dense, out rows scattered to the even pixels; the
            // others hold the (masked) addend or zero - one pass over dx unless the addend is dx itself
            hipStream_t s = as_stream(stream);
            if (addend != dx) {
                const size_t n = (size_t)G * M * d->C;
                k_zero_bf16<<<(int)((n / 8 + 255) / 256 < 4096 ? (n / 8 + 255) / 256 : 4096), 256, 0, s>>>(
                    (uint16_t*)dx, n, (const uint16_t*)addend, addend ? amask : nullptr);
                if ((rc = check_launch("k_zero_bf16"))) return rc;
            }
            const int geo[6] = {2, d->H, d->W, P, Q, 1};
            return gm::conv1x1_gemm(Mo, d->K, d->C, G, dy, Mo * d->K, wt, wt_stride, dx, M * d->C,
                                    addend ? dx : nullptr, s, "conv1x1/s2 dgrad", nullptr, nullptr, nullptr, nullptr,
                                    nullptr, geo);
        }
    }
    ConvArgs a;
    const bool full = dgrad_setup(d, dy, wt, dx, a);
    a.G = G;
    a.gs_in = (long long)d->N * P * Q * d->K;
    a.gs_wt = wt_stride;
    a.gs_out = (long long)d->N * d->H * d->W * d->C;
    a.addend = (const uint16_t*)addend;
    a.amask = addend ? amask : nullptr;
    hipStream_t s = as_stream(stream);
    if (!full && addend != dx) {  // the groups are contiguous: one pass zeroes (or copies) them all
        const size_t n = (size_t)G * d->N * d->H * d->W * d->C;
        k_zero_bf16<<<(int)((n / 8 + 255) / 256 < 4096 ? (n / 8 + 255) / 256 : 4096), 256, 0, s>>>(
            (uint16_t*)dx, n, (const uint16_t*)addend, a.amask);
        rc = check_launch("k_zero_bf16");
        if (rc) return rc;
    }
    return pick_and_launch(a, s, ws, ws_bytes);
}

// Input gradient + the statistics of the BatchNorm backward that consumes it (include/
// greedymml.h): the partial rows of (sum dz, sum dz (x - mean)) from the LDS-staged epilogue
// (k_conv_rw, k_conv_h9, k_conv_igemm_ut), then G x 4C floats for the backward's coefficients
// (gm_bn_bwd_stats_finalize_grouped / gm_bn_bwd_apply_grouped_bf16).
extern "C" size_t gm_conv2d_dgrad_bn_stats_floats(const gm_conv_desc* d, int G) {
    if (check_desc(d) || G < 1 || G > 64) return 0;
    const long long M = (long long)d->N * d->H * d->W;
    long long rows = (M + 63) / 64;  // 64 x 64 tiles: one row per 64 pixels
    if (rows < 256) rows = 256;      // k_conv_rw: one per workgroup
    return (size_t)G * 2 * d->C * (size_t)(rows + 1) + (size_t)G * 4 * d->C;
}

extern "C" int gm_conv2d_dgrad_grouped_bn_stats_bf16(const gm_conv_desc* d, int G, const void* dy, const void* wt,
                                                     long long wt_stride, void* dx, const void* bn_x,
                                                     const float* bn_coef, const float* bn_mean, float* stats,
                                                     size_t stats_floats, int* rows_out, void* ws, size_t ws_bytes,
                                                     void* stream) {
    int rc = check_dgrad(d);
    if (rc) return rc;
    GM_REQUIRE(dy && wt && dx && bn_x && bn_coef && bn_mean && stats && rows_out, "conv dgrad bn stats: null pointer");
    GM_REQUIRE(G >= 1 && G <= 64, "conv dgrad bn stats: view groups must be 1..64 (got %d)", G);
    GM_REQUIRE(G == 1 || wt_stride >= (long long)d->K * d->R * d->S * d->C ||
                   -wt_stride >= (long long)d->K * d->R * d->S * d->C,
               "conv dgrad bn stats: group weight stride %lld shorter than one weight", wt_stride);
    const size_t need = gm_conv2d_dgrad_bn_stats_floats(d, G);
    GM_REQUIRE(stats_floats >= need, "conv dgrad bn stats: %zu floats < %zu", stats_floats, need);
    const long long M = (long long)d->N * d->H * d->W;
    // one dense output class (stride 1: the parity classes of a strided input gradient would
    // share tile rows), view groups, 64-channel slices, 32-bit offsets
    if (d->stride != 1 || G < 2 || d->C % 64 != 0 || (size_t)M * d->C * 2 >= 0x7ffff000u) {
        set_error("conv dgrad bn stats: stride 1, G >= 2, C %% 64 == 0, 32-bit offsets only");
        return GM_E_UNSUP;
    }
    if (gm::conv1x1_ok(d->R, d->S, d->stride, d->stride, d->pad, d->pad, M, d->K, d->C)) {  // k_gemm_ring
        *rows_out = (int)((M + 63) / 64);
        return gm::conv1x1_gemm(M, d->K, d->C, G, dy, M * d->K, wt, wt_stride, dx, M * d->C, nullptr,
                                as_stream(stream), "conv1x1 dgrad", stats, static_cast<const uint16_t*>(bn_x),
                                bn_coef, bn_mean);
    }
    ConvArgs a;
    const bool full = dgrad_setup(d, dy, wt, dx, a);
    StemArgs sr;
    if (!full || a.ncls != 1 || stem_plan(a, sr) > 0) {
        set_error("conv dgrad bn stats: one dense output class only");
        return GM_E_UNSUP;
    }
    a.G = G;
    a.gs_in = M * d->K;
    a.gs_wt = wt_stride;
    a.gs_out = M * d->C;
    a.stats = stats;
    a.bnx = static_cast<const uint16_t*>(bn_x);
    a.bncoef = bn_coef;
    a.bnmean = bn_mean;
    rc = pick_and_launch(a, as_stream(stream), ws, ws_bytes);
    *rows_out = a.stats_rows;
    return rc;
}

extern "C" int gm_conv2d_dgrad_add_bf16(const gm_conv_desc* d, const void* dy, const void* wt, void* dx,
                                        const void* addend, void* ws, size_t ws_bytes, void* stream) {
    int rc = check_dgrad(d);
    if (rc) return rc;
    GM_REQUIRE(dy && wt && dx, "conv dgrad: null pointer");
    // addend == dx (in place) is allowed: every epilogue loads an output element's addend
    // and stores that element from the same thread, and pixels no parity class covers
    // then simply keep the addend (no zero / copy pass)
    {
        const long long M = (long long)d->N * d->H * d->W;
        if (gm::conv1x1_ok(d->R, d->S, d->stride, d->stride, d->pad, d->pad, M, d->K, d->C))
            return gm::conv1x1_gemm(M, d->K, d->C, 1, dy, 0, wt, 0, dx, 0, addend, as_stream(stream),
                                    "conv1x1 dgrad");
    }
    ConvArgs a;
    const bool full = dgrad_setup(d, dy, wt, dx, a);
    a.addend = (const uint16_t*)addend;
    hipStream_t s = as_stream(stream);
    if (!full && addend != dx) {
        const size_t n = (size_t)d->N * d->H * d->W * d->C;
        k_zero_bf16<<<(int)((n / 8 + 255) / 256 < 4096 ? (n / 8 + 255) / 256 : 4096), 256, 0, s>>>(
            (uint16_t*)dx, n, (const uint16_t*)addend);
        rc = check_launch("k_zero_bf16");
        if (rc) return rc;
    }
    return pick_and_launch(a, s, ws, ws_bytes);
}

extern "C" int gm_conv2d_dgrad_ex_bf16(const gm_conv_desc* d, const void* dy, const void* wt, void* dx, void* ws,
                                       size_t ws_bytes, void* stream) {
    return gm_conv2d_dgrad_add_bf16(d, dy, wt, dx, nullptr, ws, ws_bytes, stream);
}

extern "C" int gm_conv2d_dgrad_bf16(const gm_conv_desc* d, const void* dy, const void* wt, void* dx,
                                    void* stream) {
    return gm_conv2d_dgrad_ex_bf16(d, dy, wt, dx, nullptr, 0, stream);
}

extern "C" size_t gm_conv2d_splitk_ws_bytes_grouped(const gm_conv_desc* d, int G, int dgrad) {
    ConvArgs a;
    if (G < 1) return 0;
    if (dgrad) {
        if (check_dgrad(d)) return 0;
        dgrad_setup(d, nullptr, nullptr, nullptr, a);
    } else {
        if (check_desc(d)) return 0;
        const gm_conv_desc_hw h = to_hw(d);
        fwd_setup(&h, nullptr, nullptr, nullptr, a);
    }
    a.G = G;
    const size_t b128 = splitk_bytes(pick_tile(a)), b256 = G == 1 ? halo256_plan(a).ws : 0;
    return b128 > b256 ? b128 : b256;
}

extern "C" size_t gm_conv2d_splitk_ws_bytes(const gm_conv_desc* d, int dgrad) {
    return gm_conv2d_splitk_ws_bytes_grouped(d, 1, dgrad);
}

extern "C" int gm_conv_weight_transpose_bf16(const void* w, void* wt, int Co, int T, int Ci, void* stream) {
    GM_REQUIRE(w && wt && Co > 0 && T > 0 && Ci > 0, "weight transpose: bad args");
    const int n = Co * T * Ci;
    k_transpose_w<<<(n + 255) / 256, 256, 0, as_stream(stream)>>>((const uint16_t*)w, (uint16_t*)wt, Co, T, Ci);
    return check_launch("k_transpose_w");
}

// fp32 master weight [K][RS][C] (KRSC) -> bf16 [K][RS][Cp] (channels zero-padded to Cp)
// and, optionally, the channel-transposed bf16 copy [Cp][RS][K] used by dgrad: one pass
// instead of a cast + a transpose per convolution.
__global__ void k_weight_prep(const float* __restrict__ w, int K, int RS, int C, int Cp,
                              uint16_t* __restrict__ wb, uint16_t* __restrict__ wt) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    const int n = K * RS * Cp;
    if (i >= n) return;
    const int c = i % Cp, t = (i / Cp) % RS, k = i / (Cp * RS);
    const float v = c < C ? w[((size_t)k * RS + t) * C + c] : 0.f;
    const uint16_t h = gm::Elem<uint16_t>::f2bf(v);
    wb[i] = h;
    if (wt) wt[((size_t)c * RS + t) * K + k] = h;
}

extern "C" int gm_conv_weight_prep_bf16(const float* w, int K, int RS, int C, int Cp, void* wb, void* wt,
                                        void* stream) {
    GM_REQUIRE(w && wb && K > 0 && RS > 0 && C > 0 && Cp >= C, "weight prep: bad args");
    const int n = K * RS * Cp;
    k_weight_prep<<<(n + 255) / 256, 256, 0, gm::as_stream(stream)>>>(w, K, RS, C, Cp, (uint16_t*)wb,
                                                                       (uint16_t*)wt);
    return gm::check_launch("k_weight_prep");
}

// Multi-tensor weight prep: every trunk convolution of a step in ONE launch.  One
// workgroup per 64(k) x 64(c) tile of one tap of one weight: fp32 loads coalesced
// along c, the bf16 KRSC copy written along c, the tile transposed through LDS so the
// [C][RS][K] dgrad copy is also written along k.
__global__ __launch_bounds__(256) void k_wprep_multi(const gm_wprep* __restrict__ tab, int n) {
    __shared__ uint16_t tile[64][66];  // 132-B rows: the transposed column reads are conflict-free
    const int blk = blockIdx.x;
    int lo = 0, hi = n - 1;  // last entry whose tile_start <= blk (uniform: scalar loads)
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (tab[mid].tile_start <= blk) lo = mid;
        else hi = mid - 1;
    }
    const float* w = tab[lo].w;
    uint16_t* wb = static_cast<uint16_t*>(tab[lo].wb);
    uint16_t* wt = static_cast<uint16_t*>(tab[lo].wt);
    const int K = tab[lo].K, RS = tab[lo].RS, C = tab[lo].C, Cp = tab[lo].Cp;
    int r = blk - tab[lo].tile_start;
    const int tc = (Cp + 63) >> 6;
    const int ci = r % tc;
    r /= tc;
    const int tap = r % RS, k0 = (r / RS) * 64, c0 = ci * 64;
    // 8 consecutive elements per thread and step: two float4 loads along c, one 16-B bf16 store
    // (vector forms where the whole run is in range and aligned, element-wise otherwise)
    const bool vc = (C & 3) == 0 && (Cp & 7) == 0 && ((uintptr_t)w & 15) == 0 && ((uintptr_t)wb & 15) == 0;
    for (int i = threadIdx.x; i < 64 * 8; i += 256) {
        const int kk = i >> 3, cq = (i & 7) * 8;
        const int k = k0 + kk, c = c0 + cq;
        uint16_t h[8];
        const float* src = w + ((size_t)k * RS + tap) * C + c;
        if (vc && k < K && c + 8 <= C) {
            const float4 u0 = reinterpret_cast<const float4*>(src)[0], u1 = reinterpret_cast<const float4*>(src)[1];
            const float f[8] = {u0.x, u0.y, u0.z, u0.w, u1.x, u1.y, u1.z, u1.w};
#pragma unroll
            for (int j = 0; j < 8; ++j) h[j] = gm::Elem<uint16_t>::f2bf(f[j]);
        } else {
#pragma unroll
            for (int j = 0; j < 8; ++j) h[j] = gm::Elem<uint16_t>::f2bf((k < K && c + j < C) ? src[j] : 0.f);
        }
        if (k < K) {
            uint16_t* dst = wb + ((size_t)k * RS + tap) * Cp + c;
            if (vc && c + 8 <= Cp) {
                *reinterpret_cast<uint4*>(dst) =
                    make_uint4(h[0] | (uint32_t)h[1] << 16, h[2] | (uint32_t)h[3] << 16, h[4] | (uint32_t)h[5] << 16,
                               h[6] | (uint32_t)h[7] << 16);
            } else {
#pragma unroll
                for (int j = 0; j < 8; ++j)
                    if (c + j < Cp) dst[j] = h[j];
            }
        }
        uint32_t* row = reinterpret_cast<uint32_t*>(&tile[kk][cq]);
#pragma unroll
        for (int j = 0; j < 4; ++j) row[j] = h[2 * j] | (uint32_t)h[2 * j + 1] << 16;
    }
    if (!wt) return;
    __syncthreads();
    // the [C][RS][K] copy: 8 consecutive k of one c per thread and step, one 16-B store
    const bool vk = (K & 7) == 0 && ((uintptr_t)wt & 15) == 0;
    for (int i = threadIdx.x; i < 64 * 8; i += 256) {
        const int cc = i >> 3, kq = (i & 7) * 8;
        const int k = k0 + kq, c = c0 + cc;
        if (c >= Cp) continue;
        uint16_t h[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) h[j] = tile[kq + j][cc];
        uint16_t* dst = wt + ((size_t)c * RS + tap) * K + k;
        if (vk && k + 8 <= K) {
            *reinterpret_cast<uint4*>(dst) =
                make_uint4(h[0] | (uint32_t)h[1] << 16, h[2] | (uint32_t)h[3] << 16, h[4] | (uint32_t)h[5] << 16,
                           h[6] | (uint32_t)h[7] << 16);
        } else {
#pragma unroll
            for (int j = 0; j < 8; ++j)
                if (k + j < K) dst[j] = h[j];
        }
    }
}

extern "C" int gm_wprep_tiles(int K, int RS, int Cp) {
    if (K <= 0 || RS <= 0 || Cp <= 0) return 0;
    return ((K + 63) / 64) * RS * ((Cp + 63) / 64);
}

extern "C" int gm_conv_weight_prep_multi_bf16(const gm_wprep* table, int n, int total_tiles, void* stream) {
    GM_REQUIRE(table && n > 0 && total_tiles > 0, "weight prep multi: bad args");
    k_wprep_multi<<<total_tiles, 256, 0, gm::as_stream(stream)>>>(table, n);
    return gm::check_launch("k_wprep_multi");
}
