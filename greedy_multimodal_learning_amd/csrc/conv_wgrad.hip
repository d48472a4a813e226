// bf16 convolution weight gradient on MFMA (gfx950), NHWC activations.
//
//   dw[k, t, c] = sum_{b,p,q} dy[b,p,q,k] * x[b, p*st + r_t - pad, q*st + s_t - pad, c]
//
// GEMM view: rows = output channels k, columns = (tap, c), reduction over the
// B*P*Q output pixels.  Both operands arrive pixel-major (channels contiguous), so
// the 64-pixel x 64-channel tiles are staged in LDS as [pixel][channel] rows and
// the MFMA fragments (8 consecutive pixels per lane) are read with the gfx950
// hardware-transpose load ds_read_b64_tr_b16 (two 4-row reads per fragment).  The
// LDS row pitch is 192 B (128 B payload): for the tr read's 4-row x 16-column
// blocks this puts the 8 (row, column-block) pieces of a 32-lane half on 8
// distinct 8-bank groups, i.e. conflict-free.  Tiles 64 x 64 per workgroup (2x2
// waves of 32x32, v_mfma_f32_32x32x16_bf16), double-buffered register-staged
// loads, split-K over pixels into fp32 partial slabs, then a fixed-order reduce
// (deterministic, no atomics).
#include <cstring>

#include "gm_common.h"

namespace gm {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short short4_t __attribute__((ext_vector_type(4)));
typedef short short8_t __attribute__((ext_vector_type(8)));
typedef float floatx16 __attribute__((ext_vector_type(16)));

constexpr int kWTap = 49;
constexpr int kPitch = 96;      // LDS row pitch in bf16 elements (192 B)

struct WgradArgs {
    const uint16_t* dy;         // [N][P][Q][Kc]
    const uint16_t* x;          // [N][H][W][C]
    float* part;                // [splits][Kc][T*C]
    int N, H, W, C, logC, Kc, T, P, Q, st;
    int tiles_k, tiles_n, splits, steps_per_split;  // steps of 64 pixels
    FastDiv fd_pq, fd_q;        // pixel -> (b, p, q) without integer division
    signed char dh[kWTap], dw[kWTap];
};

typedef __attribute__((address_space(3))) short4_t lds_s4;

__device__ __forceinline__ bf16x8 tr_frag(const uint16_t* base_row0, const uint16_t* base_row4) {
    const short4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)base_row0);
    const short4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)base_row4);
    const short8_t s = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
    return __builtin_bit_cast(bf16x8, s);
}

__global__ __launch_bounds__(256) void k_conv_wgrad(WgradArgs a) {
    constexpr int BK = 64;  // pixels per step
    __shared__ __attribute__((aligned(16))) uint16_t lds[2][2][BK * kPitch];  // [buf][A|B]
    __shared__ int tapt[kWTap];
    const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
    const int wm = wave >> 1, wn = wave & 1;
    int bid = blockIdx.x;
    const int split = bid % a.splits;
    bid /= a.splits;
    const int tk = bid % a.tiles_k, tn = bid / a.tiles_k;
    const int k0 = tk * 64, n0 = tn * 64;
#pragma unroll
    for (int i = 0; i < kWTap; ++i)
        if (t == i && i < a.T) tapt[i] = ((int)(a.dh[i] + 128)) | ((int)(a.dw[i] + 128) << 8);
    __syncthreads();
    const int PQ = a.P * a.Q;
    const int M = a.N * PQ;
    const int step0 = split * a.steps_per_split;
    const int step1 = min((M + BK - 1) / BK, step0 + a.steps_per_split);
    const int lchunk = t & 7, lrow = t >> 3;  // 8 loaders per 64-channel row, rows lrow, lrow+32
    // B column chunk geometry (fixed for the workgroup): col = n0 + 8*lchunk -> (tap, c)
    const int colk = n0 + lchunk * 8;
    const int btap = colk >> a.logC, bc = colk & (a.C - 1);
    const int te = tapt[btap < a.T ? btap : 0];
    const int bdh = (te & 0xff) - 128, bdw = ((te >> 8) & 0xff) - 128;
    const bool bcol_ok = colk < a.T * a.C;
    const bool acol_ok = (k0 + lchunk * 8) < a.Kc;

    uint4 ra[2], rb[2];
    auto load = [&](int step) {
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const int m = step * BK + lrow + 32 * i;
            uint4 va = make_uint4(0, 0, 0, 0), vb = make_uint4(0, 0, 0, 0);
            if (m < M) {
                if (acol_ok) va = *(const uint4*)(a.dy + (size_t)m * a.Kc + k0 + lchunk * 8);
                const int b = (int)a.fd_pq.div((uint32_t)m), pq = m - b * PQ;
                const int p = (int)a.fd_q.div((uint32_t)pq), q = pq - p * a.Q;
                const int hi = p * a.st + bdh, wi = q * a.st + bdw;
                if (bcol_ok && (unsigned)hi < (unsigned)a.H && (unsigned)wi < (unsigned)a.W)
                    vb = *(const uint4*)(a.x + ((size_t)((b * a.H + hi) * a.W + wi) << a.logC) + bc);
            }
            ra[i] = va;
            rb[i] = vb;
        }
    };
    auto store = [&](int buf) {
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const int row = lrow + 32 * i;
            *(uint4*)&lds[buf][0][row * kPitch + lchunk * 8] = ra[i];
            *(uint4*)&lds[buf][1][row * kPitch + lchunk * 8] = rb[i];
        }
    };
    floatx16 acc;
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] = 0.f;
    // tr-read lane geometry: group g = lane>>4 reads rows 8*(g>>1)+q (+4), cols 16*(g&1)+4p
    const int g = lane >> 4, i16 = lane & 15, q4 = i16 >> 2, p4 = i16 & 3;
    const int rbase = 8 * (g >> 1) + q4;
    const int acol = wm * 32 + 16 * (g & 1) + 4 * p4;
    const int bcol = wn * 32 + 16 * (g & 1) + 4 * p4;
    if (step0 < step1) {
        load(step0);
        store(0);
    }
    __syncthreads();
    for (int s = step0; s < step1; ++s) {
        const int buf = (s - step0) & 1;
        if (s + 1 < step1) load(s + 1);
        const uint16_t* A = lds[buf][0];
        const uint16_t* Bm = lds[buf][1];
#pragma unroll
        for (int ks = 0; ks < 4; ++ks) {
            const int r0 = ks * 16 + rbase;
            const bf16x8 af = tr_frag(A + r0 * kPitch + acol, A + (r0 + 4) * kPitch + acol);
            const bf16x8 bf = tr_frag(Bm + r0 * kPitch + bcol, Bm + (r0 + 4) * kPitch + bcol);
            acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af, bf, acc, 0, 0, 0);
        }
        if (s + 1 < step1) store(buf ^ 1);
        __syncthreads();
    }
    // D[k][c]: col = lane&31 (c), row = (r&3) + 8(r>>2) + 4(lane>>5) (k)
    const int TC = a.T * a.C;
    float* out = a.part + (size_t)split * a.Kc * TC;
    const int col = n0 + wn * 32 + (lane & 31);
    if (col < TC) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int row = k0 + wm * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
            if (row < a.Kc) out[(size_t)row * TC + col] = acc[r];
        }
    }
}

// stage 1 (many splits): part2[g][i] = sum of splits 8g..8g+7 (fixed order), float4 lanes,
// grid (slab/1024, groups): parallel over splits so the reduce is bandwidth-, not latency-bound
__global__ __launch_bounds__(256) void k_wgrad_sum8(const float* part, int splits, size_t slab, float* part2) {
    const size_t i4 = ((size_t)blockIdx.x * 256 + threadIdx.x) * 4;
    if (i4 >= slab) return;
    const int g = blockIdx.y, s0 = g * 8, s1 = min(splits, s0 + 8);
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int s = s0; s < s1; ++s) {
        const float4 v = *(const float4*)(part + (size_t)s * slab + i4);
        acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
    }
    *(float4*)(part2 + (size_t)g * slab + i4) = acc;
}

// dw = sum over splits (fixed order); also the [K][T][Cpad] -> [K][T][Creal] crop
__global__ __launch_bounds__(256) void k_wgrad_reduce(const float* part, int splits, int Kc, int T, int Cp,
                                                      int Cr, int accumulate, float* dw) {
    const size_t n = (size_t)Kc * T * Cr;
    const size_t slab = (size_t)Kc * T * Cp;
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
        const size_t c = i % Cr, kt = i / Cr;
        const size_t src = kt * Cp + c;
        float v = 0.f;
        for (int s = 0; s < splits; ++s) v += part[s * slab + src];
        dw[i] = accumulate ? dw[i] + v : v;
    }
}

static int ilog2w(int v) {
    int l = 0;
    while ((1 << l) < v) ++l;
    return (1 << l) == v ? l : -1;
}

static void plan(const gm_conv_desc* d, int& P, int& Q, int& tiles_k, int& tiles_n, int& splits, int& sps) {
    P = (d->H + 2 * d->pad - d->R) / d->stride + 1;
    Q = (d->W + 2 * d->pad - d->S) / d->stride + 1;
    const int M = d->N * P * Q;
    const int steps = (M + 63) / 64;
    tiles_k = (d->K + 63) / 64;
    tiles_n = (d->R * d->S * d->C + 63) / 64;
    const int tiles = tiles_k * tiles_n;
    int want = (1024 + tiles - 1) / tiles;           // ~1024 workgroups
    if (want > steps / 4) want = steps / 4 > 0 ? steps / 4 : 1;  // >= 4 steps per split
    if (want < 1) want = 1;
    sps = (steps + want - 1) / want;
    splits = (steps + sps - 1) / sps;
}

}  // namespace gm

using namespace gm;

extern "C" size_t gm_conv2d_wgrad_scratch(const gm_conv_desc* d) {
    if (!d) return 0;
    int P, Q, tk, tn, sp, sps;
    plan(d, P, Q, tk, tn, sp, sps);
    const size_t slab = (size_t)d->K * d->R * d->S * d->C;
    const int groups = sp > 8 ? (sp + 7) / 8 : 0;
    return (size_t)(sp + groups) * slab * sizeof(float);
}

extern "C" int gm_conv2d_wgrad_bf16(const gm_conv_desc* d, const void* dy, const void* x, float* dw, int c_real,
                                    int accumulate, void* scratch, size_t scratch_bytes, void* stream) {
    GM_REQUIRE(d && dy && x && dw, "conv wgrad: null pointer");
    GM_REQUIRE(d->R * d->S <= kWTap, "conv wgrad: at most %d taps", kWTap);
    GM_REQUIRE(ilog2w(d->C) >= 3, "conv wgrad: C must be a power of two >= 8");
    GM_REQUIRE(d->K % 8 == 0, "conv wgrad: K must be a multiple of 8");
    GM_REQUIRE(c_real >= 1 && c_real <= d->C, "conv wgrad: bad c_real");
    const size_t need = gm_conv2d_wgrad_scratch(d);
    GM_REQUIRE(scratch && scratch_bytes >= need, "conv wgrad: scratch %zu < %zu", scratch_bytes, need);
    WgradArgs a;
    memset(&a, 0, sizeof(a));
    plan(d, a.P, a.Q, a.tiles_k, a.tiles_n, a.splits, a.steps_per_split);
    a.dy = (const uint16_t*)dy;
    a.x = (const uint16_t*)x;
    a.part = (float*)scratch;
    a.N = d->N; a.H = d->H; a.W = d->W; a.C = d->C; a.logC = ilog2w(d->C);
    a.Kc = d->K; a.T = d->R * d->S; a.st = d->stride;
    a.fd_pq = FastDiv((uint32_t)(a.P * a.Q));
    a.fd_q = FastDiv((uint32_t)a.Q);
    for (int r = 0; r < d->R; ++r)
        for (int s = 0; s < d->S; ++s) {
            a.dh[r * d->S + s] = (signed char)(r - d->pad);
            a.dw[r * d->S + s] = (signed char)(s - d->pad);
        }
    hipStream_t st = as_stream(stream);
    const int grid = a.tiles_k * a.tiles_n * a.splits;
    k_conv_wgrad<<<grid, 256, 0, st>>>(a);
    int rc = check_launch("k_conv_wgrad");
    if (rc) return rc;
    const size_t n = (size_t)d->K * a.T * c_real;
    int g = (int)((n + 255) / 256);
    if (g > 4096) g = 4096;
    const size_t slab = (size_t)d->K * a.T * d->C;
    const float* src = a.part;
    int nsrc = a.splits;
    if (a.splits > 8) {
        const int groups = (a.splits + 7) / 8;
        float* part2 = a.part + (size_t)a.splits * slab;
        dim3 g1((unsigned)((slab / 4 + 255) / 256), groups);
        k_wgrad_sum8<<<g1, 256, 0, st>>>(a.part, a.splits, slab, part2);
        rc = check_launch("k_wgrad_sum8");
        if (rc) return rc;
        src = part2;
        nsrc = groups;
    }
    k_wgrad_reduce<<<g, 256, 0, st>>>(src, nsrc, d->K, a.T, d->C, c_real, accumulate, dw);
    return check_launch("k_wgrad_reduce");
}
