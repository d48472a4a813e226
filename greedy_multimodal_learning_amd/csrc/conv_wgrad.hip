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
#include <algorithm>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <type_traits>
#include <utility>

#include "gm_common.h"

namespace gm {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short short4_t __attribute__((ext_vector_type(4)));
typedef short short8_t __attribute__((ext_vector_type(8)));
typedef float floatx16 __attribute__((ext_vector_type(16)));

constexpr int kWTap = 49;

struct WgradArgs {
    const uint16_t* dy;         // [N][P][Q][Kc]
    const uint16_t* x;          // [N][H][W][C]
    float* part;                // [splits][Kc][T*C]
    int N, H, W, C, logC, Kc, T, P, Q, sth, stw;
    int tiles_k, tiles_n, splits, steps_per_split;  // steps of 64 pixels
    FastDiv fd_pq, fd_q;        // pixel -> (b, p, q) without integer division
    int accumulate;             // k_conv_wgrad4 with one split: add into part (= dw) instead of storing
    int S, padh, padw;          // k_conv_wgrad4 decodes taps arithmetically
    int adv_b, adv_p, adv_q;    // one 64-pixel step in (b, p, q): 64 = adv_b*P*Q + adv_p*Q + adv_q
    signed char dh[kWTap], dw[kWTap];
    int G;                      // view groups (k_conv_wgrad4): group g reads dy + g*gs_dy, x + g*gs_x
    long long gs_dy, gs_x, gs_part;  // and writes part + g*gs_part (elements)
};

typedef __attribute__((address_space(3))) short4_t lds_s4;

__device__ __forceinline__ bf16x8 tr_frag(const uint16_t* base_row0, const uint16_t* base_row4) {
    const short4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)base_row0);
    const short4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)base_row4);
    const short8_t s = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
    return __builtin_bit_cast(bf16x8, s);
}

// ds_read_b64_tr_b16 as inline asm for k_conv_wgrad4: the builtin form makes hipcc wait
// vmcnt(0) for every LDS-DMA in flight before each transposed read (it cannot tell the
// DMA's LDS destination from the read's buffer), which serialised the next step's DMA with
// this step's MFMAs.  The asm reads are invisible to the compiler's lgkmcnt tracking, so
// the caller waits for them explicitly (wait_lgkm0 on the fragments it is about to use).
template <int OFF>
__device__ __forceinline__ short4_t tr_rd(unsigned a) {
    short4_t d;
    asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(d) : "v"(a), "i"(OFF));
    return d;
}

// fragment of k-slice ks (rows 16ks + {q, q+4}) at immediate offsets BASE + ks*16*R (+4R)
template <int BASE, int R>
__device__ __forceinline__ bf16x8 tr_frag_asm(int ks, unsigned a) {
    short4_t lo, hi;
    switch (ks) {
        case 0: lo = tr_rd<BASE>(a); hi = tr_rd<BASE + 4 * R>(a); break;
        case 1: lo = tr_rd<BASE + 16 * R>(a); hi = tr_rd<BASE + 20 * R>(a); break;
        case 2: lo = tr_rd<BASE + 32 * R>(a); hi = tr_rd<BASE + 36 * R>(a); break;
        default: lo = tr_rd<BASE + 48 * R>(a); hi = tr_rd<BASE + 52 * R>(a); break;
    }
    const short8_t s = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
    return __builtin_bit_cast(bf16x8, s);
}

// lgkmcnt(0), tied to the fragments (MT + NT of them) the next MFMAs read
template <int MT, int NT>
__device__ __forceinline__ void wait_lgkm0(bf16x8 (&a)[MT], bf16x8 (&b)[NT]) {
    if constexpr (MT > 2 || NT > 2) {  // the wait, then every fragment re-defined after it
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
        for (int i = 0; i < MT; ++i) asm volatile("" : "+v"(a[i]));
#pragma unroll
        for (int j = 0; j < NT; ++j) asm volatile("" : "+v"(b[j]));
    } else if constexpr (MT == 2 && NT == 2)
        asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(a[0]), "+v"(a[1]), "+v"(b[0]), "+v"(b[1]));
    else if constexpr (MT == 2)
        asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(a[0]), "+v"(a[1]), "+v"(b[0]));
    else if constexpr (NT == 2)
        asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(a[0]), "+v"(b[0]), "+v"(b[1]));
    else
        asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(a[0]), "+v"(b[0]));
}


__device__ __attribute__((aligned(16))) const uint4 g_wzero16[1] = {{0u, 0u, 0u, 0u}};

// Workgroup tile (64*MT) x (64*NT) of dw, 2x2 waves each owning MT*NT independent 32x32
// accumulators (the MFMAs of a k-slice do not wait on each other).  Operands are staged
// by LDS-DMA (global_load_lds_dwordx4) into two buffers, the DMA of pixel step s+1
// running under the MFMAs of step s, with the loop unrolled by the two buffers so every
// LDS fragment read is a base VGPR + immediate offset.  A DMA instruction writes 64 x
// 16 B linearly, so rows are unpadded (2*BM bytes) and a source-side XOR swizzle of the
// 16-B chunk keeps the tr-read half-waves conflict-free (the four rows a half-wave
// reads get their 64-B column window in four distinct bank quarters).  Padding taps
// read a zero block of the code object.
template <int RB>  // row bytes (128 or 256)
__device__ __forceinline__ int wswz(int row) {
    return RB >= 256 ? 4 * (row & 3) : 4 * ((row >> 1) & 1);
}

// WR = 1: the operands register-staged instead of LDS-DMA'd: global_load_dwordx4 of step
// s+2 into VGPRs while step s computes, ds_write_b128 of step s+1 into the buffer step s-1
// freed - an LDS-DMA piece costs its wave ~60-185 issue cycles among MFMAs (MI355X_MICROARCH.md
// price table), eight of them per 16-MFMA step at 128 x 128 tiles; a load + ds_write_b128
// costs ~20.  Same LDS image, same arithmetic (bit-identical results).
template <int MT, int NT, int WR = 0>
__global__ __launch_bounds__(256) void k_conv_wgrad4(WgradArgs a) {
    constexpr int BK = 64;
    constexpr int BM = 64 * MT, BN = 64 * NT;
    constexpr int RA = 2 * BM, RB = 2 * BN;          // row bytes
    constexpr int SA = BK * RA, SB = BK * RB;        // bytes per buffer
    constexpr int GA = SA / 1024 / 4, GB = SB / 1024 / 4;  // DMA instructions per wave per step
    constexpr int LPA = RA / 16, LPB = RB / 16;      // lanes per row
    extern __shared__ __attribute__((aligned(16))) uint4 wsm[];
    char* lds = reinterpret_cast<char*>(wsm);        // [A0][B0][A1][B1]
    const int t = threadIdx.x, lane = t & 63;
    const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
    const int wm = wave >> 1, wn = wave & 1;
    int bid = blockIdx.x;
    {   // XCD-major: the tiles of one pixel range share an XCD (and its L2 copy of the rows)
        const int n = gridDim.x, q = n >> 3, r = n & 7, x = bid & 7;
        bid = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + (bid >> 3);
    }
    const int tiles = a.tiles_k * a.tiles_n;
    const int grp = bid / (tiles * a.splits);  // group-major: a group's tiles share XCDs
    bid -= grp * tiles * a.splits;
    const uint16_t* __restrict__ gdy = a.dy + grp * a.gs_dy;
    const uint16_t* __restrict__ gx = a.x + grp * a.gs_x;
    const int split = bid / tiles, tile = bid - split * tiles;
    const int tk = tile % a.tiles_k, tn = tile / a.tiles_k;
    const int k0 = tk * BM, n0 = tn * BN;
    const int PQ = a.P * a.Q;
    const int M = a.N * PQ;
    const int TC = a.T * a.C;
    const int step0 = split * a.steps_per_split;
    const int step1 = min((M + BK - 1) / BK, step0 + a.steps_per_split);
    const int nst = step1 - step0;

    // A (dy) DMA lanes: row a_row[j] of the step, 16-B chunk (swizzled) of channels
    const int a_rsub = lane / LPA, a_slot = lane % LPA;
    const uint16_t* a_ptr[GA];
    int a_row[GA];
    bool a_cok[GA];
#pragma unroll
    for (int j = 0; j < GA; ++j) {
        a_row[j] = (wave * GA + j) * (64 / LPA) + a_rsub;
        const int col = k0 + ((a_slot ^ wswz<RA>(a_row[j])) << 3);
        a_cok[j] = col < a.Kc;
        a_ptr[j] = gdy + ((size_t)step0 * BK + a_row[j]) * a.Kc + (a_cok[j] ? col : 0);
    }
    // B (x) DMA lanes: fixed (tap, channel chunk) per instruction; the lane's pixel
    // (b, p, q) is decoded once and then advanced by one 64-pixel step per issue
    // (adv_*: no per-step division in the issue path)
    const int b_rsub = lane / LPB, b_slot = lane % LPB;
    int b_row[GB], b_toff[GB], b_dh[GB], b_dw[GB];
    int b_b[GB], b_p[GB], b_q[GB];
    bool b_cok[GB];
#pragma unroll
    for (int j = 0; j < GB; ++j) {
        b_row[j] = (wave * GB + j) * (64 / LPB) + b_rsub;
        const int col = n0 + ((b_slot ^ wswz<RB>(b_row[j])) << 3);
        b_cok[j] = col < TC;
        const int tap = b_cok[j] ? col >> a.logC : 0;
        const int r = tap / a.S, s = tap - r * a.S;
        b_dh[j] = r - a.padh;
        b_dw[j] = s - a.padw;
        b_toff[j] = ((b_dh[j] * a.W + b_dw[j]) << a.logC) + (col & (a.C - 1));
        const int m = step0 * BK + b_row[j];
        b_b[j] = (int)a.fd_pq.div((uint32_t)m);
        const int pq = m - b_b[j] * PQ;
        b_p[j] = (int)a.fd_q.div((uint32_t)pq);
        b_q[j] = pq - b_p[j] * a.Q;
    }
    typedef __attribute__((address_space(1))) const void* gptr_t;
    typedef __attribute__((address_space(3))) void* lptr_t;
    const void* zero = (const void*)g_wzero16;
    // the sources of step step0 + i's pieces (A: dy rows, B: gathered x rows), in call order
    // (B's pixel walk advances one step per call)
    auto sources = [&](int i, const void* (&sa)[GA], const void* (&sb)[GB]) __attribute__((always_inline)) {
        const bool full = (step0 + i + 1) * BK <= M;
#pragma unroll
        for (int j = 0; j < GA; ++j) {
            const bool ok = a_cok[j] & (full | ((step0 + i) * BK + a_row[j] < M));  // no short-circuit branch
            sa[j] = ok ? (const void*)(a_ptr[j] + (size_t)i * BK * a.Kc) : zero;
        }
#pragma unroll
        for (int j = 0; j < GB; ++j) {
            const int b = b_b[j], p = b_p[j], q = b_q[j];
            const int h0 = p * a.sth, w0 = q * a.stw;
            const int hi = h0 + b_dh[j], wi = w0 + b_dw[j];
            const bool ok = b_cok[j] & (b < a.N) & ((unsigned)hi < (unsigned)a.H) & ((unsigned)wi < (unsigned)a.W);
            const int pix = (b * a.H + h0) * a.W + w0;
            sb[j] = ok ? (const void*)(gx + (((long)pix << a.logC) + b_toff[j])) : zero;
            // next step's pixel: + 64 = (adv_b, adv_p, adv_q), one carry per component at most
            int nq = q + a.adv_q, np = p + a.adv_p, nb = b + a.adv_b;
            if (nq >= a.Q) { nq -= a.Q; ++np; }
            if (np >= a.P) { np -= a.P; ++nb; }
            b_b[j] = nb; b_p[j] = np; b_q[j] = nq;
        }
    };
    auto issue = [&](int i, int bufoff) __attribute__((always_inline)) {  // step step0 + i
        const void* sa[GA];
        const void* sb[GB];
        sources(i, sa, sb);
#pragma unroll
        for (int j = 0; j < GA; ++j)
            __builtin_amdgcn_global_load_lds((gptr_t)sa[j], (lptr_t)(lds + bufoff + (wave * GA + j) * 1024), 16, 0, 0);
#pragma unroll
        for (int j = 0; j < GB; ++j)
            __builtin_amdgcn_global_load_lds((gptr_t)sb[j], (lptr_t)(lds + bufoff + SA + (wave * GB + j) * 1024), 16, 0,
                                             0);
    };
    typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
    u32x4 ra[WR ? GA : 1], rb[WR ? GB : 1];
    auto gload = [&](int i) __attribute__((always_inline)) {  // step step0 + i into registers
        const void* sa[GA];
        const void* sb[GB];
        sources(i, sa, sb);
#pragma unroll
        for (int j = 0; j < GA; ++j) ra[WR ? j : 0] = *reinterpret_cast<const u32x4*>(sa[j]);
#pragma unroll
        for (int j = 0; j < GB; ++j) rb[WR ? j : 0] = *reinterpret_cast<const u32x4*>(sb[j]);
    };
    auto swrite = [&](int bufoff) __attribute__((always_inline)) {  // the same LDS image as issue()
#pragma unroll
        for (int j = 0; j < GA; ++j)
            *reinterpret_cast<u32x4*>(lds + bufoff + (wave * GA + j) * 1024 + lane * 16) = ra[WR ? j : 0];
#pragma unroll
        for (int j = 0; j < GB; ++j)
            *reinterpret_cast<u32x4*>(lds + bufoff + SA + (wave * GB + j) * 1024 + lane * 16) = rb[WR ? j : 0];
    };

    floatx16 acc[MT][NT];
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int j = 0; j < NT; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
    // tr-read geometry: half-wave g>>1 reads rows 8*(g>>1)+q4 (+4) of a 16-row k-slice, 4-column
    // block p4 of the 32-column fragment, 16-column half g&1.  The swizzle term depends on q4 only,
    // so (k-slice, +4 row) offsets are immediates on one base per fragment.
    const int g = lane >> 4, q4 = (lane >> 2) & 3, p4 = lane & 3;
    const int rbase = 8 * (g >> 1) + q4;
    int a_base[MT], b_base[NT];
#pragma unroll
    for (int i = 0; i < MT; ++i) {
        const int c = wm * (32 * MT) + 32 * i + 16 * (g & 1) + 4 * p4;
        a_base[i] = rbase * RA + (((c >> 3) ^ wswz<RA>(rbase)) << 4) + (c & 7) * 2;
    }
#pragma unroll
    for (int j = 0; j < NT; ++j) {
        const int c = wn * (32 * NT) + 32 * j + 16 * (g & 1) + 4 * p4;
        b_base[j] = SA + rbase * RB + (((c >> 3) ^ wswz<RB>(rbase)) << 4) + (c & 7) * 2;
    }
    unsigned a_lds[MT], b_lds[NT];  // LDS byte addresses of the fragment bases
#pragma unroll
    for (int i = 0; i < MT; ++i)
        a_lds[i] = (unsigned)(uintptr_t)(__attribute__((address_space(3))) char*)(lds + a_base[i]);
#pragma unroll
    for (int j = 0; j < NT; ++j)
        b_lds[j] = (unsigned)(uintptr_t)(__attribute__((address_space(3))) char*)(lds + b_base[j]);
    // one k-slice's fragments (asm reads; the caller waits), then its MFMAs; the next
    // slice's reads are issued before this slice's MFMAs
    // buffer 1 at an immediate offset while that fits the 16-bit field, else from its own
    // base registers (wide tiles: 64 KB buffers)
    constexpr bool kFarBuf = 2 * (SA + SB) > 65536;
    unsigned a_lds1[MT], b_lds1[NT];
#pragma unroll
    for (int i = 0; i < MT; ++i) a_lds1[i] = a_lds[i] + (SA + SB);
#pragma unroll
    for (int j = 0; j < NT; ++j) b_lds1[j] = b_lds[j] + (SA + SB);
    auto compute = [&](auto bufc) {
        constexpr int BO0 = decltype(bufc)::value;
        constexpr int BO = kFarBuf ? 0 : BO0;
        const unsigned* ab = (kFarBuf && BO0) ? a_lds1 : a_lds;
        const unsigned* bb = (kFarBuf && BO0) ? b_lds1 : b_lds;
        bf16x8 af[2][MT], bfr[2][NT];
        auto load = [&](int ks, int c) {
#pragma unroll
            for (int i = 0; i < MT; ++i) af[c][i] = tr_frag_asm<BO, RA>(ks, ab[i]);
#pragma unroll
            for (int j = 0; j < NT; ++j) bfr[c][j] = tr_frag_asm<BO, RB>(ks, bb[j]);
        };
        load(0, 0);
#pragma unroll
        for (int ks = 0; ks < 4; ++ks) {
            const int c = ks & 1;
            wait_lgkm0<MT, NT>(af[c], bfr[c]);
            if (ks < 3) load(ks + 1, c ^ 1);
            __builtin_amdgcn_sched_barrier(0);  // the next slice's reads go out before these MFMAs
#pragma unroll
            for (int i = 0; i < MT; ++i)
#pragma unroll
                for (int j = 0; j < NT; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[c][i], bfr[c][j], acc[i][j], 0, 0, 0);
            __builtin_amdgcn_sched_barrier(0);
        }
    };
    constexpr int BUF1 = SA + SB;
    using B0 = std::integral_constant<int, 0>;
    using B1 = std::integral_constant<int, BUF1>;
    int i = 0;
    if constexpr (WR) {
        // LDS stores drained, then the barrier; the clobber keeps LDS accesses on their side
        auto bar = [] { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); };
        if (nst > 0) {
            gload(0);
            swrite(0);
        }
        if (nst > 1) gload(1);
        bar();
        for (; i + 1 < nst; i += 2) {  // steps i (buffer 0) and i+1 (buffer 1)
            compute(B0{});
            swrite(BUF1);  // step i+1 (buffer 1 was freed by step i-1, before the last barrier)
            if (i + 2 < nst) gload(i + 2);
            bar();
            compute(B1{});
            if (i + 2 < nst) swrite(0);
            if (i + 3 < nst) gload(i + 3);
            bar();
        }
    } else {
        if (nst > 0) issue(0, 0);
        __syncthreads();
        for (; i + 1 < nst; i += 2) {  // steps i (buffer 0) and i+1 (buffer 1)
            issue(i + 1, BUF1);
            compute(B0{});
            __syncthreads();
            if (i + 2 < nst) issue(i + 2, 0);
            compute(B1{});
            __syncthreads();
        }
    }
    if (i < nst) compute(B0{});  // odd step count: the last step sits in buffer 0

    float* out = a.part + grp * a.gs_part + (size_t)split * a.Kc * TC;
    const bool inner = k0 + BM <= a.Kc && n0 + BN <= TC;
#pragma unroll
    for (int j = 0; j < NT; ++j) {
        const int col = n0 + wn * (32 * NT) + 32 * j + (lane & 31);
#pragma unroll
        for (int ii = 0; ii < MT; ++ii) {
            const int row0 = k0 + wm * (32 * MT) + 32 * ii + 4 * (lane >> 5);
            float* o = out + (size_t)row0 * TC + col;
            if (inner) {
                if (a.accumulate) {
#pragma unroll
                    for (int r = 0; r < 16; ++r) {
                        float* p = o + (size_t)((r & 3) + 8 * (r >> 2)) * TC;
                        *p += acc[ii][j][r];
                    }
                } else {
#pragma unroll
                    for (int r = 0; r < 16; ++r) o[(size_t)((r & 3) + 8 * (r >> 2)) * TC] = acc[ii][j][r];
                }
            } else if (col < TC) {
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int row = row0 + (r & 3) + 8 * (r >> 2);
                    if (row < a.Kc) {
                        float* p = o + (size_t)((r & 3) + 8 * (r >> 2)) * TC;
                        *p = a.accumulate ? *p + acc[ii][j][r] : acc[ii][j][r];
                    }
                }
            }
        }
    }
}

// k_wgrad_halo64: weight gradient of a 3x3 / stride-1 / pad-1 convolution with 64-channel
// multiples and W <= 62 (the ResNet-18 identity-block shapes), as 64 x (9 taps x 64) blocks of
// a view group's gradient held in the accumulators of one workgroup's four compute waves
// (wave (kh, ch): output channels 32 kh .., input channels 32 ch .., 9 taps = 9 x 32x32
// accumulators) while it walks a contiguous range of image rows.
//
// Staging unit: a "super-row" of 64 positions x 128 B = RPS = 64 / PP consecutive image rows
// of PP >= W + 2 positions each (PP = 64, 32, 16 for W <= 62, 30, 14).  In the x image,
// position m of a row holds input column m - 1 (zeros outside the image); in the dy image,
// position m holds output pixel m - 2 (two leading zeros).  Tap (rr, s) of output row p is
//   dw[rr][s] = sum over positions m of dy_p[m + 2 - s] (x) x_{p + rr - 1}[m]   (m from 0)
// per 16-position k-slice.  Operand economy (LDS fragment reads set this kernel's speed:
// halving them took the layer-1 launch from 47 to 37 us, while relaxing every wait did
// nothing): per slice ONE dy fragment is read (shift s = 2, rows m) and the shifts s = 1, 0 are
// made in registers from it and the next slice's fragment (v_permlane32_swap + v_alignbit:
// rows m + 1, m + 2 = this fragment moved up by one / two elements plus the next fragment's
// first rows); the x fragments of input rows p - 1, p, p + 1 stay in registers across output
// rows (a 4-set rotation), so per slice ONE x fragment is read (row p + 2, for the next output
// row).  2 + 2 transposed reads feed 9 MFMAs (12 before).  Kernel rows outside the image
// multiply zeroed operands.
//
// Both operands come through ds_read_b64_tr_b16 transposed reads (rows of 128 B, chunk XOR
// 4 * ((row >> 1) & 1): conflict-free for any 4 consecutive rows).  Four loader waves (one
// beside each compute wave's SIMD) keep D super-rows of LDS-DMA in flight (dy of super-row S
// with x of S + 2) under counted vmcnt waits; one raw barrier per super-row, before its second
// slice (the dy reads run three slices ahead, the x reads one image row ahead).  Each workgroup
// writes its fp32 partial slab [64][9 x 64] (split over rows; k_wgrad_sum reduces the splits in
// a fixed order).
struct WHaloArgs {
    const uint16_t* dy;  // [G][N*P][Q][K]  (P = H, Q = W)
    const uint16_t* x;   // [G][N*H][W][C]
    float* part;         // [G][splits][K][9*C] (tile (kb, cb) writes its 64 x 9 x 64 block)
    int N, H, W, rows, srows, splits, rpw;  // rows = N*H image rows per group, srows = super-rows,
                                            // rpw = super-rows per workgroup
    int K, C, kt, ct;    // channels; 64-channel tiles of dy (kt) and x (ct)
    long long gs_dy, gs_x;  // group strides (elements)
};

template <int D, int PP>
__global__ __launch_bounds__(512) void k_wgrad_halo64(WHaloArgs a) {
    static_assert(D >= 2 && (PP == 16 || PP == 32 || PP == 64), "halo64: D >= 2 super-rows in flight, PP = 16/32/64");
    constexpr int RPS = 64 / PP, SPR = PP / 16;  // image rows per super-row, k-slices per image row
    constexpr int XS = D + 3, DS = D + 1;  // x ring (super-rows R .. R+D+2), dy ring (R .. R+D)
    constexpr int SL = 8192, DSL = SL + 256;  // one super-row; dy slot + 2 zero pad positions
    constexpr int OX = 0, OD = XS * SL;       // x ring | dy ring
    extern __shared__ __attribute__((aligned(16))) uint4 wsm[];
    char* lds = reinterpret_cast<char*>(wsm);
    const int t = threadIdx.x, lane = t & 63;
    const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
    // block -> (group, 64 x 64 channel tile, split): splits innermost
    int bid = blockIdx.x;
    const int split = bid % a.splits;
    bid /= a.splits;
    const int tile = bid % (a.kt * a.ct), grp = bid / (a.kt * a.ct);
    const int kb = tile % a.kt, cb = tile / a.kt;
    const int R0 = split * a.rpw;
    const int R1 = min(a.srows, R0 + a.rpw);
    // each dy slot's two pad positions: ds_write, never a DMA target
    if (t < DS * 16) *reinterpret_cast<uint4*>(lds + OD + (t >> 4) * DSL + SL + (t & 15) * 16) = make_uint4(0, 0, 0, 0);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // visible to every wave at the first barrier

    if (wave >= 4) {
        // loader waves: all LDS-DMA, so the compute waves' MFMA stream never carries a DMA issue.
        // Piece (lw, j) = slot positions 8 (2 lw + j) .. + 7, one image row (PP is a multiple of
        // 8); lane -> position 8 (2 lw + j) + lane / 8, source chunk (lane % 8) ^ swizzle(position).
        const int lw = wave - 4;
        typedef __attribute__((address_space(1))) const void* gptr_t;
        typedef __attribute__((address_space(3))) void* lptr_t;
        const void* zero = (const void*)g_wzero16;
        const uint16_t* __restrict__ gdy = a.dy + grp * a.gs_dy + kb * 64;
        const uint16_t* __restrict__ gx = a.x + grp * a.gs_x + cb * 64;
        int sub[2], xcol[2], dpx[2], xo[2], dyo[2];
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const int pos = (2 * lw + j) * 8 + (lane >> 3);
            const int sc = ((lane & 7) ^ wswz<128>(pos)) << 3;
            sub[j] = pos / PP;
            xcol[j] = pos % PP - 1;
            dpx[j] = pos % PP - 2;
            xo[j] = xcol[j] * a.C + sc;
            dyo[j] = dpx[j] * a.K + sc;
        }
        auto dma = [&](const void* src, int off) __attribute__((always_inline)) {
            __builtin_amdgcn_global_load_lds((gptr_t)src, (lptr_t)(lds + off), 16, 0, 0);
        };
        auto issue_x = [&](int R, int xs) __attribute__((always_inline)) {  // x super-row R into slot xs
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                const int g = R * RPS + sub[j];
                const bool ok = R >= 0 && g < a.rows && xcol[j] >= 0 && xcol[j] < a.W;
                dma(ok ? (const void*)(gx + (size_t)g * a.W * a.C + xo[j]) : zero, OX + xs * SL + (2 * lw + j) * 1024);
            }
        };
        auto issue_dy = [&](int R, int ds) __attribute__((always_inline)) {  // dy super-row R into slot ds
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                const int g = R * RPS + sub[j];
                const bool ok = R < R1 && g < a.rows && dpx[j] >= 0 && dpx[j] < a.W;
                dma(ok ? (const void*)(gdy + (size_t)g * a.W * a.K + dyo[j]) : zero, OD + ds * DSL + (2 * lw + j) * 1024);
            }
        };
        auto slot = [](int v, int n) { return ((v % n) + n) % n; };
        if (R0 < R1) {
            // prologue: x super-rows R0 - 1 .. R0 + 1, then D steps of (dy S, x S + 2); step R0 landed
            issue_x(R0 - 1, slot(R0 - 1, XS));
            issue_x(R0, slot(R0, XS));
            issue_x(R0 + 1, slot(R0 + 1, XS));
            for (int i = 0; i < D; ++i) {
                issue_dy(R0 + i, slot(R0 + i, DS));
                issue_x(R0 + i + 2, slot(R0 + i + 2, XS));
            }
            asm volatile("s_waitcnt vmcnt(%0)" ::"n"(4 * (D - 1)) : "memory");
            __builtin_amdgcn_s_barrier();
        }
        int dsn = slot(R0 + D, DS), xsn = slot(R0 + D + 2, XS);  // slots of DMA step R + D
        for (int R = R0; R < R1; ++R) {
            // step R + 1 landed (later steps may stay in flight); after the barrier no compute
            // wave reads dy super-row R - 1 or x super-row R - 1 any more (their slots are the
            // ones step R + D refills; uniform counts: past the range the pieces load zeros)
            asm volatile("s_waitcnt vmcnt(%0)" ::"n"(4 * (D - 2)) : "memory");
            __builtin_amdgcn_s_barrier();
            issue_dy(R + D, dsn);
            issue_x(R + D + 2, xsn);
            dsn = dsn + 1 == DS ? 0 : dsn + 1;
            xsn = xsn + 1 == XS ? 0 : xsn + 1;
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        return;
    }

    const int kh = wave & 1, ch = wave >> 1;
    floatx16 acc[9];
#pragma unroll
    for (int i = 0; i < 9; ++i)
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[i][e] = 0.f;
    // tr-read lane geometry (k_conv_wgrad4's): half-wave g >> 1 reads rows 8 (g >> 1) + q4 (+4) of
    // a 16-row slice, 4-column block p4 of the 32-column fragment, 16-column half g & 1; lane l
    // receives channel l % 32, rows 8 (l / 32) .. + 7 (the MFMA operand layout)
    const int g = lane >> 4, q4 = (lane >> 2) & 3, p4 = lane & 3;
    const int rbase = 8 * (g >> 1) + q4;
    const int acol = kh * 32 + 16 * (g & 1) + 4 * p4;
    const int bcol = ch * 32 + 16 * (g & 1) + 4 * p4;
    const unsigned lds0 = (unsigned)(uintptr_t)(__attribute__((address_space(3))) char*)lds;
    auto rowoff = [](int row, int col) { return (unsigned)(row * 128 + ((((col >> 3) ^ wswz<128>(row))) << 4) + (col & 7) * 2); };
    const unsigned a_lane = rowoff(rbase, acol), b_lane = rowoff(rbase, bcol);
    const bool lo_half = lane < 32;
    typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
    u32x4 F[4];  // dy fragments (shift 2) of slices ks .. ks + 3 of the super-row (ring by ks % 4)
    // x fragments of image rows g - 1, g, g + 1 and the prefetched g + 2, per slice of a row;
    // rotated by register copies at each image row's end (VALU beside the MFMAs)
    u32x4 Xm[SPR], X0[SPR], Xp[SPR], Xn[SPR];
    auto rd = [&](unsigned ad) __attribute__((always_inline)) {
        short4_t lo, hi;
        asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(lo) : "v"(ad));
        asm volatile("ds_read_b64_tr_b16 %0, %1 offset:512" : "=v"(hi) : "v"(ad));
        return __builtin_bit_cast(u32x4, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
    };
    auto mfma = [&](int i, u32x4 A, u32x4 B) __attribute__((always_inline)) {
        acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, A), __builtin_bit_cast(bf16x8, B),
                                                        acc[i], 0, 0, 0);
    };
    // uniform slot bases of super-rows R (dy), R + 1 (dy, the reads two slices ahead) and
    // R - 1 .. R + 2 (x); the lane offsets are added per read
    int dsl = R0 % DS, xsl = (R0 - 1 + XS) % XS;
    auto dy_base = [&](int i) { const int d = dsl + i; return lds0 + (unsigned)(OD + (d >= DS ? d - DS : d) * DSL); };
    auto x_base = [&](int i) { const int x = xsl + i; return lds0 + (unsigned)(OX + (x >= XS ? x - XS : x) * SL); };
    // x fragment of image row R * RPS + r (r = -1 .. RPS + 1), slice kk of that row
    auto xaddr = [&](int r, int kk) __attribute__((always_inline)) {
        const int rr = r + RPS;  // >= 0: super-row R - 1 + rr / RPS
        return x_base(rr / RPS) + b_lane + (unsigned)(((rr % RPS) * PP + kk * 16) * 128);
    };

    int p = 0;  // image row (within its image) of the current output row
    if (R0 < R1) {
        __builtin_amdgcn_s_barrier();  // step R0 landed: dy R0, x R0 - 1 .. R0 + 2
        p = (int)(((long long)R0 * RPS) % a.H);
#pragma unroll
        for (int kk = 0; kk < SPR; ++kk) {
            Xm[kk] = rd(xaddr(-1, kk));
            X0[kk] = rd(xaddr(0, kk));
            Xp[kk] = rd(xaddr(1, kk));
        }
        F[0] = rd(dy_base(0) + a_lane);
        F[1] = rd(dy_base(0) + a_lane + 2048);
        F[2] = rd(dy_base(0) + a_lane + 4096);
    }
    for (int R = R0; R < R1; ++R) {
#pragma unroll
        for (int ks = 0; ks < 4; ++ks) {
            const int j = ks / SPR, kk = ks % SPR;  // image row of the super-row, slice of it
            if (ks == 1)  // super-row R + 1 landed; every wave done with super-row R - 1
                __builtin_amdgcn_s_barrier();
            // everything this slice consumes has landed: the last slice's reads were its x
            // fragment, then the dy fragment three slices ahead - only that one may still fly
            // (LDS reads return in order; no other LDS or scalar-memory op in this loop)
            asm volatile("s_waitcnt lgkmcnt(2)" : "+v"(F[ks]), "+v"(F[(ks + 1) & 3]), "+v"(Xm[kk]), "+v"(X0[kk]),
                         "+v"(Xp[kk]));
            const u32x4 f2 = F[ks], fn = F[(ks + 1) & 3];
            // kernel rows 0 / 2 outside the image take zero operands (masks, not branches: a
            // conditional MFMA costs accumulator copies)
            const unsigned mt = p != 0 ? ~0u : 0u, mb = p != a.H - 1 ? ~0u : 0u;
            const u32x4 xm = Xm[kk] & mt, x0 = X0[kk], xp = Xp[kk] & mb;
            // shift s = 2 (the fragment as read); reads for later slices threaded behind
            mfma(2, f2, xm);
            __builtin_amdgcn_sched_barrier(0);
            Xn[kk] = rd(xaddr(j + 2, kk));  // image row + 2, for the next output row
            __builtin_amdgcn_sched_barrier(0);
            mfma(5, f2, x0);
            __builtin_amdgcn_sched_barrier(0);
            // dy three slices ahead (slices 1..3 read super-row R + 1's)
            F[(ks + 3) & 3] = rd(dy_base(ks >= 1 ? 1 : 0) + a_lane + (unsigned)(((ks + 3) & 3) * 2048));
            __builtin_amdgcn_sched_barrier(0);
            mfma(8, f2, xp);
            // shifts s = 1, 0: rows m + 1, m + 2 - the fragment moved up by one / two elements,
            // the vacated top elements from lane l + 32 (lanes 0-31: this fragment's rows 8, 9)
            // or lane l - 32 of the next fragment (lanes 32-63: its rows 0, 1)
            const auto sw = __builtin_amdgcn_permlane32_swap(f2[0], fn[0], false, false);
            const unsigned donor = lo_half ? sw[1] : sw[0];
            u32x4 f1, f0;
            f1[0] = __builtin_amdgcn_alignbit(f2[1], f2[0], 16);
            f1[1] = __builtin_amdgcn_alignbit(f2[2], f2[1], 16);
            f1[2] = __builtin_amdgcn_alignbit(f2[3], f2[2], 16);
            f1[3] = __builtin_amdgcn_alignbit(donor, f2[3], 16);
            f0[0] = f2[1]; f0[1] = f2[2]; f0[2] = f2[3]; f0[3] = donor;
            mfma(1, f1, xm);
            mfma(4, f1, x0);
            mfma(7, f1, xp);
            mfma(0, f0, xm);
            mfma(3, f0, x0);
            mfma(6, f0, xp);
            __builtin_amdgcn_sched_barrier(0);
            if (kk == SPR - 1) {  // the image row ends: rotate the x rows, next output row
                // (the register copies read the prefetched fragments: their reads must have landed)
#pragma unroll
                for (int q = 0; q < SPR; ++q) asm volatile("s_waitcnt lgkmcnt(2)" : "+v"(Xn[q]));
#pragma unroll
                for (int q = 0; q < SPR; ++q) {
                    Xm[q] = X0[q];
                    X0[q] = Xp[q];
                    Xp[q] = Xn[q];
                }
                p = p + 1 == a.H ? 0 : p + 1;
            }
        }
        dsl = dsl + 1 == DS ? 0 : dsl + 1;
        xsl = xsl + 1 == XS ? 0 : xsl + 1;
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    // D[k][c]: col = lane & 31 (c), row = (e & 3) + 8 (e >> 2) + 4 (lane >> 5) (k)
    // the split's slab [K][9*C]; this tile fills rows kb*64 .., columns tap*C + cb*64 ..
    // (bf16 partials in the accumulators' own layout with 16-B stores measured no faster:
    // l1 49.6 vs 49.4 us with the sum, r04)
    const int TC = 9 * a.C;
    float* out = a.part + ((size_t)grp * a.splits + split) * ((size_t)a.K * TC);
#pragma unroll
    for (int tp = 0; tp < 9; ++tp) {
        const int col = tp * a.C + cb * 64 + ch * 32 + (lane & 31);
#pragma unroll
        for (int e = 0; e < 16; ++e) {
            const int row = kb * 64 + kh * 32 + (e & 3) + 8 * (e >> 2) + 4 * (lane >> 5);
            out[(size_t)row * TC + col] = acc[tp][e];
        }
    }
}

// k_wgrad_ring: weight gradient of a 3 x 3 convolution (any stride / padding) with K % 128 == 0
// and C % 32 == 0 - the layer-2..4 shapes k_conv_wgrad4 served at 0.15-0.23 of the MFMA peak.
// What bound k_conv_wgrad4: one 64-pixel step of LDS-DMA in flight per workgroup (issue ->
// landed is ~1 us under load, MI355X_MICROARCH.md ldsdma rows) against 16 MFMAs per wave
// (~0.25 us), so its two workgroups per CU took in ~35 GB/s; and every DMA issue sat in the
// compute waves' MFMA stream.  Here, per CU ONE workgroup of 512 threads:
//   * four LOADER waves own all LDS-DMA: a 3-slot ring of 64-pixel steps, 2 steps in flight
//     (156 KB), one raw s_barrier per step after a counted vmcnt (the step about to be read has
//     landed; the younger one stays in flight across the barrier);
//   * four COMPUTE waves never touch VMEM in the loop.  The workgroup tile is 128 output channels
//     x 288 (tap, channel) columns = a 4 x 9 grid of 32 x 32 blocks (k-block kb, column block cb);
//     compute wave w = kh + 2 ch owns k-blocks {2 kh, 2 kh + 1} x column blocks 5 ch .. 5 ch + 3
//     plus the single cell (2 kh + ch, 4) of the middle column: 9 accumulators and 9 MFMAs per
//     16-pixel k-slice, fed by 2 A + 5 B fragments (14 ds_read_b64_tr_b16) read one k-slice
//     ahead.  (r05's layout - wave w owning k-block w x all 9 column blocks - read 1 A + 9 B
//     fragments per wave, every B fragment by all four waves: 80 instead of 56 transposed reads
//     per k-slice and CU, 2.22 instead of 1.56 LDS instructions per MFMA (PMC), 2.5 % slower.)
//   * every 3x3 shape with C % 32 == 0 splits into whole tiles; 88.6 FLOP per staged byte.
// LDS slot: B (x gathered per tap) as 9 blocks of [64 px][32 columns] (64-B rows: the tr reads of a
// half-wave cover 4 rows x 64 B = all 64 banks, no swizzle), then A (dy) as 2 blocks of
// [64 px][64 k] (128-B rows, chunk XOR 4 ((row >> 1) & 1): k_conv_wgrad4's image).  Splits over the
// pixel steps write fp32 partial slabs that k_wgrad_sum reduces in a fixed order (deterministic);
// one split writes (or accumulates into) the gradient directly.
// What bounds it now (r06 A/B): the LDS-DMA feed - 52 KB staged per 64-pixel step, ~38 GB/s per CU
// at half the CUs - not the LDS reads (30 % fewer of them bought 2.5 %).
struct WRingArgs {
    const uint16_t* dy;  // [G][M][K]  (M = N*P*Q)
    const uint16_t* x;   // [G][N][H][W][C]
    float* part;         // [G][splits][K][9C], or dw (one split)
    int N, H, W, C, logC, K, P, Q, sth, stw, padh, padw, M;
    int tiles_k, tiles_n, splits, sps;  // sps: 64-pixel steps per split
    FastDiv fd_pq, fd_q;
    int adv_b, adv_p, adv_q;            // one step of 64 pixels in (b, p, q)
    long long gs_dy, gs_x, gs_part;     // group strides (elements)
    int accumulate;
};

namespace ring {
constexpr int S = 3, BK = 64;                      // ring slots, pixels per step
constexpr int BB = BK * 64, AB = BK * 128;         // bytes per B / A block
constexpr int B = 9 * BB, A = 2 * AB, SLOT = B + A;
constexpr int SLICES = BK / 16;                    // 16-pixel k-slices per step
constexpr size_t LDS = (size_t)S * SLOT;
}  // namespace ring

// one 32 x 16 fragment by two transposed reads at base + LO / + HI
template <int LO, int HI>
__device__ __forceinline__ bf16x8 ring_frag(unsigned base) {
    const short4_t lo = tr_rd<LO>(base), hi = tr_rd<HI>(base);
    return __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
}

// the compute waves (see above): wave w = kh + 2 CH
template <int CH>
__device__ __forceinline__ void ring_compute(const WRingArgs& a, int w, int lane, unsigned lds0, int nst, int grp,
                                             int split, int k0, int n0) {
    using namespace ring;
    const int kh = w & 1;
    floatx16 acc[9];  // [4 i + jj]: k-block 2 kh + i x column block 5 CH + jj; [8]: (2 kh + CH, 4)
#pragma unroll
    for (int j = 0; j < 9; ++j)
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[j][e] = 0.f;
    // tr-read geometry (k_conv_wgrad4's): half-wave g >> 1 reads rows 8 (g >> 1) + q4 (+4) of a
    // 16-row k-slice, 4-column block p4 of the 32-column fragment, 16-column half g & 1.  The A
    // image's chunk swizzle (XOR 4 on odd row pairs) flips the 64-column half's bit, so the two A
    // fragments of a lane sit at +-64 B of each other by row: two base registers.
    const int g = lane >> 4, q4 = (lane >> 2) & 3, p4 = lane & 3;
    const int rbase = 8 * (g >> 1) + q4;
    const int cin = 16 * (g & 1) + 4 * p4;
    unsigned a_l[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const int ac = 32 * i + cin;
        a_l[i] = B + kh * AB + rbase * 128 + ((((ac >> 3) ^ wswz<128>(rbase))) << 4) + (ac & 7) * 2;
    }
    const unsigned b_l = rbase * 64 + cin * 2 + 5 * CH * BB, b_4 = rbase * 64 + cin * 2 + 4 * BB;
    bf16x8 fa[2][2], fb[2][5];
    auto load_ks = [&](auto ksc, int c, unsigned sb) __attribute__((always_inline)) {
        constexpr int KS = decltype(ksc)::value;
        fa[c][0] = ring_frag<KS * 2048, KS * 2048 + 512>(sb + a_l[0]);
        fa[c][1] = ring_frag<KS * 2048, KS * 2048 + 512>(sb + a_l[1]);
        fb[c][0] = ring_frag<0 * BB + KS * 1024, 0 * BB + KS * 1024 + 256>(sb + b_l);
        fb[c][1] = ring_frag<1 * BB + KS * 1024, 1 * BB + KS * 1024 + 256>(sb + b_l);
        fb[c][2] = ring_frag<2 * BB + KS * 1024, 2 * BB + KS * 1024 + 256>(sb + b_l);
        fb[c][3] = ring_frag<3 * BB + KS * 1024, 3 * BB + KS * 1024 + 256>(sb + b_l);
        fb[c][4] = ring_frag<KS * 1024, KS * 1024 + 256>(sb + b_4);
    };
    auto load = [&](int ks, int c, unsigned sb) __attribute__((always_inline)) {
        switch (ks) {
            case 0: load_ks(std::integral_constant<int, 0>{}, c, sb); break;
            case 1: load_ks(std::integral_constant<int, 1>{}, c, sb); break;
            case 2: load_ks(std::integral_constant<int, 2>{}, c, sb); break;
            default: load_ks(std::integral_constant<int, 3>{}, c, sb); break;
        }
    };
    // lgkmcnt(0), then every fragment of buffer c re-defined after it (asm reads are invisible
    // to the compiler's own waits; the MFMAs must not be hoisted above the wait)
    auto wait_frags = [&](int c) __attribute__((always_inline)) {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        asm volatile("" : "+v"(fa[c][0]), "+v"(fa[c][1]));
#pragma unroll
        for (int j = 0; j < 5; ++j) asm volatile("" : "+v"(fb[c][j]));
        __builtin_amdgcn_sched_barrier(0);
    };
    int slot = 0;
    if (nst > 0) {
        __builtin_amdgcn_s_barrier();  // step 0 landed
        unsigned sb = lds0;
        load(0, 0, sb);
        for (int i = 0; i < nst; ++i) {
#pragma unroll
            for (int ks = 0; ks < SLICES; ++ks) {
                const int c = ks & 1;
                wait_frags(c);
                if (ks + 1 < SLICES) {
                    load(ks + 1, c ^ 1, sb);
                } else if (i + 1 < nst) {
                    // every read of this step is done: the barrier lets the loaders refill the
                    // previous step's slot and tells us step i + 1 has landed - read its first
                    // slice under this slice's MFMAs
                    __builtin_amdgcn_s_barrier();
                    slot = slot + 1 == S ? 0 : slot + 1;
                    sb = lds0 + (unsigned)slot * SLOT;
                    load(0, c ^ 1, sb);
                }
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int ii = 0; ii < 2; ++ii)
#pragma unroll
                    for (int jj = 0; jj < 4; ++jj)
                        acc[4 * ii + jj] =
                            __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[c][ii], fb[c][jj], acc[4 * ii + jj], 0, 0, 0);
                acc[8] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[c][CH], fb[c][4], acc[8], 0, 0, 0);
                __builtin_amdgcn_sched_barrier(0);
            }
        }
    }
    // D[k][col]: col = lane & 31, row = (e & 3) + 8 (e >> 2) + 4 (lane >> 5).  Direct dword stores
    // (an LDS-staged dwordx4 epilogue measured 3-4 us slower per launch: hipcc serialised its
    // stores on vmcnt(0)); the accumulate test is hoisted out of the loops (a per-element select
    // would branch and wait vmcnt(0) around every load)
    const int TC = 9 * a.C;
    float* base = a.part + grp * a.gs_part + (size_t)split * a.K * TC + (size_t)(k0 + 4 * (lane >> 5)) * TC + n0 +
                  (lane & 31);
    auto out_of = [&](int j) __attribute__((always_inline)) -> float* {
        const int kb = j < 8 ? 2 * kh + (j >> 2) : 2 * kh + CH;
        const int cb = j < 8 ? 5 * CH + (j & 3) : 4;
        return base + (size_t)(32 * kb) * TC + 32 * cb;
    };
    if (a.accumulate) {
#pragma unroll
        for (int j = 0; j < 9; ++j) {
            float* out = out_of(j);
            float v[16];
#pragma unroll
            for (int e = 0; e < 16; ++e) v[e] = out[(size_t)((e & 3) + 8 * (e >> 2)) * TC];
#pragma unroll
            for (int e = 0; e < 16; ++e) out[(size_t)((e & 3) + 8 * (e >> 2)) * TC] = v[e] + acc[j][e];
        }
    } else {
#pragma unroll
        for (int j = 0; j < 9; ++j) {
            float* out = out_of(j);
#pragma unroll
            for (int e = 0; e < 16; ++e) out[(size_t)((e & 3) + 8 * (e >> 2)) * TC] = acc[j][e];
        }
    }
}

__global__ __launch_bounds__(512) void k_wgrad_ring(WRingArgs a) {
    using namespace ring;
    constexpr int D = S - 1;  // steps in flight
    extern __shared__ __attribute__((aligned(16))) uint4 wsm[];
    char* lds = reinterpret_cast<char*>(wsm);
    const int t = threadIdx.x, lane = t & 63;
    const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
    int bid = blockIdx.x;
    {   // XCD-major: the tiles of one pixel range (split) share an XCD and its L2 copy of the rows
        const int n = gridDim.x, q = n >> 3, r = n & 7, x = bid & 7;
        bid = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + (bid >> 3);
    }
    const int tiles = a.tiles_k * a.tiles_n;
    const int grp = bid / (tiles * a.splits);
    bid -= grp * tiles * a.splits;
    const int split = bid / tiles, tile = bid - split * tiles;
    const int tk = tile % a.tiles_k, tn = tile / a.tiles_k;
    const int k0 = tk * 128, n0 = tn * 288;
    const int step0 = split * a.sps;
    const int nst = max(0, min((a.M + BK - 1) / BK, step0 + a.sps) - step0);
    const unsigned lds0 = (unsigned)(uintptr_t)(__attribute__((address_space(3))) char*)lds;

    if (wave < 4) {
        if (wave >> 1) ring_compute<1>(a, wave, lane, lds0, nst, grp, split, k0, n0);
        else ring_compute<0>(a, wave, lane, lds0, nst, grp, split, k0, n0);
        return;
    }
    // ---- loader waves: wave 4 + lw stages B rows 16 lw .. + 15 of the 9 blocks and A rows
    // 16 lw .. + 15 of both blocks (9 + 4 pieces per step) ----
    const int lw = wave - 4;
    typedef __attribute__((address_space(1))) const void* gptr_t;
    typedef __attribute__((address_space(3))) void* lptr_t;
    const void* zero = (const void*)g_wzero16;
    const uint16_t* __restrict__ gdy = a.dy + grp * a.gs_dy;
    const uint16_t* __restrict__ gx = a.x + grp * a.gs_x;
    const int brow = 16 * lw + (lane >> 2), bc = (lane & 3) * 8;
    int bdh[9], bdw[9], boff[9];
#pragma unroll
    for (int j = 0; j < 9; ++j) {
        const int n = n0 + 32 * j + bc;
        const int tap = n >> a.logC, c = n & (a.C - 1);
        const int r = tap / 3, s = tap - 3 * r;
        bdh[j] = r - a.padh;
        bdw[j] = s - a.padw;
        boff[j] = ((bdh[j] * a.W + bdw[j]) << a.logC) + c;
    }
    // A sources advance by BK pixel rows per step (no per-step 64-bit multiply)
    int arow[2];
    const uint16_t* ap[2][2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        arow[h] = 16 * lw + 8 * h + (lane >> 3);
#pragma unroll
        for (int ab = 0; ab < 2; ++ab)
            ap[h][ab] = gdy + (size_t)(step0 * BK + arow[h]) * a.K + k0 + 64 * ab +
                        (((lane & 7) ^ wswz<128>(arow[h])) << 3);
    }
    const size_t astep = (size_t)BK * a.K;
    const int PQ = a.P * a.Q;
    int m = step0 * BK + brow;
    int b = (int)a.fd_pq.div((uint32_t)m);
    int p = (int)a.fd_q.div((uint32_t)(m - b * PQ));
    int q = m - b * PQ - p * a.Q;
    auto dma = [&](const void* src, unsigned off) __attribute__((always_inline)) {
        __builtin_amdgcn_global_load_lds((gptr_t)src, (lptr_t)(lds + off), 16, 0, 0);
    };
    int slot = 0;
    auto issue = [&](int i) __attribute__((always_inline)) {  // step step0 + i into the next slot
        const unsigned sb = (unsigned)slot * SLOT;
        const int ms = (step0 + i) * BK;
        const int hi0 = p * a.sth, wi0 = q * a.stw;
        const bool rok = ms + brow < a.M;
        const long pix = ((long)(b * a.H + hi0) * a.W + wi0) << a.logC;
#pragma unroll
        for (int j = 0; j < 9; ++j) {
            const int hi = hi0 + bdh[j], wi = wi0 + bdw[j];
            const bool ok = rok & ((unsigned)hi < (unsigned)a.H) & ((unsigned)wi < (unsigned)a.W);
            dma(ok ? (const void*)(gx + pix + boff[j]) : zero, sb + j * BB + lw * 1024);
        }
        // next step's pixel: + BK = (adv_b, adv_p, adv_q), one carry per component at most
        int nq = q + a.adv_q, np = p + a.adv_p, nb = b + a.adv_b;
        if (nq >= a.Q) { nq -= a.Q; ++np; }
        if (np >= a.P) { np -= a.P; ++nb; }
        b = nb; p = np; q = nq;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const bool ok = ms + arow[h] < a.M;
#pragma unroll
            for (int ab = 0; ab < 2; ++ab) {
                dma(ok ? (const void*)ap[h][ab] : zero, sb + B + ab * AB + (2 * lw + h) * 1024);
                ap[h][ab] += astep;
            }
        }
        slot = slot + 1 == S ? 0 : slot + 1;
    };
    for (int i = 0; i < D && i < nst; ++i) issue(i);
    for (int i = 0; i < nst; ++i) {
        // step i has landed (13 pieces per step per loader wave; the D - 1 younger steps may stay
        // in flight, at the tail everything); after the barrier no compute wave reads step i - 1's
        // slot any more: step i + D refills it.  No DMA past the range, so none is in flight once
        // the last barrier has passed.
        if (i + D - 1 < nst) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(13 * (D - 1)) : "memory");
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        if (i + D < nst) issue(i + D);
    }
}

// ---------------------------------------------------------------------------------
// Weight gradient of the pixel-pair stem (7 x 4 filter over 8-channel pairs, strides
// (2, 1), 64 output channels, no padding): dw[n][r][s][c] = sum over output pixels
// (b, p, q) of dy[b][p][q][n] x[b][2p + r][q + s][c].  A workgroup walks a contiguous
// run of output rows of one image with ONE WAVE PER TAP ROW r (7 waves): per output row
// the dy row (Q x 64 channels, 128-B pixel rows, XOR-swizzled 16-B chunks) and the input
// rows 2p .. 2p + 6 (a ring of two-row units, as k_conv_stem) sit in LDS; wave r reduces
// over the row's pixels in 16-pixel k-steps: A = dy^T (two 32-channel blocks), B = the
// input row 2p + r read as the [q][(s, c)] matrix whose rows overlap (row q = pairs
// q .. q + 3, 64 B at a 16-B pitch) - both by ds_read_b64_tr_b16, so one B fragment
// feeds two MFMAs and the whole tap row (s, c) = 32 columns is one accumulator column
// block.  Operands are register-staged two rows ahead (compiler-visible LDS accesses,
// exact waits); each workgroup writes its fp32 [64][224] partial, k_wgrad_sum reduces
// them in a fixed order.  The generic kernel (k_conv_wgrad4 <1, 2>) re-staged every
// input pixel per tap through an im2col tile: 117 us alone, 142 us in the step.
struct WStemArgs {
    const uint16_t* dy;  // [G][N][P][Q][64]: the output gradient, or (BN) the stem output y
    const uint16_t* x;   // [G][N][Hi][Wi][8] (pixel pairs)
    float* part;         // [G][splits][64][R * S * 8]
    int P, Q, Wi;
    int cpi, L, splits;  // chunks per image, output rows per chunk, workgroups per group (N * cpi)
    int uchunks, upitch, ichunks;  // 16-B chunks per unit (two input rows), LDS slot bytes, chunks per image
    long long gs_dy, gs_x;
    // BN (k_wgrad_stem<R, S, true>): dy formed in the loader from the stem's BatchNorm + ReLU +
    // max-pool backward (gm_conv2d_wgrad_stem_bn_grouped_bf16)
    const uint4* gp;     // [G][N][Pp][Qp][64] bf16 pool gradient
    const uint2* pidx;   // [G][N][Pp][Qp][64] window-relative argmax bytes
    const float* fcoef;  // group g: fcoef + g * fcoef_gs = sc[64], sh[64]
    const float* bcoef;  // group g: bcoef + g * bcoef_gs = ca[64], cb[64], cc[64]
    long long fcoef_gs, bcoef_gs, gs_pool;  // floats, floats, 16-B vectors
    int Pp, Qp;
};

// BN: the stem BatchNorm + ReLU + max-pool backward of the 8-channel chunks cg of the stem output y
// at row s, columns 2 pp and 2 pp + 1 (y0, y1), exactly as k_stem_pool_bn_bwd<true> forms dx
// (batchnorm.hip): the fp32 sum, in window order, of the pool gradients whose argmax is the
// element, rounded to bf16, masked by relu(y * sc + sh), then ca * d + (cb * y + cc) rounded to
// bf16.  Both columns lie in pool column pp (the odd one also in pp + 1), so each window's data is
// read once for the pair.  pool_g / pool_i: the two LDS slots of pooled rows (slot k & 1: gradient
// [Qp][64] bf16, argmax bytes [Qp][64]); cf: sc, sh, ca, cb, cc [64] each.
__device__ __forceinline__ void stem_bn_dx2(uint4& y0, uint4& y1, int s, int pp, int cg, const char* pool_g,
                                            const char* pool_i, const float* cf, int Pp, int Qp) {
    const int k0 = s >> 1, dh = s & 1;
    const uint32_t yw[2][4] = {{y0.x, y0.y, y0.z, y0.w}, {y1.x, y1.y, y1.z, y1.w}};
    uint32_t ow[2][4];
    const bool right = pp + 1 < Qp;
    // two halves of four channels, one after the other
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        float d0[4] = {0.f, 0.f, 0.f, 0.f}, d1[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int wr = 0; wr < 2; ++wr) {
            const int k = k0 + wr;
            if (wr > dh || k >= Pp) continue;  // uniform
            const int rb = (dh - 2 * wr + 1) * 3;  // window row of row s, times 3
            const char* gk = pool_g + (k & 1) * Qp * 128 + cg * 16 + h * 8;
            const char* ik = pool_i + (k & 1) * Qp * 64 + cg * 8 + h * 4;
            const uint2 ga = *reinterpret_cast<const uint2*>(gk + pp * 128);
            const uint32_t ia = *reinterpret_cast<const uint32_t*>(ik + pp * 64);
            uint2 gb = make_uint2(0, 0);
            uint32_t ib = ~0u;  // no window right of the last pool column: never a position
            if (right) {
                gb = *reinterpret_cast<const uint2*>(gk + (pp + 1) * 128);
                ib = *reinterpret_cast<const uint32_t*>(ik + (pp + 1) * 64);
            }
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const uint32_t ba = (ia >> (8 * i)) & 0xffu, bb = (ib >> (8 * i)) & 0xffu;
                const float va = (i & 1) ? bf_hi(i < 2 ? ga.x : ga.y) : bf_lo(i < 2 ? ga.x : ga.y);
                const float vb = (i & 1) ? bf_hi(i < 2 ? gb.x : gb.y) : bf_lo(i < 2 ? gb.x : gb.y);
                // column 2pp: window (k, pp) at window column 1; column 2pp + 1: window (k, pp) at
                // column 2, then window (k, pp + 1) at column 0 (the reference's window order)
                if (ba == (uint32_t)(rb + 1)) d0[i] += va;
                if (ba == (uint32_t)(rb + 2)) d1[i] += va;
                if (bb == (uint32_t)rb) d1[i] += vb;
            }
        }
        const float4* c4 = reinterpret_cast<const float4*>(cf + cg * 8 + 4 * h);
        const float4 sc = c4[0], sh = c4[16], ca = c4[32], cb = c4[48], cc = c4[64];
        const float scv[4] = {sc.x, sc.y, sc.z, sc.w}, shv[4] = {sh.x, sh.y, sh.z, sh.w};
        const float cav[4] = {ca.x, ca.y, ca.z, ca.w}, cbv[4] = {cb.x, cb.y, cb.z, cb.w};
        const float ccv[4] = {cc.x, cc.y, cc.z, cc.w};
#pragma unroll
        for (int c = 0; c < 2; ++c) {
            float o[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int j = 4 * h + i;
                const float xf = (j & 1) ? bf_hi(yw[c][j >> 1]) : bf_lo(yw[c][j >> 1]);
                const float dr = __uint_as_float((uint32_t)Elem<uint16_t>::f2bf(c ? d1[i] : d0[i]) << 16);
                const float dm = fmaf(xf, scv[i], shv[i]) > 0.f ? dr : 0.f;
                o[i] = fmaf(cav[i], dm, fmaf(cbv[i], xf, ccv[i]));
            }
            ow[c][2 * h] = pack_bf2(o[0], o[1]);
            ow[c][2 * h + 1] = pack_bf2(o[2], o[3]);
        }
        __builtin_amdgcn_sched_barrier(0);
    }
    y0 = make_uint4(ow[0][0], ow[0][1], ow[0][2], ow[0][3]);
    y1 = make_uint4(ow[1][0], ow[1][1], ow[1][2], ow[1][3]);
}

template <int R, int S>
__global__ __launch_bounds__(64 * R) void k_wgrad_stem(WStemArgs a) {
    constexpr int NT = 64 * R;                // threads: one wave per tap row
    constexpr int TC = R * S * 8;             // dw columns per output channel
    constexpr int DPT = (1024 + NT - 1) / NT;  // dy chunks per thread per row (Q <= 128)
    constexpr int RING = 8;
    static_assert(S * 8 == 32, "k_wgrad_stem: one tap row = one 32-column accumulator block");
    extern __shared__ __attribute__((aligned(16))) uint4 wsm[];
    char* lds = reinterpret_cast<char*>(wsm);  // [dy tiles 2 x Q*128][ring 8 x upitch]
    const int t = threadIdx.x, lane = t & 63;
    const int rr = __builtin_amdgcn_readfirstlane(t >> 6);
    const int grp = blockIdx.x / a.splits, wg = blockIdx.x - grp * a.splits;
    const int b = wg / a.cpi, c = wg - b * a.cpi;
    const int p0 = c * a.L, p1 = min(a.P, p0 + a.L);
    const int tileb = a.Q * 128, dchunks = a.Q * 8;
    char* const ring = lds + 2 * tileb;
    const uint4* const gdy = reinterpret_cast<const uint4*>(a.dy + grp * a.gs_dy) + (size_t)b * a.P * dchunks;
    const uint4* const gx = reinterpret_cast<const uint4*>(a.x + grp * a.gs_x) + (size_t)b * a.ichunks;
    struct Stage {
        uint4 d[DPT];
        uint4 x;
    };
    // dy row pr and input unit u (rows 2u, 2u + 1) -> registers; zeros past the image
    auto fetch = [&](int pr, int u, Stage& st, bool with_dy = true) __attribute__((always_inline)) {
#pragma unroll
        for (int h = 0; h < DPT && with_dy; ++h) {
            const int cc = t + NT * h;
            st.d[h] = (cc < dchunks && pr < a.P) ? gdy[(size_t)pr * dchunks + cc] : make_uint4(0, 0, 0, 0);
        }
        const int gi = u * a.uchunks + t;
        st.x = (t < a.uchunks && gi < a.ichunks) ? gx[gi] : make_uint4(0, 0, 0, 0);
    };
    auto stash = [&](int pr, int u, const Stage& st, bool with_dy = true) __attribute__((always_inline)) {
        char* tile = lds + (pr & 1) * tileb;
#pragma unroll
        for (int h = 0; h < DPT && with_dy; ++h) {
            const int cc = t + NT * h;
            if (cc < dchunks) {
                const int px = cc >> 3, j = cc & 7;
                *reinterpret_cast<uint4*>(tile + px * 128 + ((j ^ wswz<128>(px)) << 4)) = st.d[h];
            }
        }
        if (t < a.uchunks) *reinterpret_cast<uint4*>(ring + (u & (RING - 1)) * a.upitch + t * 16) = st.x;
    };
    {  // prologue: dy row p0 and units p0 .. p0 + 3 (row p0's window)
        Stage s0, s1;
        fetch(p0, p0, s0, true);
        fetch(0, p0 + 1, s1, false);
        stash(p0, p0, s0, true);
        stash(0, p0 + 1, s1, false);
        fetch(0, p0 + 2, s0, false);
        fetch(0, p0 + 3, s1, false);
        stash(0, p0 + 2, s0, false);
        stash(0, p0 + 3, s1, false);
    }
    Stage sa, sb;  // iteration p stashes dy row p + 1 and unit p + 4, then fetches row p + 3, unit p + 6
    fetch(p0 + 1, p0 + 4, sa);
    fetch(p0 + 2, p0 + 5, sb);

    floatx16 acc[2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[i][e] = 0.f;
    // tr-read lane geometry: 16-lane group g reads pixel rows 8 (g >> 1) + q4 (+ 4) of a
    // 16-pixel slice, columns 16 (g & 1) + 4 p4 .. + 3; lane l receives column l % 32
    const int g4 = lane >> 4, q4 = (lane >> 2) & 3, p4 = lane & 3;
    const int krow = 8 * (g4 >> 1) + q4, col = 16 * (g4 & 1) + 4 * p4;
    auto rowoff = [](int row, int ch) { return row * 128 + ((((ch >> 3) ^ wswz<128>(row))) << 4) + (ch & 7) * 2; };
    const int nks = a.Q >> 4;
    auto iteration = [&](int p, Stage& st) __attribute__((always_inline)) {
        __syncthreads();  // row p's dy tile and units p .. p + 3 are in LDS; row p - 1's reads are done
        stash(p + 1, p + 4, st);
        fetch(p + 3, p + 6, st);
        const char* tile = lds + (p & 1) * tileb;
        const char* xrow = ring + ((p + (rr >> 1)) & (RING - 1)) * a.upitch + (rr & 1) * a.Wi * 16;
        for (int ks = 0; ks < nks; ++ks) {
            const int px = 16 * ks + krow;
            const bf16x8 A0 = tr_frag(reinterpret_cast<const uint16_t*>(tile + rowoff(px, col)),
                                      reinterpret_cast<const uint16_t*>(tile + rowoff(px + 4, col)));
            const bf16x8 A1 = tr_frag(reinterpret_cast<const uint16_t*>(tile + rowoff(px, 32 + col)),
                                      reinterpret_cast<const uint16_t*>(tile + rowoff(px + 4, 32 + col)));
            const char* xb = xrow + (px + (col >> 3)) * 16 + (col & 7) * 2;
            const bf16x8 B = tr_frag(reinterpret_cast<const uint16_t*>(xb), reinterpret_cast<const uint16_t*>(xb + 64));
            acc[0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A0, B, acc[0], 0, 0, 0);
            acc[1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A1, B, acc[1], 0, 0, 0);
        }
    };
    for (int p = p0; p < p1; p += 2) {
        iteration(p, sa);
        if (p + 1 < p1) iteration(p + 1, sb);
    }
    // the partial: dw[channel][rr * 32 + (s, c)], lane -> column, registers -> channels
    float* out = a.part + ((size_t)grp * a.splits + wg) * (64 * TC) + rr * 32 + (lane & 31);
#pragma unroll
    for (int nb = 0; nb < 2; ++nb)
#pragma unroll
        for (int e = 0; e < 16; ++e) out[(size_t)(nb * 32 + 8 * (e >> 2) + 4 * (lane >> 5) + (e & 3)) * TC] = acc[nb][e];
}

// k_wgrad_stem_bn: k_wgrad_stem with dy formed in the loader (stem_bn_dx2 above) - the stem's
// BatchNorm + ReLU + max-pool backward is never written (gm_conv2d_wgrad_stem_bn_grouped_bf16).
// Forming dy costs ~450 VALU instructions per wave and row, so the MFMA waves of ONE workgroup
// would serialise it with their MFMAs (barrier per row); here a workgroup is FOUR waves (tap rows
// {2w, 2w + 1}, wave 3 row 6 only: the busiest SIMD issues the same 28 MFMAs per row as
// k_wgrad_stem's), so two workgroups fit a CU (81 KB of LDS each, 2 waves per SIMD: up to 256
// VGPRs) and one's dy forming overlaps the other's MFMAs.  The A fragments (dy) of a k-slice feed
// both of a wave's tap rows.  Rows are prefetched three iterations ahead.  Same MFMA operands and
// order as k_wgrad_stem on the same tiles: bit-identical partials.
constexpr int kStemBnDepth = 3;  // rows of y in flight (registers; 2: 216 VGPRs, room for a split-sum wave beside it - equal in the step, profiles/r06_stem_wgrad_ab.txt)
template <int R, int S>
__global__ __launch_bounds__(256) void k_wgrad_stem_bn(WStemArgs a) {
    constexpr int NT = 256;
    constexpr int TC = R * S * 8;
    constexpr int RING = 8;
    static_assert(S * 8 == 32 && R == 7, "k_wgrad_stem_bn: the 7 x 4 pixel-pair stem");
    extern __shared__ __attribute__((aligned(16))) uint4 wsm[];
    char* lds = reinterpret_cast<char*>(wsm);  // [dy tiles 2][unit ring 8][pooled 2 x (grad, argmax)][coef]
    const int t = threadIdx.x, lane = t & 63;
    const int w = __builtin_amdgcn_readfirstlane(t >> 6);
    const int grp = blockIdx.x / a.splits, wg = blockIdx.x - grp * a.splits;
    const int b = wg / a.cpi, c = wg - b * a.cpi;
    const int p0 = c * a.L, p1 = min(a.P, p0 + a.L);
    const int tileb = a.Q * 128, dchunks = a.Q * 8;
    const int npair = a.Q * 4;   // (column pair, channel chunk) items per row, <= 2 NT (host)
    const int npool = a.Qp * 8;  // pooled vectors per row, <= 2 NT (host)
    char* const ring = lds + 2 * tileb;
    char* const pool_g = ring + RING * a.upitch;
    char* const pool_i = pool_g + 2 * a.Qp * 128;
    float* const cf = reinterpret_cast<float*>(pool_i + 2 * a.Qp * 64);
    const uint4* const gy = reinterpret_cast<const uint4*>(a.dy + grp * a.gs_dy) + (size_t)b * a.P * dchunks;
    const uint4* const gx = reinterpret_cast<const uint4*>(a.x + grp * a.gs_x) + (size_t)b * a.ichunks;
    const size_t pimg = (size_t)b * a.Pp * a.Qp * 8;
    const uint4* const gpp = a.gp + grp * a.gs_pool + pimg;
    const uint2* const gpi = a.pidx + grp * a.gs_pool + pimg;
    const int cg = t & 7;  // the channel chunk of every item of this thread (NT % 8 == 0)
    struct Stage {
        uint4 y[2][2];  // item h = t + NT h: columns 2 pp, 2 pp + 1 of chunk cg (pp = item >> 3)
        uint4 x;        // unit chunk t
    };
    struct Pool {
        uint4 g[2];  // pooled vector t + NT h
        uint2 i[2];
    };
    auto fetch = [&](int pr, int u, Stage& st) __attribute__((always_inline)) {
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int it = t + NT * h;
            const bool ok = it < npair && pr < a.P;
            const size_t o = (size_t)pr * dchunks + (size_t)(it >> 3) * 16 + cg;
            st.y[h][0] = ok ? gy[o] : make_uint4(0, 0, 0, 0);
            st.y[h][1] = ok ? gy[o + 8] : make_uint4(0, 0, 0, 0);
        }
        const int gi = u * a.uchunks + t;
        st.x = (t < a.uchunks && gi < a.ichunks) ? gx[gi] : make_uint4(0, 0, 0, 0);
    };
    auto fetch_pool = [&](int pk, Pool& pq) __attribute__((always_inline)) {
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int v = t + NT * h;
            const bool ok = pk < a.Pp && v < npool;
            const size_t o = (size_t)pk * npool + v;
            pq.g[h] = ok ? gpp[o] : make_uint4(0, 0, 0, 0);
            pq.i[h] = ok ? gpi[o] : make_uint2(0, 0);
        }
    };
    auto stash_pool = [&](int pk, const Pool& pq) __attribute__((always_inline)) {
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int v = t + NT * h;
            if (v < npool) {
                *reinterpret_cast<uint4*>(pool_g + (pk & 1) * a.Qp * 128 + v * 16) = pq.g[h];
                *reinterpret_cast<uint2*>(pool_i + (pk & 1) * a.Qp * 64 + v * 8) = pq.i[h];
            }
        }
    };
    auto stash_unit = [&](int u, const Stage& st) __attribute__((always_inline)) {
        if (t < a.uchunks) *reinterpret_cast<uint4*>(ring + (u & (RING - 1)) * a.upitch + t * 16) = st.x;
    };
    // dy row pr from y row pr (registers) and the pooled rows in LDS, into tile pr & 1
    auto stash_dy = [&](int pr, const Stage& st) __attribute__((always_inline)) {
        char* tile = lds + (pr & 1) * tileb;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int it = t + NT * h;
            if (it < npair) {
                const int pp = it >> 3;
                uint4 v0 = st.y[h][0], v1 = st.y[h][1];
                stem_bn_dx2(v0, v1, pr, pp, cg, pool_g, pool_i, cf, a.Pp, a.Qp);
                const int px = 2 * pp;
                *reinterpret_cast<uint4*>(tile + px * 128 + ((cg ^ wswz<128>(px)) << 4)) = v0;
                *reinterpret_cast<uint4*>(tile + (px + 1) * 128 + ((cg ^ wswz<128>(px + 1)) << 4)) = v1;
            }
        }
    };
    const int k0 = p0 >> 1;  // p0 is even (the host plan's L is)
    Pool pq;
    {  // prologue: units p0 .. p0 + 3, pooled rows k0, k0 + 1, the coefficients; then dy row p0
        Stage s0, s1;
        fetch(p0, p0, s0);
        fetch(a.P, p0 + 1, s1);
        fetch_pool(k0, pq);
        stash_unit(p0, s0);
        stash_unit(p0 + 1, s1);
        stash_pool(k0, pq);
        fetch_pool(k0 + 1, pq);
        if (t < 64) {
            const float* fc = a.fcoef + grp * a.fcoef_gs;
            const float* bc = a.bcoef + grp * a.bcoef_gs;
            cf[t] = fc[t];
            cf[64 + t] = fc[64 + t];
            cf[128 + t] = bc[t];
            cf[192 + t] = bc[64 + t];
            cf[256 + t] = bc[128 + t];
        }
        stash_pool(k0 + 1, pq);
        fetch(a.P, p0 + 2, s1);
        stash_unit(p0 + 2, s1);
        fetch(a.P, p0 + 3, s1);
        stash_unit(p0 + 3, s1);
        __syncthreads();  // pooled rows k0, k0 + 1 and the coefficients are in LDS
        stash_dy(p0, s0);
    }
    // iteration p stashes dy row p + 1 and unit p + 4, then fetches row p + 4, unit p + 7.  Pooled
    // row j is fetched in iteration 2j - 5 and stashed in iteration 2j - 3 (odd iterations, one
    // register set), one iteration before row 2j - 1 - its first reader - is formed, after the
    // last reader of row j - 2 (its slot) - row 2j - 3, formed in iteration 2j - 4
    Stage sa, sb, sc;
    fetch(p0 + 1, p0 + 4, sa);
    fetch(p0 + 2, p0 + 5, sb);
    if constexpr (kStemBnDepth == 3) fetch(p0 + 3, p0 + 6, sc);
    fetch_pool(k0 + 2, pq);

    floatx16 acc[2][2];  // [tap row of the wave][channel block]
#pragma unroll
    for (int r = 0; r < 2; ++r)
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int e = 0; e < 16; ++e) acc[r][i][e] = 0.f;
    const bool two = w < 3;  // wave 3: tap row 6 only
    const int g4 = lane >> 4, q4 = (lane >> 2) & 3, p4 = lane & 3;
    const int krow = 8 * (g4 >> 1) + q4, col = 16 * (g4 & 1) + 4 * p4;
    auto rowoff = [](int row, int ch) { return row * 128 + ((((ch >> 3) ^ wswz<128>(row))) << 4) + (ch & 7) * 2; };
    const int nks = a.Q >> 4;
    auto iteration = [&](int p, Stage& st) __attribute__((always_inline)) {
        __syncthreads();  // row p's dy tile and units p .. p + 3 are in LDS; row p - 1's reads are done
        stash_unit(p + 4, st);
        if (p & 1) {
            stash_pool((p + 3) >> 1, pq);
            fetch_pool((p + 5) >> 1, pq);
        }
        stash_dy(p + 1, st);
        fetch(p + kStemBnDepth + 1, p + kStemBnDepth + 4, st);
        const char* tile = lds + (p & 1) * tileb;
        // tap rows 2w, 2w + 1 read input rows 2(p + w), 2(p + w) + 1: one unit
        const char* xrow = ring + ((p + w) & (RING - 1)) * a.upitch;
        for (int ks = 0; ks < nks; ++ks) {
            const int px = 16 * ks + krow;
            const bf16x8 A0 = tr_frag(reinterpret_cast<const uint16_t*>(tile + rowoff(px, col)),
                                      reinterpret_cast<const uint16_t*>(tile + rowoff(px + 4, col)));
            const bf16x8 A1 = tr_frag(reinterpret_cast<const uint16_t*>(tile + rowoff(px, 32 + col)),
                                      reinterpret_cast<const uint16_t*>(tile + rowoff(px + 4, 32 + col)));
            const char* xb = xrow + (px + (col >> 3)) * 16 + (col & 7) * 2;
            const bf16x8 B0 = tr_frag(reinterpret_cast<const uint16_t*>(xb), reinterpret_cast<const uint16_t*>(xb + 64));
            acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A0, B0, acc[0][0], 0, 0, 0);
            acc[0][1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A1, B0, acc[0][1], 0, 0, 0);
            if (two) {
                const char* xb1 = xb + a.Wi * 16;
                const bf16x8 B1 = tr_frag(reinterpret_cast<const uint16_t*>(xb1),
                                          reinterpret_cast<const uint16_t*>(xb1 + 64));
                acc[1][0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A0, B1, acc[1][0], 0, 0, 0);
                acc[1][1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A1, B1, acc[1][1], 0, 0, 0);
            }
        }
    };
    if constexpr (kStemBnDepth == 3) {
        for (int p = p0; p < p1; p += 3) {
            iteration(p, sa);
            if (p + 1 < p1) iteration(p + 1, sb);
            if (p + 2 < p1) iteration(p + 2, sc);
        }
    } else {
        for (int p = p0; p < p1; p += 2) {
            iteration(p, sa);
            if (p + 1 < p1) iteration(p + 1, sb);
        }
    }
    // the partial: dw[channel][rr * 32 + (s, c)] for the wave's tap rows rr = 2w (+ 1)
#pragma unroll
    for (int r = 0; r < 2; ++r) {
        if (r == 1 && !two) break;
        float* out = a.part + ((size_t)grp * a.splits + wg) * (64 * TC) + (2 * w + r) * 32 + (lane & 31);
#pragma unroll
        for (int nb = 0; nb < 2; ++nb)
#pragma unroll
            for (int e = 0; e < 16; ++e)
                out[(size_t)(nb * 32 + 8 * (e >> 2) + 4 * (lane >> 5) + (e & 3)) * TC] = acc[r][nb][e];
    }
}
// The stem's weight gradient from its padded pixel-pair layout [G][K][R][Sp][2][4] (fp32) into each
// view's parameter gradient [K][R][S][C0] (the channels_last [K, C0, R, S] parameter): one launch
// for every view instead of a strided copy per view (gm_stem_dw_crop)
constexpr int kCropG = 16;
struct StemCropArgs {
    const float* dwp;
    float* dst[kCropG];
    int K, R, S, C0, Sp, accumulate;
};

__global__ __launch_bounds__(256) void k_stem_dw_crop(StemCropArgs a) {
    const int g = blockIdx.y;
    const int n = a.K * a.R * a.S * a.C0;
    const int o = blockIdx.x * 256 + threadIdx.x;
    if (o >= n) return;
    int t = o;
    const int c = t % a.C0;
    t /= a.C0;
    const int s = t % a.S;
    t /= a.S;
    const int r = t % a.R, k = t / a.R;
    const float v = a.dwp[(size_t)g * a.K * a.R * a.Sp * 8 + ((size_t)(k * a.R + r) * a.Sp + (s >> 1)) * 8 + (s & 1) * 4 + c];
    float* d = a.dst[g] + o;
    *d = a.accumulate ? *d + v : v;
}

// dw[i] (+)= sum over splits of part[s][i] in ONE launch, for the uncropped case (Cp == Cr,
// every layer but the RGB stem).  A wave covers 64/R float4 columns with R split lanes per
// column (lane r sums splits r, r+R, ..., eight loads in flight), and the R lane sums are
// combined inside the wave by a fixed xor tree (DPP row rotate, swizzle, bpermute) - a fixed
// summation order for a given shape (deterministic) and NO LDS: these sums run on the weight-
// gradient stream beside LDS-heavy kernels (k_wgrad_halo64, k_wgrad_stem hold most of a CU's
// LDS), where the former LDS combine could not place its workgroups (the stem's sum: 6.3 us
// alone, 34 us in the step).  R is picked on the host so that small slabs still spread over
// hundreds of waves.
template <int C>
__device__ __forceinline__ float wsum_dpp(float v) {
    return v + __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), C, 0xf, 0xf, false));
}
__device__ __forceinline__ float wsum_x16(float v) {
    return v + __int_as_float(__builtin_amdgcn_ds_swizzle(__float_as_int(v), 0x401f));
}
template <int R>
__global__ __launch_bounds__(256) void k_wgrad_sum(const float* __restrict__ part, int splits, size_t slab,
                                                   int accumulate, float* __restrict__ dw, long long gs_dw) {
    static_assert(R == 1 || R == 2 || R == 4 || R == 8, "k_wgrad_sum: 1, 2, 4 or 8 split lanes");
    constexpr int CPW = 64 / R, CPB = 4 * CPW;
    part += (size_t)blockIdx.y * splits * slab;  // view group blockIdx.y
    dw += blockIdx.y * gs_dw;
    const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
    const int r = lane / CPW, cw = lane - r * CPW;
    const size_t i4 = ((size_t)blockIdx.x * CPB + wave * CPW + cw) * 4;
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    if (i4 < slab) {
        const float* p = part + i4;
        int s = r;
        for (; s + 7 * R < splits; s += 8 * R) {
            float4 v[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) v[j] = *(const float4*)(p + (size_t)(s + j * R) * slab);
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                acc.x += v[j].x; acc.y += v[j].y; acc.z += v[j].z; acc.w += v[j].w;
            }
        }
        for (; s < splits; s += R) {
            const float4 v = *(const float4*)(p + (size_t)s * slab);
            acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
        }
    }
    // the split lanes of a column are lanes cw + CPW q: xor 8 (row rotate 8), 16, 32
    if constexpr (R >= 8) {
        acc.x = wsum_dpp<0x128>(acc.x); acc.y = wsum_dpp<0x128>(acc.y);
        acc.z = wsum_dpp<0x128>(acc.z); acc.w = wsum_dpp<0x128>(acc.w);
    }
    if constexpr (R >= 4) {
        acc.x = wsum_x16(acc.x); acc.y = wsum_x16(acc.y); acc.z = wsum_x16(acc.z); acc.w = wsum_x16(acc.w);
    }
    if constexpr (R >= 2) {
        acc.x += __shfl_xor(acc.x, 32); acc.y += __shfl_xor(acc.y, 32);
        acc.z += __shfl_xor(acc.z, 32); acc.w += __shfl_xor(acc.w, 32);
    }
    if (r != 0 || i4 >= slab) return;
    float4* o = (float4*)(dw + i4);
    if (accumulate) {
        const float4 v = *o;
        acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
    }
    *o = acc;
}

// dw = sum over splits (fixed order); also the [K][T][Cpad] -> [K][T][Creal] crop
__global__ __launch_bounds__(256) void k_wgrad_reduce(const float* part, int splits, int Kc, int T, int Cp,
                                                      int Cr, int accumulate, float* dw, long long gs_dw) {
    const size_t n = (size_t)Kc * T * Cr;
    const size_t slab = (size_t)Kc * T * Cp;
    part += (size_t)blockIdx.y * splits * slab;  // view group blockIdx.y
    dw += blockIdx.y * gs_dw;
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

static int wgrad_target_wgs() {
    static int w = [] {
        return 512;
    }();
    return w;
}

struct WPlan {
    int P, Q, tiles_k, tiles_n, splits, sps, mt, nt;
};

static WPlan plan(const gm_conv_desc_hw* d, int G = 1) {
    WPlan w;
    w.P = (d->H + 2 * d->pad_h - d->R) / d->stride_h + 1;
    w.Q = (d->W + 2 * d->pad_w - d->S) / d->stride_w + 1;
    const int M = d->N * w.P * w.Q;
    const int steps = (M + 63) / 64;
    const int TC = d->R * d->S * d->C;
    // 128 x 128 tiles where the shape allows (256-row / 256-column tiles at one workgroup per
    // CU measured 1.2-1.6x slower in round 2 and were dropped)
    w.mt = d->K >= 128 ? 2 : 1;
    w.nt = TC >= 128 ? 2 : 1;
    w.tiles_k = (d->K + 64 * w.mt - 1) / (64 * w.mt);
    w.tiles_n = (TC + 64 * w.nt - 1) / (64 * w.nt);
    const int tiles = w.tiles_k * w.tiles_n * G;  // the groups' tiles share the chip
    const int target = wgrad_target_wgs();
    const int min_steps = 8;
    int want = target > tiles ? target / tiles : 1;
    if (tiles >= 256) want = 1;  // the chip is full: no partial slabs
    if (want > steps / min_steps) want = steps / min_steps > 0 ? steps / min_steps : 1;
    if (want < 1) want = 1;
    w.sps = (steps + want - 1) / want;
    w.splits = (steps + w.sps - 1) / w.sps;
    return w;
}

}  // namespace gm

using namespace gm;

// operand staging of k_conv_wgrad4 (its WR argument; gm_conv_set_wgrad_staging): 0 LDS-DMA,
// 1 register-staged, 2 (default) register-staged for 1x1 filters only.  Isolated
// (tools/trunk_table.py) the register-staged form is faster on the 1x1/s2 downsample
// gradients (16.6-18.7 vs 18.0-19.6 us) and slower on every 3x3 shape (layer 4 64.6 ->
// 73.6 us, conv family 0.195 -> 0.191); in the step, where the weight gradients run beside
// the input-gradient chain, the all-register form measured 0.4 % faster on average over
// nine interleaved pairs, within the box-to-box noise.
static int g_wgrad_wr = [] {
    return 2;
}();

// weight-gradient kernel choice for 3x3 / s1 / p1 shapes with W <= 62 (gm_conv_set_wgrad_loop,
// gm_conv_set_wgrad_loop): bit 1 = k_wgrad_halo64 for 64 channels (layer 1), bit 2 = also for
// 128 channels (layer 2); bit 4 = k_wgrad_ring for the other 3x3 shapes it serves (K % 128 == 0,
// C % 32 == 0: layers 3 / 4 and the strided first convolutions); otherwise k_conv_wgrad4.
// Default 22 (bits 1, 2: r04, B = 64 two-view step: layer 1 61.9 -> 44.9 us and layer 2
// 54.6 -> 46.6 us per launch with the sum; step 3.98 -> 3.91 ms against bit 1 alone).
static int g_wgrad_loop = [] {
    return 22;
}();

template <int MT, int NT>
static int launch_wgrad4(const WgradArgs& a, int grid, hipStream_t st) {
    const size_t lds = (size_t)2 * 64 * 2 * (64 * MT + 64 * NT);
    static bool attr = false;  // idempotent, safe to race
    if (!attr) {
        (void)hipFuncSetAttribute((const void*)k_conv_wgrad4<MT, NT>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        (void)hipFuncSetAttribute((const void*)k_conv_wgrad4<MT, NT, 1>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  (int)lds);
        attr = true;
    }
    if (g_wgrad_wr == 1 || (g_wgrad_wr == 2 && a.T == 1)) k_conv_wgrad4<MT, NT, 1><<<grid, 256, lds, st>>>(a);
    else k_conv_wgrad4<MT, NT><<<grid, 256, lds, st>>>(a);
    return check_launch("k_conv_wgrad4");
}

static gm_conv_desc_hw to_hw(const gm_conv_desc* d) {
    return gm_conv_desc_hw{d->N, d->H, d->W, d->C, d->K, d->R, d->S, d->stride, d->stride, d->pad, d->pad};
}

// k_wgrad_halo64 serves 3x3 / s1 / p1 shapes with W <= 62: image rows of PP = 16, 32 or 64
// positions (PP >= W + 2), 64 / PP of them per super-row
static int halo64_pp(int W) { return W + 2 <= 16 ? 16 : (W + 2 <= 32 ? 32 : 64); }
static bool halo64_ok(const gm_conv_desc_hw* d) {
    // bit 1: 64 channels (layer 1), bit 2: up to 128 (layer 2), bit 3: up to 512 (layers 3, 4)
    const int maxc = (g_wgrad_loop & 8) ? 512 : ((g_wgrad_loop & 4) ? 128 : 64);
    return (g_wgrad_loop & 2) && d->R == 3 && d->S == 3 && d->stride_h == 1 && d->stride_w == 1 && d->pad_h == 1 &&
           d->pad_w == 1 && d->C % 64 == 0 && d->K % 64 == 0 && d->C <= maxc && d->K <= maxc && d->W <= 62 &&
           d->W >= 1 && d->H >= 64 / halo64_pp(d->W) && d->N >= 1 &&
           (long long)d->N * d->H * d->W * (d->C > d->K ? d->C : d->K) < (1ll << 31);
}
// workgroups per (view group, channel tile): 128 in all - half the
// CUs: the launch runs on the weight-gradient stream beside the input-gradient chain, and one
// workgroup per CU (512 threads, 81 KB of LDS) left no room on any CU for that chain's BN
// finalize / apply launches (C2, in the step: 64 / 96 / 128 / 160 / 256 workgroups = 3.80 /
// 3.67 / 3.63 / 3.63 / 3.70 ms; as k_wgrad_ring's half-CU grid)
static int halo64_wgs() {
    static const int w = [] {
        const int v = 128;
        return v < 8 ? 8 : v;
    }();
    return w;
}
static int halo64_splits(const gm_conv_desc_hw* d, int G) {
    const int rps = 64 / halo64_pp(d->W);
    const int srows = (d->N * d->H + rps - 1) / rps;
    const int tiles = (d->K / 64) * (d->C / 64) * G;
    int sp = halo64_wgs() / tiles;
    if (sp < 1) sp = 1;
    return sp < srows ? sp : srows;
}

// k_wgrad_ring serves 3x3 shapes (any stride / padding) with K % 128 == 0 and C a power of two
// >= 32 (gm_conv_set_wgrad_loop bit 4, default on): tiles x splits sized to one workgroup per CU
static int device_cus_w() {
    static const int cus = [] {
        int dev = 0, n = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
            return 256;
        return n;
    }();
    return cus;
}
// k_wgrad_ring's grid: HALF the CUs.  The ring runs on the weight-gradient stream beside the main
// chain's input-gradient convolutions and BatchNorms, and a workgroup holds its CU's LDS (156 KB):
// one per CU starved the main chain (C2 step 3.94 ms against 3.85 without the ring), half the CUs
// left the other half to it (3.75 ms; 64 / 96 / 160 / 192 / 224 workgroups: 3.77 / 3.77 / 3.80 /
// 3.80 / 3.80 ms, r05 interleaved A/B).  Alone a launch then takes longer (conv family 0.218 vs
// 0.228 isolated).  Measured and dropped (r05): 6 slots of 32 pixels (+0.06-0.24 ms/step), 2 slots.
struct RingPlan {
    int P, Q, M, tiles_k, tiles_n, splits, sps;
};
static bool ring_plan(const gm_conv_desc_hw* d, int G, RingPlan& r) {
    if (!(g_wgrad_loop & 16) || d->R != 3 || d->S != 3 || d->K % 128 != 0 || d->C % 32 != 0 || ilog2w(d->C) < 5 ||
        d->K < 128)
        return false;
    r.P = (d->H + 2 * d->pad_h - 3) / d->stride_h + 1;
    r.Q = (d->W + 2 * d->pad_w - 3) / d->stride_w + 1;
    if (r.P < 1 || r.Q < 1 || d->N < 1) return false;
    const long long M = (long long)d->N * r.P * r.Q;
    if (M * d->K >= (1ll << 31) || (long long)d->N * d->H * d->W * d->C >= (1ll << 31)) return false;
    r.M = (int)M;
    r.tiles_k = d->K / 128;
    r.tiles_n = d->C / 32;  // 9 C / 288
    const int tiles = r.tiles_k * r.tiles_n * G;
    constexpr int bk = ring::BK;
    const int steps = (r.M + bk - 1) / bk;
    int want = (device_cus_w() / 2) / tiles;
    if (want > steps / (512 / bk)) want = steps / (512 / bk);  // >= 512 pixels per split
    if (want < 1) want = 1;
    r.sps = (steps + want - 1) / want;
    r.splits = (steps + r.sps - 1) / r.sps;
    return true;
}

// k_wgrad_stem serves the pixel-pair stem: 8-channel pairs, 64 output channels, a 7 x 4
// filter, strides (2, 1), no padding, output rows of a multiple of 16 and <= 128 pixels
static int g_wgrad_stem = [] {
    return 1;  // 0: the stem's weight gradient takes k_conv_wgrad4
}();
struct StemWPlan {
    int P, Q, cpi, L, splits;
};
static bool stemw_plan(const gm_conv_desc_hw* d, int G, StemWPlan& w) {
    if (!g_wgrad_stem || d->C != 8 || d->K != 64 || d->R != 7 || d->S != 4 || d->stride_h != 2 || d->stride_w != 1 ||
        d->pad_h != 0 || d->pad_w != 0 || d->N < 1 || d->H < 7 || d->W < 4)
        return false;
    w.P = (d->H - 7) / 2 + 1;
    w.Q = d->W - 3;
    if (w.Q % 16 != 0 || w.Q > 128 || 2 * d->W > 448 || (long long)d->H * d->W >= (1ll << 27)) return false;
    if ((long long)d->N * w.P * w.Q * 64 >= (1ll << 31)) return false;
    const int target = 512 / G > 0 ? 512 / G : 1;
    const int cpi0 = std::max(1, std::min(w.P, target / d->N));
    w.L = (w.P + cpi0 - 1) / cpi0;
    w.L += w.L & 1;  // even: the BN form's pooled-row schedule starts on an even row
    w.cpi = (w.P + w.L - 1) / w.L;
    w.splits = d->N * w.cpi;
    return true;
}

extern "C" size_t gm_conv2d_wgrad_grouped_scratch(const gm_conv_desc_hw* d, int G) {
    if (!d || d->stride_h < 1 || d->stride_w < 1 || G < 1) return 0;
    // the launch takes the stem / halo kernels only when c_real == C and otherwise falls
    // through to k_conv_wgrad4, which this query cannot tell apart: size for the larger plan
    const WPlan w = plan(d, G);
    const size_t slab = (size_t)d->K * d->R * d->S * d->C;
    size_t need = (size_t)G * w.splits * slab * sizeof(float);
    StemWPlan sw;
    RingPlan rp;
    if (stemw_plan(d, G, sw)) need = std::max(need, (size_t)G * sw.splits * 64 * 224 * 4);
    else if (halo64_ok(d)) need = std::max(need, (size_t)G * halo64_splits(d, G) * d->K * 9 * d->C * 4);
    else if (ring_plan(d, G, rp) && rp.splits > 1) need = std::max(need, (size_t)G * rp.splits * slab * sizeof(float));
    return need;
}

extern "C" int gm_conv_set_wgrad_stem(int on) {
    g_wgrad_stem = on ? 1 : 0;
    return GM_OK;
}

extern "C" size_t gm_conv2d_wgrad_hw_scratch(const gm_conv_desc_hw* d) {
    return gm_conv2d_wgrad_grouped_scratch(d, 1);
}

extern "C" size_t gm_conv2d_wgrad_scratch(const gm_conv_desc* d) {
    if (!d) return 0;
    const gm_conv_desc_hw h = to_hw(d);
    return gm_conv2d_wgrad_hw_scratch(&h);
}


static WStemArgs stem_args(const gm_conv_desc_hw* d, const StemWPlan& sw, const void* dy, const void* x,
                           void* scratch) {
    WStemArgs s{};
    s.dy = (const uint16_t*)dy;
    s.x = (const uint16_t*)x;
    s.part = (float*)scratch;
    s.P = sw.P; s.Q = sw.Q; s.Wi = d->W;
    s.cpi = sw.cpi; s.L = sw.L; s.splits = sw.splits;
    s.uchunks = 2 * d->W;
    s.upitch = s.uchunks * 16;
    s.ichunks = d->H * d->W;
    s.gs_dy = (long long)d->N * sw.P * sw.Q * 64;
    s.gs_x = (long long)d->N * d->H * d->W * 8;
    return s;
}

template <bool BN>
static int launch_wgrad_stem(const WStemArgs& s, const StemWPlan& sw, int G, size_t lds, hipStream_t st) {
    static size_t granted = 0;
    const void* fn = BN ? (const void*)k_wgrad_stem_bn<7, 4> : (const void*)k_wgrad_stem<7, 4>;
    if (lds > granted) {
        if (hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess) {
            set_error("k_wgrad_stem: %zu B of LDS refused", lds);
            return GM_E_UNSUP;
        }
        granted = lds;
    }
    if (BN) k_wgrad_stem_bn<7, 4><<<sw.splits * G, 256, lds, st>>>(s);
    else k_wgrad_stem<7, 4><<<sw.splits * G, 448, lds, st>>>(s);
    return check_launch(BN ? "k_wgrad_stem_bn" : "k_wgrad_stem");
}

// the split sum of every split weight-gradient kernel: k_wgrad_sum with R split lanes per
// column (at most 8, inside one wave), enough waves for small slabs
static int launch_wgrad_sum(const float* part, int splits, size_t slab, int accumulate, float* dw, long long gs,
                            int G, hipStream_t st) {
    const size_t ncol = slab / 4;
    int R = 1;
    while (R < 8 && R * 2 <= splits && (ncol * R + 255) / 256 < 512) R *= 2;
    const dim3 gg((unsigned)((ncol + 256 / R - 1) / (256 / R)), (unsigned)G);
    switch (R) {
        case 1: k_wgrad_sum<1><<<gg, 256, 0, st>>>(part, splits, slab, accumulate, dw, gs); break;
        case 2: k_wgrad_sum<2><<<gg, 256, 0, st>>>(part, splits, slab, accumulate, dw, gs); break;
        case 4: k_wgrad_sum<4><<<gg, 256, 0, st>>>(part, splits, slab, accumulate, dw, gs); break;
        default: k_wgrad_sum<8><<<gg, 256, 0, st>>>(part, splits, slab, accumulate, dw, gs); break;
    }
    return check_launch("k_wgrad_sum");
}

// G view groups in one launch: group g reads dy + g*N*P*Q*K and x + g*N*H*W*C (the views
// stacked along the batch) and writes its weight gradient to dw + g*dw_stride (floats)
extern "C" int gm_conv2d_wgrad_grouped_bf16(const gm_conv_desc_hw* d, int G, const void* dy, const void* x,
                                            float* dw, long long dw_stride, int c_real, int accumulate,
                                            void* scratch, size_t scratch_bytes, void* stream) {
    GM_REQUIRE(d && dy && x && dw, "conv wgrad: null pointer");
    GM_REQUIRE(G >= 1 && G <= 64, "conv wgrad: view groups must be 1..64 (got %d)", G);
    GM_REQUIRE(d->stride_h >= 1 && d->stride_w >= 1 && d->pad_h >= 0 && d->pad_w >= 0, "conv wgrad: bad stride/pad");
    GM_REQUIRE(d->R * d->S <= kWTap, "conv wgrad: at most %d taps", kWTap);
    GM_REQUIRE(ilog2w(d->C) >= 3, "conv wgrad: C must be a power of two >= 8");
    GM_REQUIRE(d->K % 8 == 0, "conv wgrad: K must be a multiple of 8");
    GM_REQUIRE(c_real >= 1 && c_real <= d->C, "conv wgrad: bad c_real");
    const size_t slab_c = (size_t)d->K * d->R * d->S * (size_t)c_real;
    GM_REQUIRE(G == 1 || (dw_stride >= (long long)slab_c || dw_stride <= -(long long)slab_c),
               "conv wgrad: group gradient stride %lld overlaps one gradient", dw_stride);
    const size_t need = gm_conv2d_wgrad_grouped_scratch(d, G);
    GM_REQUIRE(scratch && scratch_bytes >= need, "conv wgrad: scratch %zu < %zu", scratch_bytes, need);
    hipStream_t st0 = as_stream(stream);
    auto split_sum = [&](float* part, int splits, size_t slab) {
        return launch_wgrad_sum(part, splits, slab, accumulate, dw, dw_stride, G, st0);
    };
    StemWPlan sw;
    if (stemw_plan(d, G, sw) && c_real == d->C) {
        const WStemArgs s = stem_args(d, sw, dy, x, scratch);
        int rc = launch_wgrad_stem<false>(s, sw, G, (size_t)2 * sw.Q * 128 + (size_t)8 * s.upitch, st0);
        if (rc) return rc;
        return split_sum(s.part, sw.splits, (size_t)64 * 224);
    }
    if (halo64_ok(d) && c_real == d->C) {
        WHaloArgs h;
        h.dy = (const uint16_t*)dy;
        h.x = (const uint16_t*)x;
        h.part = (float*)scratch;
        h.N = d->N; h.H = d->H; h.W = d->W;
        h.rows = d->N * d->H;
        const int pp = halo64_pp(d->W);
        h.srows = (h.rows + 64 / pp - 1) / (64 / pp);
        h.splits = halo64_splits(d, G);
        h.rpw = (h.srows + h.splits - 1) / h.splits;
        h.K = d->K; h.C = d->C; h.kt = d->K / 64; h.ct = d->C / 64;
        h.gs_dy = (long long)d->N * d->H * d->W * d->K;
        h.gs_x = (long long)d->N * d->H * d->W * d->C;
        // D = 3 super-rows of LDS-DMA in flight
        const int nblk = h.splits * h.kt * h.ct * G;
        auto go = [&](auto pc) {
            constexpr int D = 3, PP = decltype(pc)::value;
            constexpr size_t lds = (size_t)(D + 3) * 8192 + (size_t)(D + 1) * (8192 + 256);
            static bool attr = false;
            if (!attr) {
                (void)hipFuncSetAttribute((const void*)k_wgrad_halo64<D, PP>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                          (int)lds);
                attr = true;
            }
            k_wgrad_halo64<D, PP><<<nblk, 512, lds, st0>>>(h);
        };
        if (pp == 16) go(std::integral_constant<int, 16>{});
        else if (pp == 32) go(std::integral_constant<int, 32>{});
        else go(std::integral_constant<int, 64>{});
        int rc = check_launch("k_wgrad_halo64");
        if (rc) return rc;
        return launch_wgrad_sum(h.part, h.splits, (size_t)d->K * 9 * d->C, accumulate, dw, dw_stride, G, st0);
    }
    RingPlan rp;
    if (c_real == d->C && ring_plan(d, G, rp)) {
        WRingArgs r;
        memset(&r, 0, sizeof(r));
        r.dy = (const uint16_t*)dy;
        r.x = (const uint16_t*)x;
        r.N = d->N; r.H = d->H; r.W = d->W; r.C = d->C; r.logC = ilog2w(d->C); r.K = d->K;
        r.P = rp.P; r.Q = rp.Q; r.sth = d->stride_h; r.stw = d->stride_w; r.padh = d->pad_h; r.padw = d->pad_w;
        r.M = rp.M;
        r.tiles_k = rp.tiles_k; r.tiles_n = rp.tiles_n; r.splits = rp.splits; r.sps = rp.sps;
        r.fd_pq = FastDiv((uint32_t)(rp.P * rp.Q));
        r.fd_q = FastDiv((uint32_t)rp.Q);
        constexpr int BK = ring::BK;
        r.adv_b = BK / (rp.P * rp.Q);
        r.adv_p = (BK % (rp.P * rp.Q)) / rp.Q;
        r.adv_q = (BK % (rp.P * rp.Q)) % rp.Q;
        r.gs_dy = (long long)rp.M * d->K;
        r.gs_x = (long long)d->N * d->H * d->W * d->C;
        const size_t slab = (size_t)d->K * 9 * d->C;
        const bool direct = rp.splits == 1;
        r.part = direct ? dw : (float*)scratch;
        r.gs_part = direct ? dw_stride : (long long)rp.splits * (long long)slab;
        r.accumulate = direct ? accumulate : 0;
        const int grid = rp.tiles_k * rp.tiles_n * rp.splits * G;
        static bool attr = false;
        if (!attr) {
            if (hipFuncSetAttribute((const void*)k_wgrad_ring, hipFuncAttributeMaxDynamicSharedMemorySize,
                                    (int)ring::LDS) != hipSuccess) {
                set_error("k_wgrad_ring: %zu B of LDS refused", ring::LDS);
                return GM_E_UNSUP;
            }
            attr = true;
        }
        k_wgrad_ring<<<grid, 512, ring::LDS, st0>>>(r);
        const int rc = check_launch("k_wgrad_ring");
        if (rc || direct) return rc;
        return split_sum(r.part, rp.splits, slab);
    }
    WgradArgs a;
    memset(&a, 0, sizeof(a));
    const WPlan w = plan(d, G);
    a.P = w.P; a.Q = w.Q; a.tiles_k = w.tiles_k; a.tiles_n = w.tiles_n;
    a.splits = w.splits; a.steps_per_split = w.sps;
    a.dy = (const uint16_t*)dy;
    a.x = (const uint16_t*)x;
    a.part = (float*)scratch;
    a.N = d->N; a.H = d->H; a.W = d->W; a.C = d->C; a.logC = ilog2w(d->C);
    a.Kc = d->K; a.T = d->R * d->S; a.sth = d->stride_h; a.stw = d->stride_w;
    a.fd_pq = FastDiv((uint32_t)(a.P * a.Q));
    a.fd_q = FastDiv((uint32_t)a.Q);
    a.G = G;
    a.gs_dy = (long long)d->N * w.P * w.Q * d->K;
    a.gs_x = (long long)d->N * d->H * d->W * d->C;
    a.gs_part = (long long)w.splits * d->K * a.T * d->C;
    a.adv_b = 64 / (a.P * a.Q);
    a.adv_p = (64 % (a.P * a.Q)) / a.Q;
    a.adv_q = (64 % (a.P * a.Q)) % a.Q;
    for (int r = 0; r < d->R; ++r)
        for (int s = 0; s < d->S; ++s) {
            a.dh[r * d->S + s] = (signed char)(r - d->pad_h);
            a.dw[r * d->S + s] = (signed char)(s - d->pad_w);
        }
    hipStream_t st = as_stream(stream);
    const int grid = a.tiles_k * a.tiles_n * a.splits * G;
    int rc;
    const bool direct = a.splits == 1 && c_real == d->C;
    if (direct) {
        a.part = dw;
        a.gs_part = dw_stride;
        a.accumulate = accumulate;
    }
    a.S = d->S;
    a.padh = d->pad_h;
    a.padw = d->pad_w;
    if (w.mt == 2 && w.nt == 2) rc = launch_wgrad4<2, 2>(a, grid, st);
    else if (w.mt == 2) rc = launch_wgrad4<2, 1>(a, grid, st);
    else if (w.nt == 2) rc = launch_wgrad4<1, 2>(a, grid, st);
    else rc = launch_wgrad4<1, 1>(a, grid, st);
    if (rc || direct) return rc;
    const size_t slab = (size_t)d->K * a.T * d->C;
    if (c_real == d->C)  // one-launch split reduction (slab is a multiple of 4: K % 8 == 0)
        return launch_wgrad_sum(a.part, a.splits, slab, accumulate, dw, dw_stride, G, st);
    const size_t n = (size_t)d->K * a.T * c_real;
    int g = (int)((n + 255) / 256);
    if (g > 4096) g = 4096;
    k_wgrad_reduce<<<dim3(g, G), 256, 0, st>>>(a.part, a.splits, d->K, a.T, d->C, c_real, accumulate, dw,
                                               dw_stride);
    return check_launch("k_wgrad_reduce");
}


// The stem's weight gradient with dy formed in the loader (greedymml.h: the stem BatchNorm +
// ReLU + max-pool backward, never written): k_wgrad_stem<7, 4, true> on the k_wgrad_stem plan
static bool stem_bn_plan(const gm_conv_desc_hw* d, int G, StemWPlan& sw) {
    // k_wgrad_stem_bn: two (column pair, chunk) items and two pooled vectors per thread, a unit
    // chunk per thread
    return d && G >= 1 && G <= 64 && stemw_plan(d, G, sw) && sw.Q * 4 <= 2 * 256 && ((sw.Q + 1) / 2) * 8 <= 2 * 256 &&
           2 * d->W <= 256 && !(sw.L & 1);
}

extern "C" int gm_conv2d_wgrad_stem_bn_ok(const gm_conv_desc_hw* d, int G) {
    StemWPlan sw;
    return stem_bn_plan(d, G, sw) ? 1 : 0;
}

extern "C" int gm_conv2d_wgrad_stem_bn_grouped_bf16(const gm_conv_desc_hw* d, int G, const gm_stem_bn_src* src,
                                                    const void* x, float* dw, long long dw_stride, int accumulate,
                                                    void* scratch, size_t scratch_bytes, void* stream) {
    const char* fn = "gm_conv2d_wgrad_stem_bn_grouped_bf16";
    GM_REQUIRE(d && src && src->y && src->dy_pool && src->idx && src->fcoef && src->bcoef && x && dw,
               "%s: null pointer", fn);
    GM_REQUIRE(G >= 1 && G <= 64, "%s: view groups must be 1..64 (got %d)", fn, G);
    StemWPlan sw;
    if (!stem_bn_plan(d, G, sw)) {
        set_error("%s: not the pixel-pair stem shape of k_wgrad_stem with Q <= 112", fn);
        return GM_E_UNSUP;
    }
    const int Pp = (sw.P + 1) / 2, Qp = (sw.Q + 1) / 2;
    GM_REQUIRE(G == 1 || dw_stride >= 64 * 224 || dw_stride <= -64 * 224, "%s: group gradient stride overlaps", fn);
    const size_t need = gm_conv2d_wgrad_grouped_scratch(d, G);
    GM_REQUIRE(scratch && scratch_bytes >= need, "%s: scratch %zu < %zu", fn, scratch_bytes, need);
    WStemArgs s = stem_args(d, sw, src->y, x, scratch);
    s.gp = static_cast<const uint4*>(src->dy_pool);
    s.pidx = static_cast<const uint2*>(src->idx);
    s.fcoef = src->fcoef;
    s.bcoef = src->bcoef;
    s.fcoef_gs = src->fcoef_gs;
    s.bcoef_gs = src->bcoef_gs;
    s.gs_pool = (long long)d->N * Pp * Qp * 8;
    s.Pp = Pp;
    s.Qp = Qp;
    hipStream_t st = as_stream(stream);
    const size_t lds = (size_t)2 * sw.Q * 128 + (size_t)8 * s.upitch + (size_t)2 * Qp * 192 + 5 * 64 * sizeof(float);
    int rc = launch_wgrad_stem<true>(s, sw, G, lds, st);
    if (rc) return rc;
    return launch_wgrad_sum(s.part, sw.splits, (size_t)64 * 224, accumulate, dw, dw_stride, G, st);
}

extern "C" int gm_conv2d_wgrad_hw_bf16(const gm_conv_desc_hw* d, const void* dy, const void* x, float* dw,
                                       int c_real, int accumulate, void* scratch, size_t scratch_bytes,
                                       void* stream) {
    return gm_conv2d_wgrad_grouped_bf16(d, 1, dy, x, dw, 0, c_real, accumulate, scratch, scratch_bytes, stream);
}

extern "C" int gm_conv_set_wgrad_staging(int wr) {
    GM_REQUIRE(wr >= 0 && wr <= 2,
               "gm_conv_set_wgrad_staging: 0 (LDS-DMA), 1 (register-staged), 2 (register-staged for 1x1 filters)");
    g_wgrad_wr = wr;
    return GM_OK;
}

extern "C" int gm_conv_set_wgrad_loop(int mode) {
    GM_REQUIRE(mode >= 0 && mode <= 31 && !(mode & 1),
               "gm_conv_set_wgrad_loop: bit 1 halo kernel for 64 channels, bit 2 up to 128, bit 3 up to 512, "
               "bit 4 the ring kernel for 3x3 shapes with K % 128 == 0, C % 32 == 0");
    g_wgrad_loop = mode;
    return GM_OK;
}

extern "C" int gm_conv2d_wgrad_bf16(const gm_conv_desc* d, const void* dy, const void* x, float* dw, int c_real,
                                    int accumulate, void* scratch, size_t scratch_bytes, void* stream) {
    GM_REQUIRE(d, "conv wgrad: null pointer");
    const gm_conv_desc_hw h = to_hw(d);
    return gm_conv2d_wgrad_hw_bf16(&h, dy, x, dw, c_real, accumulate, scratch, scratch_bytes, stream);
}

extern "C" int gm_stem_dw_crop(const float* dwp, int G, int K, int R, int S, int C0, int Sp, float* const* dst,
                               int accumulate, void* stream) {
    GM_REQUIRE(dwp && dst && G >= 1 && G <= kCropG && K > 0 && R > 0 && S > 0 && C0 >= 1 && C0 <= 4 &&
                   Sp == (S + 1) / 2,
               "gm_stem_dw_crop: bad arguments");
    StemCropArgs a{};
    a.dwp = dwp;
    for (int g = 0; g < G; ++g) {
        GM_REQUIRE(dst[g], "gm_stem_dw_crop: null destination %d", g);
        a.dst[g] = dst[g];
    }
    a.K = K; a.R = R; a.S = S; a.C0 = C0; a.Sp = Sp; a.accumulate = accumulate ? 1 : 0;
    const int n = K * R * S * C0;
    k_stem_dw_crop<<<dim3((unsigned)((n + 255) / 256), (unsigned)G), 256, 0, as_stream(stream)>>>(a);
    return check_launch("k_stem_dw_crop");
}
