// 1x1 / stride-1 / pad-0 convolutions in NHWC are plain NT GEMMs over the pixels: the ResNet-50
// bottleneck's reduce / expand convolutions and their input gradients (C5 workload, SURVEY §8 row
// f4; torchvision Bottleneck conv1 / conv3 + downsample of layer 1, autocast bf16).  The im2col
// kernel ran them at 0.09-0.18 of the MFMA peak: most have a short reduction (K = 64-512), so a
// 128 x 128 tile is one to eight 64-deep k-steps, each paid for with a DMA round trip, a barrier
// and an epilogue - latency, not math or bytes.
//
//   Out[g][m][n] = sum_k A[g][m][k] * B[g][n][k]  (+ Addend[g][m][n]),  bf16 in/out, fp32 accumulate
//   forward: A = x [M][C], B = w [K][C] (KRSC, R = S = 1),   Out = y  [M][K]
//   dgrad:   A = dy [M][K], B = wt [C][K] (the transposed copy), Out = dx [M][C] (+ the join addend)
//
// k_gemm_ring: a PERSISTENT workgroup walks a strided list of output tiles; the (tile, k-step)
// units of its list stream through an S-slot LDS ring filled by four LOADER waves (LDS-DMA,
// S - 1 units in flight, one raw s_barrier per unit after a counted vmcnt - the pattern of
// k_wgrad_ring), so a tile's DMA, the previous tile's epilogue stores and the MFMAs overlap
// across tile boundaries; four COMPUTE waves (2 x 2, 64 pixels x BN/2 channels each) read
// ds_read_b128 fragments from 128-B rows whose 16-B chunks are XOR-swizzled by (row >> 1) & 7
// on the source side (conflict-free for the b128 lane groups), weights as the MFMA A operand
// so each lane owns 4 consecutive output channels of one pixel; the epilogue transposes each
// wave's 32-pixel halves through private fp32 LDS rows into 16-B NHWC stores through a buffer
// resource (rows past M dropped by the hardware, addend loads in flight together).
#include <cstdint>
#include <cstring>

#include "gm_common.h"

namespace gm {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float floatx16 __attribute__((ext_vector_type(16)));

struct RingGemmArgs {
    const uint16_t* A;       // [G][M][Kr]
    const uint16_t* B;       // [G][N][Kr]
    uint16_t* out;           // [G][M][N]
    const uint16_t* addend;  // [G][M][N] or null (may alias out)
    const uint8_t* amask;    // with it, optional: its 1-bit mask (mask_bf2), [G][M * N / 8]
    // A rows gathered from a strided 1x1 convolution's input (forward, stride sst > 0): row m =
    // output pixel (b, p, q) of [.][sP][sQ] reads input pixel (b, sst p, sst q) of [.][sH][sW];
    // scatter (input gradient): A = dy rows read densely, out row m written to input pixel
    // (b, sst p, sst q) of the [orows = M / (sP sQ) * sH * sW][N] output
    int sst, sH, sW, sP, sQ, scatter;
    long long orows;
    int M, N, Kr;            // per group
    int G, tiles_m, tiles_n, tiles;  // tiles = G * tiles_m * tiles_n
    long long gsA, gsB, gsO; // group strides (elements; gsB may be negative)
    // forward, optional: BatchNorm partial rows of the stored output, as ConvArgs::stats
    // (row = a wave's 64-pixel slab, group g at stats + g * 2 N (stats_rows + 1))
    float* stats;
    int stats_rows;
    // input gradient, optional (with stats): the BatchNorm backward's statistics instead
    // (ConvArgs::bnx): dz = out where x sc + sh > 0, sums of dz and dz (x - mean)
    const uint16_t* bnx;
    const float* bncoef;  // [G][2 N]
    const float* bnmean;  // [G][N]
};

// sum over the lanes xor 8, 16, 32 (the lanes sharing lane % 8): DPP row rotate by 8, a
// swizzle xor 16, a bpermute xor 32
__device__ __forceinline__ float sum_lanes_8(float v) {
    v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x128, 0xf, 0xf, false));
    v += __int_as_float(__builtin_amdgcn_ds_swizzle(__float_as_int(v), 0x401f));
    v += __shfl_xor(v, 32);
    return v;
}

__device__ __attribute__((aligned(16))) const uint4 g_rzero16[1] = {{0u, 0u, 0u, 0u}};

template <int BN, int S>
__global__ __launch_bounds__(512) void k_gemm_ring(RingGemmArgs a) {
    static_assert(BN == 64 || BN == 128, "k_gemm_ring: 64 or 128 output channels per tile");
    static_assert(S >= 2, "k_gemm_ring: at least two slots");
    constexpr int BM = 128, D = S - 1;
    constexpr int SA = BM * 128, SB = BN * 128, SLOT = SA + SB;  // bytes
    constexpr int PA = SA / 1024 / 4, PB = SB / 1024 / 4;        // DMA pieces per loader wave per unit
    constexpr int NT = BN / 64;                                  // 32-channel fragments per wave
    extern __shared__ __attribute__((aligned(16))) uint4 gsm[];
    char* lds = reinterpret_cast<char*>(gsm);
    const int t = threadIdx.x, lane = t & 63;
    const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
    const int nk = a.Kr >> 6;  // 64-deep k-steps per tile
    // this workgroup's tiles: vb, vb + gridDim.x, ...; units = tiles x k-steps.  Workgroups are
    // dealt round-robin over the 8 XCDs (b on XCD b % 8): vb gives each XCD a contiguous block of
    // every round's tile ids, so the tiles_n output-channel tiles of one pixel block run together
    // on one XCD and fetch its activation rows from HBM once (into that L2) instead of tiles_n times
    const int nb = (int)gridDim.x, b = (int)blockIdx.x;
    const int vb = nb % 8 == 0 ? (b & 7) * (nb >> 3) + (b >> 3) : b;
    const int ntiles = a.tiles > vb ? (a.tiles - 1 - vb) / nb + 1 : 0;
    const int nunits = ntiles * nk;
    auto tile_of = [&](int i, int& g, int& m0, int& n0) __attribute__((always_inline)) {
        int tl = vb + i * nb;
        const int per = a.tiles_m * a.tiles_n;
        g = tl / per;
        tl -= g * per;
        const int mt = tl / a.tiles_n;
        m0 = mt * BM;
        n0 = (tl - mt * a.tiles_n) * BN;
    };

    if (wave >= 4) {
        // ---- loader waves: A rows 32 lw .. + 31 (4 pieces of 8 rows), B rows (BN / 4) lw .. ----
        const int lw = wave - 4;
        typedef __attribute__((address_space(1))) const void* gptr_t;
        typedef __attribute__((address_space(3))) void* lptr_t;
        const void* zero = (const void*)g_rzero16;
        const int r8 = lane >> 3, ch = lane & 7;
        int slot = 0, ut = 0, uk = 0;  // next unit to issue: tile index ut, k-step uk
        int g = 0, m0 = 0, n0 = 0;
        long long ar[PA];  // this tile's A row offsets (elements; -1: past M), once per tile
        auto rows_of = [&]() __attribute__((always_inline)) {
#pragma unroll
            for (int j = 0; j < PA; ++j) {
                const int m = m0 + (lw * PA + j) * 8 + r8;
                long long o = (long long)m;
                if (a.sst && !a.scatter) {
                    const int PQ = a.sP * a.sQ, b = m / PQ, pq = m - b * PQ, p = pq / a.sQ, q = pq - p * a.sQ;
                    o = ((long long)b * a.sH + (long long)a.sst * p) * a.sW + (long long)a.sst * q;
                }
                ar[j] = m < a.M ? o * a.Kr : -1;
            }
        };
        if (nunits > 0) {
            tile_of(0, g, m0, n0);
            rows_of();
        }
        auto issue = [&]() __attribute__((always_inline)) {
            const unsigned sb = (unsigned)slot * SLOT;
            const uint16_t* Ag = a.A + g * a.gsA;
            const uint16_t* Bg = a.B + g * a.gsB;
            const int k0 = uk << 6;
#pragma unroll
            for (int j = 0; j < PA; ++j) {
                const int row = (lw * PA + j) * 8 + r8;
                const int c = (ch ^ ((row >> 1) & 7)) << 3;
                const void* src = ar[j] >= 0 ? (const void*)(Ag + ar[j] + k0 + c) : zero;
                __builtin_amdgcn_global_load_lds((gptr_t)src, (lptr_t)(lds + sb + (lw * PA + j) * 1024), 16, 0, 0);
            }
#pragma unroll
            for (int j = 0; j < PB; ++j) {
                const int row = (lw * PB + j) * 8 + r8;
                const int c = (ch ^ ((row >> 1) & 7)) << 3;
                __builtin_amdgcn_global_load_lds((gptr_t)(Bg + (size_t)(n0 + row) * a.Kr + k0 + c),
                                                 (lptr_t)(lds + sb + SA + (lw * PB + j) * 1024), 16, 0, 0);
            }
            slot = slot + 1 == S ? 0 : slot + 1;
            if (++uk == nk) {
                uk = 0;
                if (++ut < ntiles) {
                    tile_of(ut, g, m0, n0);
                    rows_of();
                }
            }
        };
        for (int i = 0; i < D && i < nunits; ++i) issue();
        for (int i = 0; i < nunits; ++i) {
            // unit i has landed (D - 1 younger ones may stay in flight; at the tail all of them)
            if (i + D - 1 < nunits) asm volatile("s_waitcnt vmcnt(%0)" ::"n"((PA + PB) * (D - 1)) : "memory");
            else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __builtin_amdgcn_s_barrier();
            if (i + D < nunits) issue();  // into the slot unit i - 1 used (every read of it is done)
        }
        return;
    }

    // ---- compute waves ----
    const int wm = wave >> 1, wn = wave & 1;
    const int fr = lane & 31, fh = lane >> 5;
    // fragment row r, 16-B chunk of k-slice ks: (2 ks + fh) ^ ((r >> 1) & 7); the XOR term is
    // per lane, the k-slice an XOR of (ks << 5) on the byte offset
    unsigned aoff[2], boff[NT];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const int r = wm * 64 + i * 32 + fr;
        aoff[i] = (unsigned)(r * 128 + ((fh ^ ((r >> 1) & 7)) << 4));
    }
#pragma unroll
    for (int j = 0; j < NT; ++j) {
        const int r = wn * (BN / 2) + j * 32 + fr;
        boff[j] = (unsigned)(SA + r * 128 + ((fh ^ ((r >> 1) & 7)) << 4));
    }
    floatx16 acc[NT][2];
    auto zero_acc = [&]() __attribute__((always_inline)) {
#pragma unroll
        for (int j = 0; j < NT; ++j)
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int e = 0; e < 16; ++e) acc[j][i][e] = 0.f;
    };
    zero_acc();
    bf16x8 fa[2][2], fb[2][NT];  // [buffer][fragment]: activations (MFMA B), weights (MFMA A)
    auto load = [&](int ks, int c, const char* base) __attribute__((always_inline)) {
        const unsigned x = (unsigned)ks << 5;
#pragma unroll
        for (int i = 0; i < 2; ++i) fa[c][i] = *reinterpret_cast<const bf16x8*>(base + (aoff[i] ^ x));
#pragma unroll
        for (int j = 0; j < NT; ++j) fb[c][j] = *reinterpret_cast<const bf16x8*>(base + (boff[j] ^ x));
    };
    int slot = 0, g = 0, m0 = 0, n0 = 0;
    if (nunits > 0) tile_of(0, g, m0, n0);
    int uk = 0, ut = 0;
    for (int i = 0; i < nunits; ++i) {
        __builtin_amdgcn_s_barrier();  // unit i landed; every wave is done with unit i - 1's slot
        const char* base = lds + slot * SLOT;
        load(0, 0, base);
#pragma unroll
        for (int ks = 0; ks < 4; ++ks) {
            const int c = ks & 1;
            if (ks < 3) load(ks + 1, c ^ 1, base);
#pragma unroll
            for (int j = 0; j < NT; ++j)
#pragma unroll
                for (int ii = 0; ii < 2; ++ii)
                    acc[j][ii] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fb[c][j], fa[c][ii], acc[j][ii], 0, 0, 0);
        }
        // slice ks + 1's fragment reads go out BEFORE slice ks's MFMAs (k_conv_h9's schedule): the
        // counted lgkmcnt then waits for slice ks's reads only
        constexpr int NR = 2 + NT, NM = 2 * NT;
        __builtin_amdgcn_sched_group_barrier(0x100, NR, 0);
#pragma unroll
        for (int ks = 0; ks < 3; ++ks) {
            __builtin_amdgcn_sched_group_barrier(0x100, NR, 0);
            __builtin_amdgcn_sched_group_barrier(0x008, NM, 0);
        }
        __builtin_amdgcn_sched_group_barrier(0x008, NM, 0);
        // every LDS read of this unit must be done before the next barrier lets the loaders refill
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        slot = slot + 1 == S ? 0 : slot + 1;
        if (++uk == nk) {
            // epilogue of tile ut: lane (fr, fh) holds pixel 64 wm + 32 ii + fr, channels
            // (BN / 2) wn + 32 j + 8 q + 4 fh + 0..3 in registers 4 q .. 4 q + 3.  Direct 8-B stores
            // from that layout touch 32 rows per instruction and held the write-heavy shapes
            // (K = 64 -> 256) at 3 TB/s; instead each 32-pixel half goes through the wave's own
            // fp32 staging rows (16-B chunks XOR-swizzled) and leaves as 16-B stores, OPR lanes per
            // contiguous row segment - the addend added in fp32 before the one rounding, as before.
            constexpr int RB = NT * 128, OPR = 4 * NT, RPI = 64 / OPR;
            char* stg = lds + S * SLOT + wave * (32 * RB);
            auto swz = [](int r, int c) { return NT == 2 ? c ^ (r & 15) : c ^ ((r >> 1) & 7); };
            uint16_t* outp = a.out + g * a.gsO;
            const size_t obytes = (size_t)a.orows * a.N * 2;
            const auto orsrc = __builtin_amdgcn_make_buffer_rsrc(outp, 0, (int)obytes, 0x00020000);
            const auto arsrc = __builtin_amdgcn_make_buffer_rsrc(
                const_cast<uint16_t*>(a.addend ? a.addend + g * a.gsO : outp), 0, (int)obytes, 0x00020000);
            typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
            const int o = lane % OPR, rr = lane / OPR;
            const unsigned nb = (unsigned)(n0 + wn * (BN / 2) + 8 * o) * 2u;
            float bs1[8], bs2[8];  // BatchNorm statistics (a.stats): channels 8 o .. + 7 of the wave
#pragma unroll
            for (int e = 0; e < 8; ++e) bs1[e] = bs2[e] = 0.f;
            float bsc[8], bsh[8], bmu[8];  // backward statistics (a.bnx): the BN's coefficients
            if (a.stats && a.bnx) {
                const int n = n0 + wn * (BN / 2) + 8 * o;
                const float* cf = a.bncoef + (size_t)g * 2 * a.N + n;
                const float* mu = a.bnmean + (size_t)g * a.N + n;
#pragma unroll
                for (int e = 0; e < 8; e += 4) {
                    const float4 c0 = *reinterpret_cast<const float4*>(cf + e);
                    const float4 c1 = *reinterpret_cast<const float4*>(cf + a.N + e);
                    const float4 c2 = *reinterpret_cast<const float4*>(mu + e);
                    bsc[e] = c0.x; bsc[e + 1] = c0.y; bsc[e + 2] = c0.z; bsc[e + 3] = c0.w;
                    bsh[e] = c1.x; bsh[e + 1] = c1.y; bsh[e + 2] = c1.z; bsh[e + 3] = c1.w;
                    bmu[e] = c2.x; bmu[e + 1] = c2.y; bmu[e + 2] = c2.z; bmu[e + 3] = c2.w;
                }
            }
            const auto xrsrc = __builtin_amdgcn_make_buffer_rsrc(
                const_cast<uint16_t*>(a.bnx ? a.bnx + g * a.gsO : outp), 0, (int)obytes, 0x00020000);
#pragma unroll
            for (int ii = 0; ii < 2; ++ii) {
#pragma unroll
                for (int j = 0; j < NT; ++j)
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        const float4 v = {acc[j][ii][4 * q], acc[j][ii][4 * q + 1], acc[j][ii][4 * q + 2],
                                          acc[j][ii][4 * q + 3]};
                        *reinterpret_cast<float4*>(stg + fr * RB + swz(fr, 8 * j + 2 * q + fh) * 16) = v;
                    }
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                unsigned off[2 * NT];
#pragma unroll
                for (int it = 0; it < 2 * NT; ++it) {
                    const int m = m0 + wm * 64 + ii * 32 + it * RPI + rr;
                    unsigned orow = (unsigned)m;
                    if (a.scatter) {  // the strided input gradient: output pixel -> input pixel row
                        const int PQ = a.sP * a.sQ, b = m / PQ, pq = m - b * PQ, p = pq / a.sQ, q = pq - p * a.sQ;
                        orow = (unsigned)((b * a.sH + a.sst * p) * a.sW + a.sst * q);
                    }
                    off[it] = m < a.M ? orow * (unsigned)a.N * 2u + nb : 0xfffffff0u;
                }
                // (the addend test hoisted out of the loops: a per-element one branches and waits
                // vmcnt around every store)
                if (a.addend) {
                    u32x4 av[2 * NT];
#pragma unroll
                    for (int it = 0; it < 2 * NT; ++it) av[it] = __builtin_amdgcn_raw_buffer_load_b128(arsrc, off[it], 0, 0);
                    if (a.amask) {  // one mask byte per 16-B chunk: byte off / 16 (past the range: 0)
                        const auto mrsrc = __builtin_amdgcn_make_buffer_rsrc(
                            const_cast<uint8_t*>(a.amask + g * a.gsO / 8), 0, (int)(obytes >> 4), 0x00020000);
                        unsigned mb[2 * NT];
#pragma unroll
                        for (int it = 0; it < 2 * NT; ++it)
                            mb[it] = __builtin_amdgcn_raw_buffer_load_b8(mrsrc, off[it] >> 4, 0, 0);
#pragma unroll
                        for (int it = 0; it < 2 * NT; ++it) {
                            av[it].x = mask_bf2(av[it].x, mb[it]);
                            av[it].y = mask_bf2(av[it].y, mb[it] >> 2);
                            av[it].z = mask_bf2(av[it].z, mb[it] >> 4);
                            av[it].w = mask_bf2(av[it].w, mb[it] >> 6);
                        }
                    }
#pragma unroll
                    for (int it = 0; it < 2 * NT; ++it) {
                        const int row = it * RPI + rr;
                        const float4 f0 = *reinterpret_cast<const float4*>(stg + row * RB + swz(row, 2 * o) * 16);
                        const float4 f1 = *reinterpret_cast<const float4*>(stg + row * RB + swz(row, 2 * o + 1) * 16);
                        const u32x4 v = {pack_bf2(f0.x + bf_lo(av[it].x), f0.y + bf_hi(av[it].x)),
                                         pack_bf2(f0.z + bf_lo(av[it].y), f0.w + bf_hi(av[it].y)),
                                         pack_bf2(f1.x + bf_lo(av[it].z), f1.y + bf_hi(av[it].z)),
                                         pack_bf2(f1.z + bf_lo(av[it].w), f1.w + bf_hi(av[it].w))};
                        __builtin_amdgcn_raw_buffer_store_b128(v, orsrc, off[it], 0, 0);
                    }
                } else if (a.stats && a.bnx) {
                    u32x4 xv[2 * NT];  // the BN input's chunks at the stored positions (rows past M: 0)
#pragma unroll
                    for (int it = 0; it < 2 * NT; ++it) xv[it] = __builtin_amdgcn_raw_buffer_load_b128(xrsrc, off[it], 0, 0);
#pragma unroll
                    for (int it = 0; it < 2 * NT; ++it) {
                        const int row = it * RPI + rr;
                        const float4 f0 = *reinterpret_cast<const float4*>(stg + row * RB + swz(row, 2 * o) * 16);
                        const float4 f1 = *reinterpret_cast<const float4*>(stg + row * RB + swz(row, 2 * o + 1) * 16);
                        const u32x4 v = {pack_bf2(f0.x, f0.y), pack_bf2(f0.z, f0.w), pack_bf2(f1.x, f1.y),
                                         pack_bf2(f1.z, f1.w)};
                        __builtin_amdgcn_raw_buffer_store_b128(v, orsrc, off[it], 0, 0);
                        const bool ok = off[it] != 0xfffffff0u;
#pragma unroll
                        for (int e = 0; e < 8; ++e) {  // dz = dy where x sc + sh > 0 (the forward's ReLU)
                            const unsigned w = v[e >> 1], xw = xv[it][e >> 1];
                            const float x = (e & 1) ? bf_hi(xw) : bf_lo(xw);
                            const float d = ok && fmaf(x, bsc[e], bsh[e]) > 0.f ? ((e & 1) ? bf_hi(w) : bf_lo(w)) : 0.f;
                            bs1[e] += d;
                            bs2[e] = fmaf(d, x - bmu[e], bs2[e]);
                        }
                    }
                } else {
#pragma unroll
                    for (int it = 0; it < 2 * NT; ++it) {
                        const int row = it * RPI + rr;
                        const float4 f0 = *reinterpret_cast<const float4*>(stg + row * RB + swz(row, 2 * o) * 16);
                        const float4 f1 = *reinterpret_cast<const float4*>(stg + row * RB + swz(row, 2 * o + 1) * 16);
                        const u32x4 v = {pack_bf2(f0.x, f0.y), pack_bf2(f0.z, f0.w), pack_bf2(f1.x, f1.y),
                                         pack_bf2(f1.z, f1.w)};
                        __builtin_amdgcn_raw_buffer_store_b128(v, orsrc, off[it], 0, 0);
                        if (a.stats) {  // the stored (bf16) values, rows past M out
                            const bool ok = off[it] != 0xfffffff0u;
#pragma unroll
                            for (int e = 0; e < 8; ++e) {
                                const unsigned w = v[e >> 1];
                                const float f = ok ? ((e & 1) ? bf_hi(w) : bf_lo(w)) : 0.f;
                                bs1[e] += f;
                                bs2[e] = fmaf(f, f, bs2[e]);
                            }
                        }
                    }
                }
                // the next half's staging writes after every read of this one
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            }
            if (a.stats) {  // the wave's 64-pixel slab: partial row (m0 + 64 wm) / 64
#pragma unroll
                for (int e = 0; e < 8; ++e) {
                    if (NT == 1) {  // lanes sharing lane % 4: first fold xor 4
                        bs1[e] += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(bs1[e]), 0x124, 0xf, 0xf, false));
                        bs2[e] += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(bs2[e]), 0x124, 0xf, 0xf, false));
                    }
                    bs1[e] = sum_lanes_8(bs1[e]);
                    bs2[e] = sum_lanes_8(bs2[e]);
                }
                if (rr == 0 && m0 + wm * 64 < a.M) {  // (a slab past M: no row)
                    const int n = n0 + wn * (BN / 2) + 8 * o, row = (m0 + wm * 64) >> 6;
                    float4* dst = reinterpret_cast<float4*>(a.stats + (size_t)g * 2 * a.N * (a.stats_rows + 1) +
                                                            ((size_t)(n >> 6) * a.stats_rows + row) * 128 + (n & 63) * 2);
                    dst[0] = make_float4(bs1[0], bs2[0], bs1[1], bs2[1]);
                    dst[1] = make_float4(bs1[2], bs2[2], bs1[3], bs2[3]);
                    dst[2] = make_float4(bs1[4], bs2[4], bs1[5], bs2[5]);
                    dst[3] = make_float4(bs1[6], bs2[6], bs1[7], bs2[7]);
                }
            }
            zero_acc();
            uk = 0;
            if (++ut < ntiles) tile_of(ut, g, m0, n0);
        }
    }
}

static int g_ring_cus = [] {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
        return 256;
    return n;
}();

// gm_conv_set_1x1_gemm: 2 (default) = 1x1 / s1 shapes and 1x1 / s2 forwards (the downsamples, A rows
// gathered) take k_gemm_ring, 1 = the s1 shapes only, 0 = the im2col kernel
int g_conv_1x1 = [] {
    return 2;
}();

bool conv1x1s_ok(int R, int S, int sh, int sw, int ph, int pw, long long M, int Kr, int N) {
    return g_conv_1x1 >= 2 && R == 1 && S == 1 && sh == 2 && sw == 2 && ph == 0 && pw == 0 && M >= 1 &&
           Kr % 64 == 0 && Kr >= 64 && (N % 128 == 0 || N == 64) && M * (long long)(Kr > N ? Kr : N) < (1ll << 30);
}

bool conv1x1_ok(int R, int S, int sh, int sw, int ph, int pw, long long M, int Kr, int N) {
    return g_conv_1x1 && R == 1 && S == 1 && sh == 1 && sw == 1 && ph == 0 && pw == 0 && M >= 1 && Kr % 64 == 0 &&
           Kr >= 64 && (N % 128 == 0 || N == 64) && M * (long long)(Kr > N ? Kr : N) < (1ll << 30);
}

// Out = A . B^T (+ addend) per group; the caller checked conv1x1_ok
int conv1x1_gemm(long long M, int Kr, int N, int G, const void* A, long long gsA, const void* B, long long gsB,
                 void* out, long long gsO, const void* addend, hipStream_t st, const char* fn, float* stats,
                 const uint16_t* bnx, const float* bncoef, const float* bnmean, const uint8_t* amask,
                 const int* sgeo) {
    RingGemmArgs r;
    memset(&r, 0, sizeof(r));
    r.orows = M;
    if (sgeo) {  // {stride, H, W, P, Q, scatter}: A rows gathered from / out rows scattered to the strided map
        r.sst = sgeo[0]; r.sH = sgeo[1]; r.sW = sgeo[2]; r.sP = sgeo[3]; r.sQ = sgeo[4]; r.scatter = sgeo[5];
        if (r.scatter) r.orows = M / ((long long)r.sP * r.sQ) * r.sH * r.sW;
    }
    r.A = (const uint16_t*)A;
    r.B = (const uint16_t*)B;
    r.out = (uint16_t*)out;
    r.addend = (const uint16_t*)addend;
    r.amask = addend ? amask : nullptr;
    r.M = (int)M; r.N = N; r.Kr = Kr; r.G = G;
    const int BN = N % 128 == 0 ? 128 : 64;
    r.tiles_m = (int)((M + 127) / 128);
    r.tiles_n = N / BN;
    r.tiles = G * r.tiles_m * r.tiles_n;
    r.gsA = gsA; r.gsB = gsB; r.gsO = gsO;
    r.stats = addend || r.scatter ? nullptr : stats;
    r.bnx = r.stats ? bnx : nullptr;
    r.bncoef = bncoef;
    r.bnmean = bnmean;
    r.stats_rows = (int)((M + 63) / 64);
    const int grid = r.tiles < g_ring_cus ? r.tiles : g_ring_cus;  // persistent: one workgroup per CU
    auto go = [&](auto bnc) -> int {
        constexpr int BNt = decltype(bnc)::value, S = 4;
        // the ring + four compute waves' fp32 staging rows (32 pixels x BN / 2 channels each)
        constexpr size_t lds = (size_t)S * (128 * 128 + BNt * 128) + 4 * 32 * (BNt / 2) * 4;
        static bool attr = false;
        if (!attr) {
            if (hipFuncSetAttribute((const void*)k_gemm_ring<BNt, S>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                    (int)lds) != hipSuccess) {
                set_error("%s: %zu B of LDS refused", fn, lds);
                return GM_E_UNSUP;
            }
            attr = true;
        }
        k_gemm_ring<BNt, S><<<grid, 512, lds, st>>>(r);
        return check_launch(fn);
    };
    return BN == 128 ? go(std::integral_constant<int, 128>{}) : go(std::integral_constant<int, 64>{});
}

}  // namespace gm

extern "C" int gm_conv_set_1x1_gemm(int on) {
    gm::g_conv_1x1 = on < 0 ? 2 : on > 2 ? 2 : on;
    return GM_OK;
}
