// Backward of the GNN edge stage (training; reference train_helper_2d.py:114-126
// backpropagates loss.backward() through model / model_b, whose message passing
// is gnn_2d.py:53-63 + PyG aggr='mean').  Forward, per target i and in-edge e
// from source j = nbr[i, e] (e < deg_i):
//
//   z1 = a_i + b_j,  m1 = relu(z1),  z2 = W2 m1 + b2,  m = relu(z2),
//   mean_i = (1 / max(deg_i, 1)) sum_e m
//
// Given g = dL/dmean [n, 128] this computes
//
//   gz2 = g_i / max(deg_i, 1) * [z2 > 0],  gm1 = W2^T gz2,  gz1 = gm1 * [z1 > 0]
//   dL/da_i  = sum_e gz1                  (target side, summed in registers)
//   dL/db_j  = sum_{(i, e): nbr[i,e] = j} gz1   (source side: per-edge gz1 is
//              written out and summed per source over the reverse adjacency by
//              edge_source_sum_kernel, in a fixed order)
//   dL/dW2   = sum_e gz2 m1^T,  dL/db2 = sum_e gz2   (per-workgroup partials,
//              reduced in a fixed order by partial_sum_kernel)
//
// Nothing is stored by the forward: z1, z2 are recomputed here.  Exact fp32
// products on v_mfma_f32_16x16x4_f32 (the three 16 x 128 x 128 GEMMs of a
// neighbour slot: z2, gm1 and the dW2 outer products); no atomics, so the
// gradients are deterministic.
#include "common.hpp"
#include "f16x3.hpp"

#include <algorithm>

namespace {

constexpr int BH = 128;  // hidden width
constexpr int BT = 16;   // targets per tile
constexpr int BWS = BH + 8;  // LDS row stride (floats): 2-way bank aliasing for both row- and column-walks

struct EdgeBwdArgs {
    const float *a, *b;
    const int32_t *nbr;
    const int32_t *deg;  // nullable: every row has k in-edges
    int64_t n;
    int k, ntiles;
    const float *w2, *b2;  // message_net_2.0 weight [128 out][128 in], bias
    const float *gmean;    // [n, 128]
    float *ga;             // [n, 128]
    float *gz1;            // [n * k, 128] per edge (row q = i k + e, or pos[q])
    float *pw2, *pb2;      // [grid][128][128], [grid][128] partials
    const int32_t *pos;    // nullable: the gz1 row of slot q (source-major order)
    const uint32_t *mask;  // MASK: the forward's z2 > 0 bits, [n * k][4] (mmpde_gnn_edge_mean_ex)
};

// MASK: the ReLU pattern of z2 comes from the forward (bit c % 32 of word c / 32
// of the slot) instead of recomputing z2 -- the gradient of exactly the function
// the forward evaluated, whose z2 summation order differs from this kernel's.
template <bool MASK>
__global__ __launch_bounds__(256, 1) void edge_bwd_kernel(EdgeBwdArgs p) {
    // Row strides (round 6, SQ_LDS_BANK_CONFLICT was 61 % of this kernel's LDS
    // cycles at one common 136-float stride): W2 and the z1 / a / g rows at
    // 144 floats (≡ 16 mod 32: the rows 4 s + g, g = 0, 1 of a 32-lane half, read
    // at 16 consecutive columns, fill all 32 banks), gz2 at 130 (≡ 2: its
    // A-operand reads, 16 rows r at column 4 s + g, fill all 32 banks)
    constexpr int WS = BWS + 8, GS = BWS - 6;
    __shared__ float w2s[BH * WS];     // W2 [c][kk], row stride WS
    __shared__ float at[BT * WS];      // a rows of the tile
    __shared__ float z1s[BT * WS];     // z1 of the current slot
    __shared__ float gz2s[BT * GS];    // gz2 of the current slot
    __shared__ float gms[BT * WS];     // g / deg of the tile
    __shared__ int srcs[BT];
    const int tid = threadIdx.x, wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
    const int r = lane & 15, g = lane >> 4;
    const int64_t nmax = p.n - 1;
    const int k = p.k;
    for (int i = tid; i < BH * BH / 4; i += 256)
        *(float4 *)&w2s[(i >> 5) * WS + 4 * (i & 31)] = ((const float4 *)p.w2)[i];
    // persistent accumulators: dW2 tiles (c tile 2 wave + ci, kk tile kj), db2
    f32x4 dw[2][8];
#pragma unroll
    for (int ci = 0; ci < 2; ++ci)
#pragma unroll
        for (int kj = 0; kj < 8; ++kj) dw[ci][kj] = (f32x4){0.0f, 0.0f, 0.0f, 0.0f};
    float db[2] = {0.0f, 0.0f};
    for (int tile = blockIdx.x; tile < p.ntiles; tile += gridDim.x) {
        const int64_t row0 = (int64_t)tile * BT;
        __syncthreads();  // the previous tile's LDS readers are done
        for (int i = tid; i < BT * BH / 4; i += 256) {
            const int rr = i >> 5, c4 = i & 31;
            const int64_t row = min(row0 + rr, nmax);
            const bool live = row0 + rr < p.n;
            const int dgv = p.deg ? p.deg[row] : k;
            const float inv_deg = live ? 1.0f / (float)max(dgv, 1) : 0.0f;
            const float4 av = ((const float4 *)(p.a + row * BH))[c4];
            const float4 gv = ((const float4 *)(p.gmean + row * BH))[c4];
            *(float4 *)&at[rr * WS + 4 * c4] = av;
            *(float4 *)&gms[rr * WS + 4 * c4] =
                make_float4(gv.x * inv_deg, gv.y * inv_deg, gv.z * inv_deg, gv.w * inv_deg);
        }
        // dL/da accumulators: rows 4 g + t, columns 16 (2 wave + ci) + r
        f32x4 gacc[2] = {(f32x4){0.0f, 0.0f, 0.0f, 0.0f}, (f32x4){0.0f, 0.0f, 0.0f, 0.0f}};
        int dgr[4];
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            const int64_t row = min(row0 + 4 * g + t, nmax);
            dgr[t] = p.deg ? p.deg[row] : k;
        }
        for (int e = 0; e < k; ++e) {
            if (tid < BT) {
                const int64_t row = min(row0 + tid, nmax);
                const int s = p.nbr[row * k + e];
                srcs[tid] = (s < 0 || s > nmax) ? 0 : s;  // padded / malformed entries: masked below
            }
            __syncthreads();
            // z1 = a + b_src
            for (int i = tid; i < BT * BH / 4; i += 256) {
                const int rr = i >> 5, c4 = i & 31;
                const float4 bv = ((const float4 *)(p.b + (int64_t)srcs[rr] * BH))[c4];
                const float4 av = *(const float4 *)&at[rr * WS + 4 * c4];
                *(float4 *)&z1s[rr * WS + 4 * c4] = make_float4(av.x + bv.x, av.y + bv.y, av.z + bv.z, av.w + bv.w);
            }
            __syncthreads();
            // z2 = W2 relu(z1) + b2 and gz2 = g / deg [z2 > 0]: wave owns columns
            // c of tiles 2 wave, 2 wave + 1 (A = relu(z1)[row][kk], B = W2[c][kk])
            float gz2v[2][4];
            if (MASK) {
                // columns 32 wave + 16 ci + r: bit 16 ci + r of word `wave`
                uint32_t mw[4];
#pragma unroll
                for (int t = 0; t < 4; ++t)
                    mw[t] = p.mask[(min(row0 + 4 * g + t, nmax) * k + e) * 4 + wave];
#pragma unroll
                for (int ci = 0; ci < 2; ++ci) {
                    const int c = 16 * (2 * wave + ci) + r;
#pragma unroll
                    for (int t = 0; t < 4; ++t) {
                        const int rr = 4 * g + t;
                        const bool on = e < dgr[t] && ((mw[t] >> (16 * ci + r)) & 1u);
                        const float v = on ? gms[rr * WS + c] : 0.0f;
                        gz2v[ci][t] = v;
                        gz2s[rr * GS + c] = v;
                    }
                }
            }
#pragma unroll
            for (int ci = 0; ci < 2 && !MASK; ++ci) {
                const int c = 16 * (2 * wave + ci) + r;
                f32x4 acc = (f32x4){0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll 8
                for (int s = 0; s < BH / 4; ++s) {
                    const float av = fmaxf(z1s[r * WS + 4 * s + g], 0.0f);
                    const float bv = w2s[c * WS + 4 * s + g];
                    acc = mfma16(av, bv, acc);
                }
                const float bb = p.b2[c];
#pragma unroll
                for (int t = 0; t < 4; ++t) {
                    const int rr = 4 * g + t;
                    const bool on = e < dgr[t] && acc[t] + bb > 0.0f;
                    const float v = on ? gms[rr * WS + c] : 0.0f;
                    gz2v[ci][t] = v;
                    gz2s[rr * GS + c] = v;
                }
            }
#pragma unroll
            for (int ci = 0; ci < 2; ++ci)
                db[ci] += gz2v[ci][0] + gz2v[ci][1] + gz2v[ci][2] + gz2v[ci][3];
            __syncthreads();
            // gm1 = W2^T gz2 (A = gz2[row][c], B = W2[c][kk]); wave owns kk tiles
            // 2 wave, 2 wave + 1; gz1 = gm1 [z1 > 0]
#pragma unroll
            for (int ci = 0; ci < 2; ++ci) {
                const int kk = 16 * (2 * wave + ci) + r;
                f32x4 acc = (f32x4){0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll 8
                for (int s = 0; s < BH / 4; ++s) {
                    const float av = gz2s[r * GS + 4 * s + g];
                    const float bv = w2s[(4 * s + g) * WS + kk];
                    acc = mfma16(av, bv, acc);
                }
#pragma unroll
                for (int t = 0; t < 4; ++t) {
                    const int rr = 4 * g + t;
                    const float v = z1s[rr * WS + kk] > 0.0f ? acc[t] : 0.0f;
                    gacc[ci][t] += v;
                    if (row0 + rr < p.n) {
                        const int64_t q = (row0 + rr) * k + e;
                        p.gz1[(p.pos ? (int64_t)p.pos[q] : q) * BH + kk] = v;
                    }
                }
            }
            // dW2[c][kk] += sum_rows gz2[row][c] relu(z1)[row][kk]  (K = the 16 rows)
#pragma unroll
            for (int ci = 0; ci < 2; ++ci) {
                const int c = 16 * (2 * wave + ci) + r;
#pragma unroll
                for (int kj = 0; kj < 8; ++kj) {
                    const int kk = 16 * kj + r;
#pragma unroll
                    for (int s = 0; s < 4; ++s) {
                        // A[c][row] = gz2[row][c] (lane: c = r, row = 4 s + g); B[row][kk]
                        const float av = gz2s[(4 * s + g) * GS + 16 * (2 * wave + ci) + r];
                        const float bv = fmaxf(z1s[(4 * s + g) * WS + kk], 0.0f);
                        dw[ci][kj] = mfma16(av, bv, dw[ci][kj]);
                    }
                }
                (void)c;
            }
            __syncthreads();  // z1s / gz2s are rewritten by the next slot
        }
#pragma unroll
        for (int ci = 0; ci < 2; ++ci) {
            const int kk = 16 * (2 * wave + ci) + r;
#pragma unroll
            for (int t = 0; t < 4; ++t) {
                const int64_t row = row0 + 4 * g + t;
                if (row < p.n) p.ga[row * BH + kk] = gacc[ci][t];
            }
        }
    }
    // partials of this workgroup: dW2 tile (c rows 4 g + t of tile 2 wave + ci, kk col)
    float *pw = p.pw2 + (int64_t)blockIdx.x * BH * BH;
#pragma unroll
    for (int ci = 0; ci < 2; ++ci)
#pragma unroll
        for (int kj = 0; kj < 8; ++kj)
#pragma unroll
            for (int t = 0; t < 4; ++t)
                pw[(16 * (2 * wave + ci) + 4 * g + t) * BH + 16 * kj + r] = dw[ci][kj][t];
    // db2: lanes g = 0..3 of a column hold disjoint rows: add them in g order
#pragma unroll
    for (int ci = 0; ci < 2; ++ci) {
        float v = db[ci];
        const float v1 = __shfl(v, r + 16, 64), v2 = __shfl(v, r + 32, 64), v3 = __shfl(v, r + 48, 64);
        if (g == 0) p.pb2[(int64_t)blockIdx.x * BH + 16 * (2 * wave + ci) + r] = ((v + v1) + v2) + v3;
    }
}

// ---------------------------------------------------------------------------
// The same backward with the three GEMMs in the fp16x3 split (every fp32
// operand scaled by a power of two and split into fp16 hi + lo; products
// hi.hi + hi.lo + lo.hi on v_mfma_f32_16x16x32_f16, fp32 accumulation: the
// forward's MMPDE_EDGE_GEMM_F16X3 arithmetic).  Scales are uniform per launch:
// relu(z1) by split_scale(max|a| + max|b|), gz2 by split_scale(max|g|) (one
// pre-pass reduction), W2 per output column (packed images, as the forward).
// One 512-thread workgroup per CU, persistent over 32-target tiles; a slot is
// one neighbour e of the tile's 32 targets (32 edges = the K of the dW2 GEMM):
//   P1  z1 = a + b_src (b rows prefetched one slot ahead into registers),
//       relu(z1) split -> LDS row-major (A of z2) and column-major (B of dW2),
//       the z1 > 0 bits (double-buffered by slot parity: two barriers a slot)
//   P2  z2 = relu(z1) W2^T (wave w: output columns 16w..), gz2 = g/deg
//       [z2 + b2 > 0][e < deg] split -> LDS row-major (A of gm1) and
//       column-major (A of dW2); db2 in fp32
//   P3  gm1 = gz2 W2 (wave w: columns 16w..), gz1 = gm1 [z1 > 0] -> grad_edge
//       and the dL/da sums; dW2 += gz2^T relu(z1) (wave w: a 2 x 4 block of tiles)
// Deterministic: fixed orders, per-workgroup partials, no atomics in the sums.
// ---------------------------------------------------------------------------
constexpr int FT = 32;          // targets per tile
constexpr int FAW = BH + 4;     // fp32 row stride of the a / g tiles
constexpr int FAS = BH + 16;    // half row stride, row-major images (288 B = 72 dwords: the
                                // A-operand reads' 16 rows x 4 chunks land on 64 distinct
                                // chunk banks, 8 ≡ 72 mod 64; 272 B left one 2-way pair per
                                // lane group; the ds_write_b16 stores are then 2-way, free)
constexpr int FCS = FT;         // half row stride, column-major images [128][32 edges]
constexpr int FKMAX = 64;       // neighbour slots per target this kernel takes

// The column-major images zb [kk][edge] and gt [c][edge] (rows of FCS = 32
// halves = four 16-B chunks) store chunk q of row x at chunk q ^ csw(x).  With
// a plain 64-B row stride the dW2 operand reads (lanes r = 16 rows, g = chunk)
// hit 4 rows per bank group -- 4-way conflicts on every ds_read_b128 -- the P1
// zb writes (64 consecutive rows, one chunk) 4-way and the P2 gt writes 8-way
// (SQ_LDS_BANK_CONFLICT was 57 % of the kernel's LDS cycles).  csw = bits 1-2
// of the row makes every ds_read_b128 lane group and every 8-lane ds_write_b128
// group conflict-free and the 8-B gt writes 2-way (the least a 16-dword row
// stride allows).  Only the layout changes: the same values, the same sums.
__device__ __forceinline__ int csw(int row) { return (row >> 1) & 3; }
// gt [c][edge] (the gz2 image) takes bits 1 and 3 of its row instead: the same
// conflict-free dW2 reads and 2-way writes, and with MASK it is also gm1's A
// operand, read transposed (ds_read_b64_tr_b16: a 32-lane half reads rows
// c0 .. c0 + 3 and c0 + 8 .. c0 + 11, which bit 3 sends to the other two
// chunks of each row) without conflicts.
__device__ __forceinline__ int gsw(int row) { return ((row >> 1) & 1) | ((row >> 2) & 2); }

typedef __fp16 fp16x4_t __attribute__((__vector_size__(4 * sizeof(__fp16))));
// ds_read_b64_tr_b16 (MI355X: per 16-lane group, lane 4q + p addresses row q's
// columns 4p .. 4p + 3 of a 4 x 16 block; lane i receives column i, row q in
// element q).  EXEC must be all ones.
__device__ __forceinline__ fp16x4_t lds_read_tr16(const _Float16 *p) {
    return __builtin_amdgcn_ds_read_tr16_b64_v4f16((__attribute__((address_space(3))) fp16x4_t *)p);
}

struct EdgeBwdF16Args {
    const float *a, *b;
    const int32_t *nbr, *deg;
    int64_t n;
    int k, ntiles;
    const char *img1, *img2;  // B images: W2 (z2 = relu(z1) W2^T), W2^T (gm1 = gz2 W2)
    const float *b2, *gmean;
    const unsigned *mx;       // max|a|, max|b|, max|g| (float bits)
    float *ga, *gz1, *pw2, *pb2;
    const int32_t *pos;       // nullable: the gz1 row of slot q (source-major order)
    const uint32_t *mask;     // MASK: the forward's z2 > 0 bits, [n * k][4] (mmpde_gnn_edge_mean_ex)
};

__device__ __forceinline__ void split1(float x, _Float16 &h, _Float16 &l) {
    h = (_Float16)x;
    l = (_Float16)(x - (float)h);
}

// Static LDS of edge_bwd_f16_kernel (the arrays below): ~141 KiB, which only
// gfx950's 160 KiB per CU holds, one workgroup per CU -- hence the launch
// bound of one 512-thread workgroup and the size check.
constexpr size_t kEdgeBwdF16Lds = sizeof(float) * 2 * FT * FAW + sizeof(_Float16) * 2 * 2 * FT * FAS +
                                  sizeof(_Float16) * 2 * 2 * BH * FCS + sizeof(_Float16) * 2 * FT * FAS +
                                  sizeof(_Float16) * 2 * BH * FCS + 2 * BH * (FT / 8) + 2 * sizeof(int) * FT * FKMAX +
                                  sizeof(int) * FT;
static_assert(kEdgeBwdF16Lds <= 160 * 1024, "edge_bwd_f16_kernel: LDS beyond gfx950's 160 KiB per CU");

// P1 of slot e + 1 in front of P3(e)'s MFMAs in one straight-line block (1),
// or after P3(e)'s epilogue (0, the round-3 order): 807-817 vs 784-795 us per
// sorted backward at cy B=16 (tools/ubench/bwd_ab.cpp, profiles/
// r04_bwd_ab.log) -- the compiler waits on every LDS operand read in the MFMA
// stream either way, so the placement buys nothing; 0.
#ifndef MMPDE_BWD_P1_FIRST
#define MMPDE_BWD_P1_FIRST 0
#endif
constexpr bool kBwdP1First = MMPDE_BWD_P1_FIRST != 0;
// SIMD-partner stagger of the MASK kernel (below): 0 off; waves 4-7 run
// 1: P1 P2 | P3, 2: P1 | P3 P2, 3: P2 | P3 P1 of each phase (0-3: P3 P1 P2).
// Measured (tools/ubench bwd_ab_st*, cy B=16, k = 35, profiles/
// r05_bwd_stagger_ab.log): 561-563 us off against 667-668 / 630 / 676-679:
// the second loop body pushes the kernel from 254 VGPRs to 44-53 spilled, which
// costs more than the overlap gains.  Off.
#ifndef MMPDE_BWD_STAGGER
#define MMPDE_BWD_STAGGER 0
#endif
constexpr int kBwdStagger = MMPDE_BWD_STAGGER;

// MASK: message_net_2's ReLU pattern comes from the forward's bits instead of
// recomputing z2 (P2 without its MFMAs; no row-major relu(z1) image).
// MASK kernel: s_setprio 1 around P3's MFMA cluster (the guide's T5; the wave
// in its MFMA phase wins issue over its SIMD partner's P1 / P2 VALU), same-box
// A/B (profiles/r06_bwd_lds_ab.log): 443-446 against 457-459 us with the same
// hash; the unmasked kernel was 1-3 % slower with it, so MASK only.  Waves 4-7
// at priority 1 for the whole launch (the guide's static form) measured no
// change and is not kept.  0 turns it off.
#ifndef MMPDE_BWD_PRIO
#define MMPDE_BWD_PRIO 1
#endif

// O32: every byte offset into b (n x 512 B) and gz1 (n k x 512 B) fits in 32
// bits, so the per-slot gathers and the per-edge stores take one 32-bit
// multiply-add over a scalar base instead of 64-bit address arithmetic.
template <bool MASK, bool O32>
__global__ __launch_bounds__(512, 1) void edge_bwd_f16_kernel(EdgeBwdF16Args p) {
    __shared__ float at[FT * FAW];             // a rows of the tile
    __shared__ float gms[FT * FAW];            // g / deg rows (0 for rows past n)
    // relu(z1) images double-buffered by slot parity (no barrier between a
    // slot's last readers and the next slot's writers)
    // MASK: no z2 GEMM, so no row-major relu(z1) image; gz2 double-buffered by
    // slot parity instead (one barrier per slot)
    constexpr int NZA = MASK ? 1 : 2, NGB = MASK ? 2 : 1;
    __shared__ _Float16 za[NZA][2][MASK ? 8 : FT * FAS];  // [slot & 1] relu(z1) sz: hi, lo, [edge][kk]
    __shared__ _Float16 zb[2][2][BH * FCS];    // the same, [kk][edge]
    // gz2 sg, [edge][c]: without MASK only (MASK reads gm1's A operand from gt
    // transposed: one image, no row-major stores)
    __shared__ _Float16 grb[MASK ? 1 : NGB][2][MASK ? 8 : FT * FAS];
    __shared__ _Float16 gtb[NGB][2][BH * FCS];  // the same, [c][edge]
    __shared__ __attribute__((aligned(16))) uint8_t zm[2][BH * (FT / 8)];  // z1 > 0, [kk][edge / 8] bits
    __shared__ int nb[FT * FKMAX];             // the tile's neighbour rows (clamped)
    __shared__ int gzr[FT * FKMAX];            // the gz1 rows of the tile's slots
    __shared__ int dg[FT];                     // degrees (0 past n)
    // MASK: the tile's z2 > 0 words, [row][slot][4] at a row stride of 4 FKMAX + 1
    // words (the 4 rows a ds_read_b32 takes sit on different banks), staged with
    // the neighbour table: P2 reads them from LDS.  (Round 5 prefetched each
    // slot's words into registers one slot ahead; the loop-carried registers made
    // the compiler copy them at the loop's back edge, waiting there -- after the
    // barrier -- for the loads just issued, every slot.)
    constexpr int MLS = 4 * FKMAX + 1;
    __shared__ uint32_t mlds[MASK ? FT * MLS : 1];
    const int tid = threadIdx.x, wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
    const int r = lane & 15, g = lane >> 4;
    const int64_t nmax = p.n - 1;
    const int k = p.k;
    const float sz = split_scale(__uint_as_float(p.mx[0]) + __uint_as_float(p.mx[1]));
    const float sg = split_scale(__uint_as_float(p.mx[2]));
    // B operands of this wave's column tile, for the whole launch
    half8 w1h[4], w1l[4], w2h[4], w2l[4];
#pragma unroll
    for (int s = 0; s < 4; ++s) {
        w1h[s] = bfrag(p.img1, 4, wave, s, 0, lane);
        w1l[s] = bfrag(p.img1, 4, wave, s, 1, lane);
        w2h[s] = bfrag(p.img2, 4, wave, s, 0, lane);
        w2l[s] = bfrag(p.img2, 4, wave, s, 1, lane);
    }
    const int col = 16 * wave + r;  // output column of z2 (c) and of gm1 (kk)
    const float un1 = pow2_inv(sz) * pow2_inv(((const float *)(p.img1 + 65536))[col]);
    const float un2 = pow2_inv(sg) * pow2_inv(((const float *)(p.img2 + 65536))[col]);
    const float bias = p.b2[col];
    f32x4 dw[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) dw[j] = (f32x4){0.0f, 0.0f, 0.0f, 0.0f};
    float db = 0.0f;
    // P1 role: column kk1 of edges 8 eg .. 8 eg + 7
    const int kk1 = tid & (BH - 1), eg = tid >> 7;
    // b[src][kk1] and the gz1 element (row, col): 32-bit byte offsets with O32
    auto b_at = [&](int src) -> float {
        if (O32) return *(const float *)((const char *)p.b + ((uint32_t)src * (BH * 4u) + (uint32_t)kk1 * 4u));
        return p.b[(int64_t)src * BH + kk1];
    };
    auto gz1_store = [&](int grow, float v) {
        if (O32) *(float *)((char *)p.gz1 + ((uint32_t)grow * (BH * 4u) + (uint32_t)col * 4u)) = v;
        else p.gz1[(int64_t)grow * BH + col] = v;
    };
    for (int tile = blockIdx.x; tile < p.ntiles; tile += gridDim.x) {
        const int64_t row0 = (int64_t)tile * FT;
        const bool tile_full = row0 + FT <= p.n;
        __syncthreads();  // the previous tile's readers are done
        for (int i = tid; i < FT * BH / 4; i += 512) {
            const int rr = i >> 5, c4 = i & 31;
            const int64_t row = min(row0 + rr, nmax);
            const bool live = row0 + rr < p.n;
            const int d = p.deg ? p.deg[row] : k;
            const float inv = live ? 1.0f / (float)max(d, 1) : 0.0f;
            const float4 av = ((const float4 *)(p.a + row * BH))[c4];
            const float4 gv = ((const float4 *)(p.gmean + row * BH))[c4];
            *(float4 *)&at[rr * FAW + 4 * c4] = av;
            *(float4 *)&gms[rr * FAW + 4 * c4] = make_float4(gv.x * inv, gv.y * inv, gv.z * inv, gv.w * inv);
        }
        for (int i = tid; i < FT * k; i += 512) {
            const int rr = i / k, e = i - rr * k;
            const int64_t q = min(row0 + rr, nmax) * k + e;
            const int s = p.nbr[q];
            nb[rr * FKMAX + e] = (s < 0 || s > nmax) ? 0 : s;  // padded / malformed: masked by e < deg
            gzr[rr * FKMAX + e] = p.pos ? p.pos[q] : (int)q;
        }
        if (tid < FT) dg[tid] = row0 + tid < p.n ? (p.deg ? p.deg[row0 + tid] : k) : 0;
        if (MASK) {  // rows row0 .. row0 + 31 of the mask are contiguous: coalesced
            for (int i = tid; i < FT * 4 * k; i += 512) {
                const int rr = i / (4 * k), w = i - rr * 4 * k;
                mlds[rr * MLS + w] = p.mask[(min(row0 + rr, nmax) * k) * 4 + w];
            }
        }
        __syncthreads();
        float bv[8];
#pragma unroll
        for (int t = 0; t < 8; ++t) bv[t] = b_at(nb[(8 * eg + t) * FKMAX]);
        // MASK (registers to spare without the z2 operands): the tile's a values
        // of P1, and g / deg and the degrees of P2, in registers for the tile
        float atv[MASK ? 8 : 1], gmv[MASK ? 8 : 1];
        int dgv[MASK ? 8 : 1];
        if (MASK) {
#pragma unroll
            for (int t = 0; t < 8; ++t) {
                atv[t] = at[(8 * eg + t) * FAW + kk1];
                const int rr = 16 * (t >> 2) + 4 * g + (t & 3);
                gmv[t] = gms[rr * FAW + col];
                dgv[t] = dg[rr];
            }
        }
        f32x4 gacc[2] = {(f32x4){0.0f, 0.0f, 0.0f, 0.0f}, (f32x4){0.0f, 0.0f, 0.0f, 0.0f}};
        // ---- P1 of slot e into buffer e & 1; issues the b loads of slot e + 1
        // (clamped at the last slot: a harmless reload)
        auto p1 = [&](int e) {
            const int sb = e & 1;
            half8 hi, lo;
            unsigned bits = 0;
#pragma unroll
            for (int t = 0; t < 8; ++t) {
                const int ed = 8 * eg + t;
                const float z = (MASK ? atv[MASK ? t : 0] : at[ed * FAW + kk1]) + bv[t];
                bits |= (z > 0.0f ? 1u : 0u) << t;
                _Float16 h, l;
                split1(fmaxf(z, 0.0f) * sz, h, l);
                hi[t] = h;
                lo[t] = l;
                if (!MASK) {
                    za[MASK ? 0 : sb][0][ed * FAS + kk1] = h;
                    za[MASK ? 0 : sb][1][ed * FAS + kk1] = l;
                }
            }
            *(half8 *)&zb[sb][0][kk1 * FCS + 8 * (eg ^ csw(kk1))] = hi;
            *(half8 *)&zb[sb][1][kk1 * FCS + 8 * (eg ^ csw(kk1))] = lo;
            zm[sb][kk1 * 4 + eg] = (uint8_t)bits;
            const int en = min(e + 1, k - 1);
#pragma unroll
            for (int t = 0; t < 8; ++t) bv[t] = b_at(nb[(8 * eg + t) * FKMAX + en]);
        };
        // ---- P2: z2 and gz2 (column c = col) of slot e
        auto p2 = [&](int e) {
            const int sb = e & 1;
            _Float16(*gr)[MASK ? 8 : FT * FAS] = grb[0];
            _Float16(*gt)[BH * FCS] = gtb[MASK ? sb : 0];
            f32x4 acc[2] = {(f32x4){0.0f, 0.0f, 0.0f, 0.0f}, (f32x4){0.0f, 0.0f, 0.0f, 0.0f}};
            if (!MASK) {
#pragma unroll
                for (int s = 0; s < 4; ++s) {
#pragma unroll
                    for (int rb = 0; rb < 2; ++rb) {
                        const half8 ah = *(const half8 *)&za[MASK ? 0 : sb][0][(16 * rb + r) * FAS + 32 * s + 8 * g];
                        const half8 al = *(const half8 *)&za[MASK ? 0 : sb][1][(16 * rb + r) * FAS + 32 * s + 8 * g];
                        acc[rb] = mfma_f16(ah, w1h[s], acc[rb]);
                        acc[rb] = mfma_f16(ah, w1l[s], acc[rb]);
                        acc[rb] = mfma_f16(al, w1h[s], acc[rb]);
                    }
                }
            }
            uint32_t mk[8];
            if (MASK) {
                // this slot's words (column tile = wave, bit r) of the lane's 8 rows
#pragma unroll
                for (int i = 0; i < 8; ++i)
                    mk[i] = mlds[(16 * (i >> 2) + 4 * g + (i & 3)) * MLS + 4 * e + (wave >> 1)];
            }
#pragma unroll
            for (int rb = 0; rb < 2; ++rb) {
                _Float16 hv[4], lv[4];
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const int rr = 16 * rb + 4 * g + q;
                    const bool z2pos = MASK ? ((mk[4 * rb + q] >> (16 * (wave & 1) + r)) & 1u) != 0
                                             : acc[rb][q] * un1 + bias > 0.0f;
                    const bool on = e < (MASK ? dgv[MASK ? 4 * rb + q : 0] : dg[rr]) && z2pos;
                    const float v = on ? (MASK ? gmv[MASK ? 4 * rb + q : 0] : gms[rr * FAW + col]) : 0.0f;
                    db += v;
                    split1(v * sg, hv[q], lv[q]);
                    if (!MASK) {
                        gr[0][rr * FAS + col] = hv[q];
                        gr[1][rr * FAS + col] = lv[q];
                    }
                }
                typedef _Float16 half4 __attribute__((ext_vector_type(4)));
                // edges 16 rb + 4 g .. + 3: chunk 2 rb + (g >> 1), half 4 (g & 1)
                const int go = col * FCS + 8 * ((2 * rb + (g >> 1)) ^ gsw(col)) + 4 * (g & 1);
                *(half4 *)&gt[0][go] = (half4){hv[0], hv[1], hv[2], hv[3]};
                *(half4 *)&gt[1][go] = (half4){lv[0], lv[1], lv[2], lv[3]};
            }
        };
        // ---- P3 of slot e: gm1 -> gz1 (column kk = col); this wave's dW2 tiles
        // With `next`, P1 of slot e + 1 (the other buffer) goes in front of
        // P3's MFMAs in the same straight-line block (its b prefetch is
        // clamped, not branched), so that the scheduler can issue its LDS
        // writes and VALU work in the MFMAs' shadow.
        auto p3 = [&](int e, bool next) {
            const int sb = e & 1;
            const _Float16(*gr)[MASK ? 8 : FT * FAS] = grb[0];
            const _Float16(*gt)[BH * FCS] = gtb[MASK ? sb : 0];
            if (next) p1(e + 1);
            f32x4 acc[2] = {(f32x4){0.0f, 0.0f, 0.0f, 0.0f}, (f32x4){0.0f, 0.0f, 0.0f, 0.0f}};
            // MASK: the A operand (gz2 [edge 16 rb + r][c = 32 s + 8 g + j]) by
            // two transposed reads of gt per (s, rb): lane 4q + p (q, p < 4) of
            // group g addresses row c = 32 s + 8 g + 4 h + q, edges 16 rb + 4 p
            // .. + 3 (chunk 2 rb + (p >> 1) ^ gsw(c), half 4 (p & 1)); gsw(c)
            // = bit 1 of q | bit 0 of g << 1 for every s, h
            const int tq = (lane & 15) >> 2, tp = lane & 3;
            const int tsw = ((tq >> 1) & 1) | ((g & 1) << 1);
            auto a_tr = [&](int plane, int s, int rb) {
                const _Float16 *b0 = &gt[plane][(32 * s + 8 * g + tq) * FCS + 8 * ((2 * rb + (tp >> 1)) ^ tsw) +
                                                 4 * (tp & 1)];
                const fp16x4_t lo4 = lds_read_tr16(b0), hi4 = lds_read_tr16(b0 + 4 * FCS);
                return __builtin_bit_cast(half8, __builtin_shufflevector(lo4, hi4, 0, 1, 2, 3, 4, 5, 6, 7));
            };
            if (MASK && MMPDE_BWD_PRIO) __builtin_amdgcn_s_setprio(1);
#pragma unroll
            for (int s = 0; s < 4; ++s) {
#pragma unroll
                for (int rb = 0; rb < 2; ++rb) {
                    const half8 ah = MASK ? a_tr(0, s, rb)
                                          : *(const half8 *)&gr[0][(16 * rb + r) * FAS + 32 * s + 8 * g];
                    const half8 al = MASK ? a_tr(1, s, rb)
                                          : *(const half8 *)&gr[1][(16 * rb + r) * FAS + 32 * s + 8 * g];
                    acc[rb] = mfma_f16(ah, w2h[s], acc[rb]);
                    acc[rb] = mfma_f16(ah, w2l[s], acc[rb]);
                    acc[rb] = mfma_f16(al, w2h[s], acc[rb]);
                }
            }
            // dW2 tiles of this wave: c tiles 2 (wave & 3) + i (i < 2) x kk tiles
            // 4 (wave >> 2) + jj (jj < 4): 4 A and 8 B fragment reads per slot
            // (a c-row of tiles would read 2 A and all 16 B fragments)
            const int cw = 32 * (wave & 3) + r;
            const int gq = 8 * (g ^ gsw(cw));  // gsw(cw + 16) = gsw(cw)
            const half8 gh0 = *(const half8 *)&gt[0][cw * FCS + gq];
            const half8 gl0 = *(const half8 *)&gt[1][cw * FCS + gq];
            const half8 gh1 = *(const half8 *)&gt[0][(cw + 16) * FCS + gq];
            const half8 gl1 = *(const half8 *)&gt[1][(cw + 16) * FCS + gq];
            // the epilogue's LDS values, read ahead of the dW2 MFMAs: the z1 > 0
            // bits of column col (bit rr of the 4 bytes), and (MASK, registers
            // to spare) the gz1 rows of the lane's 8 slots
            const uint32_t zbits = *(const uint32_t *)&zm[sb][col * 4];
            int gzrow[MASK ? 8 : 1];
            if (MASK) {
#pragma unroll
                for (int i = 0; i < 8; ++i) gzrow[i] = gzr[(16 * (i >> 2) + 4 * g + (i & 3)) * FKMAX + e];
            }
#pragma unroll
            for (int jj = 0; jj < 4; ++jj) {
                const int j = 4 * (wave >> 2) + jj;
                const int zq = (16 * j + r) * FCS + 8 * (g ^ csw(r));  // csw(16 j + r) = csw(r)
                const half8 bh = *(const half8 *)&zb[sb][0][zq];
                const half8 bl = *(const half8 *)&zb[sb][1][zq];
                dw[2 * jj] = mfma_f16(gh0, bh, dw[2 * jj]);
                dw[2 * jj] = mfma_f16(gh0, bl, dw[2 * jj]);
                dw[2 * jj] = mfma_f16(gl0, bh, dw[2 * jj]);
                dw[2 * jj + 1] = mfma_f16(gh1, bh, dw[2 * jj + 1]);
                dw[2 * jj + 1] = mfma_f16(gh1, bl, dw[2 * jj + 1]);
                dw[2 * jj + 1] = mfma_f16(gl1, bh, dw[2 * jj + 1]);
            }
            if (MASK && MMPDE_BWD_PRIO) __builtin_amdgcn_s_setprio(0);
            float gv[8];
#pragma unroll
            for (int rb = 0; rb < 2; ++rb) {
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const int rr = 16 * rb + 4 * g + q;
                    const bool pos = (zbits >> rr) & 1u;
                    const float v = pos ? acc[rb][q] * un2 : 0.0f;
                    gacc[rb][q] += v;
                    gv[4 * rb + q] = v;
                }
            }
            // the rows past n (the last tile only) keep no gz1: one uniform test
            // per tile instead of a lane branch per store
            if (tile_full) {
#pragma unroll
                for (int i = 0; i < 8; ++i)
                    gz1_store(MASK ? gzrow[MASK ? i : 0] : gzr[(16 * (i >> 2) + 4 * g + (i & 3)) * FKMAX + e], gv[i]);
            } else {
#pragma unroll
                for (int i = 0; i < 8; ++i) {
                    const int rr = 16 * (i >> 2) + 4 * g + (i & 3);
                    if (row0 + rr < p.n)
                        gz1_store(MASK ? gzrow[MASK ? i : 0] : gzr[rr * FKMAX + e], gv[i]);
                }
            }
        };
        // Per slot: P2(e) | barrier | P3(e) + P1(e + 1) | barrier.  Buffers:
        // P1(e + 1) writes za / zb / zm[(e + 1) & 1], last read by P2(e - 1)
        // and P3(e - 1), both before the previous barrier; P2(e + 1) reads
        // them after the barrier that ends P1(e + 1), and rewrites gr / gt
        // only after every wave's P3(e) (the same barrier).
        if (MASK) {
            // P2 reads no LDS image (the bits and g / deg only): P1 + P2 of a slot
            // form one phase, and with every buffer a P3 reads held by slot
            // parity, one barrier per slot -- a wave done with P3(e) builds slot
            // e + 1 while the others still multiply.  P1 / P2(e + 1) write the
            // (e + 1) & 1 buffers, last read by P3(e - 1), which every wave left
            // before the previous barrier.
            // Stagger (MI355X_MICROARCH.md, "two waves that run the SAME program
            // with one barrier per block"): waves w and w + 4 share a SIMD;
            // waves 4-7 build slot e + 1 (VALU, LDS writes, loads) before their
            // P3(e) MFMAs, waves 0-3 after theirs, so one wave of each SIMD
            // pair multiplies while the other splits.  Both orders touch
            // disjoint buffers within the phase (P3(e) reads parity e & 1, P1 /
            // P2(e + 1) write parity (e + 1) & 1), and each wave's own sums run
            // in the same order: the outputs are bitwise unchanged.
            p1(0);
            p2(0);
            __syncthreads();
            if (kBwdStagger == 0 || wave < 4) {
                for (int e = 0; e + 1 < k; ++e) {
                    p3(e, false);
                    p1(e + 1);
                    p2(e + 1);
                    __syncthreads();
                }
            } else {
                for (int e = 0; e + 1 < k; ++e) {
                    if (kBwdStagger != 3) p1(e + 1);
                    if (kBwdStagger == 1 || kBwdStagger == 3) p2(e + 1);
                    __builtin_amdgcn_sched_barrier(0);  // P3's fragment reads stay after the split
                    p3(e, false);
                    if (kBwdStagger == 2) p2(e + 1);
                    if (kBwdStagger == 3) p1(e + 1);
                    __syncthreads();
                }
            }
            p3(k - 1, false);
        } else {
            p1(0);
            __syncthreads();
            for (int e = 0; e + 1 < k; ++e) {
                p2(e);
                __syncthreads();
                if (kBwdP1First) {
                    p3(e, true);
                } else {
                    p3(e, false);
                    p1(e + 1);
                }
                __syncthreads();
            }
            p2(k - 1);
            __syncthreads();
            p3(k - 1, false);
        }
#pragma unroll
        for (int rb = 0; rb < 2; ++rb) {
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int64_t row = row0 + 16 * rb + 4 * g + q;
                if (row < p.n) p.ga[row * BH + col] = gacc[rb][q];
            }
        }
    }
    // partials: dW2[c = 32 (wave & 3) + 16 (j & 1) + 4 g + q][kk = 16 (4 (wave >> 2) + (j >> 1)) + r], db2[col]
    const float und = pow2_inv(sg) * pow2_inv(sz);
    float *pw = p.pw2 + (int64_t)blockIdx.x * BH * BH;
#pragma unroll
    for (int j = 0; j < 8; ++j)
#pragma unroll
        for (int q = 0; q < 4; ++q)
            pw[(32 * (wave & 3) + 16 * (j & 1) + 4 * g + q) * BH + 16 * (4 * (wave >> 2) + (j >> 1)) + r] =
                dw[j][q] * und;
    const float v1 = __shfl(db, r + 16, 64), v2 = __shfl(db, r + 32, 64), v3 = __shfl(db, r + 48, 64);
    if (g == 0) p.pb2[(int64_t)blockIdx.x * BH + col] = ((db + v1) + v2) + v3;
}

// max|a|, max|b|, max|g| over [n, 128] rows: per-workgroup maxima into
// part[3][gridDim.x] (no atomics: 3 x 1024 adds on one line serialised at the
// memory-side atomic unit took 148 us), reduced by maxabs3_final_kernel.
__global__ __launch_bounds__(256) void maxabs3_kernel(const float *__restrict__ a, const float *__restrict__ b,
                                                      const float *__restrict__ gm, int64_t n4,
                                                      float *__restrict__ part) {
    float m[3] = {0.0f, 0.0f, 0.0f};
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (int64_t)gridDim.x * 256) {
        const float4 x = ((const float4 *)a)[i], y = ((const float4 *)b)[i], z = ((const float4 *)gm)[i];
        m[0] = fmaxf(m[0], fmaxf(fmaxf(fabsf(x.x), fabsf(x.y)), fmaxf(fabsf(x.z), fabsf(x.w))));
        m[1] = fmaxf(m[1], fmaxf(fmaxf(fabsf(y.x), fabsf(y.y)), fmaxf(fabsf(y.z), fabsf(y.w))));
        m[2] = fmaxf(m[2], fmaxf(fmaxf(fabsf(z.x), fabsf(z.y)), fmaxf(fabsf(z.z), fabsf(z.w))));
    }
    __shared__ float red[3][4];
#pragma unroll
    for (int q = 0; q < 3; ++q) {
        const float w = wave_max(m[q]);
        if ((threadIdx.x & 63) == 0) red[q][threadIdx.x >> 6] = w;
    }
    __syncthreads();
    if (threadIdx.x < 3)
        part[threadIdx.x * gridDim.x + blockIdx.x] =
            fmaxf(fmaxf(red[threadIdx.x][0], red[threadIdx.x][1]), fmaxf(red[threadIdx.x][2], red[threadIdx.x][3]));
}

// mx[q] = max over the G per-workgroup maxima of quantity q (float bits).
__global__ __launch_bounds__(256) void maxabs3_final_kernel(const float *__restrict__ part, int G,
                                                            unsigned *__restrict__ mx) {
    __shared__ float red[4];
    const int q = blockIdx.x;
    float m = 0.0f;
    for (int i = threadIdx.x; i < G; i += 256) m = fmaxf(m, part[q * G + i]);
    m = wave_max(m);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
    __syncthreads();
    if (threadIdx.x == 0) mx[q] = __float_as_uint(fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3])));
}

__global__ __launch_bounds__(256) void transpose128_kernel(const float *__restrict__ w, float *__restrict__ wt) {
    const int i = blockIdx.x * 256 + threadIdx.x;  // 128 x 128
    wt[(i & 127) * BH + (i >> 7)] = w[i];
}

// out[j] = sum_{p in [off[j], off[j+1])} rows[edge[p]] (GATHER) or rows[p] (the
// rows of source j stored contiguously by mmpde_gnn_edge_backward_sorted).  One
// wave per source: lanes 0-31 take the even positions of the list and 32-63 the
// odd ones, four columns per lane.  Rows go in batches of 32 (16 loads in
// flight per lane, issued unconditionally: positions past the list re-read its
// last row and are masked with an opaque all-ones / zero word, since a load
// under a condition is waited for at once; non-temporal loads, the rows are
// read once); each half adds its rows in list
// order, then the odd half's sum is added to the even half's.  Both forms add
// the same values in the same order: bitwise-equal sums.
template <bool GATHER>
__device__ __forceinline__ void source_sum(const float *__restrict__ rows, const int64_t *__restrict__ off,
                                           const int64_t *__restrict__ edge, int64_t n,
                                           float *__restrict__ out) {
    const int64_t j = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    const int par = lane >> 5, c4 = lane & 31;
    if (j >= n) return;
    float4 acc = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    const int64_t q0 = off[j], qe = off[j + 1];
    for (int64_t qb = q0; qb < qe; qb += 32) {
        int64_t src[16];
#pragma unroll
        for (int t = 0; t < 16; ++t) {
            const int64_t q = min(qb + 2 * t + par, qe - 1);
            src[t] = GATHER ? edge[q] : q;
        }
        float4 v[16];
#pragma unroll
        for (int t = 0; t < 16; ++t) {
            // non-temporal: each row is read once (115 vs 162 us at cy B=16,
            // profiles/r05_loads_ab.log)
            typedef float nt4 __attribute__((ext_vector_type(4)));
            const nt4 q = __builtin_nontemporal_load((const nt4 *)(rows + src[t] * BH) + c4);
            v[t] = make_float4(q.x, q.y, q.z, q.w);
        }
#pragma unroll
        for (int t = 0; t < 16; ++t) {
            int m = qb + 2 * t + par < qe ? -1 : 0;
            asm volatile("" : "+v"(m));
            acc.x += __int_as_float(__float_as_int(v[t].x) & m);
            acc.y += __int_as_float(__float_as_int(v[t].y) & m);
            acc.z += __int_as_float(__float_as_int(v[t].z) & m);
            acc.w += __int_as_float(__float_as_int(v[t].w) & m);
        }
    }
    acc.x += __shfl_down(acc.x, 32, 64);
    acc.y += __shfl_down(acc.y, 32, 64);
    acc.z += __shfl_down(acc.z, 32, 64);
    acc.w += __shfl_down(acc.w, 32, 64);
    if (par == 0) ((float4 *)(out + j * BH))[c4] = acc;
}

__global__ __launch_bounds__(256) void edge_source_sum_kernel(const float *__restrict__ rows,
                                                              const int64_t *__restrict__ off,
                                                              const int64_t *__restrict__ edge, int64_t n,
                                                              float *__restrict__ out) {
    source_sum<true>(rows, off, edge, n, out);
}

__global__ __launch_bounds__(256) void edge_source_sum_sorted_kernel(const float *__restrict__ rows,
                                                                     const int64_t *__restrict__ off, int64_t n,
                                                                     float *__restrict__ out) {
    source_sum<false>(rows, off, nullptr, n, out);
}

// out[j][c] = sum_{p in [off[j], off[j+1])} rows[edge[p]][c] for any row width:
// one thread per (j, c), in list order.
__global__ __launch_bounds__(256) void segment_sum_kernel(const float *__restrict__ rows, int64_t width,
                                                          const int64_t *__restrict__ off,
                                                          const int64_t *__restrict__ edge, int64_t n,
                                                          float *__restrict__ out) {
    const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (t >= n * width) return;
    const int64_t j = t / width, c = t - j * width;
    float acc = 0.0f;
    for (int64_t q = off[j]; q < off[j + 1]; ++q) acc += rows[edge[q] * width + c];
    out[t] = acc;
}

// out[i] = sum_{g < G} part[g * len + i] in a fixed order: thread (group gq =
// tid / 32, i = 32 block + tid % 32) adds the partials of its eighth of g in
// order (eight loads in flight, issued unconditionally: clamped and masked),
// then the eight group sums are added in group order through LDS.
__global__ __launch_bounds__(256) void partial_sum_kernel(const float *__restrict__ part, int G, int64_t len,
                                                          float *__restrict__ out) {
    __shared__ float red[8][32];
    const int gq = threadIdx.x >> 5, l = threadIdx.x & 31;
    const int64_t i = (int64_t)blockIdx.x * 32 + l;
    const int64_t ic = min(i, len - 1);
    const int per = (G + 7) / 8;
    const int q0 = min(gq * per, G), q1 = min(q0 + per, G);
    float s = 0.0f;
    for (int q = q0; q < q1; q += 8) {
        float v[8];
#pragma unroll
        for (int t = 0; t < 8; ++t) v[t] = part[(int64_t)min(q + t, q1 - 1) * len + ic];
#pragma unroll
        for (int t = 0; t < 8; ++t) {
            int m = q + t < q1 ? -1 : 0;
            asm volatile("" : "+v"(m));
            s += __int_as_float(__float_as_int(v[t]) & m);
        }
    }
    red[gq][l] = s;
    __syncthreads();
    if (gq != 0 || i >= len) return;
#pragma unroll
    for (int u = 1; u < 8; ++u) s += red[u][l];
    out[i] = s;
}

}  // namespace

constexpr int64_t kBwdImg = (BH * BH * 4 + BH * 4) / 4;     // floats of one packed W2 image
constexpr int64_t kBwdExtra = 2 * kBwdImg + BH * BH + 64 + 3 * 1024;  // images, W2^T, maxima

extern "C" int64_t mmpde_gnn_edge_backward_partials(int *grid) {
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
        cus = 256;
    if (grid) *grid = cus > 0 ? cus : 256;
    // per-workgroup dW2 / db2 partials, then (fp16x3 mode) the two W2 images,
    // W2^T and the three maxima
    return (int64_t)(cus > 0 ? cus : 256) * (BH * BH + BH) + kBwdExtra;
}

static int edge_backward_f32(const float *a, const float *b, const int32_t *nbr, const int32_t *deg, int64_t n,
                             int k, const float *msg2_w, const float *msg2_b, const float *grad_mean,
                             const int32_t *pos, const uint32_t *mask, float *grad_a, float *grad_edge,
                             float *partials, float *grad_w2, float *grad_b2, mmpde_stream_t stream) {
    MMPDE_REQUIRE(a && b && nbr && msg2_w && msg2_b && grad_mean && grad_a && grad_edge && partials);
    MMPDE_REQUIRE(grad_w2 && grad_b2 && n > 0 && k > 0 && n <= (int64_t)INT32_MAX);
    MMPDE_REQUIRE((((uintptr_t)a | (uintptr_t)b | (uintptr_t)msg2_w | (uintptr_t)grad_mean) & 15) == 0);
    int grid = 256;
    mmpde_gnn_edge_backward_partials(&grid);
    const int64_t ntiles = (n + BT - 1) / BT;
    MMPDE_REQUIRE(ntiles < (int64_t)INT32_MAX);
    if (grid > ntiles) grid = (int)ntiles;
    float *pw2 = partials, *pb2 = partials + (int64_t)grid * BH * BH;
    EdgeBwdArgs p{a, b, nbr, deg, n, k, (int)ntiles, msg2_w, msg2_b, grad_mean, grad_a, grad_edge, pw2, pb2, pos,
                  mask};
    hipStream_t st = as_stream(stream);
    if (mask) hipLaunchKernelGGL(edge_bwd_kernel<true>, dim3(grid), dim3(256), 0, st, p);
    else hipLaunchKernelGGL(edge_bwd_kernel<false>, dim3(grid), dim3(256), 0, st, p);
    MMPDE_RET_LAUNCH();
    hipLaunchKernelGGL(partial_sum_kernel, dim3(ceil_div(BH * BH, 32)), dim3(256), 0, st, pw2, grid,
                       (int64_t)BH * BH, grad_w2);
    hipLaunchKernelGGL(partial_sum_kernel, dim3(BH / 32), dim3(256), 0, st, pb2, grid, (int64_t)BH, grad_b2);
    MMPDE_RET_LAUNCH();
    return MMPDE_OK;
}

static int edge_backward(const float *a, const float *b, const int32_t *nbr, const int32_t *deg, int64_t n, int k,
                         const float *msg2_w, const float *msg2_b, const float *grad_mean, const int32_t *pos,
                         const uint32_t *mask, float *grad_a, float *grad_edge, float *partials, float *grad_w2,
                         float *grad_b2, int edge_gemm, mmpde_stream_t stream) {
    MMPDE_REQUIRE(edge_gemm == MMPDE_EDGE_GEMM_F32 || edge_gemm == MMPDE_EDGE_GEMM_F16X3);
    if (edge_gemm == MMPDE_EDGE_GEMM_F32 || k > FKMAX)
        return edge_backward_f32(a, b, nbr, deg, n, k, msg2_w, msg2_b, grad_mean, pos, mask, grad_a, grad_edge, partials,
                                 grad_w2, grad_b2, stream);
    MMPDE_REQUIRE(a && b && nbr && msg2_w && msg2_b && grad_mean && grad_a && grad_edge && partials);
    MMPDE_REQUIRE(grad_w2 && grad_b2 && n > 0 && k > 0 && n <= (int64_t)INT32_MAX);
    MMPDE_REQUIRE((((uintptr_t)a | (uintptr_t)b | (uintptr_t)msg2_w | (uintptr_t)grad_mean |
                    (uintptr_t)partials) & 15) == 0);
    int grid = 256;
    mmpde_gnn_edge_backward_partials(&grid);
    const int64_t ntiles = (n + FT - 1) / FT;
    MMPDE_REQUIRE(ntiles < (int64_t)INT32_MAX && n * k < (int64_t)INT32_MAX);
    const int G = grid;
    if (grid > ntiles) grid = (int)ntiles;
    float *pw2 = partials, *pb2 = partials + (int64_t)G * BH * BH;
    float *ex = partials + (int64_t)G * (BH * BH + BH);
    char *img1 = (char *)ex, *img2 = (char *)(ex + kBwdImg);
    float *w2t = ex + 2 * kBwdImg;
    unsigned *mx = (unsigned *)(w2t + BH * BH);
    hipStream_t st = as_stream(stream);
    // W2 and W2^T as fp16x3 B images (f16x3.hpp layout), the split maxima
    PackSrc s1{}, s2{};
    s1.w[0] = msg2_w;
    s1.ld[0] = BH;
    s2.w[0] = w2t;
    s2.ld[0] = BH;
    hipLaunchKernelGGL(transpose128_kernel, dim3(BH * BH / 256), dim3(256), 0, st, msg2_w, w2t);
    hipLaunchKernelGGL((pack_f16x3_kernel<BH>), dim3(BH, 1), dim3(BH), 0, st, s1, 0, (int64_t)0, (int64_t)BH, img1);
    hipLaunchKernelGGL((pack_f16x3_kernel<BH>), dim3(BH, 1), dim3(BH), 0, st, s2, 0, (int64_t)0, (int64_t)BH, img2);
    MMPDE_RET_LAUNCH();
    const int64_t n4 = n * BH / 4;
    const int mg = (int)std::min<int64_t>(ceil_div(n4, 256), 1024);
    float *mpart = (float *)(mx + 64);  // 3 x mg per-workgroup maxima
    hipLaunchKernelGGL(maxabs3_kernel, dim3((unsigned)mg), dim3(256), 0, st, a, b, grad_mean, n4, mpart);
    hipLaunchKernelGGL(maxabs3_final_kernel, dim3(3), dim3(256), 0, st, mpart, mg, mx);
    MMPDE_RET_LAUNCH();
    EdgeBwdF16Args p{a, b, nbr, deg, n, k, (int)ntiles, img1, img2, msg2_b, grad_mean, mx, grad_a, grad_edge,
                     pw2, pb2, pos, mask};
    const bool o32 = n * BH * 4 < ((int64_t)1 << 32) && n * k * BH * 4 < ((int64_t)1 << 32);
    if (mask && o32) hipLaunchKernelGGL((edge_bwd_f16_kernel<true, true>), dim3(grid), dim3(512), 0, st, p);
    else if (mask) hipLaunchKernelGGL((edge_bwd_f16_kernel<true, false>), dim3(grid), dim3(512), 0, st, p);
    else if (o32) hipLaunchKernelGGL((edge_bwd_f16_kernel<false, true>), dim3(grid), dim3(512), 0, st, p);
    else hipLaunchKernelGGL((edge_bwd_f16_kernel<false, false>), dim3(grid), dim3(512), 0, st, p);
    MMPDE_RET_LAUNCH();
    hipLaunchKernelGGL(partial_sum_kernel, dim3(ceil_div(BH * BH, 32)), dim3(256), 0, st, pw2, grid,
                       (int64_t)BH * BH, grad_w2);
    hipLaunchKernelGGL(partial_sum_kernel, dim3(BH / 32), dim3(256), 0, st, pb2, grid, (int64_t)BH, grad_b2);
    MMPDE_RET_LAUNCH();
    return MMPDE_OK;
}

extern "C" int mmpde_gnn_edge_backward(const float *a, const float *b, const int32_t *nbr, const int32_t *deg,
                                       int64_t n, int k, const float *msg2_w, const float *msg2_b,
                                       const float *grad_mean, float *grad_a, float *grad_edge,
                                       float *partials, float *grad_w2, float *grad_b2,
                                       mmpde_stream_t stream) {
    return edge_backward_f32(a, b, nbr, deg, n, k, msg2_w, msg2_b, grad_mean, nullptr, nullptr, grad_a, grad_edge, partials,
                             grad_w2, grad_b2, stream);
}

extern "C" int mmpde_gnn_edge_backward_ex(const float *a, const float *b, const int32_t *nbr, const int32_t *deg,
                                          int64_t n, int k, const float *msg2_w, const float *msg2_b,
                                          const float *grad_mean, float *grad_a, float *grad_edge,
                                          float *partials, float *grad_w2, float *grad_b2, int edge_gemm,
                                          mmpde_stream_t stream) {
    return edge_backward(a, b, nbr, deg, n, k, msg2_w, msg2_b, grad_mean, nullptr, nullptr, grad_a, grad_edge,
                         partials, grad_w2, grad_b2, edge_gemm, stream);
}

extern "C" int mmpde_gnn_edge_backward_sorted(const float *a, const float *b, const int32_t *nbr,
                                              const int32_t *deg, int64_t n, int k, const float *msg2_w,
                                              const float *msg2_b, const float *grad_mean, const int32_t *slot_pos,
                                              const uint32_t *relu_mask, float *grad_a, float *grad_edge,
                                              float *partials, float *grad_w2, float *grad_b2, int edge_gemm,
                                              mmpde_stream_t stream) {
    MMPDE_REQUIRE(slot_pos);
    MMPDE_REQUIRE(!relu_mask || k <= FKMAX);
    return edge_backward(a, b, nbr, deg, n, k, msg2_w, msg2_b, grad_mean, slot_pos, relu_mask, grad_a, grad_edge,
                         partials, grad_w2, grad_b2, edge_gemm, stream);
}

extern "C" int mmpde_gnn_edge_source_sum_sorted(const float *grad_edge, const int64_t *rev_off, int64_t n,
                                                float *grad_b, mmpde_stream_t stream) {
    MMPDE_REQUIRE(grad_edge && rev_off && grad_b && n > 0);
    hipLaunchKernelGGL(edge_source_sum_sorted_kernel, dim3((unsigned)ceil_div(n, 4)), dim3(256), 0,
                       as_stream(stream), grad_edge, rev_off, n, grad_b);
    MMPDE_RET_LAUNCH();
    return MMPDE_OK;
}

extern "C" int mmpde_gnn_edge_source_sum(const float *grad_edge, const int64_t *rev_off, const int64_t *rev_edge,
                                         int64_t n, float *grad_b, mmpde_stream_t stream) {
    MMPDE_REQUIRE(grad_edge && rev_off && rev_edge && grad_b && n > 0);
    hipLaunchKernelGGL(edge_source_sum_kernel, dim3((unsigned)ceil_div(n, 4)), dim3(256), 0, as_stream(stream),
                       grad_edge, rev_off, rev_edge, n, grad_b);
    MMPDE_RET_LAUNCH();
    return MMPDE_OK;
}

extern "C" int mmpde_segment_sum(const float *rows, int64_t width, const int64_t *rev_off,
                                 const int64_t *rev_edge, int64_t n, float *out, mmpde_stream_t stream) {
    MMPDE_REQUIRE(rows && rev_off && rev_edge && out && n > 0 && width > 0);
    MMPDE_REQUIRE(n * width / 256 < (int64_t)INT32_MAX);
    hipLaunchKernelGGL(segment_sum_kernel, dim3((unsigned)ceil_div(n * width, 256)), dim3(256), 0,
                       as_stream(stream), rows, width, rev_off, rev_edge, n, out);
    MMPDE_RET_LAUNCH();
    return MMPDE_OK;
}
