// One message-passing layer of MP_PDE_Solver_2D (reference gnn_2d.py:53-69,
// GNN_Layer_FS_2D.forward/message/update) as two launches:
//
//   edge stage  mean_i = (1/k) sum_e relu(W2 relu(a_i + b_nbr(i,e)) + b2)
//   node stage  v_i = relu(U1 [h_i | mean_i | t_i] + c1)
//               h'_i = BN(h_i + relu(U2 v_i + c2))
//               a'_i, b'_i = next layer's message_net_1 node halves of h'_i
//
// a, b are message_net_1 factored exactly into a target half and a source half
// (its 260-wide input is cat(h_i, h_j, u_i-u_j, x_i-x_j, y_i-y_j, t_i), so
// W1 [h_i | h_j | du | dx | dy | t] = (W1a h_i + w.(u,x,y)_i + w_t t_i + b1)
// + (W1b h_j - w.(u,x,y)_j)); the reference's [E, 260] edge concat never
// exists and the only per-edge work is one 128x128 GEMM per edge.
//
// Edge stage (the dominant kernel): persistent, one 768-thread workgroup per
// CU walking a contiguous (XCD-local) range of 16-target tiles.  Waves 8-11 are
// producers: for neighbour slot e of a tile they gather the 16 source rows of
// b, form m = relu(a_i + b_j) in registers and store it to an LDS ring as the
// exact per-lane A operand (F16X3: scaled fp16 hi/lo halves).  Waves 0-7 are
// consumers: the two on one SIMD keep the same 32 output columns of W2 in
// registers for the whole launch and split each round's slots (even / odd),
// accumulating relu(. + b2) per target in registers (slot e of all 16 targets
// shares one accumulator row, so no cross-lane traffic); after the tile's last
// slot the odd-slot wave hands its sums to its partner through LDS, which
// writes the mean.  Sharing columns rather than splitting them halves the
// LDS operand reads (each slot is read by 4 waves, not 8).
// A workgroup's waves land on SIMDs in the order 0,2,1,3 (MI355X_MICROARCH.md),
// so waves w and w+4 share a SIMD: every SIMD pairs one MFMA stream with one
// VALU/gather stream.  One barrier per round of 4 slots; producers run
// ERING-1 rounds ahead, b rows are gathered two rounds before use.
//
// Node stage: 64 (or 32) rows per workgroup, 8 waves; every GEMM reads its
// weight operand once per workgroup (wave w owns output column tile w for all
// row blocks); activations are staged in LDS as MFMA operand images with
// per-row power-of-two scales (F16X3), and (F16X3) each workgroup stores the
// row maxima of its a', b' rows (layer.hpp).  No atomics: every output is
// deterministic.
#include "common.hpp"
#include <type_traits>
#include "f16x3.hpp"
#include "layer.hpp"

namespace {

constexpr int LH = 128;   // hidden width
constexpr int ET = 16;    // targets per edge tile
constexpr int ESL = 4;    // neighbour slots per round
constexpr int ERING = 3;  // LDS ring depth (rounds)
constexpr int EPF = ERING - 1;
constexpr int SLOT4 = 512;    // float4 per slot: 8 planes x 64 lanes = 8 KB
constexpr int NLDA = LH + 4;  // a-tile LDS row stride (floats)

// Contiguous XCD-local tile ranges (blocks b and b + 8 share an XCD): XCD x owns
// tiles [lo, hi), its workgroups i = b >> 3 take lo + i + nW * j.  Bijective
// for any grid; placement is used for speed only.
__device__ __forceinline__ void tile_schedule(int bid, int G, int ntiles, int &first, int &stride,
                                              int &count) {
    const int x = bid & 7, i = bid >> 3;
    const int q = G >> 3, rem = G & 7;
    const int nW = q + (x < rem ? 1 : 0);
    const int cum = x * q + min(x, rem);
    const int lo = (int)((int64_t)ntiles * cum / G);
    const int hi = (int)((int64_t)ntiles * (cum + nW) / G);
    first = lo + i;
    stride = nW;
    count = first < hi ? (hi - first + stride - 1) / stride : 0;
}

struct EdgeArgs {
    const float *a, *b;
    const int32_t *nbr;
    int64_t n;
    int k, ntiles;
    const float *w2, *b2;      // message_net_2.0 weight [128,128], bias
    const char *pk;            // F16X3: this layer's packed images (column scales of W2)
    const float *rsc;          // F16X3: split scale of every target row (layer.hpp row maxima)
    float *mean;               // [n, 128]
    uint64_t *stamps;          // profiling builds (PH bit 10): per-round s_memtime of block 0
    const int32_t *deg;        // RAGGED: in-degree of every target (nbr row entries past it are ignored)
    uint32_t *relu_mask;       // nullable: [n * k][4] bits z2 > 0 of every slot (training forward)
};

struct RoundCtr {  // (tile j, round rd) of a running round index
    int j, rd;
    __device__ void next(int rpt) {
        if (++rd == rpt) {
            rd = 0;
            ++j;
        }
    }
};

#ifndef MMPDE_EDGE_NC
#define MMPDE_EDGE_NC 2
#endif
constexpr int EDGE_NC = MMPDE_EDGE_NC;
#ifndef MMPDE_EDGE_NP
#define MMPDE_EDGE_NP 1
#endif
constexpr int EDGE_NP = MMPDE_EDGE_NP;

// PH: bit 0 produce, bit 1 consume (MFMA), bit 2 skip the gathers, bit 3 raise
// the consumer waves' issue priority, bit 5 replace the producer's split by a
// bare conversion, bit 6 store one ring piece in four (both timing only), bit 7
// re-read the tile's a rows every round, bit 4 (NC == 2) split each round's slots
// between the two consumer waves of a SIMD, which then own the same 32 output
// columns (half the LDS operand reads of column-split waves), bit 10 record
// per-round s_memtime stamps of block 0.  Bits other than 0, 1 and 4 are for
// profiling builds (tools/ubench); production launches use EDGE_PH.
#ifndef MMPDE_EDGE_PH
#define MMPDE_EDGE_PH 27
#endif
constexpr int EDGE_PH = MMPDE_EDGE_PH;
// relu_mask words need the SPLIT consumer layout (two waves per SIMD sharing 32
// columns, cg < 4): other profiling builds reject relu_mask at launch
constexpr bool kEdgeMaskOk = EDGE_NC == 2 && (EDGE_PH & 16);

// Slot operand layout (v_mfma_f32_16x16x32_f16; F32: v_mfma_f32_16x16x4_f32): a
// slot is the 16 x 128 message tile m[row][k] of one neighbour slot e of the
// tile's 16 targets; lane l = 16 g + row holds 8 float4-sized pieces i < 8:
//   F16X3 piece i: k = 32 (i >> 1) + 8 g + 4 (i & 1) + t -> pieces 2 s, 2 s + 1
//         are the fp16 hi / lo halves of K step s (k = 32 s + 8 g + t, t < 8);
//   F32   piece i: k = 16 i + 4 g + t (t < 4).
// stored as 8 lane-contiguous 1 KB planes (8 KB per slot).
//
// Workgroup: 4 NC consumer waves + 4 producer waves (NC consumers per SIMD: a
// workgroup's waves land on SIMDs in the order 0,2,1,3, so waves w, w + 4,
// w + 8 share one).  Producer p builds slot ESL rd + p of round rd; consumer c
// multiplies every slot by its 32 / NC output columns of W2 (held in
// registers for the whole launch).  One barrier per round; producers run EPF
// rounds ahead; b rows are gathered two rounds before use.
// RAGGED: target i averages over its first deg[i] table entries (PyG / torch_scatter
// mean over a variable in-degree: sum / max(deg, 1)); otherwise over all k.
template <bool F16X3, int PH = EDGE_PH, int NC = EDGE_NC, int NP = EDGE_NP, bool RAGGED = false>
__global__ __launch_bounds__(64 * (4 * NC + 4 * NP), 1) void gnn_edge_kernel(EdgeArgs p) {
    constexpr bool SPLIT = NC == 2 && (PH & 16);
    constexpr int CT = SPLIT ? 2 : 2 / NC;  // 16-column tiles per consumer wave
    constexpr int SPW = SPLIT ? ESL / 2 : ESL;  // slots per consumer wave and round
    constexpr int NPC = 8 / NP;  // float4 pieces of a slot lane per producer wave
    constexpr int NCT = 256 * NC;  // consumer threads
    __shared__ float4 ring[ERING * ESL * SLOT4];  // [round % ERING][slot][plane][lane]
    __shared__ float a_lds[2][ET * NLDA];        // a rows of tile j in [j & 1]
    // F16X3: the split scales of tile j's rows in [j & 7] (staged with the a rows;
    // eight deep: the consumers read a tile's until one round after its last,
    // staging runs one tile ahead of the producers)
    __shared__ float rs_ring[8][ET];
    // SPLIT: the odd-slot consumer's relu-sums of tile j, in [j & 1]
    __shared__ float4 xS[SPLIT ? 2 * 4 * CT * 64 : 1];
    const int tid = threadIdx.x;
    // wave index in an SGPR: every role / slot / liveness test below is then a
    // scalar branch (a VGPR wave index made `live` divergent: exec-masked MFMA
    // blocks and accumulator copies at every slot)
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
    const int r = lane & 15, g = lane >> 4;
    const bool producer = wave >= 4 * NC;
    int first, stride, nt;
    tile_schedule(blockIdx.x, gridDim.x, p.ntiles, first, stride, nt);
    const int k = p.k;
    const int rpt = (k + ESL - 1) / ESL;
    const int NR = nt * rpt;
    const int NIT = NR + EPF;
    const int NIT2 = (NIT + 1) & ~1;  // even: the producer's 2x-unrolled body has no tail test
    const int64_t nmax = p.n - 1;
    auto tile_row = [&](int j, int row) { return min((int64_t)(first + j * stride) * ET + row, nmax); };

    // a tiles (F16X3: scaled by their rows' split scales, |relu(a + b)| s < 2^11,
    // split8_relu_rtz): the consumer waves stage tile j + 1 while the producers
    // work on tile j, 2 / NC float4 per consumer thread.
    auto a_fetch = [&](int j, float4 *v, float *sv) {
#pragma unroll
        for (int u = 0; u < 2 / NC; ++u) {
            const int e = tid + NCT * u, row = e >> 5, c4 = e & 31;
            v[u] = *(const float4 *)(p.a + tile_row(j, row) * LH + 4 * c4);
            sv[u] = F16X3 ? p.rsc[tile_row(j, row)] : 1.0f;
        }
    };
    auto a_store = [&](int j, const float4 *v, const float *sv) {
#pragma unroll
        for (int u = 0; u < 2 / NC; ++u) {
            const int e = tid + NCT * u, row = e >> 5, c4 = e & 31;
            float4 x = v[u];
            if (F16X3) {
                const float sc = sv[u];
                x = make_float4(x.x * sc, x.y * sc, x.z * sc, x.w * sc);
                if (c4 == 0) rs_ring[j & 7][row] = sc;
            }
            *(float4 *)(&a_lds[j & 1][row * NLDA + 4 * c4]) = x;
        }
    };
    if (!producer && nt > 0) {
        float4 v[2 / NC];
        float sv[2 / NC];
        a_fetch(0, v, sv);
        a_store(0, v, sv);
    }
    __syncthreads();

    if (producer) {
        // ------------------------------------------------------------ producer
        // NP producers per slot (one per SIMD each): producer pidx builds
        // pieces i0 .. i0 + NPC - 1 of slot pidx & 3 (F16X3: K steps
        // i0 / 2 .. (i0 + NPC) / 2 - 1, hi and lo)
        const int pidx = wave - 4 * NC;
        if (PH & 2048) __builtin_amdgcn_s_setprio(2);  // profiling: producers first
        const int pw = pidx & 3, i0 = (pidx >> 2) * NPC;
        auto piece = [&](int i) {
            const int ii = i0 + i;
            return F16X3 ? 32 * (ii >> 1) + 8 * g + 4 * (ii & 1) : 16 * ii + 4 * g;
        };
        float4 acur[NPC], bv0[NPC], bv1[NPC];
        float sc = 1.0f;  // F16X3: split scale of this lane's row (r) of the tile
        // every round issues the same loads (clamped addresses past the end or
        // past k): 1 index + 8 gathers
        auto src_of = [&](const RoundCtr &c) -> uint32_t {
            return (uint32_t)p.nbr[tile_row(c.j, r) * k + min(ESL * c.rd + pw, k - 1)];
        };
        auto gather = [&](float4 *dst, uint32_t src) {
            const float *br = p.b + (int64_t)min(src, (uint32_t)nmax) * LH;  // clamped: a malformed table must not fault
#pragma unroll
            for (int i = 0; i < NPC; ++i) dst[i] = *(const float4 *)(br + piece(i));
        };
        RoundCtr cP{0, 0}, c2{0, 0}, c3{0, 0};
        uint32_t s0, s1;  // neighbour index of the round gathered next into bv0 / bv1
        // prologue in the loop's own load order (index of round R + 1, then the
        // gathers of round R): idx0, idx1, gathers0, idx2, gathers1
        {
            const uint32_t i0 = src_of(c2);
            c2.next(rpt);
            const uint32_t i1 = src_of(c2);
            c2.next(rpt);
            gather(bv0, i0);
            c3 = c2;
            s0 = src_of(c3);
            c3.next(rpt);
            gather(bv1, i1);
        }
        int slot = 0;
        // Branch-free rounds (a straight-line body keeps the compiler's
        // vector-memory waits counted): past the end and for slots past k the
        // producer still writes its ring slot (nobody reads it unmasked; after
        // the last round the slot written is neither of the rounds still being
        // consumed).
        auto body = [&](int it, float4 *bv, uint32_t &s_use, uint32_t &s_fill) {
            // the index of round it + 3 is this round's first load: a later use
            // of a register only waits for the loads issued before it
            s_fill = src_of(c3);
            c3.next(rpt);
            if (PH & 1) {
                // the a rows of a tile are the same for all its rounds: read them
                // from LDS once per tile (PH bit 7: every round)
                if ((PH & 128) || cP.rd == 0) {
                    const float *ar = &a_lds[cP.j & 1][r * NLDA];
#pragma unroll
                    for (int i = 0; i < NPC; ++i) acur[i] = *(const float4 *)(ar + piece(i));
                    if (F16X3) sc = rs_ring[cP.j & 7][r];
                }
                float4 *dst = ring + (slot * ESL + pw) * SLOT4 + i0 * 64 + lane;
                uint32_t fold = 0;
#pragma unroll
                for (int h2 = 0; h2 < NPC / 2; ++h2) {
                    const float4 &a0 = acur[2 * h2], &a1 = acur[2 * h2 + 1];
                    const float4 &b0 = bv[2 * h2], &b1 = bv[2 * h2 + 1];
                    float4 m0, m1;
                    if (F16X3) {  // relu folded into the split (split8_relu_rtz)
                        m0 = make_float4(fmaf(b0.x, sc, a0.x), fmaf(b0.y, sc, a0.y), fmaf(b0.z, sc, a0.z),
                                         fmaf(b0.w, sc, a0.w));
                        m1 = make_float4(fmaf(b1.x, sc, a1.x), fmaf(b1.y, sc, a1.y), fmaf(b1.z, sc, a1.z),
                                         fmaf(b1.w, sc, a1.w));
                        half8 hi, lo;
                        if (PH & 32) {  // profiling: conversion only, no split (wrong values)
                            const uint32_t w[4] = {
                                __builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_pkrtz(m0.x, m0.y)),
                                __builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_pkrtz(m0.z, m0.w)),
                                __builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_pkrtz(m1.x, m1.y)),
                                __builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_pkrtz(m1.z, m1.w))};
                            hi = *(const half8 *)w;
                            lo = hi;
                        } else {
                            split8_relu_rtz(m0, m1, hi, lo);
                        }
                        if (!(PH & 64) || h2 == 0) {
                            dst[(2 * h2 + 0) * 64] = *(const float4 *)&hi;
                            dst[(2 * h2 + 1) * 64] = *(const float4 *)&lo;
                        } else {  // profiling: one store in four, the rest folded (kept live)
                            const uint32_t *hw = (const uint32_t *)&hi, *lw = (const uint32_t *)&lo;
                            fold ^= hw[0] ^ hw[1] ^ hw[2] ^ hw[3] ^ lw[0] ^ lw[1] ^ lw[2] ^ lw[3];
                        }
                    } else {
                        m0 = make_float4(fmaxf(a0.x + b0.x, 0.0f), fmaxf(a0.y + b0.y, 0.0f),
                                         fmaxf(a0.z + b0.z, 0.0f), fmaxf(a0.w + b0.w, 0.0f));
                        m1 = make_float4(fmaxf(a1.x + b1.x, 0.0f), fmaxf(a1.y + b1.y, 0.0f),
                                         fmaxf(a1.z + b1.z, 0.0f), fmaxf(a1.w + b1.w, 0.0f));
                        dst[(2 * h2 + 0) * 64] = m0;
                        dst[(2 * h2 + 1) * 64] = m1;
                    }
                }
                if ((PH & 64) && fold == 0x9e3779b9u) dst[64] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
            }
            cP.next(rpt);
            // gather the round two ahead into the registers just consumed
            if (!(PH & 4)) gather(bv, s_use);
            c2.next(rpt);
            slot = slot == ERING - 1 ? 0 : slot + 1;
            if ((PH & 1024) && blockIdx.x == 0 && lane == 0 && it < 256)
                p.stamps[2 * 256 * wave + 2 * it] = __builtin_amdgcn_s_memtime();
            __syncthreads();
            if ((PH & 1024) && blockIdx.x == 0 && lane == 0 && it < 256)
                p.stamps[2 * 256 * wave + 2 * it + 1] = __builtin_amdgcn_s_memtime();
        };
        for (int it = 0; it < NIT2; it += 2) {
            body(it, bv0, s0, s1);
            body(it + 1, bv1, s1, s0);
        }
    } else {
        // ------------------------------------------------------------ consumer
        // this wave's output column tiles CT cg + cc (cc < CT); SPLIT: slots
        // hs, hs + 2 of every round
        const int cg = SPLIT ? (wave & 3) : wave;
        const int hs = SPLIT ? (wave >> 2) : 0;
        auto slotq = [&](int qq) { return SPLIT ? hs + 2 * qq : qq; };
        float4 wf[CT][8];
        half8 wh[CT][4], wl[CT][4];
        f32x4 bias[CT];  // accumulator initial value (message_net_2 bias, scaled; F16X3 per row)
        float bb0[CT];   // F16X3: the bias in the column scale (times the row scales per tile)
        float inv[CT];
#pragma unroll
        for (int cc = 0; cc < CT; ++cc) {
            const int col = 16 * (CT * cg + cc) + r;
            float bb = p.b2[col];
            if (F16X3) {
                const char *img = p.pk + kPkW2;
#pragma unroll
                for (int s4 = 0; s4 < 4; ++s4) {
                    wh[cc][s4] = bfrag(img, 4, CT * cg + cc, s4, 0, lane);
                    wl[cc][s4] = bfrag(img, 4, CT * cg + cc, s4, 1, lane);
                }
                const float sw = ((const float *)(img + 65536))[col];
                bb = bb * sw;
                inv[cc] = pow2_inv(sw);
            } else {
#pragma unroll
                for (int j = 0; j < 8; ++j) wf[cc][j] = *(const float4 *)(p.w2 + col * LH + 16 * j + 4 * g);
                inv[cc] = 1.0f;
            }
            bias[cc] = (f32x4){bb, bb, bb, bb};
            bb0[cc] = bb;
        }
        const float kdiv = (float)k;
        int dg[4] = {k, k, k, k};  // RAGGED: in-degree of this lane's rows 4 g + t of the tile
        f32x4 S[CT], Ssave[CT];
#pragma unroll
        for (int cc = 0; cc < CT; ++cc) S[cc] = (f32x4){0.0f, 0.0f, 0.0f, 0.0f};
        int pend = -1;  // SPLIT, even-slot wave: tile whose mean waits for the partner's sums
        // T: relu-sums in the scaled domain (F16X3: x sw[col] s[row], powers of
        // two); inv and the row scale undo it exactly before the division by the
        // degree
        auto write_mean = [&](int j, const f32x4 *T) {
            const int64_t row0 = (int64_t)(first + j * stride) * ET + 4 * g;
            float irs[4] = {1.0f, 1.0f, 1.0f, 1.0f};
            if (F16X3) {
#pragma unroll
                for (int t = 0; t < 4; ++t) irs[t] = pow2_inv(rs_ring[j & 7][4 * g + t]);
            }
#pragma unroll
            for (int cc = 0; cc < CT; ++cc) {
                const int col = 16 * (CT * cg + cc) + r;
#pragma unroll
                for (int t = 0; t < 4; ++t) {
                    const float div = RAGGED ? (float)max(dg[t], 1) : kdiv;
                    if (row0 + t < p.n) p.mean[(row0 + t) * LH + col] = T[cc][t] * inv[cc] * irs[t] / div;
                }
            }
        };
        auto finish_pending = [&]() {  // after the barrier that follows the partner's store
            if (SPLIT && pend >= 0) {
#pragma unroll
                for (int cc = 0; cc < CT; ++cc) {
                    const float4 o = xS[(((pend & 1) * 4 + cg) * CT + cc) * 64 + lane];
                    Ssave[cc] += (f32x4){o.x, o.y, o.z, o.w};
                }
                write_mean(pend, Ssave);
                pend = -1;
            }
        };
        RoundCtr cC{0, 0};
        int slot = 0;
        if (PH & 8) __builtin_amdgcn_s_setprio(1);
        // The next half slot is read from LDS while the current one is
        // multiplied (the next round's first half too: that round was
        // completed by the previous barrier), and each slot's relu-sum update
        // is issued after the next slot's first MFMAs.  Slots past k (last
        // round) are multiplied but not summed.
        // A operands stream through two half-slot register buffers (pieces
        // 0-3 / 4-7 of a slot lane)
        auto rd_half = [&](const float4 *src, int hf, float4 *x) {
#pragma unroll
            for (int i = 0; i < 4; ++i) x[i] = src[(4 * hf + i) * 64];
        };
        auto mma_half = [&](const float4 *x, int hf, f32x4 *acc) {
            if (F16X3) {
#pragma unroll
                for (int s = 0; s < 2; ++s) {
                    const int s4 = 2 * hf + s;
                    const half8 hi = *(const half8 *)&x[2 * s], lo = *(const half8 *)&x[2 * s + 1];
#pragma unroll
                    for (int cc = 0; cc < CT; ++cc) acc[cc] = mfma_f16(hi, wh[cc][s4], s4 == 0 ? bias[cc] : acc[cc]);
#pragma unroll
                    for (int cc = 0; cc < CT; ++cc) acc[cc] = mfma_f16(hi, wl[cc][s4], acc[cc]);
#pragma unroll
                    for (int cc = 0; cc < CT; ++cc) acc[cc] = mfma_f16(lo, wh[cc][s4], acc[cc]);
                }
            } else {
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const int jj = 4 * hf + j;
#pragma unroll
                    for (int t = 0; t < 4; ++t) {
#pragma unroll
                        for (int cc = 0; cc < CT; ++cc)
                            acc[cc] = mfma16(f4c(x[j], t), f4c(wf[cc][jj], t), jj == 0 && t == 0 ? bias[cc] : acc[cc]);
                    }
                }
            }
        };
        // relu-sum of slot e; e < k is wave-uniform (slots past k exist only
        // in a tile's last round), so it is a branch, not a select; RAGGED adds
        // the per-row e < deg select
        // (relu as v_med3(x, 0, max): one instruction, where fmaxf adds a NaN-
        // quieting canonicalize; the column scale is applied once, in write_mean)
        auto sum_into = [&](const f32x4 *acc, int e) {
            if (e >= k) return;
#pragma unroll
            for (int cc = 0; cc < CT; ++cc) {
#pragma unroll
                for (int t = 0; t < 4; ++t) {
                    float v = __builtin_amdgcn_fmed3f(acc[cc][t], 0.0f, 3.402823466e38f);
                    if (RAGGED) v = e < dg[t] ? v : 0.0f;
                    S[cc][t] += v;
                }
            }
            if constexpr (SPLIT) if (p.relu_mask) {
                // the z2 > 0 bits the backward reuses (mmpde_gnn_edge_backward_sorted):
                // ballots per (column tile cc, row t) cover rows 4 g + t, g < 4,
                // 16 columns each; lane l < 16 stores row 4 (l >> 2) + (l & 3)'s
                // word of this wave's 32 columns (CT = 2 tiles, cg < 4): one store
                // per slot.  Builds without SPLIT reject relu_mask at launch
                // (kEdgeMaskOk).
                static_assert(CT == 2, "relu mask words take two column tiles per wave");
                uint64_t bal[CT][4];
#pragma unroll
                for (int cc = 0; cc < CT; ++cc)
#pragma unroll
                    for (int t = 0; t < 4; ++t) bal[cc][t] = __ballot(acc[cc][t] > 0.0f);
                const int tl = lane & 3, gl = (lane >> 2) & 3;
                uint64_t b0 = bal[0][0], b1 = bal[CT - 1][0];
#pragma unroll
                for (int t = 1; t < 4; ++t) {
                    b0 = tl == t ? bal[0][t] : b0;
                    b1 = tl == t ? bal[CT - 1][t] : b1;
                }
                const uint32_t word = (uint32_t)((b0 >> (16 * gl)) & 0xffffu) |
                                      ((uint32_t)((b1 >> (16 * gl)) & 0xffffu) << 16);
                const int64_t row = (int64_t)(first + cC.j * stride) * ET + 4 * gl + tl;
                if (lane < 16 && row < p.n) p.relu_mask[(row * k + e) * 4 + cg] = word;
            }
        };
        float4 xa[4], xb[4], an[2 / NC];
        float asv[2 / NC];
        int js = 1;  // next a tile to stage: stored in iteration js * rpt - 1 (the
                     // producers read it from iteration js * rpt), fetched up to two
                     // iterations earlier but after the previous store
        const int lead = min(2, rpt - 1);
        for (int it = 0; it < NIT2; ++it) {
            finish_pending();
            if (js < nt) {
                const int ts = js * rpt - 1;
                if (it == ts - lead) a_fetch(js, an, asv);
                if (it == ts) {
                    a_store(js, an, asv);
                    ++js;
                }
            }
            if (it >= EPF && it < NIT && (PH & 2)) {
                const float4 *base = ring + slot * ESL * SLOT4 + lane;
                const float4 *nbase = ring + (slot == ERING - 1 ? 0 : slot + 1) * ESL * SLOT4 + lane;
                if (it == EPF) rd_half(base + slotq(0) * SLOT4, 0, xa);
                if (RAGGED && cC.rd == 0) {  // a new tile (after finish_pending used the last one's)
#pragma unroll
                    for (int t = 0; t < 4; ++t) dg[t] = p.deg[tile_row(cC.j, 4 * g + t)];
                }
                if (F16X3 && cC.rd == 0) {  // the new tile's row scales (rows 4 g + t)
#pragma unroll
                    for (int cc = 0; cc < CT; ++cc)
#pragma unroll
                        for (int t = 0; t < 4; ++t) bias[cc][t] = bb0[cc] * rs_ring[cC.j & 7][4 * g + t];
                }
                // Straight-line round: every slot is multiplied (a slot past k, in
                // a tile's last round only, holds a duplicate of the last
                // neighbour and is not summed) and the next round's first half
                // slot is read even after the last round (in-bounds, unused):
                // no branch joins, so the accumulators need no copies.
                f32x4 acc[SPW][CT];
#pragma unroll
                for (int qq = 0; qq < SPW; ++qq) {
                    rd_half(base + slotq(qq) * SLOT4, 1, xb);
                    mma_half(xa, 0, acc[qq]);
                    if (qq > 0) sum_into(acc[qq - 1], ESL * cC.rd + slotq(qq - 1));
                    if (qq < SPW - 1) rd_half(base + slotq(qq + 1) * SLOT4, 0, xa);
                    else rd_half(nbase + slotq(0) * SLOT4, 0, xa);
                    mma_half(xb, 1, acc[qq]);
                }
                sum_into(acc[SPW - 1], ESL * cC.rd + slotq(SPW - 1));
                if (cC.rd == rpt - 1) {  // tile complete: mean = sum / degree (PyG mean)
                    if (!SPLIT) {
                        write_mean(cC.j, S);
                    } else if (hs == 1) {  // hand the odd slots' sums to the partner wave
#pragma unroll
                        for (int cc = 0; cc < CT; ++cc)
                            xS[(((cC.j & 1) * 4 + cg) * CT + cc) * 64 + lane] =
                                make_float4(S[cc][0], S[cc][1], S[cc][2], S[cc][3]);
                    } else {
#pragma unroll
                        for (int cc = 0; cc < CT; ++cc) Ssave[cc] = S[cc];
                        pend = cC.j;
                    }
#pragma unroll
                    for (int cc = 0; cc < CT; ++cc) S[cc] = (f32x4){0.0f, 0.0f, 0.0f, 0.0f};
                }
                cC.next(rpt);
                slot = slot == ERING - 1 ? 0 : slot + 1;
            }
            if ((PH & 1024) && blockIdx.x == 0 && lane == 0 && it < 256)
                p.stamps[2 * 256 * wave + 2 * it] = __builtin_amdgcn_s_memtime();
            __syncthreads();
            if ((PH & 1024) && blockIdx.x == 0 && lane == 0 && it < 256)
                p.stamps[2 * 256 * wave + 2 * it + 1] = __builtin_amdgcn_s_memtime();
            if ((PH & 1024) && blockIdx.x == 0 && tid == 0 && (it == 0 || it == NIT2 - 1)) {
                // shader clock vs the 100 MHz constant clock, first / last round
                p.stamps[12 * 2 * 256 + (it ? 2 : 0)] = __builtin_amdgcn_s_memtime();
                p.stamps[12 * 2 * 256 + (it ? 3 : 1)] = __builtin_amdgcn_s_memrealtime();
            }
        }
        finish_pending();  // the loop ends with a barrier
    }
}

// ---------------------------------------------------------------------------
// Node stage
// ---------------------------------------------------------------------------
struct NodeArgs {
    const float *h, *mean;
    int64_t n;
    const float *u1, *c1;  // update_net_1.0 [128, ld_u1] (h | mean | t), bias
    int64_t ld_u1;
    const float *u2, *c2;  // update_net_2.0 [128, 128], bias
    const float *bn_w, *bn_b, *bn_rm, *bn_rv;
    float eps;
    float *h_out;
    const float *w1n, *b1n;  // next layer message_net_1.0 [128, ld_w1n], bias (NEXT)
    int64_t ld_w1n;
    float *a_out, *b_out;
    const float *u, *pos;
    mmpde_gnn_scales sc;
    const char *pk, *pkn;  // F16X3 images: this layer (U1, U2), next layer (W1)
    float *rmx_out;        // F16X3: row maxima of a', b' and their range records (layer.hpp)
    int64_t seg_n;         // rows per trajectory segment (range records)
    int parts;             // mean = sum of `parts` buffers part_stride floats apart
    int64_t part_stride;
    // div_k > 0: the buffers hold neighbour sums (F16X3 wave edge kernel); the
    // mean is their total / max(div_deg[row], 1), or / div_k without degrees
    const int32_t *div_deg = nullptr;
    int div_k = 0;
    EdgeSplit split;       // units > 0: add the wave kernel's side blocks first
};

constexpr int NLD = 132;  // fp32 staging row stride (floats)
#ifndef MMPDE_NODE_WPE
#define MMPDE_NODE_WPE 4
#endif
constexpr int NODE_WPE = MMPDE_NODE_WPE;  // node / embed launch bounds: waves per SIMD
// node / embed kernels: issue B operands one phase before their GEMMs instead
// of just before them.  EARLY_U2: update_net_2's (dead bH / bM registers);
// EARLY_B: the next projections' b' operands beside a' (measured: node
// 50.6-51.1 vs 50.0-50.2 us, embed 45.2-45.4 vs 42.8-43.0 us with 4 spills;
// off).  Same arithmetic either way.
#ifndef MMPDE_NODE_EARLY_U2
#define MMPDE_NODE_EARLY_U2 1
#endif
#ifndef MMPDE_NODE_EARLY_B
#define MMPDE_NODE_EARLY_B 0
#endif
constexpr bool NODE_EARLY_U2 = MMPDE_NODE_EARLY_U2 != 0;
// EARLY_M: update_net_1's mean-half operands beside the h-half ones at the
// start, in the last layer's kernel (with the next projections it spills);
// measured 31.9 against 31.3-31.4 us (profiles/r04_node_early_m_ab.log), so off
#ifndef MMPDE_NODE_EARLY_M
#define MMPDE_NODE_EARLY_M 0
#endif
constexpr bool NODE_EARLY_M = MMPDE_NODE_EARLY_M != 0;
constexpr bool NODE_EARLY_B = MMPDE_NODE_EARLY_B != 0;

// Operand images in LDS, per 16-row block rb and K step s (1 KB units of 64
// lanes x 16 B): F16X3 [rb][s (32-wide)][hi|lo] with lane (r, g) holding
// k = 32 s + 8 g + t; F32 [rb][s (16-wide)] with lane (r, g) holding k = 16 s + 4 g + t.
// prep(): rows of 128 fp32 values (src, row stride lds) -> image at k offset
// kofs (multiple of 128) of an image KT wide; F16X3 scales each row by a power
// of two (its max |x| -> [2^13, 2^14)) and records it in rs[row].  8 lanes per row.
// nsum > 1: src is the first of nsum buffers sum_stride floats apart, added in
// buffer order (the edge stage's per-part sums); div_k > 0: the total is then
// divided by the row's degree max(div_deg[row], 1), or by div_k (IEEE division:
// torch_scatter's mean = sum / count).
// The (row, part) item of prep's work index idx: a wave takes 8 rows x 8 parts,
// lane = 8 part + row: the 8 lanes of one ds_write_b128 group write 8
// consecutive image rows (conflict-free).
__device__ __forceinline__ void prep_item(int idx, int &row, int &part) {
    row = (idx >> 6) * 8 + (idx & 7);
    part = (idx >> 3) & 7;
}

// prep, first half: the 16 values of item (row, part) of rows src (row stride
// lds; global rows row0 + row clamped to nrows_valid - 1, else LDS rows).
__device__ __forceinline__ void prep_fetch(const float *src, int64_t lds, int64_t row0, int64_t nrows_valid,
                                           bool global, int row, int part, float4 (&x)[4]) {
    const int64_t srow = global ? min(row0 + row, nrows_valid - 1) : row;
    const float *sp = src + srow * lds + 16 * part;
#pragma unroll
    for (int q = 0; q < 4; ++q) x[q] = *(const float4 *)(sp + 4 * q);
}

// prep, second half: the fetched values x of item (row, part) (global row srow
// when global) -> the image (and copy, rs), after the optional side-block sums
// and degree division (see prep).
template <bool F16X3>
__device__ __forceinline__ void prep_finish(float4 (&x)[4], const float *src, int64_t srow, int row, int part,
                                            float4 *img, int KT, int kofs, float *rs, float *copy, int nsum,
                                            int64_t sum_stride, const int32_t *div_deg, int div_k,
                                            const EdgeSplit *split) {
    const float *sp = src + srow * LH + 16 * part;
    for (int ps = 1; ps < nsum; ++ps) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const float4 y = *(const float4 *)(sp + ps * sum_stride + 4 * q);
            x[q] = make_float4(x[q].x + y.x, x[q].y + y.y, x[q].z + y.z, x[q].w + y.w);
        }
    }
    if (split && split->units > 0) {
        // side blocks of the units u of this row's segment whose first slot
        // s0(u) = floor(u S / U) lies strictly inside the row's 16-row tile
        // t (local): t k < s0(u) < (t + 1) k
        const int64_t S = split->S, G = split->units, kk = split->k;
        int64_t sg, q, lo, hi;
        if ((uint64_t)(S + 1) * (uint64_t)(G + 1) + (uint64_t)split->seg_n < 0xffffffffull) {
            // 32-bit divisions (wave-uniform test: a 64-bit one is a long
            // instruction sequence, three per row here)
            const uint32_t sn = (uint32_t)split->seg_n, r32 = (uint32_t)srow;
            const uint32_t sg32 = r32 / sn, q32 = r32 - sg32 * sn, t = q32 / 16;
            const uint32_t S32 = (uint32_t)S, G32 = (uint32_t)G, k32 = (uint32_t)kk;
            sg = sg32;
            q = q32;
            lo = max(((t * k32 + 1) * G32 + S32 - 1) / S32, 1u);
            hi = min(((t + 1) * k32 * G32 + S32 - 1) / S32 - 1, G32 - 1);
        } else {
            sg = srow / split->seg_n;
            q = srow - sg * split->seg_n;
            const int64_t t = q / 16;
            lo = max(((t * kk + 1) * G + S - 1) / S, (int64_t)1);
            hi = min(((t + 1) * kk * G + S - 1) / S - 1, G - 1);
        }
        for (int64_t w = lo; w <= hi; ++w) {
            const float *q4 = split->side + ((sg * G + w) * 16 + (q & 15)) * 128 + 16 * part;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const float4 y = *(const float4 *)(q4 + 4 * q);
                x[q] = make_float4(x[q].x + y.x, x[q].y + y.y, x[q].z + y.z, x[q].w + y.w);
            }
        }
    }
    if (div_k > 0) {
        const float d = div_deg ? (float)max(div_deg[srow], 1) : (float)div_k;
        div_rows_rn(x, d);
    }
    if (copy) {
#pragma unroll
        for (int q = 0; q < 4; ++q) *(float4 *)(copy + row * NLD + 16 * part + 4 * q) = x[q];
    }
    const int rb = row >> 4, rr = row & 15;
    if (F16X3) {
        float m = 0.0f;
#pragma unroll
        for (int q = 0; q < 4; ++q) m = absmax4(m, x[q]);
        m = absmax_stride8(m);  // the row's 8 parts (lanes l ^ 8, ^ 16, ^ 32)
        const float s = split_scale(m);
        if (part == 0) rs[row] = s;
#pragma unroll
        for (int q = 0; q < 4; ++q) x[q] = make_float4(x[q].x * s, x[q].y * s, x[q].z * s, x[q].w * s);
        const int KS = KT / 32;
        const int ks = (kofs + 16 * part) >> 5;
        const int g0 = 2 * (part & 1);
#pragma unroll
        for (int hh = 0; hh < 2; ++hh) {
            half8 hi, lo;
            split8_rn(x[2 * hh], x[2 * hh + 1], hi, lo);
            float4 *d = img + ((rb * KS + ks) * 2) * 64 + 16 * (g0 + hh) + rr;
            d[0] = *(const float4 *)&hi;
            d[64] = *(const float4 *)&lo;
        }
    } else {
        const int KJ = KT / 16;
        const int j = (kofs >> 4) + part;
#pragma unroll
        for (int q = 0; q < 4; ++q) img[(rb * KJ + j) * 64 + 16 * q + rr] = x[q];
    }
}

template <bool F16X3, int ROWS>
__device__ __forceinline__ void prep(const float *src, int64_t lds, int64_t row0, int64_t nrows_valid,
                                     bool global, float4 *img, int KT, int kofs, float *rs,
                                     float *copy = nullptr, int t0 = -1, int nthr = 512, int nsum = 1,
                                     int64_t sum_stride = 0, const int32_t *div_deg = nullptr,
                                     int div_k = 0, const EdgeSplit *split = nullptr) {
    // threads t0 .. t0 + nthr (default: the whole workgroup) share the rows
    for (int idx = t0 < 0 ? (int)threadIdx.x : (int)threadIdx.x - t0; idx < ROWS * 8; idx += nthr) {
        int row, part;
        prep_item(idx, row, part);
        float4 x[4];
        prep_fetch(src, lds, row0, nrows_valid, global, row, part, x);
        const int64_t srow = global ? min(row0 + row, nrows_valid - 1) : row;
        prep_finish<F16X3>(x, src, srow, row, part, img, KT, kofs, rs, copy, nsum, sum_stride, div_deg, div_k,
                           split);
    }
}

// B operand fragments of NS K steps of column tile ct, loaded ahead of use.
// F16X3: packed image (KSB 32-wide K steps per column tile) steps sb0 ..;
// F32: fp32 weight row wrow (this lane's column), 16-wide steps from k = wk0.
template <bool F16X3, int NS>
struct BOps {
    half8 h[F16X3 ? NS : 1], l[F16X3 ? NS : 1];
    float4 w[F16X3 ? 1 : NS];
    __device__ __forceinline__ void load(const char *bimg, int KSB, int ct, int sb0,
                                         const float *wrow, int wk0, int lane) {
#pragma unroll
        for (int s = 0; s < NS; ++s) {
            if (F16X3) {
                h[s] = bfrag(bimg, KSB, ct, sb0 + s, 0, lane);
                l[s] = bfrag(bimg, KSB, ct, sb0 + s, 1, lane);
            } else {
                w[s] = *(const float4 *)(wrow + wk0 + 16 * s + 4 * (lane >> 4));
            }
        }
    }
};

// acc[rb] += A(image rows, K steps s0 .. s0 + NS of an image KT wide) x B.
template <bool F16X3, int RB, int NS>
__device__ __forceinline__ void gemm_tile(f32x4 *acc, const float4 *img, int KT, int s0,
                                          const BOps<F16X3, NS> &B, int lane) {
#pragma unroll
    for (int s = 0; s < NS; ++s) {
#pragma unroll
        for (int rb = 0; rb < RB; ++rb) {
            if (F16X3) {
                const int KS = KT / 32;
                const float4 h4 = img[((rb * KS + s0 + s) * 2) * 64 + lane];
                const float4 l4 = img[((rb * KS + s0 + s) * 2 + 1) * 64 + lane];
                const half8 ah = *(const half8 *)&h4, al = *(const half8 *)&l4;
                acc[rb] = mfma_f16(ah, B.h[s], acc[rb]);
                acc[rb] = mfma_f16(ah, B.l[s], acc[rb]);
                acc[rb] = mfma_f16(al, B.h[s], acc[rb]);
            } else {
                const int KJ = KT / 16;
                const float4 a = img[(rb * KJ + s0 + s) * 64 + lane];
                acc[rb] = mfma16(a.x, B.w[s].x, acc[rb]);
                acc[rb] = mfma16(a.y, B.w[s].y, acc[rb]);
                acc[rb] = mfma16(a.z, B.w[s].z, acc[rb]);
                acc[rb] = mfma16(a.w, B.w[s].w, acc[rb]);
            }
        }
    }
}

constexpr int MAX_TW = 16;  // time_window (u channels) of the fused kernels

// Per-row node values of one row: t / tmax, x / Lx, y / Ly, u_0 .. u_{tw-1}.
// fetch() issues every load first (written value by value, node_t / node_x /
// node_y's branches kept the compiler from hoisting the loads past each
// other's LDS writes: one memory round trip per value); store() writes them
// to rowv[.][tid].
struct RowValues {
    float t = 0.0f, x = 0.0f, y = 0.0f, u[MAX_TW];
    __device__ __forceinline__ void fetch(const mmpde_gnn_scales &sc, const float *pos, const float *uu,
                                          int64_t row, int tw) {
        const float *pr = sc.pos_xy ? pos + row * 2 : pos + row * 3 + 1;
        x = pr[0];
        y = pr[1];
        t = sc.pos_xy ? (sc.t_ptr ? *sc.t_ptr : sc.t) : pr[-1];
#pragma unroll
        for (int c = 0; c < MAX_TW; ++c) u[c] = c < tw ? uu[row * tw + c] : 0.0f;
    }
    template <int ROWS>
    __device__ __forceinline__ void store(float (*rowv)[ROWS], const mmpde_gnn_scales &sc, int tid, int tw) const {
        rowv[0][tid] = t * sc.inv_tmax;
        rowv[1][tid] = x * sc.inv_lx;
        rowv[2][tid] = y * sc.inv_ly;
#pragma unroll
        for (int c = 0; c < MAX_TW; ++c)
            if (c < tw) rowv[3 + c][tid] = u[c];
    }
};

// Per-column constants of a message_net_1 node projection (weight row w1r of
// this lane's column: node-term columns 256 .. 256 + tw - 1 (u_i - u_j, du holds
// the first), 256 + tw (x), 257 + tw (y), 258 + tw (t), bias, F16X3 unscale).
struct W1C {
    float du = 0.0f, dx = 0.0f, dy = 0.0f, t = 0.0f, b = 0.0f, isa = 1.0f, isb = 1.0f;
    template <bool F16X3>
    __device__ __forceinline__ void load(const float *w1r, const float *b1, const char *pk, int col,
                                         int tw) {
        du = w1r[256];
        dx = w1r[256 + tw];
        dy = w1r[257 + tw];
        t = w1r[258 + tw];
        b = b1[col];
        if (F16X3) {
            const float *su = (const float *)(pk + kPkW1 + 131072);
            isa = pow2_inv(su[col]);
            isb = pow2_inv(su[128 + col]);
        }
    }
};

// message_net_1 node halves of the rows staged in img (K = 128, F16X3 row
// scales rs): a = W1[:, :128] h + w.(u, x, y) + w_t t + b1 (column tile wave),
// b = W1[:, 128:256] h - w.(u, x, y) (column tile 8 + wave); the epilogue of
// gnn_2d.py:53-57's message_net_1 split (see the file header).  rowv: per-row
// (t, x, y, u_0 .. u_{tw-1}) planes of stride 16 RB.  bA: preloaded B operands of a.
template <bool F16X3, int RB>
__device__ __forceinline__ void proj_phase(const BOps<F16X3, F16X3 ? 4 : 8> &bA, const float4 *img,
                                           const float *rs, const float *rowv, const W1C &w,
                                           const char *pk, const float *w1r, int tw, int64_t row0,
                                           int64_t n, int64_t seg_n, float *a_out, float *b_out,
                                           float *rmx_out, uint32_t *arrived, int wave, int lane,
                                           const BOps<F16X3, F16X3 ? 4 : 8> *bBpre = nullptr) {
    constexpr int ROWS = 16 * RB, S1 = F16X3 ? 4 : 8;
    const int col = 16 * wave + (lane & 15), g = lane >> 4;
    f32x4 aA[RB], aB[RB];
#pragma unroll
    for (int rb = 0; rb < RB; ++rb) aA[rb] = aB[rb] = (f32x4){0.0f, 0.0f, 0.0f, 0.0f};
    // |a'|, |b'| of this lane's rows (16 rb + 4 g + q, column col) as bit
    // patterns (for x, y >= 0 the integer max is the float max, with no NaN
    // canonicalisation): the rows' maxima for the edge stage's split scales
    uint32_t amx[RB][4], bmx[RB][4];
#pragma unroll
    for (int rb = 0; rb < RB; ++rb)
#pragma unroll
        for (int q = 0; q < 4; ++q) amx[rb][q] = bmx[rb][q] = 0u;
    // stores at immediate offsets from one base per lane; the row test only
    // for a tile that runs past n (wave-uniform)
    const bool full = row0 + ROWS <= n;
    float *ap = a_out + (row0 + 4 * g) * LH + col, *bp = b_out + (row0 + 4 * g) * LH + col;
    // the node term w.(u, x, y) of row lr (shared by a and b)
    auto node_term = [&](int lr) {
        float node = w.du * rowv[3 * ROWS + lr];
        for (int c = 1; c < tw; ++c) node += w1r[256 + c] * rowv[(3 + c) * ROWS + lr];
        return node + w.dx * rowv[ROWS + lr] + w.dy * rowv[2 * ROWS + lr];
    };
    gemm_tile<F16X3, RB, S1>(aA, img, 128, 0, bA, lane);
    {
        if (bBpre) {  // operands of b preloaded (the weight-stationary node kernel)
            gemm_tile<F16X3, RB, S1>(aB, img, 128, 0, *bBpre, lane);
        } else {
            BOps<F16X3, S1> bB;
            bB.load(pk + kPkW1, 4, 8 + wave, 0, w1r, 128, lane);
            gemm_tile<F16X3, RB, S1>(aB, img, 128, 0, bB, lane);
        }
#pragma unroll
        for (int rb = 0; rb < RB; ++rb) {
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int lr = 16 * rb + 4 * g + q;
                if (full || row0 + lr < n) {
                    float za = aA[rb][q], zb = aB[rb][q];
                    if (F16X3) {
                        const float ir = pow2_inv(rs[lr]);
                        za = za * ir * w.isa;
                        zb = zb * ir * w.isb;
                    }
                    const float node = node_term(lr);
                    const float va = za + node + w.t * rowv[lr] + w.b;
                    const float vb = zb - node;
                    ap[(16 * rb + q) * LH] = va;
                    bp[(16 * rb + q) * LH] = vb;
                    // |v| with NaN -> 0 (fmaxf ignores a NaN, as the float max did)
                    amx[rb][q] = __builtin_bit_cast(uint32_t, fmaxf(fabsf(va), 0.0f));
                    bmx[rb][q] = __builtin_bit_cast(uint32_t, fmaxf(fabsf(vb), 0.0f));
                }
            }
        }
    }
    if (rmx_out) {
        // row maxima: over this wave's 16 columns (the 16 lanes r of one DPP
        // row: quad [1,0,3,2], quad [2,3,0,1], row_half_mirror, row_mirror), then
        // over the 8 waves without a barrier: each wave posts its maxima to LDS
        // and counts itself in (LDS atomic); the last of the 8 to arrive reduces
        // and stores the tile's rows.  (A __syncthreads here also waits for every
        // wave's a' / b' stores: 7-8 us of the 54 us node launch at cy B=16.)  The
        // max is order-free, so the record does not depend on the arrival order.
        __shared__ uint32_t red[8][ROWS][2];
#pragma unroll
        for (int rb = 0; rb < RB; ++rb) {
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                uint32_t ua = amx[rb][q], ub = bmx[rb][q];
                ua = max(ua, dpp_u<0xB1>(ua));
                ub = max(ub, dpp_u<0xB1>(ub));
                ua = max(ua, dpp_u<0x4E>(ua));
                ub = max(ub, dpp_u<0x4E>(ub));
                ua = max(ua, dpp_u<0x141>(ua));
                ub = max(ub, dpp_u<0x141>(ub));
                ua = max(ua, dpp_u<0x140>(ua));
                ub = max(ub, dpp_u<0x140>(ub));
                if ((lane & 15) == 0) {
                    red[wave][16 * rb + 4 * g + q][0] = ua;
                    red[wave][16 * rb + 4 * g + q][1] = ub;
                }
            }
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // posted before counted
        uint32_t prev = 0;
        if (lane == 0) prev = __hip_atomic_fetch_add(arrived, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        prev = __builtin_amdgcn_readfirstlane(prev);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if (prev == 7) {
            // per lane: row l >> 1, value e = l & 1 (max|a'| / max|b'|); then the
            // tile's 16-row blocks' range records (layer.hpp) by butterflies over
            // the row bits (l ^ 2 .. l ^ 16: the 16 rows of one block), each row
            // in part 0 (its block's first segment) or part 1 (the next)
            static_assert(2 * ROWS % 64 == 0, "row maxima: whole waves");
#pragma unroll
            for (int l0 = 0; l0 < 2 * ROWS; l0 += 64) {
                const int l = l0 + lane, row = l >> 1, e = l & 1;
                uint32_t m = red[0][row][e];
#pragma unroll
                for (int w2 = 1; w2 < 8; ++w2) m = max(m, red[w2][row][e]);
                const int64_t grow = row0 + row, b0 = row0 + 16 * (row >> 4);
                const bool live = grow < n;
                if (live) rmx_out[2 * grow + e] = __builtin_bit_cast(float, m);
                const bool part1 = grow >= (b0 / seg_n + 1) * seg_n;
                uint32_t mx0 = live && !part1 ? m : 0u, mx1 = live && part1 ? m : 0u;
                uint32_t mn0 = live && !part1 ? m : 0x7f800000u, mn1 = live && part1 ? m : 0x7f800000u;
                auto xmax = [&](uint32_t &v, auto O) {
                    v = max(v, __builtin_bit_cast(uint32_t, xor_lane_f<decltype(O)::value>(__builtin_bit_cast(float, v))));
                };
                auto xmin = [&](uint32_t &v, auto O) {
                    v = min(v, __builtin_bit_cast(uint32_t, xor_lane_f<decltype(O)::value>(__builtin_bit_cast(float, v))));
                };
                using X2 = std::integral_constant<int, 2>;
                using X4 = std::integral_constant<int, 4>;
                using X8 = std::integral_constant<int, 8>;
                using X16 = std::integral_constant<int, 16>;
                xmax(mx0, X2{}); xmax(mx1, X2{}); xmin(mn0, X2{}); xmin(mn1, X2{});
                xmax(mx0, X4{}); xmax(mx1, X4{}); xmin(mn0, X4{}); xmin(mn1, X4{});
                xmax(mx0, X8{}); xmax(mx1, X8{}); xmin(mn0, X8{}); xmin(mn1, X8{});
                xmax(mx0, X16{}); xmax(mx1, X16{}); xmin(mn0, X16{}); xmin(mn1, X16{});
                // lanes 0, 1 (and 32, 33) of each block hold its e = 0 / 1 results:
                // record fields {max a, max b, min a, min b} of part 0, then part 1
                if ((l & 31) < 2 && b0 < n) {
                    float *rec = rmx_out + row_max_floats(n) + 8 * (b0 / 16);
                    rec[e] = __builtin_bit_cast(float, mx0);
                    rec[2 + e] = __builtin_bit_cast(float, mn0);
                    rec[4 + e] = __builtin_bit_cast(float, mx1);
                    rec[6 + e] = __builtin_bit_cast(float, mn1);
                }
            }
        }
    }
}

// Profiling builds only (tools/ubench/node_ubench with -DMMPDE_NODE_STAMPS):
// thread 0 of every workgroup records the 100 MHz real-time clock (one clock
// for the whole chip) at the phase boundaries into g_node_stamps[block][8]
// (vector stores).
#ifdef MMPDE_NODE_STAMPS
__device__ uint64_t *g_node_stamps;
#define NODE_STAMP(i)                                                                       \
    do {                                                                                   \
        if (threadIdx.x == 0) g_node_stamps[(int64_t)blockIdx.x * 8 + (i)] = __builtin_amdgcn_s_memrealtime(); \
    } while (0)
#else
#define NODE_STAMP(i) \
    do {              \
    } while (0)
#endif

template <bool NEXT, bool F16X3, int RB>
__global__ __launch_bounds__(512, NODE_WPE) void gnn_node_kernel(NodeArgs p) {
    NODE_STAMP(0);
    constexpr int ROWS = 16 * RB;
    __shared__ float4 img[RB * 16 * 64];        // operand image, K = 256 (h | mean), then 128
    __shared__ float stage[ROWS * NLD];         // fp32 v, then h'
    __shared__ float hres[ROWS * NLD];          // fp32 h (residual)
    __shared__ float rs[4][ROWS];               // row scales: h, mean, v, h'
    __shared__ float rowv[3 + MAX_TW][ROWS];    // per row: t / tmax, x / Lx, y / Ly, u_0 .. u_{tw-1}
    __shared__ uint32_t rng_arrived;            // waves done with their row maxima (proj_phase)
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const int r = lane & 15, g = lane >> 4;
    const int col = 16 * wave + r;  // this lane's output column (tile = wave)
    if (tid == 0) rng_arrived = 0;  // read after the first barrier
    const int tw = p.sc.tw > 1 ? p.sc.tw : 1;
    constexpr int S1 = F16X3 ? 4 : 8;    // K steps per 128 columns of K
    const float *wu1 = p.u1 + (int64_t)col * p.ld_u1, *wu2 = p.u2 + (int64_t)col * LH;
    const int64_t row0 = (int64_t)blockIdx.x * ROWS;
    // everything the epilogues read from global memory is fetched up front
    // (per-row node values to LDS, per-column constants to registers), so no
    // epilogue waits on a memory round trip
    RowValues rv;
    if (tid < ROWS) rv.fetch(p.sc, p.pos, p.u, min(row0 + tid, p.n - 1), tw);
    const float u1_wt = wu1[256], u1_b = p.c1[col];
    const float u1_is = F16X3 ? pow2_inv(((const float *)(p.pk + kPkU1 + 131072))[col]) : 1.0f;
    const float u2_b = p.c2[col];
    BnAffine bn;
    bn.set(p.bn_rm[col], p.bn_rv[col], p.bn_w[col], p.bn_b[col], p.eps);
    const float u2_is = F16X3 ? pow2_inv(((const float *)(p.pk + kPkU2 + 65536))[col]) : 1.0f;
    const float *w1r = NEXT ? p.w1n + (int64_t)col * p.ld_w1n : nullptr;
    W1C w1c;
    if (NEXT) w1c.load<F16X3>(w1r, p.b1n, p.pkn, col, tw);
    // weight operands of update_net_1 / _2 loaded first: their latency hides
    // behind the activation staging
    // (RB >= 4: all three up front; smaller tiles run several workgroups per
    // CU, whose overlap hides the latency, so they load just before use)
    constexpr bool PRE = RB >= 4;
    BOps<F16X3, S1> bH, bM, bU2;
    bH.load(p.pk + kPkU1, 8, wave, 0, wu1, 0, lane);
    if (PRE || (NODE_EARLY_M && !NEXT)) bM.load(p.pk + kPkU1, 8, wave, S1, wu1, 128, lane);
    if (PRE) {
        bU2.load(p.pk + kPkU2, 4, wave, 0, wu2, 0, lane);
    }
    if (tid < ROWS) rv.store<ROWS>(rowv, p.sc, tid, tw);

    NODE_STAMP(1);
    // ---- [h | mean] -> image (K = 256)
    if constexpr (ROWS * 8 <= 256) {  // h on waves 0-3, mean on waves 4-7 at once
        if (tid < 256) prep<F16X3, ROWS>(p.h, LH, row0, p.n, true, img, 256, 0, rs[0], hres, 0, 256);
        else prep<F16X3, ROWS>(p.mean, LH, row0, p.n, true, img, 256, 128, rs[1], nullptr, 256, 256, p.parts,
                               p.part_stride, p.div_deg, p.div_k, &p.split);
    } else {
        prep<F16X3, ROWS>(p.h, LH, row0, p.n, true, img, 256, 0, rs[0], hres);
        prep<F16X3, ROWS>(p.mean, LH, row0, p.n, true, img, 256, 128, rs[1], nullptr, -1, 512, p.parts,
                          p.part_stride, p.div_deg, p.div_k, &p.split);
    }
    __syncthreads();
    NODE_STAMP(2);

    // ---- update_net_1: v = relu(U1 [h | mean | t] + c1)
    {
        f32x4 aH[RB], aM[RB];
#pragma unroll
        for (int rb = 0; rb < RB; ++rb) aH[rb] = aM[rb] = (f32x4){0.0f, 0.0f, 0.0f, 0.0f};
        gemm_tile<F16X3, RB, S1>(aH, img, 256, 0, bH, lane);
        if (!PRE && !(NODE_EARLY_M && !NEXT)) bM.load(p.pk + kPkU1, 8, wave, S1, wu1, 128, lane);
        gemm_tile<F16X3, RB, S1>(F16X3 ? aM : aH, img, 256, S1, bM, lane);
        // update_net_2's operands issued now (bH / bM are dead): in flight over
        // this epilogue, the operand prep and its two barriers
        if (!PRE && NODE_EARLY_U2) bU2.load(p.pk + kPkU2, 4, wave, 0, wu2, 0, lane);
#pragma unroll
        for (int rb = 0; rb < RB; ++rb) {
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int lr = 16 * rb + 4 * g + q;
                float v = aH[rb][q];
                if (F16X3) v = v * pow2_inv(rs[0][lr]) * u1_is + aM[rb][q] * pow2_inv(rs[1][lr]) * u1_is;
                stage[lr * NLD + col] = fmaxf(v + u1_wt * rowv[0][lr] + u1_b, 0.0f);
            }
        }
    }
    NODE_STAMP(3);
    __syncthreads();
    prep<F16X3, ROWS>(stage, NLD, 0, ROWS, false, img, 128, 0, rs[2]);
    __syncthreads();
    NODE_STAMP(4);

    // ---- update_net_2 + residual + BatchNorm(eval)
    BOps<F16X3, S1> bA, bB;
    {
        f32x4 acc[RB];
#pragma unroll
        for (int rb = 0; rb < RB; ++rb) acc[rb] = (f32x4){0.0f, 0.0f, 0.0f, 0.0f};
        if (!PRE && !NODE_EARLY_U2) bU2.load(p.pk + kPkU2, 4, wave, 0, wu2, 0, lane);
        gemm_tile<F16X3, RB, S1>(acc, img, 128, 0, bU2, lane);
        // next layer's message_net_1 operands of a' (column tile wave), and of
        // b' with NODE_EARLY_B (both in flight over the epilogue and the prep)
        if (NEXT) bA.load(p.pkn + kPkW1, 4, wave, 0, w1r, 0, lane);
        if (NEXT && NODE_EARLY_B) bB.load(p.pkn + kPkW1, 4, 8 + wave, 0, w1r, 128, lane);
        const bool full = row0 + ROWS <= p.n;
        float *hp = p.h_out + (row0 + 4 * g) * LH + col;
#pragma unroll
        for (int rb = 0; rb < RB; ++rb) {
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int lr = 16 * rb + 4 * g + q;
                float z = acc[rb][q];
                if (F16X3) z = z * pow2_inv(rs[2][lr]) * u2_is;
                const float x = hres[lr * NLD + col] + fmaxf(z + u2_b, 0.0f);
                const float y = bn(x);
                if (full || row0 + lr < p.n) hp[(16 * rb + q) * LH] = y;
                if (NEXT) stage[lr * NLD + col] = y;
            }
        }
    }
    NODE_STAMP(5);
    if constexpr (NEXT) {
        __syncthreads();
        prep<F16X3, ROWS>(stage, NLD, 0, ROWS, false, img, 128, 0, rs[3]);
        __syncthreads();
        NODE_STAMP(6);
        // ---- next layer's message_net_1 node halves
        proj_phase<F16X3, RB>(bA, img, rs[3], &rowv[0][0], w1c, p.pkn, w1r, tw, row0, p.n, p.seg_n,
                              p.a_out, p.b_out, p.rmx_out, &rng_arrived, wave, lane, NODE_EARLY_B ? &bB : nullptr);
    }
    NODE_STAMP(7);
}

// ---------------------------------------------------------------------------
// Embedding + layer 0's message_net_1 halves in one launch (gnn_2d.py:99-106,
// 122-131, then the first GNN layer's projections): per 64-row tile
//   z  = relu(BN1(W0 [u, x/Lx, y/Ly, t/tmax] + b0))        (VALU, K = 4)
//   h0 = BN4(W3 z + b3)            (F16X3: fp16x3 MFMA, W3 split in-kernel; F32: exact fp32)
//   a0, b0 = layer 0's message_net_1 node halves of h0      (F16X3 or fp32)
// ---------------------------------------------------------------------------
struct EmbedArgs {
    const float *u, *pos;
    int64_t n;
    mmpde_gnn_scales sc;
    mmpde_gnn_embed_params e;
    float *h_out;
    const float *w1, *b1;  // layer 0 message_net_1.0 [128, ld_w1], bias
    int64_t ld_w1;
    float *a_out, *b_out;
    const char *pk;        // F16X3: layer 0's packed images
    float *rmx_out;        // F16X3: layer 0's row maxima and range records
    int64_t seg_n;         // rows per trajectory segment (range records)
};

template <bool F16X3, int RB>
__global__ __launch_bounds__(512, NODE_WPE) void gnn_embed_kernel(EmbedArgs p) {
    constexpr int ROWS = 16 * RB;
    constexpr int S1 = F16X3 ? 4 : 8;
    __shared__ float4 img[RB * 8 * 64];   // K = 128 operand image
    __shared__ float stage[ROWS * NLD];   // fp32 z, then h0
    __shared__ float rs[ROWS];            // h0 row scales
    __shared__ uint32_t rng_arrived;      // waves done with their row maxima (proj_phase)
    __shared__ float rsz[ROWS];           // z row scales (F16X3 embedding GEMM)
    __shared__ float rowv[3 + MAX_TW][ROWS];  // per row: t / tmax, x / Lx, y / Ly, u_0 .. u_{tw-1}
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const int g = lane >> 4;
    const int64_t row0 = (int64_t)blockIdx.x * ROWS;
    const int col = 16 * wave + (lane & 15);
    const int tw = p.sc.tw > 1 ? p.sc.tw : 1;
    if (tid == 0) rng_arrived = 0;  // read after the first barrier
    RowValues rv;
    if (tid < ROWS) rv.fetch(p.sc, p.pos, p.u, min(row0 + tid, p.n - 1), tw);
    const mmpde_gnn_embed_params &e = p.e;
    // embedding_mlp.3 weight row of this lane's column: F32 as the exact fp32
    // B operand; F16X3 split here into the fp16 hi / lo operand with a
    // power-of-two column scale (one 128 x 128 weight: no packed image needed)
    BOps<false, 8> b3;
    BOps<true, 4> b3h;
    float w3_is = 1.0f;
    if (F16X3) {
        const float *wr = e.w3 + (int64_t)col * LH;
        float4 w[8];
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            w[2 * s] = *(const float4 *)(wr + 32 * s + 8 * g);
            w[2 * s + 1] = *(const float4 *)(wr + 32 * s + 8 * g + 4);
        }
        float m = 0.0f;
#pragma unroll
        for (int i = 0; i < 8; ++i) m = absmax4(m, w[i]);
        m = fmaxf(m, __shfl_xor(m, 16, 64));
        m = fmaxf(m, __shfl_xor(m, 32, 64));
        const float sw = split_scale(m);
        w3_is = pow2_inv(sw);
#pragma unroll
        for (int i = 0; i < 8; ++i) w[i] = make_float4(w[i].x * sw, w[i].y * sw, w[i].z * sw, w[i].w * sw);
#pragma unroll
        for (int s = 0; s < 4; ++s) split8_rn(w[2 * s], w[2 * s + 1], b3h.h[s], b3h.l[s]);
    } else {
        b3.load(nullptr, 0, 0, 0, e.w3 + (int64_t)col * LH, 0, lane);
    }
    const float h_b = e.b3[col];
    BnAffine bn4;
    bn4.set(e.bn4_rm[col], e.bn4_rv[col], e.bn4_w[col], e.bn4_b[col], e.eps);
    const float *w1r = p.w1 + (int64_t)col * p.ld_w1;
    W1C w1c;
    w1c.load<F16X3>(w1r, p.b1, p.pk, col, tw);
    // z: thread tid owns channel c = tid & 127 of rows (tid >> 7) + 4 i;
    // embedding_mlp.0 weight [128, tw + 3] over (u_0 .. u_{tw-1}, x, y, t)
    const int c = tid & 127;
    const float *zwr = e.w0 + (int64_t)c * (tw + 3);
    const float zw0 = zwr[0], zw1 = zwr[tw], zw2 = zwr[tw + 1], zw3 = zwr[tw + 2];
    const float zb = e.b0[c];
    BnAffine bn1;
    bn1.set(e.bn1_rm[c], e.bn1_rv[c], e.bn1_w[c], e.bn1_b[c], e.eps);
    if (tid < ROWS) rv.store<ROWS>(rowv, p.sc, tid, tw);
    __syncthreads();
    for (int row = tid >> 7; row < ROWS; row += 4) {
        float v = zb + zw0 * rowv[3][row];
        for (int ch = 1; ch < tw; ++ch) v += zwr[ch] * rowv[3 + ch][row];
        v = v + zw1 * rowv[1][row] + zw2 * rowv[2][row] + zw3 * rowv[0][row];
        stage[row * NLD + c] = fmaxf(bn1(v), 0.0f);
    }
    __syncthreads();
    prep<F16X3, ROWS>(stage, NLD, 0, ROWS, false, img, 128, 0, rsz);
    __syncthreads();
    BOps<F16X3, S1> bA, bB;
    {
        f32x4 acc[RB];
#pragma unroll
        for (int rb = 0; rb < RB; ++rb) acc[rb] = (f32x4){0.0f, 0.0f, 0.0f, 0.0f};
        if (F16X3) {
            gemm_tile<true, RB, 4>(acc, img, 128, 0, b3h, lane);
#pragma unroll
            for (int rb = 0; rb < RB; ++rb)
#pragma unroll
                for (int q = 0; q < 4; ++q) acc[rb][q] *= pow2_inv(rsz[16 * rb + 4 * g + q]) * w3_is;
        } else {
            gemm_tile<false, RB, 8>(acc, img, 128, 0, b3, lane);
        }
        bA.load(p.pk + kPkW1, 4, wave, 0, w1r, 0, lane);
        if (NODE_EARLY_B) bB.load(p.pk + kPkW1, 4, 8 + wave, 0, w1r, 128, lane);
        const bool full = row0 + ROWS <= p.n;
        float *hp = p.h_out + (row0 + 4 * g) * LH + col;
#pragma unroll
        for (int rb = 0; rb < RB; ++rb) {
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int lr = 16 * rb + 4 * g + q;
                const float y = bn4(acc[rb][q] + h_b);
                if (full || row0 + lr < p.n) hp[(16 * rb + q) * LH] = y;
                stage[lr * NLD + col] = y;
            }
        }
    }
    __syncthreads();
    prep<F16X3, ROWS>(stage, NLD, 0, ROWS, false, img, 128, 0, rs);
    __syncthreads();
    proj_phase<F16X3, RB>(bA, img, rs, &rowv[0][0], w1c, p.pk, w1r, tw, row0, p.n, p.seg_n,
                          p.a_out, p.b_out, p.rmx_out, &rng_arrived, wave, lane, NODE_EARLY_B ? &bB : nullptr);
}

inline bool al16(const void *q) { return ((uintptr_t)q & 15u) == 0; }

int device_cus() {
    int dev = 0, cus = 0;
    if (hipGetDevice(&dev) != hipSuccess) return 256;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus < 1)
        return 256;
    return cus;
}

}  // namespace

// Node stage rows per workgroup (16 * RB)
#ifndef MMPDE_NODE_RB
#define MMPDE_NODE_RB 2
#endif


int launch_edge_stage(const float *a, const float *b, const int32_t *nbr, const int32_t *deg,
                      int64_t n, int k, int64_t seg_n, const mmpde_gnn_layer_params *p, const char *pk,
                      const float *rmx, float *mean, float *side, int64_t side_cap,
                      EdgeSplit *split, hipStream_t st, uint32_t *relu_mask, bool rng) {
    if (split) *split = EdgeSplit{};
    MMPDE_REQUIRE(!relu_mask || (!pk && kEdgeMaskOk && al16(relu_mask)));  // the ring kernel's F32 training forward
    MMPDE_REQUIRE(a && b && nbr && p && mean && n > 0 && k > 0 && n <= (int64_t)INT32_MAX);
    MMPDE_REQUIRE(al16(a) && al16(b) && al16(p->msg2_w) && al16(mean));
    MMPDE_REQUIRE(!pk || (rmx && al16(pk) && al16(rmx)));
    const int64_t ntiles = (n + ET - 1) / ET;
    MMPDE_REQUIRE(ntiles * ((k + ESL - 1) / ESL) < (int64_t)INT32_MAX);
    const int cus = device_cus();
    // F16X3: one wave per SIMD with the operands in registers (edge_wave.hip);
    // the wave kernel leaves the side blocks and the division to the node stage
    if (pk)
        return launch_edge_wave(a, b, nbr, deg, n, k, seg_n, p->msg2_b, pk, rmx, rng, mean, side, side_cap, cus,
                                split, st);
    // F32: the exact fp32 ring kernel
    EdgeArgs e{a, b, nbr, n, k, (int)ntiles, p->msg2_w, p->msg2_b, nullptr, nullptr, mean, nullptr, deg, relu_mask};
    const int grid = ntiles < cus ? (int)ntiles : cus;
    const dim3 block(64 * (4 * EDGE_NC + 4 * EDGE_NP));
    if (deg) hipLaunchKernelGGL((gnn_edge_kernel<false, EDGE_PH, EDGE_NC, EDGE_NP, true>), dim3(grid), block, 0, st, e);
    else hipLaunchKernelGGL(gnn_edge_kernel<false>, dim3(grid), block, 0, st, e);
    MMPDE_RET_LAUNCH();
    return MMPDE_OK;
}

// Row maxima (layer.hpp) of a, b for the training forward: rmx[2 i] = max|a_i|,
// rmx[2 i + 1] = max|b_i| (a NaN counts as 0).  Half a wave per row (32 lanes x
// one float4 of each).
__global__ __launch_bounds__(256) void row_max_kernel(const float *__restrict__ a, const float *__restrict__ b,
                                                      int64_t n, float *__restrict__ rmx) {
    const int64_t row = (int64_t)blockIdx.x * 8 + (threadIdx.x >> 5);
    const int c4 = threadIdx.x & 31;
    const int64_t rr = min(row, n - 1);
    float ma = absmax4(0.0f, *(const float4 *)(a + rr * LH + 4 * c4));
    float mb = absmax4(0.0f, *(const float4 *)(b + rr * LH + 4 * c4));
#pragma unroll
    for (int o = 16; o >= 1; o >>= 1) {
        ma = fmaxf(ma, __shfl_xor(ma, o, 32));
        mb = fmaxf(mb, __shfl_xor(mb, o, 32));
    }
    if (c4 == 0 && row < n) *(float2 *)(rmx + 2 * row) = make_float2(ma, mb);
}

// Split scale of every target row (f16x3.hpp row_split_scale): rsc[i] from
// max|a_i| + max over the row's neighbours e < deg[i] (ragged tables) or k of
// max|b_nbr(i,e)|.  One thread per row.
__global__ __launch_bounds__(256) void row_scale_kernel(const float *__restrict__ rmx, const int32_t *__restrict__ nbr,
                                                        const int32_t *__restrict__ deg, int64_t n, int k,
                                                        float *__restrict__ rsc) {
    const int64_t row = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (row >= n) return;
    const int kk = deg ? max(min(deg[row], k), 1) : k;
    const float mb = nbr_bmax<36>(rmx, nbr + row * k, kk, (uint32_t)(n - 1));
    rsc[row] = row_split_scale(rmx[2 * row] + mb);
}

// The edge stage's mean from the wave kernel's neighbour sums (in mean) and
// side blocks (the node stage's prep_finish, for callers that want the mean
// itself): sums + the side blocks of the units that start strictly inside
// the row's tile, in unit order, / max(deg, 1) or / k.  8 threads per row.
__global__ __launch_bounds__(256) void edge_finish_kernel(float *__restrict__ mean, EdgeSplit sp,
                                                          const int32_t *__restrict__ deg, int64_t n) {
    const int64_t row = (int64_t)blockIdx.x * 32 + (threadIdx.x >> 3);
    const int part = threadIdx.x & 7;
    if (row >= n) return;
    float *mp = mean + row * LH + 16 * part;
    float4 x[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) x[q] = *(const float4 *)(mp + 4 * q);
    const int64_t S = sp.S, G = sp.units, kk = sp.k;
    const int64_t sg = row / sp.seg_n, ql = row - sg * sp.seg_n, t = ql / 16;
    const int64_t lo = max(((t * kk + 1) * G + S - 1) / S, (int64_t)1);
    const int64_t hi = min(((t + 1) * kk * G + S - 1) / S - 1, G - 1);
    for (int64_t w = lo; w <= hi; ++w) {
        const float *q4 = sp.side + ((sg * G + w) * 16 + (ql & 15)) * LH + 16 * part;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const float4 y = *(const float4 *)(q4 + 4 * q);
            x[q] = make_float4(x[q].x + y.x, x[q].y + y.y, x[q].z + y.z, x[q].w + y.w);
        }
    }
    div_rows_rn(x, deg ? (float)max(deg[row], 1) : (float)kk);
#pragma unroll
    for (int q = 0; q < 4; ++q) *(float4 *)(mp + 4 * q) = x[q];
}

// workspace of the F16X3 edge mean: W2's image, the row maxima, then the ring
// kernel's row scales or the wave kernel's side blocks (one per 16-row tile)
int64_t edge_mean_f16x3_ws_bytes(int64_t n) {
    const int64_t tail = ((n + 15) / 16) * 16 * LH;  // >= the n row scales
    return kLayerPack + (row_max_floats(n) + tail) * 4;
}

// The edge stage writing the mean itself, F16X3 with this call's own W2 image
// and row maxima: mmpde_gnn_edge_mean_ex, where the weights change every call.
// With relu_mask (the training forward: every slot's z2 > 0 bits for the
// backward) the persistent ring kernel on the rows' split scales; without it
// the one-wave-per-SIMD kernel of the inference forward (one segment of n rows,
// one side block per 16-row tile) and edge_finish_kernel.
int launch_edge_mean_f16x3(const float *a, const float *b, const int32_t *nbr, const int32_t *deg, int64_t n,
                           int k, const float *w2, const float *b2, float *mean, uint32_t *relu_mask, void *ws,
                           hipStream_t st) {
    MMPDE_REQUIRE(a && b && nbr && w2 && b2 && mean && ws && n > 0 && k > 0 && n <= (int64_t)INT32_MAX);
    MMPDE_REQUIRE(al16(a) && al16(b) && al16(w2) && al16(mean) && al16(ws));
    MMPDE_REQUIRE(!relu_mask || (kEdgeMaskOk && al16(relu_mask)));
    const int64_t ntiles = (n + ET - 1) / ET;
    MMPDE_REQUIRE(ntiles * ((k + ESL - 1) / ESL) < (int64_t)INT32_MAX);
    char *pk = (char *)ws;
    float *rmx = (float *)(pk + kLayerPack);
    float *rsc = rmx + row_max_floats(n);
    PackSrc src{};
    src.w[0] = w2;
    src.ld[0] = LH;
    hipLaunchKernelGGL(pack_f16x3_kernel<128>, dim3(128, 1), dim3(128), 0, st, src, 0, kPkW2, (int64_t)128, pk);
    MMPDE_RET_LAUNCH();
    hipLaunchKernelGGL(row_max_kernel, dim3((unsigned)ceil_div(n, 8)), dim3(256), 0, st, a, b, n, rmx);
    MMPDE_RET_LAUNCH();
    const int cus = device_cus();
    if (!relu_mask) {
        float *side = rsc;
        EdgeSplit split;
        const int rc = launch_edge_wave(a, b, nbr, deg, n, k, n, b2, pk, rmx, false, mean, side, ntiles, cus,
                                        &split, st);
        if (rc) return rc;
        MMPDE_REQUIRE(split.units > 0);
        hipLaunchKernelGGL(edge_finish_kernel, dim3((unsigned)ceil_div(n, 32)), dim3(256), 0, st, mean, split,
                           deg, n);
        MMPDE_RET_LAUNCH();
        return MMPDE_OK;
    }
    hipLaunchKernelGGL(row_scale_kernel, dim3((unsigned)ceil_div(n, 256)), dim3(256), 0, st, rmx, nbr, deg, n, k,
                       rsc);
    MMPDE_RET_LAUNCH();
    EdgeArgs e{a, b, nbr, n, k, (int)ntiles, w2, b2, pk, rsc, mean, nullptr, deg, relu_mask};
    const int grid = ntiles < cus ? (int)ntiles : cus;
    const dim3 block(64 * (4 * EDGE_NC + 4 * EDGE_NP));
    if (deg) hipLaunchKernelGGL((gnn_edge_kernel<true, EDGE_PH, EDGE_NC, EDGE_NP, true>), dim3(grid), block, 0, st, e);
    else hipLaunchKernelGGL(gnn_edge_kernel<true>, dim3(grid), block, 0, st, e);
    MMPDE_RET_LAUNCH();
    return MMPDE_OK;
}

// The kernel arguments of one node-stage call (validated).
static int node_args(const NodeStageCall &c, NodeArgs *out) {
    const bool sums = c.split && c.split->units > 0;
    MMPDE_REQUIRE(!sums || (c.split->side && c.split->S > 0 && c.split->k > 0 && c.split->seg_n > 0 &&
                            c.n % c.split->seg_n == 0));
    MMPDE_REQUIRE(!c.rmx_out || al16(c.rmx_out));
    MMPDE_REQUIRE(c.h && c.mean && c.u && c.pos && c.p && c.h_out && c.n > 0);
    MMPDE_REQUIRE(al16(c.h) && al16(c.mean) && al16(c.h_out));
    MMPDE_REQUIRE(c.p->upd1_ld >= 257 && (c.p->upd1_ld & 3) == 0 && al16(c.p->upd1_w) && al16(c.p->upd2_w));
    MMPDE_REQUIRE(!c.pk || (al16(c.pk) && (!c.next || c.pkn)));
    const mmpde_gnn_layer_params *p = c.p;
    NodeArgs a{c.h, c.mean, c.n, p->upd1_w, p->upd1_b, p->upd1_ld, p->upd2_w, p->upd2_b, p->bn_w, p->bn_b,
               p->bn_rm, p->bn_rv, p->eps, c.h_out, nullptr, nullptr, 0, c.a_out, c.b_out, c.u, c.pos, c.sc,
               c.pk, c.pkn, c.rmx_out, effective_seg(c.n, c.seg_n), 1, 0, sums ? c.deg : nullptr,
               sums ? c.split->k : 0};
    if (sums) a.split = *c.split;
    if (c.next) {
        MMPDE_REQUIRE(c.a_out && c.b_out && c.next->msg1_ld >= 260 && (c.next->msg1_ld & 3) == 0 &&
                      al16(c.next->msg1_w));
        a.w1n = c.next->msg1_w;
        a.b1n = c.next->msg1_b;
        a.ld_w1n = c.next->msg1_ld;
    }
    *out = a;
    return MMPDE_OK;
}

static int launch_node_stage(const NodeStageCall &c, hipStream_t st) {
    constexpr int RB = MMPDE_NODE_RB;
    NodeArgs a;
    int rc = node_args(c, &a);
    if (rc) return rc;
    const bool next = c.next != nullptr, f16 = c.pk != nullptr;
    const int64_t tiles = ceil_div(c.n, 16 * RB);
    MMPDE_REQUIRE(tiles < (int64_t)INT32_MAX);
    const dim3 grid((unsigned)tiles);
#define MMPDE_NODE(NX, SPLIT) \
    hipLaunchKernelGGL((gnn_node_kernel<NX, SPLIT, RB>), grid, dim3(512), 0, st, a)
    if (next && f16) MMPDE_NODE(true, true);
    else if (next) MMPDE_NODE(true, false);
    else if (f16) MMPDE_NODE(false, true);
    else MMPDE_NODE(false, false);
#undef MMPDE_NODE
    MMPDE_RET_LAUNCH();
    return MMPDE_OK;
}

int launch_node_stage(const float *h, const float *mean, const EdgeSplit *split, const int32_t *deg,
                      const float *u, const float *pos, int64_t n, int64_t seg_n, mmpde_gnn_scales sc,
                      const mmpde_gnn_layer_params *p, const mmpde_gnn_layer_params *next,
                      const char *pk, const char *pkn, float *rmx_out, float *h_out, float *a_out,
                      float *b_out, hipStream_t st) {
    const NodeStageCall c{h, mean, split, deg, u, pos, n, seg_n, sc, p, next, pk, pkn, rmx_out, h_out, a_out,
                          b_out};
    return launch_node_stage(c, st);
}

static int embed_args(const EmbedStageCall &c, EmbedArgs *out) {
    MMPDE_REQUIRE(c.u && c.pos && c.e && c.l0 && c.h_out && c.a_out && c.b_out && c.n > 0);
    MMPDE_REQUIRE(al16(c.e->w3) && al16(c.h_out) && al16(c.a_out) && al16(c.b_out));
    MMPDE_REQUIRE(c.l0->msg1_ld >= 260 && (c.l0->msg1_ld & 3) == 0 && al16(c.l0->msg1_w));
    MMPDE_REQUIRE(!c.pk0 || (al16(c.pk0) && c.rmx_out && al16(c.rmx_out)));
    *out = EmbedArgs{c.u, c.pos, c.n, c.sc, *c.e, c.h_out, c.l0->msg1_w, c.l0->msg1_b, c.l0->msg1_ld, c.a_out,
                     c.b_out, c.pk0, c.rmx_out, effective_seg(c.n, c.seg_n)};
    return MMPDE_OK;
}

static int launch_embed_stage(const EmbedStageCall &c, hipStream_t st) {
    constexpr int RB = MMPDE_NODE_RB;
    EmbedArgs a;
    int rc = embed_args(c, &a);
    if (rc) return rc;
    const int64_t tiles = ceil_div(c.n, 16 * RB);
    MMPDE_REQUIRE(tiles < (int64_t)INT32_MAX);
    const dim3 grid((unsigned)tiles);
    if (c.pk0) hipLaunchKernelGGL((gnn_embed_kernel<true, RB>), grid, dim3(512), 0, st, a);
    else hipLaunchKernelGGL((gnn_embed_kernel<false, RB>), grid, dim3(512), 0, st, a);
    MMPDE_RET_LAUNCH();
    return MMPDE_OK;
}

int launch_embed_stage(const float *u, const float *pos, int64_t n, int64_t seg_n, mmpde_gnn_scales sc,
                       const mmpde_gnn_embed_params *e, const mmpde_gnn_layer_params *l0,
                       const char *pk0, float *rmx_out, float *h_out, float *a_out,
                       float *b_out, hipStream_t st) {
    const EmbedStageCall c{u, pos, n, seg_n, sc, e, l0, pk0, rmx_out, h_out, a_out, b_out};
    return launch_embed_stage(c, st);
}
