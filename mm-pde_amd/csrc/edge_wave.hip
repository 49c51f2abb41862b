// GNN edge stage, F16X3, one wave per SIMD (reference gnn_2d.py:59-63 message
// + PyG aggr='mean', gnn_2d.py:36):
//
//   mean_i = (1/k) sum_e relu(W2 relu(a_i + b_nbr(i,e)) + b2)
//
// with a, b the exact node halves of message_net_1 (layer.hip header).  Every
// wave gathers, splits and multiplies its own neighbour slots: no LDS ring, no
// barrier, no producer / consumer hand-off between waves.
//
// Registers.  The whole message_net_2 operand image (8 column tiles x 4 K
// steps x fp16 hi / lo, 256 registers per lane) is pinned in AGPRs for the
// launch: v_mfma_f32_16x16x32_f16 reads its B operand straight from the
// accumulation registers, while the accumulators, the A operands and every
// VALU value live in VGPRs (this file is built with -amdgpu-mfma-vgpr-form, see
// the Makefile).  One slot (one neighbour of 16 targets) is 96 MFMAs from
// registers; the slot's split VALU (relu(a + b) -> scaled fp16 hi / lo) and its
// relu-sums are the MFMA-gap fillers of the same instruction stream.
//
// Work split: rows form trajectory segments of seg_n rows (layer.hpp
// EdgeSplit), each cut into 16-row tiles; a segment's S = tiles * k neighbour
// slots (slot = one neighbour of one 16-target tile) form one stream, cut into
// U summation units, unit u = slots [u S / U, (u + 1) S / U).  A run is the part
// of a unit inside one tile: its relu-sums accumulate in slot order; the run
// that starts at its tile's first slot stores them to out, a run that starts
// at a unit boundary inside a tile to side[s U + u] (16 x 128), and the node
// stage adds those side blocks in unit order before dividing by the degree.
// So a row's sum is a fixed function of (k, U) and the row's tile position.
// Physical waves: the wpsp waves of segment s (XCD-contiguous ranks s * wpsp
// + j) split its U units as evenly as whole units allow, wave j taking units
// [j U / wpsp, (j + 1) U / wpsp).  A wave never leaves its segment, so its
// U is a function of the segment alone (layer.hpp edge_wave_plan): a
// trajectory's result does not depend on how many trajectories are launched
// beside it (any per-rank shard of a batch sums every row in the same order).
// Split scales: one per target row (layer.hpp row maxima), computed in the
// prologue for every row of the wave's tiles from the node stage's row maxima
// and the row's neighbour list, and kept in LDS: a row's scale depends on the
// row and its neighbours only.
// Deterministic: fixed summation order, no atomics.
#include "common.hpp"
#include "f16x3.hpp"
#include "layer.hpp"

#include <cmath>

namespace {

constexpr int LH = 128;  // hidden width
constexpr int ET = 16;   // targets per tile

// Split placement (body below).  1: every MFMA gap carries at most 8 issue
// cycles of VALU: per pair j, group 2j = [relu-sum | fmas | cvt + relu of pair
// j - 1's hi], group 2j + 1 = [relu-sum | mixlo | mixhi (+ a b-row refill)]
// (v_fma_mix* issue for 8 cycles, tools/ubench/gapcost.hip).  0: the round-2
// placement, cvt + mixlo and mixhi + pk_max (12 cycles each) in one gap.
#ifndef MMPDE_EDGE_PLACE
#define MMPDE_EDGE_PLACE 1
#endif
constexpr bool kPlace8 = MMPDE_EDGE_PLACE == 1;


struct WaveArgs {
    const float *a, *b;
    const int32_t *nbr;
    const int32_t *deg;  // RAGGED: in-degree per target (nullable otherwise)
    int64_t n;
    int k;
    int64_t seg_n;            // rows per segment
    int tps;                  // 16-row tiles per segment
    int64_t S;                // slots per segment = tps * k
    int U;                    // summation units per segment
    int wpsp;                 // waves per segment (<= U)
    const float *b2;          // message_net_2.0 bias
    const char *pk;           // this layer's packed images (W2 at kPkW2)
    const float *rmx;         // row maxima of a, b (layer.hpp)
    const float *rec;         // their range records (nullable: every segment per-row)
    float *out;               // neighbour sums of the units that start a tile
    float *side;              // [G][16][128]: the unit a wave starts inside a tile
    uint64_t *stamps;         // DIAG & 256 only: [G] exit times (100 MHz clock)
};


// Rank of wave-workgroup bid: blocks b and b + 8 share an XCD; ranks number the
// blocks XCD by XCD, so each XCD walks a contiguous share of the slots (speed only).
__device__ __forceinline__ int wave_rank(int bid, int G) {
    const int x = bid & 7, i = bid >> 3;
    const int q = G >> 3, rem = G & 7;
    return x * q + min(x, rem) + i;
}

// Position in the slot stream: tile, neighbour slot e < k, global slot index.
struct SlotCtr {
    int tile, e;
    int64_t pos;
    __device__ void start(int64_t s, int k) {
        pos = s;
        tile = (int)(s / k);
        e = (int)(s - (int64_t)tile * k);
    }
    __device__ void next(int k) {
        ++pos;
        if (++e == k) {
            e = 0;
            ++tile;
        }
    }
};

// s += relu(x), as inline asm so that it keeps its place between the MFMAs
// (plain arithmetic floats to the end of the block in instruction selection).
// Only for x produced by an MFMA at least a few instructions earlier: the
// compiler cannot see this read of an MFMA result (the wave kernel reads
// column tiles six groups after their last MFMA).
__device__ __forceinline__ float relu_acc(float s, float x) {
    float t;
    asm("v_max_f32_e32 %1, 0, %2\n\tv_add_f32_e32 %0, %0, %1" : "+v"(s), "=&v"(t) : "v"(x));
    return s;
}

// A value pinned in AGPRs: the empty asm ties its input to an AGPR output, so
// the compiler places the value there (v_accvgpr_write) and the MFMAs read it
// in place.
__device__ __forceinline__ half8 pin_agpr(half8 v) {
    half8 r;
    asm("; pin %0" : "=a"(r) : "0"(v));
    return r;
}

// DIAG (profiling builds only, tools/ubench; production = 0): bit 0 skips the
// split VALU, bit 1 the relu-sums, bit 2 the b gathers (all wrong values; without
// the relu-sums the compiler drops the MFMAs they would read), bit 5 replaces the relu-sums by empty register sinks
// (MFMAs kept), bit 6 the unit stores likewise, bit 7 skips the a-row reload
// at tile switches (wrong values).
template <bool RAGGED, int DIAG = 0>
__global__ __launch_bounds__(64, 1) void gnn_edge_wave_kernel(WaveArgs p) {
    const int lane = threadIdx.x, r = lane & 15, g = lane >> 4;
    const int k = p.k;
    const int64_t nmax = p.n - 1;
    const int rank = wave_rank(blockIdx.x, gridDim.x);
    const int wpsp = p.wpsp;
    const int seg = rank / wpsp, jw = rank - seg * wpsp;
    const int u_begin = (int)((int64_t)jw * p.U / wpsp), u_end = (int)((int64_t)(jw + 1) * p.U / wpsp);
    int u_next = u_begin + 1;  // the next unit to start
    const int64_t s0 = (int64_t)u_begin * p.S / p.U, s1 = (int64_t)u_end * p.S / p.U;
    if (s0 >= s1) return;
    // slot where unit u_next starts (s1 past the wave's last unit)
    int64_t ub = u_next < u_end ? (int64_t)u_next * p.S / p.U : s1;
    // rows of this wave's segment: base + local row, local rows <= last
    const int64_t base = (int64_t)seg * p.seg_n;
    const int last = (int)p.seg_n - 1;
    // destination of the run being computed: -1 = out (it starts its tile),
    // else the side block of the unit it starts
    int run_side = s0 % k ? seg * p.U + u_begin : -1;
    // F16X3 operand piece i of this lane: k = 32 (i >> 1) + 8 g + 4 (i & 1) .. + 3
    auto piece = [&](int i) { return 32 * (i >> 1) + 8 * g + 4 * (i & 1); };
    auto unit_tile = [&](const SlotCtr &c) { return min(c.tile, p.tps - 1); };
    // global row of local row q of this segment (clamped to the segment)
    auto grow = [&](int q) { return base + min(q, last); };
    // every prefetch issues the same loads (clamped past the end)
    auto src_of = [&](const SlotCtr &c) -> uint32_t {
        const int64_t row = grow(unit_tile(c) * ET + r);
        return (uint32_t)p.nbr[row * k + c.e];
    };
    auto gather = [&](float4 *dst, uint32_t src) {
        const float *br = p.b + (int64_t)min(src, (uint32_t)nmax) * LH;  // clamped: a malformed table must not fault
#pragma unroll
        for (int i = 0; i < 8; ++i) dst[i] = *(const float4 *)(br + piece(i));
    };
    // The slot stream is software-pipelined over four positions:
    //   cC  slot q    its 96 MFMAs run in body q (operands hw/lw built in body q-1)
    //   cS  slot q+1  split in body q, between those MFMAs (b rows in X)
    //   cG  slot q+2  b rows gathered in body q, piece i into X[i] as soon as
    //                 the split has consumed slot q+1's piece i (one buffer)
    //   cI  slot q+3  neighbour index loaded in body q
    // and the relu-sums of slot q's column tiles trail its MFMAs by six groups
    // (tiles 6 and 7 finish in body q+1), so the VALU work of three slots is
    // spread across one slot's MFMA stream.
    SlotCtr cC, cS, cI;
    cC.start(s0, k);
    cS = cC;
    cS.next(k);
    cI = cS;
    cI.next(k);
    cI.next(k);
    // Split scales of the rows of this wave's tiles (at most kWaveTiles,
    // edge_wave_plan), |relu(a_i + b_j)| s_i < 2^11 (split8_relu_rtz), into LDS.
    // A segment whose range records (layer.hpp) show a narrow range -- every
    // row's bound within 2^12 of the segment's -- gives every row the
    // segment's scale (no neighbour gathers; the records go out before the W2
    // image).  Otherwise each lane takes one row of four tiles (a pass):
    // M_i = max|a_i| + max_e max|b_nbr(i,e)| from the row maxima, the index
    // loads and then the gathers all in flight together.
    constexpr int KU = 36;  // neighbour slots loaded unrolled (more: one by one)
    __shared__ float rs_lds[kWaveTiles * ET];
    const int t_first = (int)(s0 / k), t_last = min((int)((s1 - 1) / k), p.tps - 1);
    const uint32_t *rmxb = (const uint32_t *)p.rmx;
    const uint32_t nmaxu = (uint32_t)nmax;
    auto pass_row = [&](int tb) { return base + min(min(tb + g, t_last) * ET + r, last); };
    auto pass_scale = [&](int tb) {
        const int64_t row = pass_row(tb);
        const int kk = RAGGED ? max(min(p.deg[row], k), 1) : k;
        uint32_t id[KU], v[KU];
#pragma unroll
        for (int e = 0; e < KU; ++e) id[e] = (uint32_t)p.nbr[row * k + min(e, kk - 1)];
        const float ma = p.rmx[2 * row];
#pragma unroll
        for (int e = 0; e < KU; ++e) v[e] = rmxb[2 * (uint64_t)min(id[e], nmaxu) + 1];
        uint32_t m = 0;
#pragma unroll
        for (int e = 0; e < KU; ++e) m = max(m, v[e]);
        for (int e = KU; e < kk; ++e) m = max(m, rmxb[2 * (uint64_t)min((uint32_t)p.nbr[row * k + e], nmaxu) + 1]);
        if (tb + g <= t_last) rs_lds[(tb + g - t_first) * ET + r] = row_split_scale(ma + __uint_as_float(m));
    };
    // slot 0's neighbour index and a rows, then the segment's range records,
    // all before the W2 image; slot 0's b rows go out after it
    const int atile0 = unit_tile(cC);
    const uint32_t src0 = src_of(cC);
    float4 araw[8];
    {
        const float *ar = p.a + grow(atile0 * ET + r) * LH;
#pragma unroll
        for (int i = 0; i < 8; ++i) araw[i] = *(const float4 *)(ar + piece(i));
    }
    float2 seg_ml = make_float2(0.0f, 0.0f);
    if (p.rec) seg_ml = segment_stats(p.rec, p.seg_n, seg);
    __builtin_amdgcn_sched_barrier(0);  // these loads issue before the image's
    // message_net_2: B operands (AGPRs), accumulator start (bias in the column
    // scale, times the row scales of the MFMA slot's tile), column unscale
    half8 wh[8][4], wl[8][4];
    float bb0[8], inv[8];
    f32x4 bias[8];
    {
        const char *img = p.pk + kPkW2;
#pragma unroll
        for (int c = 0; c < 8; ++c) {
#pragma unroll
            for (int s = 0; s < 4; ++s) {
                wh[c][s] = pin_agpr(bfrag(img, 4, c, s, 0, lane));
                wl[c][s] = pin_agpr(bfrag(img, 4, c, s, 1, lane));
            }
            const float sw = ((const float *)(img + 65536))[16 * c + r];
            bb0[c] = p.b2[16 * c + r] * sw;
            inv[c] = pow2_inv(sw);
        }
    }
    float4 bx[8];
    gather(bx, src0);
    // narrow: L_seg >= 2^-12 M_seg (layer.hpp range records; an infinite or NaN
    // M_seg never is, and takes the per-row path)
    const bool narrow = p.rec && seg_ml.y >= 0x1p-12f * seg_ml.x;
    if (narrow) {
        const float ss = row_split_scale(seg_ml.x);
        for (int i = lane; i < (t_last - t_first + 1) * ET; i += 64) rs_lds[i] = ss;
    } else {
        for (int tb = t_first; tb <= t_last; tb += 4) pass_scale(tb);
    }
    __syncthreads();  // one wave: the LDS writes of every lane before any read
    // LDS slot of a tile's row scales (tiles past the wave's last, which only a
    // prefetch past the end touches, read the last one's)
    auto rs_of = [&](int tile) { return &rs_lds[(min(tile, t_last) - t_first) * ET]; };
    // the accumulator start of a tile's slots: rows 4 g + t of this lane
    auto set_bias = [&](int tile) {
        const float4 s4 = *(const float4 *)(rs_of(tile) + 4 * g);
#pragma unroll
        for (int c = 0; c < 8; ++c) bias[c] = (f32x4){bb0[c] * s4.x, bb0[c] * s4.y, bb0[c] * s4.z, bb0[c] * s4.w};
    };
    float4 av[8];  // a rows of the split slot's tile (scaled), this lane's pieces
    float sc = 1.0f;  // split scale of this lane's row (r) of the split slot's tile
    auto load_a = [&](int tile) {
        const float *ar = p.a + grow(tile * ET + r) * LH;
        float4 v[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) v[i] = *(const float4 *)(ar + piece(i));
        sc = rs_of(tile)[r];
#pragma unroll
        for (int i = 0; i < 8; ++i) av[i] = make_float4(v[i].x * sc, v[i].y * sc, v[i].z * sc, v[i].w * sc);
    };
    auto load_deg = [&](int *d, const SlotCtr &c) {
        const int row0 = unit_tile(c) * ET;
#pragma unroll
        for (int t = 0; t < 4; ++t) d[t] = p.deg[grow(row0 + 4 * g + t)];
    };
    // pair j (0..15) of a slot's A operand: K step j >> 2, values 2 (j & 3), +1
    // of that step (x of piece 2 (j >> 2) + ((j >> 1) & 1), components
    // 2 (j & 1), +1), as relu(a + b) scaled, split into fp16 hi / lo words.
    // Everything it reads is in registers: a memory read waited on inside the
    // MFMA stream would stall the (in-order) wave.
    auto a_piece = [&](int j) { return 2 * (j >> 2) + ((j >> 1) & 1); };
    auto split_pair = [&](int j, const float4 *X, uint32_t (*nh)[4], uint32_t (*nl)[4]) {
        const float4 &ap = av[a_piece(j)];
        const float4 &bb = X[a_piece(j)];
        const float x0 = (j & 1) ? fmaf(bb.z, sc, ap.z) : fmaf(bb.x, sc, ap.x);
        const float x1 = (j & 1) ? fmaf(bb.w, sc, ap.w) : fmaf(bb.y, sc, ap.y);
        split2_relu_rtz(x0, x1, nh[j >> 2][j & 3], nl[j >> 2][j & 3]);
    };
    f32x4 S[8];
    int dg[4] = {k, k, k, k}, dg_prev[4] = {k, k, k, k};
    uint32_t hA[4][4], lA[4][4], hB[4][4], lB[4][4];
    int atile = atile0;
    sc = rs_of(atile)[r];
#pragma unroll
    for (int i = 0; i < 8; ++i) av[i] = make_float4(araw[i].x * sc, araw[i].y * sc, araw[i].z * sc, araw[i].w * sc);
    set_bias(atile);
    if (RAGGED) load_deg(dg, cC);
#pragma unroll
    for (int j = 0; j < 16; ++j) split_pair(j, bx, hA, lA);
    gather(bx, src_of(cS));
    uint32_t i_next;  // neighbour index of the slot gathered next (slot 2)
    {
        SlotCtr c2 = cS;
        c2.next(k);
        i_next = src_of(c2);
    }
#pragma unroll
    for (int c = 0; c < 8; ++c) S[c] = (f32x4){0.0f, 0.0f, 0.0f, 0.0f};
    // column tiles 6, 7 of the previous slot, summed at the start of the next
    // body (before the first slot: relu(-big) = 0 adds nothing)
    f32x4 acc6 = (f32x4){-3.0e38f, -3.0e38f, -3.0e38f, -3.0e38f}, acc7 = acc6;
    int e_prev = 0, row0_prev = 0;
    int side_prev = -1;
    bool close_prev = false;  // the previous slot was its unit's last: write after its deferred sums
    auto relu_add = [&](f32x4 &Sc, float x, int t, int e, const int *d) {
        float v = __builtin_amdgcn_fmed3f(x, 0.0f, 3.402823466e38f);  // relu
        if (RAGGED) v = e < d[t] ? v : 0.0f;
        Sc[t] += v;
    };
    // the finished unit's sums, unscaled (by the column and row scales: a
    // power-of-two multiply, exact), to out (rows of the tile) or to
    // side[rank].  The node stage adds the side buffers and divides by the
    // degree (PyG mean = sum / count).  Stores are unconditional unless the
    // tile runs past the segment (wave-uniform test), at immediate offsets from
    // one base per lane.  row0: local row.
    auto write_unit = [&](int row0, int side_idx) {
        const bool to_side = side_idx >= 0;
        if (DIAG & 64) {  // no stores: keep the sums alive only
#pragma unroll
            for (int c = 0; c < 8; ++c) asm volatile("" ::"v"(S[c]));
            return;
        }
        const float4 s4 = *(const float4 *)(rs_of(row0 / ET) + 4 * g);
        const float irs[4] = {pow2_inv(s4.x), pow2_inv(s4.y), pow2_inv(s4.z), pow2_inv(s4.w)};
        float *o = (to_side ? p.side + (int64_t)side_idx * ET * LH : p.out + (base + row0) * LH) + 4 * g * LH + r;
        if (to_side || row0 + ET <= last + 1) {
#pragma unroll
            for (int c = 0; c < 8; ++c)
#pragma unroll
                for (int t = 0; t < 4; ++t) o[t * LH + 16 * c] = S[c][t] * (inv[c] * irs[t]);
        } else {
#pragma unroll
            for (int c = 0; c < 8; ++c)
#pragma unroll
                for (int t = 0; t < 4; ++t)
                    if (row0 + 4 * g + t <= last) o[t * LH + 16 * c] = S[c][t] * (inv[c] * irs[t]);
        }
    };
    auto body = [&](float4 *X, uint32_t (*h)[4], uint32_t (*l)[4], uint32_t (*nh)[4], uint32_t (*nl)[4]) {
        // memory: index of slot q+3 now, b rows of slot q+2 piece by piece below
        const uint32_t i_after = src_of(cI);
        cI.next(k);
        const float *brow = p.b + (int64_t)min(i_next, (uint32_t)nmax) * LH;  // clamped: a malformed table must not fault
        i_next = i_after;
        const int e = cC.e;
        {   // a rows of the split slot's tile
            const int st = unit_tile(cS);
            if (st != atile) {
                if (!(DIAG & 128)) load_a(st);
                atile = st;
            }
        }
        // Per-MFMA placement (kPlace8): every MFMA gap carries at most 8 issue
        // cycles of VALU beside the MFMA's 8 of 16, pinned by sched_barriers on
        // both sides of each MFMA.  Group G = 4 c + s (the 3 MFMAs of column
        // tile c, K step s): gap 0 the relu-sum of value G (max + add); split
        // pair j = G >> 1 over its two groups: G even gap 1 its two fmas
        // (relu(a + b) input), gap 2 cvt_pkrtz (hi) + the relu of pair j - 1's
        // hi; G odd gap 1 mixlo, gap 2 mixhi (the v_fma_mix* issue for 8 cycles
        // each) and at G = 4 p + 3 the refill of piece p, whose last pair
        // (4 p + 2) has read it.  The relu-sums trail their tile's MFMAs by six
        // groups (groups 0-5: the previous slot's tiles 6 and 7).  Measured
        // (tools/ubench/gapcost.hip: 2 v_fma_mix in one gap cost 1.48x an MFMA,
        // cvt + mix 1.32x, any 8-cycle pair 1.03-1.07x): 105.9 vs 111.8 us per
        // launch for the round-2 placement (kPlace8 = 0: cvt + mixlo and
        // mixhi + pk_max in one gap each).
        f32x4 acc[8];
        float xs0 = 0.0f, xs1 = 0.0f;
#pragma unroll
        for (int c = 0; c < 8; ++c) {
            acc[c] = bias[c];
#pragma unroll
            for (int s = 0; s < 4; ++s) {
                const half8 ah = __builtin_bit_cast(half8, h[s]), al = __builtin_bit_cast(half8, l[s]);
                const int G = 4 * c + s, j = G >> 1;
                acc[c] = mfma_f16(ah, wh[c][s], acc[c]);
                if (kPlace8) __builtin_amdgcn_sched_barrier(0);  // the gap's unit after its MFMA
                {
                    f32x4 &Sc = G >= 6 ? S[(G - 6) >> 2] : (G < 2 ? S[6] : S[7]);
                    const int t = G >= 6 ? (G - 6) & 3 : (G < 2 ? G + 2 : G - 2);
                    const float x = G >= 6 ? acc[(G - 6) >> 2][t] : (G < 2 ? acc6[t] : acc7[t]);
                    if (RAGGED) relu_add(Sc, x, t, G >= 6 ? e : e_prev, G >= 6 ? dg : dg_prev);
                    else if (DIAG & 32) asm volatile("" ::"v"(x));  // MFMAs kept, no VALU
                    else if (!(DIAG & 2)) Sc[t] = relu_acc(Sc[t], x);
                }
                __builtin_amdgcn_sched_barrier(0);
                acc[c] = mfma_f16(ah, wl[c][s], acc[c]);
                if (kPlace8) __builtin_amdgcn_sched_barrier(0);  // the gap's unit after its MFMA
                if (!(DIAG & 1)) {
                    if ((G & 1) == 0) {
                        const float4 &ap = av[a_piece(j)];
                        const float4 &bb = X[a_piece(j)];
                        xs0 = (j & 1) ? fmaf(bb.z, sc, ap.z) : fmaf(bb.x, sc, ap.x);
                        xs1 = (j & 1) ? fmaf(bb.w, sc, ap.w) : fmaf(bb.y, sc, ap.y);
                    } else if (kPlace8) {
                        split_l(xs0, nh[j >> 2][j & 3], nl[j >> 2][j & 3]);
                    } else {
                        split2_relu_rtz_b(xs1, nh[j >> 2][j & 3], nl[j >> 2][j & 3]);
                    }
                }
                __builtin_amdgcn_sched_barrier(0);
                acc[c] = mfma_f16(al, wh[c][s], acc[c]);
                if (kPlace8) __builtin_amdgcn_sched_barrier(0);  // the gap's unit after its MFMA
                if ((G & 1) == 0) {
                    if (DIAG & 1) {
                    } else if (kPlace8) {
                        split_c(xs0, xs1, nh[j >> 2][j & 3]);
                        // relu of the previous pair's hi (pair 15 of the split
                        // made in the previous body: this body's operand h, first
                        // read by group 3; applying it again to the prologue's
                        // split is harmless, relu is idempotent)
                        if (j == 0) split_p(h[3][3]);
                        else split_p(nh[(j - 1) >> 2][(j - 1) & 3]);
                    } else {
                        split2_relu_rtz_a(xs0, xs1, nh[j >> 2][j & 3], nl[j >> 2][j & 3]);
                    }
                } else {
                    if (kPlace8 && !(DIAG & 1)) split_h(xs1, nh[j >> 2][j & 3], nl[j >> 2][j & 3]);
                    if ((G & 3) == 3 && !(DIAG & 4)) X[G >> 2] = *(const float4 *)(brow + piece(G >> 2));
                }
                __builtin_amdgcn_sched_barrier(0);
                if (G == 5 && close_prev) {  // the previous unit is complete: write, restart
                    write_unit(row0_prev, side_prev);
#pragma unroll
                    for (int c2 = 0; c2 < 8; ++c2) S[c2] = (f32x4){0.0f, 0.0f, 0.0f, 0.0f};
                }
            }
        }
        acc6 = acc[6];
        acc7 = acc[7];
        e_prev = e;
        // the run closes at its tile's end, at a unit boundary and at the end
        const bool new_unit = cC.pos + 1 == ub;
        close_prev = cC.e + 1 == k || cC.pos + 1 == s1 || new_unit;
        row0_prev = unit_tile(cC) * ET;
        side_prev = run_side;
        if (RAGGED) {
#pragma unroll
            for (int t = 0; t < 4; ++t) dg_prev[t] = dg[t];
        }
        cC.next(k);
        cS.next(k);
        if (cC.e == 0) set_bias(unit_tile(cC));  // the next MFMA slot opens a tile
        if (close_prev) {  // the next run starts at cC
            run_side = new_unit && cC.e != 0 ? seg * p.U + u_next : -1;
            if (new_unit) {
                ++u_next;
                ub = u_next < u_end ? (int64_t)u_next * p.S / p.U : s1;
            }
        }
        if (RAGGED && close_prev) load_deg(dg, cC);
    };
    // (the S reset of a unit's first slot happens at group 5 of its body, after
    // the previous unit's deferred sums and write; relu-sums of the slot start
    // at group 6.  The first slot starts from S = 0.)
    for (;;) {
        body(bx, hA, lA, hB, lB);
        if (cC.pos >= s1) break;
        body(bx, hB, lB, hA, lA);
        if (cC.pos >= s1) break;
    }
    // the last slot's deferred sums, then its unit (always the last slot of one)
#pragma unroll
    for (int t = 2; t < 4; ++t) relu_add(S[6], acc6[t], t, e_prev, dg_prev);
#pragma unroll
    for (int t = 0; t < 4; ++t) relu_add(S[7], acc7[t], t, e_prev, dg_prev);
    write_unit(row0_prev, side_prev);
    if (DIAG & 256) {  // profiling builds: the wave's exit time (vector store)
        const uint64_t t = __builtin_amdgcn_s_memrealtime();
        if (lane == 0) p.stamps[blockIdx.x] = t;
    }
}

}  // namespace

// Summation units and waves of one launch (layer.hpp edge_wave_plan).
EdgePlan edge_wave_plan(int64_t nseg, int64_t S_seg, int k, int cus, int64_t side_cap) {
    EdgePlan pl;
    // U: the power of two that makes units of 22..44 slots (cylinder: 128
    // units of 43 slots), capped by the segment's slots and its share of the
    // side blocks (3 seg_n / 16 in the standard workspace): a function of the
    // segment alone
    int64_t U = 1;
    while (U * 2 * 22 <= S_seg) U *= 2;
    // a segment that fills the chip alone (>= 16384 slots: the 96 x 96 Burgers
    // grid, configs[0]) takes units of >= 11 slots, up to 1024 of them, so one
    // trajectory still runs one wave per SIMD (still a function of the segment)
    if (S_seg >= 16384)
        while (U < 1024 && U * 2 * 11 <= S_seg) U *= 2;
    const int64_t cap = S_seg < side_cap / nseg ? S_seg : side_cap / nseg;
    if (U > cap) U = cap < 1 ? 1 : cap;
    // waves per segment: one wave per SIMD over the launch, at most one per unit
    int64_t w = 4 * (int64_t)cus / nseg;
    w = w < 1 ? 1 : (w > U ? U : w);
    // ... and more (queued behind the first wave of a SIMD) while a wave would
    // span more than kWaveTiles tiles: its row scales live in LDS.  Which wave
    // runs a unit does not change any sum.
    const int64_t spu = (S_seg + U - 1) / U;  // slots per unit, at most
    auto tiles_of = [&](int64_t ww) { return (((U + ww - 1) / ww) * spu + k - 1) / k + 1; };
    while (w < U && tiles_of(w) > kWaveTiles) w = 2 * w < U ? 2 * w : U;
    pl.U = (int)U;
    pl.wpsp = tiles_of(w) <= kWaveTiles ? (int)w : 0;  // 0: no valid plan (units too long)
    pl.waves = nseg * w;
    return pl;
}

namespace {
// Kernel arguments and grid of one launch (slot split of layer.hpp EdgeSplit).
int edge_wave_setup(const float *a, const float *b, const int32_t *nbr, const int32_t *deg, int64_t n,
                    int k, int64_t seg_n, const float *msg2_b, const char *pk, const float *rmx, bool rng,
                    float *out, float *side, int64_t side_cap, int cus, WaveArgs *w, EdgeSplit *split) {
    seg_n = effective_seg(n, seg_n);
    const int64_t nseg = n / seg_n, tps = (seg_n + ET - 1) / ET, S = tps * k;
    if (!(tps < (int64_t)INT32_MAX && S < ((int64_t)1 << 40) && side_cap >= nseg)) return 0;
    const EdgePlan pl = edge_wave_plan(nseg, S, k, cus, side_cap);
    if (pl.wpsp < 1 || pl.waves > (int64_t)INT32_MAX || nseg * pl.U > (int64_t)INT32_MAX) return 0;
    *w = WaveArgs{a, b, nbr, deg, n, k, seg_n, (int)tps, S, pl.U, pl.wpsp, msg2_b, pk, rmx,
                  rng ? rmx + row_max_floats(n) : nullptr, out, side, nullptr};
    *split = EdgeSplit{side, S, pl.U, k, seg_n};
    return (int)pl.waves;
}
}  // namespace

// Profiling aid (tools/ubench): the non-ragged kernel with DIAG bits, one wave
// per SIMD, one segment of n rows; side = a [4 cus][16][128] buffer.
int launch_edge_wave_diag(const float *a, const float *b, const int32_t *nbr, int64_t n, int k,
                          const float *msg2_b, const char *pk, const float *rmx, float *out,
                          float *side, int cus, int diag, hipStream_t st) {
    WaveArgs w;
    EdgeSplit split;
    const int grid = edge_wave_setup(a, b, nbr, nullptr, n, k, n, msg2_b, pk, rmx, false, out, side,
                                     4 * (int64_t)cus, cus, &w, &split);
    MMPDE_REQUIRE(grid > 0);
#define MMPDE_DIAG(D) \
    case D: hipLaunchKernelGGL((gnn_edge_wave_kernel<false, D>), dim3(grid), dim3(64), 0, st, w); break
    switch (diag) {
        MMPDE_DIAG(1);
        MMPDE_DIAG(2);
        MMPDE_DIAG(3);
        MMPDE_DIAG(4);
        MMPDE_DIAG(7);
        MMPDE_DIAG(32);
        MMPDE_DIAG(33);
        MMPDE_DIAG(36);
        MMPDE_DIAG(64);
        MMPDE_DIAG(97);
        MMPDE_DIAG(128);
    default: hipLaunchKernelGGL((gnn_edge_wave_kernel<false, 0>), dim3(grid), dim3(64), 0, st, w); break;
    }
#undef MMPDE_DIAG
    MMPDE_RET_LAUNCH();
    return MMPDE_OK;
}

// Profiling aid (tools/ubench/edge_exit): the production launch (segments of
// seg_n rows, range records) of the kernel built with DIAG bit 8 (256), which
// stores each wave's exit time (100 MHz clock) to stamps[block] (an entry stamp
// as well made that build spill 48 VGPRs); returns the launch's wave count or a
// negative status.
int launch_edge_wave_exit_stamps(const float *a, const float *b, const int32_t *nbr, int64_t n, int k,
                                 int64_t seg_n, const float *msg2_b, const char *pk, const float *rmx,
                                 float *out, float *side, int64_t side_cap, int cus, uint64_t *stamps,
                                 hipStream_t st) {
    WaveArgs w;
    EdgeSplit split;
    const int grid = edge_wave_setup(a, b, nbr, nullptr, n, k, seg_n, msg2_b, pk, rmx, true, out, side, side_cap,
                                     cus, &w, &split);
    if (grid <= 0) return -1;
    w.stamps = stamps;
    if (stamps) hipLaunchKernelGGL((gnn_edge_wave_kernel<false, 256>), dim3(grid), dim3(64), 0, st, w);
    else hipLaunchKernelGGL((gnn_edge_wave_kernel<false, 0>), dim3(grid), dim3(64), 0, st, w);
    return hipGetLastError() == hipSuccess ? grid : -2;
}

int launch_edge_wave(const float *a, const float *b, const int32_t *nbr, const int32_t *deg, int64_t n,
                     int k, int64_t seg_n, const float *msg2_b, const char *pk, const float *rmx, bool rng,
                     float *out, float *side, int64_t side_cap, int cus, EdgeSplit *split, hipStream_t st) {
    MMPDE_REQUIRE(a && b && nbr && msg2_b && pk && rmx && out && side && split && n > 0 && k > 0);
    WaveArgs w;
    const int grid = edge_wave_setup(a, b, nbr, deg, n, k, seg_n, msg2_b, pk, rmx, rng, out, side, side_cap,
                                     cus, &w, split);
    MMPDE_REQUIRE(grid > 0);
    if (deg) hipLaunchKernelGGL((gnn_edge_wave_kernel<true>), dim3(grid), dim3(64), 0, st, w);
    else hipLaunchKernelGGL((gnn_edge_wave_kernel<false>), dim3(grid), dim3(64), 0, st, w);
    MMPDE_RET_LAUNCH();
    return MMPDE_OK;
}
