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
// Work unit = (16-target tile, part): part p of `parts` covers slots
// [p k / parts, (p + 1) k / parts) of the tile (parts > 1 balances the grid
// when tiles per wave are few).  Each wave walks a contiguous, XCD-local range
// of units as one slot stream.  Part q writes its slots' sum to out + q *
// part_stride; launch_node_stage adds the parts in part order and divides by
// the degree.  Deterministic: fixed summation order, no atomics.
#include "common.hpp"
#include "f16x3.hpp"
#include "layer.hpp"

#include <cmath>

namespace {

constexpr int LH = 128;  // hidden width
constexpr int ET = 16;   // targets per tile

struct WaveArgs {
    const float *a, *b;
    const int32_t *nbr;
    const int32_t *deg;  // RAGGED: in-degree per target (nullable otherwise)
    int64_t n;
    int k, ntiles, parts;
    int64_t part_stride;
    const float *b2;          // message_net_2.0 bias
    const char *pk;           // this layer's packed images (W2 at kPkW2)
    const uint32_t *amax_in;  // range slots of a, b
    float *out;               // mean, or the partial sums
};

// Contiguous unit range [u0, u0 + cnt) of wave-workgroup bid: blocks b and b + 8
// share an XCD, which owns a contiguous share of the units (speed only).
__device__ __forceinline__ void unit_range(int bid, int G, int nunits, int &u0, int &cnt) {
    const int x = bid & 7, i = bid >> 3;
    const int q = G >> 3, rem = G & 7;
    const int nW = q + (x < rem ? 1 : 0);
    const int cum = x * q + min(x, rem);
    const int lo = (int)((int64_t)nunits * cum / G);
    const int hi = (int)((int64_t)nunits * (cum + nW) / G);
    const int len = hi - lo;
    u0 = lo + (int)((int64_t)len * i / nW);
    cnt = lo + (int)((int64_t)len * (i + 1) / nW) - u0;
}

// Position in the slot stream: unit u (relative to u0) and slot e of that
// unit's range [e0, e1).
template <int PARTS>
struct SlotCtr {
    int u, e, e1;
    __device__ void start(int u0, int uu, int k) {
        u = uu;
        const int part = (u0 + uu) % PARTS;
        e = part * k / PARTS;
        e1 = (part + 1) * k / PARTS;
    }
    __device__ void next(int u0, int k) {
        if (++e == e1) start(u0, u + 1, k);
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
template <bool RAGGED, int PARTS, int DIAG = 0>
__global__ __launch_bounds__(64, 1) void gnn_edge_wave_kernel(WaveArgs p) {
    const int lane = threadIdx.x, r = lane & 15, g = lane >> 4;
    const int k = p.k;
    const int64_t nmax = p.n - 1;
    int u0, nu;
    unit_range(blockIdx.x, gridDim.x, p.ntiles * PARTS, u0, nu);
    if (nu <= 0) return;
    // |a + b| <= max|a| + max|b|, scaled below 2^11 (split8_relu_rtz)
    const float sc = 0.125f * split_scale(amax_read(p.amax_in) + amax_read(p.amax_in + kAmaxShards));
    // message_net_2: B operands (AGPRs), accumulator start (bias, scaled), unscale
    half8 wh[8][4], wl[8][4];
    float bias[8], inv[8];
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
            bias[c] = p.b2[16 * c + r] * sw * sc;
            inv[c] = pow2_inv(sw) * pow2_inv(sc);
        }
    }
    // F16X3 operand piece i of this lane: k = 32 (i >> 1) + 8 g + 4 (i & 1) .. + 3
    auto piece = [&](int i) { return 32 * (i >> 1) + 8 * g + 4 * (i & 1); };
    auto unit_tile = [&](const SlotCtr<PARTS> &c) { return min((u0 + c.u) / PARTS, p.ntiles - 1); };
    // every prefetch issues the same loads (clamped past the end)
    auto src_of = [&](const SlotCtr<PARTS> &c) -> uint32_t {
        const int64_t row = min((int64_t)unit_tile(c) * ET + r, nmax);
        return (uint32_t)p.nbr[row * k + min(c.e, k - 1)];
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
    SlotCtr<PARTS> cC, cS, cG, cI;
    cC.start(u0, 0, k);
    cS = cC;
    cS.next(u0, k);
    cG = cS;
    cG.next(u0, k);
    cI = cG;
    cI.next(u0, k);
    float4 av[8];  // a rows of the split slot's tile (scaled), this lane's pieces
    auto load_a = [&](int tile) {
        const float *ar = p.a + min((int64_t)tile * ET + r, nmax) * LH;
        float4 v[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) v[i] = *(const float4 *)(ar + piece(i));
#pragma unroll
        for (int i = 0; i < 8; ++i) av[i] = make_float4(v[i].x * sc, v[i].y * sc, v[i].z * sc, v[i].w * sc);
    };
    auto load_deg = [&](int *d, const SlotCtr<PARTS> &c) {
        const int64_t row0 = (int64_t)unit_tile(c) * ET;
#pragma unroll
        for (int t = 0; t < 4; ++t) d[t] = p.deg[min(row0 + 4 * g + t, nmax)];
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
    float4 bx[8];
    int atile = unit_tile(cC);
    load_a(atile);
    if (RAGGED) load_deg(dg, cC);
    gather(bx, src_of(cC));
#pragma unroll
    for (int j = 0; j < 16; ++j) split_pair(j, bx, hA, lA);
    gather(bx, src_of(cS));
    uint32_t i_next = src_of(cG);  // neighbour index of the slot gathered next
#pragma unroll
    for (int c = 0; c < 8; ++c) S[c] = (f32x4){0.0f, 0.0f, 0.0f, 0.0f};
    // column tiles 6, 7 of the previous slot, summed at the start of the next
    // body (before the first slot: relu(-big) = 0 adds nothing)
    f32x4 acc6 = (f32x4){-3.0e38f, -3.0e38f, -3.0e38f, -3.0e38f}, acc7 = acc6;
    int e_prev = 0, row0_prev = 0, part_prev = 0;
    bool close_prev = false;  // the previous slot was its unit's last: write after its deferred sums
    auto relu_add = [&](f32x4 &Sc, float x, int t, int e, const int *d) {
        float v = __builtin_amdgcn_fmed3f(x, 0.0f, 3.402823466e38f);  // relu
        if (RAGGED) v = e < d[t] ? v : 0.0f;
        Sc[t] += v;
    };
    // the finished unit's sums, unscaled (a power-of-two multiply: exact).  The
    // node stage adds the parts and divides by the degree (PyG mean = sum / count).
    // Stores are unconditional unless the tile runs past n (wave-uniform test),
    // at immediate offsets from one base per lane.
    auto write_unit = [&](int64_t row0, int part) {
        if (DIAG & 64) {  // no stores: keep the sums alive only
#pragma unroll
            for (int c = 0; c < 8; ++c) asm volatile("" ::"v"(S[c]));
            return;
        }
        float *o = p.out + part * p.part_stride + (row0 + 4 * g) * LH + r;
        if (row0 + ET <= p.n) {
#pragma unroll
            for (int c = 0; c < 8; ++c)
#pragma unroll
                for (int t = 0; t < 4; ++t) o[t * LH + 16 * c] = S[c][t] * inv[c];
        } else {
#pragma unroll
            for (int c = 0; c < 8; ++c)
#pragma unroll
                for (int t = 0; t < 4; ++t)
                    if (row0 + 4 * g + t < p.n) o[t * LH + 16 * c] = S[c][t] * inv[c];
        }
    };
    auto body = [&](float4 *X, uint32_t (*h)[4], uint32_t (*l)[4], uint32_t (*nh)[4], uint32_t (*nl)[4]) {
        // memory: index of slot q+3 now, b rows of slot q+2 piece by piece below
        const uint32_t i_after = src_of(cI);
        cI.next(u0, k);
        const float *brow = p.b + (int64_t)min(i_next, (uint32_t)nmax) * LH;  // clamped: a malformed table must not fault
        cG.next(u0, k);
        i_next = i_after;
        const int e = cC.e;
        {   // a rows of the split slot's tile
            const int st = unit_tile(cS);
            if (st != atile) {
                if (!(DIAG & 128)) load_a(st);
                atile = st;
            }
        }
        // Per-MFMA placement: every MFMA gap carries at most one 2-instruction
        // VALU unit (8 issue cycles beside the MFMA's 8 of 16), pinned by
        // sched_barriers.  Group G = 4 c + s (the 3 MFMAs of column tile c, K
        // step s): gap 0 the relu-sum of value G, gaps 1 / 2 split pair G >> 1
        // (G even: its two fmas, then cvt_pkrtz + mixlo; G odd: mixhi + pk_max,
        // then at G = 4 p + 3 the refill of piece p, whose last pair (4 p + 2)
        // has read it).  The relu-sums trail their tile's MFMAs by six groups
        // (groups 0-5: the previous slot's tiles 6 and 7).
        f32x4 acc[8];
        float xs0 = 0.0f, xs1 = 0.0f;
#pragma unroll
        for (int c = 0; c < 8; ++c) {
            acc[c] = (f32x4){bias[c], bias[c], bias[c], bias[c]};
#pragma unroll
            for (int s = 0; s < 4; ++s) {
                const half8 ah = __builtin_bit_cast(half8, h[s]), al = __builtin_bit_cast(half8, l[s]);
                const int G = 4 * c + s, j = G >> 1;
                acc[c] = mfma_f16(ah, wh[c][s], acc[c]);
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
                if (!(DIAG & 1)) {
                    if ((G & 1) == 0) {
                        const float4 &ap = av[a_piece(j)];
                        const float4 &bb = X[a_piece(j)];
                        xs0 = (j & 1) ? fmaf(bb.z, sc, ap.z) : fmaf(bb.x, sc, ap.x);
                        xs1 = (j & 1) ? fmaf(bb.w, sc, ap.w) : fmaf(bb.y, sc, ap.y);
                    } else {
                        split2_relu_rtz_b(xs1, nh[j >> 2][j & 3], nl[j >> 2][j & 3]);
                    }
                }
                __builtin_amdgcn_sched_barrier(0);
                acc[c] = mfma_f16(al, wh[c][s], acc[c]);
                if ((G & 1) == 0) {
                    if (!(DIAG & 1)) split2_relu_rtz_a(xs0, xs1, nh[j >> 2][j & 3], nl[j >> 2][j & 3]);
                } else if ((G & 3) == 3 && !(DIAG & 4)) {
                    X[G >> 2] = *(const float4 *)(brow + piece(G >> 2));
                }
                __builtin_amdgcn_sched_barrier(0);
                if (G == 5 && close_prev) {  // the previous unit is complete: write, restart
                    write_unit(row0_prev, part_prev);
#pragma unroll
                    for (int c2 = 0; c2 < 8; ++c2) S[c2] = (f32x4){0.0f, 0.0f, 0.0f, 0.0f};
                }
            }
        }
        acc6 = acc[6];
        acc7 = acc[7];
        e_prev = e;
        close_prev = cC.e + 1 == cC.e1;
        row0_prev = unit_tile(cC) * ET;
        part_prev = (u0 + cC.u) % PARTS;
        if (RAGGED) {
#pragma unroll
            for (int t = 0; t < 4; ++t) dg_prev[t] = dg[t];
        }
        cC.next(u0, k);
        cS.next(u0, k);
        if (RAGGED && close_prev) load_deg(dg, cC);
    };
    // (the S reset of a unit's first slot happens at group 5 of its body, after
    // the previous unit's deferred sums and write; relu-sums of the slot start
    // at group 6.  The first slot starts from S = 0.)
    for (;;) {
        body(bx, hA, lA, hB, lB);
        if (cC.u >= nu) break;
        body(bx, hB, lB, hA, lA);
        if (cC.u >= nu) break;
    }
    // the last slot's deferred sums, then its unit (always the last slot of one)
#pragma unroll
    for (int t = 2; t < 4; ++t) relu_add(S[6], acc6[t], t, e_prev, dg_prev);
#pragma unroll
    for (int t = 0; t < 4; ++t) relu_add(S[7], acc7[t], t, e_prev, dg_prev);
    write_unit(row0_prev, part_prev);
}

}  // namespace

// Parts per tile: the smallest count (<= max_parts, <= k) whose grid keeps the
// busiest wave within 3 % of the mean work per wave (4 waves per CU), else the
// best balanced one.  Extra parts cost one more partial buffer in the node stage.
int edge_wave_parts(int64_t ntiles, int cus, int max_parts, int k) {
    const double waves = 4.0 * cus;
    int best = 1;
    double best_eff = 0.0;
    for (int q = 1; q <= max_parts && q <= k && q <= 4; ++q) {
        const double units = (double)ntiles * q;
        const double per = units / waves;
        const double eff = units <= waves ? units / waves : per / std::ceil(per);
        if (eff >= 0.97) return q;
        if (eff > best_eff + 1e-9) {
            best_eff = eff;
            best = q;
        }
    }
    return best;
}

// Profiling aid (tools/ubench): the non-ragged parts = 2 kernel with DIAG bits.
int launch_edge_wave_diag(const float *a, const float *b, const int32_t *nbr, int64_t n, int k,
                          const float *msg2_b, const char *pk, const uint32_t *amax_in, float *out,
                          int cus, int diag, hipStream_t st) {
    const int64_t ntiles = (n + ET - 1) / ET;
    WaveArgs w{a, b, nbr, nullptr, n, k, (int)ntiles, 2, n * LH, msg2_b, pk, amax_in, out};
    const int64_t units = ntiles * 2, waves = 4 * (int64_t)cus;
    const int grid = (int)(units < waves ? units : waves);
    switch (diag) {
    case 1: hipLaunchKernelGGL((gnn_edge_wave_kernel<false, 2, 1>), dim3(grid), dim3(64), 0, st, w); break;
    case 2: hipLaunchKernelGGL((gnn_edge_wave_kernel<false, 2, 2>), dim3(grid), dim3(64), 0, st, w); break;
    case 3: hipLaunchKernelGGL((gnn_edge_wave_kernel<false, 2, 3>), dim3(grid), dim3(64), 0, st, w); break;
    case 4: hipLaunchKernelGGL((gnn_edge_wave_kernel<false, 2, 4>), dim3(grid), dim3(64), 0, st, w); break;
    case 7: hipLaunchKernelGGL((gnn_edge_wave_kernel<false, 2, 7>), dim3(grid), dim3(64), 0, st, w); break;
    case 33: hipLaunchKernelGGL((gnn_edge_wave_kernel<false, 2, 33>), dim3(grid), dim3(64), 0, st, w); break;
    case 97: hipLaunchKernelGGL((gnn_edge_wave_kernel<false, 2, 97>), dim3(grid), dim3(64), 0, st, w); break;
    case 32: hipLaunchKernelGGL((gnn_edge_wave_kernel<false, 2, 32>), dim3(grid), dim3(64), 0, st, w); break;
    case 64: hipLaunchKernelGGL((gnn_edge_wave_kernel<false, 2, 64>), dim3(grid), dim3(64), 0, st, w); break;
    case 128: hipLaunchKernelGGL((gnn_edge_wave_kernel<false, 2, 128>), dim3(grid), dim3(64), 0, st, w); break;
    case 36: hipLaunchKernelGGL((gnn_edge_wave_kernel<false, 2, 36>), dim3(grid), dim3(64), 0, st, w); break;
    default: hipLaunchKernelGGL((gnn_edge_wave_kernel<false, 2, 0>), dim3(grid), dim3(64), 0, st, w); break;
    }
    MMPDE_RET_LAUNCH();
    return MMPDE_OK;
}

int launch_edge_wave(const float *a, const float *b, const int32_t *nbr, const int32_t *deg, int64_t n,
                     int k, const float *msg2_b, const char *pk, const uint32_t *amax_in, float *out,
                     int parts, int64_t part_stride, int cus, hipStream_t st) {
    MMPDE_REQUIRE(a && b && nbr && msg2_b && pk && amax_in && out && n > 0 && k > 0);
    MMPDE_REQUIRE(parts >= 1 && parts <= 4 && parts <= k);
    MMPDE_REQUIRE(parts == 1 || part_stride >= n * LH);
    const int64_t ntiles = (n + ET - 1) / ET;
    MMPDE_REQUIRE(ntiles * parts < (int64_t)INT32_MAX && n * (int64_t)k < ((int64_t)1 << 40));
    WaveArgs w{a, b, nbr, deg, n, k, (int)ntiles, parts, part_stride, msg2_b, pk, amax_in, out};
    const int64_t waves = 4 * (int64_t)cus;   // one 64-thread workgroup per SIMD
    const int64_t units = ntiles * parts;
    const int grid = (int)(units < waves ? units : waves);
#define MMPDE_WAVE(RG, P) hipLaunchKernelGGL((gnn_edge_wave_kernel<RG, P>), dim3(grid), dim3(64), 0, st, w)
#define MMPDE_WAVE_P(RG)              \
    switch (parts) {                  \
    case 1: MMPDE_WAVE(RG, 1); break; \
    case 2: MMPDE_WAVE(RG, 2); break; \
    case 3: MMPDE_WAVE(RG, 3); break; \
    default: MMPDE_WAVE(RG, 4); break; \
    }
    if (deg) {
        MMPDE_WAVE_P(true);
    } else {
        MMPDE_WAVE_P(false);
    }
#undef MMPDE_WAVE_P
#undef MMPDE_WAVE
    MMPDE_RET_LAUNCH();
    return MMPDE_OK;
}
