// Internal (C++) interface between gnn.hip and layer.hip: the two launches of
// one message-passing layer (reference gnn_2d.py:53-69).
#pragma once
#include "common.hpp"

// F16X3 row maxima: the node / embed stage writes, for every row i of the next
// layer's message_net_1 node halves, rmx[2 i] = max_k |a_i[k]| and rmx[2 i + 1]
// = max_k |b_i[k]| (a NaN counts as 0; plain stores, no atomics, no zeroing).
// The edge stage splits target row i's messages relu(a_i + b_j) with a scale of
// the row's own (f16x3.hpp row_split_scale), from
//     M_i = max|a_i| + max_e max|b_nbr(i,e)|  >=  max_{e,k} |a_ik + b_jk|,
// so each row keeps 22 significant bits relative to its own range however far
// other rows of the trajectory lie above it (round 5's scale was one per
// trajectory segment: rows 2^14 below the segment maximum fell to an absolute
// error floor), and a row's result depends on the row and its neighbours only
// -- not on its segment or on the trajectories launched beside it.
__host__ __device__ inline int64_t row_max_floats(int64_t n) { return ((2 * n + 3) / 4) * 4; }  // 16-B multiple

// Range records beside the row maxima (the edge kernel's fast path): per
// 16-row block blk, 8 floats at rmx + row_max_floats(n) + 8 blk: {max, max, min,
// min} of the block rows' max|a|, max|b| over the rows in the block's first
// trajectory segment (part 0), then the same over its rows in the next segment
// (part 1: a block straddles at most one boundary; empty parts hold max 0, min
// +inf).  A segment whose rows all have M_i >= min max|a| + min max|b| >= 2^-12
// of M_seg = max max|a| + max max|b| loses at most 12 bits of headroom under
// ONE scale from M_seg: its error floor 2^-35 M_seg stays below 2^-23 M_i, the
// split's own 22-bit representation error -- so such a segment skips the
// per-row neighbour gathers (every row gets the segment scale); wider ranges
// take the per-row scales.
__host__ __device__ inline int64_t range_tiles(int64_t n) { return (n + 15) / 16; }
__host__ __device__ inline int64_t row_records_floats(int64_t n) { return row_max_floats(n) + 8 * range_tiles(n); }

// {M_seg, L_seg} of segment s (seg_n rows) from the range records rec (every
// lane active; four blocks per lane per pass, loaded together).
__device__ __forceinline__ float2 segment_stats(const float *rec, int64_t seg_n, int64_t s) {
    const int64_t r0 = s * seg_n, t0 = r0 / 16, t1 = (r0 + seg_n - 1) / 16;
    uint32_t ma = 0, mb = 0, na = 0x7f800000u, nb = 0x7f800000u;
    for (int64_t tb = t0; tb <= t1; tb += 256) {
        float4 v[4];
        int64_t tt[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            tt[q] = min(tb + (threadIdx.x & 63) + 64 * q, t1);
            const bool own = tt[q] * 16 >= r0;  // the block's first row lies in s: part 0
            v[q] = *(const float4 *)(rec + 8 * tt[q] + (own ? 0 : 4));
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) {  // indices past t1 re-read t1: harmless for max / min
            ma = max(ma, __float_as_uint(v[q].x));
            mb = max(mb, __float_as_uint(v[q].y));
            na = min(na, __float_as_uint(v[q].z));
            nb = min(nb, __float_as_uint(v[q].w));
        }
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
        ma = max(ma, (uint32_t)__shfl_xor((int)ma, o, 64));
        mb = max(mb, (uint32_t)__shfl_xor((int)mb, o, 64));
        na = min(na, (uint32_t)__shfl_xor((int)na, o, 64));
        nb = min(nb, (uint32_t)__shfl_xor((int)nb, o, 64));
    }
    return make_float2(__uint_as_float(ma) + __uint_as_float(mb), __uint_as_float(na) + __uint_as_float(nb));
}

// M_i's neighbour term for row `row`: max over e < kk of rmx[2 nbr[row k + e] + 1]
// (as bit patterns, indices clamped to nmax), every index load issued before
// the gathers (two memory round trips).  KU loads are unrolled (clamped to
// e < kk), the rest (kk > KU) run one by one.
template <int KU>
__device__ __forceinline__ float nbr_bmax(const float *rmx, const int32_t *nr, int kk, uint32_t nmax) {
    const uint32_t *rb = (const uint32_t *)rmx;
    uint32_t id[KU];
#pragma unroll
    for (int e = 0; e < KU; ++e) id[e] = (uint32_t)nr[min(e, kk - 1)];
    uint32_t m = 0;
#pragma unroll
    for (int e = 0; e < KU; ++e) m = max(m, rb[2 * (uint64_t)min(id[e], nmax) + 1]);
    for (int e = KU; e < kk; ++e) m = max(m, rb[2 * (uint64_t)min((uint32_t)nr[e], nmax) + 1]);
    return __uint_as_float(m);
}

// How the wave edge kernel split a layer's neighbour slots (edge_wave.hip
// header).  Rows form segments of seg_n (the trajectories; seg_n = n: one
// segment), each cut into tps = ceil(seg_n / 16) 16-row tiles and S = tps * k
// neighbour slots, cut into U summation units (unit u = slots [u S / U,
// (u + 1) S / U)).  side[s * U + u] (16 x 128) holds the sums of unit u's run
// in the tile where it starts, when it starts strictly inside that tile.  The
// node stage adds, for local row q (tile t = q / 16) of segment s,
// side[s * U + u][q % 16] of every u whose first slot lies strictly inside
// that tile, in u order, to the row's sums, then divides by the degree.
struct EdgeSplit {
    const float *side = nullptr;
    int64_t S = 0;         // slots per segment
    int units = 0, k = 0;  // summation units per segment (0: no side blocks), neighbours
    int64_t seg_n = 0;     // rows per segment
};

// Edge stage: mean[i] = (1/k) sum_e relu(W2 relu(a_i + b_nbr(i,e)) + b2)
// (message_net_2 + PyG mean aggregation); with deg != nullptr the sum runs
// over e < deg[i] and divides by max(deg[i], 1).  F16X3: pk = this layer's
// packed images, rmx = row maxima of a, b (both required); it runs the
// one-wave-per-SIMD kernel, which stores neighbour SUMS to mean plus side
// blocks (side: room for side_cap 16 x 128 blocks) and fills *split: the node
// stage then adds the side blocks and divides (pass split to launch_node_stage).
// rmx: the row maxima of a, b and their range records (F16X3, layer.hpp; rng
// false: the row maxima alone, every segment takes the per-row scales).
// F32 writes the mean itself and leaves split->units = 0.  seg_n: rows per
// trajectory segment (n: one segment; must divide n and be >= kRangeRows,
// else n is used).
int launch_edge_stage(const float *a, const float *b, const int32_t *nbr, const int32_t *deg,
                      int64_t n, int k, int64_t seg_n, const mmpde_gnn_layer_params *p, const char *pk,
                      const float *rmx, float *mean, float *side, int64_t side_cap,
                      EdgeSplit *split, hipStream_t st, uint32_t *relu_mask = nullptr, bool rng = true);

// The training forward's F16X3 edge stage (writes the mean; packs W2 and
// computes the row maxima of a, b and every row's split scale itself in ws,
// edge_mean_f16x3_ws_bytes).
int64_t edge_mean_f16x3_ws_bytes(int64_t n);
int launch_edge_mean_f16x3(const float *a, const float *b, const int32_t *nbr, const int32_t *deg, int64_t n,
                           int k, const float *w2, const float *b2, float *mean, uint32_t *relu_mask, void *ws,
                           hipStream_t st);

// Segment size the kernels use for a requested seg_n (n when seg_n is 0, does
// not divide n or is below one 16-row tile).
inline int64_t effective_seg(int64_t n, int64_t seg_n) {
    return (seg_n >= 16 && seg_n <= n && n % seg_n == 0) ? seg_n : n;
}

// Summation units per segment U and waves per segment wpsp of the wave kernel
// (waves = nseg * wpsp, about one per SIMD).  U = the power of two that makes
// units of 22..44 slots, a function of the segment alone (capped by S_seg and
// side_cap / nseg), so every launch sums a row in the same order whatever the
// segment count; wpsp = floor(4 CUs / nseg) clamped to [1, U], each wave
// taking a contiguous run of whole units, raised (more waves than SIMDs) until
// no wave spans more than kWaveTiles tiles (its row scales live in LDS).
// nseg * U <= side_cap.
constexpr int kWaveTiles = 64;
struct EdgePlan {
    int U = 1, wpsp = 1;
    int64_t waves = 1;
};
EdgePlan edge_wave_plan(int64_t nseg, int64_t S_seg, int k, int cus, int64_t side_cap);

// Edge stage, F16X3, one wave per SIMD with the message_net_2 operands in
// registers (edge_wave.hip): neighbour sums to out / side (see EdgeSplit).
// cus = compute units.
int launch_edge_wave(const float *a, const float *b, const int32_t *nbr, const int32_t *deg, int64_t n,
                     int k, int64_t seg_n, const float *msg2_b, const char *pk, const float *rmx, bool rng,
                     float *out, float *side, int64_t side_cap, int cus, EdgeSplit *split, hipStream_t st);

// Node stage (mean: the edge stage's buffer, or with split->units > 0 the wave
// kernel's sums plus side blocks divided by max(deg[row], 1) or split->k):
// h' = BN(h + relu(U2 relu(U1 [h | mean | t] + c1) + c2)) and, when
// next != nullptr, the next layer's message_net_1 node halves a', b' (and,
// F16X3, their row maxima and range records rmx_out, row_records_floats(n)).
// F16X3 when pk != nullptr (pkn: the next layer's images).
int launch_node_stage(const float *h, const float *mean, const EdgeSplit *split, const int32_t *deg,
                      const float *u, const float *pos, int64_t n, int64_t seg_n, mmpde_gnn_scales sc,
                      const mmpde_gnn_layer_params *p, const mmpde_gnn_layer_params *next,
                      const char *pk, const char *pkn, float *rmx_out, float *h_out, float *a_out,
                      float *b_out, hipStream_t st);

// The arguments of one launch_node_stage call.
struct NodeStageCall {
    const float *h, *mean;
    const EdgeSplit *split;
    const int32_t *deg;
    const float *u, *pos;
    int64_t n, seg_n;
    mmpde_gnn_scales sc;
    const mmpde_gnn_layer_params *p, *next;
    const char *pk, *pkn;
    float *rmx_out, *h_out, *a_out, *b_out;
};

// Embedding (gnn_2d.py:99-106) + layer 0's message_net_1 node halves in one
// launch: h_out = embedding_mlp(cat(u, x/Lx, y/Ly, t/tmax)), a_out / b_out as
// launch_node_stage's.  F16X3 projection when pk0 (layer 0's images) != nullptr.
int launch_embed_stage(const float *u, const float *pos, int64_t n, int64_t seg_n, mmpde_gnn_scales sc,
                       const mmpde_gnn_embed_params *e, const mmpde_gnn_layer_params *l0,
                       const char *pk0, float *rmx_out, float *h_out, float *a_out,
                       float *b_out, hipStream_t st);

// launch_embed_stage's arguments.
struct EmbedStageCall {
    const float *u, *pos;
    int64_t n, seg_n;
    mmpde_gnn_scales sc;
    const mmpde_gnn_embed_params *e;
    const mmpde_gnn_layer_params *l0;
    const char *pk0;
    float *rmx_out, *h_out, *a_out, *b_out;
};
