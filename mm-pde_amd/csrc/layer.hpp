// Internal (C++) interface between gnn.hip and layer.hip: the two launches of
// one message-passing layer (reference gnn_2d.py:53-69).
#pragma once
#include "common.hpp"

// F16X3 range records: the node / embed stage writes, per 16-row block
// (kRangeRows rows; block index = row / kRangeRows), the max |a| and max |b| of
// its rows in each of the (at most two) trajectory segments the tile touches:
// rng[tile] = {max|a| seg0, max|b| seg0, max|a| seg1, max|b| seg1}, seg0 =
// first row / seg_n (the seg1 entries are 0 when the tile lies in one
// segment).  The wave edge kernel takes its split scale from the records of
// its own segment only, so a trajectory's f16x3 result does not depend on the
// trajectories launched beside it.  Plain stores, no atomics, no zeroing.
constexpr int kRangeRows = 16;
__host__ __device__ inline int64_t range_tiles(int64_t n) { return (n + kRangeRows - 1) / kRangeRows; }

// max |a| + max |b| over segment s from the range records of the node tiles
// that hold its rows (layer.hpp kRangeRows): a block whose first row lies in s
// gives its seg0 entries, the block straddling into s from s - 1 its seg1 ones.
__device__ __forceinline__ float segment_range(const float *rng, int64_t seg_n, int64_t s) {
    const int64_t r0 = s * seg_n, t0 = r0 / kRangeRows, t1 = (r0 + seg_n - 1) / kRangeRows;
    float ma = 0.0f, mb = 0.0f;
    // four records per lane per pass, loaded together (one memory round trip for
    // segments of up to 256 records): indices past t1 re-read t1, which a max
    // takes twice harmlessly
    for (int64_t tb = t0; tb <= t1; tb += 256) {
        float4 v[4];
        int64_t tt[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            tt[q] = min(tb + (threadIdx.x & 63) + 64 * q, t1);
            v[q] = *(const float4 *)(rng + 4 * tt[q]);
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const bool own = tt[q] * kRangeRows >= r0;  // first row of the tile in s
            ma = fmaxf(ma, own ? v[q].x : v[q].z);
            mb = fmaxf(mb, own ? v[q].y : v[q].w);
        }
    }
    return wave_absmax(ma) + wave_absmax(mb);  // maxima of |x| >= 0; every lane active
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
// packed images, rng = range records of a, b (both required); it runs the
// one-wave-per-SIMD kernel, which stores neighbour SUMS to mean plus side
// blocks (side: room for side_cap 16 x 128 blocks) and fills *split: the node
// stage then adds the side blocks and divides (pass split to launch_node_stage).
// F32 writes the mean itself and leaves split->units = 0.  seg_n: rows per
// trajectory segment (n: one segment; must divide n and be >= kRangeRows,
// else n is used).
int launch_edge_stage(const float *a, const float *b, const int32_t *nbr, const int32_t *deg,
                      int64_t n, int k, int64_t seg_n, const mmpde_gnn_layer_params *p, const char *pk,
                      const float *rng, float *mean, float *side, int64_t side_cap,
                      EdgeSplit *split, hipStream_t st, uint32_t *relu_mask = nullptr);

// The training forward's F16X3 edge stage (writes the mean; packs W2 and
// computes the range records of a, b itself in ws, edge_mean_f16x3_ws_bytes).
int64_t edge_mean_f16x3_ws_bytes(int64_t n);
int launch_edge_mean_f16x3(const float *a, const float *b, const int32_t *nbr, const int32_t *deg, int64_t n,
                           int k, const float *w2, const float *b2, float *mean, uint32_t *relu_mask, void *ws,
                           hipStream_t st);

// Segment size the kernels use for a requested seg_n (n when seg_n is 0, does
// not divide n or is below kRangeRows).
inline int64_t effective_seg(int64_t n, int64_t seg_n) {
    return (seg_n >= kRangeRows && seg_n <= n && n % seg_n == 0) ? seg_n : n;
}

// Summation units per segment U and waves per segment wpsp of the wave kernel
// (waves = nseg * wpsp, about one per SIMD).  U = the power of two that makes
// units of 22..44 slots, a function of the segment alone (capped by S_seg and
// side_cap / nseg), so every launch sums a row in the same order whatever the
// segment count; wpsp = floor(4 CUs / nseg) clamped to [1, U], each wave
// taking a contiguous run of whole units.  nseg * U <= side_cap.
struct EdgePlan {
    int U = 1, wpsp = 1;
    int64_t waves = 1;
};
EdgePlan edge_wave_plan(int64_t nseg, int64_t S_seg, int cus, int64_t side_cap);

// Edge stage, F16X3, one wave per SIMD with the message_net_2 operands in
// registers (edge_wave.hip): neighbour sums to out / side (see EdgeSplit).
// cus = compute units.
int launch_edge_wave(const float *a, const float *b, const int32_t *nbr, const int32_t *deg, int64_t n,
                     int k, int64_t seg_n, const float *msg2_b, const char *pk, const float *rng,
                     float *out, float *side, int64_t side_cap, int cus, EdgeSplit *split, hipStream_t st);

// Node stage (mean: the edge stage's buffer, or with split->units > 0 the wave
// kernel's sums plus side blocks divided by max(deg[row], 1) or split->k):
// h' = BN(h + relu(U2 relu(U1 [h | mean | t] + c1) + c2)) and, when
// next != nullptr, the next layer's message_net_1 node halves a', b' (and,
// F16X3, their range records rng_out over segments of seg_n rows).  F16X3 when
// pk != nullptr (pkn: the next layer's images).
int launch_node_stage(const float *h, const float *mean, const EdgeSplit *split, const int32_t *deg,
                      const float *u, const float *pos, int64_t n, int64_t seg_n, mmpde_gnn_scales sc,
                      const mmpde_gnn_layer_params *p, const mmpde_gnn_layer_params *next,
                      const char *pk, const char *pkn, float *rng_out, float *h_out, float *a_out,
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
    float *rng_out, *h_out, *a_out, *b_out;
};

// Embedding (gnn_2d.py:99-106) + layer 0's message_net_1 node halves in one
// launch: h_out = embedding_mlp(cat(u, x/Lx, y/Ly, t/tmax)), a_out / b_out as
// launch_node_stage's.  F16X3 projection when pk0 (layer 0's images) != nullptr.
int launch_embed_stage(const float *u, const float *pos, int64_t n, int64_t seg_n, mmpde_gnn_scales sc,
                       const mmpde_gnn_embed_params *e, const mmpde_gnn_layer_params *l0,
                       const char *pk0, float *rng_out, float *h_out, float *a_out,
                       float *b_out, hipStream_t st);

// launch_embed_stage's arguments.
struct EmbedStageCall {
    const float *u, *pos;
    int64_t n, seg_n;
    mmpde_gnn_scales sc;
    const mmpde_gnn_embed_params *e;
    const mmpde_gnn_layer_params *l0;
    const char *pk0;
    float *rng_out, *h_out, *a_out, *b_out;
};
