// Internal (C++) interface between gnn.hip and layer.hip: the two launches of
// one message-passing layer (reference gnn_2d.py:53-69).
#pragma once
#include "common.hpp"

// How the wave edge kernel split a layer's neighbour slots: S = ntiles * k slots
// over G waves (wave w: slots [w S / G, (w + 1) S / G)); side[w] (16 x 128) holds
// the sums of the unit wave w starts inside a tile.  The node stage adds, for the
// tile of row i, side[w][i % 16] of every w whose first slot lies strictly inside
// that tile, in w order, to the row's sums, then divides by the degree k.
struct EdgeSplit {
    const float *side = nullptr;
    int64_t S = 0;
    int G = 0, k = 0;
};

// Edge stage: mean[i] = (1/k) sum_e relu(W2 relu(a_i + b_nbr(i,e)) + b2)
// (message_net_2 + PyG mean aggregation); with deg != nullptr the sum runs
// over e < deg[i] and divides by max(deg[i], 1).  F16X3: pk = this layer's
// packed images, amax_in = range slots of a, b (both required); it runs the
// one-wave-per-SIMD kernel, which stores neighbour SUMS to mean plus side
// blocks (side: room for side_cap 16 x 128 blocks) and fills *split: the node
// stage then adds the side blocks and divides (pass split to launch_node_stage).
// F32 writes the mean itself and leaves split->G = 0.
int launch_edge_stage(const float *a, const float *b, const int32_t *nbr, const int32_t *deg,
                      int64_t n, int k, const mmpde_gnn_layer_params *p, const char *pk,
                      const uint32_t *amax_in, float *mean, float *side, int64_t side_cap,
                      EdgeSplit *split, hipStream_t st);

// Waves of the wave kernel's slot split (one per SIMD, <= S, <= side_cap).
int edge_wave_grid(int64_t S, int cus, int64_t side_cap);

// Edge stage, F16X3, one wave per SIMD with the message_net_2 operands in
// registers (edge_wave.hip): neighbour sums to out / side (see EdgeSplit).
// cus = compute units.
int launch_edge_wave(const float *a, const float *b, const int32_t *nbr, const int32_t *deg, int64_t n,
                     int k, const float *msg2_b, const char *pk, const uint32_t *amax_in, float *out,
                     float *side, int64_t side_cap, int cus, EdgeSplit *split, hipStream_t st);

// Node stage (mean: the edge stage's buffer, or with split->G > 0 the wave
// kernel's sums plus side blocks divided by max(deg[row], 1) or split->k):
// h' = BN(h + relu(U2 relu(U1 [h | mean | t] + c1) + c2)) and, when
// next != nullptr, the next layer's message_net_1 node halves a', b' (and,
// F16X3, their range slots amax_out).  F16X3 when pk != nullptr (pkn: the next
// layer's images).
int launch_node_stage(const float *h, const float *mean, const EdgeSplit *split, const int32_t *deg,
                      const float *u, const float *pos, int64_t n, mmpde_gnn_scales sc,
                      const mmpde_gnn_layer_params *p, const mmpde_gnn_layer_params *next,
                      const char *pk, const char *pkn, uint32_t *amax_out, float *h_out, float *a_out,
                      float *b_out, hipStream_t st);

// Embedding (gnn_2d.py:99-106) + layer 0's message_net_1 node halves in one
// launch: h_out = embedding_mlp(cat(u, x/Lx, y/Ly, t/tmax)), a_out / b_out as
// launch_node_stage's.  F16X3 projection when pk0 (layer 0's images) != nullptr.
int launch_embed_stage(const float *u, const float *pos, int64_t n, mmpde_gnn_scales sc,
                       const mmpde_gnn_embed_params *e, const mmpde_gnn_layer_params *l0,
                       const char *pk0, uint32_t *amax_out, float *h_out, float *a_out,
                       float *b_out, hipStream_t st);
