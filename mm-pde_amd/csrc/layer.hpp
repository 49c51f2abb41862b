// Internal (C++) interface between gnn.hip and layer.hip: the two launches of
// one message-passing layer (reference gnn_2d.py:53-69).
#pragma once
#include "common.hpp"

// Edge stage: mean[i] = (1/k) sum_e relu(W2 relu(a_i + b_nbr(i,e)) + b2)
// (message_net_2 + PyG mean aggregation); with deg != nullptr the sum runs
// over e < deg[i] and divides by max(deg[i], 1).  F16X3: pk = this layer's
// packed images, amax_in = range slots of a, b (both required).
int launch_edge_stage(const float *a, const float *b, const int32_t *nbr, const int32_t *deg,
                      int64_t n, int k, const mmpde_gnn_layer_params *p, const char *pk,
                      const uint32_t *amax_in, float *mean, hipStream_t st);

// Node stage: h' = BN(h + relu(U2 relu(U1 [h | mean | t] + c1) + c2)) and, when
// next != nullptr, the next layer's message_net_1 node halves a', b' (and,
// F16X3, their range slots amax_out).  F16X3 when pk != nullptr (pkn: the next
// layer's images).
int launch_node_stage(const float *h, const float *mean, const float *u, const float *pos,
                      int64_t n, mmpde_gnn_scales sc, const mmpde_gnn_layer_params *p,
                      const mmpde_gnn_layer_params *next, const char *pk, const char *pkn,
                      uint32_t *amax_out, float *h_out, float *a_out, float *b_out,
                      hipStream_t st);

// Embedding (gnn_2d.py:99-106) + layer 0's message_net_1 node halves in one
// launch: h_out = embedding_mlp(cat(u, x/Lx, y/Ly, t/tmax)), a_out / b_out as
// launch_node_stage's.  F16X3 projection when pk0 (layer 0's images) != nullptr.
int launch_embed_stage(const float *u, const float *pos, int64_t n, mmpde_gnn_scales sc,
                       const mmpde_gnn_embed_params *e, const mmpde_gnn_layer_params *l0,
                       const char *pk0, uint32_t *amax_out, float *h_out, float *a_out,
                       float *b_out, hipStream_t st);
