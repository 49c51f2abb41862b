// Internal (C++) interface between gnn.hip and layer.hip: the two launches of
// one message-passing layer (reference gnn_2d.py:53-69).
#pragma once
#include "common.hpp"

// Edge stage: mean[i] = (1/k) sum_e relu(W2 relu(a_i + b_nbr(i,e)) + b2)
// (message_net_2 + PyG mean aggregation); with deg != nullptr the sum runs
// over e < deg[i] and divides by max(deg[i], 1).  F16X3: pk = this layer's
// packed images, amax_in = range slots of a, b (both required).
// F16X3 runs the one-wave-per-SIMD kernel, which may split each tile's
// neighbour slots over up to max_parts parts for grid balance: part q's mean
// of its slots goes to mean + q * part_stride and *parts_used tells the node
// stage how many buffers to add (F32: always 1).  *sums = true when the buffers
// hold neighbour SUMS (the wave kernel; the node stage then divides by the
// degree: pass div_deg = deg, div_k = k to launch_node_stage), false when they
// hold the mean.  The wave kernel requires sums != nullptr.
int launch_edge_stage(const float *a, const float *b, const int32_t *nbr, const int32_t *deg,
                      int64_t n, int k, const mmpde_gnn_layer_params *p, const char *pk,
                      const uint32_t *amax_in, float *mean, int64_t part_stride, int max_parts,
                      int *parts_used, hipStream_t st, bool *sums = nullptr);

// Parts per tile the wave edge kernel uses for ntiles tiles on cus CUs (1 .. max_parts).
int edge_wave_parts(int64_t ntiles, int cus, int max_parts, int k);

// Edge stage, F16X3, one wave per SIMD with the message_net_2 operands in
// registers (edge_wave.hip).  out + q * part_stride (q < parts <= 4) receives
// the slot range [q k / parts, (q + 1) k / parts) of every target, summed and
// (launch_node_stage adds the parts and divides by the degree).  cus = compute units.
int launch_edge_wave(const float *a, const float *b, const int32_t *nbr, const int32_t *deg, int64_t n,
                     int k, const float *msg2_b, const char *pk, const uint32_t *amax_in, float *out,
                     int parts, int64_t part_stride, int cus, hipStream_t st);

// Node stage (mean = the sum of `parts` buffers part_stride floats apart,
// divided by max(div_deg[row], 1) or div_k when div_k > 0):
// h' = BN(h + relu(U2 relu(U1 [h | mean | t] + c1) + c2)) and, when
// next != nullptr, the next layer's message_net_1 node halves a', b' (and,
// F16X3, their range slots amax_out).  F16X3 when pk != nullptr (pkn: the next
// layer's images).
int launch_node_stage(const float *h, const float *mean, int parts, int64_t part_stride,
                      const float *u, const float *pos, int64_t n, mmpde_gnn_scales sc,
                      const mmpde_gnn_layer_params *p, const mmpde_gnn_layer_params *next,
                      const char *pk, const char *pkn, uint32_t *amax_out, float *h_out, float *a_out,
                      float *b_out, hipStream_t st, const int32_t *div_deg = nullptr, int div_k = 0);

// Embedding (gnn_2d.py:99-106) + layer 0's message_net_1 node halves in one
// launch: h_out = embedding_mlp(cat(u, x/Lx, y/Ly, t/tmax)), a_out / b_out as
// launch_node_stage's.  F16X3 projection when pk0 (layer 0's images) != nullptr.
int launch_embed_stage(const float *u, const float *pos, int64_t n, mmpde_gnn_scales sc,
                       const mmpde_gnn_embed_params *e, const mmpde_gnn_layer_params *l0,
                       const char *pk0, uint32_t *amax_out, float *h_out, float *a_out,
                       float *b_out, hipStream_t st);
