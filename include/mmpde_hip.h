/*
 * mmpde_hip.h -- C-ABI of libmmpde_hip.so, the MI355X (gfx950) kernels behind
 * the MM-PDE forward step.
 *
 * The reference (Peiyannn/MM-PDE) is pure Python and has no FFI: its hot path
 * calls PyG / torch_scatter / torch_cluster / scikit-learn / cuBLAS from
 * Python.  Each entry point below replaces one of those call sites (cited
 * per function as reference file:line); the Python host mirror in
 * mm-pde_amd/mmpde_amd binds them with ctypes.
 *
 * Conventions (all entry points):
 *  - every tensor is a caller-owned, contiguous, row-major DEVICE buffer;
 *    fp32 for features / coordinates, int32 for neighbour tables;
 *  - node rows are trajectory-major: row = b * n_per + p;
 *  - `stream` is a hipStream_t; every call is asynchronous and stream-ordered,
 *    never allocates, never synchronises (safe inside hipGraph capture);
 *  - the return value is a status: 0 ok, < 0 error (see MMPDE_ERR_*);
 *    hipError_t e from a launch is returned as MMPDE_ERR_HIP_BASE - e;
 *  - calls are stateless and re-entrant (no global mutable state).
 */
#ifndef MMPDE_HIP_H
#define MMPDE_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MMPDE_OK 0
#define MMPDE_ERR_INVALID_ARG (-1)
#define MMPDE_ERR_UNSUPPORTED (-2)
#define MMPDE_ERR_HIP_BASE (-1000)

#define MMPDE_ACT_NONE 0
#define MMPDE_ACT_TANH 1
#define MMPDE_ACT_RELU 2
#define MMPDE_ACT_ELU 3 /* x > 0 ? x : expm1(x) (F.elu, alpha 1) */
#define MMPDE_PAD_ZEROS 0
#define MMPDE_PAD_CIRCULAR 1

typedef void *mmpde_stream_t; /* hipStream_t */

/* ABI version: major*10000 + minor*100 + patch */
int mmpde_version(void);
/* Static description of a status code (never NULL). */
const char *mmpde_status_string(int status);

/* ------------------------------------------------------------------------
 * Neighbour search
 * ---------------------------------------------------------------------- */

/* torch_cluster.knn_graph(x, k, batch, loop=False) for `batches` equal,
 * contiguous segments of n_per points.  Replaces reference
 * data_creator_2d.py:260 and mesh/dmm_model.py:228.
 * pos      [batches*n_per, 2] fp32
 * nbr_out  [batches*n_per, k] int32: GLOBAL source index of the e-th nearest
 *          neighbour of each query, e ordered by (d2, index), d2 =
 *          fmaf(dy, dy, dx*dx); self excluded.  PyG edge_index is
 *          [nbr_out.flatten(), repeat_interleave(arange(n), k)].
 * degenerate (nullable, device int32[1], accumulated): queries whose degree
 *          would be ragged in the reference (self not among the k+1 nearest).
 * Requires k+1 <= n_per <= 16384, k <= 63 (more than 4096 points per
 * trajectory: a slower path with the points in a 128 KB LDS block). */
int mmpde_knn_graph(const float *pos, int64_t batches, int64_t n_per, int k,
                    int32_t *nbr_out, int32_t *degenerate, mmpde_stream_t stream);

/* Static candidate table of the moved-mesh kNN entry points below, for fixed
 * points xi [n_per, 2] (128 <= n_per <= 4096) and reference points ref
 * [n_per, 2] (NULL: xi): cand_out [n_per, 128] int32 LOCAL = the 128 nearest
 * of ref_p in xi, (d2, index) order.  Built once per fixed mesh: ref = xi for
 * mmpde_knn_graph_cand; for mmpde_knn_query_cand ref = the fixed query points
 * (e.g. the uniform grid, in its own order). */
int mmpde_knn_candidates(const float *xi, const float *ref, int64_t n_per, int32_t *cand_out,
                         mmpde_stream_t stream);

/* Displacement record of moved points pos = xi + d [batches * n_per, 2]: per
 * trajectory, the box of xi cut into 16 x 16 cells and, per cell, the largest
 * |d_j| of the points whose xi_j lies in it, the largest |d_j| overall, and
 * per role (graph, query) the number of queries the candidate table could not
 * answer in the last call of that role (mmpde_knn_table_misses; calls of one
 * role on one record must not overlap).
 * cells_out: device memory of mmpde_knn_moved_cells_bytes(batches).  One
 * launch per moved mesh, shared by mmpde_knn_graph_cand and
 * mmpde_knn_query_cand. */
int64_t mmpde_knn_moved_cells_bytes(int64_t batches);
int mmpde_knn_moved_cells(const float *pos, const float *xi, int64_t batches, int64_t n_per,
                          float *cells_out, mmpde_stream_t stream);
/* out[0] (device float) = the median over the reference points p of
 * R128(p) - R_kk(p), the 128th and the kk-th nearest distance of ref_p in xi
 * (cand from mmpde_knn_candidates(xi, ref)), halved when the queries move with
 * the mesh (moved_queries != 0: the graph, whose query x_p is itself
 * displaced): the skip_above of the calls below (past that typical
 * displacement about half the lookups cannot pass).  Once per table. */
int mmpde_knn_skip_threshold(const float *xi, const float *ref, int64_t n_per, const int32_t *cand,
                             int kk, int moved_queries, float *out, mmpde_stream_t stream);
/* misses_out [batches, 2] int32 (device): per trajectory, the graph and the
 * query misses counted in the record (diagnostics; stream-ordered copy). */
int mmpde_knn_table_misses(const float *cells, int64_t batches, int32_t *misses_out,
                           mmpde_stream_t stream);

/* mmpde_knn_graph of moved points pos = xi + displacement (the DMM's moved mesh,
 * reference data_creator_2d.py:88-137 then :260), the same output bit for bit,
 * answered from the candidate table where a distance bound proves it complete
 * (|x_j - x_p| >= max(R128(xi_p) - |d_p|, dist(x_p, cell of xi_j)) - max |d|
 * over that cell, for every non-candidate j), by the full search elsewhere.
 * xi [n_per, 2] the fixed points every trajectory moves from; cand from
 * mmpde_knn_candidates(xi, NULL); cells from mmpde_knn_moved_cells(pos, xi);
 * scratch: device bytes from mmpde_knn_graph_cand_scratch_bytes (a flag per
 * query: the ones the full search answers).  skip_above > 0: a trajectory
 * whose median cell displacement (over the record's non-empty cells) exceeds
 * it goes straight to the full search (mmpde_knn_skip_threshold); <= 0: the
 * table is always tried.  k <= 63 and 128 <= n_per <= 4096, else it
 * is mmpde_knn_graph. */
int64_t mmpde_knn_graph_cand_scratch_bytes(int64_t batches, int64_t n_per);
int mmpde_knn_graph_cand(const float *pos, const float *xi, const float *cells, float skip_above,
                         int64_t batches, int64_t n_per, int k, const int32_t *cand, int32_t *nbr_out,
                         int32_t *degenerate, void *scratch, mmpde_stream_t stream);

/* sklearn NearestNeighbors(n_neighbors=k).fit(src_b).kneighbors(qry_b) per
 * trajectory b (reference data_creator_2d.py:66-78).  Distances in fp64
 * (dx*dx + dy*dy), ascending, ties by index.
 * src [batches*n_src, 2], qry [batches*n_qry, 2] fp32
 * idx_out [batches*n_qry, k] int32 LOCAL source index (0..n_src-1).
 * ties (nullable, one int32 the caller zeroes): += the number of queries
 * whose sorted fp64 distances hold an exact tie inside the first k or
 * between ranks k-1 and k -- the only inputs on which sklearn's own order (its
 * KD-tree traversal) may differ from (distance, index); parity with sklearn is
 * unpinned for those queries.
 * Requires k <= n_src <= 16384, k <= 63. */
int mmpde_knn_query(const float *src, const float *qry, int64_t batches, int64_t n_src,
                    int64_t n_qry, int k, int32_t *idx_out, int32_t *ties, mmpde_stream_t stream);

/* mmpde_knn_query of qry [batches * n_per, 2] onto moved points src = xi +
 * displacement [batches * n_per, 2] (reference data_creator_2d.py:66-78, the
 * kNN-30 query of the fixed grid onto the DMM's moved mesh), the same output
 * bit for bit, answered from mmpde_knn_candidates(xi, ref) where the bound of
 * mmpde_knn_graph_cand (with |qry_p - ref_p| in place of |d_p|) proves it
 * complete, by the full search elsewhere.  ref [n_per, 2]: the reference
 * points the table was built for (NULL: xi); cells from
 * mmpde_knn_moved_cells(src, xi).  n_src = n_qry = n_per; scratch as for
 * mmpde_knn_graph_cand; ties as for mmpde_knn_query (each query counted
 * once, by whichever kernel answered it).  k <= 64 and 128 <= n_per <= 4096,
 * else it is mmpde_knn_query. */
int mmpde_knn_query_cand(const float *src, const float *qry, const float *xi, const float *ref,
                         const float *cells, float skip_above, int64_t batches, int64_t n_per, int k,
                         const int32_t *cand, int32_t *idx_out, int32_t *ties, void *scratch,
                         mmpde_stream_t stream);

/* torch_cluster.radius_graph(pos, r, batch, loop=False, max_num_neighbors)
 * (data_creator_2d.py:257-258, connect_edge='radius'; r at :195 / :226) for
 * `batches` equal contiguous segments of n_per points, CUDA semantics: each
 * query keeps the first max_num_neighbors + 1 points of its segment in index
 * order with squared distance (fmaf(dy, dy, dx*dx), fp32) < (float)(r*r),
 * itself included, then the self loop is dropped.
 * nbr_out [n, max_num_neighbors + 1] int32 global source indices ascending,
 * padded with -1; degree_out [n] entries kept per row -- pass both to
 * mmpde_gnn_forward_ex (k = max_num_neighbors + 1, exec->degree). */
int mmpde_radius_graph(const float *pos, int64_t batches, int64_t n_per, float r,
                       int max_num_neighbors, int32_t *nbr_out, int32_t *degree_out,
                       mmpde_stream_t stream);

/* PyG edge_index (int64 [2, n*k]) from a target-major neighbour table.
 * Row 0 = source (nbr), row 1 = target. (data_creator_2d.py:260-262) */
int mmpde_edge_index_from_nbr(const int32_t *nbr, int64_t n, int k, int64_t *edge_index,
                              mmpde_stream_t stream);

/* ------------------------------------------------------------------------
 * Dense helpers
 * ---------------------------------------------------------------------- */

/* y[m, n] = act(x[m, k] . w[n, k]^T + b[n]) for skinny m (<= 4096 rows, tuned
 * for m <= 32): res_cut MLP (interpolate.py:74-82), DMM output_mlp / fc
 * layers (mesh/dmm_model.py:59-60, 175-181).  ldx / ldw / ldy are row strides
 * in elements; b nullable. */
int mmpde_linear_skinny(const float *x, int64_t ldx, int64_t m, int64_t k, const float *w,
                        int64_t ldw, const float *b, int64_t n, int act, float *y,
                        int64_t ldy, mmpde_stream_t stream);
/* The same with a device workspace of at least
 * mmpde_linear_skinny_workspace_bytes(m, n, k) bytes (0: none needed), ZEROED
 * before its first use and then reused (the call leaves its counters at zero
 * again): K is split over several workgroups per output tile so that the
 * weight stream fills the chip, and the partial tiles are added in a fixed
 * order inside the launch (results identical run to run).  A NULL / short
 * workspace falls back to no split.  Layout: 4096 ticket words (the only
 * words that must start at zero), then the partial tiles. */
int64_t mmpde_linear_skinny_workspace_bytes(int64_t m, int64_t n, int64_t k);
int mmpde_linear_skinny_ws(const float *x, int64_t ldx, int64_t m, int64_t k, const float *w,
                           int64_t ldw, const float *b, int64_t n, int act, float *y, int64_t ldy,
                           float *workspace, int64_t workspace_bytes, mmpde_stream_t stream);

/* out[b] = mean_i (pred[b, i] - labels[b, i])^2 per trajectory b (n_per values
 * each): the loss of mmpde.py:33-36 (MSELoss) kept per trajectory for the
 * sharded teacher-forced evaluation (train_helper_2d.py:184-185,193-198).
 * Fixed summation order per trajectory: independent of `batches`. */
int mmpde_traj_mse(const float *pred, const float *labels, int64_t batches, int64_t n_per,
                   float *out, mmpde_stream_t stream);

/* F.interpolate(u, size=(oh, ow), mode='bilinear', align_corners=True) of
 * `planes` contiguous h x w fp32 planes (data_creator_2d.py:102-103, moving_mesh's
 * pre-resampling of u to the DMM grid size); y [planes, oh, ow]. */
int mmpde_resample_bilinear(const float *x, int64_t planes, int h, int w, int oh, int ow, float *y,
                            mmpde_stream_t stream);

/* Direct 2-D convolution, NCHW fp32, square kernel ks, zero padding pad,
 * stride 1 or 2, fused act(conv + bias [+ residual]).  residual nullable,
 * same shape as the output.  ConvNet branch (mesh/dmm_model.py:53-57,65-81)
 * and burgers res_cut (interpolate.py:63-72). */
int mmpde_conv2d(const float *x, int64_t batches, int cin, int h, int w, const float *weight,
                 const float *bias, int cout, int ks, int stride, int pad,
                 const float *residual, int act, float *y, mmpde_stream_t stream);
/* The same with pad_mode MMPDE_PAD_ZEROS / MMPDE_PAD_CIRCULAR (nn.Conv2d
 * padding_mode='circular': indices wrap) and res_after_act = 1 for
 * residual + act(conv + bias) (BaseCNN's x + elu(conv(x)), models_cnn.py:70-76)
 * instead of act(conv + bias + residual).  act: MMPDE_ACT_* incl. ELU. */
int mmpde_conv2d_ex(const float *x, int64_t batches, int cin, int h, int w, const float *weight,
                    const float *bias, int cout, int ks, int stride, int pad, int pad_mode,
                    const float *residual, int res_after_act, int act, float *y,
                    mmpde_stream_t stream);

/* Weight and bias gradients of a stride-1 mmpde_conv2d_ex convolution (output
 * size = input size, pad = ks / 2 for odd ks) -- the training backward of
 * BaseCNN (models_cnn.py:66-83 through loss.backward(), train_helper_2d.py:
 * 121-126): dw [cout, cin, ks, ks] = sum over batches and pixels of
 * dy[b, co, y, x] * x[b, ci, y - pad + ky, x - pad + kx] (wrapped or zero
 * padded), db [cout] = sum of dy (nullable).  ks * ks <= 256.  Fixed summation
 * order: deterministic.  (The input gradient is mmpde_conv2d_ex of dy with
 * the flipped, transposed kernel.) */
int mmpde_conv2d_grad_weight(const float *x, int64_t batches, int cin, int h, int w, const float *dy,
                             int cout, int ks, int pad, int pad_mode, float *dw_out, float *db_out,
                             mmpde_stream_t stream);

/* ------------------------------------------------------------------------
 * MP_PDE_Solver_2D (reference gnn_2d.py:19-141), hidden width 128.
 * Node inputs: u [n, tw] fp32 (data.x), pos [n, 3] fp32 = (t, x, y) (data.pos).
 * time_window tw (1 .. 16) is supported by mmpde_gnn_forward[_ex]; the
 * per-stage entry points (mmpde_gnn_embed / _layer) take tw = 1.
 * pos_xy != 0: pos is [n, 2] = (x, y) and every node's t is *t_ptr (a device
 * scalar, e.g. a graph-captured step's slot) or, with t_ptr NULL, t -- the
 * rollout's form (one t per step, the moved mesh used as the positions as is).
 * ---------------------------------------------------------------------- */
typedef struct {
    float inv_lx, inv_ly, inv_tmax; /* 1/pde.Lx, 1/pde.Ly, 1/pde.tmax (gnn_2d.py:122-124) */
    int tw;                         /* time_window: channels of u (0 is read as 1) */
    int pos_xy;                     /* 0: pos = (t, x, y) rows; else (x, y) rows + t below */
    float t;                        /* pos_xy: the nodes' t when t_ptr is NULL */
    const float *t_ptr;             /* pos_xy: device scalar holding t (nullable) */
} mmpde_gnn_scales;

typedef struct {
    /* embedding_mlp: Linear(4,128) BN ReLU Linear(128,128) BN (gnn_2d.py:99-106) */
    const float *w0, *b0;                 /* [128,4], [128]   */
    const float *bn1_w, *bn1_b, *bn1_rm, *bn1_rv;
    const float *w3, *b3;                 /* [128,128], [128] */
    const float *bn4_w, *bn4_b, *bn4_rm, *bn4_rv;
    float eps;
} mmpde_gnn_embed_params;

typedef struct {
    /* GNN_Layer_FS_2D (gnn_2d.py:30-69).  msg1_w is the reference
     * message_net_1.0.weight [128, 260] (columns: h_i | h_j | du | dx | dy | t_i);
     * upd1_w is update_net_1.0.weight [128, 257] (h | mean | t). */
    const float *msg1_w, *msg1_b, *msg2_w, *msg2_b;
    const float *upd1_w, *upd1_b, *upd2_w, *upd2_b;
    const float *bn_w, *bn_b, *bn_rm, *bn_rv; /* norm.module.* */
    float eps;
    /* Row strides (elements) of msg1_w / upd1_w: multiples of 4 and >= 260 /
     * 257.  The reference message_net_1 weight is usable as-is (ld 260);
     * update_net_1's [128, 257] needs a copy padded to ld 260 so rows stay
     * 16-B aligned for dwordx4 loads (the host mirror keeps one). */
    int64_t msg1_ld, upd1_ld;
} mmpde_gnn_layer_params;

typedef struct {
    /* output_mlp Conv1d(1,4,16,s3) ReLU Conv1d(4,8,12,s3) ReLU Conv1d(8,1,8,s2)
     * (gnn_2d.py:108-114) */
    const float *c0_w, *c0_b, *c2_w, *c2_b, *c4_w, *c4_b;
    float out_scale;          /* tw = 1: pde.dt * 0.1 (gnn_2d.py:137-139) */
    const float *out_scales;  /* tw > 1: cumsum(ones(1, tw) * pde.dt * 0.1), tw device floats;
                                 out[n, tw] = out_scales[c] * output_mlp(h) */
    int tw;                   /* 0 or 1: out[n] = out_scale * output_mlp(h) */
} mmpde_gnn_head_params;

/* Bytes of device workspace mmpde_gnn_forward needs for n nodes. */
int64_t mmpde_gnn_workspace_bytes(int64_t n);

/* h_out[n,128] = embedding_mlp(cat(u, x/Lx, y/Ly, t/tmax)) */
int mmpde_gnn_embed(const float *u, const float *pos, int64_t n, mmpde_gnn_scales sc,
                    const mmpde_gnn_embed_params *p, float *workspace, float *h_out,
                    mmpde_stream_t stream);

/* One message-passing layer: h_out = BN(h + upd(h, mean_j msg(h_i, h_j, ...))).
 * nbr [n, k] int32 target-major (global source indices), fixed degree k
 * (PyG aggr='mean' over the k in-edges).  workspace >= 4*n*128 floats.
 * h_out must not alias h_in. */
int mmpde_gnn_layer(const float *h_in, const float *u, const float *pos, int64_t n, int k,
                    const int32_t *nbr, mmpde_gnn_scales sc, const mmpde_gnn_layer_params *p,
                    float *workspace, float *h_out, mmpde_stream_t stream);

/* Only the edge stage: mean[i] = (1/k) sum_e relu(W2 relu(a[i] + b[nbr[i,e]]) + b2)
 * with a, b the per-node halves of message_net_1 ([n,128] each). */
int mmpde_gnn_edge_mean(const float *a, const float *b, const int32_t *nbr, int64_t n, int k,
                        const float *msg2_w, const float *msg2_b, float *mean_out,
                        mmpde_stream_t stream);

/* Edge stage with per-target in-degrees (deg may be NULL: every row has k
 * live slots; slots e >= deg[i] are padding and ignored; mean over
 * max(deg, 1)).  Exact fp32 arithmetic: the forward of the training path
 * (train_helper_2d.py:114-126 -> gnn_2d.py:53-63 with aggr='mean'). */
int mmpde_gnn_edge_mean_deg(const float *a, const float *b, const int32_t *nbr, const int32_t *deg,
                            int64_t n, int k, const float *msg2_w, const float *msg2_b,
                            float *mean_out, mmpde_stream_t stream);

/* mmpde_gnn_edge_mean_deg in a chosen arithmetic: edge_gemm
 * MMPDE_EDGE_GEMM_F32 is mmpde_gnn_edge_mean_deg; MMPDE_EDGE_GEMM_F16X3 runs
 * message_net_2 in the fp16x3 split (the eval path's arithmetic), packing
 * W2 and the row maxima of a, b (each target row i is split with a scale of
 * its own, from max|a_i| + max over its neighbours of max|b_j|) into
 * workspace (>= mmpde_gnn_edge_mean_workspace_bytes(n, edge_gemm) bytes, 16-B
 * aligned) on every call: the f16x3 per-layer path, whose weights change
 * every iteration.  relu_mask (nullable, 16-B aligned; F32 or F16X3):
 * [n * k][4] uint32, bit c % 32 of word c / 32 of slot q = i*k + e set where
 * message_net_2's pre-activation z2[c] > 0 for that edge -- the ReLU pattern
 * mmpde_gnn_edge_backward_sorted then reuses instead of recomputing z2 (the
 * training forward: the persistent ring kernel).  F16X3 without relu_mask
 * (no backward to feed: eval / no-grad) runs the inference forward's
 * one-wave-per-SIMD kernel over one segment of n rows, then adds its side
 * blocks and divides. */
int64_t mmpde_gnn_edge_mean_workspace_bytes(int64_t n, int edge_gemm);
int mmpde_gnn_edge_mean_ex(const float *a, const float *b, const int32_t *nbr, const int32_t *deg,
                           int64_t n, int k, const float *msg2_w, const float *msg2_b, float *mean_out,
                           uint32_t *relu_mask, int edge_gemm, void *workspace, int64_t workspace_bytes,
                           mmpde_stream_t stream);

/* ---------------------------------------------------------------- training
 * Backward of the edge stage (reference: loss.backward() at
 * train_helper_2d.py:126 through GNN_Layer_FS_2D.message / aggr='mean',
 * gnn_2d.py:53-63).  Given grad_mean = dL/dmean [n,128]:
 *   grad_a [n,128]      = dL/da  (target half of message_net_1's output)
 *   grad_edge [n*k,128] = dL/dz1 per edge slot (target-major as nbr; 0 for
 *                         padding slots); dL/db = its per-source sum, see
 *                         mmpde_gnn_edge_source_sum
 *   grad_w2 [128,128], grad_b2 [128] = dL/d message_net_2.0 weight / bias.
 * partials: device scratch of mmpde_gnn_edge_backward_partials() floats.
 * z1/z2 are recomputed (nothing is kept by the forward); exact fp32 products;
 * fixed reduction order (deterministic, no atomics). */
int64_t mmpde_gnn_edge_backward_partials(int *grid);
int mmpde_gnn_edge_backward(const float *a, const float *b, const int32_t *nbr, const int32_t *deg,
                            int64_t n, int k, const float *msg2_w, const float *msg2_b,
                            const float *grad_mean, float *grad_a, float *grad_edge,
                            float *partials, float *grad_w2, float *grad_b2, mmpde_stream_t stream);
/* The same with the GEMM arithmetic chosen by edge_gemm: MMPDE_EDGE_GEMM_F32
 * (the call above) or MMPDE_EDGE_GEMM_F16X3 (the z2, gm1 and dW2 GEMMs in the
 * fp16x3 split with fp32 accumulation, as the forward's f16x3 edge stage:
 * relu(z1) and gz2 scaled by powers of two from max|a| + max|b| and max|g|,
 * W2 per column; k <= 64, else the F32 kernel).  Same outputs, same partials
 * scratch, deterministic. */
int mmpde_gnn_edge_backward_ex(const float *a, const float *b, const int32_t *nbr, const int32_t *deg,
                               int64_t n, int k, const float *msg2_w, const float *msg2_b,
                               const float *grad_mean, float *grad_a, float *grad_edge,
                               float *partials, float *grad_w2, float *grad_b2, int edge_gemm,
                               mmpde_stream_t stream);
/* grad_b[j] = sum over q in [rev_off[j], rev_off[j+1]) of grad_edge[rev_edge[q]]
 * (rev_*: the reverse adjacency, slot ids i*k+e grouped by source j, in the
 * order given; summation order fixed: the even list positions and the odd
 * ones each added in list order, then the two sums: deterministic). */
int mmpde_gnn_edge_source_sum(const float *grad_edge, const int64_t *rev_off, const int64_t *rev_edge,
                              int64_t n, float *grad_b, mmpde_stream_t stream);
/* The backward with grad_edge in source-major order: the row of slot q is
 * slot_pos[q] (mmpde_reverse_adjacency's slot_pos, a permutation of 0 ..
 * n*k-1), so that dL/db is the contiguous segmented sum
 * mmpde_gnn_edge_source_sum_sorted over rev_off: the same sums in the same
 * order as mmpde_gnn_edge_backward_ex + mmpde_gnn_edge_source_sum, read as a
 * stream instead of a gather.  n * k < 2^31.  relu_mask (nullable; F32 or F16X3,
 * k <= 64): the forward's z2 > 0 bits (mmpde_gnn_edge_mean_ex): the ReLU
 * pattern of message_net_2 is taken from it and z2 is not recomputed (one of
 * the three per-edge GEMMs dropped). */
int mmpde_gnn_edge_backward_sorted(const float *a, const float *b, const int32_t *nbr, const int32_t *deg,
                                   int64_t n, int k, const float *msg2_w, const float *msg2_b,
                                   const float *grad_mean, const int32_t *slot_pos, const uint32_t *relu_mask,
                                   float *grad_a, float *grad_edge, float *partials, float *grad_w2,
                                   float *grad_b2, int edge_gemm, mmpde_stream_t stream);
int mmpde_gnn_edge_source_sum_sorted(const float *grad_edge, const int64_t *rev_off, int64_t n, float *grad_b,
                                     mmpde_stream_t stream);
/* The same segmented sum for rows of any width: out[j, :] = sum over q in
 * [rev_off[j], rev_off[j+1]) of rows[rev_edge[q], :] (n output rows), in list
 * order.  The deterministic backward of a row gather (the kNN-30 neighbour
 * values of the training-mode interpolation, data_creator_2d.py:77-83). */
int mmpde_segment_sum(const float *rows, int64_t width, const int64_t *rev_off, const int64_t *rev_edge,
                      int64_t n, float *out, mmpde_stream_t stream);
/* The reverse adjacency those two take, built on the device: rev_edge [n_tgt *
 * k capacity] = the live slot ids q = i*k + e (e < deg[i] when deg is given)
 * grouped by source j = nbr[i, e], ascending q within a source; rev_off
 * [n_src + 1] the group offsets (rev_off[n_src] = live slots).  Sources
 * outside [0, n_src) are skipped and counted in *bad (device int32, zeroed
 * first).  slot_pos (nullable) [n_tgt * k]: the inverse permutation, the
 * position of slot q in the sorted order (dead slots after rev_off[n_src]).  Deterministic (a stable radix sort by source).  scratch:
 * mmpde_reverse_adjacency_scratch_bytes(n_tgt, k, n_src), 256-byte aligned. */
int64_t mmpde_reverse_adjacency_scratch_bytes(int64_t n_tgt, int k, int64_t n_src);
int mmpde_reverse_adjacency(const int32_t *nbr, int64_t n_tgt, int k, const int32_t *deg, int64_t n_src,
                            int64_t *rev_off, int64_t *rev_edge, int32_t *slot_pos, void *scratch,
                            int64_t scratch_bytes, int32_t *bad, mmpde_stream_t stream);

/* Weight / bias gradient of a skinny linear map over many rows (the training
 * backward of the Conv1d head as unfold + GEMM, gnn_2d.py:108-114, and of the
 * embedding's first Linear, gnn_2d.py:99-106; train_helper_2d.py:126):
 * dw [n_out, k] = dy^T x, db [n_out] = sum over rows of dy (nullable; k = 0
 * computes db alone).  x [rows, k] (row stride ldx), dy [rows, n_out] (row
 * stride ldy); k <= 64, n_out <= 128, k * n_out + n_out <= 1280.  Fixed
 * summation order: deterministic.  workspace: ..._workspace_bytes. */
int64_t mmpde_rows_grad_weight_workspace_bytes(int64_t rows, int k, int n_out);
int mmpde_rows_grad_weight(const float *x, int64_t ldx, int64_t rows, int k, const float *dy, int64_t ldy,
                           int n_out, float *dw, float *db, float *workspace, int64_t workspace_bytes,
                           mmpde_stream_t stream);

/* BatchNorm1d in training mode over rows [n, C] of x + res (res nullable; the
 * residual add of GNN_Layer_FS_2D, norm(h + update), gnn_2d.py:69; the
 * embedding's BatchNorm1d, gnn_2d.py:101,105): batch mean and biased variance
 * (Welford per thread, Chan merges in a fixed order), y = (x + res - mean) /
 * sqrt(var + eps) * weight + bias (weight / bias nullable), running_mean /
 * running_var (nullable) <- factor * (mean, unbiased var) + (1 - factor) * old.
 * stats [4 C] receives mean, invstd and the per-channel affine (kept for the
 * backward).  C % 4 == 0, C <= 1024; 16-byte aligned pointers.  workspace:
 * mmpde_batch_norm_rows_workspace_bytes(n, C) (+ 3 C floats for the backward). */
int64_t mmpde_batch_norm_rows_workspace_bytes(int64_t n, int C);
int mmpde_batch_norm_rows_train(const float *x, const float *res, int64_t n, int C, const float *weight,
                                const float *bias, float eps, float factor, float *running_mean,
                                float *running_var, float *y, float *stats, float *workspace,
                                int64_t workspace_bytes, mmpde_stream_t stream);
/* Its backward: dx = w invstd (dy - mean(dy) - xhat mean(dy xhat)) (the input
 * gradient of x and of res alike), dweight = sum dy xhat, dbias = sum dy
 * (both nullable), from the forward's stats. */
int mmpde_batch_norm_rows_backward(const float *x, const float *res, const float *dy, int64_t n, int C,
                                   const float *weight, const float *stats, float *dx, float *dweight,
                                   float *dbias, float *workspace, int64_t workspace_bytes,
                                   mmpde_stream_t stream);

/* Row GEMMs of the training path: the Linears of the train-mode GNN
 * (message_net_1 as its target / source halves, update_net_1 / _2, the
 * embedding; gnn_2d.py:53-69,99-106) and ItpNet's MLPs (interpolate.py:79-93),
 * forward and input gradient, replacing the library GEMMs torch autograd
 * would call under loss.backward() (train_helper_2d.py:126).  Exact fp32
 * products on v_mfma_f32_32x32x2_f32, deterministic.
 *
 * mmpde_rgemm: for each output part p (1 or 2 blocks of <= 128 columns,
 * ncols[p] of them) and row i < m, column c < ncols[p]:
 *   y = sum_{h<2} sum_{k<kh} A_h[i][k] * B_h(p, k, c)  (+ bias[p][c])
 *       (+ xscale[p] * sum_{e<ns[p]} xs[i][e] * XW(p, e, c))
 *   relu (relu != 0); y = omask[p][i][c] > 0 ? y : 0 (omask nullable);
 *   out[p][i][c] = y, or += y with accumulate[p].
 * A_h[i][k] = a[h][i * lda[h] + k], times (amask[h][...] > 0) when amask[h] is
 * given (same layout).  B: layout NT -> w[h][(wc[p] + c) * ldw + wk[p] + k]
 * (a Linear's weight [out, in]: y = x W^T); layout NN ->
 * w[h][(wk[p] + k) * ldw + wc[p] + c] (y = g W, the input gradient).  K halves
 * of kh columns each (kh = 0: the small segment alone); ns[p] <= 4 more input
 * columns with XW(p, e, c) = xw[p][c * ldxw + e] (NT), xw[p][e * ldxw + c] (NN). */
#define MMPDE_RGEMM_NT 0
#define MMPDE_RGEMM_NN 1
typedef struct mmpde_rgemm_args {
    int64_t m;
    int kh, layout;
    const float *w[2];
    int64_t ldw;
    const float *a[2];
    const float *amask[2];
    int64_t lda[2];
    int parts;
    float *out[2];
    int64_t ldo[2], wc[2], wk[2];
    int ncols[2];
    const float *bias[2];
    const float *omask[2];
    int64_t ldom[2];
    int accumulate[2];
    int relu;
    const float *xs; /* [m, >= ns] small input segment (row stride ldxs) */
    int64_t ldxs;
    int ns[2];
    const float *xw[2];
    int64_t ldxw;
    float xscale[2];
} mmpde_rgemm_args;
int mmpde_rgemm(const mmpde_rgemm_args *g, mmpde_stream_t stream);

/* Weight / bias gradient over the rows (K = m reduction) of a Linear with
 * gcols <= 128 outputs: with G = g * (gmask > 0) ([m, gcols], row stride ldg;
 * gmask nullable, same layout):
 *   dw[c][dwcol[s] + j] = sum_i G[i][c] x[s][i][j]      (segments s < nseg <= 3
 *                         of kx[s] columns, row stride ldx[s])
 *   dw[c][dwcol_s + e] (+)= sign_s * sum_i G[i][c] xs[i][e]   (e < ns <= 4;
 *                         accumulate_s adds to dw instead of storing)
 *   db[c] = sum_i G[i][c]                            (db nullable)
 * Rows are summed in fixed chunks of `chunk_rows` (partials in the workspace,
 * then added in chunk order): deterministic.  workspace:
 * mmpde_rgemm_tn_workspace_bytes(m, chunk_rows, sum over s of kx[s] rounded
 * up to 64, + ns + 1). */
typedef struct mmpde_rgemm_tn_args {
    int64_t m;
    int chunk_rows, gcols;
    const float *g;
    const float *gmask;
    int64_t ldg;
    int nseg;
    const float *x[3];
    int64_t ldx[3];
    int kx[3];
    int64_t dwcol[3];
    const float *xs;
    int64_t ldxs;
    int ns;
    int64_t dwcol_s;
    float sign_s;
    int accumulate_s;
    float *dw;
    int64_t lddw;
    float *db;
} mmpde_rgemm_tn_args;
int64_t mmpde_rgemm_tn_workspace_bytes(int64_t m, int chunk_rows, int cols);
int mmpde_rgemm_tn(const mmpde_rgemm_tn_args *g, void *workspace, int64_t workspace_bytes,
                   mmpde_stream_t stream);

/* Skinny row maps (one side of the map narrow: the Conv1d head's windows,
 * gnn_2d.py:108-114; the embedding's first Linear, gnn_2d.py:99-106; ItpNet's
 * 62-wide input layer, interpolate.py:79-93), forward and input gradient, on
 * the VALU (exact fp32 products summed in a fixed order; the map staged in
 * LDS).  layout MMPDE_RGEMM_NT: y[i][o] = bias[o] + sum_{k<ki} x[i][k] w[o *
 * ldw + k] for o < no (bias nullable; y = x W^T + b, W [no, ki]).  layout
 * MMPDE_RGEMM_NN: y[i][c] = sum_{o<no} x[i][o] w[o * ldw + c] for c < ki (bias
 * null; dX = dY W, W [no, ki]).  ki, no <= 128; rows i < n with strides ldx /
 * ldy. */
int mmpde_rows_small(const float *x, int64_t ldx, int64_t n, int ki, const float *w, int64_t ldw, int layout,
                     const float *bias, int no, float *y, int64_t ldy, mmpde_stream_t stream);

/* Training backward of the few-row linears (res_cut's MLP, interpolate.py:
 * 54-60,95-97, M = B rows; reference loss.backward(), train_helper_2d.py:126):
 *   mmpde_outer_rows: dw[i][j] = sum_{r<m} g[r][i] x[r][j], db[i] = sum_r
 *     g[r][i] (db nullable; r ascending, any m: rows staged 32 at a time): the
 *     weight / bias gradient;
 *   mmpde_transpose: y[c][r] = x[r][c] (rows x cols; W^T for dX = dY W through
 *     mmpde_linear_skinny);
 *   mmpde_tanh_bwd: dz[i] = dy[i] (1 - t[i]^2) (t = the forward's tanh output). */
int mmpde_outer_rows(const float *g, int64_t ldg, const float *x, int64_t ldx, int m, int64_t n, int64_t k,
                     float *dw, int64_t lddw, float *db, mmpde_stream_t stream);
int mmpde_transpose(const float *x, int64_t rows, int64_t cols, int64_t ldx, float *y, int64_t ldy,
                    mmpde_stream_t stream);
int mmpde_tanh_bwd(const float *dy, const float *t, int64_t n, float *dz, mmpde_stream_t stream);

/* The Conv1d head in train mode (gnn_2d.py:108-114,136 at time_window 1:
 * Conv1d(1, 4, 16, stride 3) -> ReLU -> Conv1d(4, 8, 12, stride 3) -> ReLU ->
 * Conv1d(8, 1, 8, stride 2) over each row of h [n, 128]; replaces the
 * output_mlp forward and its backward under loss.backward(),
 * train_helper_2d.py:126).  Weights in torch's layouts: w1 [4][1][16], b1 [4],
 * w2 [8][4][12], b2 [8], w3 [1][8][8], b3 [1].  h rows 16-B aligned (ldh % 4
 * == 0).
 *   mmpde_head_train_forward: y[i] = output_mlp(h[i]) (one value per row).
 *   mmpde_head_train_backward: from dy[i] = dL/dy[i]: dh[i][:] = dL/dh[i]
 *     (written; rows lddh apart, 16-B aligned) and grads[0 ..
 *     MMPDE_HEAD_TRAIN_GRADS) = [dW1 | db1 | dW2 | db2 | dW3 | db3] (torch
 *     layouts, concatenated); per-row terms summed over 64-row groups by a
 *     fixed butterfly, the groups in order: deterministic.  workspace >=
 *     mmpde_head_train_workspace_bytes(n). */
#define MMPDE_HEAD_TRAIN_GRADS 525
int64_t mmpde_head_train_workspace_bytes(int64_t n);
int mmpde_head_train_forward(const float *h, int64_t ldh, int64_t n, const float *w1, const float *b1,
                             const float *w2, const float *b2, const float *w3, const float *b3, float *y,
                             mmpde_stream_t stream);
int mmpde_head_train_backward(const float *h, int64_t ldh, int64_t n, const float *w1, const float *b1,
                              const float *w2, const float *b2, const float *w3, const float *b3,
                              const float *dy, float *dh, int64_t lddh, float *grads, float *workspace,
                              int64_t workspace_bytes, mmpde_stream_t stream);

/* out[n] = out_scale * output_mlp(h[:, None]) */
int mmpde_gnn_head(const float *h, int64_t n, const mmpde_gnn_head_params *p, float *out,
                   mmpde_stream_t stream);

/* Whole MP_PDE_Solver_2D.forward (gnn_2d.py:119-141): embed, n_layers layers,
 * head.  layers: array of n_layers parameter blocks.  workspace >=
 * mmpde_gnn_workspace_bytes(n). */
int mmpde_gnn_forward(const float *u, const float *pos, int64_t n, int k, const int32_t *nbr,
                      mmpde_gnn_scales sc, const mmpde_gnn_embed_params *emb,
                      const mmpde_gnn_layer_params *layers, int n_layers,
                      const mmpde_gnn_head_params *head, void *workspace, float *out,
                      mmpde_stream_t stream);

/* Arithmetic of the per-edge message_net_2 GEMM (the dominant work).
 * F32   : v_mfma_f32_16x16x4_f32, exact fp32 products, fp32 accumulate
 *         (bit-for-bit a k-ordered fmaf chain).
 * F16X3 : fp32-emulating split GEMM (Ootomo & Yokota 2022 style): every fp32
 *         operand x is scaled by a power of two (per weight column; per
 *         neighbour slot for the activations) and split into fp16 hi + lo
 *         (x = hi + lo to 2^-22 relative); the product uses hi*hi + hi*lo +
 *         lo*hi on v_mfma_f32_16x16x32_f16 with fp32 accumulation.  Applies
 *         to every GEMM of a layer (edge message_net_2 and the node
 *         GEMMs update_net_1/2, message_net_1; activations scaled per
 *         neighbour slot tile / per node row).  Error vs fp64 is measured
 *         beside F32 in tests/test_gpu_precision.py. */
#define MMPDE_EDGE_GEMM_F32 0
#define MMPDE_EDGE_GEMM_F16X3 1

/* Execution options of mmpde_gnn_forward_ex (NULL = F32, no events).  Each
 * layer is two launches: the edge stage (message_net_2 over every edge + mean
 * aggregation: the dominant kernel) and the node stage (update_net_1/2,
 * residual, BatchNorm and the next layer's message_net_1 node halves).  When
 * non-NULL, hipEventRecord(edge_begin[l]) / (edge_end[l]) / (node_end[l]) are
 * issued on `stream` immediately before layer l's edge stage, between the two
 * launches and after its node stage, so a caller can time exactly those
 * launches. */
typedef struct {
    void *const *edge_begin; /* n_layers hipEvent_t, or NULL */
    void *const *edge_end;   /* n_layers hipEvent_t, or NULL */
    int edge_gemm;           /* MMPDE_EDGE_GEMM_* */
    const void *packed;      /* F16X3: weight images from mmpde_gnn_pack_f16x3 for these
                                layers (caller-cached); NULL: packed per call into the
                                workspace */
    void *const *node_end;   /* n_layers hipEvent_t, or NULL */
    const int32_t *degree;   /* [n] in-degree of every target for a ragged nbr table (row i
                                holds degree[i] sources, the rest of its k entries are
                                ignored; PyG mean = sum / max(degree, 1)), e.g. from
                                mmpde_radius_graph; NULL: every row holds k */
    int64_t seg_n;           /* rows per trajectory segment (the graph's batch segments:
                                no edge crosses one); F16X3 takes the activation split
                                scale per segment, so a trajectory's output does not
                                depend on the others in the launch.  0 (or a value
                                that does not divide n, or < 32): one segment */
} mmpde_gnn_exec;

/* Most layers mmpde_gnn_forward_ex accepts (sizes the workspace's packed
 * weight region). */
#define MMPDE_GNN_MAX_LAYERS 16

/* F16X3 weight images (message_net_2, update_net_1, update_net_2 and
 * message_net_1 of every layer, split into scaled fp16 hi/lo MFMA operand
 * images + per-column scales).  Depends only on the weights: a caller packs
 * once per parameter change and passes it as mmpde_gnn_exec.packed. */
int64_t mmpde_gnn_pack_bytes(int n_layers);
int mmpde_gnn_pack_f16x3(const mmpde_gnn_layer_params *layers, int n_layers, void *pack,
                         mmpde_stream_t stream);

int mmpde_gnn_forward_ex(const float *u, const float *pos, int64_t n, int k, const int32_t *nbr,
                         mmpde_gnn_scales sc, const mmpde_gnn_embed_params *emb,
                         const mmpde_gnn_layer_params *layers, int n_layers,
                         const mmpde_gnn_head_params *head, void *workspace, float *out,
                         const mmpde_gnn_exec *exec, mmpde_stream_t stream);


/* ------------------------------------------------------------------------
 * DMM mesh mover (reference mesh/dmm_model.py, data_creator_2d.py:88-137)
 * ---------------------------------------------------------------------- */
typedef struct {
    /* tiny GNN branch, hidden h = 4, 3 layers (dmm_model.py:154-173) */
    const float *emb0_w, *emb0_b, *emb1_w, *emb1_b, *emb1_rm, *emb1_rv;
    const float *emb3_w, *emb3_b, *emb4_w, *emb4_b, *emb4_rm, *emb4_rv;
    const float *g_msg1_w[3], *g_msg1_b[3], *g_msg2_w[3], *g_msg2_b[3];
    const float *g_upd1_w[3], *g_upd1_b[3], *g_upd2_w[3], *g_upd2_b[3];
    const float *g_bn_w[3], *g_bn_b[3], *g_bn_rm[3], *g_bn_rv[3];
    int n_gnn_layers;
    const float *dec0_w, *dec0_b, *dec1_w, *dec1_b; /* decoding_mlp DenseNet[4,128,1] */
    const float *om0_w, *om0_b, *om2_w, *om2_b, *om4_w, *om4_b; /* output_mlp N->512->256->512 */
    float eps;
} mmpde_dmm_graph_branch;

typedef struct {
    /* ConvNet(s, 7) branch (dmm_model.py:48-81) */
    const float *c0_w, *c0_b, *c1_w, *c1_b, *c2_w, *c2_b, *c3_w, *c3_b;
    const float *fc2_w, *fc2_b, *fc3_w, *fc3_b;
    int s;
} mmpde_dmm_array_branch;

typedef struct {
    /* trunk DenseNet [2, th, L] and out_nn DenseNet [2L, L', 1] */
    const float *t0_w, *t0_b; /* [th, 2] */
    const float *t1_w, *t1_b; /* [L, th] */
    int th, latent;           /* th <= 64, latent = L (branch width) */
    const float *o0_w, *o0_b; /* [L', 2L] */
    const float *o1_w;        /* [1, L']  (its bias does not reach d(phi)/d(xi)) */
    int hidden;               /* L' */
} mmpde_dmm_head;

/* Workspace bytes for mmpde_dmm_mesh_* with B trajectories of N points. */
int64_t mmpde_dmm_workspace_bytes(int64_t batches, int64_t n_per, int latent, int hidden);

/* x = xi + d(phi)/d(xi), phi = DMM(u, xi), graph mode (cylinder).
 * Replaces moving_mesh_tri (data_creator_2d.py:115-137) incl. the two
 * autograd.grad calls, by an analytic VJP.
 * u [B, N]; grid [N, 2] = pde.ori_grid (= xi for every trajectory);
 * grid_nbr [N, 35] int32 LOCAL kNN-35 table of the fixed grid
 * (dmm_model.py:222-234, built once with mmpde_knn_graph(batches=1));
 * mesh_out [B*N, 2]. */
int mmpde_dmm_mesh_graph(const float *u, const float *grid, int64_t batches, int64_t n_per,
                         const int32_t *grid_nbr, int k, const mmpde_dmm_graph_branch *br,
                         const mmpde_dmm_head *hd, void *workspace, float *mesh_out,
                         mmpde_stream_t stream);

/* Array mode (Burgers): u [B, s, s]; xi [N, 2] (np.meshgrid xy order,
 * data_creator_2d.py:94-100).  N = s*s on the MM-PDE path; a coarser or finer
 * xi is allowed (u bilinearly pre-resampled to s x s,
 * data_creator_2d.py:102-103, mmpde_resample_bilinear), with the workspace
 * sized by mmpde_dmm_workspace_bytes(B, max(N, s*s), ...). */
int mmpde_dmm_mesh_array(const float *u, const float *xi, int64_t batches, int64_t n_per,
                         const mmpde_dmm_array_branch *br, const mmpde_dmm_head *hd,
                         void *workspace, float *mesh_out, mmpde_stream_t stream);

/* The grid side of the DMM head -- trunk(xi), Q = Wt.trunk and J = dQ/dxi
 * (dmm_model.py:196-199's trunk and out_nn first layer) -- depends on xi and the
 * weights only, not on u.  A rollout over a fixed grid prepares it once:
 * cache >= mmpde_dmm_head_cache_bytes(N, hd->hidden) bytes (16-B aligned),
 * workspace as for mmpde_dmm_mesh_*.  The _cached variants read it instead of
 * recomputing it (same xi and weights required; results are identical). */
int64_t mmpde_dmm_head_cache_bytes(int64_t n_per, int hidden);
int mmpde_dmm_head_prepare(const float *xi, int64_t n_per, const mmpde_dmm_head *hd,
                           void *workspace, void *cache, mmpde_stream_t stream);
int mmpde_dmm_mesh_graph_cached(const float *u, const float *grid, int64_t batches,
                                int64_t n_per, const int32_t *grid_nbr, int k,
                                const mmpde_dmm_graph_branch *br, const mmpde_dmm_head *hd,
                                const void *head_cache, void *workspace, float *mesh_out,
                                mmpde_stream_t stream);
int mmpde_dmm_mesh_array_cached(const float *u, const float *xi, int64_t batches, int64_t n_per,
                                const mmpde_dmm_array_branch *br, const mmpde_dmm_head *hd,
                                const void *head_cache, void *workspace, float *mesh_out,
                                mmpde_stream_t stream);

/* DMM.forward (dmm_model.py:185-219) in two calls, for callers that need phi
 * itself (DMM evaluation, dmm_utils.py) rather than the moved mesh.
 * The branch alone: branch_out [B, L] (L = hd->latent) from u on the fixed
 * grid (graph: u [B, N], grid / grid_nbr as for mmpde_dmm_mesh_graph) or from
 * u [B, s, s] (array: ConvNet.forward, dmm_model.py:65-81); workspace as for
 * mmpde_dmm_mesh_* (array: N = s*s). */
int mmpde_dmm_branch_graph(const float *u, const float *grid, int64_t batches, int64_t n_per,
                           const int32_t *grid_nbr, int k, const mmpde_dmm_graph_branch *br,
                           const mmpde_dmm_head *hd, void *workspace, float *branch_out,
                           mmpde_stream_t stream);
int mmpde_dmm_branch_array(const float *u, int64_t batches, const mmpde_dmm_array_branch *br,
                           const mmpde_dmm_head *hd, void *workspace, float *branch_out,
                           mmpde_stream_t stream);
/* phi[i] = out_nn(cat(branch[b], trunk(grid[i])))  with b = i / (n_grid / B)
 * (the reference's branch.repeat over grid rows, dmm_model.py:187-190,210-213);
 * grid [n_grid, 2] (n_grid a multiple of B); o1_b = out_nn.layers.1.bias
 * (nullable: 0); phi_out [n_grid]; second_out [n_grid, L'] = the tanh layer
 * (the rf=True second output), nullable.  workspace >=
 * mmpde_dmm_phi_workspace_bytes(B, n_grid, L, L', th) bytes, 16-B aligned. */
int64_t mmpde_dmm_phi_workspace_bytes(int64_t batches, int64_t n_grid, int latent, int hidden, int th);
int mmpde_dmm_phi(const float *branch, int64_t batches, const float *grid, int64_t n_grid,
                  const mmpde_dmm_head *hd, const float *o1_b, void *workspace, float *phi_out,
                  float *second_out, mmpde_stream_t stream);

/* ------------------------------------------------------------------------
 * ItpNet interpolation (reference interpolate.py:77-93 + data_creator_2d.py:80-83)
 * ---------------------------------------------------------------------- */
typedef struct {
    /* Linear(62,128) tanh Linear(128,64) tanh Linear(64,30): ItpNet.layers
     * (mode '1') or ItpNet.layers2 (mode '2') */
    const float *w0, *b0, *w1, *b1, *w2, *b2;
} mmpde_itp_mlp;

/* Bytes of the packed weight image mmpde_itp_pack writes. */
int64_t mmpde_itp_pack_bytes(void);
/* Re-lay the MLP weights into the MFMA operand image used by mmpde_itp_interp. */
int mmpde_itp_pack(const mmpde_itp_mlp *mlp, void *packed, mmpde_stream_t stream);

/* out[b*Nq+q] = sum_e ItpNet(nbrs, q)[e] * vals[b*Ns + idx[q,e]] (+ addend).
 * src [B*Ns,2], vals [B*Ns], qry [B*Nq,2], idx [B*Nq,30] LOCAL (from
 * mmpde_knn_query with k = 30); addend nullable [B*Nq]. */
int mmpde_itp_interp(const float *src, const float *vals, const float *qry, const int32_t *idx,
                     int64_t batches, int64_t n_src, int64_t n_qry, const void *packed,
                     const float *addend, float *out, mmpde_stream_t stream);
/* The same with a second addend, added last: out = (addend + sum) + addend2
 * (the rollout's pred = interpolate_pred(...) + model(graph_uniform),
 * train_helper_2d.py:178-185, in one launch); both nullable. */
int mmpde_itp_interp_ex(const float *src, const float *vals, const float *qry, const int32_t *idx,
                        int64_t batches, int64_t n_src, int64_t n_qry, const void *packed,
                        const float *addend, const float *addend2, float *out, mmpde_stream_t stream);

/* ------------------------------------------------------------------------
 * DMM training (reference mesh/dmm_utils.py)
 * ---------------------------------------------------------------------- */

/* Softmax kernel smoother (reference mesh/dmm_utils.py:233-249 interpolate with
 * scale = n on the n x n linspace grid, :251-267 interpolate_tri with scale =
 * sqrt(n) on a mesh of n points): out[q] = sum_j vals[j] softmax_j(-scale *
 * |pts[j] - qry[q]|).  pts [pts_sets, n_pts, 2], vals [val_sets, n_pts],
 * qry [n_q, 2]: query q uses point set q / (n_q / pts_sets) and value set
 * q / (n_q / val_sets) (both must divide n_q).  _grad: grad_qry [n_q, 2] =
 * grad_out[q] * d out[q] / d qry[q] (the VJP torch.norm / softmax autograd
 * gives, 0 for the direction of a point at distance 0). */
int mmpde_softmax_interp(const float *pts, int64_t n_pts, int64_t pts_sets, const float *vals,
                         int64_t val_sets, const float *qry, int64_t n_q, float scale, float *out,
                         mmpde_stream_t stream);
int mmpde_softmax_interp_grad(const float *pts, int64_t n_pts, int64_t pts_sets, const float *vals,
                              int64_t val_sets, const float *qry, int64_t n_q, float scale,
                              const float *grad_out, float *grad_qry, mmpde_stream_t stream);

#ifdef __cplusplus
}
#endif
#endif /* MMPDE_HIP_H */
