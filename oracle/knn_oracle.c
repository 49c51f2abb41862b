/*
 * oracle/knn_oracle.c -- TEST INFRASTRUCTURE ONLY (parity checker, never shipped).
 *
 * CPU restatement of the two nearest-neighbour searches on the MM-PDE hot path.
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load
 * the shared object built from this file.
 *
 * 1. knn_graph_oracle  -- restates torch_cluster 1.5.9 `knn_graph(x, k, batch,
 *    loop=False)` (pinned in reference env.yml:128; not vendored, not importable
 *    here).  Call sites: reference data_creator_2d.py:260 (moved / uniform mesh)
 *    and mesh/dmm_model.py:228 (DMM fixed grid).  Published algorithm: brute
 *    force per batch segment, search k+1 neighbours of every point among the
 *    points of its own segment, keep a best list sorted by distance with a
 *    strict `>` insertion test (so equal distances keep the lower index first),
 *    then drop the self loop.  Distance: squared L2 accumulated as
 *    `d += (x-y)*(x-y)` over the 2 dims, which nvcc's default --fmad=true
 *    contracts to d2 = fmaf(dy, dy, dx*dx).  We fix exactly that formula (and
 *    compile with -ffp-contract=off so nothing else is contracted).
 *    Output: nbr[q*k + e] = global source index of the e-th neighbour of query
 *    q, e ordered by (d2, index).  PyG's edge_index is then
 *    [nbr.flatten(), repeat(q, k)] (source row 0, target row 1).
 *    If fewer than k+1 points exist, or self is not among the k+1 best (more
 *    than k duplicates of the query point with lower indices), the degree would
 *    be ragged in the reference; we report it through the return value
 *    (number of such degenerate queries) and fill the row with the first k.
 *
 * 2. knn_query_oracle -- restates scikit-learn 1.3.0
 *    `NearestNeighbors(n_neighbors=k).fit(P).kneighbors(Q)` (env.yml:135) as
 *    called per trajectory at reference data_creator_2d.py:66-78.  sklearn
 *    upcasts float32 input to float64 and ranks by the reduced distance
 *    rdist = dx*dx + dy*dy (no FMA in its generic x86-64 wheels); results are
 *    sorted ascending.  sklearn leaves the order of exactly-equal distances
 *    to its heap; we fix (rdist, index) ascending.  Queries may coincide with a
 *    source point (distance 0); no self exclusion.
 *
 * 3. radius_graph_oracle -- restates torch_cluster 1.5.9 `radius_graph(x, r,
 *    batch, loop=False, max_num_neighbors=32)` (reference data_creator_2d.py:
 *    257-258, connect_edge='radius'; r from :195 / :226), CUDA path (the
 *    reference runs on cuda:0).  Published algorithm: radius_graph calls
 *    radius(x, x, r, batch, batch, max_num_neighbors + 1); its kernel scans the
 *    query's segment in index order, appends every point with squared distance
 *    (accumulated as in knn_graph: fmaf(dy, dy, dx*dx)) strictly below r*r
 *    (squared in double on the host, handed to the kernel as float) and stops
 *    after max_num_neighbors + 1 points; radius_graph then masks the self loop.
 *    Output: nbr [n, max_nn + 1] global sources in scan order padded with -1,
 *    deg [n] = entries kept.
 *
 * Parity status: torch_cluster boundary is "parity unpinned" (no reference
 * fixture exists, running the reference was denied -- SURVEY.md §8(c));
 * the sklearn boundary is pinned against sklearn 1.7.2 fixtures on tie-free
 * inputs (tests/golden/make_golden.py).
 */
#include <stdint.h>
#include <math.h>
#include <stdlib.h>
#include <string.h>

#pragma STDC FP_CONTRACT OFF

static inline float d2_graph(float qx, float qy, float px, float py) {
    /* torch_cluster: tmp = 0; tmp += (x-y)*(x-y) per dim, contracted by nvcc */
    float dx = px - qx;
    float dy = py - qy;
    float d = dx * dx;
    return fmaf(dy, dy, d);
}

/* insertion into a (dist, idx)-sorted best list of length kk, strict '>' test */
static inline void insert_f(float *bd, int64_t *bi, int kk, float d, int64_t j) {
    if (!(bd[kk - 1] > d)) return; /* fast reject; identical result */
    for (int e1 = 0; e1 < kk; ++e1) {
        if (bd[e1] > d) {
            for (int e2 = kk - 1; e2 > e1; --e2) {
                bd[e2] = bd[e2 - 1];
                bi[e2] = bi[e2 - 1];
            }
            bd[e1] = d;
            bi[e1] = j;
            return;
        }
    }
}

/* pos: [batches*n_per, 2]; nbr_out: [batches*n_per, k] (global indices)
 * returns the number of degenerate queries (ragged degree in the reference). */
int64_t knn_graph_oracle(const float *pos, int64_t batches, int64_t n_per, int k,
                         int64_t *nbr_out) {
    int kk = k + 1;
    float *bd = (float *)malloc(sizeof(float) * kk);
    int64_t *bi = (int64_t *)malloc(sizeof(int64_t) * kk);
    int64_t degenerate = 0;
    for (int64_t b = 0; b < batches; ++b) {
        const float *P = pos + 2 * b * n_per;
        for (int64_t q = 0; q < n_per; ++q) {
            for (int e = 0; e < kk; ++e) { bd[e] = 1e10f; bi[e] = -1; }
            float qx = P[2 * q], qy = P[2 * q + 1];
            for (int64_t j = 0; j < n_per; ++j) {
                float d = d2_graph(qx, qy, P[2 * j], P[2 * j + 1]);
                insert_f(bd, bi, kk, d, j);
            }
            int64_t *row = nbr_out + (b * n_per + q) * k;
            int self_seen = 0;
            for (int e = 0; e < kk; ++e) self_seen |= (bi[e] == q);
            /* drop the self loop (mask row != col); without it the reference keeps
             * k+1 edges -- here the first k, counted as degenerate */
            int w = 0;
            for (int e = 0; e < kk && w < k; ++e) {
                if (bi[e] == q) continue;
                row[w++] = (bi[e] < 0) ? -1 : b * n_per + bi[e];
            }
            if (!self_seen || bi[kk - 1] < 0) degenerate++;
        }
    }
    free(bd);
    free(bi);
    return degenerate;
}

static inline void insert_d(double *bd, int64_t *bi, int kk, double d, int64_t j) {
    /* full (d, idx) order: a later j with equal d goes after -> strict '>' */
    if (!(bd[kk - 1] > d)) return; /* fast reject; identical result */
    for (int e1 = 0; e1 < kk; ++e1) {
        if (bd[e1] > d) {
            for (int e2 = kk - 1; e2 > e1; --e2) {
                bd[e2] = bd[e2 - 1];
                bi[e2] = bi[e2 - 1];
            }
            bd[e1] = d;
            bi[e1] = j;
            return;
        }
    }
}

/* src: [batches*n_src, 2], qry: [batches*n_qry, 2]; idx_out [batches*n_qry, k]
 * holds LOCAL source indices (0..n_src-1), as sklearn returns per fit. */
int64_t knn_query_oracle(const float *src, const float *qry, int64_t batches,
                         int64_t n_src, int64_t n_qry, int k, int64_t *idx_out) {
    double *bd = (double *)malloc(sizeof(double) * k);
    int64_t *bi = (int64_t *)malloc(sizeof(int64_t) * k);
    for (int64_t b = 0; b < batches; ++b) {
        const float *S = src + 2 * b * n_src;
        const float *Q = qry + 2 * b * n_qry;
        for (int64_t q = 0; q < n_qry; ++q) {
            for (int e = 0; e < k; ++e) { bd[e] = INFINITY; bi[e] = -1; }
            double qx = (double)Q[2 * q], qy = (double)Q[2 * q + 1];
            for (int64_t j = 0; j < n_src; ++j) {
                double dx = (double)S[2 * j] - qx;
                double dy = (double)S[2 * j + 1] - qy;
                double a = dx * dx;
                double c = dy * dy;
                insert_d(bd, bi, k, a + c, j);
            }
            memcpy(idx_out + (b * n_qry + q) * k, bi, sizeof(int64_t) * k);
        }
    }
    free(bd);
    free(bi);
    return 0;
}

/* pos: [batches*n_per, 2]; nbr_out [batches*n_per, max_nn+1]; deg_out [batches*n_per] */
void radius_graph_oracle(const float *pos, int64_t batches, int64_t n_per, float r, int max_nn,
                         int64_t *nbr_out, int64_t *deg_out) {
    const float r2 = (float)((double)r * (double)r);
    const int w = max_nn + 1;
    for (int64_t b = 0; b < batches; ++b) {
        const float *P = pos + 2 * b * n_per;
        for (int64_t q = 0; q < n_per; ++q) {
            int64_t *row = nbr_out + (b * n_per + q) * w;
            int taken = 0, kept = 0;
            for (int64_t j = 0; j < n_per && taken < w; ++j) {
                if (d2_graph(P[2 * q], P[2 * q + 1], P[2 * j], P[2 * j + 1]) < r2) {
                    taken++;
                    if (j != q) row[kept++] = b * n_per + j;
                }
            }
            deg_out[b * n_per + q] = kept;
            for (int e = kept; e < w; ++e) row[e] = -1;
        }
    }
}
