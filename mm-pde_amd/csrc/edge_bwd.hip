// Backward of the GNN edge stage (training; reference train_helper_2d.py:114-126
// backpropagates loss.backward() through model / model_b, whose message passing
// is gnn_2d.py:53-63 + PyG aggr='mean').  Forward, per target i and in-edge e
// from source j = nbr[i, e] (e < deg_i):
//
//   z1 = a_i + b_j,  m1 = relu(z1),  z2 = W2 m1 + b2,  m = relu(z2),
//   mean_i = (1 / max(deg_i, 1)) sum_e m
//
// Given g = dL/dmean [n, 128] this computes
//
//   gz2 = g_i / max(deg_i, 1) * [z2 > 0],  gm1 = W2^T gz2,  gz1 = gm1 * [z1 > 0]
//   dL/da_i  = sum_e gz1                  (target side, summed in registers)
//   dL/db_j  = sum_{(i, e): nbr[i,e] = j} gz1   (source side: per-edge gz1 is
//              written out and summed per source over the reverse adjacency by
//              edge_source_sum_kernel, in a fixed order)
//   dL/dW2   = sum_e gz2 m1^T,  dL/db2 = sum_e gz2   (per-workgroup partials,
//              reduced in workgroup order by partial_sum_kernel)
//
// Nothing is stored by the forward: z1, z2 are recomputed here.  Exact fp32
// products on v_mfma_f32_16x16x4_f32 (the three 16 x 128 x 128 GEMMs of a
// neighbour slot: z2, gm1 and the dW2 outer products); no atomics, so the
// gradients are deterministic.
#include "common.hpp"

namespace {

constexpr int BH = 128;  // hidden width
constexpr int BT = 16;   // targets per tile
constexpr int BWS = BH + 8;  // LDS row stride (floats): 2-way bank aliasing for both row- and column-walks

struct EdgeBwdArgs {
    const float *a, *b;
    const int32_t *nbr;
    const int32_t *deg;  // nullable: every row has k in-edges
    int64_t n;
    int k, ntiles;
    const float *w2, *b2;  // message_net_2.0 weight [128 out][128 in], bias
    const float *gmean;    // [n, 128]
    float *ga;             // [n, 128]
    float *gz1;            // [n * k, 128] per edge (target-major, as nbr)
    float *pw2, *pb2;      // [grid][128][128], [grid][128] partials
};

__global__ __launch_bounds__(256, 1) void edge_bwd_kernel(EdgeBwdArgs p) {
    __shared__ float w2s[BH * BWS];    // W2 [c][kk], row stride BWS
    __shared__ float at[BT * BWS];     // a rows of the tile
    __shared__ float z1s[BT * BWS];    // z1 of the current slot
    __shared__ float gz2s[BT * BWS];   // gz2 of the current slot
    __shared__ float gms[BT * BWS];    // g / deg of the tile
    __shared__ int srcs[BT];
    const int tid = threadIdx.x, wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
    const int r = lane & 15, g = lane >> 4;
    const int64_t nmax = p.n - 1;
    const int k = p.k;
    for (int i = tid; i < BH * BH / 4; i += 256)
        *(float4 *)&w2s[(i >> 5) * BWS + 4 * (i & 31)] = ((const float4 *)p.w2)[i];
    // persistent accumulators: dW2 tiles (c tile 2 wave + ci, kk tile kj), db2
    f32x4 dw[2][8];
#pragma unroll
    for (int ci = 0; ci < 2; ++ci)
#pragma unroll
        for (int kj = 0; kj < 8; ++kj) dw[ci][kj] = (f32x4){0.0f, 0.0f, 0.0f, 0.0f};
    float db[2] = {0.0f, 0.0f};
    for (int tile = blockIdx.x; tile < p.ntiles; tile += gridDim.x) {
        const int64_t row0 = (int64_t)tile * BT;
        __syncthreads();  // the previous tile's LDS readers are done
        for (int i = tid; i < BT * BH / 4; i += 256) {
            const int rr = i >> 5, c4 = i & 31;
            const int64_t row = min(row0 + rr, nmax);
            const bool live = row0 + rr < p.n;
            const int dgv = p.deg ? p.deg[row] : k;
            const float inv_deg = live ? 1.0f / (float)max(dgv, 1) : 0.0f;
            const float4 av = ((const float4 *)(p.a + row * BH))[c4];
            const float4 gv = ((const float4 *)(p.gmean + row * BH))[c4];
            *(float4 *)&at[rr * BWS + 4 * c4] = av;
            *(float4 *)&gms[rr * BWS + 4 * c4] =
                make_float4(gv.x * inv_deg, gv.y * inv_deg, gv.z * inv_deg, gv.w * inv_deg);
        }
        // dL/da accumulators: rows 4 g + t, columns 16 (2 wave + ci) + r
        f32x4 gacc[2] = {(f32x4){0.0f, 0.0f, 0.0f, 0.0f}, (f32x4){0.0f, 0.0f, 0.0f, 0.0f}};
        int dgr[4];
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            const int64_t row = min(row0 + 4 * g + t, nmax);
            dgr[t] = p.deg ? p.deg[row] : k;
        }
        for (int e = 0; e < k; ++e) {
            if (tid < BT) {
                const int64_t row = min(row0 + tid, nmax);
                const int s = p.nbr[row * k + e];
                srcs[tid] = (s < 0 || s > nmax) ? 0 : s;  // padded / malformed entries: masked below
            }
            __syncthreads();
            // z1 = a + b_src
            for (int i = tid; i < BT * BH / 4; i += 256) {
                const int rr = i >> 5, c4 = i & 31;
                const float4 bv = ((const float4 *)(p.b + (int64_t)srcs[rr] * BH))[c4];
                float *zp = &z1s[rr * BWS + 4 * c4];
                const float *ap = &at[rr * BWS + 4 * c4];
                zp[0] = ap[0] + bv.x;
                zp[1] = ap[1] + bv.y;
                zp[2] = ap[2] + bv.z;
                zp[3] = ap[3] + bv.w;
            }
            __syncthreads();
            // z2 = W2 relu(z1) + b2 and gz2 = g / deg [z2 > 0]: wave owns columns
            // c of tiles 2 wave, 2 wave + 1 (A = relu(z1)[row][kk], B = W2[c][kk])
            float gz2v[2][4];
#pragma unroll
            for (int ci = 0; ci < 2; ++ci) {
                const int c = 16 * (2 * wave + ci) + r;
                f32x4 acc = (f32x4){0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll 8
                for (int s = 0; s < BH / 4; ++s) {
                    const float av = fmaxf(z1s[r * BWS + 4 * s + g], 0.0f);
                    const float bv = w2s[c * BWS + 4 * s + g];
                    acc = mfma16(av, bv, acc);
                }
                const float bb = p.b2[c];
#pragma unroll
                for (int t = 0; t < 4; ++t) {
                    const int rr = 4 * g + t;
                    const bool on = e < dgr[t] && acc[t] + bb > 0.0f;
                    const float v = on ? gms[rr * BWS + c] : 0.0f;
                    gz2v[ci][t] = v;
                    gz2s[rr * BWS + c] = v;
                }
            }
#pragma unroll
            for (int ci = 0; ci < 2; ++ci)
                db[ci] += gz2v[ci][0] + gz2v[ci][1] + gz2v[ci][2] + gz2v[ci][3];
            __syncthreads();
            // gm1 = W2^T gz2 (A = gz2[row][c], B = W2[c][kk]); wave owns kk tiles
            // 2 wave, 2 wave + 1; gz1 = gm1 [z1 > 0]
#pragma unroll
            for (int ci = 0; ci < 2; ++ci) {
                const int kk = 16 * (2 * wave + ci) + r;
                f32x4 acc = (f32x4){0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll 8
                for (int s = 0; s < BH / 4; ++s) {
                    const float av = gz2s[r * BWS + 4 * s + g];
                    const float bv = w2s[(4 * s + g) * BWS + kk];
                    acc = mfma16(av, bv, acc);
                }
#pragma unroll
                for (int t = 0; t < 4; ++t) {
                    const int rr = 4 * g + t;
                    const float v = z1s[rr * BWS + kk] > 0.0f ? acc[t] : 0.0f;
                    gacc[ci][t] += v;
                    if (row0 + rr < p.n) p.gz1[((row0 + rr) * k + e) * BH + kk] = v;
                }
            }
            // dW2[c][kk] += sum_rows gz2[row][c] relu(z1)[row][kk]  (K = the 16 rows)
#pragma unroll
            for (int ci = 0; ci < 2; ++ci) {
                const int c = 16 * (2 * wave + ci) + r;
#pragma unroll
                for (int kj = 0; kj < 8; ++kj) {
                    const int kk = 16 * kj + r;
#pragma unroll
                    for (int s = 0; s < 4; ++s) {
                        // A[c][row] = gz2[row][c] (lane: c = r, row = 4 s + g); B[row][kk]
                        const float av = gz2s[(4 * s + g) * BWS + 16 * (2 * wave + ci) + r];
                        const float bv = fmaxf(z1s[(4 * s + g) * BWS + kk], 0.0f);
                        dw[ci][kj] = mfma16(av, bv, dw[ci][kj]);
                    }
                }
                (void)c;
            }
            __syncthreads();  // z1s / gz2s are rewritten by the next slot
        }
#pragma unroll
        for (int ci = 0; ci < 2; ++ci) {
            const int kk = 16 * (2 * wave + ci) + r;
#pragma unroll
            for (int t = 0; t < 4; ++t) {
                const int64_t row = row0 + 4 * g + t;
                if (row < p.n) p.ga[row * BH + kk] = gacc[ci][t];
            }
        }
    }
    // partials of this workgroup: dW2 tile (c rows 4 g + t of tile 2 wave + ci, kk col)
    float *pw = p.pw2 + (int64_t)blockIdx.x * BH * BH;
#pragma unroll
    for (int ci = 0; ci < 2; ++ci)
#pragma unroll
        for (int kj = 0; kj < 8; ++kj)
#pragma unroll
            for (int t = 0; t < 4; ++t)
                pw[(16 * (2 * wave + ci) + 4 * g + t) * BH + 16 * kj + r] = dw[ci][kj][t];
    // db2: lanes g = 0..3 of a column hold disjoint rows: add them in g order
#pragma unroll
    for (int ci = 0; ci < 2; ++ci) {
        float v = db[ci];
        const float v1 = __shfl(v, r + 16, 64), v2 = __shfl(v, r + 32, 64), v3 = __shfl(v, r + 48, 64);
        if (g == 0) p.pb2[(int64_t)blockIdx.x * BH + 16 * (2 * wave + ci) + r] = ((v + v1) + v2) + v3;
    }
}

// out[j] = sum_{p in [off[j], off[j+1])} rows[edge[p]]: one wave per source
// row j, two columns per lane, in list order.
__global__ __launch_bounds__(256) void edge_source_sum_kernel(const float *__restrict__ rows,
                                                              const int64_t *__restrict__ off,
                                                              const int64_t *__restrict__ edge, int64_t n,
                                                              float *__restrict__ out) {
    const int64_t j = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (j >= n) return;
    float2 acc = make_float2(0.0f, 0.0f);
    for (int64_t q = off[j]; q < off[j + 1]; ++q) {
        const float2 v = ((const float2 *)(rows + edge[q] * BH))[lane];
        acc.x += v.x;
        acc.y += v.y;
    }
    ((float2 *)(out + j * BH))[lane] = acc;
}

// out[j][c] = sum_{p in [off[j], off[j+1])} rows[edge[p]][c] for any row width:
// one thread per (j, c), in list order.
__global__ __launch_bounds__(256) void segment_sum_kernel(const float *__restrict__ rows, int64_t width,
                                                          const int64_t *__restrict__ off,
                                                          const int64_t *__restrict__ edge, int64_t n,
                                                          float *__restrict__ out) {
    const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (t >= n * width) return;
    const int64_t j = t / width, c = t - j * width;
    float acc = 0.0f;
    for (int64_t q = off[j]; q < off[j + 1]; ++q) acc += rows[edge[q] * width + c];
    out[t] = acc;
}

// out[i] = sum_{g < G} part[g * len + i], in g order.
__global__ __launch_bounds__(256) void partial_sum_kernel(const float *__restrict__ part, int G, int64_t len,
                                                          float *__restrict__ out) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= len) return;
    float s = 0.0f;
    for (int q = 0; q < G; ++q) s += part[(int64_t)q * len + i];
    out[i] = s;
}

}  // namespace

extern "C" int64_t mmpde_gnn_edge_backward_partials(int *grid) {
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
        cus = 256;
    if (grid) *grid = cus > 0 ? cus : 256;
    return (int64_t)(cus > 0 ? cus : 256) * (BH * BH + BH);
}

extern "C" int mmpde_gnn_edge_backward(const float *a, const float *b, const int32_t *nbr, const int32_t *deg,
                                       int64_t n, int k, const float *msg2_w, const float *msg2_b,
                                       const float *grad_mean, float *grad_a, float *grad_edge,
                                       float *partials, float *grad_w2, float *grad_b2,
                                       mmpde_stream_t stream) {
    MMPDE_REQUIRE(a && b && nbr && msg2_w && msg2_b && grad_mean && grad_a && grad_edge && partials);
    MMPDE_REQUIRE(grad_w2 && grad_b2 && n > 0 && k > 0 && n <= (int64_t)INT32_MAX);
    MMPDE_REQUIRE((((uintptr_t)a | (uintptr_t)b | (uintptr_t)msg2_w | (uintptr_t)grad_mean) & 15) == 0);
    int grid = 256;
    mmpde_gnn_edge_backward_partials(&grid);
    const int64_t ntiles = (n + BT - 1) / BT;
    MMPDE_REQUIRE(ntiles < (int64_t)INT32_MAX);
    if (grid > ntiles) grid = (int)ntiles;
    float *pw2 = partials, *pb2 = partials + (int64_t)grid * BH * BH;
    EdgeBwdArgs p{a, b, nbr, deg, n, k, (int)ntiles, msg2_w, msg2_b, grad_mean, grad_a, grad_edge, pw2, pb2};
    hipStream_t st = as_stream(stream);
    hipLaunchKernelGGL(edge_bwd_kernel, dim3(grid), dim3(256), 0, st, p);
    MMPDE_RET_LAUNCH();
    hipLaunchKernelGGL(partial_sum_kernel, dim3(ceil_div(BH * BH, 256)), dim3(256), 0, st, pw2, grid,
                       (int64_t)BH * BH, grad_w2);
    hipLaunchKernelGGL(partial_sum_kernel, dim3(1), dim3(256), 0, st, pb2, grid, (int64_t)BH, grad_b2);
    MMPDE_RET_LAUNCH();
    return MMPDE_OK;
}

extern "C" int mmpde_gnn_edge_source_sum(const float *grad_edge, const int64_t *rev_off, const int64_t *rev_edge,
                                         int64_t n, float *grad_b, mmpde_stream_t stream) {
    MMPDE_REQUIRE(grad_edge && rev_off && rev_edge && grad_b && n > 0);
    hipLaunchKernelGGL(edge_source_sum_kernel, dim3((unsigned)ceil_div(n, 4)), dim3(256), 0, as_stream(stream),
                       grad_edge, rev_off, rev_edge, n, grad_b);
    MMPDE_RET_LAUNCH();
    return MMPDE_OK;
}

extern "C" int mmpde_segment_sum(const float *rows, int64_t width, const int64_t *rev_off,
                                 const int64_t *rev_edge, int64_t n, float *out, mmpde_stream_t stream) {
    MMPDE_REQUIRE(rows && rev_off && rev_edge && out && n > 0 && width > 0);
    MMPDE_REQUIRE(n * width / 256 < (int64_t)INT32_MAX);
    hipLaunchKernelGGL(segment_sum_kernel, dim3((unsigned)ceil_div(n * width, 256)), dim3(256), 0,
                       as_stream(stream), rows, width, rev_off, rev_edge, n, out);
    MMPDE_RET_LAUNCH();
    return MMPDE_OK;
}
