// DMM mesh mover on gfx950: x = xi + d(phi)/d(xi) (reference
// data_creator_2d.py:88-137, mesh/dmm_model.py:145-234).
//
// phi(b, n) = w_o . tanh(Wb . branch_b + Wt . trunk(xi_n) + b_o1) + b_o2, where
// out_nn's first Linear(2L, L') acts on cat(branch, trunk) (dmm_model.py:190,213).
// The branch depends only on the trajectory b, the trunk only on the grid point
// n (xi is the same fixed grid for every trajectory), so
//     z(b, n) = P[b] + Q[n],   P = Wb . branch + b_o1  [B, L'],  Q = Wt . trunk  [N, L']
// and the two autograd.grad calls of the reference reduce to the analytic VJP
//     d(phi)/d(xi)(b, n) = sum_k w_o[k] (1 - tanh^2 z_k) J[n, k, :],
//     J[n] = (Wt T1) diag(1 - s_n^2) T0,  s_n = tanh(T0 xi_n + t0b)   [L', 2]
// (trunk = DenseNet[2, th, L]: T0 [th, 2], T1 [L, th]).  Q and J depend only on the
// grid and the weights: mmpde_dmm_head_prepare computes them once into a caller-owned
// cache that later calls reuse; without a cache they are computed inside the call.
#include "common.hpp"
#include "gemm.hpp"

namespace {

// ---------------------------------------------------------------------------
// Graph-mode branch (cylinder): embedding, 3 tiny GNN layers (h = 4, tanh),
// decoding DenseNet[4,128,1].  One thread per node; the trajectory's nodes use
// the fixed grid's LOCAL neighbour table (same for every trajectory,
// dmm_model.py:222-234).
// ---------------------------------------------------------------------------
struct DmmEmbW {
    float w0[12], b0[4], bn1[16], w3[16], b3[4], bn4[16];  // bn: w, b, rm, rv
};

__global__ __launch_bounds__(256) void dmm_embed_kernel(const float *__restrict__ u,
                                                        const float2 *__restrict__ grid,
                                                        int64_t n_tot, int64_t n_per,
                                                        mmpde_dmm_graph_branch p,
                                                        float4 *__restrict__ h,
                                                        unsigned *__restrict__ zero, int n_zero) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i < n_zero) zero[i] = 0u;  // the skinny linears' split-K tickets
    if (i >= n_tot) return;
    const float2 g = grid[i % n_per];
    const float in[3] = {u[i], g.x, g.y};  // cat(x, pos_x, pos_y), dmm_model.py:205
    float z[4], o[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        float v = p.emb0_b[c];
#pragma unroll
        for (int j = 0; j < 3; ++j) v += p.emb0_w[c * 3 + j] * in[j];
        z[c] = tanhf(bn_eval(v, p.emb1_rm[c], p.emb1_rv[c], p.emb1_w[c], p.emb1_b[c], p.eps));
    }
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        float v = p.emb3_b[c];
#pragma unroll
        for (int j = 0; j < 4; ++j) v += p.emb3_w[c * 4 + j] * z[j];
        o[c] = bn_eval(v, p.emb4_rm[c], p.emb4_rv[c], p.emb4_w[c], p.emb4_b[c], p.eps);
    }
    h[i] = make_float4(o[0], o[1], o[2], o[3]);
}

// DMM GNN_Layer_FS_2D (dmm_model.py:94-142): message cat(x_i, x_j, u_i-u_j,
// px_i-px_j, py_i-py_j) (11) -> 4 tanh -> 4 tanh; mean; update cat(x, m) (8) ->
// 4 tanh -> 4 tanh; x + upd; BN.  Four lanes per node: lane `sub` of the quad
// takes edges sub, sub + 4, ..., the quad's sums meet by two xor shuffles.  The
// arithmetic lives in these helpers, shared by the two kernels below (identical
// results).
struct DmmGnnSmem {
    float W1[44], B1[4], W2[16], B2[4], V1[32], C1[4], V2[16], C2[4];
    float BW[4], BB[4], RM[4], RV[4];  // the layer's BatchNorm (eval), read at the end
    __device__ void load(const float *w1, const float *b1, const float *w2, const float *b2, const float *v1,
                         const float *c1, const float *v2, const float *c2, const float *bnw,
                         const float *bnb, const float *bnrm, const float *bnrv) {
        // every load unconditional (clamped index), the stores under the
        // conditions: a load inside an `if` is waited for where the `if` ends
        const int t = threadIdx.x;
        const int t44 = min(t, 43), t32 = min(t, 31), t16 = min(t, 15), t4 = min(t, 3);
        const float a0 = w1[t44], a1 = v1[t32], a2 = w2[t16], a3 = v2[t16];
        const float a4 = b1[t4], a5 = b2[t4], a6 = c1[t4], a7 = c2[t4];
        const float a8 = bnw[t4], a9 = bnb[t4], a10 = bnrm[t4], a11 = bnrv[t4];
        if (t < 44) W1[t] = a0;
        if (t < 32) V1[t] = a1;
        if (t < 16) {
            W2[t] = a2;
            V2[t] = a3;
        }
        if (t < 4) {
            B1[t] = a4;
            B2[t] = a5;
            C1[t] = a6;
            C2[t] = a7;
            BW[t] = a8;
            BB[t] = a9;
            RM[t] = a10;
            RV[t] = a11;
        }
    }
};

// sum[o] += message(i, j)[o]
__device__ __forceinline__ void dmm_edge_acc(const DmmGnnSmem &w, const float (&hi)[4], float ui, float2 gi,
                                             float4 hj4, float uj, float2 gj, float (&sum)[4]) {
    const float in[11] = {hi[0], hi[1], hi[2], hi[3], hj4.x, hj4.y, hj4.z, hj4.w,
                          ui - uj, gi.x - gj.x, gi.y - gj.y};
    float m1[4];
#pragma unroll
    for (int o = 0; o < 4; ++o) {
        float v = w.B1[o];
#pragma unroll
        for (int t = 0; t < 11; ++t) v += w.W1[o * 11 + t] * in[t];
        m1[o] = tanhf(v);
    }
#pragma unroll
    for (int o = 0; o < 4; ++o) {
        float v = w.B2[o];
#pragma unroll
        for (int t = 0; t < 4; ++t) v += w.W2[o * 4 + t] * m1[t];
        sum[o] += tanhf(v);
    }
}

// the quad's sums -> mean -> update -> BN (every lane of the quad returns it)
__device__ __forceinline__ float4 dmm_node_update(const DmmGnnSmem &w, const float (&hi)[4], float (&sum)[4],
                                                  int k, float eps) {
#pragma unroll
    for (int o = 0; o < 4; ++o) {
        sum[o] += xor_lane_f<1>(sum[o]);
        sum[o] += xor_lane_f<2>(sum[o]);
    }
    float cat[8];
#pragma unroll
    for (int o = 0; o < 4; ++o) {
        cat[o] = hi[o];
        cat[4 + o] = sum[o] / (float)k;
    }
    float up1[4], res[4];
#pragma unroll
    for (int o = 0; o < 4; ++o) {
        float v = w.C1[o];
#pragma unroll
        for (int t = 0; t < 8; ++t) v += w.V1[o * 8 + t] * cat[t];
        up1[o] = tanhf(v);
    }
#pragma unroll
    for (int o = 0; o < 4; ++o) {
        float v = w.C2[o];
#pragma unroll
        for (int t = 0; t < 4; ++t) v += w.V2[o * 4 + t] * up1[t];
        res[o] = bn_eval(hi[o] + tanhf(v), w.RM[o], w.RV[o], w.BW[o], w.BB[o], eps);
    }
    return make_float4(res[0], res[1], res[2], res[3]);
}

// Every source read from global memory (L2): any trajectory size.
__global__ __launch_bounds__(256) void dmm_gnn_kernel(const float4 *__restrict__ h,
                                                      const float *__restrict__ u,
                                                      const float2 *__restrict__ grid,
                                                      const int32_t *__restrict__ nbr, int k,
                                                      int64_t n_tot, int64_t n_per,
                                                      const float *__restrict__ w1,
                                                      const float *__restrict__ b1,
                                                      const float *__restrict__ w2,
                                                      const float *__restrict__ b2,
                                                      const float *__restrict__ v1,
                                                      const float *__restrict__ c1,
                                                      const float *__restrict__ v2,
                                                      const float *__restrict__ c2,
                                                      const float *__restrict__ bnw,
                                                      const float *__restrict__ bnb,
                                                      const float *__restrict__ bnrm,
                                                      const float *__restrict__ bnrv, float eps,
                                                      float4 *__restrict__ h_out) {
    __shared__ DmmGnnSmem w;
    w.load(w1, b1, w2, b2, v1, c1, v2, c2, bnw, bnb, bnrm, bnrv);
    __syncthreads();
    const int64_t i = ((int64_t)blockIdx.x * 256 + threadIdx.x) >> 2;
    const int sub = threadIdx.x & 3;
    if (i >= n_tot) return;  // whole quads leave together
    const int64_t b = i / n_per;
    const int64_t p = i - b * n_per;
    const float4 hi4 = h[i];
    const float hi[4] = {hi4.x, hi4.y, hi4.z, hi4.w};
    const float ui = u[i];
    const float2 gi = grid[p];
    float sum[4] = {0.f, 0.f, 0.f, 0.f};
    const int32_t *nr = nbr + p * k;
    // neighbour indices eight edges at a time, loaded unconditionally (clamped):
    // an index load inside the edge loop is one round trip per edge
    for (int e0 = sub; e0 < k; e0 += 32) {
        int64_t jl[8];
#pragma unroll
        for (int t = 0; t < 8; ++t) jl[t] = min((uint32_t)nr[min(e0 + 4 * t, k - 1)], (uint32_t)(n_per - 1));
#pragma unroll
        for (int t = 0; t < 8; ++t) {
            if (e0 + 4 * t >= k) break;
            const int64_t j = b * n_per + jl[t];
            dmm_edge_acc(w, hi, ui, gi, h[j], u[j], grid[jl[t]], sum);
        }
    }
    const float4 r = dmm_node_update(w, hi, sum, k, eps);
    if (sub == 0) h_out[i] = r;
}

// The same layer with the trajectory's h, u and the grid staged in LDS
// (28 B per point, dynamic): workgroup (x, b) takes kDmmLdsTargets targets of
// trajectory b, so every neighbour read is an LDS read instead of an L2
// round trip (the global kernel waits on its gathers, not on its tanh).
constexpr int kDmmLdsTargets = 128;   // 512 threads: four lanes per target
__global__ __launch_bounds__(512) void dmm_gnn_lds_kernel(const float4 *__restrict__ h,
                                                          const float *__restrict__ u,
                                                          const float2 *__restrict__ grid,
                                                          const int32_t *__restrict__ nbr, int k,
                                                          int n_per,
                                                          const float *__restrict__ w1,
                                                          const float *__restrict__ b1,
                                                          const float *__restrict__ w2,
                                                          const float *__restrict__ b2,
                                                          const float *__restrict__ v1,
                                                          const float *__restrict__ c1,
                                                          const float *__restrict__ v2,
                                                          const float *__restrict__ c2,
                                                          const float *__restrict__ bnw,
                                                          const float *__restrict__ bnb,
                                                          const float *__restrict__ bnrm,
                                                          const float *__restrict__ bnrv, float eps,
                                                          float4 *__restrict__ h_out) {
    extern __shared__ float4 dyn[];
    float4 *sh = dyn;
    float2 *sg = (float2 *)(sh + n_per);
    float *su = (float *)(sg + n_per);
    __shared__ DmmGnnSmem w;
    w.load(w1, b1, w2, b2, v1, c1, v2, c2, bnw, bnb, bnrm, bnrv);
    const int64_t base = (int64_t)blockIdx.y * n_per;
    for (int t = threadIdx.x; t < n_per; t += 512) {
        sh[t] = h[base + t];
        sg[t] = grid[t];
        su[t] = u[base + t];
    }
    __syncthreads();
    const int p = blockIdx.x * kDmmLdsTargets + (threadIdx.x >> 2);
    const int sub = threadIdx.x & 3;
    if (p >= n_per) return;  // whole quads leave together
    const float4 hi4 = sh[p];
    const float hi[4] = {hi4.x, hi4.y, hi4.z, hi4.w};
    const float ui = su[p];
    const float2 gi = sg[p];
    float sum[4] = {0.f, 0.f, 0.f, 0.f};
    const int32_t *nr = nbr + (int64_t)p * k;
    // neighbour indices eight edges at a time, loaded unconditionally (clamped):
    // an index load inside the edge loop is one round trip per edge
    for (int e0 = sub; e0 < k; e0 += 32) {
        int jl[8];
#pragma unroll
        for (int t = 0; t < 8; ++t) jl[t] = (int)min((uint32_t)nr[min(e0 + 4 * t, k - 1)], (uint32_t)(n_per - 1));
#pragma unroll
        for (int t = 0; t < 8; ++t) {
            if (e0 + 4 * t >= k) break;
            dmm_edge_acc(w, hi, ui, gi, sh[jl[t]], su[jl[t]], sg[jl[t]], sum);
        }
    }
    const float4 r = dmm_node_update(w, hi, sum, k, eps);
    if (sub == 0) h_out[base + p] = r;
}

// LDS bytes of dmm_gnn_lds_kernel's staging (0: too large, use dmm_gnn_kernel)
static size_t dmm_gnn_lds_bytes(int64_t n_per) {
    const int64_t b = n_per * (16 + 8 + 4);
    return b <= 120 * 1024 ? (size_t)b : 0;
}

// decoding_mlp DenseNet([4, 128, 1]) (dmm_model.py:173,209): d = W1 tanh(W0 h + b0) + b1
__global__ __launch_bounds__(256) void dmm_decode_kernel(const float4 *__restrict__ h,
                                                         int64_t n_tot,
                                                         const float *__restrict__ w0,
                                                         const float *__restrict__ b0,
                                                         const float *__restrict__ w1,
                                                         const float *__restrict__ b1,
                                                         float *__restrict__ out) {
    __shared__ float sW0[512], sB0[128], sW1[128];
    for (int t = threadIdx.x; t < 512; t += 256) sW0[t] = w0[t];
    if (threadIdx.x < 128) {
        sB0[threadIdx.x] = b0[threadIdx.x];
        sW1[threadIdx.x] = w1[threadIdx.x];
    }
    __syncthreads();
    // four lanes per node, lane `sub` of the quad takes hidden units sub, sub + 4, ...
    const int64_t i = ((int64_t)blockIdx.x * 256 + threadIdx.x) >> 2;
    const int sub = threadIdx.x & 3;
    if (i >= n_tot) return;  // whole quads leave together
    const float4 hv = h[i];
    float acc = 0.0f;
    for (int j = sub; j < 128; j += 4) {
        const float z = tanhf(sB0[j] + sW0[4 * j] * hv.x + sW0[4 * j + 1] * hv.y +
                              sW0[4 * j + 2] * hv.z + sW0[4 * j + 3] * hv.w);
        acc += sW1[j] * z;
    }
    acc += __shfl_xor(acc, 1, 64);
    acc += __shfl_xor(acc, 2, 64);
    if (sub == 0) out[i] = acc + b1[0];
}

// ---------------------------------------------------------------------------
// Shared head: trunk, Q, J and the mesh VJP.
// ---------------------------------------------------------------------------
// trunk hidden s = tanh(T0 xi + t0b) ([N, th]) and trunk = T1 s + t1b ([N, L]); one
// block per grid point.
__global__ __launch_bounds__(256) void trunk_kernel(const float2 *__restrict__ xi, int th,
                                                    int latent, const float *__restrict__ t0w,
                                                    const float *__restrict__ t0b,
                                                    const float *__restrict__ t1w,
                                                    const float *__restrict__ t1b,
                                                    float *__restrict__ s_out,
                                                    float *__restrict__ trunk) {
    __shared__ float s[64];
    const int64_t nidx = blockIdx.x;
    const float2 x = xi[nidx];
    if (threadIdx.x < th) {
        const float v = tanhf(t0w[threadIdx.x * 2] * x.x + t0w[threadIdx.x * 2 + 1] * x.y +
                              t0b[threadIdx.x]);
        s[threadIdx.x] = v;
        s_out[nidx * th + threadIdx.x] = v;
    }
    __syncthreads();
    for (int j = threadIdx.x; j < latent; j += 256) {
        float v = t1b[j];
        for (int m = 0; m < th; ++m) v += t1w[(int64_t)j * th + m] * s[m];
        trunk[nidx * latent + j] = v;
    }
}

// out[c][r] = in[r][c] (rows x cols -> cols x rows)
__global__ void transpose_kernel(const float *__restrict__ in, int rows, int cols,
                                 float *__restrict__ out) {
    const int e = blockIdx.x * 256 + threadIdx.x;
    if (e >= rows * cols) return;
    const int r = e / cols, c = e - r * cols;
    out[(int64_t)c * rows + r] = in[e];
}

// J[n][k][d] = sum_m Gt[m][k] (1 - s[n][m]^2) T0[m][d]; one block per grid point.
__global__ __launch_bounds__(256) void jac_kernel(const float *__restrict__ s, int th,
                                                  const float *__restrict__ gt, int hidden,
                                                  const float *__restrict__ t0w,
                                                  float2 *__restrict__ jac) {
    __shared__ float a0[64], a1[64];
    const int64_t nidx = blockIdx.x;
    if (threadIdx.x < th) {
        const float sv = s[nidx * th + threadIdx.x];
        const float ds = 1.0f - sv * sv;
        a0[threadIdx.x] = ds * t0w[threadIdx.x * 2];
        a1[threadIdx.x] = ds * t0w[threadIdx.x * 2 + 1];
    }
    __syncthreads();
    for (int kk = threadIdx.x; kk < hidden; kk += 256) {
        float j0 = 0.0f, j1 = 0.0f;
        for (int m = 0; m < th; ++m) {
            const float g = gt[(int64_t)m * hidden + kk];
            j0 += g * a0[m];
            j1 += g * a1[m];
        }
        jac[nidx * hidden + kk] = make_float2(j0, j1);
    }
}

// mesh[b*N + n] = xi[n] + sum_k w_o[k] (1 - tanh^2(P[b,k] + Q[n,k])) J[n,k]; one
// workgroup per grid point, wave w taking trajectories w, w + 4, ...
__global__ __launch_bounds__(256) void mesh_vjp_kernel(const float *__restrict__ P,
                                                       const float *__restrict__ Q,
                                                       const float2 *__restrict__ jac,
                                                       const float *__restrict__ wo,
                                                       const float2 *__restrict__ xi,
                                                       int64_t batches, int64_t n_per,
                                                       int hidden, float2 *__restrict__ mesh) {
    const int wave = threadIdx.x >> 6;
    const int lane = threadIdx.x & 63;
    const int64_t nidx = blockIdx.x;
    const float *q = Q + nidx * hidden;
    const float2 *jr = jac + nidx * hidden;
    const float2 x = xi[nidx];
    for (int64_t b = wave; b < batches; b += 4) {
        const float *pb = P + b * hidden;
        float gx = 0.0f, gy = 0.0f;
        for (int kk = lane; kk < hidden; kk += 64) {
            const float t = tanhf(pb[kk] + q[kk]);
            const float g = wo[kk] * (1.0f - t * t);
            const float2 jj = jr[kk];
            gx += g * jj.x;
            gy += g * jj.y;
        }
        gx = wave_sum_full(gx);
        gy = wave_sum_full(gy);
        if (lane == 0) mesh[b * n_per + nidx] = make_float2(gx + x.x, gy + x.y);
    }
}

// The same VJP with one wave per grid point and every trajectory: Q[n], J[n]
// and w_o are read once per grid point into registers (KPL = hidden / 64 per
// lane), P (all trajectories) once per workgroup into LDS; per-lane partial
// sums and the wave reduction are those of mesh_vjp_kernel (identical results).
template <int KPL>
__global__ __launch_bounds__(256) void mesh_vjp_wave_kernel(const float *__restrict__ P,
                                                            const float *__restrict__ Q,
                                                            const float2 *__restrict__ jac,
                                                            const float *__restrict__ wo,
                                                            const float2 *__restrict__ xi,
                                                            int batches, int n_per,
                                                            float2 *__restrict__ mesh) {
    extern __shared__ float sP[];  // [batches][64 KPL]
    constexpr int HID = 64 * KPL;
    for (int i = threadIdx.x; i < batches * HID; i += 256) sP[i] = P[i];
    __syncthreads();
    const int lane = threadIdx.x & 63;
    const int nidx = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (nidx >= n_per) return;  // wave-uniform, after the only barrier
    float q[KPL], w[KPL];
    float2 jj[KPL];
#pragma unroll
    for (int i = 0; i < KPL; ++i) {
        const int kk = lane + 64 * i;
        q[i] = Q[(int64_t)nidx * HID + kk];
        jj[i] = jac[(int64_t)nidx * HID + kk];
        w[i] = wo[kk];
    }
    const float2 x = xi[nidx];
    for (int b = 0; b < batches; ++b) {
        const float *pb = sP + b * HID;
        float gx = 0.0f, gy = 0.0f;
#pragma unroll
        for (int i = 0; i < KPL; ++i) {
            const float t = tanhf(pb[lane + 64 * i] + q[i]);
            const float g = w[i] * (1.0f - t * t);
            gx += g * jj[i].x;
            gy += g * jj[i].y;
        }
        gx = wave_sum_full(gx);
        gy = wave_sum_full(gy);
        if (lane == 0) mesh[(int64_t)b * n_per + nidx] = make_float2(gx + x.x, gy + x.y);
    }
}

// phi[i] = w_o . tanh(P[b] + Q[i]) + b_o2, b = i / per (out_nn = DenseNet[2L, L', 1]
// on cat(branch_b, trunk(grid_i)), dmm_model.py:190,213); second[i] = the tanh
// row (rf=True's second_out).  One wave per grid row.
__global__ __launch_bounds__(256) void phi_kernel(const float *__restrict__ P, const float *__restrict__ Q,
                                                  const float *__restrict__ wo, const float *__restrict__ bo,
                                                  int64_t n_grid, int64_t per, int hidden,
                                                  float *__restrict__ phi, float *__restrict__ second) {
    const int lane = threadIdx.x & 63;
    const int64_t i = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (i >= n_grid) return;
    const float *pb = P + (i / per) * hidden;
    const float *q = Q + i * hidden;
    float acc = 0.0f;
    for (int kk = lane; kk < hidden; kk += 64) {
        const float t = tanhf(pb[kk] + q[kk]);
        if (second) second[i * hidden + kk] = t;
        acc += wo[kk] * t;
    }
    acc = wave_sum_full(acc);
    if (lane == 0) phi[i] = acc + (bo ? bo[0] : 0.0f);
}

struct HeadWs {
    float *trunk, *s, *q, *t1t, *gt, *p;
    float2 *jac;
};

int64_t head_floats(int64_t batches, int64_t n_per, int latent, int hidden, int th) {
    return n_per * latent + n_per * th + n_per * hidden + (int64_t)th * latent +
           (int64_t)th * hidden + batches * hidden + 2 * n_per * hidden + 64;
}

HeadWs carve_head(float *ws, int64_t batches, int64_t n_per, int latent, int hidden, int th) {
    HeadWs h;
    auto take = [&](int64_t nf) {
        float *p = ws;
        ws += (nf + 3) & ~int64_t(3);  // keep 16-B alignment
        return p;
    };
    h.trunk = take(n_per * latent);
    h.s = take(n_per * th);
    h.q = take(n_per * hidden);
    h.t1t = take((int64_t)th * latent);
    h.gt = take((int64_t)th * hidden);
    h.p = take(batches * hidden);
    h.jac = (float2 *)take(2 * n_per * hidden);
    return h;
}

// Grid side of the head (a function of xi and the weights only): trunk, Q =
// Wt . trunk [N, L'] and J = dQ/dxi [N, L'] (float2).
int dmm_head_grid(const float *xi, int64_t n_per, const mmpde_dmm_head *hd, const HeadWs &w,
                  float *q, float2 *jac, hipStream_t st) {
    const int L = hd->latent, Lp = hd->hidden, th = hd->th;
    hipLaunchKernelGGL(trunk_kernel, dim3((unsigned)n_per), dim3(256), 0, st,
                       (const float2 *)xi, th, L, hd->t0_w, hd->t0_b, hd->t1_w, hd->t1_b, w.s,
                       w.trunk);
    MMPDE_RET_LAUNCH();
    // Q = Wt . trunk (Wt = out_nn.layers.0.weight[:, L:2L]) on MFMA
    {
        const int kh = L / 2;
        GemmArgs g{n_per, w.trunk, w.trunk + kh, L, hd->o0_w + L, hd->o0_w + L + kh, 2 * L, kh};
        EpiStore epi{q, Lp};
        const int rc = launch_gemm(g, Lp / 128, epi, st);
        if (rc) return rc;
    }
    // Gt = (Wt . T1)^T = T1^T . Wt^T  ([th, L'])
    hipLaunchKernelGGL(transpose_kernel, dim3(ceil_div((int64_t)L * th, 256)), dim3(256), 0, st,
                       hd->t1_w, L, th, w.t1t);
    MMPDE_RET_LAUNCH();
    const int rc = mmpde_linear_skinny(w.t1t, L, th, L, hd->o0_w + L, 2 * L, nullptr, Lp,
                                       MMPDE_ACT_NONE, w.gt, Lp, st);
    if (rc) return rc;
    hipLaunchKernelGGL(jac_kernel, dim3((unsigned)n_per), dim3(256), 0, st, w.s, th, w.gt, Lp,
                       hd->t0_w, jac);
    MMPDE_RET_LAUNCH();
    return MMPDE_OK;
}

bool head_ok(const mmpde_dmm_head *hd) {
    return hd->th >= 1 && hd->th <= 64 && hd->latent % 8 == 0 && hd->hidden % 128 == 0;
}

// Head cache layout: Q [N, L'] then J [N, L'] float2.
int64_t cache_floats(int64_t n_per, int hidden) { return 3 * n_per * hidden; }

// branch [B, L] -> mesh [B*N, 2]; cache: a prepared grid side (or null: computed here)
int dmm_head(const float *branch, const float *xi, int64_t batches, int64_t n_per,
             const mmpde_dmm_head *hd, float *ws, const float *cache, float *mesh_out,
             hipStream_t st, float *sk, int64_t skf) {
    const int L = hd->latent, Lp = hd->hidden, th = hd->th;
    if (!head_ok(hd)) return MMPDE_ERR_UNSUPPORTED;
    HeadWs w = carve_head(ws, batches, n_per, L, Lp, th);
    const float *q = cache ? cache : w.q;
    const float2 *jac = cache ? (const float2 *)(cache + n_per * Lp) : w.jac;
    int rc;
    if (!cache) {
        rc = dmm_head_grid(xi, n_per, hd, w, w.q, w.jac, st);
        if (rc) return rc;
    }
    // P = Wb . branch + b_o1 (Wb = out_nn.layers.0.weight[:, :L], row stride 2L)
    rc = mmpde_linear_skinny_ws(branch, L, batches, L, hd->o0_w, 2 * L, hd->o0_b, Lp, MMPDE_ACT_NONE, w.p,
                                Lp, sk, skf * (int64_t)sizeof(float), st);
    if (rc) return rc;
    const size_t lds = (size_t)batches * Lp * sizeof(float);
    if (Lp == 512 && lds <= 65536) {
        hipLaunchKernelGGL(mesh_vjp_wave_kernel<8>, dim3((unsigned)ceil_div(n_per, 4)), dim3(256),
                           lds, st, w.p, q, jac, hd->o1_w, (const float2 *)xi, (int)batches,
                           (int)n_per, (float2 *)mesh_out);
    } else {
        hipLaunchKernelGGL(mesh_vjp_kernel, dim3((unsigned)n_per), dim3(256), 0, st, w.p, q, jac,
                           hd->o1_w, (const float2 *)xi, batches, n_per, Lp, (float2 *)mesh_out);
    }
    MMPDE_RET_LAUNCH();
    return MMPDE_OK;
}

inline bool al16(const void *p) { return ((uintptr_t)p & 15u) == 0; }

}  // namespace

namespace {
// branch-side scratch (graph: 2 h buffers + decode + MLP activations; array:
// conv activations), then the shared head region, then the split-K scratch of
// the skinny linears (mmpde_linear_skinny_ws: its ticket counters first, then
// at most 16 splits of an output of at most max(batches, 64) x 2048).  The
// counters are zeroed by the branch's first kernel (dmm_embed_kernel /
// conv0) on every mesh call; every skinny call leaves them zero.
int64_t dmm_base_floats(int64_t batches, int64_t n_per, int latent, int hidden) {
    const int64_t branch_side = 2 * 4 * batches * n_per + batches * n_per + batches * 2048 +
                                8 * batches * n_per + 256;
    return branch_side + head_floats(batches, n_per, latent, hidden, 64) + 256;
}
// dense.hip kSkTickets (+ 32 floats of slack); zeroed by the branch's first
// kernel on every call
int64_t dmm_skinny_ticket_floats(int64_t) { return 4096 + 32; }
int64_t dmm_skinny_floats(int64_t batches) {
    return dmm_skinny_ticket_floats(batches) + 16 * (batches > 64 ? batches : 64) * 2048;
}

// skinny linear with the workspace's split-K scratch
int skinny(const float *x, int64_t ldx, int64_t m, int64_t k, const float *w, int64_t ldw, const float *b,
           int64_t n, int act, float *y, int64_t ldy, float *scratch, int64_t scratch_floats,
           mmpde_stream_t st) {
    return mmpde_linear_skinny_ws(x, ldx, m, k, w, ldw, b, n, act, y, ldy, scratch,
                                  scratch_floats * (int64_t)sizeof(float), st);
}

}  // namespace

extern "C" int64_t mmpde_dmm_workspace_bytes(int64_t batches, int64_t n_per, int latent,
                                             int hidden) {
    return (dmm_base_floats(batches, n_per, latent, hidden) + dmm_skinny_floats(batches)) *
           (int64_t)sizeof(float);
}

extern "C" int64_t mmpde_dmm_head_cache_bytes(int64_t n_per, int hidden) {
    return n_per > 0 && hidden > 0 ? cache_floats(n_per, hidden) * (int64_t)sizeof(float) : 0;
}

extern "C" int mmpde_dmm_head_prepare(const float *xi, int64_t n_per, const mmpde_dmm_head *hd,
                                      void *workspace, void *cache, mmpde_stream_t stream) {
    MMPDE_REQUIRE(xi && hd && workspace && cache && n_per > 0 && al16(workspace) && al16(cache));
    if (!head_ok(hd)) return MMPDE_ERR_UNSUPPORTED;
    HeadWs w = carve_head((float *)workspace, 1, n_per, hd->latent, hd->hidden, hd->th);
    float *q = (float *)cache;
    return dmm_head_grid(xi, n_per, hd, w, q, (float2 *)(q + n_per * hd->hidden),
                         as_stream(stream));
}

extern "C" int mmpde_dmm_mesh_graph(const float *u, const float *grid, int64_t batches,
                                    int64_t n_per, const int32_t *grid_nbr, int k,
                                    const mmpde_dmm_graph_branch *br, const mmpde_dmm_head *hd,
                                    void *workspace, float *mesh_out, mmpde_stream_t stream) {
    return mmpde_dmm_mesh_graph_cached(u, grid, batches, n_per, grid_nbr, k, br, hd, nullptr,
                                       workspace, mesh_out, stream);
}

namespace {
// Graph-mode branch: u [B, N] on the fixed grid -> branch [B, L]
// (dmm_model.py:197-210).  Scratch from ws (h ping-pong, decode, output_mlp
// activations); *ws_end = the first float after it.
int graph_branch(const float *u, const float *grid, int64_t batches, int64_t n_per,
                 const int32_t *grid_nbr, int k, const mmpde_dmm_graph_branch *br, int latent, float *ws,
                 float *sk, int64_t skf, float *branch, float **ws_end, hipStream_t st) {
    const int64_t nt = batches * n_per;
    float4 *h0 = (float4 *)ws;
    float4 *h1 = h0 + nt;
    float *dec = (float *)(h1 + nt);
    float *om1 = dec + ((nt + 3) & ~int64_t(3));
    float *om2 = om1 + batches * 512;
    if (ws_end) *ws_end = om2 + batches * 256;
    const int nz = (int)dmm_skinny_ticket_floats(batches);
    const dim3 g1(ceil_div(nt > nz ? nt : nz, 256)), g4(ceil_div(4 * nt, 256));  // g4: four lanes per node
    hipLaunchKernelGGL(dmm_embed_kernel, g1, dim3(256), 0, st, u, (const float2 *)grid, nt, n_per,
                       *br, h0, (unsigned *)sk, nz);
    MMPDE_RET_LAUNCH();
    size_t lds = batches <= 65535 ? dmm_gnn_lds_bytes(n_per) : 0;
    if (lds > 64 * 1024 &&
        hipFuncSetAttribute((const void *)dmm_gnn_lds_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)lds) != hipSuccess)
        lds = 0;  // the global-memory kernel
    for (int l = 0; l < br->n_gnn_layers; ++l) {
        if (lds) {
            const dim3 gl((unsigned)ceil_div(n_per, kDmmLdsTargets), (unsigned)batches);
            hipLaunchKernelGGL(dmm_gnn_lds_kernel, gl, dim3(512), lds, st, h0, u, (const float2 *)grid,
                               grid_nbr, k, (int)n_per, br->g_msg1_w[l], br->g_msg1_b[l],
                               br->g_msg2_w[l], br->g_msg2_b[l], br->g_upd1_w[l], br->g_upd1_b[l],
                               br->g_upd2_w[l], br->g_upd2_b[l], br->g_bn_w[l], br->g_bn_b[l],
                               br->g_bn_rm[l], br->g_bn_rv[l], br->eps, h1);
        } else {
            hipLaunchKernelGGL(dmm_gnn_kernel, g4, dim3(256), 0, st, h0, u, (const float2 *)grid,
                               grid_nbr, k, nt, n_per, br->g_msg1_w[l], br->g_msg1_b[l],
                               br->g_msg2_w[l], br->g_msg2_b[l], br->g_upd1_w[l], br->g_upd1_b[l],
                               br->g_upd2_w[l], br->g_upd2_b[l], br->g_bn_w[l], br->g_bn_b[l],
                               br->g_bn_rm[l], br->g_bn_rv[l], br->eps, h1);
        }
        MMPDE_RET_LAUNCH();
        float4 *t = h0;
        h0 = h1;
        h1 = t;
    }
    hipLaunchKernelGGL(dmm_decode_kernel, g4, dim3(256), 0, st, h0, nt, br->dec0_w, br->dec0_b,
                       br->dec1_w, br->dec1_b, dec);
    MMPDE_RET_LAUNCH();
    // output_mlp: Linear(N,512) tanh Linear(512,256) tanh Linear(256,L) on [B, N]
    int rc = skinny(dec, n_per, batches, n_per, br->om0_w, n_per, br->om0_b, 512, MMPDE_ACT_TANH, om1, 512,
                    sk, skf, st);
    if (rc) return rc;
    rc = skinny(om1, 512, batches, 512, br->om2_w, 512, br->om2_b, 256, MMPDE_ACT_TANH, om2, 256, sk, skf,
                st);
    if (rc) return rc;
    return skinny(om2, 256, batches, 256, br->om4_w, 256, br->om4_b, latent, MMPDE_ACT_NONE, branch, latent,
                  sk, skf, st);
}

// Array-mode branch: ConvNet.forward (dmm_model.py:65-81), u [B, s, s] ->
// branch [B, L].  conv0 also zeroes the skinny linears' tickets.
int array_branch(const float *u, int64_t batches, const mmpde_dmm_array_branch *br, int latent, float *ws,
                 float *sk, int64_t skf, float *branch, float **ws_end, hipStream_t st) {
    const int s = br->s;
    const int s1 = (s + 4 - 5) / 2 + 1;   // conv0, stride 2, pad 2
    const int s3 = (s1 + 4 - 5) / 2 + 1;  // conv3, stride 2, pad 2
    auto take = [&](int64_t nf) {
        float *p = ws;
        ws += (nf + 3) & ~int64_t(3);
        return p;
    };
    float *x1 = take(batches * 8 * s1 * s1);
    float *x2 = take(batches * 16 * s1 * s1);
    float *x3 = take(batches * 8 * s1 * s1);
    float *x4 = take(batches * s3 * s3);
    float *f2 = take(batches * 1024);
    if (ws_end) *ws_end = ws;
    int rc = mmpde_detail::conv2d(u, batches, 1, s, s, br->c0_w, br->c0_b, 8, 5, 2, 2, nullptr, MMPDE_ACT_TANH,
                                  x1, st, (unsigned *)sk, (int)dmm_skinny_ticket_floats(batches));
    if (rc) return rc;
    rc = mmpde_conv2d(x1, batches, 8, s1, s1, br->c1_w, br->c1_b, 16, 5, 1, 2, nullptr, MMPDE_ACT_TANH, x2,
                      st);
    if (rc) return rc;
    rc = mmpde_conv2d(x2, batches, 16, s1, s1, br->c2_w, br->c2_b, 8, 5, 1, 2, x1, MMPDE_ACT_TANH, x3, st);
    if (rc) return rc;
    rc = mmpde_conv2d(x3, batches, 8, s1, s1, br->c3_w, br->c3_b, 1, 5, 2, 2, nullptr, MMPDE_ACT_TANH, x4,
                      st);
    if (rc) return rc;
    rc = skinny(x4, s3 * s3, batches, s3 * s3, br->fc2_w, s3 * s3, br->fc2_b, 1024, MMPDE_ACT_TANH, f2, 1024,
                sk, skf, st);
    if (rc) return rc;
    return skinny(f2, 1024, batches, 1024, br->fc3_w, 1024, br->fc3_b, latent, MMPDE_ACT_NONE, branch, latent,
                  sk, skf, st);
}

// array scratch is sized by max(N, s*s): xi may be coarser than u's grid
// (moving_mesh's bilinear pre-resampling, data_creator_2d.py:102-103)
int64_t array_n_eff(int64_t n_per, int s) { return n_per > (int64_t)s * s ? n_per : (int64_t)s * s; }
}  // namespace

extern "C" int mmpde_dmm_mesh_graph_cached(const float *u, const float *grid, int64_t batches,
                                           int64_t n_per, const int32_t *grid_nbr, int k,
                                           const mmpde_dmm_graph_branch *br,
                                           const mmpde_dmm_head *hd, const void *head_cache,
                                           void *workspace, float *mesh_out,
                                           mmpde_stream_t stream) {
    MMPDE_REQUIRE(u && grid && grid_nbr && br && hd && workspace && mesh_out);
    MMPDE_REQUIRE(batches > 0 && n_per > k && k > 0 && br->n_gnn_layers >= 0 &&
                  br->n_gnn_layers <= 3 && al16(workspace));
    hipStream_t st = as_stream(stream);
    float *ws = (float *)workspace;
    float *sk = ws + dmm_base_floats(batches, n_per, hd->latent, hd->hidden);
    const int64_t skf = dmm_skinny_floats(batches);
    float *end = nullptr;
    // branch [B, L] right after the branch scratch, then the head region
    const int64_t nt = batches * n_per;
    float *branch = ws + 8 * nt + ((nt + 3) & ~int64_t(3)) + batches * 768;
    float *head_ws = branch + ((batches * hd->latent + 3) & ~int64_t(3));
    int rc = graph_branch(u, grid, batches, n_per, grid_nbr, k, br, hd->latent, ws, sk, skf, branch, &end, st);
    if (rc) return rc;
    return dmm_head(branch, grid, batches, n_per, hd, head_ws, (const float *)head_cache, mesh_out,
                    st, sk, skf);
}

extern "C" int mmpde_dmm_mesh_array(const float *u, const float *xi, int64_t batches,
                                    int64_t n_per, const mmpde_dmm_array_branch *br,
                                    const mmpde_dmm_head *hd, void *workspace, float *mesh_out,
                                    mmpde_stream_t stream) {
    return mmpde_dmm_mesh_array_cached(u, xi, batches, n_per, br, hd, nullptr, workspace, mesh_out,
                                       stream);
}

extern "C" int mmpde_dmm_mesh_array_cached(const float *u, const float *xi, int64_t batches,
                                           int64_t n_per, const mmpde_dmm_array_branch *br,
                                           const mmpde_dmm_head *hd, const void *head_cache,
                                           void *workspace, float *mesh_out,
                                           mmpde_stream_t stream) {
    MMPDE_REQUIRE(u && xi && br && hd && workspace && mesh_out && batches > 0 && n_per > 0);
    MMPDE_REQUIRE(br->s >= 5 && al16(workspace));
    hipStream_t st = as_stream(stream);
    float *ws = (float *)workspace;
    float *sk = ws + dmm_base_floats(batches, array_n_eff(n_per, br->s), hd->latent, hd->hidden);
    const int64_t skf = dmm_skinny_floats(batches);
    float *end = nullptr;
    // branch scratch, then branch [B, L], then the head region
    const int s1 = (br->s + 4 - 5) / 2 + 1, s3 = (s1 + 4 - 5) / 2 + 1;
    auto up4 = [](int64_t v) { return (v + 3) & ~int64_t(3); };
    float *branch = ws + 2 * up4(batches * 8 * s1 * s1) + up4(batches * 16 * s1 * s1) + up4(batches * s3 * s3) +
                    up4(batches * 1024);
    float *head_ws = branch + up4(batches * hd->latent);
    int rc = array_branch(u, batches, br, hd->latent, ws, sk, skf, branch, &end, st);
    if (rc) return rc;
    return dmm_head(branch, xi, batches, n_per, hd, head_ws, (const float *)head_cache, mesh_out, st, sk, skf);
}

// ---------------------------------------------------------------------------
// DMM.forward pieces: the branch alone and phi itself (dmm_model.py:185-219)
// ---------------------------------------------------------------------------
extern "C" int mmpde_dmm_branch_graph(const float *u, const float *grid, int64_t batches, int64_t n_per,
                                      const int32_t *grid_nbr, int k, const mmpde_dmm_graph_branch *br,
                                      const mmpde_dmm_head *hd, void *workspace, float *branch_out,
                                      mmpde_stream_t stream) {
    MMPDE_REQUIRE(u && grid && grid_nbr && br && hd && workspace && branch_out && hd->latent > 0);
    MMPDE_REQUIRE(batches > 0 && n_per > k && k > 0 && br->n_gnn_layers >= 0 &&
                  br->n_gnn_layers <= 3 && al16(workspace));
    float *ws = (float *)workspace;
    float *sk = ws + dmm_base_floats(batches, n_per, hd->latent, hd->hidden);
    return graph_branch(u, grid, batches, n_per, grid_nbr, k, br, hd->latent, ws, sk, dmm_skinny_floats(batches),
                        branch_out, nullptr, as_stream(stream));
}

extern "C" int mmpde_dmm_branch_array(const float *u, int64_t batches, const mmpde_dmm_array_branch *br,
                                      const mmpde_dmm_head *hd, void *workspace, float *branch_out,
                                      mmpde_stream_t stream) {
    MMPDE_REQUIRE(u && br && hd && workspace && branch_out && batches > 0 && hd->latent > 0 && br->s >= 5 &&
                  al16(workspace));
    float *ws = (float *)workspace;
    float *sk = ws + dmm_base_floats(batches, (int64_t)br->s * br->s, hd->latent, hd->hidden);
    return array_branch(u, batches, br, hd->latent, ws, sk, dmm_skinny_floats(batches), branch_out, nullptr,
                        as_stream(stream));
}

extern "C" int64_t mmpde_dmm_phi_workspace_bytes(int64_t batches, int64_t n_grid, int latent, int hidden,
                                                 int th) {
    if (batches <= 0 || n_grid <= 0 || latent <= 0 || hidden <= 0 || th <= 0) return 0;
    return (head_floats(batches, n_grid, latent, hidden, th) + 64) * (int64_t)sizeof(float);
}

extern "C" int mmpde_dmm_phi(const float *branch, int64_t batches, const float *grid, int64_t n_grid,
                             const mmpde_dmm_head *hd, const float *o1_b, void *workspace, float *phi_out,
                             float *second_out, mmpde_stream_t stream) {
    MMPDE_REQUIRE(branch && grid && hd && workspace && phi_out && batches > 0 && n_grid > 0);
    MMPDE_REQUIRE(n_grid % batches == 0 && al16(workspace) && ((uintptr_t)grid & 7u) == 0);
    if (!head_ok(hd)) return MMPDE_ERR_UNSUPPORTED;
    hipStream_t st = as_stream(stream);
    const int L = hd->latent, Lp = hd->hidden;
    HeadWs w = carve_head((float *)workspace, batches, n_grid, L, Lp, hd->th);
    int rc = dmm_head_grid(grid, n_grid, hd, w, w.q, w.jac, st);  // trunk(grid), Q
    if (rc) return rc;
    // P = Wb . branch + b_o1
    rc = mmpde_linear_skinny(branch, L, batches, L, hd->o0_w, 2 * L, hd->o0_b, Lp, MMPDE_ACT_NONE, w.p, Lp,
                             stream);
    if (rc) return rc;
    hipLaunchKernelGGL(phi_kernel, dim3((unsigned)ceil_div(n_grid, 4)), dim3(256), 0, st, w.p, w.q, hd->o1_w,
                       o1_b, n_grid, n_grid / batches, Lp, phi_out, second_out);
    MMPDE_RET_LAUNCH();
    return MMPDE_OK;
}
