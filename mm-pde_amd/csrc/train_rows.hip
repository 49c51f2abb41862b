// Row reductions of the training path (reference train_helper_2d.py:114-126:
// loss.backward() through MP_PDE_Solver_2D, gnn_2d.py:19-141):
//
//  * skinny weight gradients: dW = dY^T X, db = sum_rows dY for a linear map
//    with few outputs (k * n_out + n_out <= 1280: the Conv1d head written as
//    unfold + GEMM, gnn_2d.py:108-114, and the embedding's first Linear,
//    gnn_2d.py:99-106) over a very long row axis (n nodes x window positions).
//    The library GEMM with K = rows picks tiles of a 16 x 16 output and one
//    serial K loop (562-808 us per call at cy B=16, profiles/
//    r04_train_kernel_stats_f16x3.csv); here every workgroup reduces a row
//    range into partials and one wave per output sums them: HBM-bound.
//  * BatchNorm1d in train mode over [n, C] rows (torch_geometric BatchNorm =
//    nn.BatchNorm1d, gnn_2d.py:51,69,101,105) with the residual add of
//    GNN_Layer_FS_2D.forward (norm(h + upd), gnn_2d.py:69) fused in: batch
//    statistics (per-thread Welford, Chan merges in a fixed order), running
//    statistics update, the normalisation; backward with the two channel sums
//    and the elementwise input gradient.
//
// Every sum runs in a fixed order (no atomics): results are deterministic.
#include "common.hpp"

#include <algorithm>
#include <hipcub/hipcub.hpp>

namespace {

constexpr int KMAX = 64;   // x columns (k) of the weight-gradient kernel

struct RowsGradArgs {
    const float *x;
    int64_t ldx, rows;
    int k;
    const float *dy;
    int64_t ldy;
    int nout, outs;        // outs = k * nout (+ nout with the bias)
    int bias;
    int64_t rows_per;      // rows of one workgroup
    float *part;           // [gridDim.x][outs]
};

// Partials of dW (and db) over the rows [blockIdx.x * rows_per, +rows_per).
// Thread t owns output row n = t % nout -- the k weights dW[n][:] and db[n]
// in registers -- for the rows of its row group t / nout (RG = 256 / nout
// groups, rows r0 + rg, r0 + rg + RG, ...): it streams x[row][0..k) (the
// threads of one row read the same addresses) and dy[row][n].  The row groups
// are then added in a fixed order, one output column at a time: a butterfly
// within each wave and the 4 waves in order (nout a power of two <= 64), or
// the groups in order through LDS.
template <int KB, bool VEC>
__global__ __launch_bounds__(256) void rows_grad_partial_kernel(RowsGradArgs p) {
    __shared__ float red[256];
    const int tid = threadIdx.x, nout = p.nout, k = p.k;
    const int RG = 256 / nout, rg = tid / nout, n = tid - rg * nout;
    const int64_t r0 = (int64_t)blockIdx.x * p.rows_per;
    const int64_t r1 = std::min(p.rows, r0 + p.rows_per);
    float acc[KB + 1];
#pragma unroll
    for (int c = 0; c <= KB; ++c) acc[c] = 0.0f;
    if (rg < RG) {
#pragma unroll 2
        for (int64_t r = r0 + rg; r < r1; r += RG) {
            const float g = p.dy[r * p.ldy + n];
            const float *xr = p.x + r * p.ldx;
            // the whole row first, unconditionally (columns past k re-read the
            // row's last ones and are dropped): a load under the c < k test is
            // waited for where the test ends, one round trip per column group
            float xv[KB > 0 ? KB : 1];
            if (KB > 16) {  // KB = 64: column groups as loaded (a whole row in
                            // registers costs occupancy, profiles/r05_loads_ab.log)
                if (VEC) {
#pragma unroll
                    for (int c = 0; c < KB; c += 4)
                        if (c < k) {
                            const float4 v = *(const float4 *)(xr + c);
                            acc[c] = fmaf(g, v.x, acc[c]);
                            acc[c + 1] = fmaf(g, v.y, acc[c + 1]);
                            acc[c + 2] = fmaf(g, v.z, acc[c + 2]);
                            acc[c + 3] = fmaf(g, v.w, acc[c + 3]);
                        }
                } else {
#pragma unroll
                    for (int c = 0; c < KB; ++c)
                        if (c < k) acc[c] = fmaf(g, xr[c], acc[c]);
                }
                acc[KB] += g;
                continue;
            }
            if (VEC) {  // 16-byte row loads (k, ldx multiples of 4, x aligned)
#pragma unroll
                for (int c = 0; c < KB; c += 4) {
                    const float4 v = *(const float4 *)(xr + min(c, k - 4));
                    xv[c] = v.x;
                    xv[c + 1] = v.y;
                    xv[c + 2] = v.z;
                    xv[c + 3] = v.w;
                }
            } else {
#pragma unroll
                for (int c = 0; c < KB; ++c) xv[c] = xr[min(c, k - 1)];
            }
#pragma unroll
            for (int c = 0; c < KB; ++c)
                if (c < k) acc[c] = fmaf(g, xv[c], acc[c]);
            acc[KB] += g;
        }
    }
    float *pp = p.part + (int64_t)blockIdx.x * p.outs;
    const int wave = tid >> 6, lane = tid & 63;
    const bool pow2 = nout <= 64 && (nout & (nout - 1)) == 0;
#pragma unroll
    for (int c = 0; c <= KB; ++c) {
        if (c < KB && c >= k) continue;
        if (c == KB && !p.bias) continue;
        const int o = c < KB ? n * k + c : k * nout + n;
        if (pow2) {
            // lanes l = n (mod nout) of a wave hold output n: a fixed butterfly
            // over them, then the 4 waves in order
            float v = acc[c];
            for (int off = 32; off >= nout; off >>= 1) v += __shfl_xor(v, off, 64);
            __syncthreads();
            if (lane < nout) red[wave * 64 + lane] = v;
            __syncthreads();
            if (tid < nout) pp[o] = ((red[tid] + red[64 + tid]) + red[128 + tid]) + red[192 + tid];
        } else {
            // a few row groups (nout > 64, or not a power of two): in group order
            __syncthreads();
            red[tid] = acc[c];
            __syncthreads();
            if (tid < nout) {
                float v = red[tid];
                for (int q = 1; q < RG; ++q) v += red[q * nout + tid];
                pp[o] = v;
            }
        }
    }
}

// The same partials for narrow outputs (n_out <= 8) over 16-byte rows (k a
// multiple of 4, k <= 64, ldx a multiple of 4, x aligned): lanes across the
// row instead of across the outputs.  Lane (rr, cq) of a wave, cq < Q = k / 4,
// rr < R = 64 / Q, takes columns 4 cq .. 4 cq + 3 of the rows r0 + 4 R s + R w +
// rr (s = 0, 1, ...; w the wave): one float4 of x per row -- the wave's R rows
// are one contiguous run when ldx = k -- and the row's NOUT dy values (a
// broadcast within the row's lanes); it keeps 4 x NOUT weight sums (+ NOUT bias
// sums, counted from the cq = 0 lanes).  Four rows per lane are loaded at once,
// unconditionally (rows past the range re-read the last one and are masked).
// The lanes' sums then meet in LDS and each output adds its (w, rr) lanes in
// that order: fixed order, deterministic.  (rows_grad_partial_kernel puts one
// output row per thread, so the threads of a row all read the whole row: 8 x
// the L1 requests at n_out = 8, and at n_out = 1 a wave's lanes in 64 rows.)
template <int NOUT>
__global__ __launch_bounds__(256) void rows_grad_cols_kernel(RowsGradArgs p) {
    constexpr int NV = 4 * NOUT + NOUT;  // sums per lane
    __shared__ float red[256 * NV];
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const int k = p.k, Q = k >> 2, R = 64 / Q;
    const int rr = lane / Q, cq = lane - rr * Q;
    const int64_t r0 = (int64_t)blockIdx.x * p.rows_per;
    const int64_t r1 = std::min(p.rows, r0 + p.rows_per);
    float acc[4][NOUT], bacc[NOUT];
#pragma unroll
    for (int n = 0; n < NOUT; ++n) {
        bacc[n] = 0.0f;
#pragma unroll
        for (int c = 0; c < 4; ++c) acc[c][n] = 0.0f;
    }
    if (rr < R) {
        const int64_t step = 4 * (int64_t)R;
        for (int64_t rb = r0 + (int64_t)R * wave + rr; rb < r1; rb += 4 * step) {
            float4 xv[4];
            float gv[4][NOUT];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int64_t r = std::min(rb + u * step, r1 - 1);
                xv[u] = *(const float4 *)(p.x + r * p.ldx + 4 * cq);
                const float *dr = p.dy + r * p.ldy;
#pragma unroll
                for (int n = 0; n < NOUT; ++n) gv[u][n] = dr[n];
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                int m = rb + u * step < r1 ? -1 : 0;
                asm volatile("" : "+v"(m));
                const float xs[4] = {xv[u].x, xv[u].y, xv[u].z, xv[u].w};
#pragma unroll
                for (int n = 0; n < NOUT; ++n) {
                    const float g = __int_as_float(__float_as_int(gv[u][n]) & m);
#pragma unroll
                    for (int c = 0; c < 4; ++c) acc[c][n] = fmaf(g, xs[c], acc[c][n]);
                    bacc[n] += g;
                }
            }
        }
    }
    float *rl = red + tid * NV;
#pragma unroll
    for (int n = 0; n < NOUT; ++n) {
#pragma unroll
        for (int c = 0; c < 4; ++c) rl[c * NOUT + n] = acc[c][n];
        rl[4 * NOUT + n] = bacc[n];
    }
    __syncthreads();
    float *pp = p.part + (int64_t)blockIdx.x * p.outs;
    for (int o = tid; o < p.outs; o += 256) {
        int l0, slot;  // lane (cq) and sum index of output o
        if (o < k * NOUT) {
            const int n = o / k, c = o - n * k;
            l0 = c >> 2;
            slot = (c & 3) * NOUT + n;
        } else {
            l0 = 0;
            slot = 4 * NOUT + (o - k * NOUT);
        }
        float v = 0.0f;
        for (int w = 0; w < 4; ++w)
            for (int q = 0; q < R; ++q) v += red[(w * 64 + q * Q + l0) * NV + slot];
        pp[o] = v;
    }
}

// out[o] = sum_g part[g][o]: one wave per output, lane l summing g = l, l + 64,
// ... in order, then a fixed butterfly.
__global__ __launch_bounds__(256) void wave_partial_sum_kernel(const float *__restrict__ part, int G, int outs,
                                                               float *__restrict__ out0, int n0,
                                                               float *__restrict__ out1) {
    const int o = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (o >= outs) return;
    float s = 0.0f;
    for (int g = lane; g < G; g += 64) s += part[(int64_t)g * outs + o];
    s = wave_sum(s);
    if (lane == 0) {
        if (o < n0)
            out0[o] = s;
        else
            out1[o - n0] = s;
    }
}

// ---------------------------------------------------------------------------
// BatchNorm1d (train) over rows x [n, C] (+ res), C % 4 == 0, C <= 1024.
// Thread layout of the row kernels: c4 = tid % (C / 4) (a float4 of channels),
// row group rg = tid / (C / 4) of RG = 256 / (C / 4); a workgroup walks the
// rows [r0, r1) with stride RG.
// ---------------------------------------------------------------------------
struct BnRowsArgs {
    const float *x, *res;  // res nullable: the input is x + res
    const float *dy;       // backward only
    int64_t n;
    int C;
    int64_t rows_per;
    const float *mean;     // backward: the saved batch mean
    float *part;           // forward [G][2C + 4] (count, 3 pad, mean, M2); backward [G][2C]
};

__device__ __forceinline__ float4 ld4(const float *p) { return *(const float4 *)p; }
__device__ __forceinline__ float4 add4(float4 a, float4 b) {
    return make_float4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w);
}

// Chan et al. merge of (na, ma, Ma) with (nb, mb, Mb) into the first.
__device__ __forceinline__ void chan_merge(float &na, float &ma, float &Ma, float nb, float mb, float Mb) {
    const float nn = na + nb;
    if (nb == 0.0f) return;
    const float d = mb - ma, f = nb / nn;
    ma = fmaf(d, f, ma);
    Ma = Ma + Mb + d * d * na * f;
    na = nn;
}

__global__ __launch_bounds__(256) void bn_stats_partial_kernel(BnRowsArgs p) {
    __shared__ float sm[256 * 4], sM[256 * 4], sc[256];
    const int C4 = p.C >> 2, RG = 256 / C4;
    const int tid = threadIdx.x, rg = tid / C4, c4 = tid - rg * C4;
    const int64_t r0 = (int64_t)blockIdx.x * p.rows_per, r1 = std::min(p.n, r0 + p.rows_per);
    float cnt = 0.0f;
    float m[4] = {0.0f, 0.0f, 0.0f, 0.0f}, M[4] = {0.0f, 0.0f, 0.0f, 0.0f};
    if (rg < RG) {
        for (int64_t r = r0 + rg; r < r1; r += RG) {
            float4 v = ld4(p.x + r * p.C + 4 * c4);
            if (p.res) v = add4(v, ld4(p.res + r * p.C + 4 * c4));
            cnt += 1.0f;
            const float inv = 1.0f / cnt;
            const float vv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
            for (int q = 0; q < 4; ++q) {  // Welford
                const float d = vv[q] - m[q];
                m[q] = fmaf(d, inv, m[q]);
                M[q] = fmaf(d, vv[q] - m[q], M[q]);
            }
        }
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        sm[tid * 4 + q] = m[q];
        sM[tid * 4 + q] = M[q];
    }
    sc[tid] = cnt;
    __syncthreads();
    if (rg == 0) {  // merge the row groups in rg order
        float n0 = cnt;
        for (int g = 1; g < RG; ++g) {
            const int t = g * C4 + c4;
            float nb = sc[t];
            float na = n0;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                float nq = na;
                chan_merge(nq, m[q], M[q], nb, sm[t * 4 + q], sM[t * 4 + q]);
            }
            n0 = na + nb;
        }
        float *pp = p.part + (int64_t)blockIdx.x * (2 * p.C + 4);
        if (c4 == 0) pp[0] = n0;
        *(float4 *)&pp[4 + 4 * c4] = make_float4(m[0], m[1], m[2], m[3]);
        *(float4 *)&pp[4 + p.C + 4 * c4] = make_float4(M[0], M[1], M[2], M[3]);
    }
}

// Per channel (one workgroup each): merge the G partials -- thread t walks
// g = t, t + 256, ... in order, then a fixed LDS tree; mean, invstd (saved for
// the backward), the affine a = w invstd, c = b - mean a, and the running
// statistics (torch: r = (1 - f) r + f stat, the variance unbiased).
__global__ __launch_bounds__(256) void bn_stats_final_kernel(const float *__restrict__ part, int G, int C,
                                                             float eps, float factor, const float *__restrict__ w,
                                                             const float *__restrict__ b, float *__restrict__ rmean,
                                                             float *__restrict__ rvar, float *__restrict__ stats) {
    __shared__ float sn[256], sm[256], sM[256];
    const int c = blockIdx.x, t = threadIdx.x;
    const int64_t stride = 2 * C + 4;
    float na = 0.0f, ma = 0.0f, Ma = 0.0f;
    for (int g = t; g < G; g += 256) {
        const float *pp = part + (int64_t)g * stride;
        chan_merge(na, ma, Ma, pp[0], pp[4 + c], pp[4 + C + c]);
    }
    sn[t] = na;
    sm[t] = ma;
    sM[t] = Ma;
    __syncthreads();
    for (int s = 128; s >= 1; s >>= 1) {
        if (t < s) {
            chan_merge(na, ma, Ma, sn[t + s], sm[t + s], sM[t + s]);
            sn[t] = na;
            sm[t] = ma;
            sM[t] = Ma;
        }
        __syncthreads();
    }
    if (t != 0) return;
    const float var = Ma / na;
    const float invstd = 1.0f / sqrtf(var + eps);
    const float a = w ? w[c] * invstd : invstd;
    stats[c] = ma;
    stats[C + c] = invstd;
    stats[2 * C + c] = a;
    stats[3 * C + c] = (b ? b[c] : 0.0f) - ma * a;
    if (rmean) rmean[c] = factor * ma + (1.0f - factor) * rmean[c];
    if (rvar) rvar[c] = factor * (na > 1.0f ? Ma / (na - 1.0f) : var) + (1.0f - factor) * rvar[c];
}

// y = (x + res) a + c
__global__ __launch_bounds__(256) void bn_apply_kernel(const float *__restrict__ x, const float *__restrict__ res,
                                                       int64_t n4, int C4, const float *__restrict__ stats, int C,
                                                       float *__restrict__ y) {
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (int64_t)gridDim.x * 256) {
        const int c = 4 * (int)(i % C4);
        float4 v = ((const float4 *)x)[i];
        if (res) v = add4(v, ((const float4 *)res)[i]);
        const float4 a = ld4(stats + 2 * C + c), s = ld4(stats + 3 * C + c);
        ((float4 *)y)[i] = make_float4(fmaf(v.x, a.x, s.x), fmaf(v.y, a.y, s.y), fmaf(v.z, a.z, s.z),
                                       fmaf(v.w, a.w, s.w));
    }
}

// backward partials: sum dy and sum dy (x - mean) per channel
__global__ __launch_bounds__(256) void bn_bwd_partial_kernel(BnRowsArgs p) {
    __shared__ float s1[256 * 4], s2[256 * 4];
    const int C4 = p.C >> 2, RG = 256 / C4;
    const int tid = threadIdx.x, rg = tid / C4, c4 = tid - rg * C4;
    const int64_t r0 = (int64_t)blockIdx.x * p.rows_per, r1 = std::min(p.n, r0 + p.rows_per);
    float a[4] = {0.0f, 0.0f, 0.0f, 0.0f}, bsum[4] = {0.0f, 0.0f, 0.0f, 0.0f};
    if (rg < RG) {
        const float4 mu = ld4(p.mean + 4 * c4);
        const float mv[4] = {mu.x, mu.y, mu.z, mu.w};
        for (int64_t r = r0 + rg; r < r1; r += RG) {
            float4 v = ld4(p.x + r * p.C + 4 * c4);
            if (p.res) v = add4(v, ld4(p.res + r * p.C + 4 * c4));
            const float4 g = ld4(p.dy + r * p.C + 4 * c4);
            const float vv[4] = {v.x, v.y, v.z, v.w}, gg[4] = {g.x, g.y, g.z, g.w};
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                a[q] += gg[q];
                bsum[q] = fmaf(gg[q], vv[q] - mv[q], bsum[q]);
            }
        }
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        s1[tid * 4 + q] = a[q];
        s2[tid * 4 + q] = bsum[q];
    }
    __syncthreads();
    if (rg == 0) {
        for (int g = 1; g < RG; ++g) {
            const int t = g * C4 + c4;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                a[q] += s1[t * 4 + q];
                bsum[q] += s2[t * 4 + q];
            }
        }
        float *pp = p.part + (int64_t)blockIdx.x * 2 * p.C;
        *(float4 *)&pp[4 * c4] = make_float4(a[0], a[1], a[2], a[3]);
        *(float4 *)&pp[p.C + 4 * c4] = make_float4(bsum[0], bsum[1], bsum[2], bsum[3]);
    }
}

// Per channel (one workgroup each): sdy, sdyx over the partials (strided
// per-thread sums, fixed LDS tree); dgamma = sdyx invstd, dbeta = sdy; the
// input-gradient constants k1 = w invstd, k2 = sdy / n, k3 = invstd^2 sdyx / n
// (torch batch_norm_backward_elemt).
__global__ __launch_bounds__(256) void bn_bwd_final_kernel(const float *__restrict__ part, int G, int C, int64_t n,
                                                           const float *__restrict__ w,
                                                           const float *__restrict__ stats, float *__restrict__ dw,
                                                           float *__restrict__ db, float *__restrict__ kc) {
    __shared__ float r1[256], r2[256];
    const int c = blockIdx.x, t = threadIdx.x;
    float s1 = 0.0f, s2 = 0.0f;
    for (int g = t; g < G; g += 256) {
        s1 += part[(int64_t)g * 2 * C + c];
        s2 += part[(int64_t)g * 2 * C + C + c];
    }
    r1[t] = s1;
    r2[t] = s2;
    __syncthreads();
    for (int s = 128; s >= 1; s >>= 1) {
        if (t < s) {
            r1[t] += r1[t + s];
            r2[t] += r2[t + s];
        }
        __syncthreads();
    }
    if (t != 0) return;
    s1 = r1[0];
    s2 = r2[0];
    const float invstd = stats[C + c];
    if (dw) dw[c] = s2 * invstd;
    if (db) db[c] = s1;
    const float inv_n = 1.0f / (float)n;
    kc[c] = w ? w[c] * invstd : invstd;
    kc[C + c] = s1 * inv_n;
    kc[2 * C + c] = invstd * invstd * (s2 * inv_n);
}

// dx = k1 (dy - k2 - (x + res - mean) k3)
__global__ __launch_bounds__(256) void bn_bwd_apply_kernel(const float *__restrict__ x, const float *__restrict__ res,
                                                           const float *__restrict__ dy, int64_t n4, int C4,
                                                           const float *__restrict__ mean,
                                                           const float *__restrict__ kc, int C,
                                                           float *__restrict__ dx) {
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (int64_t)gridDim.x * 256) {
        const int c = 4 * (int)(i % C4);
        float4 v = ((const float4 *)x)[i];
        if (res) v = add4(v, ((const float4 *)res)[i]);
        const float4 g = ((const float4 *)dy)[i], mu = ld4(mean + c);
        const float4 k1 = ld4(kc + c), k2 = ld4(kc + C + c), k3 = ld4(kc + 2 * C + c);
        ((float4 *)dx)[i] = make_float4(k1.x * (g.x - k2.x - (v.x - mu.x) * k3.x),
                                        k1.y * (g.y - k2.y - (v.y - mu.y) * k3.y),
                                        k1.z * (g.z - k2.z - (v.z - mu.z) * k3.z),
                                        k1.w * (g.w - k2.w - (v.w - mu.w) * k3.w));
    }
}

int device_cus() {
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
        cus = 256;
    return cus;
}

// workgroups of a row kernel: >= 256 rows each, at most 4 per CU
int64_t row_blocks(int64_t rows, int64_t min_rows) {
    return std::max<int64_t>(1, std::min<int64_t>((int64_t)4 * device_cus(), (rows + min_rows - 1) / min_rows));
}

}  // namespace

// workgroups of the weight-gradient kernel: about 8 rows per thread
static int64_t rows_grad_blocks(int64_t rows, int n_out) {
    const int64_t per_block = (int64_t)(256 / n_out) * 8;
    return std::max<int64_t>(1, std::min<int64_t>((int64_t)4 * device_cus(), (rows + per_block - 1) / per_block));
}

// rows_grad_cols_kernel's shapes (the 16-byte row alignment is checked at launch)
static bool rows_grad_cols_shape(int k, int n_out) {
    return k >= 16 && k <= KMAX && k % 4 == 0 && (n_out == 1 || n_out == 2 || n_out == 4 || n_out == 8);
}

// its workgroups: at least two unrolled passes (8 rows per lane) each
static int64_t rows_grad_cols_blocks(int64_t rows, int k) {
    const int64_t per_block = 32 * (int64_t)(64 / (k / 4));
    return std::max<int64_t>(1, std::min<int64_t>((int64_t)4 * device_cus(), (rows + per_block - 1) / per_block));
}

extern "C" int64_t mmpde_rows_grad_weight_workspace_bytes(int64_t rows, int k, int n_out) {
    if (rows <= 0 || k < 0 || n_out <= 0 || n_out > 256) return 0;
    int64_t G = rows_grad_blocks(rows, n_out);
    if (rows_grad_cols_shape(k, n_out)) G = std::max(G, rows_grad_cols_blocks(rows, k));
    return G * (int64_t)(k * n_out + n_out) * 4;
}

extern "C" int mmpde_rows_grad_weight(const float *x, int64_t ldx, int64_t rows, int k, const float *dy, int64_t ldy,
                                      int n_out, float *dw, float *db, float *workspace, int64_t workspace_bytes,
                                      mmpde_stream_t stream) {
    MMPDE_REQUIRE(dy && rows > 0 && k >= 0 && k <= KMAX && n_out > 0 && n_out <= 128 && ldy >= n_out);
    MMPDE_REQUIRE(k == 0 || (x && dw && ldx >= k));
    MMPDE_REQUIRE(k > 0 || db);
    const int outs = k * n_out + (db ? n_out : 0);
    MMPDE_REQUIRE(outs <= 1280);
    MMPDE_REQUIRE(workspace && workspace_bytes >= mmpde_rows_grad_weight_workspace_bytes(rows, k, n_out));
    const bool vec = k % 4 == 0 && ldx % 4 == 0 && ((uintptr_t)x & 15) == 0;
    const bool cols = vec && rows_grad_cols_shape(k, n_out);
    const int64_t G0 = cols ? rows_grad_cols_blocks(rows, k) : rows_grad_blocks(rows, n_out);
    const int64_t per = (rows + G0 - 1) / G0, G = (rows + per - 1) / per;
    RowsGradArgs p{x, ldx, rows, k, dy, ldy, n_out, outs, db != nullptr, per, workspace};
    hipStream_t st = as_stream(stream);
    auto launch = [&](auto kern) { hipLaunchKernelGGL(kern, dim3((unsigned)G), dim3(256), 0, st, p); };
    if (cols) {
        if (n_out == 1) launch(rows_grad_cols_kernel<1>);
        else if (n_out == 2) launch(rows_grad_cols_kernel<2>);
        else if (n_out == 4) launch(rows_grad_cols_kernel<4>);
        else launch(rows_grad_cols_kernel<8>);
    } else if (k == 0)
        launch(rows_grad_partial_kernel<0, false>);
    else if (k <= 4)
        vec ? launch(rows_grad_partial_kernel<4, true>) : launch(rows_grad_partial_kernel<4, false>);
    else if (k <= 16)
        vec ? launch(rows_grad_partial_kernel<16, true>) : launch(rows_grad_partial_kernel<16, false>);
    else
        vec ? launch(rows_grad_partial_kernel<KMAX, true>) : launch(rows_grad_partial_kernel<KMAX, false>);
    MMPDE_RET_LAUNCH();
    hipLaunchKernelGGL(wave_partial_sum_kernel, dim3((unsigned)ceil_div(outs, 4)), dim3(256), 0, st, workspace,
                       (int)G, outs, dw, k * n_out, db);
    MMPDE_RET_LAUNCH();
    return MMPDE_OK;
}

extern "C" int64_t mmpde_batch_norm_rows_workspace_bytes(int64_t n, int C) {
    if (n <= 0 || C <= 0) return 0;
    return row_blocks(n, 64) * (int64_t)(2 * C + 4) * 4;
}

extern "C" int mmpde_batch_norm_rows_train(const float *x, const float *res, int64_t n, int C, const float *weight,
                                           const float *bias, float eps, float factor, float *running_mean,
                                           float *running_var, float *y, float *stats, float *workspace,
                                           int64_t workspace_bytes, mmpde_stream_t stream) {
    MMPDE_REQUIRE(x && y && stats && workspace && n > 0 && C > 0 && C % 4 == 0 && C <= 1024);
    MMPDE_REQUIRE(((((uintptr_t)x | (uintptr_t)res | (uintptr_t)y | (uintptr_t)stats | (uintptr_t)workspace)) & 15) == 0);
    MMPDE_REQUIRE(workspace_bytes >= mmpde_batch_norm_rows_workspace_bytes(n, C));
    const int64_t G0 = row_blocks(n, 64);
    const int64_t per = (n + G0 - 1) / G0, G = (n + per - 1) / per;
    BnRowsArgs p{x, res, nullptr, n, C, per, nullptr, workspace};
    hipStream_t st = as_stream(stream);
    hipLaunchKernelGGL(bn_stats_partial_kernel, dim3((unsigned)G), dim3(256), 0, st, p);
    hipLaunchKernelGGL(bn_stats_final_kernel, dim3((unsigned)C), dim3(256), 0, st, workspace, (int)G,
                       C, eps, factor, weight, bias, running_mean, running_var, stats);
    const int64_t n4 = n * C / 4;
    const unsigned blocks = (unsigned)std::min<int64_t>(ceil_div(n4, 256), (int64_t)8 * device_cus());
    hipLaunchKernelGGL(bn_apply_kernel, dim3(blocks), dim3(256), 0, st, x, res, n4, C / 4, stats, C, y);
    MMPDE_RET_LAUNCH();
    return MMPDE_OK;
}

extern "C" int mmpde_batch_norm_rows_backward(const float *x, const float *res, const float *dy, int64_t n, int C,
                                              const float *weight, const float *stats, float *dx, float *dweight,
                                              float *dbias, float *workspace, int64_t workspace_bytes,
                                              mmpde_stream_t stream) {
    MMPDE_REQUIRE(x && dy && dx && stats && workspace && n > 0 && C > 0 && C % 4 == 0 && C <= 1024);
    MMPDE_REQUIRE(((((uintptr_t)x | (uintptr_t)res | (uintptr_t)dy | (uintptr_t)dx | (uintptr_t)stats |
                     (uintptr_t)workspace)) & 15) == 0);
    MMPDE_REQUIRE(workspace_bytes >= mmpde_batch_norm_rows_workspace_bytes(n, C) + 3 * C * 4);
    const int64_t G0 = row_blocks(n, 64);
    const int64_t per = (n + G0 - 1) / G0, G = (n + per - 1) / per;
    float *kc = workspace + G * 2 * C;
    BnRowsArgs p{x, res, dy, n, C, per, stats, workspace};
    hipStream_t st = as_stream(stream);
    hipLaunchKernelGGL(bn_bwd_partial_kernel, dim3((unsigned)G), dim3(256), 0, st, p);
    hipLaunchKernelGGL(bn_bwd_final_kernel, dim3((unsigned)C), dim3(256), 0, st, workspace, (int)G, C,
                       n, weight, stats, dweight, dbias, kc);
    const int64_t n4 = n * C / 4;
    const unsigned blocks = (unsigned)std::min<int64_t>(ceil_div(n4, 256), (int64_t)8 * device_cus());
    hipLaunchKernelGGL(bn_bwd_apply_kernel, dim3(blocks), dim3(256), 0, st, x, res, dy, n4, C / 4, stats, kc, C, dx);
    MMPDE_RET_LAUNCH();
    return MMPDE_OK;
}

// ---------------------------------------------------------------------------
// Reverse adjacency of a target-major neighbour table (the source-side sums of
// the edge-stage backward, mmpde_gnn_edge_source_sum, and of row gathers,
// mmpde_segment_sum): rev_edge = the live slot ids q = i k + e grouped by
// source j = nbr[i][e], ascending q within a source (stable), rev_off [n_src +
// 1] the group offsets.  One stable LSD radix sort of (key = source, value =
// q) pairs over just the bits a source index takes (hipCUB/rocPRIM; two 8-bit
// passes for up to 65535 sources), dead and out-of-range slots keyed n_src so
// that they sort past the end; then rev_off[j] = lower_bound(keys, j).
// ---------------------------------------------------------------------------
namespace {

__global__ __launch_bounds__(256) void rev_keys_kernel(const int32_t *__restrict__ nbr, int64_t slots, int k,
                                                       const int32_t *__restrict__ deg, int32_t n_src,
                                                       int32_t *__restrict__ keys, int64_t *__restrict__ vals,
                                                       int32_t *__restrict__ bad) {
    const int64_t q = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (q >= slots) return;
    const int64_t i = q / k;
    const int e = (int)(q - i * k);
    int32_t key = n_src;
    if (!deg || e < deg[i]) {
        const int32_t j = nbr[q];
        if (j >= 0 && j < n_src)
            key = j;
        else
            atomicAdd(bad, 1);
    }
    keys[q] = key;
    vals[q] = q;
}

// off[j] = first position whose key >= j (j = 0 .. n_src)
__global__ __launch_bounds__(256) void rev_offsets_kernel(const int32_t *__restrict__ keys, int64_t slots,
                                                          int32_t n_src, int64_t *__restrict__ off) {
    const int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (j > n_src) return;
    int64_t lo = 0, hi = slots;
    while (lo < hi) {
        const int64_t mid = (lo + hi) >> 1;
        if (keys[mid] < j)
            lo = mid + 1;
        else
            hi = mid;
    }
    off[j] = lo;
}

// slot_pos[rev_edge[p]] = p
__global__ __launch_bounds__(256) void rev_pos_kernel(const int64_t *__restrict__ rev_edge, int64_t slots,
                                                      int32_t *__restrict__ pos) {
    const int64_t p = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (p < slots) pos[rev_edge[p]] = (int32_t)p;
}

int key_bits(int64_t n_src) {
    int b = 1;
    while (b < 31 && ((int64_t)1 << b) <= n_src) ++b;  // keys 0 .. n_src
    return b;
}

size_t rev_sort_temp_bytes(int64_t slots, int64_t n_src) {
    size_t tb = 0;
    if (hipcub::DeviceRadixSort::SortPairs(nullptr, tb, (const int32_t *)nullptr, (int32_t *)nullptr,
                                           (const int64_t *)nullptr, (int64_t *)nullptr, (int)slots, 0,
                                           key_bits(n_src), (hipStream_t)0) != hipSuccess)
        return (size_t)1 << 40;  // no usable size: the caller's allocation fails loudly
    return (tb + 255) / 256 * 256;
}

}  // namespace

extern "C" int64_t mmpde_reverse_adjacency_scratch_bytes(int64_t n_tgt, int k, int64_t n_src) {
    if (n_tgt <= 0 || k <= 0 || n_src <= 0) return 0;
    const int64_t slots = n_tgt * (int64_t)k;
    // keys in, keys out (int32), values in (int64), the sort's temporary storage
    return 2 * ((slots * 4 + 255) / 256 * 256) + (slots * 8 + 255) / 256 * 256 +
           (int64_t)rev_sort_temp_bytes(slots, n_src);
}

extern "C" int mmpde_reverse_adjacency(const int32_t *nbr, int64_t n_tgt, int k, const int32_t *deg, int64_t n_src,
                                       int64_t *rev_off, int64_t *rev_edge, int32_t *slot_pos, void *scratch,
                                       int64_t scratch_bytes, int32_t *bad, mmpde_stream_t stream) {
    MMPDE_REQUIRE(nbr && rev_off && rev_edge && scratch && bad && n_tgt > 0 && k > 0 && n_src > 0);
    const int64_t slots = n_tgt * (int64_t)k;
    MMPDE_REQUIRE(n_src < (int64_t)INT32_MAX && slots < (int64_t)INT32_MAX);
    MMPDE_REQUIRE(scratch_bytes >= mmpde_reverse_adjacency_scratch_bytes(n_tgt, k, n_src));
    MMPDE_REQUIRE((((uintptr_t)scratch) & 255) == 0);
    char *sp = (char *)scratch;
    int32_t *keys_in = (int32_t *)sp;
    sp += (slots * 4 + 255) / 256 * 256;
    int32_t *keys_out = (int32_t *)sp;
    sp += (slots * 4 + 255) / 256 * 256;
    int64_t *vals_in = (int64_t *)sp;
    sp += (slots * 8 + 255) / 256 * 256;
    size_t tb = rev_sort_temp_bytes(slots, n_src);
    hipStream_t st = as_stream(stream);
    if (hipMemsetAsync(bad, 0, 4, st) != hipSuccess) return MMPDE_ERR_HIP_BASE;
    hipLaunchKernelGGL(rev_keys_kernel, dim3((unsigned)ceil_div(slots, 256)), dim3(256), 0, st, nbr, slots, k, deg,
                       (int32_t)n_src, keys_in, vals_in, bad);
    MMPDE_RET_LAUNCH();
    const hipError_t e = hipcub::DeviceRadixSort::SortPairs((void *)sp, tb, keys_in, keys_out, vals_in, rev_edge,
                                                            (int)slots, 0, key_bits(n_src), st);
    if (e != hipSuccess) return MMPDE_ERR_HIP_BASE - (int)e;
    hipLaunchKernelGGL(rev_offsets_kernel, dim3((unsigned)ceil_div(n_src + 1, 256)), dim3(256), 0, st, keys_out,
                       slots, (int32_t)n_src, rev_off);
    if (slot_pos)
        hipLaunchKernelGGL(rev_pos_kernel, dim3((unsigned)ceil_div(slots, 256)), dim3(256), 0, st, rev_edge, slots,
                           slot_pos);
    MMPDE_RET_LAUNCH();
    return MMPDE_OK;
}
