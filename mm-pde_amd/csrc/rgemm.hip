// Row GEMMs of the training path (reference train_helper_2d.py:114-126:
// loss.backward() through the train-mode MP_PDE_Solver_2D, gnn_2d.py:53-69,
// 99-106, and ItpNet, interpolate.py:79-93).  The Linears act on rows (n =
// B x 2521 nodes or queries) with <= 128 outputs per block:
//
//   rgemm     y = x W^T (layout NT: the forward) or y = g W (NN: the input
//             gradient), the concatenated inputs of the reference (cat(h, agg,
//             t), cat(h_i, h_j, u_i - u_j, dx, dy, t_i)) read in place as two
//             K halves plus a <= 4-column small segment, with the bias, ReLU,
//             ReLU-backward masks and the residual accumulation fused in.
//   rgemm_tn  dW = G^T X and db = sum G over the row axis in fixed row chunks
//             (partials, then a fixed-order sum): deterministic.
//
// Exact fp32 products on v_mfma_f32_32x32x2_f32 (lane l supplies A[l & 31][l
// >> 5] and B[l >> 5][l & 31]).  A workgroup is 4 waves: rgemm covers 32 rows
// x 128 columns (each wave one 32 x 32 tile); k-lane 0 walks K half 0, k-lane
// 1 half 1, so one GEMM consumes two input tensors side by side without
// building their concatenation.  VEC: float4 row loads (kh % 4 == 0, 16-byte
// aligned rows; NT: W rows too), else one k per step.
#include "common.hpp"

namespace {

constexpr int RG_TILE = 32;

__device__ __forceinline__ float4 mask4(float4 a, const float4 &q) {
    return make_float4(q.x > 0.0f ? a.x : 0.0f, q.y > 0.0f ? a.y : 0.0f, q.z > 0.0f ? a.z : 0.0f,
                       q.w > 0.0f ? a.w : 0.0f);
}

template <int LAYOUT, bool VEC, bool AMASK, bool XS>
__global__ __launch_bounds__(256) void rgemm_kernel(mmpde_rgemm_args g) {
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int h = lane >> 5, j = lane & 31;
    const int p = blockIdx.y;
    if (32 * wave >= g.ncols[p]) return;          // a wave of columns past the part (skinny maps)
    const int64_t row0 = (int64_t)blockIdx.x * RG_TILE;
    const int64_t m = g.m;
    const int64_t row = min(row0 + j, m - 1);   // clamped: loads stay in bounds
    const int col = 32 * wave + j;                // output column within the part
    const int ncols = g.ncols[p];
    const int colc = min(col, ncols - 1);         // clamped for the W loads
    // four accumulation chains (k = 4 s + q goes to chain q), added pairwise at
    // the end: sums of kh / 4 terms per chain instead of one chain of kh
    f32x16 c0 = {0}, c1 = {0}, c2 = {0}, c3 = {0};
    if (g.kh > 0) {
        const float *ap = g.a[h] + row * g.lda[h];
        const float *mp = AMASK ? g.amask[h] + row * g.lda[h] : nullptr;
        const int64_t ldw = g.ldw;
        const int kh = g.kh;
        if (LAYOUT == MMPDE_RGEMM_NT) {
            const float *wp = g.w[h] + (g.wc[p] + colc) * ldw + g.wk[p];
            if (VEC) {
#pragma unroll 2
                for (int s = 0; s < kh; s += 4) {
                    float4 a = *(const float4 *)(ap + s);
                    if (AMASK) a = mask4(a, *(const float4 *)(mp + s));
                    const float4 w = *(const float4 *)(wp + s);
                    c0 = mfma32(a.x, w.x, c0);
                    c1 = mfma32(a.y, w.y, c1);
                    c2 = mfma32(a.z, w.z, c2);
                    c3 = mfma32(a.w, w.w, c3);
                }
            } else {
                for (int s = 0; s < kh; s += 4) {
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        const int kk = min(s + q, kh - 1);
                        float a = ap[kk];
                        if (AMASK) a = mp[kk] > 0.0f ? a : 0.0f;
                        a = s + q < kh ? a : 0.0f;
                        f32x16 &c = q == 0 ? c0 : q == 1 ? c1 : q == 2 ? c2 : c3;
                        c = mfma32(a, wp[kk], c);
                    }
                }
            }
        } else {
            const float *wp = g.w[h] + g.wk[p] * ldw + g.wc[p] + colc;
            if (VEC) {
#pragma unroll 2
                for (int s = 0; s < kh; s += 4) {
                    float4 a = *(const float4 *)(ap + s);
                    if (AMASK) a = mask4(a, *(const float4 *)(mp + s));
                    const float *w = wp + s * ldw;
                    c0 = mfma32(a.x, w[0], c0);
                    c1 = mfma32(a.y, w[ldw], c1);
                    c2 = mfma32(a.z, w[2 * ldw], c2);
                    c3 = mfma32(a.w, w[3 * ldw], c3);
                }
            } else {
                for (int s = 0; s < kh; s += 4) {
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        const int kk = min(s + q, kh - 1);
                        float a = ap[kk];
                        if (AMASK) a = mp[kk] > 0.0f ? a : 0.0f;
                        a = s + q < kh ? a : 0.0f;
                        f32x16 &c = q == 0 ? c0 : q == 1 ? c1 : q == 2 ? c2 : c3;
                        c = mfma32(a, wp[kk * ldw], c);
                    }
                }
            }
        }
    }
    const f32x16 acc = (c0 + c1) + (c2 + c3);
    if (col >= ncols) return;
    // epilogue: D[acc_row(r)][col]
    const float bias = g.bias[p] ? g.bias[p][col] : 0.0f;
    const int ns = XS ? g.ns[p] : 0;
    float xw[4] = {0.0f, 0.0f, 0.0f, 0.0f};
    if (XS) {
#pragma unroll
        for (int e = 0; e < 4; ++e)
            if (e < ns)
                xw[e] = g.xscale[p] * (LAYOUT == MMPDE_RGEMM_NT ? g.xw[p][(int64_t)col * g.ldxw + e]
                                                                : g.xw[p][(int64_t)e * g.ldxw + col]);
    }
    float *out = g.out[p];
    const float *om = g.omask[p];
    const bool accum = g.accumulate[p] != 0;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const int64_t i = row0 + acc_row(r, lane);
        if (i >= m) continue;
        float y = acc[r] + bias;
        if (XS) {
#pragma unroll
            for (int e = 0; e < 4; ++e)
                if (e < ns) y = fmaf(g.xs[i * g.ldxs + e], xw[e], y);
        }
        if (g.relu) y = fmaxf(y, 0.0f);
        if (om) y = om[i * g.ldom[p] + col] > 0.0f ? y : 0.0f;
        float *o = out + i * g.ldo[p] + col;
        *o = accum ? *o + y : y;
    }
}

// ---------------------------------------------------------------------------
// dW = G^T X over the rows.  Partials: workspace [chunks][128][cols]; the
// column space is every segment rounded up to 32 columns (segment s starts at
// base(s) = sum of the rounded widths before it), then the ns small-segment
// columns, then db.  Workgroup (kt, chunk): wave w the 32 x 32 tile (c = 32 w
// .., k = 32 kt ..) over the chunk's rows, two rows per MFMA (row parity =
// k-lane); the kt = 0 workgroups also sum the small segment and db from the
// same G values on the VALU.
// ---------------------------------------------------------------------------
struct TnArgs {
    mmpde_rgemm_tn_args g;
    int cols, kbig;  // partial columns; rounded big-segment columns
    int base[3];     // first partial column of each segment
    float *part;
};

template <bool GMASK>
__global__ __launch_bounds__(256) void rgemm_tn_partial_kernel(TnArgs t) {
    const mmpde_rgemm_tn_args &g = t.g;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int par = lane >> 5, j = lane & 31;
    const int chunk = blockIdx.y;
    const int64_t r0 = (int64_t)chunk * g.chunk_rows;
    const int64_t r1 = min(r0 + (int64_t)g.chunk_rows, g.m);
    const int c = 32 * wave + j;  // G column of this lane's A element
    if (32 * wave >= g.gcols) return;  // no G column in this wave (the reduce never reads its rows)
    const bool cl = c < g.gcols;
    const int cc = cl ? c : g.gcols - 1;
    // k-tile -> segment, column within it
    const int kt = blockIdx.x * RG_TILE;
    int seg = 0;
    while (seg < g.nseg - 1 && kt >= t.base[seg + 1]) ++seg;
    const int kl = kt - t.base[seg] + j;        // column of this lane's B element in the segment
    const bool kv = kl < g.kx[seg];
    const float *xp = g.x[seg] + (kv ? kl : g.kx[seg] - 1);
    const int64_t ldx = g.ldx[seg];
    const bool first = blockIdx.x == 0;
    const int ns = first ? g.ns : 0;
    // four accumulation chains over the row steps (step s to chain s % 4),
    // added pairwise at the end
    f32x16 ch[4] = {{0}, {0}, {0}, {0}};
    float sx[4] = {0.0f, 0.0f, 0.0f, 0.0f}, sb = 0.0f;
    // wave-uniform trip count (an MFMA reads every lane): a row past r1 (odd
    // row count, k-lane 1 of the last step) contributes zeros
    const int64_t steps = (r1 - r0 + 1) / 2;
    for (int64_t s0 = 0; s0 < steps; s0 += 4) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int64_t s = s0 + q;
            const int64_t i0 = r0 + 2 * s + par;
            const bool live = i0 < r1 && cl;
            const int64_t i = i0 < r1 ? i0 : r1 - 1;
            float a = g.g[i * g.ldg + cc];
            if (GMASK) a = g.gmask[i * g.ldg + cc] > 0.0f ? a : 0.0f;
            a = live ? a : 0.0f;
            ch[q] = mfma32(a, xp[i * ldx], ch[q]);
            if (first) {
                sb += a;
#pragma unroll
                for (int e = 0; e < 4; ++e)
                    if (e < ns) sx[e] = fmaf(a, g.xs[i * g.ldxs + e], sx[e]);
            }
        }
    }
    const f32x16 acc = (ch[0] + ch[1]) + (ch[2] + ch[3]);
    float *pp = t.part + (int64_t)chunk * 128 * t.cols;
    const int kcol = kt + j;
#pragma unroll
    for (int r = 0; r < 16; ++r) pp[(int64_t)(32 * wave + acc_row(r, lane)) * t.cols + kcol] = acc[r];
    if (first) {
        // the two row parities of column c, in a fixed order
        sb += __shfl_xor(sb, 32, 64);
#pragma unroll
        for (int e = 0; e < 4; ++e) sx[e] += __shfl_xor(sx[e], 32, 64);
        if (par == 0) {
            float *q = pp + (int64_t)c * t.cols + t.kbig;
#pragma unroll
            for (int e = 0; e < 4; ++e)
                if (e < ns) q[e] = sx[e];
            q[g.ns] = sb;
        }
    }
}

// dw / db from the partials, chunks added in order.
__global__ __launch_bounds__(256) void rgemm_tn_reduce_kernel(TnArgs t, int chunks) {
    const mmpde_rgemm_tn_args &g = t.g;
    const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (idx >= (int64_t)g.gcols * t.cols) return;
    const int c = (int)(idx / t.cols), k = (int)(idx - (int64_t)c * t.cols);
    int seg = -1, kk = 0;
    if (k < t.kbig) {
        seg = 0;
        while (seg < g.nseg - 1 && k >= t.base[seg + 1]) ++seg;
        kk = k - t.base[seg];
        if (kk >= g.kx[seg]) return;  // padding column
    }
    float s = 0.0f;
    for (int q = 0; q < chunks; ++q) s += t.part[((int64_t)q * 128 + c) * t.cols + k];
    if (seg >= 0) {
        g.dw[(int64_t)c * g.lddw + g.dwcol[seg] + kk] = s;
    } else if (k < t.kbig + g.ns) {
        float *o = g.dw + (int64_t)c * g.lddw + g.dwcol_s + (k - t.kbig);
        const float v = g.sign_s * s;
        *o = g.accumulate_s ? *o + v : v;
    } else if (g.db) {
        g.db[c] = s;
    }
}

bool al16(const void *p) { return ((uintptr_t)p & 15) == 0; }

}  // namespace

extern "C" int mmpde_rgemm(const mmpde_rgemm_args *gp, mmpde_stream_t stream) {
    MMPDE_REQUIRE(gp);
    const mmpde_rgemm_args g = *gp;
    MMPDE_REQUIRE(g.m > 0 && g.kh >= 0 && g.m < ((int64_t)1 << 36));
    MMPDE_REQUIRE(g.parts == 1 || g.parts == 2);
    MMPDE_REQUIRE(g.layout == MMPDE_RGEMM_NT || g.layout == MMPDE_RGEMM_NN);
    bool xs = false;
    for (int p = 0; p < g.parts; ++p) {
        MMPDE_REQUIRE(g.out[p] && g.ncols[p] >= 1 && g.ncols[p] <= 128 && g.ldo[p] >= g.ncols[p]);
        MMPDE_REQUIRE(g.ns[p] >= 0 && g.ns[p] <= 4);
        MMPDE_REQUIRE(g.ns[p] == 0 || (g.xs && g.xw[p]));
        MMPDE_REQUIRE(!g.omask[p] || g.ldom[p] >= g.ncols[p]);
        xs = xs || g.ns[p] > 0;
    }
    MMPDE_REQUIRE(g.kh > 0 || xs);
    bool vec = g.kh % 4 == 0;
    if (g.kh > 0) {
        MMPDE_REQUIRE((g.amask[0] == nullptr) == (g.amask[1] == nullptr));
        for (int h = 0; h < 2; ++h) {
            MMPDE_REQUIRE(g.a[h] && g.w[h] && g.lda[h] >= g.kh);
            vec = vec && al16(g.a[h]) && g.lda[h] % 4 == 0 && (!g.amask[h] || al16(g.amask[h]));
            if (g.layout == MMPDE_RGEMM_NT) vec = vec && al16(g.w[h]) && g.ldw % 4 == 0;
        }
        for (int p = 0; p < g.parts; ++p)
            if (g.layout == MMPDE_RGEMM_NT) vec = vec && g.wk[p] % 4 == 0;
    }
    const dim3 grid((unsigned)ceil_div(g.m, RG_TILE), (unsigned)g.parts);
    const bool am = g.kh > 0 && g.amask[0] != nullptr;
    hipStream_t st = as_stream(stream);
#define RG_LAUNCH(L, V, A, X) hipLaunchKernelGGL((rgemm_kernel<L, V, A, X>), grid, dim3(256), 0, st, g)
    if (g.layout == MMPDE_RGEMM_NT) {
        if (vec) {
            if (am && xs) RG_LAUNCH(MMPDE_RGEMM_NT, true, true, true);
            else if (am) RG_LAUNCH(MMPDE_RGEMM_NT, true, true, false);
            else if (xs) RG_LAUNCH(MMPDE_RGEMM_NT, true, false, true);
            else RG_LAUNCH(MMPDE_RGEMM_NT, true, false, false);
        } else {
            if (am && xs) RG_LAUNCH(MMPDE_RGEMM_NT, false, true, true);
            else if (am) RG_LAUNCH(MMPDE_RGEMM_NT, false, true, false);
            else if (xs) RG_LAUNCH(MMPDE_RGEMM_NT, false, false, true);
            else RG_LAUNCH(MMPDE_RGEMM_NT, false, false, false);
        }
    } else {
        if (vec) {
            if (am && xs) RG_LAUNCH(MMPDE_RGEMM_NN, true, true, true);
            else if (am) RG_LAUNCH(MMPDE_RGEMM_NN, true, true, false);
            else if (xs) RG_LAUNCH(MMPDE_RGEMM_NN, true, false, true);
            else RG_LAUNCH(MMPDE_RGEMM_NN, true, false, false);
        } else {
            if (am && xs) RG_LAUNCH(MMPDE_RGEMM_NN, false, true, true);
            else if (am) RG_LAUNCH(MMPDE_RGEMM_NN, false, true, false);
            else if (xs) RG_LAUNCH(MMPDE_RGEMM_NN, false, false, true);
            else RG_LAUNCH(MMPDE_RGEMM_NN, false, false, false);
        }
    }
#undef RG_LAUNCH
    MMPDE_RET_LAUNCH();
    return MMPDE_OK;
}

extern "C" int64_t mmpde_rgemm_tn_workspace_bytes(int64_t m, int chunk_rows, int cols) {
    if (m <= 0 || chunk_rows <= 0 || cols <= 0) return 0;
    return ceil_div(m, chunk_rows) * 128 * (int64_t)cols * 4;
}

extern "C" int mmpde_rgemm_tn(const mmpde_rgemm_tn_args *gp, void *workspace, int64_t workspace_bytes,
                              mmpde_stream_t stream) {
    MMPDE_REQUIRE(gp && workspace);
    const mmpde_rgemm_tn_args &g = *gp;
    MMPDE_REQUIRE(g.m > 0 && g.chunk_rows > 0 && g.chunk_rows % 2 == 0 && g.g && g.dw);
    MMPDE_REQUIRE(g.gcols >= 1 && g.gcols <= 128 && g.ldg >= g.gcols);
    MMPDE_REQUIRE(g.nseg >= 1 && g.nseg <= 3 && g.ns >= 0 && g.ns <= 4 && (g.ns == 0 || g.xs));
    TnArgs t{};
    t.g = g;
    int kbig = 0;
    for (int s = 0; s < g.nseg; ++s) {
        MMPDE_REQUIRE(g.x[s] && g.kx[s] > 0 && g.ldx[s] >= g.kx[s]);
        t.base[s] = kbig;
        kbig += (g.kx[s] + RG_TILE - 1) / RG_TILE * RG_TILE;
    }
    t.kbig = kbig;
    t.cols = kbig + g.ns + 1;
    t.part = (float *)workspace;
    const int64_t chunks = ceil_div(g.m, g.chunk_rows);
    MMPDE_REQUIRE(workspace_bytes >= mmpde_rgemm_tn_workspace_bytes(g.m, g.chunk_rows, t.cols));
    MMPDE_REQUIRE(chunks < 65536);
    hipStream_t st = as_stream(stream);
    const dim3 grid((unsigned)(kbig / RG_TILE), (unsigned)chunks);
    if (g.gmask) hipLaunchKernelGGL((rgemm_tn_partial_kernel<true>), grid, dim3(256), 0, st, t);
    else hipLaunchKernelGGL((rgemm_tn_partial_kernel<false>), grid, dim3(256), 0, st, t);
    MMPDE_RET_LAUNCH();
    const int64_t outs = (int64_t)g.gcols * t.cols;
    hipLaunchKernelGGL(rgemm_tn_reduce_kernel, dim3((unsigned)ceil_div(outs, 256)), dim3(256), 0, st, t,
                       (int)chunks);
    MMPDE_RET_LAUNCH();
    return MMPDE_OK;
}
