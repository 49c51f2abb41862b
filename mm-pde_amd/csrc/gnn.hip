// MP_PDE_Solver_2D forward on gfx950 (reference gnn_2d.py:19-141).
//
// Layout: node features are [n, 128] fp32 rows (512 B), trajectory-major.
// Per message-passing layer (gnn_2d.py:53-69) we run
//   1. node_gemm<EpiProj>  : a = W1[:, :128] h + (w_du u + w_dx x + w_dy y + w_t t + b1)
//                            b = W1[:,128:256] h - (w_du u + w_dx x + w_dy y)
//      -- message_net_1 factored exactly into a target half and a source half
//         (its 260-wide input is cat(h_i, h_j, u_i-u_j, x_i-x_j, y_i-y_j, t_i));
//   2. edge_mean_kernel    : mean_i = (1/k) sum_e relu(W2 relu(a_i + b_{nbr(i,e)}) + b2)
//      -- the only per-edge work left: one 128x128 fp32 MFMA GEMM per edge,
//         never materialised in HBM (PyG gather + scatter-mean replaced);
//   3. node_gemm<EpiUpd1>  : v = relu(U1[:, :128] h + U1[:,128:256] mean + u1_t t + c1)
//   4. node_gemm<EpiUpd2>  : h' = BN(h + relu(U2 v + c2))
// All GEMMs use v_mfma_f32_32x32x2_f32 (exact fp32 products, fp32 accumulate).
#include <vector>

#include "common.hpp"
#include "f16x3.hpp"
#include "gemm.hpp"
#include "layer.hpp"

namespace {

constexpr int H = 128;  // hidden width (gnn_2d.py:77)
// [n, H] fp32 buffers of the forward workspace: h ping-pong, a, b, and 4 for the
// edge stage's mean parts (the first doubles as the mean)
constexpr int kGnnBufs = 8;

// ---------------------------------------------------------------------------
// Embedding first half: z = relu(BN1(W0 [u, x/Lx, y/Ly, t/tmax] + b0)), one thread
// per (node, channel).  gnn_2d.py:99-102,122-131.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void embed0_kernel(const float *__restrict__ u,
                                                     const float *__restrict__ pos, int64_t n,
                                                     mmpde_gnn_scales sc,
                                                     mmpde_gnn_embed_params p,
                                                     float *__restrict__ z) {
    const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (e >= n * H) return;
    const int64_t i = e >> 7;
    const int c = (int)(e & (H - 1));
    const float in0 = u[i];
    const float in1 = node_x(sc, pos, i) * sc.inv_lx;
    const float in2 = node_y(sc, pos, i) * sc.inv_ly;
    const float in3 = node_t(sc, pos, i) * sc.inv_tmax;
    const float *w = p.w0 + c * 4;
    float v = p.b0[c] + w[0] * in0 + w[1] * in1 + w[2] * in2 + w[3] * in3;
    v = bn_eval(v, p.bn1_rm[c], p.bn1_rv[c], p.bn1_w[c], p.bn1_b[c], p.eps);
    z[e] = fmaxf(v, 0.0f);
}

struct EpiProj {  // message_net_1 split (see header comment)
    float *out_a, *out_b;
    const float *b1, *w_du, *w_dx, *w_dy, *w_t;  // bias and columns 256..259 of W1
    int64_t ldw1;
    const float *u, *pos;
    mmpde_gnn_scales sc;
    __device__ void operator()(const f32x16 &acc, int64_t row0, int col0, int lane, int64_t m,
                               int part) const {
        const int c = col0 + (lane & 31);
        const float wdu = w_du[c * ldw1], wdx = w_dx[c * ldw1], wdy = w_dy[c * ldw1];
        const float wt = w_t[c * ldw1], bb = b1[c];
        float *dst = part == 0 ? out_a : out_b;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int64_t row = row0 + acc_row(r, lane);
            if (row < m) {
                const float uu = u[row];
                const float px = node_x(sc, pos, row) * sc.inv_lx;
                const float py = node_y(sc, pos, row) * sc.inv_ly;
                const float node = wdu * uu + wdx * px + wdy * py;
                float v;
                if (part == 0) {
                    const float pt = node_t(sc, pos, row) * sc.inv_tmax;
                    v = acc[r] + node + wt * pt + bb;
                } else {
                    v = acc[r] - node;
                }
                dst[row * H + c] = v;
            }
        }
    }
};

struct EpiUpd1 {  // relu(U1 [h | mean | t] + c1), gnn_2d.py:67
    float *out;
    const float *c1, *w_t;  // w_t: column 256 of U1 (stride ldw1)
    int64_t ldw1;
    const float *pos;
    mmpde_gnn_scales sc;
    __device__ void operator()(const f32x16 &acc, int64_t row0, int col0, int lane, int64_t m,
                               int) const {
        const int c = col0 + (lane & 31);
        const float wt = w_t[c * ldw1], bb = c1[c];
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int64_t row = row0 + acc_row(r, lane);
            if (row < m) {
                const float pt = node_t(sc, pos, row) * sc.inv_tmax;
                out[row * H + c] = fmaxf(acc[r] + wt * pt + bb, 0.0f);
            }
        }
    }
};

struct EpiUpd2 {  // BN(h + relu(U2 v + c2)), gnn_2d.py:68-69,56
    float *out;
    const float *c2, *h;
    const float *bn_w, *bn_b, *bn_rm, *bn_rv;
    float eps;
    __device__ void operator()(const f32x16 &acc, int64_t row0, int col0, int lane, int64_t m,
                               int) const {
        const int c = col0 + (lane & 31);
        const float bb = c2[c], rm = bn_rm[c], rv = bn_rv[c], g = bn_w[c], be = bn_b[c];
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int64_t row = row0 + acc_row(r, lane);
            if (row < m) {
                const float x = h[row * H + c] + fmaxf(acc[r] + bb, 0.0f);
                out[row * H + c] = bn_eval(x, rm, rv, g, be, eps);
            }
        }
    }
};

struct EpiBiasBn {  // BN(W x + b): embedding_mlp.3/.4
    float *out;
    const float *b;
    const float *bn_w, *bn_b, *bn_rm, *bn_rv;
    float eps;
    __device__ void operator()(const f32x16 &acc, int64_t row0, int col0, int lane, int64_t m,
                               int) const {
        const int c = col0 + (lane & 31);
        const float bb = b[c], rm = bn_rm[c], rv = bn_rv[c], g = bn_w[c], be = bn_b[c];
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int64_t row = row0 + acc_row(r, lane);
            if (row < m) out[row * H + c] = bn_eval(acc[r] + bb, rm, rv, g, be, eps);
        }
    }
};

// ---------------------------------------------------------------------------
// Edge stage: the hot loop.  One workgroup = 32 target nodes, 4 waves; wave w
// takes neighbour slots e = w, w+4, ...  For slot e the 32x128 tile
// M1[r, :] = relu(a[tgt r] + b[nbr(tgt r, e)]) is built in registers (lane
// (r, half) owns hidden units 64*half .. 64*half+63 of row r), multiplied by
// W2^T (64 KB, staged once in LDS as the exact per-lane MFMA operand image) into
// four 32x32 accumulators initialised with b2, then relu'd and summed into
// per-wave running sums S.  Because slot e of all 32 targets shares one
// accumulator row, the per-target sum needs no cross-lane traffic.  The 4
// waves' S are reduced through the (then free) LDS image; / k gives the mean.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256, 2) void edge_mean_kernel(const float *__restrict__ a,
                                                           const float *__restrict__ b,
                                                           const int32_t *__restrict__ nbr,
                                                           int64_t n, int k,
                                                           const float *__restrict__ w2,
                                                           const float *__restrict__ b2,
                                                           float *__restrict__ out) {
    __shared__ float4 ws[4 * 16 * 64];  // [ctile][s4][lane] : 64 KB
    for (int e = threadIdx.x; e < 4 * 16 * 64; e += 256) {
        const int l = e & 63, s4 = (e >> 6) & 15, c = e >> 10;
        ws[e] = *(const float4 *)(w2 + (32 * c + (l & 31)) * H + 64 * (l >> 5) + 4 * s4);
    }
    __syncthreads();

    const int wave = threadIdx.x >> 6;
    const int lane = threadIdx.x & 63;
    const int half = lane >> 5;
    const int64_t tile0 = (int64_t)blockIdx.x * 32;
    int64_t tgt = tile0 + (lane & 31);
    if (tgt >= n) tgt = n - 1;
    const float *arow = a + tgt * H + 64 * half;
    const int32_t *nrow = nbr + tgt * k;

    float bias[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) bias[c] = b2[32 * c + (lane & 31)];

    f32x16 S[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) S[c] = (f32x16){0};

    for (int e = wave; e < k; e += 4) {
        // clamp: a malformed caller table must not fault the GPU (knn output is always valid)
        const int64_t src = min((uint32_t)nrow[e], (uint32_t)(n - 1));
        const float *brow = b + src * H + 64 * half;
        f32x16 acc[4];
#pragma unroll
        for (int c = 0; c < 4; ++c) {
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[c][r] = bias[c];
        }
#pragma unroll 2
        for (int s4 = 0; s4 < 16; ++s4) {
            const float4 av = *(const float4 *)(arow + 4 * s4);
            const float4 bv = *(const float4 *)(brow + 4 * s4);
            const float m0 = fmaxf(av.x + bv.x, 0.0f);
            const float m1 = fmaxf(av.y + bv.y, 0.0f);
            const float m2 = fmaxf(av.z + bv.z, 0.0f);
            const float m3 = fmaxf(av.w + bv.w, 0.0f);
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                const float4 w = ws[(c * 16 + s4) * 64 + lane];
                acc[c] = mfma32(m0, w.x, acc[c]);
                acc[c] = mfma32(m1, w.y, acc[c]);
                acc[c] = mfma32(m2, w.z, acc[c]);
                acc[c] = mfma32(m3, w.w, acc[c]);
            }
        }
#pragma unroll
        for (int c = 0; c < 4; ++c) {
#pragma unroll
            for (int r = 0; r < 16; ++r) S[c][r] += fmaxf(acc[c][r], 0.0f);
        }
    }

    // cross-wave reduction through the LDS image (now free): red[wave][c][r][lane]
    __syncthreads();
    float *red = (float *)ws;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
#pragma unroll
        for (int r = 0; r < 16; ++r) red[((wave * 4 + c) * 16 + r) * 64 + lane] = S[c][r];
    }
    __syncthreads();
    const int c = wave;  // each wave finalises one 32-column tile
    const float inv_cnt_div = (float)k;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        float v = 0.0f;
#pragma unroll
        for (int w = 0; w < 4; ++w) v += red[((w * 4 + c) * 16 + r) * 64 + lane];
        const int64_t row = tile0 + acc_row(r, lane);
        if (row < n) out[row * H + 32 * c + (lane & 31)] = v / inv_cnt_div;
    }
}

// ---------------------------------------------------------------------------
// Conv1d head (gnn_2d.py:108-114,136-139):
// 128 -> conv(1->4, k16, s3) 38 -> relu -> conv(4->8, k12, s3) 9 -> relu ->
// conv(8->1, k8, s2) 1, times out_scale.
// 64 nodes per 256-thread workgroup, one node per lane: the 64 h rows are
// staged in LDS (row stride 129: a wave reading one column of 64 rows hits 64
// distinct banks); wave c computes conv0 channel c (38 outputs, kept in
// registers until every wave has read h, then written over the h rows), then
// conv2 channels 2c, 2c+1 (9 outputs each) from all four conv0 channels, then
// its share of conv4; the four partial sums meet in LDS.  Weights are
// wave-uniform (scalar loads).  39 KB of LDS: several workgroups per CU.
// ---------------------------------------------------------------------------
constexpr int HN = 64;           // nodes per workgroup
constexpr int HS = H + 1;        // h row stride (floats)
constexpr int Y1S = 4 * 38 + 1;  // conv0 output row stride (floats)

// One or two problems per launch: blocks below blocks0 take problem 0's
// nodes, the rest problem 1's.
struct HeadArgs2 {
    const float *h[2];
    int64_t n[2];
    mmpde_gnn_head_params p[2];
    float *out[2];
    int64_t blocks0;
};

__global__ __launch_bounds__(256) void head_kernel(HeadArgs2 hp) {
    const bool second = (int64_t)blockIdx.x >= hp.blocks0;  // workgroup-uniform
    const float *__restrict__ h = hp.h[second ? 1 : 0];
    const int64_t n = hp.n[second ? 1 : 0];
    const mmpde_gnn_head_params &p = hp.p[second ? 1 : 0];
    float *__restrict__ out = hp.out[second ? 1 : 0];
    const int64_t bid = (int64_t)blockIdx.x - (second ? hp.blocks0 : 0);
    __shared__ float sh[HN * (Y1S > HS ? Y1S : HS)];  // h rows (stride HS), then conv0 outputs (stride Y1S)
    __shared__ float spart[4][HN];
    float *const sy1 = sh;
    const int tid = threadIdx.x, lane = tid & 63;
    const int c = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int64_t node0 = bid * HN;
    for (int i = tid; i < HN * (H / 4); i += 256) {
        const int row = i >> 5, c4 = i & 31;
        const int64_t src = min(node0 + row, n - 1);
        const float4 v = *(const float4 *)(h + src * H + 4 * c4);
        float *d = sh + row * HS + 4 * c4;
        d[0] = v.x;
        d[1] = v.y;
        d[2] = v.z;
        d[3] = v.w;
    }
    __syncthreads();
    {   // conv0, channel c
        float w[16], y[38];
#pragma unroll
        for (int t = 0; t < 16; ++t) w[t] = p.c0_w[c * 16 + t];
        const float b = p.c0_b[c];
        const float *hr = sh + lane * HS;
#pragma unroll
        for (int q0 = 0; q0 < 38; q0 += 2) {
            float x[19];
#pragma unroll
            for (int i = 0; i < 19; ++i) x[i] = hr[3 * q0 + i];
#pragma unroll
            for (int qq = 0; qq < 2; ++qq) {
                float v = b;
#pragma unroll
                for (int t = 0; t < 16; ++t) v = fmaf(w[t], x[3 * qq + t], v);
                y[q0 + qq] = fmaxf(v, 0.0f);
            }
        }
        __syncthreads();  // every wave has read the h rows
        float *yr = sy1 + lane * Y1S + c * 38;
#pragma unroll
        for (int q = 0; q < 38; ++q) yr[q] = y[q];
    }
    __syncthreads();
    float part = 0.0f;
#pragma unroll
    for (int oo = 0; oo < 2; ++oo) {  // conv2 channel co = 2c + oo, then its conv4 terms
        const int co = 2 * c + oo;
        float acc[9];
        const float b = p.c2_b[co];
#pragma unroll
        for (int q = 0; q < 9; ++q) acc[q] = b;
#pragma unroll
        for (int ci = 0; ci < 4; ++ci) {
            float y[36];
            const float *yr = sy1 + lane * Y1S + ci * 38;
#pragma unroll
            for (int i = 0; i < 36; ++i) y[i] = yr[i];
            float w[12];
#pragma unroll
            for (int t = 0; t < 12; ++t) w[t] = p.c2_w[(co * 4 + ci) * 12 + t];
#pragma unroll
            for (int q = 0; q < 9; ++q) {
#pragma unroll
                for (int t = 0; t < 12; ++t) acc[q] = fmaf(w[t], y[3 * q + t], acc[q]);
            }
        }
#pragma unroll
        for (int t = 0; t < 8; ++t) part = fmaf(p.c4_w[co * 8 + t], fmaxf(acc[t], 0.0f), part);
    }
    spart[c][lane] = part;
    __syncthreads();
    if (c == 0 && node0 + lane < n) {
        const float diff = p.c4_b[0] + ((spart[0][lane] + spart[1][lane]) +
                                        (spart[2][lane] + spart[3][lane]));
        if (p.tw <= 1) {
            out[node0 + lane] = p.out_scale * diff;
        } else {  // out [n, tw] = cumsum(dt) * diff (gnn_2d.py:137-141)
            for (int t = 0; t < p.tw; ++t) out[(node0 + lane) * p.tw + t] = p.out_scales[t] * diff;
        }
    }
}

inline bool aligned16(const void *p) { return ((uintptr_t)p & 15u) == 0; }

}  // namespace

// ===========================================================================
// C-ABI
// ===========================================================================
extern "C" int64_t mmpde_gnn_workspace_bytes(int64_t n) {
    // h ping-pong, a, b, the edge stage's sums and 3 x [n,128] for the wave edge
    // kernel's side blocks = 8 x [n,128] fp32 (the unfused per-layer API uses 4
    // of them as a, b, mean, v), then the F16X3 row maxima (layer.hpp) and
    // room for per-call weight images
    return kGnnBufs * n * H * (int64_t)sizeof(float) + row_records_floats(n) * 4 +
           (int64_t)MMPDE_GNN_MAX_LAYERS * kLayerPack;
}

extern "C" int mmpde_gnn_embed(const float *u, const float *pos, int64_t n,
                               mmpde_gnn_scales sc, const mmpde_gnn_embed_params *p,
                               float *workspace, float *h_out, mmpde_stream_t stream) {
    MMPDE_REQUIRE(u && pos && p && workspace && h_out && n > 0);
    MMPDE_REQUIRE(sc.tw <= 1);  // the per-stage entry points take one u channel
    hipStream_t st = as_stream(stream);
    hipLaunchKernelGGL(embed0_kernel, dim3(ceil_div(n * H, 256)), dim3(256), 0, st, u, pos, n,
                       sc, *p, workspace);
    MMPDE_RET_LAUNCH();
    GemmArgs g{n, workspace, workspace + 64, H, p->w3, p->w3 + 64, H, 64};
    EpiBiasBn epi{h_out, p->b3, p->bn4_w, p->bn4_b, p->bn4_rm, p->bn4_rv, p->eps};
    return launch_gemm(g, 1, epi, st);
}

extern "C" int mmpde_gnn_edge_mean(const float *a, const float *b, const int32_t *nbr,
                                   int64_t n, int k, const float *msg2_w, const float *msg2_b,
                                   float *mean_out, mmpde_stream_t stream) {
    MMPDE_REQUIRE(a && b && nbr && msg2_w && msg2_b && mean_out && n > 0 && k > 0);
    MMPDE_REQUIRE(aligned16(a) && aligned16(b) && aligned16(msg2_w));
    hipLaunchKernelGGL(edge_mean_kernel, dim3(ceil_div(n, 32)), dim3(256), 0, as_stream(stream),
                       a, b, nbr, n, k, msg2_w, msg2_b, mean_out);
    MMPDE_RET_LAUNCH();
    return MMPDE_OK;
}

extern "C" int mmpde_gnn_edge_mean_deg(const float *a, const float *b, const int32_t *nbr, const int32_t *deg,
                                       int64_t n, int k, const float *msg2_w, const float *msg2_b,
                                       float *mean_out, mmpde_stream_t stream) {
    MMPDE_REQUIRE(a && b && nbr && msg2_w && msg2_b && mean_out && n > 0 && k > 0);
    mmpde_gnn_layer_params p{};
    p.msg2_w = msg2_w;
    p.msg2_b = msg2_b;
    // exact fp32 ring kernel (no pack): the training forward of gnn_2d.py:53-63
    return launch_edge_stage(a, b, nbr, deg, n, k, n, &p, nullptr, nullptr, mean_out, nullptr, 0, nullptr,
                             as_stream(stream));
}

extern "C" int64_t mmpde_gnn_edge_mean_workspace_bytes(int64_t n, int edge_gemm) {
    return n > 0 && edge_gemm == MMPDE_EDGE_GEMM_F16X3 ? edge_mean_f16x3_ws_bytes(n) : 0;
}

extern "C" int mmpde_gnn_edge_mean_ex(const float *a, const float *b, const int32_t *nbr, const int32_t *deg,
                                      int64_t n, int k, const float *msg2_w, const float *msg2_b, float *mean_out,
                                      uint32_t *relu_mask, int edge_gemm, void *workspace, int64_t workspace_bytes,
                                      mmpde_stream_t stream) {
    MMPDE_REQUIRE(edge_gemm == MMPDE_EDGE_GEMM_F32 || edge_gemm == MMPDE_EDGE_GEMM_F16X3);
    MMPDE_REQUIRE(!relu_mask || (n * k < (int64_t)INT32_MAX && ((uintptr_t)relu_mask & 15) == 0));
    if (edge_gemm == MMPDE_EDGE_GEMM_F32) {
        if (!relu_mask) return mmpde_gnn_edge_mean_deg(a, b, nbr, deg, n, k, msg2_w, msg2_b, mean_out, stream);
        MMPDE_REQUIRE(a && b && nbr && msg2_w && msg2_b && mean_out && n > 0 && k > 0);
        mmpde_gnn_layer_params p{};
        p.msg2_w = msg2_w;
        p.msg2_b = msg2_b;
        return launch_edge_stage(a, b, nbr, deg, n, k, n, &p, nullptr, nullptr, mean_out, nullptr, 0, nullptr,
                                 as_stream(stream), relu_mask);
    }
    MMPDE_REQUIRE(n > 0 && workspace && workspace_bytes >= edge_mean_f16x3_ws_bytes(n));
    return launch_edge_mean_f16x3(a, b, nbr, deg, n, k, msg2_w, msg2_b, mean_out, relu_mask, workspace,
                                  as_stream(stream));
}

static int gnn_layer_impl(const float *h_in, const float *u, const float *pos, int64_t n, int k,
                          const int32_t *nbr, mmpde_gnn_scales sc,
                          const mmpde_gnn_layer_params *p, float *workspace, float *h_out,
                          hipEvent_t ev_begin, hipEvent_t ev_end, mmpde_stream_t stream) {
    MMPDE_REQUIRE(h_in && u && pos && nbr && p && workspace && h_out && n > 0 && k > 0);
    MMPDE_REQUIRE(h_in != h_out && aligned16(h_in) && aligned16(workspace));
    MMPDE_REQUIRE(p->msg1_ld >= 260 && (p->msg1_ld & 3) == 0 && aligned16(p->msg1_w));
    MMPDE_REQUIRE(p->upd1_ld >= 257 && (p->upd1_ld & 3) == 0 && aligned16(p->upd1_w));
    MMPDE_REQUIRE(aligned16(p->upd2_w));
    hipStream_t st = as_stream(stream);
    float *wa = workspace;
    float *wb = wa + n * H;
    float *wm = wb + n * H;
    float *wv = wm + n * H;
    int rc;
    // 1. message_net_1 split into per-node target / source halves (W1 row stride 260)
    {
        const int64_t ld = p->msg1_ld;
        GemmArgs g{n, h_in, h_in + 64, H, p->msg1_w, p->msg1_w + 64, ld, 64};
        EpiProj epi{wa, wb, p->msg1_b, p->msg1_w + 256, p->msg1_w + 257, p->msg1_w + 258,
                    p->msg1_w + 259, ld, u, pos, sc};
        rc = launch_gemm<EpiProj, true>(g, 2, epi, st);
        if (rc) return rc;
    }
    // 2. per-edge message_net_2 + mean aggregation
    if (ev_begin && hipEventRecord(ev_begin, st) != hipSuccess) return MMPDE_ERR_INVALID_ARG;
    rc = mmpde_gnn_edge_mean(wa, wb, nbr, n, k, p->msg2_w, p->msg2_b, wm, stream);
    if (rc) return rc;
    if (ev_end && hipEventRecord(ev_end, st) != hipSuccess) return MMPDE_ERR_INVALID_ARG;
    // 3. update_net_1 over cat(h, mean, t) (row stride upd1_ld, 16-B aligned rows)
    {
        const int64_t ld = p->upd1_ld;
        GemmArgs g{n, h_in, wm, H, p->upd1_w, p->upd1_w + 128, ld, 128};
        EpiUpd1 epi{wv, p->upd1_b, p->upd1_w + 256, ld, pos, sc};
        rc = launch_gemm(g, 1, epi, st);
        if (rc) return rc;
    }
    // 4. update_net_2 + residual + BatchNorm(eval)
    {
        GemmArgs g{n, wv, wv + 64, H, p->upd2_w, p->upd2_w + 64, H, 64};
        EpiUpd2 epi{h_out, p->upd2_b, h_in, p->bn_w, p->bn_b, p->bn_rm, p->bn_rv, p->eps};
        rc = launch_gemm(g, 1, epi, st);
    }
    return rc;
}

extern "C" int mmpde_gnn_layer(const float *h_in, const float *u, const float *pos, int64_t n,
                               int k, const int32_t *nbr, mmpde_gnn_scales sc,
                               const mmpde_gnn_layer_params *p, float *workspace,
                               float *h_out, mmpde_stream_t stream) {
    MMPDE_REQUIRE(sc.tw <= 1);  // the per-stage entry points take one u channel
    return gnn_layer_impl(h_in, u, pos, n, k, nbr, sc, p, workspace, h_out, nullptr, nullptr,
                          stream);
}

// The Conv1d head of one or two problems in one launch.
static int head_launch(const float *const *h, const int64_t *n, const mmpde_gnn_head_params *const *p,
                       float *const *out, int count, hipStream_t st) {
    HeadArgs2 hp;
    int64_t blocks = 0;
    for (int i = 0; i < count; ++i) {
        MMPDE_REQUIRE(h[i] && p[i] && out[i] && n[i] > 0 && p[i]->tw <= 16 && (p[i]->tw <= 1 || p[i]->out_scales));
        hp.h[i] = h[i];
        hp.n[i] = n[i];
        hp.p[i] = *p[i];
        hp.out[i] = out[i];
        if (i == 0) hp.blocks0 = ceil_div(n[0], HN);
        blocks += ceil_div(n[i], HN);
    }
    if (count == 1) {
        hp.h[1] = hp.h[0];
        hp.n[1] = hp.n[0];
        hp.p[1] = hp.p[0];
        hp.out[1] = hp.out[0];
    }
    MMPDE_REQUIRE(blocks < (int64_t)INT32_MAX);
    hipLaunchKernelGGL(head_kernel, dim3((unsigned)blocks), dim3(256), 0, st, hp);
    MMPDE_RET_LAUNCH();
    return MMPDE_OK;
}

extern "C" int mmpde_gnn_head(const float *h, int64_t n, const mmpde_gnn_head_params *p,
                              float *out, mmpde_stream_t stream) {
    MMPDE_REQUIRE(p);
    return head_launch(&h, &n, &p, &out, 1, as_stream(stream));
}

extern "C" int64_t mmpde_gnn_pack_bytes(int n_layers) {
    return n_layers < 0 ? 0 : (int64_t)n_layers * kLayerPack;
}

extern "C" int mmpde_gnn_pack_f16x3(const mmpde_gnn_layer_params *layers, int n_layers,
                                    void *pack, mmpde_stream_t stream) {
    MMPDE_REQUIRE(layers && pack && n_layers > 0 && n_layers <= MMPDE_GNN_MAX_LAYERS);
    MMPDE_REQUIRE(aligned16(pack));
    hipStream_t st = as_stream(stream);
    PackSrc w2{}, u1{}, u2{}, w1{};
    for (int l = 0; l < n_layers; ++l) {
        const mmpde_gnn_layer_params &q = layers[l];
        MMPDE_REQUIRE(q.msg1_w && q.msg2_w && q.upd1_w && q.upd2_w);
        MMPDE_REQUIRE(q.msg1_ld >= 260 && q.upd1_ld >= 257);
        w2.w[l] = q.msg2_w;
        w2.ld[l] = H;
        u1.w[l] = q.upd1_w;
        u1.ld[l] = q.upd1_ld;
        u2.w[l] = q.upd2_w;
        u2.ld[l] = H;
        w1.w[l] = q.msg1_w;
        w1.ld[l] = q.msg1_ld;
    }
    char *pk = (char *)pack;
    hipLaunchKernelGGL(pack_f16x3_kernel<128>, dim3(128, n_layers), dim3(128), 0, st, w2, 0, kPkW2, (int64_t)128, pk);
    hipLaunchKernelGGL(pack_f16x3_kernel<256>, dim3(128, n_layers), dim3(256), 0, st, u1, 0, kPkU1, (int64_t)128, pk);
    hipLaunchKernelGGL(pack_f16x3_kernel<128>, dim3(128, n_layers), dim3(128), 0, st, u2, 0, kPkU2, (int64_t)128, pk);
    hipLaunchKernelGGL(pack_f16x3_kernel<128>, dim3(256, n_layers), dim3(128), 0, st, w1, 1, kPkW1, (int64_t)256, pk);
    MMPDE_RET_LAUNCH();
    return MMPDE_OK;
}

extern "C" int mmpde_gnn_forward_ex(const float *u, const float *pos, int64_t n, int k,
                                    const int32_t *nbr, mmpde_gnn_scales sc,
                                    const mmpde_gnn_embed_params *emb,
                                    const mmpde_gnn_layer_params *layers, int n_layers,
                                    const mmpde_gnn_head_params *head, void *workspace,
                                    float *out, const mmpde_gnn_exec *exec,
                                    mmpde_stream_t stream) {
    MMPDE_REQUIRE(u && pos && nbr && emb && layers && head && workspace && out);
    MMPDE_REQUIRE(n > 0 && k > 0 && n_layers >= 0 && n_layers <= MMPDE_GNN_MAX_LAYERS);
    MMPDE_REQUIRE(aligned16(workspace));
    const int tw = sc.tw > 1 ? sc.tw : 1;
    MMPDE_REQUIRE(tw <= 16 && (head->tw > 1 ? head->tw : 1) == tw && (n_layers > 0 || tw == 1));
    for (int l = 0; l < n_layers; ++l) MMPDE_REQUIRE(layers[l].msg1_ld >= 259 + tw);
    const int mode = exec ? exec->edge_gemm : MMPDE_EDGE_GEMM_F32;
    MMPDE_REQUIRE(mode == MMPDE_EDGE_GEMM_F32 || mode == MMPDE_EDGE_GEMM_F16X3);
    hipStream_t st = as_stream(stream);
    float *ws = (float *)workspace;
    float *hb[2] = {ws, ws + n * H};
    float *wa = ws + 2 * n * H, *wb = ws + 3 * n * H, *wmean = ws + 4 * n * H;
    const char *pack = nullptr;
    // row maxima and range records of the current layer's message inputs
    // (F16X3 split scales):
    // written by the embed / node stage, read by the next edge stage
    float *rmx = ws + kGnnBufs * n * H;
    // rows per trajectory segment (the edge stage's summation units)
    const int64_t seg_n = exec ? exec->seg_n : 0;
    int rc;
    if (mode == MMPDE_EDGE_GEMM_F16X3 && n_layers > 0) {
        if (exec->packed) {
            MMPDE_REQUIRE(aligned16(exec->packed));
            pack = (const char *)exec->packed;
        } else {
            char *wpk = (char *)(ws + kGnnBufs * n * H + row_records_floats(n));
            rc = mmpde_gnn_pack_f16x3(layers, n_layers, wpk, stream);
            if (rc) return rc;
            pack = wpk;
        }
    }
    if (n_layers > 0) {
        // embedding + layer 0's message_net_1 halves (later layers get theirs
        // from the previous layer's node stage)
        rc = launch_embed_stage(u, pos, n, seg_n, sc, emb, &layers[0], pack, pack ? rmx : nullptr, hb[0],
                                wa, wb, st);
    } else {
        rc = mmpde_gnn_embed(u, pos, n, sc, emb, wmean, hb[0], stream);  // wmean: scratch
    }
    if (rc) return rc;
    int cur = 0;
    for (int l = 0; l < n_layers; ++l) {
        hipEvent_t eb = exec && exec->edge_begin ? (hipEvent_t)exec->edge_begin[l] : nullptr;
        hipEvent_t ee = exec && exec->edge_end ? (hipEvent_t)exec->edge_end[l] : nullptr;
        hipEvent_t ne = exec && exec->node_end ? (hipEvent_t)exec->node_end[l] : nullptr;
        const mmpde_gnn_layer_params *next = l + 1 < n_layers ? &layers[l + 1] : nullptr;
        const char *pk = pack ? pack + (int64_t)l * kLayerPack : nullptr;
        const char *pkn = pack && next ? pack + (int64_t)(l + 1) * kLayerPack : nullptr;
        // one row-maxima buffer serves every layer: edge stage l reads it
        // before node stage l (stream order) writes layer l + 1's
        float *rout = pack && next ? rmx : nullptr;
        if (eb && hipEventRecord(eb, st) != hipSuccess) return MMPDE_ERR_INVALID_ARG;
        EdgeSplit split;
        const int32_t *deg = exec ? exec->degree : nullptr;
        // side blocks of the wave edge kernel: the workspace after the mean
        rc = launch_edge_stage(wa, wb, nbr, deg, n, k, seg_n, &layers[l], pk, pack ? rmx : nullptr, wmean,
                               wmean + n * H, (kGnnBufs - 5) * n * H / (16 * H), &split, st);
        if (rc) return rc;
        if (ee && hipEventRecord(ee, st) != hipSuccess) return MMPDE_ERR_INVALID_ARG;
        // a, b are rewritten in place: this layer's edge stage has consumed them
        rc = launch_node_stage(hb[cur], wmean, &split, deg, u, pos, n, seg_n, sc, &layers[l], next, pk, pkn,
                               rout, hb[cur ^ 1], wa, wb, st);
        if (rc) return rc;
        if (ne && hipEventRecord(ne, st) != hipSuccess) return MMPDE_ERR_INVALID_ARG;
        cur ^= 1;
    }
    return mmpde_gnn_head(hb[cur], n, head, out, stream);
}

extern "C" int mmpde_gnn_forward(const float *u, const float *pos, int64_t n, int k,
                                 const int32_t *nbr, mmpde_gnn_scales sc,
                                 const mmpde_gnn_embed_params *emb,
                                 const mmpde_gnn_layer_params *layers, int n_layers,
                                 const mmpde_gnn_head_params *head, void *workspace, float *out,
                                 mmpde_stream_t stream) {
    return mmpde_gnn_forward_ex(u, pos, n, k, nbr, sc, emb, layers, n_layers, head, workspace, out,
                                nullptr, stream);
}
