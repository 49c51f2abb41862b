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
#include "gemm.hpp"

namespace {

constexpr int H = 128;  // hidden width (gnn_2d.py:77)

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
    const float in1 = pos[i * 3 + 1] * sc.inv_lx;
    const float in2 = pos[i * 3 + 2] * sc.inv_ly;
    const float in3 = pos[i * 3 + 0] * sc.inv_tmax;
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
                const float px = pos[row * 3 + 1] * sc.inv_lx;
                const float py = pos[row * 3 + 2] * sc.inv_ly;
                const float node = wdu * uu + wdx * px + wdy * py;
                float v;
                if (part == 0) {
                    const float pt = pos[row * 3 + 0] * sc.inv_tmax;
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
    float inv_tmax;
    __device__ void operator()(const f32x16 &acc, int64_t row0, int col0, int lane, int64_t m,
                               int) const {
        const int c = col0 + (lane & 31);
        const float wt = w_t[c * ldw1], bb = c1[c];
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int64_t row = row0 + acc_row(r, lane);
            if (row < m) {
                const float pt = pos[row * 3 + 0] * inv_tmax;
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
// Fused message-passing layer (the rollout's hot kernel): one launch per layer
//   mean_i = (1/k) sum_e relu(W2 relu(a_i + b_nbr(i,e)) + b2)           edge stage
//   v_i    = relu(U1 [h_i | mean_i | t_i] + c1)                         update_net_1
//   h'_i   = BN(h_i + relu(U2 v_i + c2))                                update_net_2, BN
//   a'_i, b'_i = next layer's message_net_1 halves of h'_i (NEXT only)  (see EpiProj)
// (gnn_2d.py:53-69 twice over: this layer's update and the next layer's
// message_net_1, so a layer costs one launch and h, a, b cross HBM once.)
//
// Workgroup = 16 target rows x 4 waves, v_mfma_f32_16x16x4_f32 throughout.
// K index map for every 128-wide operand: lane l (row l&15, group g = l>>4)
// holds k = 16 j + 4 g + t in component t of its float4 number j (j < 8), so a
// row is read as 64-B contiguous pieces and MFMA step (j, t) consumes one float
// per lane.  Edge stage: wave w takes neighbour slots e = w, w+4, ...; W2 sits
// in LDS as the exact per-lane B image (64 KB, staged once per workgroup);
// a_i stays in registers; b rows of the next slot are prefetched while the
// current slot's 16x128x128 product runs.  Slot e of all 16 targets shares one
// accumulator row, so per-target sums need no cross-lane traffic; the four
// waves' partial sums meet in LDS (the then free W2 region), which also carries
// the transposes between the epilogue GEMMs.  Deterministic: no atomics.
// ---------------------------------------------------------------------------
constexpr int FT = 16;    // target rows per workgroup
constexpr int FRP = 132;  // padded LDS row (floats): conflict-free C-layout writes

struct FusedLayerArgs {
    const float *a, *b, *h;  // [n,128]: this layer's message_net_1 halves, layer input
    const int32_t *nbr;      // [n,k] global source rows
    int64_t n;
    int k;
    const float *w2, *b2;             // message_net_2.0 [128,128], [128]
    const char *w2pk;                 // F16X3: packed W2 image + column scales
    const float *u1, *c1;             // update_net_1.0 [128, ld_u1] (h | mean | t), [128]
    int64_t ld_u1;
    const float *u2, *c2;             // update_net_2.0 [128,128], [128]
    const float *bn_w, *bn_b, *bn_rm, *bn_rv;
    float eps;
    float *h_out;
    const float *w1n, *b1n;           // next layer message_net_1.0 [128, ld_w1n], [128]
    int64_t ld_w1n;
    float *a_out, *b_out;
    const float *u, *pos;             // node input u [n], pos [n,3] = (t, x, y)
    mmpde_gnn_scales sc;
};

__device__ __forceinline__ float4 relu4_add(float4 x, float4 y) {
    return make_float4(fmaxf(x.x + y.x, 0.0f), fmaxf(x.y + y.y, 0.0f), fmaxf(x.z + y.z, 0.0f),
                       fmaxf(x.w + y.w, 0.0f));
}

__device__ __forceinline__ float f4c(const float4 &v, int t) {
    return t == 0 ? v.x : t == 1 ? v.y : t == 2 ? v.z : v.w;
}

typedef _Float16 half8 __attribute__((ext_vector_type(8)));

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
    return v;
}

// Power of two s with mx * s in [2^13, 2^14) (fp16 max 65504): the scale of
// the F16X3 split.  mx zero / subnormal / inf / nan -> 1; clamped to
// [2^-40, 2^40] so a scaled bias can never overflow fp32.
__device__ __forceinline__ float split_scale(float mx) {
    const int eb = (int)((__float_as_uint(mx) >> 23) & 0xff);
    if (eb == 0 || eb == 255) return 1.0f;
    const int se = min(max(267 - eb, 127 - 40), 127 + 40);
    return __uint_as_float((uint32_t)se << 23);
}

// ---------------------------------------------------------------------------
// F16X3 weight image of message_net_2 (per layer, once per forward): column
// col is scaled by sw[col] = split_scale(max_k |W2[col, k]|) and split into
// fp16 hi + lo, laid out as the exact per-lane B operand of
// v_mfma_f32_16x16x32_f16: [ctile c][kstep s][hi|lo][lane][8 halves] with
// lane = 16 g + (col & 15) holding k = 32 s + 8 g + j.  Followed by sw[128].
// ---------------------------------------------------------------------------
constexpr int kW2PackBytes = 65536 + 512;

struct W2PackArgs {
    const float *w2[MMPDE_GNN_MAX_LAYERS];
};

__global__ __launch_bounds__(128) void w2_pack_f16x3_kernel(W2PackArgs a, char *__restrict__ pack) {
    __shared__ float red[2];
    const int layer = blockIdx.y, col = blockIdx.x, k = threadIdx.x;
    const float w = a.w2[layer][col * H + k];
    const float m = wave_max(fabsf(w));
    if ((k & 63) == 0) red[k >> 6] = m;
    __syncthreads();
    const float sw = split_scale(fmaxf(red[0], red[1]));
    const float x = w * sw;
    const _Float16 hi = (_Float16)x;
    const _Float16 lo = (_Float16)(x - (float)hi);
    const int c = col >> 4, s = k >> 5, g = (k >> 3) & 3, j = k & 7;
    const int lane = 16 * g + (col & 15);
    _Float16 *img = (_Float16 *)(pack + (int64_t)layer * kW2PackBytes);
    img[(((c * 4 + s) * 2 + 0) * 64 + lane) * 8 + j] = hi;
    img[(((c * 4 + s) * 2 + 1) * 64 + lane) * 8 + j] = lo;
    if (k == 0) ((float *)(pack + (int64_t)layer * kW2PackBytes + 65536))[col] = sw;
}

template <bool NEXT, bool F16X3>
__global__ __launch_bounds__(256, 2) void gnn_layer_fused_kernel(FusedLayerArgs p) {
    __shared__ float4 lds4[8 * 8 * 64 + FT * FRP / 4];  // W2 image (64 KB) | a tile
    float *lds = (float *)lds4;
    float *lds_a = lds + 8 * 8 * 64 * 4;  // [16][FRP]: a rows of the tile
    const int wave = threadIdx.x >> 6;
    const int lane = threadIdx.x & 63;
    const int r = lane & 15, g = lane >> 4;
    const int tile = xcd_tile(blockIdx.x, gridDim.x);
    const int64_t tile0 = (int64_t)tile * FT;
    const int64_t tgt = min(tile0 + r, p.n - 1);

    if (F16X3) {
        for (int e = threadIdx.x; e < 8 * 8 * 64; e += 256) lds4[e] = ((const float4 *)p.w2pk)[e];
    } else {
        for (int e = threadIdx.x; e < 8 * 8 * 64; e += 256) {
            const int l = e & 63, j = (e >> 6) & 7, c = e >> 9;
            lds4[e] = *(const float4 *)(p.w2 + (16 * c + (l & 15)) * H + 16 * j + 4 * (l >> 4));
        }
    }
    for (int e = threadIdx.x; e < FT * 32; e += 256) {
        const int row = e >> 5, c4 = e & 31;
        const int64_t src = min(tile0 + row, p.n - 1);
        *(float4 *)(lds_a + row * FRP + 4 * c4) = *(const float4 *)(p.a + src * H + 4 * c4);
    }

    float bias[8];
#pragma unroll
    for (int c = 0; c < 8; ++c) bias[c] = p.b2[16 * c + r];
    f32x4 S[8];
#pragma unroll
    for (int c = 0; c < 8; ++c) S[c] = (f32x4){0.0f, 0.0f, 0.0f, 0.0f};

    // Neighbour rows: slot e's b row is loaded one slot ahead, its index two
    // slots ahead, so neither latency sits in front of the MFMAs.
    // (clamped: a malformed caller table must not fault the GPU)
    // k map of the b / a pieces: F32 float4 j holds k = 16 j + 4 g + t;
    // F16X3 float4 i holds k = 32 (i >> 1) + 8 g + 4 (i & 1) + t.
    const int32_t *nrow = p.nbr + tgt * p.k;
    const uint32_t nmax = (uint32_t)(p.n - 1);
    auto piece = [&](int i) { return F16X3 ? 32 * (i >> 1) + 8 * g + 4 * (i & 1) : 16 * i + 4 * g; };
    float4 bv[8];
    uint32_t src_next = 0;
    if (wave < p.k) {
        const int64_t src = min((uint32_t)nrow[wave], nmax);
#pragma unroll
        for (int i = 0; i < 8; ++i) bv[i] = *(const float4 *)(p.b + src * H + piece(i));
        if (wave + 4 < p.k) src_next = (uint32_t)nrow[wave + 4];
    }
    float bsw[8], isw[8];  // F16X3: bias * column scale, 1 / column scale
    if (F16X3) {
        const float *swp = (const float *)(p.w2pk + 65536);
#pragma unroll
        for (int c = 0; c < 8; ++c) {
            const float sw = swp[16 * c + r];
            bsw[c] = bias[c] * sw;
            isw[c] = 1.0f / sw;
        }
    }
    __syncthreads();
    const float4 *wimg = lds4 + lane;
    const float *arow = lds_a + r * FRP;

    for (int e = wave; e < p.k; e += 4) {
        // keep the W2 image in LDS: without this the compiler hoists the
        // loop-invariant ds_reads out of the loop (256 VGPRs) and spills them
        asm volatile("" ::: "memory");
        float4 m[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) m[i] = relu4_add(*(const float4 *)(arow + piece(i)), bv[i]);
        if (e + 4 < p.k) {
            const int64_t src = min(src_next, nmax);
#pragma unroll
            for (int i = 0; i < 8; ++i) bv[i] = *(const float4 *)(p.b + src * H + piece(i));
            if (e + 8 < p.k) src_next = (uint32_t)nrow[e + 8];
        }
        f32x4 acc[8];
        if (!F16X3) {
#pragma unroll
            for (int c = 0; c < 8; ++c) acc[c] = (f32x4){bias[c], bias[c], bias[c], bias[c]};
            float4 w[8];
#pragma unroll
            for (int c = 0; c < 8; ++c) w[c] = wimg[c * 8 * 64];
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                float4 wn[8];
                if (j < 7) {
#pragma unroll
                    for (int c = 0; c < 8; ++c) wn[c] = wimg[(c * 8 + j + 1) * 64];
                }
#pragma unroll
                for (int t = 0; t < 4; ++t) {
#pragma unroll
                    for (int c = 0; c < 8; ++c) acc[c] = mfma16(f4c(m[j], t), f4c(w[c], t), acc[c]);
                }
                if (j < 7) {
#pragma unroll
                    for (int c = 0; c < 8; ++c) w[c] = wn[c];
                }
            }
#pragma unroll
            for (int c = 0; c < 8; ++c) {
#pragma unroll
                for (int q = 0; q < 4; ++q) S[c][q] += fmaxf(acc[c][q], 0.0f);
            }
        } else {
            // slot scale: the largest message input of this neighbour slot
            float mx = 0.0f;
#pragma unroll
            for (int i = 0; i < 8; ++i) mx = fmaxf(fmaxf(fmaxf(mx, m[i].x), fmaxf(m[i].y, m[i].z)), m[i].w);
            const float sc = split_scale(wave_max(mx));
            const float isc = 1.0f / sc;
#pragma unroll
            for (int c = 0; c < 8; ++c) {
                const float bi = bsw[c] * sc;
                acc[c] = (f32x4){bi, bi, bi, bi};
            }
#pragma unroll
            for (int s4 = 0; s4 < 4; ++s4) {
                half8 hi, lo;
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const float x = f4c(m[2 * s4 + (j >> 2)], j & 3) * sc;
                    const _Float16 h = (_Float16)x;
                    hi[j] = h;
                    lo[j] = (_Float16)(x - (float)h);
                }
                half8 wh[8], wl[8];
#pragma unroll
                for (int c = 0; c < 8; ++c) {
                    const float4 a4 = wimg[((c * 4 + s4) * 2 + 0) * 64];
                    const float4 b4 = wimg[((c * 4 + s4) * 2 + 1) * 64];
                    wh[c] = *(const half8 *)&a4;
                    wl[c] = *(const half8 *)&b4;
                }
#pragma unroll
                for (int c = 0; c < 8; ++c) acc[c] = __builtin_amdgcn_mfma_f32_16x16x32_f16(hi, wh[c], acc[c], 0, 0, 0);
#pragma unroll
                for (int c = 0; c < 8; ++c) acc[c] = __builtin_amdgcn_mfma_f32_16x16x32_f16(hi, wl[c], acc[c], 0, 0, 0);
#pragma unroll
                for (int c = 0; c < 8; ++c) acc[c] = __builtin_amdgcn_mfma_f32_16x16x32_f16(lo, wh[c], acc[c], 0, 0, 0);
            }
#pragma unroll
            for (int c = 0; c < 8; ++c) {
                const float inv = isc * isw[c];
#pragma unroll
                for (int q = 0; q < 4; ++q) S[c][q] = fmaf(fmaxf(acc[c][q], 0.0f), inv, S[c][q]);
            }
        }
    }

    // ---- cross-wave sum of the edge messages: red[wave][row][col] ----------
    __syncthreads();  // every wave is done with the W2 image
    float *red = lds;                      // 4 x 16 x FRP
    float *vbuf = lds + 4 * FT * FRP;      // 16 x FRP
    float *hbuf = vbuf + FT * FRP;         // 16 x FRP
#pragma unroll
    for (int c = 0; c < 8; ++c) {
#pragma unroll
        for (int q = 0; q < 4; ++q) red[(wave * FT + 4 * g + q) * FRP + 16 * c + r] = S[c][q];
    }
    __syncthreads();
    const float kdiv = (float)p.k;

    // ---- update_net_1: v = relu(U1 [h | mean | t] + c1), cols 32 w .. 32 w + 31
    {
        f32x4 acc[2] = {(f32x4){0.0f, 0.0f, 0.0f, 0.0f}, (f32x4){0.0f, 0.0f, 0.0f, 0.0f}};
        const float *hrow = p.h + tgt * H + 4 * g;
#pragma unroll 2
        for (int j = 0; j < 8; ++j) {
            const float4 hv = *(const float4 *)(hrow + 16 * j);
            float4 mv = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
#pragma unroll
            for (int w = 0; w < 4; ++w) {
                const float4 x = *(const float4 *)(red + (w * FT + r) * FRP + 16 * j + 4 * g);
                mv.x += x.x;
                mv.y += x.y;
                mv.z += x.z;
                mv.w += x.w;
            }
            mv = make_float4(mv.x / kdiv, mv.y / kdiv, mv.z / kdiv, mv.w / kdiv);
#pragma unroll
            for (int cc = 0; cc < 2; ++cc) {
                const float *wr = p.u1 + (int64_t)(32 * wave + 16 * cc + r) * p.ld_u1 + 16 * j + 4 * g;
                const float4 wh = *(const float4 *)wr;
                const float4 wm = *(const float4 *)(wr + 128);
#pragma unroll
                for (int t = 0; t < 4; ++t) acc[cc] = mfma16(f4c(hv, t), f4c(wh, t), acc[cc]);
#pragma unroll
                for (int t = 0; t < 4; ++t) acc[cc] = mfma16(f4c(mv, t), f4c(wm, t), acc[cc]);
            }
        }
#pragma unroll
        for (int cc = 0; cc < 2; ++cc) {
            const int col = 32 * wave + 16 * cc + r;
            const float wt = p.u1[(int64_t)col * p.ld_u1 + 256], bb = p.c1[col];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int64_t row = min(tile0 + 4 * g + q, p.n - 1);
                const float pt = p.pos[row * 3 + 0] * p.sc.inv_tmax;
                vbuf[(4 * g + q) * FRP + col] = fmaxf(acc[cc][q] + wt * pt + bb, 0.0f);
            }
        }
    }
    __syncthreads();

    // ---- update_net_2 + residual + BatchNorm(eval) ----------------------------
    {
        f32x4 acc[2] = {(f32x4){0.0f, 0.0f, 0.0f, 0.0f}, (f32x4){0.0f, 0.0f, 0.0f, 0.0f}};
#pragma unroll 2
        for (int j = 0; j < 8; ++j) {
            const float4 vv = *(const float4 *)(vbuf + r * FRP + 16 * j + 4 * g);
#pragma unroll
            for (int cc = 0; cc < 2; ++cc) {
                const float4 w = *(const float4 *)(p.u2 + (32 * wave + 16 * cc + r) * H + 16 * j + 4 * g);
#pragma unroll
                for (int t = 0; t < 4; ++t) acc[cc] = mfma16(f4c(vv, t), f4c(w, t), acc[cc]);
            }
        }
#pragma unroll
        for (int cc = 0; cc < 2; ++cc) {
            const int col = 32 * wave + 16 * cc + r;
            const float bb = p.c2[col], rm = p.bn_rm[col], rv = p.bn_rv[col];
            const float gw = p.bn_w[col], gb = p.bn_b[col];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int64_t row = tile0 + 4 * g + q;
                const int64_t rowc = min(row, p.n - 1);
                const float x = p.h[rowc * H + col] + fmaxf(acc[cc][q] + bb, 0.0f);
                const float y = bn_eval(x, rm, rv, gw, gb, p.eps);
                if (row < p.n) p.h_out[row * H + col] = y;
                if (NEXT) hbuf[(4 * g + q) * FRP + col] = y;
            }
        }
    }
    if (!NEXT) return;
    __syncthreads();

    // ---- next layer's message_net_1 halves (EpiProj) -------------------------
    {
        f32x4 acc[4];
#pragma unroll
        for (int c = 0; c < 4; ++c) acc[c] = (f32x4){0.0f, 0.0f, 0.0f, 0.0f};
        // tiles 0,1: a' cols 32w+16cc (W1n[:, 0:128]); tiles 2,3: b' (W1n[:, 128:256])
#pragma unroll 2
        for (int j = 0; j < 8; ++j) {
            const float4 hv = *(const float4 *)(hbuf + r * FRP + 16 * j + 4 * g);
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                const int col = 32 * wave + 16 * (c & 1) + r;
                const float4 w = *(const float4 *)(p.w1n + (int64_t)col * p.ld_w1n + 128 * (c >> 1) + 16 * j + 4 * g);
#pragma unroll
                for (int t = 0; t < 4; ++t) acc[c] = mfma16(f4c(hv, t), f4c(w, t), acc[c]);
            }
        }
#pragma unroll
        for (int cc = 0; cc < 2; ++cc) {
            const int col = 32 * wave + 16 * cc + r;
            const float *wc = p.w1n + (int64_t)col * p.ld_w1n;
            const float wdu = wc[256], wdx = wc[257], wdy = wc[258], wt = wc[259];
            const float bb = p.b1n[col];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int64_t row = tile0 + 4 * g + q;
                if (row < p.n) {
                    const float uu = p.u[row];
                    const float px = p.pos[row * 3 + 1] * p.sc.inv_lx;
                    const float py = p.pos[row * 3 + 2] * p.sc.inv_ly;
                    const float pt = p.pos[row * 3 + 0] * p.sc.inv_tmax;
                    const float node = wdu * uu + wdx * px + wdy * py;
                    p.a_out[row * H + col] = acc[cc][q] + node + wt * pt + bb;
                    p.b_out[row * H + col] = acc[2 + cc][q] - node;
                }
            }
        }
    }
}

// ---------------------------------------------------------------------------
// Conv1d head (gnn_2d.py:108-114,136-139): one wave per node.
// 128 -> conv(1->4, k16, s3) 38 -> relu -> conv(4->8, k12, s3) 9 -> relu ->
// conv(8->1, k8, s2) 1, times out_scale.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void head_kernel(const float *__restrict__ h, int64_t n,
                                                   mmpde_gnn_head_params p,
                                                   float *__restrict__ out) {
    __shared__ float sw0[64 + 4], sw2[384 + 8], sw4[64 + 1];
    __shared__ float y1[4][4 * 38];
    __shared__ float y2[4][8 * 9];
    for (int i = threadIdx.x; i < 64; i += 256) sw0[i] = p.c0_w[i];
    for (int i = threadIdx.x; i < 4; i += 256) sw0[64 + i] = p.c0_b[i];
    for (int i = threadIdx.x; i < 384; i += 256) sw2[i] = p.c2_w[i];
    for (int i = threadIdx.x; i < 8; i += 256) sw2[384 + i] = p.c2_b[i];
    for (int i = threadIdx.x; i < 64; i += 256) sw4[i] = p.c4_w[i];
    if (threadIdx.x == 0) sw4[64] = p.c4_b[0];
    __syncthreads();
    const int wave = threadIdx.x >> 6;
    const int lane = threadIdx.x & 63;
    for (int64_t i = (int64_t)blockIdx.x * 4 + wave; i < n; i += (int64_t)gridDim.x * 4) {
        const float *hr = h + i * H;
        for (int e = lane; e < 4 * 38; e += 64) {
            const int c = e / 38, q = e - c * 38;
            float v = sw0[64 + c];
#pragma unroll
            for (int t = 0; t < 16; ++t) v += sw0[c * 16 + t] * hr[3 * q + t];
            y1[wave][e] = fmaxf(v, 0.0f);
        }
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        __builtin_amdgcn_wave_barrier();
        for (int e = lane; e < 8 * 9; e += 64) {  // 72 outputs > 64 lanes
            const int c = e / 9, q = e - c * 9;
            float v = sw2[384 + c];
            for (int ci = 0; ci < 4; ++ci) {
#pragma unroll
                for (int t = 0; t < 12; ++t) v += sw2[(c * 4 + ci) * 12 + t] * y1[wave][ci * 38 + 3 * q + t];
            }
            y2[wave][e] = fmaxf(v, 0.0f);
        }
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        __builtin_amdgcn_wave_barrier();
        {
            const int ci = lane >> 3, t = lane & 7;
            float v = sw4[ci * 8 + t] * y2[wave][ci * 9 + t];
            v = wave_sum(v);
            if (lane == 0) out[i] = p.out_scale * (v + sw4[64]);
        }
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        __builtin_amdgcn_wave_barrier();
    }
}

inline bool aligned16(const void *p) { return ((uintptr_t)p & 15u) == 0; }

}  // namespace

// ===========================================================================
// C-ABI
// ===========================================================================
extern "C" int64_t mmpde_gnn_workspace_bytes(int64_t n) {
    // h, a, b ping-pong = 6 x [n,128] fp32 (the unfused per-layer API uses
    // 4 of them as a, b, mean, v), then the F16X3 packed message_net_2 images
    return 6 * n * H * (int64_t)sizeof(float) + (int64_t)MMPDE_GNN_MAX_LAYERS * kW2PackBytes;
}

extern "C" int mmpde_gnn_embed(const float *u, const float *pos, int64_t n,
                               mmpde_gnn_scales sc, const mmpde_gnn_embed_params *p,
                               float *workspace, float *h_out, mmpde_stream_t stream) {
    MMPDE_REQUIRE(u && pos && p && workspace && h_out && n > 0);
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
        EpiUpd1 epi{wv, p->upd1_b, p->upd1_w + 256, ld, pos, sc.inv_tmax};
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
    return gnn_layer_impl(h_in, u, pos, n, k, nbr, sc, p, workspace, h_out, nullptr, nullptr,
                          stream);
}

extern "C" int mmpde_gnn_head(const float *h, int64_t n, const mmpde_gnn_head_params *p,
                              float *out, mmpde_stream_t stream) {
    MMPDE_REQUIRE(h && p && out && n > 0);
    int blocks = ceil_div(n, 4);
    if (blocks > 4096) blocks = 4096;
    hipLaunchKernelGGL(head_kernel, dim3(blocks), dim3(256), 0, as_stream(stream), h, n, *p,
                       out);
    MMPDE_RET_LAUNCH();
    return MMPDE_OK;
}

static int launch_fused_layer(const float *a, const float *b, const float *h, const float *u,
                              const float *pos, int64_t n, int k, const int32_t *nbr,
                              mmpde_gnn_scales sc, const mmpde_gnn_layer_params *p,
                              const mmpde_gnn_layer_params *next, const char *w2pk,
                              float *h_out, float *a_out, float *b_out, hipStream_t st) {
    MMPDE_REQUIRE(p->upd1_ld >= 257 && (p->upd1_ld & 3) == 0 && aligned16(p->upd1_w));
    MMPDE_REQUIRE(aligned16(p->msg2_w) && aligned16(p->upd2_w));
    FusedLayerArgs f{a, b, h, nbr, n, k, p->msg2_w, p->msg2_b, w2pk, p->upd1_w, p->upd1_b,
                     p->upd1_ld, p->upd2_w, p->upd2_b, p->bn_w, p->bn_b, p->bn_rm, p->bn_rv,
                     p->eps, h_out, nullptr, nullptr, 0, a_out, b_out, u, pos, sc};
    const dim3 grid(ceil_div(n, FT));
    if (next) {
        MMPDE_REQUIRE(next->msg1_ld >= 260 && (next->msg1_ld & 3) == 0 && aligned16(next->msg1_w));
        f.w1n = next->msg1_w;
        f.b1n = next->msg1_b;
        f.ld_w1n = next->msg1_ld;
    }
#define MMPDE_FUSED(NX, SPLIT) \
    hipLaunchKernelGGL((gnn_layer_fused_kernel<NX, SPLIT>), grid, dim3(256), 0, st, f)
    if (next && w2pk) MMPDE_FUSED(true, true);
    else if (next) MMPDE_FUSED(true, false);
    else if (w2pk) MMPDE_FUSED(false, true);
    else MMPDE_FUSED(false, false);
#undef MMPDE_FUSED
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
    const int mode = exec ? exec->edge_gemm : MMPDE_EDGE_GEMM_F32;
    MMPDE_REQUIRE(mode == MMPDE_EDGE_GEMM_F32 || mode == MMPDE_EDGE_GEMM_F16X3);
    hipStream_t st = as_stream(stream);
    float *ws = (float *)workspace;
    float *hb[2] = {ws, ws + n * H};
    float *ab[2] = {ws + 2 * n * H, ws + 3 * n * H};
    float *bb[2] = {ws + 4 * n * H, ws + 5 * n * H};
    char *pack = (char *)(ws + 6 * n * H);
    if (mode == MMPDE_EDGE_GEMM_F16X3 && n_layers > 0) {
        W2PackArgs pa{};
        for (int l = 0; l < n_layers; ++l) {
            MMPDE_REQUIRE(layers[l].msg2_w != nullptr);
            pa.w2[l] = layers[l].msg2_w;
        }
        hipLaunchKernelGGL(w2_pack_f16x3_kernel, dim3(H, n_layers), dim3(128), 0, st, pa, pack);
        MMPDE_RET_LAUNCH();
    }
    int rc = mmpde_gnn_embed(u, pos, n, sc, emb, ab[1], hb[0], stream);  // ab[1]: scratch
    if (rc) return rc;
    if (n_layers > 0) {
        // layer 0's message_net_1 halves; later layers get theirs from the fused kernel
        const mmpde_gnn_layer_params *p0 = &layers[0];
        MMPDE_REQUIRE(p0->msg1_ld >= 260 && (p0->msg1_ld & 3) == 0 && aligned16(p0->msg1_w));
        const int64_t ld = p0->msg1_ld;
        GemmArgs g{n, hb[0], hb[0] + 64, H, p0->msg1_w, p0->msg1_w + 64, ld, 64};
        EpiProj epi{ab[0], bb[0], p0->msg1_b, p0->msg1_w + 256, p0->msg1_w + 257,
                    p0->msg1_w + 258, p0->msg1_w + 259, ld, u, pos, sc};
        rc = launch_gemm<EpiProj, true>(g, 2, epi, st);
        if (rc) return rc;
    }
    int cur = 0;
    for (int l = 0; l < n_layers; ++l) {
        hipEvent_t eb = exec && exec->edge_begin ? (hipEvent_t)exec->edge_begin[l] : nullptr;
        hipEvent_t ee = exec && exec->edge_end ? (hipEvent_t)exec->edge_end[l] : nullptr;
        if (eb && hipEventRecord(eb, st) != hipSuccess) return MMPDE_ERR_INVALID_ARG;
        const mmpde_gnn_layer_params *next = l + 1 < n_layers ? &layers[l + 1] : nullptr;
        const char *w2pk = mode == MMPDE_EDGE_GEMM_F16X3 ? pack + (int64_t)l * kW2PackBytes : nullptr;
        rc = launch_fused_layer(ab[cur], bb[cur], hb[cur], u, pos, n, k, nbr, sc, &layers[l], next,
                                w2pk, hb[cur ^ 1], ab[cur ^ 1], bb[cur ^ 1], st);
        if (rc) return rc;
        if (ee && hipEventRecord(ee, st) != hipSuccess) return MMPDE_ERR_INVALID_ARG;
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
