// The Conv1d head of MP_PDE_Solver_2D in train mode (reference gnn_2d.py:108-114,
// 136: output_mlp = Conv1d(1, 4, 16, stride 3) -> ReLU -> Conv1d(4, 8, 12,
// stride 3) -> ReLU -> Conv1d(8, 1, 8, stride 2) over each node's 128 hidden
// values, time_window = 1), forward and backward in two launches instead of
// the unfold + GEMM + ReLU chain (three window matrices of up to 1.5 M rows,
// their copies, unfold's backward, ~0.48 ms per model at cy B=16).
//
// One lane per node: the node's 128 inputs and the 8 x 8 second-layer
// activations the output reads in registers, the 38 x 4 first-layer ones in
// registers (forward) or in LDS (backward: registers for the gradient terms;
// 47 KB per one-wave workgroup, three per CU) (the
// second layer's ninth position feeds no output of the last layer and gets no
// gradient).  The weights are wave-uniform (scalar loads).  The backward
// recomputes the forward, then per node: dL/dz2, the weight gradients' per-node
// terms, dL/dz1, dL/dx (written); the 525 weight / bias gradient terms are
// summed over the wave's 64 nodes in lane order (through an LDS transpose, 32
// or 24 terms at a time; the 13 bias terms by a fixed butterfly) and stored as
// the wave's partials, and a second kernel adds the partials in wave order.
// Deterministic; fp32 throughout.
#include "common.hpp"

#include <algorithm>

namespace {

constexpr int HX = 128;                          // inputs per node
constexpr int C1 = 4, K1 = 16, S1 = 3, L1 = 38;  // conv 1
constexpr int C2 = 8, K2 = 12, S2 = 3, L2U = 8;  // conv 2 (positions read by conv 3)
constexpr int K3 = 8;                            // conv 3 (one output position)
// gradient buffer: [dW1 (4x1x16) | db1 (4) | dW2 (8x4x12) | db2 (8) | dW3 (1x8x8) | db3 (1)]
constexpr int O_W1 = 0, O_B1 = O_W1 + C1 * K1, O_W2 = O_B1 + C1, O_B2 = O_W2 + C2 * C1 * K2;
constexpr int O_W3 = O_B2 + C2, O_B3 = O_W3 + C2 * K3, NG = O_B3 + 1;
static_assert(NG == MMPDE_HEAD_TRAIN_GRADS, "gradient layout");

struct HeadW {
    const float *w1, *b1, *w2, *b2, *w3, *b3;
};

__device__ __forceinline__ void load_row(const float *__restrict__ h, int64_t ldh, int64_t i, float (&x)[HX]) {
    const float4 *r = (const float4 *)(h + i * ldh);
#pragma unroll
    for (int q = 0; q < HX / 4; ++q) {
        const float4 v = r[q];
        x[4 * q] = v.x;
        x[4 * q + 1] = v.y;
        x[4 * q + 2] = v.z;
        x[4 * q + 3] = v.w;
    }
}

__device__ __forceinline__ float relu(float v) { return v > 0.0f ? v : 0.0f; }

// y1 = relu(conv1(x)), y2 = relu(conv2(y1)) at the positions conv 3 reads.  Loop
// order: output channel outermost, so each channel's taps are loaded once (a
// few scalar loads) and reused over every position; each sum in a fixed order
// (bias, then input channel, then tap)
__device__ __forceinline__ void head_fwd(const HeadW &w, const float (&x)[HX], float (&y1)[L1][C1],
                                         float (&y2)[L2U][C2]) {
#pragma unroll
    for (int o = 0; o < C1; ++o) {
        float wt[K1];
#pragma unroll
        for (int c = 0; c < K1; ++c) wt[c] = w.w1[o * K1 + c];
        const float b = w.b1[o];
#pragma unroll
        for (int l = 0; l < L1; ++l) {
            float s = b;
#pragma unroll
            for (int c = 0; c < K1; ++c) s = fmaf(wt[c], x[S1 * l + c], s);
            y1[l][o] = relu(s);
        }
    }
#pragma unroll
    for (int o = 0; o < C2; ++o) {
        float s[L2U];
        const float b = w.b2[o];
#pragma unroll
        for (int m = 0; m < L2U; ++m) s[m] = b;
#pragma unroll
        for (int ci = 0; ci < C1; ++ci) {
            float wt[K2];
#pragma unroll
            for (int c = 0; c < K2; ++c) wt[c] = w.w2[(o * C1 + ci) * K2 + c];
#pragma unroll
            for (int m = 0; m < L2U; ++m)
#pragma unroll
                for (int c = 0; c < K2; ++c) s[m] = fmaf(wt[c], y1[S2 * m + c][ci], s[m]);
        }
#pragma unroll
        for (int m = 0; m < L2U; ++m) y2[m][o] = relu(s[m]);
    }
}

// x[3l .. 3l + 15] of this lane's row (five 16-byte reads; rows 16-B aligned)
__device__ __forceinline__ void x_window(const float *xr, int l, float (&xw)[K1]) {
    const int q0 = (S1 * l) >> 2, off = S1 * l - 4 * q0;  // compile-time after unrolling
    float v[20];
#pragma unroll
    for (int q = 0; q < 5; ++q) {
        const float4 t = *(const float4 *)(xr + 4 * (q0 + q));
        v[4 * q] = t.x;
        v[4 * q + 1] = t.y;
        v[4 * q + 2] = t.z;
        v[4 * q + 3] = t.w;
    }
#pragma unroll
    for (int c = 0; c < K1; ++c) xw[c] = v[off + c];
}

__device__ __forceinline__ float head_out(const HeadW &w, const float (&y2)[L2U][C2]) {
    float s = w.b3[0];
#pragma unroll
    for (int ci = 0; ci < C2; ++ci)
#pragma unroll
        for (int c = 0; c < K3; ++c) s = fmaf(w.w3[ci * K3 + c], y2[c][ci], s);
    return s;
}

__global__ __launch_bounds__(64) void head_train_fwd_kernel(const float *__restrict__ h, int64_t ldh, int64_t n,
                                                            HeadW w, float *__restrict__ y) {
    const int64_t i = (int64_t)blockIdx.x * 64 + threadIdx.x;
    if (i >= n) return;  // no barrier below
    float x[HX], y1[L1][C1], y2[L2U][C2];
    load_row(h, ldh, i, x);
    head_fwd(w, x, y1, y2);
    y[i] = head_out(w, y2);
}

// the wave's sum of v (every lane active) stored by lane 0 as partial o
__device__ __forceinline__ void put(float *__restrict__ pp, int o, float v) {
    v = wave_sum_full(v);
    if (__lane_id() == 0) pp[o] = v;
}

constexpr int RN = 32, RP = 64 + 4;  // terms per transpose; its column pitch (16-B aligned)

// N <= RN per-node terms v[] of every lane summed over the wave's 64 lanes in
// lane order (through LDS: term t of lane l at red[t][l]; lane t reads its 64
// values as 16-byte vectors and adds them in lane order) and stored as partials
// o0 .. o0 + N - 1.  The workgroup is this one wave.
template <int N>
__device__ __forceinline__ void flush(float *red, float *__restrict__ pp, int o0, const float *v) {
    static_assert(N <= RN, "transpose width");
    const int lane = __lane_id();
#pragma unroll
    for (int t = 0; t < N; ++t) red[t * RP + lane] = v[t];
    __syncthreads();
    if (lane < N) {
        const float4 *col = (const float4 *)(red + lane * RP);
        float4 q[16];
#pragma unroll
        for (int k = 0; k < 16; ++k) q[k] = col[k];
        float s = 0.0f;
#pragma unroll
        for (int k = 0; k < 16; ++k) s = (((s + q[k].x) + q[k].y) + q[k].z) + q[k].w;
        pp[o0 + lane] = s;
    }
    __syncthreads();  // the buffer is free again
}

__global__ __launch_bounds__(64) void head_train_bwd_kernel(
    const float *__restrict__ h, int64_t ldh, int64_t n, const float *__restrict__ w1,
    const float *__restrict__ b1, const float *__restrict__ w2, const float *__restrict__ b2,
    const float *__restrict__ w3, const float *__restrict__ b3, const float *__restrict__ dy,
    float *__restrict__ dh, int64_t lddh, float *__restrict__ part) {
    // separate __restrict__ weight pointers: no store of this kernel can alias
    // them, so their wave-uniform loads stay scalar after the partial stores
    const HeadW w{w1, b1, w2, b2, w3, b3};
    __shared__ float ys[L1 * C1 * 64];  // y1, then dL/dz1, lane-minor (conflict-free)
    __shared__ float red[RN * RP];      // the gradient terms' transposes
    const int lane = threadIdx.x;
    const int64_t i0 = (int64_t)blockIdx.x * 64 + lane;
    const bool live = i0 < n;
    const int64_t i = live ? i0 : n - 1;  // every lane stays (wave sums); dead lanes add g = 0
    const float *xr = h + i * ldh;
    float y2[L2U][C2];
    const float gl = dy[i];
    {
        float x[HX], y1[L1][C1];
        load_row(h, ldh, i, x);
        head_fwd(w, x, y1, y2);
#pragma unroll
        for (int l = 0; l < L1; ++l)
#pragma unroll
            for (int ci = 0; ci < C1; ++ci) ys[(l * C1 + ci) * 64 + lane] = y1[l][ci];
    }
#define Y1(l, ci) ys[((l) * C1 + (ci)) * 64 + lane]
    const float g = live ? gl : 0.0f;
    float *pp = part + (int64_t)blockIdx.x * NG;
    // conv 3: dW3[ci][c] = g y2[c][ci], db3 = g; dL/dz2 through the ReLU
    float d2[L2U][C2];
    {
        float t3[C2 * K3];
#pragma unroll
        for (int ci = 0; ci < C2; ++ci)
#pragma unroll
            for (int c = 0; c < K3; ++c) {
                t3[ci * K3 + c] = g * y2[c][ci];
                d2[c][ci] = y2[c][ci] > 0.0f ? g * w.w3[ci * K3 + c] : 0.0f;
            }
        flush<RN>(red, pp, O_W3, t3);
        flush<RN>(red, pp, O_W3 + RN, t3 + RN);
    }
    put(pp, O_B3, g);
    // conv 2: dW2[o][ci][c] = sum_m d2[m][o] y1[3m + c][ci], db2[o] = sum_m d2[m][o]
#pragma unroll
    for (int o = 0; o < C2; ++o) {
        float t2[C1 * K2];
#pragma unroll
        for (int ci = 0; ci < C1; ++ci)
#pragma unroll
            for (int c = 0; c < K2; ++c) {
                float s = 0.0f;
#pragma unroll
                for (int m = 0; m < L2U; ++m) s = fmaf(d2[m][o], Y1(S2 * m + c, ci), s);
                t2[ci * K2 + c] = s;
            }
        flush<C1 * K2 / 2>(red, pp, O_W2 + o * C1 * K2, t2);
        flush<C1 * K2 / 2>(red, pp, O_W2 + o * C1 * K2 + C1 * K2 / 2, t2 + C1 * K2 / 2);
        float s = 0.0f;
#pragma unroll
        for (int m = 0; m < L2U; ++m) s += d2[m][o];
        put(pp, O_B2 + o, s);
    }
    // dL/dz1[l][ci] = [y1 > 0] sum over o (outer) and (m, c = l - 3m) of d2[m][o]
    // W2[o][ci][c] (in place of y1, each value read here for the last time; only
    // this lane touches its column of ys, so no barrier)
#pragma unroll
    for (int ci = 0; ci < C1; ++ci) {
        float a1[L1];
#pragma unroll
        for (int l = 0; l < L1; ++l) a1[l] = 0.0f;
#pragma unroll
        for (int o = 0; o < C2; ++o) {
            float wt[K2];
#pragma unroll
            for (int c = 0; c < K2; ++c) wt[c] = w.w2[(o * C1 + ci) * K2 + c];
#pragma unroll
            for (int m = 0; m < L2U; ++m)
#pragma unroll
                for (int c = 0; c < K2; ++c) a1[S2 * m + c] = fmaf(d2[m][o], wt[c], a1[S2 * m + c]);
        }
#pragma unroll
        for (int l = 0; l < L1; ++l) Y1(l, ci) = Y1(l, ci) > 0.0f ? a1[l] : 0.0f;
    }
    // conv 1: dW1[o][c] = sum_l dz1[l][o] x[3l + c] (l ascending), db1[o] = sum_l dz1[l][o]
    {
        float t1[C1 * K1];
#pragma unroll
        for (int t = 0; t < C1 * K1; ++t) t1[t] = 0.0f;
#pragma unroll
        for (int l = 0; l < L1; ++l) {
            float xw[K1];
            x_window(xr, l, xw);
#pragma unroll
            for (int o = 0; o < C1; ++o)
#pragma unroll
                for (int c = 0; c < K1; ++c) t1[o * K1 + c] = fmaf(Y1(l, o), xw[c], t1[o * K1 + c]);
        }
        flush<RN>(red, pp, O_W1, t1);
        flush<RN>(red, pp, O_W1 + RN, t1 + RN);
    }
#pragma unroll
    for (int o = 0; o < C1; ++o) {
        float s = 0.0f;
#pragma unroll
        for (int l = 0; l < L1; ++l) s += Y1(l, o);
        put(pp, O_B1 + o, s);
    }
    // dL/dx[j] = sum over o (outer) and (l ascending, c = j - 3l) of dz1[l][o]
    // W1[o][c], scattered channel by channel
    if (!live) return;  // the wave's sums are done
    float dx[HX];
#pragma unroll
    for (int j = 0; j < HX; ++j) dx[j] = 0.0f;
#pragma unroll
    for (int o = 0; o < C1; ++o) {
        float wt[K1];
#pragma unroll
        for (int c = 0; c < K1; ++c) wt[c] = w.w1[o * K1 + c];
#pragma unroll
        for (int l = 0; l < L1; ++l) {
            const float z = Y1(l, o);
#pragma unroll
            for (int c = 0; c < K1; ++c) dx[S1 * l + c] = fmaf(z, wt[c], dx[S1 * l + c]);
        }
    }
    float4 *dr = (float4 *)(dh + i * lddh);
#pragma unroll
    for (int q = 0; q < HX / 4; ++q) dr[q] = make_float4(dx[4 * q], dx[4 * q + 1], dx[4 * q + 2], dx[4 * q + 3]);
}

// grads[o] = sum over the waves' partials in wave order: one wave per output,
// lane l adding partials l, l + 64, ... in order, then a fixed butterfly
__global__ __launch_bounds__(256) void head_train_sum_kernel(const float *__restrict__ part, int G,
                                                             float *__restrict__ grads) {
    const int o = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (o >= NG) return;  // wave-uniform
    float s = 0.0f;
    for (int g = lane; g < G; g += 64) s += part[(int64_t)g * NG + o];
    s = wave_sum_full(s);
    if (lane == 0) grads[o] = s;
}

bool al16(const void *p) { return ((uintptr_t)p & 15) == 0; }

}  // namespace

extern "C" int64_t mmpde_head_train_workspace_bytes(int64_t n) {
    if (n <= 0) return 0;
    return (n + 63) / 64 * (int64_t)NG * (int64_t)sizeof(float);
}

extern "C" int mmpde_head_train_forward(const float *h, int64_t ldh, int64_t n, const float *w1, const float *b1,
                                        const float *w2, const float *b2, const float *w3, const float *b3,
                                        float *y, mmpde_stream_t stream) {
    MMPDE_REQUIRE(h && y && w1 && b1 && w2 && b2 && w3 && b3 && n > 0);
    MMPDE_REQUIRE(ldh >= HX && ldh % 4 == 0 && al16(h));
    const HeadW w{w1, b1, w2, b2, w3, b3};
    MMPDE_REQUIRE(n < ((int64_t)1 << 36));
    hipLaunchKernelGGL(head_train_fwd_kernel, dim3((unsigned)((n + 63) / 64)), dim3(64), 0, as_stream(stream), h,
                       ldh, n, w, y);
    MMPDE_RET_LAUNCH();
    return MMPDE_OK;
}

extern "C" int mmpde_head_train_backward(const float *h, int64_t ldh, int64_t n, const float *w1, const float *b1,
                                         const float *w2, const float *b2, const float *w3, const float *b3,
                                         const float *dy, float *dh, int64_t lddh, float *grads,
                                         float *workspace, int64_t workspace_bytes, mmpde_stream_t stream) {
    MMPDE_REQUIRE(h && dy && dh && grads && w1 && b1 && w2 && b2 && w3 && b3 && n > 0);
    MMPDE_REQUIRE(ldh >= HX && ldh % 4 == 0 && al16(h) && lddh >= HX && lddh % 4 == 0 && al16(dh));
    MMPDE_REQUIRE(workspace && workspace_bytes >= mmpde_head_train_workspace_bytes(n));
    MMPDE_REQUIRE(n < ((int64_t)1 << 36));
    const int64_t G = (n + 63) / 64;
    hipStream_t st = as_stream(stream);
    hipLaunchKernelGGL(head_train_bwd_kernel, dim3((unsigned)G), dim3(64), 0, st, h, ldh, n, w1, b1, w2, b2, w3, b3,
                       dy, dh, lddh, workspace);
    MMPDE_RET_LAUNCH();
    hipLaunchKernelGGL(head_train_sum_kernel, dim3((unsigned)ceil_div(NG, 4)), dim3(256), 0, st, workspace, (int)G,
                       grads);
    MMPDE_RET_LAUNCH();
    return MMPDE_OK;
}
