// ItpNet interpolation on gfx950 (reference interpolate.py:77-93 with the
// weighted sum of data_creator_2d.py:80-83).
//
// For every query q of trajectory b (neighbour indices from mmpde_knn_query):
//   X[q]  = [n0x, n0y, ..., n29x, n29y, qx, qy]                   (62)
//   W[q]  = L2(tanh(L1(tanh(L0(X[q])))))                         (62 -> 128 -> 64 -> 30)
//   out   = sum_e W[q, e] * vals[b, idx[q, e]]  (+ addend)
// One wave owns 32 queries and runs the three layers transposed (features on
// accumulator rows, queries on lanes) with v_mfma_f32_32x32x2_f32, so each
// layer's accumulator is directly the next layer's B operand -- no LDS or lane
// shuffles between layers.  The weights are re-laid once (mmpde_itp_pack) into
// the exact per-lane A-operand image; L0 and L1 images (64 KB) are staged in
// LDS per workgroup, the L2 image (8 KB) and biases are read from L2.
#include "common.hpp"

namespace {

constexpr int kNb = 30;                     // ItpNet.n (interpolate.py:8)
constexpr int kImg0 = 4 * 32 * 64;          // [rt][s][lane]
constexpr int kImg1 = 2 * 64 * 64;          // [gt][ks][lane]
constexpr int kImg2 = 32 * 64;              // [ks][lane]
constexpr int kBias = 128 + 64 + 32;
constexpr int kPackFloats = kImg0 + kImg1 + kImg2 + kBias;

__global__ void itp_pack_kernel(mmpde_itp_mlp m, float *__restrict__ pk) {
    const int e = blockIdx.x * 256 + threadIdx.x;
    if (e >= kPackFloats) return;
    float v = 0.0f;
    if (e < kImg0) {
        const int lane = e & 63, s = (e >> 6) & 31, rt = e >> 11;
        const int in = 2 * s + (lane >> 5);
        if (in < 62) v = m.w0[(32 * rt + (lane & 31)) * 62 + in];
    } else if (e < kImg0 + kImg1) {
        const int f = e - kImg0;
        const int lane = f & 63, ks = (f >> 6) & 63, gt = f >> 12;
        const int rt = ks >> 4, p = ks & 15;
        const int feat = 32 * rt + acc_row(p, lane);
        v = m.w1[(32 * gt + (lane & 31)) * 128 + feat];
    } else if (e < kImg0 + kImg1 + kImg2) {
        const int f = e - kImg0 - kImg1;
        const int lane = f & 63, ks = f >> 6;
        const int gt = ks >> 4, p = ks & 15;
        const int feat = 32 * gt + acc_row(p, lane);
        const int o = lane & 31;
        if (o < kNb) v = m.w2[o * 64 + feat];
    } else {
        const int f = e - kImg0 - kImg1 - kImg2;
        if (f < 128) v = m.b0[f];
        else if (f < 192) v = m.b1[f - 128];
        else if (f - 192 < kNb) v = m.b2[f - 192];
    }
    pk[e] = v;
}

__global__ __launch_bounds__(256, 2) void itp_interp_kernel(
    const float *__restrict__ src, const float *__restrict__ vals, const float *__restrict__ qry,
    const int32_t *__restrict__ idx, int64_t batches, int64_t n_src, int64_t n_qry,
    const float *__restrict__ pk, const float *__restrict__ addend, float *__restrict__ out) {
    __shared__ float4 img[(kImg0 + kImg1) / 4];  // 64 KB
    {
        const float4 *g = (const float4 *)pk;
        for (int e = threadIdx.x; e < (kImg0 + kImg1) / 4; e += 256) img[e] = g[e];
    }
    __syncthreads();
    const float *img0 = (const float *)img;
    const float *img1 = img0 + kImg0;
    const float *img2 = pk + kImg0 + kImg1;
    const float *bias = img2 + kImg2;

    const int wave = threadIdx.x >> 6;
    const int lane = threadIdx.x & 63;
    const int half = lane >> 5;
    const int64_t tiles_per_b = (n_qry + 31) / 32;
    const int64_t n_tiles = tiles_per_b * batches;

    for (int64_t tile = (int64_t)blockIdx.x * 4 + wave; tile < n_tiles;
         tile += (int64_t)gridDim.x * 4) {
        const int64_t b = tile / tiles_per_b;
        const int64_t q0 = (tile - b * tiles_per_b) * 32;
        int64_t q = q0 + (lane & 31);
        const bool valid = q < n_qry;
        if (!valid) q = n_qry - 1;
        const int64_t qrow = b * n_qry + q;
        const int32_t *ir = idx + qrow * kNb;
        const float2 *sp = (const float2 *)src + b * n_src;

        // layer-0 B operand: coordinate `half` of point s (neighbours 0..29, query, 0)
        float xin[32];
#pragma unroll
        for (int s = 0; s < kNb; ++s) {
            const float2 p = sp[min((uint32_t)ir[s], (uint32_t)(n_src - 1))];
            xin[s] = half ? p.y : p.x;
        }
        {
            const float2 p = ((const float2 *)qry)[qrow];
            xin[30] = half ? p.y : p.x;
            xin[31] = 0.0f;
        }
        // L0 row tile rt (32 of the 128 hidden units, H1^T[32 x 32q]) is computed,
        // tanh'd and immediately consumed by L1 as its k-steps (rt, p), p = register:
        // only one L0 tile is ever live.
        f32x16 a1[2];
#pragma unroll
        for (int gt = 0; gt < 2; ++gt)
#pragma unroll
            for (int r = 0; r < 16; ++r) a1[gt][r] = bias[128 + 32 * gt + acc_row(r, lane)];
#pragma unroll 1
        for (int rt = 0; rt < 4; ++rt) {
            f32x16 a0;
#pragma unroll
            for (int r = 0; r < 16; ++r) a0[r] = bias[32 * rt + acc_row(r, lane)];
#pragma unroll
            for (int s = 0; s < 32; ++s) a0 = mfma32(img0[(rt * 32 + s) * 64 + lane], xin[s], a0);
#pragma unroll
            for (int r = 0; r < 16; ++r) a0[r] = tanhf(a0[r]);
#pragma unroll
            for (int p = 0; p < 16; ++p)
#pragma unroll
                for (int gt = 0; gt < 2; ++gt)
                    a1[gt] = mfma32(img1[(gt * 64 + rt * 16 + p) * 64 + lane], a0[p], a1[gt]);
        }
#pragma unroll
        for (int gt = 0; gt < 2; ++gt)
#pragma unroll
            for (int r = 0; r < 16; ++r) a1[gt][r] = tanhf(a1[gt][r]);
        // L2: weights^T [30(32) x 32q]
        f32x16 a2;
#pragma unroll
        for (int r = 0; r < 16; ++r) a2[r] = bias[192 + acc_row(r, lane)];
#pragma unroll
        for (int gt = 0; gt < 2; ++gt)
#pragma unroll
            for (int p = 0; p < 16; ++p)
                a2 = mfma32(img2[(gt * 16 + p) * 64 + lane], a1[gt][p], a2);
        // weighted sum of the neighbour values (data_creator_2d.py:83)
        const float *vb = vals + b * n_src;
        float sum = 0.0f;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int o = acc_row(r, lane);
            if (o < kNb) sum += a2[r] * vb[min((uint32_t)ir[o], (uint32_t)(n_src - 1))];
        }
        sum += __shfl_xor(sum, 32, 64);
        if (half == 0 && valid) out[qrow] = addend ? addend[qrow] + sum : sum;
    }
}

}  // namespace

extern "C" int64_t mmpde_itp_pack_bytes(void) { return (int64_t)kPackFloats * sizeof(float); }

extern "C" int mmpde_itp_pack(const mmpde_itp_mlp *mlp, void *packed, mmpde_stream_t stream) {
    MMPDE_REQUIRE(mlp && packed && (((uintptr_t)packed) & 15u) == 0);
    hipLaunchKernelGGL(itp_pack_kernel, dim3(ceil_div(kPackFloats, 256)), dim3(256), 0,
                       as_stream(stream), *mlp, (float *)packed);
    MMPDE_RET_LAUNCH();
    return MMPDE_OK;
}

extern "C" int mmpde_itp_interp(const float *src, const float *vals, const float *qry,
                                const int32_t *idx, int64_t batches, int64_t n_src,
                                int64_t n_qry, const void *packed, const float *addend,
                                float *out, mmpde_stream_t stream) {
    MMPDE_REQUIRE(src && vals && qry && idx && packed && out);
    MMPDE_REQUIRE(batches > 0 && n_src >= kNb && n_qry > 0);
    const int64_t tiles = ((n_qry + 31) / 32) * batches;
    int blocks = ceil_div(tiles, 4);
    if (blocks > 1024) blocks = 1024;
    hipLaunchKernelGGL(itp_interp_kernel, dim3(blocks), dim3(256), 0, as_stream(stream), src, vals,
                       qry, idx, batches, n_src, n_qry, (const float *)packed, addend, out);
    MMPDE_RET_LAUNCH();
    return MMPDE_OK;
}
