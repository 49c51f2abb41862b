// ItpNet interpolation on gfx950 (reference interpolate.py:77-93 with the
// weighted sum of data_creator_2d.py:80-83).
//
// For every query q of trajectory b (neighbour indices from mmpde_knn_query):
//   X[q]  = [n0x, n0y, ..., n29x, n29y, qx, qy]                   (62)
//   W[q]  = L2(tanh(L1(tanh(L0(X[q])))))                         (62 -> 128 -> 64 -> 30)
//   out   = sum_e W[q, e] * vals[b, idx[q, e]]  (+ addend)
// One wave owns 16 queries and runs the three layers transposed (features on
// accumulator rows, queries on lanes) with exact-fp32 v_mfma_f32_16x16x4_f32.
// Lane (g, q) = (l >> 4, l & 15) holds rows 4 g + i (i < 4) of each 16-row
// accumulator tile, which is exactly the B operand of the next layer's K step
// (tile t, i) when that layer's K order is permuted to k = 16 t + 4 g + i: the
// weight images are packed in that order (mmpde_itp_pack), so no LDS or lane
// shuffles between layers.  16 queries per wave (not 32) halve each wave's
// serial MFMA chain.  Grid: two 512-thread workgroups per CU, all resident (the
// L0 and L1 images, 64 KB, are staged in LDS per workgroup; the L2 image, 8 KB,
// and the biases are read from L2); query tile t runs on workgroup t mod G, so
// every CU gets the same number of tiles (a 256-thread grid of one tile per wave
// ran the tail workgroups in a second round: 38 us at cy B=16).
#include "common.hpp"

namespace {

constexpr int kNb = 30;                     // ItpNet.n (interpolate.py:8)
constexpr int kImg0 = 8 * 16 * 64;          // [rt 16-feature tile][s K step][lane]
constexpr int kImg1 = 4 * 32 * 64;          // [rt][t * 4 + i][lane]
constexpr int kImg2 = 2 * 16 * 64;          // [rt][t * 4 + i][lane]
constexpr int kBias = 128 + 64 + 32;
constexpr int kPackFloats = kImg0 + kImg1 + kImg2 + kBias;

// lane l of a 16x16x4 A operand: row l & 15, k-index l >> 4 of the K step.
// Layer 0's K order is the input order (62 padded to 64); layers 1 and 2 take
// step (t, i) as inputs 16 t + 4 g + i, g = k-index.
__global__ void itp_pack_kernel(mmpde_itp_mlp m, float *__restrict__ pk) {
    const int e = blockIdx.x * 256 + threadIdx.x;
    if (e >= kPackFloats) return;
    float v = 0.0f;
    if (e < kImg0) {
        const int lane = e & 63, s = (e >> 6) & 15, rt = e >> 10;
        const int in = 4 * s + (lane >> 4);
        if (in < 62) v = m.w0[(16 * rt + (lane & 15)) * 62 + in];
    } else if (e < kImg0 + kImg1) {
        const int f = e - kImg0;
        const int lane = f & 63, ks = (f >> 6) & 31, rt = f >> 11;
        const int feat = 16 * (ks >> 2) + 4 * (lane >> 4) + (ks & 3);
        v = m.w1[(16 * rt + (lane & 15)) * 128 + feat];
    } else if (e < kImg0 + kImg1 + kImg2) {
        const int f = e - kImg0 - kImg1;
        const int lane = f & 63, ks = (f >> 6) & 15, rt = f >> 10;
        const int feat = 16 * (ks >> 2) + 4 * (lane >> 4) + (ks & 3);
        const int o = 16 * rt + (lane & 15);
        if (o < kNb) v = m.w2[o * 64 + feat];
    } else {
        const int f = e - kImg0 - kImg1 - kImg2;
        if (f < 128) v = m.b0[f];
        else if (f < 192) v = m.b1[f - 128];
        else if (f - 192 < kNb) v = m.b2[f - 192];
    }
    pk[e] = v;
}

constexpr int kItpThreads = 512;

__global__ __launch_bounds__(kItpThreads, 4) void itp_interp_kernel(
    const float *__restrict__ src, const float *__restrict__ vals, const float *__restrict__ qry,
    const int32_t *__restrict__ idx, int64_t batches, int64_t n_src, int64_t n_qry,
    const float *__restrict__ pk, const float *__restrict__ addend, const float *__restrict__ addend2,
    float *__restrict__ out) {
    __shared__ float4 img[(kImg0 + kImg1) / 4];  // 64 KB
    {
        const float4 *gsrc = (const float4 *)pk;
        for (int e = threadIdx.x; e < (kImg0 + kImg1) / 4; e += kItpThreads) img[e] = gsrc[e];
    }
    __syncthreads();
    const float *img0 = (const float *)img;
    const float *img1 = img0 + kImg0;
    const float *img2 = pk + kImg0 + kImg1;
    const float *bias = img2 + kImg2;

    const int wave = threadIdx.x >> 6;
    const int lane = threadIdx.x & 63;
    const int g = lane >> 4;
    const int64_t tiles_per_b = (n_qry + 15) / 16;
    const int64_t n_tiles = tiles_per_b * batches;

    // waves w and w + 4 share a SIMD: odd workgroups start on the other SIMD pair
    const int slot = (blockIdx.x & 1) ? (wave + 2) & 7 : wave;
    for (int64_t tile = (int64_t)slot * gridDim.x + blockIdx.x; tile < n_tiles;
         tile += (int64_t)gridDim.x * (kItpThreads / 64)) {
        const int64_t b = tile / tiles_per_b;
        const int64_t q0 = (tile - b * tiles_per_b) * 16;
        int64_t q = q0 + (lane & 15);
        const bool valid = q < n_qry;
        if (!valid) q = n_qry - 1;
        const int64_t qrow = b * n_qry + q;
        const int32_t *ir = idx + qrow * kNb;
        const float2 *sp = (const float2 *)src + b * n_src;

        // layer-0 B operand of K step s: input 4 s + g (neighbour 2 s + g / 2,
        // coordinate g & 1; step 15: the query's coordinates, then 0)
        float xin[16];
#pragma unroll
        for (int s = 0; s < 15; ++s) {
            const float2 p = sp[min((uint32_t)ir[2 * s + (g >> 1)], (uint32_t)(n_src - 1))];
            xin[s] = (g & 1) ? p.y : p.x;
        }
        {
            const float2 p = ((const float2 *)qry)[qrow];
            xin[15] = g == 0 ? p.x : g == 1 ? p.y : 0.0f;
        }
        // L0 row tile rt (16 of the 128 hidden units) is computed, tanh'd and
        // immediately consumed by L1 as its K steps (rt, i): one L0 tile live.
        f32x4 a1[4];
#pragma unroll
        for (int rt = 0; rt < 4; ++rt)
#pragma unroll
            for (int i = 0; i < 4; ++i) a1[rt][i] = bias[128 + 16 * rt + 4 * g + i];
#pragma unroll 1
        for (int rt = 0; rt < 8; ++rt) {
            f32x4 a0;
#pragma unroll
            for (int i = 0; i < 4; ++i) a0[i] = bias[16 * rt + 4 * g + i];
#pragma unroll
            for (int s = 0; s < 16; ++s) a0 = mfma16(img0[(rt * 16 + s) * 64 + lane], xin[s], a0);
#pragma unroll
            for (int i = 0; i < 4; ++i) a0[i] = tanhf(a0[i]);
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int r1 = 0; r1 < 4; ++r1)
                    a1[r1] = mfma16(img1[(r1 * 32 + rt * 4 + i) * 64 + lane], a0[i], a1[r1]);
        }
        // the neighbour values of this lane's outputs o = 16 r2 + 4 g + i, all
        // loaded before the L1 tanh and L2 (a load under the o < kNb test of the
        // weighted sum is waited for at once: eight dependent round trips per
        // tile; issuing them with the coordinates spills)
        const float *vb = vals + b * n_src;
        float nv[8];
#pragma unroll
        for (int r2 = 0; r2 < 2; ++r2)
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int o = min(16 * r2 + 4 * g + i, kNb - 1);
                nv[4 * r2 + i] = vb[min((uint32_t)ir[o], (uint32_t)(n_src - 1))];
            }
        // the epilogue's addends, unconditionally (a missing one reads the query
        // array in its place and is dropped below)
        const float ad1 = (addend ? addend : qry)[qrow];
        const float ad2 = (addend2 ? addend2 : qry)[qrow];
#pragma unroll
        for (int r1 = 0; r1 < 4; ++r1)
#pragma unroll
            for (int i = 0; i < 4; ++i) a1[r1][i] = tanhf(a1[r1][i]);
        // L2: weights^T [30 (32) x 16 q]
        f32x4 a2[2];
#pragma unroll
        for (int r2 = 0; r2 < 2; ++r2)
#pragma unroll
            for (int i = 0; i < 4; ++i) a2[r2][i] = bias[192 + 16 * r2 + 4 * g + i];
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int r2 = 0; r2 < 2; ++r2)
                    a2[r2] = mfma16(img2[(r2 * 16 + t * 4 + i) * 64 + lane], a1[t][i], a2[r2]);
        // weighted sum of the neighbour values (data_creator_2d.py:83): this lane's
        // outputs o = 16 r2 + 4 g + i, then the 4 lanes of the query
        float sum = 0.0f;
#pragma unroll
        for (int r2 = 0; r2 < 2; ++r2)
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int o = 16 * r2 + 4 * g + i;
                if (o < kNb) sum += a2[r2][i] * nv[4 * r2 + i];
            }
        sum += __shfl_xor(sum, 16, 64);
        sum += __shfl_xor(sum, 32, 64);
        if (g == 0 && valid) {
            float o = addend ? ad1 + sum : sum;
            if (addend2) o = o + ad2;  // (interp + res) + model(graph_uniform)
            out[qrow] = o;
        }
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
    return mmpde_itp_interp_ex(src, vals, qry, idx, batches, n_src, n_qry, packed, addend, nullptr, out,
                               stream);
}

extern "C" int mmpde_itp_interp_ex(const float *src, const float *vals, const float *qry,
                                   const int32_t *idx, int64_t batches, int64_t n_src,
                                   int64_t n_qry, const void *packed, const float *addend,
                                   const float *addend2, float *out, mmpde_stream_t stream) {
    MMPDE_REQUIRE(src && vals && qry && idx && packed && out);
    MMPDE_REQUIRE(batches > 0 && n_src >= kNb && n_qry > 0);
    const int64_t tiles = ((n_qry + 15) / 16) * batches;
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus < 1)
        cus = 256;
    int64_t blocks = 2 * (int64_t)cus;               // two resident workgroups per CU
    if (blocks > tiles) blocks = tiles;
    hipLaunchKernelGGL(itp_interp_kernel, dim3((unsigned)blocks), dim3(kItpThreads), 0, as_stream(stream), src, vals,
                       qry, idx, batches, n_src, n_qry, (const float *)packed, addend, addend2, out);
    MMPDE_RET_LAUNCH();
    return MMPDE_OK;
}
