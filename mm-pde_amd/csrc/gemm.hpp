// Node-row GEMM on v_mfma_f32_32x32x2_f32, shared by gnn.hip and dmm.hip.
#pragma once
#include "common.hpp"

namespace {

// ---------------------------------------------------------------------------
// Node GEMM: out[m, c] = epi(sum_k X[m, k] W[c, k]), 32 rows x 128 columns per
// workgroup (4 waves x one 32x32 MFMA tile).  The K dimension is split in two
// halves of KH: MFMA k-lane 0 walks (X0, W0), k-lane 1 walks (X1, W1).  This lets
// a lane stream 16-B contiguous chunks of its row and lets one GEMM consume a
// concatenated input (h | mean) without building it.
// ---------------------------------------------------------------------------
struct GemmArgs {
    int64_t m;
    const float *x0, *x1;
    int64_t ldx;
    const float *w0, *w1;
    int64_t ldw;
    int kh;
};

struct EpiStore {  // plain store, row stride ldo
    float *out;
    int64_t ldo;
    __device__ void operator()(const f32x16 &acc, int64_t row0, int col0, int lane, int64_t m,
                               int) const {
        const int c = col0 + (lane & 31);
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int64_t row = row0 + acc_row(r, lane);
            if (row < m) out[row * ldo + c] = acc[r];
        }
    }
};

// grid: (ceil(m/32), parts); part p uses weight rows [p*128, p*128+128) unless
// the epilogue re-targets (EpiProj uses part to pick the W1 half instead).
template <class Epi, bool PROJ>
__global__ __launch_bounds__(256) void node_gemm_kernel(GemmArgs g, Epi epi) {
    const int wave = threadIdx.x >> 6;
    const int lane = threadIdx.x & 63;
    const int half = lane >> 5;
    const int part = blockIdx.y;
    const int64_t row0 = (int64_t)blockIdx.x * 32;
    int64_t row = row0 + (lane & 31);
    if (row >= g.m) row = g.m - 1;
    const int col0 = PROJ ? wave * 32 : part * 128 + wave * 32;
    // PROJ: part 0 -> W1[:, 0:128] (target half), part 1 -> W1[:, 128:256] (source half)
    const int64_t wofs = PROJ ? (int64_t)part * 128 : 0;
    const float *xp = (half ? g.x1 : g.x0) + row * g.ldx;
    const float *wp = (half ? g.w1 : g.w0) + wofs + (int64_t)(col0 + (lane & 31)) * g.ldw;
    f32x16 acc = {0};
#pragma unroll 4
    for (int s = 0; s < g.kh; s += 4) {
        const float4 a = *(const float4 *)(xp + s);
        const float4 w = *(const float4 *)(wp + s);
        acc = mfma32(a.x, w.x, acc);
        acc = mfma32(a.y, w.y, acc);
        acc = mfma32(a.z, w.z, acc);
        acc = mfma32(a.w, w.w, acc);
    }
    epi(acc, row0, col0, lane, g.m, part);
}

template <class Epi, bool PROJ = false>
int launch_gemm(const GemmArgs &g, int parts, const Epi &epi, hipStream_t st) {
    if (g.m <= 0 || (g.kh & 3) != 0) return MMPDE_ERR_INVALID_ARG;
    dim3 grid(ceil_div(g.m, 32), parts);
    hipLaunchKernelGGL((node_gemm_kernel<Epi, PROJ>), grid, dim3(256), 0, st, g, epi);
    MMPDE_RET_LAUNCH();
    return MMPDE_OK;
}


}  // namespace
