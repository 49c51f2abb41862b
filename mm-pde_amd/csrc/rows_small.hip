// Skinny row maps of the training path: y = x W^T + b (the forward) and
// dX = dY W (the input gradient) when one side of the map is narrow -- the
// Conv1d head as unfold + GEMM (gnn_2d.py:108-114: 16 -> 4, 48 -> 8, 64 -> 1
// per window row) and the embedding's first Linear (4 -> 128, and back,
// gnn_2d.py:99-106).  A 32 x 32 MFMA tile would run mostly empty on these, so
// they stay on the VALU.
//
// With kin inputs and kout outputs per row (NT: kin = K, kout = N; NN: kin =
// N, kout = K), the map is staged once per workgroup in LDS as M[k][o] (k <
// kin, o < kout rounded up to 4; NT transposes W while staging).  Thread (row,
// q) computes outputs 4q .. 4q + 3 of its row: the row's inputs in registers
// (loaded by every thread of the row: one request per row), one ds_read_b128
// of M per input, a float4 store -- so the threads of a wave write whole
// contiguous runs of rows.  Persistent workgroups stride over the rows.  Sums
// run in a fixed order (k ascending): deterministic.
#include "common.hpp"

#include <algorithm>

namespace {

struct SmallArgs {
    const float *x;
    int64_t ldx, n;
    int kin, kout;
    const float *w;
    int64_t ldw;
    int layout;
    const float *bias;
    float *y;
    int64_t ldy;
    int tpr_log2;  // threads per row = 2^tpr_log2 >= kout / 4
};

// 16 of the row's inputs (k0 .. k0 + 15) into registers; VX: float4 loads
// (16-byte rows).  The loads are unconditional (indices clamped into the row;
// the FMAs skip k >= kin): a load under a condition is waited for where the
// condition ends.
template <bool VX>
__device__ __forceinline__ void load16(const float *xr, int k0, int kin, float (&v)[16]) {
    if (VX) {
#pragma unroll
        for (int k = 0; k < 16; k += 4) {
            const float4 q = *(const float4 *)(xr + min(k0 + k, kin - 4));
            v[k] = q.x;
            v[k + 1] = q.y;
            v[k + 2] = q.z;
            v[k + 3] = q.w;
        }
    } else {
#pragma unroll
        for (int k = 0; k < 16; ++k) v[k] = xr[min(k0 + k, kin - 1)];
    }
}

template <bool VX, bool VY>
__global__ __launch_bounds__(256) void rows_small_kernel(SmallArgs a) {
    extern __shared__ float4 m4[];
    float *ms = (float *)m4;
    const int kout4 = (a.kout + 3) & ~3, q4 = kout4 >> 2;
    for (int idx = threadIdx.x; idx < a.kin * kout4; idx += 256) {
        const int k = idx / kout4, o = idx - k * kout4;
        float v = 0.0f;
        if (o < a.kout)
            v = a.layout == MMPDE_RGEMM_NT ? a.w[(int64_t)o * a.ldw + k] : a.w[(int64_t)k * a.ldw + o];
        ms[idx] = v;
    }
    __syncthreads();
    const int tq = threadIdx.x & ((1 << a.tpr_log2) - 1);
    const int rpb = 256 >> a.tpr_log2;
    const int o0 = 4 * tq;
    if (o0 >= a.kout) return;  // no barrier past this point
    float4 b4 = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    if (a.bias) {
        const float *b = a.bias;
        const int l = a.kout - 1;
        b4 = make_float4(b[min(o0, l)], b[min(o0 + 1, l)], b[min(o0 + 2, l)], b[min(o0 + 3, l)]);
    }
    const int64_t stride = (int64_t)gridDim.x * rpb;
    // a few registers per thread: the latency of the row loads is covered by
    // the many waves resident per SIMD
    for (int64_t row = (int64_t)blockIdx.x * rpb + (threadIdx.x >> a.tpr_log2); row < a.n; row += stride) {
        const float *xr = a.x + row * a.ldx;
        float4 acc = b4;
        for (int k0 = 0; k0 < a.kin; k0 += 16) {
            float v[16];
            load16<VX>(xr, k0, a.kin, v);
#pragma unroll
            for (int k = 0; k < 16; ++k) {
                if (k0 + k >= a.kin) break;  // uniform
                const float4 m = m4[(k0 + k) * q4 + tq];
                acc.x = fmaf(v[k], m.x, acc.x);
                acc.y = fmaf(v[k], m.y, acc.y);
                acc.z = fmaf(v[k], m.z, acc.z);
                acc.w = fmaf(v[k], m.w, acc.w);
            }
        }
        float *yr = a.y + row * a.ldy + o0;
        if (VY && o0 + 3 < a.kout) {
            *(float4 *)yr = acc;
        } else {
            yr[0] = acc.x;
            if (o0 + 1 < a.kout) yr[1] = acc.y;
            if (o0 + 2 < a.kout) yr[2] = acc.z;
            if (o0 + 3 < a.kout) yr[3] = acc.w;
        }
    }
}

bool al16(const void *p) { return ((uintptr_t)p & 15) == 0; }

int small_cus() {
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
        cus = 256;
    return cus;
}

}  // namespace

extern "C" int mmpde_rows_small(const float *x, int64_t ldx, int64_t n, int ki, const float *w, int64_t ldw,
                                int layout, const float *bias, int no, float *y, int64_t ldy,
                                mmpde_stream_t stream) {
    MMPDE_REQUIRE(x && w && y && n > 0 && ki >= 1 && no >= 1 && n < ((int64_t)1 << 40));
    MMPDE_REQUIRE(layout == MMPDE_RGEMM_NT || layout == MMPDE_RGEMM_NN);
    SmallArgs a{};
    a.x = x;
    a.ldx = ldx;
    a.n = n;
    a.w = w;
    a.ldw = ldw;
    a.layout = layout;
    a.bias = bias;
    a.y = y;
    a.ldy = ldy;
    if (layout == MMPDE_RGEMM_NT) {
        // x [n, ki] (ldx), W [no, ki] (ldw), y [n, no] (ldy)
        MMPDE_REQUIRE(ldx >= ki && ldw >= ki && ldy >= no);
        a.kin = ki;
        a.kout = no;
    } else {
        // x = dY [n, no] (ldx), W [no, ki] (ldw), y = dX [n, ki] (ldy)
        MMPDE_REQUIRE(ldx >= no && ldw >= ki && ldy >= ki && bias == nullptr);
        a.kin = no;
        a.kout = ki;
    }
    const int kout4 = (a.kout + 3) & ~3;
    MMPDE_REQUIRE(a.kin <= 128 && a.kout <= 128 && (int64_t)a.kin * kout4 <= 16384);
    int tl = 0;
    while ((1 << tl) * 4 < a.kout) ++tl;
    a.tpr_log2 = tl;
    const int64_t rpb = 256 >> tl;
    const size_t lds = (size_t)a.kin * kout4 * 4;
    // persistent: enough workgroups for ~8 waves per SIMD, each staging the map once
    const int per_cu = std::max(1, std::min(8, (int)(131072 / std::max<size_t>(lds, 1))));
    const int64_t blocks = std::min<int64_t>((n + rpb - 1) / rpb, (int64_t)per_cu * small_cus());
    const bool vx = a.kin % 4 == 0 && ldx % 4 == 0 && al16(x);
    const bool vy = ldy % 4 == 0 && al16(y);
    hipStream_t st = as_stream(stream);
    const dim3 grid((unsigned)blocks);
#define SM_LAUNCH(VX_, VY_) hipLaunchKernelGGL((rows_small_kernel<VX_, VY_>), grid, dim3(256), lds, st, a)
    if (vx && vy) SM_LAUNCH(true, true);
    else if (vx) SM_LAUNCH(true, false);
    else if (vy) SM_LAUNCH(false, true);
    else SM_LAUNCH(false, false);
#undef SM_LAUNCH
    MMPDE_RET_LAUNCH();
    return MMPDE_OK;
}
