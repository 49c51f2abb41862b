// Shared device helpers for libmmpde_hip.so (gfx950 / CDNA4, wave64).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/mmpde_hip.h"

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

#define MMPDE_RET_LAUNCH()                                   \
    do {                                                     \
        hipError_t e_ = hipGetLastError();                   \
        if (e_ != hipSuccess) return MMPDE_ERR_HIP_BASE - (int)e_; \
    } while (0)

#define MMPDE_REQUIRE(cond)                          \
    do {                                             \
        if (!(cond)) return MMPDE_ERR_INVALID_ARG;   \
    } while (0)

static inline hipStream_t as_stream(mmpde_stream_t s) { return (hipStream_t)s; }

// v_mfma_f32_32x32x2_f32: lane l supplies A[l&31][l>>5] and B[l>>5][l&31];
// D[row][col] with col = l&31, row = (r&3) + 8*(r>>2) + 4*(l>>5) for register r.
__device__ __forceinline__ f32x16 mfma32(float a, float b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ int acc_row(int reg, int lane) {
    return (reg & 3) + 8 * (reg >> 2) + 4 * (lane >> 5);
}

// v_mfma_f32_16x16x4_f32: lane l supplies A[l&15][l>>4] and B[l>>4][l&15];
// D[4*(l>>4) + r][l&15] for register r (exact fp32, 32-cycle issue).
__device__ __forceinline__ f32x4 mfma16(float a, float b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// Blocks are dealt round-robin over the 8 XCDs (MI355X_MICROARCH.md, Workgroup
// dispatch): remap so that each XCD walks a contiguous range of tiles (its L2
// then holds the rows those tiles gather).  Bijective for any grid size; speed
// only, never correctness.
__device__ __forceinline__ int xcd_tile(int bid, int nb) {
    const int q = nb >> 3, rem = nb & 7;
    const int x = bid & 7, i = bid >> 3;
    return x < rem ? x * (q + 1) + i : rem * (q + 1) + (x - rem) * q + i;
}

// component t (compile-time after unrolling) of a float4
__device__ __forceinline__ float f4c(const float4 &v, int t) {
    return t == 0 ? v.x : t == 1 ? v.y : t == 2 ? v.z : v.w;
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
    return v;
}

// Max reductions of non-negative floats (|x| maxima, never NaN) without the
// LDS pipe (a __shfl_xor is a ds_bpermute round trip): on their bit patterns
// (for x, y >= 0, bits(max(x, y)) = max(bits(x), bits(y)), and the integer max
// needs no NaN canonicalisation), DPP within 16-lane rows, v_permlane16/32_swap
// across rows.  Every lane of the wave must be active (a DPP read of a
// disabled lane is not defined).  The swaps' outputs with both operands v:
// lane l's partner value (l ^ 16, l ^ 32) is output 0 in the upper row (half),
// output 1 in the lower (as knn.hip's xor_lane).
template <int CTRL>
__device__ __forceinline__ uint32_t dpp_u(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, 0xF, 0xF, false);
}
__device__ __forceinline__ uint32_t umax_rows16(uint32_t v) {  // max with lane ^ 16
    const auto r = __builtin_amdgcn_permlane16_swap(v, v, false, false);
    return max(v, (__lane_id() & 16) ? r[0] : r[1]);
}
__device__ __forceinline__ uint32_t umax_rows32(uint32_t v) {  // max with lane ^ 32
    const auto r = __builtin_amdgcn_permlane32_swap(v, v, false, false);
    return max(v, (__lane_id() & 32) ? r[0] : r[1]);
}
// max over the wave of v >= 0 (quad [1,0,3,2], quad [2,3,0,1], row_half_mirror,
// row_mirror, then across rows)
__device__ __forceinline__ float wave_absmax(float v) {
    uint32_t u = __builtin_bit_cast(uint32_t, v);
    u = max(u, dpp_u<0xB1>(u));
    u = max(u, dpp_u<0x4E>(u));
    u = max(u, dpp_u<0x141>(u));
    u = max(u, dpp_u<0x140>(u));
    return __builtin_bit_cast(float, umax_rows32(umax_rows16(u)));
}
// v of lane ^ O (O = 1 .. 32) without the LDS pipe; every lane active.  The
// same exchange as __shfl_xor(v, O), so a butterfly built from it adds the
// same operands in the same order as one built from __shfl_xor.
template <int O>
__device__ __forceinline__ float xor_lane_f(float v) {
    const uint32_t u = __builtin_bit_cast(uint32_t, v);
    uint32_t r;
    if constexpr (O == 1) {
        r = dpp_u<0xB1>(u);  // quad [1,0,3,2]
    } else if constexpr (O == 2) {
        r = dpp_u<0x4E>(u);  // quad [2,3,0,1]
    } else if constexpr (O == 4) {
        const uint32_t up = dpp_u<0x104>(u), dn = dpp_u<0x114>(u);  // row_shl:4 / row_shr:4
        r = (__lane_id() & 4) ? dn : up;
    } else if constexpr (O == 8) {
        r = dpp_u<0x128>(u);  // row_ror:8
    } else if constexpr (O == 16) {
        const auto q = __builtin_amdgcn_permlane16_swap(u, u, false, false);
        r = (__lane_id() & 16) ? q[0] : q[1];
    } else {
        static_assert(O == 32, "xor_lane_f: O in 1, 2, 4, 8, 16, 32");
        const auto q = __builtin_amdgcn_permlane32_swap(u, u, false, false);
        r = (__lane_id() & 32) ? q[0] : q[1];
    }
    return __builtin_bit_cast(float, r);
}
// wave_sum / wave_max with every lane active: the same butterfly (32, 16, ...,
// 1), so the same bits, without a ds_bpermute round trip per step.
__device__ __forceinline__ float wave_sum_full(float v) {
    v += xor_lane_f<32>(v);
    v += xor_lane_f<16>(v);
    v += xor_lane_f<8>(v);
    v += xor_lane_f<4>(v);
    v += xor_lane_f<2>(v);
    v += xor_lane_f<1>(v);
    return v;
}
__device__ __forceinline__ float wave_max_full(float v) {
    v = fmaxf(v, xor_lane_f<32>(v));
    v = fmaxf(v, xor_lane_f<16>(v));
    v = fmaxf(v, xor_lane_f<8>(v));
    v = fmaxf(v, xor_lane_f<4>(v));
    v = fmaxf(v, xor_lane_f<2>(v));
    v = fmaxf(v, xor_lane_f<1>(v));
    return v;
}

// max of v >= 0 over lanes l, l ^ 8, l ^ 16, ... l ^ 56 (row_ror:8 = lane ^ 8 in a 16-lane row)
__device__ __forceinline__ float absmax_stride8(float v) {
    uint32_t u = __builtin_bit_cast(uint32_t, v);
    u = max(u, dpp_u<0x128>(u));
    return __builtin_bit_cast(float, umax_rows32(umax_rows16(u)));
}

__device__ __forceinline__ float act_apply(float v, int act) {
    if (act == MMPDE_ACT_TANH) return tanhf(v);
    if (act == MMPDE_ACT_RELU) return fmaxf(v, 0.0f);
    if (act == MMPDE_ACT_ELU) return v > 0.0f ? v : expm1f(v);
    return v;
}

// Eval-mode BatchNorm1d on one channel value (torch: (x - rm) / sqrt(rv + eps) * w + b)
__device__ __forceinline__ float bn_eval(float v, float rm, float rv, float w, float b,
                                         float eps) {
    return (v - rm) / sqrtf(rv + eps) * w + b;
}

// BatchNorm (eval) folded per channel as PyTorch's CPU kernel applies it
// (alpha = w / sqrt(rv + eps), beta = b - rm alpha, y = x alpha + beta): two
// constants per channel instead of a division per element.
struct BnAffine {
    float a = 1.0f, c = 0.0f;
    __device__ __forceinline__ void set(float rm, float rv, float w, float b, float eps) {
        const float invstd = 1.0f / sqrtf(rv + eps);
        a = invstd * w;
        c = b - rm * a;
    }
    __device__ __forceinline__ float operator()(float x) const { return fmaf(x, a, c); }
};

// x / d rounded to nearest-even (IEEE binary32 division), for d > 0 with r =
// 1.0f / d (itself an IEEE division, once per row): q0 = x r, then one
// Markstein correction q0 + (x - q0 d) r, the residual exact by the fma.  That
// is the correctly rounded quotient whenever it is a normal number (checked
// against x / d on 2.0e9 random normal x for every d = 1 .. 1024,
// tools/div_check.c); quotients in the subnormal range take the division
// itself.  3 VALU instead of the ~10 of the IEEE division sequence.
// div_rows_rn: N float4 of one row by the row's d, one slow-path test per row.
template <int N>
__device__ __forceinline__ void div_rows_rn(float4 (&x)[N], float d) {
    const float r = 1.0f / d;
    float4 y[N];
    bool tiny = false;
    auto one = [&](float v) {
        const float q0 = v * r;
        tiny |= q0 != 0.0f && fabsf(q0) < 0x1p-125f;
        return fmaf(fmaf(-q0, d, v), r, q0);
    };
#pragma unroll
    for (int q = 0; q < N; ++q) y[q] = make_float4(one(x[q].x), one(x[q].y), one(x[q].z), one(x[q].w));
    if (__builtin_expect(tiny, 0)) {
#pragma unroll
        for (int q = 0; q < N; ++q) y[q] = make_float4(x[q].x / d, x[q].y / d, x[q].z / d, x[q].w / d);
    }
#pragma unroll
    for (int q = 0; q < N; ++q) x[q] = y[q];
}

// Node position fields of the GNN (mmpde_gnn_scales.pos_xy: (t, x, y) rows, or
// (x, y) rows with one t for every node), unscaled.
__device__ __forceinline__ float node_t(const mmpde_gnn_scales &sc, const float *pos, int64_t row) {
    return sc.pos_xy ? (sc.t_ptr ? *sc.t_ptr : sc.t) : pos[row * 3];
}
__device__ __forceinline__ float node_x(const mmpde_gnn_scales &sc, const float *pos, int64_t row) {
    return sc.pos_xy ? pos[row * 2] : pos[row * 3 + 1];
}
__device__ __forceinline__ float node_y(const mmpde_gnn_scales &sc, const float *pos, int64_t row) {
    return sc.pos_xy ? pos[row * 2 + 1] : pos[row * 3 + 2];
}

static inline int ceil_div(int64_t a, int64_t b) { return (int)((a + b - 1) / b); }

// library-internal entry points shared between translation units
namespace mmpde_detail {
// mmpde_conv2d (dense.hip) with a side job: threads [0, n_zero) also store 0
// to zero[] (dmm.hip's split-K tickets, zeroed by its first kernel)
__attribute__((visibility("hidden"))) int conv2d(const float *x, int64_t batches, int cin, int h,
                                                 int w, const float *weight, const float *bias,
                                                 int cout, int ks, int stride, int pad,
                                                 const float *residual, int act, float *y,
                                                 hipStream_t st, unsigned *zero, int n_zero,
                                                 int circular = 0, int res_after_act = 0);
}  // namespace mmpde_detail
