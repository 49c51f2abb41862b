// F16X3 split arithmetic shared by gnn.hip and layer.hip: power-of-two
// scales, fp16 hi/lo splits, the packed weight-image format and its packing
// kernel.  (fp32-emulating split GEMM, include/mmpde_hip.h MMPDE_EDGE_GEMM_F16X3)
#pragma once
#include "common.hpp"

namespace {

typedef _Float16 half8 __attribute__((ext_vector_type(8)));

// Power of two s with mx * s in [2^13, 2^14) (fp16 max 65504): the scale of
// the F16X3 split.  mx zero / subnormal / inf / nan -> 1; clamped to
// [2^-40, 2^40] so a scaled bias can never overflow fp32.
__device__ __forceinline__ float split_scale(float mx) {
    const int eb = (int)((__float_as_uint(mx) >> 23) & 0xff);
    if (eb == 0 || eb == 255) return 1.0f;
    const int se = min(max(267 - eb, 127 - 40), 127 + 40);
    return __uint_as_float((uint32_t)se << 23);
}

// Split scale of one target row of the edge stage (f16x3.hpp split8_relu_rtz
// needs |relu(a + b)| s < 2^11): s = split_scale(M) / 8 for a bound M >= every
// |a_ik + b_jk| of the row (layer.hpp row maxima).
__device__ __forceinline__ float row_split_scale(float M) { return 0.125f * split_scale(M); }

// 1 / s for a power of two s from split_scale (exact).
__device__ __forceinline__ float pow2_inv(float s) {
    const uint32_t eb = (__float_as_uint(s) >> 23) & 0xff;
    return __uint_as_float((254u - eb) << 23);
}

// ---------------------------------------------------------------------------
// F16X3 weight images (once per parameter change, mmpde_gnn_pack_f16x3).  A
// B-operand matrix B[k][j] = W[row(j)][koff(j) + k] (K = 128 or 256) is packed
// column by column: column j is scaled by sw[j] = split_scale(max_k |B[k][j]|)
// and split into fp16 hi + lo, laid out as the exact per-lane B operand of
// v_mfma_f32_16x16x32_f16: [ctile j/16][kstep K/32][hi|lo][lane][8 halves],
// lane = 16 g + (j & 15) holding k = 32 s + 8 g + t; followed by sw[n_cols].
// Per layer: message_net_2 (edge), update_net_1 (h | mean part), update_net_2
// and message_net_1 as the two node halves (j < 128: W1[j, 0:128] -> a;
// j >= 128: W1[j-128, 128:256] -> b).
// ---------------------------------------------------------------------------
constexpr int64_t kPkW2 = 0;                              // 128 x 128
constexpr int64_t kPkU1 = kPkW2 + 65536 + 512;            // 128 x 256
constexpr int64_t kPkU2 = kPkU1 + 131072 + 512;           // 128 x 128
constexpr int64_t kPkW1 = kPkU2 + 65536 + 512;            // 256 x 128
constexpr int64_t kLayerPack = kPkW1 + 131072 + 1024;     // bytes per layer (16-B multiple)
static_assert(kLayerPack % 16 == 0, "pack alignment");

struct PackSrc {
    const float *w[MMPDE_GNN_MAX_LAYERS];
    int64_t ld[MMPDE_GNN_MAX_LAYERS];
};

template <int K>
__global__ __launch_bounds__(K) void pack_f16x3_kernel(PackSrc src, int half_split, int64_t img_off,
                                                       int64_t n_cols, char *__restrict__ pack) {
    __shared__ float red[K / 64];
    const int layer = blockIdx.y, jcol = blockIdx.x, k = threadIdx.x;
    const int row = half_split ? (jcol & 127) : jcol;
    const int koff = half_split ? (jcol >> 7) * 128 : 0;
    const float w = src.w[layer][(int64_t)row * src.ld[layer] + koff + k];
    const float m = wave_max(fabsf(w));
    if ((k & 63) == 0) red[k >> 6] = m;
    __syncthreads();
    float mx = red[0];
#pragma unroll
    for (int i = 1; i < K / 64; ++i) mx = fmaxf(mx, red[i]);
    const float sw = split_scale(mx);
    const float x = w * sw;
    const _Float16 hi = (_Float16)x;
    const _Float16 lo = (_Float16)(x - (float)hi);
    const int c = jcol >> 4, s = k >> 5, g = (k >> 3) & 3, t = k & 7;
    const int lane = 16 * g + (jcol & 15);
    char *base = pack + (int64_t)layer * kLayerPack + img_off;
    _Float16 *img = (_Float16 *)base;
    img[(((c * (K / 32) + s) * 2 + 0) * 64 + lane) * 8 + t] = hi;
    img[(((c * (K / 32) + s) * 2 + 1) * 64 + lane) * 8 + t] = lo;
    if (k == 0) ((float *)(base + n_cols * K * 4))[jcol] = sw;
}

// B fragment (c, s, hi|lo) of a packed image with KS k-steps, as a half8.
__device__ __forceinline__ half8 bfrag(const char *img, int KS, int c, int s, int hl, int lane) {
    const float4 v = ((const float4 *)img)[((c * KS + s) * 2 + hl) * 64 + lane];
    return *(const half8 *)&v;
}

// Scaled fp16 hi/lo split of 8 consecutive-k values.
__device__ __forceinline__ void split8(const float4 &x0, const float4 &x1, float sc, half8 &hi,
                                       half8 &lo) {
#pragma unroll
    for (int t = 0; t < 8; ++t) {
        const float x = f4c(t < 4 ? x0 : x1, t & 3) * sc;
        const _Float16 h = (_Float16)x;
        hi[t] = h;
        lo[t] = (_Float16)(x - (float)h);
    }
}

// The same split as split8 with sc = 1 in 12 instructions: hi by v_cvt_pk_f16_f32
// (RN), lo = RN_f16(x - f32(hi)) by v_fma_mix (x - hi is exact in f32, so
// the result is bit-identical to split8; tools/ubench/split_check.hip).  The
// trailing s_nop covers the VALU-write -> MFMA-operand hazard, which hipcc does
// not pad for asm producers (cdna_hip_programming.md §5.7).
__device__ __forceinline__ void split8_rn(const float4 &a, const float4 &b, half8 &hi, half8 &lo) {
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
    u32x4 h, l;
    asm("v_cvt_pk_f16_f32 %0, %8, %9\n\t"
        "v_cvt_pk_f16_f32 %1, %10, %11\n\t"
        "v_cvt_pk_f16_f32 %2, %12, %13\n\t"
        "v_cvt_pk_f16_f32 %3, %14, %15\n\t"
        "v_fma_mixlo_f16 %4, %8, 1.0, -%0 op_sel_hi:[0,0,1]\n\t"
        "v_fma_mixhi_f16 %4, %9, 1.0, -%0 op_sel:[0,0,1] op_sel_hi:[0,0,1]\n\t"
        "v_fma_mixlo_f16 %5, %10, 1.0, -%1 op_sel_hi:[0,0,1]\n\t"
        "v_fma_mixhi_f16 %5, %11, 1.0, -%1 op_sel:[0,0,1] op_sel_hi:[0,0,1]\n\t"
        "v_fma_mixlo_f16 %6, %12, 1.0, -%2 op_sel_hi:[0,0,1]\n\t"
        "v_fma_mixhi_f16 %6, %13, 1.0, -%2 op_sel:[0,0,1] op_sel_hi:[0,0,1]\n\t"
        "v_fma_mixlo_f16 %7, %14, 1.0, -%3 op_sel_hi:[0,0,1]\n\t"
        "v_fma_mixhi_f16 %7, %15, 1.0, -%3 op_sel:[0,0,1] op_sel_hi:[0,0,1]\n\t"
        "s_nop 1"
        : "=&v"(h.x), "=&v"(h.y), "=&v"(h.z), "=&v"(h.w), "=&v"(l.x), "=&v"(l.y), "=&v"(l.z),
          "=&v"(l.w)
        : "v"(a.x), "v"(a.y), "v"(a.z), "v"(a.w), "v"(b.x), "v"(b.y), "v"(b.z), "v"(b.w));
    hi = *(const half8 *)&h;
    lo = *(const half8 *)&l;
}

// relu + split of 8 consecutive-k values in 16 instructions, for inputs
// scaled so that |x| < 2^11: hi = max(RTZ_f16(x), 0) (v_cvt_pkrtz + v_pk_max_f16),
// lo = clamp01(RN_f16(x - hi_rtz)) by v_fma_mix ... clamp.  With round-toward-
// zero hi, x - hi has the sign of x and |x - hi| < ulp(hi) <= 1, so the [0, 1]
// clamp is exactly the relu of the low part: (hi, lo) is the split of
// relu(x) (x = hi + lo to 2^-22 relative, like split8_rn).
__device__ __forceinline__ void split8_relu_rtz(const float4 &a, const float4 &b, half8 &hi,
                                                half8 &lo) {
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
    u32x4 h, l;
    asm("v_cvt_pkrtz_f16_f32 %0, %8, %9\n\t"
        "v_cvt_pkrtz_f16_f32 %1, %10, %11\n\t"
        "v_cvt_pkrtz_f16_f32 %2, %12, %13\n\t"
        "v_cvt_pkrtz_f16_f32 %3, %14, %15\n\t"
        "v_fma_mixlo_f16 %4, %8, 1.0, -%0 op_sel_hi:[0,0,1] clamp\n\t"
        "v_fma_mixhi_f16 %4, %9, 1.0, -%0 op_sel:[0,0,1] op_sel_hi:[0,0,1] clamp\n\t"
        "v_fma_mixlo_f16 %5, %10, 1.0, -%1 op_sel_hi:[0,0,1] clamp\n\t"
        "v_fma_mixhi_f16 %5, %11, 1.0, -%1 op_sel:[0,0,1] op_sel_hi:[0,0,1] clamp\n\t"
        "v_fma_mixlo_f16 %6, %12, 1.0, -%2 op_sel_hi:[0,0,1] clamp\n\t"
        "v_fma_mixhi_f16 %6, %13, 1.0, -%2 op_sel:[0,0,1] op_sel_hi:[0,0,1] clamp\n\t"
        "v_fma_mixlo_f16 %7, %14, 1.0, -%3 op_sel_hi:[0,0,1] clamp\n\t"
        "v_fma_mixhi_f16 %7, %15, 1.0, -%3 op_sel:[0,0,1] op_sel_hi:[0,0,1] clamp\n\t"
        "v_pk_max_f16 %0, %0, 0\n\t"
        "v_pk_max_f16 %1, %1, 0\n\t"
        "v_pk_max_f16 %2, %2, 0\n\t"
        "v_pk_max_f16 %3, %3, 0\n\t"
        "s_nop 1"
        : "=&v"(h.x), "=&v"(h.y), "=&v"(h.z), "=&v"(h.w), "=&v"(l.x), "=&v"(l.y), "=&v"(l.z),
          "=&v"(l.w)
        : "v"(a.x), "v"(a.y), "v"(a.z), "v"(a.w), "v"(b.x), "v"(b.y), "v"(b.z), "v"(b.w));
    hi = *(const half8 *)&h;
    lo = *(const half8 *)&l;
}

// split8_relu_rtz for one pair of values (4 instructions), for schedules that
// spread a slot's split between MFMAs.  No trailing s_nop: the caller
// guarantees that no MFMA reads hi / lo within the next two instructions (the
// wave kernel consumes them one slot later).
__device__ __forceinline__ void split2_relu_rtz(float x0, float x1, uint32_t &hi, uint32_t &lo) {
    asm("v_cvt_pkrtz_f16_f32 %0, %2, %3\n\t"
        "v_fma_mixlo_f16 %1, %2, 1.0, -%0 op_sel_hi:[0,0,1] clamp\n\t"
        "v_fma_mixhi_f16 %1, %3, 1.0, -%0 op_sel:[0,0,1] op_sel_hi:[0,0,1] clamp\n\t"
        "v_pk_max_f16 %0, %0, 0"
        : "=&v"(hi), "=&v"(lo)
        : "v"(x0), "v"(x1));
}

// split2_relu_rtz in two halves of two instructions, for schedules that place
// each half in its own MFMA gap: _a = hi (RTZ, before the relu) and the low
// word of lo, _b = the high word of lo and the relu of hi.
__device__ __forceinline__ void split2_relu_rtz_a(float x0, float x1, uint32_t &hi, uint32_t &lo) {
    asm("v_cvt_pkrtz_f16_f32 %0, %2, %3\n\t"
        "v_fma_mixlo_f16 %1, %2, 1.0, -%0 op_sel_hi:[0,0,1] clamp"
        : "=&v"(hi), "=&v"(lo)
        : "v"(x0), "v"(x1));
}
__device__ __forceinline__ void split2_relu_rtz_b(float x1, uint32_t &hi, uint32_t &lo) {
    asm("v_fma_mixhi_f16 %1, %2, 1.0, -%0 op_sel:[0,0,1] op_sel_hi:[0,0,1] clamp\n\t"
        "v_pk_max_f16 %0, %0, 0"
        : "+v"(hi), "+v"(lo)
        : "v"(x1));
}

// split2_relu_rtz as four single-instruction steps, for schedules that give
// every MFMA gap at most 8 issue cycles (tools/ubench/gapcost.hip: v_fma_mix*
// issue for 8 cycles, cvt / pk_max / fma for 4): C = hi (RTZ, before the
// relu), L = low word of lo, H = high word of lo (both read the pre-relu hi),
// P = the relu of hi (after L and H).  The caller keeps two instructions
// between P and the first MFMA that reads hi / lo.
__device__ __forceinline__ void split_c(float x0, float x1, uint32_t &hi) {
    asm("v_cvt_pkrtz_f16_f32 %0, %1, %2" : "=v"(hi) : "v"(x0), "v"(x1));
}
__device__ __forceinline__ void split_l(float x0, uint32_t hi, uint32_t &lo) {
    asm("v_fma_mixlo_f16 %0, %1, 1.0, -%2 op_sel_hi:[0,0,1] clamp" : "=&v"(lo) : "v"(x0), "v"(hi));
}
__device__ __forceinline__ void split_h(float x1, uint32_t hi, uint32_t &lo) {
    asm("v_fma_mixhi_f16 %0, %1, 1.0, -%2 op_sel:[0,0,1] op_sel_hi:[0,0,1] clamp" : "+v"(lo) : "v"(x1), "v"(hi));
}
__device__ __forceinline__ void split_p(uint32_t &hi) {
    asm("v_pk_max_f16 %0, %0, 0" : "+v"(hi));
}

__device__ __forceinline__ float absmax4(float m, const float4 &v) {
    return fmaxf(fmaxf(fmaxf(m, fabsf(v.x)), fmaxf(fabsf(v.y), fabsf(v.z))), fabsf(v.w));
}

__device__ __forceinline__ f32x4 mfma_f16(const half8 &a, const half8 &b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
}


}  // namespace
