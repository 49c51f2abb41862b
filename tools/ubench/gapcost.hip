// Price of VALU fillers beside v_mfma_f32_16x16x32_f16 at one wave per SIMD
// (profiling aid, not shipped): the edge kernel's MFMA-gap units, one kind per
// run, pinned one unit per MFMA gap by sched_barriers, against the bare MFMA
// stream.  64-thread workgroups, four per CU (one wave per SIMD), like the wave
// edge kernel.
//   hipcc --offload-arch=gfx950 -O3 gapcost.hip -o gapcost && ./gapcost
#include <hip/hip_runtime.h>
#include <cstdio>

typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

template <int F>
__device__ __forceinline__ void filler(float &x0, float &x1, float &y0, float &y1, uint32_t &h, uint32_t &l,
                                       float s) {
    if constexpr (F == 1) {  // 2 independent v_fma_f32
        asm volatile("v_fma_f32 %0, %2, %4, %0\n\tv_fma_f32 %1, %3, %4, %1" : "+v"(x0), "+v"(x1) : "v"(y0), "v"(y1), "v"(s));
    } else if constexpr (F == 2) {  // cvt_pkrtz + mixlo (dependent, production _a)
        asm volatile("v_cvt_pkrtz_f16_f32 %0, %2, %3\n\tv_fma_mixlo_f16 %1, %2, 1.0, -%0 op_sel_hi:[0,0,1] clamp"
                     : "=&v"(h), "+v"(l) : "v"(x0), "v"(x1));
    } else if constexpr (F == 3) {  // mixhi + pk_max (production _b)
        asm volatile("v_fma_mixhi_f16 %1, %2, 1.0, -%0 op_sel:[0,0,1] op_sel_hi:[0,0,1] clamp\n\tv_pk_max_f16 %0, %0, 0"
                     : "+v"(h), "+v"(l) : "v"(x1));
    } else if constexpr (F == 4) {  // relu-sum: max + add (dependent)
        float t;
        asm volatile("v_max_f32_e32 %1, 0, %2\n\tv_add_f32_e32 %0, %0, %1" : "+v"(x0), "=&v"(t) : "v"(y0));
    } else if constexpr (F == 5) {  // 1 v_fma_f32
        asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(x0) : "v"(y0), "v"(s));
    } else if constexpr (F == 6) {  // cvt_pkrtz alone
        asm volatile("v_cvt_pkrtz_f16_f32 %0, %1, %2" : "=v"(h) : "v"(y0), "v"(y1));
    } else if constexpr (F == 7) {  // fma_mixlo alone (independent of this gap)
        asm volatile("v_fma_mixlo_f16 %0, %1, 1.0, -%2 op_sel_hi:[0,0,1] clamp" : "+v"(l) : "v"(y0), "v"(h));
    } else if constexpr (F == 8) {  // pk_max_f16 alone
        asm volatile("v_pk_max_f16 %0, %0, 0" : "+v"(h));
    } else if constexpr (F == 9) {  // 3 independent v_fma_f32
        asm volatile("v_fma_f32 %0, %3, %5, %0\n\tv_fma_f32 %1, %4, %5, %1\n\tv_fma_f32 %2, %3, %5, %2"
                     : "+v"(x0), "+v"(x1), "+v"(y1) : "v"(y0), "v"(s), "v"(s));
    } else if constexpr (F == 10) {  // and + sub (dependent): an RTZ-11 split in fp32
        float t;
        asm volatile("v_and_b32 %1, 0xffffe000, %2\n\tv_sub_f32 %0, %2, %1" : "=v"(x0), "=&v"(t) : "v"(y0));
    } else if constexpr (F == 11) {  // 2 fmas, dependent chain
        asm volatile("v_fma_f32 %0, %1, %2, %0\n\tv_fma_f32 %0, %1, %2, %0" : "+v"(x0) : "v"(y0), "v"(s));
    } else if constexpr (F == 12) {  // cvt_pk_f16_f32 (RN) + cvt_pkrtz (independent)
        asm volatile("v_cvt_pk_f16_f32 %0, %2, %3\n\tv_cvt_pkrtz_f16_f32 %1, %3, %2" : "=v"(h), "=v"(l) : "v"(y0), "v"(y1));
    } else if constexpr (F == 13) {  // 2 fma_mix (independent of each other)
        asm volatile("v_fma_mixlo_f16 %0, %2, 1.0, -%3 op_sel_hi:[0,0,1] clamp\n\tv_fma_mixhi_f16 %1, %2, 1.0, -%3 op_sel:[0,0,1] op_sel_hi:[0,0,1] clamp"
                     : "+v"(l), "+v"(h) : "v"(y0), "v"(x1));
    } else if constexpr (F == 14) {  // v_pk_add_f16 + v_pk_mul_f16
        asm volatile("v_pk_add_f16 %0, %0, %1\n\tv_pk_mul_f16 %1, %1, %0" : "+v"(h), "+v"(l));
    }
}

// ROT: production-like rotation of units over 3-MFMA groups
template <int F, bool ROT>
__global__ __launch_bounds__(64, 1) void gap_kernel(const float4 *seed, int iters, float *out) {
    const int lane = threadIdx.x;
    const float4 s0 = seed[lane], s1 = seed[lane + 64];
    half8 a = __builtin_bit_cast(half8, s0), b = __builtin_bit_cast(half8, s1);
    f32x4 acc0 = {0, 0, 0, 0}, acc1 = {0, 0, 0, 0}, acc2 = {0, 0, 0, 0};
    float x0 = s0.x, x1 = s0.y, y0 = s1.x, y1 = s1.y, s = 1.0001f;
    uint32_t h = lane, l = lane + 1;
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            acc0 = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, acc0, 0, 0, 0);
            if (ROT) filler<4>(x0, x1, y0, y1, h, l, s);
            else filler<F>(x0, x1, y0, y1, h, l, s);
            __builtin_amdgcn_sched_barrier(0);
            acc1 = __builtin_amdgcn_mfma_f32_16x16x32_f16(b, a, acc1, 0, 0, 0);
            if (ROT) { if (j & 1) filler<3>(x0, x1, y0, y1, h, l, s); else filler<1>(x0, x1, y0, y1, h, l, s); }
            else filler<F>(x0, x1, y0, y1, h, l, s);
            __builtin_amdgcn_sched_barrier(0);
            acc2 = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, a, acc2, 0, 0, 0);
            if (ROT) { if (!(j & 1)) filler<2>(x0, x1, y0, y1, h, l, s); }
            else filler<F>(x0, x1, y0, y1, h, l, s);
            __builtin_amdgcn_sched_barrier(0);
        }
    }
    out[blockIdx.x * 64 + lane] = acc0[0] + acc1[1] + acc2[2] + x0 + x1 + y1 + (float)(h ^ l);
}

template <int F, bool ROT = false>
float run(const float4 *seed, float *out, int iters, int cus) {
    hipLaunchKernelGGL((gap_kernel<F, ROT>), dim3(4 * cus), dim3(64), 0, 0, seed, iters, out);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    hipEventRecord(a, 0);
    for (int i = 0; i < 5; ++i) hipLaunchKernelGGL((gap_kernel<F, ROT>), dim3(4 * cus), dim3(64), 0, 0, seed, iters, out);
    hipEventRecord(b, 0);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    return 1e3f * ms / 5;
}

int main() {
    int cus = 256, dev = 0;
    hipGetDevice(&dev);
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    float4 *seed;
    float *out;
    hipMalloc(&seed, 128 * 16);
    hipMemset(seed, 0x3c, 128 * 16);
    hipMalloc(&out, 4 * cus * 64 * 4);
    const int iters = 400;  // 9600 MFMAs per wave
    const double mf = 24.0 * iters;
    struct R { const char *name; float us; };
    for (int rep = 0; rep < 2; ++rep) {
        R rs[] = {{"bare MFMA", run<0>(seed, out, iters, cus)},
                  {"2 v_fma_f32 indep", run<1>(seed, out, iters, cus)},
                  {"cvt_pkrtz + mixlo (dep)", run<2>(seed, out, iters, cus)},
                  {"mixhi + pk_max_f16", run<3>(seed, out, iters, cus)},
                  {"relu-sum max + add (dep)", run<4>(seed, out, iters, cus)},
                  {"1 v_fma_f32", run<5>(seed, out, iters, cus)},
                  {"cvt_pkrtz", run<6>(seed, out, iters, cus)},
                  {"fma_mixlo", run<7>(seed, out, iters, cus)},
                  {"pk_max_f16", run<8>(seed, out, iters, cus)},
                  {"3 v_fma_f32 indep", run<9>(seed, out, iters, cus)},
                  {"and + sub (dep)", run<10>(seed, out, iters, cus)},
                  {"2 v_fma_f32 dep", run<11>(seed, out, iters, cus)},
                  {"cvt_pk + cvt_pkrtz", run<12>(seed, out, iters, cus)},
                  {"2 fma_mix", run<13>(seed, out, iters, cus)},
                  {"pk_add_f16 + pk_mul_f16", run<14>(seed, out, iters, cus)},
                  {"production rotation", run<0, true>(seed, out, iters, cus)}};
        const float base = rs[0].us;
        for (auto &r : rs)
            printf("%-28s %8.1f us  %+6.2f us  per-MFMA x%.3f\n", r.name, r.us, r.us - base, r.us / base);
        printf("(%.0f MFMAs per wave, bare = %.2f ns per MFMA)\n", mf, 1e3 * base / mf);
    }
    return 0;
}
