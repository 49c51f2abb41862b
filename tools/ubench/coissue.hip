// MFMA / VALU co-issue probe (profiling aid): one 512-thread workgroup per CU,
// waves 0-3 run a v_mfma_f32_16x16x32_f16 stream (2 accumulator chains), waves
// 4-7 (same SIMDs: waves w and w + 4 share one) run a VALU stream of the edge
// producer's instruction mix.  Reports how long each stream takes alone and
// together.
#include <hip/hip_runtime.h>
#include <cstdio>

typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

typedef float f32x16 __attribute__((ext_vector_type(16)));

template <int MODE>  // bit 0: MFMA waves work, bit 1: VALU waves work, bit 2: VALU waves use fma_mix,
                     // bit 3: the MFMA stream is v_mfma_f32_32x32x16_f16 (same MAC count)
__global__ __launch_bounds__(512, 1) void probe(float *out, int iters) {
    const int wave = threadIdx.x >> 6;
    float r = 0.0f;
    if (wave < 4) {
        if (MODE & 1) {
            half8 a, b;
            for (int i = 0; i < 8; ++i) {
                a[i] = (_Float16)(threadIdx.x * 1e-3f + i);
                b[i] = (_Float16)(1.0f / (i + 1));
            }
            if (MODE & 8) {
                f32x16 c0 = {}, c1 = {};
                for (int it = 0; it < iters; ++it) {
#pragma unroll
                    for (int j = 0; j < 6; ++j) {
                        c0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c0, 0, 0, 0);
                        c1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(b, a, c1, 0, 0, 0);
                    }
                }
                r = c0[0] + c1[1];
            } else {
                f32x4 c0 = {0, 0, 0, 0}, c1 = {0, 0, 0, 0};
                for (int it = 0; it < iters; ++it) {
#pragma unroll
                    for (int j = 0; j < 12; ++j) {
                        c0 = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c0, 0, 0, 0);
                        c1 = __builtin_amdgcn_mfma_f32_16x16x32_f16(b, a, c1, 0, 0, 0);
                    }
                }
                r = c0[0] + c1[1];
            }
        }
    } else if (MODE & 2) {
        float x0 = threadIdx.x * 1e-3f, x1 = x0 + 1, x2 = x0 + 2, x3 = x0 + 3, s = 1.0001f;
        uint32_t h = 0, l = 0;
        for (int it = 0; it < iters; ++it) {
#pragma unroll
            for (int j = 0; j < 6; ++j) {
                // per element: fma + max, per pair: cvt_pk, per element: fma_mix (or a sub)
                x0 = fmaxf(fmaf(x0, s, 0.5f), 0.0f);
                x1 = fmaxf(fmaf(x1, s, 0.5f), 0.0f);
                x2 = fmaxf(fmaf(x2, s, 0.5f), 0.0f);
                x3 = fmaxf(fmaf(x3, s, 0.5f), 0.0f);
                if (MODE & 4) {
                    asm volatile("v_cvt_pk_f16_f32 %0, %2, %3\n\t"
                                 "v_fma_mixlo_f16 %1, %2, 1.0, -%0 op_sel_hi:[0,0,1]\n\t"
                                 "v_fma_mixhi_f16 %1, %3, 1.0, -%0 op_sel:[0,0,1] op_sel_hi:[0,0,1]\n\t"
                                 : "=&v"(h), "=&v"(l) : "v"(x0), "v"(x1));
                } else {
                    asm volatile("v_cvt_pk_f16_f32 %0, %2, %3\n\t"
                                 "v_add_f32 %1, %2, %3\n\t"
                                 : "=&v"(h), "=&v"(l) : "v"(x0), "v"(x1));
                }
                x0 += __uint_as_float(h & 0x3ff) * 1e-30f;
                x2 += __uint_as_float(l & 0x3ff) * 1e-30f;
            }
        }
        r = x0 + x1 + x2 + x3;
    }
    out[blockIdx.x * 512 + threadIdx.x] = r;
}

template <int MODE>
float run(float *out, int iters) {
    hipLaunchKernelGGL(probe<MODE>, dim3(256), dim3(512), 0, 0, out, iters);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    hipEventRecord(a, 0);
    for (int i = 0; i < 5; ++i) hipLaunchKernelGGL(probe<MODE>, dim3(256), dim3(512), 0, 0, out, iters);
    hipEventRecord(b, 0);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    return 1e3f * ms / 5;
}

int main() {
    float *out;
    hipMalloc(&out, 256 * 512 * 4);
    const int iters = 4000;
    printf("us: mfma alone %.1f | valu alone %.1f (mix %.1f) | both %.1f (mix %.1f)\n", run<1>(out, iters),
           run<2>(out, iters), run<6>(out, iters), run<3>(out, iters), run<7>(out, iters));
    printf("32x32x16: mfma alone %.1f | both %.1f (mix %.1f)\n", run<9>(out, iters), run<11>(out, iters),
           run<15>(out, iters));
    return 0;
}
