// VALU issue-rate probe (profiling aid): cycles per instruction of the
// producer's instruction kinds, one wave per SIMD and two waves per SIMD.
#include <hip/hip_runtime.h>
#include <cstdio>

#define REP8(x) x x x x x x x x
#define REP64(x) REP8(REP8(x))

template <int KIND>
__global__ void probe(float *out, int iters) {
    float a = threadIdx.x * 1e-3f, b = 1.0001f, c = 0.5f, d = 0.25f;
    uint32_t hv = 0x3c003c00u, lv = 0;
    const long long t0 = clock64();
    for (int i = 0; i < iters; ++i) {
        if (KIND == 0) asm volatile(REP64("v_fma_f32 %0, %1, %2, %0\n") : "+v"(a) : "v"(b), "v"(c));
        if (KIND == 1) asm volatile(REP64("v_fma_mixlo_f16 %0, %1, 1.0, -%2 op_sel_hi:[0,0,1]\n") : "+v"(lv) : "v"(a), "v"(hv));
        if (KIND == 2) asm volatile(REP64("v_cvt_pk_f16_f32 %0, %1, %2\n") : "=v"(hv) : "v"(a), "v"(b));
        if (KIND == 3) asm volatile(REP64("v_max_f32 %0, %1, %0\n") : "+v"(a) : "v"(d));
        if (KIND == 4) {  // 8 independent chains of fma
            asm volatile(REP8("v_fma_f32 %0, %4, %5, %0\n v_fma_f32 %1, %4, %5, %1\n v_fma_f32 %2, %4, %5, %2\n v_fma_f32 %3, %4, %5, %3\n")
                         : "+v"(a), "+v"(b), "+v"(c), "+v"(d) : "v"(b), "v"(c));
        }
    }
    const long long t1 = clock64();
    if (threadIdx.x == 0 && blockIdx.x == 0) out[0] = (float)(t1 - t0);
    out[1 + blockIdx.x * blockDim.x + threadIdx.x] = a + b + c + d + __uint_as_float(hv + lv);
}

template <int KIND>
void run(const char *name, int threads, int n_instr_per_iter) {
    float *out;
    hipMalloc(&out, (1 + 256 * 1024) * 4);
    const int iters = 1000;
    hipLaunchKernelGGL(probe<KIND>, dim3(256), dim3(threads), 0, 0, out, iters);
    hipDeviceSynchronize();
    float cyc;
    hipMemcpy(&cyc, out, 4, hipMemcpyDeviceToHost);
    printf("%-28s threads/WG %4d: %.2f cycles per instruction (wave 0)\n", name, threads, cyc / (iters * (double)n_instr_per_iter));
    hipFree(out);
}

int main() {
    for (int th : {256, 512}) {
        run<0>("v_fma_f32 (dep chain)", th, 64);
        run<4>("v_fma_f32 (4 chains)", th, 32);
        run<1>("v_fma_mixlo_f16", th, 64);
        run<2>("v_cvt_pk_f16_f32", th, 64);
        run<3>("v_max_f32 (dep chain)", th, 64);
    }
    return 0;
}
