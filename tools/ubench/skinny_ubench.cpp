// Timing of linear_skinny_kernel variants on the rollout's shapes (profiling aid).
#include "../../mm-pde_amd/csrc/dense.hip"

#include <cstdio>
#include <vector>

template <int W>
static float run(const float *x, const float *w, float *y, int m, int k, int n, int it) {
    dim3 grid((n + 15) / 16, (m + 15) / 16);
    for (int i = 0; i < 3; ++i) hipLaunchKernelGGL(linear_skinny_kernel<W>, grid, dim3(W * 64), 0, 0, x, (int64_t)k, (int64_t)m, (int64_t)k, w, (int64_t)k, (const float *)nullptr, (int64_t)n, 0, y, (int64_t)n);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    hipEventRecord(a, 0);
    for (int i = 0; i < it; ++i) hipLaunchKernelGGL(linear_skinny_kernel<W>, grid, dim3(W * 64), 0, 0, x, (int64_t)k, (int64_t)m, (int64_t)k, w, (int64_t)k, (const float *)nullptr, (int64_t)n, 0, y, (int64_t)n);
    hipEventRecord(b, 0);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    return 1e3f * ms / it;
}

__global__ void empty_kernel() {}

int main() {
    const int shapes[][3] = {{16, 2521, 2048}, {16, 2048, 512}, {16, 512, 2048}, {16, 2048, 2521},
                             {16, 2521, 512}, {16, 512, 256}, {16, 256, 512}, {16, 512, 512}};
    float *x, *w, *y;
    hipMalloc(&x, 16 * 4096 * 4);
    hipMalloc(&w, 4096 * 4096 * 4);
    hipMalloc(&y, 16 * 4096 * 4);
    hipMemset(x, 0, 16 * 4096 * 4);
    hipMemset(w, 0, 4096 * 4096 * 4);
    {
        hipEvent_t a, b;
        hipEventCreate(&a);
        hipEventCreate(&b);
        hipEventRecord(a, 0);
        for (int i = 0; i < 100; ++i) hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, 0);
        hipEventRecord(b, 0);
        hipEventSynchronize(b);
        float ms;
        hipEventElapsedTime(&ms, a, b);
        printf("empty kernel: %.2f us\n", 1e3f * ms / 100);
    }
    for (auto &s : shapes) {
        const int m = s[0], k = s[1], n = s[2];
        printf("m=%d k=%d n=%d  W4 %.1f  W8 %.1f  W16 %.1f us  (%.2f MB)\n", m, k, n, run<4>(x, w, y, m, k, n, 20),
               run<8>(x, w, y, m, k, n, 20), run<16>(x, w, y, m, k, n, 20), k * n * 4e-6);
    }
    printf("err: %s\n", hipGetErrorString(hipGetLastError()));
    return 0;
}
