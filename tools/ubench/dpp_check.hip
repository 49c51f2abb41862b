// DPP / permlane max reductions (common.hpp) against __shfl_xor ones (profiling aid)
#include "../../mm-pde_amd/csrc/common.hpp"
#include <cstdio>
#include <random>
#include <vector>
__global__ void k(const float *x, float *o) {
    const int lane = threadIdx.x & 63;
    const float v = x[blockIdx.x * 64 + lane];  // >= 0
    float a = wave_max(v), b = wave_absmax(v);
    float m = v;
    m = fmaxf(m, __shfl_xor(m, 8, 64));
    m = fmaxf(m, __shfl_xor(m, 16, 64));
    m = fmaxf(m, __shfl_xor(m, 32, 64));
    const float c = absmax_stride8(v);
    float *p = o + (blockIdx.x * 64 + lane) * 4;
    p[0] = a; p[1] = b; p[2] = m; p[3] = c;
}
int main() {
    const int B = 64;
    std::vector<float> h(B * 64), o(B * 256);
    std::mt19937 rng(3);
    for (auto &v : h) v = std::uniform_real_distribution<float>(0, 1)(rng);
    float *dx, *dout;
    hipMalloc(&dx, h.size() * 4);
    hipMalloc(&dout, o.size() * 4);
    hipMemcpy(dx, h.data(), h.size() * 4, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k, dim3(B), dim3(64), 0, 0, dx, dout);
    hipMemcpy(o.data(), dout, o.size() * 4, hipMemcpyDeviceToHost);
    int bad1 = 0, bad2 = 0;
    for (int i = 0; i < B * 64; ++i) {
        bad1 += o[4 * i] != o[4 * i + 1];
        bad2 += o[4 * i + 2] != o[4 * i + 3];
        if (i < 20 && (o[4 * i + 2] != o[4 * i + 3]))
            printf("lane %d: shfl %.6f dpp %.6f (x %.6f)\n", i, o[4 * i + 2], o[4 * i + 3], h[i]);
    }
    printf("wave max mismatches %d, part max mismatches %d of %d\n", bad1, bad2, B * 64);
    return 0;
}
