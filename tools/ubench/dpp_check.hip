// DPP / permlane reductions (common.hpp) against the __shfl_xor ones they
// replace, bitwise (profiling aid): wave_absmax, absmax_stride8 (values >= 0),
// wave_sum_full, wave_max_full and xor_lane_f<1..32> on random floats of both signs.
#include "../../mm-pde_amd/csrc/common.hpp"
#include <cstdio>
#include <cstring>
#include <random>
#include <vector>
constexpr int NV = 14;
__global__ void k(const float *x, float *o) {
    const int lane = threadIdx.x & 63;
    const float v = x[blockIdx.x * 64 + lane];
    const float av = fabsf(v);
    float m = av;
    m = fmaxf(m, __shfl_xor(m, 8, 64));
    m = fmaxf(m, __shfl_xor(m, 16, 64));
    m = fmaxf(m, __shfl_xor(m, 32, 64));
    float *p = o + (blockIdx.x * 64 + lane) * NV;
    p[0] = wave_max(av);
    p[1] = wave_absmax(av);
    p[2] = m;
    p[3] = absmax_stride8(av);
    p[4] = wave_sum(v);
    p[5] = wave_sum_full(v);
    p[6] = wave_max(v);
    p[7] = wave_max_full(v);
    p[8] = __shfl_xor(v, 4, 64);
    p[9] = xor_lane_f<4>(v);
    p[10] = __shfl_xor(v, 16, 64);
    p[11] = xor_lane_f<16>(v);
    p[12] = __shfl_xor(v, 1, 64) + __shfl_xor(v, 2, 64) + __shfl_xor(v, 8, 64) + __shfl_xor(v, 32, 64);
    p[13] = xor_lane_f<1>(v) + xor_lane_f<2>(v) + xor_lane_f<8>(v) + xor_lane_f<32>(v);
}
int main() {
    const int B = 64;
    std::vector<float> h(B * 64), o(B * 64 * NV);
    std::mt19937 rng(3);
    for (auto &v : h) v = std::uniform_real_distribution<float>(-1, 1)(rng) * std::exp2(rng() % 20 - 10.0f);
    float *dx, *dout;
    if (hipMalloc(&dx, h.size() * 4) != hipSuccess || hipMalloc(&dout, o.size() * 4) != hipSuccess) return 1;
    if (hipMemcpy(dx, h.data(), h.size() * 4, hipMemcpyHostToDevice) != hipSuccess) return 1;
    hipLaunchKernelGGL(k, dim3(B), dim3(64), 0, 0, dx, dout);
    if (hipMemcpy(o.data(), dout, o.size() * 4, hipMemcpyDeviceToHost) != hipSuccess) return 1;
    int bad[7] = {0};
    for (int i = 0; i < B * 64; ++i)
        for (int t = 0; t < 7; ++t) bad[t] += memcmp(&o[NV * i + 2 * t], &o[NV * i + 2 * t + 1], 4) != 0;
    printf("bitwise mismatches of %d lanes: wave_absmax %d, absmax_stride8 %d, wave_sum_full %d, "
           "wave_max_full %d, xor4 %d, xor16 %d, xor1/2/8/32 %d\n",
           B * 64, bad[0], bad[1], bad[2], bad[3], bad[4], bad[5], bad[6]);
    int tot = 0;
    for (int t = 0; t < 7; ++t) tot += bad[t];
    return tot ? 2 : 0;
}
