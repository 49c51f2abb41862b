#include <cmath>
// Timing of the layer kernels (profiling aid, not shipped): edge stage and
// node stage variants on a cylinder-sized synthetic layer (n = B x 2521 rows,
// k = 35 in-trajectory neighbours), both arithmetic modes.
//   make -C tools/ubench && tools/ubench/fused_ubench [B] [random|local|self]
#include "../../mm-pde_amd/csrc/gnn.hip"
#include "../../mm-pde_amd/csrc/layer.hip"
#include <algorithm>
#include <cstdio>
#include <cstring>
#include <random>
#include <vector>


#define CK(x)                                                                     \
    do {                                                                          \
        hipError_t e_ = (x);                                                      \
        if (e_ != hipSuccess) {                                                   \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            return 1;                                                             \
        }                                                                         \
    } while (0)

static float *dev_random(size_t count, float lo, float hi, std::mt19937 &rng) {
    std::uniform_real_distribution<float> d(lo, hi);
    std::vector<float> h(count);
    for (auto &v : h) v = d(rng);
    float *p = nullptr;
    if (hipMalloc(&p, count * 4) != hipSuccess) return nullptr;
    hipMemcpy(p, h.data(), count * 4, hipMemcpyHostToDevice);
    return p;
}

// Ceiling check: the edge loop's MFMA count (v_mfma_f32_16x16x32_f16, 2
// accumulators, 12 per chain link) with register operands only.
__global__ __launch_bounds__(256, 2) void mfma_only_kernel(const float4 *seed, int iters, float4 *out) {
    const int lane = threadIdx.x & 63;
    const float4 s0 = seed[lane], s1 = seed[lane + 64];
    half8 a = *(const half8 *)&s0, b = *(const half8 *)&s1;
    f32x4 acc0 = {0, 0, 0, 0}, acc1 = {0, 0, 0, 0};
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int j = 0; j < 12; ++j) {
            acc0 = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, acc0, 0, 0, 0);
            acc1 = __builtin_amdgcn_mfma_f32_16x16x32_f16(b, a, acc1, 0, 0, 0);
        }
    }
    out[blockIdx.x * 256 + threadIdx.x] = make_float4(acc0[0] + acc1[0], acc0[1], acc0[2], acc1[3]);
}

template <class F>
static float time_it(F launch, int iters) {
    for (int i = 0; i < 3; ++i) launch();
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    hipEventRecord(a, 0);
    for (int i = 0; i < iters; ++i) launch();
    hipEventRecord(b, 0);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    hipEventDestroy(a);
    hipEventDestroy(b);
    return 1e3f * ms / iters;
}

int main(int argc, char **argv) {
    const int B = argc > 1 ? atoi(argv[1]) : 16, N = 2521, k = 35;
    const int64_t n = (int64_t)B * N;
    std::mt19937 rng(1);
    float *a = dev_random(n * H, -1, 1, rng), *b = dev_random(n * H, -1, 1, rng);
    float *h = dev_random(n * H, -1, 1, rng), *u = dev_random(n, -1, 1, rng);
    float *pos = dev_random(n * 3, 0, 1, rng);
    float *w1 = dev_random(128 * 260, -0.06f, 0.06f, rng), *b1 = dev_random(128, -0.06f, 0.06f, rng);
    float *w2 = dev_random(128 * 128, -0.09f, 0.09f, rng), *b2 = dev_random(128, -0.09f, 0.09f, rng);
    float *u1 = dev_random(128 * 260, -0.06f, 0.06f, rng), *c1 = dev_random(128, -0.06f, 0.06f, rng);
    float *u2 = dev_random(128 * 128, -0.09f, 0.09f, rng), *c2 = dev_random(128, -0.09f, 0.09f, rng);
    float *bnw = dev_random(128, 0.5f, 1.5f, rng), *bnb = dev_random(128, -0.1f, 0.1f, rng);
    float *bnm = dev_random(128, -0.1f, 0.1f, rng), *bnv = dev_random(128, 0.5f, 1.5f, rng);
    std::vector<int32_t> hn(n * k);
    std::uniform_int_distribution<int> di(0, N - 1);
    // argv[2]: "random" (default, in-trajectory random rows), "local" (rows of
    // the same 16-row tile: gathers hit L1/L2), "self" (every edge = the target)
    const char *pat = argc > 2 ? argv[2] : "random";
    for (int64_t i = 0; i < n; ++i)
        for (int e = 0; e < k; ++e) {
            int64_t src = (i / N) * N + di(rng);
            if (!strcmp(pat, "local")) src = std::min<int64_t>(n - 1, (i / 16) * 16 + (e % 16));
            if (!strcmp(pat, "self")) src = i;
            hn[i * k + e] = (int32_t)src;
        }
    printf("neighbour pattern: %s\n", pat);
    int32_t *nbr;
    CK(hipMalloc(&nbr, n * k * 4));
    CK(hipMemcpy(nbr, hn.data(), n * k * 4, hipMemcpyHostToDevice));
    float *ho, *ao, *bo;
    CK(hipMalloc(&ho, n * H * 4));
    CK(hipMalloc(&ao, n * H * 4));
    CK(hipMalloc(&bo, n * H * 4));
    mmpde_gnn_layer_params lp{w1, b1, w2, b2, u1, c1, u2, c2, bnw, bnb, bnm, bnv, 1e-5f, 260, 260};
    mmpde_gnn_layer_params two[2] = {lp, lp};
    char *pack;
    CK(hipMalloc(&pack, mmpde_gnn_pack_bytes(2)));
    if (mmpde_gnn_pack_f16x3(two, 2, pack, 0) != 0) return 1;
    CK(hipDeviceSynchronize());
    mmpde_gnn_scales sc{1.0f, 1.0f, 1.0f / 2.9f};
    uint32_t *amax;
    CK(hipMalloc(&amax, 4 * 2 * kAmaxShards * 4));
    {   // range slots: |a|, |b| <= 1 for the uniform [-1, 1) inputs
        std::vector<uint32_t> hs(4 * 2 * kAmaxShards, 0x3f800000u);
        CK(hipMemcpy(amax, hs.data(), hs.size() * 4, hipMemcpyHostToDevice));
    }
    float *mean;
    CK(hipMalloc(&mean, 2 * n * H * 4));
    const int it = 20;
    EdgeSplit split;
    const int64_t ntiles = (n + ET - 1) / ET;
    int cus = device_cus();
    const int grid_e = ntiles < cus ? (int)ntiles : cus;
    uint64_t *stamps;
    CK(hipMalloc(&stamps, (12 * 2 * 256 + 4) * 8));
    CK(hipMemset(stamps, 0, (12 * 2 * 256 + 4) * 8));
    EdgeArgs e32{a, b, nbr, n, k, (int)ntiles, w2, b2, nullptr, nullptr, mean, stamps};
    EdgeArgs e16{a, b, nbr, n, k, (int)ntiles, w2, b2, pack, amax, mean, stamps};
    NodeArgs nd{h, mean, n, u1, c1, 260, u2, c2, bnw, bnb, bnm, bnv, 1e-5f, ho, w1, b1, 260, ao, bo,
                u, pos, sc, pack, pack + kLayerPack, amax + 2 * kAmaxShards, 1, 0};
    printf("n=%lld k=%d  (us per launch)\n", (long long)n, k);
    auto edge = [&](auto kern, int nw, const EdgeArgs &ea) {
        return time_it([&] { hipLaunchKernelGGL(kern, dim3(grid_e), dim3(64 * nw), 0, 0, ea); }, it);
    };
    {   // variants interleaved over several repetitions (the clock drifts between
        // launches and devices differ): median per variant
        struct V { const char *name; void (*k)(EdgeArgs); const EdgeArgs *a; };
        V vs[] = {
            {"ring kernel f16x3 (PH 27)", gnn_edge_kernel<true, 27, 2, 1>, &e16},
            {"consume-only", gnn_edge_kernel<true, 26, 2, 1>, &e16},
            {"produce-only", gnn_edge_kernel<true, 25, 2, 1>, &e16},
            {"no-gather", gnn_edge_kernel<true, 31, 2, 1>, &e16},
            {"cvt-only producer", gnn_edge_kernel<true, 27 + 32, 2, 1>, &e16},
            {"quarter ring stores", gnn_edge_kernel<true, 27 + 64, 2, 1>, &e16},
            {"prio: producers 2 > consumers 1", gnn_edge_kernel<true, 27 + 2048, 2, 1>, &e16},
            {"prio: producers 2, consumers 0", gnn_edge_kernel<true, 19 + 2048, 2, 1>, &e16},
            {"prio: none", gnn_edge_kernel<true, 19, 2, 1>, &e16},
        };
        const int nv = sizeof(vs) / sizeof(vs[0]), reps = 7;
        std::vector<std::vector<float>> t(nv);
        std::vector<float> tw1, tw2;
        for (int r = 0; r < reps; ++r) {
            for (int v = 0; v < nv; ++v) t[v].push_back(edge(vs[v].k, 12, *vs[v].a));
            tw1.push_back(time_it([&] { launch_edge_wave(a, b, nbr, nullptr, n, k, b2, pack, amax, mean, mean + n * H, n / 16, cus, &split, 0); }, it));
            tw2.push_back(tw1.back());
        }
        std::sort(tw1.begin(), tw1.end());
        std::sort(tw2.begin(), tw2.end());
        printf("edge %-34s median %6.1f  min %6.1f  max %6.1f us\n", "wave kernel", tw1[reps / 2], tw1[0], tw1[reps - 1]);
        {   // wave kernel (parts 1) vs ring kernel: same per-slot arithmetic
            std::vector<float> m0(n * H), m1(n * H);
            hipLaunchKernelGGL((gnn_edge_kernel<true, 27, 2, 1>), dim3(grid_e), dim3(768), 0, 0, e16);
            CK(hipMemcpy(m0.data(), mean, n * H * 4, hipMemcpyDeviceToHost));
            if (launch_edge_wave(a, b, nbr, nullptr, n, k, b2, pack, amax, mean, mean + n * H, n / 16, cus, &split, 0)) return 1;
            CK(hipMemcpy(m1.data(), mean, n * H * 4, hipMemcpyDeviceToHost));
            double d = 0, mx = 0;
            for (size_t i = 0; i < m0.size(); ++i) {  // the wave kernel stores sums (side blocks not added)
                d = std::max(d, (double)std::fabs(m0[i] - m1[i] / k));
                mx = std::max(mx, (double)std::fabs(m0[i]));
            }
            printf("wave vs ring kernel: max|diff| %.3e (max|mean| %.3e)\n", d, mx);
        }
        for (int v = 0; v < nv; ++v) {
            std::sort(t[v].begin(), t[v].end());
            printf("edge %-34s median %6.1f  min %6.1f  max %6.1f us\n", vs[v].name, t[v][reps / 2], t[v][0],
                   t[v][reps - 1]);
        }
    }
    {   // slot-split vs column-split consumers: same sums, same order per target
        std::vector<float> m0(n * H), m1(n * H);
        hipLaunchKernelGGL((gnn_edge_kernel<true, 11, 2, 1>), dim3(grid_e), dim3(768), 0, 0, e16);
        CK(hipMemcpy(m0.data(), mean, n * H * 4, hipMemcpyDeviceToHost));
        hipLaunchKernelGGL((gnn_edge_kernel<true, 27, 2, 1>), dim3(grid_e), dim3(768), 0, 0, e16);
        CK(hipMemcpy(m1.data(), mean, n * H * 4, hipMemcpyDeviceToHost));
        double d = 0, mx = 0;
        for (size_t i = 0; i < m0.size(); ++i) {
            d = std::max(d, (double)std::fabs(m0[i] - m1[i]));
            mx = std::max(mx, (double)std::fabs(m0[i]));
        }
        printf("slot-split vs column-split: max|diff| %.3e (max|mean| %.3e)\n", d, mx);
    }
    {   // shader clock of the consume-only variant (ring operands never written)
        hipLaunchKernelGGL((gnn_edge_kernel<true, 1024 + 26, 2, 1>), dim3(grid_e), dim3(768), 0, 0, e16);
        CK(hipDeviceSynchronize());
        std::vector<uint64_t> c(4);
        CK(hipMemcpy(c.data(), stamps + 12 * 2 * 256, 4 * 8, hipMemcpyDeviceToHost));
        const double dr = (double)(c[3] - c[1]);
        printf("consume-only shader clock: %.0f MHz over %.1f us\n",
               dr > 0 ? 100.0 * (double)(c[2] - c[0]) / dr : 0.0, dr / 100.0);
        fflush(stdout);
    }
    {   // per-round barrier arrival / release times of block 0 (waves 0..7, lane 0)
        hipLaunchKernelGGL((gnn_edge_kernel<true, 1024 + 27, 2, 1>), dim3(grid_e), dim3(768), 0, 0, e16);
        CK(hipDeviceSynchronize());
        std::vector<uint64_t> st(12 * 2 * 256 + 4);
        CK(hipMemcpy(st.data(), stamps, st.size() * 8, hipMemcpyDeviceToHost));
        {
            const double dt = (double)(st[12 * 2 * 256 + 2] - st[12 * 2 * 256]);
            const double dr = (double)(st[12 * 2 * 256 + 3] - st[12 * 2 * 256 + 1]);
            printf("edge kernel shader clock (block 0, s_memtime / s_memrealtime at 100 MHz): %.0f MHz over %.1f us\n",
                   dr > 0 ? 100.0 * dt / dr : 0.0, dr / 100.0);
        }
        printf("round stamps (s_memtime, relative): it | arrive c0 c1 c2 c3 p0 p1 p2 p3 | release c0\n");
        const uint64_t t0 = st[0];
        for (int i = 0; i < 40; ++i) {
            printf("%3d |", i);
            for (int w : {0, 1, 2, 3, 4, 5, 8, 9}) printf(" %7lld", (long long)(st[2 * 256 * w + 2 * i] - t0));
            printf(" | %7lld\n", (long long)(st[2 * i + 1] - t0));
        }
    }
    printf("node f16x3 RB4 %.1f  RB2 %.1f  (last layer RB4 %.1f)  f32 RB4 %.1f\n",
           time_it([&] { hipLaunchKernelGGL((gnn_node_kernel<true, true, 4>), dim3(ceil_div(n, 64)), dim3(512), 0, 0, nd); }, it),
           time_it([&] { hipLaunchKernelGGL((gnn_node_kernel<true, true, 2>), dim3(ceil_div(n, 32)), dim3(512), 0, 0, nd); }, it),
           time_it([&] { hipLaunchKernelGGL((gnn_node_kernel<false, true, 4>), dim3(ceil_div(n, 64)), dim3(512), 0, 0, nd); }, it),
           time_it([&] { hipLaunchKernelGGL((gnn_node_kernel<true, false, 4>), dim3(ceil_div(n, 64)), dim3(512), 0, 0, nd); }, it));
    {   // MFMA ceiling: the edge stage's MFMA count (16 x 16 x 32 f16), register operands
        float4 *seed, *out;
        const int nb = (int)ntiles;
        CK(hipMalloc(&seed, 128 * 16));
        CK(hipMemset(seed, 0x3c, 128 * 16));
        CK(hipMalloc(&out, (size_t)nb * 256 * 16));
        const int iters = 9 * 96 / 24;
        printf("mfma-only ceiling (edge MFMA count, register operands, 2 waves/SIMD): %.1f us\n",
               time_it([&] { hipLaunchKernelGGL(mfma_only_kernel, dim3(nb), dim3(256), 0, 0, seed, iters, out); }, it));
    }
    CK(hipGetLastError());
    return 0;
}
