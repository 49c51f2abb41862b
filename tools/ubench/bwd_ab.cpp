// Edge-stage backward timing (profiling aid, not shipped): the fp16x3
// backward (edge_bwd_f16_kernel) at cy B=16 size (40336 targets, k = 35 random
// in-trajectory neighbours), target-major (mmpde_gnn_edge_backward_ex) and
// source-major (mmpde_gnn_edge_backward_sorted, slot positions from
// mmpde_reverse_adjacency), plus the two source sums.  Built per variant of
// the kernel's compile-time placement flags (Makefile bwd_ab_%).
//   make -C tools/ubench bwd_ab_base && tools/ubench/bwd_ab_base
// BWD_SRC: another edge_bwd.hip for a same-box A/B (built with -I mm-pde_amd/csrc)
#ifndef BWD_SRC
#define BWD_SRC "../../mm-pde_amd/csrc/edge_bwd.hip"
#endif
#include BWD_SRC
#include "../../mm-pde_amd/csrc/train_rows.hip"
#include <cstdio>
#include <random>
#include <vector>

#define CK(x)                                                                         \
    do {                                                                              \
        auto e_ = (x);                                                                \
        if (e_ != 0) {                                                                \
            fprintf(stderr, "%s:%d status %d\n", __FILE__, __LINE__, (int)e_);        \
            return 1;                                                                 \
        }                                                                             \
    } while (0)

template <class T>
static T *dev_copy(const std::vector<T> &h) {
    T *p = nullptr;
    if (hipMalloc(&p, h.size() * sizeof(T)) != hipSuccess) return nullptr;
    hipMemcpy(p, h.data(), h.size() * sizeof(T), hipMemcpyHostToDevice);
    return p;
}

int main() {
    const int B = 16, N = 2521, K = 35;
    const int64_t n = (int64_t)B * N;
    std::mt19937 rng(7);
    std::normal_distribution<float> nd(0.0f, 1.0f);
    std::vector<float> a(n * 128), b(n * 128), g(n * 128), w2(128 * 128), b2(128);
    for (auto &v : a) v = 0.5f * nd(rng);
    for (auto &v : b) v = 0.5f * nd(rng);
    for (auto &v : g) v = nd(rng);
    for (auto &v : w2) v = nd(rng) / 11.3f;
    for (auto &v : b2) v = 0.1f * nd(rng);
    std::vector<int32_t> nb(n * K);
    for (int64_t i = 0; i < n; ++i)
        for (int e = 0; e < K; ++e) nb[i * K + e] = (int32_t)(i / N * N + rng() % N);
    float *da = dev_copy(a), *db = dev_copy(b), *dg = dev_copy(g), *dw2 = dev_copy(w2), *db2 = dev_copy(b2);
    int32_t *dnb = dev_copy(nb);
    float *ga, *gb, *ge, *part, *gw2, *gb2;
    CK(hipMalloc(&ga, n * 512));
    CK(hipMalloc(&gb, n * 512));
    CK(hipMalloc(&ge, n * K * 512));
    CK(hipMalloc(&part, mmpde_gnn_edge_backward_partials(nullptr) * 4));
    CK(hipMalloc(&gw2, 128 * 128 * 4));
    CK(hipMalloc(&gb2, 128 * 4));
    int64_t *off, *edge;
    int32_t *pos, *bad;
    CK(hipMalloc(&off, (n + 1) * 8));
    CK(hipMalloc(&edge, n * K * 8));
    CK(hipMalloc(&pos, n * K * 4));
    CK(hipMalloc(&bad, 4));
    const int64_t sb = mmpde_reverse_adjacency_scratch_bytes(n, K, n);
    void *scratch;
    CK(hipMalloc(&scratch, sb));
    // relu mask (timing only: a fixed pattern, about half the bits set)
    uint32_t *mask;
    CK(hipMalloc(&mask, n * K * 16));
    CK(hipMemset(mask, 0x5a, n * K * 16));
    CK(mmpde_reverse_adjacency(dnb, n, K, nullptr, n, off, edge, pos, scratch, sb, bad, nullptr));
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    auto timed = [&](const char *what, auto fn) {
        for (int i = 0; i < 3; ++i) fn();
        hipEventRecord(e0, 0);
        const int it = 10;
        for (int i = 0; i < it; ++i) fn();
        hipEventRecord(e1, 0);
        hipEventSynchronize(e1);
        float ms = 0;
        hipEventElapsedTime(&ms, e0, e1);
        printf("  %-44s %8.1f us\n", what, 1e3 * ms / it);
    };
    printf("edge backward, n=%lld k=%d, P1_FIRST=%d\n", (long long)n, K, (int)kBwdP1First);
    timed("backward_ex f16x3 (target-major rows)", [&] {
        mmpde_gnn_edge_backward_ex(da, db, dnb, nullptr, n, K, dw2, db2, dg, ga, ge, part, gw2, gb2, 1, nullptr);
    });
    timed("source_sum (gather)", [&] { mmpde_gnn_edge_source_sum(ge, off, edge, n, gb, nullptr); });
    timed("backward_sorted f16x3 (source-major rows)", [&] {
        mmpde_gnn_edge_backward_sorted(da, db, dnb, nullptr, n, K, dw2, db2, dg, pos, nullptr, ga, ge, part, gw2,
                                       gb2, 1, nullptr);
    });
    timed("backward_sorted f16x3 + forward relu mask", [&] {
        mmpde_gnn_edge_backward_sorted(da, db, dnb, nullptr, n, K, dw2, db2, dg, pos, mask, ga, ge, part, gw2, gb2,
                                       1, nullptr);
    });
    {   // output hash of the masked sorted backward (variants must match bit for bit)
        CK(mmpde_gnn_edge_backward_sorted(da, db, dnb, nullptr, n, K, dw2, db2, dg, pos, mask, ga, ge, part, gw2,
                                          gb2, 1, nullptr));
        CK(hipDeviceSynchronize());
        uint64_t h = 1469598103934665603ull;
        auto mix = [&](const float *d, size_t cnt) {
            std::vector<uint32_t> v(cnt);
            hipMemcpy(v.data(), d, cnt * 4, hipMemcpyDeviceToHost);
            for (uint32_t x : v) h = (h ^ x) * 1099511628211ull;
        };
        mix(ga, n * 128);
        mix(ge, n * K * 128);
        mix(gw2, 128 * 128);
        mix(gb2, 128);
        printf("  output hash (ga, gz1, dW2, db2 of the masked sorted backward): %016llx\n", (unsigned long long)h);
    }
    timed("backward_sorted exact fp32 + relu mask", [&] {
        mmpde_gnn_edge_backward_sorted(da, db, dnb, nullptr, n, K, dw2, db2, dg, pos, mask, ga, ge, part, gw2, gb2,
                                       MMPDE_EDGE_GEMM_F32, nullptr);
    });
    {   // the same hash for the exact-fp32 masked sorted backward
        CK(mmpde_gnn_edge_backward_sorted(da, db, dnb, nullptr, n, K, dw2, db2, dg, pos, mask, ga, ge, part, gw2,
                                          gb2, MMPDE_EDGE_GEMM_F32, nullptr));
        CK(hipDeviceSynchronize());
        uint64_t h = 1469598103934665603ull;
        auto mix = [&](const float *d, size_t cnt) {
            std::vector<uint32_t> v(cnt);
            hipMemcpy(v.data(), d, cnt * 4, hipMemcpyDeviceToHost);
            for (uint32_t x : v) h = (h ^ x) * 1099511628211ull;
        };
        mix(ga, n * 128);
        mix(ge, n * K * 128);
        mix(gw2, 128 * 128);
        mix(gb2, 128);
        printf("  output hash (exact fp32 masked sorted backward): %016llx\n", (unsigned long long)h);
    }
    timed("source_sum_sorted (contiguous)", [&] { mmpde_gnn_edge_source_sum_sorted(ge, off, n, gb, nullptr); });
    {   // hash of the source sums (of the exact-fp32 gz1 rows above)
        CK(mmpde_gnn_edge_source_sum_sorted(ge, off, n, gb, nullptr));
        CK(hipDeviceSynchronize());
        std::vector<uint32_t> v(n * 128);
        hipMemcpy(v.data(), gb, v.size() * 4, hipMemcpyDeviceToHost);
        uint64_t h = 1469598103934665603ull;
        for (uint32_t x : v) h = (h ^ x) * 1099511628211ull;
        printf("  output hash (source_sum_sorted): %016llx\n", (unsigned long long)h);
    }
    timed("reverse_adjacency (+ slot positions)", [&] {
        mmpde_reverse_adjacency(dnb, n, K, nullptr, n, off, edge, pos, scratch, sb, bad, nullptr);
    });
    CK(hipDeviceSynchronize());
    return 0;
}
