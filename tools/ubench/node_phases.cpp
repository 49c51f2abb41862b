// Node-stage phase timing (profiling aid, not shipped): the production chain
// embed -> wave edge stage -> node stage on a cylinder-sized synthetic layer
// (B x 2521 rows, k = 35 random in-trajectory neighbours, F16X3, the rollout's
// segment size), the node kernel built with -DMMPDE_NODE_STAMPS: wave 0 of
// every workgroup stamps the shader clock at the phase boundaries.  Prints the
// launch time (hipEvents), the mean of every phase over the workgroups, and how
// many workgroups run at once.
// Then times the embed kernel (embedding + layer 0's projections) with its
// output hash.
//   make -C tools/ubench node_phases && tools/ubench/node_phases [B]
#include "../../mm-pde_amd/csrc/gnn.hip"
#include "../../mm-pde_amd/csrc/layer.hip"
#include <algorithm>
#include <cstdio>
#include <random>
#include <vector>

#define CK(x)                                                                         \
    do {                                                                              \
        hipError_t e_ = (x);                                                          \
        if (e_ != hipSuccess) {                                                       \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            return 1;                                                                 \
        }                                                                             \
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

int main(int argc, char **argv) {
    const int B = argc > 1 ? atoi(argv[1]) : 16, N = 2521, K = 35;
    const int64_t n = (int64_t)B * N;
    std::mt19937 rng(1);
    float *u = dev_random(n, -1, 1, rng), *pos = dev_random(n * 3, 0, 1, rng);
    auto W = [&](size_t c, float s) { return dev_random(c, -s, s, rng); };
    mmpde_gnn_embed_params ep{W(128 * 4, 0.5f), W(128, 0.1f), W(128, 1.0f), W(128, 0.1f), W(128, 0.1f),
                              dev_random(128, 0.5f, 1.5f, rng), W(128 * 128, 0.09f), W(128, 0.1f), W(128, 1.0f),
                              W(128, 0.1f), W(128, 0.1f), dev_random(128, 0.5f, 1.5f, rng), 1e-5f};
    mmpde_gnn_layer_params lp{W(128 * 260, 0.06f), W(128, 0.06f), W(128 * 128, 0.09f), W(128, 0.09f),
                              W(128 * 260, 0.06f), W(128, 0.06f), W(128 * 128, 0.09f), W(128, 0.09f),
                              dev_random(128, 0.5f, 1.5f, rng), W(128, 0.1f), W(128, 0.1f),
                              dev_random(128, 0.5f, 1.5f, rng), 1e-5f, 260, 260};
    mmpde_gnn_layer_params two[2] = {lp, lp};
    char *pack;
    CK(hipMalloc(&pack, mmpde_gnn_pack_bytes(2)));
    if (mmpde_gnn_pack_f16x3(two, 2, pack, 0) != 0) return 1;
    // neighbour table: k distinct random rows of the same trajectory
    std::vector<int32_t> nb(n * K);
    for (int64_t i = 0; i < n; ++i) {
        const int64_t b0 = i / N * N;
        for (int e = 0; e < K; ++e) nb[i * K + e] = (int32_t)(b0 + (rng() % N));
    }
    int32_t *nbr;
    CK(hipMalloc(&nbr, nb.size() * 4));
    CK(hipMemcpy(nbr, nb.data(), nb.size() * 4, hipMemcpyHostToDevice));
    float *ws;
    const int64_t wsb = mmpde_gnn_workspace_bytes(n);
    CK(hipMalloc(&ws, wsb));
    float *h0 = ws, *h1 = ws + n * H, *wa = ws + 2 * n * H, *wb = ws + 3 * n * H, *wm = ws + 4 * n * H;
    float *rngr = ws + kGnnBufs * n * H;
    mmpde_gnn_scales sc{1.0f, 1.0f, 1.0f / 2.9f, 1, 0, 0.0f, nullptr};
    const int nblk = (int)ceil_div(n, 32);
    uint64_t *stamps;
    CK(hipMalloc(&stamps, (size_t)nblk * 8 * 8));
    CK(hipMemcpyToSymbol(HIP_SYMBOL(g_node_stamps), &stamps, sizeof(stamps)));
    if (launch_embed_stage(u, pos, n, N, sc, &ep, &lp, pack, rngr, h0, wa, wb, 0)) return 1;
    EdgeSplit split;
    if (launch_edge_stage(wa, wb, nbr, nullptr, n, K, N, &lp, pack, rngr, wm, wm + n * H,
                          (kGnnBufs - 5) * n * H / (16 * H), &split, 0))
        return 1;
    CK(hipDeviceSynchronize());
    printf("n=%lld B=%d: edge split U=%d per segment\n", (long long)n, B, split.units);
    float *ao, *bo, *rout;
    CK(hipMalloc(&ao, n * H * 4));
    CK(hipMalloc(&bo, n * H * 4));
    CK(hipMalloc(&rout, 4 * range_tiles(n) * 4));
    auto node = [&](bool next) {
        return launch_node_stage(h0, wm, &split, nullptr, u, pos, n, N, sc, &lp, next ? &lp : nullptr, pack,
                                 next ? pack + kLayerPack : nullptr, next ? rout : nullptr, h1, ao, bo, 0);
    };
    for (int next = 1; next >= 0; --next) {
        for (int i = 0; i < 5; ++i)
            if (node(next)) return 1;
        hipEvent_t a, b;
        hipEventCreate(&a);
        hipEventCreate(&b);
        const int it = 20;
        hipEventRecord(a, 0);
        for (int i = 0; i < it; ++i) node(next);
        hipEventRecord(b, 0);
        CK(hipEventSynchronize(b));
        float ms = 0;
        hipEventElapsedTime(&ms, a, b);
        // one stamped launch
        CK(hipMemset(stamps, 0, (size_t)nblk * 64));
        node(next);
        CK(hipDeviceSynchronize());
        std::vector<uint64_t> st((size_t)nblk * 8);
        CK(hipMemcpy(st.data(), stamps, st.size() * 8, hipMemcpyDeviceToHost));
        uint64_t t0 = ~0ull, t1 = 0;
        double ph[8] = {0};
        for (int w = 0; w < nblk; ++w) {
            const uint64_t *s = &st[(size_t)w * 8];
            t0 = std::min(t0, s[0]);
            t1 = std::max(t1, s[7]);
            for (int i = 1; i <= 7; ++i) {
                if (!next && i == 6) continue;
                const int prev = (!next && i == 7) ? 5 : i - 1;
                ph[i] += (double)(s[i] - s[prev]);
            }
            ph[0] += (double)(s[7] - s[0]);
        }
        // stamps: the 100 MHz real-time clock (10 ns ticks)
        printf("%s node kernel: %.2f us per launch; the stamped launch spans %.2f us\n",
               next ? "NEXT" : "last", 1e3 * ms / it, 0.01 * (double)(t1 - t0));
        static const char *names[8] = {"whole workgroup", "constants + operand issue", "prep [h|mean] + barrier",
                                       "GEMM1 + epilogue", "barrier + prep v + barrier",
                                       "GEMM2 + epilogue (h')", "barrier + prep h' + barrier",
                                       "GEMM3 projections + stores"};
        for (int i = 0; i < 8; ++i) {
            if (!next && i == 6) continue;
            printf("  %-30s %8.2f us mean\n", names[i], 0.01 * ph[i] / nblk);
        }
        // concurrency: workgroups alive at the midpoint of every workgroup's life
        std::vector<std::pair<uint64_t, int>> ev;
        for (int w = 0; w < nblk; ++w) {
            ev.push_back({st[(size_t)w * 8], 1});
            ev.push_back({st[(size_t)w * 8 + 7], -1});
        }
        std::sort(ev.begin(), ev.end());
        int live = 0, peak = 0;
        double area = 0;
        for (size_t i = 0; i + 1 < ev.size(); ++i) {
            live += ev[i].second;
            peak = std::max(peak, live);
            area += (double)live * (double)(ev[i + 1].first - ev[i].first);
        }
        printf("  workgroups alive: peak %d, mean %.0f\n", peak, area / (double)(t1 - t0));
        // output hash (FNV-1a over h', a', b' and the range records): builds
        // of the kernel that must be bitwise equal print the same value
        uint64_t hsh = 1469598103934665603ull;
        auto fold = [&](const float *d, size_t cnt) {
            std::vector<uint32_t> v(cnt);
            hipMemcpy(v.data(), d, cnt * 4, hipMemcpyDeviceToHost);
            for (uint32_t w : v) hsh = (hsh ^ w) * 1099511628211ull;
        };
        fold(h1, n * H);
        if (next) {
            fold(ao, n * H);
            fold(bo, n * H);
            fold(rout, 4 * range_tiles(n));
        }
        printf("  output hash %016llx\n", (unsigned long long)hsh);
    }
    {   // the embed kernel (embedding + layer 0's projections), time and output hash
        auto embed = [&]() { return launch_embed_stage(u, pos, n, N, sc, &ep, &lp, pack, rngr, h0, wa, wb, 0); };
        for (int i = 0; i < 5; ++i)
            if (embed()) return 1;
        hipEvent_t a, b;
        hipEventCreate(&a);
        hipEventCreate(&b);
        const int it = 20;
        hipEventRecord(a, 0);
        for (int i = 0; i < it; ++i) embed();
        hipEventRecord(b, 0);
        CK(hipEventSynchronize(b));
        float ms = 0;
        hipEventElapsedTime(&ms, a, b);
        uint64_t hsh = 1469598103934665603ull;
        auto fold = [&](const float *d, size_t cnt) {
            std::vector<uint32_t> v(cnt);
            hipMemcpy(v.data(), d, cnt * 4, hipMemcpyDeviceToHost);
            for (uint32_t w : v) hsh = (hsh ^ w) * 1099511628211ull;
        };
        fold(h0, n * H);
        fold(wa, n * H);
        fold(wb, n * H);
        fold(rngr, 4 * range_tiles(n));
        printf("embed kernel: %.2f us per launch; output hash %016llx\n", 1e3 * ms / it, (unsigned long long)hsh);
    }
    CK(hipGetLastError());
    return 0;
}
