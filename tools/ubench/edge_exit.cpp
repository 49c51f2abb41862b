// Exit-time spread of the f16x3 wave edge kernel (profiling aid, not shipped):
// the production plan on a cylinder-sized synthetic layer (B segments of 2521
// rows, k = 35 random in-trajectory neighbours, narrow range records), the
// kernel built with DIAG bit 256 (each wave stores its exit time, 100 MHz
// clock; 0 spills, unlike an entry stamp).  Prints the launch time (hipEvents,
// production kernel) and the distribution of the waves' exit times relative to
// the last one: what a perfectly balanced launch could save.
//   make -C tools/ubench edge_exit && tools/ubench/edge_exit [B]
#include "../../mm-pde_amd/csrc/common.hpp"
#include "../../mm-pde_amd/csrc/layer.hpp"

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <random>
#include <vector>

int launch_edge_wave_exit_stamps(const float *a, const float *b, const int32_t *nbr, int64_t n, int k,
                                 int64_t seg_n, const float *msg2_b, const char *pk, const float *rmx,
                                 float *out, float *side, int64_t side_cap, int cus, uint64_t *stamps,
                                 hipStream_t st);

#define CK(x)                                                                         \
    do {                                                                              \
        hipError_t e_ = (x);                                                          \
        if (e_ != hipSuccess) {                                                       \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            return 1;                                                                 \
        }                                                                             \
    } while (0)

static float *dev_fill(size_t count, float lo, float hi, std::mt19937 &rng) {
    std::uniform_real_distribution<float> d(lo, hi);
    std::vector<float> h(count);
    for (auto &v : h) v = lo == hi ? lo : d(rng);
    float *p = nullptr;
    if (hipMalloc(&p, count * 4) != hipSuccess) return nullptr;
    if (hipMemcpy(p, h.data(), count * 4, hipMemcpyHostToDevice) != hipSuccess) return nullptr;
    return p;
}

int main(int argc, char **argv) {
    const int B = argc > 1 ? atoi(argv[1]) : 16, N = 2521, k = 35, H = 128;
    const int64_t n = (int64_t)B * N;
    std::mt19937 rng(1);
    float *a = dev_fill(n * H, -1, 1, rng), *b = dev_fill(n * H, -1, 1, rng);
    float *w2 = dev_fill(128 * 128, -0.09f, 0.09f, rng), *b2 = dev_fill(128, -0.09f, 0.09f, rng);
    float *w1big = dev_fill(128 * 260, -0.06f, 0.06f, rng);
    std::vector<int32_t> hn(n * k);
    std::uniform_int_distribution<int> di(0, N - 1);
    for (int64_t i = 0; i < n; ++i)
        for (int e = 0; e < k; ++e) hn[i * k + e] = (int32_t)((i / N) * N + di(rng));
    int32_t *nbr;
    CK(hipMalloc(&nbr, n * k * 4));
    CK(hipMemcpy(nbr, hn.data(), n * k * 4, hipMemcpyHostToDevice));
    mmpde_gnn_layer_params lp{w1big, b2, w2, b2, w1big, b2, w2, b2, b2, b2, b2, b2, 1e-5f, 260, 260};
    char *pack;
    CK(hipMalloc(&pack, mmpde_gnn_pack_bytes(1)));
    if (mmpde_gnn_pack_f16x3(&lp, 1, pack, 0) != 0) return 1;
    float *rmx = dev_fill(row_records_floats(n), 1.0f, 1.0f, rng);  // every segment narrow
    int dev = 0, cus = 256;
    CK(hipGetDevice(&dev));
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    const int64_t side_cap = (int64_t)B * 3 * N / 16;
    float *out, *side;
    CK(hipMalloc(&out, n * H * 4));
    CK(hipMalloc(&side, side_cap * 16 * H * 4));
    uint64_t *stamps;
    CK(hipMalloc(&stamps, 8 * 8192));
    auto run = [&](uint64_t *st) {
        return launch_edge_wave_exit_stamps(a, b, nbr, n, k, N, b2, pack, rmx, out, side, side_cap, cus, st, 0);
    };
    for (int i = 0; i < 20; ++i)
        if (run(nullptr) <= 0) return 1;
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const int it = 20;
    CK(hipEventRecord(e0, 0));
    for (int i = 0; i < it; ++i) run(nullptr);
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    printf("B=%d waves=%d launch %.2f us (production kernel, hipEvents over %d launches)\n", B, run(nullptr),
           1e3 * ms / it, it);
    std::vector<std::vector<double>> runs;
    for (int rep = 0; rep < 3; ++rep) {
        for (int i = 0; i < 5; ++i) run(nullptr);
        CK(hipEventRecord(e0, 0));
        const int waves = run(stamps);
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        CK(hipEventElapsedTime(&ms, e0, e1));
        std::vector<uint64_t> h(waves);
        CK(hipMemcpy(h.data(), stamps, waves * 8, hipMemcpyDeviceToHost));
        {   // per XCD (block & 7) mean exit relative to the launch's last exit, and the raw
            // per-block times for the run-to-run correlation below
            const uint64_t mx = *std::max_element(h.begin(), h.end());
            double xm[8] = {0};
            int xc[8] = {0};
            std::vector<double> r(waves);
            for (int i = 0; i < waves; ++i) {
                r[i] = 0.01 * (double)(mx - h[i]);
                xm[i & 7] += r[i];
                ++xc[i & 7];
            }
            printf("  per XCD mean exit before the last (us):");
            for (int x = 0; x < 8; ++x) printf(" %.2f", xm[x] / std::max(xc[x], 1));
            printf("\n");
            runs.push_back(r);
        }
        std::sort(h.begin(), h.end());
        const uint64_t last = h.back();
        auto before = [&](double f) { return 0.01 * (double)(last - h[(size_t)(f * (waves - 1))]); };
        double mean = 0;
        for (uint64_t t : h) mean += 0.01 * (double)(last - t);
        mean /= waves;
        printf("stamped launch %.2f us: exit before the last exit (us): first %.2f p10 %.2f p50 %.2f p90 %.2f "
               "mean %.2f\n", 1e3 * ms, before(0.0), before(0.1), before(0.5), before(0.9), mean);
    }
    {   // does a block that finishes early in one launch finish early in the next?
        const auto &x = runs[1], &y = runs[2];
        double mx = 0, my = 0;
        for (size_t i = 0; i < x.size(); ++i) mx += x[i], my += y[i];
        mx /= x.size();
        my /= y.size();
        double sxy = 0, sxx = 0, syy = 0;
        for (size_t i = 0; i < x.size(); ++i)
            sxy += (x[i] - mx) * (y[i] - my), sxx += (x[i] - mx) * (x[i] - mx), syy += (y[i] - my) * (y[i] - my);
        printf("run-to-run correlation of the blocks' exit times: %.3f\n", sxy / std::sqrt(sxx * syy + 1e-30));
    }
    return 0;
}
