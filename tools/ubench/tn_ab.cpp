// Weight-gradient row GEMM timing (profiling aid, not shipped): mmpde_rgemm_tn
// at the three train-mode GNN layer shapes of cy B=16 (n = 40336 rows;
// gnn_2d.py GnnLayerTrain.backward): dU1 (G = dv, X = [h | mean] + t, db),
// dW1 (G = da, X = h + (u, x, y, t), db) and dU2 (G = dx masked by upd, X = v,
// db).  Prints us per call (partials + fixed-order reduce) and an output hash
// per shape (variants must match bit for bit).
//   make -C tools/ubench tn_ab_base && tools/ubench/tn_ab_base
// TN_SRC: another rgemm.hip for a same-box A/B (built with -I mm-pde_amd/csrc)
#ifndef TN_SRC
#define TN_SRC "../../mm-pde_amd/csrc/rgemm.hip"
#endif
#include TN_SRC
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

static float *dev_rand(size_t cnt, std::mt19937 &rng, bool relu) {
    std::normal_distribution<float> nd(0.0f, 1.0f);
    std::vector<float> h(cnt);
    for (auto &v : h) {
        v = nd(rng);
        if (relu && v < 0.0f) v = 0.0f;
    }
    float *p = nullptr;
    if (hipMalloc(&p, cnt * 4) != hipSuccess) return nullptr;
    hipMemcpy(p, h.data(), cnt * 4, hipMemcpyHostToDevice);
    return p;
}

int main() {
    const int64_t n = 16 * 2521;
    const char *ce = getenv("TN_CHUNK");   // row chunk (256 = production; others change the bits)
    const int chunk = ce ? atoi(ce) : 256;
    std::mt19937 rng(11);
    float *G = dev_rand(n * 128, rng, false), *X1 = dev_rand(n * 128, rng, false),
          *X2 = dev_rand(n * 128, rng, false), *XS = dev_rand(n * 4, rng, false),
          *M = dev_rand(n * 128, rng, true);
    float *dw, *db, *ws;
    hipMalloc(&dw, 128 * 260 * 4);
    hipMalloc(&db, 128 * 4);
    const int64_t wsb = mmpde_rgemm_tn_workspace_bytes(n, chunk, 2 * 128 + 4 + 1);
    hipMalloc(&ws, wsb);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    struct Shape {
        const char *name;
        mmpde_rgemm_tn_args a;
        int lddw;
    };
    auto base = [&]() {
        mmpde_rgemm_tn_args a{};
        a.m = n;
        a.chunk_rows = chunk;
        a.gcols = 128;
        a.g = G;
        a.ldg = 128;
        a.dw = dw;
        a.db = db;
        a.sign_s = 1.0f;
        return a;
    };
    std::vector<Shape> shapes;
    {   // dU1: [h | mean] segments, t column (extras col 3) as the small segment
        auto a = base();
        a.nseg = 2;
        a.x[0] = X1, a.ldx[0] = 128, a.kx[0] = 128, a.dwcol[0] = 0;
        a.x[1] = X2, a.ldx[1] = 128, a.kx[1] = 128, a.dwcol[1] = 128;
        a.xs = XS + 3, a.ldxs = 4, a.ns = 1, a.dwcol_s = 256;
        a.lddw = 257;
        shapes.push_back({"dU1 (2 segs + ns 1)", a, 257});
    }
    {   // dW1: h segment, (u, x, y, t) small segment
        auto a = base();
        a.nseg = 1;
        a.x[0] = X1, a.ldx[0] = 128, a.kx[0] = 128, a.dwcol[0] = 0;
        a.xs = XS, a.ldxs = 4, a.ns = 4, a.dwcol_s = 256;
        a.lddw = 260;
        shapes.push_back({"dW1 (1 seg + ns 4)", a, 260});
    }
    {   // dU2: G masked by upd > 0
        auto a = base();
        a.nseg = 1;
        a.gmask = M;
        a.x[0] = X1, a.ldx[0] = 128, a.kx[0] = 128, a.dwcol[0] = 0;
        a.lddw = 128;
        shapes.push_back({"dU2 (gmask, 1 seg)", a, 128});
    }
    for (auto &s : shapes) {
        auto fn = [&] { return mmpde_rgemm_tn(&s.a, ws, wsb, nullptr); };
        for (int i = 0; i < 3; ++i)
            if (fn()) {
                fprintf(stderr, "mmpde_rgemm_tn failed (%s)\n", s.name);
                return 1;
            }
        const int it = 20;
        hipEventRecord(e0, 0);
        for (int i = 0; i < it; ++i) fn();
        hipEventRecord(e1, 0);
        hipEventSynchronize(e1);
        float ms = 0;
        hipEventElapsedTime(&ms, e0, e1);
        hipMemset(dw, 0, 128 * 260 * 4);
        fn();
        hipDeviceSynchronize();
        std::vector<uint32_t> hw(128 * 260), hb(128);
        hipMemcpy(hw.data(), dw, hw.size() * 4, hipMemcpyDeviceToHost);
        hipMemcpy(hb.data(), db, hb.size() * 4, hipMemcpyDeviceToHost);
        uint64_t h = 1469598103934665603ull;
        for (int r = 0; r < 128; ++r)
            for (int c = 0; c < s.lddw; ++c) h = (h ^ hw[r * s.lddw + c]) * 1099511628211ull;
        for (uint32_t x : hb) h = (h ^ x) * 1099511628211ull;
        printf("  %-22s %8.1f us   hash %016llx\n", s.name, 1e3 * ms / it, (unsigned long long)h);
    }
    return 0;
}
