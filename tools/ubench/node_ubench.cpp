// Node-stage timing (profiling aid, not shipped): tiled node kernel variants
// of layer.hip on a cylinder-sized synthetic layer (n = B x 2521 rows), F16X3,
// with a bitwise comparison of their outputs against RB2.
//   make -C tools/ubench node_ubench && tools/ubench/node_ubench [B] [parts]
#include "../../mm-pde_amd/csrc/gnn.hip"
#include "../../mm-pde_amd/csrc/layer.hip"
#include <algorithm>
#include <cstdio>
#include <cstring>
#include <functional>
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
    const int B = argc > 1 ? atoi(argv[1]) : 16, N = 2521;
    const int parts = argc > 2 ? atoi(argv[2]) : 2;
    const int64_t n = (int64_t)B * N;
    std::mt19937 rng(1);
    float *h = dev_random(n * H, -1, 1, rng), *u = dev_random(n, -1, 1, rng);
    float *mean = dev_random(4 * n * H, 0, 0.5f, rng);
    float *pos = dev_random(n * 3, 0, 1, rng);
    float *w1 = dev_random(128 * 260, -0.06f, 0.06f, rng), *b1 = dev_random(128, -0.06f, 0.06f, rng);
    float *w2 = dev_random(128 * 128, -0.09f, 0.09f, rng), *b2 = dev_random(128, -0.09f, 0.09f, rng);
    float *u1 = dev_random(128 * 260, -0.06f, 0.06f, rng), *c1 = dev_random(128, -0.06f, 0.06f, rng);
    float *u2 = dev_random(128 * 128, -0.09f, 0.09f, rng), *c2 = dev_random(128, -0.09f, 0.09f, rng);
    float *bnw = dev_random(128, 0.5f, 1.5f, rng), *bnb = dev_random(128, -0.1f, 0.1f, rng);
    float *bnm = dev_random(128, -0.1f, 0.1f, rng), *bnv = dev_random(128, 0.5f, 1.5f, rng);
    float *ho[2], *ao[2], *bo[2];
    for (int i = 0; i < 2; ++i) {
        CK(hipMalloc(&ho[i], n * H * 4));
        CK(hipMalloc(&ao[i], n * H * 4));
        CK(hipMalloc(&bo[i], n * H * 4));
    }
    mmpde_gnn_layer_params lp{w1, b1, w2, b2, u1, c1, u2, c2, bnw, bnb, bnm, bnv, 1e-5f, 260, 260};
    mmpde_gnn_layer_params two[2] = {lp, lp};
    char *pack;
    CK(hipMalloc(&pack, mmpde_gnn_pack_bytes(2)));
    if (mmpde_gnn_pack_f16x3(two, 2, pack, 0) != 0) return 1;
    float *rng_rec;  // range records written by the node stage (layer.hpp)
    CK(hipMalloc(&rng_rec, 4 * range_tiles(n) * 4));
    CK(hipDeviceSynchronize());
    mmpde_gnn_scales sc{1.0f, 1.0f, 1.0f / 2.9f, 1};
    const int cus = device_cus(), it = 20;
    printf("n=%lld parts=%d cus=%d (us per launch, median of 7)\n", (long long)n, parts, cus);
    NodeArgs nd{h, mean, n, u1, c1, 260, u2, c2, bnw, bnb, bnm, bnv, 1e-5f, ho[1], w1, b1, 260, ao[1], bo[1],
                u, pos, sc, pack, pack + kLayerPack, rng_rec, N, parts, n * H};
    nd.div_k = 35;  // the wave edge kernel's buffers hold sums (production)
    NodeArgs nt = nd;
    nt.h_out = ho[0];
    nt.a_out = ao[0];
    nt.b_out = bo[0];
    // the kernels take one or two problems (NodeArgs2): one here
    auto one = [&](const NodeArgs &a, int rows) {
        NodeArgs2 q;
        q.a[0] = q.a[1] = a;
        q.tiles0 = ceil_div(n, rows);
        return q;
    };
    auto tiled = [&](auto kern, int rows) {
        return [&, kern, rows] { hipLaunchKernelGGL(kern, dim3(ceil_div(n, rows)), dim3(512), 0, 0, one(nt, rows)); };
    };
    struct V {
        const char *name;
        std::function<void()> f;
    };
    std::vector<V> vs;
    vs.push_back({"tiled RB2", tiled(gnn_node_kernel<true, true, 2>, 32)});
    vs.push_back({"tiled RB4", tiled(gnn_node_kernel<true, true, 4>, 64)});

    vs.push_back({"tiled RB2 last layer", tiled(gnn_node_kernel<false, true, 2>, 32)});
    const int reps = 7;
    std::vector<std::vector<float>> t(vs.size());
    for (int r = 0; r < reps; ++r)
        for (size_t v = 0; v < vs.size(); ++v) t[v].push_back(time_it(vs[v].f, it));
    for (size_t v = 0; v < vs.size(); ++v) {
        std::sort(t[v].begin(), t[v].end());
        printf("node %-18s median %6.1f  min %6.1f  max %6.1f\n", vs[v].name, t[v][reps / 2], t[v][0],
               t[v][reps - 1]);
    }
    // bitwise: tiled RB2 (outputs 0) against tiled RB4 and the weight-stationary kernel (outputs 1)
    auto compare = [&](const char *name, std::function<void()> other) -> int {
        CK(hipMemset(ho[1], 0, n * H * 4));
        CK(hipMemset(ao[1], 0, n * H * 4));
        CK(hipMemset(bo[1], 0, n * H * 4));
        hipLaunchKernelGGL((gnn_node_kernel<true, true, 2>), dim3(ceil_div(n, 32)), dim3(512), 0, 0, one(nt, 32));
        CK(hipDeviceSynchronize());
        std::vector<float> rec0(4 * range_tiles(n)), rec1(4 * range_tiles(n));
        CK(hipMemcpy(rec0.data(), rng_rec, rec0.size() * 4, hipMemcpyDeviceToHost));
        other();
        CK(hipDeviceSynchronize());
        CK(hipMemcpy(rec1.data(), rng_rec, rec1.size() * 4, hipMemcpyDeviceToHost));
        for (int q = 0; q < 3; ++q) {
            std::vector<float> x(n * H), y(n * H);
            float *p0 = q == 0 ? ho[0] : q == 1 ? ao[0] : bo[0], *p1 = q == 0 ? ho[1] : q == 1 ? ao[1] : bo[1];
            CK(hipMemcpy(x.data(), p0, n * H * 4, hipMemcpyDeviceToHost));
            CK(hipMemcpy(y.data(), p1, n * H * 4, hipMemcpyDeviceToHost));
            size_t nb = 0;
            for (size_t i = 0; i < x.size(); ++i) nb += memcmp(&x[i], &y[i], 4) != 0;
            printf("%s vs RB2 array %d (h', a', b'): %zu differing words\n", name, q, nb);
        }
        size_t nr = 0;
        for (size_t i = 0; i < rec0.size(); ++i) nr += memcmp(&rec0[i], &rec1[i], 4) != 0;
        printf("%s vs RB2 range records: %zu differing words\n", name, nr);
        return 0;
    };
    if (compare("RB4", [&] { hipLaunchKernelGGL((gnn_node_kernel<true, true, 4>), dim3(ceil_div(n, 64)), dim3(512), 0, 0, one(nd, 64)); }))
        return 1;

    CK(hipGetLastError());
    return 0;
}
