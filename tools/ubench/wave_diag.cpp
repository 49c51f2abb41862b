// Where the f16x3 wave edge kernel's time goes (profiling aid, not shipped):
// the production kernel against DIAG builds with parts of its VALU / memory
// work removed (edge_wave.hip: bit 0 no split, bit 1 no relu-sums, bit 2 no b
// gathers, bit 5 relu-sums replaced by register sinks, bit 6 no stores, bit 7 no
// a-row reloads), and the
// bare MFMA stream of the same count at one wave per SIMD.  Cylinder-sized
// synthetic layer (n = B x 2521, k = 35, random in-trajectory neighbours).
//   make -C tools/ubench wave_diag && tools/ubench/wave_diag [B]
#include "../../mm-pde_amd/csrc/common.hpp"
#include "../../mm-pde_amd/csrc/f16x3.hpp"
#include "../../mm-pde_amd/csrc/layer.hpp"

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <random>
#include <vector>

int launch_edge_wave_diag(const float *a, const float *b, const int32_t *nbr, int64_t n, int k,
                          const float *msg2_b, const char *pk, const float *rng, float *out,
                          float *side, int cus, int diag, hipStream_t st);

#define CK(x)                                                                          \
    do {                                                                               \
        hipError_t e_ = (x);                                                           \
        if (e_ != hipSuccess) {                                                        \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            return 1;                                                                  \
        }                                                                              \
    } while (0)

// v_mfma_f32_16x16x32_f16 stream, one wave per SIMD, B operands in AGPRs like
// the edge kernel (2 chains; the instruction's rate is the same on 1..16).
__global__ __launch_bounds__(64, 1) void mfma_only_wave(const float4 *seed, int iters, float4 *out) {
    const int lane = threadIdx.x;
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
    out[blockIdx.x * 64 + lane] = make_float4(acc0[0] + acc1[0], acc0[1], acc0[2], acc1[3]);
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
    const int B = argc > 1 ? atoi(argv[1]) : 16, N = 2521, k = 35, H = 128;
    const int64_t n = (int64_t)B * N;
    std::mt19937 rng(1);
    float *a = dev_random(n * H, -1, 1, rng), *b = dev_random(n * H, -1, 1, rng);
    float *w2 = dev_random(128 * 128, -0.09f, 0.09f, rng), *b2 = dev_random(128, -0.09f, 0.09f, rng);
    std::vector<int32_t> hn(n * k);
    // neighbour locality: "random" (uniform in the trajectory, like a mesh in
    // random node order), "local" (within +-R of the target's index, like a
    // space-filling-curve order), "self" (every neighbour is the target)
    const char *mode = argc > 2 ? argv[2] : "random";
    const int R = argc > 3 ? atoi(argv[3]) : 24;
    std::uniform_int_distribution<int> di(0, N - 1), dl(-R, R);
    for (int64_t i = 0; i < n; ++i)
        for (int e = 0; e < k; ++e) {
            int64_t j;
            if (!strcmp(mode, "self")) j = i;
            else if (!strcmp(mode, "local")) {
                const int64_t l = std::min<int64_t>(std::max<int64_t>(i % N + dl(rng), 0), N - 1);
                j = (i / N) * N + l;
            } else j = (i / N) * N + di(rng);
            hn[i * k + e] = (int32_t)j;
        }
    printf("neighbours: %s (R = %d)\n", mode, R);
    int32_t *nbr;
    CK(hipMalloc(&nbr, n * k * 4));
    CK(hipMemcpy(nbr, hn.data(), n * k * 4, hipMemcpyHostToDevice));
    mmpde_gnn_layer_params lp{w2, b2, w2, b2, w2, b2, w2, b2, b2, b2, b2, b2, 1e-5f, 128, 128};
    // only message_net_2's image is read by the edge kernel
    char *pack;
    CK(hipMalloc(&pack, mmpde_gnn_pack_bytes(1)));
    float *w1big = dev_random(128 * 260, -0.06f, 0.06f, rng);
    lp.msg1_w = w1big;
    lp.msg1_ld = 260;
    lp.upd1_w = w1big;
    lp.upd1_ld = 260;
    if (mmpde_gnn_pack_f16x3(&lp, 1, pack, 0) != 0) return 1;
    // range records (layer.hpp): max |a| = max |b| = 1 in every node tile
    float *amax;
    {
        std::vector<float> hs(4 * range_tiles(n), 1.0f);
        CK(hipMalloc(&amax, hs.size() * 4));
        CK(hipMemcpy(amax, hs.data(), hs.size() * 4, hipMemcpyHostToDevice));
    }
    float *out, *side;
    CK(hipMalloc(&out, 2 * n * H * 4));
    int dev = 0, cus = 256;
    hipGetDevice(&dev);
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    CK(hipMalloc(&side, (size_t)4 * cus * 16 * H * 4));
    const int64_t ntiles = (n + 15) / 16;
    const double mfmas = (double)ntiles * k * 96;
    printf("n=%lld k=%d cus=%d  MFMAs per launch %.3e (%.0f per SIMD)\n", (long long)n, k, cus, mfmas,
           mfmas / (4.0 * cus));
    struct V { const char *name; int diag; };
    const V vs[] = {{"production", 0},           {"no split", 1},          {"no relu-sums", 2},
                    {"no split, no relu-sums", 3}, {"no gathers", 4},       {"no VALU, no gathers", 7},
                    
                    {"no relu VALU (sinks)", 32}, {"no stores", 64}, {"no split, no relu VALU", 33},
                    {"no split/relu VALU/stores", 97}, {"no relu VALU, no gathers", 36},
                    {"no a-row reloads", 128}};
    const int nv = sizeof(vs) / sizeof(vs[0]), reps = 7, it = 20;
    std::vector<std::vector<float>> t(nv + 1);
    float4 *seed, *mo;
    CK(hipMalloc(&seed, 128 * 16));
    CK(hipMemset(seed, 0x3c, 128 * 16));
    CK(hipMalloc(&mo, (size_t)4 * cus * 64 * 16));
    const int iters = (int)(mfmas / (4.0 * cus) / 24.0 + 0.5);
    for (int r = 0; r < reps; ++r) {
        for (int v = 0; v < nv; ++v)
            t[v].push_back(time_it([&] { launch_edge_wave_diag(a, b, nbr, n, k, b2, pack, amax, out, side, cus, vs[v].diag, 0); }, it));
        t[nv].push_back(time_it([&] { hipLaunchKernelGGL(mfma_only_wave, dim3(4 * cus), dim3(64), 0, 0, seed, iters, mo); }, it));
    }
    CK(hipGetLastError());
    {   // production and the placement variant against fp64 sums on sampled rows
        std::vector<float> ha(n * H), hb(n * H), hw(128 * 128), hbias(128), m(2 * n * H), sd(4 * cus * 16 * H);
        CK(hipMemcpy(ha.data(), a, ha.size() * 4, hipMemcpyDeviceToHost));
        CK(hipMemcpy(hb.data(), b, hb.size() * 4, hipMemcpyDeviceToHost));
        CK(hipMemcpy(hw.data(), w2, hw.size() * 4, hipMemcpyDeviceToHost));
        CK(hipMemcpy(hbias.data(), b2, hbias.size() * 4, hipMemcpyDeviceToHost));
        for (int d : {0}) {
            CK(hipMemset(out, 0, 2 * n * H * 4));
            launch_edge_wave_diag(a, b, nbr, n, k, b2, pack, amax, out, side, cus, d, 0);
            CK(hipMemcpy(m.data(), out, m.size() * 4, hipMemcpyDeviceToHost));
            CK(hipMemcpy(sd.data(), side, sd.size() * 4, hipMemcpyDeviceToHost));
            // the node stage's combine: side blocks of the waves starting inside the tile
            const int64_t S = ((n + 15) / 16) * k, G = std::min<int64_t>(4 * cus, S);
            double worst = 0;
            for (int64_t i = 0; i < n; i += 997) {
                for (int o = 0; o < H; ++o) {
                    double ref = 0, mx = 1e-30;
                    for (int e = 0; e < k; ++e) {
                        const int64_t j = hn[i * k + e];
                        double y = hbias[o];
                        for (int q = 0; q < H; ++q) {
                            double z = (double)ha[i * H + q] + (double)hb[j * H + q];
                            y += (z > 0 ? z : 0) * hw[o * H + q];
                        }
                        ref += y > 0 ? y : 0;
                        mx = std::max(mx, std::fabs(y));
                    }
                    double got = (double)m[i * H + o];
                    const int64_t t = i / 16;
                    const int64_t lo = std::max<int64_t>(((t * k + 1) * G + S - 1) / S, 1);
                    const int64_t hi = std::min<int64_t>(((t + 1) * k * G + S - 1) / S - 1, G - 1);
                    for (int64_t w = lo; w <= hi; ++w) got += sd[(w * 16 + (i & 15)) * H + o];
                    worst = std::max(worst, std::fabs(got - ref) / (k * mx));
                }
            }
            printf("diag %3d vs fp64 (sampled rows): max |err| / (k max|msg|) = %.3e\n", d, worst);
        }
    }
    {   // the schedule variants must reproduce the production sums bit for bit
        std::vector<float> m0(2 * n * H), m1(2 * n * H);
        launch_edge_wave_diag(a, b, nbr, n, k, b2, pack, amax, out, side, cus, 0, 0);
        CK(hipMemcpy(m0.data(), out, m0.size() * 4, hipMemcpyDeviceToHost));
        for (int v = 0; v < nv; ++v) {
            if (vs[v].diag != 16) continue;
            CK(hipMemset(out, 0, m1.size() * 4));
            launch_edge_wave_diag(a, b, nbr, n, k, b2, pack, amax, out, side, cus, vs[v].diag, 0);
            CK(hipMemcpy(m1.data(), out, m1.size() * 4, hipMemcpyDeviceToHost));
            size_t bad = 0;
            for (size_t i = 0; i < m0.size(); ++i) bad += memcmp(&m0[i], &m1[i], 4) != 0;
            printf("%-34s %s (%zu of %zu words differ)\n", vs[v].name, bad ? "DIFFERS" : "bitwise equal", bad, m0.size());
        }
    }
    for (int v = 0; v <= nv; ++v) {
        std::sort(t[v].begin(), t[v].end());
        printf("%-34s median %7.1f  min %7.1f  max %7.1f us\n", v < nv ? vs[v].name : "bare MFMA stream (same count)",
               t[v][reps / 2], t[v][0], t[v][reps - 1]);
    }
    return 0;
}
