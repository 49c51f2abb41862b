// The wave edge kernel's slot stream without memory (profiling aid, not
// shipped): 96 v_mfma_f32_16x16x32_f16 per slot in the production shape (8
// column tiles, accumulator chains of 12, W2 pinned in AGPRs, accumulators and A
// operands in VGPRs), with the production VALU units placed one per MFMA gap
// (edge_wave.hip, MMPDE_EDGE_PLACE 1) but fed from registers: no gathers, no
// stores, no unit bookkeeping.  Variants drop the relu-sums and / or the split,
// so the difference to the bare chains is the price of the VALU alone.
//   make -C tools/ubench slotsim && tools/ubench/slotsim
#include "../../mm-pde_amd/csrc/common.hpp"
#include "../../mm-pde_amd/csrc/f16x3.hpp"

#include <cstdio>

namespace {

__device__ __forceinline__ float relu_acc(float s, float x) {
    float t;
    asm("v_max_f32_e32 %1, 0, %2\n\tv_add_f32_e32 %0, %0, %1" : "+v"(s), "=&v"(t) : "v"(x));
    return s;
}
__device__ __forceinline__ half8 pin_agpr(half8 v) {
    half8 r;
    asm("; pin %0" : "=a"(r) : "0"(v));
    return r;
}

// V bit 0: relu-sums, bit 1: split; bit 2: pin each unit right after its MFMA;
// bit 3: b-row gathers (index 3 slots ahead, rows 2 slots ahead, production
// pipeline; the index from the table with bit 8, else arithmetic); bit 4: a-row reload every 35 slots; bit 5: unit stores every 35 slots;
// bit 6 (with bit 3): the b rows come from an LDS row buffer (528-B rows, local
// index = global index mod 64) instead of global memory; bit 7 (with 6): plus a
// fill stream of one global float4 per lane per slot written to LDS a slot later
template <int V>
__global__ __launch_bounds__(64, 1) void slot_kernel(const float4 *seed, int slots, float *out,
                                                     const float *bmat, const int32_t *nbr, const float *amat,
                                                     float *sums, int nrow) {
    const int r = threadIdx.x & 15, g = threadIdx.x >> 4;
    auto piece = [&](int i) { return 32 * (i >> 1) + 8 * g + 4 * (i & 1); };
    const int64_t base = (int64_t)blockIdx.x * 40;  // this wave's rows: 2.5 tiles
    const int lane = threadIdx.x;
    half8 wh[8][4], wl[8][4];
#pragma unroll
    for (int c = 0; c < 8; ++c)
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            const float4 v = seed[(c * 4 + s) * 64 + lane];
            wh[c][s] = pin_agpr(__builtin_bit_cast(half8, v));
            wl[c][s] = pin_agpr(__builtin_bit_cast(half8, make_float4(v.y, v.x, v.w, v.z)));
        }
    float4 av[8], X[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        av[i] = seed[(32 + i) * 64 + lane];
        X[i] = seed[(40 + i) * 64 + lane];
    }
    float sc = 0.125f;
    uint32_t hA[4][4], lA[4][4], hB[4][4], lB[4][4];
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int q = 0; q < 4; ++q) hA[s][q] = lA[s][q] = hB[s][q] = lB[s][q] = 0x3c003c00u + lane + q;
    f32x4 S[8];
#pragma unroll
    for (int c = 0; c < 8; ++c) S[c] = (f32x4){0.0f, 0.0f, 0.0f, 0.0f};
    f32x4 acc6 = (f32x4){0.0f, 0.0f, 0.0f, 0.0f}, acc7 = acc6;
    auto a_piece = [&](int j) { return 2 * (j >> 2) + ((j >> 1) & 1); };
    __shared__ float4 lrows[64 * 33];  // 64 rows of 528 B
    if (V & 64) {
        for (int i = lane; i < 64 * 33; i += 64) lrows[i] = make_float4(0.001f * i, 0.0f, 0.0f, 0.0f);
        __syncthreads();
    }
    float4 fill = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    int q_slot = 0;
    uint32_t i_next = 0, i_after = 0;
    auto body = [&](uint32_t (*h)[4], uint32_t (*l)[4], uint32_t (*nh)[4], uint32_t (*nl)[4]) {
        const float *brow = bmat;
        if (V & (8 | 256)) {
            if (V & 256)  // the neighbour index from the table (a global load per slot)
                i_after = (uint32_t)nbr[((base + (q_slot + 3) / 35 * 16 + r) % nrow) * 35 + (q_slot + 3) % 35];
            else          // an arithmetic stand-in (no load)
                i_after = (uint32_t)((q_slot * 37 + r * 131 + (int)base) & 32767);
            brow = bmat + (int64_t)min(i_next, (uint32_t)(nrow - 1)) * 128;
            if (V & 64) brow = (const float *)lrows + (i_next & 63) * 132;
            i_next = i_after;
        }
        if (V & 128) {  // fill: last slot's float4 to LDS, this slot's from global
            lrows[((q_slot * 7 + lane) & 63) * 33 + (q_slot & 31)] = fill;
            fill = *(const float4 *)(amat + ((base * 128 + (int64_t)q_slot * 512 + lane * 4) % ((int64_t)nrow * 128)));
        }
        if ((V & 16) && (q_slot + 1) % 35 == 0) {
            const float *ar = amat + ((base + (q_slot + 1) / 35 * 16 + r) % nrow) * 128;
            float4 v[8];
#pragma unroll
            for (int i = 0; i < 8; ++i) v[i] = *(const float4 *)(ar + piece(i));
#pragma unroll
            for (int i = 0; i < 8; ++i) av[i] = make_float4(v[i].x * sc, v[i].y * sc, v[i].z * sc, v[i].w * sc);
        }
        const bool close = (V & 32) && q_slot % 35 == 34;
        f32x4 acc[8];
        float xs0 = 0.0f, xs1 = 0.0f;
#pragma unroll
        for (int c = 0; c < 8; ++c) {
            acc[c] = (f32x4){sc, sc, sc, sc};
#pragma unroll
            for (int s = 0; s < 4; ++s) {
                const half8 ah = __builtin_bit_cast(half8, h[s]), al = __builtin_bit_cast(half8, l[s]);
                const int G = 4 * c + s, j = G >> 1;
                acc[c] = mfma_f16(ah, wh[c][s], acc[c]);
                if (V & 4) __builtin_amdgcn_sched_barrier(0);
                {
                    f32x4 &Sc = G >= 6 ? S[(G - 6) >> 2] : (G < 2 ? S[6] : S[7]);
                    const int t = G >= 6 ? (G - 6) & 3 : (G < 2 ? G + 2 : G - 2);
                    const float x = G >= 6 ? acc[(G - 6) >> 2][t] : (G < 2 ? acc6[t] : acc7[t]);
                    if (V & 1) Sc[t] = relu_acc(Sc[t], x);
                    else asm volatile("" ::"v"(x));
                }
                __builtin_amdgcn_sched_barrier(0);
                acc[c] = mfma_f16(ah, wl[c][s], acc[c]);
                if (V & 4) __builtin_amdgcn_sched_barrier(0);
                if (V & 2) {
                    if ((G & 1) == 0) {
                        const float4 &ap = av[a_piece(j)];
                        const float4 &bb = X[a_piece(j)];
                        xs0 = (j & 1) ? fmaf(bb.z, sc, ap.z) : fmaf(bb.x, sc, ap.x);
                        xs1 = (j & 1) ? fmaf(bb.w, sc, ap.w) : fmaf(bb.y, sc, ap.y);
                    } else {
                        split_l(xs0, nh[j >> 2][j & 3], nl[j >> 2][j & 3]);
                    }
                }
                __builtin_amdgcn_sched_barrier(0);
                acc[c] = mfma_f16(al, wh[c][s], acc[c]);
                if (V & 4) __builtin_amdgcn_sched_barrier(0);
                if (V & 2) {
                    if ((G & 1) == 0) {
                        split_c(xs0, xs1, nh[j >> 2][j & 3]);
                        if (j == 0) split_p(h[3][3]);
                        else split_p(nh[(j - 1) >> 2][(j - 1) & 3]);
                    } else {
                        split_h(xs1, nh[j >> 2][j & 3], nl[j >> 2][j & 3]);
                    }
                }
                if ((V & 8) && (G & 3) == 3) X[G >> 2] = *(const float4 *)(brow + piece(G >> 2));
                __builtin_amdgcn_sched_barrier(0);
                if (G == 5 && close) {
                    float *o = sums + ((base + q_slot / 35 * 16) % nrow + 4 * g) * 128 + r;
#pragma unroll
                    for (int c2 = 0; c2 < 8; ++c2)
#pragma unroll
                        for (int t = 0; t < 4; ++t) o[t * 128 + 16 * c2] = S[c2][t];
#pragma unroll
                    for (int c2 = 0; c2 < 8; ++c2) S[c2] = (f32x4){0.0f, 0.0f, 0.0f, 0.0f};
                }
            }
        }
        acc6 = acc[6];
        acc7 = acc[7];
        if (!(V & 2)) {  // keep the operand buffers' roles alternating
#pragma unroll
            for (int s = 0; s < 4; ++s) asm volatile("" : "+v"(nh[s][0]), "+v"(nl[s][0]));
        }
        sc = sc * 1.0000001f;
        ++q_slot;
    };
    for (int q = 0; q < slots; q += 2) {
        body(hA, lA, hB, lB);
        body(hB, lB, hA, lA);
    }
    float res = acc6[0] + acc7[1];
#pragma unroll
    for (int c = 0; c < 8; ++c) res += S[c][0] + S[c][1] + S[c][2] + S[c][3];
    out[blockIdx.x * 64 + lane] = res;
}

struct Mem { const float *b; const int32_t *nbr; const float *a; float *sums; int nrow; };
static Mem g_mem;

template <int V>
float run(const float4 *seed, int slots, float *out, int cus) {
    const Mem &m = g_mem;
    hipLaunchKernelGGL((slot_kernel<V>), dim3(4 * cus), dim3(64), 0, 0, seed, slots, out, m.b, m.nbr, m.a, m.sums, m.nrow);
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    (void)hipEventRecord(a, 0);
    for (int i = 0; i < 5; ++i) hipLaunchKernelGGL((slot_kernel<V>), dim3(4 * cus), dim3(64), 0, 0, seed, slots, out, m.b, m.nbr, m.a, m.sums, m.nrow);
    (void)hipEventRecord(b, 0);
    (void)hipEventSynchronize(b);
    float ms;
    (void)hipEventElapsedTime(&ms, a, b);
    return 1e3f * ms / 5;
}

}  // namespace

int main() {
    int cus = 256, dev = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    float4 *seed;
    float *out;
    (void)hipMalloc(&seed, 48 * 64 * 16);
    static float4 h[48 * 64];
    for (int i = 0; i < 48 * 64; ++i) h[i] = make_float4(0.01f * (i % 97), -0.02f * (i % 31), 0.5f, 0.003f * i);
    (void)hipMemcpy(seed, h, sizeof(h), hipMemcpyHostToDevice);
    (void)hipMalloc(&out, 4 * cus * 64 * 4);
    const int slots = 86;  // the cylinder B = 16 launch: 88,235 slots over 1024 waves
    {   // a cylinder-sized layer: n = 16 x 2521 rows, neighbours random in the trajectory
        const int nrow = 16 * 2521;
        float *b, *a, *sums;
        int32_t *nbr;
        (void)hipMalloc(&b, (size_t)nrow * 128 * 4);
        (void)hipMalloc(&a, (size_t)nrow * 128 * 4);
        (void)hipMalloc(&sums, (size_t)nrow * 128 * 4);
        (void)hipMalloc(&nbr, (size_t)nrow * 35 * 4);
        (void)hipMemset(b, 0, (size_t)nrow * 128 * 4);
        (void)hipMemset(a, 0, (size_t)nrow * 128 * 4);
        static int32_t hn[16 * 2521 * 35];
        uint32_t x = 12345;
        for (int i = 0; i < nrow; ++i)
            for (int e = 0; e < 35; ++e) {
                x = x * 1664525u + 1013904223u;
                hn[i * 35 + e] = (i / 2521) * 2521 + (int)((x >> 8) % 2521);
            }
        (void)hipMemcpy(nbr, hn, sizeof(hn), hipMemcpyHostToDevice);
        g_mem = Mem{b, nbr, a, sums, nrow};
    }
    struct Var { const char *name; float (*f)(const float4 *, int, float *, int); };
    const Var vs[] = {{"bare chains", run<0>},
                      {"VALU pinned", run<7>},
                      {"+ index loads only", run<7 | 256>},
                      {"+ global gathers, arithmetic index", run<7 | 8>},
                      {"+ global gathers, table index", run<7 | 8 | 256>},
                      {"+ LDS gathers, arithmetic index", run<7 | 8 | 64>},
                      {"+ LDS gathers, table index", run<7 | 8 | 64 | 256>},
                      {"all memory, global gathers", run<7 | 8 | 16 | 32 | 256>},
                      {"all memory, LDS gathers", run<7 | 8 | 16 | 32 | 64 | 256>}};
    for (int rep = 0; rep < 3; ++rep) {
        for (const auto &v : vs) printf("%-40s %7.1f us\n", v.name, v.f(seed, slots, out, cus));
        printf("--\n");
    }
    return 0;
}
