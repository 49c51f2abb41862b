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

// CU-level sharing (the LDS-staged edge design, costed without its plan): a
// 256-thread workgroup per CU, its four waves (one per SIMD) splitting the 32
// neighbour slots of one 16-target tile (8 each) at a time; b rows read from a
// double-buffered LDS row cache (104 rows of 528 B, local indices from an LDS
// table), the next tile's rows filled from global memory during the current
// tile (about 1.4 float4 per lane per slot); at each tile end the waves' partial
// sums are combined through LDS (two barriers) and stored.  V bit 0: fill
// stream on; bit 1: combine + barriers on; bit 2: per-tile prologue split
// (the first slot's split is not overlapped with MFMAs).
template <int V>
__global__ __launch_bounds__(256, 1) void cu_kernel(const float4 *seed, int tiles, float *out, const float *amat,
                                                    float *sums, int nrow) {
    constexpr int RCAP = 104, RS = 132;  // rows, row stride (floats)
    extern __shared__ float4 dyn4[];
    float *rowbuf = (float *)dyn4;                       // [2][RCAP][RS]
    float *arows = rowbuf + 2 * RCAP * RS;               // [2][16][RS]
    float *part = arows + 2 * 16 * RS;                   // [4][16][RS]
    uint8_t *lidx = (uint8_t *)(part + 4 * 16 * RS);     // [2][32][16]
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int r = lane & 15, g = lane >> 4;
    auto piece = [&](int i) { return 32 * (i >> 1) + 8 * g + 4 * (i & 1); };
    for (int i = threadIdx.x; i < 2 * RCAP * RS; i += 256) rowbuf[i] = 0.001f * (i % 977);
    for (int i = threadIdx.x; i < 2 * 16 * RS; i += 256) arows[i] = 0.002f * (i % 331);
    for (int i = threadIdx.x; i < 2 * 32 * 16; i += 256) lidx[i] = (uint8_t)((i * 37) % RCAP);
    __syncthreads();
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
    float sc = 0.125f;
    uint32_t hA[4][4], lA[4][4], hB[4][4], lB[4][4];
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int q = 0; q < 4; ++q) hA[s][q] = lA[s][q] = hB[s][q] = lB[s][q] = 0x3c003c00u + lane + q;
    f32x4 S[8];
#pragma unroll
    for (int c = 0; c < 8; ++c) S[c] = (f32x4){0.0f, 0.0f, 0.0f, 0.0f};
    f32x4 acc6 = (f32x4){-3.0e38f, -3.0e38f, -3.0e38f, -3.0e38f}, acc7 = acc6;
    auto a_piece = [&](int j) { return 2 * (j >> 2) + ((j >> 1) & 1); };
    const int64_t gbase = (int64_t)blockIdx.x * 40 * 128;
    float4 fill = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    int q_slot = 0, cur = 0, e = 0;
    const float *brow = rowbuf;
    auto split_pair = [&](int j, uint32_t (*nh)[4], uint32_t (*nl)[4]) {
        const float4 &ap = av[a_piece(j)];
        const float4 &bb = X[a_piece(j)];
        const float x0 = (j & 1) ? fmaf(bb.z, sc, ap.z) : fmaf(bb.x, sc, ap.x);
        const float x1 = (j & 1) ? fmaf(bb.w, sc, ap.w) : fmaf(bb.y, sc, ap.y);
        split2_relu_rtz(x0, x1, nh[j >> 2][j & 3], nl[j >> 2][j & 3]);
    };
    auto body = [&](uint32_t (*h)[4], uint32_t (*l)[4], uint32_t (*nh)[4], uint32_t (*nl)[4]) {
        // the b rows of slot e + 1 (this wave's next slot), index from the LDS table
        {
            const int en = min(e + 1, 7);
            const int li = lidx[(cur * 32 + wave * 8 + en) * 16 + r];
            brow = rowbuf + (cur * RCAP + li) * RS;
        }
        if (V & 1) {  // fill stream: last slot's float4 to the other buffer, this slot's from global
            rowbuf[((1 - cur) * RCAP + ((q_slot * 7 + lane) % RCAP)) * RS + 4 * (lane & 31)] = fill.x;
            fill = *(const float4 *)(amat + ((gbase + (int64_t)q_slot * 512 + lane * 4) % ((int64_t)nrow * 128)));
        }
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
                __builtin_amdgcn_sched_barrier(0);
                {
                    f32x4 &Sc = G >= 6 ? S[(G - 6) >> 2] : (G < 2 ? S[6] : S[7]);
                    const int t = G >= 6 ? (G - 6) & 3 : (G < 2 ? G + 2 : G - 2);
                    const float x = G >= 6 ? acc[(G - 6) >> 2][t] : (G < 2 ? acc6[t] : acc7[t]);
                    Sc[t] = relu_acc(Sc[t], x);
                }
                __builtin_amdgcn_sched_barrier(0);
                acc[c] = mfma_f16(ah, wl[c][s], acc[c]);
                __builtin_amdgcn_sched_barrier(0);
                if ((G & 1) == 0) {
                    const float4 &ap = av[a_piece(j)];
                    const float4 &bb = X[a_piece(j)];
                    xs0 = (j & 1) ? fmaf(bb.z, sc, ap.z) : fmaf(bb.x, sc, ap.x);
                    xs1 = (j & 1) ? fmaf(bb.w, sc, ap.w) : fmaf(bb.y, sc, ap.y);
                } else {
                    split_l(xs0, nh[j >> 2][j & 3], nl[j >> 2][j & 3]);
                }
                __builtin_amdgcn_sched_barrier(0);
                acc[c] = mfma_f16(al, wh[c][s], acc[c]);
                __builtin_amdgcn_sched_barrier(0);
                if ((G & 1) == 0) {
                    split_c(xs0, xs1, nh[j >> 2][j & 3]);
                    if (j == 0) split_p(h[3][3]);
                    else split_p(nh[(j - 1) >> 2][(j - 1) & 3]);
                } else {
                    split_h(xs1, nh[j >> 2][j & 3], nl[j >> 2][j & 3]);
                }
                if ((G & 3) == 3) X[G >> 2] = *(const float4 *)(brow + piece(G >> 2));
                __builtin_amdgcn_sched_barrier(0);
            }
        }
        acc6 = acc[6];
        acc7 = acc[7];
        sc = sc * 1.0000001f;
        ++q_slot;
        ++e;
    };
    for (int t = 0; t < tiles; ++t) {
        // tile prologue: a rows from LDS (scaled), slot 0's rows and split
        e = 0;
        {
            const float *ar = arows + (cur * 16 + r) * RS;
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                const float4 v = *(const float4 *)(ar + piece(i));
                av[i] = make_float4(v.x * sc, v.y * sc, v.z * sc, v.w * sc);
            }
            const int li = lidx[(cur * 32 + wave * 8) * 16 + r];
            const float *b0 = rowbuf + (cur * RCAP + li) * RS;
#pragma unroll
            for (int i = 0; i < 8; ++i) X[i] = *(const float4 *)(b0 + piece(i));
        }
        if (V & 4) {
#pragma unroll
            for (int j = 0; j < 16; ++j) split_pair(j, hA, lA);
        }
        for (int q = 0; q < 8; q += 2) {
            body(hA, lA, hB, lB);
            body(hB, lB, hA, lA);
        }
        // trailing relu-sums of the last slot
#pragma unroll
        for (int tt = 2; tt < 4; ++tt) S[6][tt] = relu_acc(S[6][tt], acc6[tt]);
#pragma unroll
        for (int tt = 0; tt < 4; ++tt) S[7][tt] = relu_acc(S[7][tt], acc7[tt]);
        acc6 = acc7 = (f32x4){-3.0e38f, -3.0e38f, -3.0e38f, -3.0e38f};
        if (V & 2) {  // partial sums combined through LDS, stored
            float *pw = part + (wave * 16 + 4 * g) * RS + r;
#pragma unroll
            for (int c = 0; c < 8; ++c)
#pragma unroll
                for (int tt = 0; tt < 4; ++tt) pw[tt * RS + 16 * c] = S[c][tt];
            __syncthreads();
            const int row = lane >> 2, c0 = 32 * wave + 8 * (lane & 3);
            float4 s0 = make_float4(0.f, 0.f, 0.f, 0.f), s1 = s0;
#pragma unroll
            for (int w = 0; w < 4; ++w) {
                const float4 *pp = (const float4 *)(part + (w * 16 + row) * RS + c0);
                const float4 a0 = pp[0], a1 = pp[1];
                s0 = make_float4(s0.x + a0.x, s0.y + a0.y, s0.z + a0.z, s0.w + a0.w);
                s1 = make_float4(s1.x + a1.x, s1.y + a1.y, s1.z + a1.z, s1.w + a1.w);
            }
            float4 *o = (float4 *)(sums + ((int64_t)(blockIdx.x * 16 + row) % nrow) * 128 + c0);
            o[0] = s0;
            o[1] = s1;
            __syncthreads();
        } else {
            __syncthreads();
        }
#pragma unroll
        for (int c = 0; c < 8; ++c) S[c] = (f32x4){0.0f, 0.0f, 0.0f, 0.0f};
        cur ^= 1;
    }
    out[blockIdx.x * 256 + threadIdx.x] = fill.x + S[0][0] + (float)hA[0][0] + (float)lB[1][1];
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

template <int V>
float run_cu(const float4 *seed, int tiles, float *out, int cus) {
    const Mem &m = g_mem;
    const size_t lds = (size_t)(2 * 104 * 132 + 2 * 16 * 132 + 4 * 16 * 132) * 4 + 2 * 32 * 16;
    (void)hipFuncSetAttribute((const void *)cu_kernel<V>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipLaunchKernelGGL((cu_kernel<V>), dim3(cus), dim3(256), lds, 0, seed, tiles, out, m.a, m.sums, m.nrow);
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    (void)hipEventRecord(a, 0);
    for (int i = 0; i < 5; ++i)
        hipLaunchKernelGGL((cu_kernel<V>), dim3(cus), dim3(256), lds, 0, seed, tiles, out, m.a, m.sums, m.nrow);
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
    struct VarCu { const char *name; float (*f)(const float4 *, int, float *, int); };
    const VarCu cs[] = {{"CU-level: LDS rows, no fill, no combine", run_cu<0>},
                        {"CU-level: + fill stream", run_cu<1>},
                        {"CU-level: + combine (2 barriers)", run_cu<3>},
                        {"CU-level: + per-tile prologue split", run_cu<7>}};
    for (int rep = 0; rep < 3; ++rep) {
        for (const auto &v : vs) printf("%-40s %7.1f us\n", v.name, v.f(seed, slots, out, cus));
        for (const auto &v : cs) printf("%-40s %7.1f us\n", v.name, v.f(seed, 11, out, cus));  // 11 tiles x 8 slots per wave
        printf("--\n");
    }
    return 0;
}
