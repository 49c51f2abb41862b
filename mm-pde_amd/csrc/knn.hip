// Batched exact k-nearest-neighbour search for gfx950.
//
// Replaces torch_cluster.knn_graph (reference data_creator_2d.py:260,
// mesh/dmm_model.py:228) and sklearn NearestNeighbors.kneighbors
// (data_creator_2d.py:66-78).  One wave per query; the trajectory's point set
// (<= 4096 points, <= 32 KB) is staged once per workgroup in LDS; every lane
// keeps CPL fp32 squared distances in registers (larger sets, up to 16384
// points: knn_large_kernel below).  Selection: U = the kk-th
// smallest of the 64 per-lane minima (a 64-wide bitonic sort across the wave)
// bounds the kk-th smallest key from above; the points with key <= U (a few
// dozen on a mesh; for the fp64 query key, fp32 key <= U plus a proven
// rounding margin) are compacted into a per-wave LDS list, their exact keys
// formed, and sorted by (key, index) with a 128-wide two-per-lane bitonic
// network.  Longer lists are ranked exhaustively; lists past kCap fall back to
// a full bitwise radix select over all exact keys with ties at the threshold
// taken in index order.  Every way the result is exactly the
// (distance, index)-ordered list of the reference's insertion sort,
// independent of scheduling.
//
// Distance keys (must match oracle/knn_oracle.c bit for bit):
//   graph: d2 = fmaf(dy, dy, dx*dx) in fp32  (torch_cluster under nvcc fmad)
//   query: d2 = dx*dx + dy*dy in fp64        (sklearn float64 rdist)
// Non-negative IEEE values order like their bit patterns, so keys are the
// raw bits.
#include <type_traits>

#include "common.hpp"

namespace {

constexpr int kQueriesPerBlock = 16;  // 4 per wave
constexpr int kCap = 256;             // LDS list of candidates with key <= U, per wave

// Moved-mesh displacement record (mmpde_knn_moved_cells), per trajectory:
// dcell[kCells] (-1: empty cell), box (x0, y0, hx, hy, eps), the largest
// displacement, then per role (0: graph, 1: query) the count of queries the
// candidate table could not answer in the last call (written by the
// fallback; diagnostics).
constexpr int kCellG = 16;                           // cells per axis
constexpr int kCells = kCellG * kCellG;
constexpr int kCellRec = kCells + 16;                // floats per trajectory record
__device__ __forceinline__ int32_t *cell_last_miss(const float *cells, int b) {
    return (int32_t *)(cells + (int64_t)b * kCellRec + kCells + 8);  // [role]
}
// set (plain stores of 1) by knn_cand_kernel when any query of the trajectory
// missed, zeroed with the record: a fallback workgroup of a trajectory without
// misses returns at once
__device__ __forceinline__ int32_t *cell_any_miss(const float *cells, int b) {
    return (int32_t *)(cells + (int64_t)b * kCellRec + kCells + 10);  // [role]
}
// set by knn_cand_kernel when the trajectory skipped the table (skip_above):
// the fallback then answers all its queries without reading the flags
__device__ __forceinline__ int32_t *cell_skipped(const float *cells, int b) {
    return (int32_t *)(cells + (int64_t)b * kCellRec + kCells + 12);  // [role]
}

// fp32 squared distance as raw bits: the graph key, and the query's filter key.
__device__ __forceinline__ uint32_t key_f32(float2 p, float2 q) {
#pragma clang fp contract(off)
    float dx = p.x - q.x;
    float dy = p.y - q.y;
    float a = dx * dx;
    return __float_as_uint(fmaf(dy, dy, a));
}

template <bool QUERY>
struct KeyTraits;

template <>
struct KeyTraits<false> {
    typedef uint32_t key_t;
    static constexpr int kTopBit = 30;  // valid keys are < 2^31
    __device__ static key_t key(float2 p, float2 q) { return key_f32(p, q); }
    // the filter key is the key itself
    __device__ static uint32_t filter_threshold(uint32_t u) { return u; }
};

template <>
struct KeyTraits<true> {
    typedef uint64_t key_t;
    static constexpr int kTopBit = 62;  // valid keys are < 2^63
    __device__ static key_t key(float2 p, float2 q) {
#pragma clang fp contract(off)
        double dx = (double)p.x - (double)q.x;
        double dy = (double)p.y - (double)q.y;
        double a = dx * dx;
        double c = dy * dy;
        return (key_t)__double_as_longlong(a + c);
    }
    // Candidates are filtered on the fp32 key f, whose relative error against
    // the fp64 key is <= 2^-22 (<= 4 ulp: two rounded differences, two
    // rounded products / one fma); an absolute 2^-126 covers denormal
    // flushing.  If u is the kk-th smallest fp32 lane minimum, at least kk
    // points have fp64 key <= u (1 + 2^-22) + 2^-126, hence so does every
    // point of the answer, whose fp32 key is then <= u + ~9 ulp.  A 64-ulp
    // margin over max(u, min normal) keeps every answer point a candidate.
    __device__ static uint32_t filter_threshold(uint32_t u) {
        return u >= 0x7f000000u ? 0xfffffffeu : (u < 0x00800000u ? 0x00800000u : u) + 64u;
    }
};

__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
}

// v of lane ^ j without the LDS pipe (ds_bpermute's round trip would sit on
// every step of the sorting networks): DPP quad_perm for j = 1, 2; DPP
// row_shl / row_shr by j plus a select for j = 4, 8 (row_shl:j reads lane + j);
// v_permlane16_swap / v_permlane32_swap of v with itself for j = 16, 32 (the
// swap moves odd rows of its first operand with even rows of its second /
// the upper half of the first with the lower half of the second).  j must fold
// to a constant: the networks below are fully unrolled.
__device__ __forceinline__ uint32_t xor_lane(uint32_t v, int j, int lane) {
    const int x = (int)v;
    switch (j) {
    case 1:
        return (uint32_t)__builtin_amdgcn_update_dpp(0, x, 0xB1, 0xF, 0xF, false);  // [1,0,3,2]
    case 2:
        return (uint32_t)__builtin_amdgcn_update_dpp(0, x, 0x4E, 0xF, 0xF, false);  // [2,3,0,1]
    case 4: {
        const int up = __builtin_amdgcn_update_dpp(0, x, 0x104, 0xF, 0xF, false);
        const int dn = __builtin_amdgcn_update_dpp(0, x, 0x114, 0xF, 0xF, false);
        return (uint32_t)((lane & 4) ? dn : up);
    }
    case 8: {
        const int up = __builtin_amdgcn_update_dpp(0, x, 0x108, 0xF, 0xF, false);
        const int dn = __builtin_amdgcn_update_dpp(0, x, 0x118, 0xF, 0xF, false);
        return (uint32_t)((lane & 8) ? dn : up);
    }
    case 16: {
        const auto r = __builtin_amdgcn_permlane16_swap(v, v, false, false);
        return (lane & 16) ? r[0] : r[1];
    }
    default: {  // 32
        const auto r = __builtin_amdgcn_permlane32_swap(v, v, false, false);
        return (lane & 32) ? r[0] : r[1];
    }
    }
}

// v of lane l, l wave-uniform (a kernel argument or from a ballot): v_readlane
// into an SGPR instead of a ds_bpermute round trip (the same value).
template <typename T>
__device__ __forceinline__ T lane_value(T v, int l) {
    if constexpr (sizeof(T) == 8) {
        const uint64_t u = (uint64_t)v;
        const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)u, l);
        const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(u >> 32), l);
        return (T)(((uint64_t)hi << 32) | lo);
    } else {
        return (T)__builtin_amdgcn_readlane((int)v, l);
    }
}

template <typename K>
__device__ __forceinline__ K shfl_xor_key(K v, int m, int lane) {
    if constexpr (sizeof(K) == 8) {
        const uint32_t lo = xor_lane((uint32_t)v, m, lane);
        const uint32_t hi = xor_lane((uint32_t)(v >> 32), m, lane);
        return ((K)hi << 32) | lo;
    } else {
        return xor_lane(v, m, lane);
    }
}

// Bitonic sort of one key per lane across the wave, ascending in lane order.
template <typename K>
__device__ __forceinline__ K wave_sort64(K v, int lane) {
#pragma unroll
    for (int size = 2; size <= 64; size <<= 1) {
#pragma unroll
        for (int j = size >> 1; j > 0; j >>= 1) {
            const K o = shfl_xor_key(v, j, lane);
            const bool keep_min = ((lane & j) == 0) == ((lane & size) == 0);
            v = keep_min ? (o < v ? o : v) : (o < v ? v : o);
        }
    }
    return v;
}

__device__ __forceinline__ bool ki_less(uint32_t ka, int ia, uint32_t kb, int ib) {
    // 31-bit keys and 12-bit indices: one 64-bit compare
    return (((uint64_t)ka << 32) | (uint32_t)ia) < (((uint64_t)kb << 32) | (uint32_t)ib);
}
__device__ __forceinline__ bool ki_less(uint64_t ka, int ia, uint64_t kb, int ib) {
    return ka < kb || (ka == kb && ia < ib);
}

// One compare-exchange step of the 128-wide network on register r of this
// lane against lane ^ j (same register), keeping the min iff keep_min.
template <typename K>
__device__ __forceinline__ void cx_lane(K &k, int &i, int j, bool keep_min, int lane) {
    const K ok = shfl_xor_key(k, j, lane);
    const int oi = (int)xor_lane((uint32_t)i, j, lane);
    const bool take = ki_less(ok, oi, k, i) == keep_min;
    k = take ? ok : k;
    i = take ? oi : i;
}

// Bitonic sort of 64 (key, index) pairs, one per lane, ordered
// lexicographically (the reference's tie order).  Ascending in lane.
template <typename K>
__device__ __forceinline__ void wave_sort64_ki(K &k, int &i, int lane) {
#pragma unroll
    for (int size = 2; size <= 64; size <<= 1) {
#pragma unroll
        for (int j = size >> 1; j > 0; j >>= 1)
            cx_lane(k, i, j, ((lane & j) == 0) == ((lane & size) == 0), lane);
    }
}

// Bitonic sort of 128 (key, index) pairs ordered lexicographically (the
// reference's tie order), two per lane: element p lives in lane p & 63,
// register p >> 6.  Ascending in p.
template <typename K>
__device__ __forceinline__ void wave_sort128(K &k0, int &i0, K &k1, int &i1, int lane) {
#pragma unroll
    for (int size = 2; size <= 128; size <<= 1) {
#pragma unroll
        for (int j = size >> 1; j > 0; j >>= 1) {
            if (j == 64) {  // size == 128: partners are the lane's own two registers
                const bool sw = ki_less(k1, i1, k0, i0);
                const K tk = k0;
                const int ti = i0;
                k0 = sw ? k1 : k0;
                i0 = sw ? i1 : i0;
                k1 = sw ? tk : k1;
                i1 = sw ? ti : i1;
            } else {
                // element p = lane (+64): ascending block iff (p & size) == 0
                const bool lower = (lane & j) == 0;
                cx_lane(k0, i0, j, lower == ((lane & size) == 0), lane);
                cx_lane(k1, i1, j, lower == (((lane + 64) & size) == 0), lane);
            }
        }
    }
}

// Selection and output of one query once the candidates C = {key <= thr} (m
// of them, indices in sIdx) are compacted: sort / rank C by (key, index), or
// the radix-select fallback over all cpl x 64 keys when C overflows kCap; then
// the k answers in (key, index) order (the graph variant drops the self point).
// sKey / sIdx / sSel: this wave's LDS lists.
template <bool QUERY>
__device__ __forceinline__ void knn_finish(const float2 *sP, typename KeyTraits<QUERY>::key_t *sKey,
                                           int *sIdx, int *sSel, int m, float2 q, int kk, int k, int qi,
                                           int b, int n_src, int n_q, int cpl, int lane, uint64_t below,
                                           int32_t *__restrict__ out, int32_t *__restrict__ degenerate,
                                           bool count_tie = true) {
    typedef KeyTraits<QUERY> KT;
    typedef typename KT::key_t key_t;
    key_t mk = ~key_t(0);
    int mi = 0x7fffffff;
    int rank = lane;
    // QUERY: an exact fp64 distance tie inside the first kk (order) or between
    // ranks kk - 1 and kk (set): the inputs on which sklearn's order is its
    // KD-tree's traversal, not (distance, index) -- counted in *degenerate
    bool tie = false;
    if (m <= 64) {
        // The common case (a mesh point's list holds ~1.5 kk): one pair per
        // lane, one 64-wide bitonic sort.
        wave_lds_sync();
        key_t k0 = ~key_t(0);
        int i0 = 0x7fffffff;
        if (lane < m) {
            i0 = sIdx[lane];
            k0 = KT::key(sP[i0], q);
        }
        wave_sort64_ki(k0, i0, lane);
        if (lane < kk) mi = i0;
        if (QUERY) {
            const key_t kn = (key_t)__shfl((unsigned long long)k0, (lane + 1) & 63, 64);
            tie = __ballot(lane < kk && lane + 1 < m && k0 == kn) != 0ull;
        }
    } else if (m <= 128) {
        // Two pairs per lane, one 128-wide bitonic sort.
        wave_lds_sync();
        key_t k0 = ~key_t(0), k1 = ~key_t(0);
        int i0 = 0x7fffffff, i1 = 0x7fffffff;
        if (lane < m) {
            i0 = sIdx[lane];
            k0 = KT::key(sP[i0], q);
        }
        if (lane + 64 < m) {
            i1 = sIdx[lane + 64];
            k1 = KT::key(sP[i1], q);
        }
        wave_sort128(k0, i0, k1, i1, lane);
        if (lane < kk) mi = i0;
        if (QUERY) {  // element lane + 1: lane 63's is element 64 (k1 of lane 0)
            const key_t n0 = (key_t)__shfl((unsigned long long)k0, (lane + 1) & 63, 64);
            const key_t n1 = lane_value(k1, 0);
            tie = __ballot(lane < kk && k0 == (lane == 63 ? n1 : n0)) != 0ull;
        }
    } else if (m <= kCap) {
        wave_lds_sync();
        for (int i = lane; i < m; i += 64) sKey[i] = KT::key(sP[sIdx[i]], q);
        wave_lds_sync();
        for (int i = lane; i < m; i += 64) {
            const key_t ki = sKey[i];
            const int ii = sIdx[i];
            int rk = 0, eq_after = 0;
            for (int f = 0; f < m; ++f) {
                const key_t fk = sKey[f];
                const int fi = sIdx[f];
                rk += (fk < ki) || (fk == ki && fi < ii);
                eq_after += fk == ki && fi > ii;
            }
            if (rk < kk) sSel[rk] = ii;
            tie = tie || (QUERY && rk < kk && eq_after > 0);
        }
        tie = __ballot(tie) != 0ull;
        wave_lds_sync();
        if (lane < kk) mi = sSel[lane];
    } else {
        // Fallback for adversarial point sets (hundreds of ties): full
        // radix select on all exact keys, recomputed from LDS per use so
        // that this rare path does not set the kernel's register budget.
        auto key_at = [&](int c) -> key_t {
            const int j = lane + 64 * c;
            return (j < n_src) ? KT::key(sP[j], q) : ~key_t(0);
        };
        key_t T = 0;
        for (int bit = KT::kTopBit; bit >= 0; --bit) {
            const key_t Tc = T | (key_t(1) << bit);
            int cnt = 0;
#pragma unroll 4
            for (int c = 0; c < cpl; ++c) cnt += __popcll(__ballot(key_at(c) < Tc));
            if (cnt <= kk - 1) T = Tc;
        }
        int mlt = 0;
#pragma unroll 4
        for (int c = 0; c < cpl; ++c) mlt += __popcll(__ballot(key_at(c) < T));
        const int need = kk - mlt;  // >= 1 candidates equal to T, taken in index order
        int base = 0, eq_taken = 0;
#pragma unroll 4
        for (int c = 0; c < cpl; ++c) {
            const key_t kc = key_at(c);
            const bool lt = kc < T;
            const bool eq = kc == T;
            const uint64_t em = __ballot(eq);
            const int eqrank = eq_taken + __popcll(em & below);
            const bool sel = lt || (eq && eqrank < need);
            eq_taken += __popcll(em);
            const uint64_t sm = __ballot(sel);
            if (sel) {
                const int pidx = base + __popcll(sm & below);
                sKey[pidx] = kc;
                sIdx[pidx] = lane + 64 * c;
            }
            base += __popcll(sm);
        }
        wave_lds_sync();
        if (lane < kk) {
            mk = sKey[lane];
            mi = sIdx[lane];
        }
        rank = 0;
        int dup = 0;
        for (int f = 0; f < kk; ++f) {
            const key_t fk = sKey[f];
            const int fi = sIdx[f];
            rank += (fk < mk) || (fk == mk && fi < mi);
            dup += fk == mk && fi != mi;
        }
        // ties inside the first kk, or more points at the kk-th key than taken
        tie = __ballot(lane < kk && dup > 0) != 0ull || eq_taken > need;
    }
    wave_lds_sync();  // the next query overwrites sKey / sIdx / sSel
    const int64_t row = ((int64_t)b * n_q + qi) * k;
    if (QUERY) {
        if (lane < kk) out[row + rank] = mi;
        if (tie && count_tie && lane == 0 && degenerate) atomicAdd(degenerate, 1);
    } else {
        const uint64_t smask = __ballot(lane < kk && mi == qi);
        const bool has_self = smask != 0ull;
        const int self_rank = has_self ? lane_value(rank, __ffsll((unsigned long long)smask) - 1) : kk;
        const int pos = rank - ((has_self && rank > self_rank) ? 1 : 0);
        if (lane < kk && !(has_self && mi == qi) && pos < k)
            out[row + pos] = b * n_src + mi;
        if (!has_self && lane == 0 && degenerate) atomicAdd(degenerate, 1);
    }
}

// miss != nullptr (the candidate path's fallback, grid.x = ceil(n_q / QPB)):
// miss[b n_q + i] != 0 marks the queries of trajectory b the table could not
// answer.  Every workgroup counts the trajectory's flags and ranks them in
// index order (wave ballots, no atomics).  With more than half missed it
// answers its own QPB queries as the plain search does (re-answering a few is
// harmless: same result); otherwise the missed queries of ranks x, x + grid.x,
// ... (at most QPB), so a few misses spread over many workgroups; with none it
// returns before staging the points.  Workgroup 0 records the count.
template <int CPL, bool QUERY, int QPB = kQueriesPerBlock>
__global__ __launch_bounds__(256) void knn_kernel(const float2 *__restrict__ pts,
                                                  const float2 *__restrict__ qry, int n_src,
                                                  int n_q, int k, int32_t *__restrict__ out,
                                                  int32_t *__restrict__ degenerate,
                                                  const uint8_t *__restrict__ miss = nullptr,
                                                  float *__restrict__ cells = nullptr,
                                                  int role = 0) {
    typedef KeyTraits<QUERY> KT;
    typedef typename KT::key_t key_t;
    __shared__ float2 sP[CPL * 64];
    __shared__ key_t sKey[4][kCap];
    __shared__ int sIdx[4][kCap];
    __shared__ int sSel[4][64];

    const int b = blockIdx.y;
    int q_count = n_q;  // queries of this trajectory to answer
    __shared__ int sList[QPB];
    // QUERY ties are counted for the queries the candidate kernel did not
    // answer (its miss flags, valid unless the trajectory skipped the table)
    const uint8_t *miss_cnt = miss;
    if (miss && cell_skipped(cells, b)[role]) {  // workgroup-uniform: the plain search
        miss_cnt = nullptr;
        if (blockIdx.x == 0 && threadIdx.x == 0) cell_last_miss(cells, b)[role] = n_q;
        miss = nullptr;
    }
    if (miss) {
        if (!cell_any_miss(cells, b)[role]) {  // workgroup-uniform
            if (blockIdx.x == 0 && threadIdx.x == 0) cell_last_miss(cells, b)[role] = 0;
            return;
        }
        __shared__ int sWave[4];
        const int tid = threadIdx.x, w = tid >> 6, l = tid & 63;
        const int gx = (int)gridDim.x, x = (int)blockIdx.x;
        const uint64_t below_l = l == 0 ? 0ull : (~0ull >> (64 - l));
        int total = 0;  // misses before the current chunk
        for (int c0 = 0; c0 < n_q; c0 += 256) {
            const int i = c0 + tid;
            const bool f = i < n_q && miss[(int64_t)b * n_q + i];
            const uint64_t bal = __ballot(f);
            if (l == 0) sWave[w] = __popcll(bal);
            __syncthreads();
            int before = total;
            for (int v = 0; v < w; ++v) before += sWave[v];
            const int r = before + __popcll(bal & below_l);  // rank of this miss
            if (f && r % gx == x && r / gx < QPB) sList[r / gx] = i;
            total += sWave[0] + sWave[1] + sWave[2] + sWave[3];
            __syncthreads();  // sWave is rewritten by the next chunk
        }
        if (x == 0 && tid == 0) cell_last_miss(cells, b)[role] = total;
        if (2 * total > n_q) {
            miss = nullptr;  // most missed: the plain search's own queries
        } else {
            q_count = total > x ? min((total - x + gx - 1) / gx, QPB) : 0;  // entries of this workgroup
            if (q_count == 0) return;  // workgroup-uniform: nothing to answer
        }
    }
    const float2 *P = pts + (int64_t)b * n_src;
    for (int i = threadIdx.x; i < n_src; i += 256) sP[i] = P[i];
    __syncthreads();

    const int wave = threadIdx.x >> 6;
    const int lane = threadIdx.x & 63;
    const int kk = QUERY ? k : k + 1;
    const uint64_t below = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    const int q_beg = miss ? 0 : (int)blockIdx.x * QPB;
    const int q_end = miss ? q_count : min((int)(blockIdx.x + 1) * QPB, n_q);

    for (int qe = q_beg + wave; qe < q_end; qe += 4) {
        const int qi = miss ? sList[qe] : qe;
        const float2 q = QUERY ? qry[(int64_t)b * n_q + qi] : sP[qi];
        uint32_t fkey[CPL];
        uint32_t lmin = ~0u;
#pragma unroll
        for (int c = 0; c < CPL; ++c) {
            const int j = lane + 64 * c;
            fkey[c] = (j < n_src) ? key_f32(sP[j], q) : ~0u;
            lmin = fkey[c] < lmin ? fkey[c] : lmin;
        }
        // U = kk-th smallest of the 64 lane minima.  At least kk points have
        // key <= U (one per lane whose minimum is <= U), so every key of the
        // answer, ties included, is <= U: the answer is exactly the first kk
        // of C = {key <= U} in (key, index) order.  (Query: the filter is on
        // the fp32 key, with the margin of filter_threshold; exact fp64 keys
        // are formed for C only.)  C is small (~2 kk on a mesh), so it is
        // compacted into LDS and sorted.
        const uint32_t thr = KT::filter_threshold(lane_value(wave_sort64(lmin, lane), kk - 1));
        // Compaction (order is free: the list is sorted or ranked next): every
        // lane's candidates as a bit mask, the wave's exclusive prefix of their
        // counts from the counts' bit planes (ballot + mbcnt, no LDS), then each
        // lane writes its own few entries.
        uint64_t cm = 0;
#pragma unroll
        for (int c = 0; c < CPL; ++c) cm |= (uint64_t)(fkey[c] <= thr) << c;
        const int cnt = __popcll(cm);
        int m = 0, pidx = 0;
#pragma unroll
        for (int bit = 0; bit < 6; ++bit) {  // cnt <= CPL <= 64 < 2^7: bit 6 only for 64
            const uint64_t plane = __ballot((cnt >> bit) & 1);
            m += __popcll(plane) << bit;
            pidx += __popcll(plane & below) << bit;
        }
        {
            const uint64_t plane = __ballot(cnt >> 6);
            m += __popcll(plane) << 6;
            pidx += __popcll(plane & below) << 6;
        }
        while (cm) {
            const int c = __builtin_ctzll(cm);
            cm &= cm - 1;
            if (pidx < kCap) sIdx[wave][pidx] = lane + 64 * c;
            ++pidx;
        }
        knn_finish<QUERY>(sP, sKey[wave], sIdx[wave], sSel[wave], m, q, kk, k, qi, b, n_src, n_q, CPL, lane,
                          below, out, degenerate, !miss_cnt || miss_cnt[(int64_t)b * n_q + qi] != 0);
    }
}

// Trajectories of more than 4096 points (up to kLargeMax): the same search
// with the point set in dynamic LDS (one workgroup per CU) and the keys
// recomputed from LDS instead of held in registers -- pass 1 the lane minima,
// pass 2 the compaction of C in chunks of 64 columns -- so any size fits the
// register budget.  64 queries per workgroup amortise the staging.  Same
// selection (knn_finish), same results as knn_kernel.
constexpr int kLargeMax = 16384;
constexpr int kLargeQueries = 64;

template <bool QUERY>
__global__ __launch_bounds__(256) void knn_large_kernel(const float2 *__restrict__ pts,
                                                        const float2 *__restrict__ qry, int n_src,
                                                        int n_q, int k, int32_t *__restrict__ out,
                                                        int32_t *__restrict__ degenerate) {
    typedef KeyTraits<QUERY> KT;
    typedef typename KT::key_t key_t;
    extern __shared__ float2 sP[];
    __shared__ key_t sKey[4][kCap];
    __shared__ int sIdx[4][kCap];
    __shared__ int sSel[4][64];

    const int b = blockIdx.y;
    const float2 *P = pts + (int64_t)b * n_src;
    for (int i = threadIdx.x; i < n_src; i += 256) sP[i] = P[i];
    __syncthreads();

    const int wave = threadIdx.x >> 6;
    const int lane = threadIdx.x & 63;
    const int kk = QUERY ? k : k + 1;
    const int cpl = (n_src + 63) / 64;
    const uint64_t below = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    const int q_end = min((int)(blockIdx.x + 1) * kLargeQueries, n_q);
    for (int qi = blockIdx.x * kLargeQueries + wave; qi < q_end; qi += 4) {
        const float2 q = QUERY ? qry[(int64_t)b * n_q + qi] : sP[qi];
        uint32_t lmin = ~0u;
        for (int c = 0; c < cpl; ++c) {
            const int j = lane + 64 * c;
            const uint32_t f = (j < n_src) ? key_f32(sP[j], q) : ~0u;
            lmin = f < lmin ? f : lmin;
        }
        const uint32_t thr = KT::filter_threshold(lane_value(wave_sort64(lmin, lane), kk - 1));
        int m = 0;
        for (int c0 = 0; c0 < cpl; c0 += 64) {
            const int cn = min(64, cpl - c0);
            uint64_t cm = 0;
            for (int c = 0; c < cn; ++c) {
                const int j = lane + 64 * (c0 + c);
                cm |= (uint64_t)(j < n_src && key_f32(sP[j], q) <= thr) << c;
            }
            const int cnt = __popcll(cm);
            int tot = 0, pidx = 0;
#pragma unroll
            for (int bit = 0; bit < 7; ++bit) {  // cnt <= 64 < 2^7
                const uint64_t plane = __ballot((cnt >> bit) & 1);
                tot += __popcll(plane) << bit;
                pidx += __popcll(plane & below) << bit;
            }
            pidx += m;
            while (cm) {
                const int c = __builtin_ctzll(cm);
                cm &= cm - 1;
                if (pidx < kCap) sIdx[wave][pidx] = lane + 64 * (c0 + c);
                ++pidx;
            }
            m += tot;
        }
        knn_finish<QUERY>(sP, sKey[wave], sIdx[wave], sSel[wave], m, q, kk, k, qi, b, n_src, n_q, cpl, lane,
                          below, out, degenerate);
    }
}

template <bool QUERY>
int launch_knn_large(const float2 *p, const float2 *q, int64_t batches, int ns, int nq, int k, int32_t *out,
                     int32_t *degenerate, hipStream_t st) {
    const size_t lds = (size_t)ns * sizeof(float2);
    const hipError_t e =
        hipFuncSetAttribute((const void *)knn_large_kernel<QUERY>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)lds);
    if (e != hipSuccess) return MMPDE_ERR_HIP_BASE - (int)e;
    dim3 grid(ceil_div(nq, kLargeQueries), (unsigned)batches);
    hipLaunchKernelGGL(knn_large_kernel<QUERY>, grid, dim3(256), lds, st, p, q, ns, nq, k, out, degenerate);
    MMPDE_RET_LAUNCH();
    return MMPDE_OK;
}

template <bool QUERY>
int launch_knn(const float *pts, const float *qry, int64_t batches, int64_t n_src, int64_t n_q,
               int k, int32_t *out, int32_t *degenerate, hipStream_t st) {
    const int kk = QUERY ? k : k + 1;
    if (k < 1 || kk > 64 || n_src < kk || n_src > kLargeMax || n_q < 1 || batches < 1 ||
        batches > 65535 || n_q > INT32_MAX / 64)
        return MMPDE_ERR_INVALID_ARG;
    dim3 grid(ceil_div(n_q, kQueriesPerBlock), (unsigned)batches);
    const int cpl = ceil_div(n_src, 64);
    const float2 *p = (const float2 *)pts;
    const float2 *q = (const float2 *)qry;
    const int ns = (int)n_src, nq = (int)n_q;
    if (n_src > 4096) return launch_knn_large<QUERY>(p, q, batches, ns, nq, k, out, degenerate, st);
#define MMPDE_KNN_CASE(C)                                                                     \
    if (cpl <= C) {                                                                           \
        hipLaunchKernelGGL((knn_kernel<C, QUERY>), grid, dim3(256), 0, st, p, q, ns, nq, k, out, \
                           degenerate);                                                       \
        MMPDE_RET_LAUNCH();                                                                   \
        return MMPDE_OK;                                                                      \
    }
    MMPDE_KNN_CASE(4)
    MMPDE_KNN_CASE(8)
    MMPDE_KNN_CASE(16)
    MMPDE_KNN_CASE(24)
    MMPDE_KNN_CASE(32)
    MMPDE_KNN_CASE(40)
    MMPDE_KNN_CASE(48)
    MMPDE_KNN_CASE(56)
    MMPDE_KNN_CASE(64)
#undef MMPDE_KNN_CASE
    return MMPDE_ERR_UNSUPPORTED;
}

// ---------------------------------------------------------------------------
// Moving-mesh kNN from a static candidate list (exact, with a fallback).
// The DMM moves every node x_i = xi_i + d_i only a little, so the answer for a
// query q near a fixed reference point r_p (graph: r_p = xi_p, q = x_p; query:
// r_p = the fixed query point, q = qry_p) is almost always among cand[p] = the
// 128 nearest of r_p in the fixed mesh xi ((key, index) order).  A point j
// outside cand[p] has |xi_j - r_p| >= R = sqrt(key of cand[p][127]) (up to
// rounding), hence |x_j - q| >= max(R - |q - r_p|, dist(q, cell(xi_j))) -
// |d_j|, where cell(xi_j) is the point's cell in a 16 x 16 grid over the box of
// xi and |d_j| <= dcell[cell] = the largest displacement of that cell's points
// (mmpde_knn_moved_cells, per trajectory and step).  L = the minimum of that
// bound over the cells.  If the kk-th candidate distance is below L (every
// bound with a 2^-20 relative margin, which covers the fp32 rounding), no
// non-candidate can enter the first kk in (key, index) order, so the
// candidates sorted by (key, index) ARE the answer, ties included.  Otherwise
// the query joins its trajectory's fallback list, which knn_kernel answers.  A
// far-moved node only weakens the bound of the queries near its cell.
// ---------------------------------------------------------------------------
constexpr int kCandN = 128;
constexpr float kUp = 1.0f + 1.0f / 1048576.0f, kDown = 1.0f - 1.0f / 1048576.0f;

// cand[p] = the kCandN nearest of r_p in xi, (key, index) order: one
// workgroup per point, (key << 32 | index) pairs bitonic-sorted in LDS.  Built
// once per fixed mesh (and query set).
__global__ __launch_bounds__(256) void knn_table_kernel(const float2 *__restrict__ xi,
                                                        const float2 *__restrict__ ref, int n_per,
                                                        int32_t *__restrict__ cand) {
    __shared__ uint64_t sk[4096];
    const int p = blockIdx.x;
    const float2 q = ref[p];
    for (int j = threadIdx.x; j < 4096; j += 256)
        sk[j] = j < n_per ? (((uint64_t)key_f32(xi[j], q) << 32) | (uint32_t)j) : ~0ull;
    __syncthreads();
    for (int size = 2; size <= 4096; size <<= 1)
        for (int stride = size >> 1; stride > 0; stride >>= 1) {
            for (int t = threadIdx.x; t < 2048; t += 256) {
                const int i = 2 * t - (t & (stride - 1)), l = i + stride;
                const uint64_t a = sk[i], c = sk[l];
                if ((a > c) == ((i & size) == 0)) {
                    sk[i] = c;
                    sk[l] = a;
                }
            }
            __syncthreads();
        }
    if (threadIdx.x < kCandN) cand[(int64_t)p * kCandN + threadIdx.x] = (int32_t)(uint32_t)sk[threadIdx.x];
}

// Per trajectory b (one workgroup each): the box of xi (x0, y0, cell sizes
// hx, hy, their inverses, a margin eps that covers the rounding of the cell
// assignment) and dcell[c] >= max |x_bj - xi_j| over the points j with xi_j in
// cell c (-1: empty cell).  rec[b] = {dcell[256], box[8]}.
// 1024 threads (16 waves): the point loops are 2.5 iterations per thread at
// N = 2521, and the median is a rank count (256 broadcast LDS reads per cell)
// instead of a 36-stage bitonic network with a barrier per stage.
constexpr int kCellThreads = 1024;
__global__ __launch_bounds__(kCellThreads) void knn_cells_kernel(const float2 *__restrict__ x,
                                                                 const float2 *__restrict__ xi, int n_per,
                                                                 float *__restrict__ rec) {
    constexpr int NW = kCellThreads / 64;
    __shared__ float red[NW][4];
    __shared__ uint32_t cell[kCells];
    __shared__ float srt[kCells];
    const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    float mnx = 3.0e38f, mny = 3.0e38f, mxx = -3.0e38f, mxy = -3.0e38f;
    for (int i = tid; i < n_per; i += kCellThreads) {
        const float2 c = xi[i];
        mnx = fminf(mnx, c.x);
        mny = fminf(mny, c.y);
        mxx = fmaxf(mxx, c.x);
        mxy = fmaxf(mxy, c.y);
    }
    mnx = -wave_max_full(-mnx);
    mny = -wave_max_full(-mny);
    mxx = wave_max_full(mxx);
    mxy = wave_max_full(mxy);
    if (lane == 0) {
        red[wave][0] = mnx;
        red[wave][1] = mny;
        red[wave][2] = mxx;
        red[wave][3] = mxy;
    }
    if (tid < kCells) cell[tid] = 0u;  // empty
    __syncthreads();
    float x0 = red[0][0], y0 = red[0][1], x1 = red[0][2], y1 = red[0][3];
#pragma unroll
    for (int w = 1; w < NW; ++w) {
        x0 = fminf(x0, red[w][0]);
        y0 = fminf(y0, red[w][1]);
        x1 = fmaxf(x1, red[w][2]);
        y1 = fmaxf(y1, red[w][3]);
    }
    const float hx = (x1 - x0) / kCellG, hy = (y1 - y0) / kCellG;
    const float ihx = hx > 0.0f ? 1.0f / hx : 0.0f, ihy = hy > 0.0f ? 1.0f / hy : 0.0f;
    for (int i = tid; i < n_per; i += kCellThreads) {
        const float2 a = x[(int64_t)b * n_per + i], c = xi[i];
        const float dx = a.x - c.x, dy = a.y - c.y;
        const float d = sqrtf(dx * dx + dy * dy) * kUp;
        const int cx = min(max((int)((c.x - x0) * ihx), 0), kCellG - 1);
        const int cy = min(max((int)((c.y - y0) * ihy), 0), kCellG - 1);
        // non-negative floats order like their bits; stored as bits + 1 so
        // that 0 marks an empty cell
        atomicMax(&cell[cy * kCellG + cx], __float_as_uint(d) + 1u);
    }
    __syncthreads();
    float *r = rec + (int64_t)b * kCellRec;
    // cells on threads 0 .. 255 (waves 0 - 3)
    const uint32_t v = tid < kCells ? cell[tid] : 0u;
    const float dc = v == 0u ? -1.0f : __uint_as_float(v - 1u);
    if (tid < kCells) {
        r[tid] = dc;
        // the median over the non-empty cells of their largest displacement (the
        // statistic skip_above is compared with), empty cells last
        srt[tid] = v == 0u ? 3.0e38f : dc;
    }
    const float dall = wave_max_full(fmaxf(dc, 0.0f));
    const int nonempty = __popcll(__ballot(v != 0u));
    __syncthreads();  // red (read above) and srt
    if (lane == 0 && wave < kCells / 64) {
        red[wave][0] = dall;
        red[wave][1] = __int_as_float(nonempty);
    }
    __syncthreads();
    const int ne = __float_as_int(red[0][1]) + __float_as_int(red[1][1]) + __float_as_int(red[2][1]) +
                   __float_as_int(red[3][1]);
    if (tid < kCells) {
        // rank of this cell's value in (value, cell) order; the one of rank
        // ne / 2 is element ne / 2 of the sorted list
        const float mine = srt[tid];
        int rank = 0;
        for (int u = 0; u < kCells; ++u) {
            const float o = srt[u];
            rank += (o < mine || (o == mine && u < tid)) ? 1 : 0;
        }
        if (ne > 0 && rank == ne / 2) r[kCells + 6] = mine;
    }
    if (tid == 0) {
        const float eps = 1.0e-5f * fmaxf(x1 - x0, y1 - y0);
        r[kCells + 0] = x0;
        r[kCells + 1] = y0;
        r[kCells + 2] = hx;
        r[kCells + 3] = hy;
        r[kCells + 4] = eps;
        r[kCells + 5] = fmaxf(fmaxf(red[0][0], red[1][0]), fmaxf(red[2][0], red[3][0]));
        if (ne == 0) r[kCells + 6] = 0.0f;
        for (int i = 0; i < 2; ++i) {
            cell_last_miss(rec, b)[i] = 0;
            cell_any_miss(rec, b)[i] = 0;
            cell_skipped(rec, b)[i] = 0;
        }
    }
}

// Lower bounds on |x_j - q| over every j outside cand[p] (see above), <= 0 when
// they prove nothing; every rounding step errs downward.  R = the 128th
// candidate's distance from r_p, rq = R - |q - r_p|.  The global bound takes
// the trajectory's largest displacement; the per-cell bound, per cell, the
// distance from q to the cell's box (widened by eps) less the cell's largest
// displacement (never below the global one, costlier: only when that fails).
__device__ __forceinline__ float cand_rq(const float2 *__restrict__ xi, float2 rp, int n_per,
                                         const int32_t *__restrict__ cr, float2 q) {
    const int jl = min(max(cr[kCandN - 1], 0), n_per - 1);
    const float R = sqrtf(__uint_as_float(key_f32(xi[jl], rp))) * kDown;
    const float ddx = q.x - rp.x, ddy = q.y - rp.y;
    const float dq = sqrtf(ddx * ddx + ddy * ddy) * kUp;
    return (R - dq * kUp) * kDown;
}

__device__ __forceinline__ float cand_bound_global(float rq, const float *__restrict__ rec) {
    return (rq - rec[kCells + 5] * kUp) * kDown;
}

__device__ __forceinline__ float cand_bound_cells(float rq, float2 q, const float *__restrict__ rec, int lane) {
    const float x0 = rec[kCells], y0 = rec[kCells + 1], hx = rec[kCells + 2], hy = rec[kCells + 3];
    const float eps = rec[kCells + 4];
    float L = 3.0e38f;
    // every cell's record loaded first (a load whose value decides a branch
    // is waited for at once: one memory round trip per cell group otherwise),
    // then the bound of each occupied cell (dc >= 0) taken by a select
    float dcs[kCells / 64];
#pragma unroll
    for (int t = 0; t < kCells / 64; ++t) dcs[t] = rec[lane + 64 * t];
#pragma unroll
    for (int t = 0; t < kCells / 64; ++t) {
        const int c = lane + 64 * t;
        const float dc = dcs[t];
        const int cx = c % kCellG, cy = c / kCellG;
        const float lx = x0 + cx * hx - eps, ux = x0 + (cx + 1) * hx + eps;
        const float ly = y0 + cy * hy - eps, uy = y0 + (cy + 1) * hy + eps;
        const float ex = fmaxf(fmaxf(lx - q.x, q.x - ux), 0.0f);
        const float ey = fmaxf(fmaxf(ly - q.y, q.y - uy), 0.0f);
        const float dist = sqrtf(ex * ex + ey * ey) * kDown;
        const float bound = (fmaxf(dist, rq) - dc * kUp) * kDown;
        L = dc >= 0.0f ? fminf(L, bound) : L;
    }
    return -wave_max(-L);
}

// One wave per query point: the 128 candidates' keys (two per lane), one
// 128-wide (key, index) sort; the first kk are the answer when the kk-th
// candidate is closer than the bound.  QUERY = false: the moved-mesh graph
// (fp32 keys, self dropped, global indices, as knn_finish's graph branch; ref =
// xi); true: the kNN query of qry onto the moved mesh (fp64 keys, local
// indices; ref = the fixed query points the table was built for).
template <bool QUERY>
__global__ __launch_bounds__(256) void knn_cand_kernel(const float2 *__restrict__ x,
                                                       const float2 *__restrict__ qry,
                                                       const float2 *__restrict__ xi,
                                                       const float2 *__restrict__ ref, int n_per,
                                                       int64_t n_tot, int k,
                                                       const int32_t *__restrict__ cand,
                                                       const float *__restrict__ cells,
                                                       int32_t *__restrict__ out,
                                                       int32_t *__restrict__ degenerate,
                                                       uint8_t *__restrict__ miss, float skip_above) {
    typedef KeyTraits<QUERY> KT;
    typedef typename KT::key_t key_t;
    const int lane = threadIdx.x & 63;
    const int64_t p = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (p >= n_tot) return;  // wave-uniform
    const int b = (int)(p / n_per);
    const int pl = (int)(p - (int64_t)b * n_per);
    const float *rec = cells + (int64_t)b * kCellRec;
    // a trajectory whose median cell displacement exceeds skip_above does not
    // try the table: the fallback answers all its queries (wave-uniform)
    if (skip_above > 0.0f && rec[kCells + 6] > skip_above) {
        if (pl == 0 && lane == 0) cell_skipped(cells, b)[QUERY ? 1 : 0] = 1;
        return;
    }
    const float2 *X = x + (int64_t)b * n_per;
    const float2 q = QUERY ? qry[p] : X[pl];
    const int32_t *cr = cand + (int64_t)pl * kCandN;
    const float2 rp = ref[pl];
    const float rq = cand_rq(xi, rp, n_per, cr, q);
    const int kk = QUERY ? k : k + 1;
    // a query the table cannot answer is flagged for the fallback
    auto give_up = [&]() {
        if (lane == 0) {
            miss[p] = 1;
            cell_any_miss(cells, b)[QUERY ? 1 : 0] = 1;
        }
    };

    // Given up (wave-uniform) when the bound proves nothing, or when already
    // the unmoved kk-th candidate lies beyond it: the moved one then almost
    // never passes, and the sort would be wasted.  A heuristic only -- the
    // test after the sort decides.  The per-cell bound only when the global
    // one fails.
    const int jk = min(max(cr[kk - 1], 0), n_per - 1);
    const float dk0 = sqrtf(__uint_as_float(key_f32(xi[jk], rp)));
    float L = cand_bound_global(rq, rec);
    bool cells_done = false;
    if (!(L > 0.0f) || dk0 >= L) {
        L = cand_bound_cells(rq, q, rec, lane);
        cells_done = true;
        if (!(L > 0.0f) || dk0 >= L) {
            give_up();
            return;
        }
    }
    int i0 = min(max(cr[lane], 0), n_per - 1), i1 = min(max(cr[64 + lane], 0), n_per - 1);
    key_t k0 = 0, k1 = 0;
    bool sorted = false, tie = false;  // tie: as knn_finish's (QUERY)
    if constexpr (QUERY) if (kk < 64) {
        // sklearn's fp64 order, found by the cheaper fp32 (key, index) sort and
        // checked exactly: ranks 0 .. kk-1 must be in fp64 (key, index) order
        // (adjacent pairs compared on their exact keys), and the fp32 key of
        // rank kk must exceed rank kk-1's by the 64-ulp filter margin
        // (KeyTraits<true>::filter_threshold: the fp32 key is within 2^-22
        // relative of the fp64 one), so no later candidate's fp64 key can be
        // below rank kk-1's.  Otherwise (ties, near-ties) the fp64 sort below.
        uint32_t f0 = key_f32(X[i0], q), f1 = key_f32(X[i1], q);
        int j0 = i0, j1 = i1;
        wave_sort128(f0, j0, f1, j1, lane);
        const uint64_t e0 = KT::key(X[j0], q);
        const uint64_t en = __shfl(e0, (lane + 1) & 63, 64);
        const int jn = __shfl(j0, (lane + 1) & 63, 64);
        const bool pair_ok = lane >= kk - 1 || ki_less(e0, j0, en, jn);
        const uint32_t fk = lane_value(f0, kk), fk1 = lane_value(f0, kk - 1);
        if (__ballot(!pair_ok) == 0ull && fk > KT::filter_threshold(fk1)) {
            k0 = e0;
            i0 = j0;
            sorted = true;
            // rank kk's fp64 key exceeds rank kk - 1's (the margin): ties only inside
            tie = __ballot(lane < kk - 1 && e0 == en) != 0ull;
        }
    }
    if (!sorted) {
        k0 = KT::key(X[i0], q);
        k1 = KT::key(X[i1], q);
        wave_sort128(k0, i0, k1, i1, lane);
        if (QUERY) {  // element lane + 1 (lane 63: element 64, k1 of lane 0)
            const key_t n0 = (key_t)__shfl((unsigned long long)k0, (lane + 1) & 63, 64);
            const key_t n1 = lane_value(k1, 0);
            tie = __ballot(lane < kk && k0 == (lane == 63 ? n1 : n0)) != 0ull;
        }
    }
    const key_t key_kk = lane_value(k0, kk - 1);
    float d_kk;
    if constexpr (QUERY)
        d_kk = (float)sqrt(__longlong_as_double((long long)key_kk)) * kUp;
    else
        d_kk = sqrtf(__uint_as_float(key_kk)) * kUp;
    if (!(d_kk < L) && !cells_done) L = cand_bound_cells(rq, q, rec, lane);
    if (!(d_kk < L)) {  // same on every lane
        give_up();
        return;
    }
    if (lane == 0) miss[p] = 0;
    const int mi = i0, rank = lane;
    if (QUERY) {
        if (lane < kk) out[p * k + rank] = mi;
        if (tie && lane == 0 && degenerate) atomicAdd(degenerate, 1);
    } else {
        const uint64_t smask = __ballot(lane < kk && mi == pl);
        const bool has_self = smask != 0ull;
        const int self_rank = has_self ? lane_value(rank, __ffsll((unsigned long long)smask) - 1) : kk;
        const int pos = rank - ((has_self && rank > self_rank) ? 1 : 0);
        if (lane < kk && !(has_self && mi == pl) && pos < k) out[p * k + pos] = b * n_per + mi;
        if (!has_self && lane == 0 && degenerate) atomicAdd(degenerate, 1);
    }
}

// torch_cluster radius_graph(x, r, batch, loop=False, max_num_neighbors)
// (reference data_creator_2d.py:257-258): radius(x, x, ..., max_num_neighbors
// + 1) scans the query's segment in index order and keeps the first w = max_nn
// + 1 points with d2 < r2 (the query itself included), then the self loop is
// dropped.  One wave per query, 64 candidates per step, ballot order = index
// order; stops once w points were taken.  nbr [n, w] global sources ascending,
// padded with -1; deg [n] = entries kept (w - 1 or w).
__global__ __launch_bounds__(256) void radius_kernel(const float2 *__restrict__ pts, int n_per,
                                                     float r2, int w, int32_t *__restrict__ nbr,
                                                     int32_t *__restrict__ deg) {
    const int b = blockIdx.y;
    const int q = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (q >= n_per) return;  // wave-uniform: no barrier below
    const float2 *P = pts + (int64_t)b * n_per;
    const float2 qp = P[q];
    const uint64_t below = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    int32_t *row = nbr + ((int64_t)b * n_per + q) * w;
    int taken = 0, kept = 0;
    for (int j0 = 0; j0 < n_per && taken < w; j0 += 64) {
        const int j = j0 + lane;
        const bool hit = j < n_per && key_f32(P[j], qp) < __float_as_uint(r2);
        const uint64_t hm = __ballot(hit);
        const bool take = hit && taken + __popcll(hm & below) < w;
        const uint64_t tm = __ballot(take);
        const uint64_t km = __ballot(take && j != q);  // self loop dropped
        if (take && j != q) row[kept + __popcll(km & below)] = b * n_per + j;
        taken += __popcll(tm);
        kept += __popcll(km);
    }
    for (int e = kept + lane; e < w; e += 64) row[e] = -1;
    if (lane == 0) deg[(int64_t)b * n_per + q] = kept;
}

__global__ void edge_index_kernel(const int32_t *__restrict__ nbr, int64_t n, int k,
                                  int64_t *__restrict__ ei) {
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t ne = n * k;
    if (e < ne) {
        ei[e] = nbr[e];
        ei[ne + e] = e / k;
    }
}

}  // namespace

extern "C" int mmpde_knn_graph(const float *pos, int64_t batches, int64_t n_per, int k,
                               int32_t *nbr_out, int32_t *degenerate, mmpde_stream_t stream) {
    MMPDE_REQUIRE(pos && nbr_out);
    return launch_knn<false>(pos, nullptr, batches, n_per, n_per, k, nbr_out, degenerate,
                             as_stream(stream));
}

extern "C" int mmpde_knn_candidates(const float *xi, const float *ref, int64_t n_per, int32_t *cand_out,
                                    mmpde_stream_t stream) {
    MMPDE_REQUIRE(xi && cand_out && n_per >= kCandN && n_per <= 4096);
    hipLaunchKernelGGL(knn_table_kernel, dim3((unsigned)n_per), dim3(256), 0, as_stream(stream),
                       (const float2 *)xi, (const float2 *)(ref ? ref : xi), (int)n_per, cand_out);
    MMPDE_RET_LAUNCH();
    return MMPDE_OK;
}

extern "C" int64_t mmpde_knn_moved_cells_bytes(int64_t batches) {
    return batches < 0 ? 0 : batches * kCellRec * (int64_t)sizeof(float);
}

extern "C" int mmpde_knn_moved_cells(const float *pos, const float *xi, int64_t batches, int64_t n_per,
                                     float *cells_out, mmpde_stream_t stream) {
    MMPDE_REQUIRE(pos && xi && cells_out && batches >= 1 && batches <= 65535 && n_per >= 1 &&
                  n_per <= INT32_MAX);
    hipLaunchKernelGGL(knn_cells_kernel, dim3((unsigned)batches), dim3(kCellThreads), 0, as_stream(stream),
                       (const float2 *)pos, (const float2 *)xi, (int)n_per, cells_out);
    MMPDE_RET_LAUNCH();
    return MMPDE_OK;
}

// The median over reference points p of R128(p) - R_kk(p) (the 128th and the
// kk-th candidate distance of r_p in xi), times `scale`.  One workgroup,
// bitonic sort in LDS.
__global__ __launch_bounds__(256) void knn_margin_kernel(const float2 *__restrict__ xi,
                                                         const float2 *__restrict__ ref, int n_per,
                                                         const int32_t *__restrict__ cand, int kk,
                                                         float scale, float *__restrict__ out) {
    __shared__ float sm[4096];
    for (int p = threadIdx.x; p < 4096; p += 256) {
        float m = 3.0e38f;
        if (p < n_per) {
            const float2 r = ref[p];
            const int32_t *cr = cand + (int64_t)p * kCandN;
            const int j1 = min(max(cr[kCandN - 1], 0), n_per - 1), jk = min(max(cr[kk - 1], 0), n_per - 1);
            m = sqrtf(__uint_as_float(key_f32(xi[j1], r))) - sqrtf(__uint_as_float(key_f32(xi[jk], r)));
        }
        sm[p] = m;
    }
    __syncthreads();
    for (int size = 2; size <= 4096; size <<= 1)
        for (int stride = size >> 1; stride > 0; stride >>= 1) {
            for (int t = threadIdx.x; t < 2048; t += 256) {
                const int i = 2 * t - (t & (stride - 1)), l = i + stride;
                const float a = sm[i], c = sm[l];
                if ((a > c) == ((i & size) == 0)) {
                    sm[i] = c;
                    sm[l] = a;
                }
            }
            __syncthreads();
        }
    if (threadIdx.x == 0) out[0] = scale * sm[n_per / 2];
}

__global__ void knn_misses_kernel(const float *__restrict__ cells, int batches, int32_t *__restrict__ out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < 2 * batches) out[i] = cell_last_miss(cells, i >> 1)[i & 1];
}

extern "C" int mmpde_knn_table_misses(const float *cells, int64_t batches, int32_t *misses_out,
                                      mmpde_stream_t stream) {
    MMPDE_REQUIRE(cells && misses_out && batches >= 1 && batches <= 65535);
    hipLaunchKernelGGL(knn_misses_kernel, dim3(ceil_div(2 * batches, 256)), dim3(256), 0, as_stream(stream),
                       cells, (int)batches, misses_out);
    MMPDE_RET_LAUNCH();
    return MMPDE_OK;
}

extern "C" int mmpde_knn_skip_threshold(const float *xi, const float *ref, int64_t n_per, const int32_t *cand,
                                        int kk, int moved_queries, float *out, mmpde_stream_t stream) {
    MMPDE_REQUIRE(xi && cand && out && n_per >= kCandN && n_per <= 4096 && kk >= 1 && kk <= kCandN);
    // a moved query spends the margin twice (its own offset and its
    // neighbours' displacement), a query at its reference point once
    hipLaunchKernelGGL(knn_margin_kernel, dim3(1), dim3(256), 0, as_stream(stream), (const float2 *)xi,
                       (const float2 *)(ref ? ref : xi), (int)n_per, cand, kk, moved_queries ? 0.5f : 1.0f,
                       out);
    MMPDE_RET_LAUNCH();
    return MMPDE_OK;
}

extern "C" int64_t mmpde_knn_graph_cand_scratch_bytes(int64_t batches, int64_t n_per) {
    return batches * n_per;  // the miss flags
}

// The candidate path: the candidate kernel, then the full search for the
// queries it could not answer (knn_kernel's miss mode: its cost follows the
// number of such queries, and is the plain search's when most missed).
template <bool QUERY>
static int knn_cand_launch(const float *pos, const float *qry, const float *xi, const float *ref,
                           const float *cells, float skip_above, int64_t batches, int64_t n_per, int k,
                           const int32_t *cand, int32_t *out, int32_t *degenerate, void *scratch,
                           hipStream_t st) {
    uint8_t *miss = (uint8_t *)scratch;
    const int64_t n_tot = batches * n_per;
    const float2 *x = (const float2 *)pos, *q = (const float2 *)qry, *x0 = (const float2 *)xi;
    hipLaunchKernelGGL(knn_cand_kernel<QUERY>, dim3((unsigned)ceil_div(n_tot, 4)), dim3(256), 0, st, x, q, x0,
                       (const float2 *)ref, (int)n_per, n_tot, k, cand, cells, out, degenerate, miss,
                       skip_above);
    MMPDE_RET_LAUNCH();
    dim3 grid(ceil_div(n_per, kQueriesPerBlock), (unsigned)batches);
    const int ns = (int)n_per, cpl = ceil_div(n_per, 64);
#define MMPDE_KNN_FALLBACK(C)                                                                         \
    if (cpl <= C) {                                                                                   \
        hipLaunchKernelGGL((knn_kernel<C, QUERY, kQueriesPerBlock>), grid, dim3(256), 0, st, x, QUERY ? q : x, ns, \
                           ns, k, out, degenerate, (const uint8_t *)miss, (float *)cells, QUERY ? 1 : 0); \
        MMPDE_RET_LAUNCH();                                                                           \
        return MMPDE_OK;                                                                              \
    }
    MMPDE_KNN_FALLBACK(4)
    MMPDE_KNN_FALLBACK(8)
    MMPDE_KNN_FALLBACK(16)
    MMPDE_KNN_FALLBACK(24)
    MMPDE_KNN_FALLBACK(32)
    MMPDE_KNN_FALLBACK(40)
    MMPDE_KNN_FALLBACK(48)
    MMPDE_KNN_FALLBACK(56)
    MMPDE_KNN_FALLBACK(64)
#undef MMPDE_KNN_FALLBACK
    return MMPDE_ERR_UNSUPPORTED;
}

static bool cand_path_applies(int64_t batches, int64_t n_per, int kk) {
    // the answer inside the first 64 sorted candidates; the register kernels' sizes
    return kk >= 1 && kk <= 64 && n_per >= kCandN && n_per <= 4096 && batches >= 1 && batches <= 65535 &&
           batches * n_per <= INT32_MAX;
}

extern "C" int mmpde_knn_graph_cand(const float *pos, const float *xi, const float *cells, float skip_above,
                                    int64_t batches, int64_t n_per, int k, const int32_t *cand, int32_t *nbr_out,
                                    int32_t *degenerate, void *scratch, mmpde_stream_t stream) {
    MMPDE_REQUIRE(pos && xi && cells && cand && nbr_out && scratch);
    hipStream_t st = as_stream(stream);
    if (k < 1 || !cand_path_applies(batches, n_per, k + 1))
        return launch_knn<false>(pos, nullptr, batches, n_per, n_per, k, nbr_out, degenerate, st);
    return knn_cand_launch<false>(pos, nullptr, xi, xi, cells, skip_above, batches, n_per, k, cand, nbr_out,
                                  degenerate, scratch, st);
}

extern "C" int mmpde_knn_query_cand(const float *src, const float *qry, const float *xi, const float *ref,
                                    const float *cells, float skip_above, int64_t batches, int64_t n_per, int k,
                                    const int32_t *cand, int32_t *idx_out, int32_t *ties, void *scratch,
                                    mmpde_stream_t stream) {
    MMPDE_REQUIRE(src && qry && xi && cells && cand && idx_out && scratch);
    hipStream_t st = as_stream(stream);
    if (!cand_path_applies(batches, n_per, k))
        return launch_knn<true>(src, qry, batches, n_per, n_per, k, idx_out, ties, st);
    return knn_cand_launch<true>(src, qry, xi, ref ? ref : xi, cells, skip_above, batches, n_per, k, cand,
                                 idx_out, ties, scratch, st);
}

extern "C" int mmpde_knn_query(const float *src, const float *qry, int64_t batches,
                               int64_t n_src, int64_t n_qry, int k, int32_t *idx_out, int32_t *ties,
                               mmpde_stream_t stream) {
    MMPDE_REQUIRE(src && qry && idx_out);
    return launch_knn<true>(src, qry, batches, n_src, n_qry, k, idx_out, ties, as_stream(stream));
}

extern "C" int mmpde_radius_graph(const float *pos, int64_t batches, int64_t n_per, float r,
                                  int max_num_neighbors, int32_t *nbr_out, int32_t *degree_out,
                                  mmpde_stream_t stream) {
    MMPDE_REQUIRE(pos && nbr_out && degree_out);
    MMPDE_REQUIRE(batches > 0 && batches <= 65535 && n_per > 0 && n_per <= INT32_MAX &&
                  batches * n_per <= INT32_MAX && max_num_neighbors > 0 && r > 0.0f);
    // torch_cluster squares r on the host in double and hands the kernel a float
    const float r2 = (float)((double)r * (double)r);
    hipLaunchKernelGGL(radius_kernel, dim3((unsigned)ceil_div(n_per, 4), (unsigned)batches),
                       dim3(256), 0, as_stream(stream), (const float2 *)pos, (int)n_per, r2,
                       max_num_neighbors + 1, nbr_out, degree_out);
    MMPDE_RET_LAUNCH();
    return MMPDE_OK;
}

extern "C" int mmpde_edge_index_from_nbr(const int32_t *nbr, int64_t n, int k,
                                         int64_t *edge_index, mmpde_stream_t stream) {
    MMPDE_REQUIRE(nbr && edge_index && n > 0 && k > 0);
    const int64_t ne = n * k;
    hipLaunchKernelGGL(edge_index_kernel, dim3(ceil_div(ne, 256)), dim3(256), 0,
                       as_stream(stream), nbr, n, k, edge_index);
    MMPDE_RET_LAUNCH();
    return MMPDE_OK;
}
