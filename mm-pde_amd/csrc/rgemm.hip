// Row GEMMs of the training path (reference train_helper_2d.py:114-126:
// loss.backward() through the train-mode MP_PDE_Solver_2D, gnn_2d.py:53-69,
// 99-106, and ItpNet, interpolate.py:79-93).  The Linears act on rows (n =
// B x 2521 nodes or queries) with <= 128 outputs per block:
//
//   rgemm     y = x W^T (layout NT: the forward) or y = g W (NN: the input
//             gradient), the concatenated inputs of the reference (cat(h, agg,
//             t), cat(h_i, h_j, u_i - u_j, dx, dy, t_i)) read in place as two
//             K halves plus a <= 4-column small segment, with the bias, ReLU,
//             ReLU-backward masks and the residual accumulation fused in.
//   rgemm_tn  dW = G^T X and db = sum G over the row axis in fixed row chunks
//             (partials, then a fixed-order sum): deterministic.
//
// Exact fp32 products on v_mfma_f32_32x32x2_f32 (lane l supplies A[l & 31][l
// >> 5] and B[l >> 5][l & 31]).  Operand reuse is what bounds these kernels
// (each MFMA consumes one value per lane of A and of B, 64 cycles of matrix
// work per 512 B of operands): every wave computes a 2 x 2 block of 32 x 32
// tiles, so each loaded operand feeds two MFMAs.
#include "common.hpp"

#include <algorithm>
#include <cstdlib>

namespace {


__device__ __forceinline__ float4 mask4(float4 a, const float4 &q) {
    return make_float4(q.x > 0.0f ? a.x : 0.0f, q.y > 0.0f ? a.y : 0.0f, q.z > 0.0f ? a.z : 0.0f,
                       q.w > 0.0f ? a.w : 0.0f);
}

// rgemm: one wave = 64 rows x 64 columns (row tiles rt, column tiles ct, each
// 32 x 32); workgroup = 4 waves = 128 rows x 128 columns.  K: k-lane 0 walks
// half 0, k-lane 1 half 1 (two input tensors side by side); VEC (kh % 4 == 0,
// 16-byte aligned rows; NT: W rows too): float4 operand loads, the next 4-k
// step's loaded under the current step's 16 MFMAs; two accumulation chains
// per tile (alternate 4-k steps), added at the end.
template <int LAYOUT, bool VEC, bool AMASK, bool XS>
__global__ __launch_bounds__(256, 2) void rgemm_kernel(mmpde_rgemm_args g) {
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int h = lane >> 5, j = lane & 31;
    const int p = blockIdx.y;
    const int ncols = g.ncols[p];
    const int cbase = 64 * (wave & 1);
    const int64_t row0 = (int64_t)blockIdx.x * 128 + 64 * (wave >> 1);
    const int64_t m = g.m;
    if (cbase >= ncols || row0 >= m) return;      // wave-uniform: no column / row of this wave
    const int kh = g.kh;
    f32x16 acc[2][2][2];  // [row tile][column tile][chain]
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b) acc[a][b][0] = acc[a][b][1] = (f32x16){0};
    if (kh > 0) {
        const int64_t ldw = g.ldw;
        const float *ap[2], *mp[2], *wp[2];
#pragma unroll
        for (int t = 0; t < 2; ++t) {
            const int64_t row = min(row0 + 32 * t + j, m - 1);    // clamped: loads stay in bounds
            ap[t] = g.a[h] + row * g.lda[h];
            mp[t] = AMASK ? g.amask[h] + row * g.lda[h] : nullptr;
            const int colc = min(cbase + 32 * t + j, ncols - 1);  // clamped for the W loads
            wp[t] = LAYOUT == MMPDE_RGEMM_NT ? g.w[h] + (g.wc[p] + colc) * ldw + g.wk[p]
                                             : g.w[h] + g.wk[p] * ldw + g.wc[p] + colc;
        }
        if (VEC) {
            struct Ops {
                float4 a[2], w[2];
            };
            auto load = [&](int s, Ops &o) {
#pragma unroll
                for (int t = 0; t < 2; ++t) {
                    float4 a = *(const float4 *)(ap[t] + s);
                    if (AMASK) a = mask4(a, *(const float4 *)(mp[t] + s));
                    o.a[t] = a;
                    if (LAYOUT == MMPDE_RGEMM_NT) {
                        o.w[t] = *(const float4 *)(wp[t] + s);
                    } else {
                        const float *w = wp[t] + s * ldw;
                        o.w[t] = make_float4(w[0], w[ldw], w[2 * ldw], w[3 * ldw]);
                    }
                }
            };
            auto step = [&](const Ops &o, int c) {
#pragma unroll
                for (int q = 0; q < 4; ++q)
#pragma unroll
                    for (int rt = 0; rt < 2; ++rt)
#pragma unroll
                        for (int ct = 0; ct < 2; ++ct)
                            acc[rt][ct][c] = mfma32(f4c(o.a[rt], q), f4c(o.w[ct], q), acc[rt][ct][c]);
            };
            // two 4-k steps per iteration (one per chain); the next iteration's
            // operands are loaded (clamped to the last step: in bounds, unused
            // past kh) before this iteration's 32 MFMAs
            Ops c0, c1, n0, n1;
            load(0, c0);
            load(min(4, kh - 4), c1);
            for (int s = 0; s < kh; s += 8) {
                load(min(s + 8, kh - 4), n0);
                load(min(s + 12, kh - 4), n1);
                step(c0, 0);
                if (s + 4 < kh) step(c1, 1);  // wave-uniform
                c0 = n0;
                c1 = n1;
            }
        } else {
            for (int s = 0; s < kh; s += 2) {
#pragma unroll
                for (int c = 0; c < 2; ++c) {
                    if (s + c >= kh) break;  // wave-uniform
                    const int k = s + c;
                    float a[2], w[2];
#pragma unroll
                    for (int t = 0; t < 2; ++t) {
                        a[t] = ap[t][k];
                        if (AMASK) a[t] = mp[t][k] > 0.0f ? a[t] : 0.0f;
                        w[t] = LAYOUT == MMPDE_RGEMM_NT ? wp[t][k] : wp[t][(int64_t)k * ldw];
                    }
#pragma unroll
                    for (int rt = 0; rt < 2; ++rt)
#pragma unroll
                        for (int ct = 0; ct < 2; ++ct)
                            acc[rt][ct][c] = mfma32(a[rt], w[ct], acc[rt][ct][c]);
                }
            }
        }
    }
    // epilogue: D[acc_row(r)][j] of each tile
    const float *om = g.omask[p];
    const bool accum = g.accumulate[p] != 0;
    const int ns = XS ? g.ns[p] : 0;
    float *out = g.out[p];
#pragma unroll
    for (int ct = 0; ct < 2; ++ct) {
        const int col = cbase + 32 * ct + j;
        if (col >= ncols) continue;
        const float bias = g.bias[p] ? g.bias[p][col] : 0.0f;
        float xw[4] = {0.0f, 0.0f, 0.0f, 0.0f};
        if (XS) {
#pragma unroll
            for (int e = 0; e < 4; ++e)
                if (e < ns)
                    xw[e] = g.xscale[p] * (LAYOUT == MMPDE_RGEMM_NT ? g.xw[p][(int64_t)col * g.ldxw + e]
                                                                    : g.xw[p][(int64_t)e * g.ldxw + col]);
        }
#pragma unroll
        for (int rt = 0; rt < 2; ++rt) {
            const f32x16 d = acc[rt][ct][0] + acc[rt][ct][1];
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int64_t i = row0 + 32 * rt + acc_row(r, lane);
                if (i >= m) continue;
                float y = d[r] + bias;
                if (XS) {
#pragma unroll
                    for (int e = 0; e < 4; ++e)
                        if (e < ns) y = fmaf(g.xs[i * g.ldxs + e], xw[e], y);
                }
                if (g.relu) y = fmaxf(y, 0.0f);
                if (om) y = om[i * g.ldom[p] + col] > 0.0f ? y : 0.0f;
                float *o = out + i * g.ldo[p] + col;
                *o = accum ? *o + y : y;
            }
        }
    }
}

// The weight-stationary form for kh in {32, 64, 128} (every shape of the GNN
// layers): persistent workgroups of 4 waves, wave w owning output columns
// 32 w .. 32 w + 31 of the part, its B operand (W, kh values per lane) in
// registers for the whole launch; the rows stream through LDS in tiles of 32
// (both K halves, the ReLU-backward input mask applied while staging), the
// next tile loaded into registers under the current tile's kh MFMAs and
// stored to the other LDS buffer; one barrier per tile.
template <int LAYOUT, int KH, bool AMASK, bool XS>
__global__ __launch_bounds__(256, KH == 128 ? 1 : 2) void rgemm_ws_kernel(mmpde_rgemm_args g) {
    constexpr int PITCH = 2 * KH + 4;        // floats per staged row (both halves)
    constexpr int NF4 = 32 * 2 * KH / 4;     // float4 pieces of a tile
    constexpr int PER = NF4 / 256;           // per thread
    __shared__ float xt[2][32 * PITCH];
    const int tid = threadIdx.x;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
    const int h = lane >> 5, j = lane & 31;
    const int p = blockIdx.y;
    const int ncols = g.ncols[p];
    const bool active = 32 * wave < ncols;   // wave-uniform: this wave has output columns
    const int col = 32 * wave + j;
    const int colc = min(col, ncols - 1);
    const int64_t m = g.m;
    const int64_t ntiles = (m + 31) / 32;
    // W operand: lane (j, h) holds B_h(s, colc) for s < KH
    float wreg[KH];
    {
        const int64_t ldw = g.ldw;
        if (LAYOUT == MMPDE_RGEMM_NT) {
            const float *wp = g.w[h] + (g.wc[p] + colc) * ldw + g.wk[p];
#pragma unroll
            for (int s = 0; s < KH; s += 4) {
                const float4 v = *(const float4 *)(wp + s);
                wreg[s] = v.x;
                wreg[s + 1] = v.y;
                wreg[s + 2] = v.z;
                wreg[s + 3] = v.w;
            }
        } else {
            const float *wp = g.w[h] + g.wk[p] * ldw + g.wc[p] + colc;
#pragma unroll
            for (int s = 0; s < KH; ++s) wreg[s] = wp[(int64_t)s * ldw];
        }
    }
    // staging: piece f = tid + 256 u -> row f / (KH / 2), half, float4 q; the
    // small segment's row (XS: ns <= 4 values) goes to the row's 4 pad floats.
    // Every load is unconditional (the last tile re-read past the end): a load
    // under a condition is waited for where the condition ends.
    const float *a0 = g.a[0], *a1 = g.a[1];
    const float *m0 = AMASK ? g.amask[0] : nullptr, *m1 = AMASK ? g.amask[1] : nullptr;
    const int64_t lda0 = g.lda[0], lda1 = g.lda[1];
    const int ns = XS ? g.ns[p] : 0;
    const float *xs = g.xs;
    const int64_t ldxs = g.ldxs;
    float4 stg[PER];
    float4 sxs;
    auto fetch = [&](int64_t tile) {
#pragma unroll
        for (int u = 0; u < PER; ++u) {
            const int f = tid + 256 * u;
            const int r = f / (KH / 2), rem = f % (KH / 2), hh = rem / (KH / 4), q = rem % (KH / 4);
            const int64_t row = min(tile * 32 + r, m - 1);
            const int64_t off = row * (hh ? lda1 : lda0) + 4 * q;
            float4 v = *(const float4 *)((hh ? a1 : a0) + off);
            if (AMASK) v = mask4(v, *(const float4 *)((hh ? m1 : m0) + off));
            stg[u] = v;
        }
        if (XS && tid < 32) {
            const float *xr = xs + min(tile * 32 + tid, m - 1) * ldxs;
            sxs = make_float4(xr[0], xr[min(1, ns - 1)], xr[min(2, ns - 1)], xr[min(3, ns - 1)]);
        }
    };
    auto stash = [&](float *buf) {
#pragma unroll
        for (int u = 0; u < PER; ++u) {
            const int f = tid + 256 * u;
            const int r = f / (KH / 2), rem = f % (KH / 2), hh = rem / (KH / 4), q = rem % (KH / 4);
            *(float4 *)(buf + r * PITCH + hh * KH + 4 * q) = stg[u];
        }
        if (XS && tid < 32) *(float4 *)(buf + tid * PITCH + 2 * KH) = sxs;
    };
    // epilogue constants of this lane's column
    const float bias = active && g.bias[p] ? g.bias[p][colc] : 0.0f;
    float xw[4] = {0.0f, 0.0f, 0.0f, 0.0f};
    if (XS && active) {
#pragma unroll
        for (int e = 0; e < 4; ++e)
            if (e < ns)
                xw[e] = g.xscale[p] * (LAYOUT == MMPDE_RGEMM_NT ? g.xw[p][(int64_t)colc * g.ldxw + e]
                                                                : g.xw[p][(int64_t)e * g.ldxw + colc]);
    }
    const float *om = g.omask[p];
    const bool accum = g.accumulate[p] != 0;
    const bool relu = g.relu != 0;
    const int64_t ldom = g.ldom[p], ldo = g.ldo[p];
    float *out = g.out[p];
    int64_t tile = blockIdx.x;
    if (tile >= ntiles) return;  // workgroup-uniform, before any barrier
    int cur = 0;
    fetch(tile);
    stash(xt[0]);
    __syncthreads();
    for (;;) {
        const int64_t next = tile + gridDim.x;
        const bool more = next < ntiles;  // workgroup-uniform
        fetch(min(next, ntiles - 1));
        if (active) {
            // the epilogue's row inputs (output mask, the old output values) are
            // loaded before the MFMAs, so their latency hides under them
            float em[16], eo[16];
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int64_t i = min(tile * 32 + acc_row(r, lane), m - 1);
                em[r] = om ? om[i * ldom + colc] : 1.0f;
                eo[r] = accum ? out[i * ldo + colc] : 0.0f;
            }
            const float *xr = xt[cur] + j * PITCH + h * KH;  // A: row j, half h
            f32x16 c0 = {0}, c1 = {0};
#pragma unroll
            for (int s = 0; s < KH; s += 4) {
                const float4 a = *(const float4 *)(xr + s);
                c0 = mfma32(a.x, wreg[s], c0);
                c1 = mfma32(a.y, wreg[s + 1], c1);
                c0 = mfma32(a.z, wreg[s + 2], c0);
                c1 = mfma32(a.w, wreg[s + 3], c1);
            }
            const f32x16 d = c0 + c1;
            // pin the uses of em / eo after the MFMAs (the compiler would
            // otherwise test them right after their loads, waiting there)
            const float dep = d[0];
#pragma unroll
            for (int r = 0; r < 16; ++r) asm volatile("" : "+v"(em[r]), "+v"(eo[r]) : "v"(dep));
            if (col < ncols) {
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int rr = acc_row(r, lane);
                    const int64_t i = tile * 32 + rr;
                    if (i >= m) continue;
                    float y = d[r] + bias;
                    if (XS) {
                        const float4 x4 = *(const float4 *)(xt[cur] + rr * PITCH + 2 * KH);
                        y = fmaf(x4.x, xw[0], y);   // xw[e] = 0 for e >= ns
                        y = fmaf(x4.y, xw[1], y);
                        y = fmaf(x4.z, xw[2], y);
                        y = fmaf(x4.w, xw[3], y);
                    }
                    if (relu) y = fmaxf(y, 0.0f);
                    if (om) y = em[r] > 0.0f ? y : 0.0f;
                    out[i * ldo + col] = accum ? eo[r] + y : y;
                }
            }
        }
        if (!more) break;
        stash(xt[cur ^ 1]);
        __syncthreads();  // the other buffer is complete; this one's readers are done
        cur ^= 1;
        tile = next;
    }
}

int rgemm_cus() {
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
        cus = 256;
    return cus;
}

// ---------------------------------------------------------------------------
// dW = G^T X over the rows.  Partials: workspace [chunks][128][cols]; the
// column space is every segment rounded up to 64 columns (segment s starts at
// base(s) = the sum of the rounded widths before it), then the ns
// small-segment columns, then db.  Workgroup (k block of 64 columns, chunk, c
// block of 64 columns): 4 waves over the same 64 x 64 output block, wave w
// the w-th quarter of the chunk's rows; the block is 2 x 2 tiles of 32 x 32:
// lane j of tile (ct, kt) holds c = c0 + 2 j + ct and k = k0 + 2 j + kt, so one
// float2 load of G and one of X per row feed four MFMAs (two rows per MFMA,
// row parity = k-lane).  The four waves'
// blocks are then added through LDS in wave order (fixed: deterministic).
// The k block 0 workgroups also sum the small segment and db from the same G
// values on the VALU.
// ---------------------------------------------------------------------------
struct TnArgs {
    mmpde_rgemm_tn_args g;
    int cols, kbig;  // partial columns; rounded big-segment columns
    int base[3];     // first partial column of each segment
    float *part;
    int nkb, ncb, chunks;  // k blocks, c blocks, row chunks
};

// Workgroup -> (k block, chunk, c block).  The k and c blocks of one chunk read
// the same G and X rows; workgroups are dealt to the 8 XCDs round-robin by id
// (b and b + 8 share an XCD and its L2), so the nkb * ncb blocks of chunk c take
// ids 8 (nb (c / 8) + b) + c % 8: one XCD, consecutive slots (dispatched
// together), and each row is fetched from HBM once instead of once per block.
// Ids past the last chunk exit at once.  Speed only: every block computes the
// same partial as before.
struct TnBlock {
    int kb, chunk, cb;
};
__device__ __forceinline__ TnBlock tn_block(const TnArgs &t) {
    const int id = blockIdx.x, nb = t.nkb * t.ncb;
    const int slot = id >> 3, b = slot % nb;
    return {64 * (b % t.nkb), (slot / nb) * 8 + (id & 7), 64 * (b / t.nkb)};
}

__device__ __forceinline__ float2 ld2(const float *p, bool vec) {
    return vec ? *(const float2 *)p : make_float2(p[0], p[1]);
}

// row-step batches per wave of the straight-line main loop (32 steps = the
// 64 rows of a 256-row chunk's quarter)
constexpr int kTnBatches = 8;

#ifndef MMPDE_TN_XS_OCC
#define MMPDE_TN_XS_OCC 3
#endif

template <bool GMASK, bool VEC, bool XS>
__global__ __launch_bounds__(256, GMASK && XS ? 2 : (XS ? MMPDE_TN_XS_OCC : 3)) void rgemm_tn_partial_kernel(TnArgs t) {
    constexpr int NRED = 64 + 2 + 8;  // per lane: the block (4 tiles x 16), db (2), small segment (2 x 4)
    __shared__ float red[NRED][64];
    const mmpde_rgemm_tn_args &g = t.g;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int par = lane >> 5, j = lane & 31;
    const TnBlock blk = tn_block(t);
    if (blk.chunk >= t.chunks) return;    // the whole workgroup: no barrier reached
    const int chunk = blk.chunk;
    const int gcols = g.gcols;
    const int cb = blk.cb;                // first G column of this block
    const int kb = blk.kb;                // first partial column of this block
    const int64_t c0r = (int64_t)chunk * g.chunk_rows;
    const int64_t c1r = min(c0r + (int64_t)g.chunk_rows, g.m);
    // even rows per wave, 4 * qrows >= chunk_rows (the same split as chunk_rows / 4
    // rounded up to even for every multiple of 4)
    const int64_t qrows = ((g.chunk_rows + 3) / 4 + 1) & ~(int64_t)1;
    const int64_t r0 = min(c0r + wave * qrows, c1r), r1 = min(r0 + qrows, c1r);
    // G columns c0, c0 + 1 of this lane (tiles ct = 0, 1); clamped loads, masked values
    const int c0 = cb + 2 * j;
    const bool cl0 = c0 < gcols, cl1 = c0 + 1 < gcols;
    const int cc = gcols >= 2 ? min(c0, gcols - 2) : 0;
    // X segment of this block, columns k0, k0 + 1 of this lane (tiles kt = 0, 1)
    int seg = 0;
    while (seg < g.nseg - 1 && kb >= t.base[seg + 1]) ++seg;
    const int kx = g.kx[seg];
    const int k0 = kb - t.base[seg] + 2 * j;
    const bool kl0 = k0 < kx, kl1 = k0 + 1 < kx;
    const int kc = kx >= 2 ? min(k0, kx - 2) : 0;
    const float *xp = g.x[seg] + kc;
    const int64_t ldx = g.ldx[seg];
    const float *gp = g.g + cc;
    const float *gm = GMASK ? g.gmask + cc : nullptr;
    const bool first = kb == 0;
    const int ns = first ? g.ns : 0;
    // [c tile][k tile]: four independent accumulators cover the MFMA latency
    f32x16 acc[2][2];
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b) acc[a][b] = (f32x16){0};
    float sx[2][4] = {{0.0f, 0.0f, 0.0f, 0.0f}, {0.0f, 0.0f, 0.0f, 0.0f}}, sb[2] = {0.0f, 0.0f};
    // wave-uniform trip count (an MFMA reads every lane): a row past r1 (odd
    // row count, k-lane 1 of the last step) contributes zeros
    const int64_t steps = (r1 - r0 + 1) / 2;
    const bool g1 = gcols >= 2, kx1 = kx >= 2;  // single-column operands read one value
    // batches of 4 row steps, double-buffered: the next batch's loads are
    // issued before this batch's 16 MFMAs.  The loads are unconditional and
    // keep raw values; compute() masks them (a select on a freshly loaded value
    // lets the compiler sink the load under a branch, where it is waited for
    // at once).  Single-column operands read their one column twice.  The small
    // segment's loads are issued by every block of an XS launch (its sums only
    // by k block 0): loads behind a branch on `first` left the waits at the
    // join conservative.
    struct Buf {
        float2 a[4], b[4], q[4];
        float x[4][4];
    };
    const bool xsum = XS && first;  // XS: the launch has ns > 0
    auto load = [&](int64_t s0, Buf &o) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int64_t i0 = r0 + 2 * (s0 + q) + par;
            const int64_t i = i0 < r1 ? i0 : (r1 > r0 ? r1 - 1 : min(r0, g.m - 1));
            const float *pa = gp + i * g.ldg;
            o.a[q] = VEC ? *(const float2 *)pa : make_float2(pa[0], pa[g1 ? 1 : 0]);
            const float *pb = xp + i * ldx;
            o.b[q] = VEC ? *(const float2 *)pb : make_float2(pb[0], pb[kx1 ? 1 : 0]);
            if (GMASK) {
                const float *pm = gm + i * g.ldg;
                o.q[q] = VEC ? *(const float2 *)pm : make_float2(pm[0], pm[g1 ? 1 : 0]);
            }
            if (XS) {
#pragma unroll
                for (int e = 0; e < 4; ++e) o.x[q][e] = g.xs[i * g.ldxs + min(e, g.ns - 1)];
            }
        }
    };
    auto compute = [&](int64_t s0, const Buf &o) {
        float2 av[4], bv[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int64_t i0 = r0 + 2 * (s0 + q) + par;
            const bool live = i0 < r1 && s0 + q < steps;
            float2 a = o.a[q], b = o.b[q];
            // a clamped pair past the edge read the last pair: its live first
            // column is the pair's second; dead rows and columns are zeroed
            if (cc != c0) a.x = a.y;
            if (kc != k0) b.x = b.y;
            int ma0 = live && cl0 ? -1 : 0, ma1 = live && cl1 && cc == c0 ? -1 : 0;
            if (GMASK) {
                const float2 q2 = o.q[q];
                ma0 &= (cc != c0 ? q2.y : q2.x) > 0.0f ? -1 : 0;
                ma1 &= q2.y > 0.0f ? -1 : 0;
            }
            int mb0 = kl0 ? -1 : 0, mb1 = kl1 && kc == k0 ? -1 : 0;
            asm volatile("" : "+v"(ma0), "+v"(ma1), "+v"(mb0), "+v"(mb1));
            av[q] = make_float2(__int_as_float(__float_as_int(a.x) & ma0), __int_as_float(__float_as_int(a.y) & ma1));
            bv[q] = make_float2(__int_as_float(__float_as_int(b.x) & mb0), __int_as_float(__float_as_int(b.y) & mb1));
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            acc[0][0] = mfma32(av[q].x, bv[q].x, acc[0][0]);
            acc[0][1] = mfma32(av[q].x, bv[q].y, acc[0][1]);
            acc[1][0] = mfma32(av[q].y, bv[q].x, acc[1][0]);
            acc[1][1] = mfma32(av[q].y, bv[q].y, acc[1][1]);
        }
        if (first) {
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                sb[0] += av[q].x;
                sb[1] += av[q].y;
                if (xsum) {
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        sx[0][e] = fmaf(av[q].x, o.x[q][e], sx[0][e]);
                        sx[1][e] = fmaf(av[q].y, o.x[q][e], sx[1][e]);
                    }
                }
            }
        }
    };
    if (steps > 0 && steps <= 4 * kTnBatches) {
        // the production chunk (256 rows: 32 steps per wave) as straight-line
        // code: the rolled loop below carries b0 / b1 across its back edge,
        // where the compiler waited for every outstanding load (vmcnt(0)) before
        // issuing the next batch -- each batch then paid a full memory latency
        Buf b0, b1;
        load(0, b0);
        // (sched_barrier: the scheduler hoisted the next compute's masking
        // above the loads, waiting for the batch in flight before issuing them)
#pragma unroll
        for (int s0 = 0; s0 < 4 * kTnBatches; s0 += 8) {
            load(s0 + 4, b1);
            __builtin_amdgcn_sched_barrier(0);
            compute(s0, b0);
            if (s0 + 4 >= steps) break;
            load(s0 + 8, b0);
            __builtin_amdgcn_sched_barrier(0);
            compute(s0 + 4, b1);
            if (s0 + 8 >= steps) break;
        }
    } else if (steps > 0) {
        Buf b0, b1;
        load(0, b0);
        // the next batch is loaded unconditionally (rows clamped, masked as
        // dead): a load under a condition makes the compiler wait for it
        for (int64_t s0 = 0;; s0 += 8) {
            load(s0 + 4, b1);
            compute(s0, b0);
            if (s0 + 4 >= steps) break;
            load(s0 + 8, b0);
            compute(s0 + 4, b1);
            if (s0 + 8 >= steps) break;
        }
    }
    // this wave's block, db and small-segment sums (the two row parities of a
    // column added in a fixed order); waves 1..3 hand theirs to wave 0, which
    // adds them in wave order
    if (first) {
#pragma unroll
        for (int ct = 0; ct < 2; ++ct) {
            sb[ct] += __shfl_xor(sb[ct], 32, 64);
#pragma unroll
            for (int e = 0; e < 4; ++e) sx[ct][e] += __shfl_xor(sx[ct][e], 32, 64);
        }
    }
    // one LDS block, filled by waves 1, 2, 3 in turn (19 KB instead of 57: LDS
    // no longer caps the workgroups per CU), wave 0 adding each as it lands
#pragma unroll 1
    for (int w = 1; w < 4; ++w) {
        if (wave == w) {
#pragma unroll
            for (int ct = 0; ct < 2; ++ct)
#pragma unroll
                for (int kt = 0; kt < 2; ++kt)
#pragma unroll
                    for (int r = 0; r < 16; ++r) red[(2 * ct + kt) * 16 + r][lane] = acc[ct][kt][r];
            if (first) {
#pragma unroll
                for (int ct = 0; ct < 2; ++ct) {
                    red[64 + ct][lane] = sb[ct];
#pragma unroll
                    for (int e = 0; e < 4; ++e) red[66 + 4 * ct + e][lane] = sx[ct][e];
                }
            }
        }
        __syncthreads();
        if (wave == 0) {
#pragma unroll
            for (int ct = 0; ct < 2; ++ct)
#pragma unroll
                for (int kt = 0; kt < 2; ++kt)
#pragma unroll
                    for (int r = 0; r < 16; ++r) acc[ct][kt][r] += red[(2 * ct + kt) * 16 + r][lane];
            if (first) {
#pragma unroll
                for (int ct = 0; ct < 2; ++ct) {
                    sb[ct] += red[64 + ct][lane];
#pragma unroll
                    for (int e = 0; e < 4; ++e) sx[ct][e] += red[66 + 4 * ct + e][lane];
                }
            }
        }
        __syncthreads();
    }
    if (wave != 0) return;
    if (cb >= gcols) return;
    float *pp = t.part + (int64_t)chunk * 128 * t.cols;
#pragma unroll
    for (int ct = 0; ct < 2; ++ct)
#pragma unroll
        for (int kt = 0; kt < 2; ++kt)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int c = cb + 2 * acc_row(r, lane) + ct;
                pp[(int64_t)c * t.cols + kb + 2 * j + kt] = acc[ct][kt][r];
            }
    if (first && par == 0) {
#pragma unroll
        for (int ct = 0; ct < 2; ++ct) {
            float *q = pp + (int64_t)(c0 + ct) * t.cols + t.kbig;
#pragma unroll
            for (int e = 0; e < 4; ++e)
                if (e < ns) q[e] = sx[ct][e];
            q[g.ns] = sb[ct];
        }
    }
}

// dw / db from the partials, chunks added in order.
__global__ __launch_bounds__(256) void rgemm_tn_reduce_kernel(TnArgs t, int chunks) {
    // thread (group gq = tid / 32, output idx = 32 block + tid % 32): the
    // chunks of group gq (a contiguous eighth of them) added in order, their
    // loads issued 8 at a time unconditionally (clamped, masked); then the 8
    // groups' sums added in group order through LDS: a fixed order
    __shared__ float red[8][32];
    const mmpde_rgemm_tn_args &g = t.g;
    const int gq = threadIdx.x >> 5;
    const int64_t outs = (int64_t)g.gcols * t.cols;
    const int64_t idx = (int64_t)blockIdx.x * 32 + (threadIdx.x & 31);
    const int64_t ic = min(idx, outs - 1);
    const int c = (int)(ic / t.cols), k = (int)(ic - (int64_t)c * t.cols);
    const int per = (chunks + 7) / 8;
    const int q0 = min(gq * per, chunks), q1 = min(q0 + per, chunks);
    const float *pp = t.part + (int64_t)c * t.cols + k;
    const int64_t cs = (int64_t)128 * t.cols;
    float s = 0.0f;
    for (int q = q0; q < q1; q += 8) {
        float v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = pp[(int64_t)min(q + u, q1 - 1) * cs];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            int m = q + u < q1 ? -1 : 0;
            asm volatile("" : "+v"(m));
            s += __int_as_float(__float_as_int(v[u]) & m);
        }
    }
    red[gq][threadIdx.x & 31] = s;
    __syncthreads();
    if (gq != 0 || idx >= outs) return;
#pragma unroll
    for (int u = 1; u < 8; ++u) s += red[u][threadIdx.x & 31];
    if (k < t.kbig) {
        int seg = 0;
        while (seg < g.nseg - 1 && k >= t.base[seg + 1]) ++seg;
        const int kk = k - t.base[seg];
        if (kk < g.kx[seg]) g.dw[(int64_t)c * g.lddw + g.dwcol[seg] + kk] = s;  // else a padding column
    } else if (k < t.kbig + g.ns) {
        float *o = g.dw + (int64_t)c * g.lddw + g.dwcol_s + (k - t.kbig);
        const float v = g.sign_s * s;
        *o = g.accumulate_s ? *o + v : v;
    } else if (g.db) {
        g.db[c] = s;
    }
}

bool al16(const void *p) { return ((uintptr_t)p & 15) == 0; }
bool al8(const void *p) { return ((uintptr_t)p & 7) == 0; }

}  // namespace

extern "C" int mmpde_rgemm(const mmpde_rgemm_args *gp, mmpde_stream_t stream) {
    MMPDE_REQUIRE(gp);
    const mmpde_rgemm_args g = *gp;
    MMPDE_REQUIRE(g.m > 0 && g.kh >= 0 && g.m < ((int64_t)1 << 36));
    MMPDE_REQUIRE(g.parts == 1 || g.parts == 2);
    MMPDE_REQUIRE(g.layout == MMPDE_RGEMM_NT || g.layout == MMPDE_RGEMM_NN);
    bool xs = false;
    for (int p = 0; p < g.parts; ++p) {
        MMPDE_REQUIRE(g.out[p] && g.ncols[p] >= 1 && g.ncols[p] <= 128 && g.ldo[p] >= g.ncols[p]);
        MMPDE_REQUIRE(g.ns[p] >= 0 && g.ns[p] <= 4);
        MMPDE_REQUIRE(g.ns[p] == 0 || (g.xs && g.xw[p]));
        MMPDE_REQUIRE(!g.omask[p] || g.ldom[p] >= g.ncols[p]);
        xs = xs || g.ns[p] > 0;
    }
    MMPDE_REQUIRE(g.kh > 0 || xs);
    bool vec = g.kh % 4 == 0;
    if (g.kh > 0) {
        MMPDE_REQUIRE((g.amask[0] == nullptr) == (g.amask[1] == nullptr));
        for (int h = 0; h < 2; ++h) {
            MMPDE_REQUIRE(g.a[h] && g.w[h] && g.lda[h] >= g.kh);
            vec = vec && al16(g.a[h]) && g.lda[h] % 4 == 0 && (!g.amask[h] || al16(g.amask[h]));
            if (g.layout == MMPDE_RGEMM_NT) vec = vec && al16(g.w[h]) && g.ldw % 4 == 0;
        }
        for (int p = 0; p < g.parts; ++p)
            if (g.layout == MMPDE_RGEMM_NT) vec = vec && g.wk[p] % 4 == 0;
    }
    const bool am = g.kh > 0 && g.amask[0] != nullptr;
    hipStream_t st = as_stream(stream);
    // MMPDE_RGEMM_FORM=tile (A/B aid, tools/rgemm_bench.py): the 128 x 128 tile
    // kernel for every shape
    static const bool tile_only = [] {
        const char *e = getenv("MMPDE_RGEMM_FORM");
        return e && e[0] == 't';
    }();
    if (!tile_only && vec && (g.kh == 32 || g.kh == 64 || g.kh == 128)) {
        // weight-stationary persistent form: the workgroups that fit the CUs at
        // once (two per CU; the kh = 128 form holds ~240 registers per lane,
        // one), shared by the parts
        const int64_t ntiles = (g.m + 31) / 32;
        const int per_cu = g.kh == 128 ? 1 : 2;
        const int64_t slots = std::max<int64_t>(1, (int64_t)per_cu * rgemm_cus() / g.parts);
        const dim3 wgrid((unsigned)std::min<int64_t>(ntiles, slots), (unsigned)g.parts);
#define WS_LAUNCH(L, K, A, X) hipLaunchKernelGGL((rgemm_ws_kernel<L, K, A, X>), wgrid, dim3(256), 0, st, g)
#define WS_K(L, A, X)                          \
    if (g.kh == 32) WS_LAUNCH(L, 32, A, X);    \
    else if (g.kh == 64) WS_LAUNCH(L, 64, A, X); \
    else WS_LAUNCH(L, 128, A, X);
#define WS_AX(L)                               \
    if (am && xs) { WS_K(L, true, true) }      \
    else if (am) { WS_K(L, true, false) }      \
    else if (xs) { WS_K(L, false, true) }      \
    else { WS_K(L, false, false) }
        if (g.layout == MMPDE_RGEMM_NT) {
            WS_AX(MMPDE_RGEMM_NT)
        } else {
            WS_AX(MMPDE_RGEMM_NN)
        }
#undef WS_AX
#undef WS_K
#undef WS_LAUNCH
        MMPDE_RET_LAUNCH();
        return MMPDE_OK;
    }
    const dim3 grid((unsigned)ceil_div(g.m, 128), (unsigned)g.parts);
#define RG_LAUNCH(L, V, A, X) hipLaunchKernelGGL((rgemm_kernel<L, V, A, X>), grid, dim3(256), 0, st, g)
#define RG_LAYOUT(L)                                           \
    if (vec) {                                                 \
        if (am && xs) RG_LAUNCH(L, true, true, true);          \
        else if (am) RG_LAUNCH(L, true, true, false);          \
        else if (xs) RG_LAUNCH(L, true, false, true);          \
        else RG_LAUNCH(L, true, false, false);                 \
    } else {                                                   \
        if (am && xs) RG_LAUNCH(L, false, true, true);         \
        else if (am) RG_LAUNCH(L, false, true, false);         \
        else if (xs) RG_LAUNCH(L, false, false, true);         \
        else RG_LAUNCH(L, false, false, false);                \
    }
    if (g.layout == MMPDE_RGEMM_NT) {
        RG_LAYOUT(MMPDE_RGEMM_NT)
    } else {
        RG_LAYOUT(MMPDE_RGEMM_NN)
    }
#undef RG_LAYOUT
#undef RG_LAUNCH
    MMPDE_RET_LAUNCH();
    return MMPDE_OK;
}

extern "C" int64_t mmpde_rgemm_tn_workspace_bytes(int64_t m, int chunk_rows, int cols) {
    if (m <= 0 || chunk_rows <= 0 || cols <= 0) return 0;
    return ceil_div(m, chunk_rows) * 128 * (int64_t)cols * 4;
}

extern "C" int mmpde_rgemm_tn(const mmpde_rgemm_tn_args *gp, void *workspace, int64_t workspace_bytes,
                              mmpde_stream_t stream) {
    MMPDE_REQUIRE(gp && workspace);
    const mmpde_rgemm_tn_args &g = *gp;
    MMPDE_REQUIRE(g.m > 0 && g.chunk_rows > 0 && g.chunk_rows % 2 == 0 && g.g && g.dw);
    MMPDE_REQUIRE(g.gcols >= 1 && g.gcols <= 128 && g.ldg >= g.gcols);
    MMPDE_REQUIRE(g.nseg >= 1 && g.nseg <= 3 && g.ns >= 0 && g.ns <= 4 && (g.ns == 0 || g.xs));
    TnArgs t{};
    t.g = g;
    int kbig = 0;
    bool vec = g.gcols >= 2 && g.ldg % 2 == 0 && al8(g.g) && (!g.gmask || al8(g.gmask));
    for (int s = 0; s < g.nseg; ++s) {
        MMPDE_REQUIRE(g.x[s] && g.kx[s] > 0 && g.ldx[s] >= g.kx[s]);
        t.base[s] = kbig;
        kbig += (g.kx[s] + 63) / 64 * 64;
        vec = vec && g.kx[s] >= 2 && g.ldx[s] % 2 == 0 && al8(g.x[s]);
    }
    t.kbig = kbig;
    t.cols = kbig + g.ns + 1;
    t.part = (float *)workspace;
    const int64_t chunks = ceil_div(g.m, g.chunk_rows);
    MMPDE_REQUIRE(workspace_bytes >= mmpde_rgemm_tn_workspace_bytes(g.m, g.chunk_rows, t.cols));
    MMPDE_REQUIRE(chunks < 65536);
    hipStream_t st = as_stream(stream);
    t.nkb = kbig / 64;
    t.ncb = (g.gcols + 63) / 64;
    t.chunks = (int)chunks;
    const dim3 grid((unsigned)(8 * t.nkb * t.ncb * ceil_div(chunks, 8)));
#define TN_LAUNCH(M, V, X) hipLaunchKernelGGL((rgemm_tn_partial_kernel<M, V, X>), grid, dim3(256), 0, st, t)
#define TN_X(M, V)              \
    if (g.ns > 0) TN_LAUNCH(M, V, true); \
    else TN_LAUNCH(M, V, false);
    if (g.gmask) {
        if (vec) { TN_X(true, true) }
        else { TN_X(true, false) }
    } else {
        if (vec) { TN_X(false, true) }
        else { TN_X(false, false) }
    }
#undef TN_X
#undef TN_LAUNCH
    MMPDE_RET_LAUNCH();
    const int64_t outs = (int64_t)g.gcols * t.cols;
    hipLaunchKernelGGL(rgemm_tn_reduce_kernel, dim3((unsigned)ceil_div(outs, 32)), dim3(256), 0, st, t,
                       (int)chunks);
    MMPDE_RET_LAUNCH();
    return MMPDE_OK;
}
