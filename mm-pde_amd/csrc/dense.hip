// Small dense helpers: skinny-M linear layers (res_cut MLP, DMM output_mlp /
// fc layers, the per-trajectory branch . W contraction) and a direct 2-D
// convolution (DMM ConvNet branch, Burgers res_cut).  The linears run at M = B
// (<= 32 rows), where every weight is read exactly once: weight-streaming
// (HBM-bound) kernels.
#include "common.hpp"

namespace {

// y[r, c] = act(x[r, :k] . w[c, :k] + b[c]) for M = B <= a few dozen rows: a
// weight-streaming GEMM (every weight read once).  One workgroup = one 16 x 16
// output tile (16 rows of x, 16 weight rows) and kSkW waves.  K is walked in
// chunks of 64 kSkW: the W and x tiles of a chunk are loaded cooperatively with
// lanes on consecutive k (one wave-load = 256 contiguous bytes of one row, any
// row stride or alignment -- res_cut's 2521-wide rows are not 16-B aligned) into
// registers one chunk ahead, stored to LDS, and wave w multiplies k-range
// [64 w, 64 w + 64) of the chunk with 16 v_mfma_f32_16x16x4_f32 (exact fp32
// products; lane (r, g) holds k = 16 q + 4 g + t of float4 number q).  The
// per-wave partial tiles meet in LDS in a fixed order (deterministic).
constexpr int kSkW = 8;               // waves per workgroup
constexpr int kSkMaxZ = 16;           // K splits at most

// Split K (part != nullptr): workgroup z of gridDim.z takes chunks
// [z nchz, (z + 1) nchz) of K and stores its raw tile to part[z][m][n]; the
// last of a tile's gridDim.z workgroups to finish (ticket counter, agent-scope
// release / acquire) adds the partial tiles in z order (a fixed order:
// deterministic) with the bias and activation.  Splitting K fills the chip
// when n / 16 tiles alone are too few (res_cut: 128 - 158 tiles).  The
// tickets (zero before the first launch) are reset by the reducing slice.
template <int kSkW>
__global__ __launch_bounds__(kSkW * 64) void linear_skinny_kernel(const float *__restrict__ x,
                                                                  int64_t ldx, int64_t m, int64_t k,
                                                                  const float *__restrict__ w,
                                                                  int64_t ldw,
                                                                  const float *__restrict__ b,
                                                                  int64_t n, int act,
                                                                  float *__restrict__ y, int64_t ldy,
                                                                  int nchz, float *__restrict__ part,
                                                                  unsigned *__restrict__ tickets) {
    constexpr int C = 64 * kSkW, LD = C + 4;
    __shared__ float sw[16 * LD], sx[16 * LD];
    const int tid = threadIdx.x;
    const int wave = tid >> 6;
    const int lane = tid & 63;
    const int r = lane & 15, g = lane >> 4;
    const int64_t col0 = (int64_t)blockIdx.x * 16, row0 = (int64_t)blockIdx.y * 16;
    const int K = (int)k;
    const int c0 = (int)blockIdx.z * nchz;
    const int nch = min((K + C - 1) / C - c0, nchz);
    // loader role: rows i = 0..15 of both tiles at k = kc + tid
    float lw[16], lx[16];
    auto load = [&](int kc) {
        const int kk = kc + tid;
        const bool ok = kk < K;
        const int o = ok ? kk : 0;
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            const float a = w[min(col0 + i, n - 1) * ldw + o];
            const float c = x[min(row0 + i, m - 1) * ldx + o];
            lw[i] = ok ? a : 0.0f;
            lx[i] = ok ? c : 0.0f;
        }
    };
    f32x4 acc = {0.0f, 0.0f, 0.0f, 0.0f};
    if (nch > 0) load(c0 * C);
    for (int c = 0; c < nch; ++c) {
        if (c) __syncthreads();  // chunk c - 1 consumed
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            sw[i * LD + tid] = lw[i];
            sx[i * LD + tid] = lx[i];
        }
        __syncthreads();
        if (c + 1 < nch) load((c0 + c + 1) * C);
        const float *aw = sw + r * LD + 64 * wave + 4 * g;
        const float *ax = sx + r * LD + 64 * wave + 4 * g;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const float4 wv = *(const float4 *)(aw + 16 * q);
            const float4 xv = *(const float4 *)(ax + 16 * q);
            acc = mfma16(xv.x, wv.x, acc);
            acc = mfma16(xv.y, wv.y, acc);
            acc = mfma16(xv.z, wv.z, acc);
            acc = mfma16(xv.w, wv.w, acc);
        }
    }
    __syncthreads();
    f32x4 *wpart = (f32x4 *)sw;  // [wave][lane]
    wpart[wave * 64 + lane] = acc;
    __syncthreads();
    if (wave != 0) return;
    f32x4 s = wpart[lane];
#pragma unroll
    for (int v = 1; v < kSkW; ++v) s += wpart[v * 64 + lane];
    const int64_t col = col0 + r;
    if (part) {
        float *pz = part + (int64_t)blockIdx.z * m * n;
        if (col < n) {
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int64_t row = row0 + 4 * g + q;
                // write-through (sc1) store: visible chip-wide once drained,
                // no release fence (no L2 write-back of the whole XCD)
                if (row < m)
                    __hip_atomic_store(pz + row * n + col, s[q], __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
            }
        }
        if (!tickets) return;
        // in-launch reduction (cdna_hip_programming.md, split-K hand-off, sc1
        // form): the slice that draws the last ticket of its tile adds the
        // gridDim.z partial tiles in z order (deterministic), then resets the
        // ticket.  The one storing wave drains its sc1 stores before the ticket.
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        // the ticket's address goes through a VGPR the compiler cannot fold, so the
        // atomic and the reset are vector-memory operations (never scalar-cache
        // writes)
        int vzero;
        asm volatile("v_mov_b32 %0, 0" : "=v"(vzero));
        unsigned *tk = tickets + blockIdx.y * gridDim.x + blockIdx.x + vzero;
        unsigned ticket = 0u;
        if (lane == 0) ticket = __hip_atomic_fetch_add(tk, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        // lane 0's ticket to the whole wave (register broadcast: an LDS flag
        // would need a barrier the single remaining wave cannot order by itself)
        ticket = __builtin_amdgcn_readfirstlane(ticket);
        if (ticket != gridDim.z - 1) return;
        // every slab load is an sc1 (agent-scope) load, so no acquire fence:
        // the wavefront fence only keeps the loads below the ticket
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        // every slab load issued before the first add (clamped addresses, no
        // per-load branches), then the adds in z order
        const int Z = (int)gridDim.z;
        const int64_t cc = min(col, n - 1);
        float v[kSkMaxZ][4];
#pragma unroll
        for (int zz = 0; zz < kSkMaxZ; ++zz) {
            if (zz < Z) {
                const float *pq = part + (int64_t)zz * m * n + cc;
#pragma unroll
                for (int q = 0; q < 4; ++q)
                    v[zz][q] = __hip_atomic_load(pq + min(row0 + 4 * g + q, m - 1) * n, __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_AGENT);
            }
        }
        f32x4 t = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
        for (int zz = 0; zz < kSkMaxZ; ++zz) {
            if (zz < Z) {
#pragma unroll
                for (int q = 0; q < 4; ++q) t[q] += v[zz][q];
            }
        }
        if (lane == 0) *tk = 0u;
        s = t;
    }
    if (col >= n) return;
    const float bb = b ? b[col] : 0.0f;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const int64_t row = row0 + 4 * g + q;
        if (row < m) y[row * ldy + col] = act_apply(s[q] + bb, act);
    }
}

// K splits of a skinny linear: enough workgroups for ~4 per CU over the
// output column tiles, chunks of 64 kSkW k each, at most 16 splits.  The split
// (hence every output row's summation order) depends on n and k only, not on
// the row count m, so a row's result does not depend on the rows beside it.
// The ticket block (kSkTickets words, one per output tile) bounds the tiles of
// one split launch: mmpde_linear_skinny_ws runs larger m as row blocks with
// the same split rather than unsplit (which would change a row's rounding).
inline int skinny_splits(int64_t n, int64_t k, int cus) {
    const int64_t ctiles = (n + 15) / 16;
    const int64_t chunks = (k + 64 * kSkW - 1) / (64 * kSkW);
    int64_t z = (4 * (int64_t)cus + ctiles - 1) / ctiles;
    z = z < chunks ? z : chunks;
    z = z < kSkMaxZ ? z : kSkMaxZ;
    return z > 1 ? (int)z : 1;
}

// F.interpolate(mode='bilinear', align_corners=True) of `planes` h x w planes
// to oh x ow (data_creator_2d.py:102-103): source coordinate = dst index x
// (in - 1) / (out - 1) in fp32, the two neighbours (the upper one clamped) and
// their linear weights, as PyTorch's upsample_bilinear2d computes them.  One
// thread per output element.
__global__ __launch_bounds__(256) void resample_bilinear_kernel(const float *__restrict__ x, int64_t planes,
                                                                int h, int w, int oh, int ow, float sy,
                                                                float sx, float *__restrict__ y) {
    const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (e >= planes * oh * ow) return;
    const int ox = (int)(e % ow);
    const int oy = (int)((e / ow) % oh);
    const int64_t pl = e / ((int64_t)ow * oh);
    // rounded products (no fma contraction into the lambdas below): the source
    // coordinate is an fp32 value first, as on PyTorch's side
    const float fy = __fmul_rn(sy, (float)oy), fx = __fmul_rn(sx, (float)ox);
    const int y0 = (int)fy, x0 = (int)fx;
    const int y1 = y0 + (y0 < h - 1 ? 1 : 0), x1 = x0 + (x0 < w - 1 ? 1 : 0);
    const float ly = fy - (float)y0, lx = fx - (float)x0;
    const float hy = 1.0f - ly, hx = 1.0f - lx;
    const float *p = x + pl * h * w;
    y[e] = hy * (hx * p[y0 * w + x0] + lx * p[y0 * w + x1]) + ly * (hx * p[y1 * w + x0] + lx * p[y1 * w + x1]);
}

// one thread per output element; weight [cout][cin][ks][ks] (PyTorch layout)
__global__ __launch_bounds__(256) void conv2d_kernel(const float *__restrict__ x, int64_t batches,
                                                     int cin, int h, int w,
                                                     const float *__restrict__ wt,
                                                     const float *__restrict__ bias, int cout,
                                                     int ks, int stride, int pad, int oh, int ow,
                                                     const float *__restrict__ res, int act,
                                                     float *__restrict__ y,
                                                     unsigned *__restrict__ zero, int n_zero,
                                                     int circular, int res_after_act) {
    const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const int64_t total = batches * cout * oh * ow;
    if (e < n_zero) zero[e] = 0u;  // side job for the caller (dmm.hip's split-K tickets)
    if (e >= total) return;
    const int ox = (int)(e % ow);
    const int oy = (int)((e / ow) % oh);
    const int co = (int)((e / ((int64_t)ow * oh)) % cout);
    const int64_t bb = e / ((int64_t)ow * oh * cout);
    float acc = bias ? bias[co] : 0.0f;
    for (int ci = 0; ci < cin; ++ci) {
        const float *xp = x + (bb * cin + ci) * (int64_t)h * w;
        const float *wp = wt + ((int64_t)co * cin + ci) * ks * ks;
        for (int ky = 0; ky < ks; ++ky) {
            int iy = oy * stride - pad + ky;
            if (circular) iy = ((iy % h) + h) % h;
            else if (iy < 0 || iy >= h) continue;
            for (int kx = 0; kx < ks; ++kx) {
                int ix = ox * stride - pad + kx;
                if (circular) ix = ((ix % w) + w) % w;
                else if (ix < 0 || ix >= w) continue;
                acc += wp[ky * ks + kx] * xp[iy * w + ix];
            }
        }
    }
    if (res_after_act) {
        y[e] = res[e] + act_apply(acc, act);
        return;
    }
    if (res) acc = res[e] + acc;
    y[e] = act_apply(acc, act);
}

// Weight / bias gradient of a stride-1 convolution (the backward of
// conv2d_kernel; BaseCNN training, models_cnn.py:66-83 under
// train_helper_2d.py:121-126):
//   dw[co, ci, ky, kx] = sum_{b, y, x} dy[b, co, y, x] * x[b, ci, y - pad + ky, x - pad + kx]
//   db[co]             = sum_{b, y, x} dy[b, co, y, x]        (ci == 0 workgroups)
// with circular (wrapped) or zero (skipped) padding.  One workgroup per
// (co, ci): thread t takes tap t % T (T = ks * ks) and pixel slice t / T; the
// (x, dy) planes of each batch are staged in LDS when they fit.  Every sum runs
// in a fixed order (batches, then the slice's pixels, then the slices):
// deterministic, no atomics.
constexpr int kGwThreads = 256;
template <bool LDS>
__global__ __launch_bounds__(kGwThreads) void conv2d_grad_weight_kernel(const float *__restrict__ x,
                                                                       const float *__restrict__ dy, int batches,
                                                                       int cin, int cout, int h, int w, int ks,
                                                                       int pad, int circular,
                                                                       float *__restrict__ dw,
                                                                       float *__restrict__ db) {
    extern __shared__ float sm[];  // LDS: x plane [h * w], dy plane [h * w]; then the slice sums
    const int co = (int)blockIdx.x / cin, ci = (int)blockIdx.x % cin;
    const int T = ks * ks, S = kGwThreads / T;
    const int t = threadIdx.x, tap = t % T, sl = t / T;
    const bool act = sl < S;
    const int ky = tap / ks, kx = tap % ks;
    const int hw = h * w;
    float acc = 0.0f, accb = 0.0f;
    for (int b = 0; b < batches; ++b) {
        const float *xp = x + ((int64_t)b * cin + ci) * hw;
        const float *dp = dy + ((int64_t)b * cout + co) * hw;
        const float *X = xp, *D = dp;
        if (LDS) {
            __syncthreads();  // the previous batch's planes are consumed
            for (int i = t; i < hw; i += kGwThreads) {
                sm[i] = xp[i];
                sm[hw + i] = dp[i];
            }
            __syncthreads();
            X = sm;
            D = sm + hw;
        }
        if (act) {
            for (int p = sl; p < hw; p += S) {
                const int oy = p / w, ox = p - oy * w;
                const float g = D[p];
                if (ci == 0 && tap == 0) accb += g;  // the bias sums every pixel
                int iy = oy - pad + ky, ix = ox - pad + kx;
                if (circular) {
                    iy = iy < 0 ? iy + h : (iy >= h ? iy - h : iy);
                    ix = ix < 0 ? ix + w : (ix >= w ? ix - w : ix);
                } else if (iy < 0 || iy >= h || ix < 0 || ix >= w) {
                    continue;
                }
                acc = fmaf(g, X[iy * w + ix], acc);
            }
        }
    }
    // the slices of each tap, added in slice order
    __syncthreads();
    float *part = sm;  // [S][T] (+ bias partials after)
    if (act) part[sl * T + tap] = acc;
    if (act && tap == 0) part[S * T + sl] = accb;
    __syncthreads();
    if (t < T) {
        float v = 0.0f;
        for (int q = 0; q < S; ++q) v += part[q * T + t];
        dw[(((int64_t)co * cin + ci) * ks + t / ks) * ks + t % ks] = v;
    }
    if (ci == 0 && t == 0 && db) {
        float v = 0.0f;
        for (int q = 0; q < S; ++q) v += part[S * T + q];
        db[co] = v;
    }
}

// Per-trajectory mean squared error: one workgroup per trajectory, every thread
// sums a fixed strided subset in index order, then a fixed LDS tree: the
// result depends only on that trajectory's values (not on how many
// trajectories share the launch), so a sharded evaluation reproduces the
// single-process losses bit for bit.
__global__ __launch_bounds__(256) void traj_mse_kernel(const float *__restrict__ pred,
                                                       const float *__restrict__ lab, int64_t n_per,
                                                       float *__restrict__ out) {
    __shared__ float red[256];
    const int64_t base = (int64_t)blockIdx.x * n_per;
    float s = 0.0f;
    for (int64_t i = threadIdx.x; i < n_per; i += 256) {
        const float d = pred[base + i] - lab[base + i];
        s = fmaf(d, d, s);
    }
    red[threadIdx.x] = s;
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
        if ((int)threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
        __syncthreads();
    }
    if (threadIdx.x == 0) out[blockIdx.x] = red[0] / (float)n_per;
}

// Training backward of the few-row linears (res_cut's MLP, interpolate.py:
// 54-60,95-97, at M = B rows):
//   outer_rows: dw[i][j] = sum_{r<m} g[r][i] x[r][j] and db[i] = sum_r g[r][i]
//     (r ascending).  Workgroup = a 16 (i) x 64 (j) block of dw: the block's g
//     and x columns staged in LDS (any row stride / alignment), each thread 4
//     outputs of one i; HBM-bound on the dw write.
//   transpose: y[c][r] = x[r][c] through 32 x 33 LDS tiles (dX = dY W as the
//     skinny forward of W^T).
//   tanh_bwd: dz = dy (1 - t^2) (torch's tanh_backward).
constexpr int kOrRows = 32;  // rows staged per pass (any m: passes in row order)
__global__ __launch_bounds__(256) void outer_rows_kernel(const float *__restrict__ g, int64_t ldg,
                                                         const float *__restrict__ x, int64_t ldx, int m,
                                                         int64_t n, int64_t k, float *__restrict__ dw,
                                                         int64_t lddw, float *__restrict__ db) {
    __shared__ float sg[kOrRows][16], sx[kOrRows][64];
    const int tid = threadIdx.x;
    const int64_t i0 = (int64_t)blockIdx.y * 16, j0 = (int64_t)blockIdx.x * 64;
    const int il = tid >> 4, jl = 4 * (tid & 15);
    float4 acc = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    float sb = 0.0f;
    // rows r0 .. r0 + 31 per pass, r ascending over the passes: one fixed order
    for (int r0 = 0; r0 < m; r0 += kOrRows) {
        const int mr = min(kOrRows, m - r0);
        if (r0 > 0) __syncthreads();  // the previous pass has read the tiles
        for (int e = tid; e < mr * 64; e += 256) {
            const int r = e >> 6, c = e & 63;
            const int64_t row = r0 + r;
            sx[r][c] = x[row * ldx + min(j0 + c, k - 1)];
            if (c < 16) sg[r][c] = g[row * ldg + min(i0 + c, n - 1)];
        }
        __syncthreads();
        for (int r = 0; r < mr; ++r) {
            const float gv = sg[r][il];
            const float4 xv = *(const float4 *)&sx[r][jl];
            acc.x = fmaf(gv, xv.x, acc.x);
            acc.y = fmaf(gv, xv.y, acc.y);
            acc.z = fmaf(gv, xv.z, acc.z);
            acc.w = fmaf(gv, xv.w, acc.w);
            sb += gv;
        }
    }
    const int64_t i = i0 + il, j = j0 + jl;
    if (i >= n) return;
    float *o = dw + i * lddw + j;
    if (j < k) o[0] = acc.x;
    if (j + 1 < k) o[1] = acc.y;
    if (j + 2 < k) o[2] = acc.z;
    if (j + 3 < k) o[3] = acc.w;
    if (db && blockIdx.x == 0 && jl == 0) db[i] = sb;
}

__global__ __launch_bounds__(256) void transpose_kernel(const float *__restrict__ x, int64_t rows, int64_t cols,
                                                        int64_t ldx, float *__restrict__ y, int64_t ldy) {
    __shared__ float t[32][33];
    const int64_t r0 = (int64_t)blockIdx.y * 32, c0 = (int64_t)blockIdx.x * 32;
    const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;  // 32 x 8
    for (int q = ty; q < 32; q += 8) {
        const int64_t r = r0 + q, c = c0 + tx;
        t[q][tx] = (r < rows && c < cols) ? x[r * ldx + c] : 0.0f;
    }
    __syncthreads();
    for (int q = ty; q < 32; q += 8) {
        const int64_t c = c0 + q, r = r0 + tx;
        if (c < cols && r < rows) y[c * ldy + r] = t[tx][q];
    }
}

__global__ __launch_bounds__(256) void tanh_bwd_kernel(const float *__restrict__ dy, const float *__restrict__ t,
                                                       int64_t n, float *__restrict__ dz) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const float tv = t[i];
    dz[i] = dy[i] * (1.0f - tv * tv);
}

}  // namespace

extern "C" int mmpde_outer_rows(const float *g, int64_t ldg, const float *x, int64_t ldx, int m, int64_t n,
                                int64_t k, float *dw, int64_t lddw, float *db, mmpde_stream_t stream) {
    MMPDE_REQUIRE(g && x && dw && m >= 1 && n >= 1 && k >= 1);
    MMPDE_REQUIRE(ldg >= n && ldx >= k && lddw >= k && n < ((int64_t)1 << 31) && k < ((int64_t)1 << 31));
    const dim3 grid((unsigned)((k + 63) / 64), (unsigned)((n + 15) / 16));
    hipLaunchKernelGGL(outer_rows_kernel, grid, dim3(256), 0, as_stream(stream), g, ldg, x, ldx, m, n, k, dw,
                       lddw, db);
    MMPDE_RET_LAUNCH();
    return MMPDE_OK;
}

extern "C" int mmpde_transpose(const float *x, int64_t rows, int64_t cols, int64_t ldx, float *y, int64_t ldy,
                               mmpde_stream_t stream) {
    MMPDE_REQUIRE(x && y && rows >= 1 && cols >= 1 && ldx >= cols && ldy >= rows);
    MMPDE_REQUIRE(rows < ((int64_t)1 << 36) && cols < ((int64_t)1 << 36));
    const dim3 grid((unsigned)((cols + 31) / 32), (unsigned)((rows + 31) / 32));
    hipLaunchKernelGGL(transpose_kernel, grid, dim3(256), 0, as_stream(stream), x, rows, cols, ldx, y, ldy);
    MMPDE_RET_LAUNCH();
    return MMPDE_OK;
}

extern "C" int mmpde_tanh_bwd(const float *dy, const float *t, int64_t n, float *dz, mmpde_stream_t stream) {
    MMPDE_REQUIRE(dy && t && dz && n >= 1);
    hipLaunchKernelGGL(tanh_bwd_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, as_stream(stream), dy, t,
                       n, dz);
    MMPDE_RET_LAUNCH();
    return MMPDE_OK;
}

extern "C" int mmpde_version(void) { return 12100; }

extern "C" int mmpde_traj_mse(const float *pred, const float *labels, int64_t batches, int64_t n_per,
                              float *out, mmpde_stream_t stream) {
    MMPDE_REQUIRE(pred && labels && out && batches > 0 && n_per > 0 && batches <= INT32_MAX);
    hipLaunchKernelGGL(traj_mse_kernel, dim3((unsigned)batches), dim3(256), 0, as_stream(stream), pred,
                       labels, n_per, out);
    MMPDE_RET_LAUNCH();
    return MMPDE_OK;
}

extern "C" const char *mmpde_status_string(int status) {
    if (status == MMPDE_OK) return "ok";
    if (status == MMPDE_ERR_INVALID_ARG) return "invalid argument";
    if (status == MMPDE_ERR_UNSUPPORTED) return "unsupported shape";
    if (status <= MMPDE_ERR_HIP_BASE) return hipGetErrorString((hipError_t)(MMPDE_ERR_HIP_BASE - status));
    return "unknown status";
}

static int skinny_cus() {
    int dev = 0, cus = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus < 1)
        return 256;
    return cus;
}

// split-K scratch: a FIXED block of kSkTickets ticket words (one per output
// tile; the same words for every shape, so one call's partial tiles never land
// on another call's tickets when a workspace is reused), then z partial tiles.
// A split only pays below ~4 workgroups per CU, i.e. far fewer tiles than this.
constexpr int64_t kSkTickets = 4096;
static int64_t skinny_ws_bytes(int64_t m, int64_t n, int z) {
    return z > 1 ? (kSkTickets + (int64_t)z * m * n) * (int64_t)sizeof(float) : 0;
}

extern "C" int64_t mmpde_linear_skinny_workspace_bytes(int64_t m, int64_t n, int64_t k) {
    if (m <= 0 || n <= 0 || k <= 0) return 0;
    return skinny_ws_bytes(m, n, skinny_splits(n, k, skinny_cus()));
}

extern "C" int mmpde_linear_skinny_ws(const float *x, int64_t ldx, int64_t m, int64_t k, const float *w,
                                      int64_t ldw, const float *b, int64_t n, int act, float *y, int64_t ldy,
                                      float *workspace, int64_t workspace_bytes, mmpde_stream_t stream) {
    MMPDE_REQUIRE(x && w && y && m > 0 && k > 0 && n > 0 && m <= 4096);
    MMPDE_REQUIRE(ldx >= k && ldw >= k && ldy >= n && act >= 0 && act <= 2);
    hipStream_t st = as_stream(stream);
    int z = skinny_splits(n, k, skinny_cus());
    if (!workspace || workspace_bytes < skinny_ws_bytes(m, n, z)) z = 1;
    const int chunks = ceil_div(k, 64 * kSkW);
    const int nchz = z > 1 ? ceil_div(chunks, z) : chunks;
    z = z > 1 ? ceil_div(chunks, nchz) : 1;  // no empty split
    const int64_t ctiles = ceil_div(n, 16);
    MMPDE_REQUIRE(z == 1 || ctiles <= kSkTickets);
    // a split launch holds at most kSkTickets output tiles (one ticket each):
    // more rows run as row blocks of that many tiles, one launch each, with the
    // same split (a row's summation order does not depend on m)
    const int64_t rows_per = z > 1 ? 16 * (kSkTickets / ctiles) : m;
    unsigned *tickets = z > 1 ? (unsigned *)workspace : nullptr;
    float *part = z > 1 ? workspace + kSkTickets : nullptr;
    for (int64_t r0 = 0; r0 < m; r0 += rows_per) {
        const int64_t mr = m - r0 < rows_per ? m - r0 : rows_per;
        const dim3 grid((unsigned)ctiles, (unsigned)ceil_div(mr, 16), (unsigned)z);
        hipLaunchKernelGGL(linear_skinny_kernel<kSkW>, grid, dim3(kSkW * 64), 0, st, x + r0 * ldx, ldx, mr, k, w,
                           ldw, b, n, act, y + r0 * ldy, ldy, nchz, part, tickets);
        MMPDE_RET_LAUNCH();
    }
    return MMPDE_OK;
}

extern "C" int mmpde_linear_skinny(const float *x, int64_t ldx, int64_t m, int64_t k,
                                   const float *w, int64_t ldw, const float *b, int64_t n,
                                   int act, float *y, int64_t ldy, mmpde_stream_t stream) {
    return mmpde_linear_skinny_ws(x, ldx, m, k, w, ldw, b, n, act, y, ldy, nullptr, 0, stream);
}

extern "C" int mmpde_conv2d(const float *x, int64_t batches, int cin, int h, int w,
                            const float *weight, const float *bias, int cout, int ks, int stride,
                            int pad, const float *residual, int act, float *y,
                            mmpde_stream_t stream) {
    MMPDE_REQUIRE(x && weight && y && batches > 0 && cin > 0 && cout > 0 && ks > 0);
    MMPDE_REQUIRE((stride == 1 || stride == 2) && pad >= 0 && act >= 0 && act <= 2);
    const int oh = (h + 2 * pad - ks) / stride + 1;
    const int ow = (w + 2 * pad - ks) / stride + 1;
    MMPDE_REQUIRE(oh > 0 && ow > 0);
    return mmpde_detail::conv2d(x, batches, cin, h, w, weight, bias, cout, ks, stride, pad, residual, act,
                                y, as_stream(stream), nullptr, 0);
}

extern "C" int mmpde_conv2d_ex(const float *x, int64_t batches, int cin, int h, int w, const float *weight,
                               const float *bias, int cout, int ks, int stride, int pad, int pad_mode,
                               const float *residual, int res_after_act, int act, float *y,
                               mmpde_stream_t stream) {
    MMPDE_REQUIRE(x && weight && y && batches > 0 && cin > 0 && cout > 0 && ks > 0);
    MMPDE_REQUIRE((stride == 1 || stride == 2) && pad >= 0 && act >= 0 && act <= 3);
    MMPDE_REQUIRE(pad_mode == MMPDE_PAD_ZEROS || pad_mode == MMPDE_PAD_CIRCULAR);
    MMPDE_REQUIRE(!res_after_act || residual);
    const int oh = (h + 2 * pad - ks) / stride + 1;
    const int ow = (w + 2 * pad - ks) / stride + 1;
    MMPDE_REQUIRE(oh > 0 && ow > 0 && (pad_mode == MMPDE_PAD_ZEROS || (pad <= h && pad <= w)));
    return mmpde_detail::conv2d(x, batches, cin, h, w, weight, bias, cout, ks, stride, pad, residual, act,
                                y, as_stream(stream), nullptr, 0, pad_mode == MMPDE_PAD_CIRCULAR, res_after_act);
}

namespace mmpde_detail {
int conv2d(const float *x, int64_t batches, int cin, int h, int w, const float *weight, const float *bias,
           int cout, int ks, int stride, int pad, const float *residual, int act, float *y, hipStream_t st,
           unsigned *zero, int n_zero, int circular, int res_after_act) {
    const int oh = (h + 2 * pad - ks) / stride + 1;
    const int ow = (w + 2 * pad - ks) / stride + 1;
    const int64_t total = batches * cout * oh * ow;
    const int64_t threads = total > n_zero ? total : n_zero;
    hipLaunchKernelGGL(conv2d_kernel, dim3(ceil_div(threads, 256)), dim3(256), 0, st, x, batches, cin, h, w,
                       weight, bias, cout, ks, stride, pad, oh, ow, residual, act, y, zero, n_zero, circular,
                       res_after_act);
    MMPDE_RET_LAUNCH();
    return MMPDE_OK;
}
}  // namespace mmpde_detail

extern "C" int mmpde_conv2d_grad_weight(const float *x, int64_t batches, int cin, int h, int w, const float *dy,
                                        int cout, int ks, int pad, int pad_mode, float *dw_out, float *db_out,
                                        mmpde_stream_t stream) {
    MMPDE_REQUIRE(x && dy && dw_out && batches > 0 && batches <= INT32_MAX && cin > 0 && cout > 0);
    MMPDE_REQUIRE(ks > 0 && ks * ks <= kGwThreads && pad >= 0 && h > 0 && w > 0);
    MMPDE_REQUIRE(h + 2 * pad - ks + 1 == h && w + 2 * pad - ks + 1 == w);  // stride 1, output size = input size
    MMPDE_REQUIRE(pad_mode == MMPDE_PAD_ZEROS || (pad_mode == MMPDE_PAD_CIRCULAR && pad <= h && pad <= w));
    MMPDE_REQUIRE((int64_t)cin * cout < INT32_MAX && (int64_t)h * w < INT32_MAX / 2);
    const int T = ks * ks, S = kGwThreads / T;
    const size_t part = (size_t)(S * T + S) * sizeof(float);
    const size_t planes = (size_t)2 * h * w * sizeof(float);
    const bool lds = planes <= 64 * 1024;
    const size_t shm = lds ? (planes > part ? planes : part) : part;
    const dim3 grid((unsigned)(cin * cout));
    if (lds)
        hipLaunchKernelGGL(conv2d_grad_weight_kernel<true>, grid, dim3(kGwThreads), shm, as_stream(stream), x, dy,
                           (int)batches, cin, cout, h, w, ks, pad, pad_mode == MMPDE_PAD_CIRCULAR ? 1 : 0, dw_out,
                           db_out);
    else
        hipLaunchKernelGGL(conv2d_grad_weight_kernel<false>, grid, dim3(kGwThreads), shm, as_stream(stream), x, dy,
                           (int)batches, cin, cout, h, w, ks, pad, pad_mode == MMPDE_PAD_CIRCULAR ? 1 : 0, dw_out,
                           db_out);
    MMPDE_RET_LAUNCH();
    return MMPDE_OK;
}

extern "C" int mmpde_resample_bilinear(const float *x, int64_t planes, int h, int w, int oh, int ow, float *y,
                                       mmpde_stream_t stream) {
    MMPDE_REQUIRE(x && y && planes > 0 && h > 0 && w > 0 && oh > 0 && ow > 0);
    const float sy = oh > 1 ? (float)(h - 1) / (float)(oh - 1) : 0.0f;
    const float sx = ow > 1 ? (float)(w - 1) / (float)(ow - 1) : 0.0f;
    hipLaunchKernelGGL(resample_bilinear_kernel, dim3(ceil_div(planes * oh * ow, 256)), dim3(256), 0,
                       as_stream(stream), x, planes, h, w, oh, ow, sy, sx, y);
    MMPDE_RET_LAUNCH();
    return MMPDE_OK;
}
