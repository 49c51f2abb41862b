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

template <int kSkW>
__global__ __launch_bounds__(kSkW * 64) void linear_skinny_kernel(const float *__restrict__ x,
                                                                  int64_t ldx, int64_t m, int64_t k,
                                                                  const float *__restrict__ w,
                                                                  int64_t ldw,
                                                                  const float *__restrict__ b,
                                                                  int64_t n, int act,
                                                                  float *__restrict__ y, int64_t ldy) {
    constexpr int C = 64 * kSkW, LD = C + 4;
    __shared__ float sw[16 * LD], sx[16 * LD];
    const int tid = threadIdx.x;
    const int wave = tid >> 6;
    const int lane = tid & 63;
    const int r = lane & 15, g = lane >> 4;
    const int64_t col0 = (int64_t)blockIdx.x * 16, row0 = (int64_t)blockIdx.y * 16;
    const int K = (int)k;
    const int nch = (K + C - 1) / C;
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
    load(0);
    for (int c = 0; c < nch; ++c) {
        if (c) __syncthreads();  // chunk c - 1 consumed
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            sw[i * LD + tid] = lw[i];
            sx[i * LD + tid] = lx[i];
        }
        __syncthreads();
        if (c + 1 < nch) load((c + 1) * C);
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
    f32x4 *part = (f32x4 *)sw;  // [wave][lane]
    part[wave * 64 + lane] = acc;
    __syncthreads();
    if (wave != 0) return;
    f32x4 s = part[lane];
#pragma unroll
    for (int v = 1; v < kSkW; ++v) s += part[v * 64 + lane];
    const int64_t col = col0 + r;
    if (col >= n) return;
    const float bb = b ? b[col] : 0.0f;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const int64_t row = row0 + 4 * g + q;
        if (row < m) y[row * ldy + col] = act_apply(s[q] + bb, act);
    }
}

// one thread per output element; weight [cout][cin][ks][ks] (PyTorch layout)
__global__ __launch_bounds__(256) void conv2d_kernel(const float *__restrict__ x, int64_t batches,
                                                     int cin, int h, int w,
                                                     const float *__restrict__ wt,
                                                     const float *__restrict__ bias, int cout,
                                                     int ks, int stride, int pad, int oh, int ow,
                                                     const float *__restrict__ res, int act,
                                                     float *__restrict__ y) {
    const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const int64_t total = batches * cout * oh * ow;
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
            const int iy = oy * stride - pad + ky;
            if (iy < 0 || iy >= h) continue;
            for (int kx = 0; kx < ks; ++kx) {
                const int ix = ox * stride - pad + kx;
                if (ix < 0 || ix >= w) continue;
                acc += wp[ky * ks + kx] * xp[iy * w + ix];
            }
        }
    }
    if (res) acc = res[e] + acc;
    y[e] = act_apply(acc, act);
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

}  // namespace

extern "C" int mmpde_version(void) { return 10800; }

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

extern "C" int mmpde_linear_skinny(const float *x, int64_t ldx, int64_t m, int64_t k,
                                   const float *w, int64_t ldw, const float *b, int64_t n,
                                   int act, float *y, int64_t ldy, mmpde_stream_t stream) {
    MMPDE_REQUIRE(x && w && y && m > 0 && k > 0 && n > 0 && m <= 4096);
    MMPDE_REQUIRE(ldx >= k && ldw >= k && ldy >= n && act >= 0 && act <= 2);
    hipStream_t st = as_stream(stream);
    const dim3 grid((unsigned)ceil_div(n, 16), (unsigned)ceil_div(m, 16));
    hipLaunchKernelGGL(linear_skinny_kernel<kSkW>, grid, dim3(kSkW * 64), 0, st, x, ldx, m, k, w, ldw, b,
                       n, act, y, ldy);
    MMPDE_RET_LAUNCH();
    return MMPDE_OK;
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
    const int64_t total = batches * cout * oh * ow;
    hipLaunchKernelGGL(conv2d_kernel, dim3(ceil_div(total, 256)), dim3(256), 0, as_stream(stream),
                       x, batches, cin, h, w, weight, bias, cout, ks, stride, pad, oh, ow,
                       residual, act, y);
    MMPDE_RET_LAUNCH();
    return MMPDE_OK;
}
