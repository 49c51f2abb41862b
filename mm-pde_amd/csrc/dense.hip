// Small dense helpers: skinny-M linear layers (res_cut MLP, DMM output_mlp /
// fc layers, the per-trajectory branch . W contraction) and a direct 2-D
// convolution (DMM ConvNet branch, Burgers res_cut).  These run at M = B
// (<= 32 rows), where every weight is read exactly once: they are weight-
// streaming (HBM-bound) kernels, one wave per 4 output columns, lanes striding K
// so each weight row is read coalesced.
#include "common.hpp"

namespace {

constexpr int kCols = 4;  // output columns per wave

template <int MB>
__global__ __launch_bounds__(256) void linear_skinny_kernel(const float *__restrict__ x,
                                                            int64_t ldx, int64_t m, int64_t k,
                                                            const float *__restrict__ w,
                                                            int64_t ldw,
                                                            const float *__restrict__ b,
                                                            int64_t n, int act,
                                                            float *__restrict__ y, int64_t ldy) {
    const int wave = threadIdx.x >> 6;
    const int lane = threadIdx.x & 63;
    const int64_t n0 = ((int64_t)blockIdx.x * 4 + wave) * kCols;
    if (n0 >= n) return;
    const float *wr[kCols];
#pragma unroll
    for (int j = 0; j < kCols; ++j) wr[j] = w + (n0 + j < n ? n0 + j : n - 1) * ldw;
    for (int64_t r0 = 0; r0 < m; r0 += MB) {
        float acc[kCols][MB];
#pragma unroll
        for (int j = 0; j < kCols; ++j)
#pragma unroll
            for (int i = 0; i < MB; ++i) acc[j][i] = 0.0f;
        for (int64_t kk = lane; kk < k; kk += 64) {
            float wv[kCols];
#pragma unroll
            for (int j = 0; j < kCols; ++j) wv[j] = wr[j][kk];
#pragma unroll
            for (int i = 0; i < MB; ++i) {
                const int64_t row = r0 + i;
                const float xv = row < m ? x[row * ldx + kk] : 0.0f;
#pragma unroll
                for (int j = 0; j < kCols; ++j) acc[j][i] += xv * wv[j];
            }
        }
#pragma unroll
        for (int j = 0; j < kCols; ++j) {
#pragma unroll
            for (int i = 0; i < MB; ++i) {
                const float v = wave_sum(acc[j][i]);
                const int64_t row = r0 + i, col = n0 + j;
                if (lane == 0 && row < m && col < n)
                    y[row * ldy + col] = act_apply(v + (b ? b[col] : 0.0f), act);
            }
        }
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

}  // namespace

extern "C" int mmpde_version(void) { return 10100; }

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
    dim3 grid(ceil_div(n, 4 * kCols));
    if (m <= 1)
        hipLaunchKernelGGL((linear_skinny_kernel<1>), grid, dim3(256), 0, st, x, ldx, m, k, w, ldw, b, n, act, y, ldy);
    else if (m <= 2)
        hipLaunchKernelGGL((linear_skinny_kernel<2>), grid, dim3(256), 0, st, x, ldx, m, k, w, ldw, b, n, act, y, ldy);
    else if (m <= 4)
        hipLaunchKernelGGL((linear_skinny_kernel<4>), grid, dim3(256), 0, st, x, ldx, m, k, w, ldw, b, n, act, y, ldy);
    else if (m <= 8)
        hipLaunchKernelGGL((linear_skinny_kernel<8>), grid, dim3(256), 0, st, x, ldx, m, k, w, ldw, b, n, act, y, ldy);
    else
        hipLaunchKernelGGL((linear_skinny_kernel<16>), grid, dim3(256), 0, st, x, ldx, m, k, w, ldw, b, n, act, y, ldy);
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
