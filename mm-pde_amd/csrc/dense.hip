// Small dense helpers: skinny-M linear layers (res_cut MLP, DMM output_mlp /
// fc layers, the per-trajectory branch . W contraction) and a direct 2-D
// convolution (DMM ConvNet branch, Burgers res_cut).  These run at M = B
// (<= 32 rows), where every weight is read exactly once: they are weight-
// streaming (HBM-bound) kernels, one wave per 4 output columns, lanes striding K
// so each weight row is read coalesced.
#include "common.hpp"

namespace {

constexpr int kKc = 256;  // K chunk staged in LDS

// One wave per output column (4 per workgroup, so even N = 256 fills a few
// hundred waves); the workgroup stages x[r0 : r0+MB, kc : kc+256] in LDS once
// for its 4 columns, lanes stride K (k = kc + lane + 64 t) so every weight-row
// load is a coalesced 256-B wave access for any row stride / alignment.  Each
// weight is read exactly once; fixed summation order (deterministic).
template <int MB>
__global__ __launch_bounds__(256) void linear_skinny_kernel(const float *__restrict__ x,
                                                            int64_t ldx, int64_t m, int64_t k,
                                                            const float *__restrict__ w,
                                                            int64_t ldw,
                                                            const float *__restrict__ b,
                                                            int64_t n, int act,
                                                            float *__restrict__ y, int64_t ldy) {
    __shared__ float xs[MB][kKc];
    const int wave = threadIdx.x >> 6;
    const int lane = threadIdx.x & 63;
    const int64_t col = (int64_t)blockIdx.x * 4 + wave;
    const bool colok = col < n;
    const float *wr = w + (colok ? col : n - 1) * ldw;
    for (int64_t r0 = 0; r0 < m; r0 += MB) {
        float acc[MB];
#pragma unroll
        for (int i = 0; i < MB; ++i) acc[i] = 0.0f;
        for (int64_t kc = 0; kc < k; kc += kKc) {
            float wv[4];
#pragma unroll
            for (int t = 0; t < 4; ++t) {
                const int64_t kg = kc + lane + 64 * t;
                wv[t] = kg < k ? wr[kg] : 0.0f;
            }
            __syncthreads();  // previous chunk consumed
            for (int e = threadIdx.x; e < MB * kKc; e += 256) {
                const int i = e / kKc, kk = e % kKc;
                const int64_t row = r0 + i, kg = kc + kk;
                xs[i][kk] = (row < m && kg < k) ? x[row * ldx + kg] : 0.0f;
            }
            __syncthreads();
#pragma unroll
            for (int i = 0; i < MB; ++i) {
#pragma unroll
                for (int t = 0; t < 4; ++t) acc[i] = fmaf(xs[i][lane + 64 * t], wv[t], acc[i]);
            }
        }
#pragma unroll
        for (int i = 0; i < MB; ++i) {
            const float v = wave_sum(acc[i]);
            const int64_t row = r0 + i;
            if (lane == 0 && row < m && colok)
                y[row * ldy + col] = act_apply(v + (b ? b[col] : 0.0f), act);
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

extern "C" int mmpde_version(void) { return 10200; }

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
    dim3 grid(ceil_div(n, 4));
#define MMPDE_SKINNY(MB) \
    hipLaunchKernelGGL((linear_skinny_kernel<MB>), grid, dim3(256), 0, st, x, ldx, m, k, w, ldw, b, n, act, y, ldy)
    if (m <= 1) MMPDE_SKINNY(1);
    else if (m <= 2) MMPDE_SKINNY(2);
    else if (m <= 4) MMPDE_SKINNY(4);
    else if (m <= 8) MMPDE_SKINNY(8);
    else if (m <= 16) MMPDE_SKINNY(16);
    else MMPDE_SKINNY(32);
#undef MMPDE_SKINNY
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
