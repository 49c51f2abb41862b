// Softmax kernel smoother of the DMM training loss and mesh-quality metrics
// (reference mesh/dmm_utils.py:233-249 interpolate, :251-267 interpolate_tri):
//
//   out_q = sum_j v_j w_j,   w = softmax_j(-scale |p_j - x_q|)
//
// over a point set p (the n x n linspace grid for interpolate, scale = n; a
// trajectory's mesh for interpolate_tri, scale = sqrt(n)) with per-point
// values v.  The reference materialises [queries, points] distance and weight
// tensors (the value field repeated once per query); here one wave takes one
// query, streams the points once and keeps an online softmax (running max,
// rescaled sums) per lane, merged across the wave at the end.  The VJP with
// respect to the query position (what autograd.grad(out, x) and the loss's
// backward through x + grad(phi) need):
//
//   d out_q / d x_q = sum_j w_j (v_j - out_q) ds_j / dx_q,
//   ds_j / dx_q = -scale (x_q - p_j) / |x_q - p_j|   (0 where they coincide,
//   as torch.norm's backward).
//
// Point sets and value sets are shared by consecutive queries: query q uses
// point set q / (n_q / pts_sets) and value set q / (n_q / val_sets).
#include "common.hpp"

namespace {

// Online softmax state of one lane: running max m, sum of exp(s - m), and
// sums of exp(s - m) times v, d, v d (d = ds/dx, ds/dy).
struct Acc {
    float m = -3.0e38f, z = 0.0f, zv = 0.0f, zdx = 0.0f, zdy = 0.0f, zvdx = 0.0f, zvdy = 0.0f;
    __device__ __forceinline__ void rescale(float m_new) {
        const float c = __expf(m - m_new);
        z *= c;
        zv *= c;
        zdx *= c;
        zdy *= c;
        zvdx *= c;
        zvdy *= c;
        m = m_new;
    }
    __device__ __forceinline__ void merge(const Acc &o) {
        const float mn = fmaxf(m, o.m);
        const float a = __expf(m - mn), b = __expf(o.m - mn);
        z = z * a + o.z * b;
        zv = zv * a + o.zv * b;
        zdx = zdx * a + o.zdx * b;
        zdy = zdy * a + o.zdy * b;
        zvdx = zvdx * a + o.zvdx * b;
        zvdy = zvdy * a + o.zvdy * b;
        m = mn;
    }
};

__device__ __forceinline__ Acc wave_merge(Acc a) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
        Acc b;
        b.m = __shfl_xor(a.m, o, 64);
        b.z = __shfl_xor(a.z, o, 64);
        b.zv = __shfl_xor(a.zv, o, 64);
        b.zdx = __shfl_xor(a.zdx, o, 64);
        b.zdy = __shfl_xor(a.zdy, o, 64);
        b.zvdx = __shfl_xor(a.zvdx, o, 64);
        b.zvdy = __shfl_xor(a.zvdy, o, 64);
        a.merge(b);
    }
    return a;
}

// GRAD = false: out[q]; GRAD = true: gq[q] = g[q] * d out_q / d x_q.
template <bool GRAD>
__global__ __launch_bounds__(256) void softmax_interp_kernel(const float2 *__restrict__ pts, int n_pts,
                                                             int64_t q_per_pset,
                                                             const float *__restrict__ vals,
                                                             int64_t q_per_vset,
                                                             const float2 *__restrict__ qry, int64_t n_q,
                                                             float scale, const float *__restrict__ g,
                                                             float *__restrict__ out) {
    const int lane = threadIdx.x & 63;
    const int64_t q = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (q >= n_q) return;  // wave-uniform
    const float2 *P = pts + (q / q_per_pset) * (int64_t)n_pts;
    const float *V = vals + (q / q_per_vset) * (int64_t)n_pts;
    const float2 x = qry[q];
    Acc a;
    for (int j = lane; j < n_pts; j += 64) {
        const float2 p = P[j];
        const float dx = x.x - p.x, dy = x.y - p.y;
        const float r = sqrtf(dx * dx + dy * dy);
        const float s = -scale * r;
        if (s > a.m) a.rescale(s);
        const float e = __expf(s - a.m), v = V[j];
        a.z += e;
        a.zv += e * v;
        if (GRAD) {
            const float ir = r > 0.0f ? -scale / r : 0.0f;
            const float ddx = ir * dx, ddy = ir * dy;
            a.zdx += e * ddx;
            a.zdy += e * ddy;
            a.zvdx += e * v * ddx;
            a.zvdy += e * v * ddy;
        }
    }
    a = wave_merge(a);
    if (lane == 0) {
        const float o = a.zv / a.z;
        if (GRAD) {
            // sum_j w_j (v_j - o) d_j = (zvd - o zd) / z
            const float gg = g[q];
            out[2 * q] = gg * (a.zvdx - o * a.zdx) / a.z;
            out[2 * q + 1] = gg * (a.zvdy - o * a.zdy) / a.z;
        } else {
            out[q] = o;
        }
    }
}

int check_sets(int64_t n_pts, int64_t pts_sets, int64_t val_sets, int64_t n_q) {
    if (n_pts < 1 || n_pts > INT32_MAX || pts_sets < 1 || val_sets < 1 || n_q < 1) return MMPDE_ERR_INVALID_ARG;
    if (n_q % pts_sets || n_q % val_sets) return MMPDE_ERR_INVALID_ARG;
    return MMPDE_OK;
}

}  // namespace

extern "C" int mmpde_softmax_interp(const float *pts, int64_t n_pts, int64_t pts_sets, const float *vals,
                                    int64_t val_sets, const float *qry, int64_t n_q, float scale, float *out,
                                    mmpde_stream_t stream) {
    MMPDE_REQUIRE(pts && vals && qry && out);
    const int rc = check_sets(n_pts, pts_sets, val_sets, n_q);
    if (rc) return rc;
    hipLaunchKernelGGL(softmax_interp_kernel<false>, dim3((unsigned)ceil_div(n_q, 4)), dim3(256), 0,
                       as_stream(stream), (const float2 *)pts, (int)n_pts, n_q / pts_sets, vals, n_q / val_sets,
                       (const float2 *)qry, n_q, scale, nullptr, out);
    MMPDE_RET_LAUNCH();
    return MMPDE_OK;
}

extern "C" int mmpde_softmax_interp_grad(const float *pts, int64_t n_pts, int64_t pts_sets, const float *vals,
                                         int64_t val_sets, const float *qry, int64_t n_q, float scale,
                                         const float *grad_out, float *grad_qry, mmpde_stream_t stream) {
    MMPDE_REQUIRE(pts && vals && qry && grad_out && grad_qry);
    const int rc = check_sets(n_pts, pts_sets, val_sets, n_q);
    if (rc) return rc;
    hipLaunchKernelGGL(softmax_interp_kernel<true>, dim3((unsigned)ceil_div(n_q, 4)), dim3(256), 0,
                       as_stream(stream), (const float2 *)pts, (int)n_pts, n_q / pts_sets, vals, n_q / val_sets,
                       (const float2 *)qry, n_q, scale, grad_out, grad_qry);
    MMPDE_RET_LAUNCH();
    return MMPDE_OK;
}
