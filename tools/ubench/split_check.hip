#include <hip/hip_runtime.h>
typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void split8_asm(float4 a, float4 b, half8 &hi, half8 &lo) {
    u32x4 h, l;
    asm("v_cvt_pk_f16_f32 %0, %8, %9\n\t"
        "v_cvt_pk_f16_f32 %1, %10, %11\n\t"
        "v_cvt_pk_f16_f32 %2, %12, %13\n\t"
        "v_cvt_pk_f16_f32 %3, %14, %15\n\t"
        "v_fma_mixlo_f16 %4, %8, 1.0, -%0 op_sel_hi:[0,0,1]\n\t"
        "v_fma_mixhi_f16 %4, %9, 1.0, -%0 op_sel:[0,0,1] op_sel_hi:[0,0,1]\n\t"
        "v_fma_mixlo_f16 %5, %10, 1.0, -%1 op_sel_hi:[0,0,1]\n\t"
        "v_fma_mixhi_f16 %5, %11, 1.0, -%1 op_sel:[0,0,1] op_sel_hi:[0,0,1]\n\t"
        "v_fma_mixlo_f16 %6, %12, 1.0, -%2 op_sel_hi:[0,0,1]\n\t"
        "v_fma_mixhi_f16 %6, %13, 1.0, -%2 op_sel:[0,0,1] op_sel_hi:[0,0,1]\n\t"
        "v_fma_mixlo_f16 %7, %14, 1.0, -%3 op_sel_hi:[0,0,1]\n\t"
        "v_fma_mixhi_f16 %7, %15, 1.0, -%3 op_sel:[0,0,1] op_sel_hi:[0,0,1]\n\t"
        "s_nop 1"
        : "=&v"(h.x), "=&v"(h.y), "=&v"(h.z), "=&v"(h.w), "=&v"(l.x), "=&v"(l.y), "=&v"(l.z), "=&v"(l.w)
        : "v"(a.x), "v"(a.y), "v"(a.z), "v"(a.w), "v"(b.x), "v"(b.y), "v"(b.z), "v"(b.w));
    hi = *(half8 *)&h;
    lo = *(half8 *)&l;
}
__global__ void k(const float4 *x, half8 *out) {
    int i = blockIdx.x * 64 + threadIdx.x;
    half8 hi, lo, hi2, lo2;
    float4 a = x[2 * i], b = x[2 * i + 1];
    split8_asm(a, b, hi, lo);
    float v[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
    for (int j = 0; j < 8; ++j) { _Float16 h = (_Float16)v[j]; hi2[j] = h; lo2[j] = (_Float16)(v[j] - (float)h); }
    out[4 * i] = hi; out[4 * i + 1] = lo; out[4 * i + 2] = hi2; out[4 * i + 3] = lo2;
}
int main() {
    const int n = 64 * 256;
    float *hx = (float *)malloc(n * 8 * 4);
    srand(1);
    for (int i = 0; i < n * 8; ++i) { float r = (float)rand() / RAND_MAX; hx[i] = (r - 0.3f) * powf(2.0f, (rand() % 30) - 10); }
    hx[0] = 0.0f; hx[1] = -0.0f; hx[2] = 65000.f; hx[3] = 1e-7f;
    float4 *dx; half8 *dout;
    hipMalloc(&dx, n * 32); hipMalloc(&dout, n * 64);
    hipMemcpy(dx, hx, n * 32, hipMemcpyHostToDevice);
    k<<<256, 64>>>(dx, dout);
    unsigned short *ho = (unsigned short *)malloc(n * 64);
    hipMemcpy(ho, dout, n * 64, hipMemcpyDeviceToHost);
    long bad = 0;
    for (int i = 0; i < n; ++i) for (int j = 0; j < 16; ++j) if (ho[i * 32 + j] != ho[i * 32 + 16 + j]) ++bad;
    printf("split8_asm mismatches: %ld of %d\n", bad, n * 16);
    return bad != 0;
}
