// Diagnostic: the split of a float into an rtz fp16 hi and a lo half computed two ways
// (v_fma_mixlo/hi_f16 vs v_cvt_pkrtz of the f32 remainder); prints error statistics.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cmath>
#include <vector>
#include <random>
__global__ void k(const float* a, float* out, int n) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (2 * i + 1 >= n) return;
    float a0 = a[2 * i], a1 = a[2 * i + 1];
    auto h = __builtin_amdgcn_cvt_pkrtz(a0, a1);
    unsigned hi = __builtin_bit_cast(unsigned, h);
    unsigned lo;
    asm volatile("v_fma_mixlo_f16 %0, %1, 1.0, -%2 op_sel_hi:[0,0,1]\n\t"
        "v_fma_mixhi_f16 %0, %3, 1.0, -%2 op_sel:[0,0,1] op_sel_hi:[0,0,1]"
        : "=&v"(lo) : "v"(a0), "v"(hi), "v"(a1));
    auto l2 = __builtin_amdgcn_cvt_pkrtz(a0 - (float)h[0], a1 - (float)h[1]);
    typedef _Float16 hh2 __attribute__((ext_vector_type(2)));
    hh2 L = __builtin_bit_cast(hh2, lo);
    out[4 * i + 0] = (float)h[0] + (float)L[0];
    out[4 * i + 1] = (float)h[1] + (float)L[1];
    out[4 * i + 2] = (float)h[0] + (float)l2[0];
    out[4 * i + 3] = (float)h[1] + (float)l2[1];
}
int main() {
    const int n = 1 << 20;
    std::vector<float> a(n), o(2 * n);
    std::mt19937 g(1);
    std::uniform_real_distribution<float> u(-20.f, 14.f);
    for (int i = 0; i < n; ++i) a[i] = std::ldexp(1.0f + (g() % 100000) / 1e5f, (int)u(g)) * ((i & 1) ? 1 : 1);
    float *da, *dout;
    hipMalloc(&da, n * 4); hipMalloc(&dout, 2 * n * 4);
    hipMemcpy(da, a.data(), n * 4, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k, dim3(n / 2 / 256), dim3(256), 0, 0, da, dout, n);
    hipMemcpy(o.data(), dout, 2 * n * 4, hipMemcpyDeviceToHost);
    double emix = 0, ertz = 0, mmix = 0, mrtz = 0, bmix = 0, brtz = 0;
    for (int i = 0; i < n / 2; ++i)
        for (int e = 0; e < 2; ++e) {
            double x = a[2 * i + e];
            double r1 = (o[4 * i + e] - x) / x, r2 = (o[4 * i + 2 + e] - x) / x;
            emix += r1 * r1; ertz += r2 * r2; mmix = fmax(mmix, fabs(r1)); mrtz = fmax(mrtz, fabs(r2));
            bmix += r1; brtz += r2;
        }
    printf("mix: rms %.3g max %.3g bias %.3g | rtz: rms %.3g max %.3g bias %.3g\n", sqrt(emix / n), mmix, bmix / n, sqrt(ertz / n), mrtz, brtz / n);
    // worst mix cases
    int shown = 0;
    for (int i = 0; i < n / 2 && shown < 8; ++i)
        for (int e = 0; e < 2; ++e) {
            double x = a[2 * i + e];
            if (fabs((o[4 * i + e] - x) / x) > 1e-5 && shown < 8) { printf("x %.9g mix %.9g rtz %.9g\n", x, o[4 * i + e], o[4 * i + 2 + e]); ++shown; }
        }
    return 0;
}
