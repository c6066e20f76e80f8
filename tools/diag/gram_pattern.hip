// Diagnostic: the memory-pattern ceiling of the ours-Gram backward (k_gram_bwd_s, gram_split.hip).
// The kernel reads 30 activation tensors and writes D over them in place; per stage a workgroup
// moves 16 rows x 32 channels (one 128-B line per row) of each tensor.  These kernels keep only
// that data movement (no LDS image, no MFMA, no barriers) so the rate they reach is what the
// access pattern itself allows, and compare it with other patterns:
//   quarter  the kernel's pattern: workgroup (clip, chunk, 32-channel group), 128-B lines
//   rows     workgroup (clip, chunk, quarter of the chunk), whole 512-B rows, 4 rows per stage
//   oop      quarter, D to a second set of tensors (out of place)
//   read     quarter, loads only (the Gram forward's pattern)
// each at 1 workgroup per CU (dynamic LDS as the real kernel's 116 KiB), 2 per CU, and unlimited.
// B = 256, T = 16384, 30 tensors spaced as api.hip's tensor_pad (1 MiB + 4 KiB).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

constexpr int C = 128, B = 256, T = 16384, NU = 30, NCH = 4, GSS = 16;
constexpr size_t PAD = 263168;
constexpr size_t TSTRIDE = (size_t)B * T * C + PAD;

__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
    const int xcd = bid % 8, q = nwg / 8, rr = nwg % 8;
    return (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + bid / 8;
}

__device__ __forceinline__ float4 f(float4 v) {
    return make_float4(fmaf(v.x, 0.999f, 1e-3f), fmaf(v.y, 0.999f, 1e-3f), fmaf(v.z, 0.999f, 1e-3f),
                       fmaf(v.w, 0.999f, 1e-3f));
}

// MODE 0 quarter in place, 1 rows in place, 2 quarter out of place, 3 quarter read only,
// 4 quarter over a channel-group-major layout [b][cg][t][32] in place, 5 the same read only,
// 6 rows read only, 7 quarter in place with a barrier per stage, 8 half rows (64 channels =
// 256 B per row, two workgroups per chunk) read only, 9 half rows in place
template <int MODE>
__global__ void __launch_bounds__(512) kpat(float* act, float* out, float* sink) {
    extern __shared__ float dyn[];
    const int nwg = B * NCH * 4;
    int work = xcd_remap(blockIdx.x, nwg);
    const int cg = work % 4; work /= 4;
    const int ch = work % NCH, b = work / NCH;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const float* ld[8];
    float* stp[8];
    int tbeg, tlen;
    uint32_t lofs, rstep;   // lane offset, rows per stage
    int rowl;
    const bool half = MODE == 8 || MODE == 9;
    const bool rows = MODE == 1 || MODE == 6;
    const bool cgm = MODE == 4 || MODE == 5;
    const bool ro = MODE == 3 || MODE == 5 || MODE == 6 || MODE == 8;
    uint32_t rs = C;
    if (half) {
        // workgroup (chunk, channel half, time half of the chunk): 16 tensors per thread-set
        tlen = T / NCH / 2; tbeg = ch * (T / NCH) + (cg >> 1) * tlen;
        const int uo = w & 1;
        rowl = (lane >> 4) + 4 * (w >> 1);
        lofs = 64 * (cg & 1) + 4 * (lane & 15);
        rstep = GSS;
#pragma unroll
        for (int k = 0; k < 8; ++k) {   // (tensors 16 uo + 2 k .. : two per slot, see load)
            const int u = 16 * uo + 2 * k;
            ld[k] = u < NU ? act + (size_t)u * TSTRIDE + (size_t)b * T * C : act;
            stp[k] = u < NU ? act + (size_t)u * TSTRIDE + (size_t)b * T * C : nullptr;
        }
    } else if (rows) {
        tlen = T / NCH / 4; tbeg = ch * (T / NCH) + cg * tlen;
        const int uo = w >> 1;
        rowl = (lane >> 5) + 2 * (w & 1);
        lofs = 4 * (lane & 31);
        rstep = 4;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const int u = 8 * uo + k;
            ld[k] = u < NU ? act + (size_t)u * TSTRIDE + (size_t)b * T * C : act;
            stp[k] = u < NU ? act + (size_t)u * TSTRIDE + (size_t)b * T * C : nullptr;
        }
    } else {
        tlen = T / NCH; tbeg = ch * tlen;
        const int uo = w & 3, sq = lane >> 3;
        rowl = 8 * (w >> 2) + (lane & 7);
        lofs = 32 * cg + 4 * sq;
        rstep = GSS;
        size_t cb = 0;
        if (cgm) { lofs = 4 * sq; rs = 32; cb = (size_t)cg * T * 32; }
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const int u = 8 * uo + k;
            ld[k] = u < NU ? act + (size_t)u * TSTRIDE + (size_t)b * T * C + cb : act;
            float* base = MODE == 2 ? out : act;
            stp[k] = u < NU ? base + (size_t)u * TSTRIDE + (size_t)b * T * C + cb : nullptr;
        }
    }
    float4 v[2][8], v2[2][8];
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    const int tend = tbeg + tlen;
    auto load = [&](float4 (&r)[8], int t0) {
        const int tr = min(t0, tend - (int)rstep);
#pragma unroll
        for (int k = 0; k < 8; ++k) r[k] = *reinterpret_cast<const float4*>(ld[k] + lofs + (size_t)(tr + rowl) * rs);
    };
    auto load2 = [&](float4 (&r)[8], int t0) {   // half mode: tensor u + 1 of each slot
        const int tr = min(t0, tend - (int)rstep);
#pragma unroll
        for (int k = 0; k < 8; ++k)
            r[k] = *reinterpret_cast<const float4*>(ld[k] + (16 * (w & 1) + 2 * k + 1 < NU ? TSTRIDE : 0) + lofs + (size_t)(tr + rowl) * rs);
    };
    auto stage = [&](float4 (&r)[8], float4 (&r2)[8], int t0) {
        float4 o[8], o2[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) { o[k] = f(r[k]); o2[k] = f(r2[k]); }
        load(r, t0 + 2 * rstep);
        if (half) load2(r2, t0 + 2 * rstep);
        if (half) {
            if (ro) {
#pragma unroll
                for (int k = 0; k < 8; ++k) { acc.x += o2[k].x; acc.y += o2[k].y; acc.z += o2[k].z; acc.w += o2[k].w; }
            } else {
#pragma unroll
                for (int k = 0; k < 8; ++k)
                    if (stp[k] && 16 * (w & 1) + 2 * k + 1 < NU)
                        *reinterpret_cast<float4*>(stp[k] + TSTRIDE + lofs + (size_t)(t0 + rowl) * rs) = o2[k];
            }
        }
        if (MODE == 7) __syncthreads();
        if (ro) {
#pragma unroll
            for (int k = 0; k < 8; ++k) { acc.x += o[k].x; acc.y += o[k].y; acc.z += o[k].z; acc.w += o[k].w; }
        } else {
#pragma unroll
            for (int k = 0; k < 8; ++k)
                if (stp[k]) *reinterpret_cast<float4*>(stp[k] + lofs + (size_t)(t0 + rowl) * rs) = o[k];
        }
    };
    load(v[0], tbeg);
    load(v[1], tbeg + rstep);
    if (half) { load2(v2[0], tbeg); load2(v2[1], tbeg + rstep); }
    for (int t0 = tbeg; t0 < tend; t0 += 2 * rstep) {
        stage(v[0], v2[0], t0);
        stage(v[1], v2[1], t0 + rstep);
    }
    if (ro && acc.x == 1234.5f) sink[tid] = acc.y + acc.z + acc.w + dyn[0];
}

// half rows with the register budget of a one-wave-per-SIMD kernel: 256 threads, 8-row stages,
// thread (w, l): quad l & 15, row (l >> 4) + 4 (w & 1), tensors 16 (w >> 1) + k (k < 16)
template <bool RO>
__global__ void __launch_bounds__(256, 1) kpat_h256(float* act, float* sink) {
    extern __shared__ float dyn[];
    const int nwg = B * NCH * 4;
    int work = xcd_remap(blockIdx.x, nwg);
    const int cg = work % 4; work /= 4;
    const int ch = work % NCH, b = work / NCH;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int tlen = T / NCH / 2, tbeg = ch * (T / NCH) + (cg >> 1) * tlen, tend = tbeg + tlen;
    const int rowl = (lane >> 4) + 4 * (w & 1);
    const uint32_t lofs = 64 * (cg & 1) + 4 * (lane & 15);
    float* base = act + (size_t)b * T * C;
    const int u0 = 16 * (w >> 1);
    float4 v[2][16];
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    auto load = [&](float4 (&r)[16], int t0) {
        const int tr = min(t0, tend - 8);
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            const int u = u0 + k < NU ? u0 + k : 0;
            r[k] = *reinterpret_cast<const float4*>(base + (size_t)u * TSTRIDE + lofs + (size_t)(tr + rowl) * C);
        }
    };
    auto stage = [&](float4 (&r)[16], int t0) {
        float4 o[16];
#pragma unroll
        for (int k = 0; k < 16; ++k) o[k] = f(r[k]);
        load(r, t0 + 16);
        __syncthreads();
        if (RO) {
#pragma unroll
            for (int k = 0; k < 16; ++k) { acc.x += o[k].x; acc.y += o[k].y; acc.z += o[k].z; acc.w += o[k].w; }
        } else {
#pragma unroll
            for (int k = 0; k < 16; ++k)
                if (u0 + k < NU) *reinterpret_cast<float4*>(base + (size_t)(u0 + k) * TSTRIDE + lofs + (size_t)(t0 + rowl) * C) = o[k];
        }
    };
    load(v[0], tbeg);
    load(v[1], tbeg + 8);
    for (int t0 = tbeg; t0 < tend; t0 += 16) {
        stage(v[0], t0);
        stage(v[1], t0 + 8);
    }
    if (RO && acc.x == 1234.5f) sink[tid] = acc.y + acc.z + acc.w + dyn[0];
}

int main() {
    float *act, *out, *sink;
    const size_t bytes = (size_t)(NU + 1) * TSTRIDE * 4;
    if (hipMalloc(&act, bytes) != hipSuccess || hipMalloc(&out, bytes) != hipSuccess || hipMalloc(&sink, 4096) != hipSuccess) {
        printf("alloc failed\n");
        return 1;
    }
    (void)hipMemset(act, 0, bytes);
    (void)hipMemset(out, 0, bytes);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    const double tb = (double)NU * B * T * C * 4;
    auto run = [&](auto kern, const char* name, size_t lds, double rw) {
        (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        for (int i = 0; i < 2; ++i) hipLaunchKernelGGL(kern, dim3(B * NCH * 4), dim3(512), lds, 0, act, out, sink);
        (void)hipDeviceSynchronize();
        const int n = 6;
        (void)hipEventRecord(e0, 0);
        for (int i = 0; i < n; ++i) hipLaunchKernelGGL(kern, dim3(B * NCH * 4), dim3(512), lds, 0, act, out, sink);
        (void)hipEventRecord(e1, 0);
        (void)hipEventSynchronize(e1);
        float ms;
        (void)hipEventElapsedTime(&ms, e0, e1);
        ms /= n;
        const hipError_t err = hipGetLastError();
        printf("%-8s lds %6zu  %7.3f ms  %6.3f TB/s%s\n", name, lds, ms, rw * tb / (ms * 1e-3) / 1e12,
               err == hipSuccess ? "" : hipGetErrorString(err));
        fflush(stdout);
    };
    auto run256 = [&](auto kern, const char* name, size_t lds, double rw) {
        (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        for (int i = 0; i < 2; ++i) hipLaunchKernelGGL(kern, dim3(B * NCH * 4), dim3(256), lds, 0, act, sink);
        (void)hipDeviceSynchronize();
        const int n = 6;
        (void)hipEventRecord(e0, 0);
        for (int i = 0; i < n; ++i) hipLaunchKernelGGL(kern, dim3(B * NCH * 4), dim3(256), lds, 0, act, sink);
        (void)hipEventRecord(e1, 0);
        (void)hipEventSynchronize(e1);
        float ms;
        (void)hipEventElapsedTime(&ms, e0, e1);
        ms /= n;
        printf("%-8s lds %6zu  %7.3f ms  %6.3f TB/s\n", name, lds, ms, rw * tb / (ms * 1e-3) / 1e12);
        fflush(stdout);
    };
    const size_t ldss[1] = {118784};
    for (int rep = 0; rep < 2; ++rep)
        for (size_t lds : ldss) {
            run256(kpat_h256<false>, "h256", 102400, 2.0);
            run256(kpat_h256<true>, "h256_rd", 102400, 1.0);
            run(kpat<0>, "quarter", lds, 2.0);
            run(kpat<9>, "half", lds, 2.0);
            run(kpat<1>, "rows", lds, 2.0);
            run(kpat<3>, "read", lds, 1.0);
            run(kpat<8>, "half_rd", lds, 1.0);
            run(kpat<6>, "rows_rd", lds, 1.0);
        }
    return 0;
}
