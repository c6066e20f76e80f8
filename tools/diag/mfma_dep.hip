// Diagnostic: cycles per v_mfma_f32_32x32x16_f16 for dependent vs independent accumulation
// chains, counted in shader cycles with s_memtime inside the kernel (clock-independent).  All
// operands in registers (no LDS, no global traffic in the timed loop); one wave per SIMD, 256
// workgroups.  chains k: k accumulators, MFMAs issued round-robin over them, 96 MFMAs per
// iteration.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint4 opaque(uint4 v) {
    u32x4 t = __builtin_bit_cast(u32x4, v);
    asm volatile("" : "+v"(t));
    return __builtin_bit_cast(uint4, t);
}
__device__ __forceinline__ f32x16 mf(uint4 a, uint4 b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b), c, 0, 0, 0);
}
template <int NC>
__global__ void __launch_bounds__(256, 1) kd(const uint4* src, float* out, unsigned long long* cyc, int iters) {
    const int tid = threadIdx.x, lane = tid & 63;
    uint4 a[8], b[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) { a[k] = src[k * 64 + lane]; b[k] = src[(8 + k) * 64 + lane]; }
    f32x16 acc[NC];
#pragma unroll
    for (int c = 0; c < NC; ++c)
#pragma unroll
        for (int i = 0; i < 16; ++i) acc[c][i] = 0.f;
    unsigned long long t0 = 0, t1 = 0;
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t0) :: "memory");
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int k = 0; k < 8; ++k) { a[k] = opaque(a[k]); b[k] = opaque(b[k]); }
#pragma unroll
        for (int m = 0; m < 96; ++m) acc[m % NC] = mf(a[m & 7], b[(m >> 3) & 7], acc[m % NC]);
    }
    float s = 0.f;
#pragma unroll
    for (int c = 0; c < NC; ++c)
#pragma unroll
        for (int i = 0; i < 16; ++i) s += acc[c][i];
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t1) :: "memory");
    out[blockIdx.x * 256 + tid] = s;
    if (lane == 0) atomicAdd(cyc, t1 - t0);
}
// B fragments from an LDS image as in the block kernels: per step of 3 MFMAs (a_h b_h, a_l b_h,
// a_h b_l) two ds_read_b128 (b_h, b_l) of a 528-B-stride row image, read LA steps ahead; the
// image row base moves with the iteration so nothing can be hoisted
template <int LA>
__global__ void __launch_bounds__(256, 1) kl(const uint4* src, float* out, unsigned long long* cyc, int iters) {
    __shared__ __attribute__((aligned(16))) uint8_t IMG[72 * 528];
    const int tid = threadIdx.x, lane = tid & 63, r = lane & 31, h = lane >> 5;
    for (int i = tid; i < 72 * 528 / 16; i += 256) reinterpret_cast<uint4*>(IMG)[i] = src[i % 1024];
    uint4 a[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) a[k] = src[k * 64 + lane];
    __syncthreads();
    f32x16 acc;
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[i] = 0.f;
    unsigned long long t0 = 0, t1 = 0;
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t0) :: "memory");
    for (int it = 0; it < iters; ++it) {
        const uint8_t* base = IMG + ((it & 3) + r) * 528 + h * 16;
        uint4 bh[LA + 1], bl[LA + 1];
#pragma unroll
        for (int q = 0; q < LA; ++q) { bh[q] = *reinterpret_cast<const uint4*>(base + q * 32); bl[q] = *reinterpret_cast<const uint4*>(base + 256 + q * 32); }
#pragma unroll
        for (int st = 0; st < 32; ++st) {
            const int cb = st % (LA + 1);
            acc = mf(a[st & 7], bh[cb], acc);
            if (st + LA < 32) {
                const int n = (st + LA) % (LA + 1);
                bh[n] = *reinterpret_cast<const uint4*>(base + ((st + LA) & 7) * 32 + ((st + LA) >> 3) * 528);
                bl[n] = *reinterpret_cast<const uint4*>(base + 256 + ((st + LA) & 7) * 32 + ((st + LA) >> 3) * 528);
            }
            acc = mf(a[(st + 1) & 7], bh[cb], acc);
            acc = mf(a[st & 7], bl[cb], acc);
        }
    }
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i) s += acc[i];
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t1) :: "memory");
    out[blockIdx.x * 256 + tid] = s;
    if (lane == 0) atomicAdd(cyc, t1 - t0);
}

int main() {
    std::vector<_Float16> h(16 * 64 * 8);
    for (size_t i = 0; i < h.size(); ++i) h[i] = (_Float16)((int)(i * 2654435761u % 2001) / 1000.0f - 1.0f);
    uint4* d; float* o; unsigned long long* c;
    (void)hipMalloc(&d, h.size() * 2); (void)hipMalloc(&o, 256 * 256 * 4); (void)hipMalloc(&c, 8);
    (void)hipMemcpy(d, h.data(), h.size() * 2, hipMemcpyHostToDevice);
    const int iters = 2000;
    auto run = [&](auto kern, int nc) {
        for (int rep = 0; rep < 3; ++rep) {
            (void)hipMemset(c, 0, 8);
            hipLaunchKernelGGL(kern, dim3(256), dim3(256), 0, 0, d, o, c, iters);
            (void)hipDeviceSynchronize();
        }
        unsigned long long v; (void)hipMemcpy(&v, c, 8, hipMemcpyDeviceToHost);
        printf("chains %d: %.1f shader cycles per MFMA (per wave)\n", nc, (double)v / (256 * 4) / (96.0 * iters));
    };
    run(kd<1>, 1); run(kd<2>, 2); run(kd<3>, 3); run(kd<4>, 4);
    auto runl = [&](auto kern, int la) {
        for (int rep = 0; rep < 3; ++rep) {
            (void)hipMemset(c, 0, 8);
            hipLaunchKernelGGL(kern, dim3(256), dim3(256), 0, 0, d, o, c, iters);
            (void)hipDeviceSynchronize();
        }
        unsigned long long v; (void)hipMemcpy(&v, c, 8, hipMemcpyDeviceToHost);
        printf("LDS B, lookahead %d steps: %.1f shader cycles per MFMA (per wave)\n", la, (double)v / (256 * 4) / (96.0 * iters));
    };
    runl(kl<1>, 1); runl(kl<2>, 2); runl(kl<3>, 3);
    return 0;
}
