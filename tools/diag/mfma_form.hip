// Diagnostic: cycles per v_mfma_f32_32x32x16_f16 in the split block kernels' register form --
// A (weights) pinned to AGPRs, accumulator in arch VGPRs (build with -mllvm
// -amdgpu-mfma-vgpr-form=1), B fragments read from a 528-B-stride LDS image LA steps ahead, 3
// MFMAs per step (wh bh, wl bh, wh bl) on one accumulator, 24 steps per "half" as in GEMM 1 --
// against B held in registers.  SCHED 1 adds the kernels' step3_schedule groups.  In-kernel
// s_memtime (clock-independent); one wave per SIMD, 256 workgroups.  No inline-asm memory
// instructions (the LDS reads are plain loads the compiler counts).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
constexpr int RS = 528, ROWS = 72;
__device__ __forceinline__ uint4 to_agpr(uint4 v) {
    u32x4 t = __builtin_bit_cast(u32x4, v);
    asm volatile("" : "=a"(t) : "0"(t));
    return __builtin_bit_cast(uint4, t);
}
__device__ __forceinline__ uint4 opaque(uint4 v) {
    u32x4 t = __builtin_bit_cast(u32x4, v);
    asm volatile("" : "+v"(t));
    return __builtin_bit_cast(uint4, t);
}
__device__ __forceinline__ f32x16 mf(uint4 a, uint4 b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b), c, 0, 0, 0);
}
__device__ __forceinline__ void sched3() {
    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
    __builtin_amdgcn_sched_group_barrier(0x100, 4, 0);
#pragma unroll
    for (int m = 1; m < 3; ++m) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x002, 7, 0);
        __builtin_amdgcn_sched_group_barrier(0x200, 2, 0);
    }
    __builtin_amdgcn_sched_barrier(0);
}

// MODE 0: B from LDS; MODE 1: B in registers (8 fragment pairs, rotated per tile)
template <int MODE, int LA, int SCHED>
__global__ void __launch_bounds__(256, 1) kf(const uint4* wsrc, const uint4* isrc, float* out,
                                             unsigned long long* cyc, int tiles) {
    __shared__ __attribute__((aligned(16))) uint8_t IMG[ROWS * RS];
    const int tid = threadIdx.x, lane = tid & 63, r = lane & 31, h = lane >> 5;
    for (int i = tid; i < ROWS * RS / 16; i += 256) reinterpret_cast<uint4*>(IMG)[i] = isrc[i % 2048];
    uint4 wd[3][8][2];
#pragma unroll
    for (int tp = 0; tp < 3; ++tp)
#pragma unroll
        for (int kb = 0; kb < 8; ++kb)
#pragma unroll
            for (int hl = 0; hl < 2; ++hl) wd[tp][kb][hl] = wsrc[((tp * 8 + kb) * 2 + hl) * 64 + lane];
#pragma unroll
    for (int tp = 0; tp < 3; ++tp)
#pragma unroll
        for (int kb = 0; kb < 8; ++kb)
#pragma unroll
            for (int hl = 0; hl < 2; ++hl) wd[tp][kb][hl] = to_agpr(wd[tp][kb][hl]);
    uint4 rh[8], rl[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        rh[k] = *reinterpret_cast<const uint4*>(IMG + (r + k) * RS + h * 16);
        rl[k] = *reinterpret_cast<const uint4*>(IMG + (r + k) * RS + 256 + h * 16);
    }
    __syncthreads();
    float sum = 0.f;
    unsigned long long t0 = 0, t1 = 0;
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t0) :: "memory");
    for (int t = 0; t < tiles; ++t) {
        if (MODE == 1) {
#pragma unroll
            for (int k = 0; k < 8; ++k) { rh[k] = opaque(rh[k]); rl[k] = opaque(rl[k]); }
        }
#pragma unroll
        for (int J = 0; J < 2; ++J) {
            f32x16 acc;
#pragma unroll
            for (int i = 0; i < 16; ++i) acc[i] = 0.f;
            const uint8_t* base = IMG + (32 * J + r + (t & 3)) * RS + h * 16;
            uint4 bh[LA + 1], bl[LA + 1];
            auto rd = [&](int st, int slot) {
                const int tp = st >> 3, kb = st & 7;
                if (MODE == 1) { bh[slot] = rh[(kb + tp + J) & 7]; bl[slot] = rl[(kb + tp + J) & 7]; return; }
                const uint8_t* p = base + tp * RS + kb * 32;
                bh[slot] = *reinterpret_cast<const uint4*>(p);
                bl[slot] = *reinterpret_cast<const uint4*>(p + 256);
            };
#pragma unroll
            for (int q = 0; q < LA; ++q) rd(q, q);
#pragma unroll
            for (int st = 0; st < 24; ++st) {
                const int tp = st >> 3, kb = st & 7, cb = st % (LA + 1);
                acc = mf(wd[tp][kb][0], bh[cb], acc);
                if (st + LA < 24) rd(st + LA, (st + LA) % (LA + 1));
                acc = mf(wd[tp][kb][1], bh[cb], acc);
                acc = mf(wd[tp][kb][0], bl[cb], acc);
                if (SCHED) sched3();
            }
#pragma unroll
            for (int i = 0; i < 16; ++i) sum += acc[i];
        }
    }
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t1) :: "memory");
    out[blockIdx.x * 256 + tid] = sum;
    if (lane == 0) atomicAdd(cyc, t1 - t0);
}

int main() {
    std::vector<_Float16> w(3 * 8 * 2 * 64 * 8), im(2048 * 8);
    for (size_t i = 0; i < w.size(); ++i) w[i] = (_Float16)((int)(i * 2654435761u % 2001) / 1000.0f - 1.0f);
    for (size_t i = 0; i < im.size(); ++i) im[i] = (_Float16)((int)(i * 40503u % 1999) / 1000.0f - 1.0f);
    uint4 *dw, *di; float* o; unsigned long long* c;
    (void)hipMalloc(&dw, w.size() * 2); (void)hipMalloc(&di, im.size() * 2);
    (void)hipMalloc(&o, 256 * 256 * 4); (void)hipMalloc(&c, 8);
    (void)hipMemcpy(dw, w.data(), w.size() * 2, hipMemcpyHostToDevice);
    (void)hipMemcpy(di, im.data(), im.size() * 2, hipMemcpyHostToDevice);
    const int tiles = 400;
    auto run = [&](auto kern, const char* name) {
        for (int rep = 0; rep < 3; ++rep) {
            (void)hipMemset(c, 0, 8);
            hipLaunchKernelGGL(kern, dim3(256), dim3(256), 0, 0, dw, di, o, c, tiles);
            (void)hipDeviceSynchronize();
        }
        unsigned long long v; (void)hipMemcpy(&v, c, 8, hipMemcpyDeviceToHost);
        printf("%-40s %.1f shader cycles per MFMA (per wave)\n", name, (double)v / (256 * 4) / (tiles * 2 * 72.0));
    };
    run(kf<1, 2, 0>, "reg B");
    run(kf<1, 2, 1>, "reg B, step3 schedule");
    run(kf<0, 1, 0>, "LDS B, lookahead 1");
    run(kf<0, 2, 0>, "LDS B, lookahead 2");
    run(kf<0, 3, 0>, "LDS B, lookahead 3");
    run(kf<0, 2, 1>, "LDS B, lookahead 2, step3 schedule");
    run(kf<0, 3, 1>, "LDS B, lookahead 3, step3 schedule");
    return 0;
}
