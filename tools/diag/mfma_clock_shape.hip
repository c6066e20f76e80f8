// Diagnostic: does the MFMA shape change the clock the chip holds under the split block kernels'
// load?  MI355X_MICROARCH.md (DVFS give-back, item 7) measured bare bf16 loops on random data:
// v_mfma_f32_16x16x32 delivered ~1.15x the FLOP/s of v_mfma_f32_32x32x16 at equal cycles per
// FLOP, from a higher held clock.  This runs the block kernels' GEMM-1 work per 64-position tile
// and wave (32 output channels x 64 positions x K = 384, three split-f16 products per step, A in
// AGPRs, B operands changing every tile) in both shapes on every CU for ~2.5 s each, with an
// optional VALU filler per MFMA step (the kernels issue ~3.5 VALU per MFMA), and reports wall
// TFLOP/s and the in-kernel clock (s_memtime / s_memrealtime).
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <vector>
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint4 to_agpr(uint4 v) {
    u32x4 t = __builtin_bit_cast(u32x4, v);
    asm volatile("" : "=a"(t) : "0"(t));
    return __builtin_bit_cast(uint4, t);
}
__device__ __forceinline__ f32x16 m32(uint4 a, uint4 b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b), c, 0, 0, 0);
}
__device__ __forceinline__ f32x4 m16(uint4 a, uint4 b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b), c, 0, 0, 0);
}
// one f16 ulp-scale perturbation per 32-bit word: operands differ tile to tile (random data)
__device__ __forceinline__ uint4 bump(uint4 v, uint32_t k) {
    return make_uint4(v.x ^ (k & 0x00030003u), v.y ^ ((k >> 2) & 0x00030003u), v.z ^ ((k >> 4) & 0x00030003u),
                      v.w ^ ((k >> 6) & 0x00030003u));
}

template <int SHAPE, int FILL>
__global__ void __launch_bounds__(256, 1) kshape(const uint4* wsrc, const uint4* bsrc, float* out,
                                                 unsigned long long* clk, int tiles) {
    const int lane = threadIdx.x & 63;
    uint4 w[24][2];
#pragma unroll
    for (int s = 0; s < 24; ++s)
#pragma unroll
        for (int hl = 0; hl < 2; ++hl) w[s][hl] = to_agpr(wsrc[(s * 2 + hl) * 64 + lane]);
    uint4 b[8][2];
#pragma unroll
    for (int k = 0; k < 8; ++k)
#pragma unroll
        for (int hl = 0; hl < 2; ++hl) b[k][hl] = bsrc[(k * 2 + hl) * 64 + lane];
    float f0 = lane * 1e-3f, f1 = 0.5f, f2 = 0.25f, f3 = 0.125f;
    float sum = 0.f;
    unsigned long long c0, c1, r0, r1;
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(c0) :: "memory");
    r0 = __builtin_amdgcn_s_memrealtime();
    for (int t = 0; t < tiles; ++t) {
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            b[k][0] = bump(b[k][0], t * 2654435761u + k);
            b[k][1] = bump(b[k][1], t * 40503u + k);
        }
        if (SHAPE == 0) {     // 2 column halves x 24 K-steps of 16 x 3 products = 144 MFMAs
#pragma unroll
            for (int J = 0; J < 2; ++J) {
                f32x16 acc = {};
#pragma unroll
                for (int s = 0; s < 24; ++s) {
                    const uint4 bh = b[(s + J) & 7][0], bl = b[(s + J) & 7][1];
                    acc = m32(w[s][0], bh, acc);
                    acc = m32(w[s][1], bh, acc);
                    acc = m32(w[s][0], bl, acc);
#pragma unroll
                    for (int f = 0; f < FILL; ++f) { f0 = fmaf(f0, f1, f2); f3 = fmaf(f3, f2, f1); }
                }
#pragma unroll
                for (int i = 0; i < 16; ++i) sum += acc[i];
            }
        } else {              // 2 row blocks x 4 column blocks x 12 K-steps of 32 x 3 = 288 MFMAs
#pragma unroll
            for (int J = 0; J < 2; ++J) {      // column half: 2 column blocks of 16
                f32x4 acc[2][2] = {};
#pragma unroll
                for (int s = 0; s < 12; ++s) {
#pragma unroll
                    for (int q = 0; q < 2; ++q)
#pragma unroll
                        for (int c = 0; c < 2; ++c) {
                            const uint4 bh = b[(s + 2 * J + c) & 7][0], bl = b[(s + 2 * J + c) & 7][1];
                            const int ws = (2 * s + q) % 24;
                            acc[q][c] = m16(w[ws][0], bh, acc[q][c]);
                            acc[q][c] = m16(w[ws][1], bh, acc[q][c]);
                            acc[q][c] = m16(w[ws][0], bl, acc[q][c]);
                        }
#pragma unroll
                    for (int f = 0; f < 2 * FILL; ++f) { f0 = fmaf(f0, f1, f2); f3 = fmaf(f3, f2, f1); }
                }
#pragma unroll
                for (int q = 0; q < 2; ++q)
#pragma unroll
                    for (int c = 0; c < 2; ++c)
#pragma unroll
                        for (int i = 0; i < 4; ++i) sum += acc[q][c][i];
            }
        }
    }
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(c1) :: "memory");
    r1 = __builtin_amdgcn_s_memrealtime();
    out[blockIdx.x * 256 + threadIdx.x] = sum + f0 + f3;
    if (lane == 0) {
        atomicAdd(&clk[0], c1 - c0);
        atomicAdd(&clk[1], r1 - r0);
    }
}

int main() {
    std::vector<_Float16> w(24 * 2 * 64 * 8), bb(8 * 2 * 64 * 8);
    uint32_t st = 12345;
    auto rnd = [&]() { st = st * 1664525u + 1013904223u; return (float)((st >> 9) & 0xffff) / 32768.0f - 1.0f; };
    for (auto& v : w) v = (_Float16)rnd();
    for (auto& v : bb) v = (_Float16)rnd();
    uint4 *dw, *db; float* o; unsigned long long* c;
    (void)hipMalloc(&dw, w.size() * 2); (void)hipMalloc(&db, bb.size() * 2);
    (void)hipMalloc(&o, 256 * 256 * 4); (void)hipMalloc(&c, 16);
    (void)hipMemcpy(dw, w.data(), w.size() * 2, hipMemcpyHostToDevice);
    (void)hipMemcpy(db, bb.data(), bb.size() * 2, hipMemcpyHostToDevice);
    const int tiles = 2000;       // 144 x 32768 FLOP x 2000 tiles x 1024 waves = 9.7e12 per launch
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
    auto run = [&](auto kern, const char* name) {
        for (int rep = 0; rep < 3; ++rep) {   // warm up the clock governor
            hipLaunchKernelGGL(kern, dim3(256), dim3(256), 0, 0, dw, db, o, c, tiles);
        }
        (void)hipDeviceSynchronize();
        (void)hipMemset(c, 0, 16);
        const int launches = 400;
        (void)hipEventRecord(e0, 0);
        auto h0 = std::chrono::steady_clock::now();
        int n = 0;
        for (; n < launches; ++n) {
            hipLaunchKernelGGL(kern, dim3(256), dim3(256), 0, 0, dw, db, o, c, tiles);
            if ((n & 7) == 7) {
                (void)hipDeviceSynchronize();
                if (std::chrono::duration<double>(std::chrono::steady_clock::now() - h0).count() > 2.5) { ++n; break; }
            }
        }
        (void)hipEventRecord(e1, 0);
        (void)hipEventSynchronize(e1);
        float ms;
        (void)hipEventElapsedTime(&ms, e0, e1);
        unsigned long long v[2];
        (void)hipMemcpy(v, c, 16, hipMemcpyDeviceToHost);
        const double flop = 144.0 * 32768.0 * tiles * 1024.0 * n;
        printf("%-34s %4d launches %8.3f ms each  %7.1f TF/s  clock %5.0f MHz  %.1f cyc/tile/wave\n", name, n,
               ms / n, flop / (ms * 1e-3) / 1e12, (double)v[0] / v[1] * 100.0,
               (double)v[0] / (1024.0 * tiles * n));
    };
    run(kshape<0, 0>, "32x32x16 f16, no filler");
    run(kshape<1, 0>, "16x16x32 f16, no filler");
    run(kshape<0, 4>, "32x32x16 f16, 8 VALU / 3 MFMA");
    run(kshape<1, 4>, "16x16x32 f16, 8 VALU / 3 MFMA-pairs");
    run(kshape<0, 0>, "32x32x16 f16, no filler (again)");
    run(kshape<1, 0>, "16x16x32 f16, no filler (again)");
    return 0;
}
