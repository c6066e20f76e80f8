// Diagnostic: accumulation-chain structure of the split block kernels' GEMM-1 loop.  Each step
// of the kernels is three v_mfma_f32_32x32x16_f16 (ah wh, ah wl, al wh) into ONE accumulator,
// and the 24 steps of a column half chain on it too: every MFMA waits for the previous one's
// result.  Variants (same operands, same FLOPs, one wave per SIMD, 256 workgroups):
//   chains 1: the kernels' form (all 72 MFMAs of a column half on one accumulator)
//   chains 2: ah wh and al wh on accumulator A, ah wl on B, interleaved A B A (summed at the end)
//   chains 3: one accumulator per product
//   chains 2h: the two column halves' chains interleaved step by step (two accumulators)
//   reg B: the same four with the B fragments held in registers (no LDS reads)
// B fragments are read two steps ahead (the kernels' lookahead).
// Prints the median time per launch, TF/s and the cycles per MFMA at the clock given on the
// command line (MHz; from a GRBM_GUI_ACTIVE pass, tools/diag/mfma_clock.sh).
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
constexpr int RS = 528, ROWS = 66;
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint4 opaque(uint4 v) {
    u32x4 t = __builtin_bit_cast(u32x4, v);
    asm volatile("" : "+v"(t));
    return __builtin_bit_cast(uint4, t);
}
__device__ __forceinline__ uint4 lds16(const uint8_t* p) { return *reinterpret_cast<const uint4*>(p); }
__device__ __forceinline__ f32x16 mf(uint4 a, uint4 b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b), c, 0, 0, 0);
}

template <int MODE>   // B from LDS: 1, 2, 3 chains, 4 = halves interleaved; 5..8: the same with B in registers
__global__ void __launch_bounds__(256, 1) kc(const uint4* wsrc, const uint4* img_src, float* out, int ntiles) {
    __shared__ __attribute__((aligned(16))) uint8_t IMG[ROWS * RS];
    const int tid = threadIdx.x, lane = tid & 63, r = lane & 31, h = lane >> 5;
    for (int i = tid; i < ROWS * RS / 16; i += 256) reinterpret_cast<uint4*>(IMG)[i] = img_src[i];
    uint4 wd[3][8][2];
#pragma unroll
    for (int tp = 0; tp < 3; ++tp)
#pragma unroll
        for (int kb = 0; kb < 8; ++kb)
#pragma unroll
            for (int hl = 0; hl < 2; ++hl) wd[tp][kb][hl] = wsrc[((tp * 8 + kb) * 2 + hl) * 64 + lane];
    __syncthreads();
    float sum = 0.f;
    // MODE 5..8: B fragments from registers (8 fragment pairs, opaque per tile so the compiler
    // cannot fold tiles), isolating the accumulation chains from the LDS latency
    uint4 rh[8], rl[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) { rh[k] = lds16(IMG + (r + k) * RS + h * 16); rl[k] = lds16(IMG + (r + k) * RS + 256 + h * 16); }
    for (int t = 0; t < ntiles; ++t) {
        if (MODE >= 5) {
#pragma unroll
            for (int k = 0; k < 8; ++k) { rh[k] = opaque(rh[k]); rl[k] = opaque(rl[k]); }
        }
        if (MODE == 4 || MODE == 8) {
            f32x16 a0, a1;
#pragma unroll
            for (int i = 0; i < 16; ++i) { a0[i] = 0.f; a1[i] = 0.f; }
            uint4 b0h[3], b0l[3], b1h[3], b1l[3];
            auto rd = [&](int st, int slot) {
                const int tp = st >> 3, kb = st & 7;
                if (MODE == 8) { b0h[slot] = rh[kb]; b0l[slot] = rl[kb]; b1h[slot] = rh[(kb + 1) & 7]; b1l[slot] = rl[(kb + 1) & 7]; return; }
                const uint8_t* p0 = IMG + (r + 1 + tp - 1) * RS + kb * 32 + h * 16;
                const uint8_t* p1 = IMG + (32 + r + 1 + tp - 1) * RS + kb * 32 + h * 16;
                b0h[slot] = lds16(p0); b0l[slot] = lds16(p0 + 256); b1h[slot] = lds16(p1); b1l[slot] = lds16(p1 + 256);
            };
            rd(0, 0); rd(1, 1);
#pragma unroll
            for (int st = 0; st < 24; ++st) {
                const int tp = st >> 3, kb = st & 7, cb = st % 3;
                if (st + 2 < 24) rd(st + 2, (st + 2) % 3);
                a0 = mf(wd[tp][kb][0], b0h[cb], a0);
                a1 = mf(wd[tp][kb][0], b1h[cb], a1);
                a0 = mf(wd[tp][kb][1], b0h[cb], a0);
                a1 = mf(wd[tp][kb][1], b1h[cb], a1);
                a0 = mf(wd[tp][kb][0], b0l[cb], a0);
                a1 = mf(wd[tp][kb][0], b1l[cb], a1);
            }
#pragma unroll
            for (int i = 0; i < 16; ++i) sum += a0[i] + a1[i];
            continue;
        }
#pragma unroll
        for (int J = 0; J < 2; ++J) {
            f32x16 a, b, c;
#pragma unroll
            for (int i = 0; i < 16; ++i) { a[i] = 0.f; b[i] = 0.f; c[i] = 0.f; }
            uint4 bh[3], bl[3];
            auto rd = [&](int st, int slot) {
                const int tp = st >> 3, kb = st & 7;
                if (MODE >= 5) { bh[slot] = rh[(kb + 3 * J) & 7]; bl[slot] = rl[(kb + 3 * J) & 7]; return; }
                const uint8_t* p = IMG + (32 * J + r + 1 + tp - 1) * RS + kb * 32 + h * 16;
                bh[slot] = lds16(p);
                bl[slot] = lds16(p + 256);
            };
            rd(0, 0); rd(1, 1);
#pragma unroll
            for (int st = 0; st < 24; ++st) {
                const int tp = st >> 3, kb = st & 7, cb = st % 3;
                if (st + 2 < 24) rd(st + 2, (st + 2) % 3);
                const uint4 xh = bh[cb], xl = bl[cb];
                const int nch = MODE >= 5 ? MODE - 4 : MODE;
                if (nch == 1) {
                    a = mf(wd[tp][kb][0], xh, a);
                    a = mf(wd[tp][kb][1], xh, a);
                    a = mf(wd[tp][kb][0], xl, a);
                } else if (nch == 2) {
                    a = mf(wd[tp][kb][0], xh, a);
                    b = mf(wd[tp][kb][1], xh, b);
                    a = mf(wd[tp][kb][0], xl, a);
                } else {
                    a = mf(wd[tp][kb][0], xh, a);
                    b = mf(wd[tp][kb][1], xh, b);
                    c = mf(wd[tp][kb][0], xl, c);
                }
            }
#pragma unroll
            for (int i = 0; i < 16; ++i) sum += a[i] + b[i] + c[i];
        }
    }
    out[blockIdx.x * 256 + tid] = sum;
}

int main(int argc, char** argv) {
    const double mhz = argc > 1 ? atof(argv[1]) : 0.0;
    std::mt19937 g(7);
    std::uniform_real_distribution<float> u(-1.f, 1.f);
    std::vector<_Float16> w(64 * 64 * 8 * 3), im(ROWS * RS / 2);
    for (auto& x : w) x = (_Float16)u(g);
    for (size_t i = 0; i < im.size(); ++i) { float v = u(g); im[i] = (_Float16)(v > 0 ? v * 1000.f : 0.f); }
    uint4 *dw, *di; float* dout;
    (void)hipMalloc(&dw, w.size() * 2); (void)hipMalloc(&di, im.size() * 2); (void)hipMalloc(&dout, 256 * 256 * 4);
    (void)hipMemcpy(dw, w.data(), w.size() * 2, hipMemcpyHostToDevice);
    (void)hipMemcpy(di, im.data(), im.size() * 2, hipMemcpyHostToDevice);
    hipEvent_t e0, e1; (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
    const int nt = 256;
    const char* names[8] = {"LDS B: chains 1 (kernels' form)", "LDS B: chains 2", "LDS B: chains 3", "LDS B: chains 2h (halves)",
                            "reg B: chains 1", "reg B: chains 2", "reg B: chains 3", "reg B: chains 2h (halves)"};
    std::vector<float> tm[8];
    for (int round = 0; round < 10; ++round)
        for (int m = 0; m < 8; ++m) {
            (void)hipEventRecord(e0);
            for (int k = 0; k < 5; ++k) {
                switch (m) {
                    case 0: hipLaunchKernelGGL(kc<1>, dim3(256), dim3(256), 0, 0, dw, di, dout, nt); break;
                    case 1: hipLaunchKernelGGL(kc<2>, dim3(256), dim3(256), 0, 0, dw, di, dout, nt); break;
                    case 2: hipLaunchKernelGGL(kc<3>, dim3(256), dim3(256), 0, 0, dw, di, dout, nt); break;
                    case 3: hipLaunchKernelGGL(kc<4>, dim3(256), dim3(256), 0, 0, dw, di, dout, nt); break;
                    case 4: hipLaunchKernelGGL(kc<5>, dim3(256), dim3(256), 0, 0, dw, di, dout, nt); break;
                    case 5: hipLaunchKernelGGL(kc<6>, dim3(256), dim3(256), 0, 0, dw, di, dout, nt); break;
                    case 6: hipLaunchKernelGGL(kc<7>, dim3(256), dim3(256), 0, 0, dw, di, dout, nt); break;
                    case 7: hipLaunchKernelGGL(kc<8>, dim3(256), dim3(256), 0, 0, dw, di, dout, nt); break;
                }
            }
            (void)hipEventRecord(e1); (void)hipEventSynchronize(e1);
            float ms; (void)hipEventElapsedTime(&ms, e0, e1);
            if (round >= 2) tm[m].push_back(ms / 5);
        }
    const double nmf = 256.0 * 2 * 72;   // MFMAs per wave per launch
    for (int m = 0; m < 8; ++m) {
        std::sort(tm[m].begin(), tm[m].end());
        const double ms = tm[m][tm[m].size() / 2];
        printf("%-34s median %.3f ms  %6.0f TF/s", names[m], ms, nmf * 32768 * 1024 / ms / 1e9);
        if (mhz > 0) printf("  %5.1f cycles/MFMA at %.0f MHz", ms * 1e-3 * mhz * 1e6 / nmf, mhz);
        printf("\n");
    }
    return 0;
}
