// Diagnostic: the split block kernels' GEMM-1 loop (weights as register-resident A fragments,
// a 66-row split activation image in LDS as the B operand, 3 products per step, one wave per
// SIMD, 256 workgroups) on v_mfma_f32_32x32x16_f16 vs v_mfma_f32_16x16x32_f16 at the same
// output tile per wave (32 channels x 64 columns) and the same FLOPs; random fp16 data with
// half the activations zero (relu).  Prints ms per launch of each shape (interleaved rounds).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <random>
#include <algorithm>
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
constexpr int RS = 528, ROWS = 66, NTILE = 64;
__device__ __forceinline__ uint4 to_agpr(uint4 v) {
    u32x4 t = __builtin_bit_cast(u32x4, v);
    asm volatile("" : "=a"(t) : "0"(t));
    return __builtin_bit_cast(uint4, t);
}
__device__ __forceinline__ uint4 lds16(const uint8_t* p) { return *reinterpret_cast<const uint4*>(p); }

__global__ void __launch_bounds__(256, 1) k32(const uint4* wsrc, const uint4* img_src, float* out, int ntiles) {
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
#pragma unroll
    for (int tp = 0; tp < 3; ++tp)
#pragma unroll
        for (int kb = 0; kb < 8; ++kb)
#pragma unroll
            for (int hl = 0; hl < 2; ++hl) wd[tp][kb][hl] = to_agpr(wd[tp][kb][hl]);
    __syncthreads();
    float sum = 0.f;
    for (int t = 0; t < ntiles; ++t) {
#pragma unroll
        for (int J = 0; J < 2; ++J) {
            f32x16 acc;
#pragma unroll
            for (int i = 0; i < 16; ++i) acc[i] = 0.f;
            const int Lc = 32 * J + r + 1;
            uint4 bh[3], bl[3];
            auto bread = [&](int st, uint4& xh, uint4& xl) {
                const uint8_t* p = IMG + (Lc + (st >> 3) - 1) * RS + (st & 7) * 32 + h * 16;
                xh = lds16(p); xl = lds16(p + 256);
            };
            bread(0, bh[0], bl[0]); bread(1, bh[1], bl[1]);
#pragma unroll
            for (int st = 0; st < 24; ++st) {
                const int tp = st >> 3, kb = st & 7, cb = st % 3;
                acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8, wd[tp][kb][0]), __builtin_bit_cast(f16x8, bh[cb]), acc, 0, 0, 0);
                if (st + 2 < 24) bread(st + 2, bh[(st + 2) % 3], bl[(st + 2) % 3]);
                acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8, wd[tp][kb][1]), __builtin_bit_cast(f16x8, bh[cb]), acc, 0, 0, 0);
                acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8, wd[tp][kb][0]), __builtin_bit_cast(f16x8, bl[cb]), acc, 0, 0, 0);
            }
#pragma unroll
            for (int i = 0; i < 16; ++i) sum += acc[i];
        }
    }
    out[blockIdx.x * 256 + tid] = sum;
}

// 16x16x32: wave's 32 channels = 2 M-tiles, 64 columns = 4 N-tiles; per K32 step and N-tile
// the B fragment (lane (n, q): rows column 16 N + n, channels 32 ks + 8 q .. + 8)
__global__ void __launch_bounds__(256, 1) k16(const uint4* wsrc, const uint4* img_src, float* out, int ntiles) {
    __shared__ __attribute__((aligned(16))) uint8_t IMG[ROWS * RS];
    const int tid = threadIdx.x, lane = tid & 63, n = lane & 15, q = lane >> 4;
    for (int i = tid; i < ROWS * RS / 16; i += 256) reinterpret_cast<uint4*>(IMG)[i] = img_src[i];
    uint4 wd[2][12][2];   // [m][tap * 4 + ks][hl]
#pragma unroll
    for (int m = 0; m < 2; ++m)
#pragma unroll
        for (int s = 0; s < 12; ++s)
#pragma unroll
            for (int hl = 0; hl < 2; ++hl) wd[m][s][hl] = wsrc[((m * 12 + s) * 2 + hl) * 64 + lane];
#pragma unroll
    for (int m = 0; m < 2; ++m)
#pragma unroll
        for (int s = 0; s < 12; ++s)
#pragma unroll
            for (int hl = 0; hl < 2; ++hl) wd[m][s][hl] = to_agpr(wd[m][s][hl]);
    __syncthreads();
    float sum = 0.f;
    for (int t = 0; t < ntiles; ++t) {
#pragma unroll
        for (int J = 0; J < 2; ++J) {
            f32x4 acc[2][2];
#pragma unroll
            for (int m = 0; m < 2; ++m)
#pragma unroll
                for (int N = 0; N < 2; ++N) acc[m][N] = f32x4{0.f, 0.f, 0.f, 0.f};
            uint4 bh[3][2], bl[3][2];
            auto bread = [&](int st, int slot) {
                const int tp = st >> 2, ks = st & 3;
#pragma unroll
                for (int N = 0; N < 2; ++N) {
                    const uint8_t* p = IMG + (32 * J + 16 * N + n + 1 + tp - 1) * RS + ks * 64 + q * 16;
                    bh[slot][N] = lds16(p); bl[slot][N] = lds16(p + 256);
                }
            };
            bread(0, 0); bread(1, 1);
#pragma unroll
            for (int st = 0; st < 12; ++st) {
                const int cb = st % 3;
                if (st + 2 < 12) bread(st + 2, (st + 2) % 3);
#pragma unroll
                for (int N = 0; N < 2; ++N)
#pragma unroll
                    for (int m = 0; m < 2; ++m) {
                        acc[m][N] = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, wd[m][st][0]), __builtin_bit_cast(f16x8, bh[cb][N]), acc[m][N], 0, 0, 0);
                        acc[m][N] = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, wd[m][st][1]), __builtin_bit_cast(f16x8, bh[cb][N]), acc[m][N], 0, 0, 0);
                        acc[m][N] = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, wd[m][st][0]), __builtin_bit_cast(f16x8, bl[cb][N]), acc[m][N], 0, 0, 0);
                    }
            }
#pragma unroll
            for (int m = 0; m < 2; ++m)
#pragma unroll
                for (int N = 0; N < 2; ++N) sum += acc[m][N][0] + acc[m][N][1] + acc[m][N][2] + acc[m][N][3];
        }
    }
    out[blockIdx.x * 256 + tid] = sum;
}

int main() {
    std::mt19937 g(7);
    std::uniform_real_distribution<float> u(-1.f, 1.f);
    std::vector<_Float16> w(64 * 64 * 8), im(ROWS * RS / 2);
    for (auto& x : w) x = (_Float16)u(g);
    for (size_t i = 0; i < im.size(); ++i) { float v = u(g); im[i] = (_Float16)(v > 0 ? v * 1000.f : 0.f); }
    uint4 *dw, *di; float* dout;
    (void)hipMalloc(&dw, w.size() * 2); (void)hipMalloc(&di, im.size() * 2); (void)hipMalloc(&dout, 256 * 256 * 4);
    (void)hipMemcpy(dw, w.data(), w.size() * 2, hipMemcpyHostToDevice);
    (void)hipMemcpy(di, im.data(), im.size() * 2, hipMemcpyHostToDevice);
    hipEvent_t e0, e1; (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
    const int nt = 256;
    std::vector<float> t32, t16;
    for (int round = 0; round < 12; ++round) {
        for (int which = 0; which < 2; ++which) {
            (void)hipEventRecord(e0);
            for (int k = 0; k < 5; ++k) {
                if (which == 0) hipLaunchKernelGGL(k32, dim3(256), dim3(256), 0, 0, dw, di, dout, nt);
                else hipLaunchKernelGGL(k16, dim3(256), dim3(256), 0, 0, dw, di, dout, nt);
            }
            (void)hipEventRecord(e1); (void)hipEventSynchronize(e1);
            float ms; (void)hipEventElapsedTime(&ms, e0, e1);
            if (round >= 2) (which == 0 ? t32 : t16).push_back(ms / 5);
        }
    }
    std::sort(t32.begin(), t32.end()); std::sort(t16.begin(), t16.end());
    // 256 tiles x 2 halves x 72 MFMAs (32x32x16 = 32768 flop) per wave, 1024 waves
    const double fl = 256.0 * 2 * 72 * 32768 * 1024;
    printf("32x32x16: median %.3f ms (%.0f TF/s)  16x16x32: median %.3f ms (%.0f TF/s)  ratio %.3f\n",
           t32[t32.size() / 2], fl / t32[t32.size() / 2] / 1e9, t16[t16.size() / 2], fl / t16[t16.size() / 2] / 1e9,
           t32[t32.size() / 2] / t16[t16.size() / 2]);
    return 0;
}
