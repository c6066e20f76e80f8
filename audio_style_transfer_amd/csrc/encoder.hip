// NSynth WaveNet encoder (model.py:80-127) forward and backward-to-input on gfx950.
//
// One fused kernel per residual block and direction:
//   fwd  e_{l+1} = e_l + Wr^T relu(b_d + sum_k Wd[k]^T relu(e_l)[p+k-1]) + b_r
//        (model.py:99-114; masked.py:110-160 with causal=False -> symmetric taps)
//   bwd  g_l = tot + [e_l>0] * sum_k Wd[k] ([u>0] * (Wr tot))[p-k+1],  tot = g_{l+1} + D_{l+1}
// A workgroup owns TM positions of one clip in time_to_batch order (common.h), stages the
// TM+2 input rows in LDS once, and runs both GEMMs (K = 3*128 then 128) on
// v_mfma_f32_32x32x2_f32 with fp32 accumulation; the bias/relu/residual/mask epilogues are
// fused and the relu masks leave as bits (16 B per row) for the backward.
#include <algorithm>
#include "common.h"

namespace ast {

__device__ __forceinline__ f32x16 mfma32(float a, float b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}

// acc[nt] += A[k] * B[k][colb + 32 nt] for k in [0,128): A from an LDS row (this lane's
// M-row), B (row-major [k][C]) from global/L2.  Lane half h feeds k = 4ps + 2h (+1).
template <bool RELU>
__device__ __forceinline__ void mm_k128(f32x16 (&acc)[2], const float* __restrict__ arow,
                                        bool valid, const float* __restrict__ Bm, int colb,
                                        int h) {
#pragma unroll 8
    for (int ps = 0; ps < 32; ++ps) {
        const int k0 = 4 * ps + 2 * h;
        const float2 av = *reinterpret_cast<const float2*>(arow + k0);
        float a0 = av.x, a1 = av.y;
        if (RELU) { a0 = fmaxf(a0, 0.f); a1 = fmaxf(a1, 0.f); }
        a0 = valid ? a0 : 0.f;
        a1 = valid ? a1 : 0.f;
        const float* b0 = Bm + (size_t)k0 * C + colb;
        const float b00 = b0[0], b01 = b0[32], b10 = b0[C], b11 = b0[C + 32];
        acc[0] = mfma32(a0, b00, acc[0]);
        acc[1] = mfma32(a0, b01, acc[1]);
        acc[0] = mfma32(a1, b10, acc[0]);
        acc[1] = mfma32(a1, b11, acc[1]);
    }
}

__device__ __forceinline__ int pos_to_t(int p, int n, int d) { return (p % n) * d + p / n; }

__global__ void __launch_bounds__(256) k_block_fwd(FwdArgs a) {
    __shared__ __attribute__((aligned(16))) float X[(TM + 2) * XS];
    __shared__ __attribute__((aligned(16))) float V[TM * XS];
    __shared__ __attribute__((aligned(16))) uint32_t MB[TM * 4];
    __shared__ int TT[TM + 2];
    const int tiles = a.T / TM;
    const int b = blockIdx.x / tiles;
    const int p0 = (blockIdx.x - b * tiles) * TM;
    const size_t cb = (size_t)b * a.T * C;
    const size_t mbase = (size_t)b * a.T * 4;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;

    if (tid < TM + 2) {
        const int p = p0 - 1 + tid;
        TT[tid] = (p >= 0 && p < a.T) ? pos_to_t(p, a.n, a.d) : -1;
    }
    __syncthreads();
    for (int i = tid; i < (TM + 2) * 32; i += 256) {
        const int rr = i >> 5, q = i & 31;
        const int t = TT[rr];
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
        if (t >= 0) v = *reinterpret_cast<const float4*>(a.ein + cb + (size_t)t * C + q * 4);
        float2* dst = reinterpret_cast<float2*>(&X[rr * XS + q * 4]);
        dst[0] = make_float2(v.x, v.y);
        dst[1] = make_float2(v.z, v.w);
    }
    __syncthreads();

    // e_l > 0 bits of the tile rows (consumed by the backward's relu(e_l) mask)
    for (int rr = w; rr < TM; rr += 4) {
        const float v0 = X[(rr + 1) * XS + lane], v1 = X[(rr + 1) * XS + 64 + lane];
        const unsigned long long q0 = __ballot(v0 > 0.f), q1 = __ballot(v1 > 0.f);
        if (lane == 0)
            *reinterpret_cast<uint4*>(a.me + mbase + (size_t)TT[rr + 1] * 4) =
                make_uint4((uint32_t)q0, (uint32_t)(q0 >> 32), (uint32_t)q1, (uint32_t)(q1 >> 32));
    }

    const int wm = w & 1, wn = w >> 1, r = lane & 31, h = lane >> 5;
    const int row = wm * 32 + r;
    const int m = (p0 + row) % a.n;
    const bool ok0 = m > 0, ok2 = m < a.n - 1;
    const int colb = wn * 64 + r;

    // GEMM 1: dilated conv, K = 3 taps x 128 (masked.py:154)
    f32x16 acc[2];
    for (int i = 0; i < 16; ++i) { acc[0][i] = 0.f; acc[1][i] = 0.f; }
    mm_k128<true>(acc, &X[(row + 0) * XS], ok0, a.wd + 0 * C * C, colb, h);
    mm_k128<true>(acc, &X[(row + 1) * XS], true, a.wd + 1 * C * C, colb, h);
    mm_k128<true>(acc, &X[(row + 2) * XS], ok2, a.wd + 2 * C * C, colb, h);

    {   // epilogue 1: bias (masked.py:155), relu (model.py:107), mask bits
        const float bd0 = a.bd[colb], bd1 = a.bd[colb + 32];
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            const int R0 = wm * 32 + (i & 3) + 8 * (i >> 2);
            const int R = R0 + 4 * h;
            const float u0 = acc[0][i] + bd0, u1 = acc[1][i] + bd1;
            const unsigned long long q0 = __ballot(u0 > 0.f), q1 = __ballot(u1 > 0.f);
            V[R * XS + colb] = fmaxf(u0, 0.f);
            V[R * XS + colb + 32] = fmaxf(u1, 0.f);
            if (lane == 0) {
                MB[R0 * 4 + wn * 2 + 0] = (uint32_t)q0;
                MB[R0 * 4 + wn * 2 + 1] = (uint32_t)q1;
                MB[(R0 + 4) * 4 + wn * 2 + 0] = (uint32_t)(q0 >> 32);
                MB[(R0 + 4) * 4 + wn * 2 + 1] = (uint32_t)(q1 >> 32);
            }
        }
    }
    __syncthreads();
    if (tid < TM)
        *reinterpret_cast<uint4*>(a.mu + mbase + (size_t)TT[tid + 1] * 4) =
            *reinterpret_cast<const uint4*>(&MB[tid * 4]);

    // GEMM 2: 1x1 residual projection (model.py:109-114)
    for (int i = 0; i < 16; ++i) { acc[0][i] = 0.f; acc[1][i] = 0.f; }
    mm_k128<false>(acc, &V[row * XS], true, a.wr, colb, h);
    const float br0 = a.br[colb], br1 = a.br[colb + 32];
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        const int R = wm * 32 + (i & 3) + 8 * (i >> 2) + 4 * h;
        const size_t o = cb + (size_t)TT[R + 1] * C + colb;
        a.eout[o] = X[(R + 1) * XS + colb] + (acc[0][i] + br0);
        a.eout[o + 32] = X[(R + 1) * XS + colb + 32] + (acc[1][i] + br1);
    }
}

__device__ __forceinline__ float bitf(uint32_t word, int bit) {
    return ((word >> bit) & 1u) ? 1.f : 0.f;
}

__global__ void __launch_bounds__(256) k_block_bwd(BwdArgs a) {
    __shared__ __attribute__((aligned(16))) float G[(TM + 2) * XS];
    __shared__ __attribute__((aligned(16))) float U[(TM + 2) * XS];
    __shared__ __attribute__((aligned(16))) uint32_t MU[(TM + 2) * 4];
    __shared__ __attribute__((aligned(16))) uint32_t ME[TM * 4];
    __shared__ int TT[TM + 2];
    const int tiles = a.T / TM;
    const int b = blockIdx.x / tiles;
    const int p0 = (blockIdx.x - b * tiles) * TM;
    const size_t cb = (size_t)b * a.T * C;
    const size_t mbase = (size_t)b * a.T * 4;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;

    if (tid < TM + 2) {
        const int p = p0 - 1 + tid;
        TT[tid] = (p >= 0 && p < a.T) ? pos_to_t(p, a.n, a.d) : -1;
    }
    __syncthreads();
    for (int i = tid; i < (TM + 2) * 32; i += 256) {
        const int rr = i >> 5, q = i & 31;
        const int t = TT[rr];
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
        if (t >= 0) {
            const size_t o = cb + (size_t)t * C + q * 4;
            if (a.gin) v = *reinterpret_cast<const float4*>(a.gin + o);
            if (a.din) {
                const float4 d4 = *reinterpret_cast<const float4*>(a.din + o);
                v.x += d4.x; v.y += d4.y; v.z += d4.z; v.w += d4.w;
            }
        }
        float2* dst = reinterpret_cast<float2*>(&G[rr * XS + q * 4]);
        dst[0] = make_float2(v.x, v.y);
        dst[1] = make_float2(v.z, v.w);
    }
    if (tid < TM + 2) {
        const int t = TT[tid];
        uint4 mw = make_uint4(0, 0, 0, 0);
        if (t >= 0) mw = *reinterpret_cast<const uint4*>(a.mu + mbase + (size_t)t * 4);
        *reinterpret_cast<uint4*>(&MU[tid * 4]) = mw;
        if (tid < TM)
            *reinterpret_cast<uint4*>(&ME[tid * 4]) =
                *reinterpret_cast<const uint4*>(a.me + mbase + (size_t)TT[tid + 1] * 4);
    }
    __syncthreads();

    const int wm = w & 1, wn = w >> 1, r = lane & 31, h = lane >> 5;
    const int row = wm * 32 + r;
    const int m = (p0 + row) % a.n;
    const bool ok0 = m > 0, ok2 = m < a.n - 1;
    const int colb = wn * 64 + r;

    // step 1: g_u = [u>0] * (Wr tot) for the tile rows (MFMA) ...
    f32x16 acc[2];
    for (int i = 0; i < 16; ++i) { acc[0][i] = 0.f; acc[1][i] = 0.f; }
    mm_k128<false>(acc, &G[(row + 1) * XS], true, a.wrT, colb, h);
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        const int R = wm * 32 + (i & 3) + 8 * (i >> 2) + 4 * h;
        U[(R + 1) * XS + colb] = acc[0][i] * bitf(MU[(R + 1) * 4 + wn * 2 + 0], r);
        U[(R + 1) * XS + colb + 32] = acc[1][i] * bitf(MU[(R + 1) * 4 + wn * 2 + 1], r);
    }
    // ... and for the two halo rows (VALU; they feed the neighbour taps only)
    {
        const int hr = tid >> 7, i = tid & 127;
        const int rr = hr ? TM + 1 : 0;
        float s = 0.f;
        if (TT[rr] >= 0) {
            const float* wrow = a.wr + (size_t)i * C;
            const float* grow = &G[rr * XS];
#pragma unroll 8
            for (int o = 0; o < C; ++o) s = fmaf(grow[o], wrow[o], s);
            s *= bitf(MU[rr * 4 + (i >> 5)], i & 31);
        }
        U[rr * XS + i] = s;
    }
    __syncthreads();

    // step 2: gh = sum_k Wd[k] g_u[p-k+1]  (transposed dilated conv)
    for (int i = 0; i < 16; ++i) { acc[0][i] = 0.f; acc[1][i] = 0.f; }
    mm_k128<false>(acc, &U[(row + 2) * XS], ok2, a.wdT + 0 * C * C, colb, h);
    mm_k128<false>(acc, &U[(row + 1) * XS], true, a.wdT + 1 * C * C, colb, h);
    mm_k128<false>(acc, &U[(row + 0) * XS], ok0, a.wdT + 2 * C * C, colb, h);
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        const int R = wm * 32 + (i & 3) + 8 * (i >> 2) + 4 * h;
        const size_t o = cb + (size_t)TT[R + 1] * C + colb;
        a.gout[o] = G[(R + 1) * XS + colb] + bitf(ME[R * 4 + wn * 2 + 0], r) * acc[0][i];
        a.gout[o + 32] = G[(R + 1) * XS + colb + 32] + bitf(ME[R * 4 + wn * 2 + 1], r) * acc[1][i];
    }
}

// ae_startconv (model.py:88-93): 1 -> 128 channels, K=3, d=1, input x/128 (model.py:82).
// Thread per (row, 8 channels): 16-B bf16 (32-B fp32) stores, 16 lanes per row.
constexpr int SFR = 256;   // rows per workgroup
__device__ __forceinline__ float wave_max_f(float v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v = fmaxf(v, __shfl_xor(v, off));
    return v;
}
template <typename S>
__global__ void __launch_bounds__(256) k_startconv_fwd(const float* __restrict__ x,
                                                       S* __restrict__ e0,
                                                       const float* __restrict__ w0,
                                                       const float* __restrict__ b0, int B,
                                                       int T, uint16_t* __restrict__ me0,
                                                       unsigned* __restrict__ gmax) {
    // SFR rows per workgroup, 16 lanes per row; this lane's 8 channels' weights load once
    const int m = threadIdx.x & 15;
    float wk[3][8], bk[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        wk[0][j] = w0[m * 8 + j]; wk[1][j] = w0[C + m * 8 + j]; wk[2][j] = w0[2 * C + m * 8 + j];
        bk[j] = b0[m * 8 + j];
    }
    float amax = 0.f;
    // clip-interleaved block order (block i: clip i mod B, row chunk i / B): concurrently running
    // workgroups belong to different clips, so their max atomics do not pile onto one word
    const int nper = T / SFR;
    const size_t lb = (size_t)(blockIdx.x % B) * nper + blockIdx.x / B;
    // the workgroup's SFR samples and their two neighbours, one coalesced load (zero past the clip)
    __shared__ float xs[SFR + 2];
    {
        const int t0 = (int)((lb * SFR) % T);
        const float* xc = x + (lb * SFR - t0);   // the clip's first sample
        for (int i = threadIdx.x; i < SFR + 2; i += 256) {
            const int t = t0 - 1 + i;
            xs[i] = t >= 0 && t < T ? xc[t] : 0.f;
        }
    }
    __syncthreads();
    for (int it = 0; it < SFR / 16; ++it) {
        const int r = it * 16 + (threadIdx.x >> 4);   // row within the workgroup's SFR
        const size_t rowi = lb * SFR + r;
        const float xm = xs[r], x0 = xs[r + 1], xp = xs[r + 2];
        float o[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] = e0_val(wk[0][j], wk[1][j], wk[2][j], bk[j], xm, x0, xp);
        // element j > 0 (the stored value: fp32, or its bf16 rounding)
        bool pos[8];
        if constexpr (sizeof(S) == 4) {
            if (e0) {   // (null: split mode, block 0 recomputes e_0 from x; masks and max only)
                float4* dst = reinterpret_cast<float4*>(e0 + rowi * C + m * 8);
                dst[0] = make_float4(o[0], o[1], o[2], o[3]);
                dst[1] = make_float4(o[4], o[5], o[6], o[7]);
            }
#pragma unroll
            for (int j = 0; j < 8; ++j) pos[j] = o[j] > 0.f;
        } else {
            uint32_t p[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) p[k] = pack2(o[2 * k], o[2 * k + 1]);
            *reinterpret_cast<uint4*>(e0 + rowi * C + m * 8) = make_uint4(p[0], p[1], p[2], p[3]);
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                pos[2 * k] = (short)(p[k] & 0xffffu) > 0;
                pos[2 * k + 1] = (int)p[k] >= 0x10000;
            }
        }
        if (gmax) {
#pragma unroll
            for (int j = 0; j < 8; ++j) amax = fmaxf(amax, fabsf(o[j]));
        }
        if (me0) {
            // e_0 > 0 bits for block 0's backward (dilation 1: position = time) in the MFMA
            // accumulator layout (common.h): channel 32 Q + 8 g + 4 h + j is element
            // i = 4 g + j of word (h, Q), at bit mbit(i); this lane holds Q = m / 4, g = m % 4,
            // h = 0 (elements 0..3) and h = 1 (elements 4..7)
            const int g = m & 3;
            uint32_t wd[2];
#pragma unroll
            for (int hh = 0; hh < 2; ++hh) {
                wd[hh] = 0;
#pragma unroll
                for (int j = 0; j < 4; ++j) wd[hh] |= (pos[4 * hh + j] ? 1u : 0u) << mbit(4 * g + j);
                wd[hh] |= (uint32_t)__shfl_xor((int)wd[hh], 1);
                wd[hh] |= (uint32_t)__shfl_xor((int)wd[hh], 2);
                // words (hh, Q) and (hh, Q ^ 1) in one dword (even Q low)
                const uint32_t other = (uint32_t)__shfl_xor((int)wd[hh], 4);
                wd[hh] = (m & 4) ? (other | (wd[hh] << 16)) : (wd[hh] | (other << 16));
            }
            // dwords [h0: Q0|Q1, Q2|Q3, h1: Q0|Q1, Q2|Q3]: lane m = 0 holds Q0|Q1, lane 8 Q2|Q3
            const uint32_t f0 = (uint32_t)__shfl_xor((int)wd[0], 8);
            const uint32_t f1 = (uint32_t)__shfl_xor((int)wd[1], 8);
            if (m == 0)
                *reinterpret_cast<uint4*>(me0 + rowi * 8) = make_uint4(wd[0], f0, wd[1], f1);
        }
    }
    if (gmax) {
        // max |e_0| of the workgroup's rows (one clip: T is a multiple of SFR) -> the clip's max
        amax = wave_max_f(amax);
        if ((threadIdx.x & 63) == 0)
            atomicMax(gmax + blockIdx.x % B, __float_as_uint(amax));
    }
}

// Split mode's start conv (block 0 recomputes e_0 from x, FwdArgsS::xin): only the e_0 > 0 mask
// words and the per-clip max |e_0|.  One row per lane, all 128 channels in a loop (W0 / b0 uniform:
// scalar loads), the row's eight u16 words built in registers and stored as one 16-B piece
// (64 lanes: 1 KiB contiguous) -- the same values as k_startconv_fwd's (e0_val, the same bit
// layout), without its 16-lane-per-row shuffles (0.16 -> ~0.03 ms at 256 x 16384)
__global__ void __launch_bounds__(256) k_startconv_masks(const float* __restrict__ x,
                                                         const float* __restrict__ w0,
                                                         const float* __restrict__ b0, int B, int T,
                                                         uint16_t* __restrict__ me0,
                                                         unsigned* __restrict__ gmax) {
    // clip-interleaved block order (as k_startconv_fwd): concurrent workgroups, different clips
    const int nper = T / SFR;
    const size_t lb = (size_t)(blockIdx.x % B) * nper + blockIdx.x / B;
    const size_t rowi = lb * SFR + threadIdx.x;
    const int t = (int)(rowi % (size_t)T);
    const float* xc = x + (rowi - t);
    const float xm = t > 0 ? xc[t - 1] : 0.f, x0 = xc[t], xp = t + 1 < T ? xc[t + 1] : 0.f;
    // word (h, Q) (u16 index 4 h + Q) holds channel 32 Q + 8 g + 4 h + j at bit mbit(4 g + j) =
    // 4 j + g.  Chunks of 16 channels (a runtime loop: the whole W0 / b0 in scalar registers
    // spilled): chunk k is Q = k / 2, g = 2 (k & 1) + i / 8 for its channel i
    uint64_t P0 = 0, P1 = 0;   // words (0, Q) and (1, Q) at bits 16 Q
    float amax = 0.f;
#pragma unroll 1
    for (int k = 0; k < C / 16; ++k) {
        uint32_t wh0 = 0u, wh1 = 0u;
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            const int c = 16 * k + i;
            const float o = e0_val(w0[c], w0[C + c], w0[2 * C + c], b0[c], xm, x0, xp);
            amax = fmaxf(amax, fabsf(o));
            const uint32_t bit = (o > 0.f ? 1u : 0u) << (4 * (i & 3) + (i >> 3));
            if ((i >> 2) & 1) wh1 |= bit; else wh0 |= bit;
        }
        const int sh = 16 * (k >> 1) + 2 * (k & 1);
        P0 |= (uint64_t)wh0 << sh;
        P1 |= (uint64_t)wh1 << sh;
    }
    *reinterpret_cast<uint4*>(me0 + rowi * 8) =
        make_uint4((uint32_t)P0, (uint32_t)(P0 >> 32), (uint32_t)P1, (uint32_t)(P1 >> 32));
    // the workgroup's max in one atomic (at one clip, 64 workgroups x 4 waves on one line otherwise)
    __shared__ float wmx[4];
    amax = wave_max_f(amax);
    if ((threadIdx.x & 63) == 0) wmx[threadIdx.x >> 6] = amax;
    __syncthreads();
    if (threadIdx.x == 0)
        atomicMax(gslot(gmax, blockIdx.x % B, blockIdx.x), __float_as_uint(fmaxf(fmaxf(wmx[0], wmx[1]), fmaxf(wmx[2], wmx[3]))));
}

// d loss / d x (startconv transposed, model.py:82-93, incl. the 1/128 of model.py:83):
//   gx[t] = (1/128) sum_k a_k[t - k + 1],   a_k[t] = sum_c W0[k][c] g0[t][c].
// One workgroup per SCB rows: the 16-B chunks of a row go to CPR consecutive lanes, which form
// the row's three dot products (shuffle-reduced); each row of g0 is read once, in whole lines.
constexpr int SCB = 256;
template <typename S>
__global__ void __launch_bounds__(256) k_startconv_bwd(const S* __restrict__ g0,
                                                       float* __restrict__ gx,
                                                       const float* __restrict__ w0, int B,
                                                       int T) {
    constexpr int EPC = 16 / (int)sizeof(S);   // elements per 16-B chunk
    constexpr int CPR = C / EPC;               // chunks (lanes) per row
    constexpr int RPP = 256 / CPR;             // rows per pass
    __shared__ float A[3][SCB + 2];            // a_k of rows t0 - 1 .. t0 + SCB
    const int tiles = T / SCB;
    const int b = blockIdx.x / tiles, t0 = (blockIdx.x - b * tiles) * SCB;
    const int tid = threadIdx.x, ch = tid % CPR;
    float w[3][EPC];
#pragma unroll
    for (int k = 0; k < 3; ++k)
#pragma unroll
        for (int e = 0; e < EPC; ++e) w[k][e] = w0[k * C + ch * EPC + e];
    const S* base = g0 + (size_t)b * T * C + ch * EPC;
    for (int i = tid / CPR; i < SCB + 2; i += RPP) {
        const int t = t0 - 1 + i;
        float s0 = 0.f, s1 = 0.f, s2 = 0.f;
        if (t >= 0 && t < T) {
            const uint4 v = *reinterpret_cast<const uint4*>(base + (size_t)t * C);
            const uint32_t u[4] = {v.x, v.y, v.z, v.w};
            float x[EPC];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                if constexpr (sizeof(S) == 4) {
                    x[k] = __uint_as_float(u[k]);
                } else {
                    x[2 * k] = bflo(u[k]);
                    x[2 * k + 1] = bfhi(u[k]);
                }
            }
#pragma unroll
            for (int e = 0; e < EPC; ++e) {
                s0 = fmaf(w[0][e], x[e], s0);
                s1 = fmaf(w[1][e], x[e], s1);
                s2 = fmaf(w[2][e], x[e], s2);
            }
        }
#pragma unroll
        for (int off = CPR / 2; off > 0; off >>= 1) {
            s0 += __shfl_xor(s0, off);
            s1 += __shfl_xor(s1, off);
            s2 += __shfl_xor(s2, off);
        }
        if (ch == 0) { A[0][i] = s0; A[1][i] = s1; A[2][i] = s2; }
    }
    __syncthreads();
    for (int i = tid; i < SCB; i += 256)   // t = t0 + i is image row i + 1
        gx[(size_t)b * T + t0 + i] = (A[0][i + 2] + A[1][i + 1] + A[2][i]) / 128.0f;
}

// d loss / d x from the split block-0 backward's per-wave dot products (BwdArgsS::spart):
//   a_k[t] = sum_w spart[t][w][k],  gx[t] = (a_0[t + 1] + a_1[t] + a_2[t - 1]) / 128
// (k_startconv_bwd's sums without the 2 GiB g_0 round trip; the wave partials summed in a fixed
// order, so a clip's result does not depend on its batch slot)
__global__ void __launch_bounds__(256) k_startx_gx(const float* __restrict__ sp, float* __restrict__ gx,
                                                   int B, int T) {
    const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= (size_t)B * T) return;
    const int t = (int)(i % T);
    auto ak = [&](int tt, int k) {
        const float4* q = reinterpret_cast<const float4*>(sp + (i - t + tt) * 16);
        const float v[4] = {q[0].x, q[1].x, q[2].x, q[3].x};
        const float u[4] = {q[0].y, q[1].y, q[2].y, q[3].y};
        const float z[4] = {q[0].z, q[1].z, q[2].z, q[3].z};
        const float* a = k == 0 ? v : k == 1 ? u : z;
        return ((a[0] + a[1]) + a[2]) + a[3];
    };
    float g = ak(t, 1);
    if (t + 1 < T) g = ak(t + 1, 0) + g;
    if (t > 0) g = g + ak(t - 1, 2);
    gx[i] = g * 0.0078125f;
}

// ae_bottleneck (model.py:121-127): 1x1, 128 -> 16.  Thread per (row, out channel).
template <typename S>
__global__ void __launch_bounds__(256) k_bottleneck_fwd(const S* __restrict__ e,
                                                        float* __restrict__ y,
                                                        const float* __restrict__ wb,
                                                        const float* __restrict__ bb, int B,
                                                        int T) {
    const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= (size_t)B * T * 16) return;
    const size_t rowi = i >> 4;
    const int j = (int)(i & 15);
    float s = 0.f;
    for (int c = 0; c < C; ++c) s = fmaf(ldv(e, rowi * C + c), wb[c * 16 + j], s);
    y[i] = s + bb[j];
}

// ge[row][c] (+)= sum_j Wb[c][j] gy[row][j]
template <typename S>
__global__ void __launch_bounds__(256) k_bottleneck_bwd(const float* __restrict__ gy,
                                                        S* __restrict__ ge,
                                                        const float* __restrict__ wb,
                                                        int accumulate, int B, int T) {
    const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= (size_t)B * T * C) return;
    const size_t rowi = i >> 7;
    const int c = (int)(i & 127);
    const float* g = gy + rowi * 16;
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < 16; ++j) s = fmaf(wb[c * 16 + j], g[j], s);
    stv(ge, i, accumulate ? ldv(ge, i) + s : s);
}

__global__ void __launch_bounds__(256) k_to_f32(const u16* __restrict__ src, float* __restrict__ dst,
                                                size_t n) {
    const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (i < n) dst[i] = bf2f(src[i]);
}

void launch_block_fwd(const FwdArgs& a, hipStream_t s) {
    hipLaunchKernelGGL(k_block_fwd, dim3(a.B * (a.T / TM)), dim3(256), 0, s, a);
}
void launch_block_bwd(const BwdArgs& a, hipStream_t s) {
    hipLaunchKernelGGL(k_block_bwd, dim3(a.B * (a.T / TM)), dim3(256), 0, s, a);
}
template <typename S>
void launch_startconv_fwd(const float* x, S* e0, const float* w0, const float* b0, int B, int T,
                          hipStream_t s, uint16_t* me0, unsigned* gmax) {
    hipLaunchKernelGGL(k_startconv_fwd<S>, dim3((unsigned)((size_t)B * T / SFR)), dim3(256), 0, s, x,
                       e0, w0, b0, B, T, me0, gmax);
}
void launch_startconv_masks(const float* x, const float* w0, const float* b0, int B, int T,
                            hipStream_t s, uint16_t* me0, unsigned* gmax) {
    hipLaunchKernelGGL(k_startconv_masks, dim3((unsigned)((size_t)B * T / SFR)), dim3(SFR), 0, s, x, w0,
                       b0, B, T, me0, gmax);
}
void launch_startx_gx(const float* spart, float* gx, int B, int T, hipStream_t s) {
    const size_t n = (size_t)B * T;
    hipLaunchKernelGGL(k_startx_gx, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, spart, gx, B, T);
}
template <typename S>
void launch_startconv_bwd(const S* g0, float* gx, const float* w0, int B, int T, hipStream_t s) {
    hipLaunchKernelGGL(k_startconv_bwd<S>, dim3((unsigned)(B * (T / SCB))), dim3(256), 0, s, g0,
                       gx, w0, B, T);
}
template <typename S>
void launch_bottleneck_fwd(const S* e, float* y, const float* wb, const float* bb, int B, int T,
                           hipStream_t s) {
    const size_t n = (size_t)B * T * 16;
    hipLaunchKernelGGL(k_bottleneck_fwd<S>, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, e,
                       y, wb, bb, B, T);
}
template <typename S>
void launch_bottleneck_bwd(const float* gy, S* ge, const float* wb, int accumulate, int B, int T,
                           hipStream_t s) {
    const size_t n = (size_t)B * T * C;
    hipLaunchKernelGGL(k_bottleneck_bwd<S>, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s,
                       gy, ge, wb, accumulate, B, T);
}
// zero fill of n 32-bit words: the per-call clears of the max / partial-sum / flag buffers as
// kernel nodes (a graph replay then orders them like every other node: no memset nodes)
__global__ void __launch_bounds__(256) k_zero32(uint32_t* __restrict__ p, size_t n) {
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) p[i] = 0u;
}
void launch_zero32(void* p, size_t bytes, hipStream_t s, int site) {
    const size_t n = bytes / 4;
    if (!n) return;
#ifdef ASTYLE_MEMSET_CLEARS
    // tools-only build (ASTYLE_VARIANT=memset ASTYLE_DEFS=-DASTYLE_MEMSET_CLEARS): the round-4
    // hipMemsetAsync clears, for tools/determinism2.py (graph replays); env
    // ASTYLE_MEMSET_SITES=<bit mask of sites> keeps the other sites on k_zero32 (default: all)
    static int mask = -1;
    if (mask < 0) { const char* e = getenv("ASTYLE_MEMSET_SITES"); mask = e ? atoi(e) : 0xff; }
    if (site < 0 || ((mask >> site) & 1)) {
        (void)hipMemsetAsync(p, 0, bytes, s);
        return;
    }
#endif
    const unsigned blocks = (unsigned)std::min<size_t>((n + 255) / 256, 1024);
    hipLaunchKernelGGL(k_zero32, dim3(blocks), dim3(256), 0, s, (uint32_t*)p, n);
}
void launch_to_f32(const u16* src, float* dst, size_t n, hipStream_t s) {
    hipLaunchKernelGGL(k_to_f32, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, src, dst, n);
}
template void launch_startconv_fwd<float>(const float*, float*, const float*, const float*, int, int, hipStream_t, uint16_t*, unsigned*);
template void launch_startconv_fwd<u16>(const float*, u16*, const float*, const float*, int, int, hipStream_t, uint16_t*, unsigned*);
template void launch_startconv_bwd<float>(const float*, float*, const float*, int, int, hipStream_t);
template void launch_startconv_bwd<u16>(const u16*, float*, const float*, int, int, hipStream_t);
template void launch_bottleneck_fwd<float>(const float*, float*, const float*, const float*, int, int, hipStream_t);
template void launch_bottleneck_fwd<u16>(const u16*, float*, const float*, const float*, int, int, hipStream_t);
template void launch_bottleneck_bwd<float>(const float*, float*, const float*, int, int, int, hipStream_t);
template void launch_bottleneck_bwd<u16>(const float*, u16*, const float*, int, int, int, hipStream_t);

}  // namespace ast
