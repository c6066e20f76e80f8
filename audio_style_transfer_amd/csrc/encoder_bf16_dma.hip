// bf16 encoder block forward, DMA-staged variant (precision 1; model.py:95-116).
//
// Same algebra as encoder_bf16.hip, re-cut so that TWO workgroups share each CU and overlap
// each other's MFMA phases with their load / epilogue / store phases (the one-workgroup
// persistent kernel serialises them behind its barriers):
//  * 256 threads = one wave per SIMD; wave w owns output channels 32w..32w+31 and every
//    column of a 64-position tile.  All weights live in registers as MFMA A fragments
//    (Wd^T 3 taps x 128 k: 96 VGPRs, Wr^T: 32 VGPRs); LDS holds only activations (~56 KB).
//  * Input rows stream HBM -> LDS with global_load_lds (no VGPR staging), double-buffered:
//    the next tile's rows land while this tile computes.  LDS rows are plain 256-B rows
//    whose 16-B chunks are XOR-swizzled by (row & 15) through the per-lane SOURCE address,
//    which makes the column-wise ds_read_b128 fragment reads conflict-free.  relu is applied
//    to the fragments after the read (v_pk_max_i16), so one image serves GEMM1 (relu(e))
//    and the residual (e).
//  * The barriers are raw s_barrier with an explicit lgkmcnt(0) (a __syncthreads() would
//    drain the in-flight DMA with vmcnt(0)); the DMA is retired once per tile, just before
//    the output stores, so those stores stay in flight across the next barrier.
#include "common.h"
#include <algorithm>

namespace ast {

namespace {

constexpr int P2 = 64;                 // positions per tile
constexpr int NT2 = 256;               // threads per workgroup
constexpr int NR2 = P2 + 4;            // LDS rows max (2 segments of 32 + 2 pads each)
constexpr int RB2 = 256;               // LDS row bytes (unpadded: DMA writes are lane-linear)

struct Layout2 {
    int M;       // segment length: P2 (one segment + 2 halo rows) or 32 (two padded segments)
    int nrows;   // LDS rows of a tile
};

__device__ __forceinline__ void lds_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}

__device__ __forceinline__ uint4 relu8b(uint4 v) {
    return make_uint4(relu2(v.x), relu2(v.y), relu2(v.z), relu2(v.w));
}

__device__ __forceinline__ uint32_t sign_byte(uint4 v) {
    const uint32_t d[4] = {v.x, v.y, v.z, v.w};
    uint32_t bits = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        bits |= ((short)(d[j] & 0xffffu) > 0 ? 1u : 0u) << (2 * j);
        bits |= ((short)(d[j] >> 16) > 0 ? 1u : 0u) << (2 * j + 1);
    }
    return bits;
}

// byte offset of logical 16-B chunk q of LDS row L
__device__ __forceinline__ uint32_t xoff(int L, int q) {
    return (uint32_t)(L * RB2 + ((q ^ (L & 15)) << 4));
}

__device__ __forceinline__ int acc_row2(int i, int h) { return (i & 3) + 8 * (i >> 2) + 4 * h; }

// time of LDS row L of the tile starting at position p0, or -1 (zero row)
template <bool MASKED>
__device__ __forceinline__ int row_time2(int L, int p0, const Layout2& ly, int T, int n, int d) {
    if (ly.M == P2) {
        const int p = p0 - 1 + L;
        if (p < 0 || p >= T) return -1;
        if (!MASKED) {   // halos belong to the tile's own sub-sequence only
            if (L == 0 && p0 % n == 0) return -1;
            if (L == P2 + 1 && (p0 + P2) % n == 0) return -1;
        }
        return (p % n) * d + p / n;
    }
    const int s = L / (ly.M + 2), k = L - s * (ly.M + 2);
    if (k == 0 || k == ly.M + 1) return -1;
    const int p = p0 + s * ly.M + k - 1;
    return (p % n) * d + p / n;
}

__device__ __forceinline__ int rowmap2(int c, const Layout2& ly) {
    return (c / ly.M) * (ly.M + 2) + 1 + (c % ly.M);
}

template <bool MASKED>
__global__ void __launch_bounds__(NT2, 2) k_block_fwd_dma(FwdArgsB a, Layout2 ly) {
    __shared__ __attribute__((aligned(1024))) uint8_t XS[2][NR2 * RB2];   // raw e_l rows (swizzled)
    __shared__ __attribute__((aligned(16))) u16 V[P2 * XSB];           // relu(u) by column
    __shared__ __attribute__((aligned(16))) uint32_t MB[P2 * 4];       // u > 0 bits
    __shared__ int TTb[2][NR2];
    __shared__ int RMAP[P2];
    __shared__ __attribute__((aligned(16))) float BIAS[2 * C];        // b_d, b_r
    const int tiles = a.T / P2;
    const int ntiles = a.B * tiles;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int r = lane & 31, h = lane >> 5;
    const int cb = 32 * w;

    uint4 wd[3][8], wr[8];
#pragma unroll
    for (int tp = 0; tp < 3; ++tp)
#pragma unroll
        for (int kb = 0; kb < 8; ++kb)
            wd[tp][kb] = *reinterpret_cast<const uint4*>(a.wdT + (size_t)tp * C * C + (size_t)(cb + r) * C + 16 * kb + 8 * h);
#pragma unroll
    for (int kb = 0; kb < 8; ++kb)
        wr[kb] = *reinterpret_cast<const uint4*>(a.wrT + (size_t)(cb + r) * C + 16 * kb + 8 * h);
    if (tid < C) { BIAS[tid] = a.bd[tid]; BIAS[C + tid] = a.br[tid]; }
    if (tid < P2) RMAP[tid] = rowmap2(tid, ly);

    // stage the rows of `tile` into buffer nb: DMA for live rows, zeros for pad / edge rows
    auto stage = [&](int tile, int nb) {
        tile = tile < ntiles ? tile : ntiles - 1;
        const int b = tile / tiles, p0 = (tile - b * tiles) * P2;
        const u16* src = a.ein + (size_t)b * a.T * C;
        const int p = lane & 15;
#pragma unroll
        for (int gi = 0; gi < 5; ++gi) {
            const int g = w + 4 * gi;           // 4-row group (one 1-KiB DMA instruction)
            if (4 * g >= ly.nrows) break;
            const int L = 4 * g + (lane >> 4);
            const int t = L < ly.nrows ? row_time2<MASKED>(L, p0, ly, a.T, a.n, a.d) : -1;
            if (p == 0) TTb[nb][L] = t;
            if (t >= 0)
                __builtin_amdgcn_global_load_lds(src + (uint32_t)(t * C + ((p ^ (L & 15)) << 3)),
                                                 (__attribute__((address_space(3))) void*)&XS[nb][g * 4 * RB2],
                                                 16, 0, 0);
            else
                *reinterpret_cast<uint4*>(&XS[nb][L * RB2 + p * 16]) = make_uint4(0, 0, 0, 0);
        }
    };

    stage(blockIdx.x, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    int it = 0;
    for (int tile = blockIdx.x; tile < ntiles; tile += gridDim.x, ++it) {
        const int cur = it & 1;
        const int b = tile / tiles;
        const int p0 = (tile - b * tiles) * P2;
        const uint8_t* X = XS[cur];
        const int* TT = TTb[cur];
        // (B) this tile's rows landed (each wave waited for its own DMA), previous tile done
        lds_barrier();
        stage(tile + gridDim.x, cur ^ 1);                  // in flight during this tile

        int Lc[2];
        bool ok0[2], ok2[2];
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const int c = 32 * j + r;
            Lc[j] = RMAP[c];
            ok0[j] = ok2[j] = true;
            if (MASKED) {
                const int m = (p0 + c) % a.n;
                ok0[j] = m > 0;
                ok2[j] = m < a.n - 1;
            }
        }
        // GEMM 1: u^T[co][c] = sum_{tap, ci} Wd[tap][ci][co] relu(e)[c + tap - 1][ci]
        f32x16 acc[2];
#pragma unroll
        for (int j = 0; j < 2; ++j)
            for (int i = 0; i < 16; ++i) acc[j][i] = 0.f;
        {
            uint32_t rb[2][3], rx[2][3];
#pragma unroll
            for (int j = 0; j < 2; ++j)
#pragma unroll
                for (int tp = 0; tp < 3; ++tp) {
                    const int L = Lc[j] - 1 + tp;
                    rb[j][tp] = (uint32_t)(L * RB2);
                    rx[j][tp] = (uint32_t)(L & 15);
                }
            auto frag = [&](int j, int tp, int kb) {
                const uint32_t o = rb[j][tp] + ((((uint32_t)(2 * kb + h)) ^ rx[j][tp]) << 4);
                return relu8b(*reinterpret_cast<const uint4*>(X + o));
            };
            uint4 bcur[2], bnxt[2];
#pragma unroll
            for (int j = 0; j < 2; ++j) bcur[j] = frag(j, 0, 0);
#pragma unroll
            for (int st = 0; st < 24; ++st) {
                const int tp = st >> 3, kb = st & 7;
                if (st + 1 < 24) {
#pragma unroll
                    for (int j = 0; j < 2; ++j) bnxt[j] = frag(j, (st + 1) >> 3, (st + 1) & 7);
                }
#pragma unroll
                for (int j = 0; j < 2; ++j) {
                    uint4 bv = bcur[j];
                    if (MASKED) {
                        const bool ok = tp == 0 ? ok0[j] : (tp == 2 ? ok2[j] : true);
                        if (!ok) bv = make_uint4(0, 0, 0, 0);
                    }
                    acc[j] = mfma_bf16(wd[tp][kb], bv, acc[j]);
                }
#pragma unroll
                for (int j = 0; j < 2; ++j) bcur[j] = bnxt[j];
            }
        }
        // epilogue 1: + b_d (masked.py:155), relu (model.py:107) -> V; u > 0 bits -> MB
        float bd[16];
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            const float4 v4 = *reinterpret_cast<const float4*>(&BIAS[cb + 8 * g + 4 * h]);
            bd[4 * g] = v4.x; bd[4 * g + 1] = v4.y; bd[4 * g + 2] = v4.z; bd[4 * g + 3] = v4.w;
        }
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const int c = 32 * j + r;
            uint32_t part = 0;
            float v[16];
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                const float u = acc[j][i] + bd[i];
                part |= (u > 0.f ? 1u : 0u) << acc_row2(i, h);
                v[i] = fmaxf(u, 0.f);
            }
            const uint32_t word = part | (uint32_t)__shfl_xor((int)part, 32);
            if (h == 0) MB[c * 4 + w] = word;
#pragma unroll
            for (int g = 0; g < 4; ++g)
                *reinterpret_cast<uint2*>(&V[c * XSB + cb + 8 * g + 4 * h]) =
                    make_uint2(pack2(v[4 * g], v[4 * g + 1]), pack2(v[4 * g + 2], v[4 * g + 3]));
        }
        // e_l > 0 bits (one byte = 8 channels per piece) before X is updated in place
        const size_t mbase = (size_t)b * a.T * 4;
        uint8_t* meb = reinterpret_cast<uint8_t*>(a.me + mbase);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int i = tid + NT2 * k, cc = i >> 4, q = i & 15;
            const int L = RMAP[cc];
            const uint4 v = *reinterpret_cast<const uint4*>(X + xoff(L, q));
            meb[(uint32_t)((p0 + cc) * 16 + q)] = (uint8_t)sign_byte(v);
        }
        lds_barrier();                                      // (C) V, MB complete
        a.mu[mbase + (uint32_t)((p0 + (tid >> 2)) * 4 + (tid & 3))] = MB[tid];
        // GEMM 2: y^T[co2][c] = sum_co Wr[co][co2] v[c][co]   (model.py:109-114)
#pragma unroll
        for (int j = 0; j < 2; ++j)
            for (int i = 0; i < 16; ++i) acc[j][i] = 0.f;
        {
            uint4 bcur[2], bnxt[2];
#pragma unroll
            for (int j = 0; j < 2; ++j)
                bcur[j] = *reinterpret_cast<const uint4*>(&V[(32 * j + r) * XSB + 8 * h]);
#pragma unroll
            for (int kb = 0; kb < 8; ++kb) {
                if (kb + 1 < 8) {
#pragma unroll
                    for (int j = 0; j < 2; ++j)
                        bnxt[j] = *reinterpret_cast<const uint4*>(&V[(32 * j + r) * XSB + 16 * (kb + 1) + 8 * h]);
                }
#pragma unroll
                for (int j = 0; j < 2; ++j) acc[j] = mfma_bf16(wr[kb], bcur[j], acc[j]);
#pragma unroll
                for (int j = 0; j < 2; ++j) bcur[j] = bnxt[j];
            }
        }
        // epilogue 2: e_{l+1} = e_l + (y + b_r), this wave's channels of X in place
        uint8_t* Xw = XS[cur];
        float br[16];
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            const float4 v4 = *reinterpret_cast<const float4*>(&BIAS[C + cb + 8 * g + 4 * h]);
            br[4 * g] = v4.x; br[4 * g + 1] = v4.y; br[4 * g + 2] = v4.z; br[4 * g + 3] = v4.w;
        }
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const int L = Lc[j];
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                uint2* px = reinterpret_cast<uint2*>(Xw + xoff(L, (cb >> 3) + g) + 8 * h);
                const uint2 ev = *px;
                const float o0 = bflo(ev.x) + (acc[j][4 * g + 0] + br[4 * g + 0]);
                const float o1 = bfhi(ev.x) + (acc[j][4 * g + 1] + br[4 * g + 1]);
                const float o2 = bflo(ev.y) + (acc[j][4 * g + 2] + br[4 * g + 2]);
                const float o3 = bfhi(ev.y) + (acc[j][4 * g + 3] + br[4 * g + 3]);
                *px = make_uint2(pack2(o0, o1), pack2(o2, o3));
            }
        }
        lds_barrier();                                      // (D) e_{l+1} rows complete
        // the next tile's DMA (issued at this tile's start) and the mask stores are done by
        // now; retiring them here keeps the wait off the output stores, which stay in flight
        // across the next barrier
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        u16* dst = a.eout + (size_t)b * a.T * C;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int i = tid + NT2 * k, cc = i >> 4, q = i & 15;
            const int L = RMAP[cc];
            *reinterpret_cast<uint4*>(dst + (uint32_t)(TT[L] * C + q * 8)) =
                *reinterpret_cast<const uint4*>(X + xoff(L, q));
        }
    }
}

bool pick_layout2(int n, Layout2& ly) {
    if (n % P2 == 0) { ly.M = P2; ly.nrows = P2 + 2; return false; }
    if (n == 32) { ly.M = 32; ly.nrows = 2 * 34; return false; }
    ly.M = P2; ly.nrows = P2 + 2;
    return true;
}

int g_cus2 = 0;

}  // namespace

void launch_block_fwd_dma(const FwdArgsB& a, hipStream_t s) {
    if (!g_cus2) {
        int dev = 0;
        (void)hipGetDevice(&dev);
        (void)hipDeviceGetAttribute(&g_cus2, hipDeviceAttributeMultiprocessorCount, dev);
        if (g_cus2 <= 0) g_cus2 = 256;
    }
    const int nt = a.B * (a.T / P2);
    const dim3 grid(std::min(nt, 2 * g_cus2));
    Layout2 ly;
    if (pick_layout2(a.n, ly)) hipLaunchKernelGGL(k_block_fwd_dma<true>, grid, dim3(NT2), 0, s, a, ly);
    else hipLaunchKernelGGL(k_block_fwd_dma<false>, grid, dim3(NT2), 0, s, a, ly);
}

}  // namespace ast
