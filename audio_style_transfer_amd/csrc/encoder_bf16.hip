// bf16 encoder blocks (precision 1): bf16 storage in HBM, v_mfma_f32_32x32x16_bf16 with fp32
// accumulation, fp32 epilogue math, RNE rounding on store.  Same algebra as encoder.hip
// (model.py:95-116 forward, its transpose backward), different mapping:
//   * both GEMMs run transposed — out^T[channel][row] = W^T[channel][k] * act^T[k][row] — so
//     the weights are the A operand (one 16-B global/L2 load per lane per k-block, each
//     weight byte read once per workgroup: wave w owns output channels 32w..32w+31) and the
//     staged activation rows are the B operand (ds_read_b128 from a 272-B-stride LDS image,
//     conflict-free);
//   * a tile is TMB = 128 positions in time_to_batch order (+2 halo rows);
//   * relu of the input is applied on the B fragment with v_pk_max_i16 (bf16 relu == int16
//     max with 0), so the raw rows stay in LDS for the residual;
//   * outputs are written back into the LDS tile and leave as whole 256-B rows.
#include "common.h"
#include <algorithm>

namespace ast {

__device__ __forceinline__ int pos_to_tb(int p, int n, int d) { return (p % n) * d + p / n; }

__device__ __forceinline__ uint4 relu8(uint4 v) {
    return make_uint4(relu2(v.x), relu2(v.y), relu2(v.z), relu2(v.w));
}

// accumulator register i of a 32x32 tile holds row (i&3) + 8(i>>2) + 4h (the channel here)
__device__ __forceinline__ int acc_row(int i, int h) { return (i & 3) + 8 * (i >> 2) + 4 * h; }

// Stage rows p0-1 .. p0+TMB of a clip into an LDS image (16 threads per 256-B row).  With
// ME != nullptr also emit the e>0 bit masks of the TMB centre rows: each thread turns its 8
// channels into 8 bits, 4 lanes OR their bytes into a 32-channel word, lane q=0 stores 16 B.
__device__ __forceinline__ void stage_rows(u16* Xs, const int* TT, const u16* src, size_t cb,
                                           uint32_t* me, size_t mbase, int tid) {
    for (int i = tid; i < (TMB + 2) * 16; i += 256) {
        const int rr = i >> 4, q = i & 15;
        const int t = TT[rr];
        uint4 v = make_uint4(0, 0, 0, 0);
        if (t >= 0) v = *reinterpret_cast<const uint4*>(src + cb + (size_t)t * C + q * 8);
        *reinterpret_cast<uint4*>(&Xs[rr * XSB + q * 8]) = v;
        if (me) {
            const uint32_t d[4] = {v.x, v.y, v.z, v.w};
            uint32_t bits = 0;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                bits |= ((short)(d[k] & 0xffffu) > 0 ? 1u : 0u) << (2 * k);
                bits |= ((short)(d[k] >> 16) > 0 ? 1u : 0u) << (2 * k + 1);
            }
            uint32_t m = bits << (8 * (q & 3));
            m |= (uint32_t)__shfl_xor((int)m, 1);
            m |= (uint32_t)__shfl_xor((int)m, 2);
            const int lane = tid & 63;
            const uint32_t w1 = (uint32_t)__shfl((int)m, lane + 4);
            const uint32_t w2 = (uint32_t)__shfl((int)m, lane + 8);
            const uint32_t w3 = (uint32_t)__shfl((int)m, lane + 12);
            if (q == 0 && rr >= 1 && rr <= TMB)
                *reinterpret_cast<uint4*>(me + mbase + (size_t)t * 4) = make_uint4(m, w1, w2, w3);
        }
    }
}

__device__ __forceinline__ void tile_times(int* TT, int p0, const int T, const int n, const int d,
                                           int tid) {
    if (tid < TMB + 2) {
        const int p = p0 - 1 + tid;
        TT[tid] = (p >= 0 && p < T) ? pos_to_tb(p, n, d) : -1;
    }
}

__device__ __forceinline__ void load_bias16(float (&bias)[16], const float* src, int h) {
#pragma unroll
    for (int g = 0; g < 4; ++g) {
        const float4 b4 = *reinterpret_cast<const float4*>(src + 8 * g + 4 * h);
        bias[4 * g + 0] = b4.x; bias[4 * g + 1] = b4.y; bias[4 * g + 2] = b4.z; bias[4 * g + 3] = b4.w;
    }
}

// Persistent: grid = 2 workgroups per CU; each keeps its wave's 32 output channels of Wd^T
// (3 taps x 128 k) and Wr^T as MFMA A fragments in registers for the whole launch and walks
// tiles blockIdx.x, +gridDim.x, ...
__global__ void __launch_bounds__(256, 2) k_block_fwd_bf16(FwdArgsB a) {
    __shared__ __attribute__((aligned(16))) u16 X[(TMB + 2) * XSB];
    __shared__ __attribute__((aligned(16))) u16 V[TMB * XSB];
    __shared__ __attribute__((aligned(16))) uint32_t MB[TMB * 4];
    __shared__ int TT[TMB + 2];
    const int tiles = a.T / TMB;
    const int ntiles = a.B * tiles;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int r = lane & 31, h = lane >> 5;
    const int co0 = w * 32;

    uint4 wd[3][8], wr[8];
#pragma unroll
    for (int tp = 0; tp < 3; ++tp)
#pragma unroll
        for (int kb = 0; kb < 8; ++kb)
            wd[tp][kb] = *reinterpret_cast<const uint4*>(a.wdT + (size_t)tp * C * C + (size_t)(co0 + r) * C + 8 * h + kb * 16);
#pragma unroll
    for (int kb = 0; kb < 8; ++kb)
        wr[kb] = *reinterpret_cast<const uint4*>(a.wrT + (size_t)(co0 + r) * C + 8 * h + kb * 16);

    for (int tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
        const int b = tile / tiles;
        const int p0 = (tile - b * tiles) * TMB;
        const size_t cb = (size_t)b * a.T * C;
        const size_t mbase = (size_t)b * a.T * 4;
        __syncthreads();                       // previous tile's LDS fully consumed
        tile_times(TT, p0, a.T, a.n, a.d, tid);
        __syncthreads();
        stage_rows(X, TT, a.ein, cb, a.me, mbase, tid);
        __syncthreads();

        bool ok0[4], ok2[4];
#pragma unroll
        for (int nt = 0; nt < 4; ++nt) {
            const int m = (p0 + nt * 32 + r) % a.n;
            ok0[nt] = m > 0;
            ok2[nt] = m < a.n - 1;
        }
        // GEMM 1: u^T[co][row] = sum_{tap, ci} Wd[tap][ci][co] relu(e)[row + tap - 1][ci]
        // (two passes of two 32-row N-tiles keep the accumulators at 32 VGPRs)
#pragma unroll
        for (int np = 0; np < 2; ++np) {
            f32x16 acc[2];
#pragma unroll
            for (int j = 0; j < 2; ++j)
                for (int i = 0; i < 16; ++i) acc[j][i] = 0.f;
#pragma unroll
            for (int tp = 0; tp < 3; ++tp) {
#pragma unroll
                for (int kb = 0; kb < 8; ++kb) {
#pragma unroll
                    for (int j = 0; j < 2; ++j) {
                        const int nt = 2 * np + j;
                        uint4 bv = *reinterpret_cast<const uint4*>(&X[(nt * 32 + r + tp) * XSB + kb * 16 + 8 * h]);
                        bv = relu8(bv);
                        const bool ok = tp == 0 ? ok0[nt] : (tp == 2 ? ok2[nt] : true);
                        if (!ok) bv = make_uint4(0, 0, 0, 0);
                        acc[j] = mfma_bf16(wd[tp][kb], bv, acc[j]);
                    }
                }
            }
            // epilogue 1: + bias (masked.py:155), relu (model.py:107) -> V (bf16); u>0 bits
            float bias[16];
            load_bias16(bias, a.bd + co0, h);
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                const int row = (2 * np + j) * 32 + r;
                uint32_t part = 0;
                float v[16];
#pragma unroll
                for (int i = 0; i < 16; ++i) {
                    const float u = acc[j][i] + bias[i];
                    part |= (u > 0.f ? 1u : 0u) << acc_row(i, h);
                    v[i] = fmaxf(u, 0.f);
                }
                const uint32_t word = part | (uint32_t)__shfl_xor((int)part, 32);
                if (h == 0) MB[row * 4 + w] = word;
#pragma unroll
                for (int g = 0; g < 4; ++g)
                    *reinterpret_cast<uint2*>(&V[row * XSB + co0 + 8 * g + 4 * h]) =
                        make_uint2(pack2(v[4 * g], v[4 * g + 1]), pack2(v[4 * g + 2], v[4 * g + 3]));
            }
        }
        __syncthreads();
        if (tid < TMB)
            *reinterpret_cast<uint4*>(a.mu + mbase + (size_t)TT[tid + 1] * 4) =
                *reinterpret_cast<const uint4*>(&MB[tid * 4]);

        // GEMM 2: y^T[co2][row] = sum_co Wr[co][co2] v[row][co]   (model.py:109-114)
#pragma unroll
        for (int np = 0; np < 2; ++np) {
            f32x16 acc[2];
#pragma unroll
            for (int j = 0; j < 2; ++j)
                for (int i = 0; i < 16; ++i) acc[j][i] = 0.f;
#pragma unroll
            for (int kb = 0; kb < 8; ++kb) {
#pragma unroll
                for (int j = 0; j < 2; ++j) {
                    const uint4 bv = *reinterpret_cast<const uint4*>(&V[((2 * np + j) * 32 + r) * XSB + kb * 16 + 8 * h]);
                    acc[j] = mfma_bf16(wr[kb], bv, acc[j]);
                }
            }
            // epilogue 2: e_{l+1} = e_l + (y + b_r), written over this wave's columns of X
            float bias[16];
            load_bias16(bias, a.br + co0, h);
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                const int row = (2 * np + j) * 32 + r;
#pragma unroll
                for (int g = 0; g < 4; ++g) {
                    uint2* px = reinterpret_cast<uint2*>(&X[(row + 1) * XSB + co0 + 8 * g + 4 * h]);
                    const uint2 ev = *px;
                    const float o0 = bflo(ev.x) + (acc[j][4 * g + 0] + bias[4 * g + 0]);
                    const float o1 = bfhi(ev.x) + (acc[j][4 * g + 1] + bias[4 * g + 1]);
                    const float o2 = bflo(ev.y) + (acc[j][4 * g + 2] + bias[4 * g + 2]);
                    const float o3 = bfhi(ev.y) + (acc[j][4 * g + 3] + bias[4 * g + 3]);
                    *px = make_uint2(pack2(o0, o1), pack2(o2, o3));
                }
            }
        }
        __syncthreads();
        for (int i = tid; i < TMB * 16; i += 256) {
            const int rr = i >> 4, q = i & 15;
            *reinterpret_cast<uint4*>(a.eout + cb + (size_t)TT[rr + 1] * C + q * 8) =
                *reinterpret_cast<const uint4*>(&X[(rr + 1) * XSB + q * 8]);
        }
    }
}

__global__ void __launch_bounds__(256, 2) k_block_bwd_bf16(BwdArgsB a) {
    __shared__ __attribute__((aligned(16))) u16 G[(TMB + 2) * XSB];
    __shared__ __attribute__((aligned(16))) u16 U[(TMB + 2) * XSB];
    __shared__ __attribute__((aligned(16))) uint32_t MU[(TMB + 2) * 4];
    __shared__ __attribute__((aligned(16))) uint32_t ME[TMB * 4];
    __shared__ int TT[TMB + 2];
    const int tiles = a.T / TMB;
    const int ntiles = a.B * tiles;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int r = lane & 31, h = lane >> 5;
    const int c0 = w * 32;

    uint4 wr[8], wd[3][8];
#pragma unroll
    for (int kb = 0; kb < 8; ++kb)
        wr[kb] = *reinterpret_cast<const uint4*>(a.wr + (size_t)(c0 + r) * C + 8 * h + kb * 16);
#pragma unroll
    for (int tp = 0; tp < 3; ++tp)
#pragma unroll
        for (int kb = 0; kb < 8; ++kb)
            wd[tp][kb] = *reinterpret_cast<const uint4*>(a.wd + (size_t)tp * C * C + (size_t)(c0 + r) * C + 8 * h + kb * 16);

    for (int tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
        const int b = tile / tiles;
        const int p0 = (tile - b * tiles) * TMB;
        const size_t cb = (size_t)b * a.T * C;
        const size_t mbase = (size_t)b * a.T * 4;
        __syncthreads();
        tile_times(TT, p0, a.T, a.n, a.d, tid);
        __syncthreads();
        // tot = g_{l+1} + D_{l+1}
        for (int i = tid; i < (TMB + 2) * 16; i += 256) {
            const int rr = i >> 4, q = i & 15;
            const int t = TT[rr];
            uint4 v = make_uint4(0, 0, 0, 0);
            if (t >= 0) {
                const size_t o = cb + (size_t)t * C + q * 8;
                if (a.gin && a.din) {
                    const uint4 g4 = *reinterpret_cast<const uint4*>(a.gin + o);
                    const uint4 d4 = *reinterpret_cast<const uint4*>(a.din + o);
                    v.x = pack2(bflo(g4.x) + bflo(d4.x), bfhi(g4.x) + bfhi(d4.x));
                    v.y = pack2(bflo(g4.y) + bflo(d4.y), bfhi(g4.y) + bfhi(d4.y));
                    v.z = pack2(bflo(g4.z) + bflo(d4.z), bfhi(g4.z) + bfhi(d4.z));
                    v.w = pack2(bflo(g4.w) + bflo(d4.w), bfhi(g4.w) + bfhi(d4.w));
                } else if (a.gin) {
                    v = *reinterpret_cast<const uint4*>(a.gin + o);
                } else if (a.din) {
                    v = *reinterpret_cast<const uint4*>(a.din + o);
                }
            }
            *reinterpret_cast<uint4*>(&G[rr * XSB + q * 8]) = v;
        }
        if (tid < TMB + 2) {
            const int t = TT[tid];
            uint4 mw = make_uint4(0, 0, 0, 0);
            if (t >= 0) mw = *reinterpret_cast<const uint4*>(a.mu + mbase + (size_t)t * 4);
            *reinterpret_cast<uint4*>(&MU[tid * 4]) = mw;
            if (tid < TMB)
                *reinterpret_cast<uint4*>(&ME[tid * 4]) =
                    *reinterpret_cast<const uint4*>(a.me + mbase + (size_t)TT[tid + 1] * 4);
        }
        __syncthreads();

        bool ok0[4], ok2[4];
#pragma unroll
        for (int nt = 0; nt < 4; ++nt) {
            const int m = (p0 + nt * 32 + r) % a.n;
            ok0[nt] = m > 0;
            ok2[nt] = m < a.n - 1;
        }
        // step 1: g_v^T[i][row] = sum_o Wr[i][o] tot[row][o];  g_u = [u>0] g_v -> U
#pragma unroll
        for (int np = 0; np < 2; ++np) {
            f32x16 acc[2];
#pragma unroll
            for (int j = 0; j < 2; ++j)
                for (int i = 0; i < 16; ++i) acc[j][i] = 0.f;
#pragma unroll
            for (int kb = 0; kb < 8; ++kb) {
#pragma unroll
                for (int j = 0; j < 2; ++j) {
                    const uint4 bv = *reinterpret_cast<const uint4*>(&G[((2 * np + j) * 32 + r + 1) * XSB + kb * 16 + 8 * h]);
                    acc[j] = mfma_bf16(wr[kb], bv, acc[j]);
                }
            }
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                const int row = (2 * np + j) * 32 + r;
                const uint32_t mw = MU[(row + 1) * 4 + w];
                float v[16];
#pragma unroll
                for (int i = 0; i < 16; ++i) v[i] = ((mw >> acc_row(i, h)) & 1u) ? acc[j][i] : 0.f;
#pragma unroll
                for (int g = 0; g < 4; ++g)
                    *reinterpret_cast<uint2*>(&U[(row + 1) * XSB + c0 + 8 * g + 4 * h]) =
                        make_uint2(pack2(v[4 * g], v[4 * g + 1]), pack2(v[4 * g + 2], v[4 * g + 3]));
            }
        }
        {   // the two halo rows (LDS rows 0 and TMB+1) as one more 32-column MFMA tile:
            // column r computes halo row (r & 1); lanes r = 0, 1 keep their results.
            const int hrow = (r & 1) ? TMB + 1 : 0;
            f32x16 hacc;
            for (int i = 0; i < 16; ++i) hacc[i] = 0.f;
#pragma unroll
            for (int kb = 0; kb < 8; ++kb) {
                const uint4 bv = *reinterpret_cast<const uint4*>(&G[hrow * XSB + kb * 16 + 8 * h]);
                hacc = mfma_bf16(wr[kb], bv, hacc);
            }
            if (r < 2) {
                const uint32_t mw = TT[hrow] >= 0 ? MU[hrow * 4 + w] : 0u;
                float v[16];
#pragma unroll
                for (int i = 0; i < 16; ++i) v[i] = ((mw >> acc_row(i, h)) & 1u) ? hacc[i] : 0.f;
#pragma unroll
                for (int g = 0; g < 4; ++g)
                    *reinterpret_cast<uint2*>(&U[hrow * XSB + c0 + 8 * g + 4 * h]) =
                        make_uint2(pack2(v[4 * g], v[4 * g + 1]), pack2(v[4 * g + 2], v[4 * g + 3]));
            }
        }
        __syncthreads();

        // step 2: gh^T[ci][row] = sum_{tap, co} Wd[tap][ci][co] g_u[row - tap + 1][co]
#pragma unroll
        for (int np = 0; np < 2; ++np) {
            f32x16 acc[2];
#pragma unroll
            for (int j = 0; j < 2; ++j)
                for (int i = 0; i < 16; ++i) acc[j][i] = 0.f;
#pragma unroll
            for (int tp = 0; tp < 3; ++tp) {
#pragma unroll
                for (int kb = 0; kb < 8; ++kb) {
#pragma unroll
                    for (int j = 0; j < 2; ++j) {
                        const int nt = 2 * np + j;
                        uint4 bv = *reinterpret_cast<const uint4*>(&U[(nt * 32 + r + 2 - tp) * XSB + kb * 16 + 8 * h]);
                        const bool ok = tp == 0 ? ok2[nt] : (tp == 2 ? ok0[nt] : true);
                        if (!ok) bv = make_uint4(0, 0, 0, 0);
                        acc[j] = mfma_bf16(wd[tp][kb], bv, acc[j]);
                    }
                }
            }
            // epilogue: g_l = tot + [e_l > 0] gh, over this wave's columns of G (centre rows)
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                const int row = (2 * np + j) * 32 + r;
                const uint32_t mw = ME[row * 4 + w];
#pragma unroll
                for (int g = 0; g < 4; ++g) {
                    uint2* pg = reinterpret_cast<uint2*>(&G[(row + 1) * XSB + c0 + 8 * g + 4 * h]);
                    const uint2 tv = *pg;
                    const int R = 8 * g + 4 * h;
                    const float o0 = bflo(tv.x) + (((mw >> (R + 0)) & 1u) ? acc[j][4 * g + 0] : 0.f);
                    const float o1 = bfhi(tv.x) + (((mw >> (R + 1)) & 1u) ? acc[j][4 * g + 1] : 0.f);
                    const float o2 = bflo(tv.y) + (((mw >> (R + 2)) & 1u) ? acc[j][4 * g + 2] : 0.f);
                    const float o3 = bfhi(tv.y) + (((mw >> (R + 3)) & 1u) ? acc[j][4 * g + 3] : 0.f);
                    *pg = make_uint2(pack2(o0, o1), pack2(o2, o3));
                }
            }
        }
        __syncthreads();
        for (int i = tid; i < TMB * 16; i += 256) {
            const int rr = i >> 4, q = i & 15;
            *reinterpret_cast<uint4*>(a.gout + cb + (size_t)TT[rr + 1] * C + q * 8) =
                *reinterpret_cast<const uint4*>(&G[(rr + 1) * XSB + q * 8]);
        }
    }
}

static int g_cus = 0;
static int num_cus() {
    if (!g_cus) {
        int dev = 0;
        (void)hipGetDevice(&dev);
        (void)hipDeviceGetAttribute(&g_cus, hipDeviceAttributeMultiprocessorCount, dev);
        if (g_cus <= 0) g_cus = 256;
    }
    return g_cus;
}

void launch_block_fwd_bf16(const FwdArgsB& a, hipStream_t s) {
    const int nt = a.B * (a.T / TMB);
    hipLaunchKernelGGL(k_block_fwd_bf16, dim3(std::min(nt, 2 * num_cus())), dim3(256), 0, s, a);
}
void launch_block_bwd_bf16(const BwdArgsB& a, hipStream_t s) {
    const int nt = a.B * (a.T / TMB);
    hipLaunchKernelGGL(k_block_bwd_bf16, dim3(std::min(nt, 2 * num_cus())), dim3(256), 0, s, a);
}

}  // namespace ast
