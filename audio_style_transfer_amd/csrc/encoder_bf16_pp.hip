// bf16 encoder block forward, two-group ping-pong schedule (precision 1; model.py:95-116).
//
// One persistent 512-thread workgroup per CU, split into two 4-wave groups (one wave of each
// group per SIMD).  Each group walks its own 64-position tiles (time_to_batch order,
// masked.py:57-86) through two phases separated by workgroup barriers:
//   phase a: GEMM1 (dilated conv, 48 MFMA per wave) + epilogue 1 (bias, relu, u > 0 bits)
//            + e_l > 0 bits of the tile's rows
//   phase b: GEMM2 (1x1, 16 MFMA per wave) + epilogue 2 (bias, residual) with e_{l+1} stored
//            straight from registers, commit of the next tile's prefetched rows to LDS and
//            the prefetch of the tile after it
// and the groups run one phase apart, so in every step each SIMD has one wave in an MFMA-
// heavy phase and one in a load / store / epilogue phase: the matrix cores stay fed while
// the other group's memory traffic is in flight.  Weights: Wd^T as MFMA A fragments in 96
// VGPRs per wave, Wr^T in LDS (shared by both groups).  relu(e) for GEMM1 is applied to the
// fragments after the LDS read (v_pk_max_i16), so one row image serves GEMM1 and the
// residual.
#include "common.h"
#include <algorithm>

namespace ast {

namespace {

constexpr int TP = 64;                 // positions per tile
constexpr int NRP = TP + 4;            // LDS rows max (2 segments of 32 + 2 pads each)
constexpr int NTP = 512;               // threads per workgroup
constexpr int GTH = 256;               // threads per group
constexpr int PFP = (NRP * 16 + GTH - 1) / GTH;   // 16-B pieces per thread per tile (5)
constexpr int PADP = -(1 << 28);

struct LayoutP {
    int M;       // segment length: TP (one segment + 2 halo rows) or 32 (two padded segments)
    int nrows;   // LDS rows of a tile
};

__device__ __forceinline__ uint4 relu8p(uint4 v) {
    return make_uint4(relu2(v.x), relu2(v.y), relu2(v.z), relu2(v.w));
}

__device__ __forceinline__ uint32_t sign_byte_p(uint4 v) {
    const uint32_t d[4] = {v.x, v.y, v.z, v.w};
    uint32_t bits = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        bits |= ((short)(d[j] & 0xffffu) > 0 ? 1u : 0u) << (2 * j);
        bits |= ((short)(d[j] >> 16) > 0 ? 1u : 0u) << (2 * j + 1);
    }
    return bits;
}

__device__ __forceinline__ int acc_row_p(int i, int h) { return (i & 3) + 8 * (i >> 2) + 4 * h; }

// time of LDS row L of the tile starting at position p0, or -1 (zero row)
template <bool MASKED>
__device__ __forceinline__ int row_time_p(int L, int p0, const LayoutP& ly, int T, int n, int d) {
    if (ly.M == TP) {
        const int p = p0 - 1 + L;
        if (L >= ly.nrows || p < 0 || p >= T) return -1;
        if (!MASKED) {   // halos belong to the tile's own sub-sequence only
            if (L == 0 && p0 % n == 0) return -1;
            if (L == TP + 1 && (p0 + TP) % n == 0) return -1;
        }
        return (p % n) * d + p / n;
    }
    if (L >= ly.nrows) return -1;
    const int s = L / (ly.M + 2), k = L - s * (ly.M + 2);
    if (k == 0 || k == ly.M + 1) return -1;
    const int p = p0 + s * ly.M + k - 1;
    return (p % n) * d + p / n;
}

template <bool MASKED>
__global__ void __launch_bounds__(NTP, 1) k_block_fwd_pp(FwdArgsB a, LayoutP ly) {
    __shared__ __attribute__((aligned(16))) u16 X[2][2][NRP * XSB];   // [group][buf] e_l rows
    __shared__ __attribute__((aligned(16))) u16 V[2][TP * XSB];       // [group] relu(u) by column
    __shared__ __attribute__((aligned(16))) u16 WR[C * XSB];          // Wr^T [co2][co]
    __shared__ __attribute__((aligned(16))) uint32_t MB[2][TP * 4];   // [group] u > 0 bits
    __shared__ int TTs[2][3][NRP];                                    // [group][tile % 3] row times
    __shared__ int RMAP[TP];
    __shared__ __attribute__((aligned(16))) float BIAS[2 * C];
    const int tiles = a.T / TP;
    const int ntiles = a.B * tiles;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int g = w >> 2;                  // group
    const int gt = tid & (GTH - 1);        // thread index within the group
    const int r = lane & 31, h = lane >> 5;
    const int cb = (w & 3) * 32;           // output-channel block of this wave

    uint4 wd[3][8];
#pragma unroll
    for (int tp = 0; tp < 3; ++tp)
#pragma unroll
        for (int kb = 0; kb < 8; ++kb)
            wd[tp][kb] = *reinterpret_cast<const uint4*>(a.wdT + (size_t)tp * C * C + (size_t)(cb + r) * C + 16 * kb + 8 * h);
    for (int i = tid; i < C * 16; i += NTP)
        *reinterpret_cast<uint4*>(&WR[(i >> 4) * XSB + (i & 15) * 8]) =
            *reinterpret_cast<const uint4*>(a.wrT + (size_t)(i >> 4) * C + (i & 15) * 8);
    if (tid < C) { BIAS[tid] = a.bd[tid]; BIAS[C + tid] = a.br[tid]; }
    if (tid < TP) RMAP[tid] = (tid / ly.M) * (ly.M + 2) + 1 + (tid % ly.M);

    auto tile_of = [&](int grp, int j) { return blockIdx.x + (2 * j + grp) * gridDim.x; };

    // prefetch registers of this group: piece k = LDS row (gt + k*GTH) >> 4, 16 B at q*8
    uint4 pf[PFP];
    uint32_t pfm[PFP];
    auto prefetch = [&](int j) {
        int tile = tile_of(g, j);
        tile = tile < ntiles ? tile : ntiles - 1;
        const int b = tile / tiles, p0 = (tile - b * tiles) * TP;
        const u16* src = a.ein + (size_t)b * a.T * C;
        int* TTn = TTs[g][j % 3];
#pragma unroll
        for (int k = 0; k < PFP; ++k) {
            const int i = gt + k * GTH;
            const int L = i >> 4;
            const int t = row_time_p<MASKED>(L, p0, ly, a.T, a.n, a.d);
            if ((i & 15) == 0 && L < NRP) TTn[L] = t;
            pfm[k] = t >= 0 ? 0xffffffffu : 0u;
            pf[k] = *reinterpret_cast<const uint4*>(src + (uint32_t)((t >= 0 ? t : 0) * C + (i & 15) * 8));
        }
    };
    auto commit = [&](int j) {
        u16* Xn = X[g][j & 1];
#pragma unroll
        for (int k = 0; k < PFP; ++k) {
            const int i = gt + k * GTH;
            const int L = i >> 4, q = i & 15;
            if (L >= ly.nrows) break;
            *reinterpret_cast<uint4*>(&Xn[L * XSB + q * 8]) =
                make_uint4(pf[k].x & pfm[k], pf[k].y & pfm[k], pf[k].z & pfm[k], pf[k].w & pfm[k]);
        }
    };

    // phase a of this group's tile j: GEMM1 + epilogue 1 (+ e_l > 0 bits); acc carried to b
    auto phase_a = [&](int j) {
        const int tile = tile_of(g, j);
        const int b = tile / tiles, p0 = (tile - b * tiles) * TP;
        const u16* Xc = X[g][j & 1];
        int Lc[2];
        bool ok0[2], ok2[2];
#pragma unroll
        for (int n = 0; n < 2; ++n) {
            const int c = 32 * n + r;
            Lc[n] = RMAP[c];
            ok0[n] = ok2[n] = true;
            if (MASKED) {
                const int m = (p0 + c) % a.n;
                ok0[n] = m > 0;
                ok2[n] = m < a.n - 1;
            }
        }
        f32x16 acc[2];
#pragma unroll
        for (int n = 0; n < 2; ++n)
            for (int i = 0; i < 16; ++i) acc[n][i] = 0.f;
        {
            uint4 bcur[2], bnxt[2];
            const u16* rb[2];
#pragma unroll
            for (int n = 0; n < 2; ++n) {
                rb[n] = &Xc[(Lc[n] - 1) * XSB + 8 * h];       // tap 0 row; taps 1, 2 follow
                bcur[n] = relu8p(*reinterpret_cast<const uint4*>(rb[n]));
            }
#pragma unroll
            for (int st = 0; st < 24; ++st) {
                const int tp = st >> 3, kb = st & 7;
                if (st + 1 < 24) {
                    const int tn = (st + 1) >> 3, kn = (st + 1) & 7;
#pragma unroll
                    for (int n = 0; n < 2; ++n)
                        bnxt[n] = relu8p(*reinterpret_cast<const uint4*>(rb[n] + tn * XSB + kn * 16));
                }
#pragma unroll
                for (int n = 0; n < 2; ++n) {
                    uint4 bv = bcur[n];
                    if (MASKED) {
                        const bool ok = tp == 0 ? ok0[n] : (tp == 2 ? ok2[n] : true);
                        if (!ok) bv = make_uint4(0, 0, 0, 0);
                    }
                    acc[n] = mfma_bf16(wd[tp][kb], bv, acc[n]);
                }
#pragma unroll
                for (int n = 0; n < 2; ++n) bcur[n] = bnxt[n];
            }
        }
        // epilogue 1: + b_d (masked.py:155), relu (model.py:107) -> V; u > 0 bits -> MB
        float bias[16];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const float4 v4 = *reinterpret_cast<const float4*>(&BIAS[cb + 8 * q + 4 * h]);
            bias[4 * q] = v4.x; bias[4 * q + 1] = v4.y; bias[4 * q + 2] = v4.z; bias[4 * q + 3] = v4.w;
        }
        u16* Vg = V[g];
#pragma unroll
        for (int n = 0; n < 2; ++n) {
            const int c = 32 * n + r;
            uint32_t part = 0;
            float v[16];
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                const float u = acc[n][i] + bias[i];
                part |= (u > 0.f ? 1u : 0u) << acc_row_p(i, h);
                v[i] = fmaxf(u, 0.f);
            }
            const uint32_t word = part | (uint32_t)__shfl_xor((int)part, 32);
            if (h == 0) MB[g][c * 4 + (w & 3)] = word;
#pragma unroll
            for (int q = 0; q < 4; ++q)
                *reinterpret_cast<uint2*>(&Vg[c * XSB + cb + 8 * q + 4 * h]) =
                    make_uint2(pack2(v[4 * q], v[4 * q + 1]), pack2(v[4 * q + 2], v[4 * q + 3]));
        }
        // e_l > 0 bits of the tile's 64 rows, one byte (8 channels) per piece, by position
        uint8_t* meb = reinterpret_cast<uint8_t*>(a.me + (size_t)b * a.T * 4);
#pragma unroll
        for (int k = 0; k < TP * 16 / GTH; ++k) {
            const int i = gt + k * GTH, cc = i >> 4, q = i & 15;
            const uint4 v = *reinterpret_cast<const uint4*>(&Xc[RMAP[cc] * XSB + q * 8]);
            meb[(uint32_t)((p0 + cc) * 16 + q)] = (uint8_t)sign_byte_p(v);
        }
    };

    // phase b: u > 0 bits out, GEMM2 + epilogue 2 (e_{l+1} stored from registers), then the
    // next tile's rows into the other buffer and the prefetch of the one after
    auto phase_b = [&](int j) {
        const int tile = tile_of(g, j);
        const int b = tile / tiles, p0 = (tile - b * tiles) * TP;
        const u16* Xc = X[g][j & 1];
        const int* TT = TTs[g][j % 3];
        a.mu[(size_t)b * a.T * 4 + (uint32_t)((p0 + (gt >> 2)) * 4 + (gt & 3))] = MB[g][gt];
        const u16* Vg = V[g];
        f32x16 acc[2];
#pragma unroll
        for (int n = 0; n < 2; ++n)
            for (int i = 0; i < 16; ++i) acc[n][i] = 0.f;
        {
            uint4 acur, anxt, bcur[2], bnxt[2];
            acur = *reinterpret_cast<const uint4*>(&WR[(cb + r) * XSB + 8 * h]);
#pragma unroll
            for (int n = 0; n < 2; ++n)
                bcur[n] = *reinterpret_cast<const uint4*>(&Vg[(32 * n + r) * XSB + 8 * h]);
#pragma unroll
            for (int kb = 0; kb < 8; ++kb) {
                if (kb + 1 < 8) {
                    anxt = *reinterpret_cast<const uint4*>(&WR[(cb + r) * XSB + (kb + 1) * 16 + 8 * h]);
#pragma unroll
                    for (int n = 0; n < 2; ++n)
                        bnxt[n] = *reinterpret_cast<const uint4*>(&Vg[(32 * n + r) * XSB + (kb + 1) * 16 + 8 * h]);
                }
#pragma unroll
                for (int n = 0; n < 2; ++n) acc[n] = mfma_bf16(acur, bcur[n], acc[n]);
                acur = anxt;
#pragma unroll
                for (int n = 0; n < 2; ++n) bcur[n] = bnxt[n];
            }
        }
        float bias[16];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const float4 v4 = *reinterpret_cast<const float4*>(&BIAS[C + cb + 8 * q + 4 * h]);
            bias[4 * q] = v4.x; bias[4 * q + 1] = v4.y; bias[4 * q + 2] = v4.z; bias[4 * q + 3] = v4.w;
        }
        u16* dst = a.eout + (size_t)b * a.T * C;
#pragma unroll
        for (int n = 0; n < 2; ++n) {
            const int L = RMAP[32 * n + r];
            u16* drow = dst + (uint32_t)(TT[L] * C + cb + 4 * h);
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const uint2 ev = *reinterpret_cast<const uint2*>(&Xc[L * XSB + cb + 8 * q + 4 * h]);
                const float o0 = bflo(ev.x) + (acc[n][4 * q + 0] + bias[4 * q + 0]);
                const float o1 = bfhi(ev.x) + (acc[n][4 * q + 1] + bias[4 * q + 1]);
                const float o2 = bflo(ev.y) + (acc[n][4 * q + 2] + bias[4 * q + 2]);
                const float o3 = bfhi(ev.y) + (acc[n][4 * q + 3] + bias[4 * q + 3]);
                *reinterpret_cast<uint2*>(drow + 8 * q) = make_uint2(pack2(o0, o1), pack2(o2, o3));
            }
        }
        commit(j + 1);
        prefetch(j + 2);
    };

    prefetch(0);
    commit(0);
    prefetch(1);
    __syncthreads();
    for (int s = 0;; ++s) {
        const bool done0 = tile_of(0, s >> 1) >= (unsigned)ntiles;
        const bool done1 = s == 0 ? tile_of(1, 0) >= (unsigned)ntiles : tile_of(1, (s - 1) >> 1) >= (unsigned)ntiles;
        if (done0 && done1) break;
        const int sg = s - g;
        if (sg >= 0) {
            const int j = sg >> 1;
            if (tile_of(g, j) < (unsigned)ntiles) {
                if ((sg & 1) == 0) phase_a(j);
                else phase_b(j);
            }
        }
        __syncthreads();
    }
}

bool pick_layout_p(int n, LayoutP& ly) {
    if (n % TP == 0) { ly.M = TP; ly.nrows = TP + 2; return false; }
    if (n == 32) { ly.M = 32; ly.nrows = 2 * 34; return false; }
    ly.M = TP; ly.nrows = TP + 2;
    return true;
}

int g_cus_p = 0;

}  // namespace

void launch_block_fwd_pp(const FwdArgsB& a, hipStream_t s) {
    if (!g_cus_p) {
        int dev = 0;
        (void)hipGetDevice(&dev);
        (void)hipDeviceGetAttribute(&g_cus_p, hipDeviceAttributeMultiprocessorCount, dev);
        if (g_cus_p <= 0) g_cus_p = 256;
    }
    const int nt = a.B * (a.T / TP);
    const dim3 grid(std::min((nt + 1) / 2, g_cus_p));
    LayoutP ly;
    if (pick_layout_p(a.n, ly)) hipLaunchKernelGGL(k_block_fwd_pp<true>, grid, dim3(NTP), 0, s, a, ly);
    else hipLaunchKernelGGL(k_block_fwd_pp<false>, grid, dim3(NTP), 0, s, a, ly);
}

}  // namespace ast
