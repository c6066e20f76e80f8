// bf16 encoder block backward (precision 1): d loss / d e_l for one block of model.py:95-116,
// restated by oracle/astyle_oracle.py:171-189 (encoder_backward):
//   tot = d loss / d e_{l+1}, its own direct loss term included (the chain holds it pre-added)
//   g_u = [u > 0] (W_r tot)                         1x1 conv transposed
//   g_a = sum_k W_d[k] g_u(p - k + 1)                K = 3 SAME dilated conv transposed, in
//                                                    time_to_batch positions (masked.py:110-160)
//   out = tot + [e_l > 0] g_a + D_l                  D_l: direct loss gradient of e_l, if tapped
// bf16 storage, v_mfma_f32_32x32x16_bf16 with fp32 accumulation; out is rounded to bf16 once.
//
// Same column-owning scheme as the forward (colwave.h): one workgroup per CU, persistent over
// tiles of 128 positions; wave w owns tile columns 32 w .. 32 w + 31 and all 128 channels.
// Per tile:
//  1. g_u of the own columns: A = W_r fragments (LDS), B = the own tot rows of the LDS image.
//     One-segment layouts also compute channels 32 w .. 32 w + 31 of the two halo rows.  g_u
//     (bf16) overwrites the own tot rows in place (each lane rewrites exactly the 16-B chunks it
//     read; the tot fragments stay in registers for step 3), the halo rows go to HALO.  Barrier.
//  2. g_a: 3 taps x 8 k-blocks x 4 channel tiles (taps 0 / 2 A fragments in AGPRs, tap 1 in
//     LDS), B = g_u rows p+1, p, p-1; the next tile's tot image streams in underneath.
//  3. [e_l > 0] mask, + tot and + D_l as identity MFMAs (exact), bf16, whole-row stores through
//     the wave's staging rows.  D_l arrives in registers (whole-line loads issued at the top of
//     the tile, LDS has no room for a third image) and becomes B fragments through the same
//     staging rows.
#include "colwave.h"
#include <algorithm>

namespace ast {
namespace {
using namespace cw;

template <bool MASKED, bool HAS_D>
__global__ void __launch_bounds__(FT, 1) k_block_bwd_c(BwdArgsC a, Layout ly) {
    __shared__ __attribute__((aligned(16))) uint8_t XS[2][BUFB];      // tot images, g_u in place
    __shared__ __attribute__((aligned(16))) uint8_t HALO[2 * RSB];    // g_u of the two halo rows
    __shared__ __attribute__((aligned(16))) uint4 W1[4 * 8 * 64];     // W_d tap 1 A fragments
    __shared__ __attribute__((aligned(16))) uint4 WRL[4 * 8 * 64];    // W_r A fragments
    __shared__ __attribute__((aligned(16))) uint8_t STG[4][32 * SRB]; // D / output staging, per wave

    const int tiles = a.T / TMB;
    const int ntiles = a.B * tiles;
    const int tid = threadIdx.x, lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int r = lane & 31, h = lane >> 5;

    // ---- per-launch setup (as the forward: taps 0 / 2 in AGPRs, tap 1 and W_r in LDS) --------
    // the first tile's image streams in while the weights load (it only touches XS[0])
    ImageDma<MASKED> dma;
    dma.init(w, lane, ly, a.d);
    if (blockIdx.x < ntiles) {
        dma.aim(a.tin, tile_at<MASKED>(blockIdx.x, tiles, a.n, a.d, ly), ly, a.T, a.n);
        const uint32_t lds0 = (uint32_t)(uintptr_t)&XS[0][0] + (uint32_t)(w * 1024);
#pragma unroll
        for (int j = 0; j < DPW; ++j) dma.issue(j, a.tin, a.zero, lds0, a.T, a.n, a.d);
    }
    uint4 wr0[4][8], wr2[4][8];
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int kb = 0; kb < 8; ++kb) {
            wr0[q][kb] = to_agpr(*reinterpret_cast<const uint4*>(a.wbf + ((size_t)((0 * 4 + q) * 8 + kb) * 64 + lane) * 8));
            wr2[q][kb] = to_agpr(*reinterpret_cast<const uint4*>(a.wbf + ((size_t)((2 * 4 + q) * 8 + kb) * 64 + lane) * 8));
        }
    for (int i = tid; i < 4 * 8 * 64; i += FT) {
        W1[i] = *reinterpret_cast<const uint4*>(a.wbf + ((size_t)4 * 8 * 64 + i) * 8);
        WRL[i] = *reinterpret_cast<const uint4*>(a.wrb + (size_t)i * 8);
    }
    if (tid < 2 * 64)   // group 36 of both images (colwave.h, DPW)
        *reinterpret_cast<uint4*>(&XS[tid >> 6][4 * DPW * 1024 + (tid & 63) * 16]) = make_uint4(0, 0, 0, 0);
    const uint4 id0 = identity_frag(0, r, h), id1 = identity_frag(1, r, h);
    f32x16 zf;
#pragma unroll
    for (int i = 0; i < 16; ++i) zf[i] = 0.f;

    const int c = 32 * w + r;                // this lane's tile column
    const int Lc = frow(c, ly);
    const bool onesg = ly.M == TMB;          // halo rows are real positions (else zero pad rows)
    // staged output / D rows: piece k of a half is wave column 8 k + lane / 8
    int otoff[4];
#pragma unroll
    for (int k = 0; k < 4; ++k)
        otoff[k] = MASKED ? 0 : row_toff(frow(32 * w + 8 * k + (lane >> 3), ly), ly, a.d);
    uint8_t* stg = &STG[w][0];
    __syncthreads();

    auto tile_of = [&](int tl) { return tile_at<MASKED>(tl, tiles, a.n, a.d, ly); };
    auto ctime = [&](const Tile& t, int cc, int toff) { return col_time<MASKED>(t, cc, toff, a.n, a.d); };

    // relu-mask words of a tile (this layer's positions): u > 0 and e_l > 0 of the own column,
    // u > 0 word w of the halo rows (lanes r = 0, 1; the others load a harmless duplicate)
    struct Masks { uint2 mu, me; uint32_t muh; };
    auto load_masks = [&](const Tile& t) {
        Masks m;
        const size_t row = (size_t)t.b * a.T + t.p0 + c;
        m.mu = *reinterpret_cast<const uint2*>(a.mu + row * 8 + 4 * h);
        m.me = *reinterpret_cast<const uint2*>(a.me + row * 8 + 4 * h);
        m.muh = 0;
        if (onesg) {
            const int p = min(max(r == 0 ? t.p0 - 1 : t.p0 + TMB, 0), a.T - 1);
            m.muh = a.mu[((size_t)t.b * a.T + p) * 8 + 4 * h + w];
        }
        return m;
    };

    Masks mk{};
    if (blockIdx.x < ntiles) mk = load_masks(tile_of(blockIdx.x));   // the first tile's masks
    STAMP_DECL
    int it = 0;
    for (int tile = blockIdx.x; tile < ntiles; tile += gridDim.x, ++it) {
        const int cur = it & 1;
        const Tile cu = tile_of(tile);
        // this tile's image has landed (only the previous tile's 8 output stores, issued after
        // its last DMA, may still be in flight: vmcnt counts in issue order); the barrier
        // publishes every wave's part and retires all reads of the other image
        if (it) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        STAMP(4)
        const Masks mc = mk;
        const int ntl = tile + gridDim.x < ntiles ? tile + gridDim.x : ntiles - 1;
        const Tile nx = tile_of(ntl);
        // plain loads ahead of the next tile's DMA (the vmcnt(8) above relies on the order)
        mk = load_masks(nx);
        // D_l rows of the wave's 32 columns as whole 128-B half-row lines: piece k is column
        // 8 k + lane / 8, chunk lane & 7 of half lo / hi (the staging-row order)
        uint4 dlo[4], dhi[4];
        if constexpr (HAS_D) {
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const int tt = ctime(cu, 32 * w + 8 * k + (lane >> 3), otoff[k]);
                const u16* src = a.dadd + ((size_t)cu.b * a.T + tt) * C + (lane & 7) * 8;
                dlo[k] = ld16(src);
                dhi[k] = ld16(src + 64);
            }
        }

        bool ok0 = true, ok2 = true;
        if (MASKED) {
            const int m = (cu.p0 + c) % a.n;
            ok0 = m > 0;
            ok2 = m < a.n - 1;
        }
        uint8_t* const img = &XS[cur][0];
        const uint8_t* const own = img + Lc * RSB + h * 16;   // this lane's half of its own row

        // ---- step 1: g_v = W_r tot (own columns, then the halo rows) ----
        uint4 tb[8];
        f32x16 acc[4];
#pragma unroll
        for (int kb = 0; kb < 8; ++kb) tb[kb] = lds16(own + kb * 32);
#pragma unroll
        for (int q = 0; q < 4; ++q) acc[q] = zf;
        {
            uint4 al[2][4];
#pragma unroll
            for (int q = 0; q < 4; ++q) al[0][q] = WRL[(q * 8) * 64 + lane];
#pragma unroll
            for (int kb = 0; kb < 8; ++kb) {
                if (kb + 1 < 8) {
#pragma unroll
                    for (int q = 0; q < 4; ++q) al[(kb + 1) & 1][q] = WRL[(q * 8 + kb + 1) * 64 + lane];
                }
#pragma unroll
                for (int q = 0; q < 4; ++q) acc[q] = mfma_bf16(al[kb & 1][q], tb[kb], acc[q]);
                __builtin_amdgcn_sched_barrier(0);
            }
        }
        f32x16 acch = zf;
        if (onesg) {
            const uint8_t* hr = img + (r == 1 ? (TMB + 1) * RSB : 0) + h * 16;
#pragma unroll
            for (int kb = 0; kb < 8; ++kb)
                acch = mfma_bf16(WRL[(w * 8 + kb) * 64 + lane], lds16(hr + kb * 32), acch);
        }
        // g_u = [u > 0] g_v -> bf16: own rows in place, halo rows to HALO
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            apply_mask(acc[q], mask_word(mc.mu, q));
            uint32_t o[8];
            uint4 opk[2];
            pack_tile(acc[q], o);
            swap_tile(o, opk);
#pragma unroll
            for (int gp = 0; gp < 2; ++gp)
                *reinterpret_cast<uint4*>(img + Lc * RSB + (4 * q + 2 * gp + h) * 16) = opk[gp];
        }
        if (onesg) {
            apply_mask(acch, mc.muh);
            uint32_t o[8];
            uint4 opk[2];
            pack_tile(acch, o);
            swap_tile(o, opk);
            if (r < 2) {
#pragma unroll
                for (int gp = 0; gp < 2; ++gp)
                    *reinterpret_cast<uint4*>(HALO + r * RSB + (4 * w + 2 * gp + h) * 16) = opk[gp];
            }
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        STAMP(5)

        // ---- step 2: g_a = sum_k W_d[k] g_u(p - k + 1), next tile's DMA underneath ----
        const uint8_t* const x0 = (onesg && c == TMB - 1) ? HALO + RSB + h * 16 : own + RSB;  // g_u(p + 1)
        const uint8_t* const x2 = (onesg && c == 0) ? HALO + h * 16 : own - RSB;              // g_u(p - 1)
#pragma unroll
        for (int q = 0; q < 4; ++q) acc[q] = zf;
        const uint32_t lds0 = (uint32_t)(uintptr_t)&XS[cur ^ 1][0] + (uint32_t)(w * 1024);
        dma.aim(a.tin, nx, ly, a.T, a.n);
        {
            auto bload = [&](int st) {
                const int tp = st >> 3;
                return lds16((tp == 0 ? x0 : tp == 1 ? own : x2) + (st & 7) * 32);
            };
            uint4 bl[3], al[2][4];
            bl[0] = bload(0);
            bl[1] = bload(1);
#pragma unroll
            for (int st = 0; st < 24; ++st) {
                const int tp = st >> 3, kb = st & 7;
                if (st + 2 < 24) bl[(st + 2) % 3] = bload(st + 2);
                if (st + 1 >= 8 && st + 1 < 16) {
#pragma unroll
                    for (int q = 0; q < 4; ++q) al[(st + 1) & 1][q] = W1[(q * 8 + ((st + 1) & 7)) * 64 + lane];
                }
                uint4 bv = bl[st % 3];
                if (MASKED && ((tp == 0 && !ok2) || (tp == 2 && !ok0))) bv = make_uint4(0, 0, 0, 0);
                if (tp == 0) {
#pragma unroll
                    for (int q = 0; q < 4; ++q) acc[q] = mfma_bf16(wr0[q][kb], bv, acc[q]);
                } else if (tp == 1) {
#pragma unroll
                    for (int q = 0; q < 4; ++q) acc[q] = mfma_bf16(al[st & 1][q], bv, acc[q]);
                } else {
#pragma unroll
                    for (int q = 0; q < 4; ++q) acc[q] = mfma_bf16(wr2[q][kb], bv, acc[q]);
                }
                if (st < 4) {
                    dma.issue(2 * st, a.tin, a.zero, lds0, a.T, a.n, a.d);
                    dma.issue(2 * st + 1, a.tin, a.zero, lds0, a.T, a.n, a.d);
                }
                if (st == 4) dma.issue(8, a.tin, a.zero, lds0, a.T, a.n, a.d);
#pragma unroll
                for (int m = 0; m < 4; ++m) {
                    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);   // 1 MFMA
                    __builtin_amdgcn_sched_group_barrier(0x002, 4, 0);   // up to 4 VALU
                }
                __builtin_amdgcn_sched_barrier(0);
            }
        }
        STAMP(6)

        // ---- step 3: out = tot + [e_l > 0] g_a + D_l -> bf16 -> HBM ----
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            apply_mask(acc[q], mask_word(mc.me, q));
            acc[q] = mfma_bf16(id0, tb[2 * q], acc[q]);
            acc[q] = mfma_bf16(id1, tb[2 * q + 1], acc[q]);
        }
#pragma unroll
        for (int rho = 0; rho < 2; ++rho) {
            if constexpr (HAS_D) {
                // + D_l: its half rows go through the staging rows to become B fragments
                wave_fence();
#pragma unroll
                for (int k = 0; k < 4; ++k)
                    *reinterpret_cast<uint4*>(stg + (8 * k + (lane >> 3)) * SRB + (lane & 7) * 16) = rho ? dhi[k] : dlo[k];
                wave_fence();
#pragma unroll
                for (int kbp = 0; kbp < 4; ++kbp) {
                    const uint4 df = lds16(stg + r * SRB + (2 * kbp + h) * 16);
                    const int q = 2 * rho + (kbp >> 1);
                    acc[q] = mfma_bf16((kbp & 1) ? id1 : id0, df, acc[q]);
                }
            }
            uint4 opk[2][2];
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                uint32_t o[8];
                pack_tile(acc[2 * rho + j], o);
                swap_tile(o, opk[j]);
            }
            wave_fence();
#pragma unroll
            for (int j = 0; j < 2; ++j)
#pragma unroll
                for (int gp = 0; gp < 2; ++gp)
                    *reinterpret_cast<uint4*>(stg + r * SRB + (4 * j + 2 * gp + h) * 16) = opk[j][gp];
            wave_fence();
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const uint4 v = lds16(stg + (8 * k + (lane >> 3)) * SRB + (lane & 7) * 16);
                const int tt = ctime(cu, 32 * w + 8 * k + (lane >> 3), otoff[k]);
                *reinterpret_cast<uint4*>(a.gout + ((size_t)cu.b * a.T + tt) * C + 64 * rho + (lane & 7) * 8) = v;
            }
        }
        STAMP(7)
    }
    STAMP_FLUSH(a.stamps)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

}  // namespace

void launch_block_bwd_c(const BwdArgsC& a, hipStream_t s) {
    const int nt = a.B * (a.T / TMB);
    const dim3 grid(std::min(nt, cw::num_cus()));
    Layout ly;
    if (pick_layout(a.n, ly)) {
        if (a.dadd) hipLaunchKernelGGL((k_block_bwd_c<true, true>), grid, dim3(FT), 0, s, a, ly);
        else hipLaunchKernelGGL((k_block_bwd_c<true, false>), grid, dim3(FT), 0, s, a, ly);
    } else {
        if (a.dadd) hipLaunchKernelGGL((k_block_bwd_c<false, true>), grid, dim3(FT), 0, s, a, ly);
        else hipLaunchKernelGGL((k_block_bwd_c<false, false>), grid, dim3(FT), 0, s, a, ly);
    }
}

}  // namespace ast
