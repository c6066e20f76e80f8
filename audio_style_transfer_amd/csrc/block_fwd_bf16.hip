// bf16 encoder block forward (precision 1): model.py:95-116 for one block,
//   u = dconv_d(relu(e_l)) + b_d        (masked.py:110-160, K = 3, SAME zero padding)
//   e_{l+1} = e_l + W_r^T relu(u) + b_r
// with bf16 storage, v_mfma_f32_32x32x16_bf16 and fp32 accumulation.
//
// MI355X mapping ("column-owning" waves):
//  * One 256-thread workgroup per CU (one wave per SIMD, up to 512 registers each), persistent
//    over tiles of TMB = 128 positions in time_to_batch order (masked.py:57-86).  Wave w owns
//    tile columns 32w..32w+31 and computes ALL 128 output channels of them, so nothing a wave
//    produces is read by another wave: the only barrier per tile guards the input image.
//  * Weights never leave the CU: W_d^T taps 0 and 2 sit in 256 registers as MFMA A fragments,
//    tap 1 and W_r^T sit in LDS in fragment order (one conflict-free ds_read_b128 per fragment).
//  * relu(u) never touches LDS: GEMM 1's fp32 accumulators are packed to bf16 and used directly
//    as GEMM 2's B fragments.  GEMM 2's K (channel) order is permuted on the host to match the
//    accumulator layout (WRF below).
//  * Biases enter as the accumulators' initial values, the residual e_l as two MFMAs per
//    32-channel tile against an identity fragment (exact: bf16 x 1.0 into fp32).
//  * Input rows stream HBM -> LDS by global_load_lds (no VGPR staging), double-buffered: the
//    next tile lands while this one computes.  Image rows are 272 B (256 + 16 pad), which makes
//    the column-wise fragment reads conflict-free; the DMA fills the pad slot with a harmless
//    re-read of the row's first chunk.
//  * relu masks leave as 16-bit words in the accumulator layout (bit mbit(i) = element i of one
//    lane's 32x32 tile, common.h): u > 0 by this layer's position, e_{l+1} > 0 by the NEXT layer's
//    position, so the backward applies them with no bit shuffling (block_bwd_bf16.hip).
#include "colwave.h"
#include <algorithm>
#include <type_traits>

namespace ast {
namespace {
using namespace cw;

template <bool MASKED>
__global__ void __launch_bounds__(FT, 1) k_block_fwd_c(FwdArgsC a, Layout ly) {
    __shared__ __attribute__((aligned(16))) uint8_t XS[2][BUFB];   // e_l tile images
    __shared__ __attribute__((aligned(16))) uint4 W1[4 * 8 * 64];  // W_d^T tap 1 A fragments
    __shared__ __attribute__((aligned(16))) uint4 WRL[4 * 8 * 64]; // W_r^T A fragments (K permuted)
    __shared__ __attribute__((aligned(16))) float BIAS[2 * C];     // b_d, b_r
    __shared__ __attribute__((aligned(16))) uint8_t STG[4][32 * SRB]; // output staging, per wave

    const int tiles = a.T / TMB;
    const int ntiles = a.B * tiles;
    const int tid = threadIdx.x, lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int r = lane & 31, h = lane >> 5;

    // ---- per-launch setup -------------------------------------------------------------
    // the first tile's image streams in while the weights load (it only touches XS[0])
    ImageDma<MASKED> dma;
    dma.init(w, lane, ly, a.d);
    if (blockIdx.x < ntiles) {
        dma.aim(a.ein, tile_at<MASKED>(blockIdx.x, tiles, a.n, a.d, ly), ly, a.T, a.n);
        const uint32_t lds0 = (uint32_t)(uintptr_t)&XS[0][0] + (uint32_t)(w * 1024);
#pragma unroll
        for (int j = 0; j < DPW; ++j) dma.issue(j, a.ein, a.zero, lds0, a.T, a.n, a.d);
    }
    // taps 0 and 2 live in the accumulator register file (MFMA A operands may be AGPRs): the
    // arch VGPRs stay free for accumulators, fragments and addresses.  Plain loads (the compiler
    // counts them), then a tied no-op asm that pins each fragment to AGPRs.
    uint4 wr0[4][8], wr2[4][8];
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int kb = 0; kb < 8; ++kb) {
            wr0[q][kb] = to_agpr(*reinterpret_cast<const uint4*>(a.wf + ((size_t)((0 * 4 + q) * 8 + kb) * 64 + lane) * 8));
            wr2[q][kb] = to_agpr(*reinterpret_cast<const uint4*>(a.wf + ((size_t)((2 * 4 + q) * 8 + kb) * 64 + lane) * 8));
        }
    for (int i = tid; i < 4 * 8 * 64; i += FT) {
        W1[i] = *reinterpret_cast<const uint4*>(a.wf + ((size_t)4 * 8 * 64 + i) * 8);
        WRL[i] = *reinterpret_cast<const uint4*>(a.wrf + (size_t)i * 8);
    }
    if (tid < C) { BIAS[tid] = a.bd[tid]; BIAS[C + tid] = a.br[tid]; }
    if (tid < 2 * 64)   // group 36 of both images (see DPW)
        *reinterpret_cast<uint4*>(&XS[tid >> 6][4 * DPW * 1024 + (tid & 63) * 16]) = make_uint4(0, 0, 0, 0);
    const uint4 idf[2] = {identity_frag(0, r, h), identity_frag(1, r, h)};

    const int c = 32 * w + r;                  // this lane's tile column
    const int Lc = frow(c, ly);
    const int tcoff = MASKED ? 0 : row_toff(Lc, ly, a.d);
    __syncthreads();

    // staged output rows: piece k of a round is wave column 8 k + lane / 8
    int otoff[4];
#pragma unroll
    for (int k = 0; k < 4; ++k)
        otoff[k] = MASKED ? 0 : row_toff(frow(32 * w + 8 * k + (lane >> 3), ly), ly, a.d);
    uint8_t* stg = &STG[w][0];

    auto tile_of = [&](int tl) { return tile_at<MASKED>(tl, tiles, a.n, a.d, ly); };
    auto ctime = [&](const Tile& t, int cc, int toff) { return col_time<MASKED>(t, cc, toff, a.n, a.d); };

    // ---- epilogue 2 pieces (run for the PREVIOUS tile while this tile's GEMM 1 runs) ------
    // chunk(q2): bf16 pack, e_{l+1} > 0 bits, half-wave swap: afterwards lane (n, h) holds
    // 16-B chunks 4 q2 + 2 gp + h (gp = 0, 1) of row n
    auto epi2_chunk = [&](const f32x16& acc2q, uint4 (&opk)[2], uint32_t& mebq) {
        uint32_t o[8];
        pack_tile(acc2q, o);
        mebq = pos_bits16(o);
        swap_tile(o, opk);
    };
    // round rho: channels 64 rho .. 64 rho + 63 (32-channel tiles 2 rho, 2 rho + 1) of the
    // wave's 32 rows go through the staging rows and leave as whole 128-B lines (8 lanes per
    // row half)
    auto epi2_stage = [&](int rho, const uint4 (&opk)[2][2]) {
        wave_fence();
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int gp = 0; gp < 2; ++gp)
                *reinterpret_cast<uint4*>(stg + r * SRB + (4 * j + 2 * gp + h) * 16) = opk[j][gp];
        wave_fence();
    };
    auto epi2_store = [&](int rho, const Tile& t) {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint4 v = lds16(stg + (8 * k + (lane >> 3)) * SRB + (lane & 7) * 16);
            const int tt = ctime(t, 32 * w + 8 * k + (lane >> 3), otoff[k]);
            *reinterpret_cast<uint4*>(a.eout + ((size_t)t.b * a.T + tt) * C + 64 * rho + (lane & 7) * 8) = v;
        }
    };
    auto me_store = [&](const Tile& t, const uint32_t (&meb)[4]) {
        if (a.me_next) {
            const int tc = ctime(t, c, tcoff);
            const int pn = (tc & ((1 << a.dn_log2) - 1)) * a.nn + (tc >> a.dn_log2);
            *reinterpret_cast<uint2*>(a.me_next + ((size_t)t.b * a.T + pn) * 8 + 4 * h) =
                make_uint2(meb[0] | (meb[1] << 16), meb[2] | (meb[3] << 16));
        }
    };

    f32x16 acc[4];                 // GEMM 1 accumulators
    f32x16 acc2[4];                 // GEMM 2 accumulators, carried into the next iteration
    Tile prev{0, 0, 0};
    int it = 0;
    STAMP_DECL

    // One tile per iteration, two phases:
    //  A: GEMM 1 of this tile (24 steps x 4 MFMA) with, spread over its 8 windows of 3 steps,
    //     epilogue 2 + stores of the previous tile and the DMA of the next tile
    //  B: epilogue 1 of this tile interleaved with its GEMM 2 (10 steps x 4 MFMA)
    auto body = [&](auto has_prev, int tile) {
        constexpr bool PREV = decltype(has_prev)::value;
        const int cur = it & 1;
        const Tile cu = tile_of(tile);
        // this wave's DMA of the current image is complete: vmcnt counts in issue order, and
        // only 5 stores follow the last DMA slot (step 16) of the previous iteration: the second
        // half's 4 row stores (step 18) and the u > 0 mask store of phase B; the barrier
        // publishes every wave's part and retires all reads of the other image
        if (PREV) asm volatile("s_waitcnt vmcnt(5)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        STAMP(0)

        bool ok0 = true, ok2 = true;
        if (MASKED) {
            const int m = (cu.p0 + c) % a.n;
            ok0 = m > 0;
            ok2 = m < a.n - 1;
        }
        const uint8_t* xb = &XS[cur][(Lc - 1) * RSB + h * 16];   // tap-0 row, this lane's half

        // next tile's DMA: source pointers of the wave's slots
        const int ntl = tile + gridDim.x < ntiles ? tile + gridDim.x : ntiles - 1;
        const uint32_t lds0 = (uint32_t)(uintptr_t)&XS[cur ^ 1][0] + (uint32_t)(w * 1024);
        dma.aim(a.ein, tile_of(ntl), ly, a.T, a.n);
        auto dma_slot = [&](int j) { dma.issue(j, a.ein, a.zero, lds0, a.T, a.n, a.d); };

        // ---- phase A ----
#pragma unroll
        for (int q = 0; q < 4; ++q)
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const float4 b4 = *reinterpret_cast<const float4*>(&BIAS[32 * q + 8 * g + 4 * h]);
                acc[q][4 * g + 0] = b4.x; acc[q][4 * g + 1] = b4.y;
                acc[q][4 * g + 2] = b4.z; acc[q][4 * g + 3] = b4.w;
            }
        uint4 opk[2][2];
        uint32_t meb[4];
        uint32_t o2[8];
        {
            auto bload = [&](int st) { return lds16(xb + (st >> 3) * RSB + (st & 7) * 32); };
            // B fragment of step st: relu'd (and tap-masked) one step ahead, so no MFMA waits on
            // the VALU that forms its operand
            auto bprep = [&](int st, uint4 v) {
                const int tp = st >> 3;
                v = relu8(v);
                if (MASKED && ((tp == 0 && !ok0) || (tp == 2 && !ok2))) v = make_uint4(0, 0, 0, 0);
                return v;
            };
            uint4 bl[3], al[2][4];
            bl[0] = bload(0);
            bl[1] = bload(1);
            uint4 bn = bprep(0, bl[0]);
#pragma unroll
            for (int st = 0; st < 24; ++st) {
                const int tp = st >> 3, kb = st & 7;
                if (st + 2 < 24) bl[(st + 2) % 3] = bload(st + 2);
                if (st + 1 >= 8 && st + 1 < 16) {
#pragma unroll
                    for (int q = 0; q < 4; ++q) al[(st + 1) & 1][q] = W1[(q * 8 + ((st + 1) & 7)) * 64 + lane];
                }
                const uint4 bv = bn;
                if (st + 1 < 24) bn = bprep(st + 1, bl[(st + 1) % 3]);
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
                // side work, spread so that every step carries a few independent instructions
                // between its MFMAs: epilogue 2 of the previous tile (pack / mask bits / swap of
                // 32-channel tile q2 in steps 3 q2 .. 3 q2 + 2, staging + whole-row stores in
                // steps 6-18) and the next tile's DMA (one slot every other step, 0-16).  The wait
                // at the top counts what follows the last slot (vmcnt(5)).
                if (st % 2 == 0 && st / 2 < DPW) dma_slot(st / 2);   // one slot every other step
                if (PREV) {
                    // tile q2 = 0, 1 in steps 0-5, staged at 6, stored at 10; q2 = 2, 3 in steps
                    // 7-9 and 11-13, staged at 15, stored at 18
                    constexpr int qs[24] = {0, 0, 0, 1, 1, 1, -1, 2, 2, 2, -1, 3, 3, 3, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1};
                    constexpr int ph[24] = {0, 1, 2, 0, 1, 2, -1, 0, 1, 2, -1, 0, 1, 2, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1};
                    if (qs[st] >= 0) {
                        const int q2 = qs[st];
                        if (ph[st] == 0) pack_tile(acc2[q2], o2);
                        if (ph[st] == 1) meb[q2] = pos_bits16(o2);
                        if (ph[st] == 2) swap_tile(o2, opk[q2 & 1]);
                    }
                    if (st == 6) epi2_stage(0, opk);
                    if (st == 10) epi2_store(0, prev);
                    if (st == 14) me_store(prev, meb);
                    if (st == 15) epi2_stage(1, opk);
                    if (st == 18) epi2_store(1, prev);
                }
#pragma unroll
                for (int m = 0; m < 4; ++m) {
                    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);   // 1 MFMA
                    __builtin_amdgcn_sched_group_barrier(0x002, 4, 0);   // up to 4 VALU
                }
                __builtin_amdgcn_sched_barrier(0);
            }
        }
        STAMP(1)

        // ---- phase B: epilogue 1 (relu(u) -> bf16 B fragments, u > 0 bits) with GEMM 2 ----
#pragma unroll
        for (int q2 = 0; q2 < 4; ++q2)
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const float4 b4 = *reinterpret_cast<const float4*>(&BIAS[C + 32 * q2 + 8 * g + 4 * h]);
                acc2[q2][4 * g + 0] = b4.x; acc2[q2][4 * g + 1] = b4.y;
                acc2[q2][4 * g + 2] = b4.z; acc2[q2][4 * g + 3] = b4.w;
            }
        uint4 vf[4][2];
        uint32_t mub[4];
        auto epi1a = [&](int q) {      // relu(u) -> bf16 B fragments (bias is in the accumulator)
            uint32_t pk[8];
#pragma unroll
            for (int k = 0; k < 8; ++k) pk[k] = relu2(pack2(acc[q][2 * k], acc[q][2 * k + 1]));
            vf[q][0] = make_uint4(pk[0], pk[1], pk[2], pk[3]);
            vf[q][1] = make_uint4(pk[4], pk[5], pk[6], pk[7]);
        };
        auto epi1b = [&](int q) {      // u > 0 bits
            const uint32_t pk[8] = {vf[q][0].x, vf[q][0].y, vf[q][0].z, vf[q][0].w,
                                    vf[q][1].x, vf[q][1].y, vf[q][1].z, vf[q][1].w};
            mub[q] = pos_bits16(pk);
        };
        {
            // steps 0-1: identity x e_l (the residual; B = this wave's own rows), steps 2-9:
            // W_r^T (A from LDS) x relu(u) (B in registers); fragments fetched one step ahead.
            // Epilogue 1 of tile q runs under the two steps before the first one that needs it.
            auto fetch = [&](int st, uint4 (&f)[4]) {
#pragma unroll
                for (int q2 = 0; q2 < 4; ++q2)
                    f[q2] = st >= 2 ? WRL[(q2 * 8 + (st - 2)) * 64 + lane]
                                    : lds16(xb + RSB + (2 * q2 + st) * 32);
            };
            uint4 fr[2][4];
            fetch(0, fr[0]);
#pragma unroll
            for (int st = 0; st < 10; ++st) {
                if (st + 1 < 10) fetch(st + 1, fr[(st + 1) & 1]);
                if (st < 2) {
#pragma unroll
                    for (int q2 = 0; q2 < 4; ++q2) acc2[q2] = mfma_bf16(idf[st], fr[st & 1][q2], acc2[q2]);
                } else {
                    const int k = st - 2;
#pragma unroll
                    for (int q2 = 0; q2 < 4; ++q2) acc2[q2] = mfma_bf16(fr[st & 1][q2], vf[k >> 1][k & 1], acc2[q2]);
                }
                // epilogue 1 of tile q: part a at step 2q - 2, part b at step 2q - 1 (q = 0
                // under the identity steps); the mask store after the last one
                if (st < 8) {
                    const int q = st / 2;
                    if (st % 2 == 0) epi1a(q); else epi1b(q);
                }
                if (st == 8)   // u > 0 bits by this layer's position: lane (r, h) -> words [h][0..3]
                    *reinterpret_cast<uint2*>(a.mu + ((size_t)cu.b * a.T + cu.p0 + c) * 8 + 4 * h) =
                        make_uint2(mub[0] | (mub[1] << 16), mub[2] | (mub[3] << 16));
#pragma unroll
                for (int m = 0; m < 4; ++m) {
                    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                    __builtin_amdgcn_sched_group_barrier(0x002, 5, 0);
                }
                __builtin_amdgcn_sched_barrier(0);
            }
        }
        STAMP(2)
        prev = cu;
        ++it;
    };

    int tile = blockIdx.x;
    if (tile < ntiles) {
        body(std::integral_constant<bool, false>{}, tile);
        for (tile += gridDim.x; tile < ntiles; tile += gridDim.x)
            body(std::integral_constant<bool, true>{}, tile);
        // drain: epilogue 2 of the last tile
        uint4 opk[2][2];
        uint32_t meb[4];
#pragma unroll
        for (int rho = 0; rho < 2; ++rho) {
#pragma unroll
            for (int j = 0; j < 2; ++j) epi2_chunk(acc2[2 * rho + j], opk[j], meb[2 * rho + j]);
            epi2_stage(rho, opk);
            epi2_store(rho, prev);
        }
        me_store(prev, meb);
    }
    STAMP_FLUSH(a.stamps)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

int g_cus = 0;

}  // namespace

int cw::num_cus() {
    if (!g_cus) {
        int dev = 0;
        (void)hipGetDevice(&dev);
        (void)hipDeviceGetAttribute(&g_cus, hipDeviceAttributeMultiprocessorCount, dev);
        if (g_cus <= 0) g_cus = 256;
    }
    return g_cus;
}

void launch_block_fwd_c(const FwdArgsC& a, hipStream_t s) {
    const int nt = a.B * (a.T / TMB);
    const dim3 grid(std::min(nt, cw::num_cus()));
    Layout ly;
    if (pick_layout(a.n, ly)) hipLaunchKernelGGL(k_block_fwd_c<true>, grid, dim3(FT), 0, s, a, ly);
    else hipLaunchKernelGGL(k_block_fwd_c<false>, grid, dim3(FT), 0, s, a, ly);
}

}  // namespace ast
