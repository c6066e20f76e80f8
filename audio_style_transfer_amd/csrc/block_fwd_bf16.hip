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
//    position, so the backward applies them with no bit shuffling (block_bwd in
//    encoder_bf16.hip).
#include "common.h"
#include <algorithm>
#include <type_traits>

namespace ast {
namespace {

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

constexpr int FT = 256;                  // threads: one wave per SIMD
constexpr int RSB = 272;                 // image row stride (bytes)
constexpr int FROWS = TMB + 8;           // max image rows (4 segments of 32 + 2 pads each)
constexpr int NDMA = (FROWS * RSB + 1023) / 1024;   // 37 one-KiB groups per image
constexpr int BUFB = NDMA * 1024;        // bytes per image
// The DMA fills groups 0..35 (9 per wave, no per-wave tail branch); group 36 holds only the
// last 128 B of row 135, which is a zero pad row of the 32-row segment layout (and unused by the
// others): it is zeroed once at kernel start and never written again.
constexpr int DPW = 9;
static_assert(4 * DPW * 1024 >= 135 * RSB + 128 && 4 * DPW * 1024 < FROWS * RSB,
              "DMA groups must cover every image row but the tail of row 135");
constexpr int SRB = 144;                 // staging row stride: one 128-B half row + 16 pad

struct FLayout {           // uniform per launch (see pick_flayout)
    int M;                 // segment length; TMB = one segment with two halo rows
    int nrows;             // image rows
};

__device__ __forceinline__ int frow(int c, const FLayout& ly) {   // image row of column c
    return (c / ly.M) * (ly.M + 2) + 1 + (c % ly.M);
}

// time offset of image row L from the tile's base time (unmasked layouts):
//   one segment: rows are positions p0-1 .. p0+128 of one sub-sequence, t = tb + (L-1) d
//   segments of M = n: row (s, k) is position k-1 of sub-sequence j0 + s, t = tb + (k-1) d + s
__device__ __forceinline__ int row_toff(int L, const FLayout& ly, int d) {
    if (ly.M == TMB) return (L - 1) * d;
    const int s = L / (ly.M + 2), k = L - s * (ly.M + 2);
    return (k - 1) * d + s;
}

__device__ __forceinline__ uint4 relu8(uint4 v) {
    return make_uint4(relu2(v.x), relu2(v.y), relu2(v.z), relu2(v.w));
}

__device__ __forceinline__ uint4 lds16(const uint8_t* p) { return *reinterpret_cast<const uint4*>(p); }

// 16 B per lane HBM -> LDS at lds_base + 16 * lane (global_load_lds_dwordx4).  Inline asm so the
// compiler neither counts it nor drains it with vmcnt(0) before unrelated LDS reads: the kernel
// waits for it explicitly (cdna_hip_programming.md §5.7).
__device__ __forceinline__ void dma16(const void* src, uint32_t lds_base) {
    uint32_t keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
                 "global_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(src), "s"(lds_base) : "memory");
}

template <bool MASKED>
__global__ void __launch_bounds__(FT, 1) k_block_fwd_c(FwdArgsC a, FLayout ly) {
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
    // taps 0 and 2 live in the accumulator register file (MFMA A operands may be AGPRs): the
    // arch VGPRs stay free for accumulators, fragments and addresses.  Plain loads (the compiler
    // counts them), then a tied no-op asm that pins each fragment to AGPRs.
    uint4 wr0[4][8], wr2[4][8];
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int kb = 0; kb < 8; ++kb) {
            const uint4 v0 = *reinterpret_cast<const uint4*>(a.wf + ((size_t)((0 * 4 + q) * 8 + kb) * 64 + lane) * 8);
            const uint4 v2 = *reinterpret_cast<const uint4*>(a.wf + ((size_t)((2 * 4 + q) * 8 + kb) * 64 + lane) * 8);
            u32x4 t0 = __builtin_bit_cast(u32x4, v0), t2 = __builtin_bit_cast(u32x4, v2);
            asm volatile("" : "=a"(t0) : "0"(t0));
            asm volatile("" : "=a"(t2) : "0"(t2));
            wr0[q][kb] = __builtin_bit_cast(uint4, t0);
            wr2[q][kb] = __builtin_bit_cast(uint4, t2);
        }
    for (int i = tid; i < 4 * 8 * 64; i += FT) {
        W1[i] = *reinterpret_cast<const uint4*>(a.wf + ((size_t)4 * 8 * 64 + i) * 8);
        WRL[i] = *reinterpret_cast<const uint4*>(a.wrf + (size_t)i * 8);
    }
    if (tid < C) { BIAS[tid] = a.bd[tid]; BIAS[C + tid] = a.br[tid]; }
    if (tid < 2 * 64)   // group 36 of both images (see DPW)
        *reinterpret_cast<uint4*>(&XS[tid >> 6][4 * DPW * 1024 + (tid & 63) * 16]) = make_uint4(0, 0, 0, 0);
    // identity A fragments: element e of lane (r, h) is 1 iff r == 16 sg + 8 h + e
    uint4 idf[2];
#pragma unroll
    for (int sg = 0; sg < 2; ++sg) {
        const int e = r - 16 * sg - 8 * h;
        uint32_t dw[4];
#pragma unroll
        for (int k = 0; k < 4; ++k)
            dw[k] = (e == 2 * k ? 0x3f80u : 0u) | (e == 2 * k + 1 ? 0x3f800000u : 0u);
        idf[sg] = make_uint4(dw[0], dw[1], dw[2], dw[3]);
    }

    const int c = 32 * w + r;                  // this lane's tile column
    const int Lc = frow(c, ly);
    const int tcoff = MASKED ? 0 : row_toff(Lc, ly, a.d);

    // DMA slots: group g = w + 4 j covers image bytes [1024 g, 1024 g + 1024); this lane's
    // 16 B land at row L, chunk qc (qc == 16: the pad slot, filled from chunk 0)
    int soff[DPW];       // source element offset from the tile's base row (unmasked layouts)
    int scls[DPW];       // source class: 0 row, 1 zero, 2 left halo, 3 right halo
    int srow[DPW], schk[DPW];
#pragma unroll
    for (int j = 0; j < DPW; ++j) {
        const int g = w + 4 * j;
        const int o = g * 1024 + lane * 16;
        const int L = o / RSB, qc = (o - L * RSB) >> 4;
        const int ch = qc < 16 ? qc : 0;
        srow[j] = L;
        schk[j] = ch;
        int cls = 0;
        if (L >= ly.nrows) cls = 1;
        else if (ly.M == TMB) cls = L == 0 ? 2 : (L == TMB + 1 ? 3 : 0);
        else {
            const int k = L % (ly.M + 2);
            cls = (k == 0 || k == ly.M + 1) ? 1 : 0;
        }
        scls[j] = cls;
        soff[j] = MASKED || cls == 1 ? 0 : row_toff(L, ly, a.d) * C + ch * 8;
    }
    __syncthreads();

    auto stage = [&](int tl, int buf) {          // DMA of a whole tile image (prologue)
        const int b = tl / tiles, p0 = (tl - b * tiles) * TMB;
        int m0 = 0, tb = 0;
        if (!MASKED) {
            if (ly.M == TMB) { m0 = p0 % a.n; tb = m0 * a.d + p0 / a.n; }
            else tb = p0 / a.n;
        }
        const uint32_t vmask = 1u | (!MASKED && ly.M == TMB && m0 > 0 ? 4u : 0u) |
                               (!MASKED && ly.M == TMB && m0 + TMB < a.n ? 8u : 0u);
        const uint32_t lds0 = (uint32_t)(uintptr_t)&XS[buf][0] + (uint32_t)(w * 1024);
#pragma unroll
        for (int j = 0; j < DPW; ++j) {
            const u16* src = a.zero;
            if (MASKED) {
                const int p = p0 + srow[j] - 1;
                if (scls[j] != 1 && p >= 0 && p < a.T)
                    src = a.ein + ((size_t)b * a.T + (p % a.n) * a.d + p / a.n) * C + schk[j] * 8;
            } else if ((vmask >> scls[j]) & 1u) {
                src = a.ein + ((size_t)b * a.T + tb) * C + soff[j];
            }
            dma16(src, lds0 + j * 4096);
        }
    };

    // staged output rows: piece k of a round is wave column 8 k + lane / 8
    int otoff[4];
#pragma unroll
    for (int k = 0; k < 4; ++k)
        otoff[k] = MASKED ? 0 : row_toff(frow(32 * w + 8 * k + (lane >> 3), ly), ly, a.d);
    uint8_t* stg = &STG[w][0];

    // ---- per-tile geometry ----------------------------------------------------------------
    struct Tile { int b, p0, tb; };
    auto tile_at = [&](int tl) {
        Tile t;
        t.b = tl / tiles;
        t.p0 = (tl - t.b * tiles) * TMB;
        t.tb = MASKED ? 0 : (ly.M == TMB ? (t.p0 % a.n) * a.d + t.p0 / a.n : t.p0 / a.n);
        return t;
    };
    auto col_time = [&](const Tile& t, int cc, int toff) {   // time of tile column cc
        if (MASKED) {
            const int p = t.p0 + cc;
            return (p % a.n) * a.d + p / a.n;
        }
        return t.tb + toff;
    };

    // ---- epilogue 2 pieces (run for the PREVIOUS tile while this tile's GEMM 1 runs) ------
    // chunk(q2): bf16 pack, e_{l+1} > 0 bits, half-wave swap (guide T21): afterwards lane (n, h)
    // holds 16-B chunks 4 q2 + 2 gp + h (gp = 0, 1) of row n
    auto e2_pack = [&](const f32x16& acc2q, uint32_t (&o)[8]) {
#pragma unroll
        for (int k = 0; k < 8; ++k) o[k] = pack2(acc2q[2 * k], acc2q[2 * k + 1]);
    };
    auto e2_swap = [&](const uint32_t (&o)[8], uint4 (&opk)[2]) {
#pragma unroll
        for (int gp = 0; gp < 2; ++gp) {
            const int g = 2 * gp;
            auto sx = __builtin_amdgcn_permlane32_swap(o[2 * g], o[2 * g + 2], false, false);
            auto sy = __builtin_amdgcn_permlane32_swap(o[2 * g + 1], o[2 * g + 3], false, false);
            opk[gp] = make_uint4(sx[0], sy[0], sx[1], sy[1]);
        }
    };
    auto epi2_chunk = [&](const f32x16& acc2q, uint4 (&opk)[2], uint32_t& mebq) {
        uint32_t o[8];
        e2_pack(acc2q, o);
        mebq = pos_bits16(o);
        e2_swap(o, opk);
    };
    // The staging rows are written and read by different lanes: a wave-scope fence keeps the
    // compiler from hoisting one lane's read above another lane's write (or sinking a write
    // above a read), which per-thread program order alone does not forbid.
    auto wave_fence = [] { __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront"); };
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
            const int tt = col_time(t, 32 * w + 8 * k + (lane >> 3), otoff[k]);
#ifndef ABL_NOSTORE
            *reinterpret_cast<uint4*>(a.eout + ((size_t)t.b * a.T + tt) * C + 64 * rho + (lane & 7) * 8) = v;
#else
            if (v.x == 0x12345u && tt < 0) *reinterpret_cast<uint4*>(a.eout) = v;
#endif
        }
    };
    auto me_store = [&](const Tile& t, const uint32_t (&meb)[4]) {
        if (a.me_next) {
            const int tc = col_time(t, c, tcoff);
            const int pn = (tc & ((1 << a.dn_log2) - 1)) * a.nn + (tc >> a.dn_log2);
            *reinterpret_cast<uint2*>(a.me_next + ((size_t)t.b * a.T + pn) * 8 + 4 * h) =
                make_uint2(meb[0] | (meb[1] << 16), meb[2] | (meb[3] << 16));
        }
    };

    stage(blockIdx.x, 0);
    f32x16 acc[4];                  // GEMM 1 accumulators
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
        const Tile cu = tile_at(tile);
        // this wave's DMA of the current image is complete (only the <= 10 stores of the
        // previous tile, issued after it, may still be in flight: vmcnt counts in issue order);
        // the barrier publishes every wave's part and retires all reads of the other image
        if (PREV) asm volatile("s_waitcnt vmcnt(9)" ::: "memory");
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
        const Tile nx = tile_at(ntl);
        const uint32_t lds0 = (uint32_t)(uintptr_t)&XS[cur ^ 1][0] + (uint32_t)(w * 1024);
        uint32_t vmask = 1u;
        if (!MASKED && ly.M == TMB) {
            const int m0 = nx.p0 % a.n;
            vmask |= (m0 > 0 ? 4u : 0u) | (m0 + TMB < a.n ? 8u : 0u);
        }
        const u16* nbase = a.ein + ((size_t)nx.b * a.T + nx.tb) * C;
        auto dma_slot = [&](int j) {
            const u16* src = a.zero;
            if (MASKED) {
                const int p = nx.p0 + srow[j] - 1;
                if (scls[j] != 1 && p >= 0 && p < a.T)
                    src = a.ein + ((size_t)nx.b * a.T + (p % a.n) * a.d + p / a.n) * C + schk[j] * 8;
            } else if ((vmask >> scls[j]) & 1u) {
                src = nbase + soff[j];
            }
            dma16(src, lds0 + j * 4096);
        };

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
                uint4 bv = relu8(bl[st % 3]);
                if (MASKED && ((tp == 0 && !ok0) || (tp == 2 && !ok2))) bv = make_uint4(0, 0, 0, 0);
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
                // steps 15-22) and the next tile's DMA (steps 0-7, 16, 17, where the steps carry
                // the fewest LDS reads).  The stores stay behind the last DMA (vmcnt(9) above).
#ifndef ABL_NODMA
                if (st < 4) { dma_slot(2 * st); dma_slot(2 * st + 1); }
                if (st == 4) dma_slot(8);
#endif
#ifndef ABL_NOEPI2
                if (PREV) {
                    // tile q2 = 0, 1 in steps 0-5, staged at 6, stored at 10; q2 = 2, 3 in steps
                    // 7-9 and 11-13, staged at 15, stored at 18
                    constexpr int qs[24] = {0, 0, 0, 1, 1, 1, -1, 2, 2, 2, -1, 3, 3, 3, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1};
                    constexpr int ph[24] = {0, 1, 2, 0, 1, 2, -1, 0, 1, 2, -1, 0, 1, 2, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1};
                    if (qs[st] >= 0) {
                        const int q2 = qs[st];
                        if (ph[st] == 0) e2_pack(acc2[q2], o2);
                        if (ph[st] == 1) meb[q2] = pos_bits16(o2);
                        if (ph[st] == 2) e2_swap(o2, opk[q2 & 1]);
                    }
                    if (st == 6) epi2_stage(0, opk);
                    if (st == 10) epi2_store(0, prev);
                    if (st == 14) me_store(prev, meb);
                    if (st == 15) epi2_stage(1, opk);
                    if (st == 18) epi2_store(1, prev);
                }
#endif
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

int g_cus_c = 0;
int num_cus_c() {
    if (!g_cus_c) {
        int dev = 0;
        (void)hipGetDevice(&dev);
        (void)hipDeviceGetAttribute(&g_cus_c, hipDeviceAttributeMultiprocessorCount, dev);
        if (g_cus_c <= 0) g_cus_c = 256;
    }
    return g_cus_c;
}

// Segment layout when a tile lies inside one sub-sequence (n % 128 == 0) or holds whole
// sub-sequences of >= 32 positions; otherwise one segment with per-column tap masks.
bool pick_flayout(int n, FLayout& ly) {
    if (n % TMB == 0) { ly.M = TMB; ly.nrows = TMB + 2; return false; }
    if (n < TMB && TMB % n == 0 && n >= 32) { ly.M = n; ly.nrows = (TMB / n) * (n + 2); return false; }
    ly.M = TMB; ly.nrows = TMB + 2;
    return true;
}

}  // namespace

void launch_block_fwd_c(const FwdArgsC& a, hipStream_t s) {
    const int nt = a.B * (a.T / TMB);
    const dim3 grid(std::min(nt, num_cus_c()));
    FLayout ly;
    if (pick_flayout(a.n, ly)) hipLaunchKernelGGL(k_block_fwd_c<true>, grid, dim3(FT), 0, s, a, ly);
    else hipLaunchKernelGGL(k_block_fwd_c<false>, grid, dim3(FT), 0, s, a, ly);
}

}  // namespace ast
