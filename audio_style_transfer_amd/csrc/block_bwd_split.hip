// Split-fp16 encoder block backward (precision 2): d loss / d e_l for one block of
// model.py:95-116, restated by oracle/astyle_oracle.py:171-189 (encoder_backward):
//   tot = d loss / d e_{l+1} (the chain, its own direct loss term included)
//   g_u = [u > 0] (W_r tot)                         1x1 conv transposed
//   g_a = sum_k W_d[k] g_u(p - k + 1)                K = 3 SAME dilated conv transposed, in
//                                                    time_to_batch positions (masked.py:110-160)
//   out = tot + [e_l > 0] g_a + D_l                  D_l: direct loss gradient of e_l, if tapped
// fp32 storage, split fp16 operands on v_mfma_f32_32x32x16_f16, fp32 accumulation and
// epilogue (splitwave.h).
//
// One workgroup per CU (wave w owns channels 32 w .. 32 w + 31), persistent over tiles of 64
// positions.  A tile's tot rows are DMA'd into an LDS slot and converted there, in place, to
// split tot (2^m_t, m_t from the clip's max |tot|) under the previous tile's step 2; two slots
// alternate.  Per tile i:
//   T       barrier
//   step 1  g_v = W_r tot for the tile columns (+ the two halo rows of one-segment layouts),
//           its 8 k-steps issuing tile i+1's tot-row and mask-word DMA; g_u = [u > 0] g_v 2^m_u
//           -> split g_u image (m_u from the bound |g_v| <= wrn max|tot|: no cross-wave
//           exchange), barrier
//   step 2  g_a = 3 taps x 8 k-blocks x 2 column tiles x 3 products; steps 0..8 issue tile
//           i's D_l DMA; after step 13: wait for tile i+1's rows + barrier, then steps 14..23
//           carry their in-place conversion; D_l landed + barrier
//   epi     out = tot (fp32, loaded before step 2) + [e_l > 0] g_a + D_l -> HBM; max |out|
//           -> the clip's atomic max
// Only DMA reads global memory (the compiler never waits on an in-flight DMA it cannot see).
#include "splitwave.h"
#include <algorithm>

namespace ast {
namespace {
using namespace sw;

constexpr int MSLOT = 3 * 1024;   // mask words per tile (u16 index): u > 0 [64][8] at 0, e_l > 0
                                  // [64][8] at 512, halo u > 0 [2][8] at 1024

// D_l rows: LDS row c = tile column c (64 rows, stride RS), 9 one-KiB groups per wave; unmasked
// layouts issue in the saddr form (tile base + a constant per-lane offset, rows past the tile
// re-read column 0's row)
template <bool MASKED>
struct ColDma {
    uint32_t off[DPW];
    int srow[DPW], schk[DPW];
    bool real[DPW];
    __device__ __forceinline__ void init(int w, int lane, const Layout& ly, int d) {
#pragma unroll
        for (int j = 0; j < DPW; ++j) {
            const int o = (w + 4 * j) * 1024 + lane * 16;
            const int L = o / RS, qc = (o - L * RS) >> 4;
            srow[j] = L;
            schk[j] = qc < 32 ? qc : 0;
            real[j] = L < TMS;
            off[j] = (MASKED || !real[j]) ? 0u : (uint32_t)((row_toff(frow(L, ly), ly, d) * C + schk[j] * 4) * 4);
        }
    }
    __device__ __forceinline__ void issue(int j, const float* src, const Tile& t, const float* zero,
                                          uint32_t lds0, int T, int n, int d) const {
        if (!MASKED) {
            dma16s(src + ((size_t)t.b * T + t.tb) * C, off[j], lds0 + j * 4096);
            return;
        }
        const float* p = zero;
        if (real[j]) {
            const int pp = t.p0 + srow[j];
            p = src + ((size_t)t.b * T + (pp % n) * d + pp / n) * C + schk[j] * 4;
        }
        dma16(p, lds0 + j * 4096);
    }
};

template <bool MASKED, bool ONESEG, bool HAS_D>
__global__ void __launch_bounds__(FT, 1) k_block_bwd_s(BwdArgsS a, Layout ly) {
    __shared__ __attribute__((aligned(16))) uint8_t XS[2][SLOT];    // tot images (fp32 -> split)
    __shared__ __attribute__((aligned(16))) uint8_t XG[SLOT];       // split g_u image
    __shared__ __attribute__((aligned(16))) uint8_t XD[SLOT];       // fp32 D_l rows (row = column)
    __shared__ __attribute__((aligned(16))) uint8_t MK[2][MSLOT];   // mask words
    __shared__ __attribute__((aligned(16))) uint8_t SCR[1024];      // wave 3's dummy mask group

    const int tiles = a.T / TMS;
    const int ntiles = a.B * tiles;
    const int tid = threadIdx.x, lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int r = lane & 31, h = lane >> 5;
    const uint32_t padb = MASKED ? 0u : pad_bits(ly, w, lane);   // pad rows of the pairs converted

    auto tile_of = [&](int tl) { return tile_at<MASKED>(tl, tiles, a.n, a.d, ly); };
    RowDma<MASKED> dma;
    dma.init(w, lane, ly, a.d);
    ColDma<MASKED> ddma;
    if (HAS_D) ddma.init(w, lane, ly, a.d);
    // tot rows + mask words of tile tl into slot s: wave 0 the u > 0 words of the 64 columns,
    // wave 1 the e_l > 0 words, wave 2 the halo u > 0 words (lanes 0, 1), wave 3 a dummy group
    auto issue_masks = [&](const Tile& t, int s) {
        const uint16_t* src = (const uint16_t*)a.zero;
        uint32_t dst = (uint32_t)(uintptr_t)&SCR[0];
        const size_t cb = (size_t)t.b * a.T;
        if (w == 0) src = a.mu + (cb + t.p0 + lane) * 8;
        else if (w == 1) src = a.me + (cb + t.p0 + lane) * 8;
        else if (w == 2) {
            const int p = lane == 0 ? t.p0 - 1 : t.p0 + TMS;
            if (ONESEG && lane < 2 && p >= 0 && p < a.T) src = a.mu + (cb + p) * 8;
        }
        if (w < 3) dst = (uint32_t)(uintptr_t)&MK[s][w * 1024];
        dma16(src, dst);
    };
    if (blockIdx.x < ntiles) {
        const Tile t = tile_of(blockIdx.x);
        dma.aim(a.tin, t, ly, a.T, a.n, a.d);
        const uint32_t lds0 = (uint32_t)(uintptr_t)&XS[0][0] + (uint32_t)(w * 1024);
#pragma unroll
        for (int j = 0; j < DPW; ++j) dma.issue(j, a.tin, a.zero, lds0, a.T, a.n, a.d);
        issue_masks(t, 0);
    }

    // this wave's split weight halves (A: rows = channels 32 w.., K = the other side's channels)
    uint4 wr[8][2], wd[3][8][2];
#pragma unroll
    for (int kb = 0; kb < 8; ++kb)
#pragma unroll
        for (int hl = 0; hl < 2; ++hl)
            wr[kb][hl] = a.wrb[((size_t)(w * 8 + kb) * 2 + hl) * 64 + lane];
#pragma unroll
    for (int tp = 0; tp < 3; ++tp)
#pragma unroll
        for (int kb = 0; kb < 8; ++kb)
#pragma unroll
            for (int hl = 0; hl < 2; ++hl)
                wd[tp][kb][hl] = a.wdb[((size_t)((w * 3 + tp) * 8 + kb) * 2 + hl) * 64 + lane];
    pin_all(wd, wr);
    // the g_u image's pad / unused halo rows stay zero (only column and halo rows are written)
    for (int i = tid; i < SLOT / 16; i += FT) reinterpret_cast<uint4*>(XG)[i] = make_uint4(0, 0, 0, 0);

    int Lc[2], toff[2];
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        Lc[j] = frow(32 * j + r, ly);
        toff[j] = MASKED ? 0 : row_toff(Lc[j], ly, a.d);
    }
    const int chb = 32 * w + 4 * h;
    auto ctime = [&](const Tile& t, int cc, int to) { return col_time<MASKED>(t, cc, to, a.n, a.d); };
    // the halo column tile: lane r == 0 -> image row 0 (p0 - 1), r == 1 -> row 65 (p0 + 64)
    const int Lh = r == 1 ? TMS + 1 : 0;

    if (blockIdx.x < ntiles) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        lds_barrier();
        const Tile t0 = tile_of(blockIdx.x);
        const float s0 = exp2i(scale_exp(sload(a.gmax_in + t0.b)));
        const uint32_t z0 = zero_bits<MASKED>(padb, t0, ly, a.n, w, lane);
#pragma unroll
        for (int k = 0; k < NCONV; ++k) {
            const int p = conv_pair(w, k);
            pair_write<false>(&XS[0][0], p, pair_read(&XS[0][0], p, lane), conv_scale(z0, k, s0), lane);
        }
    }

    int it = 0;
    STAMP_DECL
    for (int tile = blockIdx.x; tile < ntiles; tile += gridDim.x, ++it) {
        const int cur = it & 1;
        const Tile cu = tile_of(tile);
        const int ntile = tile + (int)gridDim.x;
        const bool has_next = ntile < ntiles;
        // T: every wave is done with the previous tile (other slot, D rows, g_u image)
        lds_barrier();
        STAMP(6)
        const Tile nt = tile_of(has_next ? ntile : tile);
        dma.aim(a.tin, nt, ly, a.T, a.n, a.d);
        const uint32_t zn = zero_bits<MASKED>(padb, nt, ly, a.n, w, lane);
        const uint32_t ldsn = (uint32_t)(uintptr_t)&XS[cur ^ 1][0] + (uint32_t)(w * 1024);
        const uint32_t ldsd = (uint32_t)(uintptr_t)&XD[0] + (uint32_t)(w * 1024);

        const float gm = sload(a.gmax_in + cu.b);
        const int m_t = scale_exp(gm);
        const int m_u = scale_exp(a.wrn * gm);
        const float s_next = has_next ? exp2i(scale_exp(sload(a.gmax_in + nt.b))) : 0.f;
        const uint8_t* xs = &XS[cur][0];
        uint8_t* xn = &XS[cur ^ 1][0];
        const uint16_t* mk = reinterpret_cast<const uint16_t*>(&MK[cur][0]);

        bool ok0[2] = {true, true}, ok2[2] = {true, true};
        if (MASKED) {
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                const int m = (cu.p0 + 32 * j + r) % a.n;
                ok0[j] = m > 0;
                ok2[j] = m < a.n - 1;
            }
        }

        // ---- step 1: g_v = W_r tot (columns, halo rows), g_u = [u > 0] g_v -> g_u image ----
        f32x16 acc[2], acch;
#pragma unroll
        for (int i = 0; i < 16; ++i) { acc[0][i] = 0.f; acc[1][i] = 0.f; acch[i] = 0.f; }
        {
            uint4 bh[2][3], bl[2][3];
            auto bload = [&](int kb, uint4 (&xh)[3], uint4 (&xl)[3]) {
#pragma unroll
                for (int j = 0; j < (ONESEG ? 3 : 2); ++j) {
                    const uint8_t* p = xs + (j < 2 ? Lc[j] : Lh) * RS + kb * 32 + h * 16;
                    xh[j] = lds16(p);
                    xl[j] = lds16(p + 256);
                }
            };
            bload(0, bh[0], bl[0]);
#pragma unroll
            for (int kb = 0; kb < 8; ++kb) {
                const int cb = kb & 1;
                // step order (step_schedule): first MFMA, DMA + next reads, the rest
                acc[0] = mfma_f16(wr[kb][0], bh[cb][0], acc[0]);
                // tile i+1's rows and mask words into the other slot (the last tile re-reads
                // itself there: unused, and the count of vector-memory ops stays fixed)
                dma.issue(kb, a.tin, a.zero, ldsn, a.T, a.n, a.d);
                if (kb == 7) {
                    dma.issue(8, a.tin, a.zero, ldsn, a.T, a.n, a.d);
                    issue_masks(nt, cur ^ 1);
                }
                if (kb + 1 < 8) bload(kb + 1, bh[cb ^ 1], bl[cb ^ 1]);
                acc[0] = mfma_f16(wr[kb][1], bh[cb][0], acc[0]);
                acc[0] = mfma_f16(wr[kb][0], bl[cb][0], acc[0]);
                acc[1] = mfma3(wr[kb][0], wr[kb][1], bh[cb][1], bl[cb][1], acc[1]);
                if (ONESEG) acch = mfma3(wr[kb][0], wr[kb][1], bh[cb][2], bl[cb][2], acch);
                step_schedule();
            }
        }
        {
            const float f = exp2i(m_u - m_t - a.kr);   // acc units 2^(m_t + k_r) -> g_u 2^m_u
            auto put = [&](f32x16& v, int row) {
#pragma unroll
                for (int g = 0; g < 4; ++g) {
                    uint2 hi, lo;
                    split4(v[4 * g] * f, v[4 * g + 1] * f, v[4 * g + 2] * f, v[4 * g + 3] * f, hi, lo);
                    uint8_t* p = XG + row * RS + 2 * (chb + 8 * g);
                    *reinterpret_cast<uint2*>(p) = hi;
                    *reinterpret_cast<uint2*>(p + 256) = lo;
                }
            };
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                apply_mask(acc[j], mk[(32 * j + r) * 8 + 4 * h + w]);
                put(acc[j], Lc[j]);
            }
            if (ONESEG) {
                apply_mask(acch, mk[1024 + r * 8 + 4 * h + w]);   // lanes r >= 2: unused
                if (r < 2) put(acch, Lh);
            }
        }
        lds_barrier();     // g_u image complete
        STAMP(7)
        // tot in fp32 for the epilogue, this lane's accumulator elements (in flight during step 2)
        float4 tv[2][4];
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const float* src = a.tin + ((size_t)cu.b * a.T + ctime(cu, 32 * j + r, toff[j])) * C + chb;
#pragma unroll
            for (int g = 0; g < 4; ++g) tv[j][g] = *reinterpret_cast<const float4*>(src + 8 * g);
        }

        // ---- step 2: g_a = sum_k W_d[k] g_u(p - k + 1), next tile converted ----
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int i = 0; i < 16; ++i) acc[j][i] = 0.f;
        {
            uint4 bh[2][2], bl[2][2];
            auto bload = [&](int st, uint4 (&xh)[2], uint4 (&xl)[2]) {
                const int tp = st >> 3, kb = st & 7;
#pragma unroll
                for (int j = 0; j < 2; ++j) {
                    const uint8_t* p = XG + (Lc[j] + 1 - tp) * RS + kb * 32 + h * 16;
                    xh[j] = lds16(p);
                    xl[j] = lds16(p + 256);
                    if (MASKED && ((tp == 0 && !ok2[j]) || (tp == 2 && !ok0[j]))) {
                        xh[j] = make_uint4(0, 0, 0, 0);
                        xl[j] = xh[j];
                    }
                }
            };
            float4 cv[2];
            bload(0, bh[0], bl[0]);
#pragma unroll
            for (int st = 0; st < 24; ++st) {
                const int tp = st >> 3, kb = st & 7, cb = st & 1;
                if (st == 14) {
                    // the next tile's rows / masks have landed (younger: the 8 tot loads and
                    // this tile's 9 D_l groups; vmcnt retires in issue order)
                    if (HAS_D) asm volatile("s_waitcnt vmcnt(17)" ::: "memory");
                    else asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
                    lds_barrier();
                }
                // step order (step_schedule): first MFMA; D_l DMA group, next reads (+ the
                // conversion's pair read); the rest with the conversion of the pair read before
                acc[0] = mfma_f16(wd[tp][kb][0], bh[cb][0], acc[0]);
                if (HAS_D && st < DPW) ddma.issue(st, a.dadd, cu, a.zero, ldsd, a.T, a.n, a.d);
                if (st + 1 < 24) bload(st + 1, bh[cb ^ 1], bl[cb ^ 1]);
                if (st >= 14) {
                    // row pair k = st - 14 read here, converted and written one step later (the
                    // last tile converts its stale other slot: unused, branch-free)
                    const int k = st - 14;
                    if (k < NCONV) cv[k & 1] = pair_read(xn, conv_pair(w, k), lane);
                    if (k > 0)
                        pair_write<false>(xn, conv_pair(w, k - 1), cv[(k - 1) & 1],
                                       conv_scale(zn, k - 1, s_next), lane);
                }
                acc[0] = mfma_f16(wd[tp][kb][1], bh[cb][0], acc[0]);
                acc[0] = mfma_f16(wd[tp][kb][0], bl[cb][0], acc[0]);
                acc[1] = mfma3(wd[tp][kb][0], wd[tp][kb][1], bh[cb][1], bl[cb][1], acc[1]);
                step_schedule();
            }
        }
        STAMP(8)
        if (HAS_D) {   // this tile's D_l rows have landed
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            lds_barrier();
        }
#ifdef ASTYLE_STAMPS
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // diagnostic: + the tot loads' wait
#endif
        STAMP(12)

        // ---- epilogue: out = tot + [e_l > 0] g_a + D_l ----
        {
            const float inv2 = exp2i(-(m_u + a.kd));
            float omax = 0.f;
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                const int c = 32 * j + r;
                apply_mask(acc[j], mk[512 + c * 8 + 4 * h + w]);
                const int t = ctime(cu, c, toff[j]);
                const uint8_t* df = XD + c * RS + 4 * chb;
                float* dst = a.gout + ((size_t)cu.b * a.T + t) * C + chb;
#pragma unroll
                for (int g = 0; g < 4; ++g) {
                    float4 o;
                    o.x = fmaf(acc[j][4 * g + 0], inv2, tv[j][g].x);
                    o.y = fmaf(acc[j][4 * g + 1], inv2, tv[j][g].y);
                    o.z = fmaf(acc[j][4 * g + 2], inv2, tv[j][g].z);
                    o.w = fmaf(acc[j][4 * g + 3], inv2, tv[j][g].w);
                    if (HAS_D) {
                        const float4 dv = *reinterpret_cast<const float4*>(df + 32 * g);
                        o.x += dv.x; o.y += dv.y; o.z += dv.z; o.w += dv.w;
                    }
                    *reinterpret_cast<float4*>(dst + 8 * g) = o;
                    omax = fmaxf(omax, fmaxf(fmaxf(fabsf(o.x), fabsf(o.y)), fmaxf(fabsf(o.z), fabsf(o.w))));
                }
            }
            omax = wave_max(omax);
            if (lane == 0) atomicMax(a.gmax_out + cu.b, __float_as_uint(omax));
        }
        STAMP(9)
    }
    STAMP_FLUSH(a.stamps)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// max |x| over each clip's n elements -> out[b] (atomic max of the float bits)
__global__ void __launch_bounds__(256) k_absmax(const float* __restrict__ x, size_t n, int chunks,
                                                unsigned* __restrict__ out) {
    const int b = blockIdx.x / chunks, ch = blockIdx.x - b * chunks;
    const size_t len = n / chunks;
    const float4* p = reinterpret_cast<const float4*>(x + (size_t)b * n + (size_t)ch * len);
    float m = 0.f;
    for (size_t i = threadIdx.x; i < len / 4; i += 256) {
        const float4 v = p[i];
        m = fmaxf(m, fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w))));
    }
    m = wave_max(m);
    if ((threadIdx.x & 63) == 0) atomicMax(out + b, __float_as_uint(m));
}

}  // namespace

void launch_block_bwd_s(const BwdArgsS& a, hipStream_t s) {
    const int nt = a.B * (a.T / TMS);
    const dim3 grid(std::min(nt, sw::num_cus()));
    Layout ly;
    const bool masked = pick_layout(a.n, ly);
    const bool oneseg = !masked && ly.M == TMS;
#define BWD_LAUNCH(M, O, D) hipLaunchKernelGGL((k_block_bwd_s<M, O, D>), grid, dim3(FT), 0, s, a, ly)
    if (masked) { if (a.dadd) BWD_LAUNCH(true, false, true); else BWD_LAUNCH(true, false, false); }
    else if (oneseg) { if (a.dadd) BWD_LAUNCH(false, true, true); else BWD_LAUNCH(false, true, false); }
    else { if (a.dadd) BWD_LAUNCH(false, false, true); else BWD_LAUNCH(false, false, false); }
#undef BWD_LAUNCH
}

void launch_absmax(const float* x, size_t per_clip, int B, unsigned* out, hipStream_t s) {
    int chunks = 1;
    while (chunks < 64 && per_clip % ((size_t)chunks * 8) == 0 && per_clip / (chunks * 2) >= 4096) chunks *= 2;
    hipLaunchKernelGGL(k_absmax, dim3(B * chunks), dim3(256), 0, s, x, per_clip, chunks, out);
}

}  // namespace ast
