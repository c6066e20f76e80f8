// ASTYLE_MFMA16=1 (round 6): the forward block kernel of block_fwd_split.hip on
// v_mfma_f32_16x16x32_f16 fragments (splitwave.h "16x16x32"; the weights are packed for it when the
// knob is set).  Same structure, phases and numerics class; the K accumulation order differs, so
// results match the default kernels to fp32 rounding, not bit for bit.  Measured (DESIGN.md §3,
// round 6): 4-5 % slower per launch than the 32x32x16 default at equal data; kept as the
// measured alternative, not the default.
//
// Split-fp16 encoder block forward (precision 2): model.py:95-116 for one block,
//   u = dconv_d(relu(e_l)) + b_d        (masked.py:110-160, K = 3, SAME zero padding)
//   e_{l+1} = e_l + W_r^T relu(u) + b_r
// fp32 storage, v_mfma_f32_16x16x32_f16 on split fp16 operands (round 6; 32x32x16 before), fp32
// accumulation and fp32 epilogues (splitwave.h).
//
// One workgroup per CU (wave w owns output channels 32 w .. 32 w + 31), persistent over tiles
// of 64 positions, one wave per SIMD: every epilogue runs in the shadow of MFMAs.  The two
// 32-column halves j of a tile are separate MFMA phases, so the epilogue of one half overlaps
// the GEMM of the other.  A tile's e_l arrives in registers (rows: unit k = image rows 8 k ..
// 8 k + 7 x wave w's 32 channels, 8 cache lines per wave instruction), loaded during phases A
// and B of the previous tile, and is converted into the LDS image (split relu(e_l), scaled by
// 2^m_e from the clip's max |e_l|) and into the wave's quarter of a residual buffer (fp32 e_l,
// double-buffered, read back by the same wave only).  Per tile i:
//   T  barrier (image i complete)
//   A  GEMM 1, column half 0 (3 taps x 8 k-blocks x 3 products); carries epilogue 2 of tile
//      i-1 (8 units of 3 steps: e_i = e_{i-1} + y + b_r back into the residual rows, e > 0
//      bits, max |e|), the flush of its half 0 (residual rows -> HBM as whole lines) and the
//      row loads of tile i+1, units 0..4
//   B  GEMM 1, column half 1; carries epilogue 1 of half 0 (u = acc 2^-(m_e+k_d) + b_d, u > 0
//      bits, v = relu(u) 2^m_v -> split v image; m_v from the bound |u| <= wdn max|e_l| + bdm),
//      the flush of epilogue 2's half 1 and the row loads of units 5..8; barrier
//   C  GEMM 2 (8 k-blocks x 3 products), half 0; carries epilogue 1 of half 1; barrier
//   D  GEMM 2, half 1; carries the conversion of tile i+1 (image + residual)
// Round-2 measurements of this structure: ~13k cycles per tile against an MFMA
// floor of 6.2k; moving the loads / conversions between phases does not change the tile time.
// non-temporal (gfx950 CPol nt) row loads and e_{l+1} stores: every row streams through once, and
// the stores are whole 128-B lines (round 6: -1.0 % per launch from the stores, -0.4 % from the
// loads, profiles/r6_diag/block_ab.txt); -DSW_FWD_DEFAULT_POLICY (A/B builds) restores the default
#ifndef SW_FWD_DEFAULT_POLICY
#define SW_LD_AUX 2
#define SW_ST_AUX 2
#endif
#include "splitwave.h"
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <type_traits>

namespace ast {
namespace {
using namespace sw;

constexpr int IROWS = 72;             // image / residual rows: 66 or 68 used, 9 units x 8 rows
constexpr int ISLOT = IROWS * RS;     // bytes per image / residual buffer
constexpr int LA = 2;                 // B-fragment lookahead (steps)

// XIN (block 0, one-segment layout, d = 1): the rows of e_0 are recomputed from the audio
// (e0_val: three samples per row, W0 / b0 of the lane's four channels in registers) instead of
// loaded, so the start conv writes no e_0 tensor (model.py:82-93 folded into block 0)
template <bool MASKED, bool ONESEG, bool XIN>
__global__ void __launch_bounds__(FT, 1) k_block_fwd_s16(FwdArgsS a, Layout) {
    // the layout as compile-time constants (pick_layout: one segment or masked: M = 64 with two
    // halo rows; else segments of SEGM = 32 with their pad rows), not the launch argument
    constexpr bool GEO1 = ONESEG || MASKED;
    const Layout ly = {GEO1 ? TMS : SEGM, GEO1 ? TMS + 2 : (TMS / SEGM) * (SEGM + 2)};
    __shared__ __attribute__((aligned(16))) uint8_t IMG[ISLOT];     // split relu(e_l) image
    __shared__ __attribute__((aligned(16))) uint8_t ER[2][ISLOT];   // fp32 e_l (residual) rows
    __shared__ __attribute__((aligned(16))) uint8_t XV[TMS * RS];   // split v image
    __shared__ __attribute__((aligned(16))) float BIAS[2 * C];      // b_d, b_r
    __shared__ __attribute__((aligned(16))) float BDS[C];           // b_d 2^m_v (the current clip's v scale)
    __shared__ __attribute__((aligned(16))) uint16_t MBU[TMS * 8];  // u > 0 words of the tile
    __shared__ __attribute__((aligned(16))) uint16_t MBE[TMS * 8];  // e_{l+1} > 0 words
    __shared__ int MBT[TMS];                                        // time of each tile column
    __shared__ uint32_t WMX[4];                                     // the drain's per-wave maxima

    const int tiles = a.T / TMS;
    const int ntiles = a.B * tiles;
    const int tid = threadIdx.x, lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int i16 = lane & 15, q4 = lane >> 4;   // 16x16x32 fragment lane (splitwave.h)
    const int G = (int)gridDim.x;
    STAMP_DECL

    auto tile_of = [&](int tl) { return tile_at<MASKED>(tl, a.ft, a.fn, a.d, ly); };
    // tiles past the end repeat the last one (loaded and converted, never used)
    auto clampt = [&](int tl) { return tl < ntiles ? tl : ntiles - 1; };

    // this wave's split weight halves, resident in AGPRs for the whole launch: every load is
    // issued before the first pin (a pin right after its load would wait for it)
    uint4 wd[3][8][2], wr[8][2];
#pragma unroll
    for (int tp = 0; tp < 3; ++tp)
#pragma unroll
        for (int kb = 0; kb < 8; ++kb)
#pragma unroll
            for (int hl = 0; hl < 2; ++hl)
                wd[tp][kb][hl] = a.wdf[((size_t)((w * 3 + tp) * 8 + kb) * 2 + hl) * 64 + lane];
#pragma unroll
    for (int kb = 0; kb < 8; ++kb)
#pragma unroll
        for (int hl = 0; hl < 2; ++hl)
            wr[kb][hl] = a.wrf[((size_t)(w * 8 + kb) * 2 + hl) * 64 + lane];
    pin_all(wd, wr);
    if (tid < C) { BIAS[tid] = a.bd[tid]; BIAS[C + tid] = a.br[tid]; }

    // image row and time offset of the lane's column 16 cb + i16 of column half j
    int Lc[2][2], toff[2][2];
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int cb = 0; cb < 2; ++cb) {
            Lc[j][cb] = frow(32 * j + 16 * cb + i16, ly);
            toff[j][cb] = MASKED ? 0 : row_toff(Lc[j][cb], ly, a.d);
        }
    const int chq = 32 * w + 4 * q4;  // first channel of this lane's sub-tiles (+ 16 rb)
    const int mg0 = q4 >> 1;          // mask group of row block 0 (mgrp: + 2 rb); word h = q4 & 1
    auto ctime = [&](const Tile& t, int cc, int to) { return col_time<MASKED>(t, cc, to, a.fn, a.d); };

    // ---- row units: unit k, lane -> image row L = 8 k + lr, channels cq .. cq + 3 ----
    const int lr = lane >> 3;
    const int cq = 32 * w + 4 * (lane & 7);
    const uint32_t imgo = (uint32_t)(lr * RS + 2 * cq);   // + 8 k RS: split row bytes
    const uint32_t ero = (uint32_t)(lr * RS + 4 * cq);    // + 8 k RS: fp32 row bytes
    // unmasked layouts: byte offset of the unit's source row from the tile's row-0 source
    // (time tb - d); rows without a source (pad rows, rows past the image) read row 1 and are
    // zeroed (bit k of padz); one-segment halos (unit 0 row 0, unit 8 row 65) are decided per
    // tile.  Masked layouts: only rows past 65 are unused
    uint32_t soff[NU];
    uint32_t padz = 0;
#pragma unroll
    for (int k = 0; k < NU; ++k) {
        const int L = 8 * k + lr;
        const bool none = MASKED ? L > TMS + 1 : (L >= ly.nrows || pad_row(L, ly));
        if (none) padz |= 1u << k;
        soff[k] = MASKED ? 0u : (uint32_t)(((none ? 0 : row_toff(L, ly, a.d)) + a.d) * C * 4 + 4 * cq);
    }
    const uint32_t row1 = (uint32_t)(a.d * C * 4 + 4 * cq), row64 = (uint32_t)(TMS * a.d * C * 4 + 4 * cq);   // image row 64 (time tb + 63 d)

    float4 ld[NU];          // rows of the next tile to convert (XIN: x[t - 1], x[t], x[t + 1])
    uint32_t xedge = 0;     // XIN: bit k = unit k's row at t = 0, bit 16 + k: at t = T - 1
    float w0r[3][4], b0r[4];
    if (XIN) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            w0r[0][i] = a.w0[cq + i]; w0r[1][i] = a.w0[C + cq + i]; w0r[2][i] = a.w0[2 * C + cq + i];
            b0r[i] = a.b0[cq + i];
        }
    }
    auto load_unit = [&](const Tile& t, int k) {
        if (XIN) {
            // row L = time tb + L - 1 (d = 1); rows outside the clip are zeroed at conversion
            const int tt = min(max(t.tb + 8 * k + lr - 1, 0), a.T - 1);
            const float* xr = a.xin + (size_t)t.b * a.T;
            ld[k] = make_float4(xr[max(tt - 1, 0)], xr[tt], xr[min(tt + 1, a.T - 1)], 0.f);
            xedge = (xedge & ~(0x10001u << k)) | (tt == 0 ? 1u << k : 0u) | (tt == a.T - 1 ? 0x10000u << k : 0u);
            return;
        }
        if (MASKED) {
            const int L = 8 * k + lr;
            // row L = position p0 + L - 1, clamped into the clip (rows 0 / 65 are real
            // neighbours when the tile starts / ends inside a sub-sequence; the tap masks of
            // gemm1h drop the ones outside a column's sub-sequence)
            const int pp = (padz >> k) & 1u ? t.p0 : min(max(t.p0 + L - 1, 0), a.T - 1);
            const float* src = a.ein + ((size_t)t.b * a.T + pos_time(pp, a.fn, a.d)) * C + cq;
            ld[k] = *reinterpret_cast<const float4*>(src);
            return;
        }
        // through a buffer resource at the tile's row-0 source: 32-bit lane offsets, no 64-bit
        // address arithmetic per unit
        const rsrc_t rs = mk_rsrc(a.ein + ((ptrdiff_t)t.b * a.T + t.tb - a.d) * C);
        uint32_t o = soff[k];
        if (ONESEG && k == 0 && lr == 0 && t.m0 == 0) o = row1;
        if (ONESEG && k == NU - 1 && lr == 1 && t.m0 + TMS >= a.n) o = row64;
        ld[k] = bld4(rs, o, 0u);
    };
    auto zero_bits_of = [&](const Tile& t) {
        uint32_t z = padz;
        if (ONESEG) {
            if (lr == 0 && t.m0 == 0) z |= 1u;
            if (lr == 1 && t.m0 + TMS >= a.n) z |= 1u << (NU - 1);
        }
        return z;
    };
    // conversion of unit k: raw fp32 -> residual buffer er; relu, scale, split -> image
    auto conv_unit = [&](int k, uint8_t* er, float s, uint32_t zb) {
        float4 v = ld[k];
        if (XIN) {   // e_0 of the lane's four channels (x[-1] = x[T] = 0)
            const float xm = (xedge >> k) & 1u ? 0.f : v.x, x0 = v.y, xp = (xedge >> (16 + k)) & 1u ? 0.f : v.z;
            v.x = e0_val(w0r[0][0], w0r[1][0], w0r[2][0], b0r[0], xm, x0, xp);
            v.y = e0_val(w0r[0][1], w0r[1][1], w0r[2][1], b0r[1], xm, x0, xp);
            v.z = e0_val(w0r[0][2], w0r[1][2], w0r[2][2], b0r[2], xm, x0, xp);
            v.w = e0_val(w0r[0][3], w0r[1][3], w0r[2][3], b0r[3], xm, x0, xp);
        }
        *reinterpret_cast<float4*>(er + ero + 8 * k * RS) = v;
        const float sk = (zb >> k) & 1u ? 0.f : s;
        v.x = __int_as_float(max(__float_as_int(v.x), 0)); v.y = __int_as_float(max(__float_as_int(v.y), 0));
        v.z = __int_as_float(max(__float_as_int(v.z), 0)); v.w = __int_as_float(max(__float_as_int(v.w), 0));
        uint32_t h01, l01, h23, l23;
        split2(v.x * sk, v.y * sk, h01, l01);
        split2(v.z * sk, v.w * sk, h23, l23);
        uint8_t* p = IMG + imgo + 8 * k * RS;
        *reinterpret_cast<uint2*>(p) = make_uint2(h01, h23);
        *reinterpret_cast<uint2*>(p + 256) = make_uint2(l01, l23);
    };

    // e_{l+1} > 0 words of a finished tile -> next layer's positions (wave w: columns 16 w..)
    auto store_me = [&](int b) {
        if (a.me_next && lane < 16) {
            const int c = 16 * w + lane;
            const int t = MBT[c];
            const int pn = (t & ((1 << a.dn_log2) - 1)) * a.nn + (t >> a.dn_log2);
            *reinterpret_cast<uint4*>(a.me_next + ((size_t)b * a.T + pn) * 8) =
                *reinterpret_cast<const uint4*>(&MBE[c * 8]);
        }
    };

    // ---- epilogue 2 of tile prv (residual rows erp), unit u = (j, g) in three parts.  e_{l+1}
    //      goes back into the residual rows it was computed from (in place: only this wave reads
    //      its quarter), and leaves for HBM from there as whole 128-B lines (flush: 8 columns x
    //      the wave's 32 channels per store); stored straight from the accumulator layout, each
    //      store would touch 32 lines 32 B at a time ----
    f32x4 acc2[2][4];                  // y of the pending epilogue 2 (sub-tiles n = 2 cb + rb)
    Tile prv = tile_of(blockIdx.x);
    float inv2p = 0.f;
    float emax = 0.f;
    uint32_t mb[2][2] = {{0u, 0u}, {0u, 0u}};
    float4 e2e, e2b, e2o;
    auto epi2_begin = [&]() {   // (emax runs on over the workgroup's consecutive tiles of one clip)
        mb[0][0] = mb[0][1] = mb[1][0] = mb[1][1] = 0u;
    };
    // unit u = (j, sub-tile g): channels chq + 16 rb .. + 3 of column 16 cb + i16
    auto epi2_part = [&](int u, int part, uint8_t* erp) {
        const int j = u >> 2, g = u & 3, rb = g & 1, cb = g >> 1;
        const int ch = chq + 16 * rb;
        if (part == 0) {
            e2e = *reinterpret_cast<const float4*>(erp + Lc[j][cb] * RS + 4 * ch);
            e2b = *reinterpret_cast<const float4*>(&BIAS[C + ch]);
        } else if (part == 1) {
            e2o.x = e2e.x + fmaf(acc2[j][g][0], inv2p, e2b.x);
            e2o.y = e2e.y + fmaf(acc2[j][g][1], inv2p, e2b.y);
            e2o.z = e2e.z + fmaf(acc2[j][g][2], inv2p, e2b.z);
            e2o.w = e2e.w + fmaf(acc2[j][g][3], inv2p, e2b.w);
            *reinterpret_cast<float4*>(erp + Lc[j][cb] * RS + 4 * ch) = e2o;
        } else {
            emax = fmaxf(emax, fmaxf(fmaxf(fabsf(e2o.x), fabsf(e2o.y)), fmaxf(fabsf(e2o.z), fabsf(e2o.w))));
            // bit mbit(4 g' + k) = 4 k + g' of the column's word h = q4 & 1 (common.h, splitwave.h mgrp)
            mb[j][cb] = or_pos_bits4(mb[j][cb], e2o.x, e2o.y, e2o.z, e2o.w, mg0 + 2 * rb);
        }
    };
    // flush piece (j, q): columns 32 j + 8 q + lr (lr = lane >> 3), channels cq .. cq + 3; part 0
    // reads the row back, part 1 stores it
    float4 fl4;
    const uint32_t fl_lane = (uint32_t)((lr * a.d * C + cq) * 4);
    auto flush_part = [&](int j, int q, int part, const uint8_t* erp) {
        const int c = 32 * j + 8 * q + lr;
        if (part == 0) {
            const int row = (MASKED || ONESEG) ? c + 1 : 34 * j + 1 + 8 * q + lr;   // frow(c)
            fl4 = *reinterpret_cast<const float4*>(erp + row * RS + 4 * cq);
        } else if (MASKED) {
            const int t = pos_time(prv.p0 + c, a.fn, a.d);
            *reinterpret_cast<float4*>(a.eout + ((size_t)prv.b * a.T + t) * C + cq) = fl4;
        } else {   // time tb + (uniform part) + lr d: the lane offset is fixed, the rest scalar
            const int tu = ONESEG ? (32 * j + 8 * q) * a.d : j + 8 * q * a.d;
            bst4(mk_rsrc(a.eout + ((size_t)prv.b * a.T + prv.tb) * C), fl_lane, (uint32_t)(tu * C * 4), fl4);
        }
    };
    // words and column times to LDS: a column's word h holds the groups of lane quads h and h + 2
    // (the lanes 32 apart); the quads 0 / 1 write it, all four the column's time (identical values)
    auto epi2_words = [&]() {
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int cb = 0; cb < 2; ++cb) {
                const int c = 32 * j + 16 * cb + i16;
                const uint32_t wv = mb[j][cb] | (uint32_t)__shfl_xor((int)mb[j][cb], 32);
                if (q4 < 2) MBE[c * 8 + 4 * q4 + w] = (uint16_t)wv;
                MBT[c] = ctime(prv, c, toff[j][cb]);
            }
    };
    // max |e_{l+1}| of clip prv.b -> gmax_out, once per run of tiles of one clip (with the
    // clip-interleaved tile order a workgroup usually keeps its clip for the whole launch)
    auto epi2_max = [&]() {
        const uint32_t m = wave_max_bits(emax);
        if (lane == 0) atomicMax(gslot(a.gmax_out, prv.b, blockIdx.x), m);
        emax = 0.f;
    };

    // ---- epilogue 1 of column half j, unit g in two parts: u, bits; v -> split v image ----
    // v = relu(u) 2^m_v = relu(acc 2^(m_v - m_e - k_d) + b_d 2^m_v): the scale folded into the fma
    // (powers of two: the same values); the u > 0 bits from the split's rtz hi halves (splitwave.h
    // nz2; SW_UBITS_EXACT: from v itself)
    f32x4 acc1[2][4];
    float a1 = 0.f;
    float bs_sv = -1.f;   // the v scale BDS holds
    uint32_t mu_w = 0;
    float4 e1v;
    // sub-tile g of column half j (rb = g & 1, cb = g >> 1); after both row blocks of a column
    // block the column's u > 0 word (the other two groups from the lane quad q4 ^ 2)
    auto epi1_part = [&](int j, int g, int part) {
        const int rb = g & 1, cb = g >> 1, ch = chq + 16 * rb;
        if (part == 0) {
            const float4 b4 = *reinterpret_cast<const float4*>(&BDS[ch]);
            e1v.x = fmaxf(fmaf(acc1[j][g][0], a1, b4.x), 0.f);
            e1v.y = fmaxf(fmaf(acc1[j][g][1], a1, b4.y), 0.f);
            e1v.z = fmaxf(fmaf(acc1[j][g][2], a1, b4.z), 0.f);
            e1v.w = fmaxf(fmaf(acc1[j][g][3], a1, b4.w), 0.f);
        } else {
            uint32_t h01, l01, h23, l23;
            split2(e1v.x, e1v.y, h01, l01);
            split2(e1v.z, e1v.w, h23, l23);
            const int c = 32 * j + 16 * cb + i16;
            uint8_t* p = XV + c * RS + 2 * ch;
            *reinterpret_cast<uint2*>(p) = make_uint2(h01, h23);
            *reinterpret_cast<uint2*>(p + 256) = make_uint2(l01, l23);
#ifdef SW_UBITS_EXACT
            mu_w = or_pos_bits4(mu_w, e1v.x, e1v.y, e1v.z, e1v.w, mg0 + 2 * rb);
            if (rb == 1) {
                const uint32_t wv = mu_w | (uint32_t)__shfl_xor((int)mu_w, 32);
                if (q4 < 2) MBU[c * 8 + 4 * q4 + w] = (uint16_t)wv;
                mu_w = 0;
            }
#else
            mu_w = or_bits4(mu_w, h01, h23, mg0 + 2 * rb);
            if (rb == 1) {
                const uint32_t wv = mask16(mu_w | (uint32_t)__shfl_xor((int)mu_w, 32));
                if (q4 < 2) MBU[c * 8 + 4 * q4 + w] = (uint16_t)wv;
                mu_w = 0;
            }
#endif
        }
    };


    // ---- GEMM 1 of column half J over the image; side work per step.  Step st = (tap, K block
    //      kb of 32, column block cb): 3 split products x 2 row blocks (splitwave.h) ----
    auto gemm1h = [&](auto j_tag, auto side, const Tile& cu) {
        constexpr int J = decltype(j_tag)::value;
        bool ok0[2] = {true, true}, ok2[2] = {true, true};
        if (MASKED) {
#pragma unroll
            for (int cb = 0; cb < 2; ++cb) {
                const int pc = cu.p0 + 32 * J + 16 * cb + i16;
                const int m = pc - (int)fdiv((uint32_t)pc, a.fn) * a.n;
                ok0[cb] = m > 0;
                ok2[cb] = m < a.n - 1;
            }
        }
#pragma unroll
        for (int n = 0; n < 4; ++n)
#pragma unroll
            for (int i = 0; i < 4; ++i) acc1[J][n][i] = 0.f;
        // B fragments are read LA steps ahead (one step ahead leaves the LDS latency exposed)
        uint4 bh[LA + 1], bl[LA + 1];
        auto bread = [&](int st, uint4& xh, uint4& xl) {
            const int tp = st >> 3, kb = (st & 7) >> 1, cb = st & 1;
            const uint8_t* p = IMG + (Lc[J][cb] + tp - 1) * RS + kb * 64 + q4 * 16;
            xh = lds16(p);
            xl = lds16(p + 256);
        };
#pragma unroll
        for (int q = 0; q < LA; ++q) bread(q, bh[q], bl[q]);
#pragma unroll
        for (int st = 0; st < 24; ++st) {
            const int tp = st >> 3, kb = (st & 7) >> 1, cb = st & 1, bi = st % (LA + 1);
            uint4 xh = bh[bi], xl = bl[bi];
            if (MASKED && ((tp == 0 && !ok0[cb]) || (tp == 2 && !ok2[cb]))) {
                xh = make_uint4(0, 0, 0, 0);
                xl = xh;
            }
            f32x4& c0 = acc1[J][2 * cb];
            f32x4& c1 = acc1[J][2 * cb + 1];
            c0 = mfma16(wd[tp][2 * kb][0], xh, c0);
            c1 = mfma16(wd[tp][2 * kb + 1][0], xh, c1);
            if (st + LA < 24) bread(st + LA, bh[(st + LA) % (LA + 1)], bl[(st + LA) % (LA + 1)]);
            side(st);
            c0 = mfma16(wd[tp][2 * kb][1], xh, c0);
            c1 = mfma16(wd[tp][2 * kb + 1][1], xh, c1);
            c0 = mfma16(wd[tp][2 * kb][0], xl, c0);
            c1 = mfma16(wd[tp][2 * kb + 1][0], xl, c1);
            step6_schedule();
        }
    };
    // ---- GEMM 2 of column half J over the v image; step st = (K block st >> 1, column block
    //      st & 1) ----
    auto gemm2h = [&](auto j_tag, auto side) {
        constexpr int J = decltype(j_tag)::value;
#pragma unroll
        for (int n = 0; n < 4; ++n)
#pragma unroll
            for (int i = 0; i < 4; ++i) acc2[J][n][i] = 0.f;
        uint4 bh[LA + 1], bl[LA + 1];
        auto bload = [&](int st, uint4& xh, uint4& xl) {
            const uint8_t* p = XV + (32 * J + 16 * (st & 1) + i16) * RS + (st >> 1) * 64 + q4 * 16;
            xh = lds16(p);
            xl = lds16(p + 256);
        };
#pragma unroll
        for (int q = 0; q < LA; ++q) bload(q, bh[q], bl[q]);
#pragma unroll
        for (int st = 0; st < 8; ++st) {
            const int kb = st >> 1, cb = st & 1, bi = st % (LA + 1);
            f32x4& c0 = acc2[J][2 * cb];
            f32x4& c1 = acc2[J][2 * cb + 1];
            c0 = mfma16(wr[2 * kb][0], bh[bi], c0);
            c1 = mfma16(wr[2 * kb + 1][0], bh[bi], c1);
            if (st + LA < 8) bload(st + LA, bh[(st + LA) % (LA + 1)], bl[(st + LA) % (LA + 1)]);
            side(st);
            c0 = mfma16(wr[2 * kb][1], bh[bi], c0);
            c1 = mfma16(wr[2 * kb + 1][1], bh[bi], c1);
            c0 = mfma16(wr[2 * kb][0], bl[bi], c0);
            c1 = mfma16(wr[2 * kb + 1][0], bl[bi], c1);
            step6_schedule();
        }
    };
    using J0 = std::integral_constant<int, 0>;
    using J1 = std::integral_constant<int, 1>;

    if (blockIdx.x >= ntiles) return;   // (grid = min(tiles, CUs): not taken)

    // prologue: the first tile's image and residual rows; the second tile's rows in flight
    float gm_c;     // max |e_l| of the current tile's clip (one scalar load per tile: the next one's)
    {
        const Tile t0 = tile_of(blockIdx.x);
#pragma unroll
        for (int k = 0; k < NU; ++k) load_unit(t0, k);
        const uint32_t z0 = zero_bits_of(t0);
        gm_c = sload_gmax(a.gmax_in, t0.b);
        const float s0 = exp2i(scale_exp(gm_c));
#pragma unroll
        for (int k = 0; k < NU; ++k) conv_unit(k, &ER[0][0], s0, z0);
    }

    STAMP(13)
    // one tile; FIRST (the peeled first tile) has no pending epilogue 2.  Peeling keeps the
    // sequence of vector-memory operations identical in every loop iteration, so the compiler's
    // counted waits for the row loads never include the epilogue's stores.
    auto tile_body = [&](auto first_tag, int tile, int it) {
        constexpr bool FIRST = decltype(first_tag)::value;
        const Tile cu = tile_of(tile);
        const Tile nt = tile_of(clampt(tile + G));
                // T: the image of this tile complete (converted during the previous phase D)
        lds_barrier();
        STAMP(0)
        const float gm = gm_c;
        const int m_e = scale_exp(gm);
        const int m_v = scale_exp(fmaf(a.wdn, gm, a.bdm));
        if (nt.b != cu.b) gm_c = sload_gmax(a.gmax_in, nt.b);   // (usually the same clip: tile order)
        const float s_next = exp2i(scale_exp(gm_c));
        const uint32_t zn = zero_bits_of(nt);
        const float sv = exp2i(m_v);
        a1 = exp2i(m_v - m_e - a.kd);
        if (sv != bs_sv) {   // the clip's v scale changed: b_d 2^m_v of this wave's channels (only
            bs_sv = sv;      // this wave reads them, in program order after these writes)
            if (lane < 32) BDS[32 * w + lane] = BIAS[32 * w + lane] * sv;
        }
        uint8_t* erp = &ER[(it & 1) ^ 1][0];   // the previous tile's residual, then the next's

        STAMP(10)
        // A: GEMM 1 half 0 + epilogue 2 of the previous tile
        if (!FIRST) {
            epi2_begin();
            gemm1h(J0{}, [&](int st) {
                epi2_part(st / 3, st % 3, erp);
                if (st >= 12 && st < 20) flush_part(0, (st - 12) >> 1, st & 1, erp);
                if (st % 3 == 1 && st < 15) load_unit(nt, st / 3);   // rows of tile i+1: units 0..4
            }, cu);
            epi2_words();
            if (cu.b != prv.b) epi2_max();
        } else {
            gemm1h(J0{}, [&](int st) { if (st % 3 == 1 && st < 15) load_unit(nt, st / 3); }, cu);
        }
        STAMP(5)
        // B: GEMM 1 half 1 + epilogue 1 of half 0
        gemm1h(J1{}, [&](int st) {
            if (st < 8) epi1_part(0, st >> 1, st & 1);
            else if (!FIRST && st < 16) flush_part(1, (st - 8) >> 1, st & 1, erp);
            if (st >= 11 && st % 3 == 2) load_unit(nt, 5 + (st - 11) / 3);   // units 5..8: 11 14 17 20
        }, cu);
        lds_barrier();   // v image half 0, u > 0 words half 0, e > 0 words of tile i-1
        STAMP(1)
        if (!FIRST) store_me(prv.b);
        // C: GEMM 2 half 0 + epilogue 1 of half 1
        gemm2h(J0{}, [&](int kb) {
            epi1_part(1, kb >> 1, kb & 1);
        });
        lds_barrier();   // v image half 1, all u > 0 words
        STAMP(2)
        if (lane < 16)   // u > 0 words of the tile (this layer's positions): wave w, columns 16 w..
            *reinterpret_cast<uint4*>(a.mu + ((size_t)cu.b * a.T + cu.p0 + 16 * w + lane) * 8) =
                *reinterpret_cast<const uint4*>(&MBU[(16 * w + lane) * 8]);
        // D: GEMM 2 half 1 + conversion of tile i+1, each unit's registers reloaded with i+2
        gemm2h(J1{}, [&](int kb) {
            conv_unit(kb, erp, s_next, zn);
            if (kb == 7) conv_unit(NU - 1, erp, s_next, zn);
        });
        STAMP(3)
        prv = cu;
        inv2p = exp2i(-(m_v + a.kr));
    };
    tile_body(std::true_type{}, (int)blockIdx.x, 0);
    int it = 1;
    for (int tile = (int)blockIdx.x + G; tile < ntiles; tile += G, ++it)
        tile_body(std::false_type{}, tile, it);
    // drain: epilogue 2 of the last tile
    {
        uint8_t* erl = &ER[(it - 1) & 1][0];
        epi2_begin();
#pragma unroll
        for (int st = 0; st < 24; ++st) epi2_part(st / 3, st % 3, erl);
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            flush_part(q >> 2, q & 3, 0, erl);
            flush_part(q >> 2, q & 3, 1, erl);
        }
        epi2_words();
        wg_max_flush(WMX, wave_max_bits(emax), gslot(a.gmax_out, prv.b, blockIdx.x));   // (its barrier: the e > 0 words too)
        store_me(prv.b);
    }
    STAMP(4)
    STAMP_FLUSH(a.stamps)
}

}  // namespace

void launch_block_fwd_s16(const FwdArgsS& a0, hipStream_t s) {
    FwdArgsS a = a0;
    a.fn = make_fdiv((uint32_t)a.n);
    a.ft = make_fdiv((uint32_t)(SW_TILE_INTERLEAVE ? a.B : a.T / TMS));
    const int nt = a.B * (a.T / TMS);
    const dim3 grid(std::min(nt, a.cus > 0 ? std::min(a.cus, sw::num_cus()) : sw::num_cus()));
    Layout ly;
    const bool masked = pick_layout(a.n, ly);
    if (a.xin && (masked || ly.M != TMS || a.d != 1)) { fprintf(stderr, "block_fwd_s: xin needs d = 1\n"); abort(); }
    if (masked) hipLaunchKernelGGL((k_block_fwd_s16<true, false, false>), grid, dim3(FT), 0, s, a, ly);
    else if (ly.M == TMS && a.xin) hipLaunchKernelGGL((k_block_fwd_s16<false, true, true>), grid, dim3(FT), 0, s, a, ly);
    else if (ly.M == TMS) hipLaunchKernelGGL((k_block_fwd_s16<false, true, false>), grid, dim3(FT), 0, s, a, ly);
    else hipLaunchKernelGGL((k_block_fwd_s16<false, false, false>), grid, dim3(FT), 0, s, a, ly);
}

}  // namespace ast
