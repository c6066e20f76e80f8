// Split-fp16 encoder block backward (precision 2): d loss / d e_l for one block of
// model.py:95-116, restated by oracle/astyle_oracle.py:171-189 (encoder_backward):
//   tot = d loss / d e_{l+1} (the chain, its own direct loss term included)
//   g_u = [u > 0] (W_r tot)                         1x1 conv transposed
//   g_a = sum_k W_d[k] g_u(p - k + 1)                K = 3 SAME dilated conv transposed, in
//                                                    time_to_batch positions (masked.py:110-160)
//   out = tot + D_l + [e_l > 0] g_a                  D_l: direct loss gradient of e_l, if tapped
// fp32 storage, split fp16 operands on v_mfma_f32_32x32x16_f16, fp32 accumulation and
// epilogue (splitwave.h).
//
// One workgroup per CU (wave w owns channels 32 w .. 32 w + 31), persistent over tiles of 64
// positions, one wave per SIMD; the structure of the forward (block_fwd_split.hip): a tile's
// tot and D_l rows arrive in registers a tile ahead in row units (8 cache lines per wave
// instruction) and are converted during the previous tile's second GEMM into the split tot
// image and the wave's quarter of a residual buffer (tot + D_l in fp32, double-buffered, read
// back by the same wave); the relu-mask words come by plain loads.  Per tile i:
//   T  barrier (tot image i complete)
//   A  g_v = W_r tot, column half 0 (8 k-steps x 3 products); carries epilogue half 1 of tile
//      i-1 (out = residual + [e_l > 0] g_a 2^-(m_u+k_d) -> HBM)
//   B  g_v column half 1; carries the rest of that epilogue and g_u of half 0 (mask, scale
//      2^m_u from the bound |g_v| <= wrn max|tot|, split -> g_u image)
//   H  (one-segment layouts, unless the workgroup's previous tile is the left neighbour: then
//      its g_u rows 64 / 65 are copied to rows 0 / 1) g_v of rows 0 / 1 (positions p0 - 1, p0;
//      the column tiles cover p0 + 1 .. p0 + 64); carries g_u of half 1; g_u of the last column
//      tile; barrier (g_u image complete, tot image free).  The left neighbour includes the
//      last tile of the previous sub-sequence (CARRY): that tile's right-halo column (p0 + 64,
//      SAME padding for its own g_a) is computed on the next sub-sequence's first position
//      instead of a zero row and set aside in g_u row 67, so the next tile's rows 0 / 1 are
//      (0, row 67) and no tile of a walk pays the halo MFMAs but its first
//   C  g_a, column half 0 (3 taps x 8 k-steps x 3 products over the g_u image); carries the
//      conversion of tile i+1 and, unit by unit behind it, the row loads of tile i+2
//   D  g_a, column half 1; carries epilogue half 0 of tile i
// The first tile is peeled so every loop iteration issues the same vector-memory sequence.
// non-temporal (nt) row loads; the stores keep the default policy: they leave the accumulator
// layout as 16-B pieces of 32 lines per instruction, which L2 merges into whole lines, and nt made
// them partial-line writes to DRAM (+75 % per launch, profiles/r6_diag/block_ab.txt)
#ifndef SW_BWD_DEFAULT_POLICY
#define SW_LD_AUX 2
#endif
#include "splitwave.h"
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <type_traits>

namespace ast {
namespace {
using namespace sw;

constexpr int IROWS = 72;             // tot image / residual rows (9 units x 8)
constexpr int ISLOT = IROWS * RS;
constexpr int GROWS = 68;             // g_u image rows (66 / 68 used; 66 takes unused halo writes)
constexpr int LA = 2;                 // B-fragment lookahead (steps)

// SX (block 0, one-segment layout, d = 1, no D_0): the start conv's backward folded into the
// epilogue -- out = d loss / d e_0 is not stored; per position the wave's three dot products
// sum_c W0[k][c] out[t][c] over its 32 channels go to spart (launch_startx_gx sums the four
// waves and forms d loss / d x): no 2 GiB g_0 round trip (model.py:82-93)
// WHOLE (one-segment layout with n == 64: every tile is a whole sub-sequence, d = T / 64): both
// halo rows (p0 - 1, p0 + 64) are SAME padding, so the column tiles cover p0 .. p0 + 63 and rows
// 0 / 65 of the g_u image stay zero: no halo MFMA tile
template <bool MASKED, bool ONESEG, bool HAS_D, bool SX, bool WHOLE>
__global__ void __launch_bounds__(FT, 1) k_block_bwd_s(BwdArgsS a, Layout) {
    // the layout as compile-time constants (pick_layout: one segment or masked: M = 64 with two
    // halo rows; else segments of SEGM = 32 with their pad rows), not the launch argument
    constexpr bool GEO1 = ONESEG || MASKED;
    const Layout ly = {GEO1 ? TMS : SEGM, GEO1 ? TMS + 2 : (TMS / SEGM) * (SEGM + 2)};
    static_assert(!WHOLE || (ONESEG && !MASKED), "WHOLE is a one-segment layout");
    __shared__ __attribute__((aligned(16))) uint8_t XS[ISLOT];        // split tot image
    __shared__ __attribute__((aligned(16))) uint8_t XG[GROWS * RS];   // split g_u image
    __shared__ __attribute__((aligned(16))) uint8_t ER[2][ISLOT];     // fp32 tot + D_l rows
    __shared__ __attribute__((aligned(16))) float W0S[SX ? 3 * C : 4];   // SX: W0 [3][C]
    __shared__ uint32_t WMX[4];                                     // the drain's per-wave maxima

    const int tiles = a.T / TMS;
    const int ntiles = a.B * tiles;
    const int tid = threadIdx.x, lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int r = lane & 31, h = lane >> 5;
    const int G = (int)gridDim.x;
    STAMP_DECL

    auto tile_of = [&](int tl) { return tile_at<MASKED>(tl, a.ft, a.fn, a.d, ly); };
    auto clampt = [&](int tl) { return tl < ntiles ? tl : ntiles - 1; };
#ifdef ASTYLE_DIAG_BWD_L2ROWS
    // diagnostic build only (tools): every row load and store addresses the workgroup's first
    // tile, so the same instruction stream runs from L2 instead of HBM (results wrong)
    const Tile t0f = tile_of(blockIdx.x);
    auto memt = [&](const Tile& t) { (void)t; return t0f; };
#else
    auto memt = [&](const Tile& t) { return t; };
#endif

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
    for (int i = tid; i < GROWS * RS / 16; i += FT) reinterpret_cast<uint4*>(XG)[i] = make_uint4(0, 0, 0, 0);
    if (SX)   // (read after the first tile's T barrier)
        for (int i = tid; i < 3 * C; i += FT) W0S[i] = a.w0[i];

    int Lc[2], toff[2];
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        Lc[j] = frow(32 * j + r, ly);
        toff[j] = MASKED ? 0 : row_toff(Lc[j], ly, a.d);
    }
    const int chb = 32 * w + 4 * h;
    auto ctime = [&](const Tile& t, int cc, int to) { return col_time<MASKED>(t, cc, to, a.fn, a.d); };
    // g_v / g_u rows.  One-segment layouts shift the two column tiles by one row: they cover
    // image rows 2..65 (positions p0 + 1 .. p0 + 64, the right halo included), and rows 0 / 1
    // (p0 - 1, p0) are either the previous tile's rows 64 / 65 (the workgroup's previous tile is
    // the left neighbour in the same sub-sequence: copied, no MFMAs) or the halo tile's
    // (lane r == 0 -> row 0, r == 1 -> row 1; lanes r >= 2 compute a copy of row 0 and write it
    // to unused row 66).  Other layouts: the tile's columns, no halo rows.
    // masked layouts have the one-segment geometry (row L = position p0 + L - 1, gathered) and
    // a tile may start / end inside a sub-sequence: the same halo rows, tap masks in g_a
    constexpr bool HALO = (ONESEG && !WHOLE) || MASKED;
    // CARRY tiles: the last tile of a sub-sequence with a next position in the clip (p0 + 64,
    // the next sub-sequence's first position, time q + 1)
    constexpr bool CARRY = ONESEG && !WHOLE && !MASKED;
    auto carry_of = [&](const Tile& t) { return CARRY && t.m0 + TMS >= a.n && t.p0 + TMS < a.T; };
    int Lv[2];
#pragma unroll
    for (int j = 0; j < 2; ++j) Lv[j] = HALO ? Lc[j] + 1 : Lc[j];
    const int Lh = r == 1 ? 1 : 0;
    const int Lhw = r < 2 ? Lh : TMS + 2;

    // ---- rows of the next tile: tot (-> split image) and D_l (-> residual) ----
    RowUnits<MASKED, ONESEG> ru;
    ru.init(w, lane, ly, a.d);
    float4 lt[NU], lg[NU];
    // unmasked layouts load through buffer resources of the tile (rs_t / rs_d, set with the tile)
    rsrc_t rs_t, rs_d;
    auto set_rs = [&](const Tile& t_) {
        const Tile t = memt(t_);
        if (!MASKED) {
            rs_t = ru.rsrc_of(a.tin, t, a.T, a.d);
            if (HAS_D) rs_d = ru.rsrc_of(a.dadd, t, a.T, a.d);
        }
    };
    auto load_unit = [&](const Tile& t_, int k) {
        const Tile t = memt(t_);
        if (MASKED) {
            lt[k] = ru.load(a.tin, t, k, a.T, a.fn, a.d);
            if (HAS_D) lg[k] = ru.load(a.dadd, t, k, a.T, a.fn, a.d);
        } else if (CARRY && k == NU - 1) {
            // unit 8 by 64-bit address: in a CARRY tile the lanes of row 65 (lr == 1) read the
            // next sub-sequence's first tot row (its D row stays the dummy: row 65's residual is
            // no output)
            const int q = t.tb - t.m0 * a.d;
            const float* pn = a.tin + ((size_t)t.b * a.T + q + 1) * C + ru.cq;
            const float* pr = reinterpret_cast<const float*>(
                reinterpret_cast<const char*>(a.tin + ((ptrdiff_t)t.b * a.T + t.tb - a.d) * C) + ru.unit_off(t, k, a.fn));
            lt[k] = *reinterpret_cast<const float4*>(carry_of(t) && ru.lr == 1 ? pn : pr);
            if (HAS_D) lg[k] = ru.loadb(rs_d, t, k, a.fn);
        } else {
            lt[k] = ru.loadb(rs_t, t, k, a.fn);
            if (HAS_D) lg[k] = ru.loadb(rs_d, t, k, a.fn);
        }
    };
    auto conv_unit = [&](int k, uint8_t* er, float s, uint32_t zb) {
        const float4 v = lt[k];
        float4 e = v;
        if (HAS_D) { e.x += lg[k].x; e.y += lg[k].y; e.z += lg[k].z; e.w += lg[k].w; }
        *reinterpret_cast<float4*>(er + ru.ero + 8 * k * RS) = e;
        const float sk = (zb >> k) & 1u ? 0.f : s;
        uint32_t h01, l01, h23, l23;
        split2s(v.x * sk, v.y * sk, h01, l01);
        split2s(v.z * sk, v.w * sk, h23, l23);
        uint8_t* p = XS + ru.imgo + 8 * k * RS;
        *reinterpret_cast<uint2*>(p) = make_uint2(h01, h23);
        *reinterpret_cast<uint2*>(p + 256) = make_uint2(l01, l23);
    };
    // zero bits of a tile's units: a CARRY tile's row 65 is real
    auto zbits = [&](const Tile& t) {
        uint32_t z = ru.zero_bits(t, a.fn);
        if (carry_of(t) && ru.lr == 1) z &= ~(1u << (NU - 1));
        return z;
    };
    // ---- relu-mask words (u16, position-indexed): u > 0 of the tile's columns and halos,
    //      e_l > 0 of its columns ----
    uint32_t mu_c[2], muh_c = 0, me_c[2], mu_n[2], muh_n = 0, me_n[2], me_p = 0;
    auto load_masks = [&](const Tile& t, uint32_t (&mu)[2], uint32_t& muh, uint32_t (&me)[2]) {
        const size_t cb = (size_t)t.b * a.T + t.p0;
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            // u > 0 of the g_v rows Lv[j]; a position past the clip reads any word (its tot row
            // is zero)
            const int pv = HALO ? min(t.p0 + 1 + 32 * j + r, a.T - 1) : t.p0 + 32 * j + r;
            mu[j] = a.mu[((size_t)t.b * a.T + pv) * 8 + 4 * h + w];
            me[j] = a.me[(cb + 32 * j + r) * 8 + 4 * h + w];
        }
        if (HALO) {     // rows 0 / 1: p0 - 1 (outside the clip at p0 == 0: its tot row is zero or tap-masked), p0
            const int p = t.p0 + (r == 1 ? 0 : -1);
            muh = a.mu[((size_t)t.b * a.T + (p < 0 ? 0 : p)) * 8 + 4 * h + w];
        }
    };

    // ---- step 1: g_v of column tile J (0, 1; 2 = the halo columns) ----
    f32x16 acc1[3];
    auto gemm1 = [&](auto j_tag, auto side) {
        constexpr int J = decltype(j_tag)::value;
        const int row = J < 2 ? Lv[J < 2 ? J : 0] : Lh;
#pragma unroll
        for (int i = 0; i < 16; ++i) acc1[J][i] = 0.f;
        uint4 bh[LA + 1], bl[LA + 1];
        auto bread = [&](int kb, uint4& xh, uint4& xl) {
            const uint8_t* p = XS + row * RS + kb * 32 + h * 16;
            xh = lds16(p);
            xl = lds16(p + 256);
        };
#pragma unroll
        for (int q = 0; q < LA; ++q) bread(q, bh[q], bl[q]);
#pragma unroll
        for (int kb = 0; kb < 8; ++kb) {
            const int cb = kb % (LA + 1);
            acc1[J] = mfma_f16(wr[kb][0], bh[cb], acc1[J]);
            if (kb + LA < 8) bread(kb + LA, bh[(kb + LA) % (LA + 1)], bl[(kb + LA) % (LA + 1)]);
            side(kb);
            acc1[J] = mfma_f16(wr[kb][1], bh[cb], acc1[J]);
            acc1[J] = mfma_f16(wr[kb][0], bl[cb], acc1[J]);
            step3_schedule();
        }
    };
    // g_u unit (J, g) in two parts: mask; scale + split -> image row
    float4 gq = make_float4(0.f, 0.f, 0.f, 0.f);
    int Lv1t = Lv[1];   // row of column tile 1 (a CARRY tile: its right-halo lane r == 31 -> row 67)
    auto gu_part = [&](int J, int g, int part, float f) {
        if (part == 0) {
            const uint32_t wd_ = J < 2 ? mu_c[J] : muh_c;
            gq.x = keep_if(acc1[J][4 * g + 0], wd_, g);
            gq.y = keep_if(acc1[J][4 * g + 1], wd_, 4 + g);
            gq.z = keep_if(acc1[J][4 * g + 2], wd_, 8 + g);
            gq.w = keep_if(acc1[J][4 * g + 3], wd_, 12 + g);
        } else {
            // the scale after the mask (f is a power of two: the same values), so that the
            // split's low half fuses with it into one v_fma_mix_f32
            uint32_t h01, l01, h23, l23;
            split2s(gq.x * f, gq.y * f, h01, l01);
            split2s(gq.z * f, gq.w * f, h23, l23);
            uint8_t* p = XG + (J == 0 ? Lv[0] : J == 1 ? Lv1t : Lhw) * RS + 2 * (chb + 8 * g);
            *reinterpret_cast<uint2*>(p) = make_uint2(h01, h23);
            *reinterpret_cast<uint2*>(p + 256) = make_uint2(l01, l23);
        }
    };

    // ---- step 2: g_a of column half J ----
    f32x16 acc2[2];
    auto gemm2 = [&](auto j_tag, auto side, const Tile& cu) {
        constexpr int J = decltype(j_tag)::value;
        bool ok0 = true, ok2 = true;
        if (MASKED) {
            const int pc = cu.p0 + 32 * J + r;
            const int m = pc - (int)fdiv((uint32_t)pc, a.fn) * a.n;
            ok0 = m > 0;
            ok2 = m < a.n - 1;
        }
#pragma unroll
        for (int i = 0; i < 16; ++i) acc2[J][i] = 0.f;
        uint4 bh[LA + 1], bl[LA + 1];
        auto bread = [&](int st, uint4& xh, uint4& xl) {
            const int tp = st >> 3, kb = st & 7;
            const uint8_t* p = XG + (Lc[J] + 1 - tp) * RS + kb * 32 + h * 16;
            xh = lds16(p);
            xl = lds16(p + 256);
        };
#pragma unroll
        for (int q = 0; q < LA; ++q) bread(q, bh[q], bl[q]);
#pragma unroll
        for (int st = 0; st < 24; ++st) {
            const int tp = st >> 3, kb = st & 7, cb = st % (LA + 1);
            uint4 xh = bh[cb], xl = bl[cb];
            if (MASKED && ((tp == 0 && !ok2) || (tp == 2 && !ok0))) {
                xh = make_uint4(0, 0, 0, 0);
                xl = xh;
            }
            acc2[J] = mfma_f16(wd[tp][kb][0], xh, acc2[J]);
            if (st + LA < 24) bread(st + LA, bh[(st + LA) % (LA + 1)], bl[(st + LA) % (LA + 1)]);
            side(st);
            acc2[J] = mfma_f16(wd[tp][kb][1], xh, acc2[J]);
            acc2[J] = mfma_f16(wd[tp][kb][0], xl, acc2[J]);
            step3_schedule();
        }
    };

    // ---- epilogue unit (J, g) of tile et in three parts: residual read; out -> HBM; max ----
    float omax = 0.f, inv2p = 0.f;
    float* dst = nullptr;
    rsrc_t rs_o;            // unmasked layouts: the stores through a resource at the tile's base time
    const uint32_t colo[2] = {(uint32_t)((toff[0] * C + chb) * 4), (uint32_t)((toff[1] * C + chb) * 4)};
    uint32_t ocol = 0;
    float4 oe, oo;
    float sk0 = 0.f, sk1 = 0.f, sk2 = 0.f;   // SX: the lane's dot products over its 16 channels
    size_t sxo = 0;                          // SX: spart float index of (column, wave)
    auto epi_begin = [&](const Tile& et_, int J) {
        const Tile et = memt(et_);
        if (SX) sxo = (((size_t)et.b * a.T + ctime(et, 32 * J + r, toff[J])) * 4 + w) * 4;
        else if (MASKED) dst = a.gout + ((size_t)et.b * a.T + ctime(et, 32 * J + r, toff[J])) * C + chb;
        else { rs_o = mk_rsrc(a.gout + ((size_t)et.b * a.T + et.tb) * C); ocol = colo[J]; }
    };
    auto epi_part = [&](int J, int g, int part, const uint8_t* er, uint32_t mw, float inv2) {
        if (part == 0) {
            oe = *reinterpret_cast<const float4*>(er + Lc[J] * RS + 4 * (chb + 8 * g));
        } else if (part == 1) {
            oo.x = fmaf(keep_if(acc2[J][4 * g + 0], mw, g), inv2, oe.x);
            oo.y = fmaf(keep_if(acc2[J][4 * g + 1], mw, 4 + g), inv2, oe.y);
            oo.z = fmaf(keep_if(acc2[J][4 * g + 2], mw, 8 + g), inv2, oe.z);
            oo.w = fmaf(keep_if(acc2[J][4 * g + 3], mw, 12 + g), inv2, oe.w);
            if (SX) {
                const float4 q0 = *reinterpret_cast<const float4*>(&W0S[chb + 8 * g]);
                const float4 q1 = *reinterpret_cast<const float4*>(&W0S[C + chb + 8 * g]);
                const float4 q2 = *reinterpret_cast<const float4*>(&W0S[2 * C + chb + 8 * g]);
                sk0 = fmaf(q0.w, oo.w, fmaf(q0.z, oo.z, fmaf(q0.y, oo.y, fmaf(q0.x, oo.x, sk0))));
                sk1 = fmaf(q1.w, oo.w, fmaf(q1.z, oo.z, fmaf(q1.y, oo.y, fmaf(q1.x, oo.x, sk1))));
                sk2 = fmaf(q2.w, oo.w, fmaf(q2.z, oo.z, fmaf(q2.y, oo.y, fmaf(q2.x, oo.x, sk2))));
            } else if (MASKED) *reinterpret_cast<float4*>(dst + 8 * g) = oo;
            else bst4(rs_o, ocol + 32 * g, 0u, oo);
        } else {
            omax = fmaxf(omax, fmaxf(fmaxf(fabsf(oo.x), fabsf(oo.y)), fmaxf(fabsf(oo.z), fabsf(oo.w))));
            if (SX && g == 3) {   // the column's 16 channels done: + the other half's 16 -> spart
                const float o0 = __shfl_xor(sk0, 32), o1 = __shfl_xor(sk1, 32), o2 = __shfl_xor(sk2, 32);
                if (h == 0)
                    *reinterpret_cast<float4*>(a.spart + sxo) = make_float4(sk0 + o0, sk1 + o1, sk2 + o2, 0.f);
                sk0 = sk1 = sk2 = 0.f;
            }
        }
    };
    auto epi_max = [&](int b) {
        const uint32_t m = wave_max_bits(omax);
        if (lane == 0) atomicMax(gslot(a.gmax_out, b, blockIdx.x), m);
        omax = 0.f;
    };
    using J0 = std::integral_constant<int, 0>;
    using J1 = std::integral_constant<int, 1>;
    using J2 = std::integral_constant<int, 2>;

    if (blockIdx.x >= ntiles) return;   // (grid = min(tiles, CUs): not taken)

    // prologue: the first tile's image, residual rows and masks; the second tile's rows in flight
    float gm_c;     // max |tot| of the current tile's clip (one scalar load per tile: the next one's)
    {
        const Tile t0 = tile_of(blockIdx.x);
        set_rs(t0);
#pragma unroll
        for (int k = 0; k < NU; ++k) load_unit(t0, k);
        load_masks(t0, mu_c, muh_c, me_c);
        const uint32_t z0 = zbits(t0);
        gm_c = sload_gmax(a.gmax_in, t0.b);
        const float s0 = exp2i(scale_exp(gm_c));
#pragma unroll
        for (int k = 0; k < NU; ++k) conv_unit(k, &ER[0][0], s0, z0);
        const Tile t1 = tile_of(clampt(blockIdx.x + G));
        set_rs(t1);
#pragma unroll
        for (int k = 0; k < NU; ++k) load_unit(t1, k);
    }

    Tile prv = tile_of(blockIdx.x);
    STAMP(14)
    auto tile_body = [&](auto first_tag, int tile, int it) {
        constexpr bool FIRST = decltype(first_tag)::value;
        const Tile cu = tile_of(tile);
        const Tile nt = tile_of(clampt(tile + G));
        const Tile n2 = tile_of(clampt(tile + 2 * G));
        set_rs(n2);   // (the previous ones' loads are all issued: units reload right after conversion)
        // T: this tile's tot image complete (converted during the previous phase C)
        lds_barrier();
        STAMP(6)
        const float gm = gm_c;
        const int m_t = scale_exp(gm);
        const int m_u = scale_exp(a.wrn * gm);
        const float f_u = exp2i(m_u - m_t - a.kr);   // acc units 2^(m_t + k_r) -> g_u 2^m_u
        const float inv2 = exp2i(-(m_u + a.kd));
        if (nt.b != cu.b) gm_c = sload_gmax(a.gmax_in, nt.b);   // (usually the same clip: tile order)
        const float s_next = exp2i(scale_exp(gm_c));
        const uint32_t zn = zbits(nt);
        uint8_t* erc = &ER[it & 1][0];          // this tile's residual
        uint8_t* ero = &ER[(it & 1) ^ 1][0];    // the previous tile's, then the next tile's

        // rows 0 / 1 from the previous tile's rows 64 / 65 when it is the left neighbour (every
        // wave its channel quarter; the previous tile's g_a reads are behind the T barrier, this
        // tile's first writes to rows 64 / 65 come in B)
        // (CARRY: the previous sub-sequence's last tile left row 65 zero and the first position's
        // g_u in row 67: rows 0 / 1 = 0 / row 67)
        const bool cont = HALO && !FIRST && prv.b == cu.b && prv.p0 + TMS == cu.p0 && (MASKED || CARRY || cu.m0 != 0);
        const bool fos = CARRY && cu.m0 == 0;
        const bool cry = carry_of(cu);
        Lv1t = cry && r == 31 ? GROWS - 1 : Lv[1];
        const int cpo = ((lane >> 2) & 1) * 256 + 64 * w + 16 * (lane & 3);   // (side work of A)
        const int csr = fos ? ((lane >> 3) ? GROWS - 1 : TMS) : TMS + (lane >> 3);
        uint4 cpv = make_uint4(0, 0, 0, 0);
        STAMP(11)
        // A: g_v half 0 + epilogue half 1 of the previous tile (parts 0..7)
        if (!FIRST) epi_begin(prv, 1);
        gemm1(J0{}, [&](int kb) {
            if (!FIRST) epi_part(1, kb / 3, kb % 3, ero, me_p, inv2p);
            if (cont && lane < 16) {   // rows 64 / 65 -> 0 / 1, read one step before the write
                if (kb == 0) {
                    cpv = lds16(XG + csr * RS + cpo);
                    if (fos && lane < 8) cpv = make_uint4(0, 0, 0, 0);
                }
                if (kb == 1) *reinterpret_cast<uint4*>(XG + (lane >> 3) * RS + cpo) = cpv;
            }
            // a CARRY tile's row 65 is SAME padding for its own g_a (after the copy's read)
            if (cry && lane < 8 && kb == 2) *reinterpret_cast<uint4*>(XG + (TMS + 1) * RS + cpo) = make_uint4(0, 0, 0, 0);
        });
        // B: g_v half 1 + the epilogue's parts 8..11 + g_u of half 0
        gemm1(J1{}, [&](int kb) {
            if (!FIRST && kb < 4) epi_part(1, (kb + 8) / 3, (kb + 8) % 3, ero, me_p, inv2p);
            gu_part(0, kb >> 1, kb & 1, f_u);
        });
        // max |out| of clip prv.b -> gmax_out once per run of tiles of one clip (omax runs on:
        // with the clip-interleaved tile order a workgroup usually keeps its clip)
        if (!FIRST && cu.b != prv.b) epi_max(prv.b);
        if (HALO && !cont) {
            // H: g_v of rows 0 / 1 + g_u of half 1; then g_u of rows 0 / 1
            gemm1(J2{}, [&](int kb) { gu_part(1, kb >> 1, kb & 1, f_u); });
#pragma unroll
            for (int q = 0; q < 8; ++q) gu_part(2, q >> 1, q & 1, f_u);
        } else {
#pragma unroll
            for (int q = 0; q < 8; ++q) gu_part(1, q >> 1, q & 1, f_u);
        }
        lds_barrier();   // g_u image complete; every wave is done with the tot image
        STAMP(7)
        // C: g_a half 0 + conversion of tile i+1, each unit's registers reloaded with tile i+2
        //    right away (a tile of latency before the next conversion: issued later, the loads'
        //    latency shows)
        gemm2(J0{}, [&](int st) {
            // unit k at step 24 k / 9 (0 2 5 8 10 13 16 18 21): spread over the phase
#pragma unroll
            for (int k = 0; k < NU; ++k)
                if (st == (24 * k) / NU) {
                    conv_unit(k, ero, s_next, zn);
                    load_unit(n2, k);
                }
            if (st == 3) load_masks(nt, mu_n, muh_n, me_n);
        }, cu);
        STAMP(8)
        // D: g_a half 1 + epilogue half 0 of this tile
        epi_begin(cu, 0);
        gemm2(J1{}, [&](int st) { if (st < 12) epi_part(0, st / 3, st % 3, erc, me_c[0], inv2); }, cu);
        STAMP(9)
        prv = cu;
        inv2p = inv2;
        me_p = me_c[1];
        me_c[0] = me_n[0]; me_c[1] = me_n[1];
        mu_c[0] = mu_n[0]; mu_c[1] = mu_n[1];
        muh_c = muh_n;
    };
    tile_body(std::true_type{}, (int)blockIdx.x, 0);
    int it = 1;
    for (int tile = (int)blockIdx.x + G; tile < ntiles; tile += G, ++it)
        tile_body(std::false_type{}, tile, it);
    // drain: epilogue half 1 of the last tile
    {
        const uint8_t* erl = &ER[(it - 1) & 1][0];
        epi_begin(prv, 1);
#pragma unroll
        for (int q = 0; q < 12; ++q) epi_part(1, q / 3, q % 3, erl, me_p, inv2p);
        wg_max_flush(WMX, wave_max_bits(omax), gslot(a.gmax_out, prv.b, blockIdx.x));
    }
    STAMP(12)
    STAMP_FLUSH(a.stamps)
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
    if ((threadIdx.x & 63) == 0) atomicMax(gslot(out, b, blockIdx.x), __float_as_uint(m));
}

}  // namespace

void launch_block_bwd_s(const BwdArgsS& a0, hipStream_t s) {
    BwdArgsS a = a0;
    a.fn = make_fdiv((uint32_t)a.n);
    a.ft = make_fdiv((uint32_t)(SW_TILE_INTERLEAVE ? a.B : a.T / TMS));
    const int nt = a.B * (a.T / TMS);
    const dim3 grid(std::min(nt, a.cus > 0 ? std::min(a.cus, sw::num_cus()) : sw::num_cus()));
    Layout ly;
    const bool masked = pick_layout(a.n, ly);
    const bool oneseg = !masked && ly.M == TMS;
    if (a.spart && (!oneseg || a.dadd || a.d != 1)) { fprintf(stderr, "block_bwd_s: spart needs d = 1, no D\n"); abort(); }
    const bool whole = oneseg && a.n == TMS;
#define BWD_LAUNCH(M, O, D, X, W) hipLaunchKernelGGL((k_block_bwd_s<M, O, D, X, W>), grid, dim3(FT), 0, s, a, ly)
    if (masked) { if (a.dadd) BWD_LAUNCH(true, false, true, false, false); else BWD_LAUNCH(true, false, false, false, false); }
    else if (whole && !a.spart) {
        if (a.dadd) BWD_LAUNCH(false, true, true, false, true); else BWD_LAUNCH(false, true, false, false, true);
    } else if (oneseg) {
        if (a.dadd) BWD_LAUNCH(false, true, true, false, false);
        else if (a.spart) BWD_LAUNCH(false, true, false, true, false);
        else BWD_LAUNCH(false, true, false, false, false);
    } else { if (a.dadd) BWD_LAUNCH(false, false, true, false, false); else BWD_LAUNCH(false, false, false, false, false); }
#undef BWD_LAUNCH
}

void launch_absmax(const float* x, size_t per_clip, int B, unsigned* out, hipStream_t s) {
    int chunks = 1;
    while (chunks < 64 && per_clip % ((size_t)chunks * 8) == 0 && per_clip / (chunks * 2) >= 4096) chunks *= 2;
    hipLaunchKernelGGL(k_absmax, dim3(B * chunks), dim3(256), 0, s, x, per_clip, chunks, out);
}

}  // namespace ast
