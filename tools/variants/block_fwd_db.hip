// Split-fp16 encoder block forward (precision 2), double-buffered image variant: the same
// block as block_fwd_split.hip (model.py:95-116, masked.py:110-160) with the same arithmetic in
// the same order (bit-identical results), scheduled differently.  block_fwd_split.hip keeps two
// fp32 residual buffers (the conversion writes tile i+1's e_l rows while tile i's wait for
// epilogue 2), so its single split image can only be refilled under GEMM 2's half 1 (24 MFMAs,
// the conversion's VALU and LDS writes exposed).  Here ONE staging buffer OB takes a tile's
// e_l again as whole lines from L2 / the Infinity Cache (its rows were loaded two tiles
// earlier), so the 38 KB freed double-buffers the image and the conversion of tile i+1 runs
// under tile i's GEMM-1 phases (144 MFMAs); the row loads move one tile further ahead.
// Per tile i (image slot i & 1):
//   T  barrier (image i complete)
//   A  GEMM 1 half 0 over image i; tile i's residual rows (8 whole-line loads); epilogue 2 of
//      tile i-1 in OB (e_i = e_{i-1} + y + b_r in place) and the flush of its half 0 (whole
//      lines -> HBM); conversion of tile i+1 units 0..4 into image i+1, row loads of tile i+2
//   B  GEMM 1 half 1; epilogue 1 of half 0, the flush of half 1, conversion units 5..8 +
//      loads; barrier
//   C  GEMM 2 half 0; epilogue 1 of half 1; barrier
//   D  GEMM 2 half 1; tile i's residual rows -> OB
// Scattering e_l / e_{l+1} in the accumulator layout instead (32 lines per wave instruction)
// made the launch 7-14 % slower than block_fwd_split.hip, and this form is 5 % slower
// (the conversion costs as many cycles under GEMM 1 as under GEMM 2).
// ASTYLE_FWD_DB selects it (block_fwd_split.hip's launcher).
#include "splitwave.h"
#include <algorithm>
#include <type_traits>

namespace ast {
namespace {
using namespace sw;

constexpr int IROWS = 72;             // image rows: 66 or 68 used, 9 units x 8 rows
constexpr int ISLOT = IROWS * RS;     // bytes per image
constexpr int LA = 2;                 // B-fragment lookahead (steps)

template <bool MASKED, bool ONESEG>
__global__ void __launch_bounds__(FT, 1) k_block_fwd_db(FwdArgsS a, Layout ly) {
    __shared__ __attribute__((aligned(16))) uint8_t IMG[2][ISLOT];  // split relu(e_l) images
    __shared__ __attribute__((aligned(16))) uint8_t XV[TMS * RS];   // split v image
    __shared__ __attribute__((aligned(16))) uint8_t OB[ISLOT];      // residual -> e_{l+1} rows (staging)
    __shared__ __attribute__((aligned(16))) float BIAS[2 * C];      // b_d, b_r
    __shared__ __attribute__((aligned(16))) float BDS[C];           // b_d 2^m_v (the current clip's v scale)
    __shared__ __attribute__((aligned(16))) uint16_t MBU[TMS * 8];  // u > 0 words of the tile
    __shared__ __attribute__((aligned(16))) uint16_t MBE[TMS * 8];  // e_{l+1} > 0 words
    __shared__ int MBT[TMS];                                        // time of each tile column

    const int tiles = a.T / TMS;
    const int ntiles = a.B * tiles;
    const int tid = threadIdx.x, lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int r = lane & 31, h = lane >> 5;
    const int G = (int)gridDim.x;
    STAMP_DECL

    auto tile_of = [&](int tl) { return tile_at<MASKED>(tl, a.ft, a.fn, a.d, ly); };
    auto clampt = [&](int tl) { return tl < ntiles ? tl : ntiles - 1; };

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

    int Lc[2], toff[2];
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        Lc[j] = frow(32 * j + r, ly);
        toff[j] = MASKED ? 0 : row_toff(Lc[j], ly, a.d);
    }
    const int chb = 32 * w + 4 * h;   // first channel of this lane's accumulator group g = 0
    auto ctime = [&](const Tile& t, int cc, int to) { return col_time<MASKED>(t, cc, to, a.fn, a.d); };

    // ---- row units (as block_fwd_split.hip): unit k, lane -> image row 8 k + lr ----
    const int lr = lane >> 3;
    const int cq = 32 * w + 4 * (lane & 7);
    const uint32_t imgo = (uint32_t)(lr * RS + 2 * cq);
    uint32_t soff[NU];
    uint32_t padz = 0;
#pragma unroll
    for (int k = 0; k < NU; ++k) {
        const int L = 8 * k + lr;
        const bool none = MASKED ? L > TMS + 1 : (L >= ly.nrows || pad_row(L, ly));
        if (none) padz |= 1u << k;
        soff[k] = MASKED ? 0u : (uint32_t)(((none ? 0 : row_toff(L, ly, a.d)) + a.d) * C * 4 + 4 * cq);
    }
    const uint32_t row1 = (uint32_t)(a.d * C * 4 + 4 * cq), row64 = (uint32_t)(TMS * a.d * C * 4 + 4 * cq);

    float4 ld[NU];          // rows of the next tile to convert
    rsrc_t rs_l;            // unmasked: the loading tile's row-0 source (set with the tile)
    auto set_load_tile = [&](const Tile& t) {
        if (!MASKED) rs_l = mk_rsrc(a.ein + ((ptrdiff_t)t.b * a.T + t.tb - a.d) * C);
    };
    auto load_unit = [&](const Tile& t, int k) {
        if (MASKED) {
            const int L = 8 * k + lr;
            const int pp = (padz >> k) & 1u ? t.p0 : min(max(t.p0 + L - 1, 0), a.T - 1);
            const float* src = a.ein + ((size_t)t.b * a.T + pos_time(pp, a.fn, a.d)) * C + cq;
            ld[k] = *reinterpret_cast<const float4*>(src);
            return;
        }
        uint32_t o = soff[k];
        if (ONESEG && k == 0 && lr == 0 && t.m0 == 0) o = row1;
        if (ONESEG && k == NU - 1 && lr == 1 && t.m0 + TMS >= a.n) o = row64;
        ld[k] = bld4(rs_l, o, 0u);
    };
    auto zero_bits_of = [&](const Tile& t) {
        uint32_t z = padz;
        if (ONESEG) {
            if (lr == 0 && t.m0 == 0) z |= 1u;
            if (lr == 1 && t.m0 + TMS >= a.n) z |= 1u << (NU - 1);
        }
        return z;
    };
    // conversion of unit k: relu, scale, split -> image img
    auto conv_unit = [&](int k, uint8_t* img, float s, uint32_t zb) {
        float4 v = ld[k];
        const float sk = (zb >> k) & 1u ? 0.f : s;
        v.x = __int_as_float(max(__float_as_int(v.x), 0)); v.y = __int_as_float(max(__float_as_int(v.y), 0));
        v.z = __int_as_float(max(__float_as_int(v.z), 0)); v.w = __int_as_float(max(__float_as_int(v.w), 0));
        uint32_t h01, l01, h23, l23;
        split2(v.x * sk, v.y * sk, h01, l01);
        split2(v.z * sk, v.w * sk, h23, l23);
        uint8_t* p = img + imgo + 8 * k * RS;
        *reinterpret_cast<uint2*>(p) = make_uint2(h01, h23);
        *reinterpret_cast<uint2*>(p + 256) = make_uint2(l01, l23);
    };

    auto store_me = [&](int b) {
        if (a.me_next && lane < 16) {
            const int c = 16 * w + lane;
            const int t = MBT[c];
            const int pn = (t & ((1 << a.dn_log2) - 1)) * a.nn + (t >> a.dn_log2);
            *reinterpret_cast<uint4*>(a.me_next + ((size_t)b * a.T + pn) * 8) =
                *reinterpret_cast<const uint4*>(&MBE[c * 8]);
        }
    };

    // ---- the staging rows OB (this wave's quarter, private to it): piece (j, q) = columns
    //      32 j + 8 q + lr, channels cq .. cq + 3, at image row frow(c); the tile's residual e_l
    //      comes in as whole lines (loaded in its phase A, written in its phase D), epilogue 2
    //      turns it into e_{l+1} in place, and the flush stores the rows as whole lines ----
    const uint32_t fl_lane = (uint32_t)((lr * a.d * C + cq) * 4);
    auto piece_row = [&](int j, int q) { return (MASKED || ONESEG) ? 32 * j + 8 * q + lr + 1 : 34 * j + 1 + 8 * q + lr; };
    auto piece_tu = [&](int j, int q) { return ONESEG ? (32 * j + 8 * q) * a.d : j + 8 * q * a.d; };
    float4 rrow[8];
    auto rr_load = [&](const Tile& t, int p) {
        const int j = p >> 2, q = p & 3;
        if (MASKED) {
            const int tm = pos_time(t.p0 + 32 * j + 8 * q + lr, a.fn, a.d);
            rrow[p] = *reinterpret_cast<const float4*>(a.ein + ((size_t)t.b * a.T + tm) * C + cq);
        } else {
            rrow[p] = bld4(mk_rsrc(a.ein + ((ptrdiff_t)t.b * a.T + t.tb) * C), fl_lane, (uint32_t)(piece_tu(j, q) * C * 4));
        }
    };
    auto rr_write = [&](int p) {
        *reinterpret_cast<float4*>(OB + piece_row(p >> 2, p & 3) * RS + 4 * cq) = rrow[p];
    };

    // ---- epilogue 2 of tile prv, unit u = (j, g) in three parts: residual read; e_{l+1} back
    //      into the staging rows; bits, max ----
    f32x16 acc2[2];
    Tile prv = tile_of(blockIdx.x);
    float inv2p = 0.f;
    float emax = 0.f;
    uint32_t mb[2] = {0u, 0u};
    float4 e2e, e2b, e2o;
    auto epi2_begin = [&]() { mb[0] = mb[1] = 0u; };
    auto epi2_part = [&](int u, int part) {
        const int j = u >> 2, g = u & 3;
        if (part == 0) {
            e2e = *reinterpret_cast<const float4*>(OB + Lc[j] * RS + 4 * (chb + 8 * g));
            e2b = *reinterpret_cast<const float4*>(&BIAS[C + chb + 8 * g]);
        } else if (part == 1) {
            e2o.x = e2e.x + fmaf(acc2[j][4 * g + 0], inv2p, e2b.x);
            e2o.y = e2e.y + fmaf(acc2[j][4 * g + 1], inv2p, e2b.y);
            e2o.z = e2e.z + fmaf(acc2[j][4 * g + 2], inv2p, e2b.z);
            e2o.w = e2e.w + fmaf(acc2[j][4 * g + 3], inv2p, e2b.w);
            *reinterpret_cast<float4*>(OB + Lc[j] * RS + 4 * (chb + 8 * g)) = e2o;
        } else {
            emax = fmaxf(emax, fmaxf(fmaxf(fabsf(e2o.x), fabsf(e2o.y)), fmaxf(fabsf(e2o.z), fabsf(e2o.w))));
            mb[j] = or_pos_bits4(mb[j], e2o.x, e2o.y, e2o.z, e2o.w, g);
        }
    };
    // flush piece (j, q) of tile prv: part 0 reads the row back, part 1 stores it
    float4 fl4;
    auto flush_part = [&](int j, int q, int part) {
        if (part == 0) {
            fl4 = *reinterpret_cast<const float4*>(OB + piece_row(j, q) * RS + 4 * cq);
        } else if (MASKED) {
            const int t = pos_time(prv.p0 + 32 * j + 8 * q + lr, a.fn, a.d);
            *reinterpret_cast<float4*>(a.eout + ((size_t)prv.b * a.T + t) * C + cq) = fl4;
        } else {
            bst4(mk_rsrc(a.eout + ((size_t)prv.b * a.T + prv.tb) * C), fl_lane, (uint32_t)(piece_tu(j, q) * C * 4), fl4);
        }
    };
    auto epi2_words = [&]() {
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const int c = 32 * j + r;
            MBE[c * 8 + 4 * h + w] = (uint16_t)mb[j];
            MBT[c] = ctime(prv, c, toff[j]);
        }
    };
    auto epi2_max = [&]() {
        const uint32_t m = wave_max_bits(emax);
        if (lane == 0) atomicMax(a.gmax_out + prv.b, m);
        emax = 0.f;
    };

    // ---- epilogue 1 (as block_fwd_split.hip) ----
    f32x16 acc1[2];
    float a1 = 0.f;
    float bs_sv = -1.f;
    uint32_t mu_w = 0;
    float4 e1v;
    auto epi1_part = [&](int j, int g, int part) {
        if (part == 0) {
            const float4 b4 = *reinterpret_cast<const float4*>(&BDS[chb + 8 * g]);
            e1v.x = fmaxf(fmaf(acc1[j][4 * g + 0], a1, b4.x), 0.f);
            e1v.y = fmaxf(fmaf(acc1[j][4 * g + 1], a1, b4.y), 0.f);
            e1v.z = fmaxf(fmaf(acc1[j][4 * g + 2], a1, b4.z), 0.f);
            e1v.w = fmaxf(fmaf(acc1[j][4 * g + 3], a1, b4.w), 0.f);
        } else {
            uint32_t h01, l01, h23, l23;
            split2(e1v.x, e1v.y, h01, l01);
            split2(e1v.z, e1v.w, h23, l23);
            uint8_t* p = XV + (32 * j + r) * RS + 2 * (chb + 8 * g);
            *reinterpret_cast<uint2*>(p) = make_uint2(h01, h23);
            *reinterpret_cast<uint2*>(p + 256) = make_uint2(l01, l23);
#ifdef SW_UBITS_EXACT
            mu_w = or_pos_bits4(mu_w, e1v.x, e1v.y, e1v.z, e1v.w, g);
            if (g == 3) {
                MBU[(32 * j + r) * 8 + 4 * h + w] = (uint16_t)mu_w;
                mu_w = 0;
            }
#else
            mu_w = or_bits4(mu_w, h01, h23, g);
            if (g == 3) {
                MBU[(32 * j + r) * 8 + 4 * h + w] = (uint16_t)mask16(mu_w);
                mu_w = 0;
            }
#endif
        }
    };

    // ---- GEMM 1 of column half J over image img ----
    auto gemm1h = [&](auto j_tag, auto side, const Tile& cu, const uint8_t* img) {
        constexpr int J = decltype(j_tag)::value;
        bool ok0 = true, ok2 = true;
        if (MASKED) {
            const int pc = cu.p0 + 32 * J + r;
            const int m = pc - (int)fdiv((uint32_t)pc, a.fn) * a.n;
            ok0 = m > 0;
            ok2 = m < a.n - 1;
        }
#pragma unroll
        for (int i = 0; i < 16; ++i) acc1[J][i] = 0.f;
        uint4 bh[LA + 1], bl[LA + 1];
        auto bread = [&](int st, uint4& xh, uint4& xl) {
            const int tp = st >> 3, kb = st & 7;
            const uint8_t* p = img + (Lc[J] + tp - 1) * RS + kb * 32 + h * 16;
            xh = lds16(p);
            xl = lds16(p + 256);
        };
#pragma unroll
        for (int q = 0; q < LA; ++q) bread(q, bh[q], bl[q]);
#pragma unroll
        for (int st = 0; st < 24; ++st) {
            const int tp = st >> 3, kb = st & 7, cb = st % (LA + 1);
            uint4 xh = bh[cb], xl = bl[cb];
            if (MASKED && ((tp == 0 && !ok0) || (tp == 2 && !ok2))) {
                xh = make_uint4(0, 0, 0, 0);
                xl = xh;
            }
            acc1[J] = mfma_f16(wd[tp][kb][0], xh, acc1[J]);
            if (st + LA < 24) bread(st + LA, bh[(st + LA) % (LA + 1)], bl[(st + LA) % (LA + 1)]);
            side(st);
            acc1[J] = mfma_f16(wd[tp][kb][1], xh, acc1[J]);
            acc1[J] = mfma_f16(wd[tp][kb][0], xl, acc1[J]);
            step3_schedule();
        }
    };
    auto gemm2h = [&](auto j_tag, auto side) {
        constexpr int J = decltype(j_tag)::value;
#pragma unroll
        for (int i = 0; i < 16; ++i) acc2[J][i] = 0.f;
        uint4 bh[LA + 1], bl[LA + 1];
        auto bload = [&](int kb, uint4& xh, uint4& xl) {
            const uint8_t* p = XV + (32 * J + r) * RS + kb * 32 + h * 16;
            xh = lds16(p);
            xl = lds16(p + 256);
        };
#pragma unroll
        for (int q = 0; q < LA; ++q) bload(q, bh[q], bl[q]);
#pragma unroll
        for (int kb = 0; kb < 8; ++kb) {
            const int cb = kb % (LA + 1);
            acc2[J] = mfma_f16(wr[kb][0], bh[cb], acc2[J]);
            if (kb + LA < 8) bload(kb + LA, bh[(kb + LA) % (LA + 1)], bl[(kb + LA) % (LA + 1)]);
            side(kb);
            acc2[J] = mfma_f16(wr[kb][1], bh[cb], acc2[J]);
            acc2[J] = mfma_f16(wr[kb][0], bl[cb], acc2[J]);
            step3_schedule();
        }
    };
    using J0 = std::integral_constant<int, 0>;
    using J1 = std::integral_constant<int, 1>;

    if (blockIdx.x >= ntiles) return;   // (grid = min(tiles, CUs): not taken)

    // prologue: the first tile's image; the second tile's rows in flight
    float gm_c;     // max |e_l| of the current tile's clip (at the top: the next one's)
    {
        const Tile t0 = tile_of(blockIdx.x);
        set_load_tile(t0);
#pragma unroll
        for (int k = 0; k < NU; ++k) load_unit(t0, k);
        const uint32_t z0 = zero_bits_of(t0);
        gm_c = sload(a.gmax_in + t0.b);
        const float s0 = exp2i(scale_exp(gm_c));
#pragma unroll
        for (int k = 0; k < NU; ++k) conv_unit(k, &IMG[0][0], s0, z0);
        const Tile t1 = tile_of(clampt(blockIdx.x + G));
        set_load_tile(t1);
#pragma unroll
        for (int k = 0; k < NU; ++k) load_unit(t1, k);
    }

    STAMP(13)
    auto tile_body = [&](auto first_tag, int tile, int it) {
        constexpr bool FIRST = decltype(first_tag)::value;
        const Tile cu = tile_of(tile);
        const Tile nt = tile_of(clampt(tile + G));
        const Tile n2 = tile_of(clampt(tile + 2 * G));
        set_load_tile(n2);   // (tile i+1's loads were all issued in the previous tile)
        lds_barrier();       // T: image i complete (converted in the previous tile's A / B)
        STAMP(0)
        const float gm = gm_c;
        const int m_e = scale_exp(gm);
        const int m_v = scale_exp(fmaf(a.wdn, gm, a.bdm));
        if (nt.b != cu.b) gm_c = sload(a.gmax_in + nt.b);   // (usually the same clip: tile order)
        const float s_next = exp2i(scale_exp(gm_c));
        const uint32_t zn = zero_bits_of(nt);
        const float sv = exp2i(m_v);
        a1 = exp2i(m_v - m_e - a.kd);
        if (sv != bs_sv) {
            bs_sv = sv;
            if (lane < 32) BDS[32 * w + lane] = BIAS[32 * w + lane] * sv;
        }
        const uint8_t* imc = &IMG[it & 1][0];
        uint8_t* imn = &IMG[(it & 1) ^ 1][0];

        STAMP(10)
        // A: GEMM 1 half 0 + this tile's residual rows (loads) + epilogue 2 of the previous tile
        //    and the flush of its half 0 + conversion units 0..4 (each unit's registers reloaded
        //    with tile i+2 right away)
        if (!FIRST) epi2_begin();
        gemm1h(J0{}, [&](int st) {
            if (st < 2) {   // (issued before this tile's row loads: their waits do not include those)
#pragma unroll
                for (int p = 0; p < 4; ++p) rr_load(cu, 4 * st + p);
            }
            if (!FIRST) {
                epi2_part(st / 3, st % 3);
                if (st >= 12 && st < 20) flush_part(0, (st - 12) >> 1, st & 1);
            }
            if (st % 5 == 2) {   // steps 2 7 12 17 22: units 0..4
                conv_unit(st / 5, imn, s_next, zn);
                load_unit(n2, st / 5);
            }
        }, cu, imc);
        if (!FIRST) {
            epi2_words();
            if (cu.b != prv.b) epi2_max();
        }
        STAMP(5)
        // B: GEMM 1 half 1 + epilogue 1 of half 0 + the flush of epilogue 2's half 1 +
        //    conversion units 5..8
        gemm1h(J1{}, [&](int st) {
            if (st < 8) epi1_part(0, st >> 1, st & 1);
            else if (!FIRST && st < 16) flush_part(1, (st - 8) >> 1, st & 1);
            if (st >= 9 && st % 4 == 1) {   // steps 9 13 17 21: units 5..8
                conv_unit(5 + (st - 9) / 4, imn, s_next, zn);
                load_unit(n2, 5 + (st - 9) / 4);
            }
        }, cu, imc);
        lds_barrier();   // v image half 0, u > 0 words half 0, e > 0 words of tile i-1
        STAMP(1)
        if (!FIRST) store_me(prv.b);
        // C: GEMM 2 half 0 + epilogue 1 of half 1
        gemm2h(J0{}, [&](int kb) { epi1_part(1, kb >> 1, kb & 1); });
        lds_barrier();   // v image half 1, all u > 0 words
        STAMP(2)
        if (lane < 16)
            *reinterpret_cast<uint4*>(a.mu + ((size_t)cu.b * a.T + cu.p0 + 16 * w + lane) * 8) =
                *reinterpret_cast<const uint4*>(&MBU[(16 * w + lane) * 8]);
        // D: GEMM 2 half 1 + this tile's residual rows into the staging rows (the flush of the
        //    previous tile's rows ended in B)
        gemm2h(J1{}, [&](int kb) { rr_write(kb); });
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
        epi2_begin();
#pragma unroll
        for (int st = 0; st < 24; ++st) epi2_part(st / 3, st % 3);
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            flush_part(q >> 2, q & 3, 0);
            flush_part(q >> 2, q & 3, 1);
        }
        epi2_words();
        epi2_max();
        lds_barrier();
        store_me(prv.b);
    }
    STAMP(4)
    STAMP_FLUSH(a.stamps)
}

}  // namespace

bool launch_block_fwd_db(const FwdArgsS& a0, hipStream_t s) {
    FwdArgsS a = a0;
    a.fn = make_fdiv((uint32_t)a.n);
    a.ft = make_fdiv((uint32_t)(SW_TILE_INTERLEAVE ? a.B : a.T / TMS));
    const int nt = a.B * (a.T / TMS);
    const dim3 grid(std::min(nt, sw::num_cus()));
    Layout ly;
    const bool masked = pick_layout(a.n, ly);
    if (masked) hipLaunchKernelGGL((k_block_fwd_db<true, false>), grid, dim3(FT), 0, s, a, ly);
    else if (ly.M == TMS) hipLaunchKernelGGL((k_block_fwd_db<false, true>), grid, dim3(FT), 0, s, a, ly);
    else hipLaunchKernelGGL((k_block_fwd_db<false, false>), grid, dim3(FT), 0, s, a, ly);
    return true;
}

}  // namespace ast
