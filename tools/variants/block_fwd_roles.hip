// Split-fp16 encoder block forward (precision 2), role-split form: model.py:95-116 for one
// block,
//   u = dconv_d(relu(e_l)) + b_d        (masked.py:110-160, K = 3, SAME zero padding)
//   e_{l+1} = e_l + W_r^T relu(u) + b_r
// with the numerics of block_fwd_split.hip (split fp16 operands, three products, fp32
// accumulation and epilogues, power-of-two scales: splitwave.h) and bit-identical results.
//
// Why roles.  The one-wave-per-SIMD kernel (block_fwd_split.hip) holds 256 weight registers per
// wave, so a SIMD has one wave and every epilogue, conversion and load has to be hand-placed in
// the shadow of that wave's own MFMAs (~10.9k cycles per 64-position tile against a 6.1k MFMA
// floor).  Here a 512-thread workgroup puts TWO waves on every SIMD:
//   waves 0..3, "dconv waves": output channels 32 w .. 32 w + 31 of GEMM 1 (the dilated conv)
//     and its epilogue 1 (u, u > 0 bits, split v image); W_d's split fragments (3 taps x 8
//     k-blocks x hi/lo = 192 registers) stay in registers;
//   waves 4..7, "residual waves": channels 32 (w-4) ..: row loads and the split image of the
//     next tile, GEMM 2 (W_r, 64 registers), epilogue 2 (residual, e > 0 bits, per-clip max,
//     stores).
// The SIMD's matrix pipe interleaves both waves' MFMAs and each wave's vector work issues in
// the other's MFMA gaps.  Neither wave uses AGPRs (both roles fit 256 registers).
//
// Pipeline (K = this workgroup's tiles; one barrier per period, all 8 waves pass every one):
//   dconv,    period k: GEMM 1 + epilogue 1 of tile k (image IMG[k&1] -> v image XV[k&1])
//   residual, period k: GEMM 2 + epilogue 2 of tile k-1 (XV[(k-1)&1] -> e_{l+1}), the mask
//             words of tiles k-1 / k-2, the conversion of tile k+1 (-> IMG[(k+1)&1]) and the
//             residual rows of tile k
// Every LDS buffer that crosses a barrier is double-buffered by tile parity.
#include "splitwave.h"
#include <algorithm>
#include <type_traits>

namespace ast {
namespace {
using namespace sw;

constexpr int FR = 512;                      // threads: two waves per SIMD
constexpr int IRW = 68;                      // image rows (66 one-segment / masked, 68 two-segment)
constexpr int ISL = IRW * RS;                // bytes per image buffer
constexpr int LA = 2;                        // B-fragment lookahead (steps), GEMM 1
constexpr int LB = 1;                        // GEMM 2 (the residual wave's registers are the scarce ones)
constexpr int L_BIAS = 0, L_BDS = L_BIAS + 2 * C * 4, L_MBU = L_BDS + C * 4, L_MBE = L_MBU + 2 * TMS * 16,
              L_XV = L_MBE + 2 * TMS * 16, L_IMG = L_XV + 2 * TMS * RS, L_END = L_IMG + 2 * ISL;
static_assert(L_END <= 163840, "LDS");

template <bool MASKED, bool ONESEG>
__global__ void __launch_bounds__(FR, 1) k_block_fwd_r(FwdArgsS a, Layout ly) {
    // one LDS block, the small arrays first (their addresses stay within the 16-bit DS offset
    // of one base register)
    __shared__ __attribute__((aligned(16))) uint8_t SM[L_END];
    float* const BIAS = reinterpret_cast<float*>(SM + L_BIAS);    // b_d, b_r
    float* const BDS = reinterpret_cast<float*>(SM + L_BDS);      // b_d 2^m_v (per dconv wave)
    auto MBU = [&](int k) { return reinterpret_cast<uint16_t*>(SM + L_MBU + (k & 1) * TMS * 16); };  // u > 0 words
    auto MBE = [&](int k) { return reinterpret_cast<uint16_t*>(SM + L_MBE + (k & 1) * TMS * 16); };  // e > 0 words
    auto XVP = [&](int k) { return SM + L_XV + (k & 1) * TMS * RS; };   // split v images
    auto IMGP = [&](int k) { return SM + L_IMG + (k & 1) * ISL; };      // split relu(e_l) images

    const int tiles = a.T / TMS;
    const int ntiles = a.B * tiles;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int w = wv & 3;
    const int r = lane & 31, h = lane >> 5;
    const int G = (int)gridDim.x;
    const int K = ((int)blockIdx.x < ntiles) ? (ntiles - (int)blockIdx.x + G - 1) / G : 0;
    STAMP_DECL

    auto tile_of = [&](int tl) { return tile_at<MASKED>(tl, a.ft, a.fn, a.d, ly); };
    auto tile_k = [&](int k) { const int tl = (int)blockIdx.x + k * G; return tile_of(tl < ntiles ? tl : ntiles - 1); };

    int Lc[2], toff[2];
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        Lc[j] = frow(32 * j + r, ly);
        toff[j] = MASKED ? 0 : row_toff(Lc[j], ly, a.d);
    }
    const int chb = 32 * w + 4 * h;   // first channel of this lane's accumulator group g = 0

    // ---- the scales of a clip: image scale 2^m_e, v scale 2^m_v (splitwave.h) ----
    int sc_b = -1;          // clip whose max gm_b holds
    float gm_b = 0.f;
    auto clip_max = [&](int b) {
        if (b != sc_b) { sc_b = b; gm_b = sload(a.gmax_in + b); }
        return gm_b;
    };

    // e_{l+1} > 0 words of a finished tile -> next layer's positions (wave w: columns 16 w..; stored by the dconv
    // waves, which have the slack)
    auto ctime = [&](const Tile& t, int cc, int to) { return col_time<MASKED>(t, cc, to, a.fn, a.d); };
    auto store_me = [&](const Tile& et, const uint16_t* mbe) {
        if (a.me_next && lane < 16) {
            const int c = 16 * w + lane;
            const int L = frow(c, ly);
            const int t = ctime(et, c, MASKED ? 0 : row_toff(L, ly, a.d));
            const int pn = (t & ((1 << a.dn_log2) - 1)) * a.nn + (t >> a.dn_log2);
            *reinterpret_cast<uint4*>(a.me_next + ((size_t)et.b * a.T + pn) * 8) =
                *reinterpret_cast<const uint4*>(&mbe[c * 8]);
        }
    };
    auto store_mu = [&](const Tile& et, const uint16_t* mbu) {
        if (lane < 16)
            *reinterpret_cast<uint4*>(a.mu + ((size_t)et.b * a.T + et.p0 + 16 * w + lane) * 8) =
                *reinterpret_cast<const uint4*>(&mbu[(16 * w + lane) * 8]);
    };

    if (wv < 4) {
        // ================= dconv wave: GEMM 1 + epilogue 1 =================
        uint4 wd[3][8][2];
#pragma unroll
        for (int tp = 0; tp < 3; ++tp)
#pragma unroll
            for (int kb = 0; kb < 8; ++kb)
#pragma unroll
                for (int hl = 0; hl < 2; ++hl)
                    wd[tp][kb][hl] = a.wdf[((size_t)((w * 3 + tp) * 8 + kb) * 2 + hl) * 64 + lane];
        constexpr int LAD = LA;
        f32x16 acc[2];          // column halves: epilogue 1 of half 0 rides in GEMM 1 half 1
        auto gemm1h = [&](auto j_tag, const uint8_t* img, const Tile& cu, auto side) {
            constexpr int J = decltype(j_tag)::value;
            bool ok0 = true, ok2 = true;
            if (MASKED) {
                const int pc = cu.p0 + 32 * J + r;
                const int m = pc - (int)fdiv((uint32_t)pc, a.fn) * a.n;
                ok0 = m > 0;
                ok2 = m < a.n - 1;
            }
#pragma unroll
            for (int i = 0; i < 16; ++i) acc[J][i] = 0.f;
            uint4 bh[LAD + 1], bl[LAD + 1];
            auto bread = [&](int st, uint4& xh, uint4& xl) {
                const int tp = st >> 3, kb = st & 7;
                const uint8_t* p = img + (Lc[J] + tp - 1) * RS + kb * 32 + h * 16;
                xh = lds16(p);
                xl = lds16(p + 256);
            };
#pragma unroll
            for (int q = 0; q < LAD; ++q) bread(q, bh[q], bl[q]);
#pragma unroll
            for (int st = 0; st < 24; ++st) {
                const int tp = st >> 3, kb = st & 7, cb = st % (LAD + 1);
                uint4 xh = bh[cb], xl = bl[cb];
                if (MASKED && ((tp == 0 && !ok0) || (tp == 2 && !ok2))) {
                    xh = make_uint4(0, 0, 0, 0);
                    xl = xh;
                }
                acc[J] = mfma_f16(wd[tp][kb][0], xh, acc[J]);
                if (st + LAD < 24) bread(st + LAD, bh[(st + LAD) % (LAD + 1)], bl[(st + LAD) % (LAD + 1)]);
                side(st);
                acc[J] = mfma_f16(wd[tp][kb][1], xh, acc[J]);
                acc[J] = mfma_f16(wd[tp][kb][0], xl, acc[J]);
            }
        };
        // epilogue 1 of column half j: v = relu(acc 2^(m_v - m_e - k_d) + b_d 2^m_v) (the scale
        // folded into the fma; powers of two: the same values), split -> v image; u > 0 bits from
        // the rtz hi halves (splitwave.h nz2)
        uint32_t mu_w = 0;
        auto epi1g = [&](int j, int g, uint8_t* xv, uint16_t* mbu, float a1) {
            const float4 b4 = *reinterpret_cast<const float4*>(&BDS[chb + 8 * g]);
            const float vx = fmaxf(fmaf(acc[j][4 * g + 0], a1, b4.x), 0.f);
            const float vy = fmaxf(fmaf(acc[j][4 * g + 1], a1, b4.y), 0.f);
            const float vz = fmaxf(fmaf(acc[j][4 * g + 2], a1, b4.z), 0.f);
            const float vw = fmaxf(fmaf(acc[j][4 * g + 3], a1, b4.w), 0.f);
            uint32_t h01, l01, h23, l23;
            split2(vx, vy, h01, l01);
            split2(vz, vw, h23, l23);
            uint8_t* p = xv + (32 * j + r) * RS + 2 * (chb + 8 * g);
            *reinterpret_cast<uint2*>(p) = make_uint2(h01, h23);
            *reinterpret_cast<uint2*>(p + 256) = make_uint2(l01, l23);
            mu_w = or_bits4(g == 0 ? 0u : mu_w, h01, h23, g);
            if (g == 3) mbu[(32 * j + r) * 8 + 4 * h + w] = (uint16_t)mask16(mu_w);
        };
        using J0 = std::integral_constant<int, 0>;
        using J1 = std::integral_constant<int, 1>;
#ifdef SW_DCONV_PRIO
        __builtin_amdgcn_s_setprio(SW_DCONV_PRIO);
#endif
        float bs_sv = -1.f;     // the v scale BDS holds
        lds_barrier();                                      // S_0: image 0 complete, BIAS
        STAMP(14)
        for (int k = 0; k <= K; ++k) {
            if (k < K) {
                const Tile cu = tile_k(k);
                const float gm = clip_max(cu.b);
                const int m_e = scale_exp(gm);
                const int m_v = scale_exp(fmaf(a.wdn, gm, a.bdm));
                const float sv = exp2i(m_v);
                const float a1 = exp2i(m_v - m_e - a.kd);
                if (sv != bs_sv) {   // only this wave reads its channels' entries, in program order
                    bs_sv = sv;
                    if (lane < 32) BDS[32 * w + lane] = BIAS[32 * w + lane] * sv;
                }
                gemm1h(J0{}, IMGP(k), cu, [&](int) {});
                STAMP(6)
                if (ONESEG) {
                    gemm1h(J1{}, IMGP(k), cu, [&](int st) {   // epilogue 1 of half 0, steps 2..9
                        if (st >= 2 && st < 10 && (st & 1) == 0) epi1g(0, (st - 2) >> 1, XVP(k), MBU(k), a1);
                    });
                } else {   // (the other layouts' residual waves need the registers)
#pragma unroll
                    for (int g = 0; g < 4; ++g) epi1g(0, g, XVP(k), MBU(k), a1);
                    gemm1h(J1{}, IMGP(k), cu, [&](int) {});
                }
                STAMP(8)
#pragma unroll
                for (int g = 0; g < 4; ++g) epi1g(1, g, XVP(k), MBU(k), a1);
                STAMP(9)
            }
            // mask words of tiles k-1 (u > 0, this role's) and k-2 (e > 0, the residual waves')
            if (k >= 1) store_mu(tile_k(k - 1), MBU(k - 1));
            if (k >= 2) store_me(tile_k(k - 2), MBE(k - 2));
            STAMP(1)
            lds_barrier();                                  // S_{k+1}
            STAMP(10)
        }
        if (K > 0) store_me(tile_k(K - 1), MBE(K - 1));
        STAMP_FLUSH(a.stamps)
        return;
    }

    // ================= residual wave =================
#ifdef SW_RESID_PRIO
    __builtin_amdgcn_s_setprio(SW_RESID_PRIO);
#endif
    uint4 wr[8][2];
#pragma unroll
    for (int kb = 0; kb < 8; ++kb)
#pragma unroll
        for (int hl = 0; hl < 2; ++hl)
            wr[kb][hl] = a.wrf[((size_t)(w * 8 + kb) * 2 + hl) * 64 + lane];
    {
        const int t = tid - 256;
        if (t < C) { BIAS[t] = a.bd[t]; BIAS[C + t] = a.br[t]; }
    }
    // ---- rows of the next tile (RowUnits: unit k = image rows 8 k .. 8 k + 7 x this wave's
    //      32 channels) -> split image ----
    RowUnits<MASKED, ONESEG> ru;
    ru.init(w, lane, ly, a.d);
    float4 ld[NU];
    // one-segment layouts: unit k's source rows are rows 8 k + lr (k < 8) = the tile's row-0
    // time + (8 k + lr) d, so no per-unit offset table (RowUnits::soff) is kept in registers
    const uint32_t lr_off = (uint32_t)(ru.lr * a.d * C * 4 + 4 * ru.cq);
    const uint32_t u8_off = ru.lr < 2 ? (uint32_t)((TMS + ru.lr) * a.d * C * 4 + 4 * ru.cq) : ru.row1;
    auto load_unit = [&](const Tile& t, int k) {
        if (MASKED) {
            ld[k] = ru.load(a.ein, t, k, a.T, a.fn, a.d);
            return;
        }
        // the tile's row-0 source (time tb - d) as the resource base, 32-bit lane offsets
        const rsrc_t rs = mk_rsrc(a.ein + ((ptrdiff_t)t.b * a.T + t.tb - a.d) * C);
        if (ONESEG) {
            uint32_t o = k < NU - 1 ? lr_off : u8_off;
            if (k == 0 && ru.lr == 0 && t.m0 == 0) o = ru.row1;
            if (k == NU - 1 && ru.lr == 1 && t.m0 + TMS >= (int)a.fn.n) o = ru.row64;
            ld[k] = bld4(rs, o, k < NU - 1 ? (uint32_t)(k * 8 * a.d * C * 4) : 0u);
        } else {
            ld[k] = bld4(rs, ru.soff[k], 0u);
        }
    };
    auto conv_unit = [&](int k, uint8_t* img, float s, uint32_t zb) {
        float4 v = ld[k];
        const float sk = (zb >> k) & 1u ? 0.f : s;
        v.x = __int_as_float(max(__float_as_int(v.x), 0)); v.y = __int_as_float(max(__float_as_int(v.y), 0));
        v.z = __int_as_float(max(__float_as_int(v.z), 0)); v.w = __int_as_float(max(__float_as_int(v.w), 0));
        uint32_t h01, l01, h23, l23;
        split2(v.x * sk, v.y * sk, h01, l01);
        split2(v.z * sk, v.w * sk, h23, l23);
        if (k < NU - 1 || ru.lr < IRW - 8 * (NU - 1)) {   // rows past the image are never read
            uint8_t* p = img + ru.imgo + 8 * k * RS;
            *reinterpret_cast<uint2*>(p) = make_uint2(h01, h23);
            *reinterpret_cast<uint2*>(p + 256) = make_uint2(l01, l23);
        }
    };

    // ---- GEMM 2 of column half J over the v image ----
    f32x16 acc2[2];         // GEMM 2 column halves (epilogue 2 of half 0 rides in half 1)
    auto gemm2h = [&](auto j_tag, const uint8_t* xv, auto side) {
        constexpr int J = decltype(j_tag)::value;
#pragma unroll
        for (int i = 0; i < 16; ++i) acc2[J][i] = 0.f;
        uint4 bh[LB + 1], bl[LB + 1];
        auto bload = [&](int kb, uint4& xh, uint4& xl) {
            const uint8_t* p = xv + (32 * J + r) * RS + kb * 32 + h * 16;
            xh = lds16(p);
            xl = lds16(p + 256);
        };
#pragma unroll
        for (int q = 0; q < LB; ++q) bload(q, bh[q], bl[q]);
#pragma unroll
        for (int kb = 0; kb < 8; ++kb) {
            const int cb = kb % (LB + 1);
            acc2[J] = mfma_f16(wr[kb][0], bh[cb], acc2[J]);
            if (kb + LB < 8) bload(kb + LB, bh[(kb + LB) % (LB + 1)], bl[(kb + LB) % (LB + 1)]);
            side(kb);
            acc2[J] = mfma_f16(wr[kb][1], bh[cb], acc2[J]);
            acc2[J] = mfma_f16(wr[kb][0], bl[cb], acc2[J]);
            __builtin_amdgcn_sched_barrier(0);   // keeps each step's side work in its step
        }
    };

    // ---- epilogue 2 (tile et, column half j): e_{l+1} = e_l + y 2^-(m_v + k_r) + b_r, stored
    //      from the accumulator layout; e > 0 bits; max |e_{l+1}| of the clip ----
    float4 res[2][4];       // residual e_l of the two column halves, accumulator layout
    // column c = 32 j + r of tile t: time tb + toff[j] (unmasked layouts; masked: gathered)
    const uint32_t colo[2] = {(uint32_t)((toff[0] * C + chb) * 4), (uint32_t)((toff[1] * C + chb) * 4)};
    auto col_base = [&](const float* ten, const Tile& t, int j) {
        return ten + ((size_t)t.b * a.T + (MASKED ? ctime(t, 32 * j + r, 0) : t.tb)) * C + (MASKED ? chb : 0);
    };
    auto load_res = [&](const Tile& et, int j) {
        if (MASKED) {
            const float* src = col_base(a.ein, et, j);
#pragma unroll
            for (int g = 0; g < 4; ++g) res[j][g] = *reinterpret_cast<const float4*>(src + 8 * g);
        } else {
            const rsrc_t rs = mk_rsrc(col_base(a.ein, et, j));
#pragma unroll
            for (int g = 0; g < 4; ++g) res[j][g] = bld4(rs, colo[j] + 32 * g, 0u);
        }
    };
    float emax = 0.f;
    int emax_b = -1;
    auto flush_max = [&]() {
        if (emax_b >= 0) {
            const uint32_t m = wave_max_bits(emax);
            if (lane == 0) atomicMax(a.gmax_out + emax_b, m);
        }
        emax = 0.f;
    };
    // epilogue 2 of column half j, accumulator group g (4 channels x the lane's column); the
    // e > 0 bits gather in mb and go to the word after group 3
    uint32_t mb = 0;
    auto epi2g = [&](const Tile& et, int j, int g, float inv2, uint16_t* mbe) {
        float* dst = const_cast<float*>(col_base(a.eout, et, j));
        const float4 b4 = *reinterpret_cast<const float4*>(&BIAS[C + chb + 8 * g]);
        float4 o;
        o.x = res[j][g].x + fmaf(acc2[j][4 * g + 0], inv2, b4.x);
        o.y = res[j][g].y + fmaf(acc2[j][4 * g + 1], inv2, b4.y);
        o.z = res[j][g].z + fmaf(acc2[j][4 * g + 2], inv2, b4.z);
        o.w = res[j][g].w + fmaf(acc2[j][4 * g + 3], inv2, b4.w);
        if (MASKED) *reinterpret_cast<float4*>(dst + 8 * g) = o;
        else bst4(mk_rsrc(dst), colo[j] + 32 * g, 0u, o);
        emax = fmaxf(emax, fmaxf(fmaxf(fabsf(o.x), fabsf(o.y)), fmaxf(fabsf(o.z), fabsf(o.w))));
        mb = or_pos_bits4(g == 0 ? 0u : mb, o.x, o.y, o.z, o.w, g);
        if (g == 3) mbe[(32 * j + r) * 8 + 4 * h + w] = (uint16_t)mb;
    };
    using J0 = std::integral_constant<int, 0>;
    using J1 = std::integral_constant<int, 1>;

    // Every vector-memory operation of the loop below is unconditional (tiles past the end are
    // clamped to a real tile: loaded and converted into an image nobody reads), so the
    // compiler's counted waits see one sequence of loads and stores on every path: a load or
    // store issued on some paths only makes it wait for everything younger on the others.
    // prologue: tile 0's image, tile 1's rows in flight; period 0: tile 1's image
    auto convert = [&](int k) {   // tile k + 1 -> IMG[(k+1)&1], units reloaded with tile k + 2
        const Tile nt = tile_k(k + 1), n2 = tile_k(k + 2);
        const float sn = exp2i(scale_exp(clip_max(nt.b)));
        const uint32_t zn = ru.zero_bits(nt, a.fn);
#pragma unroll
        for (int u = 0; u < NU; ++u) { conv_unit(u, IMGP(k + 1), sn, zn); load_unit(n2, u); }
    };
    {
        const Tile t0 = tile_k(0), t1 = tile_k(1);
#pragma unroll
        for (int k = 0; k < NU; ++k) load_unit(t0, k);
        const float s0 = exp2i(scale_exp(clip_max(t0.b)));
        const uint32_t z0 = ru.zero_bits(t0, a.fn);
#pragma unroll
        for (int k = 0; k < NU; ++k) conv_unit(k, IMGP(0), s0, z0);
#pragma unroll
        for (int k = 0; k < NU; ++k) load_unit(t1, k);
    }
    lds_barrier();                                          // S_0 (BIAS too)
    STAMP(13)
    convert(0);
    STAMP(12)
    lds_barrier();                                          // S_1
    STAMP(4)
    auto period = [&](int k) {
        // GEMM 2 + epilogue 2 of tile k - 1; conversion of tile k + 1
        const Tile et = tile_k(k - 1);
        const Tile nt = tile_k(k + 1), n2 = tile_k(k + 2);
        const float s_next = exp2i(scale_exp(clip_max(nt.b)));
        const uint32_t zn = ru.zero_bits(nt, a.fn);
        const float gm = clip_max(et.b);
        const int m_v = scale_exp(fmaf(a.wdn, gm, a.bdm));
        const float inv2 = exp2i(-(m_v + a.kr));
        if (et.b != emax_b) { flush_max(); emax_b = et.b; }
        // each half's residual rows are loaded in front of its GEMM 2 (L2-warm: the same rows
        // were loaded for the image two periods ago)
        STAMP(11)
        load_res(et, 0);
        gemm2h(J0{}, XVP(k - 1), [&](int kb) {
            if (kb < 5) { conv_unit(kb, IMGP(k + 1), s_next, zn); load_unit(n2, kb); }
            if (kb == 5) load_res(et, 1);
        });
        STAMP(0)
        gemm2h(J1{}, XVP(k - 1), [&](int kb) {
            if (kb < 4) { conv_unit(5 + kb, IMGP(k + 1), s_next, zn); load_unit(n2, 5 + kb); }
            if (kb >= 4) epi2g(et, 0, kb - 4, inv2, MBE(k - 1));
        });
        STAMP(3)
#pragma unroll
        for (int g = 0; g < 4; ++g) epi2g(et, 1, g, inv2, MBE(k - 1));
        STAMP(5)
        lds_barrier();                                      // S_{k+1}
        STAMP(4)
    };
    // period 1 is peeled: the loop is entered from a full period, so the compiler's counted
    // waits at its top see the same vector-memory history on both edges (entered from period 0,
    // its nine row loads alone, the first conversion would wait for nearly every load of the
    // previous period)
    if (K >= 1) {
        period(1);
        for (int k = 2; k <= K; ++k) period(k);
    }
    if (K > 0) flush_max();
    STAMP_FLUSH(a.stamps)
}

}  // namespace

bool launch_block_fwd_roles(const FwdArgsS& a0, hipStream_t s) {
    FwdArgsS a = a0;
    a.fn = make_fdiv((uint32_t)a.n);
    a.ft = make_fdiv((uint32_t)(SW_TILE_INTERLEAVE ? a.B : a.T / TMS));
    const int nt = a.B * (a.T / TMS);
    const dim3 grid(std::min(nt, sw::num_cus()));
    Layout ly;
    const bool masked = pick_layout(a.n, ly);
    if (masked) hipLaunchKernelGGL((k_block_fwd_r<true, false>), grid, dim3(FR), 0, s, a, ly);
    else if (ly.M == TMS) hipLaunchKernelGGL((k_block_fwd_r<false, true>), grid, dim3(FR), 0, s, a, ly);
    else hipLaunchKernelGGL((k_block_fwd_r<false, false>), grid, dim3(FR), 0, s, a, ly);
    return true;
}

}  // namespace ast
