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
// Per tile of 64 positions (one workgroup per CU, wave w owns channels 32 w .. 32 w + 31):
//   top     wait for this tile's tot rows and mask words (DMA'd during the previous tile), B1;
//           DMA this tile's D_l rows and the next tile's tot rows and mask words
//   convert tot 2^m_t -> split image (m_t from the clip's max |tot|), B2
//   step 1  g_v = W_r tot for the tile columns (+ the two halo rows of one-segment layouts),
//           g_u = [u > 0] g_v, wave max -> LDS, B3; g_u 2^m_u -> split image, D_l landed, B4
//   step 2  g_a = 3 taps x 8 k-blocks x 2 column tiles x 3 products
//   epi     out = tot + [e_l > 0] g_a + D_l -> HBM (fp32); max |out| -> the clip's atomic max
// Only DMA reads global memory (the compiler never waits on an in-flight DMA it cannot see);
// every wave issues the same vector-memory sequence: D_l (9), next rows (9), masks (1), then
// 8 row stores and 1 atomic.
#include "splitwave.h"
#include <algorithm>

namespace ast {
namespace {
using namespace sw;

constexpr int MSLOT = 3 * 1024;   // mask words per tile (u16 index): u > 0 [64][8] at 0, e_l > 0
                                  // [64][8] at 512, halo u > 0 [2][8] at 1024

// D_l rows: LDS row c = tile column c (64 rows, stride RS), 9 one-KiB groups per wave
template <bool MASKED>
struct ColDma {
    int soff[DPW], srow[DPW], schk[DPW];
    bool real[DPW];
    __device__ __forceinline__ void init(int w, int lane, const Layout& ly, int d) {
#pragma unroll
        for (int j = 0; j < DPW; ++j) {
            const int o = (w + 4 * j) * 1024 + lane * 16;
            const int L = o / RS, qc = (o - L * RS) >> 4;
            srow[j] = L;
            schk[j] = qc < 32 ? qc : 0;
            real[j] = L < TMS;
            soff[j] = (MASKED || !real[j]) ? 0 : row_toff(frow(L, ly), ly, d) * C + schk[j] * 4;
        }
    }
    __device__ __forceinline__ void issue(int j, const float* src, const Tile& t, const float* zero,
                                          uint32_t lds0, int T, int n, int d) const {
        const float* p = zero;
        if (real[j]) {
            if (MASKED) {
                const int pp = t.p0 + srow[j];
                p = src + ((size_t)t.b * T + (pp % n) * d + pp / n) * C + schk[j] * 4;
            } else {
                p = src + ((size_t)t.b * T + t.tb) * C + soff[j];
            }
        }
        dma16(p, lds0 + j * 4096);
    }
};

template <bool MASKED, bool ONESEG, bool HAS_D>
__global__ void __launch_bounds__(FT, 1) k_block_bwd_s(BwdArgsS a, Layout ly) {
    __shared__ __attribute__((aligned(16))) uint8_t XF[2][SLOT];    // fp32 tot rows
    __shared__ __attribute__((aligned(16))) uint8_t XS[SLOT];       // split tot, then split g_u
    __shared__ __attribute__((aligned(16))) uint8_t XD[SLOT];       // fp32 D_l rows (row = column)
    __shared__ __attribute__((aligned(16))) uint8_t MK[2][MSLOT];   // mask words
    __shared__ __attribute__((aligned(16))) uint8_t SCR[1024];      // wave 3's dummy mask group
    __shared__ float RED[4];

    const int tiles = a.T / TMS;
    const int ntiles = a.B * tiles;
    const int tid = threadIdx.x, lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int r = lane & 31, h = lane >> 5;

    auto tile_of = [&](int tl) { return tile_at<MASKED>(tl, tiles, a.n, a.d, ly); };
    RowDma<MASKED> dma;
    dma.init(w, lane, ly, a.d);
    ColDma<MASKED> ddma;
    if (HAS_D) ddma.init(w, lane, ly, a.d);
    // tot rows + mask words of tile tl into slot s: wave 0 the u > 0 words of the 64 columns,
    // wave 1 the e_l > 0 words, wave 2 the halo u > 0 words (lanes 0, 1), wave 3 a dummy group
    auto issue_tile = [&](int tl, int s) {
        const Tile t = tile_of(tl);
        dma.aim(a.tin, t, ly, a.T, a.n);
        const uint32_t lds0 = (uint32_t)(uintptr_t)&XF[s][0] + (uint32_t)(w * 1024);
#pragma unroll
        for (int j = 0; j < DPW; ++j) dma.issue(j, a.tin, a.zero, lds0, a.T, a.n, a.d);
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
    if (blockIdx.x < ntiles) issue_tile(blockIdx.x, 0);

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
    __syncthreads();

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

    int it = 0;
    STAMP_DECL
    for (int tile = blockIdx.x; tile < ntiles; tile += gridDim.x, ++it) {
        const int cur = it & 1;
        const Tile cu = tile_of(tile);
        if (it) asm volatile("s_waitcnt vmcnt(9)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        if (HAS_D) {
            const uint32_t lds0 = (uint32_t)(uintptr_t)&XD[0] + (uint32_t)(w * 1024);
#pragma unroll
            for (int j = 0; j < DPW; ++j) ddma.issue(j, a.dadd, cu, a.zero, lds0, a.T, a.n, a.d);
        }
        issue_tile(tile + (int)gridDim.x < ntiles ? tile + (int)gridDim.x : ntiles - 1, cur ^ 1);

        STAMP(6)
        const int m_t = scale_exp(sload(a.gmax_in + cu.b));
        convert_rows<false>(&XF[cur][0], XS, ly.nrows, exp2i(m_t), w, lane);
        lds_barrier();     // B2
        STAMP(7)

        bool ok0[2] = {true, true}, ok2[2] = {true, true};
        if (MASKED) {
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                const int m = (cu.p0 + 32 * j + r) % a.n;
                ok0[j] = m > 0;
                ok2[j] = m < a.n - 1;
            }
        }
        const uint16_t* mk = reinterpret_cast<const uint16_t*>(&MK[cur][0]);

        // ---- step 1: g_v = W_r tot (columns, halo rows), g_u = [u > 0] g_v ----
        f32x16 acc[2], acch;
#pragma unroll
        for (int i = 0; i < 16; ++i) { acc[0][i] = 0.f; acc[1][i] = 0.f; acch[i] = 0.f; }
        {
            uint4 bh[2][3], bl[2][3];
            auto bload = [&](int kb, uint4 (&xh)[3], uint4 (&xl)[3]) {
#pragma unroll
                for (int j = 0; j < (ONESEG ? 3 : 2); ++j) {
                    const uint8_t* p = XS + (j < 2 ? Lc[j] : Lh) * RS + kb * 32 + h * 16;
                    xh[j] = lds16(p);
                    xl[j] = lds16(p + 256);
                }
            };
            bload(0, bh[0], bl[0]);
#pragma unroll
            for (int kb = 0; kb < 8; ++kb) {
                const int cb = kb & 1;
                if (kb + 1 < 8) bload(kb + 1, bh[cb ^ 1], bl[cb ^ 1]);
#pragma unroll
                for (int j = 0; j < 2; ++j)
                    acc[j] = mfma3(wr[kb][0], wr[kb][1], bh[cb][j], bl[cb][j], acc[j]);
                if (ONESEG) acch = mfma3(wr[kb][0], wr[kb][1], bh[cb][2], bl[cb][2], acch);
            }
        }
        float umax = 0.f;
        {
            const float inv = exp2i(-(m_t + a.kr));
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                apply_mask(acc[j], mk[(32 * j + r) * 8 + 4 * h + w]);
#pragma unroll
                for (int i = 0; i < 16; ++i) {
                    acc[j][i] *= inv;
                    umax = fmaxf(umax, fabsf(acc[j][i]));
                }
            }
            if (ONESEG) {
                apply_mask(acch, mk[1024 + r * 8 + 4 * h + w]);   // lanes r >= 2: unused
#pragma unroll
                for (int i = 0; i < 16; ++i) {
                    acch[i] *= inv;
                    if (r < 2) umax = fmaxf(umax, fabsf(acch[i]));
                }
            }
            umax = wave_max(umax);
            if (lane == 0) RED[w] = umax;
        }
        lds_barrier();     // B3: every wave is done with the tot image
        float inv2;
        {
            const int m_u = scale_exp(fmaxf(fmaxf(RED[0], RED[1]), fmaxf(RED[2], RED[3])));
            const float su = exp2i(m_u);
            auto put = [&](const f32x16& v, int row) {
#pragma unroll
                for (int g = 0; g < 4; ++g) {
                    uint2 hi, lo;
                    split4(v[4 * g] * su, v[4 * g + 1] * su, v[4 * g + 2] * su, v[4 * g + 3] * su, hi, lo);
                    uint8_t* p = XS + row * RS + 2 * (chb + 8 * g);
                    *reinterpret_cast<uint2*>(p) = hi;
                    *reinterpret_cast<uint2*>(p + 256) = lo;
                }
            };
#pragma unroll
            for (int j = 0; j < 2; ++j) put(acc[j], Lc[j]);
            if (ONESEG && r < 2) put(acch, Lh);
            // ---- step 2 (below) works in units of 2^(m_u + k_d) ----
#pragma unroll
            for (int j = 0; j < 2; ++j)
#pragma unroll
                for (int i = 0; i < 16; ++i) acc[j][i] = 0.f;
            inv2 = exp2i(-(m_u + a.kd));
        }
        // this wave's D_l rows have landed (younger: the next tile's 9 row groups + 1 mask group)
        if (HAS_D) asm volatile("s_waitcnt vmcnt(10)" ::: "memory");
        lds_barrier();     // B4: g_u image complete (and every wave's D_l rows)
        STAMP(8)

        // ---- step 2: g_a = sum_k W_d[k] g_u(p - k + 1) ----
        {
            uint4 bh[2][2], bl[2][2];
            auto bload = [&](int st, uint4 (&xh)[2], uint4 (&xl)[2]) {
                const int tp = st >> 3, kb = st & 7;
#pragma unroll
                for (int j = 0; j < 2; ++j) {
                    const uint8_t* p = XS + (Lc[j] + 1 - tp) * RS + kb * 32 + h * 16;
                    xh[j] = lds16(p);
                    xl[j] = lds16(p + 256);
                }
            };
            bload(0, bh[0], bl[0]);
#pragma unroll
            for (int st = 0; st < 24; ++st) {
                const int tp = st >> 3, kb = st & 7, cb = st & 1;
                if (st + 1 < 24) bload(st + 1, bh[cb ^ 1], bl[cb ^ 1]);
#pragma unroll
                for (int j = 0; j < 2; ++j) {
                    uint4 xh = bh[cb][j], xl = bl[cb][j];
                    if (MASKED && ((tp == 0 && !ok2[j]) || (tp == 2 && !ok0[j]))) {
                        xh = make_uint4(0, 0, 0, 0);
                        xl = xh;
                    }
                    acc[j] = mfma3(wd[tp][kb][0], wd[tp][kb][1], xh, xl, acc[j]);
                }
            }
        }

        STAMP(9)
        // ---- epilogue: out = tot + [e_l > 0] g_a + D_l ----
        {
            float omax = 0.f;
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                const int c = 32 * j + r;
                apply_mask(acc[j], mk[512 + c * 8 + 4 * h + w]);
                const int t = ctime(cu, c, toff[j]);
                const uint8_t* tf = &XF[cur][0] + Lc[j] * RS + 4 * chb;
                const uint8_t* df = XD + c * RS + 4 * chb;
                float* dst = a.gout + ((size_t)cu.b * a.T + t) * C + chb;
#pragma unroll
                for (int g = 0; g < 4; ++g) {
                    const float4 tv = *reinterpret_cast<const float4*>(tf + 32 * g);
                    float4 o;
                    o.x = fmaf(acc[j][4 * g + 0], inv2, tv.x);
                    o.y = fmaf(acc[j][4 * g + 1], inv2, tv.y);
                    o.z = fmaf(acc[j][4 * g + 2], inv2, tv.z);
                    o.w = fmaf(acc[j][4 * g + 3], inv2, tv.w);
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
        STAMP(10)
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
