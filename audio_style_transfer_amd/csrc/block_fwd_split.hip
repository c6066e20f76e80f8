// Split-fp16 encoder block forward (precision 2): model.py:95-116 for one block,
//   u = dconv_d(relu(e_l)) + b_d        (masked.py:110-160, K = 3, SAME zero padding)
//   e_{l+1} = e_l + W_r^T relu(u) + b_r
// fp32 storage, v_mfma_f32_32x32x16_f16 on split fp16 operands, fp32 accumulation and fp32
// epilogues (splitwave.h).  The residual e_l is added in fp32 from the tile's fp32 rows.
//
// Per tile of 64 positions (one workgroup per CU, wave w owns output channels 32 w..32 w+31):
//   top     wait for this tile's fp32 rows (DMA'd during the previous tile), barrier B1;
//           store the previous tile's e_{l+1} > 0 words; DMA the next tile's rows
//   convert relu(e_l) 2^m_e -> split image (m_e from the clip's max |e_l|), barrier B2
//   GEMM 1  3 taps x 8 k-blocks x 2 column tiles x 3 products (A = W_d^T halves in AGPRs)
//   epi 1   u = acc 2^-(m_e+k_d) + b_d, u > 0 words, v = relu(u), wave max -> LDS, B3;
//           v 2^m_v -> split image (m_v from the tile's max v), u > 0 words -> HBM, B4
//   GEMM 2  8 k-blocks x 2 column tiles x 3 products (A = W_r^T halves in AGPRs)
//   epi 2   e_{l+1} = e_l + acc 2^-(m_v+k_r) + b_r -> HBM; e_{l+1} > 0 words (by the next
//           layer's positions) staged in LDS; max |e_{l+1}| -> the clip's atomic max
// Every wave issues the same vector-memory sequence after its DMA of the next tile (1 mask
// store, 8 row stores, 1 atomic), so the top-of-tile wait is vmcnt(10).
#include "splitwave.h"
#include <algorithm>

namespace ast {
namespace {
using namespace sw;

template <bool MASKED>
__global__ void __launch_bounds__(FT, 1) k_block_fwd_s(FwdArgsS a, Layout ly) {
    __shared__ __attribute__((aligned(16))) uint8_t XF[2][SLOT];   // fp32 e_l rows
    __shared__ __attribute__((aligned(16))) uint8_t XS[SLOT];      // split relu(e_l), then split v
    __shared__ __attribute__((aligned(16))) float BIAS[2 * C];     // b_d, b_r
    __shared__ __attribute__((aligned(16))) uint16_t MBU[TMS * 8]; // u > 0 words of the tile
    __shared__ __attribute__((aligned(16))) uint16_t MBE[TMS * 8]; // e_{l+1} > 0 words
    __shared__ int MBT[TMS];                                       // time of each tile column
    __shared__ float RED[4];

    const int tiles = a.T / TMS;
    const int ntiles = a.B * tiles;
    const int tid = threadIdx.x, lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int r = lane & 31, h = lane >> 5;

    auto tile_of = [&](int tl) { return tile_at<MASKED>(tl, tiles, a.n, a.d, ly); };
    RowDma<MASKED> dma;
    dma.init(w, lane, ly, a.d);
    auto issue_rows = [&](int tl, int slot) {
        dma.aim(a.ein, tile_of(tl), ly, a.T, a.n);
        const uint32_t lds0 = (uint32_t)(uintptr_t)&XF[slot][0] + (uint32_t)(w * 1024);
#pragma unroll
        for (int j = 0; j < DPW; ++j) dma.issue(j, a.ein, a.zero, lds0, a.T, a.n, a.d);
    };
    if (blockIdx.x < ntiles) issue_rows(blockIdx.x, 0);

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
    __syncthreads();

    // this lane's two tile columns (32 j + r), their image rows and time offsets
    int Lc[2], toff[2];
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        Lc[j] = frow(32 * j + r, ly);
        toff[j] = MASKED ? 0 : row_toff(Lc[j], ly, a.d);
    }
    const int chb = 32 * w + 4 * h;   // first channel of this lane's accumulator group g = 0
    auto ctime = [&](const Tile& t, int cc, int to) { return col_time<MASKED>(t, cc, to, a.n, a.d); };

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

    int it = 0, prevb = 0;
    STAMP_DECL
    for (int tile = blockIdx.x; tile < ntiles; tile += gridDim.x, ++it) {
        const int cur = it & 1;
        const Tile cu = tile_of(tile);
        // this wave's part of the tile's rows has landed (vmcnt retires in issue order; 10
        // memory ops of the previous tile follow its DMA), the barrier publishes all parts
        if (it) asm volatile("s_waitcnt vmcnt(10)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        if (it) store_me(prevb);
        issue_rows(tile + (int)gridDim.x < ntiles ? tile + (int)gridDim.x : ntiles - 1, cur ^ 1);

        STAMP(0)
        const int m_e = scale_exp(sload(a.gmax_in + cu.b));
        convert_rows<true>(&XF[cur][0], XS, ly.nrows, exp2i(m_e), w, lane);
        lds_barrier();     // B2: split image complete
        STAMP(1)

        bool ok0[2] = {true, true}, ok2[2] = {true, true};
        if (MASKED) {
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                const int m = (cu.p0 + 32 * j + r) % a.n;
                ok0[j] = m > 0;
                ok2[j] = m < a.n - 1;
            }
        }

        // ---- GEMM 1: u = sum_tap W_d[tap]^T relu(e_l)(p + tap - 1) ----
        f32x16 acc[2];
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
                    const uint8_t* p = XS + (Lc[j] + tp - 1) * RS + kb * 32 + h * 16;
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
                    if (MASKED && ((tp == 0 && !ok0[j]) || (tp == 2 && !ok2[j]))) {
                        xh = make_uint4(0, 0, 0, 0);
                        xl = xh;
                    }
                    acc[j] = mfma3(wd[tp][kb][0], wd[tp][kb][1], xh, xl, acc[j]);
                }
            }
        }

        STAMP(2)
        // ---- epilogue 1: u, u > 0 words, v = relu(u) ----
        {
            const float inv1 = exp2i(-(m_e + a.kd));
            float vmax = 0.f;
#pragma unroll
            for (int j = 0; j < 2; ++j) {
#pragma unroll
                for (int g = 0; g < 4; ++g) {
                    const float4 b4 = *reinterpret_cast<const float4*>(&BIAS[chb + 8 * g]);
                    acc[j][4 * g + 0] = fmaf(acc[j][4 * g + 0], inv1, b4.x);
                    acc[j][4 * g + 1] = fmaf(acc[j][4 * g + 1], inv1, b4.y);
                    acc[j][4 * g + 2] = fmaf(acc[j][4 * g + 2], inv1, b4.z);
                    acc[j][4 * g + 3] = fmaf(acc[j][4 * g + 3], inv1, b4.w);
                }
                MBU[(32 * j + r) * 8 + 4 * h + w] = (uint16_t)mask_bits(acc[j]);
#pragma unroll
                for (int i = 0; i < 16; ++i) {
                    acc[j][i] = fmaxf(acc[j][i], 0.f);
                    vmax = fmaxf(vmax, acc[j][i]);
                }
            }
            vmax = wave_max(vmax);
            if (lane == 0) RED[w] = vmax;
        }
        lds_barrier();     // B3: every wave is done with the relu(e_l) image
        const int m_v = scale_exp(fmaxf(fmaxf(RED[0], RED[1]), fmaxf(RED[2], RED[3])));
        {
            const float sv = exp2i(m_v);
#pragma unroll
            for (int j = 0; j < 2; ++j)
#pragma unroll
                for (int g = 0; g < 4; ++g) {
                    uint2 hi, lo;
                    split4(acc[j][4 * g] * sv, acc[j][4 * g + 1] * sv, acc[j][4 * g + 2] * sv,
                           acc[j][4 * g + 3] * sv, hi, lo);
                    uint8_t* p = XS + (32 * j + r) * RS + 2 * (chb + 8 * g);
                    *reinterpret_cast<uint2*>(p) = hi;
                    *reinterpret_cast<uint2*>(p + 256) = lo;
                }
        }
        // u > 0 words of the tile (this layer's positions): wave w stores columns 16 w .. +15
        if (lane < 16)
            *reinterpret_cast<uint4*>(a.mu + ((size_t)cu.b * a.T + cu.p0 + 16 * w + lane) * 8) =
                *reinterpret_cast<const uint4*>(&MBU[(16 * w + lane) * 8]);
        lds_barrier();     // B4: v image complete
        STAMP(3)

        // ---- GEMM 2: y = W_r^T v ----
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int i = 0; i < 16; ++i) acc[j][i] = 0.f;
        {
            uint4 bh[2][2], bl[2][2];
            auto bload = [&](int kb, uint4 (&xh)[2], uint4 (&xl)[2]) {
#pragma unroll
                for (int j = 0; j < 2; ++j) {
                    const uint8_t* p = XS + (32 * j + r) * RS + kb * 32 + h * 16;
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
            }
        }

        STAMP(4)
        // ---- epilogue 2: e_{l+1} = e_l + y + b_r ----
        {
            const float inv2 = exp2i(-(m_v + a.kr));
            float emax = 0.f;
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                const int c = 32 * j + r;
                const int t = ctime(cu, c, toff[j]);
                const uint8_t* ef = &XF[cur][0] + Lc[j] * RS + 4 * chb;
                float* dst = a.eout + ((size_t)cu.b * a.T + t) * C + chb;
#pragma unroll
                for (int g = 0; g < 4; ++g) {
                    const float4 e = *reinterpret_cast<const float4*>(ef + 32 * g);
                    const float4 b4 = *reinterpret_cast<const float4*>(&BIAS[C + chb + 8 * g]);
                    float4 o;
                    o.x = e.x + fmaf(acc[j][4 * g + 0], inv2, b4.x);
                    o.y = e.y + fmaf(acc[j][4 * g + 1], inv2, b4.y);
                    o.z = e.z + fmaf(acc[j][4 * g + 2], inv2, b4.z);
                    o.w = e.w + fmaf(acc[j][4 * g + 3], inv2, b4.w);
                    *reinterpret_cast<float4*>(dst + 8 * g) = o;
                    acc[j][4 * g + 0] = o.x; acc[j][4 * g + 1] = o.y;
                    acc[j][4 * g + 2] = o.z; acc[j][4 * g + 3] = o.w;
                    emax = fmaxf(emax, fmaxf(fmaxf(fabsf(o.x), fabsf(o.y)), fmaxf(fabsf(o.z), fabsf(o.w))));
                }
                MBE[c * 8 + 4 * h + w] = (uint16_t)mask_bits(acc[j]);
                if (w == 0 && h == 0) MBT[c] = t;
            }
            emax = wave_max(emax);
            if (lane == 0) atomicMax(a.gmax_out + cu.b, __float_as_uint(emax));
        }
        prevb = cu.b;
        STAMP(5)
    }
    STAMP_FLUSH(a.stamps)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (it) store_me(prevb);
}

}  // namespace

void launch_block_fwd_s(const FwdArgsS& a, hipStream_t s) {
    const int nt = a.B * (a.T / TMS);
    const dim3 grid(std::min(nt, sw::num_cus()));
    Layout ly;
    if (pick_layout(a.n, ly)) hipLaunchKernelGGL(k_block_fwd_s<true>, grid, dim3(FT), 0, s, a, ly);
    else hipLaunchKernelGGL(k_block_fwd_s<false>, grid, dim3(FT), 0, s, a, ly);
}

int sw::num_cus() {
    static int cus = 0;
    if (!cus) {
        int dev = 0;
        (void)hipGetDevice(&dev);
        (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
        if (cus <= 0) cus = 256;
    }
    return cus;
}

}  // namespace ast
