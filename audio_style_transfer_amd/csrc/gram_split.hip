// Channel-wise ("ours") Gram forward/backward, methods.py:62-76: on bf16 MFMA over fp32
// activations (precision 2, *_s kernels) and on fp32 MFMA (precision 0, *_f kernels, the same
// staging).  The activations stay fp32 in HBM.  Each Gram operand is carried as two
// bf16 terms, x ~ xh + xl (xh = bf16(x), xl = bf16(x - xh)), and every product as
// xh yh + xh yl + xl yh on v_mfma_*_bf16 with fp32 accumulation: the Gram is HBM-bound (10
// flop/B), so the three products cost no time, and they keep the gradient at fp32-class error
// where one bf16 product does not (an L = 2 style Gram: 1.8e-3 rel-L2 from the bf16 backward
// alone, tools/precision_emulate.py).  D leaves in fp32.
//
// Per (clip, time chunk, 32-channel group) workgroup, 8 waves x 4 channels, stages of 16 time
// rows; the next two stages' global loads (128 KiB per workgroup) are in flight while a stage
// computes:
//   fwd  G_c = E_c E_c^T      v_mfma_f32_32x32x16_bf16, A = B fragments (lane (u, h):
//                             E_u[t0 + 8 h .. + 8][c]) from an LDS image [c][u][hi t | lo t]
//   bwd  D_c = S~_c E_c       v_mfma_f32_16x16x32_bf16 (A = S~_c halves in registers, B: lane
//                             (t, kq): E_{8 kq .. + 8}[t][c]) from LDS images [c][t][u] (hi, lo);
//                             D goes back through an fp32 image [u][t][c] in two halves of 16
//                             tensors and leaves as whole 128-B lines (+ the content grad: a
//                             cg buffer, or the fused content tap computed here)
// Loads and stores move whole 128-B lines (8 lanes x 16 B per row).
#include "common.h"
#include <cstdlib>
#include <cstdio>

namespace ast {
namespace {

constexpr int GCS = 32;       // channels per workgroup
constexpr int GSS = 16;       // time rows per stage
constexpr int GWT = 512;      // threads per workgroup (8 waves x 4 channels)
constexpr int FRS = 40;       // fwd image [c][u][hi 16 | lo 16 | pad 8] row stride (bf16): 80 B
constexpr int BRS = 40;       // bwd images [c][t][u] row stride (bf16): 80 B
constexpr int ORS = 36;       // bwd output image [u][t][c] row stride (floats): 144 B

typedef float f32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
    const int xcd = bid % 8, q = nwg / 8, rr = nwg % 8;
    return (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + bid / 8;
}

__device__ __forceinline__ void decode(const GramArgs& a, int& b, int& ch, int& c0) {
    constexpr int ncg = C / GCS;
    const int nwg = a.B * a.nchunk * ncg;
    int work = xcd_remap(blockIdx.x, nwg);   // the 4 channel groups of a chunk share one XCD
    const int cgi = work % ncg; work /= ncg;
    ch = work % a.nchunk;
    b = work / a.nchunk;
    c0 = cgi * GCS;
}

// bf16 pair (x0, x1) and the pair of their remainders
__device__ __forceinline__ void split2(float x0, float x1, uint32_t& hi, uint32_t& lo) {
    hi = pack2(x0, x1);
    lo = pack2(x0 - bflo(hi), x1 - bfhi(hi));
}
// 8 values (one channel of 8 loaded float4) -> hi / lo 16-B fragment runs
template <int J>
__device__ __forceinline__ void split8(const float4 (&v)[8], uint4& hi, uint4& lo) {
    auto e = [&](int k) { return J == 0 ? v[k].x : J == 1 ? v[k].y : J == 2 ? v[k].z : v[k].w; };
    uint32_t h[4], l[4];
#pragma unroll
    for (int p = 0; p < 4; ++p) split2(e(2 * p), e(2 * p + 1), h[p], l[p]);
    hi = make_uint4(h[0], h[1], h[2], h[3]);
    lo = make_uint4(l[0], l[1], l[2], l[3]);
}

// forward.  Staging: thread (w, l) loads tensor u = 8 (w & 3) + (l & 7), channel quad l >> 3,
// rows t0 + 8 (w >> 2) + k (k = 0..7): one load instruction covers 8 whole lines.
// NST stages of loads in flight (2: 128 KiB per workgroup; 3: 192 KiB, the registers of a
// third stage fit beside the accumulators at the same two waves per SIMD)
template <int NST>
__global__ void __launch_bounds__(GWT) k_gram_fwd_s(GramArgs a) {
    __shared__ __attribute__((aligned(16))) u16 I[GCS * 32 * FRS];   // [c][u][hi t | lo t]
    int b, ch, c0;
    decode(a, b, ch, c0);
    const int tlen = a.T / a.nchunk, tbeg = ch * tlen;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int r = lane & 31, h = lane >> 5;
    const int su = 8 * (w & 3) + (lane & 7), sq = lane >> 3, tb = w >> 2;
    const bool real = su < a.nu;
    const float* src = real ? (const float*)a.act + (size_t)a.uid[su] * a.tstride +
                              (size_t)b * a.T * C + c0 + 4 * sq + (size_t)8 * tb * C
                            : (const float*)a.zero16;
    const size_t rs = real ? C : 0;
    f32x16 acc[4];
#pragma unroll
    for (int cc = 0; cc < 4; ++cc)
#pragma unroll
        for (int i = 0; i < 16; ++i) acc[cc][i] = 0.f;
    // NST stages of loads in flight (a ring of NST register sets; tlen is a multiple of 2 GSS).
    // Every load is unconditional (past the chunk a stage re-reads the chunk's last rows, an L2
    // hit) and the loop runs whole rings, the remainder after it: a conditional load made the
    // compiler copy the ring registers (v_mov) behind vmcnt(0) waits, so no stage stayed in
    // flight across a stage
    float4 v[NST][8];
    const int tend = tbeg + tlen;
    auto load = [&](float4 (&v)[8], int t0) {
        const int tr = min(t0, tend - GSS);
#pragma unroll
        for (int k = 0; k < 8; ++k) v[k] = *reinterpret_cast<const float4*>(src + (size_t)(tr + k) * rs);
    };
    auto stage = [&](float4 (&v)[8], int t0) {
        uint4 fh[4], fl[4];          // channel 4 sq + j: 8 consecutive rows, hi / lo
        split8<0>(v, fh[0], fl[0]);
        split8<1>(v, fh[1], fl[1]);
        split8<2>(v, fh[2], fl[2]);
        split8<3>(v, fh[3], fl[3]);
        load(v, t0 + NST * GSS);
        __syncthreads();
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            u16* row = &I[((4 * sq + j) * 32 + su) * FRS + 8 * tb];
            *reinterpret_cast<uint4*>(row) = fh[j];
            *reinterpret_cast<uint4*>(row + 16) = fl[j];
        }
        __syncthreads();
#pragma unroll
        for (int cc = 0; cc < 4; ++cc) {
            const u16* row = &I[((4 * w + cc) * 32 + r) * FRS + 8 * h];
            const uint4 xh = *reinterpret_cast<const uint4*>(row);
            const uint4 xl = *reinterpret_cast<const uint4*>(row + 16);
            acc[cc] = mfma_bf16(xh, xh, acc[cc]);
            acc[cc] = mfma_bf16(xh, xl, acc[cc]);
            acc[cc] = mfma_bf16(xl, xh, acc[cc]);
        }
    };
#pragma unroll
    for (int q = 0; q < NST; ++q) load(v[q], tbeg + q * GSS);
    const int nst = tlen / GSS, nring = nst / NST;
    int t0 = tbeg;
    for (int i = 0; i < nring; ++i, t0 += NST * GSS) {
#pragma unroll
        for (int q = 0; q < NST; ++q) stage(v[q], t0 + q * GSS);
    }
#pragma unroll
    for (int q = 0; q < NST - 1; ++q)
        if (q < nst - nring * NST) stage(v[q], t0 + q * GSS);
#pragma unroll
    for (int cc = 0; cc < 4; ++cc) {
        float* dst = a.gpart + (((size_t)b * a.nchunk + ch) * C + c0 + 4 * w + cc) * 1024;
#pragma unroll
        for (int i = 0; i < 16; ++i) dst[((i & 3) + 8 * (i >> 2) + 4 * h) * 32 + r] = acc[cc][i];
    }
}

// forward for few clips (k_gram_fwd_n): 8 channels per workgroup instead of 32, so a clip's
// chunk spreads over 16 workgroups instead of 4 (one clip: 64 instead of 16).  Wave w owns
// channel c0 + w and runs, stage by stage (16 rows), the same three MFMAs on the same
// fragments as k_gram_fwd_s's wave for that channel: the partials are bit-identical, so a
// clip's result does not depend on which kernel the batch size selects.  Staging: a fill is 4
// stages (64 rows); thread (w, l) loads tensor 8 (w & 3) + (l & 7), channel quad (l >> 3) & 1,
// rows 8 g .. + 8 of the fill, g = (l >> 4) + 4 (w >> 2); two fills of loads in flight.
constexpr int GCN = 8;        // channels per narrow forward workgroup
constexpr int GFN = 64;       // rows per narrow fill (4 stages)
// NFL fills of loads in flight in a ring (round 6; 2 before, with a conditional load that, as in
// the round-5 wide kernels, made the compiler drain the ring at every fill).  Loads are
// unconditional: past the chunk a fill re-reads the chunk's last fill (an L2 hit); the loop runs
// whole rings, the remainder after it.  The MFMA sequence per channel is unchanged (same bits).
// NC channels per workgroup, one wave each (8; 4 for a single clip: twice the workgroups, 16-B row
// pieces).  Staging, NC = 8: thread (w, l) loads tensor 8 (w & 3) + (l & 7), channel quad
// (l >> 3) & 1, rows 8 g .. + 8 of the fill, g = (l >> 4) + 4 (w >> 2); NC = 4: tensor 8 w + (l & 7),
// channel quad 0, g = l >> 3
template <int NFL, int NC>
__global__ void __launch_bounds__(64 * NC) k_gram_fwd_n(GramArgs a) {
    __shared__ __attribute__((aligned(16))) u16 I[(GFN / GSS) * NC * 32 * FRS];   // [stage][c][u][hi | lo]
    constexpr int ncg = C / NC;
    const int nwg = a.B * a.nchunk * ncg;
    int work = xcd_remap(blockIdx.x, nwg);
    const int cgi = work % ncg; work /= ncg;
    const int ch = work % a.nchunk, b = work / a.nchunk, c0 = cgi * NC;
    const int tlen = a.T / a.nchunk, tbeg = ch * tlen, tend = tbeg + tlen;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int r = lane & 31, h = lane >> 5;
    const int su = NC == 8 ? 8 * (w & 3) + (lane & 7) : 8 * w + (lane & 7);
    const int sq = NC == 8 ? (lane >> 3) & 1 : 0;
    const int g = NC == 8 ? (lane >> 4) + 4 * (w >> 2) : lane >> 3;
    const bool real = su < a.nu;
    const float* src = real ? (const float*)a.act + (size_t)a.uid[su] * a.tstride +
                              (size_t)b * a.T * C + c0 + 4 * sq + (size_t)8 * g * C
                            : (const float*)a.zero16;
    const size_t rs = real ? C : 0;
    f32x16 acc;
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[i] = 0.f;
    float4 v[NFL][8];
    auto load = [&](float4 (&vv)[8], int t0) {
        const int tr = min(t0, tend - GFN);
#pragma unroll
        for (int k = 0; k < 8; ++k) vv[k] = *reinterpret_cast<const float4*>(src + (size_t)(tr + k) * rs);
    };
    auto fill = [&](float4 (&vv)[8], int t0) {
        uint4 fh[4], fl[4];
        split8<0>(vv, fh[0], fl[0]);
        split8<1>(vv, fh[1], fl[1]);
        split8<2>(vv, fh[2], fl[2]);
        split8<3>(vv, fh[3], fl[3]);
        load(vv, t0 + NFL * GFN);
        __syncthreads();   // the previous fill's MFMA reads are done
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            // stage g >> 1, channel 4 sq + j, tensor su; rows 8 (g & 1) .. of the stage
            u16* row = &I[(((g >> 1) * NC + 4 * sq + j) * 32 + su) * FRS + 8 * (g & 1)];
            *reinterpret_cast<uint4*>(row) = fh[j];
            *reinterpret_cast<uint4*>(row + 16) = fl[j];
        }
        __syncthreads();
#pragma unroll
        for (int st = 0; st < GFN / GSS; ++st) {
            const u16* row = &I[((st * NC + w) * 32 + r) * FRS + 8 * h];
            const uint4 xh = *reinterpret_cast<const uint4*>(row);
            const uint4 xl = *reinterpret_cast<const uint4*>(row + 16);
            acc = mfma_bf16(xh, xh, acc);
            acc = mfma_bf16(xh, xl, acc);
            acc = mfma_bf16(xl, xh, acc);
        }
    };
#pragma unroll
    for (int q = 0; q < NFL; ++q) load(v[q], tbeg + q * GFN);
    const int nf = tlen / GFN, nring = nf / NFL;
    int t0 = tbeg;
    for (int i = 0; i < nring; ++i, t0 += NFL * GFN) {
#pragma unroll
        for (int q = 0; q < NFL; ++q) fill(v[q], t0 + q * GFN);
    }
#pragma unroll
    for (int q = 0; q < NFL - 1; ++q)
        if (q < nf - nring * NFL) fill(v[q], t0 + q * GFN);
    float* dst = a.gpart + (((size_t)b * a.nchunk + ch) * C + c0 + w) * 1024;
#pragma unroll
    for (int i = 0; i < 16; ++i) dst[((i & 3) + 8 * (i >> 2) + 4 * h) * 32 + r] = acc[i];
}

// backward.  Staging: thread (w, l) loads tensors 8 (w & 3) + k (k = 0..7), channel quad
// l >> 3, row t0 + 8 (w >> 2) + (l & 7).  Output: 16 tensors at a time through O; padding
// tensors (u >= nu) are neither read nor written.
// CONT: the fused content tap (a.cont_u >= 0); false: the round-2 kernel.  NST stages of loads
// in flight: 2 (the split of a stage into registers before the barrier) or 3 (each channel split
// straight into the image after the barrier: 24 fewer live registers pay for the third stage)
// HCG: some tensor has a content-gradient buffer to add (not the fused configs): without it
// the store loop has no branch around a load (a load there made the compiler drain every stage
// load in flight with vmcnt(0))
template <bool CONT, int NST, bool HCG>
__global__ void __launch_bounds__(GWT) k_gram_bwd_s(GramArgs a) {
    __shared__ __attribute__((aligned(16))) u16 IH[GCS * GSS * BRS];       // [c][t][u] hi
    __shared__ __attribute__((aligned(16))) u16 IL[GCS * GSS * BRS];       // [c][t][u] lo
    __shared__ __attribute__((aligned(16))) float O[16 * GSS * ORS];       // [u][t][c]
    int b, ch, c0;
    decode(a, b, ch, c0);
    const int tlen = a.T / a.nchunk, tbeg = ch * tlen, tend = tbeg + tlen;
    const int tid = threadIdx.x, lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    float omax = 0.f;   // max |D| of tensor top_u (the backward chain's first input: no k_absmax pass)
    float csd = 0.f;    // squared content error of tensor cont_u (this GRAM_CSLOT-row slot)
    __shared__ float cws[GWT / 64];
    const int i16 = lane & 15, kq = lane >> 4;
    // A fragments (16x16x32): S~_c[u = 16 m + i16][u' = 8 kq .. + 8] as bf16 hi / lo; wave w
    // owns channels 4 w .. 4 w + 3
    uint4 sa[4][2][2];
#pragma unroll
    for (int cc = 0; cc < 4; ++cc)
#pragma unroll
        for (int m = 0; m < 2; ++m) {
            const float* sm = a.smat + ((size_t)b * C + c0 + 4 * w + cc) * 1024 + (16 * m + i16) * 32 + 8 * kq;
            const float4 p = *reinterpret_cast<const float4*>(sm);
            const float4 q = *reinterpret_cast<const float4*>(sm + 4);
            uint32_t h[4], l[4];
            split2(p.x, p.y, h[0], l[0]);
            split2(p.z, p.w, h[1], l[1]);
            split2(q.x, q.y, h[2], l[2]);
            split2(q.z, q.w, h[3], l[3]);
            sa[cc][m][0] = make_uint4(h[0], h[1], h[2], h[3]);
            sa[cc][m][1] = make_uint4(l[0], l[1], l[2], l[3]);
        }
    // staging loads: tensors 8 uo + k, quad sq, row st of the stage
    const int uo = w & 3, sq = lane >> 3, st = 8 * (w >> 2) + (lane & 7);
    // per tensor a wave-uniform base (the clip's first row; scalar registers) and one 32-bit lane
    // offset for all eight (the tensors of a wave are uniform: uo = w & 3)
    const float* ld[8];
    uint32_t lrs[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        const int u = 8 * uo + k;
        ld[k] = u < a.nu ? (const float*)a.act + (size_t)a.uid[u] * a.tstride + (size_t)b * a.T * C : (const float*)a.zero16;
        lrs[k] = u < a.nu ? C : 0;
    }
    const uint32_t lofs = (uint32_t)(c0 + 4 * sq);
    // fused content tap: the 128 threads whose output pieces are tensor cont_u's (iteration
    // it = (cont_u % 16) / 4 of half cont_u / 16) load its E and phi rows at the start of each
    // stage and add coef (E - phi) to those pieces (one copy of the code, not one per piece)
    const int cit = ((a.cont_u & 15) * 128) >> 9;   // (wave-uniform test below)
    const bool cthr = CONT && cit * GWT + tid >= (a.cont_u & 15) * 128 && cit * GWT + tid < (a.cont_u & 15) * 128 + 128;
    const int cp_ = cit * GWT + tid, ctt = (cp_ >> 3) & 15, cq = cp_ & 7;
    const float* ce_src = CONT ? (const float*)a.act + (size_t)a.uid[a.cont_u & 31] * a.tstride + (size_t)b * a.T * C + c0 + 4 * cq : nullptr;
    const float* cp_src = CONT ? a.cont_phi + (size_t)b * a.cont_phi_bstride + a.cont_off + c0 + 4 * cq : nullptr;
    // NST stages of loads in flight (a ring of register sets; tlen is a multiple of 2 GSS)
    float4 vr[NST][8];
    // unconditional loads (past the chunk a stage re-reads the chunk's last stage, an L2 hit):
    // a conditional load made the compiler copy the ring registers behind vmcnt(0) waits
    auto load = [&](float4 (&v)[8], int t0) {
        const int tr = min(t0, tend - GSS);
#pragma unroll
        for (int k = 0; k < 8; ++k) v[k] = *reinterpret_cast<const float4*>(ld[k] + (lrs[k] ? lofs + (uint32_t)(tr + st) * C : 0u));
    };
    auto stage = [&](float4 (&v)[8], int t0) {
        float4 ce, cph = make_float4(0.f, 0.f, 0.f, 0.f);
        if (CONT && cthr) {
            ce = *reinterpret_cast<const float4*>(ce_src + (size_t)(t0 + ctt) * C);
            // phi rows hold only the tap's cont_ncol (a multiple of 4) channels: quads past them
            // load nothing (the row's last quad can end the caller's buffer)
            if (c0 + 4 * cq < a.cont_ncol)
                cph = *reinterpret_cast<const float4*>(cp_src + (size_t)(t0 + ctt) * a.cont_ncc);
        }
        if (NST == 2) {
            uint4 fh[4], fl[4];   // channel 4 sq + j: tensors 8 uo .. + 8 at row st, hi / lo
            split8<0>(v, fh[0], fl[0]);
            split8<1>(v, fh[1], fl[1]);
            split8<2>(v, fh[2], fl[2]);
            split8<3>(v, fh[3], fl[3]);
            load(v, t0 + NST * GSS);
            __syncthreads();   // the previous stage's image and O reads are done
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int o = ((4 * sq + j) * GSS + st) * BRS + 8 * uo;
                *reinterpret_cast<uint4*>(&IH[o]) = fh[j];
                *reinterpret_cast<uint4*>(&IL[o]) = fl[j];
            }
        } else {
            __syncthreads();   // the previous stage's image and O reads are done
            uint4 fh, fl;
#define SPLIT_ONE(J) { split8<J>(v, fh, fl); const int o = ((4 * sq + J) * GSS + st) * BRS + 8 * uo; \
                       *reinterpret_cast<uint4*>(&IH[o]) = fh; *reinterpret_cast<uint4*>(&IL[o]) = fl; }
            SPLIT_ONE(0) SPLIT_ONE(1) SPLIT_ONE(2) SPLIT_ONE(3)
#undef SPLIT_ONE
            load(v, t0 + NST * GSS);
        }
        __syncthreads();
        // D_c = S~_c E_c of column half m for the wave's 4 channels (the B fragments re-read per
        // half: only one half's accumulators are live)
        auto dhalf = [&](int m, int cc) {
            const int o = ((4 * w + cc) * GSS + i16) * BRS + 8 * kq;
            const uint4 bh = *reinterpret_cast<const uint4*>(&IH[o]);
            const uint4 bl = *reinterpret_cast<const uint4*>(&IL[o]);
            f32x4 c = {0.f, 0.f, 0.f, 0.f};
            c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, sa[cc][m][0]),
                                                       __builtin_bit_cast(bf16x8, bh), c, 0, 0, 0);
            c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, sa[cc][m][1]),
                                                       __builtin_bit_cast(bf16x8, bh), c, 0, 0, 0);
            return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, sa[cc][m][0]),
                                                          __builtin_bit_cast(bf16x8, bl), c, 0, 0, 0);
        };
        float4 cadd = make_float4(0.f, 0.f, 0.f, 0.f);
        if (CONT && cthr) {
            const int cc = c0 + 4 * cq;
            const float ev[4] = {ce.x, ce.y, ce.z, ce.w}, pv[4] = {cph.x, cph.y, cph.z, cph.w};
            float d[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                d[i] = cc + i < a.cont_ncol ? ev[i] - pv[i] : 0.f;
                csd = fmaf(d[i], d[i], csd);
            }
            cadd = make_float4(a.cont_coef * d[0], a.cont_coef * d[1], a.cont_coef * d[2], a.cont_coef * d[3]);
        }
        // lane holds D_c[u = 16 m + 4 kq + i][t = i16] for the wave's 4 channels
#pragma unroll
        for (int m = 0; m < 2; ++m) {
            f32x4 acc[4];
#pragma unroll
            for (int cc = 0; cc < 4; ++cc) acc[cc] = dhalf(m, cc);
            if (m) __syncthreads();   // the first half's O reads are done
#pragma unroll
            for (int cc = 0; cc < 4; ++cc)
#pragma unroll
                for (int i = 0; i < 4; ++i)
                    O[((4 * kq + i) * GSS + i16) * ORS + 4 * w + cc] = acc[cc][i];
            __syncthreads();
            // 16 tensors x 16 rows x 8 quads = 2048 pieces, 4 per thread: u = 16 m + (p >> 7),
            // p = it GWT + tid.  The tensor is wave-uniform (waves 2 k, 2 k + 1 take tensor 4 it + k)
            // and formed from the readfirstlane'd wave index, so a.uid[u] / a.cg[u] are scalar
            // kernel-argument loads: a per-lane index made them vector loads whose vmcnt wait
            // drained the stage loads in flight at every piece
#pragma unroll
            for (int it = 0; it < 4; ++it) {
                const int ul = 4 * it + (w >> 1), tt = (tid >> 3) & 15, q = tid & 7;
                const int u = 16 * m + ul;
                if (u < a.nu) {
                    float4 o = *reinterpret_cast<const float4*>(&O[(ul * GSS + tt) * ORS + 4 * q]);
                    const size_t off = (size_t)a.uid[u] * a.tstride + ((size_t)b * a.T + t0 + tt) * C + c0 + 4 * q;
                    const float* cg = HCG ? (const float*)a.cg[u] : nullptr;
                    if (HCG && cg) {
                        const float4 g = *reinterpret_cast<const float4*>(cg + ((size_t)b * a.T + t0 + tt) * C + c0 + 4 * q);
                        o.x += g.x; o.y += g.y; o.z += g.z; o.w += g.w;
                    }
                    if (CONT && u == a.cont_u) { o.x += cadd.x; o.y += cadd.y; o.z += cadd.z; o.w += cadd.w; }
                    *reinterpret_cast<float4*>((float*)a.actw + off) = o;
                    if (u == a.top_u)
                        omax = fmaxf(omax, fmaxf(fmaxf(fabsf(o.x), fabsf(o.y)), fmaxf(fabsf(o.z), fabsf(o.w))));
                }
            }
        }
    };
#pragma unroll
    for (int q = 0; q < NST; ++q)
        if (tbeg + q * GSS < tend) load(vr[q], tbeg + q * GSS);
    // the content errors of every GRAM_CSLOT rows -> their own slot (fixed order: wave butterfly,
    // then waves 0..7), so the loss does not depend on how time is cut into workgroups
    auto flush_c = [&](int slot) {
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) csd += __shfl_xor(csd, off);
        if (lane == 0) cws[w] = csd;
        __syncthreads();
        if (tid == 0) {
            float v = 0.f;
#pragma unroll
            for (int k = 0; k < GWT / 64; ++k) v += cws[k];
            a.cont_part[(size_t)b * a.cont_pstride + slot * (C / GCS) + c0 / GCS] = v;
        }
        csd = 0.f;
    };
    const int nring = (tlen / GSS) / NST;
    int t0 = tbeg;
    for (int i = 0; i < nring; ++i, t0 += NST * GSS) {
#pragma unroll
        for (int q = 0; q < NST; ++q) {
            stage(vr[q], t0 + q * GSS);
            if (CONT && (t0 + (q + 1) * GSS) % GRAM_CSLOT == 0) flush_c((t0 + q * GSS) / GRAM_CSLOT);
        }
    }
#pragma unroll
    for (int q = 0; q < NST - 1; ++q)
        if (t0 + q * GSS < tend) {
            stage(vr[q], t0 + q * GSS);
            if (CONT && (t0 + (q + 1) * GSS) % GRAM_CSLOT == 0) flush_c((t0 + q * GSS) / GRAM_CSLOT);
        }
    if (a.top_u >= 0) {   // one atomic per workgroup
        __shared__ float wm[GWT / 64];
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) omax = fmaxf(omax, __shfl_xor(omax, off));
        if (lane == 0) wm[w] = omax;
        __syncthreads();
        if (tid == 0) {
            float m = wm[0];
#pragma unroll
            for (int k = 1; k < GWT / 64; ++k) m = fmaxf(m, wm[k]);
            atomicMax(gslot(a.gmax_top, b, blockIdx.x), __float_as_uint(m));
        }
    }
}

// ---- backward over half rows (round 5): 64 channels per workgroup ----
// The bare data movement of this backward runs ~5.6 % faster when a workgroup's row pieces are
// 256 B (64 channels) instead of 128 B (tools/diag/gram_pattern.hip).  The S~
// fragments of 64 channels double the registers of k_gram_bwd_s's waves, so the stages are 8
// rows (half the staging registers; the 16x16x32 MFMA's columns 8..15 repeat rows 0..7 and are
// dropped -- the Gram is HBM-bound) and the split goes straight into the image after the barrier.
// 8 waves x 8 channels.  D is bit-identical to k_gram_bwd_s's (the same MFMAs per element, the
// same K order); the fused content tap's squared errors go to 128-row slots, T / 128 x 2 =
// ncpart partials per clip, each summed in a fixed order (thread over the slot's stages, wave
// butterfly, waves 0..7), whatever the chunking.  Wave pair g = w >> 1 stages and stores the
// tensors u = 8 g + k (k < 8): one set of 8 wave-uniform resources serves both.
constexpr int HCH = 64;       // channels per workgroup
constexpr int HSS = 8;        // rows per stage
constexpr int HWT = 512;      // threads
constexpr int HOR = 68;       // O row stride (floats; 16-B aligned)
constexpr int HSLOT = 128;    // rows per content-error slot

__device__ __forceinline__ void decode_h(const GramArgs& a, int& b, int& ch, int& c0) {
    const int nwg = a.B * a.nchunk * 2;
    int work = xcd_remap(blockIdx.x, nwg);   // the two channel halves of a chunk share one XCD
    const int cgi = work & 1;
    work >>= 1;
    ch = work % a.nchunk;
    b = work / a.nchunk;
    c0 = cgi * HCH;
}
// raw buffer access: a tensor's clip base in a resource (scalar registers) + one 32-bit lane
// offset shared by the 8 tensors of a thread (64-bit per-tensor lane addresses spilled); a
// resource of 0 records (a padding tensor) reads zeros and drops its stores
typedef unsigned int hu32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ __amdgpu_buffer_rsrc_t h_rsrc(const void* p, bool real) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, real ? 0x7fffffff : 0, 0x00020000);
}
// image [c][t][u] (bf16): the 16-B block of K positions 8 g .. 8 g + 7 at block g ^ hswz(c, t),
// so the staging writes (rows t & 3 x channel quads c >> 2 over 16 lanes) and the fragment
// reads (rows 0..7 of one channel) are conflict-free
__device__ __forceinline__ int hswz(int c, int t) { return ((c >> 2) ^ (t >> 2)) & 3; }

// DOOP: D goes to a buffer of its own (actw != act, ASTYLE_DOOP=1): stores through resources of
// their own (A/B only)
template <bool CONT, bool DOOP>
__global__ void __launch_bounds__(HWT) k_gram_bwd_h(GramArgs a) {
    __shared__ __attribute__((aligned(16))) u16 IH[HCH * HSS * 32];      // [c][t][u] hi
    __shared__ __attribute__((aligned(16))) u16 IL[HCH * HSS * 32];      // [c][t][u] lo
    __shared__ __attribute__((aligned(16))) float O[32 * HSS * HOR];     // [u][t][c]
    __shared__ float cws[HWT / 64];
    int b, ch, c0;
    decode_h(a, b, ch, c0);
    const int tlen = a.T / a.nchunk, tbeg = ch * tlen, tend = tbeg + tlen;
    const int tid = threadIdx.x, lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int i16 = lane & 15, kq = lane >> 4;
    float omax = 0.f;   // max |D| of tensor top_u
    float csd = 0.f;    // squared content error of tensor cont_u (this HSLOT-row slot)
    // A fragments: S~_c[u = 16 m + i16][u' = 8 kq .. + 8] as bf16 hi / lo, c = c0 + 8 w + cc
    uint4 sa[8][2][2];
#pragma unroll
    for (int cc = 0; cc < 8; ++cc)
#pragma unroll
        for (int m = 0; m < 2; ++m) {
            const float* sm = a.smat + ((size_t)b * C + c0 + 8 * w + cc) * 1024 + (16 * m + i16) * 32 + 8 * kq;
            const float4 p = *reinterpret_cast<const float4*>(sm);
            const float4 q = *reinterpret_cast<const float4*>(sm + 4);
            uint32_t h[4], l[4];
            split2(p.x, p.y, h[0], l[0]);
            split2(p.z, p.w, h[1], l[1]);
            split2(q.x, q.y, h[2], l[2]);
            split2(q.z, q.w, h[3], l[3]);
            sa[cc][m][0] = make_uint4(h[0], h[1], h[2], h[3]);
            sa[cc][m][1] = make_uint4(l[0], l[1], l[2], l[3]);
        }
    // staging loads: tensors 8 g + k (k < 8, g = w >> 1: wave-uniform), channel quad sq, row st
    // of the stage; a row piece of 64 channels = 16 lanes x 16 B
    const int g = w >> 1, sq = lane >> 2, st = (lane & 3) + 4 * (w & 1);
    __amdgpu_buffer_rsrc_t rs[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        const int u = 8 * g + k;
        rs[k] = h_rsrc(u < a.nu ? (const float*)a.act + (size_t)a.uid[u] * a.tstride + (size_t)b * a.T * C : (const float*)a.zero16, u < a.nu);
    }
    __amdgpu_buffer_rsrc_t rsw[DOOP ? 8 : 1];
    if (DOOP) {
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const int u = 8 * g + k;
            rsw[k] = h_rsrc(u < a.nu ? (const float*)a.actw + (size_t)a.uid[u] * a.tstride + (size_t)b * a.T * C : (const float*)a.zero16, u < a.nu);
        }
    }
    const uint32_t lofs = (uint32_t)(c0 + 4 * sq) * 4u;   // bytes
    // fused content tap: the 128 threads whose output pieces (iteration cont_u & 7 of the store
    // loop) are tensor cont_u's load its E and phi rows at the start of each stage
    const int ctt = (tid >> 4) & 7, cq = tid & 15;
    const bool cthr = CONT && g == (a.cont_u >> 3);
    // iterations of the store loop (wave-uniform): tensors u = 8 g + it < nu; the content
    // tensor's and the top tensor's (or -1)
    const int nlive = min(max(a.nu - 8 * g, 0), 8);
    const int cit = cthr ? a.cont_u & 7 : -1;
    const int tit = a.top_u >= 0 && (a.top_u >> 3) == g ? a.top_u & 7 : -1;
    __amdgpu_buffer_rsrc_t rce, rcp;   // the content tensor's clip and the clip's phi (+ cont_off)
    if (CONT) {
        rce = h_rsrc((const float*)a.act + (size_t)a.uid[a.cont_u & 31] * a.tstride + (size_t)b * a.T * C, true);
        rcp = h_rsrc(a.cont_phi + (size_t)b * a.cont_phi_bstride + a.cont_off, true);
    }
    float4 vr[2][8];
    // unconditional loads (past the chunk a stage re-reads the chunk's last stage, an L2 hit)
    auto load = [&](float4 (&v)[8], int t0) {
        const int tr = min(t0, tend - HSS);
        const uint32_t vo = lofs + (uint32_t)(tr + st) * (C * 4);
#pragma unroll
        for (int k = 0; k < 8; ++k) v[k] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rs[k], vo, 0, 0));
    };
    auto stage = [&](float4 (&v)[8], int t0) {
        float4 ce, cph = make_float4(0.f, 0.f, 0.f, 0.f);
        if (CONT && cthr) {
            ce = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(
                rce, ((uint32_t)(t0 + ctt) * C + (uint32_t)(c0 + 4 * cq)) * 4u, 0, 0));
            if (c0 + 4 * cq < a.cont_ncol)   // (phi rows hold only cont_ncol channels)
                cph = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(
                    rcp, ((uint32_t)(t0 + ctt) * (uint32_t)a.cont_ncc + (uint32_t)(c0 + 4 * cq)) * 4u, 0, 0));
        }
        __syncthreads();   // the previous stage's image and O reads are done
        // channel 4 sq + j: K positions 8 g .. 8 g + 7, split straight into the image
#define HSPLIT(J) { uint4 fh, fl; const int c = 4 * sq + J; \
        const int o = (c * HSS + st) * 32 + 8 * (g ^ hswz(c, st)); \
        split8<J>(v, fh, fl); *reinterpret_cast<uint4*>(&IH[o]) = fh; *reinterpret_cast<uint4*>(&IL[o]) = fl; }
        HSPLIT(0) HSPLIT(1) HSPLIT(2) HSPLIT(3)
#undef HSPLIT
        load(v, t0 + 2 * HSS);
        __syncthreads();
        // D_c = S~_c E_c for the wave's 8 channels; lane (i16, kq) holds D_c[16 m + 4 kq + i][i16 & 7]
        const int tr8 = i16 & 7;
#pragma unroll
        for (int cc = 0; cc < 8; ++cc) {
            const int cl = 8 * w + cc;
            const int o = (cl * HSS + tr8) * 32 + 8 * (kq ^ hswz(cl, tr8));
            const uint4 bh = *reinterpret_cast<const uint4*>(&IH[o]);
            const uint4 bl = *reinterpret_cast<const uint4*>(&IL[o]);
#pragma unroll
            for (int m = 0; m < 2; ++m) {
                f32x4 acc = {0.f, 0.f, 0.f, 0.f};
                acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, sa[cc][m][0]),
                                                             __builtin_bit_cast(bf16x8, bh), acc, 0, 0, 0);
                acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, sa[cc][m][1]),
                                                             __builtin_bit_cast(bf16x8, bh), acc, 0, 0, 0);
                acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, sa[cc][m][0]),
                                                             __builtin_bit_cast(bf16x8, bl), acc, 0, 0, 0);
                // (lanes i16 >= 8 hold the same values as i16 - 8: they write them again, no branch)
#pragma unroll
                for (int i = 0; i < 4; ++i) O[((16 * m + 4 * kq + i) * HSS + tr8) * HOR + cl] = acc[i];
            }
            __builtin_amdgcn_sched_barrier(0);   // one channel's fragments live at a time (registers)
        }
        float4 cadd = make_float4(0.f, 0.f, 0.f, 0.f);
        if (CONT && cthr) {
            const int cc0 = c0 + 4 * cq;
            const float ev[4] = {ce.x, ce.y, ce.z, ce.w}, pv[4] = {cph.x, cph.y, cph.z, cph.w};
            float d[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                d[i] = cc0 + i < a.cont_ncol ? ev[i] - pv[i] : 0.f;
                csd = fmaf(d[i], d[i], csd);
            }
            cadd = make_float4(a.cont_coef * d[0], a.cont_coef * d[1], a.cont_coef * d[2], a.cont_coef * d[3]);
        }
        __syncthreads();
        // 32 tensors x 8 rows x 16 quads: tensor u = 8 g + it through its staging resource rs[it]
        // (in place: act and actw are the same buffer)
        const uint32_t so = ((uint32_t)(t0 + ctt) * C + (uint32_t)(c0 + 4 * cq)) * 4u;
#pragma unroll
        for (int it = 0; it < 8; ++it) {
            const int u = 8 * g + it;
            if (it < nlive) {
                float4 o = *reinterpret_cast<const float4*>(&O[(u * HSS + ctt) * HOR + 4 * cq]);
                if (CONT && it == cit) { o.x += cadd.x; o.y += cadd.y; o.z += cadd.z; o.w += cadd.w; }
                __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(hu32x4, o), DOOP ? rsw[DOOP ? it : 0] : rs[it], so, 0, 0);
                if (it == tit)
                    omax = fmaxf(omax, fmaxf(fmaxf(fabsf(o.x), fabsf(o.y)), fmaxf(fabsf(o.z), fabsf(o.w))));
            }
        }
    };
    load(vr[0], tbeg);
    load(vr[1], tbeg + HSS);
    auto flush_c = [&](int slot) {
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) csd += __shfl_xor(csd, off);
        if (lane == 0) cws[w] = csd;
        __syncthreads();
        if (tid == 0) {
            float v = 0.f;
#pragma unroll
            for (int k = 0; k < HWT / 64; ++k) v += cws[k];
            a.cont_part[(size_t)b * a.cont_pstride + slot * (C / HCH) + c0 / HCH] = v;
        }
        csd = 0.f;
    };
    for (int t0 = tbeg; t0 < tend; t0 += 2 * HSS) {
        stage(vr[0], t0);
        if (CONT && (t0 + HSS) % HSLOT == 0) flush_c(t0 / HSLOT);
        stage(vr[1], t0 + HSS);
        if (CONT && (t0 + 2 * HSS) % HSLOT == 0) flush_c((t0 + HSS) / HSLOT);
    }
    if (a.top_u >= 0) {   // one atomic per workgroup
        __shared__ float wm[HWT / 64];
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) omax = fmaxf(omax, __shfl_xor(omax, off));
        if (lane == 0) wm[w] = omax;
        __syncthreads();
        if (tid == 0) {
            float m = wm[0];
#pragma unroll
            for (int k = 1; k < HWT / 64; ++k) m = fmaxf(m, wm[k]);
            atomicMax(gslot(a.gmax_top, b, blockIdx.x), __float_as_uint(m));
        }
    }
}

// ---- fp32 mode (precision 0): the same staging and data movement on fp32 MFMA ----
// forward: image [c][u][t] fp32 (row stride FRF floats: 80 B, conflict-free 16-B reads); the
// symmetric Gram as three v_mfma_f32_16x16x4f32 tiles (U0 U0, U0 U1, U1 U1; U = 16 tensors) per
// k-step, the fourth written as the mirror of (U0, U1): 3/4 of the MFMA cycles of one 32x32 tile.
constexpr int FRF = 20;

__global__ void __launch_bounds__(GWT) k_gram_fwd_f(GramArgs a) {
    __shared__ __attribute__((aligned(16))) float I[GCS * 32 * FRF];   // [c][u][t]
    int b, ch, c0;
    decode(a, b, ch, c0);
    const int tlen = a.T / a.nchunk, tbeg = ch * tlen;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int i16 = lane & 15, kq = lane >> 4;
    const int su = 8 * (w & 3) + (lane & 7), sq = lane >> 3, tb = w >> 2;
    const bool real = su < a.nu;
    const float* src = real ? (const float*)a.act + (size_t)a.uid[su] * a.tstride +
                              (size_t)b * a.T * C + c0 + 4 * sq + (size_t)8 * tb * C
                            : (const float*)a.zero16;
    const size_t rs = real ? C : 0;
    f32x4 acc[4][3];   // per channel: Gram tiles (U0, U0), (U0, U1), (U1, U1); (U1, U0) = mirror
#pragma unroll
    for (int cc = 0; cc < 4; ++cc)
#pragma unroll
        for (int q = 0; q < 3; ++q) acc[cc][q] = f32x4{0.f, 0.f, 0.f, 0.f};
    float4 v0[8], v1[8];
    // unconditional loads (past the chunk: its last stage again), as k_gram_fwd_s
    auto load = [&](float4 (&v)[8], int t0) {
        const int tr = min(t0, tbeg + tlen - GSS);
#pragma unroll
        for (int k = 0; k < 8; ++k) v[k] = *reinterpret_cast<const float4*>(src + (size_t)(tr + k) * rs);
    };
    auto stage = [&](float4 (&v)[8], int t0) {
        float4 f[4][2];   // channel 4 sq + j: rows 8 tb .. + 8
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            auto e = [&](int k) { return j == 0 ? v[k].x : j == 1 ? v[k].y : j == 2 ? v[k].z : v[k].w; };
            f[j][0] = make_float4(e(0), e(1), e(2), e(3));
            f[j][1] = make_float4(e(4), e(5), e(6), e(7));
        }
        load(v, t0 + 2 * GSS);
        __syncthreads();
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            float* row = &I[((4 * sq + j) * 32 + su) * FRF + 8 * tb];
            *reinterpret_cast<float4*>(row) = f[j][0];
            *reinterpret_cast<float4*>(row + 4) = f[j][1];
        }
        __syncthreads();
        // 16x16x4 tiles: lane (i16, kq) supplies tensor U + i16 at rows 4 kq .. 4 kq + 3 (k-step s
        // takes row 4 kq + s: any common permutation of K is the same Gram) for A and B alike
#pragma unroll
        for (int cc = 0; cc < 4; ++cc) {
            const float* base = &I[(4 * w + cc) * 32 * FRF + 4 * kq];
            const float4 u0 = *reinterpret_cast<const float4*>(base + i16 * FRF);
            const float4 u1 = *reinterpret_cast<const float4*>(base + (16 + i16) * FRF);
            const float a0[4] = {u0.x, u0.y, u0.z, u0.w}, a1[4] = {u1.x, u1.y, u1.z, u1.w};
#pragma unroll
            for (int st = 0; st < 4; ++st) {
                acc[cc][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(a0[st], a0[st], acc[cc][0], 0, 0, 0);
                acc[cc][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(a0[st], a1[st], acc[cc][1], 0, 0, 0);
                acc[cc][2] = __builtin_amdgcn_mfma_f32_16x16x4f32(a1[st], a1[st], acc[cc][2], 0, 0, 0);
            }
        }
    };
    load(v0, tbeg);
    load(v1, tbeg + GSS);
    for (int t0 = tbeg; t0 < tbeg + tlen; t0 += 2 * GSS) {
        stage(v0, t0);
        stage(v1, t0 + GSS);
    }
#pragma unroll
    for (int cc = 0; cc < 4; ++cc) {   // lane holds G[U + 4 kq + i][U' + i16] (C/D map of 16x16x4)
        float* dst = a.gpart + (((size_t)b * a.nchunk + ch) * C + c0 + 4 * w + cc) * 1024;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int rr = 4 * kq + i;
            dst[rr * 32 + i16] = acc[cc][0][i];
            dst[rr * 32 + 16 + i16] = acc[cc][1][i];
            dst[(16 + i16) * 32 + rr] = acc[cc][1][i];
            dst[(16 + rr) * 32 + 16 + i16] = acc[cc][2][i];
        }
    }
}

// fp32 forward for very few clips: k_gram_fwd_n's staging (8 channels, 64-row fills, wave w
// = channel c0 + w) with k_gram_fwd_f's per-channel MFMA sequence, stage by stage: the same
// partials bit for bit
__global__ void __launch_bounds__(GWT) k_gram_fwd_fn(GramArgs a) {
    __shared__ __attribute__((aligned(16))) float I[(GFN / GSS) * GCN * 32 * FRF];   // [stage][c][u][t]
    constexpr int ncg = C / GCN;
    const int nwg = a.B * a.nchunk * ncg;
    int work = xcd_remap(blockIdx.x, nwg);
    const int cgi = work % ncg; work /= ncg;
    const int ch = work % a.nchunk, b = work / a.nchunk, c0 = cgi * GCN;
    const int tlen = a.T / a.nchunk, tbeg = ch * tlen, tend = tbeg + tlen;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int i16 = lane & 15, kq = lane >> 4;
    const int su = 8 * (w & 3) + (lane & 7), sq = (lane >> 3) & 1, g = (lane >> 4) + 4 * (w >> 2);
    const bool real = su < a.nu;
    const float* src = real ? (const float*)a.act + (size_t)a.uid[su] * a.tstride +
                              (size_t)b * a.T * C + c0 + 4 * sq + (size_t)8 * g * C
                            : (const float*)a.zero16;
    const size_t rs = real ? C : 0;
    f32x4 acc[3];
#pragma unroll
    for (int q = 0; q < 3; ++q) acc[q] = f32x4{0.f, 0.f, 0.f, 0.f};
    float4 v[2][8];
    auto load = [&](float4 (&vv)[8], int t0) {
#pragma unroll
        for (int k = 0; k < 8; ++k) vv[k] = *reinterpret_cast<const float4*>(src + (size_t)(t0 + k) * rs);
    };
    auto fill = [&](float4 (&vv)[8], int t0) {
        float4 f[4][2];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            auto e = [&](int k) { return j == 0 ? vv[k].x : j == 1 ? vv[k].y : j == 2 ? vv[k].z : vv[k].w; };
            f[j][0] = make_float4(e(0), e(1), e(2), e(3));
            f[j][1] = make_float4(e(4), e(5), e(6), e(7));
        }
        if (t0 + 2 * GFN < tend) load(vv, t0 + 2 * GFN);
        __syncthreads();
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            float* row = &I[(((g >> 1) * GCN + 4 * sq + j) * 32 + su) * FRF + 8 * (g & 1)];
            *reinterpret_cast<float4*>(row) = f[j][0];
            *reinterpret_cast<float4*>(row + 4) = f[j][1];
        }
        __syncthreads();
#pragma unroll
        for (int sg = 0; sg < GFN / GSS; ++sg) {
            const float* base = &I[(sg * GCN + w) * 32 * FRF + 4 * kq];
            const float4 u0 = *reinterpret_cast<const float4*>(base + i16 * FRF);
            const float4 u1 = *reinterpret_cast<const float4*>(base + (16 + i16) * FRF);
            const float a0[4] = {u0.x, u0.y, u0.z, u0.w}, a1[4] = {u1.x, u1.y, u1.z, u1.w};
#pragma unroll
            for (int st = 0; st < 4; ++st) {
                acc[0] = __builtin_amdgcn_mfma_f32_16x16x4f32(a0[st], a0[st], acc[0], 0, 0, 0);
                acc[1] = __builtin_amdgcn_mfma_f32_16x16x4f32(a0[st], a1[st], acc[1], 0, 0, 0);
                acc[2] = __builtin_amdgcn_mfma_f32_16x16x4f32(a1[st], a1[st], acc[2], 0, 0, 0);
            }
        }
    };
    load(v[0], tbeg);
    if (tbeg + GFN < tend) load(v[1], tbeg + GFN);
    for (int t0 = tbeg; t0 < tend; t0 += 2 * GFN) {
        fill(v[0], t0);
        if (t0 + GFN < tend) fill(v[1], t0 + GFN);
    }
    float* dst = a.gpart + (((size_t)b * a.nchunk + ch) * C + c0 + w) * 1024;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int rr = 4 * kq + i;
        dst[rr * 32 + i16] = acc[0][i];
        dst[rr * 32 + 16 + i16] = acc[1][i];
        dst[(16 + i16) * 32 + rr] = acc[1][i];
        dst[(16 + rr) * 32 + 16 + i16] = acc[2][i];
    }
}

// backward: image [c][t][u] fp32, 32 floats per row with the four 8-tensor blocks swizzled
// (block kq of row t at 8 (kq ^ (t & 3)): conflict-free 16-B reads); D_c = S~_c E_c on
// v_mfma_f32_16x16x4f32: A = S~_c[u = 16 m + i16][u' = 8 kq + ks] in registers, B: lane
// (t = i16, kq) reads E_{8 kq .. + 8}[t][c] (two 16-B reads), k-step ks.  Output as the split
// kernel's (O image, whole 128-B lines, in place over E, + the content grad).
__device__ __forceinline__ int bswz(int kq, int t) { return 8 * (kq ^ (t & 3)); }

// HCG: some tensor has a content-gradient buffer (a branch around a load in the store loop
// otherwise makes the compiler drain every stage load in flight)
template <bool HCG>
__global__ void __launch_bounds__(GWT) k_gram_bwd_f(GramArgs a) {
    __shared__ __attribute__((aligned(16))) float IB[GCS * GSS * 32];     // [c][t][u]
    __shared__ __attribute__((aligned(16))) float O[16 * GSS * ORS];      // [u][t][c]
    int b, ch, c0;
    decode(a, b, ch, c0);
    const int tlen = a.T / a.nchunk, tbeg = ch * tlen, tend = tbeg + tlen;
    const int tid = threadIdx.x, lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int i16 = lane & 15, kq = lane >> 4;
    float sa[4][2][8];
#pragma unroll
    for (int cc = 0; cc < 4; ++cc)
#pragma unroll
        for (int m = 0; m < 2; ++m) {
            const float* sm = a.smat + ((size_t)b * C + c0 + 4 * w + cc) * 1024 + (16 * m + i16) * 32 + 8 * kq;
            const float4 p = *reinterpret_cast<const float4*>(sm);
            const float4 q = *reinterpret_cast<const float4*>(sm + 4);
            sa[cc][m][0] = p.x; sa[cc][m][1] = p.y; sa[cc][m][2] = p.z; sa[cc][m][3] = p.w;
            sa[cc][m][4] = q.x; sa[cc][m][5] = q.y; sa[cc][m][6] = q.z; sa[cc][m][7] = q.w;
        }
    const int uo = w & 3, sq = lane >> 3, st = 8 * (w >> 2) + (lane & 7);
    const size_t rowoff = (size_t)b * a.T * C + c0 + 4 * sq;
    const float* ld[8];
    size_t lrs[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        const int u = 8 * uo + k;
        ld[k] = u < a.nu ? (const float*)a.act + (size_t)a.uid[u] * a.tstride + rowoff : (const float*)a.zero16;
        lrs[k] = u < a.nu ? C : 0;
    }
    float4 v0[8], v1[8];
    auto load = [&](float4 (&v)[8], int t0) {   // (past the chunk: its last stage again)
        const int tr = min(t0, tend - GSS);
#pragma unroll
        for (int k = 0; k < 8; ++k) v[k] = *reinterpret_cast<const float4*>(ld[k] + (size_t)(tr + st) * lrs[k]);
    };
    auto stage = [&](float4 (&v)[8], int t0) {
        float4 f[4][2];   // channel 4 sq + j: tensors 8 uo .. + 8 at row st
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            auto e = [&](int k) { return j == 0 ? v[k].x : j == 1 ? v[k].y : j == 2 ? v[k].z : v[k].w; };
            f[j][0] = make_float4(e(0), e(1), e(2), e(3));
            f[j][1] = make_float4(e(4), e(5), e(6), e(7));
        }
        load(v, t0 + 2 * GSS);
        __syncthreads();   // the previous stage's image and O reads are done
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            float* row = &IB[((4 * sq + j) * GSS + st) * 32 + bswz(uo, st)];
            *reinterpret_cast<float4*>(row) = f[j][0];
            *reinterpret_cast<float4*>(row + 4) = f[j][1];
        }
        __syncthreads();
        f32x4 acc[4][2];
#pragma unroll
        for (int cc = 0; cc < 4; ++cc) {
            const float* row = &IB[((4 * w + cc) * GSS + i16) * 32 + bswz(kq, i16)];
            const float4 p = *reinterpret_cast<const float4*>(row);
            const float4 q = *reinterpret_cast<const float4*>(row + 4);
            const float bv[8] = {p.x, p.y, p.z, p.w, q.x, q.y, q.z, q.w};
#pragma unroll
            for (int m = 0; m < 2; ++m) {
                f32x4 c = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
                for (int ks = 0; ks < 8; ++ks)
                    c = __builtin_amdgcn_mfma_f32_16x16x4f32(sa[cc][m][ks], bv[ks], c, 0, 0, 0);
                acc[cc][m] = c;
            }
        }
        // lane holds D_c[u = 16 m + 4 kq + i][t = i16] for the wave's 4 channels
#pragma unroll
        for (int m = 0; m < 2; ++m) {
            if (m) __syncthreads();   // the first half's O reads are done
#pragma unroll
            for (int cc = 0; cc < 4; ++cc)
#pragma unroll
                for (int i = 0; i < 4; ++i)
                    O[((4 * kq + i) * GSS + i16) * ORS + 4 * w + cc] = acc[cc][m][i];
            __syncthreads();
#pragma unroll
            for (int it = 0; it < 4; ++it) {   // (wave-uniform tensor: k_gram_bwd_s)
                const int ul = 4 * it + (w >> 1), tt = (tid >> 3) & 15, q = tid & 7;
                const int u = 16 * m + ul;
                if (u < a.nu) {
                    float4 o = *reinterpret_cast<const float4*>(&O[(ul * GSS + tt) * ORS + 4 * q]);
                    const size_t off = (size_t)a.uid[u] * a.tstride + ((size_t)b * a.T + t0 + tt) * C + c0 + 4 * q;
                    const float* cg = HCG ? (const float*)a.cg[u] : nullptr;
                    if (HCG && cg) {
                        const float4 g = *reinterpret_cast<const float4*>(cg + ((size_t)b * a.T + t0 + tt) * C + c0 + 4 * q);
                        o.x += g.x; o.y += g.y; o.z += g.z; o.w += g.w;
                    }
                    *reinterpret_cast<float4*>((float*)a.actw + off) = o;
                }
            }
        }
    };
    load(v0, tbeg);
    load(v1, tbeg + GSS);
    for (int t0 = tbeg; t0 < tend; t0 += 2 * GSS) {
        stage(v0, t0);
        stage(v1, t0 + GSS);
    }
}

}  // namespace

static int gram_bwd_stages() {   // ASTYLE_GRAM_BWD_STAGES=2 / 3 (A/B; default 2 until measured)
    static int v = -1;
    if (v < 0) { const char* e = getenv("ASTYLE_GRAM_BWD_STAGES"); v = e ? atoi(e) : 2; if (v != 3) v = 2; }
    return v;
}
static int gram_stages() {   // ASTYLE_GRAM_STAGES=2 / 3 (A/B; default 3)
    static int v = -1;
    if (v < 0) { const char* e = getenv("ASTYLE_GRAM_STAGES"); v = e ? atoi(e) : 3; if (v != 2) v = 3; }
    return v;
}
void launch_gram_fwd_s(const GramArgs& a, hipStream_t s) {
    // very few clips (under 64 workgroups with 32-channel groups; measured: one clip 0.54 ->
    // 0.28 ms, 8 clips 0.65 -> 0.78 ms, the 32-B row pieces cost more than the extra
    // workgroups return): the 8-channel kernel, same bits
    if ((size_t)a.B * a.nchunk * (C / GCS) < 64 && (a.T / a.nchunk) % GFN == 0) {
        // one clip: 4 channels per workgroup (twice the workgroups) and 3 fills in flight; more
        // clips: 8 and 2 (round 6, one clip: Gram forward 0.343 -> 0.233 ms, same bits,
        // profiles/r6_diag/fewclip_ab.txt).  A/B knobs: ASTYLE_GRAM_FWDN_NC (4 / 8),
        // ASTYLE_GRAM_FWDN_FILLS (2 / 3)
        static int nfl = -1, ncw = -1;
        if (nfl < 0) { const char* e = getenv("ASTYLE_GRAM_FWDN_FILLS"); nfl = e ? atoi(e) : 0; }
        if (ncw < 0) { const char* e = getenv("ASTYLE_GRAM_FWDN_NC"); ncw = e ? atoi(e) : 0; }
        const int nc = ncw ? ncw : (a.B == 1 ? 4 : 8);
        const int nf = nfl ? nfl : (nc == 4 ? 3 : 2);
        const dim3 grid(a.B * a.nchunk * (C / nc));
        if (nc == 4) {
            if (nf <= 2) hipLaunchKernelGGL((k_gram_fwd_n<2, 4>), grid, dim3(256), 0, s, a);
            else hipLaunchKernelGGL((k_gram_fwd_n<3, 4>), grid, dim3(256), 0, s, a);
        } else {
            if (nf <= 2) hipLaunchKernelGGL((k_gram_fwd_n<2, 8>), grid, dim3(GWT), 0, s, a);
            else hipLaunchKernelGGL((k_gram_fwd_n<3, 8>), grid, dim3(GWT), 0, s, a);
        }
        return;
    }
    if (gram_stages() == 2) hipLaunchKernelGGL(k_gram_fwd_s<2>, dim3(a.B * a.nchunk * (C / GCS)), dim3(GWT), 0, s, a);
    else hipLaunchKernelGGL(k_gram_fwd_s<3>, dim3(a.B * a.nchunk * (C / GCS)), dim3(GWT), 0, s, a);
}
void launch_gram_fwd(const GramArgs& a, hipStream_t s) {
    if ((size_t)a.B * a.nchunk * (C / GCS) < 64 && (a.T / a.nchunk) % GFN == 0) {   // (as launch_gram_fwd_s)
        hipLaunchKernelGGL(k_gram_fwd_fn, dim3(a.B * a.nchunk * (C / GCN)), dim3(GWT), 0, s, a);
        return;
    }
    hipLaunchKernelGGL(k_gram_fwd_f, dim3(a.B * a.nchunk * (C / GCS)), dim3(GWT), 0, s, a);
}
void launch_gram_bwd(const GramArgs& a, hipStream_t s) {
    bool has_cg = false;
    for (int u = 0; u < a.nu; ++u) has_cg = has_cg || a.cg[u];
    if (has_cg) hipLaunchKernelGGL(k_gram_bwd_f<true>, dim3(a.B * a.nchunk * (C / GCS)), dim3(GWT), 0, s, a);
    else hipLaunchKernelGGL(k_gram_bwd_f<false>, dim3(a.B * a.nchunk * (C / GCS)), dim3(GWT), 0, s, a);
}
// Chunks of the half-row backward: the fewest whole-slot chunks, at least 4, that give >= 4096
// workgroups (depends on B and T only; the results do not depend on it)
static int gram_bwd_h_chunks(int B, int T) {
    const int slots = T / HSLOT;
    int d = 1;
    for (int k = 1; k <= slots; ++k) {
        if (slots % k) continue;
        d = k;
        if (k >= 4 && (size_t)B * k * 2 >= 4096) break;
    }
    return d;
}
static bool gram_bwd_half() {   // ASTYLE_GRAM_BWD_H=0: the 32-channel kernel (A/B)
    static int v = -1;
    if (v < 0) { const char* e = getenv("ASTYLE_GRAM_BWD_H"); v = e ? (atoi(e) != 0) : 1; }
    return v != 0;
}
bool gram_bwd_s_half(const GramArgs& a) {   // (a content-gradient buffer: the 32-channel kernel)
    if (!gram_bwd_half() || a.T % HSLOT) return false;
    for (int u = 0; u < a.nu; ++u) if (a.cg[u]) return false;
    return true;
}
void launch_gram_bwd_s(const GramArgs& a0, hipStream_t s) {
    if (gram_bwd_s_half(a0)) {
        GramArgs a = a0;
        a.nchunk = gram_bwd_h_chunks(a.B, a.T);
        const dim3 grid(a.B * a.nchunk * 2);
        const bool doop = a.actw != a.act;
        if (a.cont_u >= 0) {
            if (doop) hipLaunchKernelGGL((k_gram_bwd_h<true, true>), grid, dim3(HWT), 0, s, a);
            else hipLaunchKernelGGL((k_gram_bwd_h<true, false>), grid, dim3(HWT), 0, s, a);
        } else {
            if (doop) hipLaunchKernelGGL((k_gram_bwd_h<false, true>), grid, dim3(HWT), 0, s, a);
            else hipLaunchKernelGGL((k_gram_bwd_h<false, false>), grid, dim3(HWT), 0, s, a);
        }
        return;
    }
    const GramArgs& a = a0;
    const dim3 grid(a.B * a.nchunk * (C / GCS));
    if (a.cont_u >= 0 && (a.T / a.nchunk) % GRAM_CSLOT) {
        fprintf(stderr, "gram_bwd_s: the fused content tap needs whole %d-row chunks\n", GRAM_CSLOT);
        abort();
    }
    bool has_cg = false;
    for (int u = 0; u < a.nu; ++u) has_cg = has_cg || a.cg[u];
#define GBS(CT, NS) if (has_cg) hipLaunchKernelGGL((k_gram_bwd_s<CT, NS, true>), grid, dim3(GWT), 0, s, a); \
                    else hipLaunchKernelGGL((k_gram_bwd_s<CT, NS, false>), grid, dim3(GWT), 0, s, a);
    if (gram_bwd_stages() == 3) {
        if (a.cont_u >= 0) { GBS(true, 3) } else { GBS(false, 3) }
    } else {
        if (a.cont_u >= 0) { GBS(true, 2) } else { GBS(false, 2) }
    }
#undef GBS
}

}  // namespace ast
