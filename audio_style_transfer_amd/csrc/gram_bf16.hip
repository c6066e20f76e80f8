// bf16 channel-wise ("ours") Gram forward/backward (precision 1), methods.py:62-76.
//
// Per (clip, time chunk, 32-channel (fwd) / 64-channel (bwd) group) workgroup; per channel c the Gram is a
// 32 x 32 (tensors x tensors) product over time with fp32 accumulation:
//   fwd  G_c = E_c E_c^T   v_mfma_f32_32x32x16_bf16, A = B = one fragment:
//                          lane (u, kg) holds E_u[t0+8kg .. +8][c]
//   bwd  D_c = S~_c E_c    v_mfma_f32_16x16x32_bf16 per 16-row stage, A = S~_c (bf16, in
//                          registers), B: lane (t, kg) holds E_{8kg .. 8kg+7}[t][c]
// HBM is channels-last ([u][t][c]); the MFMA wants time- (fwd) or tensor- (bwd) contiguous
// fragments, so staging transposes 8 x 8 bf16 blocks in registers (byte permutes) into a
// padded LDS image.  Global accesses are 64-B (fwd) / whole 128-B line (bwd) row segments,
// the next stage's loads are in flight while a stage computes, and in the backward
// every load and store is unconditional (padding tensors read / re-store tensor nu-1) with
// the loop rotated so a wait for loads never drains the stage's outstanding stores.
// Block ids are remapped so the 4 channel groups of one time chunk run on one XCD (one L2).
#include "common.h"

namespace ast {

constexpr int GCG = 32;   // fwd: channels per workgroup (4 waves)
constexpr int GCB2 = 64;  // bwd: channels per workgroup (8 waves; whole 128-B line writes)
constexpr int GST = 16;   // time rows per stage
constexpr int FIS = 24;   // fwd LDS image [c][u][t] row stride (bf16): 48 B
constexpr int BIS = 40;   // bwd LDS image [c][t][u] row stride (bf16): 80 B

typedef float f32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
    const int xcd = bid % 8, q = nwg / 8, rr = nwg % 8;
    return (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + bid / 8;
}

// in[k] = 8 bf16 (elements j = 0..7) of row k  ->  out[j] = 8 bf16 (rows k = 0..7) of column j
__device__ __forceinline__ void transpose8(const uint4 (&in)[8], uint4 (&out)[8]) {
    uint32_t d[8][4];
#pragma unroll
    for (int k = 0; k < 8; ++k) { d[k][0] = in[k].x; d[k][1] = in[k].y; d[k][2] = in[k].z; d[k][3] = in[k].w; }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        uint32_t o[4];
#pragma unroll
        for (int p = 0; p < 4; ++p) {
            const uint32_t x = d[2 * p][j >> 1], y = d[2 * p + 1][j >> 1];
            o[p] = (j & 1) ? ((x >> 16) | (y & 0xffff0000u)) : ((x & 0xffffu) | (y << 16));
        }
        out[j] = make_uint4(o[0], o[1], o[2], o[3]);
    }
}

template <int G>
__device__ __forceinline__ void gram_decode(const GramArgs& a, int& b, int& ch, int& c0) {
    const int ncg = C / G;
    const int nwg = a.B * a.nchunk * ncg;
    int work = xcd_remap(blockIdx.x, nwg);
    const int cgi = work % ncg; work /= ncg;
    ch = work % a.nchunk;
    b = work / a.nchunk;
    c0 = cgi * G;
}

__global__ void __launch_bounds__(256) k_gram_fwd_bf16(GramArgs a) {
    __shared__ __attribute__((aligned(16))) u16 If[GCG * 32 * FIS];   // [c][u][t]
    const u16* act = (const u16*)a.act;
    int b, ch, c0;
    gram_decode<GCG>(a, b, ch, c0);
    const int tlen = a.T / a.nchunk, tbeg = ch * tlen;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int r = lane & 31, h = lane >> 5;
    // staging item: tensor su, 8-row time block stb, 8-channel octet so (octet fastest: 4
    // lanes cover one 64-B row segment)
    const int su = tid >> 3, stb = (tid >> 2) & 1, so = tid & 3;
    // padding tensors (su >= nu) read a 16-B zero line (row stride 0) instead of re-fetching a
    // real tensor: their Gram rows are unused
    const bool real = su < a.nu;
    const u16* src = real ? act + (size_t)a.uid[su] * a.tstride + (size_t)b * a.T * C + c0 + so * 8 +
                            (size_t)stb * 8 * C
                          : (const u16*)a.zero16;
    const size_t rs = real ? C : 0;
    f32x16 acc[8];
#pragma unroll
    for (int cc = 0; cc < 8; ++cc)
        for (int i = 0; i < 16; ++i) acc[cc][i] = 0.f;
    uint4 in[8];
    auto load = [&](int t0) {
#pragma unroll
        for (int k = 0; k < 8; ++k) in[k] = *reinterpret_cast<const uint4*>(src + (size_t)(t0 + k) * rs);
    };
    load(tbeg);
    for (int t0 = tbeg; t0 < tbeg + tlen; t0 += GST) {
        uint4 out[8];
        transpose8(in, out);
        if (t0 + GST < tbeg + tlen) load(t0 + GST);   // next stage in flight during this one
        __syncthreads();
#pragma unroll
        for (int j = 0; j < 8; ++j)
            *reinterpret_cast<uint4*>(&If[((so * 8 + j) * 32 + su) * FIS + stb * 8]) = out[j];
        __syncthreads();
#pragma unroll
        for (int cc = 0; cc < 8; ++cc) {
            const int c = w * 8 + cc;
            const uint4 f = *reinterpret_cast<const uint4*>(&If[(c * 32 + r) * FIS + 8 * h]);
            acc[cc] = mfma_bf16(f, f, acc[cc]);
        }
    }
#pragma unroll
    for (int cc = 0; cc < 8; ++cc) {
        float* dst = a.gpart + (((size_t)b * a.nchunk + ch) * C + c0 + w * 8 + cc) * 1024;
#pragma unroll
        for (int i = 0; i < 16; ++i) dst[((i & 3) + 8 * (i >> 2) + 4 * h) * 32 + r] = acc[cc][i];
    }
}

__global__ void __launch_bounds__(512) k_gram_bwd_bf16(GramArgs a) {
    __shared__ __attribute__((aligned(16))) u16 Ib[GCB2 * GST * BIS];   // [c][t][u]
    const u16* act = (const u16*)a.act;
    u16* actw = (u16*)a.actw;
    int b, ch, c0;
    gram_decode<GCB2>(a, b, ch, c0);
    const int tlen = a.T / a.nchunk, tbeg = ch * tlen, tend = tbeg + tlen;
    const int tid = threadIdx.x, lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int i16 = lane & 15, kq = lane >> 4;
    // A fragments (16x16x32): S~_c[u = 16m + i16][u' = 8kq .. +8], bf16; wave w owns 8 channels
    uint4 sa[8][2];
#pragma unroll
    for (int cc = 0; cc < 8; ++cc)
#pragma unroll
        for (int m = 0; m < 2; ++m) {
            const float* sm = a.smat + ((size_t)b * C + c0 + w * 8 + cc) * 1024 + (16 * m + i16) * 32 + 8 * kq;
            const float4 lo = *reinterpret_cast<const float4*>(sm);
            const float4 hi = *reinterpret_cast<const float4*>(sm + 4);
            sa[cc][m] = make_uint4(pack2(lo.x, lo.y), pack2(lo.z, lo.w), pack2(hi.x, hi.y), pack2(hi.z, hi.w));
        }
    // staging item: 8-tensor block ub (two waves each: scalar tensor bases), time row st,
    // octet so (8 lanes = one whole 128-B line of a row)
    const int ub = __builtin_amdgcn_readfirstlane(tid >> 7);
    const int st = (tid >> 3) & 15, so = tid & 7;
    const size_t rowoff = (size_t)b * a.T * C + c0 + so * 8 + (size_t)st * C;
    // padding slots (u >= nu) alias tensor rbk*8, the first tensor of the last real block, and
    // re-store the value its owner stores (identical bytes to the same address): they read
    // back that block and use its slot 0
    const int rbk = ub < ((a.nu - 1) >> 3) ? ub : ((a.nu - 1) >> 3);
    // tensors without a content grad read a 16-B zero line instead (no branches: every wait
    // on these loads is then countable)
    const u16* ld[8];
    u16* sp[8];
    const u16* cgp[8];
    uint32_t cgs[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        const int u = ub * 8 + k, uu = u < a.nu ? u : rbk * 8;
        ld[k] = act + (size_t)a.uid[uu] * a.tstride + rowoff;
        sp[k] = actw + (size_t)a.uid[uu] * a.tstride + rowoff;
        const u16* g = (const u16*)a.cg[uu];
        cgp[k] = g ? g + rowoff : (const u16*)a.zero16;
        cgs[k] = g ? C : 0;
    }
    uint4 nx[8];
    auto load = [&](int t0) {
#pragma unroll
        for (int k = 0; k < 8; ++k) nx[k] = *reinterpret_cast<const uint4*>(ld[k] + (size_t)t0 * C);
    };
    auto stage_in = [&]() {
        uint4 out[8];
        transpose8(nx, out);       // out[j]: channel so*8+j, tensors ub*8 .. ub*8+7
        __syncthreads();
#pragma unroll
        for (int j = 0; j < 8; ++j)
            *reinterpret_cast<uint4*>(&Ib[((so * 8 + j) * GST + st) * BIS + ub * 8]) = out[j];
    };
    load(tbeg);
    stage_in();
    for (int t0 = tbeg; t0 < tend; t0 += GST) {
        // content-grad rows of this stage (before the prefetch, so their wait leaves it in flight)
        uint4 g[8];
#pragma unroll
        for (int k = 0; k < 8; ++k)
            g[k] = *reinterpret_cast<const uint4*>(cgp[k] + (size_t)t0 * cgs[k]);
        load(t0 + GST < tend ? t0 + GST : t0);
        __syncthreads();
#pragma unroll
        for (int cc = 0; cc < 8; ++cc) {
            const int c = w * 8 + cc;
            const uint4 bf = *reinterpret_cast<const uint4*>(&Ib[(c * GST + i16) * BIS + 8 * kq]);
            f32x4 acc[2];
#pragma unroll
            for (int m = 0; m < 2; ++m)
                acc[m] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
                    __builtin_bit_cast(bf16x8, sa[cc][m]), __builtin_bit_cast(bf16x8, bf),
                    (f32x4){0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
            // lane holds D_c[u = 16m + 4kq + 0..3][t = i16]; this wave alone owns channel c
#pragma unroll
            for (int m = 0; m < 2; ++m)
                *reinterpret_cast<uint2*>(&Ib[(c * GST + i16) * BIS + 16 * m + 4 * kq]) =
                    make_uint2(pack2(acc[m][0], acc[m][1]), pack2(acc[m][2], acc[m][3]));
        }
        __syncthreads();
        uint4 in[8], out[8];
#pragma unroll
        for (int j = 0; j < 8; ++j)
            in[j] = *reinterpret_cast<const uint4*>(&Ib[((so * 8 + j) * GST + st) * BIS + rbk * 8]);
        transpose8(in, out);      // out[k]: tensor rbk*8+k, channels c0+8so .. +8
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            uint4 v = (ub * 8 + k < a.nu) ? out[k] : out[0];
            const uint4 gv = g[k];
            v.x = pack2(bflo(v.x) + bflo(gv.x), bfhi(v.x) + bfhi(gv.x));
            v.y = pack2(bflo(v.y) + bflo(gv.y), bfhi(v.y) + bfhi(gv.y));
            v.z = pack2(bflo(v.z) + bflo(gv.z), bfhi(v.z) + bfhi(gv.z));
            v.w = pack2(bflo(v.w) + bflo(gv.w), bfhi(v.w) + bfhi(gv.w));
            *reinterpret_cast<uint4*>(sp[k] + (size_t)t0 * C) = v;
        }
        if (t0 + GST < tend) stage_in();
    }
}

void launch_gram_fwd_bf16(const GramArgs& a, hipStream_t s) {
    hipLaunchKernelGGL(k_gram_fwd_bf16, dim3(a.B * a.nchunk * (C / GCG)), dim3(256), 0, s, a);
}
void launch_gram_bwd_bf16(const GramArgs& a, hipStream_t s) {
    hipLaunchKernelGGL(k_gram_bwd_bf16, dim3(a.B * a.nchunk * (C / GCB2)), dim3(512), 0, s, a);
}

}  // namespace ast
