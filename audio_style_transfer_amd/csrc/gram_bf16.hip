// bf16 channel-wise ("ours") Gram forward/backward (precision 1), methods.py:62-76.
//
// Per (clip, time chunk, 16-channel group) workgroup; per channel c the Gram is a 32x32
// (tensors x tensors) product over time, on v_mfma_f32_32x32x16_bf16 with fp32 accumulation:
//   fwd  G_c = E_c E_c^T       A = B = the same fragment: lane (u, h) holds E_u[t0+8h..+8][c]
//   bwd  D_c = S~_c E_c        A = S~_c (bf16), B: lane (t, h) holds E_{8h..8h+7}[t][c]
// HBM is channels-last ([u][t][c]) while the MFMA wants time- (fwd) or tensor- (bwd)
// contiguous fragments, so staging transposes 8x8 bf16 blocks in registers (byte permutes)
// and writes 16-B rows into an LDS image with an 80-B row stride (ds_read_b128 conflict-free).
// Block ids are remapped so the 8 channel groups of one time chunk run on one XCD (one L2).
#include "common.h"

namespace ast {

constexpr int GIS = 40;   // LDS image row stride in bf16 (80 B)
constexpr int GCG = 16;   // channels per workgroup

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

__device__ __forceinline__ void gram_decode(const GramArgs& a, int& b, int& ch, int& c0) {
    const int ncg = C / GCG;
    const int nwg = a.B * a.nchunk * ncg;
    int work = xcd_remap(blockIdx.x, nwg);
    const int cgi = work % ncg; work /= ncg;
    ch = work % a.nchunk;
    b = work / a.nchunk;
    c0 = cgi * GCG;
}

__global__ void __launch_bounds__(256) k_gram_fwd_bf16(GramArgs a) {
    __shared__ __attribute__((aligned(16))) u16 If[GCG * 32 * GIS];   // [c][u][t]
    const u16* act = (const u16*)a.act;
    int b, ch, c0;
    gram_decode(a, b, ch, c0);
    const int tlen = a.T / a.nchunk, tbeg = ch * tlen;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int r = lane & 31, h = lane >> 5;
    // staging item: tensor u, 8-row time block tb, 8-channel group q
    const int su = tid >> 3, stb = (tid >> 1) & 3, sq = tid & 1;
    const u16* src = su < a.nu ? act + (size_t)a.uid[su] * a.tstride + (size_t)b * a.T * C + c0 + sq * 8
                               : nullptr;
    f32x16 acc[4];
#pragma unroll
    for (int cc = 0; cc < 4; ++cc)
        for (int i = 0; i < 16; ++i) acc[cc][i] = 0.f;
    uint4 in[8];
    auto load = [&](int t0) {
#pragma unroll
        for (int k = 0; k < 8; ++k)
            in[k] = src ? *reinterpret_cast<const uint4*>(src + (size_t)(t0 + stb * 8 + k) * C)
                        : make_uint4(0, 0, 0, 0);
    };
    load(tbeg);
    for (int t0 = tbeg; t0 < tbeg + tlen; t0 += 32) {
        uint4 out[8];
        transpose8(in, out);
        if (t0 + 32 < tbeg + tlen) load(t0 + 32);   // next stage in flight during this one
        __syncthreads();
#pragma unroll
        for (int j = 0; j < 8; ++j)
            *reinterpret_cast<uint4*>(&If[((sq * 8 + j) * 32 + su) * GIS + stb * 8]) = out[j];
        __syncthreads();
#pragma unroll
        for (int cc = 0; cc < 4; ++cc) {
            const int c = w * 4 + cc;
#pragma unroll
            for (int kb = 0; kb < 2; ++kb) {
                const uint4 f = *reinterpret_cast<const uint4*>(&If[(c * 32 + r) * GIS + kb * 16 + 8 * h]);
                acc[cc] = mfma_bf16(f, f, acc[cc]);
            }
        }
    }
#pragma unroll
    for (int cc = 0; cc < 4; ++cc) {
        float* dst = a.gpart + (((size_t)b * a.nchunk + ch) * C + c0 + w * 4 + cc) * 1024;
#pragma unroll
        for (int i = 0; i < 16; ++i) dst[((i & 3) + 8 * (i >> 2) + 4 * h) * 32 + r] = acc[cc][i];
    }
}

__global__ void __launch_bounds__(256) k_gram_bwd_bf16(GramArgs a) {
    __shared__ __attribute__((aligned(16))) u16 Ib[GCG * 32 * GIS];   // [c][t][u]
    const u16* act = (const u16*)a.act;
    u16* actw = (u16*)a.actw;
    int b, ch, c0;
    gram_decode(a, b, ch, c0);
    const int tlen = a.T / a.nchunk, tbeg = ch * tlen;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int r = lane & 31, h = lane >> 5;
    // A fragments: S~_c[u = r][u' = kb*16 + 8h .. +8] in bf16
    uint4 sa[4][2];
#pragma unroll
    for (int cc = 0; cc < 4; ++cc) {
        const float* sm = a.smat + ((size_t)b * C + c0 + w * 4 + cc) * 1024 + r * 32 + 8 * h;
#pragma unroll
        for (int kb = 0; kb < 2; ++kb) {
            const float4 lo = *reinterpret_cast<const float4*>(sm + kb * 16);
            const float4 hi = *reinterpret_cast<const float4*>(sm + kb * 16 + 4);
            sa[cc][kb] = make_uint4(pack2(lo.x, lo.y), pack2(lo.z, lo.w), pack2(hi.x, hi.y), pack2(hi.z, hi.w));
        }
    }
    // staging item: 8-tensor block ub, time row tt, 8-channel group q
    const int sub = tid >> 6, stt = (tid >> 1) & 31, sq = tid & 1;
    const size_t rowoff = (size_t)b * a.T * C + c0 + sq * 8;
    for (int t0 = tbeg; t0 < tbeg + tlen; t0 += 32) {
        uint4 in[8], out[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const int u = sub * 8 + k;
            in[k] = u < a.nu ? *reinterpret_cast<const uint4*>(act + (size_t)a.uid[u] * a.tstride + rowoff +
                                                               (size_t)(t0 + stt) * C)
                             : make_uint4(0, 0, 0, 0);
        }
        transpose8(in, out);
        __syncthreads();
#pragma unroll
        for (int j = 0; j < 8; ++j)
            *reinterpret_cast<uint4*>(&Ib[((sq * 8 + j) * 32 + stt) * GIS + sub * 8]) = out[j];
        __syncthreads();
#pragma unroll
        for (int cc = 0; cc < 4; ++cc) {
            const int c = w * 4 + cc;
            f32x16 acc;
            for (int i = 0; i < 16; ++i) acc[i] = 0.f;
#pragma unroll
            for (int kb = 0; kb < 2; ++kb) {
                const uint4 f = *reinterpret_cast<const uint4*>(&Ib[(c * 32 + r) * GIS + kb * 16 + 8 * h]);
                acc = mfma_bf16(sa[cc][kb], f, acc);
            }
            // rows u = 8g + 4h + (0..3) of column t = r; this wave alone owns channel c
#pragma unroll
            for (int g = 0; g < 4; ++g)
                *reinterpret_cast<uint2*>(&Ib[(c * 32 + r) * GIS + 8 * g + 4 * h]) =
                    make_uint2(pack2(acc[4 * g], acc[4 * g + 1]), pack2(acc[4 * g + 2], acc[4 * g + 3]));
        }
        __syncthreads();
#pragma unroll
        for (int j = 0; j < 8; ++j)
            in[j] = *reinterpret_cast<const uint4*>(&Ib[((sq * 8 + j) * 32 + stt) * GIS + sub * 8]);
        transpose8(in, out);      // out[k]: tensor sub*8+k, channels c0+8q..+8
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const int u = sub * 8 + k;
            if (u >= a.nu) continue;
            uint4 v = out[k];
            const u16* cgp = (const u16*)a.cg[u];
            const size_t o = rowoff + (size_t)(t0 + stt) * C;
            if (cgp) {
                const uint4 g = *reinterpret_cast<const uint4*>(cgp + o);
                v.x = pack2(bflo(v.x) + bflo(g.x), bfhi(v.x) + bfhi(g.x));
                v.y = pack2(bflo(v.y) + bflo(g.y), bfhi(v.y) + bfhi(g.y));
                v.z = pack2(bflo(v.z) + bflo(g.z), bfhi(v.z) + bfhi(g.z));
                v.w = pack2(bflo(v.w) + bflo(g.w), bfhi(v.w) + bfhi(g.w));
            }
            *reinterpret_cast<uint4*>(actw + (size_t)a.uid[u] * a.tstride + o) = v;
        }
    }
}

void launch_gram_fwd_bf16(const GramArgs& a, hipStream_t s) {
    hipLaunchKernelGGL(k_gram_fwd_bf16, dim3(a.B * a.nchunk * (C / GCG)), dim3(256), 0, s, a);
}
void launch_gram_bwd_bf16(const GramArgs& a, hipStream_t s) {
    hipLaunchKernelGGL(k_gram_bwd_bf16, dim3(a.B * a.nchunk * (C / GCG)), dim3(256), 0, s, a);
}

}  // namespace ast
