// Gatys Gram (--gatys, methods.py:70-72): per style slot l, G_l = E_l^T E_l over time, a
// [C][C] = 128 x 128 channel Gram; l2-normalised per matrix (methods.py:74), no nb_channels
// truncation (methods.py:75 applies to "ours" only).  Gradient: S~_u = sum_{l -> u} dG_l +
// dG_l^T folded onto unique tensors, D_u = E_u S~_u (+ content grad), in place over E_u.
//
//   fwd  one workgroup per (clip, tensor, time chunk); 4 waves each own a 2x2 block of 32x32
//        output tiles; time tiles stream HBM -> LDS with global_load_lds (no VGPR staging),
//        double-buffered.  bf16: the LDS image is row-major [t][c] (256-B rows, 16-B chunks
//        XOR-swizzled by (row & 3) << 2 through the per-lane SOURCE address) and the MFMA
//        operands, which need 8 consecutive time steps of one channel, come out of
//        ds_read_b64_tr_b16 (hardware transpose, 2 reads per 32x32x16 fragment).
//   bwd  D^T = S~ E^T: A = S~ (LDS, symmetric), B = E rows straight from HBM (each lane reads
//        contiguous 16-B pieces of its own time row; the K order is permuted identically on
//        both operands so a lane's 8 k-steps walk one 128-B half row), C lands as 4
//        consecutive channels per lane -> 8-B (bf16) / 16-B (fp32) stores of the same rows.
#include "common.h"
#include <type_traits>
#include <cstdlib>

namespace ast {

typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef short s16x8 __attribute__((ext_vector_type(8)));
#define LDS_AS __attribute__((address_space(3)))

constexpr int GYB = 64;   // bf16 fwd: time rows per stage (16 KB)
constexpr int GYF = 32;   // fp32 fwd: time rows per stage (16 KB)
constexpr int SBS = 136;  // bwd bf16 S~ LDS row stride (272 B: ds_read_b128 conflict-free)
constexpr int SFS = 129;  // bwd fp32 S~ LDS row stride (odd: ds_read_b32 conflict-free)

__device__ __forceinline__ void glds16(const void* g, void* lds_wave_base) {
    __builtin_amdgcn_global_load_lds(g, (LDS_AS void*)lds_wave_base, 16, 0, 0);
}

__device__ __forceinline__ f32x16 mfma_f32(float a, float b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ void gatys_decode(const GatysArgs& a, int& b, int& u, int& ch) {
    int bid = blockIdx.x;
    ch = bid % a.nchunk; bid /= a.nchunk;
    u = bid % a.nu;
    b = bid / a.nu;
}

__device__ __forceinline__ void store_gpart(const GatysArgs& a, int b, int u, int ch,
                                            const f32x16 (&acc)[2][2], int w, int lane) {
    float* G = a.gpart + (((size_t)b * a.nchunk + ch) * a.nu + u) * (C * C);
    const int h = lane >> 5, col = lane & 31;
#pragma unroll
    for (int ii = 0; ii < 2; ++ii)
#pragma unroll
        for (int jj = 0; jj < 2; ++jj) {
            const int I = 2 * (w >> 1) + ii, J = 2 * (w & 1) + jj;
#pragma unroll
            for (int q = 0; q < 16; ++q) {
                const int row = 32 * I + (q & 3) + 8 * (q >> 2) + 4 * h;
                G[row * C + 32 * J + col] = acc[ii][jj][q];
            }
        }
}

__global__ void __launch_bounds__(256) k_gatys_fwd_bf16(GatysArgs a) {
    __shared__ __attribute__((aligned(1024))) u16 Ls[2][GYB * C];
    int b, u, ch;
    gatys_decode(a, b, u, ch);
    const int tlen = a.T / a.nchunk;
    const int nt = tlen / GYB;
    const u16* E = (const u16*)a.act + (size_t)a.uid[u] * a.tstride +
                   ((size_t)b * a.T + (size_t)ch * tlen) * C;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    // staging: wave w, instruction j fills rows (4w + j) * 4 + lane / 16, physical chunk lane % 16
    int srcoff[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int r = (4 * w + j) * 4 + (lane >> 4), p = lane & 15;
        srcoff[j] = r * C + ((p ^ ((r & 3) << 2)) * 8);
    }
    auto load = [&](int k, int buf) {
        const u16* src = E + (size_t)k * GYB * C;
#pragma unroll
        for (int j = 0; j < 4; ++j) glds16(src + srcoff[j], &Ls[buf][(4 * w + j) * 512]);
    };
    // transposed-read addresses (elements): row 8*kg + q (+16 s + 4 r), swizzled column
    const int kg = lane >> 5, g16 = (lane >> 4) & 1, q = (lane >> 2) & 3, p = lane & 3;
    int aoff[2], boff[2];
#pragma unroll
    for (int t = 0; t < 2; ++t) {
        const int I = 2 * (w >> 1) + t, J = 2 * (w & 1) + t;
        aoff[t] = (8 * kg + q) * C + (((4 * I + 2 * g16 + (p >> 1)) ^ (q << 2)) * 8) + (p & 1) * 4;
        boff[t] = (8 * kg + q) * C + (((4 * J + 2 * g16 + (p >> 1)) ^ (q << 2)) * 8) + (p & 1) * 4;
    }
    f32x16 acc[2][2];
#pragma unroll
    for (int ii = 0; ii < 2; ++ii)
#pragma unroll
        for (int jj = 0; jj < 2; ++jj)
            for (int e = 0; e < 16; ++e) acc[ii][jj][e] = 0.f;
    load(0, 0);
    for (int k = 0; k < nt; ++k) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (k + 1 < nt) load(k + 1, (k + 1) & 1);
        const u16* Lb = Ls[k & 1];
#pragma unroll
        for (int s = 0; s < GYB / 16; ++s) {
            s16x8 fa[2], fb[2];
#pragma unroll
            for (int t = 0; t < 2; ++t) {
                const s16x4 a0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                    (LDS_AS s16x4*)(Lb + aoff[t] + (16 * s) * C));
                const s16x4 a1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                    (LDS_AS s16x4*)(Lb + aoff[t] + (16 * s + 4) * C));
                const s16x4 b0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                    (LDS_AS s16x4*)(Lb + boff[t] + (16 * s) * C));
                const s16x4 b1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                    (LDS_AS s16x4*)(Lb + boff[t] + (16 * s + 4) * C));
                fa[t] = __builtin_shufflevector(a0, a1, 0, 1, 2, 3, 4, 5, 6, 7);
                fb[t] = __builtin_shufflevector(b0, b1, 0, 1, 2, 3, 4, 5, 6, 7);
            }
#pragma unroll
            for (int ii = 0; ii < 2; ++ii)
#pragma unroll
                for (int jj = 0; jj < 2; ++jj)
                    acc[ii][jj] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(
                        __builtin_bit_cast(bf16x8, fa[ii]), __builtin_bit_cast(bf16x8, fb[jj]),
                        acc[ii][jj], 0, 0, 0);
        }
    }
    store_gpart(a, b, u, ch, acc, w, lane);
}

__global__ void __launch_bounds__(256) k_gatys_fwd_f32(GatysArgs a) {
    __shared__ __attribute__((aligned(1024))) float Ls[2][GYF * C];
    int b, u, ch;
    gatys_decode(a, b, u, ch);
    const int tlen = a.T / a.nchunk;
    const int nt = tlen / GYF;
    const float* E = (const float*)a.act + (size_t)a.uid[u] * a.tstride +
                     ((size_t)b * a.T + (size_t)ch * tlen) * C;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    auto load = [&](int k, int buf) {
        // wave w, instruction j fills rows (4w + j) * 2 + lane / 32 (1 KiB, lane-linear)
        const float* src = E + (size_t)k * GYF * C + lane * 4;
#pragma unroll
        for (int j = 0; j < 4; ++j) glds16(src + (4 * w + j) * 256, &Ls[buf][(4 * w + j) * 256]);
    };
    const int r = lane & 31, kk = lane >> 5;
    const int I0 = 2 * (w >> 1), J0 = 2 * (w & 1);
    f32x16 acc[2][2];
#pragma unroll
    for (int ii = 0; ii < 2; ++ii)
#pragma unroll
        for (int jj = 0; jj < 2; ++jj)
            for (int e = 0; e < 16; ++e) acc[ii][jj][e] = 0.f;
    load(0, 0);
    for (int k = 0; k < nt; ++k) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (k + 1 < nt) load(k + 1, (k + 1) & 1);
        const float* Lb = Ls[k & 1] + kk * C + r;
#pragma unroll 4
        for (int s = 0; s < GYF / 2; ++s) {
            const float* row = Lb + 2 * s * C;
            const float a0 = row[32 * I0], a1 = row[32 * I0 + 32];
            const float b0 = row[32 * J0], b1 = row[32 * J0 + 32];
            acc[0][0] = mfma_f32(a0, b0, acc[0][0]);
            acc[0][1] = mfma_f32(a0, b1, acc[0][1]);
            acc[1][0] = mfma_f32(a1, b0, acc[1][0]);
            acc[1][1] = mfma_f32(a1, b1, acc[1][1]);
        }
    }
    store_gpart(a, b, u, ch, acc, w, lane);
}

// ---------------------------------------------------------------------------------------
// backward: D_u[t][:] = E_u[t][:] S~_u (+ cg_u[t][:]), in place over E_u

__global__ void __launch_bounds__(256) k_gatys_bwd_bf16(GatysArgs a) {
    __shared__ __attribute__((aligned(16))) u16 Sb[C * SBS];
    const int tilesPer = a.T / GY_ROWS;
    int bid = blockIdx.x;
    const int tile = bid % tilesPer; bid /= tilesPer;
    const int u = bid % a.nu, b = bid / a.nu;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const u16* S = a.smatb + ((size_t)b * a.nu + u) * (C * C);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        const int i = tid + 256 * k, row = i >> 4, c16 = i & 15;
        *reinterpret_cast<uint4*>(&Sb[row * SBS + c16 * 8]) =
            *reinterpret_cast<const uint4*>(S + row * C + c16 * 8);
    }
    const u16* E = (const u16*)a.act + (size_t)a.uid[u] * a.tstride + (size_t)b * a.T * C;
    u16* Ew = (u16*)a.actw + (size_t)a.uid[u] * a.tstride + (size_t)b * a.T * C;   // D (in place unless out of place)
    const u16* CG = (const u16*)a.cg[u];
    if (CG) CG += (size_t)b * a.T * C;
    const int j = lane & 31, kg = lane >> 5;
    const int rows_w = GY_ROWS / 4;
    const int t0 = tile * GY_ROWS + w * rows_w;
    auto loadB = [&](int t, uint4 (&bb)[8]) {
        const uint4* src = reinterpret_cast<const uint4*>(E + (size_t)(t + j) * C + kg * 64);
#pragma unroll
        for (int s = 0; s < 8; ++s) bb[s] = src[s];
    };
    uint4 bcur[8], bnxt[8];
    loadB(t0, bcur);
    __syncthreads();
    const u16* Ab = Sb + j * SBS + kg * 64;
    for (int n = 0; n < rows_w / 32; ++n) {
        const int t = t0 + 32 * n;
        if (n + 1 < rows_w / 32) loadB(t + 32, bnxt);
        f32x16 acc[4];
#pragma unroll
        for (int m = 0; m < 4; ++m)
            for (int e = 0; e < 16; ++e) acc[m][e] = 0.f;
#pragma unroll
        for (int s = 0; s < 8; ++s)
#pragma unroll
            for (int m = 0; m < 4; ++m)
                acc[m] = mfma_bf16(*reinterpret_cast<const uint4*>(Ab + 32 * m * SBS + 8 * s),
                                   bcur[s], acc[m]);
        // lane holds time t + j, channels 32m + 8g + 4kg + 0..3 in acc[m][4g..4g+3]
        u16* out = Ew + (size_t)(t + j) * C + 4 * kg;
        const u16* cgr = CG ? CG + (size_t)(t + j) * C + 4 * kg : nullptr;
#pragma unroll
        for (int m = 0; m < 4; ++m)
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const int c = 32 * m + 8 * g;
                float v0 = acc[m][4 * g], v1 = acc[m][4 * g + 1], v2 = acc[m][4 * g + 2],
                      v3 = acc[m][4 * g + 3];
                if (cgr) {
                    const uint2 cv = *reinterpret_cast<const uint2*>(cgr + c);
                    v0 += bflo(cv.x); v1 += bfhi(cv.x); v2 += bflo(cv.y); v3 += bfhi(cv.y);
                }
                *reinterpret_cast<uint2*>(out + c) = make_uint2(pack2(v0, v1), pack2(v2, v3));
            }
        if (n + 1 < rows_w / 32) {
#pragma unroll
            for (int s = 0; s < 8; ++s) bcur[s] = bnxt[s];
        }
    }
}

__global__ void __launch_bounds__(256) k_gatys_bwd_f32(GatysArgs a) {
    __shared__ float Sf[C * SFS];
    const int tilesPer = a.T / GY_ROWS;
    int bid = blockIdx.x;
    const int tile = bid % tilesPer; bid /= tilesPer;
    const int u = bid % a.nu, b = bid / a.nu;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const float* S = a.smat + ((size_t)b * a.nu + u) * (C * C);
    for (int i = tid; i < C * C; i += 256) Sf[(i >> 7) * SFS + (i & 127)] = S[i];
    __syncthreads();
    const float* E = (const float*)a.act + (size_t)a.uid[u] * a.tstride + (size_t)b * a.T * C;
    float* Ew = (float*)a.actw + (size_t)a.uid[u] * a.tstride + (size_t)b * a.T * C;   // D (in place unless out of place)
    const float* CG = (const float*)a.cg[u];
    if (CG) CG += (size_t)b * a.T * C;
    const int j = lane & 31, kg = lane >> 5;
    const int rows_w = GY_ROWS / 4;
    const int t0 = tile * GY_ROWS + w * rows_w;
    const float* Ab = Sf + j * SFS + kg * 64;
    for (int n = 0; n < rows_w / 32; ++n) {
        const int t = t0 + 32 * n;
        float bf[64];
        const float4* src = reinterpret_cast<const float4*>(E + (size_t)(t + j) * C + kg * 64);
#pragma unroll
        for (int s = 0; s < 16; ++s) {
            const float4 v = src[s];
            bf[4 * s] = v.x; bf[4 * s + 1] = v.y; bf[4 * s + 2] = v.z; bf[4 * s + 3] = v.w;
        }
        f32x16 acc[4];
#pragma unroll
        for (int m = 0; m < 4; ++m)
            for (int e = 0; e < 16; ++e) acc[m][e] = 0.f;
#pragma unroll
        for (int s = 0; s < 64; ++s)
#pragma unroll
            for (int m = 0; m < 4; ++m) acc[m] = mfma_f32(Ab[32 * m * SFS + s], bf[s], acc[m]);
        float* out = Ew + (size_t)(t + j) * C + 4 * kg;
        const float* cgr = CG ? CG + (size_t)(t + j) * C + 4 * kg : nullptr;
#pragma unroll
        for (int m = 0; m < 4; ++m)
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const int c = 32 * m + 8 * g;
                float4 v = make_float4(acc[m][4 * g], acc[m][4 * g + 1], acc[m][4 * g + 2],
                                       acc[m][4 * g + 3]);
                if (cgr) {
                    const float4 cv = *reinterpret_cast<const float4*>(cgr + c);
                    v.x += cv.x; v.y += cv.y; v.z += cv.z; v.w += cv.w;
                }
                *reinterpret_cast<float4*>(out + c) = v;
            }
    }
}

// ---------------------------------------------------------------------------------------
// split mode (precision 2): fp32 activations, bf16 MFMA on two-term operands x = xh + xl
// (xh = bf16(x), xl = bf16(x - xh)), products hi.hi + hi.lo + lo.hi, fp32 accumulation (the
// ours-Gram's scheme, gram_split.hip).  fwd: fp32 rows -> registers one stage ahead -> split
// into the two swizzled bf16 images of k_gatys_fwd_bf16 -> the same transposed fragment reads,
// three MFMAs per tile and k-step.  bwd: S~ split into two LDS images, E rows split per lane.

__device__ __forceinline__ void split2g(float x0, float x1, uint32_t& hi, uint32_t& lo) {
    hi = pack2(x0, x1);
    lo = pack2(x0 - bflo(hi), x1 - bfhi(hi));
}

// one 32x32 tile (I, J) of G (rows 32 I + (q & 3) + 8 (q >> 2) + 4 h, column 32 J + (lane & 31)),
// and for an off-diagonal tile of the symmetric G its mirror (J, I): four 16-B stores per lane
__device__ __forceinline__ void store_tile(float* G, int I, int J, const f32x16& acc, int lane) {
    const int h = lane >> 5, col = lane & 31;
#pragma unroll
    for (int q = 0; q < 16; ++q) G[(32 * I + (q & 3) + 8 * (q >> 2) + 4 * h) * C + 32 * J + col] = acc[q];
    if (I != J) {
#pragma unroll
        for (int g = 0; g < 4; ++g)
            *reinterpret_cast<float4*>(&G[(32 * J + col) * C + 32 * I + 8 * g + 4 * h]) =
                make_float4(acc[4 * g], acc[4 * g + 1], acc[4 * g + 2], acc[4 * g + 3]);
    }
}

// G = E^T E is symmetric: the 10 upper 32x32 tiles of the 4x4 grid are computed (waves 0 / 1:
// the diagonal pairs {0, 1} / {2, 3} as (X0, X0), (X0, X1), (X1, X1); waves 2 / 3: block w - 2
// against blocks 2 and 3) and the 6 off-diagonal ones are written twice: 30 instead of 48 MFMAs
// per 16-row k-step and workgroup
template <int NST>   // load stages in flight (2: 64 KiB per workgroup, 3: 96 KiB)
__global__ void __launch_bounds__(256) k_gatys_fwd_s(GatysArgs a) {
    __shared__ __attribute__((aligned(1024))) u16 Lh[GYB * C];   // [t][c] bf16 hi, swizzled
    __shared__ __attribute__((aligned(1024))) u16 Ll[GYB * C];   // lo
    int b, u, ch;
    gatys_decode(a, b, u, ch);
    const int tlen = a.T / a.nchunk;
    const int nt = tlen / GYB;
    const float* E = (const float*)a.act + (size_t)a.uid[u] * a.tstride +
                     ((size_t)b * a.T + (size_t)ch * tlen) * C;
    const int tid = threadIdx.x, lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    // staging: float4 f = tid + 256 k: row (tid >> 5) + 8 k, channels 4 (tid & 31) .. + 3
    const int c4 = tid & 31, r0 = tid >> 5;
    // NST stages of loads in flight (a ring of register sets)
    float4 vr[NST][8];
    // unconditional loads (past the chunk a stage re-reads its last block, an L2 hit) and whole
    // rings in the loop: a conditional load made the compiler copy the ring registers behind
    // vmcnt(0) waits, so nothing stayed in flight across a stage (the ours-Gram forward's fix)
    auto load = [&](float4 (&v)[8], int k) {
        const float* src = E + (size_t)min(k, nt - 1) * GYB * C + (size_t)r0 * C + 4 * c4;
#pragma unroll
        for (int q = 0; q < 8; ++q) v[q] = *reinterpret_cast<const float4*>(src + (size_t)(8 * q) * C);
    };
    // image element offset of (row r, channels 4 c4 ..): 16-B chunk (c4 >> 1) swizzled by
    // ((r & 3) << 2), half (c4 & 1)
    auto img = [&](int r) { return r * C + (((c4 >> 1) ^ ((r & 3) << 2)) * 8) + (c4 & 1) * 4; };
    const int kg = lane >> 5, g16 = (lane >> 4) & 1, q = (lane >> 2) & 3, p = lane & 3;
    // fragment offset of channel block X (A and B fragments of G = E^T E coincide)
    auto boff = [&](int X) { return (8 * kg + q) * C + (((4 * X + 2 * g16 + (p >> 1)) ^ (q << 2)) * 8) + (p & 1) * 4; };
    const bool diag = w < 2;
    const int X0 = diag ? 2 * w : w - 2;     // diagonal waves: blocks X0, X0 + 1; others: A = X0
    const int o0 = boff(X0), o1 = boff(diag ? X0 + 1 : 2), o2 = boff(3);
    f32x16 acc[3];
#pragma unroll
    for (int i = 0; i < 3; ++i)
        for (int e = 0; e < 16; ++e) acc[i][e] = 0.f;
    auto frag = [&](const u16* L, int off, int s) {
        const s16x4 x0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_AS s16x4*)(L + off + (16 * s) * C));
        const s16x4 x1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_AS s16x4*)(L + off + (16 * s + 4) * C));
        return __builtin_bit_cast(bf16x8, __builtin_shufflevector(x0, x1, 0, 1, 2, 3, 4, 5, 6, 7));
    };
    auto mm3 = [&](f32x16& c, const bf16x8& ah, const bf16x8& al, const bf16x8& bh, const bf16x8& bl) {
        c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bh, c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bl, c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al, bh, c, 0, 0, 0);
    };
    // the diagonal / off-diagonal waves run separate copies of the loop (DIAG a constant in
    // each), so the accumulators keep their registers across iterations.
    // Barrier invariant: waves 0-1 and 2-3 reach different s_barrier instructions,
    // which is sound because s_barrier counts waves, not instruction addresses, and both copies
    // execute the same number of barriers: `diag` is wave-uniform (w is readfirstlane'd), every
    // wave runs exactly one copy, and in both copies the trip counts (nring, the NST - 1
    // remainder stages) depend on nt and NST only, with exactly two __syncthreads per stage
    // and none elsewhere.  Any change that gives DIAG its own barrier or trip count breaks this.
    auto run = [&](auto diag_tag) {
        constexpr bool DIAG = decltype(diag_tag)::value;
        auto stage = [&](float4 (&v)[8], int k) {
            __syncthreads();   // the previous stage's fragment reads are done
#pragma unroll
            for (int qq = 0; qq < 8; ++qq) {
                const int r = r0 + 8 * qq;
                uint32_t h0, l0, h1, l1;
                split2g(v[qq].x, v[qq].y, h0, l0);
                split2g(v[qq].z, v[qq].w, h1, l1);
                *reinterpret_cast<uint2*>(&Lh[img(r)]) = make_uint2(h0, h1);
                *reinterpret_cast<uint2*>(&Ll[img(r)]) = make_uint2(l0, l1);
            }
            load(v, k + NST);   // NST stages ahead
            __syncthreads();
#pragma unroll
            for (int s = 0; s < GYB / 16; ++s) {
                const bf16x8 h0 = frag(Lh, o0, s), l0 = frag(Ll, o0, s);
                const bf16x8 h1 = frag(Lh, o1, s), l1 = frag(Ll, o1, s);
                if (DIAG) {
                    mm3(acc[0], h0, l0, h0, l0);     // (X0, X0)
                    mm3(acc[1], h0, l0, h1, l1);     // (X0, X0 + 1)
                    mm3(acc[2], h1, l1, h1, l1);     // (X0 + 1, X0 + 1)
                } else {
                    const bf16x8 h2 = frag(Lh, o2, s), l2 = frag(Ll, o2, s);
                    mm3(acc[0], h0, l0, h1, l1);     // (X0, 2)
                    mm3(acc[1], h0, l0, h2, l2);     // (X0, 3)
                }
            }
        };
#pragma unroll
        for (int q = 0; q < NST; ++q) load(vr[q], q);
        const int nring = nt / NST;
        int k = 0;
        for (int i = 0; i < nring; ++i, k += NST) {
#pragma unroll
            for (int q = 0; q < NST; ++q) stage(vr[q], k + q);
        }
#pragma unroll
        for (int q = 0; q < NST - 1; ++q)
            if (q < nt - nring * NST) stage(vr[q], k + q);
    };
    if (diag) run(std::true_type{});
    else run(std::false_type{});
    float* G = a.gpart + (((size_t)b * a.nchunk + ch) * a.nu + u) * (C * C);
    if (diag) {
        store_tile(G, X0, X0, acc[0], lane);
        store_tile(G, X0, X0 + 1, acc[1], lane);
        store_tile(G, X0 + 1, X0 + 1, acc[2], lane);
    } else {
        store_tile(G, X0, 2, acc[0], lane);
        store_tile(G, X0, 3, acc[1], lane);
    }
}

// Split Gatys backward (round 4): v_mfma_f32_16x16x32_bf16 over 16-row blocks, so a lane's E
// operand is 8 floats per k-step (32 registers a block) and three blocks stay in flight (192 KiB
// per CU at two workgroups); round 3's 32x32x16 form (64 floats per lane, one block ahead at one
// wave per SIMD) measured 28.2 against 23.9 ms per call and was removed.  Per wave: rows t0 .. t0 + 127 in 8 blocks;
// A = S~ (symmetric: S~[c][k] = S~[k][c]) split fragments from the LDS image, row c = 16 m + (l & 15),
// k = 32 s + 8 (l >> 4) .. + 7; B = E split from registers, lane (n = l & 15, q = l >> 4): row
// t + n, channels 32 s + 8 q .. + 7; D lane: row t + n, channels 16 m + 4 q .. + 3 (a float4).
// Fused content tap (a.cont_u == u, methods.py:116-117): the lane re-reads its output float4 of
// E (in L2: the workgroup streamed the row one block earlier) and phi, adds coef (E - phi) on
// channels < cont_ncol, and the workgroup's squared errors go to slot `tile` of the clip's
// content partials -- k_content's 2 GiB gradient buffer, written and read back, is gone.
typedef float f32x4g __attribute__((ext_vector_type(4)));
constexpr int GB2 = 3;   // blocks in flight
__global__ void __launch_bounds__(256) k_gatys_bwd_s2(GatysArgs a) {
    __shared__ __attribute__((aligned(16))) u16 Sh[C * SBS];   // S~ hi
    __shared__ __attribute__((aligned(16))) u16 Sl[C * SBS];   // S~ lo
    const int tilesPer = a.T / GY_ROWS;
    int bid = blockIdx.x;
    const int tile = bid % tilesPer; bid /= tilesPer;
    const int u = bid % a.nu, b = bid / a.nu;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const float* S = a.smat + ((size_t)b * a.nu + u) * (C * C);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        const int i = tid + 256 * k, row = i >> 4, c8 = i & 15;   // 8 values per piece
        const float4 x0 = *reinterpret_cast<const float4*>(S + row * C + c8 * 8);
        const float4 x1 = *reinterpret_cast<const float4*>(S + row * C + c8 * 8 + 4);
        uint32_t h[4], l[4];
        split2g(x0.x, x0.y, h[0], l[0]);
        split2g(x0.z, x0.w, h[1], l[1]);
        split2g(x1.x, x1.y, h[2], l[2]);
        split2g(x1.z, x1.w, h[3], l[3]);
        *reinterpret_cast<uint4*>(&Sh[row * SBS + c8 * 8]) = make_uint4(h[0], h[1], h[2], h[3]);
        *reinterpret_cast<uint4*>(&Sl[row * SBS + c8 * 8]) = make_uint4(l[0], l[1], l[2], l[3]);
    }
    const float* E = (const float*)a.act + (size_t)a.uid[u] * a.tstride + (size_t)b * a.T * C;
    float* Ew = (float*)a.actw + (size_t)a.uid[u] * a.tstride + (size_t)b * a.T * C;   // D (in place unless out of place)
    const float* CG = (const float*)a.cg[u];
    if (CG) CG += (size_t)b * a.T * C;
    const bool cont = u == a.cont_u;   // (workgroup-uniform)
    const bool top = u == a.top_u;
    float omax = 0.f;
    const float* PH = cont ? a.cont_phi + (size_t)b * a.cont_phi_bstride + a.cont_off : nullptr;
    float csd = 0.f;
    const int n = lane & 15, q = lane >> 4;
    const int nblk = GY_ROWS / 4 / 16;
    const int t0 = tile * GY_ROWS + w * (GY_ROWS / 4);
    float4 vr[GB2][8];   // block in flight: k-step s, halves 0 / 1 at [2 s + hf]
    auto load = [&](float4 (&v)[8], int blk) {
        const float* src = E + (size_t)(t0 + 16 * blk + n) * C + 8 * q;
#pragma unroll
        for (int k = 0; k < 8; ++k) v[k] = *reinterpret_cast<const float4*>(src + 32 * (k >> 1) + 4 * (k & 1));
    };
    __syncthreads();
    auto block = [&](float4 (&v)[8], int blk) {
        asm volatile("" ::: "memory");   // S~ fragments are re-read from LDS per block, not hoisted
        uint4 bh[4], bl[4];
#pragma unroll
        for (int s2 = 0; s2 < 4; ++s2) {
            uint32_t h[4], l[4];
            split2g(v[2 * s2].x, v[2 * s2].y, h[0], l[0]);
            split2g(v[2 * s2].z, v[2 * s2].w, h[1], l[1]);
            split2g(v[2 * s2 + 1].x, v[2 * s2 + 1].y, h[2], l[2]);
            split2g(v[2 * s2 + 1].z, v[2 * s2 + 1].w, h[3], l[3]);
            bh[s2] = make_uint4(h[0], h[1], h[2], h[3]);
            bl[s2] = make_uint4(l[0], l[1], l[2], l[3]);
        }
        if (blk + GB2 < nblk) load(v, blk + GB2);
        const int t = t0 + 16 * blk + n;
        float* out = Ew + (size_t)t * C + 4 * q;
        const float* cgr = CG ? CG + (size_t)t * C + 4 * q : nullptr;
#pragma unroll
        for (int m = 0; m < 8; ++m) {
            f32x4g c = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int s2 = 0; s2 < 4; ++s2) {
                const int o = (16 * m + n) * SBS + 32 * s2 + 8 * q;
                const uint4 ah = *reinterpret_cast<const uint4*>(&Sh[o]);
                const uint4 al = *reinterpret_cast<const uint4*>(&Sl[o]);
                c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, ah), __builtin_bit_cast(bf16x8, bh[s2]), c, 0, 0, 0);
                c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, ah), __builtin_bit_cast(bf16x8, bl[s2]), c, 0, 0, 0);
                c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, al), __builtin_bit_cast(bf16x8, bh[s2]), c, 0, 0, 0);
            }
            float4 o4 = make_float4(c[0], c[1], c[2], c[3]);
            if (cgr) {
                const float4 cv = *reinterpret_cast<const float4*>(cgr + 16 * m);
                o4.x += cv.x; o4.y += cv.y; o4.z += cv.z; o4.w += cv.w;
            }
            if (cont) {
                const int cc = 16 * m + 4 * q;
                if (cc < a.cont_ncol) {   // (phi rows hold cont_ncol channels: quads past them load nothing)
                    const float4 ev = *reinterpret_cast<const float4*>(E + (size_t)t * C + cc);
                    const float4 pv = *reinterpret_cast<const float4*>(PH + (size_t)t * a.cont_ncc + cc);
                    const float d[4] = {ev.x - pv.x, ev.y - pv.y, ev.z - pv.z, ev.w - pv.w};
                    float dd[4];
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        dd[i] = cc + i < a.cont_ncol ? d[i] : 0.f;
                        csd = fmaf(dd[i], dd[i], csd);
                    }
                    o4.x = fmaf(a.cont_coef, dd[0], o4.x); o4.y = fmaf(a.cont_coef, dd[1], o4.y);
                    o4.z = fmaf(a.cont_coef, dd[2], o4.z); o4.w = fmaf(a.cont_coef, dd[3], o4.w);
                }
            }
            *reinterpret_cast<float4*>(out + 16 * m) = o4;
            if (top) omax = fmaxf(omax, fmaxf(fmaxf(fabsf(o4.x), fabsf(o4.y)), fmaxf(fabsf(o4.z), fabsf(o4.w))));
        }
    };
#pragma unroll
    for (int k = 0; k < GB2; ++k)
        if (k < nblk) load(vr[k], k);
    for (int blk = 0; blk < nblk; blk += GB2) {
#pragma unroll
        for (int k = 0; k < GB2; ++k)
            if (blk + k < nblk) block(vr[k], blk + k);
    }
    if (top) {    // the top tensor's max |D| per clip: one atomic per workgroup (no k_absmax pass)
        __shared__ float mw[4];
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) omax = fmaxf(omax, __shfl_xor(omax, off));
        if (lane == 0) mw[w] = omax;
        __syncthreads();
        if (tid == 0) atomicMax(gslot(a.gmax_top, b, blockIdx.x), __float_as_uint(fmaxf(fmaxf(mw[0], mw[1]), fmaxf(mw[2], mw[3]))));
    }
    if (cont) {   // the workgroup's squared content error -> slot `tile` (fixed order: waves 0..3)
        __shared__ float cw[4];
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) csd += __shfl_xor(csd, off);
        if (lane == 0) cw[w] = csd;
        __syncthreads();
        if (tid == 0) a.cont_part[(size_t)b * a.cont_pstride + tile] = ((cw[0] + cw[1]) + cw[2]) + cw[3];
    }
}

// ---------------------------------------------------------------------------------------
// style loss: one workgroup per (clip, unique tensor); l2-normalise (methods.py:74), loss vs
// phi (methods.py:118-119), d/dG through the normalisation, S~ = sum dG + dG^T.

__device__ __forceinline__ float block_sum(float v, float* red) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
    __syncthreads();
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
    __syncthreads();
    return red[0] + red[1] + red[2] + red[3];
}

__global__ void __launch_bounds__(256) k_style_gatys(GatysStyleArgs a) {
    __shared__ float Tt[C * SFS];
    __shared__ float red[4];
    const int u = blockIdx.x % a.nu, b = blockIdx.x / a.nu;
    const int tid = threadIdx.x;
    constexpr int NE = C * C / 256;   // 64 elements per thread: e = tid + 256 k
    float g[NE];
#pragma unroll
    for (int k = 0; k < NE; ++k) g[k] = 0.f;
    for (int ch = 0; ch < a.nchunk; ++ch) {
        const float* src = a.gpart + (((size_t)b * a.nchunk + ch) * a.nu + u) * (C * C);
#pragma unroll
        for (int k = 0; k < NE; ++k) g[k] += src[tid + 256 * k];
    }
    float ss = 0.f;
#pragma unroll
    for (int k = 0; k < NE; ++k) ss = fmaf(g[k], g[k], ss);
    ss = block_sum(ss, red);
    const float inv = 1.0f / sqrtf(fmaxf(ss, 1e-12f));
    const float big = ss >= 1e-12f ? 1.f : 0.f;
    float sacc[NE];
#pragma unroll
    for (int k = 0; k < NE; ++k) sacc[k] = 0.f;
    float sd = 0.f;
    for (int l = 0; l < a.L; ++l) {
        if (a.lmap[l] != u) continue;
        if (a.embs) {
            float* dst = a.embs + ((size_t)b * a.L + l) * (C * C);
#pragma unroll
            for (int k = 0; k < NE; ++k) dst[tid + 256 * k] = g[k] * inv;
        }
        if (!a.phi) continue;
        const float* phi = a.phi + (size_t)b * a.phi_bstride + (size_t)l * (C * C);
        float dgn[NE];
        float dot = 0.f;
#pragma unroll
        for (int k = 0; k < NE; ++k) {
            const float gn = g[k] * inv;
            const float diff = gn - phi[tid + 256 * k];
            sd = fmaf(diff, diff, sd);
            dgn[k] = a.coef * diff;
            dot = fmaf(gn, dgn[k], dot);
        }
        dot = block_sum(dot, red);
#pragma unroll
        for (int k = 0; k < NE; ++k) sacc[k] += dgn[k] * inv - big * (g[k] * inv) * dot * inv;
    }
    if (!a.phi) return;
    sd = block_sum(sd, red);
    if (tid == 0 && a.spart) a.spart[(size_t)b * a.nu + u] = sd;
    // S~ = S + S^T through an LDS image
#pragma unroll
    for (int k = 0; k < NE; ++k) {
        const int e = tid + 256 * k;
        Tt[(e >> 7) * SFS + (e & 127)] = sacc[k];
    }
    __syncthreads();
    float* sm = a.smat ? a.smat + ((size_t)b * a.nu + u) * (C * C) : nullptr;
    u16* smb = a.smatb ? a.smatb + ((size_t)b * a.nu + u) * (C * C) : nullptr;
#pragma unroll
    for (int k = 0; k < NE; ++k) {
        const int e = tid + 256 * k, r = e >> 7, c = e & 127;
        const float v = Tt[r * SFS + c] + Tt[c * SFS + r];
        if (sm) sm[e] = v;
        if (smb) smb[e] = f2bf(v);
    }
}

void launch_gatys_fwd(const GatysArgs& a, int precision, hipStream_t s) {
    const dim3 g(a.B * a.nu * a.nchunk);
    if (precision == 1) hipLaunchKernelGGL(k_gatys_fwd_bf16, g, dim3(256), 0, s, a);
    else if (precision == 2) {   // ASTYLE_GATYS_STAGES=3: three load stages in flight (A/B; default 2)
        const char* e = getenv("ASTYLE_GATYS_STAGES");
        if (e && atoi(e) == 3) hipLaunchKernelGGL(k_gatys_fwd_s<3>, g, dim3(256), 0, s, a);
        else hipLaunchKernelGGL(k_gatys_fwd_s<2>, g, dim3(256), 0, s, a);
    }
    else hipLaunchKernelGGL(k_gatys_fwd_f32, g, dim3(256), 0, s, a);
}
void launch_gatys_bwd(const GatysArgs& a, int precision, hipStream_t s) {
    const dim3 g(a.B * a.nu * (a.T / GY_ROWS));
    if (precision == 1) hipLaunchKernelGGL(k_gatys_bwd_bf16, g, dim3(256), 0, s, a);
    else if (precision == 2) {
        hipLaunchKernelGGL(k_gatys_bwd_s2, g, dim3(256), 0, s, a);
    }
    else hipLaunchKernelGGL(k_gatys_bwd_f32, g, dim3(256), 0, s, a);
}
void launch_style_gatys(const GatysStyleArgs& a, hipStream_t s) {
    hipLaunchKernelGGL(k_style_gatys, dim3(a.B * a.nu), dim3(256), 0, s, a);
}

}  // namespace ast
