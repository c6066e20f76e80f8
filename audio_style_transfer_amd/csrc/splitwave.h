// Shared pieces of the split-fp16 block kernels (precision 2: block_fwd_split.hip,
// block_bwd_split.hip).
//
// Precision 2 keeps every tensor in HBM as fp32 (the reference's storage type) and runs the
// encoder GEMMs on v_mfma_f32_32x32x16_f16 with each fp32 operand split into two fp16 halves:
//   a ~ ah + al,  ah = rtz_f16(a s),  al = rtz_f16(a s - ah)        (22 significant bits)
//   a w ~ ah wh + ah wl + al wh                                       (al wl ~ 2^-22 dropped)
// s is a power of two that puts the largest |a| of the operand just below 2^14 (fp16 range):
// per clip for the tensors a kernel reads (the producer records max |x| per clip with one
// atomic per wave), per tile for what a kernel produces and consumes itself (max exchanged
// between the waves through LDS), per block for the weights (host).  The accumulators are in
// units of the two scales' product; the epilogues multiply them back (exact: powers of two).
// Round-toward-zero for the activation halves keeps sign(al) == sign(ah) (or al == 0), so
// relu of a split pair is the pair of relus.  tools/precision_emulate.py puts the resulting
// gradient at fp32-class error against the fp64 oracle (a bf16 two-term split is 1000x worse).
//
// Kernel shape ("channel-owning" waves): one 256-thread workgroup per CU (one wave per SIMD),
// persistent over tiles of TMS = 64 positions of one layer in time_to_batch order
// (masked.py:57-86).  Wave w owns output channels 32 w .. 32 w + 31 of every tile column: its
// share of the split weights (the A fragments, 256 registers) lives in AGPRs for the whole
// launch, and the activations are the B operand, read by all four waves from one LDS image.
// LDS per workgroup: two fp32 row slots (this tile's rows, the next tile's DMA), one split
// image (the B operand of the first GEMM, then the second GEMM's B operand written by the
// epilogue of the first).
#pragma once
#include "common.h"

namespace ast {
namespace sw {

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

constexpr int FT = 256;                  // threads: one wave per SIMD
constexpr int TMS = 64;                  // positions per tile
constexpr int RS = 528;                  // LDS row stride (bytes): 512 + 16, conflict-free
                                         // column reads (row r starts at bank 4 r)
constexpr int SLOT = 36864;              // bytes per LDS slot: up to 68 rows + DMA tail
constexpr int DPW = 9;                   // one-KiB DMA groups per wave per slot (36 groups)
static_assert(4 * DPW * 1024 == SLOT, "DMA groups tile the slot");
static_assert(68 * RS <= SLOT, "slot holds the largest layout");

struct Layout {            // uniform per launch (pick_layout)
    int M;                 // segment length; TMS = one segment with two halo rows
    int nrows;             // image rows
};

// One segment with halo rows when a tile lies inside one sub-sequence (n % 64 == 0); whole
// sub-sequences of 32 positions with their own zero pad rows (n == 32); otherwise per-column
// tap masks over 64 gathered positions (MASKED, n < 32).
inline bool pick_layout(int n, Layout& ly) {
    if (n % TMS == 0) { ly.M = TMS; ly.nrows = TMS + 2; return false; }
    if (n < TMS && TMS % n == 0 && n >= 32) { ly.M = n; ly.nrows = (TMS / n) * (n + 2); return false; }
    ly.M = TMS; ly.nrows = TMS + 2;
    return true;
}

int num_cus();

__device__ __forceinline__ int frow(int c, const Layout& ly) {   // image row of tile column c
    return (c / ly.M) * (ly.M + 2) + 1 + (c % ly.M);
}

// time offset of image row L from the tile's base time (unmasked layouts):
//   one segment: rows are positions p0-1 .. p0+64 of one sub-sequence, t = tb + (L-1) d
//   segments of M = n: row (s, k) is position k-1 of sub-sequence j0 + s, t = tb + (k-1) d + s
__device__ __forceinline__ int row_toff(int L, const Layout& ly, int d) {
    if (ly.M == TMS) return (L - 1) * d;
    const int s = L / (ly.M + 2), k = L - s * (ly.M + 2);
    return (k - 1) * d + s;
}

struct Tile { int b, p0, tb; };   // clip, first position, base time (unmasked layouts)

template <bool MASKED>
__device__ __forceinline__ Tile tile_at(int tl, int tiles, int n, int d, const Layout& ly) {
    Tile t;
    t.b = tl / tiles;
    t.p0 = (tl - t.b * tiles) * TMS;
    t.tb = MASKED ? 0 : (ly.M == TMS ? (t.p0 % n) * d + t.p0 / n : t.p0 / n);
    return t;
}

// time of tile column cc (toff = row_toff of its image row, unmasked layouts)
template <bool MASKED>
__device__ __forceinline__ int col_time(const Tile& t, int cc, int toff, int n, int d) {
    if (MASKED) {
        const int p = t.p0 + cc;
        return (p % n) * d + p / n;
    }
    return t.tb + toff;
}

__device__ __forceinline__ uint4 lds16(const uint8_t* p) { return *reinterpret_cast<const uint4*>(p); }

// 16 B per lane HBM -> LDS at lds_base + 16 * lane (global_load_lds_dwordx4).  Inline asm so the
// compiler neither counts it nor drains it before unrelated LDS reads; the kernels wait with an
// explicit vmcnt.
__device__ __forceinline__ void dma16(const void* src, uint32_t lds_base) {
    uint32_t keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
                 "global_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(src), "s"(lds_base) : "memory");
}

// One wave's share of a slot: group g = w + 4 j (j < DPW) covers slot bytes [1024 g, +1024);
// this lane's 16 B land at row L, chunk qc (qc == 32 is the row's pad chunk, filled with a
// harmless re-read of chunk 0; rows >= nrows read the zero line).
template <bool MASKED>
struct RowDma {
    int soff[DPW];       // source element offset from the tile's base row (unmasked layouts)
    int scls[DPW];       // source class: 0 row, 1 zero, 2 left halo, 3 right halo
    int srow[DPW], schk[DPW];
    const float* base;   // per tile (aim)
    uint32_t vmask;      // classes with a real source row
    Tile t;

    __device__ __forceinline__ void init(int w, int lane, const Layout& ly, int d) {
#pragma unroll
        for (int j = 0; j < DPW; ++j) {
            const int g = w + 4 * j;
            const int o = g * 1024 + lane * 16;
            const int L = o / RS, qc = (o - L * RS) >> 4;
            const int ch = qc < 32 ? qc : 0;
            srow[j] = L;
            schk[j] = ch;
            int cls = 0;
            if (L >= ly.nrows) cls = 1;
            else if (ly.M == TMS) cls = L == 0 ? 2 : (L == TMS + 1 ? 3 : 0);
            else {
                const int k = L % (ly.M + 2);
                cls = (k == 0 || k == ly.M + 1) ? 1 : 0;
            }
            if (MASKED && (L == 0 || L == TMS + 1)) cls = 1;   // no halo rows in masked layouts
            scls[j] = cls;
            soff[j] = MASKED || cls == 1 ? 0 : row_toff(L, ly, d) * C + ch * 4;
        }
    }
    // point the slots at tile nt of src ([B][T][C] fp32)
    __device__ __forceinline__ void aim(const float* src, const Tile& nt, const Layout& ly, int T, int n) {
        t = nt;
        vmask = 1u;
        if (!MASKED && ly.M == TMS) {
            const int m0 = nt.p0 % n;
            vmask |= (m0 > 0 ? 4u : 0u) | (m0 + TMS < n ? 8u : 0u);
        }
        base = src + ((size_t)nt.b * T + nt.tb) * C;
    }
    __device__ __forceinline__ void issue(int j, const float* src, const float* zero, uint32_t lds0,
                                          int T, int n, int d) const {
        const float* p = zero;
        if (MASKED) {
            const int pp = t.p0 + srow[j] - 1;
            if (scls[j] != 1 && pp >= 0 && pp < T)
                p = src + ((size_t)t.b * T + (pp % n) * d + pp / n) * C + schk[j] * 4;
        } else if ((vmask >> scls[j]) & 1u) {
            p = base + soff[j];
        }
        dma16(p, lds0 + j * 4096);
    }
};

// power-of-two exponent m with mx * 2^m in [2^13, 2^14) (0 for mx == 0 or non-finite mx)
__device__ __forceinline__ int scale_exp(float mx) {
    if (!(mx > 0.f) || !(mx < 3.0e38f)) return 0;
    int m = 14 - __builtin_amdgcn_frexp_expf(mx);
    return m < -60 ? -60 : (m > 60 ? 60 : m);
}
__device__ __forceinline__ float exp2i(int e) { return __builtin_ldexpf(1.0f, e); }

// split four fp32 values (already scaled) into rtz fp16 halves: hi / lo as 2 dwords each
__device__ __forceinline__ void split4(float a0, float a1, float a2, float a3, uint2& hi, uint2& lo) {
    const auto h01 = __builtin_amdgcn_cvt_pkrtz(a0, a1);
    const auto h23 = __builtin_amdgcn_cvt_pkrtz(a2, a3);
    const auto l01 = __builtin_amdgcn_cvt_pkrtz(a0 - (float)h01[0], a1 - (float)h01[1]);
    const auto l23 = __builtin_amdgcn_cvt_pkrtz(a2 - (float)h23[0], a3 - (float)h23[1]);
    hi = make_uint2(__builtin_bit_cast(uint32_t, h01), __builtin_bit_cast(uint32_t, h23));
    lo = make_uint2(__builtin_bit_cast(uint32_t, l01), __builtin_bit_cast(uint32_t, l23));
}

// fp32 rows [0, nrows) of slot src -> split rows of dst (hi: bytes 0..255, lo: 256..511 of the
// row), scaled by s (optionally relu'd first).  Two rows per wave instruction.
template <bool RELU>
__device__ __forceinline__ void convert_rows(const uint8_t* src, uint8_t* dst, int nrows, float s,
                                             int w, int lane) {
    const int half = lane >> 5, l = lane & 31;
    for (int pr = w; 2 * pr < nrows; pr += 4) {
        const int row = 2 * pr + half;
        const float4 v = *reinterpret_cast<const float4*>(src + row * RS + l * 16);
        float a0 = v.x, a1 = v.y, a2 = v.z, a3 = v.w;
        if (RELU) { a0 = fmaxf(a0, 0.f); a1 = fmaxf(a1, 0.f); a2 = fmaxf(a2, 0.f); a3 = fmaxf(a3, 0.f); }
        uint2 hi, lo;
        split4(a0 * s, a1 * s, a2 * s, a3 * s, hi, lo);
        *reinterpret_cast<uint2*>(dst + row * RS + l * 8) = hi;
        *reinterpret_cast<uint2*>(dst + row * RS + 256 + l * 8) = lo;
    }
}

__device__ __forceinline__ f32x16 mfma_f16(uint4 a, uint4 b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8, a),
                                                   __builtin_bit_cast(f16x8, b), c, 0, 0, 0);
}
// the three products of a split pair: acc += ah bh + al bh + ah bl
__device__ __forceinline__ f32x16 mfma3(uint4 ah, uint4 al, uint4 bh, uint4 bl, f32x16 c) {
    c = mfma_f16(ah, bh, c);
    c = mfma_f16(al, bh, c);
    return mfma_f16(ah, bl, c);
}

// tied no-op: pins a fragment to the accumulator register file (MFMA A operands may be AGPRs)
__device__ __forceinline__ uint4 to_agpr(uint4 v) {
    u32x4 t = __builtin_bit_cast(u32x4, v);
    asm volatile("" : "=a"(t) : "0"(t));
    return __builtin_bit_cast(uint4, t);
}

// LDS-only barrier: no vector-memory drain (the DMA of the next tile stays in flight)
__device__ __forceinline__ void lds_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}

// scalar load of a uniform word: a compiler-visible vector load would make the compiler wait
// for every older vector-memory op, the kernels' in-flight DMA included
__device__ __forceinline__ float sload(const float* p) {
    float v;
    asm volatile("s_load_dword %0, %1, 0x0\n\ts_waitcnt lgkmcnt(0)" : "=s"(v) : "s"(p) : "memory");
    return v;
}

__device__ __forceinline__ void pin_all(uint4 (&wd)[3][8][2], uint4 (&wr)[8][2]) {
#pragma unroll
    for (int tp = 0; tp < 3; ++tp)
#pragma unroll
        for (int kb = 0; kb < 8; ++kb)
#pragma unroll
            for (int hl = 0; hl < 2; ++hl) wd[tp][kb][hl] = to_agpr(wd[tp][kb][hl]);
#pragma unroll
    for (int kb = 0; kb < 8; ++kb)
#pragma unroll
        for (int hl = 0; hl < 2; ++hl) wr[kb][hl] = to_agpr(wr[kb][hl]);
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v = fmaxf(v, __shfl_xor(v, off));
    return v;
}

// relu-mask word of a lane's 32 x 32 accumulator tile: bit mbit(i) = acc[i] > 0 (the bf16
// path's layout, common.h)
__device__ __forceinline__ uint32_t mask_bits(const f32x16& acc) {
    uint32_t wd = 0;
#pragma unroll
    for (int i = 0; i < 16; ++i) wd |= (acc[i] > 0.f ? 1u : 0u) << mbit(i);
    return wd;
}
// zero the elements of an accumulator tile whose bit mbit(i) of mask word wd is clear
__device__ __forceinline__ void apply_mask(f32x16& acc, uint32_t wd) {
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        const int s = ((int)(wd << (31 - mbit(i)))) >> 31;   // v_bfe_i32
        acc[i] = __int_as_float(__float_as_int(acc[i]) & s);
    }
}

}  // namespace sw
}  // namespace ast
