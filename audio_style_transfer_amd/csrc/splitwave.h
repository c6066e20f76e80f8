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
constexpr int DPW = 9;                   // one-KiB DMA groups per wave per slot (36 groups)
constexpr int SLOT = 36992;              // bytes per LDS slot: 70 rows (the conversion's pairs
                                         // 0..34), the DMA fills the first 36 KiB
static_assert(4 * DPW * 1024 <= SLOT && 68 * RS <= 4 * DPW * 1024, "DMA groups cover every image row");
static_assert(70 * RS <= SLOT, "the conversion's last pair stays inside the slot");

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

// the same in the saddr form: address = base (uniform, scalar pair) + off (per lane, bytes)
__device__ __forceinline__ void dma16s(const void* base, uint32_t off, uint32_t lds_base) {
    uint32_t keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\t"
                 "global_load_lds_dwordx4 %1, %2\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(off), "s"(base), "s"(lds_base) : "memory");
}

// Image rows of a tile with no source row are zeroed at conversion (unmasked layouts): the pad
// rows of the segment layouts, and the halo rows of a one-segment tile at a sub-sequence end.
// Their DMA reads a row of the same tile instead, so every DMA address is in bounds.
__device__ __forceinline__ bool pad_row(int L, const Layout& ly) {
    if (ly.M == TMS) return false;
    const int k = L % (ly.M + 2);
    return k == 0 || k == ly.M + 1;
}
// Conversion of a slot: wave w converts row pairs conv_pair(w, k) = min(w + 4 k, 34), k < 9
// (pair 34 = rows 68, 69 lies past every image, inside the slot: converted twice, harmlessly,
// by waves 2 and 3).
// Lane bit k of the zero-row word: this lane's row 2 conv_pair(w, k) + (lane >> 5) is zeroed.
constexpr int NCONV = 9;
__device__ __forceinline__ int conv_pair(int w, int k) { return min(w + 4 * k, 34); }
__device__ __forceinline__ uint32_t pad_bits(const Layout& ly, int w, int lane) {   // per launch
    uint32_t z = 0;
    for (int k = 0; k < NCONV; ++k)
        if (pad_row(2 * conv_pair(w, k) + (lane >> 5), ly)) z |= 1u << k;
    return z;
}
template <bool MASKED>
__device__ __forceinline__ uint32_t zero_bits(uint32_t pad, const Tile& t, const Layout& ly, int n,
                                              int w, int lane) {
    if (MASKED || ly.M != TMS || w != 0) return MASKED ? 0u : pad;
    const int m0 = t.p0 % n;
    const int h = lane >> 5;
    // row 0 = pair 0 (k 0) low half, row 65 = pair 32 (k 8) high half, both wave 0
    return (h == 0 && m0 == 0 ? 1u : 0u) | (h == 1 && m0 + TMS >= n ? 1u << 8 : 0u);
}
__device__ __forceinline__ float conv_scale(uint32_t zb, int k, float s) {
    return (zb >> k) & 1u ? 0.f : s;
}

// ---- register-fed row units (block kernels): unit k (k < NU), lane -> image row
//      L = 8 k + (lane >> 3), channels cq .. cq + 3 of the wave's quarter (32 w .. 32 w + 31):
//      one wave instruction loads 8 rows x 128 B (8 cache lines).  Unmasked layouts address a
//      unit as the tile's row-0 source (time tb - d) + a constant per-lane byte offset; rows
//      without a source (pad rows, rows past the image, a one-segment halo at a sub-sequence
//      end) read a row of the tile and are zeroed at conversion (zero bit k).  Masked layouts
//      gather per lane (rows 0 and 65 have no source). ----
constexpr int NU = 9;
template <bool MASKED, bool ONESEG>
struct RowUnits {
    int lr, cq;
    uint32_t imgo, ero;      // LDS byte offsets of the lane's split / fp32 chunk in row lr
    uint32_t soff[NU];
    uint32_t padz;
    uint32_t row1, row64;

    __device__ __forceinline__ void init(int w, int lane, const Layout& ly, int d) {
        lr = lane >> 3;
        cq = 32 * w + 4 * (lane & 7);
        imgo = (uint32_t)(lr * RS + 2 * cq);
        ero = (uint32_t)(lr * RS + 4 * cq);
        padz = 0;
#pragma unroll
        for (int k = 0; k < NU; ++k) {
            const int L = 8 * k + lr;
            const bool none = MASKED ? (L == 0 || L > TMS) : (L >= ly.nrows || pad_row(L, ly));
            if (none) padz |= 1u << k;
            soff[k] = MASKED ? 0u : (uint32_t)(((none ? 0 : row_toff(L, ly, d)) + d) * C * 4 + 4 * cq);
        }
        row1 = (uint32_t)(d * C * 4 + 4 * cq);
        row64 = (uint32_t)(TMS * d * C * 4 + 4 * cq);       // image row 64 (time tb + 63 d)
    }
    // unit k of tile t of tensor src ([B][T][C] fp32)
    __device__ __forceinline__ float4 load(const float* src, const Tile& t, int k, int T, int n, int d) const {
        if (MASKED) {
            const int L = 8 * k + lr;
            const int pp = t.p0 + ((padz >> k) & 1u ? 0 : L - 1);
            return *reinterpret_cast<const float4*>(src + ((size_t)t.b * T + (pp % n) * d + pp / n) * C + cq);
        }
        const char* base = reinterpret_cast<const char*>(src + ((ptrdiff_t)t.b * T + t.tb - d) * C);
        uint32_t o = soff[k];
        if (ONESEG && k == 0 && lr == 0 && t.p0 % n == 0) o = row1;
        if (ONESEG && k == NU - 1 && lr == 1 && t.p0 % n + TMS >= n) o = row64;
        return *reinterpret_cast<const float4*>(base + o);
    }
    __device__ __forceinline__ uint32_t zero_bits(const Tile& t, int n) const {
        uint32_t z = padz;
        if (ONESEG) {
            const int m0 = t.p0 % n;
            if (lr == 0 && m0 == 0) z |= 1u;
            if (lr == 1 && m0 + TMS >= n) z |= 1u << (NU - 1);
        }
        return z;
    }
};

// x where bit k of word wd is set, else 0 (v_bfe_i32 + v_and)
__device__ __forceinline__ float keep_if(float x, uint32_t wd, int k) {
    const int s = ((int)(wd << (31 - k))) >> 31;
    return __int_as_float(__float_as_int(x) & s);
}

// one step of 3 MFMAs: the first, the next step's B reads, then the other two with side work
__device__ __forceinline__ void step3_schedule() {
    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);       // 1 MFMA
    __builtin_amdgcn_sched_group_barrier(0x100, 4, 0);       // DS reads
#pragma unroll
    for (int m = 1; m < 3; ++m) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);   // 1 MFMA
        __builtin_amdgcn_sched_group_barrier(0x002, 7, 0);   // VALU
        __builtin_amdgcn_sched_group_barrier(0x200, 2, 0);   // DS writes
    }
    __builtin_amdgcn_sched_barrier(0);
}

// One wave's share of a slot: group g = w + 4 j (j < DPW) covers slot bytes [1024 g, +1024);
// this lane's 16 B land at row L, chunk qc (qc == 32 is the row's pad chunk, filled with a
// harmless re-read of chunk 0).
//   unmasked layouts: a constant byte offset per lane from the tile's row-0 source address
//     (time tb - d; row_toff(L) + d >= 0), one saddr issue per group and no vector ALU.  Rows
//     without a source read row 1 (pad rows, rows past the image) or the nearest tile row (a halo
//     row at a sub-sequence end: rows 0 / 65 sit in groups 0 / 33, 34 = j 0 / DPW - 1) and are
//     zeroed at conversion (ZeroRows).
//   masked layouts (n < 32): gathered per lane, rows without a source read the zero line.
template <bool MASKED>
struct RowDma;

template <>
struct RowDma<false> {
    uint32_t off[DPW];
    uint32_t halt[2];    // j = 0 / DPW - 1: offset used when the lane's halo row has no source
    int hcls[2];         // 0, or 2 (row 0) / 3 (row 65) of a one-segment layout
    const float* base;   // per tile (aim)
    bool lok, rok;

    __device__ __forceinline__ void init(int w, int lane, const Layout& ly, int d) {
#pragma unroll
        for (int j = 0; j < DPW; ++j) {
            const int o = (w + 4 * j) * 1024 + lane * 16;
            const int L = o / RS, qc = (o - L * RS) >> 4;
            const int ch = qc < 32 ? qc : 0;
            const int Ls = (L >= ly.nrows || pad_row(L, ly)) ? 1 : L;
            off[j] = (uint32_t)((row_toff(Ls, ly, d) + d) * C * 4 + ch * 16);
            if (j == 0 || j == DPW - 1) {
                const int q = j == 0 ? 0 : 1;
                hcls[q] = ly.M == TMS && L == 0 ? 2 : (ly.M == TMS && L == TMS + 1 ? 3 : 0);
                halt[q] = (uint32_t)((row_toff(L == 0 ? 1 : TMS, ly, d) + d) * C * 4 + ch * 16);
            }
        }
        lok = rok = true;
    }
    __device__ __forceinline__ void aim(const float* src, const Tile& nt, const Layout& ly, int T, int n, int d) {
        if (ly.M == TMS) {
            const int m0 = nt.p0 % n;
            lok = m0 > 0;
            rok = m0 + TMS < n;
        }
        base = src + ((ptrdiff_t)nt.b * T + nt.tb - d) * C;
    }
    __device__ __forceinline__ void issue(int j, const float*, const float*, uint32_t lds0, int, int, int) const {
        uint32_t o = off[j];
        if (j == 0 || j == DPW - 1) {
            const int q = j == 0 ? 0 : 1;
            if ((hcls[q] == 2 && !lok) || (hcls[q] == 3 && !rok)) o = halt[q];
        }
        dma16s(base, o, lds0 + j * 4096);
    }
};

template <>
struct RowDma<true> {
    int srow[DPW], schk[DPW];
    bool zl[DPW];        // rows without a source (0, 65 and past the image)
    Tile t;

    __device__ __forceinline__ void init(int w, int lane, const Layout& ly, int) {
#pragma unroll
        for (int j = 0; j < DPW; ++j) {
            const int o = (w + 4 * j) * 1024 + lane * 16;
            const int L = o / RS, qc = (o - L * RS) >> 4;
            srow[j] = L;
            schk[j] = qc < 32 ? qc : 0;
            zl[j] = L >= ly.nrows || L == 0 || L == TMS + 1;
        }
    }
    __device__ __forceinline__ void aim(const float*, const Tile& nt, const Layout&, int, int, int) { t = nt; }
    __device__ __forceinline__ void issue(int j, const float* src, const float* zero, uint32_t lds0,
                                          int T, int n, int d) const {
        const float* p = zero;
        const int pp = t.p0 + srow[j] - 1;
        if (!zl[j] && pp >= 0 && pp < T)
            p = src + ((size_t)t.b * T + (pp % n) * d + pp / n) * C + schk[j] * 4;
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

// In-place conversion of one row pair of an LDS slot: fp32 rows 2 p, 2 p + 1 (as DMA'd) ->
// split rows (hi: bytes 0..255, lo: 256..511) of s x (relu(x) with RELU).  One wave
// instruction reads both rows whole before the same wave overwrites them, so the conversion is
// safe in place.  pair_read / pair_write are the two halves, for software-pipelined conversion.
__device__ __forceinline__ float4 pair_read(const uint8_t* slot, int p, int lane) {
    return *reinterpret_cast<const float4*>(slot + (2 * p + (lane >> 5)) * RS + (lane & 31) * 16);
}
template <bool RELU>
__device__ __forceinline__ void pair_write(uint8_t* slot, int p, float4 v, float s, int lane) {
    uint8_t* row = slot + (2 * p + (lane >> 5)) * RS;
    const int l = lane & 31;
    if (RELU) {   // relu as an integer max of the bits (negative floats are negative ints)
        v.x = __int_as_float(max(__float_as_int(v.x), 0)); v.y = __int_as_float(max(__float_as_int(v.y), 0));
        v.z = __int_as_float(max(__float_as_int(v.z), 0)); v.w = __int_as_float(max(__float_as_int(v.w), 0));
    }
    uint2 hi, lo;
    split4(v.x * s, v.y * s, v.z * s, v.w * s, hi, lo);
    *reinterpret_cast<uint2*>(row + l * 8) = hi;
    *reinterpret_cast<uint2*>(row + 256 + l * 8) = lo;
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

// Instruction order of one GEMM k-step (6 MFMAs): the first MFMA (its B fragments were read a
// step earlier), then the next step's LDS reads, then each remaining MFMA followed by a group of
// vector ALU / LDS-write side work that issues in its shadow.  Side work that consumes an LDS
// read issued a step earlier (the in-place conversion) then waits only for that read: LDS
// counters retire in order, so work placed after this step's reads would also wait for them.
// The step ends with a scheduling barrier.
__device__ __forceinline__ void step_schedule() {
    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);       // 1 MFMA
    __builtin_amdgcn_sched_group_barrier(0x100, 6, 0);       // DS reads
#pragma unroll
    for (int m = 1; m < 6; ++m) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);   // 1 MFMA
        __builtin_amdgcn_sched_group_barrier(0x002, 6, 0);   // up to 6 VALU
        __builtin_amdgcn_sched_group_barrier(0x200, 1, 0);   // up to 1 DS write
    }
    __builtin_amdgcn_sched_barrier(0);
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v = fmaxf(v, __shfl_xor(v, off));
    return v;
}

// [x > 0] as 0 / 1 for every non-NaN x: the bits as a signed integer clamped to [0, 1] (one
// v_med3_i32; +0 and negatives give 0)
__device__ __forceinline__ uint32_t pos_bit(float x) {
    uint32_t b;
    asm("v_med3_i32 %0, %1, 0, 1" : "=v"(b) : "v"(x));
    return b;
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
