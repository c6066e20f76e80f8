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
// A tile's input rows are loaded a tile ahead into registers (RowUnits), converted into an LDS
// split image (the first GEMM's B operand) and an fp32 residual buffer; the first GEMM's
// epilogue writes the second GEMM's split B operand.
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

struct Layout {            // uniform per launch (pick_layout)
    int M;                 // segment length; TMS = one segment with two halo rows
    int nrows;             // image rows
};

// One segment with halo rows when a tile lies inside one sub-sequence (n % 64 == 0); whole
// sub-sequences of 32 positions with their own zero pad rows (n == 32); otherwise per-column
// tap masks over 64 gathered positions (MASKED, n < 32).
// The segment layout is always n = SEGM = 32 (n < 64 dividing 64, n >= 32): the device helpers
// below divide by the constants SEGM / SEGM + 2, not by ly.M (a runtime division is ~20 VALU, and
// under register pressure the compiler recomputes these per tile, round 6)
constexpr int SEGM = 32;
inline bool pick_layout(int n, Layout& ly) {
    if (n % TMS == 0) { ly.M = TMS; ly.nrows = TMS + 2; return false; }
    if (n == SEGM) { ly.M = n; ly.nrows = (TMS / n) * (n + 2); return false; }
    ly.M = TMS; ly.nrows = TMS + 2;
    return true;
}

int num_cus();

__device__ __forceinline__ int frow(int c, const Layout& ly) {   // image row of tile column c
    return ly.M == TMS ? c + 1 : (c / SEGM) * (SEGM + 2) + 1 + (c % SEGM);
}

// time offset of image row L from the tile's base time (unmasked layouts):
//   one segment: rows are positions p0-1 .. p0+64 of one sub-sequence, t = tb + (L-1) d
//   segments of M = n: row (s, k) is position k-1 of sub-sequence j0 + s, t = tb + (k-1) d + s
__device__ __forceinline__ int row_toff(int L, const Layout& ly, int d) {
    if (ly.M == TMS) return (L - 1) * d;
    const int s = L / (SEGM + 2), k = L - s * (SEGM + 2);
    return (k - 1) * d + s;
}

struct Tile { int b, p0, tb, m0; };   // clip, first position, base time, p0 mod n

// Tile order: clip-interleaved (SW_TILE_INTERLEAVE, ft divides by B): tile tl is clip tl mod B,
// position block tl / B, so the workgroups of one round work on different clips and their
// per-clip max atomics go to different words (clip-major order puts all 1024 waves' atomics of
// a round on ONE word).  Otherwise clip-major (ft divides by T / 64).
#ifndef SW_TILE_INTERLEAVE
#define SW_TILE_INTERLEAVE 1
#endif
template <bool MASKED>
__device__ __forceinline__ Tile tile_at(int tl, const FDiv& ft, const FDiv& fn, int d, const Layout& ly) {
    Tile t;
#if SW_TILE_INTERLEAVE
    const int pb = (int)fdiv((uint32_t)tl, ft);
    t.b = tl - pb * (int)ft.n;
    t.p0 = pb * TMS;
#else
    t.b = (int)fdiv((uint32_t)tl, ft);
    t.p0 = (tl - t.b * (int)ft.n) * TMS;
#endif
    const int q = (int)fdiv((uint32_t)t.p0, fn);
    t.m0 = t.p0 - q * (int)fn.n;
    t.tb = MASKED ? 0 : (ly.M == TMS ? t.m0 * d + q : q);
    return t;
}

// time of tile column cc (toff = row_toff of its image row, unmasked layouts)
template <bool MASKED>
__device__ __forceinline__ int col_time(const Tile& t, int cc, int toff, const FDiv& fn, int d) {
    if (MASKED) {
        const int p = t.p0 + cc;
        const int q = (int)fdiv((uint32_t)p, fn);
        return (p - q * (int)fn.n) * d + q;
    }
    return t.tb + toff;
}
// position p of a layer with n positions per sub-sequence -> time (time_to_batch inverse)
__device__ __forceinline__ int pos_time(int p, const FDiv& fn, int d) {
    const int q = (int)fdiv((uint32_t)p, fn);
    return (p - q * (int)fn.n) * d + q;
}

// raw buffer access: a uniform base in the resource (scalar registers) + a 32-bit per-lane
// offset + a uniform offset, so a kernel keeps one VGPR per access stream instead of a 64-bit
// address per lane (the role-split kernels' residual waves are register-bound)
typedef __amdgpu_buffer_rsrc_t rsrc_t;
__device__ __forceinline__ rsrc_t mk_rsrc(const void* p) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, 0x7fffffff, 0x00020000);
}
// cache-policy bits of the block kernels' row loads / stores (gfx950 CPol: 2 = nt); A/B builds
// only (ASTYLE_DEFS=-DSW_LD_AUX=2 ...), the shipped kernels use the default policy
#ifndef SW_LD_AUX
#define SW_LD_AUX 0
#endif
#ifndef SW_ST_AUX
#define SW_ST_AUX 0
#endif
__device__ __forceinline__ float4 bld4(rsrc_t r, uint32_t voff, uint32_t soff) {
    return __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(r, voff, soff, SW_LD_AUX));
}
__device__ __forceinline__ void bst4(rsrc_t r, uint32_t voff, uint32_t soff, float4 v) {
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), r, voff, soff, SW_ST_AUX);
}

__device__ __forceinline__ uint4 lds16(const uint8_t* p) { return *reinterpret_cast<const uint4*>(p); }

// Image rows of a tile with no source row are zeroed at conversion (unmasked layouts): the pad
// rows of the segment layouts, and the halo rows of a one-segment tile at a sub-sequence end.
// Their DMA reads a row of the same tile instead, so every DMA address is in bounds.
__device__ __forceinline__ bool pad_row(int L, const Layout& ly) {
    if (ly.M == TMS) return false;
    const int k = L % (SEGM + 2);
    return k == 0 || k == SEGM + 1;
}
// ---- register-fed row units (block kernels): unit k (k < NU), lane -> image row
//      L = 8 k + (lane >> 3), channels cq .. cq + 3 of the wave's quarter (32 w .. 32 w + 31):
//      one wave instruction loads 8 rows x 128 B (8 cache lines).  Unmasked layouts address a
//      unit as the tile's row-0 source (time tb - d) + a constant per-lane byte offset; rows
//      without a source (pad rows, rows past the image, a one-segment halo at a sub-sequence
//      end) read a row of the tile and are zeroed at conversion (zero bit k).  Masked layouts
//      gather per lane: row L is position p0 + L - 1 (clamped into the clip; a tile may start
//      or end inside a sub-sequence, so rows 0 and 65 can be real neighbours), and the
//      per-column tap masks drop every neighbour outside the column's sub-sequence. ----
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
            const bool none = MASKED ? L > TMS + 1 : (L >= ly.nrows || pad_row(L, ly));
            if (none) padz |= 1u << k;
            soff[k] = MASKED ? 0u : (uint32_t)(((none ? 0 : row_toff(L, ly, d)) + d) * C * 4 + 4 * cq);
        }
        row1 = (uint32_t)(d * C * 4 + 4 * cq);
        row64 = (uint32_t)(TMS * d * C * 4 + 4 * cq);       // image row 64 (time tb + 63 d)
    }
    // unit k of tile t of tensor src ([B][T][C] fp32)
    __device__ __forceinline__ float4 load(const float* src, const Tile& t, int k, int T, const FDiv& fn, int d) const {
        if (MASKED) {
            const int L = 8 * k + lr;
            const int pp = (padz >> k) & 1u ? t.p0 : min(max(t.p0 + L - 1, 0), T - 1);
            return *reinterpret_cast<const float4*>(src + ((size_t)t.b * T + pos_time(pp, fn, d)) * C + cq);
        }
        const char* base = reinterpret_cast<const char*>(src + ((ptrdiff_t)t.b * T + t.tb - d) * C);
        uint32_t o = soff[k];
        if (ONESEG && k == 0 && lr == 0 && t.m0 == 0) o = row1;
        if (ONESEG && k == NU - 1 && lr == 1 && t.m0 + TMS >= (int)fn.n) o = row64;
        return *reinterpret_cast<const float4*>(base + o);
    }
    // unmasked layouts: the same rows through a buffer resource whose base is the tile's row-0
    // source (rsrc_of): one 32-bit lane offset per unit instead of a 64-bit address
    __device__ __forceinline__ rsrc_t rsrc_of(const float* src, const Tile& t, int T, int d) const {
        return mk_rsrc(src + ((ptrdiff_t)t.b * T + t.tb - d) * C);
    }
    __device__ __forceinline__ uint32_t unit_off(const Tile& t, int k, const FDiv& fn) const {
        uint32_t o = soff[k];
        if (ONESEG && k == 0 && lr == 0 && t.m0 == 0) o = row1;
        if (ONESEG && k == NU - 1 && lr == 1 && t.m0 + TMS >= (int)fn.n) o = row64;
        return o;
    }
    __device__ __forceinline__ float4 loadb(rsrc_t rs, const Tile& t, int k, const FDiv& fn) const {
        return bld4(rs, unit_off(t, k, fn), 0u);
    }
    __device__ __forceinline__ uint32_t zero_bits(const Tile& t, const FDiv& fn) const {
        uint32_t z = padz;
        if (ONESEG) {
            if (lr == 0 && t.m0 == 0) z |= 1u;
            if (lr == 1 && t.m0 + TMS >= (int)fn.n) z |= 1u << (NU - 1);
        }
        return z;
    }
};

// x where bit k of word wd is set, else +0: v_bfe_i32 + v_and (the C shift form compiles to a
// bit test, a compare and a select; the sbfe builtin to the one instruction)
__device__ __forceinline__ float keep_if(float x, uint32_t wd, int k) {
    const int s = __builtin_amdgcn_sbfe((int)wd, k, 1);   // v_bfe_i32, visible to the scheduler
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

__device__ __forceinline__ f32x16 mfma_f16(uint4 a, uint4 b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8, a),
                                                   __builtin_bit_cast(f16x8, b), c, 0, 0, 0);
}

// ---- the 16x16x32 form (ASTYLE_MFMA16=1: block_fwd_split16.hip, block_bwd_split16.hip; round 6,
//      measured no faster than the 32x32x16 default).  A wave's output tile of a
//      column half is its 32 channels x 32 columns as four 16 x 16 sub-tiles n = 2 cb + rb (row
//      block rb: channels 16 rb .. + 15 of the wave's 32; column block cb: columns 16 cb .. + 15).
//      Lane (i = lane & 15, q = lane >> 4):
//        A fragment (weights, slot s = 2 kb + rb of K block kb of 32): A[16 rb + i][32 kb + 8 q + e]
//        B fragment (image rows, K block kb):                           B[32 kb + 8 q + e][16 cb + i]
//        accumulator n, element k:                                      D[16 rb + 4 q + k][16 cb + i]
//      A step (K block kb, column block cb) reads one B fragment pair (hi, lo) and issues 3
//      products x 2 row blocks: the FLOP, operand registers and LDS bytes of a 32x32x16 step ----
typedef float f32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ f32x4 mfma16(uint4 a, uint4 b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, a),
                                                   __builtin_bit_cast(f16x8, b), c, 0, 0, 0);
}
// one 16x16x32 step: 6 MFMAs of 16 cycles, the next steps' B reads after the first pair
__device__ __forceinline__ void step6_schedule() {
    __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);       // 2 MFMAs
    __builtin_amdgcn_sched_group_barrier(0x100, 4, 0);       // DS reads
#pragma unroll
    for (int m = 1; m < 3; ++m) {
        __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);   // 2 MFMAs
        __builtin_amdgcn_sched_group_barrier(0x002, 7, 0);   // VALU
        __builtin_amdgcn_sched_group_barrier(0x200, 2, 0);   // DS writes
    }
    __builtin_amdgcn_sched_barrier(0);
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
// for every older vector-memory op, the kernels' in-flight DMA included.  The words it reads are
// per-clip maxima that atomics of the PREVIOUS launch on the same stream wrote: the kernel
// boundary (the producer's end-of-kernel release, this kernel's start acquire, which invalidates
// the scalar cache) makes them visible.  Round 5 measured the glc form (a miss in the scalar
// cache on every load): no change to the graph-replay defect of DESIGN.md §3, and +1.3 ms per
// step at one clip, where every workgroup of a launch reads the same word (configs[1]: 478 ->
// 299 iters/s); reverted
__device__ __forceinline__ float sload(const float* p) {
    float v;
    asm volatile("s_load_dword %0, %1, 0x0\n\ts_waitcnt lgkmcnt(0)" : "=s"(v) : "s"(p) : "memory");
    return v;
}

// a clip's max over its GSLOTS slots (common.h): eight scalar loads in flight, one wait.  The
// outputs are early-clobber: a load's destination must not be the base pair the later loads read
__device__ __forceinline__ float sload_gmax(const float* lvl, int b) {
    const float* p = lvl + (size_t)b * GCLIP_W;
    uint32_t v0, v1, v2, v3, v4, v5, v6, v7;
    static_assert(GSLOTS == 8 && GSLOT_W == 32, "sload_gmax: 8 slots 128 B apart");
    asm volatile("s_load_dword %0, %8, 0x0\n\ts_load_dword %1, %8, 0x80\n\t"
                 "s_load_dword %2, %8, 0x100\n\ts_load_dword %3, %8, 0x180\n\t"
                 "s_load_dword %4, %8, 0x200\n\ts_load_dword %5, %8, 0x280\n\t"
                 "s_load_dword %6, %8, 0x300\n\ts_load_dword %7, %8, 0x380\n\t"
                 "s_waitcnt lgkmcnt(0)"
                 : "=&s"(v0), "=&s"(v1), "=&s"(v2), "=&s"(v3), "=&s"(v4), "=&s"(v5), "=&s"(v6), "=&s"(v7)
                 : "s"(p) : "memory");
    return __uint_as_float(max(max(max(v0, v1), max(v2, v3)), max(max(v4, v5), max(v6, v7))));
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

// max over the wave of non-negative floats (compared as their bits), uniform result: four DPP
// steps make every row of 16 lanes uniform, then the four rows meet in scalar registers (the
// __shfl_xor form is six dependent ds_bpermute round trips, ~500 exposed cycles per tile)
__device__ __forceinline__ uint32_t wave_max_bits(float x) {
    int v = __float_as_int(x);
    v = max(v, __builtin_amdgcn_update_dpp(0, v, 0xB1, 0xF, 0xF, false));    // quad_perm [1,0,3,2]
    v = max(v, __builtin_amdgcn_update_dpp(0, v, 0x4E, 0xF, 0xF, false));    // quad_perm [2,3,0,1]
    v = max(v, __builtin_amdgcn_update_dpp(0, v, 0x141, 0xF, 0xF, false));   // row_half_mirror
    v = max(v, __builtin_amdgcn_update_dpp(0, v, 0x140, 0xF, 0xF, false));   // row_mirror
    const int a = __builtin_amdgcn_readlane(v, 0), b = __builtin_amdgcn_readlane(v, 16);
    const int c = __builtin_amdgcn_readlane(v, 32), d = __builtin_amdgcn_readlane(v, 48);
    return (uint32_t)max(max(a, b), max(c, d));
}

// The end of a block launch: the workgroup's max for its last clip in ONE global atomic, the four
// waves' maxima meeting in LDS first (round 6).  At one clip every workgroup ends on the same
// clip, and the 1024 per-wave atomics on one line serialised at L2 (~8 ns each: ~8 us of a 25-us
// launch; phase stamps showed the waves done after ~12 us).  The max is the same.
__device__ __forceinline__ void wg_max_flush(uint32_t (&slots)[4], uint32_t m, unsigned* dst) {
    if ((threadIdx.x & 63) == 0) slots[threadIdx.x >> 6] = m;
    lds_barrier();
    if (threadIdx.x == 0) atomicMax(dst, max(max(slots[0], slots[1]), max(slots[2], slots[3])));
}

// [x > 0] as 0 / 1 for every non-NaN x: the bits as a signed integer clamped to [0, 1] (one
// v_med3_i32; +0 and negatives give 0)
__device__ __forceinline__ uint32_t pos_bit(float x) {
    uint32_t b;
    asm("v_med3_i32 %0, %1, 0, 1" : "=v"(b) : "v"(x));
    return b;
}


// mask-word bits of an accumulator group g (values x0..x3 = elements 4 g .. 4 g + 3, bits
// mbit = 4 q + g): [x0 > 0] << g | [x1 > 0] << (4 + g) | [x2 > 0] << (8 + g) | [x3 > 0] << (12 + g),
// or'ed into w; 2 instructions per value
__device__ __forceinline__ uint32_t or_pos_bits4(uint32_t w, float x0, float x1, float x2, float x3, int g) {
    uint32_t t = (pos_bit(x3) << 4) | pos_bit(x2);   // each step one v_lshl_or_b32
    t = (t << 4) | pos_bit(x1);
    t = (t << 4) | pos_bit(x0);
    return (t << g) | w;
}

// ---- leaner split / bit helpers (round 3 kernels) ----
typedef unsigned short u16x2_t __attribute__((ext_vector_type(2)));

// a0, a1 >= 0 (relu'd, scaled): hi = rtz_f16 pair; lo = rtz_f16(a - hi) pair (the remainder
// formed by v_fma_mix_f32 from the packed half).  SW_LO_MIX: lo = rne_f16(a - hi) straight into
// the packed half by v_fma_mixlo/hi_f16 (one instruction per value instead of 1.5): its
// extracts are closer to fp64 (6.5e-7 vs 1.3e-6 rel-L2 at layer 29, T = 2048), but the
// gradient of the golden 'ours' case lands at 7.4e-4 from fp64 instead of 1.6e-4 (Gatys 1.3e-3
// vs 3.8e-4), both inside the fp32 rounding floor of the loss's conditioning; the default keeps
// the rtz pair, and the instruction saving measured no time (the loop is not VALU-bound).
__device__ __forceinline__ void split2(float a0, float a1, uint32_t& hi, uint32_t& lo) {
    const auto h = __builtin_amdgcn_cvt_pkrtz(a0, a1);
    hi = __builtin_bit_cast(uint32_t, h);
#ifdef SW_LO_MIX
    asm("v_fma_mixlo_f16 %0, %1, 1.0, -%2 op_sel_hi:[0,0,1]\n\t"
        "v_fma_mixhi_f16 %0, %3, 1.0, -%2 op_sel:[0,0,1] op_sel_hi:[0,0,1]"
        : "=&v"(lo) : "v"(a0), "v"(hi), "v"(a1));
#else
    lo = __builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_pkrtz(a0 - (float)h[0], a1 - (float)h[1]));
#endif
}

// the same for values of either sign (the backward's tot and g_u): hi = rtz, so a - hi has
// a's sign and lo = rtz(a - hi) keeps sign(lo) == sign(hi) or lo == 0
__device__ __forceinline__ void split2s(float a0, float a1, uint32_t& hi, uint32_t& lo) {
    split2(a0, a1, hi, lo);
}

// [x > 0] of the two halves of a relu'd hi pair as bits 0 and 16 (v_pk_min_u16 with 1): x > 0
// exactly when its rtz fp16 half is nonzero, i.e. for every x >= 2^-24 in the scaled units
// (2^-37 of the tensor's bound): smaller positive values are below fp32's own rounding noise
__device__ __forceinline__ uint32_t nz2(uint32_t hi) {
    const u16x2_t v = __builtin_elementwise_min(__builtin_bit_cast(u16x2_t, hi), (u16x2_t){1, 1});
    return __builtin_bit_cast(uint32_t, v);
}
// four values (q = 0..3: hi01, hi23) of accumulator group g into a mask accumulator w: q0 at bit
// g, q2 at 8 + g, q1 at 16 + g, q3 at 24 + g; mask16 folds that into the mbit(4 g + q) = 4 q + g
// layout of the u16 mask words (common.h)
__device__ __forceinline__ uint32_t or_bits4(uint32_t w, uint32_t hi01, uint32_t hi23, int g) {
    // (as asm: from the vector-min form the compiler emits compares and selects per half)
    uint32_t t0, t1;
    asm("v_pk_min_u16 %0, %2, %4\n\tv_pk_min_u16 %1, %3, %4\n\tv_lshl_or_b32 %0, %1, 8, %0"
        : "=&v"(t0), "=&v"(t1) : "v"(hi01), "v"(hi23), "s"(0x00010001u));
    return (t0 << g) | w;
}
__device__ __forceinline__ uint32_t mask16(uint32_t w) { return (w | (w >> 12)) & 0xffffu; }

}  // namespace sw
}  // namespace ast
