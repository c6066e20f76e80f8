// Shared pieces of the column-owning bf16 block kernels (block_fwd_bf16.hip, block_bwd_bf16.hip).
//
// Both kernels walk tiles of TMB = 128 positions of one layer in time_to_batch order
// (masked.py:57-86): one 256-thread workgroup per CU, wave w owns tile columns 32 w .. 32 w + 31
// and all 128 channels of them.  A tile's input rows (plus one halo / pad row either side of
// every segment) stream HBM -> LDS by global_load_lds into a padded image (rows of RSB bytes).
#pragma once
#include "common.h"

namespace ast {
namespace cw {

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

constexpr int FT = 256;                  // threads: one wave per SIMD
constexpr int RSB = 272;                 // image row stride (bytes): ds_read_b128 conflict-free
constexpr int FROWS = TMB + 8;           // max image rows (4 segments of 32 + 2 pads each)
constexpr int NDMA = (FROWS * RSB + 1023) / 1024;   // 37 one-KiB groups per image
constexpr int BUFB = NDMA * 1024;        // bytes per image
// The DMA fills groups 0..35 (9 per wave, no per-wave tail branch); group 36 holds only the
// last 128 B of row 135, which is a zero pad row of the 32-row segment layout (and unused by the
// others): it is zeroed once at kernel start and never written again.
constexpr int DPW = 9;
static_assert(4 * DPW * 1024 >= 135 * RSB + 128 && 4 * DPW * 1024 < FROWS * RSB,
              "DMA groups must cover every image row but the tail of row 135");
constexpr int SRB = 144;                 // staging row stride: one 128-B half row + 16 pad

struct Layout {            // uniform per launch (see pick_layout)
    int M;                 // segment length; TMB = one segment with two halo rows
    int nrows;             // image rows
};

// Segment layout when a tile lies inside one sub-sequence (n % 128 == 0) or holds whole
// sub-sequences of >= 32 positions; otherwise one segment with per-column tap masks (true).
inline bool pick_layout(int n, Layout& ly) {
    if (n % TMB == 0) { ly.M = TMB; ly.nrows = TMB + 2; return false; }
    if (n < TMB && TMB % n == 0 && n >= 32) { ly.M = n; ly.nrows = (TMB / n) * (n + 2); return false; }
    ly.M = TMB; ly.nrows = TMB + 2;
    return true;
}

int num_cus();   // block_fwd_bf16.hip

__device__ __forceinline__ int frow(int c, const Layout& ly) {   // image row of column c
    return (c / ly.M) * (ly.M + 2) + 1 + (c % ly.M);
}

// time offset of image row L from the tile's base time (unmasked layouts):
//   one segment: rows are positions p0-1 .. p0+128 of one sub-sequence, t = tb + (L-1) d
//   segments of M = n: row (s, k) is position k-1 of sub-sequence j0 + s, t = tb + (k-1) d + s
__device__ __forceinline__ int row_toff(int L, const Layout& ly, int d) {
    if (ly.M == TMB) return (L - 1) * d;
    const int s = L / (ly.M + 2), k = L - s * (ly.M + 2);
    return (k - 1) * d + s;
}

struct Tile { int b, p0, tb; };   // clip, first position, base time (unmasked layouts)

template <bool MASKED>
__device__ __forceinline__ Tile tile_at(int tl, int tiles, int n, int d, const Layout& ly) {
    Tile t;
    t.b = tl / tiles;
    t.p0 = (tl - t.b * tiles) * TMB;
    t.tb = MASKED ? 0 : (ly.M == TMB ? (t.p0 % n) * d + t.p0 / n : t.p0 / n);
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

__device__ __forceinline__ uint4 relu8(uint4 v) {
    return make_uint4(relu2(v.x), relu2(v.y), relu2(v.z), relu2(v.w));
}

__device__ __forceinline__ uint4 lds16(const uint8_t* p) { return *reinterpret_cast<const uint4*>(p); }
// 16-B global load returned by value (an aggregate copy into a register array can leave the
// array in scratch)
__device__ __forceinline__ uint4 ld16(const u16* p) { return *reinterpret_cast<const uint4*>(p); }

// 16 B per lane HBM -> LDS at lds_base + 16 * lane (global_load_lds_dwordx4).  Inline asm so the
// compiler neither counts it nor drains it with vmcnt(0) before unrelated LDS reads: the kernels
// wait for it explicitly (cdna_hip_programming.md §5.7).
__device__ __forceinline__ void dma16(const void* src, uint32_t lds_base) {
    uint32_t keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
                 "global_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(src), "s"(lds_base) : "memory");
}

// One wave's share of a tile image: group g = w + 4 j (j < DPW) covers image bytes
// [1024 g, 1024 g + 1024); this lane's 16 B of it land at row L, chunk qc (qc == 16 is the pad
// slot, filled with a harmless re-read of chunk 0).
template <bool MASKED>
struct ImageDma {
    int soff[DPW];       // source element offset from the tile's base row (unmasked layouts)
    int scls[DPW];       // source class: 0 row, 1 zero, 2 left halo, 3 right halo
    int srow[DPW], schk[DPW];
    const u16* base;     // per tile (aim)
    uint32_t vmask;      // classes with a real source row
    Tile t;

    __device__ __forceinline__ void init(int w, int lane, const Layout& ly, int d) {
#pragma unroll
        for (int j = 0; j < DPW; ++j) {
            const int g = w + 4 * j;
            const int o = g * 1024 + lane * 16;
            const int L = o / RSB, qc = (o - L * RSB) >> 4;
            const int ch = qc < 16 ? qc : 0;
            srow[j] = L;
            schk[j] = ch;
            int cls = 0;
            if (L >= ly.nrows) cls = 1;
            else if (ly.M == TMB) cls = L == 0 ? 2 : (L == TMB + 1 ? 3 : 0);
            else {
                const int k = L % (ly.M + 2);
                cls = (k == 0 || k == ly.M + 1) ? 1 : 0;
            }
            scls[j] = cls;
            soff[j] = MASKED || cls == 1 ? 0 : row_toff(L, ly, d) * C + ch * 8;
        }
    }
    // point the slots at tile nt of src ([B][T][C])
    __device__ __forceinline__ void aim(const u16* src, const Tile& nt, const Layout& ly, int T, int n) {
        t = nt;
        vmask = 1u;
        if (!MASKED && ly.M == TMB) {
            const int m0 = nt.p0 % n;
            vmask |= (m0 > 0 ? 4u : 0u) | (m0 + TMB < n ? 8u : 0u);
        }
        base = src + ((size_t)nt.b * T + nt.tb) * C;
    }
    __device__ __forceinline__ void issue(int j, const u16* src, const u16* zero, uint32_t lds0,
                                          int T, int n, int d) const {
        const u16* p = zero;
        if (MASKED) {
            const int pp = t.p0 + srow[j] - 1;
            if (scls[j] != 1 && pp >= 0 && pp < T)
                p = src + ((size_t)t.b * T + (pp % n) * d + pp / n) * C + schk[j] * 8;
        } else if ((vmask >> scls[j]) & 1u) {
            p = base + soff[j];
        }
        dma16(p, lds0 + j * 4096);
    }
};

// The staging rows are written and read by different lanes: a wave-scope fence keeps the
// compiler from hoisting one lane's read above another lane's write (or sinking a write above a
// read), which per-thread program order alone does not forbid.
__device__ __forceinline__ void wave_fence() { __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront"); }

// tied no-op: pins a fragment to the accumulator register file (MFMA A operands may be AGPRs).
// The load before it stays a plain, compiler-counted load.
__device__ __forceinline__ uint4 to_agpr(uint4 v) {
    u32x4 t = __builtin_bit_cast(u32x4, v);
    asm volatile("" : "=a"(t) : "0"(t));
    return __builtin_bit_cast(uint4, t);
}

// identity A fragment sg: element e of lane (r, h) is 1 iff r == 16 sg + 8 h + e, so
// mfma(identity_frag(sg), B fragment of k-block 2 q + sg) adds those 16 channels of a row to
// 32-channel tile q (exact: bf16 x 1.0 into fp32)
__device__ __forceinline__ uint4 identity_frag(int sg, int r, int h) {
    const int e = r - 16 * sg - 8 * h;
    uint32_t dw[4];
#pragma unroll
    for (int k = 0; k < 4; ++k)
        dw[k] = (e == 2 * k ? 0x3f80u : 0u) | (e == 2 * k + 1 ? 0x3f800000u : 0u);
    return make_uint4(dw[0], dw[1], dw[2], dw[3]);
}

// accumulator tile (32 channels x 32 columns, fp32) -> 8 packed bf16 dwords
__device__ __forceinline__ void pack_tile(const f32x16& acc, uint32_t (&o)[8]) {
#pragma unroll
    for (int k = 0; k < 8; ++k) o[k] = pack2(acc[2 * k], acc[2 * k + 1]);
}
// half-wave swap (guide T21): afterwards lane (n, h) holds 16-B chunks 4 q + 2 gp + h (gp = 0, 1)
// of row n of 32-channel tile q, in natural channel order
__device__ __forceinline__ void swap_tile(const uint32_t (&o)[8], uint4 (&opk)[2]) {
#pragma unroll
    for (int gp = 0; gp < 2; ++gp) {
        const int g = 2 * gp;
        auto sx = __builtin_amdgcn_permlane32_swap(o[2 * g], o[2 * g + 2], false, false);
        auto sy = __builtin_amdgcn_permlane32_swap(o[2 * g + 1], o[2 * g + 3], false, false);
        opk[gp] = make_uint4(sx[0], sy[0], sx[1], sy[1]);
    }
}

// word q of a lane's [4 q] u16 mask words
__device__ __forceinline__ uint32_t mask_word(uint2 v, int q) {
    return ((q < 2 ? v.x : v.y) >> (16 * (q & 1))) & 0xffffu;
}
// zero the elements of one lane's accumulator tile whose bit mbit(i) of mask word wd is clear
__device__ __forceinline__ void apply_mask(f32x16& acc, uint32_t wd) {
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        const int s = ((int)(wd << (31 - mbit(i)))) >> 31;   // v_bfe_i32
        acc[i] = __int_as_float(__float_as_int(acc[i]) & s);
    }
}

}  // namespace cw
}  // namespace ast
