// Shared definitions for the gfx950 kernels of libastyle.so.
//
// Data layout in HBM (per context, B clips of T samples, C = 128 channels):
//   act   [NB+1][B][T][C]   encoder tensors e_0 (startconv) .. e_NB; e_{l+1} = extracts[l]
//                           (model.py:116); channels-last so a time row is one 512-B line
//                           group (fp32).  Tapped tensors are overwritten in place by their
//                           direct loss gradient D during the Gram backward.
//   mu/me [NB][B][T][4]     u>0 / e_l>0 relu masks, one bit per channel (16 B per row);
//                           fp32 kernels index them by time, channel c at bit c.  bf16 kernels
//                           index them by the layer's time_to_batch position (a tile's masks
//                           are one contiguous run) as u16 words [h][q] in the 32x32 MFMA
//                           accumulator layout: bit i of word (h, q) is channel
//                           32 q + (i & 3) + 8 (i >> 2) + 4 h
//   chain [2][B][T][C]      backward ping-pong, storage type (d loss / d e_l; the bf16 chain
//                           has the direct loss gradient D_l already added)
// Dilated rows are visited in time_to_batch order (masked.py:57-86): tile position p maps to
// time t = (p % n) * d + p / n with n = T / d, so a tile's tap neighbours are p-1 / p+1 and
// the halo is 2 rows at every dilation.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stddef.h>

namespace ast {

constexpr int C = 128;
constexpr int TM = 64;        // rows per encoder tile
constexpr int XS = 130;       // LDS row stride (floats): ds_read_b64 conflict-free

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef unsigned short u16;                 // raw bf16 storage
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef short s16x2 __attribute__((ext_vector_type(2)));

// Diagnostic phase stamps (guide: In-kernel stamps).  Only -DASTYLE_STAMPS builds execute
// them; cycle deltas per phase are summed per wave and added to a.stamps[phase] at exit.  Slot
// 15 takes the wave's lifetime in s_memrealtime ticks (100 MHz): shader cycles / ticks x 100 MHz
// is the clock the kernel actually ran at.
#ifdef ASTYLE_STAMPS
#define STAMP_DECL unsigned long long st_acc[16] = {}; unsigned long long st_prev = stamp_now(); \
    const unsigned long long st_rt0 = __builtin_amdgcn_s_memrealtime();
#define STAMP(k) { const unsigned long long st_t = stamp_now(); st_acc[k] += st_t - st_prev; st_prev = st_t; }
#define STAMP_FLUSH(ptr) if (((threadIdx.x & 63) == 0) && (ptr)) { \
    st_acc[15] = __builtin_amdgcn_s_memrealtime() - st_rt0; \
    for (int k = 0; k < 16; ++k) atomicAdd(&(ptr)[k], st_acc[k]); \
    atomicMax(&(ptr)[16], st_acc[15]); atomicMin(&(ptr)[17], st_acc[15]); \
    atomicMin(&(ptr)[18], st_rt0); atomicMax(&(ptr)[19], st_rt0 + st_acc[15]); }
__device__ __forceinline__ unsigned long long stamp_now() {
    unsigned long long t;
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t) :: "memory");
    __builtin_amdgcn_sched_barrier(0);
    return t;
}
#else
#define STAMP_DECL
#define STAMP(k)
#define STAMP_FLUSH(ptr)
#endif

// bf16 path (precision 1) tile geometry
constexpr int TMB = 128;      // positions per encoder tile (colwave.h)

__device__ __forceinline__ float bf2f(u16 v) { return __uint_as_float((uint32_t)v << 16); }
__device__ __forceinline__ float bflo(uint32_t v) { return __uint_as_float(v << 16); }
__device__ __forceinline__ float bfhi(uint32_t v) { return __uint_as_float(v & 0xffff0000u); }
typedef float f32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t pack2(float a, float b) {   // RNE, one v_cvt_pk_bf16_f32
    const f32x2 x = {a, b};
    return __builtin_bit_cast(uint32_t, __builtin_convertvector(x, bf16x2));
}
__device__ __forceinline__ u16 f2bf(float a) { return (u16)(pack2(a, 0.f) & 0xffffu); }
__device__ __forceinline__ uint32_t relu2(uint32_t u) {         // bf16 relu == int16 max(v, 0)
    s16x2 v = __builtin_bit_cast(s16x2, u);
    v = __builtin_elementwise_max(v, (s16x2){0, 0});
    return __builtin_bit_cast(uint32_t, v);
}
// relu-mask word of one lane's 32x32 accumulator tile (bf16 path): bit mbit(i) = element i > 0
// for the 16 elements held as 8 packed bf16 dwords (element 2k = low half of dword k).  The bit
// order is the one pos_bits16 produces cheaply: 4 (i & 3) + (i >> 2).
__host__ __device__ constexpr int mbit(int i) { return 4 * (i & 3) + (i >> 2); }
__device__ __forceinline__ uint32_t pos_bits16(const uint32_t (&x)[8]) {
    // x - 1 with int16 saturation has its sign bit clear iff x > 0 (bf16 -0 = 0x8000 saturates)
    uint32_t t[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        const s16x2 v = __builtin_elementwise_sub_sat(__builtin_bit_cast(s16x2, x[k]), (s16x2){1, 1});
        t[k] = __builtin_bit_cast(uint32_t, v);
    }
    // bytes [t0.b1 t0.b3 t1.b1 t1.b3]: bit 7 of byte m = NOT(element 4j + m > 0)
    uint32_t z = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const uint32_t y = __builtin_amdgcn_perm(t[2 * j + 1], t[2 * j], 0x07050301u) & 0x80808080u;
        z |= y >> (7 - j);                       // bit j of byte m
    }
    z ^= 0x0f0f0f0fu;                            // element 4j + m at bit 8m + j
    const uint32_t u = z | (z >> 4);             // bytes 0, 2 hold nibbles (m = 0,1), (m = 2,3)
    return __builtin_amdgcn_perm(u, u, 0x0c0c0200u);
}

__device__ __forceinline__ f32x16 mfma_bf16(uint4 a, uint4 b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, a),
                                                    __builtin_bit_cast(bf16x8, b), c, 0, 0, 0);
}
// generic element access for kernels templated on the storage type (float | u16 = bf16)
// ae_startconv of one element (model.py:82-93): e_0[t][c] = b0[c] + sum_k W0[k][c] x[t + k - 1] / 128
// with x[-1] = x[T] = 0 (SAME).  One fixed operation order, shared by k_startconv_fwd (masks and
// max) and the split block-0 forward that recomputes e_0 from x (the two must agree bit for bit)
__device__ __forceinline__ float e0_val(float w0, float w1, float w2, float b, float xm, float x0, float xp) {
    return fmaf(w2, xp * 0.0078125f, fmaf(w1, x0 * 0.0078125f, w0 * (xm * 0.0078125f))) + b;
}

__device__ __forceinline__ float ldv(const float* p, size_t i) { return p[i]; }
__device__ __forceinline__ float ldv(const u16* p, size_t i) { return bf2f(p[i]); }
__device__ __forceinline__ void stv(float* p, size_t i, float v) { p[i] = v; }
__device__ __forceinline__ void stv(u16* p, size_t i, float v) { p[i] = f2bf(v); }

struct FwdArgs {
    const float* ein; float* eout;
    const float* wd;  const float* bd;     // wd [3][ci][co]
    const float* wr;  const float* br;     // wr [ci][co]
    uint32_t* mu; uint32_t* me;
    int B, T, d, n;
};

struct BwdArgs {
    const float* gin; const float* din; float* gout;
    const float* wr;   // [ci][co]
    const float* wrT;  // [co][ci]
    const float* wdT;  // [3][co][ci]
    const uint32_t* mu; const uint32_t* me;
    int B, T, d, n;
};

// column-owning bf16 block forward (block_fwd_bf16.hip)
struct FwdArgsC {
    unsigned long long* stamps;            // diagnostic builds (-DASTYLE_STAMPS) only
    const u16* ein; u16* eout;
    const u16* wf;         // [3 taps][4 q][8 kb][64 lanes][8] W_d^T A fragments
    const u16* wrf;        // [4 q2][8 s][64][8] W_r^T A fragments, K in accumulator order
    const float* bd; const float* br;
    uint16_t* mu;          // [B*T][2 h][4 q] u > 0 bits, this layer's positions
    uint16_t* me_next;     // [B*T][2][4] e_{l+1} > 0 bits, the next layer's positions (or null)
    const u16* zero;       // >= 256 zero bytes
    int B, T, d, n;        // dilation, n = T / d
    int dn_log2, nn;       // next layer: log2 dilation, T / dilation
};

// column-owning bf16 block backward (block_bwd_bf16.hip)
struct BwdArgsC {
    unsigned long long* stamps;            // diagnostic builds (-DASTYLE_STAMPS) only
    const u16* tin;        // d loss / d e_{l+1} incl. its direct term (chain, or D_{l+1} at the top)
    const u16* dadd;       // D_l, the direct loss gradient of e_l (or null)
    u16* gout;             // d loss / d e_l incl. D_l
    const u16* wbf;        // [3 taps][4 q][8 kb][64 lanes][8] W_d A fragments:
                           //   lane (m, h) element e = W_d[tap][ci = 32 q + m][co = 16 kb + 8 h + e]
    const u16* wrb;        // [4 q][8 kb][64][8] W_r A fragments: W_r[co = 32 q + m][o = 16 kb + 8 h + e]
    const uint16_t* mu;    // [B*T][2 h][4 q] u > 0 bits, this layer's positions
    const uint16_t* me;    // [B*T][2][4] e_l > 0 bits, this layer's positions
    const u16* zero;       // >= 256 zero bytes
    int B, T, d, n;        // dilation, n = T / d
};

// split-fp16 block kernels (precision 2: block_fwd_split.hip, block_bwd_split.hip).  Weight
// fragments are fp16 halves of W 2^k (k = kd / kr per block, host-chosen), 8 halves per lane:
//   wdf [4 w][3 tap][8 kb][2 hl][64 lanes]: lane (m, h) element e = W_d[tap][16 kb + 8 h + e][32 w + m]
//   wrf [4 w][8 kb][2 hl][64]:                                     W_r[16 kb + 8 h + e][32 w + m]
//   wrb [4 w][8 kb][2 hl][64]:                                     W_r[32 w + m][16 kb + 8 h + e]
//   wdb [4 w][3 tap][8 kb][2 hl][64]:                              W_d[tap][32 w + m][16 kb + 8 h + e]
// ASTYLE_MFMA16=1 (the 16x16x32 kernels, block_*_split16.hip): the same arrays hold 16x16x32 A
// fragments, slot s = 2 kb + rb (K block kb of 32, row block rb), lane (i, q) = (lane & 15, lane >> 4):
//   wdf: W_d[tap][32 kb + 8 q + e][32 w + 16 rb + i]     wrf: W_r[32 kb + 8 q + e][32 w + 16 rb + i]
//   wrb: W_r[32 w + 16 rb + i][32 kb + 8 q + e]          wdb: W_d[tap][32 w + 16 rb + i][32 kb + 8 q + e]
// gmax_*: per clip max |x| of a tensor as float bits (atomic max of the non-negative bit pattern),
// in GSLOTS slots per clip, one 128-B line each ([level][clip][slot][32 words], word 0 used): a
// writer takes slot blockIdx.x % GSLOTS (one per XCD under round-robin placement), a reader the
// max of the slots (round 6: at one clip every workgroup of a block launch ends on the same clip,
// and 256 atomics on one line serialised ~2 us per launch).
constexpr int GSLOTS = 8;
constexpr int GSLOT_W = 32;                 // words per slot
constexpr int GCLIP_W = GSLOTS * GSLOT_W;   // words per clip and level
__host__ __device__ inline unsigned* gslot(unsigned* lvl, int b, unsigned slot) {
    return lvl + (size_t)b * GCLIP_W + (slot % GSLOTS) * GSLOT_W;
}
// Division by a launch-invariant divisor without the signed-division expansion (~17 scalar
// instructions each): q = mulhi(x, m) >> s with m = ceil(2^(31 + l) / n), 2^l >= n, exact for
// every 0 <= x < 2^31 (Granlund-Montgomery); n = 1 passes x through.
struct FDiv {
    uint32_t n, m, s;
};
inline FDiv make_fdiv(uint32_t n) {
    FDiv f{n, 0u, 0u};
    if (n > 1) {
        uint32_t l = 0;
        while ((1ull << l) < n) ++l;
        f.m = (uint32_t)(((1ull << (31 + l)) + n - 1) / n);
        f.s = l - 1;
    }
    return f;
}
__device__ __forceinline__ uint32_t fdiv(uint32_t x, const FDiv& f) {
    return f.n == 1 ? x : __umulhi(x, f.m) >> f.s;
}

struct FwdArgsS {
    unsigned long long* stamps;            // diagnostic builds (-DASTYLE_STAMPS) only
    const float* ein; float* eout;
    const uint4* wdf; const uint4* wrf;
    const float* bd; const float* br;
    uint16_t* mu;          // [B*T][2 h][4 w] u > 0 bits, this layer's positions
    uint16_t* me_next;     // [B*T][2][4] e_{l+1} > 0 bits, the next layer's positions (or null)
    const float* gmax_in;  // [B] max |e_l|
    unsigned* gmax_out;    // [B] max |e_{l+1}| (atomic)
    const float* zero;     // >= 16 zero bytes
    int B, T, d, n;        // dilation, n = T / d
    int dn_log2, nn;       // next layer: log2 dilation, T / dilation
    int kd, kr;            // weight exponents
    float wdn, bdm;        // max_co sum_{tap,ci} |W_d|, max |b_d|: |u| <= wdn max|e_l| + bdm
    int cus;               // workgroups (CUs) the persistent grid may use; 0 = every CU
    // block 0 with the start conv folded in (xin non-null): e_l = e_0 is recomputed from the
    // audio xin [B][T] and W0 [3][C], b0 [C] (e0_val) instead of read from ein
    const float* xin; const float* w0; const float* b0;
    FDiv fn, ft;           // by n; by B (or T / 64: splitwave.h tile order): set by the launcher
};

struct BwdArgsS {
    unsigned long long* stamps;            // diagnostic builds (-DASTYLE_STAMPS) only
    const float* tin;      // d loss / d e_{l+1} incl. its direct term
    const float* dadd;     // D_l (or null)
    float* gout;           // d loss / d e_l incl. D_l
    const uint4* wrb; const uint4* wdb;
    const uint16_t* mu; const uint16_t* me;
    const float* gmax_in;  // [B] max |tot|
    unsigned* gmax_out;    // [B] max |out| (atomic)
    const float* zero;
    int B, T, d, n;
    int kd, kr;
    float wrn;             // max_ci sum_co |W_r|: |W_r tot| <= wrn max|tot|
    int cus;               // workgroups (CUs) the persistent grid may use; 0 = every CU
    // block 0 with the start conv's backward folded in (spart non-null): instead of gout, per
    // position and wave the three dot products sum_c W0[k][c] out[t][c] over the wave's 32
    // channels -> spart [B][T][4 waves][4] (k = 0..2; launch_startx_gx forms d loss / d x)
    const float* w0; float* spart;
    FDiv fn, ft;           // by n; by B (or T / 64: splitwave.h tile order): set by the launcher
};

struct GramArgs {
    const void* act; size_t tstride;       // tensor u lives at act + uid[u] * tstride elements
    void* actw;                             // same base, writable (bwd, in place)
    int nu; int uid[32];
    const void* cg[32];                     // content grad per unique tensor (bwd) or null
    float* gpart;                           // [B][nchunk][C][32][32]
    const float* smat;                      // [B][C][32][32]
    const void* zero16;                     // >= 16 zero bytes
    int B, T, nchunk;
    int top_u;                              // split bwd: unique tensor whose per-clip max |D| ...
    unsigned* gmax_top;                     // ... goes to gmax_top[b] (atomic max of float bits), or -1
    // split bwd, fused content tap (methods.py:116-117): for unique tensor cont_u (or -1) D +=
    // coef (E - phi[..., off + c]) on channels c < ncol, in place of k_content's cg buffer round
    // trip; the squared errors of every GRAM_CSLOT rows of a workgroup go to cont_part[b * cont_pstride + slot *
    // (C / 32) + channel group]
    int cont_u;
    const float* cont_phi; size_t cont_phi_bstride;
    int cont_ncc, cont_off, cont_ncol;
    float cont_coef;
    float* cont_part; size_t cont_pstride;
};

struct StyleArgs {
    const float* gpart; int nchunk;
    int L; int lmap[32]; int nu;
    int lmap_identity;                      // lmap[i] == i for every tap (no S~ fold needed)
    const float* phi; size_t phi_bstride;   // elements between clips (0 = shared)
    int nb; float coef;                     // coef = lambd * 1e3 * 2 / (nb * L * L)
    float* smat; float* spart;              // [B][C][32][32], [B][C]
    float* embs;                            // optional normalised Gram out [B][nb][L][L]
    int B;
};

// Gatys Gram (methods.py:70-72 with --gatys): G_u = E_u^T E_u [C][C] per unique tensor.
struct GatysArgs {
    const void* act; void* actw; size_t tstride;
    int nu; int uid[32];
    const void* cg[32];                     // content grad per unique tensor (bwd) or null
    float* gpart;                           // [B][nchunk][nu][C][C]
    const float* smat;                      // [B][nu][C][C]  S~ = sum_l dG_l + dG_l^T (fp32)
    const u16* smatb;                       // same, bf16 (precision 1)
    int B, T, nchunk;
    // split bwd, fused content tap (as GramArgs): tensor cont_u (or -1) gets coef (E - phi) on its
    // channels < cont_ncol; each workgroup's squared error goes to cont_part[b * cont_pstride + tile]
    int cont_u;
    const float* cont_phi; size_t cont_phi_bstride;
    int cont_ncc, cont_off, cont_ncol;
    float cont_coef;
    float* cont_part; size_t cont_pstride;
    int top_u;                              // split bwd: tensor whose per-clip max |D| (the backward
    unsigned* gmax_top;                     // chain's first input) goes to gmax_top[b], or -1
};

struct GatysStyleArgs {
    const float* gpart; int nchunk;
    int L; int lmap[32]; int nu;
    const float* phi; size_t phi_bstride;   // [B|1][L][C][C]
    float coef;                             // lambd * 1e3 * 2 / (L * C * C)
    float* smat; u16* smatb; float* spart;  // [B][nu][C][C] (x2), [B][nu]
    float* embs;                            // optional normalised Gram out [B][L][C][C]
    int B;
};

struct ContentArgs {
    const void* e; int W;                   // tensor [B][T][W] (float, or bf16 when e_bf16)
    int e_bf16, cg_bf16;
    const float* phi; size_t phi_bstride;   // [B|1][T][ncc]
    int ncc, off, ncol;
    float coef;                             // 10 * 2 / (T * ncc)
    void* cg; int accumulate;               // [B][T][W] (float, or bf16 when cg_bf16)
    float* lpart; size_t lstride;           // partial sums at lpart[b * lstride + tile]
    float* embc;                            // optional: write e[..., :ncol] into emb [B][T][ncc]
    int B, T;
};

// launchers (encoder.hip / gram.hip / optim.hip)
template <typename S>
void launch_startconv_fwd(const float* x, S* e0, const float* w0, const float* b0,
                          int B, int T, hipStream_t s, uint16_t* me0 = nullptr,
                          unsigned* gmax = nullptr);
// split mode: only the e_0 > 0 words and the per-clip max |e_0| (block 0 recomputes e_0)
void launch_startconv_masks(const float* x, const float* w0, const float* b0, int B, int T,
                            hipStream_t s, uint16_t* me0, unsigned* gmax);
void launch_startx_gx(const float* spart, float* gx, int B, int T, hipStream_t s);
// bytes: a multiple of 4; site: which clear (0 gmax_e, 1 content partials, 2 gmax_g, 3 range
// flags), used only by the tools-only memset build's per-site selection (ASTYLE_MEMSET_SITES)
void launch_zero32(void* p, size_t bytes, hipStream_t s, int site = -1);
template <typename S>
void launch_startconv_bwd(const S* g0, float* gx, const float* w0, int B, int T,
                          hipStream_t s);
void launch_block_fwd(const FwdArgs& a, hipStream_t s);
void launch_block_bwd(const BwdArgs& a, hipStream_t s);
void launch_block_fwd_c(const FwdArgsC& a, hipStream_t s);
void launch_block_bwd_c(const BwdArgsC& a, hipStream_t s);
void launch_block_fwd_s(const FwdArgsS& a, hipStream_t s);
void launch_block_fwd_s16(const FwdArgsS& a, hipStream_t s);   // ASTYLE_MFMA16=1
void launch_block_bwd_s(const BwdArgsS& a, hipStream_t s);
void launch_block_bwd_s16(const BwdArgsS& a, hipStream_t s);   // ASTYLE_MFMA16=1
void launch_absmax(const float* x, size_t per_clip, int B, unsigned* out, hipStream_t s);
template <typename S>
void launch_bottleneck_fwd(const S* e, float* y, const float* wb, const float* bb,
                           int B, int T, hipStream_t s);
template <typename S>
void launch_bottleneck_bwd(const float* gy, S* ge, const float* wb, int accumulate,
                           int B, int T, hipStream_t s);
void launch_to_f32(const u16* src, float* dst, size_t n, hipStream_t s);
void launch_gram_fwd_bf16(const GramArgs& a, hipStream_t s);
void launch_gram_bwd_bf16(const GramArgs& a, hipStream_t s);
void launch_gram_fwd(const GramArgs& a, hipStream_t s);
void launch_gram_fwd_s(const GramArgs& a, hipStream_t s);   // precision 2: bf16 MFMA, fp32 E
void launch_gram_bwd_s(const GramArgs& a, hipStream_t s);
void launch_gram_bwd(const GramArgs& a, hipStream_t s);
void launch_style_ours(const StyleArgs& a, hipStream_t s);
void launch_gatys_fwd(const GatysArgs& a, int precision, hipStream_t s);   // 0 fp32, 1 bf16, 2 split
void launch_gatys_bwd(const GatysArgs& a, int precision, hipStream_t s);
void launch_style_gatys(const GatysStyleArgs& a, hipStream_t s);
constexpr int GY_ROWS = 512;    // Gatys bwd: time rows per workgroup
void launch_content(const ContentArgs& a, hipStream_t s);
constexpr int CROWS = 64;   // rows per content workgroup
static_assert(GY_ROWS >= CROWS, "the fused Gatys content tap's T / GY_ROWS slots fit ncpart = T / CROWS");
constexpr int GRAM_CSLOT = 256;   // rows per content-error slot of the fused split Gram backward
static_assert((512 / GRAM_CSLOT) * 4 == 512 / CROWS, "fused content slots fill ncpart of one occurrence");
void launch_finalize(float* parts, const float* cpart, int ncpart, float cscale,
                     const float* spart, int nspart, float sscale, float lambd, int B,
                     hipStream_t s);
// per-clip range / finiteness flags of one loss+grad evaluation (gram.hip, ast_range_flags)
struct RangeArgs {
    const float* parts; const float* grad;  // [B][4], [B][T]
    const unsigned* gmax_e; const unsigned* gmax_g;   // split: [nblk + 1][B][GCLIP_W] per-clip maxima
    int split, nblk, B, T;
    float wdn[30], bdm[30], wrn[30];        // split: the per-block operand bounds (splitwave.h)
    int* flags;                             // [B] OR'ed (sticky)
    int* last;                              // [B] this evaluation's alone
};
void launch_range_flags(const RangeArgs& a, hipStream_t s);

// b^n by squaring: the same fp32 products on host and device, so the host-counter and the
// device-counter Adam steps agree bit for bit
__host__ __device__ inline float pow_int(float b, int n) {
    float r = 1.f;
    while (n > 0) {
        if (n & 1) r *= b;
        b *= b;
        n >>= 1;
    }
    return r;
}

// STFT regulariser (stft_reg.hip, methods.py:121-123): frames of 1024 / hop 512
int stft_frames(int T);
void launch_stft_twiddles(float2* tw, hipStream_t s);
void launch_stft_reg(const float* x, const float2* tw, float* fpart, float* gfr, float* grad,
                     float* parts, float gamma, int B, int T, hipStream_t s);

// batched device L-BFGS-B (lbfgs.hip, methods.py:132-137)
size_t lbfgs_workspace_bytes(int B, int T, int m);
void launch_lbfgs_begin(void* ws, float* x, const double* x0, const int* active, int B, int T,
                        int m, int maxiter, int maxls, double tol, double pgtol, hipStream_t s);
void launch_lbfgs_step(void* ws, float* x, const float* grad, const float* parts, int B, int T,
                       hipStream_t s);
void launch_lbfgs_state(const void* ws, int* info, double* x64, int B, int T, hipStream_t s);
int lbfgs_history_cap();
void launch_lbfgs_history(const void* ws, float* out, int cap, int B, int T, hipStream_t s);

void launch_adam(float* x, float* m, float* v, const float* g, size_t n, float lr, float b1,
                 float b2, float eps, float bc1, float bc2, hipStream_t s);
void launch_adam_dev(float* x, float* m, float* v, const float* g, size_t n, int* step_dev,
                     float lr, float b1, float b2, float eps, hipStream_t s);

// batched ADMM optimal transport between palettes (ot_admm.hip, optimal_transport.py:77-162)
size_t ot_lds_bytes(int n1, int n2);
int ot_max_cells();   // register kernel limit; larger problems run k_ot_admm_big
size_t ot_big_lds_bytes(int n1, int n2);
size_t ot_big_ws_bytes(int n1, int n2);   // per problem
void launch_ot_admm_big(const double* p_mod, const double* p_ref, int nprob, int n1, int n2, int d,
                        double eps, double miter, double* ws, double* plan, double* pal, int* iters,
                        hipStream_t s);
void launch_ot_admm(const double* p_mod, const double* p_ref, int nprob, int n1, int n2, int d,
                    double eps, double miter, double* plan, double* pal, int* iters, hipStream_t s);

}  // namespace ast
