// C ABI of libastyle.so (declared in include/astyle.h; reference interfaces cited there).
// Owns the per-device context: weights, activation workspace, tap bookkeeping, and the
// launch sequence of one loss+grad evaluation (methods.py:113-137 evaluated as
// ScipyOptimizerInterface does, methods.py:167).
#include <hip/hip_runtime.h>
#include <stdlib.h>
#include <string.h>
#include <stdio.h>
#include <string>
#include <vector>
#include <algorithm>
#include <cmath>

#include "../../include/astyle.h"
#include "common.h"
#include "ckpt.h"

using namespace ast;

namespace {

thread_local std::string g_err;
unsigned long long* g_stamps = nullptr;   // diagnostic phase stamps (ASTYLE_STAMPS builds)
static int g_stamp_row = 0;               // block launches since ast_debug_stamps: row of 20 words each
static unsigned long long* stamp_row() {  // (64 rows; a launch's max / min wave lifetime in its row)
    return g_stamps ? g_stamps + 20 * (g_stamp_row++ & 63) : nullptr;
}

int fail(int code, const std::string& msg) {
    g_err = msg;
    return code;
}

#define HIPCHK(expr)                                                                     \
    do {                                                                                 \
        hipError_t _e = (expr);                                                          \
        if (_e != hipSuccess)                                                            \
            return fail(AST_E_HIP, std::string(#expr) + ": " + hipGetErrorString(_e));  \
    } while (0)

constexpr int NBLK_MAX = 30;
constexpr int NFAM = 5;   // block fwd, block bwd, gram fwd, gram bwd, other

// weight offsets (floats) inside one device allocation
constexpr size_t W0_OFF = 0;                  // [3][128]
constexpr size_t B0_OFF = W0_OFF + 3 * C;     // [128]
constexpr size_t BLK_OFF = B0_OFF + C;
constexpr size_t WD = 0, WDT = 3 * C * C, BD = 6 * C * C, WR = BD + C, WRT = WR + C * C,
                 BR = WRT + C * C, BLK_SZ = BR + C;
constexpr size_t WB_OFF = BLK_OFF + NBLK_MAX * BLK_SZ;   // [128][16]
constexpr size_t BB_OFF = WB_OFF + C * 16;
constexpr size_t W_TOTAL = BB_OFF + 16;
// bf16 MFMA fragments (precision 1), u16 elements per block.
// MFMA A-fragment order for block_fwd_bf16.hip: WFB [3 taps][4 q][8 kb][64 lanes][8],
// lane (m, h) element e = W_d[tap][ci = 16 kb + 8 h + e][co = 32 q + m];
// WRFB [4 q2][8 s][64][8], element e = W_r[co = kperm(s, h, e)][co2 = 32 q2 + m].
// block_bwd_bf16.hip: WBFB [3][4 q][8 kb][64][8], element e = W_d[tap][32 q + m][16 kb + 8 h + e];
// WRBFB [4 q][8 kb][64][8], element e = W_r[32 q + m][16 kb + 8 h + e]
constexpr size_t WFB = 0, WRFB = 3 * C * C, WBFB = 4 * C * C, WRBFB = 7 * C * C, BLKB_SZ = 8 * C * C;
inline int kperm(int s, int h, int e) { return 32 * (s >> 1) + 16 * (s & 1) + (e & 3) + 8 * (e >> 2) + 4 * h; }
// split-fp16 fragments (precision 2), uint4 (8 fp16) units per block: WDF [4][3][8][2][64],
// WRF [4][8][2][64], WRB [4][8][2][64], WDB [4][3][8][2][64] (common.h, FwdArgsS / BwdArgsS)
constexpr size_t SWDF = 0, SWRF = 4 * 3 * 8 * 2 * 64, SWRB = SWRF + 4 * 8 * 2 * 64,
                 SWDB = SWRB + 4 * 8 * 2 * 64, SBLK = SWDB + 4 * 3 * 8 * 2 * 64;

// power-of-two exponent k that puts max |w| in [2^13, 2^14) (fp16 range, splitwave.h)
int weight_exp(const float* w, size_t n) {
    float mx = 0.f;
    for (size_t i = 0; i < n; ++i) mx = std::max(mx, std::fabs(w[i]));
    if (!(mx > 0.f) || !std::isfinite(mx)) return 0;
    int e = 0;
    (void)std::frexp(mx, &e);
    return 14 - e;
}
// fp16 halves of w 2^k (round to nearest): hi, lo = fp16(w 2^k - hi)
void split_half(float w, int k, uint16_t& hi, uint16_t& lo) {
    const float v = std::ldexp(w, k);
    const _Float16 h = (_Float16)v;
    const _Float16 l = (_Float16)(v - (float)h);
    memcpy(&hi, &h, 2);
    memcpy(&lo, &l, 2);
}

uint16_t host_bf16(float f) {   // round to nearest even
    uint32_t u;
    memcpy(&u, &f, 4);
    u += 0x7fffu + ((u >> 16) & 1u);
    return (uint16_t)(u >> 16);
}

struct Occ { int ext, tensor, off, ncol; };

}  // namespace

namespace ast {
int set_error(int code, const std::string& msg) { return fail(code, msg); }   // ckpt.cpp
}  // namespace ast

struct ast_ctx {
    ast_cfg cfg;
    int dev = 0;
    int cus = 0;                            // persistent block kernels' workgroup budget (0 = every CU)
    bool lg_front_done = false;             // ast_loss_grad_phase: phase 1 ran, phase 2 may follow
    bool lg_top_max_done = false;           // (phase 1 -> 2) the Gram bwd recorded the chain's first max
    int nblk = 0;
    bool need_bott = false;
    int nu = 0, uid[32];
    int L = 0, lmap[32];
    std::vector<Occ> occ;
    int ncc = 0;
    int nchunk = 1;
    int nchunk_b = 1;     // split ours-Gram backward: its own time chunks (see plan())
    void* cg_buf[NBLK_MAX + 1] = {};        // content grad per tensor (or null), storage type
    bool tensor_in_style[NBLK_MAX + 1] = {};
    bool tensor_has_direct_content[NBLK_MAX + 1] = {};
    // device memory
    float* wts = nullptr;
    u16* wtsb = nullptr;                    // bf16 weight copies (precision 1)
    uint4* wtss = nullptr;                  // split-fp16 weight fragments (precision 2)
    int kd[NBLK_MAX] = {}, kr[NBLK_MAX] = {};   // their exponents
    float wdn[NBLK_MAX] = {}, wrn[NBLK_MAX] = {}, bdm[NBLK_MAX] = {};   // operand bounds (splitwave.h)
    bool bf = false;                        // precision 1: bf16 activations/gradients
    bool split = false;                     // precision 2: fp32 storage, split-fp16 block GEMMs
    unsigned* gmax_e = nullptr;             // [nblk + 1][B][GCLIP_W] max |e_l| per clip, in slots (precision 2)
    unsigned* gmax_g = nullptr;             // [nblk + 1][B][GCLIP_W] max |d loss / d e_l| per clip
    size_t esz = 4;                         // bytes per stored element
    void* act = nullptr; size_t tstride = 0;
    void* dgrad = nullptr;   // style-tapped tensors' D out of place (doop; else in place over act)
    bool doop = false;       // decide_doop / timed_gram_bwd: D placement
    bool doop_tune = false;  // both placements open: the first eager evaluation times them
    float doop_ms[2] = {-1.f, -1.f};   // that timing's Gram-backward times (in place, out of place)
    uint32_t* mu = nullptr; uint32_t* me = nullptr;
    void* chain[2] = {};
    float* bott = nullptr; float* gbott = nullptr;
    float* gpart = nullptr; float* smat = nullptr; float* spart = nullptr; float* cpart = nullptr;
    u16* smatb = nullptr;                   // bf16 S~ (Gatys, precision 1)
    float2* stft_tw = nullptr;              // STFT regulariser: twiddles [1024]
    float* stft_fpart = nullptr;            //   per-frame partial sums [B][nf]
    float* stft_gfr = nullptr;              //   per-frame gradients [B][nf][1024]
    std::vector<const void*> lb_ws;         // workspaces started here with x0 (ast_lbfgs_begin)
    void* zero = nullptr;                   // 256 zero bytes
    int* rflags = nullptr;                  // [B] AST_RANGE_* OR'ed over ast_loss_grad calls since the last reset
    int* rflags_last = nullptr;             // [B] AST_RANGE_* of the last ast_loss_grad alone
    size_t gpart_elems = 0, smat_elems = 0; // per context (mode-dependent)
    int ncpart = 0;
    std::vector<void*> allocs;
    struct Guard { char* base; size_t bytes; const char* name; };
    std::vector<Guard> guards;              // ASTYLE_GUARD=1: guard bands around every buffer
    const float* phi_c = nullptr; int phi_c_shared = 0;
    const float* phi_s = nullptr; int phi_s_shared = 0;
    bool targets = false;
    bool fwd_done = false;
    // timing
    bool timing = false;
    std::vector<hipEvent_t> ev;
    int ev_used = 0;
    int timed_calls = 0;
};

namespace {

int ext_to_tensor(int ext) { return ext >= 30 ? 30 : ext + 1; }

// Number of Gram time chunks of a T-sample clip: every chunk a whole number of the kernels'
// `stage`-row stages (the kernels loop stage by stage up to the chunk end), as many chunks as
// divide evenly up to T / `target` (about `target` rows each).  T = 16384: 16 (ours), 4 (Gatys);
// T = 3584: 2 x 1792 rows (T / 1024 = 3 does not divide the 112 stages).
int gram_chunks(int T, int stage, int target) {
    const int stages = T / stage;                     // T is a multiple of 512
    int n = std::max(1, std::min(stages, T / target));
    while (stages % n) --n;
    return n;
}

int plan(const ast_cfg* c, ast_ctx* x) {
    if (c->batch < 1 || c->T < 512 || c->T % 512)
        return fail(AST_E_ARG, "T must be a positive multiple of 512 (masked.py:134,183)");
    if (c->n_cont < 1 || c->n_cont > AST_MAX_TAPS || c->n_style < 1 || c->n_style > AST_MAX_TAPS)
        return fail(AST_E_ARG, "need 1..32 content and style taps");
    if (c->cnt_channels < 1 || c->nb_channels < 1)
        return fail(AST_E_ARG, "cnt_channels / nb_channels must be >= 1");
    if (c->precision < 0 || c->precision > 2)
        return fail(AST_E_ARG, "precision must be 0 (fp32), 1 (bf16) or 2 (split: fp32 storage, split-fp16 MFMA)");
    int top = 0;
    x->need_bott = false;
    x->ncc = 0;
    x->occ.clear();
    for (int i = 0; i < c->n_cont; ++i) {
        const int e = c->cont_ids[i];
        if (e < 0 || e > 31) return fail(AST_E_ARG, "content layer ids must be in 0..31");
        const int tns = ext_to_tensor(e);
        top = std::max(top, tns);
        const int width = e == 31 ? 16 : C;
        const int ncol = std::min(c->cnt_channels, width);
        x->occ.push_back({e, tns, x->ncc, ncol});
        x->ncc += ncol;
        if (e == 31) x->need_bott = true;
        else x->tensor_has_direct_content[tns] = true;
    }
    x->nu = 0;
    x->L = c->n_style;
    for (int i = 0; i < c->n_style; ++i) {
        const int e = c->style_ids[i];
        if (e < 0 || e > 30)
            return fail(AST_E_ARG, "style layer ids must be in 0..30 (extract 31 has 16 channels; "
                                   "tf.concat with 128-channel extracts rejects it)");
        const int tns = ext_to_tensor(e);
        top = std::max(top, tns);
        int u = -1;
        for (int k = 0; k < x->nu; ++k) if (x->uid[k] == tns) u = k;
        if (u < 0) { u = x->nu++; x->uid[u] = tns; }
        x->lmap[i] = u;
        x->tensor_in_style[tns] = true;
    }
    x->nblk = top;
    // every dilation used must divide T (masked.py:134)
    const int maxd = x->nblk >= 10 ? 512 : (1 << (x->nblk - 1));
    if (c->T % maxd) return fail(AST_E_ARG, "T must be a multiple of the largest dilation");
    // Gram time chunks: a fixed length per T, whatever the batch, so a clip's partial sums (and
    // so its result, bit for bit) do not depend on how many clips share the context
    int nch = 1;
    if (c->gatys) {
        // target rows per Gatys chunk (ASTYLE_GATYS_ROWS for A/B): 8192 measured 0.2-0.4 ms / step
        // faster than 4096 (half the [C][C] partials through k_style_gatys), 16384 the same as 8192
        static int grows = -1;
        if (grows < 0) { const char* e = getenv("ASTYLE_GATYS_ROWS"); grows = e ? std::max(512, atoi(e)) : 8192; }
        nch = gram_chunks(c->T, 64, grows);    // whole 64-row stages (bf16 / split; fp32: 32)
        x->gpart_elems = (size_t)c->batch * nch * x->nu * C * C;
        x->smat_elems = (size_t)c->batch * x->nu * C * C;
    } else {
        // target rows per chunk (ASTYLE_GRAM_ROWS for A/B): 4096 measured 0.6 ms / step faster than 1024
        // in the Gram forward and 0.25 ms in k_style_ours (a quarter of the partials), 8192 the same
        static int rows = -1;
        if (rows < 0) { const char* e = getenv("ASTYLE_GRAM_ROWS"); rows = e ? std::max(512, atoi(e)) : 4096; }
        nch = gram_chunks(c->T, 32, rows);     // whole 2 x 16-row split / fp32 stages (bf16: 16)
        x->gpart_elems = (size_t)c->batch * nch * C * 1024;
        x->smat_elems = (size_t)c->batch * C * 1024;
    }
    x->nchunk = nch;
    // The split / fp32 ours-Gram backward (D = S~ E, row-independent) may cut time finer than the
    // forward, whose per-chunk Gram partials fix the summation order: at few clips the
    // forward's chunks leave most CUs idle (one clip: 16 workgroups).  Its only cross-row sums,
    // the fused content tap's squared errors, go to fixed GRAM_CSLOT-row slots, so every
    // result stays independent of the batch.  Chunks: the fewest whole-slot chunks, at least
    // the forward's count, that give >= 1024 workgroups.
    x->nchunk_b = nch;
    if ((c->precision == 2 || c->precision == 0) && !c->gatys) {   // (fp32's k_gram_bwd_f: no cross-row sums)
        const int slots = c->T / GRAM_CSLOT;
        int d = 1;
        for (int k = 1; k <= slots; ++k) {
            if (slots % k) continue;
            d = k;
            if (k >= nch && (size_t)c->batch * k * 4 >= 1024) break;
        }
        x->nchunk_b = d;
    }
    return 0;
}

// Elements between consecutive activation tensors beyond their size (ASTYLE_TPAD overrides the
// default 1 MiB + 4 KiB): at B = 256, T = 16384 a tensor is exactly 2^31 bytes, so without a pad
// the Gram kernels' 30 concurrent streams start at the same offset modulo every power of two
// (measured: Gram forward 13.2 -> 11.1-11.4 ms with the pad).
static size_t tensor_pad() {
    static long pad = -1;
    if (pad < 0) {
        const char* e = getenv("ASTYLE_TPAD");
        pad = e ? atol(e) : 263168;
        if (pad < 0) pad = 0;
        pad = (pad + 127) / 128 * 128;   // whole 512-B rows
    }
    return (size_t)pad;
}

// Where the Gram backward writes D (the direct loss gradients of the style-tapped tensors): to a
// buffer of its own (out of place, +1 activation set of memory) or over E in place.  Round 6 rule
// (DESIGN.md §2): out of place whenever the workspace with it leaves
// max(16 GiB, 10 %) of the device's memory free, in place otherwise (B > ~480 clips of 16384 on
// a 288-GB MI355X).  Out of place ran 23.8-24.1 ms in 9 of 9 processes in round 3, where in place
// ran 26.8-27.1 ms in 19 of 22 (the DRAM credit stalls of the write-over-read pattern); in round 5
// one box of five ran every in-place Gram backward at 27.1-27.3 ms; on fast boxes the two modes are
// within +-0.4 ms (round 5 and 6 A/Bs).  ASTYLE_DOOP=1 / 0 forces either mode (A/B runs).
static int doop_env() {
    static int v = -2;
    if (v == -2) { const char* e = getenv("ASTYLE_DOOP"); v = e ? (atoi(e) != 0) : -1; }
    return v;
}
// Byte offset of the D buffer inside its allocation (ASTYLE_DPAD, A/B of the Gram backward's
// read / write address interplay; a multiple of 256)
static size_t d_pad() {
    static long v = -1;
    if (v < 0) { const char* e = getenv("ASTYLE_DPAD"); v = e ? (std::max(0L, atol(e)) / 256) * 256 : 0; }
    return (size_t)v;
}

int fused_content_occ(const ast_ctx* x);

// ASTYLE_MFMA16: the split block kernels on v_mfma_f32_16x16x32_f16 (block_*_split16.hip, round 6:
// measured): 0 = neither, 1 = forward and backward, 2 = the backward only (default:
// backward -0.3..-1.2 %, forward +4 % on 16x16x32), 3 = the forward only; read once per process, since the weight fragments are packed for the kernels that will read them
static int mfma16_mode() {
    static int v = -1;
    if (v < 0) { const char* e = getenv("ASTYLE_MFMA16"); v = e ? atoi(e) : 2; if (v < 0 || v > 3) v = 2; }
    return v;
}
static bool mfma16_fwd() { const int m = mfma16_mode(); return m == 1 || m == 3; }
static bool mfma16_bwd() { const int m = mfma16_mode(); return m == 1 || m == 2; }
// (K index kk, output-channel index mm) of element e of lane ln in fragment slot kb of wave w, in
// the 32x32x16 or (m16) the 16x16x32 layout (common.h: the split weight layouts)
static void frag_index(bool m16, int kb, int ln, int e, int w, int& kk, int& mm) {
    if (m16) {
        const int ii = ln & 15, qq = ln >> 4;
        kk = 32 * (kb >> 1) + 8 * qq + e;
        mm = 32 * w + 16 * (kb & 1) + ii;
    } else {
        kk = 16 * kb + 8 * (ln >> 5) + e;
        mm = 32 * w + (ln & 31);
    }
}

size_t workspace_bytes(const ast_cfg* c, const ast_ctx* x) {
    const size_t BTC = (size_t)c->batch * c->T * C;
    const size_t es = c->precision == 1 ? 2 : 4;
    size_t n = 0;
    n += W_TOTAL * 4 + (size_t)NBLK_MAX * BLKB_SZ * 2;
    if (c->precision == 2) n += (size_t)NBLK_MAX * SBLK * 16 + 2 * (size_t)(NBLK_MAX + 1) * c->batch * GCLIP_W * 4;
    n += (size_t)(x->nblk + 1) * (BTC + tensor_pad()) * es * (x->doop ? 2 : 1);   // act (+ D)
    if (x->doop) n += d_pad();
    n += 2 * (size_t)x->nblk * c->batch * c->T * 16;        // mu, me
    n += 2 * BTC * es;                                      // chain
    int ncg = 0;
    const int fuse_u = fused_content_occ(x);   // (as ast_create: no content-gradient buffer for it)
    for (int t = 0; t <= NBLK_MAX; ++t)
        if ((x->tensor_has_direct_content[t] && !(fuse_u >= 0 && x->uid[fuse_u] == t)) || (t == 30 && x->need_bott)) ++ncg;
    n += (size_t)ncg * BTC * es;
    if (x->need_bott) n += 2 * (size_t)c->batch * c->T * 16 * 4;
    n += x->gpart_elems * 4;                                // gpart
    n += x->smat_elems * (c->gatys && es == 2 ? 6 : 4);     // smat (+ bf16 copy)
    n += (size_t)c->batch * C * 4;                          // spart
    n += 256;                                               // zero line
    n += (size_t)c->batch * 4;                              // range flags
    n += (size_t)c->batch * x->occ.size() * (c->T / CROWS) * 4;
    const int nf = stft_frames(c->T);
    if (nf) n += 1024 * 8 + (size_t)c->batch * nf * (1 + 1024) * 4;   // STFT regulariser
    return n;
}

// the D placement of a context (x->doop) on the current device: forced by ASTYLE_DOOP, else out
// of place when workspace_bytes with it leaves max(16 GiB, 10 % of the device) free
static void decide_doop(const ast_cfg* c, ast_ctx* x) {
    const int env = doop_env();
    if (env >= 0) { x->doop = env != 0; return; }
    x->doop = true;
    const size_t need = workspace_bytes(c, x);
    x->doop = false;
    size_t fr = 0, tot = 0;
    if (hipMemGetInfo(&fr, &tot) != hipSuccess) { (void)hipGetLastError(); return; }
    const size_t margin = std::max<size_t>((size_t)16 << 30, tot / 10);
    x->doop = need + margin <= fr;
}

void launch_gram_bwd_any(ast_ctx* x, const GramArgs& g, hipStream_t s);
GramArgs gram_args(ast_ctx* x);
GatysArgs gatys_args(ast_ctx* x);

// Where both placements fit (x->dgrad allocated, D at least 4 GiB) and ASTYLE_DOOP does not force
// one, the first evaluation that is not being captured into a graph times its own Gram backward in
// both placements and keeps the faster (in place only when it wins by more than 1 %, releasing the D
// buffer).  Out of place runs first: it reads E and writes D to its own buffer, so E is still there
// for the in-place run, which writes the same D over E; either way D is where the chosen placement
// reads it, and the content tap's partials and the chain's max come out the same (slot stores,
// atomic max of identical values).  The slow in-place mode depends on the physical pages a process
// got and on the data, so it is measured on the run's own data (round 6; a timing
// at create on the empty buffers mispredicted by up to 1 ms).  A capture before that evaluation
// fixes out of place (a graph holds the D buffer's address).  ~45 ms once at B = 256.
static bool capturing(hipStream_t s) {
    hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(s, &st) != hipSuccess) { (void)hipGetLastError(); return true; }
    return st != hipStreamCaptureStatusNone;
}
template <class F>
static int timed_gram_bwd(ast_ctx* x, F launch, hipStream_t s) {
    if (!x->doop_tune || !x->dgrad) { launch(x->dgrad ? x->dgrad : x->act); return 0; }
    if (capturing(s)) {   // a graph now holds the out-of-place address: keep it
        x->doop_tune = false;
        launch(x->dgrad);
        return 0;
    }
    x->doop_tune = false;
    hipEvent_t e[3];
    for (auto& ev : e) HIPCHK(hipEventCreate(&ev));
    (void)hipEventRecord(e[0], s);
    launch(x->dgrad);
    (void)hipEventRecord(e[1], s);
    launch(x->act);
    (void)hipEventRecord(e[2], s);
    hipError_t er = hipEventSynchronize(e[2]);
    float t_out = 0.f, t_in = 0.f;
    if (er == hipSuccess) er = hipEventElapsedTime(&t_out, e[0], e[1]);
    if (er == hipSuccess) er = hipEventElapsedTime(&t_in, e[1], e[2]);
    for (auto& ev : e) (void)hipEventDestroy(ev);
    if (er != hipSuccess) return fail(AST_E_HIP, hipGetErrorString(er));
    x->doop_ms[0] = t_in;
    x->doop_ms[1] = t_out;
    if (t_in < 0.99f * t_out) {   // in place: D is over E now; give the D buffer back
        void* base = (char*)x->dgrad - d_pad();
        auto it = std::find(x->allocs.begin(), x->allocs.end(), base);
        if (it != x->allocs.end()) {
            (void)hipFree(base);
            x->allocs.erase(it);
        }
        x->dgrad = nullptr;
        x->doop = false;
    }
    return 0;
}

// ASTYLE_GUARD=1 (diagnostic): every buffer gets a GUARD_BYTES band of GUARD_FILL on both
// sides; ast_debug_check_guards reports any band a kernel wrote into (out-of-bounds stores)
constexpr size_t GUARD_BYTES = 64 << 10;
constexpr int GUARD_FILL = 0x5a;
static bool guard_on() {
    static int v = -1;
    if (v < 0) { const char* e = getenv("ASTYLE_GUARD"); v = e && atoi(e) ? 1 : 0; }
    return v == 1;
}

int dalloc(ast_ctx* x, void** p, size_t bytes, const char* name = "") {
    if (guard_on()) {
        char* base = nullptr;
        HIPCHK(hipMalloc((void**)&base, bytes + 2 * GUARD_BYTES));
        HIPCHK(hipMemset(base, GUARD_FILL, bytes + 2 * GUARD_BYTES));
        x->allocs.push_back(base);
        x->guards.push_back({base, bytes, name});
        *p = base + GUARD_BYTES;
        return 0;
    }
    HIPCHK(hipMalloc(p, bytes));
    x->allocs.push_back(*p);
    return 0;
}

hipStream_t S(void* s) { return reinterpret_cast<hipStream_t>(s); }

void tmark(ast_ctx* x, hipStream_t s) {
    if (!x->timing || x->ev_used >= (int)x->ev.size()) return;
    (void)hipEventRecord(x->ev[x->ev_used++], s);
}

float* blkw(ast_ctx* x, int l) { return x->wts + BLK_OFF + (size_t)l * BLK_SZ; }
u16* blkwb(ast_ctx* x, int l) { return x->wtsb + (size_t)l * BLKB_SZ; }
void* tens(ast_ctx* x, int t) { return (char*)x->act + (size_t)t * x->tstride * x->esz; }

int run_forward(ast_ctx* x, const float* xd, hipStream_t s, bool mark = false) {
    x->lg_front_done = false;   // phase 1's state (act, gmax) is about to be overwritten
    const ast_cfg& c = x->cfg;
    if (x->split) {
        launch_zero32(x->gmax_e, (size_t)(NBLK_MAX + 1) * c.batch * GCLIP_W * 4, s, 0);
        // e_0 is not stored: block 0 recomputes it from x (FwdArgsS::xin); masks and max only
        launch_startconv_masks((const float*)xd, x->wts + W0_OFF, x->wts + B0_OFF, c.batch, c.T, s,
                               (uint16_t*)x->me, x->gmax_e);
    } else if (x->bf) launch_startconv_fwd((const float*)xd, (u16*)x->act, x->wts + W0_OFF, x->wts + B0_OFF, c.batch, c.T, s, (uint16_t*)x->me);
    else launch_startconv_fwd((const float*)xd, (float*)x->act, x->wts + W0_OFF, x->wts + B0_OFF, c.batch, c.T, s);
    if (mark) tmark(x, s);
    for (int l = 0; l < x->nblk; ++l) {
        float* w = blkw(x, l);
        const int d = 1 << (l % 10);
        uint32_t* mu = x->mu + (size_t)l * c.batch * c.T * 4;
        uint32_t* me = x->me + (size_t)l * c.batch * c.T * 4;
        if (x->split) {
            FwdArgsS a;
            a.stamps = stamp_row();
            const uint4* ws = x->wtss + (size_t)l * SBLK;
            a.ein = (const float*)tens(x, l); a.eout = (float*)tens(x, l + 1);
            a.wdf = ws + SWDF; a.wrf = ws + SWRF; a.bd = w + BD; a.br = w + BR;
            a.mu = (uint16_t*)mu;
            a.me_next = l + 1 < x->nblk ? (uint16_t*)(me + (size_t)c.batch * c.T * 4) : nullptr;
            a.gmax_in = (const float*)(x->gmax_e + (size_t)l * c.batch * GCLIP_W);
            a.gmax_out = x->gmax_e + (size_t)(l + 1) * c.batch * GCLIP_W;
            a.zero = (const float*)x->zero;
            a.B = c.batch; a.T = c.T; a.d = d; a.n = c.T / d;
            a.dn_log2 = (l + 1) % 10; a.nn = c.T >> a.dn_log2;
            a.kd = x->kd[l]; a.kr = x->kr[l];
            a.wdn = x->wdn[l]; a.bdm = x->bdm[l];
            a.cus = x->cus;
            a.xin = l == 0 ? xd : nullptr; a.w0 = x->wts + W0_OFF; a.b0 = x->wts + B0_OFF;
            if (mfma16_fwd()) launch_block_fwd_s16(a, s);
            else launch_block_fwd_s(a, s);
        } else if (x->bf) {
            FwdArgsC a;
            a.stamps = stamp_row();
            u16* wb = blkwb(x, l);
            a.ein = (const u16*)tens(x, l); a.eout = (u16*)tens(x, l + 1);
            a.wf = wb + WFB; a.wrf = wb + WRFB; a.bd = w + BD; a.br = w + BR;
            a.mu = (uint16_t*)mu;
            a.me_next = l + 1 < x->nblk ? (uint16_t*)(me + (size_t)c.batch * c.T * 4) : nullptr;
            a.zero = (const u16*)x->zero;
            a.B = c.batch; a.T = c.T; a.d = d; a.n = c.T / d;
            a.dn_log2 = (l + 1) % 10; a.nn = c.T >> a.dn_log2;
            launch_block_fwd_c(a, s);
        } else {
            FwdArgs a;
            a.ein = (const float*)tens(x, l); a.eout = (float*)tens(x, l + 1);
            a.wd = w + WD; a.bd = w + BD; a.wr = w + WR; a.br = w + BR;
            a.mu = mu; a.me = me;
            a.B = c.batch; a.T = c.T; a.d = d; a.n = c.T / d;
            launch_block_fwd(a, s);
        }
    }
    if (mark) tmark(x, s);
    if (x->need_bott) {
        if (x->bf) launch_bottleneck_fwd((const u16*)tens(x, 30), x->bott, x->wts + WB_OFF, x->wts + BB_OFF, c.batch, c.T, s);
        else launch_bottleneck_fwd((const float*)tens(x, 30), x->bott, x->wts + WB_OFF, x->wts + BB_OFF, c.batch, c.T, s);
    }
    HIPCHK(hipGetLastError());
    x->fwd_done = true;
    return 0;
}

void launch_gram_fwd_any(ast_ctx* x, const GramArgs& g, hipStream_t s) {
    if (x->bf) launch_gram_fwd_bf16(g, s);
    else if (x->split) launch_gram_fwd_s(g, s);
    else launch_gram_fwd(g, s);
}
void launch_gram_bwd_any(ast_ctx* x, const GramArgs& g, hipStream_t s) {
    if (x->bf) launch_gram_bwd_bf16(g, s);
    else if (x->split) launch_gram_bwd_s(g, s);
    else launch_gram_bwd(g, s);
}

// The split Gram backward (ours or Gatys) computes the content tap's gradient and squared error
// itself when there is exactly one content occurrence and its tensor is style-tapped (configs[2]
// and configs[4]: cont 29): k_content's cg buffer (written, then read back by the Gram backward)
// is skipped.
// ASTYLE_FUSE_CONTENT=0 keeps the separate kernel.
int fused_content_occ(const ast_ctx* x) {
    static int en = -1;
    if (en < 0) { const char* e = getenv("ASTYLE_FUSE_CONTENT"); en = e ? (atoi(e) != 0) : 1; }
    if (!en || x->cfg.precision != 2 || x->occ.size() != 1 || x->need_bott) return -1;
    const Occ& o = x->occ[0];
    if (o.ext == 31 || !x->tensor_in_style[o.tensor]) return -1;
    if (o.off % 4 || o.ncol % 4 || x->ncc % 4) return -1;   // (float4 phi reads)
    for (int u = 0; u < x->nu; ++u) if (x->uid[u] == o.tensor) return u;
    return -1;
}

GramArgs gram_args(ast_ctx* x) {
    GramArgs g;
    memset(&g, 0, sizeof(g));
    g.act = x->act; g.actw = x->dgrad ? x->dgrad : x->act; g.tstride = x->tstride;
    g.nu = x->nu;
    for (int u = 0; u < x->nu; ++u) { g.uid[u] = x->uid[u]; g.cg[u] = x->cg_buf[x->uid[u]]; }
    g.gpart = x->gpart; g.smat = x->smat; g.zero16 = x->zero;
    g.B = x->cfg.batch; g.T = x->cfg.T; g.nchunk = x->nchunk;
    g.top_u = -1; g.gmax_top = nullptr;
    g.cont_u = -1;
    return g;
}

StyleArgs style_args(ast_ctx* x) {
    StyleArgs a;
    memset(&a, 0, sizeof(a));
    a.gpart = x->gpart; a.nchunk = x->nchunk;
    a.L = x->L; a.nu = x->nu;
    a.lmap_identity = 1;
    for (int i = 0; i < x->L; ++i) {
        a.lmap[i] = x->lmap[i];
        if (x->lmap[i] != i) a.lmap_identity = 0;
    }
    a.nb = std::min(x->cfg.nb_channels, C);
    a.coef = x->cfg.lambd * 1e3f * 2.0f / (float)(a.nb * x->L * x->L);
    a.B = x->cfg.batch;
    return a;
}

GatysArgs gatys_args(ast_ctx* x) {
    GatysArgs g;
    memset(&g, 0, sizeof(g));
    g.act = x->act; g.actw = x->dgrad ? x->dgrad : x->act; g.tstride = x->tstride;
    g.nu = x->nu;
    for (int u = 0; u < x->nu; ++u) { g.uid[u] = x->uid[u]; g.cg[u] = x->cg_buf[x->uid[u]]; }
    g.gpart = x->gpart; g.smat = x->smat; g.smatb = x->smatb;
    g.B = x->cfg.batch; g.T = x->cfg.T; g.nchunk = x->nchunk;
    g.cont_u = -1;
    g.top_u = -1; g.gmax_top = nullptr;
    return g;
}

GatysStyleArgs gatys_style_args(ast_ctx* x) {
    GatysStyleArgs a;
    memset(&a, 0, sizeof(a));
    a.gpart = x->gpart; a.nchunk = x->nchunk;
    a.L = x->L; a.nu = x->nu;
    for (int i = 0; i < x->L; ++i) a.lmap[i] = x->lmap[i];
    a.coef = x->cfg.lambd * 1e3f * 2.0f / (float)(x->L * C * C);
    a.B = x->cfg.batch;
    return a;
}

}  // namespace

extern "C" {

const char* ast_last_error(void) { return g_err.c_str(); }

int ast_restore(ast_ctx* x, const char* prefix) {
    if (!x || !prefix) return fail(AST_E_ARG, "ast_restore: null argument");
    try {   // nothing may unwind through the C ABI
        Checkpoint ck;
        std::string err;
        if (ck.open(prefix, &err)) return fail(AST_E_NAME, err);
        // every encoder variable with its HWIO shape (masked.py:136-145; Saver.restore refuses a
        // variable whose shape differs, so a transposed or reshaped tensor is refused here too)
        typedef std::vector<int64_t> Shape;
        std::vector<std::pair<std::string, Shape>> names = {
            {"ae_startconv/W", {1, 3, 1, C}}, {"ae_startconv/biases", {C}},
            {"ae_bottleneck/W", {1, 1, C, 16}}, {"ae_bottleneck/biases", {16}}};
        for (int l = 1; l <= 30; ++l) {
            const std::pair<const char*, Shape> ks[4] = {{"ae_dilatedconv_%d/W", {1, 3, C, C}},
                                                         {"ae_dilatedconv_%d/biases", {C}},
                                                         {"ae_res_%d/W", {1, 1, C, C}},
                                                         {"ae_res_%d/biases", {C}}};
            for (const auto& k : ks) {
                char b[64];
                snprintf(b, sizeof b, k.first, l);
                names.emplace_back(b, k.second);
            }
        }
        auto str = [](const Shape& v) {
            std::string o = "[";
            for (size_t i = 0; i < v.size(); ++i) o += (i ? "," : "") + std::to_string(v[i]);
            return o + "]";
        };
        std::vector<float> buf;
        for (const auto& nm : names) {
            const CkptEntry* e = ck.find(nm.first);
            if (!e) return fail(AST_E_NAME, std::string(prefix) + ": no variable " + nm.first +
                                                " (Saver.restore needs every encoder variable)");
            // the shape from the file is checked before anything is allocated for it
            if (e->shape != nm.second)
                return fail(AST_E_NAME, nm.first + ": checkpoint shape " + str(e->shape) +
                                            ", the encoder expects " + str(nm.second));
            int64_t n = 1;
            for (int64_t d : nm.second) n *= d;
            buf.resize((size_t)n);
            if (ck.read_f32(*e, buf.data(), &err)) return fail(AST_E_ARG, err);
            const int rc = ast_set_weight(x, nm.first.c_str(), buf.data(), buf.size());
            if (rc) return rc;
        }
        return 0;
    } catch (const std::exception& ex) {
        return fail(AST_E_ARG, std::string("ast_restore: ") + ex.what());
    }
}

int ast_ot_admm(const double* p_mod, const double* p_ref, int nprob, int n1, int n2, int d,
                double eps, double miter, double* plan, double* pal, int* iters, void* stream) {
    if (nprob < 0 || n1 < 1 || n2 < 1 || d < 1)
        return fail(AST_E_ARG, "ast_ot_admm: need nprob >= 0 and n1, n2, d >= 1");
    // the workspace kernel runs one workgroup per problem over 10 n1 n2 fp64 iterates: ~80 B per
    // cell per ADMM iteration on one CU (2^16 cells: ~5 MB, ~0.1 ms per iteration, seconds per
    // solve at the reference's iteration counts); past that the call would run for hours
    if ((long long)n1 * n2 > (1ll << 16) || ot_big_lds_bytes(n1, n2) > 160 * 1024)
        return fail(AST_E_ARG, "ast_ot_admm: n1 * n2 must be <= 2^16 (and n1 + n2 <= 20000)");
    if (!(eps > 0.0) || !(miter >= 0.0))
        return fail(AST_E_ARG, "ast_ot_admm: eps must be > 0 and miter >= 0");
    if (nprob == 0) return 0;
    if (!p_mod || !p_ref || !plan) return fail(AST_E_ARG, "ast_ot_admm: null buffer");
    if ((long long)n1 * n2 <= ot_max_cells()) {
        launch_ot_admm(p_mod, p_ref, nprob, n1, n2, d, eps, miter, plan, pal, iters, S(stream));
        HIPCHK(hipGetLastError());
        return 0;
    }
    // larger palettes: iterates in a stream-ordered device workspace (allocated and freed on
    // the call's stream)
    void* ws = nullptr;
    HIPCHK(hipMallocAsync(&ws, ot_big_ws_bytes(n1, n2) * (size_t)nprob, S(stream)));
    launch_ot_admm_big(p_mod, p_ref, nprob, n1, n2, d, eps, miter, (double*)ws, plan, pal, iters,
                       S(stream));
    const hipError_t le = hipGetLastError();
    HIPCHK(hipFreeAsync(ws, S(stream)));
    if (le != hipSuccess) return fail(AST_E_HIP, std::string("k_ot_admm_big: ") + hipGetErrorString(le));
    return 0;
}

// Diagnostic hook (not in astyle.h): device buffer of 12 u64 phase-cycle sums that
// -DASTYLE_STAMPS builds of the bf16 block kernels accumulate into; NULL disables.
int ast_debug_stamps(void* dev_u64x20x64) {   // 64 rows of 20: [0..15] sums, [16] / [17] max / min wave lifetime, [18] / [19] first start / last end
    g_stamps = (unsigned long long*)dev_u64x20x64;
    g_stamp_row = 0;
    return 0;
}

// Diagnostic (ASTYLE_GUARD=1 contexts; not in astyle.h): device-synchronises, then checks every
// buffer's guard bands; returns the number of buffers with a written band (-1: guards off) and
// writes one line per such buffer to `report`.
int ast_debug_check_guards(ast_ctx* x, char* report, int len) {
    if (!x) return fail(AST_E_ARG, "null argument");
    if (x->guards.empty()) return -1;
    (void)hipSetDevice(x->dev);
    HIPCHK(hipDeviceSynchronize());
    std::vector<unsigned char> h(GUARD_BYTES);
    std::string rep;
    int bad = 0;
    for (const auto& g : x->guards) {
        for (int side = 0; side < 2; ++side) {
            const char* band = side ? g.base + GUARD_BYTES + g.bytes : g.base;
            HIPCHK(hipMemcpy(h.data(), band, GUARD_BYTES, hipMemcpyDeviceToHost));
            size_t first = GUARD_BYTES, last = 0, n = 0;
            for (size_t i = 0; i < GUARD_BYTES; ++i)
                if (h[i] != GUARD_FILL) { if (first == GUARD_BYTES) first = i; last = i; ++n; }
            if (n) {
                ++bad;
                char line[256];
                snprintf(line, sizeof(line), "%s (%zu bytes): %s band, %zu bytes written, offsets %lld..%lld from the buffer %s\n",
                         g.name, g.bytes, side ? "upper" : "lower", n,
                         side ? (long long)first : (long long)first - (long long)GUARD_BYTES,
                         side ? (long long)last : (long long)last - (long long)GUARD_BYTES,
                         side ? "end" : "start");
                rep += line;
            }
        }
    }
    if (report && len > 0) snprintf(report, (size_t)len, "%s", rep.c_str());
    return bad;
}

int ast_workspace_bytes(const ast_cfg* cfg, size_t* out) {
    if (!cfg || !out) return fail(AST_E_ARG, "null argument");
    ast_ctx tmp;
    tmp.cfg = *cfg;
    int rc = plan(cfg, &tmp);
    if (rc) return rc;
    decide_doop(cfg, &tmp);   // (the current device's free memory, as ast_create on it decides)
    *out = workspace_bytes(cfg, &tmp);
    return 0;
}

int ast_d_out_of_place(const ast_ctx* x, int* out, float* tuned_ms) {
    if (!x || !out) return fail(AST_E_ARG, "null argument");
    *out = x->doop ? 1 : 0;
    if (tuned_ms) { tuned_ms[0] = x->doop_ms[0]; tuned_ms[1] = x->doop_ms[1]; }
    return 0;
}

int ast_create(const ast_cfg* cfg, int hip_device, ast_ctx** out) {
    if (!cfg || !out) return fail(AST_E_ARG, "null argument");
    ast_ctx* x = new ast_ctx();
    x->cfg = *cfg;
    int rc = plan(cfg, x);
    if (rc) { delete x; return rc; }
    x->dev = hip_device;
    hipError_t e = hipSetDevice(hip_device);
    if (e != hipSuccess) { delete x; return fail(AST_E_HIP, hipGetErrorString(e)); }
    decide_doop(cfg, x);
    const ast_cfg& c = *cfg;
    const size_t BTC = (size_t)c.batch * c.T * C;
    x->tstride = BTC + tensor_pad();
    void* p;
#define ALLOC(dst, bytes) do { if ((rc = dalloc(x, &p, (bytes), #dst))) { ast_destroy(x); return rc; } dst = (decltype(dst))p; } while (0)
    x->bf = c.precision == 1;
    x->split = c.precision == 2;
    x->esz = x->bf ? 2 : 4;
    if (x->split) {
        ALLOC(x->wtss, (size_t)NBLK_MAX * SBLK * 16);
        (void)hipMemset(x->wtss, 0, (size_t)NBLK_MAX * SBLK * 16);
        ALLOC(x->gmax_e, (size_t)(NBLK_MAX + 1) * c.batch * GCLIP_W * 4);
        ALLOC(x->gmax_g, (size_t)(NBLK_MAX + 1) * c.batch * GCLIP_W * 4);
    }
    ALLOC(x->wts, W_TOTAL * 4);
    (void)hipMemset(x->wts, 0, W_TOTAL * 4);
    ALLOC(x->wtsb, (size_t)NBLK_MAX * BLKB_SZ * 2);
    (void)hipMemset(x->wtsb, 0, (size_t)NBLK_MAX * BLKB_SZ * 2);
    ALLOC(x->act, (size_t)(x->nblk + 1) * x->tstride * x->esz);
    if (x->doop) {
        ALLOC(x->dgrad, (size_t)(x->nblk + 1) * x->tstride * x->esz + d_pad());
        x->dgrad = (char*)x->dgrad + d_pad();   // (x->allocs keeps the base for hipFree)
    }
    ALLOC(x->mu, (size_t)x->nblk * c.batch * c.T * 16);
    ALLOC(x->me, (size_t)x->nblk * c.batch * c.T * 16);
    ALLOC(x->chain[0], BTC * x->esz);
    ALLOC(x->chain[1], BTC * x->esz);
    const int fuse_u = fused_content_occ(x);   // (the Gram backward adds that tap's gradient itself)
    for (int t = 0; t <= NBLK_MAX; ++t)
        if ((x->tensor_has_direct_content[t] && !(fuse_u >= 0 && x->uid[fuse_u] == t)) || (t == 30 && x->need_bott))
            ALLOC(x->cg_buf[t], BTC * x->esz);
    if (x->need_bott) {
        ALLOC(x->bott, (size_t)c.batch * c.T * 16 * 4);
        ALLOC(x->gbott, (size_t)c.batch * c.T * 16 * 4);
    }
    ALLOC(x->gpart, x->gpart_elems * 4);
    ALLOC(x->smat, x->smat_elems * 4);
    if (c.gatys && x->bf) ALLOC(x->smatb, x->smat_elems * 2);
    ALLOC(x->zero, 256);
    (void)hipMemset(x->zero, 0, 256);
    ALLOC(x->rflags, (size_t)c.batch * 4);
    (void)hipMemset(x->rflags, 0, (size_t)c.batch * 4);
    ALLOC(x->rflags_last, (size_t)c.batch * 4);
    (void)hipMemset(x->rflags_last, 0, (size_t)c.batch * 4);
    ALLOC(x->spart, (size_t)c.batch * C * 4);
    x->ncpart = (int)x->occ.size() * (c.T / CROWS);
    ALLOC(x->cpart, (size_t)c.batch * x->ncpart * 4);
    if (const int nf = stft_frames(c.T)) {
        ALLOC(x->stft_tw, 1024 * 8);
        ALLOC(x->stft_fpart, (size_t)c.batch * nf * 4);
        ALLOC(x->stft_gfr, (size_t)c.batch * nf * 1024 * 4);
        launch_stft_twiddles(x->stft_tw, nullptr);
        e = hipDeviceSynchronize();
        if (e != hipSuccess) { ast_destroy(x); return fail(AST_E_HIP, hipGetErrorString(e)); }
    }
#undef ALLOC
    x->doop_tune = doop_env() < 0 && x->dgrad &&
                   (size_t)(x->nblk + 1) * x->tstride * x->esz >= ((size_t)4 << 30);
    *out = x;
    return 0;
}

void ast_destroy(ast_ctx* x) {
    if (!x) return;
    (void)hipSetDevice(x->dev);
    for (void* p : x->allocs) (void)hipFree(p);
    for (hipEvent_t e : x->ev) (void)hipEventDestroy(e);
    delete x;
}

int ast_set_weight(ast_ctx* x, const char* name, const float* host, size_t n) {
    if (!x || !name || !host) return fail(AST_E_ARG, "null argument");
    (void)hipSetDevice(x->dev);
    std::string s(name);
    auto put = [&](size_t off, const float* src, size_t cnt) -> int {
        HIPCHK(hipMemcpy(x->wts + off, src, cnt * 4, hipMemcpyHostToDevice));
        return 0;
    };
    auto need = [&](size_t cnt) -> int {
        if (n != cnt) return fail(AST_E_NAME, s + ": expected " + std::to_string(cnt) + " elements");
        return 0;
    };
    int rc;
    if (s == "ae_startconv/W") { if ((rc = need(3 * C))) return rc; return put(W0_OFF, host, 3 * C); }
    if (s == "ae_startconv/biases") { if ((rc = need(C))) return rc; return put(B0_OFF, host, C); }
    if (s == "ae_bottleneck/W") { if ((rc = need(C * 16))) return rc; return put(WB_OFF, host, C * 16); }
    if (s == "ae_bottleneck/biases") { if ((rc = need(16))) return rc; return put(BB_OFF, host, 16); }
    int l = 0;
    char tail[32];
    if (sscanf(name, "ae_dilatedconv_%d/%31s", &l, tail) == 2 && l >= 1 && l <= NBLK_MAX) {
        const size_t base = BLK_OFF + (size_t)(l - 1) * BLK_SZ;
        if (!strcmp(tail, "W")) {
            if ((rc = need(3 * C * C))) return rc;
            std::vector<float> tr(3 * C * C);
            for (int k = 0; k < 3; ++k)
                for (int ci = 0; ci < C; ++ci)
                    for (int co = 0; co < C; ++co)
                        tr[(size_t)k * C * C + co * C + ci] = host[(size_t)k * C * C + ci * C + co];
            if ((rc = put(base + WD, host, 3 * C * C))) return rc;
            if ((rc = put(base + WDT, tr.data(), 3 * C * C))) return rc;
            std::vector<uint16_t> hb(6 * C * C), hf(3 * C * C), hg(3 * C * C);
            for (size_t i = 0; i < 3 * C * C; ++i) { hb[i] = host_bf16(host[i]); hb[3 * C * C + i] = host_bf16(tr[i]); }
            // forward fragments from W_d, backward fragments the same order from W_d^T
            for (int k = 0; k < 3; ++k)
                for (int q = 0; q < 4; ++q)
                    for (int kb = 0; kb < 8; ++kb)
                        for (int ln = 0; ln < 64; ++ln)
                            for (int e = 0; e < 8; ++e) {
                                const int ci = 16 * kb + 8 * (ln >> 5) + e, co = 32 * q + (ln & 31);
                                const size_t o = ((((size_t)k * 4 + q) * 8 + kb) * 64 + ln) * 8 + e;
                                hf[o] = hb[(size_t)k * C * C + ci * C + co];
                                hg[o] = hb[3 * C * C + (size_t)k * C * C + ci * C + co];
                            }
            u16* dst = x->wtsb + (size_t)(l - 1) * BLKB_SZ;
            HIPCHK(hipMemcpy(dst + WFB, hf.data(), 3 * C * C * 2, hipMemcpyHostToDevice));
            HIPCHK(hipMemcpy(dst + WBFB, hg.data(), 3 * C * C * 2, hipMemcpyHostToDevice));
            if (x->split) {
                // forward: element (w, tap, kb, hl, lane (m, h), e) = W_d[tap][16 kb + 8 h + e][32 w + m];
                // backward: W_d[tap][32 w + m][16 kb + 8 h + e] (ASTYLE_MFMA16: frag_index)
                const int k = weight_exp(host, 3 * C * C);
                x->kd[l - 1] = k;
                float nrm = 0.f;
                for (int co = 0; co < C; ++co) {
                    float sacc = 0.f;
                    for (int i = 0; i < 3 * C; ++i) sacc += std::fabs(host[(size_t)i * C + co]);
                    nrm = std::max(nrm, sacc);
                }
                x->wdn[l - 1] = nrm;
                std::vector<uint16_t> f(3 * C * C * 2), g(3 * C * C * 2);
                for (int w = 0; w < 4; ++w)
                    for (int tp = 0; tp < 3; ++tp)
                        for (int kb = 0; kb < 8; ++kb)
                            for (int ln = 0; ln < 64; ++ln)
                                for (int e = 0; e < 8; ++e) {
                                    int kk, mm, kb2, mb2;
                                    frag_index(mfma16_fwd(), kb, ln, e, w, kk, mm);
                                    frag_index(mfma16_bwd(), kb, ln, e, w, kb2, mb2);
                                    const size_t o = ((((size_t)(w * 3 + tp) * 8 + kb) * 2) * 64 + ln) * 8 + e;
                                    split_half(host[(size_t)tp * C * C + kk * C + mm], k, f[o], f[o + 64 * 8]);
                                    split_half(host[(size_t)tp * C * C + mb2 * C + kb2], k, g[o], g[o + 64 * 8]);
                                }
                uint4* ds = x->wtss + (size_t)(l - 1) * SBLK;
                HIPCHK(hipMemcpy(ds + SWDF, f.data(), f.size() * 2, hipMemcpyHostToDevice));
                HIPCHK(hipMemcpy(ds + SWDB, g.data(), g.size() * 2, hipMemcpyHostToDevice));
            }
            return 0;
        }
        if (!strcmp(tail, "biases")) {
            if ((rc = need(C))) return rc;
            float m = 0.f;
            for (int i = 0; i < C; ++i) m = std::max(m, std::fabs(host[i]));
            x->bdm[l - 1] = m;
            return put(base + BD, host, C);
        }
    }
    if (sscanf(name, "ae_res_%d/%31s", &l, tail) == 2 && l >= 1 && l <= NBLK_MAX) {
        const size_t base = BLK_OFF + (size_t)(l - 1) * BLK_SZ;
        if (!strcmp(tail, "W")) {
            if ((rc = need(C * C))) return rc;
            std::vector<float> tr(C * C);
            for (int ci = 0; ci < C; ++ci)
                for (int co = 0; co < C; ++co) tr[co * C + ci] = host[ci * C + co];
            if ((rc = put(base + WR, host, C * C))) return rc;
            if ((rc = put(base + WRT, tr.data(), C * C))) return rc;
            std::vector<uint16_t> hb(2 * C * C), hf(C * C), hg(C * C);
            for (size_t i = 0; i < C * C; ++i) { hb[i] = host_bf16(host[i]); hb[C * C + i] = host_bf16(tr[i]); }
            for (int q2 = 0; q2 < 4; ++q2)
                for (int st = 0; st < 8; ++st)
                    for (int ln = 0; ln < 64; ++ln)
                        for (int e = 0; e < 8; ++e) {
                            const int co = kperm(st, ln >> 5, e), co2 = 32 * q2 + (ln & 31);
                            const size_t o = (((size_t)q2 * 8 + st) * 64 + ln) * 8 + e;
                            hf[o] = hb[(size_t)co * C + co2];
                            // backward: W_r[32 q + m][16 kb + 8 h + e] = W_r^T[16 kb + 8 h + e][32 q + m]
                            hg[o] = hb[C * C + (size_t)(16 * st + 8 * (ln >> 5) + e) * C + 32 * q2 + (ln & 31)];
                        }
            u16* dst = x->wtsb + (size_t)(l - 1) * BLKB_SZ;
            HIPCHK(hipMemcpy(dst + WRFB, hf.data(), C * C * 2, hipMemcpyHostToDevice));
            HIPCHK(hipMemcpy(dst + WRBFB, hg.data(), C * C * 2, hipMemcpyHostToDevice));
            if (x->split) {
                // forward: element (w, kb, hl, lane (m, h), e) = W_r[16 kb + 8 h + e][32 w + m];
                // backward: W_r[32 w + m][16 kb + 8 h + e] (ASTYLE_MFMA16: frag_index)
                const int k = weight_exp(host, C * C);
                x->kr[l - 1] = k;
                float nrm = 0.f;
                for (int ci = 0; ci < C; ++ci) {
                    float sacc = 0.f;
                    for (int co = 0; co < C; ++co) sacc += std::fabs(host[(size_t)ci * C + co]);
                    nrm = std::max(nrm, sacc);
                }
                x->wrn[l - 1] = nrm;
                std::vector<uint16_t> f(C * C * 2), g(C * C * 2);
                for (int w = 0; w < 4; ++w)
                    for (int kb = 0; kb < 8; ++kb)
                        for (int ln = 0; ln < 64; ++ln)
                            for (int e = 0; e < 8; ++e) {
                                int kk, mm, kb2, mb2;
                                frag_index(mfma16_fwd(), kb, ln, e, w, kk, mm);
                                frag_index(mfma16_bwd(), kb, ln, e, w, kb2, mb2);
                                const size_t o = ((((size_t)w * 8 + kb) * 2) * 64 + ln) * 8 + e;
                                split_half(host[(size_t)kk * C + mm], k, f[o], f[o + 64 * 8]);
                                split_half(host[(size_t)mb2 * C + kb2], k, g[o], g[o + 64 * 8]);
                            }
                uint4* ds = x->wtss + (size_t)(l - 1) * SBLK;
                HIPCHK(hipMemcpy(ds + SWRF, f.data(), f.size() * 2, hipMemcpyHostToDevice));
                HIPCHK(hipMemcpy(ds + SWRB, g.data(), g.size() * 2, hipMemcpyHostToDevice));
            }
            return 0;
        }
        if (!strcmp(tail, "biases")) { if ((rc = need(C))) return rc; return put(base + BR, host, C); }
    }
    return fail(AST_E_NAME, "not an encoder variable: " + s);
}

int ast_forward(ast_ctx* x, const float* xd, void* stream) {
    if (!x || !xd) return fail(AST_E_ARG, "null argument");
    return run_forward(x, xd, S(stream));
}

int ast_get_extract(ast_ctx* x, int ext, float* out, void* stream) {
    if (!x || !out) return fail(AST_E_ARG, "null argument");
    if (!x->fwd_done) return fail(AST_E_STATE, "ast_forward has not run");
    const ast_cfg& c = x->cfg;
    if (ext == 31) {
        if (!x->need_bott) return fail(AST_E_ARG, "extract 31 (bottleneck) is not computed for these taps");
        HIPCHK(hipMemcpyAsync(out, x->bott, (size_t)c.batch * c.T * 16 * 4, hipMemcpyDeviceToDevice, S(stream)));
        return 0;
    }
    if (ext < 0 || ext > 30) return fail(AST_E_ARG, "extract id out of range");
    const int tns = ext_to_tensor(ext);
    if (tns > x->nblk) return fail(AST_E_ARG, "extract beyond the blocks this context runs");
    if (x->bf) {
        launch_to_f32((const u16*)tens(x, tns), out, (size_t)c.batch * c.T * C, S(stream));
        HIPCHK(hipGetLastError());
    } else {
        HIPCHK(hipMemcpyAsync(out, tens(x, tns), (size_t)c.batch * c.T * C * 4, hipMemcpyDeviceToDevice, S(stream)));
    }
    return 0;
}

int ast_content_cols(ast_ctx* x) { return x ? x->ncc : 0; }

int ast_embeds(ast_ctx* x, const float* xd, float* emb_c, float* emb_s, void* stream) {
    if (!x || !xd) return fail(AST_E_ARG, "null argument");
    hipStream_t s = S(stream);
    int rc = run_forward(x, xd, s);
    if (rc) return rc;
    const ast_cfg& c = x->cfg;
    if (emb_c) {
        for (const Occ& o : x->occ) {
            ContentArgs a;
            memset(&a, 0, sizeof(a));
            a.e = o.ext == 31 ? (const void*)x->bott : tens(x, o.tensor);
            a.e_bf16 = o.ext != 31 && x->bf;
            a.W = o.ext == 31 ? 16 : C;
            a.ncc = x->ncc; a.off = o.off; a.ncol = o.ncol;
            a.embc = emb_c; a.B = c.batch; a.T = c.T;
            launch_content(a, s);
        }
    }
    if (emb_s && c.gatys) {
        GatysArgs g = gatys_args(x);
        launch_gatys_fwd(g, x->split ? 2 : (x->bf ? 1 : 0), s);
        GatysStyleArgs a = gatys_style_args(x);
        a.embs = emb_s;
        launch_style_gatys(a, s);
    } else if (emb_s) {
        GramArgs g = gram_args(x);
        launch_gram_fwd_any(x, g, s);
        StyleArgs a = style_args(x);
        a.embs = emb_s;
        launch_style_ours(a, s);
    }
    HIPCHK(hipGetLastError());
    return 0;
}

int ast_set_targets(ast_ctx* x, const float* phi_c, int phi_c_shared, const float* phi_s,
                    int phi_s_shared) {
    if (!x || !phi_c || !phi_s) return fail(AST_E_ARG, "null argument");
    x->phi_c = phi_c; x->phi_c_shared = phi_c_shared;
    x->phi_s = phi_s; x->phi_s_shared = phi_s_shared;
    x->targets = true;
    x->lg_front_done = false;   // a phase 2 must follow a phase 1 of these targets
    return 0;
}

int ast_set_gamma(ast_ctx* x, float gamma) {
    if (!x) return fail(AST_E_ARG, "null argument");
    x->cfg.gamma = gamma;
    x->lg_front_done = false;
    return 0;
}

// ast_loss_grad in two phases (ast_loss_grad_phase): the front runs the encoder forward, the
// content taps and the Gram forward / style loss / Gram backward; the back runs the backward
// chain through the blocks, d loss / d x, the loss parts, the STFT regulariser and the flags.
static int loss_grad_front(ast_ctx* x, const float* xd, hipStream_t s) {
    const ast_cfg& c = x->cfg;
    tmark(x, s);
    int rc = run_forward(x, xd, s, true);
    if (rc) return rc;
    // content taps (methods.py:58, 116-117)
    const float ccoef = 10.0f * 2.0f / ((float)c.T * (float)x->ncc);
    const int tiles = c.T / CROWS;
    bool first_cg[NBLK_MAX + 1];
    for (int t = 0; t <= NBLK_MAX; ++t) first_cg[t] = true;
    bool first_bott = true;
    const int fuse_u = fused_content_occ(x);
    if (fuse_u >= 0)   // the Gram backward writes (T / GRAM_CSLOT) x 4 = ncpart partial slots per clip
        launch_zero32(x->cpart, (size_t)c.batch * x->ncpart * 4, s, 1);
    for (size_t i = 0; i < x->occ.size(); ++i) {
        if (fuse_u >= 0) break;
        const Occ& o = x->occ[i];
        ContentArgs a;
        memset(&a, 0, sizeof(a));
        a.W = o.ext == 31 ? 16 : C;
        a.e = o.ext == 31 ? (const void*)x->bott : tens(x, o.tensor);
        a.e_bf16 = o.ext != 31 && x->bf;
        a.cg_bf16 = o.ext != 31 && x->bf;
        a.phi = x->phi_c; a.phi_bstride = x->phi_c_shared ? 0 : (size_t)c.T * x->ncc;
        a.ncc = x->ncc; a.off = o.off; a.ncol = o.ncol; a.coef = ccoef;
        if (o.ext == 31) { a.cg = x->gbott; a.accumulate = !first_bott; first_bott = false; }
        else { a.cg = x->cg_buf[o.tensor]; a.accumulate = !first_cg[o.tensor]; first_cg[o.tensor] = false; }
        a.lpart = x->cpart + i * tiles; a.lstride = (size_t)x->ncpart;
        a.B = c.batch; a.T = c.T;
        launch_content(a, s);
    }
    if (x->need_bott) {
        if (x->bf) launch_bottleneck_bwd(x->gbott, (u16*)x->cg_buf[30], x->wts + WB_OFF, !first_cg[30], c.batch, c.T, s);
        else launch_bottleneck_bwd(x->gbott, (float*)x->cg_buf[30], x->wts + WB_OFF, !first_cg[30], c.batch, c.T, s);
    }
    // style (methods.py:62-76, 118-119)
    tmark(x, s);
    bool& top_max_done = x->lg_top_max_done;   // split: the Gram bwd recorded the top tensor's per-clip max
    top_max_done = false;
    if (c.gatys) {
        GatysArgs g = gatys_args(x);
        launch_gatys_fwd(g, x->split ? 2 : (x->bf ? 1 : 0), s);
        tmark(x, s);
        GatysStyleArgs sa = gatys_style_args(x);
        sa.phi = x->phi_s;
        sa.phi_bstride = x->phi_s_shared ? 0 : (size_t)x->L * C * C;
        sa.smat = x->smat; sa.smatb = x->smatb; sa.spart = x->spart;
        launch_style_gatys(sa, s);
        tmark(x, s);
        if (x->split && x->tensor_in_style[x->nblk]) {   // the chain's first max |tot| inside the Gatys bwd
            for (int u = 0; u < x->nu; ++u) if (x->uid[u] == x->nblk) g.top_u = u;
            g.gmax_top = x->gmax_g + (size_t)x->nblk * c.batch * GCLIP_W;
            launch_zero32(x->gmax_g, (size_t)(NBLK_MAX + 1) * c.batch * GCLIP_W * 4, s, 2);
            top_max_done = g.top_u >= 0;
        }
        if (fuse_u >= 0) {   // the split Gatys backward adds the content tap (one slot per 512-row tile)
            const Occ& o = x->occ[0];
            g.cg[fuse_u] = nullptr;
            g.cont_u = fuse_u;
            g.cont_phi = x->phi_c; g.cont_phi_bstride = x->phi_c_shared ? 0 : (size_t)c.T * x->ncc;
            g.cont_ncc = x->ncc; g.cont_off = o.off; g.cont_ncol = o.ncol; g.cont_coef = ccoef;
            g.cont_part = x->cpart; g.cont_pstride = (size_t)x->ncpart;
        }
        if ((rc = timed_gram_bwd(x, [&](void* dst) { GatysArgs gg = g; gg.actw = dst; launch_gatys_bwd(gg, x->split ? 2 : (x->bf ? 1 : 0), s); }, s)))
            return rc;
    } else {
        GramArgs g = gram_args(x);
        launch_gram_fwd_any(x, g, s);
        tmark(x, s);
        StyleArgs sa = style_args(x);
        sa.phi = x->phi_s;
        sa.phi_bstride = x->phi_s_shared ? 0 : (size_t)sa.nb * x->L * x->L;
        sa.smat = x->smat; sa.spart = x->spart;
        launch_style_ours(sa, s);
        tmark(x, s);
        if (x->split && x->tensor_in_style[x->nblk]) {   // the chain's first max |tot| inside the Gram bwd
            for (int u = 0; u < x->nu; ++u) if (x->uid[u] == x->nblk) g.top_u = u;
            g.gmax_top = x->gmax_g + (size_t)x->nblk * c.batch * GCLIP_W;
            launch_zero32(x->gmax_g, (size_t)(NBLK_MAX + 1) * c.batch * GCLIP_W * 4, s, 2);
            top_max_done = g.top_u >= 0;
        }
        if (fuse_u >= 0) {
            const Occ& o = x->occ[0];
            g.cg[fuse_u] = nullptr;
            g.cont_u = fuse_u;
            g.cont_phi = x->phi_c; g.cont_phi_bstride = x->phi_c_shared ? 0 : (size_t)c.T * x->ncc;
            g.cont_ncc = x->ncc; g.cont_off = o.off; g.cont_ncol = o.ncol; g.cont_coef = ccoef;
            g.cont_part = x->cpart; g.cont_pstride = (size_t)x->ncpart;
        }
        g.nchunk = x->nchunk_b;
        if ((rc = timed_gram_bwd(x, [&](void* dst) { GramArgs gg = g; gg.actw = dst; launch_gram_bwd_any(x, gg, s); }, s)))
            return rc;
    }
    tmark(x, s);
    x->lg_front_done = true;
    x->fwd_done = false;   // the Gram backward wrote D over the tapped tensors (in place)
    return 0;
}

static int loss_grad_back(ast_ctx* x, const float* xd, float* grad, float* parts, hipStream_t s) {
    const ast_cfg& c = x->cfg;
    const bool top_max_done = x->lg_top_max_done;
    x->lg_front_done = false;
    // backward chain through the blocks
    auto direct = [&](int t) -> const void* {   // D_t: direct loss gradient of tensor t (or null)
        return x->tensor_in_style[t] ? (x->dgrad ? (const void*)((char*)x->dgrad + (size_t)t * x->tstride * x->esz) : tens(x, t)) : x->cg_buf[t];
    };
    if (x->split && !top_max_done) {
        launch_zero32(x->gmax_g, (size_t)(NBLK_MAX + 1) * c.batch * GCLIP_W * 4, s, 2);
        const void* top = direct(x->nblk);
        if (!top) return fail(AST_E_STATE, "top block has no loss gradient");
        launch_absmax((const float*)top, (size_t)c.T * C, c.batch, x->gmax_g + (size_t)x->nblk * c.batch * GCLIP_W, s);
    }
    for (int l = x->nblk - 1; l >= 0; --l) {
        float* w = blkw(x, l);
        const int tin = l + 1;
        const void* gin = (l == x->nblk - 1) ? nullptr : x->chain[(l + 1) & 1];
        const void* din = direct(tin);
        const uint32_t* mu = x->mu + (size_t)l * c.batch * c.T * 4;
        const uint32_t* me = x->me + (size_t)l * c.batch * c.T * 4;
        const int d = 1 << (l % 10);
        if (x->split) {
            // like the bf16 chain, the chain holds d loss / d e_l with D_l already added
            BwdArgsS a;
            a.stamps = stamp_row();
            const uint4* ws = x->wtss + (size_t)l * SBLK;
            a.tin = (const float*)(gin ? gin : din);
            a.dadd = l > 0 ? (const float*)direct(l) : nullptr;
            a.gout = (float*)x->chain[l & 1];
            a.wrb = ws + SWRB; a.wdb = ws + SWDB;
            a.mu = (const uint16_t*)mu; a.me = (const uint16_t*)me;
            a.gmax_in = (const float*)(x->gmax_g + (size_t)(l + 1) * c.batch * GCLIP_W);
            a.gmax_out = x->gmax_g + (size_t)l * c.batch * GCLIP_W;
            a.zero = (const float*)x->zero;
            a.B = c.batch; a.T = c.T; a.d = d; a.n = c.T / d;
            a.kd = x->kd[l]; a.kr = x->kr[l];
            a.wrn = x->wrn[l];
            a.cus = x->cus;
            // block 0: the start conv's backward folded in; chain[0] holds the wave partials
            a.w0 = x->wts + W0_OFF;
            a.spart = l == 0 ? (float*)x->chain[0] : nullptr;
            if (mfma16_bwd()) launch_block_bwd_s16(a, s);
            else launch_block_bwd_s(a, s);
        } else if (x->bf) {
            // the bf16 chain holds d loss / d e_l with D_l already added (the kernel adds it)
            BwdArgsC a;
            a.stamps = stamp_row();
            u16* wb = blkwb(x, l);
            a.tin = (const u16*)(gin ? gin : din);
            a.dadd = l > 0 ? (const u16*)direct(l) : nullptr;
            a.gout = (u16*)x->chain[l & 1];
            a.wbf = wb + WBFB; a.wrb = wb + WRBFB;
            a.mu = (const uint16_t*)mu; a.me = (const uint16_t*)me;
            a.zero = (const u16*)x->zero;
            a.B = c.batch; a.T = c.T; a.d = d; a.n = c.T / d;
            if (!a.tin) return fail(AST_E_STATE, "top block has no loss gradient");
            launch_block_bwd_c(a, s);
        } else {
            BwdArgs a;
            a.gin = (const float*)gin; a.din = (const float*)din; a.gout = (float*)x->chain[l & 1];
            a.wr = w + WR; a.wrT = w + WRT; a.wdT = w + WDT;
            a.mu = mu; a.me = me;
            a.B = c.batch; a.T = c.T; a.d = d; a.n = c.T / d;
            launch_block_bwd(a, s);
        }
    }
    tmark(x, s);
    if (x->split) launch_startx_gx((const float*)x->chain[0], grad, c.batch, c.T, s);
    else if (x->bf) launch_startconv_bwd((const u16*)x->chain[0], grad, x->wts + W0_OFF, c.batch, c.T, s);
    else launch_startconv_bwd((const float*)x->chain[0], grad, x->wts + W0_OFF, c.batch, c.T, s);
    const int nb = std::min(c.nb_channels, C);
    if (c.gatys)
        launch_finalize(parts, x->cpart, x->ncpart, 10.0f / ((float)c.T * (float)x->ncc), x->spart,
                        x->nu, 1e3f / (float)(x->L * C * C), c.lambd, c.batch, s);
    else
        launch_finalize(parts, x->cpart, x->ncpart, 10.0f / ((float)c.T * (float)x->ncc), x->spart,
                        C, 1e3f / (float)(nb * x->L * x->L), c.lambd, c.batch, s);
    // STFT regulariser (methods.py:121-125): TF evaluates it whatever gamma is, so parts[3]
    // always holds it; its gradient enters grad only through gamma
    launch_stft_reg(xd, x->stft_tw, x->stft_fpart, x->stft_gfr, grad, parts, c.gamma, c.batch,
                    c.T, s);
    {
        RangeArgs ra;
        memset(&ra, 0, sizeof(ra));
        ra.parts = parts; ra.grad = grad;
        ra.gmax_e = x->gmax_e; ra.gmax_g = x->gmax_g;
        ra.split = x->split; ra.nblk = x->nblk; ra.B = c.batch; ra.T = c.T;
        for (int l = 0; l < NBLK_MAX; ++l) { ra.wdn[l] = x->wdn[l]; ra.bdm[l] = x->bdm[l]; ra.wrn[l] = x->wrn[l]; }
        ra.flags = x->rflags;
        ra.last = x->rflags_last;
        launch_range_flags(ra, s);
    }
    tmark(x, s);
    HIPCHK(hipGetLastError());
    if (x->timing && x->ev_used <= (int)x->ev.size()) x->timed_calls++;
    x->fwd_done = false;   // tapped tensors now hold their gradients, not activations
    return 0;
}


int ast_loss_grad(ast_ctx* x, const float* xd, float* grad, float* parts, void* stream) {
    return ast_loss_grad_phase(x, xd, grad, parts, 0, stream);
}

int ast_loss_grad_phase(ast_ctx* x, const float* xd, float* grad, float* parts, int phase, void* stream) {
    if (!x || !xd || ((phase == 0 || phase == 2) && (!grad || !parts))) return fail(AST_E_ARG, "null argument");
    if (phase < 0 || phase > 2) return fail(AST_E_ARG, "phase must be 0 (both), 1 (front) or 2 (back)");
    if (!x->targets) return fail(AST_E_STATE, "ast_set_targets has not been called");
    (void)hipSetDevice(x->dev);
    hipStream_t s = S(stream);
    if (phase != 2) {
        const int rc = loss_grad_front(x, xd, s);
        if (rc) return rc;
    } else if (!x->lg_front_done) {
        return fail(AST_E_STATE, "ast_loss_grad_phase(2) needs phase 1 first");
    }
    if (phase == 1) return 0;
    return loss_grad_back(x, xd, grad, parts, s);
}

int ast_range_flags(ast_ctx* x, int* flags, void* stream) {
    if (!x || !flags) return fail(AST_E_ARG, "null argument");
    HIPCHK(hipMemcpyAsync(flags, x->rflags, (size_t)x->cfg.batch * 4, hipMemcpyDeviceToDevice, S(stream)));
    return 0;
}

int ast_range_flags_last(ast_ctx* x, int* flags, void* stream) {
    if (!x || !flags) return fail(AST_E_ARG, "null argument");
    HIPCHK(hipMemcpyAsync(flags, x->rflags_last, (size_t)x->cfg.batch * 4, hipMemcpyDeviceToDevice, S(stream)));
    return 0;
}

int ast_set_cu_limit(ast_ctx* x, int cus) {
    if (!x) return fail(AST_E_ARG, "null argument");
    if (cus < 0) return fail(AST_E_ARG, "cu limit must be >= 0 (0 = every CU)");
    x->cus = cus;
    return 0;
}

int ast_range_flags_reset(ast_ctx* x, void* stream) {
    if (!x) return fail(AST_E_ARG, "null argument");
    launch_zero32(x->rflags, (size_t)x->cfg.batch * 4, S(stream), 3);
    return 0;
}

int ast_adam_step(ast_ctx* x, float* xd, float* m, float* v, const float* grad, int step,
                  float lr, float b1, float b2, float eps, void* stream) {
    if (!x || !xd || !m || !v || !grad || step < 1) return fail(AST_E_ARG, "bad argument");
    const float bc1 = 1.0f - pow_int(b1, step), bc2 = 1.0f - pow_int(b2, step);
    launch_adam(xd, m, v, grad, (size_t)x->cfg.batch * x->cfg.T, lr, b1, b2, eps, bc1, bc2, S(stream));
    HIPCHK(hipGetLastError());
    return 0;
}

int ast_adam_step_dev(ast_ctx* x, float* xd, float* m, float* v, const float* grad, int* step_dev,
                      float lr, float b1, float b2, float eps, void* stream) {
    if (!x || !xd || !m || !v || !grad || !step_dev) return fail(AST_E_ARG, "bad argument");
    launch_adam_dev(xd, m, v, grad, (size_t)x->cfg.batch * x->cfg.T, step_dev, lr, b1, b2, eps, S(stream));
    HIPCHK(hipGetLastError());
    return 0;
}

int ast_lbfgs_workspace_bytes(ast_ctx* x, int m, size_t* out) {
    if (!x || !out) return fail(AST_E_ARG, "null argument");
    if (m < 1 || m > 32) return fail(AST_E_ARG, "L-BFGS-B history m must be in 1..32");
    *out = lbfgs_workspace_bytes(x->cfg.batch, x->cfg.T, m);
    return 0;
}

int ast_lbfgs_begin(ast_ctx* x, void* ws, float* xd, const double* x0, const int* active, int m,
                    int maxiter, int maxls, double ftol, double gtol, void* stream) {
    if (!x || !ws || !xd) return fail(AST_E_ARG, "null argument");
    if (m < 1 || m > 32) return fail(AST_E_ARG, "L-BFGS-B history m must be in 1..32");
    if (maxiter < 1 || maxls < 1) return fail(AST_E_ARG, "maxiter and maxls must be >= 1");
    // every evaluation of the call must fit the per-call loss history (ast_lbfgs_history): at
    // most 1 + maxiter (maxls + 1) of them
    if ((long long)maxiter * (maxls + 1) + 1 > lbfgs_history_cap())
        return fail(AST_E_ARG, "maxiter * (maxls + 1) + 1 exceeds AST_LBFGS_HISTORY evaluations");
    const bool known = std::find(x->lb_ws.begin(), x->lb_ws.end(), ws) != x->lb_ws.end();
    if (!x0 && !known)
        return fail(AST_E_STATE, "continuing (x0 NULL) needs a workspace started with x0");
    if (x0 && !known) x->lb_ws.push_back(ws);
    // a new epoch: the range flags accumulate over its evaluations (include/astyle.h)
    launch_zero32(x->rflags, (size_t)x->cfg.batch * 4, S(stream), 3);
    launch_lbfgs_begin(ws, xd, x0, active, x->cfg.batch, x->cfg.T, m, maxiter, maxls, ftol, gtol,
                       S(stream));
    HIPCHK(hipGetLastError());
    return 0;
}

int ast_lbfgs_step(ast_ctx* x, void* ws, float* xd, const float* grad, const float* parts,
                   void* stream) {
    if (!x || !ws || !xd || !grad || !parts) return fail(AST_E_ARG, "null argument");
    if (std::find(x->lb_ws.begin(), x->lb_ws.end(), ws) == x->lb_ws.end())
        return fail(AST_E_STATE, "ast_lbfgs_begin (with x0) has not been called on this workspace");
    launch_lbfgs_step(ws, xd, grad, parts, x->cfg.batch, x->cfg.T, S(stream));
    HIPCHK(hipGetLastError());
    return 0;
}

int ast_lbfgs_state(ast_ctx* x, const void* ws, int* info, double* x64, void* stream) {
    if (!x || !ws || !info) return fail(AST_E_ARG, "null argument");
    if (std::find(x->lb_ws.begin(), x->lb_ws.end(), ws) == x->lb_ws.end())
        return fail(AST_E_STATE, "ast_lbfgs_begin (with x0) has not been called on this workspace");
    launch_lbfgs_state(ws, info, x64, x->cfg.batch, x->cfg.T, S(stream));
    HIPCHK(hipGetLastError());
    return 0;
}

int ast_lbfgs_history(ast_ctx* x, const void* ws, float* out, int max_evals, void* stream) {
    if (!x || !ws || !out) return fail(AST_E_ARG, "null argument");
    if (max_evals < 1 || max_evals > lbfgs_history_cap())
        return fail(AST_E_ARG, "max_evals must be in 1..AST_LBFGS_HISTORY");
    if (std::find(x->lb_ws.begin(), x->lb_ws.end(), ws) == x->lb_ws.end())
        return fail(AST_E_STATE, "ast_lbfgs_begin (with x0) has not been called on this workspace");
    launch_lbfgs_history(ws, out, max_evals, x->cfg.batch, x->cfg.T, S(stream));
    HIPCHK(hipGetLastError());
    return 0;
}

// Event layout per timed ast_loss_grad call (8 marks):
//  m0 start | startconv | m1 | blocks fwd | m2 | content | m3 gram fwd m4 style m5 gram bwd m6
//  | blocks bwd | m7 | startconv bwd + finalize | m8
int ast_timing(ast_ctx* x, int enable) {
    if (!x) return fail(AST_E_ARG, "null argument");
    (void)hipSetDevice(x->dev);
    if (enable) {
        if (x->ev.empty()) {
            x->ev.resize(9 * 512);
            for (auto& e : x->ev) HIPCHK(hipEventCreate(&e));
        }
        x->ev_used = 0;
        x->timed_calls = 0;
    }
    x->timing = enable != 0;
    return 0;
}

int ast_timing_read(ast_ctx* x, float* out, int n) {
    if (!x || !out) return fail(AST_E_ARG, "null argument");
    float fam[NFAM] = {0, 0, 0, 0, 0};
    const int per = 9;
    const int calls = std::min(x->timed_calls, x->ev_used / per);
    for (int k = 0; k < calls; ++k) {
        hipEvent_t* e = &x->ev[(size_t)k * per];
        float t[8];
        for (int i = 0; i < 8; ++i) {
            HIPCHK(hipEventSynchronize(e[i + 1]));
            HIPCHK(hipEventElapsedTime(&t[i], e[i], e[i + 1]));
        }
        fam[0] += t[1];                  // blocks fwd
        fam[1] += t[6];                  // blocks bwd
        fam[2] += t[3];                  // gram fwd
        fam[3] += t[5];                  // gram bwd
        fam[4] += t[0] + t[2] + t[4] + t[7];
    }
    float vals[7] = {fam[0], fam[1], fam[2], fam[3], fam[4], (float)calls, (float)x->nblk};
    for (int i = 0; i < n && i < 7; ++i) out[i] = vals[i];
    return 0;
}

}  // extern "C"
