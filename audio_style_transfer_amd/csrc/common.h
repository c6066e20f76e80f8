// Shared definitions for the gfx950 kernels of libastyle.so.
//
// Data layout in HBM (per context, B clips of T samples, C = 128 channels):
//   act   [NB+1][B][T][C]   encoder tensors e_0 (startconv) .. e_NB; e_{l+1} = extracts[l]
//                           (model.py:116); channels-last so a time row is one 512-B line
//                           group (fp32).  Tapped tensors are overwritten in place by their
//                           direct loss gradient D during the Gram backward.
//   mu/me [NB][B][T][4]     u>0 / e_l>0 relu masks, one bit per channel (16 B per row)
//   chain [2][B][T][C]      fp32 backward ping-pong (d loss / d e_l)
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
constexpr int GT = 32;        // Gram: time rows per stage
constexpr int GCH = 16;       // Gram: channels per workgroup
constexpr int GRS = 17;       // Gram LDS row stride (floats)
constexpr int GLS = GT * GRS + 1;   // Gram LDS layer stride (545: odd -> conflict-free)

typedef float f32x16 __attribute__((ext_vector_type(16)));

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

struct GramArgs {
    const float* act; size_t tstride;      // tensor u lives at act + uid[u] * tstride
    float* actw;                            // same base, writable (bwd, in place)
    int nu; int uid[32];
    const float* cg[32];                    // content grad per unique tensor (bwd) or null
    float* gpart;                           // [B][nchunk][C][32][32]
    const float* smat;                      // [B][C][32][32]
    int B, T, nchunk;
};

struct StyleArgs {
    const float* gpart; int nchunk;
    int L; int lmap[32]; int nu;
    const float* phi; size_t phi_bstride;   // elements between clips (0 = shared)
    int nb; float coef;                     // coef = lambd * 1e3 * 2 / (nb * L * L)
    float* smat; float* spart;              // [B][C][32][32], [B][C]
    float* embs;                            // optional normalised Gram out [B][nb][L][L]
    int B;
};

struct ContentArgs {
    const float* e; int W;                  // tensor [B][T][W]
    const float* phi; size_t phi_bstride;   // [B|1][T][ncc]
    int ncc, off, ncol;
    float coef;                             // 10 * 2 / (T * ncc)
    float* cg; int accumulate;              // [B][T][W]
    float* lpart; size_t lstride;           // partial sums at lpart[b * lstride + tile]
    float* embc;                            // optional: write e[..., :ncol] into emb [B][T][ncc]
    int B, T;
};

// launchers (encoder.hip / gram.hip / optim.hip)
void launch_startconv_fwd(const float* x, float* e0, const float* w0, const float* b0,
                          int B, int T, hipStream_t s);
void launch_startconv_bwd(const float* g0, float* gx, const float* w0, int B, int T,
                          hipStream_t s);
void launch_block_fwd(const FwdArgs& a, hipStream_t s);
void launch_block_bwd(const BwdArgs& a, hipStream_t s);
void launch_bottleneck_fwd(const float* e, float* y, const float* wb, const float* bb,
                           int B, int T, hipStream_t s);
void launch_bottleneck_bwd(const float* gy, float* ge, const float* wb, int accumulate,
                           int B, int T, hipStream_t s);
void launch_gram_fwd(const GramArgs& a, hipStream_t s);
void launch_gram_bwd(const GramArgs& a, hipStream_t s);
void launch_style_ours(const StyleArgs& a, hipStream_t s);
void launch_content(const ContentArgs& a, hipStream_t s);
constexpr int CROWS = 64;   // rows per content workgroup
void launch_finalize(float* parts, const float* cpart, int ncpart, float cscale,
                     const float* spart, int nspart, float sscale, float lambd, int B,
                     hipStream_t s);
void launch_adam(float* x, float* m, float* v, const float* g, size_t n, float lr, float b1,
                 float b2, float eps, float bc1, float bc2, hipStream_t s);

}  // namespace ast
