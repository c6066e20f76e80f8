// Channel-wise ("ours") Gram, l2-normalise, style/content losses and their gradients
// (methods.py:58-76, 113-125) on gfx950.
//
// The fp32 Gram kernels themselves (fwd G_c = E_c E_c^T, bwd D_c = S~_c E_c in place over E)
// are in gram_split.hip beside the split ones, which share their staging.
#include "common.h"

namespace ast {

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
    return v;
}

// One wave per (clip, channel): sum chunk partials, expand unique -> list, l2-normalise
// (methods.py:74), style loss vs phi (methods.py:118-119), d loss / d G, fold S = dG + dG^T
// back onto unique tensors.
__global__ void __launch_bounds__(256) k_style_ours(StyleArgs a) {
    __shared__ float Gu[4][32 * 33];
    __shared__ float dG[4][32 * 33];
    __shared__ float St[4][32 * 32];
    __shared__ uint16_t EL[1024];       // list element e -> (l << 8) | l2 (one division per block)
    __shared__ int lm[32];              // tap -> unique tensor (a by-value kernel-argument array
                                        // indexed at run time would live in scratch)
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int L = a.L, LL = L * L;
    if (tid < 32) lm[tid] = a.lmap[tid];
    for (int e = tid; e < LL; e += 256) EL[e] = (uint16_t)(((e / L) << 8) | (e % L));
    const int b = blockIdx.x / (C / 4);
    const int c = (blockIdx.x % (C / 4)) * 4 + w;
    // chunk partials: 16 independent loads in flight per lane (a serial chain of dependent
    // load-add pairs ran at 1.6 TB/s); the sum order over chunks is fixed (ch ascending)
    const float* gp = a.gpart + ((size_t)b * a.nchunk * C + c) * 1024;
    const size_t cs = (size_t)C * 1024;
    for (int e0 = 0; e0 < 1024; e0 += 256) {
        float s[4] = {0.f, 0.f, 0.f, 0.f};
        int ch = 0;
        for (; ch + 4 <= a.nchunk; ch += 4) {
            float v[4][4];
#pragma unroll
            for (int q = 0; q < 4; ++q)
#pragma unroll
                for (int k = 0; k < 4; ++k) v[q][k] = gp[(ch + q) * cs + e0 + 64 * k + lane];
#pragma unroll
            for (int q = 0; q < 4; ++q)
#pragma unroll
                for (int k = 0; k < 4; ++k) s[k] += v[q][k];
        }
        for (; ch < a.nchunk; ++ch)
#pragma unroll
            for (int k = 0; k < 4; ++k) s[k] += gp[ch * cs + e0 + 64 * k + lane];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int e = e0 + 64 * k + lane;
            Gu[w][(e >> 5) * 33 + (e & 31)] = s[k];
            St[w][e] = 0.f;
        }
    }
    __syncthreads();
    // the list Gram is re-read from LDS wherever needed: per-lane copies of the <= 16
    // elements a lane owns would cost ~250 registers and one wave per SIMD
    auto gval = [&](int e) {
        const uint32_t el = EL[e];
        return Gu[w][lm[el >> 8] * 33 + lm[el & 255]];
    };
    auto lidx = [&](int e) {
        const uint32_t el = EL[e];
        return (int)(el >> 8) * 33 + (int)(el & 255);
    };
    float ss = 0.f;
    for (int e = lane; e < LL; e += 64) {
        const float g = gval(e);
        ss = fmaf(g, g, ss);
    }
    ss = wave_sum(ss);
    const float inv = 1.0f / sqrtf(fmaxf(ss, 1e-12f));
    const bool active = c < a.nb;
    const float* phi = a.phi ? a.phi + (size_t)b * a.phi_bstride + (size_t)c * LL : nullptr;
    float sd = 0.f, dot = 0.f;
    for (int e = lane; e < LL; e += 64) {     // d loss / d Gn (raw), loss partial, <Gn, dGn>
        float dgn = 0.f;
        if (active) {
            const float gn = gval(e) * inv;
            if (a.embs) a.embs[(((size_t)b * a.nb) + c) * LL + e] = gn;
            if (phi) {
                const float diff = gn - phi[e];
                sd = fmaf(diff, diff, sd);
                dgn = a.coef * diff;
                dot = fmaf(gn, dgn, dot);
            }
        }
        dG[w][lidx(e)] = dgn;
    }
    sd = wave_sum(sd);
    dot = wave_sum(dot);
    const float big = ss >= 1e-12f ? 1.f : 0.f;
    for (int e = lane; e < LL; e += 64) {     // l2-normalise backward (each lane its own elements)
        const int i = lidx(e);
        dG[w][i] = dG[w][i] * inv - big * (gval(e) * inv) * dot * inv;
    }
    __syncthreads();
    for (int e = lane; e < LL; e += 64) {     // S = dG + dG^T folded onto unique tensors
        const uint32_t el = EL[e];
        const int l = el >> 8, l2 = el & 255;
        const float sv = dG[w][l * 33 + l2] + dG[w][l2 * 33 + l];
        if (a.lmap_identity) St[w][l * 32 + l2] = sv;     // every tap its own tensor
        else atomicAdd(&St[w][lm[l] * 32 + lm[l2]], sv);
    }
    __syncthreads();
    if (a.smat) {
        float* dst = a.smat + ((size_t)b * C + c) * 1024;
        for (int e = lane; e < 1024; e += 64) dst[e] = St[w][e];
    }
    if (lane == 0 && a.spart) a.spart[(size_t)b * C + c] = sd;
}

// Content taps (methods.py:58,116-117): cg = coef * (E[..., :ncol] - phi[..., off:off+ncol]),
// partial sums of the squared error per CROWS rows.  Optionally copies the tap into emb.
template <typename TE, typename TG>
__global__ void __launch_bounds__(256) k_content(ContentArgs a) {
    __shared__ float red[4];
    const TE* E = (const TE*)a.e;
    TG* CG = (TG*)a.cg;
    const int tilesPer = a.T / CROWS;
    const int b = blockIdx.x / tilesPer;
    const int t0 = (blockIdx.x - b * tilesPer) * CROWS;
    const int tid = threadIdx.x;
    float sd = 0.f;
    for (int i = tid; i < CROWS * a.W; i += 256) {
        const int tt = i / a.W, c = i - tt * a.W;
        const size_t row = (size_t)b * a.T + t0 + tt;
        const float e = ldv(E, row * a.W + c);
        float d = 0.f;
        if (c < a.ncol) {
            if (a.embc) a.embc[row * a.ncc + a.off + c] = e;
            if (a.phi) {
                d = e - a.phi[(size_t)b * a.phi_bstride + (size_t)(t0 + tt) * a.ncc + a.off + c];
                sd = fmaf(d, d, sd);
            }
        }
        if (CG) {
            const float gv = a.coef * d;
            stv(CG, row * a.W + c, a.accumulate ? ldv(CG, row * a.W + c) + gv : gv);
        }
    }
    sd = wave_sum(sd);
    if ((tid & 63) == 0) red[tid >> 6] = sd;
    __syncthreads();
    if (tid == 0 && a.lpart)
        a.lpart[(size_t)b * a.lstride + (blockIdx.x - b * tilesPer)] = red[0] + red[1] + red[2] + red[3];
}

// Same for the common bf16 case (128-channel tap, bf16 e and cg, ncol a multiple of 8, no emb
// copy): one thread per 16-B chunk of e / cg, the matching 32 B of phi as two float4.
__global__ void __launch_bounds__(256) k_content_bf16x8(ContentArgs a) {
    __shared__ float red[4];
    const u16* E = (const u16*)a.e;
    u16* CG = (u16*)a.cg;
    const int tilesPer = a.T / CROWS;
    const int b = blockIdx.x / tilesPer;
    const int t0 = (blockIdx.x - b * tilesPer) * CROWS;
    const int tid = threadIdx.x;
    float sd = 0.f;
#pragma unroll
    for (int it = 0; it < CROWS * (C / 8) / 256; ++it) {
        const int i = it * 256 + tid;
        const int tt = i >> 4, ch = i & 15;
        const size_t row = (size_t)b * a.T + t0 + tt;
        const uint4 ev = *reinterpret_cast<const uint4*>(E + row * C + ch * 8);
        float d[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
        if (ch * 8 < a.ncol && a.phi) {
            const float* ph = a.phi + (size_t)b * a.phi_bstride + (size_t)(t0 + tt) * a.ncc + a.off + ch * 8;
            const float4 p0 = *reinterpret_cast<const float4*>(ph);
            const float4 p1 = *reinterpret_cast<const float4*>(ph + 4);
            const float pv[8] = {p0.x, p0.y, p0.z, p0.w, p1.x, p1.y, p1.z, p1.w};
            const uint32_t eu[4] = {ev.x, ev.y, ev.z, ev.w};
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                d[2 * k] = bflo(eu[k]) - pv[2 * k];
                d[2 * k + 1] = bfhi(eu[k]) - pv[2 * k + 1];
            }
#pragma unroll
            for (int k = 0; k < 8; ++k) sd = fmaf(d[k], d[k], sd);
        }
        if (CG) {
            uint32_t o[4];
            u16* cp = CG + row * C + ch * 8;
            if (a.accumulate) {
                const uint4 old = *reinterpret_cast<const uint4*>(cp);
                const uint32_t ou[4] = {old.x, old.y, old.z, old.w};
#pragma unroll
                for (int k = 0; k < 4; ++k)
                    o[k] = pack2(bflo(ou[k]) + a.coef * d[2 * k], bfhi(ou[k]) + a.coef * d[2 * k + 1]);
            } else {
#pragma unroll
                for (int k = 0; k < 4; ++k) o[k] = pack2(a.coef * d[2 * k], a.coef * d[2 * k + 1]);
            }
            *reinterpret_cast<uint4*>(cp) = make_uint4(o[0], o[1], o[2], o[3]);
        }
    }
    sd = wave_sum(sd);
    if ((tid & 63) == 0) red[tid >> 6] = sd;
    __syncthreads();
    if (tid == 0 && a.lpart)
        a.lpart[(size_t)b * a.lstride + (blockIdx.x - b * tilesPer)] = red[0] + red[1] + red[2] + red[3];
}

// parts[b] = (content + lambd*style, content, style, 0)
__global__ void __launch_bounds__(256) k_finalize(float* parts, const float* cpart, int ncpart,
                                                  float cscale, const float* spart, int nspart,
                                                  float sscale, float lambd) {
    __shared__ float red[2][4];
    const int b = blockIdx.x, tid = threadIdx.x;
    float cs = 0.f, st = 0.f;
    if (cpart)
        for (int i = tid; i < ncpart; i += 256) cs += cpart[(size_t)b * ncpart + i];
    if (spart)
        for (int i = tid; i < nspart; i += 256) st += spart[(size_t)b * nspart + i];
    cs = wave_sum(cs);
    st = wave_sum(st);
    if ((tid & 63) == 0) { red[0][tid >> 6] = cs; red[1][tid >> 6] = st; }
    __syncthreads();
    if (tid == 0) {
        const float content = (red[0][0] + red[0][1] + red[0][2] + red[0][3]) * cscale;
        const float style = (red[1][0] + red[1][1] + red[1][2] + red[1][3]) * sscale;
        parts[b * 4 + 0] = content + lambd * style;
        parts[b * 4 + 1] = content;
        parts[b * 4 + 2] = style;
        parts[b * 4 + 3] = 0.f;
    }
}

// Per-clip flags (include/astyle.h AST_RANGE_*), OR'ed into the context's accumulated flags: non-finite loss parts or gradient; in split
// mode also every per-clip maximum the split-fp16 scales were derived from (splitwave.h
// scale_exp: in range for maxima in [2^-47, 2^74)) and the analytic intermediate bounds
// |u| <= wdn max|e_l| + bdm, |W_r tot| <= wrn max|tot|: beyond 2^74 the scaled halves would
// overflow fp16; below 2^-60 they lose significand bits.
__global__ void __launch_bounds__(256) k_range_flags(RangeArgs a) {
    // (round 6: float4 loads, four in flight per thread, and the per-level bound checks spread
    // over threads; one clip 20 -> ~5 us.  The same flags.)
    const int b = blockIdx.x, tid = threadIdx.x;
    __shared__ int sf;
    if (tid == 0) sf = 0;
    int f = 0;
    const float* g = a.grad + (size_t)b * a.T;
    if ((a.T & 3) == 0 && (reinterpret_cast<uintptr_t>(g) & 15) == 0) {
        const float4* g4 = reinterpret_cast<const float4*>(g);
        const int n4 = a.T >> 2;
        for (int i = tid; i < n4; i += 4 * 256) {
            float4 v[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) v[k] = i + 256 * k < n4 ? g4[i + 256 * k] : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
            for (int k = 0; k < 4; ++k)
                if (!isfinite(v[k].x) || !isfinite(v[k].y) || !isfinite(v[k].z) || !isfinite(v[k].w)) f = 1;
        }
    } else {
        for (int i = tid; i < a.T; i += 256)
            if (!isfinite(g[i])) f = 1;
    }
    if (tid < 4 && !isfinite(a.parts[b * 4 + tid])) f = 1;
    if (a.split && tid <= a.nblk) {   // level t = tid of the chain's operand bounds
        const float hi = 0x1p74f, lo = 0x1p-60f;
        auto chk = [&](float m, int bit) {
            if (!(m < hi)) f |= bit;
            else if (m > 0.f && m < lo) f |= 8;
        };
        const int t = tid;
        auto gread = [&](const unsigned* g, int lv) {   // the clip's max over its slots (common.h)
            const unsigned* p = g + ((size_t)lv * a.B + b) * GCLIP_W;
            unsigned m = 0;
#pragma unroll
            for (int q = 0; q < GSLOTS; ++q) m = max(m, p[q * GSLOT_W]);
            return __uint_as_float(m);
        };
        const float ge = gread(a.gmax_e, t);
        const float gg = gread(a.gmax_g, t);
        chk(ge, 2);
        chk(gg, 4);
        if (t < a.nblk) {
            if (!(fmaf(a.wdn[t], ge, a.bdm[t]) < hi)) f |= 2;
            const float gn = gread(a.gmax_g, t + 1);
            if (!(a.wrn[t] * gn < hi)) f |= 4;
        }
    }
    __syncthreads();
    if (f) atomicOr(&sf, f);
    __syncthreads();
    if (tid) return;
    f = sf;
    a.flags[b] |= f;   // sticky until ast_range_flags_reset / ast_lbfgs_begin
    a.last[b] = f;     // ast_range_flags_last: this evaluation only
}

void launch_range_flags(const RangeArgs& a, hipStream_t s) {
    hipLaunchKernelGGL(k_range_flags, dim3(a.B), dim3(256), 0, s, a);
}

void launch_style_ours(const StyleArgs& a, hipStream_t s) {
    hipLaunchKernelGGL(k_style_ours, dim3(a.B * (C / 4)), dim3(256), 0, s, a);
}
void launch_content(const ContentArgs& a, hipStream_t s) {
    const dim3 g(a.B * (a.T / CROWS));
    const bool x8 = a.e_bf16 && a.cg_bf16 && a.W == C && a.ncol % 8 == 0 && a.off % 4 == 0 &&
                    a.ncc % 4 == 0 && !a.embc;
    if (x8) hipLaunchKernelGGL(k_content_bf16x8, g, dim3(256), 0, s, a);
    else if (a.e_bf16 && a.cg_bf16) hipLaunchKernelGGL((k_content<u16, u16>), g, dim3(256), 0, s, a);
    else if (a.e_bf16) hipLaunchKernelGGL((k_content<u16, float>), g, dim3(256), 0, s, a);
    else if (a.cg_bf16) hipLaunchKernelGGL((k_content<float, u16>), g, dim3(256), 0, s, a);
    else hipLaunchKernelGGL((k_content<float, float>), g, dim3(256), 0, s, a);
}
void launch_finalize(float* parts, const float* cpart, int ncpart, float cscale,
                     const float* spart, int nspart, float sscale, float lambd, int B,
                     hipStream_t s) {
    hipLaunchKernelGGL(k_finalize, dim3(B), dim3(256), 0, s, parts, cpart, ncpart, cscale,
                       spart, nspart, sscale, lambd);
}

// Adam on the audio buffer (the north_star's optimiser; bias-corrected, PyTorch semantics).
__global__ void __launch_bounds__(256) k_adam(float* __restrict__ x, float* __restrict__ m,
                                              float* __restrict__ v,
                                              const float* __restrict__ g, size_t n, float lr,
                                              float b1, float b2, float eps, float bc1,
                                              float bc2) {
    const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const float gi = g[i];
    const float mi = b1 * m[i] + (1.f - b1) * gi;
    const float vi = b2 * v[i] + (1.f - b2) * gi * gi;
    m[i] = mi;
    v[i] = vi;
    x[i] -= lr * (mi / bc1) / (sqrtf(vi / bc2) + eps);
}

// device-counter form: step = *step_dev + 1 (bias corrections computed per thread)
__global__ void __launch_bounds__(256) k_adam_dev(float* __restrict__ x, float* __restrict__ m,
                                                  float* __restrict__ v,
                                                  const float* __restrict__ g, size_t n,
                                                  const int* __restrict__ step_dev, float lr,
                                                  float b1, float b2, float eps) {
    const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const int st = *step_dev + 1;
    const float bc1 = 1.f - pow_int(b1, st), bc2 = 1.f - pow_int(b2, st);
    const float gi = g[i];
    const float mi = b1 * m[i] + (1.f - b1) * gi;
    const float vi = b2 * v[i] + (1.f - b2) * gi * gi;
    m[i] = mi;
    v[i] = vi;
    x[i] -= lr * (mi / bc1) / (sqrtf(vi / bc2) + eps);
}

__global__ void k_step_inc(int* step_dev) { *step_dev += 1; }

void launch_adam_dev(float* x, float* m, float* v, const float* g, size_t n, int* step_dev,
                     float lr, float b1, float b2, float eps, hipStream_t s) {
    hipLaunchKernelGGL(k_adam_dev, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, x, m, v, g,
                       n, step_dev, lr, b1, b2, eps);
    hipLaunchKernelGGL(k_step_inc, dim3(1), dim3(1), 0, s, step_dev);
}

void launch_adam(float* x, float* m, float* v, const float* g, size_t n, float lr, float b1,
                 float b2, float eps, float bc1, float bc2, hipStream_t s) {
    hipLaunchKernelGGL(k_adam, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, x, m, v, g,
                       n, lr, b1, b2, eps, bc1, bc2);
}

}  // namespace ast
