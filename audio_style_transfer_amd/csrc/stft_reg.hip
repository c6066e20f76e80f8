// STFT regulariser of define_loss (methods.py:121-123) and its gradient to x, on the device.
//
//   reg = mean_{f,k} abs(Re S[f,k]) + abs(Im S[f,k]),
//   S   = stft(inv_mu_law(x), frame 1024, hop 512, periodic Hann, fft 1024, no pad_end) [nf, 513]
//   abs(v) = max(v, 1e-12) + max(0, -v), inv_mu_law the TF version (utils.py:92-104)
//
// k_stft_frames: one 256-thread workgroup per (clip, frame).  The frame (4 KB) is loaded once,
// mapped through inv_mu_law and the window, and transformed by a 1024-point radix-4 Stockham
// FFT in LDS (5 stages, one butterfly per thread per stage, twiddles from an LDS copy of the
// context's fp64-rounded table).  The 513 half-spectrum bins give the frame's partial sum;
// the gradient of the bins, d abs / d v = [v >= 1e-12] - [v < 0] (TF Maximum routes the
// gradient to its first input on ties), goes back through the same FFT:
//   d reg / d (w a)[n] = Re sum_{k<=512} (gre_k + i gim_k) e^{+2 pi i k n / N}
//                      = Re FFT(conj(gre + i gim))[n],
// times the window, stored per frame (fp32 [B][nf][1024]).
// k_stft_ola: overlap-add of the two frames that cover each sample, times d inv_mu_law / d x,
// times gamma, added to grad; the per-frame partials are summed in frame order (deterministic)
// into parts[b][3] and gamma * reg into parts[b][0].
// Work per clip is ~0.1 MFLOP per frame; the pair is HBM/latency bound at ~3 x 4 B per sample.
#include "common.h"

namespace ast {
namespace {

constexpr int NF = 1024;       // frame / fft length (tf.contrib.signal.stft defaults)
constexpr int HOP = 512;
constexpr int NBIN = NF / 2 + 1;

__device__ __forceinline__ float abs_tf(float v) { return fmaxf(v, 1e-12f) + fmaxf(0.f, -v); }
__device__ __forceinline__ float abs_tf_grad(float v) {
    return (v >= 1e-12f ? 1.f : 0.f) - (v < 0.f ? 1.f : 0.f);
}

// utils.py:99-104 inv_mu_law (TF version): value
__device__ __forceinline__ float inv_mu_law(float x) {
    const float o = (x + 0.5f) * (2.f / 256.f);
    const float a = abs_tf(o);
    const float num = fabsf(o) <= 1e-12f ? 0.f : o;
    const float out = num / a / 255.f * (exp2f(8.f * a) - 1.f);   // 256^a = 2^(8a)
    return x == 0.f ? x : out;
}

// ... and d value / d x (same formula as the oracle's inv_mu_law_tf)
__device__ __forceinline__ float inv_mu_law_grad(float x) {
    const float o = (x + 0.5f) * (2.f / 256.f);
    const float a = abs_tf(o);
    const float da = abs_tf_grad(o);
    const bool tiny = fabsf(o) <= 1e-12f;
    const float num = tiny ? 0.f : o;
    const float dnum = tiny ? 0.f : 1.f;
    const float sgn = num / a;
    const float dsgn = (dnum * a - num * da) / (a * a);
    const float p = exp2f(8.f * a);
    const float dp = p * 5.545177444479562f * da;                    // ln 256
    const float dout = (dsgn * (p - 1.f) + sgn * dp) / 255.f * (2.f / 256.f);
    return x == 0.f ? 1.f : dout;
}

__device__ __forceinline__ float2 cmul(float2 a, float2 b) {
    return make_float2(a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x);
}

// One Stockham radix-4 pass set: src -> ... -> result; returns the buffer holding the result.
// 5 passes (Ns = 1, 4, 16, 64, 256), each thread one butterfly of 4 points per pass.
__device__ __forceinline__ float2* fft1024(float2* src, float2* dst, const float2* tw, int j) {
#pragma unroll
    for (int Ns = 1; Ns < NF; Ns *= 4) {
        const int k = j & (Ns - 1);
        const int step = k * (256 / Ns);
        float2 v0 = src[j];
        float2 v1 = cmul(src[j + 256], tw[step]);
        float2 v2 = cmul(src[j + 512], tw[2 * step]);
        float2 v3 = cmul(src[j + 768], tw[3 * step]);
        const float2 s02 = make_float2(v0.x + v2.x, v0.y + v2.y);
        const float2 d02 = make_float2(v0.x - v2.x, v0.y - v2.y);
        const float2 s13 = make_float2(v1.x + v3.x, v1.y + v3.y);
        const float2 d13 = make_float2(v1.x - v3.x, v1.y - v3.y);
        const int o = (j / Ns) * Ns * 4 + k;
        dst[o] = make_float2(s02.x + s13.x, s02.y + s13.y);            // X0
        dst[o + Ns] = make_float2(d02.x + d13.y, d02.y - d13.x);       // X1 = d02 - i d13
        dst[o + 2 * Ns] = make_float2(s02.x - s13.x, s02.y - s13.y);   // X2
        dst[o + 3 * Ns] = make_float2(d02.x - d13.y, d02.y + d13.x);   // X3 = d02 + i d13
        __syncthreads();
        float2* t = src; src = dst; dst = t;
    }
    return src;
}

__device__ __forceinline__ float wave_sum_f(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    return v;
}

__global__ void __launch_bounds__(256) k_stft_frames(const float* __restrict__ x,
                                                     const float2* __restrict__ twg,
                                                     float* __restrict__ fpart,
                                                     float* __restrict__ gfr, int T, int nf,
                                                     int with_grad, float inv_nbins) {
    __shared__ float2 buf[2][NF];
    __shared__ float2 tw[NF];
    __shared__ float red[4];
    const int j = threadIdx.x;
    const int fr = blockIdx.x;                    // b * nf + f
    const int b = fr / nf, f = fr - b * nf;
    const float* xf = x + (size_t)b * T + (size_t)f * HOP;
    float win[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int n = j + 256 * i;
        const float2 t = twg[n];
        tw[n] = t;
        win[i] = 0.5f - 0.5f * t.x;               // periodic Hann: cos(2 pi n / N) = Re tw[n]
        buf[0][n] = make_float2(inv_mu_law(xf[n]) * win[i], 0.f);
    }
    __syncthreads();
    const float2* S = fft1024(buf[0], buf[1], tw, j);   // 5 passes: result in buf[1]
    float2* Z = buf[0];
    float acc = 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int k = j + 256 * i;
        float2 z = make_float2(0.f, 0.f);
        if (k < NBIN) {
            const float2 s = S[k];
            acc += abs_tf(s.x) + abs_tf(s.y);
            z = make_float2(abs_tf_grad(s.x), -abs_tf_grad(s.y));   // conj(gre + i gim)
        }
        Z[k] = z;
    }
    acc = wave_sum_f(acc);
    if ((j & 63) == 0) red[j >> 6] = acc;
    __syncthreads();
    if (j == 0) fpart[fr] = (red[0] + red[1]) + (red[2] + red[3]);
    if (!with_grad) return;
    const float2* G = fft1024(buf[0], buf[1], tw, j);
    float* gf = gfr + (size_t)fr * NF;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int n = j + 256 * i;
        gf[n] = G[n].x * win[i] * inv_nbins;
    }
}

__global__ void __launch_bounds__(256) k_stft_ola(const float* __restrict__ x,
                                                  const float* __restrict__ fpart,
                                                  const float* __restrict__ gfr,
                                                  float* __restrict__ grad,
                                                  float* __restrict__ parts, int T, int nf,
                                                  float gamma, float inv_nbins) {
    const int b = blockIdx.y;
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        float s = 0.f;
        for (int f = 0; f < nf; ++f) s += fpart[(size_t)b * nf + f];
        const float reg = s * inv_nbins;
        parts[b * 4 + 3] = reg;
        parts[b * 4 + 0] += gamma * reg;
    }
    if (gamma == 0.f) return;
    const int t = blockIdx.x * 256 + threadIdx.x;
    if (t >= T) return;
    const int f = t / HOP;
    const float* g = gfr + (size_t)b * nf * NF;
    float ga = 0.f;
    if (f - 1 >= 0 && f - 1 < nf) ga += g[(size_t)(f - 1) * NF + t - (f - 1) * HOP];
    if (f < nf) ga += g[(size_t)f * NF + t - f * HOP];
    const size_t i = (size_t)b * T + t;
    grad[i] += gamma * ga * inv_mu_law_grad(x[i]);
}

__global__ void k_twiddles(float2* tw) {
    const int n = blockIdx.x * blockDim.x + threadIdx.x;
    if (n >= NF) return;
    double s, c;
    sincospi(-2.0 * n / NF, &s, &c);               // exp(-2 pi i n / N)
    tw[n] = make_float2((float)c, (float)s);
}

}  // namespace

int stft_frames(int T) { return T >= NF ? 1 + (T - NF) / HOP : 0; }

void launch_stft_twiddles(float2* tw, hipStream_t s) {
    hipLaunchKernelGGL(k_twiddles, dim3(NF / 256), dim3(256), 0, s, tw);
}

void launch_stft_reg(const float* x, const float2* tw, float* fpart, float* gfr, float* grad,
                     float* parts, float gamma, int B, int T, hipStream_t s) {
    const int nf = stft_frames(T);
    if (nf == 0) return;          // no full frame: reg stays 0 (as the oracle)
    const float inv_nbins = 1.f / ((float)nf * (float)NBIN);
    hipLaunchKernelGGL(k_stft_frames, dim3(B * nf), dim3(256), 0, s, x, tw, fpart, gfr, T, nf,
                       (int)(gamma != 0.f), inv_nbins);
    hipLaunchKernelGGL(k_stft_ola, dim3(gamma != 0.f ? (T + 255) / 256 : 1, B), dim3(256), 0, s,
                       x, fpart, gfr, grad, parts, T, nf, gamma, inv_nbins);
}

}  // namespace ast
