// Device-resident batched L-BFGS-B: the reference's optimiser (scipy.optimize.minimize(
// method='L-BFGS-B', options={'maxiter': 100}) behind tf.contrib.opt.ScipyOptimizerInterface,
// methods.py:132-137,164-181) restated for B independent clips, so the parity-mode loop runs
// without a host round trip per evaluation and can be captured in a hipGraph.
//
// Algorithm = scipy 1.15's L-BFGS-B (v3.0, Byrd-Lu-Nocedal-Zhu / Morales-Nocedal) with no
// bounds, which reduces to:
//   * direction: col == 0 -> generalised Cauchy point z = x - g (B = I); else the quasi-Newton
//     step with H0 = I / theta, theta = y'y / s'y of the newest pair (here the two-loop
//     recursion; L-BFGS-B's compact form is the same matrix), z = x + d; d := z - x (as
//     mainlb forms it, so x + d reproduces z's rounding);
//   * line search lnsrlb: stp = min(1/||d||, 1e10) at iteration 0, else 1; MINPACK-2 dcsrch
//     (More-Thuente, ftol 1e-3, gtol 0.9, xtol 0.1, stpmin 0, stpmax 1e10); trial x = z when
//     stp == 1, else stp*d + x_base; at most maxls (20) evaluations, then restore the base
//     point and restart with an empty memory (abnormal termination if it was already empty);
//   * after an accepted step (NEW_X): iteration count against maxiter first, then
//     ||g||_inf <= pgtol, then (f_old - f) <= factr*eps * max(|f_old|, |f|, 1); then the pair
//     update, skipped when s'y <= eps * (-g_old'd * stp).
// f and g come from ast_loss_grad in fp32 and are widened to fp64, as the ScipyOptimizerInterface
// does; x is kept in fp64 and handed to the loss as fp32 (the TF variable's dtype).
//
// One 1024-thread workgroup per clip.  Every thread runs the scalar state machine redundantly
// on identical inputs (the reductions are broadcast from LDS in a fixed order, so all lanes
// agree bit for bit); vector work is split over the threads.  Thread 0 stores the state.
#include "common.h"

namespace ast {

constexpr int LB_MMAX = 32;

// per-clip scalar state (fp64 as scipy's; 512 B slot)
struct LbState {
    int phase;           // 0 idle / finished, 1 start evaluation pending, 2 line search
    int xi;              // X[xi] is the base point x_k, X[1 - xi] the trial point
    int col, head;       // stored pairs, next ring slot
    int iter, nfev, ifun, reason;
    int stage, brackt, m, maxiter;
    int maxls, pad0, pad1, pad2;
    double theta, fold, gdold, stp, dnorm;
    double finit, ginit, gtest, width, width1, stx, fx, gx, sty, fy, gy, stmin, stmax;
    double tol, pgtol;
    double rho[LB_MMAX];
};
static_assert(sizeof(LbState) <= 512, "LbState slot");

// workspace header (first 512 B): the history size the workspace was laid out with, read by
// every step / state launch, so a workspace can never be indexed with another loop's m
struct LbHeader {
    int magic, m, B, T;
};
constexpr int LB_MAGIC = 0x4c42464d;
constexpr size_t LB_HDR = 512;
// per clip, the loss parts (total, content, style, regularizer) of the first LB_HIST
// evaluations of the current minimize call, in evaluation order (methods.py:147-157 logs every
// evaluation; scipy's maxiter 100 with maxls 20 makes at most 2001)
constexpr int LB_HIST = 4096;

// reasons (ast_lbfgs_state)
enum { LB_RUNNING = 0, LB_STOP_ITER = 1, LB_CONV_PGTOL = 2, LB_CONV_REL_F = 3, LB_ABNORMAL = 4,
       LB_BAD_WORKSPACE = 5 };

namespace {

constexpr int NT = 1024;
constexpr double STPMX = 1e10;
constexpr double EPSMCH = 2.220446049250313e-16;
constexpr double LS_FTOL = 1e-3, LS_GTOL = 0.9, LS_XTOL = 0.1;

struct Ws {   // workspace views for clip b
    LbState* st;
    double* X[2];
    double* R;
    double* D;
    double* S;    // [m][T]
    double* Y;    // [m][T]
    float4* H;    // [LB_HIST] loss parts per evaluation
};

__device__ __forceinline__ Ws ws_view(void* base, int B, int T, int m, int b) {
    Ws w;
    char* p = (char*)base + LB_HDR;
    w.st = (LbState*)p + b;
    double* v = (double*)(p + (size_t)B * 512);
    const size_t per = (size_t)(4 + 2 * m) * T;     // X0 X1 R D S[m] Y[m]
    v += (size_t)b * per;
    w.X[0] = v; w.X[1] = v + T; w.R = v + 2 * (size_t)T; w.D = v + 3 * (size_t)T;
    w.S = v + 4 * (size_t)T; w.Y = v + (4 + (size_t)m) * T;
    w.H = (float4*)((double*)(p + (size_t)B * 512) + (size_t)B * per) + (size_t)b * LB_HIST;
    return w;
}

// deterministic block reductions, result broadcast to every thread
__device__ double block_sum(double v, double* red) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    __syncthreads();                       // red[] free (previous reduction fully read)
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
    __syncthreads();
    double s = 0.0;
#pragma unroll
    for (int k = 0; k < NT / 64; ++k) s += red[k];
    return s;
}

__device__ double block_max(double v, double* red) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmax(v, __shfl_xor(v, o));
    __syncthreads();
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
    __syncthreads();
    double s = 0.0;
#pragma unroll
    for (int k = 0; k < NT / 64; ++k) s = fmax(s, red[k]);
    return s;
}

// no contraction: scipy's x = stp*d + t is a rounded product then a rounded sum
__device__ __forceinline__ double mul_add_rn(double a, double b, double c) {
    return __dadd_rn(__dmul_rn(a, b), c);
}

// MINPACK-2 dcstep (More & Thuente), as called by dcsrch
__device__ void dcstep(double& stx, double& fx, double& dx, double& sty, double& fy, double& dy,
                       double& stp, double fp, double dp, int& brackt, double stpmin,
                       double stpmax) {
    const double sgnd = dp * (dx / fabs(dx));
    double stpf;
    if (fp > fx) {
        const double theta = 3.0 * (fx - fp) / (stp - stx) + dx + dp;
        const double s = fmax(fmax(fabs(theta), fabs(dx)), fabs(dp));
        double gamma = s * sqrt((theta / s) * (theta / s) - (dx / s) * (dp / s));
        if (stp < stx) gamma = -gamma;
        const double p = (gamma - dx) + theta;
        const double q = ((gamma - dx) + gamma) + dp;
        const double r = p / q;
        const double stpc = stx + r * (stp - stx);
        const double stpq = stx + ((dx / ((fx - fp) / (stp - stx) + dx)) / 2.0) * (stp - stx);
        if (fabs(stpc - stx) < fabs(stpq - stx)) stpf = stpc;
        else stpf = stpc + (stpq - stpc) / 2.0;
        brackt = 1;
    } else if (sgnd < 0.0) {
        const double theta = 3.0 * (fx - fp) / (stp - stx) + dx + dp;
        const double s = fmax(fmax(fabs(theta), fabs(dx)), fabs(dp));
        double gamma = s * sqrt((theta / s) * (theta / s) - (dx / s) * (dp / s));
        if (stp > stx) gamma = -gamma;
        const double p = (gamma - dp) + theta;
        const double q = ((gamma - dp) + gamma) + dx;
        const double r = p / q;
        const double stpc = stp + r * (stx - stp);
        const double stpq = stp + (dp / (dp - dx)) * (stx - stp);
        stpf = fabs(stpc - stp) > fabs(stpq - stp) ? stpc : stpq;
        brackt = 1;
    } else if (fabs(dp) < fabs(dx)) {
        const double theta = 3.0 * (fx - fp) / (stp - stx) + dx + dp;
        const double s = fmax(fmax(fabs(theta), fabs(dx)), fabs(dp));
        double gamma = s * sqrt(fmax(0.0, (theta / s) * (theta / s) - (dx / s) * (dp / s)));
        if (stp > stx) gamma = -gamma;
        const double p = (gamma - dp) + theta;
        const double q = (gamma + (dx - dp)) + gamma;
        const double r = p / q;
        double stpc;
        if (r < 0.0 && gamma != 0.0) stpc = stp + r * (stx - stp);
        else if (stp > stx) stpc = stpmax;
        else stpc = stpmin;
        const double stpq = stp + (dp / (dp - dx)) * (stx - stp);
        if (brackt) {
            stpf = fabs(stpc - stp) < fabs(stpq - stp) ? stpc : stpq;
            if (stp > stx) stpf = fmin(stp + 0.66 * (sty - stp), stpf);
            else stpf = fmax(stp + 0.66 * (sty - stp), stpf);
        } else {
            stpf = fabs(stpc - stp) > fabs(stpq - stp) ? stpc : stpq;
            stpf = fmin(stpmax, stpf);
            stpf = fmax(stpmin, stpf);
        }
    } else {
        if (brackt) {
            const double theta = 3.0 * (fp - fy) / (sty - stp) + dy + dp;
            const double s = fmax(fmax(fabs(theta), fabs(dy)), fabs(dp));
            double gamma = s * sqrt((theta / s) * (theta / s) - (dy / s) * (dp / s));
            if (stp > sty) gamma = -gamma;
            const double p = (gamma - dp) + theta;
            const double q = ((gamma - dp) + gamma) + dy;
            const double r = p / q;
            stpf = stp + r * (sty - stp);
        } else if (stp > stx) {
            stpf = stpmax;
        } else {
            stpf = stpmin;
        }
    }
    if (fp > fx) {
        sty = stp; fy = fp; dy = dp;
    } else {
        if (sgnd < 0.0) { sty = stx; fy = fx; dy = dx; }
        stx = stp; fx = fp; dx = dp;
    }
    stp = stpf;
}

// dcsrch START (f, g at stp = 0; stp the first trial)
__device__ void dcsrch_start(LbState& s, double f, double g, double stp) {
    s.brackt = 0;
    s.stage = 1;
    s.finit = f;
    s.ginit = g;
    s.gtest = LS_FTOL * g;
    s.width = STPMX - 0.0;
    s.width1 = s.width / 0.5;
    s.stx = 0.0; s.fx = f; s.gx = g;
    s.sty = 0.0; s.fy = f; s.gy = g;
    s.stmin = 0.0;
    s.stmax = stp + 4.0 * stp;
    s.stp = stp;
}

// dcsrch continuation: returns 1 = FG (new s.stp to evaluate), 0 = CONV / WARN (accept s.stp)
__device__ int dcsrch_iter(LbState& s, double f, double g) {
    const double stpmin = 0.0, stpmax = STPMX;
    double stp = s.stp;
    const double ftest = s.finit + stp * s.gtest;
    if (s.stage == 1 && f <= ftest && g >= 0.0) s.stage = 2;
    if (s.brackt && (stp <= s.stmin || stp >= s.stmax)) return 0;            // WARNING: rounding
    if (s.brackt && s.stmax - s.stmin <= LS_XTOL * s.stmax) return 0;         // WARNING: xtol
    if (stp == stpmax && f <= ftest && g <= s.gtest) return 0;                 // WARNING: stpmax
    if (stp == stpmin && (f > ftest || g >= s.gtest)) return 0;                // WARNING: stpmin
    if (f <= ftest && fabs(g) <= LS_GTOL * (-s.ginit)) return 0;               // CONVERGENCE
    if (s.stage == 1 && f <= s.fx && f > ftest) {
        const double fm = f - stp * s.gtest;
        double fxm = s.fx - s.stx * s.gtest;
        double fym = s.fy - s.sty * s.gtest;
        const double gm = g - s.gtest;
        double gxm = s.gx - s.gtest;
        double gym = s.gy - s.gtest;
        dcstep(s.stx, fxm, gxm, s.sty, fym, gym, stp, fm, gm, s.brackt, s.stmin, s.stmax);
        s.fx = fxm + s.stx * s.gtest;
        s.fy = fym + s.sty * s.gtest;
        s.gx = gxm + s.gtest;
        s.gy = gym + s.gtest;
    } else {
        dcstep(s.stx, s.fx, s.gx, s.sty, s.fy, s.gy, stp, f, g, s.brackt, s.stmin, s.stmax);
    }
    if (s.brackt) {
        if (fabs(s.sty - s.stx) >= 0.66 * s.width1) stp = s.stx + 0.5 * (s.sty - s.stx);
        s.width1 = s.width;
        s.width = fabs(s.sty - s.stx);
    }
    if (s.brackt) {
        s.stmin = fmin(s.stx, s.sty);
        s.stmax = fmax(s.stx, s.sty);
    } else {
        s.stmin = stp + 1.1 * (stp - s.stx);
        s.stmax = stp + 4.0 * (stp - s.stx);
    }
    stp = fmax(stp, stpmin);
    stp = fmin(stp, stpmax);
    if ((s.brackt && (stp <= s.stmin || stp >= s.stmax)) ||
        (s.brackt && s.stmax - s.stmin <= LS_XTOL * s.stmax))
        stp = s.stx;
    s.stp = stp;
    return 1;
}

// fp32 copy of a base/trial point into the buffer ast_loss_grad reads
__device__ __forceinline__ void put_x(float* xd, const double* X, int T) {
    for (int i = threadIdx.x; i < T; i += NT) xd[i] = (float)X[i];
}

// New search direction from base X[xi] with gradient R; starts the line search and writes the
// first trial point.  Returns 0, or 1 if the direction is not a descent direction even with an
// empty memory (abnormal termination).
__device__ int new_direction(LbState& s, const Ws& w, float* xd, int T, double* red, double* alpha) {
    for (int attempt = 0; attempt < 2; ++attempt) {
        const double* t = w.X[s.xi];
        double* trial = w.X[1 - s.xi];
        double* q = w.D;
        // dsub = -g (Cauchy point with B = I) or -H g (two-loop) into D
        for (int i = threadIdx.x; i < T; i += NT) q[i] = w.R[i];
        if (s.col > 0) {
            const int m = s.m;
            for (int k = 0; k < s.col; ++k) {                    // newest -> oldest
                const int j = (s.head - 1 - k + 2 * m) % m;
                const double* Sj = w.S + (size_t)j * T;
                const double* Yj = w.Y + (size_t)j * T;
                double p = 0.0;
                for (int i = threadIdx.x; i < T; i += NT) p += Sj[i] * q[i];
                const double a = s.rho[j] * block_sum(p, red);
                alpha[k] = a;
                for (int i = threadIdx.x; i < T; i += NT) q[i] -= a * Yj[i];
            }
            const double h0 = 1.0 / s.theta;
            for (int i = threadIdx.x; i < T; i += NT) q[i] *= h0;
            for (int k = s.col - 1; k >= 0; --k) {               // oldest -> newest
                const int j = (s.head - 1 - k + 2 * m) % m;
                const double* Sj = w.S + (size_t)j * T;
                const double* Yj = w.Y + (size_t)j * T;
                double p = 0.0;
                for (int i = threadIdx.x; i < T; i += NT) p += Yj[i] * q[i];
                const double beta = s.rho[j] * block_sum(p, red);
                const double c = alpha[k] - beta;
                for (int i = threadIdx.x; i < T; i += NT) q[i] += c * Sj[i];
            }
        }
        // z = x + dsub (dsub = -q), d = z - x; trial z is kept in `trial` for stp == 1
        double dd = 0.0, gd = 0.0;
        for (int i = threadIdx.x; i < T; i += NT) {
            const double z = __dadd_rn(t[i], -q[i]);
            const double d = __dadd_rn(z, -t[i]);
            trial[i] = z;
            q[i] = d;
            dd += d * d;
            gd += w.R[i] * d;
        }
        dd = block_sum(dd, red);
        gd = block_sum(gd, red);
        s.dnorm = sqrt(dd);
        if (gd >= 0.0) {                                         // lnsrlb info = -4
            if (s.col == 0) return 1;
            s.col = 0; s.head = 0; s.theta = 1.0;                // restart from an empty memory
            continue;
        }
        const double stp = s.iter == 0 ? fmin(1.0 / s.dnorm, STPMX) : 1.0;
        s.gdold = gd;
        dcsrch_start(s, s.fold, gd, stp);
        s.ifun = 1;
        if (stp != 1.0)
            for (int i = threadIdx.x; i < T; i += NT) trial[i] = mul_add_rn(stp, q[i], t[i]);
        __syncthreads();
        put_x(xd, trial, T);
        s.phase = 2;
        return 0;
    }
    return 1;
}

struct StepArgs {
    void* ws;
    float* x;
    const float* grad;
    const float* parts;
    int B, T;
};

__device__ __forceinline__ int ws_m(const void* ws) { return ((const LbHeader*)ws)->m; }
// the workspace was started (ast_lbfgs_begin with x0) for this B and T, with a valid m: no
// launch indexes a workspace through a header it did not write
__device__ __forceinline__ bool ws_ok(const void* ws, int B, int T) {
    const LbHeader h = *(const LbHeader*)ws;
    return h.magic == LB_MAGIC && h.m >= 1 && h.m <= LB_MMAX && h.B == B && h.T == T;
}

__global__ void __launch_bounds__(NT) k_lbfgs_step(StepArgs a) {
    __shared__ double red[NT / 64];
    __shared__ double alpha[LB_MMAX];
    const int b = blockIdx.x, T = a.T;
    if (!ws_ok(a.ws, a.B, T)) return;   // never started: nothing to advance (state reports it)
    const Ws w = ws_view(a.ws, a.B, T, ws_m(a.ws), b);
    LbState s = *w.st;
    if (s.phase == 0) return;
    float* xd = a.x + (size_t)b * T;
    const float* g = a.grad + (size_t)b * T;
    const double f = (double)a.parts[b * 4 + 0];
    if (threadIdx.x == 0 && s.nfev < LB_HIST)
        w.H[s.nfev] = make_float4(a.parts[b * 4 + 0], a.parts[b * 4 + 1], a.parts[b * 4 + 2],
                                  a.parts[b * 4 + 3]);
    s.nfev++;
    if (s.phase == 1) {                                          // f, g at the start point
        double gmax = 0.0;
        for (int i = threadIdx.x; i < T; i += NT) {
            const double gi = (double)g[i];
            w.R[i] = gi;
            gmax = fmax(gmax, fabs(gi));
        }
        gmax = block_max(gmax, red);
        s.fold = f;
        s.col = 0; s.head = 0; s.theta = 1.0; s.iter = 0;
        if (gmax <= s.pgtol) { s.phase = 0; s.reason = LB_CONV_PGTOL; }
        else if (new_direction(s, w, xd, T, red, alpha)) { s.phase = 0; s.reason = LB_ABNORMAL; }
    } else {                                                     // line-search evaluation
        double gd = 0.0;
        for (int i = threadIdx.x; i < T; i += NT) gd += (double)g[i] * w.D[i];
        gd = block_sum(gd, red);
        if (dcsrch_iter(s, f, gd)) {                             // FG: another trial
            s.ifun++;
            if (s.ifun - 1 >= s.maxls) {                         // iback >= maxls: give up
                __syncthreads();
                put_x(xd, w.X[s.xi], T);                         // restore the base point
                if (s.col == 0) { s.phase = 0; s.reason = LB_ABNORMAL; s.iter++; }
                else {
                    s.col = 0; s.head = 0; s.theta = 1.0;
                    if (new_direction(s, w, xd, T, red, alpha)) { s.phase = 0; s.reason = LB_ABNORMAL; }
                }
            } else {
                const double* t = w.X[s.xi];
                double* trial = w.X[1 - s.xi];
                for (int i = threadIdx.x; i < T; i += NT) {
                    const double v = mul_add_rn(s.stp, w.D[i], t[i]);
                    trial[i] = v;
                    xd[i] = (float)v;
                }
            }
        } else {                                                 // NEW_X
            s.iter++;
            const double stp = s.stp;
            double gmax = 0.0, rr = 0.0;
            const int slot = s.head;
            double* Sn = w.S + (size_t)slot * T;
            double* Yn = w.Y + (size_t)slot * T;
            for (int i = threadIdx.x; i < T; i += NT) {
                const double gi = (double)g[i];
                const double y = gi - w.R[i];
                gmax = fmax(gmax, fabs(gi));
                rr += y * y;
            }
            gmax = block_max(gmax, red);
            rr = block_sum(rr, red);
            const double fold = s.fold;
            s.xi ^= 1;                                           // the trial is the new base
            if (s.iter >= s.maxiter) { s.phase = 0; s.reason = LB_STOP_ITER; }
            else if (gmax <= s.pgtol) { s.phase = 0; s.reason = LB_CONV_PGTOL; }
            else if (fold - f <= s.tol * fmax(fmax(fabs(fold), fabs(f)), 1.0)) {
                s.phase = 0; s.reason = LB_CONV_REL_F;
            } else {
                double dr, ddum;
                if (stp == 1.0) { dr = gd - s.gdold; ddum = -s.gdold; }
                else { dr = (gd - s.gdold) * stp; ddum = -s.gdold * stp; }
                const bool upd = dr > EPSMCH * ddum;
                for (int i = threadIdx.x; i < T; i += NT) {
                    const double gi = (double)g[i];
                    if (upd) {
                        Sn[i] = stp == 1.0 ? w.D[i] : stp * w.D[i];
                        Yn[i] = gi - w.R[i];
                    }
                    w.R[i] = gi;
                }
                if (upd) {
                    s.rho[slot] = 1.0 / dr;
                    s.theta = rr / dr;
                    s.head = (s.head + 1) % s.m;
                    if (s.col < s.m) s.col++;
                }
                s.fold = f;
                __syncthreads();
                if (new_direction(s, w, xd, T, red, alpha)) { s.phase = 0; s.reason = LB_ABNORMAL; }
            }
        }
    }
    if (threadIdx.x == 0) *w.st = s;
}

__global__ void __launch_bounds__(NT) k_lbfgs_begin(void* ws, float* x, const double* x0,
                                                    const int* active, int B, int T, int m,
                                                    int maxiter, int maxls, double tol,
                                                    double pgtol) {
    const int b = blockIdx.x;
    if (!x0 && !ws_ok(ws, B, T)) return;   // a continuation needs a started workspace
    if (!x0) m = ws_m(ws);   // a continuation keeps the workspace's own history size
    const Ws w = ws_view(ws, B, T, m, b);
    LbState s = *w.st;
    if (x0 && b == 0 && threadIdx.x == 0) *(LbHeader*)ws = LbHeader{LB_MAGIC, m, B, T};
    if (x0) {
        for (int k = 0; k < (int)(sizeof(LbState) / 4); ++k) ((int*)&s)[k] = 0;
        const double* src = x0 + (size_t)b * T;
        for (int i = threadIdx.x; i < T; i += NT) w.X[0][i] = src[i];
    }
    if (!x0 && (!active || active[b])) {   // a new epoch starts from the float32 rounding of
                                            // the point (the TF variable); idle clips keep theirs
        double* X = w.X[s.xi];
        for (int i = threadIdx.x; i < T; i += NT) X[i] = (double)(float)X[i];
    }
    s.m = m; s.maxiter = maxiter; s.maxls = maxls; s.tol = tol; s.pgtol = pgtol;
    s.col = 0; s.head = 0; s.theta = 1.0; s.iter = 0; s.nfev = 0; s.ifun = 0;
    s.reason = LB_RUNNING;
    s.phase = (!active || active[b]) ? 1 : 0;
    __syncthreads();
    put_x(x + (size_t)b * T, w.X[s.xi], T);
    if (threadIdx.x == 0) *w.st = s;
}

__global__ void k_lbfgs_state(const void* ws, int* info, double* x64, int B, int T) {
    const int b = blockIdx.x;
    if (!ws_ok(ws, B, T)) {            // not a started workspace of this B, T: say so
        if (threadIdx.x == 0) {
            info[b * 4 + 0] = 0; info[b * 4 + 1] = 0; info[b * 4 + 2] = 0;
            info[b * 4 + 3] = LB_BAD_WORKSPACE;
        }
        return;
    }
    const Ws w = ws_view(const_cast<void*>(ws), B, T, ws_m(ws), b);
    const LbState& s = *w.st;
    if (threadIdx.x == 0) {
        info[b * 4 + 0] = s.phase;
        info[b * 4 + 1] = s.iter;
        info[b * 4 + 2] = s.nfev;
        info[b * 4 + 3] = s.reason;
    }
    if (x64) {
        const double* X = w.X[s.xi];
        for (int i = threadIdx.x; i < T; i += blockDim.x) x64[(size_t)b * T + i] = X[i];
    }
}

// out [B][cap][4]: the parts of evaluations 0 .. min(nfev, cap) - 1 of each clip's current (or
// last) minimize call, NaN past its count
__global__ void k_lbfgs_history(const void* ws, float4* out, int cap, int B, int T) {
    const int b = blockIdx.x;
    const bool ok = ws_ok(ws, B, T);
    const Ws w = ws_view(const_cast<void*>(ws), B, T, ok ? ws_m(ws) : 1, b);
    const int n = ok ? min(w.st->nfev, LB_HIST) : 0;
    const float q = __builtin_nanf("");
    for (int i = threadIdx.x; i < cap; i += blockDim.x)
        out[(size_t)b * cap + i] = i < n ? w.H[i] : make_float4(q, q, q, q);
}

}  // namespace

size_t lbfgs_workspace_bytes(int B, int T, int m) {
    return LB_HDR + (size_t)B * 512 + (size_t)B * (4 + 2 * (size_t)m) * T * 8 +
           (size_t)B * LB_HIST * sizeof(float4);
}

int lbfgs_history_cap() { return LB_HIST; }

void launch_lbfgs_history(const void* ws, float* out, int cap, int B, int T, hipStream_t s) {
    hipLaunchKernelGGL(k_lbfgs_history, dim3(B), dim3(256), 0, s, ws, (float4*)out, cap, B, T);
}

void launch_lbfgs_begin(void* ws, float* x, const double* x0, const int* active, int B, int T,
                        int m, int maxiter, int maxls, double tol, double pgtol, hipStream_t s) {
    hipLaunchKernelGGL(k_lbfgs_begin, dim3(B), dim3(NT), 0, s, ws, x, x0, active, B, T, m,
                       maxiter, maxls, tol, pgtol);
}

void launch_lbfgs_step(void* ws, float* x, const float* grad, const float* parts, int B, int T,
                       hipStream_t s) {
    StepArgs a{ws, x, grad, parts, B, T};
    hipLaunchKernelGGL(k_lbfgs_step, dim3(B), dim3(NT), 0, s, a);
}

void launch_lbfgs_state(const void* ws, int* info, double* x64, int B, int T, hipStream_t s) {
    hipLaunchKernelGGL(k_lbfgs_state, dim3(B), dim3(256), 0, s, ws, info, x64, B, T);
}

}  // namespace ast
