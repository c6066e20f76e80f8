// ADMM optimal transport between NMF palettes (optimal_transport.py:22-162), batched: one
// 512-thread workgroup per problem runs the whole ADMM loop on the device.
//
// Per problem: C = cost(p_mod, p_ref) / max (Euclidean rows, optimal_transport.py:22-37,82-83),
// then the reference's ADMM (rho = 100, three splitting copies: row sums in [0, 1/n1], column
// sums in [0, 1/n2], total = 1; optimal_transport.py:91-137) until every primal / dual residual
// is below eps * |Sol| or the iteration exceeds miter; then the plan and
// transform_palette(p_mod, p_ref, plan) = plan p_ref / (row sums + 1e-10) (optimal_transport.py:
// 140-148).
//
// Layout: the n1 x n2 matrices (Sol, Old, Aux[3], Lambda[3]) live in registers (C in LDS), element
// e = tid + 512 k (k < 8: n1 n2 <= 4096).  Each iteration stages Aux[0] and Aux[1] in LDS so
// that thread r sums row r and thread n1 + c sums column c (in index order, as numpy's
// per-row loop), and reduces the total and the five squared norms in fp64 across the 8 waves
// (fixed order, so a problem's result does not depend on its batch position).  Three barriers
// per iteration.  fp64 throughout (numpy's float), no contraction into fma, so the updates
// round as the reference's do; only the norms' and sums' summation order differs.
#include "common.h"

#pragma clang fp contract(off)

namespace ast {
namespace {

constexpr int OT_T = 512;
constexpr int OT_E = 8;
constexpr int OT_W = OT_T / 64;
constexpr double RHO = 1e2;

__device__ inline double wave_sum(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    return v;
}

__device__ inline double wave_max(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmax(v, __shfl_xor(v, o));
    return v;
}

__global__ void __launch_bounds__(OT_T) k_ot_admm(const double* __restrict__ p_mod,
                                                  const double* __restrict__ p_ref, int n1, int n2,
                                                  int d, double eps, double miter,
                                                  double* __restrict__ plan,
                                                  double* __restrict__ pal, int* __restrict__ iters) {
    extern __shared__ double lds[];
    const int N = n1 * n2;
    double* A0 = lds;              // [N]  Aux[0] before its projection, later the plan
    double* A1 = A0 + N;           // [N]  Aux[1]
    double* CM = A1 + N;           // [N]  the normalised cost matrix
    double* rc = CM + N;           // [n1] row corrections of Aux[0]
    double* cc = rc + n1;          // [n2] column corrections of Aux[1]
    double* redA = cc + n2;        // [OT_W]
    double* redB = redA + OT_W;    // [OT_W][5]
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const size_t pb = blockIdx.x;
    const double* P1 = p_mod + pb * n1 * d;
    const double* P2 = p_ref + pb * n2 * d;

    double c[OT_E], sol[OT_E], old[OT_E], a[3][OT_E], l[3][OT_E];   // c: staging only
    double cmax = 0.0;
#pragma unroll
    for (int k = 0; k < OT_E; ++k) {
        const int e = tid + OT_T * k;
        double v = 0.0;
        if (e < N) {
            const int i = e / n2, j = e - i * n2;
            for (int f = 0; f < d; ++f) {
                const double df = P1[(size_t)i * d + f] - P2[(size_t)j * d + f];
                v = v + df * df;
            }
            v = sqrt(v);
            cmax = fmax(cmax, v);
        }
        c[k] = v;
        sol[k] = old[k] = 0.0;
#pragma unroll
        for (int s = 0; s < 3; ++s) a[s][k] = l[s][k] = 0.0;
    }
    cmax = wave_max(cmax);
    if (lane == 0) redA[w] = cmax;
    __syncthreads();
    cmax = redA[0];
    for (int i = 1; i < OT_W; ++i) cmax = fmax(cmax, redA[i]);
#pragma unroll
    for (int k = 0; k < OT_E; ++k) {
        const int e = tid + OT_T * k;
        if (e < N) CM[e] = c[k] / cmax;
    }
    __syncthreads();                                           // redA reused below

    const double hi1 = 1.0 / (double)n1, hi2 = 1.0 / (double)n2;
    const double fN = (double)N;
    int it = 0;
    for (;;) {
        // primal update with positivity, the three splitting copies, stage Aux[0], Aux[1]
        double t2 = 0.0;
#pragma unroll
        for (int k = 0; k < OT_E; ++k) {
            const int e = tid + OT_T * k;
            if (e < N) {
                const double sa = (a[0][k] + a[1][k]) + a[2][k];
                const double sl = (l[0][k] + l[1][k]) + l[2][k];
                double s = ((-CM[e] + RHO * sa) + sl) / (3.0 * RHO);
                s = s < 0.0 ? 0.0 : s;
                sol[k] = s;
#pragma unroll
                for (int q = 0; q < 3; ++q) a[q][k] = s - l[q][k] / RHO;
                A0[e] = a[0][k];
                A1[e] = a[1][k];
                t2 += a[2][k];
            }
        }
        t2 = wave_sum(t2);
        if (lane == 0) redA[w] = t2;
        __syncthreads();
        // row sums of Aux[0] (bounds [0, 1/n1], n2 columns); column sums of Aux[1] (its
        // transpose's rows: bounds [0, 1/n2], n1 columns) — optimal_transport.py:50-74,110-112
        for (int r = tid; r < n1 + n2; r += OT_T) {
            double s = 0.0, corr = 0.0;
            if (r < n1) {
                for (int j = 0; j < n2; ++j) s += A0[r * n2 + j];
                if (s < 0.0) corr = (0.0 - s) / (double)n2;
                else if (s > hi1) corr = (hi1 - s) / (double)n2;
                rc[r] = corr;
            } else {
                const int j = r - n1;
                for (int i = 0; i < n1; ++i) s += A1[i * n2 + j];
                if (s < 0.0) corr = (0.0 - s) / (double)n1;
                else if (s > hi2) corr = (hi2 - s) / (double)n1;
                cc[j] = corr;
            }
        }
        double tot = 0.0;
        for (int i = 0; i < OT_W; ++i) tot += redA[i];
        const double corr2 = (1.0 - tot) / fN;                 // optimal_transport.py:40-47
        __syncthreads();
        // projections, dual update, residual norms
        double nr[5] = {0.0, 0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int k = 0; k < OT_E; ++k) {
            const int e = tid + OT_T * k;
            if (e < N) {
                const int i = e / n2, j = e - i * n2;
                a[0][k] = a[0][k] + rc[i];
                a[1][k] = a[1][k] + cc[j];
                a[2][k] = a[2][k] + corr2;
#pragma unroll
                for (int q = 0; q < 3; ++q) l[q][k] += RHO * (a[q][k] - sol[k]);
                const double s = sol[k];
                nr[0] += (s - old[k]) * (s - old[k]);
                nr[1] += (s - a[0][k]) * (s - a[0][k]);
                nr[2] += (s - a[1][k]) * (s - a[1][k]);
                nr[3] += (s - a[2][k]) * (s - a[2][k]);
                nr[4] += s * s;
            }
        }
#pragma unroll
        for (int q = 0; q < 5; ++q) {
            nr[q] = wave_sum(nr[q]);
            if (lane == 0) redB[w * 5 + q] = nr[q];
        }
        __syncthreads();
        double nt[5] = {0.0, 0.0, 0.0, 0.0, 0.0};
        for (int i = 0; i < OT_W; ++i)
#pragma unroll
            for (int q = 0; q < 5; ++q) nt[q] += redB[i * 5 + q];
        // optimal_transport.py:126-135 (every thread reaches the same decision)
        if ((double)it > miter) break;
        const double lim = eps * sqrt(nt[4]);
        if (sqrt(nt[0]) < lim && sqrt(nt[1]) < lim && sqrt(nt[2]) < lim && sqrt(nt[3]) < lim) break;
#pragma unroll
        for (int k = 0; k < OT_E; ++k) old[k] = sol[k];
        ++it;
    }

    // plan out; transform_palette (optimal_transport.py:140-148) from the plan in LDS
    __syncthreads();
#pragma unroll
    for (int k = 0; k < OT_E; ++k) {
        const int e = tid + OT_T * k;
        if (e < N) {
            plan[pb * N + e] = sol[k];
            A0[e] = sol[k];
        }
    }
    if (iters && tid == 0) iters[pb] = it;
    if (!pal) return;
    __syncthreads();
    for (int o = tid; o < n1 * d; o += OT_T) {
        const int i = o / d, f = o - i * d;
        double num = 0.0, den = 0.0;
        for (int j = 0; j < n2; ++j) {
            num += A0[i * n2 + j] * P2[(size_t)j * d + f];
            den += A0[i * n2 + j];
        }
        pal[pb * n1 * d + o] = num / (den + 1e-10);
    }
}

// Problems past the register kernel's n1 n2 <= 4096 cells: the same ADMM with every n1 x n2
// iterate (Sol, Old, Aux[3], Lambda[3]) and the cost matrix in a device workspace of 10 N
// doubles per problem (L2-resident for palettes of a few thousand cells), one 1024-thread
// workgroup per problem, cell e = tid + 1024 k; row / column corrections and the reductions in
// LDS.  The same fp64 operations in the same order per cell; row and column sums in index order.
constexpr int OTB_T = 1024;
constexpr int OTB_W = OTB_T / 64;

__global__ void __launch_bounds__(OTB_T) k_ot_admm_big(const double* __restrict__ p_mod,
                                                       const double* __restrict__ p_ref, int n1,
                                                       int n2, int d, double eps, double miter,
                                                       double* __restrict__ ws,
                                                       double* __restrict__ plan,
                                                       double* __restrict__ pal, int* __restrict__ iters) {
    extern __shared__ double lds[];
    const int N = n1 * n2;
    double* rc = lds;              // [n1]
    double* cc = rc + n1;          // [n2]
    double* redA = cc + n2;        // [OTB_W]
    double* redB = redA + OTB_W;   // [OTB_W][5]
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const size_t pb = blockIdx.x;
    const double* P1 = p_mod + pb * n1 * d;
    const double* P2 = p_ref + pb * n2 * d;
    double* CM = ws + pb * 10 * (size_t)N;
    double* SOL = CM + N;
    double* OLD = SOL + N;
    double* AX[3] = {OLD + N, OLD + 2 * (size_t)N, OLD + 3 * (size_t)N};
    double* LM[3] = {OLD + 4 * (size_t)N, OLD + 5 * (size_t)N, OLD + 6 * (size_t)N};

    double cmax = 0.0;
    for (int e = tid; e < N; e += OTB_T) {
        const int i = e / n2, j = e - i * n2;
        double v = 0.0;
        for (int f = 0; f < d; ++f) {
            const double df = P1[(size_t)i * d + f] - P2[(size_t)j * d + f];
            v = v + df * df;
        }
        v = sqrt(v);
        cmax = fmax(cmax, v);
        CM[e] = v;
        SOL[e] = OLD[e] = 0.0;
        for (int q = 0; q < 3; ++q) AX[q][e] = LM[q][e] = 0.0;
    }
    cmax = wave_max(cmax);
    if (lane == 0) redA[w] = cmax;
    __syncthreads();
    cmax = redA[0];
    for (int i = 1; i < OTB_W; ++i) cmax = fmax(cmax, redA[i]);
    for (int e = tid; e < N; e += OTB_T) CM[e] = CM[e] / cmax;
    __syncthreads();

    const double hi1 = 1.0 / (double)n1, hi2 = 1.0 / (double)n2;
    const double fN = (double)N;
    int it = 0;
    for (;;) {
        double t2 = 0.0;
        for (int e = tid; e < N; e += OTB_T) {
            const double sa = (AX[0][e] + AX[1][e]) + AX[2][e];
            const double sl = (LM[0][e] + LM[1][e]) + LM[2][e];
            double s = ((-CM[e] + RHO * sa) + sl) / (3.0 * RHO);
            s = s < 0.0 ? 0.0 : s;
            SOL[e] = s;
            for (int q = 0; q < 3; ++q) AX[q][e] = s - LM[q][e] / RHO;
            t2 += AX[2][e];
        }
        t2 = wave_sum(t2);
        if (lane == 0) redA[w] = t2;
        __syncthreads();   // the block's global writes are visible to the block after the barrier
        for (int r = tid; r < n1 + n2; r += OTB_T) {
            double s = 0.0, corr = 0.0;
            if (r < n1) {
                for (int j = 0; j < n2; ++j) s += AX[0][r * n2 + j];
                if (s < 0.0) corr = (0.0 - s) / (double)n2;
                else if (s > hi1) corr = (hi1 - s) / (double)n2;
                rc[r] = corr;
            } else {
                const int j = r - n1;
                for (int i = 0; i < n1; ++i) s += AX[1][i * n2 + j];
                if (s < 0.0) corr = (0.0 - s) / (double)n1;
                else if (s > hi2) corr = (hi2 - s) / (double)n1;
                cc[j] = corr;
            }
        }
        double tot = 0.0;
        for (int i = 0; i < OTB_W; ++i) tot += redA[i];
        const double corr2 = (1.0 - tot) / fN;
        __syncthreads();
        double nr[5] = {0.0, 0.0, 0.0, 0.0, 0.0};
        for (int e = tid; e < N; e += OTB_T) {
            const int i = e / n2, j = e - i * n2;
            const double s = SOL[e];
            double ax[3] = {AX[0][e] + rc[i], AX[1][e] + cc[j], AX[2][e] + corr2};
            for (int q = 0; q < 3; ++q) {
                AX[q][e] = ax[q];
                LM[q][e] += RHO * (ax[q] - s);
            }
            const double o = OLD[e];
            nr[0] += (s - o) * (s - o);
            nr[1] += (s - ax[0]) * (s - ax[0]);
            nr[2] += (s - ax[1]) * (s - ax[1]);
            nr[3] += (s - ax[2]) * (s - ax[2]);
            nr[4] += s * s;
        }
#pragma unroll
        for (int q = 0; q < 5; ++q) {
            nr[q] = wave_sum(nr[q]);
            if (lane == 0) redB[w * 5 + q] = nr[q];
        }
        __syncthreads();
        double nt[5] = {0.0, 0.0, 0.0, 0.0, 0.0};
        for (int i = 0; i < OTB_W; ++i)
#pragma unroll
            for (int q = 0; q < 5; ++q) nt[q] += redB[i * 5 + q];
        __syncthreads();   // redA / redB / rc / cc are rewritten next iteration
        if ((double)it > miter) break;
        const double lim = eps * sqrt(nt[4]);
        if (sqrt(nt[0]) < lim && sqrt(nt[1]) < lim && sqrt(nt[2]) < lim && sqrt(nt[3]) < lim) break;
        for (int e = tid; e < N; e += OTB_T) OLD[e] = SOL[e];
        ++it;
    }
    for (int e = tid; e < N; e += OTB_T) plan[pb * N + e] = SOL[e];
    if (iters && tid == 0) iters[pb] = it;
    if (!pal) return;
    __syncthreads();
    for (int o = tid; o < n1 * d; o += OTB_T) {
        const int i = o / d, f = o - i * d;
        double num = 0.0, den = 0.0;
        for (int j = 0; j < n2; ++j) {
            num += SOL[i * n2 + j] * P2[(size_t)j * d + f];
            den += SOL[i * n2 + j];
        }
        pal[pb * n1 * d + o] = num / (den + 1e-10);
    }
}

}  // namespace

size_t ot_big_lds_bytes(int n1, int n2) {
    return sizeof(double) * ((size_t)n1 + n2 + OTB_W + 5 * OTB_W);
}
size_t ot_big_ws_bytes(int n1, int n2) { return sizeof(double) * 10 * (size_t)n1 * n2; }

void launch_ot_admm_big(const double* p_mod, const double* p_ref, int nprob, int n1, int n2, int d,
                        double eps, double miter, double* ws, double* plan, double* pal, int* iters,
                        hipStream_t s) {
    (void)hipFuncSetAttribute((const void*)k_ot_admm_big, hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)ot_big_lds_bytes(n1, n2));
    hipLaunchKernelGGL(k_ot_admm_big, dim3(nprob), dim3(OTB_T), ot_big_lds_bytes(n1, n2), s, p_mod,
                       p_ref, n1, n2, d, eps, miter, ws, plan, pal, iters);
}

size_t ot_lds_bytes(int n1, int n2) {
    return sizeof(double) * (3 * (size_t)n1 * n2 + n1 + n2 + OT_W + 5 * OT_W);
}

int ot_max_cells() { return OT_T * OT_E; }

void launch_ot_admm(const double* p_mod, const double* p_ref, int nprob, int n1, int n2, int d,
                    double eps, double miter, double* plan, double* pal, int* iters, hipStream_t s) {
    (void)hipFuncSetAttribute((const void*)k_ot_admm, hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)ot_lds_bytes(n1, n2));
    hipLaunchKernelGGL(k_ot_admm, dim3(nprob), dim3(OT_T), ot_lds_bytes(n1, n2), s, p_mod, p_ref,
                       n1, n2, d, eps, miter, plan, pal, iters);
}

}  // namespace ast
