// Diagnostic: the memory pattern of the split block backward (k_block_bwd_s) without its
// compute.  One 256-thread workgroup per clip walks its 64-position tiles in order (grid = B =
// 256, the bench's walk); per tile each wave loads 9 units (8 image rows x its 32 channels, one
// 128-B line per row; rows p0 - 1 .. p0 + 64 at times tb + (L - 1) d in time_to_batch order) of
// two tensors (tot, D) a tile ahead and stores rows 1..64 of a third (out).  Does the pattern
// alone make the dilation 128 launches slower (per-layer trace: ~+100 us at d = 128)?
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr int C = 128, B = 256, T = 16384, NUU = 9;
constexpr size_t PAD = 263168;
constexpr size_t TS = (size_t)B * T * C + PAD;

struct Tl { int b, tb, m0; };

__global__ void __launch_bounds__(256, 1) kblk(const float* tin, const float* dadd, float* out, int d, int mode) {
    const int n = T / d;
    const int b = blockIdx.x;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int lr = lane >> 3, cq = 32 * w + 4 * (lane & 7);
    const int tiles = T / 64;
    auto tile = [&](int pb) {
        Tl t;
        const int p0 = pb * 64, q = p0 / n;
        t.b = b; t.m0 = p0 - q * n; t.tb = t.m0 * d + q;
        return t;
    };
    auto rowt = [&](const Tl& t, int L) {   // time of image row L (rows without a source: row 1)
        const bool none = L > 65 || (L == 0 && t.m0 == 0) || (L == 65 && t.m0 + 64 >= n);
        return t.tb + ((none ? 1 : L) - 1) * d;
    };
    float4 a[NUU], g[NUU];
    auto load = [&](const Tl& t) {
#pragma unroll
        for (int k = 0; k < NUU; ++k) {
            const size_t o = ((size_t)t.b * T + rowt(t, 8 * k + lr)) * C + cq;
            a[k] = *reinterpret_cast<const float4*>(tin + o);
            g[k] = *reinterpret_cast<const float4*>(dadd + o);
        }
    };
    Tl cur = tile(0);
    load(cur);
    for (int pb = 0; pb < tiles; ++pb) {
        float4 s[NUU];
#pragma unroll
        for (int k = 0; k < NUU; ++k)
            s[k] = make_float4(a[k].x + g[k].x, a[k].y + g[k].y, a[k].z + g[k].z, a[k].w + g[k].w);
        const Tl nx = tile(pb + 1 < tiles ? pb + 1 : pb);
        load(nx);
        if (mode == 0) {
#pragma unroll
            for (int k = 0; k < NUU; ++k) {
                const int L = 8 * k + lr;
                if (L >= 1 && L <= 64)
                    *reinterpret_cast<float4*>(out + ((size_t)cur.b * T + cur.tb + (L - 1) * d) * C + cq) = s[k];
            }
        } else if (s[0].x == 1234.5f) {
            out[threadIdx.x] = s[1].y;
        }
        __syncthreads();
        cur = nx;
    }
}

int main() {
    float* buf;
    if (hipMalloc(&buf, 3 * TS * 4) != hipSuccess) { printf("alloc failed\n"); return 1; }
    (void)hipMemset(buf, 0, 3 * TS * 4);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    const int ds[] = {1, 2, 16, 32, 64, 128, 256};
    for (int rep = 0; rep < 2; ++rep)
        for (int mode = 0; mode < 2; ++mode)
            for (int d : ds) {
                hipLaunchKernelGGL(kblk, dim3(B), dim3(256), 0, 0, buf, buf + TS, buf + 2 * TS, d, mode);
                (void)hipDeviceSynchronize();
                (void)hipEventRecord(e0, 0);
                for (int i = 0; i < 4; ++i)
                    hipLaunchKernelGGL(kblk, dim3(B), dim3(256), 0, 0, buf, buf + TS, buf + 2 * TS, d, mode);
                (void)hipEventRecord(e1, 0);
                (void)hipEventSynchronize(e1);
                float ms;
                (void)hipEventElapsedTime(&ms, e0, e1);
                ms /= 4;
                const double by = (double)B * T * C * 4 * (mode == 0 ? 3.0 : 2.0);
                printf("%s d %3d  %7.3f ms  %6.3f TB/s\n", mode == 0 ? "ld+st" : "ld   ", d, ms, by / (ms * 1e-3) / 1e12);
                fflush(stdout);
            }
    return 0;
}
