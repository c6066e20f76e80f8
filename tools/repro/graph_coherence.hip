// Minimal reproducer: data written by one kernel node of a HIP graph and read by the next node
// from a workgroup on another XCD.  Graph: bump(iter) -> produce(buf) -> consume(buf -> out);
// produce's workgroup g writes row g = iter * 1000 + g, consume's workgroup g copies row g + 1
// (written by a workgroup on another XCD: blockIdx round-robins over the 8 XCDs).  Checks out
// after every launch, eager and as graph replays.
//   hipcc --offload-arch=gfx950 -O2 -o graph_coherence graph_coherence.hip && ./graph_coherence
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); return 2; } } while (0)

constexpr int NB = 256, NT = 64;

__global__ void bump(int* iter) { if (threadIdx.x == 0 && blockIdx.x == 0) iter[0] += 1; }
__global__ void produce(float* buf, const int* iter) {
    buf[blockIdx.x * NT + threadIdx.x] = (float)(iter[0] * 1000 + (int)blockIdx.x);
}
__global__ void kmax(unsigned* gmax, const int* iter) {   // per-clip max, clip = blockIdx % 8
    if (threadIdx.x == 0) atomicMax(gmax + blockIdx.x % 8, (unsigned)(1000000 - iter[0] * 1000 + (int)blockIdx.x % 8));   // decreasing: a missed clear keeps an old max
}
__global__ void kuse(const unsigned* gmax, float* out) {
    out[blockIdx.x * NT + threadIdx.x] = (float)gmax[(blockIdx.x + 3) % 8];
}
__global__ void consume(const float* buf, float* out) {
    const int src = (blockIdx.x + 1) % NB;
    out[blockIdx.x * NT + threadIdx.x] = buf[src * NT + threadIdx.x];
}

static int check(const float* dout, int iter, const char* tag, int k) {
    std::vector<float> h(NB * NT);
    if (hipMemcpy(h.data(), dout, h.size() * 4, hipMemcpyDeviceToHost) != hipSuccess) return -1;
    int bad = 0, first = -1;
    for (int g = 0; g < NB; ++g)
        for (int t = 0; t < NT; ++t)
            if (h[g * NT + t] != (float)(iter * 1000 + (g + 1) % NB)) { if (first < 0) first = g; ++bad; }
    printf("%s %d: iter %d, %d stale values (first row %d: %g)\n", tag, k, iter, bad, first,
           first >= 0 ? h[first * NT] : 0.0);
    return bad;
}

int main() {
    float *buf, *out;
    int* iter;
    CK(hipMalloc(&buf, NB * NT * 4));
    CK(hipMalloc(&out, NB * NT * 4));
    CK(hipMalloc(&iter, 4));
    CK(hipMemset(iter, 0, 4));
    hipStream_t s;
    CK(hipStreamCreate(&s));
    int it = 0, bad_eager = 0, bad_graph = 0;
    for (int k = 0; k < 4; ++k) {
        hipLaunchKernelGGL(bump, dim3(1), dim3(64), 0, s, iter);
        hipLaunchKernelGGL(produce, dim3(NB), dim3(NT), 0, s, buf, iter);
        hipLaunchKernelGGL(consume, dim3(NB), dim3(NT), 0, s, buf, out);
        CK(hipStreamSynchronize(s));
        bad_eager += check(out, ++it, "eager", k) != 0;
    }
    hipGraph_t g;
    hipGraphExec_t ge;
    CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
    hipLaunchKernelGGL(bump, dim3(1), dim3(64), 0, s, iter);
    hipLaunchKernelGGL(produce, dim3(NB), dim3(NT), 0, s, buf, iter);
    hipLaunchKernelGGL(consume, dim3(NB), dim3(NT), 0, s, buf, out);
    CK(hipStreamEndCapture(s, &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    for (int k = 0; k < 6; ++k) {
        CK(hipGraphLaunch(ge, s));
        CK(hipStreamSynchronize(s));
        bad_graph += check(out, ++it, "graph replay", k) != 0;
    }
    printf("RESULT eager launches with stale data: %d / 4, graph replays with stale data: %d / 6\n",
           bad_eager, bad_graph);
    // second pattern: hipMemsetAsync clear -> atomicMax per clip -> readers of another clip's max
    unsigned* gmax;
    CK(hipMalloc(&gmax, 32));
    auto check2 = [&](int itv, const char* tag, int k) {
        std::vector<float> h(NB * NT);
        if (hipMemcpy(h.data(), out, h.size() * 4, hipMemcpyDeviceToHost) != hipSuccess) return -1;
        int bad = 0, first = -1;
        for (int gi = 0; gi < NB; ++gi)
            if (h[gi * NT] != (float)(1000000 - itv * 1000 + (gi + 3) % 8)) { if (first < 0) first = gi; ++bad; }
        printf("%s %d: iter %d, %d stale rows (first row %d: %g)\n", tag, k, itv, bad, first, first >= 0 ? h[first * NT] : 0.0);
        return bad;
    };
    int b2e = 0, b2g = 0;
    for (int k = 0; k < 3; ++k) {
        hipLaunchKernelGGL(bump, dim3(1), dim3(64), 0, s, iter);
        CK(hipMemsetAsync(gmax, 0, 32, s));
        hipLaunchKernelGGL(kmax, dim3(NB), dim3(64), 0, s, gmax, iter);
        hipLaunchKernelGGL(kuse, dim3(NB), dim3(NT), 0, s, gmax, out);
        CK(hipStreamSynchronize(s));
        b2e += check2(++it, "memset+max eager", k) != 0;
    }
    hipGraph_t g2;
    hipGraphExec_t ge2;
    CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
    hipLaunchKernelGGL(bump, dim3(1), dim3(64), 0, s, iter);
    CK(hipMemsetAsync(gmax, 0, 32, s));
    hipLaunchKernelGGL(kmax, dim3(NB), dim3(64), 0, s, gmax, iter);
    hipLaunchKernelGGL(kuse, dim3(NB), dim3(NT), 0, s, gmax, out);
    CK(hipStreamEndCapture(s, &g2));
    CK(hipGraphInstantiate(&ge2, g2, nullptr, nullptr, 0));
    float* junk;
    CK(hipMalloc(&junk, NB * NT * 4));
    for (int k = 0; k < 6; ++k) {
        CK(hipGraphLaunch(ge2, s));
        CK(hipStreamSynchronize(s));
        b2g += check2(++it, "memset+max graph replay", k) != 0;
        if (k >= 2) {   // eager work between replays: a memset of another buffer and a kernel
            CK(hipMemsetAsync(junk, 0x7f, 4096, s));
            hipLaunchKernelGGL(consume, dim3(NB), dim3(NT), 0, s, buf, junk);
            CK(hipStreamSynchronize(s));
        }
    }
    printf("RESULT memset+atomicMax: eager launches wrong: %d / 3, graph replays wrong: %d / 6\n", b2e, b2g);
    CK(hipGraphExecDestroy(ge2));
    CK(hipGraphDestroy(g2));
    CK(hipGraphExecDestroy(ge));
    CK(hipGraphDestroy(g));
    CK(hipStreamDestroy(s));
    return 0;
}
