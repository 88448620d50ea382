// Does stream capture on this ROCm keep (a) hipEventRecord of timing events, (b) a pinned H2D memcpy,
// (c) hipMemsetAsync inside the graph, and what does a 60-kernel chain cost as a graph vs as launches?
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s -> %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

__global__ void add_kernel(double* a, const double* b, int n) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) a[i] += b[i % 7];
}

int main() {
    const int n = 1 << 16, chain = 60;
    double *a, *b, *hb;
    CK(hipMalloc(&a, n * sizeof(double)));
    CK(hipMalloc(&b, 7 * sizeof(double)));
    CK(hipHostMalloc(&hb, 7 * sizeof(double), hipHostMallocDefault));
    for (int i = 0; i < 7; ++i) hb[i] = 1.0;
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    hipEvent_t ev[2];
    for (auto& e : ev) CK(hipEventCreate(&e));
    auto enqueue = [&](bool events) -> hipError_t {
        hipError_t e;
        if ((e = hipMemcpyAsync(b, hb, 7 * sizeof(double), hipMemcpyHostToDevice, s))) return e;
        if ((e = hipMemsetAsync(a, 0, n * sizeof(double), s))) return e;
        if (events && (e = hipEventRecord(ev[0], s))) return e;
        for (int k = 0; k < chain; ++k) hipLaunchKernelGGL(add_kernel, dim3(n / 256), dim3(256), 0, s, a, b, n);
        if (events && (e = hipEventRecord(ev[1], s))) return e;
        return hipGetLastError();
    };
    // plain launches
    CK(enqueue(true));
    CK(hipStreamSynchronize(s));
    auto t0 = std::chrono::steady_clock::now();
    for (int r = 0; r < 20; ++r) CK(enqueue(false));
    auto t1 = std::chrono::steady_clock::now();
    CK(hipStreamSynchronize(s));
    auto t2 = std::chrono::steady_clock::now();
    printf("launches: enqueue %.1f us per chain, total %.1f us per chain\n",
           std::chrono::duration<double, std::micro>(t1 - t0).count() / 20,
           std::chrono::duration<double, std::micro>(t2 - t0).count() / 20);
    // captured
    hipGraph_t g;
    hipGraphExec_t ge;
    CK(hipStreamBeginCapture(s, hipStreamCaptureModeRelaxed));
    hipError_t ce = enqueue(true);
    CK(hipStreamEndCapture(s, &g));
    printf("capture with events: %s\n", hipGetErrorString(ce));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    CK(hipGraphLaunch(ge, s));
    CK(hipStreamSynchronize(s));
    float ms = -1;
    hipError_t te = hipEventElapsedTime(&ms, ev[0], ev[1]);
    double h[2];
    CK(hipMemcpy(h, a, 2 * sizeof(double), hipMemcpyDeviceToHost));
    printf("graph result a[0]=%.1f (expect %d); event time %s %.3f ms\n", h[0], chain, hipGetErrorString(te), ms);
    hb[0] = 2.0;   // the memcpy node must re-read the pinned source at every launch
    CK(hipGraphLaunch(ge, s));
    CK(hipStreamSynchronize(s));
    CK(hipMemcpy(h, a, 2 * sizeof(double), hipMemcpyDeviceToHost));
    printf("relaunch after host change a[0]=%.1f (expect %d)\n", h[0], 2 * chain);
    t0 = std::chrono::steady_clock::now();
    for (int r = 0; r < 20; ++r) CK(hipGraphLaunch(ge, s));
    t1 = std::chrono::steady_clock::now();
    CK(hipStreamSynchronize(s));
    t2 = std::chrono::steady_clock::now();
    printf("graph: enqueue %.1f us per chain, total %.1f us per chain\n",
           std::chrono::duration<double, std::micro>(t1 - t0).count() / 20,
           std::chrono::duration<double, std::micro>(t2 - t0).count() / 20);
    return 0;
}
