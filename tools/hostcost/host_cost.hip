// Host-side cost of the calls a tracker keyframe commit enqueues: a plain kernel
// launch, hipcub radix sort / exclusive scan dispatches, a small async copy, an event record + stream wait.
// Each figure is the host time per call over many calls (enqueue only; the device is drained between sets).
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <chrono>
#include <cstdio>

__global__ void noop_kernel(int* p) {
    if (threadIdx.x == 0 && blockIdx.x == 0 && p[0] == 12345) p[1] = 1;
}

template <typename F>
static double per_call_us(F f, int reps, hipStream_t s) {
    hipStreamSynchronize(s);
    auto t0 = std::chrono::steady_clock::now();
    for (int i = 0; i < reps; ++i) f();
    auto t1 = std::chrono::steady_clock::now();
    hipStreamSynchronize(s);
    return std::chrono::duration<double, std::micro>(t1 - t0).count() / reps;
}

int main() {
    const int n = 600000;
    hipStream_t s;
    hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    uint32_t *k0, *k1;
    int *v0, *v1, *flag;
    hipMalloc(&k0, n * 4);
    hipMalloc(&k1, n * 4);
    hipMalloc(&v0, n * 4);
    hipMalloc(&v1, n * 4);
    hipMalloc(&flag, 64);
    hipMemset(k0, 0, n * 4);
    hipMemset(v0, 0, n * 4);
    size_t sort_b = 0, scan_b = 0;
    hipcub::DeviceRadixSort::SortPairs(nullptr, sort_b, k0, k1, v0, v1, n, 0, 31, s);
    hipcub::DeviceScan::ExclusiveSum(nullptr, scan_b, k0, k1, n, s);
    void* tmp;
    hipMalloc(&tmp, sort_b > scan_b ? sort_b : scan_b);
    int* h;
    hipHostMalloc((void**)&h, 64, hipHostMallocDefault);
    hipEvent_t ev;
    hipEventCreateWithFlags(&ev, hipEventDisableTiming);
    hipStream_t s2;
    hipStreamCreateWithFlags(&s2, hipStreamNonBlocking);
    for (int round = 0; round < 2; ++round) {
        const double launch = per_call_us([&] { hipLaunchKernelGGL(noop_kernel, dim3(64), dim3(256), 0, s, flag); }, 200, s);
        const double sort = per_call_us([&] {
            size_t b = sort_b;
            hipcub::DeviceRadixSort::SortPairs(tmp, b, k0, k1, v0, v1, n, 0, 31, s);
        }, 20, s);
        const double scan = per_call_us([&] {
            size_t b = scan_b;
            hipcub::DeviceScan::ExclusiveSum(tmp, b, k0, k1, n, s);
        }, 50, s);
        const double d2h = per_call_us([&] { hipMemcpyAsync(h, flag, 8, hipMemcpyDeviceToHost, s); }, 200, s);
        const double d2d = per_call_us([&] { hipMemcpyAsync(k1, k0, 4096, hipMemcpyDeviceToDevice, s); }, 200, s);
        const double evw = per_call_us([&] {
            hipEventRecord(ev, s);
            hipStreamWaitEvent(s2, ev, 0);
        }, 200, s);
        const double sync_idle = per_call_us([&] { hipStreamSynchronize(s); }, 200, s);
        std::printf("round %d host us/call: launch %.2f  hipcub sort(n=%d) %.2f  hipcub scan %.2f  D2H 8B %.2f  D2D 4KB %.2f  "
                    "event record+wait %.2f  sync(idle) %.2f\n",
                    round, launch, n, sort, scan, d2h, d2d, evw, sync_idle);
    }
    return 0;
}
