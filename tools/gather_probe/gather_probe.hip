// FETCH_SIZE calibration for the access shapes of the registration kernels (is the guide's x2
// correction, stated for wide coalesced streaming reads, right for 16-B gathers?).  Five kernels over a 4 GiB
// buffer (16x the 256 MiB Infinity Cache, so every first touch of a line misses to HBM), each reading a known
// number of bytes; run under rocprofv3 --pmc FETCH_SIZE (and TCC_EA0_RDREQ_sum / TCC_EA0_RDREQ_32B_sum) and
// compare the counters with the byte counts printed here (tools/gather_probe/run.sh).
//   stream   16 B per lane, coalesced: N bytes                           (the guide's calibration)
//   line128  random 128-B lines, 8 lanes read one line's 8 x 16 B        (a walk row: contiguous run)
//   half64   random 64-B halves of distinct lines, 4 lanes per half
//   gather16 one random 16-B point per lane, every line distinct          (the memo pass's neighbour gathers)
//   gather16x2 two 16-B points of the same 128-B line per lane pair, lines distinct
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x)                                                                              \
    do {                                                                                      \
        hipError_t e_ = (x);                                                                  \
        if (e_ != hipSuccess) {                                                               \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                      \
            std::exit(1);                                                                     \
        }                                                                                     \
    } while (0)

__global__ void stream_kernel(const float4* __restrict__ in, size_t n4, float* out) {
    float acc = 0.f;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n4; i += (size_t)gridDim.x * blockDim.x) {
        const float4 v = in[i];
        acc += v.x + v.y + v.z + v.w;
    }
    if (acc == 123.456f) out[0] = acc;   // keeps the loads
}

// lane group of G lanes reads G consecutive float4 of the line lines[t / G] (G = 8: 128 B, 4: the first 64 B)
template <int G>
__global__ void lines_kernel(const float4* __restrict__ in, const unsigned* __restrict__ lines, size_t n, float* out) {
    const size_t t = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    if (t >= n * G) return;
    const size_t line = lines[t / G];
    const float4 v = in[line * 8 + (t % G)];
    const float acc = v.x + v.y + v.z + v.w;
    if (acc == 123.456f) out[0] = acc;
}

// P points per line: lane t reads float4 (t % P) of line lines[t / P] -- P = 1: one 16-B point per line
template <int P>
__global__ void gather_kernel(const float4* __restrict__ in, const unsigned* __restrict__ lines, size_t n, float* out) {
    const size_t t = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    if (t >= n * P) return;
    const size_t line = lines[t / P];
    const float4 v = in[line * 8 + (t % P) * 3];   // points 0 and 3 of the line: both halves when P = 2
    const float acc = v.x + v.y + v.z + v.w;
    if (acc == 123.456f) out[0] = acc;
}

int main() {
    const size_t bytes = (size_t)4 << 30;
    const size_t n4 = bytes / 16, nlines = bytes / 128;
    float4* in;
    float* out;
    unsigned* lines;
    CHECK(hipMalloc(&in, bytes));
    CHECK(hipMemset(in, 0, bytes));
    CHECK(hipMalloc(&out, 4));
    const size_t m = (size_t)1 << 22;   // lines touched per gather kernel (512 MiB of distinct lines)
    std::vector<unsigned> h(m);
    // m distinct random lines: a stride permutation of the line space (odd multiplier mod 2^24)
    // (in the lower half: the streams that flush the Infinity Cache read the upper half)
    for (size_t i = 0; i < m; ++i) h[i] = (unsigned)((i * 2654435761ull + 12345) % (nlines / 2));
    CHECK(hipMalloc(&lines, m * sizeof(unsigned)));
    CHECK(hipMemcpy(lines, h.data(), m * sizeof(unsigned), hipMemcpyHostToDevice));
    const size_t sn = n4 / 4;   // 1 GiB streamed
    // every kernel twice: rocprofv3 reports each dispatch; the second run is the one to read (same counts)
    for (int rep = 0; rep < 2; ++rep) {
        CHECK(hipMemset(in, rep, 4096));
        // a 1 GiB stream before each gather kernel flushes the Infinity Cache (its lines are not re-read)
        hipLaunchKernelGGL(stream_kernel, dim3(8192), dim3(256), 0, 0, in + n4 / 2, sn, out);
        hipLaunchKernelGGL(lines_kernel<8>, dim3((m * 8 + 255) / 256), dim3(256), 0, 0, in, lines, m, out);
        hipLaunchKernelGGL(stream_kernel, dim3(8192), dim3(256), 0, 0, in + n4 / 2, sn, out);
        hipLaunchKernelGGL(lines_kernel<4>, dim3((m * 4 + 255) / 256), dim3(256), 0, 0, in, lines, m, out);
        hipLaunchKernelGGL(stream_kernel, dim3(8192), dim3(256), 0, 0, in + n4 / 2, sn, out);
        hipLaunchKernelGGL(gather_kernel<1>, dim3((m + 255) / 256), dim3(256), 0, 0, in, lines, m, out);
        hipLaunchKernelGGL(stream_kernel, dim3(8192), dim3(256), 0, 0, in + n4 / 2, sn, out);
        hipLaunchKernelGGL(gather_kernel<2>, dim3((m * 2 + 255) / 256), dim3(256), 0, 0, in, lines, m, out);
        CHECK(hipDeviceSynchronize());
    }
    std::printf("{\"stream_bytes\": %zu, \"lines\": %zu, \"line_bytes\": %zu, \"index_bytes\": %zu,\n", sn * 16, m, m * 128,
                m * sizeof(unsigned));
    std::printf(" \"algorithmic\": {\"stream\": %zu, \"line128\": %zu, \"half64\": %zu, \"gather16\": %zu, \"gather16x2\": %zu}}\n",
                sn * 16, m * 128, m * 64, m * 16, m * 32);
    CHECK(hipFree(in));
    CHECK(hipFree(out));
    CHECK(hipFree(lines));
    return 0;
}
