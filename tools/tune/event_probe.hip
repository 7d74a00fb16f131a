// What timing a launch costs the stream: back-to-back 1 GiB copy kernels (about the
// headline encode's length) launched plain, with hipEventRecord markers between them
// (bench.py's form), and with the events handed to the dispatch itself
// (hipExtLaunchKernelGGL start/stop), each with default and device-scope events.
// Prints the wall time per kernel and the mean event-timed duration.
//
//   hipcc -O3 --offload-arch=gfx950 -o tools/tune/event_probe tools/tune/event_probe.hip
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x)                                                                  \
    do {                                                                          \
        hipError_t e_ = (x);                                                      \
        if (e_ != hipSuccess) {                                                   \
            std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            std::exit(1);                                                         \
        }                                                                         \
    } while (0)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void copy_kernel(const u32x4* __restrict__ src, u32x4* __restrict__ dst, size_t n)
{
    size_t i = blockIdx.x * size_t(256) + threadIdx.x;
    if (i < n) {
        u32x4 v = __builtin_nontemporal_load(src + i);
        __builtin_nontemporal_store(v, dst + i);
    }
}

int main(int argc, char** argv)
{
    const int reps = argc > 1 ? std::atoi(argv[1]) : 40;
    const size_t bytes = size_t(1) << 30, n = bytes / 16;
    u32x4 *src, *dst;
    CHECK(hipMalloc(&src, bytes));
    CHECK(hipMalloc(&dst, bytes));
    CHECK(hipMemset(src, 1, bytes));
    hipStream_t s;
    CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    const dim3 grid(unsigned(n / 256)), block(256);
    const char* names[] = {"plain", "record default", "record device-scope", "ext-launch default",
                           "ext-launch device-scope", "1 record no-timing", "1 record no-timing dev"};
    for (int round = 0; round < 2; ++round) {
        for (int mode = 0; mode < 7; ++mode) {
            unsigned flags = (mode == 2 || mode == 4 || mode == 6) ? hipEventDisableSystemFence : 0;
            if (mode >= 5) flags |= hipEventDisableTiming;  // a completion marker only (the scratch lease's)
            std::vector<hipEvent_t> ev(2 * reps);
            for (auto& e : ev) CHECK(hipEventCreateWithFlags(&e, flags));
            for (int w = 0; w < 4; ++w) hipLaunchKernelGGL(copy_kernel, grid, block, 0, s, src, dst, n);
            CHECK(hipStreamSynchronize(s));
            auto t0 = std::chrono::steady_clock::now();
            for (int i = 0; i < reps; ++i) {
                if (mode == 0) {
                    hipLaunchKernelGGL(copy_kernel, grid, block, 0, s, src, dst, n);
                } else if (mode >= 5) {
                    hipLaunchKernelGGL(copy_kernel, grid, block, 0, s, src, dst, n);
                    CHECK(hipEventRecord(ev[2 * i], s));
                } else if (mode <= 2) {
                    CHECK(hipEventRecord(ev[2 * i], s));
                    hipLaunchKernelGGL(copy_kernel, grid, block, 0, s, src, dst, n);
                    CHECK(hipEventRecord(ev[2 * i + 1], s));
                } else {
                    hipExtLaunchKernelGGL(copy_kernel, grid, block, 0, s, ev[2 * i], ev[2 * i + 1], 0, src, dst, n);
                }
            }
            CHECK(hipStreamSynchronize(s));
            double wall = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
            double sum = 0;
            if (mode > 0 && mode < 5)
                for (int i = 0; i < reps; ++i) {
                    float ms = 0;
                    CHECK(hipEventElapsedTime(&ms, ev[2 * i], ev[2 * i + 1]));
                    sum += ms * 1e3;
                }
            std::printf("round %d  %-24s wall %8.2f us/kernel  event-timed %8.2f us/kernel\n", round, names[mode],
                        wall / reps, (mode > 0 && mode < 5) ? sum / reps : 0.0);
            for (auto& e : ev) CHECK(hipEventDestroy(e));
        }
    }
    CHECK(hipFree(src));
    CHECK(hipFree(dst));
    return 0;
}
