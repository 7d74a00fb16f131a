// What page-locking a caller's buffers per call would cost: T threads, each
// registering and unregistering its own six 4,404,020-byte buffers (one RS(6,4)
// encode call of ELECT's: 4 data + 2 parity units, ordinary malloc'd memory) in a
// loop.  Prints calls per second, data GiB/s (4 units of data per call) and CPU
// time per GiB of data, next to a plain streaming copy of the same 1.5 units per
// data unit (what the staged batcher's copies cost).
//
//   g++ -O2 -std=c++17 -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include tools/tune/register_probe.cpp \
//       -L/opt/rocm/lib -lamdhip64 -lpthread -o tools/tune/register_probe
#include <hip/hip_runtime.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <ctime>
#include <thread>
#include <vector>

static double cpu_seconds()
{
    timespec t{};
    clock_gettime(CLOCK_PROCESS_CPUTIME_ID, &t);
    return t.tv_sec + t.tv_nsec * 1e-9;
}

int main(int argc, char** argv)
{
    const double secs = argc > 1 ? std::atof(argv[1]) : 2.0;
    const size_t L = 4404020;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) {
        std::printf("no device\n");
        return 1;
    }
    (void)hipSetDevice(0);
    (void)hipFree(nullptr);
    for (int mode = 0; mode < 2; ++mode) {
        for (int T : {1, 16, 64}) {
            std::atomic<long> calls{0};
            std::atomic<bool> stop{false};
            std::atomic<int> errors{0};
            std::vector<std::thread> th;
            const double c0 = cpu_seconds();
            const auto t0 = std::chrono::steady_clock::now();
            for (int t = 0; t < T; ++t)
                th.emplace_back([&, mode] {
                    (void)hipSetDevice(0);
                    std::vector<unsigned char*> b(6);
                    for (auto& p : b) {
                        p = static_cast<unsigned char*>(std::malloc(L));
                        std::memset(p, 1, L);
                    }
                    std::vector<unsigned char> stage(L * 6);
                    while (!stop.load(std::memory_order_relaxed)) {
                        if (mode == 0) {
                            for (auto* p : b)
                                if (hipHostRegister(p, L, hipHostRegisterDefault) != hipSuccess) errors++;
                            for (auto* p : b) (void)hipHostUnregister(p);
                        } else {  // the staged path's copies: 4 units in, 2 out
                            for (int j = 0; j < 4; ++j) std::memcpy(stage.data() + j * L, b[j], L);
                            for (int j = 4; j < 6; ++j) std::memcpy(b[j], stage.data() + j * L, L);
                        }
                        calls++;
                    }
                    for (auto* p : b) std::free(p);
                });
            std::this_thread::sleep_for(std::chrono::duration<double>(secs));
            stop = true;
            for (auto& x : th) x.join();
            const double wall = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
            const double cpu = cpu_seconds() - c0;
            const double gib = calls.load() * 4.0 * L / (1u << 30);
            std::printf("%-9s T=%-3d calls/s %8.1f  data GiB/s %7.2f  core-ms/GiB %7.1f  errors %d\n",
                        mode == 0 ? "register" : "memcpy", T, calls.load() / wall, gib / wall, cpu * 1e3 / gib,
                        errors.load());
        }
    }
    return 0;
}
