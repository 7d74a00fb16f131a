// The host path as ELECT's JVM drives it, without a Python harness around it:
// T threads, each making synchronous elect_ec_encode calls (the JNI encodeImpl
// convention, EC/NativeRSEncoder.c:43-61) of one RS(6,4) stripe of 4 x L bytes
// from ordinary malloc'd buffers (ECMessageVerbHandler.java:298-314 allocates a
// direct ByteBuffer per unit; glibc serves them from the heap once its dynamic
// mmap threshold has risen, so units sit back to back: M_MMAP_THRESHOLD is
// raised here to the same effect), fresh buffers every `realloc_every` calls.
// Prints one JSON line: data GiB/s, the whole process's CPU time per GiB, the
// library's host_path_stats.  The bench.py --config hostpath figure includes
// its 64 Python caller threads; this one is the library's own cost.
//
//   hipcc -O2 -std=c++17 -I include tools/hostpath_cbench.cpp -L elect_amd -lelect_ec \
//       -Wl,-rpath,'$ORIGIN/../elect_amd' -pthread -o tools/hostpath_cbench
//   tools/hostpath_cbench [threads=64] [seconds=3] [L=4404020] [realloc_every=4]
#include <malloc.h>
#include <sys/resource.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <thread>
#include <vector>

#include "elect_ec.h"

static double cpu_seconds()
{
    rusage u{};
    getrusage(RUSAGE_SELF, &u);
    return u.ru_utime.tv_sec + u.ru_utime.tv_usec * 1e-6 + u.ru_stime.tv_sec + u.ru_stime.tv_usec * 1e-6;
}

int main(int argc, char** argv)
{
    const int T = argc > 1 ? std::atoi(argv[1]) : 64;
    const double secs = argc > 2 ? std::atof(argv[2]) : 3.0;
    const size_t L = argc > 3 ? static_cast<size_t>(std::atoll(argv[3])) : 4404020;
    const int realloc_every = argc > 4 ? std::atoi(argv[4]) : 4;
    mallopt(M_MMAP_THRESHOLD, 256 << 20);
    int ndev = 0;
    if (elect_ec_device_count(&ndev) != 0 || ndev == 0) {
        std::printf("{\"error\": \"no device\"}\n");
        return 2;
    }
    elect_ec_coder* coder = nullptr;
    if (elect_ec_coder_create(4, 2, &coder) != 0) return 2;
    std::atomic<long> calls{0};
    std::atomic<int> errors{0};
    std::atomic<bool> stop{false}, go{false};
    auto worker = [&](int t) {
        std::mt19937_64 rng(t + 1);
        std::vector<unsigned char*> u(6, nullptr);
        auto fresh = [&] {
            for (auto*& p : u) {
                std::free(p);
                p = static_cast<unsigned char*>(std::malloc(L));
                if (!p) std::abort();
            }
            for (int j = 0; j < 4; ++j)
                for (size_t i = 0; i < L; i += 4096) u[j][i] = static_cast<unsigned char>(rng());
        };
        fresh();
        while (!go.load()) std::this_thread::yield();
        long n = 0;
        while (!stop.load(std::memory_order_relaxed)) {
            const unsigned char* in[4] = {u[0], u[1], u[2], u[3]};
            unsigned char* out[2] = {u[4], u[5]};
            if (elect_ec_encode(coder, in, out, L) != 0) errors++;
            ++n;
            calls++;
            if (realloc_every > 0 && n % realloc_every == 0) fresh();  // ELECT: a new ByteBuffer per stripe
        }
        for (auto* p : u) std::free(p);
    };
    std::vector<std::thread> th;
    for (int t = 0; t < T; ++t) th.emplace_back(worker, t);
    // warm: every thread's first call (arenas, dispatchers, device), then the timed window
    go = true;
    std::this_thread::sleep_for(std::chrono::milliseconds(500));
    const long c0 = calls.load();
    const double p0 = cpu_seconds();
    const auto w0 = std::chrono::steady_clock::now();
    std::this_thread::sleep_for(std::chrono::duration<double>(secs));
    const long c1 = calls.load();
    const double p1 = cpu_seconds();
    const double wall = std::chrono::duration<double>(std::chrono::steady_clock::now() - w0).count();
    stop = true;
    for (auto& x : th) x.join();
    uint64_t st[11] = {};
    elect_ec_host_path_stats(st, 11);
    const double gib = static_cast<double>(c1 - c0) * 4.0 * L / 1073741824.0;
    std::printf("{\"metric\": \"GiB/s host-memory RS(6,4) encode, C++ callers (no Python)\", \"value\": %.2f, "
                "\"callers\": %d, \"chunk\": %zu, \"calls\": %ld, \"cpu_core_ms_per_GiB\": %.2f, "
                "\"cpu_bound_ceiling_16_cores_GiB/s\": %.1f, \"errors\": %d, \"realloc_every\": %d, "
                "\"host_path_stats\": {\"zero_copy\": %llu, \"batched\": %llu, \"direct\": %llu, \"registered\": %llu, "
                "\"register_fallback\": %llu, \"unregister_failures\": %llu}}\n",
                gib / wall, T, L, c1 - c0, (p1 - p0) * 1e3 / gib, 16e3 / ((p1 - p0) * 1e3 / gib), errors.load(),
                realloc_every, static_cast<unsigned long long>(st[0]), static_cast<unsigned long long>(st[2]),
                static_cast<unsigned long long>(st[4]), static_cast<unsigned long long>(st[5]),
                static_cast<unsigned long long>(st[6]), static_cast<unsigned long long>(st[7]));
    std::fflush(stdout);
    std::_Exit(errors.load() == 0 ? 0 : 1);
}
