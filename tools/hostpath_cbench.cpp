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
//   tools/hostpath_cbench [threads=64] [seconds=3] [L=4404020] [realloc_every=4] [pool=0]
// pool=1: the units come from elect_ec_host_alloc (page-locked pool) instead of malloc.
// Also prints, per thread of the process, the CPU time spent in the timed window
// ("threads": callers summed, every other thread by name and id, largest first),
// read from /proc/self/task: where the library's and the runtime's CPU goes.
#include <dirent.h>
#include <execinfo.h>
#include <signal.h>
#include <malloc.h>
#include <sys/resource.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <algorithm>
#include <map>
#include <mutex>
#include <set>
#include <string>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <thread>
#include <vector>

#include "elect_ec.h"

// CPU seconds of every thread of this process, by thread id (name in *names).
static std::map<long, double> thread_cpu(std::map<long, std::string>* names)
{
    std::map<long, double> out;
    const double hz = static_cast<double>(sysconf(_SC_CLK_TCK));
    DIR* d = opendir("/proc/self/task");
    if (!d) return out;
    while (dirent* e = readdir(d)) {
        if (e->d_name[0] == '.') continue;
        const long tid = std::atol(e->d_name);
        char path[64];
        std::snprintf(path, sizeof path, "/proc/self/task/%ld/stat", tid);
        FILE* f = std::fopen(path, "r");
        if (!f) continue;
        char buf[1024] = {};
        const size_t n = std::fread(buf, 1, sizeof buf - 1, f);
        std::fclose(f);
        buf[n] = 0;
        char* l = std::strchr(buf, '(');
        char* r = std::strrchr(buf, ')');
        if (!l || !r) continue;
        if (names) (*names)[tid] = std::string(l + 1, r);
        unsigned long ut = 0, st = 0;
        // fields after ") ": state(3) ... utime(14) stime(15)
        if (std::sscanf(r + 2, "%*c %*d %*d %*d %*d %*d %*u %*u %*u %*u %*u %lu %lu", &ut, &st) == 2)
            out[tid] = (ut + st) / hz;
    }
    closedir(d);
    return out;
}

// Backtrace of a thread, taken inside it by a signal (the busiest runtime thread's stack).
static void* g_bt[64];
static std::atomic<int> g_bt_n{-1};
static void bt_handler(int)
{
    g_bt_n.store(backtrace(g_bt, 64));
}

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
    const bool pool = argc > 5 && std::atoi(argv[5]) != 0;
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
    std::mutex tid_mu;
    std::set<long> caller_tids;
    auto release = [&](unsigned char* p) {
        if (!p) return;
        if (pool)
            elect_ec_host_free(p);
        else
            std::free(p);
    };
    auto worker = [&](int t) {
        {
            std::lock_guard<std::mutex> g(tid_mu);
            caller_tids.insert(static_cast<long>(syscall(SYS_gettid)));
        }
        std::mt19937_64 rng(t + 1);
        std::vector<unsigned char*> u(6, nullptr);
        auto fresh = [&] {
            for (auto*& p : u) {
                release(p);
                p = nullptr;
                if (pool) {
                    void* q = nullptr;
                    if (elect_ec_host_alloc(L, &q) != 0) std::abort();
                    p = static_cast<unsigned char*>(q);
                } else {
                    p = static_cast<unsigned char*>(std::malloc(L));
                }
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
        for (auto* p : u) release(p);
    };
    std::vector<std::thread> th;
    for (int t = 0; t < T; ++t) th.emplace_back(worker, t);
    // warm: every thread's first call (arenas, dispatchers, device), then the timed window
    go = true;
    std::this_thread::sleep_for(std::chrono::milliseconds(500));
    const long c0 = calls.load();
    std::map<long, std::string> names;
    const std::map<long, double> t0 = thread_cpu(nullptr);
    const double p0 = cpu_seconds();
    const auto w0 = std::chrono::steady_clock::now();
    std::this_thread::sleep_for(std::chrono::duration<double>(secs));
    const long c1 = calls.load();
    const double p1 = cpu_seconds();
    const std::map<long, double> t1 = thread_cpu(&names);
    const double wall = std::chrono::duration<double>(std::chrono::steady_clock::now() - w0).count();
    // what the busiest non-caller threads are doing: 50 samples of wchan ("0" = on a CPU) and the syscall number
    std::map<long, std::map<std::string, int>> samples;
    for (int k = 0; k < 50; ++k) {
        for (const auto& [tid, c] : t1) {
            if (caller_tids.count(tid)) continue;
            char path[96], w[128] = {}, sc[64] = {};
            std::snprintf(path, sizeof path, "/proc/self/task/%ld/wchan", tid);
            if (FILE* f = std::fopen(path, "r")) {
                (void)!std::fgets(w, sizeof w, f);
                std::fclose(f);
            }
            std::snprintf(path, sizeof path, "/proc/self/task/%ld/syscall", tid);
            if (FILE* f = std::fopen(path, "r")) {
                (void)!std::fscanf(f, "%63s", sc);
                std::fclose(f);
            }
            samples[tid][std::string(w[0] ? w : "?") + "|" + (sc[0] ? sc : "?")]++;
        }
        std::this_thread::sleep_for(std::chrono::milliseconds(4));
    }
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
    // per-thread CPU in the window, core-ms per GiB: callers summed, the rest by name
    double callers_s = 0;
    std::vector<std::pair<double, std::string>> others;
    for (const auto& [tid, c] : t1) {
        const auto it = t0.find(tid);
        const double d = c - (it == t0.end() ? 0.0 : it->second);
        if (caller_tids.count(tid))
            callers_s += d;
        else if (d > 0) {
            std::string top;
            for (const auto& [k, v] : samples[tid]) top += k + ":" + std::to_string(v) + " ";
            others.emplace_back(d, names[tid] + "/" + std::to_string(tid) + " [" + top + "]");
        }
    }
    std::sort(others.rbegin(), others.rend());
    // the busiest non-caller thread: 4 backtraces taken inside it
    long hot = 0;
    double hot_d = 0;
    for (const auto& [tid, c] : t1) {
        const auto it = t0.find(tid);
        const double d = c - (it == t0.end() ? 0.0 : it->second);
        if (!caller_tids.count(tid) && d > hot_d) hot = tid, hot_d = d;
    }
    if (hot && std::getenv("CBENCH_BT")) {
        void* warm[4];
        (void)backtrace(warm, 4);  // load libgcc's unwinder outside the handler
        signal(SIGUSR2, bt_handler);
        for (int k = 0; k < 4; ++k) {
            g_bt_n = -1;
            syscall(SYS_tgkill, getpid(), hot, SIGUSR2);
            for (int w = 0; w < 200 && g_bt_n.load() < 0; ++w) std::this_thread::sleep_for(std::chrono::milliseconds(1));
            std::fprintf(stderr, "--- backtrace %d of thread %ld\n", k, hot);
            if (g_bt_n.load() > 0) backtrace_symbols_fd(g_bt, g_bt_n.load(), 2);
            std::this_thread::sleep_for(std::chrono::milliseconds(20));
        }
    }
    std::printf("{\"threads_core_ms_per_GiB\": {\"callers\": %.2f", callers_s * 1e3 / gib);
    for (size_t i = 0; i < others.size() && i < 12; ++i)
        std::printf(", \"%s\": %.2f", others[i].second.c_str(), others[i].first * 1e3 / gib);
    std::printf("}, \"pool\": %d}\n", pool ? 1 : 0);
    std::fflush(stdout);
    std::_Exit(errors.load() == 0 ? 0 : 1);
}
