// Which HIP / HSA runtime thread burns a core while the host path runs, and
// what wakes it (round 5: a runtime thread "running" in 50 of 50 samples, 19-20
// core-ms per GiB at 64 callers, tools/hostpath_cbench).  One mode per run,
// 2 s each, per-thread CPU from /proc/self/task over the window:
//   idle      hipInit + a stream, nothing queued
//   kernels   an empty kernel every 0.5 ms, hipStreamSynchronize after each
//   hostfunc  an empty kernel + hipLaunchHostFunc every 0.5 ms (the batcher's completions)
//   hostfunc_burst 150 bursts per s of 3 kernels + 2 host functions (the batcher's rate)
//   event     an empty kernel + hipEventRecord + hipEventSynchronize (default event)
//   blocking  the same with a hipEventBlockingSync event
//   hsa_lock  hsa_amd_memory_lock / unlock of 4 MiB every 0.5 ms (no kernels)
//   longk_hostfunc  3 streams, each 150 times per s: a 5 ms kernel, a host function, a 1 ms kernel, a host function
//   longk_sync      the same with hipStreamSynchronize from 3 threads instead of host functions
//   longk_blocking  ... hipEventRecord + hipEventSynchronize on a hipEventBlockingSync event, 3 threads
//   longk_poll      ... hipEventRecord, then hipEventQuery every 50 us (sleeping between), 3 threads
// Round 6, cross-stream chains (the host path's gather -> code -> scatter streams), 150 per s of
// a 5 ms kernel on stream 0, then a 1 ms kernel on stream 1, then a 1 ms kernel on stream 2, each
// after the previous, the host polling the last with hipEventQuery every 50 us:
//   chain_same       all three on stream 0 (no cross-stream dependency: round 5's pattern)
//   chain_event      hipEventRecord + hipStreamWaitEvent between streams (hipEventDisableTiming)
//   chain_event_nf   ... events also hipEventDisableSystemFence
//   chain_event_dev  ... events also hipEventReleaseToDevice
//   chain_value      hipStreamWriteValue32 of a device flag behind each kernel, hipStreamWaitValue32 on the next stream
//
//   hipcc --offload-arch=gfx950 -O2 -std=c++17 tools/tune/spin_probe.cpp -L/opt/rocm/lib -lhsa-runtime64 -pthread -o tools/tune/spin_probe
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>

#include <dirent.h>
#include <execinfo.h>
#include <signal.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <string>
#include <thread>
#include <vector>

__global__ void empty_kernel(int* p)
{
    if (p && threadIdx.x == 1023) p[0] = 1;
}

// Busy for `ticks` of the 100 MHz wall clock (bounded: every wave leaves).
__global__ void wait_kernel(uint64_t ticks)
{
    const uint64_t t0 = wall_clock64();
    while (wall_clock64() - t0 < ticks) __builtin_amdgcn_s_sleep(64);
}

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
        if (std::sscanf(r + 2, "%*c %*d %*d %*d %*d %*d %*u %*u %*u %*u %*u %lu %lu", &ut, &st) == 2)
            out[tid] = (ut + st) / hz;
    }
    closedir(d);
    return out;
}

static void noop(void*) {}

static void on_segv(int sig)
{
    void* bt[64];
    const int n = backtrace(bt, 64);
    std::fprintf(stderr, "signal %d, backtrace:\n", sig);
    backtrace_symbols_fd(bt, n, 2);
    std::_Exit(128 + sig);
}

int main(int argc, char** argv)
{
    signal(SIGSEGV, on_segv);
    const std::string mode = argc > 1 ? argv[1] : "idle";
    std::fprintf(stderr, "mode %s\n", mode.c_str());
    const double secs = 2.0;
    hipStream_t s;
    if (hipStreamCreate(&s) != hipSuccess) return 2;
    hipEvent_t ev_default, ev_blocking;
    (void)hipEventCreateWithFlags(&ev_default, hipEventDisableTiming);
    (void)hipEventCreateWithFlags(&ev_blocking, hipEventDisableTiming | hipEventBlockingSync);
    std::vector<char> host(4 << 20, 1);
    hsa_agent_t gpu{};
    hsa_iterate_agents(
        [](hsa_agent_t a, void* arg) -> hsa_status_t {
            hsa_device_type_t t{};
            if (hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t) == HSA_STATUS_SUCCESS && t == HSA_DEVICE_TYPE_GPU) {
                *static_cast<hsa_agent_t*>(arg) = a;
                return HSA_STATUS_INFO_BREAK;
            }
            return HSA_STATUS_SUCCESS;
        },
        &gpu);
    // warm
    hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, s, nullptr);
    (void)hipLaunchHostFunc(s, noop, nullptr);
    (void)hipStreamSynchronize(s);
    std::this_thread::sleep_for(std::chrono::milliseconds(200));

    hipStream_t st[3];
    for (auto& x : st) (void)hipStreamCreate(&x);
    std::atomic<bool> stop{false};
    std::vector<std::thread> syncers;
    if (mode == "longk_sync" || mode == "longk_blocking" || mode == "longk_poll")
        for (int q = 0; q < 3; ++q)
            syncers.emplace_back([&, q] {
                hipEvent_t ev;
                (void)hipEventCreateWithFlags(&ev, hipEventDisableTiming | (mode == "longk_blocking" ? hipEventBlockingSync : 0));
                while (!stop.load()) {
                    hipLaunchKernelGGL(wait_kernel, dim3(1), dim3(64), 0, st[q], uint64_t{500000});
                    hipLaunchKernelGGL(wait_kernel, dim3(1), dim3(64), 0, st[q], uint64_t{100000});
                    if (mode == "longk_sync") {
                        (void)hipStreamSynchronize(st[q]);
                    } else {
                        (void)hipEventRecord(ev, st[q]);
                        if (mode == "longk_blocking")
                            (void)hipEventSynchronize(ev);
                        else
                            while (hipEventQuery(ev) == hipErrorNotReady) std::this_thread::sleep_for(std::chrono::microseconds(50));
                    }
                    std::this_thread::sleep_for(std::chrono::microseconds(300));
                }
                (void)hipEventDestroy(ev);
            });
    std::map<long, std::string> names;
    const auto t0 = thread_cpu(nullptr);
    const auto w0 = std::chrono::steady_clock::now();
    long iters = 0;
    auto elapsed = [&] { return std::chrono::duration<double>(std::chrono::steady_clock::now() - w0).count(); };
    while (elapsed() < secs) {
        if (mode == "kernels") {
            hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, s, nullptr);
            (void)hipStreamSynchronize(s);
        } else if (mode == "hostfunc") {
            hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, s, nullptr);
            (void)hipLaunchHostFunc(s, noop, nullptr);
        } else if (mode == "hostfunc_burst") {
            for (int k = 0; k < 3; ++k) {
                hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, s, nullptr);
                if (k < 2) (void)hipLaunchHostFunc(s, noop, nullptr);
            }
        } else if (mode == "event" || mode == "blocking") {
            hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, s, nullptr);
            hipEvent_t ev = mode == "event" ? ev_default : ev_blocking;
            (void)hipEventRecord(ev, s);
            (void)hipEventSynchronize(ev);
        } else if (mode == "longk_hostfunc") {
            for (int q = 0; q < 3; ++q) {
                hipLaunchKernelGGL(wait_kernel, dim3(1), dim3(64), 0, st[q], uint64_t{500000});
                (void)hipLaunchHostFunc(st[q], noop, nullptr);
                hipLaunchKernelGGL(wait_kernel, dim3(1), dim3(64), 0, st[q], uint64_t{100000});
                (void)hipLaunchHostFunc(st[q], noop, nullptr);
            }
        } else if (mode.rfind("chain_", 0) == 0) {
            static hipEvent_t ev[3];
            static uint32_t* flag = nullptr;
            static uint32_t seq = 0;
            if (!ev[0]) {
                const unsigned f = hipEventDisableTiming | (mode == "chain_event_nf" ? hipEventDisableSystemFence : 0u) |
                                   (mode == "chain_event_dev" ? hipEventReleaseToDevice : 0u);
                for (auto& e : ev) (void)hipEventCreateWithFlags(&e, f);
                (void)hipMalloc(reinterpret_cast<void**>(&flag), 2 * sizeof(uint32_t));
                (void)hipMemset(flag, 0, 2 * sizeof(uint32_t));
            }
            const bool same = mode == "chain_same", value = mode == "chain_value";
            ++seq;
            const uint64_t ticks[3] = {500000, 100000, 100000};
            for (int q = 0; q < 3; ++q) {
                hipStream_t x = same ? st[0] : st[q];
                if (q > 0 && !same) {
                    if (value)
                        (void)hipStreamWaitValue32(x, flag + q - 1, seq, hipStreamWaitValueGte, 0xFFFFFFFFu);
                    else
                        (void)hipStreamWaitEvent(x, ev[q - 1], 0);
                }
                hipLaunchKernelGGL(wait_kernel, dim3(1), dim3(64), 0, x, ticks[q]);
                if (value && q < 2) (void)hipStreamWriteValue32(x, flag + q, seq, 0);
                (void)hipEventRecord(ev[q], x);
            }
            while (hipEventQuery(ev[2]) == hipErrorNotReady) std::this_thread::sleep_for(std::chrono::microseconds(50));
        } else if (mode == "hsa_lock") {
            void* ap = nullptr;
            if (hsa_amd_memory_lock(host.data() + 4096 - (reinterpret_cast<uintptr_t>(host.data()) & 4095), 2 << 20, &gpu,
                                    1, &ap) == HSA_STATUS_SUCCESS)
                (void)hsa_amd_memory_unlock(host.data() + 4096 - (reinterpret_cast<uintptr_t>(host.data()) & 4095));
        }
        ++iters;
        std::this_thread::sleep_for(std::chrono::microseconds(mode == "hostfunc_burst"   ? 6667
                                                              : mode == "longk_hostfunc" ? 6000
                                                              : mode.rfind("chain_", 0) == 0 ? 100
                                                              : 500));
    }
    const auto t1 = thread_cpu(&names);
    const double wall = elapsed();
    stop = true;
    for (auto& t : syncers) t.join();
    for (auto& x : st) (void)hipStreamSynchronize(x);
    const long self = static_cast<long>(getpid());
    std::printf("{\"mode\": \"%s\", \"iters\": %ld, \"wall_s\": %.3f, \"threads_cpu_frac\": {", mode.c_str(), iters, wall);
    bool first = true;
    for (const auto& [tid, c] : t1) {
        const auto it = t0.find(tid);
        const double d = c - (it == t0.end() ? 0.0 : it->second);
        std::printf("%s\"%s/%ld%s\": %.3f", first ? "" : ", ", names[tid].c_str(), tid, tid == self ? "(main)" : "",
                    d / wall);
        first = false;
    }
    std::printf("}}\n");
    (void)hipStreamSynchronize(s);
    return 0;
}
