// How the HIP runtime treats overlapping hipHostRegister ranges, and what a
// page-locked-per-call DMA path really costs (round 5, the round-4 fault in
// register mode: profiles/r04/register_mode_fault.txt).
//
// Part 1 (bookkeeping only, no DMA after any unregister): on fresh anonymous
// mappings, register two page ranges in each overlap arrangement, print each
// call's status, which registration hipHostGetDevicePointer resolves every
// probe page to, then unregister (by base, or by an interior pointer) and list
// every page that is still registered afterwards: a leak.
//
// Part 2 (cost): T threads, each with six 4,404,020-byte heap buffers (mmap
// threshold raised, so buffers sit back to back and share boundary pages, as
// ELECT's direct buffers do once glibc's dynamic threshold has risen), one
// RS(6,4)-shaped call per loop: 4 H2D + 2 D2H of whole units, on the thread's
// stream.  Modes: "pageable" (hipMemcpyAsync from the pageable buffers: the
// runtime stages), "register" (each unit's interior pages registered for the
// call, interior moved by DMA, the <= 2 ragged edge pages by pageable copies,
// then unregistered).  Prints calls/s, data GiB/s, core-ms per GiB.
//
// Part 5 (relock, round 6): see relock() below.
//
//   hipcc --offload-arch=gfx950 -O2 -std=c++17 tools/tune/register_overlap_probe.cpp -L/opt/rocm/lib
//       -lhsa-runtime64 -lpthread -o tools/tune/register_overlap_probe
//   tools/tune/register_overlap_probe [all | S1..S8 | D1 | cost | unregwait | hsalock | relock]
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>
#include <malloc.h>
#include <sys/mman.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <ctime>
#include <string>
#include <thread>
#include <vector>

static const size_t P = 4096;

static double cpu_seconds()
{
    timespec t{};
    clock_gettime(CLOCK_PROCESS_CPUTIME_ID, &t);
    return t.tv_sec + t.tv_nsec * 1e-9;
}

struct Reg {
    size_t page, pages;  // range [page, page + pages) of the mapping
};

// what the runtime says about one page: registered? base offset, device pointer
static std::string page_state(uint8_t* base, size_t page, const std::vector<void*>& devs,
                              const std::vector<Reg>& regs)
{
    uint8_t* p = base + page * P + 100;
    hipPointerAttribute_t a{};
    const hipError_t e = hipPointerGetAttributes(&a, p);
    (void)hipGetLastError();
    char buf[160];
    if (e != hipSuccess || a.type != hipMemoryTypeHost) {
        std::snprintf(buf, sizeof buf, "unreg(rc=%d,type=%d)", static_cast<int>(e), static_cast<int>(a.type));
        return buf;
    }
    void* d = nullptr;
    const hipError_t e2 = hipHostGetDevicePointer(&d, p, 0);
    (void)hipGetLastError();
    int who = -1;
    for (size_t i = 0; i < regs.size(); ++i)
        if (devs[i] && d == static_cast<uint8_t*>(devs[i]) + (page - regs[i].page) * P + 100) who = static_cast<int>(i);
    const long host_off = a.hostPointer ? static_cast<long>((static_cast<uint8_t*>(a.hostPointer) - base) / P) : -1;
    std::snprintf(buf, sizeof buf, "REG(hostbase=page%ld,devptr_rc=%d,resolves_to=R%d)", host_off, static_cast<int>(e2), who);
    return buf;
}

static int scenario(const char* name, std::vector<Reg> regs, std::vector<std::pair<int, size_t>> unreg,
                    size_t npages)
{
    std::printf("\n== %s\n", name);
    const size_t bytes = (npages + 2) * P;
    auto* base = static_cast<uint8_t*>(mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0));
    if (base == MAP_FAILED) return 1;
    std::memset(base, 0x5a, bytes);
    std::vector<void*> devs(regs.size(), nullptr);
    std::vector<bool> ok(regs.size(), false);
    for (size_t i = 0; i < regs.size(); ++i) {
        const hipError_t e = hipHostRegister(base + regs[i].page * P, regs[i].pages * P, hipHostRegisterMapped);
        (void)hipGetLastError();
        ok[i] = e == hipSuccess;
        if (ok[i] && hipHostGetDevicePointer(&devs[i], base + regs[i].page * P, 0) != hipSuccess) devs[i] = nullptr;
        (void)hipGetLastError();
        std::printf("  register R%zu pages [%zu,%zu): rc=%d (%s) dev=%p\n", i, regs[i].page, regs[i].page + regs[i].pages,
                    static_cast<int>(e), hipGetErrorName(e), devs[i]);
    }
    auto snapshot = [&](const char* when) {
        std::printf("  %s:\n", when);
        for (size_t pg = 0; pg < npages; ++pg) std::printf("    page %2zu %s\n", pg, page_state(base, pg, devs, regs).c_str());
    };
    snapshot("after registering");
    for (const auto& u : unreg) {
        if (!ok[u.first]) continue;
        uint8_t* p = base + (regs[u.first].page + u.second) * P;
        const hipError_t e = hipHostUnregister(p);
        (void)hipGetLastError();
        std::printf("  unregister R%d by page %zu (%s): rc=%d (%s)\n", u.first, regs[u.first].page + u.second,
                    u.second ? "interior pointer" : "its base", static_cast<int>(e), hipGetErrorName(e));
        snapshot("  then");
    }
    int leaks = 0;
    for (size_t pg = 0; pg < npages; ++pg) {
        hipPointerAttribute_t a{};
        if (hipPointerGetAttributes(&a, base + pg * P + 100) == hipSuccess && a.type == hipMemoryTypeHost) {
            ++leaks;
            if (a.hostPointer) (void)hipHostUnregister(a.hostPointer);  // clean up before munmap
        }
        (void)hipGetLastError();
    }
    std::printf("  RESULT %s: %d page(s) still registered after every unregister%s\n", name, leaks,
                leaks ? "  <-- LEAK" : "");
    munmap(base, bytes);
    return leaks;
}

// Adjacent, disjoint registrations with DMA: a copy spanning both, then R0
// unregistered and a copy from R1's pages alone (its pages must still be mapped).
static int adjacent_dma()
{
    std::printf("\n== D1 R0=[0,4) and R1=[4,8) adjacent: DMA across both, unregister R0, DMA from R1\n");
    const size_t npages = 8, bytes = (npages + 2) * P;
    auto* base = static_cast<uint8_t*>(mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0));
    if (base == MAP_FAILED) return 1;
    for (size_t i = 0; i < bytes; ++i) base[i] = static_cast<uint8_t>(i * 7 + 3);
    uint8_t* dev = nullptr;
    if (hipMalloc(reinterpret_cast<void**>(&dev), npages * P) != hipSuccess) return 1;
    std::vector<uint8_t> back(npages * P);
    int bad = 0;
    hipError_t e0 = hipHostRegister(base, 4 * P, hipHostRegisterDefault);
    hipError_t e1 = hipHostRegister(base + 4 * P, 4 * P, hipHostRegisterDefault);
    std::printf("  register rc %d %d\n", static_cast<int>(e0), static_cast<int>(e1));
    hipError_t e = hipMemcpy(dev, base + 100, 8 * P - 200, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(back.data(), dev, 8 * P - 200, hipMemcpyDeviceToHost);
    bad += e != hipSuccess || std::memcmp(back.data(), base + 100, 8 * P - 200) != 0;
    std::printf("  copy across both: rc=%d %s\n", static_cast<int>(e), bad ? "MISMATCH" : "ok");
    e = hipHostUnregister(base);
    std::printf("  unregister R0: rc=%d\n", static_cast<int>(e));
    e = hipMemcpy(dev, base + 4 * P + 8, 4 * P - 16, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(back.data(), dev, 4 * P - 16, hipMemcpyDeviceToHost);
    const int bad2 = e != hipSuccess || std::memcmp(back.data(), base + 4 * P + 8, 4 * P - 16) != 0;
    std::printf("  copy from R1 after R0 is gone: rc=%d %s\n", static_cast<int>(e), bad2 ? "MISMATCH" : "ok");
    e = hipHostUnregister(base + 4 * P);
    std::printf("  unregister R1: rc=%d\n", static_cast<int>(e));
    (void)hipFree(dev);
    munmap(base, bytes);
    std::printf("  RESULT D1: %s\n", bad + bad2 ? "BAD" : "ok");
    return bad + bad2;
}

static int part1(const std::string& which)
{
    std::printf("# part 1: registrations on one anonymous mapping (%s)\n", which.c_str());
    int leaks = 0;
    auto want = [&](const char* id) { return which == "all" || which == id; };
    if (want("S5")) leaks += scenario("S5 R1=[0,4) then R2=[4,8) (adjacent, disjoint)", {{0, 4}, {4, 4}}, {{0, 0}, {1, 0}}, 8);
    if (want("D1")) leaks += adjacent_dma();
    if (want("S6")) leaks += scenario("S6 R1=[0,8) unregistered by an interior pointer", {{0, 8}}, {{0, 4}}, 8);
    if (want("S7")) leaks += scenario("S7 R1=[0,8) registered twice", {{0, 8}, {0, 8}}, {{0, 0}, {1, 0}}, 8);
    if (want("S1")) leaks += scenario("S1 R1=[0,8) then R2=[4,12) (R2 starts inside R1)", {{0, 8}, {4, 8}}, {{0, 0}, {1, 0}}, 12);
    if (want("S2"))
        leaks += scenario("S2 R1=[4,12) then R2=[0,8) (R2 starts before R1, overlaps; R1 freed first)", {{4, 8}, {0, 8}},
                          {{0, 0}, {1, 0}}, 12);
    if (want("S3")) leaks += scenario("S3 R1=[4,8) then R2=[0,12) (R2 contains R1)", {{4, 4}, {0, 12}}, {{0, 0}, {1, 0}}, 12);
    if (want("S4")) leaks += scenario("S4 R1=[0,12) then R2=[4,8) (R2 inside R1)", {{0, 12}, {4, 4}}, {{1, 0}, {0, 0}}, 12);
    if (want("S8")) leaks += scenario("S8 R1=[0,8) then R2=[0,12) (same base, longer)", {{0, 8}, {0, 12}}, {{0, 0}, {1, 0}}, 12);
    std::printf("# part 1 (%s) total: %d\n", which.c_str(), leaks);
    return leaks;
}

static double thread_cpu()
{
    timespec t{};
    clock_gettime(CLOCK_THREAD_CPUTIME_ID, &t);
    return t.tv_sec + t.tv_nsec * 1e-9;
}

static void part2(double secs)
{
    std::printf("\n# part 2: one RS(6,4) call per loop, 6 x 4,404,020 B heap buffers per thread (blocking sync)\n");
    mallopt(M_MMAP_THRESHOLD, 64 << 20);  // heap buffers, back to back (ELECT's after glibc's threshold rises)
    const size_t L = 4404020;
    struct Mode {
        const char* name;
        int reg;  // 0 pageable, 1 register (flags below)
        unsigned flags;
        int sem;  // concurrent register/unregister calls allowed (0: any)
    };
    const Mode modes[] = {{"pageable", 0, 0, 0},           {"reg-default", 1, hipHostRegisterDefault, 0},
                          {"reg-mapped", 1, hipHostRegisterMapped, 0}, {"reg-default-sem4", 1, hipHostRegisterDefault, 4},
                          {"reg-mapped-sem4", 1, hipHostRegisterMapped, 4}};
    for (const Mode& md : modes)
        for (int T : {1, 8, 64}) {
            std::atomic<int> sem_free{md.sem};
            auto sem_take = [&] {
                if (!md.sem) return;
                for (;;) {
                    int v = sem_free.load();
                    if (v > 0 && sem_free.compare_exchange_weak(v, v - 1)) return;
                    std::this_thread::yield();
                }
            };
            auto sem_give = [&] {
                if (md.sem) sem_free.fetch_add(1);
            };
            const int mode = md.reg;
            std::atomic<long> calls{0};
            std::atomic<bool> stop{false};
            std::atomic<int> errors{0}, regfail{0};
            std::atomic<long> reg_ns{0}, unreg_ns{0}, issue_ns{0};
            std::vector<std::thread> th;
            const double c0 = cpu_seconds();
            const auto t0 = std::chrono::steady_clock::now();
            for (int t = 0; t < T; ++t)
                th.emplace_back([&, mode] {
                    (void)hipSetDevice(0);
                    hipStream_t s;
                    (void)hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
                    hipEvent_t ev;
                    (void)hipEventCreateWithFlags(&ev, hipEventBlockingSync | hipEventDisableTiming);
                    uint8_t* dev = nullptr;
                    (void)hipMalloc(reinterpret_cast<void**>(&dev), 6 * L);
                    std::vector<uint8_t*> b(6);
                    for (auto& p : b) {
                        p = static_cast<uint8_t*>(std::malloc(L));
                        std::memset(p, 1, L);
                    }
                    while (!stop.load(std::memory_order_relaxed)) {
                        std::vector<uint8_t*> regd;
                        double r = 0, is = 0;
                        for (int j = 0; j < 6; ++j) {
                            uint8_t* h = b[j];
                            uint8_t* d = dev + j * L;
                            const bool in = j < 4;
                            const double q0 = thread_cpu();
                            if (mode == 0) {
                                if ((in ? hipMemcpyAsync(d, h, L, hipMemcpyHostToDevice, s)
                                        : hipMemcpyAsync(h, d, L, hipMemcpyDeviceToHost, s)) != hipSuccess)
                                    errors++;
                                is += thread_cpu() - q0;
                                continue;
                            }
                            const uintptr_t a = reinterpret_cast<uintptr_t>(h);
                            const uintptr_t lo = (a + P - 1) & ~(P - 1), hi = (a + L) & ~(P - 1);
                            sem_take();
                            const hipError_t re = hipHostRegister(reinterpret_cast<void*>(lo), hi - lo, md.flags);
                            sem_give();
                            if (re != hipSuccess) {
                                (void)hipGetLastError();
                                regfail++;
                            } else {
                                regd.push_back(reinterpret_cast<uint8_t*>(lo));
                            }
                            const double q1 = thread_cpu();
                            r += q1 - q0;
                            const size_t head = lo - a, mid = hi - lo, tail = a + L - hi;
                            hipError_t e = hipSuccess;
                            auto cp = [&](size_t off, size_t n) {
                                if (!n || e != hipSuccess) return;
                                e = in ? hipMemcpyAsync(d + off, h + off, n, hipMemcpyHostToDevice, s)
                                       : hipMemcpyAsync(h + off, d + off, n, hipMemcpyDeviceToHost, s);
                            };
                            cp(0, head);
                            cp(head, mid);
                            cp(head + mid, tail);
                            if (e != hipSuccess) errors++;
                            is += thread_cpu() - q1;
                        }
                        if (hipEventRecord(ev, s) != hipSuccess || hipEventSynchronize(ev) != hipSuccess) errors++;
                        const double u0 = thread_cpu();
                        for (uint8_t* x : regd) {
                            sem_take();
                            if (hipHostUnregister(x) != hipSuccess) errors++;
                            sem_give();
                        }
                        unreg_ns += static_cast<long>((thread_cpu() - u0) * 1e9);
                        reg_ns += static_cast<long>(r * 1e9);
                        issue_ns += static_cast<long>(is * 1e9);
                        calls++;
                    }
                    for (auto* p : b) std::free(p);
                    (void)hipFree(dev);
                    (void)hipEventDestroy(ev);
                    (void)hipStreamDestroy(s);
                });
            std::this_thread::sleep_for(std::chrono::duration<double>(secs));
            stop = true;
            for (auto& x : th) x.join();
            const double wall = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
            const double cpu = cpu_seconds() - c0;
            const double gib = calls.load() * 4.0 * L / (1u << 30);
            std::printf("%-16s T=%-3d calls/s %7.1f data GiB/s %6.2f | core-ms/GiB: all %7.1f register %6.1f "
                        "unregister %6.1f issue(memcpyAsync) %6.1f | errors %d regfail %d\n",
                        md.name, T, calls.load() / wall, gib / wall, cpu * 1e3 / gib,
                        reg_ns.load() * 1e-6 / gib, unreg_ns.load() * 1e-6 / gib, issue_ns.load() * 1e-6 / gib,
                        errors.load(), regfail.load());
            std::fflush(stdout);
        }
}

// Does hipHostUnregister wait for unrelated device work?  Stream A copies 2 GiB
// device-to-device a few times (tens of ms of HBM traffic); meanwhile this thread
// registers a pageable 4 MiB buffer (never used by any transfer) and unregisters
// it; the wall time of each call against A's remaining work.
static void unregwait()
{
    std::printf("\n# part 3: hipHostUnregister while another stream is busy\n");
    const size_t big = size_t{2} << 30, L = size_t{4} << 20;
    uint8_t *a = nullptr, *b = nullptr;
    if (hipMalloc(reinterpret_cast<void**>(&a), big) != hipSuccess || hipMalloc(reinterpret_cast<void**>(&b), big) != hipSuccess)
        return;
    hipStream_t s;
    (void)hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    auto* h = static_cast<uint8_t*>(std::aligned_alloc(4096, L));
    std::memset(h, 1, L);
    for (int busy = 0; busy < 2; ++busy) {
        (void)hipDeviceSynchronize();
        hipEvent_t e0, e1;
        (void)hipEventCreate(&e0);
        (void)hipEventCreate(&e1);
        (void)hipEventRecord(e0, s);
        if (busy)
            for (int i = 0; i < 8; ++i) (void)hipMemcpyAsync(b, a, big, hipMemcpyDeviceToDevice, s);
        (void)hipEventRecord(e1, s);
        const auto t0 = std::chrono::steady_clock::now();
        const hipError_t r = hipHostRegister(h, L, hipHostRegisterDefault);
        const auto t1 = std::chrono::steady_clock::now();
        const hipError_t u = hipHostUnregister(h);
        const auto t2 = std::chrono::steady_clock::now();
        const bool pending_after = hipEventQuery(e1) == hipErrorNotReady;
        (void)hipEventSynchronize(e1);
        const auto t3 = std::chrono::steady_clock::now();
        float ms = 0;
        (void)hipEventElapsedTime(&ms, e0, e1);
        auto d = [](auto x, auto y) { return std::chrono::duration<double, std::milli>(y - x).count(); };
        std::printf("other stream %s (%.1f ms of copies): register %.3f ms rc=%d, unregister %.3f ms rc=%d, "
                    "other stream still busy after unregister: %s (finished %.1f ms later)\n",
                    busy ? "busy" : "idle", ms, d(t0, t1), static_cast<int>(r), d(t1, t2), static_cast<int>(u),
                    pending_after ? "yes" : "no", d(t2, t3));
        (void)hipEventDestroy(e0);
        (void)hipEventDestroy(e1);
    }
    std::free(h);
    (void)hipFree(a);
    (void)hipFree(b);
    (void)hipStreamDestroy(s);
}

// Part 4: the HSA-level lock (hsa_amd_memory_lock, which the HSA header says
// permits overlapping locks, each with its own agent pointer): its cost, whether
// hsa_amd_memory_unlock waits for unrelated device work, and how fast a kernel
// reads / writes locked host memory through the agent pointer (the gather /
// scatter a batched zero-copy path would use).
__global__ void pcie_copy(const uint4* __restrict__ src, uint4* __restrict__ dst, size_t n16)
{
    for (size_t i = blockIdx.x * size_t{blockDim.x} + threadIdx.x; i < n16; i += size_t{gridDim.x} * blockDim.x)
        dst[i] = src[i];
}

static hsa_status_t find_gpu(hsa_agent_t a, void* out)
{
    hsa_device_type_t t;
    hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t);
    if (t == HSA_DEVICE_TYPE_GPU) {
        *static_cast<hsa_agent_t*>(out) = a;
        return HSA_STATUS_INFO_BREAK;
    }
    return HSA_STATUS_SUCCESS;
}

static void hsalock()
{
    std::printf("\n# part 4: hsa_amd_memory_lock / unlock, and kernels over locked host memory\n");
    if (hsa_init() != HSA_STATUS_SUCCESS) {
        std::printf("hsa_init failed\n");
        return;
    }
    hsa_agent_t gpu{};
    hsa_iterate_agents(find_gpu, &gpu);
    const size_t L = 4404020, N = 64;
    mallopt(M_MMAP_THRESHOLD, 1 << 30);
    std::vector<uint8_t*> bufs(N);
    for (auto& b : bufs) {
        b = static_cast<uint8_t*>(std::malloc(L));
        std::memset(b, 7, L);
    }
    // lock / unlock cost, units back to back on the heap (overlapping page ranges)
    auto d = [](auto x, auto y) { return std::chrono::duration<double, std::milli>(y - x).count(); };
    std::vector<void*> ap(N);
    double c0 = thread_cpu();
    auto t0 = std::chrono::steady_clock::now();
    int fails = 0;
    for (size_t i = 0; i < N; ++i)
        if (hsa_amd_memory_lock(bufs[i], L, &gpu, 1, &ap[i]) != HSA_STATUS_SUCCESS) ++fails;
    auto t1 = std::chrono::steady_clock::now();
    double c1 = thread_cpu();
    std::printf("lock %zu x %zu B (heap neighbours): %.3f ms wall, %.3f ms cpu (%.1f core-ms/GiB), %d failed; "
                "agent_ptr == host ptr: %s\n", N, L, d(t0, t1), (c1 - c0) * 1e3, (c1 - c0) * 1e3 / (N * L / 1073741824.0),
                fails, ap[0] == bufs[0] ? "yes" : "no");
    // kernel reads every locked unit into device memory (gather), then writes them back (scatter)
    uint8_t* dev = nullptr;
    (void)hipMalloc(reinterpret_cast<void**>(&dev), N * L);
    hipStream_t s;
    (void)hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    for (int dir = 0; dir < 2; ++dir)
        for (int rep = 0; rep < 3; ++rep) {
            hipEvent_t e0, e1;
            (void)hipEventCreate(&e0);
            (void)hipEventCreate(&e1);
            (void)hipEventRecord(e0, s);
            for (size_t i = 0; i < N; ++i) {
                const size_t n16 = L / 16;
                if (dir == 0)
                    pcie_copy<<<1024, 256, 0, s>>>(static_cast<const uint4*>(ap[i]), reinterpret_cast<uint4*>(dev + i * L), n16);
                else
                    pcie_copy<<<1024, 256, 0, s>>>(reinterpret_cast<const uint4*>(dev + i * L), static_cast<uint4*>(ap[i]), n16);
            }
            (void)hipEventRecord(e1, s);
            (void)hipEventSynchronize(e1);
            float ms = 0;
            (void)hipEventElapsedTime(&ms, e0, e1);
            std::printf("kernel %s locked host memory: %.2f ms for %.1f MB = %.1f GB/s (rc %d)\n",
                        dir ? "writes" : "reads", ms, N * L / 1e6, N * L / 1e6 / ms, static_cast<int>(hipGetLastError()));
        }
    bool ok = true;
    for (size_t i = 0; i < N && ok; ++i) ok = bufs[i][0] == 7 && bufs[i][L - 1] == 7;
    std::printf("round trip intact: %s\n", ok ? "yes" : "NO");
    // unlock while another stream is busy
    uint8_t *a = nullptr, *b = nullptr;
    const size_t big = size_t{2} << 30;
    (void)hipMalloc(reinterpret_cast<void**>(&a), big);
    (void)hipMalloc(reinterpret_cast<void**>(&b), big);
    hipEvent_t e1;
    (void)hipEventCreate(&e1);
    for (int i = 0; i < 8; ++i) (void)hipMemcpyAsync(b, a, big, hipMemcpyDeviceToDevice, s);
    (void)hipEventRecord(e1, s);
    c0 = thread_cpu();
    t0 = std::chrono::steady_clock::now();
    for (size_t i = 0; i < N; ++i) (void)hsa_amd_memory_unlock(bufs[i]);
    t1 = std::chrono::steady_clock::now();
    c1 = thread_cpu();
    const bool busy = hipEventQuery(e1) == hipErrorNotReady;
    std::printf("unlock %zu units while another stream copies: %.3f ms wall, %.3f ms cpu (%.1f core-ms/GiB); "
                "other stream still busy after: %s\n", N, d(t0, t1), (c1 - c0) * 1e3,
                (c1 - c0) * 1e3 / (N * L / 1073741824.0), busy ? "yes (unlock did not wait)" : "no");
    (void)hipEventSynchronize(e1);
    // threads: lock + unlock of 6 units per loop, T threads, 1 s
    for (int T : {1, 8, 64}) {
        std::atomic<long> loops{0};
        std::atomic<bool> stop{false};
        std::atomic<int> err{0};
        std::vector<std::thread> th;
        const double p0 = cpu_seconds();
        const auto w0 = std::chrono::steady_clock::now();
        for (int t = 0; t < T; ++t)
            th.emplace_back([&, t] {
                std::vector<uint8_t*> mine(6);
                for (auto& x : mine) {
                    x = static_cast<uint8_t*>(std::malloc(L));
                    std::memset(x, t, L);
                }
                while (!stop.load()) {
                    void* q = nullptr;
                    for (auto* x : mine)
                        if (hsa_amd_memory_lock(x, L, &gpu, 1, &q) != HSA_STATUS_SUCCESS) err++;
                    for (auto* x : mine)
                        if (hsa_amd_memory_unlock(x) != HSA_STATUS_SUCCESS) err++;
                    loops++;
                }
                for (auto* x : mine) std::free(x);
            });
        std::this_thread::sleep_for(std::chrono::seconds(1));
        stop = true;
        for (auto& x : th) x.join();
        const double wall = d(w0, std::chrono::steady_clock::now()) / 1e3, cpu = cpu_seconds() - p0;
        const double gib = loops.load() * 6.0 * L / 1073741824.0;
        std::printf("lock+unlock T=%-2d: %.0f units/s, %.1f GiB/s of units, %.1f core-ms per GiB of units, %d errors\n",
                    T, loops.load() * 6 / wall, gib / wall, cpu * 1e3 / gib, err.load());
    }
    (void)hipFree(a);
    (void)hipFree(b);
    (void)hipFree(dev);
    for (auto* x : bufs) std::free(x);
}


// Part 5 (round 6): do stale GPU mappings survive
// hsa_amd_memory_unlock?  The round-5 zero-copy fault (ECDeviceError in
// test_lone_caller_copy_fanout) was put down to "the HSA runtime keeps unlocked
// ranges cached"; this checks the mechanism.  On an anonymous mapping: lock
// pages [4, 36), read (kernel), write (kernel) and DMA-read (SDMA,
// hsa_amd_memory_async_copy) through the returned address, unlock; then the
// mapping's pages are REPLACED (munmap + mmap MAP_FIXED: new physical pages at
// the same virtual addresses, as a free + malloc can do) and refilled with a new
// pattern; then overlapping, shifted [10, 50) is locked and read / written /
// DMA'd again, and so is the identical [4, 36), and hipHostRegister of
// [8, 40) (round 5's two-layer sequence).  A stale cached translation would
// show the old pattern (or a fault) on the device side.
__global__ void fill_kernel(uint4* dst, size_t n16, uint32_t v)
{
    for (size_t i = blockIdx.x * size_t{blockDim.x} + threadIdx.x; i < n16; i += size_t{gridDim.x} * blockDim.x)
        dst[i] = make_uint4(v, v, v, v);
}

static void relock()
{
    std::printf("\n# part 5: lock, unlock, replace the pages, relock overlapping / shifted / identical\n");
    if (hsa_init() != HSA_STATUS_SUCCESS) {
        std::printf("hsa_init failed\n");
        return;
    }
    hsa_agent_t gpu{}, cpu{};
    hsa_iterate_agents(find_gpu, &gpu);
    hsa_iterate_agents(
        [](hsa_agent_t a, void* out) -> hsa_status_t {
            hsa_device_type_t t;
            hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t);
            if (t == HSA_DEVICE_TYPE_CPU) {
                *static_cast<hsa_agent_t*>(out) = a;
                return HSA_STATUS_INFO_BREAK;
            }
            return HSA_STATUS_SUCCESS;
        },
        &cpu);
    const size_t pages = 64, bytes = pages * P;
    auto* map = static_cast<uint8_t*>(mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0));
    uint8_t* dev = nullptr;
    (void)hipMalloc(reinterpret_cast<void**>(&dev), bytes);
    hipStream_t s;
    (void)hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    hsa_signal_t sig{};
    hsa_signal_create(1, 0, nullptr, &sig);
    std::vector<uint8_t> back(bytes);
    auto fill_host = [&](uint8_t v) {
        for (size_t i = 0; i < bytes; ++i) map[i] = static_cast<uint8_t>(v + i / P);
    };
    // the device's view of [lo, hi) pages through address ap: kernel read, then SDMA read, each checked against host
    auto check_view = [&](const char* tag, void* ap, size_t lo, size_t hi, uint8_t v) {
        const size_t n = (hi - lo) * P;
        (void)hipMemsetAsync(dev, 0, n, s);
        pcie_copy<<<256, 256, 0, s>>>(static_cast<const uint4*>(ap), reinterpret_cast<uint4*>(dev), n / 16);
        hipError_t e = hipMemcpyAsync(back.data(), dev, n, hipMemcpyDeviceToHost, s);
        if (e == hipSuccess) e = hipStreamSynchronize(s);
        size_t bad_k = 0;
        for (size_t i = 0; i < n; ++i) bad_k += back[i] != static_cast<uint8_t>(v + (lo * P + i) / P);
        (void)hipMemset(dev, 0, n);
        hsa_signal_store_screlease(sig, 1);
        const hsa_status_t hs = hsa_amd_memory_async_copy(dev, gpu, ap, cpu, n, 0, nullptr, sig);
        if (hs == HSA_STATUS_SUCCESS)
            hsa_signal_wait_scacquire(sig, HSA_SIGNAL_CONDITION_LT, 1, UINT64_MAX, HSA_WAIT_STATE_BLOCKED);
        (void)hipMemcpy(back.data(), dev, n, hipMemcpyDeviceToHost);
        size_t bad_d = 0;
        for (size_t i = 0; i < n; ++i) bad_d += back[i] != static_cast<uint8_t>(v + (lo * P + i) / P);
        // kernel write through the mapping, seen by the CPU at the host address
        fill_kernel<<<64, 256, 0, s>>>(static_cast<uint4*>(ap), P / 16, 0xA5A5A5A5u);
        const hipError_t ew = hipStreamSynchronize(s);
        const bool w_ok = ew == hipSuccess && map[lo * P] == 0xA5 && map[lo * P + P - 1] == 0xA5;
        for (size_t i = lo * P; i < lo * P + P; ++i) map[i] = static_cast<uint8_t>(v + i / P);  // restore
        std::printf("%-44s agent ptr %s host: kernel read %s (%zu bad), DMA read %s (%zu bad, status %d), "
                    "kernel write %s (rc %d/%d)\n",
                    tag, ap == map + lo * P ? "==" : "!=", bad_k ? "STALE" : "ok", bad_k, bad_d ? "STALE" : "ok", bad_d,
                    static_cast<int>(hs), w_ok ? "seen" : "NOT SEEN", static_cast<int>(e), static_cast<int>(ew));
    };
    auto lock = [&](size_t lo, size_t hi, void** ap) {
        return hsa_amd_memory_lock(map + lo * P, (hi - lo) * P, &gpu, 1, ap);
    };
    fill_host(10);
    void* ap = nullptr;
    hsa_status_t st = lock(4, 36, &ap);
    std::printf("lock [4, 36): status %d\n", static_cast<int>(st));
    if (st == HSA_STATUS_SUCCESS) check_view("[4, 36) locked", ap, 4, 36, 10);
    std::printf("unlock [4, 36): status %d\n", static_cast<int>(hsa_amd_memory_unlock(map + 4 * P)));
    // new physical pages at the same virtual addresses
    munmap(map, bytes);
    auto* again = static_cast<uint8_t*>(mmap(map, bytes, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS | MAP_FIXED, -1, 0));
    std::printf("remapped at the same address: %s\n", again == map ? "yes" : "NO");
    fill_host(100);
    st = lock(10, 50, &ap);
    std::printf("lock [10, 50) after the remap (overlapping, shifted): status %d\n", static_cast<int>(st));
    if (st == HSA_STATUS_SUCCESS) {
        check_view("[10, 50) relocked, shifted", ap, 10, 50, 100);
        std::printf("unlock [10, 50): status %d\n", static_cast<int>(hsa_amd_memory_unlock(map + 10 * P)));
    }
    st = lock(4, 36, &ap);
    std::printf("lock [4, 36) again (identical extent): status %d\n", static_cast<int>(st));
    if (st == HSA_STATUS_SUCCESS) {
        check_view("[4, 36) relocked, identical", ap, 4, 36, 100);
        std::printf("unlock [4, 36): status %d\n", static_cast<int>(hsa_amd_memory_unlock(map + 4 * P)));
    }
    // round 5's two-layer sequence: an HSA lock and unlock, then hipHostRegister of an overlapping range
    hipError_t he = hipHostRegister(map + 8 * P, 32 * P, hipHostRegisterMapped);
    void* hp = nullptr;
    if (he == hipSuccess) he = hipHostGetDevicePointer(&hp, map + 8 * P, 0);
    std::printf("hipHostRegister [8, 40) after the HSA unlock: rc %d\n", static_cast<int>(he));
    if (he == hipSuccess) {
        check_view("[8, 40) hipHostRegister'ed", hp, 8, 40, 100);
        std::printf("hipHostUnregister: rc %d\n", static_cast<int>(hipHostUnregister(map + 8 * P)));
    }
    (void)hipGetLastError();
    hsa_signal_destroy(sig);
    (void)hipFree(dev);
    munmap(map, bytes);
}

int main(int argc, char** argv)
{
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) {
        std::printf("no device\n");
        return 1;
    }
    const std::string what = argc > 1 ? argv[1] : "all";
    (void)hipSetDevice(0);
    if (what == "cost") (void)hipSetDeviceFlags(hipDeviceScheduleBlockingSync);
    (void)hipFree(nullptr);
    if (what == "hsalock") {
        hsalock();
        return 0;
    }
    if (what == "relock") {
        relock();
        return 0;
    }
    if (what == "unregwait") {
        unregwait();
        return 0;
    }
    if (what == "cost") {
        part2(argc > 2 ? std::atof(argv[2]) : 2.0);
        return 0;
    }
    return part1(what) ? 3 : 0;  // a scenario id (S1..S8, D1) or "all"
}
