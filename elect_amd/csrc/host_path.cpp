// host_path.cpp — host-memory path of the C ABI (include/elect_ec.h):
// the JNI calling convention, one synchronous stripe per call
// (EC/NativeRSEncoder.c:43-61 -> EC/erasure_coder.c:74-98).
#include "host_path.hpp"

#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>

#include <emmintrin.h>
#include <pthread.h>
#include <sys/prctl.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <ctime>
#include <cstring>
#include <functional>
#include <memory>
#include <map>
#include <mutex>
#include <shared_mutex>
#include <new>
#include <string>
#include <thread>
#include <vector>

namespace elect {
namespace host {
namespace {

using kern::ApplyParams;

// Waiting for the device.  Every waiting primitive of this HIP runtime spins a
// core while the work it waits for runs (hipStreamSynchronize, hipEventSynchronize
// also on hipEventBlockingSync events, and the runtime thread that runs
// hipLaunchHostFunc callbacks; tools/tune/spin_probe.cpp, profiles/r05/
// spin_probe.txt).  So the batcher's completions come from a poller thread per
// device that queries events and sleeps in between (Batcher::poller: 35 -> 17
// core-ms per GiB at 64 callers on pageable units, 28 -> 9 on pool units, the
// same GiB/s; profiles/r05/completion_poll_ab.txt), and the per-thread engine
// waits with wait_sleeping.  (Round 4's completion thread sleeping on
// hipEventBlockingSync events saved no CPU for that reason, and lost throughput:
// profiles/r04/hostwait_ab.txt.)

// Host copies into and out of the pinned staging memory, with non-temporal
// (streaming) stores: the data is not read again by this CPU (the DMA engine
// reads the arena; the caller reads its output later), so write-allocate reads
// of the destination lines would only double the host-DRAM traffic this path
// is bound by.  glibc's memcpy streams only above its non-temporal threshold,
// which 64 KiB tile copies are far below.  Callers fence (_mm_sfence) before
// the data is handed on.  (AVX-512 64-byte streaming stores measured no better:
// 64 callers the same, 16 callers 32.0-35.8 against 40.6-42.8 GiB/s,
// profiles/r04/copy_isa_ab.txt.)
void stream_copy(uint8_t* dst, const uint8_t* src, size_t n)
{
    if (n >= 4096) {
        const size_t head = (16 - (reinterpret_cast<uintptr_t>(dst) & 15)) & 15;
        std::memcpy(dst, src, head);
        dst += head;
        src += head;
        n -= head;
        const size_t body = n & ~size_t{63};
        for (size_t i = 0; i < body; i += 64) {
            const __m128i a = _mm_loadu_si128(reinterpret_cast<const __m128i*>(src + i));
            const __m128i b = _mm_loadu_si128(reinterpret_cast<const __m128i*>(src + i + 16));
            const __m128i c = _mm_loadu_si128(reinterpret_cast<const __m128i*>(src + i + 32));
            const __m128i d = _mm_loadu_si128(reinterpret_cast<const __m128i*>(src + i + 48));
            _mm_stream_si128(reinterpret_cast<__m128i*>(dst + i), a);
            _mm_stream_si128(reinterpret_cast<__m128i*>(dst + i + 16), b);
            _mm_stream_si128(reinterpret_cast<__m128i*>(dst + i + 32), c);
            _mm_stream_si128(reinterpret_cast<__m128i*>(dst + i + 48), d);
        }
        dst += body;
        src += body;
        n -= body;
    }
    std::memcpy(dst, src, n);
}

// ---------------------------------------------------------------------------
// Page-locked buffers for the callers' own units (elect_ec_host_alloc).  ELECT
// allocates a direct ByteBuffer per unit and stripe and copies the SSTable into
// it (ECMessageVerbHandler.java:298-314); when those buffers come from here,
// the batcher's gather / scatter kernels move a call's units straight between
// them and the device
// (Batcher, direct batches): no staging copies, which are most of the CPU the
// pageable path costs (1.5 bytes copied per data byte).
// Pooled by size class (64 KiB steps): ELECT frees its buffers after every
// stripe, and page-locking a 4.4 MB buffer costs far more than reusing one.
// When page-locked memory cannot be had (no device, a locked-memory limit) the
// allocation is ordinary memory, and calls on it take the staged path.
// ---------------------------------------------------------------------------
class PinnedPool {
public:
    static PinnedPool& get()
    {
        static PinnedPool* pool = new PinnedPool();  // never destroyed: buffers may outlive static teardown
        return *pool;
    }

    void* alloc(size_t bytes)
    {
        const size_t cls = std::max<size_t>(kClass, (bytes + kClass - 1) / kClass * kClass);
        // Free blocks are kept per NUMA node: a block's pages were faulted in (locked) by the
        // thread that made it, on that thread's node, and go back to a thread on the same
        // node (the one the NUMA-aware device choice gives a GPU on).
        const int node = current_node();
        {
            std::unique_lock<std::shared_mutex> lock(mu_);
            auto it = free_.find(Key{node, cls});
            if (it != free_.end() && !it->second.empty()) {
                void* p = it->second.back();
                it->second.pop_back();
                free_bytes_ -= cls;
                live_[reinterpret_cast<uintptr_t>(p)] = Block{cls, true, delta_[p], node};
                return p;
            }
        }
        void* p = nullptr;
        intptr_t delta = 0;  // device address - host address (the batches' kernels read the units there)
        bool pinned = false;
        if (kind() == kHsaLock) {  // A/B: ordinary memory locked for every agent (as the pageable path's units)
            p = std::aligned_alloc(4096, cls);
            if (!p) return nullptr;
            void* ap = nullptr;
            static const bool hsa = hsa_init() == HSA_STATUS_SUCCESS;  // once (reference counted)
            pinned = hsa && hsa_amd_memory_lock(p, cls, nullptr, 0, &ap) == HSA_STATUS_SUCCESS;
            if (pinned) delta = reinterpret_cast<intptr_t>(ap) - reinterpret_cast<intptr_t>(p);
        } else {
            const unsigned flags = hipHostMallocPortable | (kind() == kNonCoherent ? hipHostMallocNonCoherent : 0u) |
                                   (kind() == kCoherent ? hipHostMallocCoherent : 0u);
            const hipError_t e = hipHostMalloc(&p, cls, flags);
            pinned = e == hipSuccess && p;
            if (!pinned) {
                if (std::getenv("ELECT_EC_DEBUG"))
                    std::fprintf(stderr, "elect_ec_host_alloc: hipHostMalloc(%zu) failed: %s\n", cls, hipGetErrorString(e));
                (void)hipGetLastError();
                p = std::aligned_alloc(4096, cls);
                if (!p) return nullptr;
            }
        }
        if (pinned && kind() != kHsaLock) {
            void* d = nullptr;
            if (hipHostGetDevicePointer(&d, p, 0) == hipSuccess)
                delta = reinterpret_cast<intptr_t>(d) - reinterpret_cast<intptr_t>(p);
            (void)hipGetLastError();
        }
        try {
            std::unique_lock<std::shared_mutex> lock(mu_);
            live_[reinterpret_cast<uintptr_t>(p)] = Block{cls, pinned, delta, node};
            if (pinned) delta_[p] = delta;
        } catch (...) {  // no record, no buffer: nothing leaks
            release_block(p, pinned);
            return nullptr;
        }
        return p;
    }

    // How page-locked blocks are made (ELECT_EC_POOL_ALLOC): aligned_alloc +
    // hsa_amd_memory_lock for every agent ("hsalock", the default), or
    // hipHostMalloc with the runtime's default coherence ("hip"), non-coherent
    // ("nc") or coherent ("coherent").  The batches' gather / scatter kernels
    // move 64 callers' pool units at 49.3-49.4 GiB/s from locked blocks against
    // 46.9-47.7 from any hipHostMalloc kind (profiles/r05/pool_alloc_ab.txt).
    // The library reaches pool units only through kernels at their device
    // address (direct batches, zero-copy) or by CPU copies (the per-thread
    // engine).
    enum Kind { kHip, kNonCoherent, kCoherent, kHsaLock };
    static Kind kind()
    {
        static const Kind k = [] {
            const char* e = std::getenv("ELECT_EC_POOL_ALLOC");
            const std::string v = e ? e : "";
            return v == "hip" ? kHip : v == "nc" ? kNonCoherent : v == "coherent" ? kCoherent : kHsaLock;
        }();
        return k;
    }

    static void release_block(void* p, bool pinned)
    {
        if (pinned && kind() != kHsaLock) {
            (void)hipHostFree(p);
            return;
        }
        if (pinned) (void)hsa_amd_memory_unlock(p);
        std::free(p);
    }

    bool free(void* p)
    {
        Block b;
        {
            std::unique_lock<std::shared_mutex> lock(mu_);
            auto it = live_.find(reinterpret_cast<uintptr_t>(p));
            if (it == live_.end()) return false;
            b = it->second;
            live_.erase(it);
            if (b.pinned && free_bytes_ + b.size <= cap()) {
                try {
                    free_[Key{b.node, b.size}].push_back(p);
                    free_bytes_ += b.size;
                    return true;
                } catch (...) {  // no room in the free list: release the buffer below
                }
            }
        }
        release_block(p, b.pinned);
        return true;
    }

    // [p, p + n) lies inside one live page-locked block.
    bool pinned(const void* p, size_t n) const
    {
        const uintptr_t a = reinterpret_cast<uintptr_t>(p);
        std::shared_lock<std::shared_mutex> lock(mu_);
        if (live_.empty()) return false;
        auto it = live_.upper_bound(a);
        if (it == live_.begin()) return false;
        --it;
        return it->second.pinned && a + n <= it->first + it->second.size;
    }

    // Device address of p (inside a live page-locked block).
    uintptr_t device_addr(const void* p) const
    {
        const uintptr_t a = reinterpret_cast<uintptr_t>(p);
        std::shared_lock<std::shared_mutex> lock(mu_);
        auto it = live_.upper_bound(a);
        if (it == live_.begin()) return a;
        --it;
        return a + static_cast<uintptr_t>(it->second.delta);
    }

    bool any() const
    {
        std::shared_lock<std::shared_mutex> lock(mu_);
        return !live_.empty();
    }

private:
    static constexpr size_t kClass = size_t{1} << 16;
    struct Block {
        size_t size = 0;
        bool pinned = false;
        intptr_t delta = 0;  // device address - host address
        int node = -1;       // NUMA node of the thread that made it (its pages were faulted in there)
    };
    struct Key {
        int node;
        size_t cls;
        bool operator<(const Key& o) const { return node != o.node ? node < o.node : cls < o.cls; }
    };
    static int current_node()
    {
        unsigned cpu = 0, node = 0;
        return getcpu(&cpu, &node) == 0 ? static_cast<int>(node) : -1;
    }

    // free page-locked bytes kept for reuse (ELECT_EC_HOST_POOL_MB, default 4096)
    static size_t cap()
    {
        static const size_t c = [] {
            const char* e = std::getenv("ELECT_EC_HOST_POOL_MB");
            return (e ? static_cast<size_t>(std::max(0, std::atoi(e))) : size_t{4096}) << 20;
        }();
        return c;
    }

    mutable std::shared_mutex mu_;
    std::map<uintptr_t, Block> live_;
    std::map<Key, std::vector<void*>> free_;  // by (node, size class)
    std::map<void*, intptr_t> delta_;  // every page-locked block ever made (blocks are only ever reused)
    size_t free_bytes_ = 0;
};

// Bytes of input j the kernels may touch when they read the unit where it lies
// (zero-copy): a padded unit's content rounded up to the 16-byte segment, never
// past the unit.  The padded vector kernel loads the whole segment that holds a
// content end (rs_impl.hpp, gf_apply_x16<PAD>) and masks it: up to 15 bytes
// past lens[j], which on a caller pointer off 16-byte alignment can cross into
// memory that is neither registered nor in the pool.
size_t input_span(const HostOp& op, int j, size_t len)
{
    if (!op.lens) return len;
    return std::min(len, (op.lens[j] + 15) & ~size_t{15});
}

// Every byte the call's kernels may touch lies in page-locked pool buffers
// (inputs: input_span, so a zero-copy kernel reading a pool unit in place stays
// inside its block).
bool direct_op(const HostOp& op, size_t len)
{
    PinnedPool& pool = PinnedPool::get();
    if (!pool.any()) return false;
    for (int j = 0; j < op.cols; ++j) {
        const size_t n = op.lens ? op.lens[j] : len;
        if (n && !pool.pinned(op.in[j], input_span(op, j, len))) return false;
    }
    for (int r = 0; r < op.rows; ++r)
        if (!pool.pinned(op.out[r], len)) return false;
    return true;
}

// ---------------------------------------------------------------------------
// Page-locking callers' own (pageable) memory for one call: hipHostRegister,
// process-wide, through one registry.
//
// Round 4 ran batched callers' units registered per call and the GPU suite
// faulted (hipErrorIllegalAddress) in a later device-only test.  The cause,
// measured on the box (tools/tune/register_overlap_probe.cpp,
// profiles/r05/register_overlap.txt): the HIP runtime ACCEPTS a registration
// whose pages overlap a live one, in every arrangement (one range inside
// another, shifted, identical), and maps both at the same device address (the
// host address).  The first hipHostUnregister then removes the shared pages'
// mapping and bookkeeping while the other registration is still in use: after
// an identical range was registered twice, the second unregister returns
// hipErrorHostMemoryNotRegistered (the first took both down), and after
// shifted overlaps the runtime's object map is left corrupt, so that a later,
// unrelated unregister aborts the process ("Memobj map does not have ptr").
// Round 4 registered each call's page-ROUNDED ranges: ELECT's units (and the
// tests' numpy arrays) sit back to back on the heap, so a unit's first and last
// pages are shared with its neighbours, and concurrent callers registered
// overlapping ranges; a call finishing first unmapped pages another call's
// DMAs still read.  The same hazard sat in the zero-copy path below
// (host_path.cpp round 4: merged page-rounded ranges, released by base).
// Two more facts from the probe: a DMA whose host range spans two adjacent
// registrations is refused (hipErrorInvalidValue), and hipHostUnregister
// given an interior pointer aborts the process.
//
// So, with locks (hsa_amd_memory_lock; hipHostRegister is no longer used, see
// Registrar): (1) no two live locks share a page — a request that meets a live
// lock of another extent (or device) is refused here, before the runtime sees
// it; an identical request shares the live lock (refcounted); (2) every lock is
// released by the exact base it was made with, after the last transfer or
// kernel using it has completed (callers release after their batch's
// completion); (3) memory another party has registered (either end of the
// range, and for zero-copy calls either end of every unit, already known to the
// runtime) is never locked; (4) a failed unlock is counted (host_path_stats),
// never ignored silently.  The batched path locks only the pages lying wholly
// inside a unit (interior pages): those belong to that unit alone, so
// neighbours never meet, and the <= 2 partial pages at its ends travel through
// the arena.
// ---------------------------------------------------------------------------
std::atomic<uint64_t> g_unregister_failures{0};
// CPU time (ns, calling threads) spent registering, unregistering, and in the
// dispatchers' issue() (host_path_stats entries 8-10, for the A/B of this path).
std::atomic<uint64_t> g_register_cpu_ns{0}, g_unregister_cpu_ns{0}, g_issue_cpu_ns{0};
// Where a batched call's wall time goes (host_path_stats entries 11-17, ns summed over
// calls; 14 and 15 over batches, counted in entry 18): 0 entry -> units locked, 1 ->
// arena edges copied and the call counted filled, 2 -> its batch's issue starts, 3 the
// issue (dispatcher), 4 issue end -> the poller sees the batch done (device time and
// polling delay), 5 -> the caller awake, 6 -> the call returns (edges out, unlocks).
std::atomic<uint64_t> g_phase_ns[7];
std::atomic<uint64_t> g_batches{0};
thread_local int64_t t_phase_mark = 0;  // the calling thread's last phase boundary

int64_t now_ns()
{
    return std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now().time_since_epoch())
        .count();
}

// ELECT_EC_PHASE_DEBUG=<us>: report calls whose fill phase took longer (diagnostics)
}  // namespace

// Window weights equal, or (taper) 4 : ... : 4 : 2 : 1, so that the scatter left after the
// last gather is a small window's; boundaries on 64 KiB multiples, never an empty window.
int pipeline_windows(size_t len, int steps, bool taper, size_t* at)
{
    steps = std::max(1, steps);
    unsigned total = 0;
    for (int k = 0; k < steps; ++k) total += !taper || k + 2 < steps ? 4u : k + 2 == steps ? 2u : 1u;
    constexpr size_t kAlign = size_t{1} << 16;
    int n = 0;
    unsigned cum = 0;
    at[0] = 0;
    for (int k = 0; k < steps; ++k) {
        cum += !taper || k + 2 < steps ? 4u : k + 2 == steps ? 2u : 1u;
        size_t b = k + 1 == steps ? len : (len / total * cum + len % total * cum / total + kAlign / 2) / kAlign * kAlign;
        if (b > len) b = len;
        if (b > at[n]) at[++n] = b;
    }
    if (n == 0) at[n = 1] = len;  // (len 0: one empty window)
    return n;
}

namespace {

int64_t phase_debug()
{
    static const int64_t ns = [] {
        const char* e = std::getenv("ELECT_EC_PHASE_DEBUG");
        return e ? static_cast<int64_t>(std::atoi(e)) * 1000 : int64_t{0};
    }();
    return ns;
}

void add_phase(int i, int64_t from, int64_t to)
{
    if (from && to > from) g_phase_ns[i].fetch_add(static_cast<uint64_t>(to - from), std::memory_order_relaxed);
}

uint64_t thread_cpu_ns()
{
    timespec t{};
    clock_gettime(CLOCK_THREAD_CPUTIME_ID, &t);
    return static_cast<uint64_t>(t.tv_sec) * 1000000000ull + static_cast<uint64_t>(t.tv_nsec);
}

// The HSA agent of HIP device `dev`, for hsa_amd_memory_lock: the one GPU
// agent at the device's PCI domain:bus:device.function.  False when none or
// more than one matches (partitioned GPUs could share a location): the
// callers then take the staged path rather than lock for a wrong agent.
bool hsa_agent_of(int dev, hsa_agent_t* out)
{
    struct Found {
        uint32_t bdf = 0, domain = 0;
        int matches = 0;
        hsa_agent_t agent{};
    };
    static std::mutex mu;
    static std::map<int, std::pair<bool, hsa_agent_t>> cache;  // (found, agent), failures too
    std::lock_guard<std::mutex> lock(mu);
    auto it = cache.find(dev);
    if (it != cache.end()) {
        *out = it->second.second;
        return it->second.first;
    }
    static const bool init = hsa_init() == HSA_STATUS_SUCCESS;  // (reference counted: the HIP runtime holds one)
    if (!init) return false;
    char loc[64] = {};
    unsigned domain = 0, bus = 0, device = 0, function = 0;
    if (hipDeviceGetPCIBusId(loc, sizeof loc, dev) != hipSuccess ||
        std::sscanf(loc, "%x:%x:%x.%x", &domain, &bus, &device, &function) != 4) {
        (void)hipGetLastError();
        return false;
    }
    Found f;
    f.bdf = (bus << 8) | (device << 3) | function;
    f.domain = domain;
    hsa_iterate_agents(
        [](hsa_agent_t a, void* arg) -> hsa_status_t {
            auto* f = static_cast<Found*>(arg);
            hsa_device_type_t t{};
            uint32_t bdf = 0, domain = 0;
            if (hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t) != HSA_STATUS_SUCCESS || t != HSA_DEVICE_TYPE_GPU)
                return HSA_STATUS_SUCCESS;
            hsa_agent_get_info(a, static_cast<hsa_agent_info_t>(HSA_AMD_AGENT_INFO_BDFID), &bdf);
            hsa_agent_get_info(a, static_cast<hsa_agent_info_t>(HSA_AMD_AGENT_INFO_DOMAIN), &domain);
            if (bdf != f->bdf || domain != f->domain) return HSA_STATUS_SUCCESS;
            f->agent = a;
            ++f->matches;
            return HSA_STATUS_SUCCESS;
        },
        &f);
    cache[dev] = {f.matches == 1, f.agent};
    if (f.matches != 1) return false;
    *out = f.agent;
    return true;
}

class Registrar {
public:
    // Locks are hsa_amd_memory_lock for the calling device's agent: the batches'
    // kernels (and zero-copy calls) read and write the pages through the returned
    // address, and hsa_amd_memory_unlock does not wait for the device
    // (profiles/r05/register_overlap.txt part 4).  hipHostRegister is not used:
    // its hipHostUnregister waits for every queued operation on the device, other
    // streams included (part 3: 7.1 ms behind another stream's 7.1 ms of copies;
    // 485 core-ms per GiB at 64 callers, hostpath_register_ab.txt A), and one
    // locking mechanism keeps the two runtime layers from mapping one page twice.
    static Registrar& get()
    {
        static Registrar* r = new Registrar();  // never destroyed: locks may be in use at exit
        return *r;
    }

    // A reference on a lock of exactly [lo, hi) (page aligned, lo < hi) for
    // device dev: the identical live one, or a new one.  False (nothing held)
    // when [lo, hi) shares a page with a lock of another extent or device, or
    // with memory the HIP runtime already knows at either end, or when the
    // runtime refuses.  *dev_lo: the device address of lo.
    bool acquire(uintptr_t lo, uintptr_t hi, int dev, uintptr_t* dev_lo)
    {
        std::unique_lock<std::mutex> lock(mu_);
        for (;;) {
            Entry* same = nullptr;
            auto next = live_.upper_bound(lo);  // first lock starting after lo
            if (next != live_.end() && next->first < hi) return false;
            if (next != live_.begin()) {
                auto prev = std::prev(next);
                if (prev->second.end > lo) {
                    // shared only when made for the same device: a lock maps the pages for one agent
                    if (prev->first != lo || prev->second.end != hi || prev->second.dev != dev) return false;
                    same = &prev->second;
                }
            }
            if (!same) break;
            if (same->state == Entry::kLive) {
                ++same->refs;
                *dev_lo = same->dev_lo;
                return true;
            }
            if (same->state == Entry::kRetiring) return false;
            changed_.wait(lock);  // its maker is locking it: wait for the outcome
        }
        live_.emplace(lo, Entry{hi, 0, Entry::kPending, 0, dev});
        lock.unlock();
        const uint64_t t0 = thread_cpu_ns();
        void* p = reinterpret_cast<void*>(lo);
        hsa_agent_t agent{};
        void* ap = nullptr;
        const bool ok = hsa_agent_of(dev, &agent) && !known(lo) && !known(hi - 1) &&
                        hsa_amd_memory_lock(p, hi - lo, &agent, 1, &ap) == HSA_STATUS_SUCCESS;
        g_register_cpu_ns.fetch_add(thread_cpu_ns() - t0);
        lock.lock();
        auto it = live_.find(lo);
        if (ok) {
            it->second.state = Entry::kLive;
            it->second.refs = 1;
            it->second.dev_lo = reinterpret_cast<uintptr_t>(ap);
            *dev_lo = it->second.dev_lo;
        } else {
            live_.erase(it);
        }
        changed_.notify_all();
        return ok;
    }

    // Drops a reference taken by acquire(lo, ...); the last one unlocks (by lo,
    // the base it was locked with).  Only after every transfer and kernel
    // touching the pages has completed.
    void release(uintptr_t lo)
    {
        std::unique_lock<std::mutex> lock(mu_);
        auto it = live_.find(lo);
        if (it == live_.end() || it->second.state != Entry::kLive) return;
        if (--it->second.refs > 0) return;
        it->second.state = Entry::kRetiring;  // stays in the map (refusing overlaps) until it is gone
        lock.unlock();
        const uint64_t t0 = thread_cpu_ns();
        if (hsa_amd_memory_unlock(reinterpret_cast<void*>(lo)) != HSA_STATUS_SUCCESS) g_unregister_failures.fetch_add(1);
        g_unregister_cpu_ns.fetch_add(thread_cpu_ns() - t0);
        lock.lock();
        live_.erase(lo);
        changed_.notify_all();
    }

private:
    struct Entry {
        uintptr_t end;
        int refs;
        enum State { kPending, kLive, kRetiring } state;
        uintptr_t dev_lo;
        int dev;
    };

    // The HIP runtime already knows this address (registered or allocated by anyone).
    static bool known(uintptr_t a)
    {
        hipPointerAttribute_t attr{};
        const hipError_t e = hipPointerGetAttributes(&attr, reinterpret_cast<void*>(a));
        (void)hipGetLastError();
        return e != hipSuccess || attr.type != hipMemoryTypeUnregistered;
    }

    std::mutex mu_;
    std::condition_variable changed_;
    std::map<uintptr_t, Entry> live_;  // disjoint page ranges, keyed by base
};

// Callers locking or unlocking their units at once (ELECT_EC_REGISTER_SLOTS,
// default 8): hsa_amd_memory_lock / unlock contend in the driver (round 5,
// lock + unlock of 4.4 MB units: 4.7 core-ms per GiB from 8 threads, 21.7 from
// 64, profiles/r05/register_overlap.txt part 4), so the rest wait their turn.
class RegisterSlots {
public:
    static RegisterSlots& get()
    {
        static RegisterSlots s;
        return s;
    }
    void take()
    {
        std::unique_lock<std::mutex> lock(mu_);
        cv_.wait(lock, [&] { return free_ > 0; });
        --free_;
    }
    bool try_take()
    {
        std::lock_guard<std::mutex> lock(mu_);
        if (free_ <= 0) return false;
        --free_;
        return true;
    }
    // ELECT_EC_REGISTER_WAIT=0: a caller finding every slot busy is staged instead of waiting (A/B)
    static bool wait()
    {
        static const bool w = [] {
            const char* e = std::getenv("ELECT_EC_REGISTER_WAIT");
            return !(e && std::atoi(e) == 0);
        }();
        return w;
    }
    void give()
    {
        {
            std::lock_guard<std::mutex> lock(mu_);
            ++free_;
        }
        cv_.notify_one();
    }

private:
    RegisterSlots()
    {
        const char* e = std::getenv("ELECT_EC_REGISTER_SLOTS");
        free_ = e ? std::max(1, std::atoi(e)) : 8;
    }
    std::mutex mu_;
    std::condition_variable cv_;
    int free_ = 8;
};

// How a direct call's units move (Batcher, direct batches).  Unit bytes
// [lo, hi) are read (written) by the batch's gather (scatter) kernel straight
// from (to) the caller's memory at device address *_dev (the address of byte
// lo); the rest of the unit ([0, lo) and [hi, n)) goes through the arena,
// copied by the caller.  Pool units: all of it direct.  Locked units: their
// interior pages.
struct DirectPlan {
    bool direct = false;
    size_t in_lo[kern::kMaxCols] = {}, in_hi[kern::kMaxCols] = {};
    size_t out_lo[kern::kMaxRows] = {}, out_hi[kern::kMaxRows] = {};
    uintptr_t in_dev[kern::kMaxCols] = {}, out_dev[kern::kMaxRows] = {};
    uintptr_t held[kern::kMaxCols + kern::kMaxRows] = {};  // locks to release
    int nheld = 0;
};

// Per-call page locking of batched callers' pageable units (ELECT_EC_REGISTER:
// 0 off, 1 on, the default; units of at least kMinBytes): each unit's interior
// pages are locked with hsa_amd_memory_lock (Registrar), the batch's
// kernels move them over PCIe, and they are unlocked when the call's batch is
// done.  No staging copies of the interior, no DMA engine, no device wait.
struct RegisterPath {
    static constexpr size_t kMinBytes = size_t{1} << 20;
    static constexpr uintptr_t kPage = 4096;
    static constexpr uintptr_t kMinInterior = kPage * 16;  // shorter: all of the unit through the arena

    static int mode()
    {
        static const int m = [] {
            const char* e = std::getenv("ELECT_EC_REGISTER");
            return e ? std::atoi(e) : 1;
        }();
        return m;
    }

    // Interior pages of [p, p + n): [lo, hi) page aligned (lo == hi: none).
    static void interior(const void* p, size_t n, uintptr_t& lo, uintptr_t& hi)
    {
        const uintptr_t a = reinterpret_cast<uintptr_t>(p);
        lo = (a + kPage - 1) & ~(kPage - 1);
        hi = (a + n) & ~(kPage - 1);
        if (hi < lo) hi = lo;
    }

    // Locks every unit's interior pages (one lock per unit; units with equal
    // interiors share it).  False (nothing held): take the staged path.
    static bool plan(const HostOp& op, size_t len, int dev, DirectPlan& dp)
    {
        if (mode() != 1 || len < kMinBytes) return false;
        RegisterSlots& slots = RegisterSlots::get();
        if (RegisterSlots::wait())
            slots.take();
        else if (!slots.try_take())
            return false;
        Registrar& reg = Registrar::get();
        bool ok = true;
        PinnedPool& pool = PinnedPool::get();
        auto add = [&](const void* p, size_t n, size_t& lo_off, size_t& hi_off, uintptr_t& dev_addr) {
            lo_off = hi_off = 0;
            if (!ok || !p || !n) return;
            if (pool.pinned(p, n)) {  // a pool unit among pageable ones: all of it in place, no lock
                hi_off = n;
                dev_addr = pool.device_addr(p);
                return;
            }
            uintptr_t lo = 0, hi = 0;
            interior(p, n, lo, hi);
            if (hi - lo < kMinInterior) return;
            if (!reg.acquire(lo, hi, dev, &dev_addr)) {
                ok = false;
                return;
            }
            dp.held[dp.nheld++] = lo;
            const uintptr_t a = reinterpret_cast<uintptr_t>(p);
            lo_off = lo - a;
            hi_off = hi - a;
            dev_addr -= lo_off;  // the unit's base, at its device address (only [lo, hi) is read there)
        };
        for (int j = 0; j < op.cols; ++j)
            add(op.in[j], op.lens ? op.lens[j] : len, dp.in_lo[j], dp.in_hi[j], dp.in_dev[j]);
        for (int r = 0; r < op.rows; ++r) add(op.out[r], len, dp.out_lo[r], dp.out_hi[r], dp.out_dev[r]);
        if (!ok) {
            for (int i = 0; i < dp.nheld; ++i) reg.release(dp.held[i]);
            dp.nheld = 0;
        }
        slots.give();
        dp.direct = ok;
        return ok;
    }

    static void release(DirectPlan& dp)
    {
        if (!dp.nheld) return;
        RegisterSlots& slots = RegisterSlots::get();
        slots.take();
        for (int i = 0; i < dp.nheld; ++i) Registrar::get().release(dp.held[i]);
        slots.give();
        dp.nheld = 0;
    }
};

// Copy fan-out for lone callers.  One thread's staging copies (~20 GB/s) bound a
// caller that has the device to itself: a 4.4 MB RS(6,4) stripe moves 26 MB
// through them against 0.5 ms of DMA.  Such a caller spreads its copies over a
// few helper threads (ELECT_EC_COPY_THREADS, default 8; 0 disables); with many
// callers in flight every caller copies its own, as the cores are busy anyway.
struct CopyJob {
    uint8_t* dst;
    const uint8_t* src;
    size_t n;
};

// Appends dst <- src[0, n) as pieces of at most 1 MiB.
void add_copy(std::vector<CopyJob>& jobs, uint8_t* dst, const uint8_t* src, size_t n)
{
    constexpr size_t kPiece = size_t{1} << 20;
    for (size_t o = 0; o < n; o += kPiece) jobs.push_back(CopyJob{dst + o, src + o, std::min(kPiece, n - o)});
}

class CopyPool {
public:
    static CopyPool* get()
    {
        static CopyPool* pool = [] {
            const char* e = std::getenv("ELECT_EC_COPY_THREADS");
            const int n = e ? std::min(16, std::max(0, std::atoi(e))) : 8;
            return n > 0 ? new (std::nothrow) CopyPool(n) : nullptr;  // never destroyed: helpers live until exit
        }();
        return pool;
    }

    // Runs the jobs on this thread and the helpers, and returns once all are
    // done and their streamed stores fenced.  False (nothing copied) when another
    // caller holds the pool.
    bool run(const std::vector<CopyJob>& jobs)
    {
        bool idle = false;
        if (!busy_.compare_exchange_strong(idle, true)) return false;
        {
            std::lock_guard<std::mutex> lock(mu_);
            jobs_ = jobs.data();
            njobs_ = jobs.size();
            next_.store(0);
            ++gen_;
        }
        cv_go_.notify_all();
        drain(jobs.data(), jobs.size());
        _mm_sfence();
        {
            // every job is claimed; wait for the helpers that joined to finish theirs
            std::unique_lock<std::mutex> lock(mu_);
            cv_done_.wait(lock, [&] { return working_ == 0; });
            jobs_ = nullptr;  // helpers waking from here on find nothing to join
        }
        busy_.store(false);
        return true;
    }

private:
    explicit CopyPool(int n)
    {
        try {
            for (int i = 0; i < n; ++i) std::thread(&CopyPool::helper, this).detach();
        } catch (...) {  // fewer helpers (or none: callers then drain their jobs alone)
        }
    }

    void drain(const CopyJob* jobs, size_t n)
    {
        for (size_t i = next_.fetch_add(1); i < n; i = next_.fetch_add(1)) stream_copy(jobs[i].dst, jobs[i].src, jobs[i].n);
    }

    void helper()
    {
        pthread_setname_np(pthread_self(), "ec-copy");
        uint64_t seen = 0;
        std::unique_lock<std::mutex> lock(mu_);
        for (;;) {
            cv_go_.wait(lock, [&] { return gen_ != seen; });
            seen = gen_;
            if (!jobs_) continue;  // that job is over
            const CopyJob* jobs = jobs_;
            const size_t n = njobs_;
            ++working_;
            lock.unlock();
            drain(jobs, n);
            _mm_sfence();  // this thread's streamed stores, before the caller hands the data on
            lock.lock();
            if (--working_ == 0) cv_done_.notify_one();
        }
    }

    std::atomic<bool> busy_{false};
    std::mutex mu_;
    std::condition_variable cv_go_, cv_done_;
    const CopyJob* jobs_ = nullptr;  // the current job, under mu_
    size_t njobs_ = 0;
    uint64_t gen_ = 0;
    int working_ = 0;  // helpers inside the current job
    std::atomic<size_t> next_{0};
};

// Runs the copies through the pool when the caller is (nearly) alone and the
// copies are large enough to split, else on this thread.
void run_copies(const std::vector<CopyJob>& jobs, bool lone)
{
    size_t bytes = 0;
    for (const CopyJob& j : jobs) bytes += j.n;
    CopyPool* pool = lone && bytes >= (size_t{2} << 20) && jobs.size() > 1 ? CopyPool::get() : nullptr;
    if (pool && pool->run(jobs)) return;
    for (const CopyJob& j : jobs) stream_copy(j.dst, j.src, j.n);
    _mm_sfence();  // the streamed stores are visible before the data is handed on
}

// Waits for ev without spinning a core: this HIP runtime's own waits spin for as
// long as the work they wait for runs (Batcher::poller); hipEventQuery with
// sleeps from 2 up to 50 us costs ~2 % of a core instead.
hipError_t wait_sleeping(hipEvent_t ev)
{
    for (unsigned us = 2;; us = std::min(us * 2, 50u)) {
        const hipError_t e = hipEventQuery(ev);
        if (e != hipErrorNotReady) return e;
        std::this_thread::sleep_for(std::chrono::microseconds(us));
    }
}

// ---------------------------------------------------------------------------
// Host-memory path: per-thread, per-device staging engine.
// Input chunks are copied into pinned buffers, sent H2D, coded, returned D2H
// and copied out, with two slots (streams) so chunk c+1's transfers overlap
// chunk c's kernel and host copies.
// ---------------------------------------------------------------------------
class HostEngine {
public:
    static constexpr size_t kChunk = size_t{1} << 20;  // bytes per shard per pipeline step
    static constexpr int kSlots = 2;

    explicit HostEngine(int dev) : dev_(dev) {}
    ~HostEngine()
    {
        for (int s = 0; s < kSlots; ++s) {
            if (stream_[s]) (void)hipStreamDestroy(stream_[s]);
            if (ev_[s]) (void)hipEventDestroy(ev_[s]);
            if (pin_in_[s]) (void)hipHostFree(pin_in_[s]);
            if (pin_out_[s]) (void)hipHostFree(pin_out_[s]);
            if (d_in_[s]) (void)hipFree(d_in_[s]);
            if (d_out_[s]) (void)hipFree(d_out_[s]);
            if (d_scratch_[s]) (void)hipFree(d_scratch_[s]);
        }
        if (d_hash_) (void)hipFree(d_hash_);
    }

    int run(const HostOp& op, size_t len)
    {
        const size_t step = std::min(len, kChunk);
        const size_t pitch = (step + 255) & ~size_t{255};
        int rc = reserve(static_cast<size_t>(op.cols) * pitch, static_cast<size_t>(op.rows) * pitch);
        if (rc != ELECT_EC_OK) return rc;
        const size_t nchunks = (len + step - 1) / step;
        if (op.hashes) {  // every chunk's kernel adds into d_hash_; start from 31^len
            hipError_t e = hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(d_hash_),
                                             static_cast<int>(kern::pow31(len)), op.rows, stream_[0]);
            if (e == hipSuccess) e = hipStreamSynchronize(stream_[0]);
            if (e != hipSuccess) return map_hip(e);
        }
        size_t pending[kSlots] = {};
        bool busy[kSlots] = {};
        for (size_t c = 0; c < nchunks + kSlots; ++c) {
            const int s = static_cast<int>(c % kSlots);
            if (busy[s]) {  // retire the chunk that used this slot
                const hipError_t e = wait_sleeping(ev_[s]);
                if (e != hipSuccess) return map_hip(e);
                const size_t o = pending[s] * step;
                const size_t n = std::min(step, len - o);
                for (int r = 0; r < op.rows; ++r) stream_copy(op.out[r] + o, pin_out_[s] + r * pitch, n);
                _mm_sfence();
                busy[s] = false;
            }
            if (c >= nchunks) continue;
            const size_t o = c * step;
            const size_t n = std::min(step, len - o);
            hipError_t e = hipSuccess;
            uint32_t valid[kern::kMaxCols];
            if (op.lens) {  // copy and send only each column's valid bytes
                for (int j = 0; j < op.cols && e == hipSuccess; ++j) {
                    const size_t v = op.lens[j] > o ? std::min(n, op.lens[j] - o) : 0;
                    valid[j] = static_cast<uint32_t>(v);
                    if (v == 0) continue;
                    stream_copy(pin_in_[s] + j * pitch, op.in[j] + o, v);
                    _mm_sfence();
                    e = hipMemcpyAsync(d_in_[s] + j * pitch, pin_in_[s] + j * pitch, v, hipMemcpyHostToDevice,
                                       stream_[s]);
                }
            } else {
                for (int j = 0; j < op.cols; ++j) stream_copy(pin_in_[s] + j * pitch, op.in[j] + o, n);
                _mm_sfence();
                e = hipMemcpyAsync(d_in_[s], pin_in_[s], op.cols * pitch, hipMemcpyHostToDevice, stream_[s]);
            }
            if (e == hipSuccess) e = launch(op, s, pitch, n, op.lens ? valid : nullptr, o);
            if (e == hipSuccess)
                e = hipMemcpyAsync(pin_out_[s], d_out_[s], op.rows * pitch, hipMemcpyDeviceToHost, stream_[s]);
            if (e == hipSuccess) e = hipEventRecord(ev_[s], stream_[s]);
            if (e != hipSuccess) {
                (void)hipStreamSynchronize(stream_[0]);
                (void)hipStreamSynchronize(stream_[1]);
                return map_hip(e);
            }
            pending[s] = c;
            busy[s] = true;
        }
        if (op.hashes) {
            const hipError_t e = hipMemcpy(op.hashes, d_hash_, op.rows * sizeof(int32_t), hipMemcpyDeviceToHost);
            if (e != hipSuccess) return map_hip(e);
        }
        return ELECT_EC_OK;
    }

private:
    hipError_t launch(const HostOp& op, int s, size_t pitch, size_t n, const uint32_t* valid, size_t offset)
    {
        ApplyParams p;
        p.len = n;
        p.stripes = 1;
        p.cols = op.cols;
        p.rows = op.rows;
        for (int j = 0; j < op.cols; ++j) p.src[j] = col(d_in_[s], pitch, j * pitch);
        for (int r = 0; r < op.rows; ++r) p.dst[r] = col(d_out_[s], pitch, r * pitch);
        std::memcpy(p.coef, op.coef, sizeof(p.coef));
        if (valid) {
            p.padded = true;
            for (int j = 0; j < op.cols; ++j) p.clen[j] = valid[j];
        }
        if (op.hashes) {
            p.hashes = d_hash_;
            p.hash_stride = static_cast<uint32_t>(op.rows);
            p.hash_base = offset;
            p.hash_scratch = d_scratch_[s];  // per slot: the two slots' launches overlap
            p.hash_scratch_words = kScratchWords;
        }
        return kern::launch_apply(p, stream_[s]);
    }

    int reserve(size_t in_bytes, size_t out_bytes)
    {
        if (!stream_[0]) {
            for (int s = 0; s < kSlots; ++s) {
                hipError_t e = hipStreamCreateWithFlags(&stream_[s], hipStreamNonBlocking);
                if (e == hipSuccess) e = hipEventCreateWithFlags(&ev_[s], hipEventDisableTiming);
                if (e != hipSuccess) return map_hip(e);
            }
            hipError_t e = hipMalloc(reinterpret_cast<void**>(&d_hash_), kern::kMaxRows * sizeof(int32_t));
            for (int s = 0; s < kSlots && e == hipSuccess; ++s)
                e = hipMalloc(reinterpret_cast<void**>(&d_scratch_[s]), kScratchWords * sizeof(uint32_t));
            if (e != hipSuccess) return map_hip(e);
        }
        if (in_bytes > cap_in_) {
            for (int s = 0; s < kSlots; ++s) {
                if (pin_in_[s]) (void)hipHostFree(pin_in_[s]);
                if (d_in_[s]) (void)hipFree(d_in_[s]);
                pin_in_[s] = nullptr;
                d_in_[s] = nullptr;
                hipError_t e = hipHostMalloc(reinterpret_cast<void**>(&pin_in_[s]), in_bytes, hipHostMallocDefault);
                if (e == hipSuccess) e = hipMalloc(reinterpret_cast<void**>(&d_in_[s]), in_bytes);
                if (e != hipSuccess) {
                    cap_in_ = 0;
                    return map_hip(e);
                }
            }
            cap_in_ = in_bytes;
        }
        if (out_bytes > cap_out_) {
            for (int s = 0; s < kSlots; ++s) {
                if (pin_out_[s]) (void)hipHostFree(pin_out_[s]);
                if (d_out_[s]) (void)hipFree(d_out_[s]);
                pin_out_[s] = nullptr;
                d_out_[s] = nullptr;
                hipError_t e = hipHostMalloc(reinterpret_cast<void**>(&pin_out_[s]), out_bytes, hipHostMallocDefault);
                if (e == hipSuccess) e = hipMalloc(reinterpret_cast<void**>(&d_out_[s]), out_bytes);
                if (e != hipSuccess) {
                    cap_out_ = 0;
                    return map_hip(e);
                }
            }
            cap_out_ = out_bytes;
        }
        return ELECT_EC_OK;
    }

    [[maybe_unused]] int dev_;
    hipStream_t stream_[kSlots] = {};
    hipEvent_t ev_[kSlots] = {};  // behind each slot's D2H (wait_sleeping)
    uint8_t* pin_in_[kSlots] = {};
    uint8_t* pin_out_[kSlots] = {};
    uint8_t* d_in_[kSlots] = {};
    uint8_t* d_out_[kSlots] = {};
    size_t cap_in_ = 0;
    size_t cap_out_ = 0;
    int32_t* d_hash_ = nullptr;
    // Hash partials of one slot's launch.  Engine-owned rather than taken from the
    // stream-ordered pool per launch: with many caller threads, each on its own
    // streams, pool-allocated partials were corrupted (host_stress).
    static constexpr size_t kScratchWords = kern::hash_scratch_need(kChunk / 16);
    uint32_t* d_scratch_[kSlots] = {};
};

constexpr int kMaxDevices = 64;
constexpr int kMaxNumaNodes = 64;
thread_local std::unique_ptr<HostEngine> t_engines[kMaxDevices];
thread_local std::vector<CopyJob> t_jobs;  // a caller's staging copies (Batcher::submit)

// Device policy of the host-memory path (elect_ec_set_host_devices).
struct DevicePolicy {
    std::mutex mu;
    bool env_read = false;
    std::vector<int> devices;  // empty: each thread's current device
    std::vector<int> nodes;    // NUMA node of each listed device (-1: unknown)
    std::vector<unsigned> load;  // calling threads given each listed device (this generation)
    std::atomic<unsigned> generation{1};
};

DevicePolicy& policy()
{
    static DevicePolicy p;
    return p;
}

// ELECT_EC_NUMA (default 1): a calling thread gets a device on its own NUMA node
// when the list holds one (numa_pick); 0: plain round robin over the list.
bool numa_policy()
{
    static const bool on = [] {
        const char* e = std::getenv("ELECT_EC_NUMA");
        return !(e && std::atoi(e) == 0);
    }();
    return on;
}

}  // namespace

// NUMA node of HIP device `dev` from sysfs (its PCI function's numa_node), -1
// when unknown.  The box this was measured on has 2 nodes, 4 GPUs on each
// (/sys/class/drm/card*/device/numa_node, profiles/r06/numa_facts.txt).
int device_numa_node(int dev)
{
    char loc[64] = {};
    if (hipDeviceGetPCIBusId(loc, sizeof loc, dev) != hipSuccess) {
        (void)hipGetLastError();
        return -1;
    }
    unsigned domain = 0, bus = 0, device = 0, function = 0;
    if (std::sscanf(loc, "%x:%x:%x.%x", &domain, &bus, &device, &function) != 4) return -1;
    char path[128];
    std::snprintf(path, sizeof path, "/sys/bus/pci/devices/%04x:%02x:%02x.%x/numa_node", domain, bus, device, function);
    FILE* f = std::fopen(path, "r");
    if (!f) return -1;
    int node = -1;
    if (std::fscanf(f, "%d", &node) != 1) node = -1;
    std::fclose(f);
    return node >= 0 && node < kMaxNumaNodes ? node : -1;
}

namespace {

// NUMA node the calling thread runs on now (-1: unknown).
int thread_numa_node()
{
    unsigned cpu = 0, node = 0;
    if (getcpu(&cpu, &node) != 0) return -1;
    return static_cast<int>(node) < kMaxNumaNodes ? static_cast<int>(node) : -1;
}

}  // namespace

// The device a thread on NUMA node `thread_node` gets from `devices` (their
// nodes in `nodes`, the threads each already has in `load`): a least loaded
// device, one on the thread's node when one of those is among the least loaded
// (lowest index on ties).  So threads stay on their own socket while the
// sockets' threads are about even, and unbound threads that all happen to run
// on one socket at their first call still spread over every GPU: no device is
// ever more than one thread ahead of another.
// ELECT's one JVM per storage node runs concurrent_ec = 64 coding threads
// (conf/elect.yaml:598) spread over every GPU; each thread's units are
// allocated and filled by that thread (ECMessageVerbHandler.java:298-314), so
// with first-touch placement they lie on its node, and a GPU on the same node
// reads them without crossing the socket link (round 5's CPU baseline on one
// box: 90.6 GiB/s from node 0 against 75.2 from node 1, BENCH_r05 cpu_baseline).
int numa_pick(const int* devices, const int* nodes, int ndev, int thread_node, unsigned* load)
{
    int any = 0, local = -1;
    for (int i = 0; i < ndev; ++i) {
        if (load[i] < load[any]) any = i;
        if (thread_node >= 0 && nodes[i] == thread_node && (local < 0 || load[i] < load[local])) local = i;
    }
    const int pick = local >= 0 && load[local] == load[any] ? local : any;
    ++load[pick];
    return devices[pick];
}

namespace {

int parse_device_env(int ndev, std::vector<int>& out)
{
    const char* env = std::getenv("ELECT_EC_DEVICES");
    out.clear();
    if (!env || !*env) return ELECT_EC_OK;
    const std::string v(env);
    if (v == "all") {
        for (int d = 0; d < ndev; ++d) out.push_back(d);
        return ELECT_EC_OK;
    }
    size_t i = 0;
    while (i < v.size()) {
        size_t j = v.find(',', i);
        if (j == std::string::npos) j = v.size();
        const int d = std::atoi(v.substr(i, j - i).c_str());
        if (d < 0 || d >= ndev) return ELECT_EC_EINVAL;
        out.push_back(d);
        i = j + 1;
    }
    return ELECT_EC_OK;
}

// (the list's NUMA nodes, under p.mu; -1 each when the policy is off)
void read_nodes(DevicePolicy& p)
{
    p.nodes.assign(p.devices.size(), -1);
    if (numa_policy())
        for (size_t i = 0; i < p.devices.size(); ++i) p.nodes[i] = device_numa_node(p.devices[i]);
    p.load.assign(p.devices.size(), 0);
}

thread_local int t_device = -1;
thread_local unsigned t_generation = 0;

// The device this thread's host-memory calls run on.
int host_device(int ndev, int* dev)
{
    DevicePolicy& p = policy();
    {
        std::lock_guard<std::mutex> lock(p.mu);
        if (!p.env_read) {
            p.env_read = true;
            if (p.devices.empty() && parse_device_env(ndev, p.devices) != ELECT_EC_OK) p.devices.clear();
            read_nodes(p);
        }
        if (p.devices.empty()) {
            const hipError_t e = hipGetDevice(dev);
            return map_hip(e);
        }
        if (t_device < 0 || t_generation != p.generation.load()) {
            t_device = numa_pick(p.devices.data(), p.nodes.data(), static_cast<int>(p.devices.size()),
                                 numa_policy() ? thread_numa_node() : -1, p.load.data());
            t_generation = p.generation.load();
        }
    }
    *dev = t_device;
    return ELECT_EC_OK;
}

// ---------------------------------------------------------------------------
// Cross-thread batching.  ELECT makes up to concurrent_ec
// (64, conf/elect.yaml:598) synchronous one-stripe calls at once.  With
// batching on, concurrent calls of the same shape (k, m, len, coefficients,
// padded or not, hashed or not) share a pinned arena: every caller copies its
// own inputs in (in parallel; only content bytes when padded), one dispatcher
// thread per device issues ONE H2D, ONE launch over all the stripes
// ([slot][cols][pitch] layout) and ONE D2H, then each caller copies its outputs
// (and parity hashes) out.  Encodes, decodes and parity updates (as products)
// all batch.  Two arenas alternate, so one fills while the other is in flight.
//
// Units longer than 64 KiB are stored in the arena as 64 KiB tiles,
// [slot][T][cols][64 KiB] with T = ceil(len / 64 KiB), and coded through the
// tiled launch (kern::ApplyParams::tiles): every unit is then 64 KiB back to
// back, the layout HBM streams best, whatever ELECT's codeLength
// (4,404,020 B -> 68 tiles).  Callers copy their units tile by tile; the pad
// past len in each unit's last tile is never read (the tiled launch always
// runs the padded kernels, content = len or the caller's lengths).
// ---------------------------------------------------------------------------
struct BatchConfig {
    std::atomic<int> enabled{-1};  // -1: read ELECT_EC_BATCH on first use
    std::atomic<unsigned> window_us{0};
    std::atomic<size_t> arena_bytes{size_t{256} << 20};
    std::atomic<size_t> tile{size_t{1} << 16};  // ELECT_EC_BATCH_TILE_KB (0: untiled arena)
    // ELECT_EC_BATCH_SLABS: arenas per device, 2..4.  Three let one batch fill while
    // two are in flight (H2D + kernel, D2H + callers copying out): 64 callers on
    // 4.4 MB stripes 37-44.5 -> 46-50 GiB/s against two (profiles/r02_hostslabs.txt).
    std::atomic<int> slabs{3};
};

BatchConfig& batch_config()
{
    static BatchConfig c;
    if (c.enabled.load() < 0) {
        const char* e = std::getenv("ELECT_EC_BATCH");
        const char* w = std::getenv("ELECT_EC_BATCH_WINDOW_US");
        const char* a = std::getenv("ELECT_EC_BATCH_ARENA_MB");
        const char* t = std::getenv("ELECT_EC_BATCH_TILE_KB");
        const char* n = std::getenv("ELECT_EC_BATCH_SLABS");
        if (n) c.slabs = std::min(4, std::max(2, std::atoi(n)));
        if (w) c.window_us = static_cast<unsigned>(std::atoi(w));
        if (a && std::atoll(a) > 0) c.arena_bytes = static_cast<size_t>(std::atoll(a)) << 20;
        if (t && std::atoi(t) >= 0) c.tile = static_cast<size_t>(std::atoi(t)) << 10;
        int expect = -1;
        c.enabled.compare_exchange_strong(expect, (!e || std::atoi(e) > 0) ? 1 : 0);  // on unless ELECT_EC_BATCH=0
    }
    return c;
}

class Batcher {
public:
    static constexpr int kFallback = 1000;  // request does not fit (or no arena): run it directly
    static constexpr int kMaxSlabs = 4;  // arenas per device (ELECT_EC_BATCH_SLABS, default 3)
    static constexpr int kMaxSteps = 8;  // pipeline steps of a direct batch (ELECT_EC_PIPELINE_STEPS)
    // Per-slot content lengths (padded ops) and parity hashes (hashed ops) of a
    // batch: entries per arena, which caps such a batch's stripes.
    static constexpr size_t kMetaEntries = size_t{1} << 16;
    // Slots of a direct batch (each slot's unit pointers are kept in the slab).
    static constexpr size_t kMaxDirectSlots = 1024;
    // A caller fans its copies out (CopyPool) while at most this many callers are
    // in flight (ELECT_EC_COPY_FANOUT_CALLERS, default 2).
    static int lone_callers()
    {
        static const int n = [] {
            const char* e = std::getenv("ELECT_EC_COPY_FANOUT_CALLERS");
            return e ? std::max(0, std::atoi(e)) : 2;
        }();
        return n;
    }

    explicit Batcher(int dev) : dev_(dev) {}

    // dp (a direct call, dp->direct): its units move by the batch's gather /
    // scatter kernels between the caller's page-locked memory (pool buffers, or
    // units locked for the call) and the device, with no staging copies, in
    // batches of direct calls only (pipelined in steps, issue_direct);
    // bytes outside a unit's [lo, hi) (a registered unit's partial end pages)
    // go through the arena, copied by this caller.  nullptr: staged.
    int submit(const HostOp& op, size_t len, const DirectPlan* dp)
    {
        const bool direct = dp && dp->direct;
        struct InFlight {  // callers inside submit(), for the copy fan-out policy
            std::atomic<int>& n;
            explicit InFlight(std::atomic<int>& c) : n(c) { n.fetch_add(1); }
            ~InFlight() { n.fetch_sub(1); }
        } in_flight(callers_);
        // untiled: one unit per column at a 256-byte pitch; tiled: T tiles of 64 KiB
        // (direct batches are untiled: the gather pieces land at unit offsets)
        const size_t tile = direct ? 0 : batch_config().tile.load();
        // (tiled launches ride on the padded vector kernels: a wider product, the
        // update of an m >= 9 code, stays untiled rather than fail its whole batch)
        const bool tileable = op.cols <= kern::kMaxPadCols;
        const size_t tiles = tileable && tile && tile % 16 == 0 && len > tile ? (len + tile - 1) / tile : 1;
        const size_t pitch = tiles > 1 ? tile : (len + 255) & ~size_t{255};
        // the copy lists' room first: past the reservation below nothing may throw
        // (a slot reserved and never filled would stall its batch)
        std::vector<CopyJob>& jobs = t_jobs;
        jobs.clear();
        jobs.reserve(static_cast<size_t>(std::max(op.cols, op.rows)) * (tiles + (len >> 20) + 1));
        const int64_t t_sub0 = now_ns();
        std::unique_lock<std::mutex> lock(mu_);
        const int64_t t_sub1 = now_ns();
        if (init_failed_) return kFallback;
        if (!started_) {  // arenas, streams and events once, before anything is in flight
            if (init(batch_config().arena_bytes.load()) != ELECT_EC_OK) {
                release();  // whatever the failed attempt got; callers use the per-thread engine
                (void)hipGetLastError();
                init_failed_ = true;
                return kFallback;
            }
            try {
                std::thread(&Batcher::worker, this).detach();  // lives as long as the process
                std::thread(&Batcher::poller, this).detach();
            } catch (...) {  // no dispatcher: the per-thread engine serves every call
                release();
                init_failed_ = true;
                return kFallback;
            }
            started_ = true;
        }
        if (static_cast<size_t>(op.cols) * pitch * tiles > arena_ || static_cast<size_t>(op.rows) * pitch * tiles > arena_)
            return kFallback;
        Slab* slab = nullptr;
        for (;;) {
            for (Slab& s : active())
                if (s.state == Slab::kOpen && s.matches(op, len, direct) && s.reserved < s.capacity) slab = &s;
            if (!slab) {
                for (Slab& s : active())  // a different shape or a full arena closes the open batch
                    if (s.state == Slab::kOpen) s.full = true;
                for (Slab& s : active())
                    if (s.state == Slab::kFree) {
                        s.open(op, len, pitch, tiles, arena_, ++opened_, direct);
                        slab = &s;
                        break;
                    }
            }
            if (slab) break;
            cv_worker_.notify_one();  // the open batch was closed: let it leave
            cv_slot_.wait(lock);      // until an arena is free again
        }
        const int64_t t_sub2 = now_ns();
        const int slot = slab->reserved++;
        slab->readers++;
        if (slab->reserved == slab->capacity) slab->full = true;
        if (slot == 0 || slab->full) cv_worker_.notify_one();
        lock.unlock();

        // tile t of column j at slot * in_stride + (t * cols + j) * pitch (untiled: t = 0)
        const size_t in_stride = tiles * op.cols * pitch;  // == the slab's (matches())
        uint8_t* const in_base = slab->pin_in + slot * in_stride;
        for (int j = 0; j < op.cols; ++j) {
            const size_t n = op.lens ? op.lens[j] : len;  // padded: only the content bytes
            if (op.lens) slab->pin_lens[static_cast<size_t>(slot) * op.cols + j] = static_cast<uint32_t>(n);
            if (direct) {  // the gather reads [lo, hi) from the caller's buffer, the rest from the arena
                const size_t i = static_cast<size_t>(slot) * kern::kMaxCols + j;
                const size_t lo = std::min(dp->in_lo[j], n), hi = std::min(std::max(dp->in_hi[j], lo), n);
                // the unit's base at its device address ([lo, hi) is what the gather reads there)
                slab->dsrc[i] = n ? reinterpret_cast<const uint8_t*>(dp->in_dev[j]) : nullptr;
                slab->dsrc_n[i] = n;
                slab->dsrc_lo[i] = lo;
                slab->dsrc_hi[i] = hi;
                uint8_t* const at = in_base + j * pitch;  // untiled
                if (lo) add_copy(jobs, at, op.in[j], lo);
                if (hi < n) add_copy(jobs, at + hi, op.in[j] + hi, n - hi);
                continue;
            }
            for (size_t o = 0; o < n; o += pitch)  // untiled: pitch >= len, one copy
                add_copy(jobs, in_base + (o / pitch * op.cols + j) * pitch, op.in[j] + o, std::min(pitch, n - o));
        }
        if (direct) {
            for (int r = 0; r < op.rows; ++r) {
                const size_t i = static_cast<size_t>(slot) * kern::kMaxRows + r;
                const size_t lo = std::min(dp->out_lo[r], len);
                slab->ddst[i] = reinterpret_cast<uint8_t*>(dp->out_dev[r]);
                slab->ddst_lo[i] = lo;
                slab->ddst_hi[i] = std::min(std::max(dp->out_hi[r], lo), len);
            }
        }
        if (!jobs.empty()) run_copies(jobs, !direct && callers_.load() <= lone_callers());  // fenced before the H2D

        const int64_t t_filled = now_ns();
        add_phase(1, t_phase_mark, t_filled);
        if (phase_debug() && t_filled - t_phase_mark > phase_debug())
            std::fprintf(stderr, "elect_ec slow fill: %.1f us (enter %.1f, mutex %.1f, slab %.1f, copies %.1f)\n",
                         (t_filled - t_phase_mark) * 1e-3, (t_sub0 - t_phase_mark) * 1e-3, (t_sub1 - t_sub0) * 1e-3,
                         (t_sub2 - t_sub1) * 1e-3, (t_filled - t_sub2) * 1e-3);
        lock.lock();
        if (++slab->filled == slab->reserved) cv_worker_.notify_one();
        slab->done.wait(lock, [&] { return slab->state == Slab::kDone; });
        const int status = slab->status;
        t_phase_mark = now_ns();
        add_phase(2, t_filled, slab->t_issue0);
        add_phase(5, slab->t_finish, t_phase_mark);
        lock.unlock();

        if (status == ELECT_EC_OK && direct) {  // the scatter wrote [lo, hi) of each output; the rest is in the arena
            const uint8_t* const out_base = slab->pin_out + slot * (op.rows * pitch);
            jobs.clear();
            for (int r = 0; r < op.rows; ++r) {
                const size_t lo = std::min(dp->out_lo[r], len), hi = std::min(std::max(dp->out_hi[r], lo), len);
                if (lo) add_copy(jobs, op.out[r], out_base + r * pitch, lo);
                if (hi < len) add_copy(jobs, op.out[r] + hi, out_base + r * pitch + hi, len - hi);
            }
            if (!jobs.empty()) run_copies(jobs, false);
        } else if (status == ELECT_EC_OK) {
            const size_t out_stride = tiles * op.rows * pitch;
            const uint8_t* const out_base = slab->pin_out + slot * out_stride;
            jobs.clear();
            for (int r = 0; r < op.rows; ++r)
                for (size_t t = 0; t < tiles; ++t) {
                    const size_t o = t * pitch;
                    add_copy(jobs, op.out[r] + o, out_base + (t * op.rows + r) * pitch,
                             tiles > 1 ? std::min(pitch, len - o) : len);
                }
            run_copies(jobs, callers_.load() <= lone_callers());
        }
        if (status == ELECT_EC_OK && op.hashes)
            std::memcpy(op.hashes, slab->pin_hash + static_cast<size_t>(slot) * op.rows, op.rows * sizeof(int32_t));
        lock.lock();
        if (--slab->readers == 0) {
            slab->state = Slab::kFree;
            cv_slot_.notify_all();
        }
        return status;
    }

private:
    struct Shape {  // what a batch computes, copied out of its slab under mu_
        int cols = 0, rows = 0;
        size_t len = 0, pitch = 0, tiles = 1;
        bool padded = false, hashed = false, direct = false;
        uint8_t coef[kern::kMaxRows * kern::kMaxCols] = {};
    };

    // A direct batch's unit pointers, copied out of its slab under mu_ by the
    // dispatcher (the callers write them before taking mu_ to count themselves
    // filled).  issue() reads only this copy: the slab's arrays are rewritten for
    // its next batch once this one completes, and the only order between that and
    // issue()'s reads would otherwise run through the HIP streams (ThreadSanitizer,
    // profiles/r04/tsan_summary.txt).
    struct DirectSlots {
        std::vector<const uint8_t*> src;
        std::vector<size_t> src_n, src_lo, src_hi;
        std::vector<uint8_t*> dst;
        std::vector<size_t> dst_lo, dst_hi;
    };

    struct Slab {
        enum State { kFree, kOpen, kInFlight, kDone } state = kFree;
        Batcher* owner = nullptr;
        int cols = 0, rows = 0;
        size_t len = 0, pitch = 0, tiles = 1;
        uint8_t coef[kern::kMaxRows * kern::kMaxCols] = {};
        int capacity = 0, reserved = 0, filled = 0, readers = 0, status = ELECT_EC_OK;
        bool full = false;
        bool padded = false, hashed = false, direct = false;
        uint64_t seq = 0;
        std::chrono::steady_clock::time_point opened;
        uint8_t *pin_in = nullptr, *pin_out = nullptr, *d_in = nullptr, *d_out = nullptr;
        uint32_t *pin_lens = nullptr, *d_lens = nullptr;  // [slot][cols]; direct batches: [step][slot][cols]
        int32_t *pin_hash = nullptr, *d_hash = nullptr;    // [slot][rows]
        // direct batches: the arenas' and metadata's device addresses, and the
        // gather + scatter piece table (page-locked, read by the copy kernels where it lies)
        uint8_t *pin_in_dev = nullptr, *pin_out_dev = nullptr;
        uint8_t *pin_lens_dev = nullptr, *pin_hash_dev = nullptr;
        kern::CopyPiece* pieces = nullptr;
        const kern::CopyPiece* pieces_dev = nullptr;
        size_t max_pieces = 0;
        uint32_t* d_scratch = nullptr;                       // hash partials of the batch's launches
        size_t scratch_words = 0;
        // direct batches: each slot's unit pointers, input byte counts and the
        // [lo, hi) moved straight from / to the caller's memory, [slot][kMaxCols / kMaxRows]
        std::unique_ptr<const uint8_t*[]> dsrc;
        std::unique_ptr<size_t[]> dsrc_n, dsrc_lo, dsrc_hi;
        std::unique_ptr<uint8_t*[]> ddst;
        std::unique_ptr<size_t[]> ddst_lo, ddst_hi;
        std::condition_variable done;  // this batch's callers wait here for kDone
        // h2d_done: the batch's inputs have (nearly) all landed, the dispatch gate
        // (on the gather stream, behind the gate step); done_ev: behind its last
        // operation (on the scatter stream).  Both polled (Batcher::poller).
        hipStream_t stream = nullptr;  // the slab's batches, in order
        hipEvent_t h2d_done = nullptr;
        hipEvent_t done_ev = nullptr;
        int64_t t_issue0 = 0, t_issue1 = 0, t_finish = 0;  // phase marks (now_ns, under the owner's mu_)
        // early issue (Batcher::early_issue): the batch's gate number, written to the device
        // counter behind its last gather (gate_written: that write is enqueued); the bytes its
        // gathers move, and when the poller expects / saw its gate (now_ns)
        uint64_t gate_seq = 0;
        bool gate_written = false;
        size_t gather_bytes = 0;
        int64_t expect_gate = 0, t_gate = 0;
        // the bytes moved after the gate, and when the poller expects the batch done
        size_t tail_bytes = 0;
        int64_t expect_done = 0;
        bool h2d_landed = false;  // the batch in flight has passed its gate (under the owner's mu_)
        bool issued = false;      // ... and all of its work is enqueued, events recorded

        Shape shape() const
        {
            Shape sh;
            sh.cols = cols;
            sh.rows = rows;
            sh.len = len;
            sh.pitch = pitch;
            sh.tiles = tiles;
            sh.padded = padded;
            sh.hashed = hashed;
            sh.direct = direct;
            std::memcpy(sh.coef, coef, sizeof(coef));
            return sh;
        }

        bool matches(const HostOp& op, size_t n, bool d) const
        {
            return op.cols == cols && op.rows == rows && n == len && (op.lens != nullptr) == padded &&
                   (op.hashes != nullptr) == hashed && d == direct && std::memcmp(op.coef, coef, sizeof(coef)) == 0;
        }

        void open(const HostOp& op, size_t n, size_t p, size_t t, size_t arena, uint64_t order, bool d)
        {
            cols = op.cols;
            rows = op.rows;
            len = n;
            pitch = p;
            tiles = t;
            std::memcpy(coef, op.coef, sizeof(coef));
            padded = op.lens != nullptr;
            hashed = op.hashes != nullptr;
            direct = d;
            size_t cap = arena / (static_cast<size_t>(std::max(cols, rows)) * pitch * tiles);
            if (padded) cap = std::min(cap, kMetaEntries / cols);
            if (hashed) cap = std::min(cap, kMetaEntries / rows);
            if (direct) cap = std::min(cap, kMaxDirectSlots);
            capacity = static_cast<int>(cap);
            reserved = filled = readers = 0;
            status = ELECT_EC_OK;
            full = false;
            seq = order;
            opened = std::chrono::steady_clock::now();
            state = kOpen;
        }
    };

    int init(size_t arena)
    {
        arena_ = arena;
        nslabs_ = batch_config().slabs.load();
        // One stream per slab carries its batch: a batch's steps run in stream order
        // (issue_direct), and batches overlap each other on their own streams (the next
        // batch's gathers beside this one's last scatter) with no dependency between
        // streams.  (A round-6 A/B chained three per-device streams -- gathers, coding,
        // scatters -- for overlap inside a batch: waiting on events across streams
        // (hipStreamWaitEvent) kept a runtime thread at 73 % of a core, 35-44 core-ms
        // per GiB; device-side waits on memory (hipStreamWaitValue64) cost no host CPU
        // but are blit kernels of 4-20 us per handoff on the queues, and the gathers
        // ran at 46 against 53 GB/s beside concurrent scatters: no faster than one
        // step.  tools/tune/spin_probe.cpp chain_*, profiles/r06/spin_chain.txt,
        // profiles/r06/pipeline_chain_ab.txt.)
        if (early_issue()) {  // (without the counter, batches wait on the host for their gates)
            hipError_t e = hipExtMallocWithFlags(reinterpret_cast<void**>(&gate_ctr_), sizeof(uint64_t), hipMallocSignalMemory);
            if (e != hipSuccess) {
                (void)hipGetLastError();
                e = hipMalloc(reinterpret_cast<void**>(&gate_ctr_), sizeof(uint64_t));
            }
            if (e == hipSuccess) e = hipMemset(gate_ctr_, 0, sizeof(uint64_t));
            if (e != hipSuccess) {
                (void)hipGetLastError();
                if (gate_ctr_) (void)hipFree(gate_ctr_);
                gate_ctr_ = nullptr;
            }
        }
        for (Slab& s : active()) {
            s.owner = this;
            hipError_t e = hipStreamCreateWithFlags(&s.stream, hipStreamNonBlocking);
            if (e == hipSuccess) e = hipEventCreateWithFlags(&s.h2d_done, hipEventDisableTiming);
            if (e == hipSuccess) e = hipEventCreateWithFlags(&s.done_ev, hipEventDisableTiming);
            // device first: an arena too large for the device fails there, before any host pinning
            if (e == hipSuccess) e = hipMalloc(reinterpret_cast<void**>(&s.d_in), arena);
            if (e == hipSuccess) e = hipMalloc(reinterpret_cast<void**>(&s.d_out), arena);
            if (e == hipSuccess) e = hipHostMalloc(reinterpret_cast<void**>(&s.pin_in), arena, hipHostMallocDefault);
            if (e == hipSuccess) e = hipHostMalloc(reinterpret_cast<void**>(&s.pin_out), arena, hipHostMallocDefault);
            const size_t meta = kMetaEntries * sizeof(uint32_t);
            if (e == hipSuccess) e = hipHostMalloc(reinterpret_cast<void**>(&s.pin_lens), meta, hipHostMallocDefault);
            if (e == hipSuccess) e = hipMalloc(reinterpret_cast<void**>(&s.d_lens), meta);
            if (e == hipSuccess) e = hipHostMalloc(reinterpret_cast<void**>(&s.pin_hash), meta, hipHostMallocDefault);
            // one step, the smallest pieces: one per 16 KiB of the arena plus 3 per unit, both
            // ways, and the lens and hash pieces (plan_steps checks a pipelined batch's count)
            s.max_pieces = 2 * (arena / kMinPiece + 3 * kMaxDirectSlots * std::max(kern::kMaxCols, kern::kMaxRows)) +
                           2 * (meta / kMinPiece + 1);
            if (e == hipSuccess)
                e = hipHostMalloc(reinterpret_cast<void**>(&s.pieces), s.max_pieces * sizeof(kern::CopyPiece),
                                  hipHostMallocDefault);
            void* dv = nullptr;
            if (e == hipSuccess) e = hipHostGetDevicePointer(&dv, s.pieces, 0);
            s.pieces_dev = static_cast<const kern::CopyPiece*>(dv);
            if (e == hipSuccess) e = hipHostGetDevicePointer(&dv, s.pin_in, 0);
            s.pin_in_dev = static_cast<uint8_t*>(dv);
            if (e == hipSuccess) e = hipHostGetDevicePointer(&dv, s.pin_out, 0);
            s.pin_out_dev = static_cast<uint8_t*>(dv);
            if (e == hipSuccess) e = hipHostGetDevicePointer(&dv, s.pin_lens, 0);
            s.pin_lens_dev = static_cast<uint8_t*>(dv);
            if (e == hipSuccess) e = hipHostGetDevicePointer(&dv, s.pin_hash, 0);
            s.pin_hash_dev = static_cast<uint8_t*>(dv);
            if (e == hipSuccess) e = hipMalloc(reinterpret_cast<void**>(&s.d_hash), meta);
            s.scratch_words = kern::hash_scratch_need(arena / 16);  // a batch has at most arena/16 segments
            if (e == hipSuccess) e = hipMalloc(reinterpret_cast<void**>(&s.d_scratch), s.scratch_words * sizeof(uint32_t));
            if (e != hipSuccess) return map_hip(e);
            s.dsrc.reset(new (std::nothrow) const uint8_t*[kMaxDirectSlots * kern::kMaxCols]);
            s.dsrc_n.reset(new (std::nothrow) size_t[kMaxDirectSlots * kern::kMaxCols]);
            s.dsrc_lo.reset(new (std::nothrow) size_t[kMaxDirectSlots * kern::kMaxCols]);
            s.dsrc_hi.reset(new (std::nothrow) size_t[kMaxDirectSlots * kern::kMaxCols]);
            s.ddst.reset(new (std::nothrow) uint8_t*[kMaxDirectSlots * kern::kMaxRows]);
            s.ddst_lo.reset(new (std::nothrow) size_t[kMaxDirectSlots * kern::kMaxRows]);
            s.ddst_hi.reset(new (std::nothrow) size_t[kMaxDirectSlots * kern::kMaxRows]);
            if (!s.dsrc || !s.dsrc_n || !s.dsrc_lo || !s.dsrc_hi || !s.ddst || !s.ddst_lo || !s.ddst_hi)
                return ELECT_EC_ENOMEM;
        }
        try {  // the dispatcher's copies never grow past this (no allocation on its thread)
            for (auto* v : {&slots_.src_n, &slots_.src_lo, &slots_.src_hi}) v->reserve(kMaxDirectSlots * kern::kMaxCols);
            for (auto* v : {&slots_.dst_lo, &slots_.dst_hi}) v->reserve(kMaxDirectSlots * kern::kMaxRows);
            slots_.src.reserve(kMaxDirectSlots * kern::kMaxCols);
            slots_.dst.reserve(kMaxDirectSlots * kern::kMaxRows);
            gbuf_.reserve(slabs_[0].max_pieces);
            sbuf_.reserve(slabs_[0].max_pieces);
        } catch (const std::bad_alloc&) {
            return ELECT_EC_ENOMEM;
        }
        return ELECT_EC_OK;
    }

    // Frees whatever init() allocated (after a failed init: nothing is in flight).
    void release()
    {
        if (gate_ctr_) (void)hipFree(gate_ctr_);
        gate_ctr_ = nullptr;
        for (Slab& s : active()) {
            if (s.stream) (void)hipStreamDestroy(s.stream);
            s.stream = nullptr;
            for (hipEvent_t* ev : {&s.h2d_done, &s.done_ev}) {
                if (*ev) (void)hipEventDestroy(*ev);
                *ev = nullptr;
            }
            for (uint8_t* h : {s.pin_in, s.pin_out})
                if (h) (void)hipHostFree(h);
            for (void* h : {static_cast<void*>(s.pin_lens), static_cast<void*>(s.pin_hash), static_cast<void*>(s.pieces)})
                if (h) (void)hipHostFree(h);
            for (void* d : {static_cast<void*>(s.d_in), static_cast<void*>(s.d_out), static_cast<void*>(s.d_lens),
                            static_cast<void*>(s.d_hash), static_cast<void*>(s.d_scratch)})
                if (d) (void)hipFree(d);
            s.pin_in = s.pin_out = s.d_in = s.d_out = nullptr;
            s.pin_lens = s.d_lens = nullptr;
            s.pin_hash = s.d_hash = nullptr;
            s.pieces = nullptr;
            s.pieces_dev = nullptr;
            s.pin_in_dev = s.pin_out_dev = s.pin_lens_dev = s.pin_hash_dev = nullptr;
            s.d_scratch = nullptr;
        }
        arena_ = 0;
    }

    // Waits for everything queued on a slab's stream (error paths only: it spins a
    // core, see wait_sleeping).
    static void drain(Slab& s)
    {
        if (s.stream) (void)hipStreamSynchronize(s.stream);
        (void)hipGetLastError();
    }

    // Self-clocking dispatch: a batch leaves as soon as the previous batch has
    // passed its gate (its inputs have landed: a pipelined batch's last gather
    // stage is done, its last coding launch and scatter may still run beside the
    // new batch's first gathers), or at once on an idle device; callers keep
    // filling the other arenas meanwhile.  An optional window (ELECT_EC_BATCH_WINDOW_US) caps how
    // long an idle device waits for more callers; 0 = never wait.
    void worker()
    {
        pthread_setname_np(pthread_self(), ("ec-dispatch" + std::to_string(dev_)).c_str());
        set_timer_slack();
        (void)hipSetDevice(dev_);
        Slab* prev = nullptr;
        std::unique_lock<std::mutex> lock(mu_);
        for (;;) {
            Slab* s = nullptr;
            cv_worker_.wait(lock, [&] {
                s = nullptr;
                for (Slab& x : active())
                    if (x.state == Slab::kOpen && (!s || x.seq < s->seq)) s = &x;
                return s != nullptr;
            });
            uint64_t wait_for = 0;  // issue early: s's stream waits on the device for prev's gate number
            if (prev && prev->state == Slab::kInFlight) {  // asleep until the poller sees prev pass its gate
                auto passed = [&] { return prev->h2d_landed || prev->state != Slab::kInFlight; };
                if (gate_ctr_ && prev->gate_written) {
                    // ... or until shortly before it is expected to: s then leaves now and its
                    // gathers start on the device right behind prev's (no poll / issue gap)
                    const int64_t at = prev->expect_gate - static_cast<int64_t>(early_us()) * 1000;
                    cv_worker_.wait_until(lock, std::chrono::steady_clock::time_point(std::chrono::nanoseconds(at)), passed);
                    if (!passed()) wait_for = prev->gate_seq;
                } else {
                    cv_worker_.wait(lock, passed);
                }
            } else {
                const unsigned w = batch_config().window_us.load();
                if (w) cv_worker_.wait_until(lock, s->opened + std::chrono::microseconds(w), [&] { return s->full; });
            }
            s->full = true;
            s->state = Slab::kInFlight;  // no more reservations
            s->h2d_landed = false;
            cv_worker_.wait(lock, [&] { return s->filled == s->reserved; });
            const Shape shape = s->shape();  // under mu_: open() rewrites these for the slab's next batch
            const int n = s->reserved;
            if (shape.direct) {
                const size_t ni = static_cast<size_t>(n) * kern::kMaxCols, no = static_cast<size_t>(n) * kern::kMaxRows;
                slots_.src.assign(s->dsrc.get(), s->dsrc.get() + ni);
                slots_.src_n.assign(s->dsrc_n.get(), s->dsrc_n.get() + ni);
                slots_.src_lo.assign(s->dsrc_lo.get(), s->dsrc_lo.get() + ni);
                slots_.src_hi.assign(s->dsrc_hi.get(), s->dsrc_hi.get() + ni);
                slots_.dst.assign(s->ddst.get(), s->ddst.get() + no);
                slots_.dst_lo.assign(s->ddst_lo.get(), s->ddst_lo.get() + no);
                slots_.dst_hi.assign(s->ddst_hi.get(), s->ddst_hi.get() + no);
            }
            s->t_issue0 = now_ns();
            s->t_issue1 = 0;
            lock.unlock();
            const uint64_t t0 = thread_cpu_ns();
            s->gate_written = false;
            const hipError_t e = shape.direct ? issue_direct(*s, shape, n, slots_, wait_for)
                                              : issue_staged(*s, shape, n, wait_for);
            g_issue_cpu_ns.fetch_add(thread_cpu_ns() - t0);
            if (e != hipSuccess) drain(*s);  // no completion was queued: nothing of it may still run
            const int64_t t_issued = now_ns();
            add_phase(3, s->t_issue0, t_issued);
            g_batches.fetch_add(1, std::memory_order_relaxed);
            lock.lock();
            s->t_issue1 = t_issued;
            // when its gate should pass: its gathers start at issue end or behind prev's gate
            const int64_t start = std::max<int64_t>(t_issued, wait_for && prev ? prev->expect_gate : 0);
            s->expect_gate = start + static_cast<int64_t>(static_cast<double>(s->gather_bytes) * gate_ns_per_byte_);
            if (e != hipSuccess) {
                finish(s, map_hip(e));
            } else {
                s->issued = true;
                cv_poll_.notify_one();
            }
            prev = s;
        }
    }

    // ---- steps of a direct batch (round 6) ------------------------------------
    // A direct batch runs in S steps over windows of its units' bytes, all on the
    // slab's one stream, as a software pipeline of copy stages and coding
    // launches:
    //   copy(G0)  code(0)  copy(G1 + S0)  code(1)  ...  code(S-1)  copy(S[S-1])
    // Gk gathers window k of every unit, Sk scatters window k of every output;
    // one copy stage moves window k+1 in and window k-1 out at once (gather and
    // scatter pieces interleaved in one launch of the copy kernel), so both PCIe
    // directions are busy inside one call and a lone caller's call is no longer
    // gather -> code -> scatter in series (round 5: 330 + 18 + 163 us per 4.4 MB
    // RS(6,4) stripe, profiles/r06/hostprof_t1_before.txt).  Stream order is
    // the only synchronisation: code(k) follows the stage that gathered window k,
    // the stage after it scatters what code(k) wrote.  S grows with the batch's
    // input bytes (one step per ELECT_EC_STEP_KB, default 4 MiB, at most
    // ELECT_EC_PIPELINE_STEPS, default 8; windows of at least 256 KiB,
    // multiples of 64 KiB).  Each coding launch takes its window: plain where the
    // window is whole 16-byte segments, padded with the window's length for the
    // last window's partial segment (no separate byte-granular tail launch),
    // padded ops with per-step content lengths ([step][slot][cols] in the slab's
    // lens arrays, moved by the first stage), hashed ops adding each window's
    // terms (31^(window offset + i)) into entries seeded 31^len.
    struct Steps {
        int n = 1;                     // steps
        size_t at[kMaxSteps + 1] = {};  // window k is unit bytes [at[k], at[k + 1])
        size_t piece = 0;              // gather / scatter piece bytes
        static Steps one(size_t len, size_t piece)
        {
            Steps st;
            st.at[1] = len;
            st.piece = piece;
            return st;
        }
    };
    static constexpr size_t kMinWindow = size_t{256} << 10;
    static constexpr size_t kMinPiece = size_t{16} << 10;

    static int max_steps()
    {
        static const int s = [] {
            const char* e = std::getenv("ELECT_EC_PIPELINE_STEPS");
            return e ? std::min(kMaxSteps, std::max(1, std::atoi(e))) : kMaxSteps;
        }();
        return s;
    }
    static size_t step_target()
    {
        static const size_t b = [] {
            const char* e = std::getenv("ELECT_EC_STEP_KB");
            return (e && std::atoi(e) > 0 ? static_cast<size_t>(std::atoi(e)) : size_t{4096}) << 10;
        }();
        return b;
    }
    // ELECT_EC_PIECE_KB (16..64): a fixed piece size; default: 64 KiB pieces for
    // stages of at least 16 MiB (two rounds of 64 KiB pieces over the copy
    // kernels' 128 blocks; round 5's 64-caller batches measured best at 64 KiB,
    // hostpath_low_concurrency.txt), 16 KiB below, so a lone caller's few-MiB
    // stage still spreads over every copy block with a short last round.
    static size_t piece_for(size_t stage_bytes)
    {
        static const size_t fixed = [] {
            const char* e = std::getenv("ELECT_EC_PIECE_KB");
            return e ? static_cast<size_t>(std::min(64, std::max(16, std::atoi(e)))) << 10 : size_t{0};
        }();
        if (fixed) return fixed;
        return stage_bytes >= (size_t{16} << 20) ? kern::kMaxPieceBytes : kMinPiece;
    }

    // ELECT_EC_PIPELINE_ALONE (default 1): pipeline a batch only when its callers
    // are all the callers in flight on the device.  With more callers, batches
    // already overlap one another (the next batch's gathers beside this one's
    // coding and scatter), and the steps' extra launches cost more than they
    // give: 2 / 4 / 8 callers 33.6-35.4 / 38.2-39.0 / 41.8-42.7 GiB/s pipelined
    // against 39.4-40.6 / 42.2-43.9 / 44.2-45.5 in one step, one caller 29.5-30.3
    // against 27.1-29.4 on the same box (35.0 against 28.4-29.2 on another),
    // profiles/r06/pipeline_ab.txt.
    // ELECT_EC_TAPER (default 1): the last two windows a half and a quarter of the others
    // (profiles/r06/taper_ab.txt); 0: equal windows.
    static bool taper()
    {
        static const bool t = [] {
            const char* e = std::getenv("ELECT_EC_TAPER");
            return !(e && std::atoi(e) == 0);
        }();
        return t;
    }

    static bool pipeline_alone_only()
    {
        static const bool a = [] {
            const char* e = std::getenv("ELECT_EC_PIPELINE_ALONE");
            return !(e && std::atoi(e) == 0);
        }();
        return a;
    }

    Steps plan_steps(const Shape& sh, int n, const DirectSlots& d) const
    {
        size_t in_bytes = 0;
        for (int q = 0; q < n; ++q)
            for (int j = 0; j < sh.cols; ++j) in_bytes += d.src_n[static_cast<size_t>(q) * kern::kMaxCols + j];
        int s = static_cast<int>(std::min<size_t>(max_steps(), std::max<size_t>(1, (in_bytes + step_target() - 1) / step_target())));
        if (pipeline_alone_only() && callers_.load() > n) s = 1;  // other callers wait: batches overlap instead
        s = static_cast<int>(std::min<size_t>(s, std::max<size_t>(1, sh.len / kMinWindow)));
        if (sh.padded) s = static_cast<int>(std::min<size_t>(s, std::max<size_t>(1, kMetaEntries / (static_cast<size_t>(n) * sh.cols))));
        Steps st;
        st.n = pipeline_windows(sh.len, s, taper(), st.at);
        st.piece = piece_for((in_bytes + static_cast<size_t>(n) * sh.rows * sh.len) / st.n);
        return st;
    }

    // Writes the direct batch's piece table for `st`: stage k (0..S) holds the
    // gather pieces of window k (k < S) and the scatter pieces of window k-1
    // (k >= 1), interleaved in proportion so that both directions run through
    // the whole launch; stage k is [begin[k], begin[k + 1]).  False when it does
    // not fit the slab's table.
    static bool write_pieces(Slab& s, const Shape& sh, int n, const DirectSlots& d, const Steps& st, size_t* begin,
                             std::vector<kern::CopyPiece>& gbuf, std::vector<kern::CopyPiece>& sbuf)
    {
        size_t np = 0;
        for (int k = 0; k <= st.n; ++k) {
            begin[k] = np;
            if (!write_stage(s, sh, n, d, st, k, np, gbuf, sbuf)) return false;
        }
        begin[st.n + 1] = np;
        return true;
    }
    // At least the number of pieces write_pieces() writes for `st` (a unit's range
    // clipped to a window is at most three segments, each ceil(bytes / piece)).
    static size_t piece_bound(const Shape& sh, int n, const Steps& st)
    {
        size_t b = 0;
        for (int k = 0; k <= st.n; ++k) {
            if (k < st.n) b += static_cast<size_t>(n) * sh.cols * ((st.at[k + 1] - st.at[k]) / st.piece + 3);
            if (k >= 1) b += static_cast<size_t>(n) * sh.rows * ((st.at[k] - st.at[k - 1]) / st.piece + 3);
        }
        if (sh.padded) b += static_cast<size_t>(st.n) * n * sh.cols * sizeof(uint32_t) / st.piece + 1;
        return b + 1;  // (+1: the hashes)
    }
    // Stage k's pieces at s.pieces[np...), np advanced past them.
    static bool write_stage(Slab& s, const Shape& sh, int n, const DirectSlots& d, const Steps& st, int k, size_t& np,
                            std::vector<kern::CopyPiece>& gbuf, std::vector<kern::CopyPiece>& sbuf)
    {
        const size_t in_stride = sh.cols * sh.pitch, out_stride = sh.rows * sh.pitch;
        bool room = true;  // (the lists never grow past what init() reserved: no allocation here)
        auto put = [&](std::vector<kern::CopyPiece>& v, const uint8_t* from, uint8_t* to, size_t bytes) {
            for (size_t o = 0; o < bytes && room; o += st.piece) {
                if (v.size() == v.capacity()) room = false;
                else v.push_back(kern::CopyPiece{from + o, to + o, static_cast<uint32_t>(std::min(st.piece, bytes - o)), 0});
            }
        };
        // [a, b) of a unit clipped to the window [w0, w1): from + x -> to + x
        auto seg = [&](std::vector<kern::CopyPiece>& v, size_t a, size_t b, size_t w0, size_t w1, const uint8_t* from,
                       uint8_t* to) {
            const size_t x = std::max(a, w0), y = std::min(b, w1);
            if (x < y) put(v, from + x, to + x, y - x);
        };
        {
            gbuf.clear();
            sbuf.clear();
            if (k < st.n) {  // gather window k
                const size_t w0 = st.at[k], w1 = st.at[k + 1];
                if (k == 0 && sh.padded)  // the per-step content lengths ride in the first stage
                    put(gbuf, s.pin_lens_dev, reinterpret_cast<uint8_t*>(s.d_lens),
                        static_cast<size_t>(st.n) * n * sh.cols * sizeof(uint32_t));
                for (int q = 0; q < n; ++q)
                    for (int j = 0; j < sh.cols; ++j) {
                        const size_t i = static_cast<size_t>(q) * kern::kMaxCols + j;
                        const size_t nb = d.src_n[i], lo = d.src_lo[i], hi = d.src_hi[i];
                        uint8_t* const dev = s.d_in + q * in_stride + j * sh.pitch;
                        const uint8_t* const pin = s.pin_in_dev + q * in_stride + j * sh.pitch;
                        seg(gbuf, 0, lo, w0, w1, pin, dev);
                        seg(gbuf, lo, hi, w0, w1, d.src[i], dev);
                        seg(gbuf, hi, nb, w0, w1, pin, dev);
                    }
            }
            if (k >= 1) {  // scatter window k-1
                const size_t w0 = st.at[k - 1], w1 = st.at[k];
                for (int q = 0; q < n; ++q)
                    for (int r = 0; r < sh.rows; ++r) {
                        const size_t i = static_cast<size_t>(q) * kern::kMaxRows + r;
                        const size_t lo = d.dst_lo[i], hi = d.dst_hi[i];
                        const uint8_t* const dev = s.d_out + q * out_stride + r * sh.pitch;
                        uint8_t* const pin = s.pin_out_dev + q * out_stride + r * sh.pitch;
                        seg(sbuf, 0, lo, w0, w1, dev, pin);
                        seg(sbuf, lo, hi, w0, w1, dev, d.dst[i]);
                        seg(sbuf, hi, sh.len, w0, w1, dev, pin);
                    }
                if (k == st.n && sh.hashed)  // the parity hashes ride in the last stage
                    put(sbuf, reinterpret_cast<const uint8_t*>(s.d_hash), s.pin_hash_dev,
                        static_cast<size_t>(n) * sh.rows * sizeof(int32_t));
            }
            if (!room || np + gbuf.size() + sbuf.size() > s.max_pieces) return false;
            // interleave: piece i of a list of m sits at position (i + 0.5) / m of the stage
            size_t gi = 0, si = 0;
            const size_t ng = gbuf.size(), ns = sbuf.size();
            while (gi < ng || si < ns) {
                const bool take_g = si == ns || (gi < ng && (2 * gi + 1) * ns <= (2 * si + 1) * ng);
                s.pieces[np++] = take_g ? gbuf[gi++] : sbuf[si++];
            }
        }
        return true;
    }

    // ---- early issue (round 6) ---------------------------------------------------
    // A batch leaves when the previous batch has passed its gate (the poller saw its
    // gathers done): ~30-130 us of the link unused per batch between one batch's last
    // gather and the next one's first (poll interval, dispatcher wake, issue, launch;
    // 8 callers: ~70 us of each ~1.35 ms batch, profiles/r06/early_issue_ab.txt).  With
    // early issue (ELECT_EC_EARLY_ISSUE, default on) the dispatcher closes the next batch
    // ELECT_EC_EARLY_US (default 150) before the previous batch's gate is expected (its
    // gather bytes at the measured gather time per byte), and the new batch's stream first
    // waits on the device until the previous batch has written its gate number behind its
    // last gather (hipStreamWriteValue64 / hipStreamWaitValue64 on one counter per device:
    // the command processor waits, no host thread spins, profiles/r06/spin_chain.txt).  A
    // wait is enqueued only for a number whose write was enqueued.
    static bool early_issue()
    {
        static const bool on = [] {
            const char* e = std::getenv("ELECT_EC_EARLY_ISSUE");
            return !(e && std::atoi(e) == 0);
        }();
        return on;
    }
    static unsigned early_us()
    {
        static const unsigned u = [] {
            const char* e = std::getenv("ELECT_EC_EARLY_US");
            return e ? static_cast<unsigned>(std::max(0, std::atoi(e))) : 150u;
        }();
        return u;
    }
    hipError_t wait_before(Slab& s, uint64_t wait_for) const
    {
        if (!wait_for) return hipSuccess;
        return hipStreamWaitValue64(s.stream, gate_ctr_, wait_for, hipStreamWaitValueGte, ~uint64_t{0});
    }
    // The gate: (early issue) the gate number written for the next batch's stream, then the
    // host-visible event the poller queries.  In that order: a batch the dispatcher issues
    // without a device wait (the previous one seen past its gate) writes its own, higher
    // number only after the previous number has landed, so the counter never goes back.
    // Written only while other callers wait (a lone caller's next batch never overlaps).
    hipError_t record_gate(Slab& s, int n)
    {
        hipError_t e = hipSuccess;
        s.gate_written = false;
        if (gate_ctr_ && callers_.load(std::memory_order_relaxed) > n) {
            s.gate_seq = ++gate_seq_;
            e = hipStreamWriteValue64(s.stream, gate_ctr_, s.gate_seq, 0);
            s.gate_written = e == hipSuccess;
        }
        if (e == hipSuccess) e = hipEventRecord(s.h2d_done, s.stream);
        return e;
    }

    // Direct batches: each unit's [lo, hi) straight from / to its caller's
    // page-locked memory (a locked pageable unit's interior pages, or a pool
    // unit), the rest (a locked unit's partial end pages) through the arena; by
    // gather / scatter kernels reading the piece table where it lies.  s's
    // buffers, stream and events never change after init(); its shape comes from
    // the copy taken under mu_.
    hipError_t issue_direct(Slab& s, const Shape& sh, int n, const DirectSlots& d, uint64_t wait_for)
    {
        Steps st = plan_steps(sh, n, d);
        size_t begin[kMaxSteps + 2];
        // A pipelined batch's table is written stage by stage, each just before its
        // launch, so that the first gather starts after one stage's descriptors, not
        // all of them (when the table surely has room for all).
        static const bool stage_writes = [] {  // ELECT_EC_STAGE_WRITES=0: the whole table first (A/B)
            const char* e = std::getenv("ELECT_EC_STAGE_WRITES");
            return !(e && std::atoi(e) == 0);
        }();
        const bool by_stage = stage_writes && st.n > 1 && piece_bound(sh, n, st) <= s.max_pieces;
        if (by_stage) {
            begin[0] = 0;
        } else if (!write_pieces(s, sh, n, d, st, begin, gbuf_, sbuf_)) {
            st = Steps::one(sh.len, kern::kMaxPieceBytes);  // one step of 64 KiB pieces always fits
            if (!write_pieces(s, sh, n, d, st, begin, gbuf_, sbuf_)) return hipErrorInvalidValue;
        }
        const size_t in_stride = sh.cols * sh.pitch, out_stride = sh.rows * sh.pitch;
        if (sh.padded)  // [step][slot][col]: each window's share of every unit's content
            for (int t = 0; t < st.n; ++t) {
                const size_t w0 = st.at[t], w = st.at[t + 1] - w0;
                uint32_t* l = s.pin_lens + static_cast<size_t>(t) * n * sh.cols;
                for (int q = 0; q < n; ++q)
                    for (int j = 0; j < sh.cols; ++j) {
                        const size_t raw = d.src_n[static_cast<size_t>(q) * kern::kMaxCols + j];
                        l[q * sh.cols + j] = static_cast<uint32_t>(raw > w0 ? std::min(raw - w0, w) : 0);
                    }
            }
        s.gather_bytes = 0;  // (whole stages up to the last gather: pieces of both directions)
        auto stage_bytes = [&](int k) {
            if (k < st.n)
                for (size_t i = begin[k]; i < begin[k + 1]; ++i) s.gather_bytes += s.pieces[i].n;
        };
        if (!by_stage)
            for (int k = 0; k < st.n; ++k) stage_bytes(k);
        hipError_t e = wait_before(s, wait_for);
        const bool seed = sh.hashed && st.n > 1;  // windows add into entries seeded 31^len
        if (seed && e == hipSuccess)
            e = hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(s.d_hash), static_cast<int>(kern::pow31(sh.len)),
                                  static_cast<size_t>(n) * sh.rows, s.stream);
        for (int k = 0; k <= st.n && e == hipSuccess; ++k) {
            if (by_stage) {
                size_t np = begin[k];
                if (!write_stage(s, sh, n, d, st, k, np, gbuf_, sbuf_)) {
                    e = hipErrorInvalidValue;  // (piece_bound() said it fits: not reached)
                    break;
                }
                begin[k + 1] = np;
                stage_bytes(k);
            }
            e = kern::launch_copy_pieces(s.pieces_dev + begin[k], static_cast<uint32_t>(begin[k + 1] - begin[k]), s.stream);
            // the gate: the batch's last gather is done (the next batch's gathers may start beside its last scatter)
            if (e == hipSuccess && k == st.n - 1) e = record_gate(s, n);
            if (e != hipSuccess || k == st.n) break;
            const size_t w0 = st.at[k], w = st.at[k + 1] - w0;
            ApplyParams p;
            p.len = w;
            p.stripes = static_cast<uint64_t>(n);
            p.cols = sh.cols;
            p.rows = sh.rows;
            for (int j = 0; j < sh.cols; ++j) p.src[j] = col(s.d_in, in_stride, j * sh.pitch + w0);
            for (int r = 0; r < sh.rows; ++r) p.dst[r] = col(s.d_out, out_stride, r * sh.pitch + w0);
            std::memcpy(p.coef, sh.coef, sizeof(p.coef));
            if (sh.padded) {
                p.padded = true;
                p.lens = s.d_lens + static_cast<size_t>(k) * n * sh.cols;
            } else if (w % 16) {  // the unit's last partial segment, in the same launch
                p.padded = true;
                for (int j = 0; j < sh.cols; ++j) p.clen[j] = static_cast<uint32_t>(w);
            }
            if (sh.hashed) {
                p.hashes = s.d_hash;
                p.hash_stride = static_cast<uint32_t>(sh.rows);
                p.hash_base = w0;
                p.hash_seed = !seed;
                p.hash_scratch = s.d_scratch;
                p.hash_scratch_words = s.scratch_words;
            }
            e = kern::launch_apply(p, s.stream);
        }
        s.tail_bytes = 0;
        if (e == hipSuccess)
            for (size_t i = begin[st.n]; i < begin[st.n + 1]; ++i) s.tail_bytes += s.pieces[i].n;
        if (e == hipSuccess) e = hipEventRecord(s.done_ev, s.stream);
        return e;
    }

    // Staged batches (the callers copied their units into the pinned arena): one
    // H2D, one coding launch over the arena's tiles, one D2H.
    hipError_t issue_staged(Slab& s, const Shape& sh, int n, uint64_t wait_for)
    {
        const size_t in_stride = sh.tiles * sh.cols * sh.pitch;  // per slot
        const size_t out_stride = sh.tiles * sh.rows * sh.pitch;
        s.gather_bytes = n * in_stride;
        s.tail_bytes = n * out_stride;
        hipError_t e = wait_before(s, wait_for);
        if (e == hipSuccess) e = hipMemcpyAsync(s.d_in, s.pin_in, n * in_stride, hipMemcpyHostToDevice, s.stream);
        if (e == hipSuccess && sh.padded)
            e = hipMemcpyAsync(s.d_lens, s.pin_lens, static_cast<size_t>(n) * sh.cols * sizeof(uint32_t),
                               hipMemcpyHostToDevice, s.stream);
        if (e == hipSuccess) e = record_gate(s, n);
        if (e == hipSuccess) {
            // coding stripes: the slots' tiles in order (untiled: the slots)
            ApplyParams p;
            p.len = sh.tiles > 1 ? sh.pitch : sh.len;
            p.stripes = static_cast<uint64_t>(n) * sh.tiles;
            p.cols = sh.cols;
            p.rows = sh.rows;
            for (int j = 0; j < sh.cols; ++j) p.src[j] = col(s.d_in, sh.cols * sh.pitch, j * sh.pitch);
            for (int r = 0; r < sh.rows; ++r) p.dst[r] = col(s.d_out, sh.rows * sh.pitch, r * sh.pitch);
            std::memcpy(p.coef, sh.coef, sizeof(p.coef));
            if (sh.tiles > 1) {
                p.tiles = static_cast<uint32_t>(sh.tiles);
                p.unit_len = sh.len;
                p.padded = true;
                for (int j = 0; j < sh.cols; ++j) p.clen[j] = static_cast<uint32_t>(sh.len);
            }
            if (sh.padded) {
                p.padded = true;
                p.lens = s.d_lens;
            }
            if (sh.hashed) {
                p.hashes = s.d_hash;
                p.hash_stride = static_cast<uint32_t>(sh.rows);
                p.hash_seed = true;
                p.hash_scratch = s.d_scratch;
                p.hash_scratch_words = s.scratch_words;
            }
            e = kern::launch_apply(p, s.stream);
        }
        if (e == hipSuccess) e = hipMemcpyAsync(s.pin_out, s.d_out, n * out_stride, hipMemcpyDeviceToHost, s.stream);
        if (e == hipSuccess && sh.hashed)
            e = hipMemcpyAsync(s.pin_hash, s.d_hash, static_cast<size_t>(n) * sh.rows * sizeof(int32_t),
                               hipMemcpyDeviceToHost, s.stream);
        if (e == hipSuccess) e = hipEventRecord(s.done_ev, s.stream);
        return e;
    }

    // How the dispatcher learns that a batch has passed its gate (self-clocking)
    // and the callers that their batch is done: a poller thread per device
    // queries the batches' events (hipEventQuery) and sleeps ELECT_EC_POLL_US
    // (default 25) between rounds.  Every waiting primitive of this HIP runtime
    // spins a core for as long as the device work it waits for runs:
    // hipStreamSynchronize, hipEventSynchronize (hipEventBlockingSync events too)
    // 94 % of a core each behind 5 ms kernels, the runtime's host-function thread
    // 96 % (tools/tune/spin_probe.cpp, profiles/r05/spin_probe.txt), where
    // hipEventQuery every 50 us costs 2 %.  At 64 callers the callback thread
    // alone was 19-20 core-ms per GiB, and the dispatcher spinning on the H2D
    // event 53 against 35 (hostpath_register_ab.txt E); both modes were A/B
    // switches in round 5 (ELECT_EC_DISPATCH_WAIT) and are gone since.
    // The poller's sleeps and the dispatcher's timed waits end up to the thread's timer
    // slack late (Linux default 50 us): a 25 us poll round took ~75 us, and a lone caller's
    // call waited for the round after its batch was done.  ELECT_EC_TIMER_SLACK_NS (default
    // 2000; 0 leaves the default) for these two threads only (profiles/r06/slack_ab.txt).
    static void set_timer_slack()
    {
        static const long ns = [] {
            const char* e = std::getenv("ELECT_EC_TIMER_SLACK_NS");
            return e ? std::max(0L, std::atol(e)) : 2000L;
        }();
        if (ns > 0) (void)prctl(PR_SET_TIMERSLACK, static_cast<unsigned long>(ns), 0, 0, 0);
    }
    static unsigned poll_us()
    {
        static const unsigned u = [] {
            const char* e = std::getenv("ELECT_EC_POLL_US");
            return e ? static_cast<unsigned>(std::max(1, std::atoi(e))) : 25u;
        }();
        return u;
    }

    // Marks in-flight batches past their gate (waking the dispatcher) and
    // finishes completed batches (waking their callers).  Only this thread
    // finishes an issued batch, so a batch it saw issued stays in flight until
    // it finishes it.
    void poller()
    {
        pthread_setname_np(pthread_self(), ("ec-poll" + std::to_string(dev_)).c_str());
        set_timer_slack();
        (void)hipSetDevice(dev_);
        std::unique_lock<std::mutex> lock(mu_);
        for (;;) {
            cv_poll_.wait(lock, [&] {
                for (Slab& x : active())
                    if (x.state == Slab::kInFlight && x.issued) return true;
                return false;
            });
            for (Slab& x : active()) {
                if (x.state != Slab::kInFlight || !x.issued) continue;
                const bool landed = x.h2d_landed;
                lock.unlock();  // (a slab's events never change after init)
                // the batch cannot be done before it has passed its gate
                const hipError_t eh = landed ? hipSuccess : hipEventQuery(x.h2d_done);
                const hipError_t ed = eh == hipSuccess ? hipEventQuery(x.done_ev) : hipErrorNotReady;
                const bool failed = (eh != hipSuccess && eh != hipErrorNotReady) || (ed != hipSuccess && ed != hipErrorNotReady);
                if (failed) drain(x);  // nothing of the batch may still run when its callers return
                lock.lock();
                if (!landed && eh != hipErrorNotReady) {
                    x.h2d_landed = true;
                    x.t_gate = now_ns();
                    // the gather time per byte, for the next batches' expected gates (from the later of
                    // issue end and the previous gate: a batch issued early starts behind it)
                    const int64_t from = std::max(x.t_issue1, last_gate_);
                    if (x.t_issue1 && x.gather_bytes > (size_t{1} << 20) && x.t_gate > from)
                        gate_ns_per_byte_ = 0.8 * gate_ns_per_byte_ +
                                            0.2 * static_cast<double>(x.t_gate - from) / static_cast<double>(x.gather_bytes);
                    last_gate_ = x.t_gate;
                    x.expect_done = x.t_gate + static_cast<int64_t>(static_cast<double>(x.tail_bytes) * tail_ns_per_byte_);
                    cv_worker_.notify_one();
                }
                if (eh != hipSuccess && eh != hipErrorNotReady) {  // a failed batch is done, with its error
                    finish(&x, map_hip(eh));
                    continue;
                }
                if (ed == hipErrorNotReady) continue;
                if (ed == hipSuccess && x.tail_bytes > (size_t{256} << 10)) {
                    const int64_t t = now_ns();
                    tail_ns_per_byte_ = 0.8 * tail_ns_per_byte_ +
                                        0.2 * static_cast<double>(t - x.t_gate) / static_cast<double>(x.tail_bytes);
                }
                finish(&x, ed == hipSuccess ? ELECT_EC_OK : map_hip(ed));
            }
            const int64_t wake = next_poll(now_ns());
            lock.unlock();
            std::this_thread::sleep_until(std::chrono::steady_clock::time_point(std::chrono::nanoseconds(wake)));
            lock.lock();
        }
    }

    // When the poller looks next (mu_ held): poll_us() from now, or earlier when a batch
    // in flight nears the time its next event (gate, then done) is expected, and every
    // ELECT_EC_POLL_FINE_US (default 5) from then on until that event is seen.  A lone
    // caller's call no longer waits up to a whole round after its batch is done.
    // Only for events expected within kFineSpan of their batch's issue or gate (a lone
    // caller's pipelined batch, ~0.4 ms): 64 callers' ~10 ms batches gain nothing from it.
    // (Polling those less often, at half the distance to the expected event, saved no CPU:
    // profiles/r06/poll_ab.txt.)
    static constexpr int64_t kFineSpan = 2000000;
    int64_t next_poll(int64_t now) const
    {
        static const int64_t fine = [] {
            const char* e = std::getenv("ELECT_EC_POLL_FINE_US");
            return static_cast<int64_t>(e ? std::max(0, std::atoi(e)) : 5) * 1000;
        }();
        int64_t wake = now + static_cast<int64_t>(poll_us()) * 1000;
        if (!fine) return wake;
        for (int i = 0; i < nslabs_; ++i) {
            const Slab& x = slabs_[i];
            if (x.state != Slab::kInFlight || !x.issued) continue;
            const int64_t target = x.h2d_landed ? x.expect_done : x.expect_gate;
            const int64_t base = x.h2d_landed ? x.t_gate : x.t_issue1;
            if (target - base > kFineSpan) continue;  // a long batch: a round is a small share of it
            const int64_t start = target - std::max<int64_t>(10000, (target - base) / 8);
            wake = std::min(wake, now >= start ? now + fine : start);
        }
        return wake;
    }

    void finish(Slab* s, int status)  // mu_ held
    {
        s->t_finish = now_ns();
        add_phase(4, s->t_issue1, s->t_finish);
        s->status = status;
        s->issued = false;
        if (s->readers == 0) {
            s->state = Slab::kFree;
            cv_slot_.notify_all();
        } else {
            s->state = Slab::kDone;
            s->done.notify_all();
        }
    }

    int dev_;
    std::atomic<int> callers_{0};
    // One mutex; three kinds of waiter, so that a state change wakes only the
    // threads it concerns (one condition variable for all woke every caller on
    // every reservation: O(callers^2) wake-ups per batch at 64 callers).
    std::mutex mu_;
    std::condition_variable cv_worker_;  // the dispatcher
    std::condition_variable cv_poll_;    // the poller, while no batch is in flight
    DirectSlots slots_;                  // the dispatcher's copy of a direct batch's slots (its thread only)
    std::vector<kern::CopyPiece> gbuf_, sbuf_;  // a stage's gather / scatter pieces (dispatcher thread only)
    // early issue: the device counter each batch writes its gate number to behind its last gather
    // (a batch issued early waits on it, hipStreamWaitValue64), the last number handed out
    // (dispatcher thread), and the measured gather time per byte (EWMA, under mu_)
    uint64_t* gate_ctr_ = nullptr;
    uint64_t gate_seq_ = 0;
    double gate_ns_per_byte_ = 1.0 / 50.0;
    double tail_ns_per_byte_ = 1.0 / 50.0;  // after the gate, to done (poller only)
    int64_t last_gate_ = 0;  // when the poller last saw a gate pass (under mu_)
    std::condition_variable cv_slot_;    // callers waiting for an arena to reserve in
    bool started_ = false;
    bool init_failed_ = false;  // the arenas could not be allocated: every call runs directly
    size_t arena_ = 0;
    uint64_t opened_ = 0;
    Slab slabs_[kMaxSlabs];
    int nslabs_ = 3;  // set once by init()
    struct SlabRange {
        Slab* b;
        Slab* e;
        Slab* begin() const { return b; }
        Slab* end() const { return e; }
    };
    SlabRange active() { return SlabRange{slabs_, slabs_ + nslabs_}; }
};

Batcher* batcher(int dev)
{
    static std::mutex mu;
    static Batcher* all[kMaxDevices] = {};  // never destroyed: their threads live until exit
    std::lock_guard<std::mutex> lock(mu);
    if (!all[dev]) all[dev] = new (std::nothrow) Batcher(dev);
    return all[dev];
}

// ---------------------------------------------------------------------------
// Zero-copy calls (OFF by default since round 5: the batched path's per-call
// locking and gather / scatter kernels serve a lone caller faster, 24.9 against
// 19.8-20.7 GiB/s at ELECT's codeLength, and equally at two callers, 35.0 against
// 34.5, profiles/r05/hostpath_register_ab.txt G).  A caller that is alone on its
// device (no other call in flight, no other thread calling for 20 ms:
// lone_caller) has its own buffers page-locked for the duration of the call
// (hsa_amd_memory_lock since round 5, hipHostRegister before), and the kernel
// reads its units and writes its outputs over PCIe directly: no staging copies,
// no DMA stages, no helper threads.
// tools/tune/zerocopy_probe.py (RS(6,4), 4,404,020 B, one caller): 35.4 GiB/s
// against 22.1 for the staged path (register 0.02 ms and unregister 0.01 ms per
// call; kernel 0.43 ms); through the product (bench.py --config hostpath, 2 s
// runs, profiles/r03/zerocopy_hostpath.txt): 1 caller 31.9-32.2 against 22.6
// GiB/s staged, but 2 callers 35.9 against 38.8-39.3 batched.  Concurrent
// callers lose with it (registration contends in the driver: 7.8 + 12.6 ms per
// call at 64 callers, and 64 kernels reading host memory at once run at 26
// GiB/s against the batch's 44), so only a lone caller takes it.  ELECT_EC_ZEROCOPY: 0 off (default), 1 lone callers with
// units of at least kMinBytes, 2 every eligible call (tests).  Hashed calls keep
// the staged path.  Any registration failure (memory already locked by another
// call, a mapping the driver refuses) falls back to the staged path.  Units in
// the engine's page-locked pool (direct_op) need no registration: the kernel
// reads and writes them where they are.
// ---------------------------------------------------------------------------
struct ZeroCopy {
    static constexpr size_t kMinBytes = size_t{1} << 20;  // mmap-backed buffers: no page shared with another caller
    static constexpr int kMaxInFlight = 1;                // callers on the device, this one included
    static constexpr int kFallback = -1000;

    static int mode()
    {
        static const int m = [] {
            const char* e = std::getenv("ELECT_EC_ZEROCOPY");
            return e ? std::atoi(e) : 0;
        }();
        return m;
    }

    static bool eligible(const HostOp& op, size_t len, int in_flight, bool alone)
    {
        const int m = mode();
        if (m == 0 || op.hashes || len > 0xFFFFFFFFull) return false;
        return m == 2 || (len >= kMinBytes && in_flight <= kMaxInFlight && alone);
    }

    // Page-aligned, merged [begin, end) intervals covering every byte the
    // call's kernels touch (inputs: input_span), pool units left out: the pool
    // holds them locked already and the kernel addresses them at the pool's
    // device address (locking them again here, and unlocking after the
    // call, would have released pages the pool still owns).
    static std::vector<std::pair<uintptr_t, uintptr_t>> ranges(const HostOp& op, size_t len)
    {
        constexpr uintptr_t kPage = 4096;
        PinnedPool& pool = PinnedPool::get();
        std::vector<std::pair<uintptr_t, uintptr_t>> r;
        auto add = [&](const void* p, size_t n) {
            if (!p || !n || pool.pinned(p, n)) return;
            const uintptr_t a = reinterpret_cast<uintptr_t>(p);
            r.emplace_back(a & ~(kPage - 1), (a + n + kPage - 1) & ~(kPage - 1));
        };
        for (int j = 0; j < op.cols; ++j) add(op.in[j], input_span(op, j, len));
        for (int q = 0; q < op.rows; ++q) add(op.out[q], len);
        std::sort(r.begin(), r.end());
        std::vector<std::pair<uintptr_t, uintptr_t>> m;
        for (const auto& x : r) {
            if (!m.empty() && x.first <= m.back().second)
                m.back().second = std::max(m.back().second, x.second);
            else
                m.push_back(x);
        }
        return m;
    }

    // No unit's first or last byte is known to the HIP runtime (registered or
    // allocated by another party): the page-rounded ranges start before and end
    // after the units, so the registry's checks at the range ends would miss a
    // registration of exactly a unit.
    static bool units_unknown(const HostOp& op, size_t len)
    {
        auto unknown = [](const void* x) {
            hipPointerAttribute_t a{};
            const hipError_t e = hipPointerGetAttributes(&a, x);
            (void)hipGetLastError();
            return e == hipSuccess && a.type == hipMemoryTypeUnregistered;
        };
        PinnedPool& pool = PinnedPool::get();
        for (int j = 0; j < op.cols; ++j) {
            const size_t n = input_span(op, j, len);
            if (op.in[j] && n && !pool.pinned(op.in[j], n) && !(unknown(op.in[j]) && unknown(op.in[j] + n - 1)))
                return false;
        }
        for (int r = 0; r < op.rows; ++r)
            if (!pool.pinned(op.out[r], len) && !(unknown(op.out[r]) && unknown(op.out[r] + len - 1))) return false;
        return true;
    }

    // This thread's stream per device, destroyed when the thread exits (ELECT's
    // coding pools retire threads).
    struct ThreadStreams {
        hipStream_t stream[kMaxDevices] = {};
        hipEvent_t done[kMaxDevices] = {};  // the call's end (wait_sleeping)
        ~ThreadStreams()
        {
            for (int d = 0; d < kMaxDevices; ++d) {
                if (!stream[d]) continue;
                int prev = 0;
                const bool other = hipGetDevice(&prev) == hipSuccess && prev != d && hipSetDevice(d) == hipSuccess;
                (void)hipStreamDestroy(stream[d]);
                if (done[d]) (void)hipEventDestroy(done[d]);
                if (other) (void)hipSetDevice(prev);
            }
        }
    };

    // pinned: every unit already lies in the engine's page-locked pool (direct_op):
    // nothing to register, the device reads and writes the pool buffers in place.
    static int run(const HostOp& op, size_t len, bool pinned)
    {
        thread_local ThreadStreams ts;
        int dev = 0;
        if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kMaxDevices) return kFallback;
        if (!ts.stream[dev] && hipStreamCreateWithFlags(&ts.stream[dev], hipStreamNonBlocking) != hipSuccess) {
            ts.stream[dev] = nullptr;
            (void)hipGetLastError();
            return kFallback;
        }
        if (!ts.done[dev] && hipEventCreateWithFlags(&ts.done[dev], hipEventDisableTiming) != hipSuccess) {
            ts.done[dev] = nullptr;  // (the call then waits in hipStreamSynchronize)
            (void)hipGetLastError();
        }
        hipStream_t stream = ts.stream[dev];
        // through the registry: a range sharing a page with any live registration
        // (another thread's call) is refused, and the call falls back to the staged path
        // Locked with hsa_amd_memory_lock, like the batched path's units: one locking
        // mechanism in the process.  (Round 5: zero-copy calls registered with
        // hipHostRegister right after batched calls had locked and unlocked pages
        // of the same units with hsa_amd_memory_lock faulted once in the GPU suite,
        // tests/test_gpu_parity.py::test_lone_caller_copy_fanout; the HSA runtime
        // keeps unlocked ranges cached, and the two layers' mappings of one page
        // are the overlap hazard of DESIGN.md §5.2 again.)
        const auto rs = pinned ? std::vector<std::pair<uintptr_t, uintptr_t>>{} : ranges(op, len);
        if (!pinned && !units_unknown(op, len)) return kFallback;  // someone else registered a unit: staged
        std::vector<uintptr_t> dev_lo(rs.size(), 0);
        Registrar& reg = Registrar::get();
        size_t locked = 0;
        for (; locked < rs.size(); ++locked)
            if (!reg.acquire(rs[locked].first, rs[locked].second, dev, &dev_lo[locked])) break;
        int rc = kFallback;
        if (locked == rs.size()) {
            ApplyParams p;
            p.len = len;
            p.stripes = 1;
            p.cols = op.cols;
            p.rows = op.rows;
            std::memcpy(p.coef, op.coef, sizeof(p.coef));
            PinnedPool& pool = PinnedPool::get();
            auto device_of = [&](const void* x, size_t n) -> const void* {  // inside the pool or one locked range
                const uintptr_t a = reinterpret_cast<uintptr_t>(x);
                if (pinned || pool.pinned(x, n)) return reinterpret_cast<const void*>(pool.device_addr(x));
                for (size_t i = 0; i < rs.size(); ++i)
                    if (a >= rs[i].first && a < rs[i].second)
                        return reinterpret_cast<const void*>(dev_lo[i] + (a - rs[i].first));
                return nullptr;
            };
            bool ok = true;
            for (int j = 0; j < op.cols && ok; ++j) {
                const void* d = nullptr;
                if (op.in[j] && (!op.lens || op.lens[j])) ok = (d = device_of(op.in[j], input_span(op, j, len))) != nullptr;
                p.src[j] = col(d, 0, 0);
            }
            for (int q = 0; q < op.rows && ok; ++q) {
                const void* d = device_of(op.out[q], len);
                ok = d != nullptr;
                p.dst[q] = col(d, 0, 0);
            }
            if (op.lens) {  // one stripe: the per-column content lengths ride in the kernel arguments
                p.padded = true;
                for (int j = 0; j < op.cols; ++j) p.clen[j] = static_cast<uint32_t>(std::min(op.lens[j], len));
            }
            if (ok) {
                hipError_t e = kern::launch_apply(p, stream);
                // Whatever was enqueued finishes before the pages are unregistered,
                // also when a later launch of the call failed.
                hipError_t w = ts.done[dev] ? hipEventRecord(ts.done[dev], stream) : hipErrorInvalidHandle;
                w = w == hipSuccess ? wait_sleeping(ts.done[dev]) : hipStreamSynchronize(stream);
                if (e == hipSuccess) e = w;
                // A shape the single launch does not take (hipErrorInvalidValue is
                // returned before the kernels run: a wide padded update past 2^31
                // bytes, say) goes to the staged path, which splits it; the outputs
                // are rewritten there in full.  Any other error is the call's.
                rc = e == hipErrorInvalidValue ? kFallback : map_hip(e);
            }
        }
        for (size_t i = 0; i < locked; ++i) reg.release(rs[i].first);  // (the stream is synchronised above)
        return rc;
    }
};

// Host-path calls in flight per device (run_host), for the zero-copy policy.
std::atomic<int> g_in_flight[kMaxDevices];
// The last calling thread per device, and when a different thread last called:
// a caller is alone when no other thread has called for kAloneNs.  Two threads
// calling back to back are each momentarily alone between calls, and a
// zero-copy call then competes with the other's batched DMA (2 callers: 31.5-
// 34.7 GiB/s against 36.0-36.2 batched, profiles/r03/zerocopy_hostpath.txt).
std::atomic<uint64_t> g_last_caller[kMaxDevices];
std::atomic<int64_t> g_other_caller_ns[kMaxDevices];
constexpr int64_t kAloneNs = 20'000'000;

bool lone_caller(int dev)
{
    static thread_local const uint64_t me = std::hash<std::thread::id>{}(std::this_thread::get_id()) | 1u;
    const int64_t now = std::chrono::duration_cast<std::chrono::nanoseconds>(
                            std::chrono::steady_clock::now().time_since_epoch()).count();
    const uint64_t prev = g_last_caller[dev].exchange(me);
    if (prev != me && prev != 0) g_other_caller_ns[dev].store(now);  // 0: no thread has called before
    return now - g_other_caller_ns[dev].load() > kAloneNs;
}
// elect_ec_host_path_stats: zero-copy calls, zero-copy fallbacks, batched (staged), per-thread
// engine, batched direct (page-locked caller buffers, no staging copies), batched direct on
// units registered for the call (ELECT_EC_REGISTER=1), registration attempts that fell back
// to staging (no free slot, or a range refused), failed unregistrations (entry 7 is read from
// g_unregister_failures), CPU ns registering / unregistering / issuing batches (8-10).
constexpr int kStats = 19;
std::atomic<uint64_t> g_stats[kStats];

}  // namespace

int run_host(const HostOp& op, size_t len)
{
    if (len == 0) return ELECT_EC_OK;  // JEC/ErasureEncoder.java:41-44, JEC/ErasureDecoder.java:36-38
    const int64_t t_enter = now_ns();
    for (int j = 0; j < op.cols; ++j) {
        if (op.lens && op.lens[j] > len) return ELECT_EC_EINVAL;
        if (!op.in[j] && !(op.lens && op.lens[j] == 0)) return ELECT_EC_EINVAL;
    }
    for (int r = 0; r < op.rows; ++r)
        if (!op.out[r]) return ELECT_EC_EINVAL;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return ELECT_EC_ENODEV;
    int dev = 0;
    int rc = ELECT_EC_ENOMEM;
    try {
        rc = host_device(ndev, &dev);  // (parses ELECT_EC_DEVICES on first use)
    } catch (...) {
    }
    if (rc != ELECT_EC_OK) return rc;
    if (dev < 0 || dev >= kMaxDevices || dev >= ndev) return ELECT_EC_ENODEV;
    int prev = 0;
    hipError_t e = hipGetDevice(&prev);
    if (e == hipSuccess && prev != dev) e = hipSetDevice(dev);
    if (e != hipSuccess) return map_hip(e);
    struct InFlight {
        std::atomic<int>& n;
        const int now;
        explicit InFlight(std::atomic<int>& c) : n(c), now(c.fetch_add(1) + 1) {}
        ~InFlight() { n.fetch_sub(1); }
    } in_flight(g_in_flight[dev]);
    try {  // nothing may unwind into the JVM: allocation failures become status codes
        rc = Batcher::kFallback;
        // units in page-locked pool buffers (elect_ec_host_alloc) move by kernels with no
        // staging copy (batched); any other lone caller's may be page-locked for the call
        const bool direct = direct_op(op, len);
        if (ZeroCopy::eligible(op, len, in_flight.now, lone_caller(dev))) {
            rc = ZeroCopy::run(op, len, direct);
            g_stats[rc == ZeroCopy::kFallback ? 1 : 0].fetch_add(1);
            if (rc == ZeroCopy::kFallback) rc = Batcher::kFallback;
            else goto done;
        }
        if (batch_config().enabled.load() == 1) {
            Batcher* b = batcher(dev);
            DirectPlan plan;
            bool registered = false;
            if (direct) {  // pool units: all of each straight from / to the pool buffer
                PinnedPool& pool = PinnedPool::get();
                plan.direct = true;
                for (int j = 0; j < op.cols; ++j) {
                    plan.in_hi[j] = op.lens ? op.lens[j] : len;
                    plan.in_dev[j] = plan.in_hi[j] ? pool.device_addr(op.in[j]) : 0;
                }
                for (int r = 0; r < op.rows; ++r) {
                    plan.out_hi[r] = len;
                    plan.out_dev[r] = pool.device_addr(op.out[r]);
                }
            } else if (b && RegisterPath::mode() == 1 && len >= RegisterPath::kMinBytes) {
                registered = RegisterPath::plan(op, len, dev, plan);
                if (!registered) g_stats[6].fetch_add(1);
            }
            t_phase_mark = now_ns();
            add_phase(0, t_enter, t_phase_mark);
            struct Release {  // the registrations outlive the call's batch, not the call
                DirectPlan& p;
                ~Release()
                {
                    RegisterPath::release(p);
                    add_phase(6, t_phase_mark, now_ns());
                }
            } release{plan};
            rc = b ? b->submit(op, len, &plan) : ELECT_EC_ENOMEM;
            if (rc != Batcher::kFallback) g_stats[registered ? 5 : direct ? 4 : 2].fetch_add(1);
        }
        if (rc == Batcher::kFallback) {
            if (!t_engines[dev]) t_engines[dev].reset(new (std::nothrow) HostEngine(dev));
            rc = t_engines[dev] ? t_engines[dev]->run(op, len) : ELECT_EC_ENOMEM;
            g_stats[3].fetch_add(1);
        }
    } catch (const std::bad_alloc&) {
        rc = ELECT_EC_ENOMEM;
    } catch (...) {  // std::system_error: a thread could not be started
        rc = ELECT_EC_ENOMEM;
    }
done:
    if (prev != dev) (void)hipSetDevice(prev);  // the caller's current device is left as it was
    return rc;
}

int host_device_map(const int* devices, const int* nodes, int ndev, const int* thread_nodes, int nthreads, int* out)
{
    if (ndev <= 0 || nthreads < 0 || !devices || !nodes || (nthreads > 0 && (!thread_nodes || !out)))
        return ELECT_EC_EINVAL;
    try {
        std::vector<unsigned> load(static_cast<size_t>(ndev), 0);
        for (int t = 0; t < nthreads; ++t) out[t] = numa_pick(devices, nodes, ndev, thread_nodes[t], load.data());
    } catch (const std::bad_alloc&) {
        return ELECT_EC_ENOMEM;
    }
    return ELECT_EC_OK;
}

int set_host_devices(const int* devices, int n)
{
    if (n < 0 || (n > 0 && !devices)) return ELECT_EC_EINVAL;
    int ndev = 0;
    if (n > 0 && (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0)) return ELECT_EC_ENODEV;
    for (int i = 0; i < n; ++i)
        if (devices[i] < 0 || devices[i] >= ndev || devices[i] >= kMaxDevices) return ELECT_EC_EINVAL;
    DevicePolicy& p = policy();
    std::lock_guard<std::mutex> lock(p.mu);
    p.env_read = true;  // an explicit list overrides the environment
    try {
        p.devices.assign(devices, devices + n);
        read_nodes(p);
    } catch (const std::bad_alloc&) {
        p.devices.clear();
        p.nodes.clear();
        p.load.clear();
        return ELECT_EC_ENOMEM;
    }
    p.generation++;  // threads pick a device again on their next call
    return ELECT_EC_OK;
}

int host_path_stats(uint64_t* out, int n)
{
    if (n < 0 || (n > 0 && !out)) return ELECT_EC_EINVAL;
    const int w = n < kStats ? n : kStats;
    g_stats[7].store(g_unregister_failures.load());
    g_stats[8].store(g_register_cpu_ns.load());
    g_stats[9].store(g_unregister_cpu_ns.load());
    g_stats[10].store(g_issue_cpu_ns.load());
    for (int i = 0; i < 7; ++i) g_stats[11 + i].store(g_phase_ns[i].load());
    g_stats[18].store(g_batches.load());
    for (int i = 0; i < w; ++i) out[i] = g_stats[i].load();
    return w;
}

int host_alloc(size_t bytes, void** out)
{
    if (!out) return ELECT_EC_EINVAL;
    *out = nullptr;
    if (bytes == 0) return ELECT_EC_EINVAL;
    try {
        *out = PinnedPool::get().alloc(bytes);
    } catch (...) {
        *out = nullptr;
    }
    return *out ? ELECT_EC_OK : ELECT_EC_ENOMEM;
}

int host_free(void* ptr)
{
    if (!ptr) return ELECT_EC_OK;
    try {
        return PinnedPool::get().free(ptr) ? ELECT_EC_OK : ELECT_EC_EINVAL;
    } catch (...) {
        return ELECT_EC_ENOMEM;
    }
}

int host_pinned(const void* ptr, size_t bytes)
{
    return PinnedPool::get().pinned(ptr, bytes) ? 1 : 0;
}

int set_batching(int enable, unsigned window_us, size_t arena_bytes)
{
    if (enable < 0 || (enable && arena_bytes < (size_t{1} << 20))) return ELECT_EC_EINVAL;
    BatchConfig& c = batch_config();
    c.window_us = window_us;
    if (arena_bytes) c.arena_bytes = arena_bytes;
    c.enabled = enable ? 1 : 0;
    return ELECT_EC_OK;
}

}  // namespace host
}  // namespace elect
