// host_stress.cpp — concurrency stress of the host-memory C ABI under host-side
// AddressSanitizer + UndefinedBehaviorSanitizer (dev tooling; tools/sanitize/run.sh).
//
// ELECT calls the coder from up to concurrent_ec (64) threads (conf/elect.yaml:598);
// the reference is safe only with a coder per task (EC/NativeRSEncoder.c:25-29).
// Here T threads share ONE coder and mix every host entry point (encode, encode_ex
// padded/hashed, encode_update_ex, decode_ex with prefix lengths) at random
// lengths, with cross-thread batching on, then off, then on units in the engine's
// page-locked pool (direct batches).  Each result is checked by an
// independent route: decode(encode(x)) == x, update == re-encode, and the JDK
// ByteBuffer.hashCode loop written out here.  Exit 0 = no mismatch (and, under
// ASan/UBSan, no memory or UB error in the host code: batcher arenas, staging,
// per-slot lengths and hashes).
#include <atomic>
#include <cstdlib>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <random>
#include <thread>
#include <vector>

#include <hip/hip_runtime_api.h>

#include "elect_ec.h"

static std::atomic<int> g_fail{0};

static int32_t java_hash(const uint8_t* p, size_t n)
{
    uint32_t h = 1;
    for (size_t i = n; i-- > 0;) h = 31u * h + static_cast<uint32_t>(static_cast<int32_t>(static_cast<int8_t>(p[i])));
    return static_cast<int32_t>(h);
}

// A byte buffer in ordinary memory or in the engine's page-locked pool
// (elect_ec_host_alloc): calls whose every unit is pooled run as direct batches,
// moved by DMA with no staging copies.
struct Buf {
    uint8_t* p = nullptr;
    size_t n = 0;
    bool pool = false;
    Buf() = default;
    Buf(size_t len, bool pooled, uint8_t fill = 0) { make(len, pooled, fill); }
    Buf(const Buf& o)
    {
        make(o.n, o.pool, 0);
        std::memcpy(p, o.p, n);
    }
    Buf& operator=(const Buf& o)
    {
        if (this != &o) {
            drop();
            make(o.n, o.pool, 0);
            std::memcpy(p, o.p, n);
        }
        return *this;
    }
    ~Buf() { drop(); }
    void make(size_t len, bool pooled, uint8_t fill)
    {
        n = len;
        pool = pooled;
        void* q = nullptr;
        if (pooled ? elect_ec_host_alloc(len ? len : 1, &q) != 0 : !(q = std::malloc(len ? len : 1))) std::abort();
        p = static_cast<uint8_t*>(q);
        std::memset(p, fill, n);
    }
    void drop()
    {
        if (!p) return;
        if (pool)
            (void)elect_ec_host_free(p);
        else
            std::free(p);
        p = nullptr;
    }
    uint8_t* data() { return p; }
    const uint8_t* data() const { return p; }
    uint8_t* begin() { return p; }
    uint8_t* end() { return p + n; }
    uint8_t& operator[](size_t i) { return p[i]; }
    bool operator==(const Buf& o) const { return n == o.n && std::memcmp(p, o.p, n) == 0; }
};

#define CHECK(cond, ...)                                \
    do {                                                \
        if (!(cond)) {                                  \
            std::fprintf(stderr, __VA_ARGS__);          \
            std::fprintf(stderr, "  [%s:%d]\n", __FILE__, __LINE__); \
            g_fail++;                                   \
        }                                               \
    } while (0)

static void worker(const elect_ec_coder* c, int k, int m, int tid, int iters, size_t big = 0, bool pooled = false)
{
    std::mt19937_64 rng(1000 + tid);
    auto rnd = [&](size_t lo, size_t hi) { return lo + rng() % (hi - lo + 1); };
    for (int it = 0; it < iters; ++it) {
        // big: units of big/3..big bytes, so that a lone caller's copies fan out (CopyPool)
        const size_t L = big ? rnd(big / 3, big) : rng() % 4 == 0 ? rnd(1, 64) : rnd(1000, 300000);
        std::vector<Buf> d(k, Buf(L, pooled)), p(m, Buf(L, pooled));
        std::vector<size_t> lens(k);
        for (int j = 0; j < k; ++j) {
            for (auto& b : d[j]) b = static_cast<uint8_t>(rng());
            lens[j] = rng() % 3 == 0 ? L : rnd(0, L);
        }
        const bool padded = rng() & 1, hashed = rng() & 1;
        std::vector<const uint8_t*> in(k);
        std::vector<uint8_t*> out(m);
        for (int j = 0; j < k; ++j) in[j] = d[j].data();
        for (int r = 0; r < m; ++r) out[r] = p[r].data();
        int32_t hs[16] = {};
        int st = elect_ec_encode_ex(c, in.data(), padded ? lens.data() : nullptr, out.data(), L, hashed ? hs : nullptr);
        CHECK(st == 0, "t%d it%d encode_ex status %d\n", tid, it, st);
        if (padded)  // the zero-filled stripe the parity belongs to
            for (int j = 0; j < k; ++j) std::memset(d[j].data() + lens[j], 0, L - lens[j]);
        for (int r = 0; hashed && r < m; ++r)
            CHECK(hs[r] == java_hash(p[r].data(), L), "t%d it%d hash row %d (L=%zu padded=%d)\n", tid, it, r, L,
              int(padded));

        // degraded read of a random data unit from the others + parity 0, a random prefix
        const int e = static_cast<int>(rng() % k);
        std::vector<int> di;
        for (int j = 0; j < k; ++j)
            if (j != e) di.push_back(j);
        di.push_back(k);
        std::vector<const uint8_t*> sv;
        std::vector<size_t> sl;
        for (int u : di) {
            sv.push_back(u < k ? d[u].data() : p[0].data());
            sl.push_back(u < k && padded ? lens[u] : L);
        }
        const size_t pre = rnd(0, L);
        Buf rebuilt(L + 1, pooled, 0xA5);
        uint8_t* ro[1] = {rebuilt.data()};
        st = elect_ec_decode_ex(c, sv.data(), padded ? sl.data() : nullptr, di.data(), &e, 1, ro, pre,
                                ELECT_EC_DECODE_COMPAT);
        CHECK(st == 0, "t%d it%d decode_ex status %d\n", tid, it, st);
        CHECK(std::memcmp(rebuilt.data(), d[e].data(), pre) == 0 && rebuilt[pre] == 0xA5,
              "t%d it%d decode mismatch (L=%zu pre=%zu)\n", tid, it, L, pre);

        // parity update of unit t in place, then compare with a fresh encode
        const int t = static_cast<int>(rng() % k);
        Buf nw(L, pooled);
        for (auto& b : nw) b = static_cast<uint8_t>(rng());
        const size_t ul[2] = {padded ? lens[t] : L, padded ? rnd(0, L) : L};
        std::vector<const uint8_t*> ui = {d[t].data(), nw.data()};
        for (int r = 0; r < m; ++r) ui.push_back(p[r].data());
        int32_t hu[16] = {};
        st = elect_ec_encode_update_ex(c, ui.data(), padded ? ul : nullptr, t, out.data(), L, hashed ? hu : nullptr);
        CHECK(st == 0, "t%d it%d update_ex status %d\n", tid, it, st);
        std::memset(nw.data() + ul[1], 0, L - ul[1]);
        d[t] = nw;
        std::vector<Buf> q(m, Buf(L, pooled));
        std::vector<uint8_t*> qo(m);
        for (int r = 0; r < m; ++r) qo[r] = q[r].data();
        for (int j = 0; j < k; ++j) in[j] = d[j].data();
        st = elect_ec_encode(c, in.data(), qo.data(), L);
        CHECK(st == 0, "t%d it%d encode status %d\n", tid, it, st);
        for (int r = 0; r < m; ++r) {
            CHECK(p[r] == q[r], "t%d it%d update row %d mismatch\n", tid, it, r);
            CHECK(!hashed || hu[r] == java_hash(q[r].data(), L), "t%d it%d update hash row %d (L=%zu padded=%d)\n",
                  tid, it, r, L, int(padded));
        }
    }
}

// The device-resident API from many threads, each on its own stream: hashed and
// padded batch encodes checked against the host path and the JDK hash loop.
static void device_worker(const elect_ec_coder* c, int k, int m, int tid, int iters)
{
    std::mt19937_64 rng(5000 + tid);
    auto rnd = [&](size_t lo, size_t hi) { return lo + rng() % (hi - lo + 1); };
    hipStream_t st = nullptr;
    if (hipStreamCreateWithFlags(&st, hipStreamNonBlocking) != hipSuccess) {
        g_fail++;
        return;
    }
    for (int it = 0; it < iters; ++it) {
        const size_t B = rnd(1, 6), L = rng() % 3 == 0 ? rnd(1, 2000) : rnd(1024, 150000);
        const bool padded = rng() & 1;
        const size_t n = static_cast<size_t>(k + m);
        std::vector<uint8_t> h(B * n * L);
        for (auto& b : h) b = static_cast<uint8_t>(rng());
        std::vector<uint32_t> lens(B * k);
        for (auto& x : lens) x = static_cast<uint32_t>(rng() % 3 == 0 ? L : rnd(0, L));
        uint8_t* d = nullptr;
        uint32_t* dl = nullptr;
        int32_t* dh = nullptr;
        bool ok = hipMalloc(reinterpret_cast<void**>(&d), h.size()) == hipSuccess &&
                  hipMalloc(reinterpret_cast<void**>(&dl), lens.size() * 4) == hipSuccess &&
                  hipMalloc(reinterpret_cast<void**>(&dh), B * m * 4) == hipSuccess &&
                  hipMemcpyAsync(d, h.data(), h.size(), hipMemcpyHostToDevice, st) == hipSuccess &&
                  hipMemcpyAsync(dl, lens.data(), lens.size() * 4, hipMemcpyHostToDevice, st) == hipSuccess;
        CHECK(ok, "t%d it%d device setup\n", tid, it);
        elect_ec_shards data = {d, n * L, L}, par = {d + k * L, n * L, L};
        const int s = elect_ec_encode_batch_ex(c, L, B, data, padded ? dl : nullptr, par, dh, st);
        CHECK(s == 0, "t%d it%d encode_batch_ex status %d\n", tid, it, s);
        std::vector<uint8_t> got(h.size());
        std::vector<int32_t> gh(B * m);
        ok = hipMemcpyAsync(got.data(), d, got.size(), hipMemcpyDeviceToHost, st) == hipSuccess &&
             hipMemcpyAsync(gh.data(), dh, gh.size() * 4, hipMemcpyDeviceToHost, st) == hipSuccess &&
             hipStreamSynchronize(st) == hipSuccess;
        CHECK(ok, "t%d it%d device readback\n", tid, it);
        for (size_t b = 0; b < B; ++b) {
            std::vector<const uint8_t*> in(k);
            std::vector<size_t> hl(k);
            for (int j = 0; j < k; ++j) {
                in[j] = h.data() + (b * n + j) * L;
                hl[j] = padded ? lens[b * k + j] : L;
            }
            std::vector<std::vector<uint8_t>> want(m, std::vector<uint8_t>(L));
            std::vector<uint8_t*> wo(m);
            for (int r = 0; r < m; ++r) wo[r] = want[r].data();
            CHECK(elect_ec_encode_ex(c, in.data(), hl.data(), wo.data(), L, nullptr) == 0, "host encode\n");
            for (int r = 0; r < m; ++r) {
                CHECK(std::memcmp(got.data() + (b * n + k + r) * L, want[r].data(), L) == 0,
                      "t%d it%d device parity s%zu r%d (L=%zu)\n", tid, it, b, r, L);
                CHECK(gh[b * m + r] == java_hash(want[r].data(), L), "t%d it%d device hash s%zu r%d (L=%zu)\n",
                      tid, it, b, r, L);
            }
        }
        (void)hipFree(d);
        (void)hipFree(dl);
        (void)hipFree(dh);
    }
    (void)hipStreamDestroy(st);
}

int main(int argc, char** argv)
{
    const int threads = argc > 1 ? std::atoi(argv[1]) : 24;
    const int iters = argc > 2 ? std::atoi(argv[2]) : 12;
    int ndev = 0;
    if (elect_ec_device_count(&ndev) != 0 || ndev == 0) {
        std::fprintf(stderr, "no device\n");
        return 2;
    }
    elect_ec_coder* c = nullptr;
    if (elect_ec_coder_create(4, 2, &c) != 0) return 2;
    const int first = argc > 3 ? std::atoi(argv[3]) : 1;  // 1: batching on, then off; 0: off only
    for (int batching : {1, 0}) {
        if (batching > first) continue;
        elect_ec_set_batching(batching, 0, size_t{8} << 20);  // small arenas: batches close often
        std::vector<std::thread> th;
        for (int t = 0; t < threads; ++t) th.emplace_back(worker, c, 4, 2, t + 100 * batching, iters, size_t{0}, false);
        for (auto& x : th) x.join();
        std::printf("batching=%d: %d threads x %d iterations, failures so far %d\n", batching, threads, iters,
                    g_fail.load());
    }
    {  // one and two callers on multi-MB stripes: the copy fan-out, and two callers racing for it
        elect_ec_set_batching(1, 0, size_t{8} << 20);
        for (int n : {1, 2}) {
            std::vector<std::thread> th;
            for (int t = 0; t < n; ++t) th.emplace_back(worker, c, 4, 2, t + 200 + 10 * n, iters, size_t{1900000}, false);
            for (auto& x : th) x.join();
        }
        std::printf("lone callers: 1 and 2 threads x %d iterations, failures so far %d\n", iters, g_fail.load());
    }
    {  // every unit in page-locked pool buffers: direct batches (no staging copies), pool reuse across threads
        elect_ec_set_batching(1, 0, size_t{8} << 20);
        std::vector<std::thread> th;
        for (int t = 0; t < threads; ++t) th.emplace_back(worker, c, 4, 2, t + 300, iters, size_t{0}, true);
        for (auto& x : th) x.join();
        uint64_t st[5] = {};
        elect_ec_host_path_stats(st, 5);
        std::printf("pool buffers: %d threads x %d iterations, direct calls %llu, failures so far %d\n", threads, iters,
                    static_cast<unsigned long long>(st[4]), g_fail.load());
        CHECK(st[4] > 0, "no call took the direct path\n");
    }
    {  // many callers on multi-MB pageable units: interior pages locked per call (round 5), ends staged,
       // gather / scatter kernels; the registry's refcounts and exact-base releases under concurrency
        elect_ec_set_batching(1, 0, size_t{64} << 20);
        std::vector<std::thread> th;
        for (int t = 0; t < threads; ++t) th.emplace_back(worker, c, 4, 2, t + 400, iters, size_t{2400000}, false);
        for (auto& x : th) x.join();
        uint64_t st[8] = {};
        elect_ec_host_path_stats(st, 8);
        std::printf("locked pageable units: %d threads x %d iterations, locked calls %llu, unlock failures %llu, "
                    "failures so far %d\n", threads, iters, static_cast<unsigned long long>(st[5]),
                    static_cast<unsigned long long>(st[7]), g_fail.load());
        CHECK(st[5] > 0, "no call took the locked path\n");
        CHECK(st[7] == 0, "an unlock failed\n");
    }
    {
        std::vector<std::thread> th;
        for (int t = 0; t < threads; ++t) th.emplace_back(device_worker, c, 4, 2, t, iters);
        for (auto& x : th) x.join();
        std::printf("device API: %d threads x %d iterations, failures so far %d\n", threads, iters, g_fail.load());
    }
    elect_ec_coder_destroy(c);
    std::fflush(stdout);
    std::fflush(stderr);
    std::_Exit(g_fail.load() == 0 ? 0 : 1);  // skip static teardown (ASan's device allocator vs HIP's at exit)
}
