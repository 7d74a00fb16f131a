// tune_apply.hip — standalone variant sweep for the GF(2^8) batch kernel
// (dev tooling, not product).  Times kernel variants on the BASELINE shapes in
// ONE process with hipEvents (interleaved rounds, median), checks each against
// the reference variant byte for byte, and reports GB/s of algorithmic traffic
// ((cols + rows) * L per stripe) against the 8 TB/s HBM peak.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/tune/tune_apply.hip -o tune_apply
//   ./tune_apply
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../elect_amd/csrc/gf256.hpp"

#define CK(x)                                                                                   \
    do {                                                                                        \
        hipError_t e_ = (x);                                                                    \
        if (e_ != hipSuccess) {                                                                 \
            std::fprintf(stderr, "%s:%d %s -> %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            std::exit(3);                                                                       \
        }                                                                                       \
    } while (0)

using elect::gf::PermTable;
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint4 nt_load(const uint4* p)
{
    const u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
    return make_uint4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ void nt_store(const uint4& v, uint4* p)
{
    u32x4 w = {v.x, v.y, v.z, v.w};
    __builtin_nontemporal_store(w, reinterpret_cast<u32x4*>(p));
}

template <int K, int R>
struct Args {
    const uint8_t* sp[K];
    uint64_t ss[K];
    uint8_t* dp[R];
    uint64_t ds[R];
    uint32_t segs, total, magic, shift;
    PermTable tab[R][K];
};

__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c)
{
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}
__device__ __forceinline__ uint32_t lane_word(const uint4& v, int w)
{
    return w == 0 ? v.x : w == 1 ? v.y : w == 2 ? v.z : v.w;
}
__device__ __forceinline__ void set_word(uint4& v, int w, uint32_t x)
{
    if (w == 0) v.x = x;
    else if (w == 1) v.y = x;
    else if (w == 2) v.z = x;
    else v.w = x;
}

enum Mode { kGF = 0, kXor = 1, kHashAtomic = 2, kHashScratch = 3, kHashLocal = 4 };

__device__ __forceinline__ uint32_t dpow31(uint64_t e)
{
    uint32_t r = 1, b = 31;
    for (; e; e >>= 1, b *= b)
        if (e & 1) r *= b;
    return r;
}
__device__ __forceinline__ uint32_t horner31(const uint4& v)
{
    uint32_t h = 0;
#pragma unroll
    for (int w = 3; w >= 0; --w) {
        const int x = static_cast<int>(lane_word(v, w));
        const int lo = __builtin_amdgcn_sdot4(x, 0x00001F01, 0, false);
        const int hi = __builtin_amdgcn_sdot4(x, 0x1F010000, 0, false);
        const uint32_t d = static_cast<uint32_t>(__mul24(hi, 961) + lo);
        h = w == 3 ? d : h * 923521u + d;
    }
    return h;
}
__device__ __forceinline__ uint32_t wave_sum(uint32_t v)
{
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) v += static_cast<uint32_t>(__shfl_xor(static_cast<int>(v), d, 64));
    return v;
}
__device__ uint32_t* g_hash;  // set by the host before hash variants run
enum Load { kPlain = 0, kNTL = 1, kNTS = 2, kNT = 3 };

template <int K, int R, int U, int BLOCK, int MODE, int LD, bool GRIDSTRIDE, int ORDER = 0, bool ADJ = false>
__global__ __launch_bounds__(BLOCK) void kern(const Args<K, R> a)
{
    // ORDER 2: column-outer with the byte-shuffle tables staged in LDS
    // (8 dwords per coefficient: t0_lo t0_hi t1_lo t1_hi t2 pad pad pad)
    __shared__ __attribute__((aligned(16))) uint32_t tl[ORDER == 2 ? R * K * 8 : 4];
    if (ORDER == 2) {
        for (int i = threadIdx.x; i < R * K; i += BLOCK) {
            const PermTable& t = a.tab[i / K][i % K];
            tl[i * 8 + 0] = t.t0_lo; tl[i * 8 + 1] = t.t0_hi; tl[i * 8 + 2] = t.t1_lo;
            tl[i * 8 + 3] = t.t1_hi; tl[i * 8 + 4] = t.t2;
        }
        __syncthreads();
    }
    const uint32_t step = GRIDSTRIDE ? gridDim.x * (BLOCK * U) : 0;
    for (uint32_t first = blockIdx.x * (BLOCK * U) + threadIdx.x; first < a.total;
         first += GRIDSTRIDE ? step : a.total) {
        uint4 x[U][K];
        uint32_t stripe[U];
        uint64_t off[U];
        bool live[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            // ADJ: a wave's U loads per column cover U KiB back to back; else BLOCK*16 B apart
            const uint32_t idx = ADJ ? blockIdx.x * (BLOCK * U) + (threadIdx.x >> 6) * (64 * U) + u * 64 + (threadIdx.x & 63)
                                     : first + u * BLOCK;
            const uint32_t s = static_cast<uint32_t>((static_cast<uint64_t>(idx) * a.magic) >> a.shift);
            stripe[u] = s;
            off[u] = static_cast<uint64_t>(idx - s * a.segs) * 16;
            live[u] = idx < a.total;
            if (live[u]) {
#pragma unroll
                for (int j = 0; j < K; ++j) {
                    const uint4* p = reinterpret_cast<const uint4*>(a.sp[j] + s * a.ss[j] + off[u]);
                    x[u][j] = (LD & kNTL) ? nt_load(p) : *p;
                }
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (!live[u]) continue;
            uint4 acc[R];
            if (ORDER == 2 && (MODE == kGF || MODE >= kHashAtomic)) {
#pragma unroll
                for (int j = 0; j < K; ++j) {
                    uint32_t s0[4], s1[4], s2[4];
#pragma unroll
                    for (int w = 0; w < 4; ++w) {
                        const uint32_t v0 = lane_word(x[u][j], w);
                        s0[w] = v0 & 0x07070707u;
                        s1[w] = (v0 >> 3) & 0x07070707u;
                        s2[w] = (v0 >> 6) & 0x03030303u;
                    }
#pragma unroll
                    for (int r = 0; r < R; ++r) {
                        const uint4 tq = *reinterpret_cast<const uint4*>(&tl[(r * K + j) * 8]);
                        const uint32_t t2 = tl[(r * K + j) * 8 + 4];
#pragma unroll
                        for (int w = 0; w < 4; ++w) {
                            const uint32_t v = xor3(__builtin_amdgcn_perm(tq.y, tq.x, s0[w]),
                                                    __builtin_amdgcn_perm(tq.w, tq.z, s1[w]),
                                                    __builtin_amdgcn_perm(t2, t2, s2[w]));
                            set_word(acc[r], w, j == 0 ? v : (lane_word(acc[r], w) ^ v));
                        }
                    }
                }
            } else if (ORDER == 1 && MODE == kGF) {
                // column-outer: selectors of one column, then every row, then every dword
#pragma unroll
                for (int j = 0; j < K; ++j) {
                    uint32_t s0[4], s1[4], s2[4];
#pragma unroll
                    for (int w = 0; w < 4; ++w) {
                        const uint32_t v0 = lane_word(x[u][j], w);
                        s0[w] = v0 & 0x07070707u;
                        s1[w] = (v0 >> 3) & 0x07070707u;
                        s2[w] = (v0 >> 6) & 0x03030303u;
                    }
#pragma unroll
                    for (int r = 0; r < R; ++r) {
                        const PermTable& t = a.tab[r][j];
#pragma unroll
                        for (int w = 0; w < 4; ++w) {
                            const uint32_t v = xor3(__builtin_amdgcn_perm(t.t0_hi, t.t0_lo, s0[w]),
                                                    __builtin_amdgcn_perm(t.t1_hi, t.t1_lo, s1[w]),
                                                    __builtin_amdgcn_perm(t.t2, t.t2, s2[w]));
                            set_word(acc[r], w, j == 0 ? v : (lane_word(acc[r], w) ^ v));
                        }
                    }
                }
            } else
#pragma unroll
            for (int w = 0; w < 4; ++w) {
                uint32_t ar[R];
#pragma unroll
                for (int j = 0; j < K; ++j) {
                    const uint32_t v0 = lane_word(x[u][j], w);
                    if (MODE == kXor) {
#pragma unroll
                        for (int r = 0; r < R; ++r) ar[r] = j == 0 ? v0 + r : (ar[r] ^ v0);
                    } else {
                        const uint32_t s0 = v0 & 0x07070707u, s1 = (v0 >> 3) & 0x07070707u,
                                       s2 = (v0 >> 6) & 0x03030303u;
#pragma unroll
                        for (int r = 0; r < R; ++r) {
                            const PermTable& t = a.tab[r][j];
                            const uint32_t v = xor3(__builtin_amdgcn_perm(t.t0_hi, t.t0_lo, s0),
                                                    __builtin_amdgcn_perm(t.t1_hi, t.t1_lo, s1),
                                                    __builtin_amdgcn_perm(t.t2, t.t2, s2));
                            ar[r] = j == 0 ? v : (ar[r] ^ v);
                        }
                    }
                }
#pragma unroll
                for (int r = 0; r < R; ++r) set_word(acc[r], w, ar[r]);
            }
#pragma unroll
            for (int r = 0; r < R; ++r) {
                uint4* p = reinterpret_cast<uint4*>(a.dp[r] + stripe[u] * a.ds[r] + off[u]);
                if (LD & kNTS) nt_store(acc[r], p);
                else *p = acc[r];
            }
            if (MODE >= kHashAtomic) {
                const uint32_t idx = first + u * BLOCK;
                const uint32_t f = __builtin_amdgcn_readfirstlane(idx);
                const uint32_t s0 = static_cast<uint32_t>((static_cast<uint64_t>(f) * a.magic) >> a.shift);
                const uint32_t seg0 = f - s0 * a.segs;
                const uint32_t q = dpow31(16u * (threadIdx.x & 63u)) * dpow31(static_cast<uint64_t>(seg0) * 16);
#pragma unroll
                for (int r = 0; r < R; ++r) {
                    const uint32_t hv = horner31(acc[r]) * q;
                    if (MODE == kHashLocal) {
                        if (hv == 0x12345678u) g_hash[0] = hv;  // compute only
                    } else {
                        const uint32_t sum = wave_sum(hv);
                        if ((threadIdx.x & 63u) == 0) {
                            if (MODE == kHashAtomic) atomicAdd(g_hash + static_cast<uint64_t>(stripe[u]) * R + r, sum);
                            else g_hash[(static_cast<uint64_t>(idx) >> 6) * R + r] = sum;
                        }
                    }
                }
            }
        }
        if (!GRIDSTRIDE) break;
    }
}

// Persistent, software-pipelined variant: a grid of G blocks; iteration t of
// block b covers segment block t*G + b (grid-stride, so the chip still sweeps
// memory in the one-shot kernel's order), and every lane issues the loads of
// iteration t+1 before it computes and stores iteration t.
template <int K, int R, int BLOCK>
__global__ __launch_bounds__(BLOCK) void kern_pipe(const Args<K, R> a)
{
    __shared__ __attribute__((aligned(16))) uint32_t tl[R * K * 8];
    for (int i = threadIdx.x; i < R * K; i += BLOCK) {
        const PermTable& t = a.tab[i / K][i % K];
        tl[i * 8 + 0] = t.t0_lo; tl[i * 8 + 1] = t.t0_hi; tl[i * 8 + 2] = t.t1_lo;
        tl[i * 8 + 3] = t.t1_hi; tl[i * 8 + 4] = t.t2;
    }
    __syncthreads();
    const uint32_t stride = gridDim.x * BLOCK;
    uint32_t idx = blockIdx.x * BLOCK + threadIdx.x;
    auto locate = [&](uint32_t i, uint32_t& st, uint64_t& off) {
        st = static_cast<uint32_t>((static_cast<uint64_t>(i) * a.magic) >> a.shift);
        off = static_cast<uint64_t>(i - st * a.segs) * 16;
    };
    uint4 cur[K], nxt[K];
    uint32_t st;
    uint64_t off;
    if (idx < a.total) {
        locate(idx, st, off);
#pragma unroll
        for (int j = 0; j < K; ++j) cur[j] = nt_load(reinterpret_cast<const uint4*>(a.sp[j] + st * a.ss[j] + off));
    }
    for (; idx < a.total; idx += stride) {
        uint32_t st_n = 0;
        uint64_t off_n = 0;
        const bool more = idx + stride < a.total;
        if (more) {
            locate(idx + stride, st_n, off_n);
#pragma unroll
            for (int j = 0; j < K; ++j)
                nxt[j] = nt_load(reinterpret_cast<const uint4*>(a.sp[j] + st_n * a.ss[j] + off_n));
        }
        uint4 acc[R];
#pragma unroll
        for (int j = 0; j < K; ++j) {
            uint32_t s0[4], s1[4], s2[4];
#pragma unroll
            for (int w = 0; w < 4; ++w) {
                const uint32_t v0 = lane_word(cur[j], w);
                s0[w] = v0 & 0x07070707u;
                s1[w] = (v0 >> 3) & 0x07070707u;
                s2[w] = (v0 >> 6) & 0x03030303u;
            }
#pragma unroll
            for (int r = 0; r < R; ++r) {
                const uint4 tq = *reinterpret_cast<const uint4*>(&tl[(r * K + j) * 8]);
                const uint32_t t2 = tl[(r * K + j) * 8 + 4];
#pragma unroll
                for (int w = 0; w < 4; ++w) {
                    const uint32_t v = xor3(__builtin_amdgcn_perm(tq.y, tq.x, s0[w]),
                                            __builtin_amdgcn_perm(tq.w, tq.z, s1[w]),
                                            __builtin_amdgcn_perm(t2, t2, s2[w]));
                    set_word(acc[r], w, j == 0 ? v : (lane_word(acc[r], w) ^ v));
                }
            }
        }
#pragma unroll
        for (int r = 0; r < R; ++r) nt_store(acc[r], reinterpret_cast<uint4*>(a.dp[r] + st * a.ds[r] + off));
        if (more) {
#pragma unroll
            for (int j = 0; j < K; ++j) cur[j] = nxt[j];
            st = st_n;
            off = off_n;
        }
    }
}

struct Magic {
    uint32_t m, p;
};
static Magic make_magic(uint32_t d)
{
    uint32_t l = 0;
    while ((uint64_t{1} << l) < d) ++l;
    const uint32_t p = 31 + l;
    return Magic{static_cast<uint32_t>(((uint64_t{1} << p) + d - 1) / d), p};
}

struct Shape {
    const char* name;
    int K, R;
    uint64_t L, B;
    int n_units;  // stripe row count (layout [B][n_units][L])
};

template <int K, int R>
struct Runner {
    Shape sh;
    uint8_t* buf = nullptr;
    uint8_t* out_ref = nullptr;
    Args<K, R> a{};
    int dev_cus = 256;

    void setup(const Shape& s)
    {
        sh = s;
        const uint64_t bytes = s.B * s.n_units * s.L;
        CK(hipMalloc(&buf, bytes));
        CK(hipMalloc(&out_ref, s.B * R * s.L));
        // fill data with a device-side pattern via host staging (random)
        std::vector<uint8_t> h(s.n_units * s.L);
        uint64_t x = 0x243F6A8885A308D3ull;
        for (uint64_t st = 0; st < s.B; st += 64) {
            for (auto& c : h) {
                x ^= x << 13; x ^= x >> 7; x ^= x << 17;
                c = static_cast<uint8_t>(x);
            }
            for (uint64_t t = st; t < std::min(s.B, st + 64); ++t)
                CK(hipMemcpy(buf + t * s.n_units * s.L, h.data(), h.size(), hipMemcpyHostToDevice));
        }
        const uint64_t segs = s.L / 16;
        a.segs = static_cast<uint32_t>(segs);
        a.total = static_cast<uint32_t>(segs * s.B);
        Magic mg = make_magic(a.segs);
        a.magic = mg.m;
        a.shift = mg.p;
        uint8_t gen[14 * 10];
        elect::gf::cauchy_generator(K, R, gen);
        for (int j = 0; j < K; ++j) {
            a.sp[j] = buf + j * s.L;
            a.ss[j] = s.n_units * s.L;
        }
        for (int r = 0; r < R; ++r) {
            a.dp[r] = buf + (K + r) * s.L;
            a.ds[r] = s.n_units * s.L;
            for (int j = 0; j < K; ++j) a.tab[r][j] = elect::gf::perm_table(gen[(K + r) * K + j]);
        }
        hipDeviceProp_t prop;
        CK(hipGetDeviceProperties(&prop, 0));
        dev_cus = prop.multiProcessorCount;
        uint32_t* hbuf = nullptr;
        CK(hipMalloc(&hbuf, (static_cast<uint64_t>(a.total) / 64 + 64) * 4 * 4 + s.B * 16));
        CK(hipMemcpyToSymbol(HIP_SYMBOL(g_hash), &hbuf, sizeof(hbuf)));
    }

    template <int U, int BLOCK, int MODE, int LD, bool GS, int ORDER = 0, bool ADJ = false>
    float time_one(int occ_blocks_per_cu, int iters)
    {
        const uint32_t per_block = BLOCK * U;
        uint32_t grid = (a.total + per_block - 1) / per_block;
        if (GS) grid = std::min<uint32_t>(grid, dev_cus * occ_blocks_per_cu);
        // TUNE_B2B=1: launches back to back (one sync at the end), as the product
        // bench issues them; default: each launch timed alone on an idle GPU.
        static const bool b2b = std::getenv("TUNE_B2B") && std::atoi(std::getenv("TUNE_B2B")) > 0;
        std::vector<hipEvent_t> ev(2 * iters);
        for (auto& e : ev) CK(hipEventCreate(&e));
        std::vector<float> ts;
        for (int i = 0; i < iters; ++i) {
            CK(hipEventRecord(ev[2 * i]));
            hipLaunchKernelGGL((kern<K, R, U, BLOCK, MODE, LD, GS, ORDER, ADJ>), dim3(grid), dim3(BLOCK), 0, 0, a);
            CK(hipEventRecord(ev[2 * i + 1]));
            if (!b2b) CK(hipEventSynchronize(ev[2 * i + 1]));
        }
        CK(hipDeviceSynchronize());
        for (int i = 0; i < iters; ++i) {
            float ms = 0;
            CK(hipEventElapsedTime(&ms, ev[2 * i], ev[2 * i + 1]));
            ts.push_back(ms);
        }
        CK(hipGetLastError());
        std::sort(ts.begin(), ts.end());
        for (auto& e : ev) CK(hipEventDestroy(e));
        return ts[ts.size() / 2];
    }

    template <int BLOCK>
    float time_pipe(int blocks_per_cu, int iters)
    {
        const uint32_t grid = std::min<uint32_t>((a.total + BLOCK - 1) / BLOCK, dev_cus * blocks_per_cu);
        std::vector<float> ts;
        hipEvent_t e0, e1;
        CK(hipEventCreate(&e0));
        CK(hipEventCreate(&e1));
        for (int i = 0; i < iters; ++i) {
            CK(hipEventRecord(e0));
            hipLaunchKernelGGL((kern_pipe<K, R, BLOCK>), dim3(grid), dim3(BLOCK), 0, 0, a);
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms = 0;
            CK(hipEventElapsedTime(&ms, e0, e1));
            ts.push_back(ms);
        }
        CK(hipGetLastError());
        CK(hipEventDestroy(e0));
        CK(hipEventDestroy(e1));
        std::sort(ts.begin(), ts.end());
        return ts[ts.size() / 2];
    }

    // copy parity region to out_ref (reference output), compare
    void snapshot()
    {
        for (int r = 0; r < R; ++r)
            CK(hipMemcpy2D(out_ref + r * sh.L, R * sh.L, buf + (K + r) * sh.L, sh.n_units * sh.L, sh.L, sh.B,
                           hipMemcpyDeviceToDevice));
    }
    bool same()
    {
        std::vector<uint8_t> a1(sh.L), b1(sh.L);
        for (uint64_t st = 0; st < sh.B; st += std::max<uint64_t>(1, sh.B / 97)) {
            for (int r = 0; r < R; ++r) {
                CK(hipMemcpy(a1.data(), out_ref + (st * R + r) * sh.L, sh.L, hipMemcpyDeviceToHost));
                CK(hipMemcpy(b1.data(), buf + (st * sh.n_units + K + r) * sh.L, sh.L, hipMemcpyDeviceToHost));
                if (std::memcmp(a1.data(), b1.data(), sh.L) != 0) return false;
            }
        }
        return true;
    }
    void teardown()
    {
        CK(hipFree(buf));
        CK(hipFree(out_ref));
    }
};

static double alg_bytes(const Shape& s) { return double(s.B) * (s.K + s.R) * s.L; }

template <int K, int R>
static void sweep(const Shape& s)
{
    Runner<K, R> rn;
    rn.setup(s);
    const int it = std::getenv("TUNE_ITERS") ? std::atoi(std::getenv("TUNE_ITERS")) : 25;
    // reference: U=2, 256, GF, plain
    rn.template time_one<2, 256, kGF, kPlain, false>(0, 3);
    rn.snapshot();
    struct Row {
        std::string name;
        float ms;
        bool ok;
        bool check;
    };
    std::vector<Row> rows;
    auto rec = [&](const char* n, float ms, bool check) { rows.push_back({n, ms, check ? rn.same() : true, check}); };
    for (int round = 0; round < 3; ++round) {
        rows.clear();
        rec("U1 b256 nt LDS-tab (product)", rn.template time_one<1, 256, kGF, kNT, false, 2>(0, it), true);
        rec("pipelined b256 x2/CU", rn.template time_pipe<256>(2, it), true);
        rec("pipelined b256 x4/CU", rn.template time_pipe<256>(4, it), true);
        rec("pipelined b256 x8/CU", rn.template time_pipe<256>(8, it), true);
        rec("pipelined b128 x8/CU", rn.template time_pipe<128>(8, it), true);
        rec("pipelined b256 x16/CU", rn.template time_pipe<256>(16, it), true);
        rec("U1 XOR-only nt both", rn.template time_one<1, 256, kXor, kNT, false>(0, it), false);
        rec("U2 XOR-only nt both adjacent", rn.template time_one<2, 256, kXor, kNT, false, 0, true>(0, it), false);
        // restore reference output for later variants' checks
        rn.template time_one<2, 256, kGF, kPlain, false>(0, 1);
    }
    std::printf("\n== %s: K=%d R=%d L=%llu B=%llu  alg %.3f GB/launch ==\n", s.name, K, R,
                (unsigned long long)s.L, (unsigned long long)s.B, alg_bytes(s) / 1e9);
    for (auto& r : rows)
        std::printf("  %-30s %8.4f ms  %7.1f GB/s  %5.1f%% of 8 TB/s  %s\n", r.name.c_str(), r.ms,
                    alg_bytes(s) / (r.ms * 1e-3) / 1e9, 100.0 * alg_bytes(s) / (r.ms * 1e-3) / 8e12,
                    r.check ? (r.ok ? "bit-exact" : "MISMATCH") : "-");
    rn.teardown();
}

__global__ void copy_kernel(const uint4* __restrict__ in, uint4* __restrict__ out, uint64_t n)
{
    const uint64_t i = blockIdx.x * 256ull + threadIdx.x;
    if (i < n) out[i] = in[i];
}

template <bool NT>
__global__ void read_kernel(const uint4* __restrict__ in, uint32_t* sink, uint64_t n)
{
    const uint64_t i = blockIdx.x * 256ull + threadIdx.x;
    if (i >= n) return;
    const uint4 v = NT ? nt_load(in + i) : in[i];
    if ((v.x ^ v.y ^ v.z ^ v.w) == 0x9E3779B9u) sink[0] = 1;  // keeps the load live
}

template <bool NT>
__global__ void write_kernel(uint4* __restrict__ out, uint64_t n)
{
    const uint64_t i = blockIdx.x * 256ull + threadIdx.x;
    if (i >= n) return;
    const uint4 v = make_uint4(static_cast<uint32_t>(i), 1, 2, 3);
    if (NT) nt_store(v, out + i);
    else out[i] = v;
}

template <bool NT>
__global__ void copy_kernel_nt(const uint4* __restrict__ in, uint4* __restrict__ out, uint64_t n)
{
    const uint64_t i = blockIdx.x * 256ull + threadIdx.x;
    if (i >= n) return;
    if (NT) nt_store(nt_load(in + i), out + i);
    else out[i] = in[i];
}

template <class F>
static float median_ms(F&& launch, int iters = 25)
{
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    std::vector<float> ts;
    for (int i = 0; i < iters; ++i) {
        CK(hipEventRecord(e0));
        launch();
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        ts.push_back(ms);
    }
    std::sort(ts.begin(), ts.end());
    return ts[ts.size() / 2];
}

static void hbm_probe()
{
    const uint64_t bytes = 2ull << 30, n = bytes / 16;
    uint8_t *a, *b;
    uint32_t* sink;
    CK(hipMalloc(&a, bytes));
    CK(hipMalloc(&b, bytes));
    CK(hipMalloc(&sink, 64));
    CK(hipMemset(a, 7, bytes));
    const dim3 g((n + 255) / 256);
    auto rep = [&](const char* name, double moved, float ms) {
        std::printf("probe %-22s %8.4f ms  %7.1f GB/s  %5.1f%% of 8 TB/s\n", name, ms, moved / (ms * 1e-3) / 1e9,
                    100.0 * moved / (ms * 1e-3) / 8e12);
    };
    for (int round = 0; round < 2; ++round) {
        rep("read plain 2 GiB", bytes, median_ms([&] { hipLaunchKernelGGL(read_kernel<false>, g, dim3(256), 0, 0, (const uint4*)a, sink, n); }));
        rep("read nt 2 GiB", bytes, median_ms([&] { hipLaunchKernelGGL(read_kernel<true>, g, dim3(256), 0, 0, (const uint4*)a, sink, n); }));
        rep("write plain 2 GiB", bytes, median_ms([&] { hipLaunchKernelGGL(write_kernel<false>, g, dim3(256), 0, 0, (uint4*)b, n); }));
        rep("write nt 2 GiB", bytes, median_ms([&] { hipLaunchKernelGGL(write_kernel<true>, g, dim3(256), 0, 0, (uint4*)b, n); }));
        rep("copy plain 2 GiB", 2.0 * bytes, median_ms([&] { hipLaunchKernelGGL(copy_kernel_nt<false>, g, dim3(256), 0, 0, (const uint4*)a, (uint4*)b, n); }));
        rep("copy nt 2 GiB", 2.0 * bytes, median_ms([&] { hipLaunchKernelGGL(copy_kernel_nt<true>, g, dim3(256), 0, 0, (const uint4*)a, (uint4*)b, n); }));
    }
    CK(hipFree(a));
    CK(hipFree(b));
    CK(hipFree(sink));
}

// Multi-stream patterns in the stripe layout [B][6][L]: S input streams L apart
// per lane (decode/encode reads), XORed, optionally W outputs to a [B][W][L]
// buffer.  Separates "many concurrent streams" from "read:write mix".
template <int S, int W, bool NT>
__global__ void stream_kernel(const uint8_t* __restrict__ in, uint8_t* __restrict__ out, uint32_t* sink,
                              uint64_t L, uint32_t segs, uint32_t total)
{
    const uint32_t idx = blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= total) return;
    const uint32_t st = idx / segs;
    const uint64_t off = static_cast<uint64_t>(idx - st * segs) * 16;
    const uint8_t* p = in + static_cast<uint64_t>(st) * 6 * L + off;
    uint4 v = make_uint4(0, 0, 0, 0);
#pragma unroll
    for (int s = 0; s < S; ++s) {
        const uint4 x = NT ? nt_load(reinterpret_cast<const uint4*>(p + s * L)) : *reinterpret_cast<const uint4*>(p + s * L);
        v = make_uint4(v.x ^ x.x, v.y ^ x.y, v.z ^ x.z, v.w ^ x.w);
    }
    if (W == 0) {
        if ((v.x ^ v.y ^ v.z ^ v.w) == 0x9E3779B9u) sink[0] = 1;
    } else {
#pragma unroll
        for (int w = 0; w < W; ++w) {
            uint4* q = reinterpret_cast<uint4*>(out + (static_cast<uint64_t>(st) * W + w) * L + off);
            const uint4 y = make_uint4(v.x + w, v.y, v.z, v.w);
            if (NT) nt_store(y, q); else *q = y;
        }
    }
}

static void stream_probe()
{
    const uint64_t L = 65536, B = 4096;
    const uint32_t segs = L / 16, total = static_cast<uint32_t>(B * segs);
    uint8_t *a, *b;
    uint32_t* sink;
    CK(hipMalloc(&a, B * 6 * L));
    CK(hipMalloc(&b, B * 2 * L));
    CK(hipMalloc(&sink, 64));
    CK(hipMemset(a, 7, B * 6 * L));
    auto rep = [&](const char* name, double moved, float ms) {
        std::printf("stream %-26s %8.4f ms  %7.1f GB/s  %5.1f%% of 8 TB/s\n", name, ms, moved / (ms * 1e-3) / 1e9,
                    100.0 * moved / (ms * 1e-3) / 8e12);
    };
    const double seg = 16.0 * total;
    for (int blk : {128, 256}) {
        const dim3 g((total + blk - 1) / blk);
        std::printf("block %d\n", blk);
#define SP(S, W, NT) rep(#S " in " #W " out nt=" #NT, seg * (S + W), median_ms([&] { \
        hipLaunchKernelGGL((stream_kernel<S, W, NT>), g, dim3(blk), 0, 0, a, b, sink, L, segs, total); }))
        SP(1, 0, true); SP(2, 0, true); SP(4, 0, true); SP(6, 0, true);
        SP(1, 1, true); SP(4, 1, true); SP(4, 2, true); SP(4, 1, false); SP(4, 2, false);
#undef SP
    }
    CK(hipFree(a));
    CK(hipFree(b));
    CK(hipFree(sink));
}

// Cache-policy probe: the decode (4 in, 1 out) and encode (4 in, 2 out) access
// patterns of the [B][6][L] layout through buffer loads/stores with explicit
// gfx940-family CPol bits (aux: sc0 = 1, nt = 2, sc1 = 16), to see whether any
// policy other than the product's nt/nt streams HBM better.
template <int W, int LA, int SA>
__global__ void policy_kernel(const uint8_t* in, uint8_t* out, uint32_t* sink, uint32_t L, uint32_t segs,
                              uint32_t total)
{
    const uint32_t idx = blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= total) return;
    const uint32_t st = idx / segs;
    const uint32_t off = (idx - st * segs) * 16;
    const __amdgpu_buffer_rsrc_t ri =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(in + static_cast<uint64_t>(st) * 6 * L), 0, 6 * L, 0x00020000);
    uint32_t v0 = 0, v1 = 0, v2 = 0, v3 = 0;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
        const auto x = __builtin_amdgcn_raw_buffer_load_b128(ri, static_cast<int>(off + s * L), 0, LA);
        v0 ^= x[0]; v1 ^= x[1]; v2 ^= x[2]; v3 ^= x[3];
    }
    const __amdgpu_buffer_rsrc_t ro =
        __builtin_amdgcn_make_buffer_rsrc(out + static_cast<uint64_t>(st) * W * L, 0, W * L, 0x00020000);
#pragma unroll
    for (int w = 0; w < W; ++w) {
        typedef unsigned int v4u __attribute__((ext_vector_type(4)));
        const v4u y = {v0 + w, v1, v2, v3};
        __builtin_amdgcn_raw_buffer_store_b128(y, ro, static_cast<int>(off + w * L), 0, SA);
    }
}

static void policy_probe()
{
    // TUNE_ROTATE=N: launches cycle over N disjoint input/output sets, so no launch
    // finds the previous one's output lines (dirty) in L2 or the 256 MiB MALL
    const int nrot = std::getenv("TUNE_ROTATE") ? std::max(1, std::atoi(std::getenv("TUNE_ROTATE"))) : 1;
    const uint32_t L = 65536, B = 4096;
    const uint32_t segs = L / 16, total = B * segs;
    uint8_t *a0, *b0;
    uint32_t* sink;
    CK(hipMalloc(&a0, static_cast<uint64_t>(B) * 6 * L * nrot));
    CK(hipMalloc(&b0, static_cast<uint64_t>(B) * 2 * L * nrot));
    CK(hipMalloc(&sink, 64));
    CK(hipMemset(a0, 7, static_cast<uint64_t>(B) * 6 * L * nrot));
    int turn = 0;
    uint8_t *a = a0, *b = b0;
    auto next = [&] {
        const int i = turn++ % nrot;
        a = a0 + static_cast<uint64_t>(B) * 6 * L * i;
        b = b0 + static_cast<uint64_t>(B) * 2 * L * i;
    };
    std::printf("policy probe: %d rotating sets\n", nrot);
    const dim3 g((total + 255) / 256);
    const double seg = 16.0 * total;
    auto rep = [&](const char* name, double moved, float ms) {
        std::printf("policy %-34s %8.4f ms  %7.1f GB/s  %5.1f%% of 8 TB/s\n", name, ms, moved / (ms * 1e-3) / 1e9,
                    100.0 * moved / (ms * 1e-3) / 8e12);
    };
    for (int round = 0; round < 3; ++round) {
#define PP(W, LA, SA) rep(#W " out ld=" #LA " st=" #SA, seg * (4 + W), median_ms([&] { next(); \
        hipLaunchKernelGGL((policy_kernel<W, LA, SA>), g, dim3(256), 0, 0, a, b, sink, L, segs, total); }))
        rep("1 out global nt/nt (product)", seg * 5, median_ms([&] { next();
            hipLaunchKernelGGL((stream_kernel<4, 1, true>), g, dim3(256), 0, 0, a, b, sink, uint64_t{L}, segs, total); }));
        PP(1, 2, 2); PP(1, 18, 2); PP(1, 2, 0); PP(1, 2, 16); PP(1, 2, 1); PP(1, 18, 16);
        rep("2 out global nt/nt (product)", seg * 6, median_ms([&] { next();
            hipLaunchKernelGGL((stream_kernel<4, 2, true>), g, dim3(256), 0, 0, a, b, sink, uint64_t{L}, segs, total); }));
        PP(2, 2, 2); PP(2, 18, 2); PP(2, 2, 0); PP(2, 2, 16); PP(2, 2, 1); PP(2, 18, 16);
#undef PP
    }
    CK(hipFree(a0));
    CK(hipFree(b0));
    CK(hipFree(sink));
}

// Encode-shaped XOR probe with a runtime unit stride U: stripe s's unit j at
// s*6*U + j*U, L <= U bytes used per unit; units 0..3 read, 4..5 written in
// place.  Asks whether the 64 KiB sweet spot is about the unit
// stride, and whether padding the stride recovers it for other unit sizes.
__global__ void unit_stride_kernel(uint8_t* buf, uint64_t U, uint32_t segs, uint32_t total, uint32_t magic,
                                   uint32_t shift)
{
    const uint32_t idx = blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= total) return;
    const uint32_t st = static_cast<uint32_t>((static_cast<uint64_t>(idx) * magic) >> shift);
    const uint64_t off = static_cast<uint64_t>(idx - st * segs) * 16;
    uint8_t* p = buf + static_cast<uint64_t>(st) * 6 * U + off;
    uint4 v = make_uint4(0, 0, 0, 0);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const uint4 x = nt_load(reinterpret_cast<const uint4*>(p + j * U));
        v = make_uint4(v.x ^ x.x, v.y ^ x.y, v.z ^ x.z, v.w ^ x.w);
    }
    nt_store(v, reinterpret_cast<uint4*>(p + 4 * U));
    nt_store(make_uint4(v.x + 1, v.y, v.z, v.w), reinterpret_cast<uint4*>(p + 5 * U));
}

static void unit_stride_probe()
{
    struct P {
        uint64_t U, L;
    };
    const P ps[] = {{65536, 65536},     {131072, 131072},   {196608, 196608},   {262144, 262144},
                    {327680, 327680},   {1048576, 1048576}, {1114112, 1048576}, {1179648, 1048576},
                    {131072, 65536},    {196608, 131072},   {4404224, 4404016}, {4521984, 4404016},
                    {4456448, 4404016}, {16384, 16384},     {65536, 16384}};
    for (const P& p : ps) {
        const uint64_t B = (uint64_t{1} << 30) / (4 * p.L);
        uint8_t* buf;
        CK(hipMalloc(&buf, B * 6 * p.U));
        CK(hipMemset(buf, 7, B * 6 * p.U));
        const uint32_t segs = static_cast<uint32_t>(p.L / 16), total = static_cast<uint32_t>(B * segs);
        const Magic mg = make_magic(segs);
        const dim3 g((total + 255) / 256);
        const float ms = median_ms([&] {
            hipLaunchKernelGGL(unit_stride_kernel, g, dim3(256), 0, 0, buf, p.U, segs, total, mg.m, mg.p);
        });
        const double moved = 6.0 * B * p.L;
        std::printf("unit stride %8llu  L %8llu  (stride %6.2f x 64 KiB)  %8.4f ms  %7.1f GB/s  %5.1f%% of 8 TB/s\n",
                    (unsigned long long)p.U, (unsigned long long)p.L, p.U / 65536.0, ms, moved / (ms * 1e-3) / 1e9,
                    100.0 * moved / (ms * 1e-3) / 8e12);
        CK(hipFree(buf));
    }
}

// Unaligned 16-byte global access: correctness for every byte offset and the
// rate of an encode-shaped XOR pattern whose columns sit at a byte offset.
__global__ void unaligned_copy_kernel(const uint8_t* in, uint8_t* out, uint32_t n16)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n16) return;
    nt_store(nt_load(reinterpret_cast<const uint4*>(in + 16ull * i)), reinterpret_cast<uint4*>(out + 16ull * i));
}

__global__ void unaligned_encode_kernel(uint8_t* buf, uint64_t L, uint32_t segs, uint32_t total, uint32_t delta)
{
    const uint32_t idx = blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= total) return;
    const uint32_t st = idx / segs;
    const uint64_t off = static_cast<uint64_t>(idx - st * segs) * 16;
    uint8_t* p = buf + static_cast<uint64_t>(st) * 6 * L + delta + off;
    uint4 v = make_uint4(0, 0, 0, 0);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const uint4 x = nt_load(reinterpret_cast<const uint4*>(p + j * L));
        v = make_uint4(v.x ^ x.x, v.y ^ x.y, v.z ^ x.z, v.w ^ x.w);
    }
    nt_store(v, reinterpret_cast<uint4*>(p + 4 * L));
    nt_store(make_uint4(v.x + 1, v.y, v.z, v.w), reinterpret_cast<uint4*>(p + 5 * L));
}

static int unaligned_probe()
{
    const uint32_t n16 = 1 << 20;  // 16 MiB per check
    std::vector<uint8_t> h(16ull * n16 + 64), r(16ull * n16 + 64);
    for (size_t i = 0; i < h.size(); ++i) h[i] = static_cast<uint8_t>(i * 131 + (i >> 9));
    uint8_t *a, *b;
    CK(hipMalloc(&a, h.size()));
    CK(hipMalloc(&b, h.size()));
    CK(hipMemcpy(a, h.data(), h.size(), hipMemcpyHostToDevice));
    int bad = 0;
    for (uint32_t din = 0; din < 16; ++din)
        for (uint32_t dout : {0u, 1u, 3u, 4u, 8u, 13u}) {
            CK(hipMemset(b, 0, h.size()));
            hipLaunchKernelGGL(unaligned_copy_kernel, dim3(n16 / 256), dim3(256), 0, 0, a + din, b + dout, n16);
            CK(hipDeviceSynchronize());
            CK(hipMemcpy(r.data(), b, r.size(), hipMemcpyDeviceToHost));
            const bool ok = std::memcmp(r.data() + dout, h.data() + din, 16ull * n16) == 0;
            if (!ok) ++bad;
            if (!ok || dout == 0) std::printf("unaligned copy in+%u out+%u: %s\n", din, dout, ok ? "exact" : "MISMATCH");
        }
    CK(hipFree(a));
    CK(hipFree(b));
    const uint64_t L = 65536, B = 4096;
    uint8_t* buf;
    CK(hipMalloc(&buf, B * 6 * L + 64));
    CK(hipMemset(buf, 7, B * 6 * L + 64));
    const uint32_t segs = L / 16, total = static_cast<uint32_t>(B * segs);
    for (uint32_t delta : {0u, 1u, 4u, 8u, 12u}) {
        const float ms = median_ms([&] {
            hipLaunchKernelGGL(unaligned_encode_kernel, dim3(total / 256), dim3(256), 0, 0, buf, L, segs, total, delta);
        });
        const double moved = 6.0 * B * L;
        std::printf("unaligned encode pattern, columns at +%2u B: %8.4f ms  %7.1f GB/s  %5.1f%% of 8 TB/s\n", delta, ms,
                    moved / (ms * 1e-3) / 1e9, 100.0 * moved / (ms * 1e-3) / 8e12);
    }
    CK(hipFree(buf));
    return bad;
}

int main(int argc, char** argv)
{
    if (argc > 1 && std::string(argv[1]) == "unaligned") return unaligned_probe() == 0 ? 0 : 1;
    if (argc > 1 && std::string(argv[1]) == "streams") {
        stream_probe();
        return 0;
    }
    if (argc > 1 && std::string(argv[1]) == "unitstride") {
        unit_stride_probe();
        return 0;
    }
    if (argc > 1 && std::string(argv[1]) == "policy") {
        policy_probe();
        return 0;
    }
    if (argc > 1 && std::string(argv[1]) == "probe") {
        hbm_probe();
        return 0;
    }
    {
    int ndev = 0;
    CK(hipGetDeviceCount(&ndev));
    hipDeviceProp_t prop;
    CK(hipGetDeviceProperties(&prop, 0));
    std::printf("device: %s  CUs=%d\n", prop.gcnArchName, prop.multiProcessorCount);
    {  // plain copy reference: 1 GiB -> 1 GiB
        const uint64_t bytes = 1ull << 30;
        uint8_t *a, *b;
        CK(hipMalloc(&a, bytes));
        CK(hipMalloc(&b, bytes));
        CK(hipMemset(a, 1, bytes));
        hipEvent_t e0, e1;
        CK(hipEventCreate(&e0));
        CK(hipEventCreate(&e1));
        std::vector<float> ts;
        const uint64_t n = bytes / 16;
        for (int i = 0; i < 25; ++i) {
            CK(hipEventRecord(e0));
            hipLaunchKernelGGL(copy_kernel, dim3((n + 255) / 256), dim3(256), 0, 0, (const uint4*)a, (uint4*)b, n);
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            ts.push_back(ms);
        }
        std::sort(ts.begin(), ts.end());
        std::printf("float4 copy 1 GiB: %.4f ms  %.1f GB/s (read+write) = %.1f%% of 8 TB/s\n", ts[12],
                    2.0 * bytes / (ts[12] * 1e-3) / 1e9, 100.0 * 2.0 * bytes / (ts[12] * 1e-3) / 8e12);
        ts.clear();
        for (int i = 0; i < 25; ++i) {
            CK(hipEventRecord(e0));
            CK(hipMemcpyAsync(b, a, bytes, hipMemcpyDeviceToDevice, 0));
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            ts.push_back(ms);
        }
        std::sort(ts.begin(), ts.end());
        std::printf("hipMemcpy D2D 1 GiB: %.4f ms  %.1f GB/s (read+write)\n", ts[12],
                    2.0 * bytes / (ts[12] * 1e-3) / 1e9);
        CK(hipFree(a));
        CK(hipFree(b));
    }
    if (argc > 1 && std::string(argv[1]) == "main") {  // the two shapes the product benches most
        sweep<4, 2>(Shape{"RS(6,4) encode 64KiB", 4, 2, 65536, 4096, 6});
        sweep<8, 4>(Shape{"RS(12,8) encode 256KiB", 8, 4, 262144, 512, 12});
        sweep<4, 1>(Shape{"RS(6,4) decode e=1 64KiB", 4, 1, 65536, 4096, 6});
        sweep<4, 2>(Shape{"RS(6,4) encode 1MiB", 4, 2, 1048576, 256, 6});
        return 0;
    }
    sweep<4, 2>(Shape{"RS(6,4) encode 64KiB", 4, 2, 65536, 4096, 6});
    sweep<4, 1>(Shape{"RS(6,4) decode e=1 64KiB", 4, 1, 65536, 4096, 6});
    sweep<8, 2>(Shape{"RS(12,8) decode e=2 256KiB", 8, 2, 262144, 512, 12});
    sweep<8, 4>(Shape{"RS(12,8) encode 256KiB", 8, 4, 262144, 512, 12});
    sweep<4, 2>(Shape{"RS(6,4) encode 1KiB", 4, 2, 1024, 262144, 6});
    sweep<4, 2>(Shape{"RS(6,4) encode 4KiB", 4, 2, 4096, 65536, 6});
    sweep<4, 2>(Shape{"RS(6,4) encode 1MiB", 4, 2, 1048576, 256, 6});
    sweep<4, 1>(Shape{"RS(6,4) decode e=1 1KiB", 4, 1, 1024, 262144, 6});
    }
    return 0;
}
