// A/B of a bitsliced (Cauchy bit-matrix) RS(12,8) encode against the product's
// byte-shuffle kernel (EC/erasure_coder.c:43, 90 at k=8, m=4).
//
// Per lane, 32 bytes of each of the 8 data columns: the XOR-circulant sums of
// each group of 4 columns (s, u, v, w; rs_impl.hpp gf_combine_cauchy4) in the
// byte domain, an 8x8 bit transpose of every operand (three swap-move stages,
// two shifts + two bit-selects per pair) into 8 bit planes, the XOR network
// of tools/tune/gen_bitslice.py (Paar-reduced) from the 64 operand planes to
// the 32 parity planes, and the transpose back.  Bytes must equal the
// product's (elect_ec_encode_batch on the same stripes).
//
//   python tools/tune/gen_bitslice.py > tools/tune/bitslice_net.inc
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include tools/tune/bitslice_probe.hip \
//       -L elect_amd -lelect_ec -Wl,-rpath,'$ORIGIN/../../elect_amd' -o tools/tune/bitslice_probe
//   tools/tune/bitslice_probe [reps=20]
// Layout [B][12][L], B = 2048 stripes of L = 64 KiB (BASELINE configs[4]'s 512 x 256 KiB as the
// product's 64 KiB tiles).  Prints one JSON line.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "elect_ec.h"
#include "bitslice_net.inc"

#define CHECK(x)                                                                             \
    do {                                                                                     \
        hipError_t e_ = (x);                                                                 \
        if (e_ != hipSuccess) {                                                              \
            std::printf("{\"error\": \"%s at line %d\"}\n", hipGetErrorString(e_), __LINE__); \
            return 2;                                                                        \
        }                                                                                    \
    } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <int D, uint32_t MSK>
__device__ __forceinline__ void swap_move(uint32_t& a, uint32_t& b)
{
    constexpr uint32_t hi = MSK << D;
    const uint32_t na = (a & ~hi) | ((b << D) & hi);
    const uint32_t nb = (b & ~MSK) | ((a >> D) & MSK);
    a = na;
    b = nb;
}

// Register i, byte lane q, bit j  <->  register j, byte lane q, bit i (an involution).
__device__ __forceinline__ void transpose8(uint32_t* w)
{
    swap_move<4, 0x0F0F0F0Fu>(w[0], w[4]);
    swap_move<4, 0x0F0F0F0Fu>(w[1], w[5]);
    swap_move<4, 0x0F0F0F0Fu>(w[2], w[6]);
    swap_move<4, 0x0F0F0F0Fu>(w[3], w[7]);
    swap_move<2, 0x33333333u>(w[0], w[2]);
    swap_move<2, 0x33333333u>(w[1], w[3]);
    swap_move<2, 0x33333333u>(w[4], w[6]);
    swap_move<2, 0x33333333u>(w[5], w[7]);
    swap_move<1, 0x55555555u>(w[0], w[1]);
    swap_move<1, 0x55555555u>(w[2], w[3]);
    swap_move<1, 0x55555555u>(w[4], w[5]);
    swap_move<1, 0x55555555u>(w[6], w[7]);
}

__global__ __launch_bounds__(256) void bitslice_encode(const uint8_t* __restrict__ st, uint8_t* __restrict__ par,
                                                       uint32_t stripes, uint32_t L)
{
    const uint32_t segs = L / 32;
    const uint64_t idx = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
    if (idx >= static_cast<uint64_t>(stripes) * segs) return;
    const uint32_t s = static_cast<uint32_t>(idx / segs);
    const uint32_t off = static_cast<uint32_t>(idx % segs) * 32u;
    const uint8_t* base = st + static_cast<uint64_t>(s) * 12u * L + off;
    uint32_t P[64];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const u32x4* p = reinterpret_cast<const u32x4*>(base + static_cast<uint64_t>(j) * L);
        const u32x4 a = __builtin_nontemporal_load(p);
        const u32x4 b = __builtin_nontemporal_load(p + 1);
        P[8 * j + 0] = a.x, P[8 * j + 1] = a.y, P[8 * j + 2] = a.z, P[8 * j + 3] = a.w;
        P[8 * j + 4] = b.x, P[8 * j + 5] = b.y, P[8 * j + 6] = b.z, P[8 * j + 7] = b.w;
    }
#if BITSLICE_KARATSUBA
#pragma unroll
    for (int g = 0; g < 2; ++g)
#pragma unroll
        for (int d = 0; d < 8; ++d) {
            const uint32_t x0 = P[8 * (4 * g) + d], x1 = P[8 * (4 * g + 1) + d];
            const uint32_t x2 = P[8 * (4 * g + 2) + d], x3 = P[8 * (4 * g + 3) + d];
            P[8 * (4 * g) + d] = x0 ^ x1 ^ x2 ^ x3;  // s
            P[8 * (4 * g + 1) + d] = x1 ^ x3;        // u
            P[8 * (4 * g + 2) + d] = x2 ^ x3;        // v (w = x3 stays)
        }
#endif
#pragma unroll
    for (int o = 0; o < 8; ++o) transpose8(&P[8 * o]);
    uint32_t Y[32];
    BITSLICE_NET(P, Y)
#pragma unroll
    for (int a = 0; a < 4; ++a) {
        transpose8(&Y[8 * a]);
        u32x4* q = reinterpret_cast<u32x4*>(par + (static_cast<uint64_t>(s) * 4u + a) * L + off);
        __builtin_nontemporal_store(u32x4{Y[8 * a + 0], Y[8 * a + 1], Y[8 * a + 2], Y[8 * a + 3]}, q);
        __builtin_nontemporal_store(u32x4{Y[8 * a + 4], Y[8 * a + 5], Y[8 * a + 6], Y[8 * a + 7]}, q + 1);
    }
}

__global__ void fill(uint32_t* p, uint64_t n)
{
    for (uint64_t i = blockIdx.x * static_cast<uint64_t>(blockDim.x) + threadIdx.x; i < n;
         i += static_cast<uint64_t>(gridDim.x) * blockDim.x) {
        uint64_t z = i * 0x9E3779B97F4A7C15ull + 0xE1EC7;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        p[i] = static_cast<uint32_t>(z ^ (z >> 31));
    }
}

// mismatching 16-byte words between the product's parity (in st) and par
__global__ void compare(const uint8_t* st, const uint8_t* par, uint32_t stripes, uint32_t L, unsigned long long* bad)
{
    const uint64_t words = static_cast<uint64_t>(stripes) * 4 * L / 16;
    for (uint64_t i = blockIdx.x * static_cast<uint64_t>(blockDim.x) + threadIdx.x; i < words;
         i += static_cast<uint64_t>(gridDim.x) * blockDim.x) {
        const uint64_t byte = i * 16, s = byte / (4ull * L), rem = byte % (4ull * L);
        const uint4 a = *reinterpret_cast<const uint4*>(st + s * 12ull * L + 8ull * L + rem);
        const uint4 b = *reinterpret_cast<const uint4*>(par + byte);
        if (a.x != b.x || a.y != b.y || a.z != b.z || a.w != b.w) atomicAdd(bad, 1ull);
    }
}

int main(int argc, char** argv)
{
    const int reps = argc > 1 ? std::atoi(argv[1]) : 20;
    const uint32_t B = 2048, L = 65536;
    const size_t st_bytes = static_cast<size_t>(B) * 12 * L, par_bytes = static_cast<size_t>(B) * 4 * L;
    uint8_t *st = nullptr, *par = nullptr;
    unsigned long long* bad = nullptr;
    CHECK(hipMalloc(&st, st_bytes));
    CHECK(hipMalloc(&par, par_bytes));
    CHECK(hipMalloc(&bad, sizeof(*bad)));
    hipStream_t stream;
    CHECK(hipStreamCreate(&stream));
    hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, stream, reinterpret_cast<uint32_t*>(st), st_bytes / 4);
    CHECK(hipGetLastError());
    elect_ec_coder* coder = nullptr;
    if (elect_ec_coder_create(8, 4, &coder) != 0) {
        std::printf("{\"error\": \"coder\"}\n");
        return 2;
    }
    const elect_ec_shards data{st, 12ull * L, L}, parity{st + 8ull * L, 12ull * L, L};
    auto product = [&] { return elect_ec_encode_batch(coder, L, B, data, parity, stream); };
    const uint32_t grid = static_cast<uint32_t>((static_cast<uint64_t>(B) * (L / 32) + 255) / 256);
    auto bitsliced = [&] {
        hipLaunchKernelGGL(bitslice_encode, dim3(grid), dim3(256), 0, stream, st, par, B, L);
        return static_cast<int>(hipGetLastError());
    };
    if (product() != 0 || bitsliced() != 0) {
        std::printf("{\"error\": \"launch\"}\n");
        return 2;
    }
    CHECK(hipMemsetAsync(bad, 0, sizeof(*bad), stream));
    hipLaunchKernelGGL(compare, dim3(4096), dim3(256), 0, stream, st, par, B, L, bad);
    unsigned long long nbad = 0;
    CHECK(hipMemcpyAsync(&nbad, bad, sizeof(nbad), hipMemcpyDeviceToHost, stream));
    CHECK(hipStreamSynchronize(stream));
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    auto timed = [&](auto&& fn) {
        std::vector<float> t;
        for (int r = 0; r < reps + 2; ++r) {
            (void)hipEventRecord(e0, stream);
            (void)fn();
            (void)hipEventRecord(e1, stream);
            (void)hipEventSynchronize(e1);
            float ms = 0;
            (void)hipEventElapsedTime(&ms, e0, e1);
            if (r >= 2) t.push_back(ms);
        }
        std::sort(t.begin(), t.end());
        return t[t.size() / 2];
    };
    // interleaved: product, bitsliced, product, bitsliced
    const float p1 = timed(product), b1 = timed(bitsliced), p2 = timed(product), b2 = timed(bitsliced);
    const double bytes = static_cast<double>(B) * 12 * L;
    auto frac = [&](float ms) { return bytes / (ms * 1e-3) / 8e12; };
    std::printf("{\"probe\": \"RS(12,8) encode, %u x %u B stripes [B][12][L]\", \"bitsliced_equals_product\": %s, "
                "\"mismatched_16B_words\": %llu, \"product_ms\": [%.4f, %.4f], \"bitsliced_ms\": [%.4f, %.4f], "
                "\"product_frac\": [%.4f, %.4f], \"bitsliced_frac\": [%.4f, %.4f], \"form\": \"%s\"}\n",
                B, L, nbad == 0 ? "true" : "false", nbad, p1, p2, b1, b2, frac(p1), frac(p2), frac(b1), frac(b2),
                BITSLICE_KARATSUBA ? "karatsuba" : "direct");
    return nbad == 0 ? 0 : 1;
}
