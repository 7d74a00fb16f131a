// lds_probe.hip — does loading through LDS (global_load_lds_dwordx4, the
// gfx950 LDS-DMA path) stream HBM faster than global_load_dwordx4 into VGPRs?
// Tuning probe, not product code.  Read-only streams of 2 GiB, and the RS(6,4)
// encode access pattern without the GF arithmetic ([B][6][64 KiB], 4 reads and
// 2 nt writes per lane, XOR only), each loaded both ways, at the product's
// launch shapes.  hipcc --offload-arch=gfx950 -O3 -std=c++17 lds_probe.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <vector>

#define CK(x)                                                                     \
    do {                                                                          \
        hipError_t e_ = (x);                                                      \
        if (e_ != hipSuccess) {                                                   \
            std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            std::exit(1);                                                         \
        }                                                                         \
    } while (0)

typedef __attribute__((address_space(3))) void* lds_ptr;
typedef __attribute__((address_space(1))) const void* gptr;
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint4 load_nt(const uint8_t* p)
{
    const u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
    return make_uint4(v.x, v.y, v.z, v.w);
}

__device__ __forceinline__ void store_nt(uint8_t* p, const uint4& v)
{
    const u32x4 w = {v.x, v.y, v.z, v.w};
    __builtin_nontemporal_store(w, reinterpret_cast<u32x4*>(p));
}

// MODE 0: global_load_dwordx4 nt; 1: LDS-DMA (aux 0); 2: LDS-DMA nt (aux 2)
template <int MODE, int BLOCK>
__global__ __launch_bounds__(BLOCK) void read_kernel(const uint8_t* in, uint32_t* sink, uint64_t segs)
{
    __shared__ __attribute__((aligned(16))) uint32_t buf[BLOCK * 4];  // 1 KiB per wave
    const uint64_t i = blockIdx.x * static_cast<uint64_t>(blockDim.x) + threadIdx.x;
    if (i >= segs) return;
    uint4 v;
    if constexpr (MODE == 0) {
        v = load_nt(in + i * 16);
    } else {
        uint32_t* wb = buf + (threadIdx.x >> 6) * 256;
        __builtin_amdgcn_global_load_lds((gptr)(in + i * 16), (lds_ptr)wb, 16, 0, MODE == 2 ? 2 : 0);
        __builtin_amdgcn_s_waitcnt(0);
        v = *reinterpret_cast<const uint4*>(wb + (threadIdx.x & 63) * 4);
    }
    if ((v.x ^ v.y ^ v.z ^ v.w) == 0x9E3779B9u) sink[threadIdx.x & 63] = 1;
}

// The encode pattern: stripe s = idx / segs, 4 data units in, 2 parity units out.
template <int MODE, int BLOCK>
__global__ __launch_bounds__(BLOCK) void encode_pattern(uint8_t* base, uint64_t L, uint32_t segs, uint32_t total)
{
    __shared__ __attribute__((aligned(16))) uint32_t buf[BLOCK * 16];  // 4 columns x 1 KiB per wave
    const uint32_t idx = blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= total) return;
    const uint32_t st = idx / segs;
    const uint64_t off = static_cast<uint64_t>(idx - st * segs) * 16;
    uint8_t* s = base + static_cast<uint64_t>(st) * 6 * L + off;
    uint4 x[4];
    if constexpr (MODE == 0) {
#pragma unroll
        for (int j = 0; j < 4; ++j) x[j] = load_nt(s + j * L);
    } else {
        uint32_t* wb = buf + (threadIdx.x >> 6) * 1024;
#pragma unroll
        for (int j = 0; j < 4; ++j)
            __builtin_amdgcn_global_load_lds((gptr)(s + j * L), (lds_ptr)(wb + j * 256), 16, 0, MODE == 2 ? 2 : 0);
        __builtin_amdgcn_s_waitcnt(0);
#pragma unroll
        for (int j = 0; j < 4; ++j) x[j] = *reinterpret_cast<const uint4*>(wb + j * 256 + (threadIdx.x & 63) * 4);
    }
    const uint4 p = make_uint4(x[0].x ^ x[1].x ^ x[2].x ^ x[3].x, x[0].y ^ x[1].y ^ x[2].y ^ x[3].y,
                               x[0].z ^ x[1].z ^ x[2].z ^ x[3].z, x[0].w ^ x[1].w ^ x[2].w ^ x[3].w);
    store_nt(s + 4 * L, p);
    store_nt(s + 5 * L, make_uint4(p.y, p.z, p.w, p.x));
}

template <class F>
static float median_ms(F&& launch, int iters = 15)
{
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    std::vector<float> ts;
    launch();
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

// dynamic LDS that caps a launch of `block` threads at `waves` waves per CU
static size_t cap(int block, int waves, size_t static_lds)
{
    if (waves <= 0) return 0;
    const int blocks = std::max(1, waves / (block / 64));
    const size_t per = 160 * 1024 / blocks - 512;
    return per > static_lds ? per - static_lds : 0;
}

int main()
{
    const char* names[3] = {"global_load nt", "LDS-DMA", "LDS-DMA nt"};
    {
        const uint64_t bytes = 2ull << 30, segs = bytes / 16;
        uint8_t* a;
        uint32_t* sink;
        CK(hipMalloc(&a, bytes));
        CK(hipMalloc(&sink, 256));
        CK(hipMemset(a, 7, bytes));
        for (int round = 0; round < 2; ++round)
            for (int block : {256, 64})
                for (int waves : {0, 18, 24}) {
                    if (block == 256 && waves == 18) continue;
                    const dim3 g((segs + block - 1) / block);
                    const size_t lds = cap(block, waves, block * 16);
                    float ms[3];
                    if (block == 256) {
                        ms[0] = median_ms([&] { hipLaunchKernelGGL((read_kernel<0, 256>), g, dim3(block), lds, 0, a, sink, segs); });
                        ms[1] = median_ms([&] { hipLaunchKernelGGL((read_kernel<1, 256>), g, dim3(block), lds, 0, a, sink, segs); });
                        ms[2] = median_ms([&] { hipLaunchKernelGGL((read_kernel<2, 256>), g, dim3(block), lds, 0, a, sink, segs); });
                    } else {
                        ms[0] = median_ms([&] { hipLaunchKernelGGL((read_kernel<0, 64>), g, dim3(block), lds, 0, a, sink, segs); });
                        ms[1] = median_ms([&] { hipLaunchKernelGGL((read_kernel<1, 64>), g, dim3(block), lds, 0, a, sink, segs); });
                        ms[2] = median_ms([&] { hipLaunchKernelGGL((read_kernel<2, 64>), g, dim3(block), lds, 0, a, sink, segs); });
                    }
                    for (int m = 0; m < 3; ++m)
                        std::printf("read 2 GiB  block %3d cap %2d  %-15s %8.4f ms  %7.1f GB/s\n", block, waves, names[m], ms[m],
                                    bytes / (ms[m] * 1e-3) / 1e9);
                }
        CK(hipFree(a));
        CK(hipFree(sink));
    }
    {
        const uint64_t L = 65536, B = 4096;
        const uint32_t segs = L / 16, total = static_cast<uint32_t>(B * segs);
        std::vector<uint8_t*> sets(4);
        for (auto& p : sets) {
            CK(hipMalloc(&p, B * 6 * L));
            CK(hipMemset(p, 3, B * 6 * L));
        }
        const double moved = 6.0 * B * L;
        for (int round = 0; round < 2; ++round)
            for (int block : {64, 256})
                for (int waves : {18, 24, 0}) {
                    float ms[3];
                    for (int m = 0; m < 3; ++m) {
                        int turn = 0;
                        auto go = [&] {
                            uint8_t* p = sets[turn++ % sets.size()];
                            const dim3 g(total / block);
                            const size_t lds = cap(block, waves, block * 64);
                            if (block == 64) {
                                if (m == 0) hipLaunchKernelGGL((encode_pattern<0, 64>), g, dim3(block), lds, 0, p, L, segs, total);
                                if (m == 1) hipLaunchKernelGGL((encode_pattern<1, 64>), g, dim3(block), lds, 0, p, L, segs, total);
                                if (m == 2) hipLaunchKernelGGL((encode_pattern<2, 64>), g, dim3(block), lds, 0, p, L, segs, total);
                            } else {
                                if (m == 0) hipLaunchKernelGGL((encode_pattern<0, 256>), g, dim3(block), lds, 0, p, L, segs, total);
                                if (m == 1) hipLaunchKernelGGL((encode_pattern<1, 256>), g, dim3(block), lds, 0, p, L, segs, total);
                                if (m == 2) hipLaunchKernelGGL((encode_pattern<2, 256>), g, dim3(block), lds, 0, p, L, segs, total);
                            }
                        };
                        ms[m] = median_ms(go);
                    }
                    for (int m = 0; m < 3; ++m)
                        std::printf("encode pattern [4096][6][64K]  block %3d cap %2d  %-15s %8.4f ms  %7.1f GB/s  %5.1f%%\n", block,
                                    waves, names[m], ms[m], moved / (ms[m] * 1e-3) / 1e9, 100.0 * moved / (ms[m] * 1e-3) / 8e12);
                }
        for (auto p : sets) CK(hipFree(p));
    }
    return 0;
}
