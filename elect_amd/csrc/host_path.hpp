// host_path.hpp — the host-memory (JNI calling convention) path of the C ABI:
// pinned staging, per-thread streams, device policy, cross-thread batching.
#pragma once

#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>

#include "../../include/elect_ec.h"
#include "rs_kernels.hpp"

namespace elect {
namespace host {

inline int map_hip(hipError_t e)
{
    switch (e) {
    case hipSuccess: return ELECT_EC_OK;
    case hipErrorNoDevice:
    case hipErrorInvalidDevice:
    case hipErrorNoBinaryForGpu: return ELECT_EC_ENODEV;
    case hipErrorOutOfMemory: return ELECT_EC_ENOMEM;
    case hipErrorInvalidValue: return ELECT_EC_EINVAL;
    default: return ELECT_EC_EDEVICE;
    }
}

inline kern::Column col(const void* base, size_t stripe_stride, size_t offset)
{
    kern::Column c;
    c.ptr = static_cast<const uint8_t*>(base) + offset;
    c.stride = stripe_stride;
    return c;
}

// One synchronous host-memory operation: `cols` host inputs -> `rows` host outputs,
// out[r] = XOR_j coef[r*cols+j] * in[j] (a parity update is the product
// [c_r, c_r, e_r] over [old, new, P...]).  Outputs may alias inputs.
struct HostOp {
    int cols = 0;
    int rows = 0;
    const unsigned char* const* in = nullptr;
    unsigned char* const* out = nullptr;
    uint8_t coef[kern::kMaxRows * kern::kMaxCols] = {};
    const size_t* lens = nullptr;  // optional content length per input (implicit zero padding)
    int32_t* hashes = nullptr;     // optional host output: ByteBuffer.hashCode() per output row
};

// Runs op on the calling thread's device (or its assigned one, see
// set_host_devices), through cross-thread batching when that is enabled.
int run_host(const HostOp& op, size_t len);
int set_host_devices(const int* devices, int n);
int device_numa_node(int dev);  // elect_ec_device_numa_node (-1: unknown)
// The device a thread on NUMA node thread_node gets (host_device's choice; load: threads per listed device)
int numa_pick(const int* devices, const int* nodes, int ndev, int thread_node, unsigned* load);
int host_device_map(const int* devices, const int* nodes, int ndev, const int* thread_nodes, int nthreads, int* out);
// The windows a pipelined batch of units of len bytes runs over in (at most) steps steps:
// window k is [at[k], at[k + 1]); returns their number n (at[0] = 0, at[n] = len).  at: steps + 1 entries.
int pipeline_windows(size_t len, int steps, bool taper, size_t* at);
int set_batching(int enable, unsigned window_us, size_t arena_bytes);
int host_path_stats(uint64_t* out, int n);  // elect_ec_host_path_stats
int host_alloc(size_t bytes, void** out);    // elect_ec_host_alloc
int host_free(void* ptr);                    // elect_ec_host_free
int host_pinned(const void* ptr, size_t bytes);  // elect_ec_host_pinned

}  // namespace host
}  // namespace elect
