// ec_capi.cpp — the C ABI (include/elect_ec.h) over the gfx950 kernels.
//
// EC/  = src/elect/src/native/src/org/apache/cassandra/io/erasurecode
// JEC/ = src/elect/src/java/org/apache/cassandra/io/erasurecode
//
// Host work here is the reference's O(k^3) coder logic (matrix generation,
// survivor-matrix inversion, decode-row selection); every byte of stripe data
// goes through rs_kernels.hip.  There is no CPU fallback: without a device the
// calls return ELECT_EC_ENODEV.
#include "../../include/elect_ec.h"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <new>
#include <vector>

#include "gf256.hpp"
#include "host_path.hpp"
#include "rs_kernels.hpp"

struct elect_ec_coder {
    int k = 0;
    int m = 0;
    // (k+m) x k generator, rows past k+m stay zero (as the zeroed MMAX x KMAX
    // array of IsalEncoder/IsalDecoder, EC/erasure_coder.h:45-53).
    uint8_t gen[ELECT_EC_MAX_UNITS * ELECT_EC_MAX_DATA_UNITS] = {};
};

namespace {

using elect::host::col;
using elect::host::HostOp;
using elect::host::map_hip;
using elect::host::run_host;
using elect::kern::ApplyParams;
using elect::kern::Column;
using elect::kern::UpdateParams;

const uint8_t* parity_row(const elect_ec_coder* c, int r) { return c->gen + (c->k + r) * c->k; }

// processErasures + generateDecodeMatrix (EC/erasure_coder.c:161-200, 241-284).
// compat: rows r < numErasedDataUnits follow the reference's two loops, the
// rest stay zero (clearDecoder, :229-238); strict: every row reconstructs its
// unit.  A singular survivor set: strict -> ESINGULAR; compat -> the partially
// reduced inverse is used, as the reference ignores gf_invert_matrix's -1
// (:257-258), and WARN_SINGULAR is returned.
int build_decode_matrix(const elect_ec_coder* c, const int* decode_indexes, const int* erased,
                        int num_erased, int mode, uint8_t* out)
{
    const int k = c->k, n = c->k + c->m;
    if (!decode_indexes || (num_erased > 0 && !erased) || !out) return ELECT_EC_EINVAL;
    if (num_erased < 0 || num_erased > c->m) return ELECT_EC_EINVAL;  // JEC/CoderUtil.java:79-82
    if (mode != ELECT_EC_DECODE_COMPAT && mode != ELECT_EC_DECODE_STRICT) return ELECT_EC_EINVAL;
    for (int j = 0; j < k; ++j)
        if (decode_indexes[j] < 0 || decode_indexes[j] >= n) return ELECT_EC_EINVAL;
    for (int r = 0; r < num_erased; ++r)
        if (erased[r] < 0 || erased[r] >= n) return ELECT_EC_EINVAL;

    uint8_t work[ELECT_EC_MAX_DATA_UNITS * ELECT_EC_MAX_DATA_UNITS];
    uint8_t inv[ELECT_EC_MAX_DATA_UNITS * ELECT_EC_MAX_DATA_UNITS];
    for (int i = 0; i < k; ++i) std::memcpy(work + i * k, c->gen + decode_indexes[i] * k, k);
    const bool ok = elect::gf::invert(work, inv, k);
    if (!ok && mode == ELECT_EC_DECODE_STRICT) return ELECT_EC_ESINGULAR;

    std::memset(out, 0, static_cast<size_t>(num_erased) * k);
    int rows = num_erased;
    if (mode == ELECT_EC_DECODE_COMPAT) {
        rows = 0;  // numErasedDataUnits (EC/erasure_coder.c:177-182)
        for (int r = 0; r < num_erased; ++r) rows += erased[r] < k;
    }
    for (int r = 0; r < rows; ++r) {
        const int e = erased[r];
        if (e < k) {
            std::memcpy(out + r * k, inv + e * k, k);
        } else {
            const uint8_t* g = c->gen + e * k;  // parity unit: E[e] * Inv
            for (int i = 0; i < k; ++i) {
                uint8_t s = 0;
                for (int j = 0; j < k; ++j) s ^= elect::gf::mul(inv[j * k + i], g[j]);
                out[r * k + i] = s;
            }
        }
    }
    return ok ? ELECT_EC_OK : ELECT_EC_WARN_SINGULAR;
}

hipStream_t as_stream(void* s) { return static_cast<hipStream_t>(s); }

bool valid_coder(const elect_ec_coder* c) { return c && c->k >= 1 && c->m >= 1; }

// Batch geometry: num_stripes units of chunk_size bytes, untiled (tile == 0) or
// stored as ceil(chunk_size / tile) tiles of `tile` bytes, each tile coded as a
// stripe of its own (kern::ApplyParams::tiles).  Tiled launches always run the
// padded kernels: columns without explicit lengths hold chunk_size bytes.
int set_geometry(ApplyParams& p, size_t chunk_size, size_t tile, size_t num_stripes)
{
    p.len = chunk_size;
    p.stripes = num_stripes;
    if (tile == 0) return ELECT_EC_OK;
    if (tile % 16 || tile > 0x7FFFFFFFull || chunk_size > 0xFFFFFFFFull) return ELECT_EC_EINVAL;
    const uint64_t t = std::max<uint64_t>(1, (chunk_size + tile - 1) / tile);
    if (t > 0xFFFFFFFFull || num_stripes > ~uint64_t{0} / t) return ELECT_EC_EINVAL;
    p.len = tile;
    p.stripes = num_stripes * t;
    p.tiles = static_cast<uint32_t>(t);
    p.unit_len = chunk_size;
    p.padded = true;
    for (int j = 0; j < elect::kern::kMaxCols; ++j) p.clen[j] = static_cast<uint32_t>(chunk_size);
    return ELECT_EC_OK;
}

int encode_batch_impl(const elect_ec_coder* coder, size_t chunk_size, size_t tile, size_t num_stripes,
                      elect_ec_shards data, const uint32_t* d_data_lengths, elect_ec_shards parity,
                      int32_t* d_hashes, void* stream)
{
    if (!valid_coder(coder)) return ELECT_EC_EINVAL;
    if ((d_data_lengths || tile) && chunk_size > 0xFFFFFFFFull) return ELECT_EC_EINVAL;
    if (num_stripes == 0 || (chunk_size == 0 && !d_hashes)) return ELECT_EC_OK;
    if (chunk_size > 0 && (!data.base || !parity.base)) return ELECT_EC_EINVAL;
    ApplyParams p;
    const int g = set_geometry(p, chunk_size, tile, num_stripes);
    if (g != ELECT_EC_OK) return g;
    p.cols = coder->k;
    p.rows = coder->m;
    if (d_data_lengths) {
        p.padded = true;
        p.lens = d_data_lengths;
    }
    if (d_hashes) {
        p.hash_seed = true;  // the launcher produces 31^len + sum (no separate memset where it can)
        p.hashes = d_hashes;
        p.hash_stride = static_cast<uint32_t>(coder->m);
    }
    for (int j = 0; j < p.cols; ++j) p.src[j] = col(data.base, data.stripe_stride, j * data.shard_stride);
    for (int r = 0; r < p.rows; ++r) {
        p.dst[r] = col(parity.base, parity.stripe_stride, r * parity.shard_stride);
        std::memcpy(p.coef + r * p.cols, parity_row(coder, r), coder->k);
    }
    return map_hip(elect::kern::launch_apply(p, as_stream(stream)));
}

int decode_batch_impl(const elect_ec_coder* coder, size_t chunk_size, size_t tile, size_t num_stripes,
                      elect_ec_shards inputs, const uint32_t* d_input_lengths, const int* decode_indexes,
                      const int* erased_indexes, int num_erased, elect_ec_shards outputs, unsigned flags, int mode,
                      void* stream)
{
    if (!valid_coder(coder)) return ELECT_EC_EINVAL;
    if ((d_input_lengths || tile) && chunk_size > 0xFFFFFFFFull) return ELECT_EC_EINVAL;
    ApplyParams p;
    const int st = build_decode_matrix(coder, decode_indexes, erased_indexes, num_erased, mode, p.coef);
    if (st < 0) return st;
    if (num_erased == 0 || chunk_size == 0 || num_stripes == 0) return st;
    if (!inputs.base || !outputs.base) return ELECT_EC_EINVAL;
    const int g = set_geometry(p, chunk_size, tile, num_stripes);
    if (g != ELECT_EC_OK) return g;
    p.cols = coder->k;
    p.rows = num_erased;
    for (int j = 0; j < p.cols; ++j) {
        const size_t slot = (flags & ELECT_EC_INPUTS_BY_UNIT) ? static_cast<size_t>(decode_indexes[j]) : j;
        p.src[j] = col(inputs.base, inputs.stripe_stride, slot * inputs.shard_stride);
    }
    for (int r = 0; r < p.rows; ++r) {
        const size_t slot = (flags & ELECT_EC_OUTPUTS_BY_UNIT) ? static_cast<size_t>(erased_indexes[r]) : r;
        p.dst[r] = col(outputs.base, outputs.stripe_stride, slot * outputs.shard_stride);
    }
    if (d_input_lengths) {
        p.padded = true;
        p.lens = d_input_lengths;
    }
    const int rc = map_hip(elect::kern::launch_apply(p, as_stream(stream)));
    return rc != ELECT_EC_OK ? rc : st;
}

// The update as a (2+m)-column product [c_r, c_r, e_r] over [old, new, P...]
// (see elect_ec_encode_update_ex): the padded, hashed and tiled encode machinery
// serves it unchanged.
int update_batch_impl(const elect_ec_coder* coder, size_t chunk_size, size_t tile, size_t num_stripes,
                      int target_data_index, elect_ec_column old_data, elect_ec_column new_data,
                      const uint32_t* d_old_new_lengths, elect_ec_shards parity_in, elect_ec_shards parity_out,
                      int32_t* d_hashes, void* stream)
{
    if (!valid_coder(coder) || target_data_index < 0 || target_data_index >= coder->k) return ELECT_EC_EINVAL;
    // tiled launches ride on the padded vector kernels (at most kMaxPadCols columns),
    // hashed or not: refuse a wider tiled update here, not inside the launcher
    if (tile && 2 + coder->m > elect::kern::kMaxPadCols) return ELECT_EC_EINVAL;
    if ((d_old_new_lengths || tile) && chunk_size > 0xFFFFFFFFull) return ELECT_EC_EINVAL;
    if (num_stripes == 0 || (chunk_size == 0 && !d_hashes)) return ELECT_EC_OK;
    if (chunk_size > 0 && (!old_data.ptr || !new_data.ptr || !parity_in.base || !parity_out.base))
        return ELECT_EC_EINVAL;
    ApplyParams p;
    const int g = set_geometry(p, chunk_size, tile, num_stripes);
    if (g != ELECT_EC_OK) return g;
    p.cols = 2 + coder->m;
    p.rows = coder->m;
    p.src[0] = col(old_data.ptr, old_data.stripe_stride, 0);
    p.src[1] = col(new_data.ptr, new_data.stripe_stride, 0);
    for (int r = 0; r < p.rows; ++r) {
        p.src[2 + r] = col(parity_in.base, parity_in.stripe_stride, r * parity_in.shard_stride);
        p.dst[r] = col(parity_out.base, parity_out.stripe_stride, r * parity_out.shard_stride);
        const uint8_t c = parity_row(coder, r)[target_data_index];
        p.coef[r * p.cols + 0] = c;
        p.coef[r * p.cols + 1] = c;
        p.coef[r * p.cols + 2 + r] = 1;
    }
    if (d_old_new_lengths) {  // old/new padded; the old parity is full length
        p.padded = true;
        p.lens = d_old_new_lengths;
        p.lens_cols = 2;
        p.lens_stride = 2;
        for (int r = 0; r < p.rows; ++r) p.clen[2 + r] = static_cast<uint32_t>(chunk_size);
    }
    if (d_hashes) {
        p.hash_seed = true;
        p.hashes = d_hashes;
        p.hash_stride = static_cast<uint32_t>(coder->m);
    }
    return map_hip(elect::kern::launch_apply(p, as_stream(stream)));
}

// The batches calls' parameter list and grouped launch, with allocation
// failures as status codes (nothing unwinds through the C ABI).
bool reserve_params(std::vector<ApplyParams>& ps, int n)
{
    try {
        ps.resize(static_cast<size_t>(n));
        return true;
    } catch (const std::bad_alloc&) {
        return false;
    }
}

int apply_many(const std::vector<ApplyParams>& ps, int n, void* stream)
{
    try {
        return map_hip(elect::kern::launch_apply_many(ps.data(), n, as_stream(stream)));
    } catch (const std::bad_alloc&) {
        return ELECT_EC_ENOMEM;
    }
}
}  // namespace

extern "C" {

const char* elect_ec_version(void) { return "elect-ec-mi355x 0.2 (gfx950)"; }

#ifndef ELECT_EC_BUILD_ID
#define ELECT_EC_BUILD_ID "unstamped"
#endif
const char* elect_ec_build_id(void) { return ELECT_EC_BUILD_ID; }

const char* elect_ec_strerror(int status)
{
    switch (status) {
    case ELECT_EC_OK: return "ok";
    case ELECT_EC_WARN_SINGULAR: return "decode ran on a singular survivor set (compat mode)";
    case ELECT_EC_EINVAL: return "invalid argument";
    case ELECT_EC_ESINGULAR: return "survivor matrix is singular";
    case ELECT_EC_EDEVICE: return "HIP device error";
    case ELECT_EC_ENOMEM: return "out of memory";
    case ELECT_EC_ENODEV: return "no HIP device";
    default: return "unknown status";
    }
}

int elect_ec_unaligned_vector_ok(int* ok)
{
    if (!ok) return ELECT_EC_EINVAL;
    *ok = 0;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n == 0) return ELECT_EC_ENODEV;
    *ok = elect::kern::unaligned_vector_ok() ? 1 : 0;
    return ELECT_EC_OK;
}

int elect_ec_hbm_probe(int kind, const void* src, void* dst, size_t bytes, int block, int waves_per_cu, void* stream)
{
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n == 0) return ELECT_EC_ENODEV;
    return elect::host::map_hip(
        elect::kern::hbm_probe(kind, src, dst, bytes, block, waves_per_cu, static_cast<hipStream_t>(stream)));
}

int elect_ec_mix_probe(int num_in, int num_out, size_t chunk_size, size_t num_stripes, const elect_ec_column* src,
                       const uint32_t* lengths, const elect_ec_column* dst, int block, int waves_per_cu, void* stream)
{
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n == 0) return ELECT_EC_ENODEV;
    if (!src || !dst || num_in < 1 || num_in > 8 || num_out < 1 || num_out > 4) return ELECT_EC_EINVAL;
    elect::kern::Column s[8], d[4];
    for (int j = 0; j < num_in; ++j) s[j] = elect::host::col(src[j].ptr, src[j].stripe_stride, 0);
    for (int r = 0; r < num_out; ++r) d[r] = elect::host::col(dst[r].ptr, dst[r].stripe_stride, 0);
    return elect::host::map_hip(elect::kern::mix_probe(num_in, num_out, chunk_size, num_stripes, s, lengths, d, block,
                                                       waves_per_cu, static_cast<hipStream_t>(stream)));
}

int elect_ec_device_count(int* count)
{
    if (!count) return ELECT_EC_EINVAL;
    int n = 0;
    const hipError_t e = hipGetDeviceCount(&n);
    *count = e == hipSuccess ? n : 0;
    return (e == hipSuccess && n > 0) ? ELECT_EC_OK : ELECT_EC_ENODEV;
}

int elect_ec_set_host_devices(const int* devices, int n) { return elect::host::set_host_devices(devices, n); }

int elect_ec_device_numa_node(int device, int* node)
{
    if (!node) return ELECT_EC_EINVAL;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) {
        (void)hipGetLastError();
        return ELECT_EC_ENODEV;
    }
    if (device < 0 || device >= ndev) return ELECT_EC_EINVAL;
    *node = elect::host::device_numa_node(device);
    return ELECT_EC_OK;
}

int elect_ec_host_device_map(const int* devices, const int* device_nodes, int num_devices, const int* thread_nodes,
                             int num_threads, int* out)
{
    return elect::host::host_device_map(devices, device_nodes, num_devices, thread_nodes, num_threads, out);
}

// Test hook, not part of include/elect_ec.h: the windows a lone call of units of len bytes
// is pipelined over (host_path.cpp pipeline_windows); bounds: steps + 1 entries.
int elect_ec_internal_pipeline_windows(size_t len, int steps, int taper, size_t* bounds, int* n)
{
    if (!bounds || !n || steps < 1 || steps > 64) return ELECT_EC_EINVAL;
    *n = elect::host::pipeline_windows(len, steps, taper != 0, bounds);
    return ELECT_EC_OK;
}

int elect_ec_set_batching(int enable, unsigned window_us, size_t arena_bytes)
{
    return elect::host::set_batching(enable, window_us, arena_bytes);
}

int elect_ec_host_path_stats(uint64_t* out, int n) { return elect::host::host_path_stats(out, n); }

int elect_ec_host_alloc(size_t bytes, void** out) { return elect::host::host_alloc(bytes, out); }

int elect_ec_host_free(void* ptr) { return elect::host::host_free(ptr); }

int elect_ec_host_pinned(const void* ptr, size_t bytes) { return elect::host::host_pinned(ptr, bytes); }

int elect_ec_coder_create(int num_data_units, int num_parity_units, elect_ec_coder** out)
{
    if (!out) return ELECT_EC_EINVAL;
    *out = nullptr;
    const int k = num_data_units, m = num_parity_units;
    if (k < 1 || m < 1 || k > ELECT_EC_MAX_DATA_UNITS || k + m > ELECT_EC_MAX_UNITS) return ELECT_EC_EINVAL;
    auto* c = new (std::nothrow) elect_ec_coder;
    if (!c) return ELECT_EC_ENOMEM;
    c->k = k;
    c->m = m;
    elect::gf::cauchy_generator(k, m, c->gen);  // initEncodeMatrix, EC/erasure_coder.c:39-47
    *out = c;
    return ELECT_EC_OK;
}

void elect_ec_coder_destroy(elect_ec_coder* coder) { delete coder; }

int elect_ec_coder_num_data_units(const elect_ec_coder* coder) { return coder ? coder->k : ELECT_EC_EINVAL; }

int elect_ec_coder_num_parity_units(const elect_ec_coder* coder) { return coder ? coder->m : ELECT_EC_EINVAL; }

int elect_ec_coder_encode_matrix(const elect_ec_coder* coder, unsigned char* out, size_t out_len)
{
    if (!valid_coder(coder) || !out) return ELECT_EC_EINVAL;
    const size_t n = static_cast<size_t>(coder->k + coder->m) * coder->k;
    if (out_len < n) return ELECT_EC_EINVAL;
    std::memcpy(out, coder->gen, n);
    return ELECT_EC_OK;
}

int elect_ec_coder_gf_tables(const elect_ec_coder* coder, unsigned char* out, size_t out_len)
{
    if (!valid_coder(coder) || !out) return ELECT_EC_EINVAL;
    const size_t n = static_cast<size_t>(coder->m) * coder->k * 32;
    if (out_len < n) return ELECT_EC_EINVAL;
    elect::gf::isal_tables(parity_row(coder, 0), coder->m, coder->k, out);
    return ELECT_EC_OK;
}

int elect_ec_coder_invert_matrix(const elect_ec_coder* coder, const int* decode_indexes, unsigned char* out)
{
    if (!valid_coder(coder) || !decode_indexes || !out) return ELECT_EC_EINVAL;
    const int k = coder->k;
    for (int j = 0; j < k; ++j)
        if (decode_indexes[j] < 0 || decode_indexes[j] >= k + coder->m) return ELECT_EC_EINVAL;
    uint8_t work[ELECT_EC_MAX_DATA_UNITS * ELECT_EC_MAX_DATA_UNITS];
    for (int i = 0; i < k; ++i) std::memcpy(work + i * k, coder->gen + decode_indexes[i] * k, k);
    return elect::gf::invert(work, out, k) ? ELECT_EC_OK : ELECT_EC_WARN_SINGULAR;
}

int elect_ec_coder_decode_matrix(const elect_ec_coder* coder, const int* decode_indexes,
                                 const int* erased_indexes, int num_erased, int mode, unsigned char* out)
{
    if (!valid_coder(coder)) return ELECT_EC_EINVAL;
    return build_decode_matrix(coder, decode_indexes, erased_indexes, num_erased, mode, out);
}

// ---- host memory ----

int elect_ec_encode(const elect_ec_coder* coder, const unsigned char* const* data_units,
                    unsigned char* const* parity_units, size_t chunk_size)
{
    if (!valid_coder(coder) || !data_units || !parity_units) return ELECT_EC_EINVAL;
    HostOp op;
    op.cols = coder->k;
    op.rows = coder->m;
    op.in = data_units;
    op.out = parity_units;
    for (int r = 0; r < coder->m; ++r) std::memcpy(op.coef + r * op.cols, parity_row(coder, r), coder->k);
    return run_host(op, chunk_size);
}

int elect_ec_encode_ex(const elect_ec_coder* coder, const unsigned char* const* data_units,
                       const size_t* data_lengths, unsigned char* const* parity_units, size_t chunk_size,
                       int32_t* hashes)
{
    if (!valid_coder(coder) || !data_units || !parity_units) return ELECT_EC_EINVAL;
    if (data_lengths && chunk_size > 0xFFFFFFFFull) return ELECT_EC_EINVAL;
    if (hashes && chunk_size == 0) {  // hashCode of an empty buffer is 1
        for (int r = 0; r < coder->m; ++r) hashes[r] = 1;
        return ELECT_EC_OK;
    }
    HostOp op;
    op.cols = coder->k;
    op.rows = coder->m;
    op.in = data_units;
    op.out = parity_units;
    op.lens = data_lengths;
    op.hashes = hashes;
    for (int r = 0; r < coder->m; ++r) std::memcpy(op.coef + r * op.cols, parity_row(coder, r), coder->k);
    return run_host(op, chunk_size);
}

int elect_ec_encode_padded(const elect_ec_coder* coder, const unsigned char* const* data_units,
                           const size_t* data_lengths, unsigned char* const* parity_units, size_t chunk_size)
{
    if (!data_lengths) return ELECT_EC_EINVAL;
    return elect_ec_encode_ex(coder, data_units, data_lengths, parity_units, chunk_size, nullptr);
}

int elect_ec_encode_hashed(const elect_ec_coder* coder, const unsigned char* const* data_units,
                           unsigned char* const* parity_units, size_t chunk_size, int32_t* hashes)
{
    if (!hashes) return ELECT_EC_EINVAL;
    return elect_ec_encode_ex(coder, data_units, nullptr, parity_units, chunk_size, hashes);
}

int elect_ec_encode_update(const elect_ec_coder* coder, const unsigned char* const* old_new_parity,
                           int target_data_index, unsigned char* const* new_parity_units, size_t chunk_size)
{
    return elect_ec_encode_update_ex(coder, old_new_parity, nullptr, target_data_index, new_parity_units,
                                     chunk_size, nullptr);
}

int elect_ec_encode_update_ex(const elect_ec_coder* coder, const unsigned char* const* old_new_parity,
                              const size_t* old_new_lengths, int target_data_index,
                              unsigned char* const* new_parity_units, size_t chunk_size, int32_t* hashes)
{
    if (!valid_coder(coder) || !old_new_parity || !new_parity_units) return ELECT_EC_EINVAL;
    if (target_data_index < 0 || target_data_index >= coder->k) return ELECT_EC_EINVAL;
    if (old_new_lengths && chunk_size > 0xFFFFFFFFull) return ELECT_EC_EINVAL;
    if (hashes && chunk_size == 0) {
        for (int r = 0; r < coder->m; ++r) hashes[r] = 1;
        return ELECT_EC_OK;
    }
    // The update as a (2+m)-column product [c_r, c_r, e_r] over [old, new, P...]:
    // the padded and hashed encode machinery, and cross-thread batching, then
    // serve it unchanged (the host path has no separate update kernel).
    HostOp op;
    op.cols = 2 + coder->m;
    op.rows = coder->m;
    op.in = old_new_parity;
    op.out = new_parity_units;
    size_t lens[elect::kern::kMaxCols] = {};
    if (old_new_lengths) {
        lens[0] = old_new_lengths[0];
        lens[1] = old_new_lengths[1];
        for (int r = 0; r < coder->m; ++r) lens[2 + r] = chunk_size;
        op.lens = lens;
    }
    op.hashes = hashes;
    for (int r = 0; r < coder->m; ++r) {
        const uint8_t c = parity_row(coder, r)[target_data_index];
        op.coef[r * op.cols + 0] = c;
        op.coef[r * op.cols + 1] = c;
        op.coef[r * op.cols + 2 + r] = 1;
    }
    return run_host(op, chunk_size);
}

int elect_ec_decode(const elect_ec_coder* coder, const unsigned char* const* inputs, const int* decode_indexes,
                    const int* erased_indexes, int num_erased, unsigned char* const* outputs, size_t chunk_size,
                    int mode)
{
    return elect_ec_decode_ex(coder, inputs, nullptr, decode_indexes, erased_indexes, num_erased, outputs,
                              chunk_size, mode);
}

int elect_ec_decode_ex(const elect_ec_coder* coder, const unsigned char* const* inputs, const size_t* input_lengths,
                       const int* decode_indexes, const int* erased_indexes, int num_erased,
                       unsigned char* const* outputs, size_t chunk_size, int mode)
{
    if (!valid_coder(coder) || !inputs || (num_erased > 0 && !outputs)) return ELECT_EC_EINVAL;
    if (input_lengths && chunk_size > 0xFFFFFFFFull) return ELECT_EC_EINVAL;
    HostOp op;
    const int st = build_decode_matrix(coder, decode_indexes, erased_indexes, num_erased, mode, op.coef);
    if (st < 0) return st;
    if (num_erased == 0) return st;
    op.cols = coder->k;
    op.rows = num_erased;
    op.in = inputs;
    op.out = outputs;
    size_t lens[ELECT_EC_MAX_DATA_UNITS];
    if (input_lengths) {  // content past chunk_size is not needed for a chunk_size prefix
        for (int j = 0; j < coder->k; ++j) lens[j] = std::min(input_lengths[j], chunk_size);
        op.lens = lens;
    }
    const int rc = run_host(op, chunk_size);
    return rc != ELECT_EC_OK ? rc : st;
}

// ---- device resident ----

int elect_ec_encode_batch(const elect_ec_coder* coder, size_t chunk_size, size_t num_stripes,
                          elect_ec_shards data, elect_ec_shards parity, void* stream)
{
    if (!valid_coder(coder) || (!data.base && num_stripes && chunk_size) ||
        (!parity.base && num_stripes && chunk_size))
        return ELECT_EC_EINVAL;
    ApplyParams p;
    p.len = chunk_size;
    p.stripes = num_stripes;
    p.cols = coder->k;
    p.rows = coder->m;
    for (int j = 0; j < p.cols; ++j) p.src[j] = col(data.base, data.stripe_stride, j * data.shard_stride);
    for (int r = 0; r < p.rows; ++r) {
        p.dst[r] = col(parity.base, parity.stripe_stride, r * parity.shard_stride);
        std::memcpy(p.coef + r * p.cols, parity_row(coder, r), coder->k);
    }
    return map_hip(elect::kern::launch_apply(p, as_stream(stream)));
}

int elect_ec_encode_batch_ex(const elect_ec_coder* coder, size_t chunk_size, size_t num_stripes,
                             elect_ec_shards data, const uint32_t* d_data_lengths, elect_ec_shards parity,
                             int32_t* d_hashes, void* stream)
{
    return encode_batch_impl(coder, chunk_size, 0, num_stripes, data, d_data_lengths, parity, d_hashes, stream);
}

int elect_ec_encode_batch_tiled(const elect_ec_coder* coder, size_t chunk_size, size_t tile_bytes,
                                size_t num_stripes, elect_ec_shards data, const uint32_t* d_data_lengths,
                                elect_ec_shards parity, int32_t* d_hashes, void* stream)
{
    if (tile_bytes == 0) return ELECT_EC_EINVAL;
    return encode_batch_impl(coder, chunk_size, tile_bytes, num_stripes, data, d_data_lengths, parity, d_hashes,
                             stream);
}

int elect_ec_encode_batch_padded(const elect_ec_coder* coder, size_t chunk_size, size_t num_stripes,
                                 elect_ec_shards data, const uint32_t* data_lengths, elect_ec_shards parity,
                                 void* stream)
{
    if (!data_lengths) return ELECT_EC_EINVAL;
    return elect_ec_encode_batch_ex(coder, chunk_size, num_stripes, data, data_lengths, parity, nullptr, stream);
}

int elect_ec_encode_batch_hashed(const elect_ec_coder* coder, size_t chunk_size, size_t num_stripes,
                                 elect_ec_shards data, elect_ec_shards parity, int32_t* d_hashes, void* stream)
{
    if (!d_hashes) return ELECT_EC_EINVAL;
    return elect_ec_encode_batch_ex(coder, chunk_size, num_stripes, data, nullptr, parity, d_hashes, stream);
}

int elect_ec_decode_batch(const elect_ec_coder* coder, size_t chunk_size, size_t num_stripes,
                          elect_ec_shards inputs, const int* decode_indexes, const int* erased_indexes,
                          int num_erased, elect_ec_shards outputs, unsigned flags, int mode, void* stream)
{
    return elect_ec_decode_batch_ex(coder, chunk_size, num_stripes, inputs, nullptr, decode_indexes, erased_indexes,
                                    num_erased, outputs, flags, mode, stream);
}

int elect_ec_decode_batch_ex(const elect_ec_coder* coder, size_t chunk_size, size_t num_stripes,
                             elect_ec_shards inputs, const uint32_t* d_input_lengths, const int* decode_indexes,
                             const int* erased_indexes, int num_erased, elect_ec_shards outputs, unsigned flags,
                             int mode, void* stream)
{
    return decode_batch_impl(coder, chunk_size, 0, num_stripes, inputs, d_input_lengths, decode_indexes,
                             erased_indexes, num_erased, outputs, flags, mode, stream);
}

int elect_ec_decode_batch_tiled(const elect_ec_coder* coder, size_t chunk_size, size_t tile_bytes,
                                size_t num_stripes, elect_ec_shards inputs, const uint32_t* d_input_lengths,
                                const int* decode_indexes, const int* erased_indexes, int num_erased,
                                elect_ec_shards outputs, unsigned flags, int mode, void* stream)
{
    if (tile_bytes == 0) return ELECT_EC_EINVAL;
    return decode_batch_impl(coder, chunk_size, tile_bytes, num_stripes, inputs, d_input_lengths, decode_indexes,
                             erased_indexes, num_erased, outputs, flags, mode, stream);
}

int elect_ec_encode_update_batch(const elect_ec_coder* coder, size_t chunk_size, size_t num_stripes,
                                 int target_data_index, elect_ec_column old_data, elect_ec_column new_data,
                                 elect_ec_shards parity_in, elect_ec_shards parity_out, void* stream)
{
    if (!valid_coder(coder) || target_data_index < 0 || target_data_index >= coder->k) return ELECT_EC_EINVAL;
    if (chunk_size == 0 || num_stripes == 0) return ELECT_EC_OK;
    if (!old_data.ptr || !new_data.ptr || !parity_in.base || !parity_out.base) return ELECT_EC_EINVAL;
    UpdateParams p;
    p.len = chunk_size;
    p.stripes = num_stripes;
    p.rows = coder->m;
    p.old_data = col(old_data.ptr, old_data.stripe_stride, 0);
    p.new_data = col(new_data.ptr, new_data.stripe_stride, 0);
    for (int r = 0; r < p.rows; ++r) {
        p.par_in[r] = col(parity_in.base, parity_in.stripe_stride, r * parity_in.shard_stride);
        p.par_out[r] = col(parity_out.base, parity_out.stripe_stride, r * parity_out.shard_stride);
        p.coef[r] = parity_row(coder, r)[target_data_index];
    }
    return map_hip(elect::kern::launch_update(p, as_stream(stream)));
}

int elect_ec_encode_update_batch_ex(const elect_ec_coder* coder, size_t chunk_size, size_t num_stripes,
                                    int target_data_index, elect_ec_column old_data, elect_ec_column new_data,
                                    const uint32_t* d_old_new_lengths, elect_ec_shards parity_in,
                                    elect_ec_shards parity_out, int32_t* d_hashes, void* stream)
{
    if (!valid_coder(coder) || target_data_index < 0 || target_data_index >= coder->k) return ELECT_EC_EINVAL;
    if (!d_old_new_lengths && !d_hashes)
        return elect_ec_encode_update_batch(coder, chunk_size, num_stripes, target_data_index, old_data, new_data,
                                            parity_in, parity_out, stream);
    return update_batch_impl(coder, chunk_size, 0, num_stripes, target_data_index, old_data, new_data,
                             d_old_new_lengths, parity_in, parity_out, d_hashes, stream);
}

int elect_ec_encode_update_batch_tiled(const elect_ec_coder* coder, size_t chunk_size, size_t tile_bytes,
                                       size_t num_stripes, int target_data_index, elect_ec_column old_data,
                                       elect_ec_column new_data, const uint32_t* d_old_new_lengths,
                                       elect_ec_shards parity_in, elect_ec_shards parity_out, int32_t* d_hashes,
                                       void* stream)
{
    if (tile_bytes == 0) return ELECT_EC_EINVAL;
    return update_batch_impl(coder, chunk_size, tile_bytes, num_stripes, target_data_index, old_data, new_data,
                             d_old_new_lengths, parity_in, parity_out, d_hashes, stream);
}

int elect_ec_encode_batches(const elect_ec_coder* coder, const elect_ec_batch* batches, int num_batches,
                            void* stream)
{
    if (!valid_coder(coder) || num_batches < 0 || (num_batches > 0 && !batches)) return ELECT_EC_EINVAL;
    std::vector<ApplyParams> ps;
    if (!reserve_params(ps, num_batches)) return ELECT_EC_ENOMEM;
    for (int i = 0; i < num_batches; ++i) {
        const elect_ec_batch& b = batches[i];
        if (b.chunk_size && b.num_stripes && (!b.in.base || !b.out.base)) return ELECT_EC_EINVAL;
        ApplyParams& p = ps[i];
        p.len = b.chunk_size;
        p.stripes = b.num_stripes;
        p.cols = coder->k;
        p.rows = coder->m;
        for (int j = 0; j < p.cols; ++j) p.src[j] = col(b.in.base, b.in.stripe_stride, j * b.in.shard_stride);
        for (int r = 0; r < p.rows; ++r) {
            p.dst[r] = col(b.out.base, b.out.stripe_stride, r * b.out.shard_stride);
            std::memcpy(p.coef + r * p.cols, parity_row(coder, r), coder->k);
        }
    }
    return apply_many(ps, num_batches, stream);
}

int elect_ec_decode_batches(const elect_ec_coder* coder, const elect_ec_batch* batches, int num_batches,
                            const int* decode_indexes, const int* erased_indexes, int num_erased,
                            unsigned flags, int mode, void* stream)
{
    if (!valid_coder(coder) || num_batches < 0 || (num_batches > 0 && !batches)) return ELECT_EC_EINVAL;
    uint8_t coef[elect::kern::kMaxRows * elect::kern::kMaxCols] = {};
    const int st = build_decode_matrix(coder, decode_indexes, erased_indexes, num_erased, mode, coef);
    if (st < 0) return st;
    if (num_erased == 0) return st;
    std::vector<ApplyParams> ps;
    if (!reserve_params(ps, num_batches)) return ELECT_EC_ENOMEM;
    for (int i = 0; i < num_batches; ++i) {
        const elect_ec_batch& b = batches[i];
        if (b.chunk_size && b.num_stripes && (!b.in.base || !b.out.base)) return ELECT_EC_EINVAL;
        ApplyParams& p = ps[i];
        p.len = b.chunk_size;
        p.stripes = b.num_stripes;
        p.cols = coder->k;
        p.rows = num_erased;
        std::memcpy(p.coef, coef, sizeof(coef));
        for (int j = 0; j < p.cols; ++j) {
            const size_t slot = (flags & ELECT_EC_INPUTS_BY_UNIT) ? static_cast<size_t>(decode_indexes[j]) : j;
            p.src[j] = col(b.in.base, b.in.stripe_stride, slot * b.in.shard_stride);
        }
        for (int r = 0; r < p.rows; ++r) {
            const size_t slot = (flags & ELECT_EC_OUTPUTS_BY_UNIT) ? static_cast<size_t>(erased_indexes[r]) : r;
            p.dst[r] = col(b.out.base, b.out.stripe_stride, slot * b.out.shard_stride);
        }
    }
    const int rc = apply_many(ps, num_batches, stream);
    return rc != ELECT_EC_OK ? rc : st;
}

int elect_ec_apply_batch(const unsigned char* coef, int rows, int cols, size_t chunk_size, size_t num_stripes,
                         const elect_ec_column* src, const elect_ec_column* dst, void* stream)
{
    if (!coef || !src || !dst || rows < 1 || cols < 1 || rows > ELECT_EC_MAX_APPLY || cols > ELECT_EC_MAX_APPLY)
        return ELECT_EC_EINVAL;
    ApplyParams p;
    p.len = chunk_size;
    p.stripes = num_stripes;
    p.cols = cols;
    p.rows = rows;
    for (int j = 0; j < cols; ++j) {
        if (!src[j].ptr && chunk_size && num_stripes) return ELECT_EC_EINVAL;
        p.src[j] = col(src[j].ptr, src[j].stripe_stride, 0);
    }
    for (int r = 0; r < rows; ++r) {
        if (!dst[r].ptr && chunk_size && num_stripes) return ELECT_EC_EINVAL;
        p.dst[r] = col(dst[r].ptr, dst[r].stripe_stride, 0);
    }
    std::memcpy(p.coef, coef, static_cast<size_t>(rows) * cols);
    return map_hip(elect::kern::launch_apply(p, as_stream(stream)));
}

}  // extern "C"
