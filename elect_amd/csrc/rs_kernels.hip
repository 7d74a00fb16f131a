// rs_kernels.hip — launch dispatch for ELECT's Reed-Solomon path on gfx950.
//
// The kernels and their launch templates are in rs_impl.hpp (design notes
// there); the instances are built per source-column count by rs_inst.hip.
// This unit holds the dispatch (launch_apply, launch_apply_many, launch_update),
// the per-stream hash-partial scratch, the byte-granular and parity-update
// kernels and the unaligned-access probe.
#include "rs_impl.hpp"

namespace elect {
namespace kern {
namespace {

// Hash-partial scratch when the caller brings none (the device-resident API):
// one buffer per (device, stream), reused only in that stream's order.  It is
// handed to another stream (64 entries per device, least recently used first)
// only after its last use (an event recorded behind each use once 32 or more
// entries are assigned; a device-wide synchronize before that, round 6), and
// grown only after its own stream's synchronize, so a hashed call records
// nothing on the stream while few streams share the cache: a completion
// marker behind every call held the next launch back ~1.5 us (round 4,
// profiles/r04/event_cost.txt), and streams beyond 64 are rare (16 entries made
// the device-wide synchronize of a handoff routine for 17+ concurrently launching streams).
// Stream-ordered allocation (hipMallocAsync / hipFreeAsync, default or private
// pool) corrupted partials when many threads launched on their own streams:
// freed blocks were handed out again while a reduce still read them
// (tools/sanitize/host_stress; a never-freed hipMalloc variant was clean).
struct ScratchEntry {
    std::mutex mu;           // held from lease to release: launches on one stream serialise
    hipStream_t stream = nullptr;
    bool assigned = false;
    uint64_t last = 0;       // LRU tick (under the cache mutex)
    uint32_t* ptr = nullptr;
    size_t words = 0;
    hipStream_t owner = nullptr;  // the stream whose launches may still read ptr
    bool owned = false;
    // Under pressure (kPressure or more entries assigned) each release records `ev` on
    // its stream, so that a handoff waits for that stream's last use only
    // (hipStreamWaitEvent) instead of the whole device.
    bool record = false;    // this lease records on release
    hipEvent_t ev = nullptr;
    bool ev_valid = false;  // ev marks the last use (else: device-wide synchronize at handoff)
};
constexpr int kPressure = 32;

struct ScratchCache {
    std::mutex mu;
    uint64_t tick = 0;
    ScratchEntry e[64];
};

ScratchCache g_scratch[64];

// Returns with entry->mu held; scratch_release() unlocks.
hipError_t scratch_lease(hipStream_t stream, size_t words, ScratchEntry** out)
{
    // The scratch is allocated on, and cached for, the current device: a stream of
    // another device would have its kernels read memory of the wrong device.
    int dev = 0;
    hipError_t err = hipGetDevice(&dev);
    if (err != hipSuccess) return err;
    if (dev < 0 || dev >= 64) return hipErrorInvalidDevice;
    if (stream) {
        hipDevice_t sdev = 0;
        err = hipStreamGetDevice(stream, &sdev);
        if (err != hipSuccess) return err;
        if (sdev != dev) return hipErrorInvalidValue;  // include/elect_ec.h: streams of the current device
    }
    ScratchCache& c = g_scratch[dev];
    for (;;) {
        ScratchEntry* e = nullptr;
        bool pressure = false;
        {
            std::lock_guard<std::mutex> lock(c.mu);
            int assigned = 0;
            for (ScratchEntry& x : c.e) {
                assigned += x.assigned;
                if (x.assigned && x.stream == stream) e = &x;
            }
            if (!e) {  // a free entry, else the least recently used one
                for (ScratchEntry& x : c.e)
                    if (!e || (!x.assigned && e->assigned) || (x.assigned == e->assigned && x.last < e->last)) e = &x;
                e->assigned = true;
                e->stream = stream;
            }
            e->last = ++c.tick;
            // (ELECT_EC_SCRATCH_EVENTS=0: never record, round 5's device-wide synchronize at every handoff; A/B)
            static const bool events = [] {
                const char* v = std::getenv("ELECT_EC_SCRATCH_EVENTS");
                return !(v && std::atoi(v) == 0);
            }();
            pressure = events && assigned >= kPressure;
        }
        e->mu.lock();
        if (!e->assigned || e->stream != stream) {  // taken over for another stream meanwhile
            e->mu.unlock();
            continue;
        }
        // Last used on another stream (which may since have been destroyed): wait for its
        // last use (the event recorded then, device-side), else for the whole device;
        // then this stream owns the buffer.
        if (e->owned && e->owner != stream)
            err = e->ev_valid ? hipStreamWaitEvent(stream, e->ev, 0) : hipDeviceSynchronize();
        e->record = pressure;
        if (err == hipSuccess && e->words < words) {
            if (e->owned) err = hipStreamSynchronize(stream);  // its last use, on this stream
            if (err == hipSuccess && e->ptr) err = hipFree(e->ptr);
            e->ptr = nullptr;
            e->words = 0;
            if (err == hipSuccess) err = hipMalloc(reinterpret_cast<void**>(&e->ptr), words * sizeof(uint32_t));
            if (err == hipSuccess) e->words = words;
        }
        if (err != hipSuccess) {
            e->mu.unlock();
            return err;
        }
        e->owner = stream;
        e->owned = true;
        *out = e;
        return hipSuccess;
    }
}

hipError_t scratch_release(ScratchEntry* e, hipStream_t stream)
{
    e->ev_valid = false;
    if (e->record) {  // (a marker behind every call would hold the next launch back ~1.5 us: only under pressure)
        hipError_t err = e->ev ? hipSuccess : hipEventCreateWithFlags(&e->ev, hipEventDisableTiming);
        if (err == hipSuccess) err = hipEventRecord(e->ev, stream);
        e->ev_valid = err == hipSuccess;
        // a marker that could not be recorded only costs the next handoff a device-wide
        // synchronize: the launch itself stands
        if (err != hipSuccess) (void)hipGetLastError();
    }
    e->mu.unlock();
    return hipSuccess;
}

// Every (cols, rows) launcher, by source-column count (rs_inst.hip).  Padded
// variants exist for up to ELECT_EC_MAX_DATA_UNITS (kMaxPadCols = 10) columns:
// the encode shapes and ELECT's decode (k survivors).
const std::array<KernelRows, kMaxCols> kRows = {
    kernel_rows_k1(),  kernel_rows_k2(),  kernel_rows_k3(),  kernel_rows_k4(),
    kernel_rows_k5(),  kernel_rows_k6(),  kernel_rows_k7(),  kernel_rows_k8(),
    kernel_rows_k9(),  kernel_rows_k10(), kernel_rows_k11(), kernel_rows_k12(),
    kernel_rows_k13(), kernel_rows_k14(), kernel_rows_k15(), kernel_rows_k16()};

// ---------------------------------------------------------------------------
// Byte-granular path: any alignment, any (cols, rows) up to 16 x 16.
// ---------------------------------------------------------------------------
struct GenericArgs {
    const uint8_t* sp[kMaxCols];
    uint64_t ss[kMaxCols];
    uint8_t* dp[kMaxRows];
    uint64_t ds[kMaxRows];
    uint32_t len;    // bytes per stripe in this launch window (< 2^31)
    uint32_t total;  // bytes in this launch
    uint32_t magic;
    uint32_t shift;
    int cols;
    int rows;
    uint8_t coef[kMaxRows * kMaxCols];
    const uint32_t* lens;  // padded: [stripe][lstride] content lengths of columns < lcols, or null -> clen
    uint32_t lstride;
    int lcols;
    uint32_t clen[kMaxCols];
    int padded;
    uint32_t col_base;     // byte offset of this launch window inside the shard
    int32_t* hashes;       // optional parity hashes [stripe][hstride]
    uint32_t hstride;
    uint64_t hbase;        // hash offset of byte 0 of this window
};

__constant__ uint8_t d_exp[512];
__constant__ uint8_t d_log[256];

__global__ __launch_bounds__(kBlock) void gf_apply_bytes(const GenericArgs a)
{
    const uint32_t idx = blockIdx.x * kBlock + threadIdx.x;
    if (idx >= a.total) return;
    const uint32_t s = static_cast<uint32_t>((static_cast<uint64_t>(idx) * a.magic) >> a.shift);
    const uint32_t i = idx - s * a.len;
    uint8_t lx[kMaxCols];
    bool nz[kMaxCols];
    for (int j = 0; j < a.cols; ++j) {
        uint8_t v = 0;
        if (a.padded) {
            const uint32_t valid = a.lens && j < a.lcols ? a.lens[static_cast<uint64_t>(s) * a.lstride + j] : a.clen[j];
            if (a.col_base + i < valid) v = a.sp[j][s * a.ss[j] + i];
        } else {
            v = a.sp[j][s * a.ss[j] + i];
        }
        nz[j] = v != 0;
        lx[j] = d_log[v];
    }
    for (int r = 0; r < a.rows; ++r) {
        uint8_t acc = 0;
        for (int j = 0; j < a.cols; ++j) {
            const uint8_t c = a.coef[r * a.cols + j];
            if (c != 0 && nz[j]) acc ^= d_exp[d_log[c] + lx[j]];
        }
        a.dp[r][s * a.ds[r] + i] = acc;
        if (a.hashes)
            atomicAdd(reinterpret_cast<unsigned*>(a.hashes) + static_cast<uint64_t>(s) * a.hstride + r,
                      static_cast<uint32_t>(static_cast<int32_t>(static_cast<int8_t>(acc))) * dpow31(a.hbase + i));
    }
}

hipError_t launch_bytes(const ApplyParams& p, hipStream_t stream)
{
    static std::mutex mu;             // field tables go to __constant__ once per device
    static uint64_t ready_mask = 0;
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    {
        std::lock_guard<std::mutex> lock(mu);
        if (!(ready_mask & (uint64_t{1} << (dev & 63)))) {
            e = hipMemcpyToSymbol(HIP_SYMBOL(d_exp), gf::kField.exp.data(), 512);
            if (e == hipSuccess) e = hipMemcpyToSymbol(HIP_SYMBOL(d_log), gf::kField.log.data(), 256);
            if (e != hipSuccess) return e;
            ready_mask |= uint64_t{1} << (dev & 63);
        }
    }
    if (p.len > kMaxIndex) return hipErrorInvalidValue;
    GenericArgs a{};
    a.len = static_cast<uint32_t>(p.len);
    a.cols = p.cols;
    a.rows = p.rows;
    std::copy(p.coef, p.coef + kMaxRows * kMaxCols, a.coef);
    a.padded = p.padded ? 1 : 0;
    a.lstride = p.lens_stride ? p.lens_stride : static_cast<uint32_t>(p.cols);
    a.lcols = p.lens_cols ? p.lens_cols : p.cols;
    std::copy(p.clen, p.clen + kMaxCols, a.clen);
    a.col_base = p.padded ? p.col_base : 0;
    a.hstride = p.hash_stride;
    a.hbase = p.hash_base;
    const Magic mg = make_magic(a.len);
    a.magic = mg.m;
    a.shift = mg.p;
    const uint64_t per_launch = kMaxIndex / p.len;
    for (uint64_t s0 = 0; s0 < p.stripes; s0 += per_launch) {
        const uint64_t ns = std::min<uint64_t>(per_launch, p.stripes - s0);
        for (int j = 0; j < p.cols; ++j) {
            a.sp[j] = p.src[j].ptr + s0 * p.src[j].stride;
            a.ss[j] = p.src[j].stride;
        }
        for (int r = 0; r < p.rows; ++r) {
            a.dp[r] = const_cast<uint8_t*>(p.dst[r].ptr) + s0 * p.dst[r].stride;
            a.ds[r] = p.dst[r].stride;
        }
        a.lens = p.lens ? p.lens + s0 * a.lstride : nullptr;
        a.hashes = p.hashes ? p.hashes + s0 * p.hash_stride : nullptr;
        a.total = static_cast<uint32_t>(ns * p.len);
        const uint32_t grid = (a.total + kBlock - 1) / kBlock;
        hipLaunchKernelGGL(gf_apply_bytes, dim3(grid), dim3(kBlock), 0, stream, a);
        e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

// ---------------------------------------------------------------------------
// Parity update: par_out[r] = par_in[r] ^ c_r * (old ^ new), fused.
// ---------------------------------------------------------------------------
// The plain parity update runs one-wave blocks, 18 waves per CU, like the plain
// encodes (kPolicy.update_*): 81.6 -> 84.2 % of peak (uncapped 256-thread blocks
// before; caps on those, 20-28 waves, measured within noise; one-wave blocks at
// 16 / 22 waves: 83.5 / 83.8 %; profiles/r03/plain_one_wave_ab.txt).
template <int R>
struct UpdArgs {
    const uint8_t* op;
    uint64_t os;
    const uint8_t* np;
    uint64_t ns;
    const uint8_t* pip[R];
    uint64_t pis[R];
    uint8_t* pop[R];
    uint64_t pos[R];
    uint32_t segs, total, magic, shift;
    gf::PermTable tab[R];
};

template <int R>
__global__ __launch_bounds__(kBlock) void gf_update_x16(const UpdArgs<R> a)
{
    const uint32_t idx = blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= a.total) return;
    const uint32_t s = static_cast<uint32_t>((static_cast<uint64_t>(idx) * a.magic) >> a.shift);
    const uint64_t b0 = static_cast<uint64_t>(idx - s * a.segs) * 16;
    const uint4 o = load_nt(a.op + s * a.os + b0);
    const uint4 w = load_nt(a.np + s * a.ns + b0);
    uint4 pin[R];
#pragma unroll
    for (int r = 0; r < R; ++r) pin[r] = load_nt(a.pip[r] + s * a.pis[r] + b0);
    const uint4 d = make_uint4(o.x ^ w.x, o.y ^ w.y, o.z ^ w.z, o.w ^ w.w);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const Sel sl = selectors(lane_word(d, q));
#pragma unroll
        for (int r = 0; r < R; ++r)
            set_word(pin[r], q, lane_word(pin[r], q) ^ gf_lookup(a.tab[r], sl.s0, sl.s1, sl.s2));
    }
#pragma unroll
    for (int r = 0; r < R; ++r) store_nt(a.pop[r] + s * a.pos[r] + b0, pin[r]);
}

template <int R>
hipError_t launch_update_r(const UpdateParams& p, int r0, hipStream_t stream)
{
    UpdArgs<R> a{};
    const uint64_t segs64 = p.len / 16;
    if (segs64 == 0) return hipSuccess;
    if (segs64 > kMaxIndex) return hipErrorInvalidValue;
    a.segs = static_cast<uint32_t>(segs64);
    const Magic mg = make_magic(a.segs);
    a.magic = mg.m;
    a.shift = mg.p;
    for (int r = 0; r < R; ++r) a.tab[r] = gf::perm_table(p.coef[r0 + r]);
    const uint64_t per_launch = kMaxIndex / segs64;
    for (uint64_t s0 = 0; s0 < p.stripes; s0 += per_launch) {
        const uint64_t ns = std::min<uint64_t>(per_launch, p.stripes - s0);
        a.op = p.old_data.ptr + s0 * p.old_data.stride;
        a.os = p.old_data.stride;
        a.np = p.new_data.ptr + s0 * p.new_data.stride;
        a.ns = p.new_data.stride;
        for (int r = 0; r < R; ++r) {
            a.pip[r] = p.par_in[r0 + r].ptr + s0 * p.par_in[r0 + r].stride;
            a.pis[r] = p.par_in[r0 + r].stride;
            a.pop[r] = const_cast<uint8_t*>(p.par_out[r0 + r].ptr) + s0 * p.par_out[r0 + r].stride;
            a.pos[r] = p.par_out[r0 + r].stride;
        }
        a.total = static_cast<uint32_t>(ns * segs64);
        const LaunchShape sh = launch_shape(Family::kUpdate, 2, R, p.len);
        const uint32_t grid = (a.total + sh.block - 1) / sh.block;
        hipLaunchKernelGGL((gf_update_x16<R>), dim3(grid), dim3(sh.block), cap_lds(sh, 0), stream, a);
        const hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

using UpdFn = hipError_t (*)(const UpdateParams&, int, hipStream_t);
const std::array<UpdFn, kFastRows> kUpd = {&launch_update_r<1>, &launch_update_r<2>,
                                           &launch_update_r<3>, &launch_update_r<4>};

bool col_aligned(const Column& c) { return ((reinterpret_cast<uintptr_t>(c.ptr) | c.stride) & 15u) == 0; }

// The last len % 16 bytes of every stripe, as a byte-granular launch.
ApplyParams tail_of(const ApplyParams& p)
{
    ApplyParams q = p;
    const uint64_t body = p.len & ~uint64_t{15};
    for (int j = 0; j < p.cols; ++j) q.src[j].ptr = p.src[j].ptr + body;
    for (int r = 0; r < p.rows; ++r) q.dst[r].ptr = p.dst[r].ptr + body;
    q.len = p.len - body;
    q.hash_base = p.hash_base + body;
    return q;
}

// The update as a (2 + rows)-column product [c_r, c_r, e_r] over [old, new, P...].
ApplyParams update_as_apply(const UpdateParams& p)
{
    ApplyParams q;
    q.len = p.len;
    q.stripes = p.stripes;
    q.cols = 2 + p.rows;
    q.rows = p.rows;
    q.src[0] = p.old_data;
    q.src[1] = p.new_data;
    for (int r = 0; r < p.rows; ++r) {
        q.src[2 + r] = p.par_in[r];
        q.dst[r] = p.par_out[r];
        q.coef[r * q.cols + 0] = p.coef[r];
        q.coef[r * q.cols + 1] = p.coef[r];
        q.coef[r * q.cols + 2 + r] = 1;
    }
    return q;
}

}  // namespace

// One 64-lane copy at byte offsets +1 in, +3 out of a 16-byte vector per lane.
__global__ void unaligned_probe_kernel(const uint8_t* in, uint8_t* out)
{
    store_nt(out + 3 + 16 * threadIdx.x, load_nt(in + 1 + 16 * threadIdx.x));
}

namespace {
int probe_unaligned()  // 1 exact, 0 not (or the probe could not run)
{
    constexpr size_t n = 64 * 16 + 32;
    uint8_t h[n], r[n];
    for (size_t i = 0; i < n; ++i) h[i] = static_cast<uint8_t>(i * 37 + 11);
    hipStream_t st = nullptr;
    uint8_t *a = nullptr, *b = nullptr;
    bool ok = hipStreamCreateWithFlags(&st, hipStreamNonBlocking) == hipSuccess &&
              hipMalloc(reinterpret_cast<void**>(&a), n) == hipSuccess &&
              hipMalloc(reinterpret_cast<void**>(&b), n) == hipSuccess &&
              hipMemcpyAsync(a, h, n, hipMemcpyHostToDevice, st) == hipSuccess &&
              hipMemsetAsync(b, 0, n, st) == hipSuccess;
    if (ok) {
        hipLaunchKernelGGL(unaligned_probe_kernel, dim3(1), dim3(64), 0, st, a, b);
        ok = hipGetLastError() == hipSuccess && hipMemcpyAsync(r, b, n, hipMemcpyDeviceToHost, st) == hipSuccess &&
             hipStreamSynchronize(st) == hipSuccess && std::memcmp(r + 3, h + 1, 64 * 16) == 0;
    }
    if (a) (void)hipFree(a);
    if (b) (void)hipFree(b);
    if (st) (void)hipStreamDestroy(st);
    return ok ? 1 : 0;
}
}  // namespace

// gfx9 runs with SH_MEM_CONFIG alignment_mode = unaligned under ROCm's KFD, so a
// dwordx4 access at any byte offset is exact.  Measured on MI355X
// (tools/tune/tune_apply unaligned): every offset exact; an encode-shaped
// stream with columns at +1/+4/+8/+12 B runs at 74.5-77 % of peak, against
// 0.6 % for the byte-granular kernel.  Checked once per device anyway.
bool unaligned_vector_ok()
{
    static std::mutex mu;
    static int8_t state[64] = {};  // 0 unknown, 1 exact, -1 not
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return false;
    std::lock_guard<std::mutex> lock(mu);
    if (state[dev] == 0) state[dev] = probe_unaligned() ? 1 : -1;
    return state[dev] == 1;
}

// HBM ceilings measured with the same access instructions as the coding
// kernels (bench.py reports the coding kernels against them).  KIND 0 read,
// 1 write, 2 copy; 3 and 4 the coding kernels' stream mixes: four input streams
// XORed into one (decode-shaped) or two (encode-shaped) output streams, each
// `segs` segments long, the streams back to back in src / dst.  XCD: block b
// takes the (b % 8)-th eighth of the range, in order (the dispatcher deals
// blocks to the 8 XCDs round robin, so each XCD streams one contiguous eighth).
template <int KIND, bool XCD>
__global__ __launch_bounds__(kBlock) void hbm_probe_kernel(const uint8_t* in, uint8_t* out, uint64_t segs)
{
    uint64_t blk = blockIdx.x;
    if constexpr (XCD) blk = (blk % 8) * (gridDim.x / 8) + blk / 8;
    const uint64_t i = blk * blockDim.x + threadIdx.x;
    if (i >= segs) return;
    if constexpr (KIND == 0) {
        const uint4 v = load_nt(in + i * 16);
        // never true for the probe's data; keeps the load live (a per-lane vector store)
        if ((v.x ^ v.y ^ v.z ^ v.w) == 0x9E3779B9u) reinterpret_cast<uint32_t*>(out)[threadIdx.x & 63u] = 1;
    } else if constexpr (KIND == 1) {
        store_nt(out + i * 16, make_uint4(static_cast<uint32_t>(i), 1u, 2u, 3u));
    } else if constexpr (KIND == 2) {
        store_nt(out + i * 16, load_nt(in + i * 16));
    } else {
        uint4 v[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) v[j] = load_nt(in + (j * segs + i) * 16);
        const uint4 x = make_uint4(v[0].x ^ v[1].x ^ v[2].x ^ v[3].x, v[0].y ^ v[1].y ^ v[2].y ^ v[3].y,
                                   v[0].z ^ v[1].z ^ v[2].z ^ v[3].z, v[0].w ^ v[1].w ^ v[2].w ^ v[3].w);
        store_nt(out + i * 16, x);
        if constexpr (KIND == 4) store_nt(out + (segs + i) * 16, make_uint4(x.x + 1u, x.y, x.z, x.w));
    }
}

template <int KIND>
void launch_probe(bool xcd, uint64_t grid, int block, size_t lds, hipStream_t stream, const uint8_t* in, uint8_t* out,
                  uint64_t segs)
{
    if (xcd)
        hipLaunchKernelGGL((hbm_probe_kernel<KIND, true>), dim3(static_cast<uint32_t>(grid)), dim3(block), lds, stream, in,
                           out, segs);
    else
        hipLaunchKernelGGL((hbm_probe_kernel<KIND, false>), dim3(static_cast<uint32_t>(grid)), dim3(block), lds, stream,
                           in, out, segs);
}

hipError_t hbm_probe(int kind, const void* src, void* dst, size_t bytes, int block, int waves, hipStream_t stream)
{
    (void)hipGetLastError();
    const bool xcd = (kind & 0x100) != 0;
    kind &= 0xFF;
    if (kind < 0 || kind > 4 || bytes % 16 || (block != 64 && block != 128 && block != 256) || waves < 0 || !dst ||
        (kind != 1 && !src))
        return hipErrorInvalidValue;
    const uint64_t segs = bytes / 16;
    const uint64_t grid = (segs + block - 1) / block;
    if (grid == 0) return hipSuccess;
    if (grid > 0x7FFFFFFFull || (xcd && (grid % 8 || segs % block))) return hipErrorInvalidValue;
    const auto* in = static_cast<const uint8_t*>(src);
    auto* out = static_cast<uint8_t*>(dst);
    const size_t lds = cap_lds(block, 0, waves);
    switch (kind) {
    case 0: launch_probe<0>(xcd, grid, block, lds, stream, in, out, segs); break;
    case 1: launch_probe<1>(xcd, grid, block, lds, stream, in, out, segs); break;
    case 2: launch_probe<2>(xcd, grid, block, lds, stream, in, out, segs); break;
    case 3: launch_probe<3>(xcd, grid, block, lds, stream, in, out, segs); break;
    default: launch_probe<4>(xcd, grid, block, lds, stream, in, out, segs); break;
    }
    return hipGetLastError();
}

// Host <-> device gathers and scatters of the host path's direct batches
// (host_path.cpp): one block per piece of at most kMaxPieceBytes, 16-byte
// vector loads and stores at any byte offset (unaligned_vector_ok; the byte
// loop otherwise), non-temporal both ways (every byte is moved once).  One of
// the two ends is page-locked host memory, read or written over PCIe through
// its device address (a locked caller unit or an elect_ec_host_alloc /
// arena buffer, mapped at its host address): round 5 measured such kernels
// at 49 GB/s reading and 51 GB/s writing host memory
// (profiles/r05/register_overlap.txt, part 4), with no DMA engine and no
// runtime transfer call per unit.
template <bool VEC, bool NT, int U>
__global__ __launch_bounds__(kBlock) void copy_pieces_kernel(const CopyPiece* __restrict__ pieces, uint32_t n)
{
  // The piece table lies in page-locked host memory: the block's next descriptor
  // is read while this piece's data moves, so its PCIe round trip is not paid
  // between pieces (round 6: 16 KiB pieces for pipelined steps).
  CopyPiece next = blockIdx.x < n ? pieces[blockIdx.x] : CopyPiece{};
  for (uint32_t pi = blockIdx.x; pi < n; pi += gridDim.x) {
    const CopyPiece pc = next;
    if (pi + gridDim.x < n) next = pieces[pi + gridDim.x];
    const uint32_t vecs = VEC ? pc.n / 16 : 0;
    uint32_t v = threadIdx.x;
    // U loads in flight per lane before their stores
    for (; v + (U - 1) * kBlock < vecs; v += U * kBlock) {
        uint4 x[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint8_t* s = pc.src + (v + u * kBlock) * 16;
            if constexpr (NT)
                x[u] = load_nt(s);
            else
                __builtin_memcpy(&x[u], s, 16);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            uint8_t* d = pc.dst + (v + u * kBlock) * 16;
            if constexpr (NT)
                store_nt(d, x[u]);
            else
                __builtin_memcpy(d, &x[u], 16);
        }
    }
    for (; v < vecs; v += kBlock) {
        uint4 x;
        __builtin_memcpy(&x, pc.src + v * 16, 16);
        __builtin_memcpy(pc.dst + v * 16, &x, 16);
    }
    for (uint32_t b = vecs * 16 + threadIdx.x; b < pc.n; b += kBlock) pc.dst[b] = pc.src[b];
  }
}

hipError_t launch_copy_pieces(const CopyPiece* pieces, uint32_t n, hipStream_t stream)
{
    (void)hipGetLastError();
    if (n == 0) return hipSuccess;
    if (n > 0x7FFFFFFFu) return hipErrorInvalidValue;
    // ELECT_EC_COPY_VARIANT (A/B): 0 plain loads/stores, 4 in flight; 1 non-temporal, 4 in flight;
    // 2 plain, one at a time (the default since the completion poller: 64 callers 49.55-49.66
    // against 48.80-48.96 GiB/s, 8 callers 42.9-44.0 against 42.3-43.3, 3 interleaved runs,
    // profiles/r05/hostpath_low_concurrency.txt); 3 non-temporal, one at a time
    static const int variant = [] {
        const char* e = std::getenv("ELECT_EC_COPY_VARIANT");
        return e ? std::atoi(e) : 2;
    }();
    // Few blocks (ELECT_EC_COPY_BLOCKS, default 128, half a block per CU): the copies wait on
    // PCIe, and a full-chip grid of them held the coding launches of other batches off the CUs
    // (round 5 kernel trace: a 66 us encode stretched to 3.8-5.3 ms beside the copies).  64
    // callers on ELECT's codeLength, pageable units (profiles/r05/hostpath_copy_ab.txt): 64 /
    // 128 / 256 / 512 / 2048 blocks 44.7 / 47.9 / 44.4 / 39.2 / 38.1 GiB/s.
    static const uint32_t cap = [] {
        const char* e = std::getenv("ELECT_EC_COPY_BLOCKS");
        const int v = e ? std::atoi(e) : 128;
        return static_cast<uint32_t>(v > 0 ? v : 128);
    }();
    const uint32_t grid = std::min(n, cap);
    if (!unaligned_vector_ok())
        hipLaunchKernelGGL((copy_pieces_kernel<false, false, 1>), dim3(grid), dim3(kBlock), 0, stream, pieces, n);
    else if (variant == 1)
        hipLaunchKernelGGL((copy_pieces_kernel<true, true, 4>), dim3(grid), dim3(kBlock), 0, stream, pieces, n);
    else if (variant == 2)
        hipLaunchKernelGGL((copy_pieces_kernel<true, false, 1>), dim3(grid), dim3(kBlock), 0, stream, pieces, n);
    else if (variant == 3)
        hipLaunchKernelGGL((copy_pieces_kernel<true, true, 1>), dim3(grid), dim3(kBlock), 0, stream, pieces, n);
    else
        hipLaunchKernelGGL((copy_pieces_kernel<true, false, 4>), dim3(grid), dim3(kBlock), 0, stream, pieces, n);
    return hipGetLastError();
}

// Stream-mix ceiling probe (elect_ec_mix_probe): the access pattern of a coding
// launch with the GF arithmetic taken out.  NIN input columns, NOUT output
// columns, one 16-byte segment per lane of whole segments; an input with a
// content length reads only its content (the segment holding the end whole,
// masked), as the padded kernels do; every output is the XOR of the inputs.
// What a kernel of that shape could reach on this device: the bench reports
// the padded and fused-step kernels as fractions of it.
struct MixArgs {
    const uint8_t* sp[8];
    uint64_t ss[8];
    uint8_t* dp[4];
    uint64_t ds[4];
    const uint32_t* lens;  // [stripe][nin] or null (every input whole)
    uint32_t segs, total, magic, shift, len32;
};

template <int NIN, int NOUT>
__global__ __launch_bounds__(kBlock) void mix_probe_kernel(const MixArgs a)
{
    const uint32_t idx = blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= a.total) return;
    const uint32_t stripe = static_cast<uint32_t>((static_cast<uint64_t>(idx) * a.magic) >> a.shift);
    const uint32_t off = (idx - stripe * a.segs) * 16u;
    uint4 x = make_uint4(0, 0, 0, 0);
#pragma unroll
    for (int j = 0; j < NIN; ++j) {
        const uint32_t valid = a.lens ? min(a.lens[static_cast<uint64_t>(stripe) * NIN + j], a.len32) : a.len32;
        if (off >= valid) continue;
        uint4 v = load_nt(a.sp[j] + stripe * a.ss[j] + off);
        if (off + 16 > valid) v = keep_bytes(v, valid - off);
        x = make_uint4(x.x ^ v.x, x.y ^ v.y, x.z ^ v.z, x.w ^ v.w);
    }
#pragma unroll
    for (int r = 0; r < NOUT; ++r) store_nt(a.dp[r] + stripe * a.ds[r] + off, make_uint4(x.x + r, x.y, x.z, x.w));
}

hipError_t mix_probe(int nin, int nout, uint64_t len, uint64_t stripes, const Column* src, const uint32_t* lens,
                     const Column* dst, int block, int waves, hipStream_t stream)
{
    (void)hipGetLastError();
    if (nin < 1 || nin > 8 || nout < 1 || nout > 4 || (block != 64 && block != 128 && block != 256) || waves < 0)
        return hipErrorInvalidValue;
    const uint64_t segs = len / 16;
    if (segs == 0 || stripes == 0) return hipSuccess;
    if (segs * stripes > kMaxIndex || len > 0xFFFFFFFFull) return hipErrorInvalidValue;
    MixArgs a{};
    for (int j = 0; j < nin; ++j) {
        a.sp[j] = src[j].ptr;
        a.ss[j] = src[j].stride;
    }
    for (int r = 0; r < nout; ++r) {
        a.dp[r] = const_cast<uint8_t*>(dst[r].ptr);
        a.ds[r] = dst[r].stride;
    }
    a.lens = lens;
    a.segs = static_cast<uint32_t>(segs);
    a.total = static_cast<uint32_t>(segs * stripes);
    const Magic mg = make_magic(a.segs);
    a.magic = mg.m;
    a.shift = mg.p;
    a.len32 = static_cast<uint32_t>(len);
    const dim3 grid((a.total + block - 1) / block);
    const size_t lds = cap_lds(block, 0, waves);
    switch (nin * 10 + nout) {
    case 41: hipLaunchKernelGGL((mix_probe_kernel<4, 1>), grid, dim3(block), lds, stream, a); break;
    case 42: hipLaunchKernelGGL((mix_probe_kernel<4, 2>), grid, dim3(block), lds, stream, a); break;
    case 82: hipLaunchKernelGGL((mix_probe_kernel<8, 2>), grid, dim3(block), lds, stream, a); break;
    case 84: hipLaunchKernelGGL((mix_probe_kernel<8, 4>), grid, dim3(block), lds, stream, a); break;
    default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

bool apply_is_aligned(const ApplyParams& p)
{
    for (int j = 0; j < p.cols; ++j)
        if (!col_aligned(p.src[j])) return false;
    for (int r = 0; r < p.rows; ++r)
        if (!col_aligned(p.dst[r])) return false;
    return true;
}

hipError_t launch_apply_impl(const ApplyParams& p_in, hipStream_t stream)
{
    // Launch errors are read back with hipGetLastError, which also returns an
    // earlier failure of any HIP call on this thread (a failed hipMalloc, say):
    // drop that first, so only this call's launches are judged.
    (void)hipGetLastError();
    if (p_in.cols < 1 || p_in.cols > kMaxCols || p_in.rows < 1 || p_in.rows > kMaxRows) return hipErrorInvalidValue;
    if (p_in.stripes == 0) return hipSuccess;
    ApplyParams p = p_in;
    // Hashed launches wider than the widest hashed vector instance (an update of
    // an m >= 9 code: 2 + m columns) take the byte-granular kernel, which adds
    // its hash terms atomically (seeded below).
    const bool wide_hash = p.hashes && p.cols > kMaxHashCols;
    p.aligned16 = apply_is_aligned(p);
    const bool vec = p.aligned16 || unaligned_vector_ok();  // dwordx4 kernels usable
    const uint32_t tiles = std::max<uint32_t>(1, p.tiles);
    const uint64_t ulen = p.unit_len ? p.unit_len : p.len;
    if (tiles > 1 && (!p.padded || p.len == 0 || p.len % 16 || p.stripes % tiles || ulen > tiles * p.len ||
                      !vec || p.cols > kMaxPadCols || wide_hash))
        return hipErrorInvalidValue;  // tiling rides on the padded vector kernels only
    if (p.hashes && p.hash_seed) {
        // Assign mode needs the one-segment fast kernel with >= 64 segments per hashed
        // unit (every wave within two units); anything else seeds the entries and adds.
        const bool fast = vec && (!p.padded || p.cols <= kMaxPadCols) && !wide_hash;
        const uint64_t segs = (p.padded ? (p.len + 15) / 16 : p.len / 16) * tiles;
        if (!fast || segs < 64) {
            const hipError_t e = hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(p.hashes), static_cast<int>(pow31(ulen)),
                                                   p.stripes / tiles * p.hash_stride, stream);
            if (e != hipSuccess) return e;
            p.hash_seed = false;
        }
    }
    if (p.len == 0) return hipSuccess;
    if (p.padded) {
        for (int j = 0; j < p.cols; ++j)
            if ((!p.lens || (p.lens_cols && j >= p.lens_cols)) && p.clen[j] > ulen) return hipErrorInvalidValue;
        if (!vec || p.cols > kMaxPadCols || wide_hash) return launch_bytes(p, stream);
        for (int r0 = 0; r0 < p.rows; r0 += kFastRows) {
            const int nr = std::min(kFastRows, p.rows - r0);
            const hipError_t e = kRows[p.cols - 1].pad[nr - 1](p, r0, stream);
            if (e != hipSuccess) return e;
        }
        return hipSuccess;
    }
    if (!vec || wide_hash) return launch_bytes(p, stream);
    for (int r0 = 0; r0 < p.rows; r0 += kFastRows) {
        const int nr = std::min(kFastRows, p.rows - r0);
        const hipError_t e = kRows[p.cols - 1].fast[nr - 1](p, r0, stream);
        if (e != hipSuccess) return e;
    }
    return (p.len & 15) ? launch_bytes(tail_of(p), stream) : hipSuccess;
}

hipError_t launch_apply(const ApplyParams& p_in, hipStream_t stream)
{
    if (!p_in.hashes || p_in.hash_scratch || p_in.len == 0 || p_in.stripes == 0)
        return launch_apply_impl(p_in, stream);
    // hashed, no caller scratch: the stream's cached buffer (scratch_lease)
    const uint64_t segs = p_in.padded ? (p_in.len + 15) / 16 : p_in.len / 16;
    const uint64_t total = std::min<uint64_t>(segs * p_in.stripes, kMaxIndex);
    ScratchEntry* e = nullptr;
    hipError_t err = scratch_lease(stream, hash_scratch_need(total), &e);
    if (err != hipSuccess) return err;
    ApplyParams p = p_in;
    p.hash_scratch = e->ptr;
    p.hash_scratch_words = e->words;
    err = launch_apply_impl(p, stream);
    const hipError_t r = scratch_release(e, stream);
    return err != hipSuccess ? err : r;
}

// Several plain batches with one coefficient matrix: grouped into as few launches
// as the group kernel allows (kMaxGroup parts, each under 2^31 segments, whole
// 16-byte segments, vector kernels usable); anything else launches alone.
hipError_t launch_apply_many(const ApplyParams* ps, int n, hipStream_t stream)
{
    (void)hipGetLastError();  // as launch_apply_impl
    if (n < 0 || (n > 0 && !ps)) return hipErrorInvalidValue;
    std::vector<ApplyParams> grouped;
    for (int i = 0; i < n; ++i) {
        ApplyParams p = ps[i];
        if (p.cols < 1 || p.cols > kMaxCols || p.rows < 1 || p.rows > kMaxRows) return hipErrorInvalidValue;
        if (i > 0 && (p.cols != ps[0].cols || p.rows != ps[0].rows ||
                      std::memcmp(p.coef, ps[0].coef, sizeof(p.coef)) != 0))
            return hipErrorInvalidValue;  // one coefficient matrix per call
        if (p.stripes == 0 || p.len == 0) continue;
        p.aligned16 = apply_is_aligned(p);
        const bool groupable = !p.padded && !p.hashes && p.tiles <= 1 && p.len % 16 == 0 &&
                               (p.len / 16) * p.stripes <= kMaxIndex && (p.aligned16 || unaligned_vector_ok());
        if (groupable) {
            grouped.push_back(p);
            continue;
        }
        const hipError_t e = launch_apply_impl(p, stream);
        if (e != hipSuccess) return e;
    }
    // Batches group in submission order, kMaxGroup per launch.
    for (size_t g0 = 0; g0 < grouped.size();) {
        const size_t g1 = std::min(grouped.size(), g0 + kMaxGroup);
        const int m = static_cast<int>(g1 - g0);
        if (m == 1) {  // nothing to group with: the plain launcher
            const hipError_t e = launch_apply_impl(grouped[g0], stream);
            if (e != hipSuccess) return e;
        } else {
            const ApplyParams& p0 = grouped[g0];
            for (int r0 = 0; r0 < p0.rows; r0 += kFastRows) {
                const int nr = std::min(kFastRows, p0.rows - r0);
                const hipError_t e = kRows[p0.cols - 1].group[nr - 1](grouped.data() + g0, m, r0, stream);
                if (e != hipSuccess) return e;
            }
        }
        g0 = g1;
    }
    return hipSuccess;
}

hipError_t launch_update(const UpdateParams& p, hipStream_t stream)
{
    (void)hipGetLastError();  // as launch_apply_impl
    if (p.rows < 1 || p.rows > kMaxRows || p.rows + 2 > kMaxCols) return hipErrorInvalidValue;
    if (p.len == 0 || p.stripes == 0) return hipSuccess;
    bool aligned = col_aligned(p.old_data) && col_aligned(p.new_data);
    for (int r = 0; r < p.rows; ++r) aligned = aligned && col_aligned(p.par_in[r]) && col_aligned(p.par_out[r]);
    if (!aligned && !unaligned_vector_ok()) return launch_bytes(update_as_apply(p), stream);
    for (int r0 = 0; r0 < p.rows; r0 += kFastRows) {
        const int nr = std::min(kFastRows, p.rows - r0);
        const hipError_t e = kUpd[nr - 1](p, r0, stream);
        if (e != hipSuccess) return e;
    }
    return (p.len & 15) ? launch_bytes(tail_of(update_as_apply(p)), stream) : hipSuccess;
}

}  // namespace kern
}  // namespace elect
