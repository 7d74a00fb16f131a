// rs_impl.hpp — the gfx950 GF(2^8) kernels and their launch templates.
//
// Shared by rs_kernels.hip (dispatch, hash scratch, the byte-granular and
// update paths) and rs_inst.hip, which is compiled once per source-column
// count K (ELECT_EC_INST_K = 1..16) so that the few hundred kernel instances
// build in parallel.  Everything below sits in an anonymous namespace, so each
// translation unit keeps its own copies; only kernel_rows_kK() crosses units.
//
// rs_kernels.hip — gfx950 (MI355X, CDNA4) kernels for ELECT's Reed-Solomon path.
//
// The reference runs every encode/decode byte through ISA-L's ec_encode_data
// (EC/erasure_coder.c:90 and :221) and every parity update through
// ec_encode_data_update (EC/erasure_coder.c:128), one stripe per CPU thread.
// Here a launch covers a whole batch of stripes.
//
// Work unit: a 16-byte segment of one stripe.  A lane loads the segment from
// each source column (global_load_dwordx4, 1 KiB contiguous per wave
// instruction), multiplies and XOR-accumulates it into every output row in
// registers, and stores each row's 16 bytes (global_store_dwordx4).  Each input
// byte is read once and each output byte written once, so the kernel streams
// (cols + rows) x len bytes per stripe and is bound by HBM, not by ALU.
//
// GF(2^8) multiply by a wave-uniform coefficient c uses byte shuffles, not
// MFMA: split x into bit fields x[2:0], x[5:3], x[7:6]; then
//   c*x = T0[x[2:0]] ^ T1[x[5:3]] ^ T2[x[7:6]]
// (GF multiplication is linear over GF(2)).  An 8-entry byte table is two
// dwords, so ONE v_perm_b32 looks up four bytes at once.  The tables are
// staged in LDS per workgroup and read with wave-uniform (broadcast) ds_reads.
// Per data dword: 5 VALU ops for the three bit-field selectors (shared by all
// rows) + per row 3 v_perm + 2 XOR (one v_bitop3 XOR3).
//
// Tails: ELECT's chunk length (ceil(sstable_size * 1.05), StorageService.java:
// 331-339) is not a multiple of 16.  The dwordx4 kernels cover the whole
// 16-byte segments of every stripe; the last len % 16 bytes per stripe go to a
// second, byte-granular launch.  Layouts whose column starts are not all
// 16-byte aligned run the byte-granular kernel for everything (any pointer).
#pragma once

#include <hip/hip_runtime.h>

#include <algorithm>
#include <array>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <vector>

#include "rs_kernels.hpp"

namespace elect {
namespace kern {

using FastFn = hipError_t (*)(const ApplyParams&, int, hipStream_t);
using GroupFn = hipError_t (*)(const ApplyParams*, int, int, hipStream_t);
using FastRow = std::array<FastFn, kFastRows>;
using GroupRow = std::array<GroupFn, kFastRows>;

// The launchers of one source-column count K, for R = 1..4 output rows: plain,
// padded (K <= kMaxPadCols, else null) and grouped.  Defined in rs_inst.hip.
struct KernelRows {
    FastRow fast{};
    FastRow pad{};
    GroupRow group{};
};
#define ELECT_EC_DECLARE_ROWS(K) KernelRows kernel_rows_k##K();
ELECT_EC_DECLARE_ROWS(1) ELECT_EC_DECLARE_ROWS(2) ELECT_EC_DECLARE_ROWS(3) ELECT_EC_DECLARE_ROWS(4)
ELECT_EC_DECLARE_ROWS(5) ELECT_EC_DECLARE_ROWS(6) ELECT_EC_DECLARE_ROWS(7) ELECT_EC_DECLARE_ROWS(8)
ELECT_EC_DECLARE_ROWS(9) ELECT_EC_DECLARE_ROWS(10) ELECT_EC_DECLARE_ROWS(11) ELECT_EC_DECLARE_ROWS(12)
ELECT_EC_DECLARE_ROWS(13) ELECT_EC_DECLARE_ROWS(14) ELECT_EC_DECLARE_ROWS(15) ELECT_EC_DECLARE_ROWS(16)
#undef ELECT_EC_DECLARE_ROWS

namespace {


constexpr int kBlock = 256;

// q = (n * m) >> p is exact floor(n / d) for every n < 2^31 (m = ceil(2^p/d),
// p = 31 + ceil(log2 d); the rounding error m*d - 2^p < d keeps n*err < 2^p).
struct Magic {
    uint32_t m;
    uint32_t p;
};

Magic make_magic(uint32_t d)
{
    uint32_t l = 0;
    while ((uint64_t{1} << l) < d) ++l;
    const uint32_t p = 31 + l;
    const uint64_t m = ((uint64_t{1} << p) + d - 1) / d;
    return Magic{static_cast<uint32_t>(m), p};
}

constexpr uint64_t kMaxIndex = (uint64_t{1} << 31) - 1;

__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c)
{
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}

// One coefficient applied to four packed bytes, given the three selectors.
__device__ __forceinline__ uint32_t gf_lookup(const gf::PermTable& t, uint32_t s0, uint32_t s1,
                                              uint32_t s2)
{
    return xor3(__builtin_amdgcn_perm(t.t0_hi, t.t0_lo, s0),
                __builtin_amdgcn_perm(t.t1_hi, t.t1_lo, s1), __builtin_amdgcn_perm(t.t2, t.t2, s2));
}

struct Sel {
    uint32_t s0, s1, s2;
};

__device__ __forceinline__ Sel selectors(uint32_t x)
{
    return Sel{x & 0x07070707u, (x >> 3) & 0x07070707u, (x >> 6) & 0x03030303u};
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

// Streaming loads/stores: every byte is touched once, so keep it out of the
// caches' way (global_load/store ... nt).  Measured on MI355X with
// tools/tune/tune_apply.hip: +6-10 % over plain loads/stores on every BASELINE
// shape ("Kernel tuning").
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

// Partial segments (padded launches only): n < 16 valid bytes, zero filled.
__device__ __forceinline__ uint4 load_partial(const uint8_t* p, uint32_t n)
{
    uint4 v = make_uint4(0, 0, 0, 0);
#pragma unroll
    for (int w = 0; w < 4; ++w) {
        uint32_t x = 0;
#pragma unroll
        for (int b = 0; b < 4; ++b)
            if (static_cast<uint32_t>(4 * w + b) < n) x |= static_cast<uint32_t>(p[4 * w + b]) << (8 * b);
        set_word(v, w, x);
    }
    return v;
}

__device__ __forceinline__ uint4 keep_bytes(const uint4& v, uint32_t n)  // bytes [0, n) of 16
{
    uint4 o;
#pragma unroll
    for (int w = 0; w < 4; ++w) {
        const uint32_t lo = 4 * w;
        const uint32_t keep = n >= lo + 4 ? 0xFFFFFFFFu : n <= lo ? 0u : ((1u << (8 * (n - lo))) - 1u);
        set_word(o, w, lane_word(v, w) & keep);
    }
    return o;
}

__device__ __forceinline__ void store_partial(uint8_t* p, const uint4& v, uint32_t n)
{
#pragma unroll
    for (int w = 0; w < 4; ++w) {
        const uint32_t x = lane_word(v, w);
#pragma unroll
        for (int b = 0; b < 4; ++b)
            if (static_cast<uint32_t>(4 * w + b) < n) p[4 * w + b] = static_cast<uint8_t>(x >> (8 * b));
    }
}

// ---------------------------------------------------------------------------
// Fused parity hash (java.nio.ByteBuffer.hashCode), see ApplyParams::hashes.
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint32_t dpow31(uint64_t e)
{
    uint32_t r = 1, b = 31;
    for (; e; e >>= 1, b *= b)
        if (e & 1) r *= b;
    return r;
}

// sum_t sb[t] * 31^t over the 16 bytes of a segment.  v_dot4_i32_i8 reads the
// bytes as signed int8, which is Java's byte: per dword D = (b0 + 31 b1) +
// 961 (b2 + 31 b3), |D| < 2^22.  Then D0 + 31^4 D1 and D2 + 31^4 D3 as 24-bit
// multiplies (full rate; the low 32 bits are exact mod 2^32), and one 32-bit
// multiply by 31^8 (v_mul_lo_u32 is quarter rate: one instead of a three-step
// Horner chain).
__device__ __forceinline__ uint32_t horner31(const uint4& v)
{
    int d[4];
#pragma unroll
    for (int w = 0; w < 4; ++w) {
        const int x = static_cast<int>(lane_word(v, w));
        const int lo = __builtin_amdgcn_sdot4(x, 0x00001F01, 0, false);
        const int hi = __builtin_amdgcn_sdot4(x, 0x1F010000, 0, false);
        d[w] = __mul24(hi, 961) + lo;
    }
    constexpr uint32_t kP4 = 923521u;  // 31^4 (< 2^23)
    constexpr uint32_t kP8 = kP4 * kP4;  // 31^8 mod 2^32
    const uint32_t t01 = static_cast<uint32_t>(__mul24(d[1], static_cast<int>(kP4)) + d[0]);
    const uint32_t t23 = static_cast<uint32_t>(__mul24(d[3], static_cast<int>(kP4)) + d[2]);
    return t23 * kP8 + t01;
}

// 31^(16*seg) for a 32-bit segment index seg, from four 256-entry tables
// (31^(16 * j * 256^i)): four scalar loads and three multiplies instead of a
// square-and-multiply loop in the wave's epilogue.
struct SegPow {
    uint32_t t[4][256];
    constexpr SegPow() : t()
    {
        uint32_t base = 1;
        for (int i = 0; i < 16; ++i) base *= 31u;  // 31^16
        for (int i = 0; i < 4; ++i) {
            uint32_t x = 1;
            for (int j = 0; j < 256; ++j) {
                t[i][j] = x;
                x *= base;
            }
            base = x;  // base^256
        }
    }
};
__constant__ constexpr SegPow kSegPow{};

__device__ __forceinline__ uint32_t pow31_seg(uint32_t seg)
{
    return kSegPow.t[0][seg & 255u] * kSegPow.t[1][(seg >> 8) & 255u] * kSegPow.t[2][(seg >> 16) & 255u] *
           kSegPow.t[3][seg >> 24];
}

// 31^(16*lane) for lane 0..63, a compile-time table (constant memory).
struct LanePow {
    uint32_t v[64];
    constexpr LanePow() : v()
    {
        uint32_t p16 = 1;
        for (int i = 0; i < 16; ++i) p16 *= 31u;
        uint32_t x = 1;
        for (int l = 0; l < 64; ++l) {
            v[l] = x;
            x *= p16;
        }
    }
};
__constant__ constexpr LanePow kLanePow{};

// Sum over the 64 lanes, returned wave-uniform.  DPP adds (no LDS traffic):
// quad swaps and row rotates give every lane its 16-lane row sum, then the
// GFX9 row broadcasts fold rows 0+1 into row 1 and rows 0..2 into row 3, and
// lane 63 holds the total.
template <int Ctrl, int RowMask = 0xF>
__device__ __forceinline__ uint32_t dpp_add(uint32_t v)
{
    return v + static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(v), Ctrl, RowMask, 0xF, false));
}

__device__ __forceinline__ uint32_t wave_sum(uint32_t v)
{
    v = dpp_add<0xB1>(v);        // quad_perm [1,0,3,2]
    v = dpp_add<0x4E>(v);        // quad_perm [2,3,0,1]
    v = dpp_add<0x124>(v);       // row_ror:4
    v = dpp_add<0x128>(v);       // row_ror:8
    v = dpp_add<0x142, 0xA>(v);  // row_bcast:15 into rows 1 and 3
    v = dpp_add<0x143, 0xC>(v);  // row_bcast:31 into rows 2 and 3
    return static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(v), 63));
}

// ---------------------------------------------------------------------------
// Fast path: K source columns, R output rows, one 16-byte segment per lane.
// The byte-shuffle tables (5 dwords per coefficient) are staged in LDS, padded
// to 8 dwords so one ds_read_b128 + one ds_read_b32 (wave-uniform address,
// broadcast) bring a coefficient's tables into VGPRs; keeping 32 coefficients
// (RS(12,8)) in SGPRs instead spills.
// ---------------------------------------------------------------------------
template <int K, int R>
struct FastArgs {
    const uint8_t* sp[K];
    uint64_t ss[K];
    uint8_t* dp[R];
    uint64_t ds[R];
    uint32_t segs;   // whole 16-byte segments per stripe
    uint32_t total;  // segments in this launch (< 2^31)
    uint32_t magic;
    uint32_t shift;
    // padded launches only
    uint64_t len;            // bytes per shard (the last segment may be partial)
    uint32_t len32;          // min(len, 2^32-1): device lengths are clamped to it, so no load
                             // leaves a unit whatever a caller's length array holds
    const uint32_t* lens;    // [stripe][lstride] content lengths of columns < lcols, or null -> clen
    uint32_t lstride;
    uint32_t lcols;          // columns >= lcols hold clen[j] valid bytes
    uint32_t clen[K];
    uint32_t ulen32;         // min(logical unit length, 2^32-1): content lengths clamp to it
    uint32_t tiles;          // coding stripes (tiles) per logical stripe, 1 = untiled
    uint32_t tmagic, tshift; // exact division by tiles
    uint32_t hsegs;          // segments per hashed (logical) unit: tiles * segs
    uint32_t hmagic, hshift; // exact division by hsegs
    int32_t* hashes;        // optional parity hashes, [logical stripe][hstride] (row r at +r)
    uint32_t hstride;
    uint32_t hpow;          // 31^(hash offset of byte 0 of this launch window)
    uint32_t* hpart;        // per-wave partial sums [wave][R]: the wave's first stripe
    uint32_t* hpart_hi;     // assign mode: [wave][R] sums of a straddling wave's second stripe, else null
    gf::PermTable tab[R][K];
};

constexpr int kTabStride = 8;  // dwords per coefficient in LDS

__device__ __forceinline__ uint32_t div_magic(uint32_t n, uint32_t m, uint32_t sh)
{
    return static_cast<uint32_t>((static_cast<uint64_t>(n) * m) >> sh);
}

// Valid bytes of one tile (offset tb in its unit, tl bytes long) of a unit
// holding `raw` content bytes.  Untiled: tb = 0 and raw <= tl, so raw itself.
__device__ __forceinline__ uint32_t tile_valid(uint32_t raw, uint32_t tb, uint32_t tl)
{
    return raw > tb ? min(raw - tb, tl) : 0u;
}

// Content bytes of column j of coding stripe `stripe` (its logical stripe's
// length from lens, or clen), as the tile's share.
template <int K, typename A>
__device__ __forceinline__ void tile_lengths(const A& a, uint32_t stripe, uint32_t (&valid)[K], bool scalar)
{
    const uint32_t g = div_magic(stripe, a.tmagic, a.tshift);
    const uint32_t tb = (stripe - g * a.tiles) * a.len32;
    const uint32_t* l = a.lens ? a.lens + static_cast<uint64_t>(g) * a.lstride : nullptr;
#pragma unroll
    for (int j = 0; j < K; ++j) {
        uint32_t raw = a.clen[j];
        if (l && j < static_cast<int>(a.lcols)) {
            const uint32_t v = scalar ? static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(l[j])) : l[j];
            raw = min(v, a.ulen32);
        }
        valid[j] = tile_valid(raw, tb, a.len32);
    }
}

// cmask (wave-uniform): columns to include; the others are known zero for the
// whole wave and are skipped by a scalar branch (padded launches).
// Unmasked launches take columns in pairs: the six lookups of a pair fold into
// the accumulator with three XOR3s (v_bitop3), 9 VALU ops per pair, row and
// dword against 10 one column at a time (RS(12,8) encode: -48 of 887 per wave).
template <int K, int R>
__device__ __forceinline__ void gf_combine_pairs(const uint4 (&x)[K], const uint32_t* tl, uint4 (&acc)[R])
{
#pragma unroll
    for (int j = 0; j < K; j += 2) {
        constexpr int kPair = 2;
        const bool two = j + 1 < K;
        uint32_t s0[kPair][4], s1[kPair][4], s2[kPair][4];
#pragma unroll
        for (int c = 0; c < kPair; ++c)
#pragma unroll
            for (int w = 0; w < 4; ++w) {
                const Sel sl = selectors(lane_word(x[(c == 0 || !two) ? j : j + 1], w));
                s0[c][w] = sl.s0;
                s1[c][w] = sl.s1;
                s2[c][w] = sl.s2;
            }
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const uint32_t* ta = &tl[(r * K + j) * kTabStride];
            const uint4 qa = *reinterpret_cast<const uint4*>(ta);
            const uint32_t a2 = ta[4];
            uint4 qb = qa;
            uint32_t b2 = a2;
            if (two) {
                const uint32_t* tb = &tl[(r * K + j + 1) * kTabStride];
                qb = *reinterpret_cast<const uint4*>(tb);
                b2 = tb[4];
            }
#pragma unroll
            for (int w = 0; w < 4; ++w) {
                const uint32_t p0 = __builtin_amdgcn_perm(qa.y, qa.x, s0[0][w]);
                const uint32_t p1 = __builtin_amdgcn_perm(qa.w, qa.z, s1[0][w]);
                const uint32_t p2 = __builtin_amdgcn_perm(a2, a2, s2[0][w]);
                uint32_t v;
                if (!two) {  // odd K: the last column alone
                    v = j == 0 ? xor3(p0, p1, p2) : (xor3(lane_word(acc[r], w), p0, p1) ^ p2);
                } else {
                    const uint32_t q0 = __builtin_amdgcn_perm(qb.y, qb.x, s0[1][w]);
                    const uint32_t q1 = __builtin_amdgcn_perm(qb.w, qb.z, s1[1][w]);
                    const uint32_t q2 = __builtin_amdgcn_perm(b2, b2, s2[1][w]);
                    v = j == 0 ? (xor3(xor3(p0, p1, p2), q0, q1) ^ q2)
                               : xor3(xor3(xor3(lane_word(acc[r], w), p0, p1), p2, q0), q1, q2);
                }
                set_word(acc[r], w, v);
            }
        }
    }
}

template <int K, int R, bool MASKED = false>
__device__ __forceinline__ void gf_combine(const uint4 (&x)[K], const uint32_t* tl, uint4 (&acc)[R],
                                           uint32_t cmask = ~0u)
{
#ifndef AB_COMBINE1
    if constexpr (!MASKED) {
        gf_combine_pairs<K, R>(x, tl, acc);
        return;
    }
#endif
    if (MASKED) {
#pragma unroll
        for (int r = 0; r < R; ++r) acc[r] = make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int j = 0; j < K; ++j) {  // column-outer: selectors once, then every row
        if (MASKED && !(cmask & (1u << j))) continue;
        uint32_t s0[4], s1[4], s2[4];
#pragma unroll
        for (int w = 0; w < 4; ++w) {
            const Sel sl = selectors(lane_word(x[j], w));
            s0[w] = sl.s0;
            s1[w] = sl.s1;
            s2[w] = sl.s2;
        }
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const uint4 tq = *reinterpret_cast<const uint4*>(&tl[(r * K + j) * kTabStride]);
            const uint32_t t2 = tl[(r * K + j) * kTabStride + 4];
#pragma unroll
            for (int w = 0; w < 4; ++w) {
                const uint32_t v = xor3(__builtin_amdgcn_perm(tq.y, tq.x, s0[w]),
                                        __builtin_amdgcn_perm(tq.w, tq.z, s1[w]),
                                        __builtin_amdgcn_perm(t2, t2, s2[w]));
                set_word(acc[r], w, (j == 0 && !MASKED) ? v : (lane_word(acc[r], w) ^ v));
            }
        }
    }
}

// Stage the byte-shuffle tables of a launch into LDS (8 dwords per coefficient).
template <int K, int R>
__device__ __forceinline__ void stage_tables(const gf::PermTable (&tab)[R][K], uint32_t* tl)
{
    for (int i = threadIdx.x; i < R * K; i += blockDim.x) {
        const gf::PermTable& t = tab[i / K][i % K];
        tl[i * kTabStride + 0] = t.t0_lo;
        tl[i * kTabStride + 1] = t.t0_hi;
        tl[i * kTabStride + 2] = t.t1_lo;
        tl[i * kTabStride + 3] = t.t1_hi;
        tl[i * kTabStride + 4] = t.t2;
    }
    __syncthreads();
}

// HASH instances (encode shapes only) carry the parity-hash epilogue; keeping
// it out of the others saved RS(12,8) encode ~120 v_mov (acc kept live across
// the stores) and 4 VGPRs.
template <int K, int R, bool PAD, bool HASH>
__global__ __launch_bounds__(kBlock) void gf_apply_x16(const FastArgs<K, R> a)
{
    __shared__ __attribute__((aligned(16))) uint32_t tl[R * K * kTabStride];
    const uint32_t idx_raw = blockIdx.x * blockDim.x + threadIdx.x;
    const bool live = idx_raw < a.total;
    // Lanes past the end of the launch redo the last segment (identical bytes
    // to identical addresses) rather than leave the wave, so wave-wide hash
    // reductions see every lane; their hash terms are zeroed.
    const uint32_t idx = (!HASH || live) ? idx_raw : a.total - 1;
    const uint32_t stripe = static_cast<uint32_t>((static_cast<uint64_t>(idx) * a.magic) >> a.shift);
    const uint64_t off = static_cast<uint64_t>(idx - stripe * a.segs) * 16;

    uint4 x[K];
    // Padded: the content lengths of the wave's first stripe, as scalar loads
    // (wave-uniform) issued before the table staging so that their latency
    // overlaps it; lanes of a wave that straddles stripes reload theirs below.
    // (Hoisting the plain launches' data loads the same way measured 2 % slower.)
    bool uniform = false;
    uint32_t sl[K];
    const uint32_t first = __builtin_amdgcn_readfirstlane(idx_raw);
    if (PAD && a.lens && first < a.total) {  // (a wholly dead wave reads nothing)
        const uint32_t s0 = div_magic(first, a.magic, a.shift);
        const uint32_t s1 = div_magic(first + 63, a.magic, a.shift);
        uniform = s0 == s1;
        tile_lengths<K>(a, s0, sl, true);
    }

    stage_tables<K, R>(a.tab, tl);
    if (HASH ? first >= a.total : !live) return;  // HASH: only wholly dead waves leave
    if (!PAD) {
#pragma unroll
        for (int j = 0; j < K; ++j) x[j] = load_nt(a.sp[j] + stripe * a.ss[j] + off);
    }

    if (PAD) {
        uint32_t valid[K];
        if (a.lens && uniform) {
#pragma unroll
            for (int j = 0; j < K; ++j) valid[j] = sl[j];
        } else {  // all lengths first: vmcnt is in order, so interleaving would serialise
            tile_lengths<K>(a, stripe, valid, false);
        }
        // Full segments first (no loads at all past a column's content length),
        // then the one segment per unit that holds the content end, loaded whole
        // when it lies inside the unit and masked (byte loads only for a unit's
        // last, partial segment: 64 KiB units at 93 % fill ran 64 -> 71.5 % of
        // peak with this), so no load waits on another.
#pragma unroll
        for (int j = 0; j < K; ++j) {
            x[j] = make_uint4(0, 0, 0, 0);
            if (off + 16 <= valid[j]) x[j] = load_nt(a.sp[j] + stripe * a.ss[j] + off);
        }
#pragma unroll
        for (int j = 0; j < K; ++j) {
            if (off < valid[j] && off + 16 > valid[j]) {
                if (off + 16 <= a.len) {
                    x[j] = keep_bytes(load_nt(a.sp[j] + stripe * a.ss[j] + off), static_cast<uint32_t>(valid[j] - off));
                    continue;
                }
                const uint4 t = load_partial(a.sp[j] + stripe * a.ss[j] + off, static_cast<uint32_t>(valid[j] - off));
                x[j] = make_uint4(x[j].x | t.x, x[j].y | t.y, x[j].z | t.z, x[j].w | t.w);
            }
        }
    }

    uint4 acc[R];
    gf_combine<K, R>(x, tl, acc);
    if (!PAD || off + 16 <= a.len) {
#pragma unroll
        for (int r = 0; r < R; ++r) store_nt(a.dp[r] + stripe * a.ds[r] + off, acc[r]);
    } else {
        const uint32_t n = static_cast<uint32_t>(a.len - off);
#pragma unroll
        for (int r = 0; r < R; ++r) store_partial(a.dp[r] + stripe * a.ds[r] + off, acc[r], n);
    }

    if (HASH && a.hashes) {  // fused parity hash
        if (PAD && off + 16 > a.len) {  // a partial last segment: zero the bytes past len
            const uint32_t n = static_cast<uint32_t>(a.len - off);
#pragma unroll
            for (int r = 0; r < R; ++r)
#pragma unroll
                for (int w = 0; w < 4; ++w) {
                    const int lo = 4 * w;
                    const uint32_t keep = n >= static_cast<uint32_t>(lo + 4) ? 0xFFFFFFFFu
                                          : n <= static_cast<uint32_t>(lo) ? 0u : ((1u << (8 * (n - lo))) - 1u);
                    set_word(acc[r], w, lane_word(acc[r], w) & keep);
                }
        }
        // Hashed units are logical stripes (tiles of one unit are consecutive
        // coding stripes): position = flat index - the unit's first segment.
        const uint32_t last = first + 63;
        const uint32_t s_first = div_magic(first, a.hmagic, a.hshift);
        const uint32_t s_last = div_magic(last, a.hmagic, a.hshift);
        const bool whole_wave = last < a.total && s_first == s_last;  // wave-uniform
        const uint32_t hs = div_magic(idx, a.hmagic, a.hshift);       // this lane's hashed unit
        const uint32_t hseg = idx - hs * a.hsegs;                     // its segment inside it
        if (whole_wave) {  // partial sums to scratch; hash_reduce adds them per stripe
            const uint32_t seg0 = first - s_first * a.hsegs;
            const uint32_t p0 = a.hpow * pow31_seg(seg0);
            const uint32_t q = kLanePow.v[threadIdx.x & 63u] * p0;
#pragma unroll
            for (int r = 0; r < R; ++r) {
#if defined(AB_HASH_NOSUM)  // timing probes only (wrong hashes): no wave reduction / no Horner
                const uint32_t sum = horner31(acc[r]) * q;
#elif defined(AB_HASH_NOHORNER)
                const uint32_t sum = wave_sum(acc[r].x * q);
#elif defined(AB_HASH_ROWSUM)  // row sums only (4 DPP steps, no row broadcasts)
                uint32_t v = horner31(acc[r]) * q;
                v = dpp_add<0xB1>(v); v = dpp_add<0x4E>(v); v = dpp_add<0x124>(v); v = dpp_add<0x128>(v);
                const uint32_t sum = v;
#else
                const uint32_t sum = wave_sum(horner31(acc[r]) * q);
#endif
                if ((threadIdx.x & 63u) == 0) a.hpart[static_cast<uint64_t>(first >> 6) * R + r] = sum;
            }
        } else if (a.hpart_hi) {  // assign mode: a wave straddling two stripes (or the launch's end)
            const uint32_t p = live ? a.hpow * pow31_seg(hseg) : 0u;
            const bool lo = hs == s_first;
#pragma unroll
            for (int r = 0; r < R; ++r) {
                const uint32_t v = horner31(acc[r]) * p;
                const uint32_t sum_lo = wave_sum(lo ? v : 0u);
                const uint32_t sum_hi = wave_sum(lo ? 0u : v);
                if ((threadIdx.x & 63u) == 0) {
                    a.hpart[static_cast<uint64_t>(first >> 6) * R + r] = sum_lo;
                    a.hpart_hi[static_cast<uint64_t>(first >> 6) * R + r] = sum_hi;
                }
            }
        } else if (live) {
            const uint32_t p = a.hpow * pow31_seg(hseg);
#pragma unroll
            for (int r = 0; r < R; ++r)
                atomicAdd(reinterpret_cast<unsigned*>(a.hashes) + static_cast<uint64_t>(hs) * a.hstride + r,
                          horner31(acc[r]) * p);
        }
    }
}

// Plain launches whose stripes hold whole waves (segs % 64 == 0, offsets inside a
// stripe below 2^32): every wave lies in one stripe, so its column addresses
// are scalar bases (stripe * stride in SALU) plus one 32-bit lane offset, not a
// 64-bit multiply-add per column and lane (v_mad_u64_u32: 27 per lane in
// RS(12,8) encode, 15 in RS(6,4) encode).
// HASH: every wave lies inside one hashed unit, so it writes one partial per
// row (hash_reduce reads it in either mode: no wave starts outside its unit).
template <int K, int R, bool HASH>
__global__ __launch_bounds__(kBlock) void gf_apply_x16u(const FastArgs<K, R> a)
{
    __shared__ __attribute__((aligned(16))) uint32_t tl[R * K * kTabStride];
    const uint32_t idx = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t first = __builtin_amdgcn_readfirstlane(idx);  // the wave's lane 0
    const uint32_t stripe = div_magic(first, a.magic, a.shift);  // wave-uniform
    const uint32_t off = (idx - stripe * a.segs) * 16u;
    stage_tables<K, R>(a.tab, tl);
    if (first >= a.total) return;  // total % 64 == 0: waves are wholly live or wholly past the end
    uint4 x[K];
#pragma unroll
    for (int j = 0; j < K; ++j) x[j] = load_nt(a.sp[j] + static_cast<uint64_t>(stripe) * a.ss[j] + off);
    uint4 acc[R];
    gf_combine<K, R>(x, tl, acc);
#pragma unroll
    for (int r = 0; r < R; ++r) store_nt(a.dp[r] + static_cast<uint64_t>(stripe) * a.ds[r] + off, acc[r]);
    if constexpr (HASH) {
        if (a.hashes) {
            const uint32_t hs = div_magic(first, a.hmagic, a.hshift);
            const uint32_t q = kLanePow.v[threadIdx.x & 63u] * (a.hpow * pow31_seg(first - hs * a.hsegs));
#pragma unroll
            for (int r = 0; r < R; ++r) {
                const uint32_t sum = wave_sum(horner31(acc[r]) * q);
                if ((threadIdx.x & 63u) == 0) a.hpart[static_cast<uint64_t>(first >> 6) * R + r] = sum;
            }
        }
    }
}

// Padded launches with per-stripe content lengths, no hash, and L % 16 == 0:
// U segments per lane.  The lengths sit on the critical path of every data
// load (no load past a unit's content), so a wave amortises that dependent
// round trip over U x 1 KiB per column instead of 1 KiB; a wave whose 64*U
// segments lie in one stripe reads the lengths once, as scalar loads
// overlapped with the table staging.  The one segment per unit that straddles
// its content length is loaded whole (it lies inside the unit's L bytes) and
// masked, so no byte loads.  Straddling waves take a one-segment-at-a-time path.
constexpr int kAuxNT = 2;  // buffer op cache policy: nt (gfx940 family CPol)

// HASH (add mode only: entries seeded with 31^len by launch_apply): a wave
// inside one stripe sums its U*64 segments' hash terms in registers (constant
// 31^(1024u) weights per slice) and writes ONE partial per row, into the slot
// of its first 64-segment group, zeros into its other U-1 slots (hash_reduce
// adds the slots of every group wholly inside a stripe); a straddling wave
// zeroes its slots and adds per lane atomically.  So the wave reduction is paid
// once per U KiB per column instead of once per KiB (gf_apply_x16<.., HASH>).
template <int U>
struct SlicePow {  // 31^(16*64*u), u < U
    uint32_t v[U];
    constexpr SlicePow() : v()
    {
        uint32_t p = 1;
        for (int i = 0; i < 1024; ++i) p *= 31u;
        uint32_t x = 1;
        for (int u = 0; u < U; ++u) {
            v[u] = x;
            x *= p;
        }
    }
};

template <int K, int R, int U, bool HASH>
__global__ __launch_bounds__(kBlock) void gf_apply_lens(const FastArgs<K, R> a)
{
    __shared__ __attribute__((aligned(16))) uint32_t tl[R * K * kTabStride];
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t first = __builtin_amdgcn_readfirstlane(((blockIdx.x * blockDim.x + threadIdx.x) >> 6) * (64u * U));
    auto stripe_of = [&](uint32_t i) { return static_cast<uint32_t>((static_cast<uint64_t>(i) * a.magic) >> a.shift); };
    bool uniform = false;
    uint32_t s0 = 0, sl[K];
    if (first < a.total) {
        s0 = stripe_of(first);
        uniform = s0 == stripe_of(min(first + 64u * U - 1u, a.total - 1u));
        tile_lengths<K>(a, s0, sl, true);
    }
    stage_tables<K, R>(a.tab, tl);
    if (first >= a.total) return;

    if (uniform) {
        // One buffer descriptor per column whose range ends at the content
        // length rounded up to the segment: the range check turns every load
        // past it into zeros with no memory access, so all loads issue
        // unconditionally, back to back.  The one straddling segment is masked.
        __amdgpu_buffer_rsrc_t rs[K];
#pragma unroll
        for (int j = 0; j < K; ++j)
            rs[j] = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(a.sp[j] + s0 * a.ss[j]), 0,
                                                      static_cast<int>((sl[j] + 15u) & ~15u), 0x00020000);
        uint4 x[U][K];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t off = (first + u * 64u + lane - s0 * a.segs) * 16u;
#pragma unroll
            for (int j = 0; j < K; ++j) {
                const auto v = __builtin_amdgcn_raw_buffer_load_b128(rs[j], static_cast<int>(off), 0, kAuxNT);
                x[u][j] = make_uint4(v[0], v[1], v[2], v[3]);
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t off0 = (first + u * 64u - s0 * a.segs) * 16u;  // the wave's lowest offset
            const uint32_t off = off0 + lane * 16u;
#pragma unroll
            for (int j = 0; j < K; ++j)
                if (off0 < sl[j] && sl[j] < off0 + 1024u && (sl[j] & 15u))  // wave-uniform: this slice holds the content end
                    x[u][j] = keep_bytes(x[u][j], off < sl[j] ? min(sl[j] - off, 16u) : 0u);
        }
        uint32_t hacc[R];
#pragma unroll
        for (int r = 0; r < R; ++r) hacc[r] = 0;
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t idx = first + u * 64u + lane;
            if (idx >= a.total) break;
            const uint64_t off = static_cast<uint64_t>(idx - s0 * a.segs) * 16;
            // Skip the columns of empty units (ELECT's all-zero filler chunks).
            // Skipping every column that is zero for this wave slice was 2-3 %
            // slower at partial fills (interleaved A/B), though 45 % faster
            // with every unit empty; empty units get the same gain.
            uint32_t cmask = 0;
#pragma unroll
            for (int j = 0; j < K; ++j) cmask |= (sl[j] != 0 ? 1u : 0u) << j;
            uint4 acc[R];
            gf_combine<K, R, true>(x[u], tl, acc, cmask);
#pragma unroll
            for (int r = 0; r < R; ++r) store_nt(a.dp[r] + s0 * a.ds[r] + off, acc[r]);
            if constexpr (HASH) {
                constexpr SlicePow<U> kSlice{};
#pragma unroll
                for (int r = 0; r < R; ++r) hacc[r] += u == 0 ? horner31(acc[r]) : horner31(acc[r]) * kSlice.v[u];
            }
        }
        if constexpr (HASH) {
            if (a.hashes) {  // the whole wave again (the slice loop may have left early)
                const uint32_t hs = div_magic(first, a.hmagic, a.hshift);
                const uint32_t q = kLanePow.v[lane] * (a.hpow * pow31_seg(first - hs * a.hsegs));
                const uint64_t slot = first >> 6;
                // hash_reduce reads only 64-segment groups wholly inside the launch: a
                // wave reaching its end adds per lane instead (lanes past it hold 0)
                const bool tail = first + 64u * U > a.total;
#pragma unroll
                for (int r = 0; r < R; ++r) {
                    if (tail) {
                        if (hacc[r]) atomicAdd(reinterpret_cast<unsigned*>(a.hashes) + static_cast<uint64_t>(hs) * a.hstride + r,
                                               hacc[r] * q);
                        if (lane < U && first + 64u * lane < a.total) a.hpart[(slot + lane) * R + r] = 0u;
                        continue;
                    }
                    const uint32_t sum = wave_sum(hacc[r] * q);
                    if (lane < U) a.hpart[(slot + lane) * R + r] = lane == 0 ? sum : 0u;
                }
            }
        }
        return;
    }
    if (HASH && a.hashes) {  // straddling wave: its slots read as zero, terms added per lane below
#pragma unroll
        for (int r = 0; r < R; ++r)
            if (lane < U && first + 64u * lane < a.total) a.hpart[((first >> 6) + lane) * R + r] = 0u;
    }
    for (int u = 0; u < U; ++u) {  // straddling wave: per-lane stripes and lengths
        const uint32_t idx = first + u * 64u + lane;
        if (idx >= a.total) break;
        const uint32_t stripe = stripe_of(idx);
        const uint64_t off = static_cast<uint64_t>(idx - stripe * a.segs) * 16;
        uint32_t valid[K];
        tile_lengths<K>(a, stripe, valid, false);
        uint4 x[K];
#pragma unroll
        for (int j = 0; j < K; ++j) {
            x[j] = make_uint4(0, 0, 0, 0);
            if (off < valid[j]) x[j] = load_nt(a.sp[j] + stripe * a.ss[j] + off);
        }
#pragma unroll
        for (int j = 0; j < K; ++j)
            if (off < valid[j] && off + 16 > valid[j]) x[j] = keep_bytes(x[j], static_cast<uint32_t>(valid[j] - off));
        uint4 acc[R];
        gf_combine<K, R>(x, tl, acc);
#pragma unroll
        for (int r = 0; r < R; ++r) store_nt(a.dp[r] + stripe * a.ds[r] + off, acc[r]);
        if (HASH && a.hashes) {
            const uint32_t hs = div_magic(idx, a.hmagic, a.hshift);
            const uint32_t p = a.hpow * pow31_seg(idx - hs * a.hsegs);
#pragma unroll
            for (int r = 0; r < R; ++r)
                atomicAdd(reinterpret_cast<unsigned*>(a.hashes) + static_cast<uint64_t>(hs) * a.hstride + r,
                          horner31(acc[r]) * p);
        }
    }
}

// ---------------------------------------------------------------------------
// Grouped launch: several batches with the same coefficients (different chunk
// sizes, strides and stripe counts) in ONE launch of the plain kernel body.
// Block b belongs to the last part whose first block is <= b (a wave-uniform
// scan over at most kMaxGroup parts).  A batch of small launches (a strong-
// scaled mixed-size step at 8 GPUs: tens of microseconds each) otherwise pays
// one ramp-up and one drain per batch.
// ---------------------------------------------------------------------------
constexpr int kMaxGroup = 8;

template <int K, int R>
struct GroupPart {
    const uint8_t* sp[K];
    uint64_t ss[K];
    uint8_t* dp[R];
    uint64_t ds[R];
    uint32_t segs, total, magic, shift;
    uint32_t block0;  // first block of this part
};

template <int K, int R>
struct GroupArgs {
    GroupPart<K, R> part[kMaxGroup];
    int n;
    gf::PermTable tab[R][K];
};

// UNI: every part's stripes hold whole waves (segs % 64 == 0, stripe offsets
// below 2^32): scalar stripe bases, as gf_apply_x16u.
template <int K, int R, bool UNI>
__global__ __launch_bounds__(kBlock) void gf_apply_group(const GroupArgs<K, R> a)
{
    __shared__ __attribute__((aligned(16))) uint32_t tl[R * K * kTabStride];
    int p = 0;
    for (int q = 1; q < a.n; ++q)
        if (blockIdx.x >= a.part[q].block0) p = q;
    const GroupPart<K, R>& g = a.part[p];
    const uint32_t idx = (blockIdx.x - g.block0) * blockDim.x + threadIdx.x;
    stage_tables<K, R>(a.tab, tl);
    if (idx >= g.total) return;  // (UNI: whole waves)
    const uint32_t stripe = UNI ? div_magic(__builtin_amdgcn_readfirstlane(idx), g.magic, g.shift)
                                : static_cast<uint32_t>((static_cast<uint64_t>(idx) * g.magic) >> g.shift);
    const uint64_t off = UNI ? static_cast<uint64_t>(static_cast<uint32_t>((idx - stripe * g.segs) * 16u))
                             : static_cast<uint64_t>(idx - stripe * g.segs) * 16;
    uint4 x[K];
#pragma unroll
    for (int j = 0; j < K; ++j) x[j] = load_nt(g.sp[j] + stripe * g.ss[j] + off);
    uint4 acc[R];
    gf_combine<K, R>(x, tl, acc);
#pragma unroll
    for (int r = 0; r < R; ++r) store_nt(g.dp[r] + stripe * g.ds[r] + off, acc[r]);
}

// Plain launches with U segments per lane (A/B: AB_PLAIN_U > 1): a wave codes
// U adjacent 1 KiB slices per column, all U*K loads issued before any compute,
// so a wave keeps U times the bytes in flight at the same occupancy cap.
template <int K, int R, int U>
__global__ __launch_bounds__(kBlock) void gf_apply_x16m(const FastArgs<K, R> a)
{
    __shared__ __attribute__((aligned(16))) uint32_t tl[R * K * kTabStride];
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t first = ((blockIdx.x * blockDim.x + threadIdx.x) >> 6) * (64u * U);
    stage_tables<K, R>(a.tab, tl);
    if (__builtin_amdgcn_readfirstlane(first) >= a.total) return;
    uint4 x[U][K];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const uint32_t idx = min(first + u * 64u + lane, a.total - 1);  // past the end: redo the last segment
        const uint32_t stripe = static_cast<uint32_t>((static_cast<uint64_t>(idx) * a.magic) >> a.shift);
        const uint64_t off = static_cast<uint64_t>(idx - stripe * a.segs) * 16;
#pragma unroll
        for (int j = 0; j < K; ++j) x[u][j] = load_nt(a.sp[j] + stripe * a.ss[j] + off);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const uint32_t idx = first + u * 64u + lane;
        if (idx >= a.total) break;
        const uint32_t stripe = static_cast<uint32_t>((static_cast<uint64_t>(idx) * a.magic) >> a.shift);
        const uint64_t off = static_cast<uint64_t>(idx - stripe * a.segs) * 16;
        uint4 acc[R];
        gf_combine<K, R>(x[u], tl, acc);
#pragma unroll
        for (int r = 0; r < R; ++r) store_nt(a.dp[r] + stripe * a.ds[r] + off, acc[r]);
    }
}

// ---------------------------------------------------------------------------
// Persistent forms of the plain and grouped kernels: one resident wave of
// workgroups (grid = CUs x the blocks the occupancy cap lets each CU hold),
// each staging the tables ONCE and then walking the launch's blocks in a
// grid stride (virtual block b = blockIdx.x, + gridDim.x, ...).  Every
// virtual block codes exactly the segments the ordinary launch's block b
// would, so bytes, order of HBM windows and results are unchanged; what goes
// is the per-block wave launch and table staging (kernarg loads, LDS writes,
// a barrier) on the critical path of every 1 KiB per column.  No block waits
// on another: each loop ends when its next virtual block is past the launch.
// ---------------------------------------------------------------------------
template <int K, int R, bool UNI>
__global__ __launch_bounds__(kBlock) void gf_apply_x16p(const FastArgs<K, R> a, uint32_t vblocks)
{
    __shared__ __attribute__((aligned(16))) uint32_t tl[R * K * kTabStride];
    stage_tables<K, R>(a.tab, tl);
    for (uint32_t b = blockIdx.x; b < vblocks; b += gridDim.x) {
        const uint32_t idx = b * blockDim.x + threadIdx.x;
        if (idx >= a.total) break;  // (UNI: whole waves; later blocks lie further past the end)
        uint32_t stripe;
        uint64_t off;
        if constexpr (UNI) {
            stripe = div_magic(__builtin_amdgcn_readfirstlane(idx), a.magic, a.shift);
            off = static_cast<uint32_t>((idx - stripe * a.segs) * 16u);
        } else {
            stripe = static_cast<uint32_t>((static_cast<uint64_t>(idx) * a.magic) >> a.shift);
            off = static_cast<uint64_t>(idx - stripe * a.segs) * 16;
        }
        uint4 x[K];
#pragma unroll
        for (int j = 0; j < K; ++j) x[j] = load_nt(a.sp[j] + static_cast<uint64_t>(stripe) * a.ss[j] + off);
        uint4 acc[R];
        gf_combine<K, R>(x, tl, acc);
#pragma unroll
        for (int r = 0; r < R; ++r) store_nt(a.dp[r] + static_cast<uint64_t>(stripe) * a.ds[r] + off, acc[r]);
    }
}

template <int K, int R, bool UNI>
__global__ __launch_bounds__(kBlock) void gf_apply_groupp(const GroupArgs<K, R> a, uint32_t vblocks)
{
    __shared__ __attribute__((aligned(16))) uint32_t tl[R * K * kTabStride];
    stage_tables<K, R>(a.tab, tl);
    for (uint32_t b = blockIdx.x; b < vblocks; b += gridDim.x) {
        int p = 0;
        for (int q = 1; q < a.n; ++q)
            if (b >= a.part[q].block0) p = q;
        const GroupPart<K, R>& g = a.part[p];
        const uint32_t idx = (b - g.block0) * blockDim.x + threadIdx.x;
        if (idx >= g.total) continue;  // the part's last block may be partial; later blocks are other parts
        const uint32_t stripe = UNI ? div_magic(__builtin_amdgcn_readfirstlane(idx), g.magic, g.shift)
                                    : static_cast<uint32_t>((static_cast<uint64_t>(idx) * g.magic) >> g.shift);
        const uint64_t off = UNI ? static_cast<uint64_t>(static_cast<uint32_t>((idx - stripe * g.segs) * 16u))
                                 : static_cast<uint64_t>(idx - stripe * g.segs) * 16;
        uint4 x[K];
#pragma unroll
        for (int j = 0; j < K; ++j) x[j] = load_nt(g.sp[j] + stripe * g.ss[j] + off);
        uint4 acc[R];
        gf_combine<K, R>(x, tl, acc);
#pragma unroll
        for (int r = 0; r < R; ++r) store_nt(g.dp[r] + stripe * g.ds[r] + off, acc[r]);
    }
}

#ifndef AB_PAD_U4
#define AB_PAD_U4 2
#endif
// Segments per lane for gf_apply_lens: U*K 16-byte loads in flight per lane.
// U = 2 since round 3 (3 interleaved rounds, profiles/r03/padded_and_plain_u_ab.txt):
// ELECT's degraded read 77.3 -> 81.6 % of peak at 64 KiB codeLength and 80.7 ->
// 82.2 % at 4.4 MB in 64 KiB tiles, padded encode at 93 % fill 79.1 -> 80.1 %,
// full units 81.0 -> 82.3 %, random fill 69.1 -> 68.8 % (noise); U = 4 before.
template <int K>
constexpr int lens_unroll() { return K <= 4 ? AB_PAD_U4 : 1; }

// Sum the per-wave hash partials of each (stripe, row); one wave per pair:
// lanes stride over the partials, then a wave sum; lane 0 is the sole writer.
// Add mode: the waves lying wholly inside stripe s are
// [ceil(s*segs/64), floor((s+1)*segs/64)); straddling waves already added
// theirs atomically; the entry (seeded with 31^len) is incremented.
// Assign mode (hi != null, segs >= 64): every wave of [floor(s*segs/64),
// floor(((s+1)*segs-1)/64)] contributes its first-stripe sum if it starts
// inside s, else its second-stripe sum; the entry becomes seed + sum.
[[maybe_unused]] __global__ __launch_bounds__(kBlock) void hash_reduce(const uint32_t* __restrict__ part, const uint32_t* __restrict__ hi,
                                                      int32_t* hashes, uint32_t hstride, int rows, uint32_t segs,
                                                      uint32_t stripes, uint32_t seed)
{
    const uint32_t t = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;  // (stripe, row) of this wave
    if (t >= stripes * static_cast<uint32_t>(rows)) return;
    const uint32_t s = t / rows, r = t % rows, lane = threadIdx.x & 63u;
    const uint64_t start = static_cast<uint64_t>(s) * segs;
    uint32_t sum = 0;
    if (hi) {
        const uint64_t w0 = start / 64, w1 = (start + segs - 1) / 64;
        for (uint64_t w = w0 + lane; w <= w1; w += 64) sum += (w * 64 >= start ? part : hi)[w * rows + r];
    } else {
        const uint64_t w0 = (start + 63) / 64, w1 = (start + segs) / 64;
        for (uint64_t w = w0 + lane; w < w1; w += 64) sum += part[w * rows + r];
    }
    sum = wave_sum(sum);
    if (lane == 0) {
        uint32_t* h = reinterpret_cast<uint32_t*>(hashes) + static_cast<uint64_t>(s) * hstride + r;
        if (hi)
            *h = seed + sum;
        else  // add mode: launches over other windows of the same units may add concurrently (host path)
            atomicAdd(h, sum);
    }
}

// Block size by shape (the occupancy caps below are set per block size; the
// per-family choices since round 3 are in DESIGN.md §4, launch shape table):
// small chunks (<= 4 KiB per shard) run 128-thread blocks (3-4 % over 256 in
// round 1; one-wave blocks measured the same in round 3), launches of >= 16
// coefficients 128 (read-heavy) or 256 (write-heavy), and plain launches of
// fewer coefficients one-wave blocks (plain_one_wave, below).  Keeping the
// tables in SGPRs instead of LDS (no barrier) lost 1 % on RS(6,4).
#ifndef AB_BLOCK_WIDE_READ  // A/B: read-heavy launches of >= 16 coefficients (RS(12,8) decodes)
#define AB_BLOCK_WIDE_READ 128
#endif
// Write-heavy ones (RS(12,8) encodes) run 256-thread blocks since the occupancy
// caps (round 3, 3 interleaved rounds, profiles/r03/block_wide_ab.txt): 64 /
// 128 / 256 threads 75.5 / 73.9 / 76.8 % of peak; read-heavy ones keep 128
// (64: the same within noise; 256: 78 % against 85 %).
#ifndef AB_BLOCK_WIDE_WRITE  // A/B: write-heavy launches of >= 16 coefficients (RS(12,8) encodes)
#define AB_BLOCK_WIDE_WRITE 256
#endif
#ifndef AB_WAVES_HASH_PAD  // A/B: occupancy cap of padded launches with the parity hash (0: uncapped)
#define AB_WAVES_HASH_PAD 0
#endif
#ifndef AB_BLOCK_PAD_WRITE  // A/B: block size of unhashed padded write-heavy launches
#define AB_BLOCK_PAD_WRITE 128
#endif
#ifndef AB_BLOCK_HASH_PAD  // A/B: block size of padded launches with the parity hash
#define AB_BLOCK_HASH_PAD 64
#endif
#ifdef AB_BLOCK  // A/B builds (tools/ab_build.sh): one block size for every launch
inline int block_for(uint64_t, int, int) { return AB_BLOCK; }
#else
inline int block_for(uint64_t len, int cols, int rows)
{
    if (len <= 4096) return 128;
    if (cols * rows >= 16) return 2 * rows >= cols ? AB_BLOCK_WIDE_WRITE : AB_BLOCK_WIDE_READ;
    return kBlock;
}
#endif

constexpr int kMaxHashCols = 10;  // ELECT_EC_MAX_DATA_UNITS: hashed launches are encodes

// Occupancy cap for the plain streaming kernel (gf_apply_x16 without padding
// or hash): dynamic LDS that no block reads, so that at most `waves` waves of a
// launch are resident per CU (160 KiB of LDS per CU / blocks).  Fewer waves in
// flight keep fewer HBM pages open at once.  Measured (occupancy
// sweep, 3 interleaved rounds): uncapped (32 waves) -> 20 waves: RS(6,4) decode
// 77.3 -> 81.0 % of peak, the mixed config +3 %, RS(12,8) decode 77 -> 80 %;
// encodes (R >= K/2: more writes in flight) peak at 24.  PMC: the uncapped
// decode waits on DRAM read credits 6x as often (profiles/r02_pmc_occupancy_ab.txt).
// The hashed and update kernels lost with any cap (the hash epilogue wants the
// waves: ELECT's fused steps 80 -> 67 % at 20) and run uncapped.
#ifndef AB_WAVES_READ_HEAVY
#define AB_WAVES_READ_HEAVY 20
#endif
#ifndef AB_WAVES_WRITE_HEAVY
#define AB_WAVES_WRITE_HEAVY 24
#endif
// Read-heavy launches of 8 or more source columns (RS(12,8) decodes) keep twice
// the read streams open per wave: 12 waves per CU there (round 3, interleaved
// rounds on two boxes, profiles/r03/occupancy_wide_ab.txt): RS(12,8)
// two-erasure decode at 20 / 16 / 14 / 12 / 10 / 8 waves 78.2 / 79.5 / 83.0 /
// 85.2 / 75.7 / 75.7 % of peak (configs[4] 4,541 -> 4,935 GiB/s at 12, alone;
// 4,458-4,489 -> 4,765-4,775 inside the headline line), three erasures 79.1 ->
// 82.2 %; one erasure (8 coefficients, 256-thread blocks) keeps 20 (77.7 % at
// 12 against 78.1 %); 16 for every read-heavy shape cost the mixed config's
// 1-4 KiB decodes 2-4 points.
#ifndef AB_WAVES_READ_HEAVY_WIDE
#define AB_WAVES_READ_HEAVY_WIDE 12
#endif
// (write-heavy ones of 8 or more columns keep 24: RS(12,8) encode at 16 / 12
// waves 72.5 / 66.9 % against 74.6 %)
// Plain launches (no padding, no hash) of chunks above 4 KiB and fewer than 16
// coefficients run one-wave blocks, their cap set in single waves: RS(6,4)
// encode at 16 waves per CU 82.4-82.6 -> 83.6-84.2 % of peak (14: 82.0, 12:
// 75.7 %), RS(6,4) single-erasure decode at 17-18 waves 80.8-82.0 -> 83.8-84.1 %
// (15: 80.7 %), RS(12,8) single-erasure decode at 12 waves 78.8-79.0 -> 84.8-85.0 %
// (profiles/r03/plain_one_wave_ab.txt).  Finer block steps place the cap where
// 256-thread blocks (4 waves a step) cannot.  Padded, hashed and grouped
// launches keep their own shapes (padded decodes and full-size groups lose with
// one-wave blocks).
#ifndef AB_PLAIN_ONE_WAVE  // A/B: 0 = off
#define AB_PLAIN_ONE_WAVE 1
#endif
#ifndef AB_WAVES_PLAIN_WRITE
#define AB_WAVES_PLAIN_WRITE 18
#endif
#ifndef AB_WAVES_PLAIN_READ
#define AB_WAVES_PLAIN_READ 18
#endif
#ifndef AB_WAVES_PLAIN_READ_WIDE
#define AB_WAVES_PLAIN_READ_WIDE 12
#endif
// Unpadded hashed launches (the fused-hash encode) run one-wave blocks at 20
// waves per CU: 80.7 -> 81.2 % of peak (one-wave uncapped 80.4, at 24 waves
// 81.0 %; profiles/r03/plain_one_wave_ab.txt).  Unhashed padded encodes keep
// 128-thread blocks: one-wave ones at 16-20 waves gain at ELECT's fill (93 %:
// 80.4 -> 82.1 %) but lose at random fill (71.9 -> 69.5 %).
#ifndef AB_BLOCK_HASH_PLAIN  // A/B: block size of unpadded hashed launches (0: block_for)
#define AB_BLOCK_HASH_PLAIN 64
#endif
#ifndef AB_WAVES_HASH_PLAIN  // A/B: their occupancy cap (0: uncapped)
#define AB_WAVES_HASH_PLAIN 20
#endif
#ifndef AB_PAD_READ_ONE_WAVE  // A/B: padded read-heavy launches in one-wave blocks at this cap (0 = off)
#define AB_PAD_READ_ONE_WAVE 0
#endif
#ifndef AB_PLAIN_ONE_WAVE_SMALL  // A/B: chunks <= 4 KiB too (1 = on)
#define AB_PLAIN_ONE_WAVE_SMALL 0
#endif
// Grouped launches of one-wave blocks (short groups, kSmallGroupBytes) take the
// one-wave caps too: the mixed config's 8-way share 4,272 -> 4,397 GiB/s
// (profiles/r03/plain_one_wave_ab.txt).  Chunks <= 4 KiB keep 128-thread blocks
// (one-wave blocks there: 1 KiB encode -0.6, decode +1 point, the same value).
#ifndef AB_GROUP_ONE_WAVE_CAPS  // A/B: 0 = the caps of plain_waves_cap
#define AB_GROUP_ONE_WAVE_CAPS 1
#endif
inline bool plain_one_wave(uint64_t len, int cols, int rows)
{
    return AB_PLAIN_ONE_WAVE && (len > 4096 || AB_PLAIN_ONE_WAVE_SMALL) && cols * rows < 16;
}
inline int plain_one_wave_cap(int cols, int rows)
{
    if (2 * rows >= cols) return AB_WAVES_PLAIN_WRITE;
    return cols >= 8 ? AB_WAVES_PLAIN_READ_WIDE : AB_WAVES_PLAIN_READ;
}
#ifndef AB_WAVES_WRITE_HEAVY_WIDE  // A/B: write-heavy launches of 8 or more source columns (RS(12,8) encodes)
#define AB_WAVES_WRITE_HEAVY_WIDE AB_WAVES_WRITE_HEAVY
#endif
constexpr size_t kLdsPerCU = 160 * 1024;
#ifndef AB_PERSIST  // A/B builds only (tools/ab_build.sh NAME -DAB_PERSIST=1): compile the persistent
#define AB_PERSIST 0   // kernels, chosen at run time by ELECT_EC_PERSIST; measured slower
#endif
#ifndef AB_PLAIN_U  // A/B: segments per lane of plain (per-lane addressed) launches; 1 = gf_apply_x16
#define AB_PLAIN_U 1
#endif
#ifndef AB_PLAIN_U_MAX_R  // ... for launches of at most this many output rows (1: decodes only)
#define AB_PLAIN_U_MAX_R 4
#endif
#ifndef AB_PLAIN_U_WAVES  // ... and this occupancy cap (0: plain_waves_cap)
#define AB_PLAIN_U_WAVES 0
#endif

// (and narrow read-heavy ones of 128-thread blocks, chunks <= 4 KiB, keep 20 too:
// 1 KiB decodes at 16 / 24 waves 80.7 / 81.4 % against 82.4 %; write-heavy wide
// ones at 28 / 32 waves measured the same as 24)
#ifndef AB_WAVES_READ_HEAVY_SMALL  // A/B: narrow read-heavy launches of 128-thread blocks (chunks <= 4 KiB)
#define AB_WAVES_READ_HEAVY_SMALL AB_WAVES_READ_HEAVY
#endif

inline int plain_waves_cap(int cols, int rows, int block)
{
    if (2 * rows >= cols) return cols >= 8 ? AB_WAVES_WRITE_HEAVY_WIDE : AB_WAVES_WRITE_HEAVY;
    if (cols >= 8 && rows >= 2) return AB_WAVES_READ_HEAVY_WIDE;  // (>= 16 coefficients: 128-thread blocks)
    return block < kBlock ? AB_WAVES_READ_HEAVY_SMALL : AB_WAVES_READ_HEAVY;
}

inline size_t cap_lds(int block, int coefs, int waves);

// The padded per-stripe-length kernel takes the same cap: 64 KiB degraded-read
// decode (flows) 76.4 -> 77.4 %, padded encodes unchanged (3 interleaved rounds).
#ifndef AB_CAP_LENS
#define AB_CAP_LENS 1
#endif
#ifndef AB_WAVES_PAD_WRITE  // A/B: occupancy cap of padded write-heavy launches (per-stripe lengths)
#define AB_WAVES_PAD_WRITE AB_WAVES_WRITE_HEAVY
#endif
inline size_t lens_cap(int block, int coefs, int cols, int rows)
{
    // (the wide caps above were measured on the plain kernels only)
    const int waves = 2 * rows >= cols ? AB_WAVES_PAD_WRITE : (AB_PAD_READ_ONE_WAVE ? AB_PAD_READ_ONE_WAVE : AB_WAVES_READ_HEAVY);
    return AB_CAP_LENS ? cap_lds(block, coefs, AB_CAP_LENS > 1 ? AB_CAP_LENS : waves) : 0;
}

inline size_t cap_lds(int block, int coefs, int waves)
{
    if (waves <= 0) return 0;
    const int blocks = std::max(1, waves / (block / 64));
    const size_t static_lds = static_cast<size_t>(coefs) * kTabStride * sizeof(uint32_t);
    const size_t per_block = kLdsPerCU / blocks - 512;  // > kLdsPerCU / (blocks + 1): one block fewer fits
    return per_block > static_lds ? per_block - static_lds : 0;
}

// Persistent launches (gf_apply_x16p / gf_apply_groupp), in AB_PERSIST builds only:
// ELECT_EC_PERSIST = 0 (off), 1 (plain and grouped launches) or 2 (grouped only); read once.
inline int persist_mode()
{
    if constexpr (AB_PERSIST == 0) return 0;
    static const int m = [] {
        const char* e = std::getenv("ELECT_EC_PERSIST");
        return e ? std::atoi(e) : 0;
    }();
    return m;
}

// Compute units of the current device (cached per device).
inline int device_cus()
{
    static std::mutex mu;
    static int cus[64] = {};
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
    std::lock_guard<std::mutex> lock(mu);
    if (!cus[dev]) {
        int n = 0;
        cus[dev] = hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && n > 0 ? n : 256;
    }
    return cus[dev];
}

// Grid of a persistent launch: every CU holds `waves` waves (the occupancy cap)
// of `block`-thread blocks, at most the launch's own block count.
inline uint32_t persist_grid(uint64_t vblocks, int block, int waves)
{
    const uint64_t per_cu = static_cast<uint64_t>(std::max(1, waves / (block / 64)));
    return static_cast<uint32_t>(std::min<uint64_t>(vblocks, per_cu * static_cast<uint64_t>(device_cus())));
}

// Padded launches the per-stripe-length kernel can take (whole 16-byte segments,
// aligned columns).  Hashed ones with per-stripe content lengths, untiled, of at
// most 4 columns take it too, 2 segments per lane, in add mode only (launch_apply_impl
// seeds the entries for them).  Interleaved A/B against gf_apply_x16<.., HASH>
// (profiles/r02_lenshash_ab/): ELECT's fused steps at 64 KiB codeLength, encode
// 73.1 -> 74.2 %, update 74.6 -> 76.0 %; but ELECT's 4.4 MB codeLength in tiles lost
// 2 points (79.5 -> 77.6 %), full hashed units 1 % (3,762 -> 3,725 GiB/s), and
// 4 segments per lane (121 VGPRs) or 1 lost everywhere: those stay on gf_apply_x16.
// Round 3: with one-wave blocks for padded hashed launches (AB_BLOCK_HASH_PAD) the
// one-segment gf_apply_x16<.., PAD, HASH> beats it at 64 KiB codeLength too:
// encode 76.0 -> 78.1 %, update 76.7 -> 78.5 % (U = 1 / 4 in one-wave blocks:
// 72.6 / 73.5 % encode; profiles/r03/lens_hash_ab.txt), so the path is off.
#ifndef AB_LENS_HASH
#define AB_LENS_HASH 0
#endif
#ifndef AB_LENS_HASH_U
#define AB_LENS_HASH_U 2
#endif
#ifndef AB_LENS_HASH_MIN_LEN  // A/B knob: the lens path only at or above this unit length
#define AB_LENS_HASH_MIN_LEN 0
#endif
inline bool lens_eligible(const ApplyParams& p)
{
    return p.aligned16 && p.len % 16 == 0 && p.len > 0 && p.len < (uint64_t{1} << 31);
}

inline bool lens_hash_path(const ApplyParams& p)
{
    return AB_LENS_HASH && p.hashes && p.padded && p.lens && p.tiles <= 1 && p.cols <= 4 &&
           p.len >= AB_LENS_HASH_MIN_LEN && lens_eligible(p);
}

// gf_apply_x16u (and the grouped kernel's UNI form) for plain launches of
// whole-wave stripes with at least this many columns.  Interleaved A/B
// (profiles/r02_scalarbase_ab/): RS(12,8) two-erasure decode (K = 8) 79.9 ->
// 81.6 % of peak, 4,618 -> 4,716 GiB/s; RS(6,4) encode 82.7 -> 82.2 %, its
// decode +0.5, the mixed config -0.5 %: the four-column shapes keep the
// per-lane addressing.  AB builds: -DAB_SCALAR_BASE_MIN_K=99 turns it off.
#ifndef AB_SCALAR_BASE_MIN_K
#define AB_SCALAR_BASE_MIN_K 8
#endif
#ifndef AB_SCALAR_BASE_R1  // A/B: single-row plain launches (one-erasure decodes) of any width too
#define AB_SCALAR_BASE_R1 0
#endif
#ifndef AB_SCALAR_BASE_HASH  // hashed plain launches of whole-wave stripes, any width
#define AB_SCALAR_BASE_HASH 1
#endif

template <int K, int R, bool PAD>
hipError_t launch_fast_kr(const ApplyParams& p, int r0, hipStream_t stream)
{
    FastArgs<K, R> a{};
    // padded: every segment incl. a partial last one; else whole segments only
    const uint64_t segs64 = PAD ? (p.len + 15) / 16 : p.len / 16;
    if (segs64 == 0) return hipSuccess;
    if (segs64 > kMaxIndex) return hipErrorInvalidValue;
    a.segs = static_cast<uint32_t>(segs64);
    const Magic mg = make_magic(a.segs);
    a.magic = mg.m;
    a.shift = mg.p;
    a.len = p.len;
    a.len32 = static_cast<uint32_t>(std::min<uint64_t>(p.len, 0xFFFFFFFFu));
    const uint32_t tiles = std::max<uint32_t>(1, p.tiles);
    const uint64_t ulen = p.unit_len ? p.unit_len : p.len;
    a.ulen32 = static_cast<uint32_t>(std::min<uint64_t>(ulen, 0xFFFFFFFFu));
    a.tiles = tiles;
    const Magic tm = make_magic(tiles);
    a.tmagic = tm.m;
    a.tshift = tm.p;
    if (segs64 * tiles > kMaxIndex) return hipErrorInvalidValue;
    a.hsegs = static_cast<uint32_t>(segs64 * tiles);
    const Magic hm = make_magic(a.hsegs);
    a.hmagic = hm.m;
    a.hshift = hm.p;
    a.lstride = p.lens_stride ? p.lens_stride : static_cast<uint32_t>(p.cols);
    a.lcols = static_cast<uint32_t>(p.lens_cols ? p.lens_cols : p.cols);
    for (int j = 0; j < K; ++j) a.clen[j] = p.clen[j];
    a.hstride = p.hash_stride;
    a.hpow = pow31(p.hash_base);
    for (int r = 0; r < R; ++r)
        for (int j = 0; j < K; ++j) a.tab[r][j] = gf::perm_table(p.coef[(r0 + r) * p.cols + j]);
    // Padded launches with the parity hash (ELECT's fused encode and update steps)
    // run one-wave blocks: the fused encode step 80.0 -> 81.4 % of peak at ELECT's
    // codeLength (64 KiB tiles) and 74.7 -> 76.3 % at 64 KiB codeLength, the
    // update step unchanged (round 3, profiles/r03/block_hash_pad_ab.txt).
    // Unhashed padded encodes (per-unit content lengths) run 128-thread blocks:
    // 64 KiB units at random fill 70.2 -> 73.8 % of peak, at ELECT's fill (93 %)
    // 80.2 -> 80.7 %, full 82.1 -> 82.4 %; padded decodes keep 256 (64 / 128 threads:
    // -3 / -4 points) (profiles/r03/block_pad_ab.txt).
    const bool one_wave = !PAD && !p.hashes && plain_one_wave(p.len, K, R);
    const bool pad_read_one_wave = AB_PAD_READ_ONE_WAVE && PAD && !p.hashes && 2 * R < K;
    const int block = one_wave || pad_read_one_wave ? 64
                      : PAD && p.hashes ? AB_BLOCK_HASH_PAD
                      : PAD && 2 * R >= K ? std::min(AB_BLOCK_PAD_WRITE, block_for(p.len, K, R))
                      : !PAD && p.hashes && AB_BLOCK_HASH_PLAIN ? AB_BLOCK_HASH_PLAIN
                                          : block_for(p.len, K, R);
    const int plain_cap = one_wave ? plain_one_wave_cap(K, R) : plain_waves_cap(K, R, block);
    const bool hash_assign = p.hashes && p.hash_seed;  // launch_apply chose assign mode
    // stripes per launch keeping idx < 2^31, whole logical stripes (tiles) per launch
    const uint64_t per_launch = kMaxIndex / segs64 / tiles * tiles;
    for (uint64_t s0 = 0; s0 < p.stripes; s0 += per_launch) {
        const uint64_t ns = std::min<uint64_t>(per_launch, p.stripes - s0);
        for (int j = 0; j < K; ++j) {
            a.sp[j] = p.src[j].ptr + s0 * p.src[j].stride;
            a.ss[j] = p.src[j].stride;
        }
        for (int r = 0; r < R; ++r) {
            a.dp[r] = const_cast<uint8_t*>(p.dst[r0 + r].ptr) + s0 * p.dst[r0 + r].stride;
            a.ds[r] = p.dst[r0 + r].stride;
        }
        a.lens = p.lens ? p.lens + s0 / tiles * a.lstride : nullptr;
        a.hashes = p.hashes ? p.hashes + s0 / tiles * p.hash_stride + r0 : nullptr;
        a.total = static_cast<uint32_t>(ns * segs64);
        a.hpart = nullptr;
        a.hpart_hi = nullptr;
        if (a.hashes) {  // the per-wave partial sums (lo, then hi) go to the caller's scratch
            const size_t n = (static_cast<size_t>(a.total) / 64 + 1) * R;
            if (!p.hash_scratch || 2 * n > p.hash_scratch_words) return hipErrorInvalidValue;
            a.hpart = p.hash_scratch;
            if (hash_assign) a.hpart_hi = a.hpart + n;
        }
        bool lens_path = false;
        if constexpr (PAD) {
            lens_path = a.hashes ? lens_hash_path(p) && !hash_assign : (a.lens || tiles > 1) && lens_eligible(p);
#ifdef AB_NO_LENS
            lens_path = false;
#endif
            if (lens_path) {
                constexpr int U = lens_unroll<K>();
                const uint64_t threads = (static_cast<uint64_t>(a.total) + 64 * U - 1) / (64 * U) * 64;
                const dim3 grid(static_cast<uint32_t>((threads + block - 1) / block));
                if (!a.hashes)
                    hipLaunchKernelGGL((gf_apply_lens<K, R, U, false>), grid, dim3(block), lens_cap(block, R * K, K, R),
                                       stream, a);
                else if constexpr (K <= 4) {  // (lens_hash_path)
                    constexpr int UH = AB_LENS_HASH_U;
                    const uint64_t th = (static_cast<uint64_t>(a.total) + 64 * UH - 1) / (64 * UH) * 64;
                    hipLaunchKernelGGL((gf_apply_lens<K, R, UH, true>), dim3(static_cast<uint32_t>((th + block - 1) / block)),
                                       dim3(block), cap_lds(block, R * K, AB_WAVES_HASH_PAD), stream, a);
                }
            }
        }
        if (!lens_path) {
            const uint32_t grid = (a.total + block - 1) / block;
            bool scalar_base = false;
            constexpr bool kPlainU = K >= AB_SCALAR_BASE_MIN_K || (AB_SCALAR_BASE_R1 && R == 1);
            if constexpr (!PAD)
                scalar_base = (a.hashes ? AB_SCALAR_BASE_HASH != 0 && K <= kMaxHashCols : kPlainU) &&
                              a.segs % 64 == 0 && segs64 < (uint64_t{1} << 28);
            if (AB_PLAIN_U > 1 && !PAD && !a.hashes && !scalar_base && R <= AB_PLAIN_U_MAX_R) {  // A/B: U per lane
                if constexpr (!PAD && AB_PLAIN_U > 1) {
                    constexpr int U = AB_PLAIN_U;
                    const uint64_t th = (static_cast<uint64_t>(a.total) + 64 * U - 1) / (64 * U) * 64;
                    hipLaunchKernelGGL((gf_apply_x16m<K, R, U>), dim3(static_cast<uint32_t>((th + block - 1) / block)),
                                       dim3(block), cap_lds(block, R * K, AB_PLAIN_U_WAVES ? AB_PLAIN_U_WAVES : plain_cap),
                                       stream, a);
                }
            } else if (AB_PERSIST && !PAD && !a.hashes && persist_mode() == 1) {  // persistent form (gf_apply_x16p)
                if constexpr (!PAD && AB_PERSIST != 0) {
                    const int waves = plain_cap;
                    const dim3 pg(persist_grid(grid, block, waves));
                    const size_t lds = cap_lds(block, R * K, waves);
                    if constexpr (kPlainU) {
                        if (scalar_base)
                            hipLaunchKernelGGL((gf_apply_x16p<K, R, true>), pg, dim3(block), lds, stream, a, grid);
                        else
                            hipLaunchKernelGGL((gf_apply_x16p<K, R, false>), pg, dim3(block), lds, stream, a, grid);
                    } else {
                        hipLaunchKernelGGL((gf_apply_x16p<K, R, false>), pg, dim3(block), lds, stream, a, grid);
                    }
                }
            } else if (scalar_base) {
                if constexpr (!PAD && kPlainU) {
                    if (!a.hashes)
                        hipLaunchKernelGGL((gf_apply_x16u<K, R, false>), dim3(grid), dim3(block),
                                           cap_lds(block, R * K, plain_cap), stream, a);
                }
                if constexpr (!PAD && K <= kMaxHashCols) {
                    if (a.hashes)
                        hipLaunchKernelGGL((gf_apply_x16u<K, R, true>), dim3(grid), dim3(block),
                                           cap_lds(block, R * K, AB_WAVES_HASH_PLAIN), stream, a);
                }
            } else if (!a.hashes) {
                hipLaunchKernelGGL((gf_apply_x16<K, R, PAD, false>), dim3(grid), dim3(block),
                                   PAD ? 0 : cap_lds(block, R * K, plain_cap), stream, a);
            } else if constexpr (K <= kMaxHashCols) {
                // (uncapped: capping the hashed instance at 24 / 28 waves per CU cost it 5 / 3
                // points, and staging 31^(16*lane) in LDS instead of constant memory gained
                // nothing; profiles/r02_hash_ab/)
                hipLaunchKernelGGL((gf_apply_x16<K, R, PAD, true>), dim3(grid), dim3(block),
                                   PAD ? cap_lds(block, R * K, AB_WAVES_HASH_PAD) : 0, stream, a);
            }  // (launch_apply rejects hashed launches wider than kMaxHashCols)
        }
        hipError_t e = hipGetLastError();
        if (e == hipSuccess && a.hashes) {
            const uint32_t units = static_cast<uint32_t>(ns / tiles);
            const uint32_t n = units * R;  // one wave each
            hipLaunchKernelGGL(hash_reduce, dim3((n + kBlock / 64 - 1) / (kBlock / 64)), dim3(kBlock), 0, stream, a.hpart,
                               a.hpart_hi, a.hashes, a.hstride, R, a.hsegs, units, pow31(ulen));
            e = hipGetLastError();
        }
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

template <int K, bool PAD = false>
constexpr std::array<FastFn, kFastRows> fast_row_fns()
{
    return {&launch_fast_kr<K, 1, PAD>, &launch_fast_kr<K, 2, PAD>, &launch_fast_kr<K, 3, PAD>,
            &launch_fast_kr<K, 4, PAD>};
}

// Grouped launches take every groupable batch of a call, whatever its chunk
// size, in one launch of the smallest block size any part wants (block_for):
// the mixed config's 8-way share 3,879 -> 3,959 GiB/s, 4-way 4,084 -> 4,116,
// full size unchanged, against one launch per block-size class; one launch of
// 256-thread blocks lost 5 % at full size (profiles/r02_group_ab/).
// A/B builds: -DAB_GROUP_BLOCK=-1 restores one launch per class, 128 / 256 force a size.
#ifndef AB_GROUP_BLOCK
#define AB_GROUP_BLOCK 0
#endif
#ifndef AB_GROUP_SMALL_BLOCK  // A/B: block size of grouped launches under kSmallGroupBytes of source (kBlock: off)
#define AB_GROUP_SMALL_BLOCK 64
#endif
#ifndef AB_SMALL_GROUP_BYTES  // A/B: groups of at least this many source bytes keep the larger blocks
#define AB_SMALL_GROUP_BYTES (~uint64_t{0})
#endif
constexpr uint64_t kSmallGroupBytes = AB_SMALL_GROUP_BYTES;
inline int group_class(const ApplyParams& p) { return AB_GROUP_BLOCK < 0 ? block_for(p.len, p.cols, std::min(p.rows, kFastRows)) : 0; }

// Launch parts [0, n) of a group (all plain, vector-capable, whole segments,
// same coefficients) for output rows r0 .. r0+R-1.
template <int K, int R>
hipError_t launch_group_kr(const ApplyParams* ps, int n, int r0, hipStream_t stream)
{
    GroupArgs<K, R> a{};
    a.n = n;
    for (int r = 0; r < R; ++r)
        for (int j = 0; j < K; ++j) a.tab[r][j] = gf::perm_table(ps[0].coef[(r0 + r) * ps[0].cols + j]);
    int block = kBlock;
    bool uni = true;  // (used for K >= AB_SCALAR_BASE_MIN_K)
    uint64_t bytes = 0;  // source bytes of the launch
    for (int i = 0; i < n; ++i) {
        block = std::min(block, block_for(ps[i].len, K, R));
        uni = uni && (ps[i].len / 16) % 64 == 0 && ps[i].len < (uint64_t{1} << 32);
        bytes += ps[i].len * ps[i].stripes * K;
    }
    // Grouped launches run one-wave blocks with the one-wave caps of the plain
    // launches.  With round 2's caps one-wave blocks won only for short groups
    // (the mixed config's 8-way share: 4,198 -> 4,276 GiB/s; the 4-way share and
    // full size lost, profiles/r03/group_small_block_ab.txt); with the one-wave
    // caps they win at every size: 8-way share 4,272 -> 4,397, 4-way 4,312 ->
    // 4,461, 2-way 4,488 -> 4,568, full size 4,461 -> 4,531 GiB/s
    // (profiles/r03/plain_one_wave_ab.txt).
    if (bytes < kSmallGroupBytes) block = std::min(block, AB_GROUP_SMALL_BLOCK);
    if (AB_GROUP_BLOCK > 0) block = AB_GROUP_BLOCK;
    const int group_cap = AB_GROUP_ONE_WAVE_CAPS && block == 64 && K * R < 16 ? plain_one_wave_cap(K, R)
                                                                              : plain_waves_cap(K, R, block);
    uint64_t blocks = 0;
    for (int i = 0; i < n; ++i) {
        const ApplyParams& p = ps[i];
        GroupPart<K, R>& g = a.part[i];
        const uint64_t segs = p.len / 16;
        g.segs = static_cast<uint32_t>(segs);
        g.total = static_cast<uint32_t>(segs * p.stripes);
        const Magic mg = make_magic(g.segs);
        g.magic = mg.m;
        g.shift = mg.p;
        for (int j = 0; j < K; ++j) {
            g.sp[j] = p.src[j].ptr;
            g.ss[j] = p.src[j].stride;
        }
        for (int r = 0; r < R; ++r) {
            g.dp[r] = const_cast<uint8_t*>(p.dst[r0 + r].ptr);
            g.ds[r] = p.dst[r0 + r].stride;
        }
        g.block0 = static_cast<uint32_t>(blocks);
        blocks += (g.total + block - 1) / block;
    }
    if (blocks > 0xFFFFFFFFull) return hipErrorInvalidValue;
    if constexpr (AB_PERSIST != 0) {
        if (persist_mode() >= 1) {  // persistent form (gf_apply_groupp)
            const int waves = group_cap;
            const dim3 pg(persist_grid(blocks, block, waves));
            const size_t lds = cap_lds(block, R * K, waves);
            const uint32_t vb = static_cast<uint32_t>(blocks);
            if constexpr (K >= AB_SCALAR_BASE_MIN_K) {
                if (uni) {
                    hipLaunchKernelGGL((gf_apply_groupp<K, R, true>), pg, dim3(block), lds, stream, a, vb);
                    return hipGetLastError();
                }
            }
            hipLaunchKernelGGL((gf_apply_groupp<K, R, false>), pg, dim3(block), lds, stream, a, vb);
            return hipGetLastError();
        }
    }
    if constexpr (K >= AB_SCALAR_BASE_MIN_K) {
        if (uni) {
            hipLaunchKernelGGL((gf_apply_group<K, R, true>), dim3(static_cast<uint32_t>(blocks)), dim3(block),
                               cap_lds(block, R * K, group_cap), stream, a);
            return hipGetLastError();
        }
    }
    hipLaunchKernelGGL((gf_apply_group<K, R, false>), dim3(static_cast<uint32_t>(blocks)), dim3(block),
                       cap_lds(block, R * K, group_cap), stream, a);
    return hipGetLastError();
}


template <int K>
constexpr std::array<GroupFn, kFastRows> group_row_fns()
{
    return {&launch_group_kr<K, 1>, &launch_group_kr<K, 2>, &launch_group_kr<K, 3>, &launch_group_kr<K, 4>};
}

}  // namespace
}  // namespace kern
}  // namespace elect
