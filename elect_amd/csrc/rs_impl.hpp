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

// ---------------------------------------------------------------------------
// Launch policy: the block size and the occupancy cap of every launch.
//
// The cap is the number of the launch's waves resident per CU (0: uncapped),
// set with dynamic LDS that no block reads (cap_lds: 160 KiB per CU / blocks).
// Fewer waves in flight keep fewer HBM pages open: an uncapped RS(6,4) decode
// waits on DRAM read credits 6x as often (profiles/r02_pmc_occupancy_ab.txt).
// One-wave blocks let the cap move in single waves; the best points (18 waves
// for RS(6,4), 12 for RS(12,8) decodes) lie two waves above cliffs where the
// rate falls by several points.  Every entry was chosen by interleaved A/B
// runs of the product library; the evidence file is named beside it, and
// DESIGN.md §4 has the launch-shape table.  A/B builds swap the whole table
// (tools/ab_build.sh NAME -DELECT_EC_POLICY_HEADER='"file.hpp"'); the product
// compiles this one.
// ---------------------------------------------------------------------------
struct LaunchPolicy {
    // Plain launches (no padding, no hash): gf_apply_x16 / gf_apply_x16u.
    uint64_t small_len = 4096;       // chunks up to this run 128-thread blocks (round 1: +3-4 % over 256)
    int small_block = 128;
    // > 4 KiB and < 16 coefficients: one-wave blocks (profiles/r03/plain_one_wave_ab.txt: RS(6,4)
    // encode 82.5 -> 84.1 %, decode 81.6 -> 83.8 %, RS(12,8) one-erasure decode 79.0 -> 84.8 %)
    int one_wave_write_waves = 18;   // write-heavy (2R >= K): RS(6,4) encode (14: 82.0 %, 12: 75.7 %)
    int one_wave_read_waves = 18;    // read-heavy, < 8 columns: RS(6,4) decode (15: 80.7 %)
    int one_wave_read_wide_waves = 12;  // read-heavy, >= 8 columns: RS(12,8) one-erasure decode
    // >= 16 coefficients, and chunks <= 4 KiB
    int wide_write_block = 256;      // RS(12,8) encode: 64 / 128 / 256 threads 75.5 / 73.9 / 76.8 % (block_wide_ab.txt)
    int wide_read_block = 128;       // RS(12,8) decodes (64: the same; 256: 78 against 85 %)
    int write_waves = 24;            // profiles/r02_occupancy_ab/ (RS(12,8) encode at 16 / 12: 72.5 / 66.9 %)
    int read_waves = 20;             // profiles/r02_occupancy_ab/ (1 KiB decodes at 16 / 24: 80.7 / 81.4 vs 82.4 %)
    int read_wide_waves = 12;        // >= 8 columns and >= 2 rows: RS(12,8) two-erasure decode at 20 / 16 / 14 /
                                     // 12 / 10 waves 78.2 / 79.5 / 83.0 / 85.2 / 75.7 % (occupancy_wide_ab.txt)
    // Plain launches with the parity hash (the fused-hash encode): one-wave blocks;
    // the scalar-base form capped at 20 waves (80.7 -> 81.2 %, plain_one_wave_ab.txt),
    // the per-lane form uncapped (caps of 24 / 28 cost 5 / 3 points, profiles/r02_hash_ab/)
    int hashed_block = 64;
    int hashed_scalar_waves = 20;
    int hashed_lane_waves = 0;
    int hashed_scalar_base_min_cols = 1;  // hashed launches take the scalar-base form from this width up
    // Padded launches: gf_apply_x16<PAD> (uncapped) and gf_apply_lens (capped).
    int padded_write_block = 128;    // random fill 68.9 -> 71.8 %, full 82.3 -> 82.7 % (block_pad_ab.txt);
                                     // read-heavy ones keep the plain block (64 / 128: -3 / -4 points)
    int lens_write_waves = 24;       // gf_apply_lens: degraded read 76.4 -> 77.4 % at 20 (profiles/r02_lenscap_ab/)
    int lens_read_waves = 20;
    // Padded launches with the hash (ELECT's fused encode and update steps): one-wave
    // blocks, uncapped (79.6 -> 81.0 % at ELECT's codeLength; caps of 20-28 lose:
    // block_hash_pad_ab.txt)
    int padded_hashed_block = 64;
    // Grouped launches (the mixed config): one-wave blocks with the plain caps of their
    // shape (8-way share 4,198 -> 4,397 GiB/s; group_small_block_ab.txt, plain_one_wave_ab.txt)
    int group_block = 64;
    // The parity update gf_update_x16: 81.6 -> 84.2 % (plain_one_wave_ab.txt)
    int update_block = 64;
    int update_waves = 18;
    // Scalar stripe bases (gf_apply_x16u) for plain launches of whole-wave stripes with at
    // least this many columns: RS(12,8) two-erasure decode 79.9 -> 81.6 % (round 2,
    // profiles/r02_scalarbase_ab/, where four-column shapes lost 0.5 % with 256-thread blocks);
    // in one-wave blocks four-column shapes gain too: the headline step 4,511-4,521 ->
    // 4,522-4,528 GiB/s, RS(6,4) decode 84.7-84.9 -> 85.0-85.1 % (round 4, profiles/r04/policy_ab.txt)
    int scalar_base_min_cols = 4;
    // ... and for the grouped kernel's UNI form: from 4 columns the mixed config lost 1 %
    // (4,549-4,571 -> 4,507-4,538 GiB/s, policy_ab.txt)
    int group_scalar_base_min_cols = 8;
    // Plain one-wave launches that load their columns through LDS (global_load_lds_dwordx4,
    // the LDS-DMA path, then ds_read_b128) instead of into VGPRs: 0 none, 1 read-heavy ones
    // (decodes), 2 all.  The XOR-only encode pattern ran 0.8-0.9 points faster that way
    // (profiles/r04/lds_dma_probe.txt); in the product, all: RS(6,4) encode 84.15 -> 83.8 %,
    // decode 84.2-84.5 -> 84.7-85.0 %; read-heavy only: the headline step 4,507-4,511 ->
    // 4,516-4,520 GiB/s, decode 84.5-84.9 -> 85.1-85.2 %, encode unchanged (profiles/r04/lds_dma_ab.txt).
    int plain_lds_dma = 1;
    // The parity hash's per-wave sum weights each lane by 31^(16 lane) inside a DPP tree
    // (wave_poly31) instead of a per-lane table load that waits behind the parity stores.
    bool hash_dpp_weights = false;
};

#ifdef ELECT_EC_POLICY_HEADER
#include ELECT_EC_POLICY_HEADER  // defines kPolicy (A/B builds only)
#else
constexpr LaunchPolicy kPolicy{};
#endif

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

constexpr int kAuxNT = 2;  // buffer / LDS-DMA op cache policy: nt (gfx940 family CPol)

// LDS-DMA (global_load_lds_dwordx4): lane i's 16 bytes at p land at lds + 16 i;
// lds is wave-uniform.  The data is in LDS after the wave's vmcnt drains.
typedef __attribute__((address_space(3))) void* lds_ptr_t;
typedef __attribute__((address_space(1))) const void* global_ptr_t;

__device__ __forceinline__ void load_to_lds_nt(const uint8_t* p, uint8_t* lds)
{
    __builtin_amdgcn_global_load_lds((global_ptr_t)p, (lds_ptr_t)lds, 16, 0, kAuxNT);
}

// One-wave blocks only: each of the K columns' 1 KiB for the wave goes through
// stage (K KiB of LDS), then every lane reads its 16 bytes back.
template <int K>
__device__ __forceinline__ void load_columns_via_lds(const uint8_t* const (&src)[K], uint8_t* stage, uint4 (&x)[K])
{
#pragma unroll
    for (int j = 0; j < K; ++j) load_to_lds_nt(src[j], stage + j * 1024);
    __builtin_amdgcn_s_waitcnt(0);
    const uint32_t lane = threadIdx.x & 63u;
#pragma unroll
    for (int j = 0; j < K; ++j) x[j] = *reinterpret_cast<const uint4*>(stage + j * 1024 + lane * 16);
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

// Sum over the 64 lanes of v_l * 31^(16 l) (lane l's 16 bytes follow lane l-1's),
// returned wave-uniform, with no per-lane weight table: a DPP tree where each
// level adds the partner 2^i lanes up, weighted by 31^(16 * 2^i) (row_shl
// within 16-lane rows, then the four rows' sums read out and combined in SALU).
// The table form (kLanePow[lane] * v, then wave_sum) loads the weight per lane
// after the parity stores, and on gfx9 vmcnt counts those stores too: every
// wave's epilogue waited for its own stores to land.
template <int Ctrl>
__device__ __forceinline__ uint32_t dpp_read(uint32_t v)  // bound_ctrl: 0 for lanes past the row
{
    return static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(v), Ctrl, 0xF, 0xF, true));
}

struct Pow31Lanes {  // 31^(16 * n) for n = 1, 2, 4, 8, 16, 32, 48
    uint32_t b1, b2, b4, b8, b16, b32, b48;
    constexpr Pow31Lanes() : b1(1), b2(0), b4(0), b8(0), b16(0), b32(0), b48(0)
    {
        for (int i = 0; i < 16; ++i) b1 *= 31u;
        b2 = b1 * b1;
        b4 = b2 * b2;
        b8 = b4 * b4;
        b16 = b8 * b8;
        b32 = b16 * b16;
        b48 = b32 * b16;
    }
};

__device__ __forceinline__ uint32_t wave_poly31(uint32_t v)
{
    constexpr Pow31Lanes kP{};
    v += kP.b1 * dpp_read<0x101>(v);  // row_shl:1
    v += kP.b2 * dpp_read<0x102>(v);  // row_shl:2
    v += kP.b4 * dpp_read<0x104>(v);  // row_shl:4
    v += kP.b8 * dpp_read<0x108>(v);  // row_shl:8: lane 16 r holds row r's weighted sum
    const uint32_t r0 = static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(v), 0));
    const uint32_t r1 = static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(v), 16));
    const uint32_t r2 = static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(v), 32));
    const uint32_t r3 = static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(v), 48));
    return r0 + kP.b16 * r1 + kP.b32 * r2 + kP.b48 * r3;
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
    if constexpr (!MASKED) {
        gf_combine_pairs<K, R>(x, tl, acc);
        return;
    }
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

// ---------------------------------------------------------------------------
// Encodes with ISA-L's Cauchy generator (gf_gen_cauchy1_matrix,
// EC/erasure_coder.c:43): parity row i, data column j holds inv(i ^ j), so for
// k a multiple of 4 every 4 x 4 block of the parity rows (rows k+a, columns
// 4g+c) is XOR-circulant: M[a][c] = h(a ^ c) with h(t) = M[0][4g+t].  Over
// GF(2^8) (characteristic 2) such a block applies with 9 constant
// multiplications instead of 16, a two-level Karatsuba over the index bits:
//   s = x0^x1^x2^x3, u = x1^x3, v = x2^x3,
//   y0 = h0 s ^ (h0^h1) u ^ (h0^h2) v ^ H x3
//   y1 = h1 s ^ (h0^h1) u ^ (h1^h3) v ^ H x3
//   y2 = h2 s ^ (h2^h3) u ^ (h0^h2) v ^ H x3
//   y3 = h3 s ^ (h2^h3) u ^ (h1^h3) v ^ H x3        (H = h0^h1^h2^h3)
// (expand each y and the x terms cancel pairwise to y_a = sum_c h(a^c) x_c).
// Per dword of a group: 27 v_perm + 3 pre-XORs + 4 selector sets + 19 XORs =
// 65 VALU ops against 88 for the general 16-coefficient form.  RS(12,8)
// encode was VALU-bound at 80 % VALU busy and a 1.89 GHz clock
// (profiles/r04/sq_bound_pmc.txt); the block's tables: cauchy_tables().
// Bytes are identical: the same products, reassociated.
// ---------------------------------------------------------------------------
constexpr int kCauchyTabs = 9;  // tables per 4-column group: h0, h1, h0^h1, h2, h3, h2^h3, h0^h2, h1^h3, H

template <int K>
__device__ __forceinline__ void gf_combine_cauchy4(const uint4 (&x)[K], const uint32_t* tl, uint4 (&acc)[4])
{
    static_assert(K % 4 == 0, "4-column groups");
#pragma unroll
    for (int g = 0; g < K / 4; ++g) {
        uint4 q[kCauchyTabs];
        uint32_t t2[kCauchyTabs];
#pragma unroll
        for (int i = 0; i < kCauchyTabs; ++i) {
            const uint32_t* t = &tl[(g * kCauchyTabs + i) * kTabStride];
            q[i] = *reinterpret_cast<const uint4*>(t);
            t2[i] = t[4];
        }
#pragma unroll
        for (int w = 0; w < 4; ++w) {
            const uint32_t x0 = lane_word(x[4 * g + 0], w), x1 = lane_word(x[4 * g + 1], w);
            const uint32_t x2 = lane_word(x[4 * g + 2], w), x3 = lane_word(x[4 * g + 3], w);
            const uint32_t u = x1 ^ x3, v = x2 ^ x3, sm = xor3(x0, x1, v);
            const Sel ss = selectors(sm), su = selectors(u), sv = selectors(v), s3 = selectors(x3);
            auto lk = [&](int i, const Sel& sl, int f) {  // field f of table i at the selectors
                return f == 0 ? __builtin_amdgcn_perm(q[i].y, q[i].x, sl.s0)
                              : f == 1 ? __builtin_amdgcn_perm(q[i].w, q[i].z, sl.s1)
                                       : __builtin_amdgcn_perm(t2[i], t2[i], sl.s2);
            };
            auto mul = [&](int i, const Sel& sl) { return xor3(lk(i, sl, 0), lk(i, sl, 1), lk(i, sl, 2)); };
            const uint32_t m_u01 = mul(2, su), m_u23 = mul(5, su);   // (h0^h1) u, (h2^h3) u
            const uint32_t m_v02 = mul(6, sv), m_v13 = mul(7, sv);   // (h0^h2) v, (h1^h3) v
            const uint32_t m_h = mul(8, s3);                          // H x3
            const uint32_t e02 = m_v02 ^ m_h, e13 = m_v13 ^ m_h;
            const uint32_t z[4] = {m_u01 ^ e02, m_u01 ^ e13, m_u23 ^ e02, m_u23 ^ e13};
            const int hs[4] = {0, 1, 3, 4};  // tables of h0..h3
#pragma unroll
            for (int a = 0; a < 4; ++a) {
                const uint32_t y = g == 0 ? xor3(lk(hs[a], ss, 0), lk(hs[a], ss, 1), lk(hs[a], ss, 2)) ^ z[a]
                                          : xor3(xor3(lane_word(acc[a], w), lk(hs[a], ss, 0), lk(hs[a], ss, 1)),
                                                 lk(hs[a], ss, 2), z[a]);
                set_word(acc[a], w, y);
            }
        }
    }
}

// Host: whether rows r0..r0+3 of p's coefficients are XOR-circulant in every
// 4-column group (M[r0+a][4g+c] == M[r0][4g+(a^c)]), and their tables in the
// order gf_combine_cauchy4 reads them (kCauchyTabs per group, flattened).
inline bool cauchy_blocks(const uint8_t* coef, int cols, int r0, int rows)
{
    if (rows != 4 || cols % 4) return false;
    for (int g = 0; g < cols / 4; ++g)
        for (int a = 0; a < 4; ++a)
            for (int c = 0; c < 4; ++c)
                if (coef[(r0 + a) * cols + 4 * g + c] != coef[r0 * cols + 4 * g + (a ^ c)]) return false;
    return true;
}

inline void cauchy_tables(const uint8_t* coef, int cols, int r0, gf::PermTable* out)
{
    for (int g = 0; g < cols / 4; ++g) {
        const uint8_t* h = &coef[r0 * cols + 4 * g];
        const uint8_t m[kCauchyTabs] = {h[0], h[1], static_cast<uint8_t>(h[0] ^ h[1]), h[2], h[3],
                                        static_cast<uint8_t>(h[2] ^ h[3]), static_cast<uint8_t>(h[0] ^ h[2]),
                                        static_cast<uint8_t>(h[1] ^ h[3]),
                                        static_cast<uint8_t>(h[0] ^ h[1] ^ h[2] ^ h[3])};
        for (int i = 0; i < kCauchyTabs; ++i) out[g * kCauchyTabs + i] = gf::perm_table(m[i]);
    }
}

// ELECT_EC_CAUCHY=0 turns the structured form off (A/B); on by default.
inline bool cauchy_enabled()
{
    static const bool on = [] {
        const char* e = std::getenv("ELECT_EC_CAUCHY");
        return !(e && std::atoi(e) == 0);
    }();
    return on;
}

// ELECT_EC_CAUCHY_LDS=1: the structured form loads through LDS (LDS-DMA) in one-wave launches (A/B).
inline bool cauchy_lds()
{
    static const bool on = [] {
        const char* e = std::getenv("ELECT_EC_CAUCHY_LDS");
        return e && std::atoi(e) == 1;
    }();
    return on;
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
template <int K, int R, bool PAD, bool HASH, bool LDSDMA = false>
__global__ __launch_bounds__(kBlock) void gf_apply_x16(const FastArgs<K, R> a)
{
    __shared__ __attribute__((aligned(16))) uint32_t tl[R * K * kTabStride];
    __shared__ __attribute__((aligned(16))) uint8_t stage[LDSDMA ? K * 1024 : 16];  // (LDSDMA: one-wave blocks)
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
    if constexpr (!PAD && LDSDMA) {
        const uint8_t* src[K];
#pragma unroll
        for (int j = 0; j < K; ++j) src[j] = a.sp[j] + stripe * a.ss[j] + off;
        load_columns_via_lds<K>(src, stage, x);
    } else if (!PAD) {
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
#pragma unroll
            for (int r = 0; r < R; ++r) {
                uint32_t sum;
                if constexpr (kPolicy.hash_dpp_weights)
                    sum = p0 * wave_poly31(horner31(acc[r]));
                else
                    sum = wave_sum(horner31(acc[r]) * (kLanePow.v[threadIdx.x & 63u] * p0));
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
template <int K, int R, bool HASH, bool LDSDMA = false>
__global__ __launch_bounds__(kBlock) void gf_apply_x16u(const FastArgs<K, R> a)
{
    __shared__ __attribute__((aligned(16))) uint32_t tl[R * K * kTabStride];
    __shared__ __attribute__((aligned(16))) uint8_t stage[LDSDMA ? K * 1024 : 16];  // (LDSDMA: one-wave blocks)
    const uint32_t idx = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t first = __builtin_amdgcn_readfirstlane(idx);  // the wave's lane 0
    const uint32_t stripe = div_magic(first, a.magic, a.shift);  // wave-uniform
    const uint32_t off = (idx - stripe * a.segs) * 16u;
    stage_tables<K, R>(a.tab, tl);
    if (first >= a.total) return;  // total % 64 == 0: waves are wholly live or wholly past the end
    uint4 x[K];
    if constexpr (LDSDMA) {
        const uint8_t* src[K];
#pragma unroll
        for (int j = 0; j < K; ++j) src[j] = a.sp[j] + static_cast<uint64_t>(stripe) * a.ss[j] + off;
        load_columns_via_lds<K>(src, stage, x);
    } else {
#pragma unroll
        for (int j = 0; j < K; ++j) x[j] = load_nt(a.sp[j] + static_cast<uint64_t>(stripe) * a.ss[j] + off);
    }
    uint4 acc[R];
    gf_combine<K, R>(x, tl, acc);
#pragma unroll
    for (int r = 0; r < R; ++r) store_nt(a.dp[r] + static_cast<uint64_t>(stripe) * a.ds[r] + off, acc[r]);
    if constexpr (HASH) {
        if (a.hashes) {
            const uint32_t hs = div_magic(first, a.hmagic, a.hshift);
            const uint32_t p0 = a.hpow * pow31_seg(first - hs * a.hsegs);
#pragma unroll
            for (int r = 0; r < R; ++r) {
                uint32_t sum;
                if constexpr (kPolicy.hash_dpp_weights)
                    sum = p0 * wave_poly31(horner31(acc[r]));
                else
                    sum = wave_sum(horner31(acc[r]) * (kLanePow.v[threadIdx.x & 63u] * p0));
                if ((threadIdx.x & 63u) == 0) a.hpart[static_cast<uint64_t>(first >> 6) * R + r] = sum;
            }
        }
    }
}

// The Cauchy-structured plain encode (gf_combine_cauchy4): gf_apply_x16u's
// scalar-base form with the 9-multiplication combine.  92 VGPRs (the nine
// tables of a group live in VGPRs), so 20 waves per CU; asking the allocator
// for 6 / 7 / 8 waves per SIMD spilled 45 / 99 / 103 VGPRs, and the occupancy
// sweep (profiles/r05/rs12_cauchy_ab.txt) is flat above 16 waves per CU.
// LDSDMA (A/B, ELECT_EC_CAUCHY_LDS=1): one-wave blocks load their columns
// through LDS as gf_apply_x16u's LDS-DMA form does.
template <int K, bool LDSDMA = false>
__global__ __launch_bounds__(kBlock) void gf_apply_x16c(const FastArgs<K, 4> a)
{
    __shared__ __attribute__((aligned(16))) uint32_t tl[4 * K * kTabStride];
    __shared__ __attribute__((aligned(16))) uint8_t stage[LDSDMA ? K * 1024 : 16];
    const uint32_t idx = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t first = __builtin_amdgcn_readfirstlane(idx);
    const uint32_t stripe = div_magic(first, a.magic, a.shift);
    const uint32_t off = (idx - stripe * a.segs) * 16u;
    stage_tables<K, 4>(a.tab, tl);
    if (first >= a.total) return;
    uint4 x[K];
    if constexpr (LDSDMA) {
        const uint8_t* src[K];
#pragma unroll
        for (int j = 0; j < K; ++j) src[j] = a.sp[j] + static_cast<uint64_t>(stripe) * a.ss[j] + off;
        load_columns_via_lds<K>(src, stage, x);
    } else {
#pragma unroll
        for (int j = 0; j < K; ++j) x[j] = load_nt(a.sp[j] + static_cast<uint64_t>(stripe) * a.ss[j] + off);
    }
    uint4 acc[4];
    gf_combine_cauchy4<K>(x, tl, acc);
#pragma unroll
    for (int r = 0; r < 4; ++r) store_nt(a.dp[r] + static_cast<uint64_t>(stripe) * a.ds[r] + off, acc[r]);
}

// Padded launches with per-stripe content lengths, no hash, and L % 16 == 0:
// U segments per lane.  The lengths sit on the critical path of every data
// load (no load past a unit's content), so a wave amortises that dependent
// round trip over U x 1 KiB per column instead of 1 KiB; a wave whose 64*U
// segments lie in one stripe reads the lengths once, as scalar loads
// overlapped with the table staging.  The one segment per unit that straddles
// its content length is loaded whole (it lies inside the unit's L bytes) and
// masked, so no byte loads.  Straddling waves take a one-segment-at-a-time path.

template <int K, int R, int U>
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
        }
        return;
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

// Segments per lane for gf_apply_lens: U*K 16-byte loads in flight per lane.
// U = 2 since round 3 (3 interleaved rounds, profiles/r03/padded_and_plain_u_ab.txt):
// ELECT's degraded read 77.3 -> 81.6 % of peak at 64 KiB codeLength and 80.7 ->
// 82.2 % at 4.4 MB in 64 KiB tiles, padded encode at 93 % fill 79.1 -> 80.1 %,
// full units 81.0 -> 82.3 %, random fill 69.1 -> 68.8 % (noise); U = 4 before.
template <int K>
constexpr int lens_unroll() { return K <= 4 ? 2 : 1; }

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
    // Unrolled so that a lane keeps several partial loads in flight: an ELECT-size unit
    // (4.4 MB in 64 KiB tiles) has 4,352 partials per row, 68 per lane.
    if (hi) {
        const uint64_t w0 = start / 64, w1 = (start + segs - 1) / 64;
#pragma unroll 8
        for (uint64_t w = w0 + lane; w <= w1; w += 64) sum += (w * 64 >= start ? part : hi)[w * rows + r];
    } else {
        const uint64_t w0 = (start + 63) / 64, w1 = (start + segs) / 64;
#pragma unroll 8
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


struct LaunchShape {
    int block;
    int waves;  // resident waves per CU, 0 = uncapped
};

enum class Family {
    kPlain,         // gf_apply_x16 / gf_apply_x16u
    kPlainHashed,   // the same with the parity-hash epilogue
    kPadded,        // gf_apply_x16<PAD> (one length per column, or L % 16 != 0)
    kLens,          // gf_apply_lens (per-stripe content lengths, tiles)
    kPaddedHashed,  // gf_apply_x16<PAD, HASH>
    kGroup,         // gf_apply_group
    kUpdate,        // gf_update_x16
};

// The shape of a launch of `cols` source columns and `rows` output rows over
// `len`-byte chunks; scalar_base: the scalar-base form (gf_apply_x16u).
inline LaunchShape launch_shape(Family f, int cols, int rows, uint64_t len, bool scalar_base = false)
{
    const LaunchPolicy& P = kPolicy;
    const bool write_heavy = 2 * rows >= cols;
    const bool wide = cols * rows >= 16;
    // the plain caps for blocks of more than one wave
    // ELECT_EC_WRITE_WAVES overrides P.write_waves (A/B only)
    static const int write_waves = [] {
        const char* e = std::getenv("ELECT_EC_WRITE_WAVES");
        return e ? std::atoi(e) : kPolicy.write_waves;
    }();
    const int multi_cap = write_heavy ? write_waves : (cols >= 8 && rows >= 2) ? P.read_wide_waves : P.read_waves;
    const int one_wave_cap = write_heavy ? P.one_wave_write_waves
                             : cols >= 8 ? P.one_wave_read_wide_waves
                                         : P.one_wave_read_waves;
    // the plain block of a shape: 128 for small chunks, 256 / 128 for wide shapes, else 256
    const int plain_block = len <= P.small_len ? P.small_block
                            : wide            ? (write_heavy ? P.wide_write_block : P.wide_read_block)
                                              : kBlock;
    switch (f) {
    case Family::kPlain:
        if (len > P.small_len && !wide) return {64, one_wave_cap};
        return {plain_block, multi_cap};
    case Family::kPlainHashed: return {P.hashed_block, scalar_base ? P.hashed_scalar_waves : P.hashed_lane_waves};
    case Family::kPadded:
    case Family::kLens: {
        const int block = write_heavy ? std::min(P.padded_write_block, plain_block) : plain_block;
        if (f == Family::kPadded) return {block, 0};
        return {block, write_heavy ? P.lens_write_waves : P.lens_read_waves};
    }
    case Family::kPaddedHashed: return {P.padded_hashed_block, 0};
    case Family::kGroup: return {P.group_block, !wide ? one_wave_cap : multi_cap};
    case Family::kUpdate: return {P.update_block, P.update_waves};
    }
    return {kBlock, 0};
}

constexpr int kMaxHashCols = 10;  // ELECT_EC_MAX_DATA_UNITS: hashed launches are encodes
constexpr size_t kLdsPerCU = 160 * 1024;

// Dynamic LDS that caps a launch of `block`-thread blocks at `waves` resident
// waves per CU (0: none).  The block's static LDS (its coefficient tables) counts.
inline size_t cap_lds(int block, int coefs, int waves)
{
    if (waves <= 0) return 0;
    const int blocks = std::max(1, waves / (block / 64));
    const size_t static_lds = static_cast<size_t>(coefs) * kTabStride * sizeof(uint32_t);
    const size_t per_block = kLdsPerCU / blocks - 512;  // > kLdsPerCU / (blocks + 1): one block fewer fits
    return per_block > static_lds ? per_block - static_lds : 0;
}

inline size_t cap_lds(const LaunchShape& sh, int coefs, size_t extra_static = 0)
{
    const size_t d = cap_lds(sh.block, coefs, sh.waves);
    return d > extra_static ? d - extra_static : 0;
}

// Padded launches the per-stripe-length kernel can take (whole 16-byte segments,
// aligned columns).  (Hashed launches do not: a hashed form of gf_apply_lens
// gained 1 point at 64 KiB codeLength in round 2 and lost to the one-segment
// hashed kernel in one-wave blocks in round 3, profiles/r03/lens_hash_ab.txt;
// it was removed in round 4, its source is in git history before that.)
inline bool lens_eligible(const ApplyParams& p)
{
    return p.aligned16 && p.len % 16 == 0 && p.len > 0 && p.len < (uint64_t{1} << 31);
}

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
    const bool hash_assign = p.hashes && p.hash_seed;  // launch_apply chose assign mode
    // scalar stripe bases: plain launches of whole-wave stripes (kPolicy.scalar_base_min_cols
    // columns and up; hashed ones of any width)
    const bool whole_waves = !PAD && a.segs % 64 == 0 && segs64 < (uint64_t{1} << 28);
    const bool scalar_base = whole_waves && (p.hashes ? K <= kMaxHashCols && K >= kPolicy.hashed_scalar_base_min_cols
                                                      : K >= kPolicy.scalar_base_min_cols);
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
        constexpr int kCoefs = R * K;
        if constexpr (PAD) {
            if (!a.hashes && (a.lens || tiles > 1) && lens_eligible(p)) {
                constexpr int U = lens_unroll<K>();
                const LaunchShape sh = launch_shape(Family::kLens, K, R, p.len);
                const uint64_t threads = (static_cast<uint64_t>(a.total) + 64 * U - 1) / (64 * U) * 64;
                hipLaunchKernelGGL((gf_apply_lens<K, R, U>), dim3(static_cast<uint32_t>((threads + sh.block - 1) / sh.block)),
                                   dim3(sh.block), cap_lds(sh, kCoefs), stream, a);
            } else if (!a.hashes) {
                const LaunchShape sh = launch_shape(Family::kPadded, K, R, p.len);
                hipLaunchKernelGGL((gf_apply_x16<K, R, true, false>), dim3((a.total + sh.block - 1) / sh.block),
                                   dim3(sh.block), cap_lds(sh, kCoefs), stream, a);
            } else if constexpr (K <= kMaxHashCols) {
                const LaunchShape sh = launch_shape(Family::kPaddedHashed, K, R, p.len);
                hipLaunchKernelGGL((gf_apply_x16<K, R, true, true>), dim3((a.total + sh.block - 1) / sh.block),
                                   dim3(sh.block), cap_lds(sh, kCoefs), stream, a);
            }
        } else {
            const LaunchShape sh = launch_shape(a.hashes ? Family::kPlainHashed : Family::kPlain, K, R, p.len, scalar_base);
            const dim3 grid((a.total + sh.block - 1) / sh.block);
            const size_t lds = cap_lds(sh, kCoefs);
            if (!a.hashes) {
                bool launched = false;
                if constexpr (kPolicy.plain_lds_dma > 0) {  // one-wave launches load through LDS
                    // (16-byte aligned columns only: unaligned_vector_ok() vouches for global_load_dwordx4
                    // at any offset, not for the LDS-DMA load)
                    if (sh.block == 64 && p.aligned16 && (kPolicy.plain_lds_dma > 1 || 2 * R < K)) {
                        const size_t lds_d = cap_lds(sh, kCoefs, K * 1024);
                        if (scalar_base && K >= kPolicy.scalar_base_min_cols)
                            hipLaunchKernelGGL((gf_apply_x16u<K, R, false, true>), grid, dim3(sh.block), lds_d, stream, a);
                        else
                            hipLaunchKernelGGL((gf_apply_x16<K, R, false, false, true>), grid, dim3(sh.block), lds_d, stream, a);
                        launched = true;
                    }
                }
                if constexpr (R == 4 && K % 4 == 0 && K >= kPolicy.scalar_base_min_cols) {
                    // Cauchy-generator encodes: the 9-multiplication form (gf_combine_cauchy4)
                    if (!launched && scalar_base && cauchy_enabled() && cauchy_blocks(p.coef, p.cols, r0, R)) {
                        FastArgs<K, R> ac = a;
                        cauchy_tables(p.coef, p.cols, r0, &ac.tab[0][0]);
                        if (sh.block == 64 && p.aligned16 && cauchy_lds())
                            hipLaunchKernelGGL((gf_apply_x16c<K, true>), grid, dim3(sh.block), cap_lds(sh, kCoefs, K * 1024),
                                               stream, ac);
                        else
                            hipLaunchKernelGGL((gf_apply_x16c<K>), grid, dim3(sh.block), lds, stream, ac);
                        launched = true;
                    }
                }
                if constexpr (K >= kPolicy.scalar_base_min_cols) {  // (the scalar-base plain instances)
                    if (!launched && scalar_base) {
                        hipLaunchKernelGGL((gf_apply_x16u<K, R, false>), grid, dim3(sh.block), lds, stream, a);
                        launched = true;
                    }
                }
                if (!launched) hipLaunchKernelGGL((gf_apply_x16<K, R, false, false>), grid, dim3(sh.block), lds, stream, a);
            } else if constexpr (K <= kMaxHashCols) {
                if (scalar_base)
                    hipLaunchKernelGGL((gf_apply_x16u<K, R, true>), grid, dim3(sh.block), lds, stream, a);
                else
                    hipLaunchKernelGGL((gf_apply_x16<K, R, false, true>), grid, dim3(sh.block), lds, stream, a);
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
// size, in one launch (the mixed config's 8-way share 3,879 -> 3,959 GiB/s
// against one launch per block-size class, profiles/r02_group_ab/), of one-wave
// blocks with the plain caps of the shape (round 3: 8-way share 4,272 -> 4,397,
// 4-way 4,312 -> 4,461, 2-way 4,488 -> 4,568, full size 4,461 -> 4,531 GiB/s,
// profiles/r03/plain_one_wave_ab.txt).
// Launch parts [0, n) of a group (all plain, vector-capable, whole segments,
// same coefficients) for output rows r0 .. r0+R-1.
template <int K, int R>
hipError_t launch_group_kr(const ApplyParams* ps, int n, int r0, hipStream_t stream)
{
    GroupArgs<K, R> a{};
    a.n = n;
    for (int r = 0; r < R; ++r)
        for (int j = 0; j < K; ++j) a.tab[r][j] = gf::perm_table(ps[0].coef[(r0 + r) * ps[0].cols + j]);
    bool uni = true;  // every part's stripes hold whole waves: scalar stripe bases
    for (int i = 0; i < n; ++i) uni = uni && (ps[i].len / 16) % 64 == 0 && ps[i].len < (uint64_t{1} << 32);
    const LaunchShape sh = launch_shape(Family::kGroup, K, R, ps[0].len);
    const int block = sh.block;
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
    const size_t lds = cap_lds(sh, R * K);
    if (uni && K >= kPolicy.group_scalar_base_min_cols)
        hipLaunchKernelGGL((gf_apply_group<K, R, true>), dim3(static_cast<uint32_t>(blocks)), dim3(block), lds, stream, a);
    else
        hipLaunchKernelGGL((gf_apply_group<K, R, false>), dim3(static_cast<uint32_t>(blocks)), dim3(block), lds, stream, a);
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
