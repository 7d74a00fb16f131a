// rs_kernels.hpp — internal launch interface of the gfx950 GF(2^8) kernels.
//
// One kernel family serves every byte-stream operation of ELECT's coder:
//   encode        -> ec_encode_data(len, k, m, ...)          EC/erasure_coder.c:90
//   decode        -> ec_encode_data(len, k, numErased, ...)  EC/erasure_coder.c:221
//   encodeUpdate  -> ec_encode_data_update(...)              EC/erasure_coder.c:128
// all as  dst[r][i] = XOR_j coef[r][j] * src[j][i]  over a batch of stripes.
// (EC/ = src/elect/src/native/src/org/apache/cassandra/io/erasurecode)
#pragma once

#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>

#include "gf256.hpp"

namespace elect {
namespace kern {

constexpr int kMaxCols = 16;  // source columns per launch
constexpr int kMaxRows = 16;  // output rows per call (fast kernels take 4 per launch)
constexpr int kFastRows = 4;
// Widest padded (and so tiled) vector instance: ELECT_EC_MAX_DATA_UNITS.  Tiled
// launches need the padded vector kernels, so a wider product (an update of an
// m >= 9 code: 2 + m columns) must be coded untiled.
constexpr int kMaxPadCols = 10;

// A shard column over a batch of stripes: stripe s's bytes start at ptr + s*stride.
struct Column {
    const uint8_t* ptr = nullptr;
    uint64_t stride = 0;
};

struct ApplyParams {
    Column src[kMaxCols];
    Column dst[kMaxRows];  // written through (uint8_t*)ptr
    uint64_t len = 0;      // bytes per shard
    uint64_t stripes = 0;  // stripes in the batch
    int cols = 0;
    int rows = 0;
    uint8_t coef[kMaxRows * kMaxCols] = {};  // rows x cols, row-major
    // Implicit zero padding (padded == true): column j of stripe s holds only
    // lens[s * cols + j] valid bytes (device array), or clen[j] for every
    // stripe when lens is null; bytes past that read as zero.  This is ELECT's
    // zero fill up to codeLength (ECMessageVerbHandler.java:292-310) and its
    // all-zero filler chunks (:174-184), without storing or reading the zeros.
    bool padded = false;
    const uint32_t* lens = nullptr;
    uint32_t clen[kMaxCols] = {};
    // lens holds lens_stride entries per stripe (0: cols) for the first
    // lens_cols columns (0: all); the other columns hold clen[j] valid bytes.
    // ELECT's parity update pads old/new SSTables but not the old parity
    // (ECParityUpdateVerbHandler.java:643-663).
    int lens_cols = 0;
    uint32_t lens_stride = 0;
    uint32_t col_base = 0;  // internal: byte offset of a launch window inside the shard
    // Optional java.nio.ByteBuffer.hashCode() of every output row (ELECT names
    // parity by it, ECMessageVerbHandler.java:326-329):
    //   h = 31^L + sum_i sb[i] * 31^i  (mod 2^32, sb = signed byte).
    // The kernels ADD sum_i sb[i] * 31^(hash_base + i) into hashes[s*hash_stride + r]
    // with integer atomics (exact, order-independent); the caller initialises
    // every entry to 31^L first.
    int32_t* hashes = nullptr;
    uint32_t hash_stride = 0;
    uint64_t hash_base = 0;
    // hash_seed: the entries are NOT initialised; launch_apply produces
    // 31^len + sum itself.  Where every wave of the fast kernel covers at most
    // two stripes (>= 64 segments per stripe) the per-wave partials are summed
    // and assigned by hash_reduce with no memset and no atomics; otherwise the
    // launcher seeds the entries (hipMemsetD32Async) and the kernels add.
    bool hash_seed = false;
    // Optional caller-owned device scratch for the per-wave hash partials
    // (hash_scratch_need() words, used in the caller's stream order); without
    // it launch_apply leases the stream's cached buffer.
    uint32_t* hash_scratch = nullptr;
    size_t hash_scratch_words = 0;
    // Tiled units: each logical unit of unit_len bytes is stored as `tiles`
    // tiles of len bytes, tile t of logical stripe g being coding stripe
    // g * tiles + t (so `stripes` counts tiles, a multiple of `tiles`).  The
    // content lengths (lens, clen) and the hashes are per LOGICAL unit; a tile
    // holds its share of its unit's content and the bytes past unit_len are
    // never read (they code as zero).  Units of any length can then be coded
    // as 64 KiB units back to back, the layout HBM streams best.
    // Needs padded, len % 16 == 0 and the vector kernels.
    uint32_t tiles = 1;
    uint64_t unit_len = 0;  // 0: len (untiled)
    // internal (launch_apply): every column start is 16-byte aligned.  When it
    // is not, the dwordx4 kernels still run (unaligned vector access, see
    // unaligned_vector_ok) except gf_apply_lens, whose buffer loads need it.
    bool aligned16 = true;
};

// 31^e mod 2^32 (host side of the parity hash).
inline uint32_t pow31(uint64_t e)
{
    uint32_t r = 1, b = 31;
    for (; e; e >>= 1, b *= b)
        if (e & 1) r *= b;
    return r;
}

// par_out[r] = par_in[r] ^ coef[r] * (old ^ new): ec_encode_data_update with
// ELECT's old^new folding (EC/erasure_coder.c:100-142), fused into one pass.
struct UpdateParams {
    Column old_data;
    Column new_data;
    Column par_in[kMaxRows];
    Column par_out[kMaxRows];
    uint64_t len = 0;
    uint64_t stripes = 0;
    int rows = 0;
    uint8_t coef[kMaxRows] = {};
};

hipError_t launch_apply(const ApplyParams& p, hipStream_t stream);

// n batches with the same cols, rows and coefficients: the plain ones (no padding,
// hashes or tiles, whole segments) share grouped launches; the rest launch alone.
hipError_t launch_apply_many(const ApplyParams* ps, int n, hipStream_t stream);

// Scratch words a hashed launch_apply over `segments` 16-byte segments in all
// (stripes x ceil(len/16)) needs at most (row groups run one after another).
constexpr size_t hash_scratch_need(uint64_t segments) { return (segments / 64 + 1) * kFastRows * 2; }
hipError_t launch_update(const UpdateParams& p, hipStream_t stream);

// One piece of a gather / scatter between host and device memory (host path,
// direct batches): n bytes from src to dst, both device-accessible addresses.
struct CopyPiece {
    const uint8_t* src;
    uint8_t* dst;
    uint32_t n;
    uint32_t pad;
};
constexpr uint32_t kMaxPieceBytes = 1u << 16;  // callers split longer ranges

// Copies every piece of the device array `pieces` (one block each).
hipError_t launch_copy_pieces(const CopyPiece* pieces, uint32_t n, hipStream_t stream);

// True when every column start is 16-byte aligned for every stripe.
bool apply_is_aligned(const ApplyParams& p);

// True when 16-byte global loads and stores at any byte offset are exact on the
// current device (checked once per device by a tiny kernel).  Then misaligned
// layouts run the dwordx4 kernels too; otherwise the byte-granular kernel.
bool unaligned_vector_ok();

// HBM ceiling probes (diagnostics, elect_ec_hbm_probe): one 16-byte segment per
// lane with the kernels' non-temporal loads/stores, `block`-thread blocks, at
// most `waves` waves per CU (0: uncapped).  kind 0: read `bytes` of src (dst
// takes one dword per lane of a wave whose data hits a magic value: at least
// 256 bytes); 1: write `bytes` of dst; 2: copy src -> dst.
hipError_t hbm_probe(int kind, const void* src, void* dst, size_t bytes, int block, int waves, hipStream_t stream);

// Stream-mix ceiling probe (elect_ec_mix_probe): nin inputs (4 or 8; optional
// content lengths [stripe][nin], device) XORed into nout outputs (1, 2 or 4),
// whole 16-byte segments of len bytes, `block`-thread blocks, <= waves per CU.
hipError_t mix_probe(int nin, int nout, uint64_t len, uint64_t stripes, const Column* src, const uint32_t* lens,
                     const Column* dst, int block, int waves, hipStream_t stream);

}  // namespace kern
}  // namespace elect
