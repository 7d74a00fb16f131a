/*
 * elect_ec.h — C ABI of the MI355X erasure-coding engine that replaces ELECT's
 * JNI library libec.so (a thin ISA-L wrapper built by EC/genlib.sh:22-26).
 *
 * EC/  = src/elect/src/native/src/org/apache/cassandra/io/erasurecode
 * JEC/ = src/elect/src/java/org/apache/cassandra/io/erasurecode
 *
 * Plain C types only (pointers, sizes, ints); no HIP or torch types appear in
 * the signatures: a hip stream is passed as `void*` (hipStream_t), NULL = the
 * default stream of the calling thread's current device.
 *
 * Threading: a coder is immutable after elect_ec_coder_create(), so every call
 * below is re-entrant and may run concurrently on one coder or on many (the
 * reference shares per-call scratch inside the coder, EC/NativeRSEncoder.c:25-29,
 * EC/erasure_coder.h:50-65, and is safe only because ELECT makes a coder per
 * task).  create/destroy must not race with other calls on the same coder,
 * exactly as Java's write lock already ensures (JEC/NativeRSEncoder.java:33-92).
 *
 * Errors: every function returns an int status (ELECT_EC_OK = 0); nothing is
 * thrown across the ABI.  The JNI shim maps them to the Java
 * exceptions the reference raises (EC/jni_common.h:29-36).
 */
#ifndef ELECT_EC_H
#define ELECT_EC_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ELECT_EC_MAX_DATA_UNITS 10 /* KMAX, EC/erasure_coder.h:34 */
#define ELECT_EC_MAX_UNITS 14      /* MMAX, EC/erasure_coder.h:33 */
#define ELECT_EC_MAX_APPLY 16      /* rows / columns of elect_ec_apply_batch */

/* status codes */
#define ELECT_EC_OK 0
#define ELECT_EC_WARN_SINGULAR 1 /* compat decode ran on a singular survivor set, as libec.so does */
#define ELECT_EC_EINVAL (-1)     /* bad argument (counts, indexes, NULL pointers)           */
#define ELECT_EC_ESINGULAR (-2)  /* strict decode: survivor rows are not invertible           */
#define ELECT_EC_EDEVICE (-3)    /* HIP runtime error                                          */
#define ELECT_EC_ENOMEM (-4)     /* host or device allocation failed                           */
#define ELECT_EC_ENODEV (-5)     /* no usable MI355X device                                    */

/* decode modes */
#define ELECT_EC_DECODE_COMPAT 0 /* bit-exact libec.so: rows past the erased DATA count are zero
                                    (EC/erasure_coder.c:261-281) */
#define ELECT_EC_DECODE_STRICT 1 /* every erased unit (data or parity) reconstructed */

/* decode_batch layout flags */
#define ELECT_EC_INPUTS_BY_UNIT 1u  /* survivor j at inputs.base + decode_indexes[j]*shard_stride
                                       (stripe-resident layout); default: j*shard_stride */
#define ELECT_EC_OUTPUTS_BY_UNIT 2u /* output r at outputs.base + erased[r]*shard_stride
                                       (rebuild in place); default: r*shard_stride */

typedef struct elect_ec_coder elect_ec_coder;

/* A set of shards over a batch of stripes on the device: shard i of stripe s
 * starts at base + s*stripe_stride + i*shard_stride. */
typedef struct elect_ec_shards {
    void* base;
    size_t stripe_stride;
    size_t shard_stride;
} elect_ec_shards;

/* One column of an arbitrary product: stripe s at ptr + s*stripe_stride. */
typedef struct elect_ec_column {
    void* ptr;
    size_t stripe_stride;
} elect_ec_column;

const char* elect_ec_version(void);
/* Content hash of the sources this library was built from (elect_amd/build.py),
 * or "unstamped" for builds outside that recipe. */
const char* elect_ec_build_id(void);
const char* elect_ec_strerror(int status);
/* Number of visible HIP devices (0 with ELECT_EC_ENODEV when none). */
int elect_ec_device_count(int* count);
/* *ok = 1 when device-resident layouts whose shard starts are not 16-byte
 * aligned (any byte offset, e.g. a contiguous [B][k+m][L] batch with L % 16 != 0)
 * run the vector kernels on the calling thread's current device; 0 when they
 * fall back to the byte-granular kernel.  Checked once per device. */
int elect_ec_unaligned_vector_ok(int* ok);
/* Diagnostics: the HBM ceilings the coding kernels are measured against
 * (bench.py's roofline).  Enqueues one probe kernel on `stream` (a hipStream_t,
 * NULL = the null stream) of the current device: 16 bytes per lane with the
 * coding kernels' non-temporal loads and stores, `block` = 64, 128 or 256
 * threads, at most waves_per_cu resident waves per CU (0: uncapped).
 * kind 0: read `bytes` of src (dst: a device buffer of >= 256 bytes that is
 * written only if the data hits a magic value); 1: write `bytes` of dst;
 * 2: copy `bytes` from src to dst; 3 / 4: the coding kernels' stream mixes,
 * four `bytes`-long input streams back to back in src XORed into one (3,
 * decode-shaped) or two (4, encode-shaped) output streams back to back in dst.
 * kind | 0x100: XCD-major block order (each of the 8 XCDs streams one
 * contiguous eighth; needs bytes / 16 a multiple of block and the block count
 * a multiple of 8).  bytes % 16 == 0.  No reference counterpart: ELECT has no
 * device path. */
int elect_ec_hbm_probe(int kind, const void* src, void* dst, size_t bytes, int block, int waves_per_cu,
                       void* stream);

/* Stream-mix ceiling probe (diagnostics): the access pattern of a coding
 * launch without its GF arithmetic.  num_in input columns (4 or 8), each
 * reading only its content when `lengths` (device, [stripe][num_in] uint32) is
 * given (the padded kernels' pattern: content only, the segment holding the
 * end read whole and masked), XORed into num_out output columns (1, 2 or 4)
 * written in full, over whole 16-byte segments of chunk_size bytes,
 * `block`-thread blocks (64, 128, 256), at most waves_per_cu waves per CU
 * (0: uncapped).  bench.py reports the padded and fused-step kernels as
 * fractions of it.  No reference counterpart. */
int elect_ec_mix_probe(int num_in, int num_out, size_t chunk_size, size_t num_stripes, const elect_ec_column* src,
                       const uint32_t* lengths, const elect_ec_column* dst, int block, int waves_per_cu, void* stream);

/* Devices for the host-memory calls.  By default a calling thread uses its
 * current HIP device.  With a device list, each calling thread is assigned one
 * device of the list (round robin, on its first call) and keeps it, so one
 * process — ELECT runs one JVM per node — spreads its coding threads over every
 * GPU of the node.  The list can also come from the environment:
 * ELECT_EC_DEVICES=all or ELECT_EC_DEVICES=0,2,5 (read once, at the first call).
 * n = 0 restores the default.  Returns ELECT_EC_EINVAL for an unknown device. */
int elect_ec_set_host_devices(const int* devices, int n);

/* NUMA placement of the host-memory calls (round 6).  With a device list, a
 * calling thread is assigned, on its first call, a least-loaded device of the
 * list (threads already assigned to it), one on its own NUMA node (the node it
 * runs on then, getcpu) whenever one of those is among the least loaded; no
 * device is ever more than one thread ahead of another.
 * ELECT's coding threads allocate and fill their units themselves
 * (ECMessageVerbHandler.java:298-314), so with first-touch placement a GPU on
 * the thread's node reads them without crossing the socket link.
 * ELECT_EC_NUMA=0 turns the node preference off.
 * elect_ec_device_numa_node: the node of a HIP device (its PCI function's
 * sysfs numa_node; -1 unknown).  elect_ec_host_device_map (diagnostics, no
 * device needed): the devices that threads on thread_nodes[0..num_threads)
 * would get, in that order, from devices[] on device_nodes[]. */
int elect_ec_device_numa_node(int device, int* node);
int elect_ec_host_device_map(const int* devices, const int* device_nodes, int num_devices, const int* thread_nodes,
                             int num_threads, int* out);

/* Cross-thread batching of host-memory calls (on by default; ELECT_EC_BATCH=0
 * turns it off; ELECT_EC_BATCH_WINDOW_US, ELECT_EC_BATCH_ARENA_MB).  While
 * on, concurrent elect_ec_encode / elect_ec_decode calls of the same shape share
 * one pinned arena, one H2D, one kernel launch and one D2H; each call still
 * returns only when its own outputs are written.  Dispatch is self-clocking: a
 * batch leaves when the previous batch's inputs are on the device (at once on
 * an idle device, or after window_us if non-zero), so transfers pipeline.
 * arena_bytes (per direction, x3 arenas by default, ELECT_EC_BATCH_SLABS, per device) takes effect for devices
 * whose batcher has not started yet.  ELECT issues up to concurrent_ec (64)
 * such calls at once (conf/elect.yaml:598): there batching measured 4x the
 * per-thread path (46-50 vs 12.5 GiB/s on 4.4 MB stripes); a lone caller runs
 * at the per-thread path's rate (11.5-14 GiB/s). */
int elect_ec_set_batching(int enable, unsigned window_us, size_t arena_bytes);

/* Counters of the host-memory path since the process started, for diagnostics:
 * out[0] zero-copy calls (a lone caller's buffers page-locked and coded in
 * place over PCIe; ELECT_EC_ZEROCOPY=0 off (the default since round 5), 1 lone
 * callers, 2 every eligible call),
 * out[1] zero-copy attempts that fell back (registration refused), out[2]
 * calls coded through the cross-thread batcher with staging copies, out[3]
 * calls coded by the per-thread staging engine, out[4] calls coded through the
 * batcher by DMA straight from and to elect_ec_host_alloc buffers, out[5] calls
 * coded through the batcher by DMA straight from and to the caller's own
 * pageable units, page-locked for the call (ELECT_EC_REGISTER=1: each unit's
 * interior pages; its partial end pages are staged), out[6] such attempts that
 * took the staged path instead (no free registration slot, ELECT_EC_REGISTER_SLOTS,
 * or a range refused because it shares a page with a live registration of
 * another extent), out[7] unlock failures (hsa_amd_memory_unlock; 0 unless the
 * runtime's locks were disturbed by another party), out[8..10] CPU time in ns
 * spent registering, unregistering, and issuing batches in the dispatcher
 * threads, out[11..17] wall time in ns of the batched calls' phases, summed
 * over calls (locking the units; copying arena edges and joining a batch;
 * waiting for the batch's issue; the issue, per batch; issue end to the
 * poller seeing the batch done, per batch; done to the caller awake; awake to
 * return, edges out and unlocks), out[18] batches issued.  Writes min(n, 19)
 * entries; returns the count. */
int elect_ec_host_path_stats(uint64_t* out, int n);

/* Page-locked host memory for the units of host-memory calls.  ELECT allocates
 * a direct ByteBuffer per unit and stripe (ECMessageVerbHandler.java:298-314,
 * ECParityUpdateVerbHandler.java, ECRecovery.java) and copies its SSTable
 * into it; allocated here instead (NewDirectByteBuffer over this memory, see
 * INTEGRATION.md), a call whose every unit lies in such buffers is moved by DMA
 * straight between them and the device, with no staging copies: the bulk of
 * the CPU the host path costs on pageable buffers.  Pooled (64 KiB size
 * classes, ELECT_EC_HOST_POOL_MB of free buffers kept, default 4096): freeing
 * and allocating one size per stripe reuses the same page-locked memory.
 * When page-locked memory is unavailable the buffer is ordinary memory and
 * calls on it take the staged path; *out is NULL only when no memory at all
 * could be had (ELECT_EC_ENOMEM).  The blocks are ordinary memory locked with
 * hsa_amd_memory_lock for every GPU (ELECT_EC_POOL_ALLOC=hip: hipHostMalloc
 * instead), so the HIP runtime does not list them as its own pinned memory:
 * pass them to this library's calls, not to hipHostGetDevicePointer.  Usable
 * from any thread; free with
 * elect_ec_host_free (EINVAL for a pointer not from elect_ec_host_alloc). */
int elect_ec_host_alloc(size_t bytes, void** out);
int elect_ec_host_free(void* ptr);
/* 1 when [ptr, ptr + bytes) lies in one page-locked elect_ec_host_alloc buffer. */
int elect_ec_host_pinned(const void* ptr, size_t bytes);

/* ---- coder lifecycle ----
 * Replaces initEncoder / initDecoder (EC/erasure_coder.c:49-72) as called by
 * NativeRSEncoder_initImpl (EC/NativeRSEncoder.c:31-40) and NativeRSDecoder_initImpl
 * (EC/NativeRSDecoder.c:32-41); destroy replaces the destroyImpl pair
 * (EC/NativeRSEncoder.c:86-95, EC/NativeRSDecoder.c:73-82).  Host-only work.
 * Limits as the reference: 1 <= k <= 10, m >= 1, k + m <= 14. */
int elect_ec_coder_create(int num_data_units, int num_parity_units, elect_ec_coder** out);
void elect_ec_coder_destroy(elect_ec_coder* coder);
int elect_ec_coder_num_data_units(const elect_ec_coder* coder);
int elect_ec_coder_num_parity_units(const elect_ec_coder* coder);
/* (k+m) x k generator (gf_gen_cauchy1_matrix, EC/erasure_coder.c:43). */
int elect_ec_coder_encode_matrix(const elect_ec_coder* coder, unsigned char* out, size_t out_len);
/* m*k*32 bytes of ISA-L-layout tables for the parity rows (ec_init_tables,
 * EC/erasure_coder.c:57-59) — for callers that persist or compare them. */
int elect_ec_coder_gf_tables(const elect_ec_coder* coder, unsigned char* out, size_t out_len);
/* num_erased x k decode matrix exactly as processErasures/generateDecodeMatrix
 * build it (EC/erasure_coder.c:161-200, 241-284) in the given mode.  Returns
 * ELECT_EC_WARN_SINGULAR (compat) or ELECT_EC_ESINGULAR (strict) for a singular
 * survivor set. */
int elect_ec_coder_decode_matrix(const elect_ec_coder* coder, const int* decode_indexes,
                                 const int* erased_indexes, int num_erased, int mode,
                                 unsigned char* out);
/* k x k inverse of the survivor rows of the generator, in decode_indexes order
 * (gf_invert_matrix, EC/erasure_coder.c:257-258).  A singular survivor set
 * leaves the partially reduced matrix gf_invert_matrix stops at, with
 * ELECT_EC_WARN_SINGULAR.  For the verbose dumps (EC/dump.c:76-104). */
int elect_ec_coder_invert_matrix(const elect_ec_coder* coder, const int* decode_indexes, unsigned char* out);

/* ---- host memory, synchronous: the JNI calling convention ----
 * Replace encode / encodeUpdate / decode (EC/erasure_coder.h:77-79, bodies at
 * EC/erasure_coder.c:74-98, 100-142, 202-226).  Buffers are host pointers
 * (JVM direct ByteBuffers + position, EC/jni_common.c:62-108); outputs are
 * complete when the call returns.  Runs on the calling thread's current HIP
 * device through per-thread pinned staging and two streams. */
int elect_ec_encode(const elect_ec_coder* coder, const unsigned char* const* data_units,
                    unsigned char* const* parity_units, size_t chunk_size);
/* inputs: [old data, new data, old parity 0..m-1] (EC/NativeRSEncoder.c:79);
 * outputs: m new parity units; may alias the old parity inputs. */
int elect_ec_encode_update(const elect_ec_coder* coder, const unsigned char* const* old_new_parity,
                           int target_data_index, unsigned char* const* new_parity_units,
                           size_t chunk_size);
/* inputs: k survivors ordered like decode_indexes[0..k-1]; outputs: num_erased. */
int elect_ec_decode(const elect_ec_coder* coder, const unsigned char* const* inputs,
                    const int* decode_indexes, const int* erased_indexes, int num_erased,
                    unsigned char* const* outputs, size_t chunk_size, int mode);

/* Implicit zero padding (host memory): data unit j holds only data_lengths[j]
 * <= chunk_size valid bytes and reads as zero past that, exactly like ELECT's
 * zero fill up to codeLength (JEC/net/ECMessageVerbHandler.java:292-310);
 * data_units[j] may be NULL when data_lengths[j] == 0 (ELECT's all-zero filler
 * chunks, :174-184).  Only the valid bytes are copied and sent to the device. */
int elect_ec_encode_padded(const elect_ec_coder* coder, const unsigned char* const* data_units,
                           const size_t* data_lengths, unsigned char* const* parity_units,
                           size_t chunk_size);

/* encode + java.nio.ByteBuffer.hashCode() of every parity unit (hashes[r], int32),
 * fused into the encode kernel.  ELECT names parity blocks by this hash right
 * after encoding (JEC/net/ECMessageVerbHandler.java:326-329,
 * ECParityUpdateVerbHandler.java:696-699): h = 1; for i = L-1..0: h = 31*h + b[i]
 * over signed bytes, i.e. 31^L + sum_i b[i]*31^i mod 2^32. */
int elect_ec_encode_hashed(const elect_ec_coder* coder, const unsigned char* const* data_units,
                           unsigned char* const* parity_units, size_t chunk_size, int32_t* hashes);

/* ---- ELECT's two coding-node steps, each fused into one pass (host memory) ----
 * encode_ex is the whole redundancy-transition encode of
 * JEC/net/ECMessageVerbHandler.java:283-329: zero fill of each SSTable up to
 * codeLength (data_lengths, NULL = all full), encode, and the parity
 * hashCode() values that name the parity blocks (hashes, NULL = not wanted).
 * encode_padded / encode_hashed are the two halves of it. */
int elect_ec_encode_ex(const elect_ec_coder* coder, const unsigned char* const* data_units,
                       const size_t* data_lengths, unsigned char* const* parity_units,
                       size_t chunk_size, int32_t* hashes);
/* encode_update_ex is the whole parity update of ECParityUpdateVerbHandler.java:
 * 634-699: old and new SSTable contents zero filled up to codeLength
 * (old_new_lengths[0..1], NULL = both full; a NULL data pointer is allowed for a
 * zero length), P'[r] = P[r] ^ E[k+r][target] * (old ^ new) (ec_encode_data_update,
 * EC/erasure_coder.c:100-142), and hashCode() of every new parity unit (hashes,
 * NULL = not wanted; codes with m >= 9 hash on the byte-granular kernel).
 * Inputs [old, new, P0..Pm-1] as
 * elect_ec_encode_update; outputs may alias the old parity. */
int elect_ec_encode_update_ex(const elect_ec_coder* coder, const unsigned char* const* old_new_parity,
                              const size_t* old_new_lengths, int target_data_index,
                              unsigned char* const* new_parity_units, size_t chunk_size, int32_t* hashes);
/* decode_ex is the degraded-read decode of JEC/net/ECRecovery.java:128-149: each
 * survivor holds input_lengths[j] content bytes (NULL = all full) and reads as
 * zero past them (ELECT copies survivors into zero-filled codeLength buffers,
 * :130-133).  chunk_size may be only the prefix the caller needs (ECRecovery
 * keeps dataFileSize bytes of the rebuilt unit, :146-149): RS works bytewise,
 * so a prefix decode reads only that prefix of each survivor.  Lengths above
 * chunk_size are clamped to it. */
int elect_ec_decode_ex(const elect_ec_coder* coder, const unsigned char* const* inputs,
                       const size_t* input_lengths, const int* decode_indexes, const int* erased_indexes,
                       int num_erased, unsigned char* const* outputs, size_t chunk_size, int mode);

/* ---- device resident, batched, stream ordered ----
 * Many stripes per launch.  All pointers are device pointers on the calling
 * thread's current device; the call only enqueues work on `stream`.  16-byte
 * aligned bases and strides take the dwordx4 kernels; anything else is still
 * correct (byte-granular kernel). */
int elect_ec_encode_batch(const elect_ec_coder* coder, size_t chunk_size, size_t num_stripes,
                          elect_ec_shards data, elect_ec_shards parity, void* stream);
int elect_ec_decode_batch(const elect_ec_coder* coder, size_t chunk_size, size_t num_stripes,
                          elect_ec_shards inputs, const int* decode_indexes,
                          const int* erased_indexes, int num_erased, elect_ec_shards outputs,
                          unsigned flags, int mode, void* stream);
/* Zero-padded batch encode: data_lengths is a DEVICE array [num_stripes][k] of
 * uint32 content lengths; bytes past a unit's length read as zero whatever the
 * buffer holds there, and a length above chunk_size counts as chunk_size (so
 * no load ever leaves a unit).  Loads stop at the 16-byte segment holding a
 * unit's last content byte (always inside its chunk_size bytes). */
int elect_ec_encode_batch_padded(const elect_ec_coder* coder, size_t chunk_size, size_t num_stripes,
                                 elect_ec_shards data, const uint32_t* data_lengths,
                                 elect_ec_shards parity, void* stream);
/* encode_batch + parity hashes: d_hashes is a DEVICE array [num_stripes][m] of
 * int32, overwritten with each parity unit's ByteBuffer.hashCode(). */
int elect_ec_encode_batch_hashed(const elect_ec_coder* coder, size_t chunk_size, size_t num_stripes,
                                 elect_ec_shards data, elect_ec_shards parity, int32_t* d_hashes,
                                 void* stream);
/* parity_out[r] = parity_in[r] ^ E[k+r][target] * (old ^ new) for each stripe. */
int elect_ec_encode_update_batch(const elect_ec_coder* coder, size_t chunk_size,
                                 size_t num_stripes, int target_data_index,
                                 elect_ec_column old_data, elect_ec_column new_data,
                                 elect_ec_shards parity_in, elect_ec_shards parity_out,
                                 void* stream);
/* Device-resident forms of encode_ex / encode_update_ex: one launch per call.
 * d_data_lengths: DEVICE uint32 [num_stripes][k] (NULL = all full);
 * d_old_new_lengths: DEVICE uint32 [num_stripes][2], old then new content
 * length (NULL = both full); d_hashes: DEVICE int32 [num_stripes][m], overwritten
 * (NULL = not wanted; an update of an m >= 9 code hashes on the byte-granular
 * kernel, and its tiled form needs m <= 8).  parity_out may equal
 * parity_in (in place). */
int elect_ec_encode_batch_ex(const elect_ec_coder* coder, size_t chunk_size, size_t num_stripes,
                             elect_ec_shards data, const uint32_t* d_data_lengths, elect_ec_shards parity,
                             int32_t* d_hashes, void* stream);
int elect_ec_encode_update_batch_ex(const elect_ec_coder* coder, size_t chunk_size, size_t num_stripes,
                                    int target_data_index, elect_ec_column old_data, elect_ec_column new_data,
                                    const uint32_t* d_old_new_lengths, elect_ec_shards parity_in,
                                    elect_ec_shards parity_out, int32_t* d_hashes, void* stream);
/* decode_batch with survivors zero padded: d_input_lengths is a DEVICE uint32
 * [num_stripes][k] array in decode_indexes order (above chunk_size counts as
 * chunk_size). */
int elect_ec_decode_batch_ex(const elect_ec_coder* coder, size_t chunk_size, size_t num_stripes,
                             elect_ec_shards inputs, const uint32_t* d_input_lengths, const int* decode_indexes,
                             const int* erased_indexes, int num_erased, elect_ec_shards outputs,
                             unsigned flags, int mode, void* stream);
/* ---- device resident, tiled units ----
 * The three _ex calls with every unit of chunk_size bytes stored as
 * T = ceil(chunk_size / tile_bytes) tiles of tile_bytes bytes (a multiple of
 * 16; 65536 is the unit size HBM streams best, DESIGN.md §3, so ELECT's
 * codeLength of 4,404,020 B runs as 68 tiles at the 64 KiB rate).  The shard
 * descriptors address TILES: tile t of unit j of stripe s starts at
 *   base + (s*T + t) * stripe_stride + j * shard_stride
 * (a [B][T][k+m][tile] block: stripe_stride = (k+m)*tile, shard_stride = tile).
 * Content lengths (NULL = all chunk_size) and hashes are per STRIPE exactly as
 * in the _ex calls, and the bytes produced are those of coding each unit whole:
 * bytes of a unit's last tile past chunk_size are never read, and the outputs
 * there are written as zero.  Needs the vector kernels (16-byte aligned bases
 * and strides, or elect_ec_unaligned_vector_ok) and at most 10 columns. */
int elect_ec_encode_batch_tiled(const elect_ec_coder* coder, size_t chunk_size, size_t tile_bytes,
                                size_t num_stripes, elect_ec_shards data, const uint32_t* d_data_lengths,
                                elect_ec_shards parity, int32_t* d_hashes, void* stream);
int elect_ec_encode_update_batch_tiled(const elect_ec_coder* coder, size_t chunk_size, size_t tile_bytes,
                                       size_t num_stripes, int target_data_index, elect_ec_column old_data,
                                       elect_ec_column new_data, const uint32_t* d_old_new_lengths,
                                       elect_ec_shards parity_in, elect_ec_shards parity_out, int32_t* d_hashes,
                                       void* stream);
int elect_ec_decode_batch_tiled(const elect_ec_coder* coder, size_t chunk_size, size_t tile_bytes,
                                size_t num_stripes, elect_ec_shards inputs, const uint32_t* d_input_lengths,
                                const int* decode_indexes, const int* erased_indexes, int num_erased,
                                elect_ec_shards outputs, unsigned flags, int mode, void* stream);
/* ---- several device batches in one call ----
 * Batches of different chunk sizes (ELECT's mixed SSTable sizes, the mixed 1 KiB /
 * 4 KiB / 1 MiB config) coded with one coder: the same bytes as one
 * elect_ec_encode_batch / elect_ec_decode_batch per element, but batches with
 * whole 16-byte segments share one launch (up to 8 per launch), so a step of
 * many short batches pays one kernel ramp-up and drain instead of one per batch. */
typedef struct elect_ec_batch {
    size_t chunk_size;
    size_t num_stripes;
    elect_ec_shards in;   /* encode: data units; decode: survivors (or stripes, ELECT_EC_INPUTS_BY_UNIT) */
    elect_ec_shards out;  /* encode: parity units; decode: rebuilt units (or stripes, ELECT_EC_OUTPUTS_BY_UNIT) */
} elect_ec_batch;
int elect_ec_encode_batches(const elect_ec_coder* coder, const elect_ec_batch* batches, int num_batches,
                            void* stream);
/* One erasure pattern for every batch. */
int elect_ec_decode_batches(const elect_ec_coder* coder, const elect_ec_batch* batches, int num_batches,
                            const int* decode_indexes, const int* erased_indexes, int num_erased,
                            unsigned flags, int mode, void* stream);
/* General product dst[r] = XOR_j coef[r*cols+j] * src[j], rows, cols <= 16. */
int elect_ec_apply_batch(const unsigned char* coef, int rows, int cols, size_t chunk_size,
                         size_t num_stripes, const elect_ec_column* src,
                         const elect_ec_column* dst, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* ELECT_EC_H */
