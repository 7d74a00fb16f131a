/*
 * ec_oracle.h — CPU oracle for ELECT's erasure-coding hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing under elect_amd/ links, loads or calls this
 * code.  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use
 * it, and only as the checker / the timed CPU reference.
 *
 * PARITY UNPINNED.  The reference keeps its GF(2^8) arithmetic in Intel ISA-L
 * (apt package libisal-dev, version unpinned: README.md:23,29), which is not
 * vendored under /root/reference and not installed in this image.  The
 * reference's own C (EC/erasure_coder.c) includes <isa-l.h>, so it cannot be
 * built here without writing a stand-in header, which this project does not do.
 * The reference's only EC test (ErasureCodeTest.java) asserts nothing and holds
 * no vectors.  So this restatement is pinned only by (a) field facts that are
 * independent of ISA-L (GF(2^8)/0x11D axioms, generator order, RAID-6 style
 * known values) and (b) MDS round-trip properties; it is NOT pinned against a
 * run of libec.so/ISA-L.  See DESIGN.md "Oracle".
 *
 * What is restated (EC/ = src/elect/src/native/src/org/apache/cassandra/io/erasurecode):
 *   - ISA-L's public routines used by ELECT, at their call sites:
 *       gf_gen_cauchy1_matrix   EC/erasure_coder.c:43
 *       ec_init_tables          EC/erasure_coder.c:57, :192
 *       ec_encode_data          EC/erasure_coder.c:90, :221
 *       ec_encode_data_update   EC/erasure_coder.c:128
 *       gf_invert_matrix        EC/erasure_coder.c:257
 *       gf_mul                  EC/erasure_coder.c:274
 *   - ELECT's L1 coder logic (initEncoder, encode, encodeUpdate, decode with
 *     processErasures/generateDecodeMatrix and its zero-row quirk).
 *   - ISA-L's SIMD algorithm (split-nibble 32-byte tables + byte shuffle, and the
 *     GFNI affine form) for the timed CPU baseline, with a threaded batch driver.
 */
#ifndef ELECT_EC_ORACLE_H
#define ELECT_EC_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ORACLE_MMAX 14 /* EC/erasure_coder.h:33 */
#define ORACLE_KMAX 10 /* EC/erasure_coder.h:34 */

/* ---- GF(2^8), polynomial 0x11D, generator 2 (ISA-L gf_mul / gf_inv) ---- */
const unsigned char* oracle_gf_exp_table(void); /* 256 entries, exp[255] = exp[0] */
const unsigned char* oracle_gf_log_table(void); /* 256 entries, log[0] unused (0) */
unsigned char oracle_gf_mul(unsigned char a, unsigned char b);
unsigned char oracle_gf_inv(unsigned char a);

/* ---- ISA-L routines (scalar restatement) ---- */
void oracle_gf_gen_cauchy1_matrix(unsigned char* a, int m, int k);
void oracle_gf_vect_mul_init(unsigned char c, unsigned char* tbl32);
void oracle_ec_init_tables(int k, int rows, const unsigned char* a, unsigned char* g_tbls);
void oracle_ec_encode_data(int len, int srcs, int dests, const unsigned char* g_tbls,
                           unsigned char* const* src, unsigned char* const* dest);
void oracle_ec_encode_data_update(int len, int k, int rows, int vec_i,
                                  const unsigned char* g_tbls, const unsigned char* data,
                                  unsigned char* const* dest);
int oracle_gf_invert_matrix(unsigned char* in_mat, unsigned char* out_mat, int n);

/* ---- ELECT L1 coder restated (EC/erasure_coder.c) ---- */
typedef struct oracle_encoder {
    int k, m;
    unsigned char encode_matrix[ORACLE_MMAX * ORACLE_KMAX];
    unsigned char gftbls[ORACLE_MMAX * ORACLE_KMAX * 32];
} oracle_encoder;

int oracle_encoder_init(oracle_encoder* enc, int k, int m);
int oracle_encode(const oracle_encoder* enc, unsigned char* const* data,
                  unsigned char* const* parity, int len);
int oracle_encode_update(const oracle_encoder* enc, unsigned char* const* old_new_parity,
                         int target, unsigned char* const* new_parity, int len);
/* Decode matrix as ELECT builds it.  strict=0 reproduces libec.so (rows >= the
 * number of erased DATA units are zero, EC/erasure_coder.c:261-281); strict=1
 * builds a correct row for every erasure.  Returns 0, or -1 when the survivor
 * matrix is singular (the partially inverted matrix is still used when
 * strict=0, as the reference ignores the failure at EC/erasure_coder.c:257). */
int oracle_decode_matrix(int k, int m, const unsigned char* encode_matrix,
                         const int* decode_indexes, const int* erased, int num_erased,
                         int strict, unsigned char* decode_matrix /* num_erased*k */);
int oracle_decode(int k, int m, unsigned char* const* inputs, const int* decode_indexes,
                  const int* erased, int num_erased, unsigned char* const* outputs,
                  int len, int strict);

/* ---- SIMD restatement of ISA-L's dot-product kernels (CPU baseline) ---- */
enum { ORACLE_SIMD_SCALAR = 0, ORACLE_SIMD_AVX2 = 1, ORACLE_SIMD_AVX512 = 2, ORACLE_SIMD_GFNI = 3 };
int oracle_simd_best(void);
const char* oracle_simd_name(int level);
/* dest[r][i] = XOR_j gf_mul(coef(r,j), src[j][i]); g_tbls laid out as ec_init_tables. */
void oracle_ec_encode_data_simd(int level, size_t len, int k, int rows,
                                const unsigned char* g_tbls, unsigned char* const* src,
                                unsigned char* const* dest);

/* Threaded batch over stripes in a strided layout:
 *   src column j of stripe s at src + s*src_stripe + src_col_off[j]
 *   dst row    r of stripe s at dst + s*dst_stripe + dst_row_off[r]
 * coef is rows x k (row-major).  Returns wall seconds. */
double oracle_batch_apply(int level, int threads, const unsigned char* coef, int rows, int k,
                          size_t len, size_t stripes,
                          const unsigned char* src, size_t src_stripe, const int64_t* src_col_off,
                          unsigned char* dst, size_t dst_stripe, const int64_t* dst_row_off);

/* ---- ELECT's callers around the coder (JEC/net) ----
 * java.nio.ByteBuffer.hashCode() as the JDK specifies it, over [0, n) of a
 * buffer at position 0 / limit n: h = 1; for (i = n-1; i >= 0; i--)
 * h = 31*h + (int)(byte)b[i]; int32 wrap-around.  ELECT names every parity
 * block by it (ECMessageVerbHandler.java:326-329, ECParityUpdateVerbHandler.java:
 * 696-699).  A plain Horner loop, not the closed form the product uses. */
int32_t oracle_java_bytebuffer_hashcode(const unsigned char* b, size_t n);

/* splitmix64 byte stream (little-endian words) used to make fixture inputs. */
void oracle_fill_splitmix(uint64_t seed, unsigned char* buf, size_t len);

#ifdef __cplusplus
}
#endif
#endif
