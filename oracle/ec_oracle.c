/*
 * ec_oracle.c — CPU oracle for ELECT's erasure-coding path.  TEST INFRASTRUCTURE
 * ONLY; PARITY UNPINNED (see ec_oracle.h for what that means and why).
 *
 * Reference anchors (EC/ = src/elect/src/native/src/org/apache/cassandra/io/erasurecode):
 *   encode matrix  EC/erasure_coder.c:39-47  -> gf_gen_cauchy1_matrix (ISA-L)
 *   tables         EC/erasure_coder.c:57-59  -> ec_init_tables (ISA-L)
 *   encode         EC/erasure_coder.c:74-98  -> ec_encode_data (ISA-L)
 *   encodeUpdate   EC/erasure_coder.c:100-142-> ec_encode_data_update (ISA-L)
 *   decode         EC/erasure_coder.c:161-226, 241-284 -> gf_invert_matrix, gf_mul
 * The ISA-L semantics restated here follow ISA-L's published base (non-SIMD)
 * implementation (erasure_code/ec_base.c) and, for the CPU baseline, its SIMD
 * dot-product algorithm (32-byte nibble tables + byte shuffle; GFNI affine).
 */
#include "ec_oracle.h"

#include <pthread.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#if defined(__x86_64__)
#include <immintrin.h>
#endif

/* ------------------------------------------------------------------------ */
/* GF(2^8) with x^8+x^4+x^3+x^2+1 (0x11D), generator 2.                       */
/* ISA-L ships these as literal arrays (gff_base / gflog_base); generating    */
/* them from the generator gives the same field.                             */
/* ------------------------------------------------------------------------ */
static unsigned char g_exp[256];
static unsigned char g_log[256];
static pthread_once_t g_once = PTHREAD_ONCE_INIT;

static void build_field(void)
{
    unsigned v = 1;
    for (int i = 0; i < 255; i++) {
        g_exp[i] = (unsigned char)v;
        g_log[v] = (unsigned char)i;
        v <<= 1;
        if (v & 0x100u)
            v ^= 0x11Du;
    }
    g_exp[255] = g_exp[0]; /* ISA-L's table repeats 0x01 at index 255 */
    g_log[0] = 0;          /* log(0) is undefined; ISA-L stores 0 there  */
}

const unsigned char* oracle_gf_exp_table(void) { pthread_once(&g_once, build_field); return g_exp; }
const unsigned char* oracle_gf_log_table(void) { pthread_once(&g_once, build_field); return g_log; }

/* ISA-L gf_mul (ec_base.c): zero if either operand is zero, else antilog of
 * the log sum reduced mod 255.  Used by ELECT at EC/erasure_coder.c:274. */
unsigned char oracle_gf_mul(unsigned char a, unsigned char b)
{
    pthread_once(&g_once, build_field);
    if (a == 0 || b == 0)
        return 0;
    int s = g_log[a] + g_log[b];
    if (s > 254)
        s -= 255;
    return g_exp[s];
}

/* ISA-L gf_inv: inverse via exp[255 - log a]; gf_inv(0) = 0. */
unsigned char oracle_gf_inv(unsigned char a)
{
    pthread_once(&g_once, build_field);
    if (a == 0)
        return 0;
    return g_exp[255 - g_log[a]];
}

/* ISA-L gf_gen_cauchy1_matrix(a, m, k): m x k, identity on top, then
 * a[i][j] = 1/(i XOR j) for k <= i < m.  ELECT: EC/erasure_coder.c:43 calls it
 * with m = k + parity units. */
void oracle_gf_gen_cauchy1_matrix(unsigned char* a, int m, int k)
{
    memset(a, 0, (size_t)m * (size_t)k);
    for (int i = 0; i < k; i++)
        a[i * k + i] = 1;
    for (int i = k; i < m; i++)
        for (int j = 0; j < k; j++)
            a[i * k + j] = oracle_gf_inv((unsigned char)(i ^ j));
}

/* ISA-L gf_vect_mul_init: 32 bytes per coefficient c,
 * [c*x for x in 0..15] then [c*(x<<4) for x in 0..15]. */
void oracle_gf_vect_mul_init(unsigned char c, unsigned char* tbl32)
{
    for (int x = 0; x < 16; x++) {
        tbl32[x] = oracle_gf_mul(c, (unsigned char)x);
        tbl32[16 + x] = oracle_gf_mul(c, (unsigned char)(x << 4));
    }
}

/* ISA-L ec_init_tables(k, rows, a, g_tbls): row-major over (row, column), 32 B
 * each.  ELECT: EC/erasure_coder.c:57-59 (encode), :192-193 (decode). */
void oracle_ec_init_tables(int k, int rows, const unsigned char* a, unsigned char* g_tbls)
{
    for (int r = 0; r < rows; r++)
        for (int j = 0; j < k; j++)
            oracle_gf_vect_mul_init(a[r * k + j], g_tbls + 32 * (r * k + j));
}

/* ISA-L ec_encode_data_base: dest[l][i] = XOR_j gf_mul(src[j][i], v[32*(l*srcs+j)+1]).
 * The output is overwritten, not accumulated.  ELECT: EC/erasure_coder.c:90, :221. */
void oracle_ec_encode_data(int len, int srcs, int dests, const unsigned char* g_tbls,
                           unsigned char* const* src, unsigned char* const* dest)
{
    for (int l = 0; l < dests; l++) {
        for (int i = 0; i < len; i++) {
            unsigned char s = 0;
            for (int j = 0; j < srcs; j++)
                s ^= oracle_gf_mul(src[j][i], g_tbls[32 * (l * srcs + j) + 1]);
            dest[l][i] = s;
        }
    }
}

/* ISA-L ec_encode_data_update_base: dest[l][i] ^= gf_mul(data[i], coef(l, vec_i)).
 * ELECT: EC/erasure_coder.c:128. */
void oracle_ec_encode_data_update(int len, int k, int rows, int vec_i,
                                  const unsigned char* g_tbls, const unsigned char* data,
                                  unsigned char* const* dest)
{
    for (int l = 0; l < rows; l++) {
        unsigned char c = g_tbls[32 * (l * k + vec_i) + 1];
        for (int i = 0; i < len; i++)
            dest[l][i] ^= oracle_gf_mul(data[i], c);
    }
}

/* ISA-L gf_invert_matrix: Gauss-Jordan in place on in_mat, out_mat starts as
 * identity.  A zero pivot swaps in the first lower row with a non-zero entry
 * in that column; none found -> return -1 with out_mat left partially reduced
 * (ELECT ignores this at EC/erasure_coder.c:257-258 and uses out_mat as is). */
int oracle_gf_invert_matrix(unsigned char* in_mat, unsigned char* out_mat, int n)
{
    memset(out_mat, 0, (size_t)n * (size_t)n);
    for (int i = 0; i < n; i++)
        out_mat[i * n + i] = 1;

    for (int i = 0; i < n; i++) {
        if (in_mat[i * n + i] == 0) {
            int j = i + 1;
            while (j < n && in_mat[j * n + i] == 0)
                j++;
            if (j == n)
                return -1;
            for (int c = 0; c < n; c++) {
                unsigned char t = in_mat[i * n + c];
                in_mat[i * n + c] = in_mat[j * n + c];
                in_mat[j * n + c] = t;
                t = out_mat[i * n + c];
                out_mat[i * n + c] = out_mat[j * n + c];
                out_mat[j * n + c] = t;
            }
        }
        unsigned char piv = oracle_gf_inv(in_mat[i * n + i]);
        for (int c = 0; c < n; c++) {
            in_mat[i * n + c] = oracle_gf_mul(in_mat[i * n + c], piv);
            out_mat[i * n + c] = oracle_gf_mul(out_mat[i * n + c], piv);
        }
        for (int r = 0; r < n; r++) {
            if (r == i)
                continue;
            unsigned char f = in_mat[r * n + i];
            for (int c = 0; c < n; c++) {
                out_mat[r * n + c] ^= oracle_gf_mul(f, out_mat[i * n + c]);
                in_mat[r * n + c] ^= oracle_gf_mul(f, in_mat[i * n + c]);
            }
        }
    }
    return 0;
}

/* ------------------------------------------------------------------------ */
/* ELECT's coder (EC/erasure_coder.c)                                         */
/* ------------------------------------------------------------------------ */

/* initEncoder, EC/erasure_coder.c:49-64: Cauchy matrix, then tables for the
 * parity rows only (&encodeMatrix[k*k]). */
int oracle_encoder_init(oracle_encoder* enc, int k, int m)
{
    if (k < 1 || m < 1 || k > ORACLE_KMAX || k + m > ORACLE_MMAX)
        return -1;
    memset(enc, 0, sizeof(*enc));
    enc->k = k;
    enc->m = m;
    oracle_gf_gen_cauchy1_matrix(enc->encode_matrix, k + m, k);
    oracle_ec_init_tables(k, m, enc->encode_matrix + k * k, enc->gftbls);
    return 0;
}

/* encode, EC/erasure_coder.c:74-98 (the memset at :86-88 is redundant: the
 * dot product overwrites every output byte). */
int oracle_encode(const oracle_encoder* enc, unsigned char* const* data,
                  unsigned char* const* parity, int len)
{
    oracle_ec_encode_data(len, enc->k, enc->m, enc->gftbls, data, parity);
    return 0;
}

/* encodeUpdate, EC/erasure_coder.c:100-142: inputs are [old, new, P0..Pm-1];
 * newP[r] = P[r] ^ coef(r, target) * (old ^ new). */
int oracle_encode_update(const oracle_encoder* enc, unsigned char* const* old_new_parity,
                         int target, unsigned char* const* new_parity, int len)
{
    int m = enc->m;
    unsigned char* x = (unsigned char*)malloc(len > 0 ? (size_t)len : 1);
    if (!x)
        return -1;
    for (int i = 0; i < len; i++)
        x[i] = old_new_parity[0][i] ^ old_new_parity[1][i];
    for (int r = 0; r < m; r++)
        if (new_parity[r] != old_new_parity[2 + r])
            memcpy(new_parity[r], old_new_parity[2 + r], (size_t)len);
    oracle_ec_encode_data_update(len, enc->k, m, target, enc->gftbls, x, new_parity);
    free(x);
    return 0;
}

/* processErasures + generateDecodeMatrix, EC/erasure_coder.c:161-200, 241-284. */
int oracle_decode_matrix(int k, int m, const unsigned char* encode_matrix,
                         const int* decode_indexes, const int* erased, int num_erased,
                         int strict, unsigned char* decode_matrix)
{
    unsigned char tmp[ORACLE_MMAX * ORACLE_KMAX];
    unsigned char inv[ORACLE_MMAX * ORACLE_KMAX];
    (void)m;
    memset(decode_matrix, 0, (size_t)num_erased * (size_t)k);

    /* b = rows of the encode matrix for the k survivors, in input order (:248-254) */
    for (int i = 0; i < k; i++)
        memcpy(tmp + i * k, encode_matrix + decode_indexes[i] * k, (size_t)k);
    int rc = oracle_gf_invert_matrix(tmp, inv, k);
    if (rc != 0 && strict)
        return -1;

    /* numErasedDataUnits counts erased DATA shards (:177-182); the reference's
     * two row loops run only over that many leading entries (:261, :269). */
    int rows = num_erased;
    if (!strict) {
        rows = 0;
        for (int i = 0; i < num_erased; i++)
            if (erased[i] < k)
                rows++;
    }
    for (int r = 0; r < rows; r++) {
        int e = erased[r];
        if (e < k) {
            memcpy(decode_matrix + r * k, inv + e * k, (size_t)k);
        } else {
            for (int i = 0; i < k; i++) {
                unsigned char s = 0;
                for (int j = 0; j < k; j++)
                    s ^= oracle_gf_mul(inv[j * k + i], encode_matrix[e * k + j]);
                decode_matrix[r * k + i] = s;
            }
        }
    }
    return rc;
}

/* decode, EC/erasure_coder.c:202-226: init tables for numErased rows (the
 * zero rows included) and run the dot product over the k survivors. */
int oracle_decode(int k, int m, unsigned char* const* inputs, const int* decode_indexes,
                  const int* erased, int num_erased, unsigned char* const* outputs,
                  int len, int strict)
{
    unsigned char em[ORACLE_MMAX * ORACLE_KMAX];
    unsigned char dm[ORACLE_MMAX * ORACLE_KMAX];
    unsigned char tb[ORACLE_MMAX * ORACLE_KMAX * 32];
    oracle_gf_gen_cauchy1_matrix(em, k + m, k);
    int rc = oracle_decode_matrix(k, m, em, decode_indexes, erased, num_erased, strict, dm);
    if (rc != 0 && strict)
        return rc;
    oracle_ec_init_tables(k, num_erased, dm, tb);
    oracle_ec_encode_data(len, k, num_erased, tb, inputs, outputs);
    return rc;
}

/* ------------------------------------------------------------------------ */
/* SIMD restatement (CPU baseline): ISA-L's gf_Nvect_dot_prod algorithm.      */
/* Each 32-byte table splits a byte into nibbles; a byte shuffle looks up    */
/* c*lo and c*(hi<<4), XOR gives c*x.  The GFNI form multiplies by an 8x8    */
/* bit matrix per coefficient.                                               */
/* ------------------------------------------------------------------------ */
#define ORACLE_MAX_ROWS 16

static void encode_scalar_span(size_t len, int k, int rows, const unsigned char* g_tbls,
                               unsigned char* const* src, unsigned char* const* dest)
{
    /* nibble tables, scalar: same products as the log/antilog form */
    for (int r = 0; r < rows; r++) {
        for (size_t i = 0; i < len; i++) {
            unsigned char s = 0;
            for (int j = 0; j < k; j++) {
                const unsigned char* t = g_tbls + 32 * (r * k + j);
                unsigned char x = src[j][i];
                s ^= (unsigned char)(t[x & 15] ^ t[16 + (x >> 4)]);
            }
            dest[r][i] = s;
        }
    }
}

#if defined(__x86_64__)
__attribute__((target("avx2"))) static void encode_avx2_span(size_t len, int k, int rows,
                                                              const unsigned char* g_tbls,
                                                              unsigned char* const* src,
                                                              unsigned char* const* dest)
{
    const __m256i mask = _mm256_set1_epi8(0x0f);
    size_t i = 0;
    for (int r0 = 0; r0 < rows; r0 += 4) {
        int nr = rows - r0 < 4 ? rows - r0 : 4;
        for (i = 0; i + 32 <= len; i += 32) {
            __m256i acc[4] = {_mm256_setzero_si256(), _mm256_setzero_si256(),
                              _mm256_setzero_si256(), _mm256_setzero_si256()};
            for (int j = 0; j < k; j++) {
                __m256i x = _mm256_loadu_si256((const __m256i*)(src[j] + i));
                __m256i lo = _mm256_and_si256(x, mask);
                __m256i hi = _mm256_and_si256(_mm256_srli_epi64(x, 4), mask);
                for (int q = 0; q < nr; q++) {
                    const unsigned char* t = g_tbls + 32 * ((r0 + q) * k + j);
                    __m256i tl = _mm256_broadcastsi128_si256(_mm_loadu_si128((const __m128i*)t));
                    __m256i th = _mm256_broadcastsi128_si256(_mm_loadu_si128((const __m128i*)(t + 16)));
                    acc[q] = _mm256_xor_si256(acc[q], _mm256_xor_si256(_mm256_shuffle_epi8(tl, lo),
                                                                       _mm256_shuffle_epi8(th, hi)));
                }
            }
            for (int q = 0; q < nr; q++)
                _mm256_storeu_si256((__m256i*)(dest[r0 + q] + i), acc[q]);
        }
    }
    if (i < len) {
        unsigned char* s2[ORACLE_MAX_ROWS];
        unsigned char* d2[ORACLE_MAX_ROWS];
        for (int j = 0; j < k; j++) s2[j] = src[j] + i;
        for (int r = 0; r < rows; r++) d2[r] = dest[r] + i;
        encode_scalar_span(len - i, k, rows, g_tbls, s2, d2);
    }
}

__attribute__((target("avx512f,avx512bw"))) static void encode_avx512_span(
    size_t len, int k, int rows, const unsigned char* g_tbls, unsigned char* const* src,
    unsigned char* const* dest)
{
    const __m512i mask = _mm512_set1_epi8(0x0f);
    size_t i = 0;
    for (int r0 = 0; r0 < rows; r0 += 4) {
        int nr = rows - r0 < 4 ? rows - r0 : 4;
        for (i = 0; i + 64 <= len; i += 64) {
            __m512i acc[4] = {_mm512_setzero_si512(), _mm512_setzero_si512(),
                              _mm512_setzero_si512(), _mm512_setzero_si512()};
            for (int j = 0; j < k; j++) {
                __m512i x = _mm512_loadu_si512((const void*)(src[j] + i));
                __m512i lo = _mm512_and_si512(x, mask);
                __m512i hi = _mm512_and_si512(_mm512_srli_epi64(x, 4), mask);
                for (int q = 0; q < nr; q++) {
                    const unsigned char* t = g_tbls + 32 * ((r0 + q) * k + j);
                    __m512i tl = _mm512_broadcast_i32x4(_mm_loadu_si128((const __m128i*)t));
                    __m512i th = _mm512_broadcast_i32x4(_mm_loadu_si128((const __m128i*)(t + 16)));
                    acc[q] = _mm512_xor_si512(acc[q], _mm512_xor_si512(_mm512_shuffle_epi8(tl, lo),
                                                                       _mm512_shuffle_epi8(th, hi)));
                }
            }
            for (int q = 0; q < nr; q++)
                _mm512_storeu_si512((void*)(dest[r0 + q] + i), acc[q]);
        }
    }
    if (i < len) {
        unsigned char* s2[ORACLE_MAX_ROWS];
        unsigned char* d2[ORACLE_MAX_ROWS];
        for (int j = 0; j < k; j++) s2[j] = src[j] + i;
        for (int r = 0; r < rows; r++) d2[r] = dest[r] + i;
        encode_scalar_span(len - i, k, rows, g_tbls, s2, d2);
    }
}

/* 8x8 GF(2) matrix for y = c*x under 0x11D, in the operand layout of
 * vgf2p8affineqb: byte (7-i) of the qword holds the input-bit mask that
 * produces output bit i. */
static uint64_t gfni_matrix(unsigned char c)
{
    uint64_t a = 0;
    for (int i = 0; i < 8; i++) {
        unsigned row = 0;
        for (int b = 0; b < 8; b++)
            if (oracle_gf_mul(c, (unsigned char)(1u << b)) & (1u << i))
                row |= 1u << b;
        a |= (uint64_t)row << (8 * (7 - i));
    }
    return a;
}

__attribute__((target("avx512f,avx512bw,gfni"))) static void encode_gfni_span(
    size_t len, int k, int rows, const unsigned char* g_tbls, unsigned char* const* src,
    unsigned char* const* dest)
{
    __m512i mats[ORACLE_MAX_ROWS * ORACLE_MAX_ROWS];
    for (int r = 0; r < rows; r++)
        for (int j = 0; j < k; j++)
            mats[r * k + j] = _mm512_set1_epi64((long long)gfni_matrix(g_tbls[32 * (r * k + j) + 1]));
    size_t i = 0;
    for (int r0 = 0; r0 < rows; r0 += 4) {
        int nr = rows - r0 < 4 ? rows - r0 : 4;
        for (i = 0; i + 64 <= len; i += 64) {
            __m512i acc[4] = {_mm512_setzero_si512(), _mm512_setzero_si512(),
                              _mm512_setzero_si512(), _mm512_setzero_si512()};
            for (int j = 0; j < k; j++) {
                __m512i x = _mm512_loadu_si512((const void*)(src[j] + i));
                for (int q = 0; q < nr; q++)
                    acc[q] = _mm512_xor_si512(acc[q],
                                              _mm512_gf2p8affine_epi64_epi8(x, mats[(r0 + q) * k + j], 0));
            }
            for (int q = 0; q < nr; q++)
                _mm512_storeu_si512((void*)(dest[r0 + q] + i), acc[q]);
        }
    }
    if (i < len) {
        unsigned char* s2[ORACLE_MAX_ROWS];
        unsigned char* d2[ORACLE_MAX_ROWS];
        for (int j = 0; j < k; j++) s2[j] = src[j] + i;
        for (int r = 0; r < rows; r++) d2[r] = dest[r] + i;
        encode_scalar_span(len - i, k, rows, g_tbls, s2, d2);
    }
}
#endif

int oracle_simd_best(void)
{
#if defined(__x86_64__)
    __builtin_cpu_init();
    if (__builtin_cpu_supports("avx512bw") && __builtin_cpu_supports("gfni"))
        return ORACLE_SIMD_GFNI;
    if (__builtin_cpu_supports("avx512bw"))
        return ORACLE_SIMD_AVX512;
    if (__builtin_cpu_supports("avx2"))
        return ORACLE_SIMD_AVX2;
#endif
    return ORACLE_SIMD_SCALAR;
}

const char* oracle_simd_name(int level)
{
    switch (level) {
    case ORACLE_SIMD_AVX2: return "avx2-pshufb";
    case ORACLE_SIMD_AVX512: return "avx512bw-pshufb";
    case ORACLE_SIMD_GFNI: return "avx512-gfni";
    default: return "scalar";
    }
}

void oracle_ec_encode_data_simd(int level, size_t len, int k, int rows,
                                const unsigned char* g_tbls, unsigned char* const* src,
                                unsigned char* const* dest)
{
    if (rows > ORACLE_MAX_ROWS || k > ORACLE_MAX_ROWS)
        return;
#if defined(__x86_64__)
    int best = oracle_simd_best();
    if (level > best)
        level = best;
    switch (level) {
    case ORACLE_SIMD_GFNI: encode_gfni_span(len, k, rows, g_tbls, src, dest); return;
    case ORACLE_SIMD_AVX512: encode_avx512_span(len, k, rows, g_tbls, src, dest); return;
    case ORACLE_SIMD_AVX2: encode_avx2_span(len, k, rows, g_tbls, src, dest); return;
    default: break;
    }
#else
    (void)level;
#endif
    encode_scalar_span(len, k, rows, g_tbls, src, dest);
}

/* ------------------------------------------------------------------------ */
/* Threaded batch driver                                                      */
/* ------------------------------------------------------------------------ */
typedef struct batch_job {
    int level, rows, k;
    const unsigned char* tbls;
    size_t len, s0, s1;
    const unsigned char* src;
    size_t src_stripe;
    const int64_t* src_col_off;
    unsigned char* dst;
    size_t dst_stripe;
    const int64_t* dst_row_off;
} batch_job;

static void* batch_worker(void* arg)
{
    batch_job* jb = (batch_job*)arg;
    unsigned char* s[ORACLE_MAX_ROWS];
    unsigned char* d[ORACLE_MAX_ROWS];
    for (size_t st = jb->s0; st < jb->s1; st++) {
        for (int j = 0; j < jb->k; j++)
            s[j] = (unsigned char*)jb->src + st * jb->src_stripe + jb->src_col_off[j];
        for (int r = 0; r < jb->rows; r++)
            d[r] = jb->dst + st * jb->dst_stripe + jb->dst_row_off[r];
        oracle_ec_encode_data_simd(jb->level, jb->len, jb->k, jb->rows, jb->tbls, s, d);
    }
    return NULL;
}

static double now_s(void)
{
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

double oracle_batch_apply(int level, int threads, const unsigned char* coef, int rows, int k,
                          size_t len, size_t stripes,
                          const unsigned char* src, size_t src_stripe, const int64_t* src_col_off,
                          unsigned char* dst, size_t dst_stripe, const int64_t* dst_row_off)
{
    if (rows < 1 || k < 1 || rows > ORACLE_MAX_ROWS || k > ORACLE_MAX_ROWS)
        return -1.0;
    unsigned char tbls[ORACLE_MAX_ROWS * ORACLE_MAX_ROWS * 32];
    oracle_ec_init_tables(k, rows, coef, tbls);
    if (threads < 1)
        threads = 1;
    if ((size_t)threads > stripes)
        threads = stripes ? (int)stripes : 1;
    pthread_t* tid = (pthread_t*)calloc((size_t)threads, sizeof(pthread_t));
    batch_job* jobs = (batch_job*)calloc((size_t)threads, sizeof(batch_job));
    char* started = (char*)calloc((size_t)threads, 1);
    if (!tid || !jobs || !started) {
        free(tid);
        free(jobs);
        free(started);
        return -1.0;
    }
    double t0 = now_s();
    for (int t = 0; t < threads; t++) {
        batch_job* jb = &jobs[t];
        jb->level = level; jb->rows = rows; jb->k = k; jb->tbls = tbls; jb->len = len;
        jb->s0 = stripes * (size_t)t / (size_t)threads;
        jb->s1 = stripes * (size_t)(t + 1) / (size_t)threads;
        jb->src = src; jb->src_stripe = src_stripe; jb->src_col_off = src_col_off;
        jb->dst = dst; jb->dst_stripe = dst_stripe; jb->dst_row_off = dst_row_off;
        /* a thread that cannot be created (task limits) runs its share inline */
        if (t + 1 < threads) {
            started[t] = pthread_create(&tid[t], NULL, batch_worker, jb) == 0;
            if (!started[t])
                batch_worker(jb);
        }
    }
    batch_worker(&jobs[threads - 1]);
    for (int t = 0; t + 1 < threads; t++)
        if (started[t])
            pthread_join(tid[t], NULL);
    double t1 = now_s();
    free(tid);
    free(jobs);
    free(started);
    return t1 - t0;
}

/* splitmix64, one 64-bit word per 8 bytes, little-endian. */
void oracle_fill_splitmix(uint64_t seed, unsigned char* buf, size_t len)
{
    uint64_t x = seed;
    for (size_t i = 0; i < len; i += 8) {
        x += 0x9E3779B97F4A7C15ull;
        uint64_t z = x;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        z ^= z >> 31;
        for (int b = 0; b < 8 && i + (size_t)b < len; b++)
            buf[i + (size_t)b] = (unsigned char)(z >> (8 * b));
    }
}

/* JDK ByteBuffer.hashCode() loop (see ec_oracle.h); unsigned arithmetic is the
 * int32 wrap-around Java defines. */
int32_t oracle_java_bytebuffer_hashcode(const unsigned char* b, size_t n)
{
    uint32_t h = 1;
    for (size_t i = n; i-- > 0;) h = 31u * h + (uint32_t)(int32_t)(signed char)b[i];
    return (int32_t)h;
}
