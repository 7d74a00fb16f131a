/*
 * libec_jni.c — drop-in replacement for ELECT's JNI library libec.so.
 *
 * Exports the seven native methods ELECT's Java binds
 * (JEC/NativeRSEncoder.java:97-105, JEC/NativeRSDecoder.java:81-87; the
 * reference implementations are EC/NativeRSEncoder.c:31-95 and
 * EC/NativeRSDecoder.c:32-82) and forwards them to the MI355X C ABI
 * (include/elect_ec.h).  Built only where a JDK provides <jni.h>; see
 * INTEGRATION.md for the build line.  No Java code changes: ELECT keeps calling
 * System.loadLibrary("ec") (JEC/NativeRSEncoder.java:37).  Three optional
 * methods (encodeExImpl, encodeUpdateExImpl, decodeExImpl) expose the fused
 * coding-node steps to a Java that declares them, and two more
 * (allocateDirectImpl, freeDirectImpl) page-locked coding buffers.
 *
 * Differences from the reference glue, all on error paths:
 *  - every THROW returns (EC/NativeRSDecoder.c:50-52 and EC/jni_common.c:70-73,
 *    95-97 fall through after throwing), and no JNI call but the exception-safe
 *    ones runs while an exception is pending (ExceptionCheck first);
 *  - int arrays are released (EC/jni_common.c:75, 99 and EC/NativeRSDecoder.c:59-62 leak);
 *  - a negative engine status becomes a Java exception instead of being ignored;
 *  - a negative dataLen is an IllegalArgumentException (the reference memsets a
 *    negative size: EC/erasure_coder.c:86-88).
 * Standard output is libec.so's:
 *  - decodeImpl prints its three progress lines on every call, verbose or not
 *    (EC/NativeRSDecoder.c:57, 65, 68; ELECT_EC_JNI_QUIET=1 silences them);
 *  - with allowVerboseDump() true (read on every call, EC/jni_common.c:44-57),
 *    decode also prints the decoder block in EC/dump.c's format (dumpDecoder,
 *    :75-104: erased and decode indexes, encode / invert / decode matrices),
 *    after the third line, as processErasures does (EC/erasure_coder.c:195-197);
 *  - encode and encodeUpdate print nothing: the reference's only dumpEncoder
 *    call sits in initEncoder right after initCoder zeroes verbose
 *    (EC/erasure_coder.c:27, 61-63), so it never runs.
 *
 * JEC/ = src/elect/src/java/org/apache/cassandra/io/erasurecode
 * EC/  = src/elect/src/native/src/org/apache/cassandra/io/erasurecode
 */
#include <jni.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../../include/elect_ec.h"

#define EC_MAX ELECT_EC_MAX_UNITS

static void throw_java(JNIEnv* env, const char* cls, const char* msg)
{
    jclass c = (*env)->FindClass(env, cls);
    if (c != NULL)
        (*env)->ThrowNew(env, c, msg);
}

/* Map a C ABI status to the exception Java callers already handle. */
static int raise_status(JNIEnv* env, int status, const char* what)
{
    char msg[160];
    if (status >= 0)
        return 0;
    snprintf(msg, sizeof msg, "%s: %s (%d)", what, elect_ec_strerror(status), status);
    if (status == ELECT_EC_EINVAL || status == ELECT_EC_ESINGULAR)
        throw_java(env, "java/lang/IllegalArgumentException", msg);
    else
        throw_java(env, "java/io/IOException", msg);
    return 1;
}

static jfieldID coder_field(JNIEnv* env, jobject thiz)
{
    jclass clazz = (*env)->GetObjectClass(env, thiz);
    jfieldID fid = (*env)->GetFieldID(env, clazz, "nativeCoder", "J");
    if (fid == NULL) {  /* GetFieldID left NoSuchFieldError pending; report it as the reference does */
        (*env)->ExceptionClear(env);
        throw_java(env, "java/lang/UnsatisfiedLinkError", "Field nativeCoder not found");
    }
    return fid;
}

/* allowVerboseDump() (EC/jni_common.c:44-50): 1 / 0, or -1 when the call threw
 * (the exception stays pending for the caller to return with). */
static int verbose(JNIEnv* env, jobject thiz)
{
    jclass clazz = (*env)->GetObjectClass(env, thiz);
    jmethodID mid = (*env)->GetMethodID(env, clazz, "allowVerboseDump", "()Z");
    if (mid == NULL) {
        (*env)->ExceptionClear(env);
        return 0;
    }
    jboolean v = (*env)->CallBooleanMethod(env, thiz, mid);
    if ((*env)->ExceptionCheck(env))
        return -1;
    return v == JNI_TRUE;
}

/* getCoder, EC/jni_common.c:35-60.  NULL with an exception pending when the
 * field is missing; NULL with none when the coder was released. */
static elect_ec_coder* get_coder(JNIEnv* env, jobject thiz)
{
    jfieldID fid = coder_field(env, thiz);
    if (fid == NULL)
        return NULL;
    return (elect_ec_coder*)(intptr_t)(*env)->GetLongField(env, thiz, fid);
}

/* The coder of a coding call, or NULL after raising: closed coder -> IOException
 * (EC/NativeRSEncoder.c:49-51); a pending exception is left as it is. */
static elect_ec_coder* coder_for_call(JNIEnv* env, jobject thiz, const char* closed_msg)
{
    elect_ec_coder* c = get_coder(env, thiz);
    if (c == NULL && !(*env)->ExceptionCheck(env))
        throw_java(env, "java/io/IOException", closed_msg);
    return c;
}

static int bad_length(JNIEnv* env, jint dataLen)
{
    if (dataLen >= 0)
        return 0;
    throw_java(env, "java/lang/IllegalArgumentException", "negative dataLen");
    return 1;
}

/* ---- verbose dumps, in EC/dump.c's format ---- */
/* dumpCodingMatrix (EC/dump.c:46-59): n2 rows of n1 entries, decimal */
static void dump_coding_matrix(const unsigned char* buf, int n1, int n2)
{
    for (int i = 0; i < n2; i++) {
        for (int j = 0; j < n1; j++)
            printf(" %d", buf[j + i * n1]);
        printf("\n");
    }
    printf("\n");
}

/* dumpDecoder (EC/dump.c:75-104).  The reference's invert and decode matrices
 * live in zeroed MMAX x KMAX arrays (clearDecoder, EC/erasure_coder.c:229-238),
 * so rows past k (invert) and past numErased (decode) print as zeros. */
static void dump_decoder(const elect_ec_coder* c, const int* dec, const int* era, int n_era, int mode)
{
    unsigned char em[ELECT_EC_MAX_UNITS * ELECT_EC_MAX_DATA_UNITS] = {0};
    unsigned char inv[ELECT_EC_MAX_UNITS * ELECT_EC_MAX_DATA_UNITS] = {0};
    unsigned char dm[ELECT_EC_MAX_UNITS * ELECT_EC_MAX_DATA_UNITS] = {0};
    int k = elect_ec_coder_num_data_units(c), n = k + elect_ec_coder_num_parity_units(c);
    if (elect_ec_coder_decode_matrix(c, dec, era, n_era, mode, dm) < 0 || elect_ec_coder_invert_matrix(c, dec, inv) < 0)
        return;  /* an invalid call: the decode itself raises */
    elect_ec_coder_encode_matrix(c, em, sizeof em);
    printf("Recovering (numAllUnits = %d, numDataUnits = %d, numErased = %d)\n", n, k, n_era);
    printf(" - ErasedIndexes = ");
    for (int j = 0; j < n_era; j++)
        printf(" %d", era[j]);
    printf("       - DecodeIndex = ");
    for (int i = 0; i < k; i++)
        printf(" %d", dec[i]);
    printf("\n\nEncodeMatrix:\n");
    dump_coding_matrix(em, k, n);
    printf("InvertMatrix:\n");
    dump_coding_matrix(inv, k, n);
    printf("DecodeMatrix:\n");
    dump_coding_matrix(dm, k, n);
    fflush(stdout);
}

/* setCoder, EC/jni_common.c:24-33 */
static void set_coder(JNIEnv* env, jobject thiz, elect_ec_coder* c)
{
    jfieldID fid = coder_field(env, thiz);
    if (fid != NULL)
        (*env)->SetLongField(env, thiz, fid, (jlong)(intptr_t)c);
}

/* getInputs/getOutputs, EC/jni_common.c:62-108: count check, then direct
 * buffer address + offset per element.  Returns 0 on success. */
static int buffers(JNIEnv* env, jobjectArray arr, jintArray offsets, int num, unsigned char** out,
                   const char* what)
{
    if ((*env)->GetArrayLength(env, arr) != num || num > 2 + EC_MAX) {
        throw_java(env, "java/lang/InternalError", what);
        return 1;
    }
    jint* offs = (*env)->GetIntArrayElements(env, offsets, NULL);
    if (offs == NULL)
        return 1;
    for (int i = 0; i < num; i++) {
        jobject bb = (*env)->GetObjectArrayElement(env, arr, i);
        unsigned char* base = bb ? (unsigned char*)(*env)->GetDirectBufferAddress(env, bb) : NULL;
        out[i] = base ? base + offs[i] : NULL;
        if (bb)
            (*env)->DeleteLocalRef(env, bb);
        if (out[i] == NULL) {
            (*env)->ReleaseIntArrayElements(env, offsets, offs, JNI_ABORT);
            throw_java(env, "java/lang/InternalError", what);
            return 1;
        }
    }
    (*env)->ReleaseIntArrayElements(env, offsets, offs, JNI_ABORT);
    return 0;
}

/* initImpl (EC/NativeRSEncoder.c:31-41, EC/NativeRSDecoder.c:32-42): the field
 * is resolved first, so a class without it leaks no coder. */
static void init_coder(JNIEnv* env, jobject thiz, jint k, jint m)
{
    jfieldID fid = coder_field(env, thiz);
    elect_ec_coder* c = NULL;
    if (fid == NULL || raise_status(env, elect_ec_coder_create(k, m, &c), "initImpl"))
        return;
    (*env)->SetLongField(env, thiz, fid, (jlong)(intptr_t)c);
}

JNIEXPORT void JNICALL
Java_org_apache_cassandra_io_erasurecode_NativeRSEncoder_initImpl(JNIEnv* env, jobject thiz,
                                                                  jint numDataUnits, jint numParityUnits)
{
    init_coder(env, thiz, numDataUnits, numParityUnits);
}

JNIEXPORT void JNICALL
Java_org_apache_cassandra_io_erasurecode_NativeRSEncoder_encodeImpl(JNIEnv* env, jobject thiz,
                                                                    jobjectArray inputs, jintArray inputOffsets,
                                                                    jint dataLen, jobjectArray outputs,
                                                                    jintArray outputOffsets)
{
    unsigned char* in[2 + EC_MAX];
    unsigned char* out[2 + EC_MAX];
    elect_ec_coder* c = coder_for_call(env, thiz, "NativeRSRawEncoder closed");
    if (c == NULL || verbose(env, thiz) < 0 || bad_length(env, dataLen))  /* (getCoder's call) */
        return;
    int k = elect_ec_coder_num_data_units(c), m = elect_ec_coder_num_parity_units(c);
    if (buffers(env, inputs, inputOffsets, k, in, "Invalid inputs") ||
        buffers(env, outputs, outputOffsets, m, out, "Invalid outputs"))
        return;
    raise_status(env, elect_ec_encode(c, (const unsigned char* const*)in, out, (size_t)dataLen), "encode");
}

JNIEXPORT void JNICALL
Java_org_apache_cassandra_io_erasurecode_NativeRSEncoder_encodeUpdateImpl(JNIEnv* env, jobject thiz,
                                                                          jobjectArray inputs,
                                                                          jintArray inputOffsets, jint dataLen,
                                                                          jint targetUpdateDataIndex,
                                                                          jobjectArray outputs,
                                                                          jintArray outputOffsets)
{
    unsigned char* in[2 + EC_MAX];
    unsigned char* out[2 + EC_MAX];
    elect_ec_coder* c = coder_for_call(env, thiz, "NativeRSRawEncoder closed");
    if (c == NULL || verbose(env, thiz) < 0 || bad_length(env, dataLen))  /* (getCoder's call) */
        return;
    int m = elect_ec_coder_num_parity_units(c);
    if (buffers(env, inputs, inputOffsets, 2 + m, in, "Invalid inputs") ||
        buffers(env, outputs, outputOffsets, m, out, "Invalid outputs"))
        return;
    raise_status(env,
                 elect_ec_encode_update(c, (const unsigned char* const*)in, targetUpdateDataIndex, out,
                                        (size_t)dataLen),
                 "encodeUpdate");
}

/* ---- optional: ELECT's coding-node steps fused (not bound by the unchanged Java) ----
 * A maintainer who adds the matching `private native` methods to NativeRSEncoder
 *  gets ECMessageVerbHandler's zero fill + encode + parity
 * hashCode (:283-329) and ECParityUpdateVerbHandler's zero fill + encodeUpdate +
 * new-parity hashCode (:634-699) in one call each.  contentLengths (k entries for
 * encode, 2 for [old, new]) and parityHashes (>= m entries, written) may be null. */
static int content_lengths(JNIEnv* env, jintArray arr, int n, size_t* out, const size_t** use)
{
    *use = NULL;
    if (arr == NULL)
        return 0;
    jint v[EC_MAX];
    if ((*env)->GetArrayLength(env, arr) != n || n > EC_MAX) {
        throw_java(env, "java/lang/InternalError", "Invalid content lengths");
        return 1;
    }
    (*env)->GetIntArrayRegion(env, arr, 0, n, v);
    for (int i = 0; i < n; i++) {
        if (v[i] < 0) {
            throw_java(env, "java/lang/IllegalArgumentException", "negative content length");
            return 1;
        }
        out[i] = (size_t)v[i];
    }
    *use = out;
    return 0;
}

static int hash_array(JNIEnv* env, jintArray arr, int m)
{
    if (arr != NULL && (*env)->GetArrayLength(env, arr) < m) {
        throw_java(env, "java/lang/InternalError", "Invalid parity hashes");
        return 1;
    }
    return 0;
}

JNIEXPORT void JNICALL
Java_org_apache_cassandra_io_erasurecode_NativeRSEncoder_encodeExImpl(JNIEnv* env, jobject thiz,
                                                                      jobjectArray inputs, jintArray inputOffsets,
                                                                      jintArray contentLengths, jint dataLen,
                                                                      jobjectArray outputs, jintArray outputOffsets,
                                                                      jintArray parityHashes)
{
    unsigned char* in[2 + EC_MAX];
    unsigned char* out[2 + EC_MAX];
    size_t lens[EC_MAX];
    const size_t* use_lens;
    jint h[EC_MAX];
    elect_ec_coder* c = coder_for_call(env, thiz, "NativeRSRawEncoder closed");
    if (c == NULL || verbose(env, thiz) < 0 || bad_length(env, dataLen))  /* (getCoder's call) */
        return;
    int k = elect_ec_coder_num_data_units(c), m = elect_ec_coder_num_parity_units(c);
    if (buffers(env, inputs, inputOffsets, k, in, "Invalid inputs") ||
        buffers(env, outputs, outputOffsets, m, out, "Invalid outputs") ||
        content_lengths(env, contentLengths, k, lens, &use_lens) || hash_array(env, parityHashes, m))
        return;
    if (raise_status(env,
                     elect_ec_encode_ex(c, (const unsigned char* const*)in, use_lens, out, (size_t)dataLen,
                                        parityHashes ? (int32_t*)h : NULL),
                     "encodeEx"))
        return;
    if (parityHashes != NULL)
        (*env)->SetIntArrayRegion(env, parityHashes, 0, m, h);
}

JNIEXPORT void JNICALL
Java_org_apache_cassandra_io_erasurecode_NativeRSEncoder_encodeUpdateExImpl(
    JNIEnv* env, jobject thiz, jobjectArray inputs, jintArray inputOffsets, jintArray contentLengths, jint dataLen,
    jint targetUpdateDataIndex, jobjectArray outputs, jintArray outputOffsets, jintArray parityHashes)
{
    unsigned char* in[2 + EC_MAX];
    unsigned char* out[2 + EC_MAX];
    size_t lens[EC_MAX];
    const size_t* use_lens;
    jint h[EC_MAX];
    elect_ec_coder* c = coder_for_call(env, thiz, "NativeRSRawEncoder closed");
    if (c == NULL || verbose(env, thiz) < 0 || bad_length(env, dataLen))  /* (getCoder's call) */
        return;
    int m = elect_ec_coder_num_parity_units(c);
    if (buffers(env, inputs, inputOffsets, 2 + m, in, "Invalid inputs") ||
        buffers(env, outputs, outputOffsets, m, out, "Invalid outputs") ||
        content_lengths(env, contentLengths, 2, lens, &use_lens) || hash_array(env, parityHashes, m))
        return;
    if (raise_status(env,
                     elect_ec_encode_update_ex(c, (const unsigned char* const*)in, use_lens, targetUpdateDataIndex,
                                               out, (size_t)dataLen, parityHashes ? (int32_t*)h : NULL),
                     "encodeUpdateEx"))
        return;
    if (parityHashes != NULL)
        (*env)->SetIntArrayRegion(env, parityHashes, 0, m, h);
}

JNIEXPORT void JNICALL
Java_org_apache_cassandra_io_erasurecode_NativeRSEncoder_destroyImpl(JNIEnv* env, jobject thiz)
{
    elect_ec_coder* c = get_coder(env, thiz);
    if (c != NULL) {
        elect_ec_coder_destroy(c);
        set_coder(env, thiz, NULL);
    }
}

/* Optional: page-locked direct buffers for ELECT's coding buffers
 * ("Page-locked coding buffers").  Declared in NativeRSEncoder.java as
 *   static native ByteBuffer allocateDirectImpl(int capacity);
 *   static native void freeDirectImpl(ByteBuffer buffer);
 * ELECT's ByteBuffer.allocateDirect(codeLength) calls for its data and parity units
 * (ECMessageVerbHandler.java:298, 314) become allocateDirectImpl; a call whose units
 * all live in such buffers is moved by DMA with no staging copies (elect_ec_host_alloc). */
JNIEXPORT jobject JNICALL
Java_org_apache_cassandra_io_erasurecode_NativeRSEncoder_allocateDirectImpl(JNIEnv* env, jclass cls, jint capacity)
{
    void* p = NULL;
    jobject buf;
    (void)cls;
    if (capacity < 0) {
        throw_java(env, "java/lang/IllegalArgumentException", "allocateDirect: negative capacity");
        return NULL;
    }
    if (raise_status(env, elect_ec_host_alloc(capacity > 0 ? (size_t)capacity : 1, &p), "allocateDirect"))
        return NULL;
    buf = (*env)->NewDirectByteBuffer(env, p, (jlong)capacity);
    if (buf == NULL)  /* the JVM has an OutOfMemoryError pending */
        elect_ec_host_free(p);
    return buf;
}

JNIEXPORT void JNICALL
Java_org_apache_cassandra_io_erasurecode_NativeRSEncoder_freeDirectImpl(JNIEnv* env, jclass cls, jobject buffer)
{
    void* p;
    (void)cls;
    if (buffer == NULL)
        return;
    p = (*env)->GetDirectBufferAddress(env, buffer);
    if (p == NULL) {
        throw_java(env, "java/lang/IllegalArgumentException", "freeDirect: not a direct buffer");
        return;
    }
    raise_status(env, elect_ec_host_free(p), "freeDirect");
}

JNIEXPORT void JNICALL
Java_org_apache_cassandra_io_erasurecode_NativeRSDecoder_initImpl(JNIEnv* env, jobject thiz,
                                                                  jint numDataUnits, jint numParityUnits)
{
    init_coder(env, thiz, numDataUnits, numParityUnits);
}

/* ELECT_EC_JNI_QUIET=1 drops decodeImpl's three progress lines (the reference
 * prints them on every decode, EC/NativeRSDecoder.c:57, 65, 68). */
static int quiet(void)
{
    const char* s = getenv("ELECT_EC_JNI_QUIET");
    return s != NULL && strcmp(s, "1") == 0;
}

/* ELECT_EC_DECODE_MODE=strict switches off the compat zero rows for every
 * decoder in the process; the default is bit-exact libec.so. */
static int decode_mode(void)
{
    const char* s = getenv("ELECT_EC_DECODE_MODE");
    return (s != NULL && strcmp(s, "strict") == 0) ? ELECT_EC_DECODE_STRICT : ELECT_EC_DECODE_COMPAT;
}

JNIEXPORT void JNICALL
Java_org_apache_cassandra_io_erasurecode_NativeRSDecoder_decodeImpl(JNIEnv* env, jobject thiz,
                                                                    jobjectArray inputs, jintArray inputOffsets,
                                                                    jint dataLen, jintArray decodeIndexes,
                                                                    jintArray erasedIndexes, jobjectArray outputs,
                                                                    jintArray outputOffsets)
{
    unsigned char* in[2 + EC_MAX];
    unsigned char* out[2 + EC_MAX];
    int dec[EC_MAX], era[EC_MAX];
    elect_ec_coder* c = coder_for_call(env, thiz, "NativeRSRawDecoder closed");
    int v;
    if (c == NULL || (v = verbose(env, thiz)) < 0 || bad_length(env, dataLen))
        return;
    int k = elect_ec_coder_num_data_units(c), m = elect_ec_coder_num_parity_units(c);
    const int say = !quiet();
    if (say)  /* EC/NativeRSDecoder.c:57 */
        printf("NativeRSDecoder_decodeImpl, start to process: data unit = %d, parity unit = %d, data block size = %d\n",
               k, m, (int)dataLen);
    int n_dec = (*env)->GetArrayLength(env, decodeIndexes);
    int n_era = (*env)->GetArrayLength(env, erasedIndexes);
    if (n_dec < k || n_era > EC_MAX) {
        throw_java(env, "java/lang/InternalError", "Invalid decode/erased indexes");
        return;
    }
    (*env)->GetIntArrayRegion(env, decodeIndexes, 0, k, (jint*)dec);
    (*env)->GetIntArrayRegion(env, erasedIndexes, 0, n_era, (jint*)era);
    if (say)  /* :65 */
        printf("NativeRSDecoder_decodeImpl, read data: target recovery data block number = %d, the first recovery "
               "request block ID = %d\n", n_era, n_era > 0 ? era[0] : 0);
    if (buffers(env, inputs, inputOffsets, k, in, "Invalid inputs") ||
        buffers(env, outputs, outputOffsets, n_era, out, "Invalid outputs"))
        return;
    if (say)  /* :68 */
        printf("NativeRSDecoder_decodeImpl, start do decode\n");
    if (v)  /* processErasures' dumpDecoder (EC/erasure_coder.c:195-197) */
        dump_decoder(c, dec, era, n_era, decode_mode());
    else if (say)
        fflush(stdout);
    raise_status(env,
                 elect_ec_decode(c, (const unsigned char* const*)in, dec, era, n_era, out, (size_t)dataLen,
                                 decode_mode()),
                 "decode");
}

/* optional: ECRecovery's degraded-read decode (:128-149) with survivors zero
 * padded past contentLengths (k entries, decodeIndexes order; null = all full)
 * and dataLen possibly just the prefix the caller keeps. */
JNIEXPORT void JNICALL
Java_org_apache_cassandra_io_erasurecode_NativeRSDecoder_decodeExImpl(JNIEnv* env, jobject thiz,
                                                                      jobjectArray inputs, jintArray inputOffsets,
                                                                      jintArray contentLengths, jint dataLen,
                                                                      jintArray decodeIndexes, jintArray erasedIndexes,
                                                                      jobjectArray outputs, jintArray outputOffsets)
{
    unsigned char* in[2 + EC_MAX];
    unsigned char* out[2 + EC_MAX];
    int dec[EC_MAX], era[EC_MAX];
    size_t lens[EC_MAX];
    const size_t* use_lens;
    elect_ec_coder* c = coder_for_call(env, thiz, "NativeRSRawDecoder closed");
    int v;
    if (c == NULL || (v = verbose(env, thiz)) < 0 || bad_length(env, dataLen))
        return;
    int k = elect_ec_coder_num_data_units(c);
    int n_dec = (*env)->GetArrayLength(env, decodeIndexes);
    int n_era = (*env)->GetArrayLength(env, erasedIndexes);
    if (n_dec < k || n_era > EC_MAX) {
        throw_java(env, "java/lang/InternalError", "Invalid decode/erased indexes");
        return;
    }
    (*env)->GetIntArrayRegion(env, decodeIndexes, 0, k, (jint*)dec);
    (*env)->GetIntArrayRegion(env, erasedIndexes, 0, n_era, (jint*)era);
    if (buffers(env, inputs, inputOffsets, k, in, "Invalid inputs") ||
        buffers(env, outputs, outputOffsets, n_era, out, "Invalid outputs") ||
        content_lengths(env, contentLengths, k, lens, &use_lens))
        return;
    if (v)
        dump_decoder(c, dec, era, n_era, decode_mode());
    raise_status(env,
                 elect_ec_decode_ex(c, (const unsigned char* const*)in, use_lens, dec, era, n_era, out,
                                    (size_t)dataLen, decode_mode()),
                 "decodeEx");
}

JNIEXPORT void JNICALL
Java_org_apache_cassandra_io_erasurecode_NativeRSDecoder_destroyImpl(JNIEnv* env, jobject thiz)
{
    elect_ec_coder* c = get_coder(env, thiz);
    if (c != NULL) {
        elect_ec_coder_destroy(c);
        set_coder(env, thiz, NULL);
    }
}
