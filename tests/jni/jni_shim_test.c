/*
 * jni_shim_test.c — a fake JVM that loads the drop-in libec shim the way
 * System.loadLibrary("ec") does (dlopen + dlsym of the seven
 * Java_org_apache_cassandra_io_erasurecode_* names, JEC/NativeRSEncoder.java:97-105,
 * JEC/NativeRSDecoder.java:81-87) and calls them with Java-shaped arguments:
 * ByteBuffer[] arrays, int[] position offsets, a `long nativeCoder` field.
 *
 *   jni_shim_test LIB cpu          error paths; no device needed (exit 0 = pass)
 *   jni_shim_test LIB gpu OUTDIR   ErasureCodeTest.java:31-173 at codeLength 4099
 *                                  through the JNI entry points, buffers at
 *                                  non-zero positions; writes them to OUTDIR for
 *                                  the Python side to compare with
 *                                  tests/golden/erasure_code_test.json
 *
 * The fake JVM also enforces JNI rules the reference glue breaks
 * (EC/jni_common.c:70-75, EC/NativeRSDecoder.c:50-62): no JNI call other than
 * the exception-safe ones while an exception is pending, every
 * Get<Int>ArrayElements released, every local ref from GetObjectArrayElement
 * deleted.  Built against tests/jni/mock/jni.h (test double; see its header).
 */
#include <dlfcn.h>
#include <jni.h>
#include <stdarg.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define ENC_CLS "org/apache/cassandra/io/erasurecode/NativeRSEncoder"
#define DEC_CLS "org/apache/cassandra/io/erasurecode/NativeRSDecoder"

enum { K_CLASS, K_OBJECT, K_DIRECT, K_HEAP, K_OBJARR, K_INTARR };

struct _jobject {
    int kind;
    const char* cls;
    jlong native_coder;
    jboolean verbose;
    int verbose_throws; /* allowVerboseDump() throws */
    unsigned char* addr;
    jobject* elems;
    jint* ints;
    int n;
};

static struct {
    int pending;
    char exc_class[128];
    char exc_msg[256];
    int violations;
    int live_int_elems;
    int local_refs;
} vm;

static int failures;
#define EXPECT(cond)                                                                   \
    do {                                                                               \
        if (!(cond)) {                                                                 \
            fprintf(stderr, "FAIL %s:%d %s\n", __FILE__, __LINE__, #cond);             \
            ++failures;                                                                \
        }                                                                              \
    } while (0)

static void no_pending(const char* fn)
{
    if (vm.pending) {
        fprintf(stderr, "JNI violation: %s called with %s pending\n", fn, vm.exc_class);
        ++vm.violations;
    }
}

static void raise_exc(const char* cls, const char* msg)
{
    if (vm.pending) return;  /* the first exception wins, as in the JVM */
    vm.pending = 1;
    snprintf(vm.exc_class, sizeof vm.exc_class, "%s", cls);
    snprintf(vm.exc_msg, sizeof vm.exc_msg, "%s", msg ? msg : "");
}

static jobject new_obj(int kind, const char* cls)
{
    jobject o = calloc(1, sizeof *o);
    o->kind = kind;
    o->cls = cls;
    return o;
}

/* ---- the JNIEnv functions the shim uses ---------------------------------- */
static jclass m_FindClass(JNIEnv* env, const char* name)
{
    (void)env;
    no_pending("FindClass");
    return new_obj(K_CLASS, strdup(name));
}

static jint m_ThrowNew(JNIEnv* env, jclass c, const char* msg)
{
    (void)env;
    no_pending("ThrowNew");
    raise_exc(c->cls, msg);
    return 0;
}

static void m_ExceptionClear(JNIEnv* env)
{
    (void)env;
    vm.pending = 0;
}

static jclass m_GetObjectClass(JNIEnv* env, jobject o)
{
    (void)env;
    no_pending("GetObjectClass");
    return new_obj(K_CLASS, o->cls);
}

static int is_coder_class(jclass c) { return !strcmp(c->cls, ENC_CLS) || !strcmp(c->cls, DEC_CLS); }

static jfieldID m_GetFieldID(JNIEnv* env, jclass c, const char* name, const char* sig)
{
    (void)env;
    no_pending("GetFieldID");
    if (is_coder_class(c) && !strcmp(name, "nativeCoder") && !strcmp(sig, "J"))
        return (jfieldID)1;
    raise_exc("java/lang/NoSuchFieldError", name);
    return NULL;
}

static jmethodID m_GetMethodID(JNIEnv* env, jclass c, const char* name, const char* sig)
{
    (void)env;
    no_pending("GetMethodID");
    if (is_coder_class(c) && !strcmp(name, "allowVerboseDump") && !strcmp(sig, "()Z"))
        return (jmethodID)2;
    raise_exc("java/lang/NoSuchMethodError", name);
    return NULL;
}

static jboolean m_CallBooleanMethod(JNIEnv* env, jobject o, jmethodID mid, ...)
{
    (void)env;
    no_pending("CallBooleanMethod");
    if (mid == (jmethodID)2 && o->verbose_throws) {
        raise_exc("java/lang/IllegalStateException", "allowVerboseDump threw");
        return JNI_FALSE;
    }
    return mid == (jmethodID)2 ? o->verbose : JNI_FALSE;
}

static jboolean m_ExceptionCheck(JNIEnv* env)
{
    (void)env;  /* exception-safe per the JNI spec */
    return vm.pending ? JNI_TRUE : JNI_FALSE;
}

static jlong m_GetLongField(JNIEnv* env, jobject o, jfieldID f)
{
    (void)env;
    (void)f;
    no_pending("GetLongField");
    return o->native_coder;
}

static void m_SetLongField(JNIEnv* env, jobject o, jfieldID f, jlong v)
{
    (void)env;
    (void)f;
    no_pending("SetLongField");
    o->native_coder = v;
}

static jsize m_GetArrayLength(JNIEnv* env, jarray a)
{
    (void)env;
    no_pending("GetArrayLength");
    return a->n;
}

static jobject m_GetObjectArrayElement(JNIEnv* env, jobjectArray a, jsize i)
{
    (void)env;
    no_pending("GetObjectArrayElement");
    if (i < 0 || i >= a->n) {
        raise_exc("java/lang/ArrayIndexOutOfBoundsException", "");
        return NULL;
    }
    if (a->elems[i]) ++vm.local_refs;
    return a->elems[i];
}

static jint* m_GetIntArrayElements(JNIEnv* env, jintArray a, jboolean* is_copy)
{
    (void)env;
    no_pending("GetIntArrayElements");
    jint* p = malloc(sizeof(jint) * (a->n ? a->n : 1));
    memcpy(p, a->ints, sizeof(jint) * a->n);
    if (is_copy) *is_copy = JNI_TRUE;
    ++vm.live_int_elems;
    return p;
}

static void m_ReleaseIntArrayElements(JNIEnv* env, jintArray a, jint* p, jint mode)
{
    (void)env;  /* exception-safe per the JNI spec */
    if (mode != JNI_ABORT) memcpy(a->ints, p, sizeof(jint) * a->n);
    free(p);
    --vm.live_int_elems;
}

static void m_GetIntArrayRegion(JNIEnv* env, jintArray a, jsize start, jsize len, jint* buf)
{
    (void)env;
    no_pending("GetIntArrayRegion");
    if (start < 0 || len < 0 || start + len > a->n) {
        raise_exc("java/lang/ArrayIndexOutOfBoundsException", "");
        return;
    }
    memcpy(buf, a->ints + start, sizeof(jint) * len);
}

static void m_SetIntArrayRegion(JNIEnv* env, jintArray a, jsize start, jsize len, const jint* buf)
{
    (void)env;
    no_pending("SetIntArrayRegion");
    if (start < 0 || len < 0 || start + len > a->n) {
        raise_exc("java/lang/ArrayIndexOutOfBoundsException", "");
        return;
    }
    memcpy(a->ints + start, buf, sizeof(jint) * len);
}

static void* m_GetDirectBufferAddress(JNIEnv* env, jobject o)
{
    (void)env;
    no_pending("GetDirectBufferAddress");
    return o->kind == K_DIRECT ? o->addr : NULL;
}

static jobject m_NewDirectByteBuffer(JNIEnv* env, void* addr, jlong capacity)
{
    (void)env;
    no_pending("NewDirectByteBuffer");
    jobject o = new_obj(K_DIRECT, "java/nio/DirectByteBuffer");
    o->addr = addr;
    o->n = (int)capacity;
    return o;
}

static void m_DeleteLocalRef(JNIEnv* env, jobject o)
{
    (void)env;  /* exception-safe per the JNI spec */
    if (o) --vm.local_refs;
}

/* The JNI specification's table layout (tests/jni/mock/jni.h pins every slot's
 * index); the slots the shim does not call stay NULL, so calling one crashes. */
static const struct JNINativeInterface_ kEnvTable = {
    .FindClass = m_FindClass,
    .ThrowNew = m_ThrowNew,
    .ExceptionClear = m_ExceptionClear,
    .DeleteLocalRef = m_DeleteLocalRef,
    .GetObjectClass = m_GetObjectClass,
    .GetMethodID = m_GetMethodID,
    .CallBooleanMethod = m_CallBooleanMethod,
    .GetFieldID = m_GetFieldID,
    .GetLongField = m_GetLongField,
    .SetLongField = m_SetLongField,
    .GetArrayLength = m_GetArrayLength,
    .GetObjectArrayElement = m_GetObjectArrayElement,
    .GetIntArrayElements = m_GetIntArrayElements,
    .ReleaseIntArrayElements = m_ReleaseIntArrayElements,
    .GetIntArrayRegion = m_GetIntArrayRegion,
    .SetIntArrayRegion = m_SetIntArrayRegion,
    .ExceptionCheck = m_ExceptionCheck,
    .NewDirectByteBuffer = m_NewDirectByteBuffer,
    .GetDirectBufferAddress = m_GetDirectBufferAddress,
};
static JNIEnv kEnv = &kEnvTable;
static JNIEnv* env = &kEnv;

/* ---- the seven native methods, resolved by name like the JVM does --------- */
typedef void (*init_fn)(JNIEnv*, jobject, jint, jint);
typedef void (*encode_fn)(JNIEnv*, jobject, jobjectArray, jintArray, jint, jobjectArray, jintArray);
typedef void (*update_fn)(JNIEnv*, jobject, jobjectArray, jintArray, jint, jint, jobjectArray, jintArray);
typedef void (*destroy_fn)(JNIEnv*, jobject);
/* optional fused methods: (inputs, offsets, contentLengths, dataLen[, target], outputs, offsets, hashes) */
typedef void (*encode_ex_fn)(JNIEnv*, jobject, jobjectArray, jintArray, jintArray, jint, jobjectArray, jintArray,
                             jintArray);
typedef void (*update_ex_fn)(JNIEnv*, jobject, jobjectArray, jintArray, jintArray, jint, jint, jobjectArray,
                             jintArray, jintArray);
typedef void (*decode_ex_fn)(JNIEnv*, jobject, jobjectArray, jintArray, jintArray, jint, jintArray, jintArray,
                             jobjectArray, jintArray);
typedef void (*decode_fn)(JNIEnv*, jobject, jobjectArray, jintArray, jint, jintArray, jintArray, jobjectArray,
                          jintArray);

static struct {
    init_fn enc_init, dec_init;
    encode_fn encode;
    update_fn update;
    decode_fn decode;
    destroy_fn enc_destroy, dec_destroy;
    encode_ex_fn encode_ex;
    update_ex_fn update_ex;
    decode_ex_fn decode_ex;
    jobject (*alloc_direct)(JNIEnv*, jclass, jint);
    void (*free_direct)(JNIEnv*, jclass, jobject);
    int (*device_count)(int*);
    int (*host_pinned)(const void*, size_t);
} jni;

static void* sym(void* h, const char* name)
{
    void* p = dlsym(h, name);
    if (!p) {
        fprintf(stderr, "missing symbol %s\n", name);
        exit(2);
    }
    return p;
}

#define PFX "Java_org_apache_cassandra_io_erasurecode_"
static void load(const char* lib)
{
    void* h = dlopen(lib, RTLD_NOW | RTLD_LOCAL);
    if (!h) {
        fprintf(stderr, "dlopen %s: %s\n", lib, dlerror());
        exit(2);
    }
    jni.enc_init = (init_fn)sym(h, PFX "NativeRSEncoder_initImpl");
    jni.encode = (encode_fn)sym(h, PFX "NativeRSEncoder_encodeImpl");
    jni.update = (update_fn)sym(h, PFX "NativeRSEncoder_encodeUpdateImpl");
    jni.enc_destroy = (destroy_fn)sym(h, PFX "NativeRSEncoder_destroyImpl");
    jni.dec_init = (init_fn)sym(h, PFX "NativeRSDecoder_initImpl");
    jni.decode = (decode_fn)sym(h, PFX "NativeRSDecoder_decodeImpl");
    jni.dec_destroy = (destroy_fn)sym(h, PFX "NativeRSDecoder_destroyImpl");
    jni.encode_ex = (encode_ex_fn)sym(h, PFX "NativeRSEncoder_encodeExImpl");
    jni.update_ex = (update_ex_fn)sym(h, PFX "NativeRSEncoder_encodeUpdateExImpl");
    jni.decode_ex = (decode_ex_fn)sym(h, PFX "NativeRSDecoder_decodeExImpl");
    jni.alloc_direct = (jobject(*)(JNIEnv*, jclass, jint))sym(h, PFX "NativeRSEncoder_allocateDirectImpl");
    jni.free_direct = (void (*)(JNIEnv*, jclass, jobject))sym(h, PFX "NativeRSEncoder_freeDirectImpl");
    jni.device_count = (int (*)(int*))sym(h, "elect_ec_device_count");
    jni.host_pinned = (int (*)(const void*, size_t))sym(h, "elect_ec_host_pinned");
}

/* ---- Java-side object builders ------------------------------------------- */
static jobject coder_obj(const char* cls) { return new_obj(K_OBJECT, cls); }

static jobject direct_bb(unsigned char* base)
{
    jobject o = new_obj(K_DIRECT, "java/nio/DirectByteBuffer");
    o->addr = base;
    return o;
}

static jobject obj_array(int n, const jobject* e)
{
    jobject a = new_obj(K_OBJARR, "[Ljava/nio/ByteBuffer;");
    a->n = n;
    a->elems = calloc(n ? n : 1, sizeof(jobject));
    if (n) memcpy(a->elems, e, sizeof(jobject) * n);
    return a;
}

static jobject int_array(int n, const jint* v)
{
    jobject a = new_obj(K_INTARR, "[I");
    a->n = n;
    a->ints = calloc(n ? n : 1, sizeof(jint));
    if (n) memcpy(a->ints, v, sizeof(jint) * n);
    return a;
}

/* Expect exactly the Java exception `cls` (message containing `needle`), then clear it. */
static int threw(const char* cls, const char* needle)
{
    const int ok = vm.pending && !strcmp(vm.exc_class, cls) && (!needle || strstr(vm.exc_msg, needle));
    if (!ok)
        fprintf(stderr, "  expected %s(%s), got %s(%s)\n", cls, needle ? needle : "", vm.pending ? vm.exc_class : "none",
                vm.pending ? vm.exc_msg : "");
    vm.pending = 0;
    return ok;
}

static int clean(void)
{
    if (vm.pending) fprintf(stderr, "  unexpected %s(%s)\n", vm.exc_class, vm.exc_msg);
    const int ok = !vm.pending;
    vm.pending = 0;
    return ok;
}

/* n direct buffers of len bytes at position pos[i] inside their backing memory */
struct Bufs {
    int n;
    unsigned char* mem[16];
    jobject bb[16];
    jint pos[16];
};

static void bufs_init(struct Bufs* b, int n, size_t len, int pos0)
{
    b->n = n;
    for (int i = 0; i < n; ++i) {
        b->pos[i] = pos0 + 3 * i;
        b->mem[i] = calloc(len + b->pos[i] + 16, 1);
        b->bb[i] = direct_bb(b->mem[i]);
    }
}

static unsigned char* at(struct Bufs* b, int i) { return b->mem[i] + b->pos[i]; }

/* ---- cpu: error behaviour ------------------------------------------------- */
static int cpu_checks(void)
{
    jobject enc = coder_obj(ENC_CLS), dec = coder_obj(DEC_CLS);
    struct Bufs d, p;
    bufs_init(&d, 4, 16, 1);
    bufs_init(&p, 2, 16, 2);

    jni.enc_init(env, enc, 0, 2);  /* invalid k: no coder, Java sees an exception */
    EXPECT(threw("java/lang/IllegalArgumentException", "invalid argument"));
    EXPECT(enc->native_coder == 0);

    jni.enc_init(env, enc, 4, 2);
    EXPECT(clean());
    EXPECT(enc->native_coder != 0);

    /* count mismatch -> InternalError "Invalid inputs" (EC/jni_common.c:70-73) */
    jobject in3 = obj_array(3, d.bb), off3 = int_array(3, d.pos);
    jobject in4 = obj_array(4, d.bb), off4 = int_array(4, d.pos);
    jobject out2 = obj_array(2, p.bb), poff2 = int_array(2, p.pos);
    jni.encode(env, enc, in3, off3, 16, out2, poff2);
    EXPECT(threw("java/lang/InternalError", "Invalid inputs"));
    jobject out1 = obj_array(1, p.bb), poff1 = int_array(1, p.pos);
    jni.encode(env, enc, in4, off4, 16, out1, poff1);
    EXPECT(threw("java/lang/InternalError", "Invalid outputs"));

    /* a heap ByteBuffer has no direct address -> InternalError */
    jobject heap[4] = {d.bb[0], d.bb[1], new_obj(K_HEAP, "java/nio/HeapByteBuffer"), d.bb[3]};
    jobject inh = obj_array(4, heap);
    jni.encode(env, enc, inh, off4, 16, out2, poff2);
    EXPECT(threw("java/lang/InternalError", "Invalid inputs"));

    /* a null element -> InternalError */
    jobject nul[4] = {d.bb[0], NULL, d.bb[2], d.bb[3]};
    jni.encode(env, enc, obj_array(4, nul), off4, 16, out2, poff2);
    EXPECT(threw("java/lang/InternalError", "Invalid inputs"));

    /* encodeUpdate takes [old, new, P0..m-1]: m + 2 inputs */
    jni.update(env, enc, in3, off3, 16, 0, out2, poff2);
    EXPECT(threw("java/lang/InternalError", "Invalid inputs"));

    int ndev = 0;
    if (jni.device_count(&ndev) != 0 || ndev == 0) {  /* no device: compute fails loudly */
        jni.encode(env, enc, in4, off4, 16, out2, poff2);
        EXPECT(threw("java/io/IOException", "no HIP device"));
    }

    /* optional fused methods: argument checks */
    const jint cl4[4] = {16, 3, 0, 16}, cl3[3] = {16, 16, 16}, cl_neg[4] = {16, -1, 0, 16}, cl2[2] = {5, 16};
    jobject hashes2 = int_array(2, cl2), hashes1 = int_array(1, cl2);
    jni.encode_ex(env, enc, in4, off4, int_array(3, cl3), 16, out2, poff2, hashes2);
    EXPECT(threw("java/lang/InternalError", "Invalid content lengths"));
    jni.encode_ex(env, enc, in4, off4, int_array(4, cl_neg), 16, out2, poff2, NULL);
    EXPECT(threw("java/lang/IllegalArgumentException", "negative content length"));
    jni.encode_ex(env, enc, in4, off4, int_array(4, cl4), 16, out2, poff2, hashes1);
    EXPECT(threw("java/lang/InternalError", "Invalid parity hashes"));
    jni.encode_ex(env, enc, in4, off4, int_array(4, cl4), 0, out2, poff2, hashes2);  /* empty: hashCode 1 */
    EXPECT(clean());
    EXPECT(hashes2->ints[0] == 1 && hashes2->ints[1] == 1);
    jni.update_ex(env, enc, in4, off4, int_array(4, cl4), 16, 0, out2, poff2, NULL);
    EXPECT(threw("java/lang/InternalError", "Invalid content lengths"));
    jni.update_ex(env, enc, in4, off4, int_array(2, cl2), 16, 9, out2, poff2, NULL);  /* target >= k */
    EXPECT(threw("java/lang/IllegalArgumentException", "invalid argument"));
    if (ndev == 0) {
        jni.encode_ex(env, enc, in4, off4, int_array(4, cl4), 16, out2, poff2, hashes2);
        EXPECT(threw("java/io/IOException", "no HIP device"));
        jni.update_ex(env, enc, in4, off4, int_array(2, cl2), 16, 1, out2, poff2, hashes2);
        EXPECT(threw("java/io/IOException", "no HIP device"));
    }

    /* negative dataLen on the encoder's methods */
    jni.encode(env, enc, in4, off4, -1, out2, poff2);
    EXPECT(threw("java/lang/IllegalArgumentException", "negative dataLen"));
    jni.update(env, enc, in4, off4, -16, 0, out2, poff2);
    EXPECT(threw("java/lang/IllegalArgumentException", "negative dataLen"));
    jni.encode_ex(env, enc, in4, off4, NULL, -2, out2, poff2, NULL);
    EXPECT(threw("java/lang/IllegalArgumentException", "negative dataLen"));
    jni.update_ex(env, enc, in4, off4, NULL, -3, 0, out2, poff2, NULL);
    EXPECT(threw("java/lang/IllegalArgumentException", "negative dataLen"));
    enc->verbose_throws = 1;
    jni.encode(env, enc, in4, off4, 16, out2, poff2);
    EXPECT(threw("java/lang/IllegalStateException", "allowVerboseDump"));
    enc->verbose_throws = 0;

    /* destroy zeroes the field; use after destroy -> IOException (EC/NativeRSEncoder.c:46-50) */
    jni.enc_destroy(env, enc);
    EXPECT(clean());
    EXPECT(enc->native_coder == 0);
    jni.enc_destroy(env, enc);  /* idempotent */
    EXPECT(clean());
    jni.encode(env, enc, in4, off4, 16, out2, poff2);
    EXPECT(threw("java/io/IOException", "NativeRSRawEncoder closed"));
    jni.update(env, enc, in4, off4, 16, 0, out2, poff2);
    EXPECT(threw("java/io/IOException", "NativeRSRawEncoder closed"));
    jni.encode_ex(env, enc, in4, off4, NULL, 16, out2, poff2, NULL);
    EXPECT(threw("java/io/IOException", "NativeRSRawEncoder closed"));
    jni.update_ex(env, enc, in4, off4, NULL, 16, 0, out2, poff2, NULL);
    EXPECT(threw("java/io/IOException", "NativeRSRawEncoder closed"));

    /* decoder */
    jni.dec_init(env, dec, 4, 2);
    EXPECT(clean());
    EXPECT(dec->native_coder != 0);
    const jint di3[3] = {1, 2, 3}, di4[4] = {4, 1, 2, 3}, er1[1] = {0};
    jni.decode(env, dec, in4, off4, 16, int_array(3, di3), int_array(1, er1), out1, poff1);
    EXPECT(threw("java/lang/InternalError", "Invalid decode/erased indexes"));
    jni.decode(env, dec, in3, off3, 16, int_array(4, di4), int_array(1, er1), out1, poff1);
    EXPECT(threw("java/lang/InternalError", "Invalid inputs"));
    jni.decode(env, dec, in4, off4, 16, int_array(4, di4), int_array(1, er1), out2, poff2);
    EXPECT(threw("java/lang/InternalError", "Invalid outputs"));
    const jint er_bad[1] = {7};  /* engine-side validation (unit 7 of 6) surfaces as a Java exception */
    jni.decode(env, dec, in4, off4, 16, int_array(4, di4), int_array(1, er_bad), out1, poff1);
    EXPECT(threw("java/lang/IllegalArgumentException", "invalid argument"));
    const jint dl3[3] = {16, 16, 16}, dl4[4] = {16, 3, -2, 16};
    jni.decode_ex(env, dec, in4, off4, int_array(3, dl3), 16, int_array(4, di4), int_array(1, er1), out1, poff1);
    EXPECT(threw("java/lang/InternalError", "Invalid content lengths"));
    jni.decode_ex(env, dec, in4, off4, int_array(4, dl4), 16, int_array(4, di4), int_array(1, er1), out1, poff1);
    EXPECT(threw("java/lang/IllegalArgumentException", "negative content length"));
    jni.decode_ex(env, dec, in4, off4, NULL, 16, int_array(3, di3), int_array(1, er1), out1, poff1);
    EXPECT(threw("java/lang/InternalError", "Invalid decode/erased indexes"));

    /* an object without the nativeCoder field -> UnsatisfiedLinkError (EC/jni_common.h:29-36),
     * on init and on every coding call (and nothing else thrown while it is pending) */
    jobject alien = coder_obj("java/lang/Object");
    jni.enc_init(env, alien, 4, 2);
    EXPECT(threw("java/lang/UnsatisfiedLinkError", "nativeCoder"));
    jni.encode(env, alien, in4, off4, 16, out2, poff2);
    EXPECT(threw("java/lang/UnsatisfiedLinkError", "nativeCoder"));
    jni.decode(env, alien, in4, off4, 16, int_array(4, di4), int_array(1, er1), out1, poff1);
    EXPECT(threw("java/lang/UnsatisfiedLinkError", "nativeCoder"));
    jni.update_ex(env, alien, in4, off4, NULL, 16, 0, out2, poff2, NULL);
    EXPECT(threw("java/lang/UnsatisfiedLinkError", "nativeCoder"));

    /* a negative dataLen (a Java int) -> IllegalArgumentException, never a huge size_t */
    jni.decode(env, dec, in4, off4, -5, int_array(4, di4), int_array(1, er1), out1, poff1);
    EXPECT(threw("java/lang/IllegalArgumentException", "negative dataLen"));
    jni.decode_ex(env, dec, in4, off4, NULL, -1, int_array(4, di4), int_array(1, er1), out1, poff1);
    EXPECT(threw("java/lang/IllegalArgumentException", "negative dataLen"));

    /* allowVerboseDump() throwing: its exception propagates, nothing else runs */
    dec->verbose_throws = 1;
    jni.decode(env, dec, in4, off4, 16, int_array(4, di4), int_array(1, er1), out1, poff1);
    EXPECT(threw("java/lang/IllegalStateException", "allowVerboseDump"));
    dec->verbose_throws = 0;

    jni.dec_destroy(env, dec);
    EXPECT(clean());
    EXPECT(dec->native_coder == 0);
    jni.decode(env, dec, in4, off4, 16, int_array(4, di4), int_array(1, er1), out1, poff1);
    EXPECT(threw("java/io/IOException", "NativeRSRawDecoder closed"));
    jni.decode_ex(env, dec, in4, off4, NULL, 16, int_array(4, di4), int_array(1, er1), out1, poff1);
    EXPECT(threw("java/io/IOException", "NativeRSRawDecoder closed"));

    /* page-locked coding buffers: argument errors; without a device the buffer is ordinary memory */
    jclass enc_cls = new_obj(K_CLASS, ENC_CLS);
    EXPECT(jni.alloc_direct(env, enc_cls, -1) == NULL);
    EXPECT(threw("java/lang/IllegalArgumentException", "negative capacity"));
    jobject bb = jni.alloc_direct(env, enc_cls, 4099);
    EXPECT(clean() && bb != NULL && bb->kind == K_DIRECT && bb->n == 4099);
    if (bb) {
        memset(bb->addr, 0x5A, 4099);  /* the whole capacity is writable */
        jni.free_direct(env, enc_cls, bb);
        EXPECT(clean());
        jni.free_direct(env, enc_cls, bb);  /* twice: not a live buffer any more */
        EXPECT(threw("java/lang/IllegalArgumentException", "freeDirect"));
    }
    unsigned char foreign[64];
    jni.free_direct(env, enc_cls, direct_bb(foreign));
    EXPECT(threw("java/lang/IllegalArgumentException", "freeDirect"));
    jni.free_direct(env, enc_cls, new_obj(K_HEAP, "java/nio/HeapByteBuffer"));
    EXPECT(threw("java/lang/IllegalArgumentException", "not a direct buffer"));
    jni.free_direct(env, enc_cls, NULL);
    EXPECT(clean());

    EXPECT(vm.violations == 0);
    EXPECT(vm.live_int_elems == 0);
    EXPECT(vm.local_refs == 0);
    return failures;
}

/* ---- gpu: ErasureCodeTest.java through the JNI entry points --------------- */
typedef struct {
    uint64_t seed;
} JavaRandom;

static void jr_init(JavaRandom* r, int64_t s) { r->seed = ((uint64_t)s ^ 0x5DEECE66DULL) & ((1ULL << 48) - 1); }

static void jr_next_bytes(JavaRandom* r, unsigned char* b, size_t n)
{
    for (size_t i = 0; i < n;) {
        r->seed = (r->seed * 0x5DEECE66DULL + 0xBULL) & ((1ULL << 48) - 1);
        uint32_t v = (uint32_t)(int32_t)(r->seed >> 16);
        for (int k = 0; k < 4 && i < n; ++k, v >>= 8) b[i++] = (unsigned char)v;
    }
}

static void dump(const char* dir, const char* name, int idx, const unsigned char* p, size_t n)
{
    char path[1024];
    snprintf(path, sizeof path, "%s/%s%d", dir, name, idx);
    FILE* f = fopen(path, "wb");
    if (!f || fwrite(p, 1, n, f) != n) {
        fprintf(stderr, "cannot write %s\n", path);
        exit(2);
    }
    fclose(f);
}

static int gpu_erasure_code_test(const char* outdir)
{
    enum { K = 4, M = 2 };
    const jint L = 4099;
    JavaRandom rnd;
    jr_init(&rnd, 123);
    struct Bufs data, modified, parity, second, upd, out1, out2;
    bufs_init(&data, K, L, 1);
    bufs_init(&modified, K, L, 2);
    bufs_init(&parity, M, L, 5);
    bufs_init(&second, M, L, 7);
    bufs_init(&upd, M, L, 11);
    bufs_init(&out1, 1, L, 13);
    bufs_init(&out2, 1, L, 17);
    for (int i = 0; i < K; ++i) {
        jr_next_bytes(&rnd, at(&data, i), L);
        memcpy(at(&modified, i), at(&data, i), L);
    }
    jr_next_bytes(&rnd, at(&modified, 0), L);

    jobject enc = coder_obj(ENC_CLS), dec = coder_obj(DEC_CLS);
    dec->verbose = JNI_TRUE;  /* exercise the allowVerboseDump() path */
    jni.enc_init(env, enc, K, M);
    jni.dec_init(env, dec, K, M);
    EXPECT(clean());

    jni.encode(env, enc, obj_array(K, data.bb), int_array(K, data.pos), L, obj_array(M, parity.bb),
               int_array(M, parity.pos));
    EXPECT(clean());
    jni.encode(env, enc, obj_array(K, modified.bb), int_array(K, modified.pos), L, obj_array(M, second.bb),
               int_array(M, second.pos));
    EXPECT(clean());

    const jint di[K] = {4, 1, 2, 3}, er[1] = {0};
    jobject in1[K] = {parity.bb[0], data.bb[1], data.bb[2], data.bb[3]};
    jint in1_pos[K] = {parity.pos[0], data.pos[1], data.pos[2], data.pos[3]};
    jni.decode(env, dec, obj_array(K, in1), int_array(K, in1_pos), L, int_array(K, di), int_array(1, er),
               obj_array(1, out1.bb), int_array(1, out1.pos));
    EXPECT(clean());
    jobject in2[K] = {second.bb[0], modified.bb[1], modified.bb[2], modified.bb[3]};
    jint in2_pos[K] = {second.pos[0], modified.pos[1], modified.pos[2], modified.pos[3]};
    jni.decode(env, dec, obj_array(K, in2), int_array(K, in2_pos), L, int_array(K, di), int_array(1, er),
               obj_array(1, out2.bb), int_array(1, out2.pos));
    EXPECT(clean());

    jobject uin[2 + M] = {data.bb[0], modified.bb[0], parity.bb[0], parity.bb[1]};
    jint uin_pos[2 + M] = {data.pos[0], modified.pos[0], parity.pos[0], parity.pos[1]};
    jni.update(env, enc, obj_array(2 + M, uin), int_array(2 + M, uin_pos), L, 0, obj_array(M, upd.bb),
               int_array(M, upd.pos));
    EXPECT(clean());

    EXPECT(!memcmp(at(&out1, 0), at(&data, 0), L));       /* ErasureCodeTest.java:112 */
    EXPECT(!memcmp(at(&out2, 0), at(&modified, 0), L));   /* :119 */
    for (int r = 0; r < M; ++r) EXPECT(!memcmp(at(&upd, r), at(&second, r), L));
    /* bytes before each position are untouched */
    for (int r = 0; r < M; ++r)
        for (int b = 0; b < parity.pos[r]; ++b) EXPECT(parity.mem[r][b] == 0);

    for (int i = 0; i < K; ++i) dump(outdir, "data", i, at(&data, i), L);
    for (int r = 0; r < M; ++r) {
        dump(outdir, "parity", r, at(&parity, r), L);
        dump(outdir, "second", r, at(&second, r), L);
        dump(outdir, "update", r, at(&upd, r), L);
    }
    jni.enc_destroy(env, enc);
    jni.dec_destroy(env, dec);
    EXPECT(enc->native_coder == 0 && dec->native_coder == 0);
    EXPECT(vm.violations == 0);
    EXPECT(vm.live_int_elems == 0);
    EXPECT(vm.local_refs == 0);
    return failures;
}

/* JDK ByteBuffer.hashCode() loop over [p, p+n) */
static jint java_hash(const unsigned char* p, size_t n)
{
    uint32_t h = 1;
    for (size_t i = n; i-- > 0;) h = 31u * h + (uint32_t)(int32_t)(signed char)p[i];
    return (jint)h;
}

/* The optional fused methods against the seven plain ones: encodeEx over
 * SSTable contents shorter than codeLength (0xEE garbage past each) equals
 * encode over the zero-filled buffers, with the JDK hashCode of each parity;
 * encodeUpdateEx (new parity over the old, in place) equals encoding the
 * zero-filled new stripe. */
static int gpu_fused_flows(void)
{
    enum { K = 4, M = 2 };
    const jint L = 70001;
    JavaRandom rnd;
    jr_init(&rnd, 321);
    struct Bufs raw, filled, par, ref, newd, ref2;
    bufs_init(&raw, K, L, 1);
    bufs_init(&filled, K, L, 2);
    bufs_init(&par, M, L, 3);
    bufs_init(&ref, M, L, 4);
    bufs_init(&newd, 1, L, 5);
    bufs_init(&ref2, M, L, 6);
    const jint lens[K] = {L, L - 4099, 0, 17};
    for (int i = 0; i < K; ++i) {
        jr_next_bytes(&rnd, at(&raw, i), L);
        memcpy(at(&filled, i), at(&raw, i), lens[i]);  /* calloc'd: zero past the content */
        memset(at(&raw, i) + lens[i], 0xEE, L - lens[i]);
    }
    jobject enc = coder_obj(ENC_CLS);
    jni.enc_init(env, enc, K, M);
    jobject hashes = int_array(M, lens);
    jni.encode_ex(env, enc, obj_array(K, raw.bb), int_array(K, raw.pos), int_array(K, lens), L,
                  obj_array(M, par.bb), int_array(M, par.pos), hashes);
    EXPECT(clean());
    jni.encode(env, enc, obj_array(K, filled.bb), int_array(K, filled.pos), L, obj_array(M, ref.bb),
               int_array(M, ref.pos));
    EXPECT(clean());
    for (int r = 0; r < M; ++r) {
        EXPECT(!memcmp(at(&par, r), at(&ref, r), L));
        EXPECT(hashes->ints[r] == java_hash(at(&ref, r), L));
    }
    /* compaction replaces unit 1: old content lens[1] bytes, new content 5000 bytes */
    const jint ulens[2] = {lens[1], 5000};
    jr_next_bytes(&rnd, at(&newd, 0), L);
    jobject uin[2 + M] = {raw.bb[1], newd.bb[0], par.bb[0], par.bb[1]};
    jint uin_pos[2 + M] = {raw.pos[1], newd.pos[0], par.pos[0], par.pos[1]};
    jni.update_ex(env, enc, obj_array(2 + M, uin), int_array(2 + M, uin_pos), int_array(2, ulens), L, 1,
                  obj_array(M, par.bb), int_array(M, par.pos), hashes);
    EXPECT(clean());
    memset(at(&filled, 1), 0, L);
    memcpy(at(&filled, 1), at(&newd, 0), ulens[1]);
    jni.encode(env, enc, obj_array(K, filled.bb), int_array(K, filled.pos), L, obj_array(M, ref2.bb),
               int_array(M, ref2.pos));
    EXPECT(clean());
    for (int r = 0; r < M; ++r) {
        EXPECT(!memcmp(at(&par, r), at(&ref2, r), L));
        EXPECT(hashes->ints[r] == java_hash(at(&ref2, r), L));
    }
    /* degraded read of unit 1 (new content, 5000 bytes) from [P0, d0, d2, d3]: the data
     * survivors padded past their content, only the 5000-byte prefix decoded (ECRecovery) */
    jobject dec = coder_obj(DEC_CLS);
    jni.dec_init(env, dec, K, M);
    struct Bufs rb;
    bufs_init(&rb, 1, L, 7);
    memset(at(&rb, 0), 0x33, L);
    const jint di[K] = {4, 0, 2, 3}, er[1] = {1};
    const jint dlens[K] = {L, lens[0], lens[2], lens[3]};
    jobject din[K] = {par.bb[0], raw.bb[0], raw.bb[2], raw.bb[3]};
    jint din_pos[K] = {par.pos[0], raw.pos[0], raw.pos[2], raw.pos[3]};
    jni.decode_ex(env, dec, obj_array(K, din), int_array(K, din_pos), int_array(K, dlens), ulens[1], int_array(K, di),
                  int_array(1, er), obj_array(1, rb.bb), int_array(1, rb.pos));
    EXPECT(clean());
    EXPECT(!memcmp(at(&rb, 0), at(&newd, 0), ulens[1]));
    EXPECT(at(&rb, 0)[ulens[1]] == 0x33);  /* nothing past the requested prefix is written */
    jni.dec_destroy(env, dec);

    /* ELECT's encode with its units in allocateDirectImpl buffers (page-locked: the
     * engine moves them by DMA, no staging copy) equals the encode of ordinary ones */
    jclass enc_cls = new_obj(K_CLASS, ENC_CLS);
    jobject pin_in[K], pin_out[M];
    jint zero_pos[K] = {0, 0, 0, 0};
    for (int i = 0; i < K; ++i) {
        pin_in[i] = jni.alloc_direct(env, enc_cls, L);
        EXPECT(clean() && pin_in[i] != NULL && jni.host_pinned(pin_in[i]->addr, (size_t)L));
        memcpy(pin_in[i]->addr, at(&filled, i), L);
    }
    for (int r = 0; r < M; ++r) {
        pin_out[r] = jni.alloc_direct(env, enc_cls, L);
        EXPECT(clean() && pin_out[r] != NULL);
        memset(pin_out[r]->addr, 0xCC, L);
    }
    jni.encode(env, enc, obj_array(K, pin_in), int_array(K, zero_pos), L, obj_array(M, pin_out),
               int_array(M, zero_pos));
    EXPECT(clean());
    jni.encode(env, enc, obj_array(K, filled.bb), int_array(K, filled.pos), L, obj_array(M, ref.bb),
               int_array(M, ref.pos));
    EXPECT(clean());
    for (int r = 0; r < M; ++r) EXPECT(!memcmp(pin_out[r]->addr, at(&ref, r), L));
    for (int i = 0; i < K; ++i) jni.free_direct(env, enc_cls, pin_in[i]);
    for (int r = 0; r < M; ++r) jni.free_direct(env, enc_cls, pin_out[r]);
    EXPECT(clean());
    jni.enc_destroy(env, enc);
    EXPECT(vm.violations == 0);
    EXPECT(vm.live_int_elems == 0);
    EXPECT(vm.local_refs == 0);
    return failures;
}

/* ---- dump: allowVerboseDump() == true, the coder dumps on stdout ---------- *
 * Prints "=== <case>" before each call; the calls' own results (the data, or
 * an IOException without a device) are not part of the dump and are cleared. */
static int dump_cases(void)
{
    struct Bufs d, p;
    bufs_init(&d, 8, 16, 1);
    bufs_init(&p, 4, 16, 2);
    jobject enc = coder_obj(ENC_CLS), dec = coder_obj(DEC_CLS), dec12 = coder_obj(DEC_CLS);
    enc->verbose = dec->verbose = dec12->verbose = JNI_TRUE;
    jni.enc_init(env, enc, 4, 2);
    jni.dec_init(env, dec, 4, 2);
    jni.dec_init(env, dec12, 8, 4);
    EXPECT(clean());
    jobject in4 = obj_array(4, d.bb), off4 = int_array(4, d.pos);
    jobject in8 = obj_array(8, d.bb), off8 = int_array(8, d.pos);
    jobject out1 = obj_array(1, p.bb), poff1 = int_array(1, p.pos);
    jobject out2 = obj_array(2, p.bb), poff2 = int_array(2, p.pos);
    printf("=== encode RS(6,4)\n");
    fflush(stdout);
    jni.encode(env, enc, in4, off4, 16, out2, poff2);
    vm.pending = 0;
    const jint di[4] = {4, 1, 2, 3}, er[1] = {0}, ds[4] = {1, 1, 2, 3}, er2[2] = {0, 5};
    printf("=== decode RS(6,4) {4,1,2,3} erase {0}\n");
    fflush(stdout);
    jni.decode(env, dec, in4, off4, 16, int_array(4, di), int_array(1, er), out1, poff1);
    vm.pending = 0;
    printf("=== decode RS(6,4) singular {1,1,2,3} erase {0,5}\n");
    fflush(stdout);
    jni.decode(env, dec, in4, off4, 16, int_array(4, ds), int_array(2, er2), out2, poff2);
    vm.pending = 0;
    const jint di12[8] = {2, 3, 4, 5, 6, 7, 8, 10}, er12[2] = {9, 0};
    printf("=== decode RS(12,8) {2..8,10} erase {9,0}\n");
    fflush(stdout);
    jni.decode(env, dec12, in8, off8, 16, int_array(8, di12), int_array(2, er12), out2, poff2);
    vm.pending = 0;
    printf("=== encodeUpdate RS(6,4)\n");  /* verbose too: libec.so never dumps the encoder */
    fflush(stdout);
    jni.update(env, enc, in4, off4, 16, 1, out2, poff2);
    vm.pending = 0;
    enc->verbose = dec->verbose = JNI_FALSE;
    printf("=== quiet encode RS(6,4)\n");
    fflush(stdout);
    jni.encode(env, enc, in4, off4, 16, out2, poff2);
    vm.pending = 0;
    printf("=== quiet decode RS(6,4) {4,1,2,3} erase {0}\n");  /* the three lines, unconditionally */
    fflush(stdout);
    jni.decode(env, dec, in4, off4, 16, int_array(4, di), int_array(1, er), out1, poff1);
    vm.pending = 0;
    printf("=== end\n");
    jni.enc_destroy(env, enc);
    jni.dec_destroy(env, dec);
    jni.dec_destroy(env, dec12);
    EXPECT(vm.violations == 0);
    return failures;
}

int main(int argc, char** argv)
{
    if (argc < 3) {
        fprintf(stderr, "usage: %s LIB cpu | LIB dump | LIB gpu OUTDIR\n", argv[0]);
        return 2;
    }
    load(argv[1]);
    const int gpu = !strcmp(argv[2], "gpu");
    if (!strcmp(argv[2], "dump")) {
        const int rc = dump_cases();
        fprintf(stderr, "dump: %d failure(s), %d JNI violation(s)\n", rc, vm.violations);
        return rc == 0 ? 0 : 1;
    }
    int rc = gpu ? gpu_erasure_code_test(argc > 3 ? argv[3] : ".") : cpu_checks();
    if (gpu && rc == 0) rc = gpu_fused_flows();
    printf("%s: %d failure(s), %d JNI violation(s)\n", argv[2], rc, vm.violations);
    return rc == 0 ? 0 : 1;
}
