/*
 * tests/jni/mock/jni.h — TEST DOUBLE, not a JDK header.
 *
 * This image has no JDK, so the drop-in JNI shim (elect_amd/csrc/jni/libec_jni.c)
 * cannot be compiled against the JDK's <jni.h>.  This header declares the JNI
 * types and the JNIEnv function table LAID OUT AS THE JNI SPECIFICATION DEFINES
 * IT ("JNI Functions: Interface Function Table"): 235 pointer slots in the
 * specification's order (slots 0-3 reserved, FindClass at 6, ...,
 * NewDirectByteBuffer at 229, GetDirectBufferAddress at 230, up to IsVirtualThread
 * at 234), with the slots
 * the shim calls named and typed as in the JDK header and every other slot
 * kept as padding.  The static asserts below pin each named slot's index, so a
 * library built against this header calls the same table entries a JDK-built
 * one does and can be loaded by a real JVM as well as by the fake JVM in
 * tests/jni/jni_shim_test.c.  Types follow the JDK's jni.h + jni_md.h for
 * Linux/LP64 (jint = int, jlong = long, jboolean = unsigned char).
 * Production builds still use the JDK's header (build_libec.sh).
 */
#ifndef ELECT_TEST_MOCK_JNI_H
#define ELECT_TEST_MOCK_JNI_H

#include <stddef.h>

typedef int jint;
typedef long jlong;
typedef signed char jbyte;
typedef unsigned char jboolean;
typedef jint jsize;

struct _jobject;
typedef struct _jobject* jobject;
typedef jobject jclass;
typedef jobject jarray;
typedef jarray jobjectArray;
typedef jarray jintArray;
struct _jfieldID;
typedef struct _jfieldID* jfieldID;
struct _jmethodID;
typedef struct _jmethodID* jmethodID;

#define JNI_FALSE 0
#define JNI_TRUE 1
#define JNI_COMMIT 1
#define JNI_ABORT 2

#define JNIEXPORT __attribute__((visibility("default")))
#define JNICALL

struct JNINativeInterface_;
typedef const struct JNINativeInterface_* JNIEnv;

struct JNINativeInterface_ {
    void* unused_0_5[6];
    jclass (*FindClass)(JNIEnv*, const char*); /* 6 */
    void* unused_7_13[7];
    jint (*ThrowNew)(JNIEnv*, jclass, const char*); /* 14 */
    void* unused_15_16[2];
    void (*ExceptionClear)(JNIEnv*); /* 17 */
    void* unused_18_22[5];
    void (*DeleteLocalRef)(JNIEnv*, jobject); /* 23 */
    void* unused_24_30[7];
    jclass (*GetObjectClass)(JNIEnv*, jobject); /* 31 */
    void* unused_32;
    jmethodID (*GetMethodID)(JNIEnv*, jclass, const char*, const char*); /* 33 */
    void* unused_34_36[3];
    jboolean (*CallBooleanMethod)(JNIEnv*, jobject, jmethodID, ...); /* 37 */
    void* unused_38_93[56];
    jfieldID (*GetFieldID)(JNIEnv*, jclass, const char*, const char*); /* 94 */
    void* unused_95_100[6];
    jlong (*GetLongField)(JNIEnv*, jobject, jfieldID); /* 101 */
    void* unused_102_109[8];
    void (*SetLongField)(JNIEnv*, jobject, jfieldID, jlong); /* 110 */
    void* unused_111_170[60];
    jsize (*GetArrayLength)(JNIEnv*, jarray); /* 171 */
    void* unused_172;
    jobject (*GetObjectArrayElement)(JNIEnv*, jobjectArray, jsize); /* 173 */
    void* unused_174_186[13];
    jint* (*GetIntArrayElements)(JNIEnv*, jintArray, jboolean*); /* 187 */
    void* unused_188_194[7];
    void (*ReleaseIntArrayElements)(JNIEnv*, jintArray, jint*, jint); /* 195 */
    void* unused_196_202[7];
    void (*GetIntArrayRegion)(JNIEnv*, jintArray, jsize, jsize, jint*); /* 203 */
    void* unused_204_210[7];
    void (*SetIntArrayRegion)(JNIEnv*, jintArray, jsize, jsize, const jint*); /* 211 */
    void* unused_212_227[16];
    jboolean (*ExceptionCheck)(JNIEnv*); /* 228 */
    jobject (*NewDirectByteBuffer)(JNIEnv*, void*, jlong); /* 229 */
    void* (*GetDirectBufferAddress)(JNIEnv*, jobject); /* 230 */
    void* unused_231_234[4];
};

#define JNI_SLOT(name, index) \
    _Static_assert(offsetof(struct JNINativeInterface_, name) == (index) * sizeof(void*), \
                   #name " must be JNI function table slot " #index)
JNI_SLOT(FindClass, 6);
JNI_SLOT(ThrowNew, 14);
JNI_SLOT(ExceptionClear, 17);
JNI_SLOT(DeleteLocalRef, 23);
JNI_SLOT(GetObjectClass, 31);
JNI_SLOT(GetMethodID, 33);
JNI_SLOT(CallBooleanMethod, 37);
JNI_SLOT(GetFieldID, 94);
JNI_SLOT(GetLongField, 101);
JNI_SLOT(SetLongField, 110);
JNI_SLOT(GetArrayLength, 171);
JNI_SLOT(GetObjectArrayElement, 173);
JNI_SLOT(GetIntArrayElements, 187);
JNI_SLOT(ReleaseIntArrayElements, 195);
JNI_SLOT(GetIntArrayRegion, 203);
JNI_SLOT(SetIntArrayRegion, 211);
JNI_SLOT(ExceptionCheck, 228);
JNI_SLOT(NewDirectByteBuffer, 229);
JNI_SLOT(GetDirectBufferAddress, 230);
_Static_assert(sizeof(struct JNINativeInterface_) == 235 * sizeof(void*), "JNI function table size (JDK 21)");
_Static_assert(sizeof(jint) == 4 && sizeof(jlong) == 8 && sizeof(jboolean) == 1, "JNI primitive sizes");

#endif
