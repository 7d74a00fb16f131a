/*
 * tests/jni/mock/jni.h — TEST DOUBLE, not a JDK header.
 *
 * This image has no JDK, so the drop-in JNI shim (elect_amd/csrc/jni/libec_jni.c)
 * cannot be compiled against the real <jni.h>.  This file declares the JNI
 * types and exactly the JNIEnv functions the shim calls, with the JNI
 * specification's names and C calling shape ((*env)->Fn(env, ...)), so that
 * the shim's own source compiles unchanged and can be driven by a fake JVM
 * (tests/jni/jni_shim_test.c).  It is API-compatible only: the function table
 * layout is NOT the JDK's, so a library built against it can only be loaded by
 * that fake JVM.  Production builds use the JDK's header (build_libec.sh).
 */
#ifndef ELECT_TEST_MOCK_JNI_H
#define ELECT_TEST_MOCK_JNI_H

#include <stdint.h>

typedef int32_t jint;
typedef int64_t jlong;
typedef int8_t jbyte;
typedef uint8_t jboolean;
typedef jint jsize;

typedef struct _jobject* jobject;
typedef jobject jclass;
typedef jobject jarray;
typedef jobject jobjectArray;
typedef jobject jintArray;
typedef struct _jfieldID* jfieldID;
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
    jclass (*FindClass)(JNIEnv*, const char*);
    jint (*ThrowNew)(JNIEnv*, jclass, const char*);
    void (*ExceptionClear)(JNIEnv*);
    jclass (*GetObjectClass)(JNIEnv*, jobject);
    jfieldID (*GetFieldID)(JNIEnv*, jclass, const char*, const char*);
    jmethodID (*GetMethodID)(JNIEnv*, jclass, const char*, const char*);
    jboolean (*CallBooleanMethod)(JNIEnv*, jobject, jmethodID, ...);
    jlong (*GetLongField)(JNIEnv*, jobject, jfieldID);
    void (*SetLongField)(JNIEnv*, jobject, jfieldID, jlong);
    jsize (*GetArrayLength)(JNIEnv*, jarray);
    jobject (*GetObjectArrayElement)(JNIEnv*, jobjectArray, jsize);
    jint* (*GetIntArrayElements)(JNIEnv*, jintArray, jboolean*);
    void (*ReleaseIntArrayElements)(JNIEnv*, jintArray, jint*, jint);
    void (*GetIntArrayRegion)(JNIEnv*, jintArray, jsize, jsize, jint*);
    void (*SetIntArrayRegion)(JNIEnv*, jintArray, jsize, jsize, const jint*);
    void* (*GetDirectBufferAddress)(JNIEnv*, jobject);
    void (*DeleteLocalRef)(JNIEnv*, jobject);
};

#endif
