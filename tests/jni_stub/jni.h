/* Minimal JNI declarations for a syntax / type check of java/jni/hgx_jni.c in a build image without
 * a JDK (tests/test_abi.py::test_jni_shim_compiles).  Only what the shim uses; the layout of the
 * real JNINativeInterface_ is irrelevant to a -fsyntax-only check.  TEST INFRASTRUCTURE. */
#ifndef HGX_TEST_JNI_STUB_H
#define HGX_TEST_JNI_STUB_H
#include <stdint.h>
#define JNIEXPORT
#define JNICALL
#define JNI_ABORT 2
typedef int32_t jint;
typedef int64_t jlong;
typedef int8_t jbyte;
typedef uint8_t jboolean;
typedef jint jsize;
typedef struct _jobject *jobject;
typedef jobject jclass, jstring, jarray, jthrowable;
typedef jarray jintArray, jlongArray, jbyteArray;
struct JNINativeInterface_;
typedef const struct JNINativeInterface_ *JNIEnv;
struct JNINativeInterface_ {
    jclass (*FindClass)(JNIEnv *, const char *);
    jint (*ThrowNew)(JNIEnv *, jclass, const char *);
    jsize (*GetArrayLength)(JNIEnv *, jarray);
    jint *(*GetIntArrayElements)(JNIEnv *, jintArray, jboolean *);
    jlong *(*GetLongArrayElements)(JNIEnv *, jlongArray, jboolean *);
    jbyte *(*GetByteArrayElements)(JNIEnv *, jbyteArray, jboolean *);
    void (*ReleaseIntArrayElements)(JNIEnv *, jintArray, jint *, jint);
    void (*ReleaseLongArrayElements)(JNIEnv *, jlongArray, jlong *, jint);
    void (*ReleaseByteArrayElements)(JNIEnv *, jbyteArray, jbyte *, jint);
    jintArray (*NewIntArray)(JNIEnv *, jsize);
    jlongArray (*NewLongArray)(JNIEnv *, jsize);
    jbyteArray (*NewByteArray)(JNIEnv *, jsize);
    jarray (*NewDoubleArray)(JNIEnv *, jsize);
    void (*SetIntArrayRegion)(JNIEnv *, jintArray, jsize, jsize, const jint *);
    void (*SetLongArrayRegion)(JNIEnv *, jlongArray, jsize, jsize, const jlong *);
    void (*SetByteArrayRegion)(JNIEnv *, jbyteArray, jsize, jsize, const jbyte *);
    void (*SetDoubleArrayRegion)(JNIEnv *, jarray, jsize, jsize, const double *);
    void (*GetByteArrayRegion)(JNIEnv *, jbyteArray, jsize, jsize, jbyte *);
    const char *(*GetStringUTFChars)(JNIEnv *, jstring, jboolean *);
    void (*ReleaseStringUTFChars)(JNIEnv *, jstring, const char *);
    jstring (*NewStringUTF)(JNIEnv *, const char *);
    jboolean (*ExceptionCheck)(JNIEnv *);
};
#endif
