/*
 * Test-only stand-in for the JDK's jni.h (this image has no JDK): the JNI types and the six JNIEnv
 * functions sparkey-java_amd/jni/sparkey_gpu_jni.c uses, with the JNI specification's names and
 * signatures, so the shim compiles unchanged and tests/jni/harness.c can drive it with a recording
 * environment.  Not shipped; a real build compiles the shim against $JAVA_HOME/include/jni.h.
 */
#ifndef SPARKEY_TEST_JNI_H
#define SPARKEY_TEST_JNI_H
#include <stdint.h>

#define JNIEXPORT __attribute__((visibility("default")))
#define JNICALL

typedef int32_t jint;
typedef int64_t jlong;
typedef uint8_t jboolean;
typedef double jdouble;
typedef jint jsize;
typedef struct _jobject* jobject;
typedef jobject jclass;
typedef jobject jstring;
typedef jobject jarray;
typedef jarray jlongArray;
typedef jobject jthrowable;

struct JNINativeInterface_;
typedef const struct JNINativeInterface_* JNIEnv;

struct JNINativeInterface_ {
  jclass(JNICALL* FindClass)(JNIEnv* env, const char* name);
  jint(JNICALL* ThrowNew)(JNIEnv* env, jclass clazz, const char* msg);
  const char*(JNICALL* GetStringUTFChars)(JNIEnv* env, jstring str, jboolean* isCopy);
  void(JNICALL* ReleaseStringUTFChars)(JNIEnv* env, jstring str, const char* chars);
  jsize(JNICALL* GetArrayLength)(JNIEnv* env, jarray array);
  void(JNICALL* SetLongArrayRegion)(JNIEnv* env, jlongArray array, jsize start, jsize len, const jlong* buf);
};
#endif
