/* Minimal stand-in for a JDK's jni.h: only the types and the JNIEnv function-table entries
 * jvm/jni/cordagpu_jni.c uses, so that tests/test_jvm_binding.py can type-check the shim against
 * include/cordagpu.h with gcc (no JDK in this image). Test infrastructure, never linked. */
#ifndef CG_JNI_STUB_H
#define CG_JNI_STUB_H
#include <stdint.h>
#define JNIEXPORT __attribute__((visibility("default")))
#define JNICALL
#define JNI_ABORT 2
typedef int32_t jint;
typedef int64_t jlong;
typedef int32_t jsize;
typedef uint8_t jboolean;
typedef struct _jobject* jobject;
typedef jobject jclass;
typedef jobject jintArray;
struct JNINativeInterface_;
typedef const struct JNINativeInterface_* JNIEnv;
struct JNINativeInterface_ {
  jclass (*FindClass)(JNIEnv*, const char*);
  jint (*ThrowNew)(JNIEnv*, jclass, const char*);
  jsize (*GetArrayLength)(JNIEnv*, jobject);
  jint* (*GetIntArrayElements)(JNIEnv*, jintArray, jboolean*);
  void (*ReleaseIntArrayElements)(JNIEnv*, jintArray, jint*, jint);
  void* (*GetDirectBufferAddress)(JNIEnv*, jobject);
};
#endif
