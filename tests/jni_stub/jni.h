/*
 * jni.h stand-in for testing jni/kcep_jni.c without a JDK (the image has none).
 *
 * Test infrastructure only.  It declares the JNI types and a JNIEnv function table holding exactly
 * the functions kcep_jni.c calls, with the JNI specification's names and signatures; mock_jni.c
 * implements them over plain C arrays.  The shim is compiled unchanged against it, so its
 * argument handling, batch construction and C-ABI calls are what the tests exercise.  (The table's
 * layout is not the JVM's: a real build uses $JAVA_HOME/include/jni.h.)
 */
#ifndef KCEP_TEST_JNI_H
#define KCEP_TEST_JNI_H
#include <stdint.h>

typedef int32_t jint;
typedef int64_t jlong;
typedef int8_t jbyte;
typedef uint8_t jboolean;
typedef double jdouble;
typedef jint jsize;

typedef struct _jobject* jobject;
typedef jobject jclass;
typedef jobject jstring;
typedef jobject jarray;
typedef jarray jobjectArray;
typedef jarray jbyteArray;
typedef jarray jintArray;
typedef jarray jlongArray;

#define JNI_ABORT 2
#define JNIEXPORT __attribute__((visibility("default")))
#define JNICALL

struct JNINativeInterface_;
typedef const struct JNINativeInterface_* JNIEnv;

struct JNINativeInterface_ {
  jclass (*FindClass)(JNIEnv*, const char*);
  jsize (*GetArrayLength)(JNIEnv*, jarray);
  jobjectArray (*NewObjectArray)(JNIEnv*, jsize, jclass, jobject);
  jobject (*GetObjectArrayElement)(JNIEnv*, jobjectArray, jsize);
  void (*SetObjectArrayElement)(JNIEnv*, jobjectArray, jsize, jobject);
  jstring (*NewStringUTF)(JNIEnv*, const char*);
  jbyteArray (*NewByteArray)(JNIEnv*, jsize);
  jlongArray (*NewLongArray)(JNIEnv*, jsize);
  jbyte* (*GetByteArrayElements)(JNIEnv*, jbyteArray, jboolean*);
  void (*ReleaseByteArrayElements)(JNIEnv*, jbyteArray, jbyte*, jint);
  jint* (*GetIntArrayElements)(JNIEnv*, jintArray, jboolean*);
  void (*ReleaseIntArrayElements)(JNIEnv*, jintArray, jint*, jint);
  void (*SetByteArrayRegion)(JNIEnv*, jbyteArray, jsize, jsize, const jbyte*);
  void (*SetIntArrayRegion)(JNIEnv*, jintArray, jsize, jsize, const jint*);
  void (*SetLongArrayRegion)(JNIEnv*, jlongArray, jsize, jsize, const jlong*);
  void* (*GetPrimitiveArrayCritical)(JNIEnv*, jarray, jboolean*);
  void (*ReleasePrimitiveArrayCritical)(JNIEnv*, jarray, void*, jint);
  void (*GetByteArrayRegion)(JNIEnv*, jbyteArray, jsize, jsize, jbyte*);
  void (*DeleteLocalRef)(JNIEnv*, jobject);
};

#endif
