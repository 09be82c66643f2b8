/*
 * mock_jni.c -- a JNIEnv over plain C arrays, for driving jni/kcep_jni.c from Python (ctypes)
 * without a JVM.  Test infrastructure only (tests/test_jni_gpu.py, tests/test_native_cpu.py).
 *
 * Objects are `struct _jobject`: primitive arrays point at caller-owned memory (a numpy buffer,
 * so Set*Region writes are visible to the test), object arrays hold jobject slots, strings hold a
 * copy.  Every Get*Elements / GetPrimitiveArrayCritical hands out the array's own memory and
 * counts the pin; mock_pins() lets a test check that every pin was released.
 */
#include <stdlib.h>
#include <string.h>

#include "jni.h"

enum { K_PRIM = 0, K_OBJ = 1, K_STR = 2, K_CLASS = 3 };

struct _jobject {
  int kind;
  jsize len;
  size_t elem;
  void* data;
};

static long g_pins = 0;

static jobject mk(int kind, jsize len, size_t elem, void* data) {
  struct _jobject* o = calloc(1, sizeof *o);
  o->kind = kind;
  o->len = len;
  o->elem = elem;
  o->data = data;
  return o;
}

static jclass FindClass(JNIEnv* e, const char* name) { return mk(K_CLASS, 0, 0, strdup(name)); }
static jsize GetArrayLength(JNIEnv* e, jarray a) { return a->len; }
static jobjectArray NewObjectArray(JNIEnv* e, jsize n, jclass c, jobject init) {
  jobject* slots = calloc((size_t)(n ? n : 1), sizeof(jobject));
  for (jsize i = 0; i < n; i++) slots[i] = init;
  return mk(K_OBJ, n, sizeof(jobject), slots);
}
static jobject GetObjectArrayElement(JNIEnv* e, jobjectArray a, jsize i) { return ((jobject*)a->data)[i]; }
static void SetObjectArrayElement(JNIEnv* e, jobjectArray a, jsize i, jobject v) { ((jobject*)a->data)[i] = v; }
static jstring NewStringUTF(JNIEnv* e, const char* s) { return mk(K_STR, (jsize)strlen(s), 1, strdup(s)); }
static jbyteArray NewByteArray(JNIEnv* e, jsize n) { return mk(K_PRIM, n, 1, calloc((size_t)(n ? n : 1), 1)); }
static jlongArray NewLongArray(JNIEnv* e, jsize n) { return mk(K_PRIM, n, 8, calloc((size_t)(n ? n : 1), 8)); }
static void* pin(jarray a) { g_pins++; return a->data; }
static void unpin(void) { g_pins--; }
static jbyte* GetByteArrayElements(JNIEnv* e, jbyteArray a, jboolean* c) { return pin(a); }
static void ReleaseByteArrayElements(JNIEnv* e, jbyteArray a, jbyte* p, jint mode) { unpin(); }
static jint* GetIntArrayElements(JNIEnv* e, jintArray a, jboolean* c) { return pin(a); }
static void ReleaseIntArrayElements(JNIEnv* e, jintArray a, jint* p, jint mode) { unpin(); }
static void SetByteArrayRegion(JNIEnv* e, jbyteArray a, jsize at, jsize n, const jbyte* src) {
  memcpy((jbyte*)a->data + at, src, (size_t)n);
}
static void SetIntArrayRegion(JNIEnv* e, jintArray a, jsize at, jsize n, const jint* src) {
  memcpy((jint*)a->data + at, src, (size_t)n * 4);
}
static void SetLongArrayRegion(JNIEnv* e, jlongArray a, jsize at, jsize n, const jlong* src) {
  memcpy((jlong*)a->data + at, src, (size_t)n * 8);
}
static void* GetPrimitiveArrayCritical(JNIEnv* e, jarray a, jboolean* c) { return pin(a); }
static void ReleasePrimitiveArrayCritical(JNIEnv* e, jarray a, void* p, jint mode) { unpin(); }

static void GetByteArrayRegion(JNIEnv* e, jbyteArray a, jsize at, jsize n, jbyte* dst) {
  memcpy(dst, (const jbyte*)a->data + at, (size_t)n);
}
/* local refs are counted, not freed: the tests read arrays the shim has already dropped */
static long g_deleted = 0;
static void DeleteLocalRef(JNIEnv* e, jobject o) { g_deleted++; }

static const struct JNINativeInterface_ g_table = {
    FindClass, GetArrayLength, NewObjectArray, GetObjectArrayElement, SetObjectArrayElement, NewStringUTF,
    NewByteArray, NewLongArray, GetByteArrayElements, ReleaseByteArrayElements, GetIntArrayElements,
    ReleaseIntArrayElements, SetByteArrayRegion, SetIntArrayRegion, SetLongArrayRegion, GetPrimitiveArrayCritical,
    ReleasePrimitiveArrayCritical, GetByteArrayRegion, DeleteLocalRef};
static JNIEnv g_env = &g_table;

/* ---- helpers for the Python side ---- */
JNIEXPORT JNIEnv* mock_env(void) { return &g_env; }
/* a Java primitive array over caller memory (not copied) */
JNIEXPORT jobject mock_prim_array(void* data, jsize len, jint elem) { return mk(K_PRIM, len, (size_t)elem, data); }
JNIEXPORT jobject mock_obj_array(jsize len) { return NewObjectArray(&g_env, len, NULL, NULL); }
JNIEXPORT void mock_obj_set(jobject a, jsize i, jobject v) { ((jobject*)a->data)[i] = v; }
JNIEXPORT jobject mock_obj_get(jobject a, jsize i) { return ((jobject*)a->data)[i]; }
JNIEXPORT void* mock_data(jobject a) { return a ? a->data : NULL; }
JNIEXPORT jsize mock_len(jobject a) { return a ? a->len : -1; }
JNIEXPORT long mock_pins(void) { return g_pins; }
JNIEXPORT long mock_deleted_refs(void) { return g_deleted; }
