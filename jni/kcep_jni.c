/*
 * kcep_jni.c -- JNI shims between libkcep.so (include/kcep.h) and the Java side:
 *   java/com/github/fhuss/kafka/streams/cep/processor/GpuCEPProcessor.java (cep* natives) and
 *   java/com/github/fhuss/kafka/streams/cep/pattern/PatternIR.java (irb* natives, the IR builder).
 *
 * NOT BUILT in this repository: the image has no JDK, hence no jni.h.  A
 * maintainer builds it with
 *     gcc -shared -fPIC -I$JAVA_HOME/include -I$JAVA_HOME/include/linux -Iinclude \
 *         jni/kcep_jni.c -Lkafkastreams-cep_amd -lkcep -o libkcep_jni.so
 * Every shim is a thin call into the C-ABI: handles travel as jlong, errors as negative codes
 * with the message in cepLastError().  Host arrays are pinned only for the duration of the call
 * (GetPrimitiveArrayCritical); cep_push_batch stages them to the device and returns.
 *
 * Tested without a JVM: tests/test_jni_gpu.py compiles this file against tests/jni_stub/jni.h (a
 * JNIEnv with exactly the functions used here, over plain C arrays) and drives it in the order
 * GpuCEPProcessor.flush() calls it.
 */
#include <jni.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "kcep.h"

#define CLS(name) Java_com_github_fhuss_kafka_streams_cep_processor_GpuCEPProcessor_##name

static cep_session* S(jlong h) { return (cep_session*)(intptr_t)h; }

JNIEXPORT jlong JNICALL CLS(cepCompile)(JNIEnv* env, jclass c, jbyteArray ir) {
  jsize n = (*env)->GetArrayLength(env, ir);
  jbyte* p = (*env)->GetByteArrayElements(env, ir, NULL);
  cep_pattern* pat = NULL;
  int rc = cep_compile((const uint8_t*)p, (size_t)n, &pat);
  (*env)->ReleaseByteArrayElements(env, ir, p, JNI_ABORT);
  return rc ? -(jlong)rc : (jlong)(intptr_t)pat;
}

JNIEXPORT jobjectArray JNICALL CLS(cepStageNames)(JNIEnv* env, jclass c, jlong pattern) {
  cep_pattern_info info;
  if (cep_pattern_get_info((const cep_pattern*)(intptr_t)pattern, &info)) return NULL;
  jobjectArray out = (*env)->NewObjectArray(env, info.n_names, (*env)->FindClass(env, "java/lang/String"), NULL);
  for (int32_t i = 0; i < info.n_names; i++)
    (*env)->SetObjectArrayElement(env, out, i,
                                  (*env)->NewStringUTF(env, cep_pattern_name((const cep_pattern*)(intptr_t)pattern, i)));
  return out;
}

JNIEXPORT jlong JNICALL CLS(cepSessionOpen)(JNIEnv* env, jclass c, jlong pattern, jint device, jint mode,
                                            jlong max_events, jint flags, jlong max_keys, jlong max_key_words,
                                            jlong max_pool_bytes) {
  cep_opts o;
  memset(&o, 0, sizeof o);
  o.device = device;
  o.mode = mode;
  o.flags = flags;
  o.max_events = max_events;
  o.max_keys = max_keys;
  o.max_key_words = max_key_words;
  o.max_pool_bytes = max_pool_bytes;
  cep_session* s = NULL;
  int rc = cep_session_open((const cep_pattern*)(intptr_t)pattern, &o, &s);
  return rc ? -(jlong)rc : (jlong)(intptr_t)s;
}

JNIEXPORT jint JNICALL CLS(cepSessionPath)(JNIEnv* env, jclass c, jlong session) { return cep_session_path(S(session)); }

/* cols: int[] / long[] / double[] per column type (1 / 2 / 3); flags: cep_batch.flags
   (CEP_BATCH_OFFSETS_MONOTONE once the caller applied the high-water mark itself) */
JNIEXPORT jint JNICALL CLS(cepPushBatch)(JNIEnv* env, jclass c, jlong session, jint n, jintArray key,
                                         jintArray topic, jintArray partition, jlongArray offset, jlongArray ts,
                                         jintArray col_types, jobjectArray cols, jint flags) {
  const jsize nc = (*env)->GetArrayLength(env, cols);
  if (nc > 16) return CEP_E_ARG;
  jarray arrs[5 + 16];
  void* ptrs[5 + 16];
  arrs[0] = key; arrs[1] = topic; arrs[2] = partition; arrs[3] = offset; arrs[4] = ts;
  for (jsize i = 0; i < nc; i++) arrs[5 + i] = (jarray)(*env)->GetObjectArrayElement(env, cols, i);
  for (jsize i = 0; i < 5 + nc; i++) ptrs[i] = (*env)->GetPrimitiveArrayCritical(env, arrs[i], NULL);
  cep_batch b;
  memset(&b, 0, sizeof b);
  b.n = n;
  b.key_id = (const int32_t*)ptrs[0];
  b.topic = (const int32_t*)ptrs[1];
  b.partition = (const int32_t*)ptrs[2];
  b.offset = (const int64_t*)ptrs[3];
  b.ts = (const int64_t*)ptrs[4];
  b.n_cols = nc;
  b.mem = CEP_MEM_HOST;
  b.cols = (const void* const*)(ptrs + 5);
  b.flags = (uint32_t)flags;
  /* cep_push_batch borrows host columns only for the call (it copies them into the session's pinned
     staging ring before it returns), so the arrays are released -- and the JVM's GC unblocked --
     before the batch's device work is waited for */
  int rc = cep_push_batch(S(session), &b, NULL);
  for (jsize i = 5 + nc - 1; i >= 0; i--) (*env)->ReleasePrimitiveArrayCritical(env, arrs[i], ptrs[i], JNI_ABORT);
  for (jsize i = 0; i < nc; i++) (*env)->DeleteLocalRef(env, arrs[5 + i]);
  if (rc == CEP_OK) {
    cep_matches m;
    rc = cep_collect(S(session), &m);      /* waits; the CSR stays library-owned until the next push, and */
  }                                        /* cepCollect's cep_collect calls return it without device work */
  return rc;
}

/* sizes[0..1] = (n_matches, n_entries); the CSR arrays may be NULL to size them first */
JNIEXPORT jlong JNICALL CLS(cepCollect)(JNIEnv* env, jclass c, jlong session, jlongArray sizes,
                                        jlongArray match_record, jintArray match_key, jlongArray ent_off,
                                        jintArray ent_name, jlongArray ent_record) {
  cep_matches m;
  int rc = cep_collect(S(session), &m);
  if (rc) return -(jlong)rc;
  jlong sz[2] = {m.n_matches, m.n_entries};
  (*env)->SetLongArrayRegion(env, sizes, 0, 2, sz);
  if (match_record) {
    (*env)->SetLongArrayRegion(env, match_record, 0, (jsize)m.n_matches, (const jlong*)m.match_record);
    (*env)->SetIntArrayRegion(env, match_key, 0, (jsize)m.n_matches, (const jint*)m.match_key);
    (*env)->SetLongArrayRegion(env, ent_off, 0, (jsize)m.n_matches + 1, (const jlong*)m.ent_off);
    (*env)->SetIntArrayRegion(env, ent_name, 0, (jsize)m.n_entries, (const jint*)m.ent_name);
    (*env)->SetLongArrayRegion(env, ent_record, 0, (jsize)m.n_entries, (const jlong*)m.ent_record);
  }
  return m.err ? -(jlong)m.err : (jlong)m.n_matches;
}

JNIEXPORT jlongArray JNICALL CLS(cepBatchErrors)(JNIEnv* env, jclass c, jlong session) {
  int64_t n = 0;
  if (cep_batch_errors(S(session), NULL, NULL, 0, &n)) return NULL;
  int64_t* rec = malloc(sizeof(int64_t) * (size_t)(n ? n : 1));
  int32_t* code = malloc(sizeof(int32_t) * (size_t)(n ? n : 1));
  jlongArray out = NULL;
  if (rec && code && cep_batch_errors(S(session), rec, code, n, &n) == CEP_OK) {
    out = (*env)->NewLongArray(env, (jsize)(2 * n));
    for (int64_t i = 0; i < n; i++) {
      jlong pair[2] = {rec[i], code[i]};
      (*env)->SetLongArrayRegion(env, out, (jsize)(2 * i), 2, pair);
    }
  }
  free(rec);
  free(code);
  return out;
}

JNIEXPORT jlong JNICALL CLS(cepStreamPosition)(JNIEnv* env, jclass c, jlong session) {
  return (jlong)cep_stream_position(S(session));
}

JNIEXPORT jbyteArray JNICALL CLS(cepStateExport)(JNIEnv* env, jclass c, jlong session, jint lo, jint hi) {
  size_t need = 0;
  if (cep_state_export(S(session), lo, hi, NULL, 0, &need)) return NULL;
  jbyteArray out = (*env)->NewByteArray(env, (jsize)need);
  jbyte* p = (*env)->GetByteArrayElements(env, out, NULL);
  int rc = cep_state_export(S(session), lo, hi, p, need, &need);
  (*env)->ReleaseByteArrayElements(env, out, p, 0);
  return rc ? NULL : out;
}

JNIEXPORT jint JNICALL CLS(cepStateImport)(JNIEnv* env, jclass c, jlong session, jbyteArray state) {
  jsize n = (*env)->GetArrayLength(env, state);
  jbyte* p = (*env)->GetByteArrayElements(env, state, NULL);
  int rc = cep_state_import(S(session), p, (size_t)n);
  (*env)->ReleaseByteArrayElements(env, state, p, JNI_ABORT);
  return rc;
}

/* per key: its single-key blob (empty if it had no state); the keys' ids are free afterwards */
JNIEXPORT jobjectArray JNICALL CLS(cepStateEvict)(JNIEnv* env, jclass c, jlong session, jintArray keys) {
  const jsize n = (*env)->GetArrayLength(env, keys);
  int64_t* offs = malloc(sizeof(int64_t) * (size_t)(n + 1));
  jint* k = (*env)->GetIntArrayElements(env, keys, NULL);
  const uint8_t* blobs = NULL;
  int rc = offs ? cep_state_evict(S(session), (const int32_t*)k, n, &blobs, offs) : CEP_E_ARG;
  (*env)->ReleaseIntArrayElements(env, keys, k, JNI_ABORT);
  jobjectArray out = NULL;
  if (rc == CEP_OK) {
    out = (*env)->NewObjectArray(env, n, (*env)->FindClass(env, "[B"), NULL);
    for (jsize i = 0; i < n; i++) {
      const jsize len = (jsize)(offs[i + 1] - offs[i]);
      jbyteArray b = (*env)->NewByteArray(env, len);
      (*env)->SetByteArrayRegion(env, b, 0, len, (const jbyte*)(blobs + offs[i]));
      (*env)->SetObjectArrayElement(env, out, i, b);
      (*env)->DeleteLocalRef(env, b);      /* one live local ref per key would overflow the frame */
    }
  }
  free(offs);
  return out;
}

JNIEXPORT jint JNICALL CLS(cepStateImportKeys)(JNIEnv* env, jclass c, jlong session, jobjectArray blobs,
                                               jintArray keys) {
  const jsize n = (*env)->GetArrayLength(env, keys);
  if ((*env)->GetArrayLength(env, blobs) != n) return CEP_E_ARG;
  /* the blobs are copied into one buffer, each element's local ref dropped at once (a spill re-admits
     up to maxKeys / 8 keys: one live ref per key would overflow the JNI local frame) */
  size_t* lens = malloc(sizeof(size_t) * (size_t)(n ? n : 1));
  size_t* offs = malloc(sizeof(size_t) * (size_t)(n + 1));
  const void** ptrs = malloc(sizeof(void*) * (size_t)(n ? n : 1));
  if (!lens || !offs || !ptrs) { free(lens); free(offs); free((void*)ptrs); return CEP_E_ARG; }
  offs[0] = 0;
  for (jsize i = 0; i < n; i++) {
    jbyteArray a = (jbyteArray)(*env)->GetObjectArrayElement(env, blobs, i);
    lens[i] = (size_t)(*env)->GetArrayLength(env, a);
    offs[i + 1] = offs[i] + lens[i];
    (*env)->DeleteLocalRef(env, a);
  }
  uint8_t* all = malloc(offs[n] ? offs[n] : 1);
  if (!all) { free(lens); free(offs); free((void*)ptrs); return CEP_E_ARG; }
  for (jsize i = 0; i < n; i++) {
    jbyteArray a = (jbyteArray)(*env)->GetObjectArrayElement(env, blobs, i);
    (*env)->GetByteArrayRegion(env, a, 0, (jsize)lens[i], (jbyte*)(all + offs[i]));
    (*env)->DeleteLocalRef(env, a);
    ptrs[i] = all + offs[i];
  }
  jint* k = (*env)->GetIntArrayElements(env, keys, NULL);
  int rc = cep_state_import_keys(S(session), ptrs, lens, (const int32_t*)k, n);
  (*env)->ReleaseIntArrayElements(env, keys, k, JNI_ABORT);
  free(all); free(lens); free(offs); free((void*)ptrs);
  return rc;
}

JNIEXPORT jlongArray JNICALL CLS(cepStatePositions)(JNIEnv* env, jclass c, jbyteArray blob) {
  const jsize len = (*env)->GetArrayLength(env, blob);
  jbyte* p = (*env)->GetByteArrayElements(env, blob, NULL);
  int64_t n = 0;
  jlongArray out = NULL;
  if (cep_state_positions(p, (size_t)len, NULL, 0, &n) == CEP_OK) {
    int64_t* pos = malloc(sizeof(int64_t) * (size_t)(n ? n : 1));
    if (pos && cep_state_positions(p, (size_t)len, pos, n, &n) == CEP_OK) {
      out = (*env)->NewLongArray(env, (jsize)n);
      (*env)->SetLongArrayRegion(env, out, 0, (jsize)n, (const jlong*)pos);
    }
    free(pos);
  }
  (*env)->ReleaseByteArrayElements(env, blob, p, JNI_ABORT);
  return out;
}

JNIEXPORT jint JNICALL CLS(cepSetMaxKeyWords)(JNIEnv* env, jclass c, jlong session, jlong words) {
  return cep_session_set_max_key_words(S(session), words);
}

JNIEXPORT void JNICALL CLS(cepSessionClose)(JNIEnv* env, jclass c, jlong session) { cep_session_close(S(session)); }

JNIEXPORT void JNICALL CLS(cepPatternFree)(JNIEnv* env, jclass c, jlong pattern) {
  cep_pattern_free((cep_pattern*)(intptr_t)pattern);
}

JNIEXPORT jstring JNICALL CLS(cepLastError)(JNIEnv* env, jclass c) { return (*env)->NewStringUTF(env, cep_last_error()); }

/* ---- PatternIR (java/com/github/fhuss/kafka/streams/cep/pattern/PatternIR.java): the reference DSL
   lowered through the IR builder of kcep.h (cep_irb_*).  Strings travel as UTF-8 byte[] (null for a
   null Java string), so the IR carries the bytes String.getBytes(UTF_8) gives, not JNI's modified
   UTF-8; every call returns a kcep status code. ---- */
#define IRB(name) Java_com_github_fhuss_kafka_streams_cep_pattern_PatternIR_##name

static cep_irb* B(jlong h) { return (cep_irb*)(intptr_t)h; }

/* a NUL-terminated copy of a UTF-8 byte[] (NULL for null); free() it */
static char* utf8(JNIEnv* env, jbyteArray a) {
  if (!a) return NULL;
  const jsize n = (*env)->GetArrayLength(env, a);
  char* s = malloc((size_t)n + 1);
  if (!s) return NULL;
  (*env)->GetByteArrayRegion(env, a, 0, n, (jbyte*)s);
  s[n] = 0;
  return s;
}

JNIEXPORT jlong JNICALL IRB(irbNew)(JNIEnv* env, jclass c, jintArray col_types) {
  const jsize n = (*env)->GetArrayLength(env, col_types);
  jint* t = (*env)->GetIntArrayElements(env, col_types, NULL);
  cep_irb* b = NULL;
  int rc = cep_irb_new((const int32_t*)t, n, &b);
  (*env)->ReleaseIntArrayElements(env, col_types, t, JNI_ABORT);
  return rc ? -(jlong)rc : (jlong)(intptr_t)b;
}

JNIEXPORT void JNICALL IRB(irbFree)(JNIEnv* env, jclass c, jlong b) { cep_irb_free(B(b)); }

JNIEXPORT jint JNICALL IRB(irbTopic)(JNIEnv* env, jclass c, jlong b, jbyteArray topic) {
  char* t = utf8(env, topic);
  jint id = t ? cep_irb_topic(B(b), t) : -CEP_E_ARG;
  free(t);
  return id;
}

JNIEXPORT jint JNICALL IRB(irbSelect)(JNIEnv* env, jclass c, jlong b, jbyteArray name, jint level, jint strategy,
                                      jbyteArray topic) {
  char* n = utf8(env, name);
  char* t = utf8(env, topic);
  jint rc = cep_irb_select(B(b), n, level, strategy, t);
  free(n);
  free(t);
  return rc;
}

JNIEXPORT jint JNICALL IRB(irbQuantifier)(JNIEnv* env, jclass c, jlong b, jint one_or_more, jint optional, jint times) {
  return cep_irb_quantifier(B(b), one_or_more, optional, times);
}

JNIEXPORT jint JNICALL IRB(irbWithin)(JNIEnv* env, jclass c, jlong b, jlong ms) { return cep_irb_within(B(b), ms); }

JNIEXPORT jint JNICALL IRB(irbConst)(JNIEnv* env, jclass c, jlong b, jint type, jlong i, jdouble d) {
  return cep_irb_const(B(b), type, i, d);
}

JNIEXPORT jint JNICALL IRB(irbField)(JNIEnv* env, jclass c, jlong b, jint col) { return cep_irb_field(B(b), col); }

JNIEXPORT jint JNICALL IRB(irbEvent)(JNIEnv* env, jclass c, jlong b, jint what) { return cep_irb_event(B(b), what); }

JNIEXPORT jint JNICALL IRB(irbTopicEq)(JNIEnv* env, jclass c, jlong b, jbyteArray topic) {
  char* t = utf8(env, topic);
  jint rc = cep_irb_topic_eq(B(b), t);
  free(t);
  return rc;
}

JNIEXPORT jint JNICALL IRB(irbState)(JNIEnv* env, jclass c, jlong b, jbyteArray name, jint type, jint or_else) {
  char* n = utf8(env, name);
  jint rc = cep_irb_state(B(b), n, type, or_else);
  free(n);
  return rc;
}

JNIEXPORT jint JNICALL IRB(irbCurr)(JNIEnv* env, jclass c, jlong b, jint type) { return cep_irb_curr(B(b), type); }

JNIEXPORT jint JNICALL IRB(irbSeq)(JNIEnv* env, jclass c, jlong b, jint kind, jint col, jbyteArray stage) {
  char* s = utf8(env, stage);
  jint rc = cep_irb_seq(B(b), kind, col, s);
  free(s);
  return rc;
}

JNIEXPORT jint JNICALL IRB(irbOp)(JNIEnv* env, jclass c, jlong b, jint op) { return cep_irb_op(B(b), op); }

JNIEXPORT jint JNICALL IRB(irbCast)(JNIEnv* env, jclass c, jlong b, jint type) { return cep_irb_cast(B(b), type); }

JNIEXPORT jint JNICALL IRB(irbWhere)(JNIEnv* env, jclass c, jlong b, jint conj) { return cep_irb_where(B(b), conj); }

JNIEXPORT jint JNICALL IRB(irbFold)(JNIEnv* env, jclass c, jlong b, jbyteArray state, jint type) {
  char* s = utf8(env, state);
  jint rc = cep_irb_fold(B(b), s, type);
  free(s);
  return rc;
}

JNIEXPORT jbyteArray JNICALL IRB(irbFinish)(JNIEnv* env, jclass c, jlong b) {
  size_t need = 0;
  if (cep_irb_finish(B(b), NULL, 0, &need)) return NULL;
  uint8_t* buf = malloc(need ? need : 1);
  jbyteArray out = NULL;
  if (buf && cep_irb_finish(B(b), buf, need, &need) == CEP_OK) {
    out = (*env)->NewByteArray(env, (jsize)need);
    (*env)->SetByteArrayRegion(env, out, 0, (jsize)need, (const jbyte*)buf);
  }
  free(buf);
  return out;
}

/* the ids the builder gave the topics it met, in id order: the processor's topic ids must agree */
JNIEXPORT jobjectArray JNICALL IRB(irbTopics)(JNIEnv* env, jclass c, jlong b) {
  const int32_t n = cep_irb_topic_count(B(b));
  if (n < 0) return NULL;
  jobjectArray out = (*env)->NewObjectArray(env, n, (*env)->FindClass(env, "java/lang/String"), NULL);
  for (int32_t i = 0; i < n; i++) {
    jstring s = (*env)->NewStringUTF(env, cep_irb_topic_name(B(b), i));
    (*env)->SetObjectArrayElement(env, out, i, s);
    (*env)->DeleteLocalRef(env, s);
  }
  return out;
}

/* cep_compile + cep_pattern_check(CEP_SESSION_CARRY): 0 if a GpuCEPProcessor can run the IR, else the
   status (CEP_E_INVALID_PATTERN, CEP_E_UNSUPPORTED, CEP_E_BAD_IR) with the reason in irbLastError */
JNIEXPORT jint JNICALL IRB(irbProbe)(JNIEnv* env, jclass c, jbyteArray ir) {
  const jsize n = (*env)->GetArrayLength(env, ir);
  jbyte* p = (*env)->GetByteArrayElements(env, ir, NULL);
  cep_pattern* pat = NULL;
  int rc = cep_compile((const uint8_t*)p, (size_t)n, &pat);
  (*env)->ReleaseByteArrayElements(env, ir, p, JNI_ABORT);
  if (rc == CEP_OK) {
    rc = cep_pattern_check(pat, CEP_SESSION_CARRY);
    cep_pattern_free(pat);
  }
  return rc;
}

JNIEXPORT jstring JNICALL IRB(irbLastError)(JNIEnv* env, jclass c) { return (*env)->NewStringUTF(env, cep_last_error()); }

/* ---- GpuCEPProcessor: a key that outgrew the device, in the reference's own terms (KCRF) ---- */
JNIEXPORT jbyteArray JNICALL CLS(cepStateToReference)(JNIEnv* env, jclass c, jlong pattern, jbyteArray blob) {
  const jsize n = (*env)->GetArrayLength(env, blob);
  jbyte* p = (*env)->GetByteArrayElements(env, blob, NULL);
  size_t need = 0;
  jbyteArray out = NULL;
  const cep_pattern* pat = (const cep_pattern*)(intptr_t)pattern;
  if (cep_state_to_reference(pat, p, (size_t)n, NULL, 0, &need) == CEP_OK) {
    uint8_t* buf = malloc(need ? need : 1);
    if (buf && cep_state_to_reference(pat, p, (size_t)n, buf, need, &need) == CEP_OK) {
      out = (*env)->NewByteArray(env, (jsize)need);
      (*env)->SetByteArrayRegion(env, out, 0, (jsize)need, (const jbyte*)buf);
    }
    free(buf);
  }
  (*env)->ReleaseByteArrayElements(env, blob, p, JNI_ABORT);
  return out;
}
