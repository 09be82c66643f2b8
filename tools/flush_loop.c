/* flush_loop.c -- the processor-flush loop of tools/flush_probe.py in C: per batch one cep_push_batch
 * from host memory and one cep_collect, the CSR copied out as the JNI shim copies it into Java arrays.
 * It times the C-ABI alone (no Python in the loop).  Built by flush_probe.py with gcc. */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "../include/kcep.h"

static double now_us(void) {
  struct timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return t.tv_sec * 1e6 + t.tv_nsec * 1e-3;
}

static size_t copy_out(const cep_matches* m, char** sink, size_t* cap) {
  const size_t need = (size_t)m->n_matches * 20 + (size_t)m->n_entries * 12 + 8;
  if (need > *cap) {
    free(*sink);
    *cap = need * 2;
    *sink = (char*)malloc(*cap);
  }
  char* p = *sink;
  memcpy(p, m->match_record, (size_t)m->n_matches * 8); p += m->n_matches * 8;
  memcpy(p, m->match_key, (size_t)m->n_matches * 4); p += m->n_matches * 4;
  memcpy(p, m->ent_off, (size_t)(m->n_matches + 1) * 8); p += (m->n_matches + 1) * 8;
  memcpy(p, m->ent_name, (size_t)m->n_entries * 4); p += m->n_entries * 4;
  memcpy(p, m->ent_record, (size_t)m->n_entries * 8);
  return need;
}

/* Pipelined: batch i + 1 is pushed before batch i is collected (cep_collect_batch).
 * out: [total us, push us, collect us, matches] */
int flush_loop_pipelined(cep_session* s, int64_t nb, int64_t per, const int32_t* key, const int32_t* val,
                         uint32_t flags, void* stream, double* out) {
  double tp = 0, tc = 0;
  int64_t nm = 0, prev = -1;
  size_t cap = 0;
  char* sink = NULL;
  const double t00 = now_us();
  for (int64_t i = 0; i <= nb; i++) {
    const double t0 = now_us();
    if (i < nb) {
      const void* cols[1] = {val + i * per};
      cep_batch b;
      memset(&b, 0, sizeof b);
      b.n = per;
      b.key_id = key + i * per;
      b.n_cols = 1;
      b.mem = CEP_MEM_HOST;
      b.cols = cols;
      b.flags = flags;
      int rc = cep_push_batch(s, &b, stream);
      if (rc) return rc;
    }
    const double t1 = now_us();
    if (prev >= 0) {
      cep_matches m;
      int rc = cep_collect_batch(s, prev, &m);
      if (rc) return rc;
      copy_out(&m, &sink, &cap);
      nm += m.n_matches;
    }
    prev = i < nb ? cep_batch_id(s) : -1;
    const double t2 = now_us();
    tp += t1 - t0;
    tc += t2 - t1;
  }
  out[0] = now_us() - t00;
  out[1] = tp;
  out[2] = tc;
  out[3] = (double)nm;
  free(sink);
  return 0;
}

/* out: [total us, push us, collect us, matches] */
int flush_loop(cep_session* s, int64_t nb, int64_t per, const int32_t* key, const int32_t* val, uint32_t flags,
               void* stream, double* out) {
  double tp = 0, tc = 0;
  int64_t nm = 0;
  size_t cap = 0;
  char* sink = NULL;
  const double t00 = now_us();
  for (int64_t i = 0; i < nb; i++) {
    const void* cols[1] = {val + i * per};
    cep_batch b;
    memset(&b, 0, sizeof b);
    b.n = per;
    b.key_id = key + i * per;
    b.n_cols = 1;
    b.mem = CEP_MEM_HOST;
    b.cols = cols;
    b.flags = flags;
    const double t0 = now_us();
    int rc = cep_push_batch(s, &b, stream);
    if (rc) return rc;
    const double t1 = now_us();
    cep_matches m;
    rc = cep_collect(s, &m);
    if (rc) return rc;
    copy_out(&m, &sink, &cap);
    const double t2 = now_us();
    tp += t1 - t0;
    tc += t2 - t1;
    nm += m.n_matches;
  }
  out[0] = now_us() - t00;
  out[1] = tp;
  out[2] = tc;
  out[3] = (double)nm;
  free(sink);
  return 0;
}
