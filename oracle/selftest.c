/* selftest.c -- host-side sanitizer driver for the CPU oracle (test
 * infrastructure, SURVEY.md section 5 "race detection / sanitizers").
 *
 * Built twice by oracle/Makefile (selftest-asan: -fsanitize=address,undefined;
 * selftest-tsan: -fsanitize=thread) and run by tests/test_oracle_sanitizers.py.
 * It drives every oracle entry the parity tests lean on over seeded random
 * data, checks their invariants, and runs the threaded pipelines (the
 * bench's cpu_baseline, pthread Shard over all threads) against their
 * single-thread results, so a data race or an out-of-bounds access in the
 * checker shows up here instead of as a wrong "reference" answer.
 * Exit 0 = all checks passed. */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

typedef struct orc_ev orc_ev;
int64_t orc_unique(const int64_t* x, int64_t n, int64_t* y, int32_t* idx, int32_t* counts);
orc_ev* orc_ev_create(int64_t dim, const float* default_row, int64_t filter_freq,
                      int64_t steps_to_live, int64_t max_element_size,
                      float false_positive_probability, int counter_bits);
orc_ev* orc_ev_create_slot(orc_ev* primary, int slot_index, const float* default_row);
void orc_ev_free(orc_ev* ev);
int orc_ev_gather(orc_ev* ev, const int64_t* keys, int64_t n, const float* defaults,
                  const int32_t* counts, float* out);
int orc_ev_import(orc_ev* ev, const int64_t* keys, int64_t n, const float* values,
                  const int64_t* versions, const int64_t* freqs, int64_t bucket_num,
                  int64_t partition_id, int64_t partition_num);
int64_t orc_ev_size(orc_ev* ev);
int64_t orc_ev_export(orc_ev* ev, int64_t* keys, float* values, int64_t* versions,
                      int64_t* freqs);
int orc_ev_apply_sgd(orc_ev* var, float lr, const float* grad, const int64_t* keys, int64_t n,
                     int64_t gs);
int orc_ev_apply_adagrad(orc_ev* var, orc_ev* accum, float lr, const float* grad,
                         const int64_t* keys, int64_t n, int64_t gs);
int orc_sparse_segment_reduce(const float* data, int64_t data_rows, int64_t D,
                              const int32_t* idx, const int32_t* seg, int64_t n,
                              int64_t num_segments, int combiner, float* out, int64_t* out_rows);
int orc_unsorted_segment_sum(const float* data, int64_t n, int64_t D, const int32_t* seg,
                             int64_t num_segments, float* out);
int orc_pipeline_ev_lookup_sparse(orc_ev* ev, const int64_t* ids, int64_t nnz,
                                  const int32_t* seg_off, int64_t B, int combiner, int threads,
                                  float* out);
int orc_pipeline_dense_lookup_sparse(const float* table, int64_t D, const int64_t* ids,
                                     int64_t nnz, const int32_t* seg_off, int64_t B, int combiner,
                                     int threads, float* out);
typedef struct orc_pool orc_pool;
orc_pool* orc_pool_create(int threads);
void orc_pool_free(orc_pool* pl);
int64_t orc_unique_parallel(orc_pool* pool, const int64_t* x, int64_t n, int64_t* y,
                            int32_t* idx);
int orc_pipeline_ev_lookup_sparse_pool(orc_pool* pool, orc_ev* ev, const int64_t* ids,
                                       int64_t nnz, const int32_t* seg_off, int64_t B,
                                       int combiner, int serial_unique, float* out);

static uint64_t rs = 0x9E3779B97F4A7C15ULL;
static uint64_t rnd(void) {
  rs ^= rs << 13;
  rs ^= rs >> 7;
  rs ^= rs << 17;
  return rs;
}
static float frnd(void) { return (float)((rnd() >> 40) & 0xFFFFFF) / 16777216.0f - 0.5f; }

static int fails = 0;
#define CHECK(c, ...)                             \
  do {                                            \
    if (!(c)) {                                   \
      fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__); \
      fprintf(stderr, __VA_ARGS__);               \
      fprintf(stderr, "\n");                      \
      ++fails;                                    \
    }                                             \
  } while (0)

static void test_unique(void) {
  const int64_t n = 20000;
  int64_t* x = malloc(sizeof(int64_t) * n);
  int64_t* y = malloc(sizeof(int64_t) * n);
  int32_t* idx = malloc(sizeof(int32_t) * n);
  int32_t* cnt = malloc(sizeof(int32_t) * n);
  for (int64_t i = 0; i < n; ++i) x[i] = (int64_t)(rnd() % 3000) - 1000;  /* negatives too */
  const int64_t U = orc_unique(x, n, y, idx, cnt);
  int64_t tot = 0;
  for (int64_t i = 0; i < n; ++i) {
    CHECK(idx[i] >= 0 && idx[i] < U && y[idx[i]] == x[i], "unique idx at %lld", (long long)i);
  }
  for (int64_t u = 0; u < U; ++u) tot += cnt[u];
  CHECK(tot == n, "unique counts sum %lld", (long long)tot);
  /* first-occurrence order: the first position of y[u] is increasing in u */
  int64_t* first = malloc(sizeof(int64_t) * U);
  for (int64_t u = 0; u < U; ++u) first[u] = -1;
  for (int64_t i = 0; i < n; ++i)
    if (first[idx[i]] < 0) first[idx[i]] = i;
  for (int64_t u = 1; u < U; ++u) CHECK(first[u] > first[u - 1], "unique order at %lld", (long long)u);
  free(first);
  /* the parallel Unique (four threaded steps) gives the serial result */
  int64_t* y2 = malloc(sizeof(int64_t) * n);
  int32_t* idx2 = malloc(sizeof(int32_t) * n);
  for (int th = 1; th <= 8; th += 3) {
    orc_pool* pl = orc_pool_create(th);
    const int64_t U2 = orc_unique_parallel(pl, x, n, y2, idx2);
    CHECK(U2 == U && memcmp(y, y2, sizeof(int64_t) * U) == 0 &&
              memcmp(idx, idx2, sizeof(int32_t) * n) == 0,
          "parallel unique, %d threads", th);
    orc_pool_free(pl);
  }
  free(y2);
  free(idx2);
  free(x);
  free(y);
  free(idx);
  free(cnt);
}

static void test_ev_and_pipelines(void) {
  const int64_t D = 16, K = 5000, B = 4096;
  float dflt[16];
  for (int j = 0; j < D; ++j) dflt[j] = 0.25f * (float)j;
  orc_ev* ev = orc_ev_create(D, dflt, 0, 0, 0, -1.0f, 64);
  orc_ev* acc = orc_ev_create_slot(ev, 1, dflt);
  int64_t* keys = malloc(sizeof(int64_t) * K);
  float* vals = malloc(sizeof(float) * K * D);
  for (int64_t i = 0; i < K; ++i) {
    keys[i] = (int64_t)(rnd() >> 20);
    for (int j = 0; j < D; ++j) vals[i * D + j] = frnd();
  }
  CHECK(orc_ev_import(ev, keys, K, vals, NULL, NULL, 1000, 0, 1) == 0, "import");
  const int64_t sz = orc_ev_size(ev);
  CHECK(sz <= K && sz > K / 2, "size %lld", (long long)sz);
  /* multi-hot bags over imported and new keys */
  int32_t* off = malloc(sizeof(int32_t) * (B + 1));
  off[0] = 0;
  for (int64_t b = 0; b < B; ++b) off[b + 1] = off[b] + (int32_t)(rnd() % 5);
  const int64_t nnz = off[B];
  int64_t* ids = malloc(sizeof(int64_t) * (nnz ? nnz : 1));
  for (int64_t i = 0; i < nnz; ++i) ids[i] = (rnd() & 1) ? keys[rnd() % K] : (int64_t)(rnd() >> 20);
  /* the pipeline reads rows without creating: create every id first */
  float* tmp = malloc(sizeof(float) * (nnz ? nnz : 1) * D);
  CHECK(orc_ev_gather(ev, ids, nnz, NULL, NULL, tmp) == 0, "gather");
  for (int comb = 0; comb < 3; ++comb) {
    float* o1 = malloc(sizeof(float) * B * D);
    float* o8 = malloc(sizeof(float) * B * D);
    orc_pipeline_ev_lookup_sparse(ev, ids, nnz, off, B, comb, 1, o1);
    orc_pipeline_ev_lookup_sparse(ev, ids, nnz, off, B, comb, 8, o8);
    CHECK(memcmp(o1, o8, sizeof(float) * B * D) == 0, "ev pipeline threads, combiner %d", comb);
    for (int serial = 0; serial < 2; ++serial) {   /* the pooled pipeline, both Uniques */
      orc_pool* pl = orc_pool_create(6);
      orc_pipeline_ev_lookup_sparse_pool(pl, ev, ids, nnz, off, B, comb, serial, o8);
      CHECK(memcmp(o1, o8, sizeof(float) * B * D) == 0, "pooled pipeline, combiner %d", comb);
      orc_pool_free(pl);
    }
    free(o1);
    free(o8);
  }
  /* dense pipeline */
  const int64_t R = 7000;
  float* table = malloc(sizeof(float) * R * D);
  for (int64_t i = 0; i < R * D; ++i) table[i] = frnd();
  int64_t* dids = malloc(sizeof(int64_t) * (nnz ? nnz : 1));
  for (int64_t i = 0; i < nnz; ++i) dids[i] = (int64_t)(rnd() % R);
  {
    float* o1 = malloc(sizeof(float) * B * D);
    float* o8 = malloc(sizeof(float) * B * D);
    orc_pipeline_dense_lookup_sparse(table, D, dids, nnz, off, B, 1, 1, o1);
    orc_pipeline_dense_lookup_sparse(table, D, dids, nnz, off, B, 1, 8, o8);
    CHECK(memcmp(o1, o8, sizeof(float) * B * D) == 0, "dense pipeline threads");
    free(o1);
    free(o8);
  }
  /* segment reductions and the unsorted sum over the same bags */
  {
    int64_t* uq = malloc(sizeof(int64_t) * (nnz ? nnz : 1));
    int32_t* idx = malloc(sizeof(int32_t) * (nnz ? nnz : 1));
    int32_t* seg = malloc(sizeof(int32_t) * (nnz ? nnz : 1));
    const int64_t U = orc_unique(dids, nnz, uq, idx, NULL);
    float* emb = malloc(sizeof(float) * (U ? U : 1) * D);
    for (int64_t u = 0; u < U; ++u) memcpy(emb + u * D, table + uq[u] * D, sizeof(float) * D);
    for (int64_t b = 0; b < B; ++b)
      for (int32_t i = off[b]; i < off[b + 1]; ++i) seg[i] = (int32_t)b;
    float* out = malloc(sizeof(float) * B * D);
    int64_t rows = 0;
    CHECK(orc_sparse_segment_reduce(emb, U, D, idx, seg, nnz, B, 0, out, &rows) == 0, "ssr");
    float* us = malloc(sizeof(float) * B * D);
    float* pos = malloc(sizeof(float) * (nnz ? nnz : 1) * D);
    for (int64_t i = 0; i < nnz; ++i) memcpy(pos + i * D, emb + idx[i] * D, sizeof(float) * D);
    CHECK(orc_unsorted_segment_sum(pos, nnz, D, seg, B, us) == 0, "uss");
    for (int64_t i = 0; i < B * D; ++i)
      CHECK(fabsf(us[i] - out[i]) <= 1e-4f * (1.0f + fabsf(out[i])), "ssr vs uss at %lld",
            (long long)i);
    free(uq);
    free(idx);
    free(seg);
    free(emb);
    free(out);
    free(us);
    free(pos);
  }
  /* optimizer steps on distinct keys */
  {
    int64_t* uq = malloc(sizeof(int64_t) * (nnz ? nnz : 1));
    int32_t* idx = malloc(sizeof(int32_t) * (nnz ? nnz : 1));
    const int64_t U = orc_unique(ids, nnz, uq, idx, NULL);
    float* g = malloc(sizeof(float) * (U ? U : 1) * D);
    for (int64_t i = 0; i < U * D; ++i) g[i] = frnd();
    CHECK(orc_ev_apply_sgd(ev, 0.1f, g, uq, U, 1) == 0, "sgd");
    CHECK(orc_ev_apply_adagrad(ev, acc, 0.1f, g, uq, U, 2) == 0, "adagrad");
    int64_t* ek = malloc(sizeof(int64_t) * (orc_ev_size(ev) + 1));
    float* evv = malloc(sizeof(float) * (orc_ev_size(ev) + 1) * D);
    const int64_t m = orc_ev_export(ev, ek, evv, NULL, NULL);
    CHECK(m >= U, "export %lld < %lld", (long long)m, (long long)U);
    for (int64_t i = 0; i < m * D; ++i) CHECK(isfinite(evv[i]), "export value %lld", (long long)i);
    free(uq);
    free(idx);
    free(g);
    free(ek);
    free(evv);
  }
  free(table);
  free(dids);
  free(tmp);
  free(ids);
  free(off);
  free(keys);
  free(vals);
  orc_ev_free(acc);
  orc_ev_free(ev);
}

int main(void) {
  test_unique();
  test_ev_and_pipelines();
  if (fails) {
    fprintf(stderr, "%d check(s) failed\n", fails);
    return 1;
  }
  printf("oracle selftest ok\n");
  return 0;
}
