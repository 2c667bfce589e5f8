/*
 * deeprec_oracle.c -- CPU restatement of DeepRec's CPU EmbeddingVariable hot
 * path.  TEST INFRASTRUCTURE ONLY: it is the parity checker for the HIP
 * engine and the timed "cpu_baseline" leg of bench.py (kind "port").  Nothing
 * in the shipped engine (deeprec-1_amd/) may link, load or call this file.
 *
 * Parity pinning: the reference (a TensorFlow 1.15 fork built with Bazel and
 * network-fetched deps) cannot be compiled or imported in this container
 * (SURVEY.md section 8c), so this restatement is pinned against the
 * reference's own golden vectors / KATs committed under tests/golden/
 * (fused_embedding_local_ops_test.cc, segment_reduction_ali_ops_test.cc,
 * fused_embedding_ops_test.cc, embedding_variable_ops_test.py).
 *
 * Every function cites the reference file:line whose semantics it restates
 * (paths relative to the reference root).  Association order of fp32 sums is
 * replayed exactly where the reference fixes it, so the HIP engine can be
 * checked bit-exactly.
 *
 * Build: see oracle/Makefile (gcc -O2 -ffp-contract=off -fPIC -shared -pthread).
 */
#include <math.h>
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define ORC_OK 0
#define ORC_INVALID_ARGUMENT 3
#define ORC_NOT_FOUND 5
#define ORC_RESOURCE_EXHAUSTED 8

/* ------------------------------------------------------------------------ */
/* Unique with first-occurrence order.                                       */
/* unique_ali_op_util.h:192-222 (SerialComputeV1): y[j] = j-th distinct key  */
/* in order of first appearance, idx[i] = position of x[i] in y.  Counts are */
/* UniqueWithCounts (unique_ali_op.cc:137-180).                              */
/* ------------------------------------------------------------------------ */
static uint64_t orc_mix64(uint64_t k) {
  k ^= k >> 33; k *= 0xff51afd7ed558ccdULL;
  k ^= k >> 33; k *= 0xc4ceb9fe1a85ec53ULL;
  k ^= k >> 33;
  return k;
}

int64_t orc_unique(const int64_t* x, int64_t n, int64_t* y, int32_t* idx,
                   int32_t* counts) {
  if (n <= 0) return 0;
  int64_t cap = 16;
  while (cap < 2 * n) cap <<= 1;
  int64_t* slot = (int64_t*)malloc(sizeof(int64_t) * cap); /* -> y index */
  for (int64_t s = 0; s < cap; ++s) slot[s] = -1;
  int64_t u = 0;
  for (int64_t i = 0; i < n; ++i) {
    uint64_t h = orc_mix64((uint64_t)x[i]) & (uint64_t)(cap - 1);
    for (;;) {
      int64_t j = slot[h];
      if (j < 0) {
        slot[h] = u;
        y[u] = x[i];
        if (counts) counts[u] = 0;
        j = u++;
      }
      if (y[j] == x[i]) {
        idx[i] = (int32_t)j;
        if (counts) counts[j] += 1;
        break;
      }
      h = (h + 1) & (uint64_t)(cap - 1);
    }
  }
  free(slot);
  return u;
}

/* ------------------------------------------------------------------------ */
/* SparseSegment{Sum,Mean,SqrtN}[WithNumSegments], CPU ali kernel.           */
/* segment_reduction_ali_ops_util.h:30-177 (Reduce driver) and :193-318      */
/* (row reducer).  Association order per output row, num = bag length:      */
/*   num == 1 : out = L0                                                     */
/*   else     : r = num % 8 (0 -> 8, 1 -> 9);                                 */
/*              out = (((L0 + L1) + L2) ... + L_{r-1}) / m                   */
/*              (m = num, sqrt(num) for mean/sqrtn when num < 10, else 1)     */
/*              then for each further group of 8:                            */
/*              out += (((L_r + L_{r+1}) + ...) + L_{r+7})                   */
/*              then out /= num (or sqrt(num)) when num >= 10.               */
/* Missing segments are filled with 0 (default_value).                       */
/* combiner: 0 sum, 1 mean, 2 sqrtn.                                          */
/* ------------------------------------------------------------------------ */
static void orc_reduce_bag(const float* data, int64_t D, const int32_t* idx,
                           int64_t start, int64_t num, int combiner,
                           float* out) {
  if (num == 1) {
    memcpy(out, data + (int64_t)idx[start] * D, sizeof(float) * D);
    return;
  }
  int64_t r = num % 8;
  if (r == 0) r = 8;
  if (r == 1) r = 9;
  float m = 1.0f;
  if (combiner == 1 && num < 10) m = (float)num;
  if (combiner == 2 && num < 10) m = (float)sqrt((double)num);
  for (int64_t d = 0; d < D; ++d) {
    float s = data[(int64_t)idx[start] * D + d];
    for (int64_t k = 1; k < r; ++k) s = s + data[(int64_t)idx[start + k] * D + d];
    out[d] = s / m;
  }
  for (int64_t g = r; g < num; g += 8) {
    for (int64_t d = 0; d < D; ++d) {
      float s = data[(int64_t)idx[start + g] * D + d];
      for (int64_t k = 1; k < 8; ++k) s = s + data[(int64_t)idx[start + g + k] * D + d];
      out[d] = out[d] + s;
    }
  }
  if (num >= 10) {
    float q = 1.0f;
    if (combiner == 1) q = (float)num;
    if (combiner == 2) q = (float)sqrt((double)num);
    if (combiner != 0)
      for (int64_t d = 0; d < D; ++d) out[d] = out[d] / q;
  }
}

int orc_sparse_segment_reduce(const float* data, int64_t data_rows, int64_t D,
                              const int32_t* idx, const int32_t* seg, int64_t n,
                              int64_t num_segments, int combiner, float* out,
                              int64_t* out_rows) {
  int64_t last_plus_one = n > 0 ? (int64_t)seg[n - 1] + 1 : 0;
  int64_t rows = num_segments >= 0 ? num_segments : last_plus_one;
  if (num_segments >= 0 && rows < last_plus_one) return ORC_INVALID_ARGUMENT;
  if (out_rows) *out_rows = rows;
  if (!out) return ORC_OK;
  memset(out, 0, sizeof(float) * rows * D);
  int64_t start = 0;
  while (start < n) {
    int32_t s = seg[start];
    if (s < 0 || s >= rows) return ORC_INVALID_ARGUMENT;
    int64_t end = start + 1;
    while (end < n && seg[end] == s) ++end;
    if (end < n && seg[end] < s) return ORC_INVALID_ARGUMENT; /* not increasing */
    for (int64_t k = start; k < end; ++k)
      if (idx[k] < 0 || idx[k] >= data_rows) return ORC_INVALID_ARGUMENT;
    orc_reduce_bag(data, D, idx, start, end - start, combiner, out + (int64_t)s * D);
    start = end;
  }
  return ORC_OK;
}

/* ------------------------------------------------------------------------ */
/* SparseSegment{Mean,SqrtN}Grad CPU: segment_reduction_ali_ops_util.h:331-458 */
/* out[idx[i]] (=|+=) grad[seg[i]] * scale, i ascending, scale =             */
/* float(1/double(cnt)) or float(1/sqrt(double(cnt))); cnt==1 -> no scale.    */
/* is_sqrtn: 0 mean, 1 sqrtn.  (Sum grad = unsorted_segment_sum of the        */
/* gathered grad, math_grad.py:321-327; see orc_sparse_segment_sum_grad.)    */
/* ------------------------------------------------------------------------ */
int orc_sparse_segment_reduce_grad(const float* grad, int64_t grad_rows,
                                   int64_t D, const int32_t* idx,
                                   const int32_t* seg, int64_t n,
                                   int64_t out_rows, int is_sqrtn, float* out) {
  memset(out, 0, sizeof(float) * out_rows * D);
  if (out_rows == 0 || n == 0) return ORC_OK;
  if ((int64_t)seg[n - 1] + 1 > grad_rows) return ORC_INVALID_ARGUMENT;
  int32_t* cnt = (int32_t*)calloc((size_t)n, sizeof(int32_t));
  unsigned char* touched = (unsigned char*)calloc((size_t)out_rows, 1);
  int64_t start = 0;
  while (start < n) {
    int64_t end = start + 1;
    while (end < n && seg[end] == seg[start]) ++end;
    if (seg[start] < 0 || seg[start] >= grad_rows) { free(cnt); free(touched); return ORC_INVALID_ARGUMENT; }
    for (int64_t k = start; k < end; ++k) cnt[k] = (int32_t)(end - start);
    start = end;
  }
  for (int64_t i = 0; i < n; ++i) {
    int32_t o = idx[i];
    if (o < 0 || o >= out_rows) { free(cnt); free(touched); return ORC_INVALID_ARGUMENT; }
    const float* g = grad + (int64_t)seg[i] * D;
    float* dst = out + (int64_t)o * D;
    if (cnt[i] == 1) {
      if (touched[o]) for (int64_t d = 0; d < D; ++d) dst[d] = dst[d] + g[d];
      else memcpy(dst, g, sizeof(float) * D);
    } else {
      float scale = is_sqrtn ? (float)(1.0 / sqrt((double)cnt[i]))
                             : (float)(1.0 / (double)cnt[i]);
      if (touched[o]) for (int64_t d = 0; d < D; ++d) { float p = g[d] * scale; dst[d] = dst[d] + p; }
      else for (int64_t d = 0; d < D; ++d) dst[d] = g[d] * scale;
    }
    touched[o] = 1;
  }
  free(cnt);
  free(touched);
  return ORC_OK;
}

/* ------------------------------------------------------------------------ */
/* UnsortedSegmentSum CPU: segment_reduction_ops.cc:377-405.  out = 0, then  */
/* out[seg[i]] += data[i] for i ascending; seg < 0 is skipped.               */
/* ------------------------------------------------------------------------ */
int orc_unsorted_segment_sum(const float* data, int64_t n, int64_t D,
                             const int32_t* seg, int64_t num_segments,
                             float* out) {
  memset(out, 0, sizeof(float) * num_segments * D);
  for (int64_t i = 0; i < n; ++i) {
    int32_t j = seg[i];
    if (j < 0) continue;
    if (j >= num_segments) return ORC_INVALID_ARGUMENT;
    for (int64_t d = 0; d < D; ++d) out[(int64_t)j * D + d] = out[(int64_t)j * D + d] + data[i * D + d];
  }
  return ORC_OK;
}

/* Sum grad: unsorted_segment_sum(gather(grad, seg), idx, U)                 */
/* (python/ops/math_grad.py:321-327), fused without materialising the gather. */
int orc_sparse_segment_sum_grad(const float* grad, int64_t grad_rows, int64_t D,
                                const int32_t* idx, const int32_t* seg,
                                int64_t n, int64_t out_rows, float* out) {
  memset(out, 0, sizeof(float) * out_rows * D);
  for (int64_t i = 0; i < n; ++i) {
    int32_t j = idx[i];
    if (j < 0) continue;
    if (j >= out_rows || seg[i] < 0 || seg[i] >= grad_rows) return ORC_INVALID_ARGUMENT;
    for (int64_t d = 0; d < D; ++d)
      out[(int64_t)j * D + d] = out[(int64_t)j * D + d] + grad[(int64_t)seg[i] * D + d];
  }
  return ORC_OK;
}

/* Weighted path of embedding_lookup_sparse (embedding_ops.py:609-651):      */
/* gather(emb, idx) * w then SegmentSum; mean divides by the segment sum of  */
/* weights, sqrtn by sqrt(segment sum of w^2).  Sequential left-to-right sum  */
/* (the reference's Eigen reduction order is not pinned: tolerance-checked). */
int orc_weighted_segment_reduce(const float* emb, int64_t D, const int32_t* idx,
                                const float* w, const int32_t* seg, int64_t n,
                                int64_t num_segments, int combiner, float* out) {
  memset(out, 0, sizeof(float) * num_segments * D);
  float* wsum = (float*)calloc((size_t)(num_segments > 0 ? num_segments : 1), sizeof(float));
  for (int64_t i = 0; i < n; ++i) {
    int32_t s = seg[i];
    if (s < 0 || s >= num_segments) { free(wsum); return ORC_INVALID_ARGUMENT; }
    float wi = w[i];
    for (int64_t d = 0; d < D; ++d) {
      float p = emb[(int64_t)idx[i] * D + d] * wi;
      out[(int64_t)s * D + d] = out[(int64_t)s * D + d] + p;
    }
    wsum[s] = wsum[s] + (combiner == 2 ? wi * wi : wi);
  }
  if (combiner != 0) {
    for (int64_t s = 0; s < num_segments; ++s) {
      float q = combiner == 2 ? sqrtf(wsum[s]) : wsum[s];
      for (int64_t d = 0; d < D; ++d) out[s * D + d] = out[s * D + d] / q;
    }
  }
  free(wsum);
  return ORC_OK;
}

/* ------------------------------------------------------------------------ */
/* Dense-table gather (GatherFunctorCPU / HandleCopies, gather_functor.h:36- */
/* 115): out[i] = table[idx[i]]; an out-of-range index is an error.          */
/* ------------------------------------------------------------------------ */
int orc_gather(const float* table, int64_t rows, int64_t D, const int64_t* idx,
               int64_t n, float* out) {
  for (int64_t i = 0; i < n; ++i) {
    if (idx[i] < 0 || idx[i] >= rows) return ORC_INVALID_ARGUMENT;
    memcpy(out + i * D, table + idx[i] * D, sizeof(float) * D);
  }
  return ORC_OK;
}

/* clip_by_norm as used by embedding_ops._clip (embedding_ops.py:42-91 ->    */
/* clip_ops.clip_by_norm): x * max_norm / max(l2norm, max_norm).             */
void orc_clip_rows(float* rows, int64_t n, int64_t D, float max_norm) {
  for (int64_t i = 0; i < n; ++i) {
    float* r = rows + i * D;
    float l2sum = 0.0f;
    for (int64_t d = 0; d < D; ++d) l2sum = l2sum + r[d] * r[d];
    float l2norm = l2sum > 0.0f ? sqrtf(l2sum) : l2sum;
    float den = l2norm > max_norm ? l2norm : max_norm;
    for (int64_t d = 0; d < D; ++d) { float t = r[d] * max_norm; r[d] = t / den; }
  }
}

/* ------------------------------------------------------------------------ */
/* FusedEmbeddingLocalSparseLookUp (fused_embedding_local_ops_gpu.cu.cc:41-84 */
/* + combiner fused_embedding_common.cu.h:11-53): per bag, sequential sum of */
/* rows (each clipped by max_norm/l2 when max_norm >= 0 and l2 > max_norm),  */
/* then sqrtn: /sqrtf(n), mean: /n.  offsets = first nnz of each bag.         */
/* Bags are given by row ids (sp_indices[:,0]) sorted ascending.             */
/* ------------------------------------------------------------------------ */
int orc_fused_local_lookup(const float* table, int64_t rows, int64_t D,
                           const int64_t* values, const int64_t* row_ids,
                           int64_t nnz, int64_t batch, int combiner,
                           float max_norm, float* out, int32_t* offsets) {
  for (int64_t b = 0; b < batch; ++b) offsets[b] = 0x7fffffff;
  for (int64_t i = nnz - 1; i >= 0; --i) {
    if (row_ids[i] < 0 || row_ids[i] >= batch) return ORC_INVALID_ARGUMENT;
    offsets[row_ids[i]] = (int32_t)i;
  }
  float* e = (float*)malloc(sizeof(float) * (D > 0 ? D : 1));
  for (int64_t b = 0; b < batch; ++b) {
    int64_t off = offsets[b];
    int64_t cnt = (b == batch - 1 ? nnz : offsets[b + 1]) - off;
    for (int64_t d = 0; d < D; ++d) out[b * D + d] = 0.0f;
    for (int64_t k = 0; k < cnt; ++k) {
      int64_t v = values[off + k];
      if (v < 0 || v >= rows) { free(e); return ORC_INVALID_ARGUMENT; }
      memcpy(e, table + v * D, sizeof(float) * D);
      if (max_norm >= 0.0f) {
        float l2 = 0.0f;
        for (int64_t d = 0; d < D; ++d) l2 = l2 + e[d] * e[d];
        l2 = sqrtf(l2);
        if (l2 > max_norm) for (int64_t d = 0; d < D; ++d) e[d] = e[d] * (max_norm / l2);
      }
      for (int64_t d = 0; d < D; ++d) out[b * D + d] = out[b * D + d] + e[d];
    }
    for (int64_t d = 0; d < D; ++d) {
      if (combiner == 2) out[b * D + d] = out[b * D + d] / sqrtf((float)cnt);
      else if (combiner == 1) out[b * D + d] = out[b * D + d] / (float)cnt;
    }
  }
  free(e);
  return ORC_OK;
}

/* FusedEmbeddingLocalSparseLookUpGrad (fused_embedding_local_ops_gpu.cu.cc: */
/* 86-122): grad[nnz,D], row k of bag b = top_grad[b] combined (/sqrtf(n),   */
/* /n), scaled by max_norm/l2 when max_norm > 0 and l2 > max_norm.           */
int orc_fused_local_lookup_grad(const float* top_grad, const float* table,
                                int64_t rows, int64_t D, const int64_t* values,
                                const int32_t* offsets, int64_t nnz,
                                int64_t batch, int combiner, float max_norm,
                                float* grad_out) {
  for (int64_t b = 0; b < batch; ++b) {
    int64_t off = offsets[b];
    int64_t cnt = (b == batch - 1 ? nnz : offsets[b + 1]) - off;
    for (int64_t k = 0; k < cnt; ++k) {
      int64_t v = values[off + k];
      if (v < 0 || v >= rows) return ORC_INVALID_ARGUMENT;
      float scale_clip = 1.0f;
      int clip = 0;
      if (max_norm > 0.0f) {
        float l2 = 0.0f;
        for (int64_t d = 0; d < D; ++d) l2 = l2 + table[v * D + d] * table[v * D + d];
        l2 = sqrtf(l2);
        if (l2 > max_norm) { clip = 1; scale_clip = max_norm / l2; }
      }
      for (int64_t d = 0; d < D; ++d) {
        float g = top_grad[b * D + d];
        if (combiner == 2) g = g / sqrtf((float)cnt);
        else if (combiner == 1) g = g / (float)cnt;
        if (clip) g = g * scale_clip;
        grad_out[(off + k) * D + d] = g;
      }
    }
  }
  return ORC_OK;
}

/* Stable ascending order of int64 keys (bottom-up merge sort): order[] =   */
/* positions.                                                                */
static void stable_order(const int64_t* keys, int64_t n, int64_t* order) {
  for (int64_t i = 0; i < n; ++i) order[i] = i;
  int64_t* tmp = (int64_t*)malloc(sizeof(int64_t) * (n > 0 ? n : 1));
  for (int64_t w = 1; w < n; w *= 2) {
    for (int64_t lo = 0; lo < n; lo += 2 * w) {
      int64_t mid = lo + w < n ? lo + w : n;
      int64_t hi = lo + 2 * w < n ? lo + 2 * w : n;
      int64_t a = lo, b = mid, o = lo;
      while (a < mid && b < hi) tmp[o++] = (keys[order[b]] < keys[order[a]]) ? order[b++] : order[a++];
      while (a < mid) tmp[o++] = order[a++];
      while (b < hi) tmp[o++] = order[b++];
    }
    memcpy(order, tmp, sizeof(int64_t) * n);
  }
  free(tmp);
}

/* FusedEmbeddingSparsePostLookUp (fused_embedding_ops_gpus.cu.cc:285-384):  */
/* entries = the partitions' (emb row, (row, col)) pairs back to back.  Per  */
/* bag: out = 0; out += e (e *= max_norm / l2 when max_norm >= 0 and l2 >    */
/* max_norm, SumUpEmbeddingShard :72-99) over the bag's entries; then        */
/* ApplyCombiner (:101-107): / sqrtf(n), / n.  The reference's float atomics */
/* leave the order open; this restatement fixes it to ascending (row, col),  */
/* the order the engine uses (and FusedEmbeddingLocalSparseLookUp's).       */
int orc_fused_post_lookup(const float* emb, const int64_t* ind, int64_t N, int64_t B,
                          int64_t cols, int64_t D, int combiner, float max_norm, float* out,
                          int32_t* fnum) {
  int64_t* key = (int64_t*)malloc(sizeof(int64_t) * (N > 0 ? N : 1));
  int64_t* order = (int64_t*)malloc(sizeof(int64_t) * (N > 0 ? N : 1));
  float* e = (float*)malloc(sizeof(float) * (D > 0 ? D : 1));
  for (int64_t i = 0; i < N; ++i) {
    if (ind[2 * i] < 0 || ind[2 * i] >= B || ind[2 * i + 1] < 0 || ind[2 * i + 1] >= cols) {
      free(key); free(order); free(e);
      return ORC_INVALID_ARGUMENT;
    }
    key[i] = ind[2 * i] * cols + ind[2 * i + 1];
  }
  stable_order(key, N, order);
  for (int64_t i = 0; i < B * D; ++i) out[i] = 0.0f;
  for (int64_t b = 0; b < B; ++b) fnum[b] = 0;
  for (int64_t j = 0; j < N; ++j) {
    const int64_t s = order[j], b = ind[2 * s];
    for (int64_t d = 0; d < D; ++d) e[d] = emb[s * D + d];
    if (max_norm >= 0.0f) {
      float l2 = 0.0f;
      for (int64_t d = 0; d < D; ++d) l2 = l2 + e[d] * e[d];
      l2 = sqrtf(l2);
      if (l2 > max_norm) {
        const float f = max_norm / l2;
        for (int64_t d = 0; d < D; ++d) e[d] = e[d] * f;
      }
    }
    for (int64_t d = 0; d < D; ++d) out[b * D + d] = out[b * D + d] + e[d];
    fnum[b] += 1;
  }
  if (combiner != 0)
    for (int64_t b = 0; b < B; ++b) {
      const float q = combiner == 2 ? sqrtf((float)fnum[b]) : (float)fnum[b];
      for (int64_t d = 0; d < D; ++d) out[b * D + d] = out[b * D + d] / q;
    }
  free(key); free(order); free(e);
  return ORC_OK;
}

/* FusedEmbeddingSparsePostLookUpGrad, DistributeGradToShard (fused_embedding */
/* _ops_gpus.cu.cc:109-146): grad[e] = CombineGrad(top[row(e)], fnum[row])   */
/* then *= max_norm / l2(emb[e]) when max_norm >= 0 and l2 > max_norm.       */
int orc_fused_post_lookup_grad(const float* top, const float* emb, const int64_t* ind,
                               int64_t N, int64_t B, int64_t D, const int32_t* fnum,
                               int combiner, float max_norm, float* out) {
  for (int64_t i = 0; i < N; ++i) {
    const int64_t b = ind[2 * i];
    if (b < 0 || b >= B) return ORC_INVALID_ARGUMENT;
    float f = 1.0f;
    int clip = 0;
    if (max_norm >= 0.0f) {
      float l2 = 0.0f;
      for (int64_t d = 0; d < D; ++d) l2 = l2 + emb[i * D + d] * emb[i * D + d];
      l2 = sqrtf(l2);
      if (l2 > max_norm) { clip = 1; f = max_norm / l2; }
    }
    for (int64_t d = 0; d < D; ++d) {
      float g = top[b * D + d];
      if (combiner == 2) g = g / sqrtf((float)fnum[b]);
      else if (combiner == 1) g = g / (float)fnum[b];
      if (clip) g = g * f;
      out[i * D + d] = g;
    }
  }
  return ORC_OK;
}

/* Backward of the weighted embedding_lookup_sparse composition            */
/* (python/ops/embedding_ops.py:609-651) w.r.t. the unique rows: TF's        */
/* gradient chain div (RealDiv: g / weight_sum) -> segment_sum (gather by    */
/* seg) -> mul (* w) -> gather (IndexedSlices over idx) -> the dense         */
/* conversion, an UnsortedSegmentSum in ascending position from 0.           */
/* weight_sum = segment_sum(w) (mean) or sqrt(segment_sum(pow(w, 2)))        */
/* (sqrtn), accumulated from 0 in ascending position.                        */
int orc_weighted_segment_grad(const float* g, int64_t B, int64_t D, const int32_t* idx,
                              const float* w, const int32_t* seg, int64_t n, int64_t U,
                              int combiner, float* out) {
  float* q = (float*)calloc((size_t)(B > 0 ? B : 1), sizeof(float));
  for (int64_t i = 0; i < n; ++i) {
    if (seg[i] < 0 || seg[i] >= B || idx[i] < 0 || idx[i] >= U) { free(q); return ORC_INVALID_ARGUMENT; }
    q[seg[i]] = q[seg[i]] + (combiner == 2 ? w[i] * w[i] : w[i]);
  }
  if (combiner == 2)
    for (int64_t b = 0; b < B; ++b) q[b] = sqrtf(q[b]);
  memset(out, 0, sizeof(float) * U * D);
  for (int64_t i = 0; i < n; ++i) {
    const int64_t b = seg[i], u = idx[i];
    for (int64_t d = 0; d < D; ++d) {
      float t = g[b * D + d];
      if (combiner != 0) t = t / q[b];
      t = t * w[i];
      out[u * D + d] = out[u * D + d] + t;
    }
  }
  free(q);
  return ORC_OK;
}

/* Backward of clip_by_norm (clip_ops.py:164-184, applied by embedding_ops. */
/* _clip to the looked-up rows) by TF's chain rule op by op, in place on g:  */
/* l2sum = sum v*v; pred = l2sum > 0; l2 = pred ? sqrt(l2sum) : l2sum;       */
/* m = max(l2, c); gm = sum_d g * ((-(v*c)) / m) / m (RealDiv grad of y);   */
/* Maximum passes gm to l2 when l2 >= c; Sqrt: gs = (0.5 * gl2) / l2;        */
/* g' = (g / m) * c + gs * v + v * gs (the three uses of `values`).          */
void orc_clip_by_norm_grad(const float* v, float* g, int64_t n, int64_t D, float c) {
  for (int64_t i = 0; i < n; ++i) {
    const float* r = v + i * D;
    float* gr = g + i * D;
    float s = 0.0f;
    for (int64_t d = 0; d < D; ++d) s = s + r[d] * r[d];
    const int pred = s > 0.0f;
    const float l2 = pred ? sqrtf(s) : s;
    const float m = l2 > c ? l2 : c;
    float gm = 0.0f;
    for (int64_t d = 0; d < D; ++d) gm = gm + gr[d] * ((-(r[d] * c) / m) / m);
    const float gl2 = l2 >= c ? gm : 0.0f;
    const float gs = pred ? (0.5f * gl2) / l2 : 0.0f;
    for (int64_t d = 0; d < D; ++d) {
      const float a = (gr[d] / m) * c, b = gs * r[d];
      gr[d] = (a + b) + b;
    }
  }
}

/* FusedEmbeddingSparsePreLookUp partition step (fused_embedding_ops_gpus.  */
/* cu.cc:158-310, "div" over partition_shapes): ids are stably sorted, then  */
/* split by the cumulative row ranges of the partitions and rebased.  Writes */
/* out_values (rebased ids) / out_pos (original nnz position) in partition   */
/* order and part_sizes[num_partitions].                                      */
int orc_fused_pre_lookup(const int64_t* values, int64_t nnz,
                         const int64_t* part_rows, int64_t num_parts,
                         int64_t* out_values, int64_t* out_pos,
                         int64_t* part_sizes) {
  int64_t* order = (int64_t*)malloc(sizeof(int64_t) * (nnz > 0 ? nnz : 1));
  for (int64_t i = 0; i < nnz; ++i) order[i] = i;
  /* stable insertion/merge sort by id */
  for (int64_t w = 1; w < nnz; w *= 2) {
    int64_t* tmp = (int64_t*)malloc(sizeof(int64_t) * nnz);
    for (int64_t lo = 0; lo < nnz; lo += 2 * w) {
      int64_t mid = lo + w < nnz ? lo + w : nnz;
      int64_t hi = lo + 2 * w < nnz ? lo + 2 * w : nnz;
      int64_t a = lo, b = mid, o = lo;
      while (a < mid && b < hi) tmp[o++] = (values[order[b]] < values[order[a]]) ? order[b++] : order[a++];
      while (a < mid) tmp[o++] = order[a++];
      while (b < hi) tmp[o++] = order[b++];
    }
    memcpy(order, tmp, sizeof(int64_t) * nnz);
    free(tmp);
  }
  int64_t base = 0, k = 0;
  for (int64_t p = 0; p < num_parts; ++p) {
    int64_t lim = base + part_rows[p];
    int64_t c = 0;
    while (k < nnz && values[order[k]] < lim) {
      if (values[order[k]] < base) { free(order); return ORC_INVALID_ARGUMENT; }
      out_values[k] = values[order[k]] - base;
      out_pos[k] = order[k];
      ++k; ++c;
    }
    part_sizes[p] = c;
    base = lim;
  }
  free(order);
  return k == nnz ? ORC_OK : ORC_INVALID_ARGUMENT;
}

/* ------------------------------------------------------------------------ */
/* EmbeddingVariable.                                                        */
/*  - key -> ValuePtr map shared by primary and slot EVs                     */
/*    (kernels/kv_variable_ops.cc:232-238, embedding_var.h:320-339)          */
/*  - per key: version, freq, one row per emb_index allocated on first touch */
/*    by copying the caller's default (value_ptr.h:145-170)                  */
/*  - filters: Nullable / Counter / Bloom (embedding_filter.h:27-396)        */
/* ------------------------------------------------------------------------ */
#define ORC_MAX_COLS 8

typedef struct {
  int64_t key;
  int64_t version;
  int64_t freq;
  float* rows[ORC_MAX_COLS];
} orc_entry;

typedef struct {
  int64_t cap;       /* hash slots, power of two */
  int64_t* slot;     /* -> entry index, -1 empty */
  orc_entry* ent;
  int64_t n_ent, ent_cap;
  int refs;
} orc_map;

typedef struct {
  orc_map* map;
  int64_t dim;
  int emb_index;
  int primary;
  float* default_value;
  int64_t filter_freq, steps_to_live;
  /* bloom */
  int64_t k_hash, num_counter;
  int counter_bits;
  void* bloom;
  int64_t seeds[64];
  /* bf16 EV (build-defined, DESIGN "bf16 EVs"): the primary's values are */
  /* bf16; each apply computes in fp32 on the widened values and rounds    */
  /* the updated row once to nearest even.  Slots stay fp32.               */
  int bf16;
} orc_ev;

/* fp32 -> bf16 (round to nearest even, NaN -> 0x7FC0) -> fp32 */
float orc_bf16_round(float f) {
  uint32_t u;
  memcpy(&u, &f, 4);
  if ((u & 0x7FFFFFFFu) > 0x7F800000u) {
    u = 0x7FC00000u;
  } else {
    u += 0x7FFFu + ((u >> 16) & 1u);
    u &= 0xFFFF0000u;
  }
  memcpy(&f, &u, 4);
  return f;
}

static void orc_bf16_row(const orc_ev* ev, float* v) {
  if (!ev->bf16) return;
  for (int64_t d = 0; d < ev->dim; ++d) v[d] = orc_bf16_round(v[d]);
}

/* Make a primary EV a bf16 EV: its default row is rounded now, every later */
/* apply rounds the updated rows.                                            */
void orc_ev_set_bf16(orc_ev* ev) {
  ev->bf16 = 1;
  orc_bf16_row(ev, ev->default_value);
}

static orc_map* orc_map_new(void) {
  orc_map* m = (orc_map*)calloc(1, sizeof(orc_map));
  m->cap = 1024;
  m->slot = (int64_t*)malloc(sizeof(int64_t) * m->cap);
  for (int64_t i = 0; i < m->cap; ++i) m->slot[i] = -1;
  m->ent_cap = 512;
  m->ent = (orc_entry*)calloc((size_t)m->ent_cap, sizeof(orc_entry));
  m->refs = 1;
  return m;
}

static int64_t orc_map_find(orc_map* m, int64_t key) {
  uint64_t h = orc_mix64((uint64_t)key) & (uint64_t)(m->cap - 1);
  for (;;) {
    int64_t e = m->slot[h];
    if (e < 0) return -1;
    if (m->ent[e].key == key) return e;
    h = (h + 1) & (uint64_t)(m->cap - 1);
  }
}

static void orc_map_grow(orc_map* m) {
  int64_t ncap = m->cap * 2;
  int64_t* ns = (int64_t*)malloc(sizeof(int64_t) * ncap);
  for (int64_t i = 0; i < ncap; ++i) ns[i] = -1;
  for (int64_t e = 0; e < m->n_ent; ++e) {
    if (m->ent[e].key == INT64_MIN && m->ent[e].version == INT64_MIN) continue; /* removed */
    uint64_t h = orc_mix64((uint64_t)m->ent[e].key) & (uint64_t)(ncap - 1);
    while (ns[h] >= 0) h = (h + 1) & (uint64_t)(ncap - 1);
    ns[h] = e;
  }
  free(m->slot);
  m->slot = ns;
  m->cap = ncap;
}

/* LookupOrCreateKeyInternal (embedding_var.h:320-339) */
static int64_t orc_map_lookup_or_create(orc_map* m, int64_t key) {
  int64_t e = orc_map_find(m, key);
  if (e >= 0) return e;
  if (2 * (m->n_ent + 1) > m->cap) orc_map_grow(m);
  if (m->n_ent == m->ent_cap) {
    m->ent_cap *= 2;
    m->ent = (orc_entry*)realloc(m->ent, sizeof(orc_entry) * m->ent_cap);
  }
  e = m->n_ent++;
  memset(&m->ent[e], 0, sizeof(orc_entry));
  m->ent[e].key = key;
  uint64_t h = orc_mix64((uint64_t)key) & (uint64_t)(m->cap - 1);
  while (m->slot[h] >= 0) h = (h + 1) & (uint64_t)(m->cap - 1);
  m->slot[h] = e;
  return e;
}

/* BloomFilter::GenerateSeed (embedding_filter.h:252-279) */
static void orc_bloom_seeds(orc_ev* ev) {
  static const int64_t defaults[25] = {2, 3, 5, 7, 11, 13, 17, 19, 23, 29, 31, 37, 41,
                                       43, 47, 53, 59, 61, 67, 71, 73, 79, 83, 89, 97};
  int64_t k = ev->k_hash > 64 ? 64 : ev->k_hash;
  if (k < 25) {
    for (int64_t i = 0; i < k; ++i) ev->seeds[i] = defaults[i];
  } else {
    for (int64_t i = 0; i < 25; ++i) ev->seeds[i] = defaults[i];
    int64_t last = 98;
    for (int64_t i = 25; i < k; ++i) {
      for (int64_t j = last;; ++j) {
        if (j % 2 == 0) continue;
        int prime = 1;
        /* the reference loop starts at k = 0 (j % 0 is UB); effectively it  */
        /* tests divisors 2..sqrt(j)+1 -- restated that way.                 */
        for (int64_t q = 2; q <= (int64_t)sqrt((double)j) + 1; ++q)
          if (j % q == 0) { prime = 0; break; }
        if (prime) { ev->seeds[i] = j; last = j; break; }
      }
    }
  }
}

/* BloomFilter::FastHash64 (embedding_filter.h:134-148) */
uint64_t orc_fasthash64(int64_t key, uint64_t seed) {
  const uint64_t m = 0x880355f21e6d1965ULL;
  uint64_t h = seed ^ (8 * m);
  uint64_t v = (uint64_t)key;
  v ^= v >> 23; v *= 0x2127599bf4325c37ULL; v ^= v >> 47;
  h ^= v; h *= m;
  v = 0;
  v ^= v >> 23; v *= 0x2127599bf4325c37ULL; v ^= v >> 47;
  h ^= v; h *= m;
  h ^= h >> 23; h *= 0x2127599bf4325c37ULL; h ^= h >> 47;
  return h;
}

static uint64_t orc_bloom_get(orc_ev* ev, int64_t c) {
  switch (ev->counter_bits) {
    case 8: return ((uint8_t*)ev->bloom)[c];
    case 16: return ((uint16_t*)ev->bloom)[c];
    case 32: return ((uint32_t*)ev->bloom)[c];
    default: return ((uint64_t*)ev->bloom)[c];
  }
}
static void orc_bloom_add(orc_ev* ev, int64_t c, int64_t count) {
  switch (ev->counter_bits) {
    case 8: ((uint8_t*)ev->bloom)[c] += (uint8_t)count; break;
    case 16: ((uint16_t*)ev->bloom)[c] += (uint16_t)count; break;
    case 32: ((uint32_t*)ev->bloom)[c] += (uint32_t)count; break;
    default: ((uint64_t*)ev->bloom)[c] += (uint64_t)count; break;
  }
}
/* GetBloomFreq (embedding_filter.h:103-127): min over the k counters */
int64_t orc_bloom_freq(orc_ev* ev, int64_t key) {
  uint64_t mn = 0;
  for (int64_t i = 0; i < ev->k_hash; ++i) {
    int64_t c = (int64_t)(orc_fasthash64(key, (uint64_t)ev->seeds[i]) % (uint64_t)ev->num_counter);
    uint64_t v = orc_bloom_get(ev, c);
    if (i == 0 || v < mn) mn = v;
  }
  return (int64_t)mn;
}
/* AddFreq (embedding_filter.h:190-250): each counter below filter_freq += count */
static void orc_bloom_addfreq(orc_ev* ev, int64_t key, int64_t count) {
  for (int64_t i = 0; i < ev->k_hash; ++i) {
    int64_t c = (int64_t)(orc_fasthash64(key, (uint64_t)ev->seeds[i]) % (uint64_t)ev->num_counter);
    if ((int64_t)orc_bloom_get(ev, c) < ev->filter_freq) orc_bloom_add(ev, c, count);
  }
}

/* EmbeddingConfig::calc_num_hash_func / calc_num_counter (embedding_config.h:63-70) */
static void orc_bloom_params(int64_t max_element_size, float fpp, int64_t* k, int64_t* nc) {
  float loghpp = fabsf((float)(log(fpp) / log(2)));
  *k = (int64_t)ceil(loghpp);
  float loghpp2 = fabsf((float)log(fpp));
  float factor = (float)(log(2) * log(2));
  *nc = (int64_t)ceil(loghpp2 / factor * max_element_size);
}

/* InitializeKvVariableOp primary branch (kernels/kv_variable_ops.cc:173-193). */
orc_ev* orc_ev_create(int64_t dim, const float* default_row, int64_t filter_freq,
                      int64_t steps_to_live, int64_t max_element_size,
                      float false_positive_probability, int counter_bits) {
  orc_ev* ev = (orc_ev*)calloc(1, sizeof(orc_ev));
  ev->map = orc_map_new();
  ev->dim = dim;
  ev->emb_index = 0;
  ev->primary = 1;
  ev->default_value = (float*)malloc(sizeof(float) * dim);
  memcpy(ev->default_value, default_row, sizeof(float) * dim);
  ev->filter_freq = filter_freq < 0 ? 0 : filter_freq;
  ev->steps_to_live = steps_to_live;
  if (ev->filter_freq > 0 && max_element_size != 0 && false_positive_probability != -1.0f) {
    orc_bloom_params(max_element_size, false_positive_probability, &ev->k_hash, &ev->num_counter);
    ev->counter_bits = counter_bits ? counter_bits : 64;
    ev->bloom = calloc((size_t)ev->num_counter, (size_t)(ev->counter_bits / 8));
    orc_bloom_seeds(ev);
  }
  return ev;
}

/* Slot EV sharing the primary's key map (kernels/kv_variable_ops.cc:212-226): */
/* emb_index = slot_index (block_num == 1), no filter of its own.             */
orc_ev* orc_ev_create_slot(orc_ev* primary, int slot_index, const float* default_row) {
  if (slot_index <= 0 || slot_index >= ORC_MAX_COLS) return NULL;
  orc_ev* ev = (orc_ev*)calloc(1, sizeof(orc_ev));
  ev->map = primary->map;
  ev->map->refs++;
  ev->dim = primary->dim;
  ev->emb_index = slot_index;
  ev->primary = 0;
  ev->default_value = (float*)malloc(sizeof(float) * ev->dim);
  memcpy(ev->default_value, default_row, sizeof(float) * ev->dim);
  ev->steps_to_live = primary->steps_to_live;
  return ev;
}

void orc_ev_free(orc_ev* ev) {
  if (!ev) return;
  if (--ev->map->refs == 0) {
    for (int64_t e = 0; e < ev->map->n_ent; ++e)
      for (int c = 0; c < ORC_MAX_COLS; ++c) free(ev->map->ent[e].rows[c]);
    free(ev->map->ent);
    free(ev->map->slot);
    free(ev->map);
  }
  free(ev->bloom);
  free(ev->default_value);
  free(ev);
}

/* ValuePtr::GetOrAllocate (value_ptr.h:145-170) */
static float* orc_get_or_alloc(orc_ev* ev, int64_t e, const float* default_v) {
  orc_entry* en = &ev->map->ent[e];
  if (!en->rows[ev->emb_index]) {
    en->rows[ev->emb_index] = (float*)malloc(sizeof(float) * ev->dim);
    memcpy(en->rows[ev->emb_index], default_v, sizeof(float) * ev->dim);
  }
  return en->rows[ev->emb_index];
}

/* KvResourceGather / KvResourceGatherV1 (kernels/kv_variable_ops.cc:314-449) */
/* -> EmbeddingVar::LookupOrCreate -> filter_->LookupOrCreate                 */
/* (Nullable :348-353, Counter :296-320, Bloom :56-82).                       */
/* defaults: [n,D] per-index rows, or NULL for the EV's own default_value_.   */
/* counts: NULL for V0 (count 1).                                             */
int orc_ev_gather(orc_ev* ev, const int64_t* keys, int64_t n,
                  const float* defaults, const int32_t* counts, float* out) {
  const int64_t D = ev->dim;
  for (int64_t i = 0; i < n; ++i) {
    const float* dv = defaults ? defaults + i * D : ev->default_value;
    int64_t cnt = counts ? counts[i] : 1;
    if (ev->filter_freq == 0) {                      /* NullableFilter */
      int64_t e = orc_map_lookup_or_create(ev->map, keys[i]);
      memcpy(out + i * D, orc_get_or_alloc(ev, e, dv), sizeof(float) * D);
    } else if (ev->k_hash == 0) {                    /* CounterFilter */
      int64_t e = orc_map_lookup_or_create(ev->map, keys[i]);
      orc_entry* en = &ev->map->ent[e];
      if (en->freq >= ev->filter_freq) {
        memcpy(out + i * D, orc_get_or_alloc(ev, e, dv), sizeof(float) * D);
      } else {
        en->freq += cnt;
        memcpy(out + i * D, dv, sizeof(float) * D);
      }
    } else {                                         /* BloomFilter */
      if (orc_bloom_freq(ev, keys[i]) >= ev->filter_freq) {
        int64_t e = orc_map_lookup_or_create(ev->map, keys[i]);
        memcpy(out + i * D, orc_get_or_alloc(ev, e, dv), sizeof(float) * D);
      } else {
        orc_bloom_addfreq(ev, keys[i], cnt);
        memcpy(out + i * D, dv, sizeof(float) * D);
      }
    }
  }
  return ORC_OK;
}

/* EmbeddingVar::Import (embedding_var.h:187-219), the semantics the build   */
/* gives KvResourceInsert / KvResourceImportV2.  partition_num <= 0 disables */
/* the `key % bucket_num % partition_num == partition_id` filter.            */
int orc_ev_import(orc_ev* ev, const int64_t* keys, int64_t n, const float* values,
                  const int64_t* versions, const int64_t* freqs,
                  int64_t bucket_num, int64_t partition_id, int64_t partition_num) {
  const int64_t D = ev->dim;
  for (int64_t i = 0; i < n; ++i) {
    if (partition_num > 0 && keys[i] % bucket_num % partition_num != partition_id) continue;
    int64_t e = orc_map_lookup_or_create(ev->map, keys[i]);
    orc_entry* en = &ev->map->ent[e];
    if (ev->primary) {
      if (ev->filter_freq != 0) {
        int64_t f = freqs ? freqs[i] : 0;
        en->freq = f <= ev->filter_freq ? ev->filter_freq : f;
      }
      if (ev->steps_to_live != 0) en->version = versions ? versions[i] : 0;
    }
    orc_get_or_alloc(ev, e, values + i * D);
  }
  return ORC_OK;
}

int64_t orc_ev_size(orc_ev* ev) { return ev->map->n_ent; }

/* EmbeddingVar::GetSnapshot (embedding_var.h:221-243) -> KvResourceExport:  */
/* keys whose own row and primary row exist; freqs if filter_freq != 0,      */
/* versions if steps_to_live != 0.  Iteration order of the reference's hash  */
/* map is unpinned; this restatement emits keys in ascending order.          */
int64_t orc_ev_export(orc_ev* ev, int64_t* keys, float* values, int64_t* versions,
                      int64_t* freqs) {
  orc_map* m = ev->map;
  int64_t* order = (int64_t*)malloc(sizeof(int64_t) * (m->n_ent > 0 ? m->n_ent : 1));
  int64_t k = 0;
  for (int64_t e = 0; e < m->n_ent; ++e)
    if (m->ent[e].rows[ev->emb_index] && m->ent[e].rows[0]) order[k++] = e;
  /* insertion sort is fine for test sizes; use qsort-like shell sort */
  for (int64_t gap = k / 2; gap > 0; gap /= 2)
    for (int64_t i = gap; i < k; ++i)
      for (int64_t j = i; j >= gap && m->ent[order[j - gap]].key > m->ent[order[j]].key; j -= gap) {
        int64_t t = order[j]; order[j] = order[j - gap]; order[j - gap] = t;
      }
  for (int64_t i = 0; i < k; ++i) {
    orc_entry* en = &m->ent[order[i]];
    if (keys) keys[i] = en->key;
    if (values) memcpy(values + i * ev->dim, en->rows[ev->emb_index], sizeof(float) * ev->dim);
    if (versions) versions[i] = en->version;
    if (freqs) freqs[i] = ev->k_hash ? orc_bloom_freq(ev, en->key) : en->freq;
  }
  free(order);
  return k;
}

int64_t orc_ev_freq(orc_ev* ev, int64_t key) {
  if (ev->k_hash) return orc_bloom_freq(ev, key);
  int64_t e = orc_map_find(ev->map, key);
  return e < 0 ? 0 : ev->map->ent[e].freq;
}
int64_t orc_ev_version(orc_ev* ev, int64_t key) {
  int64_t e = orc_map_find(ev->map, key);
  return e < 0 ? -1 : ev->map->ent[e].version;
}
int orc_ev_has_row(orc_ev* ev, int64_t key) {
  int64_t e = orc_map_find(ev->map, key);
  return e >= 0 && ev->map->ent[e].rows[ev->emb_index] != NULL;
}

/* filter_->LookupOrCreateKey with update_version (embedding_var.h:109-121,  */
/* embedding_filter.h:322-326,355-359,84-93).  Returns the entry or -1 when  */
/* filtered (is_filter == false).                                             */
static int64_t orc_apply_key(orc_ev* var, int64_t key, int64_t gs) {
  if (var->k_hash) {
    if (orc_bloom_freq(var, key) < var->filter_freq) return -1;
  }
  int64_t e = orc_map_lookup_or_create(var->map, key);
  if (var->primary && var->steps_to_live != 0 && gs != -1) var->map->ent[e].version = gs;
  if (!var->k_hash && var->filter_freq > 0 && var->map->ent[e].freq < var->filter_freq) return -1;
  return e;
}

/* KvResourceSparseApplyGradientDescent (training_ali_ops.cc:1597-1678):     */
/* v -= lr * g                                                                */
int orc_ev_apply_sgd(orc_ev* var, float lr, const float* grad, const int64_t* keys,
                     int64_t n, int64_t gs) {
  const int64_t D = var->dim;
  for (int64_t i = 0; i < n; ++i) {
    int64_t e = orc_apply_key(var, keys[i], gs);
    if (e < 0) continue;
    float* v = orc_get_or_alloc(var, e, var->default_value);
    for (int64_t d = 0; d < D; ++d) { float p = lr * grad[i * D + d]; v[d] = v[d] - p; }
    orc_bf16_row(var, v);
  }
  return ORC_OK;
}

/* KvSparseApplyAdagrad (training_ali_ops.cc:61-145):                        */
/* a += g*g; v -= (lr * g) * rsqrt(a)                                         */
int orc_ev_apply_adagrad(orc_ev* var, orc_ev* accum, float lr, const float* grad,
                         const int64_t* keys, int64_t n, int64_t gs) {
  const int64_t D = var->dim;
  for (int64_t i = 0; i < n; ++i) {
    int64_t e = orc_apply_key(var, keys[i], gs);
    if (e < 0) continue;
    float* a = orc_get_or_alloc(accum, e, accum->default_value);
    float* v = orc_get_or_alloc(var, e, var->default_value);
    for (int64_t d = 0; d < D; ++d) {
      float g = grad[i * D + d];
      float g2 = g * g;
      a[d] = a[d] + g2;
      float lg = lr * g;
      float rs = 1.0f / sqrtf(a[d]);
      float up = lg * rs;
      v[d] = v[d] - up;
    }
    orc_bf16_row(var, v);
  }
  return ORC_OK;
}

/* KvSparseApplyAdam (training_ali_ops.cc:848-975):                          */
/* alpha = lr*sqrt(1-b2^t)/(1-b1^t); m += (g-m)(1-b1); v += (g^2-v)(1-b2);     */
/* var -= (m*alpha)/(sqrt(v)+eps)                                             */
int orc_ev_apply_adam(orc_ev* var, orc_ev* m_ev, orc_ev* v_ev, float beta1_power,
                      float beta2_power, float lr, float beta1, float beta2,
                      float eps, const float* grad, const int64_t* keys, int64_t n,
                      int64_t gs) {
  const int64_t D = var->dim;
  const float alpha = lr * sqrtf(1.0f - beta2_power) / (1.0f - beta1_power);
  for (int64_t i = 0; i < n; ++i) {
    int64_t e = orc_apply_key(var, keys[i], gs);
    if (e < 0) continue;
    float* w = orc_get_or_alloc(var, e, var->default_value);
    float* m = orc_get_or_alloc(m_ev, e, m_ev->default_value);
    float* v = orc_get_or_alloc(v_ev, e, v_ev->default_value);
    for (int64_t d = 0; d < D; ++d) {
      float g = grad[i * D + d];
      float t1 = g - m[d]; t1 = t1 * (1.0f - beta1); m[d] = m[d] + t1;
      float t2 = g * g; t2 = t2 - v[d]; t2 = t2 * (1.0f - beta2); v[d] = v[d] + t2;
      float num = m[d] * alpha;
      float den = sqrtf(v[d]) + eps;
      w[d] = w[d] - num / den;
    }
    orc_bf16_row(var, w);
  }
  return ORC_OK;
}

/* KvSparseApplyAdamAsync (training_ali_ops.cc:1404-1575).  rmsprop == 0:  */
/* alpha = lr*sqrt(1-b2p)/(1-b1p); m = m*b1 + g*(1-b1); v = v*b2 + g^2*(1-b2); */
/* var -= (m*alpha)/(sqrt(v)+eps) (:1529-1554).  rmsprop != 0 (:1506-1513):  */
/* v = v*b2 + g^2*(1-b2); m = m*b1 + rsqrt(v+eps)*lr*g; var -= m.  The beta   */
/* powers are the caller's (advanced after the apply, :1558-1559).           */
int orc_ev_apply_adam_async(orc_ev* var, orc_ev* m_ev, orc_ev* v_ev, float beta1_power,
                            float beta2_power, float lr, float beta1, float beta2, float eps,
                            int rmsprop, const float* grad, const int64_t* keys, int64_t n,
                            int64_t gs) {
  const int64_t D = var->dim;
  const float alpha = lr * sqrtf(1.0f - beta2_power) / (1.0f - beta1_power);
  for (int64_t i = 0; i < n; ++i) {
    int64_t e = orc_apply_key(var, keys[i], gs);
    if (e < 0) continue;
    float* w = orc_get_or_alloc(var, e, var->default_value);
    float* m = orc_get_or_alloc(m_ev, e, m_ev->default_value);
    float* v = orc_get_or_alloc(v_ev, e, v_ev->default_value);
    for (int64_t d = 0; d < D; ++d) {
      float g = grad[i * D + d];
      float vt = v[d] * beta2, g2 = g * g, vg = g2 * (1.0f - beta2);
      v[d] = vt + vg;
      if (rmsprop) {
        float rs = 1.0f / sqrtf(v[d] + eps);
        float st = (rs * lr) * g;
        float mt = m[d] * beta1;
        m[d] = mt + st;
        w[d] = w[d] - m[d];
      } else {
        float mt = m[d] * beta1, mg = g * (1.0f - beta1);
        m[d] = mt + mg;
        float num = m[d] * alpha;
        float den = sqrtf(v[d]) + eps;
        w[d] = w[d] - num / den;
      }
    }
    orc_bf16_row(var, w);
  }
  return ORC_OK;
}

/* KvSparseApplyAdagradDecay (training_ali_ops.cc:703-823): the decay count */
/* is element 0 of the row of the var-shaped accum_decay_power slot; when   */
/* gs / decay_step (integer division) > count: a = max(a*rate, baseline),   */
/* count += 1.  Then a += g^2; v -= (lr*g) * rsqrt(a).                       */
int orc_ev_apply_adagrad_decay(orc_ev* var, orc_ev* accum, orc_ev* power, float lr,
                               int64_t decay_step, float decay_rate, float decay_baseline,
                               const float* grad, const int64_t* keys, int64_t n, int64_t gs) {
  if (decay_step <= 0) return ORC_INVALID_ARGUMENT;
  const int64_t D = var->dim;
  for (int64_t i = 0; i < n; ++i) {
    int64_t e = orc_apply_key(var, keys[i], gs);
    if (e < 0) continue;
    float* a = orc_get_or_alloc(accum, e, accum->default_value);
    float* p = orc_get_or_alloc(power, e, power->default_value);
    float* v = orc_get_or_alloc(var, e, var->default_value);
    const int dec = (float)(gs / decay_step) > p[0];
    if (dec) p[0] = p[0] + 1.0f;
    for (int64_t d = 0; d < D; ++d) {
      float g = grad[i * D + d];
      float ad = a[d];
      if (dec) {
        ad = ad * decay_rate;
        ad = ad < decay_baseline ? decay_baseline : ad;
      }
      float g2 = g * g;
      ad = ad + g2;
      a[d] = ad;
      float lg = lr * g;
      float rs = 1.0f / sqrtf(ad);
      float up = lg * rs;
      v[d] = v[d] - up;
    }
    orc_bf16_row(var, v);
  }
  return ORC_OK;
}

/* KvResourceSparseApplyFtrl[V2] (training_ali_ops.cc:167-331), the       */
/* COMPUTE_FTRL macro (:279-307) per key with grad_to_use = g (+ 2 * l2_    */
/* shrinkage * var for V2, :308-311):                                        */
/*   new_accum = accum + gu^2                                                */
/*   linear   += gu - (new_accum^p - accum^p) / lr * var    (p = -lr_power,  */
/*               sqrt when lr_power == -0.5)                                 */
/*   norm = sqrt(sum linear^2)  (a row reduction: Eigen's order is not       */
/*          reproducible, ascending order here -> parity by tolerance)       */
/*   var = norm > l1 ? (l1 - norm) / ((new_accum^p / lr + 2 l2) norm) linear */
/*                   : 0                                                     */
/*   accum += g^2   (the plain gradient, :307)                               */
int orc_ev_apply_ftrl(orc_ev* var, orc_ev* accum_ev, orc_ev* linear_ev, float lr, float l1,
                      float l2, float lr_power, float l2_shrinkage, const float* grad,
                      const int64_t* keys, int64_t n, int64_t gs) {
  const int64_t D = var->dim;
  const int sq = lr_power == -0.5f;
  float* gu = (float*)malloc(sizeof(float) * (size_t)(D > 0 ? D : 1));
  if (!gu) return ORC_RESOURCE_EXHAUSTED;
  for (int64_t i = 0; i < n; ++i) {
    int64_t e = orc_apply_key(var, keys[i], gs);
    if (e < 0) continue;
    float* w = orc_get_or_alloc(var, e, var->default_value);
    float* a = orc_get_or_alloc(accum_ev, e, accum_ev->default_value);
    float* lin = orc_get_or_alloc(linear_ev, e, linear_ev->default_value);
    float nsq = 0.f;
    for (int64_t d = 0; d < D; ++d) {
      float g = grad[i * D + d];
      gu[d] = l2_shrinkage > 0.f ? g + 2.0f * l2_shrinkage * w[d] : g;
      float na = a[d] + gu[d] * gu[d];
      float dp = sq ? sqrtf(na) - sqrtf(a[d]) : powf(na, -lr_power) - powf(a[d], -lr_power);
      float t = dp / lr * w[d];
      lin[d] = lin[d] + (gu[d] - t);
      nsq += lin[d] * lin[d];
    }
    float norm = sqrtf(nsq);
    for (int64_t d = 0; d < D; ++d) {
      float g = grad[i * D + d];
      float na = a[d] + gu[d] * gu[d];
      if (norm > l1) {
        float eta_rec = (sq ? sqrtf(na) : powf(na, -lr_power)) / lr;
        float coef = (l1 - norm) / ((eta_rec + 2.0f * l2) * norm);
        w[d] = coef * lin[d];
      } else {
        w[d] = 0.f;
      }
      a[d] = a[d] + g * g;
    }
  }
  free(gu);
  return ORC_OK;
}

/* Dense-variable counterparts (ResourceSparseApply*, training_ops.cc),      */
/* used by the EV == dense 5-step equality idiom                              */
/* (embedding_variable_ops_test.py:825-997).  Rows indexed directly.          */
int orc_dense_apply_sgd(float* table, int64_t D, float lr, const float* grad,
                        const int64_t* idx, int64_t n) {
  for (int64_t i = 0; i < n; ++i)
    for (int64_t d = 0; d < D; ++d) { float p = grad[i * D + d] * lr; table[idx[i] * D + d] -= p; }
  return ORC_OK;
}
int orc_dense_apply_adagrad(float* table, float* accum, int64_t D, float lr,
                            const float* grad, const int64_t* idx, int64_t n) {
  for (int64_t i = 0; i < n; ++i)
    for (int64_t d = 0; d < D; ++d) {
      float g = grad[i * D + d];
      float g2 = g * g;
      accum[idx[i] * D + d] += g2;
      float lg = g * lr;
      float rs = 1.0f / sqrtf(accum[idx[i] * D + d]);
      float up = lg * rs;
      table[idx[i] * D + d] -= up;
    }
  return ORC_OK;
}

/* ------------------------------------------------------------------------ */
/* Interactions (callers of the path).                                       */
/* ------------------------------------------------------------------------ */
/* FM 2nd order (modelzoo/DeepFM/train.py:205-209):                          */
/* out[b,d] = 0.5 * ((sum_f e)^2 - sum_f e^2), accumulated in double.         */
void orc_fm2(const float* emb, int64_t B, int64_t F, int64_t D, float* out) {
  for (int64_t b = 0; b < B; ++b)
    for (int64_t d = 0; d < D; ++d) {
      double s = 0.0, q = 0.0;
      for (int64_t f = 0; f < F; ++f) {
        double e = emb[(b * F + f) * D + d];
        s += e; q += e * e;
      }
      out[b * D + d] = (float)(0.5 * (s * s - q));
    }
}

/* DLRM dot interaction (modelzoo/DLRM/train.py:150-163): strictly-lower    */
/* triangle of X X^T in row-major (i>j) order, X = [B, F, D]; double accum.  */
void orc_dot_interaction(const float* x, int64_t B, int64_t F, int64_t D, float* out) {
  int64_t P = F * (F - 1) / 2;
  for (int64_t b = 0; b < B; ++b) {
    int64_t p = 0;
    for (int64_t i = 0; i < F; ++i)
      for (int64_t j = 0; j < i; ++j) {
        double s = 0.0;
        for (int64_t d = 0; d < D; ++d) s += (double)x[(b * F + i) * D + d] * (double)x[(b * F + j) * D + d];
        out[b * P + p++] = (float)s;
      }
  }
}

/* DCN-v2 CrossNet layer (absent from the reference; build-defined spec):    */
/* x_{l+1} = x0 * (W x_l + b) + x_l, W [d, d] row-major (out, in); double.    */
void orc_crossnet_layer(const float* x0, const float* xl, const float* W, const float* bias,
                        int64_t B, int64_t d, float* out) {
  for (int64_t r = 0; r < B; ++r)
    for (int64_t o = 0; o < d; ++o) {
      double s = bias ? bias[o] : 0.0;
      for (int64_t k = 0; k < d; ++k) s += (double)W[o * d + k] * (double)xl[r * d + k];
      out[r * d + o] = (float)((double)x0[r * d + o] * s + (double)xl[r * d + o]);
    }
}

/* ------------------------------------------------------------------------ */
/* Threaded CPU pipeline for bench.py's cpu_baseline leg: the DeepRec CPU    */
/* composition of embedding_lookup_sparse over an EV (embedding_ops.py:      */
/* 587-664): Unique (serial) -> KvResourceGather (Shard over all threads,    */
/* kv_variable_ops.cc:360-362) -> SparseSegmentReduction (Shard over         */
/* threads-1 over output rows, segment_reduction_ali_ops_util.h:173-174).    */
/* ------------------------------------------------------------------------ */
typedef struct {
  orc_ev* ev;
  const int64_t* keys;
  float* out;
  int64_t lo, hi;
  const float* data; const int32_t* idx; const int32_t* seg_off; int combiner;
  const float* table; const int64_t* rows;
} orc_task;

static void* orc_gather_worker(void* p) {
  orc_task* t = (orc_task*)p;
  const int64_t D = t->ev->dim;
  for (int64_t i = t->lo; i < t->hi; ++i) {
    int64_t e = orc_map_find(t->ev->map, t->keys[i]);
    const float* src = (e >= 0 && t->ev->map->ent[e].rows[0]) ? t->ev->map->ent[e].rows[0] : t->ev->default_value;
    memcpy(t->out + i * D, src, sizeof(float) * D);
  }
  return NULL;
}
static void* orc_dense_gather_worker(void* p) {
  orc_task* t = (orc_task*)p;
  const int64_t D = t->combiner; /* reused field: D */
  for (int64_t i = t->lo; i < t->hi; ++i)
    memcpy(t->out + i * D, t->table + t->rows[i] * D, sizeof(float) * D);
  return NULL;
}
static void* orc_reduce_worker(void* p) {
  orc_task* t = (orc_task*)p;
  const int64_t D = t->ev ? t->ev->dim : (int64_t)t->rows[0];
  for (int64_t s = t->lo; s < t->hi; ++s) {
    int64_t a = t->seg_off[s], b = t->seg_off[s + 1];
    if (b > a) orc_reduce_bag(t->data, D, t->idx, a, b - a, t->combiner & 3, t->out + s * D);
    else memset(t->out + s * D, 0, sizeof(float) * D);
  }
  return NULL;
}

static void orc_run_sharded(void* (*fn)(void*), orc_task* proto, int64_t total, int threads) {
  if (threads < 1) threads = 1;
  pthread_t th[256];
  orc_task tk[256];
  if (threads > 256) threads = 256;
  for (int t = 0; t < threads; ++t) {
    tk[t] = *proto;
    tk[t].lo = total * t / threads;
    tk[t].hi = total * (t + 1) / threads;
    pthread_create(&th[t], NULL, fn, &tk[t]);
  }
  for (int t = 0; t < threads; ++t) pthread_join(th[t], NULL);
}

/* Per-feature embedding_lookup_sparse over an EV; bags given by seg_off     */
/* (CSR offsets over the batch, length B+1).  Workspace allocated inside.    */
int orc_pipeline_ev_lookup_sparse(orc_ev* ev, const int64_t* ids, int64_t nnz,
                                  const int32_t* seg_off, int64_t B, int combiner,
                                  int threads, float* out) {
  const int64_t D = ev->dim;
  int64_t* uniq = (int64_t*)malloc(sizeof(int64_t) * (nnz > 0 ? nnz : 1));
  int32_t* idx = (int32_t*)malloc(sizeof(int32_t) * (nnz > 0 ? nnz : 1));
  int64_t U = orc_unique(ids, nnz, uniq, idx, NULL);
  float* emb = (float*)malloc(sizeof(float) * (U > 0 ? U : 1) * D);
  orc_task p;
  memset(&p, 0, sizeof(p));
  p.ev = ev; p.keys = uniq; p.out = emb;
  orc_run_sharded(orc_gather_worker, &p, U, threads);
  memset(&p, 0, sizeof(p));
  p.ev = ev; p.data = emb; p.idx = idx; p.seg_off = seg_off; p.combiner = combiner; p.out = out;
  orc_run_sharded(orc_reduce_worker, &p, B, threads > 1 ? threads - 1 : 1);
  free(uniq); free(idx); free(emb);
  return ORC_OK;
}

/* Same over a dense table (ResourceGather HandleCopies + ali reduce).       */
int orc_pipeline_dense_lookup_sparse(const float* table, int64_t D, const int64_t* ids,
                                     int64_t nnz, const int32_t* seg_off, int64_t B,
                                     int combiner, int threads, float* out) {
  int64_t* uniq = (int64_t*)malloc(sizeof(int64_t) * (nnz > 0 ? nnz : 1));
  int32_t* idx = (int32_t*)malloc(sizeof(int32_t) * (nnz > 0 ? nnz : 1));
  int64_t U = orc_unique(ids, nnz, uniq, idx, NULL);
  float* emb = (float*)malloc(sizeof(float) * (U > 0 ? U : 1) * D);
  orc_task p;
  memset(&p, 0, sizeof(p));
  p.table = table; p.rows = uniq; p.out = emb; p.combiner = (int)D;
  orc_run_sharded(orc_dense_gather_worker, &p, U, threads);
  int64_t dd = D;
  memset(&p, 0, sizeof(p));
  p.rows = &dd; p.data = emb; p.idx = idx; p.seg_off = seg_off; p.combiner = combiner; p.out = out;
  orc_run_sharded(orc_reduce_worker, &p, B, threads > 1 ? threads - 1 : 1);
  free(uniq); free(idx); free(emb);
  return ORC_OK;
}

/* ------------------------------------------------------------------------ */
/* Persistent worker pool: TF's per-device CPU worker threads               */
/* (tensorflow_cpu_worker_threads()->workers, the pool Shard and the Unique  */
/* op's TaskRunner hand their tasks to), created once, not per call.         */
/* orc_pool_run(pool, fn, arg, ntasks) runs fn(arg, id, ntasks) for every    */
/* id in [0, ntasks) on the workers and returns when all have finished.      */
/* ------------------------------------------------------------------------ */
typedef void (*orc_task_fn)(void* arg, int id, int ntasks);
typedef struct {
  int n;
  pthread_t th[256];
  pthread_mutex_t mu;
  pthread_cond_t cv_work, cv_done;
  orc_task_fn fn;
  void* arg;
  int ntasks, next, pending, quit;
} orc_pool;

static void* orc_pool_main(void* p) {
  orc_pool* pl = (orc_pool*)p;
  pthread_mutex_lock(&pl->mu);
  for (;;) {
    while (!pl->quit && pl->next >= pl->ntasks) pthread_cond_wait(&pl->cv_work, &pl->mu);
    if (pl->quit) break;
    const int id = pl->next++;
    orc_task_fn fn = pl->fn;
    void* arg = pl->arg;
    const int nt = pl->ntasks;
    pthread_mutex_unlock(&pl->mu);
    fn(arg, id, nt);
    pthread_mutex_lock(&pl->mu);
    if (--pl->pending == 0) pthread_cond_signal(&pl->cv_done);
  }
  pthread_mutex_unlock(&pl->mu);
  return NULL;
}

orc_pool* orc_pool_create(int threads) {
  if (threads < 1) threads = 1;
  if (threads > 256) threads = 256;
  orc_pool* pl = (orc_pool*)calloc(1, sizeof(orc_pool));
  if (!pl) return NULL;
  pthread_mutex_init(&pl->mu, NULL);
  pthread_cond_init(&pl->cv_work, NULL);
  pthread_cond_init(&pl->cv_done, NULL);
  for (int t = 0; t < threads; ++t) {
    if (pthread_create(&pl->th[t], NULL, orc_pool_main, pl) != 0) break;
    pl->n = t + 1;
  }
  return pl;
}

int orc_pool_threads(const orc_pool* pl) { return pl ? pl->n : 0; }

void orc_pool_free(orc_pool* pl) {
  if (!pl) return;
  pthread_mutex_lock(&pl->mu);
  pl->quit = 1;
  pthread_cond_broadcast(&pl->cv_work);
  pthread_mutex_unlock(&pl->mu);
  for (int t = 0; t < pl->n; ++t) pthread_join(pl->th[t], NULL);
  pthread_cond_destroy(&pl->cv_work);
  pthread_cond_destroy(&pl->cv_done);
  pthread_mutex_destroy(&pl->mu);
  free(pl);
}

static void orc_pool_run(orc_pool* pl, orc_task_fn fn, void* arg, int ntasks) {
  if (ntasks <= 0) return;
  if (ntasks == 1 || pl->n <= 0) {   /* one task: inline, as Shard does below its cost cut */
    for (int i = 0; i < ntasks; ++i) fn(arg, i, ntasks);
    return;
  }
  pthread_mutex_lock(&pl->mu);
  pl->fn = fn;
  pl->arg = arg;
  pl->next = 0;
  pl->pending = ntasks;
  pl->ntasks = ntasks;
  pthread_cond_broadcast(&pl->cv_work);
  while (pl->pending > 0) pthread_cond_wait(&pl->cv_done, &pl->mu);
  pl->ntasks = pl->next = 0;
  pthread_mutex_unlock(&pl->mu);
}

/* ------------------------------------------------------------------------ */
/* Parallel first-occurrence Unique: ParallelComputeV1                       */
/* (unique_ali_op_util.h:226-445), the default of UniqueAliOp (serial_ =     */
/* false, unique_ali_op.cc:55-56) for N >= kPartitionLimit = 14336           */
/* (unique_ali_op_util.h:48, :651-657).  Four steps:                          */
/*  1. T1 = max(min(threads, cbrt(10 threads) + 1), 1) sections, one local    */
/*     hash map (key -> local position, insertion order) per section;       */
/*  2. T2 = max(min(threads, ceil(sum_i size_i * i / 8192)), 1) tasks mark    */
/*     each key of map l that an earlier map p < l holds (prior maps in      */
/*     ascending order, so the owner is always the earliest map's node) and  */
/*     count the duplicates;                                                 */
/*  3. per map, global indices from the prefix of the non-duplicate counts,  */
/*     the keys written at them;                                             */
/*  4. idx[i] = the global index of the node (or its owner) of x[i] in its   */
/*     section's map, T4 = max(min(threads, ceil(N / 8192)), 1) tasks.       */
/* The result equals SerialComputeV1's (first occurrence over the whole     */
/* input), which tests/test_oracle_golden.py checks against orc_unique.      */
/* ------------------------------------------------------------------------ */
typedef struct {         /* INode (unique_ali_op_util.h:230-237) */
  int64_t key;
  int64_t index;         /* local, then global index */
  int64_t owner;         /* -1, or (map << 32) | position of the earliest map's node */
} orc_inode;

typedef struct {
  int64_t lo, hi;        /* section of the input */
  int64_t cap;           /* open-addressing table: slot -> local position or -1 */
  int64_t* slot;
  orc_inode* node;       /* in insertion order */
  int64_t size;
} orc_submap;

static int64_t orc_submap_find(const orc_submap* m, int64_t k) {
  uint64_t h = orc_mix64((uint64_t)k) & (uint64_t)(m->cap - 1);
  for (;;) {
    const int64_t j = m->slot[h];
    if (j < 0) return -1;
    if (m->node[j].key == k) return j;
    h = (h + 1) & (uint64_t)(m->cap - 1);
  }
}

typedef struct {
  const int64_t* x;
  int64_t n;
  orc_submap* maps;
  int t1, t2;
  int64_t* dups;         /* [T1 * T2] */
  int64_t* goff;         /* [T1] */
  int64_t* y;
  int32_t* idx;
} orc_punique;

static void orc_pu_build(void* a, int id, int nt) {
  orc_punique* u = (orc_punique*)a;
  orc_submap* m = &u->maps[id];
  (void)nt;
  const int64_t n = m->hi - m->lo;
  m->cap = 16;
  while (m->cap < 2 * n) m->cap <<= 1;
  m->slot = (int64_t*)malloc(sizeof(int64_t) * m->cap);
  m->node = (orc_inode*)malloc(sizeof(orc_inode) * (n > 0 ? n : 1));
  for (int64_t s = 0; s < m->cap; ++s) m->slot[s] = -1;
  m->size = 0;
  for (int64_t i = m->lo; i < m->hi; ++i) {
    const int64_t k = u->x[i];
    uint64_t h = orc_mix64((uint64_t)k) & (uint64_t)(m->cap - 1);
    for (;;) {
      const int64_t j = m->slot[h];
      if (j < 0) {
        m->slot[h] = m->size;
        m->node[m->size].key = k;
        m->node[m->size].index = m->size;
        m->node[m->size].owner = -1;
        m->size++;
        break;
      }
      if (m->node[j].key == k) break;
      h = (h + 1) & (uint64_t)(m->cap - 1);
    }
  }
}

/* Partitioner (unique_ali_op_util.h:103-116): part i = (work + i) / parts   */
static void orc_part(int64_t work, int parts, int i, int64_t* lo, int64_t* hi) {
  int64_t s = 0;
  for (int j = 0; j < i; ++j) s += (work + j) / parts;
  *lo = s;
  *hi = s + (work + i) / parts;
}

static void orc_pu_dedup(void* a, int task, int nt) {
  orc_punique* u = (orc_punique*)a;
  for (int p = 0; p < u->t1 - 1; ++p) {
    const orc_submap* prior = &u->maps[p];
    for (int l = p + 1; l < u->t1; ++l) {
      orc_submap* lat = &u->maps[l];
      int64_t lo, hi, d = 0;
      orc_part(lat->size, nt, task, &lo, &hi);
      for (int64_t i = lo; i < hi; ++i) {
        if (lat->node[i].owner >= 0) continue;
        const int64_t j = orc_submap_find(prior, lat->node[i].key);
        if (j < 0) continue;
        /* GetINodeByPos: the prior node, or the node it defers to */
        lat->node[i].owner = prior->node[j].owner >= 0 ? prior->node[j].owner
                                                       : ((int64_t)p << 32) | j;
        ++d;
      }
      u->dups[l * nt + task] += d;   /* one store per (map, task): no shared line in the loop */
    }
  }
}

static void orc_pu_index(void* a, int id, int nt) {
  orc_punique* u = (orc_punique*)a;
  orc_submap* m = &u->maps[id];
  (void)nt;
  int64_t cur = u->goff[id];
  for (int64_t i = 0; i < m->size; ++i) {
    if (m->node[i].owner >= 0) continue;
    m->node[i].index = cur;
    u->y[cur] = m->node[i].key;
    ++cur;
  }
}

static void orc_pu_output(void* a, int task, int nt) {
  orc_punique* u = (orc_punique*)a;
  int64_t lo, hi;
  orc_part(u->n, nt, task, &lo, &hi);
  int mi = 0;
  for (int64_t i = lo; i < hi; ++i) {
    while (i >= u->maps[mi].hi) ++mi;
    const orc_submap* m = &u->maps[mi];
    const int64_t j = orc_submap_find(m, u->x[i]);
    const int64_t o = m->node[j].owner;
    u->idx[i] = (int32_t)(o < 0 ? m->node[j].index : u->maps[o >> 32].node[o & 0xffffffff].index);
  }
}

int64_t orc_unique_parallel(orc_pool* pool, const int64_t* x, int64_t n, int64_t* y,
                            int32_t* idx) {
  if (n <= 0) return 0;
  const int threads = pool ? pool->n : 1;
  int t1 = (int)(cbrt(10.0 * threads) + 1);
  if (t1 > threads) t1 = threads;
  if (t1 < 1) t1 = 1;
  orc_punique u;
  memset(&u, 0, sizeof(u));
  u.x = x;
  u.n = n;
  u.y = y;
  u.idx = idx;
  u.t1 = t1;
  u.maps = (orc_submap*)calloc((size_t)t1, sizeof(orc_submap));
  for (int i = 0; i < t1; ++i) orc_part(n, t1, i, &u.maps[i].lo, &u.maps[i].hi);
  orc_pool_run(pool, orc_pu_build, &u, t1);
  int64_t cost = 0;
  for (int i = 0; i < t1; ++i) cost += u.maps[i].size * i;
  int t2 = (int)((cost + 8191) / 8192);
  if (t2 > threads) t2 = threads;
  if (t2 < 1) t2 = 1;
  u.t2 = t2;
  u.dups = (int64_t*)calloc((size_t)t1 * t2, sizeof(int64_t));
  orc_pool_run(pool, orc_pu_dedup, &u, t2);
  u.goff = (int64_t*)calloc((size_t)t1, sizeof(int64_t));
  for (int i = 0; i + 1 < t1; ++i) {
    u.goff[i + 1] = u.goff[i] + u.maps[i].size;
    for (int j = 0; j < t2; ++j) u.goff[i + 1] -= u.dups[i * t2 + j];
  }
  int64_t total = u.goff[t1 - 1] + u.maps[t1 - 1].size;
  for (int j = 0; j < t2; ++j) total -= u.dups[(t1 - 1) * t2 + j];
  orc_pool_run(pool, orc_pu_index, &u, t1);
  int t4 = (int)((n + 8191) / 8192);
  if (t4 > threads) t4 = threads;
  if (t4 < 1) t4 = 1;
  orc_pool_run(pool, orc_pu_output, &u, t4);
  for (int i = 0; i < t1; ++i) {
    free(u.maps[i].slot); free(u.maps[i].node);
  }
  free(u.maps); free(u.dups); free(u.goff);
  return total;
}

/* The cpu_baseline pipeline on the persistent pool: UniqueAliOp's dispatch  */
/* (parallel for N >= 14336 unless serial, unique_ali_op_util.h:651-657) ->  */
/* KvResourceGather (Shard over the workers, kv_variable_ops.cc:360-362) ->  */
/* SparseSegmentReduction (threads - 1 shards over the output rows,          */
/* segment_reduction_ali_ops_util.h:173-174).                                 */
typedef struct {
  orc_task proto;
  int64_t total;
  void* (*fn)(void*);
} orc_shard;

static void orc_shard_task(void* a, int id, int nt) {
  orc_shard* s = (orc_shard*)a;
  orc_task t = s->proto;
  t.lo = s->total * id / nt;
  t.hi = s->total * (id + 1) / nt;
  s->fn(&t);
}

int orc_pipeline_ev_lookup_sparse_pool(orc_pool* pool, orc_ev* ev, const int64_t* ids,
                                       int64_t nnz, const int32_t* seg_off, int64_t B,
                                       int combiner, int serial_unique, float* out) {
  if (!pool || !ev) return ORC_INVALID_ARGUMENT;
  const int64_t D = ev->dim;
  const int threads = pool->n;
  int64_t* uniq = (int64_t*)malloc(sizeof(int64_t) * (nnz > 0 ? nnz : 1));
  int32_t* idx = (int32_t*)malloc(sizeof(int32_t) * (nnz > 0 ? nnz : 1));
  const int64_t U = (nnz >= 14336 && !serial_unique) ? orc_unique_parallel(pool, ids, nnz, uniq, idx)
                                                      : orc_unique(ids, nnz, uniq, idx, NULL);
  float* emb = (float*)malloc(sizeof(float) * (U > 0 ? U : 1) * D);
  orc_shard s;
  memset(&s, 0, sizeof(s));
  s.proto.ev = ev; s.proto.keys = uniq; s.proto.out = emb;
  s.total = U;
  s.fn = orc_gather_worker;
  orc_pool_run(pool, orc_shard_task, &s, U > 0 ? threads : 0);
  memset(&s, 0, sizeof(s));
  s.proto.ev = ev; s.proto.data = emb; s.proto.idx = idx; s.proto.seg_off = seg_off;
  s.proto.combiner = combiner; s.proto.out = out;
  s.total = B;
  s.fn = orc_reduce_worker;
  orc_pool_run(pool, orc_shard_task, &s, B > 0 ? (threads > 1 ? threads - 1 : 1) : 0);
  free(uniq); free(idx); free(emb);
  return ORC_OK;
}

/* ------------------------------------------------------------------------ */
/* String -> id: StringToHashBucketFast (string_to_hash_bucket_ali_op.h:     */
/* 33-63: bucket = Fingerprint64(s) % num_buckets) and the EV column's       */
/* num_buckets = INT64_MAX (feature_column_v2.py:5954-5957).                 */
/* Fingerprint64 = farmhash::Fingerprint64 (tensorflow/core/platform/        */
/* fingerprint.h:80-88), i.e. farmhashna::Hash64 of google/farmhash          */
/* @816a4ae622e964763ca0862d9dbd19324a1eaf45 (tensorflow/workspace.bzl:      */
/* 275-282; a network-fetched dependency absent from the reference tree).    */
/* Restated from farmhash's published algorithm; pinned by the reference's   */
/* golden values (fingerprint_test.cc:26-29, fingerprint_op_test.cc:64-106,  */
/* string_to_hash_bucket_op_test.py:40-50) in tests/golden/.                 */
/* ------------------------------------------------------------------------ */
static const uint64_t orc_k0 = 0xc3a5c85c97cb3127ULL;
static const uint64_t orc_k1 = 0xb492b66fbe98f273ULL;
static const uint64_t orc_k2 = 0x9ae16a3b2f90404fULL;

static uint64_t orc_fetch64(const uint8_t* p) {
  uint64_t v;
  memcpy(&v, p, 8);
  return v; /* little-endian host */
}
static uint32_t orc_fetch32(const uint8_t* p) {
  uint32_t v;
  memcpy(&v, p, 4);
  return v;
}
static uint64_t orc_rot64(uint64_t v, int s) { return s == 0 ? v : (v >> s) | (v << (64 - s)); }
static uint64_t orc_shiftmix(uint64_t v) { return v ^ (v >> 47); }
static uint64_t orc_hash_len16(uint64_t u, uint64_t v, uint64_t mul) {
  uint64_t a = (u ^ v) * mul;
  a ^= a >> 47;
  uint64_t b = (v ^ a) * mul;
  b ^= b >> 47;
  return b * mul;
}
static uint64_t orc_hash_len0to16(const uint8_t* s, uint64_t len) {
  if (len >= 8) {
    uint64_t mul = orc_k2 + len * 2;
    uint64_t a = orc_fetch64(s) + orc_k2;
    uint64_t b = orc_fetch64(s + len - 8);
    uint64_t c = orc_rot64(b, 37) * mul + a;
    uint64_t d = (orc_rot64(a, 25) + b) * mul;
    return orc_hash_len16(c, d, mul);
  }
  if (len >= 4) {
    uint64_t mul = orc_k2 + len * 2;
    uint64_t a = orc_fetch32(s);
    return orc_hash_len16(len + (a << 3), orc_fetch32(s + len - 4), mul);
  }
  if (len > 0) {
    uint8_t a = s[0], b = s[len >> 1], c = s[len - 1];
    uint32_t y = (uint32_t)a + ((uint32_t)b << 8);
    uint32_t z = (uint32_t)len + ((uint32_t)c << 2);
    return orc_shiftmix(y * orc_k2 ^ z * orc_k0) * orc_k2;
  }
  return orc_k2;
}
static uint64_t orc_hash_len17to32(const uint8_t* s, uint64_t len) {
  uint64_t mul = orc_k2 + len * 2;
  uint64_t a = orc_fetch64(s) * orc_k1;
  uint64_t b = orc_fetch64(s + 8);
  uint64_t c = orc_fetch64(s + len - 8) * mul;
  uint64_t d = orc_fetch64(s + len - 16) * orc_k2;
  return orc_hash_len16(orc_rot64(a + b, 43) + orc_rot64(c, 30) + d,
                        a + orc_rot64(b + orc_k2, 18) + c, mul);
}
static uint64_t orc_hash_len33to64(const uint8_t* s, uint64_t len) {
  uint64_t mul = orc_k2 + len * 2;
  uint64_t a = orc_fetch64(s) * orc_k2;
  uint64_t b = orc_fetch64(s + 8);
  uint64_t c = orc_fetch64(s + len - 8) * mul;
  uint64_t d = orc_fetch64(s + len - 16) * orc_k2;
  uint64_t y = orc_rot64(a + b, 43) + orc_rot64(c, 30) + d;
  uint64_t z = orc_hash_len16(y, a + orc_rot64(b + orc_k2, 18) + c, mul);
  uint64_t e = orc_fetch64(s + 16) * mul;
  uint64_t f = orc_fetch64(s + 24);
  uint64_t g = (y + orc_fetch64(s + len - 32)) * mul;
  uint64_t h = (z + orc_fetch64(s + len - 24)) * mul;
  return orc_hash_len16(orc_rot64(e + f, 43) + orc_rot64(g, 30) + h,
                        e + orc_rot64(f + a, 18) + g, mul);
}
static void orc_weak32(const uint8_t* s, uint64_t a, uint64_t b, uint64_t* o1, uint64_t* o2) {
  uint64_t w = orc_fetch64(s), x = orc_fetch64(s + 8), y = orc_fetch64(s + 16),
           z = orc_fetch64(s + 24);
  a += w;
  b = orc_rot64(b + a + z, 21);
  uint64_t c = a;
  a += x;
  a += y;
  b += orc_rot64(a, 44);
  *o1 = a + z;
  *o2 = b + c;
}

uint64_t orc_fingerprint64(const uint8_t* s, uint64_t len) {
  if (len <= 16) return orc_hash_len0to16(s, len);
  if (len <= 32) return orc_hash_len17to32(s, len);
  if (len <= 64) return orc_hash_len33to64(s, len);
  const uint64_t seed = 81;
  uint64_t x = seed, y = seed * orc_k1 + 113, z = orc_shiftmix(y * orc_k2 + 113) * orc_k2;
  uint64_t v1 = 0, v2 = 0, w1 = 0, w2 = 0, t;
  x = x * orc_k2 + orc_fetch64(s);
  const uint8_t* end = s + ((len - 1) / 64) * 64;
  const uint8_t* last64 = end + ((len - 1) & 63) - 63;
  do {
    x = orc_rot64(x + y + v1 + orc_fetch64(s + 8), 37) * orc_k1;
    y = orc_rot64(y + v2 + orc_fetch64(s + 48), 42) * orc_k1;
    x ^= w2;
    y += v1 + orc_fetch64(s + 40);
    z = orc_rot64(z + w1, 33) * orc_k1;
    orc_weak32(s, v2 * orc_k1, x + w1, &v1, &v2);
    orc_weak32(s + 32, z + w2, y + orc_fetch64(s + 16), &w1, &w2);
    t = z; z = x; x = t;
    s += 64;
  } while (s != end);
  uint64_t mul = orc_k1 + ((z & 0xff) << 1);
  s = last64;
  w1 += ((len - 1) & 63);
  v1 += w1;
  w1 += v1;
  x = orc_rot64(x + y + v1 + orc_fetch64(s + 8), 37) * mul;
  y = orc_rot64(y + v2 + orc_fetch64(s + 48), 42) * mul;
  x ^= w2 * 9;
  y += v1 * 9 + orc_fetch64(s + 40);
  z = orc_rot64(z + w1, 33) * mul;
  orc_weak32(s, v2 * mul, x + w1, &v1, &v2);
  orc_weak32(s + 32, z + w2, y + orc_fetch64(s + 16), &w1, &w2);
  t = z; z = x; x = t;
  return orc_hash_len16(orc_hash_len16(v1, w1, mul) + orc_shiftmix(y) * orc_k0 + z,
                        orc_hash_len16(v2, w2, mul) + x, mul);
}

/* StringToHashBucketFast over n strings in (offsets[n+1], bytes) layout. */
void orc_string_to_hash_bucket_fast(const uint8_t* bytes, const int64_t* offsets, int64_t n,
                                    int64_t num_buckets, int64_t* out) {
  for (int64_t i = 0; i < n; ++i)
    out[i] = (int64_t)(orc_fingerprint64(bytes + offsets[i], (uint64_t)(offsets[i + 1] - offsets[i])) %
                       (uint64_t)num_buckets);
}
