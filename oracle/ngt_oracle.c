/*
 * ngt_oracle.c -- CPU restatement of the NGT 1.13.8 distance/search hot path.
 *
 * TEST INFRASTRUCTURE ONLY (see ngt_oracle.h).  Compiled with
 * -ffp-contract=off so that every fused multiply-add below is the explicit
 * fmaf() that mirrors the reference's `vfmadd231ps` and nothing else is
 * contracted.
 */
#include "ngt_oracle.h"

#include <float.h>
#include <limits.h>
#include <math.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------------- */
/* Float reductions as emitted by the reference's AVX-512 build.             */
/* ------------------------------------------------------------------------- */

/* 16 lanes -> 8 -> 4 (lane j + lane j+8, then j + j+4), then
 * (x0+x1)+(x2+x3).  Matches the vextractf32x8/vextractf128/vunpckhps/vshufps
 * sequence of ComparatorL2 (PrimitiveComparator.h:154-155,193-196). */
static float hsum16(const float acc[16]) {
  float t8[8], t4[4];
  for (int j = 0; j < 8; j++) t8[j] = acc[j + 8] + acc[j];
  for (int j = 0; j < 4; j++) t4[j] = t8[j + 4] + t8[j];
  return (t4[0] + t4[1]) + (t4[2] + t4[3]);
}

/* PrimitiveComparator::compareL2(const float*, ...) (PrimitiveComparator.h:143-198):
 * AVX-512 16-lane accumulate of (a-b)^2 with FMA, tree reduce, sqrt in double. */
static double l2_f32(const float *a, const float *b, size_t n) {
  float acc[16] = {0};
  for (size_t i = 0; i < n; i += 16)
    for (int j = 0; j < 16; j++) {
      float v = a[i + j] - b[i + j];
      acc[j] = fmaf(v, v, acc[j]);
    }
  return sqrt((double)hsum16(acc));
}

/* PrimitiveComparator::compareL1(const float*, ...) (PrimitiveComparator.h:269-289):
 * 8-lane AVX sum of |a-b| (no FMA), horizontal ((x0+x1)+(x2+x3))+((x4+x5)+(x6+x7)). */
static double l1_f32(const float *a, const float *b, size_t n) {
  float acc[8] = {0};
  size_t i = 0;
  for (; i + 7 < n; i += 8)
    for (int j = 0; j < 8; j++) acc[j] = acc[j] + fabsf(a[i + j] - b[i + j]);
  double s = (double)(((acc[0] + acc[1]) + (acc[2] + acc[3])) +
                      ((acc[4] + acc[5]) + (acc[6] + acc[7])));
  for (; i < n; i++) s += fabs((double)(a[i] - b[i]));
  return s;
}

/* PrimitiveComparator::compareDotProduct(const float*, ...) (PrimitiveComparator.h:446-477):
 * 16-lane FMA, 16->8->4 in float, final four lanes summed in double. */
static double dot_f32(const float *a, const float *b, size_t n) {
  float acc[16] = {0};
  for (size_t i = 0; i < n; i += 16)
    for (int j = 0; j < 16; j++) acc[j] = fmaf(b[i + j], a[i + j], acc[j]);
  float t8[8], t4[4];
  for (int j = 0; j < 8; j++) t8[j] = acc[j + 8] + acc[j];
  for (int j = 0; j < 4; j++) t4[j] = t8[j + 4] + t8[j];
  return ((double)t4[0] + (double)t4[1]) + ((double)t4[2] + (double)t4[3]);
}

/* PrimitiveComparator::compareCosine(const float*, ...) (PrimitiveComparator.h:487-553). */
static double cosine_f32(const float *a, const float *b, size_t n) {
  float na[16] = {0}, nb[16] = {0}, s[16] = {0};
  for (size_t i = 0; i < n; i += 16)
    for (int j = 0; j < 16; j++) {
      na[j] = fmaf(a[i + j], a[i + j], na[j]);
      nb[j] = fmaf(b[i + j], b[i + j], nb[j]);
      s[j] = fmaf(b[i + j], a[i + j], s[j]);
    }
  double dna = hsum16(na), dnb = hsum16(nb), ds = hsum16(s);
  return ds / sqrt(dna * dnb);
}

/* compareAngleDistance / compareNormalizedAngleDistance (PrimitiveComparator.h:571-593). */
static double angle_of(double c) {
  if (c >= 1.0) return 0.0;
  if (c <= -1.0) return acos(-1.0);
  return acos(c);
}

/* PrimitiveComparator::compareSparseJaccardDistance(const float*, ...)
 * (PrimitiveComparator.h:399-418) -- including the reference's use of
 * bi[loca] in the loop guard. */
static double sparse_jaccard_f32(const float *a, const float *b, size_t size) {
  size_t loca = 0, locb = 0, count = 0;
  const uint32_t *ai = (const uint32_t *)a, *bi = (const uint32_t *)b;
  while (locb < size && ai[loca] != 0 && bi[loca] != 0) {
    int64_t sub = (int64_t)ai[loca] - (int64_t)bi[locb];
    count += sub == 0;
    loca += sub <= 0;
    locb += sub >= 0;
  }
  while (ai[loca] != 0) loca++;
  while (locb < size && bi[locb] != 0) locb++;
  return 1.0 - (double)count / (double)(loca + locb - count);
}

/* comparePoincareDistance(const float*) (PrimitiveComparator.h:608-618). */
static double poincare_f32(const float *a, const float *b, size_t n) {
  double a2 = 0.0, b2 = 0.0, c2 = l2_f32(a, b, n);
  for (size_t i = 0; i < n; i++) {
    a2 += (double)a[i] * (double)a[i];
    b2 += (double)b[i] * (double)b[i];
  }
  return acosh(1 + 2.0 * c2 * c2 / (1.0 - a2) / (1.0 - b2));
}

/* compareLorentzDistance(const float*) (PrimitiveComparator.h:630-637). */
static double lorentz_f32(const float *a, const float *b, size_t n) {
  double sum = (double)a[0] * (double)b[0];
  for (size_t i = 1; i < n; i++) sum -= (double)a[i] * (double)b[i];
  return acosh(sum);
}

/* ------------------------------------------------------------------------- */
/* uint8 comparators (exact integer arithmetic in float/double lanes).       */
/* ------------------------------------------------------------------------- */

/* compareL2(const unsigned char*, ...) (PrimitiveComparator.h:200-223): squares
 * of 16-bit differences summed in 4 float lanes (lane c takes elements c and
 * c+4 of each 8-byte group; -Ofast pairs them first), horizontal
 * (x0+x1)+(x2+x3), tail in double, sqrt. */
static double l2_u8(const uint8_t *a, const uint8_t *b, size_t n) {
  float acc[4] = {0};
  size_t i = 0;
  for (; i + 7 < n; i += 8)
    for (int c = 0; c < 4; c++) {
      int d0 = (int)a[i + c] - (int)b[i + c], d1 = (int)a[i + c + 4] - (int)b[i + c + 4];
      acc[c] = acc[c] + ((float)(d0 * d0) + (float)(d1 * d1));
    }
  double s = (double)((acc[0] + acc[1]) + (acc[2] + acc[3]));
  for (; i < n; i++) {
    int d = (int)a[i] - (int)b[i];
    s += d * d;
  }
  return sqrt(s);
}

/* compareL1(const unsigned char*, ...) (PrimitiveComparator.h:290-313). */
static double l1_u8(const uint8_t *a, const uint8_t *b, size_t n) {
  float acc[4] = {0};
  size_t i = 0;
  for (; i + 7 < n; i += 8)
    for (int c = 0; c < 4; c++) {
      int d0 = abs((int)a[i + c] - (int)b[i + c]), d1 = abs((int)a[i + c + 4] - (int)b[i + c + 4]);
      acc[c] = acc[c] + ((float)d0 + (float)d1);
    }
  double s = (double)((acc[0] + acc[1]) + (acc[2] + acc[3]));
  for (; i < n; i++) s += fabs((double)a[i] - (double)b[i]);
  return s;
}

/* compareHammingDistance (PrimitiveComparator.h:340-353): popcount over u64 words. */
static double hamming_u8(const uint8_t *a, const uint8_t *b, size_t n) {
  size_t count = 0;
  for (size_t i = 0; i + 8 <= n; i += 8) {
    uint64_t x, y;
    memcpy(&x, a + i, 8);
    memcpy(&y, b + i, 8);
    count += (size_t)__builtin_popcountll(x ^ y);
  }
  return (double)count;
}

/* compareJaccardDistance (PrimitiveComparator.h:375-391). */
static double jaccard_u8(const uint8_t *a, const uint8_t *b, size_t n) {
  size_t count = 0, de = 0;
  for (size_t i = 0; i + 8 <= n; i += 8) {
    uint64_t x, y;
    memcpy(&x, a + i, 8);
    memcpy(&y, b + i, 8);
    count += (size_t)__builtin_popcountll(x & y);
    de += (size_t)__builtin_popcountll(x | y);
  }
  return 1.0 - (double)count / (double)de;
}

/* compareDotProduct / compareCosine on uint8 (PrimitiveComparator.h:479-485, 555-568):
 * double sums of exact integer products, order-independent. */
static double dot_u8(const uint8_t *a, const uint8_t *b, size_t n) {
  double s = 0.0;
  for (size_t i = 0; i < n; i++) s += (double)a[i] * (double)b[i];
  return s;
}
static double cosine_u8(const uint8_t *a, const uint8_t *b, size_t n) {
  double na = 0.0, nb = 0.0, s = 0.0;
  for (size_t i = 0; i < n; i++) {
    na += (double)a[i] * (double)a[i];
    nb += (double)b[i] * (double)b[i];
    s += (double)a[i] * (double)b[i];
  }
  return s / sqrt(na * nb);
}
static double poincare_u8(const uint8_t *a, const uint8_t *b, size_t n) {
  double a2 = 0.0, b2 = 0.0, c2 = l2_u8(a, b, n);
  for (size_t i = 0; i < n; i++) {
    a2 += (double)a[i] * (double)a[i];
    b2 += (double)b[i] * (double)b[i];
  }
  return acosh(1 + 2.0 * c2 * c2 / (1.0 - a2) / (1.0 - b2));
}
static double lorentz_u8(const uint8_t *a, const uint8_t *b, size_t n) {
  double sum = (double)a[0] * (double)b[0];
  for (size_t i = 1; i < n; i++) sum -= (double)a[i] * (double)b[i];
  return acosh(sum);
}

/* ObjectSpaceRepository::setDistanceType (ObjectSpaceRepository.h:346-441)
 * dispatch, for both object types. */
static double compare(int metric, int otype, const void *pa, const void *pb, size_t dp) {
  if (otype == NGTO_FLOAT) {
    const float *a = (const float *)pa, *b = (const float *)pb;
    switch (metric) {
      case NGTO_L1: return l1_f32(a, b, dp);
      case NGTO_L2: return l2_f32(a, b, dp);
      case NGTO_ANGLE: return angle_of(cosine_f32(a, b, dp));
      case NGTO_COSINE: return 1.0 - cosine_f32(a, b, dp);
      case NGTO_NORMALIZED_ANGLE: return angle_of(dot_f32(a, b, dp));
      case NGTO_NORMALIZED_COSINE: {
        double v = 1.0 - dot_f32(a, b, dp);
        return v < 0.0 ? 0.0 : v;
      }
      case NGTO_NORMALIZED_L2: {
        double v = 2.0 - 2.0 * dot_f32(a, b, dp);
        return v < 0.0 ? 0.0 : sqrt(v);
      }
      case NGTO_SPARSE_JACCARD: return sparse_jaccard_f32(a, b, dp);
      case NGTO_POINCARE: return poincare_f32(a, b, dp);
      case NGTO_LORENTZ: return lorentz_f32(a, b, dp);
      case NGTO_HAMMING: return hamming_u8((const uint8_t *)pa, (const uint8_t *)pb, dp);
      case NGTO_JACCARD: return jaccard_u8((const uint8_t *)pa, (const uint8_t *)pb, dp);
      default: return l2_f32(a, b, dp);
    }
  } else {
    const uint8_t *a = (const uint8_t *)pa, *b = (const uint8_t *)pb;
    switch (metric) {
      case NGTO_L1: return l1_u8(a, b, dp);
      case NGTO_L2: return l2_u8(a, b, dp);
      case NGTO_HAMMING: return hamming_u8(a, b, dp);
      case NGTO_JACCARD: return jaccard_u8(a, b, dp);
      case NGTO_ANGLE: return angle_of(cosine_u8(a, b, dp));
      case NGTO_COSINE: return 1.0 - cosine_u8(a, b, dp);
      case NGTO_NORMALIZED_ANGLE: return angle_of(dot_u8(a, b, dp));
      case NGTO_NORMALIZED_COSINE: {
        double v = 1.0 - dot_u8(a, b, dp);
        return v < 0.0 ? 0.0 : v;
      }
      case NGTO_NORMALIZED_L2: {
        double v = 2.0 - 2.0 * dot_u8(a, b, dp);
        return v < 0.0 ? 0.0 : sqrt(v);
      }
      case NGTO_POINCARE: return poincare_u8(a, b, dp);
      case NGTO_LORENTZ: return lorentz_u8(a, b, dp);
      default: return l2_u8(a, b, dp);
    }
  }
}

float ngto_distance(int metric, int otype, const void *a, const void *b, size_t dp) {
  return (float)compare(metric, otype, a, b, dp);
}

void ngto_distances(int metric, int otype, const void *query, const void *rows,
                    size_t row_bytes, const uint32_t *ids, size_t n, size_t dp,
                    float *out) {
  for (size_t i = 0; i < n; i++)
    out[i] = ngto_distance(metric, otype, query,
                           (const uint8_t *)rows + (size_t)ids[i] * row_bytes, dp);
}

/* ObjectSpace::normalize<float> (ObjectSpace.h:251-266) as the reference's
 * -Ofast AVX-512 build vectorizes the sum: 16 FMA lanes over the unpadded
 * dimension, folded 8/4/2/1, then a sequential FMA tail.  The reference then
 * scales by vrsqrtss + one Newton step (host-CPU-dependent bits, so parity is
 * within 2 ulp, tests/golden/norm_f_d*.npz); this restatement -- like the
 * device preparation -- takes sqrtf and divides. */
int ngto_normalize_f32(float *v, size_t dim) {
  float acc[16] = {0};
  const size_t main = dim & ~(size_t)15;
  for (size_t i = 0; i < main; i++) acc[i & 15] = fmaf(v[i], v[i], acc[i & 15]);
  for (int w = 8; w >= 1; w >>= 1)
    for (int l = 0; l < w; l++) acc[l] = acc[l + w] + acc[l];
  float sum = acc[0];
  for (size_t i = main; i < dim; i++) sum = fmaf(v[i], v[i], sum);
  if (sum == 0.0f) return -1;
  sum = sqrtf(sum);
  for (size_t i = 0; i < dim; i++) v[i] = v[i] / sum;
  return 0;
}

/* ------------------------------------------------------------------------- */
/* (distance, id) heaps -- ObjectDistance ordering (Common.h:1946-1959).      */
/* ------------------------------------------------------------------------- */

typedef struct { uint32_t id; float d; } od_t;

static int od_less(od_t x, od_t y) { return x.d == y.d ? x.id < y.id : x.d < y.d; }

typedef struct { od_t *v; size_t n, cap; int max_heap; } heap_t;

static int heap_before(const heap_t *h, od_t x, od_t y) {
  return h->max_heap ? od_less(y, x) : od_less(x, y);
}
static void heap_push(heap_t *h, od_t x) {
  if (h->n == h->cap) {
    h->cap = h->cap ? h->cap * 2 : 64;
    h->v = (od_t *)realloc(h->v, h->cap * sizeof(od_t));
  }
  size_t i = h->n++;
  while (i > 0) {
    size_t p = (i - 1) / 2;
    if (!heap_before(h, x, h->v[p])) break;
    h->v[i] = h->v[p];
    i = p;
  }
  h->v[i] = x;
}
static od_t heap_pop(heap_t *h) {
  od_t top = h->v[0], x = h->v[--h->n];
  size_t i = 0;
  for (;;) {
    size_t c = 2 * i + 1;
    if (c >= h->n) break;
    if (c + 1 < h->n && heap_before(h, h->v[c + 1], h->v[c])) c++;
    if (!heap_before(h, h->v[c], x)) break;
    h->v[i] = h->v[c];
    i = c;
  }
  if (h->n) h->v[i] = x;
  return top;
}

static int od_cmp(const void *pa, const void *pb) {
  od_t a = *(const od_t *)pa, b = *(const od_t *)pb;
  return od_less(a, b) ? -1 : (od_less(b, a) ? 1 : 0);
}

/* Drain a max-heap into ascending order: ObjectDistances::moveFrom
 * (ObjectSpace.h:49-57). */
static int drain(heap_t *res, uint32_t *ids, float *dists) {
  int n = (int)res->n;
  for (int i = n - 1; i >= 0; i--) {
    od_t t = heap_pop(res);
    ids[i] = t.id;
    dists[i] = t.d;
  }
  return n;
}

int ngto_search(int metric, int otype, const void *rows, size_t row_bytes,
                size_t nrows, size_t dp, const uint64_t *edge_off,
                const uint32_t *edge_ids, const void *query,
                const uint32_t *seeds, size_t nseeds, size_t k, float epsilon,
                float radius_in, size_t edge_size, uint32_t *out_ids,
                float *out_dists, uint64_t *counters) {
  const uint8_t *base = (const uint8_t *)rows;
  /* SearchContainer::setEpsilon (Common.h:2041) and the 0 => 1.1 default
   * (Graph.cpp:403-405). */
  float coef = (float)((double)epsilon + 1.0);
  if (coef == 0.0f) coef = (float)1.1;
  float radius = radius_in;
  if (edge_size == 0) edge_size = (size_t)INT_MAX;
  uint64_t ndist = 0, nvisit = 0, nexp = 0;
  if (k == 0) { if (counters) counters[0] = counters[1] = counters[2] = 0; return 0; }

  uint8_t *checked = (uint8_t *)calloc(nrows, 1);
  heap_t unchecked = {0, 0, 0, 0}, results = {0, 0, 0, 1};

  /* setupDistances (Graph.cpp:293-338) + setupSeeds (Graph.cpp:341-367). */
  od_t *sd = (od_t *)malloc((nseeds ? nseeds : 1) * sizeof(od_t));
  for (size_t i = 0; i < nseeds; i++) {
    sd[i].id = seeds[i];
    sd[i].d = ngto_distance(metric, otype, query, base + (size_t)seeds[i] * row_bytes, dp);
  }
  ndist += nseeds;
  qsort(sd, nseeds, sizeof(od_t), od_cmp);
  for (size_t i = 0; i < nseeds; i++) {
    if (results.n < k && sd[i].d <= radius) heap_push(&results, sd[i]);
    else break;
  }
  if (results.n >= k) radius = results.v[0].d;
  for (size_t i = 0; i < nseeds; i++) {
    checked[sd[i].id] = 1;
    heap_push(&unchecked, sd[i]);
  }
  free(sd);

  /* The best-first loop (Graph.cpp:420-486). */
  float expr = coef * radius;
  uint32_t *ns = NULL;
  size_t ns_cap = 0;
  while (unchecked.n) {
    od_t target = heap_pop(&unchecked);
    if (target.d > expr) break;
    nexp++;
    uint64_t beg = edge_off[target.id], end = edge_off[target.id + 1];
    size_t deg = (size_t)(end - beg);
    if (deg > edge_size) deg = edge_size;
    if (deg > ns_cap) { ns_cap = deg; ns = (uint32_t *)realloc(ns, ns_cap * sizeof(uint32_t)); }
    size_t nns = 0;
    for (size_t e = 0; e < deg; e++)
      if (!checked[edge_ids[beg + e]]) ns[nns++] = edge_ids[beg + e];
    for (size_t i = 0; i < nns; i++) {
      uint32_t id = ns[i];
      nvisit++;
      checked[id] = 1;
      ndist++;
      float d = ngto_distance(metric, otype, query, base + (size_t)id * row_bytes, dp);
      if (d <= expr) {
        od_t r = {id, d};
        heap_push(&unchecked, r);
        if (d <= radius) {
          heap_push(&results, r);
          if (results.n >= k) {
            if (results.n > k) heap_pop(&results);
            radius = results.v[0].d;
            expr = coef * radius;
          }
        }
      }
    }
  }
  int n = drain(&results, out_ids, out_dists);
  free(ns);
  free(unchecked.v);
  free(results.v);
  free(checked);
  if (counters) {
    counters[0] = ndist;
    counters[1] = nvisit;
    counters[2] = nexp;
  }
  return n;
}

int ngto_linear_search(int metric, int otype, const void *rows, size_t row_bytes,
                       size_t nrows, size_t dp, const uint8_t *valid,
                       const void *query, size_t k, double radius,
                       uint32_t *out_ids, float *out_dists) {
  heap_t results = {0, 0, 0, 1};
  const uint8_t *base = (const uint8_t *)rows;
  for (size_t idx = 1; idx < nrows; idx++) {
    if (valid && !valid[idx]) continue;
    float d = ngto_distance(metric, otype, query, base + idx * row_bytes, dp);
    if (radius < 0.0 || d <= radius) {
      od_t r = {(uint32_t)idx, d};
      heap_push(&results, r);
      if (results.n > k) heap_pop(&results);
    }
  }
  int n = drain(&results, out_ids, out_dists);
  free(results.v);
  return n;
}

/* glibc srandom_r / random_r for TYPE_3 (degree 31, separation 3). */
void ngto_srand(ngto_rand_t *g, unsigned seed) {
  int32_t word = (int32_t)(seed == 0 ? 1 : seed);
  g->s[0] = (uint32_t)word;
  for (int i = 1; i < 31; i++) {
    int32_t hi = word / 127773, lo = word % 127773;
    word = 16807 * lo - 2836 * hi;
    if (word < 0) word += 2147483647;
    g->s[i] = (uint32_t)word;
  }
  g->f = 3;
  g->r = 0;
  for (int i = 0; i < 310; i++) ngto_rand(g);
}

int ngto_rand(ngto_rand_t *g) {
  g->s[g->f] += g->s[g->r];
  int res = (int)((g->s[g->f] >> 1) & 0x7fffffff);
  g->f = (g->f + 1) % 31;
  g->r = (g->r + 1) % 31;
  return res;
}

size_t ngto_thin_seeds(uint32_t *seeds, size_t n, unsigned leaf_id,
                       size_t seed_size, size_t k) {
  size_t ss = seed_size == 0 ? k : seed_size;
  if (ss > k) ss = k;
  if (n > ss) {
    ngto_rand_t g;
    ngto_srand(&g, leaf_id);
    for (size_t i = n; i > ss; i--) {
      double random = ((double)ngto_rand(&g) + 1.0) / ((double)RAND_MAX + 2.0);
      size_t idx = (size_t)floor((double)i * random);
      seeds[idx] = seeds[i - 1];
    }
    return ss;
  }
  return n;
}

uint32_t ngto_tree_leaf(int metric, int otype, const void *query, size_t dp,
                        uint32_t root, const void *in_pivot, size_t row_bytes,
                        const uint32_t *in_child, const float *in_border,
                        size_t children, uint64_t *ndist) {
  uint32_t node = root;
  uint64_t nd = 0;
  while (!(node & 0x80000000u)) {
    uint32_t iid = node & 0x7fffffffu;
    float d = ngto_distance(metric, otype, query,
                            (const uint8_t *)in_pivot + (size_t)iid * row_bytes, dp);
    nd++;
    const float *borders = in_border + (size_t)iid * (children - 1);
    size_t mid;
    /* radius = 0: the first region with d < border, else the last one
     * (Tree.cpp:424-456, regions sorted, front taken at :468). */
    for (mid = 0; mid < children - 1; mid++)
      if (d < borders[mid]) break;
    node = in_child[(size_t)iid * children + mid];
  }
  if (ndist) *ndist = nd;
  return node;
}

/* ------------------------------------------------------------------------- */
/* NGTQG: uint8 LUT, 4-bit ADC, quantized-graph search.                       */
/* ------------------------------------------------------------------------- */

void ngto_qg_lut(const float *query, const float *global, const float *local, size_t M,
                 size_t dsub, uint8_t *lut, float *scale, float *total_offset) {
  /* createFloatL2DistanceLookup (Quantizer.h:683-706): per subspace li and
   * centroid k = 1..16, d = sum over the subvector of (q - g - c)^2 in float.
   * The reference build contracts `d += sub * sub` into an FMA chain
   * (-Ofast); pinned by tests/golden/d20_qg (dsub = 4). */
  size_t Me = (M + 1) / 2 * 2;
  float *d = (float *)malloc(M * 16 * sizeof(float));
  float mn = FLT_MAX, mx = -FLT_MAX;
  for (size_t li = 0; li < M; li++) {
    const float *q = query + li * dsub, *g = global + li * dsub;
    for (size_t c = 1; c <= 16; c++) {
      const float *lc = local + (li * 17 + c) * dsub;
      float acc = 0.0f;
      for (size_t j = 0; j < dsub; j++) {
        float sub = q[j] - g[j] - lc[j];
        acc = fmaf(sub, sub, acc);
      }
      d[li * 16 + c - 1] = acc;
      /* one global min/max over every subspace (:724-736) */
      if (acc > mx) mx = acc;
      if (acc < mn) mn = acc;
    }
  }
  float offset = mn;
  float sc = (float)((double)(mx - mn) / 255.0);  /* (:738) */
  float tot = 0.0f;
  for (size_t li = 0; li < M; li++) {
    for (size_t c = 0; c < 16; c++) {
      int32_t t = (int32_t)roundf((d[li * 16 + c] - offset) / sc);  /* (:742) */
      lut[li * 16 + c] = (uint8_t)t;
    }
    tot += offset;  /* totalOffset (:749) */
  }
  for (size_t li = M; li < Me; li++) memset(lut + li * 16, 0, 16);  /* odd M pad (:751-757) */
  free(d);
  *scale = sc;
  *total_offset = tot;
}

void ngto_qg_adc(const uint8_t *codes, size_t n, const uint8_t *lut, size_t M, float scale,
                 float total_offset, float *out) {
  /* Block of 16 objects = 8*Me bytes: subspace m's 16 nibbles sit at bytes
   * [8m, 8m+8), object 2j in the low nibble of byte j, 2j+1 in the high
   * (QuantizedObjectProcessingStream, Quantizer.h:1295-1327).  The AVX-512
   * loop keeps two u16 accumulators per object -- even subspaces in one,
   * odd in the other -- with saturating adds (_mm512_adds_epu16, :986-1007);
   * unsigned saturating adds of non-negative terms equal min(sum, 65535).
   * Epilogue: sqrt(fma(float(E + O), scale, totalOffset)) (:1020-1031; the
   * -Ofast build contracts mul+add into vfmadd). */
  size_t Me = (M + 1) / 2 * 2;
  size_t nb = n == 0 ? 0 : (n - 1) / 16 + 1;
  for (size_t b = 0; b < nb; b++) {
    const uint8_t *blk = codes + b * 8 * Me;
    for (size_t i = 0; i < 16 && b * 16 + i < n; i++) {
      uint32_t e = 0, o = 0;
      for (size_t m = 0; m < Me; m++) {
        uint8_t byte = blk[8 * m + i / 2];
        uint32_t code = (i & 1) ? (byte >> 4) : (byte & 15);
        uint32_t v = lut[m * 16 + code];
        if (m & 1) o += v; else e += v;
      }
      if (e > 65535) e = 65535;
      if (o > 65535) o = 65535;
      out[b * 16 + i] = sqrtf(fmaf((float)(e + o), scale, total_offset));
    }
  }
}

int ngto_qg_search(const float *rows, size_t dp, size_t nrows, const uint64_t *qoff,
                   const uint32_t *qids, const uint64_t *code_off, const uint8_t *codes, size_t M,
                   const uint8_t *lut, float scale, float total_offset, const float *query,
                   const uint32_t *seeds, size_t nseeds, size_t k, float epsilon,
                   float result_expansion, float radius, uint32_t *out_ids, float *out_dists,
                   uint64_t *counters) {
  /* sc.size *= resultExpansion: size_t * float -> float -> size_t (:194-196) */
  size_t size = k;
  if (result_expansion > 1.0f) size = (size_t)((float)size * result_expansion);
  float coef = (float)((double)epsilon + 1.0);
  if (coef == 0.0f) coef = (float)1.1;  /* (:207-209) */
  uint64_t nadc = 0, nacc = 0, nexp = 0, nexact = 0;
  if (size == 0) {
    if (counters) counters[0] = counters[1] = counters[2] = counters[3] = 0;
    return 0;
  }
  uint8_t *checked = (uint8_t *)calloc(nrows, 1);
  heap_t unchecked = {0, 0, 0, 0}, results = {0, 0, 0, 1};

  /* setupDistances with the exact L2 comparator (:214) + setupSeeds (:215) */
  od_t *sd = (od_t *)malloc((nseeds ? nseeds : 1) * sizeof(od_t));
  for (size_t i = 0; i < nseeds; i++) {
    sd[i].id = seeds[i];
    sd[i].d = ngto_distance(NGTO_L2, NGTO_FLOAT, query, rows + (size_t)seeds[i] * dp, dp);
  }
  nexact += nseeds;
  qsort(sd, nseeds, sizeof(od_t), od_cmp);
  for (size_t i = 0; i < nseeds; i++) {
    if (results.n < size && sd[i].d <= radius) heap_push(&results, sd[i]);
    else break;
  }
  if (results.n >= size) radius = results.v[0].d;
  for (size_t i = 0; i < nseeds; i++) {
    checked[sd[i].id] = 1;
    heap_push(&unchecked, sd[i]);
  }
  free(sd);

  float expr = coef * radius;  /* (:216) */
  float *ds = NULL;
  size_t ds_cap = 0;
  while (unchecked.n) {
    od_t target = heap_pop(&unchecked);
    if (target.d > expr) break;  /* (:223-225) */
    nexp++;
    size_t nn = (size_t)(qoff[target.id + 1] - qoff[target.id]);
    if (nn > ds_cap) { ds_cap = nn; ds = (float *)realloc(ds, ds_cap * sizeof(float)); }
    ngto_qg_adc(codes + code_off[target.id], nn, lut, M, scale, total_offset, ds);  /* (:240) */
    nadc += nn;
    const uint32_t *nid = qids + qoff[target.id];
    for (size_t i = 0; i < nn; i++) {  /* (:241-266) */
      float d = ds[i];
      if (d <= expr) {
        if (checked[nid[i]]) continue;
        checked[nid[i]] = 1;
        nacc++;
        od_t r = {nid[i], d};
        heap_push(&unchecked, r);
        if (d <= radius) {
          heap_push(&results, r);
          if (results.n >= size) {
            if (results.n > size) heap_pop(&results);
            radius = results.v[0].d;
            expr = coef * radius;
          }
        }
      }
    }
  }
  free(ds);
  free(unchecked.v);
  free(checked);

  size_t nres = results.n;
  uint32_t *ids = (uint32_t *)malloc((nres ? nres : 1) * sizeof(uint32_t));
  float *dd = (float *)malloc((nres ? nres : 1) * sizeof(float));
  drain(&results, ids, dd);  /* moveFrom (:272) */
  free(results.v);
  int n;
  if (result_expansion >= 1.0f) {
    /* exact rerank with the index comparator, sort, resize to k (:273-299) */
    od_t *rr = (od_t *)malloc((nres ? nres : 1) * sizeof(od_t));
    for (size_t i = 0; i < nres; i++) {
      rr[i].id = ids[i];
      rr[i].d = ngto_distance(NGTO_L2, NGTO_FLOAT, query, rows + (size_t)ids[i] * dp, dp);
    }
    nexact += nres;
    qsort(rr, nres, sizeof(od_t), od_cmp);
    for (size_t i = 0; i < k; i++) {
      out_ids[i] = i < nres ? rr[i].id : 0u;
      out_dists[i] = i < nres ? rr[i].d : 0.0f;
    }
    free(rr);
    n = (int)k;
  } else {
    for (size_t i = 0; i < nres; i++) {
      out_ids[i] = ids[i];
      out_dists[i] = dd[i];
    }
    n = (int)nres;
  }
  free(ids);
  free(dd);
  if (counters) {
    counters[0] = nadc;
    counters[1] = nacc;
    counters[2] = nexp;
    counters[3] = nexact;
  }
  return n;
}

/* ------------------------------------------------------------------------- */
/* Query batches, one query per thread -- the CPU baseline bench.py times and */
/* the parity sample it checks the device against.  Each query is the single- */
/* query function above, so results do not depend on the thread count.        */
/* ------------------------------------------------------------------------- */

void ngto_search_batch(int metric, int otype, const void *rows, size_t row_bytes, size_t nrows, size_t dp,
                       const uint64_t *edge_off, const uint32_t *edge_ids, const void *queries,
                       size_t query_bytes, size_t nq, const uint32_t *seeds, const uint64_t *seed_off, size_t k,
                       float epsilon, float radius, size_t edge_size, uint32_t *out_ids, float *out_dists,
                       uint32_t *out_n, uint64_t *counters, int nthreads) {
  long q;
#ifdef _OPENMP
#pragma omp parallel for schedule(dynamic, 1) num_threads(nthreads > 0 ? nthreads : 1)
#endif
  for (q = 0; q < (long)nq; q++) {
    uint64_t c[3] = {0, 0, 0};
    int n = ngto_search(metric, otype, rows, row_bytes, nrows, dp, edge_off, edge_ids,
                        (const uint8_t *)queries + (size_t)q * query_bytes, seeds + seed_off[q],
                        (size_t)(seed_off[q + 1] - seed_off[q]), k, epsilon, radius, edge_size,
                        out_ids + (size_t)q * k, out_dists + (size_t)q * k, c);
    out_n[q] = (uint32_t)n;
    if (counters) memcpy(counters + 3 * (size_t)q, c, sizeof c);
  }
  (void)nthreads;
}

void ngto_linear_search_batch(int metric, int otype, const void *rows, size_t row_bytes, size_t nrows, size_t dp,
                              const void *queries, size_t query_bytes, size_t nq, size_t k, double radius,
                              uint32_t *out_ids, float *out_dists, uint32_t *out_n, int nthreads) {
  long q;
#ifdef _OPENMP
#pragma omp parallel for schedule(dynamic, 1) num_threads(nthreads > 0 ? nthreads : 1)
#endif
  for (q = 0; q < (long)nq; q++)
    out_n[q] = (uint32_t)ngto_linear_search(metric, otype, rows, row_bytes, nrows, dp, NULL,
                                            (const uint8_t *)queries + (size_t)q * query_bytes, k, radius,
                                            out_ids + (size_t)q * k, out_dists + (size_t)q * k);
  (void)nthreads;
}

void ngto_qg_search_batch(const float *rows, size_t dp, size_t nrows, const uint64_t *qoff, const uint32_t *qids,
                          const uint64_t *code_off, const uint8_t *codes, size_t M, const uint8_t *luts,
                          size_t lut_stride, const float *scales, const float *offsets, const float *queries,
                          size_t nq, const uint32_t *seeds, const uint64_t *seed_off, size_t k, float epsilon,
                          float result_expansion, float radius, size_t out_stride, uint32_t *out_ids,
                          float *out_dists, uint32_t *out_n, uint64_t *counters, int nthreads) {
  long q;
#ifdef _OPENMP
#pragma omp parallel for schedule(dynamic, 1) num_threads(nthreads > 0 ? nthreads : 1)
#endif
  for (q = 0; q < (long)nq; q++) {
    uint64_t c[4] = {0, 0, 0, 0};
    int n = ngto_qg_search(rows, dp, nrows, qoff, qids, code_off, codes, M, luts + (size_t)q * lut_stride,
                           scales[q], offsets[q], queries + (size_t)q * dp, seeds + seed_off[q],
                           (size_t)(seed_off[q + 1] - seed_off[q]), k, epsilon, result_expansion, radius,
                           out_ids + (size_t)q * out_stride, out_dists + (size_t)q * out_stride, c);
    out_n[q] = (uint32_t)n;
    if (counters) memcpy(counters + 4 * (size_t)q, c, sizeof c);
  }
  (void)nthreads;
}

/* ---------------------------------------------------------------------------
 * NGTQ IVF-ADC (lib/NGT/NGTQ/Quantizer.h).  The per-(subspace, centroid)
 * residual terms follow the instruction sequences of the reference's
 * -Ofast -march=native build (objdump of createFloatL2DistanceLookup,
 * QuantizedObjectDistanceFloat::operator()(Object&, size_t, void*[, LUT&])),
 * pinned by tests/golden/ngtq_n{8,16,32}.
 * ------------------------------------------------------------------------- */

/* createFloatL2DistanceLookup (:683-706): float d over the subvector. */
static float ngtq_lut_l(const float *o, const float *g, const float *l, size_t dsub) {
  float acc = 0.0f;
  size_t i = 0;
  if (dsub >= 16) {
    float a[16] = {0};
    for (; i + 16 <= dsub; i += 16)
      for (int j = 0; j < 16; j++) {
        float s = o[i + j] - (g[i + j] + l[i + j]);
        a[j] = fmaf(s, s, a[j]);
      }
    for (int h = 8; h >= 1; h >>= 1)
      for (int j = 0; j < h; j++) a[j] = a[j + h] + a[j];
    acc = a[0];
  }
  if (dsub - i >= 8) {
    float b[8];
    for (int j = 0; j < 8; j++) {
      float s = (o[i + j] - l[i + j]) - g[i + j];
      b[j] = s * s;
    }
    for (int h = 4; h >= 1; h >>= 1)
      for (int j = 0; j < h; j++) b[j] = b[j + h] + b[j];
    acc = acc + b[0];
    i += 8;
  }
  for (; i < dsub; i++) {
    float s = o[i] - (g[i] + l[i]);
    acc = fmaf(s, s, acc);
  }
  return acc;
}

/* operator()(Object&, size_t, void*, DistanceLookupTable&) (:1102-1153): the
 * 8-lane AVX block loop (dsub a multiple of 8). */
static double ngtq_sub_c(const float *o, const float *g, const float *l, size_t dsub) {
  float a[8] = {0};
  for (size_t i = 0; i < dsub; i += 8)
    for (int j = 0; j < 8; j++) {
      float s = o[i + j] - (g[i + j] + l[i + j]);
      a[j] = fmaf(s, s, a[j]);
    }
  float x[4];
  for (int j = 0; j < 4; j++) x[j] = a[j] + a[j + 4];
  return (double)((x[0] + x[1]) + (x[3] + x[2]));
}

/* getL2DistanceFloat (:579-608): the per-subspace double sum. */
static double ngtq_sub_a(const float *o, const float *g, const float *l, size_t dsub) {
  double d = 0.0;
  size_t i = 0;
  if (dsub >= 16) {
    double a[8] = {0};
    for (; i + 16 <= dsub; i += 16)
      for (int j = 0; j < 8; j++) {
        double lo = (double)(o[i + j] - (g[i + j] + l[i + j]));
        double hi = (double)(o[i + j + 8] - (g[i + j + 8] + l[i + j + 8]));
        a[j] = a[j] + fma(lo, lo, hi * hi);
      }
    for (int h = 4; h >= 1; h >>= 1)
      for (int j = 0; j < h; j++) a[j] = a[j + h] + a[j];
    d = a[0];
  }
  if (dsub - i >= 8) {
    double t[4];
    for (int j = 0; j < 4; j++) {
      double lo = (double)(o[i + j] - (g[i + j] + l[i + j]));
      double hi = (double)(o[i + j + 4] - (g[i + j + 4] + l[i + j + 4]));
      t[j] = fma(lo, lo, hi * hi);
    }
    d = d + ((t[3] + t[1]) + (t[2] + t[0]));
    i += 8;
  }
  for (; i < dsub; i++) {
    double s = (double)(o[i] - (g[i] + l[i]));
    d = fma(s, s, d);
  }
  return d;
}

static int od_cmp_desc(const void *pa, const void *pb) { return -od_cmp(pa, pb); }

size_t ngto_ngtq_aggregate(int mode, const float *query, size_t dp, const uint32_t *cent_ids,
                           const float *cent_d, size_t ncent, const float *grows, const float *local, size_t N,
                           size_t dsub, const uint64_t *list_off, size_t nlists, const uint32_t *eids,
                           const uint16_t *elids, const float *orows, size_t size, uint64_t ass,
                           uint32_t *out_ids, float *out_d) {
  /* the ResultSet of QuantizerInstance::search (:2508-2531): every aggregated
   * entry, later popped into ascending order and cut to `size` */
  size_t cap = 1024, n = 0;
  od_t *all = (od_t *)malloc(cap * sizeof(od_t));
  double *tab = (double *)malloc(N * 17 * sizeof(double));
  for (size_t ci = 0; ci < ncent; ci++) {
    uint32_t gid = cent_ids[ci];
    if (gid >= nlists) continue; /* invertedIndex[id] == 0 (:2425-2430) */
    uint64_t lo = list_off[gid], len = list_off[gid + 1] - lo;
    /* limit INT_MAX while the result set is empty (:2432) */
    uint64_t lim = n == 0 ? (uint64_t)INT_MAX : ass;
    const float *g = grows + (size_t)gid * dp;
    if (mode != 4)
      for (size_t li = 0; li < N; li++)
        for (size_t k = 1; k <= 16; k++) {
          const float *o = query + li * dsub, *gg = g + li * dsub, *l = local + (li * 17 + k) * dsub;
          tab[li * 17 + k] = mode == 1 ? (double)ngtq_lut_l(o, gg, l, dsub)
                                       : (mode == 0 ? ngtq_sub_a(o, gg, l, dsub) : ngtq_sub_c(o, gg, l, dsub));
        }
    for (uint64_t j = 0; j < len && n < lim; j++) {
      uint64_t e = lo + j;
      const uint16_t *lid = elids + e * N;
      float d;
      if (lid[0] == 0) {
        d = cent_d[ci]; /* the object is the centroid (:2275-2277) */
      } else if (mode == 4) {
        d = ngto_distance(NGTO_L2, NGTO_FLOAT, query, orows + (size_t)eids[e] * dp, dp);
      } else {
        double s = 0.0;
        for (size_t li = 0; li < N; li++) s = s + tab[li * 17 + lid[li]];
        d = (float)sqrt(s);
      }
      if (n == cap) {
        cap *= 2;
        all = (od_t *)realloc(all, cap * sizeof(od_t));
      }
      all[n].id = eids[e];
      all[n].d = d;
      n++;
    }
    if (n >= ass) break;
  }
  qsort(all, n, sizeof(od_t), od_cmp);
  size_t m = n < size ? n : size;
  if (mode == 3) { /* refineDistance (:2450-2460) */
    for (size_t i = 0; i < m; i++) all[i].d = ngto_distance(NGTO_L2, NGTO_FLOAT, query, orows + (size_t)all[i].id * dp, dp);
    qsort(all, m, sizeof(od_t), od_cmp);
  }
  for (size_t i = 0; i < m; i++) {
    out_ids[i] = all[i].id;
    out_d[i] = all[i].d;
  }
  free(all);
  free(tab);
  (void)od_cmp_desc;
  return m;
}

double ngto_ngtq_term(int mode, const float *o, const float *g, const float *l, size_t dsub) {
  return mode == 1 ? (double)ngtq_lut_l(o, g, l, dsub) : (mode == 0 ? ngtq_sub_a(o, g, l, dsub) : ngtq_sub_c(o, g, l, dsub));
}
