/* capi_threads.c -- the reference's own call pattern against the drop-in C
 * API: T threads, each issuing single-query ngt_search_index calls
 * (lib/NGT/Capi.cpp:377-406) on one handle opened with ngt_open_index, as an
 * ann-benchmarks style server would.  bench.py --mode capi runs it (no Python
 * between the callers and the library).
 *
 *   capi_threads <index_dir> <queries.f32> <nq> <dim> <k> <epsilon> <threads>
 *                <calls_per_thread> <ids_out.u32>
 *
 * queries.f32: nq x dim float32 rows; thread t issues queries
 * (t * calls + i) mod nq.  ids_out: [threads * calls][k] uint32 result ids
 * (0 padded) for the recall check.  Prints one JSON object. */
#include <math.h>
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "NGT/Capi.h"

static NGTIndex g_index;
static const float* g_q;
static int g_nq, g_dim, g_k, g_calls;
static float g_eps;
static uint32_t* g_ids;
static double* g_lat;
static pthread_barrier_t g_bar;
static int g_failed;

static double now_s(void) {
  struct timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return ts.tv_sec + ts.tv_nsec * 1e-9;
}

static void* worker(void* arg) {
  const int t = (int)(intptr_t)arg;
  NGTError err = ngt_create_error_object();
  NGTObjectDistances res = ngt_create_empty_results(err);
  double* q = (double*)malloc(sizeof(double) * g_dim);
  pthread_barrier_wait(&g_bar);
  for (int i = 0; i < g_calls; i++) {
    const int call = t * g_calls + i;
    const float* src = g_q + (size_t)(call % g_nq) * g_dim;
    for (int d = 0; d < g_dim; d++) q[d] = src[d];
    const double t0 = now_s();
    if (!ngt_search_index(g_index, q, g_dim, g_k, g_eps, -1.0f, res, err)) {
      fprintf(stderr, "ngt_search_index: %s\n", ngt_get_error_string(err));
      g_failed = 1;
      break;
    }
    g_lat[call] = now_s() - t0;
    const uint32_t n = ngt_get_result_size(res, err);
    for (uint32_t j = 0; j < n && j < (uint32_t)g_k; j++) g_ids[(size_t)call * g_k + j] = ngt_get_result(res, j, err).id;
  }
  pthread_barrier_wait(&g_bar);
  free(q);
  ngt_destroy_results(res);
  ngt_destroy_error_object(err);
  return NULL;
}

static int cmp_d(const void* a, const void* b) {
  const double x = *(const double*)a, y = *(const double*)b;
  return x < y ? -1 : x > y;
}

int main(int argc, char** argv) {
  if (argc != 10) {
    fprintf(stderr, "usage: %s index queries.f32 nq dim k epsilon threads calls ids_out\n", argv[0]);
    return 2;
  }
  g_nq = atoi(argv[3]);
  g_dim = atoi(argv[4]);
  g_k = atoi(argv[5]);
  g_eps = (float)atof(argv[6]);
  const int threads = atoi(argv[7]);
  g_calls = atoi(argv[8]);
  FILE* f = fopen(argv[2], "rb");
  if (!f) return 2;
  float* q = (float*)malloc(sizeof(float) * (size_t)g_nq * g_dim);
  if (fread(q, sizeof(float), (size_t)g_nq * g_dim, f) != (size_t)g_nq * g_dim) return 2;
  fclose(f);
  g_q = q;
  NGTError err = ngt_create_error_object();
  g_index = ngt_open_index(argv[1], err);
  if (!g_index) {
    fprintf(stderr, "ngt_open_index: %s\n", ngt_get_error_string(err));
    return 1;
  }
  const size_t total = (size_t)threads * g_calls;
  g_ids = (uint32_t*)calloc(total * g_k, sizeof(uint32_t));
  g_lat = (double*)calloc(total, sizeof(double));
  /* warm the handle (device index, filter copy, per-stream contexts) */
  {
    NGTObjectDistances res = ngt_create_empty_results(err);
    double* w = (double*)malloc(sizeof(double) * g_dim);
    for (int d = 0; d < g_dim; d++) w[d] = q[d];
    for (int i = 0; i < 3; i++) ngt_search_index(g_index, w, g_dim, g_k, g_eps, -1.0f, res, err);
    free(w);
    ngt_destroy_results(res);
  }
  pthread_barrier_init(&g_bar, NULL, (unsigned)threads + 1);
  pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * threads);
  for (int t = 0; t < threads; t++) pthread_create(&th[t], NULL, worker, (void*)(intptr_t)t);
  pthread_barrier_wait(&g_bar);
  const double t0 = now_s();
  pthread_barrier_wait(&g_bar);
  const double wall = now_s() - t0;
  for (int t = 0; t < threads; t++) pthread_join(th[t], NULL);
  if (g_failed) return 1;
  FILE* o = fopen(argv[9], "wb");
  fwrite(g_ids, sizeof(uint32_t), total * g_k, o);
  fclose(o);
  uint64_t batches = 0, served = 0;
  ngt_get_coalesce_stats(g_index, &batches, &served, err);
  double sum = 0;
  for (size_t i = 0; i < total; i++) sum += g_lat[i];
  qsort(g_lat, total, sizeof(double), cmp_d);
  printf("{\"threads\": %d, \"calls\": %zu, \"wall_s\": %.6f, \"qps\": %.1f, \"latency_ms\": {\"mean\": %.4f, "
         "\"p50\": %.4f, \"p99\": %.4f}, \"launches\": %llu, \"served\": %llu}\n",
         threads, total, wall, total / wall, 1e3 * sum / total, 1e3 * g_lat[total / 2],
         1e3 * g_lat[(size_t)(0.99 * (total - 1))], (unsigned long long)batches, (unsigned long long)served);
  ngt_close_index(g_index);
  ngt_destroy_error_object(err);
  return 0;
}
