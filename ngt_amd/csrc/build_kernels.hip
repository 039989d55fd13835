// build_kernels.hip -- gfx950 kernels of ANNG construction
// (GraphAndTreeIndex::createIndex, lib/NGT/Index.cpp:1158-1257).
//
//  * ngt_tree_insert_kernel : DVPTree::insert for one creation batch, in batch
//    order (lib/NGT/Tree.cpp:27-98): leaf descent, duplicate check, append,
//    and the leaf split -- selectPivotByMaxVariance (lib/NGT/Node.cpp:97-144),
//    splitObjects (:146-225) and recombineNodes (Tree.cpp:119-265).  The tree
//    lives in HBM (fixed-capacity node arrays); insertions are sequential by
//    definition (each may split the leaf the next one descends to), so one
//    wave runs the batch: every distance is one quad's comparator, and the
//    101 x 101 distance matrix of a split uses all 16 quads.
//  * ngt_adj_scatter_kernel : refresh rows of the padded search adjacency
//    (the first edgeSizeForSearch ids of each changed node).
#include <hip/hip_runtime.h>
#include <float.h>
#include <stdint.h>

#include "ngt_device.h"
#include "ngt_kernels.h"
#include "search_common.h"

namespace ngt_amd {

// Node.cpp:117-129 as the reference's -Ofast build (GCC, AVX2) evaluates it
// (read from its object code): the sums over a row of the distance matrix
// run in four double lanes, lane l adding x[8b + l] + x[8b + l + 4] per block
// of 8, folded (l1 + l3) + (l0 + l2); then one 4-element block
// ((y1 + y3) + (y0 + y2)) if at least 4 remain, then the rest one by one;
// pow(d, 2) is d * d contracted into FMAs (lane l: fma(lo, lo, hi * hi)), and
// both divisions by fsize are multiplies by its reciprocal.  The order matters
// when variances tie in real arithmetic (duplicate-heavy or symmetric data).
__device__ inline double pivot_variance(const float* x, uint32_t n) {
  const double inv = 1.0 / (double)n;
  const uint32_t n8 = n & ~7u;
  double s = 0.0;
  uint32_t j = 0;
  if (n > 7) {
    double a0 = 0.0, a1 = 0.0, a2 = 0.0, a3 = 0.0;
    for (uint32_t b = 0; b < n8; b += 8) {
      a0 += (double)x[b] + (double)x[b + 4];
      a1 += (double)x[b + 1] + (double)x[b + 5];
      a2 += (double)x[b + 2] + (double)x[b + 6];
      a3 += (double)x[b + 3] + (double)x[b + 7];
    }
    s = (a1 + a3) + (a0 + a2);
    j = n8;
    if (n - n8 >= 4) {
      s += ((double)x[j + 1] + (double)x[j + 3]) + ((double)x[j] + (double)x[j + 2]);
      j += 4;
    }
  }
  for (; j < n; j++) s += (double)x[j];
  const double avg = s * inv;
  double v = 0.0;
  j = 0;
  if (n > 7) {
    double a0 = 0.0, a1 = 0.0, a2 = 0.0, a3 = 0.0;
    for (uint32_t b = 0; b < n8; b += 8) {
      double lo, hi;
      lo = (double)x[b] - avg; hi = (double)x[b + 4] - avg; a0 += fma(lo, lo, hi * hi);
      lo = (double)x[b + 1] - avg; hi = (double)x[b + 5] - avg; a1 += fma(lo, lo, hi * hi);
      lo = (double)x[b + 2] - avg; hi = (double)x[b + 6] - avg; a2 += fma(lo, lo, hi * hi);
      lo = (double)x[b + 3] - avg; hi = (double)x[b + 7] - avg; a3 += fma(lo, lo, hi * hi);
    }
    v = (a1 + a3) + (a0 + a2);
    j = n8;
    if (n - n8 >= 4) {
      const double y0 = (double)x[j] - avg, y1 = (double)x[j + 1] - avg;
      const double y2 = (double)x[j + 2] - avg, y3 = (double)x[j + 3] - avg;
      v += fma(y1, y1, y3 * y3) + fma(y0, y0, y2 * y2);
      j += 4;
    }
  }
  for (; j < n; j++) {
    const double d = (double)x[j] - avg;
    v = fma(d, d, v);
  }
  return v * inv;
}


namespace {

constexpr uint32_t kLeaf = 0x80000000u;

template <int M, typename T>
__device__ __forceinline__ float quad_dist_rows(const uint8_t* a, const uint8_t* b, int dp, int g) {
  return quad_distance<M, T>(reinterpret_cast<const T*>(a), reinterpret_cast<const T*>(b), dp, g);
}

// One distance by quad 0, broadcast to the wave.
template <int M, typename T>
__device__ __forceinline__ float dist1(const uint8_t* a, const uint8_t* b, int dp) {
  const int lane = lane_id();
  float d = 0.f;
  if (lane < 4) d = quad_dist_rows<M, T>(a, b, dp, lane);
  return __shfl(d, 0, 64);
}

__device__ __forceinline__ void copy_row(uint8_t* dst, const uint8_t* src, uint64_t bytes) {
  const int lane = lane_id();
  for (uint64_t i = (uint64_t)lane * 4; i < bytes; i += 256)
    *reinterpret_cast<uint32_t*>(dst + i) = *reinterpret_cast<const uint32_t*>(src + i);
}

// ---- std::sort (libstdc++ introsort) over (distance) keys, lane 0 only -----
// Node::Object compares distances only (Node.h:66), so the order of equal
// distances is the one libstdc++'s algorithm leaves; it is restated here
// step for step (median-of-three to first, unguarded partition, threshold
// 16, final insertion sort).
struct SortItem {
  float d;
  uint32_t i;  // index into fs
};

__device__ __forceinline__ void iswap(SortItem* a, SortItem* b) {
  SortItem t = *a;
  *a = *b;
  *b = t;
}

__device__ void move_median_to_first(SortItem* result, SortItem* a, SortItem* b, SortItem* c) {
  if (a->d < b->d) {
    if (b->d < c->d) iswap(result, b);
    else if (a->d < c->d) iswap(result, c);
    else iswap(result, a);
  } else if (a->d < c->d) {
    iswap(result, a);
  } else if (b->d < c->d) {
    iswap(result, c);
  } else {
    iswap(result, b);
  }
}

__device__ SortItem* unguarded_partition(SortItem* first, SortItem* last, SortItem* pivot) {
  for (;;) {
    while (first->d < pivot->d) ++first;
    --last;
    while (pivot->d < last->d) --last;
    if (!(first < last)) return first;
    iswap(first, last);
    ++first;
  }
}

__device__ void unguarded_linear_insert(SortItem* last) {
  SortItem val = *last;
  SortItem* next = last - 1;
  while (val.d < next->d) {
    *last = *next;
    last = next;
    --next;
  }
  *last = val;
}

__device__ void insertion_sort(SortItem* first, SortItem* last) {
  if (first == last) return;
  for (SortItem* i = first + 1; i != last; ++i) {
    if (i->d < first->d) {
      SortItem val = *i;
      for (SortItem* p = i; p != first; --p) *p = *(p - 1);
      *first = val;
    } else {
      unguarded_linear_insert(i);
    }
  }
}

// libstdc++ heap sort of [first, last) (std::partial_sort(first, last, last):
// __make_heap + __sort_heap with __adjust_heap / __push_heap), used when the
// introsort depth limit is reached.
__device__ void adjust_heap(SortItem* first, int hole, int len, SortItem value) {
  const int top = hole;
  int second = hole;
  while (second < (len - 1) / 2) {
    second = 2 * (second + 1);
    if (first[second].d < first[second - 1].d) second--;
    first[hole] = first[second];
    hole = second;
  }
  if ((len & 1) == 0 && second == (len - 2) / 2) {
    second = 2 * (second + 1);
    first[hole] = first[second - 1];
    hole = second - 1;
  }
  int parent = (hole - 1) / 2;
  while (hole > top && first[parent].d < value.d) {
    first[hole] = first[parent];
    hole = parent;
    parent = (hole - 1) / 2;
  }
  first[hole] = value;
}

__device__ void heap_sort(SortItem* first, SortItem* last) {
  const int len = (int)(last - first);
  if (len < 2) return;
  for (int parent = (len - 2) / 2;; parent--) {
    adjust_heap(first, parent, len, first[parent]);
    if (parent == 0) break;
  }
  while (last - first > 1) {
    --last;
    SortItem value = *last;
    *last = *first;
    adjust_heap(first, 0, (int)(last - first), value);
  }
}

// std::sort: __introsort_loop (threshold 16, depth 2*lg(n)) then
// __final_insertion_sort.  Sub-ranges are disjoint, so processing them from
// an explicit stack instead of the recursion leaves the same result.
__device__ void std_sort(SortItem* first, SortItem* last) {
  const int n = (int)(last - first);
  if (n < 2) return;
  SortItem* sf[64];
  SortItem* sl[64];
  int sd[64];
  int sp = 0;
  sf[sp] = first; sl[sp] = last; sd[sp] = 2 * (31 - __clz(n)); sp++;
  while (sp) {
    sp--;
    SortItem* f = sf[sp];
    SortItem* l = sl[sp];
    int d = sd[sp];
    while (l - f > 16) {
      if (d == 0) {
        heap_sort(f, l);
        break;
      }
      --d;
      SortItem* mid = f + (l - f) / 2;
      move_median_to_first(f, f + 1, mid, l - 1);
      SortItem* cut = unguarded_partition(f + 1, l, f);
      sf[sp] = cut; sl[sp] = l; sd[sp] = d; sp++;
      l = cut;
    }
  }
  if (n > 16) {
    insertion_sort(first, first + 16);
    for (SortItem* i = first + 16; i != last; ++i) unguarded_linear_insert(i);
  } else {
    insertion_sort(first, last);
  }
}

}  // namespace

// ---------------------------------------------------------------------------
// DVPTree::insert for one batch, one 256-thread workgroup.  Wave 0 runs the
// sequential part (descent, duplicate check, append, the bookkeeping of a
// split); all four waves share a split's distance work.  LDS: fs ids / keys /
// cluster ids / leaf distances (101 each), sort items, variances, the
// 101 x 101 distance matrix (40.8 KB) and the batch's leaf replacements.
// ---------------------------------------------------------------------------
template <int M, typename T>
__global__ void __launch_bounds__(256) ngt_tree_insert_kernel(TreeBuildArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const int tid = threadIdx.x;
  const int lane = tid & 63, w = tid >> 6;
  const int g = tid & 3, bq = tid >> 2;  // 64 quads per workgroup
  constexpr int kQuads = 64;
  const uint32_t LS = a.leaf_size;  // leafObjectsSize (100)
  uint32_t* fs_id = reinterpret_cast<uint32_t*>(smem);
  float* fs_dist = reinterpret_cast<float*>(fs_id + 128);
  float* fs_ld = fs_dist + 128;
  int* fs_cl = reinterpret_cast<int*>(fs_ld + 128);
  SortItem* items = reinterpret_cast<SortItem*>(fs_cl + 128);
  double* var = reinterpret_cast<double*>(items + 128);
  float* D = reinterpret_cast<float*>(var + 128);  // [NF][NF]
  uint32_t* repl_leaf = reinterpret_cast<uint32_t*>(D + (size_t)(LS + 1) * (LS + 1));  // [256]
  uint32_t* repl_in = repl_leaf + 256;                                                 // [256]
  uint32_t* ctl = repl_in + 256;  // [2][2]: (leaf, fsize) of the split decided for an insert
  uint32_t nrepl = 0;             // wave 0's copy
  uint32_t it = 0;                // inserts processed: selects the ctl slot, so wave 0 (at most
                                  // one barrier ahead) never rewrites the slot the others read
  const uint64_t rb = a.row_bytes;
  auto row = [&](uint32_t id) { return a.rows + (uint64_t)id * rb; };

  for (uint32_t t = 0; t < a.n; t++) {
    if (!a.insert_flag[t]) continue;
    const uint32_t id = a.ids[t];
    const uint8_t* q = row(id);
    uint32_t* c2 = ctl + 2 * (it++ & 1);
    if (w == 0) {
      do {
        // ---- leaf descent (DVPTree::search, SearchLeaf, radius 0) -----------
        // Pre-located: the leaf found against the tree at batch start is still
        // on the object's path unless a split of this batch replaced it, and a
        // split replaces a leaf in place by an internal node whose subtree then
        // holds the path -- descend from the first such node.  A leaf that was
        // not empty at batch start keeps its pivot until it splits, so its
        // pivot distance is the pre-computed one.
        uint32_t node = a.counts[2];
        bool have_pd = false;
        float pd = 0.f;
        if (a.pre_leaf) {
          const uint32_t pl = a.pre_leaf[t];
          node = kLeaf | pl;
          uint32_t hit = 0xffffffffu;
          for (uint32_t r0 = 0; r0 < nrepl; r0 += 64) {
            const uint64_t m = ballot64(r0 + lane < nrepl && repl_leaf[r0 + lane] == pl);
            if (m) {
              hit = repl_in[r0 + __ffsll((long long)m) - 1];
              break;
            }
          }
          if (hit != 0xffffffffu) {
            node = hit;
          } else if (a.pre_count[t] != 0) {
            have_pd = true;
            pd = a.pre_dist[t];
          }
        }
        while (!(node & kLeaf)) {
          const uint32_t iid = node;
          const float d = dist1<M, T>(q, a.in_pivot + (uint64_t)iid * rb, a.dp);
          const float* b = a.in_border + (uint64_t)iid * 4;
          uint32_t mid = 0;
          for (; mid < 4; mid++)
            if (d < b[mid]) break;
          node = a.in_child[(uint64_t)iid * 5 + mid];
        }
        const uint32_t lid = node & ~kLeaf;
        uint32_t* lids = a.lf_ids + (uint64_t)lid * a.leaf_cap;
        float* ldst = a.lf_dist + (uint64_t)lid * a.leaf_cap;
        const uint32_t cnt = a.lf_count[lid];
        if (lane == 0) c2[1] = 0;
        // ---- DVPTree::insert(iobj, leaf): duplicate check (Tree.cpp:48-87) ---
        bool skip = false;
        if (cnt != 0 && !have_pd) pd = dist1<M, T>(q, a.lf_pivot + (uint64_t)lid * rb, a.dp);
        if (cnt != 0) {
          for (uint32_t base = 0; base < cnt && !skip; base += 64) {
            uint64_t eq = ballot64(base + lane < cnt && ldst[base + lane] == pd);
            while (eq) {
              const int j = __ffsll((long long)eq) - 1;
              eq &= eq - 1;
              const uint32_t loid = lids[base + j];
              const float idd = dist1<M, T>(q, row(loid), a.dp);
              if (idd == 0.0f) {
                if (loid == id && lane == 0) atomicOr(a.error, 2);  // "already existed"
                skip = true;
                break;
              }
            }
          }
        }
        if (skip) break;
        if (cnt < LS) {
          // ---- insertObject (Tree.cpp:267-313) -------------------------------
          if (cnt == 0) {
            copy_row(a.lf_pivot + (uint64_t)lid * rb, q, rb);
            if (lane == 0) {
              a.lf_has_pivot[lid] = 1;
              lids[0] = id;
              ldst[0] = 0.f;
              a.lf_count[lid] = 1;
            }
          } else if (lane == 0) {
            lids[cnt] = id;
            ldst[cnt] = pd;
            a.lf_count[lid] = cnt + 1;
          }
          break;
        }
        // ---- split (Tree.cpp:98-117): fs = leaf objects + the new one --------
        for (uint32_t i = lane; i < cnt; i += 64) fs_id[i] = lids[i];
        if (lane == 0) {
          fs_id[cnt] = id;
          c2[0] = lid;
          c2[1] = cnt + 1;
        }
      } while (false);
    }
    __syncthreads();
    const uint32_t fsize = c2[1];
    if (fsize == 0) continue;
    const uint32_t lid = c2[0];

    // selectPivotByMaxVariance (Node.cpp:97-144): D[i][j] = comparator(fs[i], fs[j]), i < j
    const uint32_t npairs = fsize * (fsize - 1) / 2;
    for (uint32_t p0 = 0; p0 < npairs; p0 += kQuads) {
      const uint32_t p = p0 + bq;
      if (p < npairs) {
        // p = hi(hi-1)/2 + lo, lo < hi
        uint32_t hi = (uint32_t)((1.0f + sqrtf(1.0f + 8.0f * (float)p)) * 0.5f);
        while (hi * (hi - 1) / 2 > p) hi--;
        while ((hi + 1) * hi / 2 <= p) hi++;
        const uint32_t lo = p - hi * (hi - 1) / 2;
        const float d = quad_dist_rows<M, T>(row(fs_id[lo]), row(fs_id[hi]), a.dp, g);
        if (g == 0) {
          D[lo * fsize + hi] = d;
          D[hi * fsize + lo] = d;
        }
      }
    }
    for (uint32_t i = tid; i < fsize; i += 256) D[i * fsize + i] = 0.f;
    __syncthreads();
    for (uint32_t i = tid; i < fsize; i += 256) var[i] = pivot_variance(D + (uint64_t)i * fsize, fsize);
    __syncthreads();
    uint32_t pv = 0;
    {
      double maxv = var[0];
      for (uint32_t i = 0; i < fsize; i++)
        if (var[i] > maxv) {
          maxv = var[i];
          pv = i;
        }
    }
    // splitObjects (Node.cpp:146-225): distance from the pivot, sort, clusters
    for (uint32_t i0 = 0; i0 < fsize; i0 += kQuads) {
      const uint32_t i = i0 + bq;
      float d = 0.f;
      if (i < fsize && i != pv) d = quad_dist_rows<M, T>(row(fs_id[pv]), row(fs_id[i]), a.dp, g);
      if (i < fsize && g == 0) fs_dist[i] = d;
    }
    __syncthreads();
    // std::sort by distance: with distinct distances every correct sort gives
    // the same order (rank = number of smaller keys); ties keep libstdc++'s
    // introsort order, restated step by step on one lane.
    bool tie = false;
    if ((uint32_t)tid < fsize) {
      const float di = fs_dist[tid];
      uint32_t rank = 0;
      for (uint32_t j = 0; j < fsize; j++) {
        const float dj = fs_dist[j];
        rank += dj < di ? 1u : 0u;
        tie |= (dj == di) && j != (uint32_t)tid;
      }
      items[rank].d = di;
      items[rank].i = (uint32_t)tid;
    }
    if (__syncthreads_or(tie)) {
      if (tid == 0) {
        for (uint32_t i = 0; i < fsize; i++) {
          items[i].d = fs_dist[i];
          items[i].i = i;
        }
        std_sort(items, items + fsize);
      }
      __syncthreads();
    }
    // permute fs into sorted order
    uint32_t sid = 0;
    float sd = 0.f;
    if ((uint32_t)tid < fsize) {
      sid = fs_id[items[tid].i];
      sd = items[tid].d;
    }
    __syncthreads();
    if ((uint32_t)tid < fsize) {
      fs_id[tid] = sid;
      fs_dist[tid] = sd;
    }
    __syncthreads();
    if (tid == 0) {
      const int csize = 5;
      int cid = csize - 1;
      int cms = ((int)fsize * cid) / csize;
      fs_cl[fsize - 1] = cid;
      for (int i = (int)fsize - 2; i >= 0; i--) {
        if (i < cms && cid > 0) {
          if (fs_dist[i] != fs_dist[i + 1]) {
            cid--;
            cms = ((int)fsize * cid) / csize;
          }
        }
        fs_cl[i] = cid;
      }
      if (cid != 0) {
        if (fs_cl[fsize - 1] == cid) {
          atomicOr(a.error, 8);  // "All of the object distances are the same!"
        } else {
          for (uint32_t i = 0; i < fsize; i++) fs_cl[i] -= cid;
        }
      }
    }
    __syncthreads();
    // leafDistance: -1 (Object::Pivot) for the first of each cluster, else the
    // distance to that first object
    for (uint32_t i0 = 0; i0 < fsize; i0 += kQuads) {
      const uint32_t i = i0 + bq;
      float ld = -1.0f;
      if (i < fsize) {
        uint32_t first = i;
        while (first > 0 && fs_cl[first - 1] == fs_cl[i]) first--;
        if (first != i) ld = quad_dist_rows<M, T>(row(fs_id[first]), row(fs_id[i]), a.dp, g);
      }
      if (i < fsize && g == 0) fs_ld[i] = ld;
    }
    __syncthreads();
    // ---- recombineNodes (Tree.cpp:119-265), wave 0 ------------------------
    if (w == 0) {
      const uint32_t targetParent = a.lf_parent[lid];
      const uint32_t targetId = kLeaf | lid;
      const uint32_t inid = a.counts[1];
      const uint32_t nl0 = a.counts[0];
      if (inid >= a.in_cap_nodes || nl0 + 4 > a.leaf_cap_nodes) {
        if (lane == 0) atomicOr(a.error, 16);  // capacity: the host grows the arrays first
      } else {
        const uint32_t ln[5] = {lid, nl0, nl0 + 1, nl0 + 2, nl0 + 3};
        bool known = false;
        for (uint32_t r0 = 0; r0 < nrepl; r0 += 64)
          known |= ballot64(r0 + lane < nrepl && repl_leaf[r0 + lane] == lid) != 0;
        if (!known && nrepl < 256) {
          if (lane == 0) {
            repl_leaf[nrepl] = lid;
            repl_in[nrepl] = inid;
          }
          nrepl++;
        }
        if (lane == 0 && (targetParent & ~kLeaf) != 0) {
          uint32_t* ch = a.in_child + (uint64_t)targetParent * 5;
          for (int c = 0; c < 5; c++)
            if (ch[c] == targetId) {
              ch[c] = inid;
              break;
            }
        }
        copy_row(a.in_pivot + (uint64_t)inid * rb, row(fs_id[0]), rb);
        // cluster pivots (leafDistance == Pivot) and the fs[0] dummies for empty children
        int maxClusterID = 0;
        for (uint32_t i = 0; i < fsize; i++) maxClusterID = fs_cl[i] > maxClusterID ? fs_cl[i] : maxClusterID;
        for (uint32_t i = 0; i < fsize; i++)
          if (fs_ld[i] == -1.0f) copy_row(a.lf_pivot + (uint64_t)ln[fs_cl[i]] * rb, row(fs_id[i]), rb);
        for (int c = maxClusterID + 1; c < 5; c++) copy_row(a.lf_pivot + (uint64_t)ln[c] * rb, row(fs_id[0]), rb);
        if (lane == 0) {
          if (fs_ld[0] != -1.0f) atomicOr(a.error, 32);  // "illegal pivot"
          // distribute fs over the cluster leaves; counts and pivot flags in
          // registers, written once
          uint32_t kc[5] = {0, 0, 0, 0, 0};
          uint8_t hp[5] = {0, 0, 0, 0, 0};
          float border[4] = {0.f, 0.f, 0.f, 0.f};
          int cid = fs_cl[0];
          a.lf_ids[(uint64_t)ln[cid] * a.leaf_cap] = fs_id[0];
          a.lf_dist[(uint64_t)ln[cid] * a.leaf_cap] = 0.0f;
          kc[cid] = 1;
          hp[cid] = 1;
          for (uint32_t i = 1; i < fsize; i++) {
            const int c = fs_cl[i];
            float ld;
            if (fs_ld[i] == -1.0f) {
              hp[c] = 1;
              ld = 0.0f;
            } else {
              ld = fs_ld[i];
            }
            a.lf_ids[(uint64_t)ln[c] * a.leaf_cap + kc[c]] = fs_id[i];
            a.lf_dist[(uint64_t)ln[c] * a.leaf_cap + kc[c]] = ld;
            kc[c]++;
            if (c != cid) {
              border[cid] = fs_dist[i];
              cid = c;
            }
          }
          for (int c = maxClusterID + 1; c < 5; c++) {
            hp[c] = 1;
            if (c < 4) border[c] = FLT_MAX;
          }
          for (int c = 0; c < 5; c++) {
            a.lf_count[ln[c]] = kc[c];
            a.lf_has_pivot[ln[c]] = hp[c];
            a.lf_parent[ln[c]] = inid;
          }
          a.in_parent[inid] = targetParent;
          for (int c = 0; c < 4; c++) a.in_border[(uint64_t)inid * 4 + c] = border[c];
          uint32_t* ch = a.in_child + (uint64_t)inid * 5;
          ch[0] = targetId;
          for (int c = 1; c < 5; c++) ch[c] = kLeaf | ln[c];
          a.counts[0] = nl0 + 4;
          a.counts[1] = inid + 1;
          if ((targetParent & ~kLeaf) == 0) a.counts[2] = inid;  // the root was this leaf
        }
      }
    }
    __threadfence();
    __syncthreads();
  }
}

// Pair distances of a creation batch: comparator(object i, object j), j < i
// (Index.cpp:690-703), one quad per pair, stored in the order the reference
// visits them.
template <int M, typename T>
__global__ void __launch_bounds__(256) ngt_batch_pairs_kernel(BatchPairArgs a) {
  const int g = threadIdx.x & 3;
  const uint64_t quad = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 2;
  const uint64_t nquads = ((uint64_t)gridDim.x * blockDim.x) >> 2;
  const uint64_t np = (uint64_t)a.n * (a.n - 1) / 2;
  for (uint64_t p = quad; p < np; p += nquads) {
    // p = i(i-1)/2 + j: i from the closed form, corrected for rounding
    uint64_t i = (uint64_t)((1.0 + sqrt(1.0 + 8.0 * (double)p)) * 0.5);
    while (i * (i - 1) / 2 > p) i--;
    while ((i + 1) * i / 2 <= p) i++;
    const uint64_t j = p - i * (i - 1) / 2;
    const T* q = reinterpret_cast<const T*>(a.batch + i * a.row_bytes);
    const T* x = row_ptr<T>(a.rows, a.row_bytes, a.ids[j]);
    const float d = quad_distance<M, T>(q, x, a.dp, g);
    if (g == 0) a.out[p] = d;
  }
}

// One wave per batch object i: the K smallest (distance, id) keys among its
// search results and the pairs (i, j < i) -- std::sort + resize on a total
// order, so K rounds of "smallest key above the previous one" select the
// same list.
__global__ void __launch_bounds__(64) ngt_batch_merge_kernel(BatchMergeArgs a) {
  const int lane = lane_id();
  for (uint32_t i = blockIdx.x; i < a.n; i += gridDim.x) {
    const uint32_t nr = a.res_n[i];
    const uint32_t c = nr + i;
    const uint64_t pb = (uint64_t)i * (i - 1) / 2;
    const uint32_t want = c < a.K ? c : a.K;
    uint64_t prev = 0, first = 0;
    for (uint32_t r = 0; r < want; r++) {
      uint64_t best = ~0ull;
      for (uint32_t t = lane; t < c; t += 64) {
        uint64_t key;
        if (t < nr) key = make_key(a.res_dists[(uint64_t)i * a.K + t], a.res_ids[(uint64_t)i * a.K + t]);
        else key = make_key(a.pair[pb + (t - nr)], a.ids[t - nr]);
        if ((r == 0 || key > prev) && key < best) best = key;
      }
      best = wave_min_u64(best);
      if (lane == 0) {
        a.out_ids[(uint64_t)i * a.K + r] = key_id(best);
        a.out_dists[(uint64_t)i * a.K + r] = key_dist(best);
      }
      if (r == 0) first = best;
      prev = best;
    }
    if (lane == 0) {
      a.out_n[i] = want;
      // the tree gets the object unless it duplicates its nearest neighbour
      a.flag[i] = (want == 0 || key_dist(first) != 0.0f) ? 1 : 0;
    }
  }
}

// Rows `nodes[i]` of the padded adjacency <- vals[i][0..stride).
__global__ void __launch_bounds__(256) ngt_adj_scatter_kernel(uint32_t* adj, uint64_t stride,
                                                              const uint32_t* nodes, const uint32_t* vals,
                                                              uint32_t n) {
  const uint64_t total = (uint64_t)n * stride;
  for (uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total;
       t += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t r = t / stride, c = t - r * stride;
    adj[(uint64_t)nodes[r] * stride + c] = vals[t];
  }
}

// dst[i] = rows[ids[i]] (row_bytes each, 16-byte aligned)
__global__ void __launch_bounds__(256) ngt_gather_rows_kernel(uint8_t* dst, const uint8_t* rows, uint64_t row_bytes,
                                                              const uint32_t* ids, uint32_t n) {
  const uint64_t per = row_bytes / 16;
  const uint64_t total = (uint64_t)n * per;
  for (uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total;
       t += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t r = t / per, c = t - r * per;
    reinterpret_cast<uint4*>(dst + r * row_bytes)[c] = reinterpret_cast<const uint4*>(rows + (uint64_t)ids[r] * row_bytes)[c];
  }
}

hipError_t launch_gather_rows(uint8_t* dst, const uint8_t* rows, uint64_t row_bytes, const uint32_t* ids, uint32_t n,
                              hipStream_t s) {
  if (n == 0) return hipSuccess;
  uint64_t blocks = ((uint64_t)n * (row_bytes / 16) + 255) / 256;
  if (blocks > 65536) blocks = 65536;
  hipLaunchKernelGGL(ngt_gather_rows_kernel, dim3((uint32_t)blocks), dim3(256), 0, s, dst, rows, row_bytes, ids, n);
  return hipGetLastError();
}

#define NGT_BUILD_DISPATCH(METRIC, OTYPE, LAUNCH)                              \
  do {                                                                         \
    if ((OTYPE) == kFloat) {                                                   \
      switch (METRIC) {                                                        \
        case kL1: LAUNCH(kL1, float); break;                                   \
        case kL2: LAUNCH(kL2, float); break;                                   \
        case kAngle: LAUNCH(kAngle, float); break;                             \
        case kCosine: LAUNCH(kCosine, float); break;                           \
        case kNormalizedAngle: LAUNCH(kNormalizedAngle, float); break;         \
        case kNormalizedCosine: LAUNCH(kNormalizedCosine, float); break;       \
        case kNormalizedL2: LAUNCH(kNormalizedL2, float); break;               \
        case kSparseJaccard: LAUNCH(kSparseJaccard, float); break;             \
        case kPoincare: LAUNCH(kPoincare, float); break;                       \
        case kLorentz: LAUNCH(kLorentz, float); break;                         \
        default: return hipErrorInvalidValue;                                  \
      }                                                                        \
    } else if ((OTYPE) == kUint8) {                                            \
      switch (METRIC) {                                                        \
        case kL1: LAUNCH(kL1, uint8_t); break;                                 \
        case kL2: LAUNCH(kL2, uint8_t); break;                                 \
        case kHamming: LAUNCH(kHamming, uint8_t); break;                       \
        case kJaccard: LAUNCH(kJaccard, uint8_t); break;                       \
        case kAngle: LAUNCH(kAngle, uint8_t); break;                           \
        case kCosine: LAUNCH(kCosine, uint8_t); break;                         \
        case kNormalizedAngle: LAUNCH(kNormalizedAngle, uint8_t); break;       \
        case kNormalizedCosine: LAUNCH(kNormalizedCosine, uint8_t); break;     \
        case kNormalizedL2: LAUNCH(kNormalizedL2, uint8_t); break;             \
        default: return hipErrorInvalidValue;                                  \
      }                                                                        \
    } else {                                                                   \
      return hipErrorInvalidValue;                                             \
    }                                                                          \
  } while (0)

hipError_t launch_tree_insert(const TreeBuildArgs& a, int metric, int otype, hipStream_t s) {
  if (a.n == 0) return hipSuccess;
  const uint32_t nf = a.leaf_size + 1;
  const size_t lds = 128 * (4 + 4 + 4 + 4) + 128 * sizeof(SortItem) + 128 * sizeof(double) +
                     (size_t)nf * nf * sizeof(float) + 2 * 256 * sizeof(uint32_t) + 4 * sizeof(uint32_t);
  if (lds > 64 * 1024) return hipErrorInvalidValue;
#define L_TI(MM, TT) hipLaunchKernelGGL((ngt_tree_insert_kernel<MM, TT>), dim3(1), dim3(256), lds, s, a)
  NGT_BUILD_DISPATCH(metric, otype, L_TI);
#undef L_TI
  return hipGetLastError();
}

hipError_t launch_batch_pairs(const BatchPairArgs& a, int metric, int otype, hipStream_t s) {
  if (a.n < 2) return hipSuccess;
  const uint64_t np = (uint64_t)a.n * (a.n - 1) / 2;
  uint64_t blocks = (np * 4 + 255) / 256;
  if (blocks > 16384) blocks = 16384;
#define L_BP(MM, TT) hipLaunchKernelGGL((ngt_batch_pairs_kernel<MM, TT>), dim3((uint32_t)blocks), dim3(256), 0, s, a)
  NGT_BUILD_DISPATCH(metric, otype, L_BP);
#undef L_BP
  return hipGetLastError();
}

hipError_t launch_batch_merge(const BatchMergeArgs& a, hipStream_t s) {
  if (a.n == 0) return hipSuccess;
  hipLaunchKernelGGL(ngt_batch_merge_kernel, dim3(a.n < 4096 ? a.n : 4096), dim3(64), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_adj_scatter(uint32_t* adj, uint64_t stride, const uint32_t* nodes, const uint32_t* vals, uint32_t n,
                              hipStream_t s) {
  if (n == 0) return hipSuccess;
  uint64_t blocks = ((uint64_t)n * stride + 255) / 256;
  if (blocks > 65536) blocks = 65536;
  hipLaunchKernelGGL(ngt_adj_scatter_kernel, dim3((uint32_t)blocks), dim3(256), 0, s, adj, stride, nodes, vals, n);
  return hipGetLastError();
}

}  // namespace ngt_amd
