// build.cpp -- ANNG construction on the MI355X:
// GraphAndTreeIndex::createIndex(threadPoolSize) (lib/NGT/Index.cpp:1158-1257)
// for graphType ANNG with the default (disabled) edge truncation.
//
// Per creation batch of batchSizeForCreation objects, in id order
// (searchMultipleQueryForCreation, Index.cpp:631-671):
//   1. seeds: DVP-tree leaf descent of every batch object with
//      useAllNodesInLeaf (searchForNNGInsertion, Index.h:1457-1479) --
//      ngt_tree_seed_kernel over the tree under construction; an empty leaf
//      falls back to getRandomSeeds over the graph (Index.h:775-801) with the
//      rand() stream of a fresh process;
//   2. the insertion searches: one ngt_graph_search_kernel launch for the batch
//      (size edgeSizeForCreation, explorationCoefficient insertionRadiusCoefficient,
//      the first edgeSizeForSearch edges of each node);
//   3. insertMultipleSearchResults (Index.cpp:673-727): the batch's pairwise
//      distances (ngt_distances_kernel), merge, sort by (distance, id), cut to
//      edgeSizeForCreation, then insertANNGNode (Graph.h:611-625) -- the node's
//      edges and the reverse edges, sorted inserts (Graph.h:845-873);
//   4. DVPTree::insert of the batch (ngt_tree_insert_kernel).
// The graph being built is host-side (sorted edge lists, the reference's
// GraphRepository); the insertion searches read a padded HBM copy of each
// node's first edgeSizeForSearch edges, refreshed for the nodes a batch touched.
#include <hip/hip_runtime.h>
#include <float.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <chrono>
#include <vector>

#include "../../include/ngt_amd.h"
#include "index_internal.h"
#include "ngt_kernels.h"

using namespace ngt_amd;

namespace {

constexpr uint32_t kLeaf = 0x80000000u;
constexpr uint32_t kLeafCap = 112;  // >= leafObjectsSize + 1, multiple of 16

template <typename T>
int grow(DevBuf<T>& b, size_t old_count, size_t new_count) {
  if (b.p && b.n >= new_count) return 0;
  T* p = nullptr;
  HIP_OK(hipMalloc((void**)&p, std::max<size_t>(new_count, 1) * sizeof(T)));
  HIP_OK(hipMemset(p, 0, std::max<size_t>(new_count, 1) * sizeof(T)));
  if (b.p && old_count) HIP_OK(hipMemcpy(p, b.p, old_count * sizeof(T), hipMemcpyDeviceToDevice));
  b.release();
  b.p = p;
  b.n = new_count;
  return 0;
}

// room for `extra_leaves` / `extra_internal` more nodes
int ensure_tree_capacity(ngt_amd_index* ix, BuildState& b, uint32_t extra_leaves, uint32_t extra_internal) {
  const uint64_t rb = ix->row_bytes;
  if (b.n_leaf + extra_leaves > b.leaf_cap_nodes) {
    const uint32_t old = b.leaf_cap_nodes;
    const uint32_t cap = std::max<uint32_t>(b.n_leaf + extra_leaves, old * 2);
    if (grow(b.lf_parent, old, cap) || grow(b.lf_count, old, cap) || grow(b.lf_has_pivot, old, cap) ||
        grow(b.lf_ids, (size_t)old * kLeafCap, (size_t)cap * kLeafCap) ||
        grow(b.lf_dist, (size_t)old * kLeafCap, (size_t)cap * kLeafCap) ||
        grow(b.lf_pivot, (size_t)old * rb, (size_t)cap * rb))
      return -1;
    b.leaf_cap_nodes = cap;
  }
  if (b.n_internal + extra_internal > b.in_cap_nodes) {
    const uint32_t old = b.in_cap_nodes;
    const uint32_t cap = std::max<uint32_t>(b.n_internal + extra_internal, old * 2);
    if (grow(b.in_parent, old, cap) || grow(b.in_child, (size_t)old * 5, (size_t)cap * 5) ||
        grow(b.in_border, (size_t)old * 4, (size_t)cap * 4) || grow(b.in_pivot, (size_t)old * rb, (size_t)cap * rb))
      return -1;
    b.in_cap_nodes = cap;
  }
  return 0;
}

bool od_less(const std::pair<uint32_t, float>& a, const std::pair<uint32_t, float>& b) {
  // ObjectDistance::operator< (Common.h:1946-1952): distance, then id
  if (a.second != b.second) return a.second < b.second;
  return a.first < b.first;
}

}  // namespace

extern "C" int ngt_amd_build_begin(ngt_amd_index* ix, const ngt_amd_build_params* prm) {
  if (!ix || !prm) return fail("ngt_amd_build_begin: bad arguments");
  if (ix->nrows == 0) return fail("ngt_amd_build_begin: set the objects first");
  if (prm->edge_size_for_creation <= 0 || prm->batch_size_for_creation <= 0)
    return fail("ngt_amd_build_begin: edge_size_for_creation and batch_size_for_creation must be > 0");
  HIP_OK(hipSetDevice(ix->device));
  ServeHold serve_hold(ix);
  delete ix->build;
  auto* b = new BuildState();
  ix->build = b;
  b->edge_size_for_creation = prm->edge_size_for_creation;
  b->edge_size_for_search = prm->edge_size_for_search;
  b->batch_size = prm->batch_size_for_creation;
  b->seed_size = prm->seed_size;
  b->epsilon_for_creation = prm->epsilon_for_creation;
  b->graph.assign(ix->nrows, {});
  b->in_graph.assign(ix->nrows, 0);
  b->rnd.seed(1);
  if (ensure_tree_capacity(ix, *b, 64, 16)) return -1;
  // the empty root leaf (DVPTree(), Tree.h:71-78): leaf 1, no parent, no objects
  const uint32_t c3[3] = {2u, 1u, kLeaf | 1u};
  HIP_OK(b->counts.upload(c3, 3));
  b->n_leaf = 2;
  b->n_internal = 1;
  b->root = kLeaf | 1u;
  // padded search adjacency: each node's first edgeSizeForSearch edges
  const int64_t es = prm->edge_size_for_search;
  if (es < 0 || es > 256) return fail("ngt_amd_build_begin: edge_size_for_search %lld unsupported", (long long)es);
  b->adj_stride = es == 0 ? 256 : (uint64_t)((es + 15) / 16 * 16);
  HIP_OK(ix->adj.alloc((size_t)ix->nrows * b->adj_stride));
  HIP_OK(hipMemset(ix->adj.p, 0, (size_t)ix->nrows * b->adj_stride * sizeof(uint32_t)));
  ix->adj_stride = b->adj_stride;
  ix->adj_version++;
  // the construction's searches read at most adj_stride edges of a list: the
  // padded copy is always the one to use (run_search never rebuilds it here)
  ix->max_degree = b->adj_stride;
  ix->has_graph = true;
  ix->edge_size_for_search = prm->edge_size_for_search;
  ix->seed_size = prm->seed_size;
  ix->seed_type = 0;
  return 0;
}

extern "C" int ngt_amd_build_insert(ngt_amd_index* ix, uint64_t first_id, uint64_t end_id) {
  if (!ix || !ix->build) return fail("ngt_amd_build_insert: call ngt_amd_build_begin first");
  HIP_OK(hipSetDevice(ix->device));
  ServeHold serve_hold(ix);
  // the insertion searches never rebuild the padded adjacency this call keeps
  // changing: build_begin set max_degree = adj_stride, so the copy always
  // holds every edge they read
  BuildState& b = *ix->build;
  hipStream_t s = ix->stream;
  const uint64_t rb = ix->row_bytes;
  if (end_id > ix->nrows) end_id = ix->nrows;
  if (first_id < 1) first_id = 1;
  std::vector<uint32_t> todo;
  for (uint64_t id = first_id; id < end_id; id++)
    if (ix->h_valid[id] && !b.in_graph[id]) todo.push_back((uint32_t)id);

  const uint32_t B = (uint32_t)b.batch_size, K = (uint32_t)b.edge_size_for_creation;
  struct Ev {
    hipEvent_t e = nullptr;
    ~Ev() {
      if (e) (void)hipEventDestroy(e);
    }
  } ev_copy;
  HIP_OK(hipEventCreateWithFlags(&ev_copy.e, hipEventDisableTiming));
  const uint32_t SS = kTreeSeedStride;
  DevBuf<uint32_t> d_ids, d_tseeds, d_tcnt, d_seeds, d_oi, d_on, d_dirty, d_vals;
  DevBuf<uint64_t> d_soff;
  DevBuf<float> d_od, d_pd;
  DevBuf<uint8_t> d_q, d_flag;
  HIP_OK(d_ids.alloc(B));
  HIP_OK(d_q.alloc((size_t)B * rb));
  HIP_OK(d_tseeds.alloc((size_t)B * SS));
  HIP_OK(d_tcnt.alloc(B));
  HIP_OK(d_oi.alloc((size_t)B * K));
  HIP_OK(d_od.alloc((size_t)B * K));
  HIP_OK(d_on.alloc(B));
  HIP_OK(d_flag.alloc(B));
  DevBuf<uint32_t> d_pleaf, d_pcnt;
  DevBuf<float> d_pdist;
  HIP_OK(d_pleaf.alloc(B));
  HIP_OK(d_pcnt.alloc(B));
  HIP_OK(d_pdist.alloc(B));
  DevBuf<uint32_t> d_mi, d_mn;
  DevBuf<float> d_md;
  HIP_OK(d_mi.alloc((size_t)B * K));
  HIP_OK(d_md.alloc((size_t)B * K));
  HIP_OK(d_mn.alloc(B));
  std::vector<uint32_t> h_tseeds((size_t)B * SS), h_tcnt(B), h_mi((size_t)B * K), h_mn(B);
  std::vector<float> h_md((size_t)B * K);
  // NGT_AMD_BUILD_PROFILE=1: per-stage wall time (stream synchronised at each mark)
  const bool prof = ngt_amd::knob("NGT_AMD_BUILD_PROFILE") != nullptr;
  double st[6] = {0, 0, 0, 0, 0, 0};
  auto t_last = std::chrono::steady_clock::now();
  DevBuf<uint64_t> d_cnt;
  std::vector<uint64_t> h_cnt;
  double k_ms = 0, dc = 0, ex = 0, ex_max = 0, c3 = 0, c5 = 0, c6 = 0, c7 = 0, c5_max = 0;
  uint64_t nsearched = 0;
  if (prof) {
    HIP_OK(d_cnt.alloc((size_t)B * NGT_AMD_COUNTERS_PER_QUERY));
    h_cnt.resize((size_t)B * NGT_AMD_COUNTERS_PER_QUERY);
  }
  auto mark = [&](int i) {
    if (!prof) return;
    (void)hipStreamSynchronize(s);
    auto t = std::chrono::steady_clock::now();
    st[i] += std::chrono::duration<double>(t - t_last).count();
    t_last = t;
  };

  for (size_t pos = 0; pos < todo.size(); pos += B) {
    const uint32_t n = (uint32_t)std::min<size_t>(B, todo.size() - pos);
    const uint32_t* ids = todo.data() + pos;
    if (ensure_tree_capacity(ix, b, 4 * n + 4, n + 1)) return -1;
    HIP_OK(hipMemcpyAsync(d_ids.p, ids, n * sizeof(uint32_t), hipMemcpyHostToDevice, s));
    HIP_OK(launch_gather_rows(d_q.p, ix->rows.p, rb, d_ids.p, n, s));

    // ---- 1. seeds: all objects of the leaf each batch object descends to --
    TreeSeedArgs t{};
    t.queries = d_q.p;
    t.query_bytes = rb;
    t.nq = n;
    t.dp = (int)ix->dp;
    t.row_bytes = rb;
    t.in_pivot = b.in_pivot.p;
    t.in_child = b.in_child.p;
    t.in_border = b.in_border.p;
    t.children = 5;
    t.root = b.root;
    t.leaf_count = b.lf_count.p;
    t.leaf_stride = kLeafCap;
    t.leaf_ids = b.lf_ids.p;
    t.seed_size = (uint32_t)std::max(b.seed_size, 0);
    t.k = K;
    t.all_leaf_nodes = 1;
    t.seeds = d_tseeds.p;
    t.seed_stride = SS;
    t.seed_count = d_tcnt.p;
    // the same descent locates each object's leaf for step 4
    t.out_leaf = d_pleaf.p;
    t.out_count = d_pcnt.p;
    t.out_pdist = d_pdist.p;
    t.leaf_pivot = b.lf_pivot.p;
    HIP_OK(launch_tree_seeds(t, ix->metric, ix->otype, s));
    HIP_OK(hipMemcpyAsync(h_tseeds.data(), d_tseeds.p, (size_t)n * SS * sizeof(uint32_t), hipMemcpyDeviceToHost, s));
    HIP_OK(hipMemcpyAsync(h_tcnt.data(), d_tcnt.p, n * sizeof(uint32_t), hipMemcpyDeviceToHost, s));
    HIP_OK(hipStreamSynchronize(s));
    mark(0);
    std::vector<uint32_t> seeds;
    std::vector<uint64_t> soff(n + 1, 0);
    for (uint32_t i = 0; i < n; i++) {
      const size_t start = seeds.size();
      for (uint32_t j = 0; j < h_tcnt[i]; j++) seeds.push_back(h_tseeds[(size_t)i * SS + j]);
      if (h_tcnt[i] == 0 && b.graph_size != 0) {
        // getSeedsFromGraph -> getRandomSeeds (Index.h:775-801, 1115-1135)
        const size_t repo = b.graph_size - 1;
        const size_t ss = std::min<size_t>(repo, (size_t)std::max(b.seed_size, 0));
        size_t empty = 0;
        while (seeds.size() - start < ss) {
          const double r = ((double)b.rnd.next() + 1.0) / ((double)2147483647 + 2.0);
          const size_t idx = (size_t)floor((double)repo * r) + 1;
          if (!b.in_graph[idx]) {
            if (++empty > repo) break;
            continue;
          }
          if (std::find(seeds.begin() + start, seeds.end(), (uint32_t)idx) != seeds.end()) continue;
          seeds.push_back((uint32_t)idx);
        }
      }
      soff[i + 1] = seeds.size();
    }

    // ---- 2. insertion searches (searchForNNGInsertion, Index.h:1457-1479) --
    if (!seeds.empty()) {
      HIP_OK(d_seeds.upload(seeds.data(), seeds.size()));
      HIP_OK(d_soff.upload(soff.data(), n + 1));
      ngt_amd_search_params p{};
      p.k = K;
      p.epsilon = b.epsilon_for_creation;
      p.radius = FLT_MAX;
      p.edge_size = -1;  // sc.edgeSize default -> edgeSizeForSearch
      p.seed_mode = NGT_AMD_SEED_GIVEN;
      p.visited_hash_log2 = 0;
      if (ngt_amd_search_device(ix, &p, d_q.p, rb, n, d_seeds.p, d_soff.p, d_oi.p, d_od.p, d_on.p,
                                prof ? d_cnt.p : nullptr, s))
        return -1;
      if (prof) {
        HIP_OK(hipMemcpyAsync(h_cnt.data(), d_cnt.p, (size_t)n * NGT_AMD_COUNTERS_PER_QUERY * sizeof(uint64_t),
                              hipMemcpyDeviceToHost, s));
        HIP_OK(hipStreamSynchronize(s));
        k_ms += ngt_amd_last_search_kernel_ms(ix);
        uint64_t mx = 0;
        for (uint32_t i = 0; i < n; i++) {
          dc += (double)h_cnt[(size_t)i * NGT_AMD_COUNTERS_PER_QUERY];
          ex += (double)h_cnt[(size_t)i * NGT_AMD_COUNTERS_PER_QUERY + 2];
          mx = std::max(mx, h_cnt[(size_t)i * NGT_AMD_COUNTERS_PER_QUERY + 2]);
          const uint64_t* c = h_cnt.data() + (size_t)i * NGT_AMD_COUNTERS_PER_QUERY;
          c3 += (double)c[3];
          c5 += (double)c[5];
          c6 += (double)c[6];
          c7 += (double)c[7];
          c5_max = std::max(c5_max, (double)c[5]);
        }
        ex_max += (double)mx;
        nsearched += n;
      }
    } else {
      HIP_OK(hipMemsetAsync(d_on.p, 0, n * sizeof(uint32_t), s));
    }
    mark(1);

    // ---- 3. pairwise distances inside the batch (Index.cpp:690-703), then the
    //         merge / sort / cut of insertMultipleSearchResults (:673-727) -------
    const uint64_t npairs = (uint64_t)n * (n - 1) / 2;
    if (npairs) HIP_OK(d_pd.alloc(npairs));
    BatchPairArgs bp{};
    bp.rows = ix->rows.p;
    bp.row_bytes = rb;
    bp.dp = (int)ix->dp;
    bp.batch = d_q.p;
    bp.ids = d_ids.p;
    bp.n = n;
    bp.out = d_pd.p;
    HIP_OK(launch_batch_pairs(bp, ix->metric, ix->otype, s));
    BatchMergeArgs bm{};
    bm.res_ids = d_oi.p;
    bm.res_dists = d_od.p;
    bm.res_n = d_on.p;
    bm.K = K;
    bm.ids = d_ids.p;
    bm.pair = d_pd.p;
    bm.n = n;
    bm.out_ids = d_mi.p;
    bm.out_dists = d_md.p;
    bm.out_n = d_mn.p;
    bm.flag = d_flag.p;
    HIP_OK(launch_batch_merge(bm, s));
    mark(2);

    // ---- 4. DVPTree::insert of the batch (device, overlaps the host graph work)
    TreeBuildArgs ta{};
    ta.rows = ix->rows.p;
    ta.row_bytes = rb;
    ta.dp = (int)ix->dp;
    ta.lf_parent = b.lf_parent.p;
    ta.lf_has_pivot = b.lf_has_pivot.p;
    ta.lf_pivot = b.lf_pivot.p;
    ta.lf_count = b.lf_count.p;
    ta.lf_ids = b.lf_ids.p;
    ta.lf_dist = b.lf_dist.p;
    ta.leaf_cap = kLeafCap;
    ta.in_parent = b.in_parent.p;
    ta.in_pivot = b.in_pivot.p;
    ta.in_child = b.in_child.p;
    ta.in_border = b.in_border.p;
    ta.counts = b.counts.p;
    ta.leaf_cap_nodes = b.leaf_cap_nodes;
    ta.in_cap_nodes = b.in_cap_nodes;
    ta.leaf_size = 100;  // LeafNode::LeafObjectsSizeMax (Node.h:618)
    ta.ids = d_ids.p;
    ta.insert_flag = d_flag.p;
    ta.pre_leaf = d_pleaf.p;
    ta.pre_count = d_pcnt.p;
    ta.pre_dist = d_pdist.p;
    ta.n = n;
    ta.error = ix->error.p;
    // the merged lists go to the host while the tree insertion runs
    HIP_OK(hipMemcpyAsync(h_mi.data(), d_mi.p, (size_t)n * K * sizeof(uint32_t), hipMemcpyDeviceToHost, s));
    HIP_OK(hipMemcpyAsync(h_md.data(), d_md.p, (size_t)n * K * sizeof(float), hipMemcpyDeviceToHost, s));
    HIP_OK(hipMemcpyAsync(h_mn.data(), d_mn.p, n * sizeof(uint32_t), hipMemcpyDeviceToHost, s));
    HIP_OK(hipEventRecord(ev_copy.e, s));
    HIP_OK(launch_tree_insert(ta, ix->metric, ix->otype, s));
    mark(4);
    HIP_OK(hipEventSynchronize(ev_copy.e));

    // ---- insertANNGNode (Graph.h:611-625): the node, then the reverse edges --
    std::vector<uint32_t> dirty;
    for (uint32_t i = 0; i < n; i++) {
      const uint32_t id = ids[i];
      auto& objs = b.graph[id];
      objs.resize(h_mn[i]);
      for (uint32_t j = 0; j < h_mn[i]; j++) objs[j] = {h_mi[(size_t)i * K + j], h_md[(size_t)i * K + j]};
      b.in_graph[id] = 1;
      b.graph_size = std::max<uint64_t>(b.graph_size, (uint64_t)id + 1);
      dirty.push_back(id);
      for (const auto& r : objs) {
        auto& node = b.graph[r.first];
        const std::pair<uint32_t, float> e{id, r.second};
        auto it = std::lower_bound(node.begin(), node.end(), e, od_less);
        if (it != node.end() && it->first == id) return fail("NGT::addEdge: already existed! %u:%u", it->first, id);
        if ((uint64_t)(it - node.begin()) < b.adj_stride) dirty.push_back(r.first);
        node.insert(it, e);
      }
    }
    mark(3);

    // ---- refresh the padded adjacency of the touched nodes -----------------
    std::sort(dirty.begin(), dirty.end());
    dirty.erase(std::unique(dirty.begin(), dirty.end()), dirty.end());
    std::vector<uint32_t> vals(dirty.size() * b.adj_stride, 0u);
    for (size_t i = 0; i < dirty.size(); i++) {
      const auto& node = b.graph[dirty[i]];
      const size_t m = std::min<size_t>(node.size(), b.adj_stride);
      for (size_t j = 0; j < m; j++) vals[i * b.adj_stride + j] = node[j].first;
    }
    HIP_OK(d_dirty.upload(dirty.data(), dirty.size()));
    HIP_OK(d_vals.upload(vals.data(), vals.size()));
    HIP_OK(launch_adj_scatter(ix->adj.p, b.adj_stride, d_dirty.p, d_vals.p, (uint32_t)dirty.size(), s));
    ix->adj_version++;
    uint32_t hc[3];
    int herr = 0;
    HIP_OK(hipMemcpyAsync(hc, b.counts.p, sizeof hc, hipMemcpyDeviceToHost, s));
    HIP_OK(hipMemcpyAsync(&herr, ix->error.p, sizeof(int), hipMemcpyDeviceToHost, s));
    HIP_OK(hipStreamSynchronize(s));
    int serr = 0;  // the insertion searches' flag (their launch context on s)
    if (take_device_error(ix, s, &serr)) return -1;
    herr |= serr;
    if (herr) {
      (void)hipMemset(ix->error.p, 0, sizeof(int));
      return fail("ngt_amd_build_insert: device error flag %d (1 unchecked-set spill full; DVP tree: 2 already "
                  "existed, 8 all split distances equal, 16 node capacity, 32 illegal pivot)", herr);
    }
    b.n_leaf = hc[0];
    b.n_internal = hc[1];
    b.root = hc[2];
    mark(5);
  }
  if (prof)
    fprintf(stderr, "build_insert %zu objects: seeds %.3f s, search %.3f s, pairs+merge %.3f s, host graph %.3f s, "
            "tree insert %.3f s, adjacency %.3f s; search kernel %.3f s, per query %.1f distances %.1f expansions, "
            "mean per-batch max expansions %.1f\n", todo.size(), st[0], st[1], st[2], st[3], st[4], st[5], k_ms / 1e3,
            dc / std::max<uint64_t>(nsearched, 1), ex / std::max<uint64_t>(nsearched, 1),
            ex_max / std::max<double>(1.0, (double)((todo.size() + B - 1) / B)));
  if (prof) {
    const double nq = (double)std::max<uint64_t>(nsearched, 1);
    // counters [3], [5..7]: spilled-visited flag, max unchecked, 0, 0 -- or, in
    // the NGT_AMD_STAMPS build, rest/pop/adjacency/eval cycles
    fprintf(stderr, "build_insert counters per query: c3 %.4g c5 %.4g (max %.4g) c6 %.4g c7 %.4g\n", c3 / nq,
            c5 / nq, c5_max, c6 / nq, c7 / nq);
  }
  return 0;
}

extern "C" int ngt_amd_build_set_graph(ngt_amd_index* ix, const uint64_t* offsets, const uint32_t* ids,
                                       const float* dists, uint64_t graph_rows) {
  if (!ix || !ix->build || !offsets || graph_rows > ix->nrows) return fail("ngt_amd_build_set_graph: bad arguments");
  if (offsets[graph_rows] && (!ids || !dists)) return fail("ngt_amd_build_set_graph: bad arguments");
  HIP_OK(hipSetDevice(ix->device));
  ServeHold serve_hold(ix);
  BuildState& b = *ix->build;
  const uint64_t S = b.adj_stride;
  std::vector<uint32_t> adj((size_t)ix->nrows * S, 0u);
  b.graph_size = 0;
  for (uint64_t v = 0; v < graph_rows; v++) {
    const uint64_t e0 = offsets[v], e1 = offsets[v + 1];
    auto& node = b.graph[v];
    node.clear();
    for (uint64_t e = e0; e < e1; e++) {
      if (ids[e] == 0 || ids[e] >= ix->nrows) return fail("ngt_amd_build_set_graph: edge %u out of range", ids[e]);
      node.push_back({ids[e], dists[e]});
      if (e - e0 < S) adj[(size_t)v * S + (e - e0)] = ids[e];
    }
    b.in_graph[v] = e1 > e0 ? 1 : 0;
    if (e1 > e0) b.graph_size = v + 1;
  }
  HIP_OK(hipMemcpy(ix->adj.p, adj.data(), adj.size() * sizeof(uint32_t), hipMemcpyHostToDevice));
  ix->adj_version++;
  return 0;
}

extern "C" int ngt_amd_build_set_tree(ngt_amd_index* ix, const uint32_t* leaf_parent, const uint64_t* leaf_off,
                                      const uint32_t* leaf_ids, const float* leaf_dists,
                                      const uint8_t* leaf_has_pivot, const void* leaf_pivot, uint32_t n_leaf,
                                      const uint32_t* in_parent, const void* in_pivot, const uint32_t* in_child,
                                      const float* in_border, uint32_t n_internal, uint32_t root) {
  if (!ix || !ix->build || !leaf_parent || !leaf_off || !leaf_has_pivot || !leaf_pivot || n_leaf < 2 ||
      n_internal < 1 || (n_internal > 1 && (!in_parent || !in_pivot || !in_child || !in_border)))
    return fail("ngt_amd_build_set_tree: bad arguments");
  HIP_OK(hipSetDevice(ix->device));
  BuildState& b = *ix->build;
  b.n_leaf = 2;
  b.n_internal = 1;
  if (ensure_tree_capacity(ix, b, n_leaf, n_internal)) return -1;
  const uint64_t rb = ix->row_bytes;
  std::vector<uint32_t> cnt(n_leaf), lids((size_t)n_leaf * kLeafCap, 0u);
  std::vector<float> ldst((size_t)n_leaf * kLeafCap, 0.f);
  for (uint32_t l = 0; l < n_leaf; l++) {
    const uint64_t c = leaf_off[l + 1] - leaf_off[l];
    if (c > kLeafCap - 1) return fail("ngt_amd_build_set_tree: leaf %u holds %llu objects", l, (unsigned long long)c);
    cnt[l] = (uint32_t)c;
    for (uint64_t j = 0; j < c; j++) {
      lids[(size_t)l * kLeafCap + j] = leaf_ids[leaf_off[l] + j];
      ldst[(size_t)l * kLeafCap + j] = leaf_dists ? leaf_dists[leaf_off[l] + j] : 0.f;
    }
  }
  HIP_OK(hipMemcpy(b.lf_count.p, cnt.data(), n_leaf * sizeof(uint32_t), hipMemcpyHostToDevice));
  HIP_OK(hipMemcpy(b.lf_ids.p, lids.data(), lids.size() * sizeof(uint32_t), hipMemcpyHostToDevice));
  HIP_OK(hipMemcpy(b.lf_dist.p, ldst.data(), ldst.size() * sizeof(float), hipMemcpyHostToDevice));
  HIP_OK(hipMemcpy(b.lf_parent.p, leaf_parent, n_leaf * sizeof(uint32_t), hipMemcpyHostToDevice));
  HIP_OK(hipMemcpy(b.lf_has_pivot.p, leaf_has_pivot, n_leaf, hipMemcpyHostToDevice));
  HIP_OK(hipMemcpy(b.lf_pivot.p, leaf_pivot, (size_t)n_leaf * rb, hipMemcpyHostToDevice));
  if (n_internal > 1) {
    HIP_OK(hipMemcpy(b.in_parent.p, in_parent, n_internal * sizeof(uint32_t), hipMemcpyHostToDevice));
    HIP_OK(hipMemcpy(b.in_pivot.p, in_pivot, (size_t)n_internal * rb, hipMemcpyHostToDevice));
    HIP_OK(hipMemcpy(b.in_child.p, in_child, (size_t)n_internal * 5 * sizeof(uint32_t), hipMemcpyHostToDevice));
    HIP_OK(hipMemcpy(b.in_border.p, in_border, (size_t)n_internal * 4 * sizeof(float), hipMemcpyHostToDevice));
  }
  const uint32_t c3[3] = {n_leaf, n_internal, root};
  HIP_OK(b.counts.upload(c3, 3));
  b.n_leaf = n_leaf;
  b.n_internal = n_internal;
  b.root = root;
  return 0;
}

extern "C" int ngt_amd_build_graph_size(const ngt_amd_index* ix, uint64_t* graph_size, uint64_t* nedges) {
  if (!ix || !ix->build || !graph_size || !nedges) return fail("ngt_amd_build_graph_size: bad arguments");
  const BuildState& b = *ix->build;
  *graph_size = b.graph_size;
  uint64_t e = 0;
  for (uint64_t v = 0; v < b.graph_size; v++) e += b.graph[v].size();
  *nedges = e;
  return 0;
}

extern "C" int ngt_amd_build_get_graph(const ngt_amd_index* ix, uint64_t* offsets, uint32_t* ids, float* dists) {
  if (!ix || !ix->build || !offsets) return fail("ngt_amd_build_get_graph: bad arguments");
  const BuildState& b = *ix->build;
  uint64_t e = 0;
  offsets[0] = 0;
  for (uint64_t v = 0; v < b.graph_size; v++) {
    for (const auto& x : b.graph[v]) {
      if (ids) ids[e] = x.first;
      if (dists) dists[e] = x.second;
      e++;
    }
    offsets[v + 1] = e;
  }
  return 0;
}

extern "C" int ngt_amd_build_tree_size(const ngt_amd_index* ix, uint32_t* n_leaf, uint32_t* n_internal,
                                       uint64_t* n_leaf_ids) {
  if (!ix || !ix->build || !n_leaf || !n_internal || !n_leaf_ids) return fail("ngt_amd_build_tree_size: bad arguments");
  const BuildState& b = *ix->build;
  HIP_OK(hipSetDevice(ix->device));
  std::vector<uint32_t> cnt(b.n_leaf);
  HIP_OK(hipMemcpy(cnt.data(), b.lf_count.p, b.n_leaf * sizeof(uint32_t), hipMemcpyDeviceToHost));
  uint64_t t = 0;
  for (uint32_t i = 1; i < b.n_leaf; i++) t += cnt[i];
  *n_leaf = b.n_leaf;
  *n_internal = b.n_internal;
  *n_leaf_ids = t;
  return 0;
}

extern "C" int ngt_amd_build_get_tree(const ngt_amd_index* ix, uint32_t* leaf_parent, uint64_t* leaf_off,
                                      uint32_t* leaf_ids, float* leaf_dists, uint8_t* leaf_has_pivot,
                                      void* leaf_pivot, uint32_t* in_parent, void* in_pivot, uint32_t* in_child,
                                      float* in_border) {
  if (!ix || !ix->build || !leaf_parent || !leaf_off || !leaf_has_pivot || !leaf_pivot || !in_parent ||
      !in_pivot || !in_child || !in_border)
    return fail("ngt_amd_build_get_tree: bad arguments");
  const BuildState& b = *ix->build;
  HIP_OK(hipSetDevice(ix->device));
  const uint64_t rb = ix->row_bytes;
  const uint32_t nl = b.n_leaf, ni = b.n_internal;
  std::vector<uint32_t> cnt(nl), lids((size_t)nl * kLeafCap);
  std::vector<float> ldst((size_t)nl * kLeafCap);
  HIP_OK(hipMemcpy(cnt.data(), b.lf_count.p, nl * sizeof(uint32_t), hipMemcpyDeviceToHost));
  HIP_OK(hipMemcpy(lids.data(), b.lf_ids.p, lids.size() * sizeof(uint32_t), hipMemcpyDeviceToHost));
  HIP_OK(hipMemcpy(ldst.data(), b.lf_dist.p, ldst.size() * sizeof(float), hipMemcpyDeviceToHost));
  HIP_OK(hipMemcpy(leaf_parent, b.lf_parent.p, nl * sizeof(uint32_t), hipMemcpyDeviceToHost));
  HIP_OK(hipMemcpy(leaf_has_pivot, b.lf_has_pivot.p, nl, hipMemcpyDeviceToHost));
  HIP_OK(hipMemcpy(leaf_pivot, b.lf_pivot.p, (size_t)nl * rb, hipMemcpyDeviceToHost));
  HIP_OK(hipMemcpy(in_parent, b.in_parent.p, ni * sizeof(uint32_t), hipMemcpyDeviceToHost));
  HIP_OK(hipMemcpy(in_pivot, b.in_pivot.p, (size_t)ni * rb, hipMemcpyDeviceToHost));
  HIP_OK(hipMemcpy(in_child, b.in_child.p, (size_t)ni * 5 * sizeof(uint32_t), hipMemcpyDeviceToHost));
  HIP_OK(hipMemcpy(in_border, b.in_border.p, (size_t)ni * 4 * sizeof(float), hipMemcpyDeviceToHost));
  uint64_t e = 0;
  leaf_off[0] = 0;
  for (uint32_t i = 0; i < nl; i++) {
    const uint32_t c = i == 0 ? 0 : cnt[i];
    for (uint32_t j = 0; j < c; j++) {
      if (leaf_ids) leaf_ids[e] = lids[(size_t)i * kLeafCap + j];
      if (leaf_dists) leaf_dists[e] = ldst[(size_t)i * kLeafCap + j];
      e++;
    }
    leaf_off[i + 1] = e;
  }
  return 0;
}
