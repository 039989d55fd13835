// kmeans_ngt.h -- NGT::Clustering::kmeansWithNGT (lib/NGT/Clustering.h:440-760)
// as NGTQ's buildMultipleLocalCodebooks drives it for the local codebooks of
// a quantized graph (lib/NGT/NGTQ/Quantizer.h:1846-1858): Head
// initialisation (:260-267), epsilon 0.10 .. 0.50 in float steps of 0.05, up
// to 20 iterations each of assignWithNGT (:440-577: one NGT search per
// centroid over the sample index, every (object, centroid, distance) entry
// sorted by std::sort on distance alone, nearest-first assignment, brute force
// for the objects no search returned, moveFartherObjectsToEmptyClusters
// :405-428) and calculateCentroid (:580-605: float means in member order).
// Host logic only: the searches are supplied by the caller (the device graph
// search, bit-identical to NGT::Index::search).  Header-only so the test
// harness (tests/golden/kmeans_harness.cpp) runs the same code against the
// reference's own search.
#pragma once
#include <math.h>
#include <stddef.h>
#include <stdint.h>

#include <algorithm>
#include <cfloat>
#include <functional>
#include <limits>
#include <string>
#include <vector>

namespace ngt_amd {
namespace kmeans {

struct Entry {
  Entry() {}
  Entry(size_t v, size_t c, double d) : vectorID((uint32_t)v), centroidID((uint32_t)c), distance(d) {}
  bool operator<(const Entry& e) const { return distance > e.distance; }  // Clustering.h:64
  uint32_t vectorID = 0;
  uint32_t centroidID = 0;
  double distance = 0.0;
};

struct Cluster {
  std::vector<Entry> members;
  std::vector<float> centroid;
};

// search(queries, size, epsilon, results): NGT::Index::search of every query
// (size results, explorationCoefficient 1 + epsilon) over the sample index
// whose object i + 1 is vectors[i]; results[q] = (id, distance) in result
// order.  False on failure.
using SearchFn = std::function<bool(const std::vector<std::vector<float>>&, size_t, float,
                                    std::vector<std::vector<std::pair<uint32_t, float>>>&)>;

// sumOfSquares of the AVX build (Clustering.h:194-214): 8-lane float partial
// sums, their sum, then the tail in double
inline double sum_of_squares(const float* a, const float* b, size_t size) {
  float lanes[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  size_t i = 0;
  for (; i + 8 <= size; i += 8)
    for (int l = 0; l < 8; l++) {
      const float v = a[i + l] - b[i + l];
      lanes[l] = fmaf(v, v, lanes[l]);
    }
  double s = lanes[0] + lanes[1] + lanes[2] + lanes[3] + lanes[4] + lanes[5] + lanes[6] + lanes[7];
  for (; i < size; i++) {
    const double d = a[i] - b[i];
    s = fma(d, d, s);
  }
  return s;
}

inline double distance_l2(const std::vector<float>& a, const std::vector<float>& b) {
  return sqrt(sum_of_squares(a.data(), b.data(), a.size()));
}

inline bool move_farther_objects_to_empty_clusters(std::vector<Cluster>& clusters, std::string& err) {
  for (size_t ci = 0; ci < clusters.size(); ci++) {
    if (!clusters[ci].members.empty()) continue;
    double mx = -DBL_MAX;
    size_t maxc = 0;
    for (size_t sc = 0; sc < clusters.size(); sc++)
      if (clusters[sc].members.size() >= 2 && clusters[sc].members.back().distance > mx) {
        maxc = sc;
        mx = clusters[sc].members.back().distance;
      }
    if (mx == -DBL_MAX) {
      err = "Clustering::moveFartherObjectsToEmptyClusters: Not found max.";
      return false;
    }
    clusters[ci].members.push_back(clusters[maxc].members.back());
    clusters[ci].members.back().centroidID = (uint32_t)ci;
    clusters[maxc].members.pop_back();
  }
  return true;
}

inline bool assign_with_ngt(const SearchFn& search, const std::vector<std::vector<float>>& vectors,
                            std::vector<Cluster>& clusters, size_t result_size, float epsilon, size_t cluster_size,
                            std::string& err) {
  const size_t n = vectors.size();
  std::vector<std::vector<float>> queries;
  for (auto& c : clusters) queries.push_back(c.centroid);
  std::vector<std::vector<std::pair<uint32_t, float>>> res;
  if (!search(queries, result_size, epsilon, res)) {
    err = "search failed";
    return false;
  }
  std::vector<Entry> sorted;
  for (size_t ci = 0; ci < clusters.size(); ci++)
    for (auto& r : res[ci]) sorted.push_back(Entry(r.first - 1, ci, r.second));
  std::vector<bool> assigned(n, false);
  std::sort(sorted.begin(), sorted.end());
  for (auto& c : clusters) c.members.clear();
  for (auto it = sorted.rbegin(); it != sorted.rend(); ++it) {
    const size_t o = it->vectorID, c = it->centroidID;
    if (clusters[c].members.size() >= cluster_size) continue;
    if (!assigned[o]) {
      assigned[o] = true;
      clusters[c].members.push_back(*it);
      clusters[c].members.back().centroidID = (uint32_t)c;
    }
  }
  std::vector<uint32_t> rest;
  for (size_t i = 0; i < n; i++)
    if (!assigned[i]) rest.push_back((uint32_t)i);
  if (cluster_size < std::numeric_limits<size_t>::max()) {
    // clusters of bounded size (Clustering.h:505-548)
    do {
      std::vector<std::vector<Entry>> na(rest.size());
      const size_t nclosest = (size_t)1 * 1024 * 1024 * 1024 / 16 / (rest.size() == 0 ? 1 : rest.size());
      for (size_t vi = 0; vi < rest.size(); vi++) {
        if (assigned[rest[vi]]) continue;
        std::vector<Entry> ds;
        for (size_t ci = 0; ci < clusters.size(); ci++) {
          if (clusters[ci].members.size() >= cluster_size) continue;
          ds.push_back(Entry(rest[vi], ci, distance_l2(vectors[rest[vi]], clusters[ci].centroid)));
        }
        std::sort(ds.begin(), ds.end());
        const size_t topk = ds.size() < nclosest ? ds.size() : nclosest;
        na[vi].assign(ds.end() - topk, ds.end());
      }
      sorted.clear();
      for (auto& v : na) sorted.insert(sorted.end(), v.begin(), v.end());
      std::sort(sorted.begin(), sorted.end());
      for (auto it = sorted.rbegin(); it != sorted.rend(); ++it) {
        const size_t o = it->vectorID, c = it->centroidID;
        if (clusters[c].members.size() >= cluster_size) continue;
        if (!assigned[o]) {
          assigned[o] = true;
          clusters[c].members.push_back(*it);
          clusters[c].members.back().centroidID = (uint32_t)c;
        }
      }
    } while (std::any_of(assigned.begin(), assigned.end(), [](bool x) { return !x; }));
  } else {
    std::vector<Entry> na(rest.size());
    for (size_t vi = 0; vi < rest.size(); vi++) {
      double mind = DBL_MAX;
      size_t minc = (size_t)-1;
      for (size_t ci = 0; ci < clusters.size(); ci++) {
        const double d = distance_l2(vectors[rest[vi]], clusters[ci].centroid);
        if (d < mind) {
          mind = d;
          minc = ci;
        }
      }
      na[vi] = Entry(rest[vi], minc, mind);
    }
    for (auto& e : na) clusters[e.centroidID].members.push_back(e);
    if (!move_farther_objects_to_empty_clusters(clusters, err)) return false;
  }
  return true;
}

// calculateCentroid (Clustering.h:580-605); < 0 on an empty cluster
inline double calculate_centroid(const std::vector<std::vector<float>>& vectors, std::vector<Cluster>& clusters) {
  double distance = 0.0;
  for (auto& c : clusters) {
    if (c.members.empty()) return -1.0;  // "Clustering: Fatal Error. No member!"
    std::vector<float> mean(vectors[0].size(), 0.0f);
    for (auto& m : c.members) {
      const std::vector<float>& v = vectors[m.vectorID];
      for (size_t i = 0; i < mean.size(); i++) mean[i] += v[i];
    }
    // `*mit /= members.size()` as the reference's -Ofast build emits it: one
    // float reciprocal, then a multiply per element (-freciprocal-math)
    const float inv = 1.0f / (float)c.members.size();
    for (auto& x : mean) x *= inv;
    distance += distance_l2(c.centroid, mean);
    c.centroid = mean;
  }
  return distance;
}

struct Params {
  float epsilon_from = 0.10f, epsilon_to = 0.50f, epsilon_step = 0.05f;  // Quantizer.h:1848-1850
  size_t maximum_iteration = 20;                                        // :1851
  size_t result_size_coefficient = 5;                                   // Clustering.h:102
  // Clustering::clusterSizeConstraint is never initialised by the constructor
  // NGTQ uses; the reference's build behaves as false (pinned by the
  // single-thread fixtures, tests/golden/qg_kmeans_st.npz)
  bool cluster_size_constraint = false;
};

// kmeansWithNGT(index, numberOfClusters, clusters) (Clustering.h:724-742):
// centroids in cluster order; returns the last diff (0 = converged), < 0 on error
inline double kmeans_with_ngt(const SearchFn& search, const std::vector<std::vector<float>>& vectors,
                              size_t nclusters, const Params& p, std::vector<std::vector<float>>& centroids,
                              std::string& err) {
  std::vector<Cluster> clusters;
  const size_t nh = nclusters > vectors.size() ? vectors.size() : nclusters;
  for (size_t i = 0; i < nh; i++) {
    Cluster c;
    c.centroid = vectors[i];
    clusters.push_back(c);
  }
  double diff = DBL_MAX;
  for (float eps = p.epsilon_from; eps <= p.epsilon_to; eps += p.epsilon_step) {
    // kmeansWithNGT(index, vectors, n, clusters, epsilon) (:648-676)
    size_t cluster_size = std::numeric_limits<size_t>::max();
    if (p.cluster_size_constraint) cluster_size = (size_t)ceil((double)vectors.size() / (double)nclusters);
    const size_t result_size = p.result_size_coefficient * vectors.size() / clusters.size();
    diff = 0.0;
    for (size_t it = 0; it < p.maximum_iteration; it++) {
      if (!assign_with_ngt(search, vectors, clusters, result_size, eps, cluster_size, err)) return -1.0;
      diff = calculate_centroid(vectors, clusters);
      if (diff < 0.0) {
        err = "Clustering: Fatal Error. No member!";
        return -1.0;
      }
      if (diff == 0.0) break;
    }
    if (diff == 0.0) break;
  }
  centroids.clear();
  for (auto& c : clusters) centroids.push_back(c.centroid);
  return diff;
}

}  // namespace kmeans
}  // namespace ngt_amd
