// coalesce.h -- serving concurrent single-query C-API callers (SURVEY.md 8(b),
// "Threading": the reference is safe for concurrent read-only searches on one
// handle, Capi.cpp:377-406 copying the query per call; the GPU build batches
// concurrent callers internally).
//
// A caller of ngt_search_index* / ngt_linear_search_index* /
// ngtqg_search_index enqueues its query and either becomes a *leader* -- it
// takes every pending request with the same search parameters (up to
// max_batch), runs them as ONE batched launch and hands each caller its rows --
// or waits until a leader has served it.  No background thread and no timed
// window: a request that finds a free leader slot launches at once, so an
// uncontended call pays nothing, and requests arriving while a batch is on the
// device accumulate into the next one (group commit).  max_leaders batches
// may be in flight together (they run on separate call streams).
//
//   NGT_AMD_COALESCE=0          every call is its own launch
//   NGT_AMD_COALESCE_LEADERS=n  batches in flight (default 2)
//   NGT_AMD_COALESCE_MAX=n      queries per batch (default 4096)
#pragma once
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "knobs.h"

#include <condition_variable>
#include <deque>
#include <exception>
#include <mutex>
#include <string>
#include <vector>

namespace ngt_amd {

// Parameters a batch must share (the kernels take them per launch).
struct CoalesceKey {
  int kind = 0;               // caller-defined (graph search, linear search, QG search)
  uint32_t size = 0;          // SearchContainer::size
  float epsilon = 0.f;
  float radius = 0.f;
  int64_t edge_size = 0;
  int seed_mode = 0;
  float expansion = 0.f;      // NGTQG result expansion
  bool operator==(const CoalesceKey& o) const {
    return kind == o.kind && size == o.size && memcmp(&epsilon, &o.epsilon, sizeof(float)) == 0 &&
           memcmp(&radius, &o.radius, sizeof(float)) == 0 && edge_size == o.edge_size &&
           seed_mode == o.seed_mode && memcmp(&expansion, &o.expansion, sizeof(float)) == 0;
  }
};

struct CoalesceReq {
  CoalesceKey key;
  const float* query = nullptr;  // [dim] floats, owned by the waiting caller
  // filled by the leader
  std::vector<uint32_t> ids;
  std::vector<float> dists;
  uint32_t n = 0;
  uint64_t counters[3] = {0, 0, 0};
  std::string err;
  bool done = false;
};

inline bool coalesce_enabled() {
  static const bool on = [] {
    const char* v = ngt_amd::knob("NGT_AMD_COALESCE");
    return !(v && atoi(v) == 0);
  }();
  return on;
}

class Coalescer {
 public:
  explicit Coalescer(uint32_t dim) : dim_(dim) {
    // 2 leaders (4 or 8: 3.1k / 2.6k vs 5.6k QPS at 32 threads)
    max_leaders_ = 2;
    max_batch_ = 4096u;
  }

  // runner(key, queries [nq][dim], nq, batch) fills every request of the batch.
  template <class F>
  void submit(CoalesceReq* r, F&& runner) {
    std::unique_lock<std::mutex> lk(mu_);
    q_.push_back(r);
    for (;;) {
      if (r->done) return;
      if (!q_.empty() && leaders_ < max_leaders_) {
        leaders_++;
        std::vector<CoalesceReq*> batch;
        const CoalesceKey k = q_.front()->key;
        for (auto it = q_.begin(); it != q_.end() && batch.size() < max_batch_;) {
          if ((*it)->key == k) {
            batch.push_back(*it);
            it = q_.erase(it);
          } else {
            ++it;
          }
        }
        lk.unlock();
        {
          // whatever the runner does (returns, throws anything), the batch is
          // marked done, the leader slot freed and the waiters woken
          struct Finish {
            Coalescer* self;
            std::unique_lock<std::mutex>& lk;
            std::vector<CoalesceReq*>& batch;
            ~Finish() {
              lk.lock();
              self->batches_++;
              self->served_ += batch.size();
              for (auto* b : batch) b->done = true;
              self->leaders_--;
              self->cv_.notify_all();
            }
          } fin{this, lk, batch};
          try {
            std::vector<float> qs(batch.size() * (size_t)dim_);
            for (size_t i = 0; i < batch.size(); i++)
              memcpy(qs.data() + i * dim_, batch[i]->query, dim_ * sizeof(float));
            runner(k, qs.data(), (uint32_t)batch.size(), batch);
          } catch (std::exception& e) {
            for (auto* b : batch) b->err = e.what();
          } catch (...) {
            for (auto* b : batch) b->err = "search failed with a non-standard exception";
          }
        }
        continue;
      }
      cv_.wait(lk);
    }
  }

  // launches issued and requests served so far (statistics for tests/bench)
  void stats(uint64_t* batches, uint64_t* served) {
    std::lock_guard<std::mutex> lk(mu_);
    *batches = batches_;
    *served = served_;
  }

 private:
  std::mutex mu_;
  std::condition_variable cv_;
  std::deque<CoalesceReq*> q_;
  int leaders_ = 0;
  int max_leaders_ = 2;
  uint32_t max_batch_ = 4096;
  uint32_t dim_;
  uint64_t batches_ = 0, served_ = 0;
};

}  // namespace ngt_amd
