// Coalescing of concurrent host Verify calls (hipbls.hip hbls_verify_batch for small n): the first
// caller of an idle queue becomes the leader, gathers more requests for at most `us` microseconds
// (or until `max_items` items are queued), runs them as ONE batch and marks every request done.
// Requests that arrive while batches run form the next batch, led by one of them as soon as fewer
// than `inflight` batches are running.  Host code only (no HIP); the batch runner is a template
// parameter so that tests/native/hostcheck.cpp drives the same state machine with a stub runner
// (tests/test_coalesce.py: every request completes exactly once, at most `inflight` batches run at
// once, late arrivals lead a second batch while the first runs).
#pragma once
#include <chrono>
#include <condition_variable>
#include <cstddef>
#include <cstdint>
#include <deque>
#include <mutex>
#include <string>
#include <vector>

namespace hb {

struct VReq {
  const uint8_t *pk = nullptr, *sig = nullptr, *msg = nullptr;
  const uint64_t* off = nullptr;
  const uint32_t* len = nullptr;
  size_t n = 0;
  uint8_t* st = nullptr;
  int rc = 0;
  std::string err;
  bool done = false;
  bool taken = false;  // in a batch (running or about to)
};

struct CoalesceParams {
  size_t us = 200;             // gathering window (HBLS_COALESCE_US; 0 = no coalescing)
  size_t max_items = 1u << 16;  // a batch closes at this many items (HBLS_COALESCE_MAX)
  size_t inflight = 3;         // batches running at once (HBLS_COALESCE_INFLIGHT)
};

struct Coalescer {
  std::mutex mu;
  std::condition_variable cv;
  std::deque<VReq*> q;
  size_t queued = 0;
  int active = 0;          // batches running (each on its own host-call context)
  bool gathering = false;  // a leader is collecting the next batch
  std::chrono::steady_clock::time_point last_end{};  // when the previous batch finished
  // observed (tests): most batches running at once, batches run
  int max_active = 0;
  size_t batches = 0;
};

// Submit `me` and return once a batch containing it has run.  run(std::vector<VReq*>&) runs a batch
// (sets st / rc / err of each request) without holding c.mu.
template <class Run>
void coalesce_submit(Coalescer& c, const CoalesceParams& p, VReq& me, Run&& run) {
  std::unique_lock<std::mutex> lk(c.mu);
  c.q.push_back(&me);
  c.queued += me.n;
  c.cv.notify_all();
  while (!me.done) {
    // a caller whose request is still queued leads the next batch when a context is free
    if (!me.taken && !c.gathering && (size_t)c.active < p.inflight) {
      c.gathering = true;
      c.active++;
      if (c.active > c.max_active) c.max_active = c.active;
      // gather more requests only in a busy period (batches running, or one finished within the
      // last few windows): a lone caller on an idle library runs at once, and under load the
      // requests that queue up meanwhile form the next batch
      const auto now = std::chrono::steady_clock::now();
      const bool busy = c.active > 1 || now - c.last_end < std::chrono::microseconds(4 * p.us) || c.q.size() > 1;
      const auto deadline = now + std::chrono::microseconds(busy ? p.us : 0);
      while (c.queued < p.max_items && std::chrono::steady_clock::now() < deadline) c.cv.wait_until(lk, deadline);
      std::vector<VReq*> batch(c.q.begin(), c.q.end());
      for (VReq* r : batch) r->taken = true;
      c.q.clear();
      c.queued = 0;
      c.gathering = false;
      c.batches++;
      c.cv.notify_all();  // the next leader may start gathering
      lk.unlock();
      run(batch);
      lk.lock();
      for (VReq* r : batch) r->done = true;
      c.active--;
      c.last_end = std::chrono::steady_clock::now();
      c.cv.notify_all();
    } else {
      c.cv.wait(lk);
    }
  }
}

}  // namespace hb
