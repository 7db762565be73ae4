// wellflow native runtime — sequence windows and the background batch prefetcher.
//
// A length-T window of series rows is ONE contiguous [T, F] block of the per-row feature
// matrix (rows are time-ordered inside each series), so gathering a [B, T, F] batch is B
// memcpys of T*F*4 bytes, spread over worker threads. The prefetcher runs those gathers on
// its own threads into a ring of caller-owned (pinned) buffers, so the host side of batch k+1
// overlaps the host->HBM copy and the GPU step of batch k (wellflow/data/native.py).
#include <algorithm>
#include <condition_variable>
#include <cstring>
#include <deque>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

#include "wf_runtime.h"

extern "C" int64_t wf_window_starts(const int64_t* groups, int64_t n, int T, int stride, int64_t* out, int64_t cap) {
  if (T <= 0 || stride <= 0) return 0;
  int64_t cnt = 0;
  int64_t i = 0;
  while (i < n) {
    int64_t j = i + 1;
    if (groups != nullptr)
      while (j < n && groups[j] == groups[i]) ++j;
    else
      j = n;
    for (int64_t s = i; s + T <= j; s += stride) {
      if (out != nullptr && cnt < cap) out[cnt] = s;
      ++cnt;
    }
    i = j;
  }
  return cnt;
}

namespace {

void gather_range(const float* rows, int F, const int64_t* starts, const int64_t* idx, int64_t b0, int64_t b1,
                  int T, float* out, const float* y, float* y_out) {
  const size_t blk = (size_t)T * (size_t)F;
  for (int64_t b = b0; b < b1; ++b) {
    const int64_t s = starts[idx != nullptr ? idx[b] : b];
    std::memcpy(out + (size_t)b * blk, rows + (size_t)s * (size_t)F, blk * sizeof(float));
    if (y != nullptr && y_out != nullptr) y_out[b] = y[s + T - 1];
  }
}

}  // namespace

extern "C" void wf_gather_windows(const float* rows, int F, const int64_t* starts, const int64_t* idx, int64_t B,
                                  int T, float* out, const float* y, float* y_out, int nthreads) {
  const size_t bytes = (size_t)B * (size_t)T * (size_t)F * sizeof(float);
  int nt = nthreads > 0 ? nthreads : (int)std::max(1u, std::thread::hardware_concurrency());
  nt = (int)std::min<int64_t>(nt, std::max<int64_t>(1, (int64_t)(bytes >> 20)));  // >= 1 MB per worker
  if (nt <= 1) {
    gather_range(rows, F, starts, idx, 0, B, T, out, y, y_out);
    return;
  }
  std::vector<std::thread> th;
  for (int i = 1; i < nt; ++i)
    th.emplace_back(gather_range, rows, F, starts, idx, B * i / nt, B * (i + 1) / nt, T, out, y, y_out);
  gather_range(rows, F, starts, idx, 0, B / nt, T, out, y, y_out);
  for (auto& t : th) t.join();
}

// ---------------------------------------------------------------- prefetcher
struct wf_prefetcher {
  const float* rows = nullptr;
  const int64_t* starts = nullptr;
  const float* y = nullptr;
  int F = 0, T = 0, B = 0;
  std::vector<float*> xs, ys;
  struct Slot {
    std::vector<int64_t> idx;
    int64_t n = 0;
    int pending = 0;  // outstanding pieces of the last submission
    uint64_t gen = 0;
  };
  std::vector<Slot> slots;
  std::mutex mu;
  std::condition_variable work_cv, done_cv;
  std::deque<std::function<void()>> q;
  std::vector<std::thread> workers;
  bool stop = false;
  int nthreads = 1;

  void loop() {
    for (;;) {
      std::function<void()> job;
      {
        std::unique_lock<std::mutex> lk(mu);
        work_cv.wait(lk, [&] { return stop || !q.empty(); });
        if (stop && q.empty()) return;
        job = std::move(q.front());
        q.pop_front();
      }
      job();
    }
  }
};

extern "C" wf_prefetcher* wf_prefetch_create(const float* rows, int F, const int64_t* starts, const float* y, int T,
                                             int B, int nslots, float* const* x_slots, float* const* y_slots,
                                             int nthreads) {
  if (nslots <= 0 || B <= 0 || T <= 0 || F <= 0) return nullptr;
  auto* p = new wf_prefetcher();
  p->rows = rows;
  p->starts = starts;
  p->y = y;
  p->F = F;
  p->T = T;
  p->B = B;
  p->xs.assign(x_slots, x_slots + nslots);
  p->ys.assign(y_slots, y_slots + nslots);
  p->slots.resize(nslots);
  p->nthreads = nthreads > 0 ? nthreads : 2;
  for (int i = 0; i < p->nthreads; ++i) p->workers.emplace_back([p] { p->loop(); });
  return p;
}

extern "C" int wf_prefetch_submit(wf_prefetcher* p, int slot, const int64_t* idx, int64_t n) {
  if (slot < 0 || slot >= (int)p->slots.size() || n < 0 || n > p->B) return -1;
  std::unique_lock<std::mutex> lk(p->mu);
  auto& s = p->slots[slot];
  p->done_cv.wait(lk, [&] { return s.pending == 0; });  // the slot's previous gather is done
  s.idx.assign(idx, idx + n);
  s.n = n;
  const int pieces = (int)std::max<int64_t>(1, std::min<int64_t>(p->nthreads, n / 64));
  s.pending = pieces;
  ++s.gen;
  for (int k = 0; k < pieces; ++k) {
    const int64_t b0 = n * k / pieces, b1 = n * (k + 1) / pieces;
    p->q.emplace_back([p, slot, b0, b1] {
      auto& sl = p->slots[slot];
      gather_range(p->rows, p->F, p->starts, sl.idx.data(), b0, b1, p->T, p->xs[slot],
                   p->y, p->ys[slot] != nullptr ? p->ys[slot] : nullptr);
      std::lock_guard<std::mutex> g(p->mu);
      if (--sl.pending == 0) p->done_cv.notify_all();
    });
  }
  lk.unlock();
  p->work_cv.notify_all();
  return 0;
}

extern "C" int64_t wf_prefetch_wait(wf_prefetcher* p, int slot) {
  if (slot < 0 || slot >= (int)p->slots.size()) return -1;
  std::unique_lock<std::mutex> lk(p->mu);
  auto& s = p->slots[slot];
  p->done_cv.wait(lk, [&] { return s.pending == 0; });
  return s.n;
}

extern "C" void wf_prefetch_destroy(wf_prefetcher* p) {
  if (p == nullptr) return;
  {
    std::lock_guard<std::mutex> g(p->mu);
    p->stop = true;
  }
  p->work_cv.notify_all();
  for (auto& t : p->workers) t.join();
  delete p;
}
