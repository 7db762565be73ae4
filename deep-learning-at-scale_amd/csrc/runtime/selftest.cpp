// wellflow native runtime self-test: exercises the CSV reader (multi-worker), the window
// gather and the prefetcher's worker threads with known answers. Built and run by
// tests/test_runtime_cpu.py under -fsanitize=thread (data races in the prefetcher / parallel
// parse) and -fsanitize=address,undefined (bounds, lifetime, UB) — the host-side race and
// memory checking of SURVEY.md §5 (GPU sanitizers are not available on the MI355X pool).
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "wf_runtime.h"

#define CHECK(c)                                                     \
  do {                                                               \
    if (!(c)) {                                                      \
      std::fprintf(stderr, "selftest FAILED %s:%d: %s\n", __FILE__, __LINE__, #c); \
      return 1;                                                      \
    }                                                                \
  } while (0)

int main(int argc, char** argv) {
  const char* path = argc > 1 ? argv[1] : "/tmp/wf_selftest.csv";
  const int N = 200000;
  {
    FILE* f = std::fopen(path, "w");
    CHECK(f != nullptr);
    for (int i = 0; i < N; ++i) {
      if (i % 1000 == 7) std::fprintf(f, "w%d,%d,notanumber\n", i % 13, i);  // dropped
      std::fprintf(f, "\"w%d\",%d,%.3f\n", i % 13, i, i * 0.5);
    }
    std::fclose(f);
  }
  const int kinds[3] = {WF_STRING, WF_INT, WF_FLOAT};
  char err[256];
  wf_table* t = wf_csv_read(path, 3, kinds, ',', 0, 8, err, sizeof(err));
  CHECK(t != nullptr);
  CHECK(wf_table_rows(t) == N);
  CHECK(wf_table_dropped(t) == N / 1000);
  const int64_t* iv = wf_table_int(t, 1);
  const float* fv = wf_table_float(t, 2);
  const int32_t* codes = wf_table_codes(t, 0);
  CHECK(wf_table_vocab_size(t, 0) == 13);
  for (int i = 0; i < N; ++i) {
    CHECK(iv[i] == i);
    CHECK(std::fabs(fv[i] - i * 0.5f) <= 1e-3f * (1.f + i));
    CHECK(codes[i] == i % 13);  // first-appearance order
  }
  wf_table_free(t);
  std::remove(path);

  // windows: 3 series of lengths 50, 10, 40; T = 8
  std::vector<int64_t> groups;
  for (int s = 0, len[3] = {50, 10, 40}; s < 3; ++s)
    for (int k = 0; k < len[s]; ++k) groups.push_back(s);
  const int64_t n = (int64_t)groups.size(), T = 8, F = 5;
  const int64_t cnt = wf_window_starts(groups.data(), n, T, 1, nullptr, 0);
  CHECK(cnt == (50 - 7) + (10 - 7) + (40 - 7));
  std::vector<int64_t> starts(cnt);
  CHECK(wf_window_starts(groups.data(), n, T, 1, starts.data(), cnt) == cnt);
  std::vector<float> rows(n * F), y(n);
  for (int64_t i = 0; i < n * F; ++i) rows[i] = (float)i;
  for (int64_t i = 0; i < n; ++i) y[i] = (float)(-i);
  std::vector<int64_t> idx(cnt);
  for (int64_t b = 0; b < cnt; ++b) idx[b] = cnt - 1 - b;
  std::vector<float> out(cnt * T * F), yo(cnt);
  wf_gather_windows(rows.data(), F, starts.data(), idx.data(), cnt, T, out.data(), y.data(), yo.data(), 4);
  for (int64_t b = 0; b < cnt; ++b) {
    const int64_t s = starts[idx[b]];
    CHECK(out[b * T * F] == (float)(s * F));
    CHECK(out[b * T * F + T * F - 1] == (float)((s + T) * F - 1));
    CHECK(yo[b] == (float)(-(s + T - 1)));
  }

  // prefetcher: 3 slots, 4 workers, many rounds
  const int B = 16, NS = 3;
  std::vector<std::vector<float>> xs(NS, std::vector<float>(B * T * F)), ys(NS, std::vector<float>(B));
  float* xp[NS];
  float* yp[NS];
  for (int k = 0; k < NS; ++k) {
    xp[k] = xs[k].data();
    yp[k] = ys[k].data();
  }
  wf_prefetcher* p = wf_prefetch_create(rows.data(), F, starts.data(), y.data(), T, B, NS, xp, yp, 4);
  CHECK(p != nullptr);
  std::vector<int64_t> bidx(B);
  for (int round = 0; round < 200; ++round) {
    const int k = round % NS;
    for (int b = 0; b < B; ++b) bidx[b] = (round * 7 + b * 3) % cnt;
    CHECK(wf_prefetch_submit(p, k, bidx.data(), B) == 0);
    if (round >= NS - 1) {
      const int kw = (round - (NS - 1)) % NS;
      CHECK(wf_prefetch_wait(p, kw) == B);
      const int r0 = round - (NS - 1);
      for (int b = 0; b < B; ++b) {
        const int64_t s = starts[(r0 * 7 + b * 3) % cnt];
        CHECK(xs[kw][b * T * F] == (float)(s * F));
        CHECK(ys[kw][b] == (float)(-(s + T - 1)));
      }
    }
  }
  wf_prefetch_destroy(p);
  std::printf("selftest ok\n");
  return 0;
}
