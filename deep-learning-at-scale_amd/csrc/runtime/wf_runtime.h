// wellflow native host runtime — C ABI (loaded with ctypes by wellflow/data/native.py).
//
// The reference hands its data path to Spark's JVM (cnn.py:49 SparkSession, cnn.py:65
// spark.read.csv, cnn.py:68 randomSplit; SURVEY.md §2.3 "Spark JVM"). Here the host side of
// that path is native C++17 with no GPU code and no torch dependency:
//   * wf_csv_read   — multithreaded headerless-CSV parse against the submission schema
//                     (int / float / string, cnn.py:53-60 mapping), rows with an unparsable
//                     or missing cell dropped and counted (Spark would null them),
//                     string columns dictionary-encoded per column;
//   * wf_window_starts / wf_gather_windows — sliding-window enumeration inside each series
//                     and the [B, T, F] batch gather (one T x F memcpy per window);
//   * wf_prefetcher — background worker threads that gather the next batches into a ring of
//                     caller-owned (pinned) host buffers while the GPU trains on the current.
#pragma once
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum { WF_INT = 0, WF_FLOAT = 1, WF_STRING = 2 };

typedef struct wf_table wf_table;

// Parse `path` (headerless unless `header`), `ncols` fields of kinds[] (WF_*), `delim`
// separator, `nthreads` workers (<= 0: hardware concurrency). NULL on error (message in err).
wf_table* wf_csv_read(const char* path, int ncols, const int* kinds, char delim, int header, int nthreads,
                      char* err, int errlen);
int64_t wf_table_rows(const wf_table* t);
int64_t wf_table_dropped(const wf_table* t);
const int64_t* wf_table_int(const wf_table* t, int col);     // WF_INT columns
const float* wf_table_float(const wf_table* t, int col);     // WF_FLOAT columns
const int32_t* wf_table_codes(const wf_table* t, int col);   // WF_STRING: code per row
int32_t wf_table_vocab_size(const wf_table* t, int col);     // distinct strings (first-seen order)
int64_t wf_table_vocab_bytes(const wf_table* t, int col);    // total bytes of the vocabulary
// vocabulary as one byte buffer + vocab_size + 1 offsets
void wf_table_vocab(const wf_table* t, int col, char* bytes, int64_t* offsets);
void wf_table_free(wf_table* t);

// First row of every length-T window (stride) that stays inside one series; groups[i] = series
// id of row i (rows in time order inside a series), NULL = one series. Returns the count;
// writes at most `cap` starts (call with out = NULL to size).
int64_t wf_window_starts(const int64_t* groups, int64_t n, int T, int stride, int64_t* out, int64_t cap);

// out[b] = rows[starts[idx[b]] : +T] ([T, F] fp32 each); y_out[b] = y[starts[idx[b]] + T - 1]
// when y / y_out are non-NULL. idx NULL = identity.
void wf_gather_windows(const float* rows, int F, const int64_t* starts, const int64_t* idx, int64_t B, int T,
                       float* out, const float* y, float* y_out, int nthreads);

typedef struct wf_prefetcher wf_prefetcher;
// `nslots` ring slots of caller-owned buffers x_slots[k] ([B, T, F] fp32) / y_slots[k] ([B]).
wf_prefetcher* wf_prefetch_create(const float* rows, int F, const int64_t* starts, const float* y, int T, int B,
                                  int nslots, float* const* x_slots, float* const* y_slots, int nthreads);
// Queue a gather of the windows idx[0..n) (n <= B; copied) into slot k (asynchronous).
int wf_prefetch_submit(wf_prefetcher* p, int slot, const int64_t* idx, int64_t n);
// Block until slot k's last submitted gather is complete; returns its row count.
int64_t wf_prefetch_wait(wf_prefetcher* p, int slot);
void wf_prefetch_destroy(wf_prefetcher* p);

#ifdef __cplusplus
}
#endif
