// wellflow — LDS tile layouts and row helpers shared by the fused MLP kernels (mlp_fused.hip,
// mlp_step.hip): 64-row chunks of the F -> 256 -> 256 -> 1 network (reference mlp.py).
#pragma once
#include "common.h"

namespace wf {
namespace {
constexpr int MF_ROWS = 64;  // rows per chunk
constexpr int MF_H = 256;    // hidden width (both layers)

// dataset row of batch row gr (indices clamped into the dataset: never an out-of-bounds read)
__device__ __forceinline__ size_t data_row(const long long* rows, int gr, long nrows) {
  if (rows == nullptr) return (size_t)gr;
  long long r = rows[gr];
  r = r < 0 ? 0 : (r >= nrows ? nrows - 1 : r);
  return (size_t)r;
}

// [64 rows][256 units] bf16 tile, 16-B chunk c (units 8c..8c+7) of row r at chunk c ^ (r & 15)
// (32 chunks per row, 512-B rows): the B-fragment reads (16 rows x one chunk) hit 16 distinct
// 16-B bank groups, as do the row-wise copy-out reads.
__device__ __forceinline__ int tile_off(int row, int unit) {
  const int c = unit >> 3;
  return row * (MF_H * 2) + ((c ^ (row & 15)) << 4) + ((unit & 7) << 1);
}
// [64 rows][64 features] bf16 input tile (8 chunks per row, 128-B rows: rows r and r + 2
// share banks, so the chunk is swizzled by (row >> 1) & 7 — 16-row fragment reads of one
// chunk hit 16 distinct bank groups)
constexpr int MF_XROW = 128;
__device__ __forceinline__ int xtile_off(int row, int chunk) { return row * MF_XROW + ((chunk ^ ((row >> 1) & 7)) << 4); }
}  // namespace
}  // namespace wf
