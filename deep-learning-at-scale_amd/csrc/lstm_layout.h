// wellflow — LSTM state layouts shared by the per-step and the persistent kernels.
#pragma once
#include "common.h"

namespace wf {

// Forward gate-column order (rows of the packed bf16 weights Wp, columns of the forward
// GEMM): a 64-column tile holds gates i,f,g,o of 16 consecutive units, so one lane's four
// 16x16 MFMA fragments carry all four gates of its unit.
__device__ __forceinline__ int gate_col(int gate, int u) { return (u >> 4) * 64 + gate * 16 + (u & 15); }
// Backward gate-column order (columns of DG, rows of the fp32 master W / its gradient,
// columns of WhhT): unit-major, gate-minor. A lane's four gate gradients of one (row,
// unit) are ONE 8-B store (16 lanes = a full 128-B line) instead of four 2-B stores.
__host__ __device__ __forceinline__ int dg_col(int gate, int u) { return 4 * u + gate; }

// Fragment-native (FN) layout of the per-(row, unit) state the backward pass re-reads
// (C, S, dc carry): 16x16 blocks, block (m>>4, u>>4) row-major over H/16 unit blocks;
// inside a block element (m, u) sits at lane ((m&15)>>2)*16 + (u&15), slot m&3 — exactly
// where the 16x16 MFMA C map puts it, so every lane moves 16-32 contiguous bytes.
// Batch rows are padded to a multiple of 16 (fn_rows).
// S (saved gates, 4 bf16 per element = 32 B per lane per block) is stored as two HALVES of
// 16 B per lane: rows 0-1 of the lane's 4 at bf16 offset lane * 8, rows 2-3 at 512 + lane * 8,
// so each 16-B store / load instruction of a wave covers 1 KiB contiguously (a lane-interleaved
// 32-B slot made every instruction touch twice the cache lines with 16-B holes; the
// forward's C / S stores were 23 % of its time, tools/pf_time.py dbg 4).
constexpr int kFnSHalf = 512;  // bf16 offset of the second half in a 16x16 S block
__host__ __device__ __forceinline__ int fn_rows(int B) { return (B + 15) & ~15; }

// Non-temporal 16-B accesses for the read-once / write-once streams (saved gates S, the
// cell-state history as read by the backward): they should not evict the operands the
// step GEMMs reuse through L2 (recurrent weights, the previous step's activations).
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint4 ld16(const void* p, int nt) {
  u32x4 v = nt ? __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p))
               : *reinterpret_cast<const u32x4*>(p);
  return make_uint4(v[0], v[1], v[2], v[3]);
}
__device__ __forceinline__ void st16(void* p, uint4 v, int nt) {
  const u32x4 w = {v.x, v.y, v.z, v.w};
  if (nt) __builtin_nontemporal_store(w, reinterpret_cast<u32x4*>(p));
  else *reinterpret_cast<u32x4*>(p) = w;
}
__device__ __forceinline__ size_t fn_block(int mrow0, int u, int H) {
  return (size_t)(mrow0 >> 4) * (H >> 4) + (u >> 4);
}

}  // namespace wf
