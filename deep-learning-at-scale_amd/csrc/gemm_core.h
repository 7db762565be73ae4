// wellflow — MFMA GEMM mainloop shared by every matmul-shaped kernel (gfx950).
//
// One workgroup = 256 threads = 4 waves laid out 2(M) x 2(N); each wave owns a
// (BM/2) x (BN/2) output tile built from v_mfma_f32_16x16x32_bf16 tiles
// (cdna_hip_programming.md §3). K advances in BK = 64 steps through a double-buffered
// LDS image filled by register staging (issue the next tile's global loads before the
// MFMAs, write them to the other LDS buffer after — §5.5 T14), one barrier per K-step.
//
// Operand layouts (logical operand X is [rows][K]):
//   K_CONTIG : X(r,k) = p[r*ld + k]     (activations, torch Linear weights [out][in])
//   MN_CONTIG: X(r,k) = p[k*ld + r]     (the "transposed" operand of a weight-gradient
//                                         GEMM, e.g. dW = dZ^T X reduces over the batch)
// K_CONTIG tiles are stored [rows][64] (128-B rows) with the 16-B chunk index XORed by
// (row>>1)&7, which makes the ds_read_b128 fragment reads conflict-free. MN_CONTIG tiles
// are stored [64 k][rows] with the 32-B chunk index XORed by (k&3)|((k>>1)&4); fragments
// come out with two ds_read_b64_tr_b16 hardware-transposed reads (T10), conflict-free
// for 128- and 256-row tiles.
#pragma once
#include <type_traits>

#include "common.h"

namespace wf {

enum : int { K_CONTIG = 0, MN_CONTIG = 1 };

typedef __attribute__((address_space(3))) bf16x4 lds_bf16x4;

// MN_CONTIG image swizzle for an R-row tile ([64 k][R] bf16, C = R/16 32-B chunks per k-row):
// data chunk j of k-row k sits in slot pos(j, hk(k)). Power-of-two C: XOR (as before);
// other C (the 288-wide weight-gradient tile): rotation mod C, still a bijection per row.
// 192-wide (C = 12) images rotate by h >> 1, not h: a 384-B k-row is 128 B mod the 256-B bank
// line, so row parity already shifts a 32-lane ds_read_b64_tr_b16 group by half a line; rotating
// by h as well put lanes (q, g) and (q, g + 1) on one bank pair for j >= 5 (PMC: 7.7 % of the
// dW kernel's cycles in bank conflicts). Rotation by h >> 1 is conflict-free for every j
// (exhaustive check over the fragment-read lane pattern). 288-wide (C = 18) images rotate by
// h >> 2: a 576-B k-row is 64 B mod the bank line, so k & 3 already spreads a group's 8-B slots
// over 4 row offsets and only the (k >> 3) & 1 half of h may rotate; rotation by h put 2-way
// conflicts on the subtiles that wrap mod 18 (PMC: 5.2 % of the 256x288 dW kernel's cycles).
// The offset table was found by exhaustive search over per-h rotations (0 conflicts for 32- and
// 64-deep images).
template <int R>
struct MnSwz {
  static constexpr int C = R / 16;
  static constexpr bool POW2 = (C & (C - 1)) == 0;
  static constexpr int RSH = C == 12 ? 1 : (C == 18 ? 2 : 0);
  __host__ __device__ static constexpr int hmask() { return POW2 ? C - 1 : 7; }
  __device__ static __forceinline__ int hk(int k) { return ((k & 3) | ((k >> 1) & 4)) & hmask(); }
  __device__ static __forceinline__ int pos(int j, int h) { return POW2 ? (j ^ h) : (j + (h >> RSH)) % C; }
  __device__ static __forceinline__ int data(int p, int h) { return POW2 ? (p ^ h) : (p + C - (h >> RSH)) % C; }
};

template <int R, int L, int NT_ = 256>
struct OpTile {
  static constexpr int NT = NT_;
  static constexpr int BK = 64;
  static constexpr int CHUNKS = R * BK / 8 / NT;  // 16-B chunks staged per thread
  static constexpr int BYTES = R * BK * 2;
  static_assert(CHUNKS >= 1 && R * BK / 8 == CHUNKS * NT, "tile / thread-count mismatch");
  static_assert(L == K_CONTIG || R >= 64, "MN_CONTIG tile needs >= 64 rows");
  static_assert(L == K_CONTIG || R % 16 == 0, "MN_CONTIG tile rows must be a multiple of 16");
  using SW = MnSwz<R>;

  __device__ static __forceinline__ int hk(int k) { return SW::hk(k); }

  // Global -> registers for the tile whose first row is row0 and first k is k0.
  // Rows >= rows or k >= kmax read as zero (the address is clamped, the value masked,
  // so the load itself is unconditional).
  __device__ static __forceinline__ void gload(const bf16_t* __restrict__ p, long ld, int rows,
                                               int kmax, int row0, int k0, uint4 (&r)[CHUNKS]) {
#pragma unroll
    for (int i = 0; i < CHUNKS; ++i) {
      const int q = threadIdx.x + i * NT;
      int gr, gk;
      if constexpr (L == K_CONTIG) {
        gr = row0 + (q >> 3);
        gk = k0 + (q & 7) * 8;
      } else {
        constexpr int CPR = R / 8;
        gk = k0 + q / CPR;
        gr = row0 + (q % CPR) * 8;
      }
      const bool ok = (gr < rows) && (gk < kmax);
      const size_t off = ok ? (L == K_CONTIG ? (size_t)gr * ld + gk : (size_t)gk * ld + gr) : 0;
      uint4 v = *reinterpret_cast<const uint4*>(p + off);
      if (!ok) v = make_uint4(0u, 0u, 0u, 0u);
      r[i] = v;
    }
  }

  __device__ static __forceinline__ void swrite(char* lds, const uint4 (&r)[CHUNKS]) {
#pragma unroll
    for (int i = 0; i < CHUNKS; ++i) {
      const int q = threadIdx.x + i * NT;
      int off;
      if constexpr (L == K_CONTIG) {
        const int row = q >> 3, c = q & 7;
        off = row * 128 + ((c ^ ((row >> 1) & 7)) << 4);
      } else {
        constexpr int CPR = R / 8;
        const int k = q / CPR, c8 = q % CPR;
        off = k * (R * 2) + (SW::pos(c8 >> 1, hk(k)) << 5) + ((c8 & 1) << 4);
      }
      *reinterpret_cast<uint4*>(lds + off) = r[i];
    }
  }

  // Lane's A/B fragment for mfma_f32_16x16x32_bf16: rows rs..rs+15 (tile-local),
  // k sub-step kk in {0,1}: lane l holds X[rs + (l&15)][32kk + 8(l>>4) + 0..7].
  __device__ static __forceinline__ bf16x8 frag(const char* lds, int rs, int kk, int lane) {
    if constexpr (L == K_CONTIG) {
      const int row = rs + (lane & 15);
      const int c = kk * 4 + (lane >> 4);
      const int off = row * 128 + ((c ^ ((row >> 1) & 7)) << 4);
      return *reinterpret_cast<const bf16x8*>(lds + off);
    } else {
      const int g = lane >> 4, q = (lane & 15) >> 2, p = lane & 3;
      const int j = rs >> 4;
      bf16x8 out;
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int k = kk * 32 + 8 * g + 4 * h + q;
        const int off = k * (R * 2) + (SW::pos(j, hk(k)) << 5) + p * 8;
        bf16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_bf16x4*)(lds + off));
        out[4 * h + 0] = v[0];
        out[4 * h + 1] = v[1];
        out[4 * h + 2] = v[2];
        out[4 * h + 3] = v[3];
      }
      return out;
    }
  }
};

// WM x WN waves (NT = 64 * WM * WN threads); 8-wave (512-thread) configurations keep two
// waves per SIMD on a 1-workgroup-per-CU grid, which the large-K LSTM GEMMs need.
template <int BM_, int BN_, int LA, int LB, int WM_ = 2, int WN_ = 2>
struct GemmCfg {
  static constexpr int BM = BM_, BN = BN_, BK = 64;
  static constexpr int WM = WM_, WN = WN_, NT = 64 * WM_ * WN_;
  static constexpr int WTM = BM / WM, WTN = BN / WN;
  static constexpr int TM = WTM / 16, TN = WTN / 16;
  static_assert(TM >= 1 && TN >= 1, "wave tile must be >= 16x16");
  static constexpr int LA_ = LA, LB_ = LB;
  using TA = OpTile<BM, LA, NT>;
  using TB = OpTile<BN, LB, NT>;
  static constexpr int STAGE = TA::BYTES + TB::BYTES;
  static constexpr int LDS_BYTES = 2 * STAGE;
};

// acc += A[m0:m0+BM, kbeg:kend] * B[n0:n0+BN, kbeg:kend]^T (operands in the layouts LA/LB).
// kbeg must be a multiple of 64; k >= kend reads as zero.
template <class C>
__device__ __forceinline__ void gemm_mainloop(const bf16_t* __restrict__ A, long lda, int M,
                                              const bf16_t* __restrict__ B, long ldb, int N,
                                              int kbeg, int kend, int m0, int n0, char* smem,
                                              f32x4 (&acc)[C::TM][C::TN]) {
  using TA = typename C::TA;
  using TB = typename C::TB;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int wm = wid / C::WN, wn = wid % C::WN;
#pragma unroll
  for (int i = 0; i < C::TM; ++i)
#pragma unroll
    for (int j = 0; j < C::TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = (kend - kbeg + C::BK - 1) / C::BK;
  if (nk <= 0) return;
  uint4 ra[TA::CHUNKS], rb[TB::CHUNKS];
  TA::gload(A, lda, M, kend, m0, kbeg, ra);
  TB::gload(B, ldb, N, kend, n0, kbeg, rb);
  TA::swrite(smem, ra);
  TB::swrite(smem + TA::BYTES, rb);
  __syncthreads();

  for (int kt = 0; kt < nk; ++kt) {
    char* cur = smem + (kt & 1) * C::STAGE;
    char* nxt = smem + ((kt & 1) ^ 1) * C::STAGE;
    const bool more = (kt + 1) < nk;
    if (more) {
      const int k0 = kbeg + (kt + 1) * C::BK;
      TA::gload(A, lda, M, kend, m0, k0, ra);
      TB::gload(B, ldb, N, kend, n0, k0, rb);
    }
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      bf16x8 a[C::TM], b[C::TN];
#pragma unroll
      for (int i = 0; i < C::TM; ++i) a[i] = TA::frag(cur, wm * C::WTM + i * 16, kk, lane);
#pragma unroll
      for (int j = 0; j < C::TN; ++j) b[j] = TB::frag(cur + TA::BYTES, wn * C::WTN + j * 16, kk, lane);
#pragma unroll
      for (int i = 0; i < C::TM; ++i)
#pragma unroll
        for (int j = 0; j < C::TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
    }
    if (more) {
      TA::swrite(nxt, ra);
      TB::swrite(nxt + TA::BYTES, rb);
    }
    __syncthreads();
  }
}

// ----------------------------------------------------------------------------------------
// Direct-to-LDS staging (global_load_lds_dwordx4): a wave-instruction writes 1 KiB of LDS
// lane-linearly (base + 16*lane), so the XOR swizzles above move onto the per-lane SOURCE
// address (cdna_hip_programming.md §5.4 rule 21) and the LDS images — hence frag() — stay
// exactly the ones the register-staged path writes. No VGPRs, no ds_write instructions.
template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

typedef __attribute__((address_space(3))) void lds_void;

template <int R, int L, int NT>
struct GldsTile {
  static constexpr int BYTES = R * 64 * 2;
  static constexpr int PIECES = BYTES / 1024;  // 1-KiB wave-instructions per tile
  static constexpr int NW = NT / 64;
  static constexpr int PER_WAVE = PIECES / NW;
  static_assert(PIECES % NW == 0 && PER_WAVE >= 1, "tile pieces must split evenly over waves");
  using SW = MnSwz<R>;

  __device__ static __forceinline__ int hk(int k) { return SW::hk(k); }

  // MN_CONTIG: the (k, column) whose 16 B land at LDS byte o of the tile image (pieces may
  // straddle k-rows when 2R does not divide 1 KiB)
  __device__ static __forceinline__ void mn_src(int o, int& k, int& col) {
    k = o / (R * 2);
    const int b = o % (R * 2);
    col = (SW::data(b >> 5, hk(k)) << 4) + (((b >> 4) & 1) << 3);
  }

  // Issue this wave's glds for the tile (row0, k0) -> lds_tile. All rows/k in range.
  __device__ static __forceinline__ void issue(const bf16_t* __restrict__ p, long ld, int row0,
                                               int k0, char* lds_tile, int wid, int lane) {
#pragma unroll
    for (int i = 0; i < PER_WAVE; ++i) {
      const int piece = i * NW + wid;
      const bf16_t* src;
      if constexpr (L == K_CONTIG) {
        const int row = piece * 8 + (lane >> 3);
        const int lc = (lane & 7) ^ ((row >> 1) & 7);
        src = p + (size_t)(row0 + row) * ld + k0 + lc * 8;
      } else {
        int k, col;
        mn_src(piece * 1024 + lane * 16, k, col);
        src = p + (size_t)(k0 + k) * ld + row0 + col;
      }
      __builtin_amdgcn_global_load_lds((const void*)src, (lds_void*)(lds_tile + piece * 1024), 16, 0, 0);
    }
  }
};

// Same contract as gemm_mainloop but for FULL tiles only (m0+BM <= M, n0+BN <= N,
// kbeg + 64*nk <= K): STAGES-deep LDS ring filled by glds, one barrier per K-step,
// counted vmcnt so STAGES-2 tiles stay in flight across it (guide §5 "Pipelining across
// barriers": raw s_barrier, never __syncthreads() while a glds is outstanding).
template <class C, int STAGES>
__device__ __forceinline__ void gemm_mainloop_glds(const bf16_t* __restrict__ A, long lda,
                                                   const bf16_t* __restrict__ B, long ldb, int kbeg,
                                                   int nk, int m0, int n0, char* smem,
                                                   f32x4 (&acc)[C::TM][C::TN]) {
  using TA = typename C::TA;
  using TB = typename C::TB;
  static_assert(STAGES >= 2 && STAGES <= 4, "2..4 stages");
  constexpr int LA_ = C::LA_, LB_ = C::LB_;
  using QA = GldsTile<C::BM, LA_, C::NT>;
  using QB = GldsTile<C::BN, LB_, C::NT>;
  constexpr int STAGE = QA::BYTES + QB::BYTES;
  constexpr int LPT = QA::PER_WAVE + QB::PER_WAVE;  // glds per wave per K-tile
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wid / C::WN, wn = wid % C::WN;
#pragma unroll
  for (int i = 0; i < C::TM; ++i)
#pragma unroll
    for (int j = 0; j < C::TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  if (nk <= 0) return;

#pragma unroll
  for (int s = 0; s < STAGES - 1; ++s) {
    if (s < nk) {
      char* st = smem + s * STAGE;
      QA::issue(A, lda, m0, kbeg + s * 64, st, wid, lane);
      QB::issue(B, ldb, n0, kbeg + s * 64, st + QA::BYTES, wid, lane);
    }
  }
  for (int t = 0; t < nk; ++t) {
    // tiles issued after t that may stay in flight: min(nk-1, t+STAGES-2) - t
    const int ahead = min(nk - 1, t + STAGES - 2) - t;
    if constexpr (STAGES >= 4) {
      if (ahead >= 2) wait_vmcnt<2 * LPT>();
      else if (ahead == 1) wait_vmcnt<LPT>();
      else wait_vmcnt<0>();
    } else if constexpr (STAGES == 3) {
      if (ahead >= 1) wait_vmcnt<LPT>();
      else wait_vmcnt<0>();
    } else {
      wait_vmcnt<0>();
    }
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    const int tn = t + STAGES - 1;
    if (tn < nk) {  // refill the stage every wave finished reading in iteration t-1
      char* st = smem + (tn % STAGES) * STAGE;
      QA::issue(A, lda, m0, kbeg + tn * 64, st, wid, lane);
      QB::issue(B, ldb, n0, kbeg + tn * 64, st + QA::BYTES, wid, lane);
    }
    const char* cur = smem + (t % STAGES) * STAGE;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      bf16x8 a[C::TM], b[C::TN];
#pragma unroll
      for (int i = 0; i < C::TM; ++i) a[i] = TA::frag(cur, wm * C::WTM + i * 16, kk, lane);
#pragma unroll
      for (int j = 0; j < C::TN; ++j) b[j] = TB::frag(cur + QA::BYTES, wn * C::WTN + j * 16, kk, lane);
#pragma unroll
      for (int i = 0; i < C::TM; ++i)
#pragma unroll
        for (int j = 0; j < C::TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
    }
  }
  // leave LDS reusable by the caller's epilogue
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// ----------------------------------------------------------------------------------------
// glds mainloop v2 — same pipeline/contract as gemm_mainloop_glds, built to keep the VALU
// out of the MFMA stream (rocprofv3 showed VALU:MFMA = 5-7:1 in v1):
//  * every per-lane address is computed ONCE: glds sources are (scalar tile base) +
//    (32-bit per-lane byte offset), the scalar base advancing by one K-step per tile;
//  * fragment reads use per-lane LDS base offsets; the K-loop is unrolled by STAGES so
//    the stage, K-substep and subtile offsets are compile-time immediates of ds_read.
template <int U, int N, class F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (U < N) {
    f(std::integral_constant<int, U>{});
    static_for<U + 1, N>(f);
  }
}

template <int R, int L, int NT>
struct GldsOperand {
  using Q = GldsTile<R, L, NT>;
  static constexpr int TILE_BYTES = Q::BYTES;
  unsigned src[Q::PER_WAVE];  // per-lane source byte offsets from the tile base
  const char* base;           // scalar: tile (row0, kbeg) base address
  long kstep_bytes;           // scalar: base advance per 64-deep K-step

  __device__ __forceinline__ void init(const bf16_t* p, long ld, int row0, int kbeg, int wid, int lane) {
#pragma unroll
    for (int i = 0; i < Q::PER_WAVE; ++i) {
      const int piece = i * Q::NW + wid;
      long off;
      if constexpr (L == K_CONTIG) {
        const int row = piece * 8 + (lane >> 3);
        const int lc = (lane & 7) ^ ((row >> 1) & 7);
        off = (long)row * ld + lc * 8;
      } else {
        int k, col;
        Q::mn_src(piece * 1024 + lane * 16, k, col);
        off = (long)k * ld + col;
      }
      src[i] = (unsigned)(off * 2);
    }
    if constexpr (L == K_CONTIG) {
      base = reinterpret_cast<const char*>(p + (size_t)row0 * ld + kbeg);
      kstep_bytes = 64 * 2;
    } else {
      base = reinterpret_cast<const char*>(p + (size_t)kbeg * ld + row0);
      kstep_bytes = 64L * ld * 2;
    }
  }

  __device__ __forceinline__ void issue(int tile, char* lds_tile, int wid) const {
    const char* b = base + (long)tile * kstep_bytes;
#pragma unroll
    for (int i = 0; i < Q::PER_WAVE; ++i)
      __builtin_amdgcn_global_load_lds((const void*)(b + src[i]),
                                       (lds_void*)(lds_tile + (i * Q::NW + wid) * 1024), 16, 0, 0);
  }
};

template <int R, int L, int WT>
struct FragReader {
  // K_CONTIG: fb[kk]; MN_CONTIG: fb[i] (one per 16-row subtile of the wave)
  static constexpr int NB = (L == K_CONTIG) ? 2 : WT / 16;
  int fb[NB];

  __device__ __forceinline__ void init(int rw, int lane) {
    const int l15 = lane & 15, g = lane >> 4;
    if constexpr (L == K_CONTIG) {
      const int s = (l15 >> 1) & 7;  // rw is a multiple of 16: the swizzle only sees l15
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) fb[kk] = (rw + l15) * 128 + (((kk * 4 + g) ^ s) << 4);
    } else {
      const int q = l15 >> 2, p = lane & 3;
      // hk(k) for k = 32kk + 8g + 4h + q does not depend on kk or h
      const int hk = (q | ((g & 1) << 2)) & MnSwz<R>::hmask();
#pragma unroll
      for (int i = 0; i < NB; ++i)
        fb[i] = (8 * g + q) * (R * 2) + (MnSwz<R>::pos((rw >> 4) + i, hk) << 5) + p * 8;
    }
  }

  // fragment of subtile i, k-substep KK, from the tile at byte offset TOFF of smem
  template <int KK, int TOFF>
  __device__ __forceinline__ bf16x8 frag(const char* smem, int i) const {
    if constexpr (L == K_CONTIG) {
      return *reinterpret_cast<const bf16x8*>(smem + fb[KK] + TOFF + i * 16 * 128);
    } else {
      bf16x8 out;
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const char* a = smem + fb[i] + TOFF + (KK * 32 + 4 * h) * (R * 2);
        bf16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_bf16x4*)a);
        out[4 * h + 0] = v[0];
        out[4 * h + 1] = v[1];
        out[4 * h + 2] = v[2];
        out[4 * h + 3] = v[3];
      }
      return out;
    }
  }
};

// PRIO (A/B, cdna_hip_programming.md §5.5 T5): 1 = s_setprio(1) around each MFMA cluster;
// 2 = the static form, waves 4-7 at priority 1 for the whole loop
template <class C, int STAGES, int PRIO = 0>
__device__ __forceinline__ void gemm_mainloop_glds2(const bf16_t* __restrict__ A, long lda,
                                                    const bf16_t* __restrict__ B, long ldb, int kbeg,
                                                    int nk, int m0, int n0, char* smem,
                                                    f32x4 (&acc)[C::TM][C::TN]) {
  static_assert(STAGES >= 2 && STAGES <= 6, "2..6 stages");
  using OA = GldsOperand<C::BM, C::LA_, C::NT>;
  using OB = GldsOperand<C::BN, C::LB_, C::NT>;
  constexpr int STAGE = OA::TILE_BYTES + OB::TILE_BYTES;
  constexpr int LPT = OA::Q::PER_WAVE + OB::Q::PER_WAVE;
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wid / C::WN, wn = wid % C::WN;
#pragma unroll
  for (int i = 0; i < C::TM; ++i)
#pragma unroll
    for (int j = 0; j < C::TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  if (nk <= 0) return;
  OA oa;
  OB ob;
  oa.init(A, lda, m0, kbeg, wid, lane);
  ob.init(B, ldb, n0, kbeg, wid, lane);
  FragReader<C::BM, C::LA_, C::WTM> fa;
  FragReader<C::BN, C::LB_, C::WTN> fbr;
  fa.init(wm * C::WTM, lane);
  fbr.init(wn * C::WTN, lane);

#pragma unroll
  for (int s = 0; s < STAGES - 1; ++s) {
    if (s < nk) {
      oa.issue(s, smem + s * STAGE, wid);
      ob.issue(s, smem + s * STAGE + OA::TILE_BYTES, wid);
    }
  }

  auto body = [&](int tt, auto uc) {
    constexpr int u = decltype(uc)::value;  // == tt % STAGES
    const int ahead = min(nk - 1, tt + STAGES - 2) - tt;
    if constexpr (STAGES >= 5) {
      if (ahead >= STAGES - 2) wait_vmcnt<(STAGES - 2) * LPT>();
      else if (ahead == 3) wait_vmcnt<3 * LPT>();
      else if (ahead == 2) wait_vmcnt<2 * LPT>();
      else if (ahead == 1) wait_vmcnt<LPT>();
      else wait_vmcnt<0>();
    } else if constexpr (STAGES >= 4) {
      if (ahead >= 2) wait_vmcnt<2 * LPT>();
      else if (ahead == 1) wait_vmcnt<LPT>();
      else wait_vmcnt<0>();
    } else if constexpr (STAGES == 3) {
      if (ahead >= 1) wait_vmcnt<LPT>();
      else wait_vmcnt<0>();
    } else {
      wait_vmcnt<0>();
    }
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    const int tn = tt + STAGES - 1;
    if (tn < nk) {
      constexpr int sn = (u + STAGES - 1) % STAGES;
      oa.issue(tn, smem + sn * STAGE, wid);
      ob.issue(tn, smem + sn * STAGE + OA::TILE_BYTES, wid);
    }
    static_for<0, 2>([&](auto kc) {
      constexpr int KK = decltype(kc)::value;
      bf16x8 a[C::TM], b[C::TN];
#pragma unroll
      for (int i = 0; i < C::TM; ++i) a[i] = fa.template frag<KK, u * STAGE>(smem, i);
#pragma unroll
      for (int j = 0; j < C::TN; ++j) b[j] = fbr.template frag<KK, u * STAGE + OA::TILE_BYTES>(smem, j);
      if constexpr (PRIO == 1) __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < C::TM; ++i)
#pragma unroll
        for (int j = 0; j < C::TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
      if constexpr (PRIO == 1) __builtin_amdgcn_s_setprio(0);
    });
  };

  if constexpr (PRIO == 2) {
    if (__builtin_amdgcn_readfirstlane(threadIdx.x) >= 256) __builtin_amdgcn_s_setprio(1);
  }
  int t = 0;
  for (; t + STAGES <= nk; t += STAGES)
    static_for<0, STAGES>([&](auto uc) { body(t + decltype(uc)::value, uc); });
  static_for<0, STAGES>([&](auto uc) {
    if (t + decltype(uc)::value < nk) body(t + decltype(uc)::value, uc);
  });
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// ----------------------------------------------------------------------------------------
// Half-step ring for the MN x MN weight-gradient GEMM: 32-deep K steps through an NSLOT-deep
// LDS ring. With 64-deep steps the 256x192 tile fits only 2 stages in 160 KiB, so each step's
// LDS-DMA had exactly one step of MFMA work (~1.5k cycles per SIMD) to land and the
// vmcnt(0) before every barrier exposed the rest of its latency (PMC: 28 % wave-wait, 54 % MFMA
// busy). 32-deep slots of the same tile (28 KiB) fit 5 deep: a piece is issued NSLOT - 1 half
// steps ahead of its use. Pieces that do not split evenly over the waves (the 192-wide image
// is 12 pieces per half step) go to the low waves, and each wave counts its own in vmcnt.
template <int R, int L, int NT, int BKD, bool GL = false>
struct GldsOpH {
  static_assert(L == MN_CONTIG, "half-step ring: MN-contiguous operands only");
  static constexpr int BYTES = R * BKD * 2;
  static constexpr int PIECES = BYTES / 1024;
  static constexpr int NW = NT / 64;
  static constexpr int MAXPW = (PIECES + NW - 1) / NW;  // pieces of the low waves
  static constexpr int REM = PIECES % NW;               // waves < REM issue MAXPW, the rest MAXPW - 1
  static_assert(BYTES % 1024 == 0 && PIECES >= NW, "tile image must be whole 1-KiB pieces, >= 1 per wave");
  using SW = MnSwz<R>;
  // buffer-resource form (buffer_load ... lds): a 32-bit per-lane voffset and a scalar step
  // offset, no 64-bit per-lane addresses (global_load_lds with 64-bit VGPR addresses spilled
  // the 288-wide tile's kernel). The workgroup's whole K range is < 2 GiB from its origin.
  unsigned src[MAXPW];
  __amdgpu_buffer_rsrc_t rsrc;
  const char* base;  // GL: the same origin as a plain pointer
  int kstep_bytes;

  __device__ __forceinline__ void init(const bf16_t* p, long ld, int row0, int kbeg, int wid, int lane) {
#pragma unroll
    for (int i = 0; i < MAXPW; ++i) {
      const int o = (i * NW + wid) * 1024 + lane * 16;
      const int k = o / (R * 2), b = o % (R * 2);
      const int col = (SW::data(b >> 5, SW::hk(k)) << 4) + (((b >> 4) & 1) << 3);
      src[i] = (unsigned)(((long)k * ld + col) * 2);
    }
    rsrc = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16_t*>(p + (size_t)kbeg * ld + row0), 0, 0x7FFFFFFF,
                                             0x00020000);
    base = reinterpret_cast<const char*>(p + (size_t)kbeg * ld + row0);
    kstep_bytes = (int)(BKD * ld * 2);
  }
  // piece i of this wave alone (DG 3: pieces placed between the MFMAs)
  __device__ __forceinline__ void issue1(int i, int step, char* lds_tile, int wid) const {
    if (i + 1 < MAXPW || REM == 0 || wid < REM)  // wave-uniform
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, (lds_void*)(lds_tile + (i * NW + wid) * 1024), 16, (int)src[i],
                                               step * kstep_bytes, 0, 0);
  }
  __device__ __forceinline__ void issue(int step, char* lds_tile, int wid) const {
    const int so = step * kstep_bytes;
#pragma unroll
    for (int i = 0; i < MAXPW; ++i) {
      if (i + 1 < MAXPW || REM == 0 || wid < REM) {  // wave-uniform
        if constexpr (GL) {
          // global_load_lds (round 6, tile 8 A/B) in its saddr form: the uniform base + step in
          // SGPRs, the 32-bit lane offset in a VGPR (the builtin made 64-bit per-lane addresses
          // and spilled). Tried because the probe charged the MUBUF form ~2x its issue time;
          // the dW GEMM measured 5 % SLOWER with it (profiles/r6/diag/glds.txt). Inline asm: M0
          // through its constraint, one wait state after the M0 write; the counted vmcnt waits
          // of the ring cover it like the builtin.
          const char* b = base + so;
          const unsigned la = (unsigned)(uintptr_t)((lds_void*)(lds_tile + (i * NW + wid) * 1024));
          asm volatile("s_nop 0\n\tglobal_load_lds_dwordx4 %0, %1" ::"v"(src[i]), "s"(b),
                       "{m0}"(__builtin_amdgcn_readfirstlane(la))
                       : "memory");
        } else
          __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, (lds_void*)(lds_tile + (i * NW + wid) * 1024), 16, (int)src[i],
                                                   so, 0, 0);
      }
    }
  }
};

// BKD = 64 with NSLOT = 2: the plain 2-stage ring of gemm_mainloop_glds2, for tiles whose
// pieces do not split evenly over the waves (the 288-wide image: 36 pieces per 64-deep step)
// DG (diagnostics, tools/dw_tiles.py tiles 9 / 10; results wrong): 1 = the ring's DMA for every
// other half step only, 2 = no fragment reads and no MFMAs (the DMA + barrier floor).
// DG 3 (tile 11, results exact): the half step's DMA pieces issued AFTER its fragment reads, one
// between every few MFMAs — a piece costs its wave ~60 issue cycles among bare MFMAs but 100-185
// in a phase of fragment reads (MI355X_MICROARCH.md, LDS-DMA piece issue cost)
template <class C, int NSLOT, int PRIO = 0, int BKD = 32, bool GL = false, int DG = 0>
__device__ __forceinline__ void gemm_mainloop_glds_h(const bf16_t* __restrict__ A, long lda,
                                                     const bf16_t* __restrict__ B, long ldb, int kbeg,
                                                     int nh, int m0, int n0, char* smem,
                                                     f32x4 (&acc)[C::TM][C::TN]) {
  static_assert(BKD == 32 || BKD == 64, "32- or 64-deep steps");
  static_assert(NSLOT >= 2 && NSLOT <= 6, "2..6 slots");
  using OA = GldsOpH<C::BM, C::LA_, C::NT, BKD, GL>;
  using OB = GldsOpH<C::BN, C::LB_, C::NT, BKD, GL>;
  static_assert(OA::REM == 0 || OB::REM == 0, "at most one operand with an uneven piece split");
  constexpr int STAGE = OA::BYTES + OB::BYTES;
  constexpr int LHI = OA::MAXPW + OB::MAXPW;                       // pieces per half step, low waves
  constexpr int LLO = LHI - ((OA::REM | OB::REM) != 0 ? 1 : 0);    // the other waves
  constexpr int NHI = OA::REM ? OA::REM : (OB::REM ? OB::REM : C::NT / 64);
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wid / C::WN, wn = wid % C::WN;
  const bool hi = wid < NHI;
#pragma unroll
  for (int i = 0; i < C::TM; ++i)
#pragma unroll
    for (int j = 0; j < C::TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  if (nh <= 0) return;
  // PRIO 3: static s_setprio 1 for the second-dispatched half of the waves (no per-cluster flips)
  if constexpr (PRIO == 3) {
    if (wid >= C::NT / 128) __builtin_amdgcn_s_setprio(1);
  }
  OA oa;
  OB ob;
  oa.init(A, lda, m0, kbeg, wid, lane);
  ob.init(B, ldb, n0, kbeg, wid, lane);
  FragReader<C::BM, C::LA_, C::WTM> fa;
  FragReader<C::BN, C::LB_, C::WTN> fbr;
  fa.init(wm * C::WTM, lane);
  fbr.init(wn * C::WTN, lane);

#pragma unroll
  for (int s = 0; s < NSLOT - 1; ++s) {
    if (s < nh) {
      oa.issue(s, smem + s * STAGE, wid);
      ob.issue(s, smem + s * STAGE + OA::BYTES, wid);
    }
  }
  auto body = [&](int tt, auto uc) {
    constexpr int u = decltype(uc)::value;  // == tt % NSLOT
    // half steps issued after tt that may stay in flight
    const int ahead = min(nh - 1, tt + NSLOT - 2) - tt;
    // keep the previous step's MFMAs above this point: sunk below the barrier they would hold
    // two steps' fragments at once (the 288-wide tile then spilled)
    __builtin_amdgcn_sched_barrier(0);
    static_for<0, NSLOT - 1>([&](auto ac) {
      constexpr int a = NSLOT - 2 - decltype(ac)::value;  // steady state (NSLOT - 2) tested first
      if (ahead == a) {
        if (hi) wait_vmcnt<a * LHI>();
        else wait_vmcnt<a * LLO>();
      }
    });
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    const int tn = tt + NSLOT - 1;
    if (DG != 3 && tn < nh && (DG != 1 || (tn & 1) == 0)) {
      constexpr int sn = (u + NSLOT - 1) % NSLOT;
      oa.issue(tn, smem + sn * STAGE, wid);
      ob.issue(tn, smem + sn * STAGE + OA::BYTES, wid);
    }
    if constexpr (DG == 2) return;
    // slot origin as an opaque per-step value: with u * STAGE folded into every fragment
    // address (beyond the 16-bit ds offset field) the compiler hoisted one address register
    // per (slot, fragment) out of the loop, and the 288-wide tile spilled them
    int so = u * STAGE;
    asm volatile("" : "+v"(so));
    const char* sl = smem + so;
    if constexpr (DG == 3) {
      static_assert(BKD == 32, "DG 3: one fragment set per half step");
      constexpr int NP = OA::MAXPW + OB::MAXPW;             // this wave's pieces (the last maybe none)
      constexpr int NM = C::TM * C::TN, GAP = NM / (NP + 1);  // MFMAs between pieces
      constexpr int sn = (u + NSLOT - 1) % NSLOT;
      const bool more = tn < nh;
      bf16x8 a[C::TM], b[C::TN];
#pragma unroll
      for (int i = 0; i < C::TM; ++i) a[i] = fa.template frag<0, 0>(sl, i);
#pragma unroll
      for (int j = 0; j < C::TN; ++j) b[j] = fbr.template frag<0, OA::BYTES>(sl, j);
      if constexpr (PRIO == 1) __builtin_amdgcn_s_setprio(1);
      static_for<0, NM>([&](auto mc) {
        constexpr int m = decltype(mc)::value, i = m / C::TN, j = m % C::TN;
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
        if constexpr ((m + 1) % GAP == 0 && (m + 1) / GAP <= NP) {
          constexpr int p = (m + 1) / GAP - 1;
          __builtin_amdgcn_sched_barrier(0);
          if (more) {
            if constexpr (p < OA::MAXPW) oa.issue1(p, tn, smem + sn * STAGE, wid);
            else ob.issue1(p - OA::MAXPW, tn, smem + sn * STAGE + OA::BYTES, wid);
          }
          __builtin_amdgcn_sched_barrier(0);
        }
      });
      if constexpr (PRIO == 1) __builtin_amdgcn_s_setprio(0);
      return;
    }
    static_for<0, BKD / 32>([&](auto kc) {
      constexpr int KK = decltype(kc)::value;
      bf16x8 a[C::TM], b[C::TN];
#pragma unroll
      for (int i = 0; i < C::TM; ++i) a[i] = fa.template frag<KK, 0>(sl, i);
#pragma unroll
      for (int j = 0; j < C::TN; ++j) b[j] = fbr.template frag<KK, OA::BYTES>(sl, j);
      if constexpr (PRIO == 1) __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < C::TM; ++i)
#pragma unroll
        for (int j = 0; j < C::TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
      if constexpr (PRIO == 1) __builtin_amdgcn_s_setprio(0);
    });
  };
  int t = 0;
  for (; t + NSLOT <= nh; t += NSLOT)
    static_for<0, NSLOT>([&](auto uc) { body(t + decltype(uc)::value, uc); });
  static_for<0, NSLOT>([&](auto uc) {
    if (t + decltype(uc)::value < nh) body(t + decltype(uc)::value, uc);
  });
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// ----------------------------------------------------------------------------------------
// Staggered wave groups (cdna_hip_programming.md §5 8-phase template, "if (wr == 1)
// s_barrier"): same tile, 2-slot 64-deep ring and operand images as gemm_mainloop_glds2, but
// every 32-deep phase is {fragment reads ; barrier ; MFMAs ; barrier} and waves 4-7 (the
// second wave on each SIMD: waves go to SIMDs cyclically) run one barrier behind waves 0-3. In
// every barrier interval one wave of a SIMD issues MFMAs while the other issues and waits for
// its fragment reads; with one barrier per step both waves read, then both multiply (the
// ring's DMA wait was not the limiter: the 5-slot half-step ring measured the same, 1.166 ms).
// Barriers b = 0, 1, .. (after the prologue's): group A reads step t's phase 0 in interval 4t,
// group B in 4t + 1, and so on. DMA(t + 1) into the slot of step t - 1 goes out after bar(4t),
// when every read of that slot has retired (each wave's lgkmcnt wait precedes its MFMAs), and
// every wave waits for its own pieces before bar(4t + 3), which precedes group A's first read
// of step t + 1 (group A: its 4th barrier of step t, group B: its 3rd).
template <class C, int PRIO = 1>
__device__ __forceinline__ void gemm_mainloop_stag(const bf16_t* __restrict__ A, long lda,
                                                   const bf16_t* __restrict__ B, long ldb, int kbeg,
                                                   int nk, int m0, int n0, char* smem,
                                                   f32x4 (&acc)[C::TM][C::TN]) {
  static_assert(C::NT == 512, "two wave groups of 4 (one wave per SIMD each)");
  using OA = GldsOperand<C::BM, C::LA_, C::NT>;
  using OB = GldsOperand<C::BN, C::LB_, C::NT>;
  constexpr int STAGE = OA::TILE_BYTES + OB::TILE_BYTES;
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wid / C::WN, wn = wid % C::WN;
  const bool grp_b = wid >= 4;
#pragma unroll
  for (int i = 0; i < C::TM; ++i)
#pragma unroll
    for (int j = 0; j < C::TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  if (nk <= 0) return;
  OA oa;
  OB ob;
  oa.init(A, lda, m0, kbeg, wid, lane);
  ob.init(B, ldb, n0, kbeg, wid, lane);
  FragReader<C::BM, C::LA_, C::WTM> fa;
  FragReader<C::BN, C::LB_, C::WTN> fbr;
  fa.init(wm * C::WTM, lane);
  fbr.init(wn * C::WTN, lane);
  auto bar = [] {
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
  };

  oa.issue(0, smem, wid);
  ob.issue(0, smem + OA::TILE_BYTES, wid);
  wait_vmcnt<0>();
  bar();
  if (grp_b) bar();  // group B runs one barrier behind

  auto body = [&](int tt, auto uc) {
    constexpr int u = decltype(uc)::value;  // == tt & 1
    const bool more = tt + 1 < nk;
    if (grp_b && more) {  // B: right after bar(4t), its last barrier of step t - 1
      oa.issue(tt + 1, smem + (u ^ 1) * STAGE, wid);
      ob.issue(tt + 1, smem + (u ^ 1) * STAGE + OA::TILE_BYTES, wid);
    }
    static_for<0, 2>([&](auto kc) {
      constexpr int KK = decltype(kc)::value;
      bf16x8 a[C::TM], b[C::TN];
#pragma unroll
      for (int i = 0; i < C::TM; ++i) a[i] = fa.template frag<KK, u * STAGE>(smem, i);
#pragma unroll
      for (int j = 0; j < C::TN; ++j) b[j] = fbr.template frag<KK, u * STAGE + OA::TILE_BYTES>(smem, j);
      if constexpr (KK == 1) {
        if (grp_b) wait_vmcnt<0>();  // B: before its 3rd barrier of the step = bar(4t + 3)
      }
      bar();
      if constexpr (KK == 0) {
        if (!grp_b && more) {  // A: right after bar(4t)
          oa.issue(tt + 1, smem + (u ^ 1) * STAGE, wid);
          ob.issue(tt + 1, smem + (u ^ 1) * STAGE + OA::TILE_BYTES, wid);
        }
      }
      if constexpr (PRIO == 1) __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < C::TM; ++i)
#pragma unroll
        for (int j = 0; j < C::TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
      if constexpr (PRIO == 1) __builtin_amdgcn_s_setprio(0);
      if constexpr (KK == 1) {
        if (!grp_b) wait_vmcnt<0>();  // A: before its 4th barrier of the step = bar(4t + 3)
      }
      bar();
    });
  };
  int t = 0;
  for (; t + 2 <= nk; t += 2) {
    body(t, std::integral_constant<int, 0>{});
    body(t + 1, std::integral_constant<int, 1>{});
  }
  if (t < nk) body(t, std::integral_constant<int, 0>{});
  if (!grp_b) bar();  // the barrier counts of the two groups meet again
}

// Output coordinates of accumulator element acc[i][j][r] (16x16 C/D map: col = lane&15,
// row = 4*(lane>>4) + r).
template <class C>
struct AccCoord {
  int mb, nb;  // wave tile origin (absolute)
  __device__ __forceinline__ AccCoord(int m0, int n0) {
    const int wid = threadIdx.x >> 6;
    mb = m0 + (wid / C::WN) * C::WTM;
    nb = n0 + (wid % C::WN) * C::WTN;
  }
  __device__ __forceinline__ int row(int i, int r) const {
    return mb + i * 16 + 4 * ((threadIdx.x & 63) >> 4) + r;
  }
  __device__ __forceinline__ int col(int j) const { return nb + j * 16 + (threadIdx.x & 15); }
};

}  // namespace wf
