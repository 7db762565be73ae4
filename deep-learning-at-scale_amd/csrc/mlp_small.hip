// wellflow — K consecutive small-batch MLP training steps (forward, backward AND Adam) in ONE
// persistent launch: the job-default batch (256 rows, reference mlp.py / config.py) of the
// F -> 256 -> 256 -> 1 network. SURVEY.md §2.4 K9-K11 + K8; round-5 VERDICT item 3(b).
//
// At 256 rows a step is ~30 us of launch-bound kernels (one-launch step, dW2, reduce, Adam:
// profiles/r6/job_default/mlp_b256_kernel_stats.csv) for ~100 MFLOP of work. Here 16 worker
// workgroups (one per CU, 4 waves) run K steps back to back with the weights and the Adam
// state resident in their registers. Worker w owns units U = O = [16w, 16w + 16) of both hidden
// layers: W1 rows U, b1[U], W2 rows O, b2[O], w3[O] (worker 0 also b3). Per step:
//   A  poll the W1 / b1 granules of this step | stage the batch (prefetched a step earlier) |
//      H1 = relu(X W1^T + b1), ALL 256 units, in LDS (4 KiB of W1 per step from L2: cheaper
//      than exchanging H1) | Z2[:, O] = H1 W2[O]^T + b2 (W2[O] fragments in VGPRs) | H2 = relu |
//      head partial p_w[r] = H2[r, O] w3[O] -> granules
//   C  poll the 16 partial granules of each row: pred = sum_w p_w + b3, dy, loss | dZ2[:, O] =
//      dy w3[O] [H2 > 0] -> publish | dW2[O, :] = dZ2[:, O]^T H1 (complete: the batch is in
//      the workgroup), db2, dw3, db3                                         == barrier ==
//   E  dH1[:, U] = dZ2 W2[:, U] (all of dZ2 + this step's W2^T block column, straight from L2 as
//      MFMA fragments) | dZ1 = dH1 [H1 > 0] | dW1[U, :] = dZ1^T X, db1
//   F  Adam on the owned parameters (registers) | publish W1[U] (bf16 pairs), b1[U], b3 as the
//      next step's granules and the W2^T block (the other parity: readers of this step's block
//      may still be in E)
// Small hand-offs are 8-B {value, tag} granules written by ONE sc1 store and polled by the
// consumer itself (MI355X_MICROARCH.md R2: no flag, no barrier; the tag names the launch and
// step). The 128-KiB dZ2 exchange is plain data behind one flag per worker (sc1 16-B stores,
// every storing wave's vmcnt(0), a workgroup barrier, ONE sc1 flag granule carrying the step's
// tag; the consumer polls the 16 flags, then sc1 loads of every handed-off byte). Buffer reuse
// needs no more: a worker reaches step k + 1's writes only after every worker's step-k granules
// of W1 arrived, i.e. after every worker finished its step-k reads. Tags only grow (launch
// ordinal x 4096 + step + 1), so no launch needs a memset.
// A spin bound turns a lost hand-off into a sticky error word (results garbage, the host
// raises) instead of a hang. Every reduction has a fixed order (no float atomics), so K fused
// steps equal K single-step launches bit for bit.
#include <type_traits>

#include "common.h"
#include "gemm_core.h"
#include "kernels.h"
#include "mlp_tiles.h"

namespace wf {

namespace {

constexpr int SB_G = 16;  // worker workgroups

// scratch (floats): granules {value, tag} of [part 16 x 256][b1 256][b3 (+ pad)][W1 256 x 16 words
// (bf16 pairs)], then the barrier-guarded blocks [dZ2 bf16 16 x 256 x 16][W2^T bf16 2 x 16 x 256 x 16]
constexpr int SBO_PART = 0, SBO_B1 = 8192, SBO_B3 = 8704, SBO_FLAG = 8736, SBO_W1 = 8768, SBO_DZ2 = 16960, SBO_W2T = 49728;
static_assert(SBO_W2T + 65536 == kMlpSmallScratch, "scratch layout");

// LDS (bytes): X [256][64 B] | H1 [256][512 B] (tile_off) | dZ2 / dZ1 own [256][16] bf16 |
// dy | y | b2, w3 own | small gradients | flag. The W2 / W2^T / W1 staging of phase F uses the
// H1 region (dead after E).
constexpr int SL_X = 0, SL_H1 = 16384, SL_Z = 147456, SL_DY = 155648, SL_Y = 156672, SL_C = 157696;
constexpr int SL_BYTES = SL_C + 1024;

typedef unsigned sb_u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) unsigned sb_g32;

__device__ __forceinline__ void sb_adam(float& p, float g, float& m, float& v, float lr, float b1, float b2, float eps,
                                        float wd, float rbc1, float rbc2) {
  // elementwise.hip adam_one (FlatAdam) with the hardware square root / reciprocal (1 ulp)
  // instead of the IEEE-exact sequences: the update's VALU count was ~1/3 of a step's Adam +
  // publish time. rbc1 / rbc2: 1 / (1 - beta^t)
  m = b1 * m + (1.f - b1) * g;
  v = b2 * v + (1.f - b2) * g * g;
  const float mh = m * rbc1, vh = v * rbc2;
  p -= lr * (mh * __builtin_amdgcn_rcpf(__builtin_amdgcn_sqrtf(vh) + eps) + wd * p);
}

__device__ __forceinline__ float sb_dloss(float d, float clip) {
  if (clip <= 0.f) return d;
  return fabsf(d) <= clip ? (d > 0.f ? 1.f : (d < 0.f ? -1.f : 0.f)) : 0.f;
}
__device__ __forceinline__ float sb_loss(float d, float clip) { return clip <= 0.f ? d * d : fminf(fabsf(d), clip); }

__device__ __forceinline__ unsigned sb_relu_pk(unsigned p) {
  typedef short s16x2 __attribute__((ext_vector_type(2)));
  return __builtin_bit_cast(unsigned, __builtin_elementwise_max(__builtin_bit_cast(s16x2, p), (s16x2){0, 0}));
}
// "d where h != 0" per 16-bit half (h a ReLU output >= 0), as mlp_step.hip mask_pk
__device__ __forceinline__ unsigned sb_mask_pk(unsigned d, unsigned h) {
  unsigned o;
  asm("v_pk_min_u16 %0, %1, %3\n\tv_pk_mul_lo_u16 %0, %2, %0" : "=&v"(o) : "v"(h), "v"(d), "s"(0x00010001u));
  return o;
}
__device__ __forceinline__ float sb_lo(unsigned q) { return __uint_as_float(q << 16); }
__device__ __forceinline__ float sb_hi(unsigned q) { return __uint_as_float(q & 0xFFFF0000u); }

template <int NFT>  // 16-feature tiles of W1 (Fp <= 16: 1, Fp <= 32: 2)
__global__ __launch_bounds__(256, 1) void mlp_small_kernel(const MlpSmallArgs a) {
  __shared__ __attribute__((aligned(16))) char lds[SL_BYTES];
  char* const Xs = lds + SL_X;
  char* const H1s = lds + SL_H1;
  char* const ZS = lds + SL_Z;
  float* const dys = reinterpret_cast<float*>(lds + SL_DY);
  float* const ys = reinterpret_cast<float*>(lds + SL_Y);
  float* const cb2 = reinterpret_cast<float*>(lds + SL_C);  // b2[O]
  float* const cw3 = cb2 + 16;                              // w3[O]
  float* const sg = cb2 + 32;                               // small gradients: db1 | db2 | dw3 | db3
  float* const sgw = cb2 + 96;                              // dw3 partials of the 4 waves [4][16]
  float* const lred = cb2 + 160;                            // block_sum scratch
  unsigned* const sflag = reinterpret_cast<unsigned*>(cb2 + 168);
  char* const W1st = H1s + 16384;   // [16 U][32] bf16

  const int tid = threadIdx.x, lane = tid & 63, l15 = lane & 15, g = lane >> 4;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int tq = l15 >> 2, tp = lane & 3;
  const int wk = blockIdx.x;
  const int B = a.B, Fp = a.Fp, K = a.K, R16 = B >> 4, KK = B >> 5;
  float* const scr = a.scr;
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)scr, 0, 0x7FFFFFFF, 0x00020000);
  auto ld16 = [&](int fo) {  // 16-B sc1 load of scratch float offset fo
    return __builtin_bit_cast(sb_u32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, fo * 4, 0, 16));
  };
  auto st16 = [&](sb_u32x4 v, int fo) { __builtin_amdgcn_raw_buffer_store_b128(v, rs, fo * 4, 0, 16); };
  auto ld4 = [&](int fo) { return __hip_atomic_load((sb_g32*)(scr + fo), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); };
  typedef unsigned sb_u32x2 __attribute__((ext_vector_type(2)));
  // an 8-B {value, tag} granule: one sc1 store, read whole by one 8- or 16-B sc1 load (untorn:
  // MI355X_MICROARCH.md R2), so a consumer polls the data itself — no flag, no barrier
  auto st8 = [&](unsigned val, unsigned tag, int fo) {
    __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(decltype(__builtin_amdgcn_raw_buffer_load_b64(rs, 0, 0, 0)),
                                                             (sb_u32x2{val, tag})), rs, fo * 4, 0, 16);
  };
  auto ld8 = [&](int fo) {
    return __builtin_bit_cast(sb_u32x2, __builtin_amdgcn_raw_buffer_load_b64(rs, fo * 4, 0, 16));
  };

  // ---- hand-off counter (sync[0]; [1] exits, [2] sticky error, [3] launches)
  sb_g32* const cnt = (sb_g32*)a.sync;
  unsigned nbar = 0;
  if (tid == 0) sflag[0] = 0u;
  (void)nbar;

  // granule poll bookkeeping: true = keep polling (not all tags seen, no failure, bound not hit)
  unsigned gspins = 0;
  auto poll_again = [&](bool ok) {
    if (__builtin_amdgcn_ballot_w64(!ok) == 0ull) return false;  // the whole wave saw its tags
    if (sflag[0] != 0u) return false;                               // failed earlier: run on
    if ((++gspins & 63u) == 0u &&
        __hip_atomic_load((sb_g32*)(a.sync + 2), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u) {
      if (lane == 0) sflag[0] = 1u;
      return false;
    }
    if (gspins > a.spin_limit) {
      __hip_atomic_store((sb_g32*)(a.sync + 2), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (lane == 0) sflag[0] = 1u;
      return false;
    }
    __builtin_amdgcn_s_sleep(1);
    return true;
  };
  // granule tags: launch ordinal (sync[3], advanced by the last worker out) x 4096 + step + 1,
  // never 0 (the zeroed scratch) and never a stale step of this or an earlier launch
  const unsigned lc = __hip_atomic_load((sb_g32*)(a.sync + 3), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  auto tagv = [&](int j) { return (lc << 12) + (unsigned)j + 1u; };
  // dZ2 hand-off: every storing wave's vmcnt(0), a workgroup barrier, then ONE sc1 flag granule
  // per worker {tag, tag}; the consumer's wave 0 polls the 16 flags (a flag only advances: a
  // later step's tag also counts), then sc1 loads of the blocks. (A counter barrier — one
  // agent-scope atomic add per worker, polled — cost the same hand-off an RMW round trip.)
  auto arrive = [&](unsigned tg) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave's sc1 stores landed
    __syncthreads();
    if (tid == 0) st8(tg, tg, SBO_FLAG + 2 * wk);
  };
  auto wait = [&](unsigned tg) {
    if (wid == 0) {
      bool more = true;
      while (more) {
        bool ok = true;
        if (lane < SB_G) ok = (int)(ld8(SBO_FLAG + 2 * lane)[0] - tg) >= 0;
        more = poll_again(ok);
      }
    }
    __syncthreads();
  };
  int kcur = 0;
  auto stamp = [&](int ph) {  // diagnostics: phase boundaries of the first 64 steps (tools/small_timeline.py)
    if (a.stamps != nullptr && tid == 0 && kcur < 64)
      a.stamps[((size_t)wk * 64 + kcur) * 16 + ph] = __builtin_amdgcn_s_memrealtime();
  };

  // ---- owned master parameters and Adam state, in registers for the whole launch
  // W2: lane (l15, g) of wave w holds W2[16wk + 4g + i][16 (4w + j) + l15], i, j < 4 (the dW2
  // accumulator layout of phase C)
  float p2[4][4], m2[4][4], v2[4][4];
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const long e = a.oW2 + (long)(16 * wk + 4 * g + i) * 256 + 16 * (4 * wid + j) + l15;
      p2[j][i] = a.p[e];
      m2[j][i] = a.m[e];
      v2[j][i] = a.v[e];
    }
  // W1: waves w < NFT, lane (l15, g): W1[16wk + 4g + i][16w + l15] (the dW1 accumulator layout)
  float p1[4] = {0.f, 0.f, 0.f, 0.f}, m1[4] = {0.f, 0.f, 0.f, 0.f}, v1[4] = {0.f, 0.f, 0.f, 0.f};
  const int f1 = 16 * wid + l15;
  const bool own1 = wid < NFT && f1 < Fp;
  if (own1) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const long e = a.oW1 + (long)(16 * wk + 4 * g + i) * Fp + f1;
      p1[i] = a.p[e];
      m1[i] = a.m[e];
      v1[i] = a.v[e];
    }
  }
  // small parameters on wave 3: lanes 0-15 b1[U], 16-31 b2[O], 32-47 w3[O], 48 b3 (worker 0)
  long es = -1;
  if (wid == 3) {
    if (lane < 16) es = a.ob1 + 16 * wk + lane;
    else if (lane < 32) es = a.ob2 + 16 * wk + lane - 16;
    else if (lane < 48) es = a.ow3 + 16 * wk + lane - 32;
    else if (lane == 48 && wk == 0) es = a.ob3;
  }
  float ps = 0.f, ms = 0.f, vs = 0.f;
  if (es >= 0) {
    ps = a.p[es];
    ms = a.m[es];
    vs = a.v[es];
  }
  const float step0 = a.step[0];

  // ---- publish the owned bf16 images (start, and phase F after each update) and refresh the
  // W2[O] A fragments of layer 2
  bf16x8 w2f[8];
  // W2 image: [256 in][16 O] bf16 staged in the dZ2 / dZ1 region (ZS; callers have every wave
  // past its ZS reads, and the next ZS writes follow a workgroup barrier), layer 2's A fragments
  // refreshed from it by transposing reads, the W2^T block of parity `par` published (16-B sc1);
  // b2 / w3 (this worker's only) to LDS
  auto publish_w2 = [&](int par) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int in = 16 * (4 * wid + j) + l15;
      *reinterpret_cast<uint2*>(ZS + in * 32 + 8 * g) = make_uint2(pk_bf16(p2[j][0], p2[j][1]), pk_bf16(p2[j][2], p2[j][3]));
    }
    if (wid == 3) {
      if (lane >= 16 && lane < 32) cb2[lane - 16] = ps;
      else if (lane >= 32 && lane < 48) cw3[lane - 32] = ps;
    }
    __syncthreads();
#pragma unroll
    for (int ks = 0; ks < 8; ++ks)
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const bf16x4 t = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_bf16x4*)(ZS + (32 * ks + 8 * g + 4 * h + tq) * 32 + 8 * tp));
#pragma unroll
        for (int e = 0; e < 4; ++e) w2f[ks][4 * h + e] = t[e];
      }
    const int wbase = SBO_W2T + (par * SB_G + wk) * 2048;  // floats
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int piece = tid + 256 * q;  // 16-B pieces of 8 KiB
      st16(*reinterpret_cast<const sb_u32x4*>(ZS + piece * 16), wbase + piece * 4);
    }
  };
  // the next step's W1 rows, b1 and b3 as granules of tag `tag` (W1 staged in the H1 region:
  // callers have every wave past its H1 reads)
  auto publish_w1 = [&](unsigned tag) {
    if (wid < 2) {  // W1 rows, zero past Fp (and the whole second tile when NFT = 1)
      bf16_t* w1s = reinterpret_cast<bf16_t*>(W1st);
#pragma unroll
      for (int i = 0; i < 4; ++i) w1s[(4 * g + i) * 32 + 16 * wid + l15] = own1 ? f2bf(p1[i]) : (bf16_t)0;
    }
    if (wid == 3) {
      if (lane < 16) st8(__float_as_uint(ps), tag, SBO_B1 + 2 * (16 * wk + lane));
      else if (lane == 48 && es >= 0) st8(__float_as_uint(ps), tag, SBO_B3);
    }
    __syncthreads();
    // W1 rows as granules {bf16 pair, tag}: thread = (unit tid / 16, word tid % 16)
    st8(*reinterpret_cast<const unsigned*>(W1st + (tid >> 4) * 64 + (tid & 15) * 4), tag,
        SBO_W1 + 2 * ((16 * wk + (tid >> 4)) * 16 + (tid & 15)));
  };

  // ---- batch prefetch: piece p = tid + 256q of the [B][64 B] X tile (row p / 4, chunk p % 4)
  // dataset row ids are fetched one step before their gathers (fetch_ids(k + 2) after
  // prefetch(k + 1)): a gather right behind its id load waited out a round trip per piece
  sb_u32x4 xv[4];
  float yv = 0.f;
  long rid[5];  // rows of the pieces q < 4 and of the target (row tid) of the next prefetch
  auto fetch_ids = [&](int k) {
#pragma unroll
    for (int q = 0; q < 5; ++q) {
      const int r = q < 4 ? (tid + 256 * q) >> 2 : tid;
      rid[q] = (r < B && k < K) ? (long)data_row(a.rows, k * B + r, a.nrows) : 0;
    }
  };
  auto prefetch = [&]() {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int piece = tid + 256 * q, r = piece >> 2, c = piece & 3;
      xv[q] = sb_u32x4{0u, 0u, 0u, 0u};
      if (r < B && 8 * c + 8 <= Fp) xv[q] = *reinterpret_cast<const sb_u32x4*>(a.X + (size_t)rid[q] * Fp + 8 * c);
    }
    yv = tid < B ? a.Y[rid[4]] : 0.f;
  };
  auto stage_x = [&]() {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int piece = tid + 256 * q, r = piece >> 2, c = piece & 3;
      if (r < B) *reinterpret_cast<sb_u32x4*>(Xs + r * 64 + ((c ^ ((r >> 2) & 3)) << 4)) = xv[q];
    }
    ys[tid] = yv;
  };

  fetch_ids(0);
  prefetch();
  fetch_ids(1);
  publish_w2(0);
  publish_w1(tagv(0));  // the step-0 granules (polled by every worker's phase A)

  const bf16x8 ones = __builtin_bit_cast(bf16x8, (sb_u32x4{0x3F803F80u, 0x3F803F80u, 0x3F803F80u, 0x3F803F80u}));
  for (int k = 0; k < K; ++k) {
    const int par = k & 1;
    kcur = k;
    stamp(0);
    // ---- A: H1 = relu(W1 X^T + b1), wave w computes units 64w .. 64w + 63 for every row tile;
    // the W1 / b1 images (published before barrier 3) requested before the X staging
    bf16x8 w1f[4];
    sb_u32x4 bvu[4];
    // this step's batch (gathered during the previous step) into LDS first: the stores overlap
    // the W1 wait (every wave's reads of Xs / ys ended before the previous step's last barrier)
    stage_x();
    {
      const unsigned tg = tagv(k);
      // light poll first: lanes 0-15 watch the LAST W1 granule of producer `lane` (written after
      // its b1 granules and the rest of its rows, but with no ordering guarantee: the full load
      // below still checks every tag); the full 16-KiB-per-wave poll every iteration cost
      // ~4 us per step in load traffic
      {
        bool more = true;
        while (more) {
          bool ok = true;
          if (lane < SB_G) ok = ld8(SBO_W1 + 2 * ((16 * lane + 15) * 16 + 15))[1] == tg;
          more = poll_again(ok);
        }
      }
      bool more = true;
      while (more) {
        bool ok = true;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int u = 16 * (4 * wid + q);
          sb_u32x4 w = sb_u32x4{0u, 0u, 0u, 0u};
          if (8 * g < Fp) {  // features 8g .. 8g + 7 = granules 4g .. 4g + 3 of the unit's row
            const sb_u32x4 v0 = ld16(SBO_W1 + 2 * ((u + l15) * 16 + 4 * g));
            const sb_u32x4 v1 = ld16(SBO_W1 + 2 * ((u + l15) * 16 + 4 * g) + 4);
            ok = ok && v0[1] == tg && v0[3] == tg && v1[1] == tg && v1[3] == tg;
            w = sb_u32x4{v0[0], v0[2], v1[0], v1[2]};
          }
          w1f[q] = __builtin_bit_cast(bf16x8, w);
          const sb_u32x4 c0 = ld16(SBO_B1 + 2 * (u + 4 * g));
          const sb_u32x4 c1 = ld16(SBO_B1 + 2 * (u + 4 * g) + 4);
          ok = ok && c0[1] == tg && c0[3] == tg && c1[1] == tg && c1[3] == tg;
          bvu[q] = sb_u32x4{c0[0], c0[2], c1[0], c1[2]};
        }
        more = poll_again(ok);
      }
    }
    __syncthreads();
    stamp(1);
    stamp(14);
    {
      f32x4 bv[4];
#pragma unroll
      for (int q = 0; q < 4; ++q)
        bv[q] = f32x4{__uint_as_float(bvu[q][0]), __uint_as_float(bvu[q][1]), __uint_as_float(bvu[q][2]),
                      __uint_as_float(bvu[q][3])};
      // two row tiles per iteration, 8 independent accumulators and the next pair's X fragments
      // read ahead (one accumulator set per tile serialised MFMA -> convert -> store: 2.9 us;
      // four tiles per iteration measured slower, 2.64 vs 2.40 us: the 128-KiB H1 store bounds it)
      auto xfrag = [&](int rt) {
        const int r = 16 * rt + l15;
        return *reinterpret_cast<const bf16x8*>(Xs + r * 64 + ((g ^ ((r >> 2) & 3)) << 4));
      };
      bf16x8 xa = xfrag(0), xb = xfrag(R16 > 1 ? 1 : 0);
      for (int rt = 0; rt < R16; rt += 2) {
        const bf16x8 na = xfrag(rt + 2 < R16 ? rt + 2 : 0), nb = xfrag(rt + 3 < R16 ? rt + 3 : 0);
        f32x4 c[2][4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          c[0][q] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w1f[q], xa, bv[q], 0, 0, 0);
          c[1][q] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w1f[q], xb, bv[q], 0, 0, 0);
        }
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int r = 16 * (rt + h) + l15;
          if (rt + h < R16) {
#pragma unroll
            for (int q = 0; q < 4; ++q)
              *reinterpret_cast<uint2*>(H1s + tile_off(r, 16 * (4 * wid + q) + 4 * g)) =
                  make_uint2(sb_relu_pk(pk_bf16(c[h][q][0], c[h][q][1])), sb_relu_pk(pk_bf16(c[h][q][2], c[h][q][3])));
          }
        }
        xa = na;
        xb = nb;
      }
    }
    __syncthreads();  // H1 complete
    stamp(2);

    // ---- layer 2 on the owned units, H2, head partials (row tiles w, w + 4, ...)
    unsigned h2p[4][2];  // H2 of the wave's row tiles as packed bf16 (units 4g .. 4g + 3)
    {
      const float4 bb = *reinterpret_cast<const float4*>(cb2 + 4 * g);
      const float4 ww = *reinterpret_cast<const float4*>(cw3 + 4 * g);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        h2p[j][0] = h2p[j][1] = 0u;
        const int rt = wid + 4 * j;
        if (rt < R16) {
          const int r = 16 * rt + l15;
          f32x4 acc = f32x4{bb.x, bb.y, bb.z, bb.w};
#pragma unroll
          for (int ks = 0; ks < 8; ++ks) {
            const bf16x8 hb = *reinterpret_cast<const bf16x8*>(H1s + tile_off(r, 32 * ks + 8 * g));
            acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w2f[ks], hb, acc, 0, 0, 0);
          }
          h2p[j][0] = sb_relu_pk(pk_bf16(acc[0], acc[1]));
          h2p[j][1] = sb_relu_pk(pk_bf16(acc[2], acc[3]));
          float hp = (sb_lo(h2p[j][0]) * ww.x + sb_hi(h2p[j][0]) * ww.y) + (sb_lo(h2p[j][1]) * ww.z + sb_hi(h2p[j][1]) * ww.w);
          const unsigned hu = __float_as_uint(hp);
          hp += __uint_as_float(__builtin_amdgcn_permlane32_swap(hu, hu, false, false)[1]);
          const unsigned tu = __float_as_uint(hp);
          hp += __uint_as_float(__builtin_amdgcn_permlane16_swap(tu, tu, false, false)[1]);
          if (g == 0) st8(__float_as_uint(hp), tagv(k), SBO_PART + 2 * (wk * 256 + r));
        }
      }
    }
    stamp(3);
    stamp(4);

    // the next batch's gathers: issued here, where the head-partial poll waits anyway (issued
    // before H1 they cost that critical-path phase ~0.5 us); xv / yv were staged in phase A
    if (k + 1 < K) {
      prefetch();        // step k + 1 (ids fetched a step ago)
      fetch_ids(k + 2);  // consumed by the next prefetch
    }
    // ---- C: prediction, dy, loss (every worker, every row; fixed summation order)
    {
      float lossv = 0.f, dyv = 0.f;
      if (tid < B) {
        // the 16 workers' partial granules of this row and b3, polled until every tag is this step's
        unsigned pv[SB_G], b3u = 0u;
        const unsigned tg = tagv(k);
        bool more = true;
        while (more) {
          bool ok = true;
#pragma unroll
          for (int w = 0; w < SB_G; ++w) {
            const sb_u32x2 v = ld8(SBO_PART + 2 * (w * 256 + tid));
            pv[w] = v[0];
            ok = ok && v[1] == tg;
          }
          const sb_u32x2 v3 = ld8(SBO_B3);
          b3u = v3[0];
          ok = ok && v3[1] == tg;
          more = poll_again(ok);
        }
        float p = 0.f;
#pragma unroll
        for (int w = 0; w < SB_G; ++w) p += __uint_as_float(pv[w]);
        p += __uint_as_float(b3u);
        const float d = p - ys[tid];
        dyv = a.dy_scale * sb_dloss(d, a.clip);
        lossv = sb_loss(d, a.clip);
        dys[tid] = dyv;
      }
      if (wk == 0) {
        const float ls = block_sum<256>(lossv, lred);
        const float s3b = block_sum<256>(dyv, lred);
        if (tid == 0) {
          if (a.loss_acc != nullptr) atomicAdd(a.loss_acc, ls);
          sg[48] = s3b;  // db3
        }
      } else {
        __syncthreads();
      }
    }
    stamp(5);
    // dZ2[:, O] = bf16(dy w3[O]) where H2 > 0 -> ZS [row][16]; dw3 partials
    {
      const float4 ww = *reinterpret_cast<const float4*>(cw3 + 4 * g);
      float s3[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int rt = wid + 4 * j;
        if (rt < R16) {
          const int r = 16 * rt + l15;
          const float dy = dys[r];
          const float h0 = sb_lo(h2p[j][0]), h1 = sb_hi(h2p[j][0]), h2 = sb_lo(h2p[j][1]), h3 = sb_hi(h2p[j][1]);
          s3[0] += h0 * dy;
          s3[1] += h1 * dy;
          s3[2] += h2 * dy;
          s3[3] += h3 * dy;
          const unsigned d0 = sb_mask_pk(pk_bf16(dy * ww.x, dy * ww.y), h2p[j][0]);
          const unsigned d1 = sb_mask_pk(pk_bf16(dy * ww.z, dy * ww.w), h2p[j][1]);
          *reinterpret_cast<uint2*>(ZS + r * 32 + 8 * g) = make_uint2(d0, d1);
        }
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        float v = s3[i];
        v += __shfl_xor(v, 1, 64);
        v += __shfl_xor(v, 2, 64);
        v += __shfl_xor(v, 4, 64);
        v += __shfl_xor(v, 8, 64);
        if (l15 == 0) sgw[wid * 16 + 4 * g + i] = v;
      }
    }
    __syncthreads();  // ZS (own dZ2) complete
    // publish dZ2[:, O] as [row][16] (B x 32 B contiguous), 16-B sc1 stores
    for (int piece = tid; piece < 2 * B; piece += 256)
      st16(*reinterpret_cast<const sb_u32x4*>(ZS + piece * 16), SBO_DZ2 + wk * 2048 + piece * 4);
    stamp(6);
    arrive(tagv(k));  // hand-off 2: dZ2 blocks

    // dW2[O, :] = dZ2[:, O]^T H1 (own; overlaps the other workers' arrivals): wave w in-tiles
    // 4w .. 4w + 3, K = rows; db2 by the ones operand (wave 0)
    f32x4 dw2a[4];
    f32x4 db2a = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int j = 0; j < 4; ++j) dw2a[j] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int kk = 0; kk < KK; ++kk) {
      bf16x8 af;
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const bf16x4 t = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (lds_bf16x4*)(ZS + (32 * kk + 8 * g + 4 * h + tq) * 32 + 8 * tp));
#pragma unroll
        for (int e = 0; e < 4; ++e) af[4 * h + e] = t[e];
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        bf16x8 bfr;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const bf16x4 t = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
              (lds_bf16x4*)(H1s + tile_off(32 * kk + 8 * g + 4 * h + tq, 16 * (4 * wid + j) + 4 * tp)));
#pragma unroll
          for (int e = 0; e < 4; ++e) bfr[4 * h + e] = t[e];
        }
        dw2a[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bfr, dw2a[j], 0, 0, 0);
      }
      if (wid == 0) db2a = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, ones, db2a, 0, 0, 0);
    }
    if (wid == 0 && l15 == 0) {
#pragma unroll
      for (int i = 0; i < 4; ++i) sg[16 + 4 * g + i] = db2a[i];
    }
    // W2, b2, w3 are complete here: their Adam update and the next step's W2 image run while
    // the other workers' dZ2 blocks arrive (t = step0 + k + 1, as FlatAdam's device counter)
    const float tstep = step0 + (float)(k + 1);
    const float rbc1 = 1.f / (1.f - __powf(a.b1, tstep)), rbc2 = 1.f / (1.f - __powf(a.b2, tstep));
    __syncthreads();  // every wave past its dZ2 (ZS) reads; db2 in LDS
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int i = 0; i < 4; ++i) sb_adam(p2[j][i], dw2a[j][i], m2[j][i], v2[j][i], a.lr, a.b1, a.b2, a.eps, a.wd, rbc1, rbc2);
    if (wid == 3 && lane >= 16 && lane < 48) {
      float gs;
      if (lane < 32) gs = sg[lane];  // db2
      else {                         // dw3: the four waves' partials in order
        const int u = lane - 32;
        gs = ((sgw[u] + sgw[16 + u]) + sgw[32 + u]) + sgw[48 + u];
      }
      sb_adam(ps, gs, ms, vs, a.lr, a.b1, a.b2, a.eps, a.wd, rbc1, rbc2);
    }
    publish_w2(par ^ 1);  // parity par ^ 1: this step's block is still being read
    // this step's W2^T column block (published before barrier 3 of the previous step)
    bf16x8 a2[8];
#pragma unroll
    for (int ks = 0; ks < 8; ++ks) {
      const int owner = 2 * ks + (g >> 1);
      a2[ks] = __builtin_bit_cast(bf16x8, ld16(SBO_W2T + ((par * SB_G + owner) * 256 + 16 * wk + l15) * 8 + 4 * (g & 1)));
    }
    stamp(7);
    wait(tagv(k));  // hand-off 2 (and the workgroup barrier: every wave is done reading ZS / H1s for dW2)
    stamp(8);

    // ---- E: dH1[:, U] = dZ2 W2[:, U] from L2 fragments (two row tiles in flight); dZ1 =
    // dH1 [H1 > 0] -> ZS
    {
      bf16x8 bz[2][8];
      auto load_bz = [&](int j, int slot) {
        const int rt = wid + 4 * j;
        if (rt < R16) {
          const int r = 16 * rt + l15;
#pragma unroll
          for (int ks = 0; ks < 8; ++ks) {
            const int owner = 2 * ks + (g >> 1);
            bz[slot][ks] = __builtin_bit_cast(bf16x8, ld16(SBO_DZ2 + owner * 2048 + r * 8 + 4 * (g & 1)));
          }
        }
      };
      load_bz(0, 0);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        if (j + 1 < 4) load_bz(j + 1, (j + 1) & 1);
        const int rt = wid + 4 * j;
        if (rt < R16) {
          const int r = 16 * rt + l15;
          f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int ks = 0; ks < 8; ++ks) acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a2[ks], bz[j & 1][ks], acc, 0, 0, 0);
          const uint2 hv = *reinterpret_cast<const uint2*>(H1s + tile_off(r, 16 * wk + 4 * g));
          *reinterpret_cast<uint2*>(ZS + r * 32 + 8 * g) =
              make_uint2(sb_mask_pk(pk_bf16(acc[0], acc[1]), hv.x), sb_mask_pk(pk_bf16(acc[2], acc[3]), hv.y));
        }
      }
    }
    __syncthreads();  // dZ1 complete
    stamp(9);
    // dW1[U, :] = dZ1^T X (wave f < NFT: feature tile f), db1 by the ones operand (wave 3)
    f32x4 dw1a = f32x4{0.f, 0.f, 0.f, 0.f}, db1a = f32x4{0.f, 0.f, 0.f, 0.f};
    if (wid < NFT || wid == 3) {
      for (int kk = 0; kk < KK; ++kk) {
        bf16x8 af;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const bf16x4 t = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
              (lds_bf16x4*)(ZS + (32 * kk + 8 * g + 4 * h + tq) * 32 + 8 * tp));
#pragma unroll
          for (int e = 0; e < 4; ++e) af[4 * h + e] = t[e];
        }
        if (wid < NFT) {
          bf16x8 bx;
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            const int r = 32 * kk + 8 * g + 4 * h + tq, f0 = 16 * wid + 4 * tp;
            const bf16x4 t = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                (lds_bf16x4*)(Xs + r * 64 + (((f0 >> 3) ^ ((r >> 2) & 3)) << 4) + ((f0 & 7) << 1)));
#pragma unroll
            for (int e = 0; e < 4; ++e) bx[4 * h + e] = t[e];
          }
          dw1a = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bx, dw1a, 0, 0, 0);
        }
        if (wid == 3) db1a = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, ones, db1a, 0, 0, 0);
      }
    }
    if (wid == 3 && l15 == 0) {
#pragma unroll
      for (int i = 0; i < 4; ++i) sg[4 * g + i] = db1a[i];
    }
    __syncthreads();  // small gradients complete; every wave done with H1s, ZS, Xs
    stamp(10);

    // ---- F: Adam on W1 / b1 / b3 (their gradients complete only now), then the next step's
    // granules
    {
#pragma unroll
      for (int i = 0; i < 4; ++i)
        if (own1) sb_adam(p1[i], dw1a[i], m1[i], v1[i], a.lr, a.b1, a.b2, a.eps, a.wd, rbc1, rbc2);
      if (wid == 3 && (lane < 16 || lane == 48) && es >= 0)
        sb_adam(ps, lane < 16 ? sg[lane] : sg[48], ms, vs, a.lr, a.b1, a.b2, a.eps, a.wd, rbc1, rbc2);
    }
    stamp(11);
    publish_w1(tagv(k + 1));
    stamp(12);
    stamp(13);
  }

  // ---- write back: master parameters, Adam state, the engine's bf16 images
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int o = 16 * wk + 4 * g + i, in = 16 * (4 * wid + j) + l15;
      const long e = a.oW2 + (long)o * 256 + in;
      a.p[e] = p2[j][i];
      a.m[e] = m2[j][i];
      a.v[e] = v2[j][i];
      if (a.shadow != nullptr) a.shadow[e] = f2bf(p2[j][i]);
      if (a.w2t != nullptr) a.w2t[(long)in * 256 + o] = f2bf(p2[j][i]);
    }
  if (own1) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const long e = a.oW1 + (long)(16 * wk + 4 * g + i) * Fp + f1;
      a.p[e] = p1[i];
      a.m[e] = m1[i];
      a.v[e] = v1[i];
      if (a.shadow != nullptr) a.shadow[e] = f2bf(p1[i]);
    }
  }
  if (es >= 0) {
    a.p[es] = ps;
    a.m[es] = ms;
    a.v[es] = vs;
    if (a.shadow != nullptr) a.shadow[es] = f2bf(ps);
  }
  // the last worker out re-zeroes the counter (every worker has passed its last wait)
  if (tid == 0) {
    if (wk == 0) a.step[0] = step0 + (float)K;
    if (__hip_atomic_fetch_add((sb_g32*)(a.sync + 1), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == SB_G - 1) {
      __hip_atomic_store(cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store((sb_g32*)(a.sync + 1), 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_fetch_add((sb_g32*)(a.sync + 3), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

}  // namespace

bool launch_mlp_small(const MlpSmallArgs& a, hipStream_t s) {
  if (a.B < 32 || a.B > 256 || a.B % 32 != 0 || a.Fp <= 0 || a.Fp > 32 || a.Fp % 8 != 0 || a.K <= 0 || a.K > 4095)
    return false;  // (tags: launch ordinal x 4096 + step + 1)
  if (a.scr == nullptr || a.sync == nullptr || a.p == nullptr || a.m == nullptr || a.v == nullptr || a.step == nullptr)
    return false;
  if (a.Fp <= 16)
    hipLaunchKernelGGL(mlp_small_kernel<1>, dim3(SB_G), dim3(256), 0, s, a);
  else
    hipLaunchKernelGGL(mlp_small_kernel<2>, dim3(SB_G), dim3(256), 0, s, a);
  return true;
}

}  // namespace wf
