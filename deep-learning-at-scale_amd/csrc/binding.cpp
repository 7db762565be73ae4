// wellflow — Python bindings for the HIP kernel library (pybind11 via torch/extension.h).
//
// Every entry point validates device, dtype, contiguity, alignment and the extents the
// kernel and its grid will touch BEFORE launching: a hand-written kernel indexing out of
// bounds can take the whole GPU node down, so shape errors must be caught on the host.
#include <torch/extension.h>
#include <ATen/hip/impl/HIPStreamMasqueradingAsCUDA.h>
#include <ATen/hip/impl/HIPGuardImplMasqueradingAsCUDA.h>

#include <cstdlib>
#include <map>
#include <type_traits>
#include <mutex>
#include <vector>

#include "kernels.h"

namespace {

using wf::bf16_t;

// A/B and diagnostic environment overrides are read only when the HIP objects are a WF_DIAG
// build (wf::dbg_mask() is ~0 there): a production _C.so reads exactly the documented knobs
// (README "Environment knobs"; tests/test_diag_cpu.py checks the set).
int diag_env(const char* name, int dflt) {
  if (wf::dbg_mask() != ~0) return dflt;
  const char* v = std::getenv(name);
  return v != nullptr ? std::atoi(v) : dflt;
}

bool disable_glds() {
  static const bool off = diag_env("WELLFLOW_NO_GLDS", 0) == 1;  // register-staged GEMM (A/B)
  return off;
}

hipStream_t cur_stream() { return c10::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream(); }

void check_t(const at::Tensor& t, at::ScalarType dt, const char* name) {
  TORCH_CHECK(t.defined(), name, ": undefined tensor");
  TORCH_CHECK(t.is_cuda(), name, ": must be a GPU tensor");
  TORCH_CHECK(t.scalar_type() == dt, name, ": expected dtype ", dt, " got ", t.scalar_type());
  TORCH_CHECK(t.is_contiguous(), name, ": must be contiguous");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(t.data_ptr()) % 16 == 0, name,
              ": data pointer must be 16-byte aligned");
}

void check_extent(const at::Tensor& t, int64_t need, const char* name) {
  TORCH_CHECK(t.numel() >= need, name, ": needs at least ", need, " elements, has ", t.numel());
}

bf16_t* bfp(const at::Tensor& t) { return reinterpret_cast<bf16_t*>(t.data_ptr()); }
float* fp(const at::Tensor& t) { return t.data_ptr<float>(); }

template <class T>
T* opt_ptr(const c10::optional<at::Tensor>& t, at::ScalarType dt, const char* name,
           int64_t need) {
  if (!t.has_value() || !t->defined()) return nullptr;
  check_t(*t, dt, name);
  check_extent(*t, need, name);
  return reinterpret_cast<T*>(t->data_ptr());
}

// Extent of a logical [rows][K] operand stored K-contiguous or MN-contiguous.
int64_t operand_extent(bool mn, int64_t rows, int64_t K, int64_t ld) {
  if (rows == 0 || K == 0) return 0;
  return mn ? (K - 1) * ld + rows : (rows - 1) * ld + K;
}

void gemm(const at::Tensor& A, bool a_mn, int64_t lda, const at::Tensor& B, bool b_mn, int64_t ldb,
          int64_t M, int64_t N, int64_t K, int64_t ksplit, c10::optional<at::Tensor> outF,
          c10::optional<at::Tensor> outH, int64_t ldo, c10::optional<at::Tensor> bias,
          c10::optional<at::Tensor> mask, int64_t ldm, double mask_scale,
          c10::optional<at::Tensor> colsum, double alpha, double beta, int64_t act, bool atomic,
          double drop_p, int64_t seed, int64_t big_tile, c10::optional<at::Tensor> seed_dev) {
  check_t(A, at::kBFloat16, "A");
  check_t(B, at::kBFloat16, "B");
  TORCH_CHECK(M > 0 && N > 0 && K > 0, "gemm: empty problem");
  TORCH_CHECK(lda % 8 == 0 && ldb % 8 == 0, "gemm: lda/ldb must be multiples of 8");
  TORCH_CHECK(a_mn ? (M % 8 == 0) : (K % 8 == 0), "gemm: A contiguous extent must be a multiple of 8");
  TORCH_CHECK(b_mn ? (N % 8 == 0) : (K % 8 == 0), "gemm: B contiguous extent must be a multiple of 8");
  TORCH_CHECK(a_mn ? lda >= M : lda >= K, "gemm: lda too small");
  TORCH_CHECK(b_mn ? ldb >= N : ldb >= K, "gemm: ldb too small");
  check_extent(A, operand_extent(a_mn, M, K, lda), "A");
  check_extent(B, operand_extent(b_mn, N, K, ldb), "B");
  TORCH_CHECK(ldo >= N, "gemm: ldo < N");
  const int64_t out_need = (M - 1) * ldo + N;
  wf::GemmEpilogue e;
  e.outF = opt_ptr<float>(outF, at::kFloat, "outF", out_need);
  e.outH = opt_ptr<bf16_t>(outH, at::kBFloat16, "outH", out_need);
  TORCH_CHECK(e.outF || e.outH, "gemm: need an output");
  TORCH_CHECK(!atomic || (e.outF && !e.outH && beta == 0.0), "gemm: atomic needs outF only, beta 0");
  TORCH_CHECK(beta == 0.0 || e.outF, "gemm: beta needs outF");
  e.ldo = ldo;
  e.bias = opt_ptr<float>(bias, at::kFloat, "bias", N);
  if (mask.has_value() && mask->defined()) TORCH_CHECK(ldm >= N, "gemm: ldm < N");
  e.mask = opt_ptr<bf16_t>(mask, at::kBFloat16, "mask", (M - 1) * ldm + N);
  e.ldm = ldm;
  e.mask_scale = (float)mask_scale;
  e.colsum = opt_ptr<float>(colsum, at::kFloat, "colsum", N);
  e.alpha = (float)alpha;
  e.beta = (float)beta;
  e.act = (int)act;
  e.atomic = atomic ? 1 : 0;
  e.drop_p = (float)drop_p;
  e.seed = (unsigned long long)seed;
  if (seed_dev.has_value() && seed_dev->defined()) {
    TORCH_CHECK(seed_dev->is_cuda() && seed_dev->scalar_type() == at::kLong && seed_dev->numel() >= 1,
                "gemm: seed_dev must be a GPU int64 tensor");
    e.seed_dev = reinterpret_cast<const long long*>(seed_dev->data_ptr<int64_t>());
  }
  e.big_tile = (int)big_tile;
  TORCH_CHECK(ksplit == 1 || atomic, "gemm: split-K needs atomic accumulation");
  e.stage_ok = (e.outH != nullptr && e.outF == nullptr && !atomic && beta == 0.0 && N % 8 == 0 &&
                ldo % 8 == 0 && (e.mask == nullptr || ldm % 8 == 0))
                   ? 1 : 0;
  // glds (whole-tile) path: the 128x128 tiles may over-read rows/cols past M / N; allow it
  // only when that stays inside both allocations (and every K chunk is 64-aligned).
  const int64_t Mc = (M + 127) / 128 * 128, Nc = (N + 127) / 128 * 128;
  int64_t kchunk = (K + std::max<int64_t>(ksplit, 1) - 1) / std::max<int64_t>(ksplit, 1);
  kchunk = (kchunk + 63) / 64 * 64;
  const bool glds_ok = (K % 64 == 0) && (kchunk % 64 == 0) &&
                       A.numel() >= operand_extent(a_mn, Mc, K, lda) + (a_mn ? 0 : 0) &&
                       B.numel() >= operand_extent(b_mn, Nc, K, ldb) &&
                       (a_mn || Mc == M || lda >= K) && (b_mn || Nc == N || ldb >= K);
  const c10::hip::OptionalHIPGuardMasqueradingAsCUDA guard(A.device());
  wf::launch_gemm(bfp(A), lda, a_mn, bfp(B), ldb, b_mn, (int)M, (int)N, (int)K, (int)ksplit, e,
                  cur_stream(), glds_ok && !disable_glds());
}

wf::LstmDims lstm_dims(int64_t B, int64_t T, int64_t F, int64_t KX, int64_t H) {
  TORCH_CHECK(B > 0 && T > 0 && H > 0, "lstm: bad dims");
  TORCH_CHECK(H % 128 == 0, "lstm: hidden size must be a multiple of 128");
  TORCH_CHECK(KX % 64 == 0 && F + 1 <= KX, "lstm: KX must be a multiple of 64 and > F");
  wf::LstmDims d;
  d.B = (int)B; d.T = (int)T; d.F = (int)F; d.KX = (int)KX; d.H = (int)H;
  d.xcd_map = diag_env("WELLFLOW_XCD_MAP", 1) == 0 ? 0 : 1;  // diagnostics: 0 = identity tile order
  d.nt = diag_env("WELLFLOW_NT", 1) == 0 ? 0 : 1;
  // WELLFLOW_PF_DBG: timing-only switches and A/B variants of the persistent kernels. Only a
  // WF_DIAG build of the HIP objects (WELLFLOW_DIAG_BUILD=1) honours them: dbg_mask() is the
  // mask the objects were compiled with, so a production _C.so ignores the variable
  // (tests/test_diag_cpu.py checks this call stays here; bench.py refuses to run with it set).
  const char* pd = std::getenv("WELLFLOW_PF_DBG");
  d.dbg = (pd != nullptr ? std::atoi(pd) : 0) & wf::dbg_mask();
  const char* sl = std::getenv("WELLFLOW_SPIN_LIMIT");  // tests: force the hand-off timeout path
  d.spin_limit = sl != nullptr ? (unsigned)std::strtoul(sl, nullptr, 10) : 0u;
  const char* ft = std::getenv("WELLFLOW_FORCE_TIMEOUT");  // tests: every hand-off wait trips its bound
  if (ft != nullptr && ft[0] == '1') d.dbg |= 1 << 21;  // fails the run loudly (STAT block)
  return d;
}

void check_lstm_state(const at::Tensor& XH, const at::Tensor& Cst, const at::Tensor& S,
                      const wf::LstmDims& d) {
  const int64_t KA = d.KX + d.H, G = 4 * d.H;
  const int64_t Bp = (d.B + 15) / 16 * 16;  // fragment-native state is padded to 16 rows
  check_t(XH, at::kBFloat16, "XH");
  check_t(Cst, at::kBFloat16, "Cst");  // bf16 cell-state history (lstm_layout.h)
  check_t(S, at::kBFloat16, "S");
  check_extent(XH, (int64_t)(d.T + 1) * d.B * KA, "XH");
  check_extent(Cst, (int64_t)(d.T + 1) * Bp * d.H, "Cst");
  check_extent(S, (int64_t)d.T * Bp * G, "S");
}

// full = false: only the feature chunks (the buffer's constant 1 column / zero padding were
// written by an earlier full pack of the same B)
void lstm_pack_x(const at::Tensor& x, const at::Tensor& XH, int64_t B, int64_t T, int64_t F,
                 int64_t KX, int64_t H, bool full) {
  auto d = lstm_dims(B, T, F, KX, H);
  check_t(x, at::kFloat, "x");
  check_extent(x, B * T * F, "x");
  check_t(XH, at::kBFloat16, "XH");
  check_extent(XH, (T + 1) * B * (KX + H), "XH");
  const c10::hip::OptionalHIPGuardMasqueradingAsCUDA guard(x.device());
  wf::launch_lstm_pack_x(fp(x), bfp(XH), d, cur_stream(), full);
}

// the batch's windows read in place from the resident row table: batch row b = rows
// starts[idx[b]] .. + T - 1 of `table` (data/features.py SeriesWindows)
void lstm_pack_x_win(const at::Tensor& table, const at::Tensor& starts, const at::Tensor& idx, const at::Tensor& XH,
                     int64_t B, int64_t T, int64_t F, int64_t KX, int64_t H, bool full) {
  auto d = lstm_dims(B, T, F, KX, H);
  check_t(table, at::kFloat, "table");
  TORCH_CHECK(table.dim() == 2 && table.size(1) == F && table.size(0) >= T, "lstm_pack_x_win: table must be [>= T][F]");
  check_t(starts, at::kLong, "starts");
  check_t(idx, at::kLong, "idx");
  check_extent(idx, B, "idx");
  TORCH_CHECK(starts.numel() >= 1, "lstm_pack_x_win: no windows");
  check_t(XH, at::kBFloat16, "XH");
  check_extent(XH, (T + 1) * B * (KX + H), "XH");
  const c10::hip::OptionalHIPGuardMasqueradingAsCUDA guard(table.device());
  wf::launch_lstm_pack_x(fp(table), bfp(XH), d, cur_stream(), full, reinterpret_cast<const long*>(starts.data_ptr<int64_t>()),
                         reinterpret_cast<const long*>(idx.data_ptr<int64_t>()), starts.numel(), table.size(0));
}

// cf32: fp32 [Bp][H] in-place state slab of the per-step path (c_{t-1} -> c_t; e.g. the
// engine's dcarry buffer, which the backward re-initialises)
void lstm_forward(const at::Tensor& XH, const at::Tensor& Wp, const at::Tensor& Cst,
                  const at::Tensor& S, const at::Tensor& cf32, int64_t B, int64_t T, int64_t F, int64_t KX,
                  int64_t H, int64_t variant) {
  auto d = lstm_dims(B, T, F, KX, H);
  d.fwd_variant = (int)variant;
  check_lstm_state(XH, Cst, S, d);
  check_t(Wp, at::kBFloat16, "Wp");
  check_extent(Wp, 4 * H * (KX + H), "Wp");
  check_t(cf32, at::kFloat, "cf32");
  check_extent(cf32, (B + 15) / 16 * 16 * H, "cf32");
  const c10::hip::OptionalHIPGuardMasqueradingAsCUDA guard(XH.device());
  auto s = cur_stream();
  for (int t = 0; t < d.T; ++t) wf::launch_lstm_fwd_step(t, bfp(XH), bfp(Wp), bfp(Cst), bfp(S), fp(cf32), d, s);
}

// A persistent kernel's sync buffer: int32, 16-B aligned, zeroed once by its owner. No launch
// resets it (csrc/persistent_sync.h: monotonic launch epochs and arrival counters), so there is
// no memset node in a captured step at all (round 2's early exit was an unaligned per-launch
// memset node under graph replay, profiles/r3_early_exit.md).
void check_sync(const at::Tensor& sync) {
  check_t(sync, at::kInt, "sync");  // check_t: 16-B aligned data pointer
}

// Raise on a failed persistent launch (status < 0: -(hipError_t)); 0 = not supported.
bool persistent_status(int st, const char* what) {
  TORCH_CHECK(st >= 0, what, ": launch failed: ", hipGetErrorString((hipError_t)(-st)));
  return st == 1;
}

// All T steps in one persistent launch per sub-batch (lstm_persistent.hip). Returns false
// (nothing launched) when the shape or device cannot host it and raises when the launch
// fails; `sync` (int32): csrc/persistent_sync.h (hand-off words) + the STAT block at its end.
bool lstm_forward_persistent(const at::Tensor& XH, const at::Tensor& Wp, const at::Tensor& Cst,
                             const at::Tensor& S, const at::Tensor& sync, int64_t B, int64_t T, int64_t F,
                             int64_t KX, int64_t H) {
  auto d = lstm_dims(B, T, F, KX, H);
  check_lstm_state(XH, Cst, S, d);
  check_t(Wp, at::kBFloat16, "Wp");
  check_extent(Wp, 4 * H * (KX + H), "Wp");
  check_sync(sync);
  const c10::hip::OptionalHIPGuardMasqueradingAsCUDA guard(XH.device());
  return persistent_status(wf::launch_lstm_fwd_persistent(bfp(XH), bfp(Wp), bfp(Cst), bfp(S),
                                                          reinterpret_cast<unsigned*>(sync.data_ptr<int>()),
                                                          sync.numel(), d, cur_stream()),
                           "persistent LSTM forward");
}

void lstm_backward(const at::Tensor& WhhT, const at::Tensor& XH, const at::Tensor& Cst,
                   const at::Tensor& S, const at::Tensor& DG, const at::Tensor& dcarry,
                   const at::Tensor& dy, const at::Tensor& w_out, int64_t B, int64_t T, int64_t F,
                   int64_t KX, int64_t H, int64_t variant, const c10::optional<at::Tensor>& sync) {
  auto d = lstm_dims(B, T, F, KX, H);
  d.bwd_variant = (int)variant;
  check_lstm_state(XH, Cst, S, d);
  check_t(WhhT, at::kBFloat16, "WhhT");
  check_extent(WhhT, H * 4 * H, "WhhT");
  check_t(DG, at::kBFloat16, "DG");
  check_extent(DG, T * B * 4 * H, "DG");
  check_t(dcarry, at::kFloat, "dcarry");
  check_extent(dcarry, (B + 15) / 16 * 16 * H, "dcarry");
  check_t(dy, at::kFloat, "dy");
  check_extent(dy, B, "dy");
  check_t(w_out, at::kFloat, "w_out");
  check_extent(w_out, H, "w_out");
  const c10::hip::OptionalHIPGuardMasqueradingAsCUDA guard(XH.device());
  auto s = cur_stream();
  if (sync.has_value()) {  // step T-1, then the persistent chain (tools/pb_time.py)
    check_sync(*sync);
    wf::launch_lstm_bwd_step(d.T - 1, bfp(WhhT), bfp(Cst), bfp(S), bfp(DG), fp(dcarry), fp(dy),
                             fp(w_out), d, s);
    TORCH_CHECK(persistent_status(wf::launch_lstm_bwd_persistent(bfp(WhhT), bfp(Cst), bfp(S), bfp(DG), fp(dcarry),
                                                                 reinterpret_cast<unsigned*>(sync->data_ptr<int>()),
                                                                 sync->numel(), d, s),
                                  "persistent LSTM backward"),
                "persistent backward refused this shape");
    return;
  }
  for (int t = d.T - 1; t >= 0; --t)
    wf::launch_lstm_bwd_step(t, bfp(WhhT), bfp(Cst), bfp(S), bfp(DG), fp(dcarry), fp(dy),
                             fp(w_out), d, s);
}

// Two persistent side streams per device for the backward pass: the serial BPTT chain
// runs on a HIGH-priority stream, the weight-gradient GEMM chunks on a LOW-priority one,
// fork/joined to the caller's stream with events (capturable in a hipGraph).
struct SideStreams {
  hipStream_t hi = nullptr, lo = nullptr;
  std::vector<hipEvent_t> ev;
};

SideStreams& side_streams(int dev, size_t nev) {
  static std::mutex mu;
  static std::map<int, SideStreams> all;
  std::lock_guard<std::mutex> g(mu);
  SideStreams& ss = all[dev];
  if (ss.hi == nullptr) {
    int least = 0, greatest = 0;
    TORCH_CHECK(hipDeviceGetStreamPriorityRange(&least, &greatest) == hipSuccess, "stream priorities");
    TORCH_CHECK(hipStreamCreateWithPriority(&ss.hi, hipStreamNonBlocking, greatest) == hipSuccess,
                "hi stream");
    TORCH_CHECK(hipStreamCreateWithPriority(&ss.lo, hipStreamNonBlocking, least) == hipSuccess,
                "lo stream");
  }
  while (ss.ev.size() < nev) {
    hipEvent_t e;
    TORCH_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming) == hipSuccess, "event");
    ss.ev.push_back(e);
  }
  return ss;
}

// Full LSTM backward: BPTT chain + dWcat = sum_t DG[t]^T XH[t] into gW (fp32 [G][KA],
// accumulated with atomics, so it must be zeroed by the caller). With chunk > 0 the dW
// GEMM is cut into chunks of `chunk` timesteps, each launched on the low-priority stream
// as soon as the chain has produced its DG slabs: compute-bound dW work fills the gaps of
// the memory/latency-bound chain instead of running after it.
// Returns true when the BPTT chain ran as the persistent kernel (false: per-step kernels).
bool lstm_backward_dw(const at::Tensor& WhhT, const at::Tensor& XH, const at::Tensor& Cst,
                      const at::Tensor& S, const at::Tensor& DG, const at::Tensor& dcarry,
                      const at::Tensor& dy, const at::Tensor& w_out, const at::Tensor& gW,
                      int64_t B, int64_t T, int64_t F, int64_t KX, int64_t H, int64_t variant,
                      int64_t chunk, int64_t ksplit, const c10::optional<at::Tensor>& sync,
                      const c10::optional<at::Tensor>& dw_slab) {
  auto d = lstm_dims(B, T, F, KX, H);
  d.bwd_variant = (int)variant;
  check_lstm_state(XH, Cst, S, d);
  check_t(WhhT, at::kBFloat16, "WhhT");
  check_extent(WhhT, H * 4 * H, "WhhT");
  check_t(DG, at::kBFloat16, "DG");
  check_extent(DG, T * B * 4 * H, "DG");
  check_t(dcarry, at::kFloat, "dcarry");
  check_extent(dcarry, (B + 15) / 16 * 16 * H, "dcarry");
  check_t(dy, at::kFloat, "dy");
  check_extent(dy, B, "dy");
  check_t(w_out, at::kFloat, "w_out");
  check_extent(w_out, H, "w_out");
  check_t(gW, at::kFloat, "gW");
  const int64_t G = 4 * H, KA = KX + H;
  check_extent(gW, G * KA, "gW");
  const c10::hip::OptionalHIPGuardMasqueradingAsCUDA guard(XH.device());
  hipStream_t main = cur_stream();

  auto dw = [&](int t0, int t1, hipStream_t s) {
    const int64_t K = (int64_t)(t1 - t0) * B;
    wf::GemmEpilogue e;
    e.outF = fp(gW);
    e.ldo = KA;
    e.atomic = 1;
    // WELLFLOW_DW_BIG: 0 = 128x128 tile, 1 = 256x128 8-wave, 2 = 128x288 4-wave,
    // 3 = 256x192 8-wave (tools/tune_lstm.py, B = 8192, split-K 32: 1.35 / 1.60 / 1.28 ms for
    // 1 / 2 / 3), 4 / 5 = 256x192 with a 5- / 4-slot 32-deep ring, 6 = 256x192 with staggered
    // wave groups, 7 (default) = 256x288 4-slot 32-deep ring (tools/dw_tiles.py: 1.107 ms vs
    // 1.166 for 3, 1.149 for 4, 1.307 for 6); shapes a tile cannot take fall back to 256x128
    static const int big = diag_env("WELLFLOW_DW_BIG", 7);
    e.big_tile = big;
    if (dw_slab.has_value()) {  // split-K partials plain-stored, one reduce (gemm.hip launch_dw_288w)
      check_t(*dw_slab, at::kFloat, "dw_slab");
      e.slab = fp(*dw_slab);
      e.slab_cap = dw_slab->numel();
    }
    const bf16_t* A = bfp(DG) + (size_t)t0 * B * G;
    const bf16_t* Bm = bfp(XH) + (size_t)t0 * B * KA;
    // whole-tile over-read of XH columns 576..639 stays inside XH (its slab T follows)
    int64_t ks = std::max<int64_t>(1, ksplit);
    int64_t kchunk = ((K + ks - 1) / ks + 63) / 64 * 64;
    const bool glds_ok = (K % 64 == 0) && (kchunk % 64 == 0) && !disable_glds();
    wf::launch_gemm(A, G, 1, Bm, KA, 1, (int)G, (int)KA, (int)K, (int)ks, e, s, glds_ok);
  };

  if (chunk <= 0) {
    // step T-1 (dh from the head), then steps T-2 .. 0 in one persistent launch when a sync
    // buffer is given and the shape fits (lstm_persistent_bwd.hip), else per-step kernels
    wf::launch_lstm_bwd_step(d.T - 1, bfp(WhhT), bfp(Cst), bfp(S), bfp(DG), fp(dcarry), fp(dy),
                             fp(w_out), d, main);
    bool done = false;
    if (sync.has_value()) {
      check_sync(*sync);
      done = persistent_status(wf::launch_lstm_bwd_persistent(bfp(WhhT), bfp(Cst), bfp(S), bfp(DG), fp(dcarry),
                                                              reinterpret_cast<unsigned*>(sync->data_ptr<int>()),
                                                              sync->numel(), d, main),
                               "persistent LSTM backward");
    }
    if (!done)
      for (int t = d.T - 2; t >= 0; --t)
        wf::launch_lstm_bwd_step(t, bfp(WhhT), bfp(Cst), bfp(S), bfp(DG), fp(dcarry), fp(dy),
                                 fp(w_out), d, main);
    dw(0, d.T, main);
    return done;
  }
  const int nchunks = (int)((T + chunk - 1) / chunk);
  SideStreams& ss = side_streams(XH.device().index(), nchunks + 3);
  TORCH_CHECK(hipEventRecord(ss.ev[0], main) == hipSuccess, "event record");
  TORCH_CHECK(hipStreamWaitEvent(ss.hi, ss.ev[0], 0) == hipSuccess, "wait");
  TORCH_CHECK(hipStreamWaitEvent(ss.lo, ss.ev[0], 0) == hipSuccess, "wait");
  int t_end = d.T, k = 0;
  for (int t = d.T - 1; t >= 0; --t) {
    wf::launch_lstm_bwd_step(t, bfp(WhhT), bfp(Cst), bfp(S), bfp(DG), fp(dcarry), fp(dy),
                             fp(w_out), d, ss.hi);
    if (t % chunk == 0) {  // DG[t .. t_end) complete
      hipEvent_t e = ss.ev[3 + k++];
      TORCH_CHECK(hipEventRecord(e, ss.hi) == hipSuccess, "event record");
      TORCH_CHECK(hipStreamWaitEvent(ss.lo, e, 0) == hipSuccess, "wait");
      dw(t, t_end, ss.lo);
      t_end = t;
    }
  }
  TORCH_CHECK(hipEventRecord(ss.ev[1], ss.hi) == hipSuccess, "event record");
  TORCH_CHECK(hipEventRecord(ss.ev[2], ss.lo) == hipSuccess, "event record");
  TORCH_CHECK(hipStreamWaitEvent(main, ss.ev[1], 0) == hipSuccess, "join");
  TORCH_CHECK(hipStreamWaitEvent(main, ss.ev[2], 0) == hipSuccess, "join");
  return false;
}

// Adam on the LSTM's flat parameters + Wp / WhhT (lstm_pack_weights' output) in one launch
void lstm_adam_pack(const at::Tensor& p, const at::Tensor& g, const at::Tensor& m, const at::Tensor& v,
                    const at::Tensor& step, double lr, double b1, double b2, double eps, double wd, double gscale,
                    bool zero_g, const at::Tensor& Wp, const at::Tensor& WhhT, int64_t H, int64_t KX) {
  for (const at::Tensor* t : {&p, &g, &m, &v}) check_t(*t, at::kFloat, "p/g/m/v");
  const int64_t n = p.numel();
  TORCH_CHECK(g.numel() == n && m.numel() == n && v.numel() == n, "lstm_adam_pack: size mismatch");
  TORCH_CHECK(KX % 32 == 0 && H % 32 == 0 && n >= 4 * H * (KX + H), "lstm_adam_pack: layout (KX, H multiples of 32)");
  for (const at::Tensor* t : {&p, &g, &m, &v})
    TORCH_CHECK(reinterpret_cast<uintptr_t>(t->data_ptr()) % 16 == 0, "lstm_adam_pack: buffers must be 16-B aligned");
  check_t(step, at::kFloat, "step");
  check_extent(step, 2, "step");
  check_t(Wp, at::kBFloat16, "Wp");
  check_t(WhhT, at::kBFloat16, "WhhT");
  check_extent(Wp, 4 * H * (KX + H), "Wp");
  check_extent(WhhT, H * 4 * H, "WhhT");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(Wp.data_ptr()) % 8 == 0, "lstm_adam_pack: Wp must be 8-B aligned");
  const c10::hip::OptionalHIPGuardMasqueradingAsCUDA guard(p.device());
  wf::launch_lstm_adam_pack(fp(p), fp(g), fp(m), fp(v), n, fp(step), (float)lr, (float)b1, (float)b2, (float)eps,
                            (float)wd, (float)gscale, zero_g ? 1 : 0, (int)KX, (int)H, bfp(Wp), bfp(WhhT), cur_stream());
}

void lstm_pack_weights(const at::Tensor& W, const at::Tensor& Wp, const at::Tensor& WhhT,
                       int64_t H, int64_t KX) {
  auto d = lstm_dims(1, 1, 0, KX, H);
  check_t(W, at::kFloat, "W");
  check_t(Wp, at::kBFloat16, "Wp");
  check_t(WhhT, at::kBFloat16, "WhhT");
  check_extent(W, 4 * H * (KX + H), "W");
  check_extent(Wp, 4 * H * (KX + H), "Wp");
  check_extent(WhhT, H * 4 * H, "WhhT");
  const c10::hip::OptionalHIPGuardMasqueradingAsCUDA guard(W.device());
  wf::launch_lstm_pack_weights(fp(W), bfp(Wp), bfp(WhhT), d, cur_stream());
}

// Regression-head input H may be a strided view of a larger bf16 buffer (e.g. the last
// timestep of XH): the raw pointer is taken from the given tensor (its storage offset).
void check_head_h(const at::Tensor& Hm, int64_t ldh, int64_t B, int64_t Hd) {
  TORCH_CHECK(Hm.is_cuda() && Hm.scalar_type() == at::kBFloat16, "H: bf16 GPU tensor");
  TORCH_CHECK(Hd % 8 == 0 && ldh % 8 == 0 && Hd <= 2048, "head: Hd, ldh multiples of 8, Hd <= 2048");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(Hm.data_ptr()) % 16 == 0, "head: H must be 16-B aligned");
  TORCH_CHECK(ldh >= Hd, "head: ldh < Hd");
  TORCH_CHECK(Hm.storage().nbytes() - Hm.storage_offset() * 2 >= (size_t)(((B - 1) * ldh + Hd) * 2),
              "head: H too small");
}

void head_fwd(const at::Tensor& Hm, int64_t ldh, int64_t B, int64_t Hd, const at::Tensor& w,
              const at::Tensor& b0, c10::optional<at::Tensor> target, const at::Tensor& pred,
              c10::optional<at::Tensor> dy, c10::optional<at::Tensor> loss_sum, double dy_scale) {
  check_head_h(Hm, ldh, B, Hd);
  TORCH_CHECK(Hd % 8 == 0 && ldh % 8 == 0, "head: Hd and ldh must be multiples of 8");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(Hm.data_ptr()) % 16 == 0, "head: H must be 16-B aligned");
  check_t(w, at::kFloat, "w");
  check_extent(w, Hd, "w");
  check_t(b0, at::kFloat, "b0");
  check_t(pred, at::kFloat, "pred");
  check_extent(pred, B, "pred");
  const c10::hip::OptionalHIPGuardMasqueradingAsCUDA guard(Hm.device());
  wf::launch_head_fwd(bfp(Hm), ldh, (int)B, (int)Hd, fp(w), fp(b0),
                      opt_ptr<float>(target, at::kFloat, "target", B), fp(pred),
                      opt_ptr<float>(dy, at::kFloat, "dy", B),
                      opt_ptr<float>(loss_sum, at::kFloat, "loss_sum", 1), (float)dy_scale,
                      cur_stream());
}

// Fused MLP backward (mlp_fused.hip) for the F -> 256 -> 256 -> 1 shape: dZ2, dZ1 and the
// bias / head gradients in one launch (the dW GEMMs stay separate).
// ReLU bitmask of the MLP's second hidden layer: int32 [B][8] (256 bits per row), 16-B aligned
static unsigned* mask_ptr(const c10::optional<at::Tensor>& M2, int64_t B) {
  if (!M2.has_value()) return nullptr;
  check_t(*M2, at::kInt, "M2");
  check_extent(*M2, B * 8, "M2");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(M2->data_ptr()) % 16 == 0, "M2 must be 16-B aligned");
  return reinterpret_cast<unsigned*>(M2->data_ptr<int>());
}

static const long long* rows_ptr(const c10::optional<at::Tensor>& rows, int64_t B) {
  if (!rows.has_value() || !rows->defined()) return nullptr;
  TORCH_CHECK(rows->is_cuda() && rows->scalar_type() == at::kLong && rows->is_contiguous(), "rows: contiguous int64 GPU tensor");
  TORCH_CHECK(rows->numel() >= B, "rows: needs ", B, " indices");
  return reinterpret_cast<const long long*>(rows->data_ptr<int64_t>());
}

// X rows read by a kernel: B rows directly, or dataset rows named by `rows`. Returns the
// dataset row count; the kernels CLAMP every index into [0, nrows) (an out-of-range index
// must never become an out-of-bounds device read, and checking here would need a host sync,
// which a captured hipGraph step cannot do).
static int64_t check_x_rows(const at::Tensor& X, int64_t Fp, int64_t B, const c10::optional<at::Tensor>& rows) {
  if (!rows.has_value() || !rows->defined()) {
    check_extent(X, B * Fp, "X");
    return B;
  }
  const int64_t nrows = X.numel() / Fp;
  TORCH_CHECK(nrows > 0, "X: empty dataset");
  return nrows;
}

bool mlp2_backward(c10::optional<at::Tensor> H1, const at::Tensor& H2, const at::Tensor& dy, const at::Tensor& w3,
                   const at::Tensor& W2, const at::Tensor& X, int64_t Fp, const at::Tensor& dZ1,
                   const at::Tensor& dZ2, c10::optional<at::Tensor> dW1, const at::Tensor& db1,
                   const at::Tensor& db2, const at::Tensor& dw3, const at::Tensor& db3, int64_t B,
                   c10::optional<at::Tensor> M2, c10::optional<at::Tensor> W1, c10::optional<at::Tensor> b1,
                   c10::optional<at::Tensor> rows, c10::optional<at::Tensor> red) {
  constexpr int64_t H = 256;
  const bool recompute = !H1.has_value() || !H1->defined();
  std::vector<const at::Tensor*> acts = {&H2, &dZ1, &dZ2};
  if (!recompute) acts.push_back(&*H1);
  for (const at::Tensor* t : acts) {
    check_t(*t, at::kBFloat16, "H/dZ");
    check_extent(*t, B * H, "H/dZ");
  }
  check_t(W2, at::kBFloat16, "W2");
  check_extent(W2, H * H, "W2");
  check_t(dy, at::kFloat, "dy");
  check_extent(dy, B, "dy");
  for (const at::Tensor* t : {&w3, &db1, &db2, &dw3}) {
    check_t(*t, at::kFloat, "w3/db");
    check_extent(*t, H, "w3/db");
  }
  check_t(db3, at::kFloat, "db3");
  check_extent(db3, 1, "db3");
  check_t(X, at::kBFloat16, "X");
  const int64_t nrows = check_x_rows(X, Fp, B, rows);
  const bf16_t* w1p = opt_ptr<bf16_t>(W1, at::kBFloat16, "W1", H * Fp);
  const float* b1p = opt_ptr<float>(b1, at::kFloat, "b1", H);
  TORCH_CHECK(!recompute || (w1p && b1p && dW1.has_value()), "mlp2_backward: H1 recompute needs W1, b1 and dW1");
  const c10::hip::OptionalHIPGuardMasqueradingAsCUDA guard(H2.device());
  return wf::launch_mlp2_bwd(recompute ? nullptr : bfp(*H1), bfp(H2), mask_ptr(M2, B), fp(dy), fp(w3), bfp(W2), bfp(X),
                             (int)Fp, bfp(dZ1), bfp(dZ2), opt_ptr<float>(dW1, at::kFloat, "dW1", H * Fp), fp(db1),
                             fp(db2), fp(dw3), fp(db3), (int)B, w1p, b1p, rows_ptr(rows, B), nrows, cur_stream(),
                             opt_ptr<float>(red, at::kFloat, "red", wf::kMlpRedFloats));
}

// dW2 [256][256] += dZ2^T relu(X W1^T + b1), H1 recomputed (mlp_fused.hip mlp2_dw2_kernel).
bool mlp2_dw2(const at::Tensor& dZ2, const at::Tensor& X, int64_t Fp, c10::optional<at::Tensor> rows,
              const at::Tensor& W1, const at::Tensor& b1, int64_t B, int64_t nsplit, const at::Tensor& dW2,
              c10::optional<at::Tensor> red) {
  constexpr int64_t H = 256;
  check_t(dZ2, at::kBFloat16, "dZ2");
  check_extent(dZ2, B * H, "dZ2");
  check_t(X, at::kBFloat16, "X");
  const int64_t nrows = check_x_rows(X, Fp, B, rows);
  check_t(W1, at::kBFloat16, "W1");
  check_extent(W1, H * Fp, "W1");
  check_t(b1, at::kFloat, "b1");
  check_extent(b1, H, "b1");
  check_t(dW2, at::kFloat, "dW2");
  check_extent(dW2, H * H, "dW2");
  const c10::hip::OptionalHIPGuardMasqueradingAsCUDA guard(dZ2.device());
  return wf::launch_mlp2_dw2(bfp(dZ2), bfp(X), (int)Fp, rows_ptr(rows, B), nrows, bfp(W1), fp(b1), (int)B, (int)nsplit,
                             fp(dW2), cur_stream(), opt_ptr<float>(red, at::kFloat, "red", wf::kMlpRedFloats));
}

// Sums the spread-reduction scratch of the 8-wave MLP training kernels into the gradients
// (mlp_fused.hip mlp2_reduce_kernel) and zeroes it; null destinations are skipped.
void mlp2_reduce(const at::Tensor& red, int64_t Fp, int64_t B, c10::optional<at::Tensor> loss_sum, const at::Tensor& db3,
                 const at::Tensor& dw3, const at::Tensor& db1, const at::Tensor& db2, const at::Tensor& dW1,
                 c10::optional<at::Tensor> dW2, int64_t dw2_rows) {
  constexpr int64_t H = 256;
  check_t(red, at::kFloat, "red");
  check_extent(red, wf::kMlpRedFloats, "red");
  TORCH_CHECK(Fp > 0 && Fp <= 64, "mlp2_reduce: Fp <= 64");
  for (const at::Tensor* t : {&dw3, &db1, &db2}) {
    check_t(*t, at::kFloat, "dw3/db");
    check_extent(*t, H, "dw3/db");
  }
  check_t(db3, at::kFloat, "db3");
  check_extent(db3, 1, "db3");
  check_t(dW1, at::kFloat, "dW1");
  check_extent(dW1, H * Fp, "dW1");
  const c10::hip::OptionalHIPGuardMasqueradingAsCUDA guard(red.device());
  TORCH_CHECK(B > 0, "mlp2_reduce: B > 0");
  wf::launch_mlp2_reduce(fp(red), (int)Fp, (int)B, opt_ptr<float>(loss_sum, at::kFloat, "loss_sum", 1), fp(db3), fp(dw3),
                         fp(db1), fp(db2), fp(dW1), opt_ptr<float>(dW2, at::kFloat, "dW2", H * H), cur_stream(),
                         (int)dw2_rows);
}

// MLP training step forward + backward in one launch (mlp_step.hip); the batch sums land in
// the spread scratch `red` (mlp2_reduce adds them), dZ2 feeds mlp2_dw2. False = not covered.
bool mlp2_step(const at::Tensor& X, int64_t Fp, const at::Tensor& W1, const at::Tensor& b1, const at::Tensor& W2,
               const at::Tensor& b2, const at::Tensor& w3, const at::Tensor& b3, const at::Tensor& y, double dy_scale,
               int64_t B, c10::optional<at::Tensor> rows, const at::Tensor& dZ2, c10::optional<at::Tensor> pred,
               const at::Tensor& red, bool dz_frag, c10::optional<at::Tensor> W2T, double clip) {
  constexpr int64_t H = 256;
  check_t(X, at::kBFloat16, "X");
  const int64_t nrows = check_x_rows(X, Fp, B, rows);
  check_t(W1, at::kBFloat16, "W1");
  check_extent(W1, H * Fp, "W1");
  check_t(W2, at::kBFloat16, "W2");
  check_extent(W2, H * H, "W2");
  for (const at::Tensor* t : {&b1, &b2, &w3}) {
    check_t(*t, at::kFloat, "bias/w3");
    check_extent(*t, H, "bias/w3");
  }
  check_t(b3, at::kFloat, "b3");
  check_extent(b3, 1, "b3");
  check_t(y, at::kFloat, "y");
  check_extent(y, nrows, "y");
  check_t(dZ2, at::kBFloat16, "dZ2");
  check_extent(dZ2, B * H, "dZ2");
  check_t(red, at::kFloat, "red");
  check_extent(red, wf::kMlpRedFloats, "red");
  for (const at::Tensor* t : {&X, &W1, &W2, &dZ2})
    TORCH_CHECK(reinterpret_cast<uintptr_t>(t->data_ptr()) % 16 == 0, "mlp2_step: bf16 operands must be 16-B aligned");
  TORCH_CHECK(B > 0, "mlp2_step: B > 0");
  const bf16_t* w2t = nullptr;
  if (W2T.has_value()) {
    check_t(*W2T, at::kBFloat16, "W2T");
    check_extent(*W2T, H * H, "W2T");
    TORCH_CHECK(reinterpret_cast<uintptr_t>(W2T->data_ptr()) % 16 == 0, "mlp2_step: W2T must be 16-B aligned");
    w2t = bfp(*W2T);
  }
  const c10::hip::OptionalHIPGuardMasqueradingAsCUDA guard(X.device());
  return wf::launch_mlp2_step(bfp(X), (int)Fp, bfp(W1), fp(b1), bfp(W2), fp(b2), fp(w3), fp(b3), fp(y), (float)dy_scale,
                              (int)B, rows_ptr(rows, B), nrows, bfp(dZ2), opt_ptr<float>(pred, at::kFloat, "pred", B),
                              fp(red), dz_frag, cur_stream(), w2t, (float)clip);
}

int64_t mlp_small_scratch_floats() { return wf::kMlpSmallScratch; }



// K small-batch MLP training steps (forward, backward, Adam) in ONE persistent launch
// (mlp_small.hip). X / Y: the dataset (bf16 [N][Fp], fp32 [N]) read through rows [K * B] (or
// contiguous from row 0); params / m / v / step: the flat parameters and FlatAdam state, updated
// in place; offs: (W1, b1, W2, b2, w3, b3) element offsets of the MlpLayout. False = not covered.
bool mlp_small_steps(const at::Tensor& X, const at::Tensor& Y, c10::optional<at::Tensor> rows, int64_t Fp, int64_t B,
                     int64_t K, const at::Tensor& params, const at::Tensor& m, const at::Tensor& v,
                     const at::Tensor& step, double lr, double b1, double b2, double eps, double wd, double dy_scale,
                     double clip, c10::optional<at::Tensor> shadow, c10::optional<at::Tensor> w2t,
                     c10::optional<at::Tensor> loss_acc, const at::Tensor& scr, const at::Tensor& sync,
                     std::vector<int64_t> offs, c10::optional<at::Tensor> stamps) {
  constexpr int64_t H = 256;
  TORCH_CHECK(offs.size() == 6, "mlp_small_steps: offs = (W1, b1, W2, b2, w3, b3)");
  TORCH_CHECK(K > 0 && B > 0, "mlp_small_steps: K, B > 0");
  check_t(X, at::kBFloat16, "X");
  check_t(Y, at::kFloat, "Y");
  int64_t nrows;
  const long long* rp = nullptr;
  if (rows.has_value() && rows->defined()) {
    rp = rows_ptr(rows, K * B);
    nrows = X.numel() / Fp;
    TORCH_CHECK(nrows > 0, "X: empty dataset");
  } else {
    check_extent(X, K * B * Fp, "X");
    nrows = K * B;
  }
  check_extent(Y, nrows, "Y");
  const int64_t n = params.numel();
  for (const at::Tensor* t : {&params, &m, &v}) {
    check_t(*t, at::kFloat, "params/m/v");
    check_extent(*t, n, "params/m/v");
  }
  TORCH_CHECK(offs[0] + H * Fp <= n && offs[2] + H * H <= n && offs[5] < n && offs[1] + H <= n && offs[3] + H <= n &&
                  offs[4] + H <= n, "mlp_small_steps: parameter offsets out of range");
  check_t(step, at::kFloat, "step");
  check_t(scr, at::kFloat, "scr");
  check_extent(scr, wf::kMlpSmallScratch, "scr");
  check_t(sync, at::kInt, "sync");
  check_extent(sync, 4, "sync");
  const c10::hip::OptionalHIPGuardMasqueradingAsCUDA guard(X.device());
  wf::MlpSmallArgs a{};
  a.X = bfp(X);
  a.Y = fp(Y);
  a.rows = rp;
  a.nrows = (long)nrows;
  a.Fp = (int)Fp;
  a.B = (int)B;
  a.K = (int)K;
  a.p = fp(params);
  a.m = fp(m);
  a.v = fp(v);
  a.step = fp(step);
  a.lr = (float)lr;
  a.b1 = (float)b1;
  a.b2 = (float)b2;
  a.eps = (float)eps;
  a.wd = (float)wd;
  a.dy_scale = (float)dy_scale;
  a.clip = (float)clip;
  a.shadow = opt_ptr<bf16_t>(shadow, at::kBFloat16, "shadow", n);
  a.w2t = opt_ptr<bf16_t>(w2t, at::kBFloat16, "w2t", H * H);
  a.loss_acc = opt_ptr<float>(loss_acc, at::kFloat, "loss_acc", 1);
  a.scr = fp(scr);
  a.sync = reinterpret_cast<unsigned*>(sync.data_ptr<int>());
  const char* sl = std::getenv("WELLFLOW_SPIN_LIMIT");  // tests: force the hand-off timeout path
  a.spin_limit = sl != nullptr ? (unsigned)std::strtoul(sl, nullptr, 10) : (1u << 22);
  a.oW1 = (long)offs[0];
  a.ob1 = (long)offs[1];
  a.oW2 = (long)offs[2];
  a.ob2 = (long)offs[3];
  a.ow3 = (long)offs[4];
  a.ob3 = (long)offs[5];
  a.stamps = reinterpret_cast<unsigned long long*>(opt_ptr<int64_t>(stamps, at::kLong, "stamps", 16 * 64 * 16));
  return wf::launch_mlp_small(a, cur_stream());
}

// dW2 from the fragment-layout dZ2 of mlp2_step(dz_frag=True) into the spread scratch's dW2
// copies (mlp_step.hip mlp2_dw2f_kernel; mlp2_reduce adds them). False = not covered.
int64_t mlp2_dw2f(const at::Tensor& dZ2F, const at::Tensor& X, int64_t Fp, c10::optional<at::Tensor> rows,
               const at::Tensor& W1, const at::Tensor& b1, int64_t B, int64_t nsplit, const at::Tensor& red) {
  constexpr int64_t H = 256;
  check_t(dZ2F, at::kBFloat16, "dZ2F");
  check_extent(dZ2F, B * H, "dZ2F");
  check_t(X, at::kBFloat16, "X");
  const int64_t nrows = check_x_rows(X, Fp, B, rows);
  check_t(W1, at::kBFloat16, "W1");
  check_extent(W1, H * Fp, "W1");
  check_t(b1, at::kFloat, "b1");
  check_extent(b1, H, "b1");
  check_t(red, at::kFloat, "red");
  check_extent(red, wf::kMlpRedFloats, "red");
  for (const at::Tensor* t : {&dZ2F, &X, &W1})
    TORCH_CHECK(reinterpret_cast<uintptr_t>(t->data_ptr()) % 16 == 0, "mlp2_dw2f: bf16 operands must be 16-B aligned");
  const c10::hip::OptionalHIPGuardMasqueradingAsCUDA guard(dZ2F.device());
  return wf::launch_mlp2_dw2f(bfp(dZ2F), bfp(X), (int)Fp, rows_ptr(rows, B), nrows, bfp(W1), fp(b1), (int)B, (int)nsplit,
                              fp(red), cur_stream());
}

// Fused MLP forward (mlp_fused.hip): both 256-wide hidden layers + head (+ MSE) in one launch.
// Returns false (nothing launched) when the shape is not covered; the caller then runs the
// per-layer GEMMs + head kernel.
bool mlp2_forward(const at::Tensor& X, int64_t Fp, const at::Tensor& W1, const at::Tensor& b1,
                  const at::Tensor& W2, const at::Tensor& b2, const at::Tensor& w3, const at::Tensor& b3,
                  c10::optional<at::Tensor> y, c10::optional<at::Tensor> H1, const at::Tensor& H2,
                  const at::Tensor& pred, c10::optional<at::Tensor> dy, c10::optional<at::Tensor> loss_sum,
                  double dy_scale, int64_t B, c10::optional<at::Tensor> M2,
                  c10::optional<at::Tensor> dw3, c10::optional<at::Tensor> db3, c10::optional<at::Tensor> rows,
                  c10::optional<at::Tensor> red) {
  constexpr int64_t H = 256;
  check_t(X, at::kBFloat16, "X");
  const int64_t nrows = check_x_rows(X, Fp, B, rows);
  check_t(W1, at::kBFloat16, "W1");
  check_extent(W1, H * Fp, "W1");
  check_t(W2, at::kBFloat16, "W2");
  check_extent(W2, H * H, "W2");
  for (const at::Tensor* t : {&b1, &b2, &w3}) {
    check_t(*t, at::kFloat, "bias/w3");
    check_extent(*t, H, "bias/w3");
  }
  check_t(b3, at::kFloat, "b3");
  bf16_t* h1p = opt_ptr<bf16_t>(H1, at::kBFloat16, "H1", B * H);
  check_t(H2, at::kBFloat16, "H2");
  check_extent(H2, B * H, "H2");
  check_t(pred, at::kFloat, "pred");
  check_extent(pred, B, "pred");
  for (const at::Tensor* t : {&X, &W1, &W2, &H2})
    TORCH_CHECK(reinterpret_cast<uintptr_t>(t->data_ptr()) % 16 == 0, "mlp2_forward: bf16 operands must be 16-B aligned");
  const int64_t ny = nrows;  // y is indexed like X
  const c10::hip::OptionalHIPGuardMasqueradingAsCUDA guard(X.device());
  return wf::launch_mlp2_fwd(bfp(X), (int)Fp, bfp(W1), fp(b1), bfp(W2), fp(b2), fp(w3), fp(b3),
                             opt_ptr<float>(y, at::kFloat, "y", ny), h1p, bfp(H2), mask_ptr(M2, B),
                             opt_ptr<float>(dw3, at::kFloat, "dw3", H), opt_ptr<float>(db3, at::kFloat, "db3", 1),
                             fp(pred),
                             opt_ptr<float>(dy, at::kFloat, "dy", B),
                             opt_ptr<float>(loss_sum, at::kFloat, "loss_sum", 1), (float)dy_scale, (int)B,
                             rows_ptr(rows, B), nrows, cur_stream(),
                             opt_ptr<float>(red, at::kFloat, "red", wf::kMlpRedFloats));
}

// head forward + MSE + head weight gradient in one pass over H (elementwise.hip); false = shape
// not covered (the caller runs head_fwd + head_bwd_w)
bool head_fwd_bwd(const at::Tensor& Hm, int64_t ldh, int64_t B, int64_t Hd, const at::Tensor& w, const at::Tensor& b0,
                  const at::Tensor& target, const at::Tensor& pred, const at::Tensor& dy,
                  c10::optional<at::Tensor> loss_sum, double dy_scale, const at::Tensor& dw, c10::optional<at::Tensor> db) {
  check_head_h(Hm, ldh, B, Hd);
  TORCH_CHECK(Hd % 8 == 0 && ldh % 8 == 0, "head: Hd and ldh must be multiples of 8");
  check_t(w, at::kFloat, "w");
  check_extent(w, Hd, "w");
  check_t(b0, at::kFloat, "b0");
  check_t(target, at::kFloat, "target");
  check_extent(target, B, "target");
  check_t(pred, at::kFloat, "pred");
  check_extent(pred, B, "pred");
  check_t(dy, at::kFloat, "dy");
  check_extent(dy, B, "dy");
  check_t(dw, at::kFloat, "dw");
  check_extent(dw, Hd, "dw");
  const c10::hip::OptionalHIPGuardMasqueradingAsCUDA guard(Hm.device());
  return wf::launch_head_fwd_bwd(bfp(Hm), ldh, (int)B, (int)Hd, fp(w), fp(b0), fp(target), fp(pred), fp(dy),
                                 opt_ptr<float>(loss_sum, at::kFloat, "loss_sum", 1), (float)dy_scale, fp(dw),
                                 opt_ptr<float>(db, at::kFloat, "db", 1), cur_stream());
}

void head_bwd_w(const at::Tensor& Hm, int64_t ldh, int64_t B, int64_t Hd, const at::Tensor& dy,
                const at::Tensor& dw, c10::optional<at::Tensor> db) {
  check_head_h(Hm, ldh, B, Hd);
  check_t(dy, at::kFloat, "dy");
  check_extent(dy, B, "dy");
  check_t(dw, at::kFloat, "dw");
  check_extent(dw, Hd, "dw");
  const c10::hip::OptionalHIPGuardMasqueradingAsCUDA guard(Hm.device());
  wf::launch_head_bwd_w(bfp(Hm), ldh, (int)B, (int)Hd, fp(dy), fp(dw),
                        opt_ptr<float>(db, at::kFloat, "db", 1), cur_stream());
}

void head_bwd_x(const at::Tensor& Hm, int64_t ldh, int64_t B, int64_t Hd, const at::Tensor& dy,
                const at::Tensor& w, bool relu_mask, const at::Tensor& dz, int64_t ldz,
                c10::optional<at::Tensor> colsum) {
  check_head_h(Hm, ldh, B, Hd);
  check_t(dy, at::kFloat, "dy");
  check_extent(dy, B, "dy");
  check_t(w, at::kFloat, "w");
  check_extent(w, Hd, "w");
  check_t(dz, at::kBFloat16, "dz");
  check_extent(dz, (B - 1) * ldz + Hd, "dz");
  TORCH_CHECK(ldz % 8 == 0, "head_bwd_x: ldz must be a multiple of 8");
  const c10::hip::OptionalHIPGuardMasqueradingAsCUDA guard(Hm.device());
  wf::launch_head_bwd_x(bfp(Hm), ldh, (int)B, (int)Hd, fp(dy), fp(w), relu_mask ? 1 : 0, bfp(dz),
                        ldz, opt_ptr<float>(colsum, at::kFloat, "colsum", Hd), cur_stream());
}

void loss(int64_t kind, const at::Tensor& pred, const at::Tensor& y, int64_t B, int64_t O,
          double clip, double scale, c10::optional<at::Tensor> loss_sum,
          c10::optional<at::Tensor> dpred, c10::optional<at::Tensor> dpredF,
          c10::optional<at::Tensor> colsum) {
  TORCH_CHECK(kind == 0 || kind == 1, "loss: kind 0 (mse) or 1 (mae_clip)");
  check_t(pred, at::kFloat, "pred");
  check_t(y, at::kFloat, "y");
  check_extent(pred, B * O, "pred");
  check_extent(y, B * O, "y");
  const c10::hip::OptionalHIPGuardMasqueradingAsCUDA guard(pred.device());
  wf::launch_loss((int)kind, fp(pred), fp(y), (int)B, (int)O, (float)clip, (float)scale,
                  opt_ptr<float>(loss_sum, at::kFloat, "loss_sum", 1),
                  opt_ptr<bf16_t>(dpred, at::kBFloat16, "dpred", B * O),
                  opt_ptr<float>(dpredF, at::kFloat, "dpredF", B * O),
                  opt_ptr<float>(colsum, at::kFloat, "colsum", O), cur_stream());
}

void adam(const at::Tensor& p, const at::Tensor& g, const at::Tensor& m, const at::Tensor& v,
          double lr, double b1, double b2, double eps, double wd, double bc1, double bc2,
          double gscale) {
  check_t(p, at::kFloat, "p");
  check_t(g, at::kFloat, "g");
  check_t(m, at::kFloat, "m");
  check_t(v, at::kFloat, "v");
  const int64_t n = p.numel();
  TORCH_CHECK(g.numel() == n && m.numel() == n && v.numel() == n, "adam: size mismatch");
  const c10::hip::OptionalHIPGuardMasqueradingAsCUDA guard(p.device());
  wf::launch_adam(fp(p), fp(g), fp(m), fp(v), n, (float)lr, (float)b1, (float)b2, (float)eps,
                  (float)wd, (float)bc1, (float)bc2, (float)gscale, cur_stream());
}

void adam_dev(const at::Tensor& p, const at::Tensor& g, const at::Tensor& m, const at::Tensor& v,
              const at::Tensor& step, double lr, double b1, double b2, double eps, double wd,
              double gscale, c10::optional<at::Tensor> shadow, bool zero_g,
              c10::optional<at::Tensor> shadow_t, int64_t t_off, int64_t t_rows, int64_t t_cols) {
  check_t(p, at::kFloat, "p");
  check_t(g, at::kFloat, "g");
  check_t(m, at::kFloat, "m");
  check_t(v, at::kFloat, "v");
  check_t(step, at::kFloat, "step");
  check_extent(step, 2, "step");  // [0] = t, [1] = completion ticket
  const int64_t n = p.numel();
  TORCH_CHECK(g.numel() == n && m.numel() == n && v.numel() == n, "adam: size mismatch");
  for (const at::Tensor* t : {&p, &g, &m, &v})
    TORCH_CHECK(reinterpret_cast<uintptr_t>(t->data_ptr()) % 16 == 0, "adam: buffers must be 16-B aligned");
  const c10::hip::OptionalHIPGuardMasqueradingAsCUDA guard(p.device());
  // shadow_t: a transposed bf16 copy of the [t_rows][t_cols] block at element t_off (e.g. the
  // MLP's W2^T, read by mlp2_step128_kernel) written in the same launch
  bf16_t* tdst = nullptr;
  if (shadow_t.has_value()) {
    TORCH_CHECK(t_off >= 0 && t_rows > 0 && t_cols > 0 && t_off + t_rows * t_cols <= n, "adam: shadow_t block outside p");
    tdst = opt_ptr<bf16_t>(shadow_t, at::kBFloat16, "shadow_t", t_rows * t_cols);
  }
  wf::launch_adam_dev(fp(p), fp(g), fp(m), fp(v), n, fp(step), (float)lr, (float)b1, (float)b2,
                      (float)eps, (float)wd, (float)gscale, opt_ptr<bf16_t>(shadow, at::kBFloat16, "shadow", n),
                      zero_g ? 1 : 0, cur_stream(), tdst, (long)t_off, (int)t_rows, (int)t_cols);
}

void sgd(const at::Tensor& p, const at::Tensor& g, const at::Tensor& vel, double lr,
         double momentum, bool nesterov, double gscale) {
  check_t(p, at::kFloat, "p");
  check_t(g, at::kFloat, "g");
  check_t(vel, at::kFloat, "vel");
  const int64_t n = p.numel();
  TORCH_CHECK(g.numel() == n && vel.numel() == n, "sgd: size mismatch");
  const c10::hip::OptionalHIPGuardMasqueradingAsCUDA guard(p.device());
  wf::launch_sgd(fp(p), fp(g), fp(vel), n, (float)lr, (float)momentum, nesterov ? 1 : 0,
                 (float)gscale, cur_stream());
}

void sgd_dev(const at::Tensor& p, const at::Tensor& g, const at::Tensor& vel, const at::Tensor& step, double lr,
             double decay, double momentum, bool nesterov, double gscale, bool zero_g) {
  check_t(p, at::kFloat, "p");
  check_t(g, at::kFloat, "g");
  check_t(vel, at::kFloat, "vel");
  check_t(step, at::kFloat, "step");
  check_extent(step, 2, "step");  // [0] = iterations, [1] = completion ticket
  const int64_t n = p.numel();
  TORCH_CHECK(g.numel() == n && vel.numel() == n, "sgd: size mismatch");
  const c10::hip::OptionalHIPGuardMasqueradingAsCUDA guard(p.device());
  wf::launch_sgd_dev(fp(p), fp(g), fp(vel), n, fp(step), (float)lr, (float)decay, (float)momentum, nesterov ? 1 : 0,
                     (float)gscale, zero_g ? 1 : 0, cur_stream());
}

void cast_bf16(const at::Tensor& src, const at::Tensor& dst) {
  check_t(src, at::kFloat, "src");
  check_t(dst, at::kBFloat16, "dst");
  TORCH_CHECK(dst.numel() >= src.numel(), "cast: dst too small");
  const c10::hip::OptionalHIPGuardMasqueradingAsCUDA guard(src.device());
  wf::launch_cast_bf16(fp(src), bfp(dst), src.numel(), cur_stream());
}

// out[r] = src[idx[r]] (rows of any dtype, contiguous, row size a multiple of 4 B; ids clamped)
void gather_rows(const at::Tensor& src, const at::Tensor& idx, const at::Tensor& out) {
  TORCH_CHECK(src.is_cuda() && idx.is_cuda() && out.is_cuda(), "gather_rows: GPU tensors");
  TORCH_CHECK(src.is_contiguous() && out.is_contiguous() && idx.is_contiguous(), "gather_rows: contiguous tensors");
  TORCH_CHECK(idx.scalar_type() == at::kLong && idx.dim() == 1, "gather_rows: idx int64 [m]");
  TORCH_CHECK(src.scalar_type() == out.scalar_type() && src.dim() >= 1 && out.dim() == src.dim(), "gather_rows: dtype / rank");
  TORCH_CHECK(src.size(0) > 0 && out.size(0) == idx.size(0), "gather_rows: out rows == idx size");
  const int64_t rb = src.numel() / src.size(0) * src.element_size();
  TORCH_CHECK(rb > 0 && rb % 4 == 0 && out.numel() / std::max<int64_t>(out.size(0), 1) * out.element_size() == rb,
              "gather_rows: row bytes must match and be a multiple of 4");
  if (idx.size(0) == 0) return;
  const c10::hip::OptionalHIPGuardMasqueradingAsCUDA guard(src.device());
  wf::launch_gather_rows(src.data_ptr(), reinterpret_cast<const long long*>(idx.data_ptr<int64_t>()), out.data_ptr(), idx.size(0), (int)rb, src.size(0),
                         cur_stream());
}

void transpose_cast_bf16(const at::Tensor& src, int64_t lds, int64_t rows, int64_t cols,
                         const at::Tensor& dst, int64_t ldd) {
  TORCH_CHECK(src.is_cuda() && src.scalar_type() == at::kFloat, "src: fp32 GPU tensor");
  check_t(dst, at::kBFloat16, "dst");
  TORCH_CHECK(lds >= cols && ldd >= rows, "transpose_cast: bad leading dims");
  TORCH_CHECK(src.storage().nbytes() - src.storage_offset() * 4 >= (size_t)(((rows - 1) * lds + cols) * 4),
              "transpose_cast: src too small");
  check_extent(dst, (cols - 1) * ldd + rows, "dst");
  const c10::hip::OptionalHIPGuardMasqueradingAsCUDA guard(src.device());
  wf::launch_transpose_cast_bf16(src.data_ptr<float>(), lds, (int)rows, (int)cols, bfp(dst), ldd,
                                 cur_stream());
}

void im2col1d(const at::Tensor& x, int64_t B, int64_t L, int64_t Cin, int64_t ksz, int64_t Kp,
              const at::Tensor& col) {
  check_t(x, at::kFloat, "x");
  check_t(col, at::kBFloat16, "col");
  const int64_t Lout = L - ksz + 1;
  TORCH_CHECK(Lout > 0 && Kp >= ksz * Cin + 1, "im2col1d: bad shape");
  check_extent(x, B * L * Cin, "x");
  check_extent(col, B * Lout * Kp, "col");
  const c10::hip::OptionalHIPGuardMasqueradingAsCUDA guard(x.device());
  wf::launch_im2col1d(fp(x), (int)B, (int)L, (int)Cin, (int)ksz, (int)Lout, (int)Kp, bfp(col),
                      cur_stream());
}

// ---- fused reference CNN (cnn_fused.hip). dims = [L, C, taps, T, Fp, Kc, O] (models/cnn.py
// CnnLayout; the dense weight has 16 rows, Op = 16).
wf::CnnDims cnn_dims(const std::vector<int64_t>& dims, double drop_p) {
  TORCH_CHECK(dims.size() == 7, "cnn: dims = [L, C, taps, T, Fp, Kc, O]");
  wf::CnnDims d;
  d.L = (int)dims[0]; d.C = (int)dims[1]; d.taps = (int)dims[2]; d.T = (int)dims[3];
  d.Fp = (int)dims[4]; d.Kc = (int)dims[5]; d.O = (int)dims[6];
  d.drop_p = (float)drop_p;
  return d;
}

bool cnn_fused_ok(const std::vector<int64_t>& dims, double drop_p) {
  return wf::cnn_fused_supported(cnn_dims(dims, drop_p));
}

std::vector<int64_t> cnn_part_sizes(int64_t B, const std::vector<int64_t>& dims) {
  auto d = cnn_dims(dims, 0.0);
  long wd = 0, wc = 0, f = 0;
  wf::cnn_part_floats((int)B, d, &wd, &wc, &f);
  return {wd, wc, f};
}

static wf::CnnDims cnn_checked(const std::vector<int64_t>& dims, double drop_p) {
  auto d = cnn_dims(dims, drop_p);
  TORCH_CHECK(wf::cnn_fused_supported(d), "cnn: shape not covered by the fused kernels");
  return d;
}

static int64_t cnn_frag_elems(const wf::CnnDims& d) { return (int64_t)d.T * (d.Fp / 16) * 64 * 4; }

int64_t cnn_small_scratch_floats() { return wf::kCnnSmallScratch; }

// K small-batch CNN training steps (forward, backward, Keras SGD) in ONE persistent launch
// (cnn_small.hip). X [N][48] / Y [N][O] fp32 through rows [K * B] (or contiguous); params / vel
// / step: flat parameters and FlatSGD state; rng: the engine's dropout step counter. False =
// not covered.
bool cnn_small_steps(const at::Tensor& X, const at::Tensor& Y, c10::optional<at::Tensor> rows, int64_t B, int64_t K,
                     std::vector<int64_t> dims, double drop_p, int64_t loss_kind, double clip, double scale,
                     int64_t seed, const at::Tensor& rng, const at::Tensor& params, const at::Tensor& vel,
                     const at::Tensor& step, double lr, double decay, double momentum, bool nesterov, double gscale,
                     c10::optional<at::Tensor> loss_acc, const at::Tensor& scr, const at::Tensor& sync,
                     int64_t filters, c10::optional<at::Tensor> stamps) {
  const wf::CnnDims d = cnn_checked(dims, drop_p);
  TORCH_CHECK(d.L == 48 && d.C == 1 && d.Fp == 112 && d.Kc == 16 && d.T == 36, "cnn_small_steps: the reference layout only");
  TORCH_CHECK(K > 0 && B > 0 && B <= 64, "cnn_small_steps: 0 < B <= 64, K > 0");
  check_t(X, at::kFloat, "X");
  check_t(Y, at::kFloat, "Y");
  int64_t nrows;
  const long long* rp = nullptr;
  if (rows.has_value() && rows->defined()) {
    rp = rows_ptr(rows, K * B);
    nrows = X.numel() / d.L;
    TORCH_CHECK(nrows > 0, "X: empty dataset");
  } else {
    nrows = K * B;
    check_extent(X, nrows * d.L, "X");
  }
  check_extent(Y, nrows * d.O, "Y");
  const int64_t n = (int64_t)d.Fp * d.Kc + 16LL * d.T * d.Fp + 16;
  for (const at::Tensor* t : {&params, &vel}) {
    check_t(*t, at::kFloat, "params/vel");
    check_extent(*t, n, "params/vel");
  }
  check_t(step, at::kFloat, "step");
  TORCH_CHECK(rng.is_cuda() && rng.scalar_type() == at::kLong && rng.numel() >= 1, "rng: int64 GPU counter");
  check_t(scr, at::kFloat, "scr");
  check_extent(scr, wf::kCnnSmallScratch, "scr");
  check_t(sync, at::kInt, "sync");
  check_extent(sync, 4, "sync");
  const c10::hip::OptionalHIPGuardMasqueradingAsCUDA guard(X.device());
  wf::CnnSmallArgs a{};
  a.X = fp(X);
  a.Y = fp(Y);
  a.rows = rp;
  a.nrows = (long)nrows;
  a.B = (int)B;
  a.K = (int)K;
  a.O = d.O;
  a.taps = d.taps;
  a.filters = (int)filters;
  a.drop = drop_p > 0.0 ? 1 : 0;
  a.loss_kind = (int)loss_kind;
  a.keep_scale = drop_p > 0.0 ? (float)(1.0 / (1.0 - drop_p)) : 1.f;
  a.clip = (float)clip;
  a.scale = (float)scale;
  a.seed = (unsigned)seed;
  a.rng = reinterpret_cast<long long*>(rng.data_ptr<int64_t>());
  a.p = fp(params);
  a.vel = fp(vel);
  a.step = fp(step);
  a.lr = (float)lr;
  a.decay = (float)decay;
  a.momentum = (float)momentum;
  a.gscale = (float)gscale;
  a.nesterov = nesterov ? 1 : 0;
  a.loss_acc = opt_ptr<float>(loss_acc, at::kFloat, "loss_acc", 1);
  a.scr = fp(scr);
  a.sync = reinterpret_cast<unsigned*>(sync.data_ptr<int>());
  const char* sl = std::getenv("WELLFLOW_SPIN_LIMIT");  // tests: force the hand-off timeout path
  a.spin_limit = sl != nullptr ? (unsigned)std::strtoul(sl, nullptr, 10) : (1u << 22);
  a.stamps = reinterpret_cast<unsigned long long*>(opt_ptr<int64_t>(stamps, at::kLong, "stamps", 28 * 64 * 16));
  return wf::launch_cnn_small(a, cur_stream());
}

void cnn_pack(const at::Tensor& Wc, const at::Tensor& Wd, const std::vector<int64_t>& dims, const at::Tensor& WcA,
              const at::Tensor& WdF, const at::Tensor& WdB) {
  auto d = cnn_checked(dims, 0.0);
  check_t(Wc, at::kFloat, "Wc");
  check_extent(Wc, (int64_t)d.Fp * d.Kc, "Wc");
  TORCH_CHECK(Wd.is_cuda() && Wd.scalar_type() == at::kFloat && Wd.is_contiguous(), "Wd: contiguous fp32 GPU tensor");
  check_extent(Wd, (int64_t)16 * d.T * d.Fp, "Wd");
  check_t(WcA, at::kBFloat16, "WcA");
  check_extent(WcA, (int64_t)d.Fp * d.Kc, "WcA");
  for (const at::Tensor* t : {&WdF, &WdB}) {
    check_t(*t, at::kBFloat16, "WdF/WdB");
    check_extent(*t, cnn_frag_elems(d), "WdF/WdB");
  }
  const c10::hip::OptionalHIPGuardMasqueradingAsCUDA guard(Wc.device());
  wf::launch_cnn_pack(fp(Wc), Wd.data_ptr<float>(), d, bfp(WcA), bfp(WdF), bfp(WdB), cur_stream());
}

// Keras SGD on the CNN's flat parameters + the bf16 operand images (cnn_pack's output) in one launch
void cnn_sgd_pack(const at::Tensor& p, const at::Tensor& g, const at::Tensor& vel, const at::Tensor& step, double lr,
                  double decay, double momentum, bool nesterov, double gscale, bool zero_g,
                  const std::vector<int64_t>& dims, const at::Tensor& WcA, const at::Tensor& WdF, const at::Tensor& WdB) {
  auto d = cnn_checked(dims, 0.0);
  for (const at::Tensor* t : {&p, &g, &vel}) check_t(*t, at::kFloat, "p/g/vel");
  const int64_t n = p.numel();
  TORCH_CHECK(g.numel() == n && vel.numel() == n, "cnn_sgd_pack: size mismatch");
  TORCH_CHECK(n >= (int64_t)d.Fp * d.Kc + (int64_t)16 * d.T * d.Fp, "cnn_sgd_pack: p shorter than the CNN layout");
  check_t(step, at::kFloat, "step");
  check_extent(step, 2, "step");
  check_t(WcA, at::kBFloat16, "WcA");
  check_extent(WcA, (int64_t)d.Fp * d.Kc, "WcA");
  for (const at::Tensor* t : {&WdF, &WdB}) {
    check_t(*t, at::kBFloat16, "WdF/WdB");
    check_extent(*t, cnn_frag_elems(d), "WdF/WdB");
  }
  const c10::hip::OptionalHIPGuardMasqueradingAsCUDA guard(p.device());
  wf::launch_cnn_sgd_pack(fp(p), fp(g), fp(vel), n, fp(step), (float)lr, (float)decay, (float)momentum, nesterov ? 1 : 0,
                          (float)gscale, zero_g ? 1 : 0, d, bfp(WcA), bfp(WdF), bfp(WdB), cur_stream());
}

static const long long* rng_ptr(const c10::optional<at::Tensor>& rng) {
  if (!rng.has_value() || !rng->defined()) return nullptr;
  TORCH_CHECK(rng->is_cuda() && rng->scalar_type() == at::kLong && rng->numel() >= 1, "rng: GPU int64 tensor");
  return reinterpret_cast<const long long*>(rng->data_ptr<int64_t>());
}

void cnn_forward(const at::Tensor& x, int64_t B, const std::vector<int64_t>& dims, double drop_p, const at::Tensor& WcA,
                 const at::Tensor& WdF, const at::Tensor& bd, c10::optional<at::Tensor> y, c10::optional<at::Tensor> dout,
                 c10::optional<at::Tensor> pred, c10::optional<at::Tensor> part, bool train, int64_t loss_kind,
                 double clip, double scale, int64_t seed, c10::optional<at::Tensor> rng) {
  auto d = cnn_checked(dims, drop_p);
  TORCH_CHECK(B > 0, "cnn_forward: B > 0");
  const int64_t rows = (B + 15) / 16 * 16;
  check_t(x, at::kFloat, "x");
  check_extent(x, B * d.L, "x");
  check_t(WcA, at::kBFloat16, "WcA");
  check_extent(WcA, (int64_t)d.Fp * d.Kc, "WcA");
  check_t(WdF, at::kBFloat16, "WdF");
  check_extent(WdF, cnn_frag_elems(d), "WdF");
  TORCH_CHECK(bd.is_cuda() && bd.scalar_type() == at::kFloat && bd.numel() >= 16, "bd: 16 fp32 values");
  long wd = 0, wc = 0, f = 0;
  wf::cnn_part_floats((int)B, d, &wd, &wc, &f);
  float *yp = nullptr, *dp = nullptr, *pp = nullptr, *part_p = nullptr;
  if (train) {
    TORCH_CHECK(loss_kind == 0 || loss_kind == 1, "cnn_forward: loss 0 (mse) or 1 (mae_clip)");
    yp = opt_ptr<float>(y, at::kFloat, "y", B * d.O);
    dp = opt_ptr<float>(dout, at::kFloat, "dout", rows * 16);
    part_p = opt_ptr<float>(part, at::kFloat, "part", f);
    TORCH_CHECK(yp && dp && part_p, "cnn_forward(train): y, dout and part are required");
  } else {
    pp = opt_ptr<float>(pred, at::kFloat, "pred", rows * 16);
    TORCH_CHECK(pp, "cnn_forward(eval): pred is required");
  }
  const c10::hip::OptionalHIPGuardMasqueradingAsCUDA guard(x.device());
  wf::launch_cnn_forward(fp(x), (int)B, d, bfp(WcA), bfp(WdF), bd.data_ptr<float>(), yp, dp, pp, part_p, train ? 1 : 0,
                         (int)loss_kind, (float)clip, (float)scale, (unsigned)(seed & 0xFFFFFFFF), rng_ptr(rng),
                         cur_stream());
}

void cnn_backward(const at::Tensor& x, int64_t B, const std::vector<int64_t>& dims, double drop_p, const at::Tensor& WcA,
                  const at::Tensor& WdB, const at::Tensor& dout, int64_t seed, c10::optional<at::Tensor> rng,
                  const at::Tensor& part_wd, const at::Tensor& part_wc) {
  auto d = cnn_checked(dims, drop_p);
  TORCH_CHECK(B > 0, "cnn_backward: B > 0");
  const int64_t rows = (B + 15) / 16 * 16;
  check_t(x, at::kFloat, "x");
  check_extent(x, B * d.L, "x");
  check_t(WcA, at::kBFloat16, "WcA");
  check_extent(WcA, (int64_t)d.Fp * d.Kc, "WcA");
  check_t(WdB, at::kBFloat16, "WdB");
  check_extent(WdB, cnn_frag_elems(d), "WdB");
  check_t(dout, at::kFloat, "dout");
  check_extent(dout, rows * 16, "dout");
  long wd = 0, wc = 0, f = 0;
  wf::cnn_part_floats((int)B, d, &wd, &wc, &f);
  check_t(part_wd, at::kFloat, "part_wd");
  check_extent(part_wd, wd, "part_wd");
  check_t(part_wc, at::kFloat, "part_wc");
  check_extent(part_wc, wc, "part_wc");
  const c10::hip::OptionalHIPGuardMasqueradingAsCUDA guard(x.device());
  wf::launch_cnn_backward(fp(x), (int)B, d, bfp(WcA), bfp(WdB), fp(dout), (unsigned)(seed & 0xFFFFFFFF), rng_ptr(rng),
                          fp(part_wd), fp(part_wc), cur_stream());
}

void cnn_reduce(const at::Tensor& part_wd, const at::Tensor& part_wc, const at::Tensor& part_f, int64_t B,
                const std::vector<int64_t>& dims, const at::Tensor& gWc, const at::Tensor& gWd, const at::Tensor& gbd,
                c10::optional<at::Tensor> loss_sum, c10::optional<at::Tensor> rng) {
  auto d = cnn_checked(dims, 0.0);
  long wd = 0, wc = 0, f = 0;
  wf::cnn_part_floats((int)B, d, &wd, &wc, &f);
  check_t(part_wd, at::kFloat, "part_wd");
  check_extent(part_wd, wd, "part_wd");
  check_t(part_wc, at::kFloat, "part_wc");
  check_extent(part_wc, wc, "part_wc");
  check_t(part_f, at::kFloat, "part_f");
  check_extent(part_f, f, "part_f");
  for (const at::Tensor* t : {&gWc, &gWd, &gbd})
    TORCH_CHECK(t->is_cuda() && t->scalar_type() == at::kFloat && t->is_contiguous(), "grads: contiguous fp32 GPU");
  check_extent(gWc, (int64_t)d.Fp * d.Kc, "gWc");
  check_extent(gWd, (int64_t)16 * d.T * d.Fp, "gWd");
  check_extent(gbd, 16, "gbd");
  long long* rp = nullptr;
  if (rng.has_value() && rng->defined()) {
    TORCH_CHECK(rng->is_cuda() && rng->scalar_type() == at::kLong && rng->numel() >= 1, "rng: GPU int64 tensor");
    rp = reinterpret_cast<long long*>(rng->data_ptr<int64_t>());
  }
  const c10::hip::OptionalHIPGuardMasqueradingAsCUDA guard(part_wd.device());
  wf::launch_cnn_reduce(fp(part_wd), fp(part_wc), fp(part_f), (int)B, d, gWc.data_ptr<float>(), gWd.data_ptr<float>(),
                        gbd.data_ptr<float>(), opt_ptr<float>(loss_sum, at::kFloat, "loss_sum", 1), rp, cur_stream());
}

// True when the HIP objects are a WF_DIAG build (WELLFLOW_DIAG_BUILD=1): timing-only switches
// and A/B variants are live. bench.py refuses to time such a build.
bool diag_build() { return wf::dbg_mask() != (1 << 21); }

// Every binding runs behind this wrapper: a kernel launch that the runtime rejected (bad grid,
// missing code object, invalid resource) raises here instead of failing silently.
template <auto F>
struct Checked;
template <class R, class... A, R (*F)(A...)>
struct Checked<F> {
  static R call(A... a) {
    (void)hipGetLastError();  // errors of earlier, foreign launches are not ours to report
    if constexpr (std::is_void_v<R>) {
      F(a...);
      check();
    } else {
      R r = F(a...);
      check();
      return r;
    }
  }
  static void check() {
    const hipError_t e = hipGetLastError();
    TORCH_CHECK(e == hipSuccess, "wellflow kernel launch failed: ", hipGetErrorString(e));
  }
};

}  // namespace

#define WF_DEF(name) m.def(#name, &Checked<&name>::call)

PYBIND11_MODULE(_C, m) {
  m.doc() = "wellflow HIP kernel library (gfx950)";
  WF_DEF(gemm);
  WF_DEF(mlp2_forward);
  WF_DEF(mlp2_backward);
  WF_DEF(mlp2_dw2);
  WF_DEF(mlp2_reduce);
  WF_DEF(mlp2_step);
  WF_DEF(mlp2_dw2f);
  WF_DEF(mlp_small_steps);
  WF_DEF(mlp_small_scratch_floats);
  WF_DEF(cnn_small_steps);
  WF_DEF(cnn_small_scratch_floats);
  WF_DEF(lstm_pack_x);
  WF_DEF(lstm_pack_x_win);
  WF_DEF(lstm_forward);
  WF_DEF(lstm_forward_persistent);
  WF_DEF(lstm_backward);
  WF_DEF(lstm_backward_dw);
  WF_DEF(lstm_pack_weights);
  WF_DEF(lstm_adam_pack);
  WF_DEF(head_fwd);
  WF_DEF(head_bwd_w);
  WF_DEF(head_fwd_bwd);
  WF_DEF(head_bwd_x);
  WF_DEF(loss);
  WF_DEF(adam);
  WF_DEF(adam_dev);
  WF_DEF(sgd);
  WF_DEF(sgd_dev);
  WF_DEF(cast_bf16);
  WF_DEF(gather_rows);
  WF_DEF(transpose_cast_bf16);
  WF_DEF(im2col1d);
  // host-only queries (no launch; callable without a GPU)
  m.def("diag_build", &diag_build);
  m.def("cnn_fused_ok", &cnn_fused_ok);
  m.def("cnn_part_sizes", &cnn_part_sizes);
  WF_DEF(cnn_pack);
  WF_DEF(cnn_sgd_pack);
  WF_DEF(cnn_forward);
  WF_DEF(cnn_backward);
  WF_DEF(cnn_reduce);
}
