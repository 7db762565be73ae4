// wellflow — host-side launcher declarations for the HIP kernel library.
// Pure HIP/C++ (no torch headers): binding.cpp validates tensors and calls these.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace wf {

typedef unsigned short bf16_t;

struct GemmEpilogue {
  float* outF = nullptr;         // fp32 output (also the beta / atomic target)
  bf16_t* outH = nullptr;        // bf16 output
  long ldo = 0;
  const float* bias = nullptr;   // [N]
  const bf16_t* mask = nullptr;  // zero the output where mask <= 0 (ReLU backward)
  long ldm = 0;
  float mask_scale = 1.f;        // multiply kept values (inverted-dropout backward)
  float* colsum = nullptr;       // [N] += column sums of the final output (bias grads)
  float alpha = 1.f, beta = 0.f;
  int act = 0;                   // 0 linear, 1 relu
  int atomic = 0;                // split-K: atomicAdd alpha*acc into outF
  float drop_p = 0.f;            // inverted dropout after the activation
  unsigned long long seed = 0;
  const long long* seed_dev = nullptr;  // optional device step counter mixed into the seed (graph replays)
  int stage_ok = 0;              // host-verified: bf16 output/mask tiles may go through LDS
  int big_tile = 0;              // MN x MN split-K weight gradient: 1 = 256x128 8-wave tile, 2 = 128x288
  float* slab = nullptr;         // split-K partial slab (256x288 dW tile, ldo == N): plain stores of
  long slab_cap = 0;             // each split's tile, then one reduce adds the splits into outF
};

void launch_gemm(const bf16_t* A, long lda, int a_mn, const bf16_t* B, long ldb, int b_mn, int M,
                 int N, int K, int ksplit, const GemmEpilogue& e, hipStream_t s,
                 bool glds_ok = false);

// ---- LSTM (single layer, batch-first input, seq-to-one regression) ----
struct LstmDims {
  int B, T, F, KX, H;  // G = 4H, KA = KX + H
  int fwd_variant = 0;  // per-step forward tile: 6 = 256x256 glds ring, else 128x128 (lstm.hip)
  int bwd_variant = 0;  // per-step backward tile: 8 = 128x128 8-wave glds ring, else 128x128
  int xcd_map = 1;      // 1: XCD-aware tile remap (default), 0: identity (diagnostics)
  int nt = 1;           // non-temporal hints on the read-once/write-once state streams
  int dbg = 0;          // persistent-kernel diagnostics (WELLFLOW_PF_DBG), masked with
                        // dbg_mask(): production builds keep only the test hook bit 21
  int row_off = 0;      // persistent kernels: first batch row of this sub-batch launch
  unsigned spin_limit = 0;  // persistent hand-off spin bound (0 = built-in; tests shrink it)
};
// WELLFLOW_PF_DBG bits the HIP objects were built to honour (persistent_guard.h kDbgMask):
// 1 << 21 (the force-timeout TEST hook) in production builds, everything in WF_DIAG builds
int dbg_mask();
// starts / idx (optional): x is a [nrows][F] row table, batch row b = the window at row starts[idx[b]]
void launch_lstm_pack_x(const float* x, bf16_t* XH, LstmDims d, hipStream_t s, bool full = true,
                        const long* starts = nullptr, const long* idx = nullptr, long nwin = 0, long nrows = 0);
// Cst: the cell-state history c_t (bf16, FN layout, slab t + 1; slab 0 = c_{-1} = 0) the backward
// reads; the per-step forward carries c in fp32 in the in-place state slab cf32 ([Bp][H], FN).
void launch_lstm_fwd_step(int t, bf16_t* XH, const bf16_t* Wp, bf16_t* Cst, bf16_t* S, float* cf32,
                          LstmDims d, hipStream_t s);
// All T forward steps in ONE persistent launch per sub-batch (lstm_persistent.hip). `sync`
// must hold lstm_persistent_sync_total(row blocks) words (16 + 16 * (B / 32 + 1) + 64 always
// suffices): a per-launch block at the start (zeroed by the launcher) and the 64-word
// completion STAT block at the end (persistent_guard.h; running totals, never cleared by a
// launch). Returns 1 launched, 0 shape / device cannot host it (nothing launched),
// < 0 = -(hipError_t) of a failed launch.
int lstm_persistent_sync_words(int row_blocks);
long lstm_persistent_sync_total(int row_blocks);
int launch_lstm_fwd_persistent(bf16_t* XH, const bf16_t* Wp, bf16_t* Cst, bf16_t* S, unsigned* sync,
                                long sync_words, LstmDims d, hipStream_t s);
// Backward steps T-2 .. 0 in ONE persistent launch per sub-batch (lstm_persistent_bwd.hip),
// after step T-1 ran (launch_lstm_bwd_step(T-1, ...)). Same `sync` contract and return
// codes as the forward.
int launch_lstm_bwd_persistent(const bf16_t* WhhT, const bf16_t* Cst, const bf16_t* S, bf16_t* DG,
                                const float* dcarry, unsigned* sync, long sync_words, LstmDims d,
                                hipStream_t s);
void launch_lstm_bwd_step(int t, const bf16_t* WhhT, const bf16_t* Cst, const bf16_t* S,
                          bf16_t* DG, float* dcarry, const float* dy, const float* w_out,
                          LstmDims d, hipStream_t s);
void launch_lstm_pack_weights(const float* W, bf16_t* Wp, bf16_t* WhhT, LstmDims d,
                              hipStream_t s);

// ---- fused MLP forward (mlp_fused.hip): F (<= 64, padded to Fp % 8 == 0) -> 256 -> 256 -> 1,
// ReLU, bias, linear head, optional MSE (y, dy = dy_scale * (pred - y), loss_sum += (pred - y)^2).
// Writes H1, H2 ([B][256] bf16: the backward's saved activations) and pred. Returns false
// (nothing launched) for shapes it does not cover.
// red (optional): the spread-reduction scratch of the 8-wave training kernels (kMlpRed* below);
// when given, their batch sums land there and launch_mlp2_reduce adds them to the gradients.
bool launch_mlp2_fwd(const bf16_t* X, int Fp, const bf16_t* W1, const float* b1, const bf16_t* W2, const float* b2,
                     const float* w3, const float* b3, const float* y, bf16_t* H1, bf16_t* H2, unsigned* M2,
                     float* dw3, float* db3, float* pred, float* dy, float* loss_sum, float dy_scale, int B,
                     const long long* rows, long nrows, hipStream_t s, float* red = nullptr);
// Mask mode (M2 != nullptr; needs y, dw3, db3): H2 is NOT written — only its ReLU bitmask M2
// ([B][8] u32, bit u of row r = word 8r + u / 32, bit u % 32) — and dw3 += H2^T dy,
// db3 += sum dy are accumulated by the forward itself.
// ---- fused MLP backward (mlp_fused.hip), everything but the dW2 GEMM: from H1, H2
// ([B][256] bf16), dy, w3 / W2 and X: dZ2 ([B][256] bf16, dW2's operand), db1, db2, dw3, db3
// and — when dW1 != nullptr — dW1 ([256][Fp], Fp <= 32) (fp32, accumulated with atomics);
// with dW1 == nullptr dZ1 ([B][256] bf16) is written for a separate dW1 GEMM instead.
// M2 != nullptr: ReLU mask of layer 2 from the forward's bitmask (H2 unused) and no dw3 / db3.
bool launch_mlp2_bwd(const bf16_t* H1, const bf16_t* H2, const unsigned* M2, const float* dy, const float* w3, const bf16_t* W2,
                     const bf16_t* X, int Fp, bf16_t* dZ1, bf16_t* dZ2, float* dW1, float* db1, float* db2,
                     float* dw3, float* db3, int B, const bf16_t* W1, const float* b1, const long long* rows,
                     long nrows, hipStream_t s, float* red = nullptr);
// H1 == nullptr: recompute H1 from X with W1 / b1 (needs dW1 != nullptr, i.e. Fp <= 32);
// rows != nullptr: dataset row indices of X (and y in the forward) per batch row.
// dW2 += dZ2^T relu(X W1^T + b1) with H1 recomputed per chunk (B % 64 == 0, Fp <= 32)
bool launch_mlp2_dw2(const bf16_t* dZ2, const bf16_t* X, int Fp, const long long* rows, long nrows, const bf16_t* W1,
                     const float* b1, int B, int nsplit, float* dW2, hipStream_t s, float* red = nullptr);
// Spread-reduction scratch (floats): kMlpRedCopies rows of kMlpRedRow slots — [loss, db3,
// dw3[256], db1[256], db2[256]] (slots from kMlpRedDW1 on are unused: every dW1 goes out as the
// per-workgroup rows below) — then kMlpRedCopies2 copies of dW2 [256 x 256].
// Zero-initialised once; mlp2_reduce sums every copy into the gradients and zeroes it again.
constexpr int kMlpRedCopies = 64, kMlpRedCopies2 = 4, kMlpRedRow = 9216;
constexpr int kMlpRedLoss = 0, kMlpRedDb3 = 1, kMlpRedDw3 = 2, kMlpRedDb1 = 258, kMlpRedDb2 = 514, kMlpRedDW1 = 770;
// then the backward's per-workgroup dW1 rows: [kMlpRedSlabRows][kMlpRedSlabRow] (plain stores,
// summed over the launch's grid by the reduce: dW1 is 4096 values per workgroup, too many
// atomic wave-instructions per CU even spread over copies)
constexpr int kMlpRedSlabRows = 256, kMlpRedSlabRow = 256 * 64;  // Fp <= 64
constexpr long kMlpRedSlabOff = (long)kMlpRedCopies * kMlpRedRow + (long)kMlpRedCopies2 * 65536;
// then the dW2 rows of the fragment-layout dW2 kernel: [kMlpRedSlab2Rows][256 x 256] (plain
// stores of each workgroup's partial tile, summed by the reduce: 8M float atomics per step
// were the dW2 kernel's bottleneck)
constexpr int kMlpRedSlab2Rows = 256;
constexpr long kMlpRedSlab2Off = kMlpRedSlabOff + (long)kMlpRedSlabRows * kMlpRedSlabRow;
constexpr long kMlpRedFloats = kMlpRedSlab2Off + (long)kMlpRedSlab2Rows * 65536;
// grid of the 8-wave training kernels for a batch (one workgroup per CU at most): the rows of
// the dW1 slab the reduce sums
int mlp2_train_grid(int B);
// K small-batch MLP training steps (forward, backward, Adam) in one persistent launch of 16
// workgroups (mlp_small.hip): hidden (256, 256), Fp <= 32, 32 <= B <= 256, B % 32 == 0.
// rows: dataset row ids [K * B] (nullptr: step k reads rows k B .. k B + B - 1 of X / Y).
// p / m / v / step: the flat fp32 parameters and FlatAdam state (updated in place);
// shadow / w2t: the engine's bf16 images written at the end; loss_acc += each step's loss sum.
// scr: kMlpSmallScratch floats; sync: 4 words zeroed once ([0] counter, [1] exits, [2] sticky
// error, [3] completed launches).
constexpr int kMlpSmallScratch = 49728 + 65536;
struct MlpSmallArgs {
  const bf16_t* X;
  const float* Y;
  const long long* rows;
  long nrows;
  int Fp, B, K;
  float* p;
  float* m;
  float* v;
  float* step;
  float lr, b1, b2, eps, wd, dy_scale, clip;
  bf16_t* shadow;
  bf16_t* w2t;
  float* loss_acc;
  float* scr;
  unsigned* sync;
  unsigned spin_limit;
  long oW1, ob1, oW2, ob2, ow3, ob3;
  unsigned long long* stamps;  // diagnostics (tools/small_timeline.py): [16][64 steps][16] s_memrealtime, or null
};
bool launch_mlp_small(const MlpSmallArgs& a, hipStream_t s);
// K small-batch training steps of the reference CNN (conv 13 taps -> 36 steps x filters, ReLU,
// dropout, dense -> O outputs, Keras SGD) in one persistent launch of ceil(filters / 4)
// workgroups (cnn_small.hip); B <= 64. X [N][48] / Y [N][O] fp32 read through rows [K * B]
// (nullptr: contiguous); p / vel / step: the flat parameters and FlatSGD state; rng: the
// engine's dropout step counter (+= K); scr: kCnnSmallScratch floats; sync: 4 words, zeroed once.
constexpr int kCnnSmallScratch = 2 * 28 * 64 * 16 * 2 + 2 * 64 * 16 * 2;
struct CnnSmallArgs {
  const float* X;
  const float* Y;
  const long long* rows;
  long nrows;
  int B, K, O, taps, filters, drop, loss_kind;
  float keep_scale, clip, scale;
  unsigned seed;
  long long* rng;
  float* p;
  float* vel;
  float* step;
  float lr, decay, momentum, gscale;
  int nesterov;
  float* loss_acc;
  float* scr;
  unsigned* sync;
  unsigned spin_limit;
  unsigned long long* stamps;  // diagnostics (tools/small_timeline.py --cnn): [G][64 steps][16], or null
};
bool launch_cnn_small(const CnnSmallArgs& a, hipStream_t s);
bool mlp_bwd8();  // the 8-wave backward is selected (WELLFLOW_MLP_BWD8, default on)
void launch_mlp2_reduce(float* red, int Fp, int B, float* loss_sum, float* db3, float* dw3, float* db1, float* db2,
                        float* dW1, float* dW2, hipStream_t s, int dw2_rows = 0);
// dw2_rows: dW2 slab rows (launch_mlp2_dw2f's return value) summed into dW2 as well
// The training step's forward + backward in ONE launch (mlp_step.hip): from X (rows), y, the
// bf16 weights and fp32 biases / head — dZ2 ([B][256] bf16, mlp2_dw2's operand), pred (optional)
// and every batch sum except dW2 (loss, db3, dw3, db1, db2, dW1) into the spread scratch `red`,
// which launch_mlp2_reduce then adds to the gradients. Fp <= 32; false = not covered.
bool launch_mlp2_step(const bf16_t* X, int Fp, const bf16_t* W1, const float* b1, const bf16_t* W2, const float* b2,
                      const float* w3, const float* b3, const float* y, float dy_scale, int B, const long long* rows,
                      long nrows, bf16_t* dZ2, float* pred, float* red, bool dz_frag, hipStream_t s,
                      const bf16_t* W2T = nullptr, float clip = 0.f);
// clip > 0: the clipped-MAE loss min(|p - y|, clip) instead of MSE (dy_scale = grad_scale then)
// W2T (optional, [256][256] bf16 = W2 transposed): with dz_frag, the 128-row-pass kernel that
// streams both weight images (mlp2_step128_kernel) instead of holding W2^T in registers.
// dz_frag: dZ2 is written in the fragment layout of launch_mlp2_dw2f (B % 64 == 0) instead of
// [B][256]: fragment (S, b) of rows 32S .. 32S + 31 x units 16b .. 16b + 15 at element
// (S * 16 + b) * 512, lane (l15, g) = 16 B = rows 32S + 8g .. + 7 of unit 16b + l15.
// dW2 from that layout without LDS (mlp_step.hip mlp2_dw2f_kernel) into the scratch's dW2 copies.
// Returns the dW2 slab rows written (> 0), or 0 = not covered (nothing launched).
int launch_mlp2_dw2f(const bf16_t* dZ2F, const bf16_t* X, int Fp, const long long* rows, long nrows, const bf16_t* W1,
                     const float* b1, int B, int nsplit, float* red, hipStream_t s);

// ---- fused reference CNN (cnn_fused.hip): Conv1D(C -> Fp, width taps / C) + ReLU + dropout ->
// Dense(T * Fp -> O) -> loss, cnn.py:110-118. Flat layout = models/cnn.py CnnLayout:
// Wc [Fp][Kc] (conv bias in column taps), Wd [Op = 16][T * Fp], bd [16].
struct CnnDims {
  int L, C, taps, T, Fp, Kc, O;  // input steps, channels, taps (= width * C), output steps, ...
  float drop_p;                   // 0 or 0.5 (one hash bit per element)
};
bool cnn_fused_supported(const CnnDims& d);
int cnn_fwd_grid(int B);
int cnn_bwd_chunks(int B);
// partial-buffer floats for a batch of B (dense-weight, conv-weight and forward partials)
long cnn_part_floats(int B, const CnnDims& d, long* wd, long* wc, long* f);
// bf16 operand images from the fp32 flat weights: WcA [Fp][Kc], WdF / WdB [T][Fp/16][64][4]
// Keras SGD over the CNN's flat parameters + the bf16 operand images of launch_cnn_pack, one launch
void launch_cnn_sgd_pack(float* p, float* g, float* vel, long n, float* step, float lr, float decay, float momentum,
                         int nesterov, float gscale, int zero_g, const CnnDims& d, bf16_t* WcA, bf16_t* WdF,
                         bf16_t* WdB, hipStream_t s);
void launch_cnn_pack(const float* Wc, const float* Wd, const CnnDims& d, bf16_t* WcA, bf16_t* WdF, bf16_t* WdB,
                     hipStream_t s);
// train = 1: dropout + loss; dout [rows >= B rounded up to 16][16] = scale * dloss/dpred, part
// [cnn_fwd_grid(B)][32] (dense-bias gradient, loss). train = 0: pred [rows][16].
void launch_cnn_forward(const float* x, int B, const CnnDims& d, const bf16_t* WcA, const bf16_t* WdF,
                        const float* bd, const float* y, float* dout, float* pred, float* part, int train,
                        int loss_kind, float clip, float scale, unsigned seed, const long long* rng, hipStream_t s);
void launch_cnn_backward(const float* x, int B, const CnnDims& d, const bf16_t* WcA, const bf16_t* WdB,
                         const float* dout, unsigned seed, const long long* rng, float* part_wd, float* part_wc,
                         hipStream_t s);
// grads += the partials; loss_sum += the loss; rng[0] += 1 (the dropout step counter)
void launch_cnn_reduce(const float* part_wd, const float* part_wc, const float* part_f, int B, const CnnDims& d,
                       float* gWc, float* gWd, float* gbd, float* loss_sum, long long* rng, hipStream_t s);

// ---- regression head (N = 1) and losses ----
void launch_head_fwd(const bf16_t* Hm, long ldh, int B, int Hd, const float* w, const float* b0,
                     const float* target, float* pred, float* dy, float* loss_sum, float dy_scale,
                     hipStream_t s);
// head forward + MSE + dw / db in one pass (Hd = 8 * a power of two <= 512); false = not covered
bool launch_head_fwd_bwd(const bf16_t* Hm, long ldh, int B, int Hd, const float* w, const float* b0,
                         const float* target, float* pred, float* dy, float* loss_sum, float dy_scale, float* dw,
                         float* db, hipStream_t s);
void launch_head_bwd_w(const bf16_t* Hm, long ldh, int B, int Hd, const float* dy, float* dw,
                       float* db, hipStream_t s);
void launch_head_bwd_x(const bf16_t* Hm, long ldh, int B, int Hd, const float* dy, const float* w,
                       int relu_mask, bf16_t* dz, long ldz, float* colsum, hipStream_t s);
// kind 0 = MSE, 1 = clipped MAE (reference mae_clip)
void launch_loss(int kind, const float* pred, const float* y, int B, int O, float clip, float scale,
                 float* loss_sum, bf16_t* dpred, float* dpredF, float* colsum, hipStream_t s);

// ---- optimizers and casts over flat fp32 buffers ----
void launch_adam(float* p, const float* g, float* m, float* v, long n, float lr, float b1,
                 float b2, float eps, float wd, float bc1, float bc2, float gscale, hipStream_t s);
// Adam over the LSTM's flat parameters + its bf16 compute copies Wp / WhhT (lstm_pack_weights) in one launch
void launch_lstm_adam_pack(float* p, float* g, float* m, float* v, long n, float* step, float lr, float b1, float b2,
                           float eps, float wd, float gscale, int zero_g, int KX, int H, bf16_t* Wp, bf16_t* WhhT,
                           hipStream_t s);
void launch_adam_dev(float* p, float* g, float* m, float* v, long n, float* step, float lr,
                     float b1, float b2, float eps, float wd, float gscale, bf16_t* shadow, int zero_g,
                     hipStream_t s, bf16_t* tdst = nullptr, long t_off = 0, int t_rows = 0, int t_cols = 0);
void launch_sgd(float* p, const float* g, float* vel, long n, float lr, float momentum,
                int nesterov, float gscale, hipStream_t s);
void launch_sgd_dev(float* p, float* g, float* vel, long n, float* step, float lr, float decay, float momentum,
                    int nesterov, float gscale, int zero_g, hipStream_t s);
void launch_cast_bf16(const float* src, bf16_t* dst, long n, hipStream_t s);
// dst[r] = src[clamp(idx[r], 0, nsrc - 1)], rows of row_bytes (multiple of 4) bytes
void launch_gather_rows(const void* src, const long long* idx, void* dst, long m, int row_bytes, long nsrc,
                        hipStream_t s);
void launch_transpose_cast_bf16(const float* src, long lds, int rows, int cols, bf16_t* dst,
                                long ldd, hipStream_t s);
void launch_im2col1d(const float* x, int B, int L, int Cin, int ksz, int Lout, int Kp,
                     bf16_t* col, hipStream_t s);

}  // namespace wf
