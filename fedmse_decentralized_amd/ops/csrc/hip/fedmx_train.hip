// Persistent fused local training of (Shrink-)Autoencoder clients on gfx950.
//
// Replaces ClientTrainer.run (src/Trainer/client_trainer.py:360-419): for every
// selected client, E epochs of mini-batch training (forward, MSE + shrink loss,
// optional FedProx proximal term, backward, Adam), a validation pass per epoch,
// patience-based early stopping and the best-model snapshot — all inside ONE
// launch with no host round trip.  Grid = one 256-thread workgroup (4 wave64,
// one per SIMD) per client; clients train concurrently on different CUs.
//
// Work split inside a workgroup (wave w = 0..3):
//   * W1a columns d in [32w, 32w+32) and W4a rows d in [32w, 32w+32) are
//     OWNED by wave w: their Adam state (param, m, v, FedProx anchor) lives in
//     that wave's VGPRs for the whole launch, in the MFMA accumulator layout of
//     their gradient tiles, so the optimizer is fused into the gradient
//     epilogue.  Layer 1 is K-split by the same column block (partial sums
//     reduced through LDS, barrier #1); layer 4 output / dY rows by the same
//     row block; dH3 = W4a^T dY is K-split again (barrier #2).
//   * The small layers W2a [16x32] / W3a [32x16] are two 16x16 gradient tiles
//     each; wave 0/1 own the two W3a tiles, wave 2/3 the two W2a tiles (Adam
//     state in registers).  Their forward/backward-data products are computed
//     redundantly by every wave from one shared LDS master, which owners
//     update after barrier #2 and readers re-read after barrier #1 of the next
//     step, so no extra synchronisation is needed.
//   * W1 never goes through LDS during training: its owned block is kept in
//     the MFMA A-operand layout, which is both what the layer-1 product reads
//     and what the dW1^T = X^T dH1 product writes (dH1 is produced directly in
//     the batch-major layout by swapping the operands of W2a^T dZ, and X is
//     streamed in both layouts).
//   * Batches of any size: a batch is processed as column tiles ("chunks") of
//     16 rows; weight gradients accumulate in the MFMA accumulators over the
//     chunks and Adam runs once per batch.  Per chunk: 2 workgroup barriers;
//     per validation chunk: 1.
//   * The layer-1 product of the next chunk is issued right after the W1 Adam
//     update, ahead of the W4 / small-tile updates, so the MFMA pipe overlaps
//     that optimizer VALU work.
//   * Global memory is touched only to stream the batches (prefetched one
//     chunk ahead) and, through LDS staging with coalesced 16-byte accesses, to
//     load / store the client state and the best-validation snapshot.
// All products run on v_mfma_f32_16x16x4_f32 (exact fp32).  Padded batch
// columns and padded features are masked out of the loss and every gradient.
#include "fedmx_train_common.h"

// (Rounds 1-5 measured, and removed, these variants of this kernel's step:
// sched_group_barrier MFMA/VALU interleavings (+9 %) and the compiler's own
// schedule (+2.5 %) against iglp_opt(0); dW4's products after barrier #2
// (+0.5 %); W4's Adam after dH1 or after the next layer-1 issue (+2.5 / +2 %);
// separately rounded Adam (+3 %); the timing-only ablations that located the
// optimizer's share of the step.  Source in git history, numbers in
// scripts/ab_variants.py and profiles/r2_*.)

namespace fedmx {

// LDS plan (floats); total < 160 KiB -> one workgroup per CU.
constexpr int L_W1 = HP * S_W1;          // 4224  master (snapshots / write-back only)
constexpr int L_W4 = DP * S_W4;          // 4608  shared, row block per wave
constexpr int L_W2 = ZP * S_W2;          // 576   shared master
constexpr int L_W3 = HP * S_W3;          // 640   shared master
constexpr int L_RED = 4 * 2 * 64 * 4;    // 2048  one partial-sum exchange buffer
constexpr int L_T32 = 32 * S_T;          // 640   [32 features][batch] transpose tile
constexpr int L_T16 = 16 * S_T;          // 320
constexpr int L_SCR = 3 * L_T32 + 2 * L_T16;  // 2560 per wave
constexpr int L_TOTAL = L_W1 + L_W4 + L_W2 + L_W3 + 3 * L_RED + 4 * L_SCR + 64;

// Per-lane state of the owned parameter blocks of wave w, lane (c = l & 15, g = l >> 4):
//   q1[t][v][r] = W1a[16t+c][32w+16v+4g+r]   (MFMA A-operand layout of layer 1:
//                 register s of tile (t,v) is the A value of k-step s, so the
//                 forward consumes the registers directly, and dW1^T tiles come
//                 out of the MFMA in exactly this layout)
//   q4[v][t][r] = W4a[32w+16v+4g+r][16t+c]   (D layout: A operand of dH3 = W4a^T dY)
// plus the owned small tile o[r]:
//   w<2 : W3a[16w+4g+r][c]                   w>=2: W2a[4g+r][16(w-2)+c]
struct Slab {
  float q1[2][2][4];
  float q4[2][2][4];
  float o[4];
};

struct Lane {
  float* w1;   // sW1 + c*S_W1 + 32w + 4g      (+ 16t*S_W1 + 16v; 4 consecutive r)
  float* w4;   // sW4 + (32w+4g)*S_W4 + c      (+ (16v+r)*S_W4 + 16t)
  float* own;  // owned small tile base (stride own_stride per r)
  int own_stride;
};

__device__ __forceinline__ void w1_to_lds(const Slab& o, const Lane& L) {
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int v = 0; v < 2; ++v)
      lds_write4(L.w1 + 16 * t * S_W1 + 16 * v, f32x4{o.q1[t][v][0], o.q1[t][v][1], o.q1[t][v][2], o.q1[t][v][3]});
}

__device__ __forceinline__ void w4_to_lds(const Slab& o, const Lane& L) {
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int v = 0; v < 2; ++v) L.w4[(16 * v + r) * S_W4 + 16 * t] = o.q4[v][t][r];
}

__device__ __forceinline__ void own_to_lds(const Slab& o, const Lane& L) {
#pragma unroll
  for (int r = 0; r < 4; ++r) L.own[r * L.own_stride] = o.o[r];
}

__device__ __forceinline__ void w4own_to_lds(const Slab& o, const Lane& L) {
  w4_to_lds(o, L);
  own_to_lds(o, L);
}

__device__ __forceinline__ void slab_to_lds(const Slab& o, const Lane& L) {
  w1_to_lds(o, L);
  w4own_to_lds(o, L);
}

__device__ __forceinline__ void lds_to_slab(Slab& o, const Lane& L) {
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int v = 0; v < 2; ++v) {
      const f32x4 q = lds_read4(L.w1 + 16 * t * S_W1 + 16 * v);
#pragma unroll
      for (int r = 0; r < 4; ++r) o.q1[t][v][r] = q[r];
    }
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int v = 0; v < 2; ++v) o.q4[v][t][r] = L.w4[(16 * v + r) * S_W4 + 16 * t];
#pragma unroll
  for (int r = 0; r < 4; ++r) o.o[r] = L.own[r * L.own_stride];
}

__device__ __forceinline__ void scale_slab(Slab& o, float f) {
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int v = 0; v < 2; ++v)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        o.q1[t][v][r] *= f;
        o.q4[t][v][r] *= f;
      }
#pragma unroll
  for (int r = 0; r < 4; ++r) o.o[r] *= f;
}

// 16x16 product summed over the two 16-wide halves of the hidden axis
// (k-steps (t, s)): L2 (W2a H1) and dZ (W3a^T dH3).  These are the dependent
// chains on the step's critical path (one accumulator: 7-8 x 40-cycle MFMA
// latency); SPLIT sums each half in its own accumulator and adds the two, so
// the chain is ~half as long.  SPLIT_CHAINS is a mask over the
// instantiations (bit 0 plain, bit 1 FedProx, bit 2 batch > 12), shared with
// fedmx_train_hw.hip (whose bit 2 has no instantiation here) so that the two
// kernels sum in the same order.  r5h A/B: plain -0.7 %, batch 64 -0.3 %,
// FedProx +1.2 % with split chains (profiles/r5_train_kernel_ab.md).
template <bool CP, bool SPLIT>
__device__ __forceinline__ f32x4 chain2(f32x4 a0, f32x4 a1, f32x4 b0, f32x4 b1) {
  f32x4 x = zero4();
  if (SPLIT) {
    f32x4 y = zero4();
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      x = mfma16(a0[s], b0[s], x);
      if (s < (CP ? 3 : 4)) y = mfma16(a1[s], b1[s], y);
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) x[r] = x[r] + y[r];
  } else {
#pragma unroll
    for (int s = 0; s < 4; ++s) x = mfma16(a0[s], b0[s], x);
#pragma unroll
    for (int s = 0; s < (CP ? 3 : 4); ++s) x = mfma16(a1[s], b1[s], x);
  }
  return x;
}

// One batch column tile ("chunk") of up to 16 rows, in the two register
// layouts the step needs:
//   f0/f1: feature-major B operand  X[b=c][32w+4g+s] / X[b=c][32w+16+4g+s]
//   b0/b1: batch-major A operand    X[b=4g+s][32w+c] / X[b=4g+s][32w+16+c]
// Rows past the chunk are zero; the bias column (DP-1) is 1 on real rows.
struct XChunk {
  f32x4 f0, f1, b0, b1;
};

// ONE: every batch is a single 16-row tile (batch <= 16, the reference's 12):
// the per-chunk bookkeeping folds away and each step is one basic block the
// scheduler can interleave (W4's optimizer VALU under the backward MFMAs).
// CP (compact, implies ONE): batch <= 12, hidden <= 27, latent <= 7 — the
// internal hidden / latent / batch orders of fedmx_train_common.h put every
// padded slot into whole k-steps, which the products over hidden (7 of 8
// k-steps), latent (2 of 4) and batch (3 of 4) skip: 95 instead of 116
// MFMAs per wave and training step, and shorter dependent chains.
template <bool PROX, bool ONE, bool CP>
__global__ __launch_bounds__(256, 1) void train_kernel(const TrainArgs A) {
  static_assert(ONE || !CP, "compact order needs single-tile batches");
  constexpr int KB = CP ? 3 : 4;   // k-steps of products over the batch
  constexpr int KZ = CP ? 2 : 4;   // k-steps of products over the latent axis
  constexpr bool SPLIT = (SPLIT_CHAINS & (PROX ? 2 : 1)) != 0;
  __shared__ __attribute__((aligned(16))) float lds[L_TOTAL];
  const int w = threadIdx.x >> 6;
  const int lane = threadIdx.x & 63;
  const int c = lane & 15;
  const int g = lane >> 4;
  float* const sW1 = lds;
  float* const sW4 = sW1 + L_W1;
  float* const sW2 = sW4 + L_W4;
  float* const sW3 = sW2 + L_W2;
  float* const sRedH1 = sW3 + L_W3;               // two buffers (parity)
  float* const sRedDH3 = sRedH1 + 2 * L_RED;
  float* const scr = sRedDH3 + L_RED + w * L_SCR;
  float* const sH1T = scr;               // H1^T                    [32][S_T]
  float* const sT0 = sH1T + L_T32;       // dY^T own rows, then dH3^T
  float* const sT1 = sT0 + L_T32;        // H3^T
  float* const sZT = sT1 + L_T32;        // Z^T (with bias row)     [16][S_T]
  float* const sDZT = sZT + L_T16;       // dZ^T                    [16][S_T]
  double* const sLoss = reinterpret_cast<double*>(sRedDH3 + L_RED + 4 * L_SCR);  // [4][4] doubles

  Lane L;
  L.w1 = sW1 + c * S_W1 + 32 * w + 4 * g;
  L.w4 = sW4 + (32 * w + 4 * g) * S_W4 + c;
  if (w < 2) {
    L.own = sW3 + (16 * w + 4 * g) * S_W3 + c;
    L.own_stride = S_W3;
  } else {
    L.own = sW2 + 4 * g * S_W2 + 16 * (w - 2) + c;
    L.own_stride = S_W2;
  }
  const float* const a4p = sW4 + (32 * w + c) * S_W4 + 4 * g;  // + 16v*S_W4 + 16t
  const float* const a2p = sW2 + c * S_W2 + 4 * g;             // + 16t
  const float* const a3p = sW3 + c * S_W3 + 4 * g;             // + 16t*S_W3
  const float* const d2p = sW2 + 4 * g * S_W2 + c;             // W2a[4g+r][16t+c]  (+ r*S_W2 + 16t)
  const float* const d3p = sW3 + 4 * g * S_W3 + c;             // W3a[16t+4g+r][c]  (+ (16t+r)*S_W3)
  const int tw = 4 * g * S_T + c;   // transpose write: [feature 4g+r (+16v)][b=c]
  const int tr = c * S_T + 4 * g;   // transpose read : [feature c (+16v)][b=4g..4g+3]
  float* const redw = sRedDH3 + (w * 2) * 256 + lane * 4;  // own dH3 partial slot (+ t*256)

  const int kslot = blockIdx.x;
  const int cid = A.client_idx[kslot];
  float* const Pg = A.params + (size_t)cid * P_PAD;
  float* const Mg = A.adam_m + (size_t)cid * P_PAD;
  float* const Vg = A.adam_v + (size_t)cid * P_PAD;
  float* const Bg = A.best + (size_t)cid * P_PAD;
  const int d_in = A.d_in, hidden = A.hidden, latent = A.latent;

  // ---- load client state: global -> LDS masters -> owned registers ----------
  STAMP(true, 28);
  Slab P, M, V, AN;
  global_to_masters_o<CP>(Mg, sW1, sW4, sW2, sW3);
  __syncthreads();
  lds_to_slab(M, L);
  __syncthreads();
  global_to_masters_o<CP>(Vg, sW1, sW4, sW2, sW3);
  __syncthreads();
  lds_to_slab(V, L);
  __syncthreads();
  // moment scales of the scaled-moment Adam (identity otherwise)
  const float c1 = 1.f - A.beta1, c2 = 1.f - A.beta2;
  if (ADAM_SCALED) {
    scale_slab(M, adam_moment_in_scale(A.beta1));
    scale_slab(V, adam_moment_in_scale(A.beta2));
  }
  if (PROX) {
    global_to_masters_o<CP>(A.anchor + (size_t)cid * P_PAD, sW1, sW4, sW2, sW3);
    __syncthreads();
    lds_to_slab(AN, L);
    __syncthreads();
  }
  global_to_masters_o<CP>(Pg, sW1, sW4, sW2, sW3);
  __syncthreads();
  lds_to_slab(P, L);   // W2/W3/W4 masters stay live; W1 lives in registers only
  STAMP(true, 29);

  const int B = A.batch;
  const float* const Xtr = A.train_x + (size_t)A.train_off[cid] * DP;
  const int n_tr = (int)(A.train_off[cid + 1] - A.train_off[cid]);
  const float* const Xva = A.valid_x + (size_t)A.valid_off[cid] * DP;
  const int n_va = (int)(A.valid_off[cid + 1] - A.valid_off[cid]);
  const int nb = (n_tr + B - 1) / B;
  const int nvb = (n_va + B - 1) / B;
  int step = A.adam_step[cid];
  int parity = 0;
  const bool bias_lane = (w == 3 && g == 3);  // feature-major: X column DP-1 (= 32*3 + 16 + 4*3 + 3)
  const bool bias_col = (w == 3 && c == 15);  // batch-major:   X column DP-1 (= 32*3 + 16 + 15), tile 1
  const int xcol = 32 * w + 4 * g;
  const float lam = A.lambda;
  const float inv_d = 1.0f / (float)d_in;
  // hidden / latent positions of this lane's D-layout registers (16t + 4g + r,
  // 4g + r) and of its batch-major column (16t + c): real / bias flags
  bool hreal_d[2][4], hbias_d[2][4], zreal_d[4], zbias_d[4], hreal_c[2];
#pragma unroll
  for (int t = 0; t < 2; ++t) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int j = hslot_of_pos<CP>(16 * t + 4 * g + r);
      hreal_d[t][r] = j < hidden;
      hbias_d[t][r] = j == h_bias_slot<CP>();
    }
    hreal_c[t] = hslot_of_pos<CP>(16 * t + c) < hidden;
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int j = zslot_of_pos<CP>(4 * g + r);
    zreal_d[r] = j < latent;
    zbias_d[r] = j == z_bias_slot<CP>();
  }
  // batch rows of this lane's tile column c and batch-major rows 4g + r (-1: padding)
  const int brow_c = batch_row_of_col<CP>(c);
  int brow_b[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) brow_b[r] = batch_row_of_col<CP>(4 * g + r);
  bool stamp_fwd = false;
  (void)stamp_fwd;

  // rows [row0, row0 + bc) of X, bc in 1..16.  Branch-free prefetch: tile
  // columns / rows past the chunk read row0 (always valid) and keep that
  // duplicated data: every product that sums over the batch meets them with an
  // exactly zero gradient (dY is scaled by 0 there, so dH3, dZ and dH1 are 0
  // too) and the loss masks them, so they never need zeroing.  The bias input
  // (feature DP-1) is set by finalize_chunk when the chunk is consumed, so
  // issuing the loads never waits.
  auto load_chunk = [&](const float* X, int row0, int bc, XChunk& x) {
    const float* src = X + (size_t)(row0 + ((unsigned)brow_c < (unsigned)bc ? brow_c : 0)) * DP + xcol;
    x.f0 = *reinterpret_cast<const f32x4*>(src);
    x.f1 = *reinterpret_cast<const f32x4*>(src + 16);
    const float* bsrc = X + (size_t)row0 * DP + 32 * w + c;
#pragma unroll
    for (int r = 0; r < (CP ? 3 : 4); ++r) {   // CP: row quad 3 is padding, never read
      const int rr = ((unsigned)brow_b[r] < (unsigned)bc) ? brow_b[r] : 0;
      x.b0[r] = bsrc[(size_t)rr * DP];
      x.b1[r] = bsrc[(size_t)rr * DP + 16];
    }
    if (CP) {
      x.b0[3] = 0.f;
      x.b1[3] = 0.f;
    }
  };
  auto finalize_chunk = [&](int bc, XChunk& x) {
    (void)bc;
#pragma unroll
    for (int r = 0; r < (CP ? 3 : 4); ++r)
      if (bias_col) x.b1[r] = 1.f;
    if (bias_lane) x.f1[3] = 1.f;
  };

  // Layer-1 partial product over this wave's 32 input columns, straight from
  // the owned registers (no LDS traffic for W1).
  auto l1_partial = [&](const XChunk& x, f32x4& acc0, f32x4& acc1) {
    acc0 = zero4();
    acc1 = zero4();
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      acc0 = mfma16(P.q1[0][0][j], x.f0[j], acc0);
      acc1 = mfma16(P.q1[1][0][j], x.f0[j], acc1);
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      acc0 = mfma16(P.q1[0][1][j], x.f1[j], acc0);
      acc1 = mfma16(P.q1[1][1][j], x.f1[j], acc1);
    }
  };

  // Rest of the forward of one chunk: layer-1 K reduction through LDS
  // (barrier #1), layers 2-3 (redundant per wave), layer 4 on own rows.  Adds
  // this lane's loss share (MSE of its own 32 features; shrink term on wave 0 /
  // lane group 0), normalised by the whole batch's row count bt.  Validation
  // keeps one tile per batch (no packing across batch boundaries): the loss
  // sums then follow the reference's per-batch order closely enough that the
  // patience decisions match it (a packed variant flipped a near-tie).
  auto forward_rest = [&](const f32x4& acc0, const f32x4& acc1, const XChunk& x, int bc, float inv_bt,
                          f32x4 (&h1)[2], f32x4& z, f32x4& zb, f32x4 (&h3)[2], f32x4 (&y)[2], float& norm_c,
                          double& lacc) {
    float* red = sRedH1 + parity * L_RED;
    const bool sf = stamp_fwd;
    lds_write4(red + (w * 2 + 0) * 256 + lane * 4, acc0);
    lds_write4(red + (w * 2 + 1) * 256 + lane * 4, acc1);
    STAMP(sf, 1);
    __syncthreads();  // barrier #1
    STAMP(sf, 2);
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      f32x4 s = lds_read4(red + t * 256 + lane * 4);
#pragma unroll
      for (int ww = 1; ww < 4; ++ww) {
        const f32x4 o = lds_read4(red + (ww * 2 + t) * 256 + lane * 4);
#pragma unroll
        for (int r = 0; r < 4; ++r) s[r] = s[r] + o[r];
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float vv = relu(s[r]);
        if (hbias_d[t][r]) vv = 1.f;
        s[r] = vv;
      }
      h1[t] = s;
    }
    parity ^= 1;
    z = chain2<CP, SPLIT>(lds_read4(a2p), lds_read4(a2p + 16), h1[0], h1[1]);
    zb = z;
#pragma unroll
    for (int r = 0; r < 4; ++r)
      if (zbias_d[r]) zb[r] = 1.f;
    {
      f32x4 acc0 = zero4(), acc1 = zero4();
      const f32x4 a0 = lds_read4(a3p);
      const f32x4 a1 = lds_read4(a3p + 16 * S_W3);
#pragma unroll
      for (int s = 0; s < KZ; ++s) {
        acc0 = mfma16(a0[s], zb[s], acc0);
        acc1 = mfma16(a1[s], zb[s], acc1);
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float v0 = relu(acc0[r]), v1 = relu(acc1[r]);
        if (hbias_d[0][r]) v0 = 1.f;
        if (hbias_d[1][r]) v1 = 1.f;
        acc0[r] = v0;
        acc1[r] = v1;
      }
      h3[0] = acc0;
      h3[1] = acc1;
    }
    {
      f32x4 acc0 = zero4(), acc1 = zero4();
      const f32x4 a00 = lds_read4(a4p);
      const f32x4 a01 = lds_read4(a4p + 16);
      const f32x4 a10 = lds_read4(a4p + 16 * S_W4);
      const f32x4 a11 = lds_read4(a4p + 16 * S_W4 + 16);
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        acc0 = mfma16(a00[s], h3[0][s], acc0);
        acc1 = mfma16(a10[s], h3[0][s], acc1);
      }
#pragma unroll
      for (int s = 0; s < (CP ? 3 : 4); ++s) {
        acc0 = mfma16(a01[s], h3[1][s], acc0);
        acc1 = mfma16(a11[s], h3[1][s], acc1);
      }
      y[0] = acc0;
      y[1] = acc1;
    }
    float sq = 0.f;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      // padded features: Y = 0 (zero W4 rows) and X = 0; only the bias
      // input (feature DP-1, X = 1) is masked
      const float d0 = y[0][r] - x.f0[r];
      const float d1 = (bias_lane && r == 3) ? 0.f : y[1][r] - x.f1[r];
      sq += d0 * d0 + d1 * d1;
    }
    const bool col_ok = (unsigned)brow_c < (unsigned)bc;
    sq = col_ok ? sq : 0.f;
    float nz = 0.f;
#pragma unroll
    for (int r = 0; r < 4; ++r) nz += zreal_d[r] ? z[r] * z[r] : 0.f;
    nz = sum_lane_groups(nz);
    norm_c = __builtin_amdgcn_sqrtf(nz);
    float contrib = sq * (inv_bt * inv_d);
    if (w == 0 && g == 0 && col_ok) contrib += lam * norm_c * inv_bt;
    lacc += (double)contrib;
  };

  // Whole forward of one validation chunk by this wave alone (see the
  // validation pass): L1 as four K-block partials (wave-order sum), L2/L3 as
  // in forward_rest, L4 for all 128 rows, loss shares per K-block.
  auto valid_chunk = [&](const float* X, int row0, int bc, float inv_bt, double& lacc) {
    // the masters are loop-invariant here; keep their reads inside the loop
    // (hoisting ~40 b128 operand reads out of it would spill the Adam slabs)
    asm volatile("" ::: "memory");
    const bool ok = (unsigned)brow_c < (unsigned)bc;
    const float* src = X + (size_t)(row0 + (ok ? brow_c : 0)) * DP + 4 * g;
    f32x4 xf[4][2];
#pragma unroll
    for (int b = 0; b < 4; ++b)
#pragma unroll
      for (int v = 0; v < 2; ++v) {
        const f32x4 q = *reinterpret_cast<const f32x4*>(src + 32 * b + 16 * v);
#pragma unroll
        for (int r = 0; r < 4; ++r) xf[b][v][r] = q[r];
      }
    if (g == 3) xf[3][1][3] = 1.f;   // bias column DP-1
    f32x4 h1[2];
    {
      // K-block partials one after another, each added to the running sum as
      // soon as it is complete: ((p0 + p1) + p2) + p3 with two live chains
      f32x4 sum0 = zero4(), sum1 = zero4();
#pragma unroll
      for (int b = 0; b < 4; ++b) {
        f32x4 p0 = zero4(), p1 = zero4();
#pragma unroll
        for (int v = 0; v < 2; ++v) {
          const f32x4 a0 = lds_read4(sW1 + c * S_W1 + 32 * b + 16 * v + 4 * g);
          const f32x4 a1 = lds_read4(sW1 + (16 + c) * S_W1 + 32 * b + 16 * v + 4 * g);
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            p0 = mfma16(a0[r], xf[b][v][r], p0);
            p1 = mfma16(a1[r], xf[b][v][r], p1);
          }
        }
        if (b == 0) {
          sum0 = p0;
          sum1 = p1;
        } else {
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            sum0[r] = sum0[r] + p0[r];
            sum1[r] = sum1[r] + p1[r];
          }
        }
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float v0 = relu(sum0[r]), v1 = relu(sum1[r]);
        if (hbias_d[0][r]) v0 = 1.f;
        if (hbias_d[1][r]) v1 = 1.f;
        sum0[r] = v0;
        sum1[r] = v1;
      }
      h1[0] = sum0;
      h1[1] = sum1;
    }
    const f32x4 z = chain2<CP, SPLIT>(lds_read4(a2p), lds_read4(a2p + 16), h1[0], h1[1]);
    f32x4 zb = z;
#pragma unroll
    for (int r = 0; r < 4; ++r)
      if (zbias_d[r]) zb[r] = 1.f;
    f32x4 h3[2];
    {
      f32x4 acc0 = zero4(), acc1 = zero4();
      const f32x4 a0 = lds_read4(a3p);
      const f32x4 a1 = lds_read4(a3p + 16 * S_W3);
#pragma unroll
      for (int s = 0; s < KZ; ++s) {
        acc0 = mfma16(a0[s], zb[s], acc0);
        acc1 = mfma16(a1[s], zb[s], acc1);
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float v0 = relu(acc0[r]), v1 = relu(acc1[r]);
        if (hbias_d[0][r]) v0 = 1.f;
        if (hbias_d[1][r]) v1 = 1.f;
        acc0[r] = v0;
        acc1[r] = v1;
      }
      h3[0] = acc0;
      h3[1] = acc1;
    }
    float nz = 0.f;
#pragma unroll
    for (int r = 0; r < 4; ++r) nz += zreal_d[r] ? z[r] * z[r] : 0.f;
    nz = sum_lane_groups(nz);
    const float norm_v = __builtin_amdgcn_sqrtf(nz);
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      f32x4 acc0 = zero4(), acc1 = zero4();
      const float* ap = sW4 + (32 * b + c) * S_W4 + 4 * g;
      const f32x4 a00 = lds_read4(ap);
      const f32x4 a01 = lds_read4(ap + 16);
      const f32x4 a10 = lds_read4(ap + 16 * S_W4);
      const f32x4 a11 = lds_read4(ap + 16 * S_W4 + 16);
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        acc0 = mfma16(a00[s], h3[0][s], acc0);
        acc1 = mfma16(a10[s], h3[0][s], acc1);
      }
#pragma unroll
      for (int s = 0; s < (CP ? 3 : 4); ++s) {
        acc0 = mfma16(a01[s], h3[1][s], acc0);
        acc1 = mfma16(a11[s], h3[1][s], acc1);
      }
      float sq = 0.f;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float d0 = acc0[r] - xf[b][0][r];
        const float d1 = (b == 3 && g == 3 && r == 3) ? 0.f : acc1[r] - xf[b][1][r];
        sq += d0 * d0 + d1 * d1;
      }
      sq = ok ? sq : 0.f;
      float contrib = sq * (inv_bt * inv_d);
      if (b == 0 && g == 0 && ok) contrib += lam * norm_v * inv_bt;
      lacc += (double)contrib;
    }
  };

  AdamStep K;
  K.one_m_b1 = 1.f - A.beta1;
  K.b2 = A.beta2;
  K.one_m_b2 = 1.f - A.beta2;
  K.eps = A.eps;
  K.two_mu = 2.f * A.mu;
  K.b1 = A.beta1;
  // beta^step as running products (python: 1 - beta ** step)
  double b1pow = pow((double)A.beta1, (double)step);
  double b2pow = pow((double)A.beta2, (double)step);
  const AdamScaledInit KI = adam_scaled_init(A.lr, A.beta1, A.beta2, A.eps);

  double min_valid = __builtin_huge_val();
  int worse = 0, ep_run = 0, best_ep = -1;

  // the step's 1/bt and dY scale 2/(bt d_in): bt is B except on an epoch's
  // last batch, so both are formed once here instead of two IEEE division
  // sequences per chunk (opaque to LLVM, which would otherwise fold the
  // per-chunk select back into one division of the selected divisor)
  const int bt_last = nb > 0 ? n_tr - (nb - 1) * B : B;
  float inv_b_full = 1.0f / (float)B, inv_b_last = 1.0f / (float)bt_last;
  float scale_full = 2.0f / (float)(B * d_in), scale_last = 2.0f / (float)(bt_last * d_in);
  asm volatile("" : "+v"(inv_b_full), "+v"(inv_b_last), "+v"(scale_full), "+v"(scale_last));
  for (int ep = 0; ep < A.epochs; ++ep) {
    double acc_tr = 0.0;
    // The epoch is a sequence of chunks (batch bi, column tile ch).  The next
    // chunk's rows are prefetched one chunk ahead, and its layer-1 partial is
    // issued at the end of the current chunk (after the Adam update of W1 when
    // the current chunk closes a batch), where it overlaps the remaining
    // optimizer work.
    int bi = 0, ch = 0;
    XChunk cur, nxt;
    f32x4 l1a = zero4(), l1b = zero4();
    if (nb > 0) {
      load_chunk(Xtr, 0, min(16, min(B, n_tr)), cur);
      finalize_chunk(min(16, min(B, n_tr)), cur);
      l1_partial(cur, l1a, l1b);
    }
    f32x4 G1[2][2], G4[2][2], Go;
    while (bi < nb) {
      const int row_b = bi * B;
      const int bt = min(B, n_tr - row_b);
      const int nch = ONE ? 1 : (bt + 15) >> 4;
      const int bc = ONE ? bt : min(16, bt - 16 * ch);
      const bool last = ONE || (ch == nch - 1);
      // next chunk position
      const int bi_n = last ? bi + 1 : bi;
      const int ch_n = last ? 0 : ch + 1;
      const bool has_next = bi_n < nb;
      const int row_n = bi_n * B + 16 * ch_n;
      const int bc_n = has_next ? min(16, min(B, n_tr - bi_n * B) - 16 * ch_n) : 0;
      const bool full_b = bi + 1 < nb;
      const float inv_bt = full_b ? inv_b_full : inv_b_last;
      if (ch == 0) {
        // bias corrections of the Adam step this batch closes (python:
        // 1 - beta ** step), computed at the batch start, off the critical path
        b1pow *= (double)A.beta1;
        b2pow *= (double)A.beta2;
        adam_step_scalars(K, KI, A.lr, b1pow, b2pow);
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
          for (int v = 0; v < 2; ++v) {
            G1[t][v] = zero4();
            G4[v][t] = zero4();
          }
        Go = zero4();
      }
      f32x4 h1[2], z, zb, h3[2], y[2];
      float norm_c;
      const bool stamp_on = (ep == 0 && bi == STAMP_STEP && ch == 0);
      STAMP(stamp_on, 0);
      stamp_fwd = FEDMX_STAMPS && stamp_on;
      forward_rest(l1a, l1b, cur, bc, inv_bt, h1, z, zb, h3, y, norm_c, acc_tr);
      STAMP(stamp_on, 3);
      if (has_next) load_chunk(Xtr, row_n, bc_n, nxt);  // prefetch

      // current W2a / W3a (all tiles, D layout) for the backward-data products;
      // owners only rewrite the masters after the batch's last barrier #2.
      float q2[2][4], q3[2][4];
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          q2[t][r] = d2p[r * S_W2 + 16 * t];
          q3[t][r] = d3p[(16 * t + r) * S_W3];
        }

      // ---- dY (masked, feature-major) and the transposes feeding dW4
      const bool col_ok = (unsigned)brow_c < (unsigned)bc;
      const float scale = col_ok ? (full_b ? scale_full : scale_last) : 0.f;
      f32x4 dy[2];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        dy[0][r] = (y[0][r] - cur.f0[r]) * scale;
        dy[1][r] = (bias_lane && r == 3) ? 0.f : (y[1][r] - cur.f1[r]) * scale;
        sT0[tw + r * S_T] = dy[0][r];
        sT0[tw + (16 + r) * S_T] = dy[1][r];
        sT1[tw + r * S_T] = h3[0][r];
        sT1[tw + (16 + r) * S_T] = h3[1][r];
      }
      // ---- dH3 partial = W4a(own rows)^T dY(own rows)   (pre-update W4)
      {
        f32x4 acc0 = zero4(), acc1 = zero4();
#pragma unroll
        for (int v = 0; v < 2; ++v)
#pragma unroll
          for (int s = 0; s < 4; ++s) {
            acc0 = mfma16(P.q4[v][0][s], dy[v][s], acc0);
            acc1 = mfma16(P.q4[v][1][s], dy[v][s], acc1);
          }
        lds_write4(redw, acc0);
        lds_write4(redw + 256, acc1);
      }
      // ---- stage H1^T, Z^T (read after barrier #2: no wave-level ordering needed)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        sH1T[tw + r * S_T] = h1[0][r];
        sH1T[tw + (16 + r) * S_T] = h1[1][r];
        sZT[tw + r * S_T] = zb[r];
      }
      STAMP(stamp_on, 4);
      wave_sync();
      // ---- dW4 (own rows) accumulated over the batch's chunks.  Operands are
      // read here (sT0 is reused for dH3^T below).
      const f32x4 w4a0 = lds_read4(sT0 + tr);
      const f32x4 w4a1 = lds_read4(sT0 + tr + 16 * S_T);
      const f32x4 w4b0 = lds_read4(sT1 + tr);
      const f32x4 w4b1 = lds_read4(sT1 + tr + 16 * S_T);
#pragma unroll
      for (int s = 0; s < KB; ++s) {
        G4[0][0] = mfma16(w4a0[s], w4b0[s], G4[0][0]);
        G4[0][1] = mfma16(w4a0[s], w4b1[s], G4[0][1]);
        G4[1][0] = mfma16(w4a1[s], w4b0[s], G4[1][0]);
        G4[1][1] = mfma16(w4a1[s], w4b1[s], G4[1][1]);
      }
      STAMP(stamp_on, 5);
      STAMP(stamp_on, 6);
      __syncthreads();  // barrier #2: dH3 partials of all waves visible
      STAMP(stamp_on, 7);
      f32x4 dh3[2];
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        f32x4 s = lds_read4(sRedDH3 + t * 256 + lane * 4);
#pragma unroll
        for (int ww = 1; ww < 4; ++ww) {
          const f32x4 o = lds_read4(sRedDH3 + (ww * 2 + t) * 256 + lane * 4);
#pragma unroll
          for (int r = 0; r < 4; ++r) s[r] = s[r] + o[r];
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          s[r] = (hreal_d[t][r] && h3[t][r] > 0.f) ? s[r] : 0.f;
        }
        dh3[t] = s;
      }
      float prox_acc = 0.f;  // sum (p - anchor)^2 of owned params (pre-update)
      // W4's Adam update + publish (its rows are read back by this wave only,
      // by the next layer-4 product).  W4 is not read again this step (its
      // dH3 product ran before barrier #2); here its VALU work overlaps the
      // backward MFMAs.
      if (last) {
        ++step;
#pragma unroll
        for (int v = 0; v < 2; ++v)
#pragma unroll
          for (int t = 0; t < 2; ++t)
            adam_update<PROX>(P.q4[v][t], M.q4[v][t], V.q4[v][t], AN.q4[v][t], G4[v][t], K, prox_acc);
        w4_to_lds(P, L);
      }
      // dH3^T for the owned dW3 tile (dY^T reads are done).  Written by every
      // wave (own scratch) so the step stays one basic block for the scheduler.
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) sT0[tw + (16 * t + r) * S_T] = dh3[t][r];
      // ---- dZ = W3a^T dH3 (pre-update W3, every wave), + shrink-loss gradient
      //      lambda/B * z / ||z|| (0 where ||z|| == 0)
      f32x4 dz = chain2<CP, SPLIT>(f32x4{q3[0][0], q3[0][1], q3[0][2], q3[0][3]},
                            f32x4{q3[1][0], q3[1][1], q3[1][2], q3[1][3]}, dh3[0], dh3[1]);
      const float shr_raw = lam * __builtin_amdgcn_rcpf((float)bt * norm_c);
      const float shr = (col_ok && norm_c > 0.f) ? shr_raw : 0.f;
#pragma unroll
      for (int r = 0; r < 4; ++r) dz[r] = zreal_d[r] ? dz[r] + shr * z[r] : 0.f;
#pragma unroll
      for (int r = 0; r < 4; ++r) sDZT[tw + r * S_T] = dz[r];
      // ---- dH1 in the batch-major layout, D[b=4g+r][h=16t+c] = sum_z dZ[b][z] W2a[z][h]
      //      (A = dZ^T D tile as is, B = W2a D layout), ReLU mask from H1^T
      //      read in the same layout; this is directly dW1's B operand.
      f32x4 dh1b[2], h1b[2];
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        h1b[t] = lds_read4(sH1T + tr + 16 * t * S_T);
        f32x4 acc = zero4();
#pragma unroll
        for (int s = 0; s < KZ; ++s) acc = mfma16(dz[s], q2[t][s], acc);
#pragma unroll
        for (int r = 0; r < 4; ++r) acc[r] = (hreal_c[t] && h1b[t][r] > 0.f) ? acc[r] : 0.f;
        dh1b[t] = acc;
      }
      STAMP(stamp_on, 8);
      // ---- dW1^T (own columns) = X^T dH1: D[d=4g+r][h=c] lands in the q1 layout
#pragma unroll
      for (int s = 0; s < KB; ++s) {
        G1[0][0] = mfma16(cur.b0[s], dh1b[0][s], G1[0][0]);
        G1[0][1] = mfma16(cur.b1[s], dh1b[0][s], G1[0][1]);
        G1[1][0] = mfma16(cur.b0[s], dh1b[1][s], G1[1][0]);
        G1[1][1] = mfma16(cur.b1[s], dh1b[1][s], G1[1][1]);
      }
      wave_sync();
      // ---- owned small tile: w<2 -> dW3 tile (h-block w) = dH3^T Z ;
      //                        w>=2 -> dW2 tile (h-block w-2) = dZ^T H1
      {
        const f32x4 a = lds_read4(w < 2 ? sT0 + tr + 16 * w * S_T : sDZT + tr);
        const f32x4 bz = lds_read4(sZT + tr);
        const f32x4 b = (w < 2) ? bz : ((w == 2) ? h1b[0] : h1b[1]);
#pragma unroll
        for (int s = 0; s < KB; ++s) Go = mfma16(a[s], b[s], Go);
      }
      STAMP(stamp_on, 9);
      if (last) {
        // W1 first: the next chunk's layer-1 product waits on it
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
          for (int v = 0; v < 2; ++v)
            adam_update<PROX>(P.q1[t][v], M.q1[t][v], V.q1[t][v], AN.q1[t][v], G1[t][v], K, prox_acc);
        STAMP(stamp_on, 10);
        // (after an epoch's last batch this works on a stale tile; the result
        // is unused and the product stays branch-free)
        finalize_chunk(bc_n, nxt);
        l1_partial(nxt, l1a, l1b);
        adam_update<PROX>(P.o, M.o, V.o, AN.o, Go, K, prox_acc);
        if (PROX) acc_tr += (double)A.mu * (double)prox_acc;
        // publish the owned small tile (read by every wave after barrier #1)
        own_to_lds(P, L);
        // Everything from barrier #2 to here is one basic block (ONE): the
        // scheduler interleaves the optimizer / mask VALU work into the MFMA
        // gaps (one wave per SIMD co-issues ~6 VALU per 16x16x4 MFMA) instead
        // of running the two streams back to back (iglp_opt(0): 1.211 vs
        // 1.231 ms with the compiler's schedule per 5-client x 5-epoch launch)
        if (ONE) __builtin_amdgcn_iglp_opt(0);
      } else {
        finalize_chunk(bc_n, nxt);
        l1_partial(nxt, l1a, l1b);
      }
      STAMP(stamp_on, 11);
      cur = nxt;
      bi = bi_n;
      ch = ch_n;
    }

    // ---- validation pass (eval mode, no grad).  The waves split the batches
    // (wave w: batches w, w+4, ...) and each runs a whole forward from the
    // LDS masters: no cross-wave reduction, no barrier per batch.  Layer 1 is
    // still summed as the training step's four K-block partials in wave
    // order and each K-block's loss share is formed as there, so every
    // per-lane fp32 loss contribution is bitwise the one the training-step
    // forward would produce.
    STAMP(ep == 0, 14);
    w1_to_lds(P, L);   // W1 master (also the source of a best-validation snapshot)
    __syncthreads();   // every wave's owned rows / tiles published
    double acc_va = 0.0;
    for (int vb = w; vb < nvb; vb += 4) {
      const int row0 = vb * B;
      const int bt = min(B, n_va - row0);
      const float inv_bt = 1.0f / (float)bt;
      for (int c0 = 0; c0 < bt; c0 += 16) {
        const int bc = min(16, bt - c0);
        STAMP(ep == 0 && vb == w && c0 == 0, 16);
        valid_chunk(Xva, row0 + c0, bc, inv_bt, acc_va);
        STAMP(ep == 0 && vb == w && c0 == 0, 17);
      }
    }
    STAMP(ep == 0, 15);
    STAMP(ep == 0, 12);
    double prox_now = 0.0;
    if (PROX) {
      float pr = 0.f;
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
          for (int v = 0; v < 2; ++v) {
            const float d1 = P.q1[t][v][r] - AN.q1[t][v][r];
            const float d4 = P.q4[v][t][r] - AN.q4[v][t][r];
            pr += d1 * d1 + d4 * d4;
          }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float d = P.o[r] - AN.o[r];
        pr += d * d;
      }
      prox_now = (double)pr;
    }
    // ---- epoch-end reduction (fixed order over waves -> identical decision everywhere)
    {
      const double s0 = wave_sum_d(acc_tr);
      const double s1 = wave_sum_d(acc_va);
      const double s2 = wave_sum_d(prox_now);
      if (lane == 0) {
        sLoss[w * 4 + 0] = s0;
        sLoss[w * 4 + 1] = s1;
        sLoss[w * 4 + 2] = s2;
      }
    }
    __syncthreads();
    const double tr_sum = sLoss[0] + sLoss[4] + sLoss[8] + sLoss[12];
    const double va_sum = sLoss[1] + sLoss[5] + sLoss[9] + sLoss[13];
    const double px_sum = sLoss[2] + sLoss[6] + sLoss[10] + sLoss[14];
    const double train_loss = nb > 0 ? tr_sum / nb : __builtin_nan("");
    double valid_loss = nvb > 0 ? va_sum / nvb : __builtin_nan("");
    if (PROX) valid_loss += (double)A.mu * px_sum;
    if (threadIdx.x == 0) {
      double* trk = A.tracking + ((size_t)kslot * A.epochs + ep) * 2;
      trk[0] = train_loss;
      trk[1] = valid_loss;
    }
    ep_run = ep + 1;
    if (valid_loss < min_valid) {
      min_valid = valid_loss;
      best_ep = ep;
      worse = 0;
      masters_to_global_o<CP>(Bg, sW1, sW4, sW2, sW3);  // save_model(): best-validation snapshot
    } else {
      ++worse;
    }
    __syncthreads();  // sLoss reuse / masters stable for the snapshot copy
    STAMP(ep == 0, 13);
    if (worse >= A.patience && worse > 0) break;
  }

  STAMP(true, 30);
  // ---- write back: params (masters), then m and v through the same staging
  w1_to_lds(P, L);
  __syncthreads();
  masters_to_global_o<CP>(Pg, sW1, sW4, sW2, sW3);
  __syncthreads();
  if (ADAM_SCALED) {
    scale_slab(M, c1);
    scale_slab(V, c2);
  }
  slab_to_lds(M, L);
  __syncthreads();
  masters_to_global_o<CP>(Mg, sW1, sW4, sW2, sW3);
  __syncthreads();
  slab_to_lds(V, L);
  __syncthreads();
  masters_to_global_o<CP>(Vg, sW1, sW4, sW2, sW3);
  if (threadIdx.x == 0) {
    A.adam_step[cid] = step;
    A.epochs_run[kslot] = ep_run;
    A.best_epoch[kslot] = best_ep;
  }
  STAMP(true, 31);
}

}  // namespace fedmx

extern "C" {

int fedmx_train_hw(const void* args, int k, hipStream_t stream);  // fedmx_train_hw.hip

// The compact shapes train on the helper-wave kernel unless the caller asks
// otherwise (TRAIN_FLAG_NO_HELPER).  Measured (r2, 5 clients x 5 epochs):
// 1.058 vs 1.090 ms, FedProx 1.137 vs 1.231 ms; bit-identical parameters
// (tests/test_kernels_gpu.py).

int fedmx_train(const void* args, int k, hipStream_t stream) {
  if (k <= 0) return 0;
  const fedmx::TrainArgs& A = *reinterpret_cast<const fedmx::TrainArgs*>(args);
  if (A.batch < 1) return -2;
  if (A.d_in < 1 || A.d_in > fedmx::DP - 1 || A.hidden < 1 || A.hidden > fedmx::HP - 1 || A.latent < 1 ||
      A.latent > fedmx::ZP - 1)
    return -3;
  const bool one = A.batch <= 16;
  // compact layer shapes; the helper-wave kernel takes any batch size there
  // (batches over 12 rows as 16-row chunks), this kernel's compact order
  // batches of <= 12 rows
  const bool cpl = A.hidden <= 27 && A.latent <= 7 && !(A.flags & fedmx::TRAIN_FLAG_NO_COMPACT);
  const bool cp = A.batch <= 12 && cpl;
  const bool hw = cpl && !(A.flags & fedmx::TRAIN_FLAG_NO_HELPER);
  if (hw) return fedmx_train_hw(args, k, stream);
  if (A.mu != 0.f) {
    if (cp)
      hipLaunchKernelGGL((fedmx::train_kernel<true, true, true>), dim3(k), dim3(256), 0, stream, A);
    else if (one)
      hipLaunchKernelGGL((fedmx::train_kernel<true, true, false>), dim3(k), dim3(256), 0, stream, A);
    else
      hipLaunchKernelGGL((fedmx::train_kernel<true, false, false>), dim3(k), dim3(256), 0, stream, A);
  } else {
    if (cp)
      hipLaunchKernelGGL((fedmx::train_kernel<false, true, true>), dim3(k), dim3(256), 0, stream, A);
    else if (one)
      hipLaunchKernelGGL((fedmx::train_kernel<false, true, false>), dim3(k), dim3(256), 0, stream, A);
    else
      hipLaunchKernelGGL((fedmx::train_kernel<false, false, false>), dim3(k), dim3(256), 0, stream, A);
  }
  return (int)hipGetLastError();
}

int fedmx_train_args_size() { return (int)sizeof(fedmx::TrainArgs); }

}  // extern "C"
