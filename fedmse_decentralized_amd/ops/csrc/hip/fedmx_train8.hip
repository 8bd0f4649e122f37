// Fused local training, 8-wave variant: two waves per SIMD.
//
// Same algorithm and numerics contract as fedmx_train.hip (ClientTrainer.run,
// src/Trainer/client_trainer.py:360-419; Appendix D of SURVEY.md), with the
// workgroup widened to 512 threads so that each SIMD runs two waves: one
// wave's optimizer / loss VALU work co-issues with the other wave's MFMAs
// (one wave per SIMD never co-executes: SQ_VALU_MFMA_COEXEC_CYCLES was 0 for
// the 4-wave kernel, profiles/r1_pmc_train2.md), and a lone wave issues VALU
// at half the SIMD's rate.
//
// Work split (wave w = 0..7, lane (c = l & 15, g = l >> 4)):
//   * W1a columns d in [16w, 16w+16) and W4a rows d in [16w, 16w+16) are
//     owned by wave w (param / Adam state in registers):
//       q1[t][r] = W1a[16t+c][16w+4g+r]   (A-operand layout of layer 1 =
//                                           D layout of dW1^T tiles)
//       q4[t][r] = W4a[16w+4g+r][16t+c]   (D layout, A operand of W4a^T dY)
//   * the four small-layer gradient tiles belong to waves 0..3 (w<2: W3a tile
//     of h-block w, w=2,3: W2a tile of h-block w-2), as in the 4-wave kernel.
//   * layer 1 and dH3 = W4a^T dY are K-split over the 8 column blocks
//     (partials reduced in a fixed wave order through LDS: barriers #1 / #2);
//     layers 2-3 and dZ / dH1 run redundantly in every wave (identical
//     values); the H1^T / H3^T / Z^T transposes they feed are staged once,
//     by wave 0, before barrier #2.
//   * dW4 runs after barrier #2 (it is first needed by the next step's
//     layer 4), directly followed by the W4 update.
//   * per step: 2 workgroup barriers, 72-76 MFMAs per wave.
// Measured on MI355X it is SLOWER than the 4-wave kernel (1.62 vs 1.39 ms for
// 5 clients x 5 epochs, profiles/r1_train8_stamps.txt): the step is bound by
// dependent MFMA chains and barrier waits, and the duplicated small-layer
// chains of the two waves sharing a SIMD contend for its matrix pipe.  Kept as
// an opt-in variant (FEDMX_TRAIN_WAVES=8) with its own numerics test.
#include "fedmx_train_common.h"

namespace fedmx {
namespace w8 {

constexpr int NW = 8;
constexpr int L_W1 = HP * S_W1;             // 4224 master (snapshots / write-back)
constexpr int L_W4 = DP * S_W4;             // 4608
constexpr int L_W2 = ZP * S_W2;             // 576
constexpr int L_W3 = HP * S_W3;             // 640
constexpr int L_RED = NW * 2 * 256;         // 4096 one partial-sum exchange buffer
constexpr int L_T32 = 32 * S_T;             // 640
constexpr int L_T16 = 16 * S_T;             // 320
constexpr int L_SHARED = 2 * L_T32 + L_T16; // H1^T, H3^T, Z^T (written by wave 0)
constexpr int L_SCR = L_T16 + L_T32 + L_T16; // per wave: dY^T own rows, dH3^T, dZ^T
constexpr int L_TOTAL = L_W1 + L_W4 + L_W2 + L_W3 + 3 * L_RED + L_SHARED + NW * L_SCR + 2 * NW * 4;
static_assert(L_TOTAL * 4 <= 160 * 1024, "LDS budget");

struct Slab {
  float q1[2][4];
  float q4[2][4];
  float o[4];
};

struct Lane {
  float* w1;   // sW1 + c*S_W1 + 16w + 4g            (+ 16t*S_W1; 4 consecutive r)
  float* w4;   // sW4 + (16w+4g)*S_W4 + c            (+ r*S_W4 + 16t)
  float* own;  // owned small tile (waves 0..3), stride own_stride per r
  int own_stride;
  bool has_own;
};

__device__ __forceinline__ void w1_to_lds(const Slab& o, const Lane& L) {
#pragma unroll
  for (int t = 0; t < 2; ++t) lds_write4(L.w1 + 16 * t * S_W1, f32x4{o.q1[t][0], o.q1[t][1], o.q1[t][2], o.q1[t][3]});
}
__device__ __forceinline__ void w4_to_lds(const Slab& o, const Lane& L) {
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int r = 0; r < 4; ++r) L.w4[r * S_W4 + 16 * t] = o.q4[t][r];
}
__device__ __forceinline__ void own_to_lds(const Slab& o, const Lane& L) {
  if (!L.has_own) return;
#pragma unroll
  for (int r = 0; r < 4; ++r) L.own[r * L.own_stride] = o.o[r];
}
__device__ __forceinline__ void slab_to_lds(const Slab& o, const Lane& L) {
  w1_to_lds(o, L);
  w4_to_lds(o, L);
  own_to_lds(o, L);
}
__device__ __forceinline__ void lds_to_slab(Slab& o, const Lane& L) {
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    const f32x4 q = lds_read4(L.w1 + 16 * t * S_W1);
#pragma unroll
    for (int r = 0; r < 4; ++r) o.q1[t][r] = q[r];
  }
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int r = 0; r < 4; ++r) o.q4[t][r] = L.w4[r * S_W4 + 16 * t];
#pragma unroll
  for (int r = 0; r < 4; ++r) o.o[r] = L.has_own ? L.own[r * L.own_stride] : 0.f;
}

// One 16-row batch tile: feature-major X[b=c][16w+4g+s] and batch-major
// X[b=4g+s][16w+c]; rows past the tile are zeroed, the bias column is 1 on
// real rows (applied by finalize when the tile is consumed).
struct XChunk {
  f32x4 f, b;
};

template <bool PROX, bool ONE>
__global__ __launch_bounds__(512, 1) void train8_kernel(const TrainArgs A) {
  __shared__ __attribute__((aligned(16))) float lds[L_TOTAL];
  const int w = threadIdx.x >> 6;
  const int lane = threadIdx.x & 63;
  const int c = lane & 15;
  const int g = lane >> 4;
  float* const sW1 = lds;
  float* const sW4 = sW1 + L_W1;
  float* const sW2 = sW4 + L_W4;
  float* const sW3 = sW2 + L_W2;
  float* const sRedH1 = sW3 + L_W3;        // two buffers (parity)
  float* const sRedDH3 = sRedH1 + 2 * L_RED;
  float* const sH1T = sRedDH3 + L_RED;     // shared transposes (wave 0 writes)
  float* const sH3T = sH1T + L_T32;
  float* const sZT = sH3T + L_T32;
  float* const scr = sZT + L_T16 + w * L_SCR;
  float* const sDYT = scr;                 // dY^T own 16 rows  [16][S_T]
  float* const sDH3T = sDYT + L_T16;       // dH3^T             [32][S_T] (waves 0,1)
  float* const sDZT = sDH3T + L_T32;       // dZ^T              [16][S_T] (waves 2,3)
  double* const sLoss = reinterpret_cast<double*>(sZT + L_T16 + NW * L_SCR);  // [8][4] doubles

  Lane L;
  L.w1 = sW1 + c * S_W1 + 16 * w + 4 * g;
  L.w4 = sW4 + (16 * w + 4 * g) * S_W4 + c;
  L.has_own = w < 4;
  if (w < 2) {
    L.own = sW3 + (16 * w + 4 * g) * S_W3 + c;
    L.own_stride = S_W3;
  } else {
    L.own = sW2 + 4 * g * S_W2 + 16 * ((w - 2) & 1) + c;
    L.own_stride = S_W2;
  }
  const float* const a4p = sW4 + (16 * w + c) * S_W4 + 4 * g;  // + 16t
  const float* const a2p = sW2 + c * S_W2 + 4 * g;             // + 16t
  const float* const a3p = sW3 + c * S_W3 + 4 * g;             // + 16t*S_W3
  const float* const d2p = sW2 + 4 * g * S_W2 + c;             // W2a[4g+r][16t+c]
  const float* const d3p = sW3 + 4 * g * S_W3 + c;             // W3a[16t+4g+r][c]
  const int tw = 4 * g * S_T + c;   // transpose write: [feature 4g+r (+16t)][b=c]
  const int tr = c * S_T + 4 * g;   // transpose read : [feature c (+16t)][b=4g..4g+3]

  const int kslot = blockIdx.x;
  const int cid = A.client_idx[kslot];
  float* const Pg = A.params + (size_t)cid * P_PAD;
  float* const Mg = A.adam_m + (size_t)cid * P_PAD;
  float* const Vg = A.adam_v + (size_t)cid * P_PAD;
  float* const Bg = A.best + (size_t)cid * P_PAD;
  const int d_in = A.d_in, hidden = A.hidden, latent = A.latent;

  STAMP(true, 28);
  Slab P, M, V, AN;
  global_to_masters(Mg, sW1, sW4, sW2, sW3);
  __syncthreads();
  lds_to_slab(M, L);
  __syncthreads();
  global_to_masters(Vg, sW1, sW4, sW2, sW3);
  __syncthreads();
  lds_to_slab(V, L);
  __syncthreads();
  if (PROX) {
    global_to_masters(A.anchor + (size_t)cid * P_PAD, sW1, sW4, sW2, sW3);
    __syncthreads();
    lds_to_slab(AN, L);
    __syncthreads();
  }
  global_to_masters(Pg, sW1, sW4, sW2, sW3);
  __syncthreads();
  lds_to_slab(P, L);
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
  const bool bias_lane = (w == NW - 1 && g == 3);  // feature-major: column DP-1 = 16*7 + 4*3 + 3
  const bool bias_col = (w == NW - 1 && c == 15);  // batch-major:   column DP-1 = 16*7 + 15
  const int xcol = 16 * w + 4 * g;
  const float lam = A.lambda;
  const float inv_d = 1.0f / (float)d_in;
  float fm[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) fm[r] = (xcol + r < d_in) ? 1.f : 0.f;
  bool stamp_fwd = false;
  (void)stamp_fwd;

  auto load_chunk = [&](const float* X, int row0, int bc, XChunk& x) {
    const float* src = X + (size_t)(row0 + (c < bc ? c : 0)) * DP + xcol;
    x.f = *reinterpret_cast<const f32x4*>(src);
    const float* bsrc = X + (size_t)row0 * DP + 16 * w + c;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int rr = (4 * g + r < bc) ? 4 * g + r : 0;
      x.b[r] = bsrc[(size_t)rr * DP];
    }
  };
  auto finalize_chunk = [&](int bc, XChunk& x) {
    const bool ok = c < bc;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const bool okr = 4 * g + r < bc;
      x.f[r] = ok ? x.f[r] : 0.f;
      x.b[r] = okr ? (bias_col ? 1.f : x.b[r]) : 0.f;
    }
    if (bias_lane) x.f[3] = 1.f;
  };
  auto load_chunk_f = [&](const float* X, int row0, int bc, XChunk& x) {
    const bool ok = c < bc;
    const f32x4 f = *reinterpret_cast<const f32x4*>(X + (size_t)(row0 + (ok ? c : 0)) * DP + xcol);
#pragma unroll
    for (int r = 0; r < 4; ++r) x.f[r] = ok ? f[r] : 0.f;
    if (bias_lane) x.f[3] = 1.f;
  };

  auto l1_partial = [&](const XChunk& x, f32x4& acc0, f32x4& acc1) {
    acc0 = zero4();
    acc1 = zero4();
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      acc0 = mfma16(P.q1[0][j], x.f[j], acc0);
      acc1 = mfma16(P.q1[1][j], x.f[j], acc1);
    }
  };

  auto forward_rest = [&](const f32x4& acc0, const f32x4& acc1, const XChunk& x, int bc, float inv_bt,
                          f32x4 (&h1)[2], f32x4& z, f32x4& zb, f32x4 (&h3)[2], f32x4& y, float& norm_c,
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
      for (int ww = 1; ww < NW; ++ww) {
        const f32x4 o = lds_read4(red + (ww * 2 + t) * 256 + lane * 4);
#pragma unroll
        for (int r = 0; r < 4; ++r) s[r] = s[r] + o[r];
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float vv = fmaxf(s[r], 0.f);
        if (16 * t + 4 * g + r == HP - 1) vv = 1.f;
        s[r] = vv;
      }
      h1[t] = s;
    }
    parity ^= 1;
    z = zero4();
    {
      const f32x4 a0 = lds_read4(a2p);
      const f32x4 a1 = lds_read4(a2p + 16);
#pragma unroll
      for (int s = 0; s < 4; ++s) z = mfma16(a0[s], h1[0][s], z);
#pragma unroll
      for (int s = 0; s < 4; ++s) z = mfma16(a1[s], h1[1][s], z);
    }
    zb = z;
    if (g == 3) zb[3] = 1.f;
    {
      f32x4 c0 = zero4(), c1 = zero4();
      const f32x4 a0 = lds_read4(a3p);
      const f32x4 a1 = lds_read4(a3p + 16 * S_W3);
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        c0 = mfma16(a0[s], zb[s], c0);
        c1 = mfma16(a1[s], zb[s], c1);
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float v0 = fmaxf(c0[r], 0.f), v1 = fmaxf(c1[r], 0.f);
        if (16 + 4 * g + r == HP - 1) v1 = 1.f;
        c0[r] = v0;
        c1[r] = v1;
      }
      h3[0] = c0;
      h3[1] = c1;
    }
    {
      // own 16 output rows; two accumulators (one per h k-block) shorten the chain
      f32x4 y0 = zero4(), y1 = zero4();
      const f32x4 a0 = lds_read4(a4p);
      const f32x4 a1 = lds_read4(a4p + 16);
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        y0 = mfma16(a0[s], h3[0][s], y0);
        y1 = mfma16(a1[s], h3[1][s], y1);
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) y[r] = y0[r] + y1[r];
    }
    float sq = 0.f;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float d0 = (y[r] - x.f[r]) * fm[r];
      sq += d0 * d0;
    }
    sq = (c < bc) ? sq : 0.f;
    float nz = 0.f;
#pragma unroll
    for (int r = 0; r < 4; ++r) nz += (4 * g + r < latent) ? z[r] * z[r] : 0.f;
    nz = sum_lane_groups(nz);
    norm_c = __builtin_amdgcn_sqrtf(nz);
    float contrib = sq * (inv_bt * inv_d);
    if (w == 0 && g == 0 && c < bc) contrib += lam * norm_c * inv_bt;
    lacc += (double)contrib;
  };

  AdamStep K;
  K.one_m_b1 = 1.f - A.beta1;
  K.b2 = A.beta2;
  K.one_m_b2 = 1.f - A.beta2;
  K.eps = A.eps;
  K.two_mu = 2.f * A.mu;
  double b1pow = pow((double)A.beta1, (double)step);
  double b2pow = pow((double)A.beta2, (double)step);

  double min_valid = __builtin_huge_val();
  int worse = 0, ep_run = 0, best_ep = -1;

  for (int ep = 0; ep < A.epochs; ++ep) {
    double acc_tr = 0.0;
    int bi = 0, ch = 0;
    XChunk cur, nxt;
    f32x4 l1a = zero4(), l1b = zero4();
    if (nb > 0) {
      const int bc0 = min(16, min(B, n_tr));
      load_chunk(Xtr, 0, bc0, cur);
      finalize_chunk(bc0, cur);
      l1_partial(cur, l1a, l1b);
    }
    f32x4 G1[2], G4[2], Go;
    while (bi < nb) {
      const int row_b = bi * B;
      const int bt = min(B, n_tr - row_b);
      const int nch = ONE ? 1 : (bt + 15) >> 4;
      const int bc = ONE ? bt : min(16, bt - 16 * ch);
      const bool last = ONE || (ch == nch - 1);
      const int bi_n = last ? bi + 1 : bi;
      const int ch_n = last ? 0 : ch + 1;
      const bool has_next = bi_n < nb;
      const int row_n = bi_n * B + 16 * ch_n;
      const int bc_n = has_next ? min(16, min(B, n_tr - bi_n * B) - 16 * ch_n) : 0;
      const float inv_bt = 1.0f / (float)bt;
      if (ch == 0) {
        G1[0] = G1[1] = G4[0] = G4[1] = Go = zero4();
      }
      f32x4 h1[2], z, zb, h3[2], y;
      float norm_c;
      const bool stamp_on = (ep == 0 && bi == STAMP_STEP && ch == 0);
      STAMP(stamp_on, 0);
      stamp_fwd = FEDMX_STAMPS && stamp_on;
      forward_rest(l1a, l1b, cur, bc, inv_bt, h1, z, zb, h3, y, norm_c, acc_tr);
      STAMP(stamp_on, 3);
      if (has_next) load_chunk(Xtr, row_n, bc_n, nxt);

      float q2[2][4], q3[2][4];
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          q2[t][r] = d2p[r * S_W2 + 16 * t];
          q3[t][r] = d3p[(16 * t + r) * S_W3];
        }

      // ---- dY (own 16 rows, feature-major), dH3 partial = W4a(own rows)^T dY
      const float scale = (c < bc) ? 2.0f / (float)(bt * d_in) : 0.f;
      f32x4 dy;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        dy[r] = (y[r] - cur.f[r]) * (scale * fm[r]);
        sDYT[tw + r * S_T] = dy[r];
      }
      {
        f32x4 a0 = zero4(), a1 = zero4();
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          a0 = mfma16(P.q4[0][s], dy[s], a0);
          a1 = mfma16(P.q4[1][s], dy[s], a1);
        }
        lds_write4(sRedDH3 + (w * 2 + 0) * 256 + lane * 4, a0);
        lds_write4(sRedDH3 + (w * 2 + 1) * 256 + lane * 4, a1);
      }
      if (w == 0) {  // shared transposes (identical in every wave)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          sH1T[tw + r * S_T] = h1[0][r];
          sH1T[tw + (16 + r) * S_T] = h1[1][r];
          sH3T[tw + r * S_T] = h3[0][r];
          sH3T[tw + (16 + r) * S_T] = h3[1][r];
          sZT[tw + r * S_T] = zb[r];
        }
      }
      STAMP(stamp_on, 4);
      STAMP(stamp_on, 5);
      STAMP(stamp_on, 6);
      __syncthreads();  // barrier #2: dH3 partials, transposes and own dY^T visible
      STAMP(stamp_on, 7);
      // ---- dW4 (own rows) = dY^T H3, accumulated over the batch's chunks
      {
        const f32x4 a = lds_read4(sDYT + tr);
        const f32x4 b0 = lds_read4(sH3T + tr);
        const f32x4 b1 = lds_read4(sH3T + tr + 16 * S_T);
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          G4[0] = mfma16(a[s], b0[s], G4[0]);
          G4[1] = mfma16(a[s], b1[s], G4[1]);
        }
      }
      f32x4 dh3[2];
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        f32x4 s = lds_read4(sRedDH3 + t * 256 + lane * 4);
#pragma unroll
        for (int ww = 1; ww < NW; ++ww) {
          const f32x4 o = lds_read4(sRedDH3 + (ww * 2 + t) * 256 + lane * 4);
#pragma unroll
          for (int r = 0; r < 4; ++r) s[r] = s[r] + o[r];
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int h = 16 * t + 4 * g + r;
          s[r] = (h < hidden && h3[t][r] > 0.f) ? s[r] : 0.f;
        }
        dh3[t] = s;
      }
      float prox_acc = 0.f;
      if (last) {
        ++step;
        b1pow *= (double)A.beta1;
        b2pow *= (double)A.beta2;
        K.neg_step_size = (float)(-((double)A.lr / (1.0 - b1pow)));
        K.bc2s = (float)sqrt(1.0 - b2pow);
        K.inv_bc2s = 1.0f / K.bc2s;
#pragma unroll
        for (int t = 0; t < 2; ++t) adam4<PROX>(P.q4[t], M.q4[t], V.q4[t], AN.q4[t], G4[t], K, prox_acc);
        w4_to_lds(P, L);  // own rows: read back by this wave's next layer-4 product
      }
      if (w < 2) {
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
          for (int r = 0; r < 4; ++r) sDH3T[tw + (16 * t + r) * S_T] = dh3[t][r];
      }
      f32x4 dz = zero4();
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int s = 0; s < 4; ++s) dz = mfma16(q3[t][s], dh3[t][s], dz);
      const float shr_raw = lam * __builtin_amdgcn_rcpf((float)bt * norm_c);
      const float shr = (c < bc && norm_c > 0.f) ? shr_raw : 0.f;
#pragma unroll
      for (int r = 0; r < 4; ++r) dz[r] = (4 * g + r < latent) ? dz[r] + shr * z[r] : 0.f;
      if (w == 2 || w == 3) {
#pragma unroll
        for (int r = 0; r < 4; ++r) sDZT[tw + r * S_T] = dz[r];
      }
      f32x4 dh1b[2], h1b[2];
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        h1b[t] = lds_read4(sH1T + tr + 16 * t * S_T);
        f32x4 acc = zero4();
#pragma unroll
        for (int s = 0; s < 4; ++s) acc = mfma16(dz[s], q2[t][s], acc);
#pragma unroll
        for (int r = 0; r < 4; ++r) acc[r] = (16 * t + c < hidden && h1b[t][r] > 0.f) ? acc[r] : 0.f;
        dh1b[t] = acc;
      }
      STAMP(stamp_on, 8);
      // ---- dW1^T (own 16 columns) = X^T dH1 -> q1 layout
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        G1[0] = mfma16(cur.b[s], dh1b[0][s], G1[0]);
        G1[1] = mfma16(cur.b[s], dh1b[1][s], G1[1]);
      }
      if (w < 4) {
        wave_sync();
        f32x4 a, b;
        if (w < 2) {
          a = lds_read4(sDH3T + tr + 16 * w * S_T);
          b = lds_read4(sZT + tr);
        } else {
          a = lds_read4(sDZT + tr);
          b = (w == 2) ? h1b[0] : h1b[1];
        }
#pragma unroll
        for (int s = 0; s < 4; ++s) Go = mfma16(a[s], b[s], Go);
      }
      STAMP(stamp_on, 9);
      if (last) {
#pragma unroll
        for (int t = 0; t < 2; ++t) adam4<PROX>(P.q1[t], M.q1[t], V.q1[t], AN.q1[t], G1[t], K, prox_acc);
        STAMP(stamp_on, 10);
        if (has_next) {
          finalize_chunk(bc_n, nxt);
          l1_partial(nxt, l1a, l1b);
        }
        if (w < 4) {
          adam4<PROX>(P.o, M.o, V.o, AN.o, Go, K, prox_acc);
          own_to_lds(P, L);
        }
        if (PROX) acc_tr += (double)A.mu * (double)prox_acc;
      } else {
        finalize_chunk(bc_n, nxt);
        l1_partial(nxt, l1a, l1b);
      }
      STAMP(stamp_on, 11);
      cur = nxt;
      bi = bi_n;
      ch = ch_n;
    }

    // ---- validation pass
    double acc_va = 0.0;
    for (int vb = 0; vb < nvb; ++vb) {
      const int row0 = vb * B;
      const int bt = min(B, n_va - row0);
      const float inv_bt = 1.0f / (float)bt;
      for (int c0 = 0; c0 < bt; c0 += 16) {
        const int bc = min(16, bt - c0);
        XChunk xv;
        STAMP(ep == 0 && vb == 1 && c0 == 0, 16);
        load_chunk_f(Xva, row0 + c0, bc, xv);
        f32x4 a0, a1;
        l1_partial(xv, a0, a1);
        f32x4 h1[2], z, zb, h3[2], y;
        float norm_c;
        STAMP(ep == 0 && vb == 1 && c0 == 0, 17);
        forward_rest(a0, a1, xv, bc, inv_bt, h1, z, zb, h3, y, norm_c, acc_va);
        STAMP(ep == 0 && vb == 1 && c0 == 0, 18);
      }
    }
    STAMP(ep == 0, 12);
    double prox_now = 0.0;
    if (PROX) {
      float pr = 0.f;
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float d1 = P.q1[t][r] - AN.q1[t][r];
          const float d4 = P.q4[t][r] - AN.q4[t][r];
          pr += d1 * d1 + d4 * d4;
        }
      if (w < 4) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float d = P.o[r] - AN.o[r];
          pr += d * d;
        }
      }
      prox_now = (double)pr;
    }
    w1_to_lds(P, L);
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
    double tr_sum = 0.0, va_sum = 0.0, px_sum = 0.0;
#pragma unroll
    for (int ww = 0; ww < NW; ++ww) {
      tr_sum += sLoss[ww * 4 + 0];
      va_sum += sLoss[ww * 4 + 1];
      px_sum += sLoss[ww * 4 + 2];
    }
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
      masters_to_global(Bg, sW1, sW4, sW2, sW3);
    } else {
      ++worse;
    }
    __syncthreads();
    STAMP(ep == 0, 13);
    if (worse >= A.patience && worse > 0) break;
  }

  STAMP(true, 30);
  w1_to_lds(P, L);
  __syncthreads();
  masters_to_global(Pg, sW1, sW4, sW2, sW3);
  __syncthreads();
  slab_to_lds(M, L);
  __syncthreads();
  masters_to_global(Mg, sW1, sW4, sW2, sW3);
  __syncthreads();
  slab_to_lds(V, L);
  __syncthreads();
  masters_to_global(Vg, sW1, sW4, sW2, sW3);
  if (threadIdx.x == 0) {
    A.adam_step[cid] = step;
    A.epochs_run[kslot] = ep_run;
    A.best_epoch[kslot] = best_ep;
  }
  STAMP(true, 31);
}

}  // namespace w8
}  // namespace fedmx

extern "C" {

int fedmx_train8(const void* args, int k, hipStream_t stream) {
  if (k <= 0) return 0;
  const fedmx::TrainArgs& A = *reinterpret_cast<const fedmx::TrainArgs*>(args);
  if (A.batch < 1) return -2;
  if (A.d_in < 1 || A.d_in > fedmx::DP - 1 || A.hidden < 1 || A.hidden > fedmx::HP - 1 || A.latent < 1 ||
      A.latent > fedmx::ZP - 1)
    return -3;
  // single-tile batches only: the multi-tile bookkeeping does not fit the
  // 256-register budget of two waves per SIMD (callers use fedmx_train)
  if (A.batch > 16) return -4;
  if (A.mu != 0.f)
    hipLaunchKernelGGL((fedmx::w8::train8_kernel<true, true>), dim3(k), dim3(512), 0, stream, A);
  else
    hipLaunchKernelGGL((fedmx::w8::train8_kernel<false, true>), dim3(k), dim3(512), 0, stream, A);
  return (int)hipGetLastError();
}

}  // extern "C"
