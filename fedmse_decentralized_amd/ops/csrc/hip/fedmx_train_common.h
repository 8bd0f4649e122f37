// Shared pieces of the fused local-training kernels (fedmx_train.hip: 4 waves,
// fedmx_train_hw.hip: 4 main + 4 helper waves): kernel arguments, the fused Adam update, the
// in-kernel timestamp macro and the dense <-> LDS-master parameter staging.
#pragma once
#include "fedmx_common.h"

// Build variants of the training kernels (the only two compile-time switches
// of the training sources besides the launch-time tunables of
// fedmx_train_hw.hip; every other variant measured in rounds 1-5 lives in git
// history and in profiles/r*_train_*):
//   FEDMX_EXACT_ADAM=1  torch's exact Adam rounding sequence (IEEE square root
//                       and divisions: adam4) instead of the scaled-moment
//                       form (adam4s); libfedmx_hip_exact.so, the long-horizon
//                       parity test
//   FEDMX_STAMPS=1      in-kernel s_memtime phase stamps (libfedmx_hip_stamps.so,
//                       scripts/train_stamps.py)
// (FEDMX_HW_PROX_TU is no variant: it selects which part of
// fedmx_train_hw.hip a translation unit holds -- fedmx_train_hw_prox.hip,
// the FedProx instantiation under its own compiler flags)
#ifndef FEDMX_EXACT_ADAM
#define FEDMX_EXACT_ADAM 0
#endif

namespace fedmx {

struct TrainArgs {
  float* params;            // [C, P_PAD]
  float* adam_m;            // [C, P_PAD]
  float* adam_v;            // [C, P_PAD]
  const float* anchor;      // [C, P_PAD] FedProx anchor (previous global model)
  float* best;              // [C, P_PAD] best-validation snapshot (model.cpt content)
  int32_t* adam_step;       // [C]
  const float* train_x;     // [rows, DP]
  const int64_t* train_off; // [C+1]
  const float* valid_x;     // [rows, DP]
  const int64_t* valid_off; // [C+1]
  const int32_t* client_idx;  // [k] store rows to train
  double* tracking;         // [k, epochs, 2] (train_loss, valid_loss)
  int32_t* epochs_run;      // [k]
  int32_t* best_epoch;      // [k]
  int32_t epochs, batch, patience, d_in, hidden, latent;
  float lr, beta1, beta2, eps, lambda, mu;
  uint64_t* stamps;         // [8 waves][32] s_memtime stamps of one step (FEDMX_STAMPS builds), or null
  int32_t flags;            // TRAIN_FLAG_* bits
  int32_t pad0;
  int32_t* err;             // or null: set to 1 by a launch that failed (a flag wait ran out,
                            // fedmx_train_hw.hip); read by elect_wsum_kernel, which then skips
                            // the round's aggregation and adoption (engine/device_round.py)
  float* vws;               // or null: [k][fedmx_train_av_slot()] workspace of the helper-wave
                            // kernel's validator workgroups (epoch snapshots, flags); zeroed once
  uint32_t vseq;            // launch number (> 0, distinct per launch on this workspace): stamps
                            // the workspace's flags, so no launch reads another's
  int32_t pad1;
};
constexpr int32_t TRAIN_FLAG_NO_COMPACT = 1;  // identity-order kernels even where the compact order applies
constexpr int32_t TRAIN_FLAG_HELPER = 2;      // helper-wave kernel (fedmx_train_hw.hip) for the compact shapes
constexpr int32_t TRAIN_FLAG_NO_HELPER = 4;   // never the helper-wave kernel
constexpr int32_t TRAIN_FLAG_ASYNC_VALID = 16;  // set by the launcher (fedmx_train_hw): validator workgroups
constexpr int32_t TRAIN_FLAG_TEST_DROP_W4 = 8;   // tests only: one W4 hand-off is never published (a
                                                 // flag-wait timeout in the FedProx helper-wave kernel)
constexpr int32_t TRAIN_FLAG_TEST_MUTE_VALIDATOR = 32;   // tests only: client slot 0's validator never answers
                                                         // (a decision-wait timeout, 0.2 s)

// In-kernel phase timestamps (build with -DFEDMX_STAMPS=1): wave w's lane 0 of
// workgroup 0 records s_memtime at fixed points of training step STAMP_STEP
// of epoch 0 and of the first validation batch.
#ifndef FEDMX_STAMPS
#define FEDMX_STAMPS 0
#endif
constexpr int STAMP_STEP = 20;
#if FEDMX_STAMPS
#define STAMP(cond, i)                                                                          \
  do {                                                                                          \
    if ((cond) && A.stamps != nullptr && blockIdx.x == 0 && lane == 0)                          \
      A.stamps[w * 32 + (i)] = __builtin_amdgcn_s_memtime();                                   \
  } while (0)
#else
#define STAMP(cond, i) \
  do {                 \
  } while (0)
#endif

struct AdamStep {
  float one_m_b1, b2, one_m_b2, inv_bc2s, bc2s, eps, neg_step_size, two_mu;
  float b1, kd, ed;   // scaled form (adam4s)
};

// Scaled-moment Adam (both training kernels; not in FEDMX_EXACT_ADAM builds): the kernel keeps
//   mh = m / (1-b1),  vh = v / (1-b2)
// in registers for the whole launch (scaled on load, unscaled on write-back),
// which turns torch's update into
//   mh = b1*mh + g ;  vh = b2*vh + g*g ;
//   p  = p + mh / (sqrt(vh)*kd + ed)
// with the per-step scalars  S  = -(lr/bc1)*(1-b1),
//   kd = sqrt(1-b2) / (sqrt(bc2)*S),  ed = eps / S
// (algebraically torch's  p -= lr/bc1 * m / (sqrt(v)/sqrt(bc2) + eps)):
// 5 VALU + 2 transcendental issues per parameter instead of 8 + 2 — the
// optimizer is ~35 % of the training launch (ablation, profiles/r2_*).
// Rounding differs from the unscaled form in the last bits only.
template <bool PROX>
__device__ __forceinline__ void adam4s(float (&p)[4], float (&m)[4], float (&v)[4], const float (&a)[4], f32x4 g,
                                       const AdamStep& K, float& prox_acc) {
  float gr[4], t0[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) gr[r] = g[r];
  if (PROX) {
#pragma unroll
    for (int r = 0; r < 4; ++r) t0[r] = p[r] - a[r];
#pragma unroll
    for (int r = 0; r < 4; ++r) prox_acc += t0[r] * t0[r];
#pragma unroll
    for (int r = 0; r < 4; ++r) gr[r] = gr[r] + K.two_mu * t0[r];
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) t0[r] = v[r] * K.b2;
#pragma unroll
  for (int r = 0; r < 4; ++r) v[r] = __builtin_fmaf(gr[r], gr[r], t0[r]);
#pragma unroll
  for (int r = 0; r < 4; ++r) m[r] = __builtin_fmaf(K.b1, m[r], gr[r]);
#pragma unroll
  for (int r = 0; r < 4; ++r) t0[r] = __builtin_amdgcn_sqrtf(v[r]);
#pragma unroll
  for (int r = 0; r < 4; ++r) t0[r] = __builtin_fmaf(t0[r], K.kd, K.ed);
#pragma unroll
  for (int r = 0; r < 4; ++r) t0[r] = __builtin_amdgcn_rcpf(t0[r]);
#pragma unroll
  for (int r = 0; r < 4; ++r) p[r] = __builtin_fmaf(m[r], t0[r], p[r]);
}

// adam4s's per-step scalars (both training kernels, so the helper-wave and
// the 4-wave kernels stay bit-identical): with 1/S = (b1^t - 1) / (lr (1-b1))
//   ed = eps / S,  kd = sqrt(1-b2) / (sqrt(bc2) S) = sqrt(1-b2) (1/S) rsqrt(bc2)
// -- only 1/S changes linearly per step: no f64 division or square root on
// the step's path (the f32 rsqrt of bc2 is <= 1 ulp)
struct AdamScaledInit {
  double r_lrc1;   // 1 / (lr (1 - b1))
  double sq_c2;    // sqrt(1 - b2)
  double eps;
};
__device__ __forceinline__ AdamScaledInit adam_scaled_init(float lr, float beta1, float beta2, float eps) {
  return AdamScaledInit{1.0 / ((double)lr * (double)(1.f - beta1)), sqrt((double)(1.f - beta2)), (double)eps};
}
__device__ __forceinline__ void adam_scaled_step(AdamStep& K, const AdamScaledInit& I, double b1pow, double b2pow) {
  const double inv_s = (b1pow - 1.0) * I.r_lrc1;
  K.ed = (float)(I.eps * inv_s);
  K.kd = (float)(I.sq_c2 * inv_s) * __builtin_amdgcn_rsqf((float)(1.0 - b2pow));
}
// moment scale on load (m / (1-b1), v / (1-b2)); the write-back multiplies by 1-b
__device__ __forceinline__ float adam_moment_in_scale(float beta) { return (float)(1.0 / (double)(1.f - beta)); }

// torch.optim.Adam single-tensor update (no weight decay / amsgrad), the
// FEDMX_EXACT_ADAM build:
//   m.lerp_(g, 1-b1); v.mul_(b2).addcmul_(g, g, 1-b2)
//   p.addcdiv_(m, sqrt(v)/sqrt(bc2) + eps, -lr/bc1)
// torch's CPU op sequence, rounding for rounding (checked against torch 2.10
// on the CPU: lerp and addcmul fused, `(sqrt(v) / bc2s) + eps` and addcdiv's
// `p + (value * m) / denom` separately rounded); only torch's vectorised sqrt
// (SLEEF, 0.5001 ulp: ~0.6 % of inputs off by one ulp) differs from the IEEE
// square root used here (54 % slower launch than adam4s,
// profiles/r4_train_hw_experiments.md; tests/test_long_horizon_gpu.py).
// Four elements (one accumulator register quad) at a time, stage-major.
template <bool PROX>
__device__ __forceinline__ void adam4(float (&p)[4], float (&m)[4], float (&v)[4], const float (&a)[4], f32x4 g,
                                      const AdamStep& K, float& prox_acc) {
  float gr[4], t0[4], t1[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) gr[r] = g[r];
  if (PROX) {
#pragma unroll
    for (int r = 0; r < 4; ++r) t0[r] = p[r] - a[r];
#pragma unroll
    for (int r = 0; r < 4; ++r) prox_acc += t0[r] * t0[r];
#pragma unroll
    for (int r = 0; r < 4; ++r) gr[r] = gr[r] + K.two_mu * t0[r];
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) t0[r] = gr[r] - m[r];
#pragma unroll
  for (int r = 0; r < 4; ++r) m[r] = __builtin_fmaf(K.one_m_b1, t0[r], m[r]);
#pragma unroll
  for (int r = 0; r < 4; ++r) t0[r] = v[r] * K.b2;
#pragma unroll
  for (int r = 0; r < 4; ++r) t1[r] = K.one_m_b2 * gr[r];
#pragma unroll
  for (int r = 0; r < 4; ++r) v[r] = __builtin_fmaf(t1[r], gr[r], t0[r]);
#pragma unroll
  for (int r = 0; r < 4; ++r) t0[r] = __fsqrt_rn(v[r]);
#pragma unroll
  for (int r = 0; r < 4; ++r) t0[r] = t0[r] / K.bc2s + K.eps;   // (-ffp-contract=off: two roundings)
#pragma unroll
  for (int r = 0; r < 4; ++r) t1[r] = K.neg_step_size * m[r];
#pragma unroll
  for (int r = 0; r < 4; ++r) t1[r] = t1[r] / t0[r];
#pragma unroll
  for (int r = 0; r < 4; ++r) p[r] = p[r] + t1[r];
}

// L2 / dZ products as two accumulator chains, per instantiation (bit 0
// plain, bit 1 FedProx, bit 2 batch > 12): chain2 in both training kernels
constexpr int SPLIT_CHAINS = 5;

// the build's Adam form: scaled moments (moments in registers as m/(1-b1),
// v/(1-b2) for the whole launch) unless FEDMX_EXACT_ADAM
constexpr bool ADAM_SCALED = !FEDMX_EXACT_ADAM;
template <bool PROX>
__device__ __forceinline__ void adam_update(float (&p)[4], float (&m)[4], float (&v)[4], const float (&a)[4], f32x4 g,
                                            const AdamStep& K, float& prox_acc) {
  if constexpr (ADAM_SCALED)
    adam4s<PROX>(p, m, v, a, g, K, prox_acc);
  else
    adam4<PROX>(p, m, v, a, g, K, prox_acc);
}
// the per-step scalars of the build's form for the step whose bias
// corrections are 1 - b1pow, 1 - b2pow
__device__ __forceinline__ void adam_step_scalars(AdamStep& K, const AdamScaledInit& I, float lr, double b1pow,
                                                  double b2pow) {
  if constexpr (ADAM_SCALED) {
    adam_scaled_step(K, I, b1pow, b2pow);
  } else {
    K.neg_step_size = (float)(-((double)lr / (1.0 - b1pow)));
    K.bc2s = (float)sqrt(1.0 - b2pow);
    K.inv_bc2s = 1.0f / K.bc2s;
  }
}

// ---- compact internal order (train_kernel<.., CP = true>) --------------------
// For the reference shapes (hidden <= 27, latent <= 7, batch <= 12) the kernel
// keeps the hidden and latent axes of its LDS masters / register tiles in a
// permuted order in which every padded slot falls into whole MFMA k-steps, so
// contractions over hidden, latent and batch skip those k-steps:
//   hidden: storage index h -> slot j (h < 27: j = h; bias h = HP-1: j = 27;
//           pads 27..30: j = 28..31) -> position 16(ks>>2) + 4(j&3) + (ks&3),
//           ks = j>>2; slots 28..31 are exactly k-step (t=1, s=3).
//   latent: storage z -> slot j (z < 7: j = z; bias: 7; pads: 8..15) ->
//           position 4(j&3) + (j>>2); slots 0..7 are k-steps s = 0, 1.
//   batch : tile column (lane) p holds batch row 3(p>>2) + (p&3) for p&3 < 3;
//           columns 3, 7, 11, 15 (= k-step s = 3 of every product that sums
//           over the batch) are always padding.
// CP = false is the identity order (position = storage index, lane = row).
template <bool CP>
__device__ __forceinline__ int hslot_of_pos(int p) {
  return CP ? 16 * (p >> 4) + 4 * (p & 3) + ((p >> 2) & 3) : p;
}
template <bool CP>
__device__ __forceinline__ int hpos_of_storage(int h) {
  if (!CP) return h;
  const int j = h < 27 ? h : (h == HP - 1 ? 27 : h + 1);
  const int ks = j >> 2;
  return 16 * (ks >> 2) + 4 * (j & 3) + (ks & 3);
}
template <bool CP>
__device__ __forceinline__ int zslot_of_pos(int p) {
  return CP ? 4 * (p & 3) + (p >> 2) : p;
}
template <bool CP>
__device__ __forceinline__ int zpos_of_storage(int z) {
  if (!CP) return z;
  const int j = z < 7 ? z : (z == ZP - 1 ? 7 : z + 1);
  return 4 * (j & 3) + (j >> 2);
}
template <bool CP>
constexpr int h_bias_slot() { return CP ? 27 : HP - 1; }
template <bool CP>
constexpr int z_bias_slot() { return CP ? 7 : ZP - 1; }
// batch row held by tile column p, or -1 for a padding column
template <bool CP>
__device__ __forceinline__ int batch_row_of_col(int p) {
  return CP ? ((p & 3) == 3 ? -1 : 3 * (p >> 2) + (p & 3)) : p;
}

// dense global [P_PAD] (storage order) <-> LDS masters (internal order).
// 256 threads x 9 float4 = P_PAD: every thread issues all nine global loads
// before its first LDS write (one memory latency per pass, not nine), and
// gathers its LDS reads into float4 stores on the way out.  The four
// matrices start at multiples of 4 floats, so no float4 straddles two.
constexpr int STAGE_PER_THREAD = P_PAD / 4 / 256;
static_assert(STAGE_PER_THREAD * 4 * 256 == P_PAD, "staging assumes 256 threads");

// the staging thread index, opaque to the optimiser: every staging pass
// forms its LDS addresses afresh instead of keeping the ~40 addresses of the
// first pass live (spilled) across the whole launch for the write-back
// (only the 256 staging threads call the staging passes: the range keeps
// their per-element branches resolved at compile time)
__device__ __forceinline__ int stage_tid() {
  int t = (int)threadIdx.x;
  asm volatile("" : "+v"(t));
  __builtin_assume(t >= 0 && t < 256);
  return t;
}

template <bool CP>
__device__ __forceinline__ float* master_slot(int e, int i, float* sW1, float* sW4, float* sW2, float* sW3) {
  // LDS address of storage element e + i (e a multiple of 4, i in 0..3)
  if (e < OFF_W2) return &sW1[hpos_of_storage<CP>(e / DP) * S_W1 + (e % DP) + i];
  if (e < OFF_W3) {
    const int q = e - OFF_W2;
    return &sW2[zpos_of_storage<CP>(q / HP) * S_W2 + hpos_of_storage<CP>(q % HP + i)];
  }
  if (e < OFF_W4) {
    const int q = e - OFF_W3;
    return &sW3[hpos_of_storage<CP>(q / ZP) * S_W3 + zpos_of_storage<CP>(q % ZP + i)];
  }
  const int q = e - OFF_W4;
  return &sW4[(q / HP) * S_W4 + hpos_of_storage<CP>(q % HP + i)];
}

// a staging thread's share of one padded parameter-sized tensor (the load
// half of global_to_masters_o: a kernel can issue several tensors' loads in
// one memory round trip, then write them to the masters one at a time)
__device__ __forceinline__ void stage_load(const float* __restrict__ src, f32x4 (&val)[STAGE_PER_THREAD]) {
  const f32x4* s4 = reinterpret_cast<const f32x4*>(src);
#pragma unroll
  for (int k = 0; k < STAGE_PER_THREAD; ++k) val[k] = s4[threadIdx.x + 256 * k];
}

template <bool CP>
__device__ __forceinline__ void vals_to_masters_o(const f32x4 (&val)[STAGE_PER_THREAD], float* sW1, float* sW4,
                                                  float* sW2, float* sW3) {
  const int tid = stage_tid();
#pragma unroll
  for (int k = 0; k < STAGE_PER_THREAD; ++k) {
    const int e = 4 * (tid + 256 * k);
    if (e < OFF_W2 || !CP) {   // rows permuted at most: one float4
      lds_write4(master_slot<CP>(e, 0, sW1, sW4, sW2, sW3), val[k]);
    } else {
#pragma unroll
      for (int i = 0; i < 4; ++i) *master_slot<CP>(e, i, sW1, sW4, sW2, sW3) = val[k][i];
    }
  }
}

template <bool CP>
__device__ __forceinline__ void global_to_masters_o(const float* __restrict__ src, float* sW1, float* sW4,
                                                    float* sW2, float* sW3) {
  const f32x4* s4 = reinterpret_cast<const f32x4*>(src);
  f32x4 val[STAGE_PER_THREAD];
#pragma unroll
  for (int k = 0; k < STAGE_PER_THREAD; ++k) val[k] = s4[threadIdx.x + 256 * k];
  const int tid = stage_tid();
#pragma unroll
  for (int k = 0; k < STAGE_PER_THREAD; ++k) {
    const int e = 4 * (tid + 256 * k);
    if (e < OFF_W2 || !CP) {   // rows permuted at most: one float4
      lds_write4(master_slot<CP>(e, 0, sW1, sW4, sW2, sW3), val[k]);
    } else {
#pragma unroll
      for (int i = 0; i < 4; ++i) *master_slot<CP>(e, i, sW1, sW4, sW2, sW3) = val[k][i];
    }
  }
}

// CLEAR_BU: the helper-wave kernel's in-launch bias units (the last element
// of W1, W2, W3 and W4, fedmx_train_hw.hip, "bias units") are written as 0
template <bool CP, bool CLEAR_BU = false>
__device__ __forceinline__ void masters_to_global_o(float* __restrict__ dst, float* sW1, float* sW4, float* sW2,
                                                    float* sW3) {
  f32x4* d4 = reinterpret_cast<f32x4*>(dst);
  f32x4 val[STAGE_PER_THREAD];
  const int tid = stage_tid();
#pragma unroll
  for (int k = 0; k < STAGE_PER_THREAD; ++k) {
    const int e = 4 * (tid + 256 * k);
    if (e < OFF_W2 || !CP) {
      val[k] = lds_read4(master_slot<CP>(e, 0, sW1, sW4, sW2, sW3));
    } else {
#pragma unroll
      for (int i = 0; i < 4; ++i) val[k][i] = *master_slot<CP>(e, i, sW1, sW4, sW2, sW3);
    }
    if (CLEAR_BU && (e == OFF_W1 + HP * DP - 4 || e == OFF_W2 + ZP * HP - 4 || e == OFF_W3 + HP * ZP - 4 ||
                     e == OFF_W4 + DP * HP - 4))
      val[k][3] = 0.f;
  }
#pragma unroll
  for (int k = 0; k < STAGE_PER_THREAD; ++k) d4[tid + 256 * k] = val[k];
}

}  // namespace fedmx
