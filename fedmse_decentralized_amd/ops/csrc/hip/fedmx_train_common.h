// Shared pieces of the fused local-training kernels (fedmx_train.hip: 4 waves,
// fedmx_train8.hip: 8 waves): kernel arguments, the fused Adam update, the
// in-kernel timestamp macro and the dense <-> LDS-master parameter staging.
#pragma once
#include "fedmx_common.h"

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
  uint64_t* stamps;         // [4 waves][32] s_memtime stamps of one step (FEDMX_STAMPS builds), or null
};

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
};

// torch.optim.Adam single-tensor update (no weight decay / amsgrad):
//   m.lerp_(g, 1-b1); v.mul_(b2).addcmul_(g, g, 1-b2)
//   p.addcdiv_(m, sqrt(v)/sqrt(bc2) + eps, -lr/bc1)
// Default build: hardware sqrt / reciprocal (<= 1 ulp each) instead of the
// IEEE division sequences — 4x fewer instructions on the critical path.
template <bool PROX>
__device__ __forceinline__ void adam_update(float& p, float& m, float& v, float a, float grad, const AdamStep& K,
                                            float& prox_acc) {
  float gr = grad;
  if (PROX) {
    const float dp = p - a;
    prox_acc += dp * dp;
    gr = gr + K.two_mu * dp;
  }
  m = m + K.one_m_b1 * (gr - m);
  v = v * K.b2 + (K.one_m_b2 * gr) * gr;
#if FEDMX_EXACT_ADAM
  const float den = __fsqrt_rn(v) / K.bc2s + K.eps;
  p = p + K.neg_step_size * (m / den);
#else
  const float den = __builtin_amdgcn_sqrtf(v) * K.inv_bc2s + K.eps;
  p = p + K.neg_step_size * (m * __builtin_amdgcn_rcpf(den));
#endif
}

// Four elements (one accumulator register quad) at a time, stage-major: every
// stage issues four independent scalar ops, so consecutive VALU instructions
// never depend on each other (no hazard s_nops between dependent packed ops,
// which the packed-fp32 form paid on gfx950) and the scheduler can slot them
// into MFMA gaps.  Same operation order per element as adam_update.
template <bool PROX>
__device__ __forceinline__ void adam4(float (&p)[4], float (&m)[4], float (&v)[4], const float (&a)[4], f32x4 g,
                                      const AdamStep& K, float& prox_acc) {
#if FEDMX_EXACT_ADAM
#pragma unroll
  for (int r = 0; r < 4; ++r) adam_update<PROX>(p[r], m[r], v[r], a[r], g[r], K, prox_acc);
#else
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
  for (int r = 0; r < 4; ++r) t1[r] = K.one_m_b1 * gr[r];
#pragma unroll
  for (int r = 0; r < 4; ++r) m[r] = m[r] + K.one_m_b1 * t0[r];
#pragma unroll
  for (int r = 0; r < 4; ++r) t0[r] = v[r] * K.b2;
#pragma unroll
  for (int r = 0; r < 4; ++r) t1[r] = (K.one_m_b2 * gr[r]) * gr[r];
#pragma unroll
  for (int r = 0; r < 4; ++r) v[r] = t0[r] + t1[r];
#pragma unroll
  for (int r = 0; r < 4; ++r) t0[r] = __builtin_amdgcn_sqrtf(v[r]);
#pragma unroll
  for (int r = 0; r < 4; ++r) t0[r] = t0[r] * K.inv_bc2s + K.eps;
#pragma unroll
  for (int r = 0; r < 4; ++r) t1[r] = __builtin_amdgcn_rcpf(t0[r]);
#pragma unroll
  for (int r = 0; r < 4; ++r) t1[r] = m[r] * t1[r];
#pragma unroll
  for (int r = 0; r < 4; ++r) p[r] = p[r] + K.neg_step_size * t1[r];
#endif
}

// dense global [P_PAD] <-> LDS masters
__device__ __forceinline__ void global_to_masters(const float* __restrict__ src, float* sW1, float* sW4,
                                                  float* sW2, float* sW3) {
  const f32x4* s4 = reinterpret_cast<const f32x4*>(src);
  for (int i = threadIdx.x; i < P_PAD / 4; i += blockDim.x) {
    const f32x4 val = s4[i];
    int e = i * 4;
    if (e < OFF_W2) {
      lds_write4(&sW1[(e / DP) * S_W1 + (e % DP)], val);
    } else if (e < OFF_W3) {
      e -= OFF_W2;
      lds_write4(&sW2[(e / HP) * S_W2 + (e % HP)], val);
    } else if (e < OFF_W4) {
      e -= OFF_W3;
      lds_write4(&sW3[(e / ZP) * S_W3 + (e % ZP)], val);
    } else {
      e -= OFF_W4;
      lds_write4(&sW4[(e / HP) * S_W4 + (e % HP)], val);
    }
  }
}

__device__ __forceinline__ void masters_to_global(float* __restrict__ dst, const float* sW1, const float* sW4,
                                                  const float* sW2, const float* sW3) {
  f32x4* d4 = reinterpret_cast<f32x4*>(dst);
  for (int i = threadIdx.x; i < P_PAD / 4; i += blockDim.x) {
    int e = i * 4;
    f32x4 val;
    if (e < OFF_W2) {
      val = lds_read4(&sW1[(e / DP) * S_W1 + (e % DP)]);
    } else if (e < OFF_W3) {
      e -= OFF_W2;
      val = lds_read4(&sW2[(e / HP) * S_W2 + (e % HP)]);
    } else if (e < OFF_W4) {
      e -= OFF_W3;
      val = lds_read4(&sW3[(e / ZP) * S_W3 + (e % ZP)]);
    } else {
      e -= OFF_W4;
      val = lds_read4(&sW4[(e / HP) * S_W4 + (e % HP)]);
    }
    d4[i] = val;
  }
}


}  // namespace fedmx
