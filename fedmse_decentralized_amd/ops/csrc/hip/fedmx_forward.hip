// Batched SAE/AE inference on gfx950: per-row reconstruction SSE and latents.
//
// Replaces every no-grad forward of the reference:
//   * vote scoring      (src/Trainer/client_trainer.py:226-238, batches of 128)
//   * FedMSE weights    (src/Trainer/client_trainer.py:118-124, whole dev set)
//   * verification      (src/Trainer/model_verifier.py:86-99)
//   * AE anomaly scores (src/Evaluator/evaluator.py:56-62)
//   * SAE latents       (src/Evaluator/evaluator.py:80-94)
// One launch covers any list of (parameter vector, row block) pairs — e.g. all
// clients' test and train sets at once.  Each 256-thread workgroup stages one
// client's weights in LDS (40 KB, padded strides) and its 4 waves stream
// 16-row tiles: 4 chained fp32 MFMA layers with the activations kept in
// registers between layers (transposed orientation, see fedmx_common.h).
#include "fedmx_forward_common.h"

namespace fedmx {

// ---------------------------------------------------------------------------
// Early scoring (engine/device_round.py): the vote / FedMSE forwards run on a
// second stream while the round's training kernel is still going, each block
// waiting for its own model's done flag (TrainArgs::done).  Spins are bounded
// by a wall-clock limit (s_memrealtime): on expiry the block records
// an error code in `err` (mapped host memory, checked by the host when it
// collects the round) and carries on, so no wait can hang the device.
// s_sleep(8) (~512 clocks) repeats between two polls of a done flag
#ifndef FEDMX_POLL_SLEEPS
#define FEDMX_POLL_SLEEPS 1
#endif
__device__ inline bool seq_before(int32_t have, int32_t want) { return (int32_t)((uint32_t)have - (uint32_t)want) < 0; }

__device__ inline void record_error(int32_t* err, int32_t code) {
  if (err != nullptr) __hip_atomic_store(err, code, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// thread 0 spins, then the whole block acquires (its later loads of the model
// see the trainer's released stores)
__device__ inline void block_wait_flag(const int32_t* flag, int32_t seq, int32_t* err, uint64_t timeout) {
  if (threadIdx.x == 0) {
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    while (seq_before(__hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT), seq)) {
      for (int i = 0; i < FEDMX_POLL_SLEEPS; ++i) __builtin_amdgcn_s_sleep(8);
      if (__builtin_amdgcn_s_memrealtime() - t0 > timeout) {
        record_error(err, 1);
        break;
      }
    }
  }
  __syncthreads();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
}

// One wave: returns once `target` training workgroups have started (the
// counter TrainArgs::started), i.e. every trainer of the round is resident.
// Launched on the scoring stream right before the waiting forward: until it
// returns, none of the forward's blocks occupies a CU a trainer still needs.
__global__ __launch_bounds__(64) void start_gate_kernel(const int32_t* started, int32_t target, int32_t* err,
                                                        uint64_t timeout) {
  if (threadIdx.x != 0) return;
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  while (seq_before(__hip_atomic_load(started, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT), target)) {
    __builtin_amdgcn_s_sleep(8);
    if (__builtin_amdgcn_s_memrealtime() - t0 > timeout) {
      record_error(err, 2);
      break;
    }
  }
}

template <bool WAIT>
__global__ __launch_bounds__(256) void fwd_rows_kernel(const FwdDesc* __restrict__ descs, int32_t* err,
                                                       uint64_t timeout) {
  __shared__ __attribute__((aligned(16))) float sW1[HP * S_W1];
  __shared__ __attribute__((aligned(16))) float sW2[ZP * S_W2];
  __shared__ __attribute__((aligned(16))) float sW3[HP * S_W3];
  __shared__ __attribute__((aligned(16))) float sW4[DP * S_W4];

  const FwdDesc d = descs[blockIdx.x];
  if (d.nrows <= 0) return;   // alignment filler of an XCD-grouped descriptor list (whole block)
  if (WAIT && d.wait_seq != 0) block_wait_flag(d.wait_flag, d.wait_seq, err, timeout);
  if (fwd_compact_ok(d)) {
    stage_params<true>(d.params, sW1, sW2, sW3, sW4);
    __syncthreads();
    fwd_rows_block<true>(d, sW1, sW2, sW3, sW4, threadIdx.x >> 6, 4, d.sse);
  } else {
    stage_params<false>(d.params, sW1, sW2, sW3, sW4);
    __syncthreads();
    fwd_rows_block<false>(d, sW1, sW2, sW3, sW4, threadIdx.x >> 6, 4, d.sse);
  }
}

// ---------------------------------------------------------------------------
// weighted_sum: out[p] = sum_k w[k] * stack[k][p], accumulated in k order with
// separately rounded multiply and add (the reference's python `sum()` over
// float32 tensors, src/Trainer/client_trainer.py:107-130), so every rank that
// runs the same plan gets a bit-identical aggregate.
__global__ __launch_bounds__(256) void weighted_sum_kernel(const float* __restrict__ stack,
                                                           const float* __restrict__ w, int K, int P,
                                                           float* __restrict__ out) {
  const int i = (blockIdx.x * blockDim.x + threadIdx.x) * 4;
  if (i >= P) return;
  f32x4 acc = zero4();
  for (int k = 0; k < K; ++k) {
    const f32x4 v = *reinterpret_cast<const f32x4*>(stack + (size_t)k * P + i);
    const float wk = w[k];
#pragma unroll
    for (int r = 0; r < 4; ++r) acc[r] = (k == 0) ? __fmul_rn(v[r], wk) : __fadd_rn(acc[r], __fmul_rn(v[r], wk));
  }
  *reinterpret_cast<f32x4*>(out + i) = acc;
}

// ---------------------------------------------------------------------------
// param_drift: out[m] = sum_t || hist[m] - new ||_2 over the 8 state-dict
// tensors t (src/Trainer/model_verifier.py:79-84).  seg[p] = tensor id of
// padded slot p (-1 = padding).  One workgroup per history vector.
__global__ __launch_bounds__(1024) void param_drift_kernel(const float* __restrict__ hist,
                                                           const float* __restrict__ newp,
                                                           const int* __restrict__ seg, float* __restrict__ out) {
  __shared__ float part[8][16];
  const float* h = hist + (size_t)blockIdx.x * P_PAD;
  float acc[8];
#pragma unroll
  for (int t = 0; t < 8; ++t) acc[t] = 0.f;
  for (int p = threadIdx.x; p < P_PAD; p += blockDim.x) {
    const int s = seg[p];
    const float df = h[p] - newp[p];
#pragma unroll
    for (int t = 0; t < 8; ++t) acc[t] += (s == t) ? df * df : 0.0f;
  }
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
#pragma unroll
  for (int t = 0; t < 8; ++t) {
    float v = wave_sum(acc[t]);
    if (lane == 0) part[t][wave] = v;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    const int nw = blockDim.x >> 6;
    float tot = 0.f;
    for (int t = 0; t < 8; ++t) {
      float s2 = 0.f;
      for (int w = 0; w < nw; ++w) s2 += part[t][w];
      tot += sqrtf(s2);
    }
    out[blockIdx.x] = tot;
  }
}


// Layout probe: D = A*B for A[i][k] = i + 100k, B[k][j] = 1000k + j through
// the documented lane maps; the host checks D against numpy (asymmetric B
// catches a transposed C/D map).
// the constant-rate clock the bounded waits use (s_memrealtime), for calibration
__global__ void probe_realtime_kernel(uint64_t* out) {
  if (threadIdx.x == 0) out[0] = __builtin_amdgcn_s_memrealtime();
}

__global__ void probe_mfma_kernel(float* out) {
  const int l = threadIdx.x;
  const float a = (float)((l & 15) + 100 * (l >> 4));
  const float b = (float)(1000 * (l >> 4) + (l & 15));
  f32x4 acc = mfma16(a, b, zero4());
#pragma unroll
  for (int r = 0; r < 4; ++r) out[(4 * (l >> 4) + r) * 16 + (l & 15)] = acc[r];
}

}  // namespace fedmx

// ============================================================================
// C ABI
// ============================================================================
extern "C" {

int fedmx_forward_rows(const void* descs, int nblocks, hipStream_t stream) {
  if (nblocks <= 0) return 0;
  hipLaunchKernelGGL(fedmx::fwd_rows_kernel<false>, dim3(nblocks), dim3(256), 0, stream,
                     reinterpret_cast<const fedmx::FwdDesc*>(descs), nullptr, (uint64_t)0);
  return (int)hipGetLastError();
}

// early scoring: the start gate, then the forward whose blocks wait for their
// model's done flag (FwdDesc::wait_seq / wait_flag); timeout in microseconds
// (timeout in s_memrealtime ticks: ops/_hip.realtime_ticks_per_us calibrates the clock)
int fedmx_forward_rows_wait(const void* descs, int nblocks, const int32_t* started, int32_t target, int32_t* err,
                            int64_t timeout_ticks, hipStream_t stream) {
  if (nblocks <= 0) return 0;
  if (started == nullptr || timeout_ticks <= 0) return -1;
  const uint64_t ticks = (uint64_t)timeout_ticks;
  hipLaunchKernelGGL(fedmx::start_gate_kernel, dim3(1), dim3(64), 0, stream, started, target, err, ticks);
  hipLaunchKernelGGL(fedmx::fwd_rows_kernel<true>, dim3(nblocks), dim3(256), 0, stream,
                     reinterpret_cast<const fedmx::FwdDesc*>(descs), err, ticks);
  return (int)hipGetLastError();
}

int fedmx_weighted_sum(const float* stack, const float* w, int K, int P, float* out, hipStream_t stream) {
  if (P % 4 != 0) return -1;
  const int nthreads = P / 4;
  hipLaunchKernelGGL(fedmx::weighted_sum_kernel, dim3((nthreads + 255) / 256), dim3(256), 0, stream, stack, w, K,
                     P, out);
  return (int)hipGetLastError();
}

int fedmx_param_drift(const float* hist, int M, const float* newp, const int* seg, float* out,
                      hipStream_t stream) {
  if (M <= 0) return 0;
  hipLaunchKernelGGL(fedmx::param_drift_kernel, dim3(M), dim3(1024), 0, stream, hist, newp, seg, out);
  return (int)hipGetLastError();
}

int fedmx_probe_realtime(uint64_t* out, hipStream_t stream) {
  hipLaunchKernelGGL(fedmx::probe_realtime_kernel, dim3(1), dim3(64), 0, stream, out);
  return (int)hipGetLastError();
}

int fedmx_probe_mfma(float* out, hipStream_t stream) {
  hipLaunchKernelGGL(fedmx::probe_mfma_kernel, dim3(1), dim3(64), 0, stream, out);
  return (int)hipGetLastError();
}

int fedmx_fwd_desc_size() { return (int)sizeof(fedmx::FwdDesc); }

}  // extern "C"
