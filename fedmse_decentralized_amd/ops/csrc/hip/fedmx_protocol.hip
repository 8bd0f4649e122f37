// Device-resident round protocol (fixed-compat fast path): the decisions the
// host otherwise takes between stream synchronisations, as tiny kernels that
// read their inputs from device memory, so a whole federated round is one
// stream of launches with no host round trip.
//
//  * elect_kernel        : aggregator election (src/Trainer/client_trainer.py:249-285,
//                          driver src/main.py:281-288) over the all-reduced
//                          vote scores and a host-drawn noise table, the
//                          aggregation-cap bookkeeping (:78, :279, :300-303)
//                          and the FedAvg / FedMSE weights (:107-130)
//  * gather_wsum_kernel  : sum_j w_j * theta_{row_j} in selection order, the
//                          same separately-rounded fp32 order as
//                          weighted_sum_kernel (bit-identical aggregate)
//  * decide_adopt_kernel : ModelVerifier rule (src/Trainer/model_verifier.py:72-99)
//                          per hosted receiver + update_from_peers adoption
//                          (client_trainer.py:174-206): accepted receivers load
//                          the aggregate and re-anchor FedProx, the history is
//                          always the last received aggregate; the aggregator
//                          itself loads the aggregate without re-anchoring
//  * copy_f64_kernel     : device -> mapped host report slots
// Every kernel is a no-op when the election found no aggregator.
#include "fedmx_common.h"

namespace fedmx {

struct ElectArgs {
  const int32_t* sel;      // [k] global client ids, selection order
  const double* vec;       // [N][4]: vote score, -, dev MSE (seg out[0]), dev MSE (seg out[1])
  const double* noise;     // [k][k-1] U(0,1) draws, voter-major
  int32_t* agg_counts;     // [N]
  float* weights;          // [k] out
  int32_t* state;          // [4] out: aggregator (-1: none), voter
  int32_t* report;         // [2] out (mapped host memory): aggregator, voter
  int32_t k, cap, rule;    // rule 0: mean (avg / fedprox), 1: 1/MSE (mse_avg)
  int32_t pad;
};
static_assert(sizeof(ElectArgs) == 72, "ElectArgs layout is shared with Python");

__global__ void elect_kernel(const ElectArgs A) {
  if (threadIdx.x != 0) return;
  int agg = -1, voter = -1;
  for (int vi = 0; vi < A.k && agg < 0; ++vi) {
    const int v = A.sel[vi];
    const double* u = A.noise + (size_t)vi * (A.k - 1);
    int best = -1, j = 0;
    double best_s = 0.0;
    for (int ci = 0; ci < A.k; ++ci) {
      const int c = A.sel[ci];
      if (c == v) continue;
      const double f = 1.0 + (u[j++] - 0.5) * 0.0002;
      const double s = A.vec[(size_t)c * 4] * f;
      // ascending stable sort, first candidate below the cap
      if (A.agg_counts[c] < A.cap && (best < 0 || s < best_s)) {
        best = c;
        best_s = s;
      }
    }
    if (best >= 0) {
      agg = best;
      voter = v;
    }
  }
  A.state[0] = agg;
  A.state[1] = voter;
  A.report[0] = agg;
  A.report[1] = voter;
  if (agg < 0) return;
  A.agg_counts[agg] += 1;
  if (A.rule == 1) {
    double tot = 0.0;
    for (int j = 0; j < A.k; ++j) tot += 1.0 / A.vec[(size_t)A.sel[j] * 4 + 3];
    for (int j = 0; j < A.k; ++j) A.weights[j] = (float)((1.0 / A.vec[(size_t)A.sel[j] * 4 + 3]) / tot);
  } else {
    const float w = (float)(1.0 / (double)A.k);
    for (int j = 0; j < A.k; ++j) A.weights[j] = w;
  }
}

struct WsumArgs {
  const float* base;       // row-major [*, P]
  const int64_t* rows;     // [k] source rows (selection order)
  const float* weights;    // [k]
  const int32_t* state;    // aggregator flag
  float* out;              // [P]
  int32_t k, P;
};
static_assert(sizeof(WsumArgs) == 48, "WsumArgs layout is shared with Python");

__global__ __launch_bounds__(256) void gather_wsum_kernel(const WsumArgs A) {
  if (A.state[0] < 0) return;
  const int i = (blockIdx.x * blockDim.x + threadIdx.x) * 4;
  if (i >= A.P) return;
  f32x4 acc = zero4();
  for (int k = 0; k < A.k; ++k) {
    const f32x4 v = *reinterpret_cast<const f32x4*>(A.base + (size_t)A.rows[k] * A.P + i);
    const float wk = A.weights[k];
#pragma unroll
    for (int r = 0; r < 4; ++r) acc[r] = (k == 0) ? __fmul_rn(v[r], wk) : __fadd_rn(acc[r], __fmul_rn(v[r], wk));
  }
  *reinterpret_cast<f32x4*>(A.out + i) = acc;
}

struct DecideArgs {
  float* params;           // [n_local, P] hosted clients
  float* anchor;           // [n_local, P]
  float* hist;             // [n_local, P] last received aggregate
  const float* agg;        // [P]
  const int32_t* state;    // aggregator
  const double* mse;       // [n_local][2] score_reduce output; [.][1] = MSE of agg on the receiver's data
  const float* drift;      // [n_local] drift of hist vs agg
  int32_t* has_hist;       // [n_local]
  double* hist_perf;       // [n_local]
  int32_t* rejected;       // [n_local]
  double* rej_vec;         // [N] out: rejected count per receiver (global id)
  double thr, pthr;
  int32_t start, n_local, P, pad;
};
static_assert(sizeof(DecideArgs) == 120, "DecideArgs layout is shared with Python");

__global__ __launch_bounds__(256) void decide_adopt_kernel(const DecideArgs A) {
  const int a = A.state[0];
  if (a < 0) return;
  const int cl = blockIdx.x;
  const int c = A.start + cl;
  __shared__ int s_ok;
  const size_t off = (size_t)cl * A.P;
  const f32x4* src = reinterpret_cast<const f32x4*>(A.agg);
  const int n4 = A.P / 4;
  if (c == a) {  // the aggregator loads its aggregate (anchor unchanged)
    for (int i = threadIdx.x; i < n4; i += blockDim.x) reinterpret_cast<f32x4*>(A.params + off)[i] = src[i];
    return;
  }
  if (threadIdx.x == 0) {
    const double perf = 1.0 / (1.0 + A.mse[(size_t)cl * 2 + 1]);
    int ok;
    if (!A.has_hist[cl]) {
      ok = 1;  // the first received model is accepted unconditionally
      A.has_hist[cl] = 1;
    } else {
      const double change = perf - A.hist_perf[cl];
      ok = ((double)A.drift[cl] <= A.thr) && (change >= -A.pthr);
    }
    A.hist_perf[cl] = perf;
    const int rj = ok ? 0 : A.rejected[cl] + 1;
    A.rejected[cl] = rj;
    A.rej_vec[c] = (double)rj;
    s_ok = ok;
  }
  __syncthreads();
  const bool ok = s_ok != 0;
  for (int i = threadIdx.x; i < n4; i += blockDim.x) {
    const f32x4 v = src[i];
    reinterpret_cast<f32x4*>(A.hist + off)[i] = v;
    if (ok) {
      reinterpret_cast<f32x4*>(A.params + off)[i] = v;
      reinterpret_cast<f32x4*>(A.anchor + off)[i] = v;
    }
  }
}

__global__ __launch_bounds__(256) void copy_f64_kernel(double* __restrict__ dst, const double* __restrict__ src,
                                                       int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) dst[i] = src[i];
}

// two independent copies in one launch (blockIdx.y selects the pair)
__global__ __launch_bounds__(256) void copy2_f64_kernel(double* __restrict__ d0, const double* __restrict__ s0, int n0,
                                                        double* __restrict__ d1, const double* __restrict__ s1,
                                                        int n1) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (blockIdx.y == 0) {
    if (i < n0) d0[i] = s0[i];
  } else if (i < n1) {
    d1[i] = s1[i];
  }
}

}  // namespace fedmx

extern "C" {

int fedmx_copy2_f64(double* d0, const double* s0, int n0, double* d1, const double* s1, int n1, hipStream_t stream) {
  const int n = max(n0, n1);
  if (n <= 0) return 0;
  hipLaunchKernelGGL(fedmx::copy2_f64_kernel, dim3((n + 255) / 256, 2), dim3(256), 0, stream, d0, s0, n0, d1, s1, n1);
  return (int)hipGetLastError();
}

int fedmx_elect(const void* args, hipStream_t stream) {
  hipLaunchKernelGGL(fedmx::elect_kernel, dim3(1), dim3(64), 0, stream, *reinterpret_cast<const fedmx::ElectArgs*>(args));
  return (int)hipGetLastError();
}

int fedmx_gather_wsum(const void* args, hipStream_t stream) {
  const fedmx::WsumArgs& A = *reinterpret_cast<const fedmx::WsumArgs*>(args);
  if (A.P % 4 != 0 || A.k < 1) return -1;
  const int n4 = A.P / 4;
  hipLaunchKernelGGL(fedmx::gather_wsum_kernel, dim3((n4 + 255) / 256), dim3(256), 0, stream, A);
  return (int)hipGetLastError();
}

int fedmx_decide_adopt(const void* args, hipStream_t stream) {
  const fedmx::DecideArgs& A = *reinterpret_cast<const fedmx::DecideArgs*>(args);
  if (A.n_local <= 0) return 0;
  if (A.P % 4 != 0) return -1;
  hipLaunchKernelGGL(fedmx::decide_adopt_kernel, dim3(A.n_local), dim3(256), 0, stream, A);
  return (int)hipGetLastError();
}

int fedmx_copy_f64(double* dst, const double* src, int n, hipStream_t stream) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(fedmx::copy_f64_kernel, dim3((n + 255) / 256), dim3(256), 0, stream, dst, src, n);
  return (int)hipGetLastError();
}

int fedmx_protocol_sizes(int* out) {
  out[0] = (int)sizeof(fedmx::ElectArgs);
  out[1] = (int)sizeof(fedmx::WsumArgs);
  out[2] = (int)sizeof(fedmx::DecideArgs);
  return 0;
}

}  // extern "C"
