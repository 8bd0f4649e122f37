// Detection scoring on gfx950: SAE-CEN centroid distances and exact ROC-AUC.
//
// cen_score: reference CentroidBasedOneClassClassifier (src/Model/Centroid.py:15-35)
//   fit    : sklearn StandardScaler on the train latents (float64 accumulation,
//            corrected two-pass variance, near-constant features -> scale 1)
//   score  : sklearn transforms the float32 latent array in place (float64
//            arithmetic, float32 storage) and scipy's cdist to the origin runs
//            in float64; reproduced operation by operation.
// auc: sklearn roc_curve + auc (src/Evaluator/evaluator.py:21-28) — the area
//   under the tie-aware ROC equals the Mann-Whitney statistic with ties
//   counted 1/2.  One 1024-thread workgroup per client: the smaller class is bitonic-sorted
//   in LDS (<= 8192 keys), every element of the other class binary-searches
//   it, integer counts are reduced exactly.
#include "fedmx_common.h"
#include <float.h>

namespace fedmx {

struct CenDesc {
  const float* train_lat;  // [n_train, stride]
  const float* test_lat;   // [n_test, stride]
  double* out;             // [n_test]
  int32_t n_train;
  int32_t n_test;
  int32_t latent;
  int32_t stride;
};
static_assert(sizeof(CenDesc) == 40, "CenDesc layout is shared with Python");

// All latent dimensions are reduced together: one wave-shuffle + LDS pass per
// statistic (3 block reductions instead of 3 per dimension).
__device__ __forceinline__ void block_sum_vec(double* v, int m, double* s_red /*[4][ZP]*/) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
  for (int j = 0; j < ZP; ++j) {
    if (j >= m) break;
    double x = v[j];
    for (int o = 32; o >= 1; o >>= 1) x += __shfl_xor(x, o, 64);
    if (lane == 0) s_red[wv * ZP + j] = x;
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < ZP; ++j)
    if (j < m) v[j] = s_red[j] + s_red[ZP + j] + s_red[2 * ZP + j] + s_red[3 * ZP + j];
  __syncthreads();
}

__global__ __launch_bounds__(256) void cen_score_kernel(const CenDesc* __restrict__ descs) {
  const CenDesc d = descs[blockIdx.x];
  __shared__ double s_red[4 * ZP];
  __shared__ double s_mean[ZP];
  __shared__ double s_scale[ZP];
  const int tid = threadIdx.x;
  const int m = d.latent;
  double acc[ZP], acc2[ZP];
  // mean (float64 sums of float32 values)
#pragma unroll
  for (int j = 0; j < ZP; ++j) acc[j] = 0.0;
  for (int r = tid; r < d.n_train; r += blockDim.x) {
    const float* row = d.train_lat + (size_t)r * d.stride;
#pragma unroll
    for (int j = 0; j < ZP; ++j)
      if (j < m) acc[j] += (double)row[j];
  }
  block_sum_vec(acc, m, s_red);
  double mean[ZP];
#pragma unroll
  for (int j = 0; j < ZP; ++j) mean[j] = (j < m) ? acc[j] / d.n_train : 0.0;
  // corrected two-pass variance: (sum (x-m)^2 - (sum (x-m))^2 / n) / n
#pragma unroll
  for (int j = 0; j < ZP; ++j) {
    acc[j] = 0.0;
    acc2[j] = 0.0;
  }
  for (int r = tid; r < d.n_train; r += blockDim.x) {
    const float* row = d.train_lat + (size_t)r * d.stride;
#pragma unroll
    for (int j = 0; j < ZP; ++j) {
      if (j < m) {
        const double df = (double)row[j] - mean[j];
        acc[j] += df;
        acc2[j] += df * df;
      }
    }
  }
  block_sum_vec(acc, m, s_red);
  block_sum_vec(acc2, m, s_red);
  if (tid == 0) {
    const double n = (double)d.n_train;
#pragma unroll
    for (int j = 0; j < ZP; ++j) {
      if (j >= m) break;
      const double var = (acc2[j] - acc[j] * acc[j] / n) / n;
      const double eps = DBL_EPSILON;
      const double upper = n * eps * var + (n * mean[j] * eps) * (n * mean[j] * eps);
      s_mean[j] = mean[j];
      s_scale[j] = (var <= upper) ? 1.0 : sqrt(var);
    }
  }
  __syncthreads();
  // test rows are split over gridDim.y workgroups per client (each refits the
  // tiny train statistics above)
  for (int r = blockIdx.y * blockDim.x + tid; r < d.n_test; r += blockDim.x * gridDim.y) {
    double acc = 0.0;
    for (int j = 0; j < d.latent; ++j) {
      const float t0 = (float)((double)d.test_lat[(size_t)r * d.stride + j] - s_mean[j]);
      const float t1 = (float)((double)t0 / s_scale[j]);
      const double v = (double)t1;
      acc += v * v;
    }
    d.out[r] = sqrt(acc);
  }
}

// ---------------------------------------------------------------------------
struct AucDesc {
  const void* score;     // float32 or float64 [n]
  const int32_t* label;  // [n] (non-zero = positive / abnormal)
  double* out;           // [1]
  int32_t n;
  int32_t score_is_f64;
  float score_scale;     // multiply float32 scores by this (1/D for AE SSE -> mean)
  int32_t pad;
};
static_assert(sizeof(AucDesc) == 40, "AucDesc layout is shared with Python");

constexpr int AUC_MAX_SORT = 8192;

__device__ __forceinline__ double clean(double v) {
  // numpy.nan_to_num: nan -> 0, +-inf -> +-DBL_MAX
  if (v != v) return 0.0;
  if (v == INFINITY) return DBL_MAX;
  if (v == -INFINITY) return -DBL_MAX;
  return v;
}

__device__ __forceinline__ double load_score(const AucDesc& d, int i) {
  if (d.score_is_f64) return clean(reinterpret_cast<const double*>(d.score)[i]);
  const float f = reinterpret_cast<const float*>(d.score)[i] * d.score_scale;
  return clean((double)f);
}

__global__ __launch_bounds__(1024) void auc_kernel(const AucDesc* __restrict__ descs) {
  const AucDesc d = descs[blockIdx.x];
  extern __shared__ double keys[];  // [AUC_MAX_SORT]
  __shared__ int s_cnt[2];
  __shared__ unsigned long long s_acc[2];
  const int tid = threadIdx.x;
  if (tid < 2) {
    s_cnt[tid] = 0;
    s_acc[tid] = 0ull;
  }
  __syncthreads();
  // class counts
  int npos = 0;
  for (int i = tid; i < d.n; i += blockDim.x) npos += (d.label[i] != 0);
  atomicAdd(&s_cnt[0], npos);
  __syncthreads();
  const int P = s_cnt[0];
  const int N = d.n - P;
  if (P == 0 || N == 0) {
    if (tid == 0) d.out[0] = __builtin_nan("");
    return;
  }
  // sort the smaller class
  const int sort_pos = (P <= N) ? 1 : 0;
  const int m = sort_pos ? P : N;
  if (m > AUC_MAX_SORT) {
    if (tid == 0) d.out[0] = -1.0;  // caller falls back to the host path
    return;
  }
  int m2 = 1;
  while (m2 < m) m2 <<= 1;
  // compact the class into LDS (order irrelevant: it gets sorted)
  for (int i = tid; i < m2; i += blockDim.x) keys[i] = INFINITY;
  __syncthreads();
  if (tid == 0) s_cnt[1] = 0;
  __syncthreads();
  for (int i = tid; i < d.n; i += blockDim.x) {
    const int isp = (d.label[i] != 0);
    if (isp == sort_pos) {
      const int slot = atomicAdd(&s_cnt[1], 1);
      keys[slot] = load_score(d, i);
    }
  }
  __syncthreads();
  // bitonic sort ascending (+inf padding stays at the end)
  for (int k = 2; k <= m2; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int i = tid; i < m2; i += blockDim.x) {
        const int ixj = i ^ j;
        if (ixj > i) {
          const double a = keys[i], b = keys[ixj];
          const bool up = ((i & k) == 0);
          if ((a > b) == up) {
            keys[i] = b;
            keys[ixj] = a;
          }
        }
      }
      __syncthreads();
    }
  }
  // for each element of the other class: #sorted < v and #sorted == v
  unsigned long long less = 0, eq = 0;
  for (int i = tid; i < d.n; i += blockDim.x) {
    const int isp = (d.label[i] != 0);
    if (isp == sort_pos) continue;
    const double v = load_score(d, i);
    int lo = 0, hi = m;  // lower_bound
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (keys[mid] < v) lo = mid + 1; else hi = mid;
    }
    const int lb = lo;
    hi = m;  // upper_bound
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (keys[mid] <= v) lo = mid + 1; else hi = mid;
    }
    less += (unsigned long long)lb;
    eq += (unsigned long long)(lo - lb);
  }
  atomicAdd(&s_acc[0], less);
  atomicAdd(&s_acc[1], eq);
  __syncthreads();
  if (tid == 0) {
    const double L = (double)s_acc[0], E = (double)s_acc[1];
    const double pairs = (double)P * (double)N;
    // sorted = positives: pairs (neg v, pos) with pos < v count against the AUC
    const double auc = sort_pos ? (pairs - L - 0.5 * E) / pairs : (L + 0.5 * E) / pairs;
    d.out[0] = auc;
  }
}

}  // namespace fedmx

extern "C" {

int fedmx_cen_score(const void* descs, int n, hipStream_t stream) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(fedmx::cen_score_kernel, dim3(n, 8), dim3(256), 0, stream,
                     reinterpret_cast<const fedmx::CenDesc*>(descs));
  return (int)hipGetLastError();
}

int fedmx_auc(const void* descs, int n, hipStream_t stream) {
  if (n <= 0) return 0;
  static bool attr_set = false;
  if (!attr_set) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(fedmx::auc_kernel),
                                       hipFuncAttributeMaxDynamicSharedMemorySize,
                                       fedmx::AUC_MAX_SORT * (int)sizeof(double));
    if (e != hipSuccess) return (int)e;
    attr_set = true;
  }
  hipLaunchKernelGGL(fedmx::auc_kernel, dim3(n), dim3(1024), fedmx::AUC_MAX_SORT * sizeof(double), stream,
                     reinterpret_cast<const fedmx::AucDesc*>(descs));
  return (int)hipGetLastError();
}

int fedmx_cen_desc_size() { return (int)sizeof(fedmx::CenDesc); }
int fedmx_auc_desc_size() { return (int)sizeof(fedmx::AucDesc); }

}  // extern "C"
