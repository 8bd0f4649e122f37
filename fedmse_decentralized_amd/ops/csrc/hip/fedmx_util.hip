// Small protocol kernels on gfx950 (all launch-latency sized; the point is to
// keep every per-round reduction on the device so a round needs only a few
// host synchronisations).
//
//  * score_reduce  : per-row SSE segments -> (vote score, mean MSE)
//      vote score = mean over batches of 128 rows of the batch MSE
//      (calculate_mse_score, src/Trainer/client_trainer.py:226-241);
//      mean MSE   = sum SSE / (n * D) (fed_mse_avg / verifier,
//      src/Trainer/client_trainer.py:118-124, src/Trainer/model_verifier.py:95-99)
//  * broadcast_rows: dst[idx[i]] = src for the accepted receivers (adopt the
//      aggregate + refresh the FedProx anchor, client_trainer.py:191-195)
//  * standardize_ddof1 (LDS-staged): vote-data normalisation
//      (client_trainer.py:220-223)
#include "fedmx_reduce_common.h"

namespace fedmx {

// One workgroup of 1024 threads per segment (fedmx_reduce_common.h).
__device__ __forceinline__ void score_reduce_block(const SegDesc& d, int d_in) {
  __shared__ double s_w[SCORE_WAVES];
  const float* p = d.sse;
  score_reduce_seg<SCORE_THREADS>(
      d, d_in, s_w, [p](int i) { return p[i]; },
      [p](int i) { return *reinterpret_cast<const f32x4*>(p + i); });
}

__global__ __launch_bounds__(SCORE_THREADS) void score_reduce_kernel(const SegDesc* __restrict__ descs, int d_in) {
  score_reduce_block(descs[blockIdx.x], d_in);
}

// row copies riding the same launch (CopyDesc, fedmx_reduce_common.h)

__global__ __launch_bounds__(SCORE_THREADS) void score_reduce_copy_kernel(const SegDesc* __restrict__ descs, int n,
                                                                          int d_in,
                                                                          const CopyDesc* __restrict__ copies) {
  if ((int)blockIdx.x < n) {
    score_reduce_block(descs[blockIdx.x], d_in);
    return;
  }
  copy_desc_block(copies[blockIdx.x - n]);
}

__global__ __launch_bounds__(256) void broadcast_rows_kernel(float* __restrict__ dst0, float* __restrict__ dst1,
                                                             const int32_t* __restrict__ idx, int n,
                                                             const float* __restrict__ src, int P) {
  const int i4 = blockIdx.x * blockDim.x + threadIdx.x;  // float4 index within a row
  const int row = blockIdx.y;
  if (row >= n || i4 * 4 >= P) return;
  const f32x4 v = reinterpret_cast<const f32x4*>(src)[i4];
  const size_t base = (size_t)idx[row] * P;
  reinterpret_cast<f32x4*>(dst0 + base)[i4] = v;
  if (dst1 != nullptr) reinterpret_cast<f32x4*>(dst1 + base)[i4] = v;
}

// (x - mean) / (std_unbiased + 1e-8) per real column.  Rows are staged in LDS
// in chunks of up to 256 rows (128 KB); 1024 threads = 8 row groups x 128
// columns; column sums in float64, row groups combined in fixed order.
constexpr int STD_CHUNK = 256;
constexpr int STD_GROUPS = 8;

__global__ __launch_bounds__(1024) void standardize_lds_kernel(const float* __restrict__ x, int n, int d_in,
                                                               float* __restrict__ y) {
  __shared__ __attribute__((aligned(16))) float tile[STD_CHUNK * DP];
  __shared__ double s_part[STD_GROUPS][DP];
  __shared__ float s_mean[DP];
  __shared__ float s_den[DP];
  const int tid = threadIdx.x;
  const int col = tid & (DP - 1);
  const int grp = tid >> 7;  // row group handled by this thread
  const int nthr = blockDim.x;
  double sum = 0.0;
  for (int r0 = 0; r0 < n; r0 += STD_CHUNK) {
    const int rows = min(STD_CHUNK, n - r0);
    for (int i = tid; i < rows * DP / 4; i += nthr)
      reinterpret_cast<f32x4*>(tile)[i] = reinterpret_cast<const f32x4*>(x + (size_t)r0 * DP)[i];
    __syncthreads();
    for (int r = grp; r < rows; r += STD_GROUPS) sum += (double)tile[r * DP + col];
    __syncthreads();
  }
  s_part[grp][col] = sum;
  __syncthreads();
  double tot = 0.0;
#pragma unroll
  for (int g = 0; g < STD_GROUPS; ++g) tot += s_part[g][col];
  const double mean = tot / n;
  __syncthreads();
  double q = 0.0;
  const bool single = (n <= STD_CHUNK);
  for (int r0 = 0; r0 < n; r0 += STD_CHUNK) {
    const int rows = min(STD_CHUNK, n - r0);
    if (!single) {
      for (int i = tid; i < rows * DP / 4; i += nthr)
        reinterpret_cast<f32x4*>(tile)[i] = reinterpret_cast<const f32x4*>(x + (size_t)r0 * DP)[i];
      __syncthreads();
    }
    for (int r = grp; r < rows; r += STD_GROUPS) {
      const double df = (double)tile[r * DP + col] - mean;
      q += df * df;
    }
    __syncthreads();
  }
  s_part[grp][col] = q;
  __syncthreads();
  if (grp == 0) {
    double qq = 0.0;
#pragma unroll
    for (int g = 0; g < STD_GROUPS; ++g) qq += s_part[g][col];
    const double var = qq / (n > 1 ? (n - 1) : 1);
    s_mean[col] = (float)mean;
    s_den[col] = (float)sqrt(var) + 1e-8f;
  }
  __syncthreads();
  for (int r0 = 0; r0 < n; r0 += STD_CHUNK) {
    const int rows = min(STD_CHUNK, n - r0);
    if (!single) {
      for (int i = tid; i < rows * DP / 4; i += nthr)
        reinterpret_cast<f32x4*>(tile)[i] = reinterpret_cast<const f32x4*>(x + (size_t)r0 * DP)[i];
      __syncthreads();
    }
    for (int i = tid; i < rows * DP; i += nthr) {
      const int cc = i & (DP - 1);
      y[(size_t)r0 * DP + i] = (cc < d_in) ? (tile[i] - s_mean[cc]) / s_den[cc] : 0.f;
    }
    __syncthreads();
  }
}

}  // namespace fedmx

extern "C" {

int fedmx_score_reduce_copy(const void* descs, int n, int d_in, const void* copies, int ncopy, hipStream_t stream) {
  if (n + ncopy <= 0) return 0;
  hipLaunchKernelGGL(fedmx::score_reduce_copy_kernel, dim3(n + ncopy), dim3(fedmx::SCORE_THREADS), 0, stream,
                     reinterpret_cast<const fedmx::SegDesc*>(descs), n, d_in,
                     reinterpret_cast<const fedmx::CopyDesc*>(copies));
  return (int)hipGetLastError();
}

int fedmx_score_reduce(const void* descs, int n, int d_in, hipStream_t stream) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(fedmx::score_reduce_kernel, dim3(n), dim3(fedmx::SCORE_THREADS), 0, stream,
                     reinterpret_cast<const fedmx::SegDesc*>(descs), d_in);
  return (int)hipGetLastError();
}

int fedmx_broadcast_rows(float* dst0, float* dst1, const int32_t* idx, int n, const float* src, int P,
                         hipStream_t stream) {
  if (n <= 0) return 0;
  if (P % 4 != 0) return -1;
  const int n4 = P / 4;
  hipLaunchKernelGGL(fedmx::broadcast_rows_kernel, dim3((n4 + 255) / 256, n), dim3(256), 0, stream, dst0, dst1, idx,
                     n, src, P);
  return (int)hipGetLastError();
}

int fedmx_standardize_lds(const float* x, int n, int d_in, float* y, hipStream_t stream) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(fedmx::standardize_lds_kernel, dim3(1), dim3(1024), 0, stream, x, n, d_in, y);
  return (int)hipGetLastError();
}

int fedmx_seg_desc_size() { return (int)sizeof(fedmx::SegDesc); }

}  // extern "C"
