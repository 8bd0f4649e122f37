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
#include "fedmx_common.h"

namespace fedmx {

struct SegDesc {
  const float* sse;  // [n]
  int32_t n;
  int32_t batch;     // rows per vote batch (128); <= 0: single batch
  double* out;       // [2]: vote score, mean MSE
};
static_assert(sizeof(SegDesc) == 24, "SegDesc layout is shared with Python");

constexpr int SCORE_THREADS = 1024;
constexpr int SCORE_WAVES = SCORE_THREADS / 64;

__device__ __forceinline__ double block_sum_d(double v, double* s_w) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  if (lane == 0) s_w[wv] = v;
  __syncthreads();
  double r = 0.0;
#pragma unroll
  for (int w = 0; w < SCORE_WAVES; ++w) r += s_w[w];   // fixed order
  __syncthreads();
  return r;
}

// One workgroup of 1024 threads per segment.  A single-batch segment (the
// dev-set MSE: 6.7K rows at 10 clients, 53K at 80) is summed with float4 loads,
// four per thread in flight, so the latency-bound pass is a few round trips
// instead of one per 256 rows; batched segments (the 128-row vote batches)
// are reduced one batch after another.
__device__ __forceinline__ void score_reduce_block(const SegDesc& d, int d_in) {
  __shared__ double s_w[SCORE_WAVES];
  const int tid = threadIdx.x;
  const int bs = d.batch > 0 ? d.batch : (d.n > 0 ? d.n : 1);
  const int nb = (d.n + bs - 1) / bs;
  double vote = 0.0, tot = 0.0;
  if (nb == 1) {
    const float* p = d.sse;
    const int n = d.n;
    const int head = min(n, (int)((4 - ((reinterpret_cast<uintptr_t>(p) >> 2) & 3)) & 3));
    const int n4 = (n - head) >> 2;
    const f32x4* q = reinterpret_cast<const f32x4*>(p + head);
    double s = 0.0;
    if (tid < head) s += (double)p[tid];
    int i = tid;
    for (; i + 3 * SCORE_THREADS < n4; i += 4 * SCORE_THREADS) {
      const f32x4 a = q[i], b = q[i + SCORE_THREADS], c = q[i + 2 * SCORE_THREADS], e = q[i + 3 * SCORE_THREADS];
      s += (double)a[0]; s += (double)a[1]; s += (double)a[2]; s += (double)a[3];
      s += (double)b[0]; s += (double)b[1]; s += (double)b[2]; s += (double)b[3];
      s += (double)c[0]; s += (double)c[1]; s += (double)c[2]; s += (double)c[3];
      s += (double)e[0]; s += (double)e[1]; s += (double)e[2]; s += (double)e[3];
    }
    for (; i < n4; i += SCORE_THREADS) {
      const f32x4 a = q[i];
      s += (double)a[0]; s += (double)a[1]; s += (double)a[2]; s += (double)a[3];
    }
    const int t0 = head + 4 * n4;
    if (t0 + tid < n) s += (double)p[t0 + tid];
    tot = block_sum_d(s, s_w);
    vote = n > 0 ? tot / ((double)n * d_in) : 0.0;
  } else {
    for (int b = 0; b < nb; ++b) {
      const int r0 = b * bs;
      const int r1 = min(d.n, r0 + bs);
      double s = 0.0;
      for (int r = r0 + tid; r < r1; r += SCORE_THREADS) s += (double)d.sse[r];
      s = block_sum_d(s, s_w);
      tot += s;
      vote += s / ((double)(r1 - r0) * d_in);
    }
  }
  if (tid == 0) {
    d.out[0] = nb > 0 ? vote / nb : __builtin_inf();
    d.out[1] = d.n > 0 ? tot / ((double)d.n * d_in) : __builtin_nan("");
  }
}

__global__ __launch_bounds__(SCORE_THREADS) void score_reduce_kernel(const SegDesc* __restrict__ descs, int d_in) {
  score_reduce_block(descs[blockIdx.x], d_in);
}

// row copies riding the same launch (the multi-rank exchange's pack of the
// locally selected models into the send buffer: it needs the trained
// parameters only, so it runs beside the score reduction instead of as a
// launch of its own on the round's critical path)
struct CopyDesc {
  const float* src;
  float* dst;
  int32_t nfloats;   // multiple of 4
  int32_t pad;
};
static_assert(sizeof(CopyDesc) == 24, "CopyDesc layout is shared with Python");

__global__ __launch_bounds__(SCORE_THREADS) void score_reduce_copy_kernel(const SegDesc* __restrict__ descs, int n,
                                                                          int d_in,
                                                                          const CopyDesc* __restrict__ copies) {
  if ((int)blockIdx.x < n) {
    score_reduce_block(descs[blockIdx.x], d_in);
    return;
  }
  const CopyDesc c = copies[blockIdx.x - n];
  const f32x4* s4 = reinterpret_cast<const f32x4*>(c.src);
  f32x4* d4 = reinterpret_cast<f32x4*>(c.dst);
  for (int i = threadIdx.x; i < c.nfloats / 4; i += SCORE_THREADS) d4[i] = s4[i];
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
