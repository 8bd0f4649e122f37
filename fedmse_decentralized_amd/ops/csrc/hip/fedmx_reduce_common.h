// Per-segment score reduction (shared by score_reduce_kernel of
// fedmx_util.hip and the fused forward + reduction of fedmx_forward.hip, so
// both produce bit-identical vote scores and MSEs):
//   vote score = mean over batches of `batch` rows of the batch MSE
//   (calculate_mse_score, src/Trainer/client_trainer.py:226-241);
//   mean MSE   = sum SSE / (n * D) (fed_mse_avg / verifier,
//   src/Trainer/client_trainer.py:118-124, src/Trainer/model_verifier.py:95-99).
//
// The summation order is that of 1,024 threads: virtual thread v keeps one
// float64 accumulator over its elements, each 64-lane virtual wave sums by
// butterfly and the 16 wave sums add in wave order.  A workgroup of NT
// threads emulates them exactly: thread t runs v = t + NT j (j < 1024 / NT),
// real wave w's accumulator j holds virtual wave w + (NT / 64) j, whose
// butterfly it runs, so the order -- and the result -- does not depend on NT.
#pragma once
#include "fedmx_common.h"

namespace fedmx {

struct SegDesc {
  const float* sse;  // [n]
  int32_t n;
  int32_t batch;     // rows per vote batch (128); <= 0: single batch
  double* out;       // [2]: vote score, mean MSE
};
static_assert(sizeof(SegDesc) == 24, "SegDesc layout is shared with Python");

constexpr int SCORE_THREADS = 1024;   // the virtual workgroup whose order every NT reproduces
constexpr int SCORE_WAVES = SCORE_THREADS / 64;

template <int NT>
__device__ __forceinline__ double block_sum_virtual(double (&s)[SCORE_THREADS / NT], double* s_w) {
  constexpr int VT = SCORE_THREADS / NT;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
  for (int j = 0; j < VT; ++j) {
    double v = s[j];
    for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
    if (lane == 0) s_w[wv + (NT / 64) * j] = v;
  }
  __syncthreads();
  double r = 0.0;
#pragma unroll
  for (int w = 0; w < SCORE_WAVES; ++w) r += s_w[w];   // fixed order
  __syncthreads();
  return r;
}

// `ld1(i)` loads element i of the segment, `ld4(i)` the four elements from i
// (p + i 16-byte aligned).  A single-batch segment (the dev-set MSE: 6.7 K
// rows at 10 clients, 53 K at 80) is summed with float4 loads, four per
// virtual thread in flight; batched segments (the 128-row vote batches) are
// reduced one batch after another.  Thread 0 writes d.out.
template <int NT, class LD1, class LD4>
__device__ __forceinline__ void score_reduce_seg(const SegDesc& d, int d_in, double* s_w, LD1 ld1, LD4 ld4) {
  static_assert(NT % 64 == 0 && SCORE_THREADS % NT == 0, "NT must divide the virtual workgroup in whole waves");
  constexpr int VT = SCORE_THREADS / NT;
  const int tid = threadIdx.x;
  const int bs = d.batch > 0 ? d.batch : (d.n > 0 ? d.n : 1);
  const int nb = (d.n + bs - 1) / bs;
  double vote = 0.0, tot = 0.0;
  double s[VT];
  if (nb == 1) {
    const int n = d.n;
    const int head = min(n, (int)((4 - ((reinterpret_cast<uintptr_t>(d.sse) >> 2) & 3)) & 3));
    const int n4 = (n - head) >> 2;
#pragma unroll
    for (int j = 0; j < VT; ++j) {
      const int v = tid + NT * j;
      double a = 0.0;
      if (v < head) a += (double)ld1(v);
      int i = v;
      for (; i + 3 * SCORE_THREADS < n4; i += 4 * SCORE_THREADS) {
        const f32x4 x0 = ld4(head + 4 * i), x1 = ld4(head + 4 * (i + SCORE_THREADS)),
                    x2 = ld4(head + 4 * (i + 2 * SCORE_THREADS)), x3 = ld4(head + 4 * (i + 3 * SCORE_THREADS));
        a += (double)x0[0]; a += (double)x0[1]; a += (double)x0[2]; a += (double)x0[3];
        a += (double)x1[0]; a += (double)x1[1]; a += (double)x1[2]; a += (double)x1[3];
        a += (double)x2[0]; a += (double)x2[1]; a += (double)x2[2]; a += (double)x2[3];
        a += (double)x3[0]; a += (double)x3[1]; a += (double)x3[2]; a += (double)x3[3];
      }
      for (; i < n4; i += SCORE_THREADS) {
        const f32x4 x0 = ld4(head + 4 * i);
        a += (double)x0[0]; a += (double)x0[1]; a += (double)x0[2]; a += (double)x0[3];
      }
      const int t0 = head + 4 * n4;
      if (t0 + v < n) a += (double)ld1(t0 + v);
      s[j] = a;
    }
    tot = block_sum_virtual<NT>(s, s_w);
    vote = n > 0 ? tot / ((double)n * d_in) : 0.0;
  } else {
    for (int b = 0; b < nb; ++b) {
      const int r0 = b * bs;
      const int r1 = min(d.n, r0 + bs);
#pragma unroll
      for (int j = 0; j < VT; ++j) {
        double a = 0.0;
        for (int r = r0 + tid + NT * j; r < r1; r += SCORE_THREADS) a += (double)ld1(r);
        s[j] = a;
      }
      const double sb = block_sum_virtual<NT>(s, s_w);
      tot += sb;
      vote += sb / ((double)(r1 - r0) * d_in);
    }
  }
  if (tid == 0) {
    d.out[0] = nb > 0 ? vote / nb : __builtin_inf();
    d.out[1] = d.n > 0 ? tot / ((double)d.n * d_in) : __builtin_nan("");
  }
}

// score_reduce_seg's order with the segment staged through LDS `buf`
// (STAGE floats, 16-byte aligned), every staging load of a chunk in flight
// at once: the last-arriver reduction of fwd_reduce_kernel, whose direct
// loads would otherwise be a chain of dependent round trips (one per 128-row
// vote batch).  Single batch: virtual thread v's float4 sequence is
// q[v], q[v + 1024], ... in increasing order (score_reduce_seg's unrolled and
// remainder loops together), so chunks of STAGE / 4 float4 (a multiple of
// 1024) keep every virtual thread's order; batched: chunks of whole batches.
// `g1` / `g4` load from the segment as in score_reduce_seg.
template <int NT, int STAGE, class G1, class G4>
__device__ __forceinline__ void score_reduce_staged(const SegDesc& d, int d_in, double* s_w, float* buf, G1 g1,
                                                    G4 g4) {
  static_assert(STAGE % (4 * SCORE_THREADS) == 0 && (STAGE / 4) % NT == 0, "chunks must keep the virtual order");
  constexpr int VT = SCORE_THREADS / NT;
  constexpr int CH4 = STAGE / 4;
  const int tid = threadIdx.x;
  const int bs = d.batch > 0 ? d.batch : (d.n > 0 ? d.n : 1);
  const int nb = (d.n + bs - 1) / bs;
  if (nb > 1 && bs > STAGE) {
    score_reduce_seg<NT>(d, d_in, s_w, g1, g4);
    return;
  }
  double vote = 0.0, tot = 0.0;
  double a[VT];
  if (nb == 1) {
    const int n = d.n;
    const int head = min(n, (int)((4 - ((reinterpret_cast<uintptr_t>(d.sse) >> 2) & 3)) & 3));
    const int n4 = (n - head) >> 2;
#pragma unroll
    for (int j = 0; j < VT; ++j) {
      const int v = tid + NT * j;
      a[j] = 0.0;
      if (v < head) a[j] += (double)g1(v);
    }
    for (int c0 = 0; c0 < n4; c0 += CH4) {
      const int cnt = min(CH4, n4 - c0);
      f32x4 r[CH4 / NT];
#pragma unroll
      for (int u = 0; u < CH4 / NT; ++u)
        if (tid + NT * u < cnt) r[u] = g4(head + 4 * (c0 + tid + NT * u));
#pragma unroll
      for (int u = 0; u < CH4 / NT; ++u)
        if (tid + NT * u < cnt) lds_write4(buf + 4 * (tid + NT * u), r[u]);
      __syncthreads();
#pragma unroll
      for (int j = 0; j < VT; ++j)
        for (int i = tid + NT * j; i < cnt; i += SCORE_THREADS) {
          const f32x4 x = lds_read4(buf + 4 * i);
          a[j] += (double)x[0]; a[j] += (double)x[1]; a[j] += (double)x[2]; a[j] += (double)x[3];
        }
      __syncthreads();
    }
    const int t0 = head + 4 * n4;
#pragma unroll
    for (int j = 0; j < VT; ++j) {
      const int v = tid + NT * j;
      if (t0 + v < n) a[j] += (double)g1(t0 + v);
    }
    tot = block_sum_virtual<NT>(a, s_w);
    vote = n > 0 ? tot / ((double)n * d_in) : 0.0;
  } else {
    const int R = (STAGE / bs) * bs;   // whole batches per chunk
    for (int c0 = 0; c0 < d.n; c0 += R) {
      const int cnt = min(R, d.n - c0);
      float r[STAGE / NT];
#pragma unroll
      for (int u = 0; u < STAGE / NT; ++u)
        if (tid + NT * u < cnt) r[u] = g1(c0 + tid + NT * u);
#pragma unroll
      for (int u = 0; u < STAGE / NT; ++u)
        if (tid + NT * u < cnt) buf[tid + NT * u] = r[u];
      __syncthreads();
      for (int r0 = 0; r0 < cnt; r0 += bs) {
        const int r1 = min(cnt, r0 + bs);
#pragma unroll
        for (int j = 0; j < VT; ++j) {
          double s = 0.0;
          for (int q = r0 + tid + NT * j; q < r1; q += SCORE_THREADS) s += (double)buf[q];
          a[j] = s;
        }
        const double sb = block_sum_virtual<NT>(a, s_w);   // (its closing barrier guards the next chunk)
        tot += sb;
        vote += sb / ((double)(r1 - r0) * d_in);
      }
    }
  }
  if (tid == 0) {
    d.out[0] = nb > 0 ? vote / nb : __builtin_inf();
    d.out[1] = d.n > 0 ? tot / ((double)d.n * d_in) : __builtin_nan("");
  }
}

// Row copies riding a reduction launch (the multi-rank exchange's pack of the
// locally selected models into the send buffer: it needs the trained
// parameters only, so it runs beside the score reduction instead of as a
// launch of its own on the round's critical path).
struct CopyDesc {
  const float* src;
  float* dst;
  int32_t nfloats;   // multiple of 4
  int32_t pad;
};
static_assert(sizeof(CopyDesc) == 24, "CopyDesc layout is shared with Python");

__device__ __forceinline__ void copy_desc_block(const CopyDesc& c) {
  const f32x4* s4 = reinterpret_cast<const f32x4*>(c.src);
  f32x4* d4 = reinterpret_cast<f32x4*>(c.dst);
  for (int i = threadIdx.x; i < c.nfloats / 4; i += blockDim.x) d4[i] = s4[i];
}

}  // namespace fedmx
