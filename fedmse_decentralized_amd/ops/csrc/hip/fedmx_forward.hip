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
#include "fedmx_common.h"

namespace fedmx {

struct FwdDesc {
  const float* params;  // [P_PAD] padded parameter vector
  const float* x;       // [nrows, DP] input rows (already offset to the block)
  float* sse;           // [nrows] per-row sum of squared error over d < d_in, or null
  float* lat;           // [nrows, lat_stride] latents (first `latent` columns), or null
  int32_t nrows;
  int32_t lat_stride;
  int32_t d_in;
  int32_t latent;
  int32_t hidden;
  int32_t pad0;
  int64_t pad1;
};
static_assert(sizeof(FwdDesc) == 64, "FwdDesc layout is shared with Python");

__device__ __forceinline__ void stage_params(const float* __restrict__ p, float* sW1, float* sW2, float* sW3,
                                             float* sW4) {
  const f32x4* p4 = reinterpret_cast<const f32x4*>(p);
  for (int i = threadIdx.x; i < P_PAD / 4; i += blockDim.x) {
    f32x4 v = p4[i];
    int e = i * 4;
    if (e < OFF_W2) {
      int r = e / DP, c = e % DP;
      lds_write4(&sW1[r * S_W1 + c], v);
    } else if (e < OFF_W3) {
      e -= OFF_W2;
      int r = e / HP, c = e % HP;
      lds_write4(&sW2[r * S_W2 + c], v);
    } else if (e < OFF_W4) {
      e -= OFF_W3;
      int r = e / ZP, c = e % ZP;
      lds_write4(&sW3[r * S_W3 + c], v);
    } else {
      e -= OFF_W4;
      int r = e / HP, c = e % HP;
      lds_write4(&sW4[r * S_W4 + c], v);
    }
  }
}

__global__ __launch_bounds__(256) void fwd_rows_kernel(const FwdDesc* __restrict__ descs) {
  __shared__ __attribute__((aligned(16))) float sW1[HP * S_W1];
  __shared__ __attribute__((aligned(16))) float sW2[ZP * S_W2];
  __shared__ __attribute__((aligned(16))) float sW3[HP * S_W3];
  __shared__ __attribute__((aligned(16))) float sW4[DP * S_W4];

  const FwdDesc d = descs[blockIdx.x];
  stage_params(d.params, sW1, sW2, sW3, sW4);
  __syncthreads();

  const int wave = threadIdx.x >> 6;
  const int lane = threadIdx.x & 63;
  const int c = lane & 15;  // batch column (B operand / D column) and A-operand row
  const int g = lane >> 4;  // lane group: k sub-index / D row quad
  const int ntiles = (d.nrows + 15) >> 4;

  // X[row][16u + 4g + j] for u = 0..7 : the lane's B-operand values for layer 1
  // (k-step s = 4u + j supplies k = 16u + 4g + j) and its reference values for
  // the layer-4 output rows it holds (Y^T[16u + 4g + j][row]).  The next
  // tile's rows are loaded while this one computes (one tile ahead).
  auto load_tile = [&](int tile, f32x4 (&xt)[8]) {
    const int row = tile * 16 + c;
    const int rr = row < d.nrows ? row : 0;   // padding rows: any valid row, masked at the end
    const float* xr = d.x + (size_t)rr * DP + 4 * g;
#pragma unroll
    for (int u = 0; u < 8; ++u) xt[u] = *reinterpret_cast<const f32x4*>(xr + 16 * u);
  };
  f32x4 xn[8];
  if (wave < ntiles) load_tile(wave, xn);
  for (int tile = wave; tile < ntiles; tile += 4) {
    const int row = tile * 16 + c;
    const bool valid = row < d.nrows;
    f32x4 x[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) x[u] = xn[u];
    if (tile + 4 < ntiles) load_tile(tile + 4, xn);
    if (g == 3) x[7][3] = 1.0f;  // column DP-1 feeds the b1 column of W1a

    // ---- layer 1: H1^T[h][b] = sum_d W1a[h][d] X^T[d][b]
    f32x4 h1[2];
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      f32x4 acc = zero4();
      const float* wrow = &sW1[(16 * t + c) * S_W1 + 4 * g];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        f32x4 a = lds_read4(wrow + 16 * u);
#pragma unroll
        for (int j = 0; j < 4; ++j) acc = mfma16(a[j], x[u][j], acc);
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float v = fmaxf(acc[r], 0.0f);
        if (16 * t + 4 * g + r == HP - 1) v = 1.0f;
        acc[r] = v;
      }
      h1[t] = acc;
    }
    // ---- layer 2: Z^T[z][b] = sum_h W2a[z][h] H1^T[h][b]
    f32x4 z = zero4();
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      f32x4 a = lds_read4(&sW2[c * S_W2 + 16 * t + 4 * g]);
#pragma unroll
      for (int s = 0; s < 4; ++s) z = mfma16(a[s], h1[t][s], z);
    }
    if (d.lat != nullptr && valid) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int zi = 4 * g + r;
        if (zi < d.latent) d.lat[(size_t)row * d.lat_stride + zi] = z[r];
      }
    }
    if (d.sse == nullptr) continue;
    if (g == 3) z[3] = 1.0f;  // latent row ZP-1 feeds the b3 column of W3a
    // ---- layer 3: H3^T[h][b] = relu(sum_z W3a[h][z] Z^T[z][b])
    f32x4 h3[2];
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      f32x4 acc = zero4();
      f32x4 a = lds_read4(&sW3[(16 * t + c) * S_W3 + 4 * g]);
#pragma unroll
      for (int s = 0; s < 4; ++s) acc = mfma16(a[s], z[s], acc);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float v = fmaxf(acc[r], 0.0f);
        if (16 * t + 4 * g + r == HP - 1) v = 1.0f;
        acc[r] = v;
      }
      h3[t] = acc;
    }
    // ---- layer 4 + squared error: Y^T[d][b] = sum_h W4a[d][h] H3^T[h][b]
    float part = 0.0f;
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      f32x4 acc = zero4();
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        f32x4 a = lds_read4(&sW4[(16 * u + c) * S_W4 + 16 * t + 4 * g]);
#pragma unroll
        for (int s = 0; s < 4; ++s) acc = mfma16(a[s], h3[t][s], acc);
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int dc = 16 * u + 4 * g + r;
        const float df = acc[r] - x[u][r];
        part += (dc < d.d_in) ? df * df : 0.0f;
      }
    }
    part = sum_lane_groups(part);
    if (g == 0 && valid) d.sse[row] = part;
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
  hipLaunchKernelGGL(fedmx::fwd_rows_kernel, dim3(nblocks), dim3(256), 0, stream,
                     reinterpret_cast<const fedmx::FwdDesc*>(descs));
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

int fedmx_probe_mfma(float* out, hipStream_t stream) {
  hipLaunchKernelGGL(fedmx::probe_mfma_kernel, dim3(1), dim3(64), 0, stream, out);
  return (int)hipGetLastError();
}

int fedmx_fwd_desc_size() { return (int)sizeof(fedmx::FwdDesc); }

}  // extern "C"
