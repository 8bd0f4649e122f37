// Batched SAE/AE inference of one row block (shared by fwd_rows_kernel and
// the fused verification kernel of fedmx_protocol.hip, so both produce
// bit-identical per-row SSE): the descriptor, LDS staging of one padded
// parameter vector, and the 16-row tile loop of `nwaves` waves.
#pragma once
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

// ---- compact forward order (CP = true; shapes with d_in <= 115, hidden <= 27,
// latent <= 7 — every reference shape).  The LDS images are permuted so that
// every k-step of an MFMA whose four k values are all padding can be skipped
// (125 instead of 144 MFMAs per 16-row tile):
//   hidden: storage h -> slot j (h < 27: j = h; bias HP-1: 27; pads: 28..31)
//           at position 16(ks>>2) + 4(j&3) + (ks&3), ks = j>>2: the pads are
//           k-step (t=1, s=3) of every contraction over hidden, and the
//           k-order of the remaining steps is h = 0, 1, ..., 26, bias;
//   latent: storage z -> slot j (z < 7: j = z; bias: 7; pads: 8..15) at
//           position 4(j&3) + (j>>2): pads are k-steps s = 2, 3;
//   input : W1 columns 113 <-> 116, 114 <-> 120, 127 (bias) <-> 124, so
//           k-step (u=7, j=0) carries x[112], x[113], x[114] and the bias and
//           k-steps (7, 1..3) are padding; the rows' x[113] / x[114] reach
//           lane groups 1 / 2 by one cross-lane read each.  The nonzero
//           terms of layer 1 keep their accumulation order (bit-identical to
//           CP = false); layers 2-4 now sum in natural hidden / latent order.
// Same permutations as the training kernel's compact internal order
// (fedmx_train_common.h: hpos_of_storage / zpos_of_storage).
__device__ __forceinline__ int fwd_hpos(int h) {
  const int j = h < 27 ? h : (h == HP - 1 ? 27 : h + 1);
  const int ks = j >> 2;
  return 16 * (ks >> 2) + 4 * (j & 3) + (ks & 3);
}
__device__ __forceinline__ int fwd_zpos(int z) {
  const int j = z < 7 ? z : (z == ZP - 1 ? 7 : z + 1);
  return 4 * (j & 3) + (j >> 2);
}
__device__ __forceinline__ int fwd_xcol(int d) {
  switch (d) {
    case 113: return 116;
    case 116: return 113;
    case 114: return 120;
    case 120: return 114;
    case 127: return 124;
    case 124: return 127;
    default: return d;
  }
}
constexpr int FWD_H_BIAS_POS = 30;   // fwd_hpos(HP - 1)
constexpr int FWD_Z_BIAS_POS = 13;   // fwd_zpos(ZP - 1)

__device__ __forceinline__ bool fwd_compact_ok(const FwdDesc& d) {
  return d.d_in <= 115 && d.hidden <= 27 && d.latent <= 7;
}

template <bool CP>
__device__ __forceinline__ void stage_param4(float* sW1, float* sW2, float* sW3, float* sW4, int i, f32x4 v) {
  int e = i * 4;
  if (e < OFF_W2) {
    int r = e / DP, c = e % DP;
    if (!CP) {
      lds_write4(&sW1[r * S_W1 + c], v);
    } else if (c < 112) {
      lds_write4(&sW1[fwd_hpos(r) * S_W1 + c], v);
    } else {
#pragma unroll
      for (int k = 0; k < 4; ++k) sW1[fwd_hpos(r) * S_W1 + fwd_xcol(c + k)] = v[k];
    }
  } else if (e < OFF_W3) {
    e -= OFF_W2;
    int r = e / HP, c = e % HP;
    if (!CP) {
      lds_write4(&sW2[r * S_W2 + c], v);
    } else {
#pragma unroll
      for (int k = 0; k < 4; ++k) sW2[fwd_zpos(r) * S_W2 + fwd_hpos(c + k)] = v[k];
    }
  } else if (e < OFF_W4) {
    e -= OFF_W3;
    int r = e / ZP, c = e % ZP;
    if (!CP) {
      lds_write4(&sW3[r * S_W3 + c], v);
    } else {
#pragma unroll
      for (int k = 0; k < 4; ++k) sW3[fwd_hpos(r) * S_W3 + fwd_zpos(c + k)] = v[k];
    }
  } else {
    e -= OFF_W4;
    int r = e / HP, c = e % HP;
    if (!CP) {
      lds_write4(&sW4[r * S_W4 + c], v);
    } else {
#pragma unroll
      for (int k = 0; k < 4; ++k) sW4[r * S_W4 + fwd_hpos(c + k)] = v[k];
    }
  }
}

// The parameter vector (2,304 float4) is staged with all of a thread's
// loads issued before its LDS writes: one global round trip per workgroup of
// >= 256 threads (9 float4 per thread) instead of one per 256 / 512 elements.
template <bool CP>
__device__ __forceinline__ void stage_params(const float* __restrict__ p, float* sW1, float* sW2, float* sW3,
                                             float* sW4) {
  const f32x4* p4 = reinterpret_cast<const f32x4*>(p);
  constexpr int N4 = P_PAD / 4;
  constexpr int U = (N4 + 255) / 256;
  const int nt = blockDim.x;
  for (int i0 = threadIdx.x; i0 < N4; i0 += U * nt) {
    f32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (i0 + u * nt < N4) v[u] = p4[i0 + u * nt];
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (i0 + u * nt < N4) stage_param4<CP>(sW1, sW2, sW3, sW4, i0 + u * nt, v[u]);
  }
}

// Waves `wave` (of `nwaves`) stream the block's 16-row tiles (PREFETCH: the
// next tile's rows load while this one computes — off when every wave takes
// at most one tile, which saves 32 VGPRs): 4 chained fp32
// MFMA layers with the activations kept in registers between layers
// (transposed orientation, see fedmx_common.h).  `sse` (global or LDS, row
// indexed) receives per-row sums of squared error over d < d_in.
template <bool CP, bool PREFETCH = true>
__device__ __forceinline__ void fwd_rows_block(const FwdDesc& d, const float* sW1, const float* sW2,
                                               const float* sW3, const float* sW4, int wave, int nwaves,
                                               float* sse) {
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
  if (PREFETCH && wave < ntiles) load_tile(wave, xn);
  for (int tile = wave; tile < ntiles; tile += nwaves) {
    const int row = tile * 16 + c;
    const bool valid = row < d.nrows;
    f32x4 x[8];
    if (PREFETCH) {
#pragma unroll
      for (int u = 0; u < 8; ++u) x[u] = xn[u];
      if (tile + nwaves < ntiles) load_tile(tile + nwaves, xn);
    } else {
      load_tile(tile, x);
    }
    if (CP) {
      // k-step (7, 0) carries x[112], x[113], x[114] and the bias (W1
      // columns 116 / 120 / 124 hold W1[:, 113] / W1[:, 114] / b1)
      const float x113 = __shfl(x[7][1], c, 64);
      const float x114 = __shfl(x[7][2], c, 64);
      if (g == 1) x[7][0] = x113;
      if (g == 2) x[7][0] = x114;
      if (g == 3) x[7][0] = 1.0f;
    } else if (g == 3) {
      x[7][3] = 1.0f;  // column DP-1 feeds the b1 column of W1a
    }
    constexpr int H_BIAS = CP ? FWD_H_BIAS_POS : HP - 1;

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
        for (int j = 0; j < 4; ++j)
          if (!CP || u < 7 || j == 0) acc = mfma16(a[j], x[u][j], acc);
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float v = relu(acc[r]);
        if (16 * t + 4 * g + r == H_BIAS) v = 1.0f;
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
      for (int s = 0; s < 4; ++s)
        if (!CP || t == 0 || s < 3) z = mfma16(a[s], h1[t][s], z);
    }
    if (d.lat != nullptr && valid) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int zi = CP ? 4 * r + g : 4 * g + r;   // latent index held by D row 4g + r
        if (zi < d.latent) d.lat[(size_t)row * d.lat_stride + zi] = z[r];
      }
    }
    if (sse == nullptr) continue;
    if (CP) {
      if (g == 3) z[1] = 1.0f;  // latent position 13 feeds the b3 column of W3a
    } else if (g == 3) {
      z[3] = 1.0f;  // latent row ZP-1 feeds the b3 column of W3a
    }
    // ---- layer 3: H3^T[h][b] = relu(sum_z W3a[h][z] Z^T[z][b])
    f32x4 h3[2];
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      f32x4 acc = zero4();
      f32x4 a = lds_read4(&sW3[(16 * t + c) * S_W3 + 4 * g]);
#pragma unroll
      for (int s = 0; s < (CP ? 2 : 4); ++s) acc = mfma16(a[s], z[s], acc);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float v = relu(acc[r]);
        if (16 * t + 4 * g + r == H_BIAS) v = 1.0f;
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
        for (int s = 0; s < 4; ++s)
          if (!CP || t == 0 || s < 3) acc = mfma16(a[s], h3[t][s], acc);
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int dc = 16 * u + 4 * g + r;
        const float df = acc[r] - x[u][r];
        part += (dc < d.d_in) ? df * df : 0.0f;
      }
    }
    part = sum_lane_groups(part);
    if (g == 0 && valid) sse[row] = part;
  }
}

}  // namespace fedmx
