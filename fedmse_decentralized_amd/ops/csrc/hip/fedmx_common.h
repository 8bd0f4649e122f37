// Shared definitions for the fedmx gfx950 (CDNA4 / MI355X) kernels.
//
// Model layout: see fedmse_decentralized_amd/models/layout.py.  Four
// bias-augmented weight matrices, row-major, one flat fp32 vector per client:
//   W1a [HP=32][DP=128]  (bias b1 in column DP-1)
//   W2a [ZP=16][HP=32]   (bias b2 in column HP-1)
//   W3a [HP=32][ZP=16]   (bias b3 in column ZP-1)
//   W4a [DP=128][HP=32]  (bias b4 in column HP-1)
// The activation feeding each layer carries a constant 1 in its last padded
// row/column so that y = W_aug * [x; 1].
//
// All GEMM work uses the exact-fp32 matrix core instruction
// v_mfma_f32_16x16x4_f32 (64 lanes, D[16x16] += A[16x4] * B[4x16]).  Lane
// maps (wave64):
//   A operand : lane l supplies A[i = l & 15][k = l >> 4]
//   B operand : lane l supplies B[k = l >> 4][j = l & 15]
//   C/D       : lane l holds D[row = 4*(l >> 4) + reg][col = l & 15], reg 0..3
// Every kernel works in the "transposed" orientation: activations are
// [feature][batch] tiles with the batch on the 16 columns (lanes) so that a
// layer's D tile is directly the next layer's B operand (the next product
// sums over D's row index: lane group g supplies k = 4g + s at k-step s, which
// is exactly its own register s).  Only weight-gradient products (which sum
// over the batch = the lane index) need an LDS transpose.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace fedmx {

constexpr int DP = 128;
constexpr int HP = 32;
constexpr int ZP = 16;
constexpr int OFF_W1 = 0;
constexpr int OFF_W2 = OFF_W1 + HP * DP;
constexpr int OFF_W3 = OFF_W2 + ZP * HP;
constexpr int OFF_W4 = OFF_W3 + HP * ZP;
constexpr int P_PAD = OFF_W4 + DP * HP;  // 9216

// LDS row strides (floats) chosen so the per-lane ds_read_b128 A-operand
// reads of 16 lanes land on distinct 16-byte bank slots (stride = 4 mod 64).
constexpr int S_W1 = DP + 4;  // 132
constexpr int S_W2 = HP + 4;  // 36
constexpr int S_W3 = ZP + 4;  // 20
constexpr int S_W4 = HP + 4;  // 36
constexpr int S_T = 20;       // [feature][batch16] transpose scratch

typedef float f32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ f32x4 mfma16(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ f32x4 zero4() { return f32x4{0.f, 0.f, 0.f, 0.f}; }

// ReLU as ONE integer v_max_i32 on the float's bits: a negative float (sign
// bit set) is a negative int, so max(bits, 0) is +0.0 for it (and for -0.0)
// and the float itself otherwise -- max(x, 0) for every non-NaN x.
// fmaxf(x, 0.f) (or an fmed3 with 0 and +inf, which the compiler folds into
// it) on an MFMA result costs two VALU instructions: the compiler cannot
// prove the accumulator canonical and quiets it first (v_max_f32 x, x).
__device__ __forceinline__ float relu(float x) {
  return __builtin_bit_cast(float, max(__builtin_bit_cast(int, x), 0));
}

__device__ __forceinline__ f32x4 lds_read4(const float* p) {
  return *reinterpret_cast<const f32x4*>(p);
}
__device__ __forceinline__ void lds_write4(float* p, f32x4 v) {
  *reinterpret_cast<f32x4*>(p) = v;
}

// Order this wave's LDS accesses (other lanes' writes visible to later reads
// of this wave) without a workgroup barrier.
__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Sum across the 4 lane groups that share a column (lanes c, c+16, c+32, c+48).
__device__ __forceinline__ float sum_lane_groups(float v) {
  v += __shfl_xor(v, 16, 64);
  v += __shfl_xor(v, 32, 64);
  return v;
}
__device__ __forceinline__ double sum_lane_groups_d(double v) {
  v += __shfl_xor(v, 16, 64);
  v += __shfl_xor(v, 32, 64);
  return v;
}
__device__ __forceinline__ double wave_sum_d(double v) {
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_sum(float v) {
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

}  // namespace fedmx
