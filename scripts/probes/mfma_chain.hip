// Probe: is a dependent chain of v_mfma_f32_16x16x4_f32 bit-identical when
// issued back to back (each MFMA reads the previous one's accumulator
// directly) and when interleaved with an independent chain?  Random fp32
// operands; 8-step chains as in the training kernel's layer-1 partial.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>

typedef float f32x4 __attribute__((ext_vector_type(4)));

// inline asm so the compiler can neither merge the identical chains nor
// reorder the issue sequence; every MFMA names its accumulator as srcC
#define MFMA(acc, a, b) asm volatile("v_mfma_f32_16x16x4_f32 %0, %1, %2, %0" : "+v"(acc) : "v"(a), "v"(b))
#define SETTLE() asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory")

__device__ void load(const float* A, const float* B, const float* A2, float* a, float* b, float* a2) {
  const int l = threadIdx.x;
  for (int j = 0; j < 8; ++j) {
    a[j] = A[j * 64 + l];
    b[j] = B[j * 64 + l];
    a2[j] = A2[j * 64 + l];
  }
}

__device__ void store(float* out, int slot, f32x4 x) {
  const int l = threadIdx.x;
  for (int r = 0; r < 4; ++r) out[(slot * 64 + l) * 4 + r] = x[r];
}

__global__ void chains(const float* A, const float* B, const float* A2, float* out) {
  float a[8], b[8], a2[8];
  load(A, B, A2, a, b, a2);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  // slot 0: back to back, one accumulator
  f32x4 x = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int j = 0; j < 8; ++j) MFMA(x, a[j], b[j]);
  SETTLE();
  // slot 1: interleaved with an independent chain (slot 3)
  f32x4 y = {0.f, 0.f, 0.f, 0.f}, z = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    MFMA(y, a[j], b[j]);
    MFMA(z, a2[j], b[j]);
  }
  SETTLE();
  // slot 2: every step waits for the previous result to settle
  f32x4 w = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    MFMA(w, a[j], b[j]);
    SETTLE();
  }
  store(out, 0, x);
  store(out, 1, y);
  store(out, 2, w);
  store(out, 3, z);
}

int main() {
  const int n = 8 * 64;
  float *hA = (float*)malloc(n * 4), *hB = (float*)malloc(n * 4), *hA2 = (float*)malloc(n * 4);
  srand(7);
  for (int i = 0; i < n; ++i) {
    hA[i] = (float)rand() / RAND_MAX * 2.f - 1.f;
    hB[i] = ((float)rand() / RAND_MAX * 2.f - 1.f) * 3.7f;
    hA2[i] = (float)rand() / RAND_MAX;
  }
  float *A, *B, *A2, *O;
  hipMalloc(&A, n * 4); hipMalloc(&B, n * 4); hipMalloc(&A2, n * 4); hipMalloc(&O, 4 * 64 * 4 * 4);
  hipMemcpy(A, hA, n * 4, hipMemcpyHostToDevice);
  hipMemcpy(B, hB, n * 4, hipMemcpyHostToDevice);
  hipMemcpy(A2, hA2, n * 4, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(chains, dim3(1), dim3(64), 0, 0, A, B, A2, O);
  float hO[4 * 64 * 4];
  hipMemcpy(hO, O, sizeof(hO), hipMemcpyDeviceToHost);
  int d_xy = 0, d_xw = 0, d_yw = 0;
  for (int i = 0; i < 256; ++i) {
    d_xy += memcmp(&hO[i], &hO[256 + i], 4) != 0;
    d_xw += memcmp(&hO[i], &hO[512 + i], 4) != 0;
    d_yw += memcmp(&hO[256 + i], &hO[512 + i], 4) != 0;
  }
  // fp32 fmaf-chain reference in the k order g = 0..3 within each step
  int d_ref = 0;
  for (int m = 0; m < 16; ++m)
    for (int nn = 0; nn < 16; ++nn) {
      float acc = 0.f;
      for (int j = 0; j < 8; ++j)
        for (int g = 0; g < 4; ++g) acc = fmaf(hA[j * 64 + g * 16 + m], hB[j * 64 + g * 16 + nn], acc);
      // D layout: lane (c = nn, g' = m / 4) holds D[m][nn] in register m % 4
      const int lane = (m / 4) * 16 + nn;
      d_ref += memcmp(&acc, &hO[(2 * 64 + lane) * 4 + (m % 4)], 4) != 0;
    }
  printf("{\"back_to_back_vs_interleaved\": %d, \"back_to_back_vs_padded\": %d, \"interleaved_vs_padded\": %d, "
         "\"padded_vs_fmaf_chain\": %d, \"of\": 256}\n", d_xy, d_xw, d_yw, d_ref);
  return 0;
}
