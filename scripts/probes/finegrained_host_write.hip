// Can the host write fine-grained device memory directly (large BAR), and do
// kernels see every rewrite?  Descriptor-ring pattern: the host rewrites a
// 1 KB block between launches (no device sync in between on the "ahead"
// arm), the kernel sums it with per-lane (vector) and uniform (scalar) loads;
// every result is checked.  Also: CPU cost of writing the block.
#include <hip/hip_runtime.h>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <cstdint>

__global__ void sum_kernel(const uint32_t* p, int n, uint32_t* out, int slot) {
  uint32_t s = 0;
  for (int i = threadIdx.x; i < n; i += blockDim.x) s += p[i];
  for (int o = 32; o >= 1; o >>= 1) s += __shfl_xor(s, o, 64);
  const uint32_t u = p[n - 1];   // uniform address: scalar load
  if (threadIdx.x == 0) {
    out[2 * slot] = s;
    out[2 * slot + 1] = u;
  }
}

int main() {
  const int n = 256;   // 1 KB
  const int iters = 256;
  uint32_t *fine, *out;
  if (hipExtMallocWithFlags((void**)&fine, 1 << 20, hipDeviceMallocFinegrained) != hipSuccess) {
    printf("{\"alloc\": false}\n");
    return 0;
  }
  (void)hipHostMalloc(&out, 8 * iters, hipHostMallocMapped);
  uint32_t want[iters], wantu[iters];
  double wr_us = 0;
  int bad_sync = 0, bad_ahead = 0;
  // arm 1: write, launch, sync (same block rewritten every iteration)
  for (int it = 0; it < iters; ++it) {
    uint32_t src[n];
    want[it] = 0;
    for (int i = 0; i < n; ++i) {
      src[i] = (uint32_t)(i * 7 + 1 + it * 131);
      want[it] += src[i];
    }
    wantu[it] = src[n - 1];
    auto t0 = std::chrono::steady_clock::now();
    std::memcpy(fine, src, sizeof(src));
    std::atomic_thread_fence(std::memory_order_seq_cst);
    auto t1 = std::chrono::steady_clock::now();
    wr_us += std::chrono::duration<double, std::micro>(t1 - t0).count();
    hipLaunchKernelGGL(sum_kernel, dim3(1), dim3(64), 0, 0, fine, n, out, it);
    (void)hipDeviceSynchronize();
    bad_sync += (out[2 * it] != want[it]) + (out[2 * it + 1] != wantu[it]);
  }
  // arm 2: a ring of 8 blocks written ahead while earlier launches run
  for (int it = 0; it < iters; ++it) {
    uint32_t* blk = fine + (it % 8) * n;
    if (it >= 8) {
      // the block's previous use must be done: wait for the launch 8 back
      while (__atomic_load_n(&out[2 * (it - 8)], __ATOMIC_ACQUIRE) == 0xffffffffu) {}
    }
    uint32_t src[n];
    want[it] = 0;
    for (int i = 0; i < n; ++i) {
      src[i] = (uint32_t)(i * 3 + 5 + it * 977);
      want[it] += src[i];
    }
    wantu[it] = src[n - 1];
    std::memcpy(blk, src, sizeof(src));
    std::atomic_thread_fence(std::memory_order_seq_cst);
    out[2 * it] = 0xffffffffu;
    hipLaunchKernelGGL(sum_kernel, dim3(1), dim3(64), 0, 0, blk, n, out, it);
    if (it % 8 == 7) (void)hipDeviceSynchronize();
  }
  (void)hipDeviceSynchronize();
  for (int it = 0; it < iters; ++it) bad_ahead += (out[2 * it] != want[it]) + (out[2 * it + 1] != wantu[it]);
  printf("{\"alloc\": true, \"host_write_1KB_us\": %.3f, \"stale_reads_sync\": %d, \"stale_reads_ring\": %d, "
         "\"checks\": %d}\n", wr_us / iters, bad_sync, bad_ahead, 4 * iters);
  return 0;
}
