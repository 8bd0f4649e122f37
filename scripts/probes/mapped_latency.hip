// Latency of dependent loads by one GPU thread: device memory (HBM / L2),
// host memory mapped into the GPU (pinned, hipHostMalloc), and fine-grained
// device memory written by the host.  Pointer chase of N hops, timed with
// events over several launches.  Answers: what does one descriptor read from
// the mapped ring cost a kernel on the round's critical path?
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

__global__ void chase(const uint32_t* __restrict__ p, int hops, uint32_t* out) {
  uint32_t i = 0;
  for (int h = 0; h < hops; ++h) i = __builtin_nontemporal_load(p + i);
  out[0] = i;
}

__global__ void empty_kernel(uint32_t* out) {
  if (threadIdx.x == 1000) out[0] = 1;
}

static float time_chase(const uint32_t* p, int hops, uint32_t* out, int reps) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  hipLaunchKernelGGL(chase, dim3(1), dim3(1), 0, 0, p, hops, out);
  hipEventRecord(a, 0);
  for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(chase, dim3(1), dim3(1), 0, 0, p, hops, out);
  hipEventRecord(b, 0);
  hipEventSynchronize(b);
  float ms = 0;
  hipEventElapsedTime(&ms, a, b);
  return 1000.f * ms / reps;
}

int main() {
  const int n = 1 << 16;   // 256 KB ring: stride 4 KB + 64 B so every hop is a new line / page
  std::vector<uint32_t> h(n);
  const uint32_t stride = 1040;
  for (int i = 0; i < n; ++i) h[i] = (uint32_t)((i + stride) % n);
  uint32_t *dev, *host, *fine, *out;
  hipMalloc(&dev, n * 4);
  hipMemcpy(dev, h.data(), n * 4, hipMemcpyHostToDevice);
  hipHostMalloc(&host, n * 4, hipHostMallocMapped);
  for (int i = 0; i < n; ++i) host[i] = h[i];
  int fine_ok = hipExtMallocWithFlags((void**)&fine, n * 4, hipDeviceMallocFinegrained) == hipSuccess;
  if (fine_ok) hipMemcpy(fine, h.data(), n * 4, hipMemcpyHostToDevice);
  hipMalloc(&out, 64);
  hipDeviceSynchronize();
  const int reps = 50;
  float base = 0;
  {
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, 0, out);
    hipEventRecord(a, 0);
    for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, 0, out);
    hipEventRecord(b, 0);
    hipEventSynchronize(b);
    hipEventElapsedTime(&base, a, b);
    base = 1000.f * base / reps;
  }
  printf("{\"empty_kernel_us\": %.2f", base);
  for (int hops : {1, 4, 16, 64}) {
    printf(", \"device_hops%d_us\": %.2f", hops, time_chase(dev, hops, out, reps));
    printf(", \"mapped_host_hops%d_us\": %.2f", hops, time_chase(host, hops, out, reps));
    if (fine_ok) printf(", \"finegrained_dev_hops%d_us\": %.2f", hops, time_chase(fine, hops, out, reps));
  }
  printf("}\n");
  return 0;
}
