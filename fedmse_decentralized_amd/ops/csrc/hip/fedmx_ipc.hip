// One-shot exchange over peer-mapped memory: the per-round all-gather (and
// the small float64 all-reduce) of the multi-GPU federation without RCCL.
//
// on the 8x MI355X node every GPU has a direct xGMI
// link to each of its 7 peers, and the round's exchange is a few hundred KB
// per rank, so what matters is latency, not ring bandwidth.  Each rank owns
// one RECEIVE AREA in uncached device memory, exported with hipIpcGetMemHandle
// and opened by every other rank (parallel/ipc.py).  A collective is two
// launches on the caller's stream, no host synchronisation and no stream
// hand-off to a communicator stream:
//
//   push:  every workgroup (chunk c, destination peer d) stores its chunk of
//          this rank's contribution straight into d's receive area (remote
//          stores over xGMI), then a system-scope release publishes flag
//          (parity, self, c) = seq in d's area;
//   wait:  every workgroup (chunk c, source peer s) spins (bounded) on flag
//          (parity, s, c) of its OWN area, then copies that chunk into the
//          caller's gathered tensor [world][n_words] (regular device memory),
//          or, for the reduce, sums the ranks' vectors in rank order.  The
//          rank's own block never goes through the area: it is read from src.
//
// Receive area layout (32-bit words):
//   data  [2 parities][world][slot_words]
//   flags [2 parities][world][IPC_MAX_CHUNKS]   (int32, zero-initialised)
// Flags carry the call's sequence number (1, 2, ...), parity = seq & 1.  Double
// buffering by parity is enough: a rank pushes call seq+2 into parity p only
// after its own wait of call seq+1 saw every peer's push of seq+1, and each
// peer pushed seq+1 after consuming call seq's data in stream order.
//
// The receive area is allocated uncached (hipDeviceMallocUncached): stores
// arriving over the fabric are never hidden behind a stale line of the
// receiver's L2.  A wait that sees no flag within the timeout records an error
// in the host-visible status word and lets the launch drain (the host raises);
// no wave spins forever.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#include "fedmx_common.h"

namespace fedmx {

constexpr int IPC_MAX_WORLD = 16;
constexpr int IPC_MAX_CHUNKS = 64;

struct IpcArgs {
  unsigned long long area[IPC_MAX_WORLD];  // receive area of every rank as mapped in this process
  const float* src;                        // this rank's contribution (n_words 32-bit words)
  void* out;                               // wait: gathered [world][n_words] f32, or reduce output f64[n_words/2]
  int* status;                             // host-visible error word (0 = ok)
  long long timeout_ticks;                 // wall_clock64() ticks
  int world, rank, n_words, slot_words;
  int parity, seq, chunks, chunk_words;
};

__device__ __forceinline__ int* ipc_flag(unsigned long long area, const IpcArgs& A, int src, int c) {
  int* flags = reinterpret_cast<int*>(area) + (size_t)2 * A.world * A.slot_words;
  return flags + ((size_t)A.parity * A.world + src) * IPC_MAX_CHUNKS + c;
}

__device__ __forceinline__ const float* ipc_data(unsigned long long area, const IpcArgs& A, int src) {
  return reinterpret_cast<const float*>(area) + ((size_t)A.parity * A.world + src) * A.slot_words;
}

// grid (chunks, world): chunk c of this rank's contribution -> rank blockIdx.y
// (its own block never leaves the rank: the wait reads it from src)
__global__ __launch_bounds__(256) void ipc_push_kernel(const IpcArgs A) {
  const int c = blockIdx.x, dst = blockIdx.y;
  if (dst == A.rank) return;
  float* d = const_cast<float*>(ipc_data(A.area[dst], A, A.rank));
  const int lo = c * A.chunk_words;
  const int hi = min(lo + A.chunk_words, A.n_words);
  for (int i = lo + 4 * (int)threadIdx.x; i < hi; i += 4 * (int)blockDim.x)
    *reinterpret_cast<f32x4*>(d + i) = *reinterpret_cast<const f32x4*>(A.src + i);
  // every thread's stores are performed at system scope before the flag
  __threadfence_system();
  __syncthreads();
  if (threadIdx.x == 0)
    __hip_atomic_store(ipc_flag(A.area[dst], A, A.rank, c), A.seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// thread 0 of the workgroup waits until flag >= seq (bounded); all threads then
// acquire at system scope
__device__ __forceinline__ void ipc_wait_flag(const IpcArgs& A, int* flag) {
  if (threadIdx.x == 0) {
    const long long t0 = (long long)wall_clock64();
    while ((int)(__hip_atomic_load(flag, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) - A.seq) < 0) {
      if ((long long)wall_clock64() - t0 > A.timeout_ticks) {
        if (A.status) __hip_atomic_store(A.status, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        break;
      }
      __builtin_amdgcn_s_sleep(2);
    }
  }
  __syncthreads();
  __atomic_thread_fence(__ATOMIC_ACQUIRE);   // system scope: no stale line of the area survives
}

// grid (chunks, world): chunk c of rank blockIdx.y's contribution, own area -> out
__global__ __launch_bounds__(256) void ipc_wait_gather_kernel(const IpcArgs A) {
  const int c = blockIdx.x, s = blockIdx.y;
  const unsigned long long mine = A.area[A.rank];
  if (s != A.rank) ipc_wait_flag(A, ipc_flag(mine, A, s, c));
  const float* src = s == A.rank ? A.src : ipc_data(mine, A, s);
  float* out = reinterpret_cast<float*>(A.out) + (size_t)s * A.n_words;
  const int lo = c * A.chunk_words;
  const int hi = min(lo + A.chunk_words, A.n_words);
  for (int i = lo + 4 * (int)threadIdx.x; i < hi; i += 4 * (int)blockDim.x)
    *reinterpret_cast<f32x4*>(out + i) = *reinterpret_cast<const f32x4*>(src + i);
}

// grid ceil(n/256): out[i] = sum over ranks (in rank order) of their f64 vectors
// (single chunk per rank); every rank forms bit-identical sums
__global__ __launch_bounds__(256) void ipc_wait_reduce_f64_kernel(const IpcArgs A) {
  const unsigned long long mine = A.area[A.rank];
  if (threadIdx.x == 0) {
    for (int s = 0; s < A.world; ++s) {
      if (s == A.rank) continue;
      int* flag = ipc_flag(mine, A, s, 0);
      const long long t0 = (long long)wall_clock64();
      while ((int)(__hip_atomic_load(flag, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) - A.seq) < 0) {
        if ((long long)wall_clock64() - t0 > A.timeout_ticks) {
          if (A.status) __hip_atomic_store(A.status, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          break;
        }
        __builtin_amdgcn_s_sleep(2);
      }
    }
  }
  __syncthreads();
  __atomic_thread_fence(__ATOMIC_ACQUIRE);
  const int n = A.n_words / 2;
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  double acc = 0.0;
  for (int s = 0; s < A.world; ++s)
    acc += reinterpret_cast<const double*>(s == A.rank ? A.src : ipc_data(mine, A, s))[i];
  reinterpret_cast<double*>(A.out)[i] = acc;
}

static int ipc_check(const IpcArgs& A) {
  if (A.world < 1 || A.world > IPC_MAX_WORLD || A.rank < 0 || A.rank >= A.world) return -1;
  if (A.n_words < 0 || A.n_words > A.slot_words || (A.n_words & 3) || (A.slot_words & 3)) return -1;
  if (A.chunks < 1 || A.chunks > IPC_MAX_CHUNKS || (A.chunk_words & 3)) return -1;
  if ((long long)A.chunks * A.chunk_words < A.n_words) return -1;
  if (A.parity != (A.seq & 1) || A.seq <= 0) return -1;
  for (int r = 0; r < A.world; ++r)
    if (!A.area[r]) return -1;
  return 0;
}

}  // namespace fedmx

extern "C" {

int fedmx_ipc_args_size(void) { return (int)sizeof(fedmx::IpcArgs); }
int fedmx_ipc_handle_size(void) { return (int)sizeof(hipIpcMemHandle_t); }
int fedmx_ipc_max_world(void) { return fedmx::IPC_MAX_WORLD; }
int fedmx_ipc_max_chunks(void) { return fedmx::IPC_MAX_CHUNKS; }

// wall_clock64() rate of the current device, kHz
int fedmx_ipc_wall_khz(void) {
  int dev = 0, khz = 0;
  if (hipGetDevice(&dev) != hipSuccess) return -1;
  if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev) != hipSuccess) return -1;
  return khz;
}

// Uncached, zeroed device allocation plus its IPC handle (handle_out: fedmx_ipc_handle_size() bytes).
int fedmx_ipc_alloc(size_t bytes, void** ptr, void* handle_out) {
  *ptr = nullptr;
  hipError_t e = hipExtMallocWithFlags(ptr, bytes, hipDeviceMallocUncached);
  if (e != hipSuccess) return (int)e;
  e = hipMemset(*ptr, 0, bytes);
  if (e == hipSuccess) e = hipDeviceSynchronize();
  if (e == hipSuccess) {
    hipIpcMemHandle_t h;
    e = hipIpcGetMemHandle(&h, *ptr);
    if (e == hipSuccess) memcpy(handle_out, &h, sizeof h);
  }
  if (e != hipSuccess) {
    (void)hipFree(*ptr);
    *ptr = nullptr;
    // a failed HIP call stays the thread's "last error": torch would report it
    // at its next unrelated call (the 8-process rehearsal's extras did)
    (void)hipGetLastError();
  }
  return (int)e;
}

int fedmx_ipc_open(const void* handle, void** ptr) {
  hipIpcMemHandle_t h;
  memcpy(&h, handle, sizeof h);
  *ptr = nullptr;
  const hipError_t e = hipIpcOpenMemHandle(ptr, h, hipIpcMemLazyEnablePeerAccess);
  if (e != hipSuccess) (void)hipGetLastError();
  return (int)e;
}

int fedmx_ipc_close(void* ptr) { return (int)hipIpcCloseMemHandle(ptr); }

int fedmx_ipc_free(void* ptr) { return (int)hipFree(ptr); }

int fedmx_ipc_push(const void* args, hipStream_t stream) {
  const fedmx::IpcArgs& A = *reinterpret_cast<const fedmx::IpcArgs*>(args);
  if (fedmx::ipc_check(A)) return -1;
  hipLaunchKernelGGL(fedmx::ipc_push_kernel, dim3(A.chunks, A.world), dim3(256), 0, stream, A);
  return (int)hipGetLastError();
}

int fedmx_ipc_wait_gather(const void* args, hipStream_t stream) {
  const fedmx::IpcArgs& A = *reinterpret_cast<const fedmx::IpcArgs*>(args);
  if (fedmx::ipc_check(A) || !A.out) return -1;
  hipLaunchKernelGGL(fedmx::ipc_wait_gather_kernel, dim3(A.chunks, A.world), dim3(256), 0, stream, A);
  return (int)hipGetLastError();
}

int fedmx_ipc_wait_reduce_f64(const void* args, hipStream_t stream) {
  const fedmx::IpcArgs& A = *reinterpret_cast<const fedmx::IpcArgs*>(args);
  if (fedmx::ipc_check(A) || !A.out || A.chunks != 1 || (A.n_words & 1)) return -1;
  const int n = A.n_words / 2;
  if (n == 0) return 0;
  hipLaunchKernelGGL(fedmx::ipc_wait_reduce_f64_kernel, dim3((n + 255) / 256), dim3(256), 0, stream, A);
  return (int)hipGetLastError();
}

}  // extern "C"
