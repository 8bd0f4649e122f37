// Persistent fused local training with HELPER WAVES (gfx950, 8 wave64 per
// client: two per SIMD).  Same math, same per-lane data layouts and the same
// results as train_kernel<PROX, ONE=true, CP=true> (fedmx_train.hip), for the
// reference shapes (batch <= 12, hidden <= 27, latent <= 7).
//
// Why: one wave per SIMD exposes every dependency stall of the step's serial
// chain L1 -> L2 -> L3 -> L4 -> dH3 -> dZ -> dH1 -> dW1 -> Adam(W1) -> L1.
// Timing ablations of fedmx_train.hip (scripts/ab_variants.py abl_*) put the
// W4 gradient + Adam work at ~9.5 % of the launch although nothing on the
// chain waits for it before the next step's layer 4.  Here that work moves to
// a second wave on each SIMD, which issues while the first one stalls:
//
//   waves 0..3 ("main", one per SIMD): the chain exactly as in train_kernel,
//     minus dW4 / W4's Adam.  W4's rows come back each step from LDS (the
//     master for layer 4 as before, plus a copy in the dH3 A-operand layout).
//   waves 4..7 ("helper" h, on the SIMD of main w = h - 4): own W4 rows
//     [32w, 32w+32) with their Adam state (param, m, v, FedProx anchor) in
//     registers.  Between barrier #2 of step s and barrier #1 of step s+1 a
//     helper reads main w's dY^T / H3^T tiles, forms dW4 (12 MFMAs), runs the
//     Adam update and publishes W4(s+1) (master rows + A-operand copy).  The
//     two workgroup barriers of the step are the only synchronisation.
//   validation: all 8 waves share the epoch's validation batches -- in a
//     second workgroup per client, the "validator", while the trainer runs
//     ahead into the next epoch (asynchronous validation, below), or in the
//     trainer itself at every epoch's end (launches whose 2k workgroups would
//     not all be resident at once).
//
// Barrier sequence (every wave executes exactly this): prologue staging
// (2 per state tensor), per training step #1 / #2, per epoch: masters
// published, loss exchange, snapshot (asynchronous: masters published, one
// decision barrier at step AV_CHECK, the publication; a roll-back: one);
// epilogue write-back.
#include "fedmx_train_common.h"

// Per-instantiation choices.  Each is a bit mask over the kernel's
// instantiations -- bit 0: batch <= 12 without FedProx (the benchmark's),
// bit 1: batch <= 12 with FedProx, bit 2: MULTI (batch > 12, either) --
// because the same removal of VALU work measured faster in one and slower in
// another (r5 A/B, one box, two passes, train launch us: plain / FedProx /
// batch 64):
//   scaled Adam only       885.5 / 973 / 698.5
//   + bias units + masks   900.5 / 953 / 680
//   + ping-pong            877.5 / 977 / 696.5
//   + all three            889   / 986 / 661
// so each instantiation gets its fastest combination.
//
// BIAS_UNITS: the constant-1 "bias units" of H1, Z and H3 (the slots that feed
// b2, b3 and b4 through the next layer's bias column) come out of the products
// themselves instead of being set by a select after every product: inside the
// launch W1's bias row, W2's bias row and W3's bias row hold a single 1 (in the
// input-bias column, the H1-bias column and the Z-bias column), so
// relu(1 * 1) = 1, 1 * 1 = 1 and relu(1 * 1) = 1 exactly; W4's row of the
// input-bias "feature" holds a 1 in the H3-bias column, so X's constant-1
// column is reconstructed exactly and needs no mask in the loss and dY.  Their
// gradients are zero (the dH1 / dZ / dH3 masks already exclude the bias slots;
// the bias feature's dY is exactly 0), so Adam never moves them; the global
// parameters (aggregation, checkpoints) never see them: set on staging in,
// cleared on staging out (bias_units_*).
constexpr int BIAS_UNITS = 6;
// VALUE_MASKS: the backward masks test values, not slot tables: every padded
// hidden / latent slot holds exactly 0 (zero weights, relu(0) = 0, zero
// gradients), so "real and positive" is "positive" except at the one bias
// slot, which a per-lane threshold (2 > the bias unit's 1) or a single-slot
// select excludes: one compare + select per element instead of compare +
// scalar AND + select, and no select at all on the latent axis but the bias
// slot's
constexpr int VALUE_MASKS = 6;
// PINGPONG: the step loop unrolled by two with the current / prefetched chunk
// buffers swapping roles (instead of copying the prefetched chunk's 16
// registers into the current one after every step)
constexpr int PINGPONG = 5;
// SPLIT_CHAINS (fedmx_train.hip, the same mask keeps the two kernels
// bit-identical): the L2 / dZ products as two accumulator chains (chain2)
// W4FLAG_ROLES: the FedProx instantiation hands W4(s+1) and each step's Adam
// scalars from helper w to main w through an LDS flag the main waits on right
// before layer 4, and barrier #1 is a main-waves-only LDS flag exchange: the
// helpers then no longer gate the mains' layer-1 exchange (r4 A/B: FedProx
// launch -3.3 %, the plain launch +6 % -- without FedProx the helpers' path is
// short enough that the flag polls only add latency to the mains')
constexpr int W4FLAG_ROLES = 2;
// bound on one flag wait (polls); a wait that runs out marks the launch failed
// (epochs_run = -1000) instead of hanging the GPU
// (~1 ms of polls, vs ~3 us for a whole training step; after one wait has run
// out the wave waits no more, so a broken hand-off ends the launch quickly)
constexpr int HW_SPIN_LIMIT = 1 << 16;
// (Rounds 3-5 also measured, and removed: a software-pipelined W1 Adam /
// layer-1 (+4.2 %), layer 1's second hidden tile and its backward on the
// helpers (+22.6 %), the eight dH3 partial reads issued together (+6.5 %),
// iglp_opt(1) / no scheduling hint (+1.6 / +12.6 %), a step loop with no
// workgroup barrier at all (LDS flags for barrier #2 too), packed-fp32 Adam
// (+2 %), X's bias column set after each load instead of stored in the packed
// rows, and the timing-only ablations of the step; source in git history,
// numbers in profiles/r3_train_hw_experiments.md, r4_train_hw_experiments.md,
// r5_train_kernel_ab.md.)

// Asynchronous validation (TRAIN_FLAG_ASYNC_VALID, set by the launcher when
// TrainArgs.vws is given and 2k workgroups fit the device at once): the
// epoch-end validation pass (~24,000 cycles of the trainer's 8 waves per epoch,
// r5 stamps) moves to a second workgroup per client, the "validator", on
// another CU.  At the end of epoch e the trainer copies its LDS masters to
// the workspace (write-through stores, drained, then one flag: no fences),
// keeps its waves' Adam moments in a per-thread record of its own and goes on
// with epoch e+1 without waiting.  The validator runs the
// same validation code on the copy (same tiles, waves and fp64 order), writes
// the valid loss, the best snapshot (save_model) and a stamped decision word
// (stop or continue, the best epoch).  The trainer reads that word at step
// AV_CHECK of epoch e+1 (or at its end, for epochs that short): on "stop" it
// discards the speculative steps -- masters and moments come back from the
// workspace, the step count from a register -- and leaves as the synchronous
// kernel would have after epoch e.  Every result (parameters, moments, best
// snapshot, tracking, epochs run, best epoch) is the synchronous kernel's
// (tests/test_async_validation_gpu.py).  Measured (profiles/r5_train_kernel_ab.md):
// plain launch 874 -> 842 us, bench +3.5 %, paper configuration +4.6 %; the
// FedProx and batch > 12 instantiations measured slower and keep the
// synchronous epoch tail.
constexpr int ASYNC_VALID = 1;   // instantiation mask (bit 0 plain, bit 1 FedProx, bit 2 batch > 12)
constexpr int AV_CHECK = 6;      // step of epoch e+1 before which the trainer needs epoch e's decision
// wall_clock64() ticks (100 MHz on gfx950) one cross-workgroup wait may take
// before the launch reports itself failed (an epoch of a large client can
// take many milliseconds; a validator that never runs must not hang the GPU)
constexpr long long AV_TIMEOUT = 1000000000LL;
static_assert(AV_CHECK % 2 == 0, "the ping-pong step loop checks between step pairs");

typedef int i32x4 __attribute__((ext_vector_type(4)));
// (Round 3 also measured, and removed, seven schedule variants of this step --
// dH3 partial reads in flight together, the bias column by address select,
// helper-formed next-step Adam scalars, a software-pipelined tail, helper
// delays and issue priorities for either role: all slower or neutral,
// profiles/r3_train_hw_experiments.md; source in git history before this note.)

namespace fedmx {
namespace hw {

// In-kernel phase stamps (-DFEDMX_STAMPS=1 builds, scripts/train_stamps.py):
// row w8 (0..7: mains then helpers) of A.stamps, columns as in fedmx_train.hip.
#if FEDMX_STAMPS
#define HSTAMP(cond, i)                                                                         \
  do {                                                                                          \
    if ((cond) && A.stamps != nullptr && blockIdx.x == 0 && lane == 0)                          \
      A.stamps[w8 * 32 + (i)] = __builtin_amdgcn_s_memtime();                                  \
  } while (0)
// asynchronous-validation timeline of client slot 0 (trainer and validator,
// wave 0 lane 0): wall_clock64() ticks (one clock for every CU)
#define AVSTAMP(cond, i)                                                                     \
  do {                                                                                       \
    if ((cond) && A.stamps != nullptr && kslot == 0 && threadIdx.x == 0)                     \
      A.stamps[(i)] = (uint64_t)wall_clock64();                                              \
  } while (0)
#else
#define HSTAMP(cond, i) \
  do {                  \
  } while (0)
#define AVSTAMP(cond, i) \
  do {                   \
  } while (0)
#endif

constexpr int L_W1 = HP * S_W1;          // 4224
constexpr int L_W4 = DP * S_W4;          // 4608
constexpr int L_W2 = ZP * S_W2;          // 576
constexpr int L_W3 = HP * S_W3;          // 640
constexpr int L_RED = 4 * 2 * 64 * 4;    // 2048
constexpr int L_T32 = 32 * S_T;          // 640
constexpr int L_T16 = 16 * S_T;          // 320
constexpr int L_SCR = 4 * L_T32 + 2 * L_T16;  // 3200 per main wave (dY^T, H3^T, H1^T, dH3^T | Z^T, dZ^T)
constexpr int L_Q4 = 4 * 4 * 64 * 4;     // 4096 W4 rows in the dH3 A-operand layout [w][v][t][lane][4]
constexpr int L_TOTAL = L_W1 + L_W4 + L_W2 + L_W3 + 3 * L_RED + 4 * L_SCR + L_Q4 + 128;
static_assert(L_TOTAL * 4 <= 160 * 1024, "LDS budget");

// asynchronous validation workspace of one client slot (floats): the LDS
// masters region [sW1 | sW4 | sW2 | sW3] as it is (padded strides, bias
// units), then the flags (ready: u64 at 0, the epoch's FedProx term: f64 at 2,
// decision: u64 at 32, its own 128-byte line), then every thread's Adam
// moments (mains: M, V slabs, 40 floats; helpers: M4, V4, 32)
constexpr int AV_L_M = L_W1 + L_W4 + L_W2 + L_W3;   // 10048
constexpr int AV_FLAGS = 64;
constexpr int AV_R = 512 * 40;
constexpr int AV_SLOT = AV_L_M + AV_FLAGS + AV_R;
static_assert(AV_L_M % 4 == 0 && AV_SLOT % 64 == 0, "workspace alignment");
constexpr unsigned AV_FAIL = 0xffffffffu;   // decision word (low half) of a validator whose wait ran out
// Memory-model argument (VERDICT r5 Next #2c).  Trainer and validator run on
// different CUs, usually on different XCDs, whose L2s are not coherent with
// each other; each CU's vector L1 is never refreshed by another CU's stores.
// The two hand-offs therefore follow the write-through recipe of
// cdna_hip_programming.md §6 Guideline 16 and MI355X_MICROARCH.md
// § visibility, which measures them valid without release / acquire fences
// (each fence: ~1.7-6.5 us, an L2 write-back or L1 invalidate):
//  * snapshot + FedProx term, trainer -> validator (R1, table row 1 "ONE lane
//    of each storing workgroup, for ALL that workgroup's stores: an sc1 flag
//    store"):  (1) EVERY store of the payload is sc1: 16-B
//    raw_buffer_store_b128 with aux 16 (av_store16) for the masters, an 8-B
//    relaxed agent-scope atomic store (global_store_dwordx2 sc1) for the
//    FedProx term;  (2) every storing wave drains (s_waitcnt vmcnt(0),
//    av_drain) before the workgroup barrier, and thread 0 then stores the
//    ready flag -- after its own drain of the FedProx term -- as an 8-B
//    relaxed agent-scope atomic (sc1);  (3) the validator's thread 0 polls
//    the flag with relaxed agent-scope atomic loads (global_load_dwordx2 sc1),
//    reads the FedProx term the same way after the match, and every other
//    wave loads only behind the workgroup barrier thread 0 then joins;
//    (4) EVERY load of the payload is an sc1 buffer load to registers
//    (av_load16, raw_buffer_load_b128 aux 16: it bypasses the validator CU's
//    L1, and sc1 makes the access coherent at agent scope, i.e. it is served
//    from the memory side of the XCD L2s, where the trainer's write-through
//    stores have landed before its flag).  The workspace is hipMalloc memory
//    (the torch caching allocator) and both roles run one workgroup per CU
//    (132 KB of LDS each): the row's memory / occupancy cells hold too.
//  * decision, validator -> trainer (R2): the data is the flag -- one aligned
//    8-B granule {launch number vseq, stop bit, epoch + 1, best epoch + 1}
//    written by one relaxed agent-scope atomic store and polled by one
//    relaxed agent-scope atomic load; the trainer uses nothing but the
//    granule's own bits.  The best snapshot the validator writes (plain
//    stores) is read only after the launch (kernel boundary).
//  * the trainer's own moment records (av_rec) and its roll-back reads of the
//    snapshot (sc1 loads of its own sc1 stores) stay on one CU.
// Every wait is bounded (AV_TIMEOUT); a launch number per launch tags every
// flag, so stale words of earlier launches never match (zeroed once).
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ __amdgpu_buffer_rsrc_t av_rsrc(float* p) {
  return __builtin_amdgcn_make_buffer_rsrc(p, (short)0, AV_L_M * 4, 0x00020000);
}
__device__ __forceinline__ void av_store16(__amdgpu_buffer_rsrc_t r, int i, f32x4 v) {
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), r, i * 16, 0, 16);   // aux 16: sc1
}
__device__ __forceinline__ f32x4 av_load16(__amdgpu_buffer_rsrc_t r, int i) {
  return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, i * 16, 0, 16));   // sc1
}
__device__ __forceinline__ void av_drain() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }
// flags / decisions / the FedProx term: 8-byte GLOBAL (never flat) agent-scope atomics
typedef __attribute__((address_space(1))) unsigned long long gu64;
__device__ __forceinline__ unsigned long long av_ld(unsigned long long* p) {
  return __hip_atomic_load((gu64*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void av_st(unsigned long long* p, unsigned long long v) {
  __hip_atomic_store((gu64*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// (thread 0 of a trainer) the low half of the decision word `dec` once it is
// stamped `seq` and covers epoch need - 1, or AV_FAIL when the wait runs out.
// (Inlined: a call anywhere in the step loop, even on its cold check branch,
// makes the register allocator spill around it inside the loop.)
__device__ __forceinline__ unsigned av_wait_decision(unsigned long long* dec, unsigned long long seq, int need,
                                                     long long timeout) {
  const long long t0 = (long long)wall_clock64();
  for (;;) {
    const unsigned long long d = av_ld(dec);
    if ((d & 0xffffffff00000000ull) == seq) {
      const unsigned lo = (unsigned)d;
      if (lo == AV_FAIL || (int)((lo >> 1) & 0x7fffu) >= need) return lo;
    }
    if ((long long)wall_clock64() - t0 > timeout) return AV_FAIL;
    __builtin_amdgcn_s_sleep(2);
  }
}

// main-wave optimizer state: W1 column block (MFMA A-operand layout) + small tile
struct MSlab {
  float q1[2][2][4];
  float o[4];
};
// helper-wave optimizer state: W4 row block (D layout, see fedmx_train.hip)
struct HSlab {
  float q4[2][2][4];
};

// storage-order float4 index of each bias-unit entry (the last element of
// W1 [HP][DP], W2 [ZP][HP], W3 [HP][ZP]: their bias row, bias column)
constexpr int BU_W1 = (OFF_W1 + HP * DP - 4) / 4;
constexpr int BU_W2 = (OFF_W2 + ZP * HP - 4) / 4;
constexpr int BU_W3 = (OFF_W3 + HP * ZP - 4) / 4;
// and W4's row for the input-bias "feature" DP-1, H3-bias column: the
// reconstruction of X's constant-1 column is then exactly 1, so its error
// (and its dY, and its gradient) is 0 without a select
constexpr int BU_W4 = (OFF_W4 + DP * HP - 4) / 4;
// staging thread's share (stage_load layout): mark / clear the bias units
__device__ __forceinline__ void bias_units_set(f32x4 (&val)[STAGE_PER_THREAD], float one) {
#pragma unroll
  for (int k = 0; k < STAGE_PER_THREAD; ++k) {
    const int q = threadIdx.x + 256 * k;
    if (q == BU_W1 || q == BU_W2 || q == BU_W3 || q == BU_W4) val[k][3] = one;
  }
}

struct Lane {
  float* w1;   // sW1 + c*S_W1 + 32w + 4g
  float* w4;   // sW4 + (32w+4g)*S_W4 + c
  float* own;
  int own_stride;
};
__device__ __forceinline__ void w1_to_lds(const MSlab& o, const Lane& L) {
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int v = 0; v < 2; ++v)
      lds_write4(L.w1 + 16 * t * S_W1 + 16 * v, f32x4{o.q1[t][v][0], o.q1[t][v][1], o.q1[t][v][2], o.q1[t][v][3]});
}
__device__ __forceinline__ void own_to_lds(const MSlab& o, const Lane& L) {
#pragma unroll
  for (int r = 0; r < 4; ++r) L.own[r * L.own_stride] = o.o[r];
}
__device__ __forceinline__ void lds_to_mslab(MSlab& o, const Lane& L) {
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int v = 0; v < 2; ++v) {
      const f32x4 q = lds_read4(L.w1 + 16 * t * S_W1 + 16 * v);
#pragma unroll
      for (int r = 0; r < 4; ++r) o.q1[t][v][r] = q[r];
    }
#pragma unroll
  for (int r = 0; r < 4; ++r) o.o[r] = L.own[r * L.own_stride];
}
__device__ __forceinline__ void w4_to_lds(const HSlab& o, const Lane& L) {
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int v = 0; v < 2; ++v) L.w4[(16 * v + r) * S_W4 + 16 * t] = o.q4[v][t][r];
}
__device__ __forceinline__ void lds_to_hslab(HSlab& o, const Lane& L) {
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int v = 0; v < 2; ++v) o.q4[v][t][r] = L.w4[(16 * v + r) * S_W4 + 16 * t];
}

// asynchronous validation: a thread's Adam moments <-> its workspace record
// (registers as they are: the scaled form of ADAM_SCALED included)
__device__ __forceinline__ f32x4 q4v(const float (&a)[4]) { return f32x4{a[0], a[1], a[2], a[3]}; }
__device__ __forceinline__ void q4set(float (&a)[4], f32x4 v) {
#pragma unroll
  for (int r = 0; r < 4; ++r) a[r] = v[r];
}
__device__ __forceinline__ void mslab_dump(float* rec, const MSlab& M, const MSlab& V) {
  f32x4* q = reinterpret_cast<f32x4*>(rec);
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int v = 0; v < 2; ++v) {
      q[2 * t + v] = q4v(M.q1[t][v]);
      q[5 + 2 * t + v] = q4v(V.q1[t][v]);
    }
  q[4] = q4v(M.o);
  q[9] = q4v(V.o);
}
__device__ __forceinline__ void mslab_restore(const float* rec, MSlab& M, MSlab& V) {
  const f32x4* q = reinterpret_cast<const f32x4*>(rec);
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int v = 0; v < 2; ++v) {
      q4set(M.q1[t][v], q[2 * t + v]);
      q4set(V.q1[t][v], q[5 + 2 * t + v]);
    }
  q4set(M.o, q[4]);
  q4set(V.o, q[9]);
}
__device__ __forceinline__ void hslab_dump(float* rec, const HSlab& M, const HSlab& V) {
  f32x4* q = reinterpret_cast<f32x4*>(rec);
#pragma unroll
  for (int v = 0; v < 2; ++v)
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      q[2 * v + t] = q4v(M.q4[v][t]);
      q[4 + 2 * v + t] = q4v(V.q4[v][t]);
    }
}
__device__ __forceinline__ void hslab_restore(const float* rec, HSlab& M, HSlab& V) {
  const f32x4* q = reinterpret_cast<const f32x4*>(rec);
#pragma unroll
  for (int v = 0; v < 2; ++v)
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      q4set(M.q4[v][t], q[2 * v + t]);
      q4set(V.q4[v][t], q[4 + 2 * v + t]);
    }
}

// compact-order product over the two halves of the hidden axis (7 k-steps).
// SPLIT (SPLIT_CHAINS, per instantiation; fedmx_train.hip the same
// order): each half in its own accumulator, interleaved, then added -- a
// 4-long dependent MFMA chain instead of 7 (40-cycle result latency vs
// 32-cycle issue) on the main waves' serial path (z after barrier #1, dZ
// after barrier #2)
template <bool SPLIT>
__device__ __forceinline__ f32x4 chain2(f32x4 a0, f32x4 a1, f32x4 b0, f32x4 b1) {
  f32x4 x = zero4();
  if (SPLIT) {
    f32x4 y = zero4();
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      x = mfma16(a0[s], b0[s], x);
      if (s < 3) y = mfma16(a1[s], b1[s], y);
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) x[r] = x[r] + y[r];
  } else {
#pragma unroll
    for (int s = 0; s < 4; ++s) x = mfma16(a0[s], b0[s], x);
#pragma unroll
    for (int s = 0; s < 3; ++s) x = mfma16(a1[s], b1[s], x);
  }
  return x;
}

struct XChunk {
  f32x4 f0, f1, b0, b1;
};
// one 16-row validation tile's rows as the lane holds them (valid_compute)
struct VTile {
  f32x4 xf[4][2];
};

// MULTI (batch > 12; VERDICT r3 Next #7, the thesis's batch-64 runs): the
// step loop runs over 16-row chunks (a batch's chunks in turn, natural batch
// order, 4 batch k-steps); every chunk is a forward / backward with the
// step's two barriers, the weight gradients accumulate over the batch's
// chunks, and Adam plus the W4 / scalar hand-off follow the batch's last
// chunk.  Loss and gradient scales use the batch's row count, the column
// masks the chunk's.  (A first version in 12-row compact-order chunks ran
// 15 % slower than the 4-wave kernel at batch 64: six chunks per batch
// instead of four.)
template <bool PROX, bool MULTI>
__global__ __launch_bounds__(512, 1) void train_kernel_hw(const TrainArgs A) {
  // this instantiation's bit in the BIAS_UNITS, VALUE_MASKS, PINGPONG,
  // SPLIT_CHAINS, W4FLAG_ROLES and ASYNC_VALID masks
  constexpr int ROLE = MULTI ? 4 : (PROX ? 2 : 1);
  // W4 / Adam scalars handed over by LDS flag (per-helper K slots), barrier #1
  // a main-waves-only flag exchange
  constexpr bool W4FLAG = (W4FLAG_ROLES & ROLE) != 0;
  constexpr bool CP = true;
  constexpr bool CPB = !MULTI;       // compact batch order (12 rows of 16 columns)
  constexpr int KB = CPB ? 3 : 4;    // k-steps of products over the batch
  constexpr int KZ = 2;   // k-steps of products over the latent axis
  constexpr bool BU = (BIAS_UNITS & ROLE) != 0;
  constexpr bool VMASK = (VALUE_MASKS & ROLE) != 0;
  constexpr bool PPONG = (PINGPONG & ROLE) != 0;
  constexpr bool SPLIT = (SPLIT_CHAINS & ROLE) != 0;
  // asynchronous validation (a mask over the instantiations like the choices
  // above: FedProx and batch > 12 measured slower with it compiled in)
  constexpr bool AVOK = (ASYNC_VALID & ROLE) != 0;
  const bool av_launch = (A.flags & TRAIN_FLAG_ASYNC_VALID) != 0;   // grid: k trainers, then k validators
  const int nk = av_launch ? (int)gridDim.x / 2 : (int)gridDim.x;
  if (av_launch && !AVOK && (int)blockIdx.x >= nk) return;
  const bool av = AVOK && av_launch;
  const bool validator = av && (int)blockIdx.x >= nk;
  __shared__ __attribute__((aligned(16))) float lds[L_TOTAL];
  const int w8 = threadIdx.x >> 6;
  const bool helper = w8 >= 4;
  const int w = w8 & 3;           // main wave index / the main wave a helper serves
  const int lane = threadIdx.x & 63;
  const int c = lane & 15;
  const int g = lane >> 4;
  const bool stager = threadIdx.x < 256;
  float* const sW1 = lds;
  float* const sW4 = sW1 + L_W1;
  float* const sW2 = sW4 + L_W4;
  float* const sW3 = sW2 + L_W2;
  float* const sRedH1 = sW3 + L_W3;               // two buffers (parity)
  float* const sRedDH3 = sRedH1 + 2 * L_RED;
  float* const scr = sRedDH3 + L_RED + w * L_SCR;
  float* const sT0 = scr;                // dY^T own rows   (main -> helper)
  float* const sT1 = sT0 + L_T32;        // H3^T            (main -> helper)
  float* const sH1T = sT1 + L_T32;       // H1^T
  float* const sT2 = sH1T + L_T32;       // dH3^T
  float* const sZT = sT2 + L_T32;        // Z^T (with bias row)
  float* const sDZT = sZT + L_T16;       // dZ^T
  float* const sQ4 = sRedDH3 + L_RED + 4 * L_SCR;   // [w][v][t][lane][4]
  double* const sLoss = reinterpret_cast<double*>(sQ4 + L_Q4);  // [8 waves][4]
  // per-step Adam scalars (helper -> main), double-buffered by step parity:
  // [kd, ed, -, -] (EXACT_ADAM: [neg_step_size, inv_bc2s, bc2s, -]); W4FLAG:
  // one pair per helper
  float* const sK = reinterpret_cast<float*>(sLoss + 32);
  // W4FLAG: [0..3] layer-1 partials of step count v written by main w;
  // [4..7] W4 / Adam scalars for step count v published by helper w
  int* const sFlag = reinterpret_cast<int*>(sK + 32);
  // [12]: OR of every wave's spin_fail, read by thread 0 after the last barrier
  int* const sFail = sFlag + 12;
  bool spin_fail = false;
  auto flag_set = [&](int i, int v) {
    if (lane == 0) __hip_atomic_store(sFlag + i, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
  };
  // n = 4: one 16-byte volatile LDS read polls four flags (one round trip; four
  // acquire loads would each wait for the previous one), then one acquire fence
  auto flag_wait = [&](int i0, int n, int v) {
    for (int it = 0; !spin_fail; ++it) {
      int m;
      // (explicit LDS address space: a generic volatile pointer becomes a flat load)
      if (n == 4) {
        const i32x4 q = *(const volatile __attribute__((address_space(3))) i32x4*)(sFlag + i0);
        m = min(min(q[0], q[1]), min(q[2], q[3]));
      } else {
        m = *(const volatile __attribute__((address_space(3))) int*)(sFlag + i0);
      }
      if (m >= v) break;
      if (it >= HW_SPIN_LIMIT) {
        spin_fail = true;
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
  };

  Lane L;
  L.w1 = sW1 + c * S_W1 + 32 * w + 4 * g;
  L.w4 = sW4 + (32 * w + 4 * g) * S_W4 + c;
  if (w < 2) {
    L.own = sW3 + (16 * w + 4 * g) * S_W3 + c;
    L.own_stride = S_W3;
  } else {
    L.own = sW2 + 4 * g * S_W2 + 16 * (w - 2) + c;
    L.own_stride = S_W2;
  }
  float* const q4p = sQ4 + (w * 4 * 64 + lane) * 4;   // + (2v + t) * 256
  const float* const a4p = sW4 + (32 * w + c) * S_W4 + 4 * g;
  const float* const a2p = sW2 + c * S_W2 + 4 * g;
  const float* const a3p = sW3 + c * S_W3 + 4 * g;
  const float* const d2p = sW2 + 4 * g * S_W2 + c;
  const float* const d3p = sW3 + 4 * g * S_W3 + c;
  const int tw = 4 * g * S_T + c;
  const int tr = c * S_T + 4 * g;
  // owned small tile's operands (wave-uniform choice, made once): w < 2: dW3
  // tile = dH3^T(rows 16w..) Z; w >= 2: dW2 tile = dZ^T H1(tile w-2)
  const float* const sm_a = w < 2 ? sT2 + tr + 16 * w * S_T : sDZT + tr;
  const float* const sm_b = w < 2 ? sZT + tr : sH1T + tr + 16 * (w - 2) * S_T;
  float* const redw = sRedDH3 + (w * 2) * 256 + lane * 4;

  const int kslot = validator ? (int)blockIdx.x - nk : (int)blockIdx.x;
  const int cid = A.client_idx[kslot];
  float* const Pg = A.params + (size_t)cid * P_PAD;
  float* const Mg = A.adam_m + (size_t)cid * P_PAD;
  float* const Vg = A.adam_v + (size_t)cid * P_PAD;
  float* const Bg = A.best + (size_t)cid * P_PAD;
  const int d_in = A.d_in, hidden = A.hidden, latent = A.latent;

  const int B = A.batch;
  const float* const Xtr = A.train_x + (size_t)A.train_off[cid] * DP;
  const int n_tr = (int)(A.train_off[cid + 1] - A.train_off[cid]);
  const float* const Xva = A.valid_x + (size_t)A.valid_off[cid] * DP;
  const int n_va = (int)(A.valid_off[cid + 1] - A.valid_off[cid]);
  const int nb = (n_tr + B - 1) / B;
  // MULTI: 16-row chunks per epoch ((nb - 1) full batches + the last one)
  const int nsteps = MULTI ? (nb > 0 ? (nb - 1) * ((B + 15) / 16) + (n_tr - (nb - 1) * B + 15) / 16 : 0) : nb;
  const int nvb = (n_va + B - 1) / B;
  const int nvt = (n_va + 15) / 16;   // 16-row validation tiles
  int step = A.adam_step[cid];
  int parity = 0;
  const bool bias_lane = (w == 3 && g == 3);
  const int xcol = 32 * w + 4 * g;
  const float lam = A.lambda;
  const float inv_d = 1.0f / (float)d_in;
  bool hreal_d[2][4], hbias_d[2][4], zreal_d[4], zbias_d[4], hreal_c[2];
#pragma unroll
  for (int t = 0; t < 2; ++t) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int j = hslot_of_pos<CP>(16 * t + 4 * g + r);
      hreal_d[t][r] = j < hidden;
      hbias_d[t][r] = j == h_bias_slot<CP>();
    }
    hreal_c[t] = hslot_of_pos<CP>(16 * t + c) < hidden;
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int j = zslot_of_pos<CP>(4 * g + r);
    zreal_d[r] = j < latent;
    zbias_d[r] = j == z_bias_slot<CP>();
  }
  // VALUE_MASKS: the bias slots in the register tiles (compact
  // order): H3 / dH3 D-layout row 30 = tile 1, (g, r) = (3, 2); H1^T row 30 =
  // tile 1, column lane c = 14; Z D-layout row 13 = (g, r) = (3, 1)
  const float thr_h3b = (g == 3) ? 2.f : 0.f;
  const float thr_h1b = (c == 14) ? 2.f : 0.f;
  const bool z_bias_lane = (g == 3);
  const int brow_c = batch_row_of_col<CPB>(c);
  int brow_b[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) brow_b[r] = batch_row_of_col<CPB>(4 * g + r);

  // one batch chunk of X in both register layouts the step uses (f: layer
  // 1's B operand over this wave's 32 columns; b: dW1's, batch on k).  The
  // packed training / validation rows already hold the constant 1 in the
  // bias column DP-1 (ClientStore._concat; it feeds W1a's b1).
  // Rows past the client's end (an epoch's last chunk) are read as they are:
  // the next client's rows or the buffer's zero tail (ClientStore), finite
  // values in batch columns every product masks.  So each load is a uniform
  // row base plus a per-lane offset formed once, with no per-step clamping.
  // (padding columns, brow_c = -1, read the chunk's row 0; every row < 12)
  const unsigned offf = (unsigned)((brow_c < 0 ? 0 : brow_c) * DP + xcol);
  unsigned offb[KB];
#pragma unroll
  for (int r = 0; r < KB; ++r) offb[r] = (unsigned)(brow_b[r] * DP + 32 * w + c);   // CPB: r < 3 real rows
  auto load_chunk = [&](const float* X, int row0, int bc, XChunk& x) {
    (void)bc;
    const float* base = X + (size_t)row0 * DP;
    x.f0 = *reinterpret_cast<const f32x4*>(base + offf);
    x.f1 = *reinterpret_cast<const f32x4*>(base + offf + 16);   // cols DP-4..DP-1 on the bias lane
#pragma unroll
    for (int r = 0; r < KB; ++r) {   // CPB: row quad 3 is padding, never read
      x.b0[r] = base[offb[r]];
      x.b1[r] = base[offb[r] + 16];
    }
    if (CPB) {
      x.b0[3] = 0.f;
      x.b1[3] = 0.f;
    }
  };
  // whole forward of one 16-row validation TILE by one wave (any of the 8).
  // The reference's validation loss is the mean over its batch-B DataLoader
  // batches of each batch's mean loss (`src/Trainer/client_trainer.py:387-404`):
  // every row contributes its own loss / bt(its batch), so the rows need not
  // be grouped by batch — 16-row tiles cover the 170-row validation sets in
  // 11 forwards instead of 15 batch-of-12 chunks (the validation is
  // matrix-pipe bound: 3 instead of 4 forwards on the busiest SIMD).  Each
  // row's fp32 contribution is the batch-chunk form's; only the fp64 sums
  // are grouped differently.
  // (split into the row loads and the forward: the validator workgroup of
  // asynchronous validation loads its tiles once per launch)
  auto valid_load = [&](const float* X, int row0, int n_rows, VTile& t) {
    const int row = row0 + c;
    const bool ok = row < n_rows;
    const float* src = X + (size_t)(ok ? row : 0) * DP + 4 * g;
#pragma unroll
    for (int b = 0; b < 4; ++b)
#pragma unroll
      for (int v = 0; v < 2; ++v) {
        const f32x4 q = *reinterpret_cast<const f32x4*>(src + 32 * b + 16 * v);
#pragma unroll
        for (int r = 0; r < 4; ++r) t.xf[b][v][r] = q[r];
      }
  };
  auto valid_compute = [&](const VTile& t, int row0, int n_rows, double& lacc) {
    const int row = row0 + c;
    const bool ok = row < n_rows;
    const int bstart = ok ? (row / B) * B : 0;
    const float inv_bt = ok ? 1.0f / (float)min(B, n_rows - bstart) : 0.f;
    const auto& xf = t.xf;
    f32x4 h1[2];
    {
      f32x4 sum0 = zero4(), sum1 = zero4();
#pragma unroll
      for (int b = 0; b < 4; ++b) {
        f32x4 p0 = zero4(), p1 = zero4();
#pragma unroll
        for (int v = 0; v < 2; ++v) {
          const f32x4 a0 = lds_read4(sW1 + c * S_W1 + 32 * b + 16 * v + 4 * g);
          const f32x4 a1 = lds_read4(sW1 + (16 + c) * S_W1 + 32 * b + 16 * v + 4 * g);
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            p0 = mfma16(a0[r], xf[b][v][r], p0);
            p1 = mfma16(a1[r], xf[b][v][r], p1);
          }
        }
        if (b == 0) {
          sum0 = p0;
          sum1 = p1;
        } else {
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            sum0[r] = sum0[r] + p0[r];
            sum1[r] = sum1[r] + p1[r];
          }
        }
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float v0 = relu(sum0[r]), v1 = relu(sum1[r]);
        if (!BU && hbias_d[0][r]) v0 = 1.f;
        if (!BU && hbias_d[1][r]) v1 = 1.f;
        sum0[r] = v0;
        sum1[r] = v1;
      }
      h1[0] = sum0;
      h1[1] = sum1;
    }
    const f32x4 z = chain2<SPLIT>(lds_read4(a2p), lds_read4(a2p + 16), h1[0], h1[1]);
    f32x4 zb = z;
#pragma unroll
    for (int r = 0; r < 4; ++r)
      if (!BU && zbias_d[r]) zb[r] = 1.f;
    f32x4 h3[2];
    {
      f32x4 acc0 = zero4(), acc1 = zero4();
      const f32x4 a0 = lds_read4(a3p);
      const f32x4 a1 = lds_read4(a3p + 16 * S_W3);
#pragma unroll
      for (int s = 0; s < KZ; ++s) {
        acc0 = mfma16(a0[s], zb[s], acc0);
        acc1 = mfma16(a1[s], zb[s], acc1);
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float v0 = relu(acc0[r]), v1 = relu(acc1[r]);
        if (!BU && hbias_d[0][r]) v0 = 1.f;
        if (!BU && hbias_d[1][r]) v1 = 1.f;
        acc0[r] = v0;
        acc1[r] = v1;
      }
      h3[0] = acc0;
      h3[1] = acc1;
    }
    float nz = 0.f;
    if (VMASK) {
      // (padded latent slots are 0; the bias slot is row (g, r) = (3, 1))
      nz = z[0] * z[0] + (z_bias_lane ? 0.f : z[1] * z[1]) + z[2] * z[2] + z[3] * z[3];
    } else {
#pragma unroll
      for (int r = 0; r < 4; ++r) nz += zreal_d[r] ? z[r] * z[r] : 0.f;
    }
    nz = sum_lane_groups(nz);
    const float norm_v = __builtin_amdgcn_sqrtf(nz);
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      f32x4 acc0 = zero4(), acc1 = zero4();
      const float* ap = sW4 + (32 * b + c) * S_W4 + 4 * g;
      const f32x4 a00 = lds_read4(ap);
      const f32x4 a01 = lds_read4(ap + 16);
      const f32x4 a10 = lds_read4(ap + 16 * S_W4);
      const f32x4 a11 = lds_read4(ap + 16 * S_W4 + 16);
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        acc0 = mfma16(a00[s], h3[0][s], acc0);
        acc1 = mfma16(a10[s], h3[0][s], acc1);
      }
#pragma unroll
      for (int s = 0; s < 3; ++s) {
        acc0 = mfma16(a01[s], h3[1][s], acc0);
        acc1 = mfma16(a11[s], h3[1][s], acc1);
      }
      float sq = 0.f;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float d0 = acc0[r] - xf[b][0][r];
        const float d1 = (!BU && b == 3 && g == 3 && r == 3) ? 0.f : acc1[r] - xf[b][1][r];
        sq += d0 * d0 + d1 * d1;
      }
      sq = ok ? sq : 0.f;
      float contrib = sq * (inv_bt * inv_d);
      if (b == 0 && g == 0 && ok) contrib += lam * norm_v * inv_bt;
      lacc += (double)contrib;
    }
  };
  auto valid_chunk = [&](const float* X, int row0, int n_rows, double& lacc) {
    asm volatile("" ::: "memory");
    VTile t;
    valid_load(X, row0, n_rows, t);
    valid_compute(t, row0, n_rows, lacc);
  };

  AdamStep K;
  K.one_m_b1 = 1.f - A.beta1;
  K.b1 = A.beta1;
  K.b2 = A.beta2;
  K.one_m_b2 = 1.f - A.beta2;
  K.eps = A.eps;
  K.two_mu = 2.f * A.mu;
  double b1pow = pow((double)A.beta1, (double)step);
  double b2pow = pow((double)A.beta2, (double)step);
  // adam4s: p += mh / (sqrt(vh) * kd + ed) (fedmx_train_common.h)
  const AdamScaledInit KI = adam_scaled_init(A.lr, A.beta1, A.beta2, A.eps);
  auto next_constants = [&]() {
    b1pow *= (double)A.beta1;
    b2pow *= (double)A.beta2;
    adam_step_scalars(K, KI, A.lr, b1pow, b2pow);
  };
  // moment scales of adam4s (load: m / (1-b1), v / (1-b2); write-back: inverse)
  const float m_in = adam_moment_in_scale(A.beta1), v_in = adam_moment_in_scale(A.beta2);
  auto scale4 = [](float (&q)[4], float s) {
#pragma unroll
    for (int r = 0; r < 4; ++r) q[r] *= s;
  };

  double min_valid = __builtin_huge_val();
  int worse = 0, ep_run = 0, best_ep = -1;

  // Epoch tail, identical barrier sequence for both roles: validation (wave
  // w8 takes batches w8, w8+8, ...), fixed-order loss exchange, tracking,
  // patience decision, best-validation snapshot.  True: stop training.
  auto epoch_tail = [&](int ep, double acc_tr, double prox_now) -> bool {
    HSTAMP(ep == 0, 12);
    __syncthreads();   // masters published (W1 by mains, W4 by helpers, small tiles)
    double acc_va = 0.0;
    HSTAMP(ep == 0, 14);
    for (int vt = w8; vt < nvt; vt += 8) {
      HSTAMP(ep == 0 && vt == w8, 16);
      valid_chunk(Xva, 16 * vt, n_va, acc_va);
      HSTAMP(ep == 0 && vt == w8, 17);
    }
    HSTAMP(ep == 0, 15);
    {
      const double s0 = wave_sum_d(acc_tr);
      const double s1 = wave_sum_d(acc_va);
      const double s2 = wave_sum_d(prox_now);
      if (lane == 0) {
        sLoss[w8 * 4 + 0] = s0;
        sLoss[w8 * 4 + 1] = s1;
        sLoss[w8 * 4 + 2] = s2;
      }
    }
    __syncthreads();
    double tr_sum = 0.0, va_sum = 0.0, px_sum = 0.0;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      tr_sum += sLoss[i * 4 + 0];
      va_sum += sLoss[i * 4 + 1];
      px_sum += sLoss[i * 4 + 2];
    }
    const double train_loss = nb > 0 ? tr_sum / nb : __builtin_nan("");
    double valid_loss = nvb > 0 ? va_sum / nvb : __builtin_nan("");
    if (PROX) valid_loss += (double)A.mu * px_sum;
    if (threadIdx.x == 0) {
      double* trk = A.tracking + ((size_t)kslot * A.epochs + ep) * 2;
      trk[0] = train_loss;
      trk[1] = valid_loss;
    }
    ep_run = ep + 1;
    if (valid_loss < min_valid) {
      min_valid = valid_loss;
      best_ep = ep;
      worse = 0;
      if (stager) masters_to_global_o<CP, BU>(Bg, sW1, sW4, sW2, sW3);  // save_model(): best snapshot
    } else {
      ++worse;
    }
    __syncthreads();   // sLoss reuse / masters stable for the snapshot copy
    HSTAMP(ep == 0, 13);
    return worse >= A.patience && worse > 0;
  };

  // ---- asynchronous validation (ASYNC_VALID, see the top of the file)
  // (the workspace addresses are formed where they are used, from the kernel
  // arguments: nothing of this stays live through the step loop, whose
  // FedProx and batch > 12 instantiations sit at the register limit)
  auto av_ws = [&]() -> float* { return A.vws + (size_t)kslot * AV_SLOT; };
  auto av_ready = [&]() { return reinterpret_cast<unsigned long long*>(av_ws() + AV_L_M); };
  auto av_px = [&]() { return reinterpret_cast<unsigned long long*>(av_ws() + AV_L_M + 2); };
  auto av_dec = [&]() { return reinterpret_cast<unsigned long long*>(av_ws() + AV_L_M + 32); };
  auto av_rec = [&]() { return av_ws() + AV_L_M + AV_FLAGS + 40 * threadIdx.x; };
  auto av_seq = [&]() { return (unsigned long long)A.vseq << 32; };
  // (TRAIN_FLAG_TEST_MUTE_VALIDATOR, tests only: 0.2 s instead of 10 s)
  auto av_timeout = [&]() -> long long {
    return (A.flags & TRAIN_FLAG_TEST_MUTE_VALIDATOR) ? AV_TIMEOUT / 50 : AV_TIMEOUT;
  };
  bool av_break = false;   // the validator stopped the client: roll back to the last published epoch
  // (thread 0) the decision word's low half once it covers epoch need - 1, or AV_FAIL
  auto av_wait_dec = [&](int need) -> unsigned {
    if (spin_fail) return AV_FAIL;   // (one wait that ran out ends the launch's waiting)
    const unsigned lo = av_wait_decision(av_dec(), av_seq(), need, av_timeout());
    if (lo == AV_FAIL) spin_fail = true;
    return lo;
  };
  auto av_stop = [](unsigned lo) { return lo != AV_FAIL && (lo & 1u) != 0; };
  // trainer, both roles, one workgroup barrier: epoch ep-1's decision
  // (thread 0 waits for it); true = stop
  auto av_check = [&](int ep) -> bool {
    HSTAMP(ep == 1, 20);
    AVSTAMP(ep == 2, 23);   // trainer: epoch 1's decision needed
    if (threadIdx.x == 0) sFlag[16] = (int)av_wait_dec(ep);
    AVSTAMP(ep == 2, 24);   // trainer: ... received
    __syncthreads();
    HSTAMP(ep == 1, 21);
    return av_stop((unsigned)sFlag[16]);
  };
  // trainer, end of epoch ep, both roles: the masters of epoch ep complete in
  // LDS; an epoch shorter than AV_CHECK steps reads epoch ep-1's decision
  // here.  True: it said stop -- roll back instead of publishing.
  auto av_epoch_begin = [&](int ep) -> bool {
    HSTAMP(ep == 0, 18);
    __syncthreads();
    return ep > 0 && nsteps <= AV_CHECK && av_check(ep);
  };
  // ... then publish epoch ep: LDS masters -> workspace, train loss, FedProx
  // term, ready flag (the role then writes its own moments to av_rec, which
  // only the same thread reads back, after a roll-back)
  auto av_epoch_publish = [&](int ep, double acc_tr, double prox_now) {
    const __amdgpu_buffer_rsrc_t rs = av_rsrc(av_ws());
    for (int i = threadIdx.x; i < AV_L_M / 4; i += 512) av_store16(rs, i, lds_read4(lds + 4 * i));
    const double s0 = wave_sum_d(acc_tr);
    const double s2 = wave_sum_d(prox_now);
    if (lane == 0) {
      sLoss[w8 * 4 + 0] = s0;
      sLoss[w8 * 4 + 2] = s2;
    }
    av_drain();   // every storing wave, before the barrier behind which lane 0 signals
    __syncthreads();
    if (threadIdx.x == 0) {
      double tr_sum = 0.0, px_sum = 0.0;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        tr_sum += sLoss[i * 4 + 0];
        px_sum += sLoss[i * 4 + 2];
      }
      A.tracking[((size_t)kslot * A.epochs + ep) * 2] = nb > 0 ? tr_sum / nb : __builtin_nan("");
      // (the FedProx term, 0 without FedProx, and a drain before the flag in
      // every instantiation: without them the plain launch measured 12 us
      // slower, r5z -- the flag then queues behind the waves' moment records)
      av_st(av_px(), __builtin_bit_cast(unsigned long long, px_sum));
      av_drain();
      av_st(av_ready(), av_seq() | (unsigned)(ep + 1));
      AVSTAMP(ep == 1, 22);   // trainer: epoch 1 published
    }
    HSTAMP(ep == 0, 19);
    ep_run = ep + 1;
  };
  // trainer, both roles: the masters of the last published epoch back into
  // LDS (the role restores its moments from av_rec after this; this thread's
  // own stores of them are ordered before its loads).  The leading barrier
  // orders the main waves' w1_to_lds of the discarded epoch (which a stop
  // decided inside the step loop reaches without av_epoch_begin's barrier)
  // before every wave's roll-back writes to the same LDS.
  auto av_rollback_lds = [&]() {
    __syncthreads();
    const __amdgpu_buffer_rsrc_t rs = av_rsrc(av_ws());
    for (int i = threadIdx.x; i < AV_L_M / 4; i += 512) lds_write4(lds + 4 * i, av_load16(rs, i));
    __syncthreads();
  };

  // ============================= validator =====================================
  // (the synchronous epoch_tail's validation, loss order, patience rule and
  // best snapshot, on the trainer's published copy of each epoch)
  if (validator) {
    // (TRAIN_FLAG_TEST_MUTE_VALIDATOR, tests only: client slot 0's validator
    // never answers, so its trainer's decision wait runs out and the launch
    // must report itself failed)
    if ((A.flags & TRAIN_FLAG_TEST_MUTE_VALIDATOR) && kslot == 0) return;
    double min_v = __builtin_huge_val();
    int worse_v = 0, best_v = -1;
    // the validation rows do not change: each wave loads its (first two)
    // tiles once, while it waits for the first epoch
    VTile vx0, vx1;
    if (w8 < nvt) valid_load(Xva, 16 * w8, n_va, vx0);
    if (w8 + 8 < nvt) valid_load(Xva, 16 * (w8 + 8), n_va, vx1);
    for (int ep = 0; ep < A.epochs; ++ep) {
      if (threadIdx.x == 0) {
        const unsigned long long want = av_seq() | (unsigned)(ep + 1);
        const long long t0 = (long long)wall_clock64();
        int ok = 1;
        while (av_ld(av_ready()) != want) {
          if ((long long)wall_clock64() - t0 > av_timeout()) {
            ok = 0;
            break;
          }
          __builtin_amdgcn_s_sleep(2);
        }
        sFlag[16] = ok;
        AVSTAMP(ep == 1, 25);   // validator: epoch 1 seen
        // (the polling lane loads after its poll matched; sc1, like every load of the hand-off)
        sLoss[3] = ok ? __builtin_bit_cast(double, av_ld(av_px())) : 0.0;
      }
      __syncthreads();
      if (!sFlag[16]) {   // the trainer never published: its launch reports itself failed
        if (threadIdx.x == 0)
          av_st(av_dec(), av_seq() | AV_FAIL);
        return;
      }
      {
        const __amdgpu_buffer_rsrc_t rs = av_rsrc(av_ws());
        for (int i = threadIdx.x; i < AV_L_M / 4; i += 512) lds_write4(lds + 4 * i, av_load16(rs, i));
      }
      __syncthreads();
      double acc_va = 0.0;   // (the tiles in epoch_tail's order: w8, w8 + 8, ...)
      if (w8 < nvt) valid_compute(vx0, 16 * w8, n_va, acc_va);
      if (w8 + 8 < nvt) valid_compute(vx1, 16 * (w8 + 8), n_va, acc_va);
      for (int vt = w8 + 16; vt < nvt; vt += 8) valid_chunk(Xva, 16 * vt, n_va, acc_va);
      const double s1 = wave_sum_d(acc_va);
      if (lane == 0) sLoss[w8 * 4 + 1] = s1;
      __syncthreads();
      AVSTAMP(ep == 1, 26);   // validator: validation pass done
      double va_sum = 0.0;
#pragma unroll
      for (int i = 0; i < 8; ++i) va_sum += sLoss[i * 4 + 1];
      double valid_loss = nvb > 0 ? va_sum / nvb : __builtin_nan("");
      if (PROX) valid_loss += (double)A.mu * sLoss[3];
      if (threadIdx.x == 0) A.tracking[((size_t)kslot * A.epochs + ep) * 2 + 1] = valid_loss;
      const bool better = valid_loss < min_v;
      if (better) {
        min_v = valid_loss;
        best_v = ep;
        worse_v = 0;
      } else {
        ++worse_v;
      }
      const bool stop = worse_v >= A.patience && worse_v > 0;
      // the decision first (the trainer waits for nothing else), then the best
      // snapshot from this workgroup's LDS copy, which the trainer never touches
      if (threadIdx.x == 0)
        av_st(av_dec(), av_seq() | ((unsigned)(best_v + 1) << 16) | ((unsigned)(ep + 1) << 1) | (stop ? 1u : 0u));
      AVSTAMP(ep == 1, 27);   // validator: decision stored
      if (better && stager) masters_to_global_o<CP, BU>(Bg, sW1, sW4, sW2, sW3);  // save_model(): best snapshot
      if (stop) return;
      __syncthreads();   // masters and sLoss read before the next epoch's copy
    }
    return;
  }
  // prologue staging: the stagers issue the loads of every state tensor
  // (m, v, [anchor], params) in one memory round trip, then each tensor
  // passes through the masters in turn (the barrier sequence of one global_to_masters_o pass per tensor)
  HSTAMP(true, 28);
  if (threadIdx.x < 13) sFlag[threadIdx.x] = 0;   // flags + failure word (the staging barriers follow)
  f32x4 pv_m[STAGE_PER_THREAD], pv_v[STAGE_PER_THREAD], pv_a[STAGE_PER_THREAD], pv_p[STAGE_PER_THREAD];
  if (stager) {
    stage_load(Mg, pv_m);
    stage_load(Vg, pv_v);
    if (PROX) stage_load(A.anchor + (size_t)cid * P_PAD, pv_a);
    stage_load(Pg, pv_p);
    if (BU) {
      bias_units_set(pv_p, 1.f);
      if (PROX) bias_units_set(pv_a, 1.f);   // (p - anchor = 0 there: no proximal pull)
    }
  }
  auto stage_vals = [&](const f32x4 (&v)[STAGE_PER_THREAD]) {
    if (stager) vals_to_masters_o<CP>(v, sW1, sW4, sW2, sW3);
    __syncthreads();
  };

  if (helper) {
    // =========================== helper waves ===================================
    HSlab P4, M4, V4, AN4;
    stage_vals(pv_m);
    lds_to_hslab(M4, L);
    __syncthreads();
    stage_vals(pv_v);
    lds_to_hslab(V4, L);
    __syncthreads();
    if (ADAM_SCALED) {
#pragma unroll
      for (int v = 0; v < 2; ++v)
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          scale4(M4.q4[v][t], m_in);
          scale4(V4.q4[v][t], v_in);
        }
    }
    if (PROX) {
      stage_vals(pv_a);
      lds_to_hslab(AN4, L);
      __syncthreads();
    }
    stage_vals(pv_p);
    lds_to_hslab(P4, L);
    auto publish_q4 = [&]() {
#pragma unroll
      for (int v = 0; v < 2; ++v)
#pragma unroll
        for (int t = 0; t < 2; ++t)
          lds_write4(q4p + (2 * v + t) * 256, f32x4{P4.q4[v][t][0], P4.q4[v][t][1], P4.q4[v][t][2], P4.q4[v][t][3]});
    };
    publish_q4();
    // The step's Adam scalars (f64 bias corrections: ~6 % of the main waves'
    // step when they computed them, r3 ablation) are formed here one
    // step ahead and handed over through LDS.
    int js = 0;   // step index within the launch
    auto publish_k = [&]() {
      next_constants();
      const f32x4 kq = ADAM_SCALED ? f32x4{K.kd, K.ed, 0.f, 0.f} : f32x4{K.neg_step_size, K.inv_bc2s, K.bc2s, 0.f};
      if (W4FLAG) {
        if (lane == 0) lds_write4(sK + 8 * w + 4 * (js & 1), kq);
      } else if (lane == 0 && w8 == 4) {
        lds_write4(sK + 4 * (js & 1), kq);
      }
    };
    publish_k();   // step 0's
    if (W4FLAG) flag_set(4 + w, 1);   // W4 / scalars of launch step 0 published
    for (int ep = 0; ep < A.epochs; ++ep) {
      double acc_tr = 0.0;
      // W4 gradient + Adam between barrier #2 of step s and barrier #1 of s+1
      int mb = 0, mch = 0;   // MULTI: batch / chunk of this step
      f32x4 G4[2][2];
      for (int bi = 0; bi < nsteps; ++bi) {
        // (asynchronous validation: the mains' check before step AV_CHECK)
        if (AVOK && av && ep > 0 && bi == AV_CHECK && av_check(ep)) {
          av_break = true;
          break;
        }
        const bool hs = (ep == 0 && bi == STAMP_STEP);
        const int nch = MULTI ? (min(B, n_tr - mb * B) + 15) / 16 : 1;
        const bool first_ch = !MULTI || mch == 0;
        const bool last_ch = !MULTI || mch + 1 == nch;
        if (MULTI) {
          if (last_ch) {
            ++mb;
            mch = 0;
          } else {
            ++mch;
          }
        }
        HSTAMP(hs, 0);
        if (!W4FLAG) __syncthreads();   // barrier #1 (main: layer-1 partials)
        HSTAMP(hs, 2);
        __syncthreads();   // barrier #2 (main: dY^T / H3^T of this step written)
        HSTAMP(hs, 7);
        const f32x4 w4a0 = lds_read4(sT0 + tr);
        const f32x4 w4a1 = lds_read4(sT0 + tr + 16 * S_T);
        const f32x4 w4b0 = lds_read4(sT1 + tr);
        const f32x4 w4b1 = lds_read4(sT1 + tr + 16 * S_T);
        if (first_ch) {
#pragma unroll
          for (int v = 0; v < 2; ++v)
#pragma unroll
            for (int t = 0; t < 2; ++t) G4[v][t] = zero4();
        }
#pragma unroll
        for (int s = 0; s < KB; ++s) {
          G4[0][0] = mfma16(w4a0[s], w4b0[s], G4[0][0]);
          G4[0][1] = mfma16(w4a0[s], w4b1[s], G4[0][1]);
          G4[1][0] = mfma16(w4a1[s], w4b0[s], G4[1][0]);
          G4[1][1] = mfma16(w4a1[s], w4b1[s], G4[1][1]);
        }
        if (!last_ch) continue;   // MULTI: W4's Adam after the batch's last chunk
        HSTAMP(hs, 8);

        float prox_acc = 0.f;
#pragma unroll
        for (int v = 0; v < 2; ++v)
#pragma unroll
          for (int t = 0; t < 2; ++t)
            adam_update<PROX>(P4.q4[v][t], M4.q4[v][t], V4.q4[v][t], AN4.q4[v][t], G4[v][t], K, prox_acc);
        if (PROX) acc_tr += (double)A.mu * (double)prox_acc;
        HSTAMP(hs, 10);
        // publish W4(s+1): master rows (layer 4, validation, snapshots) and the
        // dH3 A-operand copy; main w reads both after barrier #1 of step s+1
        w4_to_lds(P4, L);
        publish_q4();
        ++js;
        publish_k();   // step js's scalars, read by the mains after its barrier #1
        // (TRAIN_FLAG_TEST_DROP_W4, tests only: helper 0 never publishes launch
        // step 3's W4, so main wave 0's bounded wait for it runs out and the
        // launch must report itself failed)
        if (W4FLAG && !((A.flags & TRAIN_FLAG_TEST_DROP_W4) && w == 0 && js == 3))
          flag_set(4 + w, js + 1);   // W4(js) ready for main w's layer 4
        HSTAMP(hs, 11);
      }
      double prox_now = 0.0;
      if (PROX) {
        float pr = 0.f;
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
          for (int r = 0; r < 4; ++r)
#pragma unroll
            for (int v = 0; v < 2; ++v) {
              const float d4 = P4.q4[v][t][r] - AN4.q4[v][t][r];
              pr += d4 * d4;
            }
        prox_now = (double)pr;
      }
      if (av) {
        if (av_break || av_epoch_begin(ep)) {   // stopped after epoch ep-1: discard epoch ep
          av_break = true;
          av_rollback_lds();
          hslab_restore(av_rec(), M4, V4);
          break;
        }
        av_epoch_publish(ep, acc_tr, prox_now);
        if (ep + 1 < A.epochs) hslab_dump(av_rec(), M4, V4);   // (own roll-back record: after the publication, undrained)
      } else if (epoch_tail(ep, acc_tr, prox_now)) {
        break;
      }
    }
    // write back (barriers as the main branch; the mains stage to global)
    if (ADAM_SCALED) {
#pragma unroll
      for (int v = 0; v < 2; ++v)
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          scale4(M4.q4[v][t], K.one_m_b1);
          scale4(V4.q4[v][t], K.one_m_b2);
        }
    }
    __syncthreads();
    __syncthreads();
    w4_to_lds(M4, L);
    __syncthreads();
    __syncthreads();
    w4_to_lds(V4, L);
    if (spin_fail && lane == 0) __hip_atomic_fetch_or(sFail, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    __syncthreads();
    HSTAMP(true, 31);
    return;
  }

  // ============================= main waves =====================================
  int js = 0;   // step index within the launch (selects the Adam-scalar slot)
  int step_e = step;   // asynchronous validation: the Adam step count of the last published epoch
  MSlab P, M, V, AN;
  stage_vals(pv_m);
  lds_to_mslab(M, L);
  __syncthreads();
  stage_vals(pv_v);
  lds_to_mslab(V, L);
  __syncthreads();
  auto scale_mslab = [&](MSlab& o, float sc) {
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int v = 0; v < 2; ++v) scale4(o.q1[t][v], sc);
    scale4(o.o, sc);
  };
  if (ADAM_SCALED) {
    scale_mslab(M, m_in);
    scale_mslab(V, v_in);
  }
  if (PROX) {
    stage_vals(pv_a);
    lds_to_mslab(AN, L);
    __syncthreads();
  }
  stage_vals(pv_p);
  lds_to_mslab(P, L);   // W2/W3/W4 masters stay live; W1 lives in registers only
  HSTAMP(true, 29);

  auto l1_partial = [&](const XChunk& x, f32x4& acc0, f32x4& acc1) {
    acc0 = zero4();
    acc1 = zero4();
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      acc0 = mfma16(P.q1[0][0][j], x.f0[j], acc0);
      acc1 = mfma16(P.q1[1][0][j], x.f0[j], acc1);
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      acc0 = mfma16(P.q1[0][1][j], x.f1[j], acc0);
      acc1 = mfma16(P.q1[1][1][j], x.f1[j], acc1);
    }
  };

  // the step's 1/bt and dY scale 2/(bt d_in): bt is B except on an epoch's
  // last batch, so both are formed once here (IEEE divisions, the same values
  // as per step) instead of two division sequences in every step
  const int bt_last = nb > 0 ? n_tr - (nb - 1) * B : B;
  float inv_b_full = 1.0f / (float)B, inv_b_last = 1.0f / (float)bt_last;
  float scale_full = 2.0f / (float)(B * d_in), scale_last = 2.0f / (float)(bt_last * d_in);
  // opaque to the optimiser: it would otherwise fold the per-step select of
  // two quotients back into one division of the selected divisor
  asm volatile("" : "+v"(inv_b_full), "+v"(inv_b_last), "+v"(scale_full), "+v"(scale_last));
  for (int ep = 0; ep < A.epochs; ++ep) {
    double acc_tr = 0.0;
    XChunk cur, nxt;
    f32x4 l1a = zero4(), l1b = zero4();
    if (nb > 0) {
      load_chunk(Xtr, 0, min(B, n_tr), cur);
      l1_partial(cur, l1a, l1b);
    }
    int mb = 0, mch = 0;   // MULTI: batch / chunk of this step
    f32x4 G1[2][2], Go;
    // one training step on chunk `cur`, prefetching into `nxt`; the loop runs
    // it twice per iteration with the two chunk buffers' roles swapped (no
    // 16-register copy of the prefetched chunk per step: PINGPONG)
    auto train_step = [&](const int bi, XChunk& cur, XChunk& nxt) {
      // MULTI: this step is chunk mch of batch mb (16 rows from row_b); the
      // batch's row count bt sets the scales, the chunk's bc the masks
      const int row_b = MULTI ? mb * B + 16 * mch : bi * B;
      const int bt = MULTI ? min(B, n_tr - mb * B) : min(B, n_tr - row_b);
      const int nch = MULTI ? (bt + 15) / 16 : 1;
      const bool first_ch = !MULTI || mch == 0;
      const bool last_ch = !MULTI || mch + 1 == nch;
      const int bc = MULTI ? min(16, bt - 16 * mch) : bt;
      const bool has_next_b = MULTI ? mb + 1 < nb : bi + 1 < nb;
      const bool has_next = MULTI ? (!last_ch || has_next_b) : has_next_b;
      const int row_n = MULTI ? (last_ch ? (mb + 1) * B : row_b + 16) : (bi + 1) * B;
      const int bc_n = has_next ? min(B, n_tr - row_n) : 0;
      const float inv_bt = has_next_b ? inv_b_full : inv_b_last;
      if (MULTI) {
        if (last_ch) {
          ++mb;
          mch = 0;
        } else {
          ++mch;
        }
      }
      const bool ms = (ep == 0 && bi == STAMP_STEP);
      HSTAMP(ms, 0);
      if (first_ch) {
        Go = zero4();
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
          for (int v = 0; v < 2; ++v) G1[t][v] = zero4();
      }

      // ---- forward: layer-1 K reduction (barrier #1), layers 2-4, loss
      f32x4 h1[2], z, zb, h3[2], y[2], q4[2][2];
      float norm_c;
      {
        float* red = sRedH1 + parity * L_RED;
        lds_write4(red + (w * 2 + 0) * 256 + lane * 4, l1a);
        lds_write4(red + (w * 2 + 1) * 256 + lane * 4, l1b);
        HSTAMP(ms, 1);
        if (W4FLAG) {
          flag_set(w, js + 1);        // (release: the partial writes above complete first)
          flag_wait(0, 4, js + 1);    // every main wave's partial of this step
        } else {
          __syncthreads();  // barrier #1
        }
        HSTAMP(ms, 2);
        auto read_helper_state = [&]() {
          // this step's Adam scalars (helper-published)
          const f32x4 kk = lds_read4(W4FLAG ? sK + 8 * w + 4 * (js & 1) : sK + 4 * (js & 1));
          if (ADAM_SCALED) {
            K.kd = kk[0];
            K.ed = kk[1];
          } else {
            K.neg_step_size = kk[0];
            K.inv_bc2s = kk[1];
            K.bc2s = kk[2];
          }
          // W4(s) rows in the dH3 A-operand layout (helper-published)
#pragma unroll
          for (int v = 0; v < 2; ++v)
#pragma unroll
            for (int t = 0; t < 2; ++t) q4[v][t] = lds_read4(q4p + (2 * v + t) * 256);
        };
        if (!W4FLAG) read_helper_state();
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          f32x4 s = lds_read4(red + t * 256 + lane * 4);
#pragma unroll
          for (int ww = 1; ww < 4; ++ww) {
            const f32x4 o = lds_read4(red + (ww * 2 + t) * 256 + lane * 4);
#pragma unroll
            for (int r = 0; r < 4; ++r) s[r] = s[r] + o[r];
          }
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            float vv = relu(s[r]);
            if (!BU && hbias_d[t][r]) vv = 1.f;
            s[r] = vv;
          }
          h1[t] = s;
        }
        parity ^= 1;
        z = chain2<SPLIT>(lds_read4(a2p), lds_read4(a2p + 16), h1[0], h1[1]);
        zb = z;
#pragma unroll
        for (int r = 0; r < 4; ++r)
          if (!BU && zbias_d[r]) zb[r] = 1.f;
        {
          f32x4 acc0 = zero4(), acc1 = zero4();
          const f32x4 a0 = lds_read4(a3p);
          const f32x4 a1 = lds_read4(a3p + 16 * S_W3);
#pragma unroll
          for (int s = 0; s < KZ; ++s) {
            acc0 = mfma16(a0[s], zb[s], acc0);
            acc1 = mfma16(a1[s], zb[s], acc1);
          }
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            float v0 = relu(acc0[r]), v1 = relu(acc1[r]);
            if (!BU && hbias_d[0][r]) v0 = 1.f;
            if (!BU && hbias_d[1][r]) v1 = 1.f;
            acc0[r] = v0;
            acc1[r] = v1;
          }
          h3[0] = acc0;
          h3[1] = acc1;
        }
        if (W4FLAG) {
          flag_wait(4 + w, 1, js + 1);   // helper w has published W4(s) and the scalars
          read_helper_state();
        }
        if (last_ch) ++js;
        {
          f32x4 acc0 = zero4(), acc1 = zero4();
          const f32x4 a00 = lds_read4(a4p);
          const f32x4 a01 = lds_read4(a4p + 16);
          const f32x4 a10 = lds_read4(a4p + 16 * S_W4);
          const f32x4 a11 = lds_read4(a4p + 16 * S_W4 + 16);
#pragma unroll
          for (int s = 0; s < 4; ++s) {
            acc0 = mfma16(a00[s], h3[0][s], acc0);
            acc1 = mfma16(a10[s], h3[0][s], acc1);
          }
#pragma unroll
          for (int s = 0; s < 3; ++s) {
            acc0 = mfma16(a01[s], h3[1][s], acc0);
            acc1 = mfma16(a11[s], h3[1][s], acc1);
          }
          y[0] = acc0;
          y[1] = acc1;
        }
        float sq = 0.f;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float d0 = y[0][r] - cur.f0[r];
          const float d1 = (!BU && bias_lane && r == 3) ? 0.f : y[1][r] - cur.f1[r];
          sq += d0 * d0 + d1 * d1;
        }
        const bool col_ok = (unsigned)brow_c < (unsigned)bc;
        sq = col_ok ? sq : 0.f;
        float nz = 0.f;
        if (VMASK) {
          nz = z[0] * z[0] + (z_bias_lane ? 0.f : z[1] * z[1]) + z[2] * z[2] + z[3] * z[3];
        } else {
#pragma unroll
          for (int r = 0; r < 4; ++r) nz += zreal_d[r] ? z[r] * z[r] : 0.f;
        }
        nz = sum_lane_groups(nz);
        norm_c = __builtin_amdgcn_sqrtf(nz);
        float contrib = sq * (inv_bt * inv_d);
        if (w == 0 && g == 0 && col_ok) contrib += lam * norm_c * inv_bt;
        acc_tr += (double)contrib;
        HSTAMP(ms, 3);
      }
      if (has_next) load_chunk(Xtr, row_n, bc_n, nxt);  // prefetch

      float q2[2][4], q3[2][4];
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          q2[t][r] = d2p[r * S_W2 + 16 * t];
          q3[t][r] = d3p[(16 * t + r) * S_W3];
        }

      // ---- dY (masked, feature-major); dY^T / H3^T for the helper's dW4
      const bool col_ok = (unsigned)brow_c < (unsigned)bc;
      const float scale = col_ok ? (has_next_b ? scale_full : scale_last) : 0.f;
      f32x4 dy[2];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        dy[0][r] = (y[0][r] - cur.f0[r]) * scale;
        dy[1][r] = (!BU && bias_lane && r == 3) ? 0.f : (y[1][r] - cur.f1[r]) * scale;
        sT0[tw + r * S_T] = dy[0][r];
        sT0[tw + (16 + r) * S_T] = dy[1][r];
        sT1[tw + r * S_T] = h3[0][r];
        sT1[tw + (16 + r) * S_T] = h3[1][r];
      }
      // ---- dH3 partial = W4a(own rows)^T dY(own rows)   (W4(s))
      {
        f32x4 acc0 = zero4(), acc1 = zero4();
#pragma unroll
        for (int v = 0; v < 2; ++v)
#pragma unroll
          for (int s = 0; s < 4; ++s) {
            acc0 = mfma16(q4[v][0][s], dy[v][s], acc0);
            acc1 = mfma16(q4[v][1][s], dy[v][s], acc1);
          }
        lds_write4(redw, acc0);
        lds_write4(redw + 256, acc1);
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        sH1T[tw + r * S_T] = h1[0][r];
        sH1T[tw + (16 + r) * S_T] = h1[1][r];
        sZT[tw + r * S_T] = zb[r];
      }
      HSTAMP(ms, 4);
      __syncthreads();  // barrier #2: dH3 partials of all waves visible
      HSTAMP(ms, 7);
      f32x4 dh3[2];
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        f32x4 s = lds_read4(sRedDH3 + t * 256 + lane * 4);
#pragma unroll
        for (int ww = 1; ww < 4; ++ww) {
          const f32x4 o = lds_read4(sRedDH3 + (ww * 2 + t) * 256 + lane * 4);
#pragma unroll
          for (int r = 0; r < 4; ++r) s[r] = s[r] + o[r];
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          if (VMASK)
            s[r] = (h3[t][r] > ((t == 1 && r == 2) ? thr_h3b : 0.f)) ? s[r] : 0.f;
          else
            s[r] = (hreal_d[t][r] && h3[t][r] > 0.f) ? s[r] : 0.f;
        }
        dh3[t] = s;
      }
      float prox_acc = 0.f;
      if (last_ch) ++step;
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) sT2[tw + (16 * t + r) * S_T] = dh3[t][r];
      // ---- dZ = W3a^T dH3 (+ shrink-loss gradient)
      f32x4 dz = chain2<SPLIT>(f32x4{q3[0][0], q3[0][1], q3[0][2], q3[0][3]},
                        f32x4{q3[1][0], q3[1][1], q3[1][2], q3[1][3]}, dh3[0], dh3[1]);
      const float shr_raw = lam * __builtin_amdgcn_rcpf((float)bt * norm_c);
      const float shr = (col_ok && norm_c > 0.f) ? shr_raw : 0.f;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        if (VMASK)
          dz[r] = (r == 1 && z_bias_lane) ? 0.f : dz[r] + shr * z[r];
        else
          dz[r] = zreal_d[r] ? dz[r] + shr * z[r] : 0.f;
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) sDZT[tw + r * S_T] = dz[r];
      // ---- dH1 (batch-major) with the ReLU mask from H1^T
      f32x4 dh1b[2], h1b[2];
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        h1b[t] = lds_read4(sH1T + tr + 16 * t * S_T);
        dh1b[t] = zero4();
        f32x4 acc = zero4();
#pragma unroll
        for (int s = 0; s < KZ; ++s) acc = mfma16(dz[s], q2[t][s], acc);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          if (VMASK)
            acc[r] = (h1b[t][r] > (t == 1 ? thr_h1b : 0.f)) ? acc[r] : 0.f;
          else
            acc[r] = (hreal_c[t] && h1b[t][r] > 0.f) ? acc[r] : 0.f;
        }
        dh1b[t] = acc;
      }
      HSTAMP(ms, 8);
      // ---- dW1^T (own columns) = X^T dH1
#pragma unroll
      for (int s = 0; s < KB; ++s) {
        G1[0][0] = mfma16(cur.b0[s], dh1b[0][s], G1[0][0]);
        G1[0][1] = mfma16(cur.b1[s], dh1b[0][s], G1[0][1]);
        G1[1][0] = mfma16(cur.b0[s], dh1b[1][s], G1[1][0]);
        G1[1][1] = mfma16(cur.b1[s], dh1b[1][s], G1[1][1]);
      }
      wave_sync();
      // ---- owned small tile: w<2 -> dW3 tile = dH3^T Z ; w>=2 -> dW2 tile = dZ^T H1
      {
        const f32x4 a = lds_read4(sm_a);
        const f32x4 b = lds_read4(sm_b);   // (Z^T, or H1^T's tile of this wave)
#pragma unroll
        for (int s = 0; s < KB; ++s) Go = mfma16(a[s], b[s], Go);
      }
      HSTAMP(ms, 9);
      auto adam_w1 = [&](int t, int v) {
        adam_update<PROX>(P.q1[t][v], M.q1[t][v], V.q1[t][v], AN.q1[t][v], G1[t][v], K, prox_acc);
      };
      {
        // W1 first: the next chunk's layer-1 product waits on it
        // (MULTI: the batch's last chunk only)
        if (last_ch) {
#pragma unroll
          for (int t = 0; t < 2; ++t)
#pragma unroll
            for (int v = 0; v < 2; ++v) adam_w1(t, v);
        }
        HSTAMP(ms, 10);
        // (after an epoch's last batch this works on a stale tile; unused)
        l1_partial(nxt, l1a, l1b);
      }
      if (last_ch) {
        adam_update<PROX>(P.o, M.o, V.o, AN.o, Go, K, prox_acc);
        if (PROX) acc_tr += (double)A.mu * (double)prox_acc;
        own_to_lds(P, L);   // read by every wave after barrier #1
      }
      HSTAMP(ms, 11);
      __builtin_amdgcn_iglp_opt(0);
    };
    // (asynchronous validation: the decision on epoch ep-1 before step
    // AV_CHECK, an even step, so the chunk buffers keep their roles)
    if constexpr (PPONG) {
      int bi = 0;
      for (; bi + 1 < nsteps; bi += 2) {
        if (AVOK && av && ep > 0 && bi == AV_CHECK && av_check(ep)) {
          av_break = true;
          break;
        }
        train_step(bi, cur, nxt);
        train_step(bi + 1, nxt, cur);
      }
      if (bi < nsteps && !av_break) {
        if (AVOK && av && ep > 0 && bi == AV_CHECK && av_check(ep))   // (an epoch of AV_CHECK + 1 steps)
          av_break = true;
        else
          train_step(bi, cur, nxt);
      }
    } else {
      for (int bi = 0; bi < nsteps; ++bi) {
        if (AVOK && av && ep > 0 && bi == AV_CHECK && av_check(ep)) {
          av_break = true;
          break;
        }
        train_step(bi, cur, nxt);
        cur = nxt;
      }
    }
    w1_to_lds(P, L);   // W1 master (validation, snapshot)
    double prox_now = 0.0;
    if (PROX) {
      float pr = 0.f;
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
          for (int v = 0; v < 2; ++v) {
            const float d1 = P.q1[t][v][r] - AN.q1[t][v][r];
            pr += d1 * d1;
          }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float d = P.o[r] - AN.o[r];
        pr += d * d;
      }
      prox_now = (double)pr;
    }
    if (av) {
      if (av_break || av_epoch_begin(ep)) {   // stopped after epoch ep-1: discard epoch ep
        av_break = true;
        av_rollback_lds();
        mslab_restore(av_rec(), M, V);
        step = step_e;
        break;
      }
      av_epoch_publish(ep, acc_tr, prox_now);
      if (ep + 1 < A.epochs) mslab_dump(av_rec(), M, V);   // (own roll-back record: after the publication, undrained)
      step_e = step;
    } else if (epoch_tail(ep, acc_tr, prox_now)) {
      break;
    }
  }

  // ---- write back: params (masters), then m and v through the same staging
  HSTAMP(true, 30);
  __syncthreads();
  masters_to_global_o<CP, BU>(Pg, sW1, sW4, sW2, sW3);
  if (ADAM_SCALED) {
    scale_mslab(M, K.one_m_b1);
    scale_mslab(V, K.one_m_b2);
  }
  __syncthreads();
  w1_to_lds(M, L);
  own_to_lds(M, L);
  __syncthreads();
  masters_to_global_o<CP>(Mg, sW1, sW4, sW2, sW3);
  __syncthreads();
  w1_to_lds(V, L);
  own_to_lds(V, L);
  if (spin_fail && lane == 0) __hip_atomic_fetch_or(sFail, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  __syncthreads();   // (the helpers' last: every wave's failure bit is in sFail)
  masters_to_global_o<CP>(Vg, sW1, sW4, sW2, sW3);
  HSTAMP(true, 31);
  if (threadIdx.x == 0) {
    // a flag wait of any wave ran out: the launch's results are invalid
    bool failed = *(volatile int*)sFail != 0;
    int best = best_ep;
    if (av && ep_run > 0) {
      // the validator's word on the last epoch kept (after a roll-back: the
      // stop decision itself); its best epoch
      const unsigned lo = av_break ? (unsigned)sFlag[16] : av_wait_dec(ep_run);
      if (lo == AV_FAIL)
        failed = true;
      else
        best = (int)(lo >> 16) - 1;
    }
    A.adam_step[cid] = step;
    A.epochs_run[kslot] = failed ? -1000 : ep_run;
    A.best_epoch[kslot] = best;
    if (failed && A.err != nullptr) *A.err = 1;
  }
}

}  // namespace hw
}  // namespace fedmx

#ifdef FEDMX_HW_PROX_TU
// fedmx_train_hw_prox.hip: this TU holds the FedProx instantiation for batch
// <= 12 only, compiled with its own scheduler flags (ops/build.py SOURCE_FLAGS)
extern "C" int fedmx_train_hw_prox_launch(const void* args, int grid, hipStream_t stream) {
  const fedmx::TrainArgs A = *reinterpret_cast<const fedmx::TrainArgs*>(args);
  hipLaunchKernelGGL((fedmx::hw::train_kernel_hw<true, false>), dim3(grid), dim3(512), 0, stream, A);
  return (int)hipGetLastError();
}
#else
extern "C" int fedmx_train_hw_prox_launch(const void* args, int grid, hipStream_t stream);

extern "C" {

static int g_last_grid = 0;   // workgroups of the last helper-wave launch (tests: 2k = validators ran)
int fedmx_train_hw_last_grid(void) { return g_last_grid; }

// Helper-wave training launch for the compact reference shapes; returns -4
// when the shapes need the general kernel (fedmx_train).
int fedmx_train_hw(const void* args, int k, hipStream_t stream) {
  if (k <= 0) return 0;
  fedmx::TrainArgs A = *reinterpret_cast<const fedmx::TrainArgs*>(args);
  if (!(A.batch >= 1 && A.d_in >= 1 && A.d_in <= fedmx::DP - 1 && A.hidden >= 1 && A.hidden <= 27 &&
        A.latent >= 1 && A.latent <= 7))
    return -4;
  const bool multi = A.batch > 12;   // 16-row chunks per batch
  // asynchronous validation: one validator workgroup per client beside the
  // trainers, only when all 2k workgroups (one per CU: 132 KB of LDS each)
  // can be resident at once -- a trainer waits for its validator's decisions
  int grid = k;
  A.flags &= ~fedmx::TRAIN_FLAG_ASYNC_VALID;
  const int role = multi ? 4 : (A.mu != 0.f ? 2 : 1);   // the kernel's ROLE
  // (the decision word packs epoch + 1 into 15 bits: ADVICE r5)
  if ((ASYNC_VALID & role) && A.vws != nullptr && A.vseq != 0 && A.epochs >= 1 && A.epochs < 32767) {
    static int cus = 0;
    if (cus == 0) {
      int dev = 0;
      if (hipGetDevice(&dev) != hipSuccess ||
          hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
        cus = -1;
    }
    if (2 * k <= cus) {
      A.flags |= fedmx::TRAIN_FLAG_ASYNC_VALID;
      grid = 2 * k;
    }
  }
  g_last_grid = grid;
  if (A.mu != 0.f) {
    if (multi)
      hipLaunchKernelGGL((fedmx::hw::train_kernel_hw<true, true>), dim3(grid), dim3(512), 0, stream, A);
    else
      return fedmx_train_hw_prox_launch(&A, grid, stream);   // (fedmx_train_hw_prox.hip)
  } else {
    if (multi)
      hipLaunchKernelGGL((fedmx::hw::train_kernel_hw<false, true>), dim3(grid), dim3(512), 0, stream, A);
    else
      hipLaunchKernelGGL((fedmx::hw::train_kernel_hw<false, false>), dim3(grid), dim3(512), 0, stream, A);
  }
  return (int)hipGetLastError();
}

// floats of one client slot of TrainArgs.vws
int fedmx_train_av_slot(void) { return fedmx::hw::AV_SLOT; }

}  // extern "C"
#endif  // FEDMX_HW_PROX_TU
