// Device-resident round protocol (fixed-compat fast path): the decisions the
// host otherwise takes between stream synchronisations, as tiny kernels that
// read their inputs from device memory, so a whole federated round is one
// stream of launches with no host round trip.
//
//  * elect_wsum_kernel   : aggregator election (src/Trainer/client_trainer.py:249-285,
//                          driver src/main.py:281-288) over the gathered vote
//                          scores and a host-drawn noise table, the FedAvg /
//                          FedMSE weights (:107-130), and the aggregate
//                          sum_j w_j * theta_{row_j} in selection order with the
//                          separately-rounded fp32 order of weighted_sum_kernel
//                          (bit-identical aggregate)
//  * decide_adopt_kernel : aggregation-cap bookkeeping (:78, :279, :300-303),
//                          verification MSE + parameter drift reductions and
//                          the ModelVerifier rule (src/Trainer/model_verifier.py:72-99)
//                          per hosted receiver + update_from_peers adoption
//                          (client_trainer.py:174-206): accepted receivers load
//                          the aggregate and re-anchor FedProx, the history is
//                          always the last received aggregate; the aggregator
//                          itself loads the aggregate without re-anchoring
//  * verify_decide_kernel: the verification forward of the aggregate on each
//                          hosted receiver's data, decide_adopt and the
//                          evaluation snapshot in ONE launch (a workgroup per
//                          receiver: its rows fit one block, so no cross-block
//                          step); bit-identical to fwd_rows + decide_adopt + copy
//  * copy_f64_kernel     : device -> mapped host report slots
// Every kernel is a no-op when the election found no aggregator.
#include "fedmx_forward_common.h"

namespace fedmx {

struct ElectArgs {
  const int32_t* sel;      // [k] global client ids, selection order
  const double* vec;       // [N][4]: vote score, -, dev MSE (seg out[0]), dev MSE (seg out[1])
  const double* noise;     // [k][k-1] U(0,1) draws, voter-major
  int32_t* agg_counts;     // [N]
  float* weights;          // [k] out
  int32_t* state;          // [4] out: aggregator (-1: none), voter
  int32_t* report;         // [2] out (mapped host memory): aggregator, voter
  int32_t k, cap, rule;    // rule 0: mean (avg / fedprox), 1: 1/MSE (mse_avg),
                           // 2: host-computed weights hw (sample-weighted FedAvg)
  int32_t mode;            // bit 0 clear: first voter decides (client_trainer.py:249-285 +
                           //   main.py:284-288); set: majority of every selected voter's ballot
                           //   (legacy GlobalAggregator.select_aggregator; ties: selection order);
                           // bit 1: thesis vote cap (candidates scored above vote_cap, or NaN,
                           //   are never voted for, Thesis p.20 Alg. 4.2);
                           // bit 2: thesis random fallback when nobody was voted for (Thesis
                           //   p.25 §4.3.4): eligible[floor(fallback_u * n_eligible)]
  const int32_t* rec;      // [k] record index (4-double units into vec) of each selection, or
                           // null: the client id (multi-rank: records read in place from the exchange buffer)
  const float* hw;         // rule 2: [k] weights (they depend on the selection only)
  double vote_cap;         // mode bit 1
  double fallback_u;       // mode bit 2: this round's uniform draw (host, every round)
  const int32_t* err;      // or null: err_n training-failure words (TrainArgs.err), err_stride
  int32_t err_n, err_stride;   // ints apart (one per rank: the exchange rows carry them); any
                               // set -> no aggregator, report[0] = ELECT_TRAIN_FAILED
};
static_assert(sizeof(ElectArgs) == 120, "ElectArgs layout is shared with Python");
constexpr int32_t ELECT_TRAIN_FAILED = -3;

__device__ __forceinline__ int train_failed(const ElectArgs& E) {
  int f = 0;
  if (E.err != nullptr)
    for (int r = 0; r < E.err_n; ++r) f |= E.err[(size_t)r * E.err_stride];
  return f;
}

struct WsumArgs {
  const float* base;       // row-major [*, P]
  const int64_t* rows;     // [k] source rows (selection order)
  const float* weights;    // [k]
  const int32_t* state;    // aggregator flag
  float* out;              // [P]
  int32_t k, P;
};
static_assert(sizeof(WsumArgs) == 48, "WsumArgs layout is shared with Python");

// Election and aggregation in one launch: every workgroup replays the
// (tiny, k <= a few hundred) election from the same inputs — identical
// results, no inter-block communication — then reduces its slice of the
// aggregate.  Workgroup 0 publishes the aggregator / voter / weights; the
// aggregation-cap count is bumped later by decide_adopt (a single writer,
// after every workgroup here has read the counts).
template <bool WIDE>
__global__ __launch_bounds__(256) void elect_wsum_kernel(const ElectArgs E, const WsumArgs W) {
  __shared__ float s_w[1024];
  __shared__ int64_t s_rows[1024];
  __shared__ int s_agg;
  const int tid = threadIdx.x;
  // the source rows live in the mapped descriptor ring (host memory): one
  // parallel load here instead of one dependent PCIe round trip per row below
  for (int j = tid; j < W.k; j += blockDim.x) s_rows[j] = W.rows[j];
  if (E.k <= 64) {
    // Small selections (every reference config): wave 0 stages the inputs
    // with one parallel load each; each candidate lane forms its noisy score
    // with the current voter's noise row (mapped host memory: one PCIe round
    // trip per voter tried, normally just the first), then the reference's
    // serial first-minimum scan runs over the lanes.  Same double arithmetic
    // as the serial loop below (bit-identical decisions).
    __shared__ double s_inv[64];
    if (tid < 64) {
      const int lane = tid;
      const int k = E.k;
      int c = -1, cnt = 0;
      double vs = 0.0, mse = 1.0;
      // (loaded with the other inputs; checked once the election is formed)
      const int failed = train_failed(E);
      if (lane < k) {
        c = E.sel[lane];
        const int ri = E.rec != nullptr ? E.rec[lane] : c;
        vs = E.vec[(size_t)ri * 4];
        mse = E.vec[(size_t)ri * 4 + 3];
        cnt = E.agg_counts[c];
      }
      int agg = -1, voter = -1;
      int my_votes = 0;   // majority: ballots naming this lane's client
      for (int vi = 0; vi < k && (agg < 0 || (E.mode & 1)); ++vi) {
        const int v = __shfl(c, vi, 64);
        // candidate lane ci != vi draws noise entry j = ci - (ci > vi)
        bool cand = lane < k && lane != vi && cnt < E.cap;
        double sc = 0.0;
        if (lane < k && lane != vi) {
          const double f = 1.0 + (E.noise[(size_t)vi * (k - 1) + lane - (lane > vi ? 1 : 0)] - 0.5) * 0.0002;
          sc = vs * f;
        }
        if (E.mode & 2) cand = cand && (sc <= E.vote_cap);
        // the serial scan of the reference loop over the candidates' lanes
        // (uniform across the wave; NaN scores behave exactly as there)
        int best = -1;
        double best_s = 0.0;
        for (int ci = 0; ci < k; ++ci) {
          const double s_ci = __shfl(sc, ci, 64);
          const int ok_ci = __shfl(cand ? 1 : 0, ci, 64);
          if (ok_ci && (best < 0 || s_ci < best_s)) {
            best = ci;
            best_s = s_ci;
          }
        }
        if (best >= 0) {
          agg = __shfl(c, best, 64);
          voter = v;
          if (lane == best) ++my_votes;
        }
      }
      if (E.mode & 1) {
        // most ballots wins, ties to the earliest in selection order
        int top = -1, top_votes = 0;
        for (int ci = 0; ci < k; ++ci) {
          const int vc = __shfl(my_votes, ci, 64);
          if (vc > top_votes) {
            top = ci;
            top_votes = vc;
          }
        }
        agg = top >= 0 ? __shfl(c, top, 64) : -1;
        voter = -1;
      }
      if (agg < 0 && (E.mode & 4)) {
        // random eligible aggregator: the idx-th eligible lane in selection order
        const unsigned long long m = __ballot(lane < k && cnt < E.cap);
        const int n_e = __popcll(m);
        if (n_e > 0) {
          int idx = (int)(E.fallback_u * (double)n_e);
          if (idx > n_e - 1) idx = n_e - 1;
          int pick = 0, seen = 0;
          for (int ci = 0; ci < k; ++ci)
            if ((m >> ci) & 1ull) {
              if (seen == idx) {
                pick = ci;
                break;
              }
              ++seen;
            }
          agg = __shfl(c, pick, 64);
          voter = -1;
        }
      }
      // a failed training launch: its clients' parameters are invalid, so
      // nothing is aggregated or adopted this round (the host raises)
      if (failed) agg = -1;
      if (lane == 0) s_agg = agg;
      if (agg >= 0) {
        if (E.rule == 1) {
          if (lane < k) s_inv[lane] = 1.0 / mse;
          __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
          __builtin_amdgcn_wave_barrier();
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
          double tot = 0.0;
          for (int j = 0; j < k; ++j) tot += s_inv[j];   // selection order, as the serial form
          if (lane < k) s_w[lane] = (float)(s_inv[lane] / tot);
        } else if (E.rule == 2) {
          if (lane < k) s_w[lane] = E.hw[lane];
        } else if (lane < k) {
          s_w[lane] = (float)(1.0 / (double)k);
        }
      }
      if (blockIdx.x == 0 && lane == 0) {
        E.state[0] = agg;
        E.state[1] = voter;
        E.report[0] = failed ? ELECT_TRAIN_FAILED : agg;
        E.report[1] = voter;
      }
      if (blockIdx.x == 0 && agg >= 0 && lane < k) E.weights[lane] = s_w[lane];
    }
  } else if (tid == 0) {
    int agg = -1, voter = -1;
    int* s_votes = reinterpret_cast<int*>(s_w);   // majority tally (s_w is written after it)
    if (E.mode & 1)
      for (int j = 0; j < E.k; ++j) s_votes[j] = 0;
    for (int vi = 0; vi < E.k && (agg < 0 || (E.mode & 1)); ++vi) {
      const int v = E.sel[vi];
      const double* u = E.noise + (size_t)vi * (E.k - 1);
      int best = -1, best_ci = -1, j = 0;
      double best_s = 0.0;
      for (int ci = 0; ci < E.k; ++ci) {
        const int c = E.sel[ci];
        if (c == v) continue;
        const double f = 1.0 + (u[j++] - 0.5) * 0.0002;
        const double sc = E.vec[(size_t)(E.rec != nullptr ? E.rec[ci] : c) * 4] * f;
        if (E.agg_counts[c] < E.cap && (!(E.mode & 2) || sc <= E.vote_cap) && (best < 0 || sc < best_s)) {
          best = c;
          best_ci = ci;
          best_s = sc;
        }
      }
      if (best >= 0) {
        agg = best;
        voter = v;
        if (E.mode & 1) ++s_votes[best_ci];
      }
    }
    if (E.mode & 1) {
      int top = -1, top_votes = 0;
      for (int ci = 0; ci < E.k; ++ci)
        if (s_votes[ci] > top_votes) {
          top = ci;
          top_votes = s_votes[ci];
        }
      agg = top >= 0 ? E.sel[top] : -1;
      voter = -1;
    }
    if (agg < 0 && (E.mode & 4)) {
      int n_e = 0;
      for (int j = 0; j < E.k; ++j) n_e += E.agg_counts[E.sel[j]] < E.cap ? 1 : 0;
      if (n_e > 0) {
        int idx = (int)(E.fallback_u * (double)n_e);
        if (idx > n_e - 1) idx = n_e - 1;
        for (int j = 0, seen = 0; j < E.k; ++j)
          if (E.agg_counts[E.sel[j]] < E.cap) {
            if (seen == idx) {
              agg = E.sel[j];
              break;
            }
            ++seen;
          }
        voter = -1;
      }
    }
    const int failed = train_failed(E);
    if (failed) agg = -1;
    s_agg = agg;
    if (agg >= 0) {
      if (E.rule == 1) {
        double tot = 0.0;
        for (int j = 0; j < E.k; ++j) tot += 1.0 / E.vec[(size_t)(E.rec != nullptr ? E.rec[j] : E.sel[j]) * 4 + 3];
        for (int j = 0; j < E.k; ++j)
          s_w[j] = (float)((1.0 / E.vec[(size_t)(E.rec != nullptr ? E.rec[j] : E.sel[j]) * 4 + 3]) / tot);
      } else if (E.rule == 2) {
        for (int j = 0; j < E.k; ++j) s_w[j] = E.hw[j];
      } else {
        const float w = (float)(1.0 / (double)E.k);
        for (int j = 0; j < E.k; ++j) s_w[j] = w;
      }
    }
    if (blockIdx.x == 0) {
      E.state[0] = agg;
      E.state[1] = voter;
      E.report[0] = failed ? ELECT_TRAIN_FAILED : agg;
      E.report[1] = voter;
      if (agg >= 0)
        for (int j = 0; j < E.k; ++j) E.weights[j] = s_w[j];
    }
  }
  __syncthreads();
  if (s_agg < 0) return;
  if (WIDE) {
    // large selections (k > 8, e.g. the 8-rank job's 40): one element per
    // thread and up to 64 selected rows' loads in flight before the first
    // add — the float4 form below waits for 5 dependent rounds at k = 40
    // (20.1 -> 13.2 us); for k <= 8 the float4 form is faster (6.5 vs 8.5 us)
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= W.P) return;
    constexpr int U = 64;
    float acc = 0.f;
    for (int k0 = 0; k0 < W.k; k0 += U) {
      float v[U];
#pragma unroll
      for (int u = 0; u < U; ++u)
        if (k0 + u < W.k) v[u] = W.base[(size_t)s_rows[k0 + u] * W.P + i];
#pragma unroll
      for (int u = 0; u < U; ++u)
        if (k0 + u < W.k)
          acc = (k0 + u == 0) ? __fmul_rn(v[u], s_w[k0 + u]) : __fadd_rn(acc, __fmul_rn(v[u], s_w[k0 + u]));
    }
    W.out[i] = acc;
    return;
  }
  const int i = (blockIdx.x * blockDim.x + threadIdx.x) * 4;
  if (i >= W.P) return;
  // eight independent row loads in flight, added strictly in selection order
  // (the separately rounded fp32 order of weighted_sum_kernel)
  f32x4 acc = zero4();
  constexpr int U = 8;
  for (int k0 = 0; k0 < W.k; k0 += U) {
    f32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (k0 + u < W.k) v[u] = *reinterpret_cast<const f32x4*>(W.base + (size_t)s_rows[k0 + u] * W.P + i);
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (k0 + u < W.k) {
        const float wk = s_w[k0 + u];
#pragma unroll
        for (int r = 0; r < 4; ++r)
          acc[r] = (k0 + u == 0) ? __fmul_rn(v[u][r], wk) : __fadd_rn(acc[r], __fmul_rn(v[u][r], wk));
      }
    }
  }
  *reinterpret_cast<f32x4*>(W.out + i) = acc;
}

struct DecideArgs {
  float* params;           // [n_local, P] hosted clients
  float* anchor;           // [n_local, P]
  float* hist;             // [n_local, P] last received aggregate
  const float* agg;        // [P]
  const int32_t* state;    // aggregator
  const float* sse;        // verification forward: per-row SSE of agg on each receiver's data
  const int32_t* sse_off;  // [n_local] row offset of receiver cl's segment in sse
  const int32_t* sse_n;    // [n_local] rows of that segment
  const int32_t* seg;      // [P] state-dict tensor id of each padded slot (-1 = padding)
  int32_t* agg_counts;     // [N] aggregation-cap counts (bumped here, workgroup 0)
  int32_t* has_hist;       // [n_local]
  double* hist_perf;       // [n_local]
  int32_t* rejected;       // [n_local]
  double* rej_out;         // [N] rejected count per receiver (global id)
  double thr, pthr;
  int32_t start, n_local, P, d_in;
  int32_t mode;            // 0: receivers verify (ModelVerifier); 1: centralised push (legacy
                           //    GlobalAggregator.update): every hosted client, the aggregator
                           //    included, loads the aggregate and re-anchors FedProx, no verification;
                           // 2: thesis rule (Thesis p.20-22 Alg. 4.3): accept iff the aggregate's
                           //    MSE on the receiver's data is finite and <= (1 + thr) x the MSE of
                           //    the receiver's own current model there (fused kernel only);
                           // 3: as 0 with a RELATIVE drift threshold: accept iff
                           //    drift <= thr x sum_tensors ||history||_2 and dperf >= -pthr
  int32_t pad;
};
static_assert(sizeof(DecideArgs) == 152, "DecideArgs layout is shared with Python");

// One 1024-thread workgroup per hosted client.  The verification MSE and the
// parameter drift are reduced here with exactly the arithmetic of
// score_reduce_kernel (threads 0..255) and param_drift_kernel (all 1024
// threads), so decisions are bit-identical to the host-decision path.
__global__ __launch_bounds__(1024) void decide_adopt_kernel(const DecideArgs A) {
  const int a = A.state[0];
  if (a < 0) return;
  if (blockIdx.x == 0 && threadIdx.x == 0) A.agg_counts[a] += 1;
  const int cl = blockIdx.x;
  if (cl >= A.n_local) return;
  const int c = A.start + cl;
  const int had_hist = A.has_hist[cl];  // read by every thread before thread 0 updates it
  __shared__ int s_ok;
  __shared__ double s_d[4];
  __shared__ float part[8][16];
  const size_t off = (size_t)cl * A.P;
  const f32x4* src = reinterpret_cast<const f32x4*>(A.agg);
  const int n4 = A.P / 4;
  if (A.mode == 1) {  // centralised push: load + re-anchor, nothing verified
    for (int i = threadIdx.x; i < n4; i += blockDim.x) {
      reinterpret_cast<f32x4*>(A.params + off)[i] = src[i];
      reinterpret_cast<f32x4*>(A.anchor + off)[i] = src[i];
    }
    return;
  }
  if (c == a) {  // the aggregator loads its aggregate (anchor unchanged)
    for (int i = threadIdx.x; i < n4; i += blockDim.x) reinterpret_cast<f32x4*>(A.params + off)[i] = src[i];
    return;
  }
  const int tid = threadIdx.x;
  const int lane = tid & 63, wv = tid >> 6;
  // ---- MSE of the aggregate on this receiver's data (score_reduce, one batch)
  double mse = 0.0;
  {
    const float* sp = A.sse + A.sse_off[cl];
    const int n = A.sse_n[cl];
    double sv = 0.0;
    if (tid < 256) {
#pragma unroll 8
      for (int r = tid; r < n; r += 256) sv += (double)sp[r];
    }
    for (int o = 32; o >= 1; o >>= 1) sv += __shfl_xor(sv, o, 64);
    if (lane == 0 && wv < 4) s_d[wv] = sv;
    __syncthreads();
    const double tot = s_d[0] + s_d[1] + s_d[2] + s_d[3];
    mse = n > 0 ? tot / ((double)n * A.d_in) : __builtin_nan("");
  }
  // ---- drift of the receiver's history vs the aggregate (param_drift)
  float drift = 0.f, hnorm = 0.f;
  const bool rel = A.mode == 3;
  __shared__ float part_h[8][16];
  if (had_hist) {
    const float* h = A.hist + off;
    float acc[8], acch[8];
#pragma unroll
    for (int t = 0; t < 8; ++t) acc[t] = acch[t] = 0.f;
    for (int p = tid; p < A.P; p += blockDim.x) {
      const int sg = A.seg[p];
      const float df = h[p] - A.agg[p];
#pragma unroll
      for (int t = 0; t < 8; ++t) acc[t] += (sg == t) ? df * df : 0.0f;
      if (rel) {
#pragma unroll
        for (int t = 0; t < 8; ++t) acch[t] += (sg == t) ? h[p] * h[p] : 0.0f;
      }
    }
#pragma unroll
    for (int t = 0; t < 8; ++t) {
      const float v = wave_sum(acc[t]);
      if (lane == 0) part[t][wv] = v;
      if (rel) {
        const float vh = wave_sum(acch[t]);
        if (lane == 0) part_h[t][wv] = vh;
      }
    }
    __syncthreads();
    if (tid == 0) {
      const int nw = blockDim.x >> 6;
      float tot = 0.f, toth = 0.f;
      for (int t = 0; t < 8; ++t) {
        float s2 = 0.f, h2 = 0.f;
        for (int w = 0; w < nw; ++w) {
          s2 += part[t][w];
          if (rel) h2 += part_h[t][w];
        }
        tot += sqrtf(s2);
        toth += sqrtf(h2);
      }
      drift = tot;
      hnorm = toth;
    }
  }
  if (tid == 0) {
    const double perf = 1.0 / (1.0 + mse);
    int ok;
    if (!had_hist) {
      ok = 1;  // the first received model is accepted unconditionally
      A.has_hist[cl] = 1;
    } else {
      const double change = perf - A.hist_perf[cl];
      const double lim = rel ? A.thr * (double)hnorm : A.thr;
      ok = ((double)drift <= lim) && (change >= -A.pthr);
    }
    A.hist_perf[cl] = perf;
    const int rj = ok ? 0 : A.rejected[cl] + 1;
    A.rejected[cl] = rj;
    A.rej_out[c] = (double)rj;
    s_ok = ok;
  }
  __syncthreads();
  const bool ok = s_ok != 0;
  for (int i = tid; i < n4; i += blockDim.x) {
    const f32x4 v = src[i];
    reinterpret_cast<f32x4*>(A.hist + off)[i] = v;
    if (ok) {
      reinterpret_cast<f32x4*>(A.params + off)[i] = v;
      reinterpret_cast<f32x4*>(A.anchor + off)[i] = v;
    }
  }
}

// ---------------------------------------------------------------------------
// Fused verification: per hosted client one 512-thread workgroup stages the
// aggregate, runs the shared batched forward (fwd_rows_block, 8 waves) over
// its verification rows into LDS, then does decide_adopt's work with the same
// reductions (MSE: 256-thread strided sum; drift: each thread plays two of
// decide_adopt's 1024 threads, partial sums combined in the same order) and
// writes the evaluation / artefact snapshots of its rows in the same pass.
// (512 threads: the forward keeps its registers — at 1024 it spilled.)
constexpr int VERIFY_MAX_ROWS = 4096;

struct VerifyArgs {
  DecideArgs D;               // sse / sse_off / sse_n unused
  const int64_t* vx;          // [n_local] address of each receiver's verification rows [n, DP]
  const int32_t* vn;          // [n_local] their row counts (<= VERIFY_MAX_ROWS)
  float* eval_params;         // [n_local, P] parameter snapshot for the side-stream evaluation
  float* best_stage;          // [n_local, P] best-model snapshot for the artefact writer
  const float* best;          // [n_local, P]
  int32_t latent, hidden;
};
static_assert(sizeof(VerifyArgs) == sizeof(DecideArgs) + 48, "VerifyArgs layout is shared with Python");

// (r2 timing-only ablations of this kernel -- no forward 13.4 us, no drift
// 18.9 us, no adoption pass 21.4 us, of 24.6 us -- are in git history and
// profiles/r2_verify_ablations.md)
// REL: the relative drift limit (mode 3) is compiled in only where it is used
template <bool CP, bool REL>
__global__ __launch_bounds__(512) void verify_decide_kernel(const VerifyArgs V) {
  const DecideArgs& A = V.D;
  __shared__ __attribute__((aligned(16))) float sW1[HP * S_W1];
  __shared__ __attribute__((aligned(16))) float sW2[ZP * S_W2];
  __shared__ __attribute__((aligned(16))) float sW3[HP * S_W3];
  __shared__ __attribute__((aligned(16))) float sW4[DP * S_W4];
  __shared__ float s_sse[VERIFY_MAX_ROWS];
  __shared__ int s_ok;
  __shared__ double s_d[4];
  __shared__ float part[8][16];
  __shared__ float part_h[8][16];
  const int a = A.state[0];
  if (a >= 0 && blockIdx.x == 0 && threadIdx.x == 0) A.agg_counts[a] += 1;
  if ((int)blockIdx.x >= A.n_local) {
    // workgroups n_local..2n_local-1: the artefact snapshot best -> best_stage
    // of client blockIdx.x - n_local (independent of every decision, so it
    // runs beside the verification instead of in its adoption pass)
    const int cl2 = blockIdx.x - A.n_local;
    if (cl2 >= A.n_local) return;
    const size_t o2 = (size_t)cl2 * A.P;
    const f32x4* b = reinterpret_cast<const f32x4*>(V.best + o2);
    f32x4* bs = reinterpret_cast<f32x4*>(V.best_stage + o2);
    for (int i = threadIdx.x; i < A.P / 4; i += blockDim.x) bs[i] = b[i];
    return;
  }
  const int cl = blockIdx.x;
  const int c = A.start + cl;
  const int tid = threadIdx.x;
  const int lane = tid & 63, wv = tid >> 6;
  const size_t off = (size_t)cl * A.P;
  const int n4 = A.P / 4;
  const f32x4* src = reinterpret_cast<const f32x4*>(A.agg);
  f32x4* prm = reinterpret_cast<f32x4*>(A.params + off);
  f32x4* evp = reinterpret_cast<f32x4*>(V.eval_params + off);
  bool ok = false, load = false;
  if (a >= 0 && A.mode == 1) {
    load = ok = true;   // centralised push: every hosted client loads and re-anchors
  } else if (a >= 0 && c == a) {
    load = true;   // the aggregator loads its aggregate (anchor / history unchanged)
  } else if (a >= 0) {
    const int had_hist = A.has_hist[cl];
    // ---- SSE rows of the aggregate on this receiver's data (fwd_rows arithmetic)
    FwdDesc d;
    d.params = A.agg;
    d.x = reinterpret_cast<const float*>(V.vx[cl]);
    d.sse = s_sse;
    d.lat = nullptr;
    d.nrows = V.vn[cl];
    d.lat_stride = V.latent;
    d.d_in = A.d_in;
    d.latent = V.latent;
    d.hidden = V.hidden;
    {
      stage_params<CP>(A.agg, sW1, sW2, sW3, sW4);
      __syncthreads();
      fwd_rows_block<CP>(d, sW1, sW2, sW3, sW4, wv, 8, s_sse);
    }
    __syncthreads();
    // ---- MSE (score_reduce / decide_adopt order)
    auto mse_of_rows = [&]() -> double {
      const int n = d.nrows;
      double sv = 0.0;
      if (tid < 256) {
#pragma unroll 8
        for (int r = tid; r < n; r += 256) sv += (double)s_sse[r];
      }
      for (int o = 32; o >= 1; o >>= 1) sv += __shfl_xor(sv, o, 64);
      if (lane == 0 && wv < 4) s_d[wv] = sv;
      __syncthreads();
      const double tot = s_d[0] + s_d[1] + s_d[2] + s_d[3];
      __syncthreads();   // s_d / s_sse reusable
      return n > 0 ? tot / ((double)n * A.d_in) : __builtin_nan("");
    };
    const double mse = mse_of_rows();
    double old_mse = 0.0;
    if (A.mode == 2) {
      // thesis rule: the receiver's own current model on the same rows
      stage_params<CP>(A.params + off, sW1, sW2, sW3, sW4);
      __syncthreads();
      fwd_rows_block<CP>(d, sW1, sW2, sW3, sW4, wv, 8, s_sse);
      __syncthreads();
      old_mse = mse_of_rows();
    }
    // ---- drift of the receiver's history vs the aggregate (param_drift order:
    // virtual threads vt = tid and tid + 512 of a 1024-thread block, each
    // summing p = vt, vt + 1024, ... in increasing order).  All of a
    // thread's loads are issued before the first add: one memory round trip
    // instead of one per 4 elements (6 dependent rounds, ~5 us of the kernel).
    float drift = 0.f, hnorm = 0.f;
    const bool rel = REL && A.mode == 3;
    if (had_hist && (A.mode == 0 || rel)) {
      const float* h = A.hist + off;
      constexpr int NJ = (P_PAD + 1023) / 1024;
      int sg[2][NJ];
      float df[2][NJ], hv[2][NJ];
#pragma unroll
      for (int q = 0; q < 2; ++q)
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
          const int p = tid + 512 * q + 1024 * j;
          sg[q][j] = -1;
          df[q][j] = 0.f;
          hv[q][j] = 0.f;
          if (p < P_PAD) {
            sg[q][j] = A.seg[p];
            hv[q][j] = h[p];
            df[q][j] = hv[q][j] - A.agg[p];
          }
        }
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        float acc[8];
#pragma unroll
        for (int t = 0; t < 8; ++t) acc[t] = 0.f;
#pragma unroll
        for (int j = 0; j < NJ; ++j)
#pragma unroll
          for (int t = 0; t < 8; ++t) acc[t] += (sg[q][j] == t) ? df[q][j] * df[q][j] : 0.0f;
#pragma unroll
        for (int t = 0; t < 8; ++t) {
          const float v = wave_sum(acc[t]);
          if (lane == 0) part[t][wv + 8 * q] = v;
        }
        if (rel) {   // relative threshold: the history's own per-tensor norms, same order
#pragma unroll
          for (int t = 0; t < 8; ++t) acc[t] = 0.f;
#pragma unroll
          for (int j = 0; j < NJ; ++j)
#pragma unroll
            for (int t = 0; t < 8; ++t) acc[t] += (sg[q][j] == t) ? hv[q][j] * hv[q][j] : 0.0f;
#pragma unroll
          for (int t = 0; t < 8; ++t) {
            const float v = wave_sum(acc[t]);
            if (lane == 0) part_h[t][wv + 8 * q] = v;
          }
        }
      }
      __syncthreads();
      if (tid == 0) {
        float tot = 0.f, toth = 0.f;
        for (int t = 0; t < 8; ++t) {
          float s2 = 0.f, h2 = 0.f;
          for (int w = 0; w < 16; ++w) {
            s2 += part[t][w];
            if (rel) h2 += part_h[t][w];
          }
          tot += sqrtf(s2);
          toth += sqrtf(h2);
        }
        drift = tot;
        hnorm = toth;
      }
    }
    if (tid == 0) {
      const double perf = 1.0 / (1.0 + mse);
      int okk;
      if (A.mode == 2) {
        okk = __builtin_isfinite(mse) && mse <= old_mse * (1.0 + A.thr);
        A.has_hist[cl] = 1;
      } else if (!had_hist) {
        okk = 1;  // the first received model is accepted unconditionally
        A.has_hist[cl] = 1;
      } else {
        const double change = perf - A.hist_perf[cl];
        const double lim = rel ? A.thr * (double)hnorm : A.thr;
        okk = ((double)drift <= lim) && (change >= -A.pthr);
      }
      A.hist_perf[cl] = perf;
      const int rj = okk ? 0 : A.rejected[cl] + 1;
      A.rejected[cl] = rj;
      A.rej_out[c] = (double)rj;
      s_ok = okk;
    }
    __syncthreads();
    ok = s_ok != 0;
    load = ok;
  }
  // ---- adoption + history + snapshots in one pass over the row
  // (ModelVerifier receivers, absolute or relative drift limit: the history
  // becomes the received aggregate whatever the decision)
  const bool receiver = a >= 0 && c != a && (A.mode == 0 || A.mode == 3);
  constexpr int UA = (P_PAD / 4 + 511) / 512;   // every element of the row in one pass of loads
  f32x4 v[UA], pv[UA];
#pragma unroll
  for (int u = 0; u < UA; ++u) {
    const int i = tid + 512 * u;
    if (i < n4) {
      v[u] = src[i];
      pv[u] = load ? v[u] : prm[i];
    }
  }
#pragma unroll
  for (int u = 0; u < UA; ++u) {
    const int i = tid + 512 * u;
    if (i < n4) {
      if (load) {
        prm[i] = v[u];
        if (ok) reinterpret_cast<f32x4*>(A.anchor + off)[i] = v[u];
      }
      if (receiver) reinterpret_cast<f32x4*>(A.hist + off)[i] = v[u];
      evp[i] = pv[u];
    }
  }
}

// ---------------------------------------------------------------------------
// Split verification (round 6, VERDICT r5 Next #7): the same decisions,
// adoption and snapshots as verify_decide_kernel (modes 0 / 1 / 3: every
// variant but the thesis rule), with each receiver's work spread over
// `splits` forward workgroups and one drift workgroup instead of one
// workgroup doing all of it in turn (r2 ablations of the fused kernel: the
// forward 11.2 us, the drift 5.7 us, the adoption pass 3.2 us of 24.6).
//
//   workgroup (cl, p < splits): the aggregate's per-row SSE on rows
//       [p T 16, (p+1) T 16) of receiver cl's verification data (T tiles per
//       split; fwd_rows_block, so the rows' SSE are bit-identical to the
//       fused kernel's), published to the scratch row block with sc1 stores;
//   workgroup (cl, splits): the drift of cl's history against the aggregate
//       (the fused kernel's code and order), published as one 8-byte granule;
//   every workgroup then adds 1 to cl's arrival counter, and the LAST one
//       (its add returned splits) reloads the SSE rows into LDS with sc1
//       loads, reduces them in the fused kernel's order, decides, adopts and
//       resets the counter to 0 for the next launch.
// Hand-off (cdna_hip_programming.md §6 Guideline 16 R1; MI355X_MICROARCH.md
// § visibility table row 1, "all those lanes add to ONE unsharded counter,
// the workgroup whose add came last"): every storing wave drains its sc1
// stores, then the workgroup barrier, then ONE lane's agent-scope atomic add;
// the last arriver's other waves load after the barrier its lane then
// joins, every load of the handed-off bytes an sc1 load; hipMalloc memory,
// one workgroup of this kernel per CU at most (60 KB of LDS: 2 per CU fit,
// the row allows one -- the scratch is written by one workgroup and read by
// one, never by two on the same CU at once in one launch, so no L1 copy can
// be stale).  No workgroup waits: the last arriver does the work, so the
// grid needs no co-residency.
struct VerifySplitArgs {
  float* sse;                 // [n_local][VERIFY_MAX_ROWS] per-row SSE scratch
  unsigned long long* drift;  // [n_local] granule {float drift, float history norm}
  uint32_t* count;            // [n_local] arrivals; zero between launches (zeroed once; the last arriver resets)
  int32_t splits;             // forward workgroups per receiver (>= 1)
  int32_t pad;
  uint32_t* done;             // or null: [2] = {departed workgroups (zero between launches), hand-off word}
  uint32_t seq;               // written to done[1] by the launch's last departing workgroup
  int32_t pad2;
};
static_assert(sizeof(VerifySplitArgs) == 48, "VerifySplitArgs layout is shared with Python");

// The side-stream hand-off (round 6): the round's evaluation on the side
// stream reads what this kernel writes for it -- the evaluation snapshot
// (eval_params), the artefact snapshot (best_stage) and the rejection counts
// (rej_out) -- and nothing else of it.  Those are written with sc1 stores;
// every workgroup drains them, passes the workgroup barrier and adds 1 to
// done[0] (one lane, agent scope); the last one (its add returned the grid
// size - 1) resets done[0] and stores `seq` into done[1], on which
// side_wait_kernel polls (cdna_hip_programming.md §6 Guideline 16 R1, the
// hand-off the verification's own last-arriver step uses).  The evaluation
// kernels behind side_wait_kernel start with their dispatch's acquire, so no
// stale L2 line of the snapshots survives into them.  The round's main
// stream then needs no event between this kernel and the next training
// launch (engine/device_round.py; profiles/r6_device_events_ab.md: the
// event's marker packet costs the main stream ~2.6 us per round).
__device__ __forceinline__ void vs_depart(const VerifySplitArgs& S) {
  typedef __attribute__((address_space(1))) uint32_t gu32;
  if (S.done == nullptr) return;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    const uint32_t old = __hip_atomic_fetch_add((gu32*)S.done, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (old == gridDim.x - 1) {
      __hip_atomic_store((gu32*)S.done, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store((gu32*)(S.done + 1), S.seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

typedef unsigned int u32x4v __attribute__((ext_vector_type(4)));
__device__ __forceinline__ __amdgpu_buffer_rsrc_t vs_rsrc(float* p, int bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(p, (short)0, bytes, 0x00020000);
}
constexpr int SC1 = 16;   // buffer instruction cache-policy bits: sc1

template <bool CP, bool REL>
__global__ __launch_bounds__(512) void verify_split_kernel(const VerifyArgs V, const VerifySplitArgs S) {
  typedef __attribute__((address_space(1))) unsigned long long gu64;
  typedef __attribute__((address_space(1))) uint32_t gu32;
  const DecideArgs& A = V.D;
  __shared__ __attribute__((aligned(16))) float sW1[HP * S_W1];
  __shared__ __attribute__((aligned(16))) float sW2[ZP * S_W2];
  __shared__ __attribute__((aligned(16))) float sW3[HP * S_W3];
  __shared__ __attribute__((aligned(16))) float sW4[DP * S_W4];
  __shared__ __attribute__((aligned(16))) float s_sse[VERIFY_MAX_ROWS];
  __shared__ int s_ok, s_last;
  __shared__ double s_d[4];
  __shared__ float part[8][16];
  __shared__ float part_h[8][16];
  const int a = A.state[0];
  const int per = S.splits + 1;
  const int nver = A.n_local * per;
  if (a >= 0 && blockIdx.x == 0 && threadIdx.x == 0) A.agg_counts[a] += 1;
  if ((int)blockIdx.x >= nver) {
    // the artefact snapshot best -> best_stage (as in verify_decide_kernel)
    const int cl2 = blockIdx.x - nver;
    if (cl2 < A.n_local) {
      const size_t o2 = (size_t)cl2 * A.P;
      const f32x4* b = reinterpret_cast<const f32x4*>(V.best + o2);
      const __amdgpu_buffer_rsrc_t bs = vs_rsrc(V.best_stage + o2, 4 * A.P);   // (side-stream input)
      for (int i = threadIdx.x; i < A.P / 4; i += blockDim.x)
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4v, b[i]), bs, 16 * i, 0, SC1);
    }
    vs_depart(S);
    return;
  }
  const int cl = blockIdx.x / per, role = blockIdx.x % per;
  const int c = A.start + cl;
  const int tid = threadIdx.x;
  const int lane = tid & 63, wv = tid >> 6;
  const size_t off = (size_t)cl * A.P;
  const bool verifying = a >= 0 && A.mode != 1 && c != a;
  const bool rel = REL && A.mode == 3;
  const int had_hist = verifying ? A.has_hist[cl] : 0;   // (the last arriver updates it after every add)
  const int n = V.vn[cl];
  float* const sse_g = S.sse + (size_t)cl * VERIFY_MAX_ROWS;
  if (verifying && role < S.splits) {
    // ---- forward share: T tiles from tile role * T
    const int ntiles = (n + 15) >> 4;
    const int T = (ntiles + S.splits - 1) / S.splits;
    const int row0 = min(n, role * T * 16);
    const int nr = min(n - row0, T * 16);
    if (nr > 0) {
      FwdDesc d;
      d.params = A.agg;
      d.x = reinterpret_cast<const float*>(V.vx[cl]) + (size_t)row0 * DP;
      d.sse = s_sse;
      d.lat = nullptr;
      d.nrows = nr;
      d.lat_stride = V.latent;
      d.d_in = A.d_in;
      d.latent = V.latent;
      d.hidden = V.hidden;
      stage_params<CP>(A.agg, sW1, sW2, sW3, sW4);
      __syncthreads();
      fwd_rows_block<CP>(d, sW1, sW2, sW3, sW4, wv, 8, s_sse);
      __syncthreads();
      // publish the rows' SSE: 16-byte sc1 stores (row0 is a multiple of 16)
      const __amdgpu_buffer_rsrc_t rs = vs_rsrc(sse_g + row0, 4 * ((nr + 3) & ~3));
      for (int i = tid; i < (nr + 3) >> 2; i += 512)
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4v, lds_read4(s_sse + 4 * i)), rs, 16 * i, 0,
                                               16);
    }
  } else if (verifying && had_hist && (A.mode == 0 || rel)) {
    // ---- drift (verify_decide_kernel's code and summation order)
    const float* h = A.hist + off;
    constexpr int NJ = (P_PAD + 1023) / 1024;
    int sg[2][NJ];
    float df[2][NJ], hv[2][NJ];
#pragma unroll
    for (int q = 0; q < 2; ++q)
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const int p = tid + 512 * q + 1024 * j;
        sg[q][j] = -1;
        df[q][j] = 0.f;
        hv[q][j] = 0.f;
        if (p < P_PAD) {
          sg[q][j] = A.seg[p];
          hv[q][j] = h[p];
          df[q][j] = hv[q][j] - A.agg[p];
        }
      }
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      float acc[8];
#pragma unroll
      for (int t = 0; t < 8; ++t) acc[t] = 0.f;
#pragma unroll
      for (int j = 0; j < NJ; ++j)
#pragma unroll
        for (int t = 0; t < 8; ++t) acc[t] += (sg[q][j] == t) ? df[q][j] * df[q][j] : 0.0f;
#pragma unroll
      for (int t = 0; t < 8; ++t) {
        const float v = wave_sum(acc[t]);
        if (lane == 0) part[t][wv + 8 * q] = v;
      }
      if (rel) {
#pragma unroll
        for (int t = 0; t < 8; ++t) acc[t] = 0.f;
#pragma unroll
        for (int j = 0; j < NJ; ++j)
#pragma unroll
          for (int t = 0; t < 8; ++t) acc[t] += (sg[q][j] == t) ? hv[q][j] * hv[q][j] : 0.0f;
#pragma unroll
        for (int t = 0; t < 8; ++t) {
          const float v = wave_sum(acc[t]);
          if (lane == 0) part_h[t][wv + 8 * q] = v;
        }
      }
    }
    __syncthreads();
    if (tid == 0) {
      float tot = 0.f, toth = 0.f;
      for (int t = 0; t < 8; ++t) {
        float s2 = 0.f, h2 = 0.f;
        for (int w = 0; w < 16; ++w) {
          s2 += part[t][w];
          if (rel) h2 += part_h[t][w];
        }
        tot += sqrtf(s2);
        toth += sqrtf(h2);
      }
      const unsigned long long g = (unsigned long long)__builtin_bit_cast(uint32_t, tot) |
                                   ((unsigned long long)__builtin_bit_cast(uint32_t, toth) << 32);
      __hip_atomic_store((gu64*)(S.drift + cl), g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  // ---- arrival: every storing wave drained, one lane adds; the last one decides
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0) {
    const uint32_t old = __hip_atomic_fetch_add((gu32*)(S.count + cl), 1u, __ATOMIC_RELAXED,
                                                __HIP_MEMORY_SCOPE_AGENT);
    s_last = old == (uint32_t)(per - 1);
    if (s_last) __hip_atomic_store((gu32*)(S.count + cl), 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  if (!s_last) {
    vs_depart(S);
    return;
  }
  bool ok = false, load = false;
  if (a >= 0 && A.mode == 1) {
    load = ok = true;   // centralised push: every hosted client loads and re-anchors
  } else if (a >= 0 && c == a) {
    load = true;   // the aggregator loads its aggregate (anchor / history unchanged)
  } else if (a >= 0) {
    // the rows' SSE back into LDS (sc1 loads), then the fused kernel's MSE order
    {
      const __amdgpu_buffer_rsrc_t rs = vs_rsrc(sse_g, 4 * ((n + 3) & ~3));
      for (int i = tid; i < (n + 3) >> 2; i += 512)
        lds_write4(s_sse + 4 * i, __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, 16 * i, 0, 16)));
    }
    __syncthreads();
    double sv = 0.0;
    if (tid < 256) {
#pragma unroll 8
      for (int r = tid; r < n; r += 256) sv += (double)s_sse[r];
    }
    for (int o = 32; o >= 1; o >>= 1) sv += __shfl_xor(sv, o, 64);
    if (lane == 0 && wv < 4) s_d[wv] = sv;
    __syncthreads();
    const double tot = s_d[0] + s_d[1] + s_d[2] + s_d[3];
    const double mse = n > 0 ? tot / ((double)n * A.d_in) : __builtin_nan("");
    if (tid == 0) {
      float drift = 0.f, hnorm = 0.f;
      if (had_hist && (A.mode == 0 || rel)) {
        const unsigned long long g = __hip_atomic_load((gu64*)(S.drift + cl), __ATOMIC_RELAXED,
                                                       __HIP_MEMORY_SCOPE_AGENT);
        drift = __builtin_bit_cast(float, (uint32_t)g);
        hnorm = __builtin_bit_cast(float, (uint32_t)(g >> 32));
      }
      const double perf = 1.0 / (1.0 + mse);
      int okk;
      if (!had_hist) {
        okk = 1;  // the first received model is accepted unconditionally
        A.has_hist[cl] = 1;
      } else {
        const double change = perf - A.hist_perf[cl];
        const double lim = rel ? A.thr * (double)hnorm : A.thr;
        okk = ((double)drift <= lim) && (change >= -A.pthr);
      }
      A.hist_perf[cl] = perf;
      const int rj = okk ? 0 : A.rejected[cl] + 1;
      A.rejected[cl] = rj;
      __hip_atomic_store((gu64*)(A.rej_out + c), __builtin_bit_cast(unsigned long long, (double)rj),
                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);   // (side-stream input)
      s_ok = okk;
    }
    __syncthreads();
    ok = s_ok != 0;
    load = ok;
  }
  // ---- adoption + history + snapshots in one pass over the row (as verify_decide_kernel)
  const bool receiver = a >= 0 && c != a && (A.mode == 0 || A.mode == 3);
  const int n4 = A.P / 4;
  const f32x4* src = reinterpret_cast<const f32x4*>(A.agg);
  f32x4* prm = reinterpret_cast<f32x4*>(A.params + off);
  const __amdgpu_buffer_rsrc_t evp = vs_rsrc(V.eval_params + off, 4 * A.P);   // (side-stream input)
  constexpr int UA = (P_PAD / 4 + 511) / 512;
  f32x4 v[UA], pv[UA];
#pragma unroll
  for (int u = 0; u < UA; ++u) {
    const int i = tid + 512 * u;
    if (i < n4) {
      v[u] = src[i];
      pv[u] = load ? v[u] : prm[i];
    }
  }
#pragma unroll
  for (int u = 0; u < UA; ++u) {
    const int i = tid + 512 * u;
    if (i < n4) {
      if (load) {
        prm[i] = v[u];
        if (ok) reinterpret_cast<f32x4*>(A.anchor + off)[i] = v[u];
      }
      if (receiver) reinterpret_cast<f32x4*>(A.hist + off)[i] = v[u];
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4v, pv[u]), evp, 16 * i, 0, SC1);
    }
  }
  vs_depart(S);
}

// The side stream's wait for the verification's hand-off word (vs_depart):
// one lane polls done[1] until it reaches `seq` (bounded: past timeout_ticks
// it sets the host-visible status word and exits, and the host raises when
// it collects the round).  Nothing else -- the evaluation kernels behind it
// acquire at their own dispatch.
__global__ __launch_bounds__(64) void side_wait_kernel(uint32_t* word, uint32_t seq, int* status,
                                                       long long timeout_ticks) {
  typedef __attribute__((address_space(1))) uint32_t gu32;
  if (threadIdx.x != 0) return;
  const long long t0 = (long long)wall_clock64();
  while ((int)(__hip_atomic_load((gu32*)word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) - seq) < 0) {
    if ((long long)wall_clock64() - t0 > timeout_ticks) {
      if (status) __hip_atomic_store(status, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      break;
    }
    __builtin_amdgcn_s_sleep(2);
  }
}

__global__ __launch_bounds__(256) void copy_f64_kernel(double* __restrict__ dst, const double* __restrict__ src,
                                                       int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) dst[i] = src[i];
}

// two independent copies in one launch (blockIdx.y selects the pair)
__global__ __launch_bounds__(256) void copy2_f64_kernel(double* __restrict__ d0, const double* __restrict__ s0, int n0,
                                                        double* __restrict__ d1, const double* __restrict__ s1,
                                                        int n1) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (blockIdx.y == 0) {
    if (i < n0) d0[i] = s0[i];
  } else if (i < n1) {
    d1[i] = s1[i];
  }
}

// Row gather / scatter: dst[(didx ? didx[i] : i) * dstride + j] =
// src[(sidx ? sidx[i] : i) * sstride + j] for i < n, j < len (floats; len and
// the strides are multiples of 4).  Index arrays usually live in the mapped
// descriptor ring, so packing the multi-rank exchange needs no host copies.
__global__ __launch_bounds__(256) void copy_rows_kernel(float* __restrict__ dst, int dstride,
                                                        const int32_t* __restrict__ didx,
                                                        const float* __restrict__ src, int sstride,
                                                        const int32_t* __restrict__ sidx, int len) {
  const int i = blockIdx.y;
  const int j = (blockIdx.x * blockDim.x + threadIdx.x) * 4;
  if (j >= len) return;
  const size_t d = (size_t)(didx ? didx[i] : i) * dstride + j;
  const size_t s = (size_t)(sidx ? sidx[i] : i) * sstride + j;
  *reinterpret_cast<f32x4*>(dst + d) = *reinterpret_cast<const f32x4*>(src + s);
}

}  // namespace fedmx

extern "C" {

int fedmx_copy_rows(float* dst, int dstride, const int32_t* didx, const float* src, int sstride, const int32_t* sidx,
                    int n, int len, hipStream_t stream) {
  if (n <= 0 || len <= 0) return 0;
  if (len % 4 || dstride % 4 || sstride % 4 || n > 65535) return -1;
  hipLaunchKernelGGL(fedmx::copy_rows_kernel, dim3((len / 4 + 255) / 256, n), dim3(256), 0, stream, dst, dstride,
                     didx, src, sstride, sidx, len);
  return (int)hipGetLastError();
}

int fedmx_copy2_f64(double* d0, const double* s0, int n0, double* d1, const double* s1, int n1, hipStream_t stream) {
  const int n = max(n0, n1);
  if (n <= 0) return 0;
  hipLaunchKernelGGL(fedmx::copy2_f64_kernel, dim3((n + 255) / 256, 2), dim3(256), 0, stream, d0, s0, n0, d1, s1, n1);
  return (int)hipGetLastError();
}

int fedmx_decide_adopt(const void* args, hipStream_t stream) {
  const fedmx::DecideArgs& A = *reinterpret_cast<const fedmx::DecideArgs*>(args);
  if (A.P % 4 != 0 || A.P != fedmx::P_PAD) return -1;
  // at least one workgroup: it bumps the replicated aggregation-cap count
  hipLaunchKernelGGL(fedmx::decide_adopt_kernel, dim3(A.n_local > 0 ? A.n_local : 1), dim3(1024), 0, stream, A);
  return (int)hipGetLastError();
}

int fedmx_elect_wsum(const void* eargs, const void* wargs, hipStream_t stream) {
  const fedmx::ElectArgs& E = *reinterpret_cast<const fedmx::ElectArgs*>(eargs);
  const fedmx::WsumArgs& W = *reinterpret_cast<const fedmx::WsumArgs*>(wargs);
  if (W.P % 4 != 0 || W.k < 1 || E.k > 1024) return -1;
  if (W.k > 8)
    hipLaunchKernelGGL(fedmx::elect_wsum_kernel<true>, dim3((W.P + 255) / 256), dim3(256), 0, stream, E, W);
  else
    hipLaunchKernelGGL(fedmx::elect_wsum_kernel<false>, dim3((W.P / 4 + 255) / 256), dim3(256), 0, stream, E, W);
  return (int)hipGetLastError();
}

// Split verification (modes 0 / 1 / 3); -5: the thesis rule (mode 2) needs
// the fused kernel
int fedmx_verify_split(const void* args, const void* sargs, hipStream_t stream) {
  const fedmx::VerifyArgs& V = *reinterpret_cast<const fedmx::VerifyArgs*>(args);
  const fedmx::VerifySplitArgs& S = *reinterpret_cast<const fedmx::VerifySplitArgs*>(sargs);
  if (V.D.P % 4 != 0 || V.D.P != fedmx::P_PAD || S.splits < 1 || S.splits > 64) return -1;
  if (V.D.mode == 2) return -5;
  const int nl = V.D.n_local;
  // n_local x (splits forward + 1 drift) workgroups, then n_local snapshot copies
  const dim3 grid(nl > 0 ? nl * (S.splits + 1) + nl : 1);
  const bool cp = V.D.d_in <= 115 && V.hidden <= 27 && V.latent <= 7;
  if (V.D.mode == 3) {
    if (cp)
      hipLaunchKernelGGL((fedmx::verify_split_kernel<true, true>), grid, dim3(512), 0, stream, V, S);
    else
      hipLaunchKernelGGL((fedmx::verify_split_kernel<false, true>), grid, dim3(512), 0, stream, V, S);
  } else if (cp) {
    hipLaunchKernelGGL((fedmx::verify_split_kernel<true, false>), grid, dim3(512), 0, stream, V, S);
  } else {
    hipLaunchKernelGGL((fedmx::verify_split_kernel<false, false>), grid, dim3(512), 0, stream, V, S);
  }
  return (int)hipGetLastError();
}

int fedmx_side_wait(void* word, uint32_t seq, void* status, long long timeout_ticks, hipStream_t stream) {
  hipLaunchKernelGGL(fedmx::side_wait_kernel, dim3(1), dim3(64), 0, stream, reinterpret_cast<uint32_t*>(word), seq,
                     reinterpret_cast<int*>(status), timeout_ticks);
  return (int)hipGetLastError();
}

int fedmx_verify_split_args_size(void) { return (int)sizeof(fedmx::VerifySplitArgs); }

int fedmx_verify_decide(const void* args, hipStream_t stream) {
  const fedmx::VerifyArgs& V = *reinterpret_cast<const fedmx::VerifyArgs*>(args);
  if (V.D.P % 4 != 0 || V.D.P != fedmx::P_PAD) return -1;
  // n_local verification workgroups + n_local snapshot-copy workgroups
  const dim3 grid(V.D.n_local > 0 ? 2 * V.D.n_local : 1);
  // compact forward order for the reference shapes (fedmx_forward_common.h)
  const bool cp = V.D.d_in <= 115 && V.hidden <= 27 && V.latent <= 7;
  if (V.D.mode == 3) {
    if (cp)
      hipLaunchKernelGGL((fedmx::verify_decide_kernel<true, true>), grid, dim3(512), 0, stream, V);
    else
      hipLaunchKernelGGL((fedmx::verify_decide_kernel<false, true>), grid, dim3(512), 0, stream, V);
  } else if (cp) {
    hipLaunchKernelGGL((fedmx::verify_decide_kernel<true, false>), grid, dim3(512), 0, stream, V);
  } else {
    hipLaunchKernelGGL((fedmx::verify_decide_kernel<false, false>), grid, dim3(512), 0, stream, V);
  }
  return (int)hipGetLastError();
}

int fedmx_copy_f64(double* dst, const double* src, int n, hipStream_t stream) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(fedmx::copy_f64_kernel, dim3((n + 255) / 256), dim3(256), 0, stream, dst, src, n);
  return (int)hipGetLastError();
}

int fedmx_protocol_sizes(int* out) {
  out[0] = (int)sizeof(fedmx::ElectArgs);
  out[1] = (int)sizeof(fedmx::WsumArgs);
  out[2] = (int)sizeof(fedmx::DecideArgs);
  out[3] = (int)sizeof(fedmx::VerifyArgs);
  return 0;
}

}  // extern "C"
