// mr_ensemble.hip — combination models and the reference's threshold mAP on
// the device, over dense models of one context's shard (n_te x width of the
// context's out_dtype, NaN = no pair). MR = MusicRecommender.scala:
//   getLinearCombinationModel(P)      MR:317-351  out = ubm*alpha + ibm*(1-alpha)
//   getAggregationModel(P)            MR:361-418  pair index < (int)(p*P) -> ibm, else ubm
//   getStochasticCombinationModel(P)  MR:429-481  nextFloat() < p -> ibm, else ubm; the
//                                     reference's java.util.Random is unseeded, here a
//                                     seeded counter-based stream over the pair index
//   evaluateModel                     MR:521-639  global min/max (MR:524-525), per-class
//                                     confusion counts at the thresholds (MR:541-553):
//                                     0.0..0.9 (10, MR:590) or 0.0..1.0 (11, the
//                                     distributed evaluation, distributed.scala:395);
//                                     AP per class and the mean (mr_eval_map[_device])
// The pair index is the position of (u, s) in the driver's sorted model
// (main.scala:57-59 sorts by (user, song): the interned order, heard songs
// skipped): idx(u, s) = pair_base + u*n_s - te_off[u] + s - |{t in T(u): t < s}|.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <vector>

#include "mr_engine.h"

namespace mr_host {
int fail(int code, const char* fmt, ...);  // thread-local error slot (mr_engine.hip)
}

namespace {

using mr_host::fail;

#define MR_HIP(call)                                                                            \
  do {                                                                                          \
    hipError_t e_ = (call);                                                                     \
    if (e_ != hipSuccess)                                                                       \
      return fail(e_ == hipErrorOutOfMemory ? MR_E_OOM : MR_E_HIP, "%s failed: %s (%s:%d)", #call, \
                  hipGetErrorString(e_), __FILE__, __LINE__);                                   \
  } while (0)

constexpr int kThreads = 256;
// Thresholds: the first n of 0.0, 0.1, ..., 1.0 — n = 10 for MusicRecommender's
// evaluateModel (MR:590: 0.0 :: ... :: 0.9 :: Nil), n = 11 for the distributed
// evaluation (distributed.scala:395: Array(0.0, ..., 1.0)); the same literals.
constexpr int kThresholds = 11;  // the most any evaluation uses
#define MR_THRESHOLDS {0.0, 0.1, 0.2, 0.3, 0.4, 0.5, 0.6, 0.7, 0.8, 0.9, 1.0}
__constant__ double kThr[kThresholds] = MR_THRESHOLDS;
constexpr double kThrHost[kThresholds] = MR_THRESHOLDS;

inline int thresholds_or_default(int n) { return n == 0 ? 10 : n; }

// ---- combination models -----------------------------------------------------
struct CombParams {
  int n_te, width, song_lo, n_songs, kind;
  double param;
  unsigned long long seed;
  long long pair_base, threshold;
  const long long* te_off;
  const int* te_songs;
  const void* ubm;
  const void* ibm;
  void* out;
};

// splitmix64 finaliser over (seed, pair index): a stateless stream, so every
// pair's draw is independent of launch geometry and shard count.
__host__ __device__ inline unsigned long long splitmix64(unsigned long long z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
// 24 random bits / 2^24, the distribution of java.util.Random.nextFloat.
__host__ __device__ inline float pair_uniform(unsigned long long seed, long long idx) {
  const unsigned long long z = splitmix64(seed + (unsigned long long)(idx + 1) * 0x9E3779B97F4A7C15ull);
  return (float)(unsigned)(z >> 40) * (1.0f / 16777216.0f);
}

#ifndef MR_COMB_PER
#define MR_COMB_PER 8  // C5: 86.44 vs 87.00 ms per step at 4 (profiles/r04/s35)
#endif
constexpr int kCombPer = MR_COMB_PER;  // songs per thread (strided by kThreads: coalesced)

// One (user, kThreads * kCombPer-song block) per workgroup. The pair index
// needs |{t in T(u): t < s}|: one binary search per block for the first heard
// song at or after the block, then the few heard songs inside the block are
// walked per element (T(u) is sorted; rows are short).
template <typename OutT>
__global__ __launch_bounds__(kThreads) void k_combine(CombParams p) {
  const int u = blockIdx.y;
  const int i0 = blockIdx.x * kThreads * kCombPer + threadIdx.x;
  const size_t row = (size_t)u * p.width;
  const OutT* ubm = reinterpret_cast<const OutT*>(p.ubm) + row;
  const OutT* ibm = reinterpret_cast<const OutT*>(p.ibm) + row;
  OutT* out = reinterpret_cast<OutT*>(p.out) + row;
  OutT a4[kCombPer], b4[kCombPer];
#pragma unroll
  for (int r = 0; r < kCombPer; ++r) {
    const int i = i0 + r * kThreads;
    a4[r] = i < p.width ? ubm[i] : (OutT)0;
    b4[r] = i < p.width ? ibm[i] : (OutT)0;
  }
  if (p.kind == MR_COMB_LINEAR) {  // MR:327: rank1 * alpha + rank2 * (1 - alpha); NaN stays NaN
#pragma unroll
    for (int r = 0; r < kCombPer; ++r) {
      const int i = i0 + r * kThreads;
      if (i < p.width) out[i] = (OutT)((double)a4[r] * p.param + (double)b4[r] * (1.0 - p.param));
    }
    return;
  }
  const long long t0 = p.te_off[u], t1 = p.te_off[u + 1];
  const int s_blk = p.song_lo + blockIdx.x * kThreads * kCombPer;  // first song of the block
  long long a = t0, b = t1;  // first song of T(u) >= s_blk (uniform over the block)
  while (a < b) {
    const long long m = (a + b) >> 1;
    if (p.te_songs[m] < s_blk) a = m + 1; else b = m;
  }
#pragma unroll
  for (int r = 0; r < kCombPer; ++r) {
    const int i = i0 + r * kThreads;
    if (i >= p.width) continue;
    const int s = p.song_lo + i;
    long long j = a;  // first song of T(u) >= s
    while (j < t1 && p.te_songs[j] < s) ++j;
    if (j < t1 && p.te_songs[j] == s) {  // heard: no pair (MR:109)
      out[i] = (OutT)NAN;
      continue;
    }
    const long long idx = p.pair_base + (long long)u * p.n_songs - t0 + s - (j - t0);
    const bool take_ibm = p.kind == MR_COMB_AGGREGATION ? idx < p.threshold                   // MR:380-381
                                                        : (double)pair_uniform(p.seed, idx) < p.param;  // MR:414-415
    out[i] = take_ibm ? b4[r] : a4[r];
  }
}

// The driver's three combinations in one pass (mr_combine_all_device): each
// block reads its ubm / ibm elements once and writes the linear, aggregation
// and stochastic outputs with k_combine's exact expressions; with part != null
// it also leaves the min / max of each output over its pairs (NaN skipped, in
// the element type, as k_minmax) in part[block][6].
struct Comb3Params {
  int n_te, width, song_lo, n_songs;
  double alpha, p_sto;
  unsigned long long seed;
  long long pair_base, threshold;
  const long long* te_off;
  const int* te_songs;
  const void* ubm;
  const void* ibm;
  void* out[3];  // linear, aggregation, stochastic
  double* part;
};
template <typename OutT>
__global__ __launch_bounds__(kThreads) void k_combine3(Comb3Params p) {
  __shared__ double sm[6][kThreads];
  const int u = blockIdx.y;
  const int i0 = blockIdx.x * kThreads * kCombPer + threadIdx.x;
  const size_t row = (size_t)u * p.width;
  const OutT* ubm = reinterpret_cast<const OutT*>(p.ubm) + row;
  const OutT* ibm = reinterpret_cast<const OutT*>(p.ibm) + row;
  OutT* o_lin = reinterpret_cast<OutT*>(p.out[0]) + row;
  OutT* o_agg = reinterpret_cast<OutT*>(p.out[1]) + row;
  OutT* o_sto = reinterpret_cast<OutT*>(p.out[2]) + row;
  OutT a4[kCombPer], b4[kCombPer];
#pragma unroll
  for (int r = 0; r < kCombPer; ++r) {
    const int i = i0 + r * kThreads;
    a4[r] = i < p.width ? ubm[i] : (OutT)0;
    b4[r] = i < p.width ? ibm[i] : (OutT)0;
  }
  const long long t0 = p.te_off[u], t1 = p.te_off[u + 1];
  const int s_blk = p.song_lo + blockIdx.x * kThreads * kCombPer;  // first song of the block
  long long a = t0, b = t1;  // first song of T(u) >= s_blk (uniform over the block)
  while (a < b) {
    const long long m = (a + b) >> 1;
    if (p.te_songs[m] < s_blk) a = m + 1; else b = m;
  }
  OutT mn[3], mx[3];
#pragma unroll
  for (int c = 0; c < 3; ++c) { mn[c] = (OutT)INFINITY; mx[c] = (OutT)-INFINITY; }
  auto track = [&](int c, OutT x) {
    if (x != x) return;
    mn[c] = x < mn[c] ? x : mn[c];
    mx[c] = x > mx[c] ? x : mx[c];
  };
#pragma unroll
  for (int r = 0; r < kCombPer; ++r) {
    const int i = i0 + r * kThreads;
    if (i >= p.width) continue;
    const OutT lin = (OutT)((double)a4[r] * p.alpha + (double)b4[r] * (1.0 - p.alpha));  // MR:327
    o_lin[i] = lin;
    track(0, lin);
    const int s = p.song_lo + i;
    long long j = a;  // first song of T(u) >= s
    while (j < t1 && p.te_songs[j] < s) ++j;
    if (j < t1 && p.te_songs[j] == s) {  // heard: no pair (MR:109)
      o_agg[i] = (OutT)NAN;
      o_sto[i] = (OutT)NAN;
      continue;
    }
    const long long idx = p.pair_base + (long long)u * p.n_songs - t0 + s - (j - t0);
    const OutT agg = idx < p.threshold ? b4[r] : a4[r];                               // MR:380-381
    const OutT sto = (double)pair_uniform(p.seed, idx) < p.p_sto ? b4[r] : a4[r];     // MR:414-415
    o_agg[i] = agg;
    o_sto[i] = sto;
    track(1, agg);
    track(2, sto);
  }
  if (!p.part) return;
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    sm[2 * c][threadIdx.x] = (double)mn[c];
    sm[2 * c + 1][threadIdx.x] = (double)mx[c];
  }
  __syncthreads();
  for (int h = kThreads / 2; h > 0; h >>= 1) {
    if ((int)threadIdx.x < h)
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        sm[2 * c][threadIdx.x] = fmin(sm[2 * c][threadIdx.x], sm[2 * c][threadIdx.x + h]);
        sm[2 * c + 1][threadIdx.x] = fmax(sm[2 * c + 1][threadIdx.x], sm[2 * c + 1][threadIdx.x + h]);
      }
    __syncthreads();
  }
  if (threadIdx.x < 6) p.part[((size_t)blockIdx.y * gridDim.x + blockIdx.x) * 6 + threadIdx.x] = sm[threadIdx.x][0];
}

// part[n][6] (min, max, min, max, min, max) -> part2[gridDim.x][6]
__global__ __launch_bounds__(kThreads) void k_minmax6(const double* part, long long n, double* part2) {
  __shared__ double sm[6][kThreads];
  double v[6] = {INFINITY, -INFINITY, INFINITY, -INFINITY, INFINITY, -INFINITY};
  for (long long b = (long long)blockIdx.x * kThreads + threadIdx.x; b < n; b += (long long)gridDim.x * kThreads)
#pragma unroll
    for (int c = 0; c < 6; ++c) v[c] = (c & 1) ? fmax(v[c], part[b * 6 + c]) : fmin(v[c], part[b * 6 + c]);
#pragma unroll
  for (int c = 0; c < 6; ++c) sm[c][threadIdx.x] = v[c];
  __syncthreads();
  for (int h = kThreads / 2; h > 0; h >>= 1) {
    if ((int)threadIdx.x < h)
#pragma unroll
      for (int c = 0; c < 6; ++c)
        sm[c][threadIdx.x] = (c & 1) ? fmax(sm[c][threadIdx.x], sm[c][threadIdx.x + h])
                                     : fmin(sm[c][threadIdx.x], sm[c][threadIdx.x + h]);
    __syncthreads();
  }
  if (threadIdx.x < 6) part2[(size_t)blockIdx.x * 6 + threadIdx.x] = sm[threadIdx.x][0];
}

// ---- evaluation ------------------------------------------------------------
constexpr int kMinmaxPer = 8;  // loads in flight per thread per iteration

template <typename OutT>
__global__ __launch_bounds__(kThreads) void k_minmax(const OutT* d, long long n, double* part) {
  __shared__ double smn[kThreads], smx[kThreads];
  OutT mn = (OutT)INFINITY, mx = (OutT)-INFINITY;  // min/max are exact in the element type
  const long long stride = (long long)gridDim.x * kThreads;
  for (long long i0 = (long long)blockIdx.x * kThreads + threadIdx.x; i0 < n; i0 += stride * kMinmaxPer) {
    OutT x[kMinmaxPer];
#pragma unroll
    for (int r = 0; r < kMinmaxPer; ++r) {
      const long long i = i0 + r * stride;
      x[r] = i < n ? d[i] : (OutT)NAN;
    }
#pragma unroll
    for (int r = 0; r < kMinmaxPer; ++r) {
      if (x[r] != x[r]) continue;
      mn = x[r] < mn ? x[r] : mn;
      mx = x[r] > mx ? x[r] : mx;
    }
  }
  smn[threadIdx.x] = (double)mn;
  smx[threadIdx.x] = (double)mx;
  __syncthreads();
  for (int h = kThreads / 2; h > 0; h >>= 1) {
    if ((int)threadIdx.x < h) {
      smn[threadIdx.x] = fmin(smn[threadIdx.x], smn[threadIdx.x + h]);
      smx[threadIdx.x] = fmax(smx[threadIdx.x], smx[threadIdx.x + h]);
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    part[2 * blockIdx.x] = smn[0];
    part[2 * blockIdx.x + 1] = smx[0];
  }
}

struct EvalParams {
  int n_te, width, song_lo, users_per_block, n_thr;
  double mn, mx;
  const void* dense;
  int* pred;  // [width][n_thr]: users with (x - min) / (max - min) > t_i (MR:529)
  int* tp;    // [width][n_thr]: of those, users whose labels hold the song (MR:545)
  const int* lab_u;
  const int* lab_s;
  long long n_lab;
  float xt_f[kThresholds];   // smallest score with (x - min) / (max - min) > t_i (f32 models)
  double xt_d[kThresholds];  // the same for f64 models
};

// The level test (x - mn) / (mx - mn) > t of MR:529 is monotone in x (fp64
// subtraction and division by a positive range are monotone under rounding),
// so it equals x >= xt with xt the smallest score of the model's element type
// that passes. Found on the host by bisection over the ordered bit patterns of
// that type, with the same fp64 expression: exact, and the kernel then needs
// n_thr compares per element instead of an fp64 division.
template <typename T, typename U>
T level_floor(double mn, double mx, double t) {
  constexpr int B = sizeof(T) * 8;
  const U sign = (U)1 << (B - 1);
  auto key = [&](T x) { U b; std::memcpy(&b, &x, sizeof b); return (b & sign) ? (U)~b : (U)(b | sign); };
  auto val = [&](U k) { U b = (k & sign) ? (U)(k & ~sign) : (U)~k; T x; std::memcpy(&x, &b, sizeof x); return x; };
  auto pass = [&](U k) { return ((double)val(k) - mn) / (mx - mn) > t; };
  U lo = key(-INFINITY), hi = key(INFINITY);  // NaN patterns lie outside [lo, hi]
  if (!pass(hi)) return (T)NAN;               // nothing passes (mx == mn: 0 / 0)
  while (lo < hi) {                           // smallest passing key
    const U m = lo + (hi - lo) / 2;
    if (pass(m)) hi = m; else lo = m + 1;
  }
  return val(lo);
}

__device__ __forceinline__ int levels(double x, double mn, double mx, int n_thr) {
  const double v = (x - mn) / (mx - mn);  // MR:529 (NaN > t is false)
  int c = 0;
#pragma unroll
  for (int t = 0; t < kThresholds; ++t) c += (t < n_thr && v > kThr[t]) ? 1 : 0;
  return c;  // thresholds ascend: predicted at t_i for every i < c
}

// one thread per song column, a block of users per blockIdx.y (rows read coalesced)
#ifndef MR_EVAL_U
#define MR_EVAL_U 16  // C5: 86.53 vs 87.00 ms per step at 8 (profiles/r04/s35)
#endif
template <typename OutT>
__global__ __launch_bounds__(kThreads) void k_eval_pred(EvalParams p) {
  const int i = blockIdx.x * kThreads + threadIdx.x;
  if (i >= p.width) return;
  const int u0 = blockIdx.y * p.users_per_block, u1 = min(p.n_te, u0 + p.users_per_block);
  const OutT* d = reinterpret_cast<const OutT*>(p.dense);
  OutT xt[kThresholds];
#pragma unroll
  for (int t = 0; t < kThresholds; ++t)  // unused slots: +inf, never reached
    xt[t] = t < p.n_thr ? (sizeof(OutT) == 4 ? (OutT)p.xt_f[t] : (OutT)p.xt_d[t]) : (OutT)INFINITY;
  int cnt[kThresholds];
#pragma unroll
  for (int t = 0; t < kThresholds; ++t) cnt[t] = 0;
  constexpr int U = MR_EVAL_U;  // rows in flight per thread
  for (int ub = u0; ub < u1; ub += U) {
    OutT x[U];
#pragma unroll
    for (int r = 0; r < U; ++r) x[r] = ub + r < u1 ? d[(size_t)(ub + r) * p.width + i] : (OutT)NAN;
#pragma unroll
    for (int r = 0; r < U; ++r)
#pragma unroll
      for (int t = 0; t < kThresholds; ++t) cnt[t] += x[r] >= xt[t] ? 1 : 0;  // NaN (no pair): never
  }
  if (gridDim.y == 1) {  // one user block: this thread owns the song's counts (no zeroing, no atomics)
#pragma unroll
    for (int t = 0; t < kThresholds; ++t)
      if (t < p.n_thr) p.pred[(size_t)i * p.n_thr + t] = cnt[t];
    return;
  }
#pragma unroll
  for (int t = 0; t < kThresholds; ++t)
    if (cnt[t]) atomicAdd(&p.pred[(size_t)i * p.n_thr + t], cnt[t]);
}

template <typename OutT>
__global__ __launch_bounds__(kThreads) void k_eval_tp(EvalParams p) {
  const long long j = (long long)blockIdx.x * kThreads + threadIdx.x;
  if (j >= p.n_lab) return;
  const int u = p.lab_u[j], g = p.lab_s[j] - p.song_lo;
  if (g < 0 || g >= p.width) return;  // other shard, or a label-only song (never predicted)
  const double x = (double)reinterpret_cast<const OutT*>(p.dense)[(size_t)u * p.width + g];
  if (x != x) return;
  const int c = levels(x, p.mn, p.mx, p.n_thr);
  for (int t = 0; t < c; ++t) atomicAdd(&p.tp[(size_t)g * p.n_thr + t], 1);
}

// AP of the label classes cls[0..n) of the shard (shard-local song ids, np =
// their label counts pos, all > 0; MR:588-618), the host fold's exact double
// operations (mr_eval_map) per class.
__global__ __launch_bounds__(kThreads) void k_eval_ap(int n, int n_thr, const int* cls, const int* cpos,
                                                      const int* pred, const int* tp, double* ap) {
  const int c = blockIdx.x * kThreads + threadIdx.x;
  if (c >= n) return;
  const int g = cls[c];
  const int np = cpos[c];
  double P[kThresholds], R[kThresholds];
#pragma unroll
  for (int t = 0; t < kThresholds; ++t) {
    const size_t i = (size_t)g * n_thr + (t < n_thr ? t : 0);
    P[t] = pred[i] > 0 ? (double)tp[i] / (double)pred[i] : 0.0;
    R[t] = (double)tp[i] / (double)np;
  }
  // AP = sum over i of: (R_i - R_{i+1}) * P_i, (R_{n-2} - 0.0) * P_{n-2} at
  // i = n - 2, 0 at i = n - 1 (MR:601-609, distributed.scala:405-413), left fold
  double a = 0.0;
#pragma unroll
  for (int t = 0; t < kThresholds; ++t) {
    if (t >= n_thr) break;
    const double term = t == n_thr - 1 ? 0.0 : t == n_thr - 2 ? (R[t] - 0.0) * P[t] : (R[t] - R[t + 1]) * P[t];
    a = a + term;
  }
  ap[c] = a;
}

// The label classes' rows of the shard's counts, in a class-indexed block
// that every rank lays out alike (the global class list): out[0][c][t] =
// pred, out[1][c][t] = tp of class c when its song is in [song_lo, song_hi),
// else 0 — so summing the blocks over ranks (one all-reduce) gives the counts
// of MR:541-553 over every test user, whatever the layout.
__global__ __launch_bounds__(kThreads) void k_eval_gather(int n_cls, int n_thr, int song_lo, int width,
                                                          const int* cls, const int* pred, const int* tp,
                                                          int* out) {
  const int j = blockIdx.x * kThreads + threadIdx.x;
  if (j >= n_cls * n_thr) return;
  const int c = j / n_thr, t = j - c * n_thr;
  const int g = cls[c] - song_lo;
  const bool in = g >= 0 && g < width;
  out[j] = in ? pred[(size_t)g * n_thr + t] : 0;
  out[(size_t)n_cls * n_thr + j] = in ? tp[(size_t)g * n_thr + t] : 0;
}

template <typename T>
struct Tmp {  // scratch device buffer of one call, stream-ordered (pool allocator: no device sync)
  T* p = nullptr;
  hipStream_t st = nullptr;
  ~Tmp() { if (p) (void)hipFreeAsync(p, st); }
};

// pred / tp counts of the shard into the device buffers d_pred / d_tp
// ([width][n_thr], stream-ordered on the context stream; the caller frees
// them), for n_models dense models in turn: the labels are staged once, and
// after model i's counts are queued after(i) queues what consumes them (the
// buffers are reused by model i + 1, in stream order).
template <typename After>
int eval_counts(mr_ctx* ctx, int n_models, const void* const* dense, const double* mn, const double* mx,
                const int64_t* lab_off, const int32_t* lab_songs, int n_thr, mr_view& v, Tmp<int>& d_pred,
                Tmp<int>& d_tp, After&& after) {
  if (!ctx || !dense || !lab_off || !mn || !mx || n_models < 1) return fail(MR_E_INVALID, "null argument");
  for (int i = 0; i < n_models; ++i)
    if (!dense[i]) return fail(MR_E_INVALID, "null dense model %d", i);
  if (n_thr != 10 && n_thr != 11)
    return fail(MR_E_INVALID, "%d thresholds: 10 (MR:590) or 11 (distributed.scala:395)", n_thr);
  int rc = mr_view_get(ctx, &v);
  if (rc) return rc;
  MR_HIP(hipSetDevice(v.device));
  const int width = v.song_hi - v.song_lo, n_te = v.n_test_users;
  const long long n_lab = lab_off[n_te];
  if (n_lab > 0 && !lab_songs) return fail(MR_E_INVALID, "null label songs");
  std::vector<int32_t> lu((size_t)std::max<long long>(1, n_lab)), ls((size_t)std::max<long long>(1, n_lab));
  for (int u = 0; u < n_te; ++u)
    for (int64_t j = lab_off[u]; j < lab_off[u + 1]; ++j) {
      if (j < 0 || j >= n_lab || lab_off[u + 1] < lab_off[u]) return fail(MR_E_INVALID, "bad label CSR");
      lu[j] = u;
      ls[j] = lab_songs[j];
    }
  hipStream_t st = (hipStream_t)v.stream;
  Tmp<int> d_lu, d_ls;
  d_pred.st = d_tp.st = d_lu.st = d_ls.st = st;
  const size_t nc = (size_t)width * n_thr;
  MR_HIP(hipMallocAsync(reinterpret_cast<void**>(&d_pred.p), std::max<size_t>(1, nc) * 4, st));
  MR_HIP(hipMallocAsync(reinterpret_cast<void**>(&d_tp.p), std::max<size_t>(1, nc) * 4, st));
  MR_HIP(hipMallocAsync(reinterpret_cast<void**>(&d_lu.p), lu.size() * 4, st));
  MR_HIP(hipMallocAsync(reinterpret_cast<void**>(&d_ls.p), ls.size() * 4, st));
  MR_HIP(hipMemcpyAsync(d_lu.p, lu.data(), lu.size() * 4, hipMemcpyHostToDevice, st));
  MR_HIP(hipMemcpyAsync(d_ls.p, ls.data(), ls.size() * 4, hipMemcpyHostToDevice, st));
  // (song block x user block) workgroups: ~1024 of them fill the chip (a
  // thread keeps 16 rows' loads in flight); a user block per workgroup row
  // adds its counts atomically, so split the users only when the songs alone
  // give too few workgroups (narrow shards). One user block (the whole model
  // of a wide shard, any user count): plain stores, no zeroing, no atomics —
  // the atomics, not the model's bytes, were the pass's cost at a few hundred
  // users (C5's 250-user blocks at 8 GPUs: 0.84 ms per model).
  const int sx = (width + kThreads - 1) / kThreads;
  const int uy = std::max(1, std::min((n_te + 15) / 16, (1024 + sx - 1) / sx));
  const bool f64 = v.out_dtype == MR_OUT_F64;
  for (int i = 0; i < n_models; ++i) {
    if (uy > 1) MR_HIP(hipMemsetAsync(d_pred.p, 0, nc * 4, st));
    MR_HIP(hipMemsetAsync(d_tp.p, 0, nc * 4, st));
    EvalParams ep{n_te, width, v.song_lo, (n_te + uy - 1) / uy, n_thr, mn[i], mx[i], dense[i], d_pred.p, d_tp.p,
                  d_lu.p, d_ls.p, n_lab};
    for (int t = 0; t < n_thr; ++t) {
      const double thr = kThrHost[t];
      ep.xt_f[t] = level_floor<float, uint32_t>(mn[i], mx[i], thr);
      ep.xt_d[t] = level_floor<double, uint64_t>(mn[i], mx[i], thr);
    }
    if (width > 0) {
      if (f64) hipLaunchKernelGGL(k_eval_pred<double>, dim3(sx, uy), dim3(kThreads), 0, st, ep);
      else hipLaunchKernelGGL(k_eval_pred<float>, dim3(sx, uy), dim3(kThreads), 0, st, ep);
      MR_HIP(hipGetLastError());
    }
    if (n_lab > 0) {
      const int lb = (int)((n_lab + kThreads - 1) / kThreads);
      if (f64) hipLaunchKernelGGL(k_eval_tp<double>, dim3(lb), dim3(kThreads), 0, st, ep);
      else hipLaunchKernelGGL(k_eval_tp<float>, dim3(lb), dim3(kThreads), 0, st, ep);
      MR_HIP(hipGetLastError());
    }
    if ((rc = after(i))) return rc;
  }
  // the label staging is freed in stream order after these kernels (Tmp)
  return MR_OK;
}

}  // namespace

extern "C" {

int mr_combine_device(mr_ctx* ctx, int kind, double param, uint64_t seed, int64_t pair_base, int64_t n_pairs,
                      const void* ubm, const void* ibm, void* out) {
  if (!ctx || !ubm || !ibm || !out) return fail(MR_E_INVALID, "null argument");
  if (kind != MR_COMB_LINEAR && kind != MR_COMB_AGGREGATION && kind != MR_COMB_STOCHASTIC)
    return fail(MR_E_INVALID, "unknown combination kind %d", kind);
  // MR:366-369 / MR:434-437: the reference prints and calls System.exit(-1)
  if (kind != MR_COMB_LINEAR && !(param >= 0.0 && param <= 1.0))
    return fail(MR_E_INVALID, "percentage/probability %g must be between 0 and 1", param);
  mr_view v;
  int rc = mr_view_get(ctx, &v);
  if (rc) return rc;
  if (pair_base < 0 || n_pairs < 0) return fail(MR_E_INVALID, "negative pair_base / n_pairs");
  MR_HIP(hipSetDevice(v.device));
  const int width = v.song_hi - v.song_lo;
  CombParams cp{v.n_test_users, width, v.song_lo, v.n_songs, kind, param, (unsigned long long)seed,
                (long long)pair_base, (long long)(param * (double)n_pairs),  // (p * length).toInt, MR:371
                reinterpret_cast<const long long*>(v.te_off), v.te_songs, ubm, ibm, out};
  hipStream_t st = (hipStream_t)v.stream;
  for (int y0 = 0; y0 < v.n_test_users; y0 += 65535) {
    CombParams q = cp;
    const int ny = std::min(65535, v.n_test_users - y0);
    const size_t esz = v.out_dtype == MR_OUT_F64 ? 8 : 4;
    q.n_te = ny;
    q.te_off = cp.te_off + y0;  // values index the whole te_songs: pairs before user y0 + u are
    q.pair_base = cp.pair_base + (long long)y0 * v.n_songs;  // (y0 + u) * n_s - te_off[y0 + u]
    q.ubm = (const char*)ubm + (size_t)y0 * width * esz;
    q.ibm = (const char*)ibm + (size_t)y0 * width * esz;
    q.out = (char*)out + (size_t)y0 * width * esz;
    dim3 grid((width + kThreads * kCombPer - 1) / (kThreads * kCombPer), ny);
    if (v.out_dtype == MR_OUT_F64) hipLaunchKernelGGL(k_combine<double>, grid, dim3(kThreads), 0, st, q);
    else hipLaunchKernelGGL(k_combine<float>, grid, dim3(kThreads), 0, st, q);
    MR_HIP(hipGetLastError());
  }
  MR_HIP(hipStreamSynchronize(st));
  return MR_OK;
}

int mr_combine_all_device(mr_ctx* ctx, double alpha, double ibm_percentage, double ibm_probability, uint64_t seed,
                          int64_t pair_base, int64_t n_pairs, const void* ubm, const void* ibm, void* out_linear,
                          void* out_aggregation, void* out_stochastic, double* minmax) {
  if (!ctx || !ubm || !ibm || !out_linear || !out_aggregation || !out_stochastic)
    return fail(MR_E_INVALID, "null argument");
  // MR:366-369 / MR:434-437: the reference prints and calls System.exit(-1)
  if (!(ibm_percentage >= 0.0 && ibm_percentage <= 1.0) || !(ibm_probability >= 0.0 && ibm_probability <= 1.0))
    return fail(MR_E_INVALID, "percentage %g / probability %g must be between 0 and 1", ibm_percentage,
                ibm_probability);
  mr_view v;
  int rc = mr_view_get(ctx, &v);
  if (rc) return rc;
  if (pair_base < 0 || n_pairs < 0) return fail(MR_E_INVALID, "negative pair_base / n_pairs");
  MR_HIP(hipSetDevice(v.device));
  const int width = v.song_hi - v.song_lo;
  const size_t esz = v.out_dtype == MR_OUT_F64 ? 8 : 4;
  Comb3Params cp{v.n_test_users, width, v.song_lo, v.n_songs, alpha, ibm_probability, (unsigned long long)seed,
                 (long long)pair_base, (long long)(ibm_percentage * (double)n_pairs),  // (p * length).toInt, MR:371
                 reinterpret_cast<const long long*>(v.te_off), v.te_songs, ubm, ibm,
                 {out_linear, out_aggregation, out_stochastic}, nullptr};
  hipStream_t st = (hipStream_t)v.stream;
  const int gx = (width + kThreads * kCombPer - 1) / (kThreads * kCombPer);
  const long long nblk = (long long)gx * v.n_test_users;
  Tmp<double> part, part2;
  part.st = part2.st = st;
  constexpr int kRed = 256;  // k_minmax6 blocks
  if (minmax && nblk > 0) {
    MR_HIP(hipMallocAsync(reinterpret_cast<void**>(&part.p), (size_t)nblk * 6 * sizeof(double), st));
    MR_HIP(hipMallocAsync(reinterpret_cast<void**>(&part2.p), (size_t)kRed * 6 * sizeof(double), st));
  }
  for (int y0 = 0; gx > 0 && y0 < v.n_test_users; y0 += 65535) {
    Comb3Params q = cp;
    const int ny = std::min(65535, v.n_test_users - y0);
    q.n_te = ny;
    q.te_off = cp.te_off + y0;  // values index the whole te_songs (see mr_combine_device)
    q.pair_base = cp.pair_base + (long long)y0 * v.n_songs;
    q.ubm = (const char*)ubm + (size_t)y0 * width * esz;
    q.ibm = (const char*)ibm + (size_t)y0 * width * esz;
    for (int c = 0; c < 3; ++c) q.out[c] = (char*)cp.out[c] + (size_t)y0 * width * esz;
    q.part = part.p ? part.p + (size_t)y0 * gx * 6 : nullptr;
    dim3 grid(gx, ny);
    if (v.out_dtype == MR_OUT_F64) hipLaunchKernelGGL(k_combine3<double>, grid, dim3(kThreads), 0, st, q);
    else hipLaunchKernelGGL(k_combine3<float>, grid, dim3(kThreads), 0, st, q);
    MR_HIP(hipGetLastError());
  }
  if (minmax) {
    double h[kRed * 6];
    for (int c = 0; c < 6; ++c) minmax[c] = (c & 1) ? -INFINITY : INFINITY;
    if (nblk > 0) {
      hipLaunchKernelGGL(k_minmax6, dim3(kRed), dim3(kThreads), 0, st, part.p, nblk, part2.p);
      MR_HIP(hipGetLastError());
      MR_HIP(hipMemcpyAsync(h, part2.p, sizeof h, hipMemcpyDeviceToHost, st));
      MR_HIP(hipStreamSynchronize(st));
      for (int b = 0; b < kRed; ++b)
        for (int c = 0; c < 6; ++c)
          minmax[c] = (c & 1) ? std::fmax(minmax[c], h[b * 6 + c]) : std::fmin(minmax[c], h[b * 6 + c]);
    }
  }
  MR_HIP(hipStreamSynchronize(st));
  return MR_OK;
}

int mr_eval_minmax_device(mr_ctx* ctx, const void* dense, double* mn, double* mx) {
  if (!ctx || !dense || !mn || !mx) return fail(MR_E_INVALID, "null argument");
  mr_view v;
  int rc = mr_view_get(ctx, &v);
  if (rc) return rc;
  MR_HIP(hipSetDevice(v.device));
  const long long n = (long long)v.n_test_users * (v.song_hi - v.song_lo);
  const int blocks = (int)std::max<long long>(1, std::min<long long>(4096, (n + kThreads - 1) / kThreads));
  hipStream_t st = (hipStream_t)v.stream;
  Tmp<double> part;
  part.st = st;
  MR_HIP(hipMallocAsync(reinterpret_cast<void**>(&part.p), (size_t)blocks * 2 * sizeof(double), st));
  if (v.out_dtype == MR_OUT_F64)
    hipLaunchKernelGGL(k_minmax<double>, dim3(blocks), dim3(kThreads), 0, st, (const double*)dense, n, part.p);
  else
    hipLaunchKernelGGL(k_minmax<float>, dim3(blocks), dim3(kThreads), 0, st, (const float*)dense, n, part.p);
  MR_HIP(hipGetLastError());
  std::vector<double> h((size_t)blocks * 2);
  MR_HIP(hipMemcpyAsync(h.data(), part.p, h.size() * sizeof(double), hipMemcpyDeviceToHost, st));
  MR_HIP(hipStreamSynchronize(st));
  double a = INFINITY, b = -INFINITY;
  for (int i = 0; i < blocks; ++i) {
    a = std::fmin(a, h[2 * i]);
    b = std::fmax(b, h[2 * i + 1]);
  }
  *mn = a;
  *mx = b;
  return MR_OK;
}

int mr_eval_counts_device(mr_ctx* ctx, const void* dense, double mn, double mx, const int64_t* lab_off,
                          const int32_t* lab_songs, int32_t* pred_counts, int32_t* tp_counts, int32_t n_thresholds) {
  if (!pred_counts || !tp_counts) return fail(MR_E_INVALID, "null argument");
  const int n_thr = thresholds_or_default(n_thresholds);
  mr_view v;
  Tmp<int> d_pred, d_tp;
  int rc = eval_counts(ctx, 1, &dense, &mn, &mx, lab_off, lab_songs, n_thr, v, d_pred, d_tp, [](int) { return 0; });
  if (rc) return rc;
  hipStream_t st = (hipStream_t)v.stream;
  const size_t nc = (size_t)(v.song_hi - v.song_lo) * n_thr;
  MR_HIP(hipMemcpyAsync(pred_counts, d_pred.p, nc * 4, hipMemcpyDeviceToHost, st));
  MR_HIP(hipMemcpyAsync(tp_counts, d_tp.p, nc * 4, hipMemcpyDeviceToHost, st));
  MR_HIP(hipStreamSynchronize(st));
  return MR_OK;
}

int mr_eval_map_device(mr_ctx* ctx, const void* dense, double mn, double mx, const int64_t* lab_off,
                       const int32_t* lab_songs, const int32_t* pos, int32_t n_label_songs, double* map_out,
                       int32_t n_thresholds) {
  if (!pos || !map_out) return fail(MR_E_INVALID, "null argument");
  const int n_thr = thresholds_or_default(n_thresholds);
  mr_view v;
  Tmp<int> d_pred, d_tp;
  int rc = eval_counts(ctx, 1, &dense, &mn, &mx, lab_off, lab_songs, n_thr, v, d_pred, d_tp, [](int) { return 0; });
  if (rc) return rc;
  hipStream_t st = (hipStream_t)v.stream;
  const int width = v.song_hi - v.song_lo;
  // Only the label classes (pos > 0, ascending) cross PCIe: their ids and
  // counts in, their AP out (C5: ~1/10 of the shard's songs).
  std::vector<int32_t> cls, cpos;
  for (int g = 0; g < width; ++g)
    if (pos[v.song_lo + g] > 0) { cls.push_back(g); cpos.push_back(pos[v.song_lo + g]); }
  const int nc = (int)cls.size();
  Tmp<int> d_cls, d_cpos;
  Tmp<double> d_ap;
  d_cls.st = d_cpos.st = d_ap.st = st;
  std::vector<double> ap((size_t)std::max(1, nc));
  if (nc > 0) {
    MR_HIP(hipMallocAsync(reinterpret_cast<void**>(&d_cls.p), (size_t)nc * 4, st));
    MR_HIP(hipMallocAsync(reinterpret_cast<void**>(&d_cpos.p), (size_t)nc * 4, st));
    MR_HIP(hipMallocAsync(reinterpret_cast<void**>(&d_ap.p), (size_t)nc * 8, st));
    MR_HIP(hipMemcpyAsync(d_cls.p, cls.data(), (size_t)nc * 4, hipMemcpyHostToDevice, st));
    MR_HIP(hipMemcpyAsync(d_cpos.p, cpos.data(), (size_t)nc * 4, hipMemcpyHostToDevice, st));
    hipLaunchKernelGGL(k_eval_ap, dim3((nc + kThreads - 1) / kThreads), dim3(kThreads), 0, st, nc, n_thr, d_cls.p,
                       d_cpos.p, d_pred.p, d_tp.p, d_ap.p);
    MR_HIP(hipGetLastError());
    MR_HIP(hipMemcpyAsync(ap.data(), d_ap.p, (size_t)nc * 8, hipMemcpyDeviceToHost, st));
  }
  MR_HIP(hipStreamSynchronize(st));
  double total = 0.0;  // classes in song-id order, as mr_eval_map (MR:625-627)
  for (int c = 0; c < nc; ++c) total += ap[c];
  *map_out = n_label_songs > 0 ? total / (double)n_label_songs : NAN;
  return MR_OK;
}

int mr_eval_class_counts_device(mr_ctx* ctx, int32_t n_models, const void* const* dense, const double* mn,
                                const double* mx, const int64_t* lab_off, const int32_t* lab_songs, int32_t n_classes,
                                const int32_t* classes, int32_t* counts, int32_t n_thresholds) {
  if (!counts || (n_classes > 0 && !classes) || n_classes < 0) return fail(MR_E_INVALID, "null argument");
  for (int32_t c = 1; c < n_classes; ++c)
    if (classes[c] <= classes[c - 1]) return fail(MR_E_INVALID, "classes not strictly ascending at %d", (int)c);
  const int n_thr = thresholds_or_default(n_thresholds);
  mr_view v;
  Tmp<int> d_pred, d_tp, d_cls;
  const size_t blk = (size_t)2 * n_classes * n_thr;  // one model's block
  auto gather = [&](int i) -> int {
    if (n_classes == 0) return 0;
    hipStream_t st = (hipStream_t)v.stream;
    if (!d_cls.p) {  // the class list, staged once (after eval_counts resolved the context)
      d_cls.st = st;
      MR_HIP(hipMallocAsync(reinterpret_cast<void**>(&d_cls.p), (size_t)n_classes * 4, st));
      MR_HIP(hipMemcpyAsync(d_cls.p, classes, (size_t)n_classes * 4, hipMemcpyHostToDevice, st));
    }
    const int n = n_classes * n_thr;
    hipLaunchKernelGGL(k_eval_gather, dim3((n + kThreads - 1) / kThreads), dim3(kThreads), 0, st, n_classes, n_thr,
                       v.song_lo, v.song_hi - v.song_lo, d_cls.p, d_pred.p, d_tp.p, counts + (size_t)i * blk);
    MR_HIP(hipGetLastError());
    return 0;
  };
  int rc = eval_counts(ctx, n_models, dense, mn, mx, lab_off, lab_songs, n_thr, v, d_pred, d_tp, gather);
  if (rc) return rc;
  MR_HIP(hipStreamSynchronize((hipStream_t)v.stream));  // the host staging (labels, classes) has been read
  return MR_OK;
}

int mr_eval_map_counts_device(mr_ctx* ctx, int32_t n_models, int32_t n_classes, const int32_t* class_pos,
                              const int32_t* counts, int32_t n_label_songs, double* maps_out, int32_t n_thresholds) {
  if (!ctx || !maps_out || n_models < 1 || n_classes < 0 || (n_classes > 0 && (!class_pos || !counts)))
    return fail(MR_E_INVALID, "null argument");
  for (int32_t c = 0; c < n_classes; ++c)
    if (class_pos[c] <= 0) return fail(MR_E_INVALID, "class %d has no positive (pos %d)", (int)c, (int)class_pos[c]);
  const int n_thr = thresholds_or_default(n_thresholds);
  if (n_thr != 10 && n_thr != 11)
    return fail(MR_E_INVALID, "%d thresholds: 10 (MR:590) or 11 (distributed.scala:395)", n_thr);
  mr_view v;
  int rc = mr_view_get(ctx, &v);
  if (rc) return rc;
  MR_HIP(hipSetDevice(v.device));
  hipStream_t st = (hipStream_t)v.stream;
  const size_t nap = (size_t)n_models * n_classes;
  std::vector<double> ap(std::max<size_t>(1, nap));
  if (n_classes > 0) {
    // every model's classes as one launch: AP row m * n_classes + c reads
    // model m's block, pred at [m][0][c][t], tp at [m][1][c][t] — tp is the
    // pred pointer + n_classes * n_thr, so index the classes of model m as
    // m * 2 * n_classes + c
    std::vector<int32_t> cls(nap), cpos(nap);
    for (int m = 0; m < n_models; ++m)
      for (int c = 0; c < n_classes; ++c) {
        cls[(size_t)m * n_classes + c] = 2 * m * n_classes + c;
        cpos[(size_t)m * n_classes + c] = class_pos[c];
      }
    Tmp<int> d_cls, d_cpos;
    Tmp<double> d_ap;
    d_cls.st = d_cpos.st = d_ap.st = st;
    MR_HIP(hipMallocAsync(reinterpret_cast<void**>(&d_cls.p), nap * 4, st));
    MR_HIP(hipMallocAsync(reinterpret_cast<void**>(&d_cpos.p), nap * 4, st));
    MR_HIP(hipMallocAsync(reinterpret_cast<void**>(&d_ap.p), nap * 8, st));
    MR_HIP(hipMemcpyAsync(d_cls.p, cls.data(), nap * 4, hipMemcpyHostToDevice, st));
    MR_HIP(hipMemcpyAsync(d_cpos.p, cpos.data(), nap * 4, hipMemcpyHostToDevice, st));
    hipLaunchKernelGGL(k_eval_ap, dim3((unsigned)((nap + kThreads - 1) / kThreads)), dim3(kThreads), 0, st, (int)nap,
                       n_thr, d_cls.p, d_cpos.p, counts, counts + (size_t)n_classes * n_thr, d_ap.p);
    MR_HIP(hipGetLastError());
    MR_HIP(hipMemcpyAsync(ap.data(), d_ap.p, nap * 8, hipMemcpyDeviceToHost, st));
  }
  MR_HIP(hipStreamSynchronize(st));
  for (int m = 0; m < n_models; ++m) {
    double total = 0.0;  // classes in song-id order, as mr_eval_map (MR:625-627)
    for (int c = 0; c < n_classes; ++c) total += ap[(size_t)m * n_classes + c];
    maps_out[m] = n_label_songs > 0 ? total / (double)n_label_songs : NAN;
  }
  return MR_OK;
}

}  // extern "C"
