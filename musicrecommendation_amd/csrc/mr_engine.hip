// mr_engine.hip — MI355X (gfx950) collaborative-filtering similarity engine.
//
// Replaces the per-pair scoring MapReduce of the reference
// (src/main/scala/music_recommandation/MusicRecommender.scala, "MR"):
//   getModel(rank)            MR:105-111   (all unheard (user, song) pairs)
//   UBM cosine + rank         MR:140-166
//   IBM cosine + rank         MR:230-257
// by a two-stage sparse computation (SURVEY.md §0.1 "two-hop identity"):
//   stage 1, per test user u, one weight per train neighbour v
//       ibm: y_v = Σ_{s2 ∈ T(u) ∩ S(v)} q(s2),   q(s2) = rint(2^F / sqrt c(s2))
//       ubm: o_v = |T(u) ∩ S(v)|,  q_v = rint(2^F · o_v / (sqrt|T(u)| · sqrt|S(v)|))
//   stage 2, per (u, song tile) an LDS int64 accumulator
//       acc[s] = Σ_{v ∈ N(u), s ∈ S(v)} weight_v
//       ibm: score = acc·2^-F / sqrt c(s);  ubm: score = acc·2^-F
//     + dense write (NaN for heard songs, MR:109) + the tile's top-k
//   stage 3, per test user, the top-k over all tiles, done inside the same
//       launch by the workgroup that finishes the user's last tile.
// Two launch shapes:
//   fused    (small train sets): ONE kernel; every (u, tile) workgroup
//            rebuilds u's neighbour weights in LDS (k_score<.., FUSED=true>);
//   separate (large train sets): k_neighbours writes compacted neighbour
//            lists, then k_score<.., FUSED=false> reads them.
// ItemBasedModel on large train sets, the co-listening route (round 3,
// DESIGN.md §4b): per run, an index of C[s2][s] = |L_tr(s2) ∩ L_tr(s)| for
// every test-visible song s2 (k_cooc_light / k_cooc_light_wave: LDS hash per
// row; k_cooc_build: LDS counters per (row, tile)), then per (u, tile)
//       acc[s] = Σ_{s2 ∈ T(u)} q(s2) · C[s2][s]      (k_score_wide<.., COOC>)
//   — the same int64 sum as stage 1 + stage 2 with the two sums exchanged.
// Integer accumulation is associative, so every launch geometry, shard count,
// route and the CPU fixed-point oracle (oracle/fixedpoint.c) give
// bit-identical scores and hence identical top-k order. Built with
// -ffp-contract=off.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <climits>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <limits>
#include <mutex>
#include <string>
#include <vector>

#ifndef MR_TILE_ROWS
#define MR_TILE_ROWS 32  // threshold rows of the fused tile top-k (C2: 17.9 us vs 18.3 at 16; 8 < k falls back, 26.6)
#endif

#include "mr_engine.h"
#include "mr_internal.h"
#include "mr_par.h"


namespace {

constexpr int kThreads = 256;             // 4 waves of 64
constexpr int kWaves = kThreads / 64;
constexpr int kMaxTopK = 64;
constexpr int kMaxBlockSongs = 16384;     // 128 KiB of int64 accumulators (LDS is 160 KiB)
constexpr int kLdsBytes = 160 * 1024;     // LDS per workgroup (CU) on gfx950
constexpr int kMaxWideBlockSongs = 65536; // wide shape: uint16 tile-local ids, LDS-bound in practice
constexpr int kMaxLdsTrainUsers = 16384;  // stage-1 dense neighbour array in LDS (int64), one chunk
constexpr int kStage1Chunk = 4096;        // larger train sets: stage 1 in LDS chunks of train users (C4
                                          // batch 21.3 vs 21.9 ms at 8192, 23.8 at 16384, 22.5 at 2048;
                                          // profiles/r02/c4/stage1_chunk_sweep.txt)
constexpr int kMaxChunks = 2048;          // => n_train_users <= 8.4M
constexpr int kMaxFusedTrainUsers = 4096; // fused path: Y (32 KiB) + tile live together
constexpr long long kKeyNone = -1;        // valid keys are bit patterns of doubles >= 0
constexpr int kMaxTopkTile = 1024;        // songs per tile for the register top-k (4 per lane)
constexpr int kMaxTopkLarge = 16;         // k limit of the wide-tile top-k (per-thread running lists)
constexpr int kFusedPre = 4;              // fused shape: tile entries per thread prefetched before stage 1
constexpr int kWideMapDefault = 1;        // wide-shape block mapping (wide_map_opt)

thread_local std::string g_err = "no error";

int fail(int code, const char* fmt, ...) {
  char buf[1024];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  g_err = buf;
  return code;
}

}  // namespace

namespace mr_host {
// Error slot used by mr_host.cpp (same thread-local message as the device part).
int fail(int code, const char* fmt, ...) {
  char buf[1024];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  g_err = buf;
  return code;
}
}  // namespace mr_host

namespace {

#define MR_HIP(call)                                                                   \
  do {                                                                                 \
    hipError_t e_ = (call);                                                            \
    if (e_ != hipSuccess)                                                              \
      return fail(e_ == hipErrorOutOfMemory ? MR_E_OOM : MR_E_HIP, "%s failed: %s (%s:%d)", \
                  #call, hipGetErrorString(e_), __FILE__, __LINE__);                   \
  } while (0)

// ---------------------------------------------------------------------------
// LDS layout of k_score (bytes; every region 16-byte aligned).
// ---------------------------------------------------------------------------
struct ScoreLds {
  int acc, y, heard, s_lo, s_w, s_pre, s_scan, wk, ws, fk, fs, flag, cpre, stg, gm, stage_lists, total;
};
// threshold top-k scratch of a 256-thread block with up to 64 rows
// (= topk_scratch_bytes<kThreads, 64>())
constexpr int kTopkScratch256 = (64 + 1) * 12 + 4 + 64 * 4 + 256 * 4;

// Separate shape, stage 2: per-wave staging of one round of neighbours
// (kStgItems segments: start, exclusive prefix of lengths, weight).
constexpr int kStgItems = 256;
constexpr int kStgBytes = kStgItems * 8 + kStgItems * 4 + (kStgItems + 4) * 4;  // q, a, pre

__host__ __device__ inline int align16(int x) { return (x + 15) & ~15; }
__host__ __device__ inline int merge_lists_per_pass(int k);

// Region A (offset 0) holds the tile accumulators (+ the fused path's
// neighbour array Y); after the tile's own top-k it is reused to stage tile
// candidate lists for the in-launch merge (stage_lists lists per pass), and
// by the wide-tile top-k for its per-thread lists. n_chunks: separate shape's
// stage-1 chunk count (prefix of the per-chunk neighbour counts).
__host__ __device__ inline ScoreLds score_lds(int bs, int fused_ntr, int k, int n_tiles, int n_chunks = 0) {
  ScoreLds L;
  const int fused = fused_ntr > 0 ? 1 : 0;
  const int kk = k > 0 ? k : 1;
  const int per = merge_lists_per_pass(kk);
  L.stage_lists = (k > 0 && n_tiles > 1) ? (n_tiles < per ? n_tiles : per) : 0;
  int a_bytes = bs * 8 + fused_ntr * 8;
  const int st_bytes = L.stage_lists * kk * 8 + align16(L.stage_lists * kk * 4);
  const int wide_bytes = (k > 0 && bs > kMaxTopkTile) ? kThreads * kk * 8 + kThreads * kk * 4 : 0;
  if (wide_bytes > a_bytes) a_bytes = wide_bytes;
  int o = 0;
  L.acc = o; L.y = bs * 8; o = align16(a_bytes > st_bytes ? a_bytes : st_bytes);
  L.heard = o; o = align16(o + (bs / 32) * 4);
  L.s_lo = o; o += fused * kThreads * 8;
  L.s_w = o; o += fused * kThreads * 8;
  L.s_pre = o; o = align16(o + (kThreads + 1) * 4);
  L.s_scan = o; o = align16(o + kWaves * 4);
  L.wk = o; o = align16(o + kWaves * kMaxTopK * 8);
  L.ws = o; o = align16(o + kWaves * kMaxTopK * 4);
  L.fk = o; o = align16(o + kMaxTopK * 8);
  L.fs = o; o = align16(o + kMaxTopK * 4);
  L.flag = o; o = align16(o + 16);
  L.cpre = o; o = align16(o + (n_chunks > 0 ? (n_chunks + 1) * 4 : 0));
  L.stg = o; o = align16(o + (n_chunks > 0 ? kWaves * kStgBytes : 0));
  L.gm = o; o = align16(o + kTopkScratch256);
  L.total = o;
  return L;
}

// ---------------------------------------------------------------------------
// device helpers
// ---------------------------------------------------------------------------

// Diagnostic build only (-DMR_STAMPS, libmr_engine_stamps.so): thread 0 of
// each scoring workgroup records s_memrealtime (100 MHz) at phase boundaries
// into a debug buffer; the production build compiles these away.
constexpr int kStampSlots = 32;  // [0,16): s_memrealtime, [16,32): s_memtime
__device__ __forceinline__ void stamp_at(long long* sb, int i) {
#ifdef MR_STAMPS
  if (sb && threadIdx.x == 0) {
    sb[i] = (long long)__builtin_amdgcn_s_memrealtime();
    sb[16 + i] = (long long)__builtin_amdgcn_s_memtime();
  }
#endif
}
// k_cooc_build's stamps: s_memrealtime only, 8 slots per workgroup
__device__ __forceinline__ void stamp_rt(long long* sb, int i) {
#ifdef MR_STAMPS
  if (sb && threadIdx.x == 0) sb[i] = (long long)__builtin_amdgcn_s_memrealtime();
#endif
}
// the same from lane 0 of every wave (one index row per wave)
__device__ __forceinline__ void stamp_rt_wave(long long* sb, int i) {
#ifdef MR_STAMPS
  if (sb && (threadIdx.x & 63) == 0) sb[i] = (long long)__builtin_amdgcn_s_memrealtime();
#endif
}
__device__ __forceinline__ void stamp_val(long long* sb, int i, long long v, bool wave = false) {
#ifdef MR_STAMPS
  if (sb && (wave ? (threadIdx.x & 63) == 0 : threadIdx.x == 0)) sb[i] = v;
#endif
}
#ifdef MR_STAMPS
#define MR_STAMP(i) stamp_at(p.stamps ? p.stamps + ((size_t)blockIdx.y * gridDim.x + blockIdx.x) * kStampSlots : nullptr, (i))
#else
#define MR_STAMP(i) do {} while (0)
#endif

// Inclusive wave prefix sum. DPP (no LDS round trip): row_shr 1/2/4/8 scan
// each row of 16 lanes (a source outside the row reads the 0 of `old`),
// row_bcast 15 / 31 add the rows below. MR_NO_DPP: the ds_bpermute chain.
__device__ __forceinline__ int wave_incl_scan(int x) {
#ifndef MR_NO_DPP
  x += __builtin_amdgcn_update_dpp(0, x, 0x111, 0xf, 0xf, false);  // row_shr:1
  x += __builtin_amdgcn_update_dpp(0, x, 0x112, 0xf, 0xf, false);  // row_shr:2
  x += __builtin_amdgcn_update_dpp(0, x, 0x114, 0xf, 0xf, false);  // row_shr:4
  x += __builtin_amdgcn_update_dpp(0, x, 0x118, 0xf, 0xf, false);  // row_shr:8
  x += __builtin_amdgcn_update_dpp(0, x, 0x142, 0xa, 0xf, false);  // row_bcast:15 -> rows 1, 3
  x += __builtin_amdgcn_update_dpp(0, x, 0x143, 0xc, 0xf, false);  // row_bcast:31 -> rows 2, 3
#else
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const int y = __shfl_up(x, d, 64);
    if (lane >= d) x += y;
  }
#endif
  return x;
}

// Lane `l`'s value to the whole wave through a scalar register (v_readlane:
// no LDS round trip, unlike __shfl's ds_bpermute). Every lane must be active.
__device__ __forceinline__ int wave_lane(int x, int l) { return __builtin_amdgcn_readlane(x, l); }

// Doubles as unsigned keys in the same order (negatives: bits inverted;
// others: sign bit set), so integer atomicMin / atomicMax give min / max.
__host__ __device__ inline unsigned long long ordered_key(double x) {
  unsigned long long b;
  memcpy(&b, &x, sizeof b);
  return (b >> 63) ? ~b : (b | (1ull << 63));
}
__host__ __device__ inline double ordered_value(unsigned long long k) {
  const unsigned long long b = (k >> 63) ? (k & ~(1ull << 63)) : ~k;
  double x;
  memcpy(&x, &b, sizeof x);
  return x;
}

// Block-wide exclusive scan of one int per thread (256 threads). `sbuf` holds kWaves ints.
__device__ __forceinline__ int block_excl_scan(int x, int* total, int* sbuf) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int incl = wave_incl_scan(x);
  if (lane == 63) sbuf[w] = incl;
  __syncthreads();
  int off = 0, tot = 0;
#pragma unroll
  for (int i = 0; i < kWaves; ++i) {
    int s = sbuf[i];
    off += (i < w) ? s : 0;
    tot += s;
  }
  __syncthreads();
  *total = tot;
  return off + incl - x;
}

// Total order of recommendation candidates: score (key) descending, song ascending.
__device__ __forceinline__ bool cand_before(long long ka, int sa, long long kb, int sb) {
  return ka > kb || (ka == kb && sa < sb);
}

// ---------------------------------------------------------------------------
// Top-k selection, all in registers + DPP (no LDS round trips on the chain).
// ---------------------------------------------------------------------------

// 32-bit wave reductions on DPP: row_shr 1/2/4/8 leave each row's result in
// its lane 15, row_bcast 15/31 carry the rows into lane 63, readlane
// broadcasts it (as an SGPR value) to the whole wave. Sources outside a row
// keep the lane's own value (idempotent ops only).
// One DPP reduction step as a single VALU op: x = op(x[src lane], x). Lanes
// whose source is outside the row/pattern are not written (bound_ctrl off),
// i.e. keep x: right for idempotent ops. The s_nop covers the VALU-write ->
// DPP-read hazard the compiler cannot see through inline asm.
#define MR_DPP(op, x, mod) asm volatile("s_nop 1\n\t" op " %0, %0, %0 " mod : "+v"(x))
#define MR_DPP_REDUCE(op, x)                                          \
  do {                                                                \
    MR_DPP(op, x, "row_shr:1 row_mask:0xf bank_mask:0xf");            \
    MR_DPP(op, x, "row_shr:2 row_mask:0xf bank_mask:0xf");            \
    MR_DPP(op, x, "row_shr:4 row_mask:0xf bank_mask:0xf");            \
    MR_DPP(op, x, "row_shr:8 row_mask:0xf bank_mask:0xf");            \
    MR_DPP(op, x, "row_bcast:15 row_mask:0xa bank_mask:0xf");         \
    MR_DPP(op, x, "row_bcast:31 row_mask:0xc bank_mask:0xf");         \
    asm volatile("s_nop 1" ::: "memory");                             \
  } while (0)

__device__ __forceinline__ int wave_max_i32(int x) {
  MR_DPP_REDUCE("v_max_i32_dpp", x);
  return __builtin_amdgcn_readlane(x, 63);
}
__device__ __forceinline__ unsigned wave_max_u32(unsigned x) {
  MR_DPP_REDUCE("v_max_u32_dpp", x);
  return (unsigned)__builtin_amdgcn_readlane((int)x, 63);
}
__device__ __forceinline__ int wave_min_i32(int x) {
  MR_DPP_REDUCE("v_min_i32_dpp", x);
  return __builtin_amdgcn_readlane(x, 63);
}

// Wave-wide best candidate in the (key desc, song asc) order, returned to
// every lane: max of the high key words; if one lane holds it (the common
// case) its low word and song are read with readlane, else max of the low
// words among the tied lanes, then (if still tied) min song among those.
// "No candidate" is (-1, INT_MAX): its high word -1 is below every valid one.
__device__ __forceinline__ void wave_argmax(long long& k, int& s) {
  const int hi = (int)(k >> 32);
  const unsigned lo = (unsigned)(k & 0xffffffffll);
  const int H = wave_max_i32(hi);
  unsigned long long m = __ballot(hi == H);
  unsigned Lo;
  if (__popcll(m) == 1) {
    const int l = __ffsll((long long)m) - 1;
    Lo = (unsigned)__builtin_amdgcn_readlane((int)lo, l);
    s = __builtin_amdgcn_readlane(s, l);
  } else {
    Lo = wave_max_u32(hi == H ? lo : 0u);
    m = __ballot(hi == H && lo == Lo);
    if (__popcll(m) == 1) {
      s = __builtin_amdgcn_readlane(s, __ffsll((long long)m) - 1);
    } else {
      s = wave_min_i32((hi == H && lo == Lo) ? s : INT_MAX);
    }
  }
  k = (long long)(((unsigned long long)(unsigned)H << 32) | Lo);
}

// Branch-free "take b if it comes first".
__device__ __forceinline__ void take_if_before(long long& ka, int& sa, long long kb, int sb) {
  const bool t = cand_before(kb, sb, ka, sa);
  ka = t ? kb : ka;
  sa = t ? sb : sa;
}

// (k, s) <- the better of itself and lane CTRL's (a DPP pattern whose sources
// all lie in the row: quad_perm, row_mirror, row_half_mirror).
template <int CTRL>
__device__ __forceinline__ void dpp_take(long long& k, int& s) {
  const unsigned lo = (unsigned)__builtin_amdgcn_update_dpp(0, (int)(unsigned)(unsigned long long)k, CTRL, 0xf, 0xf,
                                                            false);
  const int hi = __builtin_amdgcn_update_dpp(0, (int)(k >> 32), CTRL, 0xf, 0xf, false);
  const int os = __builtin_amdgcn_update_dpp(0, s, CTRL, 0xf, 0xf, false);
  take_if_before(k, s, (long long)(((unsigned long long)(unsigned)hi << 32) | lo), os);
}

// Best of each aligned group of GS lanes (GS <= 16), in every lane of the
// group: quad xor 1, quad xor 2, then the half-row and row mirrors pair the
// quads and the half-rows. DPP: no LDS round trip per step.
template <int GS>
__device__ __forceinline__ void group_best(long long& k, int& s) {
  static_assert(GS == 1 || GS == 2 || GS == 4 || GS == 8 || GS == 16, "group size");
  if constexpr (GS >= 2) dpp_take<0xB1>(k, s);   // quad_perm [1,0,3,2]
  if constexpr (GS >= 4) dpp_take<0x4E>(k, s);   // quad_perm [2,3,0,1]
  if constexpr (GS >= 8) dpp_take<0x141>(k, s);  // row_half_mirror
  if constexpr (GS >= 16) dpp_take<0x140>(k, s); // row_mirror
}

// Sort M register candidates of a lane descending (odd-even transposition).
template <int M>
__device__ __forceinline__ void lane_sort(long long (&rk)[M], int (&rs)[M]) {
#pragma unroll
  for (int round = 0; round < M; ++round) {
#pragma unroll
    for (int j = round & 1; j + 1 < M; j += 2) {
      const bool sw = cand_before(rk[j + 1], rs[j + 1], rk[j], rs[j]);
      const long long k0 = rk[j], k1 = rk[j + 1];
      const int s0 = rs[j], s1 = rs[j + 1];
      rk[j] = sw ? k1 : k0;
      rk[j + 1] = sw ? k0 : k1;
      rs[j] = sw ? s1 : s0;
      rs[j + 1] = sw ? s0 : s1;
    }
  }
}

// One wave's top-k from M register candidates per lane (any order; key < 0
// = none): sort each lane's M, then k rounds of "argmax of the lane heads,
// the winning lane shifts its list". Lane 0 writes out_k/out_s[0..k),
// missing slots (-1, -1).
template <int M, bool SORTED = false>
__device__ __forceinline__ void wave_topk_regs(long long (&rk)[M], int (&rs)[M], int k, long long* out_k,
                                               int* out_s) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int j = 0; j < M; ++j)
    if (rk[j] < 0) { rk[j] = kKeyNone; rs[j] = INT_MAX; }
  if (!SORTED) lane_sort<M>(rk, rs);  // SORTED: the lane's list is already in order
  int r = 0;
  for (; r < k; ++r) {
    long long bk = rk[0];
    int bs = rs[0];
    wave_argmax(bk, bs);
    if (bk < 0) break;  // wave-uniform
    if (lane == 0) { out_k[r] = bk; out_s[r] = bs; }
    const bool win = rk[0] == bk && rs[0] == bs;  // songs are unique: one winner
#pragma unroll
    for (int j = 0; j + 1 < M; ++j) {
      rk[j] = win ? rk[j + 1] : rk[j];
      rs[j] = win ? rs[j + 1] : rs[j];
    }
    rk[M - 1] = win ? kKeyNone : rk[M - 1];
    rs[M - 1] = win ? INT_MAX : rs[M - 1];
  }
  for (int i = r + lane; i < k; i += 64) { out_k[i] = kKeyNone; out_s[i] = -1; }
}

// Tournament over L <= 256 sorted lists (desc, (-1,-1)-padded) of length k
// in LDS, run by ONE wave: lane l owns lists l, l+64, l+128, l+192, keeps
// each head and the element after it in registers (the LDS read for the
// next-but-one is issued when a list advances and is needed one win later).
__device__ __forceinline__ void wave_merge_lists(int L, int k, const long long* lk, const int* ls,
                                                 long long* out_k, int* out_s) {
  const int lane = threadIdx.x & 63;
  int pos[4];
  long long hk[4], nk[4];
  int hs[4], ns[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int l = lane + 64 * j;
    pos[j] = 0;
    hk[j] = nk[j] = kKeyNone;
    hs[j] = ns[j] = INT_MAX;
    if (l < L) {
      hk[j] = lk[(size_t)l * k];
      hs[j] = ls[(size_t)l * k];
      if (k > 1) {
        nk[j] = lk[(size_t)l * k + 1];
        ns[j] = ls[(size_t)l * k + 1];
      }
    }
    if (hk[j] < 0) { hk[j] = kKeyNone; hs[j] = INT_MAX; }
    if (nk[j] < 0) { nk[j] = kKeyNone; ns[j] = INT_MAX; }
  }
  int r = 0;
  for (; r < k; ++r) {
    long long bk = hk[0];
    int bs = hs[0];
#pragma unroll
    for (int j = 1; j < 4; ++j) take_if_before(bk, bs, hk[j], hs[j]);
    wave_argmax(bk, bs);
    if (bk < 0) break;  // wave-uniform
    if (lane == 0) { out_k[r] = bk; out_s[r] = bs; }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if (hk[j] == bk && hs[j] == bs) {  // the owner advances this list
        hk[j] = nk[j];
        hs[j] = ns[j];
        ++pos[j];
        nk[j] = kKeyNone;
        ns[j] = INT_MAX;
        if (pos[j] + 1 < k) {
          const int l = lane + 64 * j;
          nk[j] = lk[(size_t)l * k + pos[j] + 1];
          ns[j] = ls[(size_t)l * k + pos[j] + 1];
          if (nk[j] < 0) { nk[j] = kKeyNone; ns[j] = INT_MAX; }
        }
      }
    }
  }
  for (int i = r + lane; i < k; i += 64) { out_k[i] = kKeyNone; out_s[i] = -1; }
}

// Block top-k of n <= 1024 candidates get(i) into out (LDS). n <= 256: one
// wave holds 4 per lane and selects alone; otherwise every wave selects from
// its 256 (i = w*64 + lane + 256 j), then wave 0 merges the 4 sorted lists.
// All threads call it; it ends with a barrier.
template <typename Get>
__device__ __forceinline__ void block_topk(int n, int k, Get get, long long* wk, int* ws, long long* out_k,
                                           int* out_s) {
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  long long rk[4];
  int rs[4];
  if (n <= 256) {
    if (w == 0) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        rk[j] = kKeyNone;
        rs[j] = INT_MAX;
        if (lane + 64 * j < n) get(lane + 64 * j, rk[j], rs[j]);
      }
      wave_topk_regs<4>(rk, rs, k, out_k, out_s);
    }
    __syncthreads();
    return;
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int i = w * 64 + lane + kThreads * j;
    rk[j] = kKeyNone;
    rs[j] = INT_MAX;
    if (i < n) get(i, rk[j], rs[j]);
  }
  wave_topk_regs<4>(rk, rs, k, wk + w * k, ws + w * k);
  __syncthreads();
  if (w == 0) wave_merge_lists(kWaves, k, wk, ws, out_k, out_s);
  __syncthreads();
}

// Insert (key, song) into a lane's descending register list of kMaxTopkLarge
// slots (first k used); thr tracks the k-th key (candidates at or below it
// cannot enter, except equal keys with a lower song id, which the caller
// excludes by visiting songs in ascending order per lane).
template <int KS>
__device__ __forceinline__ void lane_list_insert(long long (&tk)[KS], int (&ts)[KS], int k, long long key, int song,
                                                 long long& thr) {
  long long ck = key;
  int cs = song;
#pragma unroll
  for (int t = 0; t < KS; ++t) {
    const bool b = t < k && cand_before(ck, cs, tk[t], ts[t]);
    const long long ok = tk[t];
    const int os = ts[t];
    tk[t] = b ? ck : tk[t];
    ts[t] = b ? cs : ts[t];
    ck = b ? ok : ck;
    cs = b ? os : cs;
  }
  long long nt = kKeyNone;
#pragma unroll
  for (int t = 0; t < KS; ++t) nt = (t == k - 1) ? tk[t] : nt;
  thr = nt;
}

// Block top-k (k <= kMaxTopkLarge) of n candidates get(i), any n: every thread
// keeps a running list over i = tid + kThreads*j (ascending, so ties keep the
// lower song), the 256 lists go to LDS (lk/ls: kThreads*k slots, may alias
// the storage get() reads — a barrier separates them), each wave merges its
// 64 lists, wave 0 merges the kWaves results. Ends with a barrier.
template <typename Get>
__device__ __forceinline__ void block_topk_wide(int n, int k, Get get, long long* lk, int* ls, long long* wk,
                                                int* ws, long long* out_k, int* out_s) {
  const int tid = threadIdx.x, w = tid >> 6;
  long long tk[kMaxTopkLarge];
  int ts[kMaxTopkLarge];
#pragma unroll
  for (int t = 0; t < kMaxTopkLarge; ++t) { tk[t] = kKeyNone; ts[t] = INT_MAX; }
  long long thr = kKeyNone;
  for (int i = tid; i < n; i += kThreads) {
    long long key;
    int song;
    get(i, key, song);
    if (key > thr) lane_list_insert(tk, ts, k, key, song, thr);
  }
  __syncthreads();
#pragma unroll
  for (int t = 0; t < kMaxTopkLarge; ++t)
    if (t < k) { lk[tid * k + t] = tk[t]; ls[tid * k + t] = tk[t] >= 0 ? ts[t] : -1; }
  __syncthreads();
  wave_merge_lists(64, k, lk + (size_t)w * 64 * k, ls + (size_t)w * 64 * k, wk + w * k, ws + w * k);
  __syncthreads();
  if (w == 0) wave_merge_lists(kWaves, k, wk, ws, out_k, out_s);
  __syncthreads();
}

// Block top-k by threshold, for large n. Candidates are totally ordered by
// (key desc, song asc) (cand_before), so the k-th best of the NT/16 row bests
// (16-lane groups) is a lower bound tau on the k-th best entry (those k are k
// distinct entries): every top-k entry comes before or equal to tau. A second
// pass collects those entries (about k of them, ties included: the bound is a
// (key, song) pair) into ck/cs (cap <= 256 slots), and every candidate's rank
// among them (pairwise comparisons spread over the block) is its output slot.
// Each thread passes the best of its own keys (mk, ms) — get(i) for
// i = tid + NT j, which the caller has usually just produced. Scratch gm:
// topk_scratch_bytes(NT). Returns false, uniformly, when the candidates
// overflow cap or k > NT/16: the caller then runs the general per-thread-list
// path. All threads call it; it ends with a barrier. Every phase is spread
// over the whole block: no single-wave serial chain.
template <int NT, int NG = NT / 16>
__host__ __device__ constexpr int topk_scratch_bytes() {
  return (NG + 1) * 12 + 4 + NG * 4 + 256 * 4;
}
// The best (key desc, song asc) of a thread's keys get(i), i = tid + NT j.
static_assert(topk_scratch_bytes<256, 64>() == kTopkScratch256, "score_lds scratch size");
template <int NT, typename Get>
__device__ __forceinline__ void thread_best(int n, Get get, long long& mk, int& ms) {
  mk = kKeyNone;
  ms = INT_MAX;
#pragma unroll 4
  for (int i = threadIdx.x; i < n; i += NT) {
    long long key;
    int song;
    get(i, key, song);
    if (key >= 0) take_if_before(mk, ms, key, song);
  }
}
// A top-k list's global destination: key / song (and score = the key's
// double, NaN for none, when non-null), written by the thread that ranked the
// slot — sc1 stores for an in-launch hand-off — instead of through LDS; the
// caller orders the stores (no barrier after them). key == nullptr: LDS out.
struct TopkDst {
  long long* key = nullptr;
  int* song = nullptr;
  double* score = nullptr;
  bool sc1 = false;
};
__device__ __forceinline__ void topk_dst_write(const TopkDst& d, int slot, long long key, int song) {
  if (d.sc1) {
    __hip_atomic_store(d.key + slot, key, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(d.song + slot, song, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  } else {
    d.key[slot] = key;
    d.song[slot] = song;
  }
  if (d.score) d.score[slot] = key >= 0 ? __longlong_as_double(key) : (double)NAN;
}

// key / bs for shard-local songs (< 2^24) without an integer division: the
// fp32 quotient is within one of the truth, then corrected
#ifndef MR_LIGHT_CAS1
#define MR_LIGHT_CAS1 1
#endif
#ifndef MR_LIGHT_FDIV
#define MR_LIGHT_FDIV 1
#endif
__device__ __forceinline__ int tile_of(int key, int bs, float inv_bs) {
  if (!MR_LIGHT_FDIV) return key / bs;
  int t = (int)((float)key * inv_bs);
  t -= t * bs > key ? 1 : 0;
  t += (t + 1) * bs <= key ? 1 : 0;
  return t;
}

// Comparisons per thread past which rank_survivors hands its candidates to one
// wave (k rounds of a wave-wide best) instead of ranking them all at once. The
// fused shape's 256 threads rank up to 128 survivors themselves: a UserBasedModel
// tile with many equal scores at tau (C1) otherwise spent ~4 us in the one-wave
// select — C1 15.0 -> 10.5 us per step, C2 unchanged (profiles/r06/s47).
#ifndef MR_RANK_Q_FUSED
#define MR_RANK_Q_FUSED 64
#endif
#ifndef MR_RANK_Q_WIDE
#define MR_RANK_Q_WIDE 16
#endif
#ifndef MR_MERGE_INTERLEAVE
#define MR_MERGE_INTERLEAVE 1  // C2 9.84-9.88 vs 9.91-9.93 us per step, profiles/r06/s54
#endif
#ifndef MR_RANK_UNROLL_FUSED
#define MR_RANK_UNROLL_FUSED 4
#endif
template <int NT>
constexpr int kRankQ = NT <= 256 ? MR_RANK_Q_FUSED : MR_RANK_Q_WIDE;
template <int NT>
constexpr int kRankU = NT <= 256 ? MR_RANK_UNROLL_FUSED : 1;  // the wide kernels: one comparison at a time

// Ranks of nc <= 256 survivor candidates ck/cs among themselves (total order
// (key desc, song asc)): rank < k -> output slot; slots past nc get (-1, -1).
// crank: 256 zeroed ints. All threads call it; it ends with a barrier (not
// after the stores to a global dst).
template <int NT>
__device__ __forceinline__ void rank_survivors(int nc, int k, const long long* ck, const int* cs, int* crank,
                                               long long* out_k, int* out_s, const TopkDst& dst = TopkDst{}) {
  const int tid = threadIdx.x, lane = tid & 63;
  if (nc * nc > kRankQ<NT> * NT) {  // many ties at tau: one wave selects (4 candidates per lane)
    if (tid < 64) {
      long long rk[4];
      int rs[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int c = lane + 64 * j;
        rk[j] = c < nc ? ck[c] : kKeyNone;
        rs[j] = c < nc ? cs[c] : INT_MAX;
      }
      wave_topk_regs<4>(rk, rs, k, out_k, out_s);
    }
    __syncthreads();
    if (dst.key)
      for (int r = tid; r < k; r += NT) topk_dst_write(dst, r, out_k[r], out_s[r]);
    return;
  }
  if (nc > 0) {  // candidate ranks: nc x nc comparisons, <= 16 per thread
    const int sl = NT / nc;  // slices per candidate (nc <= 256 <= NT)
    const int per = (nc + sl - 1) / sl;
    if (tid < sl * nc) {
      const int i = tid % nc, j0 = (tid / nc) * per;
      const long long mine = ck[i];
      const int mines = cs[i];
      int c = 0;
      const int je = min(nc, j0 + per);
      int j = j0;
      // (a tie-heavy tile's slices run up to 64 comparisons: the fused shape
      // keeps the LDS reads of kRankU of them in flight instead of one round
      // trip each — C1 10.47 -> 9.65 us per step at 4, 10.14 at 8,
      // profiles/r06/s51)
      constexpr int U = kRankU<NT>;
      if constexpr (U > 1) {
        for (; j + U <= je; j += U) {
          long long o[U];
          int os[U];
#pragma unroll
          for (int r = 0; r < U; ++r) { o[r] = ck[j + r]; os[r] = cs[j + r]; }
#pragma unroll
          for (int r = 0; r < U; ++r) c += cand_before(o[r], os[r], mine, mines) ? 1 : 0;
        }
      }
      for (; j < je; ++j) c += cand_before(ck[j], cs[j], mine, mines) ? 1 : 0;
      if (c) atomicAdd(&crank[i], c);
    }
  }
  __syncthreads();
  if (dst.key) {
    if (tid < nc && crank[tid] < k) topk_dst_write(dst, crank[tid], ck[tid], cs[tid]);
    if (tid >= nc && tid < k) topk_dst_write(dst, tid, kKeyNone, -1);  // fewer than k entries
    return;
  }
  if (tid < nc && crank[tid] < k) { out_k[crank[tid]] = ck[tid]; out_s[crank[tid]] = cs[tid]; }
  if (tid >= nc && tid < k) { out_k[tid] = kKeyNone; out_s[tid] = -1; }  // fewer than k entries
  __syncthreads();
}


// The threshold of block_topk_threshold: every thread passes the best (mk,
// ms) of its own entries; returns, uniformly, tau = the k-th best of the NG
// row bests (k <= NG), or (0, INT_MAX) — "every valid key" — when fewer than
// k rows hold a valid entry. Zeroes the scratch's survivor counter and ranks
// (gm: topk_scratch_bytes(NT)); ends with a barrier.
template <int NT, int NG = NT / 16>
__device__ __forceinline__ void block_tau(int k, long long mk, int ms, unsigned char* gm, long long& tau_k,
                                          int& tau_s, long long* sb = nullptr) {
  constexpr int GS = NT / NG;  // threads per row
  static_assert(NT % 64 == 0 && NT % NG == 0 && NG <= 64 && GS <= 64 && NT * 16 >= NG * NG,
                "block shape");
  long long* gk = reinterpret_cast<long long*>(gm);    // [NG + 1]: row bests, then tau
  int* gs = reinterpret_cast<int*>(gk + NG + 1);       // [NG + 1]
  int* counter = gs + NG + 1;                          // [1]
  int* grank = counter + 1;                            // [NG]
  int* crank = grank + NG;                             // [256]
  const int tid = threadIdx.x, lane = tid & 63;
#ifndef MR_NO_DPP
  if constexpr (GS <= 16) {
    group_best<GS>(mk, ms);
  } else
#endif
  {
#pragma unroll
    for (int d = 1; d < GS; d <<= 1) {
      const long long ok = __shfl_xor(mk, d, 64);
      const int os = __shfl_xor(ms, d, 64);
      take_if_before(mk, ms, ok, os);
    }
  }
  if ((lane & (GS - 1)) == 0) { gk[tid / GS] = mk; gs[tid / GS] = ms; }
  if (tid < NG) grank[tid] = 0;
  if (tid == 0) *counter = 0;
  __syncthreads();
  stamp_at(sb, 9);
  {  // rank of every row best: NG x NG comparisons, NG / (NT / NG) per thread
    constexpr int SL = NT / NG, PER = (NG + SL - 1) / SL;
    const int i = tid % NG, j0 = (tid / NG) * PER;
    const long long mine = gk[i];
    const int mines = gs[i];
    int c = 0;
#pragma unroll
    for (int jj = 0; jj < PER; ++jj) {
      const int j = j0 + jj;
      if (j < NG) {
        const long long o = gk[j];
        const int os = gs[j];
        c += (cand_before(o, os, mine, mines) || (o == mine && os == mines && j < i)) ? 1 : 0;
      }
    }
    if (c) atomicAdd(&grank[i], c);
  }
  __syncthreads();
  if (tid < NG && grank[tid] == k - 1) { gk[NG] = gk[tid]; gs[NG] = gs[tid]; }  // exactly one row
  if (tid < 256) crank[tid] = 0;
  __syncthreads();
  stamp_at(sb, 10);
  tau_k = gk[NG];
  tau_s = gs[NG];
  if (tau_k < 0) { tau_k = 0; tau_s = INT_MAX; }  // fewer than k valid row bests: every valid key
}

// NG rows of NT / NG threads: more rows give a tighter tau (fewer survivors
// to rank) for NG^2 / NT comparisons per thread.
template <int NT, typename Get, int NG = NT / 16>
__device__ __forceinline__ bool block_topk_threshold(int n, int k, Get get, long long mk, int ms, unsigned char* gm,
                                                     long long* ck, int* cs, int cap, long long* out_k, int* out_s,
                                                     long long* sb = nullptr, const TopkDst& dst = TopkDst{}) {
  long long* gk = reinterpret_cast<long long*>(gm);
  int* gs = reinterpret_cast<int*>(gk + NG + 1);
  int* counter = gs + NG + 1;
  int* crank = counter + 1 + NG;
  const int tid = threadIdx.x;
  if (k > NG || k <= 0 || cap > 256) return false;
  long long tk;
  int tsg;
  block_tau<NT, NG>(k, mk, ms, gm, tk, tsg, sb);
  // (Compacting survivors per wave by ballot, one atomic per wave, measured
  // slower: C2 14.30 vs 14.11 us per step, profiles/r02/c2_topk_ab.txt.)
#pragma unroll 4
  for (int i = tid; i < n; i += NT) {
    long long key;
    int song;
    get(i, key, song);
    if (key >= 0 && !cand_before(tk, tsg, key, song)) {
      const int pos = atomicAdd(counter, 1);
      if (pos < cap) { ck[pos] = key; cs[pos] = song; }
    }
  }
  __syncthreads();
  stamp_at(sb, 11);
  const int nc = *counter;
  if (nc > cap) return false;
  rank_survivors<NT>(nc, k, ck, cs, crank, out_k, out_s, dst);
  return true;
}

constexpr int kMergeStageBytes = 32 * 1024;  // LDS staging of tile lists per merge pass
__host__ __device__ inline int merge_lists_per_pass(int k) {
  const int kk = k > 0 ? k : 1;
  int l = kMergeStageBytes / (12 * kk);
  return l > 256 ? 256 : (l < 2 ? 2 : l);
}

// Wave-private LDS hand-off: wait for this wave's LDS ops, keep the compiler
// from reordering across it (a single wave needs no s_barrier).
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// sc1 (L2-coherent, agent-scope) stores/loads for the in-launch hand-off of
// tile candidates to the user's last workgroup (MI355X_MICROARCH.md, "Valid
// forms", row 1: sc1 stores, vmcnt(0), barrier, one agent atomic add per
// workgroup; the last adder loads with sc1 loads).
template <typename T>
__device__ __forceinline__ void st_sc1(T* p, T v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
template <typename T>
__device__ __forceinline__ T ld_sc1(const T* p) {
  return __hip_atomic_load(const_cast<T*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// ---------------------------------------------------------------------------
// stage 1, separate shape: one workgroup per test user, dense LDS array over
// the train users, compacted (v, weight) lists to global. MR:140-149 / MR:230-239.
// ---------------------------------------------------------------------------
struct NbrParams {
  int n_tr;
  int user0;                 // first test user of this launch
  int cap;                   // neighbour-list capacity per user (= n_chunks * chunk)
  int frac_bits;
  int chunk, n_chunks;       // train users per stage-1 chunk (blockIdx.x), chunks per user
  const long long* te_off;   // [n_te+1]
  const int* te_songs;
  const long long* trs_off;  // song -> train users CSR [n_s+1]
  const int* trs_users;
  const long long* q_song;   // ibm: rint(2^F / sqrt c(s))
  const double* sqrt_tr;     // sqrt(|S(v)|) with duplicates (MR:147)
  const double* sqrt_te;     // sqrt(|T(u)|) with duplicates
  int* nbr_v;                // [batch][cap]: chunk c's list at c * chunk
  long long* nbr_q;          // [batch][cap]
  int* nbr_cnt;              // [batch][n_chunks]
  const int* sbound;         // [n_s][n_chunks+1]: first trs_users index of each chunk (n_chunks > 1)
};

// First index in the sorted trs_users[lo, hi) whose user is >= v.
__device__ __forceinline__ long long lower_bound_user(const int* trs_users, long long lo, long long hi, int v) {
  while (lo < hi) {
    const long long m = (lo + hi) >> 1;
    if (trs_users[m] < v) lo = m + 1; else hi = m;
  }
  return lo;
}

// Accumulate Y[v] += w(s2) over v ∈ L_tr(s2), s2 ∈ T(u): a flattened walk over
// the listener lists of T(u), 256 songs of T(u) at a time; add(v, w) performs
// the (integer, order-independent) accumulation. mark(s2) is called once per
// song of T(u) (heard-song bookkeeping). ranged: only listeners v in [v0, v1)
// (a stage-1 chunk; the sorted lists are cut by binary search).
template <int MODEL, typename Add, typename Mark>
__device__ __forceinline__ void walk_neighbours(long long t0, long long t1, const int* te_songs,
                                                const long long* trs_off, const int* trs_users,
                                                const long long* q_song, long long* s_lo, long long* s_w,
                                                int* s_pre, int* s_scan, Add add, Mark mark, bool ranged = false,
                                                int v0 = 0, int v1 = 0, const int* sbound = nullptr,
                                                int chunk_idx = 0, int nc1 = 0, const int2* te_rng = nullptr,
                                                const long long* te_q = nullptr, long long* sb = nullptr) {
  const int tid = threadIdx.x;
  for (long long base = t0; base < t1; base += kThreads) {
    const int n = (int)min((long long)kThreads, t1 - base);
    int len = 0;
    if (tid < n && te_rng && !ranged) {
      // listener range and weight of each song of T(u) resolved at load time
      // (mr_load: the songsToUsersMap lookup of MR:232 per test-visible song):
      // loaded beside te_songs, one dependent level fewer
      const int s2 = te_songs[base + tid];
      const int2 r = te_rng[base + tid];
      len = r.y;
      s_lo[tid] = r.x;
      s_w[tid] = (MODEL == MR_IBM) ? te_q[base + tid] : 1ll;
      mark(s2);
    } else if (tid < n) {
      const int s2 = te_songs[base + tid];
      long long lo = trs_off[s2], hi = trs_off[s2 + 1];
      if (ranged && sbound) {  // precomputed chunk boundaries of L_tr(s2) (mr_load)
        const int* b = sbound + (size_t)s2 * nc1 + chunk_idx;
        lo = b[0];
        hi = b[1];
      } else if (ranged) {
        lo = lower_bound_user(trs_users, lo, hi, v0);
        hi = lower_bound_user(trs_users, lo, hi, v1);
      }
      len = (int)(hi - lo);
      s_lo[tid] = lo;
      s_w[tid] = (MODEL == MR_IBM) ? q_song[s2] : 1ll;
      mark(s2);
    }
    int total;
    const int pre = block_excl_scan(len, &total, s_scan);
    s_pre[tid] = pre;
    if (tid == 0) s_pre[kThreads] = total;
    __syncthreads();
    stamp_at(sb, 10);  // (diagnostic build) the batch's songs resolved and scanned
    // 16 flattened entries per thread in flight: the listener loads of one
    // batch are issued together, then their accumulations.
    // Segment search (j with s_pre[j] <= i < s_pre[j+1]): groups of 4
    // entries advance in lockstep for ceil(log2 n) halvings (their LDS reads
    // overlap); groups past the block's last entry are skipped uniformly.
    // (A per-entry loop serialised entries x log2 n dependent LDS reads: 7.3 us
    // of stage 1 for C2's heaviest user; 16-wide lockstep with fixed 8 steps
    // cost more than it saved.)
    const int nsteps = n > 1 ? 32 - __clz(n - 1) : 0;
    for (int i0 = tid; i0 < total; i0 += 16 * kThreads) {
      const int ib = i0 - tid;  // block-uniform
      int v[16];
      unsigned long long wv[16];
#pragma unroll
      for (int r = 0; r < 16; ++r) { v[r] = -1; wv[r] = 0ull; }
#pragma unroll
      for (int g2 = 0; g2 < 4; g2 += 2) {  // two groups of 4 at a time
        if (ib + g2 * 4 * kThreads >= total) break;
        if (ib + (g2 + 1) * 4 * kThreads < total) {
          // both groups hold entries (heavy users): 8 searches in lockstep, so
          // the second group's LDS reads overlap the first's (C2's heaviest
          // user: stage 1 4.9 -> 4.5 us)
          int a[8], b[8];
#pragma unroll
          for (int e = 0; e < 8; ++e) { a[e] = 0; b[e] = n; }
          for (int st = 0; st < nsteps; ++st) {
#pragma unroll
            for (int e = 0; e < 8; ++e) {
              const int i = i0 + (g2 * 4 + e) * kThreads;
              const int m = (a[e] + b[e]) >> 1;
              if (s_pre[m] <= i) a[e] = m; else b[e] = m;
            }
          }
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const int i = i0 + (g2 * 4 + e) * kThreads;
            if (i < total) {
              v[g2 * 4 + e] = trs_users[s_lo[a[e]] + (i - s_pre[a[e]])];
              wv[g2 * 4 + e] = (unsigned long long)s_w[a[e]];
            }
          }
          continue;
        }
        const int g = g2;  // one group of 4
        int a[4], b[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) { a[e] = 0; b[e] = n; }
        for (int st = 0; st < nsteps; ++st) {
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int i = i0 + (g * 4 + e) * kThreads;
            const int m = (a[e] + b[e]) >> 1;
            if (s_pre[m] <= i) a[e] = m; else b[e] = m;  // size 1: m = a, stays
          }
        }
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int i = i0 + (g * 4 + e) * kThreads;
          if (i < total) {
            v[g * 4 + e] = trs_users[s_lo[a[e]] + (i - s_pre[a[e]])];
            wv[g * 4 + e] = (unsigned long long)s_w[a[e]];
          }
        }
      }
#pragma unroll
      for (int r = 0; r < 16; ++r)
        if (v[r] >= 0) add(v[r], wv[r]);
    }
    stamp_at(sb, 11);  // (diagnostic build) thread 0's searches, listener loads and adds issued
    __syncthreads();
  }
}

// Y indexed by v - v0 (v0 = 0 unless ranged).
template <int MODEL>
__device__ __forceinline__ void accumulate_neighbours(unsigned long long* Y, long long t0, long long t1,
                                                      const int* te_songs, const long long* trs_off,
                                                      const int* trs_users, const long long* q_song,
                                                      long long* s_lo, long long* s_w, int* s_pre, int* s_scan,
                                                      unsigned* heard, int blo, int bhi, bool ranged = false,
                                                      int v0 = 0, int v1 = 0, const int* sbound = nullptr,
                                                      int chunk_idx = 0, int nc1 = 0, const int2* te_rng = nullptr,
                                                      const long long* te_q = nullptr, long long* sb = nullptr) {
  walk_neighbours<MODEL>(
      t0, t1, te_songs, trs_off, trs_users, q_song, s_lo, s_w, s_pre, s_scan,
      [&](int v, unsigned long long w) { atomicAdd(&Y[v - v0], w); },
      [&](int s2) {
        if (heard && s2 >= blo && s2 < bhi) atomicOr(&heard[(s2 - blo) >> 5], 1u << ((s2 - blo) & 31));
      },
      ranged, v0, v1, sbound, chunk_idx, nc1, te_rng, te_q, sb);
}

// Neighbour weight from the stage-1 sum: ibm uses it as is; ubm turns the
// distinct-overlap count into the fixed-point cosine (MR:142-148).
template <int MODEL>
__device__ __forceinline__ long long neighbour_weight(unsigned long long y, double rs_u, double sqrt_tr_v,
                                                      double two_f) {
  if (MODEL == MR_IBM) return (long long)y;
  const double c = (double)(long long)y / (rs_u * sqrt_tr_v);
  return (long long)rint(c * two_f);
}

template <int MODEL>
__global__ __launch_bounds__(kThreads) void k_neighbours(NbrParams p) {
  extern __shared__ __align__(16) unsigned char smem_raw[];
  unsigned long long* Y = reinterpret_cast<unsigned long long*>(smem_raw);         // [n_tr]
  long long* s_lo = reinterpret_cast<long long*>(smem_raw + align16(p.chunk * 8));  // [256]
  long long* s_w = s_lo + kThreads;                                                // [256]
  int* s_pre = reinterpret_cast<int*>(s_w + kThreads);                             // [257]
  int* s_scan = s_pre + kThreads + 4;                                              // [kWaves]

  const int c = blockIdx.x;
  const int bu = blockIdx.y;
  const int u = p.user0 + bu;
  const int tid = threadIdx.x;
  const int cv0 = c * p.chunk, cv1 = min(p.n_tr, cv0 + p.chunk), cw = cv1 - cv0;
  for (int i = tid; i < cw; i += kThreads) Y[i] = 0ull;
  __syncthreads();
  accumulate_neighbours<MODEL>(Y, p.te_off[u], p.te_off[u + 1], p.te_songs, p.trs_off, p.trs_users, p.q_song,
                               s_lo, s_w, s_pre, s_scan, nullptr, 0, 0, p.n_chunks > 1, cv0, cv1, p.sbound, c,
                               p.n_chunks + 1);

  // Compaction, order kept: wave w owns the contiguous quarter [w*q, (w+1)*q)
  // of the chunk, counts its non-zeros by ballot (rows of 64, conflict-free
  // LDS reads), one scan of the 4 wave totals, then writes by ballot rank.
  const double two_f = ldexp(1.0, p.frac_bits);
  const double rs_u = p.sqrt_te[u];
  int* out_v = p.nbr_v + (size_t)bu * p.cap + (size_t)c * p.chunk;
  long long* out_q = p.nbr_q + (size_t)bu * p.cap + (size_t)c * p.chunk;
  const int lane = tid & 63, w = tid >> 6;
  const int q4 = (cw + kWaves * 64 - 1) / (kWaves * 64) * 64;  // per-wave span, multiple of 64
  const int wb = min(cw, w * q4), we = min(cw, wb + q4);
  int nz = 0;
  for (int i0 = wb; i0 < we; i0 += 64) {
    const int i = i0 + lane;
    nz += __popcll(__ballot(i < we && Y[i] != 0ull));
  }
  if (lane == 0) s_scan[w] = nz;
  __syncthreads();
  int base = 0, written = 0;
#pragma unroll
  for (int x = 0; x < kWaves; ++x) {
    base += x < w ? s_scan[x] : 0;
    written += s_scan[x];
  }
  const unsigned long long below = lane ? (~0ull >> (64 - lane)) : 0ull;
  for (int i0 = wb; i0 < we; i0 += 64) {
    const int i = i0 + lane;
    const unsigned long long y = i < we ? Y[i] : 0ull;
    const unsigned long long m = __ballot(y != 0ull);
    if (y != 0ull) {
      const int pos = base + __popcll(m & below);
      const int v = cv0 + i;
      out_v[pos] = v;
      out_q[pos] = neighbour_weight<MODEL>(y, rs_u, MODEL == MR_UBM ? p.sqrt_tr[v] : 0.0, two_f);
    }
    base += __popcll(m);
  }
  if (tid == 0) p.nbr_cnt[(size_t)bu * p.n_chunks + c] = written;
}

// ---------------------------------------------------------------------------
// stage 2 (+ fused stage 1, + stage 3): one workgroup per (song tile, test
// user). MR:159-166 (ubm rank), MR:249-257 (ibm rank), MR:105-111 (pairs).
// ---------------------------------------------------------------------------
#ifndef MR_FUSED_SCHED
#define MR_FUSED_SCHED 1  // fused stage 1 from mr_load's walk schedule (0: the per-step segment search)
#endif
#ifndef MR_SCHED_SE
#define MR_SCHED_SE 8     // fused stage 1: schedule entries per thread per batch (C2 per step: 4 9.92-10.00,
                          // 6 10.26-10.33, 8 9.93-9.95, 12 10.27-10.30, 16 10.99-11.02 us; profiles/r06/s33-s34)
#endif
#ifndef MR_COUNTER_STRIDE
#define MR_COUNTER_STRIDE 64  // words between two users' hand-off counters: one 256-B line each.
                              // Every tile's agent-scope add on its user's counter is a memory-side
                              // atomic; packed (1), the 220 adds of a C2 step hit one line and
                              // serialise: 12.20-12.23 vs 11.95-11.99 us per step (profiles/r06/s29-s30)
#endif
constexpr int kCounterStride = MR_COUNTER_STRIDE;
struct ScoreParams {
  int n_tr;
  int user0;
  int song_lo, song_hi, width;   // shard [lo, hi), width = hi - lo
  int block_songs, n_tiles;
  int frac_bits, topk, dense;
  const long long* te_off;
  const int* te_songs;
  const int* toff;               // tile-major train CSR: [n_tiles * n_tr + 1]; tile t, user v ->
                                 //   tsongs[toff[t*n_tr+v] .. toff[t*n_tr+v+1])
  const unsigned short* tsongs;  // tile-local song ids (s - tile start), rows sorted
  const unsigned* tpack;         // fused shape: the same entries as (train user << 16) | tile-local song
  const int2* te_rng;            // fused shape: per te_songs entry, (trs_off[s2], c_tr(s2))
  const long long* te_q;         // fused shape: per te_songs entry, q_song[s2]
  // fused shape: stage 1's walk schedule (mr_load) — per test user, one entry
  // per (song of T(u), listener) in song order: (trs_users index, song's slot
  // in T(u)); sched_off[u] .. sched_off[u + 1]. Null: the in-kernel search.
  const uint2* te_sched;
  const long long* sched_off;
  const double* sqrt_c;          // sqrt(c(s)) (train+test, dups), MR:237
  // fused stage 1 inputs
  const long long* trs_off;
  const int* trs_users;
  const long long* q_song;
  const double* sqrt_tr;
  const double* sqrt_te;
  // separate stage 1 outputs
  int cap;
  int chunk, n_chunks;           // per-chunk neighbour lists (k_neighbours)
  int n_users, xcd_remap;        // users of this launch; 1 = all tiles of a user on one XCD
  int merge_rows;                // threshold rows of the in-launch merge (16 / 32 / 64; MR_MERGE_ROWS)
  const int* nbr_v;
  const long long* nbr_q;
  const int* nbr_cnt;
  // outputs
  void* dense_out;               // [n_te][width] float or double
  long long* cand_key;           // [n_te][n_tiles][k] tile candidates
  int* cand_song;
  unsigned* counter;             // [n_te] tiles finished (reset by the last tile)
  long long* top_key;            // [n_te][k]
  int* top_song;
  double* top_score;
  long long* stamps;             // diagnostic build: [grid][8] phase timestamps
  int topk_lists;                // 1: skip the threshold top-k (mr_options.topk_lists)
  // co-listening route (wide shape, ibm; k_cooc_build's index)
  int n_rows, nseg;              // index rows; segment descriptors per LDS pass
  const int* te_row;             // per te_songs entry: its index row, -1 = no train listener
  const long long* seg_off;      // [tile][row]: first pool entry of the row's tile segment
  const int* seg_len;            // [tile][row]: its entries
  const unsigned* pool;          // entries (tile-local song << kCoocCntBits) | C[s2][s]
  // wide shape, dense output: ordered keys of each user's min / max stored
  // score ([user] min, [mm_n + user] max; mr_dense_minmax), or null
  unsigned long long* mm_key;
  int mm_n;
  // wide shape, top-k-only runs: the candidate-only tile top-k
  // (wide_cand_topk) over fp32 approximations with 1/sqrt(c(s)) as fp32
  int cand;
  const float* rsq_c;
};

template <int MODEL, typename OutT, bool FUSED>
__global__ __launch_bounds__(kThreads) void k_score(ScoreParams p) {
  extern __shared__ __align__(16) unsigned char smem_raw[];
  const int bs = p.block_songs;
  const ScoreLds L = score_lds(bs, FUSED ? p.n_tr : 0, p.topk, p.n_tiles, FUSED ? 0 : p.n_chunks);
  unsigned long long* acc = reinterpret_cast<unsigned long long*>(smem_raw + L.acc);
  unsigned* heard = reinterpret_cast<unsigned*>(smem_raw + L.heard);
  long long* wk = reinterpret_cast<long long*>(smem_raw + L.wk);
  int* ws = reinterpret_cast<int*>(smem_raw + L.ws);
  long long* fk = reinterpret_cast<long long*>(smem_raw + L.fk);
  int* fs = reinterpret_cast<int*>(smem_raw + L.fs);
  int* flag = reinterpret_cast<int*>(smem_raw + L.flag);

  int tile = blockIdx.x;
  int bu = blockIdx.y;
  if (p.xcd_remap) {
    // Blocks are dealt round-robin over the 8 XCDs (MI355X_MICROARCH.md, speed
    // only): give XCD x the users bu = 8j + x, all their tiles back to back,
    // so a user's neighbour rows are fetched into one L2 and re-read there.
    const int lin = blockIdx.y * gridDim.x + blockIdx.x;
    const int slot = lin >> 3;
    bu = (slot / p.n_tiles) * 8 + (lin & 7);
    tile = slot % p.n_tiles;
    if (bu >= p.n_users) return;  // grid padded to a multiple of 8 users
  }
  const int u = p.user0 + bu;
  const int tid = threadIdx.x;
  const int blo = p.song_lo + tile * bs;
  const int bhi = min(p.song_hi, blo + bs);
  const int bw = bhi - blo;
  const double two_f = ldexp(1.0, p.frac_bits);
#ifdef MR_STAMPS
  long long* sb = p.stamps ? p.stamps + ((size_t)blockIdx.y * gridDim.x + blockIdx.x) * kStampSlots : nullptr;
#endif
  MR_STAMP(0);

  for (int i = tid; i < bw; i += kThreads) acc[i] = 0ull;
  for (int i = tid; i < bs / 32; i += kThreads) heard[i] = 0u;
  const long long t0 = p.te_off[u], t1 = p.te_off[u + 1];
  // Fused stage 1 from the walk schedule: its first loads (this thread's
  // first song of T(u) for the heard bitmap, its first kSE schedule entries)
  // are issued before every prefetch below — the vector-memory counter
  // retires loads in issue order, so waiting on them then does not wait on
  // the prefetches issued after them. (Unconditional loads at clamped
  // indices, validity re-derived from the index at use: a predicated load
  // compiles to a branch with a full wait.)
  const bool sched = FUSED && p.te_sched != nullptr;
  constexpr int kSE = MR_SCHED_SE;  // schedule entries per thread in flight
  long long se0 = 0, se1 = 0;
  int hs0 = -1;
  uint2 sc1[kSE];
  if (sched) {
    se0 = p.sched_off[u];
    se1 = p.sched_off[u + 1];
    if (t1 > t0) hs0 = p.te_songs[min(t0 + tid, t1 - 1)];  // (block-uniform guards: an empty user reads nothing)
    if (se1 > se0) {
#pragma unroll
      for (int r = 0; r < kSE; ++r) sc1[r] = p.te_sched[min(se0 + tid + (long long)r * kThreads, se1 - 1)];
    }
  }
  // Prefetch this thread's epilogue scales (hidden behind stages 1-2): songs
  // tid + 256 j of the tile, j < kFusedPre (the whole tile up to 1024 songs).
  double sc[kFusedPre];
#pragma unroll
  for (int j = 0; j < kFusedPre; ++j) {
    const int i = tid + j * kThreads;
    sc[j] = (MODEL == MR_IBM && i < bw) ? p.sqrt_c[blo + i] : 1.0;
  }

  if (FUSED) {
    // Stage 2's inputs do not depend on the test user: the tile's entries
    // (train user, song) are one contiguous run of tpack (tile-major CSR), so
    // they are loaded now, coalesced, 4 per thread, and land while stage 1
    // runs; stage 2 is then LDS work only (Y[v] lookups + atomics), balanced
    // over the block whatever the segment lengths. (The per-neighbour segment
    // walk it replaces waited on up to 3 dependent load batches for heavy
    // listeners: 3.0 us median, 4.3 us max per C2 tile.)
    const int e0 = p.toff[(size_t)tile * p.n_tr], e1 = p.toff[(size_t)(tile + 1) * p.n_tr];
    unsigned pk[kFusedPre];
#pragma unroll
    for (int j = 0; j < kFusedPre; ++j) {
      const int i = e0 + tid + j * kThreads;
      pk[j] = i < e1 ? p.tpack[i] : 0xffffffffu;
    }
    double str[kFusedPre];  // ubm: sqrt|S(v)| of this thread's first train users
#pragma unroll
    for (int r = 0; r < kFusedPre; ++r) {
      const int v = tid + r * kThreads;
      str[r] = (MODEL == MR_UBM && v < p.n_tr) ? p.sqrt_tr[v] : 1.0;
    }
    unsigned long long* Y = reinterpret_cast<unsigned long long*>(smem_raw + L.y);
    int v[kSE];
    unsigned long long wv[kSE];
    auto gather = [&]() {  // (clamped entries are real ones: loads always in bounds)
#pragma unroll
      for (int r = 0; r < kSE; ++r) {
        v[r] = p.trs_users[sc1[r].x];
        wv[r] = (MODEL == MR_IBM) ? (unsigned long long)p.te_q[t0 + sc1[r].y] : 1ull;
      }
    };
    const bool any = sched && se1 > se0;  // (block-uniform: a user without entries gathers nothing)
    for (int i = tid; i < p.n_tr; i += kThreads) Y[i] = 0ull;
    __syncthreads();
    if (sched) {
      // Stage 1 from the walk schedule: every (song of T(u), listener) entry
      // names its trs_users index and its song's slot in T(u), so the entries
      // are loaded coalesced (the first kSE per thread above), with no
      // per-step prefix scan, barrier or segment search before the listener
      // gather; the gather (trs_users) and the Y adds are this step's work.
      if (any) gather();  // (issued before the zeroing barrier instead: slower, profiles/r06/s33)
      // the tile's heard songs, after the first gather is issued (their
      // wait then covers loads the adds need next anyway)
      auto mark = [&](int s2) {
        if (s2 >= blo && s2 < bhi) atomicOr(&heard[(s2 - blo) >> 5], 1u << ((s2 - blo) & 31));
      };
      if (t0 + tid < t1) mark(hs0);
      for (long long i = t0 + tid + kThreads; i < t1; i += kThreads) mark(p.te_songs[i]);  // |T(u)| > 256
#ifdef MR_STAMPS
      stamp_at(sb, 10);
#endif
      for (long long i0 = se0 + tid; any;) {
#pragma unroll
        for (int r = 0; r < kSE; ++r)
          if (i0 + (long long)r * kThreads < se1) atomicAdd(&Y[v[r]], wv[r]);
        i0 += (long long)kSE * kThreads;
        if (i0 >= se1) break;  // (users with more than kSE x 256 entries: the next batch)
#pragma unroll
        for (int r = 0; r < kSE; ++r) sc1[r] = p.te_sched[min(i0 + (long long)r * kThreads, se1 - 1)];
        gather();
      }
#ifdef MR_STAMPS
      stamp_at(sb, 11);
#endif
      __syncthreads();
    } else
    accumulate_neighbours<MODEL>(Y, t0, t1, p.te_songs, p.trs_off, p.trs_users, p.q_song,
                                 reinterpret_cast<long long*>(smem_raw + L.s_lo),
                                 reinterpret_cast<long long*>(smem_raw + L.s_w),
                                 reinterpret_cast<int*>(smem_raw + L.s_pre),
                                 reinterpret_cast<int*>(smem_raw + L.s_scan), heard, blo, bhi, false, 0, 0,
                                 nullptr, 0, 0, p.te_rng, p.te_q,
#ifdef MR_STAMPS
                                 sb
#else
                                 nullptr
#endif
    );
    MR_STAMP(1);
    if (MODEL == MR_UBM) {  // overlap counts -> fixed-point cosines (MR:142-148), in place
      const double rs_u = p.sqrt_te[u];
      for (int v = tid, r = 0; v < p.n_tr; v += kThreads, ++r) {
        const unsigned long long y = Y[v];
        if (y != 0ull) {
          double sv;
          if (r < kFusedPre) {  // static register index: no scratch spill
            sv = str[0];
#pragma unroll
            for (int x = 1; x < kFusedPre; ++x) sv = r == x ? str[x] : sv;
          } else {
            sv = p.sqrt_tr[v];
          }
          Y[v] = (unsigned long long)neighbour_weight<MODEL>(y, rs_u, sv, two_f);
        }
      }
      __syncthreads();
    }
#pragma unroll
    for (int j = 0; j < kFusedPre; ++j) {
      if (pk[j] == 0xffffffffu) continue;
      const unsigned long long y = Y[pk[j] >> 16];
      if (y != 0ull) atomicAdd(&acc[pk[j] & 0xffffu], y);
    }
    for (int i = e0 + tid + kFusedPre * kThreads; i < e1; i += kThreads) {  // tiles of > 1024 entries
      const unsigned e = p.tpack[i];
      const unsigned long long y = Y[e >> 16];
      if (y != 0ull) atomicAdd(&acc[e & 0xffffu], y);
    }
  } else {
    __syncthreads();
    for (long long i = t0 + tid; i < t1; i += kThreads) {
      const int s = p.te_songs[i];
      if (s >= blo && s < bhi) atomicOr(&heard[(s - blo) >> 5], 1u << ((s - blo) & 31));
    }
    // Prefix of the per-chunk neighbour counts: entry k of the user's
    // flattened list lives in chunk c with cpre[c] <= k < cpre[c+1].
    int* cpre = reinterpret_cast<int*>(smem_raw + L.cpre);
    int* s_scan = reinterpret_cast<int*>(smem_raw + L.s_scan);
    const int nch = p.n_chunks;
    int cnt = 0;
    for (int c0 = 0; c0 < nch; c0 += kThreads) {
      const int cc = c0 + tid;
      const int x = cc < nch ? p.nbr_cnt[(size_t)bu * nch + cc] : 0;
      int tot;
      const int pre = block_excl_scan(x, &tot, s_scan);
      if (cc < nch) cpre[cc] = cnt + pre;
      cnt += tot;
    }
    if (tid == 0) cpre[nch] = cnt;
    __syncthreads();
    MR_STAMP(1);
    const int* nv = p.nbr_v + (size_t)bu * p.cap;
    const long long* nq = p.nbr_q + (size_t)bu * p.cap;
    // Load-balanced scatter: each wave takes rounds of kStgItems neighbours
    // (R per lane), stages their tile segments (start, length prefix, weight)
    // in LDS, then its lanes walk the round's flattened entries, E per lane in
    // flight — segment lengths are heavy-tailed (heavy listeners dominate
    // N(u)), so per-lane segment loops would leave the wave waiting on its
    // longest segment.
    const int lane = tid & 63, w = tid >> 6;
    unsigned char* stg = smem_raw + L.stg + w * kStgBytes;
    unsigned long long* st_q = reinterpret_cast<unsigned long long*>(stg);
    int* st_a = reinterpret_cast<int*>(stg + kStgItems * 8);
    int* st_pre = st_a + kStgItems;
    constexpr int R = kStgItems / 64;
    constexpr int E = 16;
    const int* toff_t = p.toff + (size_t)tile * p.n_tr;
    // Software pipeline over rounds (one wave): round i is scattered while the
    // row offsets of round i+1 and the list entries of round i+2 are in
    // flight, so one memory latency covers three dependent levels.
    int cur = 0;  // this lane's chunk (its items ascend)
    auto load_list = [&](int k0, int (&v)[R], unsigned long long (&q)[R]) {
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const int k = k0 + r * 64 + lane;
        v[r] = -1;
        q[r] = 0ull;
        if (k < cnt) {
          while (cur + 1 < nch && cpre[cur + 1] <= k) ++cur;
          const size_t idx = (size_t)cur * p.chunk + (k - cpre[cur]);
          v[r] = nv[idx];
          q[r] = (unsigned long long)nq[idx];
        }
      }
    };
    auto load_offsets = [&](const int (&v)[R], int (&a)[R], int (&b)[R]) {
#pragma unroll
      for (int r = 0; r < R; ++r) {
        a[r] = b[r] = 0;
        if (v[r] >= 0) {
          a[r] = toff_t[v[r]];
          b[r] = toff_t[v[r] + 1];
        }
      }
    };
    const int step = kWaves * kStgItems;
    int v0[R], a0[R], b0[R], v1[R], a1[R], b1[R], v2[R];
    unsigned long long q0[R], q1[R], q2[R];
    int k0 = w * kStgItems;
    load_list(k0, v0, q0);
    load_offsets(v0, a0, b0);
    load_list(k0 + step, v1, q1);
    for (; k0 < cnt; k0 += step) {
      int run = 0;
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const int len = b0[r] - a0[r];
        const int incl = wave_incl_scan(len);
        const int it = r * 64 + lane;
        st_a[it] = a0[r];
        st_pre[it] = run + incl - len;
        st_q[it] = q0[r];
        run += __shfl(incl, 63, 64);
      }
      if (lane == 0) st_pre[kStgItems] = run;
      wave_lds_sync();
      load_offsets(v1, a1, b1);            // round i+1
      load_list(k0 + 2 * step, v2, q2);    // round i+2
      for (int j0 = 0; j0 < run; j0 += 64 * E) {
        int song[E], it[E];
#pragma unroll
        for (int e = 0; e < E; ++e) {
          const int j = j0 + e * 64 + lane;
          song[e] = -1;
          it[e] = 0;
          if (j < run) {
            int lo = 0, hi = kStgItems;  // last item with st_pre[item] <= j
#pragma unroll
            for (int st = 0; st < 8; ++st) {
              const int m = (lo + hi) >> 1;
              if (st_pre[m] <= j) lo = m; else hi = m;
            }
            song[e] = (int)p.tsongs[st_a[lo] + (j - st_pre[lo])];
            it[e] = lo;
          }
        }
#pragma unroll
        for (int e = 0; e < E; ++e)
          if (song[e] >= 0) atomicAdd(&acc[song[e]], st_q[it[e]]);
      }
      wave_lds_sync();  // the next round overwrites the staging
#pragma unroll
      for (int r = 0; r < R; ++r) {
        a0[r] = a1[r]; b0[r] = b1[r]; q0[r] = q1[r];
        v1[r] = v2[r]; q1[r] = q2[r];
      }
    }
  }
  __syncthreads();
  MR_STAMP(2);

  // Epilogue: scores -> dense row segment; keys stay in LDS for the top-k.
  const double inv_f = ldexp(1.0, -p.frac_bits);
  OutT* out = reinterpret_cast<OutT*>(p.dense_out) + (size_t)u * p.width + (blo - p.song_lo);
  // The thread's best (key desc, song asc) is tracked on the way (the
  // threshold top-k starts from it; songs ascend per thread).
  long long mk = kKeyNone;
  int ms = INT_MAX;
#pragma unroll
  for (int j = 0; j < kFusedPre; ++j) {
    const int i = tid + j * kThreads;
    if (i < bw) {
      const bool h = (heard[i >> 5] >> (i & 31)) & 1u;
      double score = (double)(long long)acc[i] * inv_f;
      if (MODEL == MR_IBM) score = score / sc[j];
      if (p.dense) out[i] = h ? (OutT)NAN : (OutT)score;
      const long long key = h ? kKeyNone : __double_as_longlong(score);
      acc[i] = (unsigned long long)key;
      if (key > mk) { mk = key; ms = blo + i; }
    }
  }
  for (int i = tid + kFusedPre * kThreads; i < bw; i += kThreads) {  // tiles wider than 1024 songs
    const bool h = (heard[i >> 5] >> (i & 31)) & 1u;
    double score = (double)(long long)acc[i] * inv_f;
    if (MODEL == MR_IBM) score = score / p.sqrt_c[blo + i];
    if (p.dense) out[i] = h ? (OutT)NAN : (OutT)score;
    const long long key = h ? kKeyNone : __double_as_longlong(score);
    acc[i] = (unsigned long long)key;
    if (key > mk) { mk = key; ms = blo + i; }
  }
  const int k = p.topk;
  if (k <= 0) return;
  __syncthreads();
  MR_STAMP(3);

  // Tile top-k -> fk/fs (LDS): per-wave DPP rounds, then a 4-list tournament;
  // wide tiles: per-thread running lists, merged per wave, then across waves.
  auto get_key = [&](int i, long long& key, int& song) {
    key = (long long)acc[i];
    song = blo + i;
  };
  bool thr_done = false;  // threshold pass first (about k candidates, ranked in parallel)
  // The tile's list goes straight from the ranking threads to its global
  // slots (sc1 for the hand-off; the user's outputs when the tile is the
  // whole shard), not through LDS + a barrier + a copy loop.
  long long* ck = p.cand_key + (size_t)u * p.n_tiles * k;
  int* cs = p.cand_song + (size_t)u * p.n_tiles * k;
  TopkDst tdst;
#ifndef MR_TOPK_VIA_LDS
  if (p.n_tiles == 1) {
    tdst.key = p.top_key + (size_t)u * k;
    tdst.song = p.top_song + (size_t)u * k;
    tdst.score = p.top_score + (size_t)u * k;
  } else {
    tdst.key = ck + (size_t)tile * k;
    tdst.song = cs + (size_t)tile * k;
    tdst.sc1 = true;
  }
#endif
  if (!p.topk_lists && k <= kThreads / 16) {
#ifdef MR_STAMPS
    long long* sbt = sb ? sb + 3 : nullptr;  // sub-phase stamps in slots 12-14
#else
    long long* sbt = nullptr;
#endif
    thr_done = block_topk_threshold<kThreads, decltype(get_key), MR_TILE_ROWS>(
        bw, k, get_key, mk, ms, smem_raw + L.gm, wk, ws, kWaves * kMaxTopK, fk, fs, sbt, tdst);
  }
  const bool direct = thr_done && tdst.key;
  if (thr_done) {
  } else if (bs <= kMaxTopkTile) {
    block_topk(bw, k, get_key, wk, ws, fk, fs);
  } else {
    long long* lk = reinterpret_cast<long long*>(smem_raw + L.acc);
    int* ls = reinterpret_cast<int*>(smem_raw + L.acc + kThreads * k * 8);
    block_topk_wide(bw, k, get_key, lk, ls, wk, ws, fk, fs);
  }
  MR_STAMP(4);

  if (p.n_tiles == 1) {  // the tile is the whole shard: publish directly
    if (!direct)
      for (int r = tid; r < k; r += kThreads) {
        const size_t o = (size_t)u * k + r;
        p.top_key[o] = fk[r];
        p.top_song[o] = fs[r];
        p.top_score[o] = fk[r] >= 0 ? __longlong_as_double(fk[r]) : (double)NAN;
      }
    return;
  }

  // Publish the tile's candidates (sc1), then count the tile in.
  // Ordering: this is the measured valid hand-off of MI355X_MICROARCH.md
  // ("Hand-offs measured with sc1 loads in place of the acquire", row 1):
  // every byte stored sc1 (write-through, dropped from L1/L2), every storing
  // wave waits vmcnt(0) (inline asm with a memory clobber, so the compiler
  // cannot sink a store below it), a workgroup barrier, ONE lane's agent-scope
  // atomic add; the last adder's workgroup reads only after a barrier it
  // joins, with sc1 loads (L1 bypassed). A release/acquire fence pair at agent
  // scope would lower to buffer_wbl2 sc1 + buffer_inv sc1 — a write-back of
  // the XCD's whole L2 (≈1.7-6.5 us per the guide's price table) on every
  // tile's critical path — and adds nothing this protocol needs on gfx950.
  if (!direct)
    for (int r = tid; r < k; r += kThreads) {
      st_sc1(&ck[(size_t)tile * k + r], fk[r]);
      st_sc1(&cs[(size_t)tile * k + r], fs[r]);
    }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0) {
    const unsigned old = __hip_atomic_fetch_add(&p.counter[(size_t)u * kCounterStride], 1u, __ATOMIC_RELAXED,
                                                __HIP_MEMORY_SCOPE_AGENT);
    *flag = (old == (unsigned)(p.n_tiles - 1));
  }
  __syncthreads();
  MR_STAMP(5);
#ifdef MR_STAMPS
  if (tid == 0 && sb)
    sb[15] = (long long)(*flag) | ((long long)__builtin_amdgcn_s_getreg((20 << 0) | (0 << 6) | (3 << 11)) << 8);
#endif
  if (!*flag) return;

  bool merged_direct = false;  // the merge's select wrote the user's outputs itself
  // Last tile of user u: tournament over the tiles' sorted candidate lists,
  // staged into LDS region A with sc1 loads (stage_lists lists per pass; the
  // running top-k is list 0 of every later pass). (A prune-by-max-k-th-key +
  // rank-counting merge measured 28.4 vs 26.2 us per C2 step: its rank loop is
  // a chain of dependent LDS reads.)
  {
    long long* mk = reinterpret_cast<long long*>(smem_raw + L.acc);
    int* ms = reinterpret_cast<int*>(smem_raw + L.acc + L.stage_lists * k * 8);
    const int w = tid >> 6;
    int done = 0, off = 0;
    merged_direct = false;
#ifndef MR_MERGE_VIA_LDS
    // At most one candidate per thread (C2: 22 tiles x 10 <= 256): each thread
    // loads its candidate into registers and the threshold select reads it
    // there — no LDS staging pass and barrier before the select.
    const int nck = p.n_tiles * k;
    if (!p.topk_lists && nck <= kThreads && k <= kThreads / 16 && p.merge_rows == 32) {
      long long rk = kKeyNone;
      int rs = INT_MAX;
      if (tid < nck) {
#if MR_MERGE_INTERLEAVE
        // thread t holds position t / n_tiles of tile t % n_tiles: a threshold
        // row is one list position over 8 tiles, not 8 positions of one tile
        const int ci = (tid % p.n_tiles) * k + tid / p.n_tiles;
#else
        const int ci = tid;
#endif
        rk = ld_sc1(&ck[ci]);
        rs = ld_sc1(&cs[ci]);
      }
      MR_STAMP(6);
      auto get_r = [&](int, long long& key, int& song) { key = rk; song = rs; };  // called for i = tid only
      TopkDst mdst;
      mdst.key = p.top_key + (size_t)u * k;
      mdst.song = p.top_song + (size_t)u * k;
      mdst.score = p.top_score + (size_t)u * k;
      merged_direct = block_topk_threshold<kThreads, decltype(get_r), 32>(
          nck, k, get_r, rk >= 0 ? rk : kKeyNone, rk >= 0 ? rs : INT_MAX, smem_raw + L.gm, wk, ws,
          kWaves * kMaxTopK, fk, fs, nullptr, mdst);
      MR_STAMP(8);
    }
#endif
    while (!merged_direct && done < p.n_tiles) {
      const int nl = min(p.n_tiles - done, L.stage_lists - off);
      // 4 candidates per thread in flight per batch (loads first, then LDS)
      for (int i0 = tid; i0 < nl * k; i0 += 4 * kThreads) {
        long long lk4[4];
        int ls4[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int i = i0 + r * kThreads;
          lk4[r] = kKeyNone;
          ls4[r] = -1;
          if (i < nl * k) {
            lk4[r] = ld_sc1(&ck[(size_t)done * k + i]);
            ls4[r] = ld_sc1(&cs[(size_t)done * k + i]);
          }
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int i = i0 + r * kThreads;
          if (i < nl * k) {
            mk[off * k + i] = lk4[r];
            ms[off * k + i] = ls4[r];
          }
        }
      }
      for (int i = tid; i < off * k; i += kThreads) {
        mk[i] = fk[i];
        ms[i] = fs[i];
      }
      __syncthreads();
      MR_STAMP(6);
      bool merged = false;
      TopkDst mdst;  // the user's outputs, written by the ranking threads
#ifndef MR_TOPK_VIA_LDS
      mdst.key = p.top_key + (size_t)u * k;
      mdst.song = p.top_song + (size_t)u * k;
      mdst.score = p.top_score + (size_t)u * k;
#endif
      // (A threshold on the sorted lists' HEADS — the k-th best head — measured
      // 16.7 vs 14.0 us per C2 step: it is a much looser bound than the row
      // bests, ~5x the survivors to rank; profiles/r02/c2_merge_heads_ab.txt.)
      if (!p.topk_lists && done == 0 && nl == p.n_tiles && k <= kThreads / 16) {  // one pass: threshold select
        auto get_c = [&](int i, long long& key, int& song) { key = mk[i]; song = ms[i]; };
        long long bk;
        int bsg;
        thread_best<kThreads>(nl * k, get_c, bk, bsg);
        if (p.merge_rows == 16)
          merged = block_topk_threshold<kThreads, decltype(get_c), 16>(nl * k, k, get_c, bk, bsg, smem_raw + L.gm,
                                                                      wk, ws, kWaves * kMaxTopK, fk, fs, nullptr, mdst);
        else if (p.merge_rows == 64)
          merged = block_topk_threshold<kThreads, decltype(get_c), 64>(nl * k, k, get_c, bk, bsg, smem_raw + L.gm,
                                                                      wk, ws, kWaves * kMaxTopK, fk, fs, nullptr, mdst);
        else
          merged = block_topk_threshold<kThreads, decltype(get_c), 32>(nl * k, k, get_c, bk, bsg, smem_raw + L.gm,
                                                                      wk, ws, kWaves * kMaxTopK, fk, fs, nullptr, mdst);
      }
      if (!merged) {
        if (w == 0) wave_merge_lists(nl + off, k, mk, ms, fk, fs);
        __syncthreads();
      }
      MR_STAMP(8);
      merged_direct = merged && mdst.key;
      done += nl;
      off = 1;
    }
  }
  if (!merged_direct)
    for (int r = tid; r < k; r += kThreads) {
      const size_t o = (size_t)u * k + r;
      p.top_key[o] = fk[r];
      p.top_song[o] = fs[r];
      p.top_score[o] = fk[r] >= 0 ? __longlong_as_double(fk[r]) : (double)NAN;
    }
  if (tid == 0) p.counter[(size_t)u * kCounterStride] = 0u;  // ready for the next launch (kernel boundary orders it)
  MR_STAMP(9);
}

// ---------------------------------------------------------------------------
// wide shape (large train sets, config 4): one (test user, 16k-song tile)
// per NT-thread workgroup. The 128 KiB tile admits one workgroup per CU, so
// the workgroup itself is wide (NT = 1024: 4 waves per SIMD) to keep enough
// independent neighbour visits in flight; the per-(v, tile) segments are
// short (|S(v)| / n_tiles), heavy-tailed work is spread by the hardware over
// 16 waves. Tile candidates go to cand_key/cand_song; k_topk_merge reduces
// them per user in a second launch. MR:159-166 / MR:249-257.
// ---------------------------------------------------------------------------
template <int NT>
__device__ __forceinline__ int block_excl_scan_nt(int x, int* total, int* sbuf) {
  constexpr int NW = NT / 64;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int incl = wave_incl_scan(x);
  if (lane == 63) sbuf[w] = incl;
  __syncthreads();
  int off = 0, tot = 0;
#pragma unroll
  for (int i = 0; i < NW; ++i) {
    const int v = sbuf[i];
    off += (i < w) ? v : 0;
    tot += v;
  }
  __syncthreads();
  *total = tot;
  return off + incl - x;
}

template <int NT>
struct WideLds {
  int acc, heard, cpre, s_scan, wk, ws, fk, fs, gm, total;
  WideLds<1024> as_wide() const { return WideLds<1024>{acc, heard, cpre, s_scan, wk, ws, fk, fs, gm, total}; }
};
template <int NT>
__host__ __device__ inline WideLds<NT> wide_lds(int bs, int k, int n_chunks) {
  constexpr int NW = NT / 64;
  const int kk = k > 0 ? k : 1;
  WideLds<NT> L;
  int o = 0;
  L.acc = o; o = align16(o + bs * 8);
  L.heard = o; o = align16(o + (bs / 32) * 4);
  L.cpre = o; o = align16(o + (n_chunks + 1) * 4);
  L.s_scan = o; o = align16(o + NW * 4);
  L.wk = o; o = align16(o + NW * kk * 8);
  L.ws = o; o = align16(o + NW * kk * 4);
  L.fk = o; o = align16(o + kk * 8);
  L.fs = o; o = align16(o + kk * 4);
  L.gm = o; o = align16(o + topk_scratch_bytes<NT>());
  L.total = o;
  return L;
}

constexpr int kWideThreads = 1024;
#ifndef MR_WIDE_R
#define MR_WIDE_R 4         // neighbours per thread per iteration (wide kernel, 3-level software pipeline):
                            // 4 vs 2 at C5's ubm model 61.7 vs 66.0 ms, C3 1.108 vs 1.119 ms (ibm) —
                            // 3: 63.1, 6: 71.0, 8 spills (profiles/r04/s27, s28; round 2 measured 2
                            // ahead by 2 % at C4 on an older kernel, profiles/r02/c4/pipeline_ab.txt)
#endif
#ifndef MR_WIDE_SEG
#define MR_WIDE_SEG 12      // first entries of every segment loaded in one batch (wide kernel; swept 2-16)
#endif
#ifndef MR_WIDE_Z16
#define MR_WIDE_Z16 1       // wide kernel: the accumulators zeroed by 16-B LDS stores
#endif
#ifndef MR_WIDE_EB
#define MR_WIDE_EB 8        // wide-kernel epilogue: songs per thread whose scale loads are issued together
#endif
#ifndef MR_COOC_U
#define MR_COOC_U 4         // co-listening route: 16-B pool loads (4 entries) per thread in flight
#endif
#ifndef MR_COOC_DU
#define MR_COOC_DU 4        // co-listening route: dense rows whose loads are issued together
#endif
#ifndef MR_COOC_DS
#define MR_COOC_DS 8        // co-listening route: dense-pass songs per thread per block (8 or 16)
#endif
#ifndef MR_COOC_SPLIT
#define MR_COOC_SPLIT 1     // co-listening scoring: the dense pass's u32 half-weight sums (frac_bits <= 32)
#endif
#ifndef MR_COOC_DOT2
#define MR_COOC_DOT2 1      // co-listening scoring: the split dense pass two rows per v_dot2_u32_u16
#endif
typedef unsigned short us2_t __attribute__((ext_vector_type(2)));
#ifndef MR_COOC_NOZERO
#define MR_COOC_NOZERO 1    // co-listening scoring: acc zeroed only when the first pass has no dense row
#endif
#ifndef MR_GROUP_STUB
#define MR_GROUP_STUB 0     // timing-only builds of k_cooc_group's emission (1: no sparse stores, 2: pass A only)
#endif
#ifndef MR_COOC_DPF
#define MR_COOC_DPF 1       // co-listening scoring: the first descriptor pass's row lookups issued before the zeroing
#endif
#ifndef MR_COOC_PF
#define MR_COOC_PF 0        // co-listening scoring: per-song scales prefetched per thread (songs tid + NT e;
                            // 0 = none)
#endif
#ifndef MR_COOC_R
#define MR_COOC_R 2         // co-listening index build: listeners per thread per iteration
#endif
#ifndef MR_COOC_NT16
#define MR_COOC_NT16 512    // co-listening index build, u16-pair counters: threads per workgroup (4 per CU)
#endif
#ifndef MR_COOC_P16
#define MR_COOC_P16 1       // 0: every heavy row with u32 counters (A/B)
#endif
#ifndef MR_COOC_NT
#define MR_COOC_NT 1024     // co-listening index build: threads per workgroup
#endif
// 16-B vector of 4-B-aligned words (global_load_dwordx4 needs dword alignment only)
typedef unsigned u32x4_a4 __attribute__((ext_vector_type(4), aligned(4)));
// Co-listening index entries: (tile-local song << kCoocCntBits) | count, so
// tiles <= 32768 songs and counts < 131072 (mr_load checks both).
constexpr int kCoocCntBits = 17;
// seg_len of a dense segment (<= -3): a byte per song of the tile, the count
// saturated at the build's sat value (255), then -seg_len - 3 sparse entries
// carrying each larger count's excess (count - sat) — the dense pass adds
// min(count, sat) · q, the sparse walk the rest.
// The ORDER of the entries inside a sparse segment or a dense segment's excess
// tail is unspecified (LDS atomics place them: the touched-song list, the
// excess counter, the light rows' hash order and tile cursors), so two builds
// of the same index may differ byte for byte; every consumer sums the entries
// (order-free integer adds), so the scores never do. Compare indexes as sets.
constexpr int kCoocDenseTail = -3;
// Count-byte order of a dense segment: lane-interleaved blocks of 64 x DS
// songs (DS = MR_COOC_DS). In each block, the DS-byte chunk t holds songs t,
// t + 64, ..., t + 64 (DS - 1) of the block: the scoring's dense pass loads
// chunk t in lane t (coalesced, as before) and adds its DS sums into acc at
// songs t + 64 i — consecutive across the wave, so the LDS read-modify-writes
// are free of bank conflicts (song-ordered chunks put the lanes' u64 adds
// 8 x DS bytes apart: 16-way conflicts at DS = 8). The segment holds whole
// blocks (songs past the tile: count 0).
constexpr int kDenseDS = MR_COOC_DS;
constexpr int kDenseBlock = 64 * kDenseDS;
__host__ __device__ inline int cooc_dense_words(int bw) {
  return (bw + kDenseBlock - 1) / kDenseBlock * (kDenseBlock / 4);
}
// the song of byte i of chunk c
__host__ __device__ inline int cooc_dense_song(int c, int i) { return (c >> 6) * kDenseBlock + 64 * i + (c & 63); }
constexpr int kCoocDenseDiv = 3;
#ifndef MR_COOC_BIG_ROW
#define MR_COOC_BIG_ROW 2048  // C4 44.74 vs 45.16 ms at 4096, 8x1 6.06 vs 6.10 (profiles/r04/s43, s44)
#endif
constexpr int kCoocBigRow = MR_COOC_BIG_ROW;  // listeners from which a heavy row's tiles get a workgroup each  // dense when non-zeros * this >= the tile's songs (MR_COOC_DENSE_DIV)
constexpr unsigned kCoocCntMask = (1u << kCoocCntBits) - 1u;
constexpr int kCoocMaxTile = 1 << (32 - kCoocCntBits);


// Stage 2 of the wide shape as a walk over a list of train users: entry k <
// cnt of the list is (v, w) = load_list(k) (v = -1 past the end); every
// tile-local song x of v's segment in this tile (tsongs[toff_t[v] ..
// toff_t[v+1])) gets acc[x] += w by an LDS atomic. R entries per thread per
// iteration. Used by the two-hop scoring (list = the test user's neighbours,
// w = their int64 weights) and by the co-listening index build (list = one
// song's train listeners, w = 1).
template <int NT, int R, int kSeg, typename WT, typename LoadList, typename Add>
__device__ __forceinline__ void walk_tile_lists(int tid, int cnt, LoadList&& load_list, const int* toff_t,
                                                const unsigned short* tsongs, Add&& add) {
  // Software pipeline over iterations: iteration i gathers its segments
  // while the toff pairs of i+1 and the list entries of i+2 are in flight
  // (one memory latency covers the three dependent levels).
  auto load_offs = [&](const int (&v)[R], int (&a)[R], int (&b)[R]) {
#pragma unroll
    for (int r = 0; r < R; ++r) {
      a[r] = b[r] = 0;
      if (v[r] >= 0) { a[r] = toff_t[v[r]]; b[r] = toff_t[v[r] + 1]; }
    }
  };
  int v0[R], a0[R], b0[R], v1[R], a1[R], b1[R], v2[R];
  WT q0[R], q1[R], q2[R];
  load_list(tid, v0, q0);
  load_offs(v0, a0, b0);
  load_list(tid + R * NT, v1, q1);
  for (int k0 = tid; k0 < cnt; k0 += R * NT) {
#ifndef MR_WIDE_U16
    // a segment's first kSeg entries as 8-B words (4 tile-local ids each)
    // from the aligned word holding entry a0: kW loads instead of kSeg
    // 2-B loads (C4 21.9 vs 22.9 ms per 704-user batch, C3 1.093 vs 1.141 ms
    // per step; MR_WIDE_U16 builds the 2-B form, profiles/r02/c4/vec_seg_ab.txt)
    constexpr int kW = (kSeg + 3) / 4 + 1;
    const uint2* tw = reinterpret_cast<const uint2*>(tsongs);
    uint2 sw[R][kW];
    int so[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const int wb = a0[r] >> 2;
      const int we = b0[r] > a0[r] ? (b0[r] + 3) >> 2 : wb;
      so[r] = a0[r] & 3;
#pragma unroll
      for (int j = 0; j < kW; ++j) sw[r][j] = wb + j < we ? tw[wb + j] : make_uint2(0u, 0u);
    }
#else
    int sg[R][kSeg];
#pragma unroll
    for (int r = 0; r < R; ++r)
#pragma unroll
      for (int j = 0; j < kSeg; ++j) sg[r][j] = a0[r] + j < b0[r] ? (int)tsongs[a0[r] + j] : -1;
#endif
    load_offs(v1, a1, b1);                 // iteration i+1
    load_list(k0 + 2 * R * NT, v2, q2);    // iteration i+2
#pragma unroll
    for (int r = 0; r < R; ++r) {
#ifndef MR_WIDE_U16
#pragma unroll
      for (int j = 0; j < kSeg; ++j) {
        if (a0[r] + j < b0[r]) {
          const int e = (j & 3) + so[r];  // 0..6: word j/4 or the next one
          const uint2 wv = e >= 4 ? sw[r][(j >> 2) + 1] : sw[r][j >> 2];
          const unsigned x = ((e & 3) < 2 ? wv.x : wv.y) >> ((e & 1) * 16);
          add(x & 0xffffu, q0[r]);
        }
      }
#else
#pragma unroll
      for (int j = 0; j < kSeg; ++j)
        if (sg[r][j] >= 0) add((unsigned)sg[r][j], q0[r]);
#endif
      for (int x0 = a0[r] + kSeg; x0 < b0[r]; x0 += kSeg) {
        int st[kSeg];
#pragma unroll
        for (int j = 0; j < kSeg; ++j) st[j] = x0 + j < b0[r] ? (int)tsongs[x0 + j] : -1;
#pragma unroll
        for (int j = 0; j < kSeg; ++j)
          if (st[j] >= 0) add((unsigned)st[j], q0[r]);
      }
    }
#pragma unroll
    for (int r = 0; r < R; ++r) {
      a0[r] = a1[r]; b0[r] = b1[r]; q0[r] = q1[r];
      v1[r] = v2[r]; q1[r] = q2[r];
    }
  }
  (void)v0;
}

// Candidate-only tile top-k of the wide kernel, for top-k-only runs (no
// dense row, no min / max): the epilogue computes the exact fp64 score of
// every song only to rank it, and ~k of a tile's ~19k songs leave the tile.
// Here every song gets an fp32 approximation from its integer accumulator —
// a ≈ acc / sqrt(c(s)) (ibm; acc for ubm) with a 4-B table of 1/sqrt(c) —
// kept in registers (songs i = tid + NT e, e < EMAX); tau is the k-th best
// row best of those (block_tau); only songs with a >= tau · (1 − 2^-17) get
// the exact key (the same fp64 ops as the all-songs epilogue: the oracle's)
// and are ranked exactly (rank_survivors).
// Why no top-k song is lost: a carries ≤ 5·2^-24 relative error (the two
// halves of acc converted, fma, the table's rounding, the product), the fp64
// key ≤ 2^-52. The k songs behind tau have exact scores ≥ tau(1 − δ)/(1 + δ),
// so the k-th best exact score is too, and any song ranked at or above it has
// a ≥ tau(1 − 2δ − 2ε) > tau(1 − 2^-17). Ties of exact scores have equal
// approximations (same acc, same c). Returns false, uniformly, when the
// survivors overflow cap (e.g. fewer than k positive scores: tau = 0); acc
// is untouched, so the caller then runs the all-songs path.
#ifndef MR_CAND_EB
#define MR_CAND_EB 4  // wide_cand_topk: songs per thread whose loads are issued together (5 / 7 slower, 10 spilled)
#endif
#ifndef MR_CAND_PRE
#define MR_CAND_PRE 1  // the first batch's scales loaded by the caller before stage 2's last barrier
#endif
template <int MODEL, int NT, int EMAX>
__device__ __forceinline__ bool wide_cand_topk(const ScoreParams& p, const unsigned long long* acc,
                                               const unsigned* heard, int blo, int bw, int k, unsigned char* gm,
                                               long long* ck, int* cs, int cap, long long* fk, int* fs,
                                               long long* sb, bool have_rv, const float (&pre_rv)[MR_CAND_EB]) {
  constexpr int NG = NT / 16;
  const int tid = threadIdx.x;
  float ap[EMAX];
  // the thread's best approximation and its slot: songs ascend with e, so a
  // strictly larger value is the (key desc, song asc) order's better one
  float ba = -1.f;
  int be = -1;
  constexpr int EB = MR_CAND_EB;
#pragma unroll
  for (int e0 = 0; e0 < EMAX; e0 += EB) {
    unsigned long long av[EB];
    float rv[EB];
#pragma unroll
    for (int j = 0; j < EB; ++j) {
      const int i = tid + (e0 + j) * NT;
      av[j] = 0ull;
      rv[j] = 0.f;
      if (e0 + j < EMAX && i < bw) {
        av[j] = acc[i];
        // (loading these at the kernel's start, in flight during stage 2, ran
        // 41.46 vs 41.08 ms at C4: profiles/r05/s2)
        rv[j] = MODEL != MR_IBM ? 1.f : (e0 == 0 && have_rv) ? pre_rv[j] : p.rsq_c[blo + i];
      }
    }
#pragma unroll
    for (int j = 0; j < EB; ++j) {
      const int e = e0 + j;
      if (e >= EMAX) continue;
      const int i = tid + e * NT;
      float a = -1.f;
      if (i < bw && !((heard[i >> 5] >> (i & 31)) & 1u)) {
        const float hi = (float)(unsigned)(av[j] >> 32), lo = (float)(unsigned)av[j];
        a = __fmaf_rn(hi, 4294967296.f, lo) * rv[j];
      }
      be = a > ba ? e : be;
      ba = a > ba ? a : ba;
      ap[e] = a;
    }
  }
  // (non-negative floats order as their bit patterns: the key of a)
  const long long mk = be >= 0 ? (long long)__float_as_uint(ba) : kKeyNone;
  const int ms = be >= 0 ? blo + tid + be * NT : INT_MAX;
  MR_STAMP(3);
  long long tk;
  int tsg;
  block_tau<NT, NG>(k, mk, ms, gm, tk, tsg, sb);
  int* counter = reinterpret_cast<int*>(reinterpret_cast<long long*>(gm) + NG + 1) + NG + 1;
  int* crank = counter + 1 + NG;
  const float thr = __uint_as_float((unsigned)tk) * (1.f - 0x1p-17f);  // tk = 0 (none): every song
  const double inv_f = ldexp(1.0, -p.frac_bits);
  // the thread's survivors as a bit mask (heard / past the tile: a = -1), then
  // a compact loop over the set bits (a few per tile: no unrolled 20-way body)
  unsigned sm = 0u;
#pragma unroll
  for (int e = 0; e < EMAX; ++e) sm |= ap[e] >= thr ? 1u << e : 0u;
  while (sm) {
    const int e = __builtin_ctz(sm);
    sm &= sm - 1u;
    const int i = tid + e * NT;
    double score = (double)(long long)acc[i] * inv_f;
    if (MODEL == MR_IBM) score = score / p.sqrt_c[blo + i];
    const int pos = atomicAdd(counter, 1);
    if (pos < cap) { ck[pos] = __double_as_longlong(score); cs[pos] = blo + i; }
  }
  __syncthreads();
  stamp_at(sb, 11);
  const int nc = *counter;
  if (nc > cap) return false;
  rank_survivors<NT>(nc, k, ck, cs, crank, fk, fs);
  return true;
}
constexpr int kCandE = 20;  // wide_cand_topk: songs per thread (tiles <= 20 x NT songs)

// KS: register slots of the per-thread lists (10: k = 10 exactly, the
// default, compiled in; 16: any k <= 16 at run time).
template <int MODEL, typename OutT, int NT, int KS, bool COOC>
__global__ __launch_bounds__(NT) void k_score_wide(ScoreParams p) {
  constexpr int NW = NT / 64;
  extern __shared__ __align__(16) unsigned char smem_raw[];
  const int bs = p.block_songs;
  const WideLds<NT> L = wide_lds<NT>(bs, p.topk, p.n_chunks);
  unsigned long long* acc = reinterpret_cast<unsigned long long*>(smem_raw + L.acc);
  unsigned* heard = reinterpret_cast<unsigned*>(smem_raw + L.heard);
  int* cpre = reinterpret_cast<int*>(smem_raw + L.cpre);
  int* s_scan = reinterpret_cast<int*>(smem_raw + L.s_scan);

  // Block -> (user, tile), speed only (blocks are dealt round-robin over the
  // 8 XCDs): xcd_remap 1 = all tiles of a user on one XCD (the user's
  // neighbour list is fetched into one L2); 2 = the (tile, user) pairs in
  // tile-major order cut into 8 contiguous ranges, one per XCD, so the CUs of
  // an XCD sweep the SAME tile's train-side rows (toff, tsongs: read almost
  // whole by every user) for consecutive users at once and share them in L2.
  const int lin = blockIdx.y * gridDim.x + blockIdx.x;
  const int slot = lin >> 3;
  int bu, tile;
  if (p.xcd_remap == 2) {
    const int per_xcd = (gridDim.x * gridDim.y) >> 3;  // gridDim.y padded to a multiple of 8
    const int pidx = (lin & 7) * per_xcd + slot;
    tile = pidx / gridDim.y;
    bu = pidx - tile * gridDim.y;
  } else if (p.xcd_remap == 3) {  // tile-major: every XCD on the same tile at once
    tile = lin / gridDim.y;
    bu = lin - tile * gridDim.y;
  } else {
    bu = (slot / p.n_tiles) * 8 + (lin & 7);
    tile = slot % p.n_tiles;
  }
  if (bu >= p.n_users) return;  // grid padded to a multiple of 8 users
  const int u = p.user0 + bu;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int blo = p.song_lo + tile * bs;
  const int bhi = min(p.song_hi, blo + bs);
  const int bw = bhi - blo;
  MR_STAMP(0);

  // co-listening route: the epilogue's per-song scales of this thread's songs
  // (i = tid + NT e) loaded now, in flight while stage 2 runs (a tile's
  // scales are the same for every user: L2 hits, but three dependent batches
  // of them were ~2 us of the epilogue)
  constexpr bool kPF = COOC && MR_COOC_PF > 0;
  constexpr int PF = kPF ? MR_COOC_PF : 1;
  double scp[PF];
  if constexpr (kPF) {
#pragma unroll
    for (int e = 0; e < PF; ++e) {
      const int i = tid + e * NT;
      scp[e] = i < bw ? p.sqrt_c[blo + i] : 1.0;
    }
  }
  // co-listening route: the first descriptor pass's row lookups (te_row /
  // te_songs, then seg_len / seg_off / q_song) issued around the zeroing and
  // the heard bitmap instead of after them (two dependent loads off the
  // descriptor phase's critical path)
  constexpr bool kDPF = COOC && MR_COOC_DPF;
  int pf_r = -1, pf_s = 0, pf_sl = 0;
  long long pf_off = 0;
  unsigned long long pf_q = 0ull;
  if constexpr (kDPF) {
    const long long a = p.te_off[u];
    if (tid < min<long long>(p.nseg, p.te_off[u + 1] - a)) {
      pf_r = p.te_row[a + tid];
      pf_s = p.te_songs[a + tid];
    }
  }
  // co-listening route (MR_COOC_NOZERO): a first descriptor pass with dense
  // rows STORES every song's dense sum (the pass covers the whole tile), so
  // acc is zeroed here only for users without index rows, else after the
  // first pass's scan when it has no dense row
  auto zero_acc = [&]() {
#if MR_WIDE_Z16  // 16-B stores: two songs per store (acc is 16-B aligned; bs is even)
    for (int i = tid; 2 * i < bw; i += NT) reinterpret_cast<ulonglong2*>(acc)[i] = make_ulonglong2(0ull, 0ull);
#else
    for (int i = tid; i < bw; i += NT) acc[i] = 0ull;
#endif
  };
  if (!(COOC && MR_COOC_NOZERO) || p.te_off[u + 1] == p.te_off[u]) zero_acc();
  if constexpr (kDPF) {
    if (pf_r >= 0) {
      pf_sl = p.seg_len[(size_t)tile * p.n_rows + pf_r];
      pf_off = p.seg_off[(size_t)tile * p.n_rows + pf_r];
      pf_q = (unsigned long long)p.q_song[pf_s];
    }
  }
  for (int i = tid; i < bs / 32; i += NT) heard[i] = 0u;
  __syncthreads();
  for (long long i = p.te_off[u] + tid; i < p.te_off[u + 1]; i += NT) {
    const int s = p.te_songs[i];
    if (s >= blo && s < bhi) atomicOr(&heard[(s - blo) >> 5], 1u << ((s - blo) & 31));
  }
  const int nch = p.n_chunks;
  int cnt = 0;
  if constexpr (!COOC) {
    for (int c0 = 0; c0 < nch; c0 += NT) {
      const int cc = c0 + tid;
      const int x = cc < nch ? p.nbr_cnt[(size_t)bu * nch + cc] : 0;
      int tot;
      const int pre = block_excl_scan_nt<NT>(x, &tot, s_scan);
      if (cc < nch) cpre[cc] = cnt + pre;
      cnt += tot;
    }
    if (tid == 0) cpre[nch] = cnt;
  }
  __syncthreads();
  MR_STAMP(1);

  bool have_rv = false;  // (COOC, p.cand: pass A's first scales loaded at the end of stage 2)
  float pre_rv[MR_CAND_EB];
  if constexpr (COOC) {
    // stage 2 from the co-listening index: acc[s] += q(s2) * C[s2][s] over
    // u's index rows' segments in this tile. Dense segments (every song's
    // count) are summed per song by the thread that owns it, in registers;
    // sparse segments are walked as one flattened list (coalesced pool reads,
    // LDS atomics). Descriptors of up to nseg rows per pass live in the top-k
    // scratch, which is free until the epilogue.
    long long* m_off = reinterpret_cast<long long*>(smem_raw + L.wk);
    unsigned long long* m_q = reinterpret_cast<unsigned long long*>(m_off + p.nseg);
    long long* d_off = reinterpret_cast<long long*>(m_q + p.nseg);
    unsigned long long* d_q = reinterpret_cast<unsigned long long*>(d_off + p.nseg);
    int* m_pre = reinterpret_cast<int*>(d_q + p.nseg);
    int* d_fmt = m_pre + p.nseg + 1;
    const long long t0 = p.te_off[u], t1 = p.te_off[u + 1];
    const int* slen = p.seg_len + (size_t)tile * p.n_rows;
    const long long* soff = p.seg_off + (size_t)tile * p.n_rows;
    for (long long c0 = t0; c0 < t1; c0 += p.nseg) {
      const int ns = (int)min<long long>(p.nseg, t1 - c0);
      int len = 0, isd = 0, fmt = 0;
      long long off = 0, tail_off = -1;
      unsigned long long q = 0ull;
      if (tid < ns) {
        int r, sl = 0;
        if (kDPF && c0 == t0) {  // (prefetched above)
          r = pf_r;
          sl = pf_sl;
          off = pf_off;
          q = pf_q;
        } else {
          r = p.te_row[c0 + tid];
          if (r >= 0) {
            sl = slen[r];
            off = soff[r];
            q = (unsigned long long)p.q_song[p.te_songs[c0 + tid]];
          }
        }
        if (r >= 0) {
          if (sl < 0) {  // saturated count bytes, then the excess entries
            isd = 1;
            fmt = sl;
            len = kCoocDenseTail - sl;
            tail_off = off + cooc_dense_words(bw);
          } else {
            len = sl;
          }
        }
      }
      // one scan of (entries << 8 | dense): nseg <= 255 rows of < 32768
      // entries each per pass (mr_load), so both sums fit
      int tot_pk;
      const int pk = block_excl_scan_nt<NT>((len << 8) | isd, &tot_pk, s_scan);
      const int pre = pk >> 8, dpre = pk & 255;
      const int total = tot_pk >> 8, nd = tot_pk & 255;
      if (tid < ns) {
        m_off[tid] = (tail_off >= 0 ? tail_off : off) - pre;
        m_q[tid] = q;
        m_pre[tid] = pre;
        if (isd) { d_off[dpre] = off; d_q[dpre] = q; d_fmt[dpre] = fmt; }
      }
      if (tid == 0) m_pre[ns] = total;
      __syncthreads();
      MR_STAMP(12);  // (the last descriptor pass's) descriptors ready
      const bool store = MR_COOC_NOZERO && c0 == t0;  // the first pass: dense sums stored, else zeroed here
      if (store && nd == 0) {
        zero_acc();
        __syncthreads();
      }
      if (nd > 0) {
        // DS songs per thread per block of DS * NT, every dense row summed in
        // registers (DS = 8: one 8-B load per row; 16: one 16-B load per row,
        // half the blocks per tile)
        constexpr int DS = kDenseDS;
        typedef unsigned dvec_t __attribute__((ext_vector_type(DS / 4)));
        // chunk c = b0 / DS: songs cooc_dense_song(c, i) (wave-uniform block)
        constexpr int DU = MR_COOC_DU;  // dense rows per step, their loads issued together
#if MR_COOC_SPLIT
        if (p.frac_bits <= 32) {
          // q <= 2^32: its 16-bit halves times the count bytes summed in u32
          // (v_mad_u32_u24; <= 255 rows x 255 x 2^16 < 2^32), the row
          // descriptors read from lanes (v_readlane: scalar, no LDS round trip
          // before each row's load)
          for (int b0 = DS * tid; (b0 & ~(kDenseBlock - 1)) < bw; b0 += DS * NT) {
            unsigned lo[DS], hi[DS];
#pragma unroll
            for (int i = 0; i < DS; ++i) lo[i] = hi[i] = 0u;
            for (int g0 = 0; g0 < nd; g0 += 64) {
              const int dj = g0 + lane, ng = min(64, nd - g0);
              const long long mo = dj < nd ? d_off[dj] : 0;
              const unsigned long long mq = dj < nd ? d_q[dj] : 0ull;
              const int mo_lo = (int)(unsigned)mo, mo_hi = (int)(mo >> 32), mq_lo = (int)(unsigned)mq,
                        mq_hi = (int)(mq >> 32);
              for (int d0 = 0; d0 < ng; d0 += DU) {
                dvec_t v0[DU];
                unsigned ql[DU], qh[DU];
#pragma unroll
                for (int j = 0; j < DU; ++j) {
                  const int d = d0 + j;
                  v0[j] = dvec_t(0u);
                  ql[j] = qh[j] = 0u;
                  if (d < ng) {
                    const long long off = (long long)(((unsigned long long)(unsigned)__builtin_amdgcn_readlane(mo_hi, d)
                                                       << 32) |
                                                      (unsigned)__builtin_amdgcn_readlane(mo_lo, d));
                    const unsigned long long q =
                        ((unsigned long long)(unsigned)__builtin_amdgcn_readlane(mq_hi, d) << 32) |
                        (unsigned)__builtin_amdgcn_readlane(mq_lo, d);
                    ql[j] = (unsigned)(q & 0xffffu);
                    qh[j] = (unsigned)(q >> 16);
                    v0[j] = *reinterpret_cast<const dvec_t*>(p.pool + off + (b0 >> 2));
                  }
                }
#if MR_COOC_DOT2
                // two rows per v_dot2_u32_u16: a song's two count bytes as a
                // u16 pair (one v_perm_b32) times the rows' weight halves —
                // 1.5 VALU per count byte; a row with q = 2^32 (q >> 16 =
                // 2^16, one listener) takes the u24 path with its partner
                static_assert(DU % 2 == 0, "row pairs");
#pragma unroll
                for (int j = 0; j < DU; j += 2) {
                  if (qh[j] <= 0xffffu && qh[j + 1] <= 0xffffu) {
                    const us2_t qlp = __builtin_bit_cast(us2_t, ql[j] | (ql[j + 1] << 16));
                    const us2_t qhp = __builtin_bit_cast(us2_t, qh[j] | (qh[j + 1] << 16));
#pragma unroll
                    for (int i = 0; i < DS; ++i) {
                      const unsigned sel = 0x0c000c00u | ((4u + (i & 3)) << 16) | (unsigned)(i & 3);
                      const us2_t c2 = __builtin_bit_cast(us2_t, __builtin_amdgcn_perm(v0[j + 1][i >> 2], v0[j][i >> 2], sel));
                      lo[i] = __builtin_amdgcn_udot2(c2, qlp, lo[i], false);
                      hi[i] = __builtin_amdgcn_udot2(c2, qhp, hi[i], false);
                    }
                  } else {
#pragma unroll
                    for (int jj = j; jj < j + 2; ++jj)
#pragma unroll
                      for (int i = 0; i < DS; ++i) {
                        const unsigned c = (v0[jj][i >> 2] >> (8 * (i & 3))) & 0xffu;
                        lo[i] += __umul24(c, ql[jj]);
                        hi[i] += __umul24(c, qh[jj]);
                      }
                  }
                }
#else
#pragma unroll
                for (int j = 0; j < DU; ++j) {
#pragma unroll
                  for (int i = 0; i < DS; ++i) {
                    const unsigned c = (v0[j][i >> 2] >> (8 * (i & 3))) & 0xffu;
                    lo[i] += __umul24(c, ql[j]);
                    hi[i] += __umul24(c, qh[j]);
                  }
                }
#endif
              }
            }
#pragma unroll
            for (int i = 0; i < DS; ++i) {
              const int col = cooc_dense_song(b0 / DS, i);
              const unsigned long long v = ((unsigned long long)hi[i] << 16) + lo[i];
              if (col < bw) acc[col] = store ? v : acc[col] + v;
            }
          }
        } else
#endif
        for (int b0 = DS * tid; (b0 & ~(kDenseBlock - 1)) < bw; b0 += DS * NT) {
          unsigned long long aa[DS];
#pragma unroll
          for (int i = 0; i < DS; ++i) aa[i] = 0ull;
          for (int d0 = 0; d0 < nd; d0 += DU) {
            dvec_t v0[DU];
            unsigned long long qd[DU];
#pragma unroll
            for (int j = 0; j < DU; ++j) {
              const int d = d0 + j;
              qd[j] = 0ull;
              v0[j] = dvec_t(0u);
              if (d < nd) {
                qd[j] = d_q[d];
                v0[j] = *reinterpret_cast<const dvec_t*>(p.pool + d_off[d] + (b0 >> 2));
              }
            }
#pragma unroll
            for (int j = 0; j < DU; ++j) {
#pragma unroll
              for (int i = 0; i < DS; ++i) {
                const unsigned c = (v0[j][i >> 2] >> (8 * (i & 3))) & 0xffu;
                aa[i] += (unsigned long long)c * qd[j];
              }
            }
          }
#pragma unroll
          for (int i = 0; i < DS; ++i) {
            const int col = cooc_dense_song(b0 / DS, i);
            if (col < bw) acc[col] = store ? aa[i] : acc[col] + aa[i];
          }
        }
        __syncthreads();  // the sparse walk's atomics may hit any song
      }
      MR_STAMP(13);  // dense rows summed
      // 4 consecutive entries per thread and load (one 16-B load when they
      // lie in one segment, else entry by entry), U loads in flight
      constexpr int U = MR_COOC_U;
      // the thread's current row: entries up to ce at pool[co + e], weight cq
      int cur = -1, ce = 0;
      long long co = 0;
      unsigned long long cq = 0ull;
      const unsigned pad_x = (unsigned)lane << kCoocCntBits;
      for (int e0 = 4 * tid; e0 < total; e0 += 4 * U * NT) {
        unsigned x[U][4];
        unsigned long long wq[U][4];
#pragma unroll
        for (int j = 0; j < U; ++j) {
          const int e = e0 + j * 4 * NT;
#pragma unroll
          for (int i = 0; i < 4; ++i) { x[j][i] = pad_x; wq[j][i] = 0ull; }
          if (e < total) {
            while (e >= ce) { ++cur; ce = m_pre[cur + 1]; co = m_off[cur]; cq = m_q[cur]; }
            if (e + 3 < ce) {
              const u32x4_a4 v = *reinterpret_cast<const u32x4_a4*>(p.pool + co + e);
              x[j][0] = v.x; x[j][1] = v.y; x[j][2] = v.z; x[j][3] = v.w;
#pragma unroll
              for (int i = 0; i < 4; ++i) wq[j][i] = cq;
            } else {
#pragma unroll
              for (int i = 0; i < 4; ++i) {
                const int ei = e + i;
                if (ei < total) {
                  while (ei >= ce) { ++cur; ce = m_pre[cur + 1]; co = m_off[cur]; cq = m_q[cur]; }
                  x[j][i] = p.pool[co + ei];
                  wq[j][i] = cq;
                }
              }
            }
          }
        }
        // (no branch per entry: a slot past the list adds 0 at song lane < 64,
        // distinct per lane — inside acc, never read past bw)
#pragma unroll
        for (int j = 0; j < U; ++j)
#pragma unroll
          for (int i = 0; i < 4; ++i)
            atomicAdd(&acc[x[j][i] >> kCoocCntBits], (unsigned long long)(x[j][i] & kCoocCntMask) * wq[j][i]);
      }
      if (MR_CAND_PRE && p.cand && c0 + p.nseg >= t1) {  // the last pass: pass A's first scales
#pragma unroll
        for (int e = 0; e < MR_CAND_EB; ++e) {
          const int i = tid + e * NT;
          pre_rv[e] = i < bw ? p.rsq_c[blo + i] : 0.f;
        }
        have_rv = true;
      }
      __syncthreads();  // the next pass rewrites the descriptors
      MR_STAMP(14);  // sparse segments walked
    }
  } else {
  // stage 2: R neighbours per thread in flight; each segment's first kSeg
  // entries are loaded in the same batch, longer tails loop.
    const int* nv = p.nbr_v + (size_t)bu * p.cap;
    const long long* nq = p.nbr_q + (size_t)bu * p.cap;
    constexpr int R = MR_WIDE_R, kSeg = MR_WIDE_SEG;
    int cur = 0;
    auto load_list = [&](int k0, int (&v)[R], unsigned long long (&q)[R]) {
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const int k = k0 + r * NT;
        v[r] = -1;
        q[r] = 0ull;
        if (k < cnt) {
          while (cur + 1 < nch && cpre[cur + 1] <= k) ++cur;
          const size_t idx = (size_t)cur * p.chunk + (k - cpre[cur]);
          v[r] = nv[idx];
          q[r] = (unsigned long long)nq[idx];
        }
      }
    };
    walk_tile_lists<NT, R, kSeg, unsigned long long>(tid, cnt, load_list, p.toff + (size_t)tile * p.n_tr, p.tsongs,
                                                     [&](unsigned x, unsigned long long q) { atomicAdd(&acc[x], q); });
  }
  __syncthreads();
  MR_STAMP(2);

  long long* wk = reinterpret_cast<long long*>(smem_raw + L.wk);
  int* ws = reinterpret_cast<int*>(smem_raw + L.ws);
  long long* fk = reinterpret_cast<long long*>(smem_raw + L.fk);
  int* fs = reinterpret_cast<int*>(smem_raw + L.fs);
  const int k = KS == 10 ? 10 : p.topk;
  // top-k-only runs: the candidate-only tile top-k (p.cand: no dense row, no
  // min / max, 1 <= k <= NT / 16, bw <= kCandE * NT — set by the host)
  bool have = false;
#ifdef MR_STAMPS
  long long* sbp = p.stamps ? p.stamps + ((size_t)blockIdx.y * gridDim.x + blockIdx.x) * kStampSlots : nullptr;
#else
  long long* sbp = nullptr;
#endif
  if (p.cand) {
    have = wide_cand_topk<MODEL, NT, kCandE>(p, acc, heard, blo, bw, k, smem_raw + L.gm, wk, ws,
                                             min(256, NW * k), fk, fs, sbp, have_rv, pre_rv);
    MR_STAMP(6);
  }
  if (!have) {
  // epilogue: scores -> dense row segment; keys back into acc. 8 songs per
  // thread per batch (the per-song scale loads in flight together), and the
  // thread's best key (thread_best order: i = tid + NT j) tracked on the way
  // for the threshold top-k.
  const double inv_f = ldexp(1.0, -p.frac_bits);
  OutT* out = reinterpret_cast<OutT*>(p.dense_out) + (size_t)u * p.width + (blo - p.song_lo);
  long long mk = kKeyNone;
  int ms = INT_MAX;
  OutT lmn = (OutT)INFINITY, lmx = (OutT)-INFINITY;  // stored scores' min / max (p.mm_key)
  auto store = [&](int i, bool h, double score) {
    const OutT o = h ? (OutT)NAN : (OutT)score;
    out[i] = o;
    if (!h) {
      lmn = o < lmn ? o : lmn;
      lmx = o > lmx ? o : lmx;
    }
  };
  constexpr int EB = MR_WIDE_EB;
  int i_start = tid;
  if constexpr (kPF) {  // the prefetched songs first
#pragma unroll
    for (int e = 0; e < PF; ++e) {
      const int i = tid + e * NT;
      if (i >= bw) continue;
      const bool h = (heard[i >> 5] >> (i & 31)) & 1u;
      double score = (double)(long long)acc[i] * inv_f;
      score = score / scp[e];
      if (p.dense) store(i, h, score);
      const long long key = h ? kKeyNone : __double_as_longlong(score);
      acc[i] = (unsigned long long)key;
      if (key >= 0) take_if_before(mk, ms, key, blo + i);
    }
    i_start = tid + PF * NT;
  }
  for (int i0 = i_start; i0 < bw; i0 += EB * NT) {
    double sc[EB];
    unsigned long long av[EB];
#pragma unroll
    for (int e = 0; e < EB; ++e) {
      const int i = i0 + e * NT;
      sc[e] = 1.0;
      av[e] = 0ull;
      if (i < bw) {
        av[e] = acc[i];
        if (MODEL == MR_IBM) sc[e] = p.sqrt_c[blo + i];
      }
    }
#pragma unroll
    for (int e = 0; e < EB; ++e) {
      const int i = i0 + e * NT;
      if (i >= bw) continue;
      const bool h = (heard[i >> 5] >> (i & 31)) & 1u;
      double score = (double)(long long)av[e] * inv_f;
      if (MODEL == MR_IBM) score = score / sc[e];
      if (p.dense) store(i, h, score);
      const long long key = h ? kKeyNone : __double_as_longlong(score);
      acc[i] = (unsigned long long)key;
      if (key >= 0) take_if_before(mk, ms, key, blo + i);
    }
  }
  if (p.mm_key) {  // the wave's min / max, one atomic each per wave (ordered keys)
    double a = (double)lmn, b = (double)lmx;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      a = fmin(a, __shfl_xor(a, o, 64));
      b = fmax(b, __shfl_xor(b, o, 64));
    }
    if (lane == 0) {
      atomicMin(&p.mm_key[u], ordered_key(a));
      atomicMax(&p.mm_key[p.mm_n + u], ordered_key(b));
    }
  }
  if (p.topk <= 0) return;
  __syncthreads();
  MR_STAMP(3);

  // tile top-k: per-thread running lists (songs ascend per thread), per-wave
  // register tournament, then wave 0 over the NW wave lists.
  auto get_key = [&](int i, long long& key, int& song) { key = (long long)acc[i]; song = blo + i; };
  // (mk, ms): this thread's best key, from the epilogue
  const bool fast = !p.topk_lists && block_topk_threshold<NT>(bw, k, get_key, mk, ms, smem_raw + L.gm, wk, ws,
                                                              min(256, NW * k), fk, fs);
  MR_STAMP(6);
  if (!fast) {  // many ties at the threshold: per-thread running lists
    long long tk[KS];
    int ts[KS];
#pragma unroll
    for (int t = 0; t < KS; ++t) { tk[t] = kKeyNone; ts[t] = INT_MAX; }
    long long thr = kKeyNone;
    for (int i = tid; i < bw; i += NT) {
      const long long key = (long long)acc[i];
      if (key > thr) lane_list_insert(tk, ts, k, key, blo + i, thr);
    }
    wave_topk_regs<KS, true>(tk, ts, k, wk + w * k, ws + w * k);
    __syncthreads();
    if (w == 0) wave_merge_lists(NW, k, wk, ws, fk, fs);
    __syncthreads();
  }
  }  // !have
  MR_STAMP(7);
  MR_STAMP(8);
  MR_STAMP(4);
  if (p.n_tiles == 1) {
    for (int r = tid; r < k; r += NT) {
      const size_t o = (size_t)u * k + r;
      p.top_key[o] = fk[r];
      p.top_song[o] = fs[r];
      p.top_score[o] = fk[r] >= 0 ? __longlong_as_double(fk[r]) : (double)NAN;
    }
  } else {
    const size_t o = ((size_t)bu * p.n_tiles + tile) * k;  // batch-local user
    for (int r = tid; r < k; r += NT) {
      p.cand_key[o + r] = fk[r];
      p.cand_song[o + r] = fs[r];
    }
  }
  MR_STAMP(5);
  (void)lane;
}

// ---------------------------------------------------------------------------
// Co-listening index (ibm_route 2), built at the start of every ibm run: for
// index row r (a test-visible song s2 = row_song[r] with train listeners) and
// song tile t, the counts C[s2][s] = |L_tr(s2) ∩ L_tr(s)| (the distinct-user
// numerator of MR:232-235) of every song s of the tile with C > 0: a sparse
// segment of packed entries (tile-local s << kCoocCntBits) | C, or a dense one
// (every song's count, u16 / u32) when a third of the tile is non-zero.
// Heavy rows: one workgroup per row (k_cooc_build), its tiles in turn — LDS
// counters, the row's listeners walked over the tile-major train CSR like the
// two-hop stage 2 (weight 1), then the segment written at a running offset
// from row_base[r] (the host's bound on the row's words). Light rows: one
// workgroup per row with an LDS hash of its listeners' whole rows
// (k_cooc_light). Rows come sorted by listener count, heaviest first.
// ---------------------------------------------------------------------------
struct CoocParams {
  int n_tr, n_rows, n_tiles, block_songs, song_lo, song_hi;
  const int* toff;               // tile-major train CSR (ScoreParams.toff / tsongs)
  const unsigned short* tsongs;
  const long long* trs_off;      // train song -> users CSR (renumbered users, ascending)
  const int* trs_users;
  const int* row_song;           // [n_rows]
  const long long* row_base;     // [n_rows] first pool entry of the row
  unsigned* pool;
  long long* seg_off;            // [tile][row]
  int* seg_len;                  // [tile][row]
  const int* rows;               // the rows of this launch (index rows, heaviest first)
  // k_cooc_light: the shard's train rows (renumbered users, shard-local song ids)
  const long long* sr_off;
  const unsigned* sr_songs;
  const int* row_slots;          // [n_rows] a light row's hash slots | lane-group log2 (kLightGlogShift)
  int dense_div;                 // dense segment when non-zeros * dense_div >= tile songs (0: never)
  int force32;                   // 1: every heavy row as a >= 65536-listener row (tests: the saturated format)
  unsigned sat;                  // saturation of the dense count bytes (255; tests lower it)
  long long* stamps;             // diagnostic build: [workgroup][8] s_memrealtime at phase ends
  unsigned* row_nnz;             // [n_rows] non-zero counts of the row over the shard (zeroed per run)
  int n_big;                     // k_cooc_build: the first n_big rows of the launch one workgroup per
                                 //   (row, tile), each tile's segment at row_base + tile * tcap
  int tcap;                      //   (words per tile of those rows); the rest one workgroup per row
  // k_cooc_group: the tile groups (grp tiles each), and per (row, listener) a
  // record of lrec_words u32 words — word 0 the listener's first entry in
  // sr_songs, then u16 starts (relative to it) of every tile group g =
  // 0..n_grp — in the row's listener order, the row's first record at rdesc.z
  // (built at load by k_lrec from the per-user records of k_urec)
  int grp, n_grp;
  const unsigned* lrec;
  int lrec_words;
  // k_cooc_light*: per (light row, listener) the listener's shard-row range
  // [a, b) of sr_songs as two u32, in the row's order, the row's first at
  // rdesc.z (built at load by k_llrec): one 8-B load instead of the listener
  // id and then its two sr_off words
  const unsigned* llrec;
  long long* lstamps;            // diagnostic build: [light row of the launch][8] (k_cooc_light*)
  // k_cooc_light* / k_cooc_group: the launch's rows as {row, row_slots value,
  // first listener in trs_users, listeners} (one load instead of rows ->
  // row_slots / row_song -> trs_off: three dependent ones)
  const int4* rdesc;
};

template <bool P16>
__host__ __device__ inline int cooc_words(int bs) { return P16 ? (bs + 1) / 2 : bs; }
// songs first touched during the walk (u16, tile-local): a sparse segment of
// at most this many non-zeros is written from the list, without a scan of the
// tile (sized so 4 / 2 workgroups of a 19,456-song tile still fit one CU)
template <bool P16>
__host__ __device__ constexpr int cooc_list_cap() { return P16 ? 960 : 1984; }
template <bool P16>
__host__ __device__ inline int cooc_build_lds(int bs) {
  return align16(cooc_words<P16>(bs) * 4) + 16 * 4 + 32 + cooc_list_cap<P16>() * 2;
}

// Light rows (k_cooc_light): an LDS hash table of packed slots
// ((shard-local song + 1) << kLightCntBits) | count, at most kLightSlots;
// a row is light when its entry bound fits half the slots, its listener count
// fits kLightCntBits and the shard's songs fit the key bits.
constexpr int kLightCntBits = 12;
constexpr unsigned kLightCntMask = (1u << kLightCntBits) - 1u;
constexpr int kLightSlots = 32768;
constexpr int kLightMaxTiles = 256;
constexpr int kLightMaxWidth = (1 << (32 - kLightCntBits)) - 2;
// row_slots of a light row as uploaded: the table's slots (a power of 2 <= 2^15)
// | log2(lanes per listener) << kLightGlogShift (rows_walk)
constexpr int kLightGlogShift = 24;
constexpr int kLightSlotsMask = (1 << kLightGlogShift) - 1;
// Light rows run in the smallest of four table sizes that holds them (the
// rows are latency-bound, so smaller tables = more workgroups per CU):
// 4096 slots / 256 threads (7 per CU), 8192 / 512 (4), 16384 / 512 (2),
// 32768 / 1024 (1). Tier 0 is the largest (launched first).
constexpr int kLightTiers = 6;     // tiers 4, 5 (2048 / 1024 slots): one wave per row (k_cooc_light_wave)
#ifndef MR_WAVE_ROWS
#define MR_WAVE_ROWS 1  // C4 8x1: 5.95 vs 6.03 ms at 4, 5.99 at 2 (profiles/r04/s54, s55)
#endif
constexpr int kWaveRowsPerBlock = MR_WAVE_ROWS;
constexpr int kWaveMaxTiles = 64;  // the wave tiers' per-row tile counters
__host__ __device__ constexpr int light_tier_slots(int t) { return 32768 >> t; }
// a table of S slots holds a row whose entry bound is at most S * 4/5 (the
// bound counts every listener's songs; the distinct ones are far fewer)
__host__ __device__ constexpr long long light_bound_max(long long slots) { return slots * 4 / 5; }
// k_cooc_light's LDS layout (byte offsets): the hash table, then the per-tile
// counts and cursors of the emission.
template <int NT, int SMAX>
struct LightLds {
  static constexpr int tab = 0;
  static constexpr int tcnt = tab + SMAX * 4;
  static constexpr int tpos = tcnt + kLightMaxTiles * 4;
  static constexpr int total = tpos + kLightMaxTiles * 4;
  static_assert(total % 16 == 0, "k_cooc_light LDS size");
};
template <int NT, int SMAX>
__host__ __device__ constexpr int cooc_light_lds() {
  return LightLds<NT, SMAX>::total;
}

// A dense segment's count bytes (cooc_dense_song order, saturated at sat)
// at out[0, dwords), the excess (count - sat) of larger counts as entries
// from out[dwords] on (*tail: their LDS counter). Lanes read consecutive
// songs' counters and store consecutive chunks (CHUNK) or words.
template <int NT, bool CHUNK, typename CountOf>
__device__ __forceinline__ void cooc_write_dense(unsigned* out, int bw, int dwords, unsigned sat, int* tail,
                                                 CountOf&& count_of) {
  constexpr int WPC = kDenseDS / 4;  // words per chunk
  if constexpr (CHUNK) {  // a whole chunk per thread, one store (k_cooc_group: 17.85 vs 18.27 ms at C4)
    typedef unsigned chunk_t __attribute__((ext_vector_type(WPC)));
    for (int c = threadIdx.x; c < dwords / WPC; c += NT) {
      chunk_t v = chunk_t(0u);
#pragma unroll
      for (int i = 0; i < kDenseDS; ++i) {
        const int col = cooc_dense_song(c, i);
        const unsigned n = col < bw ? count_of(col) : 0u;
        v[i >> 2] |= min(n, sat) << (8 * (i & 3));
        if (n > sat) out[dwords + atomicAdd(tail, 1)] = ((unsigned)col << kCoocCntBits) | (n - sat);
      }
      reinterpret_cast<chunk_t*>(out)[c] = v;
    }
    return;
  }
  // a word per thread (k_cooc_build: the chunk's registers spilled, 1.04 vs 0.71 ms)
  for (int x = threadIdx.x; x < dwords; x += NT) {  // word x: bytes 4 (x % WPC) .. +3 of chunk x / WPC
    const int c = x / WPC, i0 = 4 * (x % WPC);
    unsigned wv = 0u;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int col = cooc_dense_song(c, i0 + j);
      const unsigned n = col < bw ? count_of(col) : 0u;
      wv |= min(n, sat) << (8 * j);
      if (n > sat) out[dwords + atomicAdd(tail, 1)] = ((unsigned)col << kCoocCntBits) | (n - sat);
    }
    out[x] = wv;
  }
}

// One finished tile of an index row (counters in LDS, count_of(i) = song i's
// count, `total` non-zeros, the first `cap` of them listed in `touched`)
// written at pool[off]: a dense segment (a count byte per song, saturated at
// p.sat, then the excess entries) when total * dense_div >= bw, else a sparse
// one (from the touched list when it holds every non-zero, else a song-ordered
// compaction). Sets seg_off / seg_len of (tile, r); returns the segment's
// words. Called by the whole workgroup (barriers inside); *s_tail is zero on
// entry; the caller synchronises before the counters or s_scan are reused.
template <int NT, typename CountOf>
__device__ __forceinline__ int cooc_emit_tile(const CoocParams& p, int r, int tile, int bw, long long off, int total,
                                              const unsigned short* touched, int kCap, int* s_tail, int* s_scan,
                                              CountOf&& count_of) {
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const unsigned long long below = lane ? (~0ull >> (64 - lane)) : 0ull;
    // Dense segment when at least a third of the tile's songs are non-zero:
    // a count byte per song (no index, no atomics on the consumer side; the
    // rare counts above sat carried by excess entries). Segments are whole
    // 16-B words.
    const bool dense = p.dense_div > 0 && (long long)total * p.dense_div >= bw;
    const int dwords = cooc_dense_words(bw);  // a dense segment's u8 count words, whole 16-B words
    int words = (total + 3) & ~3;
    unsigned* out = p.pool + off;
    if (dense) {
      // every song's count as a byte saturated at sat (255), the excess
      // (count - sat) of the few larger counts as sparse entries after them
      // (own counter: s_nz is still being read for `total` by other waves)
      cooc_write_dense<NT, false>(out, bw, dwords, p.sat, s_tail, count_of);
      __syncthreads();
      const int tail = *s_tail;
      words = (dwords + tail + 3) & ~3;
      if (tid == 0) {
        p.seg_off[(size_t)tile * p.n_rows + r] = off;
        p.seg_len[(size_t)tile * p.n_rows + r] = kCoocDenseTail - tail;
      }
    } else if (total <= kCap) {  // the touched list holds every non-zero song
      if (tid == 0) {
        p.seg_off[(size_t)tile * p.n_rows + r] = off;
        p.seg_len[(size_t)tile * p.n_rows + r] = total;
      }
      for (int k = tid; k < total; k += NT) {
        const unsigned x = touched[k];
        out[k] = (x << kCoocCntBits) | count_of((int)x);
      }
    } else {  // compaction: wave w owns songs [wb, we); its run of the segment is
              // reserved by one LDS atomic (*s_tail is free here: no excess
              // entries), so the waves' runs land in arrival order (order
              // inside a segment is unspecified) and no workgroup barrier
      if (tid == 0) {
        p.seg_off[(size_t)tile * p.n_rows + r] = off;
        p.seg_len[(size_t)tile * p.n_rows + r] = total;
      }
      const int q4 = (bw + NT - 1) / NT * 64;
      const int wb = min(bw, w * q4), we = min(bw, wb + q4);
      int nz = 0;
      for (int i0 = wb; i0 < we; i0 += 64) {
        const int i = i0 + lane;
        nz += __popcll(__ballot(i < we && count_of(i) != 0u));
      }
      int base = 0;
      if (lane == 0 && nz > 0) base = atomicAdd(s_tail, nz);
      base = wave_lane(base, 0);
      for (int i0 = wb; i0 < we; i0 += 64) {
        const int i = i0 + lane;
        const unsigned c = i < we ? count_of(i) : 0u;
        const unsigned long long m = __ballot(c != 0u);
        if (c) out[base + __popcll(m & below)] = ((unsigned)i << kCoocCntBits) | c;
        base += __popcll(m);
      }
    }
    return words;
}

// P16: two u16 counters per LDS word (rows with < 65536 listeners: half the
// LDS, twice the workgroups per CU), else one u32 counter per song.
template <int NT, bool P16>
__global__ __launch_bounds__(NT, (P16 ? 4 : 2) * NT / 256) void k_cooc_build(CoocParams p) {
  extern __shared__ __align__(16) unsigned char smem_raw[];
  const int bs = p.block_songs;
  unsigned* cnt = reinterpret_cast<unsigned*>(smem_raw);
  int* s_scan = reinterpret_cast<int*>(smem_raw + align16(cooc_words<P16>(bs) * 4));
  int* s_nz = s_scan + 16;      // songs first touched in this tile
  int* s_tail = s_scan + 17;    // excess entries of this tile's dense segment
  unsigned short* touched = reinterpret_cast<unsigned short*>(s_scan + 16 + 8);
  constexpr int kCap = cooc_list_cap<P16>();
  auto count_of = [&](int i) -> unsigned {
    if constexpr (P16) return (cnt[i >> 1] >> ((i & 1) << 4)) & 0xffffu;
    else return cnt[i];
  };
  // big rows: one workgroup per (row, tile) at a fixed offset; the others:
  // one workgroup per row, its tiles in turn at a running offset
  const int nbt = p.n_big * p.n_tiles;
  const bool big = (int)blockIdx.x < nbt;
  const int ri = big ? (int)blockIdx.x / p.n_tiles : p.n_big + ((int)blockIdx.x - nbt);
  const int r = p.rows[ri];
  const int t_begin = big ? (int)blockIdx.x - ri * p.n_tiles : 0;
  const int t_end = big ? t_begin + 1 : p.n_tiles;
  const int tid = threadIdx.x;
  long long* sb = p.stamps ? p.stamps + (size_t)blockIdx.x * 8 : nullptr;
  stamp_rt(sb, 0);
  const int s2 = p.row_song[r];
  const long long a = p.trs_off[s2];
  const int n = (int)(p.trs_off[s2 + 1] - a);
  const int* lst = p.trs_users + a;
  constexpr int R = MR_COOC_R, kSeg = MR_WIDE_SEG;
  auto load_list = [&](int k0, int (&v)[R], unsigned (&q)[R]) {
#pragma unroll
    for (int j = 0; j < R; ++j) {
      const int k = k0 + j * NT;
      v[j] = k < n ? lst[k] : -1;
      q[j] = 1u;
    }
  };
  // the row's tiles one after another: its segments are laid out in tile
  // order from row_base[r] (no reservation atomics; the capacity bound holds)
  long long off = p.row_base[r] + (long long)t_begin * p.tcap;  // (t_begin = 0 unless big)
  unsigned row_nz = 0u;
  for (int tile = t_begin; tile < t_end; ++tile) {
    const int blo = p.song_lo + tile * bs;
    const int bw = min(p.song_hi, blo + bs) - blo;
    for (int i = tid; i < cooc_words<P16>(bw); i += NT) cnt[i] = 0u;
    if (tid == 0) { *s_nz = 0; *s_tail = 0; }
    __syncthreads();
    walk_tile_lists<NT, R, kSeg, unsigned>(tid, n, load_list, p.toff + (size_t)tile * p.n_tr, p.tsongs,
                                           [&](unsigned x, unsigned) {
                                             bool first;
                                             if constexpr (P16) {
                                               const unsigned sh = (x & 1) << 4;
                                               first = ((atomicAdd(&cnt[x >> 1], 1u << sh) >> sh) & 0xffffu) == 0u;
                                             } else {
                                               first = atomicAdd(&cnt[x], 1u) == 0u;
                                             }
                                             if (first) {
                                               const int k = atomicAdd(s_nz, 1);
                                               if (k < kCap) touched[k] = (unsigned short)x;
                                             }
                                           });
    __syncthreads();
    if (tile == t_begin) stamp_rt(sb, 1);  // the first tile's walk done
    const int total = *s_nz;
    const int words = cooc_emit_tile<NT>(p, r, tile, bw, off, total, touched, kCap, s_tail, s_scan, count_of);
    off += words;
    row_nz += (unsigned)total;
    __syncthreads();  // the next tile rezeroes the counters
    if (tile == t_begin) {  // the first tile emitted (one pass: slot 3 = slot 2)
      stamp_rt(sb, 2);
      stamp_rt(sb, 3);
    }
  }
  if (tid == 0 && row_nz) atomicAdd(&p.row_nnz[r], row_nz);
  // slots 5-7: big, listeners, -1 = this kernel (k_cooc_group writes its group count there)
  stamp_rt(sb, 4);
  stamp_val(sb, 5, big ? 1 : 0);
  stamp_val(sb, 6, n);
  stamp_val(sb, 7, -1);
}

// Insert one shard-local song into a light row's LDS hash table (packed
// ((song + 1) << kLightCntBits) | count slots, open addressing, linear probing,
// CAS insert; S = mask + 1 slots, hash = the top log2(S) bits of key * φ).
#ifndef MR_LIGHT_INSERT
#define MR_LIGHT_INSERT 0  // 0: slot by slot; 1: 4-slot probes (one 16-B LDS read per step: slower,
                           // r04 session 4: C4 8x1 rank 8.29 vs 7.07 ms);
                           // 8, 9: timing-only stubs (wrong counts: no probing / a bare add)
#endif
__device__ __forceinline__ void light_insert(unsigned* tab, unsigned mask, int sh, unsigned key) {
  const unsigned tag = (key + 1u) << kLightCntBits;
  unsigned h = (key * 2654435761u) >> sh;
#if MR_LIGHT_INSERT == 9
  atomicAdd(&tab[h], 1u);
  (void)tag;
  (void)mask;
#elif MR_LIGHT_INSERT == 8
  unsigned x = tab[h];
  if (x == 0u) x = atomicCAS(&tab[h], 0u, tag | 1u);
  if (x != 0u) atomicAdd(&tab[h], 1u);
  (void)mask;
#elif MR_LIGHT_INSERT == 1
  // linear probing over aligned groups of 4 slots, read 16 B at a time: the
  // same probe order as slot by slot (home slot first, wrapping), so a key is
  // always found before the first empty slot after its home; about a quarter
  // of the dependent LDS reads on long clusters
  unsigned g = h & ~3u;
  int i = (int)(h & 3u);
  for (;;) {
    const uint4 q = *reinterpret_cast<const uint4*>(tab + g);
    const unsigned v[4] = {q.x, q.y, q.z, q.w};
    for (; i < 4; ++i) {
      unsigned x = v[i];
      if (x == 0u) {
        x = atomicCAS(&tab[g + i], 0u, tag | 1u);
        if (x == 0u) return;
      }
      if ((x & ~kLightCntMask) == tag) {
        atomicAdd(&tab[g + i], 1u);
        return;
      }
    }
    g = (g + 4u) & mask;
    i = 0;
  }
#else
  for (;;) {
    unsigned x = tab[h];
    if (x == 0u) {
      x = atomicCAS(&tab[h], 0u, tag | 1u);
      if (x == 0u) return;
    }
    if ((x & ~kLightCntMask) == tag) {
      atomicAdd(&tab[h], 1u);
      return;
    }
    h = (h + 1u) & mask;
  }
#endif
}

// An index row's listener walk, by listener: the n_lanes lanes form groups of
// G = 2^glog lanes (G <= 64: a group never spans two waves); group i takes the
// listeners i, i + n_lanes / G, ... of the row and its G lanes read the
// listener's entries sr_songs[a .. b) (range(v, a, b): the whole shard row
// for light rows, a tile group's part of it for k_cooc_group; sorted, shard-
// local ids) in 16-B chunks, lane j the chunks at 4j, 4j + 4G, ..., every
// entry inserted: ins(k, m) takes a lane's keys of two chunks, k[0 .. m). G is chosen per row on the host from its entries per
// listener (mr_load: about 6 entries per lane). Software-pipelined: the next
// listener's row bounds and the id after it are loaded while the current
// row's first two chunks are inserted. No listener descriptors in LDS, no
// block scans, no barriers — the flattened walk this replaced advanced every
// lane through the chunk's descriptors one LDS read at a time, a serial chain
// of ~NT / (entries per listener) reads per entry (C4 8x1: 12 entries per
// listener, 1024-lane chunks, 3.0 ms for tier 0). sr_songs is padded by 4
// entries, so a chunk's 16-B load never leaves the buffer.
#ifndef MR_WALK_R
#define MR_WALK_R 2  // listeners per lane group per iteration of rows_walk (loads issued together)
#endif
template <typename Ids, typename Range, typename Ins>
__device__ __forceinline__ void rows_walk(int lane_id, int n_lanes, int glog, Ids&& lst, int n, Range&& range,
                                          const unsigned* sr_songs, Ins&& ins) {
  constexpr int R = MR_WALK_R;
  const int G = 1 << glog;
  const int grp = lane_id >> glog, j = lane_id & (G - 1);
  const int step = n_lanes >> glog;
  const int stride = step * R;  // listeners per iteration of all groups
  auto chunk = [&](long long x, long long b, u32x4_a4& c) -> int {
    const long long m = b - x;
    c = u32x4_a4{0u, 0u, 0u, 0u};
    if (m <= 0) return 0;
    c = *reinterpret_cast<const u32x4_a4*>(sr_songs + x);
    return m >= 4 ? 4 : (int)m;
  };
  // the listener's keys of this iteration as one batch: k[0 .. m) valid (a
  // chunk's valid entries are a prefix, and the second chunk has entries only
  // when the first is full, so the two chunks' valid keys are a prefix of 8)
  auto put2 = [&](const u32x4_a4& c0, int m0, const u32x4_a4& c1, int m1) {
    const unsigned k[8] = {c0.x, c0.y, c0.z, c0.w, c1.x, c1.y, c1.z, c1.w};
    ins(k, m0 + m1);
  };
  // iteration i: listeners grp + i * stride + r * step, r < R; the next
  // iteration's row ranges and the one after's ids are loaded while this
  // iteration's first chunks are inserted
  long long a0[R], b0[R];
  int v1[R];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const int l = grp + r * step, l1 = l + stride;
    a0[r] = b0[r] = 0;
    if (l < n) range(lst(l), a0[r], b0[r]);
    v1[r] = l1 < n ? lst(l1) : -1;
  }
  for (int l0 = grp; l0 < n; l0 += stride) {
    u32x4_a4 c[R][2];
    int m[R][2];
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const long long x0 = a0[r] + 4 * j;
      m[r][0] = chunk(x0, b0[r], c[r][0]);
      m[r][1] = chunk(x0 + 4 * G, b0[r], c[r][1]);
    }
    long long a1[R], b1[R];
    int v2[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
      a1[r] = b1[r] = 0;
      if (v1[r] >= 0) range(v1[r], a1[r], b1[r]);
      const int l2 = l0 + 2 * stride + r * step;
      v2[r] = l2 < n ? lst(l2) : -1;
    }
#pragma unroll
    for (int r = 0; r < R; ++r) put2(c[r][0], m[r][0], c[r][1], m[r][1]);
#pragma unroll
    for (int r = 0; r < R; ++r)
      for (long long x = a0[r] + 4 * j + 8 * G; x < b0[r]; x += 8 * G) {
        u32x4_a4 c0, c1;
        const int m0 = chunk(x, b0[r], c0);
        const int m1 = chunk(x + 4 * G, b0[r], c1);
        put2(c0, m0, c1, m1);
      }
#pragma unroll
    for (int r = 0; r < R; ++r) {
      a0[r] = a1[r];
      b0[r] = b1[r];
      v1[r] = v2[r];
    }
  }
}

// A lane's batch of keys (k[0 .. m), m <= 8) into a light row's table as a
// queue: each step probes ONE slot for the key at the head, a finished key
// pops and the next one starts at its home slot the very next step. The wave
// therefore runs max over lanes of (Σ probes of the lane's keys) steps, not
// Σ over keys of (max over lanes of its probes), the per-key loop's cost on
// long linear-probing clusters (C4 8x1: ~30 of a light row's ~40 us walk).
__device__ __forceinline__ void light_insert_queue(unsigned* tab, unsigned mask, int sh, const unsigned (&k)[8],
                                                   int m) {
#if MR_LIGHT_INSERT >= 8
  for (int i = 0; i < 8; ++i)
    if (i < m) light_insert(tab, mask, sh, k[i]);
#else
  if (m <= 0) return;
  unsigned q[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) q[i] = k[i];
  unsigned tag = (q[0] + 1u) << kLightCntBits;
  unsigned h = (q[0] * 2654435761u) >> sh;
  int left = m;
  while (left > 0) {
#if MR_LIGHT_CAS1
    // the CAS first: a new key (most keys: counts of light rows are mostly 1)
    // takes one LDS round trip instead of a read and then the CAS
    unsigned x = atomicCAS(&tab[h], 0u, tag | 1u);
    bool done = x == 0u;
#else
    unsigned x = tab[h];
    bool done = false;
    if (x == 0u) {
      x = atomicCAS(&tab[h], 0u, tag | 1u);
      done = x == 0u;
    }
#endif
    if (!done && (x & ~kLightCntMask) == tag) {
      atomicAdd(&tab[h], 1u);
      done = true;
    }
    if (done) {
      --left;
#pragma unroll
      for (int i = 0; i < 7; ++i) q[i] = q[i + 1];
      tag = (q[0] + 1u) << kLightCntBits;
      h = (q[0] * 2654435761u) >> sh;
    } else {
      h = (h + 1u) & mask;
    }
  }
#endif
}

// range of rows_walk: listener v's whole shard row
struct ShardRow {
  const unsigned* rec;  // the row's first (a, b) record
  __device__ __forceinline__ void operator()(int x, long long& a, long long& b) const {
    const uint2 r = reinterpret_cast<const uint2*>(rec)[x];
    a = r.x;
    b = r.y;
  }
};

// Light index rows: one workgroup per row (instead of one per (row, tile)).
// The row's listeners' whole shard rows (sr_off / sr_songs) are walked by
// listener (rows_walk: groups of lanes per listener) into an LDS hash table
// of counts (light_insert), then the table is emitted tile by tile: per-tile
// counts, their prefix -> the row's segment of every tile (seg_off / seg_len,
// empty tiles included), entries placed by LDS cursors (order inside a
// segment is arbitrary; the consumer's sums are order-free).
template <int NT, int SMAX>
__global__ __launch_bounds__(NT) void k_cooc_light(CoocParams p) {
  extern __shared__ __align__(16) unsigned char smem_raw[];
  using Lay = LightLds<NT, SMAX>;
  unsigned* tab = reinterpret_cast<unsigned*>(smem_raw + Lay::tab);
  int* tcnt = reinterpret_cast<int*>(smem_raw + Lay::tcnt);
  int* tpos = reinterpret_cast<int*>(smem_raw + Lay::tpos);
  const int4 rd = p.rdesc[blockIdx.x];  // {row, slots | lane-group log2, listener list start, listeners}
  const int r = rd.x;
  const int tid = threadIdx.x;
  long long* sb = p.lstamps ? p.lstamps + (size_t)blockIdx.x * 8 : nullptr;
  stamp_rt(sb, 0);
  const int S = rd.y & kLightSlotsMask;
  const unsigned mask = (unsigned)S - 1u;
  const int sh = 32 - __builtin_ctz((unsigned)S);  // multiplicative hash: top log2(S) bits
  for (int i = tid; 4 * i < S; i += NT) reinterpret_cast<uint4*>(tab)[i] = make_uint4(0u, 0u, 0u, 0u);  // (S: a power of 2 >= 1024)
  for (int i = tid; i < p.n_tiles; i += NT) { tcnt[i] = 0; tpos[i] = 0; }
  const int n = rd.w;
  const unsigned* lst = p.llrec + 2 * (size_t)(unsigned)rd.z;  // the row's listeners' ranges
  __syncthreads();  // the table and the tile counters are zero
  stamp_rt(sb, 1);
  rows_walk(tid, NT, rd.y >> kLightGlogShift, [](int l) { return l; }, n, ShardRow{lst}, p.sr_songs,
            [&](const unsigned (&k)[8], int m) { light_insert_queue(tab, mask, sh, k, m); });
  __syncthreads();
  stamp_rt(sb, 2);
  // emit: per-tile counts, segment offsets, then the entries
  const int bs = p.block_songs;
  const float inv_bs = 1.0f / (float)bs;
  for (int i = tid; i < S; i += NT) {
    const unsigned x = tab[i];
    if (x) atomicAdd(&tcnt[tile_of((int)((x >> kLightCntBits) - 1u), bs, inv_bs)], 1);
  }
  __syncthreads();
  stamp_rt(sb, 3);
  if (tid < 64) {  // prefix over <= kLightMaxTiles tiles by one wave
    int run = 0;
    if (tid == 0) {
      int nz = 0;
      for (int t = 0; t < p.n_tiles; ++t) nz += tcnt[t];
      p.row_nnz[r] = (unsigned)nz;
    }
    for (int t0 = 0; t0 < p.n_tiles; t0 += 64) {
      const int t = t0 + tid;
      const int c = t < p.n_tiles ? tcnt[t] : 0;
      const int inc = wave_incl_scan(c);
      if (t < p.n_tiles) {
        tpos[t] = run + inc - c;
        p.seg_off[(size_t)t * p.n_rows + r] = p.row_base[r] + run + inc - c;
        p.seg_len[(size_t)t * p.n_rows + r] = c;
      }
      run += wave_lane(inc, 63);
    }
  }
  __syncthreads();
  unsigned* out = p.pool + p.row_base[r];
  for (int i = tid; i < S; i += NT) {
    const unsigned x = tab[i];
    if (x) {
      const int key = (int)((x >> kLightCntBits) - 1u);
      const int t = tile_of(key, bs, inv_bs);
      const int pos = atomicAdd(&tpos[t], 1);
      out[pos] = ((unsigned)(key - t * bs) << kCoocCntBits) | (x & kLightCntMask);
    }
  }
  __syncthreads();
  stamp_rt(sb, 4);
  stamp_val(sb, 5, n);
  stamp_val(sb, 6, S);
  stamp_val(sb, 7, NT);
}

// The smallest light rows, one wave per row (kWaveRowsPerBlock rows per
// workgroup, each wave with its own table and tile counters in LDS): the same
// walk, hash and emission as k_cooc_light with wave scans and no workgroup
// barriers, so 16 rows per CU are in flight (the rows are latency-bound).
template <int SW>
__host__ __device__ constexpr int cooc_wave_bytes() { return SW * 4 + 2 * kWaveMaxTiles * 4; }
template <int SW>
__global__ __launch_bounds__(64 * kWaveRowsPerBlock) void k_cooc_light_wave(CoocParams p, int n_launch) {
  extern __shared__ __align__(16) unsigned char smem_raw[];
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int ri = blockIdx.x * kWaveRowsPerBlock + w;
  if (ri >= n_launch) return;  // the whole wave (no workgroup barrier below)
  unsigned char* base = smem_raw + (size_t)w * cooc_wave_bytes<SW>();
  unsigned* tab = reinterpret_cast<unsigned*>(base);
  int* tcnt = reinterpret_cast<int*>(tab + SW);
  int* tpos = tcnt + kWaveMaxTiles;
  const int4 rd = p.rdesc[ri];
  const int r = rd.x;
  long long* sb = p.lstamps ? p.lstamps + (size_t)ri * 8 : nullptr;
  stamp_rt_wave(sb, 0);
  const int S = rd.y & kLightSlotsMask;
  const unsigned mask = (unsigned)S - 1u;
  const int sh = 32 - __builtin_ctz((unsigned)S);
  for (int i = lane; 4 * i < S; i += 64) reinterpret_cast<uint4*>(tab)[i] = make_uint4(0u, 0u, 0u, 0u);
  for (int i = lane; i < p.n_tiles; i += 64) { tcnt[i] = 0; tpos[i] = 0; }
  const int n = rd.w;
  const unsigned* lst = p.llrec + 2 * (size_t)(unsigned)rd.z;  // the row's listeners' ranges
  wave_lds_sync();  // the table and the tile counters are zero
  stamp_rt_wave(sb, 1);
  rows_walk(lane, 64, rd.y >> kLightGlogShift, [](int l) { return l; }, n, ShardRow{lst}, p.sr_songs,
            [&](const unsigned (&k)[8], int m) { light_insert_queue(tab, mask, sh, k, m); });
  wave_lds_sync();
  stamp_rt_wave(sb, 2);
  const int bs = p.block_songs;
  const float inv_bs = 1.0f / (float)bs;
  for (int i = lane; i < S; i += 64) {
    const unsigned x = tab[i];
    if (x) atomicAdd(&tcnt[tile_of((int)((x >> kLightCntBits) - 1u), bs, inv_bs)], 1);
  }
  wave_lds_sync();
  {
    int run = 0;
    for (int t0 = 0; t0 < p.n_tiles; t0 += 64) {
      const int t = t0 + lane;
      const int c = t < p.n_tiles ? tcnt[t] : 0;
      const int inc = wave_incl_scan(c);
      if (t < p.n_tiles) {
        tpos[t] = run + inc - c;
        p.seg_off[(size_t)t * p.n_rows + r] = p.row_base[r] + run + inc - c;
        p.seg_len[(size_t)t * p.n_rows + r] = c;
      }
      run += wave_lane(inc, 63);
    }
    if (lane == 0) p.row_nnz[r] = (unsigned)run;
  }
  wave_lds_sync();
  stamp_rt_wave(sb, 3);  // tile counts and offsets done
  unsigned* out = p.pool + p.row_base[r];
  for (int i = lane; i < S; i += 64) {
    const unsigned x = tab[i];
    if (x) {
      const int key = (int)((x >> kLightCntBits) - 1u);
      const int t = tile_of(key, bs, inv_bs);
      const int pos = atomicAdd(&tpos[t], 1);
      out[pos] = ((unsigned)(key - t * bs) << kCoocCntBits) | (x & kLightCntMask);
    }
  }
  wave_lds_sync();
  stamp_rt_wave(sb, 4);
  stamp_val(sb, 5, n, true);
  stamp_val(sb, 6, S, true);
  stamp_val(sb, 7, 64, true);
}

// k_cooc_group: the heavy rows under 65536 listeners, a tile GROUP per pass —
// grp tiles' u16 counters (two per LDS word) side by side in LDS, so one walk
// of the row's listeners serves grp tiles. Each listener's entries of the
// group are one contiguous run of its shard row (user-major sr_songs: the
// songs ascend, so tiles do), found through the (row, listener) record (lrec:
// 16 contiguous bytes per listener of the row hold its base and every group's
// start; round 4 read a listener id and then a per-user record line, 10 GB of
// lines per C4 step for ~0.1 GB used, profiles/r05/group_lines_c4.json).
// k_cooc_build's walk
// gathered, per (row, tile, listener), a toff pair and a tile segment from two
// tile-major arrays: two whole lines for ~5 entries, 20 times per listener at
// C4 (107 GB of fetches per step for ~6 GB of entries).
constexpr int kMaxGroupTiles = 8;
__host__ __device__ inline int cooc_group_lds(int bs, int g) {
  // counters; per tile: excess entries (+ spare words); per (tile, wave): non-zeros
  return align16(g * bs * 2) + 3 * kMaxGroupTiles * 4 + kMaxGroupTiles * 16 * 4;
}

// Bit 15 / bit 31 of the result set iff the low / high u16 half of x is non-zero
// (the low 15 bits + 0x7fff carry into bit 15; OR-ing x catches bit 15 itself).
__device__ __forceinline__ unsigned nz_halves(unsigned x) {
  return (((x & 0x7fff7fffu) + 0x7fff7fffu) | x) & 0x80008000u;
}
// Non-zero u16 counters among the 8 of a 16-B chunk. k_cooc_group zeroes the
// counters up to the last chunk's end, so a tile's padding past its bw songs
// counts nothing.
__device__ __forceinline__ int nz_pairs8(const uint4& w) {
  return __popc(nz_halves(w.x) | (nz_halves(w.y) >> 1) | (nz_halves(w.z) >> 2) | (nz_halves(w.w) >> 3));
}

// All tiles [t0, t0 + ntg) of a k_cooc_group pass written from their u16
// counters (tile k's at cnt + k * bs / 2): pass A counts every tile's
// non-zeros per WAVE (16-B LDS chunks, the wave's sum to s_wcnt[k][w], no
// atomics), ONE barrier, then every thread derives the same segment offsets
// from those sums — a sparse segment its non-zeros, a dense one its count
// bytes plus room for as many excess entries as it has non-zeros (an upper
// bound: within the row's pool bound, see mr_load), so no tile waits for the
// previous tile's excess count — and its wave's start inside each segment
// (the waves before it: pass B visits the same chunks as pass A); pass B
// writes every tile (dense: count bytes + excess entries; sparse: each wave
// compacts at DPP-scanned prefixes from its own start, no LDS cursor), ONE
// barrier, and thread 0 records the segments. s_tail [ntg] is zero on entry;
// every wave writes its s_wcnt entries. Advances *off (rows at a running
// offset) and *row_nz. (The per-wave starts replace an LDS atomic on one
// cursor word per wave and chunk row, which the 16 waves serialized on.)
template <int NT>
__device__ __forceinline__ void cooc_emit_group16(const CoocParams& p, int r, bool big, int t0, int ntg, int bs,
                                                  int width, const unsigned* cnt, int* s_wcnt, int* s_tail,
                                                  long long* off, unsigned* row_nz, long long* sb = nullptr) {
  constexpr int NW = NT / 64;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  for (int k = 0; k < ntg; ++k) {
    const int bw = min(width, (t0 + k + 1) * bs) - (t0 + k) * bs;
    const uint4* cv = reinterpret_cast<const uint4*>(cnt + (size_t)k * (bs >> 1));
    const int nch = (bw + 7) >> 3;
    int nz = 0;
    for (int c = tid; c < nch; c += NT) nz += nz_pairs8(cv[c]);
    const int ws = wave_lane(wave_incl_scan(nz), 63);
    if (lane == 0) s_wcnt[k * NW + w] = ws;
  }
  __syncthreads();
  stamp_rt(sb, 3);  // (diagnostic build: pass A of the first group)
  // tile k's non-zeros, and this wave's first entry among them (lane x reads
  // wave x's count; one scan, two lane reads)
  const int ws_id = __builtin_amdgcn_readfirstlane(w);
  auto tile_counts = [&](int k, int& total, int& wbase) {
    const int c = lane < NW ? s_wcnt[k * NW + lane] : 0;
    const int inc = wave_incl_scan(c);
    total = wave_lane(inc, 63);
    wbase = wave_lane(inc - c, ws_id);
  };
  long long o = *off;
  for (int k = 0; k < ntg; ++k) {
    const int tile = t0 + k;
    const int bw = min(width, (tile + 1) * bs) - tile * bs;
    int total, wbase;
    tile_counts(k, total, wbase);
    const bool dense = p.dense_div > 0 && (long long)total * p.dense_div >= bw;
#if MR_GROUP_STUB == 2  // timing-only build: pass A only
    if (!big) o += dense ? ((cooc_dense_words(bw) + total + 3) & ~3) : ((total + 3) & ~3);
    *row_nz += (unsigned)total;
    continue;
#endif
    const int dwords = cooc_dense_words(bw);
    const long long seg = big ? p.row_base[r] + (long long)tile * p.tcap : o;
    const unsigned* cw = cnt + (size_t)k * (bs >> 1);
    unsigned* out = p.pool + seg;
    if (dense) {
      cooc_write_dense<NT, true>(out, bw, dwords, p.sat, &s_tail[k],
                           [&](int col) { return (cw[col >> 1] >> ((col & 1) << 4)) & 0xffffu; });
    } else {
      const uint4* cv = reinterpret_cast<const uint4*>(cw);
      const int nch = (bw + 7) >> 3;
      unsigned run = (unsigned)wbase;  // this wave's next entry
      for (int c0 = 0; c0 < nch; c0 += NT) {  // wave-uniform trip count (scans inside)
        const int c = c0 + tid;
        uint4 w4 = make_uint4(0u, 0u, 0u, 0u);
        if (c < nch) w4 = cv[c];
        const int n = nz_pairs8(w4);  // (zero past the tile)
        const int incl = wave_incl_scan(n);
        unsigned pos = run + (unsigned)(incl - n);
        run += (unsigned)wave_lane(incl, 63);
        const unsigned ww[4] = {w4.x, w4.y, w4.z, w4.w};
        const unsigned key0 = (unsigned)(c * 8) << kCoocCntBits;
#if MR_GROUP_STUB != 1  // (1: timing-only build without the sparse stores)
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const unsigned v = (ww[i >> 1] >> ((i & 1) << 4)) & 0xffffu;
          if (v) out[pos++] = (key0 | ((unsigned)i << kCoocCntBits)) | v;
        }
#else
        if ((int)pos < 0) out[0] = ww[0];
#endif
      }
    }
    if (!big) o += dense ? ((dwords + total + 3) & ~3) : ((total + 3) & ~3);
    *row_nz += (unsigned)total;
  }
  __syncthreads();
  if (tid == 0) {
    long long q = *off;
    for (int k = 0; k < ntg; ++k) {
      const int tile = t0 + k;
      const int bw = min(width, (tile + 1) * bs) - tile * bs;
      int total = 0;
      for (int x = 0; x < NW; ++x) total += s_wcnt[k * NW + x];
      const bool dense = p.dense_div > 0 && (long long)total * p.dense_div >= bw;
      p.seg_off[(size_t)tile * p.n_rows + r] = big ? p.row_base[r] + (long long)tile * p.tcap : q;
      p.seg_len[(size_t)tile * p.n_rows + r] = dense ? kCoocDenseTail - s_tail[k] : total;
      if (!big) q += dense ? ((cooc_dense_words(bw) + total + 3) & ~3) : ((total + 3) & ~3);
    }
  }
  *off = o;
}

// range of rows_walk: record x's entries of tile group g (lrec: the
// listener's base and group starts, one 16-B record in the row's order)
struct GroupRange {
  const unsigned* rec;
  int words, g;
  __device__ __forceinline__ void operator()(int x, long long& a, long long& b) const {
    const unsigned* q = rec + (size_t)x * words;
    const unsigned short* st = reinterpret_cast<const unsigned short*>(q + 1);
    const long long base = q[0];
    a = base + st[g];
    b = base + st[g + 1];
  }
};

// A k_cooc_group pass's counters zeroed up to the last 16-B chunk's end (the
// emission's chunk counts need no bound test), and its per-tile excess
// counters.
template <int NT>
__device__ __forceinline__ void group_zero(unsigned* cnt, int gw, int* s_tail) {
  uint4* c4 = reinterpret_cast<uint4*>(cnt);
  for (int i = threadIdx.x; i < (gw + 7) >> 3; i += NT) c4[i] = make_uint4(0u, 0u, 0u, 0u);
  if (threadIdx.x < kMaxGroupTiles) s_tail[threadIdx.x] = 0;
}

// Entries x .. x + 3 of sr_songs below b (a prefix of the chunk) or none.
__device__ __forceinline__ int group_chunk(const unsigned* songs, unsigned x, unsigned b, u32x4_a4& c) {
  c = u32x4_a4{0u, 0u, 0u, 0u};
  if (x >= b) return 0;
  c = *reinterpret_cast<const u32x4_a4*>(songs + x);
  const unsigned m = b - x;
  return m >= 4u ? 4 : (int)m;
}

// Song key's counter + 1 (u16 pairs: song x's counter is the half x & 1 of
// word x >> 1; a fire-and-forget LDS add). MR_GROUP_PAD: no branch per key —
// an invalid slot adds 0 to the lane's own word (< 64, inside the counters).
#ifndef MR_GROUP_PAD
#define MR_GROUP_PAD 1
#endif
__device__ __forceinline__ void group_inc(unsigned* cnt, unsigned key, bool ok, unsigned lo0) {
#if MR_GROUP_PAD
  const unsigned x = ok ? key - lo0 : 2u * (threadIdx.x & 63u);
  atomicAdd(&cnt[x >> 1], ok ? 1u << ((x & 1u) << 4) : 0u);
#else
  if (ok) {
    const unsigned x = key - lo0;
    atomicAdd(&cnt[x >> 1], 1u << ((x & 1u) << 4));
  }
#endif
}
// A chunk's m valid songs counted.
__device__ __forceinline__ void group_add(unsigned* cnt, const u32x4_a4& c, int m, unsigned lo0) {
  const unsigned k[4] = {c.x, c.y, c.z, c.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) group_inc(cnt, k[i], i < m, lo0);
}

// k_cooc_group's rows under kCoocBigRow listeners, every tile group in turn
// with the walk software-pipelined ACROSS groups: each lane group holds up to
// kGroupPipeR listeners for the whole row (mr_load caps the lanes per listener
// so that the row fits: n <= (NT >> glog) * kGroupPipeR), their ids and record
// bases are loaded once, the next group's end is loaded while this group is
// walked, and the next group's first two chunks per listener are issued before
// this group's emission, so they land while the tiles are written. The
// per-group walk of rows_walk repeated the whole dependent chain (listener id
// -> record -> chunk, ~3 x 3-5 us under load) for every group: C4 1x1 15.4 us
// of a group pass's ~32 (profiles/r04/s9).
#ifndef MR_GROUP_PIPE
#define MR_GROUP_PIPE 1
#endif
#ifndef MR_GROUP_PIPE_R
#define MR_GROUP_PIPE_R 4
#endif
constexpr int kGroupPipeR = MR_GROUP_PIPE_R;
template <int NT>
__device__ __forceinline__ void cooc_group_pipelined(const CoocParams& p, int r, const unsigned* lst, int n, int glog,
                                                     int width, unsigned* cnt, int* s_wcnt, int* s_tail,
                                                     long long* sb, long long* off, unsigned* row_nz) {
  constexpr int R = kGroupPipeR;
  const int tid = threadIdx.x;
  const int L = 1 << glog, j = tid & (L - 1), lg = tid >> glog, step = NT >> glog;
  const int bs = p.block_songs, GT = p.grp, nt = p.n_tiles, ng = p.n_grp, words = p.lrec_words;
  const unsigned* songs = p.sr_songs;
  // listener i of this lane group: record lg + i * step of the row (lst: the
  // row's first record); its entries of the current group: [a, b) of
  // sr_songs (records hold 32-bit bases, mr_load)
  int v[R];
  unsigned base[R], a[R], b[R];
#pragma unroll
  for (int i = 0; i < R; ++i) {
    const int l = lg + i * step;
    v[i] = l < n ? l : -1;
  }
#pragma unroll
  for (int i = 0; i < R; ++i) {
    base[i] = a[i] = b[i] = 0u;
    if (v[i] >= 0) {
      const unsigned* q = lst + (size_t)v[i] * words;
      const unsigned short* st = reinterpret_cast<const unsigned short*>(q + 1);
      base[i] = q[0];
      a[i] = base[i] + st[0];
      b[i] = base[i] + st[1];
    }
  }
  u32x4_a4 c[R][2];
  int m[R][2];
#pragma unroll
  for (int i = 0; i < R; ++i) {
    const unsigned x = a[i] + 4u * j;
    m[i][0] = group_chunk(songs, x, b[i], c[i][0]);
    m[i][1] = group_chunk(songs, x + 4u * L, b[i], c[i][1]);
  }
  for (int gi = 0; gi < ng; ++gi) {
    const int t0 = gi * GT, t1 = min(nt, t0 + GT);
    const unsigned lo0 = (unsigned)(t0 * bs);  // shard-local first song of the group
    const int gw = min(width, t1 * bs) - t0 * bs;
    group_zero<NT>(cnt, gw, s_tail);
    // the next group's end (its start is this group's end)
    unsigned e[R];
#pragma unroll
    for (int i = 0; i < R; ++i) {
      e[i] = b[i];
      if (v[i] >= 0 && gi + 1 < ng)
        e[i] = base[i] + reinterpret_cast<const unsigned short*>(lst + (size_t)v[i] * words + 1)[gi + 2];
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < R; ++i) {
      group_add(cnt, c[i][0], m[i][0], lo0);
      group_add(cnt, c[i][1], m[i][1], lo0);
    }
#pragma unroll
    for (int i = 0; i < R; ++i)
      for (unsigned x = a[i] + 4u * j + 8u * L; x < b[i]; x += 8u * L) {
        u32x4_a4 d0, d1;
        const int m0 = group_chunk(songs, x, b[i], d0);
        const int m1 = group_chunk(songs, x + 4u * L, b[i], d1);
        group_add(cnt, d0, m0, lo0);
        group_add(cnt, d1, m1, lo0);
      }
    __syncthreads();
    if (gi == 0) stamp_rt(sb, 1);  // the first group's walk done
    // the next group's first chunks: in flight while this group is emitted
    if (gi + 1 < ng) {
#pragma unroll
      for (int i = 0; i < R; ++i) {
        a[i] = b[i];
        b[i] = e[i];
        const unsigned x = a[i] + 4u * j;
        m[i][0] = group_chunk(songs, x, b[i], c[i][0]);
        m[i][1] = group_chunk(songs, x + 4u * L, b[i], c[i][1]);
      }
    }
    cooc_emit_group16<NT>(p, r, false, t0, t1 - t0, bs, width, cnt, s_wcnt, s_tail, off, row_nz,
                          gi == 0 ? sb : nullptr);
    // thread 0 reads s_wcnt / s_tail after the emission's closing barrier: keep
    // the next group's zeroing behind it
    __syncthreads();
    if (gi == 0) stamp_rt(sb, 2);  // the first group's tiles emitted
  }
}

template <int NT>
__global__ __launch_bounds__(NT) void k_cooc_group(CoocParams p) {
  extern __shared__ __align__(16) unsigned char smem_raw[];
  const int bs = p.block_songs, G = p.grp, ng = p.n_grp;
  const int width = p.song_hi - p.song_lo;
  unsigned* cnt = reinterpret_cast<unsigned*>(smem_raw);
  int* s_tail = reinterpret_cast<int*>(smem_raw + align16(G * bs * 2));  // [grp] excess entries per dense tile
  int* s_wcnt = s_tail + 3 * kMaxGroupTiles;  // [grp][NT / 64] non-zeros per tile and wave
  const int tid = threadIdx.x;
  // big rows (the first n_big): one workgroup per (row, group), a row's groups
  // on one XCD (blocks are dealt round-robin over the 8 XCDs: slot k of XCD x
  // takes row x + 8 (k / ng), group k % ng — the groups share the listeners'
  // records in that XCD's L2); the other rows one workgroup each, every group
  // in turn at a running pool offset
  const int lin = blockIdx.x;
  const int nbg = (p.n_big + 7) / 8 * 8 * ng;
  const bool big = lin < nbg;
  int ri, g_begin, g_end;
  if (big) {
    const int slot = lin >> 3;
    ri = (lin & 7) + 8 * (slot / ng);
    g_begin = slot % ng;
    g_end = g_begin + 1;
    if (ri >= p.n_big) return;
  } else {
    ri = p.n_big + (lin - nbg);
    g_begin = 0;
    g_end = ng;
  }
  const int4 rd = p.rdesc[ri];
  const int r = rd.x;
  const int n = rd.w;
  // the row's listener records (lrec, from rd.z): no listener id, no per-user
  // record line on the way to the shard-row chunks
  const unsigned* lst = p.lrec + (size_t)(unsigned)rd.z * p.lrec_words;
  const int glog = rd.y >> kLightGlogShift;
  long long* sb = p.stamps ? p.stamps + (size_t)blockIdx.x * 8 : nullptr;
  stamp_rt(sb, 0);
  long long off = p.row_base[r];
  unsigned row_nz = 0u;
#if MR_GROUP_PIPE
  if (!big && n <= (NT >> glog) * kGroupPipeR) {
    cooc_group_pipelined<NT>(p, r, lst, n, glog, width, cnt, s_wcnt, s_tail, sb, &off, &row_nz);
    g_end = g_begin;  // (every group done)
  }
#endif
  for (int gi = g_begin; gi < g_end; ++gi) {
    const int t0 = gi * G, t1 = min(p.n_tiles, t0 + G);
    const int lo0 = t0 * bs;  // shard-local first song of the group
    const int gw = min(width, t1 * bs) - lo0;
    group_zero<NT>(cnt, gw, s_tail);
    __syncthreads();
    // fire-and-forget adds (no returned value, no per-entry bookkeeping)
    rows_walk(tid, NT, glog, [](int l) { return l; }, n, GroupRange{lst, p.lrec_words, gi}, p.sr_songs,
              [&](const unsigned (&k)[8], int m) {
#pragma unroll
                for (int i = 0; i < 8; ++i) group_inc(cnt, k[i], i < m, (unsigned)lo0);
              });
    __syncthreads();
    if (gi == g_begin) stamp_rt(sb, 1);  // the first group's walk done
    // tile k's counters start at word k * bs / 2 (bs is a multiple of 256: 16-B aligned)
    cooc_emit_group16<NT>(p, r, big, t0, t1 - t0, bs, width, cnt, s_wcnt, s_tail, &off, &row_nz,
                          gi == g_begin ? sb : nullptr);
    // thread 0 reads s_wcnt / s_tail after the emission's closing barrier: keep
    // the next group's zeroing behind it (the dc4df36 race class)
    __syncthreads();
    if (gi == g_begin) stamp_rt(sb, 2);  // the first group's tiles emitted
  }
  if (tid == 0 && row_nz) atomicAdd(&p.row_nnz[r], row_nz);
  stamp_rt(sb, 4);
  stamp_val(sb, 5, big ? 1 : 0);
  stamp_val(sb, 6, n);
  stamp_val(sb, 7, big ? 1 : p.n_grp);
}

// The records of k_cooc_group, built once per load: one thread per train user
// walks its sorted shard row and writes its base and the start of every tile.
__global__ __launch_bounds__(256) void k_urec(const long long* sr_off, const unsigned* sr_songs, int n_tr, int n_tiles,
                                              int bs, int words, unsigned* rec) {
  const int v = blockIdx.x * 256 + threadIdx.x;
  if (v >= n_tr) return;
  const long long a = sr_off[v], b = sr_off[v + 1];
  unsigned* q = rec + (size_t)v * words;
  q[0] = (unsigned)a;
  unsigned short* st = reinterpret_cast<unsigned short*>(q + 1);
  long long x = a;
  for (int t = 0; t <= n_tiles; ++t) {
    const unsigned lim = (unsigned)t * (unsigned)bs;
    while (x < b && sr_songs[x] < lim) ++x;
    st[t] = (unsigned short)(t == n_tiles ? b - a : x - a);
  }
}

// k_cooc_group's per-(row, listener) records, built once per load from the
// per-user records: one workgroup per u16 heavy row (rd.z: its first record,
// rd.w: its listeners), the listener's base and its tile-group starts.
__global__ __launch_bounds__(256) void k_lrec(const int4* rdesc, const int* row_song, const long long* trs_off,
                                              const int* trs_users, const unsigned* urec, int urec_words,
                                              int n_tiles, int grp, int n_grp, int words, unsigned* lrec) {
  const int4 rd = rdesc[blockIdx.x];
  const long long s0 = trs_off[row_song[rd.x]];
  for (int l = threadIdx.x; l < rd.w; l += 256) {
    const unsigned* q = urec + (size_t)trs_users[s0 + l] * urec_words;
    const unsigned short* st = reinterpret_cast<const unsigned short*>(q + 1);
    unsigned* o = lrec + (size_t)((unsigned)rd.z + l) * words;
    o[0] = q[0];
    unsigned short* os = reinterpret_cast<unsigned short*>(o + 1);
    for (int g = 0; g < 2 * (words - 1); ++g) os[g] = g <= n_grp ? st[min(n_tiles, g * grp)] : 0;
  }
}

// The light rows' per-(row, listener) shard-row ranges, built once per load:
// one workgroup per light row (rd.z: its first record, rd.w: its listeners).
__global__ __launch_bounds__(256) void k_llrec(const int4* rdesc, const int* row_song, const long long* trs_off,
                                               const int* trs_users, const long long* sr_off, uint2* llrec) {
  const int4 rd = rdesc[blockIdx.x];
  const long long s0 = trs_off[row_song[rd.x]];
  for (int l = threadIdx.x; l < rd.w; l += 256) {
    const int v = trs_users[s0 + l];
    llrec[(size_t)(unsigned)rd.z + l] = make_uint2((unsigned)sr_off[v], (unsigned)sr_off[v + 1]);
  }
}

// Light-row tier t (light_tier_slots): its table size and workgroup width
// fixed at compile time. light_tier_call(t, stream, n, &params, ..) launches
// n rows; with params == nullptr it sets the kernel's LDS attribute instead.
__host__ __device__ constexpr int light_tier_nt(int t) { return t == 0 ? 1024 : t == 3 ? 256 : 512; }
inline int light_tier(int slots, int n_tiles) {
  const int last = n_tiles <= kWaveMaxTiles ? kLightTiers - 1 : 3;  // wave tiers hold <= 64 tile counters
  int t = 0;
  while (t + 1 <= last && light_tier_slots(t + 1) >= slots) ++t;
  return t;
}
template <int T>
int light_tier_go(hipStream_t st, int n, const CoocParams* lp) {
  constexpr int NT = light_tier_nt(T), S = light_tier_slots(T);
  const int lds = cooc_light_lds<NT, S>();
  if (!lp) {
    MR_HIP(hipFuncSetAttribute((const void*)k_cooc_light<NT, S>, hipFuncAttributeMaxDynamicSharedMemorySize, lds));
    return MR_OK;
  }
  hipLaunchKernelGGL((k_cooc_light<NT, S>), dim3(n), dim3(NT), (size_t)lds, st, *lp);
  MR_HIP(hipGetLastError());
  return MR_OK;
}
template <int SW>
int light_wave_go(hipStream_t st, int n, const CoocParams* lp) {
  const int lds = cooc_wave_bytes<SW>() * kWaveRowsPerBlock;
  if (!lp) {
    MR_HIP(hipFuncSetAttribute((const void*)k_cooc_light_wave<SW>, hipFuncAttributeMaxDynamicSharedMemorySize, lds));
    return MR_OK;
  }
  hipLaunchKernelGGL(k_cooc_light_wave<SW>, dim3((n + kWaveRowsPerBlock - 1) / kWaveRowsPerBlock),
                     dim3(64 * kWaveRowsPerBlock), (size_t)lds, st, *lp, n);
  MR_HIP(hipGetLastError());
  return MR_OK;
}
int light_tier_call(int t, hipStream_t st, int n, const CoocParams* lp, const CoocParams&) {
  switch (t) {
    case 0: return light_tier_go<0>(st, n, lp);
    case 1: return light_tier_go<1>(st, n, lp);
    case 2: return light_tier_go<2>(st, n, lp);
    case 3: return light_tier_go<3>(st, n, lp);
    case 4: return light_wave_go<2048>(st, n, lp);
    default: return light_wave_go<1024>(st, n, lp);
  }
}

// ---------------------------------------------------------------------------
// top-k over a dense model buffer (any model of the context's shape, e.g. a
// combination model, MR:317-481): one 1024-thread workgroup per test user,
// per-thread running lists, per-wave register tournament, wave 0 merges.
// Keys are the bit patterns of the (non-negative) scores; a negative score
// sets *neg (the caller reports MR_E_INVALID: no total order in int64 keys).
// ---------------------------------------------------------------------------
struct DenseTopkParams {
  int user0, width, song_lo, k;
  const void* dense;
  long long* top_key;
  int* top_song;
  double* top_score;
  unsigned* neg;
};

template <typename OutT>
__global__ __launch_bounds__(kWideThreads) void k_topk_dense(DenseTopkParams p) {
  constexpr int NT = kWideThreads, NW = NT / 64;
  __shared__ long long wk[NW * kMaxTopkLarge];
  __shared__ int ws[NW * kMaxTopkLarge];
  __shared__ long long fk[kMaxTopkLarge];
  __shared__ int fs[kMaxTopkLarge];
  const int u = p.user0 + blockIdx.x;
  const int tid = threadIdx.x, w = tid >> 6, k = p.k;
  const OutT* row = reinterpret_cast<const OutT*>(p.dense) + (size_t)u * p.width;
  long long tk[kMaxTopkLarge];
  int ts[kMaxTopkLarge];
#pragma unroll
  for (int t = 0; t < kMaxTopkLarge; ++t) { tk[t] = kKeyNone; ts[t] = INT_MAX; }
  long long thr = kKeyNone;
  bool neg = false;
  for (int i = tid; i < p.width; i += NT) {
    const double x = (double)row[i];
    if (x != x) continue;  // NaN: no pair (heard song, MR:109)
    if (x < 0.0) { neg = true; continue; }
    const long long key = __double_as_longlong(x + 0.0);  // -0.0 -> +0.0
    if (key > thr) lane_list_insert(tk, ts, k, key, p.song_lo + i, thr);
  }
  if (neg) atomicOr(p.neg, 1u);
  wave_topk_regs<kMaxTopkLarge, true>(tk, ts, k, wk + w * k, ws + w * k);
  __syncthreads();
  if (w == 0) wave_merge_lists(NW, k, wk, ws, fk, fs);
  __syncthreads();
  for (int r = tid; r < k; r += NT) {
    const size_t o = (size_t)u * k + r;
    p.top_key[o] = fk[r];
    p.top_song[o] = fs[r];
    p.top_score[o] = fk[r] >= 0 ? __longlong_as_double(fk[r]) : (double)NAN;
  }
}

// auto shape: wide from this many (test user x train user) pairs of work
// (scripts/shape_sweep.py, profiles/r01_final/shape_sweep.txt: at 500 train x
// 256 test users wide 0.101 ms vs fused 0.112; C2's 500 x 10 stays fused)
constexpr long long kWideMinUserPairs = 100000;

// ---------------------------------------------------------------------------
// Top-k merge over lists (exchange step after a song-shard all-gather).
// Element (u, l, r) of the input: key at keys[u*user_stride + l*list_stride_k +
// r], song at songs[u*user_stride + l*list_stride_s + r] (the strides differ
// for gathered record blocks: keys and songs of one shard in one block).
// ---------------------------------------------------------------------------
struct MergeParams {
  int n_lists, k_in, k_out;
  long long user_stride, list_stride_k, list_stride_s;
  const long long* keys;
  const int* songs;
  long long* out_keys;    // [n_users][k_out]
  int* out_songs;
  double* out_scores;     // may be null
};

// Bytes of one shard's top-k record block: n int64 keys then n int32 songs,
// padded to 16 B (the block stride of a gathered exchange buffer).
inline int64_t topk_record_bytes(size_t n) { return (int64_t)((12 * n + 15) / 16 * 16); }

__host__ __device__ inline int merge_lds_bytes(int k) {
  return align16(merge_lists_per_pass(k) * k * 12) + align16(kMaxTopK * 12);
}

__global__ __launch_bounds__(kThreads) void k_topk_merge(MergeParams p) {
  extern __shared__ __align__(16) unsigned char smem_raw[];
  const int k = p.k_out;
  const int per = merge_lists_per_pass(k);
  long long* mk = reinterpret_cast<long long*>(smem_raw);
  int* ms = reinterpret_cast<int*>(mk + per * k);
  long long* fk = reinterpret_cast<long long*>(smem_raw + align16(per * k * 12));
  int* fs = reinterpret_cast<int*>(fk + kMaxTopK);
  const int bu = blockIdx.x;
  const int tid = threadIdx.x;
  const long long* keys = p.keys + (size_t)bu * p.user_stride;
  const int* songs = p.songs + (size_t)bu * p.user_stride;
  int done = 0, off = 0;
  while (done < p.n_lists) {
    const int nl = min(p.n_lists - done, per - off);
    for (int i = tid; i < nl * k; i += kThreads) {
      const int l = done + i / k, r = i - (i / k) * k;
      const bool in = r < p.k_in;
      mk[off * k + i] = in ? keys[(size_t)l * p.list_stride_k + r] : kKeyNone;
      ms[off * k + i] = in ? songs[(size_t)l * p.list_stride_s + r] : -1;
    }
    for (int i = tid; i < off * k; i += kThreads) {
      mk[i] = fk[i];
      ms[i] = fs[i];
    }
    __syncthreads();
    if ((tid >> 6) == 0) wave_merge_lists(nl + off, k, mk, ms, fk, fs);
    __syncthreads();
    done += nl;
    off = 1;
  }
  const size_t o = (size_t)bu * k;
  for (int r = tid; r < k; r += kThreads) {
    p.out_keys[o + r] = fk[r];
    p.out_songs[o + r] = fs[r];
    if (p.out_scores) p.out_scores[o + r] = fk[r] >= 0 ? __longlong_as_double(fk[r]) : (double)NAN;
  }
}

// ---------------------------------------------------------------------------
// Stage-1 chunk boundaries of every listener list, built once by mr_load:
// sbound[s][cc] = first index i of L_tr(s) = trs_users[trs_off[s] ..
// trs_off[s+1]) (ascending) with trs_users[i] >= cc * chunk. One binary search
// per entry (C4: 95M entries; was a host loop plus a 380 MB upload).
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_sbound(const long long* trs_off, const int* trs_users, int n_s, int nc1,
                                                int chunk, int* sbound) {
  const size_t total = (size_t)n_s * nc1;
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < total; i += (size_t)gridDim.x * 256) {
    const int s = (int)(i / nc1);
    const long long bound = (long long)(int)(i - (size_t)s * nc1) * chunk;
    long long a = trs_off[s], b = trs_off[s + 1];
    while (a < b) {
      const long long m = (a + b) >> 1;
      if (trs_users[m] < bound) a = m + 1; else b = m;
    }
    sbound[i] = (int)a;
  }
}

// ---------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------
template <typename T>
struct DevBuf {
  T* p = nullptr;
  size_t n = 0;
  bool own = true;  // false: a view into another buffer's allocation
  void release() {
    if (p && own) (void)hipFree(p);
    p = nullptr;
    n = 0;
    own = true;
  }
};

template <typename T>
int dev_alloc(DevBuf<T>& b, size_t n) {
  b.release();
  if (n == 0) n = 1;
  MR_HIP(hipMalloc(reinterpret_cast<void**>(&b.p), n * sizeof(T)));
  b.n = n;
  return MR_OK;
}

template <typename T>
int dev_upload(DevBuf<T>& b, const T* src, size_t n, hipStream_t st) {
  int rc = dev_alloc(b, n);
  if (rc) return rc;
  if (n) MR_HIP(hipMemcpyAsync(b.p, src, n * sizeof(T), hipMemcpyHostToDevice, st));
  return MR_OK;
}

using ScoreKernel = void (*)(ScoreParams);
using NbrKernel = void (*)(NbrParams);

// Launch shapes (mr_options.stage1 / mr_launch_info).
enum Shape { kShapeSeparate = 0, kShapeFused = 1, kShapeWide = 3 };

}  // namespace

struct mr_ctx {
  mr_options opt{};
  int dev_share = 1;  // contexts of this process on the device (mr_internal::set_device_share)
  hipStream_t stream = nullptr;
  bool loaded = false;
  bool ran = false;
  bool fused = false;
  int shape = kShapeSeparate;
  int last_model = -1;
  int n_tr = 0, n_te = 0, n_s = 0;
  int song_lo = 0, song_hi = 0, width = 0;
  int block_songs = 0, n_tiles = 0;
  int cap = 0, batch = 0;
  int chunk = 1, n_chunks = 1;  // separate shape: stage-1 chunks of train users
  size_t score_lds = 0, nbr_lds = 0, merge_lds = 0, wide_lds = 0;
  ScoreKernel score_kernel[2] = {nullptr, nullptr};  // [model]
  NbrKernel nbr_kernel[2] = {nullptr, nullptr};
  DevBuf<long long> tr_off, te_off, trs_off, q_song, cand_key, top_key, nbr_q;
  DevBuf<int> te_songs, trs_users, toff, nbr_v, nbr_cnt, cand_song, top_song;
  DevBuf<unsigned short> tsongs;
  DevBuf<unsigned> tpack;  // fused shape: tile entries as (train user << 16) | tile-local song
  DevBuf<int2> te_rng;     // fused shape: listener range of every test-visible song
  DevBuf<long long> te_q;  // fused shape: its ibm weight q_song
  DevBuf<uint2> te_sched;  // fused shape: stage 1's walk schedule (ScoreParams::te_sched)
  DevBuf<long long> sched_off;
  DevBuf<int> sbound;  // stage-1 chunk boundaries of every listener list (n_chunks > 1)
  DevBuf<unsigned> counter;
  DevBuf<double> sqrt_c, sqrt_tr, sqrt_te, top_score;
  DevBuf<float> rsq_c;  // wide shape: 1 / sqrt(c(s)) as fp32 (wide_cand_topk's approximations)
  bool cand_on = false; // wide shape, top-k only: the candidate-only tile top-k (MR_WIDE_CAND=0: off)
  DevBuf<unsigned char> dense;
  DevBuf<long long> stamps;
  // Pinned staging of large D2H copies (d2h_staged): two buffers, lazily
  // allocated, kept for the context's life.
  hipEvent_t stage_ev[2] = {nullptr, nullptr};
  // Kernel timing ring: 3 events per timed batch (before stage 1, before the
  // score kernel, after it), recorded without host synchronisation and
  // resolved in flush_timing (mr_kernel_times, ring full).
  static constexpr int kRing = 1024;
  std::vector<hipEvent_t> ring;
  int ring_used = 0;
  bool ring_has_stage1[kRing] = {};
  long long launches[3] = {0, 0, 0};
  double ms[3] = {0, 0, 0};
  // Timing window (mr_timing_begin/end): two events on the stream around any
  // number of mr_run calls, no per-launch events.
  hipEvent_t win[2] = {nullptr, nullptr};
  bool win_open = false;
  bool win_stopped = false;  // mr_timing_stop recorded win[1]
  void* dense_override = nullptr;  // mr_run_into: caller's device buffer for this run's dense model
  DevBuf<unsigned long long> mm_key;  // wide dense runs: per-user min / max keys of the stored scores
  bool mm_on = false, mm_valid = false;
  hipGraph_t graph = nullptr;          // mr_graph_capture: n steps of mr_run
  hipGraphExec_t graph_exec = nullptr;
  int graph_steps = 0;
  DevBuf<unsigned> flag;           // mr_topk_dense_device: negative-score flag
  long long win_launches = 0;
  // co-listening route (mr_options.ibm_route, k_cooc_build)
  int ibm_route = 1;               // 1 two-hop, 2 co-listening index
  int cooc_nt = 1024;              // threads of the co-listening scoring workgroups (MR_COOC_NT)
  size_t cooc_score_lds = 0;
  int n_rows = 0, nseg = 0;
  long long pool_cap = 0;
  size_t cooc_lds = 0;
  ScoreKernel cooc_kernel = nullptr;
  DevBuf<int> row_song, te_row, seg_len;
  DevBuf<long long> row_base, seg_off;
  DevBuf<unsigned> pool;
  DevBuf<unsigned> row_nnz;        // per run: each index row's non-zeros over the shard
  std::vector<int32_t> row_users;  // test users whose T(u) holds the row's song
  std::vector<int64_t> row_reads;  // per row: c_tr(s2) + Σ_{v ∈ L_tr(s2)} |S(v) ∩ shard| (mr_cooc_bytes)
  std::vector<int32_t> row_listeners;  // per row: c_tr(s2)
  std::vector<uint8_t> row_light;  // per row: built by the light-row kernels
  long long build_reads = 0;       // Σ_r c_tr(s2) + Σ_{v ∈ L_tr(s2)} |S(v) ∩ shard| (mr_cooc_stats)
  bool cooc_ran = false;           // an ibm run on route 2 since the load (its row_nnz are current)
  hipStream_t side[2] = {nullptr, nullptr};  // light-row build streams (created with the context)
  hipEvent_t side_fork = nullptr, side_join[2] = {nullptr, nullptr};
  int n_heavy = 0, n_light = 0;    // rows built per (row, tile) / per row (k_cooc_light)
  int n_light_tier[6] = {0, 0, 0, 0, 0, 0};  // light rows per table tier (light_tier_slots), in launch order
  int n_heavy32 = 0;               // the first heavy rows: >= 65536 listeners (u32 counters)
  int n_big16 = 0, tcap16 = 0, tcap32 = 0;  // big u16 rows after them; per-tile slot words
  int dense_div = 0, force32 = 0;  // k_cooc_build's dense-segment rule
  unsigned sat = 255;
  size_t bstamp_off = 0;           // diagnostic build: k_cooc_build's stamps in the stamps buffer
  size_t lstamp_off = 0;           //   and the light rows' (one slot block per light row, launch order)
  DevBuf<int> rows_order, row_slots;  // heavy rows then light rows; light rows' hash slots
  DevBuf<int4> rdesc;              // rows_order's rows as {row, row_slots, listener start, listeners}
  DevBuf<long long> sr_off;        // light rows / k_cooc_group: the shard's train rows
  DevBuf<unsigned> sr_songs;
  DevBuf<unsigned> urec;           // k_cooc_group: per-user tile starts (load-time only: lrec's source)
  DevBuf<unsigned> lrec;           // k_cooc_group: per-(row, listener) base + tile-group starts
  DevBuf<uint2> llrec;             // k_cooc_light*: per-(row, listener) shard-row ranges
  int grp = 0, n_grp = 0, urec_words = 0, lrec_words = 0;
  int group_nt = 1024;             // threads per k_cooc_group workgroup (MR_COOC_GNT)

  void release_data() {
    tr_off.release(); te_off.release(); trs_off.release(); q_song.release();
    cand_key.release(); top_key.release(); nbr_q.release();
    tsongs.release(); tpack.release(); te_rng.release(); te_q.release(); te_sched.release(); sched_off.release(); te_songs.release(); trs_users.release(); toff.release(); sbound.release();
    nbr_v.release(); nbr_cnt.release(); cand_song.release(); top_song.release();
    counter.release();
    sqrt_c.release(); sqrt_tr.release(); sqrt_te.release(); top_score.release();
    rsq_c.release(); cand_on = false;
    dense.release();
    mm_key.release(); mm_on = mm_valid = false;
    stamps.release();
    flag.release();
    row_song.release(); te_row.release(); seg_len.release(); row_base.release(); seg_off.release();
    pool.release();
    rows_order.release(); row_slots.release(); sr_off.release(); sr_songs.release(); row_nnz.release();
    urec.release(); lrec.release(); llrec.release(); rdesc.release(); grp = n_grp = urec_words = lrec_words = 0;
    row_users.clear(); row_reads.clear(); row_listeners.clear(); row_light.clear();
    build_reads = 0; cooc_ran = false;
    ibm_route = 1; n_rows = 0; nseg = 0; pool_cap = 0; cooc_kernel = nullptr; n_heavy = n_light = n_heavy32 = 0;
    for (int& x : n_light_tier) x = 0;
    if (graph_exec) (void)hipGraphExecDestroy(graph_exec);
    if (graph) (void)hipGraphDestroy(graph);
    graph_exec = nullptr;
    graph = nullptr;
    graph_steps = 0;
    loaded = ran = false;
  }
};

namespace {

// Smallest i in [0, n) with bad(i), or -1: every worker scans its range in
// order and stops at its first hit.
template <class F>
int64_t first_bad(int64_t n, F&& bad, int64_t grain = 1 << 14) {
  std::atomic<int64_t> best{INT64_MAX};
  mr_par::parallel_for(n, [&](int64_t lo, int64_t hi, int) {
    for (int64_t i = lo; i < hi && i < best.load(std::memory_order_relaxed); ++i)
      if (bad(i)) {
        int64_t cur = best.load();
        while (i < cur && !best.compare_exchange_weak(cur, i)) {}
        return;
      }
  }, grain);
  const int64_t b = best.load();
  return b == INT64_MAX ? -1 : b;
}

// Sorted strictly ascending columns in [0, n_cols), checked in parallel; the
// first bad row (in row order) is reported. Offsets are checked first, so the
// column pass only reads inside [off[0], off[n_rows]).
int validate_csr(const char* what, int n_rows, int n_cols, const int64_t* off, const int32_t* col) {
  if (!off || (off[n_rows] > 0 && !col)) return fail(MR_E_INVALID, "%s: null CSR array", what);
  if (off[0] != 0) return fail(MR_E_INVALID, "%s: offsets[0] = %lld != 0", what, (long long)off[0]);
  const int64_t r0 = first_bad(n_rows, [&](int64_t r) { return off[r + 1] < off[r]; });
  if (r0 >= 0) return fail(MR_E_INVALID, "%s: offsets decrease at row %d", what, (int)r0);
  const int64_t r1 = first_bad(n_rows, [&](int64_t r) {
    for (int64_t i = off[r]; i < off[r + 1]; ++i)
      if (col[i] < 0 || col[i] >= n_cols || (i > off[r] && col[i] <= col[i - 1])) return true;
    return false;
  }, 1 << 10);
  if (r1 >= 0) {
    const int r = (int)r1;
    for (int64_t i = off[r]; i < off[r + 1]; ++i) {
      if (col[i] < 0 || col[i] >= n_cols)
        return fail(MR_E_INVALID, "%s: row %d has column %d outside [0,%d)", what, r, col[i], n_cols);
      if (i > off[r] && col[i] <= col[i - 1])
        return fail(MR_E_INVALID, "%s: row %d is not sorted strictly ascending", what, r);
    }
  }
  if (off[n_rows] >= (int64_t)INT32_MAX)
    return fail(MR_E_INVALID, "%s: %lld entries exceed the int32 index range", what, (long long)off[n_rows]);
  return MR_OK;
}

// Worker ranges over [0, n) with about equal weight: range w = [cut[w], cut[w+1])
// of a prefix-summed weight (CSR offsets: rows of power-law length).
std::vector<int64_t> weighted_cuts(const int64_t* prefix, int64_t n, int parts) {
  std::vector<int64_t> cut(parts + 1, n);
  cut[0] = 0;
  const int64_t total = prefix[n] - prefix[0];
  for (int w = 1; w < parts; ++w) {
    const int64_t target = prefix[0] + total * w / parts;
    cut[w] = std::max(cut[w - 1], (int64_t)(std::lower_bound(prefix, prefix + n + 1, target) - prefix));
    cut[w] = std::min(cut[w], n);
  }
  return cut;
}

// Rows of the in-launch merge's threshold pass: 32 (C2 step 20.4 us vs 22.9 at
// 16 rows and 20.8 at 64, profiles/r01_final/c2_merge_rows.txt);
// MR_MERGE_ROWS=16/32/64 overrides it for experiments.
int merge_rows_opt() {
  static const int rows = [] {
    const char* e = std::getenv("MR_MERGE_ROWS");
    const int r = e ? std::atoi(e) : 32;
    return (r == 16 || r == 64) ? r : 32;
  }();
  return rows;
}

// Wide-shape block mapping (ScoreParams.xcd_remap): 1 = tiles of a user on
// one XCD, 2 = one tile's users per XCD; MR_WIDE_MAP=1/2 overrides.
// Light index rows by k_cooc_light (default) or every row per (row, tile)
// (MR_COOC_LIGHT=0: A/B experiments and tests; read at each mr_load).
// Largest light-row table (MR_COOC_LIGHT_MAX slots, a power of 2 in
// [1024, kLightSlots]; rows above it go to the heavy-row kernels) and the
// table's load bound (MR_COOC_LIGHT_LOAD: entry bound <= this % of the slots,
// default 80): A/B experiments, read at each mr_load.
// Default: the largest table (kLightSlots) — unless the shard is narrow enough
// for k_cooc_group to hold ALL its tiles in one pass (C4 over 8 GPUs: 3 tiles
// of 15.6k songs): then one listener walk with fire-and-forget counter adds
// beats hashing for the larger rows, and light rows stop at kLightSlotsNarrow.
constexpr int64_t kLightSlotsNarrow = 8192;  // C4 8 x 1: 6.20 vs 6.32 ms (16k), profiles/r04/s20
int64_t cooc_light_max_opt(bool narrow) {
  const char* e = std::getenv("MR_COOC_LIGHT_MAX");
  int64_t v = e ? std::atoll(e) : (narrow ? kLightSlotsNarrow : kLightSlots);
  int64_t s = 1024;
  while (s * 2 <= std::min<int64_t>(v, kLightSlots)) s *= 2;
  return s;
}
int64_t cooc_light_load_opt() {
  const char* e = std::getenv("MR_COOC_LIGHT_LOAD");
  const int64_t v = e ? std::atoll(e) : 80;
  return std::min<int64_t>(100, std::max<int64_t>(10, v));
}
bool cooc_light_opt() {
  const char* e = std::getenv("MR_COOC_LIGHT");
  return !(e && std::atoi(e) == 0);
}
// fused stage 1 from the load-time walk schedule (MR_FUSED_SCHED=0 at load:
// the per-step segment search, as past the schedule's size cap)
bool fused_sched_opt() {
  const char* e = std::getenv("MR_FUSED_SCHED");
  return MR_FUSED_SCHED && !(e && std::atoi(e) == 0);
}
// Heavy u16 rows by tile groups (k_cooc_group, default) or per tile
// (MR_COOC_GROUP=0: k_cooc_build<512, true>; A/B experiments and tests; read
// at each mr_load).
// Threads per co-listening scoring workgroup: 1024 (default) or 512
// (MR_COOC_NT=512: with a narrower block_songs, two or three workgroups per
// CU; A/B experiments, read at each mr_load).
int cooc_nt_opt() {
  const char* e = std::getenv("MR_COOC_NT");
  return e && std::atoi(e) == 512 ? 512 : 1024;
}
// Tiles per k_cooc_group pass at most (MR_COOC_GRP; default: as many as the
// LDS holds, up to kMaxGroupTiles): fewer tiles = fewer bytes of LDS per
// workgroup, more workgroups per CU, more listener walks (A/B experiments).
// Threads per k_cooc_group workgroup: 1024 (default) or 512 (MR_COOC_GNT=512:
// with MR_COOC_GRP=2, two workgroups per CU; A/B experiments).
int cooc_group_nt_opt() {
  const char* e = std::getenv("MR_COOC_GNT");
  return e && std::atoi(e) == 512 ? 512 : 1024;
}
int cooc_group_max_opt() {
  const char* e = std::getenv("MR_COOC_GRP");
  const int v = e ? std::atoi(e) : 0;
  return v > 0 ? v : kMaxGroupTiles;
}
bool cooc_group_opt() {
  const char* e = std::getenv("MR_COOC_GROUP");
  return !(e && std::atoi(e) == 0);
}
// Light rows on side streams (default) or on the context stream
// (MR_COOC_SIDE=0: A/B experiments; read at each run).
bool cooc_side_opt() {
  const char* e = std::getenv("MR_COOC_SIDE");
  return !(e && std::atoi(e) == 0);
}
// Dense-segment rule of k_cooc_build (MR_COOC_DENSE_DIV, default kCoocDenseDiv;
// 0 = sparse only) and u32 dense counts for every row (MR_COOC_DENSE32=1):
// experiments and tests, read at each mr_load.
int cooc_dense_div_opt() {
  const char* e = std::getenv("MR_COOC_DENSE_DIV");
  return e ? std::max(0, std::atoi(e)) : kCoocDenseDiv;
}
int cooc_dense32_opt() {
  const char* e = std::getenv("MR_COOC_DENSE32");
  return e && std::atoi(e) == 1 ? 1 : 0;
}
// Saturation of the dense segments' count bytes (255; MR_COOC_SAT lowers it
// so tests see excess entries on small data).
unsigned cooc_sat_opt() {
  const char* e = std::getenv("MR_COOC_SAT");
  const long v = e ? std::atol(e) : 255;
  return (unsigned)std::min<long>(255, std::max<long>(1, v));
}

// Auto route rule: the co-listening route when its estimated device time is
// below the two-hop route's. Per-unit costs fitted on one MI355X
// (profiles/r03/cooc/route_model.txt): two-hop 5.75 ps per estimated
// (tile, test user, neighbour) visit, neighbours estimated by Σ_{s2∈T(u)}
// c_tr(s2) capped at n_tr (C4 286 ms of stage-2 time); co-listening build
// 35 ps per heavy (row, tile, listener) visit and 12.8 ps per light-row entry,
// scoring 0.49 ps per estimated consumed entry (bound of the row's non-zeros),
// plus a latency floor of 28 ns per light row and 24 ns per heavy (row, tile)
// workgroup (C3: 0.30 ms for 10.7k light rows). C3 -> two-hop (0.77 vs 0.38 ms
// estimated; 1.53 vs 1.09 measured), C4 / C5 -> co-listening (62 vs 286 ms,
// 28 vs 58 ms estimated).
bool cooc_pays(double v_est, double e_est, const std::vector<int64_t>& bound, const std::vector<int64_t>& reads,
               const std::vector<int32_t>& row_song, const std::vector<int32_t>& col_tr, int n_tiles) {
  double build = 0.0;
  for (size_t r = 0; r < row_song.size(); ++r) {
    const double c = col_tr[row_song[r]];
    if (bound[r] <= light_bound_max(kLightSlots) && c <= kLightCntMask) build += 12.8e-12 * (double)(reads[r] - c) + 28e-9;
    else build += n_tiles * (35e-12 * c + 24e-9);
  }
  return build + 0.49e-12 * e_est < 5.75e-12 * v_est;
}

int wide_map_opt() {
  static const int m = [] {
    const char* e = std::getenv("MR_WIDE_MAP");
    const int v = e ? std::atoi(e) : 0;
    return v >= 1 && v <= 3 ? v : kWideMapDefault;
  }();
  return m;
}

int auto_block_songs(int width, int n_te, bool fused, int k, int n_tr) {
  // Separate: aim for >= ~1024 workgroups, tiles of 256..16384 songs; with top-k a tile
  // is at most kMaxTopkTile songs (4 candidates per lane in registers); the
  // fused path keeps the neighbour array beside the tile (<= 8192).
  // Large train sets (chunked stage 1): every tile re-walks the user's whole
  // neighbour list, so take the widest tile (wide top-k, k <= 16).
  long long cover = ((long long)width + 255) / 256 * 256;  // no point in a tile wider than the shard
  if (!fused && n_tr > kMaxLdsTrainUsers && k <= kMaxTopkLarge)
    return (int)std::max<long long>(256, std::min<long long>(kMaxBlockSongs, cover));
  const long long cap = k > 0 ? kMaxTopkTile : (fused ? 8192 : kMaxBlockSongs);
  // Fused: every tile repeats stage 1 and adds a candidate list to the
  // user's merge, so aim for ~256 workgroups (C2: 22 tiles of 768 songs,
  // 14.5 us vs 15.2 at 512 and 14.7 at 1024 once stage 2 became LDS-only,
  // scripts/c2_bs_sweep.py, profiles/r02).
  const long long target = fused ? 256 : 1024;
  long long want = ((long long)width * std::max(1, n_te) + target - 1) / target;
  long long bs = ((want + 255) / 256) * 256;
  bs = std::max<long long>(256, std::min<long long>(cap, bs));
  return (int)std::max<long long>(256, std::min(bs, cover));
}

template <int MODEL>
void pick_kernels(mr_ctx* c) {
  const bool f64 = c->opt.out_dtype == MR_OUT_F64;
  if (c->fused)
    c->score_kernel[MODEL] = f64 ? k_score<MODEL, double, true> : k_score<MODEL, float, true>;
  else
    c->score_kernel[MODEL] = f64 ? k_score<MODEL, double, false> : k_score<MODEL, float, false>;
  if (c->shape == kShapeWide) {
    if (c->opt.topk == 10)
      c->score_kernel[MODEL] = f64 ? k_score_wide<MODEL, double, kWideThreads, 10, false>
                                   : k_score_wide<MODEL, float, kWideThreads, 10, false>;
    else
      c->score_kernel[MODEL] = f64 ? k_score_wide<MODEL, double, kWideThreads, kMaxTopkLarge, false>
                                   : k_score_wide<MODEL, float, kWideThreads, kMaxTopkLarge, false>;
    if constexpr (MODEL == MR_IBM) {
      if (c->ibm_route == 2 && c->cooc_nt == 512) {
        if (c->opt.topk == 10)
          c->cooc_kernel = f64 ? k_score_wide<MR_IBM, double, 512, 10, true> : k_score_wide<MR_IBM, float, 512, 10, true>;
        else
          c->cooc_kernel = f64 ? k_score_wide<MR_IBM, double, 512, kMaxTopkLarge, true>
                               : k_score_wide<MR_IBM, float, 512, kMaxTopkLarge, true>;
      } else if (c->ibm_route == 2) {
        if (c->opt.topk == 10)
          c->cooc_kernel = f64 ? k_score_wide<MR_IBM, double, kWideThreads, 10, true>
                               : k_score_wide<MR_IBM, float, kWideThreads, 10, true>;
        else
          c->cooc_kernel = f64 ? k_score_wide<MR_IBM, double, kWideThreads, kMaxTopkLarge, true>
                               : k_score_wide<MR_IBM, float, kWideThreads, kMaxTopkLarge, true>;
      }
    }
  }
  c->nbr_kernel[MODEL] = k_neighbours<MODEL>;
}

// Launch-shape rule of mr_load (also answers mr_shard_tile_songs before any
// load). auto (scripts/shape_sweep.py, profiles/r01_final/shape_sweep.txt):
// wide beats separate above 4096 train users, and fused from ~1e5 (test user x
// train user) pairs; fused for small sets (C2). Round 2 also measured a
// "pull" shape (dense Yt slab gathered per song) and a "user" shape (one
// 1024-thread workgroup per test user): never faster, removed in round 3.
int pick_shape(const mr_options& o, int n_tr, int n_te) {
  const int k = o.topk;
  if (o.stage1 == 1) return kShapeFused;
  if (o.stage1 == 2) return kShapeSeparate;
  if (o.stage1 == 4) return kShapeWide;
  if (n_tr > kMaxFusedTrainUsers && k <= kMaxTopkLarge) return kShapeWide;
  if ((long long)n_te * n_tr >= kWideMinUserPairs && k <= kMaxTopkLarge) return kShapeWide;
  return n_tr <= kMaxFusedTrainUsers ? kShapeFused : kShapeSeparate;
}

// Train users per stage-1 chunk (separate / wide shapes).
int stage1_chunk_for(const mr_options& o, int n_tr) {
  return o.stage1_chunk > 0 ? std::min(o.stage1_chunk, std::max(1, n_tr))
         : n_tr <= kMaxLdsTrainUsers ? std::max(1, n_tr) : kStage1Chunk;
}

// The widest wide-shape tile (a multiple of 256 songs) whose LDS fits one CU.
int wide_bmax(int k, int n_chunks) {
  int bmax = 256;
  while (bmax + 256 <= 65536 && wide_lds<kWideThreads>(bmax + 256, k, n_chunks).total <= kLdsBytes) bmax += 256;
  return bmax;
}

}  // namespace

// Every input check of mr_load (sizes, CSR shapes, sorted rows, id ranges,
// duplicate-counting lengths, song counts), in parallel; the distinct train
// listeners per song come back in *col_tr.
static int check_dataset(const mr_dataset* d, std::vector<int32_t>& col_tr) {
  mr_par::PhaseTrace trace("MR_LOAD_TRACE", "mr_load");
  const int n_tr = d->n_train_users, n_te = d->n_test_users, n_s = d->n_songs;
  if (n_tr < 0 || n_te <= 0 || n_s <= 0)
    return fail(MR_E_INVALID, "bad sizes: n_train_users=%d n_test_users=%d n_songs=%d", n_tr, n_te, n_s);
  if (n_tr > kMaxChunks * kStage1Chunk)
    return fail(MR_E_INVALID, "n_train_users=%d exceeds the stage-1 limit %d of this build", n_tr,
                kMaxChunks * kStage1Chunk);
  int rc;
  if ((rc = validate_csr("train user->songs", n_tr, n_s, d->tr_off, d->tr_songs))) return rc;
  if ((rc = validate_csr("test user->songs", n_te, n_s, d->te_off, d->te_songs))) return rc;
  if (!d->song_count || !d->tr_len || !d->te_len) return fail(MR_E_INVALID, "null count arrays");
  {  // lengths count duplicates: >= the distinct count, and nobody is empty (MR:44-46)
    const int64_t v = first_bad(n_tr, [&](int64_t v) {
      const int64_t deg = d->tr_off[v + 1] - d->tr_off[v];
      return deg <= 0 || d->tr_len[v] < deg;
    });
    if (v >= 0)
      return fail(MR_E_INVALID, "train user %d: %lld distinct songs but length %d", (int)v,
                  (long long)(d->tr_off[v + 1] - d->tr_off[v]), d->tr_len[v]);
    const int64_t u = first_bad(n_te, [&](int64_t u) {
      const int64_t deg = d->te_off[u + 1] - d->te_off[u];
      return deg <= 0 || d->te_len[u] < deg;
    });
    if (u >= 0)
      return fail(MR_E_INVALID, "test user %d: %lld distinct songs but length %d", (int)u,
                  (long long)(d->te_off[u + 1] - d->te_off[u]), d->te_len[u]);
  }
  const int64_t nnz_tr = d->tr_off[n_tr];
  // Workers of the bulk passes: ranges of users with about equal entries.
  const int W = (int)std::max<int64_t>(1, std::min<int64_t>(mr_par::usable_cores(), nnz_tr >> 18));
  // Distinct listeners per song: train (per-worker histograms) and test.
  col_tr.assign(n_s, 0);
  std::vector<int32_t> col_te(n_s, 0);
  {
    std::vector<std::vector<int32_t>> h(W);
    const std::vector<int64_t> cut = weighted_cuts(d->tr_off, n_tr, W);
    mr_par::parallel_for(W, [&](int64_t w0, int64_t w1, int) {
      for (int64_t w = w0; w < w1; ++w) {
        h[w].assign(n_s, 0);
        for (int64_t i = d->tr_off[cut[w]]; i < d->tr_off[cut[w + 1]]; ++i) h[w][d->tr_songs[i]]++;
      }
    }, 1, W);
    mr_par::parallel_for(n_s, [&](int64_t a, int64_t b, int) {
      for (int w = 0; w < W; ++w)
        for (int64_t s2 = a; s2 < b; ++s2) col_tr[s2] += h[w][s2];
    }, 4096);
  }
  for (int64_t i = 0; i < d->te_off[n_te]; ++i) col_te[d->te_songs[i]]++;
  {
    const int64_t s_bad = first_bad(n_s, [&](int64_t s2) {
      return d->song_count[s2] < col_tr[s2] + col_te[s2] || d->song_count[s2] <= 0;
    });
    if (s_bad >= 0)
      return fail(MR_E_INVALID, "song %d: count %d below its %d distinct listeners (or zero)", (int)s_bad,
                  d->song_count[s_bad], col_tr[s_bad] + col_te[s_bad]);
  }
  trace("validate");
  return MR_OK;
}

extern "C" {

const char* mr_last_error(void) { return g_err.c_str(); }
const char* mr_version(void) { return "mr_engine 0.2 (gfx950)"; }

int mr_options_default(mr_options* opt) {
  if (!opt) return fail(MR_E_INVALID, "null options");
  std::memset(opt, 0, sizeof *opt);
  opt->device = 0;
  opt->frac_bits = 32;
  opt->song_lo = 0;
  opt->song_hi = 0;
  opt->block_songs = 0;
  opt->out_dtype = MR_OUT_F32;
  opt->topk = 10;
  opt->dense = 1;
  opt->time_kernels = 0;
  opt->stage1 = 0;
  return MR_OK;
}

int mr_create(const mr_options* opt, mr_ctx** out) {
  if (!out) return fail(MR_E_INVALID, "null output pointer");
  *out = nullptr;
  mr_options o;
  if (opt) o = *opt; else mr_options_default(&o);
  if (o.frac_bits < 8 || o.frac_bits > 40) return fail(MR_E_INVALID, "frac_bits %d outside [8,40]", o.frac_bits);
  if (o.topk < 0 || o.topk > kMaxTopK) return fail(MR_E_INVALID, "topk %d outside [0,%d]", o.topk, kMaxTopK);
  if (o.out_dtype != MR_OUT_F32 && o.out_dtype != MR_OUT_F64) return fail(MR_E_INVALID, "bad out_dtype %d", o.out_dtype);
  if (o.block_songs < 0 || o.block_songs > (o.stage1 == 4 ? kMaxWideBlockSongs : kMaxBlockSongs) ||
      (o.block_songs % 256) != 0)
    return fail(MR_E_INVALID, "block_songs %d must be a multiple of 256 in [0,%d]", o.block_songs,
                o.stage1 == 4 ? kMaxWideBlockSongs : kMaxBlockSongs);
  if (o.stage1 < 0 || o.stage1 > 4 || o.stage1 == 3)
    return fail(MR_E_INVALID, "stage1 %d is not 0 (auto), 1 (fused), 2 (separate) or 4 (wide)", o.stage1);
  if (o.topk_lists != 0 && o.topk_lists != 1) return fail(MR_E_INVALID, "topk_lists %d not 0 or 1", o.topk_lists);
  if (o.ibm_route < 0 || o.ibm_route > 2)
    return fail(MR_E_INVALID, "ibm_route %d is not 0 (auto), 1 (two-hop) or 2 (co-listening index)", o.ibm_route);
  if (!o.dense && o.topk == 0) return fail(MR_E_INVALID, "dense=0 and topk=0: nothing to compute");
  if (o.stage1_chunk < 0 || o.stage1_chunk > kMaxLdsTrainUsers)
    return fail(MR_E_INVALID, "stage1_chunk %d outside [0,%d]", o.stage1_chunk, kMaxLdsTrainUsers);
  int ndev = 0;
  MR_HIP(hipGetDeviceCount(&ndev));
  if (o.device < 0 || o.device >= ndev) return fail(MR_E_INVALID, "device %d not present (%d devices)", o.device, ndev);
  MR_HIP(hipSetDevice(o.device));
  mr_ctx* c = new mr_ctx();
  c->opt = o;
  hipError_t e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking);
  if (e != hipSuccess) {
    delete c;
    return fail(MR_E_HIP, "hipStreamCreate: %s", hipGetErrorString(e));
  }
  for (int i = 0; i < 2 && e == hipSuccess; ++i) e = hipStreamCreateWithFlags(&c->side[i], hipStreamNonBlocking);
  if (e == hipSuccess) e = hipEventCreateWithFlags(&c->side_fork, hipEventDisableTiming);
  for (int i = 0; i < 2 && e == hipSuccess; ++i) e = hipEventCreateWithFlags(&c->side_join[i], hipEventDisableTiming);
  if (e != hipSuccess) {
    mr_destroy(c);
    return fail(MR_E_HIP, "side streams: %s", hipGetErrorString(e));
  }
  for (auto& ev : c->win) {
    e = hipEventCreate(&ev);
    if (e != hipSuccess) {
      ev = nullptr;
      mr_destroy(c);
      return fail(MR_E_HIP, "hipEventCreate: %s", hipGetErrorString(e));
    }
  }
  if (o.time_kernels) {
    c->ring.resize((size_t)mr_ctx::kRing * 3);
    for (auto& ev : c->ring) {
      e = hipEventCreate(&ev);
      if (e != hipSuccess) {
        ev = nullptr;
        mr_destroy(c);
        return fail(MR_E_HIP, "hipEventCreate: %s", hipGetErrorString(e));
      }
    }
  }
  *out = c;
  return MR_OK;
}

int mr_destroy(mr_ctx* c) {
  if (!c) return MR_OK;
  (void)hipSetDevice(c->opt.device);
  if (c->stream) (void)hipStreamSynchronize(c->stream);
  c->release_data();
  for (int i = 0; i < 2; ++i) {
    if (c->stage_ev[i]) (void)hipEventDestroy(c->stage_ev[i]);
  }
  for (auto& ev : c->ring) if (ev) (void)hipEventDestroy(ev);
  for (auto& ev : c->win) if (ev) (void)hipEventDestroy(ev);
  for (int i = 0; i < 2; ++i) {
    if (c->side[i]) { (void)hipStreamSynchronize(c->side[i]); (void)hipStreamDestroy(c->side[i]); }
    if (c->side_join[i]) (void)hipEventDestroy(c->side_join[i]);
  }
  if (c->side_fork) (void)hipEventDestroy(c->side_fork);
  if (c->stream) (void)hipStreamDestroy(c->stream);
  delete c;
  return MR_OK;
}

void* mr_stream(const mr_ctx* c) { return c ? (void*)c->stream : nullptr; }

int mr_load(mr_ctx* c, const mr_dataset* d) {
  if (!c || !d) return fail(MR_E_INVALID, "null argument");
  mr_par::PhaseTrace trace("MR_LOAD_TRACE", "mr_load");
  MR_HIP(hipSetDevice(c->opt.device));
  MR_HIP(hipStreamSynchronize(c->stream));
  c->ring_used = 0;
  c->release_data();
  const int n_tr = d->n_train_users, n_te = d->n_test_users, n_s = d->n_songs;
  std::vector<int32_t> col_tr;
  int rc;
  if ((rc = check_dataset(d, col_tr))) return rc;
  const int64_t nnz_tr = d->tr_off[n_tr];
  const int W = (int)std::max<int64_t>(1, std::min<int64_t>(mr_par::usable_cores(), nnz_tr >> 18));
  std::vector<int64_t> trs_off((size_t)n_s + 1, 0);
  for (int s2 = 0; s2 < n_s; ++s2) trs_off[s2 + 1] = trs_off[s2] + col_tr[s2];
  trace("counts");
  // Train users renumbered by distinct-song count, descending (ties by id),
  // unless opt.train_order = 1: the users of one wave then have segments of
  // similar length in every song tile, so no lane waits on one heavy
  // listener's long tail (heavy listeners dominate every neighbourhood).
  // Results do not change: every accumulation is an order-free integer sum
  // and the outputs are indexed by test user and song only. (A stable
  // counting sort by degree.)
  std::vector<int32_t> perm(std::max(1, n_tr));  // new id -> caller's id
  if (c->opt.train_order == 0 && n_tr > 0) {
    int64_t max_deg = 0;
    for (int v = 0; v < n_tr; ++v) max_deg = std::max(max_deg, d->tr_off[v + 1] - d->tr_off[v]);
    std::vector<int64_t> at((size_t)max_deg + 1, 0);
    for (int v = 0; v < n_tr; ++v) at[max_deg - (d->tr_off[v + 1] - d->tr_off[v])]++;
    int64_t run = 0;
    for (auto& x : at) { const int64_t n = x; x = run; run += n; }
    for (int v = 0; v < n_tr; ++v) perm[at[max_deg - (d->tr_off[v + 1] - d->tr_off[v])]++] = v;
  } else {
    for (int v = 0; v < n_tr; ++v) perm[v] = v;
  }
  std::vector<int64_t> p_off((size_t)n_tr + 1, 0);
  mr_par::parallel_for(n_tr, [&](int64_t a, int64_t b, int) {
    for (int64_t v = a; v < b; ++v) p_off[v] = d->tr_off[perm[v] + 1] - d->tr_off[perm[v]];
  });
  p_off[n_tr] = mr_par::exclusive_scan(p_off.data(), (int64_t)n_tr);
  mr_par::buffer<int32_t> p_songs((size_t)std::max<int64_t>(1, nnz_tr));
  std::vector<int32_t> p_len(std::max(1, n_tr));
  mr_par::parallel_dynamic(n_tr, 2048, [&](int64_t v, int) {
    const int o = perm[v];
    std::copy(d->tr_songs + d->tr_off[o], d->tr_songs + d->tr_off[o + 1], p_songs.begin() + p_off[v]);
    p_len[v] = d->tr_len[o];
  });
  const int64_t* tr_off = p_off.data();
  const int32_t* tr_songs = p_songs.data();
  const int32_t* tr_len = p_len.data();
  trace("renumber");
  // Transpose song -> train users, lists ascending in v: worker w owns a
  // contiguous range of (new) users and a private cursor per song.
  const std::vector<int64_t> ucut = weighted_cuts(tr_off, n_tr, W);
  mr_par::buffer<int32_t> trs_users((size_t)std::max<int64_t>(1, trs_off[n_s]));
  {
    std::vector<std::vector<int64_t>> pos(W);
    mr_par::parallel_for(W, [&](int64_t w0, int64_t w1, int) {
      for (int64_t w = w0; w < w1; ++w) {
        pos[w].assign(n_s, 0);
        for (int64_t i = tr_off[ucut[w]]; i < tr_off[ucut[w + 1]]; ++i) pos[w][tr_songs[i]]++;
      }
    }, 1, W);
    mr_par::parallel_for(n_s, [&](int64_t a, int64_t b, int) {
      for (int64_t s2 = a; s2 < b; ++s2) {
        int64_t at = trs_off[s2];
        for (int w = 0; w < W; ++w) {
          const int64_t n = pos[w][s2];
          pos[w][s2] = at;
          at += n;
        }
      }
    }, 4096);
    mr_par::parallel_for(W, [&](int64_t w0, int64_t w1, int) {
      for (int64_t w = w0; w < w1; ++w)
        for (int64_t v = ucut[w]; v < ucut[w + 1]; ++v)
          for (int64_t i = tr_off[v]; i < tr_off[v + 1]; ++i) trs_users[pos[w][tr_songs[i]]++] = (int32_t)v;
    }, 1, W);
  }
  trace("transpose");
  // Shard geometry and launch shape.
  const int lo = c->opt.song_lo, hi = c->opt.song_hi > 0 ? c->opt.song_hi : n_s;
  if (lo < 0 || hi > n_s || lo >= hi) return fail(MR_E_INVALID, "song shard [%d,%d) invalid for %d songs", lo, hi, n_s);
  const int width = hi - lo;
  const int k = c->opt.topk;
  const int shape = pick_shape(c->opt, n_tr, n_te);
  const bool fused = shape == kShapeFused, wide = shape == kShapeWide;
  if (wide && k > kMaxTopkLarge)
    return fail(MR_E_INVALID, "wide shape keeps topk <= %d (got %d)", kMaxTopkLarge, k);
  if (fused && n_tr > kMaxFusedTrainUsers)
    return fail(MR_E_INVALID, "fused stage 1 needs n_train_users <= %d (got %d)", kMaxFusedTrainUsers, n_tr);
  // Stage 1 of the separate / wide shapes: one LDS chunk of train users per workgroup.
  const int chunk = stage1_chunk_for(c->opt, n_tr);
  if ((n_tr + chunk - 1) / chunk > kMaxChunks)
    return fail(MR_E_INVALID, "stage1_chunk %d gives more than %d chunks", chunk, kMaxChunks);
  const int n_chunks = (std::max(1, n_tr) + chunk - 1) / chunk;
  int bs;
  if (wide) {
    // the widest tile the LDS holds (every tile re-walks the user's whole
    // neighbour list), then balanced: n_tiles = ceil(width / max), bs =
    // ceil(width / n_tiles) rounded up to 256
    const int bmax = wide_bmax(k, n_chunks);
    const long long nt = ((long long)width + bmax - 1) / bmax;
    bs = c->opt.block_songs > 0 ? c->opt.block_songs
                                : (int)std::min<long long>(bmax, (((long long)width + nt - 1) / nt + 255) / 256 * 256);
    if (wide_lds<kWideThreads>(bs, k, n_chunks).total > kLdsBytes)
      return fail(MR_E_INVALID, "wide shape: block_songs %d needs more than %d B of LDS", bs, kLdsBytes);
  } else {
    bs = c->opt.block_songs > 0 ? c->opt.block_songs : auto_block_songs(width, n_te, fused, k, n_tr);
  }
  if (fused && bs > 8192) return fail(MR_E_INVALID, "fused stage 1 needs block_songs <= 8192 (got %d)", bs);
  if (!wide && k > kMaxTopkLarge && bs > kMaxTopkTile)
    return fail(MR_E_INVALID, "with topk > %d block_songs must be <= %d (got %d)", kMaxTopkLarge, kMaxTopkTile, bs);
  const int n_tiles = (width + bs - 1) / bs;
  // Per-song / per-user fixed-point tables, computed once on the host with
  // correctly rounded std::sqrt (java.lang.Math.sqrt semantics, MR:147/237).
  const int F = c->opt.frac_bits;
  const double two_f = std::ldexp(1.0, F);
  std::vector<double> sqrt_c(n_s), sqrt_tr(std::max(1, n_tr)), sqrt_te(n_te);
  std::vector<long long> q_song(n_s);
  std::vector<float> rsq_c(n_s);
  mr_par::parallel_for(n_s, [&](int64_t a, int64_t b, int) {
    for (int64_t s2 = a; s2 < b; ++s2) {
      sqrt_c[s2] = std::sqrt((double)d->song_count[s2]);
      q_song[s2] = (long long)std::nearbyint(two_f / sqrt_c[s2]);
      rsq_c[s2] = sqrt_c[s2] > 0.0 ? (float)(1.0 / sqrt_c[s2]) : 0.f;
    }
  });
  mr_par::parallel_for(n_tr, [&](int64_t a, int64_t b, int) {
    for (int64_t v = a; v < b; ++v) sqrt_tr[v] = std::sqrt((double)tr_len[v]);
  });
  for (int u = 0; u < n_te; ++u) sqrt_te[u] = std::sqrt((double)d->te_len[u]);
  // Tile-major train CSR over the shard's songs: for tile t, user v, the
  // tile-local ids of S(v) ∩ [lo + t*bs, lo + (t+1)*bs) live at
  // tsongs[toff[t*n_tr + v] .. toff[t*n_tr + v + 1]) (entries ordered by
  // (tile, user, song)), so neighbouring users' segments share cache lines.
  // Every user writes only its own (tile, user) slots: parallel over users.
  const size_t n_tv = (size_t)n_tiles * n_tr;
  mr_par::buffer<int32_t> toff(n_tv + 1);
  mr_par::parallel_for((int64_t)n_tv, [&](int64_t a, int64_t b, int) { std::fill(toff.begin() + a, toff.begin() + b, 0); });
  mr_par::parallel_for(W, [&](int64_t w0, int64_t w1, int) {
    for (int64_t w = w0; w < w1; ++w)
      for (int64_t v = ucut[w]; v < ucut[w + 1]; ++v)
        for (int64_t i = tr_off[v]; i < tr_off[v + 1]; ++i) {
          const int s2 = tr_songs[i];
          if (s2 >= lo && s2 < hi) toff[(size_t)((s2 - lo) / bs) * n_tr + v]++;
        }
  }, 1, W);
  const int64_t n_entries = mr_par::exclusive_scan(toff.data(), (int64_t)n_tv);
  toff[n_tv] = (int32_t)n_entries;
  // padded to whole 8-B words (+1): the wide kernel loads a segment's ids as
  // aligned 4-id words
  mr_par::buffer<uint16_t> tsongs((std::max<int64_t>(1, n_entries) + 3) / 4 * 4 + 4);
  std::fill(tsongs.begin() + n_entries, tsongs.end(), (uint16_t)0);
  mr_par::parallel_for(W, [&](int64_t w0, int64_t w1, int) {
    for (int64_t w = w0; w < w1; ++w)
      for (int64_t v = ucut[w]; v < ucut[w + 1]; ++v) {
        int cur_t = -1;
        int32_t at = 0;
        for (int64_t i = tr_off[v]; i < tr_off[v + 1]; ++i) {  // songs ascend, so tiles do
          const int s2 = tr_songs[i];
          if (s2 < lo || s2 >= hi) continue;
          const int t = (s2 - lo) / bs;
          if (t != cur_t) {
            cur_t = t;
            at = toff[(size_t)t * n_tr + v];
          }
          tsongs[at++] = (uint16_t)(s2 - lo - t * bs);
        }
      }
  }, 1, W);
  trace("tiles");
  // Separate / wide shapes: test-user batches so the neighbour lists fit 8 GiB.
  const int cap = n_chunks * chunk;
  // one launch's neighbour lists (batch x cap x 12 B): an eighth of the free
  // device memory, 8-32 GiB (C5's 2,000 users in one launch on a 288 GB
  // MI355X; allocated at the first two-hop run, ensure_nbr)
  size_t free_b0 = 0, total_b0 = 0;
  MR_HIP(hipMemGetInfo(&free_b0, &total_b0));
  const size_t budget = std::min<size_t>((size_t)32 << 30, std::max<size_t>((size_t)8 << 30, free_b0 / 8)) /
                        (size_t)std::max(1, c->dev_share);
  const int batch = fused ? n_te
                          : (int)std::max<size_t>(1, std::min<size_t>(std::min(n_te, 65528),
                                                                      budget / ((size_t)cap * 12)));

  // ItemBasedModel route (mr_options.ibm_route). The co-listening index has
  // one row per distinct test-visible song with train listeners, heaviest
  // first; row r's pool range holds at most min(width, Σ_{v ∈ L_tr(s2)}
  // |S(v) ∩ shard|) entries (its non-zero counts over the shard's songs).
  int route = 1;
  std::vector<int32_t> row_song, te_row;
  std::vector<int64_t> row_base;
  std::vector<int32_t> heavy_rows, light_rows, row_slots;
  int dense_div = kCoocDenseDiv;
  int n_heavy32 = 0, n_big16 = 0, tcap16 = 0, tcap32 = 0;
  int32_t max_shard_deg = 0;
  int grp = 0, n_grp = 0, urec_words = 0, lrec_words = 0;  // k_cooc_group (0: the per-tile k_cooc_build)
  std::vector<int64_t> row_reads;
  int64_t pool_cap = 0;
  {
    const char* why = nullptr;
    int32_t max_c = 0;
    if (!wide) why = "the wide shape only";
    else if (bs > kCoocMaxTile) why = "song tiles <= 32768";
    if (!why && c->opt.ibm_route != 1) {
      const int64_t nte = d->te_off[n_te];
      std::vector<int32_t> row_of(n_s, -1);
      for (int64_t i = 0; i < nte; ++i) {
        const int s2 = d->te_songs[i];
        if (col_tr[s2] > 0 && row_of[s2] < 0) { row_of[s2] = 0; row_song.push_back(s2); }
      }
      std::sort(row_song.begin(), row_song.end(), [&](int x, int y) {
        return col_tr[x] != col_tr[y] ? col_tr[x] > col_tr[y] : x < y;
      });
      for (size_t r = 0; r < row_song.size(); ++r) {
        row_of[row_song[r]] = (int32_t)r;
        max_c = std::max(max_c, col_tr[row_song[r]]);
      }
      te_row.resize(std::max<int64_t>(1, nte));
      for (int64_t i = 0; i < nte; ++i) te_row[i] = row_of[d->te_songs[i]];
      if (max_c > (int32_t)kCoocCntMask) why = "train listener counts < 131072";
      // the row descriptors hold 32-bit listener-list starts and k_urec's
      // records 32-bit shard-row bases (shard entries <= train entries)
      else if (trs_off[n_s] >= (int64_t)INT32_MAX) why = "train entries < 2^31";
      else if ((long long)row_song.size() * n_tiles > INT32_MAX) why = "rows x tiles < 2^31";
    }
    if (!why && c->opt.ibm_route != 1) {
      // |S(v) ∩ [lo, hi)| of every (renumbered) train user, then the row bounds
      std::vector<int32_t> deg((size_t)std::max(1, n_tr));
      mr_par::parallel_for(n_tr, [&](int64_t a, int64_t b, int) {
        for (int64_t v = a; v < b; ++v) {
          const int32_t* r0 = tr_songs + tr_off[v];
          const int32_t* r1 = tr_songs + tr_off[v + 1];
          deg[v] = (int32_t)(std::lower_bound(r0, r1, hi) - std::lower_bound(r0, r1, lo));
        }
      });
      for (int v = 0; v < n_tr; ++v) max_shard_deg = std::max(max_shard_deg, deg[v]);
      const int64_t nr = (int64_t)row_song.size();
      row_base.assign((size_t)nr + 1, 0);
      row_reads.assign((size_t)nr, 0);
      mr_par::parallel_for(nr, [&](int64_t a, int64_t b, int) {
        for (int64_t r = a; r < b; ++r) {
          const int s2 = row_song[r];
          int64_t sum = 0;
          for (int64_t i = trs_off[s2]; i < trs_off[s2 + 1]; ++i) sum += deg[trs_users[i]];
          row_reads[r] = (trs_off[s2 + 1] - trs_off[s2]) + sum;
          row_base[r] = std::min<int64_t>(sum, width);  // the row's non-zeros: its sparse bound
        }
      }, 256);
      // auto: the cost model of cooc_pays (the rows' bounds = sparse entry bounds here)
      if (c->opt.ibm_route == 0) {
        double e_est = 0.0;
        for (int64_t i = 0; i < d->te_off[n_te]; ++i)
          if (te_row[i] >= 0) e_est += (double)row_base[te_row[i]];
        double v_est = 0.0;
        for (int u = 0; u < n_te; ++u) {
          double sc = 0.0;
          for (int64_t i = d->te_off[u]; i < d->te_off[u + 1]; ++i) sc += col_tr[d->te_songs[i]];
          v_est += std::min<double>(sc, n_tr);
        }
        if (!cooc_pays(v_est * n_tiles, e_est, row_base, row_reads, row_song, col_tr, n_tiles))
          why = "a cheaper estimate than the two-hop route (auto)";
      }
    }
    if (!why && c->opt.ibm_route != 1) {
      // light rows (k_cooc_light): the bound fits half the hash slots
      const int64_t nr = (int64_t)row_song.size();
      const bool light_ok = width <= kLightMaxWidth && n_tiles <= kLightMaxTiles && cooc_light_opt();
      // a light row's table: the smallest power of 2 of at least bound * 100 / lload slots (the
      // entry bound at most lload % of the slots), at most light_slots_max (MR_COOC_LIGHT_MAX /
      // MR_COOC_LIGHT_LOAD: A/B knobs; defaults 32768 slots, 80 %)
      // narrow shard: the group kernel would hold every tile in one pass
      // (the conditions of its set-up below, before the heavy rows are known)
      bool narrow = false;
      if (cooc_group_opt() && 1 + (n_tiles + 2) / 2 <= 32 && max_shard_deg <= 65535 &&
          n_tiles <= std::min(kMaxGroupTiles, cooc_group_max_opt()))
        narrow = cooc_group_lds(bs, n_tiles) <= kLdsBytes;
      const int64_t lload = cooc_light_load_opt(), light_slots_max = cooc_light_max_opt(narrow);
      dense_div = cooc_dense_div_opt();
      // a dense segment holds whole interleaved blocks (cooc_dense_words):
      // the words past its songs' bytes, over every tile, on each heavy row's bound
      int64_t dense_pad = 0;
      for (int t = 0; t < n_tiles; ++t) {
        const int bw = (int)(std::min<int64_t>(width, (int64_t)(t + 1) * bs) - (int64_t)t * bs);
        dense_pad += cooc_dense_words(bw) - (bw + 3) / 4;
      }
      // whole 16-B words: every row's bound stays a multiple of 4 words, so
      // every row (placed by the exclusive scan below) starts 16-B aligned for
      // the scorer's dvec_t loads and k_cooc_group's chunk_t stores
      dense_pad = (dense_pad + 3) & ~(int64_t)3;
      row_slots.assign((size_t)std::max<int64_t>(1, nr), 0);
      for (int64_t r = 0; r < nr; ++r) {
        if (light_ok && row_base[r] * 100 <= light_slots_max * lload && col_tr[row_song[r]] <= (int32_t)kLightCntMask) {
          int sl = 1024;
          while ((int64_t)sl * lload < row_base[r] * 100) sl <<= 1;
          row_slots[r] = sl;
          // lanes per listener of rows_walk: the largest power of 2 G <= 16
          // with 6 G <= the row's shard entries per listener (>= 6 per lane)
          const int64_t c = col_tr[row_song[r]];
          const int64_t per = c > 0 ? (row_reads[r] - c) / c : 0;
          int glog = 0;
          while (glog < 4 && ((int64_t)6 << (glog + 1)) <= per) ++glog;
          row_slots[r] |= glog << kLightGlogShift;
          light_rows.push_back((int32_t)r);
          row_base[r] = (row_base[r] + 3) & ~(int64_t)3;
        } else {
          // k_cooc_build: a tile's segment is sparse (its non-zeros) or dense
          // (<= kCoocDenseDiv x its non-zeros, <= the tile's songs), in whole
          // 16-B words (32-B for u32 counts)
          // (dense: count bytes <= kCoocDenseDiv / 4 x the non-zeros, + excess entries <= the non-zeros)
          const int64_t nz = row_base[r];
          const int64_t dn = std::max<int64_t>(1, std::min<int64_t>(dense_div, width)) * nz;
          row_base[r] = ((std::min<int64_t>(width, dn) + nz + 3) & ~(int64_t)3) + 8 * (int64_t)n_tiles + dense_pad;
          heavy_rows.push_back((int32_t)r);
        }
      }
      // heavy rows whose counts may pass 65535 first (u32 counters), the rest
      // keep their order (u16-pair counters, k_cooc_build<.., true>)
      const bool all32 = !MR_COOC_P16 || cooc_dense32_opt();
      std::stable_partition(heavy_rows.begin(), heavy_rows.end(), [&](int32_t r) {
        return all32 || col_tr[row_song[r]] >= 65536;
      });
      for (int32_t r : heavy_rows) n_heavy32 += (all32 || col_tr[row_song[r]] >= 65536) ? 1 : 0;
      // Big rows (>= kCoocBigRow listeners, and every u32 row): one workgroup
      // per (row, tile), each tile a fixed slot of tcap words (the larger of a
      // dense segment and the longest sparse one), so the row's tiles run in
      // parallel. Rows are heaviest first, so the big rows of each kind lead.
      const int sparse_max = dense_div > 0 ? (bs + dense_div - 1) / dense_div : bs;
      // a dense segment: the count bytes + at most one excess entry per song
      tcap32 = (std::max(sparse_max, cooc_dense_words(bs) + bs) + 7) & ~7;
      tcap16 = tcap32;
      n_big16 = 0;
      for (size_t i = n_heavy32; i < heavy_rows.size(); ++i) {
        if (col_tr[row_song[heavy_rows[i]]] < kCoocBigRow) break;
        n_big16++;
      }
      for (size_t i = 0; i < heavy_rows.size(); ++i)
        if ((int)i < n_heavy32 + n_big16)
          row_base[heavy_rows[i]] = (int64_t)n_tiles * ((int)i < n_heavy32 ? tcap32 : tcap16);
      // The u16 heavy rows by tile groups (k_cooc_group) when the per-user
      // records fit (one 128-B line: n_tiles <= 61, u16 starts: shard rows
      // < 65536 songs): the widest group whose counters fit the LDS.
      urec_words = 1 + (n_tiles + 2) / 2;
      if (cooc_group_opt() && (int)heavy_rows.size() > n_heavy32 && urec_words <= 32 && max_shard_deg <= 65535) {
        grp = std::min(std::min(n_tiles, kMaxGroupTiles), cooc_group_max_opt());
        while (grp > 0 && cooc_group_lds(bs, grp) > kLdsBytes) --grp;
      }
      if (grp > 0) {
        int w2 = 1;
        while (w2 < urec_words) w2 <<= 1;
        urec_words = w2;
        n_grp = (n_tiles + grp - 1) / grp;
        // lanes per listener of rows_walk: ~6 entries of the group per lane
        for (size_t i = n_heavy32; i < heavy_rows.size(); ++i) {
          const int32_t r = heavy_rows[i];
          const int64_t cr = col_tr[row_song[r]];
          const int64_t per = cr > 0 ? (row_reads[r] - cr) / cr * grp / n_tiles : 0;
          int glog = 0;
          while (glog < 4 && ((int64_t)6 << (glog + 1)) <= per) ++glog;
          // rows under kCoocBigRow listeners: every listener held by a lane
          // group for the whole row (cooc_group_pipelined)
          if ((int)i >= n_heavy32 + n_big16)
            while (glog > 0 && cr > (int64_t)(cooc_group_nt_opt() >> glog) * kGroupPipeR) --glog;
          row_slots[r] = glog << kLightGlogShift;
        }
      } else {
        urec_words = 0;
      }
      pool_cap = mr_par::exclusive_scan(row_base.data(), nr);
      row_base[nr] = pool_cap;
      for (int64_t r = 0; r < nr; ++r)
        if (row_base[r] & 3)
          return fail(MR_E_STATE, "co-listening index: row %lld starts at word %lld (not 16-B aligned)",
                      (long long)r, (long long)row_base[r]);
      // the pool and the per-(row, listener) record tables built beside it:
      // lrec (the u16 heavy rows' listeners, lrec_words each), llrec (8 B per
      // light-row listener) and urec (alive during the load), against half the
      // free device memory (the share of it a group's context may use)
      double rec_b = 0.0;
      {
        int64_t n_lrec = 0, n_llrec = 0;
        for (size_t i = 0; i < heavy_rows.size(); ++i)
          if (grp > 0 && (int)i >= n_heavy32) n_lrec += col_tr[row_song[heavy_rows[i]]];
        for (int32_t r : light_rows) n_llrec += col_tr[row_song[r]];
        int lw = 1;
        const int ng = grp > 0 ? (n_tiles + grp - 1) / grp : 0;
        while (2 * (lw - 1) < ng + 1) lw <<= 1;
        rec_b = 4.0 * (double)n_lrec * lw + 8.0 * (double)n_llrec + 4.0 * (double)n_tr * urec_words;
      }
      size_t free_b = 0, total_b = 0;
      MR_HIP(hipMemGetInfo(&free_b, &total_b));
      if ((double)pool_cap * 4.0 + rec_b > 0.5 * (double)free_b / std::max(1, c->dev_share))
        why = "a pool within half the free device memory";
    }
    if (c->opt.ibm_route == 2 && why)
      return fail(MR_E_INVALID, "ibm_route 2 (co-listening index) needs %s", why);
    route = (c->opt.ibm_route != 1 && !why) ? 2 : 1;
    trace("route");
  }

  hipStream_t st = c->stream;
  if ((rc = dev_upload(c->tr_off, reinterpret_cast<const long long*>(tr_off), (size_t)n_tr + 1, st))) return rc;
  if ((rc = dev_upload(c->te_off, reinterpret_cast<const long long*>(d->te_off), (size_t)n_te + 1, st))) return rc;
  if ((rc = dev_upload(c->te_songs, d->te_songs, (size_t)d->te_off[n_te], st))) return rc;
  if ((rc = dev_upload(c->trs_off, reinterpret_cast<const long long*>(trs_off.data()), trs_off.size(), st))) return rc;
  if ((rc = dev_upload(c->trs_users, trs_users.data(), (size_t)trs_off[n_s], st))) return rc;
  if ((rc = dev_upload(c->q_song, q_song.data(), q_song.size(), st))) return rc;
  if ((rc = dev_upload(c->sqrt_c, sqrt_c.data(), sqrt_c.size(), st))) return rc;
  if (wide && (rc = dev_upload(c->rsq_c, rsq_c.data(), rsq_c.size(), st))) return rc;
  if ((rc = dev_upload(c->sqrt_tr, sqrt_tr.data(), sqrt_tr.size(), st))) return rc;
  if ((rc = dev_upload(c->sqrt_te, sqrt_te.data(), sqrt_te.size(), st))) return rc;
  if ((rc = dev_upload(c->toff, toff.data(), toff.size(), st))) return rc;
  if ((rc = dev_upload(c->tsongs, tsongs.data(), tsongs.size(), st))) return rc;
  if (!fused && n_chunks > 1) {
    // Chunk boundaries of every listener list (sorted by train user), built on
    // the device from the uploaded transpose: the chunked stage 1 reads its
    // sub-list bounds instead of searching (n_s x (n_chunks + 1) ints).
    const int nc1 = n_chunks + 1;
    const size_t n_sb = (size_t)n_s * nc1;
    if ((rc = dev_alloc(c->sbound, n_sb))) return rc;
    const int grid = (int)std::min<size_t>(8192, (n_sb + 255) / 256);
    hipLaunchKernelGGL(k_sbound, dim3(grid), dim3(256), 0, st, c->trs_off.p, c->trs_users.p, n_s, nc1, chunk,
                       c->sbound.p);
    MR_HIP(hipGetLastError());
  }
  if (fused) {  // n_tr <= 4096 and bs <= 65536: both halves fit 16 bits
    std::vector<uint32_t> tpack(tsongs.size(), 0u);
    for (size_t t = 0; t < (size_t)n_tiles; ++t)
      for (int v = 0; v < n_tr; ++v)
        for (int32_t i = toff[t * n_tr + v]; i < toff[t * n_tr + v + 1]; ++i)
          tpack[i] = ((uint32_t)v << 16) | tsongs[i];
    if ((rc = dev_upload(c->tpack, tpack.data(), tpack.size(), st))) return rc;
    // The songsToUsersMap lookup (MR:232) of every test-visible song, resolved
    // once: its listener range in trs_users and its ibm weight.
    const size_t nte = (size_t)d->te_off[n_te];
    std::vector<int2> rng(std::max<size_t>(1, nte));
    std::vector<long long> tq(std::max<size_t>(1, nte));
    for (size_t i = 0; i < nte; ++i) {
      const int s2 = d->te_songs[i];
      rng[i] = make_int2((int)trs_off[s2], (int)(trs_off[s2 + 1] - trs_off[s2]));
      tq[i] = q_song[s2];
    }
    if ((rc = dev_upload(c->te_rng, rng.data(), rng.size(), st))) return rc;
    if ((rc = dev_upload(c->te_q, tq.data(), tq.size(), st))) return rc;
    // Stage 1's walk schedule: per test user, its (song, listener) entries in
    // song order as (trs_users index, slot of the song in T(u)) — the segment
    // each flattened entry falls in, which the kernel otherwise finds per step
    // by a prefix scan and a binary search. Index metadata like te_rng (it
    // names positions, not listener ids or weights); skipped past 2^26 entries.
    std::vector<long long> h_sched_off((size_t)n_te + 1, 0);
    for (int u = 0; u < n_te; ++u) {
      long long n = 0;
      for (long long i = d->te_off[u]; i < d->te_off[u + 1]; ++i) n += rng[(size_t)i].y;
      h_sched_off[(size_t)u + 1] = h_sched_off[(size_t)u] + n;
    }
    const long long n_sched = h_sched_off[(size_t)n_te];
    if (fused_sched_opt() && n_sched <= (1ll << 26)) {
      std::vector<uint2> sched(std::max<long long>(1, n_sched));
      size_t o = 0;
      for (int u = 0; u < n_te; ++u)
        for (long long i = d->te_off[u]; i < d->te_off[u + 1]; ++i)
          for (int e = 0; e < rng[(size_t)i].y; ++e)
            sched[o++] = make_uint2((unsigned)(rng[(size_t)i].x + e), (unsigned)(i - d->te_off[u]));
      if ((rc = dev_upload(c->te_sched, sched.data(), sched.size(), st))) return rc;
      if ((rc = dev_upload(c->sched_off, h_sched_off.data(), h_sched_off.size(), st))) return rc;
    }
  }  // (separate / wide shapes: neighbour lists allocated by the first two-hop run, ensure_nbr)
  if (route == 2) {
    const size_t nr = row_song.size();
    if ((rc = dev_upload(c->row_song, row_song.data(), nr, st))) return rc;
    if ((rc = dev_upload(c->te_row, te_row.data(), te_row.size(), st))) return rc;
    if ((rc = dev_upload(c->row_base, reinterpret_cast<const long long*>(row_base.data()), nr + 1, st))) return rc;
    if ((rc = dev_alloc(c->row_nnz, nr))) return rc;
    if ((rc = dev_alloc(c->seg_off, nr * n_tiles))) return rc;
    if ((rc = dev_alloc(c->seg_len, nr * n_tiles))) return rc;
    if ((rc = dev_alloc(c->pool, (size_t)pool_cap))) return rc;
    // heavy rows, then light rows with large tables, then the small-table ones
    std::stable_sort(light_rows.begin(), light_rows.end(), [&](int32_t x, int32_t y) {
      return light_tier(row_slots[x] & kLightSlotsMask, n_tiles) < light_tier(row_slots[y] & kLightSlotsMask, n_tiles);
    });
    std::vector<int32_t> order(heavy_rows);
    order.insert(order.end(), light_rows.begin(), light_rows.end());
    if ((rc = dev_upload(c->rows_order, order.data(), order.size(), st))) return rc;
    int64_t n_lrec = 0;   // k_cooc_group's records: the u16 heavy rows' listeners
    int64_t n_llrec = 0;  // k_cooc_light*'s records: the light rows' listeners
    {
      std::vector<int4> rd(std::max<size_t>(1, order.size()));
      for (size_t i = 0; i < order.size(); ++i) {
        const int32_t r = order[i], s2 = row_song[r];
        const int cnt = (int)(trs_off[s2 + 1] - trs_off[s2]);
        int z = (int)trs_off[s2];  // the first listener in trs_users
        if (grp > 0 && (int)i >= n_heavy32 && i < heavy_rows.size()) {  // the first record in lrec
          z = (int)n_lrec;
          n_lrec += cnt;
        } else if (i >= heavy_rows.size()) {  // a light row: its first range record in llrec
          z = (int)n_llrec;
          n_llrec += cnt;
        }
        rd[i] = make_int4(r, row_slots[r], z, cnt);
      }
      if ((rc = dev_upload(c->rdesc, rd.data(), rd.size(), st))) return rc;
      MR_HIP(hipStreamSynchronize(st));
    }
    if ((rc = dev_upload(c->row_slots, row_slots.data(), row_slots.size(), st))) return rc;
    if (!light_rows.empty() || grp > 0) {
      // the shard's train rows, shard-local song ids (k_cooc_light's and
      // k_cooc_group's input)
      std::vector<int64_t> so((size_t)n_tr + 1, 0);
      mr_par::parallel_for(n_tr, [&](int64_t a, int64_t b, int) {
        for (int64_t v = a; v < b; ++v) {
          const int32_t* r0 = tr_songs + tr_off[v];
          const int32_t* r1 = tr_songs + tr_off[v + 1];
          so[v] = std::lower_bound(r0, r1, hi) - std::lower_bound(r0, r1, lo);
        }
      });
      so[n_tr] = mr_par::exclusive_scan(so.data(), (int64_t)n_tr);
      // + 4 zero entries: rows_walk's 16-B chunk loads never leave the buffer
      mr_par::buffer<uint32_t> ss((size_t)so[n_tr] + 4);
      std::fill(ss.begin() + so[n_tr], ss.end(), 0u);
      mr_par::parallel_for(n_tr, [&](int64_t a, int64_t b, int) {
        for (int64_t v = a; v < b; ++v) {
          const int32_t* r0 = std::lower_bound(tr_songs + tr_off[v], tr_songs + tr_off[v + 1], lo);
          for (int64_t i = 0; i < so[v + 1] - so[v]; ++i) ss[so[v] + i] = (uint32_t)(r0[i] - lo);
        }
      });
      if ((rc = dev_upload(c->sr_off, reinterpret_cast<const long long*>(so.data()), so.size(), st))) return rc;
      if ((rc = dev_upload(c->sr_songs, ss.data(), ss.size(), st))) return rc;
      if (!light_rows.empty()) {  // the light rows' listener ranges
        if ((rc = dev_alloc(c->llrec, (size_t)std::max<int64_t>(1, n_llrec)))) return rc;
        hipLaunchKernelGGL(k_llrec, dim3((unsigned)light_rows.size()), dim3(256), 0, st,
                           c->rdesc.p + heavy_rows.size(), c->row_song.p, c->trs_off.p, c->trs_users.p, c->sr_off.p,
                           c->llrec.p);
        MR_HIP(hipGetLastError());
      }
      if (grp > 0) {  // k_cooc_group's records, on the device: per user (tile starts), then per (row, listener)
        if ((rc = dev_alloc(c->urec, (size_t)std::max(1, n_tr) * urec_words))) return rc;
        hipLaunchKernelGGL(k_urec, dim3((std::max(1, n_tr) + 255) / 256), dim3(256), 0, st, c->sr_off.p,
                           c->sr_songs.p, n_tr, n_tiles, bs, urec_words, c->urec.p);
        MR_HIP(hipGetLastError());
        lrec_words = 1;  // base + (n_grp + 1) u16 starts, a power of 2 of words
        while (2 * (lrec_words - 1) < n_grp + 1) lrec_words <<= 1;
        if ((rc = dev_alloc(c->lrec, (size_t)std::max<int64_t>(1, n_lrec) * lrec_words))) return rc;
        const int n16 = (int)heavy_rows.size() - n_heavy32;
        if (n16 > 0)
          hipLaunchKernelGGL(k_lrec, dim3(n16), dim3(256), 0, st, c->rdesc.p + n_heavy32, c->row_song.p,
                             c->trs_off.p, c->trs_users.p, c->urec.p, urec_words, n_tiles, grp, n_grp, lrec_words,
                             c->lrec.p);
        MR_HIP(hipGetLastError());
        MR_HIP(hipStreamSynchronize(st));
        c->urec.release();  // (lrec holds what the runs need)
      }
      MR_HIP(hipStreamSynchronize(st));  // so / ss die here
    }
  }
  if (k > 0) {
    // wide: per-tile candidates of one launch (a neighbour batch; the
    // co-listening route launches up to 65528 users at once)
    const int cand_users = !wide ? n_te : route == 2 ? std::max(batch, std::min(n_te, 65528)) : batch;
    const size_t nc = (size_t)cand_users * n_tiles * k;
    if ((rc = dev_alloc(c->cand_key, nc))) return rc;
    if ((rc = dev_alloc(c->cand_song, nc))) return rc;
    // keys then songs in ONE record block: the send buffer of the song-shard
    // exchange (one all-gather of rec bytes per shard, mr_topk_merge_records_async)
    const size_t nk = (size_t)n_te * k;
    if ((rc = dev_alloc(c->top_key, (size_t)topk_record_bytes(nk) / 8))) return rc;
    c->top_song.p = reinterpret_cast<int*>(c->top_key.p + nk);
    c->top_song.n = nk;
    c->top_song.own = false;
    if ((rc = dev_alloc(c->top_score, (size_t)n_te * k))) return rc;
    // (the in-launch hand-off's per-user counters, one line each: fused / separate shapes only)
    const size_t n_ctr = wide ? (size_t)n_te : (size_t)n_te * kCounterStride;
    if ((rc = dev_alloc(c->counter, n_ctr))) return rc;
    MR_HIP(hipMemsetAsync(c->counter.p, 0, n_ctr * sizeof(unsigned), st));
  }
  const size_t esz = c->opt.out_dtype == MR_OUT_F64 ? 8 : 4;
  if ((rc = dev_alloc(c->dense, c->opt.dense ? (size_t)n_te * width * esz : 1))) return rc;
  if ((rc = dev_alloc(c->flag, 1))) return rc;

  c->fused = fused;
  c->shape = shape;
  c->ibm_route = route;
  c->cooc_nt = cooc_nt_opt();
  {  // the candidate-only tile top-k (wide_cand_topk): top-k-only wide runs
    const char* e = std::getenv("MR_WIDE_CAND");
    const int nt = route == 2 ? c->cooc_nt : kWideThreads;  // the scoring kernel's threads
    c->cand_on = wide && !c->opt.dense && k >= 1 && k <= nt / 16 && !c->opt.topk_lists && bs <= kCandE * nt &&
                 !(e && e[0] == '0');
  }
  c->wide_lds = wide ? (size_t)wide_lds<kWideThreads>(bs, k, n_chunks).total : 0;
  pick_kernels<MR_UBM>(c);
  pick_kernels<MR_IBM>(c);
  c->score_lds = wide ? c->wide_lds
                      : (size_t)score_lds(bs, fused ? n_tr : 0, k, n_tiles, fused ? 0 : n_chunks).total;
  if (c->score_lds > 160 * 1024)
    return fail(MR_E_INVALID, "scoring kernel needs %zu B of LDS (> 160 KiB): lower block_songs or topk",
                c->score_lds);
  c->nbr_lds = (size_t)align16(chunk * 8) + kThreads * 16 + (kThreads + 4 + kWaves) * 4;
  for (int m = 0; m < 2; ++m) {
    MR_HIP(hipFuncSetAttribute((const void*)c->score_kernel[m], hipFuncAttributeMaxDynamicSharedMemorySize,
                               (int)c->score_lds));
    MR_HIP(hipFuncSetAttribute((const void*)c->nbr_kernel[m], hipFuncAttributeMaxDynamicSharedMemorySize,
                               (int)c->nbr_lds));
  }
  if (route == 2) {
    c->n_rows = (int)row_song.size();
    c->pool_cap = pool_cap;
    // the score kernel's row descriptors (40 B each: sparse + dense views) in its top-k scratch
    const WideLds<kWideThreads> WL = c->cooc_nt == 512 ? wide_lds<512>(bs, k, n_chunks).as_wide()
                                                       : wide_lds<kWideThreads>(bs, k, n_chunks);
    c->cooc_score_lds = (size_t)WL.total;
    // (<= 255 per pass: the scoring packs a pass's entry and dense-row prefix sums in one int)
    c->nseg = std::min(std::min(c->cooc_nt, (WL.total - WL.wk - 8) / 40), 255);
    if (c->nseg < 16) return fail(MR_E_INVALID, "co-listening route: no LDS for row descriptors");
    c->cooc_lds = (size_t)cooc_build_lds<false>(bs);
    c->n_heavy = (int)heavy_rows.size();
    c->build_reads = 0;
    for (int64_t x : row_reads) c->build_reads += x;
    c->row_users.assign(row_song.size(), 0);
    for (size_t i = 0; i < (size_t)d->te_off[n_te]; ++i)
      if (te_row[i] >= 0) c->row_users[te_row[i]]++;
    c->row_reads = row_reads;
    c->row_listeners.resize(row_song.size());
    for (size_t r = 0; r < row_song.size(); ++r) c->row_listeners[r] = col_tr[row_song[r]];
    c->row_light.assign(row_song.size(), 0);
    for (int32_t r : light_rows) c->row_light[r] = 1;
    c->n_heavy32 = n_heavy32;
    c->n_big16 = n_big16;
    c->grp = grp;
    c->n_grp = n_grp;
    c->urec_words = urec_words;
    c->lrec_words = lrec_words;
    c->group_nt = cooc_group_nt_opt();
    if (grp > 0)
      MR_HIP(hipFuncSetAttribute(c->group_nt == 512 ? (const void*)k_cooc_group<512> : (const void*)k_cooc_group<1024>,
                                 hipFuncAttributeMaxDynamicSharedMemorySize, cooc_group_lds(bs, grp)));
    c->tcap16 = tcap16;
    c->tcap32 = tcap32;
    c->dense_div = dense_div;
    c->force32 = cooc_dense32_opt();
    c->sat = cooc_sat_opt();
    c->n_light = (int)light_rows.size();
    for (int& x : c->n_light_tier) x = 0;
    for (int32_t r : light_rows) c->n_light_tier[light_tier(row_slots[r] & kLightSlotsMask, n_tiles)]++;
    for (int t = 0; t < kLightTiers; ++t)
      if (int rc2 = light_tier_call(t, nullptr, 0, nullptr, CoocParams{})) return rc2;
    MR_HIP(hipFuncSetAttribute((const void*)c->cooc_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                               (int)c->cooc_score_lds));
    MR_HIP(hipFuncSetAttribute((const void*)k_cooc_build<MR_COOC_NT, false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                               (int)c->cooc_lds));
    MR_HIP(hipFuncSetAttribute((const void*)k_cooc_build<MR_COOC_NT16, true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                               cooc_build_lds<true>(bs)));
  }
  if (wide && k > 0) {
    c->merge_lds = (size_t)merge_lds_bytes(k);
    MR_HIP(hipFuncSetAttribute((const void*)k_topk_merge, hipFuncAttributeMaxDynamicSharedMemorySize,
                               (int)c->merge_lds));
  }
#ifdef MR_STAMPS
  // scoring workgroups' slots, then (co-listening route) 8 per k_cooc_build workgroup
  const size_t stamp_users = (size_t)std::max(batch, route == 2 ? std::min(n_te, 65528) : 0) + 8;
  // scoring workgroups, then 8 per build workgroup (per (row, tile) bound + slack for the
  // group grid's padding), then 8 per light row
  const size_t build_wgs = (size_t)heavy_rows.size() * n_tiles + 64 * (size_t)std::max(1, n_tiles);
  const size_t n_stamps = (size_t)n_tiles * stamp_users * kStampSlots + build_wgs * 8 + light_rows.size() * 8;
  if ((rc = dev_alloc(c->stamps, n_stamps))) return rc;
  MR_HIP(hipMemsetAsync(c->stamps.p, 0, n_stamps * 8, st));
  c->bstamp_off = (size_t)n_tiles * stamp_users * kStampSlots;
  c->lstamp_off = c->bstamp_off + build_wgs * 8;
#endif
  MR_HIP(hipStreamSynchronize(st));  // host vectors die at return
  trace("upload");

  c->n_tr = n_tr; c->n_te = n_te; c->n_s = n_s;
  c->song_lo = lo; c->song_hi = hi; c->width = width;
  c->block_songs = bs; c->n_tiles = n_tiles;
  c->cap = cap; c->batch = batch;
  c->chunk = chunk; c->n_chunks = n_chunks;
  c->loaded = true;
  c->ran = false;
  return MR_OK;
}

int mr_route_info(const mr_ctx* c, int32_t* route, int32_t* n_rows, int64_t* pool_entries) {
  if (!c) return fail(MR_E_INVALID, "null context");
  if (!c->loaded) return fail(MR_E_STATE, "mr_route_info before mr_load");
  if (route) *route = c->ibm_route;
  if (n_rows) *n_rows = c->n_rows;
  if (pool_entries) *pool_entries = c->pool_cap;
  return MR_OK;
}

int mr_topk_mode(const mr_ctx* c, int32_t* candidate_only) {
  if (!c || !candidate_only) return fail(MR_E_INVALID, "null argument");
  if (!c->loaded) return fail(MR_E_STATE, "mr_topk_mode before mr_load");
  *candidate_only = c->cand_on ? 1 : 0;
  return MR_OK;
}

int mr_cooc_stats(mr_ctx* c, int64_t* index_nnz, int64_t* consumed, int64_t* build_reads) {
  if (!c) return fail(MR_E_INVALID, "null context");
  if (!c->loaded || c->ibm_route != 2) return fail(MR_E_STATE, "mr_cooc_stats needs a context on ibm_route 2");
  if (!c->cooc_ran) return fail(MR_E_STATE, "mr_cooc_stats before an ibm run");
  MR_HIP(hipSetDevice(c->opt.device));
  std::vector<unsigned> nnz((size_t)std::max(1, c->n_rows), 0u);
  if (c->n_rows > 0)
    MR_HIP(hipMemcpyAsync(nnz.data(), c->row_nnz.p, (size_t)c->n_rows * 4, hipMemcpyDeviceToHost, c->stream));
  MR_HIP(hipStreamSynchronize(c->stream));
  int64_t tot = 0, use = 0;
  for (int r = 0; r < c->n_rows; ++r) {
    tot += nnz[r];
    use += (int64_t)nnz[r] * c->row_users[r];
  }
  if (index_nnz) *index_nnz = tot;
  if (consumed) *consumed = use;
  if (build_reads) *build_reads = c->build_reads;
  return MR_OK;
}

int mr_cooc_bytes(mr_ctx* c, mr_cooc_bytes_t* out) {
  if (!c || !out) return fail(MR_E_INVALID, "null argument");
  if (!c->loaded || c->ibm_route != 2) return fail(MR_E_STATE, "mr_cooc_bytes needs a context on ibm_route 2");
  if (!c->cooc_ran) return fail(MR_E_STATE, "mr_cooc_bytes before an ibm run");
  MR_HIP(hipSetDevice(c->opt.device));
  const int nr = c->n_rows, nt = c->n_tiles;
  std::vector<int32_t> len((size_t)std::max(1, nr) * nt, 0);
  if (nr > 0)
    MR_HIP(hipMemcpyAsync(len.data(), c->seg_len.p, (size_t)nr * nt * 4, hipMemcpyDeviceToHost, c->stream));
  MR_HIP(hipStreamSynchronize(c->stream));
  mr_cooc_bytes_t b{};
  for (int r = 0; r < nr; ++r) {
    int64_t seg = 0;  // Σ_t min(4 nnz(r, t), songs of t)
    int64_t sp = 0, ds = 0;  // the written encoding: sparse entries, dense songs
    for (int t = 0; t < nt; ++t) {
      const int blo = c->song_lo + t * c->block_songs;
      const int64_t bw = std::min(c->song_hi, blo + c->block_songs) - blo;
      const int32_t l = len[(size_t)t * nr + r];
      // a dense segment (l <= kCoocDenseTail) holds >= bw / dense_div >= bw / 4 non-zeros
      seg += l >= 0 ? std::min<int64_t>(4 * (int64_t)l, bw) : bw;
      if (l >= 0) sp += l;
      else { ds += bw; sp += kCoocDenseTail - l; }
    }
    b.index_sparse_entries += sp;
    b.index_dense_songs += ds;
    b.consumed_sparse_entries += sp * c->row_users[r];
    b.consumed_dense_songs += ds * c->row_users[r];
    if (c->row_light[r]) {
      b.light_rows++;
      b.light_reads += c->row_reads[r];
      b.light_index_bytes += seg;
    } else {
      b.heavy_rows++;
      b.heavy_reads += c->row_reads[r];
      b.heavy_index_bytes += seg;
      // listener walks: one per tile (k_cooc_build), one per tile group (k_cooc_group: u16 rows)
      const bool u32row = c->force32 || c->row_listeners[r] >= 65536;
      b.heavy_visits += (int64_t)c->row_listeners[r] * (c->grp > 0 && !u32row ? c->n_grp : nt);
    }
    b.consumed_bytes += seg * c->row_users[r];
  }
  b.group_tiles = c->grp;
  b.n_groups = c->grp > 0 ? c->n_grp : nt;
  *out = b;
  return MR_OK;
}

int mr_shard_info(const mr_ctx* c, int32_t* lo, int32_t* hi, int32_t* n_te) {
  if (!c) return fail(MR_E_INVALID, "null context");
  if (!c->loaded) return fail(MR_E_STATE, "mr_shard_info before mr_load");
  if (lo) *lo = c->song_lo;
  if (hi) *hi = c->song_hi;
  if (n_te) *n_te = c->n_te;
  return MR_OK;
}

int mr_launch_info(const mr_ctx* c, int32_t* fused, int32_t* block_songs, int32_t* n_tiles) {
  if (!c) return fail(MR_E_INVALID, "null context");
  if (!c->loaded) return fail(MR_E_STATE, "mr_launch_info before mr_load");
  if (fused) *fused = c->shape;
  if (block_songs) *block_songs = c->block_songs;
  if (n_tiles) *n_tiles = c->n_tiles;
  return MR_OK;
}

int mr_batch_info(const mr_ctx* c, int32_t* batch, int32_t* chunk, int32_t* n_chunks) {
  if (!c) return fail(MR_E_INVALID, "null context");
  if (!c->loaded) return fail(MR_E_STATE, "mr_batch_info before mr_load");
  if (batch) *batch = c->batch;
  if (chunk) *chunk = c->chunk;
  if (n_chunks) *n_chunks = c->n_chunks;
  return MR_OK;
}

int mr_shard_tile_songs(const mr_options* opt, int32_t n_train_users, int32_t n_test_users, int32_t* tile_songs) {
  if (!tile_songs) return fail(MR_E_INVALID, "null output pointer");
  mr_options o;
  if (opt) o = *opt; else mr_options_default(&o);
  if (n_train_users < 0 || n_test_users <= 0)
    return fail(MR_E_INVALID, "bad sizes: n_train_users=%d n_test_users=%d", n_train_users, n_test_users);
  *tile_songs = 0;
  if (pick_shape(o, n_train_users, n_test_users) != kShapeWide || o.topk > kMaxTopkLarge) return MR_OK;
  const int chunk = stage1_chunk_for(o, n_train_users);
  const int n_chunks = (std::max(1, n_train_users) + chunk - 1) / chunk;
  *tile_songs = o.block_songs > 0 ? o.block_songs : wide_bmax(o.topk, n_chunks);
  return MR_OK;
}

int mr_shard_tile_songs_n(const mr_options* opt, int32_t n_train_users, int32_t n_test_users, int32_t n_songs,
                          int32_t n_shards, int32_t* tile_songs) {
  if (n_songs <= 0 || n_shards < 1) return fail(MR_E_INVALID, "bad sizes: n_songs=%d n_shards=%d", n_songs, n_shards);
  int rc = mr_shard_tile_songs(opt, n_train_users, n_test_users, tile_songs);
  if (rc || *tile_songs == 0 || n_shards == 1 || (opt && opt->block_songs > 0)) return rc;
  // a multiple of n_shards tiles over the songs: every shard the same whole
  // number of (slightly narrower) tiles (C4 over 8 shards: 24 tiles of 16,128
  // songs, 3 per shard, instead of 20 of 19,456 cut 3/3/3/3/2/2/2/2)
  const long long t0 = ((long long)n_songs + *tile_songs - 1) / *tile_songs;
  const long long t = (t0 + n_shards - 1) / n_shards * n_shards;
  *tile_songs = (int32_t)((((long long)n_songs + t - 1) / t + 255) / 256 * 256);
  return MR_OK;
}

}  // extern "C"

namespace {

int flush_timing(mr_ctx* c) {
  if (c->ring_used == 0) return MR_OK;
  MR_HIP(hipEventSynchronize(c->ring[(size_t)(c->ring_used - 1) * 3 + 2]));
  for (int i = 0; i < c->ring_used; ++i) {
    hipEvent_t* e = &c->ring[(size_t)i * 3];
    float t;
    if (c->ring_has_stage1[i]) { MR_HIP(hipEventElapsedTime(&t, e[0], e[1])); c->ms[0] += t; c->launches[0]++; }
    MR_HIP(hipEventElapsedTime(&t, e[1], e[2])); c->ms[1] += t; c->launches[1]++;
  }
  c->ring_used = 0;
  return MR_OK;
}

// The co-listening route of an ibm run: the index build (k_cooc_build, in
// the stage-1 timing slot), then the scoring kernel over all test users (in
// launches of <= 65528 users) and the per-user merge of the tile lists.
int run_cooc(mr_ctx* c) {
  hipStream_t st = c->stream;
  const bool timed = c->opt.time_kernels != 0;
  const int k = c->opt.topk;
  hipEvent_t* ev = nullptr;
  if (timed) {
    if (c->ring_used == mr_ctx::kRing) {
      int rc = flush_timing(c);
      if (rc) return rc;
    }
    ev = &c->ring[(size_t)c->ring_used * 3];
    c->ring_has_stage1[c->ring_used] = true;
    c->ring_used++;
    MR_HIP(hipEventRecord(ev[0], st));
  }
  if (c->n_rows > 0) {
    MR_HIP(hipMemsetAsync(c->row_nnz.p, 0, (size_t)c->n_rows * sizeof(unsigned), st));
    const bool side = c->side[0] && c->n_light > 0 && cooc_side_opt();
    if (side) {
      MR_HIP(hipEventRecord(c->side_fork, st));
      for (int i = 0; i < 2; ++i) MR_HIP(hipStreamWaitEvent(c->side[i], c->side_fork, 0));
    }
    CoocParams cp{c->n_tr, c->n_rows, c->n_tiles, c->block_songs, c->song_lo, c->song_hi, c->toff.p, c->tsongs.p,
                  c->trs_off.p, c->trs_users.p, c->row_song.p, c->row_base.p, c->pool.p,
                  c->seg_off.p, c->seg_len.p, c->rows_order.p, c->sr_off.p, c->sr_songs.p, c->row_slots.p,
                  c->dense_div, c->force32, 255u, c->stamps.p ? c->stamps.p + c->bstamp_off : nullptr,
                  c->row_nnz.p};
    cp.sat = c->sat;
    // heavy rows: >= 65536 listeners with u32 counters, then the rest with u16 pairs
    const int n32 = c->n_heavy32, n16 = c->n_heavy - c->n_heavy32;
    if (n32 > 0) {  // all big: one workgroup per (row, tile)
      CoocParams hp = cp;
      hp.n_big = n32;
      hp.tcap = c->tcap32;
      hipLaunchKernelGGL((k_cooc_build<MR_COOC_NT, false>), dim3(n32 * c->n_tiles), dim3(MR_COOC_NT), c->cooc_lds, st,
                         hp);
      MR_HIP(hipGetLastError());
    }
    if (n16 > 0 && c->grp > 0) {  // by tile groups: big rows per (row, group), the others per row
      CoocParams hp = cp;
      hp.rows = c->rows_order.p + n32;
      hp.n_big = c->n_big16;
      hp.tcap = c->tcap16;
      hp.lrec = c->lrec.p;
      hp.lrec_words = c->lrec_words;
      hp.grp = c->grp;
      hp.n_grp = c->n_grp;
      hp.rdesc = c->rdesc.p + n32;
      if (hp.stamps) hp.stamps += (size_t)n32 * c->n_tiles * 8;
      const int nblk = (c->n_big16 + 7) / 8 * 8 * c->n_grp + (n16 - c->n_big16);
      const size_t glds = (size_t)cooc_group_lds(c->block_songs, c->grp);
      if (c->group_nt == 512)
        hipLaunchKernelGGL(k_cooc_group<512>, dim3(nblk), dim3(512), glds, st, hp);
      else
        hipLaunchKernelGGL(k_cooc_group<1024>, dim3(nblk), dim3(1024), glds, st, hp);
      MR_HIP(hipGetLastError());
    } else if (n16 > 0) {
      CoocParams hp = cp;
      hp.rows = c->rows_order.p + n32;
      hp.n_big = c->n_big16;
      hp.tcap = c->tcap16;
      if (hp.stamps) hp.stamps += (size_t)n32 * c->n_tiles * 8;
      hipLaunchKernelGGL((k_cooc_build<MR_COOC_NT16, true>), dim3(c->n_big16 * c->n_tiles + n16 - c->n_big16),
                         dim3(MR_COOC_NT16),
                         (size_t)cooc_build_lds<true>(c->block_songs), st, hp);
      MR_HIP(hipGetLastError());
    }
    // light rows on two side streams (tiers 0-1 and 2-3), concurrent with
    // the heavy rows on the context stream: the launches' tails overlap
    // (8 x 1 shards: most rows are light, 4 short launches per step)
    int lr = c->n_heavy;
    for (int t = 0; t < kLightTiers; ++t) {
      if (c->n_light_tier[t] == 0) continue;
      CoocParams lp = cp;
      lp.rows = c->rows_order.p + lr;
      lp.rdesc = c->rdesc.p + lr;
      lp.llrec = reinterpret_cast<const unsigned*>(c->llrec.p);
      lp.lstamps = c->stamps.p ? c->stamps.p + c->lstamp_off + (size_t)(lr - c->n_heavy) * 8 : nullptr;
      hipStream_t ls = side ? c->side[t < 2 ? 0 : 1] : st;
      if (int rc2 = light_tier_call(t, ls, c->n_light_tier[t], &lp, lp)) return rc2;
      lr += c->n_light_tier[t];
    }
    if (side)
      for (int i = 0; i < 2; ++i) {
        MR_HIP(hipEventRecord(c->side_join[i], c->side[i]));
        MR_HIP(hipStreamWaitEvent(st, c->side_join[i], 0));
      }
  }
  if (timed) MR_HIP(hipEventRecord(ev[1], st));
  for (int y0 = 0; y0 < c->n_te; y0 += 65528) {
    const int ny = std::min(65528, c->n_te - y0);
    const int remap = wide_map_opt();
    ScoreParams sp{};
    sp.chunk = c->chunk; sp.n_chunks = c->n_chunks;
    sp.n_users = ny; sp.xcd_remap = remap;
    sp.merge_rows = merge_rows_opt();
    sp.n_tr = c->n_tr;
    sp.user0 = y0;
    sp.song_lo = c->song_lo; sp.song_hi = c->song_hi; sp.width = c->width;
    sp.block_songs = c->block_songs; sp.n_tiles = c->n_tiles;
    sp.frac_bits = c->opt.frac_bits; sp.topk = k; sp.dense = c->opt.dense;
    sp.te_off = c->te_off.p; sp.te_songs = c->te_songs.p;
    sp.sqrt_c = c->sqrt_c.p; sp.q_song = c->q_song.p;
    sp.n_rows = c->n_rows; sp.nseg = c->nseg;
    sp.te_row = c->te_row.p; sp.seg_off = c->seg_off.p; sp.seg_len = c->seg_len.p; sp.pool = c->pool.p;
    sp.dense_out = c->dense_override ? c->dense_override : (void*)c->dense.p;
    sp.cand_key = c->cand_key.p; sp.cand_song = c->cand_song.p; sp.counter = c->counter.p;
    sp.top_key = c->top_key.p; sp.top_song = c->top_song.p; sp.top_score = c->top_score.p;
    sp.stamps = y0 == 0 ? c->stamps.p : nullptr;  // diagnostic build: the first launch
    sp.topk_lists = c->opt.topk_lists;
    if (c->mm_on) { sp.mm_key = c->mm_key.p; sp.mm_n = c->n_te; }
    sp.cand = c->cand_on && !sp.mm_key; sp.rsq_c = c->rsq_c.p;
    hipLaunchKernelGGL(c->cooc_kernel, dim3(c->n_tiles, (ny + 7) / 8 * 8), dim3(c->cooc_nt), c->cooc_score_lds, st, sp);
    MR_HIP(hipGetLastError());
    if (k > 0 && c->n_tiles > 1) {
      MergeParams mp{c->n_tiles, k, k, (long long)c->n_tiles * k, (long long)k, (long long)k, c->cand_key.p,
                     c->cand_song.p, c->top_key.p + (size_t)y0 * k, c->top_song.p + (size_t)y0 * k,
                     c->top_score.p + (size_t)y0 * k};
      hipLaunchKernelGGL(k_topk_merge, dim3(ny), dim3(kThreads), c->merge_lds, st, mp);
      MR_HIP(hipGetLastError());
    }
    if (c->win_open) c->win_launches++;
  }
  if (timed) MR_HIP(hipEventRecord(ev[2], st));
  return MR_OK;
}

// The two-hop shapes' neighbour lists (batch x cap entries), allocated when a
// two-hop run first needs them: a context that only runs the co-listening
// route (C4's north star) never holds them. Not during graph capture
// (mr_graph_capture calls this first).
int ensure_nbr(mr_ctx* c) {
  if (c->shape == kShapeFused || (c->nbr_v.p && c->nbr_q.p && c->nbr_cnt.p)) return MR_OK;
  int rc;
  if ((rc = dev_alloc(c->nbr_v, (size_t)c->batch * c->cap))) return rc;
  if ((rc = dev_alloc(c->nbr_q, (size_t)c->batch * c->cap))) return rc;
  if ((rc = dev_alloc(c->nbr_cnt, (size_t)c->batch * c->n_chunks))) return rc;
  return MR_OK;
}

int run_model(mr_ctx* c, int model) {
  if (model == MR_IBM && c->ibm_route == 2) {
    c->cooc_ran = true;
    return run_cooc(c);
  }
  hipStream_t st = c->stream;
  const bool timed = c->opt.time_kernels != 0;
  const int k = c->opt.topk;
  for (int user0 = 0; user0 < c->n_te; user0 += c->batch) {
    const int nb = std::min(c->batch, c->n_te - user0);
    hipEvent_t* ev = nullptr;
    if (timed) {
      if (c->ring_used == mr_ctx::kRing) {
        int rc = flush_timing(c);
        if (rc) return rc;
      }
      ev = &c->ring[(size_t)c->ring_used * 3];
      c->ring_has_stage1[c->ring_used] = c->shape != kShapeFused;
      c->ring_used++;
      MR_HIP(hipEventRecord(ev[0], st));
    }
    if (c->shape == kShapeSeparate || c->shape == kShapeWide) {
      if (!c->nbr_v.p || !c->nbr_q.p || !c->nbr_cnt.p) {
        if (int rc0 = ensure_nbr(c)) return rc0;
      }
      NbrParams np{c->n_tr, user0, c->cap, c->opt.frac_bits, c->chunk, c->n_chunks, c->te_off.p, c->te_songs.p,
                   c->trs_off.p, c->trs_users.p, c->q_song.p, c->sqrt_tr.p, c->sqrt_te.p, c->nbr_v.p, c->nbr_q.p,
                   c->nbr_cnt.p, c->n_chunks > 1 ? c->sbound.p : nullptr};
      for (int y0 = 0; y0 < nb; y0 += 65535) {
        NbrParams q = np;
        q.user0 = user0 + y0;
        q.nbr_v += (size_t)y0 * c->cap;
        q.nbr_q += (size_t)y0 * c->cap;
        q.nbr_cnt += (size_t)y0 * c->n_chunks;
        hipLaunchKernelGGL(c->nbr_kernel[model], dim3(c->n_chunks, std::min(65535, nb - y0)), dim3(kThreads),
                           c->nbr_lds, st, q);
      }
      MR_HIP(hipGetLastError());
    }
    if (timed) MR_HIP(hipEventRecord(ev[1], st));
    for (int y0 = 0; y0 < nb; y0 += 65528) {
      const int ny = std::min(65528, nb - y0);
      // separate shape: all tiles of a user on one XCD (grid padded to 8 users)
      const bool wide = c->shape == kShapeWide;
      int remap = (c->shape == kShapeSeparate && c->n_tiles > 1) || wide;
      if (wide) remap = wide_map_opt();
      const int gy = remap ? (ny + 7) / 8 * 8 : ny;
      ScoreParams sp{};
      sp.chunk = c->chunk; sp.n_chunks = c->n_chunks;
      sp.n_users = ny; sp.xcd_remap = remap;
      sp.merge_rows = merge_rows_opt();
      sp.n_tr = c->n_tr;
      sp.user0 = user0 + y0;
      sp.song_lo = c->song_lo; sp.song_hi = c->song_hi; sp.width = c->width;
      sp.block_songs = c->block_songs; sp.n_tiles = c->n_tiles;
      sp.frac_bits = c->opt.frac_bits; sp.topk = k; sp.dense = c->opt.dense;
      sp.te_off = c->te_off.p; sp.te_songs = c->te_songs.p;
      sp.toff = c->toff.p; sp.tsongs = c->tsongs.p; sp.tpack = c->tpack.p; sp.sqrt_c = c->sqrt_c.p;
      sp.te_rng = c->te_rng.p; sp.te_q = c->te_q.p;  // fused shape (else null)
      sp.te_sched = c->te_sched.p; sp.sched_off = c->sched_off.p;
#ifdef MR_NO_TERNG  // A/B experiments: stage 1 looks the listener ranges up itself
      sp.te_rng = nullptr;
#endif
      sp.trs_off = c->trs_off.p; sp.trs_users = c->trs_users.p; sp.q_song = c->q_song.p;
      sp.sqrt_tr = c->sqrt_tr.p; sp.sqrt_te = c->sqrt_te.p;
      sp.cap = c->cap;
      sp.nbr_v = c->fused ? nullptr : c->nbr_v.p + (size_t)y0 * c->cap;
      sp.nbr_q = c->fused ? nullptr : c->nbr_q.p + (size_t)y0 * c->cap;
      sp.nbr_cnt = c->fused ? nullptr : c->nbr_cnt.p + (size_t)y0 * c->n_chunks;
      sp.dense_out = c->dense_override ? c->dense_override : (void*)c->dense.p;
      sp.cand_key = c->cand_key.p; sp.cand_song = c->cand_song.p; sp.counter = c->counter.p;
      sp.top_key = c->top_key.p; sp.top_song = c->top_song.p; sp.top_score = c->top_score.p;
      sp.stamps = c->stamps.p ? c->stamps.p + (size_t)y0 * c->n_tiles * kStampSlots : nullptr;
      sp.topk_lists = c->opt.topk_lists;
      if (c->mm_on && wide) { sp.mm_key = c->mm_key.p; sp.mm_n = c->n_te; }
      sp.cand = wide && c->cand_on && !sp.mm_key; sp.rsq_c = c->rsq_c.p;
      hipLaunchKernelGGL(c->score_kernel[model], dim3(c->n_tiles, gy), dim3(wide ? kWideThreads : kThreads),
                         c->score_lds, st, sp);
      MR_HIP(hipGetLastError());
      if (wide && k > 0 && c->n_tiles > 1) {  // per-user top-k over the tiles' candidates
        MergeParams mp{c->n_tiles, k, k, (long long)c->n_tiles * k, (long long)k, (long long)k, c->cand_key.p, c->cand_song.p,
                       c->top_key.p + (size_t)(user0 + y0) * k, c->top_song.p + (size_t)(user0 + y0) * k,
                       c->top_score.p + (size_t)(user0 + y0) * k};
        hipLaunchKernelGGL(k_topk_merge, dim3(ny), dim3(kThreads), c->merge_lds, st, mp);
        MR_HIP(hipGetLastError());
      }
      if (c->win_open) c->win_launches++;
    }
    if (timed) MR_HIP(hipEventRecord(ev[2], st));
  }
  return MR_OK;
}

}  // namespace

namespace mr_internal {

// Device -> host copy of `rows` rows of `row_bytes` (source pitch spitch,
// destination pitch dpitch), synchronous on the context stream. Small copies
// and pinned destinations go straight through the DMA engine; large copies
// into pageable memory (a fresh numpy array) are staged through two pinned
// 64 MiB buffers: chunk i+1 is in flight while the host threads copy chunk i
// out — and take the destination's first-touch page faults in parallel
// (hipMemcpy from pageable memory: 9.9 GB/s at C3, one thread; staged: 47-51
// GB/s into a fresh numpy array, profiles/r03/d2h_c3.json). The two pinned
// buffers are one process-wide pool (portable pinned memory, allocated on first
// use and kept for the process: pinning 128 MiB costs ~14 ms, which a fresh
// engine per call would pay every time — 29 vs 50 GB/s); one staged copy runs
// at a time (the host threads are the bottleneck anyway).
namespace {
struct StagePool {
  std::mutex m;
  void* buf[2] = {nullptr, nullptr};
};
StagePool& stage_pool() {
  static StagePool* p = new StagePool;  // never destroyed: outlives the HIP runtime's teardown order
  return *p;
}
}  // namespace

int d2h_staged(mr_ctx* c, void* dst, size_t dpitch, const void* src, size_t spitch, size_t row_bytes, size_t rows) {
  const size_t total = row_bytes * rows;
  if (total == 0) return MR_OK;
  hipPointerAttribute_t attr;
  const bool pinned = hipPointerGetAttributes(&attr, dst) == hipSuccess && attr.type == hipMemoryTypeHost;
  (void)hipGetLastError();  // pageable memory is "not a HIP pointer": not an error here
  constexpr size_t kStage = (size_t)64 << 20;
  if (pinned || total < ((size_t)8 << 20) || row_bytes > kStage) {
    MR_HIP(hipMemcpy2DAsync(dst, dpitch, src, spitch, row_bytes, rows, hipMemcpyDeviceToHost, c->stream));
    MR_HIP(hipStreamSynchronize(c->stream));
    return MR_OK;
  }
  StagePool& pool = stage_pool();
  std::lock_guard<std::mutex> lock(pool.m);
  for (int i = 0; i < 2; ++i) {
    if (!pool.buf[i]) MR_HIP(hipHostMalloc(&pool.buf[i], kStage, hipHostMallocPortable));
    if (!c->stage_ev[i]) MR_HIP(hipEventCreateWithFlags(&c->stage_ev[i], hipEventDisableTiming));
  }
  const size_t per = kStage / row_bytes;  // rows per chunk
  const size_t n_chunks = (rows + per - 1) / per;
  auto enqueue = [&](size_t k) -> int {
    const size_t r0 = k * per, nr = std::min(per, rows - r0);
    MR_HIP(hipMemcpy2DAsync(pool.buf[k & 1], row_bytes, static_cast<const char*>(src) + r0 * spitch, spitch,
                            row_bytes, nr, hipMemcpyDeviceToHost, c->stream));
    MR_HIP(hipEventRecord(c->stage_ev[k & 1], c->stream));
    return MR_OK;
  };
  int rc = enqueue(0);
  if (!rc && n_chunks > 1) rc = enqueue(1);
  if (rc) return rc;
  for (size_t k = 0; k < n_chunks; ++k) {
    MR_HIP(hipEventSynchronize(c->stage_ev[k & 1]));
    const size_t r0 = k * per, nr = std::min(per, rows - r0);
    const char* from = static_cast<const char*>(pool.buf[k & 1]);
    char* to = static_cast<char*>(dst) + r0 * dpitch;
    if (dpitch == row_bytes) {
      mr_par::parallel_for((int64_t)(nr * row_bytes), [&](int64_t a, int64_t b, int) {
        std::memcpy(to + a, from + a, (size_t)(b - a));
      }, (int64_t)4 << 20);
    } else {
      mr_par::parallel_for((int64_t)nr, [&](int64_t a, int64_t b, int) {
        for (int64_t r = a; r < b; ++r) std::memcpy(to + r * dpitch, from + r * row_bytes, row_bytes);
      }, std::max<int64_t>(1, ((int64_t)4 << 20) / (int64_t)row_bytes));
    }
    if (k + 2 < n_chunks && (rc = enqueue(k + 2))) return rc;  // the buffer just emptied
  }
  return MR_OK;
}

namespace {
int launch_merge(mr_ctx* c, int32_t n_shards, int32_t n_te, int32_t k, const MergeParams& mp) {
  const int lds = merge_lds_bytes(k);
  if (lds > 160 * 1024) return fail(MR_E_INVALID, "merge of %d lists x %d needs too much LDS", n_shards, k);
  MR_HIP(hipFuncSetAttribute((const void*)k_topk_merge, hipFuncAttributeMaxDynamicSharedMemorySize, lds));
  for (int y0 = 0; y0 < n_te; y0 += 65535) {
    MergeParams q = mp;
    q.keys += (size_t)y0 * k;
    q.songs += (size_t)y0 * k;
    q.out_keys += (size_t)y0 * k;
    q.out_songs += (size_t)y0 * k;
    if (q.out_scores) q.out_scores += (size_t)y0 * k;
    hipLaunchKernelGGL(k_topk_merge, dim3(std::min(65535, n_te - y0)), dim3(kThreads), lds, c->stream, q);
  }
  MR_HIP(hipGetLastError());
  return MR_OK;
}
}  // namespace

int merge_async(mr_ctx* c, int32_t n_shards, int32_t n_te, int32_t k, const int32_t* songs_in,
                const int64_t* keys_in, int32_t* songs_out, int64_t* keys_out, double* scores_out) {
  if (!c || !songs_in || !keys_in || !songs_out || !keys_out) return fail(MR_E_INVALID, "null argument");
  if (n_shards <= 0 || n_te <= 0 || k <= 0 || k > kMaxTopK) return fail(MR_E_INVALID, "bad merge shape");
  MR_HIP(hipSetDevice(c->opt.device));
  MergeParams mp{n_shards, k, k, k, (long long)n_te * k, (long long)n_te * k, reinterpret_cast<const long long*>(keys_in),
                 songs_in, reinterpret_cast<long long*>(keys_out), songs_out, scores_out};
  return launch_merge(c, n_shards, n_te, k, mp);
}

int merge_records_async(mr_ctx* c, int32_t n_shards, int32_t n_te, int32_t k, const void* records, int64_t rec_bytes,
                        int32_t* songs_out, int64_t* keys_out, double* scores_out) {
  if (!c || !records || !songs_out || !keys_out) return fail(MR_E_INVALID, "null argument");
  if (n_shards <= 0 || n_te <= 0 || k <= 0 || k > kMaxTopK) return fail(MR_E_INVALID, "bad merge shape");
  const size_t nk = (size_t)n_te * k;
  if (rec_bytes < (int64_t)(12 * nk) || rec_bytes % 8)
    return fail(MR_E_INVALID, "record blocks of %lld B cannot hold %zu keys + songs (multiple of 8 B needed)",
                (long long)rec_bytes, nk);
  MR_HIP(hipSetDevice(c->opt.device));
  const char* base = static_cast<const char*>(records);
  MergeParams mp{n_shards, k, k, k, rec_bytes / 8, rec_bytes / 4, reinterpret_cast<const long long*>(base),
                 reinterpret_cast<const int*>(base + 8 * nk), reinterpret_cast<long long*>(keys_out), songs_out,
                 scores_out};
  return launch_merge(c, n_shards, n_te, k, mp);
}

int topk_records(mr_ctx* c, void** records, int64_t* rec_bytes) {
  if (!c || !records || !rec_bytes) return fail(MR_E_INVALID, "null argument");
  if (!c->loaded || c->opt.topk <= 0) return fail(MR_E_STATE, "no top-k lists (not loaded or topk = 0)");
  *records = c->top_key.p;
  *rec_bytes = topk_record_bytes((size_t)c->n_te * c->opt.topk);
  return MR_OK;
}

int set_error(int code, const char* msg) { return fail(code, "%s", msg); }

int set_device_share(mr_ctx* c, int n) {
  if (!c || n < 1) return fail(MR_E_INVALID, "set_device_share: null context or share < 1");
  c->dev_share = n;
  return MR_OK;
}

int validate_dataset(const mr_dataset* d) {
  if (!d) return fail(MR_E_INVALID, "null dataset");
  std::vector<int32_t> col_tr;
  return check_dataset(d, col_tr);
}

}  // namespace mr_internal

extern "C" {

int mr_run(mr_ctx* c, int model) {
  if (!c) return fail(MR_E_INVALID, "null context");
  if (!c->loaded) return fail(MR_E_STATE, "mr_run before mr_load");
  if (model != MR_UBM && model != MR_IBM) return fail(MR_E_INVALID, "unknown model %d", model);
  MR_HIP(hipSetDevice(c->opt.device));
  // wide dense runs leave each user's min / max stored score (mr_dense_minmax)
  c->mm_valid = false;
  c->mm_on = c->shape == kShapeWide && c->opt.dense && c->n_te > 0;
  if (c->mm_on) {
    int rc0 = MR_OK;
    if (!c->mm_key.p && (rc0 = dev_alloc(c->mm_key, (size_t)2 * c->n_te))) return rc0;
    MR_HIP(hipMemsetAsync(c->mm_key.p, 0xff, (size_t)c->n_te * 8, c->stream));  // min keys: the largest
    MR_HIP(hipMemsetAsync(c->mm_key.p + c->n_te, 0, (size_t)c->n_te * 8, c->stream));  // max keys: the smallest
  }
  int rc = run_model(c, model);
  const bool mm = c->mm_on;
  c->mm_on = false;
  if (rc) return rc;
  c->mm_valid = mm;
  c->ran = true;
  c->last_model = model;
  return MR_OK;
}

int mr_dense_minmax(mr_ctx* c, double* mn, double* mx) {
  if (!c || !mn || !mx) return fail(MR_E_INVALID, "null argument");
  if (!c->mm_valid)
    return fail(MR_E_STATE, "no dense min / max: the last mr_run / mr_run_into was not a wide-shape dense run");
  MR_HIP(hipSetDevice(c->opt.device));
  std::vector<unsigned long long> h((size_t)2 * c->n_te);
  MR_HIP(hipMemcpyAsync(h.data(), c->mm_key.p, h.size() * 8, hipMemcpyDeviceToHost, c->stream));
  MR_HIP(hipStreamSynchronize(c->stream));
  unsigned long long a = ~0ull, b = 0ull;
  for (int u = 0; u < c->n_te; ++u) {
    a = std::min(a, h[u]);
    b = std::max(b, h[(size_t)c->n_te + u]);
  }
  // (no pair anywhere: +inf / -inf, as mr_eval_minmax_device)
  *mn = a == ~0ull ? INFINITY : ordered_value(a);
  *mx = b == 0ull ? -INFINITY : ordered_value(b);
  return MR_OK;
}

int mr_graph_capture(mr_ctx* c, int model, int32_t n_steps) {
  if (!c) return fail(MR_E_INVALID, "null context");
  c->mm_valid = false;
  if (!c->loaded) return fail(MR_E_STATE, "mr_graph_capture before mr_load");
  if (model != MR_UBM && model != MR_IBM) return fail(MR_E_INVALID, "unknown model %d", model);
  if (n_steps < 1 || n_steps > 100000) return fail(MR_E_INVALID, "n_steps %d outside [1,100000]", n_steps);
  if (c->opt.time_kernels) return fail(MR_E_STATE, "graph capture of a context with time_kernels=1");
  MR_HIP(hipSetDevice(c->opt.device));
  MR_HIP(hipStreamSynchronize(c->stream));
  if (!(model == MR_IBM && c->ibm_route == 2)) {  // no allocation inside the capture
    if (int rc0 = ensure_nbr(c)) return rc0;
  }
  if (c->graph_exec) { MR_HIP(hipGraphExecDestroy(c->graph_exec)); c->graph_exec = nullptr; }
  if (c->graph) { MR_HIP(hipGraphDestroy(c->graph)); c->graph = nullptr; }
  c->graph_steps = 0;
  MR_HIP(hipStreamBeginCapture(c->stream, hipStreamCaptureModeThreadLocal));
  int rc = MR_OK;
  const long long counted = c->win_launches;  // captured launches are not runs
  for (int i = 0; i < n_steps && rc == MR_OK; ++i) rc = run_model(c, model);
  c->win_launches = counted;
  hipGraph_t g = nullptr;
  const hipError_t e = hipStreamEndCapture(c->stream, &g);
  if (rc) { if (g) (void)hipGraphDestroy(g); return rc; }
  if (e != hipSuccess) return fail(MR_E_HIP, "hipStreamEndCapture: %s", hipGetErrorString(e));
  c->graph = g;
  MR_HIP(hipGraphInstantiate(&c->graph_exec, c->graph, nullptr, nullptr, 0));
  c->graph_steps = n_steps;
  c->last_model = model;
  return MR_OK;
}

int mr_graph_launch(mr_ctx* c) {
  if (c) c->mm_valid = false;  // (graph replays leave no dense min / max)
  if (!c) return fail(MR_E_INVALID, "null context");
  if (!c->graph_exec) return fail(MR_E_STATE, "no captured graph (mr_graph_capture)");
  MR_HIP(hipSetDevice(c->opt.device));
  MR_HIP(hipGraphLaunch(c->graph_exec, c->stream));
  if (c->win_open) c->win_launches += c->graph_steps;
  c->ran = true;
  return MR_OK;
}

int mr_sync(mr_ctx* c) {
  if (!c) return fail(MR_E_INVALID, "null context");
  MR_HIP(hipStreamSynchronize(c->stream));
  return MR_OK;
}

int mr_device_outputs(const mr_ctx* c, void** dense, int32_t** ts, int64_t** tk, double** tsc) {
  if (!c) return fail(MR_E_INVALID, "null context");
  if (!c->ran) return fail(MR_E_STATE, "no mr_run yet");
  if (dense) *dense = c->opt.dense ? (void*)c->dense.p : nullptr;
  if (ts) *ts = c->top_song.p;
  if (tk) *tk = reinterpret_cast<int64_t*>(c->top_key.p);
  if (tsc) *tsc = c->top_score.p;
  return MR_OK;
}

int mr_copy_dense(mr_ctx* c, void* out) {
  if (!c || !out) return fail(MR_E_INVALID, "null argument");
  if (!c->ran) return fail(MR_E_STATE, "no mr_run yet");
  if (!c->opt.dense) return fail(MR_E_STATE, "context created with dense=0");
  MR_HIP(hipSetDevice(c->opt.device));
  const size_t row = (size_t)c->width * (c->opt.out_dtype == MR_OUT_F64 ? 8 : 4);
  return mr_internal::d2h_staged(c, out, row, c->dense.p, row, row, (size_t)c->n_te);
}

int mr_copy_topk(mr_ctx* c, int32_t* songs, double* scores, int64_t* keys) {
  if (!c) return fail(MR_E_INVALID, "null context");
  if (!c->ran) return fail(MR_E_STATE, "no mr_run yet");
  if (c->opt.topk <= 0) return fail(MR_E_STATE, "context created with topk=0");
  MR_HIP(hipSetDevice(c->opt.device));
  const size_t n = (size_t)c->n_te * c->opt.topk;
  if (songs) MR_HIP(hipMemcpyAsync(songs, c->top_song.p, n * 4, hipMemcpyDeviceToHost, c->stream));
  if (scores) MR_HIP(hipMemcpyAsync(scores, c->top_score.p, n * 8, hipMemcpyDeviceToHost, c->stream));
  if (keys) MR_HIP(hipMemcpyAsync(keys, c->top_key.p, n * 8, hipMemcpyDeviceToHost, c->stream));
  MR_HIP(hipStreamSynchronize(c->stream));
  return MR_OK;
}

int mr_copy_topk_device(mr_ctx* c, int32_t* songs, int64_t* keys) {
  if (!c) return fail(MR_E_INVALID, "null context");
  if (!c->ran) return fail(MR_E_STATE, "no mr_run yet");
  if (c->opt.topk <= 0) return fail(MR_E_STATE, "context created with topk=0");
  MR_HIP(hipSetDevice(c->opt.device));
  const size_t n = (size_t)c->n_te * c->opt.topk;
  if (songs) MR_HIP(hipMemcpyAsync(songs, c->top_song.p, n * 4, hipMemcpyDeviceToDevice, c->stream));
  if (keys) MR_HIP(hipMemcpyAsync(keys, c->top_key.p, n * 8, hipMemcpyDeviceToDevice, c->stream));
  MR_HIP(hipStreamSynchronize(c->stream));
  return MR_OK;
}

int mr_copy_topk_device_async(mr_ctx* c, int32_t* songs, int64_t* keys) {
  if (!c) return fail(MR_E_INVALID, "null context");
  if (!c->loaded) return fail(MR_E_STATE, "mr_copy_topk_device_async before mr_load");
  if (c->opt.topk <= 0) return fail(MR_E_STATE, "context created with topk=0");
  MR_HIP(hipSetDevice(c->opt.device));
  const size_t n = (size_t)c->n_te * c->opt.topk;
  if (songs) MR_HIP(hipMemcpyAsync(songs, c->top_song.p, n * 4, hipMemcpyDeviceToDevice, c->stream));
  if (keys) MR_HIP(hipMemcpyAsync(keys, c->top_key.p, n * 8, hipMemcpyDeviceToDevice, c->stream));
  return MR_OK;
}

int mr_topk_merge_device_async(mr_ctx* c, int32_t n_shards, int32_t n_te, int32_t k, const int32_t* songs_in,
                               const int64_t* keys_in, int32_t* songs_out, int64_t* keys_out, double* scores_out) {
  return mr_internal::merge_async(c, n_shards, n_te, k, songs_in, keys_in, songs_out, keys_out, scores_out);
}

int mr_topk_record_bytes(int32_t n_te, int32_t k, int64_t* rec_bytes) {
  if (!rec_bytes || n_te < 0 || k <= 0 || k > kMaxTopK) return fail(MR_E_INVALID, "bad record shape");
  *rec_bytes = topk_record_bytes((size_t)n_te * k);
  return MR_OK;
}

int mr_topk_merge_records_async(mr_ctx* c, int32_t n_shards, int32_t n_te, int32_t k, const void* records,
                                int64_t rec_bytes, int32_t* songs_out, int64_t* keys_out, double* scores_out) {
  return mr_internal::merge_records_async(c, n_shards, n_te, k, records, rec_bytes, songs_out, keys_out, scores_out);
}

int mr_score_dense(mr_ctx* c, int model, void* out) {
  int rc = mr_run(c, model);
  if (rc) return rc;
  return mr_copy_dense(c, out);
}

int mr_topk(mr_ctx* c, int model, int k, int32_t* songs, double* scores, int64_t* keys) {
  if (!c) return fail(MR_E_INVALID, "null context");
  if (k != c->opt.topk) return fail(MR_E_INVALID, "k=%d differs from the context's topk=%d", k, c->opt.topk);
  int rc = mr_run(c, model);
  if (rc) return rc;
  return mr_copy_topk(c, songs, scores, keys);
}

int mr_topk_merge_device(mr_ctx* c, int32_t n_shards, int32_t n_te, int32_t k, const int32_t* songs_in,
                         const int64_t* keys_in, const double* /*scores_in*/, int32_t* songs_out,
                         int64_t* keys_out, double* scores_out) {
  const int rc = mr_internal::merge_async(c, n_shards, n_te, k, songs_in, keys_in, songs_out, keys_out, scores_out);
  if (rc) return rc;
  MR_HIP(hipStreamSynchronize(c->stream));
  return MR_OK;
}

int mr_debug_stamps(mr_ctx* c, int64_t* out, int64_t n) {
  if (!c || !out) return fail(MR_E_INVALID, "null argument");
  if (!c->stamps.p) return fail(MR_E_STATE, "library built without -DMR_STAMPS");
  MR_HIP(hipSetDevice(c->opt.device));
  const size_t m = std::min<size_t>((size_t)n, c->stamps.n);
  MR_HIP(hipMemcpyAsync(out, c->stamps.p, m * 8, hipMemcpyDeviceToHost, c->stream));
  MR_HIP(hipStreamSynchronize(c->stream));
  return (int)MR_OK;
}

int mr_timing_begin(mr_ctx* c) {
  if (!c) return fail(MR_E_INVALID, "null context");
  MR_HIP(hipSetDevice(c->opt.device));
  MR_HIP(hipEventRecord(c->win[0], c->stream));
  c->win_open = true;
  c->win_stopped = false;
  c->win_launches = 0;
  return MR_OK;
}

int mr_timing_stop(mr_ctx* c) {
  if (!c) return fail(MR_E_INVALID, "null context");
  if (!c->win_open) return fail(MR_E_STATE, "mr_timing_stop without mr_timing_begin");
  MR_HIP(hipSetDevice(c->opt.device));
  if (!c->win_stopped) MR_HIP(hipEventRecord(c->win[1], c->stream));
  c->win_stopped = true;
  return MR_OK;
}

int mr_timing_end(mr_ctx* c, int64_t* launches, double* total_ms) {
  if (!c) return fail(MR_E_INVALID, "null context");
  if (!c->win_open) return fail(MR_E_STATE, "mr_timing_end without mr_timing_begin");
  MR_HIP(hipSetDevice(c->opt.device));
  if (!c->win_stopped) MR_HIP(hipEventRecord(c->win[1], c->stream));
  c->win_stopped = false;
  MR_HIP(hipEventSynchronize(c->win[1]));
  float t = 0.f;
  MR_HIP(hipEventElapsedTime(&t, c->win[0], c->win[1]));
  c->win_open = false;
  if (launches) *launches = c->win_launches;
  if (total_ms) *total_ms = t;
  return MR_OK;
}

int mr_kernel_times(mr_ctx* c, int32_t which, int64_t* launches, double* total_ms, int32_t reset) {
  if (!c) return fail(MR_E_INVALID, "null context");
  if (which < 0 || which > 2) return fail(MR_E_INVALID, "kernel index %d outside [0,2]", which);
  MR_HIP(hipSetDevice(c->opt.device));
  int rc = flush_timing(c);
  if (rc) return rc;
  if (launches) *launches = c->launches[which];
  if (total_ms) *total_ms = c->ms[which];
  if (reset) { c->launches[which] = 0; c->ms[which] = 0.0; }
  return MR_OK;
}

int mr_run_into(mr_ctx* c, int model, void* dense_dev) {
  if (!c || !dense_dev) return fail(MR_E_INVALID, "null argument");
  if (!c->loaded) return fail(MR_E_STATE, "mr_run_into before mr_load");
  if (!c->opt.dense) return fail(MR_E_STATE, "context created with dense=0");
  c->dense_override = dense_dev;
  const int rc = mr_run(c, model);
  c->dense_override = nullptr;
  return rc;
}

int mr_view_get(const mr_ctx* c, mr_view* v) {
  if (!c || !v) return fail(MR_E_INVALID, "null argument");
  if (!c->loaded) return fail(MR_E_STATE, "mr_view_get before mr_load");
  std::memset(v, 0, sizeof *v);
  v->n_test_users = c->n_te;
  v->n_songs = c->n_s;
  v->song_lo = c->song_lo;
  v->song_hi = c->song_hi;
  v->out_dtype = c->opt.out_dtype;
  v->device = c->opt.device;
  v->te_off = reinterpret_cast<const int64_t*>(c->te_off.p);
  v->te_songs = c->te_songs.p;
  v->stream = (void*)c->stream;
  return MR_OK;
}

int mr_topk_dense_device(mr_ctx* c, const void* dense_dev, int32_t k) {
  if (!c || !dense_dev) return fail(MR_E_INVALID, "null argument");
  if (!c->loaded) return fail(MR_E_STATE, "mr_topk_dense_device before mr_load");
  if (k != c->opt.topk || k <= 0 || k > kMaxTopkLarge)
    return fail(MR_E_INVALID, "k=%d must equal the context's topk (%d) and be in [1,%d]", k, c->opt.topk,
                kMaxTopkLarge);
  MR_HIP(hipSetDevice(c->opt.device));
  MR_HIP(hipMemsetAsync(c->flag.p, 0, sizeof(unsigned), c->stream));
  const bool f64 = c->opt.out_dtype == MR_OUT_F64;
  for (int y0 = 0; y0 < c->n_te; y0 += 65535) {
    DenseTopkParams tp{y0, c->width, c->song_lo, k, dense_dev, c->top_key.p, c->top_song.p, c->top_score.p,
                       c->flag.p};
    const int ny = std::min(65535, c->n_te - y0);
    if (f64) hipLaunchKernelGGL(k_topk_dense<double>, dim3(ny), dim3(kWideThreads), 0, c->stream, tp);
    else hipLaunchKernelGGL(k_topk_dense<float>, dim3(ny), dim3(kWideThreads), 0, c->stream, tp);
    MR_HIP(hipGetLastError());
  }
  unsigned neg = 0;
  MR_HIP(hipMemcpyAsync(&neg, c->flag.p, sizeof neg, hipMemcpyDeviceToHost, c->stream));
  MR_HIP(hipStreamSynchronize(c->stream));
  if (neg) return fail(MR_E_INVALID, "dense model has negative scores: top-k keys need scores >= 0");
  c->ran = true;
  return MR_OK;
}

}  // extern "C"
