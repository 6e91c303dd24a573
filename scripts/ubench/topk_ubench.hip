// Micro-benchmark of the top-k primitives (cycles via s_memtime), one wave.
#include <hip/hip_runtime.h>
#include <climits>
#include <cstdio>
#include <cstring>
#include <vector>
constexpr int kThreads = 256;
constexpr int kWaves = 4;
constexpr long long kKeyNone = -1;
__device__ __forceinline__ void stamp_at(long long*, int) {}
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
template <int M>
__device__ __forceinline__ void wave_topk_regs(long long (&rk)[M], int (&rs)[M], int k, long long* out_k,
                                               int* out_s) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int j = 0; j < M; ++j)
    if (rk[j] < 0) { rk[j] = kKeyNone; rs[j] = INT_MAX; }
  lane_sort<M>(rk, rs);
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


__global__ void k_bench(long long* out, const long long* keys, int which, int k) {
  __shared__ long long lk[256 * 10];
  __shared__ int ls[256 * 10];
  __shared__ long long ok[64];
  __shared__ int os[64];
  const int lane = threadIdx.x;
  for (int i = lane; i < 66 * 10; i += 64) { lk[i] = keys[i]; ls[i] = i; }
  __syncthreads();
  long long t0 = __builtin_amdgcn_s_memtime();
  long long acc = 0;
  if (which == 0) {  // 10 dependent argmaxes
    long long kk = keys[lane];
    int s = lane;
    for (int r = 0; r < 10; ++r) { wave_argmax(kk, s); kk = keys[(lane + r + (int)(kk & 7)) % 640]; acc += s; }
  } else if (which == 1) {  // wave top-k of 256 in registers
    long long rk[4]; int rs[4];
    for (int j = 0; j < 4; ++j) { rk[j] = keys[lane + 64 * j]; rs[j] = lane + 64 * j; }
    wave_topk_regs<4>(rk, rs, k, ok, os);
  } else if (which == 2) {  // tournament over 66 lists of 10
    // sort each list first (host gives random keys): lists are ls-sorted below via keys order
    wave_merge_lists(66, 10, lk, ls, ok, os);
  } else if (which == 3) {  // 10 x (3 wave reductions only)
    int x = (int)keys[lane];
    for (int r = 0; r < 10; ++r) { x = wave_max_i32(x) + lane; acc += x; }
  }
  asm volatile("s_waitcnt lgkmcnt(0) vmcnt(0)" ::: "memory");
  long long t1 = __builtin_amdgcn_s_memtime();
  if (lane == 0) { out[0] = t1 - t0; out[1] = ok[0] + acc; }
}

int main() {
  const int n = 66 * 10;
  std::vector<long long> h(n);
  unsigned long long x = 88172645463325252ull;
  for (int l = 0; l < 66; ++l) {  // 66 sorted descending lists of 10 realistic keys (double bits)
    double v = 10.0;
    for (int r = 0; r < 10; ++r) {
      x ^= x << 13; x ^= x >> 7; x ^= x << 17;
      v -= (double)(x % 100000) * 1e-6;
      long long b; memcpy(&b, &v, 8); h[l * 10 + r] = b;
    }
  }
  long long *d, *o;
  hipMalloc(&d, n * 8); hipMalloc(&o, 16);
  hipMemcpy(d, h.data(), n * 8, hipMemcpyHostToDevice);
  const char* names[] = {"10 x wave_argmax", "wave_topk_regs<4> k=10 (256 cand)", "wave_merge_lists 66x10", "10 x wave_max_i32"};
  for (int w = 0; w < 4; ++w) {
    long long best = 1ll << 60;
    for (int rep = 0; rep < 20; ++rep) {
      hipLaunchKernelGGL(k_bench, dim3(1), dim3(64), 0, 0, o, d, w, 10);
      long long r[2];
      hipMemcpy(r, o, 16, hipMemcpyDeviceToHost);
      if (r[0] < best) best = r[0];
    }
    printf("%-40s %8lld cycles\n", names[w], best);
  }
  return 0;
}
