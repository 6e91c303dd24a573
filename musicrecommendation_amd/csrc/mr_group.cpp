// mr_group.cpp — multi-GPU behind the C ABI: one handle over G contexts.
//
// The reference fans ONE driver call out over song partitions:
//   getItemBasedModel2 = ctx.parallelize(songs, numberSlices).map(getRanks2).collect.flatten
//   (src/main/scala/distributed.scala:477-479; getUserBasedModel2 :459-461), and over test
//   users in strategy 1 (getItemBasedModel1 :468-470).
// Here one mr_group_run fans out over G = n_song_shards x n_user_blocks engine
// contexts (a 2-D layout: song-id range shards x test-user blocks). Each context
// scores its (user block, song range) on its own GPU and stream; the contexts of
// one user block then exchange their per-user top-k lists with ONE all-gather
// and merge them by (key desc, song asc) — bit-identical to one context, since
// the keys are fixed-point sums (any shard count gives the same integers).
//
// Transports of the exchange:
//   RCCL  every context on its own device: one communicator per user block
//         (ncclCommInitAll over the block's devices, xGMI), ncclAllGather under
//         ncclGroupStart/End on the contexts' streams, the merge kernel on every
//         device. librccl is dlopen'ed when the first RCCL group is created.
//   COPY  every context on ONE device (logical shards, e.g. a 1-GPU box): the
//         block's first context gathers the lists with device copies, ordered by
//         events, and merges them.
// The dense model stays column-sharded on the devices; mr_group_allgather_dense
// assembles full rows on every device of a block (RCCL all-gather of equal-size
// padded shard blocks + strided on-device copies), mr_group_copy_dense collects
// them on the host (≙ collect.flatten).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <dlfcn.h>

#include <algorithm>
#include <cstdarg>
#include <cstdlib>
#include <map>
#include <mutex>
#include <cstdio>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "mr_engine.h"
#include "mr_internal.h"

namespace {

using mr_internal::set_error;

int gfail(int code, const char* fmt, ...) __attribute__((format(printf, 2, 3)));
int gfail(int code, const char* fmt, ...) {
  char buf[1024];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  return set_error(code, buf);
}

#define G_HIP(call)                                                                              \
  do {                                                                                           \
    hipError_t e_ = (call);                                                                      \
    if (e_ != hipSuccess)                                                                        \
      return gfail(e_ == hipErrorOutOfMemory ? MR_E_OOM : MR_E_HIP, "%s failed: %s (%s:%d)", #call, \
                   hipGetErrorString(e_), __FILE__, __LINE__);                                  \
  } while (0)

// ---- RCCL, loaded on first use ------------------------------------------------
struct Rccl {
  bool tried = false, ok = false;
  std::string why;
  decltype(&ncclCommInitAll) comm_init_all = nullptr;
  decltype(&ncclCommDestroy) comm_destroy = nullptr;
  decltype(&ncclAllGather) all_gather = nullptr;
  decltype(&ncclGroupStart) group_start = nullptr;
  decltype(&ncclGroupEnd) group_end = nullptr;
  decltype(&ncclGetErrorString) error_string = nullptr;
  bool shared_devices = false;  // the test library's marker (several ranks per device)
};

// The library: MR_RCCL_LIB when set (tests/fake_rccl runs the multi-context
// path on one GPU), else librccl. One handle per path, loaded once.
Rccl& rccl_at(const std::string& path) {
  static std::mutex mu;
  static std::map<std::string, Rccl> libs;
  std::lock_guard<std::mutex> lock(mu);
  Rccl& r = libs[path];
  if (r.tried) return r;
  r.tried = true;
  void* h = nullptr;
  if (!path.empty()) {
    h = dlopen(path.c_str(), RTLD_NOW | RTLD_LOCAL);
  } else {
    for (const char* name : {"librccl.so.1", "/opt/rocm/lib/librccl.so.1", "librccl.so"}) {
      h = dlopen(name, RTLD_NOW | RTLD_LOCAL);
      if (h) break;
    }
  }
  if (!h) {
    const char* e = dlerror();
    r.why = std::string("dlopen(") + (path.empty() ? "librccl.so.1" : path) + "): " + (e ? e : "?");
    return r;
  }
  r.comm_init_all = reinterpret_cast<decltype(r.comm_init_all)>(dlsym(h, "ncclCommInitAll"));
  r.comm_destroy = reinterpret_cast<decltype(r.comm_destroy)>(dlsym(h, "ncclCommDestroy"));
  r.all_gather = reinterpret_cast<decltype(r.all_gather)>(dlsym(h, "ncclAllGather"));
  r.group_start = reinterpret_cast<decltype(r.group_start)>(dlsym(h, "ncclGroupStart"));
  r.group_end = reinterpret_cast<decltype(r.group_end)>(dlsym(h, "ncclGroupEnd"));
  r.error_string = reinterpret_cast<decltype(r.error_string)>(dlsym(h, "ncclGetErrorString"));
  // a test library (tests/fake_rccl) exports this marker; it alone accepts
  // several communicator ranks on one device
  r.shared_devices = dlsym(h, "mr_fake_rccl_shared_devices") != nullptr;
  r.ok = r.comm_init_all && r.comm_destroy && r.all_gather && r.group_start && r.group_end && r.error_string;
  if (!r.ok) r.why = "the RCCL library lacks a required symbol";
  return r;
}

std::string rccl_path() {
  const char* e = std::getenv("MR_RCCL_LIB");
  return e ? std::string(e) : std::string();
}

#define G_NCCL(call)                                                                             \
  do {                                                                                           \
    ncclResult_t r_ = (call);                                                                    \
    if (r_ != ncclSuccess)                                                                       \
      return gfail(MR_E_RCCL, "%s failed: %s (%s:%d)", #call, G->rc->error_string(r_), __FILE__, \
                   __LINE__);                                                                    \
  } while (0)

template <typename T>
struct Buf {
  T* p = nullptr;
  int dev = 0;
  void release() {
    if (p) {
      (void)hipSetDevice(dev);
      (void)hipFree(p);
    }
    p = nullptr;
  }
};

template <typename T>
int alloc(Buf<T>& b, int dev, size_t n) {
  b.release();
  b.dev = dev;
  G_HIP(hipSetDevice(dev));
  G_HIP(hipMalloc(reinterpret_cast<void**>(&b.p), std::max<size_t>(1, n) * sizeof(T)));
  return MR_OK;
}

struct Member {
  mr_ctx* ctx = nullptr;
  int dev = 0;
  int block = 0, shard = 0;
  int user_lo = 0, user_hi = 0, song_lo = 0, song_hi = 0;
  hipStream_t stream = nullptr;  // the context's own stream
  hipEvent_t done = nullptr;     // end of this member's part of the last run / exchange
  ncclComm_t comm = nullptr;     // RCCL: communicator of the member's user block
  Buf<unsigned char> grec;       // gathered top-k record blocks [G_s][rec] (keys, then songs)
  int64_t rec = 0;               // bytes of one record block of this member's user block
  Buf<long long> mkey;           // merged [n_bk][k] lists
  Buf<int> msong;
  Buf<double> mscore;
  Buf<unsigned char> send, recv;  // RCCL dense: [n_bk][w_max] own shard, [G_s][n_bk][w_max] gathered
};

}  // namespace

struct mr_group {
  mr_options opt{};
  mr_group_options gopt{};
  int transport = MR_TRANSPORT_COPY;
  int n_s = 0, n_te = 0, w_max = 0;
  bool loaded = false, ran = false;
  std::vector<Member> m;  // index b * G_s + g
  std::vector<int> dev_of;
  Rccl* rc = nullptr;     // the RCCL library of this group (RCCL transport)

  int gs() const { return gopt.n_song_shards; }
  int gu() const { return gopt.n_user_blocks; }
  Member& at(int b, int g) { return m[(size_t)b * gs() + g]; }
  size_t esz() const { return opt.out_dtype == MR_OUT_F64 ? 8 : 4; }
  bool exchange() const { return opt.topk > 0 && (gs() > 1 || transport == MR_TRANSPORT_RCCL); }

  void release_members() {
    for (auto& x : m) {
      if (x.ctx) {
        (void)hipSetDevice(x.dev);
        (void)hipStreamSynchronize(x.stream);
      }
    }
    for (auto& x : m) {
      x.grec.release(); x.mkey.release(); x.msong.release(); x.mscore.release();
      x.send.release(); x.recv.release();
      if (x.comm && rc) (void)rc->comm_destroy(x.comm);
      x.comm = nullptr;
      if (x.done) { (void)hipSetDevice(x.dev); (void)hipEventDestroy(x.done); }
      x.done = nullptr;
      if (x.ctx) mr_destroy(x.ctx);
      x.ctx = nullptr;
    }
    loaded = ran = false;
  }
};

namespace {

// Song-range shards with ~equal Σ_s (c_tr(s) + 1) (stage-2 entries + one output
// per song) — the same rule as sharding.song_shards.
// Shard boundaries balancing sum(c_tr(s) + 1) (sharding.song_shards); with
// tile > 0 each boundary then moves the least so that no shard is wider than
// M tiles, M = ceil(ceil(n_songs / tile) / n): the wide kernel's work is one
// neighbour-list walk per (test user, tile), so a shard a few songs past a
// whole number of tiles pays a whole extra tile (C4 4 x 2: 6 tiles on one
// shard, 51.0 vs 47.5 ms per rank, profiles/r02/layouts_c4.txt).
std::vector<int> song_bounds(const mr_dataset* d, int n, int tile = 0) {
  std::vector<long long> cost(d->n_songs, 1);
  for (int64_t i = 0; i < d->tr_off[d->n_train_users]; ++i) cost[d->tr_songs[i]]++;
  for (int s = 1; s < d->n_songs; ++s) cost[s] += cost[s - 1];
  const long long total = cost.back();
  std::vector<int> b{0};
  for (int g = 1; g < n; ++g) {
    const double target = (double)(total * g) / n;
    const int i = (int)(std::lower_bound(cost.begin(), cost.end(), target,
                                         [](long long c, double t) { return (double)c < t; }) -
                        cost.begin());
    b.push_back(std::min(std::max(i + 1, b.back() + 1), d->n_songs - (n - g)));
  }
  b.push_back(d->n_songs);
  if (tile > 0) {
    const long long n_s = d->n_songs, tiles = (n_s + tile - 1) / tile;
    const long long cap = (tiles + n - 1) / n * tile;  // songs per shard at most
    for (int g = 1; g < n; ++g) {
      long long x = std::max<long long>(b[g], n_s - (long long)(n - g) * cap);
      x = std::min<long long>(x, b[g - 1] + cap);
      x = std::max<long long>(x, b[g - 1] + 1);
      b[g] = (int)std::min<long long>(x, n_s - (n - g));
    }
  }
  return b;
}

int wait_member(Member& dst, const Member& src) {
  G_HIP(hipSetDevice(src.dev));
  G_HIP(hipEventRecord(src.done, src.stream));
  G_HIP(hipSetDevice(dst.dev));
  G_HIP(hipStreamWaitEvent(dst.stream, src.done, 0));
  return MR_OK;
}

int run_group(mr_group* G, int model) {
  const int k = G->opt.topk;
  const bool rc_mode = G->transport == MR_TRANSPORT_RCCL;
  // The next run must not overwrite a member's lists / dense block before the
  // last exchange has read them: every member waits on its block root (COPY)
  // — in RCCL mode each member's collective sits on its own stream already.
  if (G->ran && !rc_mode && G->exchange())
    for (int b = 0; b < G->gu(); ++b)
      for (int g = 1; g < G->gs(); ++g) {
        int rc = wait_member(G->at(b, g), G->at(b, 0));
        if (rc) return rc;
      }
  for (auto& x : G->m) {
    const int rc = (rc_mode && G->opt.dense) ? mr_run_into(x.ctx, model, x.send.p) : mr_run(x.ctx, model);
    if (rc) return rc;
  }
  if (!G->exchange()) return MR_OK;
  const int gs = G->gs();
  if (rc_mode) {
    Rccl& R = *G->rc;
    G_NCCL(R.group_start());
    // ONE all-gather per member: its top-k record block (keys, then songs;
    // n_bk x k x 12 B) into [G_s][rec]. Every call between ncclGroupStart and
    // ncclGroupEnd; an error still closes the group (thread-global state).
    auto enqueue = [&]() -> int {
      for (auto& x : G->m) {
        void* rec;
        int64_t bytes;
        int rc = mr_internal::topk_records(x.ctx, &rec, &bytes);
        if (rc) return rc;
        if (bytes != x.rec) return gfail(MR_E_STATE, "record block of %lld B, %lld expected", (long long)bytes, (long long)x.rec);
        G_HIP(hipSetDevice(x.dev));
        G_NCCL(R.all_gather(rec, x.grec.p, (size_t)bytes / 8, ncclInt64, x.comm, x.stream));
      }
      return MR_OK;
    };
    const int erc = enqueue();
    const ncclResult_t end = R.group_end();
    if (erc) return erc;
    if (end != ncclSuccess) return gfail(MR_E_RCCL, "ncclGroupEnd: %s", R.error_string(end));
    for (auto& x : G->m) {
      const int rc = mr_internal::merge_records_async(x.ctx, gs, x.user_hi - x.user_lo, k, x.grec.p, x.rec, x.msong.p,
                                                      reinterpret_cast<int64_t*>(x.mkey.p), x.mscore.p);
      if (rc) return rc;
    }
    return MR_OK;
  }
  for (int b = 0; b < G->gu(); ++b) {  // COPY: the block root gathers the record blocks and merges
    Member& r = G->at(b, 0);
    for (int g = 0; g < gs; ++g) {
      Member& x = G->at(b, g);
      if (g > 0) {
        int rc = wait_member(r, x);
        if (rc) return rc;
      }
      void* rec;
      int64_t bytes;
      int rc = mr_internal::topk_records(x.ctx, &rec, &bytes);
      if (rc) return rc;
      G_HIP(hipSetDevice(r.dev));
      G_HIP(hipMemcpyAsync(r.grec.p + (size_t)g * r.rec, rec, (size_t)bytes, hipMemcpyDeviceToDevice, r.stream));
    }
    const int rc = mr_internal::merge_records_async(r.ctx, gs, r.user_hi - r.user_lo, k, r.grec.p, r.rec, r.msong.p,
                                                    reinterpret_cast<int64_t*>(r.mkey.p), r.mscore.p);
    if (rc) return rc;
  }
  return MR_OK;
}

int sync_all(mr_group* G) {
  for (auto& x : G->m) {
    G_HIP(hipSetDevice(x.dev));
    G_HIP(hipStreamSynchronize(x.stream));
  }
  return MR_OK;
}

const void* member_dense(mr_group* G, Member& x) {
  if (G->transport == MR_TRANSPORT_RCCL) return x.send.p;
  void* d = nullptr;
  if (mr_device_outputs(x.ctx, &d, nullptr, nullptr, nullptr)) return nullptr;
  return d;
}

}  // namespace

extern "C" {

int mr_song_shards(const mr_dataset* d, int32_t n_shards, int32_t* bounds) {
  if (!d || !bounds || !d->tr_off || (d->tr_off[d->n_train_users] > 0 && !d->tr_songs))
    return gfail(MR_E_INVALID, "null argument");
  if (n_shards < 1 || d->n_songs < n_shards)
    return gfail(MR_E_INVALID, "%d song shards over %d songs", n_shards, d->n_songs);
  for (int64_t i = 0; i < d->tr_off[d->n_train_users]; ++i)
    if (d->tr_songs[i] < 0 || d->tr_songs[i] >= d->n_songs) return gfail(MR_E_INVALID, "song id out of range");
  const std::vector<int> b = song_bounds(d, n_shards);
  std::copy(b.begin(), b.end(), bounds);
  return MR_OK;
}

int mr_song_shards_tiled(const mr_dataset* d, int32_t n_shards, int32_t tile_songs, int32_t* bounds) {
  const int rc = mr_song_shards(d, n_shards, bounds);
  if (rc || tile_songs <= 0) return rc;
  const std::vector<int> b = song_bounds(d, n_shards, tile_songs);
  std::copy(b.begin(), b.end(), bounds);
  return MR_OK;
}

int mr_group_options_default(mr_group_options* g) {
  if (!g) return gfail(MR_E_INVALID, "null group options");
  std::memset(g, 0, sizeof *g);
  g->n_song_shards = 1;
  g->n_user_blocks = 1;
  g->transport = MR_TRANSPORT_AUTO;
  return MR_OK;
}

int mr_group_create(const mr_options* opt, const mr_group_options* gopt, mr_group** out) {
  if (!out) return gfail(MR_E_INVALID, "null output pointer");
  *out = nullptr;
  mr_options o;
  if (opt) o = *opt; else mr_options_default(&o);
  mr_group_options go;
  if (gopt) go = *gopt; else mr_group_options_default(&go);
  if (go.n_song_shards < 1 || go.n_user_blocks < 1 || (long long)go.n_song_shards * go.n_user_blocks > 4096)
    return gfail(MR_E_INVALID, "layout %d song shards x %d user blocks invalid", go.n_song_shards, go.n_user_blocks);
  if (go.transport < MR_TRANSPORT_AUTO || go.transport > MR_TRANSPORT_RCCL)
    return gfail(MR_E_INVALID, "bad transport %d", go.transport);
  if (go.n_devices < 0 || (go.n_devices > 0 && !go.devices))
    return gfail(MR_E_INVALID, "n_devices %d with a null device list", go.n_devices);
  if (o.song_lo != 0 || o.song_hi != 0)
    return gfail(MR_E_INVALID, "song_lo/song_hi are set by the group (its shard layout)");
  const int G = go.n_song_shards * go.n_user_blocks;
  int ndev = 0;
  G_HIP(hipGetDeviceCount(&ndev));
  std::vector<int> dev(G);
  for (int i = 0; i < G; ++i) {
    dev[i] = go.n_devices > 0 ? go.devices[i % go.n_devices] : o.device;
    if (dev[i] < 0 || dev[i] >= ndev) return gfail(MR_E_INVALID, "device %d not present (%d devices)", dev[i], ndev);
  }
  std::vector<int> distinct(dev);
  std::sort(distinct.begin(), distinct.end());
  const int n_distinct = (int)(std::unique(distinct.begin(), distinct.end()) - distinct.begin());
  int transport = go.transport;
  if (transport == MR_TRANSPORT_AUTO) transport = n_distinct > 1 ? MR_TRANSPORT_RCCL : MR_TRANSPORT_COPY;
  if (transport == MR_TRANSPORT_COPY && n_distinct > 1)
    return gfail(MR_E_INVALID, "COPY transport keeps every context on one device (%d devices given)", n_distinct);
  // RCCL needs one distinct device per context; only a library that exports
  // the test marker (tests/fake_rccl, loaded through MR_RCCL_LIB: the
  // multi-context path on one GPU) may be handed shared devices — real RCCL,
  // whatever path names it, is never asked for two ranks on one GPU.
  Rccl* R = nullptr;
  if (transport == MR_TRANSPORT_RCCL) {
    R = &rccl_at(rccl_path());
    if (n_distinct != G && !(R->ok && R->shared_devices))
      return gfail(MR_E_INVALID, "RCCL transport needs one distinct device per context (%d contexts, %d devices)", G,
                   n_distinct);
    if (!R->ok) return gfail(MR_E_RCCL, "RCCL unavailable: %s", R->why.c_str());
  }
  mr_group* g = new mr_group();
  g->opt = o;
  g->gopt = go;
  g->gopt.devices = nullptr;  // not retained
  g->transport = transport;
  g->rc = R;
  g->dev_of = dev;
  g->m.resize(G);
  for (int i = 0; i < G; ++i) {
    Member& x = g->m[i];
    x.dev = dev[i];
    x.block = i / go.n_song_shards;
    x.shard = i % go.n_song_shards;
    mr_options oi = o;
    oi.device = x.dev;
    int rc = mr_create(&oi, &x.ctx);
    if (rc == MR_OK) {
      x.stream = (hipStream_t)mr_stream(x.ctx);
      hipError_t e = hipSetDevice(x.dev);
      if (e == hipSuccess) e = hipEventCreateWithFlags(&x.done, hipEventDisableTiming);
      if (e != hipSuccess) rc = gfail(MR_E_HIP, "hipEventCreate: %s", hipGetErrorString(e));
    }
    if (rc) {
      std::string msg = mr_last_error();
      g->release_members();
      delete g;
      return set_error(rc, msg.c_str());
    }
  }
  if (transport == MR_TRANSPORT_RCCL) {
    for (int b = 0; b < go.n_user_blocks; ++b) {
      std::vector<ncclComm_t> comms(go.n_song_shards);
      std::vector<int> devs(go.n_song_shards);
      for (int s = 0; s < go.n_song_shards; ++s) devs[s] = g->at(b, s).dev;
      const ncclResult_t r = R->comm_init_all(comms.data(), go.n_song_shards, devs.data());
      if (r != ncclSuccess) {
        g->release_members();
        delete g;
        return gfail(MR_E_RCCL, "ncclCommInitAll over %d devices: %s", go.n_song_shards, R->error_string(r));
      }
      for (int s = 0; s < go.n_song_shards; ++s) g->at(b, s).comm = comms[s];
    }
  }
  *out = g;
  return MR_OK;
}

int mr_group_destroy(mr_group* g) {
  if (!g) return MR_OK;
  g->release_members();
  delete g;
  return MR_OK;
}

int mr_group_load(mr_group* g, const mr_dataset* d) {
  if (!g || !d) return gfail(MR_E_INVALID, "null argument");
  // mr_load's checks first: song_bounds below indexes by the caller's song ids
  if (int rc = mr_internal::validate_dataset(d)) return rc;
  if (d->n_test_users < g->gu() || d->n_songs < g->gs())
    return gfail(MR_E_INVALID, "%d test users / %d songs cannot form %d user blocks x %d song shards",
                 d->n_test_users, d->n_songs, g->gu(), g->gs());
  int rc = sync_all(g);
  if (rc) return rc;
  g->loaded = g->ran = false;
  // A reload frees the old contexts' device data before the new ones load
  // (else device memory peaks at two full loads). The contexts themselves are
  // recreated below: the shard geometry is a creation option.
  for (auto& x : g->m) {
    if (x.ctx) mr_destroy(x.ctx);
    x.ctx = nullptr;
    x.stream = nullptr;
  }
  int tile = 0;  // the wide shape's tile when the contexts will use it (mr_shard_tile_songs)
  if (int rc = mr_shard_tile_songs_n(&g->opt, d->n_train_users, d->n_test_users / g->gu(), d->n_songs, g->gs(), &tile))
    return rc;
  const std::vector<int> sb = song_bounds(d, g->gs(), tile);
  // Per user block: a view of the dataset over its test users (te_off rebased).
  std::vector<std::vector<int64_t>> te_off(g->gu());
  std::vector<mr_dataset> views(g->gu(), *d);
  for (int b = 0; b < g->gu(); ++b) {
    const int lo = (int)((long long)d->n_test_users * b / g->gu());
    const int hi = (int)((long long)d->n_test_users * (b + 1) / g->gu());
    te_off[b].resize(hi - lo + 1);
    for (int u = lo; u <= hi; ++u) te_off[b][u - lo] = d->te_off[u] - d->te_off[lo];
    views[b].n_test_users = hi - lo;
    views[b].te_off = te_off[b].data();
    views[b].te_songs = d->te_songs + d->te_off[lo];
    views[b].te_len = d->te_len + lo;
    for (int s = 0; s < g->gs(); ++s) {
      Member& x = g->at(b, s);
      x.user_lo = lo; x.user_hi = hi;
      x.song_lo = sb[s]; x.song_hi = sb[s + 1];
    }
  }
  int w_max = 0;
  for (int s = 0; s < g->gs(); ++s) w_max = std::max(w_max, sb[s + 1] - sb[s]);
  // Load every context in parallel (each builds its shard's host-side index).
  std::vector<int> rcs(g->m.size(), MR_OK);
  std::vector<std::string> msgs(g->m.size());
  {
    std::vector<std::thread> th;
    for (size_t i = 0; i < g->m.size(); ++i)
      th.emplace_back([&, i] {
        Member& x = g->m[i];
        mr_options oi = g->opt;
        oi.device = x.dev;
        oi.song_lo = x.song_lo;
        oi.song_hi = x.song_hi;
        // the shard geometry is a creation option of a context: recreate it
        mr_ctx* c = nullptr;
        int r = mr_create(&oi, &c);
        if (r == MR_OK) {  // contexts on the same device split its neighbour-list budget
          int share = 0;
          for (const Member& y : g->m) share += y.dev == x.dev ? 1 : 0;
          r = mr_internal::set_device_share(c, share);
        }
        if (r == MR_OK) r = mr_load(c, &views[x.block]);
        if (r != MR_OK) {
          msgs[i] = mr_last_error();
          if (c) mr_destroy(c);
          rcs[i] = r;
          return;
        }
        x.ctx = c;
        x.stream = (hipStream_t)mr_stream(c);
      });
    for (auto& t : th) t.join();
  }
  for (size_t i = 0; i < g->m.size(); ++i)
    if (rcs[i]) return set_error(rcs[i], ("context " + std::to_string(i) + ": " + msgs[i]).c_str());
  // Exchange buffers.
  const int k = g->opt.topk;
  const bool rc_mode = g->transport == MR_TRANSPORT_RCCL;
  for (auto& x : g->m) {
    const size_t n = (size_t)(x.user_hi - x.user_lo) * std::max(k, 1);
    const bool holds = rc_mode || x.shard == 0;  // gathers + merges here
    x.rec = 0;
    if (k > 0 && (rc = mr_topk_record_bytes(x.user_hi - x.user_lo, k, &x.rec))) return rc;
    if (g->exchange() && holds) {
      if ((rc = alloc(x.grec, x.dev, (size_t)x.rec * g->gs())) || (rc = alloc(x.mkey, x.dev, n)) ||
          (rc = alloc(x.msong, x.dev, n)) || (rc = alloc(x.mscore, x.dev, n)))
        return rc;
    }
    if (rc_mode && g->opt.dense)
      if ((rc = alloc(x.send, x.dev, (size_t)(x.user_hi - x.user_lo) * w_max * g->esz()))) return rc;
    x.recv.release();
  }
  g->n_s = d->n_songs;
  g->n_te = d->n_test_users;
  g->w_max = w_max;
  g->loaded = true;
  return MR_OK;
}

int mr_group_info(const mr_group* g, int32_t i, int32_t* song_lo, int32_t* song_hi, int32_t* user_lo,
                  int32_t* user_hi, int32_t* device) {
  if (!g) return gfail(MR_E_INVALID, "null group");
  if (i < 0 || i >= (int)g->m.size()) return gfail(MR_E_INVALID, "context %d outside [0,%zu)", i, g->m.size());
  if (!g->loaded) return gfail(MR_E_STATE, "mr_group_info before mr_group_load");
  const Member& x = g->m[i];
  if (song_lo) *song_lo = x.song_lo;
  if (song_hi) *song_hi = x.song_hi;
  if (user_lo) *user_lo = x.user_lo;
  if (user_hi) *user_hi = x.user_hi;
  if (device) *device = x.dev;
  return MR_OK;
}

int mr_group_transport(const mr_group* g, int32_t* transport) {
  if (!g || !transport) return gfail(MR_E_INVALID, "null argument");
  *transport = g->transport;
  return MR_OK;
}

int mr_group_shape(const mr_group* g, int32_t* n_contexts, int32_t* n_test, int32_t* n_songs) {
  if (!g) return gfail(MR_E_INVALID, "null group");
  if (!g->loaded) return gfail(MR_E_STATE, "mr_group_shape before mr_group_load");
  if (n_contexts) *n_contexts = (int32_t)g->m.size();
  if (n_test) *n_test = g->n_te;
  if (n_songs) *n_songs = g->n_s;
  return MR_OK;
}

mr_ctx* mr_group_context(mr_group* g, int32_t i) {
  if (!g || i < 0 || i >= (int)g->m.size() || !g->loaded) {
    gfail(MR_E_INVALID, "no context %d", i);
    return nullptr;
  }
  return g->m[i].ctx;
}

int mr_group_run(mr_group* g, int model) {
  if (!g) return gfail(MR_E_INVALID, "null group");
  if (!g->loaded) return gfail(MR_E_STATE, "mr_group_run before mr_group_load");
  if (model != MR_UBM && model != MR_IBM) return gfail(MR_E_INVALID, "unknown model %d", model);
  const int rc = run_group(g, model);
  if (rc) return rc;
  g->ran = true;
  return MR_OK;
}

int mr_group_sync(mr_group* g) {
  if (!g) return gfail(MR_E_INVALID, "null group");
  return sync_all(g);
}

int mr_group_copy_topk(mr_group* g, int32_t* songs, double* scores, int64_t* keys) {
  if (!g) return gfail(MR_E_INVALID, "null group");
  if (!g->ran) return gfail(MR_E_STATE, "no mr_group_run yet");
  const int k = g->opt.topk;
  if (k <= 0) return gfail(MR_E_STATE, "group created with topk=0");
  for (int b = 0; b < g->gu(); ++b) {
    Member& r = g->at(b, 0);
    const size_t n = (size_t)(r.user_hi - r.user_lo) * k, o = (size_t)r.user_lo * k;
    const int32_t* ts = r.msong.p;
    const int64_t* tk = reinterpret_cast<const int64_t*>(r.mkey.p);
    const double* tsc = r.mscore.p;
    if (!g->exchange()) {
      int32_t* a;
      int64_t* bk;
      double* c;
      int rc = mr_device_outputs(r.ctx, nullptr, &a, &bk, &c);
      if (rc) return rc;
      ts = a; tk = bk; tsc = c;
    }
    G_HIP(hipSetDevice(r.dev));
    if (songs) G_HIP(hipMemcpyAsync(songs + o, ts, n * 4, hipMemcpyDeviceToHost, r.stream));
    if (keys) G_HIP(hipMemcpyAsync(keys + o, tk, n * 8, hipMemcpyDeviceToHost, r.stream));
    if (scores) G_HIP(hipMemcpyAsync(scores + o, tsc, n * 8, hipMemcpyDeviceToHost, r.stream));
  }
  return sync_all(g);
}

int mr_group_topk(mr_group* g, int model, int k, int32_t* songs, double* scores, int64_t* keys) {
  if (!g) return gfail(MR_E_INVALID, "null group");
  if (k != g->opt.topk) return gfail(MR_E_INVALID, "k=%d differs from the group's topk=%d", k, g->opt.topk);
  int rc = mr_group_run(g, model);
  if (rc) return rc;
  return mr_group_copy_topk(g, songs, scores, keys);
}

int mr_group_device_topk(mr_group* g, int32_t i, int32_t** songs, int64_t** keys, double** scores) {
  if (!g) return gfail(MR_E_INVALID, "null group");
  if (!g->ran) return gfail(MR_E_STATE, "no mr_group_run yet");
  if (i < 0 || i >= (int)g->m.size()) return gfail(MR_E_INVALID, "context %d outside [0,%zu)", i, g->m.size());
  Member& x = g->m[i];
  if (!g->exchange()) return mr_device_outputs(x.ctx, nullptr, songs, keys, scores);
  if (!x.msong.p) return gfail(MR_E_INVALID, "context %d holds no merged lists (COPY: the block's first context does)", i);
  if (songs) *songs = x.msong.p;
  if (keys) *keys = reinterpret_cast<int64_t*>(x.mkey.p);
  if (scores) *scores = x.mscore.p;
  return MR_OK;
}

int mr_group_copy_dense(mr_group* g, void* out) {
  if (!g || !out) return gfail(MR_E_INVALID, "null argument");
  if (!g->ran) return gfail(MR_E_STATE, "no mr_group_run yet");
  if (!g->opt.dense) return gfail(MR_E_STATE, "group created with dense=0");
  const size_t e = g->esz();
  if (int rc = sync_all(g)) return rc;
  // one context at a time through its pinned staging (d2h_staged): the
  // host threads of the staged copy serve one transfer at once
  for (auto& x : g->m) {
    const void* src = member_dense(g, x);
    if (!src) return gfail(MR_E_STATE, "context without a dense model");
    const size_t w = (size_t)(x.song_hi - x.song_lo);
    G_HIP(hipSetDevice(x.dev));
    if (int rc = mr_internal::d2h_staged(x.ctx, static_cast<char*>(out) + ((size_t)x.user_lo * g->n_s + x.song_lo) * e,
                                         (size_t)g->n_s * e, src, w * e, w * e, (size_t)(x.user_hi - x.user_lo)))
      return rc;
  }
  return MR_OK;
}

int mr_group_score_dense(mr_group* g, int model, void* out) {
  int rc = mr_group_run(g, model);
  if (rc) return rc;
  return mr_group_copy_dense(g, out);
}

int mr_group_allgather_dense(mr_group* g, void* const* dst) {
  mr_group* G = g;  // G_NCCL reports through G->rc
  if (!g || !dst) return gfail(MR_E_INVALID, "null argument");
  if (!g->ran) return gfail(MR_E_STATE, "no mr_group_run yet");
  if (!g->opt.dense) return gfail(MR_E_STATE, "group created with dense=0");
  const size_t e = g->esz();
  const int gs = g->gs();
  if (g->transport == MR_TRANSPORT_RCCL) {
    for (auto& x : g->m) {
      if (!x.recv.p) {
        int rc = alloc(x.recv, x.dev, (size_t)gs * (x.user_hi - x.user_lo) * g->w_max * e);
        if (rc) return rc;
      }
    }
    Rccl& R = *g->rc;
    const ncclDataType_t t = g->opt.out_dtype == MR_OUT_F64 ? ncclFloat64 : ncclFloat32;
    G_NCCL(R.group_start());
    auto enqueue = [&]() -> int {
      for (auto& x : g->m) {
        G_HIP(hipSetDevice(x.dev));
        G_NCCL(R.all_gather(x.send.p, x.recv.p, (size_t)(x.user_hi - x.user_lo) * g->w_max, t, x.comm, x.stream));
      }
      return MR_OK;
    };
    const int erc = enqueue();
    const ncclResult_t end = R.group_end();
    if (erc) return erc;
    if (end != ncclSuccess) return gfail(MR_E_RCCL, "ncclGroupEnd: %s", R.error_string(end));
    for (auto& x : g->m) {  // [G_s][n_bk][w_max] -> rows of n_songs
      const size_t nbk = (size_t)(x.user_hi - x.user_lo);
      G_HIP(hipSetDevice(x.dev));
      for (int s = 0; s < gs; ++s) {
        const Member& y = g->at(x.block, s);
        const size_t w = (size_t)(y.song_hi - y.song_lo);
        G_HIP(hipMemcpy2DAsync(static_cast<char*>(dst[&x - g->m.data()]) + (size_t)y.song_lo * e, (size_t)g->n_s * e,
                               x.recv.p + (size_t)s * nbk * g->w_max * e, w * e, w * e, nbk,
                               hipMemcpyDeviceToDevice, x.stream));
      }
    }
    return sync_all(g);
  }
  for (auto& x : g->m) {  // COPY: every context's rows from its block's shards
    const size_t nbk = (size_t)(x.user_hi - x.user_lo);
    for (int s = 0; s < gs; ++s) {
      Member& y = g->at(x.block, s);
      if (&y != &x) {
        int rc = wait_member(x, y);
        if (rc) return rc;
      }
      const void* src = member_dense(g, y);
      if (!src) return gfail(MR_E_STATE, "context without a dense model");
      const size_t w = (size_t)(y.song_hi - y.song_lo);
      G_HIP(hipSetDevice(x.dev));
      G_HIP(hipMemcpy2DAsync(static_cast<char*>(dst[&x - g->m.data()]) + (size_t)y.song_lo * e, (size_t)g->n_s * e,
                             src, w * e, w * e, nbk, hipMemcpyDeviceToDevice, x.stream));
    }
  }
  return sync_all(g);
}

}  // extern "C"
