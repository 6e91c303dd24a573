// mr_host.cpp — host-side part of the engine's C ABI (no GPU needed):
//  * parallel TSV ingest + string interning + CSR build, replacing extractData /
//    songs / songsToUsersMap / importTestLabels (MusicRecommender.scala MR:26-91);
//  * the per-shard top-k merge on the host (exchange step of a song-sharded run).
//
// Ingest, every phase on all usable cores (mr_par.h):
//  1. read   — each file pread in parallel ranges into one buffer;
//  2. parse  — the buffer cut at line starts into one part per thread; a part
//              splits its lines (Java String.split("\t") semantics) and interns
//              user / song names in its own open-addressing table (no shared state);
//  3. intern — per name kind, every part's distinct names sorted, then merged
//              over key ranges cut by sampled splitters (one range per thread,
//              a heap merge per range): the global ids come out in lexicographic
//              order directly (main.scala:57-59's sort key), no global hash table;
//  4. CSR    — rows remapped to global ids, counted, scattered, and each row
//              sorted + de-duplicated (counts keep duplicates, MR:44-46, MR:147).
// The C4 shape (48.4M rows, 1M users, 385k songs) is the size this is built for.
#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <memory>
#include <string>
#include <string_view>
#include <thread>
#include <vector>

#include "mr_engine.h"
#include "mr_par.h"

namespace mr_host {
// Error slot shared with the device part through these two functions
// (mr_last_error lives in mr_engine.hip).
int fail(int code, const char* fmt, ...);
}  // namespace mr_host

namespace {

using sv = std::string_view;

// Threads of the ingest: MR_INGEST_THREADS, else every usable core (<= 64).
int n_threads() {
  const char* e = std::getenv("MR_INGEST_THREADS");
  const int t = e ? std::atoi(e) : mr_par::usable_cores();
  return std::max(1, std::min(t, 64));
}

using Trace = mr_par::PhaseTrace;

// ---- 1. read -------------------------------------------------------------------
struct Text {
  mr_par::buffer<char> p;  // uninitialised: the reads fill it (no 3 GB zero pass)
  size_t n = 0;
  const char* data() const { return p.data(); }
};

int read_file(const char* path, Text& out) {
  const int fd = ::open(path, O_RDONLY);
  if (fd < 0) return mr_host::fail(MR_E_IO, "cannot open %s", path);
  struct stat st;
  if (::fstat(fd, &st) != 0 || st.st_size < 0) {
    ::close(fd);
    return mr_host::fail(MR_E_IO, "cannot size %s", path);
  }
  out.n = (size_t)st.st_size;
  try {
    out.p.resize(std::max<size_t>(1, out.n));
  } catch (const std::bad_alloc&) {
    ::close(fd);
    return mr_host::fail(MR_E_OOM, "cannot hold %s (%zu B)", path, out.n);
  }
  std::atomic<bool> bad{false};
  mr_par::parallel_for(
      (int64_t)out.n,
      [&](int64_t lo, int64_t hi, int) {
        while (lo < hi) {
          const ssize_t got = ::pread(fd, out.p.data() + lo, (size_t)std::min<int64_t>(hi - lo, 1 << 30), lo);
          if (got <= 0) {
            bad = true;
            return;
          }
          lo += got;
        }
      },
      (int64_t)32 << 20, n_threads());
  ::close(fd);
  if (bad) return mr_host::fail(MR_E_IO, "short read of %s", path);
  return MR_OK;
}

// ---- 2. parse ------------------------------------------------------------------
inline uint64_t hash_name(const char* p, size_t n) {
  uint64_t h = 0x9E3779B97F4A7C15ull ^ (uint64_t)n;
  while (n >= 8) {
    uint64_t w;
    std::memcpy(&w, p, 8);
    h = (h ^ w) * 0xBF58476D1CE4E5B9ull;
    h ^= h >> 31;
    p += 8;
    n -= 8;
  }
  uint64_t w = 0;
  std::memcpy(&w, p, n);
  h ^= w;  // murmur3 fmix64: every input bit reaches the low (slot) bits
  h ^= h >> 33;
  h *= 0xFF51AFD7ED558CCDull;
  h ^= h >> 33;
  h *= 0xC4CEB9FE1A85EC53ull;
  h ^= h >> 33;
  return h;
}

// Open-addressing interning table of one part: names in first-seen order,
// their bytes copied into a compact arena (a probe then touches the 8-B slot
// and the arena, both cache-friendly for the popular names, never the text).
struct NameTable {
  std::vector<uint64_t> slot;  // (hash >> 32) << 32 | (id + 1); 0 = empty
  std::vector<uint64_t> off;   // arena offset of name id
  std::vector<uint32_t> len;
  std::vector<char> arena;
  uint64_t mask = 0;

  NameTable() {
    slot.assign(1 << 12, 0);
    mask = slot.size() - 1;
    arena.reserve(1 << 16);
  }
  size_t size() const { return off.size(); }
  sv name(size_t id) const { return sv(arena.data() + off[id], len[id]); }
  void grow() {
    std::vector<uint64_t> old(slot.size() * 2, 0);
    old.swap(slot);
    mask = slot.size() - 1;
    for (uint64_t e : old) {
      if (!e) continue;
      const uint32_t id = (uint32_t)e - 1;
      uint64_t i = hash_name(arena.data() + off[id], len[id]) & mask;
      while (slot[i]) i = (i + 1) & mask;
      slot[i] = e;
    }
  }
  void prefetch(uint64_t h) const { __builtin_prefetch(&slot[h & mask]); }
  void prefetch_name(uint64_t h) const {  // the first tag match's bytes
    const uint64_t t = h >> 32;
    for (uint64_t i = h & mask;; i = (i + 1) & mask) {
      const uint64_t e = slot[i];
      if (!e) return;
      if ((e >> 32) == t) {
        __builtin_prefetch(arena.data() + off[(uint32_t)e - 1]);
        return;
      }
    }
  }
  int get(const char* p, size_t n, uint64_t h) {
    const uint64_t t = h >> 32;
    uint64_t i = h & mask;
    while (uint64_t e = slot[i]) {
      if ((e >> 32) == t) {
        const uint32_t id = (uint32_t)e - 1;
        if (len[id] == n && std::memcmp(arena.data() + off[id], p, n) == 0) return (int)id;
      }
      i = (i + 1) & mask;
    }
    const uint32_t id = (uint32_t)off.size();
    off.push_back(arena.size());
    len.push_back((uint32_t)n);
    arena.insert(arena.end(), p, p + n);
    slot[i] = (t << 32) | (id + 1);
    if (off.size() * 2 > slot.size()) grow();
    return (int)id;
  }
  std::vector<sv> names() const {
    std::vector<sv> v(size());
    for (size_t i = 0; i < v.size(); ++i) v[i] = name(i);
    return v;
  }
};

struct Part {  // one thread's share of one file
  NameTable users, songs;
  std::vector<sv> user_names, song_names;  // views of the tables' arenas, after parsing
  std::vector<int32_t> ru, rs;  // rows as part-local ids (global ids after remap)
  size_t err_off = SIZE_MAX;
  int err_fields = 0;
};

// Lines are split in batches: every line's song hash is computed and its slot
// prefetched, then the candidate names' bytes, then the lookups run — the
// table's cache misses overlap instead of serialising (~6x at C4 size).
void parse_chunk(const char* p, size_t a, size_t b, Part& c) {
  constexpr int B = 16;
  struct Line {
    size_t start;
    const char *u, *s;
    uint32_t ul, sl;
    uint64_t h;
  } L[B];
  sv last_user;
  int last_uid = -1;
  size_t i = a;
  while (i < b) {
    int n = 0;
    for (; n < B && i < b; ++n) {
      const char* nl = static_cast<const char*>(std::memchr(p + i, '\n', b - i));
      const size_t end = nl ? (size_t)(nl - p) : b;
      size_t le = end;
      if (le > i && p[le - 1] == '\r') --le;  // getLines strips \r\n
      int nf = 0, last_ne = -1;
      sv f0, f1;
      size_t s = i;
      while (true) {
        const char* t = static_cast<const char*>(std::memchr(p + s, '\t', le - s));
        const size_t fe = t ? (size_t)(t - p) : le;
        if (fe > s) last_ne = nf;
        if (nf == 0) f0 = sv(p + s, fe - s);
        else if (nf == 1) f1 = sv(p + s, fe - s);
        ++nf;
        if (!t) break;
        s = fe + 1;
      }
      if (last_ne + 1 != 3) {  // scala.MatchError (MR:34): Array(u, s, _) after split
        c.err_off = i;
        c.err_fields = last_ne + 1;
        return;
      }
      Line& x = L[n];
      x.start = i;
      x.u = f0.data();
      x.ul = (uint32_t)f0.size();
      x.s = f1.data();
      x.sl = (uint32_t)f1.size();
      x.h = hash_name(x.s, x.sl);
      c.songs.prefetch(x.h);
      i = nl ? end + 1 : b;
    }
    for (int k = 0; k < n; ++k) c.songs.prefetch_name(L[k].h);
    for (int k = 0; k < n; ++k) {
      const Line& x = L[k];
      // the triplet files are grouped by user: most lines repeat the last user
      const sv u(x.u, x.ul);
      if (last_uid < 0 || u != last_user) {
        last_uid = c.users.get(x.u, x.ul, hash_name(x.u, x.ul));
        last_user = u;
      }
      c.ru.push_back(last_uid);
      c.rs.push_back(c.songs.get(x.s, x.sl, x.h));
    }
  }
}

int parse_file(const char* path, const Text& text, std::vector<Part>& parts) {
  const size_t n = text.n;
  // chunks of >= 1 MiB (MR_INGEST_MIN_CHUNK overrides, e.g. to split small files in tests)
  const char* mc = std::getenv("MR_INGEST_MIN_CHUNK");
  const size_t min_chunk = mc ? std::max<size_t>(1, (size_t)std::atoll(mc)) : ((size_t)1 << 20);
  const int T = (int)std::max<size_t>(1, std::min<size_t>((size_t)n_threads(), n / min_chunk + 1));
  std::vector<size_t> cut(T + 1, n);
  cut[0] = 0;
  for (int t = 1; t < T; ++t) {
    size_t x = std::max(cut[t - 1], n * t / T);
    while (x < n && x > 0 && text.p[x - 1] != '\n') ++x;
    cut[t] = x;
  }
  parts.clear();
  parts.resize(T);
  mr_par::parallel_for(
      T,
      [&](int64_t lo, int64_t hi, int) {
        for (int64_t t = lo; t < hi; ++t) {
          parts[t].ru.reserve((cut[t + 1] - cut[t]) / 48 + 16);
          parts[t].rs.reserve((cut[t + 1] - cut[t]) / 48 + 16);
          parse_chunk(text.data(), cut[t], cut[t + 1], parts[t]);
          parts[t].user_names = parts[t].users.names();
          parts[t].song_names = parts[t].songs.names();
        }
      },
      1, T);
  size_t bad = SIZE_MAX;
  int fields = 0;
  for (auto& c : parts)
    if (c.err_off < bad) { bad = c.err_off; fields = c.err_fields; }
  if (bad != SIZE_MAX) {
    const size_t lineno = 1 + (size_t)std::count(text.data(), text.data() + bad, '\n');
    return mr_host::fail(MR_E_PARSE, "%s:%zu: expected 3 tab-separated fields, got %d", path, lineno, fields);
  }
  return MR_OK;
}

// ---- 3. intern -----------------------------------------------------------------
// Global lexicographic interning of the distinct names of several parts.
struct Interned {
  std::vector<sv> names;                 // distinct, sorted
  std::vector<std::vector<int32_t>> id;  // per part: part-local id -> global id
};

Interned intern(const std::vector<const std::vector<sv>*>& parts) {
  const int P = (int)parts.size();
  Interned out;
  out.id.resize(P);
  size_t total = 0;
  for (int p = 0; p < P; ++p) total += parts[p]->size();
  // 1. key ranges: splitters at the quantiles of a regular sample of every part
  //    (the parts overlap heavily, so ranges hold similar distinct counts)
  const int R = (int)std::max<size_t>(1, std::min<size_t>((size_t)n_threads() * 4, total / 4096 + 1));
  std::vector<sv> sample;
  for (int p = 0; p < P; ++p) {
    const size_t m = parts[p]->size(), step = std::max<size_t>(1, m / ((size_t)R * 16));
    for (size_t i = step / 2; i < m; i += step) sample.push_back((*parts[p])[i]);
  }
  std::sort(sample.begin(), sample.end());
  std::vector<sv> split;  // range r = [split[r-1], split[r])
  for (int r = 1; r < R && !sample.empty(); ++r) {
    const sv k = sample[sample.size() * r / R];
    if (split.empty() || split.back() < k) split.push_back(k);
  }
  const int NR = (int)split.size() + 1;
  // 2. every part's names cut into ranges (local ids per (part, range))
  std::vector<std::vector<int32_t>> in((size_t)P * NR);
  mr_par::parallel_dynamic(P, 1, [&](int64_t p, int) {
    const std::vector<sv>& nm = *parts[p];
    out.id[p].resize(nm.size());
    for (size_t i = 0; i < nm.size(); ++i) {
      const int r = (int)(std::upper_bound(split.begin(), split.end(), nm[i]) - split.begin());
      in[(size_t)p * NR + r].push_back((int32_t)i);
    }
  });
  // 3. per range: distinct names by hashing, sorted; the ranges concatenate in
  //    lexicographic order, so a name's global id = range base + rank in range
  std::vector<std::vector<sv>> rnames(NR);
  mr_par::parallel_dynamic(NR, 1, [&](int64_t r, int) {
    size_t m = 0;
    for (int p = 0; p < P; ++p) m += in[(size_t)p * NR + r].size();
    size_t cap = 64;
    while (cap < 2 * m) cap *= 2;
    std::vector<int32_t> slot(cap, -1);
    auto& names = rnames[r];
    for (int p = 0; p < P; ++p)
      for (int32_t i : in[(size_t)p * NR + r]) {
        const sv s = (*parts[p])[i];
        size_t k = hash_name(s.data(), s.size()) & (cap - 1);
        while (slot[k] >= 0 && names[slot[k]] != s) k = (k + 1) & (cap - 1);
        if (slot[k] < 0) {
          slot[k] = (int32_t)names.size();
          names.push_back(s);
        }
        out.id[p][i] = slot[k];
      }
    std::vector<int32_t> order(names.size()), rank(names.size());
    for (size_t i = 0; i < order.size(); ++i) order[i] = (int32_t)i;
    std::sort(order.begin(), order.end(), [&](int32_t x, int32_t y) { return names[x] < names[y]; });
    std::vector<sv> sorted(names.size());
    for (size_t j = 0; j < order.size(); ++j) {
      rank[order[j]] = (int32_t)j;
      sorted[j] = names[order[j]];
    }
    names.swap(sorted);
    for (int p = 0; p < P; ++p)
      for (int32_t i : in[(size_t)p * NR + r]) out.id[p][i] = rank[out.id[p][i]];
  });
  std::vector<int32_t> base(NR + 1, 0);
  for (int r = 0; r < NR; ++r) base[r + 1] = base[r] + (int32_t)rnames[r].size();
  out.names.resize(base[NR]);
  mr_par::parallel_dynamic(NR, 1, [&](int64_t r, int) {
    std::copy(rnames[r].begin(), rnames[r].end(), out.names.begin() + base[r]);
    for (int p = 0; p < P; ++p)
      for (int32_t i : in[(size_t)p * NR + r]) out.id[p][i] += base[r];
  });
  return out;
}

// ---- 4. CSR --------------------------------------------------------------------
struct Rows {  // (user, song) global ids of one part
  const std::vector<int32_t>* u;
  const std::vector<int32_t>* s;
};

// Rows -> CSR by user with sorted distinct columns; len[u] = row length with
// duplicates (MR:147). Deterministic whatever the scatter order: every row is
// sorted afterwards. Runs of equal users (the files are grouped by user) take
// one atomic each.
template <class OffVec, class ColVec>
void build_csr(int n_users, const std::vector<Rows>& rows, OffVec& off, ColVec& col, std::vector<int32_t>* len) {
  std::vector<int64_t> start((size_t)n_users + 1, 0);
  mr_par::parallel_dynamic((int64_t)rows.size(), 1, [&](int64_t p, int) {
    const auto& U = *rows[p].u;
    for (size_t i = 0; i < U.size();) {
      size_t j = i + 1;
      while (j < U.size() && U[j] == U[i]) ++j;
      __atomic_fetch_add(&start[U[i]], (int64_t)(j - i), __ATOMIC_RELAXED);
      i = j;
    }
  });
  if (len) {
    len->resize(n_users);
    mr_par::parallel_for(n_users, [&](int64_t lo, int64_t hi, int) {
      for (int64_t u = lo; u < hi; ++u) (*len)[u] = (int32_t)start[u];
    });
  }
  const int64_t total = mr_par::exclusive_scan(start.data(), (int64_t)n_users);
  start[n_users] = total;
  std::vector<int64_t> cur(start.begin(), start.end() - 1);
  mr_par::buffer<int32_t> tmp((size_t)std::max<int64_t>(1, total));
  mr_par::parallel_dynamic((int64_t)rows.size(), 1, [&](int64_t p, int) {
    const auto& U = *rows[p].u;
    const auto& S = *rows[p].s;
    for (size_t i = 0; i < U.size();) {
      size_t j = i + 1;
      while (j < U.size() && U[j] == U[i]) ++j;
      const int64_t at = __atomic_fetch_add(&cur[U[i]], (int64_t)(j - i), __ATOMIC_RELAXED);
      std::copy(S.begin() + i, S.begin() + j, tmp.begin() + at);
      i = j;
    }
  });
  std::vector<int64_t> uniq((size_t)n_users + 1, 0);
  mr_par::parallel_dynamic(n_users, 1024, [&](int64_t u, int) {
    auto b = tmp.begin() + start[u], e = tmp.begin() + start[u + 1];
    if (!std::is_sorted(b, e)) std::sort(b, e);
    uniq[u] = std::unique(b, e) - b;
  });
  const int64_t nnz = mr_par::exclusive_scan(uniq.data(), (int64_t)n_users);
  uniq[n_users] = nnz;
  col.resize((size_t)nnz);
  mr_par::parallel_for(n_users, [&](int64_t lo, int64_t hi, int) {
    for (int64_t u = lo; u < hi; ++u)
      std::copy(tmp.begin() + start[u], tmp.begin() + start[u] + (uniq[u + 1] - uniq[u]), col.begin() + uniq[u]);
  }, 4096);
  off.assign(uniq.begin(), uniq.end());
}

// Names of one kind as one NUL-separated blob (mr_corpus_name hands out
// pointers into it) built in parallel.
struct NameBlob {
  std::vector<char> bytes;
  std::vector<int64_t> at;  // [n + 1] start of name i
  size_t size() const { return at.empty() ? 0 : at.size() - 1; }
  void append_sorted(const std::vector<sv>& names) {  // appends after the current names
    const size_t n0 = size();
    if (at.empty()) at.push_back(0);
    at.resize(n0 + names.size() + 1);
    for (size_t i = 0; i < names.size(); ++i) at[n0 + i + 1] = at[n0 + i] + (int64_t)names[i].size() + 1;
    bytes.resize((size_t)at.back());
    mr_par::parallel_for((int64_t)names.size(), [&](int64_t lo, int64_t hi, int) {
      for (int64_t i = lo; i < hi; ++i) {
        char* o = bytes.data() + at[n0 + i];
        std::memcpy(o, names[i].data(), names[i].size());
        o[names[i].size()] = '\0';
      }
    });
  }
  const char* get(size_t i) const { return bytes.data() + at[i]; }
  int64_t len(size_t i) const { return at[i + 1] - at[i] - 1; }
};

}  // namespace

struct mr_corpus {
  NameBlob song_names;  // n_songs + n_extra (label-only songs last)
  NameBlob train_names, test_names;
  int n_songs = 0, n_extra = 0, n_label_songs = 0;
  std::vector<int64_t> tr_off, te_off, lab_off;
  mr_par::buffer<int32_t> tr_songs, te_songs, lab_songs;
  std::vector<int32_t> song_count, tr_len, te_len;
};

namespace {

std::vector<const std::vector<sv>*> user_names(const std::vector<Part>& parts) {
  std::vector<const std::vector<sv>*> v;
  for (auto& p : parts) v.push_back(&p.user_names);
  return v;
}

// Remap a part's rows from part-local to global ids, in place.
void remap_rows(Part& p, const std::vector<int32_t>& uid, const std::vector<int32_t>& sid) {
  for (size_t i = 0; i < p.ru.size(); ++i) {
    p.ru[i] = uid[p.ru[i]];
    p.rs[i] = sid[p.rs[i]];
  }
}

int find_sorted(const std::vector<sv>& sorted, sv s) {
  auto it = std::lower_bound(sorted.begin(), sorted.end(), s);
  return it != sorted.end() && *it == s ? (int)(it - sorted.begin()) : -1;
}

}  // namespace

extern "C" {

int mr_corpus_from_tsv(const char* train_path, const char* test_path, const char* labels_path,
                       mr_corpus** out) {
  if (!train_path || !test_path || !out) return mr_host::fail(MR_E_INVALID, "null argument");
  *out = nullptr;
  Trace trace("MR_INGEST_TRACE", "ingest");
  Text tr_text, te_text, lab_text;
  std::vector<Part> tr, te, lab;
  int rc;
  if ((rc = read_file(train_path, tr_text))) return rc;
  trace("read");
  if ((rc = parse_file(train_path, tr_text, tr))) return rc;
  trace("parse");
  if ((rc = read_file(test_path, te_text)) || (rc = parse_file(test_path, te_text, te))) return rc;
  if (labels_path && ((rc = read_file(labels_path, lab_text)) || (rc = parse_file(labels_path, lab_text, lab))))
    return rc;
  trace("test+lab");

  // songs = distinct songs of train ∪ test (MR:38, MR:51, MR:58); users per file
  std::vector<const std::vector<sv>*> song_parts;
  for (auto& p : tr) song_parts.push_back(&p.song_names);
  for (auto& p : te) song_parts.push_back(&p.song_names);
  Interned songs, trainU, testU;
  {
    std::thread a([&] { trainU = intern(user_names(tr)); });
    testU = intern(user_names(te));
    songs = intern(song_parts);
    a.join();
  }
  trace("intern");
  // train and test users must be disjoint (dataExtraction.ipynb:149,301)
  for (const sv& u : testU.names)
    if (find_sorted(trainU.names, u) >= 0)
      return mr_host::fail(MR_E_INVALID, "user %s is in both the train and the test file", std::string(u).c_str());

  auto* c = new mr_corpus();
  const int n_s = (int)songs.names.size(), n_tr = (int)trainU.names.size(), n_te = (int)testU.names.size();
  c->n_songs = n_s;
  const size_t np_tr = tr.size(), np_te = te.size();
  mr_par::parallel_dynamic((int64_t)(np_tr + np_te), 1, [&](int64_t i, int) {
    if ((size_t)i < np_tr) remap_rows(tr[i], trainU.id[i], songs.id[i]);
    else remap_rows(te[i - np_tr], testU.id[i - np_tr], songs.id[i]);
  });
  // c(s) = songsToUsersMap(s).length: train AND test lines, duplicates counted (MR:41, MR:60-62)
  {
    const int P = (int)(np_tr + np_te);
    std::vector<std::vector<int32_t>> hist(P);
    mr_par::parallel_dynamic(P, 1, [&](int64_t i, int) {
      const Part& p = (size_t)i < np_tr ? tr[i] : te[i - np_tr];
      hist[i].assign(n_s, 0);
      for (int32_t s : p.rs) hist[i][s]++;
    });
    c->song_count.assign(n_s, 0);
    mr_par::parallel_for(n_s, [&](int64_t lo, int64_t hi, int) {
      for (int i = 0; i < P; ++i)
        for (int64_t s = lo; s < hi; ++s) c->song_count[s] += hist[i][s];
    }, 4096);
  }
  trace("remap+c(s)");
  std::vector<Rows> tr_rows, te_rows;
  for (auto& p : tr) tr_rows.push_back({&p.ru, &p.rs});
  for (auto& p : te) te_rows.push_back({&p.ru, &p.rs});
  build_csr(n_tr, tr_rows, c->tr_off, c->tr_songs, &c->tr_len);
  build_csr(n_te, te_rows, c->te_off, c->te_songs, &c->te_len);
  for (auto& p : tr) { std::vector<int32_t>().swap(p.ru); std::vector<int32_t>().swap(p.rs); }
  trace("csr");

  // Labels (importTestLabels, MR:70-91): newSongs = distinct label songs; label
  // songs outside `songs` are numbered after them lexicographically. Rows of
  // users that are not test users are never looked up (MR:545) but their songs
  // still count as label songs.
  std::vector<sv> lab_distinct, extra;
  std::vector<std::vector<int32_t>> lu(lab.size()), ls(lab.size());  // per part: local -> id (-1 = none)
  mr_par::parallel_dynamic((int64_t)lab.size(), 1, [&](int64_t p, int) {
    const auto& un = lab[p].user_names;
    const auto& snm = lab[p].song_names;
    lu[p].resize(un.size());
    ls[p].resize(snm.size());
    for (size_t i = 0; i < un.size(); ++i) lu[p][i] = find_sorted(testU.names, un[i]);
    for (size_t i = 0; i < snm.size(); ++i) ls[p][i] = find_sorted(songs.names, snm[i]);
  });
  for (size_t p = 0; p < lab.size(); ++p)
    for (size_t i = 0; i < lab[p].song_names.size(); ++i) {
      lab_distinct.push_back(lab[p].song_names[i]);
      if (ls[p][i] < 0) extra.push_back(lab[p].song_names[i]);
    }
  std::sort(lab_distinct.begin(), lab_distinct.end());
  c->n_label_songs = (int)(std::unique(lab_distinct.begin(), lab_distinct.end()) - lab_distinct.begin());
  std::sort(extra.begin(), extra.end());
  extra.erase(std::unique(extra.begin(), extra.end()), extra.end());
  c->n_extra = (int)extra.size();
  std::vector<std::vector<int32_t>> lab_u(lab.size()), lab_s(lab.size());
  std::vector<Rows> lab_rows;
  for (size_t p = 0; p < lab.size(); ++p) {
    for (size_t i = 0; i < lab[p].ru.size(); ++i) {
      const int u = lu[p][lab[p].ru[i]];
      if (u < 0) continue;
      int s = ls[p][lab[p].rs[i]];
      if (s < 0) s = n_s + find_sorted(extra, lab[p].song_names[lab[p].rs[i]]);
      lab_u[p].push_back(u);
      lab_s[p].push_back(s);
    }
    lab_rows.push_back({&lab_u[p], &lab_s[p]});
  }
  build_csr(n_te, lab_rows, c->lab_off, c->lab_songs, nullptr);

  c->song_names.append_sorted(songs.names);
  c->song_names.append_sorted(extra);
  c->train_names.append_sorted(trainU.names);
  c->test_names.append_sorted(testU.names);
  trace("labels+names");
  *out = c;
  return MR_OK;
}

int mr_corpus_dataset(const mr_corpus* c, mr_dataset* d) {
  if (!c || !d) return mr_host::fail(MR_E_INVALID, "null argument");
  std::memset(d, 0, sizeof *d);
  d->n_train_users = (int32_t)c->train_names.size();
  d->n_test_users = (int32_t)c->test_names.size();
  d->n_songs = c->n_songs;
  d->tr_off = c->tr_off.data();
  d->tr_songs = c->tr_songs.data();
  d->te_off = c->te_off.data();
  d->te_songs = c->te_songs.data();
  d->song_count = c->song_count.data();
  d->tr_len = c->tr_len.data();
  d->te_len = c->te_len.data();
  return MR_OK;
}

int mr_corpus_labels(const mr_corpus* c, const int64_t** off, const int32_t** songs, int32_t* n_label_songs,
                     int32_t* n_extra_songs) {
  if (!c) return mr_host::fail(MR_E_INVALID, "null corpus");
  if (off) *off = c->lab_off.data();
  if (songs) *songs = c->lab_songs.data();
  if (n_label_songs) *n_label_songs = c->n_label_songs;
  if (n_extra_songs) *n_extra_songs = c->n_extra;
  return MR_OK;
}

static const NameBlob* blob_of(const mr_corpus* c, int32_t kind) {
  return kind == 0 ? &c->song_names : kind == 1 ? &c->train_names : kind == 2 ? &c->test_names : nullptr;
}

const char* mr_corpus_name(const mr_corpus* c, int32_t kind, int32_t id) {
  if (!c || id < 0) return nullptr;
  const NameBlob* v = blob_of(c, kind);
  if (!v || (size_t)id >= v->size()) return nullptr;
  return v->get((size_t)id);
}

int mr_corpus_names(const mr_corpus* c, int32_t kind, char* buf, int64_t buf_size, int64_t* bytes_needed) {
  if (!c || !bytes_needed) return mr_host::fail(MR_E_INVALID, "null argument");
  const NameBlob* v = blob_of(c, kind);
  if (!v) return mr_host::fail(MR_E_INVALID, "bad name kind %d", kind);
  const int64_t total = (int64_t)v->bytes.size();  // every name + its terminator
  *bytes_needed = total;
  if (!buf) return MR_OK;
  if (buf_size < total) return mr_host::fail(MR_E_INVALID, "name buffer of %lld B, %lld needed", (long long)buf_size, (long long)total);
  if (total) std::memcpy(buf, v->bytes.data(), (size_t)total);
  for (size_t i = 0; i < v->size(); ++i) buf[v->at[i + 1] - 1] = '\n';  // NUL terminators -> newlines
  return MR_OK;
}

int mr_corpus_free(mr_corpus* c) {
  delete c;
  return MR_OK;
}

int mr_topk_merge_host(int32_t n_shards, int32_t n_te, int32_t k, const int32_t* songs_in, const int64_t* keys_in,
                       const double* /*scores_in*/, int32_t* songs_out, int64_t* keys_out, double* scores_out) {
  if (!songs_in || !keys_in || !songs_out || !keys_out) return mr_host::fail(MR_E_INVALID, "null argument");
  if (n_shards <= 0 || n_te < 0 || k <= 0) return mr_host::fail(MR_E_INVALID, "bad merge shape");
  std::vector<std::pair<int64_t, int32_t>> cand;
  for (int u = 0; u < n_te; ++u) {
    cand.clear();
    for (int g = 0; g < n_shards; ++g)
      for (int r = 0; r < k; ++r) {
        const size_t i = ((size_t)g * n_te + u) * k + r;
        if (keys_in[i] >= 0) cand.emplace_back(keys_in[i], songs_in[i]);
      }
    std::sort(cand.begin(), cand.end(), [](const std::pair<int64_t, int32_t>& a, const std::pair<int64_t, int32_t>& b) {
      return a.first > b.first || (a.first == b.first && a.second < b.second);
    });
    for (int r = 0; r < k; ++r) {
      const size_t o = (size_t)u * k + r;
      if (r < (int)cand.size()) {
        keys_out[o] = cand[r].first;
        songs_out[o] = cand[r].second;
        if (scores_out) {
          double d;
          std::memcpy(&d, &cand[r].first, 8);
          scores_out[o] = d;
        }
      } else {
        keys_out[o] = -1;
        songs_out[o] = -1;
        if (scores_out) scores_out[o] = NAN;
      }
    }
  }
  return MR_OK;
}

int mr_eval_map(int32_t n_classes, const int32_t* pred, const int32_t* tp, const int32_t* pos,
                int32_t n_label_songs, double* map_out, int32_t n_thresholds) {
  if (!pred || !tp || !pos || !map_out || n_classes < 0) return mr_host::fail(MR_E_INVALID, "bad argument");
  const int T = n_thresholds == 0 ? 10 : n_thresholds;  // 10: MR:590; 11: distributed.scala:395
  if (T != 10 && T != 11) return mr_host::fail(MR_E_INVALID, "%d thresholds: 10 or 11", n_thresholds);
  double total = 0.0;
  for (int g = 0; g < n_classes; ++g) {
    if (pos[g] <= 0) continue;  // AP = 0 for classes nobody holds
    double P[11], R[11];
    for (int t = 0; t < T; ++t) {
      const size_t i = (size_t)g * T + t;
      P[t] = pred[i] > 0 ? (double)tp[i] / (double)pred[i] : 0.0;  // precision, MR:563-568
      R[t] = (double)tp[i] / (double)pos[g];                        // recall, MR:576-581
    }
    double ap = 0.0;  // MR:601-609 / distributed.scala:405-413, summed left to right
    for (int t = 0; t < T; ++t) {
      const double term = t == T - 1 ? 0.0 : t == T - 2 ? (R[t] - 0.0) * P[t] : (R[t] - R[t + 1]) * P[t];
      ap = ap + term;
    }
    total += ap;
  }
  *map_out = n_label_songs > 0 ? total / (double)n_label_songs : NAN;
  return MR_OK;
}

}  // extern "C"
