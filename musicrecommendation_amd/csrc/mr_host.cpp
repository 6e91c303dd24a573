// mr_host.cpp — host-side part of the engine's C ABI (no GPU needed):
//  * parallel TSV ingest + string interning + CSR build, replacing extractData /
//    songs / songsToUsersMap / importTestLabels (MusicRecommender.scala MR:26-91);
//  * the per-shard top-k merge on the host (exchange step of a song-sharded run).
#include <algorithm>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <string>
#include <string_view>
#include <thread>
#include <unordered_map>
#include <vector>

#include "mr_engine.h"

namespace mr_host {
// Error slot shared with the device part through these two functions
// (mr_last_error lives in mr_engine.hip).
int fail(int code, const char* fmt, ...);
}  // namespace mr_host

namespace {

// ---- parallel TSV reader -------------------------------------------------------
// The whole file is read into memory and cut into per-thread chunks at line
// starts; every thread splits its lines (Java String.split("\t") semantics:
// trailing empty fields dropped, then exactly 3 fields, MR:34-35) into string
// views and interns user / song names in thread-local tables. The tables are
// merged afterwards (distinct names only), so the hot loop touches no shared
// state.
using sv = std::string_view;

int read_file(const char* path, std::vector<char>& out) {
  FILE* f = std::fopen(path, "rb");
  if (!f) return mr_host::fail(MR_E_IO, "cannot open %s", path);
  std::fseek(f, 0, SEEK_END);
  const long n = std::ftell(f);
  std::fseek(f, 0, SEEK_SET);
  if (n < 0) { std::fclose(f); return mr_host::fail(MR_E_IO, "cannot size %s", path); }
  out.resize((size_t)n);
  const size_t got = n ? std::fread(out.data(), 1, (size_t)n, f) : 0;
  std::fclose(f);
  if (got != (size_t)n) return mr_host::fail(MR_E_IO, "short read of %s", path);
  return MR_OK;
}

struct Local {  // one thread's share of one file
  std::unordered_map<sv, int> uid, sid;
  std::vector<sv> unames, snames;
  std::vector<int> ru, rs;
  size_t err_off = SIZE_MAX;
  int err_fields = 0;
};

void parse_chunk(const char* p, size_t a, size_t b, Local& c) {
  size_t i = a;
  while (i < b) {
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
    if (last_ne + 1 != 3) {  // scala.MatchError (MR:34)
      c.err_off = i;
      c.err_fields = last_ne + 1;
      return;
    }
    auto u = c.uid.try_emplace(f0, (int)c.unames.size());
    if (u.second) c.unames.push_back(f0);
    auto so = c.sid.try_emplace(f1, (int)c.snames.size());
    if (so.second) c.snames.push_back(f1);
    c.ru.push_back(u.first->second);
    c.rs.push_back(so.first->second);
    i = nl ? end + 1 : b;
  }
}

int n_threads() {
  const char* e = std::getenv("MR_INGEST_THREADS");
  int t = e ? std::atoi(e) : (int)std::thread::hardware_concurrency();
  return std::max(1, std::min(t, 32));
}

int parse_file(const char* path, const std::vector<char>& text, std::vector<Local>& parts) {
  const size_t n = text.size();
  // chunks of >= 1 MiB (MR_INGEST_MIN_CHUNK overrides, e.g. to split small files in tests)
  const char* mc = std::getenv("MR_INGEST_MIN_CHUNK");
  const size_t min_chunk = mc ? std::max<size_t>(1, (size_t)std::atoll(mc)) : ((size_t)1 << 20);
  const int T = (int)std::max<size_t>(1, std::min<size_t>((size_t)n_threads(), n / min_chunk + 1));
  std::vector<size_t> cut(T + 1, n);
  cut[0] = 0;
  for (int t = 1; t < T; ++t) {
    size_t x = std::max(cut[t - 1], n * t / T);
    while (x < n && x > 0 && text[x - 1] != '\n') ++x;
    cut[t] = x;
  }
  parts.assign(T, Local());
  std::vector<std::thread> th;
  for (int t = 0; t < T; ++t) {
    parts[t].ru.reserve((cut[t + 1] - cut[t]) / 48 + 16);
    parts[t].rs.reserve((cut[t + 1] - cut[t]) / 48 + 16);
    th.emplace_back(parse_chunk, text.data(), cut[t], cut[t + 1], std::ref(parts[t]));
  }
  for (auto& x : th) x.join();
  size_t bad = SIZE_MAX;
  int fields = 0;
  for (auto& c : parts)
    if (c.err_off < bad) { bad = c.err_off; fields = c.err_fields; }
  if (bad != SIZE_MAX) {
    const size_t lineno = 1 + (size_t)std::count(text.begin(), text.begin() + (long)bad, '\n');
    return mr_host::fail(MR_E_PARSE, "%s:%zu: expected 3 tab-separated fields, got %d", path, lineno, fields);
  }
  return MR_OK;
}

struct Table {
  // interning in first-seen order, re-numbered lexicographically at the end
  std::unordered_map<sv, int> id;
  std::vector<sv> names;
  int get(sv s) {
    auto it = id.try_emplace(s, (int)names.size());
    if (it.second) names.push_back(s);
    return it.first->second;
  }
  // old id -> new lexicographic id
  std::vector<int> lex_order() const {
    std::vector<int> idx(names.size());
    for (size_t i = 0; i < idx.size(); ++i) idx[i] = (int)i;
    std::sort(idx.begin(), idx.end(), [&](int a, int b) { return names[a] < names[b]; });
    std::vector<int> remap(names.size());
    for (size_t r = 0; r < idx.size(); ++r) remap[idx[r]] = (int)r;
    return remap;
  }
};

struct Row {
  int user;
  int song;
};

// Merge the per-thread tables of one file into the global user / song tables
// and append its rows (global first-seen ids).
void merge_parts(std::vector<Local>& parts, Table& users, Table& songs, std::vector<Row>& rows) {
  size_t total = 0;
  for (auto& c : parts) total += c.ru.size();
  rows.reserve(rows.size() + total);
  for (auto& c : parts) {
    std::vector<int> ug(c.unames.size()), sg(c.snames.size());
    for (size_t i = 0; i < ug.size(); ++i) ug[i] = users.get(c.unames[i]);
    for (size_t i = 0; i < sg.size(); ++i) sg[i] = songs.get(c.snames[i]);
    for (size_t r = 0; r < c.ru.size(); ++r) rows.push_back({ug[c.ru[r]], sg[c.rs[r]]});
    std::vector<int>().swap(c.ru);
    std::vector<int>().swap(c.rs);
  }
}

}  // namespace

struct mr_corpus {
  std::vector<std::string> song_names;   // n_songs + n_extra (label-only songs last)
  std::vector<std::string> train_names, test_names;
  int n_songs = 0, n_extra = 0, n_label_songs = 0;
  std::vector<int64_t> tr_off, te_off, lab_off;
  std::vector<int32_t> tr_songs, te_songs, lab_songs;
  std::vector<int32_t> song_count, tr_len, te_len;
};

namespace {

// Build CSR rows (sorted unique) + duplicate-counting lengths: counting sort
// by user, then sort + unique inside each row.
void build_rows(int n_users, const std::vector<Row>& rows, std::vector<int64_t>& off,
                std::vector<int32_t>& col, std::vector<int32_t>* len) {
  std::vector<int64_t> start((size_t)n_users + 1, 0);
  for (const Row& r : rows) start[(size_t)r.user + 1]++;
  for (int u = 0; u < n_users; ++u) start[u + 1] += start[u];
  std::vector<int32_t> tmp(rows.size());
  {
    std::vector<int64_t> cur(start.begin(), start.end() - 1);
    for (const Row& r : rows) tmp[cur[r.user]++] = r.song;
  }
  off.assign((size_t)n_users + 1, 0);
  if (len) len->assign(n_users, 0);
  col.clear();
  col.reserve(rows.size());
  for (int u = 0; u < n_users; ++u) {
    auto b = tmp.begin() + start[u], e = tmp.begin() + start[u + 1];
    if (len) (*len)[u] = (int32_t)(e - b);
    std::sort(b, e);
    col.insert(col.end(), b, std::unique(b, e));
    off[u + 1] = (int64_t)col.size();
  }
}

}  // namespace

extern "C" {

int mr_corpus_from_tsv(const char* train_path, const char* test_path, const char* labels_path,
                       mr_corpus** out) {
  if (!train_path || !test_path || !out) return mr_host::fail(MR_E_INVALID, "null argument");
  *out = nullptr;
  std::vector<char> tr_text, te_text, lab_text;
  std::vector<Local> tr, te, lab;
  int rc;
  if ((rc = read_file(train_path, tr_text)) || (rc = parse_file(train_path, tr_text, tr))) return rc;
  if ((rc = read_file(test_path, te_text)) || (rc = parse_file(test_path, te_text, te))) return rc;
  if (labels_path && ((rc = read_file(labels_path, lab_text)) || (rc = parse_file(labels_path, lab_text, lab))))
    return rc;

  Table songs, trainU, testU;
  std::vector<Row> tr_rows, te_rows;
  merge_parts(tr, trainU, songs, tr_rows);
  merge_parts(te, testU, songs, te_rows);
  for (auto& kv : testU.id)
    if (trainU.id.count(kv.first))
      return mr_host::fail(MR_E_INVALID, "user %s is in both the train and the test file",
                           std::string(kv.first).c_str());

  auto* c = new mr_corpus();
  const std::vector<int> srm = songs.lex_order(), trm = trainU.lex_order(), term = testU.lex_order();
  c->n_songs = (int)songs.names.size();
  c->song_names.resize(c->n_songs);
  for (size_t i = 0; i < srm.size(); ++i) c->song_names[srm[i]] = std::string(songs.names[i]);
  c->train_names.resize(trm.size());
  for (size_t i = 0; i < trm.size(); ++i) c->train_names[trm[i]] = std::string(trainU.names[i]);
  c->test_names.resize(term.size());
  for (size_t i = 0; i < term.size(); ++i) c->test_names[term[i]] = std::string(testU.names[i]);
  c->song_count.assign(c->n_songs, 0);
  for (auto& r : tr_rows) { r.user = trm[r.user]; r.song = srm[r.song]; c->song_count[r.song]++; }
  for (auto& r : te_rows) { r.user = term[r.user]; r.song = srm[r.song]; c->song_count[r.song]++; }
  build_rows((int)c->train_names.size(), tr_rows, c->tr_off, c->tr_songs, &c->tr_len);
  build_rows((int)c->test_names.size(), te_rows, c->te_off, c->te_songs, &c->te_len);

  // Labels (importTestLabels, MR:70-91): newSongs = distinct label songs,
  // label songs outside `songs` are numbered after them lexicographically.
  Table extra;
  std::vector<Row> lab_rows;
  std::unordered_map<sv, int> label_song_set;
  std::vector<std::pair<int, sv>> pending;  // (test user, extra song name)
  for (auto& part : lab)
    for (size_t r = 0; r < part.ru.size(); ++r) {
      const sv un = part.unames[part.ru[r]], sn = part.snames[part.rs[r]];
      label_song_set.emplace(sn, 1);
      auto tu = testU.id.find(un);
      auto si = songs.id.find(sn);
      if (si == songs.id.end()) extra.get(sn);
      if (tu == testU.id.end()) continue;  // never looked up by the reference (MR:545)
      if (si != songs.id.end()) lab_rows.push_back({term[tu->second], srm[si->second]});
      else pending.emplace_back(term[tu->second], sn);
    }
  const std::vector<int> erm = extra.lex_order();
  c->n_extra = (int)extra.names.size();
  c->song_names.resize(c->n_songs + c->n_extra);
  for (size_t i = 0; i < erm.size(); ++i) c->song_names[c->n_songs + erm[i]] = std::string(extra.names[i]);
  for (auto& pr : pending) lab_rows.push_back({pr.first, c->n_songs + erm[extra.id[pr.second]]});
  c->n_label_songs = (int)label_song_set.size();
  build_rows((int)c->test_names.size(), lab_rows, c->lab_off, c->lab_songs, nullptr);
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

const char* mr_corpus_name(const mr_corpus* c, int32_t kind, int32_t id) {
  if (!c || id < 0) return nullptr;
  const std::vector<std::string>* v =
      kind == 0 ? &c->song_names : kind == 1 ? &c->train_names : kind == 2 ? &c->test_names : nullptr;
  if (!v || (size_t)id >= v->size()) return nullptr;
  return (*v)[id].c_str();
}

int mr_corpus_names(const mr_corpus* c, int32_t kind, char* buf, int64_t buf_size, int64_t* bytes_needed) {
  if (!c || !bytes_needed) return mr_host::fail(MR_E_INVALID, "null argument");
  const std::vector<std::string>* v =
      kind == 0 ? &c->song_names : kind == 1 ? &c->train_names : kind == 2 ? &c->test_names : nullptr;
  if (!v) return mr_host::fail(MR_E_INVALID, "bad name kind %d", kind);
  int64_t total = 0;
  for (const auto& s : *v) total += (int64_t)s.size() + 1;
  *bytes_needed = total;
  if (!buf) return MR_OK;
  if (buf_size < total) return mr_host::fail(MR_E_INVALID, "name buffer of %lld B, %lld needed", (long long)buf_size, (long long)total);
  char* o = buf;
  for (const auto& s : *v) {
    std::memcpy(o, s.data(), s.size());
    o += s.size();
    *o++ = '\n';
  }
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
                int32_t n_label_songs, double* map_out) {
  if (!pred || !tp || !pos || !map_out || n_classes < 0) return mr_host::fail(MR_E_INVALID, "bad argument");
  double total = 0.0;
  for (int g = 0; g < n_classes; ++g) {
    if (pos[g] <= 0) continue;  // AP = 0 for classes nobody holds
    double P[10], R[10];
    for (int t = 0; t < 10; ++t) {
      const size_t i = (size_t)g * 10 + t;
      P[t] = pred[i] > 0 ? (double)tp[i] / (double)pred[i] : 0.0;  // precision, MR:563-568
      R[t] = (double)tp[i] / (double)pos[g];                        // recall, MR:576-581
    }
    double ap = 0.0;  // MR:601-609, summed left to right
    for (int t = 0; t < 10; ++t) {
      const double term = t == 9 ? 0.0 : t == 8 ? (R[8] - 0.0) * P[8] : (R[t] - R[t + 1]) * P[t];
      ap = ap + term;
    }
    total += ap;
  }
  *map_out = n_label_songs > 0 ? total / (double)n_label_songs : NAN;
  return MR_OK;
}

}  // extern "C"
