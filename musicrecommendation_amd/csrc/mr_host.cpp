// mr_host.cpp — host-side part of the engine's C ABI (no GPU needed):
//  * TSV ingest + string interning + CSR build, replacing extractData /
//    songs / songsToUsersMap / importTestLabels (MusicRecommender.scala MR:26-91);
//  * the per-shard top-k merge on the host (exchange step of a song-sharded run).
#include <algorithm>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <string>
#include <unordered_map>
#include <vector>

#include "mr_engine.h"

namespace mr_host {
// Error slot shared with the device part through these two functions
// (mr_last_error lives in mr_engine.hip).
int fail(int code, const char* fmt, ...);
}  // namespace mr_host

namespace {

struct Table {
  // interning in first-seen order, re-numbered lexicographically at the end
  std::unordered_map<std::string, int> id;
  std::vector<std::string> names;
  int get(const std::string& s) {
    auto it = id.find(s);
    if (it != id.end()) return it->second;
    int k = (int)names.size();
    id.emplace(s, k);
    names.push_back(s);
    return k;
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

// Split like Java's String.split("\t"): trailing empty fields are dropped;
// the reference then pattern-matches exactly three fields (MR:34-35).
int parse_file(const char* path, std::vector<std::pair<std::string, std::string>>& out) {
  std::ifstream in(path, std::ios::binary);
  if (!in) return mr_host::fail(MR_E_IO, "cannot open %s", path);
  std::string line;
  size_t lineno = 0;
  std::vector<std::string> f;
  while (std::getline(in, line)) {
    ++lineno;
    if (!line.empty() && line.back() == '\r') line.pop_back();  // getLines strips \r\n
    f.clear();
    size_t a = 0;
    while (true) {
      size_t b = line.find('\t', a);
      if (b == std::string::npos) { f.emplace_back(line.substr(a)); break; }
      f.emplace_back(line.substr(a, b - a));
      a = b + 1;
    }
    while (!f.empty() && f.back().empty()) f.pop_back();
    if (f.size() != 3)
      return mr_host::fail(MR_E_PARSE, "%s:%zu: expected 3 tab-separated fields, got %zu", path, lineno, f.size());
    out.emplace_back(std::move(f[0]), std::move(f[1]));
  }
  return MR_OK;
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

// Build CSR rows (sorted unique) + duplicate-counting lengths.
void build_rows(int n_users, const std::vector<Row>& rows, std::vector<int64_t>& off,
                std::vector<int32_t>& col, std::vector<int32_t>* len) {
  std::vector<std::vector<int32_t>> per(n_users);
  for (const Row& r : rows) per[r.user].push_back(r.song);
  off.assign(n_users + 1, 0);
  if (len) len->assign(n_users, 0);
  col.clear();
  for (int u = 0; u < n_users; ++u) {
    auto& v = per[u];
    if (len) (*len)[u] = (int32_t)v.size();
    std::sort(v.begin(), v.end());
    v.erase(std::unique(v.begin(), v.end()), v.end());
    col.insert(col.end(), v.begin(), v.end());
    off[u + 1] = (int64_t)col.size();
  }
}

}  // namespace

extern "C" {

int mr_corpus_from_tsv(const char* train_path, const char* test_path, const char* labels_path,
                       mr_corpus** out) {
  if (!train_path || !test_path || !out) return mr_host::fail(MR_E_INVALID, "null argument");
  *out = nullptr;
  std::vector<std::pair<std::string, std::string>> tr, te, lab;
  int rc;
  if ((rc = parse_file(train_path, tr))) return rc;
  if ((rc = parse_file(test_path, te))) return rc;
  if (labels_path && (rc = parse_file(labels_path, lab))) return rc;

  Table songs, trainU, testU;
  std::vector<Row> tr_rows, te_rows;
  tr_rows.reserve(tr.size());
  te_rows.reserve(te.size());
  for (auto& l : tr) tr_rows.push_back({trainU.get(l.first), songs.get(l.second)});
  for (auto& l : te) te_rows.push_back({testU.get(l.first), songs.get(l.second)});
  for (auto& kv : testU.id)
    if (trainU.id.count(kv.first))
      return mr_host::fail(MR_E_INVALID, "user %s is in both the train and the test file", kv.first.c_str());

  auto* c = new mr_corpus();
  const std::vector<int> srm = songs.lex_order(), trm = trainU.lex_order(), term = testU.lex_order();
  c->n_songs = (int)songs.names.size();
  c->song_names.resize(c->n_songs);
  for (size_t i = 0; i < srm.size(); ++i) c->song_names[srm[i]] = songs.names[i];
  c->train_names.resize(trm.size());
  for (size_t i = 0; i < trm.size(); ++i) c->train_names[trm[i]] = trainU.names[i];
  c->test_names.resize(term.size());
  for (size_t i = 0; i < term.size(); ++i) c->test_names[term[i]] = testU.names[i];
  c->song_count.assign(c->n_songs, 0);
  for (auto& r : tr_rows) { r.user = trm[r.user]; r.song = srm[r.song]; c->song_count[r.song]++; }
  for (auto& r : te_rows) { r.user = term[r.user]; r.song = srm[r.song]; c->song_count[r.song]++; }
  build_rows((int)c->train_names.size(), tr_rows, c->tr_off, c->tr_songs, &c->tr_len);
  build_rows((int)c->test_names.size(), te_rows, c->te_off, c->te_songs, &c->te_len);

  // Labels (importTestLabels, MR:70-91): newSongs = distinct label songs,
  // label songs outside `songs` are numbered after them lexicographically.
  Table extra;
  std::vector<Row> lab_rows;
  std::unordered_map<std::string, int> label_song_set;
  std::unordered_map<std::string, int> song_id;
  song_id.reserve(c->song_names.size());
  for (int s = 0; s < c->n_songs; ++s) song_id.emplace(c->song_names[s], s);
  std::vector<std::pair<int, std::string>> pending;  // (test user, extra song name)
  for (auto& l : lab) {
    label_song_set.emplace(l.second, 1);
    auto tu = testU.id.find(l.first);
    auto si = song_id.find(l.second);
    if (si == song_id.end()) extra.get(l.second);
    if (tu == testU.id.end()) continue;  // never looked up by the reference (MR:545)
    if (si != song_id.end()) lab_rows.push_back({term[tu->second], si->second});
    else pending.emplace_back(term[tu->second], l.second);
  }
  const std::vector<int> erm = extra.lex_order();
  c->n_extra = (int)extra.names.size();
  c->song_names.resize(c->n_songs + c->n_extra);
  for (size_t i = 0; i < erm.size(); ++i) c->song_names[c->n_songs + erm[i]] = extra.names[i];
  for (auto& p : pending) lab_rows.push_back({p.first, c->n_songs + erm[extra.id[p.second]]});
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
