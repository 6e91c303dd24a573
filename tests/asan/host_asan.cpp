// tests/asan/host_asan.cpp — TEST HARNESS: the engine's host-only C++ (TSV
// ingest mr_host.cpp, model files mr_modelio.cpp) built with
// -fsanitize=address,undefined by g++ and driven through its C ABI on the
// fixtures, malformed input and forced multi-chunk parses. Exit 0 = clean.
// Usage: host_asan TRAIN TEST LABELS BADFILE TMPDIR
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <vector>

#include "mr_engine.h"

namespace mr_host {
static std::string last;
int fail(int code, const char* fmt, ...) {  // the engine library's error slot, stubbed
  char buf[1024];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  last = buf;
  return code;
}
}  // namespace mr_host

static int failures = 0;
#define CHECK(c)                                                  \
  do {                                                            \
    if (!(c)) {                                                   \
      ++failures;                                                 \
      std::fprintf(stderr, "FAIL %s:%d: %s\n", __FILE__, __LINE__, #c); \
    }                                                             \
  } while (0)

int main(int argc, char** argv) {
  if (argc < 6) return 2;
  const std::string tmp = argv[5];
  for (const char* chunk : {"0", "64"}) {  // default chunking, then tiny chunks (many threads)
    if (std::strcmp(chunk, "0")) setenv("MR_INGEST_MIN_CHUNK", chunk, 1);
    mr_corpus* c = nullptr;
    CHECK(mr_corpus_from_tsv(argv[1], argv[2], argv[3], &c) == MR_OK);
    if (!c) return 1;
    mr_dataset d;
    CHECK(mr_corpus_dataset(c, &d) == MR_OK);
    CHECK(d.n_train_users > 0 && d.n_test_users > 0 && d.n_songs > 0);
    const int64_t* lo;
    const int32_t* ls;
    int32_t nl = 0, nx = 0;
    CHECK(mr_corpus_labels(c, &lo, &ls, &nl, &nx) == MR_OK);
    // model files: write the dense model of made-up scores, read it back
    std::vector<const char*> un(d.n_test_users), sn(d.n_songs);
    for (int u = 0; u < d.n_test_users; ++u) un[u] = mr_corpus_name(c, 2, u);
    for (int s = 0; s < d.n_songs; ++s) sn[s] = mr_corpus_name(c, 0, s);
    std::vector<double> dense((size_t)d.n_test_users * d.n_songs), back(dense.size());
    std::mt19937_64 rng(7);
    for (size_t i = 0; i < dense.size(); ++i)
      dense[i] = (rng() % 5 == 0) ? NAN : std::ldexp((double)(rng() >> 11), -53 + (int)(rng() % 20));
    const std::string path = tmp + "/model.txt";
    for (int order = 0; order < 2; ++order) {
      CHECK(mr_model_write_tsv(path.c_str(), d.n_test_users, d.n_songs, un.data(), sn.data(), dense.data(), order) ==
            MR_OK);
      CHECK(mr_model_read_tsv(path.c_str(), d.n_test_users, d.n_songs, un.data(), sn.data(), back.data()) == MR_OK);
      for (size_t i = 0; i < dense.size(); ++i)
        CHECK((std::isnan(dense[i]) && std::isnan(back[i])) || dense[i] == back[i]);
    }
    CHECK(mr_corpus_free(c) == MR_OK);
  }
  unsetenv("MR_INGEST_MIN_CHUNK");
  mr_corpus* bad = nullptr;
  CHECK(mr_corpus_from_tsv(argv[4], argv[2], nullptr, &bad) == MR_E_PARSE && !bad);
  CHECK(mr_corpus_from_tsv("/nonexistent/x.txt", argv[2], nullptr, &bad) == MR_E_IO && !bad);
  char buf[64];
  std::mt19937_64 rng(3);
  for (int i = 0; i < 20000; ++i) {
    uint64_t bits = rng();
    double x;
    std::memcpy(&x, &bits, 8);
    const int n = mr_java_double_string(x, buf, sizeof buf);
    CHECK(n > 0 && n < (int)sizeof buf);
    if (std::isfinite(x)) CHECK(std::strtod(buf, nullptr) == x);
  }
  CHECK(mr_java_double_string(1.0, buf, 2) == MR_E_INVALID);
  // host merge + mAP fold on small arrays
  const int32_t s_in[2 * 1 * 3] = {5, 9, -1, 2, 7, 8};
  const int64_t k_in[2 * 1 * 3] = {100, 50, -1, 100, 60, 10};
  int32_t so[3];
  int64_t ko[3];
  double sc[3];
  CHECK(mr_topk_merge_host(2, 1, 3, s_in, k_in, nullptr, so, ko, sc) == MR_OK);
  CHECK(so[0] == 2 && so[1] == 5 && so[2] == 7);
  const int32_t pred[2 * 10] = {3, 3, 2, 2, 1, 1, 1, 0, 0, 0, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1};
  const int32_t tp[2 * 10] = {1, 1, 1, 1, 1, 1, 1, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
  const int32_t pos[2] = {1, 2};
  double map = -1;
  CHECK(mr_eval_map(2, pred, tp, pos, 3, &map, 10) == MR_OK && map >= 0 && map <= 1);
  const int32_t pred11[2 * 11] = {3, 3, 2, 2, 1, 1, 1, 0, 0, 0, 0, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 0};
  const int32_t tp11[2 * 11] = {1, 1, 1, 1, 1, 1, 1, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
  CHECK(mr_eval_map(2, pred11, tp11, pos, 3, &map, 11) == MR_OK && map >= 0 && map <= 1);
  CHECK(mr_eval_map(2, pred11, tp11, pos, 3, &map, 12) == MR_E_INVALID);
  std::printf("host asan: %s\n", failures ? "FAIL" : "ok");
  return failures ? 1 : 0;
}
