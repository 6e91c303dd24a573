/*
 * jni/test_shim.c — TEST HARNESS (plain C, gcc): the exact call sequences the
 * JNI shim makes, on the known-answer test of SURVEY.md §4.2, without a JDK.
 *
 *  1. always: error codes. A null options pointer, a null dataset, bad group
 *     layouts, Java array lengths that disagree with the sizes (ne_load checks
 *     them before the engine reads a byte), and — on a box without a GPU —
 *     mr_create / ne_create fail with a negative code and a message (never
 *     exit, never a CPU fallback).
 *  2. with a GPU: the single-context sequence
 *       mr_options_default -> mr_create -> mr_load -> mr_score_dense -> mr_destroy
 *     and the shim's group sequence (ne_create -> ne_load -> ne_score_dense /
 *     ne_topk -> ne_destroy, one context and 2 song shards x 2 user blocks),
 *     both BIT-identical to the fixed-point oracle (oracle/fixedpoint.c,
 *     test infrastructure) and within 1e-9 of the hand-derived KAT values
 *     (MusicRecommender.scala MR:140-166, MR:230-257).
 * Exit 0 = pass; prints "gpu: skipped" when no device is visible.
 *
 * KAT: train A:{s1,s2,s3} B:{s2,s3} C:{s3,s4}; test-visible X:{s1,s4} Y:{s2};
 * c = {s1:2, s2:3, s3:3, s4:2} (train + test listens, MR:60-62).
 */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include "nativeengine.h"

/* oracle/fixedpoint.c (liboracle.so) */
typedef struct fp_data {
  int32_t n_train, n_test, n_songs;
  const int64_t* tr_off; const int32_t* tr_songs;
  const int64_t* te_off; const int32_t* te_songs;
  const int32_t* song_count; const int32_t* tr_len; const int32_t* te_len;
} fp_data;
int fp_model(const fp_data* d, int model, int frac_bits, int32_t song_lo, int32_t song_hi, int32_t user_lo,
             int32_t user_hi, double* dense, int32_t k, int32_t* top_songs, int64_t* top_keys);

static int failures = 0;
#define CHECK(cond, ...)                                \
  do {                                                  \
    if (!(cond)) {                                      \
      ++failures;                                       \
      fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__); \
      fprintf(stderr, __VA_ARGS__);                     \
      fprintf(stderr, "\n");                            \
    }                                                   \
  } while (0)

/* ids: songs s1..s4 = 0..3, train A,B,C = 0..2, test X,Y = 0..1 */
static const int64_t TR_OFF[] = {0, 3, 5, 7};
static const int32_t TR_SONGS[] = {0, 1, 2, 1, 2, 2, 3};
static const int64_t TE_OFF[] = {0, 2, 3};
static const int32_t TE_SONGS[] = {0, 3, 1};
static const int32_t SONG_COUNT[] = {2, 3, 3, 2};
static const int32_t TR_LEN[] = {3, 2, 2};
static const int32_t TE_LEN[] = {2, 1};
enum { NTR = 3, NTE = 2, NS = 4 };
/* Java lengths of the load arrays (tr_off, tr_songs, te_off, te_songs, song_count, tr_len, te_len) */
static const int64_t LENS[7] = {NTR + 1, 7, NTE + 1, 3, NS, NTR, NTE};

/* SURVEY.md §4.2 (NaN = heard song, no pair) */
static const double KAT_IBM[NTE][NS] = {{NAN, 0.40824829046386296, 0.8164965809277259, NAN},
                                        {0.40824829046386296, NAN, 0.6666666666666667, 0.0}};
static const double KAT_UBM[NTE][NS] = {{NAN, 0.40824829046386296, 0.9082482904638629, NAN},
                                        {0.5773502691896258, NAN, 1.2844570503761732, 0.0}};

static mr_dataset kat(void) {
  mr_dataset d;
  memset(&d, 0, sizeof d);
  d.n_train_users = NTR; d.n_test_users = NTE; d.n_songs = NS;
  d.tr_off = TR_OFF; d.tr_songs = TR_SONGS; d.te_off = TE_OFF; d.te_songs = TE_SONGS;
  d.song_count = SONG_COUNT; d.tr_len = TR_LEN; d.te_len = TE_LEN;
  return d;
}

static int same_bits(double a, double b) {
  uint64_t x, y;
  memcpy(&x, &a, 8);
  memcpy(&y, &b, 8);
  return x == y || (isnan(a) && isnan(b));
}

static void check_dense(const char* what, int model, const double* got) {
  const fp_data fd = {NTR, NTE, NS, TR_OFF, TR_SONGS, TE_OFF, TE_SONGS, SONG_COUNT, TR_LEN, TE_LEN};
  double exp[NTE * NS];
  CHECK(fp_model(&fd, model, 32, 0, NS, 0, NTE, exp, 0, NULL, NULL) == 0, "oracle failed");
  const double(*kat_v)[NS] = model == MR_IBM ? KAT_IBM : KAT_UBM;
  for (int u = 0; u < NTE; ++u)
    for (int s = 0; s < NS; ++s) {
      const double g = got[u * NS + s], e = exp[u * NS + s], k = kat_v[u][s];
      CHECK(same_bits(g, e), "%s model %d (u=%d,s=%d): %.17g != oracle %.17g", what, model, u, s, g, e);
      CHECK(isnan(g) == isnan(k), "%s: heard-song mask differs at (%d,%d)", what, u, s);
      if (!isnan(k)) CHECK(fabs(g - k) <= 1e-9 * fabs(k), "%s (u=%d,s=%d): %.17g vs KAT %.17g", what, u, s, g, k);
    }
}

static void check_topk(const char* what, int model, int k, const int32_t* songs, const double* scores) {
  const fp_data fd = {NTR, NTE, NS, TR_OFF, TR_SONGS, TE_OFF, TE_SONGS, SONG_COUNT, TR_LEN, TE_LEN};
  int32_t ts[NTE * 8];
  int64_t tk[NTE * 8];
  CHECK(fp_model(&fd, model, 32, 0, NS, 0, NTE, NULL, k, ts, tk) == 0, "oracle failed");
  for (int i = 0; i < NTE * k; ++i) {
    CHECK(songs[i] == ts[i], "%s model %d top-k slot %d: song %d != oracle %d", what, model, i, songs[i], ts[i]);
    double e;
    memcpy(&e, &tk[i], 8);
    if (ts[i] >= 0) CHECK(same_bits(scores[i], e), "%s top-k score slot %d", what, i);
  }
}

static void error_codes(void) {
  CHECK(mr_options_default(NULL) == MR_E_INVALID, "mr_options_default(NULL)");
  CHECK(strlen(mr_last_error()) > 0, "empty error message");
  CHECK(mr_create(NULL, NULL) == MR_E_INVALID, "mr_create(NULL, NULL)");
  CHECK(mr_load(NULL, NULL) == MR_E_INVALID, "mr_load(NULL, NULL)");
  CHECK(mr_group_load(NULL, NULL) == MR_E_INVALID, "mr_group_load(NULL, NULL)");
  mr_group_options go;
  CHECK(mr_group_options_default(&go) == MR_OK, "mr_group_options_default");
  go.n_song_shards = 0;
  mr_group* g = 0;
  CHECK(mr_group_create(NULL, &go, &g) == MR_E_INVALID && !g, "0 song shards accepted");
  mr_dataset d = kat();
  int32_t b[3];
  CHECK(mr_song_shards(&d, 2, b) == MR_OK && b[0] == 0 && b[2] == NS && b[1] > 0 && b[1] < NS, "mr_song_shards");
  CHECK(mr_song_shards(&d, NS + 1, b) == MR_E_INVALID, "more shards than songs accepted");
  /* Java array lengths are checked before anything is read (NativeScoring's
   * arrays, jni/mr_jni.c): each wrong length is an error naming the array */
  static const char* arr[7] = {"trOff", "trSongs", "teOff", "teSongs", "songCount", "trLen", "teLen"};
  for (int i = 0; i < 7; ++i) {
    int64_t lens[7];
    memcpy(lens, LENS, sizeof lens);
    lens[i] -= 1;
    CHECK(ne_load(NULL, NTR, NTE, NS, TR_OFF, TR_SONGS, TE_OFF, TE_SONGS, SONG_COUNT, TR_LEN, TE_LEN, lens) ==
              MR_E_INVALID && strstr(ne_error(), arr[i]),
          "short %s accepted (%s)", arr[i], ne_error());
  }
  CHECK(ne_load(NULL, NTR, NTE, NS, TR_OFF, TR_SONGS, TE_OFF, TE_SONGS, SONG_COUNT, TR_LEN, TE_LEN, LENS) ==
            MR_E_INVALID && strstr(ne_error(), "handle"),
        "null handle accepted (%s)", ne_error());
  CHECK(ne_score_dense(NULL, MR_IBM, NULL, 0) == MR_E_INVALID, "ne_score_dense(NULL) accepted");
  CHECK(ne_topk(NULL, MR_IBM, 3, NULL, 0, NULL, 0) == MR_E_INVALID, "ne_topk(NULL) accepted");
}

int main(void) {
  error_codes();
  mr_options o;
  mr_options_default(&o);
  o.out_dtype = MR_OUT_F64;
  o.topk = 3;
  mr_ctx* c = 0;
  const int rc = mr_create(&o, &c);
  if (rc != MR_OK) {  /* no GPU: the compute entry points refuse, loudly */
    CHECK(rc == MR_E_HIP || rc == MR_E_INVALID, "mr_create without a GPU returned %d", rc);
    CHECK(!c, "context returned on failure");
    const int32_t dev0 = 0;
    CHECK(ne_create(&dev0, 1, 1, 1, 3, 1) == 0, "ne_create without a GPU succeeded");
    printf("error codes: %s\ngpu: skipped (%s)\n", failures ? "FAIL" : "ok", mr_last_error());
    return failures ? 1 : 0;
  }
  /* 2a. the single-context sequence of INTEGRATION.md */
  mr_dataset d = kat();
  CHECK(mr_load(c, &d) == MR_OK, "mr_load: %s", mr_last_error());
  double dense[NTE * NS];
  for (int model = 0; model < 2; ++model) {
    CHECK(mr_score_dense(c, model, dense) == MR_OK, "mr_score_dense: %s", mr_last_error());
    check_dense("context", model, dense);
  }
  mr_dataset bad = kat();
  int32_t unsorted[] = {1, 0, 2, 1, 2, 2, 3};
  bad.tr_songs = unsorted;
  CHECK(mr_load(c, &bad) == MR_E_INVALID, "unsorted CSR accepted");
  CHECK(mr_run(c, MR_IBM) == MR_E_STATE, "mr_run after a failed load accepted");
  CHECK(mr_destroy(c) == MR_OK, "mr_destroy");
  /* 2b. the shim's group sequence: one context, then 2 song shards x 2 user blocks */
  const int layouts[2][2] = {{1, 1}, {2, 2}};
  for (int l = 0; l < 2; ++l) {
    const int32_t dev0 = 0;
    mr_group* g = ne_create(&dev0, 1, layouts[l][0], layouts[l][1], 3, 1);
    CHECK(g != 0, "ne_create: %s", ne_error());
    if (!g) continue;
    CHECK(ne_load(g, NTR, NTE, NS, TR_OFF, TR_SONGS, TE_OFF, TE_SONGS, SONG_COUNT, TR_LEN, TE_LEN, LENS) == MR_OK,
          "ne_load: %s", ne_error());
    for (int model = 0; model < 2; ++model) {
      CHECK(ne_score_dense(g, model, dense, NTE * NS) == MR_OK, "ne_score_dense: %s", ne_error());
      check_dense(l ? "group 2x2" : "group 1x1", model, dense);
      CHECK(ne_score_dense(g, model, dense, NTE * NS - 1) == MR_E_INVALID, "short dense array accepted");
      int32_t songs[NTE * 4];
      double scores[NTE * 4];
      CHECK(ne_topk(g, model, 3, songs, NTE * 3, scores, NTE * 3) == MR_OK, "ne_topk: %s", ne_error());
      check_topk(l ? "group 2x2" : "group 1x1", model, 3, songs, scores);
      CHECK(ne_topk(g, model, 3, songs, NTE * 3 - 1, scores, NTE * 3) == MR_E_INVALID, "short songs array accepted");
      CHECK(ne_topk(g, model, 4, songs, NTE * 4, scores, NTE * 4) == MR_E_INVALID, "k != the handle's topk accepted");
    }
    CHECK(ne_destroy(g) == MR_OK, "ne_destroy");
  }
  printf("error codes + gpu KAT sequences: %s\n", failures ? "FAIL" : "ok");
  return failures ? 1 : 0;
}
