/*
 * oracle/literal.c — TEST INFRASTRUCTURE ONLY (parity checker and the timed
 * CPU baseline of bench.py). Never linked into or called by the product path.
 *
 * A literal C restatement of the reference's scoring loop nests, over STRING
 * ids with linear `contains` scans, exactly as the Scala code does them
 * (reference: src/main/scala/music_recommandation/MusicRecommender.scala, MR):
 *
 *   getModel / getModelP                 MR:105-111 / MR:119-125
 *     for s <- songs; u <- testUsers; if !T(u).contains(s) yield rank(u, s)
 *   UBM cosineSimilarity                  MR:140-149
 *     num = songs.map(song => T(u1).contains(song) && S(u2).contains(song) ? 1 : 0).sum
 *     den = sqrt(T(u1).length) * sqrt(S(u2).length); den != 0 ? num/den : 0.0
 *   UBM rank                              MR:159-166
 *     (for u2 <- trainUsers if S(u2).contains(song) yield cos(user, u2)).sum
 *   IBM cosineSimilarity                  MR:230-239
 *     num = trainUsers.map(v => L(s1).contains(v) && L(s2).contains(v) ? 1 : 0).sum
 *     den = sqrt(L(s1).length) * sqrt(L(s2).length)
 *   IBM rank                              MR:249-257
 *     (for s2 <- songs if s2 != song if T(user).contains(s2) yield cos(song, s2)).sum
 *
 * `.sum` on an Array[Double] is a left fold from 0.0 in element order; the
 * only thing this restatement cannot reproduce is the order of the JVM
 * HashSet behind `songs`/`trainUsers` (MR:51, MR:28), which moves results by
 * a few ulps. Map lookups (`m(key)`) are O(1) hashed in Scala and are direct
 * array indexing here. The parallel variant splits the flattened (s, u) pair
 * space over pthreads like getModelP's songs.par x testUsers.par; every
 * rank() itself runs sequentially, so par == seq bit for bit (README:254-261).
 *
 * Lists are given as arrays of C strings: lst_off[i]..lst_off[i+1] index into
 * `lst` (the reference's Array[String] values, duplicates kept, in the
 * reference's prepend order).
 */
#include <math.h>
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

typedef struct lit_data {
  int32_t n_songs, n_train, n_test;
  const char* const* songs;        /* songs (MR:58)                      */
  const char* const* train_users;  /* trainUsers (MR:55)                 */
  const char* const* test_users;   /* testUsers (MR:56)                  */
  /* trainUsersToSongsMap: per train user, its songs (dups kept) */
  const int64_t* tr_off; const char* const* tr_lst;
  /* testUsersToSongsMap: per test user */
  const int64_t* te_off; const char* const* te_lst;
  /* songsToUsersMap: per song (same order as `songs`), train AND test users (dups kept) */
  const int64_t* su_off; const char* const* su_lst;
} lit_data;

/* Array[String].contains: linear scan with String.equals. */
static int contains(const char* const* lst, int64_t lo, int64_t hi, const char* x) {
  for (int64_t i = lo; i < hi; ++i)
    if (lst[i] == x || strcmp(lst[i], x) == 0) return 1;
  return 0;
}

/* ---- UBM (MR:140-166) ---- */
static double ubm_cos(const lit_data* d, int u, int v) {
  long num = 0;
  for (int s = 0; s < d->n_songs; ++s)
    if (contains(d->te_lst, d->te_off[u], d->te_off[u + 1], d->songs[s]) &&
        contains(d->tr_lst, d->tr_off[v], d->tr_off[v + 1], d->songs[s]))
      num += 1;
  const double den = sqrt((double)(d->te_off[u + 1] - d->te_off[u])) *
                     sqrt((double)(d->tr_off[v + 1] - d->tr_off[v]));
  return den != 0 ? (double)num / den : 0.0;
}

static double ubm_rank(const lit_data* d, int u, int s) {
  double acc = 0.0;
  for (int v = 0; v < d->n_train; ++v)
    if (contains(d->tr_lst, d->tr_off[v], d->tr_off[v + 1], d->songs[s])) acc += ubm_cos(d, u, v);
  return acc;
}

/* ---- IBM (MR:230-257) ---- */
static double ibm_cos(const lit_data* d, int s1, int s2) {
  long num = 0;
  for (int v = 0; v < d->n_train; ++v)
    if (contains(d->su_lst, d->su_off[s1], d->su_off[s1 + 1], d->train_users[v]) &&
        contains(d->su_lst, d->su_off[s2], d->su_off[s2 + 1], d->train_users[v]))
      num += 1;
  const double den = sqrt((double)(d->su_off[s1 + 1] - d->su_off[s1])) *
                     sqrt((double)(d->su_off[s2 + 1] - d->su_off[s2]));
  return den != 0 ? (double)num / den : 0.0;
}

static double ibm_rank(const lit_data* d, int u, int s) {
  double acc = 0.0;
  for (int s2 = 0; s2 < d->n_songs; ++s2) {
    if (s2 == s || strcmp(d->songs[s2], d->songs[s]) == 0) continue;
    if (contains(d->te_lst, d->te_off[u], d->te_off[u + 1], d->songs[s2])) acc += ibm_cos(d, s, s2);
  }
  return acc;
}

/* ---- driver (MR:105-125) ---- */
typedef struct job {
  const lit_data* d;
  int model;
  int64_t p0, p1;       /* flattened pair range [p0, p1) of s-major x u-minor */
  double* out;          /* [n_test][n_songs], NaN for heard (no pair emitted) */
  int64_t emitted;
} job;

static void* worker(void* arg) {
  job* j = (job*)arg;
  const lit_data* d = j->d;
  for (int64_t p = j->p0; p < j->p1; ++p) {
    const int s = (int)(p / d->n_test), u = (int)(p % d->n_test);
    double* o = j->out + (size_t)u * d->n_songs + s;
    if (contains(d->te_lst, d->te_off[u], d->te_off[u + 1], d->songs[s])) { *o = NAN; continue; }
    *o = j->model == 0 ? ubm_rank(d, u, s) : ibm_rank(d, u, s);
    j->emitted++;
  }
  return NULL;
}

/*
 * Score the (s, u) pairs p in [pair_lo, pair_hi) of the s-major x u-minor
 * enumeration (pair_hi <= 0 means all pairs) with `threads` pthreads
 * (threads <= 1: sequential getModel). model 0 = UBM, 1 = IBM.
 * out: n_test x n_songs doubles (only the covered pairs are written).
 * Returns the number of emitted (unheard) pairs, or -1 on error.
 */
int64_t lit_model(const lit_data* d, int model, int threads, int64_t pair_lo, int64_t pair_hi, double* out) {
  const int64_t total = (int64_t)d->n_songs * d->n_test;
  if (pair_hi <= 0 || pair_hi > total) pair_hi = total;
  if (pair_lo < 0) pair_lo = 0;
  if (threads < 1) threads = 1;
  if (threads > 256) threads = 256;
  job jobs[256];
  pthread_t tids[256];
  const int64_t n = pair_hi - pair_lo;
  for (int t = 0; t < threads; ++t) {
    jobs[t].d = d;
    jobs[t].model = model;
    jobs[t].p0 = pair_lo + n * t / threads;
    jobs[t].p1 = pair_lo + n * (t + 1) / threads;
    jobs[t].out = out;
    jobs[t].emitted = 0;
  }
  if (threads == 1) {
    worker(&jobs[0]);
    return jobs[0].emitted;
  }
  for (int t = 0; t < threads; ++t)
    if (pthread_create(&tids[t], NULL, worker, &jobs[t]) != 0) return -1;
  int64_t emitted = 0;
  for (int t = 0; t < threads; ++t) {
    pthread_join(tids[t], NULL);
    emitted += jobs[t].emitted;
  }
  return emitted;
}
