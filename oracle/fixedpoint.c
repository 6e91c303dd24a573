/*
 * oracle/fixedpoint.c — TEST INFRASTRUCTURE ONLY (the bit-exact checker of the
 * HIP engine). Never linked into or called by the product path.
 *
 * The reference's scores (MusicRecommender.scala, MR) rewritten with the
 * two-hop identity of SURVEY.md §0.1 and int64 fixed-point accumulation:
 *
 *   IBM (MR:230-257): rank_i(u,s) = Σ_{s2∈T(u)} num(s,s2) / (sqrt c(s)·sqrt c(s2))
 *                   = (1/sqrt c(s)) · Σ_{v∈U_tr, s∈S(v)} Σ_{s2∈T(u)∩S(v)} 1/sqrt c(s2)
 *       fixed point: q(s2) = rint(2^F / sqrt c(s2)),  acc[s] = Σ_v Σ_{s2} q(s2),
 *                    score = (acc · 2^-F) / sqrt c(s)
 *   UBM (MR:140-166): rank_u(u,s) = Σ_{v∈U_tr, s∈S(v)} |T(u)∩S(v)| / (sqrt|T(u)|·sqrt|S(v)|)
 *       fixed point: q_v = rint((o_v / (sqrt|T(u)|·sqrt|S(v)|)) · 2^F),
 *                    acc[s] = Σ_v q_v,  score = acc · 2^-F
 *
 * Every floating-point operation here is the same IEEE operation, in the same
 * order, as in the HIP kernels (mr_engine.hip; both built without FP
 * contraction), and the integer sums are order-independent, so the engine
 * must match this oracle BIT FOR BIT (dense scores and top-k order). Against
 * the literal restatement (literal.c) it differs by the fixed-point rounding
 * only: relative error <= 2^-(F+1) / min term (SURVEY.md §7 hard part 1).
 *
 * Input: the interned CSR dataset (same layout as mr_dataset in
 * include/mr_engine.h). The per-song/per-user sqrt tables are recomputed here
 * with libm's correctly rounded sqrt.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

typedef struct fp_data {
  int32_t n_train, n_test, n_songs;
  const int64_t* tr_off; const int32_t* tr_songs;
  const int64_t* te_off; const int32_t* te_songs;
  const int32_t* song_count; const int32_t* tr_len; const int32_t* te_len;
} fp_data;

static int before(int64_t ka, int32_t sa, int64_t kb, int32_t sb) {
  return ka > kb || (ka == kb && sa < sb);
}

/*
 * model 0 = UBM, 1 = IBM. Scores songs [song_lo, song_hi) for test users
 * [user_lo, user_hi). dense (may be NULL): (user_hi-user_lo) x (song_hi-song_lo)
 * doubles, NaN for heard songs. top (may be NULL): k candidates per user,
 * ordered by (key desc, song asc), key = bit pattern of the double score,
 * missing entries song -1 / key -1. Returns 0, or -1 on allocation failure.
 */
int fp_model(const fp_data* d, int model, int frac_bits, int32_t song_lo, int32_t song_hi, int32_t user_lo,
             int32_t user_hi, double* dense, int32_t k, int32_t* top_songs, int64_t* top_keys) {
  const int n_tr = d->n_train, n_s = d->n_songs;
  const int width = song_hi - song_lo;
  const double two_f = ldexp(1.0, frac_bits), inv_f = ldexp(1.0, -frac_bits);
  /* transpose train u->s into s->u */
  int64_t* trs_off = calloc((size_t)n_s + 1, sizeof(int64_t));
  int32_t* trs_users = malloc(sizeof(int32_t) * (size_t)(d->tr_off[n_tr] + 1));
  int64_t* fill = malloc(sizeof(int64_t) * ((size_t)n_s + 1));
  int64_t* y = malloc(sizeof(int64_t) * ((size_t)n_tr + 1));
  int64_t* q = malloc(sizeof(int64_t) * ((size_t)n_tr + 1));
  int64_t* acc = malloc(sizeof(int64_t) * ((size_t)width + 1));
  int64_t* keys = malloc(sizeof(int64_t) * ((size_t)width + 1));
  char* heard = malloc((size_t)width + 1);
  double* sqrt_c = malloc(sizeof(double) * (size_t)n_s);
  int64_t* q_song = malloc(sizeof(int64_t) * (size_t)n_s);
  if (!trs_off || !trs_users || !fill || !y || !q || !acc || !keys || !heard || !sqrt_c || !q_song) {
    free(trs_off); free(trs_users); free(fill); free(y); free(q); free(acc); free(keys); free(heard);
    free(sqrt_c); free(q_song);
    return -1;
  }
  for (int v = 0; v < n_tr; ++v)
    for (int64_t i = d->tr_off[v]; i < d->tr_off[v + 1]; ++i) trs_off[d->tr_songs[i] + 1]++;
  for (int s = 0; s < n_s; ++s) trs_off[s + 1] += trs_off[s];
  memcpy(fill, trs_off, sizeof(int64_t) * (size_t)n_s);
  for (int v = 0; v < n_tr; ++v)
    for (int64_t i = d->tr_off[v]; i < d->tr_off[v + 1]; ++i) trs_users[fill[d->tr_songs[i]]++] = v;
  for (int s = 0; s < n_s; ++s) {
    sqrt_c[s] = sqrt((double)d->song_count[s]);
    q_song[s] = (int64_t)nearbyint(two_f / sqrt_c[s]);
  }

  for (int u = user_lo; u < user_hi; ++u) {
    /* stage 1: neighbour weights (MR:140-149 / MR:230-239) */
    memset(y, 0, sizeof(int64_t) * (size_t)n_tr);
    for (int64_t i = d->te_off[u]; i < d->te_off[u + 1]; ++i) {
      const int s2 = d->te_songs[i];
      const int64_t w = model == 1 ? q_song[s2] : 1;
      for (int64_t j = trs_off[s2]; j < trs_off[s2 + 1]; ++j) y[trs_users[j]] += w;
    }
    const double rs_u = sqrt((double)d->te_len[u]);
    for (int v = 0; v < n_tr; ++v) {
      if (y[v] == 0) { q[v] = 0; continue; }
      if (model == 1) {
        q[v] = y[v];
      } else {
        const double c = (double)y[v] / (rs_u * sqrt((double)d->tr_len[v]));
        q[v] = (int64_t)rint(c * two_f);
      }
    }
    /* stage 2: acc[s] = Σ_{v: s∈S(v)} q_v (MR:159-166 / MR:249-257) */
    memset(acc, 0, sizeof(int64_t) * (size_t)width);
    memset(heard, 0, (size_t)width);
    for (int v = 0; v < n_tr; ++v) {
      if (q[v] == 0 && y[v] == 0) continue;
      for (int64_t j = d->tr_off[v]; j < d->tr_off[v + 1]; ++j) {
        const int s = d->tr_songs[j];
        if (s >= song_lo && s < song_hi) acc[s - song_lo] += q[v];
      }
    }
    for (int64_t i = d->te_off[u]; i < d->te_off[u + 1]; ++i) {
      const int s = d->te_songs[i];
      if (s >= song_lo && s < song_hi) heard[s - song_lo] = 1;
    }
    double* row = dense ? dense + (size_t)(u - user_lo) * width : NULL;
    for (int i = 0; i < width; ++i) {
      double score = (double)acc[i] * inv_f;
      if (model == 1) score = score / sqrt_c[song_lo + i];
      if (row) row[i] = heard[i] ? NAN : score;
      int64_t key;
      memcpy(&key, &score, 8);
      keys[i] = heard[i] ? -1 : key;
    }
    /* top-k by (key desc, song asc): k passes, each the best after the previous */
    if (k > 0 && top_songs && top_keys) {
      int64_t pk = INT64_MAX;
      int32_t ps = -1;
      for (int r = 0; r < k; ++r) {
        int64_t bk = -1;
        int32_t bs = INT32_MAX;
        for (int i = 0; i < width; ++i) {
          const int32_t s = song_lo + i;
          if (keys[i] >= 0 && before(pk, ps, keys[i], s) && before(keys[i], s, bk, bs)) { bk = keys[i]; bs = s; }
        }
        const size_t o = (size_t)(u - user_lo) * k + r;
        if (bk < 0) { top_keys[o] = -1; top_songs[o] = -1; continue; }
        top_keys[o] = bk; top_songs[o] = bs;
        pk = bk; ps = bs;
      }
    }
  }
  free(trs_off); free(trs_users); free(fill); free(y); free(q); free(acc); free(keys); free(heard);
  free(sqrt_c); free(q_song);
  return 0;
}
