/* jni/nativeengine.c — see nativeengine.h. */
#include "nativeengine.h"

#include <stdarg.h>
#include <stdio.h>
#include <string.h>

static _Thread_local char ne_msg[512];
static _Thread_local int ne_own;  /* 1: ne_msg holds the last error */

static int ne_fail(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(ne_msg, sizeof ne_msg, fmt, ap);
  va_end(ap);
  ne_own = 1;
  return MR_E_INVALID;
}

static int ne_rc(int rc) {  /* an engine call's result: its message is mr_last_error() */
  ne_own = 0;
  return rc;
}

const char* ne_error(void) { return ne_own ? ne_msg : mr_last_error(); }

mr_group* ne_create(const int32_t* devices, int32_t n_devices, int32_t song_shards, int32_t user_blocks,
                    int32_t topk, int32_t out_f64) {
  mr_options o;
  mr_group_options go;
  ne_own = 0;
  if (mr_options_default(&o) != MR_OK || mr_group_options_default(&go) != MR_OK) return 0;
  o.topk = topk;
  o.out_dtype = out_f64 ? MR_OUT_F64 : MR_OUT_F32;
  go.n_song_shards = song_shards;
  go.n_user_blocks = user_blocks;
  go.n_devices = n_devices;
  go.devices = devices;
  mr_group* g = 0;
  if (mr_group_create(&o, &go, &g) != MR_OK) return 0;
  return g;
}

int ne_load(mr_group* g, int32_t n_tr, int32_t n_te, int32_t n_s, const int64_t* tr_off, const int32_t* tr_songs,
            const int64_t* te_off, const int32_t* te_songs, const int32_t* song_count, const int32_t* tr_len,
            const int32_t* te_len, const int64_t len[7]) {
  if (!len) return ne_fail("null lengths");
  if (n_tr < 0 || n_te < 0 || n_s < 0) return ne_fail("negative sizes %d / %d / %d", n_tr, n_te, n_s);
  const int64_t want_fixed[7] = {(int64_t)n_tr + 1, -1, (int64_t)n_te + 1, -1, n_s, n_tr, n_te};
  static const char* names[7] = {"trOff", "trSongs", "teOff", "teSongs", "songCount", "trLen", "teLen"};
  const void* arr[7] = {tr_off, tr_songs, te_off, te_songs, song_count, tr_len, te_len};
  for (int i = 0; i < 7; ++i) {
    if (want_fixed[i] >= 0 && len[i] != want_fixed[i])
      return ne_fail("%s has %lld elements, %lld expected", names[i], (long long)len[i], (long long)want_fixed[i]);
    if (!arr[i] && len[i] > 0) return ne_fail("%s is null", names[i]);
  }
  /* the offsets are readable now: the column arrays must match their ends */
  if (len[1] != tr_off[n_tr])
    return ne_fail("trSongs has %lld elements, trOff[nTr] = %lld", (long long)len[1], (long long)tr_off[n_tr]);
  if (len[3] != te_off[n_te])
    return ne_fail("teSongs has %lld elements, teOff[nTe] = %lld", (long long)len[3], (long long)te_off[n_te]);
  if (!g) return ne_fail("null handle");
  mr_dataset d;
  memset(&d, 0, sizeof d);
  d.n_train_users = n_tr;
  d.n_test_users = n_te;
  d.n_songs = n_s;
  d.tr_off = tr_off;
  d.tr_songs = tr_songs;
  d.te_off = te_off;
  d.te_songs = te_songs;
  d.song_count = song_count;
  d.tr_len = tr_len;
  d.te_len = te_len;
  return ne_rc(mr_group_load(g, &d));  /* copies: the JNI wrapper unpins right after */
}

static int ne_shape(mr_group* g, int32_t* n_te, int32_t* n_s) {
  if (!g) return ne_fail("null handle");
  const int rc = mr_group_shape(g, 0, n_te, n_s);
  return rc ? ne_rc(rc) : MR_OK;
}

int ne_score_dense(mr_group* g, int32_t model, double* out, int64_t out_len) {
  int32_t n_te = 0, n_s = 0;
  int rc = ne_shape(g, &n_te, &n_s);
  if (rc) return rc;
  if (out_len != (int64_t)n_te * n_s)
    return ne_fail("out has %lld elements, nTe * nS = %lld (use topk past Int.MaxValue pairs)", (long long)out_len,
                   (long long)n_te * n_s);
  if (!out && out_len) return ne_fail("out is null");
  return ne_rc(mr_group_score_dense(g, model, out));
}

int ne_topk(mr_group* g, int32_t model, int32_t k, int32_t* songs, int64_t songs_len, double* scores,
            int64_t scores_len) {
  int32_t n_te = 0, n_s = 0;
  int rc = ne_shape(g, &n_te, &n_s);
  if (rc) return rc;
  if (k <= 0) return ne_fail("k = %d", k);
  if (songs_len != (int64_t)n_te * k || scores_len != (int64_t)n_te * k)
    return ne_fail("songs / scores have %lld / %lld elements, nTe * k = %lld", (long long)songs_len,
                   (long long)scores_len, (long long)n_te * k);
  if ((!songs || !scores) && n_te) return ne_fail("null output array");
  return ne_rc(mr_group_topk(g, model, k, songs, scores, 0));
}

int ne_destroy(mr_group* g) { return mr_group_destroy(g); }
