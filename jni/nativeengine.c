/* jni/nativeengine.c — see nativeengine.h. */
#include "nativeengine.h"

#include <string.h>

mr_group* ne_create(const int32_t* devices, int32_t n_devices, int32_t song_shards, int32_t user_blocks,
                    int32_t topk, int32_t out_f64) {
  mr_options o;
  mr_group_options go;
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
            const int32_t* te_len) {
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
  return mr_group_load(g, &d);  /* copies: the JNI wrapper unpins right after */
}

int ne_score_dense(mr_group* g, int32_t model, double* out) { return mr_group_score_dense(g, model, out); }

int ne_topk(mr_group* g, int32_t model, int32_t k, int32_t* songs, double* scores) {
  return mr_group_topk(g, model, k, songs, scores, 0);
}

int ne_destroy(mr_group* g) { return mr_group_destroy(g); }
