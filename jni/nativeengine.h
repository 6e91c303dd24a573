/*
 * jni/nativeengine.h — the JNI-free core of the JNI shim (jni/mr_jni.c).
 *
 * Each function is exactly the call sequence one Java native method makes on
 * the engine's C ABI (include/mr_engine.h), with plain C types, so the
 * sequence is compiled and exercised here (jni/test_shim.c, gcc) even though
 * the image has no JDK. The JNI wrappers only pin/unpin Java arrays around
 * these calls and turn a negative code into an exception carrying
 * ne_error(). Every handle is a multi-GPU group (mr_group_*): one GPU is the
 * group of one context, several GPUs get song shards x user blocks and the
 * in-library RCCL all-gather — the reference's single driver call
 * (getItemBasedModel2, distributed.scala:477-479) keeps reaching every GPU from
 * one JVM thread.
 *
 * Java hands over arrays whose lengths the JVM knows and C does not: every
 * entry takes those lengths and checks them against the sizes the call
 * implies BEFORE the engine reads or writes a byte (MR_E_INVALID otherwise), so
 * a short Java array is an IllegalArgumentException, never a heap overrun.
 */
#ifndef NATIVEENGINE_H
#define NATIVEENGINE_H

#include <stdint.h>

#include "mr_engine.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Last error of the calling thread: the shim's own length checks, else mr_last_error(). */
const char* ne_error(void);

/* NativeEngine.create(devices, songShards, userBlocks, topk, f64): 0 = error. */
mr_group* ne_create(const int32_t* devices, int32_t n_devices, int32_t song_shards, int32_t user_blocks,
                    int32_t topk, int32_t out_f64);
/* NativeEngine.load(...): the interned CSR of MusicRecommender's maps (MR:26-62).
 * len[0..6] = Java lengths of tr_off, tr_songs, te_off, te_songs, song_count,
 * tr_len, te_len; they must be n_tr+1, tr_off[n_tr], n_te+1, te_off[n_te], n_s,
 * n_tr, n_te. */
int ne_load(mr_group* g, int32_t n_tr, int32_t n_te, int32_t n_s, const int64_t* tr_off, const int32_t* tr_songs,
            const int64_t* te_off, const int32_t* te_songs, const int32_t* song_count, const int32_t* tr_len,
            const int32_t* te_len, const int64_t len[7]);
/* NativeEngine.scoreDense(model, out): out = n_te x n_s doubles (f64 handle), NaN = heard
 * (replaces getModel(rank), MR:105-111, for rank = UBM MR:140-166 / IBM MR:230-257);
 * out_len must be n_te * n_s. */
int ne_score_dense(mr_group* g, int32_t model, double* out, int64_t out_len);
/* NativeEngine.topk(model, k, songs, scores): n_te x k, (score desc, song asc);
 * both lengths must be n_te * k. */
int ne_topk(mr_group* g, int32_t model, int32_t k, int32_t* songs, int64_t songs_len, double* scores,
            int64_t scores_len);
int ne_destroy(mr_group* g);

#ifdef __cplusplus
}
#endif
#endif
