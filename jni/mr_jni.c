/*
 * jni/mr_jni.c — JNI shim: music_recommandation.NativeEngine (scala/) -> C ABI.
 *
 * Built only where a JDK exists (`make -C jni jni JAVA_HOME=...`; this image has
 * none). Every method pins its Java arrays with Get/ReleasePrimitiveArrayCritical,
 * makes the ONE core call of jni/nativeengine.c (compiled and exercised without a
 * JDK by jni/test_shim.c) and turns a negative return code into a Java exception
 * carrying mr_last_error() — the reference signals nothing itself (Map.apply's
 * NoSuchElementException, MatchError, System.exit at MR:326); the engine never
 * exits the JVM.
 */
#include <jni.h>
#include <stdint.h>

#include "nativeengine.h"

static void throw_rt(JNIEnv* env, const char* cls) {
  (*env)->ThrowNew(env, (*env)->FindClass(env, cls), mr_last_error());
}

/* long create(int[] devices, int songShards, int userBlocks, int topk) — f64 models */
JNIEXPORT jlong JNICALL Java_music_1recommandation_NativeEngine_00024_create(JNIEnv* env, jobject self,
                                                                             jintArray devices, jint songShards,
                                                                             jint userBlocks, jint topk) {
  (void)self;
  const jsize n = devices ? (*env)->GetArrayLength(env, devices) : 0;
  jint* d = n ? (*env)->GetIntArrayElements(env, devices, NULL) : NULL;
  mr_group* g = ne_create((const int32_t*)d, n, songShards, userBlocks, topk, 1);
  if (d) (*env)->ReleaseIntArrayElements(env, devices, d, JNI_ABORT);
  if (!g) throw_rt(env, "java/lang/IllegalStateException");
  return (jlong)(intptr_t)g;
}

/* void load(long h, int nTr, int nTe, int nS, long[] trOff, int[] trSongs, long[] teOff, int[] teSongs,
 *           int[] songCount, int[] trLen, int[] teLen) */
JNIEXPORT void JNICALL Java_music_1recommandation_NativeEngine_00024_load(
    JNIEnv* env, jobject self, jlong h, jint nTr, jint nTe, jint nS, jlongArray trOff, jintArray trSongs,
    jlongArray teOff, jintArray teSongs, jintArray songCount, jintArray trLen, jintArray teLen) {
  (void)self;
  jarray a[7] = {trOff, trSongs, teOff, teSongs, songCount, trLen, teLen};
  void* p[7];
  for (int i = 0; i < 7; ++i) p[i] = (*env)->GetPrimitiveArrayCritical(env, a[i], NULL);
  const int rc = ne_load((mr_group*)(intptr_t)h, nTr, nTe, nS, p[0], p[1], p[2], p[3], p[4], p[5], p[6]);
  for (int i = 6; i >= 0; --i) (*env)->ReleasePrimitiveArrayCritical(env, a[i], p[i], JNI_ABORT);
  if (rc != MR_OK) throw_rt(env, "java/lang/IllegalArgumentException");
}

/* void scoreDense(long h, int model, double[] out)  (out: nTe * nS, NaN = heard song) */
JNIEXPORT void JNICALL Java_music_1recommandation_NativeEngine_00024_scoreDense(JNIEnv* env, jobject self, jlong h,
                                                                                jint model, jdoubleArray out) {
  (void)self;
  double* o = (*env)->GetPrimitiveArrayCritical(env, out, NULL);
  const int rc = ne_score_dense((mr_group*)(intptr_t)h, model, o);
  (*env)->ReleasePrimitiveArrayCritical(env, out, o, 0);
  if (rc != MR_OK) throw_rt(env, "java/lang/RuntimeException");
}

/* void topk(long h, int model, int k, int[] songs, double[] scores)  (nTe * k each) */
JNIEXPORT void JNICALL Java_music_1recommandation_NativeEngine_00024_topk(JNIEnv* env, jobject self, jlong h,
                                                                          jint model, jint k, jintArray songs,
                                                                          jdoubleArray scores) {
  (void)self;
  int32_t* s = (*env)->GetPrimitiveArrayCritical(env, songs, NULL);
  double* sc = (*env)->GetPrimitiveArrayCritical(env, scores, NULL);
  const int rc = ne_topk((mr_group*)(intptr_t)h, model, k, s, sc);
  (*env)->ReleasePrimitiveArrayCritical(env, scores, sc, 0);
  (*env)->ReleasePrimitiveArrayCritical(env, songs, s, 0);
  if (rc != MR_OK) throw_rt(env, "java/lang/RuntimeException");
}

/* void destroy(long h) */
JNIEXPORT void JNICALL Java_music_1recommandation_NativeEngine_00024_destroy(JNIEnv* env, jobject self, jlong h) {
  (void)env;
  (void)self;
  ne_destroy((mr_group*)(intptr_t)h);
}
