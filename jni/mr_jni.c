/*
 * jni/mr_jni.c — JNI shim: music_recommandation.NativeEngine (scala/) -> C ABI.
 *
 * Built only where a JDK exists (`make -C jni jni JAVA_HOME=...`; this image has
 * none). Every method checks its Java arrays (non-null; lengths handed to the
 * JDK-free core of jni/nativeengine.c, compiled and exercised without a JDK by
 * jni/test_shim.c, which checks them against the sizes the call implies before
 * the engine touches a byte), pins them with Get/ReleasePrimitiveArrayCritical
 * (a NULL pin is an OutOfMemoryError), makes the ONE core call and turns a
 * negative return code into a Java exception carrying ne_error() — the
 * reference signals nothing itself (Map.apply's NoSuchElementException,
 * MatchError, System.exit at MR:326); the engine never exits the JVM.
 */
#include <jni.h>
#include <stdint.h>

#include "nativeengine.h"

static void throw_msg(JNIEnv* env, const char* cls, const char* msg) {
  jclass c = (*env)->FindClass(env, cls);
  if (c) (*env)->ThrowNew(env, c, msg);
}

static void throw_rc(JNIEnv* env, int rc, const char* cls) {
  throw_msg(env, rc == MR_E_INVALID ? "java/lang/IllegalArgumentException" : cls, ne_error());
}

/* Pin n arrays; on a NULL pin release the ones already pinned, throw, return 0. */
static int pin_all(JNIEnv* env, jarray* a, void** p, int n) {
  for (int i = 0; i < n; ++i) {
    p[i] = (*env)->GetPrimitiveArrayCritical(env, a[i], NULL);
    if (!p[i]) {
      for (int j = i - 1; j >= 0; --j) (*env)->ReleasePrimitiveArrayCritical(env, a[j], p[j], JNI_ABORT);
      throw_msg(env, "java/lang/OutOfMemoryError", "GetPrimitiveArrayCritical failed");
      return 0;
    }
  }
  return 1;
}

/* long create(int[] devices, int songShards, int userBlocks, int topk) — f64 models */
JNIEXPORT jlong JNICALL Java_music_1recommandation_NativeEngine_00024_create(JNIEnv* env, jobject self,
                                                                             jintArray devices, jint songShards,
                                                                             jint userBlocks, jint topk) {
  (void)self;
  const jsize n = devices ? (*env)->GetArrayLength(env, devices) : 0;
  jint* d = n ? (*env)->GetIntArrayElements(env, devices, NULL) : NULL;
  if (n && !d) {
    throw_msg(env, "java/lang/OutOfMemoryError", "GetIntArrayElements failed");
    return 0;
  }
  mr_group* g = ne_create((const int32_t*)d, n, songShards, userBlocks, topk, 1);
  if (d) (*env)->ReleaseIntArrayElements(env, devices, d, JNI_ABORT);
  if (!g) throw_msg(env, "java/lang/IllegalStateException", ne_error());
  return (jlong)(intptr_t)g;
}

/* void load(long h, int nTr, int nTe, int nS, long[] trOff, int[] trSongs, long[] teOff, int[] teSongs,
 *           int[] songCount, int[] trLen, int[] teLen) */
JNIEXPORT void JNICALL Java_music_1recommandation_NativeEngine_00024_load(
    JNIEnv* env, jobject self, jlong h, jint nTr, jint nTe, jint nS, jlongArray trOff, jintArray trSongs,
    jlongArray teOff, jintArray teSongs, jintArray songCount, jintArray trLen, jintArray teLen) {
  (void)self;
  jarray a[7] = {trOff, trSongs, teOff, teSongs, songCount, trLen, teLen};
  int64_t len[7];
  void* p[7];
  for (int i = 0; i < 7; ++i) {
    if (!a[i]) {
      throw_msg(env, "java/lang/NullPointerException", "NativeEngine.load: null array");
      return;
    }
    len[i] = (*env)->GetArrayLength(env, a[i]);
  }
  if (!pin_all(env, a, p, 7)) return;
  const int rc = ne_load((mr_group*)(intptr_t)h, nTr, nTe, nS, p[0], p[1], p[2], p[3], p[4], p[5], p[6], len);
  for (int i = 6; i >= 0; --i) (*env)->ReleasePrimitiveArrayCritical(env, a[i], p[i], JNI_ABORT);
  if (rc != MR_OK) throw_rc(env, rc, "java/lang/IllegalArgumentException");
}

/* void scoreDense(long h, int model, double[] out)  (out: nTe * nS, NaN = heard song) */
JNIEXPORT void JNICALL Java_music_1recommandation_NativeEngine_00024_scoreDense(JNIEnv* env, jobject self, jlong h,
                                                                                jint model, jdoubleArray out) {
  (void)self;
  if (!out) {
    throw_msg(env, "java/lang/NullPointerException", "NativeEngine.scoreDense: null array");
    return;
  }
  jarray a[1] = {out};
  void* p[1];
  const int64_t n = (*env)->GetArrayLength(env, out);
  if (!pin_all(env, a, p, 1)) return;
  const int rc = ne_score_dense((mr_group*)(intptr_t)h, model, p[0], n);
  (*env)->ReleasePrimitiveArrayCritical(env, out, p[0], rc == MR_OK ? 0 : JNI_ABORT);
  if (rc != MR_OK) throw_rc(env, rc, "java/lang/RuntimeException");
}

/* void topk(long h, int model, int k, int[] songs, double[] scores)  (nTe * k each) */
JNIEXPORT void JNICALL Java_music_1recommandation_NativeEngine_00024_topk(JNIEnv* env, jobject self, jlong h,
                                                                          jint model, jint k, jintArray songs,
                                                                          jdoubleArray scores) {
  (void)self;
  if (!songs || !scores) {
    throw_msg(env, "java/lang/NullPointerException", "NativeEngine.topk: null array");
    return;
  }
  jarray a[2] = {songs, scores};
  void* p[2];
  const int64_t ns = (*env)->GetArrayLength(env, songs), nsc = (*env)->GetArrayLength(env, scores);
  if (!pin_all(env, a, p, 2)) return;
  const int rc = ne_topk((mr_group*)(intptr_t)h, model, k, p[0], ns, p[1], nsc);
  const jint mode = rc == MR_OK ? 0 : JNI_ABORT;
  (*env)->ReleasePrimitiveArrayCritical(env, scores, p[1], mode);
  (*env)->ReleasePrimitiveArrayCritical(env, songs, p[0], mode);
  if (rc != MR_OK) throw_rc(env, rc, "java/lang/RuntimeException");
}

/* void destroy(long h) */
JNIEXPORT void JNICALL Java_music_1recommandation_NativeEngine_00024_destroy(JNIEnv* env, jobject self, jlong h) {
  (void)env;
  (void)self;
  ne_destroy((mr_group*)(intptr_t)h);
}
