package music_recommandation

/**
 * JNI binding of the MI355X engine (jni/mr_jni.c -> jni/nativeengine.c -> include/mr_engine.h).
 *
 * One handle = one multi-GPU group (mr_group_*): `devices` lists the GPUs, the
 * engine splits the songs into `songShards` ranges (balanced by listener entries)
 * and the test users into `userBlocks`, one context per (block, shard) and GPU;
 * the shards of a block exchange their top-k lists with an in-library RCCL
 * all-gather. One GPU = Array(0), 1, 1. Calls are synchronous and must come from
 * one thread at a time (the driver's, main.scala:37-40). Errors arrive as
 * exceptions carrying the engine's message; the engine never exits the JVM.
 *
 * Not compiled in the build image (no JDK / scalac); jni/test_shim.c exercises
 * the same call sequences against libmr_engine.so.
 */
object NativeEngine {
  System.loadLibrary("mr_jni")

  val UBM = 0 // getUserBasedModel, MusicRecommender.scala:132-170
  val IBM = 1 // getItemBasedModel, MusicRecommender.scala:222-261

  @native def create(devices: Array[Int], songShards: Int, userBlocks: Int, topk: Int): Long
  @native def load(h: Long, nTr: Int, nTe: Int, nS: Int, trOff: Array[Long], trSongs: Array[Int],
                   teOff: Array[Long], teSongs: Array[Int], songCount: Array[Int],
                   trLen: Array[Int], teLen: Array[Int]): Unit
  /** out: nTe * nS scores, row-major by interned test user; NaN = song already heard (MR:109). */
  @native def scoreDense(h: Long, model: Int, out: Array[Double]): Unit
  /** songs / scores: nTe * k, per test user by (score desc, song id asc); song -1 = empty slot. */
  @native def topk(h: Long, model: Int, k: Int, songs: Array[Int], scores: Array[Double]): Unit
  @native def destroy(h: Long): Unit
}
