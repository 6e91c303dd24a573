package music_recommandation

/**
 * The batched replacement of `getModel(rank)` (MusicRecommender.scala:105-111)
 * for the two similarity models, as a trait the reference class mixes in:
 *
 *   class MusicRecommender(...) extends NativeScoring { ... }
 *
 * with its private fields made visible to the trait (drop `private` on
 * `songs`, `trainUsers`, `testUsers`, `trainUsersToSongsMap`,
 * `testUsersToSongsMap`, `songsToUsersMap`, MusicRecommender.scala:51-62) and
 * the two entry points redirected:
 *
 *   def getUserBasedModel: Array[(String, (String, Double))] = nativeModel(NativeEngine.UBM)
 *   def getItemBasedModel: Array[(String, (String, Double))] = nativeModel(NativeEngine.IBM)
 *
 * The pair set and values are the reference's (c(s) counts train AND test
 * listens, MR:60-62/237; lengths keep duplicates, MR:147; heard songs emit no
 * pair, MR:109); the emission order is the reference's own: s-major over its
 * `songs` array, u-minor over its `testUsers` array (MR:106-108). Scores are
 * int64 fixed point (2^-32), within 1e-7 relative of the Scala fp64 sums.
 *
 * Not compiled in the build image (no JDK / scalac).
 */
trait NativeScoring {
  def songs: Array[String]
  def trainUsers: Array[String]
  def testUsers: Array[String]
  def trainUsersToSongsMap: Map[String, Array[String]]
  def testUsersToSongsMap: Map[String, Array[String]]
  def songsToUsersMap: Map[String, Array[String]]

  /** GPUs of this process and the layout; one GPU by default. */
  def nativeDevices: Array[Int] = Array(0)
  def nativeSongShards: Int = nativeDevices.length
  def nativeUserBlocks: Int = 1
  def nativeTopK: Int = 10

  // Interning in lexicographic order (Ordering.String, the driver's sort key main.scala:57-59).
  private lazy val songIds: Array[String] = songs.sorted
  private lazy val songIdx: Map[String, Int] = songIds.zipWithIndex.toMap
  private lazy val trIds: Array[String] = trainUsers.sorted
  private lazy val teIds: Array[String] = testUsers.sorted
  private lazy val teIdx: Map[String, Int] = teIds.zipWithIndex.toMap

  /** CSR of distinct sorted song ids per user + the duplicate-counting lengths (MR:147). */
  private def csr(ids: Array[String], m: Map[String, Array[String]]): (Array[Long], Array[Int], Array[Int]) = {
    val rows = ids.map(u => m(u).map(songIdx).distinct.sorted)
    (rows.scanLeft(0L)(_ + _.length), rows.flatten, ids.map(u => m(u).length))
  }

  private lazy val handle: Long = {
    val h = NativeEngine.create(nativeDevices, nativeSongShards, nativeUserBlocks, nativeTopK)
    val (trOff, trSongs, trLen) = csr(trIds, trainUsersToSongsMap)
    val (teOff, teSongs, teLen) = csr(teIds, testUsersToSongsMap)
    NativeEngine.load(h, trIds.length, teIds.length, songIds.length, trOff, trSongs, teOff, teSongs,
                      songIds.map(s => songsToUsersMap(s).length), trLen, teLen)
    sys.addShutdownHook(NativeEngine.destroy(h))
    h
  }

  /** getModel(rank) for rank = UBM / IBM: every (test user, unheard song) pair.
   *
   * The dense model has nTe x nS cells, one JVM array: above Int.MaxValue cells
   * (the full Taste Profile: 10,000 x 384,546 = 3.85e9) neither it nor the
   * reference's pair array can exist, so the size is computed as a Long and such
   * a request fails with a clear exception instead of wrapping negative; use
   * nativeRecommendations (top-k lists) at that scale. Indices below stay Int:
   * they are < nTe * nS <= Int.MaxValue. */
  def nativeModel(model: Int): Array[(String, (String, Double))] = {
    val nS = songIds.length
    val cells = teIds.length.toLong * nS
    if (cells > Int.MaxValue - 8)  // the JVM's largest array
      throw new IllegalArgumentException(
        s"dense model of ${teIds.length} test users x $nS songs = $cells cells exceeds a JVM array; " +
        "use nativeRecommendations(model) for the per-user top-k lists")
    val out = new Array[Double](cells.toInt)
    NativeEngine.scoreDense(handle, model, out)
    for {
      s <- songs
      u <- testUsers
      x = out(teIdx(u) * nS + songIdx(s))
      if !x.isNaN
    } yield u -> (s, x)
  }

  /** Per test user, the k best unheard songs with their scores (score desc, song asc). */
  def nativeRecommendations(model: Int): Map[String, Array[(String, Double)]] = {
    val k = nativeTopK
    val songsOut = new Array[Int](teIds.length * k)
    val scoresOut = new Array[Double](teIds.length * k)
    NativeEngine.topk(handle, model, k, songsOut, scoresOut)
    teIds.zipWithIndex.map { case (u, i) =>
      u -> (0 until k).filter(j => songsOut(i * k + j) >= 0)
                      .map(j => songIds(songsOut(i * k + j)) -> scoresOut(i * k + j)).toArray
    }.toMap
  }
}
