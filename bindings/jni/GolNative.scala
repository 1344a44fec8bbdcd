// GolNative.scala -- the Scala side of bindings/jni/gol_jni.c: the native
// method table and one backend worker actor per GPU that replaces the cell
// actors (CellActor.scala:10-102 + NextStateCellGathererActor.scala:21-60)
// of a backend.  Status: a source file the CPU suite cross-checks against
// gol_jni.c (tests/test_jni_glue.py: every @native def has its JNI entry
// point and back); never compiled here -- the image has no JDK or scalac.
// INTEGRATION.md describes the frontend side.
package gameoflife

import akka.actor.{Actor, ActorRef}

object GolNative {
  System.loadLibrary("gol_jni")

  // every Int-returning method returns the gol_* status code (0 = ok);
  // Long-returning ones return the value, or the negated status code
  @native def create(w: Long, h: Long, row0: Long, rows: Long, topology: Int, birth: Int, survive: Int,
                     device: Int, visWidth: Long, visHeight: Long): Long
  @native def destroy(h: Long): Unit
  @native def lastError(h: Long): String
  @native def seed(h: Long, seed: Long): Int
  @native def load(h: Long, packed: java.nio.IntBuffer, wordsPerRow: Long): Int
  @native def step(h: Long, gens: Int, hashes: java.nio.LongBuffer): Int
  @native def epoch(h: Long): Long
  @native def hash(h: Long, out: java.nio.LongBuffer): Int
  @native def snapshot(h: Long, packed: java.nio.IntBuffer, wordsPerRow: Long): Int
  @native def snapshotAsync(h: Long, packed: java.nio.IntBuffer, wordsPerRow: Long): Int
  @native def snapshotWait(h: Long): Long
  @native def snapshotQuery(h: Long): Int
  @native def hostAlloc(bytes: Long): java.nio.ByteBuffer
  @native def hostFree(buf: java.nio.ByteBuffer): Unit
  @native def getCell(h: Long, x: Long, y: Long): Int
  @native def checkpointBytes(h: Long): Long
  @native def checkpoint(h: Long, out: java.nio.ByteBuffer): Int
  @native def checkpointAsync(h: Long, out: java.nio.ByteBuffer): Int
  @native def restore(h: Long, in: java.nio.ByteBuffer): Int
  @native def replay(h: Long, gens: Int, above: java.nio.IntBuffer, below: java.nio.IntBuffer, wordsPerRow: Long,
                     hashes: java.nio.LongBuffer): Int
  @native def commUniqueId(): Array[Byte]
  @native def commInit(h: Long, id: Array[Byte], rank: Int, n: Int): Int
  @native def commAbort(h: Long): Int
  @native def commAllreduce(h: Long, values: java.nio.LongBuffer, count: Int): Int
  @native def shardRows(height: Long, rank: Int, n: Int, out: java.nio.LongBuffer): Int
  @native def setTuning(h: Long, bandRows: Int, gensPerPass: Int, wordsPerLane: Int): Int
  @native def profileEnable(h: Long, on: Boolean): Int
  @native def profileStats(h: Long, out: java.nio.ByteBuffer): Int
  @native def runtimeInfo(): String

  /** A non-zero status becomes the exception Akka's supervisor restarts on
    * (BoardCreator.scala:42-45). */
  def check(h: Long, rc: Int): Unit =
    if (rc != 0) throw new IllegalStateException(lastError(h))

  /** A Long result, or the exception its negated status code stands for. */
  def value(h: Long, v: Long): Long = {
    if (v < 0) check(h, (-v).toInt)
    v
  }

  def waitEpoch(h: Long): Long = value(h, snapshotWait(h))
}

/** What a worker reports in place of one CellStateMsg per cell and epoch
  * (CellActor.scala:89): its shard's partial state hash of every generation
  * (the shards' partials sum, mod 2^64, to the board's hash). */
case class EpochHashes(row0: Long, firstEpoch: Int, hashes: Seq[Long])

/** A background board dump for the LoggerActor (LoggerActor.scala:30-46
  * prints y rows of x entries for a board of size (x, y)). */
case class BoardDump(row0: Long, epoch: Long, packed: java.nio.ByteBuffer)

/** One per GPU: owns rows [row0, row0 + rows) of the board (replaces the
  * cells BoardCreator.deplyActorWithPosition spread over backends,
  * BoardCreator.scala:65-70). */
class GpuBackendWorker(size: BoardSize, row0: Long, rows: Long, device: Int, loggerRef: ActorRef,
                       dumpEvery: Int /* epochs between LoggerActor board dumps */)
    extends Actor {
  import CellActor._

  // reference geometry: (w+1) x (h+1) cells, neighbours in [0,w) x [0,h)
  // (BoardCreator.scala:47-53, package.scala:17-28); rule B3/S23 here, or
  // ref-effective (0x000 / 0x1FF) for the reference's own rule
  private val h = GolNative.create(size._1 + 1, size._2 + 1, row0, rows, /*GOL_REF_CLIPPED*/ 1,
                                   /*birth*/ 0x008, /*survive*/ 0x00C, device,
                                   /*visWidth*/ size._1, /*visHeight*/ size._2)
  private var epoch = 0
  private val hashes = java.nio.ByteBuffer.allocateDirect(8 * 1024)
    .order(java.nio.ByteOrder.nativeOrder()).asLongBuffer()

  // LoggerActor's board dump every `dumpEvery` epochs, in the background
  private val words = (size._1 + 1 + 31) / 32
  private val dumps = Array.fill(2)(GolNative.hostAlloc(4L * rows * words))   // double-buffered
  private var dumpPending = false
  private var next = 0

  override def postStop(): Unit = { GolNative.destroy(h); dumps.foreach(GolNative.hostFree) }

  def receive: Receive = {
    case CurrentEpochMsg(target) if target > epoch =>      // CellActor.scala:63-65
      while (epoch < target) {                             // catch up, CellActor.scala:41-47,86,
        val n = math.min(target - epoch, hashes.capacity)  // at most one buffer of hashes per call
        GolNative.check(h, GolNative.step(h, n, hashes))
        loggerRef ! EpochHashes(row0, epoch + 1, (0 until n).map(hashes.get))
        epoch += n
        if (dumpEvery > 0 && epoch % dumpEvery == 0) {
          // the previous dump is complete once waited for; the logger owns it
          // until the next-but-one dump reuses the buffer
          if (dumpPending) loggerRef ! BoardDump(row0, GolNative.waitEpoch(h), dumps(next ^ 1))
          GolNative.check(h, GolNative.snapshotAsync(h, dumps(next).asIntBuffer, words))  // overlaps the next steps
          dumpPending = true
          next ^= 1
        }
      }
  }
}
