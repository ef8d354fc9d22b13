package glint.models.server.gpu

import scala.collection.mutable

import akka.actor.{ActorLogging, ActorRef}
import glint.messages.server.logic.AcknowledgeReceipt
import glint.messages.server.request._
import glint.messages.server.response.{ResponseDouble, ResponseFloat, ResponseInt, ResponseLong}
import glint.models.server.{PartialMatrix, PartialVector}
import glint.partitioning.Partition
import glint.partitioning.cyclic.CyclicPartition
import glint.partitioning.range.RangePartition
import spire.implicits._

/**
  * JNI bindings of libglint_gpu.so (include/glint_gpu.h) -- integration/jni/glint_jni.c. One typed
  * entry point per value type of the reference's partial models. Pushes return a ticket: the push
  * is applied in order on the shard's GPU stream, and `await(ticket)` returns once it (and every
  * earlier push of the shard) is applied; pulls are ordered after every enqueued push.
  */
object GpuShard {
  System.loadLibrary("glint_jni")

  final val I32 = 0
  final val I64 = 1
  final val F32 = 2
  final val F64 = 3

  @native def createRange(device: Int, dtype: Int, start: Long, end: Long, cols: Int): Long
  @native def createCyclic(device: Int, dtype: Int, index: Int, parts: Int, keys: Long, cols: Int): Long
  @native def destroy(handle: Long): Unit
  @native def zero(handle: Long): Unit
  @native def await(handle: Long, ticket: Long): Unit

  @native def vecPushD(handle: Long, keys: Array[Long], values: Array[Double], flags: Int): Long
  @native def vecPushF(handle: Long, keys: Array[Long], values: Array[Float], flags: Int): Long
  @native def vecPushL(handle: Long, keys: Array[Long], values: Array[Long], flags: Int): Long
  @native def vecPushI(handle: Long, keys: Array[Long], values: Array[Int], flags: Int): Long
  @native def matPushD(handle: Long, rows: Array[Long], cols: Array[Int], values: Array[Double], flags: Int): Long
  @native def matPushF(handle: Long, rows: Array[Long], cols: Array[Int], values: Array[Float], flags: Int): Long
  @native def matPushL(handle: Long, rows: Array[Long], cols: Array[Int], values: Array[Long], flags: Int): Long
  @native def matPushI(handle: Long, rows: Array[Long], cols: Array[Int], values: Array[Int], flags: Int): Long

  @native def vecPullD(handle: Long, keys: Array[Long], out: Array[Double]): Unit
  @native def vecPullF(handle: Long, keys: Array[Long], out: Array[Float]): Unit
  @native def vecPullL(handle: Long, keys: Array[Long], out: Array[Long]): Unit
  @native def vecPullI(handle: Long, keys: Array[Long], out: Array[Int]): Unit
  @native def matPullD(handle: Long, rows: Array[Long], cols: Array[Int], out: Array[Double]): Unit
  @native def matPullF(handle: Long, rows: Array[Long], cols: Array[Int], out: Array[Float]): Unit
  @native def matPullL(handle: Long, rows: Array[Long], cols: Array[Int], out: Array[Long]): Unit
  @native def matPullI(handle: Long, rows: Array[Long], cols: Array[Int], out: Array[Int]): Unit
  @native def matPullRowsD(handle: Long, rows: Array[Long], out: Array[Double]): Unit
  @native def matPullRowsF(handle: Long, rows: Array[Long], out: Array[Float]): Unit
  @native def matPullRowsL(handle: Long, rows: Array[Long], out: Array[Long]): Unit
  @native def matPullRowsI(handle: Long, rows: Array[Long], out: Array[Int]): Unit

  /** Pipelined pulls: `pullAsync` enqueues a pull (kind 0 get, 1 matrix get, 2 getRows) behind every
    * enqueued push and returns a handle; `pullFinish*` waits for it and fills the result array. */
  @native def pullAsync(handle: Long, kind: Int, rows: Array[Long], cols: Array[Int]): Long
  @native def pullFinishD(pending: Long, out: Array[Double]): Unit
  @native def pullFinishF(pending: Long, out: Array[Float]): Unit
  @native def pullFinishL(pending: Long, out: Array[Long]): Unit
  @native def pullFinishI(pending: Long, out: Array[Int]): Unit

  /** Sent by an actor to itself behind a burst of Pull messages (see GpuShardActor). */
  private[gpu] case object FlushPulls

  /** The shard of `partition` on GPU `device` (range or cyclic layout, as the partitioner chose). */
  def create(partition: Partition, dtype: Int, cols: Int, device: Int): Long = partition match {
    case p: RangePartition => createRange(device, dtype, p.start, p.end, cols)
    // CyclicPartition keeps numberOfKeys private; any key count giving the same size is equivalent
    case p: CyclicPartition =>
      createCyclic(device, dtype, p.index, p.numberOfPartitions, (p.size - 1).toLong * p.numberOfPartitions + p.index + 1, cols)
  }

  /** GPU for a partition: partitions are spread round-robin over the server's GPUs. */
  def deviceFor(partition: Partition): Int = partition.index % sys.props.getOrElse("glint.gpus", "8").toInt
}

/**
  * The GPU half of a partial model actor. `receive` and PushLogic are those of the reference's
  * PartialVector*/PartialMatrix* actors (e.g. PartialVectorDouble.scala:17-23) with one change in
  * timing: a push is enqueued (its update runs on the GPU in message order) and `updateFinished(id)`
  * -- which makes the id acknowledgeable -- runs when the AcknowledgeReceipt for it arrives, after
  * `await(ticket)`. The client's PushFSM (PushFSM.scala:88-120) sends that acknowledgement request
  * right after the push, so the actor answers it exactly as before, once the push is applied, and
  * meanwhile takes the next messages. The await covers every push enqueued before it, so all of them
  * become acknowledgeable then (`pending` holds only pushes newer than the last awaited one).
  *
  * Errors happen where the reference's happen: the library checks a message's keys when it is
  * enqueued, so an out-of-partition key throws ArrayIndexOutOfBoundsException from the Push (or Pull)
  * message itself, with nothing of it applied; Akka restarts the actor, postStop frees the shard and
  * the new instance allocates a zeroed one (the reference's restart re-creates `new Array[V](size)`).
  * The client's AcknowledgeReceipt then reaches the new actor and is answered NotAcknowledgeReceipt
  * (PushLogic.scala:44-49), and a Pull after the restart is answered from the zeroed shard.
  *
  * Pulls are pipelined the same way: a Pull enqueues its gather (pullAsync; it sees every push
  * enqueued before it, as get() sees every update before it) and its answer is held. The first held
  * pull sends FlushPulls to the actor itself; that message queues behind everything already in the
  * mailbox, so when it arrives the burst has been taken, and the held pulls are answered in arrival
  * order after their waits (the first wait covers most of the burst). The reference answers each Pull
  * in `receive` (PartialVectorDouble.scala:18); here a burst of Pulls costs one GPU round trip instead
  * of one per message. A restart answers the held pulls first (postStop).
  */
trait GpuShardActor extends ActorLogging { this: akka.actor.Actor =>
  protected def shard: Long
  private val pending = mutable.HashMap.empty[Int, Long]  // push id -> ticket
  private val held = mutable.ArrayBuffer.empty[() => Unit]  // answers of enqueued pulls, in arrival order

  /** Holds the answer of an enqueued pull (`answer` finishes it and replies to its sender). */
  protected def hold(answer: () => Unit): Unit = {
    held += answer
    if (held.size == 1) self ! GpuShard.FlushPulls
  }

  /** Answers every held pull, in arrival order. Every held answer runs even if an earlier one throws
    * (its pullFinish frees its native handle on every path, and the other senders still get their
    * replies); the first exception is rethrown afterwards, so the actor fails on it as the
    * reference's get() would inside `receive`. */
  protected def flushPulls(): Unit = {
    val answers = held.toList
    held.clear()
    var first: Throwable = null
    answers.foreach { a =>
      try a()
      catch { case t: Throwable => if (first == null) first = t }
    }
    if (first != null) throw first
  }

  protected def enqueued(id: Int, ticket: Long): Unit = pending.put(id, ticket)

  /** AcknowledgeReceipt(id) of an enqueued push: wait for it, then mark it -- and every push enqueued
    * before it, which the same wait covers -- received (PushLogic.updateFinished). */
  protected def settle(message: Any, finished: Int => Unit): Unit = message match {
    case AcknowledgeReceipt(id) =>
      pending.get(id).foreach { ticket =>
        GpuShard.await(shard, ticket)
        val done = pending.collect { case (i, t) if t <= ticket => i }.toList
        done.foreach { i => pending.remove(i); finished(i) }
      }
    case _ =>
  }

  override def postStop(): Unit = {
    try flushPulls() finally GpuShard.destroy(shard)
  }
}

// ---- vectors: PartialVector{Double,Float,Long,Int}.scala --------------------------------------------
class GpuPartialVectorDouble(partition: Partition) extends PartialVector[Double](partition) with GpuShardActor {
  override val data: Array[Double] = Array.emptyDoubleArray  // lives in HBM
  protected val shard: Long = GpuShard.create(partition, GpuShard.F64, 0, GpuShard.deviceFor(partition))
  override def update(keys: Array[Long], values: Array[Double]): Boolean = {
    GpuShard.await(shard, GpuShard.vecPushD(shard, keys, values, 0)); true
  }
  override def get(keys: Array[Long]): Array[Double] = {
    val out = new Array[Double](keys.length); GpuShard.vecPullD(shard, keys, out); out
  }
  override def receive: Receive = {
    case pull: PullVector =>
      val to = sender(); val out = new Array[Double](pull.keys.length)
      val p = GpuShard.pullAsync(shard, 0, pull.keys, null)
      hold(() => { GpuShard.pullFinishD(p, out); to ! ResponseDouble(out) })
    case GpuShard.FlushPulls => flushPulls()
    case push: PushVectorDouble => enqueued(push.id, GpuShard.vecPushD(shard, push.keys, push.values, 0))
    case x => settle(x, updateFinished); handleLogic(x, sender)
  }
}

class GpuPartialVectorFloat(partition: Partition) extends PartialVector[Float](partition) with GpuShardActor {
  override val data: Array[Float] = Array.emptyFloatArray
  protected val shard: Long = GpuShard.create(partition, GpuShard.F32, 0, GpuShard.deviceFor(partition))
  override def update(keys: Array[Long], values: Array[Float]): Boolean = {
    GpuShard.await(shard, GpuShard.vecPushF(shard, keys, values, 0)); true
  }
  override def get(keys: Array[Long]): Array[Float] = {
    val out = new Array[Float](keys.length); GpuShard.vecPullF(shard, keys, out); out
  }
  override def receive: Receive = {
    case pull: PullVector =>
      val to = sender(); val out = new Array[Float](pull.keys.length)
      val p = GpuShard.pullAsync(shard, 0, pull.keys, null)
      hold(() => { GpuShard.pullFinishF(p, out); to ! ResponseFloat(out) })
    case GpuShard.FlushPulls => flushPulls()
    case push: PushVectorFloat => enqueued(push.id, GpuShard.vecPushF(shard, push.keys, push.values, 0))
    case x => settle(x, updateFinished); handleLogic(x, sender)
  }
}

class GpuPartialVectorLong(partition: Partition) extends PartialVector[Long](partition) with GpuShardActor {
  override val data: Array[Long] = Array.emptyLongArray
  protected val shard: Long = GpuShard.create(partition, GpuShard.I64, 0, GpuShard.deviceFor(partition))
  override def update(keys: Array[Long], values: Array[Long]): Boolean = {
    GpuShard.await(shard, GpuShard.vecPushL(shard, keys, values, 0)); true
  }
  override def get(keys: Array[Long]): Array[Long] = {
    val out = new Array[Long](keys.length); GpuShard.vecPullL(shard, keys, out); out
  }
  override def receive: Receive = {
    case pull: PullVector =>
      val to = sender(); val out = new Array[Long](pull.keys.length)
      val p = GpuShard.pullAsync(shard, 0, pull.keys, null)
      hold(() => { GpuShard.pullFinishL(p, out); to ! ResponseLong(out) })
    case GpuShard.FlushPulls => flushPulls()
    case push: PushVectorLong => enqueued(push.id, GpuShard.vecPushL(shard, push.keys, push.values, 0))
    case x => settle(x, updateFinished); handleLogic(x, sender)
  }
}

class GpuPartialVectorInt(partition: Partition) extends PartialVector[Int](partition) with GpuShardActor {
  override val data: Array[Int] = Array.emptyIntArray
  protected val shard: Long = GpuShard.create(partition, GpuShard.I32, 0, GpuShard.deviceFor(partition))
  override def update(keys: Array[Long], values: Array[Int]): Boolean = {
    GpuShard.await(shard, GpuShard.vecPushI(shard, keys, values, 0)); true
  }
  override def get(keys: Array[Long]): Array[Int] = {
    val out = new Array[Int](keys.length); GpuShard.vecPullI(shard, keys, out); out
  }
  override def receive: Receive = {
    case pull: PullVector =>
      val to = sender(); val out = new Array[Int](pull.keys.length)
      val p = GpuShard.pullAsync(shard, 0, pull.keys, null)
      hold(() => { GpuShard.pullFinishI(p, out); to ! ResponseInt(out) })
    case GpuShard.FlushPulls => flushPulls()
    case push: PushVectorInt => enqueued(push.id, GpuShard.vecPushI(shard, push.keys, push.values, 0))
    case x => settle(x, updateFinished); handleLogic(x, sender)
  }
}

// ---- matrices: PartialMatrix{Double,Float,Long,Int}.scala (rows live row-major in HBM) ---------------
// Row pulls answer with the flattened rows x cols array: what ResponseSerializer sends for
// ResponseRows* (ResponseSerializer.scala:52-61) and what the client's AsyncBigMatrix* decodes.
class GpuPartialMatrixDouble(partition: Partition, cols: Int) extends PartialMatrix[Double](partition, cols)
  with GpuShardActor {
  override val data: Array[Array[Double]] = Array.empty[Array[Double]]
  protected val shard: Long = GpuShard.create(partition, GpuShard.F64, cols, GpuShard.deviceFor(partition))
  override def update(rows: Array[Long], cs: Array[Int], values: Array[Double]): Boolean = {
    GpuShard.await(shard, GpuShard.matPushD(shard, rows, cs, values, 0)); true
  }
  override def get(rows: Array[Long], cs: Array[Int]): Array[Double] = {
    val out = new Array[Double](rows.length); GpuShard.matPullD(shard, rows, cs, out); out
  }
  def getRowsFlat(rows: Array[Long]): Array[Double] = {
    val out = new Array[Double](rows.length * cols); GpuShard.matPullRowsD(shard, rows, out); out
  }
  // PartialMatrix.getRows (PartialMatrix.scala:37-46) reads data(row), which lives in HBM here: the
  // rows come back flat in one pull and are cut into cols-long arrays (MatrixBenchmark.scala:73,99)
  override def getRows(rows: Array[Long]): Array[Array[Double]] = {
    val flat = getRowsFlat(rows)
    Array.tabulate(rows.length)(i => java.util.Arrays.copyOfRange(flat, i * cols, (i + 1) * cols))
  }
  override def receive: Receive = {
    case pull: PullMatrix =>
      val to = sender(); val out = new Array[Double](pull.rows.length)
      val p = GpuShard.pullAsync(shard, 1, pull.rows, pull.cols)
      hold(() => { GpuShard.pullFinishD(p, out); to ! ResponseDouble(out) })
    case pull: PullMatrixRows =>
      val to = sender(); val out = new Array[Double](pull.rows.length * cols)
      val p = GpuShard.pullAsync(shard, 2, pull.rows, null)
      hold(() => { GpuShard.pullFinishD(p, out); to ! ResponseDouble(out) })
    case GpuShard.FlushPulls => flushPulls()
    case push: PushMatrixDouble => enqueued(push.id, GpuShard.matPushD(shard, push.rows, push.cols, push.values, 0))
    case x => settle(x, updateFinished); handleLogic(x, sender)
  }
}

class GpuPartialMatrixFloat(partition: Partition, cols: Int) extends PartialMatrix[Float](partition, cols)
  with GpuShardActor {
  override val data: Array[Array[Float]] = Array.empty[Array[Float]]
  protected val shard: Long = GpuShard.create(partition, GpuShard.F32, cols, GpuShard.deviceFor(partition))
  override def update(rows: Array[Long], cs: Array[Int], values: Array[Float]): Boolean = {
    GpuShard.await(shard, GpuShard.matPushF(shard, rows, cs, values, 0)); true
  }
  override def get(rows: Array[Long], cs: Array[Int]): Array[Float] = {
    val out = new Array[Float](rows.length); GpuShard.matPullF(shard, rows, cs, out); out
  }
  def getRowsFlat(rows: Array[Long]): Array[Float] = {
    val out = new Array[Float](rows.length * cols); GpuShard.matPullRowsF(shard, rows, out); out
  }
  // PartialMatrix.getRows (PartialMatrix.scala:37-46) reads data(row), which lives in HBM here: the
  // rows come back flat in one pull and are cut into cols-long arrays (MatrixBenchmark.scala:73,99)
  override def getRows(rows: Array[Long]): Array[Array[Float]] = {
    val flat = getRowsFlat(rows)
    Array.tabulate(rows.length)(i => java.util.Arrays.copyOfRange(flat, i * cols, (i + 1) * cols))
  }
  override def receive: Receive = {
    case pull: PullMatrix =>
      val to = sender(); val out = new Array[Float](pull.rows.length)
      val p = GpuShard.pullAsync(shard, 1, pull.rows, pull.cols)
      hold(() => { GpuShard.pullFinishF(p, out); to ! ResponseFloat(out) })
    case pull: PullMatrixRows =>
      val to = sender(); val out = new Array[Float](pull.rows.length * cols)
      val p = GpuShard.pullAsync(shard, 2, pull.rows, null)
      hold(() => { GpuShard.pullFinishF(p, out); to ! ResponseFloat(out) })
    case GpuShard.FlushPulls => flushPulls()
    case push: PushMatrixFloat => enqueued(push.id, GpuShard.matPushF(shard, push.rows, push.cols, push.values, 0))
    case x => settle(x, updateFinished); handleLogic(x, sender)
  }
}

class GpuPartialMatrixLong(partition: Partition, cols: Int) extends PartialMatrix[Long](partition, cols)
  with GpuShardActor {
  override val data: Array[Array[Long]] = Array.empty[Array[Long]]
  protected val shard: Long = GpuShard.create(partition, GpuShard.I64, cols, GpuShard.deviceFor(partition))
  override def update(rows: Array[Long], cs: Array[Int], values: Array[Long]): Boolean = {
    GpuShard.await(shard, GpuShard.matPushL(shard, rows, cs, values, 0)); true
  }
  override def get(rows: Array[Long], cs: Array[Int]): Array[Long] = {
    val out = new Array[Long](rows.length); GpuShard.matPullL(shard, rows, cs, out); out
  }
  def getRowsFlat(rows: Array[Long]): Array[Long] = {
    val out = new Array[Long](rows.length * cols); GpuShard.matPullRowsL(shard, rows, out); out
  }
  // PartialMatrix.getRows (PartialMatrix.scala:37-46) reads data(row), which lives in HBM here: the
  // rows come back flat in one pull and are cut into cols-long arrays (MatrixBenchmark.scala:73,99)
  override def getRows(rows: Array[Long]): Array[Array[Long]] = {
    val flat = getRowsFlat(rows)
    Array.tabulate(rows.length)(i => java.util.Arrays.copyOfRange(flat, i * cols, (i + 1) * cols))
  }
  override def receive: Receive = {
    case pull: PullMatrix =>
      val to = sender(); val out = new Array[Long](pull.rows.length)
      val p = GpuShard.pullAsync(shard, 1, pull.rows, pull.cols)
      hold(() => { GpuShard.pullFinishL(p, out); to ! ResponseLong(out) })
    case pull: PullMatrixRows =>
      val to = sender(); val out = new Array[Long](pull.rows.length * cols)
      val p = GpuShard.pullAsync(shard, 2, pull.rows, null)
      hold(() => { GpuShard.pullFinishL(p, out); to ! ResponseLong(out) })
    case GpuShard.FlushPulls => flushPulls()
    case push: PushMatrixLong => enqueued(push.id, GpuShard.matPushL(shard, push.rows, push.cols, push.values, 0))
    case x => settle(x, updateFinished); handleLogic(x, sender)
  }
}

class GpuPartialMatrixInt(partition: Partition, cols: Int) extends PartialMatrix[Int](partition, cols)
  with GpuShardActor {
  override val data: Array[Array[Int]] = Array.empty[Array[Int]]
  protected val shard: Long = GpuShard.create(partition, GpuShard.I32, cols, GpuShard.deviceFor(partition))
  override def update(rows: Array[Long], cs: Array[Int], values: Array[Int]): Boolean = {
    GpuShard.await(shard, GpuShard.matPushI(shard, rows, cs, values, 0)); true
  }
  override def get(rows: Array[Long], cs: Array[Int]): Array[Int] = {
    val out = new Array[Int](rows.length); GpuShard.matPullI(shard, rows, cs, out); out
  }
  def getRowsFlat(rows: Array[Long]): Array[Int] = {
    val out = new Array[Int](rows.length * cols); GpuShard.matPullRowsI(shard, rows, out); out
  }
  // PartialMatrix.getRows (PartialMatrix.scala:37-46) reads data(row), which lives in HBM here: the
  // rows come back flat in one pull and are cut into cols-long arrays (MatrixBenchmark.scala:73,99)
  override def getRows(rows: Array[Long]): Array[Array[Int]] = {
    val flat = getRowsFlat(rows)
    Array.tabulate(rows.length)(i => java.util.Arrays.copyOfRange(flat, i * cols, (i + 1) * cols))
  }
  override def receive: Receive = {
    case pull: PullMatrix =>
      val to = sender(); val out = new Array[Int](pull.rows.length)
      val p = GpuShard.pullAsync(shard, 1, pull.rows, pull.cols)
      hold(() => { GpuShard.pullFinishI(p, out); to ! ResponseInt(out) })
    case pull: PullMatrixRows =>
      val to = sender(); val out = new Array[Int](pull.rows.length * cols)
      val p = GpuShard.pullAsync(shard, 2, pull.rows, null)
      hold(() => { GpuShard.pullFinishI(p, out); to ! ResponseInt(out) })
    case GpuShard.FlushPulls => flushPulls()
    case push: PushMatrixInt => enqueued(push.id, GpuShard.matPushI(shard, push.rows, push.cols, push.values, 0))
    case x => settle(x, updateFinished); handleLogic(x, sender)
  }
}
