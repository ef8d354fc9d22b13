package glint.models.server.gpu

import akka.actor.ActorLogging
import glint.messages.server.request.{PullMatrix, PullMatrixRows, PullVector, PushMatrixDouble, PushVectorDouble}
import glint.messages.server.response.{ResponseDouble, ResponseRowsDouble}
import glint.models.server.{PartialMatrix, PartialVector}
import glint.partitioning.Partition
import glint.partitioning.cyclic.CyclicPartition
import glint.partitioning.range.RangePartition
import spire.implicits._

/**
  * JNI bindings of libglint_gpu.so (include/glint_gpu.h) -- see integration/jni/glint_jni.c.
  */
object GpuShard {
  System.loadLibrary("glint_jni")

  final val F64 = 3
  @native def createRange(device: Int, dtype: Int, start: Long, end: Long, cols: Int): Long
  @native def createCyclic(device: Int, dtype: Int, index: Int, parts: Int, keys: Long, cols: Int): Long
  @native def destroy(handle: Long): Unit
  @native def zero(handle: Long): Unit
  @native def vecPush(handle: Long, keys: Array[Long], values: AnyRef, deterministic: Int): Unit
  @native def vecPull(handle: Long, keys: Array[Long], out: AnyRef): Unit
  @native def matPush(handle: Long, rows: Array[Long], cols: Array[Int], values: AnyRef, deterministic: Int): Unit
  @native def matPull(handle: Long, rows: Array[Long], cols: Array[Int], out: AnyRef): Unit
  @native def matPullRows(handle: Long, rows: Array[Long], out: AnyRef): Unit

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
  * PartialVectorDouble with its data in HBM. `receive` and PushLogic are exactly those of
  * PartialVectorDouble (src/main/scala/glint/models/server/PartialVectorDouble.scala:17-23); only
  * update/get run on the GPU. An out-of-partition key throws ArrayIndexOutOfBoundsException from
  * update/get as on the JVM, so Akka restarts the actor, whose constructor allocates a new, zeroed
  * shard (the reference's restart re-creates `new Array[Double](size)`).
  */
class GpuPartialVectorDouble(partition: Partition) extends PartialVector[Double](partition) with ActorLogging {

  override val data: Array[Double] = Array.emptyDoubleArray  // lives in HBM
  private val shard: Long = GpuShard.create(partition, GpuShard.F64, 0, GpuShard.deviceFor(partition))

  override def update(keys: Array[Long], values: Array[Double]): Boolean = {
    GpuShard.vecPush(shard, keys, values, 0)
    true
  }

  override def get(keys: Array[Long]): Array[Double] = {
    val out = new Array[Double](keys.length)
    GpuShard.vecPull(shard, keys, out)
    out
  }

  override def postStop(): Unit = GpuShard.destroy(shard)

  override def receive: Receive = {
    case pull: PullVector => sender ! ResponseDouble(get(pull.keys))
    case push: PushVectorDouble =>
      update(push.keys, push.values)
      updateFinished(push.id)
    case x => handleLogic(x, sender)
  }
}

/**
  * PartialMatrixDouble with its rows in HBM (row-major, PartialMatrixDouble.scala:19-28).
  */
class GpuPartialMatrixDouble(partition: Partition, cols: Int) extends PartialMatrix[Double](partition, cols)
  with ActorLogging {

  override val data: Array[Array[Double]] = Array.empty[Array[Double]]  // lives in HBM
  private val shard: Long = GpuShard.create(partition, GpuShard.F64, cols, GpuShard.deviceFor(partition))

  override def update(rows: Array[Long], cols: Array[Int], values: Array[Double]): Boolean = {
    GpuShard.matPush(shard, rows, cols, values, 0)
    true
  }

  override def get(rows: Array[Long], cols: Array[Int]): Array[Double] = {
    val out = new Array[Double](rows.length)
    GpuShard.matPull(shard, rows, cols, out)
    out
  }

  /** Rows as one flattened array: reply with ResponseDouble directly (what the serializer makes of
    * ResponseRowsDouble anyway, ResponseSerializer.scala:52-61, and what AsyncBigMatrixDouble expects). */
  def getRowsFlat(rows: Array[Long]): Array[Double] = {
    val out = new Array[Double](rows.length * this.cols)
    GpuShard.matPullRows(shard, rows, out)
    out
  }

  override def postStop(): Unit = GpuShard.destroy(shard)

  override def receive: Receive = {
    case pull: PullMatrix => sender ! ResponseDouble(get(pull.rows, pull.cols))
    case pull: PullMatrixRows => sender ! ResponseDouble(getRowsFlat(pull.rows))
    case push: PushMatrixDouble =>
      update(push.rows, push.cols, push.values)
      updateFinished(push.id)
    case x => handleLogic(x, sender)
  }
}
