// GGMLHipBackend.kt — the reference-side binding a maintainer adds to llama.kotlin
// (src/nativeMain/kotlin/ai/solace/llamakotlin/core/), over the cinterop of include/lk_hip.h.
//
// It implements the reference's GGMLBackend plugin interface (K/core/GGMLBackend.kt:90-157)
// for exactly one op: MUL_MAT with src0 in {Q4_0, Q4_1, Q8_0, Q2_K, Q4_K, Q8_K} (or F32/F16
// general) and F32 activations, keeping the host ByteArrays authoritative (K/core/GGMLAlloc.kt:271). Every
// other node is left to GGMLCpuBackend. Not compiled in this repository (no Kotlin/Native
// toolchain offline); it is the integration contract the C-ABI tests in tests/test_abi.py pin.
package ai.solace.llamakotlin.core

import ai.solace.llamakotlin.hip.*
import kotlinx.cinterop.*

/** lk_status -> the exception computeMatMul throws (K/core/GGMLComputeOps.kt:1435-1565). */
private fun checkStatus(st: Int) {
    if (st == LK_OK.toInt()) return
    val msg = lk_last_error()?.toKString() ?: "lk_hip status $st"
    when (st) {
        LK_ERR_INVALID_ARG.toInt() -> throw IllegalArgumentException(msg)
        LK_ERR_NOT_IMPLEMENTED.toInt() -> throw NotImplementedError(msg)
        LK_ERR_OUT_OF_BOUNDS.toInt() -> throw IndexOutOfBoundsException(msg)
        LK_ERR_NO_BUFFER.toInt() -> throw IllegalStateException(msg)
        else -> throw IllegalStateException("HIP device error: $msg")
    }
}

/** GGMLType -> lk_type: the ids of GGMLType.fromValue (K/core/GGMLTypes.kt:145-168). The enum's
 *  ordinals differ from those ids past Q8_K (BITNET_1_58 sits at ordinal 14), so map by name. */
private fun lkTypeId(t: GGMLType): Int = when (t) {
    GGMLType.Q1_5_K -> LK_TYPE_Q1_5_K.toInt()
    GGMLType.I8 -> LK_TYPE_I8.toInt()
    GGMLType.I16 -> LK_TYPE_I16.toInt()
    GGMLType.I32 -> LK_TYPE_I32.toInt()
    GGMLType.I64 -> LK_TYPE_I64.toInt()
    GGMLType.BITNET_1_58 -> LK_TYPE_BITNET_1_58.toInt()
    else -> t.ordinal  // F32 .. Q8_K: ordinal == fromValue id
}

/** Fill an lk_tensor from a GGMLTensor whose bytes live in a pinned ByteArray. */
private fun fill(t: lk_tensor, src: GGMLTensor, base: CPointer<ByteVar>?, bytes: Int) {
    t.type = lkTypeId(src.type)
    for (i in 0 until 4) {
        t.ne[i] = src.ne[i]
        t.nb[i] = src.nb[i]
    }
    t.data = base
    t.buf_bytes = bytes.toULong()
    t.data_offset = src.dataOffset
}

/**
 * computeMatMul(graphAllocator, context, a, b, dst) on the MI355X: same signature, same
 * destination-tensor semantics, same exceptions. Weights are mirrored on the device once per
 * (ByteArray, offset, size, generation) by lk_weights_pin; activations and dst are copied per call.
 * Pass a new weightGeneration after rewriting a weight's bytes in place (include/lk_hip.h).
 */
fun computeMatMulHip(graphAllocator: GGMLGraphAllocator, @Suppress("unused") context: GGMLContext,
                     a: GGMLTensor, b: GGMLTensor, dst: GGMLTensor, weightGeneration: ULong = 0u,
                     shards: Int = 1, firstDevice: Int = 0) {
    val bufA = graphAllocator.buffers.getOrNull(a.bufferId)
    val bufB = graphAllocator.buffers.getOrNull(b.bufferId)
    val bufD = graphAllocator.buffers.getOrNull(dst.bufferId)
    memScoped {
        val la = alloc<lk_tensor>()
        val lb = alloc<lk_tensor>()
        val ld = alloc<lk_tensor>()
        // Pin the three ByteArrays for the duration of the call (the library copies what it needs).
        (bufA ?: ByteArray(0)).usePinned { pa ->
            (bufB ?: ByteArray(0)).usePinned { pb ->
                (bufD ?: ByteArray(0)).usePinned { pd ->
                    fill(la, a, if (bufA != null && bufA.isNotEmpty()) pa.addressOf(0) else null, bufA?.size ?: 0)
                    fill(lb, b, if (bufB != null && bufB.isNotEmpty()) pb.addressOf(0) else null, bufB?.size ?: 0)
                    fill(ld, dst, if (bufD != null && bufD.isNotEmpty()) pd.addressOf(0) else null, bufD?.size ?: 0)
                    val quant = a.type == GGMLType.Q4_0 || a.type == GGMLType.Q4_1 || a.type == GGMLType.Q8_0
                    if (shards > 1) {
                        // rows of A over the node's GPUs (shard r on device (firstDevice + r) mod lk_device_count())
                        if (quant && a.ne[0] % 32L == 0L)
                            checkStatus(lk_weights_pin_sharded_at(la.ptr, weightGeneration, shards, firstDevice))
                        checkStatus(lk_mul_mat_sharded_at(la.ptr, lb.ptr, ld.ptr, shards, firstDevice))
                    } else {
                        if (quant) checkStatus(lk_weights_pin(la.ptr, weightGeneration))
                        checkStatus(lk_mul_mat(la.ptr, lb.ptr, ld.ptr))
                    }
                }
            }
        }
    }
}

/**
 * The direct dot products computeDotProduct{F32Q41, F32Q80, Q80Q80, Q40Q40, Q41Q41, Q80Q40}
 * (core/GGMLComputeOps.kt:349-629) for every (row, col) of tensorA's rows x tensorB's columns
 * in one call: out[row * N + col], bit-identical to the Kotlin functions (same element
 * expressions, k in order, no fused multiply-add). kind = LK_DOT_* of lk_hip.h.
 */
fun computeDotProductMatrixHip(graphAllocator: GGMLGraphAllocator, kind: Int, tensorA: GGMLTensor,
                               tensorB: GGMLTensor, commonDimK: Int): FloatArray {
    val bufA = graphAllocator.buffers.getOrNull(tensorA.bufferId)
    val bufB = graphAllocator.buffers.getOrNull(tensorB.bufferId)
    val out = FloatArray(maxOf(tensorA.ne[1].toInt(), 0) * maxOf(tensorB.ne[0].toInt(), 0))
    memScoped {
        val la = alloc<lk_tensor>()
        val lb = alloc<lk_tensor>()
        (bufA ?: ByteArray(0)).usePinned { pa ->
            (bufB ?: ByteArray(0)).usePinned { pb ->
                out.usePinned { po ->
                    fill(la, tensorA, if (bufA != null && bufA.isNotEmpty()) pa.addressOf(0) else null, bufA?.size ?: 0)
                    fill(lb, tensorB, if (bufB != null && bufB.isNotEmpty()) pb.addressOf(0) else null, bufB?.size ?: 0)
                    checkStatus(lk_dot_direct(kind, la.ptr, lb.ptr, commonDimK.toLong(),
                                              if (out.isNotEmpty()) po.addressOf(0) else null))
                }
            }
        }
    }
    return out
}

/** computeDotProductQ80Q80(graphAllocator, a, b, row, col, K) through the matrix call (one element). */
fun computeDotProductQ80Q80Hip(graphAllocator: GGMLGraphAllocator, a: GGMLTensor, b: GGMLTensor,
                               row: Int, col: Int, commonDimK: Int): Float =
    computeDotProductMatrixHip(graphAllocator, LK_DOT_Q8_0_Q8_0, a, b, commonDimK)[row * b.ne[0].toInt() + col]

/**
 * A GGMLBackend that offloads MUL_MAT to the MI355X and defers everything else to the CPU backend.
 *
 * graphCompute (K/core/GGMLCpuBackend.kt:167-176 contract) walks the graph in node order
 * (computeGraph, K/core/GGMLComputeOps.kt:2515-2523) and cuts it into runs of consecutive
 * offloadable MUL_MAT nodes. Each run is one lk_graph (include/lk_hip.h), created once and cached
 * by the run's full tensor descriptors and the weight generation: weights stay mirrored in HBM,
 * independent nodes of a dependency level share one launch, and the device part is replayed as a
 * HIP graph. Every result reaches the ByteArrays by default: the graph may be one split of a larger
 * one (GGMLScheduler.executeGraphSplit, K/core/GGMLScheduler.kt:245-258, flags no outputs), whose
 * later splits may read any of them. With wholeGraphs = true (the caller passes whole graphs) only
 * results that leave the run go back (flagged isOutput(), K/core/GGMLTypes.kt:268, read by a node
 * outside the run, or read by no node at all). Nodes the backend does not offload run one at a time
 * on GGMLCpuBackend between the runs.
 *
 * shards > 1 (default): every offloaded node runs as lk_mul_mat_sharded — shard r of its rows on
 * GPU (device + r) mod lk_device_count(), results gathered through the host dst (the path the
 * one-GPU boxes test; shards may exceed the GPU count).
 * shards > 1 with rcclGraphs = true: the GPUs device, device + 1, … device + shards − 1 share every
 * run — one RCCL communicator per GPU (lk_comm_init_all), each run one lk_graph_create_sharded
 * graph: rank r computes rows [r·M/P, (r+1)·M/P) of every weight with only that shard pinned on its
 * GPU, and an in-place all-gather over xGMI per dependency level hands every GPU the whole result
 * (SURVEY §8e). This one-thread-drives-P-GPUs form has not run at P > 1 on hardware yet (the
 * one-process-per-GPU form is what the bench's multi-GPU run uses); when fewer than `shards` GPUs
 * are visible the backend falls back to the default form instead of failing.
 *
 * Residency contract: the host ByteArrays stay authoritative. Call bumpWeightGeneration()
 * whenever GGMLGraphAllocator re-places or rewrites tensor bytes (allocateGraph,
 * K/core/GGMLAlloc.kt:404-480) and evictBuffer(old) when reserve replaces a buffer (:392, :638).
 */
class GGMLHipBackend(private val device: Int = 0, private val shards: Int = 1,
                     private val wholeGraphs: Boolean = false,
                     private val rcclGraphs: Boolean = false) : GGMLBackend {
    private val cpu = GGMLCpuBackend()

    /** rcclGraphs and shards > 1 with that many GPUs from `device` on: rank r's communicator on GPU
     *  device + r (lk_comm_init_all), shared by every sharded run; null otherwise. */
    private val comms: CPointer<CPointerVar<lk_comm>>? =
        if (rcclGraphs && shards > 1 && device + shards <= lk_device_count()) {
            val arr = nativeHeap.allocArray<CPointerVar<lk_comm>>(shards)
            memScoped {
                val devs = allocArray<IntVar>(shards)
                for (r in 0 until shards) devs[r] = device + r
                val st = lk_comm_init_all(shards, devs, arr)
                if (st != LK_OK.toInt()) nativeHeap.free(arr)
                checkStatus(st)  // a constructor that cannot build its communicators throws
            }
            arr
        } else null

    /** The generation cached weight mirrors are current for (lk_weights_pin semantics). */
    var weightGeneration: ULong = 0u
        private set

    /** One cached lk_graph: the handle plus the pins that keep its ByteArrays' addresses valid
     *  (the graph copies inputs from and results to those addresses on every compute). */
    private class Run(val handle: CPointer<lk_graph>, val pins: List<Pinned<ByteArray>>) {
        fun close() {
            lk_graph_destroy(handle)
            pins.forEach { it.unpin() }
        }
    }

    /** Access-ordered LRU of runs, keyed by descriptors + write-back mask + generation. */
    private val runs = object : LinkedHashMap<List<Long>, Run>(16, 0.75f, true) {
        override fun removeEldestEntry(eldest: MutableMap.MutableEntry<List<Long>, Run>?): Boolean {
            if (size <= MAX_CACHED_RUNS) return false
            eldest?.value?.close()
            return true
        }
    }

    init {
        checkStatus(lk_init(device))
    }

    override fun getGuid(): String = "HIP-GFX950-LK"
    override fun getName(): String = "HIP"
    override fun free() {
        dropRuns()
        comms?.let { arr ->
            for (r in 0 until shards) lk_comm_destroy(arr[r])
            nativeHeap.free(arr)
        }
        lk_shutdown()
    }
    override fun getDefaultBufferType(): GGMLBackendBufferType = cpu.getDefaultBufferType()  // host ByteArrays stay authoritative

    /** The weight bytes changed in place: every cached run is dropped, the next compute pins the
     *  current bytes under the new generation (superseding the old mirrors). */
    fun bumpWeightGeneration(): ULong {
        weightGeneration++
        dropRuns()
        return weightGeneration
    }

    /** A ByteArray the allocator is about to drop or replace: forget its device mirrors. */
    fun evictBuffer(buffer: ByteArray) {
        dropRuns()
        if (buffer.isEmpty()) return
        buffer.usePinned { checkStatus(lk_weights_evict_buffer(it.addressOf(0), buffer.size.toULong())) }
    }

    private fun dropRuns() {
        runs.values.forEach { it.close() }
        runs.clear()
    }

    override fun supportsOp(tensor: GGMLTensor): Boolean {
        if (tensor.op != GGMLOp.MUL_MAT) return false
        val a = tensor.src[0] ?: return false
        val b = tensor.src[1] ?: return false
        val quant = (a.type == GGMLType.Q4_0 || a.type == GGMLType.Q4_1 || a.type == GGMLType.Q8_0 ||
            a.type == GGMLType.Q2_K || a.type == GGMLType.Q4_K || a.type == GGMLType.Q8_K) &&
            b.type == GGMLType.F32 && tensor.type == GGMLType.F32
        val general = (a.type == GGMLType.F32 && b.type == GGMLType.F32 && tensor.type == GGMLType.F32) ||
            (a.type == GGMLType.F16 && b.type == GGMLType.F16 && tensor.type == GGMLType.F16)
        return quant || general
    }

    override fun supportsBufferType(bufferType: GGMLBackendBufferType): Boolean = bufferType.isHost()

    override fun graphCompute(graph: GGMLCGraph): GGMLStatus {
        val ga = graph.allocator ?: return GGMLStatus.FAILED
        return try {
            val nodes = (0 until graph.nNodes).mapNotNull { graph.nodes[it] }
            var i = 0
            while (i < nodes.size) {
                if (!supportsOp(nodes[i])) {
                    // one-node graph on the CPU backend (K/core/GGMLCpuBackend.kt:167-176)
                    val one = GGMLCGraph(size = 1, nNodes = 1, nodes = arrayOf(nodes[i]), allocator = ga)
                    if (cpu.graphCompute(one) != GGMLStatus.SUCCESS) return GGMLStatus.FAILED
                    i++
                    continue
                }
                var j = i
                while (j < nodes.size && supportsOp(nodes[j])) j++
                if (shards > 1 && comms == null) {
                    // row shards node by node through the host dst (lk_mul_mat_sharded)
                    for (k in i until j) {
                        val n = nodes[k]
                        computeMatMulHip(ga, GGMLContext(), n.src[0]!!, n.src[1]!!, n, weightGeneration, shards, device)
                    }
                } else {
                    computeRun(ga, nodes, i, j)  // one lk_graph (row-sharded over the GPUs with comms)
                }
                i = j
            }
            GGMLStatus.SUCCESS
        } catch (e: Exception) {
            println("GGMLHipBackend: Error computing graph: ${e.message}")
            GGMLStatus.FAILED
        }
    }

    /** Nodes [from, to) of `all` (every one offloadable) as one cached lk_graph. */
    private fun computeRun(ga: GGMLGraphAllocator, all: List<GGMLTensor>, from: Int, to: Int) {
        val run = all.subList(from, to)
        val inRun = run.toHashSet()
        val readBy = HashMap<GGMLTensor, MutableList<GGMLTensor>>()
        for (n in all) for (s in n.src) if (s != null) readBy.getOrPut(s) { mutableListOf() }.add(n)
        val writeBack = run.map { n ->
            val readers = readBy[n].orEmpty()
            !wholeGraphs || n.isOutput() || readers.isEmpty() || readers.any { it !in inRun }
        }
        val bufs = ArrayList<ByteArray?>()
        fun buf(t: GGMLTensor): ByteArray? = ga.buffers.getOrNull(t.bufferId)
        val key = ArrayList<Long>(run.size * 3 * 12 + 1)
        key.add(weightGeneration.toLong())
        for ((k, n) in run.withIndex()) {
            for (t in listOf(n.src[0]!!, n.src[1]!!, n)) {
                val b = buf(t)
                bufs.add(b)
                key.add(lkTypeId(t.type).toLong())
                for (d in 0 until 4) { key.add(t.ne[d]); key.add(t.nb[d].toLong()) }
                key.add(t.dataOffset.toLong())
                key.add(b?.let { identityHash(it) } ?: 0L)
                key.add(b?.size?.toLong() ?: 0L)
            }
            key.add(if (writeBack[k]) 1L else 0L)
        }
        val cached = runs[key]
        if (cached != null) {
            checkStatus(lk_graph_compute(cached.handle))
            return
        }
        // pin every ByteArray the run touches for the graph's lifetime (one Pinned per array)
        val distinct = bufs.filterNotNull().filter { it.isNotEmpty() }.distinctBy { identityHash(it) }
        val pins = distinct.map { it.pin() }
        fun addr(b: ByteArray?): CPointer<ByteVar>? =
            if (b == null || b.isEmpty()) null else pins.first { it.get() === b }.addressOf(0)
        val created = memScoped {
            val n = run.size
            val la = allocArray<lk_tensor>(n)
            val lb = allocArray<lk_tensor>(n)
            val ld = allocArray<lk_tensor>(n)
            val outs = allocArray<UByteVar>(n)
            for ((k, node) in run.withIndex()) {
                val a = node.src[0]!!
                val b = node.src[1]!!
                fill(la[k], a, addr(buf(a)), buf(a)?.size ?: 0)
                fill(lb[k], b, addr(buf(b)), buf(b)?.size ?: 0)
                fill(ld[k], node, addr(buf(node)), buf(node)?.size ?: 0)
                outs[k] = if (writeBack[k]) 1u else 0u
            }
            val h = alloc<CPointerVar<lk_graph>>()
            val st = if (comms != null) lk_graph_create_sharded(comms, shards, la, lb, ld, n, outs, weightGeneration, h.ptr)
                     else lk_graph_create(la, lb, ld, n, outs, weightGeneration, h.ptr)
            if (st != LK_OK.toInt()) {
                pins.forEach { it.unpin() }
                checkStatus(st)
            }
            Run(h.value!!, pins)
        }
        runs[key] = created
        checkStatus(lk_graph_compute(created.handle))
    }

    private fun identityHash(b: ByteArray): Long = b.usePinned { it.addressOf(0).rawValue.toLong() }

    companion object {
        const val MAX_CACHED_RUNS = 32
    }
}
