// GGUFHipLoader.kt — reference-side binding of include/lk_gguf.h (GGUF quantized-tensor
// loading, SURVEY §8f row 1). Drop-in next to K/gguf/ModelLoader.kt, whose loadFromFile is a
// stub and whose loadTensorData loads F32 only (K/gguf/ModelLoader.kt:13-15, :78-96).
//
// The file is memory-mapped by the library; tensors land in llama.kotlin's block layout
// (upstream Q4_0/Q4_1 nibbles are repacked on the GPU), in a ByteArray owned by the
// graph allocator, ready for computeMatMul / computeMatMulHip. Not compiled here.
package ai.solace.llamakotlin.gguf

import ai.solace.llamakotlin.core.*
import ai.solace.llamakotlin.hip.*
import kotlinx.cinterop.*

private fun ggufCheck(st: Int) {
    if (st == LK_OK.toInt()) return
    val msg = lk_last_error()?.toKString() ?: "lk_gguf status $st"
    when (st) {
        LK_ERR_INVALID_ARG.toInt() -> throw IllegalArgumentException(msg)
        LK_ERR_OUT_OF_BOUNDS.toInt() -> throw IndexOutOfBoundsException(msg)
        LK_ERR_NOT_IMPLEMENTED.toInt() -> throw NotImplementedError(msg)
        else -> throw IllegalStateException(msg)
    }
}

/** lk_type (GGMLType.fromValue ids) -> GGMLType. */
private fun ggmlType(id: Int): GGMLType =
    GGMLType.fromValue(id) ?: throw NotImplementedError("no GGMLType for lk_type $id")

class HipLoadedModel internal constructor(private val handle: CPointer<lk_gguf>) {
    private val cache = mutableMapOf<String, GGMLTensor>()

    val version: UInt get() = lk_gguf_version(handle)
    val tensorCount: Long get() = lk_gguf_tensor_count(handle)

    fun getStringValue(key: String): String? = memScoped {
        val i = lk_gguf_find_key(handle, key)
        if (i < 0 || lk_gguf_kv_type(handle, i) != LK_GGUF_STRING.toInt()) return null
        val s = alloc<CPointerVar<ByteVar>>()
        val n = alloc<ULongVar>()
        ggufCheck(lk_gguf_kv_get_string(handle, i, -1, s.ptr, n.ptr))
        s.value!!.readBytes(n.value.toInt()).decodeToString()
    }

    fun getTensorNames(): List<String> = memScoped {
        val info = alloc<lk_gguf_tensor_info>()
        (0 until tensorCount).map { i ->
            ggufCheck(lk_gguf_get_tensor_info(handle, i, info.ptr))
            info.name!!.toKString()
        }
    }

    /** LoadedModel.getTensor (K/gguf/ModelLoader.kt:40-48) for every type llama.kotlin names. */
    fun getTensor(name: String, graphAllocator: GGMLGraphAllocator): GGMLTensor? = cache[name] ?: memScoped {
        val i = lk_gguf_find_tensor(handle, name)
        if (i < 0) return null
        val info = alloc<lk_gguf_tensor_info>()
        ggufCheck(lk_gguf_get_tensor_info(handle, i, info.ptr))
        val ne = LongArray(info.n_dims) { d -> info.ne[d] }
        val t = graphAllocator.allocateTensor(ggmlType(info.type), ne)
        t.name = name
        val buf = graphAllocator.buffers[t.bufferId]!!
        buf.usePinned { p ->
            ggufCheck(lk_gguf_load_tensor(handle, i, p.addressOf(t.dataOffset.toInt()),
                                          (buf.size - t.dataOffset.toInt()).toULong(), 0, null))
        }
        cache[name] = t
        t
    }

    fun close() = lk_gguf_close(handle)
}

object HipModelLoader {
    /** ModelLoader.loadFromFile with upstream (llama.cpp) type ids; kotlinIds = true reads them
     *  as GGMLType.fromValue like GGUFParser.kt:93. */
    fun loadFromFile(path: String, kotlinIds: Boolean = false): HipLoadedModel = memScoped {
        val h = alloc<CPointerVar<lk_gguf>>()
        ggufCheck(lk_gguf_open_file(path, if (kotlinIds) LK_GGUF_KOTLIN_IDS else LK_GGUF_UPSTREAM_IDS, h.ptr))
        HipLoadedModel(h.value!!)
    }
}
