"""ggml_hip — MI355X (gfx950) backend for llama.kotlin's quantized MUL_MAT path.

Host-side mirror of the reference's operator/plugin API for this path, over the
C-ABI in include/lk_hip.h (liblk_hip.so, hand-written HIP kernels):

  computeMatMul(graphAllocator, context, a, b, dst)  core/GGMLComputeOps.kt:1435
  GGMLTensor / GGMLGraphAllocator / GGMLType          core/GGMLTypes.kt, core/GGMLAlloc.kt
  GGMLHipBackend (GGMLBackend)                        core/GGMLBackend.kt:90-157
  dequantizeTensor / quantizeTensor (device)          core/GGMLComputeOps.kt:918 / :1040
  computeDotProductMatrix (direct Q x Q / F32 x Q)    core/GGMLComputeOps.kt:349-629
  RowShardedMulMat (rows over GPUs + RCCL gather)     new: the reference is single-device
  GGUFParser / ModelLoader / LoadedModel              gguf/GGUFParser.kt, gguf/ModelLoader.kt

There is no CPU compute path in this package: a missing liblk_hip.so raises.
"""
from . import _lib
from ._lib import (HipDeviceError, IllegalArgumentException, IllegalStateException, IndexOutOfBoundsException,
                   NotOffloadedError)
from .backend import GGMLBackendRegistry, GGMLHipBackend, GGMLStatus
from .ops import (DotKind, MulMatPlan, ResidentGraph, computeDotProductF32Q41, computeDotProductF32Q80, computeDotProductMatrix,
                  computeDotProductQ40Q40, computeDotProductQ41Q41, computeDotProductQ80Q40, computeDotProductQ80Q80, computeMatMul,
                  computeMatMulSharded, dequantizeTensor, quantizeTensor, setSyncWaitBound, syncCountersSum, syncTimeouts, debugRoute, debugScratchEpoch, debugPokeGemmCounter, scratchRelease, scratchBytes, to_lk, validateMatMul, weightsCachedBytes, weightsCachedCount,
                  weightsEvict, weightsEvictAll, weightsEvictBuffer, weightsPin, weightsPinSharded)
from .gguf import GGUFContext, GGUFParser, GGUFTensorInfo, GGUFType, LoadedModel, ModelLoader
from .sharded import Comm, P2PChain, P2PGroup, P2PMulMatPlan, RowShardedMulMat, ShardedMulMatPlan, row_slice, shard_rows, shard_view
from .tensor import (GGMLCGraph, GGMLContext, GGMLGraphAllocator, GGMLOp, GGMLTensor, GGMLType,
                     calculateContiguousStrides, calculateTensorByteSize)

__all__ = [
    "syncTimeouts", "setSyncWaitBound", "syncCountersSum", "debugRoute", "debugScratchEpoch", "debugPokeGemmCounter", "scratchRelease", "scratchBytes",
    "GGMLType", "GGMLTensor", "GGMLGraphAllocator", "GGMLContext", "GGMLCGraph", "GGMLOp",
    "calculateContiguousStrides", "calculateTensorByteSize",
    "computeMatMul", "computeMatMulSharded", "weightsPinSharded", "validateMatMul", "MulMatPlan", "ResidentGraph", "dequantizeTensor", "quantizeTensor", "weightsPin",
    "weightsEvictAll", "weightsEvict", "weightsEvictBuffer", "weightsCachedBytes", "weightsCachedCount", "to_lk", "DotKind", "computeDotProductMatrix", "computeDotProductF32Q41",
    "computeDotProductF32Q80", "computeDotProductQ80Q80", "computeDotProductQ40Q40", "computeDotProductQ41Q41",
    "computeDotProductQ80Q40",
    "GGMLHipBackend", "GGMLStatus", "GGMLBackendRegistry",
    "RowShardedMulMat", "row_slice", "shard_rows", "Comm", "ShardedMulMatPlan", "shard_view", "P2PGroup", "P2PMulMatPlan", "P2PChain",
    "GGUFParser", "GGUFContext", "GGUFTensorInfo", "GGUFType", "ModelLoader", "LoadedModel",
    "IllegalArgumentException", "IndexOutOfBoundsException", "IllegalStateException", "NotOffloadedError",
    "HipDeviceError",
]


def load_library():
    """Load liblk_hip.so now (raises ImportError if it was not built)."""
    return _lib.load()
