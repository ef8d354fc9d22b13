"""glint_amd -- MI355X-native push/pull reduction plane for Glint's parameter server.

The per-server vector/matrix shards of Glint (src/main/scala/glint/models/server/) live in HBM;
push is a hand-written HIP scatter-add and pull a gather (glint_amd/csrc/glint_gpu.hip), exposed
through the C ABI in include/glint_gpu.h. Importing this package loads that library and fails
loudly if it is missing: there is no CPU fallback.
"""
from . import _native

_native.load()

from .errors import (ArrayIndexOutOfBoundsException, GlintDeviceError,  # noqa: E402
                     IndexOutOfBoundsException, ModelCreationException)
from .partitioning import (CyclicPartition, CyclicPartitioner, RangePartition,  # noqa: E402
                           RangePartitioner)
from .shard import PartialMatrix, PartialVector  # noqa: E402
from .client import BigMatrix, BigVector, Client  # noqa: E402

__all__ = [
    "PartialVector", "PartialMatrix", "RangePartition", "RangePartitioner", "CyclicPartition",
    "CyclicPartitioner", "Client", "BigVector", "BigMatrix", "IndexOutOfBoundsException",
    "ArrayIndexOutOfBoundsException", "GlintDeviceError", "ModelCreationException",
]
