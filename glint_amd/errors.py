"""Exception types the reference's callers observe, so host code and tests read like Glint's.

The JVM raises ``IndexOutOfBoundsException`` from the partitioners (RangePartitioner.scala:30-32,
CyclicPartitioner.scala:20) and ``ArrayIndexOutOfBoundsException`` from the shard loops
(PartialVector.scala:38-39 on an out-of-partition key). The C ABI reports the latter as
GLINT_EOUTOFRANGE; the binding raises the same-named exception.
"""


class IndexOutOfBoundsException(IndexError):
    """java.lang.IndexOutOfBoundsException."""


class ArrayIndexOutOfBoundsException(IndexOutOfBoundsException):
    """java.lang.ArrayIndexOutOfBoundsException (a subclass, as on the JVM)."""

    def __init__(self, msg: str = "", record: int = -1):
        super().__init__(msg)
        self.record = record


class GlintDeviceError(RuntimeError):
    """HIP runtime failure (GLINT_EDEVICE), including 'no GPU present'."""


class ModelCreationException(RuntimeError):
    """glint.exceptions.ModelCreationException (ModelCreationException.scala:8)."""
