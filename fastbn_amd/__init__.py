"""fastbn_amd -- MI355X-native FastBN hot paths (junction-tree inference, PC-stable CI sweep).

Python mirror of the reference's operator API over the C-ABI in ``include/fastbn.h``
(``libfastbn.so``, built in-tree by ``__graft_entry__.build()``).  The classes keep the
reference's names and argument meaning:

* ``JunctionTree(network, device).EvaluateAccuracy(...)`` / ``.infer(evidence)``
  -- ``JunctionTree`` + ``Inference`` (include/JunctionTree.h:19-94, include/Inference.h:23-49)
* ``PCStable(alpha, depth).StructLearnCompData(dataset, group_size)``
  -- include/PCStable.h:23-59
* ``IndependenceTest(dataset, alpha).IndependenceResult(x, y, z)``
  -- include/IndependenceTest.h:30-56

There is no CPU fallback: if the HIP library is missing, importing works but every call raises.
"""
from .api import (  # noqa: F401
    FastBNError,
    Network,
    Dataset,
    JunctionTree,
    IndependenceTest,
    PCStable,
    PCResult,
    orient_skeleton,
    shd_bif,
    lib,
    load_libsvm,
    write_csv,
    write_libsvm,
    device_count,
    kernel_options,
)

__all__ = ["FastBNError", "Network", "Dataset", "JunctionTree", "IndependenceTest", "PCStable", "PCResult", "orient_skeleton", "shd_bif",
           "lib", "load_libsvm", "write_csv", "write_libsvm", "device_count", "kernel_options"]
