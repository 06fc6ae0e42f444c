"""hivemall_amd — an MI355X-native (gfx950 / CDNA4) classical machine-learning engine with
Apache Hivemall's SQL function surface.

Layers ("Layer map of the new framework"):
  sql/        HiveQL-subset frontend (N7)
  functions   registry of Hivemall SQL function names -> implementations (N6)
  models/     learners (N5): linear family, FM, FFM, MF/BPR, trees, topic models, ...
  ops/        device ops: gfx950 HIP kernels (csrc/kernels) + C++ CPU twins (csrc/host) (N3/N4)
  parallel/   process-per-GPU runtime, RCCL model mixing over xGMI (N2)
  io/         model tables, datasets, synthetic generators (N1)
"""
__version__ = "0.1.0"


def hivemall_version() -> str:
    """``hivemall_version()`` UDF."""
    return __version__
