"""hetseq_amd: MI355X-native heterogeneous data-parallel BERT training (HetSeq capabilities).

``torch`` is imported before any in-tree native module can load: the HIP kernel and RCCL
engine modules must bind to the HIP runtime torch brings (one libamdhip64 per process).
"""
import torch  # noqa: F401
