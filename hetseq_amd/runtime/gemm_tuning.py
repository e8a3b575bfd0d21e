"""Measured library-GEMM selection (hipBLASLt / rocBLAS) via PyTorch TunableOp.

hipBLASLt's heuristic picks a poor tile for several BERT shapes (e.g. the
[4096 x 768] x [768 x 2304] QKV projection ran at 91 TF/s on MT96x32x128).
TunableOp times every hipBLASLt and rocBLAS solution for each GEMM shape once
and keeps the fastest.  Tables measured on MI355X (gfx950, ROCm 7 /
hipBLASLt of this image) are committed under ``configs/tunableop/`` and
loaded at start-up; shapes missing from the table are tuned on first use
(during warm-up) unless ``HETSEQ_GEMM_TUNING=0``.  Rows carry validators
(PyTorch / HIP / hipBLASLt / rocBLAS versions, GPU arch), so a table from a
different software stack is ignored rather than misapplied.
"""
from __future__ import annotations

import os
import tempfile

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
TABLE_DIR = os.path.join(ROOT, "configs", "tunableop")
_done = False


def enable(dtype_tag="fp32", tune_missing=None):
    """Turn on TunableOp for this process and load the committed table for ``dtype_tag``."""
    global _done
    if _done or not torch.cuda.is_available() or os.environ.get("HETSEQ_GEMM_TUNING", "1") == "0":
        return False
    import torch.cuda.tunable as tn

    if tune_missing is None:
        tune_missing = os.environ.get("HETSEQ_GEMM_TUNE_MISSING", "0") == "1"
    tn.enable(True)
    tn.tuning_enable(bool(tune_missing))
    if "PYTORCH_TUNABLEOP_MAX_TUNING_DURATION_MS" not in os.environ:
        tn.set_max_tuning_duration(100)
    # results of new tunings go to a private file (never into the repository) unless
    # HETSEQ_TUNABLEOP_OUT names one (tools/gpu_tune.sh uses that to refresh the tables)
    out = os.environ.get("HETSEQ_TUNABLEOP_OUT")
    if not out:
        out = os.path.join(tempfile.mkdtemp(prefix="hetseq_tunableop_"), "tunableop_%s.csv" % dtype_tag)
    tn.set_filename(out, insert_device_ordinal=True)
    for tag in ("fp32", "bf16") if dtype_tag == "bf16" else ("fp32",):
        path = os.path.join(TABLE_DIR, "gfx950_%s.csv" % tag)
        if os.path.exists(path):
            tn.read_file(path)
    _done = True
    return True


def configure(args):
    """Entry-point hook (train.py, bench.py): load the measured library-GEMM table and the
    per-call-site engine choices for ``args.dtype`` unless ``--no-gemm-tuning``."""
    if not torch.cuda.is_available() or getattr(args, "cpu", False) or not getattr(args, "gemm_tuning", True):
        return False
    dt = getattr(args, "dtype", "fp32")
    enable(dt, tune_missing=True if getattr(args, "gemm_tune_missing", False) else None)
    load_engine_choices(dt)
    return True


def reset():
    """Undo :func:`enable` (tests: no TunableOp state leaks from one test into the next)."""
    global _done
    if torch.cuda.is_available():
        import torch.cuda.tunable as tn

        tn.tuning_enable(False)
        tn.enable(False)
    _done = False


CHOICE_DIR = os.path.join(ROOT, "configs", "gemm_choices")


def load_engine_choices(dtype_tag="fp32"):
    """Preload the per-call-site engine choices (HIP kernel vs library, split-K) measured on
    gfx950 and committed under ``configs/gemm_choices/`` (written by ``bench.py
    --gemm-choices``), so a run needs no measuring in its first step.  Sites missing from
    the file are still measured on first use; ``HETSEQ_GEMM_CHOICES=measure`` ignores the
    file.  Entries measured under another fp32 engine policy are skipped."""
    if os.environ.get("HETSEQ_GEMM_CHOICES", "") == "measure" or not torch.cuda.is_available():
        return False
    from hetseq_amd.ops import gemm as G

    path = os.environ.get("HETSEQ_GEMM_CHOICES_FILE")
    if not path:  # per fp32 engine policy (gfx950_fp32_h3.json, ...), else the dtype's file
        path = os.path.join(CHOICE_DIR, "gfx950_%s_%s.json" % (dtype_tag, G.fp32_mode()))
        if dtype_tag != "fp32" or not os.path.exists(path):
            path = os.path.join(CHOICE_DIR, "gfx950_%s.json" % dtype_tag)
    if not os.path.exists(path):
        return False
    return G.load_choices(path)


def results():
    """The (op, shape, solution, ms) rows TunableOp holds for this process."""
    if not _done:
        return []
    import torch.cuda.tunable as tn

    return list(tn.get_results())
