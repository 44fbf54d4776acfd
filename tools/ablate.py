#!/usr/bin/env python3
"""Time ablation builds of the engine in ONE process family on one GPU (bench-shaped
workload): each variant runs as a child process with TBE_LIB pointing at its build and
prints per-stage ms.  Variants are built beforehand in this container:
    python tools/ablate.py --build
then on the GPU box:
    python tools/ablate.py --run
"""
import argparse
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUTDIR = os.path.join(ROOT, "tools", "ablate_libs")
VARIANT_SETS = {
    "queue": {
        "base_q": ([], ["--workload", "queue", "--no-drain-variant"]),
        "noring_q": (["TBE_Q_NO_RING_WRITE"], ["--workload", "queue", "--no-drain-variant"]),
        "r1only_q": (["TBE_Q_R1_ONLY"], ["--workload", "queue", "--no-drain-variant"]),
        "sepTick_q": ([], ["--workload", "queue", "--no-drain-variant", "--no-fuse-tick"]),
    },
    "ring": {
        "base_q": ([], ["--workload", "queue", "--no-drain-variant"]),
        "noring_q": (["TBE_Q_NO_RING_WRITE"], ["--workload", "queue", "--no-drain-variant"]),
        "sector_q": (["TBE_Q_RING_SECTOR_AB"], ["--workload", "queue", "--no-drain-variant"]),
    },
    "qfold": {
        "base_q": ([], ["--workload", "queue", "--no-drain-variant"]),
        "r1only_q": (["TBE_Q_R1_ONLY"], ["--workload", "queue", "--no-drain-variant"]),
        "noring_q": (["TBE_Q_NO_RING_WRITE"], ["--workload", "queue", "--no-drain-variant"]),
        "r1noring_q": (["TBE_Q_R1_ONLY", "TBE_Q_NO_RING_WRITE"], ["--workload", "queue", "--no-drain-variant"]),
    },
    "hot": {
        "slots4096_z": ([], ["--workload", "zipf", "--no-host-buffer", "--no-strdir"]),
        "slots2048_z": (["TBE_HOT_SLOT_BITS=11"], ["--workload", "zipf", "--no-host-buffer", "--no-strdir"]),
        "wideall_z": (["TBE_WIDE_MIN_SHIFT=11"], ["--workload", "zipf", "--no-host-buffer", "--no-strdir"]),
        "base_u": ([], ["--workload", "uniform", "--no-host-buffer", "--no-strdir"]),
        "wideall_u": (["TBE_WIDE_MIN_SHIFT=11"], ["--workload", "uniform", "--no-host-buffer", "--no-strdir"]),
    },
    "recnt": {
        "base_u": ([], ["--workload", "uniform", "--no-host-buffer", "--no-strdir"]),
        "base_z": ([], ["--workload", "zipf", "--no-host-buffer", "--no-strdir"]),
    },
    "qshape": {
        "base_q": ([], ["--workload", "queue", "--no-drain-variant"]),
        "b1024i2w8_q": (["TBE_Q_BLOCK=1024", "TBE_Q_ITEMS=2", "TBE_Q_WAVES=8"], ["--workload", "queue", "--no-drain-variant"]),
        "b1024i1w8_q": (["TBE_Q_BLOCK=1024", "TBE_Q_ITEMS=1", "TBE_Q_WAVES=8"], ["--workload", "queue", "--no-drain-variant"]),
    },
    "histhot": {
        "base_z": ([], ["--workload", "zipf", "--no-host-buffer", "--no-strdir"]),
        "hotw8_z": (["TBE_HIST_HOT_WAVES=8"], ["--workload", "zipf", "--no-host-buffer", "--no-strdir"]),
        "hotw4_z": (["TBE_HIST_HOT_WAVES=4"], ["--workload", "zipf", "--no-host-buffer", "--no-strdir"]),
    },
    "aper": {
        "base_a": ([], ["--workload", "approx"]),
        "per8w5_a": (["TBE_A_PER=8", "TBE_A_WAVES=5"], ["--workload", "approx"]),
        "per8w4_a": (["TBE_A_PER=8", "TBE_A_WAVES=4"], ["--workload", "approx"]),
        "per6w5_a": (["TBE_A_PER=6", "TBE_A_WAVES=5"], ["--workload", "approx"]),
    },
    "afold": {
        "base_a": ([], ["--workload", "approx"]),
        "r1only_a": (["TBE_A_R1_ONLY"], ["--workload", "approx"]),
    },
    "hist": {
        "base_u": ([], ["--workload", "uniform", "--no-host-buffer", "--no-strdir"]),
        "a2w6_u": (["TBE_HIST_AHEAD=2", "TBE_HIST_WAVES=6"], ["--workload", "uniform", "--no-host-buffer", "--no-strdir"]),
        "blk2048_u": (["TBE_HIST_BLOCKS=2048"], ["--workload", "uniform", "--no-host-buffer", "--no-strdir"]),
        "blk512_u": (["TBE_HIST_BLOCKS=512"], ["--workload", "uniform", "--no-host-buffer", "--no-strdir"]),
    },
    "unscatter": {
        "base_u": ([], ["--workload", "uniform", "--no-host-buffer", "--no-strdir"]),
        "b512i16_u": (["TBE_UN_BLOCK=512", "TBE_UN_ITEMS=16"], ["--workload", "uniform", "--no-host-buffer", "--no-strdir"]),
        "b1024i16_u": (["TBE_UN_BLOCK=1024", "TBE_UN_ITEMS=16"], ["--workload", "uniform", "--no-host-buffer", "--no-strdir"]),
        "b256i16_u": (["TBE_UN_BLOCK=256", "TBE_UN_ITEMS=16"], ["--workload", "uniform", "--no-host-buffer", "--no-strdir"]),
        "b512i8_u": (["TBE_UN_BLOCK=512", "TBE_UN_ITEMS=8"], ["--workload", "uniform", "--no-host-buffer", "--no-strdir"]),
    },
    "probe": {
        "base_z": ([], ["--workload", "zipf", "--no-host-buffer", "--no-strdir"]),
        "base_u": ([], ["--workload", "uniform", "--no-host-buffer", "--no-strdir"]),
        "hist2_u": (["TBE_HIST_AHEAD=2"], ["--workload", "uniform", "--no-host-buffer", "--no-strdir"]),
    },
    "qwalk": {
        "walk_q": ([], ["--workload", "queue"]),
        "rounds_q": (["TBE_Q_TAIL_WALK=0"], ["--workload", "queue"]),
    },
    "fold": {
        "base_u": ([], ["--workload", "uniform", "--no-host-buffer", "--no-strdir"]),
        "copyonly_u": (["TBE_FOLD_COPY_ONLY"], ["--workload", "uniform", "--no-host-buffer", "--no-strdir"]),
        "r1only_u": (["TBE_FOLD_R1_ONLY"], ["--workload", "uniform", "--no-host-buffer", "--no-strdir"]),
    },
    "r04": {
        "base_u": ([], ["--workload", "uniform", "--no-host-buffer", "--no-strdir", "--no-sparse"]),
        "unall_u": ([], ["--workload", "uniform", "--no-host-buffer", "--no-strdir", "--no-sparse", "--unscatter-all"]),
        "histrec_u": ([], ["--workload", "uniform", "--no-host-buffer", "--no-strdir", "--no-sparse", "--hist-records"]),
        "s0w6_u": (["TBE_SCATTER0_WAVES=6"], ["--workload", "uniform", "--no-host-buffer", "--no-strdir", "--no-sparse"]),
        "base_z": ([], ["--workload", "zipf", "--no-host-buffer", "--no-strdir"]),
        "unall_z": ([], ["--workload", "zipf", "--no-host-buffer", "--no-strdir", "--unscatter-all"]),
        "s0w6_z": (["TBE_SCATTER0_WAVES=6"], ["--workload", "zipf", "--no-host-buffer", "--no-strdir"]),
        "histrec_z": ([], ["--workload", "zipf", "--no-host-buffer", "--no-strdir", "--hist-records"]),
        "base_q": ([], ["--workload", "queue", "--no-drain-variant"]),
        "unall_q": ([], ["--workload", "queue", "--no-drain-variant", "--unscatter-all"]),
        "base_a": ([], ["--workload", "approx"]),
        "unall_a": ([], ["--workload", "approx", "--unscatter-all"]),
    },
    "r04b": {
        "base_u": ([], ["--workload", "uniform", "--no-host-buffer", "--no-strdir", "--no-sparse"]),
        "rerank_u": ([], ["--workload", "uniform", "--no-host-buffer", "--no-strdir", "--no-sparse", "--rerank"]),
        "unall_u": ([], ["--workload", "uniform", "--no-host-buffer", "--no-strdir", "--no-sparse", "--unscatter-all"]),
        "pf768_u": (["TBE_FOLD_PREFETCH=768"], ["--workload", "uniform", "--no-host-buffer", "--no-strdir", "--no-sparse"]),
        "pf1536_u": (["TBE_FOLD_PREFETCH=1536"], ["--workload", "uniform", "--no-host-buffer", "--no-strdir", "--no-sparse"]),
        "pf384_u": (["TBE_FOLD_PREFETCH=384"], ["--workload", "uniform", "--no-host-buffer", "--no-strdir", "--no-sparse"]),
        "base_z": ([], ["--workload", "zipf", "--no-host-buffer", "--no-strdir"]),
        "rerank_z": ([], ["--workload", "zipf", "--no-host-buffer", "--no-strdir", "--rerank"]),
        "base_q": ([], ["--workload", "queue", "--no-drain-variant"]),
        "rerank_q": ([], ["--workload", "queue", "--no-drain-variant", "--rerank"]),
        "base_a": ([], ["--workload", "approx"]),
        "rerank_a": ([], ["--workload", "approx", "--rerank"]),
    },
    "r04c": {
        "base_u": ([], ["--workload", "uniform", "--no-host-buffer", "--no-strdir", "--no-sparse"]),
        "pf0_u": (["TBE_FOLD_PREFETCH=0"], ["--workload", "uniform", "--no-host-buffer", "--no-strdir", "--no-sparse"]),
        "pf192_u": (["TBE_FOLD_PREFETCH=192"], ["--workload", "uniform", "--no-host-buffer", "--no-strdir", "--no-sparse"]),
        "pf256_u": (["TBE_FOLD_PREFETCH=256"], ["--workload", "uniform", "--no-host-buffer", "--no-strdir", "--no-sparse"]),
        "pf512_u": (["TBE_FOLD_PREFETCH=512"], ["--workload", "uniform", "--no-host-buffer", "--no-strdir", "--no-sparse"]),
        "unall_u": ([], ["--workload", "uniform", "--no-host-buffer", "--no-strdir", "--no-sparse", "--unscatter-all"]),
        "base_z": ([], ["--workload", "zipf", "--no-host-buffer", "--no-strdir"]),
        "pf0_z": (["TBE_FOLD_PREFETCH=0"], ["--workload", "zipf", "--no-host-buffer", "--no-strdir"]),
        "pf256_z": (["TBE_FOLD_PREFETCH=256"], ["--workload", "zipf", "--no-host-buffer", "--no-strdir"]),
    },
    "r04d": {
        "base_u": ([], ["--workload", "uniform", "--no-host-buffer", "--no-strdir", "--no-sparse"]),
        "pfmin0_u": (["TBE_FOLD_PREFETCH_MIN=0"], ["--workload", "uniform", "--no-host-buffer", "--no-strdir", "--no-sparse"]),
        "pfmin768_u": (["TBE_FOLD_PREFETCH_MIN=768"], ["--workload", "uniform", "--no-host-buffer", "--no-strdir", "--no-sparse"]),
        "pf0_u": (["TBE_FOLD_PREFETCH=0"], ["--workload", "uniform", "--no-host-buffer", "--no-strdir", "--no-sparse"]),
        "base_z": ([], ["--workload", "zipf", "--no-host-buffer", "--no-strdir"]),
        "pfmin0_z": (["TBE_FOLD_PREFETCH_MIN=0"], ["--workload", "zipf", "--no-host-buffer", "--no-strdir"]),
        "pfmin768_z": (["TBE_FOLD_PREFETCH_MIN=768"], ["--workload", "zipf", "--no-host-buffer", "--no-strdir"]),
        "pf0_z": (["TBE_FOLD_PREFETCH=0"], ["--workload", "zipf", "--no-host-buffer", "--no-strdir"]),
    },
    "r04e": {
        "base_q": ([], ["--workload", "queue", "--no-drain-variant"]),
        "qpf384_q": (["TBE_QFOLD_PREFETCH=384"], ["--workload", "queue", "--no-drain-variant"]),
        "qpf768_q": (["TBE_QFOLD_PREFETCH=768"], ["--workload", "queue", "--no-drain-variant"]),
        "base_a": ([], ["--workload", "approx"]),
        "apf384_a": (["TBE_AFOLD_PREFETCH=384"], ["--workload", "approx"]),
        "base_z": ([], ["--workload", "zipf", "--no-host-buffer", "--no-strdir"]),
        "hotw8_z": (["TBE_HIST_HOT_WAVES=8"], ["--workload", "zipf", "--no-host-buffer", "--no-strdir"]),
        "base_u": ([], ["--workload", "uniform", "--no-host-buffer", "--no-strdir", "--no-sparse"]),
        "hotw8_u": (["TBE_HIST_HOT_WAVES=8"], ["--workload", "uniform", "--no-host-buffer", "--no-strdir", "--no-sparse"]),
    },
    "r04f": {
        "base_u": ([], ["--workload", "uniform", "--no-host-buffer", "--no-strdir", "--no-sparse"]),
        "base_z": ([], ["--workload", "zipf", "--no-host-buffer", "--no-strdir"]),
        "base_q": ([], ["--workload", "queue", "--no-drain-variant"]),
    },
    "r04g": {
        "base_u": ([], ["--workload", "uniform", "--no-host-buffer", "--no-strdir", "--no-sparse"]),
        "base_z": ([], ["--workload", "zipf", "--no-host-buffer", "--no-strdir"]),
    },
    "wipE": {
        "base_a": ([], ["--workload", "approx"]),
        "base_u": ([], ["--workload", "uniform", "--no-host-buffer", "--no-strdir", "--no-sparse"]),
        "nomemset_u": ([], ["--workload", "uniform", "--no-host-buffer", "--no-strdir", "--no-sparse"], "wip_no_memsets.patch"),
        "base_z": ([], ["--workload", "zipf", "--no-host-buffer", "--no-strdir"]),
        "nomemset_z": ([], ["--workload", "zipf", "--no-host-buffer", "--no-strdir"], "wip_no_memsets.patch"),
        "hotpipe_z": ([], ["--workload", "zipf", "--no-host-buffer", "--no-strdir"], "wip_hot_summary_pipelined.patch"),
    },
    "wipF": {
        "base_z": ([], ["--workload", "zipf", "--no-host-buffer", "--no-strdir"]),
        "hotpipe_z": ([], ["--workload", "zipf", "--no-host-buffer", "--no-strdir"], "wip_hot_summary_pipelined.patch"),
    },
    "rows12": {   # round 6: the fold's copy-only floor with 16-byte rows and with 3/4 of the bytes
        "base_u": ([], ["--workload", "uniform", "--no-host-buffer", "--no-strdir", "--no-sparse"]),
        "copyonly_u": (["TBE_FOLD_COPY_ONLY"], ["--workload", "uniform", "--no-host-buffer", "--no-strdir", "--no-sparse"]),
        "copy34_u": (["TBE_FOLD_COPY_ONLY", "TBE_COPY_ROWS=1536"], ["--workload", "uniform", "--no-host-buffer", "--no-strdir", "--no-sparse"]),
    },
    "solo": {   # round 6: the dense fold's last rounds (<= 64 pending) in one wave, or the whole workgroup
        "base_u": ([], ["--workload", "uniform", "--no-host-buffer", "--no-strdir", "--no-sparse"]),
        "solo0_u": (["TBE_WIDE_SOLO=0"], ["--workload", "uniform", "--no-host-buffer", "--no-strdir", "--no-sparse"]),
        "base_z": ([], ["--workload", "zipf", "--no-host-buffer", "--no-strdir"]),
        "solo0_z": (["TBE_WIDE_SOLO=0"], ["--workload", "zipf", "--no-host-buffer", "--no-strdir"]),
    },
    "qfloors6": {   # round 6: where config D's fold time goes
        "base_q": ([], ["--workload", "queue", "--no-host-buffer", "--no-strdir", "--no-drain-variant"]),
        "r1only_q": (["TBE_Q_R1_ONLY"], ["--workload", "queue", "--no-host-buffer", "--no-strdir", "--no-drain-variant"]),
        "noring_q": (["TBE_Q_NO_RING_WRITE"], ["--workload", "queue", "--no-host-buffer", "--no-strdir", "--no-drain-variant"]),
        "notick_q": (["TBE_Q_TICK_SKIP"], ["--workload", "queue", "--no-host-buffer", "--no-strdir", "--no-drain-variant"]),
    },
    "tickft": {   # round 6: the fused tick's row times by req_time_rel, or tb_step's 64-bit path
        "base_q": ([], ["--workload", "queue", "--no-host-buffer", "--no-strdir"]),
        "tickft0_q": (["TBE_TICK_FT=0"], ["--workload", "queue", "--no-host-buffer", "--no-strdir"]),
    },
    "relbase": {   # round 6: req_time_rel's base 2^31 us below the batch's first time, or pack_base (wb = 33 in D)
        "base_q": ([], ["--workload", "queue", "--no-host-buffer", "--no-strdir", "--no-drain-variant"]),
        "rb0_q": (["TBE_REL_BASE=0", "TBE_TICK_FT=0"], ["--workload", "queue", "--no-host-buffer", "--no-strdir", "--no-drain-variant"]),
        "base_u": ([], ["--workload", "uniform", "--no-host-buffer", "--no-strdir", "--no-sparse"]),
        "rb0_u": (["TBE_REL_BASE=0", "TBE_TICK_FT=0"], ["--workload", "uniform", "--no-host-buffer", "--no-strdir", "--no-sparse"]),
    },
    "qh32": {   # round 6: 32-bit queue headers (QueueLimit <= 1024) or 64-bit ones
        "base_q": ([], ["--workload", "queue", "--no-host-buffer", "--no-strdir", "--no-drain-variant"]),
        "qh64_q": (["TBE_QH32=0"], ["--workload", "queue", "--no-host-buffer", "--no-strdir", "--no-drain-variant"]),
    },
    "qh32b": {   # the same as bench.py --workload queue runs it (20 + 5 batches, draining variant)
        "base_q": ([], ["--workload", "queue", "--no-strdir", "--steps", "20", "--warmup", "5"]),
        "qh64_q": (["TBE_QH32=0"], ["--workload", "queue", "--no-strdir", "--steps", "20", "--warmup", "5"]),
    },
    "qvar": {   # run-to-run spread of config D's fold in the bench's schedule, with and without ring stores
        "base_q": ([], ["--workload", "queue", "--no-strdir", "--steps", "20", "--warmup", "5"]),
        "noring_q": (["TBE_Q_NO_RING_WRITE"], ["--workload", "queue", "--no-strdir", "--steps", "20", "--warmup", "5"]),
    },
    "qtail": {   # round 6: the queue fold's pending requests after round 1 by the walk (tree) or by owner rounds on the list + solo wave (patch)
        "base_q": ([], ["--workload", "queue", "--no-host-buffer", "--no-strdir", "--no-drain-variant"]),
        "rounds_q": ([], ["--workload", "queue", "--no-host-buffer", "--no-strdir", "--no-drain-variant"], "diag/q_tail_rounds.patch"),
    },
    "pf6": {   # round 6 (final tree): the dense fold's prefetch distance
        "base_u": ([], ["--workload", "uniform", "--no-host-buffer", "--no-strdir", "--no-sparse"]),
        "pf256_u": (["TBE_FOLD_PREFETCH=256"], ["--workload", "uniform", "--no-host-buffer", "--no-strdir", "--no-sparse"]),
        "pf512_u": (["TBE_FOLD_PREFETCH=512"], ["--workload", "uniform", "--no-host-buffer", "--no-strdir", "--no-sparse"]),
        "pfmin512_u": (["TBE_FOLD_PREFETCH_MIN=512"], ["--workload", "uniform", "--no-host-buffer", "--no-strdir", "--no-sparse"]),
    },
    "floors": {
        "base_u": ([], ["--workload", "uniform", "--no-host-buffer", "--no-strdir", "--no-sparse"]),
        "copyonly_u": (["TBE_FOLD_COPY_ONLY"], ["--workload", "uniform", "--no-host-buffer", "--no-strdir", "--no-sparse"]),
        "r1only_u": (["TBE_FOLD_R1_ONLY"], ["--workload", "uniform", "--no-host-buffer", "--no-strdir", "--no-sparse"]),
        "copyonly_pf0_u": (["TBE_FOLD_COPY_ONLY", "TBE_FOLD_PREFETCH=0"], ["--workload", "uniform", "--no-host-buffer", "--no-strdir", "--no-sparse"]),
    },
    "tick": {
        "skip_q": ([], ["--workload", "queue", "--no-host-buffer", "--no-strdir"]),
    },
    "hs": {
        "small_u": ([], ["--workload", "uniform", "--no-host-buffer", "--no-strdir", "--no-sparse"]),
        "small_z": ([], ["--workload", "zipf", "--no-host-buffer", "--no-strdir"]),
    },
    "seg": {
        "base_z": ([], ["--workload", "zipf", "--no-host-buffer", "--no-strdir"]),
    },
    "pipe": {
        "base_u": ([], ["--workload", "uniform", "--no-host-buffer", "--no-strdir", "--no-sparse"]),
        "nopipe_u": ([], ["--workload", "uniform", "--no-host-buffer", "--no-strdir", "--no-sparse", "--no-pipeline"]),
        "base_z": ([], ["--workload", "zipf", "--no-host-buffer", "--no-strdir"]),
        "nopipe_z": ([], ["--workload", "zipf", "--no-host-buffer", "--no-strdir", "--no-pipeline"]),
    },
    "events": {
        "base_u": ([], ["--workload", "uniform", "--no-host-buffer", "--no-strdir", "--no-sparse"]),
        "tev_u": ([], ["--workload", "uniform", "--no-host-buffer", "--no-strdir", "--no-sparse", "--timed-stage-events"]),
        "base_z": ([], ["--workload", "zipf", "--no-host-buffer", "--no-strdir"]),
        "tev_z": ([], ["--workload", "zipf", "--no-host-buffer", "--no-strdir", "--timed-stage-events"]),
    },
    "hotmin": {
        "never_u": (["TBE_HOT_SPARSE_MIN_LOG2=40"], ['--workload', 'uniform', '--no-host-buffer', '--no-strdir', '--sweep-log2', '16,18,20,22']),
        "hm20_u": (["TBE_HOT_SPARSE_MIN_LOG2=20"], ['--workload', 'uniform', '--no-host-buffer', '--no-strdir', '--sweep-log2', '16,18,20,22']),
        "never_z": (["TBE_HOT_SPARSE_MIN_LOG2=40"], ['--workload', 'uniform', '--no-host-buffer', '--no-strdir', '--sweep-log2', '16,18,20,22', '--sweep-zipf']),
        "hm20_z": (["TBE_HOT_SPARSE_MIN_LOG2=20"], ['--workload', 'uniform', '--no-host-buffer', '--no-strdir', '--sweep-log2', '16,18,20,22', '--sweep-zipf']),
    },
    "r05b": {   # the queue kind pipelined or not (its sampler variants were removed with their hook)
        "base_u": ([], ["--workload", "uniform", "--no-host-buffer", "--no-strdir", "--no-sparse"]),
        "base_z": ([], ["--workload", "zipf", "--no-host-buffer", "--no-strdir"]),
        "base_q": ([], ["--workload", "queue", "--no-host-buffer", "--no-strdir", "--no-drain-variant"]),
        "nopipe_q": ([], ["--workload", "queue", "--no-host-buffer", "--no-strdir", "--no-drain-variant", "--no-pipeline"]),
    },
    "r05q": {   # the queue kind pipelined (batch b+1's partition beside batch b's fold) or not
        "base_q": ([], ["--workload", "queue", "--no-host-buffer", "--no-strdir", "--no-drain-variant"]),
        "nopipe_q": ([], ["--workload", "queue", "--no-host-buffer", "--no-strdir", "--no-drain-variant", "--no-pipeline"]),
    },
    "uniform": {
        "base_u": ([], ["--workload", "uniform"]),
        "hist2_u": (["TBE_HIST_AHEAD=2"], ["--workload", "uniform"]),
        "wb768_u": (["TBE_WIDE_BLOCK=768", "TBE_WIDE_PER=2"], ["--workload", "uniform"]),
        "r1only_u": (["TBE_FOLD_R1_ONLY"], ["--workload", "uniform"]),
    },
}
# name: (build defines, extra bench args); ABLATE_SET picks the set (default: queue)
VARIANTS = VARIANT_SETS[os.environ.get("ABLATE_SET", "queue")]


def _build_defs(defs):
    """Compiler defines of a variant; entries "ENV:NAME=VALUE" are run-time environment
    settings of the child process instead (e.g. ENV:TBE_CU_SPLIT=4) and share the base build."""
    return [d for d in defs if not d.startswith("ENV:")]


def _env_defs(defs):
    return dict(d[4:].split("=", 1) for d in defs if d.startswith("ENV:"))


def lib_path(defs, patch=None):
    defs = _build_defs(defs)
    tag = "_".join(defs).replace("=", "") or "base"
    if patch:
        tag = os.path.splitext(os.path.basename(patch))[0] + ("_" + tag if defs else "")
    return os.path.join(OUTDIR, f"libtbe_{tag}.so")


def build_patched(m, defs, patch, out):
    """An experiment kept out of the tree's own sources: tools/<patch> (diff -ru of csrc/)
    applied to a scratch copy of the sources, built like build.py builds libtbe.so."""
    import shutil
    import tempfile
    with tempfile.TemporaryDirectory() as tmp:
        pkg = os.path.join(tmp, "distributedratelimiting.redis_amd")
        shutil.copytree(os.path.join(ROOT, "distributedratelimiting.redis_amd", "csrc"), os.path.join(pkg, "csrc"))
        shutil.copytree(os.path.join(ROOT, "include"), os.path.join(tmp, "include"))
        subprocess.run(["patch", "-p1", "-s", "-d", pkg, "-i", os.path.join(ROOT, "tools", patch)], check=True)
        srcs = [os.path.join(pkg, "csrc", os.path.basename(d)) for d in m.DEPS if d.endswith(".hip")]
        cmd = [m.hipcc()] + list(m.HIPCC_FLAGS) + [f"-D{d}" for d in defs] + [
            "-I", os.path.join(tmp, "include"), "-o", out] + srcs
        subprocess.run(cmd, check=True)


def build():
    import importlib.util
    spec = importlib.util.spec_from_file_location(
        "_b", os.path.join(ROOT, "distributedratelimiting.redis_amd", "build.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    os.makedirs(OUTDIR, exist_ok=True)
    for name, v in VARIANTS.items():
        defs, patch = _build_defs(v[0]), (v[2] if len(v) > 2 else None)
        lib = lib_path(defs, patch)
        if patch:
            build_patched(m, defs, patch, lib)
        else:
            m.build_engine(defines=defs, out=lib)   # sha256-stamped: rebuilt when sources change
        print("built", name)


def run(rounds: int, steps: int):
    results = {}
    for r in range(rounds):
        for name, v in VARIANTS.items():
            defs, extra = v[0], v[1]
            env = dict(os.environ, TBE_LIB=lib_path(defs, v[2] if len(v) > 2 else None), **_env_defs(defs))
            args = ["--steps", str(steps), "--cpu-seconds", "0"] + ([] if "--no-strdir" in extra else ["--no-host-buffer", "--no-strdir"])
            if "--warmup" not in extra:
                args += ["--warmup", "3"]
            out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args + extra, env=env,
                                 capture_output=True, text=True, timeout=300)
            line = [l for l in out.stdout.splitlines() if l.startswith("{")]
            if not line:
                print(name, "FAILED", out.stderr[-2000:])
                continue
            d = json.loads(line[0])
            results.setdefault(name, []).append(d["stage_ms_per_step"])
            print(r, name, d["ms_per_step"], d["stage_ms_per_step"],
                  (d.get("roofline") or {}).get("avg_launch_ms"), d.get("host_buffer_decisions_per_s"),
                  d.get("host_buffer_pinned_decisions_per_s"), flush=True)
            for b in d.get("batch_sweep") or []:
                print("   sweep", name, b["batch"], b["ms_per_batch"], b["latency_ms"], b["fold"][:14],
                      b["stage_ms_per_batch"], flush=True)
    print(json.dumps(results))


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--build", action="store_true")
    ap.add_argument("--run", action="store_true")
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--steps", type=int, default=5)
    a = ap.parse_args()
    if a.build:
        build()
    if a.run:
        run(a.rounds, a.steps)
