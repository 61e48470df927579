"""ctypes binding of libkge_hip.so (the C-ABI declared in include/kge_hip.h).

This is the Python-side stub a maintainer of the reference would add next to
tensorflow_codes/model.py. There is deliberately NO fallback: if the
shared library is missing or fails to load, every scoring call raises.
"""
from __future__ import annotations

import ctypes
import os
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("KGE_HIP_LIB", os.path.join(_HERE, "libkge_hip.so"))

# enum kge_fn (include/kge_hip.h)
FN_IDS = {
    "TransE": 0,
    "DistMult": 1,
    "ComplEx": 2,
    "RotatE": 3,
    "InterHT": 4,
    "pRotatE": 5,
}
# enum kge_mode — the TF reference's integer mode codes (model.py:124,203; supervisor.py:18)
HEAD_BATCH, TAIL_BATCH, SINGLE = 0, 1, 3

_c_i64 = ctypes.c_int64
_c_f = ctypes.c_float
_c_p = ctypes.c_void_p
_c_i = ctypes.c_int



class Forms(ctypes.Structure):
    """struct kge_forms (include/kge_hip.h): an explicit kernel-form choice for the _ex entry points (A/B runs
    and the bitwise cross-form tests); `forms(step_order="xcd", tile_rows=3)` builds one, the rest left to the
    library."""
    _fields_ = [("step_order", ctypes.c_int), ("xcd_phases", ctypes.c_int), ("tile_rows", ctypes.c_int),
                ("tile_q2slots", ctypes.c_int), ("tile_waves", ctypes.c_int), ("gemm_form", ctypes.c_int),
                ("transparse_form", ctypes.c_int)]


_ORDERS = {"row": 0, "xcd": 1, "tile": 2}


def forms(step_order=None, xcd_phases=0, tile_rows=0, tile_q2slots=None, tile_waves=0, gemm_form=0,
          transparse_form=0):
    so = -1 if step_order is None else (_ORDERS[step_order] if isinstance(step_order, str) else int(step_order))
    return Forms(so, int(xcd_phases), int(tile_rows or 0), -1 if tile_q2slots is None else int(tile_q2slots),
                 int(tile_waves or 0), int(gemm_form), int(transparse_form))


# exported symbol -> (restype, argtypes)
SIGNATURES = {
    "kge_abi_version": (_c_i, []),
    "kge_last_error": (ctypes.c_char_p, []),
    "kge_max_dim": (_c_i64, [_c_i]),
    "kge_step_forward_order": (_c_i, [_c_i64, _c_i64]),
    "kge_score_indexed": (
        _c_i,
        [_c_i, _c_i, _c_p, _c_i64, _c_i64, _c_p, _c_i64, _c_i64, _c_i64, _c_p, _c_p, _c_i64,
         _c_i64, _c_i64, _c_i64, _c_f, _c_f, _c_f, _c_p, _c_i64, _c_p],
    ),
    "kge_step_forward": (
        _c_i,
        [_c_i, _c_i, _c_p, _c_i64, _c_i64, _c_p, _c_i64, _c_i64, _c_i64, _c_p, _c_p, _c_i64,
         _c_i64, _c_i64, _c_i64, _c_f, _c_f, _c_f, _c_f, _c_i, _c_p, _c_i64, _c_p, _c_p, _c_p, _c_p, _c_p],
    ),
    "kge_score_indexed_ex": (
        _c_i,
        [_c_i, _c_i, _c_p, _c_i64, _c_i64, _c_p, _c_i64, _c_i64, _c_i64, _c_p, _c_p, _c_i64,
         _c_i64, _c_i64, _c_i64, _c_f, _c_f, _c_f, _c_p, _c_i64, _c_p, _c_p],
    ),
    "kge_step_forward_ex": (
        _c_i,
        [_c_i, _c_i, _c_p, _c_i64, _c_i64, _c_p, _c_i64, _c_i64, _c_i64, _c_p, _c_p, _c_i64,
         _c_i64, _c_i64, _c_i64, _c_f, _c_f, _c_f, _c_f, _c_i, _c_p, _c_i64, _c_p, _c_p, _c_p, _c_p, _c_p, _c_p],
    ),
    "kge_step_plan_size": (_c_i64, [_c_i, _c_i64, _c_i64, _c_i64, _c_i64, _c_i64, _c_i64, _c_i64, _c_i64]),
    "kge_step_plan": (
        _c_i, [_c_i, _c_i, _c_i64, _c_i64, _c_i64, _c_i64, _c_i64, _c_p, _c_p, _c_i64, _c_i64, _c_i64, _c_i64, _c_p,
               _c_p]),
    "kge_step_forward_planned": (
        _c_i,
        [_c_i, _c_i, _c_p, _c_i64, _c_i64, _c_p, _c_i64, _c_i64, _c_i64, _c_i64, _c_i64, _c_i64, _c_f, _c_f, _c_f,
         _c_f, _c_i, _c_p, _c_p, _c_p, _c_i64, _c_i, _c_p, _c_p, _c_i64, _c_p, _c_p, _c_p, _c_p],
    ),
    "kge_step_planner_create": (
        _c_i, [_c_p, _c_i, _c_p, _c_i64, _c_i64, _c_p, _c_i64, _c_i64, _c_i64, _c_i64, _c_i64, _c_i64, _c_f, _c_f, _c_f,
               _c_f, _c_i, _c_p, _c_p, _c_i64, _c_p]),
    "kge_step_planner_set_modulus": (_c_i, [_c_p, _c_f]),
    "kge_step_planner_set_sweep": (_c_i, [_c_p, _c_i]),
    "kge_step_planner_plan": (_c_i, [_c_p, _c_p, _c_p, _c_i64, _c_i]),
    "kge_step_planner_step": (_c_i, [_c_p, _c_p, _c_p, _c_i64, _c_i, _c_p, _c_p, _c_p, _c_p]),
    "kge_step_planner_destroy": (_c_i, [_c_p]),
    "kge_step_finish": (
        _c_i,
        [_c_i, _c_p, _c_i64, _c_i64, _c_p, _c_i64, _c_i64, _c_i64, _c_p, _c_i64, _c_i64,
         _c_f, _c_f, _c_f, _c_p, _c_i64, _c_i64, _c_f, _c_i, _c_p, _c_p, _c_p, _c_p],
    ),
    "kge_score_sharded": (
        _c_i,
        [_c_i, _c_i, _c_p, _c_i64, _c_p, _c_i64, _c_i64, _c_i64, _c_p, _c_i64, _c_i64, _c_i64,
         _c_p, _c_p, _c_i64, _c_i64, _c_i64, _c_i64, _c_f, _c_f, _c_f, _c_p, _c_i64, _c_p],
    ),
    "kge_gather_rows": (
        _c_i, [_c_p, _c_i64, _c_i64, _c_i64, _c_p, _c_i64, _c_i64, _c_i64, _c_p, _c_i64, _c_p]),
    "kge_build_id": (ctypes.c_char_p, []),
    "kge_source_hash": (ctypes.c_char_p, []),
    "kge_shard_plan": (
        _c_i, [_c_p, _c_p, _c_i64, _c_i64, _c_i64, _c_i64, _c_i, _c_i, _c_i, _c_i, _c_i, _c_p, _c_p, _c_p, _c_p, _c_p,
               _c_p, _c_p, _c_p]),
    "kge_shard_gather_queries": (
        _c_i, [_c_p, _c_i64, _c_i64, _c_i64, _c_p, _c_i64, _c_i, _c_i, _c_i64, _c_i, _c_i, _c_i, _c_i, _c_p, _c_p,
               _c_p, _c_p, _c_p, _c_p]),
    "kge_shard_score": (
        _c_i,
        [_c_i, _c_i, _c_p, _c_i64, _c_i64, _c_p, _c_p, _c_i64, _c_i64, _c_i64, _c_p, _c_i64, _c_i64, _c_i64,
         _c_p, _c_i64, _c_i64, _c_i64, _c_f, _c_f, _c_f, _c_p, _c_p, _c_p, _c_p, _c_p, _c_i, _c_i, _c_i64,
         _c_i64, _c_p, _c_p],
    ),
    "kge_shard_finish": (
        _c_i, [_c_p, _c_p, _c_p, _c_p, _c_p, _c_i64, _c_i64, _c_i64, _c_i64, _c_i, _c_i, _c_i, _c_f, _c_i, _c_p,
               _c_i64, _c_p, _c_p, _c_p, _c_p]),
    "kge_comm_unique_id": (_c_i, [_c_p]),
    "kge_comm_loopback_group": (_c_p, [_c_i]),
    "kge_comm_loopback_group_destroy": (_c_i, [_c_p]),
    "kge_comm_loopback_init": (_c_i, [_c_p, _c_p, _c_i]),
    "kge_comm_init": (_c_i, [_c_p, _c_p, _c_i, _c_i]),
    "kge_comm_destroy": (_c_i, [_c_p]),
    "kge_comm_all_to_allv": (_c_i, [_c_p, _c_p, _c_p, _c_p, _c_p, _c_p]),
    "kge_comm_all_reduce_sum": (_c_i, [_c_p, _c_p, _c_i64, _c_p]),
    "kge_shard_exec_workspace_size": (_c_i64, [_c_i64, _c_i64, _c_i64, _c_i, _c_i]),
    "kge_shard_exec_host_ints": (_c_i64, [_c_i, _c_i]),
    "kge_shard_exec_create": (
        _c_i, [_c_p, _c_p, _c_i, _c_i, _c_i64, _c_i64, _c_i64, _c_i64, _c_i64, _c_i64, _c_i, _c_i, _c_i, _c_p, _c_i64,
               _c_p, _c_i64]),
    "kge_shard_exec_destroy": (_c_i, [_c_p]),
    "kge_shard_exec_host_wait_us": (ctypes.c_double, [_c_p, _c_i]),
    "kge_shard_exec_timings": (_c_i, [_c_p, _c_p, _c_i]),
    "kge_comm_size": (_c_i, [_c_p]),
    "kge_shard_exec_plan": (_c_i, [_c_p, _c_p, _c_p, _c_i64, _c_i, _c_p]),
    "kge_shard_exec_step": (
        _c_i, [_c_p, _c_p, _c_i64, _c_i64, _c_p, _c_i64, _c_i64, _c_i64, _c_p, _c_p, _c_i64, _c_i, _c_f, _c_f, _c_f,
               _c_f, _c_i, _c_p, _c_p, _c_i, _c_p, _c_i64, _c_p, _c_p, _c_p, _c_p]),
    "kge_eval_query": (
        _c_i, [_c_i, _c_i, _c_p, _c_i64, _c_i64, _c_p, _c_i64, _c_i64, _c_p, _c_i64, _c_i64, _c_p, _c_i64, _c_p]),
    "kge_eval_query_planes": (
        _c_i, [_c_i, _c_i, _c_p, _c_i64, _c_i64, _c_p, _c_i64, _c_i64, _c_p, _c_i64, _c_i64, _c_p, _c_i64, _c_p]),
    "kge_gemm_nt": (_c_i, [_c_p, _c_i64, _c_p, _c_i64, _c_p, _c_i64, _c_i64, _c_i64, _c_i64, _c_p]),
    "kge_gemm_nt_bf16x3": (_c_i, [_c_p, _c_i64, _c_p, _c_i64, _c_p, _c_i64, _c_i64, _c_i64, _c_i64, _c_p]),
    "kge_gemm_nt_bf16x3_ex": (_c_i, [_c_p, _c_i64, _c_p, _c_i64, _c_p, _c_i64, _c_i64, _c_i64, _c_i64, _c_p, _c_p]),
    "kge_split_bf16x3_bytes": (_c_i64, [_c_i64, _c_i64]),
    "kge_split_bf16x3": (_c_i, [_c_p, _c_i64, _c_i64, _c_i64, _c_p, _c_i64, _c_p]),
    "kge_gemm_nt_bf16x3_planes": (_c_i, [_c_p, _c_i64, _c_p, _c_i64, _c_i64, _c_p, _c_i64, _c_i64, _c_i64, _c_p]),
    "kge_eval_rank_planes_workspace_size": (_c_i64, [_c_i64, _c_i64]),
    "kge_eval_rank_planes": (_c_i, [_c_p, _c_i64, _c_p, _c_i64, _c_i64, _c_i64, _c_i64, _c_p, _c_p, _c_p, _c_i64, _c_p,
                                    _c_p, ctypes.c_size_t, _c_p]),
    "kge_eval_rank_planes_ex": (_c_i, [_c_p, _c_i64, _c_p, _c_i64, _c_i64, _c_i64, _c_i64, _c_p, _c_p, _c_p, _c_i64,
                                       _c_p, _c_p, ctypes.c_size_t, _c_p, _c_p]),
    "kge_eval_rank_planes_phases": (_c_i, [_c_p, _c_i64, _c_p, _c_i64, _c_i64, _c_i64, _c_i64, _c_p, _c_p, _c_p,
                                           _c_i64, _c_p, _c_p, ctypes.c_size_t, _c_i, _c_p, _c_p]),
    "kge_gemm_nt_bf16x3_planes_ex": (_c_i, [_c_p, _c_i64, _c_p, _c_i64, _c_i64, _c_p, _c_i64, _c_i64, _c_i64, _c_p,
                                            _c_p]),
    "kge_rank_filtered": (_c_i, [_c_p, _c_i64, _c_i64, _c_i64, _c_p, _c_p, _c_p, _c_p, _c_p]),
    "kge_score_dense": (
        _c_i,
        [_c_i, _c_i, _c_p, _c_i64, _c_p, _c_i64, _c_i64, _c_p, _c_i64, _c_i64, _c_i64, _c_i64,
         _c_f, _c_f, _c_f, _c_p, _c_i64, _c_p],
    ),
    "kge_score_dense_bwd": (
        _c_i,
        [_c_i, _c_i, _c_p, _c_i64, _c_p, _c_i64, _c_i64, _c_p, _c_i64, _c_i64, _c_i64, _c_i64,
         _c_f, _c_f, _c_f, _c_p, _c_i64, _c_p, _c_p, _c_p, _c_p, _c_p],
    ),
    "kge_neg_reduce": (_c_i, [_c_p, _c_i64, _c_i64, _c_i64, _c_f, _c_i, _c_p, _c_p]),
    "kge_neg_reduce_bwd": (
        _c_i, [_c_p, _c_i64, _c_i64, _c_i64, _c_f, _c_i, _c_i, _c_p, _c_p, _c_i64, _c_p]),
    "kge_log_sigmoid": (_c_i, [_c_p, _c_i64, _c_p, _c_p]),
    "kge_log_sigmoid_bwd": (_c_i, [_c_p, _c_p, _c_i64, _c_p, _c_p]),
    "kge_adam_update": (
        _c_i, [_c_p, _c_p, _c_p, _c_p, _c_i64, _c_f, _c_f, _c_f, _c_f, _c_i64, _c_i, _c_i, _c_p]),
    "kge_step_backward_workspace_size": (_c_i64, [_c_i, _c_i64, _c_i64, _c_i64, _c_i64]),
    "kge_step_backward": (
        _c_i,
        [_c_i, _c_i, _c_p, _c_i64, _c_i64, _c_p, _c_i64, _c_i64, _c_i64, _c_p, _c_p, _c_i64,
         _c_i64, _c_i64, _c_i64, _c_f, _c_f, _c_f, _c_f, _c_i, _c_i, _c_p, _c_i64, _c_p, _c_p, _c_p,
         _c_p, _c_p, _c_p, _c_p, _c_p, _c_i64, _c_p],
    ),
    "kge_step_backward_adam_workspace_size": (_c_i64, [_c_i, _c_i64, _c_i64, _c_i64, _c_i64, _c_i64, _c_i64]),
    "kge_step_backward_adam": (
        _c_i,
        [_c_i, _c_i, _c_p, _c_i64, _c_i64, _c_p, _c_i64, _c_i64, _c_i64, _c_p, _c_p, _c_i64,
         _c_i64, _c_i64, _c_i64, _c_f, _c_f, _c_p, _c_f, _c_f, _c_i, _c_i, _c_p, _c_i64, _c_p, _c_p, _c_p,
         _c_p, _c_p, _c_p, _c_p, _c_p, _c_p, _c_f, _c_f, _c_f, _c_f, _c_i64, _c_i, _c_p, _c_p, _c_i64, _c_p],
    ),
    "kge_train_step_workspace_size": (_c_i64, [_c_i, _c_i64, _c_i64, _c_i64, _c_i64, _c_i64, _c_i64]),
    "kge_train_step": (
        _c_i,
        [_c_i, _c_i, _c_p, _c_i64, _c_i64, _c_p, _c_i64, _c_i64, _c_i64, _c_p, _c_p, _c_i64,
         _c_i64, _c_i64, _c_i64, _c_f, _c_f, _c_f, _c_i, _c_i, _c_p, _c_p, _c_p, _c_p, _c_p,
         _c_p, _c_p, _c_p, _c_p, _c_f, _c_f, _c_f, _c_f, _c_i64, _c_i, _c_p, _c_i64, _c_p],
    ),
    "kge_sampler_create": (_c_p, [_c_p, _c_i64, _c_i64, _c_i64, _c_i64, _c_i]),
    "kge_sampler_seed": (_c_i, [_c_p, ctypes.c_uint32]),
    "kge_sampler_get": (_c_i, [_c_p, _c_p, _c_i64, _c_p, _c_p, _c_p]),
    "kge_sampler_destroy": (None, [_c_p]),
    "kge_transparse_score": (_c_i, [_c_i, _c_p, _c_i64, _c_i64, _c_p, _c_i64, _c_i64, _c_p, _c_p, _c_p, _c_p, _c_i64,
                                    _c_i64, _c_i64, _c_i64, _c_f, _c_p, _c_i64, _c_p, _c_p]),
    "kge_transparse_score_workspace_size": (ctypes.c_size_t, [_c_i, _c_i64, _c_i64, _c_i64]),
    "kge_transparse_score_ex": (_c_i, [_c_i, _c_p, _c_i64, _c_i64, _c_p, _c_i64, _c_i64, _c_p, _c_p, _c_p, _c_p,
                                       _c_i64, _c_i64, _c_i64, _c_i64, _c_f, _c_p, _c_i64, _c_p, _c_p, _c_p,
                                       ctypes.c_size_t, _c_p]),
    "kge_transparse_step_workspace_size": (ctypes.c_size_t, [_c_i64, _c_i64, _c_i64]),
    # (mode, ent, nent, ent_ld, rel, nrel, rel_ld, W, mask, pos, neg, neg_ld, B, N, d, gamma, T, adversarial,
    #  neg_scores, ns_ld, out_neg, pos_scores, out_pos, workspace, workspace_bytes, stream)
    "kge_transparse_step_forward": (_c_i, [_c_i, _c_p, _c_i64, _c_i64, _c_p, _c_i64, _c_i64, _c_p, _c_p, _c_p, _c_p,
                                           _c_i64, _c_i64, _c_i64, _c_i64, _c_f, _c_f, _c_i, _c_p, _c_i64, _c_p, _c_p,
                                           _c_p, _c_p, ctypes.c_size_t, _c_p]),
    "kge_transparse_bwd_workspace_size": (ctypes.c_size_t, [_c_i, _c_i64, _c_i64, _c_i64, _c_i64, _c_i64]),
    "kge_transparse_premul": (_c_i, [_c_p, _c_p, _c_i64, _c_p, _c_p]),
    "kge_transparse_score_bwd": (_c_i, [_c_i, _c_p, _c_i64, _c_i64, _c_p, _c_i64, _c_i64, _c_p, _c_p, _c_p, _c_p, _c_p,
                                        _c_i64, _c_i64, _c_i64, _c_i64, _c_p, _c_p, _c_i64, _c_p, _c_p, _c_p, _c_p,
                                        ctypes.c_size_t, _c_p]),
    "kge_step_loss": (_c_i, [_c_p, _c_p, _c_p, _c_i64, _c_p, _c_p, _c_p]),
    "kge_crc32c": (ctypes.c_uint32, [_c_p, _c_i64]),
    "kge_tfrecord_open": (_c_p, [_c_p, _c_i64, _c_i]),
    "kge_tfrecord_next": (_c_i, [_c_p, _c_p]),
    "kge_tfrecord_copy": (_c_i, [_c_p, _c_p, _c_p, _c_p, _c_p]),
    "kge_tfrecord_rewind": (_c_i, [_c_p]),
    "kge_tfrecord_close": (None, [_c_p]),
    "kge_tfrecord_writer_open": (_c_p, [ctypes.c_char_p]),
    "kge_tfrecord_write_example": (_c_i, [_c_p, _c_p, _c_i64, _c_p, _c_i64, _c_p, _c_i64, _c_p, _c_i64]),
    "kge_tfrecord_writer_close": (_c_i, [_c_p]),
    "kge_score_bwd_workspace_size": (_c_i64, [_c_i, _c_i, _c_i64, _c_i64, _c_i64]),
    "kge_score_indexed_bwd": (
        _c_i,
        [_c_i, _c_i, _c_p, _c_i64, _c_i64, _c_p, _c_i64, _c_i64, _c_i64, _c_p, _c_p, _c_i64,
         _c_i64, _c_i64, _c_i64, _c_f, _c_f, _c_f, _c_p, _c_i64, _c_p, _c_p, _c_p, _c_p, _c_p],
    ),
    "kge_shard_nq": (_c_i, [_c_i]),
    "kge_shard_train_workspace_size": (_c_i64, [_c_i, _c_i64, _c_i64, _c_i64, _c_i64, _c_i64, _c_i64]),
    "kge_shard_train_forward": (_c_i, [_c_i, _c_i, _c_p, _c_i64, _c_i64, _c_i64, _c_p, _c_p, _c_i64, _c_p, _c_i64, _c_i64, _c_i64, _c_p, _c_p, _c_i64, _c_i64, _c_i64, _c_i64, _c_i64, _c_i, _c_i, _c_f, _c_f, _c_f, _c_i, _c_i, _c_p, _c_p, _c_p, _c_p, _c_i64, _c_p]),
    "kge_shard_train_combine": (_c_i, [_c_i, _c_i, _c_p, _c_i64, _c_i64, _c_i64, _c_p, _c_p, _c_i64, _c_p, _c_i64, _c_i64, _c_i64, _c_p, _c_p, _c_i64, _c_i64, _c_i64, _c_i64, _c_i64, _c_i, _c_i, _c_f, _c_f, _c_f, _c_i, _c_i, _c_p, _c_p, _c_p, _c_p, _c_p, _c_p, _c_p, _c_i64, _c_p]),
    "kge_shard_train_backward": (_c_i, [_c_i, _c_i, _c_p, _c_i64, _c_i64, _c_i64, _c_p, _c_p, _c_i64, _c_p, _c_i64, _c_i64, _c_i64, _c_p, _c_p, _c_i64, _c_i64, _c_i64, _c_i64, _c_i64, _c_i, _c_i, _c_f, _c_f, _c_f, _c_i, _c_i, _c_p, _c_p, _c_p, _c_p, _c_p, _c_p, _c_p, _c_p, _c_f, _c_f, _c_f, _c_f, _c_i64, _c_i, _c_p, _c_i64, _c_p]),
}

_lock = threading.Lock()
_lib = None


class KGEHipError(RuntimeError):
    """A libkge_hip.so entry point returned a non-zero status (message from kge_last_error)."""


def load(path: str | None = None):
    """Load libkge_hip.so once. torch is imported first so that the library binds to the HIP
    runtime torch already loaded (same SONAME libamdhip64.so.7) and shares its streams."""
    global _lib
    with _lock:
        if _lib is not None and path is None:
            return _lib
        import torch  # noqa: F401  (HIP runtime first)

        p = path or LIB_PATH
        if not os.path.exists(p):
            raise KGEHipError(
                f"libkge_hip.so not found at {p}: build it with `make -C {_HERE}` or "
                "`python -c 'import __graft_entry__ as g; g.build()'` (there is no CPU fallback)")
        lib = ctypes.CDLL(p)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        if lib.kge_abi_version() != 1:
            raise KGEHipError(f"ABI version mismatch: {lib.kge_abi_version()} != 1")
        if path is None:
            _lib = lib
        return lib


def source_hash(root: str | None = None) -> str:
    """The sha256 (16 hex digits) of the sources libkge_hip.so is built from, by the Makefile's recipe
    (make's byte-order sort of: include/kge_hip.h by absolute path, Makefile, csrc/*.{hip,cpp,h}). It
    equals the loaded library's kge_source_hash() exactly when the library was built from this tree."""
    import glob
    import hashlib

    pkg = root or _HERE
    top = os.path.dirname(os.path.abspath(pkg))
    rel = ["Makefile"] + [os.path.relpath(p, pkg) for ext in ("hip", "cpp", "h")
                          for p in glob.glob(os.path.join(pkg, "csrc", "*." + ext))]
    files = [os.path.join(top, "include", "kge_hip.h")] + [os.path.join(pkg, r) for r in sorted(rel)]
    h = hashlib.sha256()
    for f in files:
        with open(f, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


def build_id() -> dict:
    """Provenance of the loaded library: its build id string and source hash, and whether that hash
    matches the sources in this tree."""
    lib = load()
    sh = lib.kge_source_hash().decode()
    return {"build_id": lib.kge_build_id().decode(), "source_hash": sh, "source_hash_matches_tree": sh == source_hash()}


def check(rc: int, what: str) -> None:
    if rc != 0:
        msg = load().kge_last_error().decode(errors="replace")
        raise KGEHipError(f"{what} failed (rc={rc}): {msg}")
