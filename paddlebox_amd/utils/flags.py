"""FLAGS_* registry (PaddleBox flag set, reference platform/flags.cc:926-1013).

Backed by the native registry in ``_pbx_host`` when built (so C++ components
see the same values); otherwise a Python dict seeded from the environment.

Flags accepted for compatibility whose mechanism does not exist in this
design (documented, not silently ignored):

* ``enable_pullpush_dedup_keys`` -- live: false selects the single-shard GPU step
  without a key dedup (per-occurrence probe + leader-elected push merge).
* ``padbox_record_pool_max_size``, ``padbox_slotpool_thread_num``,
  ``enbale_slotpool_auto_clear``, ``enable_slotpool_wait_release``,
  ``enable_slotrecord_reset_shrink`` -- there is no SlotRecord object pool:
  the pass lives in a columnar CSR store (``csrc/host/slot_dataset.h``).
* ``padbox_enable_gc`` -- intermediate tensors are freed by reference
  counting / the HIP graph's memory pool.
* ``enable_pull_box_padding_zero`` -- an empty slot always pools to zeros
  (the fused pull writes every output row), the flag's ``true`` behaviour.
* ``padbox_auc_runner_mode`` -- AucRunner mode is entered by
  ``BoxWrapper.initialize_auc_runner`` (``auc_runner_mode()`` reports it).
* ``padbox_enable_sharding_stage`` -- optimizer-state sharding is chosen by
  the fleet strategy / ``ShardedFlatAdam``.
* ``padbox_fc_precision`` (this engine's, not the reference's) -- operand
  precision of the fluid ``fc`` chains the lowering fuses: ``fp32`` (default,
  the reference fc precision: the exact-fp32 MFMA tower, or library fp32
  GEMMs for chains the tower does not take), ``fp32x3`` (fp32 storage and
  accumulation, every product as three bf16 MFMAs on hi + lo halves --
  finer than the TF32 math the reference's fp32 fc runs on by default,
  phi/backends/gpu/gpu_context.cc:65-67,580-588; the bench headline) or
  ``bf16`` (bf16 MFMA operands, fp32 accumulate).
* ``padbox_train_steps_per_graph`` / ``padbox_pipelined_front`` (this
  engine's) -- the graphed ``train_from_dataset`` loop: training steps per
  captured HIP graph (0 = auto) and the pipelined front (each step pools the
  next batch right after its sparse push).
* ``padbox_dataset_merge_thread_num`` -- feed-pass keys are registered by
  the loader threads themselves (KeyAgent); their count comes from
  ``set_thread``.  (``padbox_dataset_shuffle_thread_num`` is live: the
  global shuffle's serializer threads.)
"""
from __future__ import annotations

import os
from typing import Dict

_DEFAULTS: Dict[str, str] = {
    "enable_pullpush_dedup_keys": "true",
    "enable_pull_box_padding_zero": "true",
    "padbox_record_pool_max_size": "2000000",
    "padbox_slotrecord_extend_dim": "2",
    "padbox_slotpool_thread_num": "1",
    "padbox_dataset_shuffle_thread_num": "20",
    "padbox_dataset_merge_thread_num": "20",
    "padbox_dataset_disable_shuffle": "false",
    "padbox_dataset_disable_polling": "false",
    "padbox_dataset_enable_unrollinstance": "false",
    "padbox_auc_runner_mode": "false",
    "padbox_disable_ins_shuffle": "false",
    "padbox_enable_gc": "true",
    "padbox_enable_print_op_debug": "false",
    "enable_print_dump_field_debug": "false",
    "enable_print_dump_info_debug": "false",
    "padbox_enable_sharding_stage": "false",
    "padbox_dump_debug_lineid": "",
    "use_gpu_replica_cache": "false",
    "gpu_replica_cache_dim": "8",
    "fix_dayid": "false",
    "enable_binding_train_cpu": "true",
    "enable_sync_dense_moment": "false",
    "enable_dense_nccl_barrier": "false",
    "enable_shuffle_by_searchid": "false",
    "enbale_slotpool_auto_clear": "false",
    "enable_slotpool_wait_release": "false",
    "enable_slotrecord_reset_shrink": "false",
    "enable_ins_parser_file": "false",
    "enable_ins_parser_add_file_path": "false",
    "lineid_have_extend_info": "false",
    "dump_filed_same_as_aibox": "false",
    "enable_dump_main_program": "false",
    "enable_debug_print_metrics_info": "false",
    "check_nan_inf": "false",
    "enable_force_hbm_recyle": "false",
    "enable_force_mem_recyle": "false",
    "padbox_max_keys_per_batch": "0",
    "padbox_device_pass": "true",
    "padbox_device_pass_max_gb": "64",
    "padbox_fc_precision": "fp32",
    "padbox_train_steps_per_graph": "0",
    "padbox_pipelined_front": "true",
}
_py: Dict[str, str] = {k: os.environ.get("FLAGS_" + k, v) for k, v in _DEFAULTS.items()}


def _native():
    try:
        from .. import _native as n

        return n.host() if n.host_available() else None
    except Exception:  # pragma: no cover
        return None


def get(name: str) -> str:
    h = _native()
    if h is not None:
        return h.flag_get(name)
    return _py[name]


def get_bool(name: str) -> bool:
    return get(name).lower() in ("1", "true", "yes")


def get_int(name: str) -> int:
    return int(get(name))


def set_flags(d: Dict[str, object]):
    """paddle.set_flags({'FLAGS_x': v}) equivalent (prefix optional)."""
    h = _native()
    for k, v in d.items():
        k = k[6:] if k.startswith("FLAGS_") else k
        sv = str(v).lower() if isinstance(v, bool) else str(v)
        if k not in _py:
            raise KeyError(f"unknown flag {k}")
        if h is not None:
            h.flag_set(k, sv)
        if k not in _py:
            raise KeyError(f"unknown flag {k}")
        _py[k] = sv


def get_flags(names) -> Dict[str, str]:
    if isinstance(names, str):
        names = [names]
    return {("FLAGS_" + n if not n.startswith("FLAGS_") else n): get(n.replace("FLAGS_", "", 1)) for n in names}


def all_flags() -> Dict[str, str]:
    h = _native()
    return dict(h.flags_all()) if h is not None else dict(_py)
