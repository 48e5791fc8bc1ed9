// PaddleBox-compatible flag set (names/defaults from reference
// paddle/fluid/platform/flags.cc:926-1013, fw/boxps_worker.cc:43-58,
// fw/data_set.cc:42, fw/fleet/metrics.cc:29).  Settable via FLAGS_<name> env
// vars or paddlebox_amd.utils.flags.set_flags().
#include "runtime.h"

namespace pbx {

void register_default_flags() {
  auto& f = Flags::ins();
  f.define("enable_pullpush_dedup_keys", "true", "dedup keys before pull/push");
  f.define("enable_pull_box_padding_zero", "true", "zero [1,size] output for an empty slot");
  f.define("padbox_record_pool_max_size", "2000000", "SlotRecord pool cap");
  f.define("padbox_slotrecord_extend_dim", "2", "extra floats per record (PCOC q values)");
  f.define("padbox_slotpool_thread_num", "1", "slot pool release threads");
  f.define("padbox_dataset_shuffle_thread_num", "20", "dataset shuffle threads");
  f.define("padbox_dataset_merge_thread_num", "20", "dataset merge threads");
  f.define("padbox_dataset_disable_shuffle", "false", "disable inter-node shuffle");
  f.define("padbox_dataset_disable_polling", "false", "disable rank-strided filelist");
  f.define("padbox_dataset_enable_unrollinstance", "false", "call parser UnrollInstance after load");
  f.define("padbox_auc_runner_mode", "false", "AucRunner slot-importance mode");
  f.define("padbox_disable_ins_shuffle", "false", "disable per-pass instance shuffle");
  f.define("padbox_enable_gc", "true", "eager tensor release in the worker");
  f.define("padbox_enable_print_op_debug", "false", "log each op");
  f.define("enable_print_dump_field_debug", "false", "dump debug");
  f.define("enable_print_dump_info_debug", "false", "dump debug");
  f.define("padbox_enable_sharding_stage", "false", "optimizer-state sharding stage");
  f.define("padbox_dump_debug_lineid", "", "line id to trace in dumps");
  f.define("use_gpu_replica_cache", "false", "enable the replicated GPU cache");
  f.define("gpu_replica_cache_dim", "8", "replica cache dim");
  f.define("fix_dayid", "false", "do not subtract the UTC+8 offset in make_day_id");
  f.define("enable_binding_train_cpu", "true", "pin worker threads");
  f.define("enable_sync_dense_moment", "false", "also sync Adam moments");
  f.define("enable_dense_nccl_barrier", "false", "barrier around dense sync timing");
  f.define("enable_shuffle_by_searchid", "false", "shuffle records by search id");
  f.define("enbale_slotpool_auto_clear", "false", "slot pool auto clear");
  f.define("enable_slotpool_wait_release", "false", "wait slot pool release");
  f.define("enable_slotrecord_reset_shrink", "false", "shrink records on reset");
  f.define("enable_ins_parser_file", "false", "parser whole-file mode");
  f.define("enable_ins_parser_add_file_path", "false", "append file path to ins id");
  f.define("lineid_have_extend_info", "false", "dump format");
  f.define("dump_filed_same_as_aibox", "false", "dump format");
  f.define("enable_dump_main_program", "false", "write per-device op list");
  f.define("enable_debug_print_metrics_info", "false", "log metric internals");
  f.define("check_nan_inf", "false", "per-batch nan/inf check + scope dump + abort");
  f.define("enable_force_hbm_recyle", "false", "release HBM pool at EndPass");
  f.define("enable_force_mem_recyle", "false", "force host memory release / disable slot pool");
  f.define("padbox_max_keys_per_batch", "0", "override engine key capacity (0 = auto)");
  f.define("padbox_device_pass", "true", "keep the pass's record store in HBM and assemble batches on the GPU");
  f.define("padbox_device_pass_max_gb", "64", "largest pass (GB of HBM) kept device-resident");
  f.define("padbox_fc_precision", "fp32", "fluid fc chains: fp32 (exact, reference) or bf16 MFMA operands");
  f.define("padbox_train_steps_per_graph", "0", "graphed train loop: training steps per HIP graph (0 = auto)");
  f.define("padbox_pipelined_front", "true", "graphed train loop: pool the next batch after the sparse push");
}

}  // namespace pbx
