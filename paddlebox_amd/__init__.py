"""paddlebox_amd -- a MI355X-native large-scale sparse CTR training engine with
the capabilities of PaddleBox (BoxPS GPU parameter server, fused CTR ops,
pass-based slot datasets, paddle.fluid-compatible API).

Subpackages
  ps/        sparse parameter server: GPU cuckoo table, CPU table, engine,
             pass lifecycle, tiers, checkpoints
  ops/       CTR operators (HIP kernels + fp32 references)
  data/      slot records, parsers, datasets, synthetic Criteo generator
  models/    DeepFM, Wide&Deep, DCN-V2
  parallel/  RCCL process groups, key all-to-all, dense sync, sharding
  metrics/   AUC family calculators and the metric registry
  runtime/   trainer / worker / dump / profiling timers
  fluid/     paddle.fluid-compatible front-end
  utils/     flags, timers, logging, day ids
"""
__version__ = "0.1.0"
