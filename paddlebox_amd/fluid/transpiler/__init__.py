"""``fluid.transpiler`` surface: collective transpilers (the ones PaddleBox
scripts use for dense data parallelism) and the pserver transpiler config
objects (accepted for API compatibility; BoxPS replaces the pserver path)."""
from . import collective  # noqa: F401
from .collective import GradAllReduce, LocalSGD, MultiThread, SingleProcessMultiThread  # noqa: F401


class DistributeTranspilerConfig:
    """Attribute bag of ``fluid.DistributeTranspilerConfig`` (pserver mode is
    not on the BoxPS path; the fields are kept so scripts that set them run)."""

    def __init__(self):
        self.slice_var_up = True
        self.split_method = None
        self.min_block_size = 8192
        self.enable_dc_asgd = False
        self.mode = "pserver"
        self.print_log = False
        self.wait_port = True
        self.runtime_split_send_recv = False
        self.sync_mode = True
        self.nccl_comm_num = 1
        self.use_hierarchical_allreduce = False
        self.hierarchical_allreduce_inter_nranks = 0
        self.collective_mode = None


class DistributeTranspiler:
    """``mode="collective"`` / ``"nccl2"`` configs dispatch to the collective
    transpilers; pserver transpilation is not provided (BoxPS is the sparse
    parameter server)."""

    def __init__(self, config: DistributeTranspilerConfig = None):
        self.config = config or DistributeTranspilerConfig()

    def transpile(self, trainer_id, program=None, pservers="127.0.0.1:6174", trainers=1, sync_mode=True,
                  startup_program=None, current_endpoint="127.0.0.1:6174"):
        from ..framework import default_main_program, default_startup_program

        program = program or default_main_program()
        startup_program = startup_program or default_startup_program()
        if self.config.mode in ("collective", "nccl2"):
            cls = LocalSGD if self.config.collective_mode == "local_sgd" else GradAllReduce
            eps = trainers if isinstance(trainers, str) else ",".join(f"127.0.0.1:{6170 + i}" for i in range(trainers))
            cls().transpile(startup_program, program, trainer_id, eps, current_endpoint)
            return
        raise NotImplementedError("pserver transpilation is not part of the BoxPS path; use BoxPSOptimizer")
