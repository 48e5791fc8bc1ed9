from .nn import *  # noqa: F401,F403
from .nn import (_elementwise, _pull_box_sparse, _pull_cache_value, _store_q_value,  # noqa: F401
                 continuous_value_model, data, data_norm, fc, lookup_input, masked_data_norm, pull_box_sparse)
from . import collective  # noqa: F401,E402
