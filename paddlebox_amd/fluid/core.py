"""``paddle.fluid.core`` objects used by PaddleBox scripts.

``BoxWrapper``, ``BoxPS`` (the BoxHelper pass driver) and ``BoxFileMgr``
mirror the pybind surface in ``paddle/fluid/pybind/box_helper_py.cc:37-216``.
"""
from __future__ import annotations

import threading
from typing import Optional

from ..ps.box_wrapper import BoxWrapper as _BoxWrapper
from ..utils.dayid import make_day_id
from ..utils.fs import BoxFileMgr  # noqa: F401
from .framework import (CPUPlace, CUDAPinnedPlace, CUDAPlace, LoDTensor, Scope,  # noqa: F401
                        is_compiled_with_cuda)


def BoxWrapper(embedx_dim: int = 8, expand_embed_dim: int = 0, feature_type: int = 0,  # noqa: N802
               pull_embedx_scale: float = 1.0, **kw) -> _BoxWrapper:
    """Handle to the process-wide BoxWrapper (created on first call, like
    ``BoxWrapper::SetInstance``; later calls return the same instance)."""
    inst = _BoxWrapper._instance
    if inst is None or kw.get("new", False):
        kw.pop("new", None)
        inst = _BoxWrapper(embedx_dim, expand_embed_dim, feature_type, pull_embedx_scale, **kw)
    return inst


class BoxPS:
    """BoxHelper (``fw/fleet/box_wrapper.h:1043-1295``): drives one dataset
    through the pass lifecycle.

    * ``read_ins_into_memory`` / ``load_into_memory``: BeginFeedPass ->
      load -> key registration -> EndFeedPass (``ReadData2Memory``);
    * ``preload_into_memory`` + ``wait_feed_pass_done``: the same, with the
      file loading overlapped with training of the previous pass;
    * ``begin_pass`` / ``end_pass``: stage the pass working set into HBM /
      write it back.
    """

    def __init__(self, dataset):
        self.dataset = dataset
        self.box = _BoxWrapper.get_instance()
        dataset.box = self.box
        self._date: Optional[str] = None
        self._preload: Optional[threading.Thread] = None

    def set_date(self, year: int, month: int, day: int):
        self._date = f"{year:04d}{month:02d}{day:02d}"
        self.dataset.set_date(self._date)
        self.box.day_id = make_day_id(year, month, day)

    def begin_pass(self):
        self.box.begin_pass()

    def end_pass(self, need_save_delta: bool = False):
        self.box.end_pass(need_save_delta)

    def read_ins_into_memory(self):
        # the loader threads register feasigns into the feed-pass agent
        self.dataset.load_into_memory(register_keys=True)

    load_into_memory = read_ins_into_memory

    def preload_into_memory(self):
        self.dataset.preload_into_memory()

    def wait_feed_pass_done(self):
        self.dataset.wait_preload_done(register_keys=True)

    def slots_shuffle(self, slots):
        self.dataset.slots_shuffle(slots)
