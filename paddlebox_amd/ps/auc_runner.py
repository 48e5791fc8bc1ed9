"""AucRunner: slot-importance evaluation by feature replacement.

The reference runs it inside BoxWrapper (``InitializeAucRunner``,
``GetRandomReplace``, ``AddReplaceFeasign``, ``RecordReplace`` /
``RecordReplaceBack``, box_wrapper.h:906-1011, box_wrapper.cc:212-368):
every instance is paired with a reservoir-sampled other instance, and an
evaluation phase replaces one slot group's feasigns by the partner's,
measures AUC, and restores them.  A slot whose replacement costs AUC
matters; a noise slot costs nothing.

The per-record work is native (csrc/host/auc_runner.cc over the columnar
pass store); this class maps slot names to store columns and drives it.
"""
from __future__ import annotations

from typing import Callable, Dict, List, Sequence

import torch

from .. import _native


class AucRunner:
    def __init__(self, slot_eval: Sequence[Sequence[str]], thread_num: int = 4, pool_size: int = 10000,
                 seed: int = 0):
        self.groups: List[List[str]] = [list(g) for g in slot_eval]
        self.names = sorted({s for g in self.groups for s in g})
        self._n = _native.host().AucRunner(int(pool_size), int(thread_num), int(seed))
        self._bound = None  # dataset the runner sampled
        self.last_slots: List[str] = []

    @staticmethod
    def _index(dataset, names: Sequence[str]) -> List[int]:
        all_names = dataset._native.sparse_slot_names()
        u64 = dataset._native.sparse_slot_u64_index()
        pos = {n: u for n, u in zip(all_names, u64)}
        missing = [n for n in names if n not in pos]
        if missing:
            raise KeyError(f"AucRunner: unknown sparse slots {missing}")
        return [pos[n] for n in names]

    def covers(self, dataset, slots: Sequence[str]) -> bool:
        return self._bound is dataset and set(slots) <= set(self.names)

    def prepare(self, dataset) -> torch.Tensor:
        """GetRandomReplace for the loaded pass; returns the candidate
        feasigns (AddReplaceFeasign) so the caller can register them."""
        if self._n.replaced():
            raise RuntimeError("AucRunner.prepare: restore the replaced slots (slots_shuffle([])) first")
        if not dataset._configured:
            dataset._configure()
        self._n.set_eval_slots(self._index(dataset, self.names))
        self._n.sample(dataset._native)
        self._bound = dataset
        return self._n.candidate_keys()

    def shuffle(self, dataset, slots: Sequence[str]) -> int:
        """RecordReplaceBack of the previous group, RecordReplace of ``slots``."""
        if self._bound is not dataset:
            raise RuntimeError("AucRunner.shuffle: dataset was not prepared by this runner")
        n = int(self._n.shuffle(dataset._native, self._index(dataset, slots)))
        self.last_slots = list(slots)
        return n

    def pool_entries(self) -> int:
        return int(self._n.pool_entries())

    def slot_importance(self, dataset, evaluate: Callable[[], float]) -> Dict[str, float]:
        """Run ``evaluate()`` (returns AUC on the dataset as currently
        replaced) once unreplaced and once per slot group; returns
        {"base": auc, "<group>": auc, ...}."""
        out = {"base": None}
        self.shuffle(dataset, [])
        out["base"] = float(evaluate())
        for g in self.groups:
            self.shuffle(dataset, g)
            out[",".join(g)] = float(evaluate())
        self.shuffle(dataset, [])
        return out
