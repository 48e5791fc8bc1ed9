"""Metric registry with the nine BoxWrapper calculator kinds.

Reference: ``BoxWrapper::InitMetric`` (``fw/fleet/box_wrapper.cc:916-1025``),
the ``MetricMsg`` family (``:265-886``) and ``GetMetricMsg`` /
``GetContinueMetricMsg`` / ``GetNanInfMetricMsg`` (``:1027-1083``).

Per-batch accumulation runs on the GPU (histogram kernel into a device
``[2, buckets]`` f64 table, no per-batch D2H -- the reference copies preds and
labels to the host every batch, ``metrics.cc:115-136``); ``get_metric_msg``
all-reduces the tables over the process group and computes on the host with
the native calculator (``csrc/host/metrics.cc``).
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple

import torch
import torch.distributed as dist

from .. import _native
from ..ops.ctr import auc_accumulate

KINDS = (
    "AucCalculator",
    "MultiTaskAucCalculator",
    "CmatchRankAucCalculator",
    "MaskAucCalculator",
    "MultiMaskAucCalculator",
    "CmatchRankMaskAucCalculator",
    "FloatMaskAucCalculator",
    "ContinueMaskCalculator",
    "NanInfCalculator",
    "WuAucCalculator",
)


def parse_cmatch_rank(x: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
    """high 32 bits = cmatch, low 8 bits = rank (box_wrapper.h:364-368)."""
    x = x.to(torch.int64)
    return (x >> 32) & 0xFFFFFFFF, x & 0xFF


def _parse_group(group: str) -> List[Tuple[int, int]]:
    out = []
    for item in [g for g in group.replace(",", " ").split() if g]:
        a, b = item.split("_")
        out.append((int(a), int(b)))
    return out


@dataclass
class Metric:
    method: str
    name: str
    label_var: str
    pred_var: str
    cmatch_rank_var: str = ""
    mask_var: str = ""
    phase: int = -1
    cmatch_rank_group: str = ""
    ignore_rank: bool = False
    bucket_size: int = 1_000_000
    sample_scale_var: str = ""
    uid_var: str = ""
    pred_list: List[str] = field(default_factory=list)
    mask_list: List[str] = field(default_factory=list)
    # state
    calc: object = None
    dev_table: Optional[torch.Tensor] = None
    dev_stats: Optional[torch.Tensor] = None

    def reset_device(self):
        if self.dev_table is not None:
            self.dev_table.zero_()
            self.dev_stats.zero_()


class MetricRegistry:
    def __init__(self, group=None):
        self.metrics: Dict[str, Metric] = {}
        self.group = group
        self.phase = 1  # reference phase_: join=1 / update=0
        self.phase_num = 2

    # -- phases (box_wrapper.h:770-773,890-891)
    def flip_phase(self):
        self.phase = (self.phase + 1) % self.phase_num

    def set_phase(self, p: int):
        self.phase = p

    def init_metric(self, method: str, name: str, label_varname: str, pred_varname: str,
                    cmatch_rank_varname: str = "", mask_varname: str = "", metric_phase: int = -1,
                    cmatch_rank_group: str = "", ignore_rank: bool = False, bucket_size: int = 1_000_000,
                    mode_collect_in_gpu: bool = True, max_batch_size: int = 0, sample_scale_varname: str = "",
                    uid_varname: str = ""):
        if method not in KINDS:
            raise ValueError(f"unknown metric method {method}")
        m = Metric(method, name, label_varname, pred_varname, cmatch_rank_varname, mask_varname, metric_phase,
                   cmatch_rank_group, ignore_rank, bucket_size, sample_scale_varname, uid_varname)
        if method == "MultiTaskAucCalculator":
            m.pred_list = [p for p in pred_varname.replace(",", " ").split() if p]
        if method == "MultiMaskAucCalculator":
            m.mask_list = [p for p in mask_varname.replace(",", " ").split() if p]
        m.calc = _native.host().AucCalculator(bucket_size)
        self.metrics[name] = m
        return m

    def get_metric_name_list(self, metric_phase: int = -1) -> List[str]:
        return [n for n, m in self.metrics.items() if metric_phase == -1 or m.phase in (-1, metric_phase)]

    # -- accumulation ---------------------------------------------------
    def add_batch(self, fetch: Dict[str, torch.Tensor]):
        """Accumulate every registered metric of the current phase from the
        batch's named tensors (preds, labels, masks, cmatch_rank, uids).
        Metrics a kernel already accumulated for this batch (``fetch.
        fused_metrics``: the fused tower's AUC) are skipped."""
        done = getattr(fetch, "fused_metrics", ())
        for name, m in self.metrics.items():
            if m.phase != -1 and m.phase != self.phase:
                continue
            if name in done:
                continue
            self._add(m, fetch)

    def _dev_tables(self, m: Metric, device):
        if m.dev_table is None or m.dev_table.device != device:
            m.dev_table = torch.zeros(2 * m.bucket_size, dtype=torch.float64, device=device)
            m.dev_stats = torch.zeros(5, dtype=torch.float64, device=device)
        return m.dev_table, m.dev_stats

    def _add(self, m: Metric, fetch):
        label = fetch[m.label_var].reshape(-1).float()
        mask = None
        if m.method in ("MaskAucCalculator", "CmatchRankMaskAucCalculator", "FloatMaskAucCalculator",
                        "ContinueMaskCalculator") and m.mask_var:
            mask = (fetch[m.mask_var].reshape(-1) != 0).float()
        if m.method == "MultiMaskAucCalculator":
            mask = torch.ones_like(label)
            for mv in m.mask_list:
                mask = mask * (fetch[mv].reshape(-1) != 0).float()
        if m.method in ("CmatchRankAucCalculator", "CmatchRankMaskAucCalculator"):
            cm, rk = parse_cmatch_rank(fetch[m.cmatch_rank_var].reshape(-1))
            sel = torch.zeros_like(label, dtype=torch.bool)
            for c, r in _parse_group(m.cmatch_rank_group):
                sel |= (cm == c) if m.ignore_rank else ((cm == c) & (rk == r))
            sel = sel.float()
            mask = sel if mask is None else mask * sel
        if m.method == "MultiTaskAucCalculator":
            cm, rk = parse_cmatch_rank(fetch[m.cmatch_rank_var].reshape(-1))
            pred = torch.zeros_like(label)
            sel = torch.zeros_like(label, dtype=torch.bool)
            for (c, r), pv in zip(_parse_group(m.cmatch_rank_group), m.pred_list):
                hit = (cm == c) & (rk == r) & ~sel
                pred = torch.where(hit, fetch[pv].reshape(-1).float(), pred)
                sel |= hit
            self._hist(m, pred, label, sel.float())
            return
        if m.method == "NanInfCalculator":
            m.calc.add_nan_inf(fetch[m.pred_var].reshape(-1).float().detach().cpu().contiguous())
            return
        pred = fetch[m.pred_var].reshape(-1).float()
        if m.method == "WuAucCalculator":
            m.calc.add_uid(pred.detach().cpu().contiguous(), label.cpu().contiguous(),
                           fetch[m.uid_var].reshape(-1).to(torch.int64).cpu().contiguous())
            self._hist(m, pred, label, mask)
            return
        if m.method == "FloatMaskAucCalculator":
            keep = mask.cpu() != 0 if mask is not None else slice(None)
            m.calc.add_float_label(pred.detach().cpu().contiguous(), label.cpu().contiguous(),
                                   None if mask is None else mask.cpu().contiguous())
            return
        if m.method == "ContinueMaskCalculator":
            m.calc.add_continue(pred.detach().cpu().contiguous(), label.cpu().contiguous(),
                                None if mask is None else mask.cpu().contiguous())
            return
        if m.sample_scale_var:
            scale = fetch[m.sample_scale_var].reshape(-1).float()
            # sample-scaled histogram on the host (rare path)
            p, l, s = pred.detach().cpu(), label.cpu(), scale.cpu()
            for v in torch.unique(s).tolist():
                sel = s == v
                m.calc.add(p[sel].contiguous(), l[sel].contiguous(), None, float(v))
            return
        self._hist(m, pred, label, mask)

    def _hist(self, m: Metric, pred, label, mask):
        tab, st = self._dev_tables(m, pred.device)
        auc_accumulate(pred.detach(), label, tab, st, None if mask is None else mask.contiguous())

    # -- results ----------------------------------------------------------
    def _reduce(self, t: torch.Tensor) -> torch.Tensor:
        if dist.is_available() and dist.is_initialized() and dist.get_world_size(self.group) > 1:
            t = t.clone()
            dist.all_reduce(t, group=self.group)
        return t

    def _collect(self, m: Metric):
        """Device histogram + host calculator state -> globally reduced
        (tables[2,T], err[5])."""
        host_t, host_e = m.calc.tables()
        if m.dev_table is not None:
            dt = m.dev_table.view(2, -1).to(host_t.device)
            host_t = host_t + dt.cpu()
            host_e = host_e + m.dev_stats.cpu()
        dev = m.dev_table.device if m.dev_table is not None else torch.device("cpu")
        if dist.is_available() and dist.is_initialized() and dist.get_world_size(self.group) > 1:
            backend = dist.get_backend(self.group)
            td = torch.device("cuda", torch.cuda.current_device()) if backend == "nccl" else torch.device("cpu")
            host_t = self._reduce(host_t.to(td)).cpu()
            host_e = self._reduce(host_e.to(td)).cpu()
        return host_t.contiguous(), host_e.contiguous()

    def get_metric_msg(self, name: str) -> List[float]:
        """[auc, bucket_error, mae, rmse, actual_ctr, predicted_ctr,
        actual/predicted (copc), size]; resets the metric."""
        m = self.metrics[name]
        if m.method == "WuAucCalculator":
            m.calc.compute_wuauc()
            res = [m.calc.uauc, m.calc.wuauc, m.calc.user_cnt, m.calc.size]
            self._reset(m)
            return res
        t, e = self._collect(m)
        m.calc.compute(t, e)
        c = m.calc
        copc = c.actual_ctr / c.predicted_ctr if c.predicted_ctr > 0 else 0.0
        res = [c.auc, c.bucket_error, c.mae, c.rmse, c.actual_ctr, c.predicted_ctr, copc, c.size]
        if _debug_metrics():
            # FLAGS_enable_debug_print_metrics_info (fw/fleet/metrics.cc:29)
            _log().info("metric %s [%s phase=%s]: auc=%.6f bucket_error=%.6f mae=%.6f rmse=%.6f actual_ctr=%.6f "
                        "predicted_ctr=%.6f copc=%.6f size=%d", name, m.method, getattr(m, "phase", -1), *res[:7],
                        int(res[7]))
        self._reset(m)
        return res

    def get_continue_metric_msg(self, name: str) -> List[float]:
        """[mae, rmse, actual_value, predicted_value, size]"""
        m = self.metrics[name]
        _, e = self._collect(m)
        m.calc.compute_continue(e)
        c = m.calc
        res = [c.mae, c.rmse, c.actual_value, c.predicted_value, c.size]
        self._reset(m)
        return res

    def get_nan_inf_metric_msg(self, name: str) -> List[float]:
        """[nan_cnt, inf_cnt, nan_inf_rate, size]"""
        m = self.metrics[name]
        m.calc.compute_nan_inf()
        c = m.calc
        vals = torch.tensor([c.nan_cnt, c.inf_cnt, c.nan_inf_size], dtype=torch.float64)
        if dist.is_available() and dist.is_initialized() and dist.get_world_size(self.group) > 1 and \
                dist.get_backend(self.group) == "gloo":
            vals = self._reduce(vals)
        n, i, s = vals.tolist()
        res = [n, i, (n + i) / s if s > 0 else 0.0, s]
        self._reset(m)
        return res

    def _reset(self, m: Metric):
        m.calc.reset()
        m.reset_device()


def _debug_metrics() -> bool:
    from ..utils import flags as _fl

    try:
        return _fl.get_bool("enable_debug_print_metrics_info")
    except Exception:
        return False


def _log():
    from ..utils.log import logger

    return logger()
