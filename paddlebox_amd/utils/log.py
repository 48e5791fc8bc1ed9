"""Structured JSON-lines logging per pass (throughput, stage times, tiers)."""
from __future__ import annotations

import json
import logging
import os
import sys
import time

_logger = logging.getLogger("paddlebox_amd")
if not _logger.handlers:
    h = logging.StreamHandler(sys.stderr)
    h.setFormatter(logging.Formatter("[%(asctime)s %(levelname)s pbx] %(message)s"))
    _logger.addHandler(h)
    _logger.setLevel(os.environ.get("PBX_LOG_LEVEL", "INFO"))


def logger():
    return _logger


class JsonlLog:
    def __init__(self, path: str = None):
        self.path = path

    def write(self, **rec):
        rec.setdefault("ts", time.time())
        line = json.dumps(rec)
        if self.path:
            with open(self.path, "a") as f:
                f.write(line + "\n")
        else:
            _logger.info(line)
