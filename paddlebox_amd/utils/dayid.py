"""Day ids for passes (BoxWrapper make_day_id, reference
``fw/fleet/box_wrapper.cc:38-76``): days since 1970 using the
leap-year-every-4 month table, minus 8 hours (UTC+8) unless FLAGS_fix_dayid."""
from __future__ import annotations

from . import flags as _flags

MINUTE = 60
HOUR = 60 * MINUTE
DAY = 24 * HOUR
YEAR = 365 * DAY
_GMONTH = [0]
for _d in (31, 29, 31, 30, 31, 30, 31, 31, 30, 31, 30):
    _GMONTH.append(_GMONTH[-1] + DAY * _d)


def make_day_id(y: int, m: int, d: int, fix_dayid: bool = None) -> int:
    year = y - 1970
    mon = m - 1
    res = YEAR * year + DAY * ((year + 1) // 4)
    res += _GMONTH[mon]
    if mon > 1 and ((year + 2) % 4):
        res -= DAY
    res += DAY * (d - 1)
    if fix_dayid is None:
        fix_dayid = _flags.get_bool("fix_dayid")
    if fix_dayid:
        return int(res // 86400)
    return int((res - 8 * 3600) / 86400)  # C truncation toward zero


def make_day_id_str(date: str) -> int:
    date = str(date)
    return make_day_id(int(date[0:4]), int(date[4:6]), int(date[6:8]))
