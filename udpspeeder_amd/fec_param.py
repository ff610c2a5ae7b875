"""FEC parameter table: the ``-f x1:y1,x2:y2,...`` grammar of UDPspeeder.

Mirrors ``fec_parameter_t::rs_from_str`` (fec_manager.h:40-136): the list is
expanded into a dense table ``rs_par[x-1] = (x, y)`` for x = 1..x_last.  Below
the first point every x gets the first y (fec_manager.h:95-102); between two
points y is interpolated as ``pre_y + (now_y - pre_y) * (x - pre_x) / dist +
0.9999`` in double and truncated (fec_manager.h:122), clamped so x + y <= 255
(fec_manager.h:124-127).  Invalid input returns None where the reference
returns -1 (fec_manager.h:43-69).  The C3 workload uses this table to pick m
for each k.
"""
from __future__ import annotations

import re
from typing import List, Optional, Tuple

MAX_FEC_PACKET_NUM = 255  # fec_manager.h:18
# sscanf(tok, "%d:%d") (fec_manager.h:52): optional leading white space and
# sign before each number, ':' right after the first; the rest is ignored
_XY = re.compile(r"[ \t\n\v\f\r]*([+-]?[0-9]+):[ \t\n\v\f\r]*([+-]?[0-9]+)")


def rs_from_str(s: str) -> Optional[List[Tuple[int, int]]]:
    # string_to_vec(s, ",") (common.cpp:919-934) is strtok: empty tokens vanish
    parts = [p for p in s.split(",") if p]
    pars = []
    for p in parts:
        m = _XY.match(p)
        if not m:
            return None
        x, y = int(m.group(1)), int(m.group(2))
        if x < 1 or y < 0 or x + y > MAX_FEC_PACKET_NUM:
            return None
        pars.append((x, y))
    if not pars:
        return None
    for i in range(1, len(pars)):
        if pars[i][0] <= pars[i - 1][0]:
            return None
    table = {}
    x0, y0 = pars[0]
    for i in range(1, x0 + 1):
        table[i] = y0
    for i in range(1, len(pars)):
        now_x, now_y = pars[i]
        pre_x, pre_y = pars[i - 1]
        table[now_x] = now_y
        for j in range(pre_x + 1, now_x):
            dist = float(now_x - pre_x)
            in_y = int(pre_y + (now_y - pre_y) * (j - pre_x) / dist + 0.9999)
            if j + in_y > MAX_FEC_PACKET_NUM:
                in_y = MAX_FEC_PACKET_NUM - j
            table[j] = in_y
    return [(x, table[x]) for x in range(1, pars[-1][0] + 1)]


def rs_to_str(table: List[Tuple[int, int]]) -> str:
    """fec_parameter_t::rs_to_str (fec_manager.h:138-152)."""
    return ",".join(f"{x}:{y}" for (x, y) in table)
