"""Plain-text table rendering compatible with PrettyTable's default style.

The reference prints its census with ``prettytable.PrettyTable`` (who_use_gpu.py:5,11,22),
which is not installed in this image, so the framework renders the same
box style itself: ``+---+`` rules, ``|`` separators, one space of padding, centred cells
(PrettyTable puts the odd padding space right for odd-width text, left for even).
"""
from __future__ import annotations

from typing import Sequence


def _center(text: str, width: int) -> str:
    excess = width - len(text)
    if excess <= 0:
        return text
    if excess % 2:
        if len(text) % 2:
            return " " * (excess // 2) + text + " " * (excess // 2 + 1)
        return " " * (excess // 2 + 1) + text + " " * (excess // 2)
    return " " * (excess // 2) + text + " " * (excess // 2)


def render(header: Sequence[str], rows: Sequence[Sequence[object]], align: str = "c") -> str:
    cells = [[str(c) for c in r] for r in rows]
    widths = [len(h) for h in header]
    for r in cells:
        for i, c in enumerate(r):
            widths[i] = max(widths[i], len(c))
    rule = "+" + "+".join("-" * (w + 2) for w in widths) + "+"

    def fmt(r):
        parts = []
        for c, w in zip(r, widths):
            if align == "l":
                parts.append(" " + c.ljust(w) + " ")
            elif align == "r":
                parts.append(" " + c.rjust(w) + " ")
            else:
                parts.append(" " + _center(c, w) + " ")
        return "|" + "|".join(parts) + "|"

    out = [rule, fmt(header), rule]
    out += [fmt(r) for r in cells]
    out.append(rule)
    return "\n".join(out)


def render_csv(header: Sequence[str], rows: Sequence[Sequence[object]]) -> str:
    import csv
    import io

    buf = io.StringIO()
    w = csv.writer(buf, lineterminator="\n")
    w.writerow(header)
    w.writerows(rows)
    return buf.getvalue().rstrip("\n")
