"""Compare two print_tensor-format dumps tensor by tensor (layer triage).

The counterpart of the reference's compare_tensors.py (its parse_file and
comparison loop, compare_tensors.py:6-146): a dump is a sequence of blocks

    <name> = {ne0, ne1, ne2, ne3}
        [ ... printed values (3 head + 3 tail per row, "%12.4f") ... ]
        sum = <float>

as written by tensor.h print_tensor_generic (the reference under --verbose)
and by llmi_session_dump (this repo).  Blocks pair by name and occurrence
(the n-th "Qcur-0" of one file with the n-th of the other); for each pair
the report gives both sums, |delta sum| and the MSE over the printed values.
Names present in only one file are listed separately (the reference prints
more intermediates than the device path materialises).  No plotting.

    python scripts/compare_dumps.py ref.txt ours.txt [--tol 1e-3]

Exit status 1 when a pair's |delta sum| > tol * max(1, |sum_ref|).
"""
from __future__ import annotations

import argparse
import math
import re
import sys
from collections import defaultdict
from typing import Dict, List, Tuple

_SUM = re.compile(r"^\s*sum\s+=\s+(\S+)")
_NAME = re.compile(r"^\s*([^=\[\]]+?)\s+=\s+\{([^}]*)\}")
_NUM = re.compile(r"[-+]?(?:\d+\.\d+|\.\d+|\d+)(?:[eE][-+]?\d+)?|[-+]?nan|[-+]?inf")


def parse(text: str) -> List[dict]:
    """Blocks of a dump, in file order: name, shape, printed values, sum."""
    out: List[dict] = []
    cur = None
    for line in text.splitlines():
        m = _SUM.match(line)
        if m and cur is not None:
            cur["sum"] = float(m.group(1))
            out.append(cur)
            cur = None
            continue
        m = _NAME.match(line)
        if m:
            cur = {"name": m.group(1).strip(), "shape": [int(v) for v in m.group(2).split(",")], "values": []}
            continue
        if cur is not None:
            cur["values"] += [float(v) for v in _NUM.findall(line)]
    return out


def pair(a: List[dict], b: List[dict]) -> Tuple[List[Tuple[str, int, dict, dict]], List[str], List[str]]:
    """(name, occurrence, block a, block b) for every name in both files."""
    idx_b: Dict[Tuple[str, int], dict] = {}
    seen: Dict[str, int] = defaultdict(int)
    for t in b:
        idx_b[(t["name"], seen[t["name"]])] = t
        seen[t["name"]] += 1
    seen_a: Dict[str, int] = defaultdict(int)
    pairs, only_a = [], []
    for t in a:
        k = (t["name"], seen_a[t["name"]])
        seen_a[t["name"]] += 1
        if k in idx_b:
            pairs.append((k[0], k[1], t, idx_b.pop(k)))
        else:
            only_a.append(k[0])
    only_b = sorted({k[0] for k in idx_b})
    return pairs, sorted(set(only_a)), only_b


def mse(x: List[float], y: List[float]) -> float:
    n = min(len(x), len(y))
    if n == 0:
        return 0.0
    return sum((x[i] - y[i]) ** 2 for i in range(n)) / n


def compare(text_a: str, text_b: str, tol: float = 1e-3):
    """Rows (name, occurrence, sum_a, sum_b, |d sum|, mse, ok) + unmatched names."""
    pairs, only_a, only_b = pair(parse(text_a), parse(text_b))
    rows = []
    for name, occ, ta, tb in pairs:
        d = abs(ta["sum"] - tb["sum"])
        ok = (ta["shape"] == tb["shape"]) and (d <= tol * max(1.0, abs(ta["sum"])) or
                                                (math.isnan(ta["sum"]) and math.isnan(tb["sum"])))
        rows.append((name, occ, ta["sum"], tb["sum"], d, mse(ta["values"], tb["values"]), ok))
    return rows, only_a, only_b


def main() -> int:
    p = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    p.add_argument("a")
    p.add_argument("b")
    p.add_argument("--tol", type=float, default=1e-3, help="relative |delta sum| bound")
    a = p.parse_args()
    rows, only_a, only_b = compare(open(a.a).read(), open(a.b).read(), a.tol)
    print(f"{'tensor':48s} {'#':>3s} {'sum a':>14s} {'sum b':>14s} {'|d sum|':>10s} {'mse':>10s}")
    bad = 0
    for name, occ, sa, sb, d, m, ok in rows:
        bad += not ok
        print(f"{name[:48]:48s} {occ:3d} {sa:14.6f} {sb:14.6f} {d:10.3g} {m:10.3g}{'' if ok else '  <-- differs'}")
    if only_a:
        print(f"only in {a.a}: {', '.join(only_a[:12])}{' ...' if len(only_a) > 12 else ''}")
    if only_b:
        print(f"only in {a.b}: {', '.join(only_b[:12])}{' ...' if len(only_b) > 12 else ''}")
    print(f"{len(rows)} pairs, {bad} outside tolerance")
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
