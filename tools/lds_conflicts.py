"""LDS bank-conflict census from a rocprofv3 --pmc run with SQ_LDS_BANK_CONFLICT,
SQ_LDS_IDX_ACTIVE and SQ_INSTS_LDS (tools/gpu/r2_ldsconf.sh): per kernel (base name + grid),
the extra conflict cycles as a fraction of all LDS-array cycles, summed over its dispatches.

usage: python tools/lds_conflicts.py <pmc output dir> [top]
"""
import csv
import glob
import os
import sys
from collections import defaultdict

from prof_summary import base


def main():
    root = sys.argv[1]
    top = int(sys.argv[2]) if len(sys.argv) > 2 else 25
    path = glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True)[0]
    agg = defaultdict(lambda: defaultdict(float))
    calls = defaultdict(set)
    for r in csv.DictReader(open(path)):
        key = (base(r["Kernel_Name"]), r.get("Grid_Size", r.get("Grid_Size_X", "")))
        agg[key][r["Counter_Name"]] += float(r["Counter_Value"])
        calls[key].add(r.get("Dispatch_Id", ""))
    rows = []
    for k, v in agg.items():
        act = v.get("SQ_LDS_IDX_ACTIVE", 0.0)
        conf = v.get("SQ_LDS_BANK_CONFLICT", 0.0)
        rows.append((conf, act, v.get("SQ_INSTS_LDS", 0.0), len(calls[k]), k))
    rows.sort(reverse=True)
    print(f"source: {path}")
    print(f"{'kernel':40s} {'grid':>10s} {'calls':>6s} {'conflict cyc':>14s} {'LDS active cyc':>15s} {'conf/active':>11s}")
    for conf, act, ins, n, (name, grid) in rows[:top]:
        frac = conf / act if act else 0.0
        print(f"{name[:40]:40s} {grid:>10s} {n:6d} {conf:14.3e} {act:15.3e} {frac:11.3f}")


if __name__ == "__main__":
    main()
