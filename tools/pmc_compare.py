"""Per-dispatch PMC counters of selected kernels from rocprofv3 counter-collection CSVs, averaged per
(kernel, grid) group -- to compare one kernel in the train step against the same kernel launched alone.
Each CSV is one pass (MI355X_MICROARCH.md "rocprofv3 PMC slots": one block's slots per pass).  With
GRBM_GUI_ACTIVE and the dispatch's timestamps the effective clock is GRBM_GUI_ACTIVE / 8 / duration
(the counter sums the 8 XCDs; the guide's DVFS item), with TCC_HIT / TCC_MISS the L2 hit rate.

usage: python tools/pmc_compare.py <regex> <label>=<csv>[,<csv>...] ...
"""
import csv
import os
import re
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from prof_summary import base  # noqa: E402


def load(paths, rx):
    """{(kernel, grid): {counter: [values per dispatch], "_dur_ns": [...]}}"""
    out = defaultdict(lambda: defaultdict(list))
    for p in paths:
        seen = set()
        with open(p) as f:
            for r in csv.DictReader(f):
                name = base(r["Kernel_Name"])
                if not re.search(rx, name):
                    continue
                k = (name, int(r["Grid_Size"]))
                out[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
                did = (r.get("Dispatch_Id") or r.get("Correlation_Id"), k)
                if did not in seen and r.get("Start_Timestamp") and r.get("End_Timestamp"):
                    seen.add(did)
                    out[k]["_dur_ns"].append(float(r["End_Timestamp"]) - float(r["Start_Timestamp"]))
    return out


def main():
    rx = sys.argv[1]
    for arg in sys.argv[2:]:
        label, paths = arg.split("=", 1)
        data = load(paths.split(","), rx)
        for (name, grid), c in sorted(data.items()):
            mean = {n: sum(v) / len(v) for n, v in c.items() if v}
            n = max(len(v) for v in c.values())
            line = f"{label:10s} {name:32s} grid={grid:8d} n={n:4d}"
            dur = mean.get("_dur_ns")
            if dur:
                line += f" dur={dur / 1e3:8.1f}us"
                if "GRBM_GUI_ACTIVE" in mean:
                    line += f" clock={mean['GRBM_GUI_ACTIVE'] / 8 / dur:5.2f}GHz"
            if "TCC_HIT_sum" in mean and "TCC_MISS_sum" in mean:
                tot = mean["TCC_HIT_sum"] + mean["TCC_MISS_sum"]
                line += f" L2hit={mean['TCC_HIT_sum'] / max(tot, 1):5.3f}"
            for k2 in sorted(mean):
                if k2 not in ("_dur_ns",):
                    line += f" {k2}={mean[k2]:.4g}"
            print(line)


if __name__ == "__main__":
    main()
