"""Effective GPU clock per kernel from a rocprofv3 GRBM_GUI_ACTIVE pass (MI355X_MICROARCH.md
§DVFS: GRBM_GUI_ACTIVE is summed over the 8 XCDs, so clock = value / 8 / kernel wall time; it reads
high on dispatches shorter than ~0.3 ms).  Groups by (kernel base name, grid); prints the
dispatch-weighted clock of the groups that take the most time, and the SQ-pass MFMA-busy fraction
when an SQ counter file is given (SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x GRBM cycles / 8)).

usage: python tools/eff_clock.py GRBM.csv [SQ.csv] > out.txt
"""
import csv
import sys
from collections import defaultdict

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.abspath(__file__)))
from prof_summary import base  # noqa: E402


def load(path, counter):
    out = {}
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] == counter:
            out[r["Dispatch_Id"]] = (base(r["Kernel_Name"]), int(r["Grid_Size"]), float(r["Counter_Value"]),
                                     int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    return out


def main():
    g = load(sys.argv[1], "GRBM_GUI_ACTIVE")
    mf = load(sys.argv[2], "SQ_VALU_MFMA_BUSY_CYCLES") if len(sys.argv) > 2 else {}
    agg = defaultdict(lambda: [0.0, 0.0, 0, 0.0])   # grbm cycles/8, ns, n, mfma busy
    for d, (k, grid, v, ns) in g.items():
        a = agg[(k, grid)]
        a[0] += v / 8
        a[1] += ns
        a[2] += 1
    for d, (k, grid, v, ns) in mf.items():
        if (k, grid) in agg:
            agg[(k, grid)][3] += v
    tot_ns = sum(a[1] for a in agg.values())
    tot_cyc = sum(a[0] for a in agg.values())
    print(f"all dispatches: {tot_cyc / tot_ns:.3f} GHz effective over {tot_ns / 1e6:.1f} ms of kernel time")
    print(f"{'kernel':50s} {'grid':>9s} {'n':>4s} {'ms':>8s} {'GHz':>6s} {'mfma busy':>9s}")
    for (k, grid), (cyc, ns, n, busy) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:25]:
        mb = f"{busy / (1024 * cyc):9.3f}" if mf and cyc else ""
        print(f"{k[:50]:50s} {grid:9d} {n:4d} {ns / 1e6:8.2f} {cyc / ns:6.3f} {mb}")


if __name__ == "__main__":
    main()
