"""Per-stream view of one training step from a rocprofv3 kernel trace: for the last full step
(delimited by the optimizer's opt_adam launches), each stream's busy time, and the kernels of
the main stream grouped by name with their time inside that step, plus the idle gaps.

usage: python tools/stream_timeline.py <kernel_trace.csv> [top]
"""
import csv
import sys
from collections import defaultdict

sys.path.insert(0, __file__.rsplit("/", 1)[0])
from prof_summary import base  # noqa: E402


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    top = int(sys.argv[2]) if len(sys.argv) > 2 else 30
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    adam = [i for i, r in enumerate(rows) if "opt_adam" in r["Kernel_Name"]]
    lo, hi = adam[-2] + 1, adam[-1] + 1
    step = rows[lo:hi]
    t0, t1 = int(step[0]["Start_Timestamp"]), int(step[-1]["End_Timestamp"])
    print(f"step window {(t1 - t0) / 1e6:.3f} ms, {len(step)} dispatches")
    by_q = defaultdict(list)
    for r in step:
        by_q[(r["Queue_Id"], r["Stream_Id"])].append(r)
    for q, rs in sorted(by_q.items(), key=lambda kv: -len(kv[1])):
        busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rs)
        print(f"queue {q[0]} stream {q[1]}: {len(rs)} dispatches, busy {busy / 1e6:.3f} ms")
    main_q = max(by_q, key=lambda k: len(by_q[k]))
    rs = by_q[main_q]
    gaps = 0
    for a, b in zip(rs, rs[1:]):
        g = int(b["Start_Timestamp"]) - int(a["End_Timestamp"])
        if g > 0:
            gaps += g
    print(f"main stream idle gaps inside the step: {gaps / 1e6:.3f} ms")
    agg = defaultdict(lambda: [0, 0])
    for r in rs:
        k = base(r["Kernel_Name"])
        agg[k][0] += 1
        agg[k][1] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    print(f"{'main-stream kernel':50s} {'calls':>6s} {'ms':>8s}")
    for k, (n, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:top]:
        print(f"{k[:50]:50s} {n:6d} {t / 1e6:8.3f}")
    for q, rs2 in by_q.items():
        if q == main_q:
            continue
        agg2 = defaultdict(lambda: [0, 0])
        for r in rs2:
            k = base(r["Kernel_Name"])
            agg2[k][0] += 1
            agg2[k][1] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        print(f"-- queue {q[0]} stream {q[1]}")
        for k, (n, t) in sorted(agg2.items(), key=lambda kv: -kv[1][1])[:12]:
            print(f"{k[:50]:50s} {n:6d} {t / 1e6:8.3f}")


if __name__ == "__main__":
    main()
