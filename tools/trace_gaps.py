#!/usr/bin/env python3
"""Per-step GPU busy vs wall time, per-stream busy time and the largest idle gaps from a
rocprofv3 kernel trace.

usage: trace_gaps.py <run_kernel_trace.csv> [marker_kernel_substring]
One step = the kernels between the last two launches of the marker kernel (default: the fused Adam).
"""
import collections
import csv
import sys


def union(iv):
    tot, cur_s, cur_e = 0, None, None
    for s, e in sorted(iv):
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                tot += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    return tot + (cur_e - cur_s if cur_e is not None else 0)


def main():
    path = sys.argv[1]
    marker = sys.argv[2] if len(sys.argv) > 2 else "adam_flat"
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows) if marker in r["Kernel_Name"]]
    a, b = idx[-2], idx[-1]
    step = rows[a + 1:b + 1]
    t0, t1 = int(rows[a]["End_Timestamp"]), int(step[-1]["End_Timestamp"])
    iv = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in step]
    busy = sum(e - s for s, e in iv)
    print("step: wall %.3f ms, kernel time %.3f ms, GPU busy (union) %.3f ms, %d kernels"
          % ((t1 - t0) / 1e6, busy / 1e6, union(iv) / 1e6, len(step)))
    per = collections.defaultdict(list)
    for r in step:
        per[r.get("Stream_Id", r.get("Queue_Id"))].append(r)
    for sid, rs in sorted(per.items(), key=lambda kv: -len(kv[1])):
        u = union([(int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rs])
        top = collections.Counter()
        for r in rs:
            top[r["Kernel_Name"][:60]] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        print("stream %s: %d kernels, busy %.3f ms; top: %s" % (sid, len(rs), u / 1e6, "; ".join(
            "%s %.2f" % (k, v / 1e6) for k, v in top.most_common(4))))
    gaps = []
    end = t0
    for r in step:
        s = int(r["Start_Timestamp"])
        if s - end > 2000:
            gaps.append(((s - end) / 1e3, r["Kernel_Name"][:60]))
        end = max(end, int(r["End_Timestamp"]))
    print("device idle gaps > 2us: total %.3f ms in %d gaps" % (sum(g for g, _ in gaps) / 1e3, len(gaps)))
    for g in sorted(gaps, reverse=True)[:10]:
        print("  %8.1f us  before %s" % g)


if __name__ == "__main__":
    main()
