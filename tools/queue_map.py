#!/usr/bin/env python3
"""Stream -> hardware-queue placement of a traced run (rocprofv3 --kernel-trace, rocpd sqlite).

    python tools/queue_map.py gpurun_out/qmap/run_results.db [--top 4]

One row per (HIP stream, HW queue) pair: dispatches, busy time, and the kernels that dominate it,
so each role (compute stream, weight-gradient side stream, RCCL comm stream) can be matched to its
queue.  Then the pairwise overlap: for every two queues, the wall time during which both had a
kernel running (a role sharing a queue with another would show zero overlap and serialise).
"""
import argparse
import collections
import re
import sqlite3


def short(name, n=60):
    name = re.sub(r"\(.*", "", name)
    return name if len(name) <= n else name[:n - 3] + "..."


def busy_intervals(iv):
    """Union of [start, end) intervals (sorted, merged)."""
    out = []
    for s, e in sorted(iv):
        if out and s <= out[-1][1]:
            out[-1][1] = max(out[-1][1], e)
        else:
            out.append([s, e])
    return out


def overlap(a, b):
    i = j = 0
    tot = 0
    while i < len(a) and j < len(b):
        s, e = max(a[i][0], b[j][0]), min(a[i][1], b[j][1])
        if e > s:
            tot += e - s
        if a[i][1] < b[j][1]:
            i += 1
        else:
            j += 1
    return tot


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--top", type=int, default=4)
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    rows = list(c.execute("select stream_id, queue_id, coalesce(stream, ''), coalesce(queue, ''), name, start, end "
                          "from kernels"))
    per = collections.defaultdict(lambda: {"n": 0, "t": 0, "names": collections.Counter(), "iv": []})
    queues = collections.defaultdict(list)
    for sid, qid, sname, qname, name, s, e in rows:
        d = per[(sid, qid, sname, qname)]
        d["n"] += 1
        d["t"] += e - s
        d["names"][short(name)] += e - s
        d["iv"].append((s, e))
        queues[qid].append((s, e))
    print("| stream id | stream | HW queue id | queue | dispatches | busy ms | top kernels (share of busy) |")
    print("|---|---|---|---|---|---|---|")
    for (sid, qid, sname, qname), d in sorted(per.items(), key=lambda kv: -kv[1]["t"]):
        top = ", ".join("%s %.0f%%" % (k, 100.0 * v / d["t"]) for k, v in d["names"].most_common(a.top))
        print("| %s | %s | %s | %s | %d | %.2f | %s |" % (sid, sname, qid, qname, d["n"], d["t"] / 1e6, top))
    streams_per_queue = collections.defaultdict(set)
    for (sid, qid, _, _) in per:
        streams_per_queue[qid].add(sid)
    shared = {q: s for q, s in streams_per_queue.items() if len(s) > 1}
    print("\nstreams: %d, HW queues: %d, queues shared by several streams: %s"
          % (len({k[0] for k in per}), len(queues), shared or "none"))
    merged = {q: busy_intervals(iv) for q, iv in queues.items()}
    qs = sorted(merged)
    if len(qs) > 1:
        print("\n| queue pair | both busy ms | busy ms (first) | busy ms (second) |")
        print("|---|---|---|---|")
        for i in range(len(qs)):
            for j in range(i + 1, len(qs)):
                ov = overlap(merged[qs[i]], merged[qs[j]])
                bi = sum(e - s for s, e in merged[qs[i]])
                bj = sum(e - s for s, e in merged[qs[j]])
                print("| %s / %s | %.2f | %.2f | %.2f |" % (qs[i], qs[j], ov / 1e6, bi / 1e6, bj / 1e6))


if __name__ == "__main__":
    main()
