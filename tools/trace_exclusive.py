"""Per-kernel busy time that no other kernel overlaps (exclusive) vs total, from a rocprofv3 kernel trace, over the
last N steps' span: which kernels sit on the critical path and which run under others (side streams).
python tools/trace_exclusive.py <run_kernel_trace.csv> [top]"""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
top = int(sys.argv[2]) if len(sys.argv) > 2 else 20
ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
# sweep: at each elementary interval, the set of running kernels; exclusive time goes to a kernel running alone
points = sorted({t for s, e, _ in ev for t in (s, e)})
starts = collections.defaultdict(list)
ends = collections.defaultdict(list)
for i, (s, e, n) in enumerate(ev):
    starts[s].append(i)
    ends[e].append(i)
active = set()
excl = collections.Counter()
total = collections.Counter()
shared = collections.Counter()
busy = idle = 0
for a, b in zip(points, points[1:]):
    for i in ends[a]:
        active.discard(i)
    for i in starts[a]:
        active.add(i)
    d = b - a
    if not active:
        idle += d
        continue
    busy += d
    if len(active) == 1:
        excl[ev[next(iter(active))][2]] += d
    for i in active:
        shared[ev[i][2]] += d / len(active)
for s, e, n in ev:
    total[n] += e - s
span = ev[-1][1] - ev[0][0]
print(f"span {span/1e6:.1f} ms, busy {busy/1e6:.1f} ms, idle {idle/1e6:.1f} ms")
print(f"{'kernel':70s} {'total_ms':>9s} {'excl_ms':>8s} {'share_ms':>9s}")
for n, t in total.most_common(top):
    print(f"{n[:70]:70s} {t/1e6:9.2f} {excl[n]/1e6:8.2f} {shared[n]/1e6:9.2f}")
