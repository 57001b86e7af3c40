"""Per-stream busy time and idle gaps from a rocprofv3 kernel trace (csv): is a step GPU-bound or launch-bound?
    python tools/timeline_gaps.py <kernel_trace.csv> [last_ms]"""
import csv
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
last_ms = float(sys.argv[2]) if len(sys.argv) > 2 else 60.0
sk = next(k for k in rows[0] if "Start" in k)
ek = next(k for k in rows[0] if "End" in k)
qk = next((k for k in rows[0] if k.lower() in ("stream_id", "queue_id")), None)
t_end = max(int(r[ek]) for r in rows)
t0 = t_end - int(last_ms * 1e6)
rows = [r for r in rows if int(r[sk]) >= t0]
by = defaultdict(list)
for r in rows:
    by[r[qk] if qk else "all"].append((int(r[sk]), int(r[ek]), r["Kernel_Name"][:60]))
span = (t_end - min(int(r[sk]) for r in rows)) / 1e6
print(f"window {span:.2f} ms, {len(rows)} kernels, streams/queues: {len(by)} (key {qk})")
allv = sorted((s, e) for v in by.values() for s, e, _ in v)
busy, cur_s, cur_e = 0, None, None
for s, e in allv:
    if cur_e is None or s > cur_e:
        if cur_e is not None:
            busy += cur_e - cur_s
        cur_s, cur_e = s, e
    else:
        cur_e = max(cur_e, e)
busy += cur_e - cur_s
print(f"any-stream busy {busy / 1e6:.2f} ms of {span:.2f} ({100 * busy / 1e6 / span:.1f} %)")
for q, v in sorted(by.items(), key=lambda kv: -len(kv[1])):
    v.sort()
    b = sum(e - s for s, e, _ in v)
    gaps = [v[i + 1][0] - v[i][1] for i in range(len(v) - 1)]
    big = sorted(((g, v[i][2], v[i + 1][2]) for i, g in enumerate(gaps) if g > 20000), reverse=True)[:5]
    print(f"stream {q}: {len(v)} kernels, busy {b / 1e6:.2f} ms, gaps>2us total {sum(g for g in gaps if g > 2000) / 1e6:.2f} ms")
    for g, a, c in big:
        print(f"    gap {g / 1e3:.1f} us after {a} -> {c}")
