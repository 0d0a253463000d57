"""Summarise a rocprofv3 kernel trace of bench.py: per-step kernel time vs wall time and the largest
idle gaps between consecutive kernels (name before -> name after)."""
import csv
import collections
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
k = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0][-48:]) for r in rows]
# keep the last 40% of dispatches (timed steps)
k = k[int(len(k) * 0.6):]
busy = sum(e - s for s, e, _ in k)
wall = k[-1][1] - k[0][0]
print(f"dispatches {len(k)}  busy {busy/1e3:.1f} us  wall {wall/1e3:.1f} us  idle {100*(1-busy/wall):.1f}%")
gaps = collections.defaultdict(list)
for (s0, e0, n0), (s1, e1, n1) in zip(k, k[1:]):
    gaps[(n0, n1)].append(max(0, s1 - e0))
tot = sorted(((sum(v), len(v), key) for key, v in gaps.items()), reverse=True)
for t, n, (a, b) in tot[:14]:
    print(f"{t/1e3:9.1f} us over {n:4d}  {a:>48s} -> {b}")
dur = collections.defaultdict(list)
for s, e, n in k:
    dur[n].append(e - s)
print("--- kernels (avg us, count)")
for n, v in sorted(dur.items(), key=lambda kv: -sum(kv[1])):
    print(f"{sum(v)/len(v)/1e3:9.2f} {len(v):5d}  {n}")
