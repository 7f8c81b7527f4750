"""From a rocprofv3 kernel trace: how much of the conv kernels' busy time overlaps across queues/streams."""
import csv, sys
rows = []
for r in csv.DictReader(open(sys.argv[1])):
    if "wino3" in r["Kernel_Name"]:
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r.get("Stream_Id", r.get("Queue_Id"))))
rows.sort()
rows = rows[len(rows) // 2:]  # steady state
t0, t1 = rows[0][0], max(r[1] for r in rows)
busy = 0; cur = None
for s, e, _ in rows:
    if cur is None or s > cur[1]:
        if cur: busy += cur[1] - cur[0]
        cur = [s, e]
    else:
        cur[1] = max(cur[1], e)
busy += cur[1] - cur[0]
tot = sum(e - s for s, e, _ in rows)
print(f"conv kernels {len(rows)}, span {(t1-t0)/1e6:.1f} ms, union busy {busy/1e6:.1f} ms, sum {tot/1e6:.1f} ms, "
      f"overlap factor {tot/busy:.3f}, streams {sorted(set(r[2] for r in rows))}")
gaps = [rows[i+1][0] - max(r[1] for r in rows[:i+1]) for i in range(min(len(rows)-1, 4000))]
gaps = [g for g in gaps if g > 0]
print(f"idle gaps between conv kernels: n={len(gaps)}, total {sum(gaps)/1e6:.1f} ms, mean {sum(gaps)/max(len(gaps),1)/1e3:.1f} us")
