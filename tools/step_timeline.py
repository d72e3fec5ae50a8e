"""One DIP training step as a timeline, from a rocprofv3 kernel_trace.csv.

    python tools/step_timeline.py <run_kernel_trace.csv> [step_index_from_end=2]

A step starts at a k_sn_gram dispatch.  Prints every kernel of the chosen step in start order:
start offset and duration (us), queue, grid, name; then the step's wall time, the busy time of
each queue and the summed idle gaps between consecutive kernels of the first queue.
"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
back = int(sys.argv[2]) if len(sys.argv) > 2 else 2
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
starts = [i for i, r in enumerate(rows) if "k_sn_gram(" in r["Kernel_Name"]]
if len(starts) < back + 1:
    sys.exit("not enough steps in the trace")
a, b = starts[-back - 1], starts[-back]
step = rows[a:b]
t0 = int(step[0]["Start_Timestamp"])
qkey = "Queue_Id" if "Queue_Id" in step[0] else ("Stream_Id" if "Stream_Id" in step[0] else None)
busy = {}
print(f"{'start':>8} {'dur':>7} {'q':>3} {'s':>3} {'grid':>16}  kernel")
for r in step:
    s, e = int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0
    q = r.get(qkey, "?") if qkey else "?"
    busy[q] = busy.get(q, 0) + (e - s)
    grid = f"{r['Grid_Size_X']}x{r['Grid_Size_Y']}x{r['Grid_Size_Z']}"
    name = r["Kernel_Name"].replace("lrs::", "").split("(")[0][:70]
    sid = r.get("Stream_Id", "?")
    print(f"{s / 1e3:8.1f} {(e - s) / 1e3:7.1f} {q:>3} {sid:>3} {grid:>16}  {name}")
wall = int(rows[b]["Start_Timestamp"]) - t0
print(f"step wall {wall / 1e3:.1f} us, {len(step)} kernels; busy per queue: "
      + ", ".join(f"{q}: {v / 1e3:.1f} us" for q, v in busy.items()))
