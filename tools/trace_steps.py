"""Per-step anatomy of DIP training steps from a rocprofv3 kernel trace (the rocpd .db that
`rocprofv3 --kernel-trace` writes, or its kernel_trace.csv): steps are delimited by k_adam.  Prints,
averaged over the last --steps steps, the step wall, per-queue busy time, the idle time of the
union of queues (no kernel running anywhere), the launch-to-launch gaps on each queue, and the
kernel count.  With --timeline, the last step kernel by kernel.

    python tools/trace_steps.py gpurun_out/d1/trace_g36/run_results.db [--steps 10] [--timeline]
"""
import argparse
import csv
import sqlite3
import statistics


def load(path):
    if path.endswith(".db"):
        c = sqlite3.connect(path)
        rows = c.execute("select name, queue_id, start, end, grid_x, grid_y, grid_z from kernels order by start").fetchall()
        return [dict(name=r[0], q=r[1], s=r[2], e=r[3], grid=f"{r[4]}x{r[5]}x{r[6]}") for r in rows]
    out = []
    with open(path) as f:
        for r in csv.DictReader(f):
            out.append(dict(name=r["Kernel_Name"], q=int(r["Queue_Id"]), s=int(r["Start_Timestamp"]),
                            e=int(r["End_Timestamp"]), grid=f"{r['Grid_Size_X']}x{r['Grid_Size_Y']}x{r['Grid_Size_Z']}"))
    return sorted(out, key=lambda k: k["s"])


def short(n):
    n = n.split("(")[0]
    return n.replace("void ", "").replace("lrs::", "").replace("(anonymous namespace)::", "")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("path")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--timeline", action="store_true")
    a = ap.parse_args()
    ks = load(a.path)
    adam = [i for i, k in enumerate(ks) if "k_adam" in k["name"]]
    if len(adam) < a.steps + 1:
        raise SystemExit(f"only {len(adam)} k_adam launches")
    res = []
    for t in range(len(adam) - a.steps, len(adam)):
        lo, hi = adam[t - 1] + 1, adam[t] + 1
        step = ks[lo:hi]
        t0, t1 = ks[adam[t - 1]]["e"], ks[adam[t]]["e"]
        busy = {}
        for k in step:
            busy[k["q"]] = busy.get(k["q"], 0) + (k["e"] - k["s"])
        # idle time of the union of all queues
        iv = sorted((k["s"], k["e"]) for k in step)
        idle, cur = 0, t0
        for s, e in iv:
            if s > cur:
                idle += s - cur
            cur = max(cur, e)
        idle += max(0, t1 - cur)
        res.append(dict(wall=t1 - t0, busy=busy, idle=idle, n=len(step), step=step, t0=t0))
    med = lambda f: statistics.median(f(r) for r in res)
    print(f"{a.path}: last {a.steps} steps")
    print(f"  wall {med(lambda r: r['wall']) / 1e3:.1f} us, kernels {med(lambda r: r['n'])}, "
          f"all-queues idle {med(lambda r: r['idle']) / 1e3:.1f} us")
    qs = sorted({q for r in res for q in r["busy"]})
    for q in qs:
        print(f"  queue {q}: busy {med(lambda r: r['busy'].get(q, 0)) / 1e3:.1f} us")
    if a.timeline:
        r = res[-1]
        print(f"{'start':>8} {'dur':>7} {'gap':>6} {'q':>3} {'grid':>16}  kernel")
        last = {}
        for k in r["step"]:
            gap = (k["s"] - last[k["q"]]) / 1e3 if k["q"] in last else 0.0
            last[k["q"]] = k["e"]
            print(f"{(k['s'] - r['t0']) / 1e3:8.1f} {(k['e'] - k['s']) / 1e3:7.1f} {gap:6.1f} {k['q']:3d} {k['grid']:>16}  {short(k['name'])[:70]}")


if __name__ == "__main__":
    main()
