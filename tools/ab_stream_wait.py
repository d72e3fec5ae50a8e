"""A/B of the stream orderings of the outer iteration (the DIP stream against the caller's, the
low-rank stream against the main one): lrs_stream_wait (device-scope event) vs torch's wait_stream,
on a bench line (configs[2] by default, --workload pnp configs[1]), interleaved rounds in one process.

    python tools/ab_stream_wait.py [--rounds 3] [--steps 3] [--workload dip|pnp]"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "lrs-pnp-dip_amd"))

ap = argparse.ArgumentParser()
ap.add_argument("--rounds", type=int, default=3)
ap.add_argument("--steps", type=int, default=3)
ap.add_argument("--workload", default="dip", choices=["dip", "pnp"])
a = ap.parse_args()
sys.argv = ["bench.py", "--steps", str(a.steps), "--warmup", "1" if a.workload == "dip" else "2", "--no-cpu-baseline",
            "--workload", a.workload]
import bench  # noqa: E402
from lrspnp import dip, dist as D  # noqa: E402

args = bench.parse()
ctx = D.init_from_env(args.backend)
for r in range(a.rounds):
    for flag in (False, True):
        dip.DEVICE_SCOPE_WAITS = flag
        out = (bench.main_dip if a.workload == "dip" else bench.main_pnp)(args, ctx)
        print(f"round {r} {'lrs_stream_wait' if flag else 'torch wait_stream'}: {out['value']:.4f} outer it/s, "
              f"{out['ms_per_step']:.2f} ms", flush=True)
