"""GPU-side cost of a cross-stream fork (event record on the main stream + wait on a side stream).

A chain of dependent ~15-us matmuls on the main stream, with and without a fork after every one
(the side stream waits on the event and runs a small matmul): the main chain's extra time per fork
is what a fork costs the critical path.  Host enqueue stays far ahead (the GPU is the bottleneck)."""
import time

import torch

torch.cuda.set_device(0)
n, reps = 1536, 200
a = torch.randn(n, n, device="cuda")
b = torch.randn(n, n, device="cuda") / n ** 0.5
c = torch.randn(256, 256, device="cuda")
main = torch.cuda.current_stream()
side = torch.cuda.Stream()
evs = [torch.cuda.Event() for _ in range(reps)]


def run(mode):
    x = a
    for i in range(reps):
        x = x @ b
        if mode >= 1:
            evs[i].record(main)
            if mode == 2:
                side.wait_event(evs[i])
                with torch.cuda.stream(side):
                    c @ c
    if mode == 2:
        main.wait_stream(side)
    return x


for mode in (0, 1, 2, 0, 1, 2):
    run(mode)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    t0 = time.perf_counter()
    run(mode)
    t1 = time.perf_counter()
    e1.record()
    torch.cuda.synchronize()
    name = ["plain", "record only", "record + side wait + side kernel"][mode]
    print(f"{name:34s} {e0.elapsed_time(e1) / reps * 1e3:8.2f} us per step (host {1e6 * (t1 - t0) / reps:6.1f} us)")
