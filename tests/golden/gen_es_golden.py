"""Early-stopping golden: the reference's own get_DIP_out + EarlyStop + myMetric + torch_to_np
(main_LRS_PnP_DIP_1-LiP.py:71-118, 208-264), run in the BUILD CONTAINER only.

    python tests/golden/gen_es_golden.py

The four `def`s / the class are loaded from /root/reference with `ast` (no module-level code) and
get_DIP_out runs unmodified.  Its network is replaced by a recorder whose forward returns a fixed,
seeded output trajectory (so the ES decisions depend only on the trajectory, not on training), and
EarlyStop is subclassed only to log every check_stop(current, epoch) call.  Saved (es_golden.npz),
per trajectory k:
  traj{k}     (T, C, H, W) float32   the outputs the network "produced" at steps 0..T-1
  ret{k}      int64                  the step at which get_DIP_out returned (-1: ran out, returned None)
  var{k}      (n,) float64           every variance cur_var handed to check_stop (float32 numpy values)
  epoch{k}    (n,) int64             the matching epochs
  best{k}, best_epoch{k}, wait{k}    EarlyStop's final state
Nothing of the reference's source is saved.
"""
from __future__ import annotations

import ast
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference"
SCRIPT = "main_LRS_PnP_DIP_1-LiP.py"
C, H, W, T = 2, 12, 12, 170


def load_reference(extra):
    src = open(os.path.join(REF, SCRIPT)).read()
    keep = {"get_DIP_out", "torch_to_np", "myMetric", "EarlyStop"}
    body = [n for n in ast.parse(src).body
            if isinstance(n, (ast.FunctionDef, ast.ClassDef)) and n.name in keep]
    assert {n.name for n in body} == keep
    g = dict(extra)
    exec(compile(ast.Module(body=body, type_ignores=[]), os.path.join(REF, SCRIPT), "exec"), g)
    return g


def trajectories():
    rng = np.random.default_rng(2024)
    base = rng.random((C, H, W)).astype(np.float32)
    t = np.arange(T)
    amp = [
        0.2 * np.exp(-t / 20.0) + 0.002 * np.maximum(t - 70, 0),        # falls, then rises: stops
        0.3 / (1.0 + t / 8.0),                                          # keeps falling: never stops
        0.05 * (1.0 + 0.5 * np.sin(t / 6.0)),                           # oscillates: stops on a plateau
    ]
    out = []
    for a in amp:
        noise = rng.standard_normal((T, C, H, W)).astype(np.float32)
        out.append((base[None] + a[:, None, None, None].astype(np.float32) * noise).astype(np.float32))
    return out


def main():
    import torch

    trajs = trajectories()
    res = {}
    for k, traj in enumerate(trajs):
        calls = {"n": 0}

        class Recorder(torch.nn.Module):
            def __init__(self, *a, **kw):
                super().__init__()
                self.p = torch.nn.Parameter(torch.zeros(1))

            def cuda(self, *a, **kw):
                return self

            def forward(self, x):
                i = calls["n"]
                calls["n"] += 1
                return torch.from_numpy(traj[i][None].copy()) + 0.0 * self.p

        log = []
        g = load_reference({"torch": torch, "np": np, "my_Lipschitz_Unet": Recorder,
                            "mask_bkg": torch.ones(1, 1, H, W), "print": lambda *a, **kw: None})
        Base = g["EarlyStop"]
        holder = {}

        class LoggedEarlyStop(Base):
            def __init__(self, *a, **kw):
                super().__init__(*a, **kw)
                holder["es"] = self

            def check_stop(self, current, cur_epoch):
                log.append((float(current), int(cur_epoch), type(current).__name__))
                return super().check_stop(current, cur_epoch)

        g["EarlyStop"] = LoggedEarlyStop
        x = torch.zeros(1, C, H, W)
        out = g["get_DIP_out"](torch.zeros(1, C, H, W), x, num_iter=T, learning_rate=0.1, show_every=1)
        ret = calls["n"] - 1 if out is not None else -1
        es = holder["es"]
        print(f"trajectory {k}: returned at step {ret}, {len(log)} checks, best {es.best_score:.6e} at "
              f"{es.best_epoch}, variance dtype {log[0][2] if log else '-'}")
        res[f"traj{k}"] = traj
        res[f"ret{k}"] = np.int64(ret)
        res[f"var{k}"] = np.array([v for v, _, _ in log], np.float64)
        res[f"epoch{k}"] = np.array([e for _, e, _ in log], np.int64)
        res[f"best{k}"] = np.float64(es.best_score)
        res[f"best_epoch{k}"] = np.int64(es.best_epoch)
        res[f"wait{k}"] = np.int64(es.wait_count)
    res["size"], res["patience"] = np.int64(30), np.int64(60)
    np.savez_compressed(os.path.join(HERE, "es_golden.npz"), **res)


if __name__ == "__main__":
    sys.exit(main())
