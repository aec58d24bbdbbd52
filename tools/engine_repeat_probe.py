#!/usr/bin/env python3
"""Run-to-run spread of the native unet_bn f32 training step (csrc/engine.cpp) in one process: two handles on the
same weights and tiles (one with a one-rank RCCL communicator, i.e. the bucketed all-reduce on its own stream, when
--comm), several steps, each step started from the same weights on both handles; prints per step the layers whose
gradients differ beyond rounding (cosine, largest element error relative to the layer's largest gradient).
Localises an intermittent mismatch of tests/test_engine.py::test_native_unet_bn_bucketed_comm_and_errors.

    python tools/engine_repeat_probe.py [--reps 6] [--comm 1]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import _adipose_pkg  # noqa: E402,F401

import numpy as np  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=6)
    ap.add_argument("--comm", type=int, default=1)
    args = ap.parse_args()
    from adipose_amd.engine import NativeUNetBN, comm_destroy, comm_init, comm_unique_id, train_cfg
    from tests.test_engine import _bn_case
    L, S_, B, lr = 3, 64, 2, 1e-3
    w, x, y = _bn_case(L, S_, B, seed=6)
    a = NativeUNetBN(tile=S_, max_batch=B, dtype="f32", levels=L)
    b = NativeUNetBN(tile=S_, max_batch=B, dtype="f32", levels=L)
    a.set_weights(w)
    b.set_weights(w)
    comm = None
    if args.comm:
        comm = comm_init(1, comm_unique_id(), 0)
        b.set_comm(comm)
    cfg = train_cfg(use_hard_mining=False)
    for rep in range(args.reps):
        b.set_weights(a.get_weights())
        a.train_step(x, y, lr, cfg)
        b.train_step(x, y, lr, cfg)
        ga, gb = a.get_grads(), b.get_grads()
        worst, bad = (1.0, 0.0, ""), []
        for n in ga:
            for si, (u, v) in enumerate(zip(ga[n], gb[n])):
                u, v = np.asarray(u, np.float64).ravel(), np.asarray(v, np.float64).ravel()
                c = float(u @ v / (np.linalg.norm(u) * np.linalg.norm(v) + 1e-30))
                r = float(np.abs(u - v).max() / max(np.abs(v).max(), 1e-12))
                if r > worst[1]:
                    worst = (c, r, f"{n}/{si}")
                if r > 1e-3:
                    i = int(np.abs(u - v).argmax())
                    bad.append((n, si, round(c, 7), round(r, 5), i, float(u[i]), float(v[i]), u.size))
        print(f"rep {rep}: worst {worst[2]} cos {worst[0]:.7f} rel {worst[1]:.2e}; beyond 1e-3: {bad}", flush=True)
    if comm is not None:
        b.set_comm(None)
        comm_destroy(comm)
    a.close()
    b.close()


if __name__ == "__main__":
    main()
