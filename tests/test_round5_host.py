"""CPU tests of round-5 host utilities: the hard synthetic histology set behind the bench's Dice@val leg
(data.synthetic_tile_hard / synthetic_stream_hard) and the timed-step kernel breakdown (tools/kstats.py)."""
import csv
import json
import os
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def test_hard_synthetic_tiles_are_seeded_and_not_trivial():
    """Same seed -> the same tiles; different seeds -> different tiles; uint8 RGB images and {0, 1} masks whose fat
    fraction sits well inside (0, 1) (a task that neither all-background nor all-fat solves)."""
    import _adipose_pkg  # noqa: F401
    from adipose_amd.data import synthetic_stream_hard
    x1, y1 = synthetic_stream_hard(11, 2, 128)
    x2, y2 = synthetic_stream_hard(11, 2, 128)
    x3, _ = synthetic_stream_hard(12, 2, 128)
    assert tuple(x1.shape) == (2, 128, 128, 3) and tuple(y1.shape) == (2, 128, 128)
    assert str(x1.dtype) == "torch.uint8" and str(y1.dtype) == "torch.float32"
    assert (x1 == x2).all() and (y1 == y2).all()
    assert not (x1 == x3).all()
    vals = set(np.unique(y1.numpy()).tolist())
    assert vals <= {0.0, 1.0}
    frac = float(y1.mean())
    assert 0.1 < frac < 0.9, frac
    # stain noise: the image is not a function of the mask alone (fat pixels are not one colour)
    fat = x1.numpy()[y1.numpy() > 0.5]
    assert fat.std(axis=0).min() > 2.0


def _trace(path, steps, warmup, kernels_per_step):
    """A fake rocprofv3 kernel trace: (warmup + steps) steps of `kernels_per_step` (name, duration) launches, each step
    ending with adam_kernel, 1 us gaps; plus 5 allocation fills before the first step."""
    rows, t = [], 1000
    for i in range(5):
        rows.append({"Kernel_Name": "fill_kernel(float*)", "Start_Timestamp": t, "End_Timestamp": t + 500})
        t += 600
    for _ in range(warmup + steps):
        for name, dur in kernels_per_step + [("adam_kernel(float*)", 2000)]:
            rows.append({"Kernel_Name": name, "Start_Timestamp": t, "End_Timestamp": t + dur})
            t += dur + 1000
    with open(path, "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=["Kernel_Name", "Start_Timestamp", "End_Timestamp"])
        w.writeheader()
        w.writerows(rows)


def test_kstats_counts_only_the_timed_steps(tmp_path):
    kp = [("void igemm_fwd_halop_kernel<false, 1, 64>(FwdArgs)", 100000), ("bn_apply_kernel(float*)", 20000)]
    tr = tmp_path / "kt_kernel_trace.csv"
    _trace(tr, steps=4, warmup=2, kernels_per_step=kp)
    bench = tmp_path / "bench.json"
    bench.write_text(json.dumps({"warmup": 2, "steps": 4, "ms_per_step": 0.125}) + "\n")
    out = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "kstats.py"), str(tr), str(bench)],
                         capture_output=True, text=True, check=True).stdout
    assert "timed steps only: 4 steps after 2 warm-up steps" in out
    line = [ln for ln in out.splitlines() if ln.startswith("igemm_fwd_halop_kernel")][0]
    assert "calls/step=  1.00" in line and "avg=    100.0us" in line
    assert "fill_kernel" not in out   # (allocation fills before the first step are not step time)
    # kernel time per step 0.100 + 0.020 + 0.002 ms; the span adds the three 1-us gaps of a step
    assert "kernel time per step: 0.122 ms" in out
    assert "wall span per step (kernels + gaps): 0.125 ms" in out


def test_kstats_rejects_a_short_trace(tmp_path):
    tr = tmp_path / "kt_kernel_trace.csv"
    _trace(tr, steps=2, warmup=1, kernels_per_step=[("k_kernel(float*)", 1000)])
    bench = tmp_path / "bench.json"
    bench.write_text(json.dumps({"warmup": 2, "steps": 4, "ms_per_step": 1.0}) + "\n")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "kstats.py"), str(tr), str(bench)],
                       capture_output=True, text=True)
    assert r.returncode != 0 and "adam_kernel" in (r.stderr + r.stdout)
