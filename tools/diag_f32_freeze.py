"""One-off: the f32 frozen-encoder native step vs the Python schedule with the f32 tap kernel on and off,
per-layer count of weights that differ by more than 1e-6 after two steps."""
import sys
import numpy as np
import torch
sys.path.insert(0, ".")
sys.path.insert(0, "tests")
import _adipose_pkg  # noqa: E402,F401
import test_engine as T  # noqa: E402
from oracle import torch_ref as R  # noqa: E402
from adipose_amd import ops  # noqa: E402
from adipose_amd.engine import NativeAdiposeV3, train_cfg  # noqa: E402

w = R.adipose_v3_keras_weights(seed=865, deep_supervision=True)
for tap in (1, 0):
    ops.set_option("f32_tap", tap)
    for freeze in (True, False):
        x, y = T._train_data(7)
        net, tr = T._python_trainer(w, "f32", lr=1e-3, freeze=freeze)
        eng = NativeAdiposeV3(tile=T.S, max_batch=2, dtype="f32")
        eng.set_weights(w)
        xd, yd = torch.from_numpy(x).cuda(), torch.from_numpy(y).cuda()
        for step in range(2):
            tr.train_step(xd, yd)
            tr.read_metrics()
            eng.train_step(x, y, 1e-3, train_cfg(freeze_encoder=freeze))
        a, b = eng.get_weights(), net.get_weights()
        for k in a:
            for i, (u, v) in enumerate(zip(a[k], b[k])):
                d = np.abs(np.asarray(u, np.float32).ravel() - np.asarray(v, np.float32).ravel())
                nb = int((d > 1e-6).sum())
                if nb:
                    print(f"tap={tap} freeze={freeze} {k}[{i}] n_big={nb}/{d.size} worst={d.max():.3g}", flush=True)
        eng.close()
        print(f"tap={tap} freeze={freeze} done", flush=True)
