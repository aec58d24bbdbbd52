"""One-off: run-to-run spread of the unet_bn bf16 per-layer gradients (same net, same weights and batch, five
forward + backward passes, no optimizer step) under wgrad_bna_maxch = 1 and 2, and against the f32 oracle."""
import sys
import torch
sys.path.insert(0, ".")
sys.path.insert(0, "tests")
import _adipose_pkg  # noqa: E402,F401
import test_gpu_network as T  # noqa: E402
from oracle import torch_ref as R  # noqa: E402
from adipose_amd import ops  # noqa: E402
from adipose_amd.nets import UNetBN  # noqa: E402
from adipose_amd.trainer import LossConfig, Trainer  # noqa: E402

B, L, S = 2, 3, 64
w = R.unet_bn_keras_weights(levels=L, base=64, in_ch=3, seed=5)
x, y = T.synth_batch(B, S, C=3, seed=9)
for maxch in (1, 2, 0):
    ops.set_option("wgrad_bna_maxch", maxch)
    if maxch == 0:
        ops.set_option("wgrad_bna", 0)
    net = UNetBN(B, S, levels=L, base=64, in_ch=3, dtype="bf16", device="cuda")
    net.set_weights(w)
    tr = Trainer(net, LossConfig(use_hard_mining=False))
    runs = []
    for step in range(5):
        T._unet_bn_step(net, tr, x, y, B)
        runs.append({n: [torch.as_tensor(g).double().flatten() for g in net.get_layer_grads(n)] for n in w})
    worst = {}
    for r in runs[1:]:
        for n in w:
            for si, (a, b) in enumerate(zip(runs[0][n], r[n])):
                c = float(a @ b / (a.norm() * b.norm() + 1e-30))
                worst[(n, si)] = min(worst.get((n, si), 1.0), c)
    low = sorted(worst.items(), key=lambda kv: kv[1])[:6]
    print("maxch", maxch, "lowest run-to-run cosines", [(k[0], k[1], round(v, 5)) for k, v in low], flush=True)
    ops.set_option("wgrad_bna_maxch", None)
    ops.set_option("wgrad_bna", None)
    del net, tr
