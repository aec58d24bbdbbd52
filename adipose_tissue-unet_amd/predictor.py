"""Inference surface: predictor, batched test-time augmentation, sliding-window + blending.

Mirrors (same names, arguments, return values):
  * AdiposeUNet / predict_single / predict   segmentation_inference.py:83-158,
                                              full_evaluation_enhanced.py:1157-1353
  * TestTimeAugmentation                      segmentation_inference.py:181-229,
                                              full_evaluation_enhanced.py:522-600
  * SlidingWindowInference, GaussianBlender,  full_evaluation_enhanced.py:115-329
    LinearBlender

MI355X-first differences (same results): all TTA views of a tile run as ONE batched forward (the
view transform is folded into adp_prep_input's load, the inverse transform + mean into adp_tta_merge),
sliding-window tiles are read in place from the HBM-resident image, several tiles x views are batched
per forward, and blending accumulates on the GPU (adp_blend_accum). With a torch.distributed process
group, sliding-window positions are sharded by contiguous tile rows across ranks; each rank blends its tiles
into a ROW BAND of the frame (its tiles' rows plus the tile overlap) and the bands are added into rank 0's frame
by point-to-point transfers in rank order (BandCanvas; SURVEY.md §8e: a reduce of row-band buffers to rank 0, RCCL
having no gather), so no rank but 0 holds a full-frame canvas (BASELINE.json config 4).
"""
from __future__ import annotations

import math
import time

import numpy as np
import torch

from . import ops
from .nets import AdiposeV3Net

INFER_CPAD = (64, 64, 64, 64)   # adipose_v3 channel-stride granule per level for bf16 inference (nets.py)
TTA_VIEWS = {"minimal": [0, 4], "basic": [0, 4, 5, 1], "full": [0, 1, 2, 3, 4, 5, 6, 7]}


def _to_dev(image, device):
    """Host arrays are uploaded once; device tensors (possibly strided windows) are used in place."""
    if isinstance(image, np.ndarray):
        return torch.from_numpy(np.ascontiguousarray(image, dtype=np.float32)).to(device)
    if image.dtype != torch.float32 or not image.is_cuda:
        raise TypeError("device images must be float32 CUDA tensors")
    return image


class HipUnetPredictor:
    """GPU predictor: predict_single(image, mean, std) -> (S,S) float32 probabilities (main_out)."""

    def __init__(self, net, max_batch=8):
        self.net = net
        self.device = net.device
        self.max_batch = max_batch
        self._packed_step = None

    @property
    def use_deep_supervision(self):
        return getattr(self.net, "ds", False)

    def _forward(self, batch):
        net = self.net
        outs = net.forward(batch, train=False, pack=True)
        return outs["main_out"]

    def predict_views(self, images, mean, std, views):
        """images: list/tensor of (S,S) tiles (device or host, may be strided windows); returns
        (len(images), S, S) device tensor of TTA-merged probabilities."""
        n_img = len(images)
        nv = len(views)
        S = images[0].shape[-1]
        out = torch.empty((n_img, S, S), dtype=torch.float32, device=self.device)
        per = max(1, self.max_batch // nv)
        for i0 in range(0, n_img, per):
            chunk = images[i0:i0 + per]
            B = len(chunk) * nv
            a = self.net.acts(B)
            for t, img in enumerate(chunk):
                src = _to_dev(img, self.device)[None]
                for k, v in enumerate(views):
                    ops.prep_input(src, a["x"][t * nv + k: t * nv + k + 1], mean=mean, std=std, view=v)
            p = self._forward(B)
            for t in range(len(chunk)):
                if nv == 1:
                    ops.cast(p[t], out[i0 + t])
                else:
                    ops.tta_merge(p[t * nv:(t + 1) * nv], views, out[i0 + t])
        return out

    def predict_single(self, image, mean, std):
        """segmentation_inference.py:153-158 — returns a new float32 numpy array."""
        return self.predict_views([image], mean, std, [0])[0].cpu().numpy()


class AdiposeUNet:
    """Inference wrapper with the reference's method surface (build_model / load_weights /
    predict_single / predict). ``dtype='f32'`` reproduces the reference's fp32 numerics."""

    def __init__(self, tile_size=1024, dtype="f32", device="cuda", max_batch=8):
        self.net = None
        self.use_deep_supervision = False
        self.tile_size = tile_size
        self.dtype = dtype
        self.device = device
        self.max_batch = max_batch
        self._pred = None

    def build_model(self, init_nb: int = 44, dropout_rate: float = 0.3, use_deep_supervision: bool = False):
        self.use_deep_supervision = use_deep_supervision
        # inference layout: 64/128/192/384 strides put every level on the persistent halo / tap64 kernels
        # (432 tiles/s at 1024^2 vs 377 for 48/88 strides on the full-resolution levels)
        cpad = INFER_CPAD if self.dtype == "bf16" else None
        self.net = AdiposeV3Net(1, self.tile_size, dtype=self.dtype, device=self.device, init_nb=init_nb, cpad=cpad,
                                dropout_rate=dropout_rate, deep_supervision=use_deep_supervision)
        self._pred = HipUnetPredictor(self.net, self.max_batch)
        return self.net

    def load_weights(self, weights_path: str):
        from .checkpoint import load_weights
        load_weights(self.net, weights_path, by_name=True, skip_mismatch=False)
        print(f"✓ Loaded weights from {weights_path}")

    def predict_single(self, image, mean, std):
        return self._pred.predict_single(image, mean, std)

    def predict_views(self, images, mean, std, views):
        return self._pred.predict_views(images, mean, std, views)

    def predict(self, image, mean, std, use_tta=False, tta_mode="basic"):
        """full_evaluation_enhanced.py:1323-1353 -> (pred, timing_info)"""
        t0 = time.time()
        if not use_tta:
            pred = self.predict_single(image, mean, std)
            return pred, {"num_augmentations": 1, "total_time": time.time() - t0, "tta_enabled": False}
        tta = TestTimeAugmentation(mode=tta_mode)
        pred, info = tta.predict_with_tta(self, image, mean, std, return_timing=True)
        info["tta_enabled"] = True
        info["tta_mode"] = tta_mode
        return pred, info


class TestTimeAugmentation:
    """D4-subset TTA. With a GPU predictor (has ``predict_views``) all views run as one batch;
    any other duck-typed predictor gets the reference's per-view host loop."""

    __test__ = False  # not a pytest class

    def __init__(self, mode: str = "basic"):
        mode = (mode or "basic").lower()
        if mode not in TTA_VIEWS:
            mode = "basic"
        self.mode = mode
        self.views = TTA_VIEWS[mode]
        r = lambda k: (lambda x: np.rot90(x, k))  # noqa: E731
        fh = lambda x: np.flip(x, 1)  # noqa: E731
        fv = lambda x: np.flip(x, 0)  # noqa: E731
        table = {0: (lambda x: x, lambda x: x), 1: (r(1), r(3)), 2: (r(2), r(2)), 3: (r(3), r(1)), 4: (fh, fh),
                 5: (fv, fv), 6: (lambda x: fh(np.rot90(x, 1)), lambda x: np.rot90(fh(x), 3)),
                 7: (lambda x: fv(np.rot90(x, 1)), lambda x: np.rot90(fv(x), 3))}
        self.transforms = [table[v] for v in self.views]

    def predict_with_tta(self, model, image, mean, std, return_timing=False):
        start = time.time()
        if hasattr(model, "predict_views"):
            avg = model.predict_views([image], mean, std, self.views)[0].cpu().numpy()
        else:
            preds = [deaug(model.predict_single(aug(image), mean, std)).astype(np.float32)
                     for aug, deaug in self.transforms]
            avg = np.mean(preds, axis=0).astype(np.float32)
        if return_timing:
            return avg, {"num_augmentations": len(self.views), "total_time": time.time() - start}
        return avg


class GaussianBlender:
    """full_evaluation_enhanced.py:115-183 — w = exp(-r^2 / (2 (0.25 T)^2)) normalised to max 1."""

    def __init__(self, tile_size: int = 1024, sigma_factor: float = 0.25):
        self.tile_size = tile_size
        self.sigma = tile_size * sigma_factor
        c = tile_size / 2
        y, x = np.ogrid[0:tile_size, 0:tile_size]
        w = np.exp(-((x - c) ** 2 + (y - c) ** 2) / (2 * self.sigma ** 2))
        self.weight_map = (w / w.max()).astype(np.float32)
        self._dev = {}
        self.floor = 1e-8

    def device_weights(self, device, th=None, tw=None):
        key = (str(device), th, tw)
        if key not in self._dev:
            w = self.weight_map if th is None else self.weight_map[:th, :tw]
            self._dev[key] = torch.from_numpy(np.ascontiguousarray(w)).to(device)
        return self._dev[key]

    def reconstruct(self, tiles, positions, output_shape):
        return _gpu_reconstruct(self, tiles, positions, output_shape)


class LinearBlender:
    """full_evaluation_enhanced.py:186-204 — plain average (count floor 1)."""

    floor = 1.0

    def device_weights(self, device, th=None, tw=None):
        return None

    def reconstruct(self, tiles, positions, output_shape):
        return _gpu_reconstruct(self, tiles, positions, output_shape)


def band_rows(positions, tile):
    """Rows [y0, y1) the tiles at `positions` (top-left corners) cover; (0, 0) for none."""
    if not positions:
        return 0, 0
    return min(y for y, _ in positions), max(y for y, _ in positions) + tile


def _p2p_cpu(group):
    import torch.distributed as dist
    return dist.get_backend(group) == "gloo"   # (gloo's send / recv take host tensors)


class BandCanvas:
    """Blend accumulators (acc, wsum) of one (H, W) output plane, held for rows [y0, y1) only.

    Sharded sliding-window inference (the path it shards is full_evaluation_enhanced.py:286-329):
    every rank but 0 allocates just the band its tiles cover (their rows plus the tile overlap) and blends into it at
    row offset y0; rank 0 holds the whole frame (band (0, H)). reduce_to_root() adds the other ranks' bands into
    rank 0's frame in rank order -- one send of the 2 x band buffer per rank, received and added by rank 0 -- so the
    sum's association depends only on the sharding (deterministic), and the result equals the one-rank canvas up to
    f32 rounding of the different association. Full-frame worst case per rank before: 2 x H x W f32 (512 MiB at
    8192^2); now 2 x band x W on ranks > 0."""

    def __init__(self, shape, rows, device):
        H, W = int(shape[0]), int(shape[1])
        self.H, self.W = H, W
        self.y0, self.y1 = int(rows[0]), int(max(rows[0], rows[1]))
        self.buf = torch.zeros((2, self.y1 - self.y0, W), dtype=torch.float32, device=device)
        self.acc, self.ws = self.buf[0], self.buf[1]

    def add(self, tile, weight, y, x):
        ops.blend_accum(tile, weight, self.acc, self.ws, y - self.y0, x)

    def reduce_to_root(self, group, bands):
        """bands[q]: rows (y0, y1) of rank q's band (rank 0: its frame). Returns True on rank 0, whose (acc, ws)
        then hold the sums over all ranks; the other ranks send their band and return False."""
        import torch.distributed as dist
        r, n = dist.get_rank(group), dist.get_world_size(group)
        host = _p2p_cpu(group)
        if r != 0:
            if self.y1 > self.y0:
                dist.send(self.buf.cpu() if host else self.buf, dist.get_global_rank(group, 0), group=group)
            return False
        if (self.y0, self.y1) != (0, self.H):
            raise ValueError("rank 0's canvas must cover the whole frame")
        # every band's receive is posted at once (round 6), so the transfers overlap; the adds still run in rank order
        # (waiting on rank q while the later bands keep arriving): the sum's association stays the sharding's
        posted = []
        for q in range(1, n):
            y0, y1 = int(bands[q][0]), int(bands[q][1])
            if y1 <= y0:
                continue
            tmp = torch.empty((2, y1 - y0, self.W), dtype=torch.float32, device="cpu" if host else self.buf.device)
            posted.append((y0, y1, tmp, dist.irecv(tmp, dist.get_global_rank(group, q), group=group)))
        for y0, y1, tmp, work in posted:
            work.wait()
            tmp = tmp.to(self.buf.device)
            for k in range(2):
                dst = self.buf[k, y0:y1]
                if dst.is_cuda and dst.numel() % 8 == 0:
                    ops.add_mask(dst, dst, b=tmp[k])
                else:
                    dst.add_(tmp[k])
        return True

    def finalize(self, floor_):
        out = torch.empty_like(self.acc)
        ops.blend_finalize(self.acc, self.ws, out, floor_)
        return out


def _bcast_frame(frame, shape, dev, group):
    """Rank 0's finished (H, W) map to every rank of `group` (frame = None on the receiving ranks)."""
    import torch.distributed as dist
    host = _p2p_cpu(group)
    buf = frame if frame is not None else torch.empty(shape, dtype=torch.float32, device=dev)
    tb = buf.cpu() if host else buf
    dist.broadcast(tb, dist.get_global_rank(group, 0), group=group)
    return tb.to(dev) if host else tb


def _gpu_reconstruct(blender, tiles, positions, output_shape):
    dev = torch.device("cuda", torch.cuda.current_device())
    h, w = output_shape
    acc = torch.zeros((h, w), dtype=torch.float32, device=dev)
    ws = torch.zeros((h, w), dtype=torch.float32, device=dev)
    for t, (y, x) in zip(tiles, positions):
        td = _to_dev(t, dev)
        th, tw = td.shape
        if th != tw:
            raise ValueError("blend tiles must be square")
        ops.blend_accum(td, blender.device_weights(dev, th, tw), acc, ws, y, x)
    out = torch.empty_like(acc)
    ops.blend_finalize(acc, ws, out, blender.floor)
    return out.cpu().numpy()


class SlidingWindowInference:
    """full_evaluation_enhanced.py:207-329 with GPU batching / blending and optional rank sharding."""

    def __init__(self, tile_size: int = 1024, overlap: float = 0.5, blend_mode: str = "gaussian",
                 process_group=None, verbose=True):
        self.tile_size = tile_size
        self.overlap = max(0.0, min(overlap, 0.75))
        self.stride = int(tile_size * (1 - self.overlap))
        self.blend_mode = blend_mode
        self.blender = GaussianBlender(tile_size) if blend_mode == "gaussian" else LinearBlender()
        self.group = process_group
        if verbose:
            print(f"[SlidingWindow] Initialized: tile={tile_size}, stride={self.stride}, "
                  f"overlap={overlap:.1%}, blend={blend_mode}")

    def extract_tile_positions(self, image_shape):
        h, w = image_shape[:2]
        T, s = self.tile_size, self.stride
        ys = max(1, math.ceil((h - T) / s) + 1)
        xs = max(1, math.ceil((w - T) / s) + 1)
        pos = []
        for yi in range(ys):
            for xi in range(xs):
                y = min(yi * s, h - T)
                x = min(xi * s, w - T)
                if y >= 0 and x >= 0 and y + T <= h and x + T <= w:
                    pos.append((y, x))
        return pos

    def extract_tiles(self, image):
        pos = self.extract_tile_positions(image.shape)
        T = self.tile_size
        return [image[y:y + T, x:x + T] for y, x in pos], pos

    def shard(self, positions, rank=None):
        """Contiguous runs of tile positions per rank (tile rows stay together)."""
        if self.group is None:
            return positions
        import torch.distributed as dist
        r, n = dist.get_rank(self.group) if rank is None else rank, dist.get_world_size(self.group)
        per = math.ceil(len(positions) / n)
        return positions[r * per:(r + 1) * per]

    def predict_with_sliding_window(self, image, model, mean, std, use_tta=False, tta_mode="basic",
                                    return_device=False, broadcast=False):
        """The blended probability map of `image` (full_evaluation_enhanced.py:286-329).

        With a process group (rank-sharded tiles, round 5): the bands are reduced to rank 0, which returns the map;
        the other ranks return None unless broadcast=True, which sends rank 0's finished map to every rank (one
        H x W f32 broadcast) so that every rank returns it, as the single-process call does."""
        if not hasattr(model, "predict_views"):
            raise TypeError("GPU sliding window needs a HIP predictor (AdiposeUNet / HipUnetPredictor)")
        dev = model.net.device if hasattr(model, "net") else torch.device("cuda")
        img = _to_dev(image, dev)
        h, w = img.shape
        T = self.tile_size
        positions = self.extract_tile_positions((h, w))
        mine = self.shard(positions)
        views = TTA_VIEWS[(tta_mode or "basic").lower()] if use_tta else [0]
        bands = None
        if self.group is None:
            canvas = BandCanvas((h, w), (0, h), dev)
        else:   # rank 0: the frame; others: the row band of their tiles
            import torch.distributed as dist
            n = dist.get_world_size(self.group)
            bands = [(0, h)] + [band_rows(self.shard(positions, q), T) for q in range(1, n)]
            canvas = BandCanvas((h, w), bands[dist.get_rank(self.group)], dev)
        wmap = self.blender.device_weights(dev, T, T)
        per = max(1, getattr(model, "max_batch", 8) // len(views))
        for i0 in range(0, len(mine), per):
            chunk = mine[i0:i0 + per]
            tiles = [img[y:y + T, x:x + T] for y, x in chunk]
            probs = model.predict_views(tiles, mean, std, views)
            for (y, x), p in zip(chunk, probs):
                canvas.add(p, wmap, y, x)
        if self.group is not None and not canvas.reduce_to_root(self.group, bands):
            if not broadcast:
                return None   # (the blended frame lives on rank 0 only)
            out = _bcast_frame(None, (h, w), dev, self.group)
        else:
            out = canvas.finalize(self.blender.floor)
            if self.group is not None and broadcast:
                _bcast_frame(out, (h, w), dev, self.group)
        return out if return_device else out.cpu().numpy()
