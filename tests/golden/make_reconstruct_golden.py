"""Golden vectors for full-slide reconstruction (Segmentation/reconstruct_full_images.py), generated HERE
from the reference's own functions. The module imports cv2 / tifffile / tensorflow at load time; none is
installed (ordinary ImportError), so they are satisfied by make_golden's inert stubs and, for the two
calls reconstruct_slide makes, by a small in-memory file table:
  cv2.imread(path, IMREAD_GRAYSCALE) -> the tile's PIL "L" conversion (the build reads tiles with PIL,
  so the golden pins everything after decoding); cv2.imread(path, IMREAD_COLOR) -> the tile as BGR;
  cv2.cvtColor(BGR2RGB) -> channel reversal; tifffile.imread(path) -> the mask array.
Model: make_golden.fake_predictor (deterministic, asymmetric). Data only is written
(tests/golden/reconstruct.npz); no reference source is stored. Usage:
    python tests/golden/make_reconstruct_golden.py [/root/reference]
"""
import contextlib
import io
import os
import sys
import tempfile
import types
from pathlib import Path

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import make_golden  # noqa: E402

REF = sys.argv[1] if len(sys.argv) > 1 else "/root/reference"
T, STRIDE = 64, 32


def slide_cases(rng):
    """(slide_id, grid rows, grid cols, missing tiles, tiles without mask, mask scale, full_shape)"""
    return [("slideA", 3, 3, set(), set(), 255.0, (128, 128)),
            ("slide_B x", 3, 4, {(1, 2)}, {(0, 1), (2, 3)}, 1.0, (100, 130))]


def main():
    make_golden.REF = REF
    fe, _ = make_golden.load_reference()
    import reconstruct_full_images as rf  # noqa: E402
    from PIL import Image
    rng = np.random.default_rng(2024)
    files = {}
    masks = {}
    rf.cv2 = types.SimpleNamespace(
        IMREAD_GRAYSCALE=0, IMREAD_COLOR=1, COLOR_BGR2RGB=4,
        imread=lambda p, flag: files[p][0] if flag == 0 else files[p][1][..., ::-1].copy(),
        cvtColor=lambda a, code: a[..., ::-1].copy())
    rf.tiff = types.SimpleNamespace(imread=lambda p: masks[p])
    rf.tqdm = lambda it, **k: it
    out = {}
    quiet = contextlib.redirect_stdout(io.StringIO())
    names = ["6 BEEF Shoulder -1_grid_5x5_r1_c2_r0_c1.jpg", "slide_name_r5_c3.jpg", "a_r10_c0.png",
             "bad_name.jpg", "x_rA_c1.jpg", "r1_c2.jpg", "only_c3.jpg"]
    parsed = []
    for n in names:
        try:
            s, r, c = rf.parse_tile_filename(n)
            parsed.append(f"{s}|{r}|{c}")
        except ValueError:
            parsed.append("ValueError")
    out["parse_names"], out["parse_out"] = np.array(names), np.array(parsed)
    with tempfile.TemporaryDirectory() as td:
        img_dir, msk_dir = Path(td) / "images", Path(td) / "masks"
        img_dir.mkdir()
        msk_dir.mkdir()
        for sid, nr, nc, missing, nomask, scale, shape in slide_cases(rng):
            for r in range(nr):
                for c in range(nc):
                    if (r, c) in missing:
                        continue
                    stem = f"{sid}_r{r}_c{c}"
                    base = rng.integers(40, 220, size=(1, 1, 3))
                    rgb = np.clip(base + rng.normal(0, 25, size=(T, T, 3)), 0, 255).astype(np.uint8)
                    gray = np.asarray(Image.fromarray(rgb).convert("L"), np.float32)
                    files[str(img_dir / f"{stem}.jpg")] = (gray, rgb)
                    (img_dir / f"{stem}.jpg").write_bytes(b"")
                    out[f"tile_{stem}"] = rgb
                    if (r, c) not in nomask:
                        m = (rng.random((T, T)) > 0.6).astype(np.float32) * np.float32(scale)
                        masks[str(msk_dir / f"{stem}.tif")] = m.astype(np.uint8)
                        (msk_dir / f"{stem}.tif").write_bytes(b"")
                        out[f"mask_{stem}"] = m.astype(np.uint8)
        slides = rf.group_tiles_by_slide(img_dir, msk_dir)
        model = make_golden.fake_predictor()
        for k, (sid, nr, nc, missing, nomask, scale, shape) in enumerate(slide_cases(rng)):
            info = slides[sid]
            out[f"group_{k}_tiles"] = np.array([f"{r}|{c}|{Path(i).name}|{Path(m).name if m else ''}"
                                                for r, c, i, m in info["tiles"]])
            out[f"group_{k}_ranges"] = np.array([*info["row_range"], *info["col_range"]])
            exp = rf.create_expected_grid(info["row_range"], info["col_range"])
            out[f"group_{k}_missing"] = np.array(sorted(rf.find_missing_tiles(exp, info["positions"])))
            out[f"group_{k}_inferred"] = np.array(rf.infer_full_image_dimensions(info["positions"], T, STRIDE))
            out[f"group_{k}_shape"] = np.array(shape)
            for mode, blender in (("gaussian", fe.GaussianBlender(tile_size=T, sigma_factor=0.25)),
                                  ("linear", fe.LinearBlender())):
                for tta in (None, "basic"):
                    with quiet:
                        rgbf, pred, gt = rf.reconstruct_slide(model, info["tiles"], shape, T, STRIDE, 120.0, 40.0,
                                                              blender, None, tta is not None, tta or "basic")
                    key = f"rec_{k}_{mode}_{tta or 'none'}"
                    out[key + "_rgb"], out[key + "_pred"] = rgbf, pred
                    out[key + "_gt"] = gt
    np.savez_compressed(os.path.join(HERE, "reconstruct.npz"), **out)
    print("wrote", os.path.join(HERE, "reconstruct.npz"), len(out), "arrays")


if __name__ == "__main__":
    main()
