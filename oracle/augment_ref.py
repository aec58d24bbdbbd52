"""CPU oracle (test infrastructure only) for the training-time augmentations of src/utils/data.py:13-264
and the percentile normalisation of :398-429.

The numpy parts restate the reference functions line by line (same RandomState call order, same float32
/ float64 evaluation) and are pinned by tests/golden/augment.npz, generated from the reference's own
functions by tests/golden/make_augment_golden.py. OpenCV is not installed here, so the five cv2 calls
the reference makes are restated from OpenCV's documented semantics (class Cv2Restated, below) and are
"parity unpinned": resize INTER_LINEAR / INTER_NEAREST, GaussianBlur(ksize=(0,0)), remap INTER_LINEAR /
INTER_NEAREST. The pipelines take a cv2-like object, so the recording stub of the golden script can be
substituted to check the call sequence.
"""
import numpy as np


def gaussian_taps(sigma, dtype=np.float32):
    """cv2.getGaussianKernel(ksize, sigma) for ksize = round(8 sigma + 1) | 1 (f32/f64 images)."""
    n = int(round(sigma * 4 * 2 + 1)) | 1
    x = np.arange(n, dtype=np.float64) - (n - 1) * 0.5
    t = np.exp(-0.5 / (sigma * sigma) * x * x)
    return (t / t.sum()).astype(dtype), (n - 1) // 2


def _reflect101(p, n):
    if n == 1:
        return np.zeros_like(p)
    p = np.abs(p)
    period = 2 * n - 2
    p = p % period
    return np.where(p >= n, period - p, p)


def _reflect(p, n):
    period = 2 * n
    p = np.where(p < 0, -p - 1, p) % period
    return np.where(p >= n, period - 1 - p, p)


class Cv2Restated:
    INTER_LINEAR, INTER_NEAREST, BORDER_REFLECT, BORDER_CONSTANT = 1, 0, 2, 0

    @staticmethod
    def GaussianBlur(src, ksize, sigma):
        src = np.asarray(src)
        dt = np.float64 if src.dtype == np.float64 else np.float32
        w, r = gaussian_taps(sigma, np.float32)
        w = w.astype(dt)
        H, W = src.shape
        out = src.astype(dt)
        for axis in (1, 0):
            n = W if axis == 1 else H
            acc = np.zeros_like(out)
            for t in range(-r, r + 1):
                idx = _reflect101(np.arange(n) + t, n)
                acc = acc + w[t + r] * (out[:, idx] if axis == 1 else out[idx, :])
            out = acc
        return out

    @staticmethod
    def resize(src, dsize, interpolation):
        src = np.asarray(src, np.float32)
        H, W = src.shape
        Wn, Hn = dsize
        sy, sx = np.float32(H) / np.float32(Hn), np.float32(W) / np.float32(Wn)
        yr, xr = np.arange(Hn, dtype=np.float32), np.arange(Wn, dtype=np.float32)
        if interpolation == 0:
            ys = np.minimum(np.floor(yr * sy).astype(np.int64), H - 1)
            xs = np.minimum(np.floor(xr * sx).astype(np.int64), W - 1)
            return src[ys][:, xs]

        def coords(r, s, n):
            f = (r + np.float32(0.5)) * s - np.float32(0.5)
            i0 = np.floor(f).astype(np.int64)
            f = (f - i0).astype(np.float32)
            f = np.where(i0 < 0, np.float32(0), f)
            i0 = np.maximum(i0, 0)
            f = np.where(i0 >= n - 1, np.float32(0), f)
            i0 = np.minimum(i0, n - 1)
            return i0, np.minimum(i0 + 1, n - 1), f.astype(np.float32)

        y0, y1, fy = coords(yr, sy, H)
        x0, x1, fx = coords(xr, sx, W)
        fy, fx = fy[:, None], fx[None, :]
        a, b = src[y0][:, x0], src[y0][:, x1]
        c, d = src[y1][:, x0], src[y1][:, x1]
        one = np.float32(1)
        return ((a * (one - fx) + b * fx) * (one - fy) + (c * (one - fx) + d * fx) * fy).astype(np.float32)

    @staticmethod
    def remap(src, map1, map2, interpolation, borderMode=None, borderValue=0):
        src = np.asarray(src, np.float32)
        H, W = src.shape
        mx, my = np.asarray(map1, np.float32), np.asarray(map2, np.float32)
        if interpolation == 0:
            xn, yn = np.rint(mx).astype(np.int64), np.rint(my).astype(np.int64)
            ok = (xn >= 0) & (xn < W) & (yn >= 0) & (yn < H)
            return np.where(ok, src[np.clip(yn, 0, H - 1), np.clip(xn, 0, W - 1)], np.float32(0)).astype(np.float32)
        X = np.rint(mx * np.float32(32)).astype(np.int64)
        Y = np.rint(my * np.float32(32)).astype(np.int64)
        x0, y0 = X >> 5, Y >> 5
        fx = ((X & 31) * np.float32(1 / 32)).astype(np.float32)
        fy = ((Y & 31) * np.float32(1 / 32)).astype(np.float32)
        xa, xb, ya, yb = _reflect(x0, W), _reflect(x0 + 1, W), _reflect(y0, H), _reflect(y0 + 1, H)
        one = np.float32(1)
        return ((src[ya, xa] * (one - fx) + src[ya, xb] * fx) * (one - fy)
                + (src[yb, xa] * (one - fx) + src[yb, xb] * fx) * fy).astype(np.float32)


CV2 = Cv2Restated()


# ---------------------------------------------------------------- data.py:13-145, restated
def random_rotation_90(image, mask, rng):
    k = rng.randint(0, 4)
    if k == 0:
        return image, mask
    return np.rot90(image, k), np.rot90(mask, k)


def random_flip(image, mask, rng):
    if rng.random() > 0.5:
        image, mask = np.fliplr(image), np.fliplr(mask)
    if rng.random() > 0.5:
        image, mask = np.flipud(image), np.flipud(mask)
    return image, mask


def random_brightness(image, factor_range, rng):
    factor = rng.uniform(*factor_range)
    return np.clip(image * np.float32(factor), 0, 255)


def random_contrast(image, factor_range, rng):
    mean = image.mean()
    factor = rng.uniform(*factor_range)
    return np.clip((image - mean) * np.float32(factor) + mean, 0, 255)


def random_gamma(image, gamma_range, rng):
    gamma = rng.uniform(*gamma_range)
    normalized = image / np.float32(255.0)
    return (np.power(normalized, np.float32(gamma)) * np.float32(255.0)).astype(image.dtype)


def random_gaussian_blur(image, sigma_range, prob, rng, cv2=CV2):
    if rng.random() > prob:
        return image
    sigma = rng.uniform(*sigma_range)
    if sigma < 0.1:
        return image
    return cv2.GaussianBlur(image, (0, 0), sigma)


def random_gaussian_noise(image, std_range, prob, rng):
    if rng.random() > prob:
        return image
    std = rng.uniform(*std_range)
    noise = rng.normal(0, std, image.shape)
    return np.clip(image + noise, 0, 255)


def random_scale(image, mask, scale_range, prob, rng, cv2=CV2):
    if rng.random() > prob:
        return image, mask
    scale = rng.uniform(*scale_range)
    h, w = image.shape[:2]
    new_h, new_w = int(h * scale), int(w * scale)
    image_s = cv2.resize(image, (new_w, new_h), interpolation=cv2.INTER_LINEAR)
    mask_s = cv2.resize(mask, (new_w, new_h), interpolation=cv2.INTER_NEAREST)
    if scale > 1.0:
        y0, x0 = (new_h - h) // 2, (new_w - w) // 2
        return image_s[y0:y0 + h, x0:x0 + w], mask_s[y0:y0 + h, x0:x0 + w]
    ph, pw = (h - new_h) // 2, (w - new_w) // 2
    pad = ((ph, h - new_h - ph), (pw, w - new_w - pw))
    return np.pad(image_s, pad, mode="reflect"), np.pad(mask_s, pad, mode="constant", constant_values=0)


def elastic_fields(shape, alpha, sigma, rng, cv2=CV2):
    dx = cv2.GaussianBlur((rng.rand(*shape) * 2 - 1), (0, 0), sigma) * alpha
    dy = cv2.GaussianBlur((rng.rand(*shape) * 2 - 1), (0, 0), sigma) * alpha
    return dx, dy


def elastic_transform(image, mask, alpha, sigma, rng, cv2=CV2):
    shape = image.shape[:2]
    dx, dy = elastic_fields(shape, alpha, sigma, rng, cv2)
    x, y = np.meshgrid(np.arange(shape[1]), np.arange(shape[0]))
    iy, ix = (y + dy).astype(np.float32), (x + dx).astype(np.float32)
    return (cv2.remap(image, ix, iy, cv2.INTER_LINEAR, borderMode=cv2.BORDER_REFLECT),
            cv2.remap(mask, ix, iy, cv2.INTER_NEAREST, borderMode=cv2.BORDER_CONSTANT, borderValue=0))


def augment_pair_heavy(image, mask, rng, cv2=CV2):
    image, mask = random_rotation_90(image, mask, rng)
    image, mask = random_flip(image, mask, rng)
    image, mask = random_scale(image, mask, (0.9, 1.1), 0.5, rng, cv2)
    if rng.random() > 0.7:
        image, mask = elastic_transform(image, mask, 15, 3, rng, cv2)
    if rng.random() > 0.3:
        image = random_brightness(image, (0.8, 1.2), rng)
    if rng.random() > 0.3:
        image = random_contrast(image, (0.8, 1.2), rng)
    if rng.random() > 0.3:
        image = random_gamma(image, (0.8, 1.2), rng)
    image = random_gaussian_blur(image, (0, 1.0), 0.2, rng, cv2)
    image = random_gaussian_noise(image, (0, 5), 0.2, rng)
    return np.asarray(image).astype(np.float32), np.asarray(mask).astype(np.float32)


def augment_pair_moderate(image, mask, rng, cv2=CV2):
    image, mask = random_rotation_90(image, mask, rng)
    image, mask = random_flip(image, mask, rng)
    image, mask = random_scale(image, mask, (0.95, 1.05), 0.3, rng, cv2)
    if rng.random() > 0.85:
        image, mask = elastic_transform(image, mask, 8, 3, rng, cv2)
    if rng.random() > 0.5:
        image = random_brightness(image, (0.9, 1.1), rng)
    if rng.random() > 0.5:
        image = random_contrast(image, (0.9, 1.1), rng)
    image = random_gaussian_blur(image, (0, 0.8), 0.15, rng, cv2)
    return np.asarray(image).astype(np.float32), np.asarray(mask).astype(np.float32)


def augment_pair_light(image, mask, rng, cv2=CV2):
    image, mask = random_rotation_90(image, mask, rng)
    image, mask = random_flip(image, mask, rng)
    if rng.random() > 0.7:
        image = random_brightness(image, (0.95, 1.05), rng)
    return np.asarray(image).astype(np.float32), np.asarray(mask).astype(np.float32)


def augment_pair_tta_style(image, mask, rng, cv2=CV2):
    transform_id = rng.randint(0, 8)
    if transform_id >= 4:
        image, mask = np.fliplr(image), np.fliplr(mask)
    if transform_id % 4:
        image, mask = np.rot90(image, transform_id % 4), np.rot90(mask, transform_id % 4)
    if rng.random() > 0.7:
        image, mask = random_scale(image, mask, (0.95, 1.05), 1.0, rng, cv2)
    if rng.random() > 0.4:
        image = random_brightness(image, (0.85, 1.15), rng)
    if rng.random() > 0.4:
        image = random_contrast(image, (0.85, 1.15), rng)
    if rng.random() > 0.5:
        image = random_gamma(image, (0.85, 1.15), rng)
    image = random_gaussian_blur(image, (0, 0.7), 0.15, rng, cv2)
    return np.asarray(image).astype(np.float32), np.asarray(mask).astype(np.float32)


def normalize_percentile_np123(image, p_low=1.0, p_high=99.0):
    """normalize_image(method='percentile') as evaluated under the reference's pinned numpy 1.23.5
    (requirements.txt:9): value-based casting keeps the array arithmetic in float32."""
    image = np.asarray(image, np.float32)
    plow, phigh = np.percentile(image, (p_low, p_high))
    scale = max(phigh - plow, 1e-3)
    return np.clip((image - np.float32(plow)) / np.float32(scale), np.float32(0), np.float32(1)).astype(np.float32)

