"""CPU oracle for the training-data augmentation -- TEST INFRASTRUCTURE ONLY.

Restates, call for call, what the reference's generators do
(/root/reference/main.py:71-98: ImageDataGenerator(rescale=1/255,
rotation_range=90, horizontal_flip=True, vertical_flip=True, zoom_range=0.2),
flow_from_directory(..., shuffle=True, seed=1), zipped input/target streams).
That code lives in Keras 2.2.4's dependency keras_preprocessing 1.0.x
(image.py: Iterator._flow_index, ImageDataGenerator.get_random_transform /
apply_transform / standardize, apply_affine_transform,
transform_matrix_offset_center), which is not vendored under /root/reference
and not installed here: the random stream below follows its published source
(global numpy RNG, seeded with seed + total_batches_seen before every batch)
and is "parity unpinned" against Keras itself.  The warp calls
scipy.ndimage.affine_transform(order=1, mode='nearest') -- the very function
keras_preprocessing calls -- so the pixel arithmetic is pinned.
"""
import numpy as np
import scipy.ndimage as ndi


def get_random_transform(img_shape, rotation_range=0.0, zoom_range=(1.0, 1.0), horizontal_flip=False,
                         vertical_flip=False, shear_range=0.0):
    """Global-RNG draws in keras_preprocessing's order (no shifts)."""
    theta = np.random.uniform(-rotation_range, rotation_range) if rotation_range else 0
    shear = np.random.uniform(-shear_range, shear_range) if shear_range else 0
    if zoom_range[0] == 1 and zoom_range[1] == 1:
        zx, zy = 1, 1
    else:
        zx, zy = np.random.uniform(zoom_range[0], zoom_range[1], 2)
    fh = (np.random.random() < 0.5) * horizontal_flip
    fv = (np.random.random() < 0.5) * vertical_flip
    return dict(theta=theta, tx=0, ty=0, shear=shear, zx=zx, zy=zy, flip_horizontal=fh, flip_vertical=fv)


def transform_matrix_offset_center(matrix, x, y):
    o_x = float(x) / 2 + 0.5
    o_y = float(y) / 2 + 0.5
    offset_matrix = np.array([[1, 0, o_x], [0, 1, o_y], [0, 0, 1]])
    reset_matrix = np.array([[1, 0, -o_x], [0, 1, -o_y], [0, 0, 1]])
    return np.dot(np.dot(offset_matrix, matrix), reset_matrix)


def apply_affine_transform(x, theta=0, shear=0, zx=1, zy=1):
    """x [H, W, C] float32 -> float32 (row 0, col 1, channel 2; fill 'nearest')."""
    m = None
    if theta != 0:
        t = np.deg2rad(theta)
        m = np.array([[np.cos(t), -np.sin(t), 0], [np.sin(t), np.cos(t), 0], [0, 0, 1]])
    if shear != 0:
        s = np.deg2rad(shear)
        sm = np.array([[1, -np.sin(s), 0], [0, np.cos(s), 0], [0, 0, 1]])
        m = sm if m is None else np.dot(m, sm)
    if zx != 1 or zy != 1:
        z = np.array([[zx, 0, 0], [0, zy, 0], [0, 0, 1]])
        m = z if m is None else np.dot(m, z)
    if m is None:
        return x
    h, w = x.shape[0], x.shape[1]
    m = transform_matrix_offset_center(m, h, w)
    xc = np.rollaxis(x, 2, 0)
    chans = [ndi.affine_transform(c, m[:2, :2], m[:2, 2], order=1, mode="nearest", cval=0.0) for c in xc]
    return np.rollaxis(np.stack(chans, axis=0), 0, 3)


def apply_transform(x, p, rescale=None):
    x = apply_affine_transform(x, p["theta"], p.get("shear", 0), p["zx"], p["zy"])
    if p["flip_horizontal"]:
        x = x[:, ::-1]
    if p["flip_vertical"]:
        x = x[::-1]
    x = np.ascontiguousarray(x)
    if rescale:
        x *= rescale
    return x


def flow(frames, batch_size, seed, nbatches, shuffle=True, **kw):
    """Yield (index_array, params) of keras Iterator batches over len(frames)."""
    n = len(frames)
    batch_index, seen, index_array = 0, 0, None
    for _ in range(nbatches):
        np.random.seed(seed + seen)
        if batch_index == 0:
            index_array = np.random.permutation(n) if shuffle else np.arange(n)
        cur = (batch_index * batch_size) % n
        batch_index = batch_index + 1 if n > cur + batch_size else 0
        seen += 1
        idx = index_array[cur:cur + batch_size]
        yield idx, [get_random_transform(frames[j].shape, **kw) for j in idx]
