"""keras.preprocessing.image.ImageDataGenerator for the reference's training
pipeline, with the per-frame transform on the GPU.

/root/reference/main.py:71-98 builds two generators with identical arguments
(rescale=1/255, rotation_range=90, horizontal_flip, vertical_flip,
zoom_range=0.2) over 'data/train/input1' and 'data/train/output1' with the same
seed, and zips them: the two streams draw the same permutation and the same
random transforms, so SDR input and HDR target stay paired.

The random stream here is Keras 2.2.4's (keras_preprocessing 1.0.x), call for
call: before every batch ``np.random.seed(seed + total_batches_seen)``; at an
epoch start a ``permutation`` of the files (shuffle=True); then per frame
``get_random_transform``: uniform(-rot, rot), [shifts/shear if set],
uniform(zoom lo, hi, 2), random() < 0.5 (h-flip), random() < 0.5 (v-flip).  A
private ``RandomState`` replays it, so a zip of two generators pairs exactly
as the reference's does, without touching numpy's global state.

The transform itself (transform_matrix_offset_center(rotation @ zoom), scipy
affine_transform order 1 / 'nearest', flips, x *= rescale) runs in
``cnnitmo_augment_affine`` (csrc/augment.hip) on a whole batch at once; PNG
decode and the nearest-neighbour resize to target_size stay on host threads.
Batches are yielded as float32 CUDA tensors [B, H, W, 3] (``output='numpy'``
for host arrays), which Model.fit_generator consumes without a host round
trip.
"""
from __future__ import annotations

import concurrent.futures as cf
import os

import numpy as np

WHITE_LIST = ("png", "jpg", "jpeg", "bmp", "ppm", "tif", "tiff")


def _pair(v):
    if np.isscalar(v):
        return (1.0 - float(v), 1.0 + float(v))
    v = tuple(float(x) for x in v)
    if len(v) != 2:
        raise ValueError(f"zoom_range should be a float or a tuple or list of two floats. Received: {v}")
    return v


def offset_center(matrix, h, w):
    """keras_preprocessing transform_matrix_offset_center."""
    o_x, o_y = float(h) / 2 + 0.5, float(w) / 2 + 0.5
    offset = np.array([[1, 0, o_x], [0, 1, o_y], [0, 0, 1]])
    reset = np.array([[1, 0, -o_x], [0, 1, -o_y], [0, 0, 1]])
    return np.dot(np.dot(offset, matrix), reset)


class ImageDataGenerator:
    """The subset of keras ImageDataGenerator the reference uses (+ shifts and shear,
    which share the affine kernel).  fill_mode 'nearest' only (the Keras default)."""

    def __init__(self, rescale=None, rotation_range=0.0, width_shift_range=0.0, height_shift_range=0.0,
                 shear_range=0.0, zoom_range=0.0, horizontal_flip=False, vertical_flip=False,
                 fill_mode="nearest", cval=0.0, data_format="channels_last", dtype="float32", **kwargs):
        unsupported = {k: v for k, v in kwargs.items() if v not in (None, False, 0, 0.0)}
        if unsupported:
            raise NotImplementedError(f"ImageDataGenerator options not on the path: {sorted(unsupported)}")
        if fill_mode != "nearest":
            raise NotImplementedError("fill_mode other than 'nearest'")
        if data_format != "channels_last" or dtype != "float32":
            raise NotImplementedError("channels_last float32 only")
        self.rescale = rescale
        self.rotation_range = float(rotation_range)
        self.width_shift_range = width_shift_range
        self.height_shift_range = height_shift_range
        self.shear_range = float(shear_range)
        self.zoom_range = _pair(zoom_range)
        self.horizontal_flip = bool(horizontal_flip)
        self.vertical_flip = bool(vertical_flip)

    # ---- Keras 2.2.4 random stream ------------------------------------------------
    def get_random_transform(self, img_shape, rng):
        """keras_preprocessing get_random_transform, drawing from `rng` (a RandomState)."""
        h, w = img_shape[0], img_shape[1]
        theta = rng.uniform(-self.rotation_range, self.rotation_range) if self.rotation_range else 0
        tx = ty = 0
        if self.height_shift_range:
            tx = self._shift(self.height_shift_range, rng)
            if np.max(self.height_shift_range) < 1:
                tx *= h
        if self.width_shift_range:
            ty = self._shift(self.width_shift_range, rng)
            if np.max(self.width_shift_range) < 1:
                ty *= w
        shear = rng.uniform(-self.shear_range, self.shear_range) if self.shear_range else 0
        if self.zoom_range[0] == 1 and self.zoom_range[1] == 1:
            zx, zy = 1, 1
        else:
            zx, zy = rng.uniform(self.zoom_range[0], self.zoom_range[1], 2)
        flip_h = (rng.random_sample() < 0.5) * self.horizontal_flip
        flip_v = (rng.random_sample() < 0.5) * self.vertical_flip
        return {"theta": theta, "tx": tx, "ty": ty, "shear": shear, "zx": zx, "zy": zy,
                "flip_horizontal": flip_h, "flip_vertical": flip_v}

    @staticmethod
    def _shift(rg, rng):
        try:  # 1-D array-like or int
            return rng.choice(rg) * rng.choice([-1, 1])
        except ValueError:  # floating point
            return rng.uniform(-rg, rg)

    @staticmethod
    def affine(params, h, w):
        """(matrix [2x3] float64, flip bits) for one frame -- apply_affine_transform's
        transform_matrix (identity when no transform)."""
        m = None
        theta = params.get("theta", 0)
        if theta != 0:
            t = np.deg2rad(theta)
            m = np.array([[np.cos(t), -np.sin(t), 0], [np.sin(t), np.cos(t), 0], [0, 0, 1]])
        tx, ty = params.get("tx", 0), params.get("ty", 0)
        if tx != 0 or ty != 0:
            s = np.array([[1, 0, tx], [0, 1, ty], [0, 0, 1]])
            m = s if m is None else np.dot(m, s)
        shear = params.get("shear", 0)
        if shear != 0:
            sh = np.deg2rad(shear)
            s = np.array([[1, -np.sin(sh), 0], [0, np.cos(sh), 0], [0, 0, 1]])
            m = s if m is None else np.dot(m, s)
        zx, zy = params.get("zx", 1), params.get("zy", 1)
        if zx != 1 or zy != 1:
            z = np.array([[zx, 0, 0], [0, zy, 0], [0, 0, 1]])
            m = z if m is None else np.dot(m, z)
        if m is None:
            m = np.eye(3)
        else:
            m = offset_center(m, h, w)
        flips = (1 if params.get("flip_horizontal") else 0) | (2 if params.get("flip_vertical") else 0)
        return m[:2].reshape(-1).astype(np.float64), flips

    # ---- the GPU transform ---------------------------------------------------------
    def transform_batch(self, frames, params, out=None):
        """frames: uint8/float32 [B,H,W,C] (numpy or CUDA tensor) -> fp32 CUDA tensor."""
        import torch
        from . import ops
        src = torch.as_tensor(frames)
        if not src.is_cuda:
            src = src.pin_memory().cuda(non_blocking=True) if src.dtype == torch.uint8 else src.cuda()
        src = src.contiguous()
        b, h, w, c = src.shape
        mats, flips = zip(*[self.affine(p, h, w) for p in params])
        m = torch.as_tensor(np.stack(mats)).cuda()
        f = torch.as_tensor(np.asarray(flips, np.int32)).cuda()
        if out is None:
            out = torch.empty((b, h, w, c), dtype=torch.float32, device=src.device)
        scale = float(self.rescale) if self.rescale else 1.0
        ops.augment_affine(src, m, f, scale, out)
        return out

    # ---- iterators -------------------------------------------------------------------
    def flow_from_directory(self, directory, target_size=(256, 256), color_mode="rgb", classes=None,
                            class_mode="categorical", batch_size=32, shuffle=True, seed=None,
                            interpolation="nearest", output="cuda", workers=8, rank=None, world=None, **kwargs):
        """``batch_size`` is per rank; ``rank``/``world`` default to the initialised
        torch.distributed group (pass ``world=1`` for an unsharded stream)."""
        return DirectoryIterator(directory, self, target_size, color_mode, classes, class_mode, batch_size,
                                 shuffle, seed, interpolation, output, workers, rank, world)

    def flow(self, x, y=None, batch_size=32, shuffle=True, seed=None, output="cuda", rank=None, world=None):
        return ArrayIterator(x, y, self, batch_size, shuffle, seed, output, rank, world)


def _shard(rank, world):
    """(rank, world) for a generator: explicit values, else the initialised
    torch.distributed group, else (0, 1)."""
    if world is None:
        try:
            from .dist import rank_world
            r, w = rank_world()
        except ImportError:  # pragma: no cover
            r, w = 0, 1
        return (r if rank is None else int(rank)), w
    world = int(world)
    rank = 0 if rank is None else int(rank)
    if world < 1 or not 0 <= rank < world:
        raise ValueError(f"rank {rank} out of range for world {world}")
    return rank, world


class Iterator:
    """keras_preprocessing Iterator: batch index stream + seeded permutation.

    Rank sharding: with ``world`` > 1 every rank replays the
    SAME stream for a global batch of ``batch_size * world`` frames -- the same
    reseeding, permutation and per-frame random transforms -- and keeps its
    contiguous share (``np.array_split`` of the global batch; a short last batch is
    split as evenly as possible, and one with fewer frames than ranks is dropped on
    every rank -- no rank may get an empty batch).  The union over ranks is therefore
    the single-process stream at the global batch size (less such a dropped tail), and
    two generators with the same seed stay paired on every rank (main.py:82-100's
    ``zip``).  ``last_global_batch`` is the frame count of the global batch last drawn:
    Model.fit_generator normalises each rank's gradient by it (global-batch mean)."""

    def __init__(self, n, batch_size, shuffle, seed, rank=None, world=None):
        self.rank, self.world = _shard(rank, world)
        if self.world > 1 and seed is None:
            raise ValueError("a rank-sharded generator needs a seed shared by all ranks")
        if self.world > 1 and n < self.world:
            raise ValueError(f"{n} samples cannot be sharded over {self.world} ranks")
        self.n, self.batch_size, self.shuffle, self.seed = n, batch_size, shuffle, seed
        self.global_batch = batch_size * self.world
        self.batch_index = 0
        self.total_batches_seen = 0
        self.last_global_batch = None
        self.index_array = None
        self.rng = np.random.RandomState(seed)
        self._gen = self._flow_index()

    def _local(self, m):
        """[lo, hi) of this rank's share of a global batch of m frames."""
        q, rem = divmod(m, self.world)
        lo = self.rank * q + min(self.rank, rem)
        return lo, lo + q + (1 if self.rank < rem else 0)

    def reset(self):
        self.batch_index = 0

    def _set_index_array(self):
        self.index_array = np.arange(self.n)
        if self.shuffle:
            self.index_array = self.rng.permutation(self.n)

    def _flow_index(self):
        self.reset()
        while True:
            if self.seed is not None:
                self.rng.seed(self.seed + self.total_batches_seen)
            if self.batch_index == 0:
                self._set_index_array()
            bs = self.global_batch
            cur = (self.batch_index * bs) % self.n
            if self.n > cur + bs:
                self.batch_index += 1
            else:
                self.batch_index = 0
            self.total_batches_seen += 1
            blk = self.index_array[cur:cur + bs]
            if len(blk) < self.world:  # a tail too short to give every rank a frame
                continue
            yield blk

    def __len__(self):
        full, tail = divmod(self.n, self.global_batch)
        return full + (1 if tail >= self.world else 0)

    def __iter__(self):
        return self

    def __next__(self):
        blk = next(self._gen)
        self.last_global_batch = len(blk)
        return self._batch(blk)

    next = __next__


def _list_files(directory, classes):
    if not classes:
        classes = sorted(d for d in os.listdir(directory) if os.path.isdir(os.path.join(directory, d)))
    files, labels = [], []
    for ci, cls in enumerate(classes):
        root = os.path.join(directory, cls)
        for dirpath, _, names in sorted(os.walk(root), key=lambda t: t[0]):
            for nm in sorted(names):
                if nm.lower().endswith(tuple("." + e for e in WHITE_LIST)):
                    files.append(os.path.join(dirpath, nm))
                    labels.append(ci)
    return classes, files, np.asarray(labels, np.int32)


def load_img(path, target_size=None, color_mode="rgb", interpolation="nearest"):
    """keras load_img + img_to_array, kept as uint8 [H, W, C]."""
    from PIL import Image
    modes = {"nearest": Image.NEAREST, "bilinear": Image.BILINEAR, "bicubic": Image.BICUBIC}
    with Image.open(path) as im:
        im = im.convert("L" if color_mode == "grayscale" else "RGB")
        if target_size is not None:
            wh = (target_size[1], target_size[0])
            if im.size != wh:
                im = im.resize(wh, modes[interpolation])
        a = np.asarray(im)
    return a[..., None] if a.ndim == 2 else a


class DirectoryIterator(Iterator):
    def __init__(self, directory, gen, target_size, color_mode, classes, class_mode, batch_size, shuffle,
                 seed, interpolation, output, workers, rank=None, world=None):
        if class_mode not in (None, "input", "sparse", "categorical", "binary"):
            raise ValueError(f"Invalid class_mode: {class_mode}")
        self.gen, self.target_size = gen, tuple(target_size)
        self.color_mode, self.class_mode, self.interpolation = color_mode, class_mode, interpolation
        self.output = output
        self.class_names, self.filenames, self.classes = _list_files(directory, classes)
        self.num_classes = len(self.class_names)
        self.class_indices = dict(zip(self.class_names, range(self.num_classes)))
        self._pool = cf.ThreadPoolExecutor(max_workers=workers)
        print(f"Found {len(self.filenames)} images belonging to {self.num_classes} classes.")
        super().__init__(len(self.filenames), batch_size, shuffle, seed, rank, world)

    def _batch(self, index_array):
        # the random stream covers the whole (global) batch; this rank keeps its share
        shape = tuple(self.target_size) + ((1,) if self.color_mode == "grayscale" else (3,))
        params = [self.gen.get_random_transform(shape, self.rng) for _ in index_array]
        lo, hi = self._local(len(index_array))
        index_array, params = index_array[lo:hi], params[lo:hi]
        frames = list(self._pool.map(
            lambda j: load_img(self.filenames[j], self.target_size, self.color_mode, self.interpolation),
            index_array))
        x = self.gen.transform_batch(np.stack(frames), params)
        if self.output == "numpy":
            x = x.cpu().numpy()
        if self.class_mode is None:
            return x
        if self.class_mode == "input":
            return x, x.clone() if hasattr(x, "clone") else x.copy()
        y = self.classes[index_array]
        if self.class_mode == "categorical":
            y = np.eye(self.num_classes, dtype=np.float32)[y]
        elif self.class_mode == "binary":
            y = y.astype(np.float32)
        return x, y


class ArrayIterator(Iterator):
    """keras NumpyArrayIterator (flow): frames already in memory (uint8 or float)."""

    def __init__(self, x, y, gen, batch_size, shuffle, seed, output, rank=None, world=None):
        self.x = np.asarray(x)
        if self.x.ndim != 4:
            raise ValueError(f"Input data in `NumpyArrayIterator` should have rank 4. Got {self.x.shape}")
        self.y = None if y is None else np.asarray(y)
        self.gen, self.output = gen, output
        super().__init__(self.x.shape[0], batch_size, shuffle, seed, rank, world)

    def _batch(self, index_array):
        params = [self.gen.get_random_transform(self.x.shape[1:], self.rng) for _ in index_array]
        lo, hi = self._local(len(index_array))
        index_array, params = index_array[lo:hi], params[lo:hi]
        frames = self.x[index_array]
        if frames.dtype != np.uint8:
            frames = frames.astype(np.float32)
        x = self.gen.transform_batch(frames, params)
        if self.output == "numpy":
            x = x.cpu().numpy()
        return x if self.y is None else (x, self.y[index_array])
