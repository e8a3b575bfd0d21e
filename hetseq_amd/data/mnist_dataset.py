"""MNIST without torchvision (reference: data/mnist_dataset.py:11-75).

Reads the torchvision legacy ``processed/{training,test}.pt`` tuple
``(uint8[N,28,28], int64[N])`` with ``torch.load(weights_only=True)``, or raw
IDX files (``train-images-idx3-ubyte`` ...).  The per-sample transform is
the reference's ``ToTensor()`` + ``Normalize((0.1307,), (0.3081,))``
(uint8/255, then (x-0.1307)/0.3081) applied to the whole batch in the
collater instead of through PIL per sample.  A sample is ``(img[1,28,28],
target)``; a batch is ``[float32[B,1,28,28], int64[B]]``.
"""
from __future__ import annotations

import gzip
import os
import struct

import numpy as np
import torch
import torch.utils.data

MEAN, STD = 0.1307, 0.3081


def _read_idx(path):
    op = gzip.open if path.endswith(".gz") else open
    with op(path, "rb") as f:
        magic = struct.unpack(">I", f.read(4))[0]
        nd = magic & 0xFF
        dims = struct.unpack(">" + "I" * nd, f.read(4 * nd))
        data = np.frombuffer(f.read(), dtype=np.uint8)
    return data.reshape(dims)


def load_mnist_file(path):
    if path.endswith(".pt"):
        images, labels = torch.load(path, map_location="cpu", weights_only=True)
        return images.to(torch.uint8), labels.to(torch.int64)
    raise ValueError("unsupported MNIST file: " + path)


def find_split_file(path, split):
    """Mirror of the reference's lookup (reference: tasks.py:307-327) minus the download."""
    if os.path.isdir(path):
        if os.path.exists(os.path.join(path, "MNIST/processed/")):
            path = os.path.join(path, "MNIST/processed/")
        elif os.path.basename(os.path.normpath(path)) != "processed":
            raw = os.path.join(path, "MNIST/raw/") if os.path.isdir(os.path.join(path, "MNIST/raw/")) else path
            idx = _idx_pair(raw, split)
            if idx is not None:
                return idx
            raise FileNotFoundError(
                "MNIST not found under {} (no network: place processed/{{training,test}}.pt or raw IDX files there, "
                "or generate synthetic ones with tools/make_synthetic_mnist.py)".format(path))
    files = [os.path.join(path, f) for f in os.listdir(path)] if os.path.isdir(path) else [path]
    files = select_split_files(files, split)
    assert len(files) == 1, "no suitable file in split ***{}***".format(split)
    return files[0]


def select_split_files(files, split):
    """Files of a split: the reference matches ``split in path`` on the FULL path
    (reference: tasks.py:240-241, Q10), so a directory named e.g. ``test_128``
    selects everything.  Match on the file name first and fall back to the
    reference's full-path rule only when no file name matches."""
    by_name = sorted(f for f in files if split in os.path.basename(f))
    if by_name:
        return by_name
    by_path = sorted(f for f in files if split in f)
    if by_path:
        import warnings

        warnings.warn("split '{}' matched only through directory names (reference full-path rule)".format(split))
    return by_path


def _idx_pair(raw, split):
    prefix = "train" if split in ("train", "training") else "t10k"
    for ext in ("", ".gz"):
        im = os.path.join(raw, prefix + "-images-idx3-ubyte" + ext)
        lb = os.path.join(raw, prefix + "-labels-idx1-ubyte" + ext)
        if os.path.exists(im) and os.path.exists(lb):
            return (im, lb)
    return None


class MNISTDataset(torch.utils.data.Dataset):
    def __init__(self, path):
        if isinstance(path, tuple):
            self.image = torch.from_numpy(_read_idx(path[0]).copy())
            self.label = torch.from_numpy(_read_idx(path[1]).astype(np.int64))
        else:
            self.image, self.label = load_mnist_file(path)
        self.path = path
        self._len = len(self.image)

    def __getitem__(self, index):
        img = self.image[index].to(torch.float32).div_(255.0).sub_(MEAN).div_(STD).unsqueeze(0)
        return img, int(self.label[index])

    def __len__(self):
        return self._len

    def ordered_indices(self):
        return np.arange(len(self))

    constant_num_tokens = 1

    def num_tokens(self, index):
        return 1

    def collater(self, samples):
        if len(samples) == 0:
            return None
        imgs = torch.stack([s[0] for s in samples])
        return [imgs, torch.tensor([s[1] for s in samples], dtype=torch.int64)]

    def set_epoch(self, epoch):
        pass
