"""Data: DistributedSampler, on-device synthetic batches, MNIST IDX reader.

* :class:`DistributedSampler` — index-for-index identical to
  ``torch.utils.data.distributed.DistributedSampler`` (main.py:109,115;
  SURVEY §2b F9): ``randperm`` seeded ``seed + epoch``, wrap-around padding to
  ``ceil(N/R)*R`` (or truncation with ``drop_last``), strided slice
  ``[rank::R]``. Shards therefore match torch exactly (tests assert it).
* :class:`SyntheticBatches` — BASELINE.json mandates synthetic data: a pool of
  random batches generated once ON the GPU (normalised like real inputs,
  channels_last for conv nets) and cycled, so the input pipeline costs nothing
  inside the timed step.
* :class:`MNISTIdx` — reads the raw MNIST IDX files if they exist locally
  (no download; torchvision is not available), applying the reference's
  ``ToTensor`` + ``Normalize(0.1307, 0.3081)`` (main.py:107-108).
"""
from __future__ import annotations

import gzip
import math
import os
from typing import Iterator, Optional, Sequence, Tuple

import torch
from torch.utils.data import Dataset, Sampler


class DistributedSampler(Sampler):
    def __init__(self, dataset, num_replicas: Optional[int] = None, rank: Optional[int] = None, shuffle: bool = True,
                 seed: int = 0, drop_last: bool = False):
        if num_replicas is None or rank is None:
            from .. import distributed as dist

            num_replicas = dist.get_world_size() if num_replicas is None else num_replicas
            rank = dist.get_rank() if rank is None else rank
        if rank >= num_replicas or rank < 0:
            raise ValueError(f"Invalid rank {rank}, rank should be in the interval [0, {num_replicas - 1}]")
        self.dataset = dataset
        self.num_replicas = num_replicas
        self.rank = rank
        self.epoch = 0
        self.drop_last = drop_last
        n = len(dataset)
        if drop_last and n % num_replicas != 0:
            self.num_samples = math.ceil((n - num_replicas) / num_replicas)
        else:
            self.num_samples = math.ceil(n / num_replicas)
        self.total_size = self.num_samples * num_replicas
        self.shuffle = shuffle
        self.seed = seed

    def __iter__(self) -> Iterator[int]:
        n = len(self.dataset)
        if self.shuffle:
            g = torch.Generator()
            g.manual_seed(self.seed + self.epoch)
            indices = torch.randperm(n, generator=g).tolist()
        else:
            indices = list(range(n))
        if not self.drop_last:
            pad = self.total_size - len(indices)
            if pad <= len(indices):
                indices += indices[:pad]
            else:
                indices += (indices * math.ceil(pad / len(indices)))[:pad]
        else:
            indices = indices[: self.total_size]
        assert len(indices) == self.total_size
        return iter(indices[self.rank: self.total_size: self.num_replicas])

    def __len__(self) -> int:
        return self.num_samples

    def set_epoch(self, epoch: int) -> None:
        self.epoch = epoch


class SyntheticBatches:
    """Cycle over ``pool`` pre-generated device batches of (input, target)."""

    def __init__(self, batch_size: int, input_shape: Sequence[int], num_classes: int, device,
                 dtype: torch.dtype = torch.float32, channels_last: bool = False, pool: int = 4, seed: int = 1234,
                 target_shape: Optional[Sequence[int]] = None, integer_inputs: Optional[int] = None):
        g = torch.Generator(device="cpu")
        g.manual_seed(seed)
        self.batches = []
        for _ in range(pool):
            if integer_inputs is not None:
                x = torch.randint(0, integer_inputs, (batch_size, *input_shape), generator=g)
            else:
                x = torch.randn((batch_size, *input_shape), generator=g).to(dtype)
            tshape = (batch_size,) if target_shape is None else (batch_size, *target_shape)
            y = torch.randint(0, num_classes, tshape, generator=g)
            x = x.to(device)
            if channels_last and x.dim() == 4:
                x = x.contiguous(memory_format=torch.channels_last)
            self.batches.append((x, y.to(device)))
        self.i = 0

    def __iter__(self):
        return self

    def __next__(self) -> Tuple[torch.Tensor, torch.Tensor]:
        b = self.batches[self.i % len(self.batches)]
        self.i += 1
        return b


class SyntheticDataset(Dataset):
    """Deterministic CPU dataset of MNIST-shaped samples (for sampler/DataLoader paths).

    ``learnable=True`` (the default): a class-conditional task in place of the
    absent MNIST files — every class has a fixed smooth 28x28 template (the
    same for every ``seed``: train and test splits share them) and a sample
    is ``signal * template[y] + noise`` with unit Gaussian noise, so a model's
    test accuracy climbs epoch by epoch as the reference's printout does
    (main.py:93-95). ``learnable=False``: labels independent of the inputs
    (pure throughput data)."""

    TEMPLATE_SEED = 20260101

    def __init__(self, n: int = 60000, shape=(1, 28, 28), num_classes: int = 10, seed: int = 0,
                 learnable: bool = True, signal: float = 0.1):
        g = torch.Generator()
        g.manual_seed(seed)
        self.y = torch.randint(0, num_classes, (n,), generator=g)
        noise = torch.randn((n, *shape), generator=g)
        if learnable:
            self.x = noise.add_(self.templates(shape, num_classes)[self.y], alpha=signal)
        else:
            self.x = noise

    @classmethod
    def templates(cls, shape=(1, 28, 28), num_classes: int = 10) -> torch.Tensor:
        """[num_classes, *shape] unit-variance smooth patterns (a 7x7 random
        grid upsampled bilinearly: digit-scale strokes, not pixel noise)."""
        g = torch.Generator()
        g.manual_seed(cls.TEMPLATE_SEED)
        c = shape[0]
        coarse = torch.randn((num_classes, c, 7, 7), generator=g)
        t = torch.nn.functional.interpolate(coarse, size=tuple(shape[1:]), mode="bilinear", align_corners=False)
        t = t - t.mean(dim=(1, 2, 3), keepdim=True)
        return t / t.std(dim=(1, 2, 3), keepdim=True)

    def __len__(self):
        return len(self.x)

    def __getitem__(self, i):
        return self.x[i], self.y[i]


def _read_idx(path: str) -> torch.Tensor:
    opener = gzip.open if path.endswith(".gz") else open
    with opener(path, "rb") as f:
        data = f.read()
    magic = int.from_bytes(data[0:4], "big")
    ndim = magic & 0xFF
    dims = [int.from_bytes(data[4 + 4 * i: 8 + 4 * i], "big") for i in range(ndim)]
    off = 4 + 4 * ndim
    return torch.frombuffer(bytearray(data[off:]), dtype=torch.uint8).reshape(dims)


class MNISTIdx(Dataset):
    MEAN, STD = 0.1307, 0.3081

    def __init__(self, root: str, train: bool = True):
        stem = "train" if train else "t10k"
        cands = [os.path.join(root, d) for d in ("", "MNIST/raw", "raw")]
        img = lbl = None
        for c in cands:
            for ext in ("", ".gz"):
                pi = os.path.join(c, f"{stem}-images-idx3-ubyte{ext}")
                pl = os.path.join(c, f"{stem}-labels-idx1-ubyte{ext}")
                if os.path.exists(pi) and os.path.exists(pl):
                    img, lbl = pi, pl
                    break
            if img:
                break
        if img is None:
            raise FileNotFoundError(f"MNIST IDX files not found under {root} (no download in this environment)")
        x = _read_idx(img).float().div_(255.0)
        self.x = ((x - self.MEAN) / self.STD).unsqueeze(1)
        self.y = _read_idx(lbl).long()

    def __len__(self):
        return len(self.y)

    def __getitem__(self, i):
        return self.x[i], self.y[i]
