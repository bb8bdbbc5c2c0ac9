"""Language-modelling batch sampling (reference contract K17, ``tests/adapters.py:401-421``).

``get_batch`` draws ``batch_size`` start offsets uniformly from
``[0, len(dataset) - context_length)`` and returns ``x = data[s:s+ctx]`` and
``y = data[s+1:s+1+ctx]`` as int64 tensors on ``device``.  Works on in-memory
arrays and ``np.memmap`` token files alike (one fancy-index gather, no Python
loop).  GPU copies go through pinned host memory with ``non_blocking=True``.

:class:`BatchLoader` is the training-loop version: a background thread samples
and pins the next batches while the GPU works, and each rank of a
data-parallel job draws from its own RNG stream.
"""

from __future__ import annotations

import queue
import threading

import numpy as np
import torch


def _sample(dataset: np.ndarray, batch_size: int, context_length: int, rng: np.random.Generator):
    n = len(dataset)
    if n <= context_length:
        raise ValueError(f"dataset of {n} tokens is too short for context_length {context_length}")
    starts = rng.integers(0, n - context_length, size=batch_size)
    idx = starts[:, None] + np.arange(context_length + 1)[None, :]
    window = np.asarray(dataset[idx]).astype(np.int64, copy=False)
    return torch.from_numpy(np.ascontiguousarray(window[:, :-1])), torch.from_numpy(np.ascontiguousarray(window[:, 1:]))


def get_batch(dataset: np.ndarray, batch_size: int, context_length: int, device: str | torch.device,
              rng: np.random.Generator | None = None) -> tuple[torch.Tensor, torch.Tensor]:
    rng = rng if rng is not None else np.random.default_rng()
    x, y = _sample(dataset, batch_size, context_length, rng)
    device = torch.device(device)
    if device.type == "cuda":
        x = x.pin_memory().to(device, non_blocking=True)
        y = y.pin_memory().to(device, non_blocking=True)
    elif device.type != "cpu":
        x, y = x.to(device), y.to(device)
    return x, y


class BatchLoader:
    """Prefetching batch iterator over a token array.

    ``seed`` should differ per data-parallel rank (the trainer uses
    ``base_seed + rank``) so ranks see independent samples.
    """

    def __init__(self, dataset: np.ndarray, batch_size: int, context_length: int, device: str | torch.device,
                 seed: int = 0, prefetch: int = 4):
        self.dataset = dataset
        self.batch_size = batch_size
        self.context_length = context_length
        self.device = torch.device(device)
        self.rng = np.random.default_rng(seed)
        self._q: queue.Queue = queue.Queue(maxsize=max(prefetch, 1))
        self._stop = threading.Event()
        self._thread = threading.Thread(target=self._worker, daemon=True)
        self._thread.start()

    def _worker(self):
        pin = self.device.type == "cuda"
        while not self._stop.is_set():
            x, y = _sample(self.dataset, self.batch_size, self.context_length, self.rng)
            if pin:
                x, y = x.pin_memory(), y.pin_memory()
            while not self._stop.is_set():
                try:
                    self._q.put((x, y), timeout=0.1)
                    break
                except queue.Full:
                    continue

    def __iter__(self):
        return self

    def __next__(self) -> tuple[torch.Tensor, torch.Tensor]:
        x, y = self._q.get()
        if self.device.type == "cuda":
            return x.to(self.device, non_blocking=True), y.to(self.device, non_blocking=True)
        return x, y

    def close(self):
        self._stop.set()
        self._thread.join(timeout=2)
