"""Training-batch negative sampler: drop-in for the upstream KnowledgeGraphEmbedding
`TrainDataset` / `BidirectionalOneShotIterator` (codes/dataloader.py, absent from the snapshot;
the reference's call sites are compress_data/main.py:64-90), running in the C++ sampler of
libkge_hip.so (kge_sampler_*).

Negative ids are bit-exact with upstream's numpy code for the same numpy RNG state: construct with
`seed=s` to reproduce `np.random.seed(s)` followed by the same sequence of __getitem__ calls.
Batches are produced in host memory (numpy) and moved to the device by the caller (pinned copies
overlap with compute on a side stream).
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch

from . import _lib
from ._lib import HEAD_BATCH, TAIL_BATCH, check

_MODES = {"head-batch": HEAD_BATCH, "tail-batch": TAIL_BATCH, 0: HEAD_BATCH, 1: TAIL_BATCH}


class TrainDataset:
    """upstream TrainDataset(triples, nentity, nrelation, negative_sample_size, mode)."""

    def __init__(self, triples, nentity, nrelation, negative_sample_size, mode, seed=0):
        self.triples = np.ascontiguousarray(np.asarray(triples, dtype=np.int64).reshape(-1, 3))
        self.len = len(self.triples)
        self.nentity = int(nentity)
        self.nrelation = int(nrelation)
        self.negative_sample_size = int(negative_sample_size)
        self.mode = mode if isinstance(mode, str) else {HEAD_BATCH: "head-batch", TAIL_BATCH: "tail-batch"}[mode]
        lib = _lib.load()
        self._h = lib.kge_sampler_create(self.triples.ctypes.data, self.len, self.nentity, self.nrelation,
                                         self.negative_sample_size, _MODES[self.mode])
        if not self._h:
            raise _lib.KGEHipError(lib.kge_last_error().decode())
        self.seed(seed)

    def seed(self, seed: int):
        check(_lib.load().kge_sampler_seed(self._h, ctypes.c_uint32(int(seed) & 0xFFFFFFFF)), "kge_sampler_seed")

    def __len__(self):
        return self.len

    def sample(self, idx):
        """__getitem__ for every index in `idx`, in order -> (pos [B,3] int64, neg [B,N] int64, w [B] f32)."""
        idx = np.ascontiguousarray(np.asarray(idx, dtype=np.int64).reshape(-1))
        B, N = len(idx), self.negative_sample_size
        pos = np.empty((B, 3), dtype=np.int64)
        neg = np.empty((B, N), dtype=np.int64)
        w = np.empty((B,), dtype=np.float32)
        check(_lib.load().kge_sampler_get(self._h, idx.ctypes.data, B, pos.ctypes.data, neg.ctypes.data,
                                          w.ctypes.data), "kge_sampler_get")
        return pos, neg, w

    def __getitem__(self, idx):
        pos, neg, w = self.sample([idx])
        return (torch.from_numpy(pos[0]), torch.from_numpy(neg[0]), torch.from_numpy(w[:1]), self.mode)

    @staticmethod
    def collate_fn(data):
        positive_sample = torch.stack([_[0] for _ in data], dim=0)
        negative_sample = torch.stack([_[1] for _ in data], dim=0)
        subsample_weight = torch.cat([_[2] for _ in data], dim=0)
        mode = data[0][3]
        return positive_sample, negative_sample, subsample_weight, mode

    def batches(self, batch_size, shuffle=True, rng=None, drop_last=True, prefetch=0):
        """Endless batches (pos, neg, weight, mode) like a DataLoader over this dataset. With
        prefetch > 0 a host thread samples ahead (the C++ sampler releases the GIL), so sampling
        overlaps the GPU step; the batches and their order are unchanged."""
        rng = rng or np.random.RandomState(0)

        def produce():
            while True:
                order = rng.permutation(self.len) if shuffle else np.arange(self.len)
                stop = self.len - (self.len % batch_size if drop_last else 0)
                for s in range(0, stop, batch_size):
                    pos, neg, w = self.sample(order[s:s + batch_size])
                    yield torch.from_numpy(pos), torch.from_numpy(neg), torch.from_numpy(w), self.mode

        if prefetch <= 0:
            yield from produce()
            return
        import queue
        import threading

        q: queue.Queue = queue.Queue(maxsize=prefetch)
        stop = threading.Event()

        def worker():
            try:
                for item in produce():
                    while not stop.is_set():
                        try:
                            q.put(item, timeout=0.1)
                            break
                        except queue.Full:
                            continue
                    if stop.is_set():
                        return
            except BaseException as e:  # noqa: BLE001 (re-raised in the consumer)
                q.put(e)

        threading.Thread(target=worker, daemon=True).start()
        try:
            while True:
                item = q.get()
                if isinstance(item, BaseException):
                    raise item
                yield item
        finally:
            stop.set()

    def __del__(self):
        h = getattr(self, "_h", None)
        if h:
            try:
                _lib.load().kge_sampler_destroy(h)
            except Exception:  # noqa: BLE001 (interpreter shutdown)
                pass
            self._h = None


class BidirectionalOneShotIterator:
    """upstream BidirectionalOneShotIterator: alternates head-batch and tail-batch batches."""

    def __init__(self, dataloader_head, dataloader_tail):
        self.iterator_head = iter(dataloader_head)
        self.iterator_tail = iter(dataloader_tail)
        self.step = 0

    def __iter__(self):
        return self

    def __next__(self):
        self.step += 1
        if self.step % 2 == 0:
            return next(self.iterator_head)
        return next(self.iterator_tail)
