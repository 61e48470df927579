"""TF-free reader / writer of the reference's on-disk training batches (libkge_hip.so kge_tfrecord_*).

Reference: tensorflow_codes/run.py:40-66 (parse_tfrecord_fn, reshape_function, TFRecordDataset +
repeat at run.py:87-90) and compress_data/main.py:104-131 + compress_data/utils.py:35-42 (the
writer). Records are parsed by the C++ library; this module reshapes them as reshape_function does
and can prefetch on a host thread (the ctypes calls release the GIL) into pinned buffers.
"""
from __future__ import annotations

import ctypes
import os
import queue
import threading

import numpy as np
import torch

from . import _lib
from ._lib import KGEHipError, check


def _paths_arg(paths):
    if isinstance(paths, (str, os.PathLike)):
        paths = [paths]
    enc = [os.fsencode(p) for p in paths]
    arr = (ctypes.c_char_p * len(enc))(*enc)
    return arr, len(enc)


class TFRecordDataset:
    """tf.data.TFRecordDataset(paths).map(parse_tfrecord_fn): iterates dicts of numpy arrays
    {"positive_sample", "negative_sample", "subsampling_weight", "mode"} (flat, as to_dense gives)."""

    def __init__(self, paths, verify_crc=True):
        self._paths = [paths] if isinstance(paths, (str, os.PathLike)) else list(paths)
        self.verify_crc = verify_crc

    def __iter__(self):
        lib = _lib.load()
        arr, n = _paths_arg(self._paths)
        h = lib.kge_tfrecord_open(arr, n, 1 if self.verify_crc else 0)
        if not h:
            raise KGEHipError(lib.kge_last_error().decode())
        try:
            counts = np.zeros(4, dtype=np.int64)
            while True:
                rc = lib.kge_tfrecord_next(h, counts.ctypes.data)
                if rc == 0:
                    return
                check(rc if rc < 0 else 0, "kge_tfrecord_next")
                pos = np.empty(counts[0], np.int64)
                neg = np.empty(counts[1], np.int64)
                w = np.empty(counts[2], np.float32)
                mode = np.empty(counts[3], np.int64)
                check(lib.kge_tfrecord_copy(h, pos.ctypes.data, neg.ctypes.data, w.ctypes.data, mode.ctypes.data),
                      "kge_tfrecord_copy")
                yield {"positive_sample": pos, "negative_sample": neg, "subsampling_weight": w, "mode": mode}
        finally:
            lib.kge_tfrecord_close(h)


def reshape_function(example, batch_size):
    """run.py:54-66: (positive [B,-1], negative [B,-1], weight [B,-1], mode [B]) as torch tensors."""
    def rs(a, shape):
        a = np.asarray(a)
        if a.size % batch_size or (len(shape) == 1 and a.size != batch_size):
            raise ValueError(f"cannot reshape {a.size} values to {shape}")
        return torch.from_numpy(a.reshape(shape))

    return (rs(example["positive_sample"], (batch_size, -1)), rs(example["negative_sample"], (batch_size, -1)),
            rs(example["subsampling_weight"], (batch_size, -1)), rs(example["mode"], (batch_size,)))


def load_batches(paths, batch_size, repeat=True, prefetch=2, pin_memory=False, verify_crc=True):
    """run.py:86-90: TFRecordDataset -> parse -> reshape -> repeat(). Yields the 4-tuples the Trainer
    consumes. With prefetch > 0 a host thread parses ahead (bounded queue)."""
    def produce():
        while True:
            n = 0
            for ex in TFRecordDataset(paths, verify_crc):
                b = reshape_function(ex, batch_size)
                if pin_memory and torch.cuda.is_available():
                    b = tuple(t.pin_memory() for t in b)
                n += 1
                yield b
            if not repeat or n == 0:
                return

    if prefetch <= 0:
        yield from produce()
        return
    q: queue.Queue = queue.Queue(maxsize=prefetch)
    stop = threading.Event()
    end = object()

    def worker():
        try:
            for b in produce():
                while not stop.is_set():
                    try:
                        q.put(b, timeout=0.1)
                        break
                    except queue.Full:
                        continue
                if stop.is_set():
                    return
            q.put(end)
        except BaseException as e:  # noqa: BLE001 (re-raised in the consumer)
            q.put(e)

    t = threading.Thread(target=worker, daemon=True)
    t.start()
    try:
        while True:
            item = q.get()
            if item is end:
                return
            if isinstance(item, BaseException):
                raise item
            yield item
    finally:
        stop.set()


class TFRecordWriter:
    """tf.io.TFRecordWriter + create_example (compress_data/utils.py:35-42)."""

    def __init__(self, path):
        lib = _lib.load()
        self._h = lib.kge_tfrecord_writer_open(os.fsencode(path))
        if not self._h:
            raise KGEHipError(lib.kge_last_error().decode())

    def write(self, positive_sample, negative_sample, subsampling_weight, mode):
        p = np.ascontiguousarray(np.asarray(positive_sample, dtype=np.int64).reshape(-1))
        n = np.ascontiguousarray(np.asarray(negative_sample, dtype=np.int64).reshape(-1))
        w = np.ascontiguousarray(np.asarray(subsampling_weight, dtype=np.float32).reshape(-1))
        m = np.ascontiguousarray(np.asarray(mode, dtype=np.int64).reshape(-1))
        check(_lib.load().kge_tfrecord_write_example(self._h, p.ctypes.data, p.size, n.ctypes.data, n.size,
                                                     w.ctypes.data, w.size, m.ctypes.data, m.size),
              "kge_tfrecord_write_example")

    def close(self):
        if self._h:
            h, self._h = self._h, None
            check(_lib.load().kge_tfrecord_writer_close(h), "kge_tfrecord_writer_close")

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


def write_file_tfrecords(batches, output_dir, batch_size, split_number=17, dataset_name=None):
    """compress_data/main.py:104-131: spreads len(batches)//split_number batches over `split_number`
    files named <dataset>-<idx>.tfrec, skipping batches whose size is not batch_size."""
    batches = list(batches)
    name = dataset_name or os.path.basename(os.path.normpath(output_dir))
    per_file = len(batches) // split_number
    it = iter(batches)
    paths = []
    for idx in range(split_number):
        path = os.path.join(output_dir, f"{name}-{idx}.tfrec")
        paths.append(path)
        with TFRecordWriter(path) as wr:
            for _ in range(per_file):
                pos, neg, w, mode = next(it)
                if np.asarray(pos).shape[0] != batch_size:
                    continue
                wr.write(pos, neg, w, mode)
    return paths
