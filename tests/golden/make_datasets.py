"""Generates tests/golden/<dataset>_ids.npz: the reference's own triples as integer id arrays, so that
bench.py can take the positives of SURVEY §8(d) from the real data on the GPU box (where
/root/reference does not exist) without reading text files there.

Run from the repo root, in this container:  python tests/golden/make_datasets.py [--reference /root/reference]

Ids follow the reference's dictionaries (data/<name>/entities.dict, relations.dict: "<id>\t<name>"),
read exactly as the upstream loader does (read_triple: h, r, t per line -> (entity2id[h],
relation2id[r], entity2id[t])). Stored as int32 [T, 3] (every id < 2^31), compressed.

  wn18rr     train.txt           (C2's positives)
  FB15k-237  valid.txt+test.txt  (C3: the snapshot has no train split, .MISSING_LARGE_BLOBS)
  YAGO3-10   valid.txt+test.txt  (C4: likewise)
  FB15k      valid.txt           (C5's queries and filter set: train/test are missing)
"""
from __future__ import annotations

import argparse
import os

import numpy as np

OUT = os.path.dirname(os.path.abspath(__file__))

SETS = {
    "wn18rr": ("wn18rr", ["train.txt"]),
    "fb15k237": ("FB15k-237", ["valid.txt", "test.txt"]),
    "yago3_10": ("YAGO3-10", ["valid.txt", "test.txt"]),
    "fb15k": ("FB15k", ["valid.txt"]),
}


def read_dict(path):
    d = {}
    with open(path) as f:
        for line in f:
            i, name = line.rstrip("\n").split("\t")
            d[name] = int(i)
    return d


def read_triples(path, e2i, r2i):
    out = []
    with open(path) as f:
        for line in f:
            h, r, t = line.rstrip("\n").split("\t")
            out.append((e2i[h], r2i[r], e2i[t]))
    return np.asarray(out, dtype=np.int32).reshape(-1, 3)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reference", default="/root/reference")
    a = ap.parse_args()
    for key, (d, files) in SETS.items():
        base = os.path.join(a.reference, "data", d)
        e2i = read_dict(os.path.join(base, "entities.dict"))
        r2i = read_dict(os.path.join(base, "relations.dict"))
        tri = np.concatenate([read_triples(os.path.join(base, f), e2i, r2i) for f in files])
        np.savez_compressed(os.path.join(OUT, f"{key}_ids.npz"), triples=tri, nentity=np.int64(len(e2i)),
                            nrelation=np.int64(len(r2i)), source=np.array(f"data/{d}/" + "+".join(files)))
        print(key, tri.shape, len(e2i), len(r2i))


if __name__ == "__main__":
    main()
