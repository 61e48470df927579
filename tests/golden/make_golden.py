"""Generates the committed golden fixtures tests/golden/*.npz from the CPU oracle (fp64).

Run from the repo root:  python tests/golden/make_golden.py [--reference /root/reference]

The reference pins no numeric results (PARITY UNPINNED), so these fixtures freeze
the oracle's restatement of tensorflow_codes/model.py and the upstream score functions on seeded
inputs. The countries_S1 fixture uses the reference's own data files (data/countries_S1/*.dict,
train.txt) as inputs: the triples are read here, in this container, and stored as ids in the npz,
so nothing reads /root/reference at test time.
"""
from __future__ import annotations

import argparse
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from oracle import kge_oracle as O  # noqa: E402

OUT = os.path.dirname(os.path.abspath(__file__))

FN_SPECS = {
    # name: (de, dr, tr) in upstream/TF flag terms -> (entity_dim, relation_dim) multipliers
    "TransE": (1, 1),
    "DistMult": (1, 1),
    "ComplEx": (2, 2),
    "RotatE": (2, 1),
    "pRotatE": (1, 1),
    "InterHT": (2, 3),
}


def _read_dict(path):
    d = {}
    with open(path) as f:
        for line in f:
            i, name = line.strip().split("\t")
            d[name] = int(i)
    return d


def _scores_all_modes(name, ent, rel, pos, neg, gamma, rng, modulus):
    e64, r64 = ent.double(), rel.double()
    out = {}
    for mode, tag in ((0, "head"), (1, "tail"), (3, "single")):
        out[f"score_{tag}"] = O.score(name, e64, r64, pos, neg, mode, gamma, rng, modulus).numpy()
    return out


def make_random(name, d, seed, E=97, R=7, B=4, N=16, gamma=12.0):
    em, rm = FN_SPECS[name]
    ent, rel, rng = O.make_tables(E, R, em * d, rm * d, gamma, d, seed=seed)
    g = np.random.RandomState(seed)
    pos = torch.from_numpy(np.stack([g.randint(E, size=B), g.randint(R, size=B), g.randint(E, size=B)], 1))
    neg = torch.from_numpy(g.randint(E, size=(B, N)))
    modulus = 0.5 * rng
    res = dict(ent=ent.numpy(), rel=rel.numpy(), pos=pos.numpy(), neg=neg.numpy(),
               gamma=np.float64(gamma), embedding_range=np.float64(rng), modulus=np.float64(modulus),
               hidden_dim=np.int64(d))
    res.update(_scores_all_modes(name, ent, rel, pos, neg, gamma, rng, modulus))
    s = torch.from_numpy(res["score_tail"])
    res["adv_reduce_tail"] = O.adv_reduce(s).numpy()
    res["mean_reduce_tail"] = O.mean_reduce(s).numpy()
    return res


def make_train(name, d, seed, E=53, R=5, B=6, N=8, gamma=9.0):
    """TF train-step loss (supervisor.py:17-23) + gradients w.r.t. both tables (tape.gradient)."""
    em, rm = FN_SPECS[name]
    ent, rel, rng = O.make_tables(E, R, em * d, rm * d, gamma, d, seed=seed)
    g = np.random.RandomState(seed + 100)
    pos = torch.from_numpy(np.stack([g.randint(E, size=B), g.randint(R, size=B), g.randint(E, size=B)], 1))
    neg = torch.from_numpy(g.randint(E, size=(B, N)))
    w = torch.from_numpy(g.uniform(0.1, 1.0, size=(B, 1)))
    res = dict(ent=ent.numpy(), rel=rel.numpy(), pos=pos.numpy(), neg=neg.numpy(), weight=w.numpy(),
               gamma=np.float64(gamma), embedding_range=np.float64(rng), hidden_dim=np.int64(d))
    for mode in (0, 1):
        e64 = ent.double().requires_grad_(True)
        r64 = rel.double().requires_grad_(True)
        loss = O.tf_train_loss(name, e64, r64, pos, neg, w, torch.tensor([mode]), gamma, rng, 0.5 * rng)
        loss.backward()
        res[f"loss_mode{mode}"] = loss.detach().numpy()
        res[f"d_ent_mode{mode}"] = e64.grad.numpy()
        res[f"d_rel_mode{mode}"] = r64.grad.numpy()
    return res


def make_countries(ref):
    """C1: countries_S1 TransE d=50 N=4 B=8 on the reference's own triples."""
    base = os.path.join(ref, "data", "countries_S1")
    e2i = _read_dict(os.path.join(base, "entities.dict"))
    r2i = _read_dict(os.path.join(base, "relations.dict"))
    triples = []
    with open(os.path.join(base, "train.txt")) as f:
        for line in f:
            h, r, t = line.strip().split("\t")
            triples.append((e2i[h], r2i[r], e2i[t]))
    E, R, d, gamma = len(e2i), len(r2i), 50, 24.0
    ent, rel, rng = O.make_tables(E, R, d, d, gamma, d, seed=0)
    pos = torch.tensor(triples[:8], dtype=torch.int64)
    neg = torch.from_numpy(np.random.RandomState(2).randint(E, size=(8, 4)))
    res = dict(ent=ent.numpy(), rel=rel.numpy(), pos=pos.numpy(), neg=neg.numpy(),
               gamma=np.float64(gamma), embedding_range=np.float64(rng), modulus=np.float64(0.0),
               hidden_dim=np.int64(d), nentity=np.int64(E), nrelation=np.int64(R))
    res.update(_scores_all_modes("TransE", ent, rel, pos, neg, gamma, rng, None))
    for mode in (0, 1, 3):
        res[f"tf_call_mode{mode}"] = O.tf_call("TransE", ent.double(), rel.double(), pos, neg, mode, gamma, rng).numpy()
    return res


def make_c2_rows():
    """C2-shaped InterHT rows (d=1000, -de -tr, gamma=24) on a 64-row slice, B=2, N=8."""
    d, E, R, gamma = 1000, 64, 11, 24.0
    ent, rel, rng = O.make_tables(E, R, 2 * d, 3 * d, gamma, d, seed=0)
    g = np.random.RandomState(1)
    pos = torch.from_numpy(np.stack([g.randint(E, size=2), g.randint(R, size=2), g.randint(E, size=2)], 1))
    neg = torch.from_numpy(np.random.RandomState(2).randint(E, size=(2, 8)))
    res = dict(ent=ent.numpy(), rel=rel.numpy(), pos=pos.numpy(), neg=neg.numpy(),
               gamma=np.float64(gamma), embedding_range=np.float64(rng), modulus=np.float64(0.0),
               hidden_dim=np.int64(d))
    res.update(_scores_all_modes("InterHT", ent, rel, pos, neg, gamma, rng, None))
    for mode in (0, 1, 3):
        res[f"tf_call_mode{mode}"] = O.tf_call("InterHT", ent.double(), rel.double(), pos, neg, mode, gamma, rng).numpy()
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reference", default="/root/reference")
    a = ap.parse_args()
    files = {}
    for name in FN_SPECS:
        for d in (8, 64):
            files[f"rand_{name}_d{d}.npz"] = make_random(name, d, seed=d)
        files[f"train_{name}_d16.npz"] = make_train(name, 16, seed=3)
    files["c1_countries_S1_TransE.npz"] = make_countries(a.reference)
    files["c2_wn18rr_InterHT_rows.npz"] = make_c2_rows()
    for fname, arrs in files.items():
        np.savez_compressed(os.path.join(OUT, fname), **arrs)
        print(fname, os.path.getsize(os.path.join(OUT, fname)))


if __name__ == "__main__":
    main()
