"""ORACLE (independent cross-check) — pure-Python scalar loops, small cases only. TEST
INFRASTRUCTURE ONLY (see oracle/kge_oracle.py for the rules and the parity-unpinned note).

A second restatement of the same formulas written element by element in float64 Python floats,
sharing no code with kge_oracle.py, so an op-order or split/chunk mistake in one shows up as a
mismatch against the other.
  InterHT  : tensorflow_codes/model.py:207-224
  TransE / DistMult / ComplEx / RotatE / pRotatE : upstream KnowledgeGraphEmbedding/codes/model.py
"""
from __future__ import annotations

import math

PI = 3.14159265358979323846
PI_PROTATE = 3.14159262358979323846


def _norm(v):
    return math.sqrt(sum(x * x for x in v))


def score_one(name, h, r, t, mode, gamma, embedding_range=None, modulus=None):
    """Score one (h, r, t) triple given as Python lists; mode is 'head-batch', 'tail-batch' or
    'single'. Returns a float."""
    if name == "InterHT":
        d = len(h) // 2
        ah, bh = h[:d], h[d:]
        at, bt = t[:d], t[d:]
        rm = r[d:2 * d]
        nah, nbh, nat, nbt = _norm(ah), _norm(bh), _norm(at), _norm(bt)
        s = 0.0
        for i in range(d):
            x = (ah[i] / nah) * (bt[i] / nbt + 1.0) - (at[i] / nat) * (bh[i] / nbh + 1.0) + rm[i]
            s += abs(x)
        return gamma - s
    if name == "TransE":
        return gamma - sum(abs(h[i] + r[i] - t[i]) for i in range(len(h)))
    if name == "DistMult":
        return sum(h[i] * r[i] * t[i] for i in range(len(h)))
    if name == "ComplEx":
        d = len(h) // 2
        s = 0.0
        for i in range(d):
            # Re(h * r * conj(t))
            hr_re = h[i] * r[i] - h[d + i] * r[d + i]
            hr_im = h[i] * r[d + i] + h[d + i] * r[i]
            s += hr_re * t[i] + hr_im * t[d + i]
        return s
    if name == "RotatE":
        d = len(h) // 2
        s = 0.0
        for i in range(d):
            ph = r[i] / (embedding_range / PI)
            c, sn = math.cos(ph), math.sin(ph)
            re = h[i] * c - h[d + i] * sn - t[i]
            im = h[i] * sn + h[d + i] * c - t[d + i]
            s += math.sqrt(re * re + im * im)
        return gamma - s
    if name == "pRotatE":
        k = embedding_range / PI_PROTATE
        s = sum(abs(math.sin(h[i] / k + r[i] / k - t[i] / k)) for i in range(len(h)))
        return gamma - s * modulus
    raise ValueError(name)


def log_sigmoid(x):
    return min(x, 0.0) - math.log1p(math.exp(-abs(x)))


def adv_reduce_row(scores, temperature=1.0):
    m = max(temperature * s for s in scores)
    e = [math.exp(temperature * s - m) for s in scores]
    z = sum(e)
    return sum(ei / z * log_sigmoid(-s) for ei, s in zip(e, scores))


def score_batch(name, ent, rel, pos, neg, mode, gamma, embedding_range=None, modulus=None):
    """Nested-list version of kge_oracle.score: ent/rel are lists of rows, pos [[h,r,t]], neg
    [[ids]]. Returns [B][N]."""
    out = []
    for b, (h, r, t) in enumerate(pos):
        row = []
        if mode == "single":
            row.append(score_one(name, ent[h], rel[r], ent[t], mode, gamma, embedding_range, modulus))
        else:
            for c in neg[b]:
                hh, tt = (c, t) if mode == "head-batch" else (h, c)
                row.append(score_one(name, ent[hh], rel[r], ent[tt], mode, gamma, embedding_range,
                                     modulus))
        out.append(row)
    return out
