"""ORACLE — CPU restatement of the reference's KGE scoring path. TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module, and
only as the checker / the timed CPU baseline — never as the product path.

PARITY UNPINNED. The reference pins no numeric result for this path: it ships no golden vectors,
fixtures or unit tests; TensorFlow is not installed (ModuleNotFoundError, an
ordinary import error), and the upstream PyTorch KnowledgeGraphEmbedding submodule that holds
TransE/DistMult/ComplEx/RotatE/pRotatE is an empty directory (version unpinned). This module is
therefore a restatement, op for op, of
  * tensorflow_codes/model.py (TF, read as text):  gathers :127-199, InterHT :207-224,
    TranSparse :226-235, call/blend :114-125,201-205, reductions :145,168-171,195-198
  * tensorflow_codes/supervisor.py:15-28          train-step loss
  * the published upstream KnowledgeGraphEmbedding/codes/model.py (Sun et al., ICLR 2019 code):
    TransE / DistMult / ComplEx / RotatE / pRotatE, KGEModel.forward, train_step loss.
It is cross-checked against an independent pure-Python loop restatement (oracle/loops.py) on
small cases, and it freezes its own outputs as tests/golden/*.npz (regression, not pinning).

Everything here is plain torch on the CPU, dtype selectable (float64 for the parity oracle,
float32 for the timed "reference-faithful" CPU baseline, which materialises [B, N, d] tensors
exactly like the reference graph does).
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

PI = 3.14159265358979323846          # upstream RotatE
PI_PROTATE = 3.14159262358979323846  # upstream pRotatE (sic)

SPLIT_ENTITY = ("ComplEx", "RotatE", "InterHT")


# ------------------------------------------------------------------------------------------------
# score functions on gathered tensors: head [B, Nh, *], relation [B, 1, *], tail [B, Nt, *]
# ------------------------------------------------------------------------------------------------
def interht(head, relation, tail, mode, gamma, u=1.0):
    """tensorflow_codes/model.py:207-224."""
    a_head, b_head = torch.chunk(head, 2, dim=2)                 # :208 tf.split(head, 2, axis=2)
    re_head, re_mid, re_tail = torch.chunk(relation, 3, dim=2)   # :209 (Q6: only re_mid used)
    a_tail, b_tail = torch.chunk(tail, 2, dim=2)                 # :210
    e_h = torch.ones_like(b_head)                                # :212
    e_t = torch.ones_like(b_tail)                                # :213
    a_head = a_head / torch.linalg.vector_norm(a_head, ord=2, dim=-1, keepdim=True)  # :215 (Q7)
    a_tail = a_tail / torch.linalg.vector_norm(a_tail, ord=2, dim=-1, keepdim=True)  # :216
    b_head = b_head / torch.linalg.vector_norm(b_head, ord=2, dim=-1, keepdim=True)  # :217
    b_tail = b_tail / torch.linalg.vector_norm(b_tail, ord=2, dim=-1, keepdim=True)  # :218
    b_head = b_head + u * e_h                                    # :219
    b_tail = b_tail + u * e_t                                    # :220
    score = a_head * b_tail - a_tail * b_head + re_mid           # :222
    return gamma - torch.linalg.vector_norm(score, ord=1, dim=2)  # :223


def transparse(head, relation, tail, mode, gamma, weight, mask):
    """tensorflow_codes/model.py:226-235 (Q9: p_tail is computed from the head)."""
    def normalize(x):
        return x / torch.linalg.vector_norm(x, ord=2, dim=-1, keepdim=True)
    p_head = normalize(torch.matmul(head, mask * weight))
    p_tail = normalize(torch.matmul(head, mask * weight))
    relation = normalize(relation)
    score = p_head * relation - p_tail
    return gamma - torch.linalg.vector_norm(score, ord=1, dim=2)


def transe(head, relation, tail, mode, gamma):
    """upstream KGEModel.TransE."""
    if mode == "head-batch":
        score = head + (relation - tail)
    else:
        score = (head + relation) - tail
    return gamma - torch.norm(score, p=1, dim=2)


def distmult(head, relation, tail, mode, gamma=None):
    """upstream KGEModel.DistMult."""
    if mode == "head-batch":
        score = head * (relation * tail)
    else:
        score = (head * relation) * tail
    return score.sum(dim=2)


def complex_(head, relation, tail, mode, gamma=None):
    """upstream KGEModel.ComplEx."""
    re_head, im_head = torch.chunk(head, 2, dim=2)
    re_relation, im_relation = torch.chunk(relation, 2, dim=2)
    re_tail, im_tail = torch.chunk(tail, 2, dim=2)
    if mode == "head-batch":
        re_score = re_relation * re_tail + im_relation * im_tail
        im_score = re_relation * im_tail - im_relation * re_tail
        score = re_head * re_score + im_head * im_score
    else:
        re_score = re_head * re_relation - im_head * im_relation
        im_score = re_head * im_relation + im_head * re_relation
        score = re_score * re_tail + im_score * im_tail
    return score.sum(dim=2)


def rotate(head, relation, tail, mode, gamma, embedding_range):
    """upstream KGEModel.RotatE."""
    re_head, im_head = torch.chunk(head, 2, dim=2)
    re_tail, im_tail = torch.chunk(tail, 2, dim=2)
    phase_relation = relation / (embedding_range / PI)
    re_relation = torch.cos(phase_relation)
    im_relation = torch.sin(phase_relation)
    if mode == "head-batch":
        re_score = re_relation * re_tail + im_relation * im_tail
        im_score = re_relation * im_tail - im_relation * re_tail
        re_score = re_score - re_head
        im_score = im_score - im_head
    else:
        re_score = re_head * re_relation - im_head * im_relation
        im_score = re_head * im_relation + im_head * re_relation
        re_score = re_score - re_tail
        im_score = im_score - im_tail
    score = torch.stack([re_score, im_score], dim=0)
    score = score.norm(dim=0)
    return gamma - score.sum(dim=2)


def protate(head, relation, tail, mode, gamma, embedding_range, modulus):
    """upstream KGEModel.pRotatE."""
    phase_head = head / (embedding_range / PI_PROTATE)
    phase_relation = relation / (embedding_range / PI_PROTATE)
    phase_tail = tail / (embedding_range / PI_PROTATE)
    if mode == "head-batch":
        score = phase_head + (phase_relation - phase_tail)
    else:
        score = (phase_head + phase_relation) - phase_tail
    score = torch.sin(score)
    score = torch.abs(score)
    return gamma - score.sum(dim=2) * modulus


MODE_NAMES = {0: "head-batch", 1: "tail-batch", 3: "single"}


def model_func(name, head, relation, tail, mode, gamma, embedding_range=None, modulus=None):
    """Dispatch like KGEModel.model_func / TFKGEModel.model_func (model.py:109-112)."""
    m = MODE_NAMES.get(mode, "tail-batch") if isinstance(mode, int) else mode
    if name == "InterHT":
        return interht(head, relation, tail, m, gamma)
    if name == "TransE":
        return transe(head, relation, tail, m, gamma)
    if name == "DistMult":
        return distmult(head, relation, tail, m)
    if name == "ComplEx":
        return complex_(head, relation, tail, m)
    if name == "RotatE":
        return rotate(head, relation, tail, m, gamma, embedding_range)
    if name == "pRotatE":
        return protate(head, relation, tail, m, gamma, embedding_range, modulus)
    raise ValueError(name)


# ------------------------------------------------------------------------------------------------
# gathers (model.py:127-199 / upstream KGEModel.forward)
# ------------------------------------------------------------------------------------------------
def gather_rows(ent, rel, pos, neg, mode):
    """Returns (head, relation, tail) exactly as the reference gathers them."""
    if mode in (3, "single"):                                     # model.py:127-137
        head = ent[pos[:, 0]].unsqueeze(1)
        relation = rel[pos[:, 1]].unsqueeze(1)
        tail = ent[pos[:, 2]].unsqueeze(1)
    elif mode in (0, "head-batch"):                               # model.py:148-159
        B, N = neg.shape
        head = ent[neg.reshape(-1)].reshape(B, N, -1)
        relation = rel[pos[:, 1]].unsqueeze(1)
        tail = ent[pos[:, 2]].unsqueeze(1)
    else:                                                         # model.py:174-185
        B, N = neg.shape
        head = ent[pos[:, 0]].unsqueeze(1)
        relation = rel[pos[:, 1]].unsqueeze(1)
        tail = ent[neg.reshape(-1)].reshape(B, N, -1)
    return head, relation, tail


def score(name, ent, rel, pos, neg, mode, gamma, embedding_range=None, modulus=None):
    """Raw scores [B, N] ([B, 1] single) — upstream KGEModel.forward semantics."""
    head, relation, tail = gather_rows(ent, rel, pos, neg, mode)
    return model_func(name, head, relation, tail, mode, gamma, embedding_range, modulus)


def transparse_score(ent, rel, W, mask, pos, neg, mode, gamma):
    """TranSparse branches of TFKGEModel (model.py:127-192 with the W/mask gathers of :139-142,
    :161-164, :187-190): raw scores [B, N] (head-batch) or [B, 1] (single, tail-batch: Q9)."""
    head, relation, tail = gather_rows(ent, rel, pos, neg, mode)
    b_W = W[pos[:, 1]]
    b_mask = mask[pos[:, 1]]
    return transparse(head, relation, tail, mode, gamma, b_W, b_mask)


def tf_call_transparse(ent, rel, W, mask, pos, neg, mode, gamma):
    """TFKGEModel.call for TranSparse, all three branches blended as model.py:114-125 does."""
    p_score = F.logsigmoid(transparse_score(ent, rel, W, mask, pos, neg, 3, gamma))
    head_score = adv_reduce(transparse_score(ent, rel, W, mask, pos, neg, 0, gamma))
    tail_score = adv_reduce(transparse_score(ent, rel, W, mask, pos, neg, 1, gamma))
    negative_condition = 1.0 if mode == 0 else 0.0
    n_score = head_score * negative_condition + tail_score * (1 - negative_condition)
    condition = 1.0 if mode == 3 else 0.0
    return p_score * condition + n_score * (1 - condition)


def adv_reduce(s, temperature=1.0):
    """model.py:168-171 / 195-198 (Q3): sum softmax(s*T) * logsigmoid(-s), keepdims."""
    return torch.sum(torch.softmax(s * temperature, dim=1) * F.logsigmoid(-s), dim=1, keepdim=True)


def mean_reduce(s):
    """upstream non-adversarial: logsigmoid(-s).mean(dim=1)."""
    return F.logsigmoid(-s).mean(dim=1, keepdim=True)


def tf_call(name, ent, rel, pos, neg, mode, gamma, embedding_range=None, modulus=None):
    """TFKGEModel.call(((pos, neg), mode)) -> [B, 1], faithful to Q2: all three branches are
    evaluated and blended with 0/1 float masks (model.py:117-125,201-205)."""
    p_score = F.logsigmoid(score(name, ent, rel, pos, neg, 3, gamma, embedding_range, modulus))
    head_score = adv_reduce(score(name, ent, rel, pos, neg, 0, gamma, embedding_range, modulus))
    tail_score = adv_reduce(score(name, ent, rel, pos, neg, 1, gamma, embedding_range, modulus))
    negative_condition = 1.0 if mode == 0 else 0.0
    n_score = head_score * negative_condition + tail_score * (1 - negative_condition)
    condition = 1.0 if mode == 3 else 0.0
    return p_score * condition + n_score * (1 - condition)


def tf_call_useful(name, ent, rel, pos, neg, mode, gamma, embedding_range=None, modulus=None):
    """Same output as tf_call but only the selected branch is computed (the 'useful-only' work)."""
    if mode == 3:
        return F.logsigmoid(score(name, ent, rel, pos, neg, 3, gamma, embedding_range, modulus))
    m = 0 if mode == 0 else 1
    return adv_reduce(score(name, ent, rel, pos, neg, m, gamma, embedding_range, modulus))


def tf_train_loss(name, ent, rel, pos, neg, weight, mode, gamma, embedding_range=None, modulus=None,
                  call=tf_call):
    """supervisor.py:17-23: the loss the TF train step differentiates."""
    weight = weight.reshape(-1, 1)
    negative_score = call(name, ent, rel, pos, neg, int(mode[0]), gamma, embedding_range, modulus)
    positive_score = call(name, ent, rel, pos, neg, 3, gamma, embedding_range, modulus)
    positive_sample_loss = -torch.sum(weight * positive_score) / torch.sum(weight)
    negative_sample_loss = -torch.sum(weight * negative_score) / torch.sum(weight)
    return (positive_sample_loss + negative_sample_loss) / 2


def upstream_train_loss(name, ent, rel, pos, neg, weight, mode, gamma, embedding_range=None,
                        modulus=None, adversarial=True, temperature=1.0, uni_weight=False,
                        regularization=0.0):
    """upstream KGEModel.train_step loss (self-adversarial weights detached)."""
    negative_score = score(name, ent, rel, pos, neg, mode, gamma, embedding_range, modulus)
    if adversarial:
        negative_score = (torch.softmax(negative_score * temperature, dim=1).detach()
                          * F.logsigmoid(-negative_score)).sum(dim=1)
    else:
        negative_score = F.logsigmoid(-negative_score).mean(dim=1)
    positive_score = score(name, ent, rel, pos, neg, "single", gamma, embedding_range, modulus)
    positive_score = F.logsigmoid(positive_score).squeeze(dim=1)
    weight = weight.reshape(-1)
    if uni_weight:
        positive_sample_loss = -positive_score.mean()
        negative_sample_loss = -negative_score.mean()
    else:
        positive_sample_loss = -(weight * positive_score).sum() / weight.sum()
        negative_sample_loss = -(weight * negative_score).sum() / weight.sum()
    loss = (positive_sample_loss + negative_sample_loss) / 2
    if regularization != 0.0:
        loss = loss + regularization * (ent.norm(p=3) ** 3 + rel.norm(p=3).norm(p=3) ** 3)
    return loss


# ------------------------------------------------------------------------------------------------
# table construction (model.py:49-91 / upstream __init__)
# ------------------------------------------------------------------------------------------------
def tf_dims(name, hidden_dim, de=False, dr=False, tr=False):
    """model.py:65-78 (Q5: -dr is dead unless ComplEx, which cannot be built without it)."""
    relation_dim = hidden_dim * 2 if dr else hidden_dim
    entity_dim = hidden_dim * 2 if de else hidden_dim
    if tr:
        relation_dim = hidden_dim * 3
    elif not (name == "ComplEx" and dr):
        relation_dim = hidden_dim
    return entity_dim, relation_dim


def make_tables(nentity, nrelation, entity_dim, relation_dim, gamma, hidden_dim, seed=0,
                dtype=torch.float32, epsilon=2.0):
    """Q8: U(-(gamma+eps)/d, +(gamma+eps)/d) for both tables; same generator sequence as
    customknowledgegraphembedding_amd.model._KGEBase._init_tables."""
    init_range = float((torch.tensor([gamma], dtype=torch.float32)
                        + torch.tensor(epsilon, dtype=torch.float32)) / hidden_dim)
    g = torch.Generator().manual_seed(int(seed))
    ent = torch.empty(nentity, entity_dim).uniform_(-init_range, init_range, generator=g)
    rel = torch.empty(nrelation, relation_dim).uniform_(-init_range, init_range, generator=g)
    return ent.to(dtype), rel.to(dtype), init_range


# ------------------------------------------------------------------------------------------------
# optimizer (supervisor.py:26 optimizer.apply_gradients; run.py:111 tf.keras.optimizers.Adam)
# ------------------------------------------------------------------------------------------------
def keras_adam_step(p, g, m, v, t, lr, beta1=0.9, beta2=0.999, epsilon=1e-7):
    """Keras Adam `update_step`, dense form (sparse IndexedSlices gradients are deduplicated by
    summation before the update, which makes the sparse and dense forms equal). Returns (p, m, v)."""
    alpha = lr * (1 - beta2 ** t) ** 0.5 / (1 - beta1 ** t)
    m = m + (g - m) * (1 - beta1)
    v = v + (g * g - v) * (1 - beta2)
    p = p - (m * alpha) / (torch.sqrt(v) + epsilon)
    return p, m, v


def lrfn(epoch, num_replicas=1):
    """run.py:69-84: linear warm-up over 5 epochs to 5e-5 * replicas, then 0.8**epoch decay."""
    LR_START, LR_MAX, LR_MIN = 0.00001, 0.00005 * num_replicas, 0.00001
    LR_RAMPUP_EPOCHS, LR_SUSTAIN_EPOCHS, LR_EXP_DECAY = 5.0, 0.0, 0.8
    if float(epoch) < LR_RAMPUP_EPOCHS:
        return (LR_MAX - LR_START) / LR_RAMPUP_EPOCHS * float(epoch) + LR_START
    if float(epoch) < LR_RAMPUP_EPOCHS + LR_SUSTAIN_EPOCHS:
        return LR_MAX
    return (LR_MAX - LR_MIN) * LR_EXP_DECAY ** (float(epoch) - LR_RAMPUP_EPOCHS - LR_SUSTAIN_EPOCHS) + LR_MIN


# ------------------------------------------------------------------------------------------------
# link-prediction evaluation (upstream KGEModel.test_step + TestDataset, restated)
# ------------------------------------------------------------------------------------------------
def eval_ranks(name, ent, rel, pos, mode, all_true, gamma, embedding_range=None, modulus=None):
    """Upstream TestDataset/test_step: for each (h, r, t) the candidates are all entities; a
    candidate that forms another true triple is replaced by the positive with filter_bias -1
    (`tmp[rand] = (-1, head)`, `tmp[head] = (0, head)`); scores + bias are argsorted descending and
    the rank is 1 + the position of the positive's slot. Returns int64 ranks [B]."""
    E = ent.shape[0]
    true = set(map(tuple, all_true))
    ranks = []
    for h, r, t in pos.tolist():
        neg, bias = [], []
        for e in range(E):
            trip = (e, r, t) if mode == "head-batch" else (h, r, e)
            filtered = trip in true and e != (h if mode == "head-batch" else t)
            neg.append((h if mode == "head-batch" else t) if filtered else e)
            bias.append(-1.0 if filtered else 0.0)
        p = torch.tensor([[h, r, t]], dtype=torch.int64)
        n = torch.tensor([neg], dtype=torch.int64)
        s = score(name, ent, rel, p, n, mode, gamma, embedding_range, modulus)[0] + torch.tensor(bias, dtype=ent.dtype)
        order = torch.argsort(s, descending=True)
        slot = h if mode == "head-batch" else t
        ranks.append(int((order == slot).nonzero()[0, 0]) + 1)
    return torch.tensor(ranks, dtype=torch.int64)


def eval_query_dense(name, ent, rel, pos, mode):
    """The query side Q [B, K] of DistMult / ComplEx all-entity scoring, so that score(e) = Q . ent[e] (the
    candidate enters both formulas linearly: distmult / complex_ above with the candidate's factors pulled out;
    upstream DistMult / ComplEx head-batch and tail-batch)."""
    h, r, t = ent[pos[:, 0]], rel[pos[:, 1]], ent[pos[:, 2]]
    if name == "DistMult":
        return r * t if mode == "head-batch" else h * r
    if name != "ComplEx":
        raise ValueError(name)
    re_h, im_h = torch.chunk(h, 2, dim=1)
    re_r, im_r = torch.chunk(r, 2, dim=1)
    re_t, im_t = torch.chunk(t, 2, dim=1)
    if mode == "head-batch":
        return torch.cat([re_r * re_t + im_r * im_t, re_r * im_t - im_r * re_t], dim=1)
    return torch.cat([re_h * re_r - im_h * im_r, re_h * im_r + im_h * re_r], dim=1)


def eval_scores_dense(name, ent, rel, pos, mode):
    """S [B, E] = Q . ent^T: every entity's score as the candidate (DistMult / ComplEx)."""
    return eval_query_dense(name, ent, rel, pos, mode) @ ent.T


def eval_ranks_dense(name, ent, rel, pos, mode, all_true, rtol=1e-6, atol=None):
    """eval_ranks (upstream test_step's filtered rank) for DistMult / ComplEx over every entity at once:
    S = Q . ent^T, rank = 1 + #(unfiltered e != truth with S[e] > S[truth]) (a filtered candidate carries the
    positive's score - 1, below it). Also returns the bounds [lo, hi] of the rank under a score perturbation of
    rtol * sum_k |Q_k ent[e]_k| per candidate (the accuracy bound of an fp32 evaluation), or of atol when given
    ([B]: one bound per query's scores; [B, E]: one per score): lo counts the candidates above the truth by more than
    both perturbations, hi those not below it by more. Returns (ranks, lo, hi), int64 [B]."""
    E = ent.shape[0]
    col = 0 if mode == "head-batch" else 2
    Q = eval_query_dense(name, ent, rel, pos, mode)
    S = Q @ ent.T
    if atol is None:
        T = rtol * (Q.abs() @ ent.abs().T)
    else:
        T = torch.as_tensor(atol, dtype=S.dtype)
        T = T.expand_as(S) if T.dim() == 2 else T.reshape(-1, 1).expand_as(S)
    others = {}  # (r, t) -> true heads, or (h, r) -> true tails
    for h, r, t in map(tuple, all_true):
        key, e = ((r, t), h) if mode == "head-batch" else ((h, r), t)
        others.setdefault(key, set()).add(e)
    ranks, lo, hi = [], [], []
    for i, (h, r, t) in enumerate(pos.tolist()):
        truth = (h, r, t)[col]
        keep = torch.ones(E, dtype=torch.bool)
        keep[truth] = False
        filt = others.get((r, t) if mode == "head-batch" else (h, r), set())
        if filt:
            keep[torch.tensor(sorted(filt), dtype=torch.int64)] = False
        d = S[i] - S[i, truth]
        tol = T[i] + T[i, truth]
        ranks.append(1 + int(((d > 0) & keep).sum()))
        lo.append(1 + int(((d > tol) & keep).sum()))
        hi.append(1 + int(((d > -tol) & keep).sum()))
    return (torch.tensor(ranks, dtype=torch.int64), torch.tensor(lo, dtype=torch.int64),
            torch.tensor(hi, dtype=torch.int64))


# ------------------------------------------------------------------------------------------------
# negative sampler: upstream TrainDataset.__getitem__ with numpy itself (the reference's own RNG and
# set-membership code, so this part of the oracle is pinned by numpy, not restated)
# ------------------------------------------------------------------------------------------------
def upstream_train_dataset(triples, nentity, negative_sample_size, mode):
    """Returns getitem(idx) -> (positive_sample, negative_sample, subsampling_weight) computed
    exactly as upstream TrainDataset does, drawing from numpy's GLOBAL RandomState."""
    import numpy as np

    triples = [tuple(map(int, t)) for t in triples]
    count = {}
    for h, r, t in triples:  # count_frequency(start=4)
        count[(h, r)] = count.get((h, r), 3) + 1
        count[(t, -r - 1)] = count.get((t, -r - 1), 3) + 1
    true_head, true_tail = {}, {}
    for h, r, t in triples:  # get_true_head_and_tail
        true_tail.setdefault((h, r), []).append(t)
        true_head.setdefault((r, t), []).append(h)
    true_head = {k: np.array(list(set(v))) for k, v in true_head.items()}
    true_tail = {k: np.array(list(set(v))) for k, v in true_tail.items()}

    def getitem(idx):
        head, relation, tail = triples[idx]
        w = count[(head, relation)] + count[(tail, -relation - 1)]
        w = torch.sqrt(1 / torch.Tensor([w]))
        lst, size = [], 0
        while size < negative_sample_size:
            neg = np.random.randint(nentity, size=negative_sample_size * 2)
            if mode == "head-batch":
                mask = np.in1d(neg, true_head[(relation, tail)], assume_unique=True, invert=True)
            else:
                mask = np.in1d(neg, true_tail[(head, relation)], assume_unique=True, invert=True)
            neg = neg[mask]
            lst.append(neg)
            size += neg.size
        neg = np.concatenate(lst)[:negative_sample_size]
        return np.array([head, relation, tail]), neg, w.numpy()

    return getitem
