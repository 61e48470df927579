"""Filtered link-prediction evaluation against all entities: the upstream `KGEModel.test_step`
(KnowledgeGraphEmbedding/codes/model.py, absent from the snapshot; its TestDataset builds, per test
triple and mode, a candidate list over every entity in which the other true triples are replaced by
the positive with bias -1; ranks come from argsort). BASELINE config C5.

The scores of a query batch against all E entities are computed on the GPU:
  * DistMult / ComplEx: S = Q . E^T at fp32 accuracy on the bf16 matrix cores (kge_eval_query +
    kge_gemm_nt_bf16x3: bf16x3 split in registers, six products, fp32 accumulation);
  * every other score function: the fused VALU scorer with candidate ids 0..E-1 (row stride 0).
Ranks are exact integers from kge_rank_filtered: rank = 1 + #(unfiltered e != truth with
s_e > s_truth). Ties count in the positive's favour; upstream's unstable argsort leaves them
arbitrary, which no test here exercises (continuous random scores). test_step ranks DistMult / ComplEx batches
without materialising S (kge_eval_rank_planes: the same ranks).
"""
from __future__ import annotations

from collections import defaultdict

import numpy as np
import torch

from . import ops
from . import _lib
from ._lib import FN_IDS, HEAD_BATCH, TAIL_BATCH, check

MFMA_FNS = ("DistMult", "ComplEx")


def build_filter(queries: np.ndarray, mode: str, all_true_triples) -> tuple[np.ndarray, np.ndarray]:
    """CSR (ptr [M+1], ids) of the entities upstream's filter pushes below the positive:
    head-batch (h, r, t): every h' != h with (h', r, t) true; tail-batch: every t' != t with
    (h, r, t') true. Ids are distinct and sorted within a row."""
    by_rt, by_hr = defaultdict(set), defaultdict(set)
    for h, r, t in all_true_triples:
        by_rt[(int(r), int(t))].add(int(h))
        by_hr[(int(h), int(r))].add(int(t))
    ptr = np.zeros(len(queries) + 1, dtype=np.int64)
    rows = []
    for i, (h, r, t) in enumerate(np.asarray(queries, dtype=np.int64)):
        if mode == "head-batch":
            s = by_rt.get((int(r), int(t)), set()) - {int(h)}
        else:
            s = by_hr.get((int(h), int(r)), set()) - {int(t)}
        ids = np.array(sorted(s), dtype=np.int64)
        rows.append(ids)
        ptr[i + 1] = ptr[i] + len(ids)
    ids = np.concatenate(rows) if rows else np.zeros(0, dtype=np.int64)
    return ptr, ids


def split_planes(x: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
    """x [rows, K] fp32 as three bf16 planes (kge_split_bf16x3: uint8 storage of [3][rows][K rounded to 16]),
    the operand form of kge_gemm_nt_bf16x3_planes."""
    lib = _lib.load()
    rows, K = x.shape
    nbytes = int(lib.kge_split_bf16x3_bytes(rows, K))
    if out is None or out.numel() < nbytes:
        out = torch.empty(max(nbytes, 16), dtype=torch.uint8, device=x.device)
    check(lib.kge_split_bf16x3(x.data_ptr(), rows, K, x.stride(0), out.data_ptr(), rows,
                               torch.cuda.current_stream(x.device).cuda_stream), "kge_split_bf16x3")
    return out


PLANES_MAX_BYTES = (1 << 32) - 16  # the plane GEMM's 32-bit buffer offsets (kge_split_bf16x3 refuses past it)


def entity_planes(model) -> torch.Tensor | None:
    """The entity table's bf16 planes for one evaluation pass (DistMult / ComplEx), made once and passed to
    every score_all call of the pass: the table does not change while it is evaluated. None for the other
    score functions, and None where the planes do not fit (PLANES_MAX_BYTES, or no device memory for their
    1.5x the table): score_all then splits the operands at staging (kge_gemm_nt_bf16x3), at the same accuracy."""
    if model.model_name not in MFMA_FNS:
        return None
    ent = model.entity_embedding.detach()
    if int(_lib.load().kge_split_bf16x3_bytes(ent.shape[0], ent.shape[1])) >= PLANES_MAX_BYTES:
        return None
    try:
        return split_planes(ent)
    except torch.OutOfMemoryError:
        return None


_Q_PLANES = {}


def score_all(model, positive_sample: torch.Tensor, mode: str, out: torch.Tensor | None = None,
              planes: torch.Tensor | None = None) -> torch.Tensor:
    """[B, E] scores of every entity as the candidate (head-batch or tail-batch). DistMult / ComplEx: pass
    `planes` = entity_planes(model), made once per evaluation pass (without it the call splits the table
    itself: kge_gemm_nt_bf16x3, the operands split at staging)."""
    m = ops.mode_id(mode)
    ent, rel = model.entity_embedding.detach(), model.relation_embedding.detach()
    B, E = positive_sample.shape[0], ent.shape[0]
    dev = ent.device
    if out is None:
        out = torch.empty((B, E), dtype=torch.float32, device=dev)
    st = torch.cuda.current_stream(dev).cuda_stream
    if model.model_name == "TranSparse":
        # head-batch: every entity as the head (stride-0 candidate rows); tail-batch scores do not
        # depend on the tail (Q9), so the [B, 1] score is broadcast to every candidate
        if m == HEAD_BATCH:
            cand = torch.arange(E, device=dev, dtype=torch.int64).unsqueeze(0).expand(B, E)
            return ops.transparse_score_raw(m, ent, rel, model.W.detach(), model.mask, positive_sample, cand,
                                            model._gamma_f, out=out)
        s = ops.transparse_score_raw(m, ent, rel, model.W.detach(), model.mask, positive_sample, None,
                                     model._gamma_f)
        out.copy_(s.expand(B, E))
        return out
    if model.model_name in MFMA_FNS:
        K = ent.shape[1]
        lib = _lib.load()
        fq = FN_IDS[model.model_name]
        # S = Q . E^T at fp32 accuracy on the bf16 matrix cores (bf16x3 terms, six products): from the pass's
        # entity planes and the batch's query planes (kge_eval_query_planes: the query rows written as planes, one
        # launch), or with the operands split at staging
        if planes is not None and model._D % 4 == 0 and ent.data_ptr() % 16 == 0 and rel.data_ptr() % 16 == 0:
            key = (str(dev), st)
            nbytes = int(lib.kge_split_bf16x3_bytes(B, K))
            qp = _Q_PLANES.get(key)
            if qp is None or qp.numel() < nbytes:
                qp = _Q_PLANES[key] = torch.empty(nbytes, dtype=torch.uint8, device=dev)
            check(lib.kge_eval_query_planes(fq, m, ent.data_ptr(), E, ent.stride(0), rel.data_ptr(), rel.shape[0],
                                            rel.stride(0), positive_sample.data_ptr(), B, model._D, qp.data_ptr(), B,
                                            st), "kge_eval_query_planes")
            check(lib.kge_gemm_nt_bf16x3_planes(qp.data_ptr(), B, planes.data_ptr(), E, K, out.data_ptr(),
                                                out.stride(0), B, E, st), "kge_gemm_nt_bf16x3_planes")
            return out
        Q = torch.empty((B, K), dtype=torch.float32, device=dev)
        check(lib.kge_eval_query(fq, m, ent.data_ptr(), E, ent.stride(0), rel.data_ptr(),
                                 rel.shape[0], rel.stride(0), positive_sample.data_ptr(), B, model._D, Q.data_ptr(),
                                 Q.stride(0), st), "kge_eval_query")
        if planes is not None:
            key = (str(dev), st)
            qp = _Q_PLANES[key] = split_planes(Q, _Q_PLANES.get(key))
            check(lib.kge_gemm_nt_bf16x3_planes(qp.data_ptr(), B, planes.data_ptr(), E, K, out.data_ptr(),
                                                out.stride(0), B, E, st), "kge_gemm_nt_bf16x3_planes")
        else:
            check(lib.kge_gemm_nt_bf16x3(Q.data_ptr(), Q.stride(0), ent.data_ptr(), ent.stride(0), out.data_ptr(),
                                         out.stride(0), B, E, K, st), "kge_gemm_nt_bf16x3")
        return out
    cand = torch.arange(E, device=dev, dtype=torch.int64).unsqueeze(0).expand(B, E)  # row stride 0
    modulus = float(model.modulus.detach().reshape(-1)[0]) if model.model_name == "pRotatE" else 0.0
    return ops.score_indexed_raw(FN_IDS[model.model_name], m, ent, rel, model._rel_off, positive_sample, cand,
                                 model._D, model._gamma_f, model._range_f, modulus, out=out)


_RANK_WS = {}


def _planes_rank_ok(model, planes) -> bool:
    """Whether the ranks-from-planes path applies: DistMult / ComplEx with entity planes, float4 rows."""
    if model.model_name not in MFMA_FNS or planes is None:
        return False
    ent, rel = model.entity_embedding, model.relation_embedding
    return model._D % 4 == 0 and ent.data_ptr() % 16 == 0 and rel.data_ptr() % 16 == 0


def rank_planes(model, positive_sample: torch.Tensor, mode: str, planes: torch.Tensor, truth: torch.Tensor,
                filter_ptr: torch.Tensor | None = None, filter_ids: torch.Tensor | None = None,
                nfilter: int | None = None) -> torch.Tensor | None:
    """Filtered ranks of a query batch straight from the entity planes, without the [B, E] score matrix
    (kge_eval_rank_planes: the truth's and the filter entries' scores with the GEMM's own arithmetic, the plane GEMM
    counting per row the entities above the truth, the filter correction): rank_filtered(score_all(...))'s ranks
    exactly. DistMult / ComplEx with planes; None where the query-plane form does not apply (then score_all +
    rank_filtered). filter_ptr must start at 0; nfilter = filter_ptr[-1] (read from the device when not given)."""
    if not _planes_rank_ok(model, planes):
        return None
    ent, rel = model.entity_embedding.detach(), model.relation_embedding.detach()
    lib = _lib.load()
    m = ops.mode_id(mode)
    B, E, K = positive_sample.shape[0], ent.shape[0], ent.shape[1]
    dev = ent.device
    st = torch.cuda.current_stream(dev).cuda_stream
    key = (str(dev), st)
    nbytes = int(lib.kge_split_bf16x3_bytes(B, K))
    qp = _Q_PLANES.get(key)
    if qp is None or qp.numel() < nbytes:
        qp = _Q_PLANES[key] = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    check(lib.kge_eval_query_planes(FN_IDS[model.model_name], m, ent.data_ptr(), E, ent.stride(0), rel.data_ptr(),
                                    rel.shape[0], rel.stride(0), positive_sample.data_ptr(), B, model._D, qp.data_ptr(),
                                    B, st), "kge_eval_query_planes")
    nf = (int(filter_ptr[-1]) if nfilter is None else int(nfilter)) if filter_ptr is not None else 0
    wsb = int(lib.kge_eval_rank_planes_workspace_size(B, nf))
    ws = _RANK_WS.get(key)
    if ws is None or ws.numel() < wsb:
        ws = _RANK_WS[key] = torch.empty(max(wsb, 16), dtype=torch.uint8, device=dev)
    ranks = torch.empty(B, dtype=torch.int64, device=dev)
    check(lib.kge_eval_rank_planes(qp.data_ptr(), B, planes.data_ptr(), E, K, B, E, truth.data_ptr(),
                                   None if filter_ptr is None else filter_ptr.data_ptr(),
                                   None if filter_ids is None else filter_ids.data_ptr(), nf, ranks.data_ptr(),
                                   ws.data_ptr(), ws.numel(), st), "kge_eval_rank_planes")
    return ranks


class RankPipeline:
    """rank_planes over consecutive query batches on two streams: batch i runs its whole chain (query planes,
    kge_eval_rank_planes_phases' pair scores, counting GEMM and finish) on stream i % 2, with a query-plane buffer and
    a workspace of its own. The counting GEMM holds every CU's VGPRs while its blocks run, so a single stream leaves
    the CUs of its last partial round idle (944 tiles = 3.7 rounds at C5) and runs the small kernels between GEMMs;
    with two streams the next batch's kernels and GEMM blocks fill them. submit() returns the batch's ranks tensor,
    valid on the caller's stream after flush(). Same ranks as rank_planes, batch by batch. DistMult / ComplEx with
    entity planes only (rank_planes' domain). Inputs given as CPU tensors are uploaded on the batch's stream; device
    inputs must already be complete (the streams wait for the caller's stream only in the constructor and in
    wait_caller())."""

    def __init__(self, model, planes: torch.Tensor, max_rows: int, max_filter: int, forms: dict | None = None):
        if model.model_name not in MFMA_FNS or planes is None:
            raise ValueError("RankPipeline: DistMult / ComplEx with entity planes")
        self.m, self.planes = model, planes
        self.ent, self.rel = model.entity_embedding.detach(), model.relation_embedding.detach()
        dev = self.ent.device
        self.lib = _lib.load()
        K = self.ent.shape[1]
        qb = int(self.lib.kge_split_bf16x3_bytes(max_rows, K))
        wb = max(int(self.lib.kge_eval_rank_planes_workspace_size(max_rows, max_filter)), 16)
        self.qp = [torch.empty(qb, dtype=torch.uint8, device=dev) for _ in range(2)]
        self.ws = [torch.empty(wb, dtype=torch.uint8, device=dev) for _ in range(2)]
        self.max_rows, self.max_filter = max_rows, max_filter
        self.main = torch.cuda.current_stream(dev)
        self.streams = [torch.cuda.Stream(dev), torch.cuda.Stream(dev)]
        self.forms = forms
        self.i = 0
        self.wait_caller()  # the tables and planes as the caller's stream left them

    def wait_caller(self):
        """Both streams wait for the caller's stream: after the caller rewrote the tables or the planes."""
        for st in self.streams:
            st.wait_stream(self.main)

    def submit(self, positive_sample, mode, truth, filter_ptr=None, filter_ids=None, nfilter=None, events=None):
        """Queue one batch; `events` (optional pair of timing events) are recorded on the batch's stream around its
        counting GEMM."""
        B = positive_sample.shape[0]
        if filter_ptr is not None and nfilter is None:
            nfilter = int(filter_ptr[-1])
        nf = int(nfilter) if filter_ptr is not None else 0
        if B > self.max_rows or nf > self.max_filter:
            raise ValueError("RankPipeline: batch or filter larger than the pipeline was sized for")
        E, K = self.ent.shape
        slot = self.i & 1
        self.i += 1
        st = self.streams[slot]
        dev = self.ent.device
        fp, _keep = ops._forms_ptr(self.forms)
        with torch.cuda.stream(st):
            ranks = torch.empty(B, dtype=torch.int64, device=dev)
            positive_sample, truth, filter_ptr, filter_ids = (
                None if t is None else t.to(dev) for t in (positive_sample, truth, filter_ptr, filter_ids))
            check(self.lib.kge_eval_query_planes(FN_IDS[self.m.model_name], ops.mode_id(mode), self.ent.data_ptr(), E,
                                                 self.ent.stride(0), self.rel.data_ptr(), self.rel.shape[0],
                                                 self.rel.stride(0), positive_sample.data_ptr(), B, self.m._D,
                                                 self.qp[slot].data_ptr(), B, st.cuda_stream), "kge_eval_query_planes")
            args = (self.qp[slot].data_ptr(), B, self.planes.data_ptr(), E, K, B, E, truth.data_ptr(),
                    None if filter_ptr is None else filter_ptr.data_ptr(),
                    None if filter_ids is None else filter_ids.data_ptr(), nf, ranks.data_ptr(),
                    self.ws[slot].data_ptr(), self.ws[slot].numel())
            for ph in (1, 2, 4):  # KGE_RANK_PAIRS, KGE_RANK_COUNT (events around it), KGE_RANK_FINISH
                if ph == 2 and events is not None:
                    events[0].record(st)
                check(self.lib.kge_eval_rank_planes_phases(*args, ph, fp, st.cuda_stream), "kge_eval_rank_planes")
                if ph == 2 and events is not None:
                    events[1].record(st)
            for t in (positive_sample, truth, filter_ptr, filter_ids):
                if t is not None and t.device.type == "cuda":
                    t.record_stream(st)
        ranks.record_stream(self.main)
        return ranks

    def flush(self):
        """The caller's stream waits for both streams (every submitted batch's ranks)."""
        for st in self.streams:
            self.main.wait_stream(st)


def rank_filtered(scores: torch.Tensor, truth: torch.Tensor, filter_ptr: torch.Tensor | None = None,
                  filter_ids: torch.Tensor | None = None) -> torch.Tensor:
    M, N = scores.shape
    ranks = torch.empty(M, dtype=torch.int64, device=scores.device)
    if filter_ids is not None and filter_ids.numel() == 0:  # every row's filter list empty: no filter
        filter_ptr = filter_ids = None
    rc = _lib.load().kge_rank_filtered(scores.data_ptr(), M, N, scores.stride(0), truth.data_ptr(),
                                       None if filter_ptr is None else filter_ptr.data_ptr(),
                                       None if filter_ids is None else filter_ids.data_ptr(), ranks.data_ptr(),
                                       torch.cuda.current_stream(scores.device).cuda_stream)
    check(rc, "kge_rank_filtered")
    return ranks


def metrics_from_ranks(ranks: np.ndarray) -> dict:
    r = np.asarray(ranks, dtype=np.float64)
    return {"MRR": float(np.mean(1.0 / r)), "MR": float(np.mean(r)), "HITS@1": float(np.mean(r <= 1.0)),
            "HITS@3": float(np.mean(r <= 3.0)), "HITS@10": float(np.mean(r <= 10.0))}


def average_precision(y_true, y_score) -> float:
    """Average precision = area under the precision-recall curve, as sklearn's
    average_precision_score (the metric upstream test_step reports as auc_pr for countries):
    sum over distinct score thresholds (descending) of (R_n - R_{n-1}) * P_n."""
    y_true = np.asarray(y_true, dtype=np.float64).reshape(-1)
    y_score = np.asarray(y_score, dtype=np.float64).reshape(-1)
    order = np.argsort(-y_score, kind="mergesort")
    y_true, y_score = y_true[order], y_score[order]
    last = np.r_[np.where(np.diff(y_score) != 0)[0], y_true.size - 1]  # last index of each tie group
    tps = np.cumsum(y_true)[last]
    fps = (last + 1) - tps
    if tps[-1] == 0:
        return 0.0
    precision = tps / (tps + fps)
    recall = tps / tps[-1]
    return float(np.sum(np.diff(np.r_[0.0, recall]) * precision))


def read_regions(data_path, entity2id):
    """Upstream run.py: the countries datasets' candidate regions (data/countries_S*/regions.list)."""
    import os

    with open(os.path.join(data_path, "regions.list")) as fin:
        return [entity2id[line.strip()] for line in fin if line.strip()]


def countries_auc_pr(model, test_triples, regions):
    """Upstream test_step for args.countries: every test (h, r, t) is scored against every candidate
    region (single mode, on the GPU); y_true marks the true region; auc_pr = average precision."""
    dev = model.entity_embedding.device
    sample, y_true = [], []
    for h, r, t in np.asarray(test_triples, dtype=np.int64).reshape(-1, 3).tolist():
        for region in regions:
            y_true.append(1 if region == t else 0)
            sample.append((h, r, region))
    pos = torch.tensor(sample, dtype=torch.int64, device=dev)
    with torch.no_grad():
        y_score = model.score(ops.SINGLE, pos).reshape(-1).cpu().numpy()
    return {"auc_pr": average_precision(np.array(y_true), y_score)}


def test_step(model, test_triples, all_true_triples, args=None, batch_size=None):
    """Upstream `KGEModel.test_step(model, test_triples, all_true_triples, args)`: filtered MRR,
    MR and HITS@{1,3,10} over head-batch and tail-batch ranking of every test triple; with
    args.countries, the AUC-PR over args.regions instead."""
    if args is not None and getattr(args, "countries", False):
        return countries_auc_pr(model, test_triples, args.regions)
    bs = batch_size or int(getattr(args, "test_batch_size", 1024) or 1024)
    dev = model.entity_embedding.device
    triples = np.asarray(test_triples, dtype=np.int64).reshape(-1, 3)
    # multi-GPU: replicas. Each rank ranks a strided share of the test triples against its own copy
    # of the table; the integer ranks are all-gathered before the metrics (no collective while scoring)
    import torch.distributed as dist

    world = dist.get_world_size() if (dist.is_available() and dist.is_initialized()) else 1
    if world > 1:
        triples = triples[dist.get_rank()::world]
    all_ranks = []
    with torch.no_grad():
        planes = entity_planes(model)  # once per evaluation pass (DistMult / ComplEx)
        if _planes_rank_ok(model, planes) and len(triples):
            # ranks straight from the planes (no [B, E] score matrix), batches pipelined over two streams
            filt = {m: build_filter(triples, m, all_true_triples) for m in ("head-batch", "tail-batch")}
            starts = range(0, len(triples), bs)
            maxf = max(int(ptr[min(s + bs, len(triples))] - ptr[s]) for ptr, _ in filt.values() for s in starts)
            pipe = RankPipeline(model, planes, min(bs, len(triples)), maxf)
            for mode in ("head-batch", "tail-batch"):
                col = 0 if mode == "head-batch" else 2
                ptr, ids = filt[mode]
                for s in starts:
                    q = triples[s:s + bs]
                    p = ptr[s:s + len(q) + 1]
                    pos = torch.from_numpy(q)
                    all_ranks.append(pipe.submit(pos, mode, pos[:, col].contiguous(), torch.from_numpy(p - p[0]),
                                                 torch.from_numpy(ids[p[0]:p[-1]]), int(p[-1] - p[0])))
            pipe.flush()
            all_ranks = [r.cpu().numpy() for r in all_ranks]
        for mode in (() if all_ranks else ("head-batch", "tail-batch")):
            col = 0 if mode == "head-batch" else 2
            ptr, ids = build_filter(triples, mode, all_true_triples)
            for s in range(0, len(triples), bs):
                q = triples[s:s + bs]
                pos = torch.from_numpy(q).to(dev)
                p = ptr[s:s + len(q) + 1]
                fptr = torch.from_numpy(p - p[0]).to(dev)
                fids = torch.from_numpy(ids[p[0]:p[-1]]).to(dev)
                truth = pos[:, col].contiguous()
                r = rank_filtered(score_all(model, pos, mode, planes=planes), truth, fptr, fids)
                all_ranks.append(r.cpu().numpy())
    ranks = np.concatenate(all_ranks) if all_ranks else np.zeros(0, dtype=np.int64)
    if world > 1:
        gathered = [None] * world
        dist.all_gather_object(gathered, ranks)
        ranks = np.concatenate(gathered)
    return metrics_from_ranks(ranks)


__all__ = ["build_filter", "score_all", "rank_filtered", "rank_planes", "RankPipeline", "metrics_from_ranks", "test_step", "entity_planes",
           "split_planes", "HEAD_BATCH", "TAIL_BATCH"]
