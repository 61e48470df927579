"""Multi-GPU scoring: one process per GPU, torch.distributed over RCCL (backend "nccl") on xGMI.

Two layouts:

* Replicas (C2 WN18RR, C3 FB15k-237; any table that fits one GPU's 288 GB): every rank holds the
  whole table and scores its own batch rows; the data path has no collective (bench.py --gpus N).
* Row-sharded owner-computes (`ShardedKGE`; C4 YAGO3-10 as the north star names it, and any table
  larger than one GPU): rank r owns entity rows [lo_r, hi_r). The global batch (W*B rows) is known
  to every rank (the sampler seed is replicated, so no ids move). One step:
    1. query-entity rows: each rank gathers the rows it owns (zeros elsewhere)      kge_gather_rows
       -> SUM all-reduce [W*B, ent_dim]                                              RCCL
    2. every rank scores the candidates it owns (others exactly 0, no traffic) and
       the positives whose tail it owns                                              kge_score_sharded
    3. SUM reduce-scatter of the [W*B, N+1] partial scores -> each rank's home rows  RCCL
    4. home rank: self-adversarial reduction + logsigmoid of its B rows               kge_neg_reduce/...
  Each (row, candidate) has exactly one owner, so the SUMs add exact zeros: the sharded scores
  equal the unsharded ones bitwise. (An out-of-range candidate id has no owner and scores 0 here;
  the unsharded kernels and the gather scheme score it against a zero row, as TF-GPU gather does.) Table rows never cross xGMI; per step a rank moves
  W*B*ent_dim*4 bytes of query rows and W*B*(N+1)*4 bytes of scores.
  Pipelining: the global batch is cut into K chunks (each chunk = B/K rows of every home rank, so
  the reduce-scatter of a chunk still lands on the home ranks). All chunks' query all-reduces are
  issued up front; chunk k is scored as soon as its all-reduce completes while chunk k+1's
  all-reduce and chunk k-1's reduce-scatter run on RCCL's stream, so the collectives hide behind
  the scoring kernels.

* Row-sharded gather (`ShardedKGE.step_forward_gather`, the north star's literal scheme, kept beside
  owner-computes as SURVEY §8e asks so the two can be measured against each other): every rank
  fetches the rows its own B home rows need. Per step a rank dedups its ids (sorted unique), sends
  each owner the ids in that owner's range (all-to-all), receives the rows (all-to-all), and scores
  locally on the fetched cache with the unsharded kernels (kge_step_forward). Moves ~|unique rows| x
  ent_dim x 4 bytes per rank (C4 at 8 ranks: ~45k rows, ~89 MB) instead of owner-computes' queries
  + scores, which is why owner-computes is the default.

The GPU kernels are reached through a small backend object (`HipShardKernels`); tests on CPU swap
in an oracle-backed backend to check the orchestration with gloo (tests/test_distributed_cpu.py).
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from . import ops
from ._lib import FN_IDS, HEAD_BATCH, SINGLE, TAIL_BATCH, check
from . import _lib
from .model import _dims_for


def shard_bounds(nentity: int, world: int, rank: int):
    """Block partition of entity rows: the first (nentity % world) ranks get one extra row."""
    base, extra = divmod(nentity, world)
    lo = rank * base + min(rank, extra)
    hi = lo + base + (1 if rank < extra else 0)
    return lo, hi


class HipShardKernels:
    """libkge_hip.so entry points used by ShardedKGE (device tensors, torch's current stream)."""

    @staticmethod
    def gather_rows(table, lo, ids, id_stride, n, out):
        rc = _lib.load().kge_gather_rows(table.data_ptr(), table.shape[0], table.stride(0), lo, ids.data_ptr(),
                                         id_stride, n, out.shape[1], out.data_ptr(), out.stride(0),
                                         torch.cuda.current_stream(table.device).cuda_stream)
        check(rc, "kge_gather_rows")

    @staticmethod
    def score_sharded(fn, mode, qent, rel, rel_off, shard, lo, pos, neg, D, gamma, emb_range, modulus, out):
        B = pos.shape[0]
        N = 1 if mode == SINGLE else neg.shape[1]
        rc = _lib.load().kge_score_sharded(
            fn, mode, qent.data_ptr(), qent.stride(0), rel.data_ptr(), rel.shape[0], rel.stride(0), rel_off,
            shard.data_ptr(), shard.shape[0], shard.stride(0), lo, pos.data_ptr(),
            None if mode == SINGLE else neg.data_ptr(), 0 if mode == SINGLE else neg.stride(0), B, N, D,
            float(gamma), float(emb_range), float(modulus), out.data_ptr(), out.stride(0),
            torch.cuda.current_stream(shard.device).cuda_stream)
        check(rc, "kge_score_sharded")

    @staticmethod
    def neg_reduce(scores, temperature, adversarial):
        return ops.neg_reduce_raw(scores, temperature, adversarial)

    @staticmethod
    def step_forward(fn, mode, ent, rel, rel_off, pos, neg, D, gamma, emb_range, modulus, temperature, adversarial):
        out_neg, out_pos, ns, _ = ops.step_forward_raw(fn, mode, ent, rel, rel_off, pos, neg, D, gamma, emb_range,
                                                       modulus, temperature, adversarial)
        return out_neg, out_pos, ns

    @staticmethod
    def log_sigmoid(x):
        return ops.log_sigmoid_raw(x)

    # ---- row-sharded train step (kge_shard_train_*; include/kge_hip.h) ----
    @staticmethod
    def train_alloc(sk, Bg, N):
        lib = _lib.load()
        rel = sk.relation_embedding
        nbytes = lib.kge_shard_train_workspace_size(sk.fn, sk.shard.shape[0], rel.shape[0], rel.stride(0), Bg, N, sk.D)
        if nbytes < 0:
            raise ValueError("bad shape for the sharded train step")
        dev = sk.device
        nq = lib.kge_shard_nq(sk.fn)
        f32 = dict(dtype=torch.float32, device=dev)
        return {"ws": torch.empty(max(nbytes, 1), dtype=torch.uint8, device=dev),
                "stats": torch.empty((Bg, 4), **f32), "dq": torch.empty((2 * Bg, nq * sk.D), **f32),
                "out_neg": torch.empty(Bg, **f32), "out_pos_raw": torch.empty(Bg, **f32),
                "out_pos": torch.empty(Bg, **f32), "loss": torch.empty(sk.world, **f32)}

    @staticmethod
    def _prefix(sk, bufs, mode, qent, qent_pos, pos, neg, w):
        rel = sk.relation_embedding
        Bg, N = neg.shape
        return (sk.fn, mode, sk.shard.data_ptr(), sk.shard.shape[0], sk.shard.stride(0), sk.lo, qent.data_ptr(),
                qent_pos.data_ptr(), qent.stride(0), rel.data_ptr(), rel.shape[0], rel.stride(0), sk.rel_off,
                pos.data_ptr(), neg.data_ptr(), neg.stride(0), Bg, N, sk.D, Bg // sk.world, sk.world, sk.rank,
                float(sk.gamma), float(sk.emb_range), float(sk.temperature), int(sk.adversarial), int(sk.detach),
                w.data_ptr())

    @classmethod
    def train_forward(cls, sk, bufs, mode, qent, qent_pos, pos, neg, w):
        st = torch.cuda.current_stream(sk.device).cuda_stream
        rc = _lib.load().kge_shard_train_forward(*cls._prefix(sk, bufs, mode, qent, qent_pos, pos, neg, w),
                                                 bufs["stats"].data_ptr(), bufs["dq"].data_ptr(), bufs["ws"].data_ptr(),
                                                 bufs["ws"].numel(), st)
        check(rc, "kge_shard_train_forward")

    @classmethod
    def train_combine(cls, sk, bufs, mode, qent, qent_pos, pos, neg, w, stats_all):
        st = torch.cuda.current_stream(sk.device).cuda_stream
        rc = _lib.load().kge_shard_train_combine(*cls._prefix(sk, bufs, mode, qent, qent_pos, pos, neg, w),
                                                 stats_all.data_ptr(), bufs["dq"].data_ptr(),
                                                 bufs["out_neg"].data_ptr(), bufs["out_pos_raw"].data_ptr(),
                                                 bufs["out_pos"].data_ptr(), bufs["ws"].data_ptr(), bufs["ws"].numel(),
                                                 st)
        check(rc, "kge_shard_train_combine")

    @classmethod
    def train_backward(cls, sk, bufs, mode, qent, qent_pos, pos, neg, w, step, loss_sum):
        st = torch.cuda.current_stream(sk.device).cuda_stream
        a = sk.adam
        rc = _lib.load().kge_shard_train_backward(
            *cls._prefix(sk, bufs, mode, qent, qent_pos, pos, neg, w), bufs["dq"].data_ptr(),
            bufs["loss"].data_ptr(), None if loss_sum is None else loss_sum.data_ptr(), a["m_ent"].data_ptr(),
            a["v_ent"].data_ptr(), a["m_rel"].data_ptr(), a["v_rel"].data_ptr(), float(a["lr"]), float(a["b1"]),
            float(a["b2"]), float(a["eps"]), int(step), int(a["keras"]), bufs["ws"].data_ptr(), bufs["ws"].numel(), st)
        check(rc, "kge_shard_train_backward")
        return bufs["loss"]


class TorchComm:
    """Collectives of the sharded step over torch.distributed (RCCL on ROCm, gloo on CPU)."""

    def __init__(self, group=None):
        self.group = group

    def all_gather_cat(self, t):
        """[W, *t.shape], rank-major."""
        W = dist.get_world_size(self.group)
        parts = [torch.empty_like(t) for _ in range(W)]
        dist.all_gather(parts, t.contiguous(), group=self.group)  # any backend (RCCL, gloo), any device
        return torch.stack(parts)

    def all_reduce_sum_(self, t):
        dist.all_reduce(t, op=dist.ReduceOp.SUM, group=self.group)
        return t


class ThreadComm:
    """The same collectives between W threads of ONE process (one Python thread per simulated rank,
    all on one device and stream): used to run the W-rank sharded step on a single GPU. Sums are
    taken in rank order, as RCCL's result is the same on every rank."""

    def __init__(self, world):
        import threading
        self.world = world
        self._barrier = threading.Barrier(world, timeout=120)  # a failed rank breaks it instead of hanging
        self._slots = [None] * world

    def _exchange(self, rank, t):
        self._slots[rank] = t
        self._barrier.wait()
        got = list(self._slots)
        self._barrier.wait()
        return got

    def all_gather_cat(self, t, rank):
        return torch.stack(self._exchange(rank, t.contiguous()))

    def all_reduce_sum_(self, t, rank):
        parts = self._exchange(rank, t.clone())
        acc = parts[0].clone()
        for x in parts[1:]:
            acc += x
        t.copy_(acc)
        return t


def run_threads(fns):
    """Runs fns[r]() on one thread per simulated rank; returns their results (re-raises the first error)."""
    import threading
    res, err = [None] * len(fns), []

    def go(r):
        try:
            res[r] = fns[r]()
        except BaseException as e:  # noqa: BLE001
            err.append(e)

    th = [threading.Thread(target=go, args=(r,)) for r in range(len(fns))]
    for t in th:
        t.start()
    for t in th:
        t.join()
    if err:
        raise err[0]
    return res


def _reduce_scatter_rows(full, world, rank, group):
    """SUM over ranks of `full` [W*B, C], returning this rank's [B, C] block. RCCL has a native
    reduce-scatter; gloo (CPU tests) falls back to all-reduce + slice."""
    B = full.shape[0] // world
    if full.is_cuda:
        out = torch.empty((B,) + tuple(full.shape[1:]), dtype=full.dtype, device=full.device)
        dist.reduce_scatter_tensor(out, full, op=dist.ReduceOp.SUM, group=group)
        return out
    dist.all_reduce(full, op=dist.ReduceOp.SUM, group=group)
    return full[rank * B:(rank + 1) * B].contiguous()


def _reduce_scatter_rows_into(out, full, world, rank, group):
    """Async SUM reduce-scatter of `full` [W*b, C] into this rank's `out` [b, C] (a contiguous row
    block). Returns the work handle (None when it completed synchronously: gloo fallback)."""
    b = full.shape[0] // world
    if full.is_cuda:
        return dist.reduce_scatter_tensor(out, full, op=dist.ReduceOp.SUM, group=group, async_op=True)
    dist.all_reduce(full, op=dist.ReduceOp.SUM, group=group)
    out.copy_(full[rank * b:(rank + 1) * b])
    return None


class ShardedKGE:
    """Row-sharded owner-computes forward of supervisor.py:17-18 (both model calls).

    The shard is the slice [lo, hi) of exactly the table TFKGEModel(seed) would build, so sharded
    results can be compared with the unsharded model row for row.
    """

    def __init__(self, model_name, nentity, nrelation, hidden_dim, gamma, double_entity_embedding=False,
                 double_relation_embedding=False, triple_relation_embedding=False, device=None, seed=0,
                 group=None, kernels=None, full_tables=None, world=None, rank=None, comm=None):
        """world / rank / comm override torch.distributed: a ThreadComm runs W simulated ranks as
        threads of one process (single-GPU tests and measurements of the sharded step)."""
        from .model import TFKGEModel

        self.group = group
        if world is None:
            self.world = dist.get_world_size(group) if dist.is_initialized() else 1
            self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        else:
            self.world, self.rank = int(world), int(rank)
        self.comm = comm if comm is not None else (TorchComm(group) if self.world > 1 else None)
        self.kernels = kernels or HipShardKernels()
        self.model_name = model_name
        self.fn = FN_IDS[model_name]
        self.nentity = nentity
        self.lo, self.hi = shard_bounds(nentity, self.world, self.rank)
        if full_tables is None:
            ref = TFKGEModel(model_name, nentity, nrelation, hidden_dim, gamma, double_entity_embedding,
                             double_relation_embedding, triple_relation_embedding, device="cpu", seed=seed)
            ent, rel = ref.entity_embedding.detach(), ref.relation_embedding.detach()
            self.gamma, self.emb_range = ref._gamma_f, ref._range_f
            self.modulus = float(ref.modulus.reshape(-1)[0]) if model_name == "pRotatE" else 0.0
        else:
            ent, rel, self.gamma, self.emb_range, self.modulus = full_tables
        self.entity_dim, self.relation_dim = ent.shape[1], rel.shape[1]
        self.D, self.rel_off = _dims_for(model_name, self.entity_dim, self.relation_dim)
        dev = device if device is not None else ("cuda" if torch.cuda.is_available() else "cpu")
        self.shard = ent[self.lo:self.hi].contiguous().to(dev)
        self.relation_embedding = rel.contiguous().to(dev)  # replicated (R rows)
        self.device = torch.device(dev)
        # train-step options (supervisor.py:15-26 TF semantics by default: self-adversarial, T = 1,
        # softmax not detached; Keras Adam) and state
        self.temperature, self.adversarial, self.detach = 1.0, True, False
        self.adam = None
        self.step = 0
        self.loss_sum = None
        self._bufs = {}

    @classmethod
    def from_model(cls, model, group=None, kernels=None, world=None, rank=None, comm=None):
        """A sharded view of an existing TFKGEModel / KGEModel: this rank's shard IS rows [lo, hi) of the
        model's entity table (a view: updates land in the model's own storage) and the relation table
        is the model's (updated identically on every rank). Rows outside the shard go stale during
        training until `sync_entity_table` re-broadcasts every rank's block."""
        ent = model.entity_embedding.data
        rel = model.relation_embedding.data
        modulus = float(model.modulus.reshape(-1)[0]) if model.model_name == "pRotatE" else 0.0
        return cls(model.model_name, model.nentity, model.nrelation, model.hidden_dim, model._gamma_f,
                   device=ent.device, group=group, kernels=kernels, world=world, rank=rank, comm=comm,
                   full_tables=(ent, rel, model._gamma_f, model._range_f, modulus))

    def sync_entity_table(self, table):
        """Every rank's block of rows -> `table` [E, ent_dim] on every rank (one broadcast per rank)."""
        if self.world == 1:
            return table
        for r in range(self.world):
            lo, hi = shard_bounds(self.nentity, self.world, r)
            blk = table[lo:hi]
            if r == self.rank and blk.data_ptr() != self.shard.data_ptr():
                blk.copy_(self.shard)
            dist.broadcast(blk, src=r, group=self.group)
        return table

    def configure_optimizer(self, lr=5e-5, betas=(0.9, 0.999), eps=None, semantics="keras"):
        """Adam over this rank's shard and the replicated relation table (supervisor.py:26; run.py:111
        Keras Adam by default). Every rank applies the same relation update, so the replicas stay equal."""
        if eps is None:
            eps = 1e-7 if semantics == "keras" else 1e-8
        self.adam = {"m_ent": torch.zeros_like(self.shard), "v_ent": torch.zeros_like(self.shard),
                     "m_rel": torch.zeros_like(self.relation_embedding),
                     "v_rel": torch.zeros_like(self.relation_embedding),
                     "lr": lr, "b1": betas[0], "b2": betas[1], "eps": eps, "keras": semantics == "keras"}
        self.step = 0
        return self

    def _coll(self, name, t):
        if self.world == 1:
            return t.unsqueeze(0) if name == "gather" else t
        if isinstance(self.comm, ThreadComm):
            return self.comm.all_gather_cat(t, self.rank) if name == "gather" else self.comm.all_reduce_sum_(t, self.rank)
        return self.comm.all_gather_cat(t) if name == "gather" else self.comm.all_reduce_sum_(t)

    def assemble_queries(self, pos_g, mode):
        """The query-entity rows of every global batch row: (qent [Bg, ent_dim] = E[pos[:, 2 if head
        else 0]], qent_pos [Bg, ent_dim] = E[pos[:, 0]]): owners gather their rows, one SUM all-reduce."""
        Bg = pos_g.shape[0]
        cols = [2, 0] if mode == HEAD_BATCH else [0]
        rows = torch.empty((len(cols), Bg, self.entity_dim), dtype=torch.float32, device=self.device)
        for i, c in enumerate(cols):
            self.kernels.gather_rows(self.shard, self.lo, pos_g[:, c:], 3, Bg, rows[i])
        rows = self._coll("sum", rows)
        return rows[0], rows[-1]

    def train_step(self, pos_g, neg_g, weight_g, mode):
        """One row-sharded train step (supervisor.py:15-26 over the W replicas' batches, SUM gradient
        aggregation): pos_g [Bg, 3], neg_g [Bg, N], weight_g [Bg] — the global batch (home rank h's
        replica batch is rows [h Bg/W, (h+1) Bg/W)), identical on every rank. Updates this rank's
        shard and the relation table in place; returns this rank's replica loss (0-dim tensor).
        Collectives per step: one SUM all-reduce of the query rows, one all-gather of [Bg, 4] row
        statistics, one SUM all-reduce of the [2 Bg, nq D] query gradients."""
        if self.adam is None:
            self.configure_optimizer()
        mode = ops.mode_id(mode)
        if mode not in (HEAD_BATCH, TAIL_BATCH):
            raise ValueError("train_step needs a negative mode (0 or 1)")
        Bg, N = neg_g.shape
        if Bg % self.world:
            raise ValueError("global batch must split evenly over ranks")
        w = weight_g.reshape(-1).to(torch.float32).contiguous()
        k = self.kernels
        key = (Bg, N)
        if key not in self._bufs:
            self._bufs = {key: k.train_alloc(self, Bg, N)}
        bufs = self._bufs[key]
        if self.loss_sum is None:
            self.loss_sum = torch.zeros((), dtype=torch.float32, device=self.device)
        qent, qent_pos = self.assemble_queries(pos_g, mode)
        k.train_forward(self, bufs, mode, qent, qent_pos, pos_g, neg_g, w)
        stats_all = self._coll("gather", bufs["stats"])
        k.train_combine(self, bufs, mode, qent, qent_pos, pos_g, neg_g, w, stats_all)
        self._coll("sum", bufs["dq"])
        loss = k.train_backward(self, bufs, mode, qent, qent_pos, pos_g, neg_g, w, self.step + 1, self.loss_sum)
        self.step += 1
        self.last_losses = loss  # every replica's loss [W] (identical on every rank)
        return loss[self.rank]

    def step_forward(self, pos_g, neg_g, mode, temperature=1.0, adversarial=True, chunks=None):
        """pos_g [W*B, 3], neg_g [W*B, N] (the global batch, identical on every rank) ->
        (out_neg [B], out_pos [B], scores [B, N]) for this rank's home rows [rank*B, (rank+1)*B)."""
        mode = ops.mode_id(mode)
        if mode not in (HEAD_BATCH, TAIL_BATCH):
            raise ValueError("step_forward needs a negative mode (0 or 1)")
        WB, N = neg_g.shape
        W = self.world
        if WB % W:
            raise ValueError("global batch must split evenly over ranks")
        B = WB // W
        K = max(1, min(int(chunks if chunks is not None else (4 if W > 1 else 1)), B))
        while B % K:
            K -= 1
        Bk = B // K
        k = self.kernels
        dev = self.device
        qcols = [2, 0] if mode == HEAD_BATCH else [0]
        dist_on = W > 1

        # chunk k = rows h*B + k*Bk + [0, Bk) of every home rank h, in h-major order
        def chunk_rows(kk):
            if K == 1:
                return pos_g, neg_g
            base = torch.arange(W, device=pos_g.device, dtype=torch.int64) * B + kk * Bk
            idx = (base[:, None] + torch.arange(Bk, device=pos_g.device, dtype=torch.int64)[None, :]).reshape(-1)
            return pos_g.index_select(0, idx), neg_g.index_select(0, idx)

        # 1. query-entity rows (t for head-batch, h otherwise; plus the positives' h rows in head-batch):
        #    owner-gathered, SUM all-reduce; every chunk's all-reduce is in flight before any scoring
        batches, rows_k, ar = [], [], []
        for kk in range(K):
            pk, nk = chunk_rows(kk)
            rows = torch.empty((len(qcols), W * Bk, self.entity_dim), dtype=torch.float32, device=dev)
            for i, c in enumerate(qcols):
                k.gather_rows(self.shard, self.lo, pk[:, c:], 3, W * Bk, rows[i])
            ar.append(dist.all_reduce(rows, op=dist.ReduceOp.SUM, group=self.group, async_op=True)
                      if dist_on else None)
            batches.append((pk, nk))
            rows_k.append(rows)
        # 2. owner-computes scores per chunk, 3. SUM reduce-scatter of the chunk to the home ranks
        home = torch.empty((B, N + 1), dtype=torch.float32, device=dev)
        pending = []
        for kk in range(K):
            if ar[kk] is not None:
                ar[kk].wait()
            pk, nk = batches[kk]
            rows = rows_k[kk]
            qe, ph = rows[0], rows[-1]
            part = home if not dist_on else torch.empty((W * Bk, N + 1), dtype=torch.float32, device=dev)
            k.score_sharded(self.fn, mode, qe, self.relation_embedding, self.rel_off, self.shard, self.lo, pk, nk,
                            self.D, self.gamma, self.emb_range, self.modulus, part)
            k.score_sharded(self.fn, SINGLE, ph, self.relation_embedding, self.rel_off, self.shard, self.lo, pk,
                            None, self.D, self.gamma, self.emb_range, self.modulus, part[:, N:])
            if dist_on:
                pending.append((_reduce_scatter_rows_into(home[kk * Bk:(kk + 1) * Bk], part, W, self.rank,
                                                          self.group), part))
        for h, _ in pending:
            if h is not None:
                h.wait()
        scores = home[:, :N].contiguous()
        # 4. per-row reductions on the home rank
        out_neg = k.neg_reduce(scores, temperature, adversarial)
        out_pos = k.log_sigmoid(home[:, N].contiguous())
        return out_neg, out_pos, scores

    def step_forward_gather(self, pos_g, neg_g, mode, temperature=1.0, adversarial=True):
        """Same contract and results as step_forward (bitwise: the same rows reach the same kernel
        arithmetic), by fetching the home rows' entity rows from their owners (all-to-all)."""
        mode = ops.mode_id(mode)
        if mode not in (HEAD_BATCH, TAIL_BATCH):
            raise ValueError("step_forward_gather needs a negative mode (0 or 1)")
        WB, N = neg_g.shape
        W, r = self.world, self.rank
        if WB % W:
            raise ValueError("global batch must split evenly over ranks")
        B = WB // W
        dev = self.device
        pos_h = pos_g[r * B:(r + 1) * B].contiguous()
        neg_h = neg_g[r * B:(r + 1) * B].contiguous()
        ids = torch.cat([neg_h.reshape(-1), pos_h[:, 0], pos_h[:, 2]])
        inr = (ids >= 0) & (ids < self.nentity)
        U = torch.unique(ids[inr])  # sorted ascending
        bounds = torch.tensor([shard_bounds(self.nentity, W, o)[0] for o in range(W)] + [self.nentity],
                              dtype=torch.int64, device=U.device)
        edges = torch.searchsorted(U, bounds)
        need = (edges[1:] - edges[:-1]).to(torch.int64)  # rows this rank needs from each owner
        if W > 1:
            allneed = [torch.empty_like(need) for _ in range(W)]
            dist.all_gather(allneed, need, group=self.group)
            C = torch.stack(allneed).cpu()  # C[q, o]: rows requester q needs from owner o
        else:
            C = need.cpu().view(1, 1)
        send_ids = C[r].tolist()                   # my requests, grouped by owner (U is owner-ordered)
        recv_ids = C[:, r].tolist()                # requests addressed to me, per requester
        if W > 1:
            req = torch.empty(sum(recv_ids), dtype=torch.int64, device=U.device)
            dist.all_to_all_single(req, U, recv_ids, send_ids, group=self.group)
        else:
            req = U
        rows_out = torch.empty((req.numel(), self.entity_dim), dtype=torch.float32, device=dev)
        if req.numel():
            self.kernels.gather_rows(self.shard, self.lo, req.to(dev), 1, req.numel(), rows_out)
        cache = torch.zeros((U.numel() + 1, self.entity_dim), dtype=torch.float32, device=dev)  # + zero row
        if W > 1:
            dist.all_to_all_single(cache[:U.numel()], rows_out, [c * 1 for c in send_ids], recv_ids,
                                   group=self.group)
        else:
            cache[:U.numel()] = rows_out
        # home ids -> cache rows (out-of-range ids -> the zero row, TF-GPU gather semantics)
        loc = torch.searchsorted(U, ids.clamp(0, max(self.nentity - 1, 0)))
        loc = torch.where(inr, loc, torch.full_like(loc, U.numel()))
        neg_l = loc[:B * N].view(B, N).contiguous()
        pos_l = pos_h.clone()
        pos_l[:, 0] = loc[B * N:B * N + B]
        pos_l[:, 2] = loc[B * N + B:]
        out_neg, out_pos, scores = self.kernels.step_forward(
            self.fn, mode, cache, self.relation_embedding, self.rel_off, pos_l.to(dev), neg_l.to(dev), self.D,
            self.gamma, self.emb_range, self.modulus, temperature, adversarial)
        return out_neg, out_pos, scores
