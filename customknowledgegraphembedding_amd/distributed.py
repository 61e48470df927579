"""Multi-GPU scoring: one process per GPU, torch.distributed over RCCL (backend "nccl") on xGMI.

Two layouts:

* Replicas (C2 WN18RR, C3 FB15k-237; any table that fits one GPU's 288 GB): every rank holds the
  whole table and scores its own batch rows; the data path has no collective (bench.py --gpus N).
* Row-sharded owner-computes (`ShardedKGE`; C4 YAGO3-10 as the north star names it, and any table
  larger than one GPU): rank r owns entity rows [lo_r, hi_r). The global batch (W*B rows, home rank h
  owning rows [h B, (h+1) B)) is known to every rank (the sampler seed is replicated, so no ids move),
  so every rank can work out from the ids alone who owns which row and in which order it will send it:
  the collectives carry payload only. One step (`step_forward`):
    0. plan: ownership counts and ranks of the batch's candidates and query rows,     kge_shard_plan
       and this rank's bucket: its owned candidates per row grouped by XCD slice
       (made a step ahead, on a side stream: it overlaps the previous step's scoring)
    1. query rows (the negative call's query entity only): each owner gathers the
       rows it owns, compacted; one ALL-TO-ALL sends that block to every rank           RCCL
    2. every rank scores only the candidates it owns (its bucket: no walk over the
       other ranks' ids), writing the scores compacted per row (column order, the
       row's positive last) into one block per home rank                               kge_shard_score
       (head-batch positives: the owner of the head, with the tail from step 1)
    3. one ALL-TO-ALL: home h receives exactly the scores of its rows, no indices       RCCL
    4. home rank: scatter by the same ranks, self-adversarial reduction, logsigmoid     kge_shard_finish
  Each (row, candidate) has exactly one owner and is moved once: the sharded scores equal the
  unsharded ones bitwise. (An id without an owner — out of range — scores 0 here; the unsharded
  kernels score it against a zero row, as TF-GPU gather does.) Per step and rank the collectives
  move ~7/8 of (W B ent_dim) query floats in and ~7/8 of (B (N+1)) scores in, against 2 x ncol times
  those queries and W times those scores for the zero-padded SUM all-reduce / reduce-scatter of
  round 2. Pipelining: the global batch is cut into K chunks of W/K whole homes; every chunk's query
  exchange is issued up front, chunk k is scored as soon as its rows arrived, and its score
  all-to-all runs on RCCL's stream while chunk k+1 is scored. At W = 1 the step is the unsharded
  fused forward.

* Row-sharded gather (`ShardedKGE.step_forward_gather`, the north star's literal scheme, kept beside
  owner-computes as SURVEY §8e asks so the two can be measured against each other): every rank
  fetches the rows its own B home rows need. Per step a rank dedups its ids (sorted unique), sends
  each owner the ids in that owner's range (all-to-all), receives the rows (all-to-all), and scores
  locally on the fetched cache with the unsharded kernels (kge_step_forward). Moves ~|unique rows| x
  ent_dim x 4 bytes per rank (C4 at 8 ranks: ~45k rows, ~89 MB) instead of owner-computes' queries
  + scores, which is why owner-computes is the default.

Every collective goes through a communicator object (`TorchComm`: one torch.distributed call per
method; `ThreadComm`: the same methods between W threads of one process, so a W-rank step runs on
one GPU). The GPU kernels are reached through a backend object (`HipShardKernels`); tests on CPU swap
in an oracle-backed backend to check the orchestration with gloo (tests/test_distributed_cpu.py).
"""
from __future__ import annotations

import collections
import warnings

import numpy as np
import torch
import torch.distributed as dist

from . import ops
from ._lib import FN_IDS, HEAD_BATCH, SINGLE, TAIL_BATCH, KGEHipError, check
from . import _lib
from .model import _dims_for


# widest per-half dimension the row-sharded train kernels take (kge_shard_train_*: kFwdGradMaxG float4
# groups per lane, six accumulators per element in registers); wider models train on the dense path
SHARD_MAX_D = 1024


def shard_bounds(nentity: int, world: int, rank: int):
    """Block partition of entity rows: the first (nentity % world) ranks get one extra row."""
    base, extra = divmod(nentity, world)
    lo = rank * base + min(rank, extra)
    hi = lo + base + (1 if rank < extra else 0)
    return lo, hi


def default_chunks(world: int, chunks=None) -> int:
    """Chunks of the pipelined sharded forward: a divisor of W (each chunk is W/K whole homes),
    the largest <= the request (default 2: at the C4 size on MI355X a rank's scoring takes 63 us in one
    launch, 69 us in two, 85 us in four (launch ramp-up and tail per chunk), while two chunks already
    hide half of each all-to-all behind scoring)."""
    want = max(1, min(int(chunks if chunks is not None else 2), world))
    while world % want:
        want -= 1
    return want


KGE_SHARD_TWO_COLUMNS = 1  # include/kge_hip.h


def query_cols(mode: int, flags: int = 0):
    """Columns of pos whose entity rows the exchange moves: the negative call's query entity (head-batch:
    the tail, else the head) and, with KGE_SHARD_TWO_COLUMNS in head-batch mode, the positive call's (the
    head). Without it the head-batch positive is scored by the owner of its head."""
    return [2, 0] if (mode == HEAD_BATCH and flags & KGE_SHARD_TWO_COLUMNS) else ([2] if mode == HEAD_BATCH else [0])


def positive_col(mode: int, flags: int = 0):
    """Column of pos whose owner scores the positive (kge_shard_plan's candidate N)."""
    return 0 if (mode == HEAD_BATCH and not flags & KGE_SHARD_TWO_COLUMNS) else 2


# ------------------------------------------------------------------------------------------------
# communicators
# ------------------------------------------------------------------------------------------------
class _Done:
    """Handle of a collective that already completed."""

    def wait(self):
        return None


class TorchComm:
    """Every collective of the row-sharded steps, one torch.distributed call each (RCCL on ROCm
    device tensors, gloo on CPU tensors). async_op=True returns the work handle."""

    def __init__(self, group=None):
        self.group = group

    @property
    def world(self):
        return dist.get_world_size(self.group)

    @property
    def rank(self):
        return dist.get_rank(self.group)

    @staticmethod
    def _h(h):
        return _Done() if h is None else h

    def all_gather_into(self, out, inp, async_op=False):
        """out [W * inp.numel()] (any shape, contiguous) <- every rank's inp, rank-major."""
        return self._h(dist.all_gather_into_tensor(out.view(-1), inp.contiguous().view(-1), group=self.group,
                                                   async_op=async_op))

    def all_to_all(self, out, inp, out_splits, in_splits, async_op=False):
        """inp [sum(in_splits)] -> rank d gets inp's d-th piece; out [sum(out_splits)] holds the pieces
        sent to this rank, source-rank-major (torch.distributed.all_to_all_single)."""
        return self._h(dist.all_to_all_single(out, inp, [int(x) for x in out_splits], [int(x) for x in in_splits],
                                              group=self.group, async_op=async_op))

    def all_reduce_sum_(self, t, async_op=False):
        h = self._h(dist.all_reduce(t, op=dist.ReduceOp.SUM, group=self.group, async_op=async_op))
        return h if async_op else t

    def broadcast_(self, t, src):
        dist.broadcast(t, src=src, group=self.group)
        return t

    def all_gather_cat(self, t):
        """[W, *t.shape], rank-major."""
        out = torch.empty((self.world,) + tuple(t.shape), dtype=t.dtype, device=t.device)
        self.all_gather_into(out, t)
        return out


class NativeComm:
    """The RCCL communicator of libkge_hip.so (kge_comm_*, csrc/kge_comm.hip): the row-sharded step's
    collectives issued from C++ by the native executor (ShardedKGE.use_native), with no torch.distributed
    call on the per-step path. Made collectively, one per process: rank 0's 128-byte RCCL id reaches every
    rank through torch.distributed (`group`, any backend)."""

    def __init__(self, group=None, device=None):
        import ctypes
        lib = _lib.load()
        self.world, self.rank = dist.get_world_size(group), dist.get_rank(group)
        buf = ctypes.create_string_buffer(128)
        if self.rank == 0:
            check(lib.kge_comm_unique_id(ctypes.addressof(buf)), "kge_comm_unique_id")
        on_dev = dist.get_backend(group) == "nccl"
        idt = torch.frombuffer(bytearray(buf.raw), dtype=torch.uint8).clone()
        if on_dev:
            idt = idt.to(device if device is not None else torch.device("cuda", torch.cuda.current_device()))
        dist.broadcast(idt, src=dist.get_global_rank(group, 0) if group is not None else 0, group=group)
        buf = ctypes.create_string_buffer(bytes(idt.cpu().tolist()), 128)
        h = ctypes.c_void_p()
        check(lib.kge_comm_init(ctypes.addressof(h), ctypes.addressof(buf), self.world, self.rank), "kge_comm_init")
        self.handle = h.value

    def all_to_all(self, out, inp, out_splits, in_splits, async_op=False):
        """TorchComm.all_to_all's contract (float tensors) through ncclAllToAllv on torch's current stream."""
        import ctypes
        W = self.world
        sc, rc = (ctypes.c_int64 * W)(*[int(x) for x in in_splits]), (ctypes.c_int64 * W)(*[int(x) for x in out_splits])
        check(_lib.load().kge_comm_all_to_allv(self.handle, inp.data_ptr(), ctypes.addressof(sc), out.data_ptr(),
                                               ctypes.addressof(rc), _st(inp)), "kge_comm_all_to_allv")
        return _Done()

    def all_reduce_sum_(self, t, async_op=False):
        check(_lib.load().kge_comm_all_reduce_sum(self.handle, t.data_ptr(), t.numel(), _st(t)), "kge_comm_all_reduce_sum")
        return _Done() if async_op else t

    def close(self):
        if getattr(self, "handle", None):
            check(_lib.load().kge_comm_destroy(self.handle), "kge_comm_destroy")
            self.handle = None


class _NativeHandle:
    def __init__(self, handle, world, rank):
        self.handle, self.world, self.rank = handle, world, rank


class LoopbackGroup:
    """W native communicators of ONE process (kge_comm_loopback_*): the native executor's W-rank step on
    one GPU, one host thread per rank (run_threads) and one compute stream per rank (ranks sharing a stream
    would wait on each other's queued work), as ThreadComm runs the Python path. comm(r) -> rank r's."""

    def __init__(self, world):
        import ctypes
        lib = _lib.load()
        self.world = world
        self._g = lib.kge_comm_loopback_group(world)
        if not self._g:
            check(-22, "kge_comm_loopback_group")
        self._comms = []
        for r in range(world):
            h = ctypes.c_void_p()
            check(lib.kge_comm_loopback_init(ctypes.addressof(h), self._g, r), "kge_comm_loopback_init")
            self._comms.append(_NativeHandle(h.value, world, r))

    def comm(self, rank):
        return self._comms[rank]

    def close(self):
        lib = _lib.load()
        for c in self._comms:
            check(lib.kge_comm_destroy(c.handle), "kge_comm_destroy")
        self._comms = []
        if self._g:
            check(lib.kge_comm_loopback_group_destroy(self._g), "kge_comm_loopback_group_destroy")
            self._g = None


class NativeShardExec:
    """One rank's row-sharded forward step as ONE C call (kge_shard_exec_*, csrc/kge_comm.hip): the plan of
    the next batch, the query exchange, owner-computes scoring, the score exchange and the finish, with the
    collectives on the executor's communication stream (RCCL through `comm`, a NativeComm) and the step's
    kernels on torch's current stream. comm None: world 1 (the pieces are device copies), or `probe` at any
    world (collectives skipped, outputs meaningless: the host-cost probe). The workspace and the pinned
    summary buffers are torch allocations owned here."""

    def __init__(self, sk, Bg, N, comm=None, probe=False, chunks=None, one_stream=False, timing=False):
        import ctypes
        lib = _lib.load()
        W, K = sk.world, default_chunks(sk.world, chunks)
        self.lib, self.Bg, self.N, self.B, self.K = lib, Bg, N, Bg // W, K
        nbytes = lib.kge_shard_exec_workspace_size(Bg, N, sk.entity_dim, W, K)
        check(int(nbytes) if nbytes < 0 else 0, "kge_shard_exec_workspace_size")
        self.ws = torch.empty(nbytes + 256, dtype=torch.uint8, device=sk.device)
        ws = (self.ws.data_ptr() + 255) & ~255
        hi = lib.kge_shard_exec_host_ints(W, K)
        self.host = torch.empty(hi, dtype=torch.int32, pin_memory=True)
        h = ctypes.c_void_p()
        # KGE_EXEC_PROBE, KGE_EXEC_ONE_STREAM, KGE_EXEC_TIMING
        flags = (1 if probe else 0) | (2 if one_stream else 0) | (4 if timing else 0)
        check(lib.kge_shard_exec_create(ctypes.addressof(h), None if comm is None else comm.handle, flags,
                                        sk.fn, sk.nentity, sk.shard.shape[0], sk.entity_dim, sk.D, Bg, N, W, sk.rank,
                                        K, ws, nbytes, self.host.data_ptr(), hi), "kge_shard_exec_create")
        self.handle = h.value
        self.sk = sk
        self.comm = comm
        # the batches planned ahead, oldest first: (pos, neg, mode, their tensor versions). The plan stream reads
        # their ids asynchronously, and the C side matches a step to its plan by pointer: holding the tensors
        # here until their step keeps the caching allocator from handing their memory to another batch, and the
        # versions catch an in-place change of the ids between plan and step (the plan would be stale)
        self._fifo = collections.deque()
        self.broken = None  # the error of a failed step: the executor (and, under RCCL, its peers) is unusable

    def _live(self):
        if self.broken is not None:
            raise KGEHipError(f"the native executor failed earlier ({self.broken}); an exec error is fatal to its "
                              "communicator: make a new ShardedKGE / NativeComm")

    def plan(self, pos_g, neg_g, mode):
        self._live()
        check(self.lib.kge_shard_exec_plan(self.handle, pos_g.data_ptr(), neg_g.data_ptr(), neg_g.stride(0), mode,
                                           _st(neg_g)), "kge_shard_exec_plan")
        self._fifo.append((pos_g, neg_g, mode, pos_g._version, neg_g._version))

    def step(self, pos_g, neg_g, mode, temperature, adversarial, nxt=None):
        self._live()
        if self._fifo:
            p0, n0, m0, v0, w0 = self._fifo[0]
            if p0 is not pos_g or n0 is not neg_g or m0 != mode:
                raise KGEHipError("NativeShardExec.step: the oldest batch planned ahead is another batch or mode "
                                  "(steps must consume the planned batches in order)")
            if pos_g._version != v0 or neg_g._version != w0:
                raise KGEHipError("NativeShardExec.step: the batch's ids changed in place after it was planned")
        sk, B, N = self.sk, self.B, self.N
        out = torch.empty(B * (N + 3), dtype=torch.float32, device=sk.device)
        base = out.data_ptr()
        sh, rel = sk.shard, sk.relation_embedding
        npos, nneg, nmode = (nxt[0].data_ptr(), nxt[1].data_ptr(), nxt[2]) if nxt is not None else (None, None, 0)
        try:
            check(self.lib.kge_shard_exec_step(
                self.handle, sh.data_ptr(), sh.stride(0), sk.lo, rel.data_ptr(), rel.shape[0], rel.stride(0),
                sk.rel_off, pos_g.data_ptr(), neg_g.data_ptr(), neg_g.stride(0), mode, sk.gamma, sk.emb_range,
                sk.modulus, temperature, int(adversarial), npos, nneg, nmode, base, N, base + B * N * 4,
                base + B * (N + 1) * 4, base + B * (N + 2) * 4, _st(sh)), "kge_shard_exec_step")
        except KGEHipError as e:
            self.broken = str(e)
            raise
        if self._fifo:
            self._fifo.popleft()
        if nxt is not None:
            self._fifo.append((nxt[0], nxt[1], nxt[2], nxt[0]._version, nxt[1]._version))
        return out[B * N:B * (N + 1)], out[B * (N + 2):], out[:B * N].view(B, N)

    def timings(self):
        """KGE_EXEC_TIMING executors: the last step's device spans in us (kge_shard_exec_timings): step,
        query gather, finish, and per chunk (query all-to-all, scoring, score all-to-all)."""
        import ctypes
        n = 3 + 3 * self.K
        buf = (ctypes.c_float * n)()
        check(self.lib.kge_shard_exec_timings(self.handle, ctypes.addressof(buf), n), "kge_shard_exec_timings")
        v = list(buf)
        return {"step_us": v[0], "gather_us": v[1], "finish_us": v[2],
                "query_a2a_us": [v[3 + 3 * k] for k in range(self.K)],
                "score_us": [v[4 + 3 * k] for k in range(self.K)],
                "score_a2a_us": [v[5 + 3 * k] for k in range(self.K)]}

    def host_wait_us(self, reset=True):
        return float(self.lib.kge_shard_exec_host_wait_us(self.handle, int(reset)))

    def close(self):
        """Destroys the executor (its streams and events); its buffers go with this object. Not done at
        garbage collection: an executor left open at exit is reclaimed with the process."""
        if getattr(self, "handle", None):
            torch.cuda.synchronize(self.sk.device)
            check(self.lib.kge_shard_exec_destroy(self.handle), "kge_shard_exec_destroy")
            self.handle = None


class ThreadComm:
    """The same collectives between W threads of ONE process (one Python thread per simulated rank,
    all on one device and stream): used to run the W-rank sharded steps on a single GPU. Sums are
    taken in rank order, as RCCL's result is the same on every rank. `view(rank)` is the per-rank
    communicator (TorchComm's methods); ShardedKGE takes the ThreadComm itself and makes the view."""

    def __init__(self, world):
        import threading
        self.world = world
        self._barrier = threading.Barrier(world, timeout=120)  # a failed rank breaks it instead of hanging
        self._slots = [None] * world

    def view(self, rank):
        return _ThreadCommRank(self, rank)

    def _exchange(self, rank, t):
        self._slots[rank] = t
        self._barrier.wait()
        got = list(self._slots)
        self._barrier.wait()
        return got

    # rank-explicit forms (kept for callers holding the shared object)
    def all_gather_cat(self, t, rank):
        return self.view(rank).all_gather_cat(t)

    def all_reduce_sum_(self, t, rank):
        return self.view(rank).all_reduce_sum_(t)


class _ThreadCommRank:
    def __init__(self, shared, rank):
        self.shared, self.rank, self.world = shared, rank, shared.world

    def all_gather_into(self, out, inp, async_op=False):
        parts = self.shared._exchange(self.rank, inp.contiguous())
        flat = out.view(-1)
        n = parts[0].numel()
        for r, x in enumerate(parts):
            flat[r * n:(r + 1) * n].copy_(x.view(-1))
        return _Done()

    def all_to_all(self, out, inp, out_splits, in_splits, async_op=False):
        got = self.shared._exchange(self.rank, (inp, [int(x) for x in in_splits]))
        at = 0
        for src, (x, splits) in enumerate(got):
            n = splits[self.rank]
            if n != int(out_splits[src]):
                raise RuntimeError(f"all_to_all: rank {src} sends {n} to rank {self.rank}, which expects "
                                   f"{int(out_splits[src])}")
            off = sum(splits[:self.rank])
            if n:
                out[at:at + n].copy_(x[off:off + n])
            at += n
        return _Done()

    def all_reduce_sum_(self, t, async_op=False):
        parts = self.shared._exchange(self.rank, t.clone())
        acc = parts[0].clone()
        for x in parts[1:]:
            acc += x
        t.copy_(acc)
        return _Done() if async_op else t

    def broadcast_(self, t, src):
        parts = self.shared._exchange(self.rank, t)
        if src != self.rank:
            t.copy_(parts[src])
        return t

    def all_gather_cat(self, t):
        return torch.stack(self.shared._exchange(self.rank, t.contiguous()))


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


# ------------------------------------------------------------------------------------------------
# the exchange plan of one global batch
# ------------------------------------------------------------------------------------------------
class ShardPlan:
    """Ownership counts and ranks of one global batch (kge_shard_plan; identical on every rank but for
    the bucket). Device arrays: cnt, hpre [W, Bg], qown, qslot [ncol, Bg], and (the forward's plans)
    rank `rank`'s bucket [Bg, N+1, 2] / bucket_start [Bg, 9]: its owned candidates per row grouped by XCD
    slice, the input of kge_shard_score. `summary()` -> (tot [W, W], qtot [K, ncol, W]) on the host:
    tot[h, o] = scores of home h's rows owned by rank o (the score all-to-all's split sizes), qtot[k, c,
    o] = chunk k's column-c query rows owned by o (the query all-to-all's). The host copy is issued
    asynchronously when the plan is made: a plan made one step ahead costs no host wait."""

    def __init__(self, world, chunks, mode, Bg, N, cnt, hpre, qown, qslot, summary_dev, summary_host, event,
                 flags=0, rank=None, bucket=None, bucket_start=None):
        self.world, self.chunks, self.mode, self.Bg, self.N, self.flags = world, chunks, mode, Bg, N, flags
        self.ncol = len(query_cols(mode, flags))
        self.cnt, self.hpre, self.qown, self.qslot = cnt, hpre, qown, qslot
        self.rank, self.bucket, self.bucket_start = rank, bucket, bucket_start
        self._dev, self._host, self._event = summary_dev, summary_host, event
        self._parsed = None

    def use_on(self, stream):
        """A plan made on a side stream (ShardedKGE.plan(stream=...)): `stream` waits for it, and its device
        arrays are marked as used there (the caching allocator must not hand them to the side stream's next
        plan while this stream's kernels still read them)."""
        if getattr(self, "stream", None) is None or self.stream == stream:
            return
        stream.wait_event(self._event)
        for t in (self.cnt, self.hpre, self.qown, self.qslot, self._dev, self.bucket, self.bucket_start):
            if t is not None:
                t.record_stream(stream)
        self.stream = stream

    def layout(self, rank):
        """This rank's split sizes of the forward's exchange, as Python ints (computed once per plan):
        per chunk k, the query all-to-all (send offset and length into the all-chunk send block, received
        rows, out / in splits in floats of ent_dim rows: set by ShardedKGE) and the score all-to-all (in
        splits, send length, out splits, received length). The host path of step_forward reads only this."""
        lay = self.__dict__.get("_layout")
        if lay is not None and lay[0] == rank:
            return lay[1]
        tot, qtot = self.summary()
        W, K = self.world, self.chunks
        hpc = W // K
        qper = qtot.sum(1).tolist()  # [K][W] query rows of chunk k owned by o
        totl = tot.tolist()
        k_home = rank // hpc
        chunks = []
        for k in range(K):
            per = qper[k]
            sin = [totl[h][rank] if k * hpc <= h < (k + 1) * hpc else 0 for h in range(W)]
            sout = totl[rank] if k == k_home else [0] * W
            chunks.append({"qper": per, "q_mine": per[rank], "q_rows": sum(per), "s_in": sin, "s_send": sum(sin),
                           "s_out": sout, "s_recv": sum(sout)})
        lay = {"chunks": chunks, "k_home": k_home, "q_send_rows": W * sum(c["q_mine"] for c in chunks)}
        self._layout = (rank, lay)
        return lay

    def summary(self):
        if self._parsed is None:
            if self._event is not None:
                self._event.synchronize()
            s = self._host.numpy().astype(np.int64)
            W, K, nc = self.world, self.chunks, self.ncol
            self._parsed = (s[:W * W].reshape(W, W), s[W * W:W * W + K * nc * W].reshape(K, nc, W))
        return self._parsed


# ------------------------------------------------------------------------------------------------
# kernels
# ------------------------------------------------------------------------------------------------
def _st(t):
    return torch.cuda.current_stream(t.device).cuda_stream


class HipShardKernels:
    """libkge_hip.so entry points used by ShardedKGE (device tensors, torch's current stream)."""

    @staticmethod
    def gather_rows(table, lo, ids, id_stride, n, out):
        rc = _lib.load().kge_gather_rows(table.data_ptr(), table.shape[0], table.stride(0), lo, ids.data_ptr(),
                                         id_stride, n, out.shape[1], out.data_ptr(), out.stride(0), _st(table))
        check(rc, "kge_gather_rows")

    @staticmethod
    def score_sharded(fn, mode, qent, rel, rel_off, shard, lo, pos, neg, D, gamma, emb_range, modulus, out):
        B = pos.shape[0]
        N = 1 if mode == SINGLE else neg.shape[1]
        rc = _lib.load().kge_score_sharded(
            fn, mode, qent.data_ptr(), qent.stride(0), rel.data_ptr(), rel.shape[0], rel.stride(0), rel_off,
            shard.data_ptr(), shard.shape[0], shard.stride(0), lo, pos.data_ptr(),
            None if mode == SINGLE else neg.data_ptr(), 0 if mode == SINGLE else neg.stride(0), B, N, D,
            float(gamma), float(emb_range), float(modulus), out.data_ptr(), out.stride(0), _st(shard))
        check(rc, "kge_score_sharded")

    # ---- the O(information) exchange of the sharded forward (kge_shard_*; include/kge_hip.h) ----
    @staticmethod
    def plan(sk, pos_g, neg_g, mode, chunks, flags=0):
        Bg, N = neg_g.shape
        W = sk.world
        nc = len(query_cols(mode, flags))
        i32 = dict(dtype=torch.int32, device=neg_g.device)
        cnt, hpre = torch.empty((W, Bg), **i32), torch.empty((W, Bg), **i32)
        qown, qslot = torch.empty((nc, Bg), **i32), torch.empty((nc, Bg), **i32)
        summ = torch.empty(W * W + chunks * nc * W, **i32)
        bucket = bstart = None
        if flags == 0:  # the forward: this rank's bucket for kge_shard_score
            bucket, bstart = torch.empty((Bg, N + 1, 2), **i32), torch.empty((Bg, 9), **i32)
        rc = _lib.load().kge_shard_plan(pos_g.data_ptr(), neg_g.data_ptr(), neg_g.stride(0), Bg, N, sk.nentity, W,
                                        chunks, mode, flags, sk.rank, cnt.data_ptr(), hpre.data_ptr(),
                                        qown.data_ptr(), qslot.data_ptr(), summ.data_ptr(),
                                        None if bucket is None else bucket.data_ptr(),
                                        None if bstart is None else bstart.data_ptr(), _st(neg_g))
        check(rc, "kge_shard_plan")
        host = sk._pinned(summ.numel())
        host.copy_(summ, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        return ShardPlan(W, chunks, mode, Bg, N, cnt, hpre, qown, qslot, summ, host, ev, flags, sk.rank, bucket,
                         bstart)

    @staticmethod
    def gather_queries(sk, plan, pos_g, k, send, qidx, st=None):
        """Query rows this rank owns -> send (chunk k's block, or k = -1: every chunk's, back to back)."""
        rc = _lib.load().kge_shard_gather_queries(
            sk.shard.data_ptr(), sk.shard.shape[0], sk.shard.stride(0), sk.lo, pos_g.data_ptr(), plan.Bg,
            plan.chunks, k, sk.entity_dim, sk.world, sk.rank, plan.mode, plan.flags, plan.qown.data_ptr(),
            plan.qslot.data_ptr(), plan._dev.data_ptr(), send.data_ptr() if send.numel() else None, qidx.data_ptr(),
            st if st is not None else _st(sk.shard))
        check(rc, "kge_shard_gather_queries")

    @staticmethod
    def score_compact(sk, qblock, qidx, pos_g, neg_g, plan, row0, rows, send, st=None):
        """Owned scores (negatives and positives) of rows [row0, row0 + rows) (whole homes) -> send,
        compacted (kge_shard_score over the plan's bucket). Row offsets into the plan's arrays are taken by
        pointer arithmetic (no tensor slicing on the host path)."""
        if plan.rank != sk.rank or plan.bucket is None:
            raise ValueError("kge_shard_score needs a forward plan made by this rank (its bucket)")
        if send.numel() == 0:  # this rank owns none of these rows' candidates
            return
        hB = plan.Bg // sk.world
        rel = sk.relation_embedding
        me = sk.rank
        bk, bs, hp, cn = plan.bucket, plan.bucket_start, plan.hpre, plan.cnt
        rc = _lib.load().kge_shard_score(
            sk.fn, plan.mode, qblock.data_ptr(), qblock.shape[0], qblock.stride(0), qidx.data_ptr(),
            rel.data_ptr(), rel.shape[0], rel.stride(0), sk.rel_off, sk.shard.data_ptr(), sk.shard.shape[0],
            sk.shard.stride(0), sk.lo, pos_g.data_ptr() + row0 * pos_g.stride(0) * 8, rows, plan.N, sk.D,
            float(sk.gamma), float(sk.emb_range), float(sk.modulus), bk.data_ptr() + row0 * bk.stride(0) * 4,
            bs.data_ptr() + row0 * bs.stride(0) * 4, hp.data_ptr() + (me * hp.stride(0) + row0) * 4,
            cn.data_ptr() + (me * cn.stride(0) + row0) * 4, plan._dev.data_ptr(), sk.world, me, hB, row0 // hB,
            send.data_ptr(), st if st is not None else _st(sk.shard))
        check(rc, "kge_shard_score")

    @staticmethod
    def shard_finish(sk, plan, recv, pos_g, neg_g, temperature, adversarial, st=None):
        W, r = sk.world, sk.rank
        B, N = plan.Bg // W, plan.N
        # the four outputs in one allocation: scores [B, N], out_neg, pos_raw, out_pos [B]
        out = torch.empty(B * (N + 3), dtype=torch.float32, device=neg_g.device)
        base = out.data_ptr()
        rc = _lib.load().kge_shard_finish(
            recv.data_ptr() if recv.numel() else None, plan._dev.data_ptr(), plan.hpre.data_ptr(), pos_g.data_ptr(),
            neg_g.data_ptr(), neg_g.stride(0), plan.Bg, N, sk.nentity, W, r, plan.mode, float(temperature),
            int(adversarial), base, N, base + B * N * 4, base + B * (N + 1) * 4, base + B * (N + 2) * 4,
            st if st is not None else _st(neg_g))
        check(rc, "kge_shard_finish")
        return out[B * N:B * (N + 1)], out[B * (N + 2):], out[:B * N].view(B, N)

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
        rc = _lib.load().kge_shard_train_forward(*cls._prefix(sk, bufs, mode, qent, qent_pos, pos, neg, w),
                                                 bufs["stats"].data_ptr(), bufs["dq"].data_ptr(), bufs["ws"].data_ptr(),
                                                 bufs["ws"].numel(), _st(sk.shard))
        check(rc, "kge_shard_train_forward")

    @classmethod
    def train_combine(cls, sk, bufs, mode, qent, qent_pos, pos, neg, w, stats_all):
        rc = _lib.load().kge_shard_train_combine(*cls._prefix(sk, bufs, mode, qent, qent_pos, pos, neg, w),
                                                 stats_all.data_ptr(), bufs["dq"].data_ptr(),
                                                 bufs["out_neg"].data_ptr(), bufs["out_pos_raw"].data_ptr(),
                                                 bufs["out_pos"].data_ptr(), bufs["ws"].data_ptr(), bufs["ws"].numel(),
                                                 _st(sk.shard))
        check(rc, "kge_shard_train_combine")

    @classmethod
    def train_backward(cls, sk, bufs, mode, qent, qent_pos, pos, neg, w, step, loss_sum):
        a = sk.adam
        rc = _lib.load().kge_shard_train_backward(
            *cls._prefix(sk, bufs, mode, qent, qent_pos, pos, neg, w), bufs["dq"].data_ptr(),
            bufs["loss"].data_ptr(), None if loss_sum is None else loss_sum.data_ptr(), a["m_ent"].data_ptr(),
            a["v_ent"].data_ptr(), a["m_rel"].data_ptr(), a["v_rel"].data_ptr(), float(a["lr"]), float(a["b1"]),
            float(a["b2"]), float(a["eps"]), int(step), int(a["keras"]), bufs["ws"].data_ptr(), bufs["ws"].numel(),
            _st(sk.shard))
        check(rc, "kge_shard_train_backward")
        return bufs["loss"]


# ------------------------------------------------------------------------------------------------
# the row-sharded model
# ------------------------------------------------------------------------------------------------
class ShardedKGE:
    """Row-sharded owner-computes forward of supervisor.py:17-18 (both model calls) and train step
    (supervisor.py:15-26 across replicas).

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
        if isinstance(comm, ThreadComm):
            comm = comm.view(self.rank)
        self.comm = comm if comm is not None else (TorchComm(group) if self.world > 1 else None)
        # the exchange runs through self.comm (W > 1). At W = 1 the steps skip it (it is the identity) unless a
        # communicator was given and `exchange` is set: tests run the whole collective path under RCCL on one GPU
        self.exchange = self.world > 1
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
            self.modulus = float(ref.modulus.detach().reshape(-1)[0]) if model_name == "pRotatE" else 0.0
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
        self.loss_sum = None  # optional 0-dim fp32 device tensor: the step adds W * sum(replica losses)
        self._bufs = {}
        self._wsb = {}
        self._native_cfg, self._native = None, {}
        self._pin, self._pin_i = [], 0

    @classmethod
    def from_model(cls, model, group=None, kernels=None, world=None, rank=None, comm=None):
        """A sharded view of an existing TFKGEModel / KGEModel: this rank's shard IS rows [lo, hi) of the
        model's entity table (a view: updates land in the model's own storage) and the relation table
        is the model's (updated identically on every rank). Rows outside the shard go stale during
        training until `sync_entity_table` re-broadcasts every rank's block. With a ThreadComm (W
        simulated ranks of one process) each rank gets its own copy of the relation table: W in-place
        relation updates of one shared tensor would compound. Training through such a view therefore
        leaves `model.relation_embedding` unchanged: call `sync_relation_table(model.relation_embedding)`
        (from any one rank) to copy the replicas' table back."""
        ent = model.entity_embedding.data
        rel = model.relation_embedding.data
        if isinstance(comm, (ThreadComm, _ThreadCommRank)):
            rel = rel.clone()
        modulus = float(model.modulus.detach().reshape(-1)[0]) if model.model_name == "pRotatE" else 0.0
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
            self.comm.broadcast_(blk, r)
        return table

    def sync_relation_table(self, table):
        """This rank's relation table -> `table` (the replicas' tables are identical after every step). With
        a ThreadComm, from_model gave each simulated rank a copy; this writes the trained one back."""
        if table.data_ptr() != self.relation_embedding.data_ptr():
            table.copy_(self.relation_embedding)
        return table

    def configure_optimizer(self, lr=5e-5, betas=(0.9, 0.999), eps=None, semantics="keras"):
        """Adam over this rank's shard and the replicated relation table (supervisor.py:26; run.py:111
        Keras Adam by default). Every rank applies the same relation update, so the replicas stay equal.
        The entity moments exist only for this rank's rows (Trainer keeps them as views of the
        optimizer's full-table state, whose rows outside the shard are never advanced by this rank)."""
        if eps is None:
            eps = 1e-7 if semantics == "keras" else 1e-8
        self.adam = {"m_ent": torch.zeros_like(self.shard), "v_ent": torch.zeros_like(self.shard),
                     "m_rel": torch.zeros_like(self.relation_embedding),
                     "v_rel": torch.zeros_like(self.relation_embedding),
                     "lr": lr, "b1": betas[0], "b2": betas[1], "eps": eps, "keras": semantics == "keras"}
        self.step = 0
        return self

    # ---- the exchange (§ module docstring) ----
    def _pinned(self, n):
        """A pinned host int32 buffer for a plan's summary (a ring of four: plans made ahead stay valid)."""
        if len(self._pin) < 4 or self._pin[self._pin_i].numel() < n:
            buf = torch.empty(max(n, 64), dtype=torch.int32, pin_memory=torch.cuda.is_available())
            if len(self._pin) < 4:
                self._pin.append(buf)
                self._pin_i = len(self._pin) - 1
            else:
                self._pin[self._pin_i] = buf
        out = self._pin[self._pin_i][:n]
        self._pin_i = (self._pin_i + 1) % 4
        return out

    def plan(self, pos_g, neg_g, mode, chunks=None, flags=0, stream=None):
        """The exchange plan of a global batch (kge_shard_plan, two launches, the split sizes copied to the
        host asynchronously). Make it one step ahead and pass it to step_forward(plan=...) so the host never
        waits for it; with `stream` (a side stream) its integer work also overlaps the current step's
        gather-bound scoring on the device (the side stream first waits for the current stream's queued
        work, which made the ids)."""
        mode = ops.mode_id(mode)
        if mode not in (HEAD_BATCH, TAIL_BATCH):
            raise ValueError("the sharded step needs a negative mode (0 or 1)")
        WB = neg_g.shape[0]
        if WB % self.world:
            raise ValueError("global batch must split evenly over ranks")
        K = default_chunks(self.world, chunks)
        if stream is None:
            p = self.kernels.plan(self, pos_g, neg_g, mode, K, flags)
        else:
            stream.wait_stream(torch.cuda.current_stream(self.device))
            with torch.cuda.stream(stream):
                p = self.kernels.plan(self, pos_g, neg_g, mode, K, flags)
            p.stream = stream
        p.ids = (pos_g.data_ptr(), neg_g.data_ptr())  # step_forward(plan=...) checks it is this batch's plan
        return p

    def _ws(self, name, n, dtype=torch.float32):
        """A view of n elements of this rank's persistent exchange buffer `name` (grown by 1.25x when too
        small). Reuse across steps is stream-ordered: every collective that touches a buffer is waited for on
        the current stream before the step returns, so the next step's kernels come after it."""
        b = self._wsb.get(name)
        if b is None or b.numel() < n or b.dtype != dtype:
            b = torch.empty(max(int(n * 1.25), 1), dtype=dtype, device=self.device)
            self._wsb[name] = b
        return b[:n]

    def _exchange_queries(self, plan, pos_g, st=None):
        """Every chunk's query rows: each owner's compacted rows sent to every rank (one gather launch for
        all chunks, then one async all-to-all per chunk). Returns [(block [rows, ent_dim], qidx [ncol,
        Bg/K] into it, handle)] per chunk and the send buffer to keep alive."""
        W, K, d = self.world, plan.chunks, self.entity_dim
        lay = plan.layout(self.rank)
        send = self._ws("q_send", lay["q_send_rows"] * d)
        qidx = self._ws("q_idx", plan.ncol * plan.Bg, torch.int64).view(plan.ncol, plan.Bg)
        self.kernels.gather_queries(self, plan, pos_g, -1, send, qidx, st=st)
        Rk = plan.Bg // K
        out, at = [], 0
        for k, c in enumerate(lay["chunks"]):
            n = W * c["q_mine"] * d
            block = self._ws(f"q_block{k}", c["q_rows"] * d).view(c["q_rows"], d)
            h = self.comm.all_to_all(block.view(-1), send[at:at + n], [p * d for p in c["qper"]], [c["q_mine"] * d] * W,
                                     async_op=True)
            out.append((block, qidx[:, k * Rk:(k + 1) * Rk], h))
            at += n
        return out, send

    def use_native(self, comm=None, probe=False, one_stream=None, timing=False):
        """Run step_forward through the native executor (NativeShardExec: one C call per rank-step, RCCL
        issued from C++): `comm` a NativeComm (W > 1, or W = 1 through RCCL), None at W = 1 (device copies),
        or `probe` (collectives skipped: host-cost measurement only). One executor per batch shape.
        one_stream: the collectives on the step's own stream (KGE_EXEC_ONE_STREAM), the default: at C4 x 8 a
        rank-step's kernels run back to back in 100 us of device time that way, against 144-161 us with the
        collectives on a communication stream, whose cross-stream event hops (the dependent queue's wake-up)
        cost more than the overlap they buy (profiles/r04_native_timeline.txt); KGE_SHARD_ONE_STREAM=0 keeps
        the communication stream. With one stream the batch is one chunk unless `chunks` is given."""
        import os
        if comm is None and self.world > 1 and not probe:
            raise ValueError("the native executor needs a NativeComm at world > 1")
        if one_stream is None:
            one_stream = os.environ.get("KGE_SHARD_ONE_STREAM", "1") != "0"
        for ex in getattr(self, "_native", {}).values():
            ex.close()
        self._native_cfg = (comm, bool(probe), bool(one_stream), bool(timing))
        self._native = {}
        return self

    def _native_exec(self, Bg, N, chunks):
        if chunks is None and self._native_cfg[2]:
            chunks = 1  # one stream: no exchange overlaps scoring, and one scoring launch is the shortest
        key = (Bg, N, default_chunks(self.world, chunks))
        ex = self._native.get(key)
        if ex is None:
            comm, probe, one, timing = self._native_cfg
            ex = self._native[key] = NativeShardExec(self, Bg, N, comm=comm, probe=probe, chunks=chunks, one_stream=one,
                                                     timing=timing)
        return ex

    @staticmethod
    def _native_batch(pos_g, neg_g, mode):
        m = ops.mode_id(mode)
        if m not in (HEAD_BATCH, TAIL_BATCH):
            raise ValueError("the sharded step needs a negative mode (0 or 1)")
        if pos_g.stride() != (3, 1) or neg_g.stride(1) != 1:
            raise ValueError("the native step needs contiguous pos [Bg, 3] and row-major neg [Bg, N]")
        return m

    def plan_native(self, pos_g, neg_g, mode, chunks=None):
        """Plans a batch ahead for the native step (kge_shard_exec_plan, on the executor's plan stream after the
        current stream's queued work): up to three plans wait; step_forward consumes them in order, and each
        step given `nxt` plans that batch too. Planning two batches ahead lets the host run two steps ahead
        of the device."""
        if self._native_cfg is None:
            raise ValueError("plan_native needs use_native() first")
        m = self._native_batch(pos_g, neg_g, mode)
        Bg, N = neg_g.shape
        if Bg % self.world:
            raise ValueError("global batch must split evenly over ranks")
        self._native_exec(Bg, N, chunks).plan(pos_g, neg_g, m)

    def _native_step(self, pos_g, neg_g, mode, temperature, adversarial, chunks, nxt):
        m = self._native_batch(pos_g, neg_g, mode)
        Bg, N = neg_g.shape
        if Bg % self.world:
            raise ValueError("global batch must split evenly over ranks")
        ex = self._native_exec(Bg, N, chunks)
        if nxt is not None:
            nm = self._native_batch(nxt[0], nxt[1], nxt[2])
            if tuple(nxt[1].shape) != (Bg, N):
                raise ValueError("the batch planned ahead must have this batch's shape")
            nxt = (nxt[0], nxt[1], nm)
        return ex.step(pos_g, neg_g, m, temperature, adversarial, nxt)

    def step_forward(self, pos_g, neg_g, mode, temperature=1.0, adversarial=True, chunks=None, plan=None, nxt=None):
        """pos_g [W*B, 3], neg_g [W*B, N] (the global batch, identical on every rank) ->
        (out_neg [B], out_pos [B], scores [B, N]) for this rank's home rows [rank*B, (rank+1)*B).
        Collectives: per chunk one all-to-all of compacted query rows and one all-to-all of compacted
        owned scores, both through self.comm. At W = 1 the exchange is the identity and the step is the
        unsharded fused forward (kge_step_forward; the same scores bitwise).
        Host path (it bounds the step at W = 8: bench rank_host_cost): the split sizes come from the plan's
        cached layout, the exchange buffers are persistent (self._ws), the kernels get pointers and the
        stream handle computed once.
        After use_native(...) the whole step is one C call (NativeShardExec; `plan` must then be None): it
        consumes the oldest batch planned ahead (plan_native / an earlier step's `nxt`; planned inline if none
        waits), and `nxt` = (pos, neg, mode) of the batch after the planned ones is planned on the side."""
        W, me = self.world, self.rank
        if self._native_cfg is not None and plan is None:
            return self._native_step(pos_g, neg_g, mode, temperature, adversarial, chunks, nxt)
        if not self.exchange:
            m = ops.mode_id(mode)
            if m not in (HEAD_BATCH, TAIL_BATCH):
                raise ValueError("step_forward needs a negative mode (0 or 1)")
            return self.kernels.step_forward(self.fn, m, self.shard, self.relation_embedding, self.rel_off, pos_g,
                                             neg_g, self.D, self.gamma, self.emb_range, self.modulus, temperature,
                                             adversarial)
        if plan is None:
            plan = self.plan(pos_g, neg_g, mode, chunks)
        if plan.rank != me:
            raise ValueError("the plan was made by another rank (its bucket is that rank's)")
        if plan.mode != ops.mode_id(mode) or (plan.Bg, plan.N) != tuple(neg_g.shape):
            raise ValueError(f"the plan was made for mode {plan.mode}, batch {plan.Bg} x {plan.N}; this step is mode "
                             f"{ops.mode_id(mode)}, batch {tuple(neg_g.shape)}")
        ids = getattr(plan, "ids", None)
        if ids is not None and ids != (pos_g.data_ptr(), neg_g.data_ptr()):
            raise ValueError("the plan was made for other pos/neg tensors than this step's")
        cur = torch.cuda.current_stream(self.device) if self.device.type == "cuda" else None
        if getattr(plan, "stream", None) is not None:  # made on a side stream
            plan.use_on(cur)
        st = cur.cuda_stream if cur is not None else None
        K = plan.chunks
        Rk = plan.Bg // K
        lay = plan.layout(me)
        # 1. every chunk's query exchange in flight before any scoring
        qx, _qsend = self._exchange_queries(plan, pos_g, st)
        # 2. owner-computes scores per chunk, compacted per home; 3. all-to-all to the home ranks
        pending, recv = [], None
        for k, c in enumerate(lay["chunks"]):
            block, qidx, h = qx[k]
            h.wait()
            send = self._ws(f"s_send{k}", c["s_send"])
            self.kernels.score_compact(self, block, qidx[0], pos_g, neg_g, plan, k * Rk, Rk, send, st=st)
            out = self._ws("s_recv", c["s_recv"]) if k == lay["k_home"] else self._ws(f"s_none{k}", 0)
            if k == lay["k_home"]:
                recv = out
            pending.append(self.comm.all_to_all(out, send, c["s_out"], c["s_in"], async_op=True))
        for h in pending:
            h.wait()
        # 4. scatter to the home rows, reductions
        return self.kernels.shard_finish(self, plan, recv, pos_g, neg_g, temperature, adversarial, st=st)

    def collective_bytes(self, plan):
        """Bytes this rank receives per step through the forward's collectives (payload only)."""
        tot, qtot = plan.summary()
        W, me = self.world, self.rank
        q = int(sum(qtot[k, :, o].sum() for k in range(plan.chunks) for o in range(W) if o != me)) * self.entity_dim * 4
        s = sum(int(tot[me, o]) for o in range(W) if o != me) * 4
        return {"query_rows": q, "scores": s}

    def assemble_queries(self, pos_g, mode):
        """The query-entity rows of every global batch row: (qent [Bg, ent_dim] = E[pos[:, 2 if head
        else 0]], qent_pos [Bg, ent_dim] = E[pos[:, 0]]): owners' compacted rows, one all-to-all, then a
        local gather into batch-row order."""
        Bg = pos_g.shape[0]
        rows = torch.empty((2 if ops.mode_id(mode) == HEAD_BATCH else 1, Bg, self.entity_dim), dtype=torch.float32,
                           device=self.device)
        if not self.exchange:
            for i, c in enumerate(query_cols(ops.mode_id(mode), KGE_SHARD_TWO_COLUMNS)):
                self.kernels.gather_rows(self.shard, self.lo, pos_g[:, c:], 3, Bg, rows[i])
            return rows[0], rows[-1]
        plan = self.plan(pos_g, pos_g[:, :0], mode, chunks=1, flags=KGE_SHARD_TWO_COLUMNS)
        ((block, qidx, h),), qsend = self._exchange_queries(plan, pos_g)
        h.wait()
        del qsend
        for c in range(plan.ncol):
            self.kernels.gather_rows(block, 0, qidx[c], 1, Bg, rows[c])
        return rows[0], rows[-1]

    def train_step(self, pos_g, neg_g, weight_g, mode):
        """One row-sharded train step (supervisor.py:15-26 over the W replicas' batches, SUM gradient
        aggregation): pos_g [Bg, 3], neg_g [Bg, N], weight_g [Bg] — the global batch (home rank h's
        replica batch is rows [h Bg/W, (h+1) Bg/W)), identical on every rank. Updates this rank's
        shard and the relation table in place; returns this rank's replica loss (0-dim tensor).
        Collectives per step: one all-to-all of the compacted query rows, one all-gather of [Bg, 4] row
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
        qent, qent_pos = self.assemble_queries(pos_g, mode)
        k.train_forward(self, bufs, mode, qent, qent_pos, pos_g, neg_g, w)
        stats_all = self._gather_cat(bufs["stats"])
        k.train_combine(self, bufs, mode, qent, qent_pos, pos_g, neg_g, w, stats_all)
        if self.exchange:
            self.comm.all_reduce_sum_(bufs["dq"])
        loss = k.train_backward(self, bufs, mode, qent, qent_pos, pos_g, neg_g, w, self.step + 1, self.loss_sum)
        self.step += 1
        self.last_losses = loss  # every replica's loss [W] (identical on every rank)
        return loss[self.rank]

    def _gather_cat(self, t):
        return self.comm.all_gather_cat(t) if self.exchange else t.unsqueeze(0)

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
        C = self._gather_cat(need).cpu()  # C[q, o]: rows requester q needs from owner o
        send_ids = C[r].tolist()                   # my requests, grouped by owner (U is owner-ordered)
        recv_ids = C[:, r].tolist()                # requests addressed to me, per requester
        if W > 1:
            req = torch.empty(sum(recv_ids), dtype=torch.int64, device=U.device)
            self.comm.all_to_all(req, U, recv_ids, send_ids)
        else:
            req = U
        rows_out = torch.empty((req.numel(), self.entity_dim), dtype=torch.float32, device=dev)
        if req.numel():
            self.kernels.gather_rows(self.shard, self.lo, req.to(dev), 1, req.numel(), rows_out)
        cache = torch.zeros((U.numel() + 1, self.entity_dim), dtype=torch.float32, device=dev)  # + zero row
        if W > 1:
            self.comm.all_to_all(cache[:U.numel()].view(-1), rows_out.view(-1),
                                 [c * self.entity_dim for c in send_ids], [c * self.entity_dim for c in recv_ids])
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


def warn_dense_fallback(model, world, reason):
    """One-time warning: a multi-replica Trainer that cannot use the row-sharded fused step all-reduces
    the dense table gradients every step (supervisor.py:26 under tf.distribute)."""
    nbytes = sum(p.numel() * p.element_size() for p in model.parameters() if p.requires_grad)
    warnings.warn(f"Trainer at {world} replicas falls back to the dense-gradient path ({reason}): every step "
                  f"all-reduces {nbytes / 1e6:.1f} MB of table gradients (the row-sharded fused step moves "
                  f"O(batch) bytes instead)", RuntimeWarning, stacklevel=3)
