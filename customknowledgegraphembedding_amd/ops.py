"""Tensor-level wrappers around libkge_hip.so with autograd.

Every function here runs the hand-written HIP kernels; there is no eager-PyTorch or CPU fallback.
Tensors must be fp32 (tables/scores) / int64 (indices) on a ROCm device; the launch goes on
torch's current stream, so these ops compose with the rest of a torch program and with
torch.cuda graphs.

Reference correspondence (file:line in /root/reference):
  score_indexed      -> TFKGEModel.single_mode/head_batch_mode/tail_batch_mode gathers + model_func
                        (tensorflow_codes/model.py:127-144,148-166,174-192); upstream KGEModel.forward
  score_dense        -> model_func[name](head, relation, tail, mode) (model.py:109-112,207-235)
  neg_reduce         -> sum(softmax(s*1) * log_sigmoid(-s)) (model.py:168-171,195-198, Q3) and the
                        upstream adversarial / mean reduction in train_step
  log_sigmoid        -> tf.math.log_sigmoid (model.py:145)
"""
from __future__ import annotations

import torch

from . import _lib
from ._lib import FN_IDS, HEAD_BATCH, SINGLE, TAIL_BATCH, check


def ctypes_ptr(t):
    return None if t is None else t.data_ptr()


def _stream(device) -> int:
    return torch.cuda.current_stream(device).cuda_stream


def _need_gpu(*ts):
    for t in ts:
        if t is not None and t.device.type != "cuda":
            raise _lib.KGEHipError(
                f"libkge_hip.so runs on ROCm devices only; got a tensor on {t.device} "
                "(there is no CPU fallback)")


def _fp32(t, name):
    if t.dtype != torch.float32:
        raise TypeError(f"{name} must be float32, got {t.dtype}")
    if t.dim() < 1 or t.stride(-1) != 1:
        raise ValueError(f"{name} must be row-contiguous (stride(-1) == 1)")


def _i64(t, name):
    if t.dtype != torch.int64:
        raise TypeError(f"{name} must be int64, got {t.dtype}")


def fn_id(name: str) -> int:
    try:
        return FN_IDS[name]
    except KeyError:
        raise ValueError(f"model {name} not supported (have {sorted(FN_IDS)})") from None


def mode_id(mode) -> int:
    """Accept the TF integer codes (Q1: 0 head-batch, 3 single, anything else tail-batch) and the
    upstream strings."""
    if isinstance(mode, str):
        m = {"head-batch": HEAD_BATCH, "tail-batch": TAIL_BATCH, "single": SINGLE}.get(mode)
        if m is None:
            raise ValueError(f"mode {mode} not supported")
        return m
    mode = int(mode)
    if mode == 0:
        return HEAD_BATCH
    if mode == 3:
        return SINGLE
    return TAIL_BATCH  # model.py:124 — every non-zero negative mode falls into tail-batch


# ----------------------------------------------------------------------------------------------
# raw launches (no autograd)
# ----------------------------------------------------------------------------------------------
def _forms_ptr(forms):
    """A kge_forms for the _ex entry points (None: the library's choice) -> (ctypes pointer, keep-alive)."""
    import ctypes
    if forms is None:
        return None, None
    if isinstance(forms, dict):
        forms = _lib.forms(**forms)
    return ctypes.addressof(forms), forms


def score_indexed_raw(fn, mode, ent, rel, rel_off, pos, neg, D, gamma, emb_range, modulus=0.0,
                      out=None, forms=None):
    _need_gpu(ent, rel, pos, neg)
    _fp32(ent, "entity_embedding")
    _fp32(rel, "relation_embedding")
    _i64(pos, "positive_sample")
    if pos.dim() != 2 or pos.shape[1] != 3 or not pos.is_contiguous():
        raise ValueError("positive_sample must be a contiguous [B, 3] int64 tensor")
    B = pos.shape[0]
    if mode == SINGLE:
        N, neg_ld, neg_p = 1, 0, None
    else:
        _i64(neg, "negative_sample")
        if neg.dim() != 2 or neg.shape[0] != B or neg.stride(1) != 1:
            raise ValueError("negative_sample must be a row-contiguous [B, N] int64 tensor")
        N, neg_ld, neg_p = neg.shape[1], neg.stride(0), neg.data_ptr()
    if out is None:
        out = torch.empty((B, N), dtype=torch.float32, device=ent.device)
    fp, _keep = _forms_ptr(forms)
    rc = _lib.load().kge_score_indexed_ex(
        fn, mode, ent.data_ptr(), ent.shape[0], ent.stride(0), rel.data_ptr(), rel.shape[0],
        rel.stride(0), rel_off, pos.data_ptr(), neg_p, neg_ld, B, N, D, float(gamma),
        float(emb_range), float(modulus), out.data_ptr(), out.stride(0), fp, _stream(ent.device))
    check(rc, "kge_score_indexed")
    return out


def score_indexed_bwd_raw(fn, mode, ent, rel, rel_off, pos, neg, D, gamma, emb_range, modulus,
                          d_scores, d_ent, d_rel, d_modulus=None):
    B = pos.shape[0]
    if mode == SINGLE:
        N, neg_ld, neg_p = 1, 0, None
    else:
        N, neg_ld, neg_p = neg.shape[1], neg.stride(0), neg.data_ptr()
    d_scores = d_scores.contiguous()
    rc = _lib.load().kge_score_indexed_bwd(
        fn, mode, ent.data_ptr(), ent.shape[0], ent.stride(0), rel.data_ptr(), rel.shape[0],
        rel.stride(0), rel_off, pos.data_ptr(), neg_p, neg_ld, B, N, D, float(gamma),
        float(emb_range), float(modulus), d_scores.data_ptr(), d_scores.stride(0),
        d_ent.data_ptr(), d_rel.data_ptr(), ctypes_ptr(d_modulus), None, _stream(ent.device))
    check(rc, "kge_score_indexed_bwd")


def step_forward_raw(fn, mode, ent, rel, rel_off, pos, neg, D, gamma, emb_range, modulus=0.0,
                     temperature=1.0, adversarial=True, neg_scores=None, cand_stats=None, forms=None):
    """Both model calls of supervisor.py:17-18 in one launch -> (out_neg [B], out_pos [B],
    neg_scores [B, N], pos_scores [B]). `cand_stats` ([B*N, 2] fp32, optional) receives InterHT's
    per-candidate inverse half-norms for the streaming backward."""
    _need_gpu(ent, rel, pos, neg)
    _fp32(ent, "entity_embedding")
    _fp32(rel, "relation_embedding")
    _i64(pos, "positive_sample")
    _i64(neg, "negative_sample")
    if mode not in (HEAD_BATCH, TAIL_BATCH):
        raise ValueError("step_forward needs a negative mode (0 head-batch or 1 tail-batch)")
    if pos.dim() != 2 or pos.shape[1] != 3 or not pos.is_contiguous():
        raise ValueError("positive_sample must be a contiguous [B, 3] int64 tensor")
    B, N = neg.shape
    if neg.stride(1) != 1 or B != pos.shape[0]:
        raise ValueError("negative_sample must be a row-contiguous [B, N] int64 tensor")
    dev = ent.device
    if neg_scores is None:
        neg_scores = torch.empty((B, N), dtype=torch.float32, device=dev)
    out_neg = torch.empty((B,), dtype=torch.float32, device=dev)
    out_pos = torch.empty((B,), dtype=torch.float32, device=dev)
    pos_scores = torch.empty((B,), dtype=torch.float32, device=dev)
    fp, _keep = _forms_ptr(forms)
    rc = _lib.load().kge_step_forward_ex(
        fn, mode, ent.data_ptr(), ent.shape[0], ent.stride(0), rel.data_ptr(), rel.shape[0],
        rel.stride(0), rel_off, pos.data_ptr(), neg.data_ptr(), neg.stride(0), B, N, D,
        float(gamma), float(emb_range), float(modulus), float(temperature), int(bool(adversarial)),
        neg_scores.data_ptr(), neg_scores.stride(0), out_neg.data_ptr(), pos_scores.data_ptr(),
        out_pos.data_ptr(), None if cand_stats is None else cand_stats.data_ptr(), fp, _stream(dev))
    check(rc, "kge_step_forward")
    return out_neg, out_pos, neg_scores, pos_scores


class StepPlanner:
    """step_forward_raw with the tile scorer's id-only setup made one step AHEAD (kge_step_planner_*: the handle
    form of kge_step_plan / kge_step_forward_planned): a step loop that knows its next batch (run.py's prefetching
    input pipeline, run.py:40-66) hands it to the current step, whose launch's tail blocks plan it, so the next
    step's blocks start on their sorted candidates at once. Outputs are bitwise step_forward_raw's.

        sp = StepPlanner(fn, ent, rel, rel_off, D, B, N, gamma, emb_range)
        sp.plan(pos0, neg0, mode0)                    # the first batch's plan: one launch
        out = sp.step(nxt=(pos1, neg1, mode1))        # batch 0's step + batch 1's plan
        out = sp.step(nxt=(pos2, neg2, mode2))        # batch 1's step + ...

    A plan is a snapshot of its batch's ids (the planned step reads no id but the plan's). The planner keeps
    the tensors of the batch being planned until the step that consumes the plan, and two plan buffers
    (the step reads one while its tail blocks write the other). The tables may change between steps (they are
    read at step time); the launch stream is torch's current stream when the planner is made. `available(...)`
    is False when the tile form does not apply (use step_forward_raw). A step costs the host one 9-argument
    C call: the tables, shapes and buffers live in the library's handle."""

    def __init__(self, fn, ent, rel, rel_off, D, B, N, gamma, emb_range, modulus=0.0, temperature=1.0,
                 adversarial=True):
        import ctypes
        _need_gpu(ent, rel)
        _fp32(ent, "entity_embedding")
        _fp32(rel, "relation_embedding")
        self.fn, self.ent, self.rel, self.rel_off, self.D = fn, ent, rel, rel_off, D
        self.B, self.N = B, N
        lib = _lib.load()
        nbytes = self.plan_size(fn, ent, rel, rel_off, D, B, N)
        if nbytes <= 0:
            raise _lib.KGEHipError("kge_step_plan_size is 0: the tile form does not apply to this shape "
                                   "(use step_forward_raw)")
        self._bufs = [torch.empty(nbytes, dtype=torch.uint8, device=ent.device) for _ in range(2)]
        h = ctypes.c_void_p()
        check(lib.kge_step_planner_create(
            ctypes.addressof(h), fn, ent.data_ptr(), ent.shape[0], ent.stride(0), rel.data_ptr(), rel.shape[0],
            rel.stride(0), rel_off, B, N, D, float(gamma), float(emb_range), float(modulus), float(temperature),
            int(bool(adversarial)), self._bufs[0].data_ptr(), self._bufs[1].data_ptr(), nbytes,
            _stream(ent.device)), "kge_step_planner_create")
        self._h = h.value
        self._lib = lib
        self._step_fn = lib.kge_step_planner_step
        self._planned = False
        self._held = None      # the tensors the waiting plan was made from (kept alive until its step)
        self._pshape, self._nshape = (B, 3), (B, N)
        self._out_ok = None

    @staticmethod
    def plan_size(fn, ent, rel, rel_off, D, B, N):
        return int(_lib.load().kge_step_plan_size(fn, ent.shape[0], ent.stride(0), rel.shape[0], rel.stride(0),
                                                  rel_off, B, N, D))

    @classmethod
    def available(cls, fn, ent, rel, rel_off, D, B, N):
        return cls.plan_size(fn, ent, rel, rel_off, D, B, N) > 0

    def _check_batch(self, pos, neg, mode):
        if mode not in (HEAD_BATCH, TAIL_BATCH):
            raise ValueError("a planned step needs a negative mode (0 head-batch or 1 tail-batch)")
        if pos.shape != self._pshape or neg.shape != self._nshape:
            raise ValueError(f"a planned batch must be pos [{self.B}, 3] and neg [{self.B}, {self.N}]")
        if pos.dtype != torch.int64 or neg.dtype != torch.int64 or pos.device != self.ent.device or \
                neg.device != self.ent.device:
            raise TypeError("a planned batch must be int64 tensors on the tables' device")
        if pos.stride() != (3, 1) or neg.stride(1) != 1:
            raise ValueError("pos must be contiguous and neg row-contiguous")

    def set_sweep(self, alternate):
        """1: the tile sweep's direction alternates step by step (kge_step_planner_set_sweep); 0: ascending."""
        check(self._lib.kge_step_planner_set_sweep(self._h, int(alternate)), "kge_step_planner_set_sweep")

    def set_modulus(self, modulus):
        check(self._lib.kge_step_planner_set_modulus(self._h, float(modulus)), "kge_step_planner_set_modulus")

    def plan(self, pos, neg, mode):
        """The plan of the batch the next step() scores (a run's first batch; later ones come from step)."""
        self._check_batch(pos, neg, mode)
        check(self._lib.kge_step_planner_plan(self._h, pos.data_ptr(), neg.data_ptr(), neg.stride(0), mode),
              "kge_step_planner_plan")
        self._planned, self._held = True, (pos, neg)

    def outputs(self):
        """A set of output tensors for step(out=...): (out_neg [B], out_pos [B], neg_scores [B, N], pos_scores [B])."""
        dev = self.ent.device
        return (torch.empty((self.B,), dtype=torch.float32, device=dev),
                torch.empty((self.B,), dtype=torch.float32, device=dev),
                torch.empty((self.B, self.N), dtype=torch.float32, device=dev),
                torch.empty((self.B,), dtype=torch.float32, device=dev))

    def _check_outputs(self, out):
        """the planner writes neg_scores with row stride N and the three row outputs densely, fp32, on
        the tables' device; anything else would be written silently wrong."""
        if not isinstance(out, (tuple, list)) or len(out) != 4:
            raise ValueError("StepPlanner.step: out must be (out_neg, out_pos, neg_scores, pos_scores)")
        shapes = ((self.B,), (self.B,), (self.B, self.N), (self.B,))
        strides = ((1,), (1,), (self.N, 1), (1,))
        for t, shp, std, nm in zip(out, shapes, strides, ("out_neg", "out_pos", "neg_scores", "pos_scores")):
            if not isinstance(t, torch.Tensor) or t.dtype != torch.float32 or t.device != self.ent.device:
                raise TypeError(f"StepPlanner.step: {nm} must be a float32 tensor on {self.ent.device}")
            if tuple(t.shape) != shp or (t.numel() > 1 and tuple(t.stride()) != std):
                raise ValueError(f"StepPlanner.step: {nm} must have shape {shp} and strides {std}")

    def step(self, nxt=None, out=None):
        """Both model calls on the planned batch -> (out_neg [B], out_pos [B], neg_scores [B, N],
        pos_scores [B]); with nxt = (pos, neg, mode) the same launch plans that batch for the next step.
        `out`: outputs to write (from outputs(); neg_scores contiguous), else fresh tensors."""
        if not self._planned:
            raise RuntimeError("StepPlanner.step: no batch planned (call plan() first, or pass nxt to step)")
        if out is not None and out is not self._out_ok:
            self._check_outputs(out)
            self._out_ok = out  # a caller reusing one set of outputs pays the check once
        out_neg, out_pos, neg_scores, pos_scores = out if out is not None else self.outputs()
        if nxt is None:
            rc = self._step_fn(self._h, None, None, 0, 0, neg_scores.data_ptr(), out_neg.data_ptr(),
                               pos_scores.data_ptr(), out_pos.data_ptr())
        else:
            npos, nneg, nmode = nxt
            self._check_batch(npos, nneg, nmode)
            rc = self._step_fn(self._h, npos.data_ptr(), nneg.data_ptr(), nneg.stride(0), nmode,
                               neg_scores.data_ptr(), out_neg.data_ptr(), pos_scores.data_ptr(), out_pos.data_ptr())
        check(rc, "kge_step_planner_step")
        if nxt is None:
            self._planned, self._held = False, None
        else:
            self._held = (nxt[0], nxt[1])
        return out_neg, out_pos, neg_scores, pos_scores

    def __del__(self):
        h = getattr(self, "_h", None)
        if h:
            try:
                self._lib.kge_step_planner_destroy(h)
            except Exception:  # noqa: BLE001 (interpreter teardown)
                pass
            self._h = None


def step_finish_raw(fn, ent, rel, rel_off, pos, D, gamma, emb_range, neg_scores, modulus=0.0,
                    temperature=1.0, adversarial=True):
    """Second launch of step_forward_raw: positives + per-row reductions of `neg_scores`."""
    B, N = neg_scores.shape
    dev = ent.device
    out_neg = torch.empty((B,), dtype=torch.float32, device=dev)
    out_pos = torch.empty((B,), dtype=torch.float32, device=dev)
    pos_scores = torch.empty((B,), dtype=torch.float32, device=dev)
    rc = _lib.load().kge_step_finish(
        fn, ent.data_ptr(), ent.shape[0], ent.stride(0), rel.data_ptr(), rel.shape[0], rel.stride(0),
        rel_off, pos.data_ptr(), B, D, float(gamma), float(emb_range), float(modulus),
        neg_scores.data_ptr(), N, neg_scores.stride(0), float(temperature), int(bool(adversarial)),
        out_neg.data_ptr(), pos_scores.data_ptr(), out_pos.data_ptr(), _stream(dev))
    check(rc, "kge_step_finish")
    return out_neg, out_pos, pos_scores


def _dense_shapes(mode, head, relation, tail):
    B = head.shape[0]
    if mode == HEAD_BATCH:
        N = head.shape[1]
    elif mode == TAIL_BATCH:
        N = tail.shape[1]
    else:
        N = 1
    return B, N


def _rows(t):
    """[B, n, w] (or [B, w]) tensor whose rows are contiguous -> (tensor, row stride)."""
    if t.dim() == 2:
        t = t.unsqueeze(1)
    if t.stride(-1) != 1 or (t.shape[1] > 1 and t.stride(0) != t.shape[1] * t.stride(1)):
        t = t.contiguous()
    ld = t.stride(1) if t.shape[1] > 1 else t.stride(0)
    return t, ld


def score_dense_raw(fn, mode, head, relation, tail, rel_off, D, gamma, emb_range, modulus=0.0):
    _need_gpu(head, relation, tail)
    for t, n in ((head, "head"), (relation, "relation"), (tail, "tail")):
        _fp32(t, n)
    B, N = _dense_shapes(mode, head, relation, tail)
    head, hld = _rows(head)
    tail, tld = _rows(tail)
    relation, rld = _rows(relation)
    out = torch.empty((B, N), dtype=torch.float32, device=head.device)
    rc = _lib.load().kge_score_dense(
        fn, mode, head.data_ptr(), hld, relation.data_ptr(), rld, rel_off, tail.data_ptr(), tld,
        B, N, D, float(gamma), float(emb_range), float(modulus), out.data_ptr(), out.stride(0),
        _stream(head.device))
    check(rc, "kge_score_dense")
    return out


def neg_reduce_raw(scores, temperature=1.0, adversarial=True):
    _need_gpu(scores)
    _fp32(scores, "scores")
    B, N = scores.shape
    out = torch.empty((B,), dtype=torch.float32, device=scores.device)
    rc = _lib.load().kge_neg_reduce(scores.data_ptr(), B, N, scores.stride(0), float(temperature),
                                    int(bool(adversarial)), out.data_ptr(), _stream(scores.device))
    check(rc, "kge_neg_reduce")
    return out


def log_sigmoid_raw(x):
    _need_gpu(x)
    x = x.contiguous()
    out = torch.empty_like(x)
    rc = _lib.load().kge_log_sigmoid(x.data_ptr(), x.numel(), out.data_ptr(), _stream(x.device))
    check(rc, "kge_log_sigmoid")
    return out



def transparse_premul(W, mask):
    """M = mask * W (kge_transparse_premul)."""
    M = torch.empty_like(W)
    check(_lib.load().kge_transparse_premul(W.data_ptr(), mask.data_ptr(), W.numel(), M.data_ptr(),
                                            _stream(W.device)), "kge_transparse_premul")
    return M


def _want_premul(W, pos, neg, mode):
    """Premultiply the relation matrices when there are fewer of them than row blocks: one pass over
    R*d*d floats then saves every block the mask reads."""
    if W.numel() % 4 or W.data_ptr() % 16:
        return False
    rows = pos.shape[0] * (neg.shape[1] if (mode_id(mode) == HEAD_BATCH and neg is not None) else 1)
    return W.shape[0] * 4 <= max(1, rows // 128)


_WS_CACHE = {}


def _workspace(device, nbytes):
    """A scratch buffer of at least nbytes on `device`, reused across calls on torch's current stream (the
    library's workspaces carry nothing between calls)."""
    if nbytes <= 0:
        return None
    key = (str(device), torch.cuda.current_stream(device).cuda_stream)
    ws = _WS_CACHE.get(key)
    if ws is None or ws.numel() < nbytes:
        ws = torch.empty(nbytes, dtype=torch.uint8, device=device)
        _WS_CACHE[key] = ws
    return ws


def transparse_score_raw(mode, ent, rel, W, mask, pos, neg, gamma, stats=None, out=None, M=None, forms=None,
                         split=True):
    """TranSparse raw scores (model.py:226-235): [B, N] for head-batch, [B, 1] for single and
    tail-batch (Q9). `stats` (optional [rows, 2] fp32) receives the per-row backward statistics.
    `M` (optional) = transparse_premul(W, mask), used instead of forming mask * W in the loads.
    `split` (single / tail-batch): the projection split over the columns through a workspace
    (kge_transparse_score_ex), else one block per relation's row chunk."""
    _need_gpu(ent, rel, W, mask, pos, neg)
    for t, n in ((ent, "ent"), (rel, "rel"), (W, "W"), (mask, "mask")):
        _fp32(t, n)
    _i64(pos, "pos")
    if not (W.is_contiguous() and mask.is_contiguous()):
        raise ValueError("W and mask must be contiguous [R, d, d]")
    m = mode_id(mode)
    B, d = pos.shape[0], ent.shape[1]
    if rel.shape[1] != d or tuple(W.shape) != (rel.shape[0], d, d) or W.shape != mask.shape:
        raise ValueError("TranSparse needs entity_dim == relation_dim == d and W, mask [R, d, d]")
    if pos.stride(1) != 1 or pos.stride(0) != 3:
        pos = pos.contiguous()
    head = m == HEAD_BATCH
    N = neg.shape[1] if head else 1
    if head:
        _i64(neg, "neg")
        if neg.stride(1) != 1:
            neg = neg.contiguous()
    if out is None:
        out = torch.empty((B, N), dtype=torch.float32, device=ent.device)
    lib = _lib.load()
    nbytes = int(lib.kge_transparse_score_workspace_size(m, rel.shape[0], B, d)) if split else 0
    ws = _workspace(ent.device, nbytes)
    fp, _keep = _forms_ptr(forms)
    Wp, maskp = (M.data_ptr(), None) if M is not None else (W.data_ptr(), mask.data_ptr())
    rc = lib.kge_transparse_score_ex(
        m, ent.data_ptr(), ent.shape[0], ent.stride(0), rel.data_ptr(), rel.shape[0], rel.stride(0), Wp, maskp,
        pos.data_ptr(), neg.data_ptr() if head else None, neg.stride(0) if head else 0, B, N, d, float(gamma),
        out.data_ptr(), out.stride(0), None if stats is None else stats.data_ptr(), fp,
        None if ws is None else ws.data_ptr(), nbytes, _stream(ent.device))
    check(rc, "kge_transparse_score")
    return out


def transparse_step_forward_raw(mode, ent, rel, W, mask, pos, neg, gamma, temperature=1.0, adversarial=True, M=None):
    """Both calls of supervisor.py:17-18 for TranSparse (kge_transparse_step_forward): returns (neg_scores,
    out_neg [B], pos_scores [B], out_pos [B]); neg_scores is [B, N] for head-batch, [B, 1] for tail-batch (Q9).
    Bitwise transparse_score_raw + neg_reduce_raw / log_sigmoid_raw. No autograd (see TFKGEModel.step_forward)."""
    _need_gpu(ent, rel, W, mask, pos, neg)
    for t, n in ((ent, "ent"), (rel, "rel"), (W, "W"), (mask, "mask")):
        _fp32(t, n)
    _i64(pos, "pos")
    m = mode_id(mode)
    if m not in (HEAD_BATCH, TAIL_BATCH):
        raise ValueError("transparse_step_forward needs the batch's negative mode (0 or 1)")
    if not (W.is_contiguous() and mask.is_contiguous()):
        raise ValueError("W and mask must be contiguous [R, d, d]")
    B, d = pos.shape[0], ent.shape[1]
    if rel.shape[1] != d or tuple(W.shape) != (rel.shape[0], d, d) or W.shape != mask.shape:
        raise ValueError("TranSparse needs entity_dim == relation_dim == d and W, mask [R, d, d]")
    if pos.stride(1) != 1 or pos.stride(0) != 3:
        pos = pos.contiguous()
    _i64(neg, "neg")
    if neg.stride(1) != 1:
        neg = neg.contiguous()
    N = neg.shape[1] if m == HEAD_BATCH else 1
    dev = ent.device
    ns = torch.empty((B, N), dtype=torch.float32, device=dev)
    out_neg = torch.empty((B,), dtype=torch.float32, device=dev)
    ps = torch.empty((B,), dtype=torch.float32, device=dev)
    out_pos = torch.empty((B,), dtype=torch.float32, device=dev)
    lib = _lib.load()
    nbytes = int(lib.kge_transparse_step_workspace_size(rel.shape[0], B, d))
    ws = _workspace(dev, nbytes)
    Wp, maskp = (M.data_ptr(), None) if M is not None else (W.data_ptr(), mask.data_ptr())
    rc = lib.kge_transparse_step_forward(
        m, ent.data_ptr(), ent.shape[0], ent.stride(0), rel.data_ptr(), rel.shape[0], rel.stride(0), Wp, maskp,
        pos.data_ptr(), neg.data_ptr(), neg.stride(0), B, neg.shape[1], d, float(gamma), float(temperature),
        int(bool(adversarial)), ns.data_ptr(), ns.stride(0), out_neg.data_ptr(), ps.data_ptr(), out_pos.data_ptr(),
        None if ws is None else ws.data_ptr(), nbytes, _stream(dev))
    check(rc, "kge_transparse_step_forward")
    return ns, out_neg, ps, out_pos


def transparse_score_bwd_raw(mode, ent, rel, W, mask, pos, neg, stats, d_scores, d_ent, d_rel, d_W, M=None):
    """Accumulates the TranSparse gradients into d_ent, d_rel, d_W (deterministic)."""
    m = mode_id(mode)
    B, d = pos.shape[0], ent.shape[1]
    head = m == HEAD_BATCH
    N = neg.shape[1] if head else 1
    d_scores = d_scores.contiguous() if d_scores.stride(-1) != 1 else d_scores
    lib = _lib.load()
    nbytes = lib.kge_transparse_bwd_workspace_size(m, ent.shape[0], rel.shape[0], B, N, d)
    ws = torch.empty(max(int(nbytes), 1), dtype=torch.uint8, device=ent.device)
    rc = lib.kge_transparse_score_bwd(
        m, ent.data_ptr(), ent.shape[0], ent.stride(0), rel.data_ptr(), rel.shape[0], rel.stride(0), W.data_ptr(),
        mask.data_ptr(), None if M is None else M.data_ptr(), pos.data_ptr(), neg.data_ptr() if head else None,
        neg.stride(0) if head else 0, B, N, d, stats.data_ptr(), d_scores.data_ptr(), d_scores.stride(0), d_ent.data_ptr(), d_rel.data_ptr(),
        d_W.data_ptr(), ws.data_ptr(), ws.numel(), _stream(ent.device))
    check(rc, "kge_transparse_score_bwd")

# ----------------------------------------------------------------------------------------------
# autograd
# ----------------------------------------------------------------------------------------------
class _ScoreIndexed(torch.autograd.Function):
    @staticmethod
    def forward(ctx, ent, rel, modulus_t, pos, neg, fn, mode, rel_off, D, gamma, emb_range):
        modulus = float(modulus_t.item()) if (fn == FN_IDS["pRotatE"]) else 0.0
        out = score_indexed_raw(fn, mode, ent, rel, rel_off, pos, neg, D, gamma, emb_range, modulus)
        ctx.save_for_backward(ent, rel, pos, neg if neg is not None else pos)
        ctx.cfg = (fn, mode, rel_off, D, gamma, emb_range, modulus, neg is not None,
                   None if modulus_t is None else modulus_t.shape)
        return out

    @staticmethod
    def backward(ctx, d_scores):
        ent, rel, pos, neg = ctx.saved_tensors
        fn, mode, rel_off, D, gamma, emb_range, modulus, has_neg, mod_shape = ctx.cfg
        has_mod = mod_shape is not None
        d_ent = torch.zeros_like(ent)
        d_rel = torch.zeros_like(rel)
        d_mod = torch.zeros(1, dtype=torch.float32, device=ent.device) if has_mod else None
        score_indexed_bwd_raw(fn, mode, ent, rel, rel_off, pos, neg if has_neg else None, D, gamma,
                              emb_range, modulus, d_scores, d_ent, d_rel, d_mod)
        if has_mod:
            d_mod = d_mod.view(mod_shape)
        return d_ent, d_rel, d_mod, None, None, None, None, None, None, None, None


class _ScoreDense(torch.autograd.Function):
    @staticmethod
    def forward(ctx, head, relation, tail, fn, mode, rel_off, D, gamma, emb_range, modulus):
        out = score_dense_raw(fn, mode, head, relation, tail, rel_off, D, gamma, emb_range, modulus)
        ctx.save_for_backward(head, relation, tail)
        ctx.cfg = (fn, mode, rel_off, D, gamma, emb_range, modulus)
        return out

    @staticmethod
    def backward(ctx, d_scores):
        head, relation, tail = ctx.saved_tensors
        fn, mode, rel_off, D, gamma, emb_range, modulus = ctx.cfg
        B, N = _dense_shapes(mode, head, relation, tail)
        h, hld = _rows(head)
        t, tld = _rows(tail)
        r, rld = _rows(relation)
        dh = torch.zeros_like(h)
        dt = torch.zeros_like(t)
        dr = torch.zeros_like(r)
        d_scores = d_scores.contiguous()
        rc = _lib.load().kge_score_dense_bwd(
            fn, mode, h.data_ptr(), hld, r.data_ptr(), rld, rel_off, t.data_ptr(), tld, B, N, D,
            float(gamma), float(emb_range), float(modulus), d_scores.data_ptr(), d_scores.stride(0),
            dh.data_ptr(), dr.data_ptr(), dt.data_ptr(), None, _stream(h.device))
        check(rc, "kge_score_dense_bwd")
        return (dh.view(head.shape), dr.view(relation.shape), dt.view(tail.shape),
                None, None, None, None, None, None, None)


class _NegReduce(torch.autograd.Function):
    @staticmethod
    def forward(ctx, scores, temperature, adversarial, detach):
        scores = scores.contiguous()
        out = neg_reduce_raw(scores, temperature, adversarial)
        ctx.save_for_backward(scores)
        ctx.cfg = (temperature, adversarial, detach)
        return out

    @staticmethod
    def backward(ctx, d_out):
        (scores,) = ctx.saved_tensors
        temperature, adversarial, detach = ctx.cfg
        B, N = scores.shape
        d_out = d_out.contiguous()
        d_s = torch.empty_like(scores)
        rc = _lib.load().kge_neg_reduce_bwd(
            scores.data_ptr(), B, N, scores.stride(0), float(temperature), int(bool(adversarial)),
            int(bool(detach)), d_out.data_ptr(), d_s.data_ptr(), d_s.stride(0),
            _stream(scores.device))
        check(rc, "kge_neg_reduce_bwd")
        return d_s, None, None, None


class _LogSigmoid(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        out = log_sigmoid_raw(x)
        ctx.save_for_backward(x)
        return out

    @staticmethod
    def backward(ctx, d_out):
        (x,) = ctx.saved_tensors
        x = x.contiguous()
        d_out = d_out.contiguous()
        d_x = torch.empty_like(x)
        rc = _lib.load().kge_log_sigmoid_bwd(x.data_ptr(), d_out.data_ptr(), x.numel(),
                                             d_x.data_ptr(), _stream(x.device))
        check(rc, "kge_log_sigmoid_bwd")
        return d_x


class _StepForward(torch.autograd.Function):
    """Differentiable fused forward of supervisor.py:17-18 (GradientTape through both calls)."""

    @staticmethod
    def forward(ctx, ent, rel, modulus_t, pos, neg, fn, mode, rel_off, D, gamma, emb_range,
                temperature, adversarial, detach):
        modulus = float(modulus_t.item()) if (fn == FN_IDS["pRotatE"]) else 0.0
        stats = (torch.empty((neg.shape[0] * neg.shape[1], 2), dtype=torch.float32, device=ent.device)
                 if fn == FN_IDS["InterHT"] else None)
        out_neg, out_pos, ns, ps = step_forward_raw(fn, mode, ent, rel, rel_off, pos, neg, D, gamma,
                                                    emb_range, modulus, temperature, adversarial, cand_stats=stats)
        ctx.save_for_backward(ent, rel, pos, neg, ns, ps, stats if stats is not None else ps)
        ctx.has_stats = stats is not None
        ctx.cfg = (fn, mode, rel_off, D, gamma, emb_range, modulus, temperature, adversarial, detach,
                   None if modulus_t is None else modulus_t.shape)
        return out_neg, out_pos

    @staticmethod
    def backward(ctx, d_neg, d_pos):
        """kge_step_backward: deterministic two-phase backward (no float atomics); it overwrites
        every row of the gradient tables, so they are allocated uninitialised."""
        ent, rel, pos, neg, ns, ps, stats = ctx.saved_tensors
        stats = stats if ctx.has_stats else None
        (fn, mode, rel_off, D, gamma, emb_range, modulus, temperature, adversarial, detach,
         mod_shape) = ctx.cfg
        lib = _lib.load()
        B, N = ns.shape
        dev = ent.device
        d_neg = torch.zeros(B, device=dev) if d_neg is None else d_neg.contiguous()
        d_pos = torch.zeros(B, device=dev) if d_pos is None else d_pos.contiguous()
        d_ent = torch.empty_like(ent)
        d_rel = torch.empty_like(rel)
        d_mod = torch.empty(1, dtype=torch.float32, device=dev) if mod_shape is not None else None
        nbytes = lib.kge_step_backward_workspace_size(fn, ent.shape[0], B, N, D)
        ws = torch.empty(max(nbytes, 1), dtype=torch.uint8, device=dev)
        rc = lib.kge_step_backward(
            fn, mode, ent.data_ptr(), ent.shape[0], ent.stride(0), rel.data_ptr(), rel.shape[0], rel.stride(0),
            rel_off, pos.data_ptr(), neg.data_ptr(), neg.stride(0), B, N, D, float(gamma), float(emb_range),
            float(modulus), float(temperature), int(bool(adversarial)), int(bool(detach)), ns.data_ptr(),
            ns.stride(0), ps.data_ptr(), d_neg.data_ptr(), d_pos.data_ptr(), d_ent.data_ptr(), d_rel.data_ptr(),
            ctypes_ptr(d_mod), ctypes_ptr(stats), ws.data_ptr(), ws.numel(), _stream(dev))
        check(rc, "kge_step_backward")
        if d_mod is not None:
            d_mod = d_mod.view(mod_shape)
        return (d_ent, d_rel, d_mod) + (None,) * 11


class _TranSparse(torch.autograd.Function):
    @staticmethod
    def forward(ctx, ent, rel, W, mask, pos, neg, mode, gamma):
        m = mode_id(mode)
        pos = pos.contiguous()
        neg = neg.contiguous() if (m == HEAD_BATCH) else None
        rows = pos.shape[0] * (neg.shape[1] if neg is not None else 1)
        stats = torch.empty((rows, 2), dtype=torch.float32, device=ent.device)
        M = transparse_premul(W, mask) if _want_premul(W, pos, neg, m) else None
        out = transparse_score_raw(m, ent, rel, W, mask, pos, neg, gamma, stats=stats, M=M)
        ctx.save_for_backward(ent, rel, W, mask, pos, neg if neg is not None else pos, stats,
                              M if M is not None else stats)
        ctx.cfg = (m, neg is not None, M is not None)
        return out

    @staticmethod
    def backward(ctx, d_scores):
        ent, rel, W, mask, pos, neg, stats, M = ctx.saved_tensors
        m, has_neg, has_m = ctx.cfg
        d_ent, d_rel, d_W = torch.zeros_like(ent), torch.zeros_like(rel), torch.zeros_like(W)
        transparse_score_bwd_raw(m, ent, rel, W, mask, pos, neg if has_neg else None, stats, d_scores, d_ent, d_rel,
                                 d_W, M=M if has_m else None)
        return d_ent, d_rel, d_W, None, None, None, None, None


def transparse_score(mode, ent, rel, W, mask, pos, neg, gamma):
    """TranSparse gather + score (model.py:139-142,161-164,187-190,226-235), differentiable w.r.t.
    ent, rel and W -> [B, N] (head-batch) or [B, 1] (single / tail-batch)."""
    return _TranSparse.apply(ent, rel, W, mask, pos, neg, mode, float(gamma))


def step_loss_raw(out_neg, out_pos, weight, want_grad=True):
    """supervisor.py:19-23 in one HIP launch -> (loss 0-dim, d_out [B] or None)."""
    _need_gpu(out_neg, out_pos, weight)
    B = out_neg.numel()
    n, p_, w = (t.reshape(-1).contiguous().to(torch.float32) for t in (out_neg, out_pos, weight))
    loss = torch.empty((), dtype=torch.float32, device=n.device)
    d_out = torch.empty(B, dtype=torch.float32, device=n.device) if want_grad else None
    check(_lib.load().kge_step_loss(n.data_ptr(), p_.data_ptr(), w.data_ptr(), B, loss.data_ptr(), ctypes_ptr(d_out),
                                    _stream(n.device)), "kge_step_loss")
    return loss, d_out


class _StepLoss(torch.autograd.Function):
    @staticmethod
    def forward(ctx, out_neg, out_pos, weight):
        loss, d_out = step_loss_raw(out_neg, out_pos, weight)
        ctx.save_for_backward(d_out)
        ctx.shapes = (out_neg.shape, out_pos.shape)
        return loss

    @staticmethod
    def backward(ctx, g):
        (d_out,) = ctx.saved_tensors
        d = d_out * g
        return d.view(ctx.shapes[0]), d.view(ctx.shapes[1]), None


def step_loss(out_neg, out_pos, weight):
    """The weighted loss of supervisor.py:19-23, differentiable w.r.t. both outputs."""
    return _StepLoss.apply(out_neg, out_pos, weight)


def step_forward(fn, mode, ent, rel, pos, neg, D, gamma, emb_range, rel_off=0, modulus=None,
                 temperature=1.0, adversarial=True, detach=False):
    """Fused, differentiable forward of both model calls of one train step -> (neg [B], pos [B])."""
    return _StepForward.apply(ent, rel, modulus, pos, neg, fn, mode, rel_off, D, gamma, emb_range,
                              float(temperature), bool(adversarial), bool(detach))


def score_indexed(fn, mode, ent, rel, pos, neg, D, gamma, emb_range, rel_off=0, modulus=None):
    """Fused gather + score -> raw scores [B, N] ([B, 1] for single). Differentiable w.r.t. the
    tables (and the pRotatE modulus)."""
    return _ScoreIndexed.apply(ent, rel, modulus, pos, None if mode == SINGLE else neg, fn, mode,
                               rel_off, D, gamma, emb_range)


def score_dense(fn, mode, head, relation, tail, D, gamma, emb_range, rel_off=0, modulus=0.0):
    """model_func plugin on pre-gathered rows -> [B, N]."""
    return _ScoreDense.apply(head, relation, tail, fn, mode, rel_off, D, gamma, emb_range,
                             float(modulus))


def neg_reduce(scores, temperature=1.0, adversarial=True, detach=False):
    """[B, N] -> [B]: sum softmax(T*s)*logsigmoid(-s) (adversarial) or mean logsigmoid(-s)."""
    return _NegReduce.apply(scores, float(temperature), bool(adversarial), bool(detach))


def log_sigmoid(x):
    return _LogSigmoid.apply(x)
