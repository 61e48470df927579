"""Benchmark of the KGE negative-sample scoring step on MI355X.

Metric (BASELINE.json): scored (pos+neg) triples/s, WN18RR InterHT d=1000 n_neg=256, 1/2/4/8 GPU.
One step = the forward of supervisor.py:17-18 on one batch, i.e. TFKGEModel.call for the batch's
negative mode (head/tail alternating, model.py:148-199) and for mode 3 (single, model.py:127-146):
  * fused gather + InterHT score of B*N negatives   -> [B, N]   (kernel score_fwd_kernel)
  * self-adversarial reduction                      -> [B, 1]   (neg_reduce_kernel)
  * fused gather + score of the B positives         -> [B, 1]   (score_fwd_kernel, single)
  * logsigmoid of the positives                     -> [B, 1]   (log_sigmoid_kernel)
Scored triples per step = B*N + B (the reference's redundant branches, Q2, are not counted).

Multi-GPU: one process per GPU; each rank scores its own batch with its own replica of the table
(weak scaling, no collective in the data path); timing = max over ranks. `--gpus N` (N > 1) outside
torchrun starts the N ranks itself: `python -m torch.distributed.run --nproc-per-node N` as a child
process, before this process makes any GPU call; the parent exits with the children's status.
Under torchrun (WORLD_SIZE set) the world size comes from the environment.

Positives: the reference's own triples where the snapshot has them (tests/golden/
<dataset>_ids.npz, made by tests/golden/make_datasets.py): WN18RR train.txt for C2 (RandomState(0)
permutation, read sequentially), FB15k-237 / YAGO3-10 valid+test for C3 / C4; negatives
RandomState(2).randint(E, (B, N)).

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--workload c2|c3|c4|...] [--dry-run]
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import statistics
import subprocess
import sys
import time

import numpy as np
import torch  # importing torch makes no GPU call; the package (and its HIP library) loads in main()

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "scored (pos+neg) triples/sec, WN18RR InterHT d=1000 n_neg=256, 1/2/4/8 GPU"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec

WORKLOADS = {
    # BASELINE.json configs[1]: the metric's config
    "c2": dict(name="WN18RR InterHT d=1000 -de -tr gamma=24 n_neg=256 bz=512", fn="InterHT",
               nentity=40943, nrelation=11, hidden_dim=1000, gamma=24.0, de=True, tr=True, dr=False,
               B=512, N=256, dataset="wn18rr"),
    # configs[2]
    "c3": dict(name="FB15k-237 RotatE d=1000 -de gamma=9 n_neg=256 bz=512", fn="RotatE",
               nentity=14541, nrelation=237, hidden_dim=1000, gamma=9.0, de=True, tr=False, dr=False,
               B=512, N=256, dataset="fb15k237"),
    # configs[3] (single-GPU replica form)
    "c4": dict(name="YAGO3-10 DistMult d=500 gamma=24 n_neg=1024 bz=512", fn="DistMult",
               nentity=123182, nrelation=37, hidden_dim=500, gamma=24.0, de=False, tr=False, dr=False,
               B=512, N=1024, dataset="yago3_10"),
    # configs[3] as the north star states it: entity table row-sharded over the ranks
    # (owner-computes, distributed.ShardedKGE; bz=512 per rank)
    # configs[4]: FB15k link-prediction eval, each query vs all 14 951 entities, filtered ranks
    # (DistMult d=1000 assumed); a step = one batch of 4096 queries, one mode
    "c5": dict(name="FB15k filtered eval DistMult d=1000, 4096 queries/step vs all 14951 entities",
               fn="DistMult", nentity=14951, nrelation=1345, hidden_dim=1000, gamma=24.0, de=False, tr=False,
               dr=False, B=4096, N=14951, eval=True),
    # TranSparse (model.py:226-235; in the reference's model_func dict, not in a BASELINE config):
    # WN18RR-sized graph, d=500, head-batch (the only mode whose scores depend on the negatives, Q9)
    "c6": dict(name="WN18RR-sized TranSparse d=500 gamma=12 n_neg=256 bz=512 head-batch", fn="TranSparse",
               nentity=40943, nrelation=11, hidden_dim=500, gamma=12.0, de=False, tr=False, dr=False,
               B=512, N=256, transparse=True),
    "c4s": dict(name="YAGO3-10 DistMult d=500 gamma=24 n_neg=1024 bz=512/rank, row-sharded owner-computes",
                fn="DistMult", nentity=123182, nrelation=37, hidden_dim=500, gamma=24.0, de=False, tr=False,
                dr=False, B=512, N=1024, sharded=True, dataset="yago3_10"),
    # the same, with the all-to-all row-fetch scheme (both schemes, measured side by side)
    "c4g": dict(name="YAGO3-10 DistMult d=500 gamma=24 n_neg=1024 bz=512/rank, row-sharded all-to-all row fetch",
                fn="DistMult", nentity=123182, nrelation=37, hidden_dim=500, gamma=24.0, de=False, tr=False,
                dr=False, B=512, N=1024, sharded=True, scheme="gather", dataset="yago3_10"),
}


def library_sha256():
    import hashlib
    path = os.path.join(ROOT, "customknowledgegraphembedding_amd", "libkge_hip.so")
    with open(path, "rb") as f:
        return hashlib.sha256(f.read()).hexdigest()


def loaded_source_hash():
    """kge_source_hash() of the loaded libkge_hip.so (the sources it was built from)."""
    from customknowledgegraphembedding_amd import _lib
    return _lib.load().kge_source_hash().decode()


def pmc_traffic(workload, kernel_prefixes):
    """Fabric (L2 <-> memory) bytes per step of the kernels `kernel_prefixes` (each: the mean over its
    head/tail instantiations, summed over the prefixes) from the committed rocprofv3 --pmc summary of
    this workload (profiles/pmc_<workload>.json, scripts/pmc.sh + scripts/pmc_summary.py: FETCH_SIZE x 2
    + WRITE_SIZE, the gfx950 corrections). (None, reason) when no summary was committed, or when it was
    measured on a library built from other sources than the one loaded now (kge_source_hash: stale)."""
    # KGE_PMC_DIR: summaries made in this same session (scripts/gpu_r03_final.sh) before they are committed
    path = os.path.join(os.environ.get("KGE_PMC_DIR") or os.path.join(ROOT, "profiles"), f"pmc_{workload}.json")
    try:
        with open(path) as f:
            summ = json.load(f)
        rows = summ["kernels"]
    except (OSError, ValueError, KeyError):
        return None, "no PMC summary committed"
    have = loaded_source_hash()
    if summ.get("source_hash") != have:
        return None, (f"stale: {os.path.relpath(path, ROOT)} was measured on sources {summ.get('source_hash')}, "
                      f"the loaded library is built from {have}")
    total = 0.0
    for pre in kernel_prefixes:
        got = [r["hbm_read_bytes_corrected"] + r.get("hbm_write_bytes", 0.0) for r in rows
               if r.get("kernel", "").startswith(pre + "<") or r.get("kernel", "") == pre]
        got = [g for g in got if g == g]
        if not got:
            return None, f"{os.path.relpath(path, ROOT)} has no {pre}"
        total += sum(got) / len(got)
    return total, os.path.relpath(path, ROOT)


def pmc_l2_requests(workload, kernel_prefixes):
    """Bytes the kernels request from L2 per step: (TCC_HIT_sum + TCC_MISS_sum) x 128 B lines, from the same
    PMC summary as pmc_traffic (None when it is missing or stale)."""
    path = os.path.join(os.environ.get("KGE_PMC_DIR") or os.path.join(ROOT, "profiles"), f"pmc_{workload}.json")
    try:
        with open(path) as f:
            summ = json.load(f)
        rows = summ["kernels"]
    except (OSError, ValueError, KeyError):
        return None
    if summ.get("source_hash") != loaded_source_hash():
        return None
    total = 0.0
    for pre in kernel_prefixes:
        got = [(r["TCC_HIT_sum"] + r["TCC_MISS_sum"]) * 128.0 for r in rows
               if (r.get("kernel", "").startswith(pre + "<") or r.get("kernel", "") == pre) and "TCC_HIT_sum" in r]
        if not got:
            return None
        total += sum(got) / len(got)
    return total


def roofline_hbm(step_bytes, traffic, traffic_src, kern_avg_s, **extra):
    """The HBM roofline object of a gather-bound step. `frac` is on the COUNTER bytes (the PMC passes'
    FETCH_SIZE x 2 + WRITE_SIZE of the same kernels, per launch) whenever a summary of this build
    exists: the algorithmic-bytes fraction can pass 1 when repeat gathers hit L2 / the Infinity Cache,
    the counter fraction cannot. The algorithmic figure (SURVEY §8d bytes) is reported beside it."""
    alg = step_bytes / kern_avg_s / 1e9
    r = {"bound": "hbm", "peak": HBM_PEAK_GBS, "unit": "GB/s", "traffic": traffic, "traffic_unit": "bytes/step",
         "traffic_source": traffic_src, "achieved_algorithmic": alg, "frac_algorithmic": alg / HBM_PEAK_GBS,
         "algorithmic_bytes_per_launch": step_bytes, "kernel_avg_us": kern_avg_s * 1e6}
    if traffic:
        ach = traffic / kern_avg_s / 1e9
        r.update({"achieved": ach, "frac": ach / HBM_PEAK_GBS, "frac_basis": "counter bytes (PMC)",
                  "frac_counter": ach / HBM_PEAK_GBS})
    else:
        r.update({"achieved": alg, "frac": alg / HBM_PEAK_GBS, "frac_basis": "algorithmic bytes (no PMC summary "
                  "of this build)", "frac_counter": None})
    r.update(extra)
    return r


# the L2-served gather rate of MI355X_MICROARCH.md §"Indexed rows: gather into LDS" (rows shared by every
# workgroup, served by the XCD's L2: 16.8-18.8 TB/s chip-wide), the ceiling of a kernel whose repeat gathers hit L2
L2_GATHER_PEAK_GBS = 18800.0


def l2_gather_roofline(l2_bytes, kern_avg_s):
    """Second roofline for a gather kernel that no longer reaches HBM for most rows: bytes requested from L2
    (PMC TCC_HIT + TCC_MISS lines) per step over the L2-served gather ceiling."""
    if not l2_bytes:
        return None
    ach = l2_bytes / kern_avg_s / 1e9
    return {"achieved": ach, "peak": L2_GATHER_PEAK_GBS, "unit": "GB/s", "frac": ach / L2_GATHER_PEAK_GBS,
            "l2_request_bytes_per_step": l2_bytes,
            "peak_source": "MI355X_MICROARCH.md, indexed rows gathered from the XCD's L2: 16.8-18.8 TB/s chip-wide"}


def dims(w):
    d = w["hidden_dim"]
    ent = 2 * d if w["de"] else d
    if w["tr"]:
        rel = 3 * d
    elif w["dr"]:
        rel = 2 * d
    else:
        rel = d
    D = ent // 2 if w["fn"] in ("ComplEx", "RotatE", "InterHT") else ent
    rel_used = rel // 3 if w["fn"] == "InterHT" else rel
    return ent, rel, D, rel_used


def algorithmic_bytes(w):
    """per negative launch = B*N*(4*ent_dim + 8 idx + 4 score) + the shared query
    side B*(4*ent_dim + 4*rel_used + 24); per positive launch B*(8*ent_dim + 4*rel_used + 28)."""
    ent, _, _, rel_used = dims(w)
    B, N = w["B"], w["N"]
    neg = B * N * (4 * ent + 8 + 4) + B * (4 * ent + 4 * rel_used + 24)
    pos = B * (8 * ent + 4 * rel_used + 28)
    return neg, pos


def load_triples(w):
    """The reference's triples of the workload's dataset (tests/golden/<dataset>_ids.npz), or None."""
    key = w.get("dataset")
    if not key:
        return None
    path = os.path.join(ROOT, "tests", "golden", f"{key}_ids.npz")
    with np.load(path) as z:  # allow_pickle=False: plain int arrays
        tri = z["triples"].astype(np.int64)
        assert int(z["nentity"]) == w["nentity"] and int(z["nrelation"]) == w["nrelation"], path
    return tri


def positives(w, rank, n_batches, world=1):
    """[n_batches] x [B, 3] positives: the dataset's triples in a RandomState(0) permutation, read
    sequentially (rank r takes every world-th batch), or uniform random ids without a dataset."""
    E, R, B = w["nentity"], w["nrelation"], w["B"]
    tri = load_triples(w)
    out = []
    if tri is None:
        for i in range(n_batches):
            g = np.random.RandomState(1 + 1000 * rank + i)
            out.append(np.stack([g.randint(E, size=B), g.randint(R, size=B), g.randint(E, size=B)], 1))
        return out, "uniform random (h, r, t)"
    perm = np.random.RandomState(0).permutation(len(tri))
    for i in range(n_batches):
        k = (i * world + rank) * B
        idx = perm[np.arange(k, k + B) % len(tri)]
        out.append(tri[idx])
    return out, f"reference triples tests/golden/{w['dataset']}_ids.npz (RandomState(0) permutation)"


def rank_batches(w, rank, n_batches=8, world=1):
    """Host ids of rank `rank`'s batches: ([(pos [B,3], neg [B,N])], positives source). Ranks read
    disjoint positives (batch i of rank r is sequential batch i * world + r); negatives
    RandomState(2 + 1000 rank + i).randint(E, (B, N))."""
    E, B, N = w["nentity"], w["B"], w["N"]
    pos_l, src = positives(w, rank, n_batches, world)
    return [(pos_l[i], np.random.RandomState(2 + 1000 * rank + i).randint(E, size=(B, N)))
            for i in range(n_batches)], src


def make_inputs(w, rank, device, n_batches=8, world=1):
    from customknowledgegraphembedding_amd.model import TFKGEModel
    m = TFKGEModel(w["fn"], w["nentity"], w["nrelation"], w["hidden_dim"], w["gamma"],
                   double_entity_embedding=w["de"], double_relation_embedding=w["dr"],
                   triple_relation_embedding=w["tr"], device=device, seed=0)
    host, src = rank_batches(w, rank, n_batches, world)
    batches = [(torch.from_numpy(p).to(device), torch.from_numpy(n).to(device)) for p, n in host]
    m.positives_source = src
    return m, batches


def cpu_baseline_inputs(w, rows):
    """The CPU baseline's sample: the first `rows` rows of rank 0's batch 0, the GPU line's own inputs."""
    (pos, neg), = rank_batches(w, 0, 1)[0][:1]
    src = rank_batches(w, 0, 1)[1]
    return torch.from_numpy(pos[:rows]), torch.from_numpy(neg[:rows]), src


def run_step(m, pos, neg, mode, fn, ev=None):
    """Forward of supervisor.py:17-18 (both model calls) = kge_step_forward: ONE launch of the fused
    step kernel (block per batch row: the negatives' gather + score, then the row's positive and
    self-adversarial reduction), bracketed by events on torch's current stream (the launch stream)."""
    ent, rel = m.entity_embedding.detach(), m.relation_embedding.detach()
    if ev is not None:
        ev[0].record()
    out = ops.step_forward_raw(fn, mode, ent, rel, m._rel_off, pos, neg, m._D, m._gamma_f, m._range_f)
    if ev is not None:
        ev[1].record()
    return out


class StepRunner:
    """The headline step loop: step i scores batch i % len(batches) in mode i % 2. With a planner
    (ops.StepPlanner, the default where the tile form applies; KGE_BENCH_UNPLANNED=1 turns it off) step i is
    kge_step_forward_planned on the plan step i - 1 made in its launch's tail, and it makes step i + 1's plan
    the same way: one plan per step, inside the step. Without one, step i is kge_step_forward (its setup in
    the scoring launch)."""

    def __init__(self, m, batches, fn, planned=True):
        self.m, self.batches, self.fn = m, batches, fn
        ent, rel = m.entity_embedding.detach(), m.relation_embedding.detach()
        B, N = batches[0][1].shape
        mod = float(m.modulus.detach().reshape(-1)[0]) if m.model_name == "pRotatE" else 0.0
        self.planner = None
        if planned and ops.StepPlanner.available(fn, ent, rel, m._rel_off, m._D, B, N):
            self.planner = ops.StepPlanner(fn, ent, rel, m._rel_off, m._D, B, N, m._gamma_f, m._range_f,
                                           modulus=mod)
        self.next_i = None  # the step the pending plan is for
        # two output sets, alternating (a training loop double-buffers what the next step overwrites)
        self.outs = [self.planner.outputs() for _ in range(2)] if self.planner is not None else None

    def batch(self, i):
        return self.batches[i % len(self.batches)]

    def __call__(self, i, mode=None):
        """Step i (mode: i % 2 unless forced; a forced-mode run plans the next step in the same mode)."""
        md = i % 2 if mode is None else mode
        pos, neg = self.batch(i)
        if self.planner is None:
            return run_step(self.m, pos, neg, md, self.fn)
        if self.next_i != (i, md):
            self.planner.plan(pos, neg, md)  # the chain starts here (a run's first step, or a new chain)
        npos, nneg = self.batch(i + 1)
        nmd = (i + 1) % 2 if mode is None else mode
        out = self.planner.step(nxt=(npos, nneg, nmd), out=self.outs[i % 2])
        self.next_i = (i + 1, nmd)
        return out


def _global_batches(w, world, n, device):
    """n global batches of world x B rows (identical on every rank: the replicas' batches replicated
    by seed): YAGO3-10 positives (RandomState(0) permutation), RandomState negatives."""
    E, B, N = w["nentity"], w["B"], w["N"]
    WB = world * B
    tri = load_triples(w)
    perm = np.random.RandomState(0).permutation(len(tri))
    out = []
    for i in range(n):
        idx = perm[np.arange(i * WB, (i + 1) * WB) % len(tri)]
        neg = np.random.RandomState(200 + i).randint(E, size=(WB, N))
        wt = np.random.RandomState(300 + i).uniform(0.1, 1.0, size=WB).astype(np.float32)
        out.append((torch.from_numpy(tri[idx]).to(device), torch.from_numpy(neg).to(device),
                    torch.from_numpy(wt).to(device)))
    return out


def sharded_bench(w, a, world, rank, device, dist_on, train=False):
    """c4s: ShardedKGE.step_forward (or, with train, ShardedKGE.train_step: the whole row-sharded
    train step with Keras Adam) on the global batch; the timed step includes every collective.
    Returns the elapsed seconds of a.steps steps (this rank)."""
    from customknowledgegraphembedding_amd.distributed import ShardedKGE
    sk = ShardedKGE(w["fn"], w["nentity"], w["nrelation"], w["hidden_dim"], w["gamma"],
                    double_entity_embedding=w["de"], double_relation_embedding=w["dr"],
                    triple_relation_embedding=w["tr"], device=device, seed=0)
    batches = _global_batches(w, world, 4, device)
    if train:
        sk.configure_optimizer(lr=5e-5)

        def step(b, i):
            return sk.train_step(b[0], b[1], b[2], i % 2)
    elif w.get("scheme") == "gather":
        def step(b, i):
            return sk.step_forward_gather(b[0], b[1], i % 2)
    elif sk.world > 1 and dist_on and os.environ.get("KGE_SHARD_NATIVE", "0") == "1":
        # the native executor (one C call per rank-step, RCCL issued from C++ through its own communicator):
        # each step also plans the next batch, on the executor's plan stream, overlapping this step
        from customknowledgegraphembedding_amd.distributed import NativeComm
        sk.use_native(NativeComm(device=device))
        sk.plan_native(batches[0][0], batches[0][1], 0)  # two batches planned ahead, then each step plans the
        sk.plan_native(batches[1][0], batches[1][1], 1)  # batch two steps later

        def step(b, i):
            nb = batches[(i + 2) % 4]
            return sk.step_forward(b[0], b[1], i % 2, nxt=(nb[0], nb[1], i % 2))
    else:
        # the exchange plan of step i + 1 (kge_shard_plan: ownership counts and ranks from the ids, its
        # split sizes copied to the host asynchronously) is issued before step i's work, so the host
        # never waits for it; it is device work inside the timed region like the rest of the step, on a
        # side stream (KGE_PLAN_STREAM=main: the step's own stream) where it overlaps step i's scoring
        # (the Python host path, the default of this standalone workload; KGE_SHARD_NATIVE=1: the native
        # executor, which the headline's N > 1 section runs after checking it, rowshard_multi)
        plans = {}
        side = torch.cuda.Stream(device) if os.environ.get("KGE_PLAN_STREAM", "side") == "side" else None

        def step(b, i):
            if sk.world == 1:  # no exchange: the step is the unsharded fused forward
                return sk.step_forward(b[0], b[1], i % 2)
            nb = batches[(i + 1) % 4]
            plan = plans.pop(i, None) or sk.plan(b[0], b[1], i % 2)
            plans[i + 1] = sk.plan(nb[0], nb[1], (i + 1) % 2, stream=side)
            return sk.step_forward(b[0], b[1], i % 2, plan=plan)
    for i in range(a.warmup):
        step(batches[i % 4], i)
    torch.cuda.synchronize()
    if dist_on:
        import torch.distributed as tdist
        tdist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(a.warmup, a.warmup + a.steps):
        step(batches[i % 4], i)
    torch.cuda.synchronize()
    if dist_on:
        tdist.barrier()
    return time.perf_counter() - t0


# The native executor's two forms measured at N > 1: the collectives on the step's own stream with
# one chunk (the default: no cross-stream event hops, profiles/r04_native_timeline.txt), and on a communication
# stream with two chunks (half of each exchange under the other chunk's scoring)
ROWSHARD_VARIANTS = (("one_stream_1chunk", dict(one_stream=True, chunks=1)),
                     ("two_stream_2chunk", dict(one_stream=False, chunks=2)))
ROWSHARD_DEFAULT = "one_stream_1chunk"
ROWSHARD_RANK_KEYS = ("rank", "step_us", "kernel_busy_us", "query_a2a_us", "score_a2a_us", "host_wait_us",
                      "host_call_us")


def _gather_objects(obj, world):
    import torch.distributed as tdist
    out = [None] * world
    tdist.all_gather_object(out, obj)
    return out


def _max_over_ranks(x, device):
    import torch.distributed as tdist
    t = torch.tensor([x], dtype=torch.float64, device=device)
    tdist.all_reduce(t, op=tdist.ReduceOp.MAX)
    return float(t.item())


def rowshard_report(w, world, steps, variants, per_rank, n_ranks_seen, native_status, matches):
    """The N > 1 row-sharded record (yago3_10_rowshard): the per-variant max-over-ranks step times, the selected
    form's throughput, every rank's diagnosis (device spans of one step from the executor's timing events, the
    host time per call and its wait for plans), what the communicator saw, and whether the native step's
    outputs equal the torch.distributed path's on the same batch (its first cross-process run checks itself)."""
    trip = (w["B"] * w["N"] + w["B"]) * world
    var = {k: {"ms_per_step": v * 1e3, "triples_per_s": trip / v} for k, v in variants.items()}
    sel = ROWSHARD_DEFAULT if (ROWSHARD_DEFAULT in var and native_status == "ok" and matches) else "torchcomm_python"
    return {"workload": w["name"], "n_gpus": world, "global_batch": w["B"] * world, "n_neg": w["N"], "steps": steps,
            "selected": sel, "triples_per_s": var[sel]["triples_per_s"], "ms_per_step": var[sel]["ms_per_step"],
            "variants": var, "per_rank": per_rank, "n_ranks_seen": n_ranks_seen, "native_status": native_status,
            "native_matches_torchcomm": matches,
            "what": "distributed.ShardedKGE.step_forward: entity table row-sharded over the ranks, owner-computes "
                    "scoring, one RCCL all-to-all of the owners' compacted query rows and one of the owned scores; "
                    "variants: the native executor (one C call per rank-step, ncclAllToAllv from C++) with the "
                    "collectives on the step's stream (1 chunk) or on a communication stream (2 chunks), and the "
                    "Python path over torch.distributed; selected: the native default when its communicator "
                    "checked out and its outputs equal the Python path's bitwise, else the Python path"}


def rowshard_multi(w, a, world, rank, device):
    """N > 1: the row-sharded forward step through (1) the Python path over torch.distributed (RCCL via torch)
    and (2) the native executor in both ROWSHARD_VARIANTS, after a known-answer check of the native communicator
    (ncclCommCount, one all-to-all of rank-tagged values) agreed on by every rank; then one diagnosis pass with
    the executor's timing events. A native failure is recorded (native_status) and the Python path stands."""
    import torch.distributed as tdist
    from customknowledgegraphembedding_amd.distributed import NativeComm, ShardedKGE, TorchComm
    sk = ShardedKGE(w["fn"], w["nentity"], w["nrelation"], w["hidden_dim"], w["gamma"], device=device, seed=0,
                    comm=TorchComm())
    sk.exchange = True  # the exchange path at every world size (at world 1 its pieces are a rank's own)
    batches = _global_batches(w, world, 4, device)
    lib = kge.load()
    variants = {}

    def timed(step, n_warm, n):
        for i in range(n_warm):
            step(i)
        torch.cuda.synchronize()
        tdist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(n_warm, n_warm + n):
            step(i)
        torch.cuda.synchronize()
        tdist.barrier()
        return _max_over_ranks(time.perf_counter() - t0, device)

    # (1) the Python path: plans made a step ahead on a side stream
    plans, side = {}, torch.cuda.Stream(device)

    def py_step(i):
        b, nb = batches[i % 4], batches[(i + 1) % 4]
        plan = plans.pop(i, None) or sk.plan(b[0], b[1], i % 2)
        plans[i + 1] = sk.plan(nb[0], nb[1], (i + 1) % 2, stream=side)
        return sk.step_forward(b[0], b[1], i % 2, plan=plan)
    ref = [t.clone() for t in sk.step_forward(batches[0][0], batches[0][1], 0)]
    variants["torchcomm_python"] = timed(py_step, a.warmup, a.steps) / a.steps
    # (2) the native communicator, checked before any executor uses it
    status, comm, seen = "ok", None, None
    try:
        comm = NativeComm(device=device)
        seen = int(lib.kge_comm_size(comm.handle))
        send = torch.tensor([rank * 1000.0 + o for o in range(world)], device=device)
        recv = torch.empty(world, device=device)
        comm.all_to_all(recv, send, [1] * world, [1] * world)
        torch.cuda.synchronize()
        want = torch.tensor([o * 1000.0 + rank for o in range(world)], device=device)
        if seen != world or not torch.equal(recv, want):
            status = f"known-answer check failed: ncclCommCount {seen}, all-to-all {recv.tolist()}"
    except Exception as e:  # noqa: BLE001
        status = "native communicator: " + repr(e)
    bad = torch.tensor([0 if status == "ok" else 1], device=device)
    tdist.all_reduce(bad, op=tdist.ReduceOp.MAX)  # every rank takes the native path, or none does
    if status == "ok" and int(bad.item()):
        status = "another rank's native communicator check failed"
    matches = None
    per_rank = {"rank": rank}
    if status == "ok":
        for name, cfg in ROWSHARD_VARIANTS:
            sk.use_native(comm, one_stream=cfg["one_stream"])
            ch = cfg["chunks"]
            got = [t.clone() for t in sk.step_forward(batches[0][0], batches[0][1], 0, chunks=ch)]
            same = all(bool(((x == y) | (torch.isnan(x) & torch.isnan(y))).all()) for x, y in zip(got, ref))
            matches = same if matches is None else (matches and same)
            sk.plan_native(batches[1][0], batches[1][1], 1, chunks=ch)
            sk.plan_native(batches[2][0], batches[2][1], 0, chunks=ch)

            def nat_step(i, ch=ch):
                b, nb = batches[(i + 1) % 4], batches[(i + 3) % 4]
                return sk.step_forward(b[0], b[1], (i + 1) % 2, chunks=ch, nxt=(nb[0], nb[1], (i + 3) % 2))
            variants[name] = timed(nat_step, a.warmup, a.steps) / a.steps
        # diagnosis: the default form with timing events, a few steps; device spans of each, host time per call
        cfg = dict(ROWSHARD_VARIANTS)[ROWSHARD_DEFAULT]
        sk.use_native(comm, one_stream=cfg["one_stream"], timing=True)
        ch = cfg["chunks"]
        sk.plan_native(batches[0][0], batches[0][1], 0, chunks=ch)
        sk.plan_native(batches[1][0], batches[1][1], 1, chunks=ch)
        spans, calls, waits = [], [], []
        ex = None
        for i in range(8):
            b, nb = batches[i % 4], batches[(i + 2) % 4]
            t0 = time.perf_counter()
            sk.step_forward(b[0], b[1], i % 2, chunks=ch, nxt=(nb[0], nb[1], i % 2))
            calls.append((time.perf_counter() - t0) * 1e6)
            ex = ex or next(iter(sk._native.values()))
            waits.append(ex.host_wait_us())
            spans.append(ex.timings())
        torch.cuda.synchronize()
        tdist.barrier()
        sp = spans[2:]  # after the first steps' ramp
        per_rank.update({
            "step_us": statistics.median(x["step_us"] for x in sp),
            "kernel_busy_us": statistics.median(x["gather_us"] + x["finish_us"] + sum(x["score_us"]) for x in sp),
            "query_a2a_us": statistics.median(sum(x["query_a2a_us"]) for x in sp),
            "score_a2a_us": statistics.median(sum(x["score_a2a_us"]) for x in sp),
            "host_wait_us": statistics.median(waits[2:]), "host_call_us": statistics.median(calls[2:]),
            "spans_of_one_step": sp[-1]})
        sk.use_native(None, probe=True)  # closes the executors
        comm.close()
    else:
        per_rank.update({k: None for k in ROWSHARD_RANK_KEYS if k != "rank"})
    per = _gather_objects(per_rank, world)
    return rowshard_report(w, world, a.steps, variants, per, seen, status, matches)


def rank0_step_parts(ranks, pos, neg, mode, chunks=None):
    """Rank 0's device work of one row-sharded forward step, as closures over inputs prepared untimed
    with every simulated rank's contributions (ranks: ShardedKGE of ranks 0..W-1 on one GPU): plan_fn
    (the plan with rank 0's bucket), gather (the query gather of every chunk, one launch), score (compact
    scoring of every chunk), finish (scatter + reductions)."""
    from customknowledgegraphembedding_amd.distributed import HipShardKernels as HK
    r0 = ranks[0]
    world, device = r0.world, r0.device
    Bg = pos.shape[0]
    plans = [sk.plan(pos, neg, mode, chunks) for sk in ranks]  # identical but for each rank's bucket
    plan = plans[0]
    tot, qtot = plan.summary()
    K = plan.chunks
    Rk, hpc = Bg // K, world // K
    blocks, qidxs, sends = [], [], []
    for k in range(K):
        per = [int(qtot[k, :, o].sum()) for o in range(world)]
        pieces = []
        for sk in ranks:  # every owner's compacted rows: the query all-to-all's output
            snd = torch.empty((world, per[sk.rank], r0.entity_dim), dtype=torch.float32, device=device)
            qidx = torch.empty((plan.ncol, Rk), dtype=torch.int64, device=device)
            HK.gather_queries(sk, plans[sk.rank], pos, k, snd, qidx)
            pieces.append(snd[0])
        blocks.append(torch.cat(pieces))
        qidxs.append(qidx)
        sends.append(torch.empty(int(sum(tot[h, 0] for h in range(k * hpc, (k + 1) * hpc))), dtype=torch.float32,
                                 device=device))
    # home 0's score all-to-all output: every owner's block of home 0's rows, in rank order
    recv = []
    for sk in ranks:
        snd = torch.empty(int(sum(tot[h, sk.rank] for h in range(hpc))), dtype=torch.float32, device=device)
        HK.score_compact(sk, blocks[0], qidxs[0][0], pos, neg, plans[sk.rank], 0, Rk, snd)
        recv.append(snd[:int(tot[0, sk.rank])])
    recv = torch.cat(recv)
    q_send = torch.empty(sum(world * int(qtot[k, :, 0].sum()) for k in range(K)) * r0.entity_dim,
                         dtype=torch.float32, device=device)
    q_idx = torch.empty((plan.ncol, Bg), dtype=torch.int64, device=device)

    def score():
        for k in range(K):
            HK.score_compact(r0, blocks[k], qidxs[k][0], pos, neg, plan, k * Rk, Rk, sends[k])

    return {"plan": plan, "chunks": K, "plan_fn": lambda: HK.plan(r0, pos, neg, mode, K),
            "gather": lambda: HK.gather_queries(r0, plan, pos, -1, q_send, q_idx), "score": score,
            "finish": lambda: HK.shard_finish(r0, plan, recv, pos, neg, 1.0, True)}


class _PrefilledComm:
    """One rank's communicator stand-in for measuring its host cost: every collective returns at once and
    its output buffers keep what they hold (the scores computed from them are garbage; only the host time
    is read). No other rank exists, so no other thread contends for the GIL."""

    def __init__(self, world, rank):
        self.world, self.rank = world, rank

    def all_to_all(self, out, inp, out_splits, in_splits, async_op=False):
        from customknowledgegraphembedding_amd.distributed import _Done
        return _Done()


def rank_host_cost(tables, world, device, steps=20):
    """CPU time one rank's thread spends issuing ShardedKGE.step_forward at `world` ranks (full C4 size): one
    real rank (rank 0) with a prefilled-buffer communicator, the device held behind a sleep kernel so that no
    host call waits for the GPU. Returns per-step microseconds of the plan made a step ahead (plan) and of
    the step given that plan (step), and whether the device was still held when the host finished (if not,
    the host waited and the figure is an upper bound)."""
    from customknowledgegraphembedding_amd.distributed import ShardedKGE
    w = WORKLOADS["c4s"]
    sk = ShardedKGE("DistMult", w["nentity"], w["nrelation"], w["hidden_dim"], w["gamma"], device=device,
                    world=world, rank=0, comm=_PrefilledComm(world, 0), full_tables=tables)
    batches = _global_batches(w, world, 4, device)
    side = torch.cuda.Stream(device)
    plans = [sk.plan(batches[i % 4][0], batches[i % 4][1], i % 2) for i in range(steps)]
    for p in plans:
        p.summary()  # resolved before the timed region: step_forward then never waits for the device
    for i in range(3):
        sk.step_forward(batches[i % 4][0], batches[i % 4][1], i % 2, plan=plans[i])
        sk.plan(batches[i % 4][0], batches[i % 4][1], i % 2, stream=side)
    torch.cuda.synchronize()

    def held(f):
        torch.cuda._sleep(200_000_000)  # hold the device queue (far longer than the host loop)
        t0 = time.perf_counter()
        f()
        el = time.perf_counter() - t0
        probe = torch.cuda.Event()
        probe.record()
        still = not probe.query()
        torch.cuda.synchronize()
        return el / steps * 1e6, still

    plan_us, held_p = held(lambda: [sk.plan(batches[i % 4][0], batches[i % 4][1], i % 2, stream=side)
                                    for i in range(steps)])
    step_us, held_s = held(lambda: [sk.step_forward(batches[i % 4][0], batches[i % 4][1], i % 2, plan=plans[i])
                                    for i in range(steps)])
    out = {"python_path": {"plan": plan_us, "step": step_us, "total": plan_us + step_us,
                           "device_held_throughout": held_p and held_s, "steps": steps,
                           "what": "host time of one rank's ShardedKGE.plan (next step, side stream) + "
                                   f"step_forward(plan=...) at W={world}, C4 full size; collectives stubbed (return "
                                   "at once), device queue held behind a sleep kernel: the Python + ctypes + launch "
                                   "cost per rank-step, before any torch.distributed call"}}
    out["native"] = native_host_cost(tables, world, device, batches, 4 * steps)
    out["per_rank_step_us"] = out["native"]["step_us"]
    return out


def native_host_cost(tables, world, device, batches, steps):
    """Host time of one rank's native row-sharded step (ShardedKGE.use_native: ONE C call that issues the
    query gather, per chunk the query all-to-all, the owner-computes scoring and the score all-to-all, the
    finish, and the NEXT batch's plan) at `world` ranks, C4 full size, collectives skipped (KGE_EXEC_PROBE;
    an RCCL ncclAllToAllv call's own host cost is measured beside it in scripts/shard_host_probe.py). The
    device runs the steps back to back; the host time the calls spent blocked on the plans' summaries (the
    device pacing the host) is subtracted."""
    from customknowledgegraphembedding_amd.distributed import ShardedKGE
    w = WORKLOADS["c4s"]
    sk = ShardedKGE("DistMult", w["nentity"], w["nrelation"], w["hidden_dim"], w["gamma"], device=device,
                    world=world, rank=0, comm=_PrefilledComm(world, 0), full_tables=tables).use_native(probe=True)
    nb = len(batches)
    at = [0]  # the plan-ahead chain continues across the calls: step i plans batch i + 2
    for i in range(2):
        sk.plan_native(batches[i][0], batches[i][1], i % 2)

    def run(n):
        for i in range(at[0], at[0] + n):
            p, q, _ = batches[i % nb]
            np_, nq, _ = batches[(i + 2) % nb]
            sk.step_forward(p, q, i % 2, nxt=(np_, nq, i % 2))
        at[0] += n

    run(6)
    torch.cuda.synchronize()
    ex = next(iter(sk._native.values()))
    lib = kge.load()
    lib.kge_shard_exec_host_wait_us(ex.handle, 1)
    # per call: its wall time minus the time it spent blocked on the plan's summary; the median over the calls
    # (a mean let a few host stalls, and waits outside the plan wait, swing it 32-92 us between runs of one box)
    per, blocked = [], 0.0
    t0 = time.perf_counter()
    for _ in range(steps):
        c0 = time.perf_counter()
        run(1)
        c1 = time.perf_counter()
        wt = lib.kge_shard_exec_host_wait_us(ex.handle, 1)
        blocked += wt
        per.append((c1 - c0) * 1e6 - wt)
    el = time.perf_counter() - t0
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    run(steps)
    torch.cuda.synchronize()
    dev_us = (time.perf_counter() - t1) / steps * 1e6
    ex.close()
    return {"step_us": statistics.median(per), "step_us_mean": (el * 1e6 - blocked) / steps,
            "blocked_us_per_step": blocked / steps,
            "wall_us_per_step": dev_us, "steps": steps, "chunks": ex.K,
            "what": f"host time per rank-step of the native executor at W={world} (one ctypes call: gather, "
                    f"{ex.K} x (query all-to-all, scoring, score all-to-all), finish, next plan), C4 full size, "
                    "collectives skipped; step_us: median over the calls of the call's time minus its wait for the "
                    "plan's summary (step_us_mean: the mean); wall_us_per_step: the same steps with the device "
                    "pacing them"}


def shard_sim_bench(device, world=8, reps=10, v1=None):
    """Single-GPU evidence for the row-sharded scaling at the full C4 size (YAGO3-10
    DistMult d=500, E=123182, N=1024, global batch of world x 512 rows):
      * rank 0's own kernels of one step (plan, per-chunk query gather and compact scoring, finish),
        timed alone with events on the launch stream: the per-GPU compute of an N-GPU step;
      * the payload rank 0's collectives carry per step, and the RCCL bandwidth a step needs to reach
        6x the 1-GPU row-sharded throughput `v1` (triples/s) when the collectives do not overlap;
      * the sharded train step's kernels of rank 0 (forward, combine, backward)."""
    from customknowledgegraphembedding_amd.distributed import HipShardKernels, ShardedKGE, ThreadComm
    from customknowledgegraphembedding_amd.model import TFKGEModel
    w = WORKLOADS["c4s"]
    E, d, N = w["nentity"], w["hidden_dim"], w["N"]
    pos, neg, wt = _global_batches(w, world, 1, device)[0]
    Bg = pos.shape[0]
    B = Bg // world
    full = TFKGEModel("DistMult", E, w["nrelation"], d, w["gamma"], device=device, seed=0)
    ent, rel = full.entity_embedding.detach(), full.relation_embedding.detach()
    tables = (ent, rel, full._gamma_f, full._range_f, 0.0)
    fn = FN_IDS["DistMult"]

    def timed(f, n=reps, queue=True):
        """Device time of f() per call: the launches are queued behind a sleep kernel, so the events bracket
        back-to-back GPU work and not the host's launch rate (ctypes launches cost ~10 us each here)."""
        f()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        if queue:
            torch.cuda._sleep(50_000_000)
        e0.record()
        for _ in range(n):
            f()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / n * 1e3  # us

    unsharded_us = timed(lambda: ops.score_indexed_raw(fn, 0, ent, rel, 0, pos, neg, d, full._gamma_f, full._range_f))
    step_us = timed(lambda: ops.step_forward_raw(fn, 0, ent, rel, 0, pos, neg, d, full._gamma_f, full._range_f))
    comm = ThreadComm(world)
    ranks = [ShardedKGE("DistMult", E, w["nrelation"], d, w["gamma"], device=device, world=world, rank=r, comm=comm,
                        full_tables=tables) for r in range(world)]
    # rank 0 alone: the kernels of one step, with the other ranks' contributions prepared untimed
    HK = HipShardKernels
    r0 = ranks[0]
    parts = rank0_step_parts(ranks, pos, neg, 0)
    plan, K = parts["plan"], parts["chunks"]
    t_plan = timed(parts["plan_fn"])
    t_gather = timed(parts["gather"])
    t_score = timed(parts["score"])
    t_finish = timed(parts["finish"])
    # the plan is made a step ahead on a side stream (sharded_bench, KGE_PLAN_STREAM): off the critical path
    rank_us = t_gather + t_score + t_finish
    cb = r0.collective_bytes(plan)
    coll = cb["query_rows"] + cb["scores"]
    B_ = Bg // world
    out = {"workload": f"C4 YAGO3-10 DistMult d=500 N=1024, global batch {world} x 512 (YAGO3-10 positives), "
                       f"entity table split over {world} simulated ranks",
           "rank_step_kernels_us": {"plan_side_stream": t_plan, "query_gather": t_gather, "compact_scoring": t_score,
                                    "finish": t_finish, "critical_path": rank_us},
           "host_us_per_rank_step": rank_host_cost(tables, world, device),
           "unsharded_global_kernel_us": unsharded_us,
           "unsharded_global_step_us": step_us,
           "rank_scoring_over_unsharded": t_score / unsharded_us,
           "collective_bytes_per_rank_step": cb,
           "zero_padded_round2_bytes_per_rank_step": {"query_rows_allreduce_ring": 2 * (world - 1) * Bg * d * 4 * 2 // world,
                                                       "scores_reduce_scatter": (world - 1) * B_ * (N + 1) * 4},
           "chunks": K,
           "what": "rank_step_kernels_us: rank 0's kernels of one 8-rank step, device time (queued behind a sleep "
                   "kernel): its per-GPU compute in an 8-GPU step (critical_path: without the plan, which the "
                   "step makes a step ahead on a side stream); collective_bytes_per_rank_step: what its two "
                   "all-to-alls carry; six_x_target: the RCCL rate those bytes need for 6x the 1-GPU line"}
    if v1:
        t6 = world * B_ * (N + 1) / (6.0 * v1) * 1e6  # us per step at 6x the 1-GPU throughput
        out["six_x_target"] = {"one_gpu_triples_per_s": v1, "step_budget_us": t6,
                               "collective_budget_us_without_overlap": t6 - rank_us,
                               "rccl_gbps_needed_without_overlap": (coll / ((t6 - rank_us) * 1e-6) / 1e9
                                                                    if t6 > rank_us else None)}
    # the sharded train step's kernels of rank 0 (forward, combine, backward), collectives priced by size
    sk = ShardedKGE("DistMult", E, w["nrelation"], d, w["gamma"], device=device, world=world, rank=0,
                    full_tables=tables).configure_optimizer(lr=5e-5)
    qent = ent[pos[:, 2]].contiguous()  # head-batch query rows (the all-gather's result)
    qpos = ent[pos[:, 0]].contiguous()
    bufs = HK.train_alloc(sk, Bg, N)
    HK.train_forward(sk, bufs, 0, qent, qpos, pos, neg, wt)
    stats_all = bufs["stats"].unsqueeze(0).expand(world, -1, -1).contiguous()
    t_fwd = timed(lambda: HK.train_forward(sk, bufs, 0, qent, qpos, pos, neg, wt))
    t_comb = timed(lambda: HK.train_combine(sk, bufs, 0, qent, qpos, pos, neg, wt, stats_all))
    t_bwd = timed(lambda: HK.train_backward(sk, bufs, 0, qent, qpos, pos, neg, wt, 3, None))
    out["rank_train_step_kernels_us"] = {"forward": t_fwd, "combine": t_comb, "backward": t_bwd,
                                         "total": t_fwd + t_comb + t_bwd}
    out["train_collective_bytes_per_rank_step"] = {
        "query_rows_alltoall": (world - 1) * 2 * Bg // world * d * 4,
        "stats_allgather": (world - 1) * Bg * 16, "query_grad_allreduce_ring": 2 * (world - 1) * 2 * Bg * d * 4 // world}
    return out


def eval_bench(w, a, device, world=1, rank=0, dist_on=False):
    """c5: upstream test_step's scoring + filtered ranking for batches of queries: kge_eval_query +
    kge_gemm_nt (fp32 MFMA, events around it) + kge_rank_filtered. Multi-GPU = replicas: every rank
    holds the (60 MB) table and ranks its own query batches (weak scaling, no collective in the
    data path); value = all ranks' queries / max elapsed. Returns the JSON line."""
    from customknowledgegraphembedding_amd import evaluate
    from customknowledgegraphembedding_amd.model import KGEModel
    m = KGEModel(w["fn"], w["nentity"], w["nrelation"], w["hidden_dim"], w["gamma"], device=device, seed=0)
    E, R, Bq = w["nentity"], w["nrelation"], w["B"]
    g = np.random.RandomState(7)
    true = np.stack([g.randint(E, size=200000), g.randint(R, size=200000), g.randint(E, size=200000)], 1)
    batches = []
    for i in range(4):
        q = true[(rank * 4 + i) * Bq:(rank * 4 + i + 1) * Bq]
        mode = "head-batch" if i % 2 == 0 else "tail-batch"
        ptr, ids = evaluate.build_filter(q, mode, true)
        col = 0 if mode == "head-batch" else 2
        pos = torch.from_numpy(q).to(device)
        batches.append((pos, mode, pos[:, col].contiguous(), torch.from_numpy(ptr).to(device),
                        torch.from_numpy(ids).to(device), int(ptr[-1])))
    S = torch.empty((Bq, E), dtype=torch.float32, device=device)
    K = m.entity_embedding.shape[1]
    ent = m.entity_embedding.detach()
    Q = torch.empty((Bq, K), dtype=torch.float32, device=device)
    lib = __import__("customknowledgegraphembedding_amd._lib", fromlist=["load"]).load()
    # planes (default): ranks straight from the planes, batches alternating between two streams
    # (evaluate.RankPipeline: batch i + 1's kernels fill the CUs batch i's GEMM leaves idle); planes1: one stream
    # (kge_eval_rank_planes); planes_s: the plane GEMM writing S, then kge_rank_filtered (round 5); staging: the
    # round-4 form
    split = os.environ.get("KGE_BENCH_EVAL_SPLIT", "planes")
    qp = torch.empty(int(lib.kge_split_bf16x3_bytes(Bq, K)), dtype=torch.uint8, device=device)
    ep = torch.empty(int(lib.kge_split_bf16x3_bytes(E, K)), dtype=torch.uint8, device=device)
    rws = torch.empty(int(lib.kge_eval_rank_planes_workspace_size(Bq, max(b[5] for b in batches))) + 16,
                      dtype=torch.uint8, device=device)
    pipe = evaluate.RankPipeline(m, ep, Bq, max(b[5] for b in batches)) if split == "planes" else None

    def entity_pass():
        """The start of an evaluation pass: the entity table's bf16 planes (evaluate.entity_planes), once per pass."""
        if split in ("planes", "planes1", "planes_s"):
            lib.kge_split_bf16x3(ent.data_ptr(), E, K, ent.stride(0), ep.data_ptr(), E,
                                 torch.cuda.current_stream().cuda_stream)
        if pipe is not None:
            pipe.wait_caller()

    def step(b, ev=None):
        """One query batch: Q = h*r or r*t written as bf16 planes (kge_eval_query_planes), S = Q . E^T
        (kge_gemm_nt_bf16x3_planes on the pass's entity planes, events around it; or kge_eval_query +
        kge_gemm_nt_bf16x3, the staging form), exact filtered ranks."""
        pos, mode, truth, fptr, fids = b[:5]
        if pipe is not None:  # the query planes and pair scores on the side stream, events around the GEMM
            return pipe.submit(pos, mode, truth, fptr, fids, b[5], events=ev)
        st = torch.cuda.current_stream().cuda_stream
        md = 0 if mode == "head-batch" else 1
        rel_ = m.relation_embedding
        if split in ("planes1", "planes_s"):
            lib.kge_eval_query_planes(FN_IDS[w["fn"]], md, ent.data_ptr(), E, ent.stride(0), rel_.data_ptr(), R,
                                      rel_.stride(0), pos.data_ptr(), Bq, m._D, qp.data_ptr(), Bq, st)
        else:
            lib.kge_eval_query(FN_IDS[w["fn"]], md, ent.data_ptr(), E, ent.stride(0), rel_.data_ptr(), R,
                               rel_.stride(0), pos.data_ptr(), Bq, m._D, Q.data_ptr(), K, st)
        if ev is not None:
            ev[0].record()
        if split == "planes1":
            ranks = torch.empty(Bq, dtype=torch.int64, device=device)
            lib.kge_eval_rank_planes(qp.data_ptr(), Bq, ep.data_ptr(), E, K, Bq, E, truth.data_ptr(), fptr.data_ptr(),
                                     fids.data_ptr(), b[5], ranks.data_ptr(), rws.data_ptr(), rws.numel(), st)
            if ev is not None:
                ev[1].record()
            return ranks
        if split == "planes_s":
            lib.kge_gemm_nt_bf16x3_planes(qp.data_ptr(), Bq, ep.data_ptr(), E, K, S.data_ptr(), E, Bq, E, st)
        else:
            lib.kge_gemm_nt_bf16x3(Q.data_ptr(), K, ent.data_ptr(), ent.stride(0), S.data_ptr(), E, Bq, E, K, st)
        if ev is not None:
            ev[1].record()
        return evaluate.rank_filtered(S, truth, fptr, fids)

    entity_pass()
    for i in range(a.warmup):
        step(batches[i % 4])
    if pipe is not None:
        pipe.flush()
    torch.cuda.synchronize()
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(a.steps)]
    if dist_on:
        import torch.distributed as tdist
        tdist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ranks = []
    entity_pass()  # the timed region is one evaluation pass: its entity planes are made inside it
    for i in range(a.steps):
        ranks.append(step(batches[i % 4], evs[i]))
    if pipe is not None:
        pipe.flush()
    torch.cuda.synchronize()
    if dist_on:
        tdist.barrier()
    dt = time.perf_counter() - t0
    gemm_s = statistics.mean(e0.elapsed_time(e1) for e0, e1 in evs) / 1e3
    overlapped_s = None
    if pipe is not None:
        # the GEMMs of consecutive batches overlap (two streams): each one's events also span the other stream's
        # work, so the per-launch figure is the GEMMs' span (first start to last end) over the launches
        overlapped_s = gemm_s
        gemm_s = evs[0][0].elapsed_time(evs[-1][1]) / 1e3 / a.steps
    flops = 2.0 * Bq * E * K            # the fp32 contraction
    kp = (K + 15) // 16 * 16
    mfma_flops = 6 * 2.0 * Bq * E * kp  # bf16 MFMA work executed (six products, K padded to 16)
    r = torch.cat(ranks)
    if dist_on:
        t = torch.tensor([dt], device=device, dtype=torch.float64)
        tdist.all_reduce(t, op=tdist.ReduceOp.MAX)
        dt = float(t.item())
        allr = [torch.empty_like(r) for _ in range(world)]
        tdist.all_gather(allr, r)
        r = torch.cat(allr)
    met = evaluate.metrics_from_ranks(r.cpu().numpy())
    return {"metric": f"ranked queries/sec, {w['name']}", "value": Bq * a.steps * world / dt, "unit": "queries/s",
            "n_gpus": world, "steps": a.steps, "warmup": a.warmup, "ms_per_step": dt / a.steps * 1e3,
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f32",
            "gemm_numerics": "fp32 operands split once at staging into 3 bf16 terms each (24 significant bits), the six "
                             "products A_i.B_j^T with i + j <= 2 on v_mfma_f32_32x32x16_bf16, fp32 accumulation: error "
                             "vs fp64 within the fp32 MFMA path's (tests/test_eval_gpu.py)",
            "data": "synthetic triples (random init: MRR is not a quality number)",
            "config": {"workload": w["name"], "queries_per_step": Bq * world, "entities": E, "K": K,
                       "parallelism": f"replicas{world}" if world > 1 else "single"},
            "roofline": {"bound": "mfma", "achieved": mfma_flops / gemm_s / 1e12, "peak": 2500.0, "unit": "TFLOP/s",
                         "frac": mfma_flops / gemm_s / 1e12 / 2500.0, "traffic": None,
                         "kernel": ("gemm_nt_x3l_kernel<true> (the counting phase of kge_eval_rank_planes_phases, "
                                    "events around it: 256 x 256 tiles from the query planes and the entity bf16 planes "
                                    "copied global -> LDS by LDS-DMA loads into three stages, six products per 16 k on "
                                    "v_mfma_f32_32x32x16_bf16, each row's count of scores above its truth in the "
                                    "epilogue: no score matrix), with the batch's query planes, pair scores "
                                    "(pair_dot_x3_kernel) and rank_finish_kernel on the same stream; batches alternate "
                                    "between two streams (evaluate.RankPipeline), so a GEMM's events also span the other "
                                    "stream's kernels that share its CUs; the entity planes made once per evaluation "
                                    "pass, inside the timed region" if split == "planes" else
                                    "kge_eval_rank_planes on one stream: pair_dot_x3_kernel + gemm_nt_x3l_kernel<true> + "
                                    "rank_finish_kernel, events around the three" if split == "planes1" else
                                    "gemm_nt_x3l_kernel (256 x 256 tiles from the query and entity bf16 planes by "
                                    "LDS-DMA, S written, then kge_rank_filtered)" if split == "planes_s" else
                                    "gemm_nt_x3s_kernel (256 x 256 tiles, operands split once at staging into bf16 "
                                    "planes, six products per 16 k on v_mfma_f32_32x32x16_bf16)"),
                         "kernel_avg_us": gemm_s * 1e6,
                         **({"kernel_avg_us_what": "span of the overlapping GEMM launches (first start to last end, "
                                                   "events on both streams) / launches",
                             "overlapped_launch_avg_us": overlapped_s * 1e6} if overlapped_s is not None else {}),
                         "fp32_equivalent_tflops": flops / gemm_s / 1e12,
                         "fp32_equivalent_over_fp32_mfma_peak": flops / gemm_s / 1e12 / 157.3},
            "filtered_metrics": met, "build": kge.build_id()}


def transparse_bench(w, a, device):
    """c6: TranSparse scoring step = both calls of supervisor.py:17-18 in kge_transparse_step_forward (head-batch
    negatives [B, N] on the bf16x3 MFMA forms with their row reduction, the positives [B, 1] with their
    logsigmoid; events around the call), after the mask product (kge_transparse_premul); plus the autograd train
    step (deterministic backward + HIP Adam) as a side measurement."""
    from customknowledgegraphembedding_amd.model import TFKGEModel
    from customknowledgegraphembedding_amd.optim import Adam
    from customknowledgegraphembedding_amd.supervisor import Strategy, Sum, Trainer
    m = TFKGEModel("TranSparse", w["nentity"], w["nrelation"], w["hidden_dim"], w["gamma"], device=device, seed=0)
    E, R, B, N, d = w["nentity"], w["nrelation"], w["B"], w["N"], w["hidden_dim"]
    batches = []
    for i in range(4):
        g = np.random.RandomState(1 + i)
        pos = np.stack([g.randint(E, size=B), g.randint(R, size=B), g.randint(E, size=B)], 1)
        neg = np.random.RandomState(2 + i).randint(E, size=(B, N))
        batches.append((torch.from_numpy(pos).to(device), torch.from_numpy(neg).to(device)))
    ent, rel, W, mask = m.entity_embedding.detach(), m.relation_embedding.detach(), m.W.detach(), m.mask

    def step(b, ev=None):
        # supervisor.py:17-18 both calls: kge_transparse_step_forward (the head-batch scores and their row
        # reduction, the positives' scores and logsigmoid; events around that call)
        pos, neg = b
        M = ops.transparse_premul(W, mask) if ops._want_premul(W, pos, neg, 0) else None
        if ev is not None:
            ev[0].record()
        _, on, _, op = ops.transparse_step_forward_raw(0, ent, rel, W, mask, pos, neg, m._gamma_f, M=M)
        if ev is not None:
            ev[1].record()
        return on, op

    for i in range(a.warmup):
        step(batches[i % 4])
    torch.cuda.synchronize()
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(a.steps)]
    t0 = time.perf_counter()
    for i in range(a.steps):
        step(batches[i % 4], evs[i])
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    k_s = statistics.mean(e0.elapsed_time(e1) for e0, e1 in evs) / 1e3
    flops = 2.0 * (B * N + B) * d * d
    # the default forms run the bf16x3 forward (float4 rows: d % 4 == 0, aligned tables). Executed MFMA products
    # of the call: head-batch 256-column super-tiles x 16-deep chunks; the positives' split form 128-column x
    # 16-deep blocks
    x3 = d % 4 == 0
    dp, dk = (d + 255) // 256 * 256, (d + 15) // 16 * 16
    mfma_flops = 6 * 2.0 * B * N * dp * dk + 6 * 2.0 * B * ((d + 127) // 128 * 128) * dk
    train = None
    if a.train_steps > 0:
        wts = torch.ones(B, 1, device=device)
        data = [(pos, neg, wts, torch.tensor([0])) for pos, neg in batches]

        def cycle():
            while True:
                yield from data

        tr = Trainer(Strategy(), data, m, Adam([p for p in m.parameters() if p.requires_grad], lr=5e-5), Sum())
        it = cycle()
        tr.train_step(it)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        for _ in range(a.train_steps):
            tr.train_step(it)
        torch.cuda.synchronize()
        tdt = (time.perf_counter() - t1) / a.train_steps
        train = {"ms_per_step": tdt * 1e3, "triples_per_s": (B * N + B) / tdt, "steps": a.train_steps,
                 "what": "supervisor.py:13-30 with TranSparse: fwd (MFMA) + loss + deterministic MFMA backward "
                         "(kge_transparse_score_bwd) + Keras Adam (kge_adam_update) over E, R and W"}
    return {"metric": f"scored triples/sec (pos+neg, one fused scoring step), {w['name']}",
            "value": (B * N + B) * a.steps / dt, "unit": "triples/s", "n_gpus": 1, "steps": a.steps,
            "warmup": a.warmup, "ms_per_step": dt / a.steps * 1e3, "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "f32", "data": "synthetic (random tables, uniform random ids)",
            "config": {"workload": w["name"], "global_batch": B, "n_neg": N, "d": d},
            "roofline": ({"bound": "mfma", "achieved": mfma_flops / k_s / 1e12, "peak": 2500.0, "unit": "TFLOP/s",
                          "frac": mfma_flops / k_s / 1e12 / 2500.0, "traffic": None,
                          "kernel": "kge_transparse_step_forward: " + ts_kernel_name() + " with the row reduction in "
                                    "its epilogue; ts_fwd_x3g_kernel (columns x K split) + ts_xk_finish_kernel with "
                                    "the logsigmoid",
                          "kernel_avg_us": k_s * 1e6, "fp32_equivalent_tflops": flops / k_s / 1e12,
                          "fp32_equivalent_over_fp32_mfma_peak": flops / k_s / 1e12 / 157.3}
                         if x3 else
                         {"bound": "mfma", "achieved": flops / k_s / 1e12, "peak": 157.3, "unit": "TFLOP/s",
                          "frac": flops / k_s / 1e12 / 157.3, "traffic": None,
                          "kernel": "ts_rows_kernel<TS_FWD> (v_mfma_f32_32x32x2_f32)", "kernel_avg_us": k_s * 1e6}),
            "train_step": train, "build": kge.build_id()}


def ts_kernel_name():
    """The head-batch TranSparse forward kernel the default forms select (kge_transparse.hip launch_rows<TS_FWD>:
    d % 4 == 0, aligned tables, d <= 1024)."""
    return ("ts_fwd_x3s_kernel (256 negatives of one batch row per block, M_r chunks staged once for all of them; "
            "operands split once at staging into bf16 planes, six products on v_mfma_f32_32x32x16_bf16, fp32 "
            "accumulation)")


def train_step_bench(m, batches, steps, warmup):
    """supervisor.py:13-30 train step (fused forward, HIP backward, HIP Keras Adam) on the same
    workload: reported beside the scoring metric, never as `value`."""
    from customknowledgegraphembedding_amd.optim import Adam
    from customknowledgegraphembedding_amd.supervisor import Strategy, Sum, Trainer

    B = batches[0][0].shape[0]
    w = torch.ones(B, 1, device=batches[0][0].device)
    data = [(pos, neg, w, torch.tensor([i % 2])) for i, (pos, neg) in enumerate(batches)]

    def cycle():
        while True:
            yield from data

    tr = Trainer(Strategy(), data, m, Adam(m.parameters(), lr=5e-5), Sum())
    it = cycle()
    for _ in range(warmup):
        tr.train_step(it)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        tr.train_step(it)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / steps
    N = batches[0][1].shape[1]
    return {"ms_per_step": dt * 1e3, "triples_per_s": (B * N + B) / dt, "steps": steps, "fused": tr.fused,
            "what": "supervisor.py:13-30 in one C-ABI call (kge_train_step): forward with the backward's query "
                    "pass fused in (one gather of every candidate row), loss, deterministic entity-major backward "
                    "with Keras Adam fused in (4 launches per step)" if tr.fused else
                    "fwd + loss + deterministic bwd (kge_step_backward) + Keras Adam (kge_adam_update)"}


def pipeline_bench(w, a, device):
    """run.py's input pipeline in front of the train step (run.py:40-66,86-90 -> supervisor.Trainer):
    C2-shaped batches written as the reference's TFRecord files (compress_data/main.py:104-131 layout,
    17 files), read back by the C++ reader (CRC verified) on a prefetch thread, moved to the GPU and
    trained on with kge_train_step. Reports the reader alone, the train step on device-resident
    batches, and the end-to-end rate (the slower of the two bounds it)."""
    import shutil
    import tempfile

    from customknowledgegraphembedding_amd import tfrecord
    from customknowledgegraphembedding_amd.optim import Adam
    from customknowledgegraphembedding_amd.supervisor import Strategy, Sum, Trainer

    m, dev_batches = make_inputs(w, 0, device)
    B, N = w["B"], w["N"]
    host = []
    for i, (pos, neg) in enumerate(dev_batches):
        wt = torch.from_numpy(np.random.RandomState(7 + i).uniform(0.1, 1.0, size=(B, 1)).astype(np.float32))
        host.append((pos.cpu(), neg.cpu(), wt, torch.full((B,), i % 2, dtype=torch.int64)))
    d = tempfile.mkdtemp(prefix="kge_tfrec_")
    try:
        paths = tfrecord.write_file_tfrecords(host * 4, d, B, split_number=17)
        nbytes = sum(os.path.getsize(p) for p in paths)
        # the reader alone (one pass over every file, no prefetch thread)
        t0 = time.perf_counter()
        nrec = sum(1 for _ in tfrecord.load_batches(paths, B, repeat=False, prefetch=0))
        read_s = (time.perf_counter() - t0) / nrec
        # train step on device-resident batches vs fed from the files
        data = [(p.to(device), n.to(device), wt.to(device), md) for p, n, wt, md in host]

        def cycle():
            while True:
                yield from data

        def run(it, steps):
            tr = Trainer(Strategy(), None, m, Adam(m.parameters(), lr=5e-5), Sum())
            for _ in range(5):
                tr.train_step(it)
            torch.cuda.synchronize()
            t = time.perf_counter()
            for _ in range(steps):
                tr.train_step(it)
            torch.cuda.synchronize()
            return (time.perf_counter() - t) / steps

        resident_s = run(cycle(), a.steps)
        fed_s = run(iter(tfrecord.load_batches(paths, B, repeat=True, prefetch=4)), a.steps)
    finally:
        shutil.rmtree(d, ignore_errors=True)
    return {"metric": "scored (pos+neg) triples/sec through the train step fed from TFRecord files, "
                      + w["name"], "value": (B * N + B) / fed_s, "unit": "triples/s", "n_gpus": 1,
            "steps": a.steps, "warmup": 5, "ms_per_step": fed_s * 1e3, "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "f32",
            "data": "synthetic C2 batches written as reference-layout TFRecord files (17 files), read back",
            "config": {"workload": "run.py pipeline: " + w["name"], "global_batch": B, "n_neg": N,
                       "parallelism": "single"},
            "reader_ms_per_batch": read_s * 1e3, "reader_mb_per_s": nbytes / (read_s * nrec) / 1e6,
            "train_step_resident_ms": resident_s * 1e3, "tfrecord_bytes_per_batch": nbytes / nrec}


def cpu_baseline(w, budget_s=15.0, rows=64):
    """The oracle's torch-CPU fp32 restatement of the reference graph (model.py:114-235 with all
    three branches per call, Q2; two calls per step as supervisor.py:17-18) on a bounded sample:
    `rows` batch rows x N negatives of the same workload. Returns a dict for the JSON line."""
    from oracle import kge_oracle as O
    cores = int(os.environ.get("OMP_NUM_THREADS", "0")) or len(os.sched_getaffinity(0))
    cores = max(1, min(cores, len(os.sched_getaffinity(0))))
    torch.set_num_threads(cores)
    ent_dim, rel_dim, D, _ = dims(w)
    ent, rel, rng = O.make_tables(w["nentity"], w["nrelation"], ent_dim, rel_dim, w["gamma"],
                                  w["hidden_dim"], seed=0, dtype=torch.float32)
    # the same inputs as the timed GPU steps: the first `rows` rows of rank 0's batch 0 (make_inputs)
    N = w["N"]
    pos, neg, src = cpu_baseline_inputs(w, rows)
    mod = 0.5 * rng

    def faithful(mode):
        with torch.no_grad():
            O.tf_call(w["fn"], ent, rel, pos, neg, mode, w["gamma"], rng, mod)
            O.tf_call(w["fn"], ent, rel, pos, neg, 3, w["gamma"], rng, mod)

    def useful(mode):
        with torch.no_grad():
            O.tf_call_useful(w["fn"], ent, rel, pos, neg, mode, w["gamma"], rng, mod)
            O.tf_call_useful(w["fn"], ent, rel, pos, neg, 3, w["gamma"], rng, mod)

    res = {}
    for tag, f in (("faithful", faithful), ("useful", useful)):
        f(0)  # warm-up
        times = []
        t_end = time.perf_counter() + budget_s / 2
        i = 0
        while (len(times) < 3 or time.perf_counter() < t_end) and len(times) < 50:
            t0 = time.perf_counter()
            f(i % 2)
            times.append(time.perf_counter() - t0)
            i += 1
        res[tag] = (statistics.median(times), len(times))
    triples = rows * N + rows
    try:
        cpu_model = [l for l in open("/proc/cpuinfo") if l.startswith("model name")][0].split(":")[1].strip()
    except Exception:  # noqa: BLE001
        cpu_model = "unknown"
    return {
        "value": triples / res["faithful"][0],
        "unit": "triples/s",
        "cores": cores,
        "kind": "port",
        "sample": (f"the first {rows} batch rows x {N} negatives of the GPU line's batch 0 ({w['name']}; positives: "
                   f"{src}, negatives RandomState(2).randint(E)): oracle torch-CPU fp32 restatement of the reference "
                   f"TF graph (2 calls/step, all 3 branches each, Q2), median of {res['faithful'][1]} steps"),
        "useful_only_value": triples / res["useful"][0],
        "cpu_model": cpu_model,
    }


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(a, argv):
    """`bench.py --gpus N` outside torchrun: run the N ranks as children of this process (this
    process never touches the GPU) and return their exit status. Rank 0 prints the JSON line."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={a.gpus}",
           "--master-addr", "127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__)] + list(argv)
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env.setdefault("OMP_NUM_THREADS", "1")
    return subprocess.call(cmd, env=env)


def dry_run(a, world, rank):
    """CPU rehearsal of the launcher and the multi-rank timing contract (gloo; no kernels, no GPU):
    barrier, K timed no-op steps, max over ranks, one JSON line from rank 0."""
    import torch
    import torch.distributed as tdist
    if world > 1:
        tdist.init_process_group("gloo")
    t0 = time.perf_counter()
    for _ in range(a.steps):
        pass
    if world > 1:
        tdist.barrier()
    el = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([el], dtype=torch.float64)
        tdist.all_reduce(t, op=tdist.ReduceOp.MAX)
        el = float(t.item())
        seen = torch.tensor([rank], dtype=torch.int64)
        tdist.all_reduce(seen, op=tdist.ReduceOp.SUM)
        ranks_seen = int(seen.item())
    else:
        ranks_seen = 0
    line = {"metric": METRIC, "value": 0.0, "unit": "triples/s", "n_gpus": world, "steps": a.steps,
            "warmup": a.warmup, "ms_per_step": el / max(1, a.steps) * 1e3, "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "f32", "data": "dry run (no kernels)",
            "config": {"workload": "dry-run", "parallelism": f"replicas{world}"},
            "dry_run": True, "rank_sum": ranks_seen}
    if world > 1:
        # the N > 1 row-sharded record's shape (rowshard_report), every rank's entry gathered as on the GPU
        per = _gather_objects({k: (rank if k == "rank" else 0.0) for k in ROWSHARD_RANK_KEYS}, world)
        line["yago3_10_rowshard"] = rowshard_report(
            WORKLOADS["c4s"], world, a.steps, {k: max(el, 1e-9) for k in ["torchcomm_python"] +
                                               [n for n, _ in ROWSHARD_VARIANTS]}, per, world, "ok", True)
    if rank == 0:
        print(json.dumps(line), flush=True)
    if world > 1:
        tdist.destroy_process_group()


SHARDED_TIMEOUT_S = float(os.environ.get("KGE_BENCH_SHARDED_TIMEOUT", "240"))


SHARDED_TIMEOUT_STATUS = 3  # exit status of a run whose row-sharded side section hung (headline printed)


def sharded_watchdog(line, rank, timeout_s):
    """A timer on every rank around the row-sharded side section: if it has not finished after timeout_s
    (a collective that never completes), rank 0 prints the headline line it already holds, with the section
    marked as timed out, and every rank leaves with status SHARDED_TIMEOUT_STATUS, so the harness can tell
    the hang from a clean run (all ranks' timers start together, after the headline's barrier-bracketed
    measurement). The printed text is serialised HERE, before the section starts writing into `line`, so
    the timer thread never iterates a dict the main thread is changing. Cancelled when the section returns."""
    import threading

    marked = dict(line)
    marked["yago3_10_rowshard_error"] = f"timeout after {timeout_s:.0f} s (collective hang); headline kept"
    text = json.dumps(marked)

    def fire():
        if rank == 0:
            print(text, flush=True)
        sys.stdout.flush()
        sys.stderr.flush()
        os._exit(SHARDED_TIMEOUT_STATUS)

    t = threading.Timer(timeout_s, fire)
    t.daemon = True
    t.start()
    return t


def sharded_single(line, ws, sa, device):
    """c4s at one GPU: the unsharded fused forward through ShardedKGE (no exchange at one rank)."""
    el = sharded_bench(ws, sa, 1, 0, device, False)
    line["yago3_10_rowshard"] = {
        "workload": ws["name"], "n_gpus": 1, "global_batch": ws["B"], "n_neg": ws["N"],
        "triples_per_s": (ws["B"] * ws["N"] + ws["B"]) * sa.steps / el,
        "ms_per_step": el / sa.steps * 1e3, "steps": sa.steps,
        "what": "distributed.ShardedKGE.step_forward at 1 rank: the unsharded fused forward (no exchange)"}


def sharded_lines(line, a, world, rank, device, dist):
    """c4s beside the headline: ShardedKGE.step_forward (at N > 1 the self-checking, per-rank diagnosed
    rowshard_multi) and .train_step at this world size, and at one GPU the simulated 8-rank step
    (shard_sim_bench)."""
    ws = WORKLOADS["c4s"]
    sa = argparse.Namespace(**{**vars(a), "steps": a.sharded_steps, "warmup": 3})
    if dist:
        line["yago3_10_rowshard"] = rowshard_multi(ws, sa, world, rank, device)
    else:
        sharded_single(line, ws, sa, device)
    el = sharded_bench(ws, sa, world, rank, device, dist, train=True)
    if dist:
        el = _max_over_ranks(el, device)
    line["yago3_10_rowshard_train"] = {
        "workload": ws["name"] + ", train step", "n_gpus": world, "global_batch": ws["B"] * world,
        "n_neg": ws["N"], "triples_per_s": (ws["B"] * ws["N"] + ws["B"]) * world * sa.steps / el,
        "ms_per_step": el / sa.steps * 1e3, "steps": sa.steps,
        "what": "distributed.ShardedKGE.train_step: supervisor.py:15-26 over the replicas' batches (SUM "
                "gradients, Keras Adam) with the entity table row-sharded: owned candidates only, one gather "
                "per candidate row, RCCL all-to-all of the owners' query rows, all-gather of [Bg,4] row stats, "
                "all-reduce of query gradients; Adam on the shard"}
    if world == 1:
        line["yago3_10_shard_sim8"] = shard_sim_bench(device, v1=line["yago3_10_rowshard"]["triples_per_s"])


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--workload", default="c2", choices=sorted(WORKLOADS) + ["pipeline"])
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-budget", type=float, default=15.0)
    ap.add_argument("--train-steps", type=int, default=50, help="train-step side measurement (0 = skip)")
    ap.add_argument("--event-group", type=int, default=5,
                    help="timing events bracket groups of this many consecutive launches")
    ap.add_argument("--sharded-steps", type=int, default=20,
                    help="side measurement of the YAGO3-10 row-sharded step (c4s) at the same world size (0 = skip)")
    ap.add_argument("--sharded-train", action="store_true", help="c4s/c4g: time the row-sharded TRAIN step")
    ap.add_argument("--dry-run", action="store_true",
                    help="CPU/gloo rehearsal of the launcher and timing contract (no GPU, no kernels)")
    a = ap.parse_args(argv)

    if "WORLD_SIZE" not in os.environ and a.gpus > 1:
        return launch_ranks(a, argv)  # before any GPU call in this process
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != a.gpus and rank == 0:
        print(f"bench.py: --gpus {a.gpus} but WORLD_SIZE={world}; using WORLD_SIZE", file=sys.stderr)
    if a.dry_run:
        return dry_run(a, world, rank)

    global kge, ops, FN_IDS
    import customknowledgegraphembedding_amd as kge  # noqa: F401
    from customknowledgegraphembedding_amd import ops
    from customknowledgegraphembedding_amd._lib import FN_IDS
    dist = world > 1
    if dist:
        import torch.distributed as tdist
        torch.cuda.set_device(local)
        tdist.init_process_group("nccl", device_id=torch.device("cuda", local))
    device = torch.device("cuda", local)
    torch.cuda.set_device(device)

    if a.workload == "pipeline":
        print(json.dumps(pipeline_bench(WORKLOADS["c2"], a, device)), flush=True)
        return
    w = WORKLOADS[a.workload]
    fn = FN_IDS.get(w["fn"])
    B, N = w["B"], w["N"]
    if w.get("eval") or w.get("transparse"):
        line = (eval_bench(w, a, device, world, rank, dist) if w.get("eval")
                else transparse_bench(w, a, device))
        if rank == 0:
            print(json.dumps(line), flush=True)
        if dist:
            tdist.destroy_process_group()
        return
    if w.get("sharded"):
        elapsed = sharded_bench(w, a, world, rank, device, dist, train=a.sharded_train)
        if dist:
            t = torch.tensor([elapsed], device=device, dtype=torch.float64)
            tdist.all_reduce(t, op=tdist.ReduceOp.MAX)
            elapsed = float(t.item())
        ent, _, _, rel_used = dims(w)
        owned_bytes = B * N * (4 * ent + 12)  # per rank per step, on average
        line = {"metric": f"scored (pos+neg) triples/sec, {w['name']}", "value": (B * N + B) * a.steps * world / elapsed,
                "unit": "triples/s", "n_gpus": world, "steps": a.steps, "warmup": a.warmup,
                "ms_per_step": elapsed / a.steps * 1e3, "higher_is_better": True, "scaling": "weak",
                "vs_baseline": None, "dtype": "f32", "data": "synthetic global batch replicated by seed",
                "config": {"workload": w["name"], "global_batch": B * world, "n_neg": N,
                           "parallelism": f"rowshard{world}", "scheme": w.get("scheme", "owner-computes")},
                "roofline": {"bound": "hbm", "achieved": owned_bytes / (elapsed / a.steps) / 1e9,
                             "peak": HBM_PEAK_GBS, "unit": "GB/s",
                             "frac": owned_bytes / (elapsed / a.steps) / 1e9 / HBM_PEAK_GBS, "traffic": None,
                             "kernel": "whole sharded step (plan, query all-gather, compact scoring, score "
                                       "all-to-all, finish)"},
                "build": kge.build_id()}
        if rank == 0:
            print(json.dumps(line), flush=True)
        if dist:
            tdist.destroy_process_group()
        return
    m, batches = make_inputs(w, rank, device, world=world)

    def barrier():
        if dist:
            tdist.barrier()

    runner = StepRunner(m, batches, fn, planned=os.environ.get("KGE_BENCH_UNPLANNED", "0") != "1")
    for i in range(a.warmup):
        runner(i)
    torch.cuda.synchronize()

    # kernel timing: event pairs bracket groups of `ev_group` consecutive launches (every other
    # group), so the event packets are amortised over several kernels and kept off most launches
    # (a bracket around every single launch adds ~3 us to each step)
    ev_group = max(1, a.event_group)
    evs = {}
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    host_us = []  # host time of each step's calls (the loop is host-bound if these reach the device step)
    for i in range(a.steps):
        g, r = divmod(i, ev_group)
        if g % 2 == 0 and r == 0 and i + ev_group <= a.steps:
            evs[g] = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
            evs[g][0].record()
        h0 = time.perf_counter()
        runner(a.warmup + i)  # continues the warmup's plan chain: one plan per timed step, made inside it
        host_us.append((time.perf_counter() - h0) * 1e6)
        if g in evs and r == ev_group - 1:
            evs[g][1].record()
    torch.cuda.synchronize()
    barrier()
    elapsed = time.perf_counter() - t0
    kern_ms = [evs[g][0].elapsed_time(evs[g][1]) / ev_group for g in sorted(evs)]
    # SURVEY §8d per-mode STEP times (both launches of a step and the gap between them, device time), after the
    # timed region, timed like kern_ms: a group of ev_group same-mode steps is queued first (untimed, it keeps
    # the device busy), then one event pair brackets the next ev_group, so the first launch's host latency does
    # not land inside the pair
    per_mode = {}
    for mode in (0, 1):
        e = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
        for i in range(2 * ev_group):
            if i == ev_group:
                e[0].record()
            runner(i, mode)
        e[1].record()
        torch.cuda.synchronize()
        per_mode[mode] = e[0].elapsed_time(e[1]) / ev_group
    # the same step without the plan made ahead (kge_step_forward: the tile kernel's setup in the scoring
    # launch), device time per step over the same alternating batches: what the plan saves. Planned and
    # unplanned blocks alternate (three rounds each, the planned runner continuing its own plan chain), so both
    # figures see the same clock and cache state
    unplanned_us = planned_us = None
    if runner.planner is not None:
        plain = StepRunner(m, batches, fn, planned=False)
        acc = {"planned": [], "unplanned": []}
        nxt = a.warmup + a.steps
        for rnd in range(3):
            for key in (("planned", "unplanned") if rnd % 2 == 0 else ("unplanned", "planned")):
                e = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                for i in range(4 * ev_group):
                    if i == 2 * ev_group:
                        e[0].record()
                    if key == "planned":
                        runner(nxt)
                        nxt += 1
                    else:
                        plain(i)
                e[1].record()
                torch.cuda.synchronize()
                acc[key].append(e[0].elapsed_time(e[1]) / (2 * ev_group) * 1e3)
        planned_us, unplanned_us = statistics.median(acc["planned"]), statistics.median(acc["unplanned"])
    head_ms, tail_ms = [per_mode[0]], [per_mode[1]]
    if not kern_ms:  # fewer steps than one event group
        kern_ms = head_ms + tail_ms
    if dist:
        t = torch.tensor([elapsed], device=device, dtype=torch.float64)
        tdist.all_reduce(t, op=tdist.ReduceOp.MAX)
        elapsed = float(t.item())

    neg_bytes, pos_bytes = algorithmic_bytes(w)
    step_bytes = neg_bytes + pos_bytes  # the fused kernel moves both calls' bytes
    order = int(kge.load().kge_step_forward_order(w["nentity"], N))  # 0 row-major, 1 XCD-sliced, 2 tiles
    step_kernels = {0: ["step_fwd_kernel"], 1: ["step_fwd_xcd_kernel", "neg_rows_kernel"],
                    2: ["step_fwd_tile_kernel", "neg_rows_kernel"]}[order]
    traffic, traffic_src = pmc_traffic(a.workload, step_kernels)
    kern_avg_s = statistics.mean(kern_ms) / 1e3
    # head and tail reported separately (steps alternate head, tail, ...)
    # unique-row bytes of one step (row reuse inside a batch; the algorithmic bytes count every gather)
    ent_dim_, _, _, _ = dims(w)
    pos0, neg0 = batches[0]
    uniq = torch.unique(torch.cat([neg0.reshape(-1), pos0[:, 0], pos0[:, 2]])).numel()
    triples = (B * N + B) * a.steps * world
    value = triples / elapsed
    line = {
        "metric": METRIC if a.workload == "c2" else f"scored (pos+neg) triples/sec, {w['name']}",
        "value": value,
        "unit": "triples/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": elapsed / a.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic U(-(gamma+2)/d,(gamma+2)/d) tables (seed 0); positives: " + m.positives_source +
                "; negatives RandomState(2).randint(E); 8 distinct batches resident in HBM, mode alternating head/tail",
        "config": {"workload": w["name"], "global_batch": B * world, "n_neg": N, "hidden_dim": w["hidden_dim"],
                   "score_function": w["fn"], "parallelism": f"replicas{world}" if world > 1 else "single"},
        "roofline": roofline_hbm(
            step_bytes, traffic, traffic_src, kern_avg_s,
            l2_gather=l2_gather_roofline(pmc_l2_requests(a.workload, step_kernels), kern_avg_s),
            kernel={0: "step_fwd_kernel (negatives + positives + row reductions, one launch)",
                    1: "step_fwd_xcd_kernel + neg_rows_kernel (the step's two launches: negatives and positives "
                       "gathered in XCD-sliced ascending-id order, then the row reductions)",
                    2: "step_fwd_tile_kernel + neg_rows_kernel (the step's two launches: negatives and positives "
                       "in row-group x XCD-slice tiles, queries in LDS, each block's candidates swept in entity "
                       "order, planned a step ahead by the previous launch's tail blocks; then the row "
                       "reductions)"}[order],
            step_us_head_batch=head_ms[0] * 1e3, step_us_tail_batch=tail_ms[0] * 1e3,
            step_plan=("kge_step_forward_planned: each step's id-only setup (row groups, entity-sorted candidate "
                       "lists) made by the previous step's tail blocks; one plan per timed step"
                       if runner.planner is not None else "none (kge_step_forward)"),
            unplanned_step_us=unplanned_us, planned_step_us=planned_us,
            plan_ab=("device us per step, medians of three interleaved blocks of planned and unplanned steps "
                     "after the timed region"),
            host_us_per_step_median=statistics.median(host_us), event_group_step_us=[x * 1e3 for x in kern_ms],
            unique_row_bytes_per_step=uniq * ent_dim_ * 4, row_reuse=(B * N + 2 * B) / max(1, uniq)),
        "build": kge.build_id(),
    }
    if a.train_steps > 0:
        line["train_step"] = train_step_bench(m, batches, a.train_steps, 5)
    if a.sharded_steps > 0 and a.workload == "c2":
        # the north star's YAGO3-10 row-sharded configuration at this world size (weak scaling: bz=512 per
        # rank), measured beside the headline replica metric; a failure there is recorded in the line and
        # does not cost the headline
        # across processes the section's collectives are its first RCCL use: a hang there must not cost the
        # headline line either (sharded_watchdog)
        dog = sharded_watchdog(line, rank, SHARDED_TIMEOUT_S) if dist else None
        try:
            sharded_lines(line, a, world, rank, device, dist)
        except Exception as e:  # noqa: BLE001
            import traceback
            traceback.print_exc()
            line["yago3_10_rowshard_error"] = repr(e)
        finally:
            if dog is not None:
                dog.cancel()
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        line["cpu_baseline"] = cpu_baseline(w, a.cpu_budget)
    if rank == 0:
        print(json.dumps(line), flush=True)
    if dist:
        tdist.destroy_process_group()


if __name__ == "__main__":
    sys.exit(main() or 0)
