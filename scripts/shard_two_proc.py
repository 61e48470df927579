"""Two processes on one GPU running ShardedKGE.step_forward (plan, query all-gather, compact scoring, score
all-to-all, finish) and ShardedKGE.train_step over torch.distributed (TorchComm): the forward checked bitwise
against the unsharded kernels, the train step against the oracle's replicated-SUM step. gloo carries the device tensors (RCCL cannot place two ranks
on one device); the orchestration, buffers and kernels are the ones an N-GPU RCCL run uses.

    python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
        --master-port 29511 scripts/shard_two_proc.py
Launch it from a process that has not touched the GPU (torchrun's parent does not)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from customknowledgegraphembedding_amd.distributed import ShardedKGE  # noqa: E402
from tests.test_shard_train_gpu import _batches, _oracle_run  # noqa: E402


def main():
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    dev = "cuda"
    out = {}
    # the forward: every home's scores / reductions bitwise equal the unsharded kernels'
    import numpy as np
    import customknowledgegraphembedding_amd as kge
    from customknowledgegraphembedding_amd import ops
    for name, N in (("DistMult", 300), ("InterHT", 40)):
        E, R, d, Bh = 5003, 5, 64, 8
        de, tr = name == "InterHT", name == "InterHT"
        m = kge.TFKGEModel(name, E, R, d, 9.0, double_entity_embedding=de, triple_relation_embedding=tr,
                           device=dev, seed=3)
        sk = ShardedKGE.from_model(m)
        g = np.random.RandomState(11)
        pos = torch.from_numpy(np.stack([g.randint(E, size=world * Bh), g.randint(R, size=world * Bh),
                                         g.randint(E, size=world * Bh)], 1)).to(dev)
        neg = torch.from_numpy(g.randint(E, size=(world * Bh, N))).to(dev)
        ent, rel = m.entity_embedding.detach(), m.relation_embedding.detach()
        ok_fwd = True
        for mode in (0, 1):
            o_neg, o_pos, s = sk.step_forward(pos, neg, mode)
            w_neg, w_pos, w_s, _ = ops.step_forward_raw(kge.FN_IDS[name], mode, ent, rel, m._rel_off, pos, neg, m._D,
                                                        m._gamma_f, m._range_f)
            sl = slice(rank * Bh, (rank + 1) * Bh)
            ok_fwd &= bool(torch.equal(s, w_s[sl]) and torch.equal(o_neg, w_neg[sl]) and torch.equal(o_pos, w_pos[sl]))
        plan = sk.plan(pos, neg, 0)
        out["forward_" + name] = {"bitwise_equal_unsharded": ok_fwd, "collective_bytes": sk.collective_bytes(plan)}
    for name in ("InterHT", "DistMult", "RotatE"):
        E, R, d, Bh, N, gamma, lr = 97, 5, 40, 6, 24, 9.0, 2e-3
        de, dr, tr = name in ("InterHT", "RotatE"), False, name == "InterHT"
        batches = _batches(E, R, world * Bh, N, 3, seed=world)
        sk = ShardedKGE(name, E, R, d, gamma, de, dr, tr, device=dev, seed=7)
        sk.configure_optimizer(lr=lr)
        losses = [float(sk.train_step(p.to(dev), n.to(dev), w.to(dev), m)) for p, n, w, m in batches]
        torch.cuda.synchronize()
        lb, ent_ref, rel_ref = _oracle_run(name, E, R, d, gamma, world, batches, lr)
        out[name] = {"loss_rel_err": max(abs(a - b[rank]) / max(1.0, abs(b[rank])) for a, b in zip(losses, lb)),
                     "shard_err_over_lr": float((sk.shard.cpu().double() - ent_ref[sk.lo:sk.hi]).abs().max()) / lr,
                     "rel_err_over_lr": float((sk.relation_embedding.cpu().double() - rel_ref).abs().max()) / lr}
    ok = all(v["bitwise_equal_unsharded"] if k.startswith("forward_") else
             (v["loss_rel_err"] < 1e-4 and v["shard_err_over_lr"] < 5e-2 and v["rel_err_over_lr"] < 5e-2)
             for k, v in out.items())
    print(json.dumps({"rank": rank, "world": world, "ok": ok, **out}), flush=True)
    dist.destroy_process_group()
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
